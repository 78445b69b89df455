// comm.cpp — RCCL and loopback implementations of wc::Comm.
#include "comm.hpp"

#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "../common/hip_util.hpp"
#include "../kernels/kernels.hpp"

namespace wc {


#define WC_NCCL_CHECK(expr)                                                                          \
  do {                                                                                                \
    ncclResult_t r_ = (expr);                                                                         \
    if (r_ != ncclSuccess)                                                                            \
      ::wc::fail(std::string("RCCL error ") + ncclGetErrorString(r_) + " at " + __FILE__ + ":" +     \
                 std::to_string(__LINE__) + " in " #expr);                                           \
  } while (0)

Comm::Comm() {
  if (const char* e = std::getenv("WC_COMM_TIMEOUT_S")) {
    const double t = std::atof(e);
    if (t > 0) timeout_s_ = t;
  }
  if (const char* e = std::getenv("WC_COMM_FAULT"); e && *e) {
    char* end = nullptr;
    fault_rank_ = (int)std::strtol(e, &end, 10);
    fault_at_ = (end && *end == ':') ? std::strtoull(end + 1, nullptr, 10) : 1;
  }
}

namespace {
std::atomic<uint64_t> g_collectives{0}, g_host_waits{0};
}
uint64_t Comm::collectives_total() { return g_collectives.load(); }
uint64_t Comm::host_waits_total() { return g_host_waits.load(); }
void Comm::count_host_wait() { ++g_host_waits; }

void Comm::tick(int rank) {
  if (failed()) fail("communicator failed earlier: " + failed_);
  ++calls_;
  ++g_collectives;
  if (rank == fault_rank_ && calls_ == fault_at_) {
    const std::string why = "injected comm fault (WC_COMM_FAULT) at collective " + std::to_string(calls_) +
                            " of rank " + std::to_string(rank);
    abort(why);
    fail(why);
  }
}

void Comm::sync(hipStream_t s) {
  if (failed()) fail("communicator failed earlier: " + failed_);
  count_host_wait();
  WC_HIP_CHECK(hipStreamSynchronize(s));
}

void Comm::wait_word(const uint32_t* word, uint32_t want, hipStream_t s) {
  if (failed()) fail("communicator failed earlier: " + failed_);
  count_host_wait();
  const double t0 = now_seconds();
  for (uint64_t it = 1;; ++it) {
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == want) break;
    if ((it & 0x3FFF) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q != hipErrorNotReady) {
        WC_HIP_CHECK(q);
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) != want) fail("publish launch completed without its sequence word");
        break;
      }
      std::string why;
      if (!poll_error(why) && now_seconds() - t0 > timeout_s())
        why = std::string(backend()) + " collective made no progress for " + std::to_string((int)timeout_s()) +
              " s (WC_COMM_TIMEOUT_S)";
      if (!why.empty()) {
        abort(why);
        fail(why + "; communicator aborted");
      }
    }
    __builtin_ia32_pause();
  }
  std::string why;
  if (poll_error(why)) {
    abort(why);
    fail(why + "; communicator aborted");
  }
}

namespace {

ncclRedOp_t to_nccl(RedOp op) {
  switch (op) {
    case RedOp::Sum: return ncclSum;
    case RedOp::Min: return ncclMin;
    default: return ncclMax;
  }
}

class RcclComm final : public Comm {
 public:
  RcclComm(ncclComm_t c, int rank, int size, int device) : c_(c), rank_(rank), size_(size), dev_(device) {
    WC_HIP_CHECK(hipSetDevice(device));
    dev_malloc(&scratch_, 8);
  }
  ~RcclComm() override {
    (void)hipFree(scratch_);
    if (c_) (void)ncclCommDestroy(c_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* backend() const override { return "rccl"; }
  // An in-place collective over one rank is the identity: no launch (RCCL
  // issued a copy kernel for it, ~5 us each).
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    tick(rank_);
    if (size_ == 1 && send == recv) return;
    WC_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, c_, s));
  }
  void reduce_scatter_u64(const uint64_t* send, uint64_t* recv, size_t count, RedOp op, hipStream_t s) override {
    tick(rank_);
    if (size_ == 1 && send == recv) return;
    WC_NCCL_CHECK(ncclReduceScatter(send, recv, count, ncclUint64, to_nccl(op), c_, s));
  }
  void alltoallv(const void* send, const size_t* send_off, const size_t* send_bytes, void* recv,
                 const size_t* recv_off, const size_t* recv_bytes, hipStream_t s) override {
    tick(rank_);
    WC_NCCL_CHECK(ncclGroupStart());
    for (int p = 0; p < size_; ++p) {
      if (send_bytes[p])
        WC_NCCL_CHECK(ncclSend(static_cast<const uint8_t*>(send) + send_off[p], send_bytes[p], ncclUint8, p, c_, s));
      if (recv_bytes[p])
        WC_NCCL_CHECK(ncclRecv(static_cast<uint8_t*>(recv) + recv_off[p], recv_bytes[p], ncclUint8, p, c_, s));
    }
    WC_NCCL_CHECK(ncclGroupEnd());
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
    tick(rank_);
    if (bytes) WC_NCCL_CHECK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, c_, s));
  }
  void group_begin() override { WC_NCCL_CHECK(ncclGroupStart()); }
  void group_end() override { WC_NCCL_CHECK(ncclGroupEnd()); }
  void barrier(hipStream_t s) override {
    tick(rank_);
    WC_NCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclUint64, ncclSum, c_, s));
    sync(s);
  }
  // Watchdog wait: a peer that died or diverged leaves our collective kernel
  // spinning forever under a plain hipStreamSynchronize.
  void sync(hipStream_t s) override {
    if (failed()) fail("communicator failed earlier: " + failed_);
    count_host_wait();
    const double t0 = now_seconds();
    for (;;) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) WC_HIP_CHECK(q);
      ncclResult_t ar = ncclSuccess;
      WC_NCCL_CHECK(ncclCommGetAsyncError(c_, &ar));
      std::string why;
      if (ar != ncclSuccess && ar != ncclInProgress) why = std::string("RCCL async error: ") + ncclGetErrorString(ar);
      else if (now_seconds() - t0 > timeout_s())
        why = "RCCL collective made no progress for " + std::to_string((int)timeout_s()) + " s (WC_COMM_TIMEOUT_S)";
      if (!why.empty()) {
        abort(why);
        fail(why + " on rank " + std::to_string(rank_) + "; communicator aborted");
      }
      std::this_thread::yield();
    }
  }
  bool poll_error(std::string& why) override {
    if (!c_) return false;
    ncclResult_t ar = ncclSuccess;
    WC_NCCL_CHECK(ncclCommGetAsyncError(c_, &ar));
    if (ar == ncclSuccess || ar == ncclInProgress) return false;
    why = std::string("RCCL async error: ") + ncclGetErrorString(ar);
    return true;
  }
  void abort(const std::string& why) override {
    Comm::abort(why);
    if (c_) {
      WC_LOG(LOG_WARN, "rank %d: aborting RCCL communicator: %s", rank_, why.c_str());
      (void)ncclCommAbort(c_);
      c_ = nullptr;
    }
  }

 private:
  ncclComm_t c_;
  int rank_, size_, dev_;
  void* scratch_ = nullptr;
};

// Shared state of one loopback group: the page-locked metadata the ranks'
// transfer kernels read (kernels.hpp LbShared, src/kernels/comm.hip), the
// per-slot ready / done events, and the arrival rendezvous.
struct Hub {
  explicit Hub(int n) : n(n) {
    WC_CHECK(n >= 1 && n <= LB_MAX_RANKS, "loopback: 1..64 ranks");
    WC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sh), sizeof(LbShared), hipHostMallocCoherent));
    std::memset(sh, 0, sizeof(LbShared));
    ready.resize((size_t)LB_RING * n);
    done.resize((size_t)LB_RING * n);
    for (auto* v : {&ready, &done})
      for (auto& e : *v) WC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  ~Hub() {
    for (auto* v : {&ready, &done})
      for (auto& e : *v)
        if (e) (void)hipEventDestroy(e);
    if (sh) (void)hipHostFree(sh);
  }
  int n;
  LbShared* sh = nullptr;
  std::vector<hipEvent_t> ready, done;  // [slot * n + rank]
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;  // a rank failed: every current and later rendezvous throws
  std::string why;
  // Every rank has ENQUEUED up to this point (a host rendezvous on the calls,
  // never on the GPU: no stream is waited for).
  void arrive() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) fail("loopback peer failed: " + why);
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
      if (gen == g) fail("loopback peer failed: " + why);
    }
  }
  bool is_aborted() {
    std::lock_guard<std::mutex> lk(mu);
    return aborted;
  }
  void abort(const std::string& w) {
    std::lock_guard<std::mutex> lk(mu);
    if (!aborted) {
      aborted = true;
      why = w;
      __atomic_store_n(&sh->aborted, 1u, __ATOMIC_SEQ_CST);  // transfers already queued skip their copies
    }
    cv.notify_all();
  }
};

// Loopback ranks, one per thread, every rank's stream on one device (or on
// peer-accessible devices: the transfer kernel reads the peers' buffers
// directly).  A collective is ENQUEUED like an RCCL collective, never waited
// for: each rank records "ready" on its stream behind its earlier work; after
// the arrival rendezvous every peer's ready event exists, so the stream waits
// on all of them (hipStreamWaitEvent) and runs the transfer kernel, which
// reads the peers' buffer addresses from the page-locked metadata; then
// "done" is recorded, a second rendezvous, and the stream waits for every
// peer's done (a send buffer is reusable once the collective completes on the
// stream, as with RCCL).  Nothing is complete until the stream gets there: a
// host read of a collective's output before sync() sees stale data, exactly
// as with RCCL.  Only arrival rendezvous block the host (for the peers to
// CALL the collective); every event waited on was recorded before the wait
// was enqueued, so streams sharing a hardware queue (GPU_MAX_HW_QUEUES) never
// wait on work queued behind them.
class LoopbackComm final : public Comm {
 public:
  LoopbackComm(std::shared_ptr<Hub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  ~LoopbackComm() override = default;
  int rank() const override { return rank_; }
  int size() const override { return hub_->n; }
  const char* backend() const override { return "loopback"; }
  void abort(const std::string& why) override {
    Comm::abort(why);
    hub_->abort("rank " + std::to_string(rank_) + ": " + failed_);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    tick(rank_);
    LbMeta& m = begin();
    m.send = reinterpret_cast<uint64_t>(send);
    m.recv = reinterpret_cast<uint64_t>(recv);
    enqueue(LB_ALLGATHER, bytes, 0, 0, s);
  }
  void reduce_scatter_u64(const uint64_t* send, uint64_t* recv, size_t count, RedOp op, hipStream_t s) override {
    tick(rank_);
    LbMeta& m = begin();
    m.send = reinterpret_cast<uint64_t>(send);
    m.recv = reinterpret_cast<uint64_t>(recv);
    enqueue(LB_REDUCE_SCATTER, count, (uint32_t)op, 0, s);
  }
  void alltoallv(const void* send, const size_t* send_off, const size_t* /*send_bytes*/, void* recv,
                 const size_t* recv_off, const size_t* recv_bytes, hipStream_t s) override {
    tick(rank_);
    LbMeta& m = begin();
    m.send = reinterpret_cast<uint64_t>(send);
    m.recv = reinterpret_cast<uint64_t>(recv);
    for (int p = 0; p < hub_->n; ++p) {
      m.soff[p] = send_off[p];
      m.roff[p] = recv_off[p];
      m.rbytes[p] = recv_bytes[p];
    }
    enqueue(LB_ALLTOALLV, 0, 0, 0, s);
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
    tick(rank_);
    LbMeta& m = begin();
    m.send = reinterpret_cast<uint64_t>(buf);
    m.recv = reinterpret_cast<uint64_t>(buf);
    enqueue(LB_BROADCAST, bytes, 0, (uint32_t)root, s);
  }
  void barrier(hipStream_t s) override {
    tick(rank_);
    begin();
    enqueue(~0u, 0, 0, 0, s);  // events only
    sync(s);
  }
  bool poll_error(std::string& why) override {
    if (!hub_->is_aborted()) return false;
    why = "loopback peer failed: " + hub_->why;
    return true;
  }
  // Watchdog wait, as RcclComm::sync (a failed peer is reported).
  void sync(hipStream_t s) override {
    if (failed()) fail("communicator failed earlier: " + failed_);
    count_host_wait();
    const double t0 = now_seconds();
    for (;;) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) WC_HIP_CHECK(q);
      if (now_seconds() - t0 > timeout_s()) {
        const std::string why = "loopback collective made no progress for " + std::to_string((int)timeout_s()) +
                                " s (WC_COMM_TIMEOUT_S)";
        abort(why);
        fail(why + " on rank " + std::to_string(rank_));
      }
      std::this_thread::yield();
    }
    if (hub_->is_aborted()) fail("loopback peer failed: " + hub_->why);
    since_sync_ = 0;
  }

 private:
  // Next sequence number and this rank's metadata slot for it.  The slot's previous collective was begun LB_RING collectives ago: if this
  // rank has not completed a sync() since then, the peers' transfer kernels of
  // that collective (which read this metadata when they RUN, not when they are
  // enqueued) may still be queued — wait for its done events before
  // overwriting it.  After a sync() every earlier collective is complete on
  // every peer (this rank's stream waited for all their done events).
  LbMeta& begin() {
    seq_ = (uint32_t)(seq_ + 1);
    slot_ = seq_ % LB_RING;
    Hub& h = *hub_;
    if (++since_sync_ > (uint32_t)LB_RING)
      for (int p = 0; p < h.n; ++p) WC_HIP_CHECK(hipEventSynchronize(h.done[(size_t)slot_ * h.n + p]));
    return h.sh->meta[slot_ * h.n + rank_];
  }
  void enqueue(uint32_t kind, uint64_t count, uint32_t op, uint32_t root, hipStream_t s) {
    Hub& h = *hub_;
    const size_t base = (size_t)slot_ * h.n;
    WC_HIP_CHECK(hipEventRecord(h.ready[base + rank_], s));
    h.arrive();  // every peer's metadata is written and its ready event recorded
    for (int p = 0; p < h.n; ++p)
      if (p != rank_) WC_HIP_CHECK(hipStreamWaitEvent(s, h.ready[base + p], 0));
    if (kind != ~0u) launch_loopback_xfer(LbXfer{h.sh, kind, (uint32_t)h.n, (uint32_t)rank_, slot_, op, root, count}, s);
    WC_HIP_CHECK(hipEventRecord(h.done[base + rank_], s));
    h.arrive();  // every peer's done event recorded
    for (int p = 0; p < h.n; ++p)
      if (p != rank_) WC_HIP_CHECK(hipStreamWaitEvent(s, h.done[base + p], 0));
  }
  std::shared_ptr<Hub> hub_;
  int rank_;
  uint32_t seq_ = 0, slot_ = 0;
  uint32_t since_sync_ = 0;  // collectives begun since this rank's last completed sync()
};

}  // namespace

std::string rccl_unique_id() {
  static_assert(sizeof(ncclUniqueId) == RCCL_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  WC_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof id);
}

std::unique_ptr<Comm> make_rccl_comm(const std::string& unique_id, int rank, int size, int device) {
  WC_CHECK(unique_id.size() == sizeof(ncclUniqueId), "bad RCCL unique id");
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof id);
  WC_HIP_CHECK(hipSetDevice(device));
  ncclComm_t c;
  const ncclResult_t r = ncclCommInitRank(&c, size, id, rank);
  // Two ranks on one GPU: RCCL 2.27 refuses them at init with
  // "NCCL WARN Duplicate GPU detected : rank 0 and rank 1 both on CUDA device
  // 8e000" and ncclInvalidUsage (measured on MI355X, profiles/r6_rccl_one_gpu.md)
  // — one rank per GPU; the loopback communicator shares a GPU instead
  if (r == ncclInvalidUsage)
    fail("RCCL refused rank " + std::to_string(rank) + " of " + std::to_string(size) + " on device " +
         std::to_string(device) + " (ncclInvalidUsage): RCCL allows one rank per GPU (\"Duplicate GPU detected\" when "
         "two ranks share one); give every rank its own GPU, or use --virtual-ranks (loopback) on one GPU");
  if (r != ncclSuccess) fail(std::string("RCCL error ") + ncclGetErrorString(r) + " in ncclCommInitRank");
  return std::unique_ptr<Comm>(new RcclComm(c, rank, size, device));
}

std::vector<std::unique_ptr<Comm>> make_rccl_comms_all(const std::vector<int>& devices) {
  std::vector<ncclComm_t> cs(devices.size());
  WC_NCCL_CHECK(ncclCommInitAll(cs.data(), (int)devices.size(), devices.data()));
  std::vector<std::unique_ptr<Comm>> out;
  for (size_t i = 0; i < devices.size(); ++i)
    out.emplace_back(new RcclComm(cs[i], (int)i, (int)devices.size(), devices[i]));
  return out;
}

std::vector<std::unique_ptr<Comm>> make_loopback_comms(int n, const std::vector<int>& devices) {
  WC_CHECK(devices.empty() || (int)devices.size() == n, "loopback: one device per rank");
  int prev = 0;
  WC_HIP_CHECK(hipGetDevice(&prev));
  for (int a : devices)
    for (int b : devices) {
      if (a == b) continue;
      int ok = 0;
      WC_HIP_CHECK(hipDeviceCanAccessPeer(&ok, a, b));
      WC_CHECK(ok, "loopback ranks on devices " + std::to_string(a) + " and " + std::to_string(b) +
                       ": no peer access between them (the transfer kernel reads peer buffers directly)");
      WC_HIP_CHECK(hipSetDevice(a));
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();  // not an error: clear it
      else WC_HIP_CHECK(e);
    }
  WC_HIP_CHECK(hipSetDevice(prev));
  auto hub = std::make_shared<Hub>(n);
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r) out.emplace_back(new LoopbackComm(hub, r));
  return out;
}

}  // namespace wc
