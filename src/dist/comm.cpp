// comm.cpp — RCCL and loopback implementations of wc::Comm.
#include "comm.hpp"

#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "../common/hip_util.hpp"

namespace wc {

void launch_combine_u64(uint64_t* dst, const uint64_t* src, uint64_t n, int op, hipStream_t s);  // merge.hip

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

void Comm::tick(int rank) {
  if (failed()) fail("communicator failed earlier: " + failed_);
  ++calls_;
  if (rank == fault_rank_ && calls_ == fault_at_) {
    const std::string why = "injected comm fault (WC_COMM_FAULT) at collective " + std::to_string(calls_) +
                            " of rank " + std::to_string(rank);
    abort(why);
    fail(why);
  }
}

void Comm::sync(hipStream_t s) {
  if (failed()) fail("communicator failed earlier: " + failed_);
  WC_HIP_CHECK(hipStreamSynchronize(s));
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
    WC_HIP_CHECK(hipMalloc(&scratch_, 8));
  }
  ~RcclComm() override {
    (void)hipFree(scratch_);
    if (c_) (void)ncclCommDestroy(c_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* backend() const override { return "rccl"; }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    tick(rank_);
    WC_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, c_, s));
  }
  void reduce_scatter_u64(const uint64_t* send, uint64_t* recv, size_t count, RedOp op, hipStream_t s) override {
    tick(rank_);
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

// Shared rendezvous for loopback ranks.
struct Hub {
  explicit Hub(int n) : n(n), offs(n, nullptr), ptrs(n, nullptr) {}
  int n;
  std::vector<const size_t*> offs;  // alltoallv: each rank's send offsets
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<const void*> ptrs;
  bool aborted = false;  // a rank failed: every current and later wait throws
  std::string why;
  void wait_all() {
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
  void abort(const std::string& w) {
    std::lock_guard<std::mutex> lk(mu);
    if (!aborted) {
      aborted = true;
      why = w;
    }
    cv.notify_all();
  }
};

class LoopbackComm final : public Comm {
 public:
  LoopbackComm(std::shared_ptr<Hub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  ~LoopbackComm() override {
    if (scratch_) (void)hipFree(scratch_);
  }
  int rank() const override { return rank_; }
  int size() const override { return hub_->n; }
  const char* backend() const override { return "loopback"; }
  void abort(const std::string& why) override {
    Comm::abort(why);
    hub_->abort("rank " + std::to_string(rank_) + ": " + failed_);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    tick(rank_);
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->ptrs[rank_] = send;
    hub_->wait_all();
    for (int r = 0; r < hub_->n; ++r)
      WC_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + (size_t)r * bytes, hub_->ptrs[r], bytes,
                                  hipMemcpyDefault, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->wait_all();  // senders may reuse their buffers after everyone copied
  }
  void reduce_scatter_u64(const uint64_t* send, uint64_t* recv, size_t count, RedOp op, hipStream_t s) override {
    tick(rank_);
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->ptrs[rank_] = send;
    hub_->wait_all();
    if (count > scratch_n_) {  // grown once, reused: no allocation per collective
      if (scratch_) WC_HIP_CHECK(hipFree(scratch_));
      WC_HIP_CHECK(hipMalloc(&scratch_, count * 8));
      scratch_n_ = count;
    }
    uint64_t* tmp = scratch_;
    for (int r = 0; r < hub_->n; ++r) {
      const uint64_t* src = static_cast<const uint64_t*>(hub_->ptrs[r]) + (size_t)rank_ * count;
      if (!count) break;
      if (r == 0) {
        WC_HIP_CHECK(hipMemcpyAsync(recv, src, count * 8, hipMemcpyDefault, s));
      } else {
        WC_HIP_CHECK(hipMemcpyAsync(tmp, src, count * 8, hipMemcpyDefault, s));
        launch_combine_u64(recv, tmp, count, (int)op, s);
      }
    }
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->wait_all();
  }
  void alltoallv(const void* send, const size_t* send_off, const size_t* /*send_bytes*/, void* recv,
                 const size_t* recv_off, const size_t* recv_bytes, hipStream_t s) override {
    tick(rank_);
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->ptrs[rank_] = send;
    hub_->offs[rank_] = send_off;
    hub_->wait_all();
    for (int r = 0; r < hub_->n; ++r)
      if (recv_bytes[r])
        WC_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[r],
                                    static_cast<const uint8_t*>(hub_->ptrs[r]) + hub_->offs[r][rank_], recv_bytes[r],
                                    hipMemcpyDefault, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->wait_all();
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
    tick(rank_);
    WC_HIP_CHECK(hipStreamSynchronize(s));
    if (rank_ == root) hub_->ptrs[root] = buf;
    hub_->wait_all();
    if (rank_ != root && bytes) WC_HIP_CHECK(hipMemcpyAsync(buf, hub_->ptrs[root], bytes, hipMemcpyDefault, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->wait_all();
  }
  void barrier(hipStream_t s) override {
    tick(rank_);
    WC_HIP_CHECK(hipStreamSynchronize(s));
    hub_->wait_all();
  }

 private:
  std::shared_ptr<Hub> hub_;
  int rank_;
  uint64_t* scratch_ = nullptr;  // reduce-scatter staging (device of this rank)
  size_t scratch_n_ = 0;
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
  WC_NCCL_CHECK(ncclCommInitRank(&c, size, id, rank));
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

std::vector<std::unique_ptr<Comm>> make_loopback_comms(int n) {
  auto hub = std::make_shared<Hub>(n);
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < n; ++r) out.emplace_back(new LoopbackComm(hub, r));
  return out;
}

}  // namespace wc
