// comm.hpp — collective interface used by the cross-GPU merge.
//
// The reference has no communication at all.  Backends:
//  * RcclComm      RCCL over xGMI; either one process per GPU (unique id shared
//                  by the launcher, e.g. torch.distributed's store) or one
//                  process driving all GPUs (ncclCommInitAll, the CLI).
//  * LoopbackComm  N virtual ranks in one process (threads), any devices —
//                  exercises sharding + merge at N = 1..8 on a single GPU.
// All buffers are device pointers on the caller's current device and every
// call is ordered on the given stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace wc {

enum class RedOp { Sum, Min, Max };

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* backend() const = 0;
  // recv[r * bytes ...] = rank r's send (bytes each).
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // recv[count] = op over ranks of send[rank * count ... + count).
  virtual void reduce_scatter_u64(const uint64_t* send, uint64_t* recv, size_t count, RedOp op, hipStream_t s) = 0;
  // Personalised exchange (the MapReduce shuffle): bytes [send_off[p], +send_bytes[p]) of
  // `send` go to rank p, which receives them at recv + recv_off[me].  Arrays have size().
  virtual void alltoallv(const void* send, const size_t* send_off, const size_t* send_bytes, void* recv,
                         const size_t* recv_off, const size_t* recv_bytes, hipStream_t s) = 0;
  virtual void broadcast(void* buf, size_t bytes, int root, hipStream_t s) = 0;
  // Bracket several collectives / point-to-point exchanges into ONE launch
  // (RCCL group); no-op for backends that run each call on its own.
  virtual void group_begin() {}
  virtual void group_end() {}
  virtual void barrier(hipStream_t s) = 0;
  // Wait for everything queued on s (collectives included) — the merge's only
  // host sync points.  RCCL polls the stream and ncclCommGetAsyncError; an
  // async error, or no progress within timeout_s(), aborts the communicator
  // (ncclCommAbort) and throws instead of hanging the job.
  virtual void sync(hipStream_t s);
  // Wait for a page-locked word that a publish launch on s stores last
  // (system-scope release): a host spin wakes within a microsecond of the
  // store, where sync()'s stream query waits for the completion signal (~20-30
  // us of GPU idle between merged jobs).  The same watchdog as sync(): the
  // backend's async error and the timeout are polled while spinning.
  void wait_word(const uint32_t* word, uint32_t want, hipStream_t s);
  // Mark the communicator failed: later calls throw, and peers blocked in a
  // collective of the loopback backend wake up and throw.
  virtual void abort(const std::string& why) { failed_ = why.empty() ? "aborted" : why; }
  bool failed() const { return !failed_.empty(); }
  double timeout_s() const { return timeout_s_; }
  // Process-wide counters (tests): collectives enqueued, and host waits of
  // the communicators (sync(); barrier() waits through it) — a merge's host
  // waits must not grow with its collective count.
  static uint64_t collectives_total();
  static uint64_t host_waits_total();

 protected:
  Comm();
  // A failure the backend knows of without waiting (RCCL: ncclCommGetAsyncError;
  // loopback: a peer aborted) -> true and the reason.
  virtual bool poll_error(std::string& why) {
    (void)why;
    return false;
  }
  // Called at the top of every collective: throws once the communicator has
  // failed, and implements fault injection — WC_COMM_FAULT=<rank>[:<n>] makes
  // rank <rank> fail its n-th collective (default 1st) as a simulated comm
  // failure, for tests of the failure path.
  void tick(int rank);
  static void count_host_wait();
  std::string failed_;

 private:
  double timeout_s_ = 300.0;  // WC_COMM_TIMEOUT_S
  int fault_rank_ = -1;
  uint64_t fault_at_ = 0, calls_ = 0;
};

// RCCL.  unique_id is the 128-byte ncclUniqueId blob.
constexpr int RCCL_ID_BYTES = 128;
std::string rccl_unique_id();
std::unique_ptr<Comm> make_rccl_comm(const std::string& unique_id, int rank, int size, int device);
std::vector<std::unique_ptr<Comm>> make_rccl_comms_all(const std::vector<int>& devices);

// In-process virtual ranks (call each rank's methods from its own thread;
// every rank's stream on one device, or on devices with peer access enabled:
// the transfer kernel reads the peers' buffers directly).
// devices (optional, one per rank): distinct devices must be peer-accessible —
// the transfer kernel reads the peers' buffers directly — and peer access is
// enabled between every pair here (refused with an error when unsupported).
std::vector<std::unique_ptr<Comm>> make_loopback_comms(int n, const std::vector<int>& devices = {});

}  // namespace wc
