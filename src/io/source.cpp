#include "source.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../common/hip_util.hpp"
#include "../kernels/keys.hpp"

namespace wc {

uint64_t file_size(const std::string& path) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) fail("cannot stat " + path + ": " + std::strerror(errno));
  return (uint64_t)st.st_size;
}

namespace {
// Byte accessor abstraction so file and memory shards share one rule.
template <class Get>
ShardRange owned_range(uint64_t n, int rank, int world, Get get) {
  ShardRange r;
  const uint64_t s = n / world * rank, e = (rank == world - 1) ? n : n / world * (rank + 1);
  uint64_t b = s;
  if (s > 0 && !is_delim(get(s - 1)))  // the token straddling s belongs to the previous shard
    while (b < e && !is_delim(get(b))) ++b;
  if (b >= e) {  // no token starts in this shard
    r.begin = r.end = e;
    return r;
  }
  uint64_t x = e;  // finish the last owned token past e
  if (e > 0 && !is_delim(get(e - 1)))
    while (x < n && !is_delim(get(x))) ++x;
  r.begin = b;
  r.end = x;
  return r;
}
}  // namespace

ShardRange shard_range_mem(const uint8_t* p, uint64_t n, int rank, int world) {
  return owned_range(n, rank, world, [&](uint64_t i) { return (uint32_t)p[i]; });
}

ShardRange shard_range(const std::string& path, int rank, int world) {
  const uint64_t n = file_size(path);
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) fail("cannot open " + path + ": " + std::strerror(errno));
  // small read-through cache for the boundary scans
  std::vector<uint8_t> buf(1 << 16);
  uint64_t buf_off = ~0ull, buf_len = 0;
  auto get = [&](uint64_t i) -> uint32_t {
    if (i < buf_off || i >= buf_off + buf_len) {
      buf_off = i;
      const ssize_t k = ::pread(fd, buf.data(), buf.size(), (off_t)i);
      buf_len = k > 0 ? (uint64_t)k : 0;
      if (!buf_len) return ' ';
    }
    return buf[i - buf_off];
  };
  ShardRange r = owned_range(n, rank, world, get);
  ::close(fd);
  return r;
}

FileSource::FileSource(const std::string& path, uint64_t begin, uint64_t end) : pos_(begin), end_(end) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) fail("cannot open " + path + ": " + std::strerror(errno));
}

FileSource::~FileSource() {
  if (fd_ >= 0) ::close(fd_);
}

namespace {
// Persistent reader threads, one pool PER CALLING THREAD (thread_local below):
// the CLI runs one streaming thread per GPU, each bound to its GPU's NUMA node,
// and its pool's workers inherit that CPU mask; concurrent callers never share
// a pool.  Threads spawned per 64 MiB piece cost tens of us each and capped the
// split at 4 (16 MiB slices); the stream read at 54 GB/s against 75 GB/s
// standalone (profiles/r4_session3.md §10).
//
// Task claims go through ONE 64-bit ticket = generation << 32 | next index,
// advanced by compare-exchange only while its generation is the caller's: a
// worker still inside help() of an earlier run can never claim (or count) a
// task of the next run, and run() returns only when every task of its own
// generation has finished (the tasks' captures live on the caller's stack).
class ReadPool {
 public:
  explicit ReadPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~ReadPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // f(0) .. f(tasks - 1) over the workers and the caller; returns when all ran.
  void run(unsigned tasks, const std::function<void(unsigned)>& f) {
    std::lock_guard<std::mutex> one(run_m_);  // one run at a time (re-entry from another thread waits)
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &f;
      ntasks_ = tasks;
      done_.store(0);
      gen = ++gen_;
      ticket_.store(gen << 32);
    }
    cv_.notify_all();
    help(gen);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [&] { return done_.load() == tasks; });
    job_ = nullptr;
  }

 private:
  void help(uint64_t gen) {
    for (;;) {
      uint64_t t = ticket_.load();
      unsigned i;
      do {
        if ((t >> 32) != gen) return;  // a later run: not ours
        i = (unsigned)t;
        if (i >= ntasks_) return;      // ntasks_ is this generation's while t's generation is
      } while (!ticket_.compare_exchange_weak(t, t + 1));
      (*job_)(i);  // the run cannot end (nor job_ change) before this task is counted
      if (done_.fetch_add(1) + 1 == ntasks_) {
        std::lock_guard<std::mutex> g(m_);
        done_cv_.notify_all();
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      uint64_t gen;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        gen = seen = gen_;
      }
      help(gen);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(unsigned)>* job_ = nullptr;
  std::atomic<uint64_t> ticket_{0};
  std::atomic<unsigned> done_{0};
  std::atomic<unsigned> ntasks_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};
}  // namespace

uint64_t pread_parallel(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
  // One thread copies ~5-8 GB/s out of the page cache, below PCIe Gen5 x16
  // (57 GB/s measured pinned H2D): large reads are split over WC_IO_THREADS
  // (default 16) persistent threads, 4 MiB minimum per slice.
  static const unsigned kThreads = [] {
    const char* e = std::getenv("WC_IO_THREADS");
    const long v = e ? std::strtol(e, nullptr, 10) : 16;
    return (unsigned)std::max(1l, std::min(64l, v));
  }();
  constexpr uint64_t kMinSlice = 4ull << 20;
  const unsigned t = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(kThreads, n / kMinSlice));
  auto slice = [&](uint64_t b, uint64_t e, uint64_t& got, int& err) {
    got = 0;
    err = 0;
    while (b + got < e) {
      const ssize_t k = ::pread(fd, dst + b + got, std::min<uint64_t>(e - b - got, 1ull << 30), (off_t)(off + b + got));
      if (k < 0) {
        if (errno == EINTR) continue;
        err = errno;
        return;
      }
      if (k == 0) return;  // end of file
      got += (uint64_t)k;
    }
  };
  std::vector<uint64_t> got(t), lo(t);
  std::vector<int> err(t);
  const uint64_t per = (n + t - 1) / t;
  for (unsigned i = 0; i < t; ++i) lo[i] = std::min(n, (uint64_t)i * per);
  const std::function<void(unsigned)> task = [&](unsigned i) { slice(lo[i], std::min(n, lo[i] + per), got[i], err[i]); };
  if (t == 1) {
    task(0);
  } else {
    thread_local ReadPool pool(kThreads - 1);  // + the caller; this thread's own pool (its CPU mask)
    pool.run(t, task);
  }
  uint64_t total = 0;  // contiguous prefix: a short slice ends the read
  for (unsigned i = 0; i < t; ++i) {
    if (err[i]) fail(std::string("read error: ") + std::strerror(err[i]));
    total += got[i];
    if (lo[i] + got[i] < std::min(n, lo[i] + per)) break;
  }
  return total;
}

uint64_t FileSource::read(uint8_t* dst, uint64_t cap) {
  const uint64_t want = std::min<uint64_t>(cap, end_ - pos_);
  const uint64_t got = want ? pread_parallel(fd_, dst, want, pos_) : 0;
  pos_ += got;
  return got;
}

ReplaySource::ReplaySource(const uint8_t* pool, uint64_t pool_bytes, uint64_t total)
    : pool_(pool), pool_bytes_(pool_bytes), total_(total) {
  WC_CHECK(pool_bytes > 0 && is_delim(pool[pool_bytes - 1]), "replay pool must end with a delimiter");
}

uint64_t ReplaySource::read(uint8_t* dst, uint64_t cap) {
  uint64_t got = 0;
  while (got < cap && produced_ < total_) {
    const uint64_t k = std::min({cap - got, pool_bytes_ - pos_, total_ - produced_});
    std::memcpy(dst + got, pool_ + pos_, k);
    got += k;
    produced_ += k;
    pos_ = (pos_ + k) % pool_bytes_;
  }
  return got;
}

std::string read_file(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) fail("cannot open " + path + ": " + std::strerror(errno));
  std::string out;
  char buf[1 << 16];
  for (;;) {
    const ssize_t k = ::read(fd, buf, sizeof buf);
    if (k < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      fail("read error on " + path);
    }
    if (k == 0) break;
    out.append(buf, (size_t)k);
  }
  ::close(fd);
  return out;
}

}  // namespace wc
