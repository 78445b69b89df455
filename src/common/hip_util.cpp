#include "hip_util.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>

namespace wc {

void fail(const std::string& msg) { throw Error(msg); }

int poison_level() {
  static const int v = std::getenv("WC_POISON") ? std::atoi(std::getenv("WC_POISON")) : 0;
  return v;
}

namespace {
void poison(void* p, size_t bytes) {
  if (!p || !bytes) return;
  WC_HIP_CHECK(hipDeviceSynchronize());  // nothing queued still uses the region (arena reuse)
  WC_HIP_CHECK(hipMemset(p, 0xA5, bytes));
  WC_HIP_CHECK(hipDeviceSynchronize());
}
}  // namespace

void dev_malloc(void** p, size_t bytes) {
  *p = nullptr;
  WC_HIP_CHECK(hipMalloc(p, bytes));
  if (poison_level() >= 1) poison(*p, bytes);
}

DeviceArena::~DeviceArena() {
  if (base_) (void)hipFree(base_);
}

void DeviceArena::reserve(size_t bytes) {
  if (bytes <= cap_) {
    used_ = 0;
    return;
  }
  // work already launched may still write the old store (the engine's merge
  // zeroing rides in a job's first launch): drained before it is freed
  if (base_) WC_HIP_CHECK(hipDeviceSynchronize());
  if (base_) WC_HIP_CHECK(hipFree(base_));
  base_ = nullptr;
  cap_ = used_ = 0;
  dev_malloc(&base_, bytes);
  cap_ = bytes;
  ++gen_;
}

void DeviceArena::reset() {
  if (poison_level() >= 2 && used_) poison(base_, used_);
  used_ = 0;
}

void* DeviceArena::take(size_t bytes, size_t align) {
  size_t off = (used_ + align - 1) / align * align;
  if (off + bytes > cap_)
    fail("device arena exhausted: need " + std::to_string(off + bytes) + " of " + std::to_string(cap_));
  used_ = off + bytes;
  return base_ + off;
}

PinnedBuffer::~PinnedBuffer() {
  if (p_) (void)hipHostFree(p_);
}

PinnedBuffer& PinnedBuffer::operator=(PinnedBuffer&& o) noexcept {
  if (this != &o) {
    if (p_) (void)hipHostFree(p_);
    p_ = o.p_;
    n_ = o.n_;
    o.p_ = nullptr;
    o.n_ = 0;
  }
  return *this;
}

void PinnedBuffer::resize(size_t bytes) {
  if (bytes <= n_) return;
  if (p_) WC_HIP_CHECK(hipHostFree(p_));
  p_ = nullptr;
  n_ = 0;
  WC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_), bytes, hipHostMallocDefault));
  n_ = bytes;
}

Range::Range(const char* name) { roctxRangePush(name); }
Range::~Range() { roctxRangePop(); }

int log_level() {
  static const int lvl = [] {
    const char* e = std::getenv("WC_LOG");
    if (!e || !*e) return (int)LOG_WARN;
    const std::string v(e);
    if (v == "debug" || v == "2") return (int)LOG_DEBUG;
    if (v == "info" || v == "1") return (int)LOG_INFO;
    return (int)LOG_WARN;
  }();
  return lvl;
}

void log_printf(int level, const char* fmt, ...) {
  static const double t0 = now_seconds();
  static const char* tag[] = {"warn", "info", "debug"};
  char line[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(line, sizeof(line), fmt, ap);
  va_end(ap);
  // one fprintf per line: lines of concurrent rank threads do not interleave
  std::fprintf(stderr, "[wc %s %9.3f] %s\n", tag[level < 0 ? 0 : level > 2 ? 2 : level], now_seconds() - t0, line);
}

double now_seconds() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

int device_cu_count(int device) {
  static std::mutex mu;
  static std::vector<int> cache;
  std::lock_guard<std::mutex> g(mu);
  if ((int)cache.size() <= device) cache.resize(device + 1, 0);
  if (!cache[device]) {
    hipDeviceProp_t p;
    WC_HIP_CHECK(hipGetDeviceProperties(&p, device));
    cache[device] = p.multiProcessorCount;
  }
  return cache[device];
}

}  // namespace wc
