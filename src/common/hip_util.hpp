// hip_util.hpp — error checking, device arena, timers, roctx ranges.
//
// Reference parity: the reference checks no return code anywhere
// (/root/reference/main.cu:143-161); every HIP call here goes
// through WC_HIP_CHECK and throws wc::Error with file:line.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace wc {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] void fail(const std::string& msg);

#define WC_HIP_CHECK(expr)                                                                     \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      ::wc::fail(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" + \
                 std::to_string(__LINE__) + " in " #expr);                                     \
  } while (0)

#define WC_CHECK(cond, msg)                                                                      \
  do {                                                                                           \
    if (!(cond)) ::wc::fail(std::string("check failed: ") + (msg) + " at " + __FILE__ + ":" +   \
                            std::to_string(__LINE__));                                          \
  } while (0)

// Debug mode WC_POISON=1 (a test switch, off by default): every device
// allocation of the engine, the merge and the communicators is filled with
// the byte 0xA5 when it is made, and with WC_POISON=2 every DeviceArena region
// also when the arena is reset for reuse — so no kernel or host path can
// silently depend on fresh memory reading as zeros (the reference's own bug
// class: dev_pairs never initialised, main.cu:144).
int poison_level();
// hipMalloc + (WC_POISON) the fill, device-synchronous.
void dev_malloc(void** p, size_t bytes);
template <class T>
inline void dev_malloc(T** p, size_t bytes) {
  void* v = nullptr;
  dev_malloc(&v, bytes);
  *p = static_cast<T*>(v);
}

// Bump allocator over ONE hipMalloc: nothing in the hot path allocates
// (cdna_hip_programming.md Guideline 9).
class DeviceArena {
 public:
  DeviceArena() = default;
  ~DeviceArena();
  DeviceArena(const DeviceArena&) = delete;
  DeviceArena& operator=(const DeviceArena&) = delete;
  void reserve(size_t bytes);  // (re)allocate backing store; invalidates pointers
  void* take(size_t bytes, size_t align = 256);
  template <class T>
  T* take_n(size_t n) {
    return static_cast<T*>(take(n * sizeof(T)));
  }
  void reset();  // WC_POISON=2: the regions handed out so far are poisoned
  size_t capacity() const { return cap_; }
  size_t used() const { return used_; }
  uint64_t generation() const { return gen_; }  // bumped by every reallocation

 private:
  uint8_t* base_ = nullptr;
  size_t cap_ = 0, used_ = 0;
  uint64_t gen_ = 0;
};

// Pinned host buffer (hipHostMalloc) RAII.
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t bytes) { resize(bytes); }
  ~PinnedBuffer();
  PinnedBuffer(PinnedBuffer&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  PinnedBuffer& operator=(PinnedBuffer&& o) noexcept;
  PinnedBuffer(const PinnedBuffer&) = delete;
  void resize(size_t bytes);
  uint8_t* data() const { return p_; }
  size_t size() const { return n_; }

 private:
  uint8_t* p_ = nullptr;
  size_t n_ = 0;
};

// Scoped roctx range (no-op when the profiler is not attached).
class Range {
 public:
  explicit Range(const char* name);
  ~Range();
};

double now_seconds();

// Diagnostics on stderr (stdout stays reference-identical).
// WC_LOG=warn (default) | info | debug  (or 0 / 1 / 2).
enum LogLevel { LOG_WARN = 0, LOG_INFO = 1, LOG_DEBUG = 2 };
int log_level();
void log_printf(int level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#define WC_LOG(level, ...)                                            \
  do {                                                                \
    if ((level) <= ::wc::log_level()) ::wc::log_printf((level), __VA_ARGS__); \
  } while (0)

// Number of compute units of the current device (cached per device).
int device_cu_count(int device);

}  // namespace wc
