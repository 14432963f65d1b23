// L0 platform layer: error propagation, RAII device/pinned buffers, timers,
// roctx ranges and rank-prefixed logging.
//
// Parity notes (reference -> here):
//   include/utils/exceptions.hpp:13-153  ErrorChecker (syncs after EVERY call)
//       -> PSOUP_HIP_CHECK / PSOUP_ROCFFT_CHECK: throw with file:line + rank
//          context and never synchronise; PSOUP_DEBUG_SYNC=1 restores the
//          sync-after-launch behaviour for debugging.
//   include/utils/utils.hpp:20-80  Utils::device_malloc/h2dcpy/...
//       -> DeviceBuffer<T>/PinnedBuffer<T> (RAII, async copies on a stream).
//   include/utils/stopwatch.hpp:9-142  Stopwatch (gettimeofday, seconds)
//       -> Stopwatch (steady_clock, seconds, accumulating) + GpuTimer.
//   include/utils/nvtx.hpp:1-24  PUSH/POP_NVTX_RANGE -> RoctxRange (roctx).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace psoup {

// ---------------------------------------------------------------- errors ----
class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& msg) : std::runtime_error(msg) {}
};

int log_rank();                 // rank used as log prefix (-1 = none)
void set_log_rank(int rank);
bool debug_sync_enabled();      // PSOUP_DEBUG_SYNC env var

// Runtime switches that change candidate numerics (kernel variant flag words,
// numerics-affecting env knobs), recorded by name for the checkpoint identity
// (checkpoint.cpp make_run_identity): spills from a run with other switches
// are never resumed.
void set_numerics_flag(const std::string& name, long value);
std::string numerics_flags();   // "name=value ..." sorted by name

// One-time device start-up, outside every stage timer: HIP loads a
// translation unit's code object at the first launch of one of its kernels
// (tens of ms for the set the search uses), and the first allocation sets up
// the device's memory state.  Every kernel TU registers a no-op launch
// (device_common.hpp); warm_device() runs them all and a small
// allocation on the current device and waits.  Returns the seconds taken.
using WarmFn = void (*)(hipStream_t);
bool register_warmup(WarmFn fn);
double warm_device();

[[noreturn]] void throw_error(const std::string& what, const char* file, int line);

#define PSOUP_THROW(msg)                                                   \
  do {                                                                     \
    std::ostringstream _psoup_os;                                          \
    _psoup_os << msg;                                                      \
    ::psoup::throw_error(_psoup_os.str(), __FILE__, __LINE__);             \
  } while (0)

#define PSOUP_CHECK(cond, msg)                                             \
  do {                                                                     \
    if (!(cond)) PSOUP_THROW("check failed: " #cond ": " << msg);          \
  } while (0)

#define PSOUP_HIP_CHECK(expr)                                              \
  do {                                                                     \
    hipError_t _psoup_e = (expr);                                          \
    if (_psoup_e != hipSuccess)                                            \
      PSOUP_THROW("HIP error " << hipGetErrorName(_psoup_e) << " ("        \
                               << hipGetErrorString(_psoup_e)              \
                               << ") in " #expr);                          \
  } while (0)

// Called after each kernel launch: catches launch-configuration errors
// without a device sync; in debug mode also synchronises the stream so the
// faulting kernel is named.
void post_launch_check(const char* kernel, hipStream_t stream);

// ---------------------------------------------------------------- logging ---
enum class LogLevel { Quiet = 0, Info = 1, Verbose = 2 };
void set_log_level(LogLevel lvl);
LogLevel log_level();
void log_info(const std::string& msg);
void log_verbose(const std::string& msg);

// ---------------------------------------------------------------- buffers ---
template <class T>
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t n) { resize(n); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : ptr_(o.ptr_), n_(o.n_), cap_(o.cap_) {
    o.ptr_ = nullptr;
    o.n_ = o.cap_ = 0;
  }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
      release();
      ptr_ = o.ptr_;
      n_ = o.n_;
      cap_ = o.cap_;
      o.ptr_ = nullptr;
      o.n_ = o.cap_ = 0;
    }
    return *this;
  }
  // Grows (never shrinks) the allocation; contents are not preserved.
  void resize(size_t n) {
    if (n <= cap_) {
      n_ = n;
      return;
    }
    release();
    if (n > 0) PSOUP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&ptr_), n * sizeof(T)));
    n_ = cap_ = n;
  }
  void release() {
    if (ptr_) (void)hipFree(ptr_);
    ptr_ = nullptr;
    n_ = cap_ = 0;
  }
  void zero_async(hipStream_t s) {
    if (n_) PSOUP_HIP_CHECK(hipMemsetAsync(ptr_, 0, n_ * sizeof(T), s));
  }
  T* data() const { return ptr_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }

 private:
  T* ptr_ = nullptr;
  size_t n_ = 0;
  size_t cap_ = 0;
};

template <class T>
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t n) { resize(n); }
  ~PinnedBuffer() { release(); }
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  void resize(size_t n) {
    if (n <= cap_) {
      n_ = n;
      return;
    }
    release();
    if (n > 0) PSOUP_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ptr_), n * sizeof(T), hipHostMallocDefault));
    n_ = cap_ = n;
  }
  void release() {
    if (ptr_) (void)hipHostFree(ptr_);
    ptr_ = nullptr;
    n_ = cap_ = 0;
  }
  T* data() const { return ptr_; }
  size_t size() const { return n_; }
  T& operator[](size_t i) { return ptr_[i]; }
  const T& operator[](size_t i) const { return ptr_[i]; }

 private:
  T* ptr_ = nullptr;
  size_t n_ = 0;
  size_t cap_ = 0;
};

// RAII stream / event owners.
class Stream {
 public:
  Stream() { PSOUP_HIP_CHECK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking)); }
  ~Stream() {
    if (s_) (void)hipStreamDestroy(s_);
  }
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  hipStream_t get() const { return s_; }
  void sync() const { PSOUP_HIP_CHECK(hipStreamSynchronize(s_)); }

 private:
  hipStream_t s_ = nullptr;
};

class Event {
 public:
  explicit Event(bool timing = false) {
    PSOUP_HIP_CHECK(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming));
  }
  ~Event() {
    if (e_) (void)hipEventDestroy(e_);
  }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  void record(hipStream_t s) { PSOUP_HIP_CHECK(hipEventRecord(e_, s)); }
  void sync() { PSOUP_HIP_CHECK(hipEventSynchronize(e_)); }
  hipEvent_t get() const { return e_; }

 private:
  hipEvent_t e_ = nullptr;
};

// ---------------------------------------------------------------- timers ----
// Accumulating wall-clock stopwatch; get_time() returns SECONDS (the
// reference's Stopwatch::getTime also returns seconds despite its comment).
class Stopwatch {
 public:
  void start() {
    t0_ = clock::now();
    running_ = true;
  }
  void stop() {
    if (running_) acc_ += std::chrono::duration<double>(clock::now() - t0_).count();
    running_ = false;
  }
  void reset() {
    acc_ = 0.0;
    running_ = false;
  }
  void add(double seconds) { acc_ += seconds; }  // externally measured interval (e.g. GPU events)
  double get_time() const {
    double t = acc_;
    if (running_) t += std::chrono::duration<double>(clock::now() - t0_).count();
    return t;
  }

 private:
  using clock = std::chrono::steady_clock;
  clock::time_point t0_{};
  double acc_ = 0.0;
  bool running_ = false;
};

// GPU-side interval timer (hipEvent pair), accumulates milliseconds.
class GpuTimer {
 public:
  GpuTimer() : a_(true), b_(true) {}
  void start(hipStream_t s) { a_.record(s); }
  void stop(hipStream_t s) {
    b_.record(s);
    pending_ = true;
  }
  double elapsed_ms() {
    if (pending_) {
      b_.sync();
      float ms = 0.f;
      PSOUP_HIP_CHECK(hipEventElapsedTime(&ms, a_.get(), b_.get()));
      acc_ += ms;
      pending_ = false;
    }
    return acc_;
  }

 private:
  Event a_, b_;
  bool pending_ = false;
  double acc_ = 0.0;
};

// --------------------------------------------------------------- roctx ------
// Named ranges visible in rocprofv3 --marker-trace (same names as the
// reference's NVTX ranges: "Dedisperse", "DM-Loop", "Acceleration-Loop",
// "Harmonic summing").
class RoctxRange {
 public:
  explicit RoctxRange(const char* name);
  ~RoctxRange();
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;

 private:
  bool active_;
};

void roctx_push(const char* name);
void roctx_pop();

// ---------------------------------------------------------------- device ----
struct DeviceInfo {
  int id = 0;
  std::string name;
  std::string arch;  // gcnArchName, e.g. gfx950:sramecc+:xnack-
  int major = 0;
  int minor = 0;
  int multiprocessors = 0;
  size_t total_mem = 0;
};
int device_count();
// Lets `device` read and write `peer`'s memory directly over xGMI (hipDeviceEnablePeerAccess,
// idempotent); false where the pair cannot (the copies then stage through the host) or is one device.
bool enable_peer_access(int device, int peer);
DeviceInfo device_info(int device);
int runtime_version();
int driver_version();

// Largest power of two STRICTLY less than val (reference utils.hpp:12-18:
// `while (n*2 < val) n *= 2`), so an exact 2^k input yields 2^(k-1).
inline uint64_t prev_power_of_two(uint64_t val) {
  uint64_t n = 1;
  while (n * 2 < val) n *= 2;
  return n;
}

// fn(i0, i1) over contiguous ranges of [0, n) on up to max_threads threads
// (one range per thread, the calling thread included); exceptions rethrown.
template <class F>
void parallel_ranges(size_t n, unsigned max_threads, F&& fn) {
  const unsigned hw = std::max(1u, std::min(max_threads, std::thread::hardware_concurrency()));
  const size_t nt = std::max<size_t>(1, std::min<size_t>(hw, n));
  if (nt == 1) {
    if (n) fn(size_t(0), n);
    return;
  }
  std::vector<std::exception_ptr> err(nt);
  std::vector<std::thread> th;
  auto run = [&](size_t t) {
    try {
      fn(n * t / nt, n * (t + 1) / nt);
    } catch (...) {
      err[t] = std::current_exception();
    }
  };
  for (size_t t = 1; t < nt; ++t) th.emplace_back(run, t);
  run(0);
  for (auto& x : th) x.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// fn(i) for every i in [0, n) on up to max_threads threads taking indices one
// at a time (uneven items: a candidate list's association trees); exceptions
// rethrown.
template <class F>
void parallel_each(size_t n, unsigned max_threads, F&& fn) {
  std::atomic<size_t> next{0};
  parallel_ranges(std::min<size_t>(n, max_threads), max_threads, [&](size_t, size_t) {
    for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
  });
}

// Small fixed-size host worker pool for data-parallel host stages (peak
// clustering / harmonic distillation of a trial batch).  parallel_for(n, fn)
// runs fn(i) for i in [0, n) over the workers plus the calling thread and
// returns when all are done; exceptions are rethrown in the caller.
class HostPool {
 public:
  explicit HostPool(int workers);
  ~HostPool();
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;
  int size() const { return static_cast<int>(threads_.size()) + 1; }
  void parallel_for(int n, const std::function<void(int)>& fn);

 private:
  void loop();
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int n_ = 0, next_ = 0, active_ = 0;
  uint64_t generation_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
};

// FIFO of host tasks run asynchronously by `workers` threads (the engine's
// per-DM acceleration distillation, overlapped with the GPU's next batches).
// wait() blocks until every submitted task has finished and rethrows the
// first exception a task raised; the destructor waits without rethrowing.
class TaskQueue {
 public:
  explicit TaskQueue(int workers);
  ~TaskQueue();
  TaskQueue(const TaskQueue&) = delete;
  TaskQueue& operator=(const TaskQueue&) = delete;
  void submit(std::function<void()> fn);
  void wait();

 private:
  void loop();
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::deque<std::function<void()>> q_;
  int busy_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
};

}  // namespace psoup
