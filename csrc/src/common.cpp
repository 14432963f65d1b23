#include "psoup/common.hpp"

#include <chrono>

#include <vector>

#include <map>

#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <cstring>
#include <iostream>
#include <mutex>

namespace psoup {

namespace {
std::atomic<int> g_rank{-1};
std::atomic<int> g_level{static_cast<int>(LogLevel::Info)};
std::mutex g_log_mutex;

std::string prefix() {
  int r = g_rank.load();
  if (r < 0) return "";
  return "[rank " + std::to_string(r) + "] ";
}
}  // namespace

namespace {
std::mutex g_numerics_mu;
std::map<std::string, long>& numerics_map() {
  static std::map<std::string, long> m;
  return m;
}
}  // namespace

void set_numerics_flag(const std::string& name, long value) {
  std::lock_guard<std::mutex> lk(g_numerics_mu);
  numerics_map()[name] = value;
}

std::string numerics_flags() {
  std::lock_guard<std::mutex> lk(g_numerics_mu);
  std::string s;
  for (const auto& [k, v] : numerics_map()) s += (s.empty() ? "" : " ") + k + "=" + std::to_string(v);
  return s;
}

namespace {
std::vector<WarmFn>& warm_list() {
  static std::vector<WarmFn> v;  // filled by static initialisers of the kernel TUs
  return v;
}
}  // namespace

bool register_warmup(WarmFn fn) {
  warm_list().push_back(fn);
  return true;
}

double warm_device() {
  const auto t0 = std::chrono::steady_clock::now();
  void* p = nullptr;
  PSOUP_HIP_CHECK(hipMalloc(&p, 256));
  for (WarmFn fn : warm_list()) fn(nullptr);
  PSOUP_HIP_CHECK(hipDeviceSynchronize());
  PSOUP_HIP_CHECK(hipFree(p));
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int log_rank() { return g_rank.load(); }
void set_log_rank(int rank) { g_rank.store(rank); }

bool debug_sync_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("PSOUP_DEBUG_SYNC");
    return v && std::strcmp(v, "0") != 0;
  }();
  return on;
}

void throw_error(const std::string& what, const char* file, int line) {
  std::ostringstream os;
  os << prefix() << what << " [" << file << ":" << line << "]";
  throw Error(os.str());
}

void post_launch_check(const char* kernel, hipStream_t stream) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    PSOUP_THROW("launch of " << kernel << " failed: " << hipGetErrorName(e) << " ("
                             << hipGetErrorString(e) << ")");
  if (debug_sync_enabled()) {
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess)
      PSOUP_THROW("kernel " << kernel << " faulted: " << hipGetErrorName(e) << " ("
                            << hipGetErrorString(e) << ")");
  }
}

void set_log_level(LogLevel lvl) { g_level.store(static_cast<int>(lvl)); }
LogLevel log_level() { return static_cast<LogLevel>(g_level.load()); }

void log_info(const std::string& msg) {
  if (g_level.load() < static_cast<int>(LogLevel::Info)) return;
  std::lock_guard<std::mutex> lk(g_log_mutex);
  std::cout << prefix() << msg << std::endl;
}

void log_verbose(const std::string& msg) {
  if (g_level.load() < static_cast<int>(LogLevel::Verbose)) return;
  std::lock_guard<std::mutex> lk(g_log_mutex);
  std::cout << prefix() << msg << std::endl;
}

RoctxRange::RoctxRange(const char* name) : active_(true) { roctxRangePushA(name); }
RoctxRange::~RoctxRange() {
  if (active_) roctxRangePop();
}

void roctx_push(const char* name) { roctxRangePushA(name); }
void roctx_pop() { roctxRangePop(); }

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

bool enable_peer_access(int device, int peer) {
  if (device == peer) return false;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, device, peer) != hipSuccess || !can) return false;
  int prev = 0;
  PSOUP_HIP_CHECK(hipGetDevice(&prev));
  PSOUP_HIP_CHECK(hipSetDevice(device));
  const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  PSOUP_HIP_CHECK(hipSetDevice(prev));
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();  // (clear the sticky status of the benign error)
    return true;
  }
  PSOUP_HIP_CHECK(e);
  return true;
}

DeviceInfo device_info(int device) {
  hipDeviceProp_t p;
  PSOUP_HIP_CHECK(hipGetDeviceProperties(&p, device));
  DeviceInfo d;
  d.id = device;
  d.name = p.name;
  d.arch = p.gcnArchName;
  d.major = p.major;
  d.minor = p.minor;
  d.multiprocessors = p.multiProcessorCount;
  d.total_mem = p.totalGlobalMem;
  return d;
}

int runtime_version() {
  int v = 0;
  (void)hipRuntimeGetVersion(&v);
  return v;
}

int driver_version() {
  int v = 0;
  (void)hipDriverGetVersion(&v);
  return v;
}

HostPool::HostPool(int workers) {
  for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { loop(); });
}

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void HostPool::loop() {
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
    if (stop_) return;
    seen = generation_;
    ++active_;
    while (next_ < n_) {
      const int i = next_++;
      lk.unlock();
      try {
        (*job_)(i);
      } catch (...) {
        lk.lock();
        if (!err_) err_ = std::current_exception();
        lk.unlock();
      }
      lk.lock();
    }
    if (--active_ == 0) done_cv_.notify_all();
  }
}

void HostPool::parallel_for(int n, const std::function<void(int)>& fn) {
  if (n <= 0) return;
  if (threads_.empty() || n == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  std::unique_lock<std::mutex> lk(mu_);
  job_ = &fn;
  n_ = n;
  next_ = 0;
  err_ = nullptr;
  ++generation_;
  ++active_;  // the caller works too
  cv_.notify_all();
  while (next_ < n_) {
    const int i = next_++;
    lk.unlock();
    try {
      fn(i);
    } catch (...) {
      lk.lock();
      if (!err_) err_ = std::current_exception();
      lk.unlock();
    }
    lk.lock();
  }
  --active_;
  done_cv_.wait(lk, [&] { return active_ == 0; });
  job_ = nullptr;
  n_ = 0;
  if (err_) std::rethrow_exception(err_);
}

TaskQueue::TaskQueue(int workers) {
  for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { loop(); });
}

TaskQueue::~TaskQueue() {
  {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [&] { return q_.empty() && busy_ == 0; });
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void TaskQueue::submit(std::function<void()> fn) {
  if (threads_.empty()) {
    fn();
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(fn));
  }
  cv_.notify_one();
}

void TaskQueue::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
    if (q_.empty()) return;  // stop_ with nothing left
    std::function<void()> fn = std::move(q_.front());
    q_.pop_front();
    ++busy_;
    lk.unlock();
    try {
      fn();
    } catch (...) {
      lk.lock();
      if (!err_) err_ = std::current_exception();
      lk.unlock();
    }
    lk.lock();
    --busy_;
    if (q_.empty() && busy_ == 0) idle_cv_.notify_all();
  }
}

void TaskQueue::wait() {
  std::unique_lock<std::mutex> lk(mu_);
  idle_cv_.wait(lk, [&] { return q_.empty() && busy_ == 0; });
  if (err_) {
    std::exception_ptr e = err_;
    err_ = nullptr;
    std::rethrow_exception(e);
  }
}

}  // namespace psoup
