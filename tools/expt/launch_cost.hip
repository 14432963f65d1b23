// Host cost of a kernel launch on a stream with and without an outstanding
// cross-stream wait (hipStreamWaitEvent on an event of another stream that
// has not completed).  The native pipeline's traces showed ~60 us per launch
// on the engine stream after it joined its sub-batch stream, against ~5 us
// before the join (profiles/r6_host/).
//   hipcc --offload-arch=gfx950 -O2 tools/expt/launch_cost.hip -o /tmp/launch_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void spin_kernel(unsigned long long ticks, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

// memory-bound: streams n floats (HBM traffic while the host launches)
__global__ void copy_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    b[i] = a[i];
}

__global__ void tiny_kernel(int* out, int v) {
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// median host time of n tiny launches on s
static double launches(hipStream_t s, int* buf, int n = 20) {
  std::vector<double> t;
  for (int i = 0; i < n; ++i) {
    const double a = now_us();
    hipLaunchKernelGGL(tiny_kernel, dim3(64), dim3(64), 0, s, buf, i);
    t.push_back(now_us() - a);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const unsigned long long ticks = static_cast<unsigned long long>(rate_khz) * 5;  // 5 ms
  hipStream_t A, B, C;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  int* buf = nullptr;
  CK(hipMalloc(&buf, 1 << 20));
  // warm
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, B, 1ull, buf);
  launches(A, buf);
  launches(B, buf);
  launches(C, buf);
  CK(hipDeviceSynchronize());

  auto report = [](const char* what, double us) { std::printf("%-72s %8.1f us/launch\n", what, us); };
  report("idle stream", launches(A, buf));
  CK(hipDeviceSynchronize());

  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, A, ticks, buf);
  report("behind a 5 ms kernel on the same stream", launches(A, buf));
  CK(hipDeviceSynchronize());

  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, B, ticks, buf);
  CK(hipEventRecord(ev, B));
  CK(hipStreamWaitEvent(A, ev, 0));
  report("after waiting on another stream's pending event", launches(A, buf));
  report("  ... a third stream meanwhile", launches(C, buf));
  report("  ... the other (waited-on) stream meanwhile", launches(B, buf));
  CK(hipDeviceSynchronize());
  report("  ... the waiting stream once everything drained", launches(A, buf));

  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, B, ticks / 100, buf);
  CK(hipEventRecord(ev, B));
  CK(hipEventSynchronize(ev));
  CK(hipStreamWaitEvent(A, ev, 0));
  report("after waiting on a completed event", launches(A, buf));
  CK(hipDeviceSynchronize());

  // the waiting stream has its own long work queued before the wait
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, A, ticks, buf);
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, B, ticks / 2, buf);
  CK(hipEventRecord(ev, B));
  CK(hipStreamWaitEvent(A, ev, 0));
  report("own 5 ms kernel, then a wait on a 2.5 ms kernel elsewhere", launches(A, buf));
  CK(hipDeviceSynchronize());

  // fork / join like the engine's sub-batch pipeline, then more launches
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, A, ticks / 5, buf);
  CK(hipEventRecord(ev, A));
  CK(hipStreamWaitEvent(B, ev, 0));
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, A, ticks, buf);
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, B, ticks, buf);
  hipEvent_t join;
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventRecord(join, B));
  CK(hipStreamWaitEvent(A, join, 0));
  report("fork/join (engine sub-batches), then launches on the joined stream", launches(A, buf));
  CK(hipDeviceSynchronize());

  // the join done by a marker kernel on the other stream instead: B records,
  // A launches its next kernels only after a host-side wait (not used:
  // reference point) -- and the join through a tiny kernel on A behind the wait
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, A, ticks, buf);
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, B, ticks, buf);
  CK(hipEventRecord(join, B));
  CK(hipStreamWaitEvent(A, join, 0));
  hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, A, buf, 0);
  report("join, one launch, then launches", launches(A, buf));
  CK(hipDeviceSynchronize());
  // every CU busy: many spinning workgroups on B, launches on A
  hipLaunchKernelGGL(spin_kernel, dim3(8192), dim3(256), 0, B, ticks, buf);
  report("all CUs busy with spinning workgroups on another stream", launches(A, buf));
  CK(hipDeviceSynchronize());
  // HBM saturated: 2 GiB copies on B (about 0.5 ms each), launches on A
  const size_t n4 = (size_t(1) << 31) / 16;
  float4 *x = nullptr, *y = nullptr;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&y, n4 * 16));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, B, x, y, n4);
  report("HBM-bound copies running on another stream", launches(A, buf));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, A, x, y, n4);
  report("HBM-bound copies queued on the same stream", launches(A, buf));
  CK(hipDeviceSynchronize());
  // the engine's pattern: copies on A and B, then A joins B, then launches
  for (int i = 0; i < 10; ++i) {
    hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, A, x, y, n4);
    hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, B, x, y, n4);
  }
  CK(hipEventRecord(join, B));
  CK(hipStreamWaitEvent(A, join, 0));
  report("HBM-bound copies on both, A joined B, then launches on A", launches(A, buf));
  CK(hipDeviceSynchronize());
  std::printf("DONE\n");
  return 0;
}
