// Time-domain acceleration resampling.
// Reference: src/kernels.cu:308-379 (K5 resample_kernel, K6 resample_kernelII,
// one launch per acceleration).  Here one launch resamples a whole batch of K
// accelerations (blockIdx.y = trial) so the whitened input series stays
// L2/Infinity-Cache resident while K outputs stream to HBM, and the read
// index is clamped (the reference can read index N for a < 0).
#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

__global__ void __launch_bounds__(256) resample_batch_kernel(const float* __restrict__ in, uint64_t n,
                                                             float* __restrict__ out, uint64_t out_stride,
                                                             const double* __restrict__ afs) {
  const int k = blockIdx.y;
  const double af = afs[k];
  const double size = static_cast<double>(n);
  float* o = out + static_cast<uint64_t>(k) * out_stride;
  const uint64_t n4 = n / 4;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t v = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; v < n4; v += stride) {
    uint64_t i = v * 4;
    float4 r;
    r.x = in[dev::accel_index_ii(af, size, i, n - 1)];
    r.y = in[dev::accel_index_ii(af, size, i + 1, n - 1)];
    r.z = in[dev::accel_index_ii(af, size, i + 2, n - 1)];
    r.w = in[dev::accel_index_ii(af, size, i + 3, n - 1)];
    reinterpret_cast<float4*>(o)[v] = r;
  }
  for (uint64_t i = n4 * 4 + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    o[i] = in[dev::accel_index_ii(af, size, i, n - 1)];
}

__global__ void __launch_bounds__(256) resample_v1_kernel(const float* __restrict__ in, uint64_t n,
                                                          float* __restrict__ out, double af) {
  const double h = static_cast<double>(n) / 2.0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    double d = static_cast<double>(i);
    double r = rint(d + af * (((d - h) * (d - h)) - (h * h)));
    if (r < 0.0) r = 0.0;
    uint64_t j = static_cast<uint64_t>(r);
    if (j > n - 1) j = n - 1;
    out[i] = in[j];
  }
}

}  // namespace

void resample_batch(const float* in, uint64_t n, float* out, uint64_t out_stride, const double* af, int K,
                    hipStream_t s) {
  PSOUP_CHECK(K >= 1 && K <= 65535, "bad batch " << K);
  PSOUP_CHECK(out_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0, "resample output alignment");
  unsigned gx = dev::grid_for(n / 4 + 1, 256, 1024);
  dim3 grid(gx, static_cast<unsigned>(K));
  resample_batch_kernel<<<grid, 256, 0, s>>>(in, n, out, out_stride, af);
  post_launch_check("resample_batch_kernel", s);
}

void resample_v1(const float* in, uint64_t n, float* out, double af, hipStream_t s) {
  resample_v1_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(in, n, out, af);
  post_launch_check("resample_v1_kernel", s);
}

}  // namespace kern
}  // namespace psoup
