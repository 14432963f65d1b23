// Time-series kernels: u8 trial -> f32 with mean padding, f32 statistics.
// Replaces K29 conversion_kernel + K9 GPU_mean + K10 GPU_fill
// (src/kernels.cu:440-463, 1144-1170): one exact integer reduction and one
// fused convert+pad pass, with the mean read on the device (no D2H scalar).
#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

__global__ void __launch_bounds__(256) u8_sum_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                     unsigned long long* __restrict__ sum, uint64_t in_stride) {
  in += blockIdx.y * in_stride;
  sum += blockIdx.y;
  __shared__ unsigned long long scratch[4];
  unsigned long long acc = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t nvec = n / 16;
  const uint4* in4 = reinterpret_cast<const uint4*>(in);
  const bool aligned = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  if (aligned) {
    for (uint64_t v = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; v < nvec; v += stride) {
      uint4 w = in4[v];
      uint32_t words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t x = words[q];
        // byte-sum of a dword via two 16-bit lanes
        uint32_t pairs = (x & 0x00FF00FFu) + ((x >> 8) & 0x00FF00FFu);
        acc += (pairs & 0xFFFFu) + (pairs >> 16);
      }
    }
    for (uint64_t i = nvec * 16 + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
      acc += in[i];
  } else {
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) acc += in[i];
  }
  acc = dev::block_sum(acc, scratch);
  if (threadIdx.x == 0) atomicAdd(sum, acc);
}

__global__ void __launch_bounds__(256) u8_to_f32_pad_kernel(const uint8_t* __restrict__ in, uint64_t nvalid,
                                                            float* __restrict__ out, uint64_t n,
                                                            const unsigned long long* __restrict__ sum,
                                                            uint64_t in_stride, uint64_t out_stride) {
  in += blockIdx.y * in_stride;
  out += blockIdx.y * out_stride;
  sum += blockIdx.y;
  const float mean = nvalid ? static_cast<float>(static_cast<double>(*sum) / static_cast<double>(nvalid)) : 0.f;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  // 4 samples per thread per step
  const uint64_t n4 = n / 4;
  const bool aligned4 = (reinterpret_cast<uintptr_t>(in) & 3) == 0;
  for (uint64_t v = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; v < n4; v += stride) {
    uint64_t i = v * 4;
    float4 r;
    if (i + 4 <= nvalid && aligned4) {
      const uchar4 b = *reinterpret_cast<const uchar4*>(in + i);  // one dword load
      r = make_float4(b.x, b.y, b.z, b.w);
    } else if (i + 4 <= nvalid) {
      r.x = in[i];
      r.y = in[i + 1];
      r.z = in[i + 2];
      r.w = in[i + 3];
    } else {
      r.x = (i < nvalid) ? static_cast<float>(in[i]) : mean;
      r.y = (i + 1 < nvalid) ? static_cast<float>(in[i + 1]) : mean;
      r.z = (i + 2 < nvalid) ? static_cast<float>(in[i + 2]) : mean;
      r.w = (i + 3 < nvalid) ? static_cast<float>(in[i + 3]) : mean;
    }
    reinterpret_cast<float4*>(out)[v] = r;
  }
  for (uint64_t i = n4 * 4 + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    out[i] = i < nvalid ? static_cast<float>(in[i]) : mean;
}

// Partial sums of x and x^2 (double) -> partials[2*block]
__global__ void __launch_bounds__(256) f32_moments_kernel(const float* __restrict__ x, uint64_t n,
                                                          double* __restrict__ partials) {
  __shared__ double scratch[4];
  double s = 0.0, s2 = 0.0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    double v = x[i];
    s += v;
    s2 += v * v;
  }
  s = dev::block_sum(s, scratch);
  s2 = dev::block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = s;
    partials[2 * blockIdx.x + 1] = s2;
  }
}

}  // namespace

// Final reduction shared with spectrum.hip: stats = {mean, rms, std} as the
// reference's stats::stats (float mean/rms, std = sqrt(rms^2 - mean^2)).
__global__ void __launch_bounds__(256) stats_finalize_kernel(const double* __restrict__ partials, int npart,
                                                             uint64_t n, float* __restrict__ stats, int pstride) {
  __shared__ double scratch[4];
  partials += static_cast<uint64_t>(blockIdx.x) * pstride;  // batch item blockIdx.x
  stats += 4 * blockIdx.x;
  double s = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < npart; i += blockDim.x) {
    s += partials[2 * i];
    s2 += partials[2 * i + 1];
  }
  s = dev::block_sum(s, scratch);
  s2 = dev::block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    float fs = static_cast<float>(s), fs2 = static_cast<float>(s2), fn = static_cast<float>(n);
    float mean = fs / fn;
    float rms = sqrtf(fs2 / fn);
    float var = rms * rms - mean * mean;
    stats[0] = mean;
    stats[1] = rms;
    stats[2] = sqrtf(fmaxf(var, 0.f));
  }
}

void u8_sum(const uint8_t* in, uint64_t n, unsigned long long* sum, hipStream_t s, int count, uint64_t in_stride) {
  PSOUP_CHECK(count >= 1 && count <= 65535, "u8_sum: bad count");
  PSOUP_HIP_CHECK(hipMemsetAsync(sum, 0, sizeof(unsigned long long) * count, s));
  if (n == 0) return;
  // few blocks per series: every block ends in one 64-bit atomic on the
  // series' sum, and 256 of them on one address serialise (57 us for ten
  // 2^20 series in the config-4 trace)
  const dim3 grid(dev::grid_for(n / 16 + 1, 256, count > 1 ? 32 : 1024), static_cast<unsigned>(count));
  u8_sum_kernel<<<grid, 256, 0, s>>>(in, n, sum, in_stride);
  post_launch_check("u8_sum_kernel", s);
}

void u8_to_f32_pad(const uint8_t* in, uint64_t nvalid, float* out, uint64_t n, const unsigned long long* sum,
                   hipStream_t s, int count, uint64_t in_stride, uint64_t out_stride) {
  PSOUP_CHECK((reinterpret_cast<uintptr_t>(out) & 15) == 0 && out_stride % 4 == 0, "output must be 16-byte aligned");
  PSOUP_CHECK(count >= 1 && count <= 65535, "u8_to_f32_pad: bad count");
  const dim3 grid(dev::grid_for(n / 4 + 1, 256, count > 1 ? 1024 : 2048), static_cast<unsigned>(count));
  u8_to_f32_pad_kernel<<<grid, 256, 0, s>>>(in, nvalid, out, n, sum, in_stride, out_stride);
  post_launch_check("u8_to_f32_pad_kernel", s);
}

void f32_stats(const float* x, uint64_t n, double* partials, int npartials, float* stats_out, hipStream_t s) {
  PSOUP_CHECK(npartials >= 1, "need partial buffer");
  unsigned grid = dev::grid_for(n, 256, static_cast<unsigned>(npartials));
  f32_moments_kernel<<<grid, 256, 0, s>>>(x, n, partials);
  post_launch_check("f32_moments_kernel", s);
  stats_finalize_kernel<<<1, 256, 0, s>>>(partials, static_cast<int>(grid), n, stats_out, 0);
  post_launch_check("stats_finalize_kernel", s);
}

}  // namespace kern
}  // namespace psoup
