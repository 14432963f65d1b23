// Spectrum formation and running-median whitening.
// Reference: src/kernels.cu:215-252 (K2 amplitude, K3 interbin), :469-494 (K4
// normalise), :875-1034 (K22 median_scrunch5, K23 linear_stretch, K24
// divide_c_by_f), :1036-1069 (K25 zap), include/transforms/dereddener.hpp:
// 44-66 (piecewise median assembly).  Here the stretch + piecewise select +
// complex divide + zap is ONE pass (deredden_zap) and the interbin spectrum
// is formed together with its mean/rms partial sums (interbin_stats).
#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

__global__ void stats_finalize_kernel(const double* __restrict__ partials, int npart, uint64_t n,
                                      float* __restrict__ stats, int pstride);

namespace {

__global__ void __launch_bounds__(256) form_amplitude_kernel(const float2* __restrict__ X, uint64_t nbins,
                                                             float* __restrict__ out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins; i += stride)
    out[i] = dev::amplitude(X[i]);
}

__global__ void __launch_bounds__(256) form_interbin_kernel(const float2* __restrict__ X, uint64_t nbins,
                                                            float* __restrict__ out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins; i += stride) {
    float2 xl = i > 0 ? X[i - 1] : make_float2(0.f, 0.f);
    out[i] = dev::interbin(X[i], xl);
  }
}

__global__ void __launch_bounds__(256) normalise_kernel(float* __restrict__ x, uint64_t n, float mean,
                                                        float sigma) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    v -= mean;
    v /= sigma;
    x[i] = v;
  }
}

__global__ void __launch_bounds__(256) normalise_dev_kernel(float* __restrict__ x, uint64_t n,
                                                            const float* __restrict__ stats, float scale) {
  const float mean = stats[0] * scale;
  const float sigma = stats[2] * scale;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    v -= mean;
    v /= sigma;
    x[i] = v;
  }
}

__global__ void __launch_bounds__(256) median5_amp_kernel(const float2* __restrict__ X, uint64_t nout,
                                                          float* __restrict__ out, uint64_t xstride,
                                                          uint64_t ostride) {
  X += blockIdx.y * xstride;
  out += blockIdx.y * ostride;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nout; i += stride) {
    const float2* p = X + 5 * i;
    out[i] = dev::median5(dev::amplitude(p[0]), dev::amplitude(p[1]), dev::amplitude(p[2]),
                          dev::amplitude(p[3]), dev::amplitude(p[4]));
  }
}

__global__ void __launch_bounds__(256) median5_kernel(const float* __restrict__ in, uint64_t nout,
                                                      float* __restrict__ out, uint64_t istride, uint64_t ostride) {
  in += blockIdx.y * istride;
  out += blockIdx.y * ostride;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nout; i += stride) {
    const float* p = in + 5 * i;
    out[i] = dev::median5(p[0], p[1], p[2], p[3], p[4]);
  }
}

__global__ void median_small_kernel(const float* __restrict__ in, int count, float* __restrict__ out,
                                    uint64_t istride, uint64_t ostride) {
  if (threadIdx.x != 0) return;
  in += blockIdx.x * istride;
  out += blockIdx.x * ostride;
  float r;
  if (count == 1) r = in[0];
  else if (count == 2) r = 0.5f * (in[0] + in[1]);
  else if (count == 3) r = dev::median3(in[0], in[1], in[2]);
  else r = dev::median4(in[0], in[1], in[2], in[3]);
  out[0] = r;
}

// linear_stretch_functor (kernels.cu:983-999) evaluated at output index i
__device__ __forceinline__ float stretch_at(const float* __restrict__ in, uint64_t in_count, float step,
                                            uint64_t i) {
  float x = static_cast<float>(static_cast<unsigned>(i)) * step;
  unsigned j = static_cast<unsigned>(x);
  if (j >= in_count) j = static_cast<unsigned>(in_count - 1);
  float frac = x - static_cast<float>(j);
  float a = in[j];
  if (frac > 1e-5f && j + 1 < in_count) return a + frac * (in[j + 1] - a);
  return a;
}

__global__ void __launch_bounds__(256) deredden_zap_kernel(float2* __restrict__ X, uint64_t nbins,
                                                           const float* __restrict__ m5, uint64_t n5, float step5,
                                                           const float* __restrict__ m25, uint64_t n25,
                                                           float step25, const float* __restrict__ m125,
                                                           uint64_t n125, float step125, int64_t pos5,
                                                           int64_t pos25, const uint32_t* __restrict__ zapmask,
                                                           uint64_t xstride, uint64_t mstride) {
  X += blockIdx.y * xstride;  // batch item blockIdx.y: its spectrum and medians
  m5 += blockIdx.y * mstride;
  m25 += blockIdx.y * mstride;
  m125 += blockIdx.y * mstride;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t k = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; k < nbins; k += stride) {
    float2 x;
    if (k < 5) {
      x = make_float2(0.f, 0.f);
    } else {
      float med;
      if (static_cast<int64_t>(k) >= pos25) med = stretch_at(m125, n125, step125, k);
      else if (static_cast<int64_t>(k) >= pos5) med = stretch_at(m25, n25, step25, k);
      else med = stretch_at(m5, n5, step5, k);
      x = dev::cdiv_real(X[k], med);
    }
    if (zapmask && ((zapmask[k >> 5] >> (k & 31)) & 1u)) x = make_float2(1.f, 0.f);
    X[k] = x;
  }
}

__global__ void __launch_bounds__(256) interbin_moments_kernel(const float2* __restrict__ X, uint64_t nbins,
                                                               float* __restrict__ P,
                                                               double* __restrict__ partials, uint64_t xstride,
                                                               int pstride) {
  __shared__ double scratch[4];
  X += blockIdx.y * xstride;
  partials += static_cast<uint64_t>(blockIdx.y) * pstride;
  double s = 0.0, s2 = 0.0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins; i += stride) {
    float2 xl = i > 0 ? X[i - 1] : make_float2(0.f, 0.f);
    float v = dev::interbin(X[i], xl);
    if (P) P[i] = v;
    s += v;
    s2 += static_cast<double>(v) * v;
  }
  s = dev::block_sum(s, scratch);
  s2 = dev::block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = s;
    partials[2 * blockIdx.x + 1] = s2;
  }
}

// deredden_zap and interbin_moments in one pass, out of place: item b's
// spectrum X -> out (dereddened, zapped), with the interbin partial sums of
// out over the same grid and loop order as interbin_moments_kernel (so the
// statistics are bit-identical).  The left neighbour is dereddened again from
// X rather than read back from out, which other workgroups write.
__global__ void __launch_bounds__(256) deredden_zap_moments_kernel(
    const float2* __restrict__ X, float2* __restrict__ out, uint64_t nbins, const float* __restrict__ m5, uint64_t n5,
    float step5, const float* __restrict__ m25, uint64_t n25, float step25, const float* __restrict__ m125,
    uint64_t n125, float step125, int64_t pos5, int64_t pos25, const uint32_t* __restrict__ zapmask, uint64_t xstride,
    uint64_t ostride, uint64_t mstride, double* __restrict__ partials, int pstride) {
  __shared__ double scratch[4];
  X += blockIdx.y * xstride;
  out += blockIdx.y * ostride;
  m5 += blockIdx.y * mstride;
  m25 += blockIdx.y * mstride;
  m125 += blockIdx.y * mstride;
  partials += static_cast<uint64_t>(blockIdx.y) * pstride;
  auto dz = [&](uint64_t k) {  // deredden_zap_kernel's value of bin k
    float2 x;
    if (k < 5) {
      x = make_float2(0.f, 0.f);
    } else {
      float med;
      if (static_cast<int64_t>(k) >= pos25) med = stretch_at(m125, n125, step125, k);
      else if (static_cast<int64_t>(k) >= pos5) med = stretch_at(m25, n25, step25, k);
      else med = stretch_at(m5, n5, step5, k);
      x = dev::cdiv_real(X[k], med);
    }
    if (zapmask && ((zapmask[k >> 5] >> (k & 31)) & 1u)) x = make_float2(1.f, 0.f);
    return x;
  };
  double s = 0.0, s2 = 0.0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins; i += stride) {
    const float2 x = dz(i);
    out[i] = x;
    const float2 xl = i > 0 ? dz(i - 1) : make_float2(0.f, 0.f);
    const float v = dev::interbin(x, xl);
    s += v;
    s2 += static_cast<double>(v) * v;
  }
  s = dev::block_sum(s, scratch);
  s2 = dev::block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = s;
    partials[2 * blockIdx.x + 1] = s2;
  }
}

float stretch_step(uint64_t in_count, uint64_t out_count) {
  if (out_count <= 1 || in_count == 0) return 0.f;
  return static_cast<float>(in_count - 1) / static_cast<float>(out_count - 1);
}

}  // namespace

void form_amplitude(const float2* X, uint64_t nbins, float* out, hipStream_t s) {
  form_amplitude_kernel<<<dev::grid_for(nbins, 256), 256, 0, s>>>(X, nbins, out);
  post_launch_check("form_amplitude_kernel", s);
}

void form_interbin(const float2* X, uint64_t nbins, float* out, hipStream_t s) {
  form_interbin_kernel<<<dev::grid_for(nbins, 256), 256, 0, s>>>(X, nbins, out);
  post_launch_check("form_interbin_kernel", s);
}

void normalise(float* x, uint64_t n, float mean, float sigma, hipStream_t s) {
  normalise_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(x, n, mean, sigma);
  post_launch_check("normalise_kernel", s);
}

void normalise_dev(float* x, uint64_t n, const float* stats, float scale, hipStream_t s) {
  normalise_dev_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(x, n, stats, scale);
  post_launch_check("normalise_dev_kernel", s);
}

void median5_amp(const float2* X, uint64_t nbins, float* out, hipStream_t s, int batch, uint64_t xstride,
                 uint64_t ostride) {
  uint64_t nout = nbins / 5;
  if (nout == 0) PSOUP_THROW("median5_amp needs >= 5 bins");
  PSOUP_CHECK(batch >= 1 && batch <= 65535, "median5_amp: bad batch");
  const dim3 grid(dev::grid_for(nout, 256, batch > 1 ? 512 : 2048), static_cast<unsigned>(batch));
  median5_amp_kernel<<<grid, 256, 0, s>>>(X, nout, out, xstride, ostride);
  post_launch_check("median5_amp_kernel", s);
}

void median5(const float* in, uint64_t count, float* out, hipStream_t s, int batch, uint64_t istride,
             uint64_t ostride) {
  if (count == 0) return;
  PSOUP_CHECK(batch >= 1 && batch <= 65535, "median5: bad batch");
  if (count < 5) {
    median_small_kernel<<<static_cast<unsigned>(batch), 64, 0, s>>>(in, static_cast<int>(count), out, istride,
                                                                     ostride);
    post_launch_check("median_small_kernel", s);
    return;
  }
  uint64_t nout = count / 5;
  const dim3 grid(dev::grid_for(nout, 256, batch > 1 ? 512 : 2048), static_cast<unsigned>(batch));
  median5_kernel<<<grid, 256, 0, s>>>(in, nout, out, istride, ostride);
  post_launch_check("median5_kernel", s);
}

void deredden_zap(float2* X, uint64_t nbins, const float* m5, uint64_t n5, const float* m25, uint64_t n25,
                  const float* m125, uint64_t n125, int64_t pos5, int64_t pos25, const uint32_t* zapmask,
                  hipStream_t s, int batch, uint64_t xstride, uint64_t mstride) {
  PSOUP_CHECK(n5 >= 1 && n25 >= 1 && n125 >= 1, "running median needs >= 125 bins");
  PSOUP_CHECK(batch >= 1 && batch <= 65535, "deredden_zap: bad batch");
  const dim3 grid(dev::grid_for(nbins, 256, batch > 1 ? 512 : 2048), static_cast<unsigned>(batch));
  deredden_zap_kernel<<<grid, 256, 0, s>>>(X, nbins, m5, n5, stretch_step(n5, nbins), m25, n25,
                                           stretch_step(n25, nbins), m125, n125, stretch_step(n125, nbins), pos5,
                                           pos25, zapmask, xstride, mstride);
  post_launch_check("deredden_zap_kernel", s);
}

void interbin_stats(const float2* X, uint64_t nbins, float* P, double* partials, int npartials, float* stats,
                    hipStream_t s, int batch, uint64_t xstride) {
  PSOUP_CHECK(batch >= 1 && batch <= 65535 && (batch == 1 || P == nullptr), "interbin_stats: bad batch");
  const unsigned gx = dev::grid_for(nbins, 256, static_cast<unsigned>(npartials));
  interbin_moments_kernel<<<dim3(gx, static_cast<unsigned>(batch)), 256, 0, s>>>(X, nbins, P, partials, xstride,
                                                                                 2 * npartials);
  post_launch_check("interbin_moments_kernel", s);
  stats_finalize_kernel<<<static_cast<unsigned>(batch), 256, 0, s>>>(partials, static_cast<int>(gx), nbins, stats,
                                                                      2 * npartials);
  post_launch_check("stats_finalize_kernel", s);
}

void deredden_zap_stats(const float2* X, float2* out, uint64_t nbins, const float* m5, uint64_t n5, const float* m25,
                        uint64_t n25, const float* m125, uint64_t n125, int64_t pos5, int64_t pos25,
                        const uint32_t* zapmask, double* partials, int npartials, float* stats, hipStream_t s,
                        int batch, uint64_t xstride, uint64_t ostride, uint64_t mstride) {
  PSOUP_CHECK(n5 >= 1 && n25 >= 1 && n125 >= 1, "running median needs >= 125 bins");
  PSOUP_CHECK(batch >= 1 && batch <= 65535 && X != out, "deredden_zap_stats: bad batch / in place");
  const unsigned gx = dev::grid_for(nbins, 256, static_cast<unsigned>(npartials));  // as interbin_stats
  deredden_zap_moments_kernel<<<dim3(gx, static_cast<unsigned>(batch)), 256, 0, s>>>(
      X, out, nbins, m5, n5, stretch_step(n5, nbins), m25, n25, stretch_step(n25, nbins), m125, n125,
      stretch_step(n125, nbins), pos5, pos25, zapmask, xstride, ostride, mstride, partials, 2 * npartials);
  post_launch_check("deredden_zap_moments_kernel", s);
  stats_finalize_kernel<<<static_cast<unsigned>(batch), 256, 0, s>>>(partials, static_cast<int>(gx), nbins, stats,
                                                                      2 * npartials);
  post_launch_check("stats_finalize_kernel", s);
}

}  // namespace kern
}  // namespace psoup
