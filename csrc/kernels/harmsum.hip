// Search hot path: interbinned+normalised spectra for a batch of acceleration
// trials, then a fused incoherent harmonic sum + threshold + wave-aggregated
// compaction.
//
// Reference: src/kernels.cu:33-99 (K1 harmonic_sum_kernel, writes up to five
// full summed spectra through a float** table), :231-252 (K3 interbin),
// :469-494 (K4 normalise), :384-416 (K7 thrust::copy_if + D2H per spectrum),
// include/transforms/peakfinder.hpp:77-94 (per-level bounds).  Here the
// summed spectra are never materialised: each level is thresholded in
// registers and only (trial, level, bin, S/N) records are appended.
//
// Numerics reproduce the reference exactly: the gather index
// (int)(i*m/2^h + 0.5) is computed as (i*m + 2^(h-1)) >> h, additions follow
// the reference order (level 2 adds 3/4 before 1/4), and each level is scaled
// by the double constant rsqrt(2^h) before rounding to float.
#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

__constant__ double c_level_scale[6] = {1.0, 0.70710678118654752440, 0.5, 0.35355339059327376220, 0.25,
                                        0.17677669529663688110};

__global__ void __launch_bounds__(256) interbin_normalise_batch_kernel(const float2* __restrict__ X,
                                                                       uint64_t xstride, float* __restrict__ P,
                                                                       uint64_t pstride, uint64_t nbins_out,
                                                                       const float* __restrict__ stats,
                                                                       float nscale) {
  const int k = blockIdx.y;
  const float2* x = X + static_cast<uint64_t>(k) * xstride;
  float* p = P + static_cast<uint64_t>(k) * pstride;
  const float mean = stats[0] * nscale;
  const float sigma = stats[2] * nscale;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins_out; i += stride) {
    float2 xl = i > 0 ? x[i - 1] : make_float2(0.f, 0.f);
    float v = dev::interbin(x[i], xl);
    v -= mean;
    v /= sigma;
    p[i] = v;
  }
}

// Real-input FFT recovered from an M = N/2 point complex FFT of the packed
// series z[m] = x[2m] + i x[2m+1]:
//   X[k] = (Z[k] + conj Z[M-k])/2 - i/2 e^{-2 pi i k/N} (Z[k] - conj Z[M-k]),  k = 0..M
// (indices mod M); za = Z[k mod M], zb = Z[(M-k) mod M].  Replaces rocFFT's
// separate r2c post-processing pass.
__device__ __forceinline__ float2 r2c_combine(float2 za, float2 zb, uint64_t k, uint64_t M) {
  const float ex = 0.5f * (za.x + zb.x), ey = 0.5f * (za.y - zb.y);
  const float dx = 0.5f * (za.x - zb.x), dy = 0.5f * (za.y + zb.y);
  const float ox = dy, oy = -dx;  // -i * d
  float s, c;
  sincospif(-static_cast<float>(k) / static_cast<float>(M), &s, &c);
  return make_float2(ex + c * ox - s * oy, ey + c * oy + s * ox);
}

__device__ __forceinline__ uint64_t zaddr(uint64_t k, int log2_row, uint64_t pitch) {
  return (k >> log2_row) * pitch + (k & ((uint64_t(1) << log2_row) - 1));
}

// One workgroup per tile of 256 bins k in [k0, k0+256), k <= M/2: both the
// ascending bins k and their mirrors M-k come from the same loads
// Z[k], Z[M-k]; one halo bin each side feeds the interbin neighbour.
__global__ void __launch_bounds__(256) r2c_interbin_normalise_batch_kernel(
    const float2* __restrict__ Z, uint64_t M, uint64_t zstride, int log2_row, uint64_t pitch, float* __restrict__ P,
    uint64_t pstride, uint64_t nbins_out, const float* __restrict__ stats, float nscale) {
  __shared__ float2 A[258];  // A[u] = X[k0 - 1 + u]
  __shared__ float2 D[258];  // D[u] = X[M - (k0 - 1 + u)]
  const int kk = blockIdx.y;
  const int t = threadIdx.x;
  const float2* z = Z + static_cast<uint64_t>(kk) * zstride;
  float* p = P + static_cast<uint64_t>(kk) * pstride;
  const float mean = stats[0] * nscale;
  const float sigma = stats[2] * nscale;
  const uint64_t half = M / 2;
  auto pair = [&](int64_t k, int u) {
    if (k < 0 || static_cast<uint64_t>(k) > half + 1) {
      A[u] = D[u] = make_float2(0.f, 0.f);
      return;
    }
    const uint64_t uk = static_cast<uint64_t>(k);
    const uint64_t a = uk & (M - 1), b = (M - uk) & (M - 1);
    const float2 za = z[zaddr(a, log2_row, pitch)], zb = z[zaddr(b, log2_row, pitch)];
    A[u] = r2c_combine(za, zb, uk, M);
    D[u] = r2c_combine(zb, za, M - uk, M);
  };
  for (uint64_t k0 = static_cast<uint64_t>(blockIdx.x) * 256; k0 <= half;
       k0 += static_cast<uint64_t>(gridDim.x) * 256) {
    pair(static_cast<int64_t>(k0 + t), t + 1);
    if (t == 0) pair(static_cast<int64_t>(k0) - 1, 0);
    if (t == 1) pair(static_cast<int64_t>(k0 + 256), 257);
    __syncthreads();
    const uint64_t k = k0 + t;
    if (k <= half) {
      if (k < nbins_out) {
        const float2 xl = k > 0 ? A[t] : make_float2(0.f, 0.f);
        p[k] = (dev::interbin(A[t + 1], xl) - mean) / sigma;
      }
      const uint64_t j = M - k;  // mirrored bin (> M/2), neighbour X[j-1] = D[t+2]
      if (j > half && j < nbins_out) p[j] = (dev::interbin(D[t + 1], D[t + 2]) - mean) / sigma;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void emit(bool pred, uint32_t seg, int idx, float snr, PeakRecord* __restrict__ out,
                                     uint32_t* __restrict__ count, uint32_t capacity) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0ull) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll(static_cast<long long>(mask)) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(count, static_cast<uint32_t>(__popcll(mask)));
  base = __shfl(base, leader, 64);
  if (pred) {
    const unsigned long long lt = (lane == 0) ? 0ull : (mask & ((1ull << lane) - 1ull));
    const uint32_t pos = base + static_cast<uint32_t>(__popcll(lt));
    if (pos < capacity) out[pos] = PeakRecord{seg, idx, snr};
  }
}

template <int NLEV>
__global__ void __launch_bounds__(256) harmonic_peaks_kernel(const float* __restrict__ P, uint64_t pstride,
                                                             int lo, int hi, HarmParams hp,
                                                             PeakRecord* __restrict__ out,
                                                             uint32_t* __restrict__ count) {
  const int k = blockIdx.y;
  const float* p = P + static_cast<uint64_t>(k) * pstride;
  const float thr = hp.thresh;
  const uint32_t seg0 = static_cast<uint32_t>(k) * 8u;
  const int stride = gridDim.x * blockDim.x;
  for (int base = lo + blockIdx.x * blockDim.x; base < hi; base += stride) {
    const int i = base + threadIdx.x;
    const bool valid = i < hi;
    const int ii = valid ? i : lo;
    float val = p[ii];
    emit(valid && ii >= hp.start[0] && ii < hp.end[0] && val > thr, seg0, ii, val, out, count, hp.capacity);
    if constexpr (NLEV >= 1) {
      const long long li = ii;
      val += p[(li + 1) >> 1];
      float o = static_cast<float>(static_cast<double>(val) * c_level_scale[1]);
      emit(valid && ii >= hp.start[1] && ii < hp.end[1] && o > thr, seg0 + 1, ii, o, out, count, hp.capacity);
    }
    if constexpr (NLEV >= 2) {
      const long long li = ii;
      val += p[(li * 3 + 2) >> 2];
      val += p[(li * 1 + 2) >> 2];
      float o = static_cast<float>(static_cast<double>(val) * c_level_scale[2]);
      emit(valid && ii >= hp.start[2] && ii < hp.end[2] && o > thr, seg0 + 2, ii, o, out, count, hp.capacity);
    }
    if constexpr (NLEV >= 3) {
      const long long li = ii;
#pragma unroll
      for (int m = 1; m < 8; m += 2) val += p[(li * m + 4) >> 3];
      float o = static_cast<float>(static_cast<double>(val) * c_level_scale[3]);
      emit(valid && ii >= hp.start[3] && ii < hp.end[3] && o > thr, seg0 + 3, ii, o, out, count, hp.capacity);
    }
    if constexpr (NLEV >= 4) {
      const long long li = ii;
#pragma unroll
      for (int m = 1; m < 16; m += 2) val += p[(li * m + 8) >> 4];
      float o = static_cast<float>(static_cast<double>(val) * c_level_scale[4]);
      emit(valid && ii >= hp.start[4] && ii < hp.end[4] && o > thr, seg0 + 4, ii, o, out, count, hp.capacity);
    }
    if constexpr (NLEV >= 5) {
      const long long li = ii;
#pragma unroll
      for (int m = 1; m < 32; m += 2) val += p[(li * m + 16) >> 5];
      float o = static_cast<float>(static_cast<double>(val) * c_level_scale[5]);
      emit(valid && ii >= hp.start[5] && ii < hp.end[5] && o > thr, seg0 + 5, ii, o, out, count, hp.capacity);
    }
  }
}

__global__ void __launch_bounds__(256) harmonic_sums_kernel(const float* __restrict__ p, uint64_t nbins,
                                                            int nlevels, float* __restrict__ out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins; i += stride) {
    const long long li = static_cast<long long>(i);
    float val = p[i];
    if (nlevels > 0) {
      val += p[(li + 1) >> 1];
      out[i] = static_cast<float>(static_cast<double>(val) * c_level_scale[1]);
    }
    if (nlevels > 1) {
      val += p[(li * 3 + 2) >> 2];
      val += p[(li + 2) >> 2];
      out[nbins + i] = static_cast<float>(static_cast<double>(val) * c_level_scale[2]);
    }
    for (int h = 3; h <= nlevels && h <= 5; ++h) {
      const int den = 1 << h;
      for (int m = 1; m < den; m += 2) val += p[(li * m + den / 2) >> h];
      out[static_cast<uint64_t>(h - 1) * nbins + i] = static_cast<float>(static_cast<double>(val) * c_level_scale[h]);
    }
  }
}

}  // namespace

void interbin_normalise_batch(const float2* X, uint64_t nbins, uint64_t xstride, float* P, uint64_t pstride,
                              int K, uint64_t nbins_out, const float* stats, float nscale, hipStream_t s) {
  (void)nbins;
  PSOUP_CHECK(K >= 1 && K <= 65535, "bad batch");
  if (nbins_out == 0) return;
  dim3 grid(dev::grid_for(nbins_out, 256, 1024), static_cast<unsigned>(K));
  interbin_normalise_batch_kernel<<<grid, 256, 0, s>>>(X, xstride, P, pstride, nbins_out, stats, nscale);
  post_launch_check("interbin_normalise_batch_kernel", s);
}

void r2c_interbin_normalise_batch(const float2* Z, uint64_t M, uint64_t zstride, int log2_row, uint64_t row_pitch,
                                  float* P, uint64_t pstride, int K, uint64_t nbins_out, const float* stats,
                                  float nscale, hipStream_t s) {
  PSOUP_CHECK(K >= 1 && K <= 65535, "bad batch");
  PSOUP_CHECK(M >= 2 && (M & (M - 1)) == 0, "r2c: M must be a power of two");
  PSOUP_CHECK(nbins_out <= M + 1, "nbins_out beyond the spectrum");
  PSOUP_CHECK(log2_row >= 0 && log2_row < 63 && (uint64_t(1) << log2_row) <= M, "r2c: bad row layout");
  if (nbins_out == 0) return;
  dim3 grid(dev::grid_for(M / 2 + 1, 256, 2048), static_cast<unsigned>(K));
  r2c_interbin_normalise_batch_kernel<<<grid, 256, 0, s>>>(Z, M, zstride, log2_row, row_pitch, P, pstride, nbins_out,
                                                           stats, nscale);
  post_launch_check("r2c_interbin_normalise_batch_kernel", s);
}

void harmonic_peaks_batch(const float* P, uint64_t nbins, uint64_t pstride, int K, const HarmParams& hp,
                          PeakRecord* out, uint32_t* count, hipStream_t s) {
  PSOUP_CHECK(hp.nlevels >= 0 && hp.nlevels <= kMaxHarmLevels, "nlevels out of range");
  PSOUP_CHECK(nbins < (1ull << 31), "spectrum too long for int32 indices");
  int lo = static_cast<int>(nbins), hi = 0;
  for (int h = 0; h <= hp.nlevels; ++h) {
    if (hp.end[h] > hp.start[h]) {
      lo = std::min(lo, hp.start[h]);
      hi = std::max(hi, hp.end[h]);
    }
  }
  PSOUP_CHECK(hi <= static_cast<int>(nbins), "search range beyond spectrum");
  if (hi <= lo) return;
  dim3 grid(dev::grid_for(static_cast<uint64_t>(hi - lo), 256, 1024), static_cast<unsigned>(K));
  switch (hp.nlevels) {
    case 0: harmonic_peaks_kernel<0><<<grid, 256, 0, s>>>(P, pstride, lo, hi, hp, out, count); break;
    case 1: harmonic_peaks_kernel<1><<<grid, 256, 0, s>>>(P, pstride, lo, hi, hp, out, count); break;
    case 2: harmonic_peaks_kernel<2><<<grid, 256, 0, s>>>(P, pstride, lo, hi, hp, out, count); break;
    case 3: harmonic_peaks_kernel<3><<<grid, 256, 0, s>>>(P, pstride, lo, hi, hp, out, count); break;
    case 4: harmonic_peaks_kernel<4><<<grid, 256, 0, s>>>(P, pstride, lo, hi, hp, out, count); break;
    default: harmonic_peaks_kernel<5><<<grid, 256, 0, s>>>(P, pstride, lo, hi, hp, out, count); break;
  }
  post_launch_check("harmonic_peaks_kernel", s);
}

void harmonic_sums(const float* P, uint64_t nbins, int nlevels, float* out, hipStream_t s) {
  harmonic_sums_kernel<<<dev::grid_for(nbins, 256), 256, 0, s>>>(P, nbins, nlevels, out);
  post_launch_check("harmonic_sums_kernel", s);
}

}  // namespace kern
}  // namespace psoup
