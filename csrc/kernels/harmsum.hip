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

#include <climits>
#include <cmath>
#include <type_traits>
#include <vector>
#include <mutex>
#include <map>

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
  const float rsig = 1.0f / sigma;  // one division per thread; per bin dev::div_rn
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nbins_out; i += stride) {
    float2 xl = i > 0 ? x[i - 1] : make_float2(0.f, 0.f);
    float v = dev::interbin(x[i], xl);
    p[i] = dev::div_rn(v - mean, sigma, rsig);
  }
}

// Real-input FFT recovered from an M = N/2 point complex FFT of the packed
// series z[m] = x[2m] + i x[2m+1]:
//   X[k] = (Z[k] + conj Z[M-k])/2 - i/2 e^{-2 pi i k/N} (Z[k] - conj Z[M-k]),  k = 0..M
// (indices mod M); za = Z[k mod M], zb = Z[(M-k) mod M].  Replaces rocFFT's
// separate r2c post-processing pass.
// (c, s) = (cos, sin) of -pi k / M (dev::r2c_combine, shared with the fused
// pass B of fft4step.hip).
using dev::r2c_combine;

// Address of bin k = k2 + 2^log2_row * k1 in a (possibly blocked) layout:
// (k2 >> lw) * blk + k1 * pitch + (k2 & (2^lw - 1)).
__device__ __forceinline__ uint64_t zaddr(uint64_t k, int log2_row, uint64_t pitch, uint64_t blk, int lw) {
  const uint64_t k2 = k & ((uint64_t(1) << log2_row) - 1);
  return (k2 >> lw) * blk + (k >> log2_row) * pitch + (k2 & ((uint64_t(1) << lw) - 1));
}

// One workgroup per tile of 1024 bins k in [k0, k0+1024), k <= M/2, four
// bins per thread 256 apart (so every load instruction reads 64 consecutive
// bins, whatever the spectrum layout): both the ascending bins k and their
// mirrors M-k come from the same pair of loads Z[k], Z[M-k] (all eight loads
// of a thread are issued before any is used); one halo bin each side feeds
// the interbin neighbour.  One sincospi per thread: the twiddles of the other
// three bins are W^k * W^(256u), precomputed per block.
constexpr int kR2cBpt = 4;
constexpr int kR2cTile = 256 * kR2cBpt;

__global__ void __launch_bounds__(256) r2c_interbin_normalise_batch_kernel(
    const float2* __restrict__ Z, uint64_t M, uint64_t zstride, int log2_row, uint64_t pitch, uint64_t blk, int lw,
    float* __restrict__ P, uint64_t pstride, uint64_t nbins_out, const float* __restrict__ stats, float nscale,
    const uint32_t* __restrict__ tsrc) {
  __shared__ float2 A[kR2cTile + 2];  // A[u] = X[k0 - 1 + u]
  __shared__ float2 D[kR2cTile + 2];  // D[u] = X[M - (k0 - 1 + u)]
  const int kk = blockIdx.y;
  const int t = threadIdx.x;
  const float2* z = Z + static_cast<uint64_t>(kk) * zstride;
  float* p = P + static_cast<uint64_t>(kk) * pstride;
  if (tsrc) stats += 4 * tsrc[kk];  // multi-series batch: this trial's whitening stats
  const float mean = stats[0] * nscale;
  const float sigma = stats[2] * nscale;
  const float rsig = 1.0f / sigma;  // one division per thread; per bin dev::div_rn
  const uint64_t half = M / 2;
  const float invM = 1.0f / static_cast<float>(M);  // M a power of two: x * invM == x / M exactly
  float2 wu[kR2cBpt];  // W^(256 u), W = e^{-i pi / M}
#pragma unroll
  for (int u = 0; u < kR2cBpt; ++u)
    sincospif(-static_cast<float>(256 * u) * invM, &wu[u].y, &wu[u].x);
  auto halo = [&](int64_t k, int u) {
    if (k < 0 || static_cast<uint64_t>(k) > half + 1) {
      A[u] = D[u] = make_float2(0.f, 0.f);
      return;
    }
    const uint64_t uk = static_cast<uint64_t>(k);
    const float2 za = z[zaddr(uk & (M - 1), log2_row, pitch, blk, lw)];
    const float2 zb = z[zaddr((M - uk) & (M - 1), log2_row, pitch, blk, lw)];
    float sn, cs;
    sincospif(-static_cast<float>(uk) * invM, &sn, &cs);
    A[u] = r2c_combine(za, zb, cs, sn);
    D[u] = r2c_combine(zb, za, -cs, sn);  // angle -pi (M-k)/M = -pi + pi k/M
  };
  for (uint64_t k0 = static_cast<uint64_t>(blockIdx.x) * kR2cTile; k0 <= half;
       k0 += static_cast<uint64_t>(gridDim.x) * kR2cTile) {
    const uint64_t kb = k0 + static_cast<uint64_t>(t);
    float2 za[kR2cBpt], zb[kR2cBpt];
#pragma unroll
    for (int u = 0; u < kR2cBpt; ++u) {
      const uint64_t k = kb + 256 * u;
      const bool ok = k <= half + 1;
      za[u] = ok ? z[zaddr(k & (M - 1), log2_row, pitch, blk, lw)] : make_float2(0.f, 0.f);
      zb[u] = ok ? z[zaddr((M - k) & (M - 1), log2_row, pitch, blk, lw)] : make_float2(0.f, 0.f);
    }
    if (t == 0) halo(static_cast<int64_t>(k0) - 1, 0);
    if (t == 1) halo(static_cast<int64_t>(k0 + kR2cTile), kR2cTile + 1);
    float sn, cs;
    sincospif(-static_cast<float>(kb) * invM, &sn, &cs);
#pragma unroll
    for (int u = 0; u < kR2cBpt; ++u) {
      const float c = cs * wu[u].x - sn * wu[u].y, s = cs * wu[u].y + sn * wu[u].x;  // W^(kb+256u)
      const int slot = t + 256 * u + 1;
      A[slot] = r2c_combine(za[u], zb[u], c, s);
      D[slot] = r2c_combine(zb[u], za[u], -c, s);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kR2cBpt; ++u) {
      const uint64_t k = kb + 256 * u;
      const int slot = t + 256 * u + 1;
      if (k <= half) {
        if (k < nbins_out) {
          const float2 xl = k > 0 ? A[slot - 1] : make_float2(0.f, 0.f);
          p[k] = dev::div_rn(dev::interbin(A[slot], xl) - mean, sigma, rsig);
        }
        const uint64_t j = M - k;  // mirrored bin (> M/2), neighbour X[j-1] = D[slot+1]
        if (j > half && j < nbins_out) p[j] = dev::div_rn(dev::interbin(D[slot], D[slot + 1]) - mean, sigma, rsig);
      }
    }
    __syncthreads();
  }
}

// The same from a row-major half spectrum Zr[k2 * zp + k1] = Z[k2 + n2 k1]
// (the rocFFT row pass of the long-series four-step FFT writes each row's
// transform contiguously): a workgroup takes a tile of 32 k2 x 64 k1 with
// k1 < n1/2, loads rows r0 - 1 .. r0 + 32 of it and the mirror rows (each
// wave instruction one contiguous 512-byte row piece), forms X[k] and
// X[M - k] of every loaded bin into LDS, and writes P[k] (32 consecutive k
// per k1) and P[M - k] -- the transpose happens in LDS, every global access
// is a whole row piece.  Bins k < M/2 and their mirrors (M/2, M]; bin M/2 by
// block (0, 0).
// (128 rows: one workgroup writes whole 128-byte Q lines and 512-byte P
// runs; 32 rows x 64 columns wrote 32-byte Q pieces, +37 us per 2^26 trial)
constexpr int kRowsTr = 128, kRowsTc = 16;
constexpr int kRowsN = kRowsTr + 3;                        // loaded rows: k2 = r0 - 1 .. r0 + kRowsTr + 1
constexpr int kRowsPer = 256 / kRowsTc;                    // rows per load pass
constexpr int kRowsLd = (kRowsN + kRowsPer - 1) / kRowsPer;  // loaded rows per thread
__global__ void __launch_bounds__(256) r2c_interbin_normalise_rows_kernel(
    const float2* __restrict__ Z, uint64_t zp, uint64_t zstride, int log2_n2, uint64_t n1, float* __restrict__ P,
    uint64_t pstride, uint64_t nbins_out, const float* __restrict__ stats, float nscale,
    const uint32_t* __restrict__ tsrc, uint8_t* __restrict__ Q, uint64_t qstride) {
  __shared__ float2 XA[kRowsN][kRowsTc + 1];  // X[kb(rr, cc)] (+1: conflict-free column reads)
  __shared__ float2 XD[kRowsN][kRowsTc + 1];  // X[M - kb(rr, cc)]
  const int kk = blockIdx.y;
  const int t = threadIdx.x;
  const uint64_t n2 = uint64_t(1) << log2_n2, M = n1 << log2_n2, half = M / 2;
  const uint64_t ntr = n2 / kRowsTr;
  const uint64_t r0 = (blockIdx.x % ntr) * kRowsTr, c0 = (blockIdx.x / ntr) * kRowsTc;
  const float2* z = Z + static_cast<uint64_t>(kk) * zstride;
  float* p = P + static_cast<uint64_t>(kk) * pstride;
  uint8_t* q = Q ? Q + static_cast<uint64_t>(kk) * qstride : nullptr;
  if (tsrc) stats += 4 * tsrc[kk];
  const float mean = stats[0] * nscale;
  const float sigma = stats[2] * nscale;
  const float rsig = 1.0f / sigma;
  const float invM = 1.0f / static_cast<float>(M);
  // Forward bins k2 in [r0, r0 + 32), mirror bins M - k for k2 in (r0, r0 + 32]
  // (so both come in aligned groups of four); workgroup-uniform skip
  const bool fwd_any = r0 + n2 * c0 < nbins_out;
  const bool mir_any = M - (r0 + kRowsTr) - n2 * (c0 + kRowsTc - 1) < nbins_out;
  if (fwd_any || mir_any) {
    // bin of row rr (0 .. 34), column cc: kb = r0 - 1 + rr + n2 (c0 + cc) (-1: X[-1] = 0).
    // Every pair's two loads issued before any is used.
    const int cc = t & (kRowsTc - 1);
    float2 za[kRowsLd], zb[kRowsLd];
#pragma unroll
    for (int i = 0; i < kRowsLd; ++i) {
      const int rr = t / kRowsTc + kRowsPer * i;
      const int64_t kb = static_cast<int64_t>(r0) - 1 + rr + static_cast<int64_t>(n2 * (c0 + cc));
      za[i] = zb[i] = make_float2(0.f, 0.f);
      if (rr < kRowsN && kb >= 0) {
        const uint64_t k = static_cast<uint64_t>(kb), mk = (M - k) & (M - 1);
        za[i] = z[(k & (n2 - 1)) * zp + (k >> log2_n2)];
        zb[i] = z[(mk & (n2 - 1)) * zp + (mk >> log2_n2)];
      }
    }
#pragma unroll
    for (int i = 0; i < kRowsLd; ++i) {
      const int rr = t / kRowsTc + kRowsPer * i;
      if (rr < kRowsN) {
        const int64_t kb = static_cast<int64_t>(r0) - 1 + rr + static_cast<int64_t>(n2 * (c0 + cc));
        float2 xa = make_float2(0.f, 0.f), xd = make_float2(0.f, 0.f);
        if (kb >= 0) {
          float sn, cs;
          sincospif(-static_cast<float>(kb) * invM, &sn, &cs);
          xa = r2c_combine(za[i], zb[i], cs, sn);
          xd = r2c_combine(zb[i], za[i], -cs, sn);  // angle -pi (M-k)/M = -pi + pi k/M
        }
        XA[rr][cc] = xa;
        XD[rr][cc] = xd;
      }
    }
    __syncthreads();
    // Thread (g = t % 32, column c = t / 32 (+ 8)): four consecutive bins per
    // side as one 16-byte P store and one 4-byte Q store (32 lanes: 512
    // contiguous bytes of P, one 128-byte Q line).  Forward: k2 = r0 + 4g ..
    // +3 (rows 4g+1 .. 4g+4, neighbour the row above); mirror: j = M - k for
    // k2 = r0 + 4g + 4 .. +1 (rows 4g+5 .. 4g+2, neighbour X[M - k - 1] the
    // row below), ascending j.
    const int g = t & (kRowsTr / 4 - 1);
    auto q8x4 = [](const float (&v)[4]) {
      return static_cast<uint32_t>(dev::q8(v[0])) | (static_cast<uint32_t>(dev::q8(v[1])) << 8) |
             (static_cast<uint32_t>(dev::q8(v[2])) << 16) | (static_cast<uint32_t>(dev::q8(v[3])) << 24);
    };
#pragma unroll
    for (int h = 0; h < kRowsTc / (256 / (kRowsTr / 4)); ++h) {
      const int c = t / (kRowsTr / 4) + (256 / (kRowsTr / 4)) * h;
      const uint64_t kc = n2 * (c0 + c);
      const uint64_t k = r0 + 4 * g + kc;  // first forward bin (multiple of 4)
      if (k < nbins_out) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = dev::div_rn(dev::interbin(XA[4 * g + 1 + e][c], XA[4 * g + e][c]) - mean, sigma, rsig);
        if (k + 4 <= nbins_out) {
          *reinterpret_cast<float4*>(p + k) = make_float4(v[0], v[1], v[2], v[3]);
          if (q) *reinterpret_cast<uint32_t*>(q + k) = q8x4(v);
        } else {
          for (int e = 0; e < 4 && k + e < nbins_out; ++e) {
            p[k + e] = v[e];
            if (q) q[k + e] = dev::q8(v[e]);
          }
        }
      }
      // first mirror bin (a multiple of 4, >= M/2: bin M/2 itself is written
      // once, below, so a group starting there stores its other three alone)
      const uint64_t j = M - (r0 + 4 * g + 4 + kc);
      if (j < nbins_out && j + 3 > half) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)  // bin j + e = M - (k2 = r0 + 4g + 4 - e)
          v[e] = dev::div_rn(dev::interbin(XD[4 * g + 5 - e][c], XD[4 * g + 6 - e][c]) - mean, sigma, rsig);
        if (j > half && j + 4 <= nbins_out) {
          *reinterpret_cast<float4*>(p + j) = make_float4(v[0], v[1], v[2], v[3]);
          if (q) *reinterpret_cast<uint32_t*>(q + j) = q8x4(v);
        } else {
          for (int e = 0; e < 4 && j + e < nbins_out; ++e) {
            if (j + e <= half) continue;
            p[j + e] = v[e];
            if (q) q[j + e] = dev::q8(v[e]);
          }
        }
      }
    }
  }
  if (blockIdx.x == 0 && t == 0) {
    // bin M/2 (k2 = 0, k1 = n1/2: its own mirror) and bin M (the mirror of 0)
    auto zat = [&](uint64_t k) { return z[(k & (n2 - 1)) * zp + (k >> log2_n2)]; };
    auto xk = [&](uint64_t k) {
      float sn, cs;
      sincospif(-static_cast<float>(k) * invM, &sn, &cs);
      return r2c_combine(zat(k), zat((M - k) & (M - 1)), cs, sn);
    };
    if (half < nbins_out) {
      const float v = dev::div_rn(dev::interbin(xk(half), xk(half - 1)) - mean, sigma, rsig);
      p[half] = v;
      if (q) q[half] = dev::q8(v);
    }
    if (M < nbins_out) {
      // X[M] = combine(Z[0], Z[0], -1, 0); its neighbour X[M - 1] = mirror of bin 1
      const float2 z0 = zat(0), z1 = zat(1), zm1 = zat(M - 1);
      float sn, cs;
      sincospif(-invM, &sn, &cs);
      const float v = dev::div_rn(dev::interbin(r2c_combine(z0, z0, -1.0f, 0.0f), r2c_combine(zm1, z1, -cs, sn)) - mean,
                                  sigma, rsig);
      p[M] = v;
      if (q) q[M] = dev::q8(v);
    }
  }
}

// Tiled spectrum layout written by fft4 pass B (kFft4TileX):
// bin k = k2 + n2*k1 at X_t[k2/8][k1/8][k2%8][k1%8]; a (k2-octet, k1-octet)
// pair is one contiguous 512-byte chunk.
__device__ __forceinline__ uint64_t taddr(uint64_t k, int log2_n2, uint64_t n1) {
  const uint64_t k2 = k & ((uint64_t(1) << log2_n2) - 1), k1 = k >> log2_n2;
  return (k2 >> 3) * (8 * n1) + (k1 >> 3) * 64 + (k2 & 7) * 8 + (k1 & 7);
}

// One workgroup per tile of 8 rows k1 in [g0, g0+8) (g0 < n1/2) x 256
// columns k2 in [c0, c0+256): thread t owns column c0+t of all 8 rows, so its
// 8 bins are 64 contiguous bytes of X_t (4 x 16-byte loads) and so are their
// mirrors M-k = (n2-k2) + n2*(n1-1-k1) (reversed).  Rows k1 < n1/2 produce
// every bin below M/2 and, as mirrors, every bin above it; bin M/2 is done by
// block (0,0).  P rows are written coalesced in natural order.
// Row twiddles W^(r n2) = e^{-i pi r / n1}, r = 0..7 (kernel argument: SGPRs)
struct RowTw8 {
  float c[8], s[8];
};

// The whitener's half spectrum X[0..M] from the tiled four-step output: the
// tile of r2c_interbin_tiled_kernel (8 rows x 256 columns, 64 contiguous
// bytes per lane and mirror) without the interbin step, so every load is a
// 16-byte vector and every row of the output a contiguous 2 KiB store (the
// generic r2c_half_kernel reads one 8-byte element per 64-byte segment).
__global__ void __launch_bounds__(256) r2c_half_tiled_kernel(const float2* __restrict__ Z, int log2_n2, uint64_t n1,
                                                             uint64_t zstride, float2* __restrict__ X,
                                                             uint64_t xstride, RowTw8 rtw) {
  const uint64_t n2 = uint64_t(1) << log2_n2;
  const uint64_t M = n1 * n2, half = M / 2;
  const float invM = 1.0f / static_cast<float>(M);  // M a power of two: x * invM == x / M exactly
  const int t = threadIdx.x;
  const float2* z = Z + static_cast<uint64_t>(blockIdx.z) * zstride;
  float2* x = X + static_cast<uint64_t>(blockIdx.z) * xstride;
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.y) * 8;
  const uint64_t k2 = static_cast<uint64_t>(blockIdx.x) * 256 + t;
  auto xbin = [&](uint64_t k, float2& xa, float2& xm) {  // generic: X[k] and X[M-k]
    const float2 za = z[taddr(k & (M - 1), log2_n2, n1)];
    const float2 zb = z[taddr((M - k) & (M - 1), log2_n2, n1)];
    float sn, cs;
    sincospif(-static_cast<float>(k) * invM, &sn, &cs);
    xa = r2c_combine(za, zb, cs, sn);
    xm = r2c_combine(zb, za, -cs, sn);
  };
  if (k2 == 0) {
    // column 0 pairs row k1 with row n1 - k1 (not n1 - 1 - k1)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint64_t k = (g0 + r) * n2;
      float2 xa, xm;
      xbin(k, xa, xm);
      x[k] = xa;
      x[M - k] = xm;  // k = 0: bin M
    }
  } else {
    const float4* sa = reinterpret_cast<const float4*>(z + (k2 >> 3) * (8 * n1) + (g0 >> 3) * 64 + (k2 & 7) * 8);
    const uint64_t m2 = n2 - k2, m1 = n1 - 8 - g0;  // mirror column, first mirror row (rows reversed)
    const float4* sb = reinterpret_cast<const float4*>(z + (m2 >> 3) * (8 * n1) + (m1 >> 3) * 64 + (m2 & 7) * 8);
    float2 za[8], zb[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 a = sa[u], b = sb[u];
      za[2 * u] = make_float2(a.x, a.y);
      za[2 * u + 1] = make_float2(a.z, a.w);
      zb[7 - 2 * u] = make_float2(b.x, b.y);
      zb[6 - 2 * u] = make_float2(b.z, b.w);
    }
    float sn, cs;
    sincospif(-static_cast<float>(g0 * n2 + k2) * invM, &sn, &cs);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float ws = rtw.s[r], wc = rtw.c[r];  // W^(r n2)
      const float c = __builtin_fmaf(cs, wc, -(sn * ws)), sv = __builtin_fmaf(cs, ws, sn * wc);
      const uint64_t k = (g0 + r) * n2 + k2;
      x[k] = r2c_combine(za[r], zb[r], c, sv);
      x[M - k] = r2c_combine(zb[r], za[r], -c, sv);
    }
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && t == 0) {  // bin M/2 (row n1/2, column 0)
    float2 xa, xm;
    xbin(half, xa, xm);
    x[half] = xa;
  }
}

// The whitener's inverse: x[m] = conj(Z[m]) in natural order from the tiled
// four-step output, 8 rows x 256 columns per workgroup: each lane reads its
// column's 8 rows as 64 contiguous bytes, each row is stored as 2 KiB.
__global__ void __launch_bounds__(256) c2r_post_tiled_kernel(const float2* __restrict__ Z, int log2_n2, uint64_t n1,
                                                             uint64_t zstride, float2* __restrict__ x,
                                                             uint64_t ostride) {
  const uint64_t n2 = uint64_t(1) << log2_n2;
  const float2* z = Z + static_cast<uint64_t>(blockIdx.z) * zstride;
  float2* o = x + static_cast<uint64_t>(blockIdx.z) * ostride;
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.y) * 8;
  const uint64_t k2 = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  const float4* sa = reinterpret_cast<const float4*>(z + (k2 >> 3) * (8 * n1) + (g0 >> 3) * 64 + (k2 & 7) * 8);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 a = sa[u];
    o[(g0 + 2 * u) * n2 + k2] = make_float2(a.x, -a.y);
    o[(g0 + 2 * u + 1) * n2 + k2] = make_float2(a.z, -a.w);
  }
}

// The same inverse written straight into the search pass A's padded input
// (fft4_pad_input's row layout, which it replaces): natural float2 m = j R + r
// (R = 2^log2_r float2 per row) goes to row j at r, a row's first `head`
// float2 also to the previous row's pad (a padded row holds the next row's
// head), and the last row's pad is zero -- the bytes fft4_pad_input writes.
__global__ void __launch_bounds__(256) c2r_post_tiled_pad_kernel(const float2* __restrict__ Z, int log2_n2,
                                                                 uint64_t n1, uint64_t zstride,
                                                                 float2* __restrict__ xp, uint64_t pstride,
                                                                 int log2_r, uint32_t pitch, uint32_t head,
                                                                 uint32_t nrows) {
  const uint64_t n2 = uint64_t(1) << log2_n2;
  const float2* z = Z + static_cast<uint64_t>(blockIdx.z) * zstride;
  float2* o = xp + static_cast<uint64_t>(blockIdx.z) * pstride;
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.y) * 8;
  const uint64_t k2 = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  const uint32_t rlen = 1u << log2_r, rmask = rlen - 1u;
  auto put = [&](uint64_t m, float2 v) {
    const uint32_t j = static_cast<uint32_t>(m >> log2_r), r = static_cast<uint32_t>(m) & rmask;
    o[static_cast<uint64_t>(j) * pitch + r] = v;
    if (r < head) {
      if (j > 0) o[static_cast<uint64_t>(j - 1) * pitch + rlen + r] = v;
      else o[static_cast<uint64_t>(nrows - 1) * pitch + rlen + r] = make_float2(0.f, 0.f);
    }
  };
  const float4* sa = reinterpret_cast<const float4*>(z + (k2 >> 3) * (8 * n1) + (g0 >> 3) * 64 + (k2 & 7) * 8);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 a = sa[u];
    put((g0 + 2 * u) * n2 + k2, make_float2(a.x, -a.y));
    put((g0 + 2 * u + 1) * n2 + k2, make_float2(a.z, -a.w));
  }
}

// The search's r2c + interbin + normalise on that tile.  Interbin
// neighbours come by cross-lane shuffles: lane l's left neighbour X[k-1] is
// lane l-1's ascending bin and its mirror neighbour X[M-(k+1)] is lane l+1's
// mirrored bin; only the values crossing a wave edge (and the tile's two halo
// columns) go through 640 bytes of LDS, so occupancy is set by registers
// (8 workgroups/CU; two 16.5 KiB LDS planes held it to 4).  With Q, the
// harmonic sum's screening bytes dev::q8(P) are stored alongside P.
__global__ void __launch_bounds__(256) r2c_interbin_tiled_shfl_kernel(
    const float2* __restrict__ Z, int log2_n2, uint64_t n1, uint64_t zstride, float* __restrict__ P,
    uint64_t pstride, uint64_t nbins_out, const float* __restrict__ stats, float nscale,
    const float2* __restrict__ rt, const uint32_t* __restrict__ tsrc, uint8_t* __restrict__ Q, uint64_t qstride) {
  __shared__ float2 eA[5][8];  // eA[w][r]: X left of wave w's lane 0 (w = 0: the tile's halo column c0 - 1)
  __shared__ float2 eD[5][8];  // eD[w][r]: mirror X of wave w's lane 0 (w = 4: the halo column c0 + 256)
  const uint64_t n2 = uint64_t(1) << log2_n2;
  const uint64_t M = n1 * n2, half = M / 2;
  const int kk = blockIdx.z;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float2* z = Z + static_cast<uint64_t>(kk) * zstride;
  float* p = P ? P + static_cast<uint64_t>(kk) * pstride : nullptr;
  uint8_t* q = Q ? Q + static_cast<uint64_t>(kk) * qstride : nullptr;
  if (tsrc) stats += 4 * tsrc[kk];
  const float mean = stats[0] * nscale;
  const float sigma = stats[2] * nscale;
  const float rsig = 1.0f / sigma;  // one division per thread; per bin dev::div_rn
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.y) * 8;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * 256;
  auto put = [&](uint64_t k, float v) {
    if (p) p[k] = v;
    if (q) q[k] = dev::q8(v);
  };
  // every bin k <= M/2 with the table twiddle of k, its mirror M - k with
  // (-c, s): each value is a function of Z and k alone (harmonic_peaks_q8_kernel
  // recomputes bins the same way)
  auto xbin = [&](uint64_t k, float2& xa, float2& xm) {  // generic: X[k] and X[M-k], k <= M/2
    const float2 za = z[taddr(k & (M - 1), log2_n2, n1)];
    const float2 zb = z[taddr((M - k) & (M - 1), log2_n2, n1)];
    const float2 tw = dev::r2c_tw(rt, static_cast<uint32_t>(k));
    xa = r2c_combine(za, zb, tw.x, tw.y);
    xm = r2c_combine(zb, za, -tw.x, tw.y);
  };
  const uint64_t k2 = c0 + t;
  float2 xa[8], xm[8];
  if (k2 == 0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) xbin((g0 + r) * n2, xa[r], xm[r]);
  } else {
    const float4* sa = reinterpret_cast<const float4*>(z + (k2 >> 3) * (8 * n1) + (g0 >> 3) * 64 + (k2 & 7) * 8);
    const uint64_t m2 = n2 - k2, m1 = n1 - 8 - g0;
    const float4* sb = reinterpret_cast<const float4*>(z + (m2 >> 3) * (8 * n1) + (m1 >> 3) * 64 + (m2 & 7) * 8);
    float2 za[8], zb[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 a = sa[u], b = sb[u];
      za[2 * u] = make_float2(a.x, a.y);
      za[2 * u + 1] = make_float2(a.z, a.w);
      zb[7 - 2 * u] = make_float2(b.x, b.y);
      zb[6 - 2 * u] = make_float2(b.z, b.w);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float2 tw = dev::r2c_tw(rt, static_cast<uint32_t>((g0 + r) * n2 + k2));
      xa[r] = r2c_combine(za[r], zb[r], tw.x, tw.y);
      xm[r] = r2c_combine(zb[r], za[r], -tw.x, tw.y);
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int r = 0; r < 8; ++r) eA[w + 1][r] = xa[r];
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) eD[w][r] = xm[r];
  }
  if (t < 8) {  // halos: column c0-1 (ascending neighbour) and c0+256 (mirror neighbour) of row t
    const uint64_t row = (g0 + t) * n2 + c0;
    float2 ha, hm;
    if (row > 0) {
      xbin(row - 1, ha, hm);
      eA[0][t] = ha;
    } else {
      eA[0][t] = make_float2(0.f, 0.f);
    }
    xbin(row + 256, ha, hm);
    eD[4][t] = row + 256 == half ? ha : hm;  // bin M/2 in its ascending form, as it is stored
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    float2 xl = make_float2(__shfl_up(xa[r].x, 1, 64), __shfl_up(xa[r].y, 1, 64));
    float2 xr = make_float2(__shfl_down(xm[r].x, 1, 64), __shfl_down(xm[r].y, 1, 64));
    if (lane == 0) xl = eA[w][r];
    if (lane == 63) xr = eD[w + 1][r];
    const uint64_t k = (g0 + r) * n2 + k2;
    if (k < nbins_out) {
      if (k == 0) xl = make_float2(0.f, 0.f);
      put(k, dev::div_rn(dev::interbin(xa[r], xl) - mean, sigma, rsig));
    }
    const uint64_t j = M - k;
    if (j < nbins_out) put(j, dev::div_rn(dev::interbin(xm[r], xr) - mean, sigma, rsig));
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && t == 0 && half < nbins_out) {  // bin M/2 (row n1/2, column 0)
    float2 ha, hm, la, lm;
    xbin(half, ha, hm);
    xbin(half - 1, la, lm);
    put(half, dev::div_rn(dev::interbin(ha, la) - mean, sigma, rsig));
  }
}

// The records of levels [h0, h1] of one bin group with one atomic per wave
// (not one per level): on peak-heavy (RFI) spectra every bin group of a tile
// crosses on several levels, and the single global counter's atomics were
// the emission cost.  Each level's crossings are one chunk in lane (= idx)
// order behind its descriptor {kPeakChunk | count << 16 | segment, first
// idx, position}: the clustering (peakcluster.hip) then sorts chunks, not
// crossings.  Segments are < 2^16 (checked on the host).
template <int NL>
__device__ __forceinline__ void emit_levels(const bool (&pred)[NL], int h0, int h1, uint32_t seg0, int idx,
                                            const float (&snr)[NL], PeakRecord* __restrict__ out,
                                            uint32_t* __restrict__ count, const HarmParams& hp) {
  const int lane = threadIdx.x & 63;
  unsigned long long mask[NL];
  uint32_t tot = 0;
#pragma unroll
  for (int h = 0; h < NL; ++h) {
    mask[h] = (h >= h0 && h <= h1) ? __ballot(pred[h]) : 0ull;
    tot += mask[h] ? static_cast<uint32_t>(__popcll(mask[h])) + 1u : 0u;  // + its descriptor
  }
  if (tot == 0) return;
  // the workgroup's record region (kPeakRegionStride): block-uniform, a
  // multiplicative hash of the block index.  (blockIdx & mask put a bright
  // pulsar's tile of every trial of an 8-trial XCD group into the same 8 of
  // 64 regions: one region overflowed and the whole batch was recomputed --
  // config 3 sliced over 8 ranks, 1.7M records in 85 trials, 9.8 -> 4.9 ms.)
  const uint32_t rg = hp.region_log2 ? (blockIdx.x * 2654435761u) >> (32 - hp.region_log2) : 0u;
  const uint32_t capacity = hp.capacity >> hp.region_log2;
  const uint32_t pos0 = rg * capacity;
  out += pos0;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(count + rg * kPeakRegionStride, tot);
  base = __shfl(base, 0, 64);
  const unsigned long long lt = (lane == 0) ? 0ull : ((1ull << lane) - 1ull);
#pragma unroll
  for (int h = 0; h < NL; ++h) {
    if (mask[h] == 0ull) continue;  // wave-uniform
    const uint32_t cnt = static_cast<uint32_t>(__popcll(mask[h]));
    const uint32_t first = base + 1u;  // the chunk's first crossing
    if (pred[h]) {
      const uint32_t below = static_cast<uint32_t>(__popcll(mask[h] & lt));
      if (below == 0 && base < capacity)  // the chunk's lowest lane: the descriptor (absolute position)
        out[base] = PeakRecord{kPeakChunk | (cnt << 16) | (seg0 + static_cast<uint32_t>(h)), idx,
                               __uint_as_float(pos0 + first)};
      const uint32_t pos = first + below;
      if (pos < capacity) out[pos] = PeakRecord{seg0 + static_cast<uint32_t>(h), idx, snr[h]};
    }
    base = first + cnt;
  }
}

// LDS-staged fused harmonic sum.  A workgroup owns a tile of B = 256*BPT
// bins [b0, b0+B) of one trial.  Every gather the tile needs -- level h,
// odd numerator m: P[(i*m + 2^(h-1)) >> h] -- falls in one contiguous
// range of length ~B*m/2^h, so the tile first copies the fundamental and
// each of those ranges into LDS with coalesced loads (they are L2-hot:
// neighbouring tiles need overlapping ranges), then every thread sums its
// bins from LDS.  Even numerators repeat the previous level's terms and
// are not re-read (as in the reference recurrence).
template <int NLEV, int BPT_ = 0>
struct HarmTile {
  static constexpr int BPT = BPT_ > 0 ? BPT_ : (NLEV <= 3 ? 8 : (NLEV == 4 ? 4 : 2));
  static constexpr int B = 256 * BPT;
  static constexpr int NREG = 1 << NLEV;  // (fundamental) + sum_{h=1..NLEV} 2^(h-1) gather ranges
  static constexpr int maxlen(int h, int m) { return h == 0 ? B : (((B - 1) * m) >> h) + 2; }
  static constexpr int chunks(int h, int m) { return (maxlen(h, m) + 3) / 4; }  // 16-byte chunks
  static constexpr int region(int h, int m) { return h == 0 ? 0 : (1 << (h - 1)) + (m - 1) / 2; }
  // LDS offset (floats, multiple of 4) of gather range r >= 1; the fundamental stays in registers
  static constexpr int offset(int r) {
    int off = 0;
    for (int h = 1; h <= NLEV; ++h)
      for (int m = 1; m < (1 << h); m += 2) {
        if (region(h, m) == r) return off;
        off += 4 * chunks(h, m);
      }
    return off;
  }
  static constexpr int TOTAL = offset(NREG) > 0 ? offset(NREG) : 4;
  static constexpr int iters() {  // 16-byte staging loads per thread
    int n = 0;
    for (int h = 1; h <= NLEV; ++h)
      for (int m = 1; m < (1 << h); m += 2) n += (chunks(h, m) + 255) / 256;
    return n;
  }
  static constexpr int ITERS = iters() > 0 ? iters() : 1;
};

typedef float f4u_h __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-byte load

// 4 consecutive bins a .. a+3 of spectrum p; bins past `last` read bin
// `last` (never used).
__device__ __forceinline__ f4u_h load_chunk(const float* __restrict__ p, int a, int last) {
  if (a + 3 <= last) return *reinterpret_cast<const f4u_h*>(p + a);
  return f4u_h{p[min(a, last)], p[min(a + 1, last)], p[min(a + 2, last)], p[min(a + 3, last)]};
}

// Block order: with xcd_trials (K % 8 == 0) XCD x (blockIdx % 8 under
// round-robin dispatch) runs trials x, x+8, ... and each trial's tiles in
// increasing order, so the recently streamed part of that trial's spectrum
// -- where the high-numerator gather ranges lie -- is in the XCD's own L2.
// Conservative pre-thresholds on the unscaled running sums: o_h > thresh
// implies sum_h > lo[h] (lo[h] sits a relative 1e-5 below thresh / scale_h),
// so a bin group whose sums all stay at or below lo[] cannot hold a peak and
// skips the exact double-scaled levels and range checks.
struct HarmPre {
  float lo[6];
};

template <int NLEV, int BPT_ = 0>
__global__ void __launch_bounds__(256) harmonic_peaks_kernel(const float* __restrict__ P, uint64_t pstride,
                                                             int lo, int hi, HarmParams hp,
                                                             PeakRecord* __restrict__ out,
                                                             uint32_t* __restrict__ count, int ntiles,
                                                             int xcd_trials, HarmPre pre) {
  using Tl = HarmTile<NLEV, BPT_>;
  constexpr int B = Tl::B;
  __shared__ __attribute__((aligned(16))) float lds[Tl::TOTAL];
  const uint32_t bid = blockIdx.x;
  int k, tile;
  if (xcd_trials & 1) {
    const uint32_t slot = bid >> 3;
    k = static_cast<int>((slot / ntiles) * 8 + (bid & 7u));
    tile = static_cast<int>(slot % ntiles);
  } else {
    k = static_cast<int>(bid / ntiles);
    tile = static_cast<int>(bid % ntiles);
  }
  const float* p = P + static_cast<uint64_t>(k) * pstride;
  const int t = threadIdx.x;
  const int b0 = lo + tile * B;
  const int last = hi - 1;
  // ---- fundamental straight into registers (coalesced)
  float fund[Tl::BPT];
#pragma unroll
  for (int u = 0; u < Tl::BPT; ++u) fund[u] = p[min(b0 + t + 256 * u, last)];
  // ---- stage every gather range in 16-byte chunks: all loads are issued
  // before the first LDS store (fixed trip counts).  Only values at indices
  // < hi are ever used; chunks reaching past `last` are gathered per element.
  f4u_h tmp[Tl::ITERS];
  {
    int it = 0;
#pragma unroll
    for (int h = 1; h <= NLEV; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        const int half = 1 << (h - 1);
        const int r0 = (b0 * m + half) >> h;
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          tmp[it] = load_chunk(p, r0 + 4 * (t + 256 * e), last);
      }
    }
  }
  {
    int it = 0;
#pragma unroll
    for (int h = 1; h <= NLEV; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        float4* dst = reinterpret_cast<float4*>(lds + Tl::offset(Tl::region(h, m)));
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          if (t + 256 * e < Tl::chunks(h, m))
            dst[t + 256 * e] = make_float4(tmp[it].x, tmp[it].y, tmp[it].z, tmp[it].w);
      }
    }
  }
  __syncthreads();
  const float thr = hp.thresh;
  const uint32_t seg0 = (static_cast<uint32_t>(k) + hp.trial_base) * 8u;
  bool inner = true;  // block-uniform: the whole tile lies inside every level's search range
#pragma unroll
  for (int h = 0; h <= NLEV; ++h) inner = inner & (b0 >= hp.start[h]) & (b0 + B <= hp.end[h]);
  // Gather offsets are affine in u: for i = i0 + 256u,
  // (i*m + 2^(h-1)) >> h = ((i0*m + 2^(h-1)) >> h) + u*(m << (8-h)) exactly
  // (256m is a multiple of 2^h), so each term's LDS address is formed once per
  // thread and the per-bin reads use immediate offsets.
  const int i0 = b0 + t;
  int lo_h[NLEV + 1], hi_h[NLEV + 1];
#pragma unroll
  for (int h = 0; h <= NLEV; ++h) {
    lo_h[h] = hp.start[h];
    hi_h[h] = hp.end[h];
  }
#define PS_BASE(h, m) (Tl::offset(Tl::region(h, m)) + (((i0 * (m) + (1 << ((h) - 1))) >> (h)) - ((b0 * (m) + (1 << ((h) - 1))) >> (h))))
  int base[Tl::NREG];
  if constexpr (NLEV >= 1) base[1] = PS_BASE(1, 1);
  if constexpr (NLEV >= 2) {
    base[2] = PS_BASE(2, 1);
    base[3] = PS_BASE(2, 3);
  }
  if constexpr (NLEV >= 3) {
#pragma unroll
    for (int m = 1; m < 8; m += 2) base[4 + m / 2] = PS_BASE(3, m);
  }
  if constexpr (NLEV >= 4) {
#pragma unroll
    for (int m = 1; m < 16; m += 2) base[8 + m / 2] = PS_BASE(4, m);
  }
  if constexpr (NLEV >= 5) {
#pragma unroll
    for (int m = 1; m < 32; m += 2) base[16 + m / 2] = PS_BASE(5, m);
  }
#undef PS_BASE
#pragma unroll
  for (int u = 0; u < Tl::BPT; ++u) {
    const int i = i0 + u * 256;
    const bool valid = i < hi;
    float val = fund[u];  // fundamental P[i]
    float sum[NLEV + 1];  // unscaled running sum after each level
    sum[0] = val;
#define PS_TERM(h, m) lds[base[(1 << ((h) - 1)) + (m) / 2] + u * ((m) << (8 - (h)))]
    if constexpr (NLEV >= 1) {
      val += PS_TERM(1, 1);
      sum[1] = val;
    }
    if constexpr (NLEV >= 2) {
      val += PS_TERM(2, 3);  // reference order: 3/4 before 1/4
      val += PS_TERM(2, 1);
      sum[2] = val;
    }
    if constexpr (NLEV >= 3) {
#pragma unroll
      for (int m = 1; m < 8; m += 2) val += PS_TERM(3, m);
      sum[3] = val;
    }
    if constexpr (NLEV >= 4) {
#pragma unroll
      for (int m = 1; m < 16; m += 2) val += PS_TERM(4, m);
      sum[4] = val;
    }
    if constexpr (NLEV >= 5) {
#pragma unroll
      for (int m = 1; m < 32; m += 2) val += PS_TERM(5, m);
      sum[5] = val;
    }
#undef PS_TERM
    bool cand = false;
#pragma unroll
    for (int h = 0; h <= NLEV; ++h) cand = cand | (sum[h] > pre.lo[h]);
    if (__ballot(cand) == 0ull) continue;  // the usual no-peak case: one compare per level
    // exact levels: each scaled by the double constant rsqrt(2^h) before rounding to float
    float o[NLEV + 1];
#pragma unroll
    for (int h = 0; h <= NLEV; ++h) {
      if (h == 2)
        o[h] = sum[h] * 0.5f;  // == (float)((double)sum * 0.5): exact scaling
      else if (h == 4)
        o[h] = sum[h] * 0.25f;
      else
        o[h] = h == 0 ? sum[0] : static_cast<float>(static_cast<double>(sum[h]) * c_level_scale[h]);
    }
    // branch-free predicates (bitwise, no short-circuit)
    bool pred[NLEV + 1];
    bool any = false;
#pragma unroll
    for (int h = 0; h <= NLEV; ++h) {
      const bool in_range = inner | ((i >= lo_h[h]) & (i < hi_h[h]));
      pred[h] = valid & in_range & (o[h] > thr);
      any = any | pred[h];
    }
    if (__ballot(any) == 0ull) continue;  // one ballot per bin group in the (usual) no-peak case
    emit_levels<NLEV + 1>(pred, 0, NLEV, seg0, i, o, out, count, hp);
  }
}

// Two-phase form (harmonic_set_flags bit 5, tuning): levels 1..NLEV-1 are
// staged, summed and thresholded first, then the top level's ranges reuse
// the same LDS -- 16.4 instead of 28.8 KiB and about half the staging
// registers at NLEV = 3, so more workgroups share a CU.  Same sums in the
// same order, same records (emitted level by level; the host sorts each
// (trial, level) segment).
template <int NLEV>
struct HarmTile2 {
  using T = HarmTile<NLEV, 0>;
  static constexpr int SPLIT = 1 << (NLEV - 1);  // first region of the top level
  static constexpr int P1 = T::offset(SPLIT);    // floats of levels 1..NLEV-1
  static constexpr int P2 = T::TOTAL - P1;       // floats of level NLEV
  static constexpr int LDS = P1 > P2 ? P1 : P2;
  static constexpr int iters(int hlo, int hhi) {
    int n = 0;
    for (int h = hlo; h <= hhi; ++h)
      for (int m = 1; m < (1 << h); m += 2) n += (T::chunks(h, m) + 255) / 256;
    return n;
  }
  static constexpr int IT = iters(1, NLEV - 1) > iters(NLEV, NLEV) ? iters(1, NLEV - 1) : iters(NLEV, NLEV);
};

template <int NLEV>
__global__ void __launch_bounds__(256) harmonic_peaks2_kernel(const float* __restrict__ P, uint64_t pstride, int lo,
                                                              int hi, HarmParams hp, PeakRecord* __restrict__ out,
                                                              uint32_t* __restrict__ count, int ntiles, int xcd_trials,
                                                              HarmPre pre) {
  static_assert(NLEV >= 2, "two phases need at least two levels");
  using Tl = HarmTile<NLEV, 0>;
  using T2 = HarmTile2<NLEV>;
  constexpr int B = Tl::B;
  __shared__ __attribute__((aligned(16))) float lds[T2::LDS];
  const uint32_t bid = blockIdx.x;
  int k, tile;
  if (xcd_trials & 1) {
    const uint32_t slot = bid >> 3;
    k = static_cast<int>((slot / ntiles) * 8 + (bid & 7u));
    tile = static_cast<int>(slot % ntiles);
  } else {
    k = static_cast<int>(bid / ntiles);
    tile = static_cast<int>(bid % ntiles);
  }
  const float* p = P + static_cast<uint64_t>(k) * pstride;
  const int t = threadIdx.x;
  const int b0 = lo + tile * B;
  const int last = hi - 1;
  const int i0 = b0 + t;
  // stage the gather ranges of levels [HLO, HHI] at LDS offset base 0
  auto stage = [&](auto hlo_c, auto hhi_c) {
    constexpr int HLO = decltype(hlo_c)::value, HHI = decltype(hhi_c)::value;
    constexpr int BASE = Tl::offset(1 << (HLO - 1));
    f4u_h tmp[T2::IT];
    int it = 0;
#pragma unroll
    for (int h = HLO; h <= HHI; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        const int r0 = (b0 * m + (1 << (h - 1))) >> h;
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          tmp[it] = load_chunk(p, r0 + 4 * (t + 256 * e), last);
      }
    }
    it = 0;
#pragma unroll
    for (int h = HLO; h <= HHI; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        float4* dst = reinterpret_cast<float4*>(lds + Tl::offset(Tl::region(h, m)) - BASE);
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          if (t + 256 * e < Tl::chunks(h, m)) dst[t + 256 * e] = make_float4(tmp[it].x, tmp[it].y, tmp[it].z, tmp[it].w);
      }
    }
  };
  // LDS index of term (h, m) for bin i0 + 256 u (affine in u, see harmonic_peaks_kernel)
  auto term = [&](int h, int m, int base_off, int u) {
    const int r = Tl::region(h, m);
    const int b = Tl::offset(r) - base_off + (((i0 * m + (1 << (h - 1))) >> h) - ((b0 * m + (1 << (h - 1))) >> h));
    return lds[b + u * (m << (8 - h))];
  };
  float fund[Tl::BPT];
#pragma unroll
  for (int u = 0; u < Tl::BPT; ++u) fund[u] = p[min(b0 + t + 256 * u, last)];
  stage(std::integral_constant<int, 1>{}, std::integral_constant<int, NLEV - 1>{});
  __syncthreads();
  const float thr = hp.thresh;
  const uint32_t seg0 = (static_cast<uint32_t>(k) + hp.trial_base) * 8u;
  bool inner = true;
#pragma unroll
  for (int h = 0; h <= NLEV; ++h) inner = inner & (b0 >= hp.start[h]) & (b0 + B <= hp.end[h]);
  // emit the exact-scaled records of levels [h0, h1] for bin i from the unscaled sums
  auto check = [&](const float* sum, int h0, int h1, int i, bool valid) {
    bool cand = false;
    for (int h = h0; h <= h1; ++h) cand = cand | (sum[h] > pre.lo[h]);
    if (__ballot(cand) == 0ull) return;
    bool any = false;
    bool pred[NLEV + 1];
    float o[NLEV + 1];
#pragma unroll
    for (int h = 0; h <= NLEV; ++h) {
      if (h < h0 || h > h1) {
        pred[h] = false;
        o[h] = 0.f;
        continue;
      }
      if (h == 2)
        o[h] = sum[h] * 0.5f;
      else if (h == 4)
        o[h] = sum[h] * 0.25f;
      else
        o[h] = h == 0 ? sum[0] : static_cast<float>(static_cast<double>(sum[h]) * c_level_scale[h]);
      const bool in_range = inner | ((i >= hp.start[h]) & (i < hp.end[h]));
      pred[h] = valid & in_range & (o[h] > thr);
      any = any | pred[h];
    }
    if (__ballot(any) == 0ull) return;
    emit_levels<NLEV + 1>(pred, h0, h1, seg0, i, o, out, count, hp);
  };
  float run[Tl::BPT];  // running sum after level NLEV - 1
#pragma unroll
  for (int u = 0; u < Tl::BPT; ++u) {
    const int i = i0 + u * 256;
    float val = fund[u];
    float sum[NLEV + 1];
    sum[0] = val;
    val += term(1, 1, 0, u);
    sum[1] = val;
    if constexpr (NLEV >= 3) {
      val += term(2, 3, 0, u);  // reference order: 3/4 before 1/4
      val += term(2, 1, 0, u);
      sum[2] = val;
    }
    if constexpr (NLEV >= 4) {
#pragma unroll
      for (int m = 1; m < 8; m += 2) val += term(3, m, 0, u);
      sum[3] = val;
    }
    if constexpr (NLEV >= 5) {
#pragma unroll
      for (int m = 1; m < 16; m += 2) val += term(4, m, 0, u);
      sum[4] = val;
    }
    run[u] = val;
    check(sum, 0, NLEV - 1, i, i < hi);
  }
  __syncthreads();  // phase-1 ranges no longer read
  stage(std::integral_constant<int, NLEV>{}, std::integral_constant<int, NLEV>{});
  __syncthreads();
  constexpr int BASE2 = Tl::offset(1 << (NLEV - 1));
#pragma unroll
  for (int u = 0; u < Tl::BPT; ++u) {
    const int i = i0 + u * 256;
    float val = run[u];
    if constexpr (NLEV == 2) {
      val += term(2, 3, BASE2, u);
      val += term(2, 1, BASE2, u);
    } else {
#pragma unroll
      for (int m = 1; m < (1 << NLEV); m += 2) val += term(NLEV, m, BASE2, u);
    }
    float sum[NLEV + 1];
#pragma unroll
    for (int h = 0; h < NLEV; ++h) sum[h] = 0.f;
    sum[NLEV] = val;
    check(sum, NLEV, NLEV, i, i < hi);
  }
}

// Screened harmonic sum (harmonic_peaks_batch with Q).  The tile stages
// the gather ranges of the screening bytes (dev::q8) instead of P: 16 bins
// per 16-byte load, a quarter of the bytes.  Each level's integer sum of
// bytes s_h (2^h terms) is compared with lim[h], chosen on the host so that
// an fp32 sum above the pre-threshold lo[h] always gives s_h > lim[h]: every
// byte below 254 is within 1/8 of its bin, so (s_h - 127 * 2^h) / 4 + 2^h / 8
// + 0.25 bounds the fp32 sum (0.25 covers its rounding: the terms are below
// 32 in magnitude), lim = floor(4 (lo - 2^h / 8 - 0.25) + 127 * 2^h) - 1.  A
// bin whose sums pass, or whose terms include a byte >= 254 (out of the byte
// range either way), is summed again exactly in the reference order -- the
// same values and records as harmonic_peaks_kernel.
template <int NLEV, int BPT>
struct HarmTileQ {
  static constexpr int B = 256 * BPT;
  static constexpr int NREG = 1 << NLEV;
  static constexpr int maxlen(int h, int m) { return (((B - 1) * m) >> h) + 2; }
  // 16-byte chunks staged per range, from the 16-byte boundary at or below its first bin
  static constexpr int chunks(int h, int m) { return (maxlen(h, m) + 30) / 16; }
  static constexpr int region(int h, int m) { return (1 << (h - 1)) + (m - 1) / 2; }
  static constexpr int offset(int r) {  // bytes, a multiple of 16
    int off = 0;
    for (int h = 1; h <= NLEV; ++h)
      for (int m = 1; m < (1 << h); m += 2) {
        if (region(h, m) == r) return off;
        off += 16 * chunks(h, m);
      }
    return off;
  }
  static constexpr int TOTAL = offset(NREG) > 0 ? offset(NREG) : 16;
  static constexpr int iters() {
    int n = 0;
    for (int h = 1; h <= NLEV; ++h)
      for (int m = 1; m < (1 << h); m += 2) n += (chunks(h, m) + 255) / 256;
    return n;
  }
  static constexpr int ITERS = iters() > 0 ? iters() : 1;
};

struct HarmLim {
  int v[6];
};

// 16 screening bytes a .. a+15 of row q; bytes past `last` repeat byte `last`
// (they only feed bins at or beyond the end of the search range)
__device__ __forceinline__ uint4 load_q16(const uint8_t* __restrict__ q, int a, int last) {
  if (a + 15 <= last) return *reinterpret_cast<const uint4*>(q + a);
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) v |= static_cast<uint32_t>(q[min(a + 4 * j + e, last)]) << (8 * e);
    w[j] = v;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Bin b of trial spectrum z exactly as r2c_interbin_tiled_shfl_kernel stores
// it (HarmFromX): X[b] from Z[b], Z[M-b] and the table twiddle of min(b, M-b)
// (mirror form above M/2), interbinned with X[b-1], normalised.
__device__ __forceinline__ float2 x_canon(const float2* __restrict__ z, uint32_t b, uint32_t M, int log2_n2,
                                          uint32_t n1, const float2* __restrict__ rt) {
  const float2 za = z[taddr(b & (M - 1), log2_n2, n1)];
  const float2 zb = z[taddr((M - b) & (M - 1), log2_n2, n1)];
  const bool up = b <= M / 2;
  const float2 tw = dev::r2c_tw(rt, up ? b : M - b);
  return r2c_combine(za, zb, up ? tw.x : -tw.x, tw.y);
}

// SRC: where the exact sums read a bin -- 0: P (natural order), 1:
// recomputed from the tiled spectrum X (HarmFromX), 2: the blocked P of
// fft4_rowpass_spectrum (spec_pblk_index).  Q rows start fx.qshift bytes
// before bin 0 (staging chunks stay 16-byte aligned in memory).
// (waves_per_eu(7): the register budget of 7 waves per SIMD; the allocator
// then fits 64 VGPRs, 8 waves, where it took 80 unconstrained)
template <int NLEV, int BPT, int SRC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7)))
harmonic_peaks_q8_kernel(const float* __restrict__ P, uint64_t pstride, const uint8_t* __restrict__ Q,
                         uint64_t qstride, int lo, int hi, HarmParams hp, PeakRecord* __restrict__ out,
                         uint32_t* __restrict__ count, int ntiles, int xcd_trials, HarmLim lim, HarmFromX fx) {
  using Tl = HarmTileQ<NLEV, BPT>;
  constexpr int B = Tl::B;
  __shared__ __attribute__((aligned(16))) uint8_t lds[Tl::TOTAL];
  const uint32_t bid = blockIdx.x;
  int k, tile;
  if (xcd_trials & 1) {
    const uint32_t slot = bid >> 3;
    k = static_cast<int>((slot / ntiles) * 8 + (bid & 7u));
    tile = static_cast<int>(slot % ntiles);
  } else {
    k = static_cast<int>(bid / ntiles);
    tile = static_cast<int>(bid % ntiles);
  }
  constexpr bool FROMX = SRC == 1;
  const float* p = FROMX ? nullptr : P + static_cast<uint64_t>(k) * pstride;
  const int qs = fx.qshift;
  const uint8_t* q = Q + static_cast<uint64_t>(k) * qstride + qs;  // q[b]: bin b; q + a aligned iff (a + qs) % 16 == 0
  const int t = threadIdx.x;
  const int b0 = lo + tile * B;
  const int last = hi - 1;
  int fund[BPT];
  // Interior tiles (block-uniform b0 + B <= hi: every bin and every staged
  // range below hi) load without clamps: one per-thread offset, the rest
  // scalar bases and immediate offsets (the clamped forms took ~100 VALU of
  // a wave's ~400).
  const bool interior = b0 + B <= hi;
  uint4 tmp[Tl::ITERS];
  if (interior) {
    const uint8_t* qf = q + (b0 + t);
#pragma unroll
    for (int u = 0; u < BPT; ++u) fund[u] = qf[256 * u];
    // each range as a buffer resource built in SGPRs (base = its first chunk,
    // num_records = the rest of the row: a load past the row returns zeros),
    // the thread's 16 t as the vector offset
    const uint32_t vo = 16u * static_cast<uint32_t>(t);
    int it = 0;
#pragma unroll
    for (int h = 1; h <= NLEV; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        // byte offset of the range's first chunk from the row start (16-byte aligned, >= 0)
        const int r0 = ((((b0 * m + (1 << (h - 1))) >> h) + qs) & ~15);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(q - qs + r0), 0, static_cast<int>(qstride) - r0, 0x00020000);
        // (only the range's chunks: the threads past them would read up to 4 KiB beyond it)
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          if (t + 256 * e < Tl::chunks(h, m))
            tmp[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 4096u * e, 0, 0));
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < BPT; ++u) fund[u] = q[min(b0 + t + 256 * u, last)];
    int it = 0;
#pragma unroll
    for (int h = 1; h <= NLEV; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        const int r0 = ((((b0 * m + (1 << (h - 1))) >> h) + qs) & ~15) - qs;
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          tmp[it] = load_q16(q, r0 + 16 * (t + 256 * e), last);
      }
    }
  }
  {
    int it = 0;
#pragma unroll
    for (int h = 1; h <= NLEV; ++h) {
#pragma unroll
      for (int m = 1; m < (1 << h); m += 2) {
        uint4* dst = reinterpret_cast<uint4*>(lds + Tl::offset(Tl::region(h, m)));
#pragma unroll
        for (int e = 0; e < (Tl::chunks(h, m) + 255) / 256; ++e, ++it)
          if (t + 256 * e < Tl::chunks(h, m)) dst[t + 256 * e] = tmp[it];
      }
    }
  }
  __syncthreads();
  const float thr = hp.thresh;
  const uint32_t seg0 = (static_cast<uint32_t>(k) + hp.trial_base) * 8u;
  bool inner = true;  // block-uniform: the whole tile lies inside every level's search range
#pragma unroll
  for (int h = 0; h <= NLEV; ++h) inner = inner & (b0 >= hp.start[h]) & (b0 + B <= hp.end[h]);
  const int i0 = b0 + t;
  // byte offset in LDS of term (h, m) of bin i0; bin i0 + 256 u adds u * (m << (8 - h))
#define PS_QBASE(h, m) \
  (Tl::offset(Tl::region(h, m)) + (((i0 * (m) + (1 << ((h) - 1))) >> (h)) - (((((b0 * (m) + (1 << ((h) - 1))) >> (h)) + qs) & ~15) - qs)))
  int base[Tl::NREG];
  if constexpr (NLEV >= 1) base[1] = PS_QBASE(1, 1);
  if constexpr (NLEV >= 2) {
    base[2] = PS_QBASE(2, 1);
    base[3] = PS_QBASE(2, 3);
  }
  if constexpr (NLEV >= 3) {
#pragma unroll
    for (int m = 1; m < 8; m += 2) base[4 + m / 2] = PS_QBASE(3, m);
  }
  if constexpr (NLEV >= 4) {
#pragma unroll
    for (int m = 1; m < 16; m += 2) base[8 + m / 2] = PS_QBASE(4, m);
  }
  if constexpr (NLEV >= 5) {
#pragma unroll
    for (int m = 1; m < 32; m += 2) base[16 + m / 2] = PS_QBASE(5, m);
  }
#undef PS_QBASE
  // screen: bit u of cm = bin i0 + 256 u must be summed exactly
  uint32_t cm = 0;
#pragma unroll
  for (int u = 0; u < BPT; ++u) {
    const int i = i0 + u * 256;
    int sq = fund[u], mx = sq;
    bool cand = sq > lim.v[0];
#define PS_QTERM(h, m)                                                                  \
  {                                                                                     \
    const int v = lds[base[(1 << ((h) - 1)) + (m) / 2] + u * ((m) << (8 - (h)))];       \
    sq += v;                                                                            \
    mx = max(mx, v);                                                                    \
  }
    if constexpr (NLEV >= 1) {
      PS_QTERM(1, 1)
      cand = cand | (sq > lim.v[1]);
    }
    if constexpr (NLEV >= 2) {
      PS_QTERM(2, 3)
      PS_QTERM(2, 1)
      cand = cand | (sq > lim.v[2]);
    }
    if constexpr (NLEV >= 3) {
#pragma unroll
      for (int m = 1; m < 8; m += 2) PS_QTERM(3, m)
      cand = cand | (sq > lim.v[3]);
    }
    if constexpr (NLEV >= 4) {
#pragma unroll
      for (int m = 1; m < 16; m += 2) PS_QTERM(4, m)
      cand = cand | (sq > lim.v[4]);
    }
    if constexpr (NLEV >= 5) {
#pragma unroll
      for (int m = 1; m < 32; m += 2) PS_QTERM(5, m)
      cand = cand | (sq > lim.v[5]);
    }
#undef PS_QTERM
    cand = cand | (mx >= 254);
    cm |= cand ? (1u << u) : 0u;
  }
  if (b0 + B > hi) {  // the last tile (block-uniform): its bins at or past hi are not searched
#pragma unroll
    for (int u = 0; u < BPT; ++u)
      if (i0 + u * 256 >= hi) cm &= ~(1u << u);
  }
  if (__ballot(cm != 0u) == 0ull) return;  // the usual no-peak case: the whole wave is done
  // exact sums, one bin group at a time (not unrolled: the exact path is rare)
  const float2* z = nullptr;
  float mean = 0.f, sigma = 1.f, rsig = 1.f;
  uint32_t M = 0;
  if constexpr (FROMX) {
    z = fx.X + static_cast<uint64_t>(k) * fx.xstride;
    const float* st = fx.tsrc ? fx.stats + 4 * fx.tsrc[k] : fx.stats;
    mean = st[0] * fx.nscale;
    sigma = st[2] * fx.nscale;
    rsig = 1.0f / sigma;  // as the r2c kernel
    M = fx.n1 << fx.log2_n2;
  }
  auto pv = [&](int b) -> float {
    if constexpr (FROMX) {
      const uint32_t ub = static_cast<uint32_t>(b);
      const float2 x0 = x_canon(z, ub, M, fx.log2_n2, fx.n1, fx.rt);
      const float2 xl = ub > 0 ? x_canon(z, ub - 1, M, fx.log2_n2, fx.n1, fx.rt) : make_float2(0.f, 0.f);
      return dev::div_rn(dev::interbin(x0, xl) - mean, sigma, rsig);
    } else if constexpr (SRC == 2) {
      return p[spec_pblk_index(static_cast<uint32_t>(b), fx.log2_n2, fx.n1)];
    } else {
      return p[b];
    }
  };
  // (levels <= 3 from P: two bin groups per round, all their 2 x 2^NLEV
  // loads issued before the first sum -- one memory round trip per pair of
  // groups on peak-heavy tiles, where most groups have candidates)
  auto level_out = [&](const float (&sum)[NLEV + 1], int i, bool cand, bool (&pred)[NLEV + 1],
                       float (&o)[NLEV + 1]) {
#pragma unroll
    for (int h = 0; h <= NLEV; ++h) {
      if (h == 2)
        o[h] = sum[h] * 0.5f;
      else if (h == 4)
        o[h] = sum[h] * 0.25f;
      else
        o[h] = h == 0 ? sum[0] : static_cast<float>(static_cast<double>(sum[h]) * c_level_scale[h]);
      const bool in_range = inner | ((i >= hp.start[h]) & (i < hp.end[h]));
      pred[h] = cand & in_range & (o[h] > thr);
    }
  };
  if constexpr (!FROMX && NLEV <= 3 && BPT % 2 == 0) {
    constexpr int NT = 1 << NLEV;  // terms per bin
#pragma unroll 1
    for (int u = 0; u < BPT; u += 2) {
      const bool c0 = (cm >> u) & 1u, c1 = (cm >> (u + 1)) & 1u;
      if (__ballot(c0 | c1) == 0ull) continue;
      float tv[2][NT];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int i = i0 + (u + e) * 256;
        const bool c = e ? c1 : c0;
        // reference order: the fundamental, 1/2, then 3/4 before 1/4, then m/8 ascending
        int b[NT];
        b[0] = i;
        if constexpr (NLEV >= 1) b[1] = (i + 1) >> 1;
        if constexpr (NLEV >= 2) {
          b[2] = (i * 3 + 2) >> 2;
          b[3] = (i + 2) >> 2;
        }
        if constexpr (NLEV >= 3) {
#pragma unroll
          for (int m = 1; m < 8; m += 2) b[4 + m / 2] = (i * m + 4) >> 3;
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) tv[e][q] = c ? pv(b[q]) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int i = i0 + (u + e) * 256;
        float sum[NLEV + 1];
        float val = tv[e][0];
        sum[0] = val;
        if constexpr (NLEV >= 1) {
          val += tv[e][1];
          sum[1] = val;
        }
        if constexpr (NLEV >= 2) {
          val += tv[e][2];
          val += tv[e][3];
          sum[2] = val;
        }
        if constexpr (NLEV >= 3) {
#pragma unroll
          for (int q = 4; q < 8; ++q) val += tv[e][q];
          sum[3] = val;
        }
        bool pred[NLEV + 1];
        float o[NLEV + 1];
        level_out(sum, i, e ? c1 : c0, pred, o);
        emit_levels<NLEV + 1>(pred, 0, NLEV, seg0, i, o, out, count, hp);
      }
    }
    return;
  }
#pragma unroll 1
  for (int u = 0; u < BPT; ++u) {
    const bool cand = (cm >> u) & 1u;
    if (__ballot(cand) == 0ull) continue;
    const int i = i0 + u * 256;
    bool pred[NLEV + 1];
    float o[NLEV + 1];
#pragma unroll
    for (int h = 0; h <= NLEV; ++h) {
      pred[h] = false;
      o[h] = 0.f;
    }
    if (cand) {
      // the fp32 sums in the reference order (harmonic_peaks_kernel)
      float val = pv(i);
      float sum[NLEV + 1];
      sum[0] = val;
      if constexpr (NLEV >= 1) {
        val += pv((i + 1) >> 1);
        sum[1] = val;
      }
      if constexpr (NLEV >= 2) {
        val += pv((i * 3 + 2) >> 2);  // reference order: 3/4 before 1/4
        val += pv((i + 2) >> 2);
        sum[2] = val;
      }
      // (levels 3+ in runtime loops when the bins are recomputed: unrolled,
      // their loads in flight took 106-370 VGPRs and the occupancy of the
      // whole kernel)
      if constexpr (NLEV >= 3) {
        if constexpr (FROMX) {
#pragma unroll 1
          for (int m = 1; m < 8; m += 2) val += pv((i * m + 4) >> 3);
        } else {
#pragma unroll
          for (int m = 1; m < 8; m += 2) val += pv((i * m + 4) >> 3);
        }
        sum[3] = val;
      }
      if constexpr (NLEV >= 4) {
        if constexpr (FROMX) {
#pragma unroll 1
          for (int m = 1; m < 16; m += 2) val += pv((i * m + 8) >> 4);
        } else {
#pragma unroll
          for (int m = 1; m < 16; m += 2) val += pv((i * m + 8) >> 4);
        }
        sum[4] = val;
      }
      if constexpr (NLEV >= 5) {
        if constexpr (FROMX) {
#pragma unroll 1
          for (int m = 1; m < 32; m += 2) val += pv((i * m + 16) >> 5);
        } else {
#pragma unroll
          for (int m = 1; m < 32; m += 2) val += pv((i * m + 16) >> 5);
        }
        sum[5] = val;
      }
#pragma unroll
      for (int h = 0; h <= NLEV; ++h) {
        if (h == 2)
          o[h] = sum[h] * 0.5f;
        else if (h == 4)
          o[h] = sum[h] * 0.25f;
        else
          o[h] = h == 0 ? sum[0] : static_cast<float>(static_cast<double>(sum[h]) * c_level_scale[h]);
        const bool in_range = inner | ((i >= hp.start[h]) & (i < hp.end[h]));
        pred[h] = in_range & (o[h] > thr);
      }
    }
    emit_levels<NLEV + 1>(pred, 0, NLEV, seg0, i, o, out, count, hp);
  }
}

__global__ void __launch_bounds__(256) quantize_q8_kernel(const float* __restrict__ P, uint64_t pstride, uint64_t n,
                                                          uint8_t* __restrict__ Q, uint64_t qstride) {
  const float* p = P + blockIdx.y * pstride;
  uint8_t* q = Q + blockIdx.y * qstride;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    q[i] = dev::q8(p[i]);
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

// ------------------------------------------------ whitening real FFTs ----
// The whitener's N-point real transforms on the four-step passes (K = 1):
//   forward: z[m] = x[2m] + i x[2m+1] -> Z = FFT_M(z) (passes A+B, spectrum
//            layout L) -> X[k] = r2c_combine(Z[k], Z[M-k]), k = 0..M, natural;
//   inverse: Z'[k] = conj((X[k] + conj X[M-k]) + i W^k (X[k] - conj X[M-k])),
//            W = e^{2 pi i/N}; passes A+B give FFT_M(Z') = conj(N-unnormalised
//            IFFT_M), so x[2m] + i x[2m+1] = conj(out[m]) (rocFFT C2R scale).
__device__ __forceinline__ uint64_t xaddr(uint64_t k, const XLayoutArgs& L) {
  return L.tiled ? taddr(k, L.log2_row, L.n1) : zaddr(k, L.log2_row, L.row_pitch, L.blk_pitch, L.log2_blk);
}

__global__ void __launch_bounds__(256) r2c_half_kernel(const float2* __restrict__ Z, uint64_t M, XLayoutArgs L,
                                                       float2* __restrict__ X, uint64_t zstride, uint64_t xstride) {
  Z += blockIdx.y * zstride;
  X += blockIdx.y * xstride;
  const float invM = 1.0f / static_cast<float>(M);  // M a power of two: x * invM == x / M exactly
  for (uint64_t k = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; k <= M;
       k += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const float2 za = Z[xaddr(k & (M - 1), L)];
    const float2 zb = Z[xaddr((M - k) & (M - 1), L)];
    float sn, cs;
    sincospif(-static_cast<float>(k) * invM, &sn, &cs);
    X[k] = r2c_combine(za, zb, cs, sn);
  }
}

__global__ void __launch_bounds__(256) c2r_pre_kernel(const float2* __restrict__ X, uint64_t M,
                                                      float2* __restrict__ out, uint64_t xstride, uint64_t ostride) {
  X += blockIdx.y * xstride;
  out += blockIdx.y * ostride;
  const float invM = 1.0f / static_cast<float>(M);  // M a power of two: x * invM == x / M exactly
  for (uint64_t k = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; k < M;
       k += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const float2 a = X[k], b = X[M - k];
    const float ex = a.x + b.x, ey = a.y - b.y;  // X[k] + conj X[M-k]
    const float dx = a.x - b.x, dy = a.y + b.y;  // X[k] - conj X[M-k]
    float sn, cs;
    sincospif(static_cast<float>(k) * invM, &sn, &cs);
    const float wx = cs * dx - sn * dy, wy = cs * dy + sn * dx;  // W^k d
    // e + i (W^k d), conjugated
    out[k] = make_float2(ex - wy, -(ey + wx));
  }
}

__global__ void __launch_bounds__(256) c2r_post_kernel(const float2* __restrict__ Z, uint64_t M, XLayoutArgs L,
                                                       float2* __restrict__ x, uint64_t zstride, uint64_t ostride) {
  Z += blockIdx.y * zstride;
  x += blockIdx.y * ostride;
  for (uint64_t m = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; m < M;
       m += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const float2 v = Z[xaddr(m, L)];
    x[m] = make_float2(v.x, -v.y);
  }
}

}  // namespace

namespace {
// bit 0: XCD-per-trial block order; bit 1: no pre-threshold (testing);
// bit 2: the search engine's screened sum off; bit 3: its exact sums
// recomputed from the spectrum X (unfused engines); bit 5: the fp32 3-level
// kernel in two staging phases; bit 6: the engine's fused spectrum pass
// (fft4_rowpass_spectrum: pass B writes P and Q, no X and no r2c pass);
// bits 8-15: dynamic-LDS occupancy cap in KiB of the two-phase kernel;
// bit 16: the screened kernel up to 3 levels with 16 bins per thread (a
// 4096-bin tile: twice the staging per workgroup in flight; bench +2.7% over
// 8); bit 17: 32 bins per thread.
// Engines read bits 2, 3 and 6 when they are built.
int g_harm_flags = 1 | 8 | 32 | 64 | (10 << 8) | 65536;

// Mixed-radix n = m p (p a power of two, m odd): gather of the m strided
// columns, and the length-m combination with the twiddles W_n^(n1 k)
// (double-precision recurrence per output).
__global__ void __launch_bounds__(256) mixed_gather_kernel(const float* __restrict__ src, uint64_t n, uint32_t m,
                                                           int log2p, int mode, float2* __restrict__ dst) {
  const uint64_t pmask = (uint64_t(1) << log2p) - 1, half = n / 2;
  const float2* X = reinterpret_cast<const float2*>(src);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t j = (i >> log2p) + m * (i & pmask);  // n1 + m n2
    float2 v;
    if (mode == 0) {
      v = make_float2(src[j], 0.f);
    } else {
      const float2 a = j <= half ? X[j] : X[n - j];
      v = j <= half ? make_float2(a.x, -a.y) : a;  // conj(Xfull[j]), Xfull[n-j] = conj X[j]
    }
    dst[i] = v;
  }
}

__global__ void __launch_bounds__(256) mixed_combine_kernel(const float2* __restrict__ Z, uint64_t zstride,
                                                            XLayoutArgs L, uint64_t n, uint32_t m, uint64_t pmask,
                                                            int mode, uint64_t nout, void* __restrict__ out) {
  for (uint64_t k = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; k < nout;
       k += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t a = xaddr(k & pmask, L);
    double sn, cs;
    sincospi(-2.0 * static_cast<double>(k) / static_cast<double>(n), &sn, &cs);
    double wr = 1.0, wi = 0.0, ar = 0.0, ai = 0.0;
    for (uint32_t n1 = 0; n1 < m; ++n1) {
      const float2 z = Z[n1 * zstride + a];
      ar += wr * z.x - wi * z.y;
      ai += wr * z.y + wi * z.x;
      const double t = wr * cs - wi * sn;
      wi = wr * sn + wi * cs;
      wr = t;
    }
    if (mode == 0)
      reinterpret_cast<float2*>(out)[k] = make_float2(static_cast<float>(ar), static_cast<float>(ai));
    else
      reinterpret_cast<float*>(out)[k] = static_cast<float>(ar);
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
                                  uint64_t blk_pitch, int log2_blk, float* P, uint64_t pstride, int K,
                                  uint64_t nbins_out, const float* stats, float nscale, hipStream_t s,
                                  const uint32_t* tsrc) {
  PSOUP_CHECK(K >= 1 && K <= 65535, "bad batch");
  PSOUP_CHECK(M >= 2 && (M & (M - 1)) == 0, "r2c: M must be a power of two");
  PSOUP_CHECK(nbins_out <= M + 1, "nbins_out beyond the spectrum");
  PSOUP_CHECK(log2_row >= 0 && log2_row < 63 && (uint64_t(1) << log2_row) <= M, "r2c: bad row layout");
  if (nbins_out == 0) return;
  dim3 grid(dev::grid_for((M / 2 + 1 + kR2cBpt - 1) / kR2cBpt, 256, 2048), static_cast<unsigned>(K));
  PSOUP_CHECK(log2_blk >= 0 && log2_blk <= log2_row, "r2c: bad block layout");
  r2c_interbin_normalise_batch_kernel<<<grid, 256, 0, s>>>(Z, M, zstride, log2_row, row_pitch, blk_pitch, log2_blk, P,
                                                           pstride, nbins_out, stats, nscale, tsrc);
  post_launch_check("r2c_interbin_normalise_batch_kernel", s);
}

void r2c_interbin_normalise_rows(const float2* Z, uint64_t zp, uint64_t zstride, int log2_n2, uint64_t n1, float* P,
                                 uint64_t pstride, int K, uint64_t nbins_out, const float* stats, float nscale,
                                 hipStream_t s, const uint32_t* tsrc, uint8_t* Q, uint64_t qstride) {
  PSOUP_CHECK(K >= 1 && K <= 65535, "bad batch");
  PSOUP_CHECK((uint64_t(1) << log2_n2) >= kRowsTr && n1 >= 2 * kRowsTc && (n1 & (n1 - 1)) == 0 && zp >= n1,
              "r2c rows: layout");
  PSOUP_CHECK(pstride % 4 == 0 && (reinterpret_cast<uintptr_t>(P) & 15) == 0 && (!Q || qstride % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(Q) & 3) == 0,
              "r2c rows: P / Q alignment");
  const uint64_t M = n1 << log2_n2;
  PSOUP_CHECK(M < (uint64_t(1) << 31) && nbins_out <= M + 1, "r2c rows: length");
  if (nbins_out == 0) return;
  const uint64_t tiles = ((uint64_t(1) << log2_n2) / kRowsTr) * (n1 / 2 / kRowsTc);
  PSOUP_CHECK(tiles < (uint64_t(1) << 31), "r2c rows: grid");
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(K));
  r2c_interbin_normalise_rows_kernel<<<grid, 256, 0, s>>>(Z, zp, zstride, log2_n2, n1, P, pstride, nbins_out, stats,
                                                          nscale, tsrc, Q, qstride);
  post_launch_check("r2c_interbin_normalise_rows_kernel", s);
}

const float2* r2c_twiddle_table(uint64_t M) {
  PSOUP_CHECK(M >= 2 && (M & (M - 1)) == 0 && M <= (uint64_t(1) << 31), "r2c_twiddle_table: M " << M);
  int dev = 0;
  PSOUP_HIP_CHECK(hipGetDevice(&dev));
  static std::mutex mu;
  static std::map<std::pair<int, uint64_t>, float2*> cache;  // per device and length, kept for the process
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(dev, M);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const uint64_t nh = ((M / 2) >> 11) + 1;
  std::vector<float2> h(2048 + nh);
  auto w = [M](double num) {
    const double a = -M_PI * num / static_cast<double>(M);
    return make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a)));
  };
  for (uint64_t j = 0; j < 2048; ++j) h[j] = w(static_cast<double>(j));
  for (uint64_t a = 0; a < nh; ++a) h[2048 + a] = w(static_cast<double>(a << 11));
  float2* d = nullptr;
  PSOUP_HIP_CHECK(hipMalloc(&d, h.size() * sizeof(float2)));
  PSOUP_HIP_CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
  cache[key] = d;
  return d;
}

void r2c_interbin_normalise_tiled(const float2* X, int n1, int n2, uint64_t xstride, float* P, uint64_t pstride,
                                  int K, uint64_t nbins_out, const float* stats, float nscale, hipStream_t s,
                                  const uint32_t* tsrc, uint8_t* Q, uint64_t qstride, const float2* rt) {
  PSOUP_CHECK(K >= 1 && K <= 65535, "bad batch");
  PSOUP_CHECK(n1 >= 16 && n2 >= 256 && (n1 & (n1 - 1)) == 0 && (n2 & (n2 - 1)) == 0, "r2c tiled: bad geometry");
  PSOUP_CHECK(nbins_out <= static_cast<uint64_t>(n1) * n2 + 1, "nbins_out beyond the spectrum");
  PSOUP_CHECK((reinterpret_cast<uintptr_t>(X) & 15) == 0 && xstride % 2 == 0, "r2c tiled: alignment");
  if (nbins_out == 0) return;
  int lg = 0;
  while ((1 << lg) < n2) ++lg;
  // row blocks beyond the last one holding a bin < nbins_out write nothing
  dim3 grid(static_cast<unsigned>(n2 / 256), r2c_tiled_row_blocks(nbins_out, n1, n2), static_cast<unsigned>(K));
  if (!rt) rt = r2c_twiddle_table(static_cast<uint64_t>(n1) * n2);
  PSOUP_CHECK(P || Q, "r2c tiled: no output");
  PSOUP_CHECK(!Q || qstride >= nbins_out, "r2c tiled: screening row too short");
  r2c_interbin_tiled_shfl_kernel<<<grid, 256, 0, s>>>(X, lg, static_cast<uint64_t>(n1), xstride, P, pstride, nbins_out,
                                                      stats, nscale, rt, tsrc, Q, qstride);
  post_launch_check("r2c_interbin_tiled_shfl_kernel", s);
}

void mixed_gather(const float* src, uint64_t n, uint32_t m, uint64_t p, int mode, float2* dst, hipStream_t s) {
  PSOUP_CHECK(p >= 2 && (p & (p - 1)) == 0 && m >= 1 && n == static_cast<uint64_t>(m) * p, "mixed_gather: bad shape");
  int lg = 0;
  while ((uint64_t(1) << lg) < p) ++lg;
  mixed_gather_kernel<<<dev::grid_for(n, 256, 4096), 256, 0, s>>>(src, n, m, lg, mode, dst);
  post_launch_check("mixed_gather_kernel", s);
}

void mixed_combine(const float2* Z, uint64_t zstride, const XLayoutArgs& L, uint64_t n, uint32_t m, uint64_t p,
                   int mode, void* out, hipStream_t s) {
  PSOUP_CHECK(p >= 2 && (p & (p - 1)) == 0 && m >= 1 && n == static_cast<uint64_t>(m) * p, "mixed_combine: bad shape");
  const uint64_t nout = mode == 0 ? n / 2 + 1 : n;
  mixed_combine_kernel<<<dev::grid_for(nout, 256, 4096), 256, 0, s>>>(Z, zstride, L, n, m, p - 1, mode, nout, out);
  post_launch_check("mixed_combine_kernel", s);
}

void fft4_r2c_half(const float2* Z, uint64_t M, const XLayoutArgs& L, float2* X, hipStream_t s, int count,
                   uint64_t zstride, uint64_t xstride) {
  PSOUP_CHECK(M >= 2 && (M & (M - 1)) == 0, "r2c_half: M must be a power of two");
  PSOUP_CHECK(count >= 1 && count <= 65535, "r2c_half: bad count");
  const uint64_t n1 = L.n1, n2 = L.tiled ? (uint64_t(1) << L.log2_row) : 0;
  if (L.tiled && n1 >= 16 && n2 >= 256 && n1 * n2 == M && (reinterpret_cast<uintptr_t>(Z) & 15) == 0 &&
      zstride % 2 == 0) {
    RowTw8 rtw;
    for (int r = 0; r < 8; ++r) {
      const double a = -M_PI * r / static_cast<double>(n1);
      rtw.c[r] = static_cast<float>(std::cos(a));
      rtw.s[r] = static_cast<float>(std::sin(a));
    }
    const dim3 grid(static_cast<unsigned>(n2 / 256), static_cast<unsigned>(n1 / 16), static_cast<unsigned>(count));
    r2c_half_tiled_kernel<<<grid, 256, 0, s>>>(Z, L.log2_row, n1, zstride, X, xstride, rtw);
    post_launch_check("r2c_half_tiled_kernel", s);
    return;
  }
  const dim3 grid(dev::grid_for(M + 1, 256, count > 1 ? 1024 : 4096), static_cast<unsigned>(count));
  r2c_half_kernel<<<grid, 256, 0, s>>>(Z, M, L, X, zstride, xstride);
  post_launch_check("r2c_half_kernel", s);
}

void fft4_c2r_pre(const float2* X, uint64_t M, float2* out, hipStream_t s, int count, uint64_t xstride,
                  uint64_t ostride) {
  PSOUP_CHECK(M >= 2 && (M & (M - 1)) == 0, "c2r_pre: M must be a power of two");
  PSOUP_CHECK(count >= 1 && count <= 65535, "c2r_pre: bad count");
  const dim3 grid(dev::grid_for(M, 256, count > 1 ? 1024 : 4096), static_cast<unsigned>(count));
  c2r_pre_kernel<<<grid, 256, 0, s>>>(X, M, out, xstride, ostride);
  post_launch_check("c2r_pre_kernel", s);
}

void fft4_c2r_post(const float2* Z, uint64_t M, const XLayoutArgs& L, float* x, hipStream_t s, int count,
                   uint64_t zstride, uint64_t ostride) {
  PSOUP_CHECK((reinterpret_cast<uintptr_t>(x) & 7) == 0 && ostride % 2 == 0, "c2r_post: output alignment");
  PSOUP_CHECK(count >= 1 && count <= 65535, "c2r_post: bad count");
  const uint64_t n1 = L.n1, n2 = L.tiled ? (uint64_t(1) << L.log2_row) : 0;
  if (L.tiled && n1 >= 8 && n2 >= 256 && n1 * n2 == M && (reinterpret_cast<uintptr_t>(Z) & 15) == 0 &&
      zstride % 2 == 0) {
    const dim3 grid(static_cast<unsigned>(n2 / 256), static_cast<unsigned>(n1 / 8), static_cast<unsigned>(count));
    c2r_post_tiled_kernel<<<grid, 256, 0, s>>>(Z, L.log2_row, n1, zstride, reinterpret_cast<float2*>(x), ostride / 2);
    post_launch_check("c2r_post_tiled_kernel", s);
    return;
  }
  const dim3 grid(dev::grid_for(M, 256, count > 1 ? 1024 : 4096), static_cast<unsigned>(count));
  c2r_post_kernel<<<grid, 256, 0, s>>>(Z, M, L, reinterpret_cast<float2*>(x), zstride, ostride / 2);
  post_launch_check("c2r_post_kernel", s);
}

bool fft4_c2r_post_pad(const float2* Z, uint64_t M, const XLayoutArgs& L, float* xpad, const Fft4Geom& gs,
                       hipStream_t s, int count, uint64_t zstride, uint64_t pstride) {
  const uint64_t n1 = L.n1, n2 = L.tiled ? (uint64_t(1) << L.log2_row) : 0;
  const uint64_t rlen = static_cast<uint64_t>(gs.n1), rows = static_cast<uint64_t>(gs.n2);
  const bool ok = L.tiled && n1 >= 8 && n2 >= 256 && n1 * n2 == M && (reinterpret_cast<uintptr_t>(Z) & 15) == 0 &&
                  zstride % 2 == 0 && !fft4_strip_layout(gs) && !gs.rows_ext && rlen * rows == M &&
                  (rlen & (rlen - 1)) == 0 && gs.inpitch % 2 == 0 && gs.inpitch >= 2 * rlen &&
                  (gs.inpitch - 2 * rlen) / 2 <= rlen && rows * gs.inpitch <= gs.insize && pstride % 2 == 0 &&
                  (reinterpret_cast<uintptr_t>(xpad) & 7) == 0 && gs.insize < (1ull << 32);
  if (!ok) return false;
  PSOUP_CHECK(count >= 1 && count <= 65535, "c2r_post_pad: bad count");
  const dim3 grid(static_cast<unsigned>(n2 / 256), static_cast<unsigned>(n1 / 8), static_cast<unsigned>(count));
  c2r_post_tiled_pad_kernel<<<grid, 256, 0, s>>>(Z, L.log2_row, n1, zstride, reinterpret_cast<float2*>(xpad),
                                                 pstride / 2, __builtin_ctzll(rlen),
                                                 static_cast<uint32_t>(gs.inpitch / 2),
                                                 static_cast<uint32_t>((gs.inpitch - 2 * rlen) / 2),
                                                 static_cast<uint32_t>(rows));
  post_launch_check("c2r_post_tiled_pad_kernel", s);
  return true;
}

void harmonic_set_flags(int flags) {
  g_harm_flags = flags;
  set_numerics_flag("harm_flags", flags);
}
int harmonic_flags() { return g_harm_flags; }

void quantize_q8(const float* P, uint64_t pstride, uint64_t n, int K, uint8_t* Q, uint64_t qstride, hipStream_t s) {
  PSOUP_CHECK(K >= 1 && K <= 65535 && qstride >= n, "quantize_q8: bad shape");
  if (n == 0) return;
  quantize_q8_kernel<<<dim3(dev::grid_for(n, 256, 1024), static_cast<unsigned>(K)), 256, 0, s>>>(P, pstride, n, Q,
                                                                                                 qstride);
  post_launch_check("quantize_q8_kernel", s);
}

void harmonic_peaks_batch(const float* P, uint64_t nbins, uint64_t pstride, int K, const HarmParams& hp,
                          PeakRecord* out, uint32_t* count, hipStream_t s, const uint8_t* Q, uint64_t qstride,
                          const HarmFromX* fx) {
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
  PSOUP_CHECK((static_cast<uint64_t>(K) + hp.trial_base) * 8 <= 65536, "chunk descriptors hold 16-bit segments");
  PSOUP_CHECK(hp.region_log2 >= 0 && hp.region_log2 <= 8 && hp.capacity % (1u << hp.region_log2) == 0,
              "harmonic_peaks_batch: record regions must divide the capacity");
  if (hi <= lo) return;
  // the gathers of level h read bin (i m + 2^(h-1)) >> h, m < 2^h: int32 up to
  // hi 2^nlevels (2^27-point series: 2^26 bins x 8 at 3 levels)
  PSOUP_CHECK(static_cast<int64_t>(hi) << hp.nlevels < (int64_t(1) << 31), "spectrum too long for the int32 gather math");
  const int xcd = (g_harm_flags & 1) && (K % 8 == 0) ? 1 : 0;
  // bits 8-15: dynamic LDS occupancy cap, measured for (and applied to) the
  // two-phase 3-level kernel only (the other kernels keep their full occupancy)
  const size_t dyn_lds2 = static_cast<size_t>((g_harm_flags >> 8) & 0xff) * 1024;
  HarmPre pre;
  {
    static const double scale[6] = {1.0, 0.70710678118654752440, 0.5, 0.35355339059327376220, 0.25,
                                    0.17677669529663688110};
    for (int h = 0; h < 6; ++h) {
      const double t = static_cast<double>(hp.thresh) / scale[h];
      // rounding to float and the double product can move o_h by < 2^-23
      // relative; 1e-5 relative margin (and an absolute one near 0) is safe
      const double lo = t - std::fabs(t) * 1e-5 - 1e-30;
      float f = static_cast<float>(lo);
      if (static_cast<double>(f) > lo) f = std::nextafter(f, -INFINITY);
      pre.lo[h] = (g_harm_flags & 2) ? -INFINITY : f;  // bit 1: disable the pre-threshold (testing)
    }
  }
  auto ntiles_of = [&](int B) { return (hi - lo + B - 1) / B; };
  if (Q) {
    PSOUP_CHECK((reinterpret_cast<uintptr_t>(Q) & 15) == 0 && qstride % 16 == 0 && qstride >= static_cast<uint64_t>(hi),
                "harmonic_peaks_batch: screening rows must be 16-byte aligned and cover the search range");
    HarmLim lim;
    for (int h = 0; h < 6; ++h) {
      const double n = std::ldexp(1.0, h);
      const double x = 4.0 * (static_cast<double>(pre.lo[h]) - n / 8.0 - 0.25) + 127.0 * n;
      // above INT_MAX no byte sum passes; below INT_MIN + 1 every bin does (no UB in the cast)
      const double fl = std::isfinite(x) ? std::floor(x) : x;
      lim.v[h] = !(fl > static_cast<double>(INT_MIN) + 1.0) ? INT_MIN
                 : fl >= static_cast<double>(INT_MAX)     ? INT_MAX
                                                          : static_cast<int>(fl) - 1;
    }
    HarmFromX fxv;
    int src = 0;
    if (fx) {
      fxv = *fx;
      const uint64_t M = static_cast<uint64_t>(fxv.n1) << fxv.log2_n2;
      PSOUP_CHECK(fxv.qshift >= 0 && fxv.qshift < 16 && qstride >= static_cast<uint64_t>(hi) + fxv.qshift,
                  "harmonic_peaks_batch: screening row shift");
      if (fxv.pblk) {
        PSOUP_CHECK(P && fxv.n1 >= 16 && M < (uint64_t(1) << 31) && static_cast<uint64_t>(hi) <= M + 1 &&
                        pstride >= M + 1,
                    "harmonic_peaks_batch: bad blocked spectrum");
        src = 2;
      } else {
        PSOUP_CHECK(fxv.X && fxv.rt && fxv.stats && fxv.n1 >= 16 && M < (uint64_t(1) << 31) &&
                        static_cast<uint64_t>(hi) <= M + 1,
                    "harmonic_peaks_batch: bad spectrum for the exact recompute");
        src = 1;
      }
    }
    auto oneq_bp = [&](auto nl_c, auto bp_c) {
      constexpr int NL = decltype(nl_c)::value, BP = decltype(bp_c)::value;
      const int nt = ntiles_of(HarmTileQ<NL, BP>::B);
      PSOUP_CHECK(static_cast<int64_t>(nt) * K < (int64_t(1) << 31), "harmonic grid too large");
      const dim3 grid(static_cast<unsigned>(nt * K));
      if (src == 1)
        harmonic_peaks_q8_kernel<NL, BP, 1><<<grid, 256, 0, s>>>(P, pstride, Q, qstride, lo, hi, hp, out, count, nt,
                                                                 xcd, lim, fxv);
      else if (src == 2)
        harmonic_peaks_q8_kernel<NL, BP, 2><<<grid, 256, 0, s>>>(P, pstride, Q, qstride, lo, hi, hp, out, count, nt,
                                                                 xcd, lim, fxv);
      else
        harmonic_peaks_q8_kernel<NL, BP, 0><<<grid, 256, 0, s>>>(P, pstride, Q, qstride, lo, hi, hp, out, count, nt,
                                                                 xcd, lim, fxv);
    };
    // bins per thread: 8 up to 3 levels (16 with flag bit 16), else 4
    auto oneq = [&](auto nl_c) {
      constexpr int NL = decltype(nl_c)::value;
      if constexpr (NL <= 3) {
        if (g_harm_flags & 131072)
          oneq_bp(nl_c, std::integral_constant<int, 32>{});
        else if (g_harm_flags & 65536)
          oneq_bp(nl_c, std::integral_constant<int, 16>{});
        else
          oneq_bp(nl_c, std::integral_constant<int, 8>{});
      } else {
        oneq_bp(nl_c, std::integral_constant<int, 4>{});
      }
    };
    switch (hp.nlevels) {
      case 0: oneq(std::integral_constant<int, 0>{}); break;
      case 1: oneq(std::integral_constant<int, 1>{}); break;
      case 2: oneq(std::integral_constant<int, 2>{}); break;
      case 3: oneq(std::integral_constant<int, 3>{}); break;
      case 4: oneq(std::integral_constant<int, 4>{}); break;
      default: oneq(std::integral_constant<int, 5>{}); break;
    }
    post_launch_check("harmonic_peaks_q8_kernel", s);
    return;
  }
  auto one = [&](auto nl_c, auto bp_c) {
    constexpr int NL = decltype(nl_c)::value, BP = decltype(bp_c)::value;
    const int nt = ntiles_of(HarmTile<NL, BP>::B);
    PSOUP_CHECK(static_cast<int64_t>(nt) * K < (int64_t(1) << 31), "harmonic grid too large");
    harmonic_peaks_kernel<NL, BP><<<dim3(static_cast<unsigned>(nt * K)), 256, 0, s>>>(P, pstride, lo, hi, hp, out,
                                                                                      count, nt, xcd, pre);
  };
  using I = std::integral_constant<int, 0>;
  switch (hp.nlevels) {
    case 0: one(I{}, I{}); break;
    case 1: one(std::integral_constant<int, 1>{}, I{}); break;
    case 2: one(std::integral_constant<int, 2>{}, I{}); break;
    case 3:
      if (g_harm_flags & 32) {  // two staging phases (levels 1-2, then 3) in 16.4 KiB of LDS
        const int nt = ntiles_of(HarmTile<3, 0>::B);
        PSOUP_CHECK(static_cast<int64_t>(nt) * K < (int64_t(1) << 31), "harmonic grid too large");
        harmonic_peaks2_kernel<3><<<dim3(static_cast<unsigned>(nt * K)), 256, dyn_lds2, s>>>(P, pstride, lo, hi, hp,
                                                                                           out, count, nt, xcd, pre);
      } else {
        one(std::integral_constant<int, 3>{}, I{});
      }
      break;
    case 4: one(std::integral_constant<int, 4>{}, I{}); break;
    default: one(std::integral_constant<int, 5>{}, I{}); break;
  }
  post_launch_check("harmonic_peaks_kernel", s);
}

void harmonic_sums(const float* P, uint64_t nbins, int nlevels, float* out, hipStream_t s) {
  harmonic_sums_kernel<<<dev::grid_for(nbins, 256), 256, 0, s>>>(P, nbins, nlevels, out);
  post_launch_check("harmonic_sums_kernel", s);
}

}  // namespace kern
}  // namespace psoup
