// Candidate folding and fold optimisation.
//
// Reference: src/kernels.cu:597-651 (K13 fold_time_series_kernel: one block
// per subint, LDS atomics, counts start at 1), :655-865 (K14-K20 shift ramps,
// boxcar templates, multiply/collapse), include/transforms/folder.hpp:235-334
// (FoldOptimiser::optimise: 64-pt FFTs of every subint, 64 linear drifts,
// 63 boxcar widths, a 4032x64 inverse FFT, |.|, argmax).
//
// Here: (1) fold_accumulate fuses the v1 acceleration resampler (K5) into
// the fold and runs many blocks per subint with register run-length
// accumulation before LDS atomics, writing deterministic partial sums;
// (2) fold_optimise is ONE workgroup per candidate doing every step in LDS
// and registers, its 64-point DFTs as register FFTs.
// The template search uses the identity
//     IFFT(P . FFT(boxcar_w))[j] = sum_{m<w} IFFT(P)[j-m]
// so the 63 widths are sliding-window sums of one 64-pt inverse DFT per drift
// instead of 4032 inverse FFTs; the argmax index order (template, shift, bin)
// and first-maximum tie rule of thrust::max_element are kept.
#include <cmath>

#include "device_common.hpp"
#include "dft_reg.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

using namespace dreg;  // cadd / cmul / dft<64> / idft<64> (dft_reg.hpp)

constexpr int kNb = 64;  // bins (the reference hard-codes 64 bins x 16 subints)
constexpr int kNi = 16;

__global__ void __launch_bounds__(256) fold_accumulate_kernel(const float* __restrict__ in, uint64_t n,
                                                              const FoldJob* __restrict__ jobs, int nbins,
                                                              int nints, int chunk, int nchunk,
                                                              float* __restrict__ psum,
                                                              int32_t* __restrict__ pcount) {
  // Deterministic accumulation: every thread owns one float slot per bin
  // (slot[bin][thread]); a fixed-order reduction follows.  Float LDS
  // atomics would make folds (and the folded S/N) vary run to run.
  __shared__ float slot[kNb * 256];
  __shared__ int lcnt[kNb];
  const int job = blockIdx.z;
  const int subint = blockIdx.y;
  const int ch = blockIdx.x;
  for (int b = 0; b < nbins; ++b) slot[b * 256 + threadIdx.x] = 0.f;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) lcnt[b] = 0;
  __syncthreads();
  const FoldJob J = jobs[job];
  in += J.series * n;
  const uint64_t nps = n / nints;
  const uint64_t beg = static_cast<uint64_t>(subint) * nps + static_cast<uint64_t>(ch) * chunk;
  const uint64_t end = min(beg + static_cast<uint64_t>(chunk), static_cast<uint64_t>(subint + 1) * nps);
  const double h = static_cast<double>(n) / 2.0;
  const int per = (chunk + blockDim.x - 1) / blockDim.x;
  const uint64_t my0 = beg + static_cast<uint64_t>(threadIdx.x) * per;
  const uint64_t my1 = min(my0 + per, end);
  int cur = -1;
  float rs = 0.f;
  int rc = 0;
  for (uint64_t j = my0; j < my1; ++j) {
    double ip;
    double fp = modf(static_cast<double>(j) * J.tsamp_by_period, &ip);
    int b = static_cast<int>(floor(fp * nbins));
    b = b < 0 ? 0 : (b >= nbins ? nbins - 1 : b);
    double d = static_cast<double>(j);
    double r = rint(d + J.af * (((d - h) * (d - h)) - (h * h)));
    if (r < 0.0) r = 0.0;
    uint64_t src = static_cast<uint64_t>(r);
    if (src > n - 1) src = n - 1;
    float v = in[src];
    if (b != cur) {
      if (cur >= 0) {
        slot[cur * 256 + threadIdx.x] += rs;
        atomicAdd(&lcnt[cur], rc);
      }
      cur = b;
      rs = 0.f;
      rc = 0;
    }
    rs += v;
    rc++;
  }
  if (cur >= 0) {
    slot[cur * 256 + threadIdx.x] += rs;
    atomicAdd(&lcnt[cur], rc);
  }
  __syncthreads();
  // 4 threads per bin, 64 slots each, then a fixed-order combine
  const int b = threadIdx.x >> 2, q = threadIdx.x & 3;
  float s = 0.f;
  if (b < nbins)
    for (int k = 0; k < 64; ++k) s += slot[b * 256 + q * 64 + k];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  const uint64_t o = ((static_cast<uint64_t>(job) * nints + subint) * nchunk + ch) * nbins;
  if (b < nbins && q == 0) {
    psum[o + b] = s;
    pcount[o + b] = lcnt[b];
  }
}

__global__ void __launch_bounds__(256) fold_reduce_kernel(const float* __restrict__ psum,
                                                          const int32_t* __restrict__ pcount, int total,
                                                          int nbins, int nchunk, float* __restrict__ fold) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;  // (job*nints+subint)*nbins + bin
  if (gid >= total) return;
  const int bin = gid % nbins;
  const int js = gid / nbins;
  float s = 0.f;
  int c = 1;  // reference counts start at 1 (kernels.cu:614)
  for (int k = 0; k < nchunk; ++k) {
    const uint64_t o = (static_cast<uint64_t>(js) * nchunk + k) * nbins + bin;
    s += psum[o];
    c += pcount[o];
  }
  fold[gid] = s / static_cast<float>(c);
}

__global__ void fold_shift_table_kernel(float2* __restrict__ table, int nbins, int nints, float two_pi) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int size = nbins * nbins * nints;
  if (idx >= size) return;
  const float subint = static_cast<float>(static_cast<unsigned>(idx) / nbins % nints);
  const unsigned shift_idx = static_cast<unsigned>(idx) / (nbins * nints);
  const unsigned bin = static_cast<unsigned>(idx) % nbins;
  const float shiftmag = static_cast<float>(static_cast<int>(shift_idx) - nbins / 2);
  const float shift = subint / static_cast<float>(nints) * shiftmag;
  float ramp = static_cast<float>(bin) * two_pi / static_cast<float>(nbins);
  if (bin > static_cast<unsigned>(nbins / 2)) ramp -= two_pi;
  const float ph = -1.f * ramp * shift;
  float sn, cs;
  sincosf(ph, &sn, &cs);
  const float e = expf(0.f);
  table[idx] = make_float2(cs * e, sn * e);
}

// |S|^2 / (t + 1) of a template response (the reference ranks |S| / sqrt(t + 1),
// the same order); one explicit fma so both passes below compute it bitwise
// alike under any contraction setting.
__device__ __forceinline__ float template_power(float2 S, float inv_w) {
  return __builtin_fmaf(S.y, S.y, S.x * S.x) * inv_w;
}

// One block (256 threads) per candidate fold [kNi][kNb].  The DFTs of steps
// 1, 3 and 5 are 64-point radix-8 FFTs in registers (dft_reg.hpp: packed-f32
// butterflies, literal twiddles) -- ~550 packed VALU instructions per
// transform where a 64 x 64 DFT-matrix product costs 64x more multiply-adds
// (as four real 64^3 GEMMs on the f32 MFMA: 512 v_mfma_f32_32x32x2f32 of
// 64 cycles per candidate vs ~2.2k cycles for the 64 row FFTs of step 3).
// Step 4 (every boxcar width at every drift and phase: 258k template
// responses per candidate, the bulk of the work) runs on each thread's
// rotated copy of its drift row in registers with compile-time indices.
__global__ void __launch_bounds__(256) fold_optimise_kernel(const float* __restrict__ folds,
                                                            const float2* __restrict__ shift_table,
                                                            float* __restrict__ opt_fold,
                                                            float* __restrict__ opt_prof,
                                                            int32_t* __restrict__ opt_int,
                                                            float* __restrict__ opt_val) {
  constexpr int P = kNb + 1;                 // padded LDS rows (complex)
  __shared__ float2 F[kNi * P];              // per-subint forward DFT [i][b]
  __shared__ float2 prof[kNb * P];           // [shift][bin] collapsed profiles
  __shared__ float2 Q[kNb * P];              // [shift][j] inverse DFT (DC removed)
  __shared__ float red_v[256];
  __shared__ int red_i[256];
  const int tid = threadIdx.x;
  const int cand = blockIdx.x;
  const float* f = folds + static_cast<uint64_t>(cand) * kNi * kNb;
  // 1. F[i][b] = sum_t f[i][t] e^{-2 pi i b t / 64}
  if (tid < kNi) {
    float2 x[kNb];
    const float4* src = reinterpret_cast<const float4*>(f + tid * kNb);
#pragma unroll
    for (int q = 0; q < kNb / 4; ++q) {
      const float4 v = src[q];
      x[4 * q] = make_float2(v.x, 0.f);
      x[4 * q + 1] = make_float2(v.y, 0.f);
      x[4 * q + 2] = make_float2(v.z, 0.f);
      x[4 * q + 3] = make_float2(v.w, 0.f);
    }
    dft<kNb>(x);
#pragma unroll
    for (int b = 0; b < kNb; ++b) F[tid * P + b] = x[b];
  }
  __syncthreads();
  // 2. drifts and subint collapse: prof[s][b] = sum_i F[i][b] * shift[s][i][b]
  {
    const int b = tid & (kNb - 1), sg = tid >> 6;
    float2 Fi[kNi];
#pragma unroll
    for (int i = 0; i < kNi; ++i) Fi[i] = F[i * P + b];
    for (int s = sg; s < kNb; s += 4) {
      float2 acc = make_float2(0.f, 0.f);
#pragma unroll
      for (int i = 0; i < kNi; ++i) acc = cadd(acc, cmul(Fi[i], shift_table[(s * kNi + i) * kNb + b]));
      prof[s * P + b] = acc;
    }
  }
  __syncthreads();
  // 3. Q[s][j] = sum_{b>=1} prof[s][b] e^{+2 pi i b j / 64}   (template bin 0 is zeroed)
  if (tid < kNb) {
    float2 x[kNb];
    x[0] = make_float2(0.f, 0.f);
#pragma unroll
    for (int b = 1; b < kNb; ++b) x[b] = prof[tid * P + b];
    idft<kNb>(x);
#pragma unroll
    for (int j = 0; j < kNb; ++j) Q[tid * P + j] = x[j];
  }
  __syncthreads();
  // 4. boxcar widths 1..63 as sliding sums of Q; argmax over (template, shift,
  // bin) with the first-maximum rule of thrust::max_element (index
  // t * 4096 + s * 64 + j): the maximum first, then the first index holding it
  const int s = tid >> 2, q = tid & 3;       // drift row s, bins j = 16 q + jj
  float best = -1.f;
  {
    float2 rot[kNb];                          // rot[x] = Q[s][(16 q + x) mod 64]
#pragma unroll
    for (int x = 0; x < kNb; ++x) rot[x] = Q[s * P + ((16 * q + x) & (kNb - 1))];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      float2 S = make_float2(0.f, 0.f);
#pragma unroll
      for (int t = 0; t < kNb - 1; ++t) {
        S = cadd(S, rot[(jj - t) & (kNb - 1)]);
        best = fmaxf(best, template_power(S, 1.0f / static_cast<float>(t + 1)));
      }
    }
  }
  red_v[tid] = best;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red_v[tid] = fmaxf(red_v[tid], red_v[tid + w]);
    __syncthreads();
  }
  const float gbest = red_v[0];
  int besti = 0x7fffffff;
  if (best == gbest) {  // the (few) threads holding the maximum locate its first index
    for (int jj = 0; jj < 16; ++jj) {
      float2 S = make_float2(0.f, 0.f);
      const int j = 16 * q + jj;
      for (int t = 0; t < kNb - 1; ++t) {
        S = cadd(S, Q[s * P + ((j - t) & (kNb - 1))]);
        const int idx = t * (kNb * kNb) + s * kNb + j;
        if (template_power(S, 1.0f / static_cast<float>(t + 1)) == gbest && idx < besti) besti = idx;
      }
    }
  }
  red_i[tid] = besti;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red_i[tid] = min(red_i[tid], red_i[tid + w]);
    __syncthreads();
  }
  const int am = red_i[0];
  const int opt_template = am / (kNb * kNb);
  const int opt_shift = (am / kNb) % kNb;
  const int opt_bin = am % kNb;
  // 5. optimal subints: Re(IDFT_b(F[i][b] * shift[s*][i][b]))[t]
  float* of = opt_fold + static_cast<uint64_t>(cand) * kNi * kNb;
  if (tid < kNi) {
    float2 x[kNb];
#pragma unroll
    for (int b = 0; b < kNb; ++b) x[b] = cmul(F[tid * P + b], shift_table[(opt_shift * kNi + tid) * kNb + b]);
    idft<kNb>(x);
    float4* dst = reinterpret_cast<float4*>(of + tid * kNb);
#pragma unroll
    for (int u = 0; u < kNb / 4; ++u) dst[u] = make_float4(x[4 * u].x, x[4 * u + 1].x, x[4 * u + 2].x, x[4 * u + 3].x);
  }
  // 6. optimal profile: Re(IDFT(prof[s*]))[j] (DC included)
  if (tid < kNb) {
    const float2 qv = Q[opt_shift * P + tid];
    opt_prof[static_cast<uint64_t>(cand) * kNb + tid] = qv.x + prof[opt_shift * P].x;
  }
  if (tid == 0) {
    opt_int[3 * cand + 0] = opt_template;
    opt_int[3 * cand + 1] = opt_shift;
    opt_int[3 * cand + 2] = opt_bin;
    opt_val[cand] = sqrtf(gbest);
  }
}

}  // namespace

void fold_accumulate(const float* in, uint64_t n, const FoldJob* jobs, int njobs, int nbins, int nints, int chunk,
                     float* psum, int32_t* pcount, hipStream_t s) {
  if (njobs <= 0) return;
  PSOUP_CHECK(n >= static_cast<uint64_t>(nints), "series shorter than nints");
  const uint64_t nps = n / nints;
  const int nchunk = static_cast<int>((nps + chunk - 1) / chunk);
  dim3 grid(static_cast<unsigned>(nchunk), static_cast<unsigned>(nints), static_cast<unsigned>(njobs));
  PSOUP_CHECK(nbins >= 1 && nbins <= kNb, "fold_accumulate supports up to 64 bins");
  fold_accumulate_kernel<<<grid, 256, 0, s>>>(in, n, jobs, nbins, nints, chunk, nchunk, psum, pcount);
  post_launch_check("fold_accumulate_kernel", s);
}

void fold_reduce(const float* psum, const int32_t* pcount, int njobs, int nbins, int nints, int nchunk, float* fold,
                 hipStream_t s) {
  const int total = njobs * nints * nbins;
  if (total <= 0) return;
  fold_reduce_kernel<<<(total + 255) / 256, 256, 0, s>>>(psum, pcount, total, nbins, nchunk, fold);
  post_launch_check("fold_reduce_kernel", s);
}

void fold_shift_table(float2* table, int nbins, int nints, hipStream_t s) {
  const int size = nbins * nbins * nints;
  const float two_pi = static_cast<float>(2 * 3.14159265359);
  fold_shift_table_kernel<<<(size + 255) / 256, 256, 0, s>>>(table, nbins, nints, two_pi);
  post_launch_check("fold_shift_table_kernel", s);
}

void fold_optimise(const float* folds, int nfold, const float2* shift_table, float* opt_fold, float* opt_prof,
                   int32_t* opt_int, float* opt_val, hipStream_t s) {
  if (nfold <= 0) return;
  fold_optimise_kernel<<<nfold, 256, 0, s>>>(folds, shift_table, opt_fold, opt_prof, opt_int, opt_val);
  post_launch_check("fold_optimise_kernel", s);
}

}  // namespace kern
}  // namespace psoup
