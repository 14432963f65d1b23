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
// (2) fold_optimise is ONE workgroup per candidate doing every step in LDS.
// The template search uses the identity
//     IFFT(P . FFT(boxcar_w))[j] = sum_{m<w} IFFT(P)[j-m]
// so the 63 widths are sliding-window sums of one 64-pt inverse DFT per drift
// instead of 4032 inverse FFTs; the argmax index order (template, shift, bin)
// and first-maximum tie rule of thrust::max_element are kept.
#include <cmath>

#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

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

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// One block (256 threads) per candidate fold [kNi][kNb].
__global__ void __launch_bounds__(256) fold_optimise_kernel(const float* __restrict__ folds,
                                                            const float2* __restrict__ shift_table,
                                                            float* __restrict__ opt_fold,
                                                            float* __restrict__ opt_prof,
                                                            int32_t* __restrict__ opt_int,
                                                            float* __restrict__ opt_val) {
  __shared__ float2 tw[kNb];                 // e^{+2 pi i m/64}
  __shared__ float fin[kNi * kNb];           // input fold
  __shared__ float2 F[kNi * kNb];            // per-subint forward DFT
  __shared__ float2 prof[kNb * kNb];         // [shift][bin] collapsed profiles
  __shared__ float2 Q[kNb * kNb];            // [shift][j] inverse DFT (DC removed)
  __shared__ float red_v[256];
  __shared__ int red_i[256];
  const int tid = threadIdx.x;
  const int cand = blockIdx.x;
  const float* f = folds + static_cast<uint64_t>(cand) * kNi * kNb;
  if (tid < kNb) {
    double sn, cs;
    sincospi(2.0 * tid / kNb, &sn, &cs);
    tw[tid] = make_float2(static_cast<float>(cs), static_cast<float>(sn));
  }
  for (int i = tid; i < kNi * kNb; i += 256) fin[i] = f[i];
  __syncthreads();
  // 1. forward DFT of each subint: F[i][b] = sum_t f[i][t] e^{-2 pi i b t/64}
  for (int o = tid; o < kNi * kNb; o += 256) {
    const int i = o / kNb, b = o % kNb;
    float re = 0.f, im = 0.f;
    for (int t = 0; t < kNb; ++t) {
      const float2 w = tw[(b * t) & (kNb - 1)];
      const float v = fin[i * kNb + t];
      re += v * w.x;
      im -= v * w.y;
    }
    F[o] = make_float2(re, im);
  }
  __syncthreads();
  // 2. apply drifts and collapse subints: prof[s][b] = sum_i F[i][b] * shift[s][i][b]
  for (int o = tid; o < kNb * kNb; o += 256) {
    const int s = o / kNb, b = o % kNb;
    float2 acc = make_float2(0.f, 0.f);
    for (int i = 0; i < kNi; ++i) {
      const float2 v = cmul(F[i * kNb + b], shift_table[(s * kNi + i) * kNb + b]);
      acc.x += v.x;
      acc.y += v.y;
    }
    prof[o] = acc;
  }
  __syncthreads();
  // 3. Q[s][j] = sum_{b>=1} prof[s][b] e^{+2 pi i b j/64}   (template bin 0 is zeroed)
  for (int o = tid; o < kNb * kNb; o += 256) {
    const int s = o / kNb, j = o % kNb;
    float re = 0.f, im = 0.f;
    for (int b = 1; b < kNb; ++b) {
      const float2 p = prof[s * kNb + b];
      const float2 w = tw[(b * j) & (kNb - 1)];
      re += p.x * w.x - p.y * w.y;
      im += p.x * w.y + p.y * w.x;
    }
    Q[o] = make_float2(re, im);
  }
  __syncthreads();
  // 4. boxcar widths 1..63 as sliding sums; argmax over (template, shift, bin)
  float best = -1.f;
  int besti = 0x7fffffff;
  for (int o = tid; o < kNb * kNb; o += 256) {
    const int s = o / kNb, j = o % kNb;
    float sr = 0.f, si = 0.f;
    for (int t = 0; t < kNb - 1; ++t) {
      const float2 q = Q[s * kNb + ((j - t) & (kNb - 1))];
      sr += q.x;
      si += q.y;
      const float v = sqrtf(sr * sr + si * si) / sqrtf(static_cast<float>(t + 1));
      const int idx = t * (kNb * kNb) + s * kNb + j;
      if (v > best || (v == best && idx < besti)) {
        best = v;
        besti = idx;
      }
    }
  }
  red_v[tid] = best;
  red_i[tid] = besti;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) {
      const float v2 = red_v[tid + w];
      const int i2 = red_i[tid + w];
      if (v2 > red_v[tid] || (v2 == red_v[tid] && i2 < red_i[tid])) {
        red_v[tid] = v2;
        red_i[tid] = i2;
      }
    }
    __syncthreads();
  }
  const int am = red_i[0];
  const int opt_template = am / (kNb * kNb);
  const int opt_shift = (am / kNb) % kNb;
  const int opt_bin = am % kNb;
  // 5. optimal subints: Re(IDFT_b(F[i][b] * shift[s*][i][b]))[t]
  float* of = opt_fold + static_cast<uint64_t>(cand) * kNi * kNb;
  for (int o = tid; o < kNi * kNb; o += 256) {
    const int i = o / kNb, t = o % kNb;
    float re = 0.f;
    for (int b = 0; b < kNb; ++b) {
      const float2 v = cmul(F[i * kNb + b], shift_table[(opt_shift * kNi + i) * kNb + b]);
      const float2 w = tw[(b * t) & (kNb - 1)];
      re += v.x * w.x - v.y * w.y;
    }
    of[o] = re;
  }
  // 6. optimal profile: Re(IDFT(prof[s*]))[j] (DC included)
  if (tid < kNb) {
    const float2 q = Q[opt_shift * kNb + tid];
    opt_prof[static_cast<uint64_t>(cand) * kNb + tid] = q.x + prof[opt_shift * kNb].x;
  }
  if (tid == 0) {
    opt_int[3 * cand + 0] = opt_template;
    opt_int[3 * cand + 1] = opt_shift;
    opt_int[3 * cand + 2] = opt_bin;
    opt_val[cand] = red_v[0];
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
