// Fast Folding Algorithm (FFA) periodicity search kernels (gfx950 / CDNA4).
//
// The reference ships only the options of its FFA pipeline
// (include/utils/cmdline.hpp:35-50, 211-292: FFACmdLineOptions,
// read_ffa_cmdline_options; Makefile:41-42 target `ffaster`, whose source
// and FFAster library are not in the tree).  This is the MI355X-native
// search behind those options:
//
//   detrend (block means, linear trend between block centres) + normalise
//   -> per octave: real-factor downsampling (exact piecewise-constant
//      integration) so that the octave's periods span [nb0, 2 nb0) bins
//   -> for every integer base period P: the M x P folded matrix (rows padded
//      to a power of two with zeros) goes through log2(M2) radix-2 FFA
//      stages, all periods of a chunk batched in one launch per stage; the
//      first stages run on LDS-resident 16-row blocks (one HBM round trip
//      for four stages)
//   -> one wavefront per folded profile: circular prefix sums in LDS,
//      boxcar matched filter over a geometric width ladder, best S/N;
//      only threshold crossings are emitted (ballot-free: one record per
//      wave, one atomic).
//
// FFA convention (Staelin 1969): block of m rows from its two halves H, T
// (each already transformed): out[s] = H[s/2] + roll(T[s/2], -(s+1)/2), i.e.
// out[s][b] = H[s/2][b] + T[s/2][(b + (s+1)/2) mod P].  After log2(M2)
// stages row s holds the fold at period P + s/(M2-1) bins.
#include "device_common.hpp"
#include "psoup/ffa.hpp"

#include <algorithm>

namespace psoup {
namespace kern {

namespace {

// Exact per-block byte sums: blockIdx.y = trend block, x splits it.
__global__ void __launch_bounds__(256) block_sums_kernel(const uint8_t* __restrict__ in, uint64_t n, uint64_t w,
                                                         unsigned long long* __restrict__ sums) {
  __shared__ unsigned long long scratch[4];
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.y) * w;
  const uint64_t b1 = b0 + w < n ? b0 + w : n;
  unsigned long long acc = 0;
  for (uint64_t i = b0 + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < b1;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    acc += in[i];
  acc = dev::block_sum(acc, scratch);
  if (threadIdx.x == 0 && acc) atomicAdd(&sums[blockIdx.y], acc);
}

__global__ void block_means_kernel(const unsigned long long* __restrict__ sums, uint64_t n, uint64_t w, int nblk,
                                   float* __restrict__ means) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += gridDim.x * blockDim.x) {
    const uint64_t b0 = static_cast<uint64_t>(b) * w;
    const uint64_t cnt = (b0 + w < n ? b0 + w : n) - b0;
    means[b] = static_cast<float>(static_cast<double>(sums[b]) / static_cast<double>(cnt));
  }
}

// x[i] = in[i] - trend(i); trend is linear between block centres (flat
// beyond the first/last centre).
__global__ void __launch_bounds__(256) detrend_kernel(const uint8_t* __restrict__ in, uint64_t n, uint64_t w,
                                                      const float* __restrict__ means, int nblk,
                                                      float* __restrict__ out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const double half = 0.5 * static_cast<double>(w);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    const double pos = (static_cast<double>(i) - half) / static_cast<double>(w);  // in block-centre units
    float trend;
    if (pos <= 0.0 || nblk == 1) {
      trend = means[0];
    } else if (pos >= nblk - 1) {
      trend = means[nblk - 1];
    } else {
      const int b = static_cast<int>(pos);
      const float fr = static_cast<float>(pos - b);
      trend = means[b] + fr * (means[b + 1] - means[b]);
    }
    out[i] = static_cast<float>(in[i]) - trend;
  }
}

// out[j] = integral of the piecewise-constant x over [j f, (j+1) f).
__global__ void __launch_bounds__(256) downsample_kernel(const float* __restrict__ x, uint64_t n, double f,
                                                         float* __restrict__ out, uint64_t nout) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t j = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; j < nout; j += stride) {
    const double a = static_cast<double>(j) * f, b = a + f;
    const uint64_t i0 = static_cast<uint64_t>(a), i1 = static_cast<uint64_t>(b);
    float acc;
    if (i0 == i1) {
      acc = x[i0] * static_cast<float>(b - a);
    } else {
      acc = x[i0] * static_cast<float>(static_cast<double>(i0 + 1) - a);
      for (uint64_t i = i0 + 1; i < i1; ++i) acc += x[i];
      if (i1 < n) acc += x[i1] * static_cast<float>(b - static_cast<double>(i1));
    }
    out[j] = acc;
  }
}

// Arena row r of period p: rows < M from the series, the rest zero.
__global__ void __launch_bounds__(256) fill_kernel(const float* __restrict__ ds, const FfaPeriod* __restrict__ per,
                                                   float* __restrict__ arena) {
  const FfaPeriod pp = per[blockIdx.y];
  for (int r = blockIdx.x; r < pp.m2; r += gridDim.x) {
    float* dst = arena + pp.offset + static_cast<uint64_t>(r) * pp.p;
    const float* src = ds + static_cast<uint64_t>(r) * pp.p;
    for (int b = threadIdx.x; b < pp.p; b += blockDim.x) dst[b] = r < pp.m ? src[b] : 0.f;
  }
}

// Stages 0..L-1 (L = min(kLdsRows log2, log2 M2)) on LDS-resident blocks of
// 2^L consecutive rows: one read and one write of the arena for L stages.
constexpr int kLdsLog2 = 4;
constexpr int kLdsRows = 1 << kLdsLog2;
constexpr int kLdsFloats = 16384;  // 64 KiB: 16 rows x 1024 bins
constexpr int kMaxProfile = 2048;
constexpr int kMaxProfileLds = kMaxProfile;

// 1024 threads = 16 rows x 64 bin lanes: thread (r, c) owns row r, bins
// c, c+64, ...; no per-element division, every thread busy whatever P is.
__global__ void __launch_bounds__(1024) stages_lds_kernel(const FfaPeriod* __restrict__ per, float* __restrict__ arena,
                                                          int maxp_lds) {
  __shared__ float buf[2][kLdsFloats];
  const FfaPeriod pp = per[blockIdx.y];
  const int L = pp.log2m2 < kLdsLog2 ? pp.log2m2 : kLdsLog2;
  const int rows = 1 << L;
  const int P = pp.p;
  if (P > maxp_lds || L == 0) return;
  const int r = threadIdx.x >> 6, c = threadIdx.x & 63;
  const bool live = r < rows;
  for (int blk = blockIdx.x; blk * rows < pp.m2; blk += gridDim.x) {
    float* g = arena + pp.offset + static_cast<uint64_t>(blk) * rows * P;
    if (live)
      for (int b = c; b < P; b += 64) buf[0][r * P + b] = g[r * P + b];
    __syncthreads();
    int cur = 0;
    for (int st = 0; st < L; ++st) {
      const int m = 2 << st, h = m >> 1;
      if (live) {
        const float* src = buf[cur];
        float* dst = buf[cur ^ 1];
        const int base = r & ~(m - 1), so = r & (m - 1);
        const int j = so >> 1, sh = ((so + 1) >> 1) % P;
        const float* hrow = src + (base + j) * P;
        const float* trow = src + (base + h + j) * P;
        for (int b = c; b < P; b += 64) {
          int bt = b + sh;
          bt -= (bt >= P) ? P : 0;
          dst[r * P + b] = hrow[b] + trow[bt];
        }
      }
      __syncthreads();
      cur ^= 1;
    }
    if (live)
      for (int b = c; b < P; b += 64) g[r * P + b] = buf[cur][r * P + b];
    __syncthreads();
  }
}

// One global ping-pong pass covering stages st and st+1 (radix 4: rows
// i, q+i, 2q+i, 3q+i of a 4q block -> rows 4i..4i+3, q = 2^st), or stage st
// alone when it is the period's last (radix 2).  Sums are formed in the
// radix-2 order, (X0 + X1[+a]) + (X2[+c] + X3[+d]).  The group's input rows
// are staged in LDS and read back with the circular shifts.
__global__ void __launch_bounds__(256) pass_kernel(const FfaPeriod* __restrict__ per, const float* __restrict__ in,
                                                   float* __restrict__ out, int st) {
  __shared__ float rows[4][kMaxProfileLds];
  const FfaPeriod pp = per[blockIdx.y];
  if (st >= pp.log2m2) return;
  const int P = pp.p;
  const bool r4 = st + 1 < pp.log2m2;
  const int q = 1 << st;
  const int ngroups = r4 ? pp.m2 >> 2 : pp.m2 >> 1;
  const float* src = in + pp.offset;
  float* dst = out + pp.offset;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    if (r4) {
      const int blk = g >> st, i = g & (q - 1);
      const int base = blk * 4 * q;
      for (int k = 0; k < 4; ++k) {
        const float* rsrc = src + static_cast<uint64_t>(base + k * q + i) * P;
        for (int b = threadIdx.x; b < P; b += blockDim.x) rows[k][b] = rsrc[b];
      }
      __syncthreads();
      // out[4i+u][b] = (X0[b] + X1[b+a_u]) + (X2[b+c_u] + X3[b+d_u])
      const int a0 = i % P, a1 = (i + 1) % P;
      const int c0 = (2 * i) % P, c1 = (2 * i + 1) % P, c2 = (2 * i + 2) % P;
      const int d0 = (3 * i) % P, d1 = (3 * i + 1) % P, d2 = (3 * i + 2) % P, d3 = (3 * i + 3) % P;
      auto wrap = [P](int x) { return x >= P ? x - P : x; };
      float* o = dst + static_cast<uint64_t>(base + 4 * i) * P;
      for (int b = threadIdx.x; b < P; b += blockDim.x) {
        const float x0 = rows[0][b];
        const float l0 = x0 + rows[1][wrap(b + a0)], l1 = x0 + rows[1][wrap(b + a1)];
        o[b] = l0 + (rows[2][wrap(b + c0)] + rows[3][wrap(b + d0)]);
        o[P + b] = l0 + (rows[2][wrap(b + c1)] + rows[3][wrap(b + d1)]);
        o[2 * P + b] = l1 + (rows[2][wrap(b + c1)] + rows[3][wrap(b + d2)]);
        o[3 * P + b] = l1 + (rows[2][wrap(b + c2)] + rows[3][wrap(b + d3)]);
      }
      __syncthreads();
    } else {
      const int blk = g >> st, j = g & (q - 1);
      const int base = blk * 2 * q;
      const float* hrow = src + static_cast<uint64_t>(base + j) * P;
      const float* trow = src + static_cast<uint64_t>(base + q + j) * P;
      const int s0 = j % P, s1 = (j + 1) % P;
      float* o = dst + static_cast<uint64_t>(base + 2 * j) * P;
      for (int b = threadIdx.x; b < P; b += blockDim.x) {
        const float hv = hrow[b];
        int t0 = b + s0, t1 = b + s1;
        t0 -= t0 >= P ? P : 0;
        t1 -= t1 >= P ? P : 0;
        o[b] = hv + trow[t0];
        o[P + b] = hv + trow[t1];
      }
    }
  }
}

// One wavefront per profile: circular prefix sums, boxcar S/N ladder.

__global__ void __launch_bounds__(256) snr_kernel(const FfaPeriod* __restrict__ per, const float* __restrict__ a0,
                                                  const float* __restrict__ a1, int lds_stages, FfaSnrParams sp,
                                                  FfaPeak* __restrict__ out, uint32_t* __restrict__ count,
                                                  uint32_t capacity, float* __restrict__ best_out) {
  __shared__ float pre[4][kMaxProfile + 1];
  const FfaPeriod pp = per[blockIdx.y];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s0 = blockIdx.x * 4 + wave;
  const bool active = s0 < pp.m2;  // wave-uniform; every wave still reaches the barrier
  const int s = active ? s0 : pp.m2 - 1;
  const int P = pp.p;
  // the result sits in a1 after an odd number of global ping-pong stages
  const float* prof = (ffa_result_in_second(pp, lds_stages) ? a1 : a0) + pp.offset + static_cast<uint64_t>(s) * P;
  float* C = pre[wave];
  // contiguous chunk per lane, exclusive scan of chunk sums across the wave
  // prefix sums over the profile viewed as rows of 64: coalesced loads, a
  // 64-lane inclusive scan per row plus the running carry (conflict-free LDS)
  if (lane == 0) C[0] = 0.f;
  float carry = 0.f;
  for (int b0 = 0; b0 < P; b0 += 64) {
    const int b = b0 + lane;
    float v = b < P ? prof[b] : 0.f;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float u = __shfl_up(v, off, 64);
      if (lane >= off) v += u;
    }
    if (b < P) C[b + 1] = carry + v;
    carry += __shfl(v, 63, 64);
  }
  __syncthreads();  // prefix sums are wave-local; all four waves reach this barrier
  const float total = C[P];
  const float var = static_cast<float>(pp.m) * sp.var_per_bin;
  // per-lane best over (width, phase), one wave reduction at the end
  float best = -1e30f;
  int best_w = 0;
  for (int wi = 0; wi < sp.nwidths; ++wi) {
    const int w = sp.widths[wi];
    if (w >= P) break;
    float mx = -1e30f;
    for (int ph = lane; ph < P; ph += 64) {
      const int e = ph + w;
      const float sum = e <= P ? C[e] - C[ph] : total - C[ph] + C[e - P];
      mx = fmaxf(mx, sum);
    }
    const float snr = mx * rsqrtf(static_cast<float>(w) * var);
    if (snr > best) {
      best = snr;
      best_w = w;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ob = __shfl_xor(best, off, 64);
    const int ow = __shfl_xor(best_w, off, 64);
    if (ob > best || (ob == best && ow < best_w)) {  // ties: narrowest width (deterministic)
      best = ob;
      best_w = ow;
    }
  }
  if (lane == 0 && active) {
    if (best_out) best_out[pp.best_offset + s] = best;
    if (best > sp.thresh) {
      const uint32_t pos = atomicAdd(count, 1u);
      if (pos < capacity) out[pos] = FfaPeak{static_cast<int32_t>(blockIdx.y), s, best, best_w};
    }
  }
}

}  // namespace

void ffa_detrend(const uint8_t* in, uint64_t n, uint64_t window, unsigned long long* sums, float* block_means,
                 float* out, hipStream_t s) {
  PSOUP_CHECK(n > 0 && window > 0, "ffa_detrend: empty input");
  const uint64_t nblk = (n + window - 1) / window;
  PSOUP_CHECK(nblk < 65536, "ffa_detrend: too many trend blocks");
  PSOUP_HIP_CHECK(hipMemsetAsync(sums, 0, nblk * sizeof(unsigned long long), s));
  const unsigned splits = dev::grid_for(window, 256 * 16, 256);
  block_sums_kernel<<<dim3(splits, static_cast<unsigned>(nblk)), 256, 0, s>>>(in, n, window, sums);
  post_launch_check("ffa block_sums_kernel", s);
  block_means_kernel<<<dev::grid_for(nblk, 256, 64), 256, 0, s>>>(sums, n, window, static_cast<int>(nblk),
                                                                 block_means);
  post_launch_check("ffa block_means_kernel", s);
  detrend_kernel<<<dev::grid_for(n, 256, 4096), 256, 0, s>>>(in, n, window, block_means, static_cast<int>(nblk), out);
  post_launch_check("ffa detrend_kernel", s);
}

void ffa_downsample(const float* x, uint64_t n, double f, float* out, uint64_t nout, hipStream_t s) {
  PSOUP_CHECK(f >= 1.0 && static_cast<double>(nout) * f <= static_cast<double>(n) + 1e-6,
              "ffa_downsample: bad factor/length");
  if (nout == 0) return;
  downsample_kernel<<<dev::grid_for(nout, 256, 4096), 256, 0, s>>>(x, n, f, out, nout);
  post_launch_check("ffa downsample_kernel", s);
}

int ffa_max_profile() { return kMaxProfile; }

bool ffa_uses_lds(int max_p) { return max_p * kLdsRows <= kLdsFloats; }

void ffa_transform(const float* ds, const FfaPeriod* d_periods, int nper, int max_m2, int max_log2m2, int max_p,
                   float* arena0, float* arena1, hipStream_t s) {
  PSOUP_CHECK(nper > 0 && nper < 65536 && max_p > 0 && max_p <= kMaxProfile, "ffa_transform: bad period set");
  const unsigned gx = static_cast<unsigned>(max_m2 < 4096 ? max_m2 : 4096);
  fill_kernel<<<dim3(gx, nper), 256, 0, s>>>(ds, d_periods, arena0);
  post_launch_check("ffa fill_kernel", s);
  int first = 0;
  if (ffa_uses_lds(max_p)) {
    const int nb = (max_m2 + kLdsRows - 1) / kLdsRows;
    stages_lds_kernel<<<dim3(static_cast<unsigned>(nb < 4096 ? nb : 4096), nper), 1024, 0, s>>>(d_periods, arena0,
                                                                                                 kLdsFloats / kLdsRows);
    post_launch_check("ffa stages_lds_kernel", s);
    first = kLdsLog2;
  }
  float* bufs[2] = {arena0, arena1};
  // radix-4 passes (two stages each); a period with one stage left does it
  // as a radix-2 group in the same pass
  const unsigned gp = static_cast<unsigned>(std::max(1, std::min(max_m2 / 2, 4096)));
  for (int st = first, k = 0; st < max_log2m2; st += 2, ++k)
    pass_kernel<<<dim3(gp, nper), 256, 0, s>>>(d_periods, bufs[k & 1], bufs[(k + 1) & 1], st);
  if (max_log2m2 > first) post_launch_check("ffa pass_kernel", s);
}

void ffa_snr(const FfaPeriod* d_periods, int nper, int max_m2, int max_p, const float* arena0, const float* arena1,
             const FfaSnrParams& sp, FfaPeak* out, uint32_t* count, uint32_t capacity, float* best, hipStream_t s) {
  const bool lds_used = ffa_uses_lds(max_p);
  PSOUP_CHECK(sp.nwidths > 0 && sp.nwidths <= kFfaMaxWidths, "ffa_snr: width ladder");
  PSOUP_CHECK(max_p <= kMaxProfile, "ffa_snr: profile too long");
  const unsigned gx = static_cast<unsigned>((max_m2 + 3) / 4);
  snr_kernel<<<dim3(gx, nper), 256, 0, s>>>(d_periods, arena0, arena1, lds_used ? kLdsLog2 : 0, sp, out, count,
                                            capacity, best);
  post_launch_check("ffa snr_kernel", s);
}

}  // namespace kern
}  // namespace psoup
