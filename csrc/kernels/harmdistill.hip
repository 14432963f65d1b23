// Per-trial harmonic distillation on the device: the reference's
// HarmonicDistiller(freq_tol, max_harm, keep_related=false,
// fractional_harms=true) (include/transforms/distiller.hpp:63-108), run for
// every acceleration trial on its cluster peaks (src/pipeline_multi.cu:233-238)
// -- the host hot spot on candidate-heavy (RFI) data, SURVEY.md §7.4 item 6.
//
// BaseDistiller (distiller.hpp:27-59) sorts by S/N and then lets every
// surviving candidate, in that order, remove the later candidates related to
// it.  One workgroup per trial here:
//   1. gather the trial's cluster peaks (all levels) into LDS, with their
//      frequencies float(idx * factor[level]) as the host forms them;
//   2. bitonic sort by descending S/N (64-bit keys: order-preserving S/N bits,
//      load position); a tie anywhere hands the trial to the host, whose
//      std::sort breaks ties in the reference's (introsort) order;
//   3. the greedy scan in blocks of 64 candidates: the block's 64 x 64
//      relation bits come from wave ballots (one row per wave step), one lane
//      resolves the block's survivors from them (the greedy order inside the
//      block), and the survivors then clear every later candidate they relate
//      to, each wave owning 64-candidate words of the unique mask;
//   4. compact the unique candidates in S/N order.
// The relation is the host's fast form (candidates.cpp HarmonicDistiller::run,
// valid for tol <= 1e-3 and keep_related = false), with identical double
// expressions; contraction is off so no FMA changes a rounding.
#include "device_common.hpp"

namespace psoup {
namespace kern {
namespace {

constexpr uint32_t kSmallCap = 1024;

__device__ __forceinline__ uint32_t ordered_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float snr_of(uint32_t ob) {
  return __uint_as_float((ob & 0x80000000u) ? (ob & 0x7fffffffu) : ~ob);
}

// Is candidate (freq, nh) related to the fundamental fundi?  The host's fast
// relation (candidates.cpp): for each kk only the nearest integer jj.
__device__ __forceinline__ bool harm_related(double fundi_freq, double freq, int nh, const HarmDistillParams& p) {
#pragma clang fp contract(off)
  const float max_denominator = static_cast<float>(1u << nh);
  const double x1 = freq / fundi_freq;
  for (int kk = 1; kk <= max_denominator; ++kk) {
    const double x = kk * x1;
    if (!(x < p.max_harm + 2.0)) break;
    const int j0 = static_cast<int>(::round(x));  // lround: half away from zero
    if (j0 < 1 || j0 > p.max_harm || ::fabs(x - j0) > 1.5 * p.tol * j0 + 1e-9) continue;
    const double ratio = kk * freq / (j0 * fundi_freq);
    if (ratio > p.lower_tol && ratio < p.upper_tol) return true;
  }
  return false;
}

template <uint32_t CAP, int TH>
__global__ void __launch_bounds__(TH) harm_distill_kernel(const uint2* __restrict__ clust,
                                                          const uint2* __restrict__ segtab, HarmDistillParams p,
                                                          uint32_t lo_n, uint2* __restrict__ out,
                                                          uint2* __restrict__ ttab, uint32_t* __restrict__ total) {
  constexpr uint32_t kWords = CAP / 64;
  constexpr int kWaves = TH / 64;
  __shared__ uint64_t key[CAP];      // ~(S/N order bits << 32 | load position): ascending sort
  __shared__ uint32_t rec[CAP];      // load order: idx | level << 29
  __shared__ float frq[CAP];         // load order: frequency
  __shared__ uint32_t srec[CAP];     // S/N order
  __shared__ float sfrq[CAP];
  __shared__ float ssnr[CAP];
  __shared__ uint64_t uniq[kWords];  // bit c of word w: candidate 64 w + c still unique
  __shared__ uint64_t rel[64];       // in-block relation rows
  __shared__ uint32_t segoff[6], segn[6];
  __shared__ uint32_t wpre[kWords + 1];
  __shared__ uint32_t base_s;
  __shared__ int tie_s;
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const uint32_t k = blockIdx.x;
  const int L = p.nlevels + 1;
  // 1. size of the trial, and who handles it
  uint32_t n = 0;
  bool raw = false;
  for (int h = 0; h < L; ++h) {
    const uint2 e = segtab[8 * k + h];
    raw = raw || (e.y & kClusterRaw);
    n += e.y & ~kClusterRaw;
  }
  if (raw || n > CAP) {
    if (t == 0 && CAP > kSmallCap) ttab[k] = make_uint2(0u, kHarmHost);
    return;
  }
  if (n == 0) {
    if (t == 0 && lo_n == 0) ttab[k] = make_uint2(0u, 0u);
    return;
  }
  if (n <= lo_n) return;
  if (t == 0) {
    uint32_t acc = 0;
    for (int h = 0; h < L; ++h) {
      const uint2 e = segtab[8 * k + h];
      segoff[h] = e.x;
      segn[h] = acc;  // first load position of level h
      acc += e.y;
    }
    tie_s = 0;
  }
  __syncthreads();
  for (uint32_t i = t; i < n; i += TH) {
    int h = 0;
    while (h + 1 < L && i >= segn[h + 1]) ++h;
    const uint2 v = clust[segoff[h] + (i - segn[h])];
    rec[i] = v.x | (static_cast<uint32_t>(h) << 29);
    frq[i] = static_cast<float>(static_cast<double>(static_cast<int>(v.x)) * p.factor[h]);
    key[i] = ~((static_cast<uint64_t>(ordered_bits(__uint_as_float(v.y))) << 32) | i);
  }
  uint32_t P = 2;
  while (P < n) P <<= 1;
  __syncthreads();
  // 2. bitonic sort, ascending comparators only; positions >= n act as +inf
  for (uint32_t kk = 2; kk <= P; kk <<= 1) {
    const uint32_t hh = kk >> 1;
    for (uint32_t q = t; q < P / 2; q += TH) {
      const uint32_t lo = (q / hh) * kk + (q & (hh - 1)), hi = lo ^ (kk - 1);
      if (hi < n) {
        const uint64_t a = key[lo], b = key[hi];
        if (a > b) {
          key[lo] = b;
          key[hi] = a;
        }
      }
    }
    __syncthreads();
    for (uint32_t j = kk >> 2; j > 0; j >>= 1) {
      for (uint32_t q = t; q < P / 2; q += TH) {
        const uint32_t lo = 2 * j * (q / j) + (q & (j - 1)), hi = lo + j;
        if (hi < n) {
          const uint64_t a = key[lo], b = key[hi];
          if (a > b) {
            key[lo] = b;
            key[hi] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = t; i < n; i += TH) {
    const uint64_t kv = ~key[i];
    const uint32_t pos = static_cast<uint32_t>(kv);
    srec[i] = rec[pos];
    sfrq[i] = frq[pos];
    // the S/N itself (the order bits are a bijection of the float bits)
    const float si = snr_of(static_cast<uint32_t>(kv >> 32));
    ssnr[i] = si;
    // equal S/N (as floats: +0 == -0) next to each other: a tie
    if (i + 1 < n && snr_of(static_cast<uint32_t>(~key[i + 1] >> 32)) == si) tie_s = 1;
  }
  const uint32_t nw = (n + 63) / 64;
  for (uint32_t w = t; w < nw; w += TH) {
    const uint32_t c = min(64u, n - 64 * w);
    uniq[w] = c == 64 ? ~0ull : ((1ull << c) - 1);
  }
  __syncthreads();
  if (tie_s) {
    if (t == 0) ttab[k] = make_uint2(0u, kHarmHost);
    return;
  }
  // 3. greedy scan, 64 candidates per block
  for (uint32_t b = 0; b < nw; ++b) {
    const uint32_t r0 = 64 * b;
    const uint32_t nb = min(64u, n - r0);
    const uint64_t m0 = uniq[b];
    // (i) relation rows of the block: wave wv computes rows wv, wv + kWaves, ...
    for (uint32_t r = wv; r < nb; r += kWaves) {
      bool bit = false;
      const uint32_t c = lane;
      if ((m0 >> r & 1) && c > r && c < nb && (m0 >> c & 1)) {
        const uint32_t rc = srec[r0 + c];
        bit = harm_related(sfrq[r0 + r], sfrq[r0 + c], static_cast<int>(rc >> 29), p);
      }
      const uint64_t row = __ballot(bit);
      if (lane == 0) rel[r] = row;
    }
    __syncthreads();
    // (ii) the block's survivors in greedy order
    if (t == 0) {
      uint64_t m = m0;
      for (uint32_t r = 0; r < nb; ++r)
        if (m >> r & 1) m &= ~rel[r];
      uniq[b] = m;
    }
    __syncthreads();
    // (iii) survivors clear the later candidates they relate to
    const uint64_t m = uniq[b];
    if (m != 0) {
      for (uint32_t w = b + 1 + wv; w < nw; w += kWaves) {
        const uint32_t j = 64 * w + lane;
        const uint64_t word = uniq[w];
        bool alive = (word >> lane & 1) != 0;
        if (alive) {
          const double f = sfrq[j];
          const int nh = static_cast<int>(srec[j] >> 29);
          uint64_t mm = m;
          while (mm) {
            const int r = __builtin_ctzll(mm);
            mm &= mm - 1;
            if (harm_related(sfrq[r0 + r], f, nh, p)) {
              alive = false;
              break;
            }
          }
        }
        const uint64_t nwd = __ballot(alive);
        if (lane == 0) uniq[w] = nwd;
      }
    }
    __syncthreads();
  }
  // 4. compaction in S/N order
  if (t == 0) {
    uint32_t acc = 0;
    for (uint32_t w = 0; w < nw; ++w) {
      wpre[w] = acc;
      acc += static_cast<uint32_t>(__builtin_popcountll(uniq[w]));
    }
    base_s = atomicAdd(total, acc);
    ttab[k] = make_uint2(base_s, acc);
  }
  __syncthreads();
  for (uint32_t i = t; i < n; i += TH) {
    const uint32_t w = i >> 6, c = i & 63;
    const uint64_t word = uniq[w];
    if (word >> c & 1)
      out[base_s + wpre[w] + static_cast<uint32_t>(__builtin_popcountll(word & ((1ull << c) - 1)))] =
          make_uint2(srec[i], __float_as_uint(ssnr[i]));
  }
}

}  // namespace

void harm_distill_batch(const uint2* d_clust, const uint2* d_segtab, int ntrials, const HarmDistillParams& p,
                        uint2* d_out, uint2* d_ttab, uint32_t* d_total, hipStream_t s) {
  if (ntrials <= 0) return;
  PSOUP_CHECK(p.nlevels >= 0 && p.nlevels <= 5, "harm_distill_batch: nlevels " << p.nlevels);
  PSOUP_CHECK(p.tol <= 1e-3f, "harm_distill_batch: the device relation needs freq_tol <= 1e-3");
  PSOUP_HIP_CHECK(hipMemsetAsync(d_total, 0, sizeof(uint32_t), s));
  // small trials (<= 1024 peaks, ~30 KiB LDS, several workgroups per CU),
  // then the large ones (<= kHarmCap); the large kernel also flags the
  // trials left to the host
  harm_distill_kernel<kSmallCap, 256><<<ntrials, 256, 0, s>>>(d_clust, d_segtab, p, 0u, d_out, d_ttab, d_total);
  post_launch_check("harm_distill_kernel<small>", s);
  harm_distill_kernel<kHarmCap, 512><<<ntrials, 512, 0, s>>>(d_clust, d_segtab, p, kSmallCap, d_out, d_ttab,
                                                              d_total);
  post_launch_check("harm_distill_kernel<large>", s);
}

}  // namespace kern
}  // namespace psoup
