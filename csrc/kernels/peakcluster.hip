// GPU peak clustering: the reference's per-(trial, harmonic level) peak
// clustering (include/transforms/peakfinder.hpp:24-55, identify_unique_peaks)
// done on the device, so only the cluster peaks -- not every threshold
// crossing -- travel to the host.
//
// The reference scans the idx-sorted crossings of one spectrum: a cluster
// starts at the first unclaimed crossing (its anchor), absorbs every later
// crossing with idx - anchor < gap, and the anchor moves to any absorbed
// crossing of strictly larger S/N; the cluster's peak is the final anchor.
// Two facts make that parallel:
//   (1) a crossing i with a strictly larger crossing in (idx_i, idx_i + gap)
//       is never a cluster peak, and removing all such crossings leaves every
//       cluster's peak and boundaries unchanged (every crossing of a cluster
//       before its peak is of this kind; the peak is the first survivor);
//   (2) among the survivors an anchor never moves, so clusters are greedy
//       gap-windows: within a "run" of survivors spaced < gap apart the peaks
//       are the run's first survivor, then the first survivor >= anchor + gap,
//       and so on; a survivor >= gap after the previous survivor starts a run.
// So the peaks of a whole segment are one chain: the first survivor, then
// next(i) = the first survivor with idx >= idx_i + gap, and so on (a run's
// last anchor has every later survivor of its run within the gap, so its
// next is the following run's start).
// peak_cluster_kernel: one workgroup per segment (trial x level): bitonic
// sort by idx in LDS, the window test (1) and next() in parallel (a suffix
// scan gives the next survivor at or after any position), one thread follows
// the chain (one LDS read per peak), a scan compacts the peaks in idx order.
// Segments over kClusterCap crossings are left to the host (flagged in the
// segment table with their raw, unsorted range).
#include <cstdlib>

#include "device_common.hpp"

namespace psoup {
namespace kern {
namespace {

constexpr int kClThreads = 512;
constexpr uint32_t kClSmall = 4096;  // segments up to this size: the small-LDS kernel (3 workgroups per CU)
constexpr int kSegLds = 8192;        // segments a batch may have for the LDS-aggregated hist/scatter
constexpr int kRecPerThread = 16;    // records per thread in hist/scatter blocks (256 threads)

// Hillis-Steele scans over one value per thread (TH threads).
template <int TH = kClThreads>
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t* sc, uint32_t* total) {
  const int t = threadIdx.x;
  sc[t] = v;
  __syncthreads();
  for (int off = 1; off < TH; off <<= 1) {
    const uint32_t a = t >= off ? sc[t - off] : 0u;
    __syncthreads();
    sc[t] += a;
    __syncthreads();
  }
  const uint32_t incl = sc[t];
  if (total) *total = sc[TH - 1];
  __syncthreads();
  return incl - v;
}

// Per-segment counts: each block counts its records in LDS and adds the
// non-zero counts to the global ones (one atomic per block and segment, not
// per record: heavy segments get tens of thousands of records).
__global__ void __launch_bounds__(256) seg_hist_kernel(const PeakRecord* __restrict__ in,
                                                       const uint32_t* __restrict__ count, uint32_t cap,
                                                       uint32_t nseg, uint32_t* __restrict__ segcnt) {
  __shared__ uint32_t lc[kSegLds];
  const uint32_t n = min(*count, cap);
  const uint32_t base = blockIdx.x * 256u * kRecPerThread;
  if (base >= n) return;
  for (uint32_t i = threadIdx.x; i < nseg; i += 256) lc[i] = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    const uint32_t i = base + r * 256u + threadIdx.x;
    if (i < n) {
      const uint32_t sg = in[i].seg;
      if (sg < nseg) atomicAdd(&lc[sg], 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nseg; i += 256)
    if (lc[i]) atomicAdd(&segcnt[i], lc[i]);
}

__global__ void __launch_bounds__(kClThreads) seg_scan_kernel(const uint32_t* __restrict__ segcnt, uint32_t nseg,
                                                              uint32_t* __restrict__ segoff) {
  __shared__ uint32_t sc[kClThreads];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < nseg; b += kClThreads) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < nseg ? segcnt[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_sum(v, sc, &tot);
    if (i < nseg) segoff[i] = carry + ex;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
}

// Records grouped by segment: LDS ranks within the block, one global atomic
// per (block, segment) reserves the block's range of the segment.
__global__ void __launch_bounds__(256) seg_scatter_kernel(const PeakRecord* __restrict__ in,
                                                          const uint32_t* __restrict__ count, uint32_t cap,
                                                          uint32_t nseg, const uint32_t* __restrict__ segoff,
                                                          uint32_t* __restrict__ cursor, uint2* __restrict__ out) {
  __shared__ uint32_t lc[kSegLds];
  __shared__ uint32_t lb[kSegLds];
  const uint32_t n = min(*count, cap);
  const uint32_t base = blockIdx.x * 256u * kRecPerThread;
  if (base >= n) return;
  for (uint32_t i = threadIdx.x; i < nseg; i += 256) lc[i] = 0;
  __syncthreads();
  PeakRecord rec[kRecPerThread];
  uint32_t rank[kRecPerThread];
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    const uint32_t i = base + r * 256u + threadIdx.x;
    rec[r].seg = 0xffffffffu;
    if (i < n) {
      rec[r] = in[i];
      if (rec[r].seg < nseg) rank[r] = atomicAdd(&lc[rec[r].seg], 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nseg; i += 256)
    if (lc[i]) lb[i] = segoff[i] + atomicAdd(&cursor[i], lc[i]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r)
    if (rec[r].seg < nseg)
      out[lb[rec[r].seg] + rank[r]] = make_uint2(static_cast<uint32_t>(rec[r].idx), __float_as_uint(rec[r].snr));
}

// One workgroup per segment with lo_n < n <= CAP crossings (the small
// kernel also writes the empty segments' entries, the large one the raw
// entries of segments over its capacity).
template <uint32_t CAP, int kClThreads>
__global__ void __launch_bounds__(kClThreads) peak_cluster_kernel(const uint2* __restrict__ sorted,
                                                                  const uint32_t* __restrict__ segoff,
                                                                  const uint32_t* __restrict__ segcnt, int gap,
                                                                  uint32_t lo_n, uint2* __restrict__ out,
                                                                  uint2* __restrict__ segtab,
                                                                  uint32_t* __restrict__ total, int mode) {
  // mode bits 0-7: timing phase cut (PSOUP_CLUSTER_STOP); bit 8: register
  // stages in the sort (PSOUP_CLUSTER_RSORT=1, opt-in until measured on the GPU)
  const int stop_after = mode & 255;
  const bool rsort = (mode & 256) != 0;
  constexpr uint32_t R = (CAP + kClThreads - 1) / kClThreads;  // rows of kClThreads positions
  __shared__ uint2 key[CAP];      // (idx, snr bits)
  __shared__ uint16_t jmp[CAP];   // next survivor at/after a position, then chain jumps
  __shared__ uint8_t flag[CAP];   // bit 0: survives the window test, bit 1: cluster peak
  __shared__ uint32_t sc[kClThreads];
  __shared__ uint32_t wcnt[kClThreads / 64];   // per wave: first survivor of the row
  __shared__ uint32_t rw[R * (kClThreads / 64)];  // per (row, wave): peak count, then its output offset
  __shared__ uint32_t base_s, first_s;
  const int t = threadIdx.x;
  const uint32_t seg = blockIdx.x;
  const uint32_t n = segcnt[seg], off = segoff[seg];
  if (n <= lo_n || n > CAP) {
    if (t == 0) {
      if (n == 0 && lo_n == 0) segtab[seg] = make_uint2(0u, 0u);
      if (n > CAP && CAP > kClSmall) segtab[seg] = make_uint2(off, n | kClusterRaw);
    }
    return;
  }
  for (uint32_t i = t; i < n; i += kClThreads) key[i] = sorted[off + i];
  uint32_t P = 2;
  while (P < n) P <<= 1;
  __syncthreads();
  // bitonic sort with ascending comparators only (a "flip" stage then half
  // cleaners per merge size): positions >= n act as +inf and never move, so
  // comparators reaching them are skipped -- no padding.  Every stage whose
  // pairs lie inside one aligned 16-position chunk runs in registers: each
  // chunk is sorted there first (merge sizes 2..16), and after the LDS stages
  // of each larger merge size its last four half cleaners (j = 8, 4, 2, 1) are
  // one register pass -- 66 barriers and LDS round trips instead of 105 at
  // P = 16384 (opt-in, `rsort`; the all-LDS form is the default).
  auto cswap = [&](uint32_t lo, uint32_t hi) {
    const uint2 a = key[lo], b = key[hi];
    if (static_cast<int>(a.x) > static_cast<int>(b.x)) {
      key[lo] = b;
      key[hi] = a;
    }
  };
  constexpr int B = 16;
  auto rswap = [](uint2& a, uint2& b) {
    const bool sw = static_cast<int>(a.x) > static_cast<int>(b.x);
    const uint2 lo = sw ? b : a, hi = sw ? a : b;
    a = lo;
    b = hi;
  };
  auto chunk_pass = [&](bool full) {
    for (uint32_t c = t; c * B < P; c += kClThreads) {
      const uint32_t b0 = c * B;
      uint2 r[B];
#pragma unroll
      for (int i = 0; i < B; ++i) r[i] = b0 + i < n ? key[b0 + i] : make_uint2(0x7fffffffu, 0u);
      if (full) {
#pragma unroll
        for (int k = 2; k <= B; k <<= 1) {
#pragma unroll
          for (int i = 0; i < B; ++i)
            if ((i & (k >> 1)) == 0) rswap(r[i], r[i ^ (k - 1)]);
#pragma unroll
          for (int j = k >> 2; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < B; ++i)
              if ((i & j) == 0) rswap(r[i], r[i + j]);
        }
      } else {
#pragma unroll
        for (int j = B >> 1; j > 0; j >>= 1)
#pragma unroll
          for (int i = 0; i < B; ++i)
            if ((i & j) == 0) rswap(r[i], r[i + j]);
      }
#pragma unroll
      for (int i = 0; i < B; ++i)
        if (b0 + i < n) key[b0 + i] = r[i];
    }
    __syncthreads();
  };
  if (rsort) {
    chunk_pass(true);
    for (uint32_t k = 2 * B; k <= P; k <<= 1) {
      const uint32_t h = k >> 1;
      for (uint32_t q = t; q < P / 2; q += kClThreads) {
        const uint32_t lo = (q / h) * k + (q & (h - 1)), hi = lo ^ (k - 1);
        if (hi < n) cswap(lo, hi);
      }
      __syncthreads();
      for (uint32_t j = k >> 2; j >= static_cast<uint32_t>(B); j >>= 1) {
        for (uint32_t q = t; q < P / 2; q += kClThreads) {
          const uint32_t lo = 2 * j * (q / j) + (q & (j - 1)), hi = lo + j;
          if (hi < n) cswap(lo, hi);
        }
        __syncthreads();
      }
      chunk_pass(false);
    }
  } else {
    for (uint32_t k = 2; k <= P; k <<= 1) {
      const uint32_t h = k >> 1;
      for (uint32_t q = t; q < P / 2; q += kClThreads) {
        const uint32_t lo = (q / h) * k + (q & (h - 1)), hi = lo ^ (k - 1);
        if (hi < n) cswap(lo, hi);
      }
      __syncthreads();
      for (uint32_t j = k >> 2; j > 0; j >>= 1) {
        for (uint32_t q = t; q < P / 2; q += kClThreads) {
          const uint32_t lo = 2 * j * (q / j) + (q & (j - 1)), hi = lo + j;
          if (hi < n) cswap(lo, hi);
        }
        __syncthreads();
      }
    }
  }
  if (stop_after == 1) return;  // timing only (PSOUP_CLUSTER_STOP): load + sort
  // Every phase below gives position i = r * kClThreads + t to thread t
  // (row r): consecutive lanes touch consecutive LDS words, and wave ballots
  // order the survivors / peaks inside a row.
  constexpr uint32_t kW = kClThreads / 64;
  const uint32_t nrow = (n + kClThreads - 1) / kClThreads;
  const int lane = t & 63, w = t >> 6;
  // (1) window test
  uint32_t mysurv = 0;
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    if (i >= n) break;
    const int xi = static_cast<int>(key[i].x);
    const float si = __uint_as_float(key[i].y);
    bool keep = true;
    for (uint32_t j = i + 1; j < n && static_cast<int>(key[j].x) - xi < gap; ++j)
      if (__uint_as_float(key[j].y) > si) {
        keep = false;
        break;
      }
    flag[i] = keep ? 1 : 0;
    mysurv += keep ? 1u : 0u;
  }
  uint32_t totsurv;
  block_excl_sum<kClThreads>(mysurv, sc, &totsurv);  // (its barriers also publish flag)
  if (stop_after == 2) return;  // timing only: + window test
  // (3) next survivor at or after every position: rows from the last, a
  // row's waves from their ballots, the carry from the rows after it
  uint32_t carry = n;
  for (uint32_t r = nrow; r-- > 0;) {
    const uint32_t i = r * kClThreads + t;
    const bool sv = i < n && (flag[i] & 1);
    const uint64_t mask = __ballot(sv);
    if (lane == 0) wcnt[w] = mask ? r * kClThreads + w * 64 + static_cast<uint32_t>(__builtin_ctzll(mask)) : n;
    __syncthreads();
    uint32_t c = carry;
    for (int v = static_cast<int>(kW) - 1; v > w; --v) c = wcnt[v] < n ? wcnt[v] : c;
    const uint64_t ge = mask >> lane;
    if (i < n) jmp[i] = static_cast<uint16_t>(ge ? i + static_cast<uint32_t>(__builtin_ctzll(ge)) : c);
    uint32_t rowfirst = n;
    for (uint32_t v = 0; v < kW; ++v) rowfirst = min(rowfirst, wcnt[v]);
    carry = rowfirst < n ? rowfirst : carry;
    __syncthreads();
  }
  // next(i): the first survivor with idx >= idx_i + gap (at most gap - 1
  // positions ahead have smaller idx: distinct bins)
  uint32_t nx[R];
  if (t == 0) first_s = jmp[0];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = r * kClThreads + t;
    nx[r] = n;
    if (i < n && (flag[i] & 1)) {
      const int target = static_cast<int>(key[i].x) + gap;
      uint32_t p = i + 1;
      while (p < n && static_cast<int>(key[p].x) < target) ++p;
      nx[r] = p < n ? jmp[p] : n;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = r * kClThreads + t;
    if (i < n && (flag[i] & 1)) jmp[i] = static_cast<uint16_t>(nx[r]);
  }
  __syncthreads();
  if (t == 0 && first_s < n) flag[first_s] = 3;
  __syncthreads();
  if (stop_after == 3) return;  // timing only: + next survivor / next()
  // (2) the chain from the first survivor, by pointer doubling: after round
  // m every survivor within 2^(m+1) - 1 jumps of the start is marked
  for (uint32_t span = 1; span < totsurv; span <<= 1) {
    uint32_t tgt[R], nj[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = r * kClThreads + t;
      tgt[r] = n;
      nj[r] = n;
      if (i < n && (flag[i] & 1)) {
        const uint32_t j = jmp[i];
        if (j < n) {
          if (flag[i] & 2) tgt[r] = j;
          nj[r] = jmp[j];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = r * kClThreads + t;
      if (tgt[r] < n) flag[tgt[r]] = 3;
      if (i < n && (flag[i] & 1)) jmp[i] = static_cast<uint16_t>(nj[r]);
    }
    __syncthreads();
  }
  if (stop_after == 4) return;  // timing only: + chain marking
  // compaction of the peaks in idx order: per (row, wave) counts, their
  // exclusive scan (one thread), then ballot ranks inside each wave
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    const uint64_t mask = __ballot(i < n && (flag[i] >> 1));
    if (lane == 0) rw[r * kW + w] = static_cast<uint32_t>(__builtin_popcountll(mask));
  }
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (uint32_t q = 0; q < nrow * kW; ++q) {
      const uint32_t c = rw[q];
      rw[q] = acc;
      acc += c;
    }
    base_s = atomicAdd(total, acc);
    segtab[seg] = make_uint2(base_s, acc);
  }
  __syncthreads();
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    const bool pk = i < n && (flag[i] >> 1);
    const uint64_t mask = __ballot(pk);
    if (pk)
      out[base_s + rw[r * kW + w] + static_cast<uint32_t>(__builtin_popcountll(mask & ((1ull << lane) - 1)))] = key[i];
  }
}

// Fallbacks for batches with more than kSegLds segments: one global atomic per record.
__global__ void __launch_bounds__(256) seg_hist_global_kernel(const PeakRecord* __restrict__ in,
                                                              const uint32_t* __restrict__ count, uint32_t cap,
                                                              uint32_t nseg, uint32_t* __restrict__ segcnt) {
  const uint32_t n = min(*count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t sg = in[i].seg;
    if (sg < nseg) atomicAdd(&segcnt[sg], 1u);
  }
}

__global__ void __launch_bounds__(256) seg_scatter_global_kernel(const PeakRecord* __restrict__ in,
                                                                 const uint32_t* __restrict__ count, uint32_t cap,
                                                                 uint32_t nseg, const uint32_t* __restrict__ segoff,
                                                                 uint32_t* __restrict__ cursor,
                                                                 uint2* __restrict__ out) {
  const uint32_t n = min(*count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const PeakRecord r = in[i];
    if (r.seg >= nseg) continue;
    const uint32_t pos = segoff[r.seg] + atomicAdd(&cursor[r.seg], 1u);
    out[pos] = make_uint2(static_cast<uint32_t>(r.idx), __float_as_uint(r.snr));
  }
}

}  // namespace

void peak_cluster_batch(const PeakRecord* d_peaks, const uint32_t* d_count, uint32_t cap, uint32_t nseg, int gap,
                        uint32_t* d_work, uint2* d_sorted, uint2* d_out, uint2* d_segtab, uint32_t* d_total,
                        hipStream_t s) {
  if (nseg == 0) return;
  PSOUP_CHECK(gap >= 1, "peak_cluster_batch: gap must be positive");
  uint32_t* segcnt = d_work;
  uint32_t* segoff = d_work + nseg;
  uint32_t* cursor = d_work + 2 * nseg;
  PSOUP_HIP_CHECK(hipMemsetAsync(d_work, 0, 3ull * nseg * sizeof(uint32_t), s));
  PSOUP_HIP_CHECK(hipMemsetAsync(d_total, 0, sizeof(uint32_t), s));
  if (nseg <= static_cast<uint32_t>(kSegLds)) {
    const uint64_t per = 256ull * kRecPerThread;
    const unsigned g = static_cast<unsigned>(std::max<uint64_t>(1, (static_cast<uint64_t>(cap) + per - 1) / per));
    seg_hist_kernel<<<g, 256, 0, s>>>(d_peaks, d_count, cap, nseg, segcnt);
    post_launch_check("seg_hist_kernel", s);
    seg_scan_kernel<<<1, kClThreads, 0, s>>>(segcnt, nseg, segoff);
    post_launch_check("seg_scan_kernel", s);
    seg_scatter_kernel<<<g, 256, 0, s>>>(d_peaks, d_count, cap, nseg, segoff, cursor, d_sorted);
    post_launch_check("seg_scatter_kernel", s);
  } else {
    const unsigned g = dev::grid_for(cap, 256, 4096);
    seg_hist_global_kernel<<<g, 256, 0, s>>>(d_peaks, d_count, cap, nseg, segcnt);
    post_launch_check("seg_hist_global_kernel", s);
    seg_scan_kernel<<<1, kClThreads, 0, s>>>(segcnt, nseg, segoff);
    post_launch_check("seg_scan_kernel", s);
    seg_scatter_global_kernel<<<g, 256, 0, s>>>(d_peaks, d_count, cap, nseg, segoff, cursor, d_sorted);
    post_launch_check("seg_scatter_global_kernel", s);
  }
  static const int stop = [] {  // timing experiments only: end the kernels after a phase
    const char* e = std::getenv("PSOUP_CLUSTER_STOP");
    const char* r = std::getenv("PSOUP_CLUSTER_RSORT");
    return (e ? std::atoi(e) : 99) | (r && std::atoi(r) == 1 ? 256 : 0);
  }();
  peak_cluster_kernel<kClSmall, kClThreads><<<nseg, kClThreads, 0, s>>>(d_sorted, segoff, segcnt, gap, 0u, d_out,
                                                                         d_segtab, d_total, stop);
  post_launch_check("peak_cluster_kernel<small>", s);
  // the large kernel holds a CU's LDS alone: 1024 threads (16 waves) hide the
  // LDS latency of its dependent sort / scan steps (PSOUP_CLUSTER_TH=512: the
  // previous shape)
  static const bool th512 = [] {
    const char* e = std::getenv("PSOUP_CLUSTER_TH");
    return e && std::atoi(e) == 512;
  }();
  if (th512)
    peak_cluster_kernel<kClusterCap, 512><<<nseg, 512, 0, s>>>(d_sorted, segoff, segcnt, gap, kClSmall, d_out,
                                                                d_segtab, d_total, stop);
  else
    peak_cluster_kernel<kClusterCap, 1024><<<nseg, 1024, 0, s>>>(d_sorted, segoff, segcnt, gap, kClSmall, d_out,
                                                                  d_segtab, d_total, stop);
  post_launch_check("peak_cluster_kernel<large>", s);
}

}  // namespace kern
}  // namespace psoup
