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
// Input: the harmonic kernel's records (harmsum.hip emit_levels): every
// (wave, bin group, level) with crossings wrote one chunk -- a descriptor
// {kPeakChunk | count << 16 | segment, first idx, position} and its `count`
// crossings, idx-ascending, at that position.  Chunks of one segment cover
// disjoint 64-bin groups, so the segment in idx order is its chunks in
// first-idx order: only the descriptors (~1/20 of the records on dense RFI
// spectra) are grouped by segment and sorted.
// peak_cluster_kernel: one workgroup per segment (trial x level): radix
// sort of its chunk descriptors in LDS, the crossings gathered in idx order,
// the window test (1) and next() in parallel (a suffix scan gives the next
// survivor at or after any position), each run's chain followed by the thread
// of its start, a scan compacts the peaks in idx order.  Segments over
// kClusterCap crossings are left to the host (flagged in the segment table
// with their raw, unsorted range).
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

// A chunk descriptor's segment and crossing count (kPeakChunk records only).
__device__ __forceinline__ uint32_t chunk_seg(uint32_t f) { return f & 0xffffu; }
__device__ __forceinline__ uint32_t chunk_count(uint32_t f) { return (f >> 16) & 0x7fu; }
// A descriptor the clustering may use: its segment in the batch and all its
// crossings written (a batch over the record capacity -- recomputed by the
// engine with a larger buffer -- has chunks cut at the capacity: those are
// skipped, so no kernel reads past the n records held).
__device__ __forceinline__ bool chunk_ok(const PeakRecord& r, uint32_t nseg, uint32_t n) {
  return (r.seg & kPeakChunk) && chunk_seg(r.seg) < nseg &&
         static_cast<uint64_t>(__float_as_uint(r.snr)) + chunk_count(r.seg) <= n;
}

// Where the records are (kernels.hpp kPeakRegionStride): 2^log2 regions of
// capr records, region r's count at count[r * kPeakRegionStride] (log2 = 0:
// one region, count[0], capr = the capacity).
struct RecRegions {
  const uint32_t* count;
  uint32_t capr;
  int log2;
};
// the end (absolute, exclusive) of the records held in the region of position i
__device__ __forceinline__ uint32_t region_end(const RecRegions& g, uint32_t i) {
  const uint32_t r = g.log2 ? i / g.capr : 0u;
  return r * g.capr + min(g.count[r * kPeakRegionStride], g.capr);
}

// Per-segment chunk and crossing counts: each block counts its descriptors
// in LDS and adds the non-zero counts to the global ones (one atomic per
// block and segment).
__global__ void __launch_bounds__(256) seg_hist_kernel(const PeakRecord* __restrict__ in, RecRegions g,
                                                       uint32_t nseg, uint32_t* __restrict__ segcnt,
                                                       uint32_t* __restrict__ segdcnt) {
  __shared__ uint32_t lr[kSegLds], lc[kSegLds];
  const uint32_t base = blockIdx.x * 256u * kRecPerThread;
  const uint32_t n = region_end(g, base);  // blocks never straddle regions (capr % 4096 == 0)
  if (base >= n) return;
  for (uint32_t i = threadIdx.x; i < nseg; i += 256) lr[i] = lc[i] = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    const uint32_t i = base + r * 256u + threadIdx.x;
    if (i < n) {
      const PeakRecord r = in[i];
      if (chunk_ok(r, nseg, n)) {
        atomicAdd(&lc[chunk_seg(r.seg)], 1u);
        atomicAdd(&lr[chunk_seg(r.seg)], chunk_count(r.seg));
      }
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nseg; i += 256)
    if (lc[i]) {
      atomicAdd(&segdcnt[i], lc[i]);
      atomicAdd(&segcnt[i], lr[i]);
    }
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

// Chunk descriptors grouped by segment as {first idx, position, count}: LDS
// ranks within the block, one global atomic per (block, segment) reserves
// the block's range of the segment.
__global__ void __launch_bounds__(256) seg_scatter_kernel(const PeakRecord* __restrict__ in, RecRegions g,
                                                          uint32_t nseg, const uint32_t* __restrict__ segdoff,
                                                          uint32_t* __restrict__ cursor, uint4* __restrict__ out) {
  __shared__ uint32_t lc[kSegLds];
  __shared__ uint32_t lb[kSegLds];
  const uint32_t base = blockIdx.x * 256u * kRecPerThread;
  const uint32_t n = region_end(g, base);
  if (base >= n) return;
  for (uint32_t i = threadIdx.x; i < nseg; i += 256) lc[i] = 0;
  __syncthreads();
  PeakRecord rec[kRecPerThread];
  uint32_t rank[kRecPerThread];
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    const uint32_t i = base + r * 256u + threadIdx.x;
    rec[r].seg = 0u;
    if (i < n) {
      rec[r] = in[i];
      if (!chunk_ok(rec[r], nseg, n)) rec[r].seg = 0u;
      else rank[r] = atomicAdd(&lc[chunk_seg(rec[r].seg)], 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nseg; i += 256)
    if (lc[i]) lb[i] = segdoff[i] + atomicAdd(&cursor[i], lc[i]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r)
    if (rec[r].seg & kPeakChunk)
      out[lb[chunk_seg(rec[r].seg)] + rank[r]] = make_uint4(static_cast<uint32_t>(rec[r].idx),
                                                             __float_as_uint(rec[r].snr), chunk_count(rec[r].seg), 0u);
}

// Phase timestamps (tools/expt/cluster_bench.py --trace): when set, thread 0
// of each workgroup of the large kernel records the wall clock (100 MHz) at
// fixed points; a scalar load of a __constant__ pointer, nothing else.
__constant__ unsigned long long* g_cl_trace = nullptr;
constexpr int kClTraceEvents = 8;
__device__ __forceinline__ void cl_trace(int ev) {
  unsigned long long* tr = g_cl_trace;
  if (tr != nullptr && threadIdx.x == 0) tr[blockIdx.x * kClTraceEvents + ev] = wall_clock64();
}

// Exclusive scan of one value per thread over the block (TH threads): wave
// scans by shuffles, one wave scans the wave totals; two barriers.
template <int TH>
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t* wtot, uint32_t* total) {
  constexpr int W = TH / 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(incl, off, 64);
    if (lane >= off) incl += u;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  if (w == 0) {
    uint32_t x = lane < W ? wtot[lane] : 0u, xi = x;
#pragma unroll
    for (int off = 1; off < W; off <<= 1) {
      const uint32_t u = __shfl_up(xi, off, 64);
      if (lane >= off) xi += u;
    }
    if (lane < W) wtot[lane] = xi - x;  // exclusive wave offsets
    if (lane == W - 1 && total) *total = xi;
  }
  __syncthreads();
  return wtot[w] + incl - v;
}

// One workgroup per segment with lo_n < n <= CAP crossings (the small
// kernel also writes the empty segments' entries, the large one the raw
// entries of segments over its capacity).
//
// 1. Order the segment's m chunk descriptors by first idx: a rank sort (each
//    thread counts the smaller first idx among all m, broadcast LDS reads)
//    when m <= kClThreads -- the usual case: dense RFI runs give ~40
//    crossings per chunk -- else an LSD radix sort with 4-bit digits of
//    first idx - min (keys in registers between passes, stable ranks by wave
//    ballots, counts scanned per (digit, row, wave)).  The sorted chunk
//    indices end in the jump table.
// 2. Gather the crossings in idx order into LDS as two arrays (idx, snr):
//    sorted chunk p starts at the counts of chunks 0 .. p-1.
// 3. Window test, next() and run starts from the 32 positions after (or
//    before) a crossing, fetched as independent 16-byte LDS reads of the idx
//    / snr / flag arrays -- not a dependent walk (gap - 1 <= 29 positions
//    can lie within the gap: distinct bins).
// 4. The next survivor at or after every position (per-row ballots, rows
//    from the last), each run's chain followed by its start's thread, and a
//    compaction of the peaks in idx order.
template <uint32_t CAP, int kClThreads>
__global__ void __launch_bounds__(kClThreads) peak_cluster_kernel(const PeakRecord* __restrict__ recs,
                                                                  const uint4* __restrict__ desc,
                                                                  const uint32_t* __restrict__ segoff,
                                                                  const uint32_t* __restrict__ segcnt,
                                                                  const uint32_t* __restrict__ segdoff,
                                                                  const uint32_t* __restrict__ segdcnt, int gap,
                                                                  uint32_t lo_n, uint2* __restrict__ out,
                                                                  uint2* __restrict__ segtab,
                                                                  uint32_t* __restrict__ total,
                                                                  uint2* __restrict__ raw) {
  constexpr uint32_t R = (CAP + kClThreads - 1) / kClThreads;  // rows of kClThreads positions
  constexpr uint32_t kW = kClThreads / 64;
  constexpr uint32_t kCnt = 16 * R * kW;  // radix counts (digit, row, wave)
  constexpr uint32_t kPad = 36;           // window reads run up to 35 positions past / before the data
  // crossings: idx at kidx[kPad + i], snr at ksnr[kPad + i]; before the gather
  // the same memory holds the radix sort's (first idx, chunk) keys
  __shared__ __attribute__((aligned(16))) uint32_t kmem[2 * (CAP + 2 * kPad)];
  __shared__ uint16_t jmp[CAP > 2 * kCnt ? CAP : 2 * kCnt];  // sorted chunks, then next survivor / chain jumps
  __shared__ __attribute__((aligned(16))) uint8_t flag[CAP + 2 * kPad];  // at kPad + i: bit 0 survivor, 1 peak, 2 run start
  __shared__ uint32_t sc[kClThreads];
  __shared__ uint32_t rw[R * (kClThreads / 64)];  // per (row, wave): peak count, then its output offset
  __shared__ uint32_t base_s, lo_s, hi_s;
  uint32_t* const kidx = kmem;
  float* const ksnr = reinterpret_cast<float*>(kmem + CAP + 2 * kPad);
  uint2* const key = reinterpret_cast<uint2*>(kmem);  // radix keys (first idx, chunk)
  const int t = threadIdx.x;
  // workgroups go round-robin over the 8 XCDs and the segment ids are trial
  // x 8 + level, so blockIdx = segment would put every trial's level-h segment
  // on XCD h (the big high levels of a peak-heavy batch on 2 of 8 XCDs): XCD
  // x takes the contiguous eighth x of the segments instead (all levels)
  const uint32_t nseg = gridDim.x;
  const uint32_t seg = (nseg & 7u) == 0 ? (blockIdx.x & 7u) * (nseg >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const uint32_t n = segcnt[seg];                        // crossings
  const uint32_t m = segdcnt[seg], doff = segdoff[seg];  // chunks
  const uint4* dsc = desc + doff;
  if (n <= lo_n || n > CAP) {
    if (n == 0 && lo_n == 0 && t == 0) segtab[seg] = make_uint2(0u, 0u);
    if (n > CAP && CAP > kClSmall) {
      // over capacity: the raw crossings (any order) at raw[segoff ..] for the
      // host; chunk j's crossings after chunks 0 .. j-1's
      uint32_t carry = 0;
      for (uint32_t j0 = 0; j0 < m; j0 += kClThreads) {
        const uint32_t j = j0 + t;
        const uint4 d = j < m ? dsc[j] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t ex = block_scan_excl<kClThreads>(d.z, sc, &base_s);
        const uint32_t tot = base_s;
        for (uint32_t q = 0; q < d.z; ++q) {
          const PeakRecord r = recs[d.y + q];
          raw[segoff[seg] + carry + ex + q] = make_uint2(static_cast<uint32_t>(r.idx), __float_as_uint(r.snr));
        }
        carry += tot;
        __syncthreads();
      }
      if (t == 0) segtab[seg] = make_uint2(segoff[seg], n | kClusterRaw);
    }
    return;
  }
  const int lane = t & 63, w = t >> 6;
  if (CAP > kClSmall) cl_trace(0);
  // ---- 1. chunk order -> jmp[p] = chunk at sorted position p
  if (m <= static_cast<uint32_t>(kClThreads)) {
    uint32_t* fi = kmem;  // first idx of every chunk (distinct: disjoint 64-bin groups)
    const uint32_t mine = t < static_cast<int>(m) ? dsc[t].x : 0u;
    if (t < static_cast<int>(m)) fi[t] = mine;
    if (t < 4) fi[m + t] = 0xffffffffu;  // pad to a multiple of four
    __syncthreads();
    if (t < static_cast<int>(m)) {
      uint32_t rank = 0;
      const uint4* f4 = reinterpret_cast<const uint4*>(fi);
      for (uint32_t j = 0; j < (m + 3) / 4; ++j) {
        const uint4 v = f4[j];  // every lane reads the same 16 bytes: a broadcast
        rank += (v.x < mine) + (v.y < mine) + (v.z < mine) + (v.w < mine);
      }
      jmp[rank] = static_cast<uint16_t>(t);
    }
    __syncthreads();
  } else {
    uint2 kv[R];
    int lo = 0x7fffffff, hi = -0x7fffffff;
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = r * kClThreads + t;
      kv[r] = i < m ? make_uint2(dsc[i].x, i) : make_uint2(0u, 0u);
      if (i < m) {
        lo = min(lo, static_cast<int>(kv[r].x));
        hi = max(hi, static_cast<int>(kv[r].x));
      }
    }
    if (t == 0) {
      lo_s = 0x7fffffffu;
      hi_s = 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    __syncthreads();
    if (lane == 0) {
      atomicMin(&lo_s, static_cast<uint32_t>(lo));
      atomicMax(&hi_s, static_cast<uint32_t>(hi));
    }
    __syncthreads();
    const uint32_t base = lo_s, span = hi_s - lo_s;
    const int passes = span == 0 ? 1 : (32 - __builtin_clz(span) + 3) / 4;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(jmp);  // [digit][row][wave]
    constexpr uint32_t kPer = (kCnt + kClThreads - 1) / kClThreads;  // counts scanned per thread
    for (int ps = 0; ps < passes; ++ps) {
      const int shift = 4 * ps;
      uint32_t dig[R], rank[R];
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) {
        const uint32_t i = r * kClThreads + t;
        dig[r] = i < m ? ((kv[r].x - base) >> shift) & 15u : 16u;
        rank[r] = 0;
        if (r * kClThreads + w * 64 < m) {  // wave-uniform: the row's wave holds keys
#pragma unroll
          for (uint32_t d = 0; d < 16; ++d) {
            const uint64_t mk = __ballot(dig[r] == d);
            if (dig[r] == d) rank[r] = static_cast<uint32_t>(__builtin_popcountll(mk & ((1ull << lane) - 1)));
            if (lane == 0) cnt[(d * R + r) * kW + w] = static_cast<uint32_t>(__builtin_popcountll(mk));
          }
        } else if (lane == 0) {
#pragma unroll
          for (uint32_t d = 0; d < 16; ++d) cnt[(d * R + r) * kW + w] = 0u;
        }
      }
      __syncthreads();
      {
        uint32_t loc[kPer], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
          const uint32_t e = t * kPer + q;
          loc[q] = e < kCnt ? cnt[e] : 0u;
          sum += loc[q];
        }
        uint32_t run = block_scan_excl<kClThreads>(sum, sc, nullptr);
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
          const uint32_t e = t * kPer + q;
          if (e < kCnt) cnt[e] = run;
          run += loc[q];
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t r = 0; r < R; ++r)
        if (dig[r] < 16) key[cnt[(dig[r] * R + r) * kW + w] + rank[r]] = kv[r];
      __syncthreads();
#pragma unroll
      for (uint32_t r = 0; r < R; ++r) {
        const uint32_t i = r * kClThreads + t;
        if (i < m) kv[r] = key[i];
      }
      __syncthreads();  // the next pass's counts and scatter overwrite cnt / key
    }
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = r * kClThreads + t;
      if (i < m) jmp[i] = static_cast<uint16_t>(kv[r].y);
    }
    __syncthreads();
  }
  if (CAP > kClSmall) cl_trace(1);
  // ---- 2. the crossings in idx order (thread t owns the consecutive sorted
  // chunks [t q, t q + q))
  {
    const uint32_t q = (m + kClThreads - 1) / kClThreads;
    const uint32_t p0 = t * q, p1 = min(m, p0 + q);
    uint32_t sum = 0;
    for (uint32_t p = p0; p < p1; ++p) sum += dsc[jmp[p]].z;
    uint32_t dst = kPad + block_scan_excl<kClThreads>(sum, sc, nullptr);
    for (uint32_t p = p0; p < p1; ++p) {
      const uint4 d = dsc[jmp[p]];
      for (uint32_t c = 0; c < d.z; ++c) {
        const PeakRecord r = recs[d.y + c];
        kidx[dst + c] = static_cast<uint32_t>(r.idx);
        ksnr[dst + c] = r.snr;
      }
      dst += d.z;
    }
    // pads: idx far outside every window (before: never within the gap,
    // after: never below a target); flags clear
    if (t < static_cast<int>(kPad)) {
      kidx[t] = 0x80000000u;  // as int: below everything
      ksnr[t] = 0.f;
      kidx[kPad + n + t] = 0x7fffffffu;
      ksnr[kPad + n + t] = 0.f;
      flag[t] = 0;
      flag[kPad + n + t] = 0;
    }
    __syncthreads();
  }
  if (CAP > kClSmall) cl_trace(2);
  // Every phase below gives position i = r * kClThreads + t to thread t
  // (row r): consecutive lanes touch consecutive LDS words, and wave ballots
  // order the survivors / peaks inside a row.
  const uint32_t nrow = (n + kClThreads - 1) / kClThreads;
  // ---- 3a. window test: survives iff no strictly larger crossing among the
  // following positions within the gap (at most 29 of them).  The window's
  // end p (the first position with idx >= idx_i + gap) comes first -- a run of
  // consecutive bins reaches it exactly gap positions ahead, else a 5-step
  // binary search (past n the pads read 0x7fffffff) -- so the 32 S/N values
  // after i need one compare each, their bits masked to the window; p - i - 1
  // (<= 29) is kept in flag bits 3..7 for 3c
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    if (i >= n) break;
    const int xi = static_cast<int>(kidx[kPad + i]);
    const float si = ksnr[kPad + i];
    const int tgt = xi + gap;
    uint32_t cnt;  // window positions i + 1 .. i + cnt
    if (i + gap < n && static_cast<int>(kidx[kPad + i + gap]) == tgt) {
      cnt = static_cast<uint32_t>(gap) - 1;
    } else {
      cnt = 0;
#pragma unroll
      for (uint32_t st = 16; st >= 1; st >>= 1)
        if (static_cast<int>(kidx[kPad + i + cnt + st]) < tgt) cnt += st;
    }
    const uint32_t a = (kPad + i + 1) & ~3u, sh = (kPad + i + 1) - a;  // aligned base, offset of i + 1 (0..3)
    const uint32_t win = ((1u << cnt) - 1u) << sh;                     // bits of positions a + off in the window
    uint32_t gt = 0;                                                   // bit off: S/N at a + off above si
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const float4 sv = *reinterpret_cast<const float4*>(ksnr + a + 4 * v);
      const float ss[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) gt |= ss[e] > si ? (1u << (4 * v + e)) : 0u;
    }
    flag[kPad + i] = static_cast<uint8_t>(((gt & win) == 0 ? 1u : 0u) | (cnt << 3));
  }
  __syncthreads();
  if (CAP > kClSmall) cl_trace(3);
  // ---- 3b. next survivor at or after every position, with two barriers:
  // the first survivor of every 64-position block (a wave's part of a row,
  // block q = r kW + w covers positions 64 q ..), one wave's suffix minimum
  // over the blocks, then each position from its own wave's ballot or the
  // suffix of the blocks after its own
  const uint32_t nblk = nrow * kW;
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    const uint64_t mask = __ballot(i < n && (flag[kPad + i] & 1));
    if (lane == 0) rw[r * kW + w] = mask ? r * kClThreads + w * 64 + static_cast<uint32_t>(__builtin_ctzll(mask)) : n;
  }
  __syncthreads();
  if (w == 0) {
    constexpr uint32_t kPerB = (R * kW + 63) / 64;  // blocks per lane
    uint32_t v[kPerB + 1];
    v[kPerB] = n;
#pragma unroll
    for (int e = static_cast<int>(kPerB) - 1; e >= 0; --e) {
      const uint32_t q = static_cast<uint32_t>(lane) * kPerB + static_cast<uint32_t>(e);
      v[e] = min(q < nblk ? rw[q] : n, v[e + 1]);
    }
    uint32_t x = v[0];  // suffix minimum over the lanes from this one
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_down(x, off, 64);
      if (lane + off < 64) x = min(x, y);
    }
    uint32_t after = __shfl_down(x, 1, 64);  // the lanes after this one
    if (lane == 63) after = n;
#pragma unroll
    for (uint32_t e = 0; e < kPerB; ++e) {
      const uint32_t q = static_cast<uint32_t>(lane) * kPerB + e;
      if (q < nblk) sc[q] = min(v[e], after);  // first survivor at or after block q
    }
  }
  __syncthreads();
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    const uint64_t ge = __ballot(i < n && (flag[kPad + i] & 1)) >> lane;
    const uint32_t q = r * kW + w;
    const uint32_t nxt = q + 1 < nblk ? sc[q + 1] : n;
    if (i < n) jmp[i] = static_cast<uint16_t>(ge ? i + static_cast<uint32_t>(__builtin_ctzll(ge)) : nxt);
  }
  __syncthreads();
  if (CAP > kClSmall) cl_trace(4);
  // ---- 3c. next(i): the first survivor with idx >= idx_i + gap = the next
  // survivor from the first position not below that target; a survivor
  // starts a run when no survivor lies within the gap before it (bit 2).
  // Both are written in place: a survivor's own jump entry is never read
  // here (the next survivor at or after a survivor is itself), and bit 2
  // leaves the survivor bit readers test unchanged -- so the row loop keeps
  // no per-row registers and stays a loop.
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    if (i >= n || !(flag[kPad + i] & 1)) continue;
    const int xi = static_cast<int>(kidx[kPad + i]);
    // the first position with idx >= idx_i + gap (3a's window end)
    const uint32_t p = i + 1 + (static_cast<uint32_t>(flag[kPad + i]) >> 3);
    const uint32_t nx = p < n ? ((flag[kPad + p] & 1) ? p : jmp[p]) : n;
    // run start: no survivor within the gap before i; fast path: the
    // previous position is a survivor within the gap.  Else k = the first
    // position with idx > idx_i - gap (a binary search over the 32 before i;
    // the pads before position 0 read as far below), and i starts a run iff
    // the next survivor at or after k is i itself (a survivor's own entry:
    // itself; a non-survivor's jump entry is never overwritten here)
    bool start = true;
    if (i > 0 && (flag[kPad + i - 1] & 1) && xi - static_cast<int>(kidx[kPad + i - 1]) < gap) {
      start = false;
    } else {
      const int lim = xi - gap;  // (pads: INT_MIN, at or below every limit)
      uint32_t far = 0;          // positions of [i - 32, i) at or below idx_i - gap: a prefix
#pragma unroll
      for (uint32_t st = 16; st >= 1; st >>= 1)
        if (static_cast<int>(kidx[kPad + i - 32 + far + st - 1]) <= lim) far += st;
      const uint32_t k = i - 32 + far + (static_cast<int>(kidx[kPad + i - 32 + far]) <= lim ? 1u : 0u);
      const uint32_t ns = k >= i ? i : ((flag[kPad + k] & 1) ? k : static_cast<uint32_t>(jmp[k]));
      start = ns >= i;
    }
    jmp[i] = static_cast<uint16_t>(nx);
    if (start) flag[kPad + i] = 5;
  }
  __syncthreads();
  if (CAP > kClSmall) cl_trace(5);
  // ---- 4. the chains: within a run an anchor never moves, so the run's
  // peaks are its start, then next(), next(next()), ... until the chain
  // reaches the following run's start; each run start's thread follows its run
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    if (i >= n || !(flag[kPad + i] & 4)) continue;
    uint32_t p = i;
    do {
      flag[kPad + p] = static_cast<uint8_t>(flag[kPad + p] | 2);
      p = jmp[p];
    } while (p < n && !(flag[kPad + p] & 4));
  }
  __syncthreads();
  if (CAP > kClSmall) cl_trace(6);
  // compaction of the peaks in idx order: per (row, wave) counts, their
  // exclusive scan, then ballot ranks inside each wave
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    const uint64_t mask = __ballot(i < n && (flag[kPad + i] & 2));
    if (lane == 0) rw[r * kW + w] = static_cast<uint32_t>(__builtin_popcountll(mask));
  }
  __syncthreads();
  {
    static_assert(R * kW <= kClThreads, "one (row, wave) count per thread");
    const uint32_t v = static_cast<uint32_t>(t) < nrow * kW ? rw[t] : 0u;
    const uint32_t ex = block_scan_excl<kClThreads>(v, sc, &base_s);
    if (static_cast<uint32_t>(t) < nrow * kW) rw[t] = ex;
    __syncthreads();
    const uint32_t acc = base_s;  // the segment's peak count
    __syncthreads();
    if (t == 0) {
      base_s = atomicAdd(total, acc);
      segtab[seg] = make_uint2(base_s, acc);
    }
  }
  __syncthreads();
  for (uint32_t r = 0; r < nrow; ++r) {
    const uint32_t i = r * kClThreads + t;
    const bool pk = i < n && (flag[kPad + i] & 2);
    const uint64_t mask = __ballot(pk);
    if (pk)
      out[base_s + rw[r * kW + w] + static_cast<uint32_t>(__builtin_popcountll(mask & ((1ull << lane) - 1)))] =
          make_uint2(kidx[kPad + i], __float_as_uint(ksnr[kPad + i]));
  }
  if (CAP > kClSmall) cl_trace(7);
}

// Fallbacks for batches with more than kSegLds segments: one global atomic per descriptor.
__global__ void __launch_bounds__(256) seg_hist_global_kernel(const PeakRecord* __restrict__ in, RecRegions g,
                                                              uint32_t cap, uint32_t nseg,
                                                              uint32_t* __restrict__ segcnt,
                                                              uint32_t* __restrict__ segdcnt) {
  const uint32_t lim = g.log2 ? cap : min(*g.count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += gridDim.x * blockDim.x) {
    const uint32_t n = region_end(g, i);
    if (i >= n) continue;
    const PeakRecord r = in[i];
    if (chunk_ok(r, nseg, n)) {
      atomicAdd(&segdcnt[chunk_seg(r.seg)], 1u);
      atomicAdd(&segcnt[chunk_seg(r.seg)], chunk_count(r.seg));
    }
  }
}

__global__ void __launch_bounds__(256) seg_scatter_global_kernel(const PeakRecord* __restrict__ in, RecRegions g,
                                                                 uint32_t cap, uint32_t nseg,
                                                                 const uint32_t* __restrict__ segdoff,
                                                                 uint32_t* __restrict__ cursor,
                                                                 uint4* __restrict__ out) {
  const uint32_t lim = g.log2 ? cap : min(*g.count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += gridDim.x * blockDim.x) {
    const uint32_t n = region_end(g, i);
    if (i >= n) continue;
    const PeakRecord r = in[i];
    if (!chunk_ok(r, nseg, n)) continue;
    const uint32_t sg = chunk_seg(r.seg);
    out[segdoff[sg] + atomicAdd(&cursor[sg], 1u)] =
        make_uint4(static_cast<uint32_t>(r.idx), __float_as_uint(r.snr), chunk_count(r.seg), 0u);
  }
}

// The regions' total into *total, or 2^log2 x the fullest region's count
// when one overflowed (> the capacity: the engine's re-run with a larger
// buffer then fits every region).
__global__ void __launch_bounds__(64) peak_regions_total_kernel(const uint32_t* __restrict__ count, int log2,
                                                                uint32_t capr, uint32_t* __restrict__ total) {
  const uint32_t R = 1u << log2;
  unsigned long long sum = 0;
  uint32_t mx = 0;
  for (uint32_t r = threadIdx.x; r < R; r += 64) {
    const uint32_t c = count[r * kPeakRegionStride];
    sum += c;
    mx = max(mx, c);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    sum += __shfl_xor(sum, off, 64);
    mx = max(mx, __shfl_xor(mx, off, 64));
  }
  if (threadIdx.x == 0)
    *total = mx > capr ? static_cast<uint32_t>(min(static_cast<unsigned long long>(mx) << log2, 0x80000000ull))
                       : static_cast<uint32_t>(sum);
}

}  // namespace

void peak_regions_total(const uint32_t* d_rcount, int region_log2, uint32_t cap, uint32_t* d_total, hipStream_t s) {
  PSOUP_CHECK(region_log2 >= 0 && region_log2 <= 8 && cap % (1u << region_log2) == 0, "peak_regions_total: regions");
  peak_regions_total_kernel<<<1, 64, 0, s>>>(d_rcount, region_log2, cap >> region_log2, d_total);
  post_launch_check("peak_regions_total_kernel", s);
}

void peak_cluster_set_trace(unsigned long long* d_events) {
  PSOUP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_cl_trace), &d_events, sizeof(d_events)));
}

void peak_cluster_batch(const PeakRecord* d_peaks, const uint32_t* d_count, uint32_t cap, uint32_t nseg, int gap,
                        uint32_t* d_work, uint2* d_sorted, uint2* d_out, uint2* d_segtab, uint32_t* d_total,
                        hipStream_t s, int region_log2) {
  if (nseg == 0) return;
  PSOUP_CHECK(region_log2 >= 0 && region_log2 <= 8 &&
                  (region_log2 == 0 || (cap >> region_log2) % (256u * kRecPerThread) == 0) &&
                  cap % (1u << region_log2) == 0,
              "peak_cluster_batch: record regions must be whole multiples of 4096 records");
  const RecRegions rg{d_count, cap >> region_log2, region_log2};
  // the window phases read the 32 positions next to a crossing: gap - 1 <= 29
  // of them can lie within the gap (the reference's min_gap is 30)
  PSOUP_CHECK(gap >= 1 && gap <= 30, "peak_cluster_batch: gap must be in [1, 30]");
  PSOUP_CHECK(nseg <= 65536, "peak_cluster_batch: segment ids are 16-bit in the chunk descriptors");
  uint32_t* segcnt = d_work;              // crossings per segment
  uint32_t* segoff = d_work + nseg;       // their exclusive scan (raw segments' offsets)
  uint32_t* segdcnt = d_work + 2 * nseg;  // chunks per segment
  uint32_t* segdoff = d_work + 3 * nseg;
  uint32_t* cursor = d_work + 4 * nseg;
  uint4* desc = reinterpret_cast<uint4*>(d_sorted);  // chunks <= cap / 2: the first cap entries
  uint2* raw = d_sorted + cap;
  PSOUP_HIP_CHECK(hipMemsetAsync(d_work, 0, 5ull * nseg * sizeof(uint32_t), s));
  PSOUP_HIP_CHECK(hipMemsetAsync(d_total, 0, sizeof(uint32_t), s));
  if (nseg <= static_cast<uint32_t>(kSegLds)) {
    const uint64_t per = 256ull * kRecPerThread;
    const unsigned g = static_cast<unsigned>(std::max<uint64_t>(1, (static_cast<uint64_t>(cap) + per - 1) / per));
    seg_hist_kernel<<<g, 256, 0, s>>>(d_peaks, rg, nseg, segcnt, segdcnt);
    post_launch_check("seg_hist_kernel", s);
    seg_scan_kernel<<<1, kClThreads, 0, s>>>(segcnt, nseg, segoff);
    post_launch_check("seg_scan_kernel", s);
    seg_scan_kernel<<<1, kClThreads, 0, s>>>(segdcnt, nseg, segdoff);
    post_launch_check("seg_scan_kernel", s);
    seg_scatter_kernel<<<g, 256, 0, s>>>(d_peaks, rg, nseg, segdoff, cursor, desc);
    post_launch_check("seg_scatter_kernel", s);
  } else {
    const unsigned g = dev::grid_for(cap, 256, 4096);
    seg_hist_global_kernel<<<g, 256, 0, s>>>(d_peaks, rg, cap, nseg, segcnt, segdcnt);
    post_launch_check("seg_hist_global_kernel", s);
    seg_scan_kernel<<<1, kClThreads, 0, s>>>(segcnt, nseg, segoff);
    post_launch_check("seg_scan_kernel", s);
    seg_scan_kernel<<<1, kClThreads, 0, s>>>(segdcnt, nseg, segdoff);
    post_launch_check("seg_scan_kernel", s);
    seg_scatter_global_kernel<<<g, 256, 0, s>>>(d_peaks, rg, cap, nseg, segdoff, cursor, desc);
    post_launch_check("seg_scatter_global_kernel", s);
  }
  peak_cluster_kernel<kClSmall, kClThreads><<<nseg, kClThreads, 0, s>>>(
      d_peaks, desc, segoff, segcnt, segdoff, segdcnt, gap, 0u, d_out, d_segtab, d_total, raw);
  post_launch_check("peak_cluster_kernel<small>", s);
  // the large kernel holds a CU's LDS alone: 1024 threads (16 waves)
  peak_cluster_kernel<kClusterCap, 1024><<<nseg, 1024, 0, s>>>(
      d_peaks, desc, segoff, segcnt, segdoff, segdcnt, gap, kClSmall, d_out, d_segtab, d_total, raw);
  post_launch_check("peak_cluster_kernel<large>", s);
}

}  // namespace kern
}  // namespace psoup
