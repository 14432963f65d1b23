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
// peak_cluster_kernel: one workgroup per segment (trial x level): bitonic
// sort by idx in LDS, the window test (1) in parallel, runs marked with a
// max-scan, one thread walks each run (2), a scan compacts the peaks in idx
// order.  Segments over kClusterCap crossings are left to the host (flagged
// in the segment table with their raw, unsorted range).
#include "device_common.hpp"

namespace psoup {
namespace kern {
namespace {

constexpr int kClThreads = 512;

// Hillis-Steele scans over one value per thread (kClThreads); returns the
// exclusive sum / the inclusive max of the preceding threads' values.
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t* sc, uint32_t* total) {
  const int t = threadIdx.x;
  sc[t] = v;
  __syncthreads();
  for (int off = 1; off < kClThreads; off <<= 1) {
    const uint32_t a = t >= off ? sc[t - off] : 0u;
    __syncthreads();
    sc[t] += a;
    __syncthreads();
  }
  const uint32_t incl = sc[t];
  if (total) *total = sc[kClThreads - 1];
  __syncthreads();
  return incl - v;
}

__device__ __forceinline__ int block_excl_max(int v, int* sc) {
  const int t = threadIdx.x;
  sc[t] = v;
  __syncthreads();
  for (int off = 1; off < kClThreads; off <<= 1) {
    const int a = t >= off ? sc[t - off] : -1;
    __syncthreads();
    sc[t] = max(sc[t], a);
    __syncthreads();
  }
  const int prev = t > 0 ? sc[t - 1] : -1;
  __syncthreads();
  return prev;
}

__global__ void __launch_bounds__(256) seg_hist_kernel(const PeakRecord* __restrict__ in,
                                                       const uint32_t* __restrict__ count, uint32_t cap,
                                                       uint32_t nseg, uint32_t* __restrict__ segcnt) {
  const uint32_t n = min(*count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = in[i].seg;
    if (s < nseg) atomicAdd(&segcnt[s], 1u);
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

__global__ void __launch_bounds__(256) seg_scatter_kernel(const PeakRecord* __restrict__ in,
                                                          const uint32_t* __restrict__ count, uint32_t cap,
                                                          uint32_t nseg, const uint32_t* __restrict__ segoff,
                                                          uint32_t* __restrict__ cursor, uint2* __restrict__ out) {
  const uint32_t n = min(*count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const PeakRecord r = in[i];
    if (r.seg >= nseg) continue;
    const uint32_t pos = segoff[r.seg] + atomicAdd(&cursor[r.seg], 1u);
    out[pos] = make_uint2(static_cast<uint32_t>(r.idx), __float_as_uint(r.snr));
  }
}

__global__ void __launch_bounds__(kClThreads) peak_cluster_kernel(const uint2* __restrict__ sorted,
                                                                  const uint32_t* __restrict__ segoff,
                                                                  const uint32_t* __restrict__ segcnt, int gap,
                                                                  uint2* __restrict__ out, uint2* __restrict__ segtab,
                                                                  uint32_t* __restrict__ total) {
  __shared__ uint2 key[kClusterCap];    // (idx, snr bits)
  __shared__ uint8_t flag[kClusterCap];  // bit 0: survives the window test, bit 1: cluster peak
  __shared__ uint32_t sc[kClThreads];
  __shared__ uint32_t base_s;
  const int t = threadIdx.x;
  const uint32_t seg = blockIdx.x;
  const uint32_t n = segcnt[seg], off = segoff[seg];
  if (n == 0 || n > kClusterCap) {
    if (t == 0) segtab[seg] = n == 0 ? make_uint2(0u, 0u) : make_uint2(off, n | kClusterRaw);
    return;
  }
  uint32_t P = 64;
  while (P < n) P <<= 1;
  for (uint32_t i = t; i < P; i += kClThreads)
    key[i] = i < n ? sorted[off + i] : make_uint2(0x7fffffffu, 0u);  // pads sort last
  __syncthreads();
  // bitonic sort, ascending idx (distinct within a segment; idx >= 0)
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = t; i < P / 2; i += kClThreads) {
        const uint32_t lo = 2 * j * (i / j) + (i & (j - 1)), hi = lo + j;
        const uint2 a = key[lo], b = key[hi];
        if ((static_cast<int>(a.x) > static_cast<int>(b.x)) == ((lo & k) == 0)) {
          key[lo] = b;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  // (1) window test over a contiguous chunk per thread
  const uint32_t C = (P + kClThreads - 1) / kClThreads;
  const uint32_t b0 = min(static_cast<uint32_t>(t) * C, n), b1 = min(b0 + C, n);
  int last = -1;  // this chunk's last survivor
  for (uint32_t i = b0; i < b1; ++i) {
    const int xi = static_cast<int>(key[i].x);
    const float si = __uint_as_float(key[i].y);
    bool keep = true;
    for (uint32_t j = i + 1; j < n && static_cast<int>(key[j].x) - xi < gap; ++j)
      if (__uint_as_float(key[j].y) > si) {
        keep = false;
        break;
      }
    flag[i] = keep ? 1 : 0;
    if (keep) last = static_cast<int>(i);
  }
  // the survivor before this chunk (max-scan of chunk-last positions)
  int prev = block_excl_max(last, reinterpret_cast<int*>(sc));
  // (2) one thread per run: from each run start, greedy gap windows
  for (uint32_t i = b0; i < b1; ++i) {
    if (!(flag[i] & 1)) continue;
    const int xi = static_cast<int>(key[i].x);
    const bool start = prev < 0 || xi - static_cast<int>(key[prev].x) >= gap;
    prev = static_cast<int>(i);
    if (!start) continue;
    int anchor = xi, lastx = xi;
    flag[i] = 3;
    for (uint32_t j = i + 1; j < n; ++j) {
      if (!(flag[j] & 1)) continue;
      const int xj = static_cast<int>(key[j].x);
      if (xj - lastx >= gap) break;  // the next run (its own walker)
      lastx = xj;
      if (xj - anchor >= gap) {
        anchor = xj;
        flag[j] = 3;
      }
    }
  }
  __syncthreads();
  // compaction of the peaks, idx order
  uint32_t cnt = 0;
  for (uint32_t i = b0; i < b1; ++i) cnt += flag[i] >> 1;
  uint32_t npk;
  const uint32_t ex = block_excl_sum(cnt, sc, &npk);
  if (t == 0) {
    base_s = atomicAdd(total, npk);
    segtab[seg] = make_uint2(base_s, npk);
  }
  __syncthreads();
  uint32_t o = base_s + ex;
  for (uint32_t i = b0; i < b1; ++i)
    if (flag[i] >> 1) out[o++] = key[i];
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
  const unsigned g = dev::grid_for(cap, 256, 4096);
  seg_hist_kernel<<<g, 256, 0, s>>>(d_peaks, d_count, cap, nseg, segcnt);
  post_launch_check("seg_hist_kernel", s);
  seg_scan_kernel<<<1, kClThreads, 0, s>>>(segcnt, nseg, segoff);
  post_launch_check("seg_scan_kernel", s);
  seg_scatter_kernel<<<g, 256, 0, s>>>(d_peaks, d_count, cap, nseg, segoff, cursor, d_sorted);
  post_launch_check("seg_scatter_kernel", s);
  peak_cluster_kernel<<<nseg, kClThreads, 0, s>>>(d_sorted, segoff, segcnt, gap, d_out, d_segtab, d_total);
  post_launch_check("peak_cluster_kernel", s);
}

}  // namespace kern
}  // namespace psoup
