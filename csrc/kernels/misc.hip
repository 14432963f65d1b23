// Multi-beam coincidence and cross-correlation helpers.
// Reference: src/kernels.cu:1073-1100 (K26 coincidence_kernel over a float**
// table of beams, no bounds check), :1104-1139 (K27 conjugate, K28 complex
// multiply).  The coincidencer is split into a per-beam indicator (so beams
// on different GPUs can be summed by an RCCL all-reduce over xGMI) and a
// final threshold.
#include <algorithm>

#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

__global__ void __launch_bounds__(256) count_above_kernel(const float* __restrict__ x, uint64_t n, float thresh,
                                                          uint8_t* __restrict__ counts) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    counts[i] = static_cast<uint8_t>(counts[i] + (x[i] > thresh ? 1 : 0));
}

__global__ void __launch_bounds__(256) add_counts_kernel(const uint8_t* __restrict__ a, uint64_t n,
                                                         uint8_t* __restrict__ acc) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    acc[i] = static_cast<uint8_t>(acc[i] + a[i]);
}

__global__ void __launch_bounds__(256) coincidence_mask_kernel(const uint8_t* __restrict__ counts, uint64_t n,
                                                               int beam_thresh, float* __restrict__ mask) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    mask[i] = static_cast<float>(static_cast<int>(counts[i]) < beam_thresh);
}

__global__ void __launch_bounds__(256) conjugate_kernel(float2* __restrict__ x, uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    x[i].y *= -1.0f;
}

// One launch copying up to kGatherRows scattered rows (16-byte multiples)
// into consecutive rows of dst: blockIdx.y = row.
__global__ void __launch_bounds__(256) gather_rows_kernel(RowPtrs src, uint64_t nvec, uint4* __restrict__ dst,
                                                          uint64_t dst_stride_vec) {
  const uint4* __restrict__ s = reinterpret_cast<const uint4*>(src.p[blockIdx.y]);
  uint4* __restrict__ d = dst + blockIdx.y * dst_stride_vec;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nvec; i += stride) d[i] = s[i];
}

__global__ void __launch_bounds__(256) cmul_kernel(const float2* __restrict__ x, float2* __restrict__ y, uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float2 a = x[i], b = y[i];
    y[i] = make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
  }
}

}  // namespace

void add_counts(const uint8_t* a, uint64_t n, uint8_t* acc, hipStream_t s) {
  add_counts_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(a, n, acc);
  post_launch_check("add_counts_kernel", s);
}

void count_above(const float* x, uint64_t n, float thresh, uint8_t* counts, hipStream_t s) {
  count_above_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(x, n, thresh, counts);
  post_launch_check("count_above_kernel", s);
}

void coincidence_mask(const uint8_t* counts, uint64_t n, int beam_thresh, float* mask, hipStream_t s) {
  coincidence_mask_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(counts, n, beam_thresh, mask);
  post_launch_check("coincidence_mask_kernel", s);
}

void conjugate(float2* x, uint64_t n, hipStream_t s) {
  conjugate_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(x, n);
  post_launch_check("conjugate_kernel", s);
}

void gather_rows(const uint8_t* const* rows, int nrows, uint64_t nbytes, uint8_t* dst, uint64_t dst_stride,
                 hipStream_t s) {
  PSOUP_CHECK(nbytes % 16 == 0 && dst_stride % 16 == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0,
              "gather_rows: 16-byte rows");
  for (int r0 = 0; r0 < nrows; r0 += kGatherRows) {
    RowPtrs rp{};
    const int n = nrows - r0 < kGatherRows ? nrows - r0 : kGatherRows;
    for (int i = 0; i < n; ++i) {
      PSOUP_CHECK((reinterpret_cast<uintptr_t>(rows[r0 + i]) & 15) == 0, "gather_rows: row alignment");
      rp.p[i] = rows[r0 + i];
    }
    const uint64_t nvec = nbytes / 16;
    const dim3 grid(static_cast<unsigned>(std::min<uint64_t>((nvec + 255) / 256, 256)), static_cast<unsigned>(n));
    gather_rows_kernel<<<grid, 256, 0, s>>>(rp, nvec, reinterpret_cast<uint4*>(dst + r0 * dst_stride), dst_stride / 16);
    post_launch_check("gather_rows_kernel", s);
  }
}

void cmul_inplace(const float2* x, float2* y, uint64_t n, hipStream_t s) {
  cmul_kernel<<<dev::grid_for(n, 256), 256, 0, s>>>(x, y, n);
  post_launch_check("cmul_kernel", s);
}

}  // namespace kern
}  // namespace psoup
