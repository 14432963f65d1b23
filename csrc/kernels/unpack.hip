// Corner turn: packed time-major SIGPROC samples -> channel-major int8 rows.
// (dedisp performs the same unpack + transpose internally; the reference tree
// carries an unused copy of its transpose in include/transforms/transpose.hpp.)
// Tile: 256 samples x 64 channels through LDS, 64-byte coalesced row stores.
#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

constexpr int TS = 256;  // samples per tile
constexpr int TC = 64;   // channels per tile
constexpr int LDS_ROW = TS + 16;

__global__ void __launch_bounds__(256) unpack_transpose_kernel(const uint8_t* __restrict__ packed,
                                                               uint64_t nsamps, int nchans, int nbits,
                                                               int8_t* __restrict__ out, uint64_t out_stride,
                                                               int bias) {
  __shared__ __attribute__((aligned(16))) int8_t tile[TC * LDS_ROW];
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * TS;
  const int c0 = blockIdx.y * TC;
  const uint64_t bps = static_cast<uint64_t>(nchans) * nbits / 8;
  const int mask = (1 << nbits) - 1;
  const int per_byte = 8 / nbits;
  // ---- read: thread t unpacks sample t0+t for channels [c0, c0+TC)
  {
    const uint64_t t = t0 + threadIdx.x;
    const int nc = min(TC, nchans - c0);
    if (t < nsamps) {
      const uint8_t* src = packed + t * bps + (static_cast<uint64_t>(c0) * nbits) / 8;
      const int nbytes = (nc * nbits + 7) / 8;
      for (int b = 0; b < nbytes; ++b) {
        const int byte = src[b];
#pragma unroll 8
        for (int q = 0; q < per_byte; ++q) {
          const int c = b * per_byte + q;
          if (c < nc) tile[c * LDS_ROW + threadIdx.x] = static_cast<int8_t>(((byte >> (q * nbits)) & mask) - bias);
        }
      }
    }
  }
  __syncthreads();
  // ---- write: 4 threads per channel row, 64 bytes each
  const int row = threadIdx.x >> 2;
  const int seg = threadIdx.x & 3;
  const int c = c0 + row;
  if (c < nchans) {
    const uint64_t tbeg = t0 + seg * 64;
    int8_t* dst = out + static_cast<uint64_t>(c) * out_stride + tbeg;
    const int8_t* srcl = tile + row * LDS_ROW + seg * 64;
    if (tbeg + 64 <= nsamps && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        reinterpret_cast<int4*>(dst)[q] = reinterpret_cast<const int4*>(srcl)[q];
    } else {
      for (int q = 0; q < 64; ++q)
        if (tbeg + q < nsamps) dst[q] = srcl[q];
    }
  }
}

}  // namespace

void unpack_transpose(const uint8_t* packed, uint64_t nsamps, int nchans, int nbits, int8_t* out,
                      uint64_t out_stride, int bias, hipStream_t s) {
  PSOUP_CHECK(nbits == 1 || nbits == 2 || nbits == 4 || nbits == 8, "nbits must be 1/2/4/8");
  PSOUP_CHECK((static_cast<uint64_t>(nchans) * nbits) % 8 == 0, "nchans*nbits must be a multiple of 8");
  PSOUP_CHECK(out_stride >= nsamps, "out_stride too small");
  if (nsamps == 0) return;
  uint64_t gx = (nsamps + TS - 1) / TS;
  PSOUP_CHECK(gx < (1ull << 31), "too many samples");
  dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>((nchans + TC - 1) / TC));
  unpack_transpose_kernel<<<grid, 256, 0, s>>>(packed, nsamps, nchans, nbits, out, out_stride, bias);
  post_launch_check("unpack_transpose_kernel", s);
}

}  // namespace kern
}  // namespace psoup
