// Brute-force incoherent dedispersion (replaces the external dedisp library
// called from include/transforms/dedisperser.hpp:98-113).
//
// Input: channel-major int8 rows x[c][t] = raw - bias (unpack_transpose).
// Output: DM-major uint8 trials, out[d][t] = (uint8) clamp(scale * S, 0, 255),
//   S = sum over unkilled channels of raw[c][t + off(c,d)], off = (int)(dm*delay[c] + 0.5)
// scale = 192 / (in_range * nchans) (= 255/(in_range*nchans) * 3*1024/255/16,
// dedisp's 8-bit output scaling; exactly 1.0 for 2-bit x 64 channels).
//
// Two kernels produce bit-identical output:
//   dedisperse_direct_kernel  VALU reference: one thread = 4 samples of 1 DM.
//   dedisperse_mfma_kernel    v_mfma_i32_32x32x32_i8: the DM sum is a GEMM of
//     shifted data (A: 32 samples x 32 (channel,shift) pairs) with a one-hot
//     selection matrix (B: 32 (channel,shift) pairs x 32 DMs); see below.
#include <algorithm>
#include <cstdlib>
#include <utility>
#include <vector>

#include "device_common.hpp"
#include "psoup/kernels.hpp"

namespace psoup {
namespace kern {

namespace {

__device__ __forceinline__ uint8_t scale_out(int sum, float scale) {
  float v = static_cast<float>(sum) * scale;
  v = fminf(fmaxf(v, 0.f), 255.f);
  return static_cast<uint8_t>(v);
}

__global__ void __launch_bounds__(256) dedisperse_direct_kernel(const int8_t* __restrict__ x, uint64_t stride,
                                                                int nchans, const int32_t* __restrict__ offsets,
                                                                const int32_t* __restrict__ kill,
                                                                uint64_t out_nsamps, uint8_t* __restrict__ out,
                                                                uint64_t out_stride, float scale, int bias_total) {
  const int d = blockIdx.y;
  const uint64_t t = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
  if (t >= out_nsamps) return;
  const int32_t* off = offsets + static_cast<uint64_t>(d) * nchans;
  int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  const bool full = t + 4 <= out_nsamps;
  for (int c = 0; c < nchans; ++c) {
    if (!kill[c]) continue;
    const int8_t* p = x + static_cast<uint64_t>(c) * stride + t + off[c];
    if (full) {
      s0 += p[0];
      s1 += p[1];
      s2 += p[2];
      s3 += p[3];
    } else {
      s0 += p[0];
      if (t + 1 < out_nsamps) s1 += p[1];
      if (t + 2 < out_nsamps) s2 += p[2];
      if (t + 3 < out_nsamps) s3 += p[3];
    }
  }
  uint8_t* o = out + static_cast<uint64_t>(d) * out_stride + t;
  o[0] = scale_out(s0 + bias_total, scale);
  if (t + 1 < out_nsamps) o[1] = scale_out(s1 + bias_total, scale);
  if (t + 2 < out_nsamps) o[2] = scale_out(s2 + bias_total, scale);
  if (t + 3 < out_nsamps) o[3] = scale_out(s3 + bias_total, scale);
}


// ------------------------------------------------------------------ MFMA ----
// out[t][d] = sum_k A[t][k] * B[k][d] with k = (channel c, shift j in a block of
// 16 consecutive shifts starting at sb):
//   A[t][(c,j)] = x[c][t + sb + j]               (16 consecutive bytes per lane)
//   B[(c,j)][d] = (off(c,d) - sb == j)           (one-hot, built from a delta byte)
// One v_mfma_i32_32x32x32_i8 covers two (c, sb) blocks (lane half h = block h)
// for 32 samples x 32 DMs; a wave owns 4 such sample tiles (128 samples) so
// each one-hot B fragment is reused 4x.  Workgroup = 4 waves = 512 samples of
// one 32-DM tile.  Exact int32 accumulation => identical to the VALU kernel.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

constexpr int kMfmaWaveTiles = 4;                       // 32-sample tiles per wave
constexpr int kMfmaWgSamples = 4 * 32 * kMfmaWaveTiles;  // 512

__global__ void __launch_bounds__(256) dedisperse_mfma_kernel(
    const int8_t* __restrict__ x, uint64_t stride, const int4* __restrict__ steps, const int8_t* __restrict__ deltas,
    const int2* __restrict__ tile_info, int ndm, int d_skip, uint64_t out_nsamps, uint8_t* __restrict__ out,
    uint64_t out_stride, float scale, int bias_total, uint64_t ntime_tiles) {
  const int tile = blockIdx.x;  // DM tile (fastest: concurrent WGs share the x window in L2)
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int2 ti = tile_info[tile];  // {first step, step count}: ragged per-tile step lists
  const int ns = ti.y;
  const int4* st = steps + ti.x;
  const int8_t* dl = deltas + static_cast<uint64_t>(ti.x) * 64;
  for (uint64_t tt = blockIdx.y; tt < ntime_tiles; tt += gridDim.y) {
    const uint64_t t0 = tt * kMfmaWgSamples + static_cast<uint64_t>(wave) * (32 * kMfmaWaveTiles);
    v16i acc[kMfmaWaveTiles];
#pragma unroll
    for (int m = 0; m < kMfmaWaveTiles; ++m)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][e] = 0;
    for (int s = 0; s < ns; ++s) {
      const int4 stp = st[s];
      const int c = h ? stp.z : stp.x;
      const int sb = h ? stp.w : stp.y;
      const int delta = dl[s * 64 + lane];
      v4i b;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        b[q] = (delta >= 0 && (delta >> 2) == q) ? (1 << ((delta & 3) * 8)) : 0;
      const int8_t* row = x + static_cast<uint64_t>(c) * stride;
#pragma unroll
      for (int m = 0; m < kMfmaWaveTiles; ++m) {
        const uint64_t a0 = t0 + m * 32 + r + static_cast<int64_t>(sb);
        const uint64_t al = a0 & ~3ull;
        const int sh = static_cast<int>(a0 & 3ull);
        const uint32_t* p = reinterpret_cast<const uint32_t*>(row + al);
        const u32x4_a4 w = *reinterpret_cast<const u32x4_a4*>(p);
        const uint32_t w4 = p[4];
        v4i a;
        a[0] = static_cast<int>(__builtin_amdgcn_alignbyte(w[1], w[0], sh));
        a[1] = static_cast<int>(__builtin_amdgcn_alignbyte(w[2], w[1], sh));
        a[2] = static_cast<int>(__builtin_amdgcn_alignbyte(w[3], w[2], sh));
        a[3] = static_cast<int>(__builtin_amdgcn_alignbyte(w4, w[3], sh));
        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[m], 0, 0, 0);
      }
    }
    // C/D layout (32x32): col = lane&31 (DM), row = (reg&3) + 8*(reg>>2) + 4*(lane>>5) (sample)
    // DMs before the range's first (its first tile's leading d_skip) are not stored
    const int d = tile * 32 + r - d_skip;
    if (d >= 0 && d < ndm) {
      uint8_t* o = out + static_cast<uint64_t>(d) * out_stride;
#pragma unroll
      for (int m = 0; m < kMfmaWaveTiles; ++m) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint64_t t = t0 + m * 32 + 8 * g + 4 * h;
          uint32_t packed = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            packed |= static_cast<uint32_t>(scale_out(acc[m][4 * g + e] + bias_total, scale)) << (8 * e);
          if (t + 4 <= out_nsamps) {
            *reinterpret_cast<uint32_t*>(o + t) = packed;
          } else {
            for (int e = 0; e < 4; ++e)
              if (t + e < out_nsamps) o[t + e] = static_cast<uint8_t>(packed >> (8 * e));
          }
        }
      }
    }
  }
}


// ------------------------------------------------------------------ VALU ----
// Packed-byte kernel for wide DM tiles (offset spread across the tile >> 16
// samples, where the one-hot MFMA GEMM is mostly zeros).  Workgroup = 4 waves
// = 4*DPT DMs x 1024 samples; lane = 16 consecutive samples, wave = DPT DMs.
// Channel-outer / DM-inner: one channel's window (1024 + spread bytes) is
// re-read by the workgroup's DMs straight from L1.  Per channel and DM a lane
// loads 20 bytes (dwordx4 + dword at the dword-aligned offset) and v_perm
// picks the even / odd bytes at the wave-uniform misalignment into two 16-bit
// lanes, so one 32-bit add accumulates two samples.  Sums are of raw
// (unbiased) bytes: x ^ 0x80 restores raw for bias-128 8-bit data.  16-bit
// lanes hold max_raw * nactive <= 65535 (WIDE = false, nbits <= 4 at <= 4369
// channels); otherwise they are flushed to 32-bit sums every 256 channels.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int DPT, bool WIDE, bool XOR>
__global__ void __launch_bounds__(256) dedisperse_valu_kernel(
    const int8_t* __restrict__ x, uint64_t stride, const int32_t* __restrict__ active, int nactive,
    const int32_t* __restrict__ offT, int ldo, int d_base, int ndm, uint64_t out_nsamps, uint8_t* __restrict__ out,
    uint64_t out_stride, float scale) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int dm0 = blockIdx.x * (4 * DPT) + wave * DPT;  // relative to d_base
  const uint64_t tb = static_cast<uint64_t>(blockIdx.y) * 1024;  // workgroup's first sample
  const uint32_t lo = static_cast<uint32_t>(lane) * 16;          // lane's byte offset from tb
  const uint64_t t = tb + lo;
  uint32_t pk[DPT][8];
  int wide[WIDE ? DPT : 1][WIDE ? 16 : 1];
#pragma unroll
  for (int j = 0; j < DPT; ++j)
#pragma unroll
    for (int q = 0; q < 8; ++q) pk[j][q] = 0;
  if constexpr (WIDE) {
#pragma unroll
    for (int j = 0; j < DPT; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) wide[j][q] = 0;
  }
  auto flush = [&]() {
    if constexpr (WIDE) {
#pragma unroll
      for (int j = 0; j < DPT; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          wide[j][4 * i + 0] += pk[j][2 * i] & 0xFFFF;
          wide[j][4 * i + 2] += pk[j][2 * i] >> 16;
          wide[j][4 * i + 1] += pk[j][2 * i + 1] & 0xFFFF;
          wide[j][4 * i + 3] += pk[j][2 * i + 1] >> 16;
          pk[j][2 * i] = 0;
          pk[j][2 * i + 1] = 0;
        }
    }
  };
  // Two register sets of 20-byte windows (A: even channels, B: odd): the next
  // channel's DPT loads are in flight while this one's are accumulated.
  u32x4 wa[DPT], wb[DPT];
  uint32_t wa4[DPT], wb4[DPT];
  uint32_t sha[DPT], shb[DPT];
  auto load = [&](int ci, u32x4* w, uint32_t* w4, uint32_t* sh) {
    // uniform row base (SGPRs) + 32-bit lane offset
    const int8_t* row = x + static_cast<uint64_t>(active[ci]) * stride + tb;
    const int32_t* o = offT + static_cast<uint64_t>(ci) * ldo + d_base + dm0;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const int off = o[j];
      const int8_t* rb = row + (off & ~3);
      w[j] = *reinterpret_cast<const u32x4_a4*>(rb + lo);
      w4[j] = *reinterpret_cast<const uint32_t*>(rb + lo + 16);
      sh[j] = static_cast<uint32_t>(off & 3);
    }
  };
  auto accumulate = [&](u32x4* w, uint32_t* w4, const uint32_t* sh) {
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      if constexpr (XOR) {
        w[j] ^= 0x80808080u;
        w4[j] ^= 0x80808080u;
      }
      const uint32_t selE = 0x0C000C00u | sh[j] | ((sh[j] + 2) << 16);  // bytes sh, sh+2 -> 16-bit lanes
      const uint32_t selO = selE + 0x00010001u;                        // bytes sh+1, sh+3
      pk[j][0] += __builtin_amdgcn_perm(w[j][1], w[j][0], selE);
      pk[j][1] += __builtin_amdgcn_perm(w[j][1], w[j][0], selO);
      pk[j][2] += __builtin_amdgcn_perm(w[j][2], w[j][1], selE);
      pk[j][3] += __builtin_amdgcn_perm(w[j][2], w[j][1], selO);
      pk[j][4] += __builtin_amdgcn_perm(w[j][3], w[j][2], selE);
      pk[j][5] += __builtin_amdgcn_perm(w[j][3], w[j][2], selO);
      pk[j][6] += __builtin_amdgcn_perm(w4[j], w[j][3], selE);
      pk[j][7] += __builtin_amdgcn_perm(w4[j], w[j][3], selO);
    }
  };
  load(0, wa, wa4, sha);
  int ci = 0;
  for (; ci + 1 < nactive; ci += 2) {
    load(ci + 1, wb, wb4, shb);
    accumulate(wa, wa4, sha);
    if (WIDE && (ci & 255) == 255) flush();
    load(min(ci + 2, nactive - 1), wa, wa4, sha);  // branch-free (a spare reload at the end)
    accumulate(wb, wb4, shb);
    if (WIDE && ((ci + 1) & 255) == 255) flush();
  }
  if (ci < nactive) accumulate(wa, wa4, sha);  // odd count: A holds the last channel
  flush();
  if (t >= out_nsamps) return;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int d = dm0 + j;
    if (d >= ndm) break;
    uint32_t ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int s4[4];
      if constexpr (WIDE) {
        s4[0] = wide[j][4 * i];
        s4[1] = wide[j][4 * i + 1];
        s4[2] = wide[j][4 * i + 2];
        s4[3] = wide[j][4 * i + 3];
      } else {
        s4[0] = static_cast<int>(pk[j][2 * i] & 0xFFFF);
        s4[1] = static_cast<int>(pk[j][2 * i + 1] & 0xFFFF);
        s4[2] = static_cast<int>(pk[j][2 * i] >> 16);
        s4[3] = static_cast<int>(pk[j][2 * i + 1] >> 16);
      }
      ob[i] = static_cast<uint32_t>(scale_out(s4[0], scale)) | (static_cast<uint32_t>(scale_out(s4[1], scale)) << 8) |
              (static_cast<uint32_t>(scale_out(s4[2], scale)) << 16) |
              (static_cast<uint32_t>(scale_out(s4[3], scale)) << 24);
    }
    uint8_t* orow = out + static_cast<uint64_t>(d) * out_stride + t;
    if (t + 16 <= out_nsamps) {
      *reinterpret_cast<u32x4*>(orow) = u32x4{ob[0], ob[1], ob[2], ob[3]};
    } else {
      for (uint64_t e = 0; t + e < out_nsamps; ++e) orow[e] = static_cast<uint8_t>(ob[e >> 2] >> (8 * (e & 3)));
    }
  }
}


// LDS-staged variant of the packed-byte kernel (narrow sample: nbits <= 4).
// Per channel the workgroup (32 DMs x 1024 samples) stages the channel's
// window -- from the tile's smallest offset, 16-byte aligned, 1024 + spread
// + 32 bytes -- once, with aligned dwordx4 loads one channel ahead (double
// buffer, one barrier per channel); each lane then reads its 32 bytes per DM
// as two conflict-free ds_read_b128 and picks 5 words at the wave-uniform
// word offset (uniform branch) before the same v_perm/add accumulation.
// wmin[tile][ci]: the window start (relative to the sample) of tile and channel.
constexpr int kLdsWinWords = 2048;  // largest staged window: 8 KiB (two 4 KiB passes)

template <int Q>
__device__ __forceinline__ void lds_accumulate(const uint32_t* w, uint32_t sh, uint32_t (&pk)[8]) {
  const uint32_t selE = 0x0C000C00u | sh | ((sh + 2) << 16);
  const uint32_t selO = selE + 0x00010001u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pk[2 * i] += __builtin_amdgcn_perm(w[Q + i + 1], w[Q + i], selE);
    pk[2 * i + 1] += __builtin_amdgcn_perm(w[Q + i + 1], w[Q + i], selO);
  }
}

// Byte-lane accumulation (BYTES): a lane's 16 samples of one DM are the four
// dwords at the wave-uniform byte shift (v_alignbyte) added as packed bytes --
// four adds per channel instead of eight v_perm + eight adds -- and spilled to
// the 16-bit sums every `flush` channels (flush * max raw value <= 255, so no
// byte carries).
template <int Q>
__device__ __forceinline__ void lds_accumulate_bytes(const uint32_t* w, uint32_t sh, uint32_t (&acc)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] += __builtin_amdgcn_alignbyte(w[Q + i + 1], w[Q + i], sh);
}

template <bool XOR, int PASSES, int DPT, int CPB, bool BYTES = false>
__global__ void __launch_bounds__(256) dedisperse_lds_kernel(
    const int8_t* __restrict__ x, uint64_t stride, const int32_t* __restrict__ active, int nactive,
    const int32_t* __restrict__ offT, int ldo, int d_base, int d_skip, int ndm, const int32_t* __restrict__ wmin,
    uint64_t out_nsamps, uint8_t* __restrict__ out, uint64_t out_stride, float scale, int flush) {
  // CPB channels' windows per LDS buffer (one barrier per CPB channels),
  // double-buffered; each window is PASSES x 4 KiB
  __shared__ __attribute__((aligned(16))) uint32_t win[2][CPB * PASSES * 1024];
  // workgroup = 4*DPT DMs (DPT = 8: one 32-DM tile; 4: half a tile, more
  // workgroups per CU to hide the channel-window loads)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // d_base is a multiple of the workgroup's 4*DPT DMs, so every workgroup
  // lies in one absolute 32-DM tile of the window table; its first d_skip
  // DMs (before the range) are computed but not stored
  const int dm0 = blockIdx.x * (4 * DPT) + wave * DPT;  // relative to d_base
  const int tile = (d_base + static_cast<int>(blockIdx.x) * 4 * DPT) / 32;
  const uint64_t tb = static_cast<uint64_t>(blockIdx.y) * 1024;
  const uint64_t t = tb + static_cast<uint64_t>(lane) * 16;
  const int32_t* wm = wmin + static_cast<uint64_t>(tile) * nactive;
  uint32_t pk[DPT][8];
#pragma unroll
  for (int j = 0; j < DPT; ++j)
#pragma unroll
    for (int q = 0; q < 8; ++q) pk[j][q] = 0;
  uint32_t acc[DPT][4];  // BYTES: packed byte sums since the last spill
#pragma unroll
  for (int j = 0; j < DPT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = 0;
  auto spill = [&]() {
#pragma unroll
    for (int j = 0; j < DPT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pk[j][2 * i] += acc[j][i] & 0x00FF00FFu;            // samples 4i, 4i+2
        pk[j][2 * i + 1] += (acc[j][i] >> 8) & 0x00FF00FFu;  // samples 4i+1, 4i+3
        acc[j][i] = 0;
      }
  };
  u32x4 r[CPB][PASSES];
  // every thread stages 16 bytes per pass and channel (predicating the loads
  // to the launch's largest window measured slower: 2.57 vs 2.2 ms per chunk)
  auto gload = [&](int c0) {
#pragma unroll
    for (int q = 0; q < CPB; ++q) {
      const int ci = min(c0 + q, nactive - 1);  // past the end: a harmless reload
      const int8_t* row = x + static_cast<uint64_t>(active[ci]) * stride + tb + wm[ci];
#pragma unroll
      for (int p = 0; p < PASSES; ++p)
        r[q][p] = *reinterpret_cast<const u32x4*>(row + 4096 * p + 16 * threadIdx.x);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < CPB; ++q)
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        if constexpr (XOR) r[q][p] ^= 0x80808080u;
        *reinterpret_cast<u32x4*>(&win[buf][(q * PASSES + p) * 1024 + 4 * threadIdx.x]) = r[q][p];
      }
  };
  auto compute = [&](int ci, const uint32_t* wbase) {
    const int w0 = wm[ci];
    const int32_t* o = offT + static_cast<uint64_t>(ci) * ldo + d_base + dm0;
    // all DPT windows' LDS reads first (latency overlapped), then the sums:
    // two 16-byte-aligned ds_read_b128 per DM, words picked at the
    // wave-uniform offset (a dword-aligned b128 + b32 form measured slower)
    int rel[DPT];
    uint32_t w[DPT][8];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      rel[j] = o[j] - w0;  // >= 0, wave-uniform
      const uint32_t* src = wbase + 4 * lane + ((rel[j] >> 4) << 2);
      const u32x4 a = *reinterpret_cast<const u32x4*>(src);
      const u32x4 b = *reinterpret_cast<const u32x4*>(src + 4);
      w[j][0] = a[0]; w[j][1] = a[1]; w[j][2] = a[2]; w[j][3] = a[3];
      w[j][4] = b[0]; w[j][5] = b[1]; w[j][6] = b[2]; w[j][7] = b[3];
    }
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const uint32_t sh = static_cast<uint32_t>(rel[j] & 3);
      if constexpr (BYTES) {
        switch ((rel[j] >> 2) & 3) {  // uniform
          case 0: lds_accumulate_bytes<0>(w[j], sh, acc[j]); break;
          case 1: lds_accumulate_bytes<1>(w[j], sh, acc[j]); break;
          case 2: lds_accumulate_bytes<2>(w[j], sh, acc[j]); break;
          default: lds_accumulate_bytes<3>(w[j], sh, acc[j]); break;
        }
      } else {
        switch ((rel[j] >> 2) & 3) {  // uniform
          case 0: lds_accumulate<0>(w[j], sh, pk[j]); break;
          case 1: lds_accumulate<1>(w[j], sh, pk[j]); break;
          case 2: lds_accumulate<2>(w[j], sh, pk[j]); break;
          default: lds_accumulate<3>(w[j], sh, pk[j]); break;
        }
      }
    }
    if constexpr (BYTES) {
      if ((ci + 1) % flush == 0) spill();  // wave-uniform
    }
  };
  gload(0);
  lstore(0);
  __syncthreads();
  for (int c0 = 0, it = 0; c0 < nactive; c0 += CPB, ++it) {
    const int buf = it & 1;
    if (c0 + CPB < nactive) gload(c0 + CPB);  // in flight during these channels' sums
#pragma unroll 1
    for (int q = 0; q < CPB; ++q)
      if (c0 + q < nactive) compute(c0 + q, &win[buf][q * PASSES * 1024]);
    if (c0 + CPB < nactive) lstore(buf ^ 1);
    __syncthreads();
  }
  if constexpr (BYTES) spill();
  if (t >= out_nsamps) return;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    if (dm0 + j >= ndm) break;  // ndm counts from d_base
    const int d = dm0 + j - d_skip;
    if (d < 0) continue;
    uint32_t ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s0 = static_cast<int>(pk[j][2 * i] & 0xFFFF), s2 = static_cast<int>(pk[j][2 * i] >> 16);
      const int s1 = static_cast<int>(pk[j][2 * i + 1] & 0xFFFF), s3 = static_cast<int>(pk[j][2 * i + 1] >> 16);
      ob[i] = static_cast<uint32_t>(scale_out(s0, scale)) | (static_cast<uint32_t>(scale_out(s1, scale)) << 8) |
              (static_cast<uint32_t>(scale_out(s2, scale)) << 16) | (static_cast<uint32_t>(scale_out(s3, scale)) << 24);
    }
    uint8_t* orow = out + static_cast<uint64_t>(d) * out_stride + t;
    if (t + 16 <= out_nsamps) {
      *reinterpret_cast<u32x4*>(orow) = u32x4{ob[0], ob[1], ob[2], ob[3]};
    } else {
      for (uint64_t e = 0; t + e < out_nsamps; ++e) orow[e] = static_cast<uint8_t>(ob[e >> 2] >> (8 * (e & 3)));
    }
  }
}

// ------------------------------------------------------- MFMA, LDS-fed ----
// The one-hot GEMM of dedisperse_mfma_kernel with its A operand built from
// LDS instead of global memory: per 16-channel group the workgroup (one
// 32-DM tile x 1024 samples) stages each channel's window
// [t0 + w0, t0 + w0 + 1280) -- w0 = the tile's smallest offset of the
// channel, rounded down to 16 bytes -- with aligned dwordx4 loads one group
// ahead (double buffer, one barrier per group); a lane's 16 shifted bytes
// come from five dword LDS reads and v_alignbyte.  Only tiles whose offset
// spread fits the window take this path (low DM, few 16-shift blocks per
// channel: there the one-hot MFMA beats the packed-byte VALU kernel).  Plan:
// build_mfma_lds_plan (packed step words + window-relative DM offsets per
// channel group, staged in LDS with the windows: the step loop is LDS + MFMA
// only -- a per-step global one-hot load measured 3.7x the MFMA time).
constexpr int kMlWin = 1280;  // staged bytes per channel: 1024 samples + spread + the 20-byte read
constexpr int kMlTs = 1024;   // samples per workgroup (4 waves x 8 tiles of 32)

template <int CG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) dedisperse_mfma_lds_kernel(
    const int8_t* __restrict__ x, uint64_t stride, const int32_t* __restrict__ active, int nactive,
    const uint32_t* __restrict__ steps, const uint8_t* __restrict__ relo, const int2* __restrict__ ginfo,
    int ngroups, const int32_t* __restrict__ wmin, int ndm, int d_skip, uint64_t out_nsamps,
    uint8_t* __restrict__ out, uint64_t out_stride, float scale, int bias_total) {
  // per buffer: CG windows, then kMfmaLdsMaxSteps step words, then the
  // CG x 32 relo bytes (all 16-byte units)
  constexpr int kWinU = CG * kMlWin / 16;            // window units
  constexpr int kStepU = kMfmaLdsMaxSteps * 4 / 16;  // step-word units
  constexpr int kReloU = CG * 32 / 16;               // relo units
  constexpr int kBufW = (kWinU + kStepU + kReloU) * 4;
  __shared__ __attribute__((aligned(16))) uint32_t win[2][kBufW];
  const int tile = blockIdx.x;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.y) * kMlTs;
  const int2* gi = ginfo + static_cast<uint64_t>(tile) * ngroups;
  const int32_t* wm = wmin + static_cast<uint64_t>(tile) * nactive;
  const uint8_t* rl = relo + static_cast<uint64_t>(tile) * ngroups * CG * 32;
  constexpr int kV = kWinU / 256;  // 16-byte window loads per thread per group
  static_assert(kV * 256 == kWinU && kStepU + kReloU <= 256, "staging shape");
  u32x4 rg[kV + 1];
  const bool extra = threadIdx.x < kStepU + kReloU;
  auto gload = [&](int g) {
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      const int e = v * 256 + static_cast<int>(threadIdx.x);  // 16-byte unit in the group's windows
      const int q = e / (kMlWin / 16), u = e - q * (kMlWin / 16);
      const int ci = min(g * CG + q, nactive - 1);  // past the last channel: a harmless reload
      rg[v] = *reinterpret_cast<const u32x4*>(x + static_cast<uint64_t>(active[ci]) * stride + t0 + wm[ci] + 16 * u);
    }
    if (extra) {
      const int e = static_cast<int>(threadIdx.x);
      rg[kV] = e < kStepU ? *reinterpret_cast<const u32x4*>(steps + gi[g].x + 4 * e)  // padded past the end
                          : *reinterpret_cast<const u32x4*>(rl + static_cast<uint64_t>(g) * CG * 32 + 16 * (e - kStepU));
    }
  };
  auto lstore = [&](int b) {
#pragma unroll
    for (int v = 0; v < kV; ++v) *reinterpret_cast<u32x4*>(&win[b][4 * (v * 256 + threadIdx.x)]) = rg[v];
    if (extra) *reinterpret_cast<u32x4*>(&win[b][4 * (kWinU + threadIdx.x)]) = rg[kV];
  };
  // MFMA row r of sub-tile m is sample w*256 + 8r + m: the eight sub-tiles of
  // a lane read the 23 consecutive window bytes from 8r, so one 7-dword LDS
  // read per lane and step feeds all eight MFMAs (rel is a multiple of 4, so
  // each sub-tile's byte shift m & 3 is a compile-time constant)
  v16i acc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[m][e] = 0;
  const int sbase = wave * 256 + 8 * r;  // this lane's first sample in the window, before the block shift
  gload(0);
  lstore(0);
  __syncthreads();
  for (int g = 0; g < ngroups; ++g) {
    const int b = g & 1;
    if (g + 1 < ngroups) gload(g + 1);
    const int nst = gi[g].y;
    const uint32_t* wb = win[b];
    const uint32_t* sw = wb + kWinU * 4;
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(sw + kMfmaLdsMaxSteps);
    // Pipelined over the group's steps, unrolled by two so the register
    // halves swap roles instead of being copied: while step s's eight MFMAs
    // issue, the lane's window words and one-hot position for step s+1 and
    // the (uniform, broadcast) step word for s+2 are in flight.  All from
    // LDS: the step loop issues no global or scalar load.
    struct Frag {
      uint32_t w[7];  // the lane's 28 window bytes
      int rv;         // relo byte of (slot, DM)
      uint32_t hw;    // the lane's step half-word
    };
    auto lread = [&](uint32_t word, Frag& f) {  // issue only: nothing here waits on LDS
      f.hw = h ? (word >> 16) : (word & 0xFFFF);
      const int slot = static_cast<int>(f.hw & 15), rel = static_cast<int>((f.hw >> 4) & 255);
      const uint32_t* p = wb + ((slot * kMlWin + rel + sbase) >> 2);
#pragma unroll
      for (int k = 0; k < 7; ++k) f.w[k] = p[k];
      f.rv = rb[slot * 32 + r];  // unconditional: no divergent branch
    };
    auto mfma8 = [&](const Frag& f) {
      // one-hot column: byte dl of the 16-byte K-half (dl outside [0, 16)
      // -- negative or >= 16 -- gives (dl >> 2) outside 0..3: all zero)
      const int dl = (f.hw & 4096) ? -1 : f.rv - static_cast<int>((f.hw >> 4) & 255);
      const uint32_t* w = f.w;
      v4i bf;
#pragma unroll
      for (int q = 0; q < 4; ++q) bf[q] = ((dl >> 2) == q) ? (1 << ((dl & 3) * 8)) : 0;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int q = m >> 2;
        const uint32_t sh = static_cast<uint32_t>(m & 3);
        v4i a;
        a[0] = static_cast<int>(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh));
        a[1] = static_cast<int>(__builtin_amdgcn_alignbyte(w[q + 2], w[q + 1], sh));
        a[2] = static_cast<int>(__builtin_amdgcn_alignbyte(w[q + 3], w[q + 2], sh));
        a[3] = static_cast<int>(__builtin_amdgcn_alignbyte(w[q + 4], w[q + 3], sh));
        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bf, acc[m], 0, 0, 0);
      }
    };
    if (nst > 0) {
      const int last = nst - 1;
      Frag fA, fB;
      lread(sw[0], fA);
      uint32_t wordN = sw[min(1, last)];  // step s+1's word
      for (int s = 0; s < nst; s += 2) {
        // (sched_barrier: keep the prefetch reads in front of the MFMAs;
        // left alone the scheduler sinks them and waits on them at once)
        const uint32_t wordN2 = sw[min(s + 2, last)];
        lread(wordN, fB);  // step s+1 (a harmless re-read past the end)
        __builtin_amdgcn_sched_barrier(0);
        mfma8(fA);  // step s
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 > last) break;
        wordN = sw[min(s + 3, last)];
        lread(wordN2, fA);  // step s+2
        __builtin_amdgcn_sched_barrier(0);
        mfma8(fB);  // step s+1
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (g + 1 < ngroups) lstore(b ^ 1);
    __syncthreads();
  }
  // C/D layout (32x32): col = lane&31 (DM), row = (reg&3) + 8*(reg>>2) + 4*(lane>>5);
  // sub-tiles m = 0..7 of a (lane, reg) are the 8 consecutive samples 8*row + m
  const int d = tile * 32 + r - d_skip;  // the first tile's leading d_skip DMs are not stored
  if (d < 0 || d >= ndm) return;
  uint8_t* o = out + static_cast<uint64_t>(d) * out_stride;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
    const uint64_t t = t0 + wave * 256 + 8 * row;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) lo |= static_cast<uint32_t>(scale_out(acc[m][e] + bias_total, scale)) << (8 * m);
#pragma unroll
    for (int m = 0; m < 4; ++m) hi |= static_cast<uint32_t>(scale_out(acc[m + 4][e] + bias_total, scale)) << (8 * m);
    if (t + 8 <= out_nsamps) {
      *reinterpret_cast<uint2*>(o + t) = make_uint2(lo, hi);
    } else {
      for (int m = 0; m < 8; ++m)
        if (t + m < out_nsamps) o[t + m] = static_cast<uint8_t>((m < 4 ? lo : hi) >> (8 * (m & 3)));
    }
  }
}


// ------------------------------------------------ packed 2-bit, VALU SWAR --
// Narrow data (nbits <= 2: values 0..3) kept a second time as 2-bit fields,
// 16 samples per dword (sample t of row c at bit 2 (t & 15) of dword t / 16):
// a lane's 32 samples of one DM and channel are two dwords at a wave-uniform
// bit shift (v_alignbit of three LDS dwords: 0.375 LDS bytes per sample
// instead of the byte kernel's 2), added as nibble lanes (even / odd fields
// masked apart: 4 adds per 32 samples), spilled to byte lanes every 4
// channels (4 x 3 <= 15) and to 16-bit lanes every 64 (16 x 12 <= 255).
// Workgroup: 4 waves x DPW DMs x 2048 samples; per channel the workgroup's
// window (from the 32-DM tile's smallest offset, 64-sample aligned) is staged
// in LDS, 8 channels per buffer, double-buffered.
constexpr int k2bTs = 2048;    // samples per workgroup (64 lanes x 32)
constexpr int k2bCpb = 8;      // channels per LDS buffer (32 threads each)
constexpr int k2bWinDw = 384;  // largest staged window per channel (dwords = 16 samples)

__global__ void __launch_bounds__(256) pack2_kernel(const int8_t* __restrict__ x, uint64_t stride,
                                                    uint32_t* __restrict__ out, uint64_t stride2, uint64_t dw0,
                                                    uint64_t ndw) {
  const int8_t* row = x + static_cast<uint64_t>(blockIdx.y) * stride;
  uint32_t* orow = out + static_cast<uint64_t>(blockIdx.y) * stride2;
  for (uint64_t j = dw0 + static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; j < dw0 + ndw;
       j += static_cast<uint64_t>(gridDim.x) * 256) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(row + 16 * j);
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t b = v[i];  // four samples, one per byte, each 0..3
      const uint32_t p = (b & 3u) | ((b >> 6) & 0xCu) | ((b >> 12) & 0x30u) | ((b >> 18) & 0xC0u);
      w |= p << (8 * i);
    }
    orow[j] = w;
  }
}

template <int DPW>
__global__ void __launch_bounds__(256) dedisperse_2bit_kernel(
    const uint32_t* __restrict__ x2, uint64_t stride2, const int32_t* __restrict__ active, int nactive,
    const int32_t* __restrict__ offT, int ldo, int d_base, int d_skip, int ndm, const int32_t* __restrict__ wmin,
    int wvec, uint64_t out_nsamps, uint8_t* __restrict__ out, uint64_t out_stride, float scale) {
  __shared__ __attribute__((aligned(16))) uint32_t win[2][k2bCpb * k2bWinDw];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int dm0 = static_cast<int>(blockIdx.x) * (4 * DPW) + wave * DPW;  // relative to d_base
  const int tile = (d_base + static_cast<int>(blockIdx.x) * 4 * DPW) / 32;  // 4 DPW divides 32
  const uint64_t tb = static_cast<uint64_t>(blockIdx.y) * k2bTs;
  const int32_t* wm = wmin + static_cast<uint64_t>(tile) * nactive;
  uint32_t a4[DPW][4], a8[DPW][8], a16[DPW][16];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
#pragma unroll
    for (int m = 0; m < 4; ++m) a4[j][m] = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m) a8[j][m] = 0;
#pragma unroll
    for (int m = 0; m < 16; ++m) a16[j][m] = 0;
  }
  auto flush4 = [&]() {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        a8[j][2 * m] += a4[j][m] & 0x0F0F0F0Fu;
        a8[j][2 * m + 1] += (a4[j][m] >> 4) & 0x0F0F0F0Fu;
        a4[j][m] = 0;
      }
  };
  auto flush8 = [&]() {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        a16[j][2 * m] += a8[j][m] & 0x00FF00FFu;
        a16[j][2 * m + 1] += (a8[j][m] >> 8) & 0x00FF00FFu;
        a8[j][m] = 0;
      }
  };
  // Staging, per group of k2bCpb channels, one group ahead (double buffer):
  // thread (q = t / 32, e = t % 32) loads 16-byte vectors e, e + 32, e + 64
  // of channel q's window (wvec vectors: a launch-wide bound); threads t <
  // k2bCpb * 4 DPW also write one entry of the group's rel table (a DM
  // offset minus the channel's window start: the compute reads it from LDS,
  // uniform).  The indices behind those loads -- the window channel's row
  // (active) and start (wmin), the rel entry's offset and window start --
  // are loaded a further group ahead and parked in LDS with the windows, so
  // no global load waits on another issued in the same group (one dependent
  // round trip per 8 channels was most of the kernel at 2^20).
  constexpr int kRel = k2bCpb * 4 * DPW;  // rel entries per group
  static_assert(kRel <= 256, "one rel entry per thread");
  __shared__ int rel_l[2][kRel];
  __shared__ int4 idx_l[2][256];
  const int sq = threadIdx.x >> 5, se = threadIdx.x & 31;
  const int rq = static_cast<int>(threadIdx.x) / (4 * DPW), rk = static_cast<int>(threadIdx.x) % (4 * DPW);
  const bool rthread = static_cast<int>(threadIdx.x) < kRel;
  auto iload = [&](int c0) {  // {row, window start, rel offset, rel window start} of group c0
    const int ci = min(c0 + sq, nactive - 1);  // past the end: a harmless reload
    int4 v = make_int4(active[ci], wm[ci], 0, 0);
    if (rthread) {
      const int cr = min(c0 + rq, nactive - 1);
      v.z = offT[static_cast<uint64_t>(cr) * ldo + d_base + static_cast<int>(blockIdx.x) * 4 * DPW + rk];
      v.w = wm[cr];
    }
    return v;
  };
  u32x4 r[3];
  int relv = 0;
  auto gload = [&](const int4 ix) {
    const uint32_t* row = x2 + static_cast<uint64_t>(ix.x) * stride2 + ((tb + (ix.y & ~63)) >> 4);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (se + 32 * i < wvec) r[i] = *reinterpret_cast<const u32x4*>(row + 4 * (se + 32 * i));
    relv = ix.z - (ix.w & ~63);  // >= 0
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (se + 32 * i < wvec) *reinterpret_cast<u32x4*>(&win[buf][sq * k2bWinDw + 4 * (se + 32 * i)]) = r[i];
    if (rthread) rel_l[buf][threadIdx.x] = relv;
  };
  auto compute = [&](int ci, int q, const uint32_t* wb, const int* rl) {
    uint32_t d[DPW][3], sh[DPW];
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int rel = rl[q * 4 * DPW + wave * DPW + j];  // >= 0, wave-uniform (an LDS broadcast)
      sh[j] = 2u * static_cast<uint32_t>(rel & 15);
      const uint32_t* src = wb + 2 * lane + (rel >> 4);
      d[j][0] = src[0];
      d[j][1] = src[1];
      d[j][2] = src[2];
    }
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const uint32_t u0 = __builtin_amdgcn_alignbit(d[j][1], d[j][0], sh[j]);
      const uint32_t u1 = __builtin_amdgcn_alignbit(d[j][2], d[j][1], sh[j]);
      a4[j][0] += u0 & 0x33333333u;
      a4[j][1] += (u0 >> 2) & 0x33333333u;
      a4[j][2] += u1 & 0x33333333u;
      a4[j][3] += (u1 >> 2) & 0x33333333u;
    }
    if ((ci & 3) == 3) flush4();    // wave-uniform
    if ((ci & 63) == 63) flush8();
  };
  gload(iload(0));
  if (k2bCpb < nactive) idx_l[1][threadIdx.x] = iload(k2bCpb);  // group 1's indices
  lstore(0);
  __syncthreads();
  for (int c0 = 0, it = 0; c0 < nactive; c0 += k2bCpb, ++it) {
    const int buf = it & 1;
    const bool more = c0 + k2bCpb < nactive, more2 = c0 + 2 * k2bCpb < nactive;
    int4 nx = make_int4(0, 0, 0, 0);
    if (more) {
      gload(idx_l[buf ^ 1][threadIdx.x]);       // group + 1's windows, in flight during the sums
      if (more2) nx = iload(c0 + 2 * k2bCpb);  // group + 2's indices
    }
#pragma unroll 2
    for (int q = 0; q < k2bCpb; ++q)
      if (c0 + q < nactive) compute(c0 + q, q, &win[buf][q * k2bWinDw], rel_l[buf]);
    if (more) lstore(buf ^ 1);
    if (more2) idx_l[buf][threadIdx.x] = nx;  // (group + 2 uses buffer `buf` again)
    __syncthreads();
  }
  flush4();
  flush8();
  const uint64_t t = tb + static_cast<uint64_t>(lane) * 32;
  if (t >= out_nsamps) return;
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    if (dm0 + j >= ndm) break;  // ndm counts from d_base
    const int dd = dm0 + j - d_skip;
    if (dd < 0) continue;
    // sample s of word wi: a16[2 (4 wi + k) + ((s >> 2) & 1)] half s >> 3,
    // k = 0, 2, 1, 3 for s & 3 = 0, 1, 2, 3 (even fields, then odd)
    uint32_t ob[8];
#pragma unroll
    for (int wi = 0; wi < 2; ++wi)
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // output dword g of the word: samples 4g .. 4g+3
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int sidx = 4 * g + e;
          constexpr int kk[4] = {0, 2, 1, 3};
          const uint32_t h = a16[j][2 * (4 * wi + kk[e]) + ((sidx >> 2) & 1)];
          const int sum = static_cast<int>((sidx >> 3) ? (h >> 16) : (h & 0xFFFFu));
          v |= static_cast<uint32_t>(scale_out(sum, scale)) << (8 * e);
        }
        ob[4 * wi + g] = v;
      }
    uint8_t* orow = out + static_cast<uint64_t>(dd) * out_stride + t;
    if (t + 32 <= out_nsamps) {
      *reinterpret_cast<u32x4*>(orow) = u32x4{ob[0], ob[1], ob[2], ob[3]};
      *reinterpret_cast<u32x4*>(orow + 16) = u32x4{ob[4], ob[5], ob[6], ob[7]};
    } else {
      for (uint64_t e = 0; t + e < out_nsamps; ++e) orow[e] = static_cast<uint8_t>(ob[e >> 2] >> (8 * (e & 3)));
    }
  }
}

}  // namespace

void dedisperse_direct(const int8_t* chan_major, uint64_t chan_stride, int nchans, const int32_t* offsets,
                       const int32_t* killmask, int ndm, uint64_t out_nsamps, uint8_t* out, uint64_t out_stride,
                       float scale, int bias, int nactive, hipStream_t s) {
  if (ndm <= 0 || out_nsamps == 0) return;
  PSOUP_CHECK(ndm <= 65535, "too many DMs per launch");
  uint64_t gx = (out_nsamps + 1023) / 1024;
  dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(ndm));
  dedisperse_direct_kernel<<<grid, 256, 0, s>>>(chan_major, chan_stride, nchans, offsets, killmask, out_nsamps,
                                                 out, out_stride, scale, bias * nactive);
  post_launch_check("dedisperse_direct_kernel", s);
}


void build_mfma_dedisp_plan(const int32_t* offsets, int ndm, int nchans, const int32_t* killmask,
                            MfmaDedispPlan& plan) {
  const int ntiles = (ndm + 31) / 32;
  plan.ntiles = ntiles;
  std::vector<std::vector<int32_t>> tsteps(static_cast<size_t>(ntiles));
  std::vector<std::vector<int8_t>> tdeltas(static_cast<size_t>(ntiles));
  int max_steps = 1;
  for (int T = 0; T < ntiles; ++T) {
    auto off = [&](int dd, int c) {
      int d = std::min(T * 32 + dd, ndm - 1);  // pad the last tile with the last DM
      return offsets[static_cast<size_t>(d) * nchans + c];
    };
    std::vector<std::pair<int, int>> blocks;
    for (int c = 0; c < nchans; ++c) {
      if (killmask && !killmask[c]) continue;
      int smin = off(0, c), smax = off(0, c);
      for (int dd = 1; dd < 32; ++dd) {
        smin = std::min(smin, off(dd, c));
        smax = std::max(smax, off(dd, c));
      }
      PSOUP_CHECK(smin >= 0, "negative dispersion offset (foff > 0 is not supported)");
      for (int sb = smin; sb <= smax; sb += 16) blocks.emplace_back(c, sb);
    }
    if (blocks.size() % 2) blocks.push_back(std::make_pair(-1, -1));  // dummy half (zero one-hot)
    const int nst = static_cast<int>(blocks.size() / 2);
    auto& S = tsteps[T];
    auto& D = tdeltas[T];
    S.resize(static_cast<size_t>(nst) * 4);
    D.resize(static_cast<size_t>(nst) * 64);
    for (int s = 0; s < nst; ++s) {
      for (int hh = 0; hh < 2; ++hh) {
        auto blk = blocks[2 * s + hh];
        const bool dummy = blk.first < 0;
        const int c = dummy ? blocks[2 * s].first : blk.first;
        const int sb = dummy ? blocks[2 * s].second : blk.second;
        S[4 * s + 2 * hh] = c;
        S[4 * s + 2 * hh + 1] = sb;
        for (int rr = 0; rr < 32; ++rr) {
          int delta = -1;
          if (!dummy && T * 32 + rr < ndm) {
            const int dv = off(rr, c) - sb;
            if (dv >= 0 && dv < 16) delta = dv;
          }
          D[static_cast<size_t>(s) * 64 + hh * 32 + rr] = static_cast<int8_t>(delta);
        }
      }
    }
    max_steps = std::max(max_steps, nst);
  }
  plan.max_steps = max_steps;
  size_t total = 0;
  for (const auto& S : tsteps) total += S.size() / 4;
  plan.steps.assign(total * 4, 0);
  plan.deltas.assign(total * 64, static_cast<int8_t>(-1));
  plan.tile_info.assign(static_cast<size_t>(ntiles) * 2, 0);
  size_t at = 0;
  for (int T = 0; T < ntiles; ++T) {
    const size_t nst = tsteps[T].size() / 4;
    PSOUP_CHECK(at + nst < (1ull << 31), "MFMA dedispersion plan too large");
    plan.tile_info[2 * T] = static_cast<int32_t>(at);
    plan.tile_info[2 * T + 1] = static_cast<int32_t>(nst);
    std::copy(tsteps[T].begin(), tsteps[T].end(), plan.steps.begin() + at * 4);
    std::copy(tdeltas[T].begin(), tdeltas[T].end(), plan.deltas.begin() + at * 64);
    at += nst;
  }
}

void dedisperse_mfma(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_steps, const int8_t* d_deltas,
                     const int32_t* d_tile_info, int ntiles, int ndm, uint64_t out_nsamps, uint8_t* out,
                     uint64_t out_stride, float scale, int bias_total, hipStream_t s, int d_skip) {
  if (ndm <= 0 || out_nsamps == 0) return;
  PSOUP_CHECK(ntiles <= 65535, "too many DM tiles");
  PSOUP_CHECK(d_skip >= 0 && d_skip < 32 && d_skip + ndm <= 32 * ntiles, "dedisperse_mfma: bad tile range");
  const uint64_t ntt = (out_nsamps + kMfmaWgSamples - 1) / kMfmaWgSamples;
  dim3 grid(static_cast<unsigned>(ntiles), static_cast<unsigned>(std::min<uint64_t>(ntt, 65535)));
  dedisperse_mfma_kernel<<<grid, 256, 0, s>>>(chan_major, chan_stride, reinterpret_cast<const int4*>(d_steps),
                                               d_deltas, reinterpret_cast<const int2*>(d_tile_info), ndm, d_skip,
                                               out_nsamps,
                                               out, out_stride, scale,
                                               bias_total, ntt);
  post_launch_check("dedisperse_mfma_kernel", s);
}

void dedisperse_valu(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_active, int nactive,
                     const int32_t* d_offT, int ldo, int d_base, int ndm, uint64_t out_nsamps, uint8_t* out,
                     uint64_t out_stride, float scale, int nbits, int bias, hipStream_t s) {
  if (ndm <= 0 || out_nsamps == 0 || nactive <= 0) return;
  PSOUP_CHECK(bias == 0 || bias == 128, "dedisperse_valu: bias must be 0 or 128");
  PSOUP_CHECK((chan_stride & 3) == 0 && (out_stride & 15) == 0, "dedisperse_valu: stride alignment");
  const uint64_t max_raw = (1ull << std::min(nbits, 8)) - 1;
  const bool wide = max_raw * static_cast<uint64_t>(nactive) > 65535;
  const int dpt = wide ? 4 : 8;
  const uint64_t ty = (out_nsamps + 1023) / 1024;
  PSOUP_CHECK(ty <= 0x7FFFFFFF, "dedisperse_valu: series too long");
  dim3 grid(static_cast<unsigned>((ndm + 4 * dpt - 1) / (4 * dpt)), static_cast<unsigned>(ty));
  PSOUP_CHECK(d_base + static_cast<int>(grid.x) * 4 * dpt <= ldo, "dedisperse_valu: offset table too narrow");
#define PSOUP_VALU_LAUNCH(D, W, X)                                                                            \
  dedisperse_valu_kernel<D, W, X><<<grid, 256, 0, s>>>(chan_major, chan_stride, d_active, nactive, d_offT, ldo, \
                                                       d_base, ndm, out_nsamps, out, out_stride, scale)
  if (wide) {
    if (bias == 128)
      PSOUP_VALU_LAUNCH(4, true, true);
    else
      PSOUP_VALU_LAUNCH(4, true, false);
  } else {
    if (bias == 128)
      PSOUP_VALU_LAUNCH(8, false, true);
    else
      PSOUP_VALU_LAUNCH(8, false, false);
  }
#undef PSOUP_VALU_LAUNCH
  post_launch_check("dedisperse_valu_kernel", s);
}

void build_mfma_lds_plan(const int32_t* offsets, int ndm, int nchans, const int32_t* killmask, MfmaLdsPlan& plan,
                         int tile0, int tile1, int d_first) {
  constexpr int CG = kMfmaLdsGroup;
  std::vector<int> active;
  for (int c = 0; c < nchans; ++c)
    if (!killmask || killmask[c]) active.push_back(c);
  const int na = static_cast<int>(active.size());
  const int ntiles = (ndm + 31) / 32;
  const int ngroups = (na + CG - 1) / CG;
  plan.ntiles = ntiles;
  plan.ngroups = ngroups;
  plan.nactive = na;
  plan.steps.clear();
  plan.relo.assign(static_cast<size_t>(ntiles) * std::max(1, ngroups) * CG * 32, 0);
  plan.ginfo.assign(static_cast<size_t>(ntiles) * std::max(1, ngroups) * 2, 0);
  plan.wmin.assign(static_cast<size_t>(ntiles) * std::max(1, na), 0);
  plan.tile_ok.assign(static_cast<size_t>(ntiles), 0);
  plan.tile_steps.assign(static_cast<size_t>(ntiles), 0);
  // tiles outside [tile0, tile1) stay not-ok (no steps); offsets hold the
  // rows of DMs [d_first, ...)
  if (tile1 < 0 || tile1 > ntiles) tile1 = ntiles;
  tile0 = std::max(0, tile0);
  PSOUP_CHECK(d_first <= tile0 * 32, "MFMA-LDS plan: offsets start after the first tile");
  for (int T = tile0; T < tile1; ++T) {
    auto off = [&](int dd, int c) {
      const int d = std::min(T * 32 + dd, ndm - 1);  // pad the last tile with the last DM
      return offsets[static_cast<size_t>(d - d_first) * nchans + c];
    };
    bool ok = true;
    std::vector<int> lo(static_cast<size_t>(na)), hi(static_cast<size_t>(na));
    for (int ci = 0; ci < na; ++ci) {
      int a = off(0, active[ci]), b = a;
      for (int dd = 1; dd < 32; ++dd) {
        a = std::min(a, off(dd, active[ci]));
        b = std::max(b, off(dd, active[ci]));
      }
      PSOUP_CHECK(a >= 0, "negative dispersion offset (foff > 0 is not supported)");
      lo[ci] = a;
      hi[ci] = b;
      const int w0 = a & ~15;
      plan.wmin[static_cast<size_t>(T) * na + ci] = w0;
      // the last block starts at most (hi - w0) bytes in; a lane reads 7
      // dwords from there + 256 * wave + 8 * row (<= 1016): 1044 bytes past it
      if ((hi[ci] - w0) + 1044 > kMfmaLdsWindow) ok = false;
    }
    plan.tile_ok[static_cast<size_t>(T)] = ok ? 1 : 0;
    if (!ok) continue;  // the VALU kernels take this tile
    int tsteps = 0;
    for (int g = 0; g < ngroups; ++g) {
      std::vector<std::pair<int, int>> blocks;  // (slot, rel)
      for (int ci = g * CG; ci < std::min(na, (g + 1) * CG); ++ci) {
        const int w0 = plan.wmin[static_cast<size_t>(T) * na + ci];
        // blocks start on a multiple of 4 (w0 is one of 16): every window
        // offset rel is 4-aligned, so the kernel's byte shifts are static
        for (int sb = lo[ci] & ~3; sb <= hi[ci]; sb += 16) blocks.emplace_back(ci - g * CG, sb - w0);
      }
      if (blocks.size() % 2) blocks.push_back(std::make_pair(-1, -1));  // empty half (zero one-hot)
      const int nst = static_cast<int>(blocks.size() / 2);
      PSOUP_CHECK(nst <= kMfmaLdsMaxSteps, "MFMA-LDS plan: too many steps in a channel group");
      while (plan.steps.size() % 4) plan.steps.push_back(0);  // 16-byte aligned group start
      plan.ginfo[(static_cast<size_t>(T) * ngroups + g) * 2] = static_cast<int32_t>(plan.steps.size());
      plan.ginfo[(static_cast<size_t>(T) * ngroups + g) * 2 + 1] = nst;
      for (int st = 0; st < nst; ++st) {
        uint32_t word = 0;
        for (int hh = 0; hh < 2; ++hh) {
          const auto blk = blocks[static_cast<size_t>(2 * st + hh)];
          const bool empty = blk.first < 0;
          const auto use = empty ? blocks[static_cast<size_t>(2 * st)] : blk;  // a valid address
          PSOUP_CHECK(use.second >= 0 && use.second < 256, "MFMA-LDS plan: window offset");
          const uint32_t half = static_cast<uint32_t>(use.first) | (static_cast<uint32_t>(use.second) << 4) |
                                (empty ? 4096u : 0u);
          word |= half << (16 * hh);
        }
        plan.steps.push_back(static_cast<int32_t>(word));
      }
      for (int ci = g * CG; ci < std::min(na, (g + 1) * CG); ++ci) {
        const int w0 = plan.wmin[static_cast<size_t>(T) * na + ci];
        uint8_t* dst = &plan.relo[((static_cast<size_t>(T) * ngroups + g) * CG + (ci - g * CG)) * 32];
        for (int rr = 0; rr < 32; ++rr) {
          const int v = off(rr, active[ci]) - w0;  // padded DMs repeat the last one (never stored)
          PSOUP_CHECK(v >= 0 && v < 256, "MFMA-LDS plan: relative offset");
          dst[rr] = static_cast<uint8_t>(v);
        }
      }
      tsteps += nst;
    }
    plan.tile_steps[static_cast<size_t>(T)] = tsteps;
    PSOUP_CHECK(plan.steps.size() < (1ull << 31), "MFMA-LDS dedispersion plan too large");
  }
  plan.steps.resize(plan.steps.size() + kMfmaLdsMaxSteps, 0);  // the staging reads a full step block
}

void dedisperse_mfma_lds(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_active, int nactive,
                         const int32_t* d_steps, const uint8_t* d_relo, const int32_t* d_ginfo, int ngroups,
                         const int32_t* d_wmin, int ntiles, int ndm, uint64_t out_nsamps, uint8_t* out,
                         uint64_t out_stride, float scale, int bias_total, hipStream_t s, int d_skip) {
  if (ndm <= 0 || out_nsamps == 0 || nactive <= 0) return;
  PSOUP_CHECK(ntiles >= 1 && ntiles <= 65535 && d_skip >= 0 && d_skip < 32 && d_skip + ndm <= 32 * ntiles,
              "dedisperse_mfma_lds: bad tile range");
  PSOUP_CHECK((chan_stride & 15) == 0, "dedisperse_mfma_lds: stride alignment");
  const uint64_t ty = (out_nsamps + kMlTs - 1) / kMlTs;
  if (ty > 65535) {  // beyond one grid: consecutive shifted time ranges (as dedisperse_2bit)
    constexpr uint64_t kSpan = 65535ull * kMlTs;
    for (uint64_t t0 = 0; t0 < out_nsamps; t0 += kSpan)
      dedisperse_mfma_lds(chan_major + t0, chan_stride, d_active, nactive, d_steps, d_relo, d_ginfo, ngroups, d_wmin,
                          ntiles, ndm, std::min(kSpan, out_nsamps - t0), out + t0, out_stride, scale, bias_total, s,
                          d_skip);
    return;
  }
  dim3 grid(static_cast<unsigned>(ntiles), static_cast<unsigned>(ty));
  dedisperse_mfma_lds_kernel<kMfmaLdsGroup><<<grid, 256, 0, s>>>(
      chan_major, chan_stride, d_active, nactive, reinterpret_cast<const uint32_t*>(d_steps), d_relo,
      reinterpret_cast<const int2*>(d_ginfo), ngroups, d_wmin, ndm, d_skip, out_nsamps, out, out_stride, scale,
      bias_total);
  post_launch_check("dedisperse_mfma_lds_kernel", s);
}

bool dedisperse_lds_fits(int nbits, int nactive, int max_window) {
  const uint64_t max_raw = (1ull << std::min(nbits, 8)) - 1;
  return max_raw * static_cast<uint64_t>(nactive) <= 65535 && max_window <= 4 * kLdsWinWords;
}

void dedisperse_lds(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_active, int nactive,
                    const int32_t* d_offT, int ldo, int d0, int ndm, const int32_t* d_wmin, int max_window,
                    uint64_t out_nsamps, uint8_t* out, uint64_t out_stride, float scale, int nbits, int bias,
                    hipStream_t s) {
  if (ndm <= 0 || out_nsamps == 0 || nactive <= 0) return;
  PSOUP_CHECK(d0 >= 0, "dedisperse_lds: negative first DM");
  PSOUP_CHECK(dedisperse_lds_fits(nbits, nactive, max_window), "dedisperse_lds: window or sums too large");
  PSOUP_CHECK((chan_stride & 15) == 0 && (out_stride & 15) == 0, "dedisperse_lds: stride alignment");
  const uint64_t ty = (out_nsamps + 1023) / 1024;
  if (ty > 65535) {  // beyond one grid: consecutive shifted time ranges (as dedisperse_2bit)
    constexpr uint64_t kSpan = 65535ull * 1024;
    for (uint64_t t0 = 0; t0 < out_nsamps; t0 += kSpan)
      dedisperse_lds(chan_major + t0, chan_stride, d_active, nactive, d_offT, ldo, d0, ndm, d_wmin, max_window,
                     std::min(kSpan, out_nsamps - t0), out + t0, out_stride, scale, nbits, bias, s);
    return;
  }
  // DMs per wave: a launch of <= 8 DMs (the headline bench's per-rank chunk)
  // fills 8-DM workgroups instead of half-empty 16-DM ones; otherwise 4
  // (config-4 DM list: 141 ms vs 173 ms at 8).  Two-pass windows (> 4096
  // samples) are built for 4 only.
  const bool two = max_window > 4096;
  const int dpt = ndm <= 8 && !two ? 2 : 4;
  // workgroups start on multiples of their 4*dpt DMs (one absolute tile's
  // window each): a range from any DM starts at the workgroup boundary below
  // it and skips the DMs before d0
  const int d_base = d0 / (4 * dpt) * (4 * dpt), d_skip = d0 - d_base;
  dim3 grid(static_cast<unsigned>((ndm + d_skip + 4 * dpt - 1) / (4 * dpt)), static_cast<unsigned>(ty));
  PSOUP_CHECK(d_base + static_cast<int>(grid.x) * 4 * dpt <= ldo, "dedisperse_lds: offset table too narrow");
  const bool xr = bias == 128;
  // byte-lane sums (narrow unsigned samples: flush * max raw value <= 255;
  // one channel per barrier: 140 ms vs 153 / 185 ms at 2 / 4)
  const int max_raw = (1 << std::min(nbits, 8)) - 1;
  const int flush = max_raw > 0 ? 255 / max_raw : 255;
  const bool bytes = !xr && nbits <= 4 && flush >= 1 && !two;
  if (bytes) {
    if (dpt == 4)
      dedisperse_lds_kernel<false, 1, 4, 1, true><<<grid, 256, 0, s>>>(chan_major, chan_stride, d_active, nactive,
                                                                       d_offT, ldo, d_base, d_skip, ndm + d_skip,
                                                                       d_wmin, out_nsamps, out, out_stride, scale,
                                                                       flush);
    else
      dedisperse_lds_kernel<false, 1, 2, 1, true><<<grid, 256, 0, s>>>(chan_major, chan_stride, d_active, nactive,
                                                                       d_offT, ldo, d_base, d_skip, ndm + d_skip,
                                                                       d_wmin, out_nsamps, out, out_stride, scale,
                                                                       flush);
    post_launch_check("dedisperse_lds_kernel", s);
    return;
  }
#define PSOUP_LDS_LAUNCH(X, P, D, C)                                                                           \
  dedisperse_lds_kernel<X, P, D, C><<<grid, 256, 0, s>>>(chan_major, chan_stride, d_active, nactive, d_offT, ldo, \
                                                         d_base, d_skip, ndm + d_skip, d_wmin, out_nsamps, out,      \
                                                         out_stride, scale, 255)
#define PSOUP_LDS_ONE(X)          \
  if (two)                         \
    PSOUP_LDS_LAUNCH(X, 2, 4, 1);  \
  else if (dpt == 2)               \
    PSOUP_LDS_LAUNCH(X, 1, 2, 1);  \
  else                             \
    PSOUP_LDS_LAUNCH(X, 1, 4, 1);
  if (xr) {
    PSOUP_LDS_ONE(true)
  } else {
    PSOUP_LDS_ONE(false)
  }
#undef PSOUP_LDS_ONE
#undef PSOUP_LDS_LAUNCH
  post_launch_check("dedisperse_lds_kernel", s);
}


void pack2_rows(const int8_t* chan_major, uint64_t chan_stride, int nrows, uint32_t* out, uint64_t stride2, uint64_t t0,
                uint64_t ns, hipStream_t s) {
  if (ns == 0 || nrows <= 0) return;
  PSOUP_CHECK(t0 % 16 == 0 && (chan_stride & 15) == 0, "pack2_rows: alignment");
  const uint64_t dw0 = t0 / 16, ndw = (ns + 15) / 16;
  PSOUP_CHECK(16 * (dw0 + ndw) <= chan_stride && dw0 + ndw <= stride2, "pack2_rows: past the rows");
  PSOUP_CHECK(nrows <= 65535, "pack2_rows: too many rows");
  dim3 grid(static_cast<unsigned>(std::min<uint64_t>((ndw + 255) / 256, 1024)), static_cast<unsigned>(nrows));
  pack2_kernel<<<grid, 256, 0, s>>>(chan_major, chan_stride, out, stride2, dw0, ndw);
  post_launch_check("pack2_kernel", s);
}

int dedisperse_2bit_window(int max_spread) { return ((k2bTs + max_spread + 48 + 63) / 64 + 1) * 4; }
bool dedisperse_2bit_fits(int nactive, int max_spread) {
  return nactive <= 21845 && dedisperse_2bit_window(max_spread) <= k2bWinDw;
}

void dedisperse_2bit(const uint32_t* x2, uint64_t stride2, const int32_t* d_active, int nactive, const int32_t* d_offT,
                     int ldo, int d0, int ndm, const int32_t* d_wmin, int max_spread, int max_offset,
                     uint64_t out_nsamps, uint8_t* out, uint64_t out_stride, float scale, hipStream_t s) {
  if (ndm <= 0 || out_nsamps == 0 || nactive <= 0) return;
  PSOUP_CHECK(dedisperse_2bit_fits(nactive, max_spread), "dedisperse_2bit: window or sums too large");
  PSOUP_CHECK((out_stride & 15) == 0 && d0 >= 0, "dedisperse_2bit: stride alignment");
  const uint64_t ty = (out_nsamps + k2bTs - 1) / k2bTs;
  PSOUP_CHECK(16 * stride2 >= ty * k2bTs + static_cast<uint64_t>(max_offset) +
                                   16ull * static_cast<uint64_t>(dedisperse_2bit_window(max_spread)) &&
                  stride2 % 4 == 0,
              "dedisperse_2bit: packed rows too short for the windows");
  if (ty > 65535) {
    // longer than one grid (2^26 samples and up): consecutive time ranges of
    // 65535 tiles, input and output shifted by the same number of samples
    constexpr uint64_t kSpan = 65535ull * k2bTs;
    static_assert(k2bTs % 64 == 0, "shifted packed rows stay 16-byte aligned");
    for (uint64_t t0 = 0; t0 < out_nsamps; t0 += kSpan) {
      dedisperse_2bit(x2 + t0 / 16, stride2, d_active, nactive, d_offT, ldo, d0, ndm, d_wmin, max_spread, max_offset,
                      std::min(kSpan, out_nsamps - t0), out + t0, out_stride, scale, s);
    }
    return;
  }
  // DMs per wave: 4 (16-DM workgroups); a launch of <= 8 DMs from an 8-DM
  // boundary (the headline bench's per-rank chunk) takes 8-DM workgroups
  // instead of computing 8 DMs it does not store
  const int dpw = (ndm <= 8 && (d0 % 8) + ndm <= 8) ? 2 : 4;
  const int d_base = d0 / (4 * dpw) * (4 * dpw), d_skip = d0 - d_base;
  dim3 grid(static_cast<unsigned>((ndm + d_skip + 4 * dpw - 1) / (4 * dpw)), static_cast<unsigned>(ty));
  PSOUP_CHECK(d_base + static_cast<int>(grid.x) * 4 * dpw <= ldo, "dedisperse_2bit: offset table too narrow");
  if (dpw == 2)
    dedisperse_2bit_kernel<2><<<grid, 256, 0, s>>>(x2, stride2, d_active, nactive, d_offT, ldo, d_base, d_skip,
                                                   ndm + d_skip, d_wmin, dedisperse_2bit_window(max_spread) / 4,
                                                   out_nsamps, out, out_stride, scale);
  else
    dedisperse_2bit_kernel<4><<<grid, 256, 0, s>>>(x2, stride2, d_active, nactive, d_offT, ldo, d_base, d_skip,
                                                   ndm + d_skip, d_wmin, dedisperse_2bit_window(max_spread) / 4,
                                                   out_nsamps, out, out_stride, scale);
  post_launch_check("dedisperse_2bit_kernel", s);
}

}  // namespace kern
}  // namespace psoup
