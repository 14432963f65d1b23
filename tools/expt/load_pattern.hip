// Load-pattern microbenchmark for fft4 pass A's input reads: K "trials" of
// 256 workgroups x 256 threads, each thread loading 8 spans (q) of 16 floats,
// two workgroups per CU (72 KiB of LDS each), input resident in L2/MALL (one
// 34 MB series shared by every trial, as in a real acceleration batch).
//   rows     : lane = row j (rows 16 KiB apart), 4 x 16-byte loads per span at
//              an arbitrary dword offset (pass A today)
//   rows16   : the same, 16-byte aligned
//   rowsx2   : 8 x 8-byte loads per span
//   contig   : every load instruction reads 1 KiB contiguous (upper bound)
//   tdword   : transposed copy, 16 dword loads per span, 256 B per instruction
// build: hipcc --offload-arch=gfx950 -O3 load_pattern.hip -o load_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
constexpr int N1 = 2048, N2 = 2048, T = 256, PITCH = 2 * N1 + 32;

__device__ __forceinline__ double apos(double af, double size, double d) { return d + d * af * (d - size); }

template <int MODE>
__global__ void __launch_bounds__(256) lk(const float* __restrict__ in, float* __restrict__ out, int K, int shift) {
  extern __shared__ float pad[];
  if (threadIdx.x == 1023) pad[0] = 0.f;
  const int k = blockIdx.x % K, cb = blockIdx.x / K;
  const int c0 = cb * 8, t = threadIdx.x;
  const int s = shift + k * 3;  // per-trial shift (consecutive accelerations: a few samples apart)
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int j = t + q * T;
    if (MODE == 0 || MODE == 1) {
      const int off = MODE == 0 ? s : (s & ~3);
      const f4u* src = reinterpret_cast<const f4u*>(in + (size_t)j * PITCH + 2 * c0 + off);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f4u w = src[u];
        acc += w.x + w.y + w.z + w.w;
      }
    } else if (MODE == 2) {
      const f2u* src = reinterpret_cast<const f2u*>(in + (size_t)j * PITCH + 2 * c0 + s);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f2u w = src[u];
        acc += w.x + w.y;
      }
    } else if (MODE == 3) {
      const f4u* src = reinterpret_cast<const f4u*>(in + (size_t)(((cb * 8 + q) % 512) * 4096)) + t;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f4u w = src[u * T];
        acc += w.x + w.y + w.z + w.w;
      }
    } else if (MODE == 4) {  // transposed: row = 2*c0 + e + s (+pad), column j
      const float* src = in + (size_t)(2 * c0 + s + 64) * (N2 + 32) + j;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc += src[(size_t)e * (N2 + 32)];
    } else if (MODE == 5) {  // transposed via buffer loads with SGPR offsets
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), 0, 0x7fffffff, 0x00020000);
      const unsigned vo = ((2 * c0 + s + 64) * (N2 + 32) + j) * 4u;
#pragma unroll
      for (int e = 0; e < 17; ++e)
        acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, e * (N2 + 32) * 4, 0));
    } else if (MODE == 9) {  // MODE 7's varying rows, shift from fp32 arithmetic (no double)
      const float aff = (200.0f + 1.464f * k) * 64e-6f / (2 * 299792458.0f);
      const float p = 4096.0f * j + 2.0f * c0;
      const int sh = (int)rintf(aff * p * (p - 8388608.0f));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), 0, 0x7fffffff, 0x00020000);
      const unsigned row = (unsigned)(2 * c0 + sh + 2048);
      const unsigned vo = (row * (N2 + 32) + j) * 4u;
#pragma unroll
      for (int e = 0; e < 17; ++e)
        acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, e * (N2 + 32) * 4, 0));
    } else if (MODE == 10) {  // rows pattern (plain layout) with the realistic varying shift, fp32
      const float aff = (200.0f + 1.464f * k) * 64e-6f / (2 * 299792458.0f);
      const float p = 4096.0f * j + 2.0f * c0;
      const int sh = (int)rintf(aff * p * (p - 8388608.0f));
      const f4u* src = reinterpret_cast<const f4u*>(in + (size_t)j * PITCH + 2 * c0 + 2048 + sh);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f4u w = src[u];
        acc += w.x + w.y + w.z + w.w;
      }
    } else if (MODE == 11 || MODE == 12) {  // 8 lanes per row (c = t & 7), 8 bytes per lane, rows g + 32 m
      if (q == 0) {
        const int c = t & 7, g = t >> 3;
        const float aff = (200.0f + 1.464f * k) * 64e-6f / (2 * 299792458.0f);
#pragma unroll
        for (int m = 0; m < 64; ++m) {
          const int jj = g + 32 * m;
          int sh = s;
          if (MODE == 12) {
            const float p = 4096.0f * jj + 2.0f * c0;
            sh = 2048 + (int)rintf(aff * p * (p - 8388608.0f));
          }
          const f2u w = *reinterpret_cast<const f2u*>(in + (size_t)jj * PITCH + 2 * (c0 + c) + sh);
          acc += w.x + w.y;
        }
      }
    } else if (MODE == 13 || MODE == 14) {  // 4 lanes per row (2 columns each), 16 bytes per lane, rows g + 64 m
      if (q == 0) {
        const int cp = t & 3, g = t >> 2;
        const float aff = (200.0f + 1.464f * k) * 64e-6f / (2 * 299792458.0f);
#pragma unroll
        for (int m = 0; m < 32; ++m) {
          const int jj = g + 64 * m;
          int sh = s;
          if (MODE == 14) {
            const float p = 4096.0f * jj + 2.0f * c0;
            sh = 2048 + (int)rintf(aff * p * (p - 8388608.0f));
          }
          const f4u w = *reinterpret_cast<const f4u*>(in + (size_t)jj * PITCH + 2 * c0 + 4 * cp + sh);
          acc += w.x + w.y + w.z + w.w;
        }
      }
    } else if (MODE == 7 || MODE == 8) {  // transposed, realistic per-row shift (varies along j), buffer loads
      // shift of row j for trial k at acceleration 200 + 1.464 k m/s^2 (the parabola, 0..-375 samples)
      const double af = (200.0 + 1.464 * k) * 64e-6 / (2 * 299792458.0);
      const double p = 4096.0 * j + 2.0 * c0;
      const int sh = (int)rint(af * p * (p - 8388608.0));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), 0, 0x7fffffff, 0x00020000);
      const unsigned row = MODE == 7 ? (unsigned)(2 * c0 + sh + 2048) : (unsigned)(2 * c0 + 2048 - 100);
      const unsigned vo = (row * (N2 + 32) + j) * 4u;
#pragma unroll
      for (int e = 0; e < 17; ++e)
        acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, e * (N2 + 32) * 4, 0));
    } else {  // MODE 6: + the exact double-precision span classification per q
      const double af = (200.0 + 1.464 * k) * 64e-6 / (2 * 299792458.0), size = 8388608.0;
      const double d0 = (double)(4096u * (unsigned)j + 2u * (unsigned)c0), d1 = d0 + 15.0;
      const double r0 = apos(af, size, d0), r1 = apos(af, size, d1);
      const double q0 = rint(r0), q1 = rint(r1);
      const bool ok = (0.5 - fabs(r0 - q0) > 1e-7) && (0.5 - fabs(r1 - q1) > 1e-7) && q0 >= 0.0 &&
                      fabs(0.5 * (d0 + d1) - 0.5 * size) > 8192.0;
      const int sh = ok ? (int)(q0 - d0) : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in), 0, 0x7fffffff, 0x00020000);
      const unsigned vo = ((2 * c0 + (sh & 255) + 64) * (N2 + 32) + j) * 4u;
#pragma unroll
      for (int e = 0; e < 17; ++e)
        acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, e * (N2 + 32) * 4, 0));
    }
  }
  if (acc == 1234.5f) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 32;
  const size_t nin = (size_t)(2 * N1 + 4096 + 64) * (N2 + 32) + (1 << 20);
  float *in, *out;
  if (hipMalloc(&in, nin * 4) != hipSuccess || hipMalloc(&out, 1 << 22) != hipSuccess) return 1;
  (void)hipMemset(in, 0, nin * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](const char* name, auto fn) {
    fn();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) fn();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 10 / K;
    printf("%-12s %7.2f us/trial (%.0f GB/s of span data)\n", name, us, 8.0 * N1 * N2 / (us * 1e-6) / 1e9);
  };
  const int grid = (N1 / 8) * K;
  const int lds = 74752;
  time("rows", [&] { lk<0><<<grid, 256, lds>>>(in, out, K, 5); });
  time("rows16", [&] { lk<1><<<grid, 256, lds>>>(in, out, K, 5); });
  time("rowsx2", [&] { lk<2><<<grid, 256, lds>>>(in, out, K, 5); });
  time("contig", [&] { lk<3><<<grid, 256, lds>>>(in, out, K, 5); });
  time("tdword", [&] { lk<4><<<grid, 256, lds>>>(in, out, K, 5); });
  time("tbuffer", [&] { lk<5><<<grid, 256, lds>>>(in, out, K, 5); });
  time("tshift", [&] { lk<7><<<grid, 256, lds>>>(in, out, K, 5); });
  time("tnoshift", [&] { lk<8><<<grid, 256, lds>>>(in, out, K, 5); });
  time("tshift32", [&] { lk<9><<<grid, 256, lds>>>(in, out, K, 5); });
  time("rowshift32", [&] { lk<10><<<grid, 256, lds>>>(in, out, K, 5); });
  time("tbuf+f64", [&] { lk<6><<<grid, 256, lds>>>(in, out, K, 5); });
  time("lane8", [&] { lk<11><<<grid, 256, lds>>>(in, out, K, 5); });
  time("lane8shift", [&] { lk<12><<<grid, 256, lds>>>(in, out, K, 5); });
  time("lane4x16", [&] { lk<13><<<grid, 256, lds>>>(in, out, K, 5); });
  time("lane4x16sh", [&] { lk<14><<<grid, 256, lds>>>(in, out, K, 5); });
  time("rows", [&] { lk<0><<<grid, 256, lds>>>(in, out, K, 5); });
  return 0;
}
