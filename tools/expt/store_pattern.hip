// Store-pattern microbenchmark for the four-step FFT passes: K trials x M
// complex (M = 2^22, 33.5 MB per trial) written by 256-thread workgroups that
// each own an 8-transform x 2048-point block (128 KiB), in the patterns the
// passes use, with the passes' occupancy (72 KiB of LDS per workgroup: two
// workgroups per CU) or unconstrained.
//   tileY   : Y_t[i/8][k2/8][i%8][k2%8]: per store instruction 8 lanes x 8 B
//             = 64 B pieces, 512 B apart (fft4 pass A default)
//   blocked : each lane 64 contiguous bytes as 4 x 16 B, lanes 64 B apart
//   contig  : each store instruction 64 lanes x 16 B = 1 KiB contiguous
// build: hipcc --offload-arch=gfx950 -O3 store_pattern.hip -o store_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int L = 2048, T = 256;
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int MODE, bool NT>
__global__ void __launch_bounds__(256) wblock(float2* __restrict__ Y, int K, size_t ystride) {
  extern __shared__ float pad[];
  if (threadIdx.x == 1023) pad[0] = 0.f;
  const int nbt = L / 8;  // blocks per trial (8 columns each)
  const int k = blockIdx.x % K, cb = blockIdx.x / K;
  const int c0 = cb * 8, t = threadIdx.x;
  float2* yk = Y + (size_t)k * ystride;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k2 = t + q * T;
    if (MODE == 0) {  // tileY
      float2* dst = yk + (size_t)c0 * L + (k2 >> 3) * 64 + (k2 & 7);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const v2f v = {(float)c, (float)q};
        v2f* d = reinterpret_cast<v2f*>(dst + c * 8);
        if (NT) __builtin_nontemporal_store(v, d); else *d = v;
      }
    } else if (MODE == 1) {  // blocked: Y_b[c0/8][k2][c]
      v4f* dst = reinterpret_cast<v4f*>(yk + (size_t)c0 * L + (size_t)k2 * 8);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const v4f v = {(float)c, (float)q, 1.f, 2.f};
        if (NT) __builtin_nontemporal_store(v, dst + c); else dst[c] = v;
      }
    } else {  // contiguous 1 KiB per instruction
      v4f* dst = reinterpret_cast<v4f*>(yk + (size_t)c0 * L) + q * 4 * T;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const v4f v = {(float)c, (float)q, 1.f, 2.f};
        if (NT) __builtin_nontemporal_store(v, dst + c * T + t); else dst[c * T + t] = v;
      }
    }
  }
  (void)nbt;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 32;
  const size_t M = (size_t)L * L, ystride = M + 64;
  float2* Y;
  if (hipMalloc(&Y, ystride * K * sizeof(float2)) != hipSuccess) return 1;
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
    printf("%-34s %7.2f us/trial %6.0f GB/s\n", name, us, M * 8.0 / (us * 1e-6) / 1e9);
  };
  const int grid = (L / 8) * K;
  for (int lds : {74752, 0}) {
    char n[64];
#define RUN(MODE, NT, label)                                                                  \
  snprintf(n, sizeof n, "%s%s lds=%d", label, NT ? " nt" : "", lds);                          \
  time(n, [&] { wblock<MODE, NT><<<grid, 256, lds>>>(Y, K, ystride); });
    RUN(0, false, "tileY") RUN(0, true, "tileY") RUN(1, false, "blocked") RUN(1, true, "blocked")
    RUN(2, false, "contig") RUN(2, true, "contig")
  }
  return 0;
}
