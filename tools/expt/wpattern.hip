// Write-pattern microbenchmark: cost of natural-order spectrum writes from a
// row-decomposed FFT pass (each workgroup owns 7-8 consecutive rows k2 of
// P[k1*n2 + k2] for all k1: 28-32 byte chunks 8 KB apart) vs contiguous writes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int N1 = 2048, N2 = 2048;

// contiguous: each WG writes 16 rows' worth of floats contiguously
__global__ void __launch_bounds__(512) wcontig(float* P, int K) {
  const int per = 16 * N1;
  const int blk = blockIdx.x;
  float* p = P + (size_t)blk * per;
  for (int i = threadIdx.x; i < per; i += 512) p[i] = (float)i;
}

// chunked: WG b (per trial) writes rows [rb, rb+R) of P[k1*N2 + k2] for all k1,
// twice (ascending + mirror block), each thread owning k1 = t + 256 q.
template <int R, int STEP, bool REMAP, bool LANET>
__global__ void __launch_bounds__(512) wchunk(float* P, int K, int nb) {
  const unsigned hw = blockIdx.x, G = gridDim.x;
  const unsigned lb = REMAP ? (hw & 7u) * (G >> 3) + (hw >> 3) : hw;
  const int trial = lb / nb, b = lb % nb;
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
  float* p = P + (size_t)trial * ((size_t)N1 * N2 + 64);
  const int r0 = grp == 0 ? STEP * b + 1 : N2 - STEP * b - R;
  if (r0 < 0 || r0 + R > N2) return;
  if (LANET) {
    // lane-transposed: 8 lanes cover one k1's (up to) 8 rows, so each store
    // instruction writes 8 chunks of 32 bytes
    const int sub = t & 7, kk = t >> 3;  // 32 k1 per pass
#pragma unroll
    for (int pass = 0; pass < 64; ++pass) {
      const int k1 = kk + 32 * pass;
      if (sub < R) p[(size_t)k1 * N2 + r0 + sub] = (float)(sub + pass);
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k1 = t + 256 * q;
#pragma unroll
      for (int c = 0; c < R; ++c) p[(size_t)k1 * N2 + r0 + c] = (float)(c + q);
    }
  }
}

__global__ void __launch_bounds__(256) rcontig(const float4* __restrict__ P, size_t n4, float* out) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    float4 v = P[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
}
__global__ void __launch_bounds__(256) wcontig4(float4* __restrict__ P, size_t n4) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    P[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// write-only with occupancy limited by dynamic LDS (lds_bytes per WG)
__global__ void __launch_bounds__(256) wocc(float4* __restrict__ P, size_t n4) {
  extern __shared__ float pad[];
  if (threadIdx.x == 1023) pad[0] = 0.f;  // never true; keeps the allocation
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    P[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
// same, but each thread writes 32 x 16 B in one burst at the end (FFT-like)
__global__ void __launch_bounds__(256) wburst(float4* __restrict__ P, size_t n4) {
  extern __shared__ float pad[];
  if (threadIdx.x == 1023) pad[0] = 0.f;
  const size_t per = 256 * 32;
  const size_t nblk = n4 / per;
  for (size_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    float4* d = P + b * per;
#pragma unroll
    for (int j = 0; j < 32; ++j) d[j * 256 + threadIdx.x] = make_float4(1.f, 2.f, 3.f, (float)j);
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 32;
  float* P;
  const size_t per = (size_t)N1 * N2 + 64;
  hipMalloc(&P, per * K * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](const char* name, auto fn) {
    fn();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 10 / K;
    printf("%-28s %8.2f us/trial  %7.0f GB/s\n", name, us, N1 * (double)N2 * 4 / (us * 1e-6) / 1e9);
  };
  {
    const size_t n4 = per * K / 4;
    float* o;
    hipMalloc(&o, 64);
    time("read-only float4 (grid 8192)", [&] { rcontig<<<8192, 256>>>((const float4*)P, n4, o); });
    time("write-only float4 (grid 8192)", [&] { wcontig4<<<8192, 256>>>((float4*)P, n4); });
    time("write-only float4 (grid 2048)", [&] { wcontig4<<<2048, 256>>>((float4*)P, n4); });
  }
  {
    const size_t n4 = per * K / 4;
    for (int wgs : {1, 2, 4, 8}) {
      const size_t lds = 160 * 1024 / wgs - 1024;
      char name[64];
      snprintf(name, sizeof(name), "write-only, %d WG/CU", wgs);
      time(name, [&] { wocc<<<256 * wgs, 256, lds>>>((float4*)P, n4); });
      snprintf(name, sizeof(name), "write burst, %d WG/CU", wgs);
      time(name, [&] { wburst<<<256 * wgs, 256, lds>>>((float4*)P, n4); });
    }
  }
  const int nbc = (N1 * N2) / (16 * N1);
  time("contiguous", [&] { wcontig<<<nbc * K, 512>>>(P, K); });
  const int nb7 = (N2 / 2 + 6) / 7;
  time("7-row chunks", [&] { wchunk<7, 7, false, false><<<nb7 * K, 512>>>(P, K, nb7); });
  time("7-row chunks remap", [&] { wchunk<7, 7, true, false><<<nb7 * K, 512>>>(P, K, nb7); });
  time("7-row chunks lanes", [&] { wchunk<7, 7, false, true><<<nb7 * K, 512>>>(P, K, nb7); });
  time("7-row chunks remap+lanes", [&] { wchunk<7, 7, true, true><<<nb7 * K, 512>>>(P, K, nb7); });
  const int nb8 = N2 / 16;
  time("8-row chunks remap+lanes", [&] { wchunk<8, 8, true, true><<<nb8 * K, 512>>>(P, K, nb8); });
  return 0;
}
