// Cost of the harmonic sum's record emission pattern (harmsum.hip
// emit_levels): every wave with crossings reserves its chunk (descriptor +
// crossings) with one device-scope atomicAdd on a single counter, then its
// lanes write 12-byte records.  Variants: 0 = one counter (as now), 1 = one
// counters per block class (blockIdx % R, separate 128-byte lines, R = 8 /
// 64 / 256), 2 = no atomic (positions from the wave id: the write cost alone).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/atomic_bench tools/expt/atomic_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

struct Rec {
  uint32_t a;
  int32_t b;
  float c;
};

template <int MODE>
__global__ void __launch_bounds__(256) emit(Rec* out, uint32_t* ctr, int chunks_per_wave, int per_chunk,
                                            uint32_t cap, uint32_t R) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t* c = MODE == 1 ? ctr + (blockIdx.x & (R - 1)) * 32u : ctr;
  for (int j = 0; j < chunks_per_wave; ++j) {
    const uint32_t tot = static_cast<uint32_t>(per_chunk) + 1u;
    uint32_t base = 0;
    if constexpr (MODE == 2) {
      base = (wave * chunks_per_wave + j) * tot;
    } else {
      if (lane == 0) base = atomicAdd(c, tot);
      base = __shfl(base, 0, 64);
      if (MODE == 1) base = (blockIdx.x & (R - 1)) * (cap / R) + base;
    }
    if (lane < per_chunk + 1) {
      const uint32_t pos = base + lane;
      if (pos < cap) out[pos] = Rec{pos, lane, 1.0f};
    }
  }
}

int main(int argc, char** argv) {
  const int nchunks = argc > 1 ? atoi(argv[1]) : 776742;  // one peak-heavy batch (cluster_replay)
  const int per = argc > 2 ? atoi(argv[2]) : 25;
  const int cpw = argc > 3 ? atoi(argv[3]) : 1;
  const int waves = (nchunks + cpw - 1) / cpw;
  const int blocks = (waves + 3) / 4;
  const uint32_t cap = static_cast<uint32_t>(static_cast<uint64_t>(blocks) * 4 * cpw * (per + 1) + 64);
  Rec* out;
  uint32_t* ctr;
  if (hipMalloc(&out, sizeof(Rec) * static_cast<size_t>(cap)) != hipSuccess) return 1;
  if (hipMalloc(&ctr, 256 * 32 * sizeof(uint32_t)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int modes[5] = {0, 1, 1, 1, 2};
  const uint32_t regs[5] = {1, 8, 64, 256, 1};
  for (int v = 0; v < 5; ++v) {
    const int mode = modes[v];
    const uint32_t R = regs[v];
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      (void)hipMemset(ctr, 0, 256 * 32 * sizeof(uint32_t));
      (void)hipEventRecord(e0);
      if (mode == 0) emit<0><<<blocks, 256>>>(out, ctr, cpw, per, cap, R);
      if (mode == 1) emit<1><<<blocks, 256>>>(out, ctr, cpw, per, cap, R);
      if (mode == 2) emit<2><<<blocks, 256>>>(out, ctr, cpw, per, cap, R);
      if (hipGetLastError() != hipSuccess) return 3;
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r > 0 && ms < best) best = ms;
    }
    printf("mode %d (%s, R %u): chunks %d x %d records, %d per wave: %.3f ms\n", mode,
           mode == 0 ? "one counter" : mode == 1 ? "R counters" : "no atomic", R, nchunks, per + 1, cpw, best);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  (void)hipFree(out);
  (void)hipFree(ctr);
  return 0;
}
