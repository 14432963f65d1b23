// Fused four-step FFT for the acceleration search (gfx950 / CDNA4).
//
// The acceleration trials need, per trial k, the spectrum of the resampled
// whitened series x_k[p] = in[idx_k(p)] (resampleII, kernels.cu:338-379) --
// an N-point real FFT, done as the M = N/2 point complex FFT of
// z[m] = x[2m] + i x[2m+1] (real-FFT post-processing fused into the interbin
// kernel, harmsum.hip).  The reference runs resample -> cuFFT R2C as separate
// passes per trial (pipeline_multi.cu:203-214); rocFFT needs five passes over
// HBM for M = 2^22.  Here the whole chain is two passes, M = N1 x N2:
//
//   pass A (columns, length N2): resample straight from the L2/Infinity-Cache
//     resident input, DFT over the strided index j of z[N1 j + i], multiply
//     by W_M^{i k2}, write Y[k2][i];
//   pass B (rows, length N1): DFT over i of row k2, write X[k2 + N2 k1]
//     in natural order.
//
// A workgroup transforms 8 adjacent columns (pass A) or rows (pass B), so
// every global row segment it touches is 64 bytes (8 complex values); it runs
// as two halves of L/8 threads, each half owning 4 of the 8 transforms and
// each thread 8 points of each of its 4 transforms (32 complex values in
// VGPRs).  The two halves write the two 32-byte halves of every 64-byte
// segment at the same time, so L2 merges them into whole lines.  Transforms
// are Stockham radix-8 (+ a final radix-4/2 stage) with LDS exchanges between
// stages; LDS stays at 72 KiB per workgroup so two workgroups (16 waves)
// share a CU.  Twiddles come from small host-built tables (double precision).
// Block ids are remapped so that each XCD (blockIdx % 8 under round-robin
// dispatch) works on a contiguous range of (column block, trial) pairs: the
// trials of one column block, whose resampled reads overlap, share one L2.
#include "device_common.hpp"
#include "dft_reg.hpp"
#include "psoup/kernels.hpp"

#include <cmath>

namespace psoup {
namespace kern {

namespace {

constexpr int kPts = 8;     // points per thread per transform
constexpr int kSplit = 11;  // W_M^a = hi[a >> kSplit] * lo[a & (2^kSplit - 1)]
constexpr int kLdsBudget = 74752;  // bytes per workgroup: two workgroups per CU
// Channel planes in the exchange buffer are kChanPad complex elements apart
// beyond the padded length: with a plane stride that is a multiple of 64
// elements the compiler pairs two channels' accesses into ds_read2st64_b64 /
// ds_write2st64_b64, which run at half the LDS rate of two ds_read_b64.
constexpr int kChanPad = 8;

// CPT = transforms per thread, SUB = thread groups per workgroup; the
// workgroup covers CH = CPT*SUB adjacent columns/rows (8: 64-byte row
// segments, two workgroups per CU; 16: 128-byte segments, one per CU).
template <int L, int CPT, int SUB>
struct Cfg {
  static constexpr int CH = CPT * SUB;  // transforms per workgroup (blocked layout width when SUB == 1)
  static_assert(CH == 8 || (SUB == 1 && CPT == 10), "workgroups cover 8 transforms (10: the fused spectrum pass)");
  static constexpr int T = L / kPts;                     // threads per group
  static constexpr int THREADS = T * SUB;
  static constexpr int PAD = L + L / 8 + kChanPad;       // complex elements per channel plane
  // Workgroups of fewer than 256 threads (L < 2048) get a proportional
  // share: at L = 1024 the full 73 KiB let the 128-thread workgroup exchange
  // all 8 channels in one round but held the CU to 2 workgroups (1 wave per SIMD)
  static constexpr int BUDGET = THREADS >= 256 ? kLdsBudget : kLdsBudget / 256 * THREADS;
  static constexpr int CG0 = BUDGET / (SUB * 2 * PAD * 4);
  static constexpr int CG = CG0 >= CPT ? CPT : (CG0 >= 4 ? 4 : (CG0 >= 2 ? 2 : 1));  // channels per exchange round
  static constexpr int GROUP_FLOATS = 2 * CG * PAD;
  static constexpr int LDS_FLOATS = SUB * GROUP_FLOATS;
};

template <int CPT>
using Vec = float2[CPT][kPts];
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-byte load
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int lds_pad(int x) { return x + (x >> 3); }
using namespace dreg;  // butterflies, packed complex arithmetic, dft<N> (dft_reg.hpp)

// One Stockham iteration's arithmetic (Govindaraju et al. formulation): for
// virtual thread j' = t + b*T, points v[b + r*B] = data[j' + r*L/R] are
// twiddled by W_{Ns R}^{r (j' mod Ns)} and transformed in place.
// Where the Stockham stages read W_L^m.  Global: the length-L table.  LDS
// (TwLds): the entries the stages of a length-L transform use -- every m <
// D, and multiples of S in [D, L/2) -- staged once per workgroup, so no
// stage waits on a global round trip after its exchange.
struct TwGlobal {
  const float2* __restrict__ p;
  __device__ __forceinline__ float2 operator()(int m) const { return p[m]; }
};
template <int L>
struct TwLds {
  static constexpr int D = L <= 1024 ? L / 2 : 512;
  static constexpr int S = L <= 1024 ? 1 : (L == 2048 ? 16 : 4);
  static constexpr int N = D + (L / 2 - D) / S;  // staged entries
  __host__ __device__ static constexpr int slot(int m) { return m < D ? m : D + (m - D) / S; }
  __host__ __device__ static constexpr int index(int e) { return e < D ? e : D + (e - D) * S; }
  // every twiddle index stage_compute reads for this L is staged
  static constexpr bool covers() {
    for (int ns = 1; ns < L; ns *= 8) {
      const int r = L / ns >= 8 ? 8 : L / ns;
      if (ns == 1) continue;
      const int scale = L / (ns * r);
      for (int jm = 0; jm < ns; ++jm) {
        const int a = jm * scale, b = 4 * jm * scale;
        if (a >= L / 2 || (a >= D && (a - D) % S != 0)) return false;
        if (r == 8 && (b >= L / 2 || (b >= D && (b - D) % S != 0))) return false;
      }
    }
    return true;
  }
  const float2* __restrict__ p;
  __device__ __forceinline__ float2 operator()(int m) const { return p[slot(m)]; }
};

template <int L, int CPT, int Ns, int R, class TW>
__device__ __forceinline__ void stage_compute(Vec<CPT>& v, int t, const TW& twL) {
  constexpr int T = L / kPts, B = kPts / R;
#pragma unroll
  for (int b = 0; b < B; ++b) {
    if constexpr (Ns > 1) {
      const int jm = (t + b * T) & (Ns - 1);
      constexpr int scale = L / (Ns * R);
      // W^{r jm scale}, r < R: two table reads (w1, w4) and short products
      // (at most two multiplications deep) instead of R-1 table reads
      float2 w[R];
      w[1] = twL(jm * scale);
      if constexpr (R >= 4) {
        w[2] = cmul(w[1], w[1]);
        w[3] = cmul(w[2], w[1]);
      }
      if constexpr (R == 8) {
        w[4] = twL(4 * jm * scale);
        w[5] = cmul(w[4], w[1]);
        w[6] = cmul(w[4], w[2]);
        w[7] = cmul(w[4], w[3]);
      }
#pragma unroll
      for (int r = 1; r < R; ++r) {
#pragma unroll
        for (int c = 0; c < CPT; ++c) v[c][b + r * B] = cmul(v[c][b + r * B], w[r]);
      }
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      if constexpr (R == 8)
        fft8(v[c][b], v[c][b + B], v[c][b + 2 * B], v[c][b + 3 * B], v[c][b + 4 * B], v[c][b + 5 * B],
             v[c][b + 6 * B], v[c][b + 7 * B]);
      else if constexpr (R == 4)
        fft4(v[c][b], v[c][b + B], v[c][b + 2 * B], v[c][b + 3 * B]);
      else
        fft2(v[c][b], v[c][b + B]);
    }
  }
}

// Scatter to the Stockham destination (j'/Ns)*Ns*R + j' mod Ns + r*Ns, then
// gather back in the uniform pattern t + q*T.
template <int L, int CPT, int CG, int Ns, int R>
__device__ __forceinline__ void exchange(Vec<CPT>& v, float* __restrict__ lds, int t) {
  constexpr int T = L / kPts, B = kPts / R, PAD = L + L / 8 + kChanPad;  // plane stride, complex elements
  float2* buf = reinterpret_cast<float2*>(lds);                   // 8-byte ds_write_b64 / ds_read_b64
#pragma unroll
  for (int g = 0; g < CPT; g += CG) {
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int j = t + b * T;
      const int base = (j / Ns) * Ns * R + (j & (Ns - 1));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int idx = lds_pad(base + r * Ns);
#pragma unroll
        for (int cc = 0; cc < CG; ++cc)
          if (g + cc < CPT) buf[cc * PAD + idx] = v[g + cc][b + r * B];  // (the last round may be short)
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const int idx = lds_pad(t + q * T);
#pragma unroll
      for (int cc = 0; cc < CG; ++cc)
        if (g + cc < CPT) v[g + cc][q] = buf[cc * PAD + idx];
    }
    __syncthreads();
  }
}

// Full forward DFT of length L on the thread's CPT channels (lds = its group's
// region); input and output both in the pattern v[c][q] <-> element t + q*T.
// Phase timestamps (tools/expt/fft4_trace.py): when g_fft4_trace is set,
// thread 0 of each workgroup records the shader clock at fixed points of the
// kernel (start, loads issued, after every FFT stage and exchange, end).
// (__constant__: read with a scalar load, so a trace point costs an lgkmcnt
// wait, not a vmcnt(0) that would drain every global load in flight)
__constant__ unsigned long long* g_fft4_trace = nullptr;
constexpr int kTraceEvents = 12;
__device__ __forceinline__ void trace_event(int ev) {
  unsigned long long* tr = g_fft4_trace;
  if (tr != nullptr && threadIdx.x == 0) tr[blockIdx.x * kTraceEvents + ev] = __builtin_readcyclecounter();
}

template <int L, int CPT, int CG, int Ns, class TW>
__device__ __forceinline__ void fft_stages(Vec<CPT>& v, float* __restrict__ lds, int t, const TW& twL, int ev = 2) {
  constexpr int R = (L / Ns >= 8) ? 8 : L / Ns;
  stage_compute<L, CPT, Ns, R>(v, t, twL);
  trace_event(ev);
  if constexpr (Ns * R < L) {
    exchange<L, CPT, CG, Ns, R>(v, lds, t);
    trace_event(ev + 1);
    fft_stages<L, CPT, CG, Ns * R>(v, lds, t, twL, ev + 2);
  }
}
template <int L, int CPT, int CG, int Ns>
__device__ __forceinline__ void fft_stages(Vec<CPT>& v, float* __restrict__ lds, int t,
                                           const float2* __restrict__ twL, int ev = 2) {
  fft_stages<L, CPT, CG, Ns>(v, lds, t, TwGlobal{twL}, ev);
}

// S consecutive resampled samples x[p0 .. p0+S-1] (resampleII indices,
// kernels.cu:338-379).  The read index is evaluated exactly, in double, at
// both ends of the span.  The shift idx(p) - p is monotone on a span away
// from the parabola's vertex n/2 and changes by at most one there (|af| n < 1e-3
// for physical accelerations), so with both ends rounding by a margin:
//   * equal end shifts: every sample has that shift and the S values are one
//     contiguous load of the padded input (S = 16: four 16-byte loads);
//   * end shifts one apart: a binary search over the span (log2 S exact
//     evaluations) finds the first sample with the new shift, and the values
//     come from one S+4-float window with a per-element select;
// anything else (spans near the vertex or the series edges, end values within
// 1e-7 of a rounding tie) is gathered per element.  All index math is 32-bit
// (series < 2^31 samples; checked on the host).
constexpr double kVertexGuard = 8192.0;  // spans this close to n/2 take the per-element path

template <int S>  // S = samples per span, a multiple of 4
__device__ __forceinline__ void load_resampled(const float* __restrict__ in, const float* __restrict__ in_pad,
                                               uint32_t n, int log2row, uint32_t inpitch, double af, double size,
                                               uint32_t p0, float (&x)[S]) {
  const double d0 = static_cast<double>(p0), d1 = d0 + static_cast<double>(S - 1);
  const double r0 = dev::accel_pos_ii(af, size, d0), r1 = dev::accel_pos_ii(af, size, d1);
  const double q0 = rint(r0), q1 = rint(r1);
  const bool ok = (0.5 - fabs(r0 - q0) > 1e-7) && (0.5 - fabs(r1 - q1) > 1e-7) && q0 >= 1.0 &&
                  q1 <= static_cast<double>(n - 1) && fabs(0.5 * (d0 + d1) - 0.5 * size) > kVertexGuard;
  const double ds = (q1 - q0) - static_cast<double>(S - 1);  // change of the shift over the span
  const uint32_t rowmask = (1u << log2row) - 1u;
  auto addr = [&](uint32_t i) { return (i >> log2row) * inpitch + (i & rowmask); };
  if (ok && ds == 0.0) {
    const f4u* src = reinterpret_cast<const f4u*>(in_pad + addr(static_cast<uint32_t>(q0)));
#pragma unroll
    for (int u = 0; u < S / 4; ++u) {
      const f4u w = src[u];
      x[4 * u] = w.x;
      x[4 * u + 1] = w.y;
      x[4 * u + 2] = w.z;
      x[4 * u + 3] = w.w;
    }
  } else if (ok && fabs(ds) == 1.0) {
    // samples e < hi keep the first shift s0, samples e >= hi have s0 + ds
    const double s0 = q0 - d0;
    int lo = 0, hi = S - 1;
#pragma unroll
    for (int it = 0; (1 << it) < S - 1; ++it) {
      const int mid = (lo + hi) >> 1;
      const double dm = d0 + static_cast<double>(mid);
      const bool same = rint(dev::accel_pos_ii(af, size, dm)) - dm == s0;
      lo = same ? mid : lo;
      hi = same ? hi : mid;
    }
    // window w[v] = x_in[q0 - 1 + v], v < S + 4 (the padded row holds the next row's head)
    float w[S + 4];
    const f4u* src = reinterpret_cast<const f4u*>(in_pad + addr(static_cast<uint32_t>(q0) - 1u));
#pragma unroll
    for (int u = 0; u < S / 4 + 1; ++u) {
      const f4u v = src[u];
      w[4 * u] = v.x;
      w[4 * u + 1] = v.y;
      w[4 * u + 2] = v.z;
      w[4 * u + 3] = v.w;
    }
    const bool up = ds > 0.0;
#pragma unroll
    for (int e = 0; e < S; ++e) x[e] = e < hi ? w[e + 1] : (up ? w[e + 2] : w[e]);
  } else {
#pragma unroll
    // (from the padded copy: the engine may whiten straight into it and
    // leave the unpadded series unwritten, fft4_c2r_post_pad)
    for (int i = 0; i < S; ++i) x[i] = in_pad[addr(dev::accel_index_ii32(af, size, p0 + static_cast<uint32_t>(i), n - 1))];
  }
}

// Table layout (float2): [tw_N2 (N2)] [tw_N1 (N1)] [lo (2^kSplit)] [hi (M >> kSplit)]
// [ox (N1 x GX)]: ox[col * GX + k2] = W_M^{col P k2}, the k2 part of the
// one-exchange pass A's four-step twiddles (GX = onex_g(N2), P = N2 / GX);
// [hk (N1)] [hr (N2/2 + 1)]: e^{-i pi k1 / N1} and e^{-i pi r / M}, the two
// factors of the real-FFT post-processing twiddle e^{-i pi (r + N2 k1) / M}
// (fused spectrum pass).
struct TableOffsets {
  uint64_t n2, n1, lo, hi, ox, hk, hr, total;
};
__host__ __device__ constexpr int onex_g(int N2) { return N2 >= 2048 ? 64 : 32; }
__host__ __device__ inline TableOffsets table_offsets(int N1, int N2) {
  const uint64_t M = static_cast<uint64_t>(N1) * N2;
  TableOffsets o;
  o.n2 = 0;
  o.n1 = o.n2 + N2;
  o.lo = o.n1 + N1;
  o.hi = o.lo + (1u << kSplit);
  o.ox = o.hi + (M >> kSplit);
  o.hk = o.ox + static_cast<uint64_t>(N1) * onex_g(N2);
  o.hr = o.hk + N1;
  o.total = o.hr + N2 / 2 + 1;
  return o;
}

__device__ __forceinline__ float2 twiddle_M(uint32_t a, const float2* __restrict__ lo, const float2* __restrict__ hi) {
  return cmul(hi[a >> kSplit], lo[a & ((1u << kSplit) - 1)]);
}

template <int CPT>
__device__ __forceinline__ void store_row(float2* __restrict__ dst, const Vec<CPT>& v, int q) {
  f4v* d = reinterpret_cast<f4v*>(dst);
#pragma unroll
  for (int c = 0; c < CPT; c += 2) d[c / 2] = f4v{v[c][q].x, v[c][q].y, v[c + 1][q].x, v[c + 1][q].y};
}

// 4 x 4 transpose of 16-byte pieces within each lane quad: afterwards lane
// j holds at [r] what lane r of its quad held at [j].  Two exchange stages
// (partners j ^ 1, then j ^ 2) with DPP quad permutes, no LDS.
template <int CTRL>
__device__ __forceinline__ f4v dpp4(const f4v& x) {
  return f4v{__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x.x), CTRL, 0xF, 0xF, false)),
             __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x.y), CTRL, 0xF, 0xF, false)),
             __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x.z), CTRL, 0xF, 0xF, false)),
             __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x.w), CTRL, 0xF, 0xF, false))};
}
__device__ __forceinline__ void quad_transpose(f4v (&a)[4], int j) {
  // stage 1 (bit 0 of row and piece): keep a[i] where i & 1 == j & 1, else the partner's a[i ^ 1]
  {
    const f4v p0 = dpp4<0xB1>(a[1]), p1 = dpp4<0xB1>(a[0]), p2 = dpp4<0xB1>(a[3]), p3 = dpp4<0xB1>(a[2]);
    const bool odd = j & 1;
    a[0] = odd ? p0 : a[0];
    a[1] = odd ? a[1] : p1;
    a[2] = odd ? p2 : a[2];
    a[3] = odd ? a[3] : p3;
  }
  // stage 2 (bit 1): keep a[i] where i & 2 == j & 2, else the partner's a[i ^ 2]
  {
    const f4v p0 = dpp4<0x4E>(a[2]), p1 = dpp4<0x4E>(a[3]), p2 = dpp4<0x4E>(a[0]), p3 = dpp4<0x4E>(a[1]);
    const bool hi = j & 2;
    a[0] = hi ? p0 : a[0];
    a[1] = hi ? p1 : a[1];
    a[2] = hi ? a[2] : p2;
    a[3] = hi ? a[3] : p3;
  }
}

// XCD-aware block order (remap = true): logical block
// b' = (b % 8) * (nblocks / 8) + b / 8, so each XCD's share of the grid is one
// contiguous logical range (nblocks is a multiple of 8).
__device__ __forceinline__ uint32_t logical_block(uint32_t nblocks, bool remap) {
  const uint32_t b = blockIdx.x;
  return remap ? (b & 7u) * (nblocks >> 3) + (b >> 3) : b;
}

// Input copy with rows of 2*N1 floats at a pitch of 2*N1 + 32 (the pad holds
// the next row's head, so a span starting in a row is contiguous).  Pass A's
// lanes read rows 2*N1 floats apart; the odd pitch spreads them over memory
// channels instead of one.
__global__ void __launch_bounds__(256) fft4_pad_input_kernel(const float* __restrict__ in, uint64_t n,
                                                             float* __restrict__ out, uint64_t rowlen,
                                                             uint64_t pitch, uint64_t total, uint64_t in_stride,
                                                             uint64_t out_stride) {
  in += blockIdx.y * in_stride;
  out += blockIdx.y * out_stride;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t u = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; u < total; u += stride) {
    const uint64_t row = u / pitch, r = u - row * pitch;
    const uint64_t src = row * rowlen + r;
    out[u] = src < n ? in[src] : 0.f;
  }
}

// The same copy in 16-byte vectors with 32-bit indices (rowlen, pitch, n and
// the strides multiples of 4 floats, 16-byte aligned pointers): a vector never
// straddles a row or the series end.
__global__ void __launch_bounds__(256) fft4_pad_input_vec_kernel(const float4* __restrict__ in, uint32_t n4,
                                                                 float4* __restrict__ out, uint32_t rowlen4,
                                                                 uint32_t pitch4, uint32_t total4, uint64_t in_stride4,
                                                                 uint64_t out_stride4) {
  in += blockIdx.y * in_stride4;
  out += blockIdx.y * out_stride4;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < total4; u += stride) {
    const uint32_t row = u / pitch4, r = u - row * pitch4;
    const uint32_t src = row * rowlen4 + r;
    out[u] = src < n4 ? in[src] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Strip layout of the padded input (kFft4StripInput, one-exchange pass A):
// strip b holds floats [16 b, 16 b + kStripW) of every row (rows of 2*N1
// floats; the last strip's tail is the next row's head), rows of a strip
// contiguous: element (row j, strip b, e) at (b * N2 + j) * kStripW + e.  A
// lane's four resampled samples start at offset (col & 15) <= 15 of the
// strip its first sample falls in, so kStripW = 20 always covers them, and a
// wave's 16 consecutive rows (at most two strips) are one or two contiguous
// ~1.3 KiB ranges.  1.25 x the series in floats.
constexpr int kStripW = 20;
__host__ __device__ constexpr uint64_t strip_floats(int n1, int n2) {
  return static_cast<uint64_t>(n1 / 8) * static_cast<uint64_t>(n2) * kStripW;
}
// (at column lengths 512 and 1024 the Stockham pass A measured faster: bench
// at 2^22 40.4k vs 37.3k trials/s, at 2^21 55.5k vs 53.4k)
__host__ __device__ inline bool onex_colpass(int n2, int f) {
  return (f & kFft4OneX) && (f & kFft4Blocked) && (f & kFft4TileY) && n2 == 2048;
}
__host__ __device__ inline bool strip_input(int n2, int f) { return (f & kFft4StripInput) && onex_colpass(n2, f); }
// the padded input of g is in strips: the one-exchange pass A reads them
// (always for the whitener's zero-shift transforms)
inline bool strip_layout(const Fft4Geom& g, int f) {
  return strip_input(g.n2, f) || (g.zero_shift && onex_colpass(g.n2, f));
}
// pass A writes row-pair Y for the fused spectrum pass: the one-exchange
// kernel always can, the tiled-Y Stockham kernel with kFft4PairY
__host__ __device__ inline bool pair_y_layout(int n2, int f) {
  return onex_colpass(n2, f) || ((f & kFft4PairY) && (f & kFft4Blocked) && (f & kFft4TileY));
}

// Strip-layout copies, one thread per strip row (b, j): out[(b N2 + j) 20 +
// e] = x[j rowlen + 16 b + e], e < 20, where x is the series (float, or
// 8-bit with the row mean past nvalid) and zero past n.  Consecutive lanes
// take consecutive rows of a strip, so a wave's stores are one contiguous
// 5 KiB range; its loads hit 64 rows at once and the other strips of those
// rows (the neighbouring waves) read the same lines out of L2.  The source
// span of a strip row starts at a multiple of 16 elements: with an aligned
// row base it is a 16-byte vector load sequence.
__device__ __forceinline__ void store_strip_row(float* __restrict__ o, const float (&x)[kStripW]) {
  f4v* d = reinterpret_cast<f4v*>(o);
#pragma unroll
  for (int u = 0; u < kStripW / 4; ++u) d[u] = f4v{x[4 * u], x[4 * u + 1], x[4 * u + 2], x[4 * u + 3]};
}

// 8-bit rows -> strips through LDS: a workgroup stages R consecutive rows
// (coalesced 16-byte loads; row pitch rowlen + 16 bytes, so the strip-row
// reads below spread over the banks) plus the head of the next row (the last
// strip's 4-float tail), then writes R rows of every strip: per strip one
// contiguous 80 R-byte range.  Samples past nvalid are the row mean, past n
// zero (as u8_to_f32_pad + fft4_pad_input).
constexpr int kStripLdsBytes = 32768;
__global__ void __launch_bounds__(256) fft4_strips_u8_kernel(const uint8_t* __restrict__ in, uint64_t nvalid, uint64_t n,
                                                             const unsigned long long* __restrict__ sum,
                                                             float* __restrict__ out, uint32_t rowlen, uint32_t nrows,
                                                             int log2_r, uint64_t in_stride, uint64_t out_stride) {
  __shared__ __attribute__((aligned(16))) uint8_t st[kStripLdsBytes + 16 * 17 + 16];
  in += blockIdx.y * in_stride;
  out += blockIdx.y * out_stride;
  const uint32_t R = 1u << log2_r, pitch = rowlen + 16, j0 = blockIdx.x * R;
  const float mean = nvalid ? static_cast<float>(static_cast<double>(sum[blockIdx.y]) / static_cast<double>(nvalid))
                            : 0.f;
  // stage rows j0 .. j0 + R - 1 whole and the first 16 bytes of row j0 + R
  const uint32_t c16 = rowlen >> 4, nchunks = R * c16 + 1;
  for (uint32_t i = threadIdx.x; i < nchunks; i += blockDim.x) {
    const uint32_t r = i / c16, c = i - r * c16;
    const uint64_t s0 = static_cast<uint64_t>(j0 + r) * rowlen + 16u * c;
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (s0 + 16 <= nvalid) {
      w = *reinterpret_cast<const uint4*>(in + s0);
    } else if (s0 < nvalid) {
      uint32_t wd[4] = {0u, 0u, 0u, 0u};
      for (uint32_t e = 0; e < 16 && s0 + e < nvalid; ++e) wd[e >> 2] |= static_cast<uint32_t>(in[s0 + e]) << (8 * (e & 3));
      w = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    }
    *reinterpret_cast<uint4*>(st + r * pitch + 16u * c) = w;
  }
  __syncthreads();
  const uint32_t nstrips = rowlen >> 4, total = nstrips << log2_r;
  for (uint32_t u = threadIdx.x; u < total; u += blockDim.x) {
    const uint32_t b = u >> log2_r, jj = u & (R - 1u);
    const uint4 w = *reinterpret_cast<const uint4*>(st + jj * pitch + 16u * b);
    const uint32_t tail = 16u * b + 16u < rowlen ? *reinterpret_cast<const uint32_t*>(st + jj * pitch + 16u * b + 16u)
                                                 : *reinterpret_cast<const uint32_t*>(st + (jj + 1u) * pitch);
    const uint32_t wd[5] = {w.x, w.y, w.z, w.w, tail};
    const uint64_t s0 = static_cast<uint64_t>(j0 + jj) * rowlen + 16u * b;
    float x[kStripW];
    if (s0 + kStripW <= nvalid) {
#pragma unroll
      for (int e = 0; e < kStripW; ++e) x[e] = static_cast<float>((wd[e >> 2] >> (8 * (e & 3))) & 255u);
    } else {
#pragma unroll
      for (int e = 0; e < kStripW; ++e)
        x[e] = s0 + e < nvalid ? static_cast<float>((wd[e >> 2] >> (8 * (e & 3))) & 255u) : (s0 + e < n ? mean : 0.f);
    }
    store_strip_row(out + (static_cast<uint64_t>(b) * nrows + j0 + jj) * kStripW, x);
  }
}

__global__ void __launch_bounds__(256) fft4_pad_strips_kernel(const float* __restrict__ in, uint64_t n,
                                                              float* __restrict__ out, uint32_t rowlen,
                                                              int log2_nrows, uint32_t nstriprows, uint64_t in_stride,
                                                              uint64_t out_stride, bool aligned) {
  in += blockIdx.y * in_stride;
  out += blockIdx.y * out_stride;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < nstriprows; u += stride) {
    const uint32_t b = u >> log2_nrows, j = u & ((1u << log2_nrows) - 1u);
    const uint64_t s0 = static_cast<uint64_t>(j) * rowlen + 16u * b;
    float x[kStripW];
    if (aligned && s0 + kStripW <= n) {
      const f4v* src = reinterpret_cast<const f4v*>(in + s0);
#pragma unroll
      for (int u4 = 0; u4 < kStripW / 4; ++u4) {
        const f4v w = src[u4];
        x[4 * u4] = w.x;
        x[4 * u4 + 1] = w.y;
        x[4 * u4 + 2] = w.z;
        x[4 * u4 + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < kStripW; ++e) x[e] = s0 + e < n ? in[s0 + e] : 0.f;
    }
    store_strip_row(out + static_cast<uint64_t>(u) * kStripW, x);
  }
}

// Kernel variants: MODE bit 0 = blocked Y/X layouts (CPT 8);
// bit 2 = tiled Y (pass A -> pass B): Y_t[i/8][k2/8][i%8][k2%8], so a pass-B
// lane reads its rows' values as contiguous 16-byte vectors and eight lanes
// cover 512 contiguous bytes.
// bit 3 = tiled X: X_t[k2/8][k1/8][k2%8][k1%8] (read by r2c_interbin_normalise_tiled).
// bit 4 = row-pair Y (pass A -> fused spectrum pass): Y_p[k2/2][i][k2%2].
constexpr int kModeBlocked = 1, kModeTileY = 4, kModeTileX = 8, kModePairY = 16;

// Pass A input sources: the padded series, resampled per trial (in_pad), or
// for the whitener's plain FFTs (Fft4Geom::u8 / c2r) the 8-bit rows or the
// half spectra themselves.  Separate instantiations, so the search's kernel
// keeps its registers.
constexpr int kSrcPad = 0, kSrcU8 = 1, kSrcC2R = 2, kSrcF32 = 3, kSrcStrips = 4;

// Pass A.  Logical block = column block * K + trial (trial fastest).
template <int L, int CPT, int SUB, int MODE, int SRC = kSrcPad>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, Cfg<L, CPT, SUB>::THREADS), amdgpu_waves_per_eu(2))) fft4_colpass_kernel(
    const float* __restrict__ in, const float* __restrict__ in_pad, uint64_t n, const double* __restrict__ afs, int K,
    float2* __restrict__ Y, Fft4Geom g, const float2* __restrict__ tab, int flags) {
  using C = Cfg<L, CPT, SUB>;
  constexpr bool kBlocked = MODE & kModeBlocked, kTileY = MODE & kModeTileY, kPairY = MODE & kModePairY;
  static_assert(!kTileY || (CPT == 8 && SUB == 1), "tiled Y: 8 transforms per thread");
  static_assert(!kPairY || kTileY, "row-pair Y: the tiled-Y kernel shape");
  __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];
  constexpr int T = C::T;
  const int grp = threadIdx.x / T;
  const int t = threadIdx.x - grp * T;
  const uint32_t lb = logical_block(gridDim.x, !(flags & kFft4NoRemap));
  trace_event(0);
  const int N1 = g.n1;
  int k = static_cast<int>(lb % static_cast<uint32_t>(K));
  int c0 = static_cast<int>(lb / static_cast<uint32_t>(K)) * C::CH + grp * CPT;
  if ((flags & kFft4GroupXcd) && (K & 7) == 0) {
    // 8 consecutive trials x column blocks 2p, 2p+1 (16 workgroups reading
    // nearly the same input lines) share one XCD, in consecutive slots
    const uint32_t b = blockIdx.x;
    const uint32_t G = ((b >> 7) << 3) | (b & 7u), w = (b >> 3) & 15u;
    const uint32_t kg = static_cast<uint32_t>(K) >> 3;
    k = static_cast<int>(8 * (G % kg) + (w & 7u));
    c0 = static_cast<int>(2 * (G / kg) + (w >> 3)) * C::CH + grp * CPT;
  } else if (flags & kFft4PairXcd) {
    // column blocks 2p and 2p+1 of a trial (the two 64-byte halves of every
    // input line) run on the same XCD, 8 dispatch slots apart
    const uint32_t b = blockIdx.x;
    const uint32_t s = (b >> 3) & 1u, u = ((b >> 4) << 3) | (b & 7u);
    k = static_cast<int>(u % static_cast<uint32_t>(K));
    c0 = static_cast<int>(2 * (u / static_cast<uint32_t>(K)) + s) * C::CH + grp * CPT;
  }
  const int log2row = __builtin_ctz(static_cast<unsigned>(2 * N1));
  const TableOffsets to = table_offsets(N1, L);
  const double af = afs[k];
  const uint64_t src = __builtin_amdgcn_readfirstlane(  // series this trial resamples (workgroup-uniform)
      static_cast<uint32_t>(g.tsrc ? g.tsrc[k] : static_cast<uint64_t>(k)));
  const double size = static_cast<double>(n);
  Vec<CPT> v;
  if constexpr (SRC == kSrcU8) {
    // the whitener's forward input straight from the 8-bit row: row j's
    // columns c0 .. c0+CPT-1 are 2 CPT consecutive bytes (one 16-byte load)
    static_assert(CPT == 8 || CPT == 4, "8-bit rows: 16- or 8-byte loads");
    const uint8_t* row = g.u8 + src * g.src_stride;
    const uint64_t nvalid = g.u8_nvalid;
    const float mean = nvalid ? static_cast<float>(static_cast<double>(g.u8sum[src]) / static_cast<double>(nvalid))
                              : 0.f;
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const uint64_t s0 = 2 * (static_cast<uint64_t>(N1) * (t + q * T) + c0);
      float x[2 * CPT];
      if (s0 + 2 * CPT <= nvalid) {
        uint32_t wd[CPT / 2];
        if constexpr (CPT == 8) {
          const uint4 w = *reinterpret_cast<const uint4*>(row + s0);
          wd[0] = w.x, wd[1] = w.y, wd[2] = w.z, wd[3] = w.w;
        } else {
          const uint2 w = *reinterpret_cast<const uint2*>(row + s0);
          wd[0] = w.x, wd[1] = w.y;
        }
#pragma unroll
        for (int e = 0; e < 2 * CPT; ++e) x[e] = static_cast<float>((wd[e >> 2] >> (8 * (e & 3))) & 255u);
      } else {
#pragma unroll
        for (int e = 0; e < 2 * CPT; ++e) x[e] = s0 + e < nvalid ? static_cast<float>(row[s0 + e]) : (s0 + e < n ? mean : 0.f);
      }
#pragma unroll
      for (int c = 0; c < CPT; ++c) v[c][q] = make_float2(x[2 * c], x[2 * c + 1]);
    }
  } else if constexpr (SRC == kSrcStrips) {
    // the padded input in column strips (fft4_pad_input_u8): row j's columns
    // c0 .. c0+CPT-1 are 2 CPT consecutive floats of strip 2 c0 / 16, and a
    // wave's consecutive rows are consecutive 80-byte strip rows
    static_assert((2 * CPT) % 4 == 0 && 2 * CPT <= 16, "strip reads");
    const float* sp = in_pad + src * g.pad_tstride + (static_cast<uint64_t>((2 * c0) >> 4) * L) * kStripW + ((2 * c0) & 15);
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const f4u* p4 = reinterpret_cast<const f4u*>(sp + static_cast<uint64_t>(t + q * T) * kStripW);
#pragma unroll
      for (int u = 0; u < CPT / 2; ++u) {
        const f4u w = p4[u];
        v[2 * u][q] = make_float2(w.x, w.y);
        v[2 * u + 1][q] = make_float2(w.z, w.w);
      }
    }
  } else if constexpr (SRC == kSrcF32) {
    // plain FFT of an unpadded series: row j's columns are 2 CPT consecutive
    // floats (no resampling, so no padded copy and no window)
    const float* row = in + src * g.in_tstride;
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const f4v* p4 = reinterpret_cast<const f4v*>(row + 2 * (static_cast<uint64_t>(N1) * (t + q * T) + c0));
#pragma unroll
      for (int u = 0; u < CPT / 2; ++u) {
        const f4v w = p4[u];
        v[2 * u][q] = make_float2(w.x, w.y);
        v[2 * u + 1][q] = make_float2(w.z, w.w);
      }
    }
  } else if constexpr (SRC == kSrcC2R) {
    // the whitener's inverse input from the half spectrum: z[m] = e + i W^m d,
    // conjugated, e = X[m] + conj X[M-m], d = X[m] - conj X[M-m] (fft4_c2r_pre)
    const float2* X = g.c2r + src * g.src_stride;
    const uint32_t M = static_cast<uint32_t>(N1) * L;
    const float invM = 1.0f / static_cast<float>(M);
    // one row at a time: X[m0 .. m0+CPT) and X[M-m0-CPT+1 .. M-m0] as 16-byte
    // loads (dword-aligned: the spectra are M + 1 bins apart)
    static_assert(CPT % 2 == 0, "c2r: pairs of bins per load");
    float2 a[1][CPT], b[1][CPT];
    auto load_row = [&](int q, int) {
      const uint32_t m0 = static_cast<uint32_t>(N1) * (t + q * T) + c0;
      const f4u* pa = reinterpret_cast<const f4u*>(X + m0);
      const f4u* pb = reinterpret_cast<const f4u*>(X + (M - m0 - (CPT - 1)));
#pragma unroll
      for (int u = 0; u < CPT / 2; ++u) {
        const f4u wa = pa[u], wb = pb[u];
        a[0][2 * u] = make_float2(wa.x, wa.y);
        a[0][2 * u + 1] = make_float2(wa.z, wa.w);
        // pb[u] holds X[M-m0-(CPT-1)+2u], X[M-m0-(CPT-2)+2u]: columns CPT-1-2u, CPT-2-2u
        b[0][CPT - 1 - 2 * u] = make_float2(wb.x, wb.y);
        b[0][CPT - 2 - 2 * u] = make_float2(wb.z, wb.w);
      }
    };
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      load_row(q, 0);
      const uint32_t m0 = static_cast<uint32_t>(N1) * (t + q * T) + c0;
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const uint32_t m = m0 + c;
        const float2 av = a[0][c], bv = b[0][c];
        const float ex = av.x + bv.x, ey = av.y - bv.y;
        const float dx = av.x - bv.x, dy = av.y + bv.y;
        float sn, cs;
        sincospif(static_cast<float>(m) * invM, &sn, &cs);
        const float wx = cs * dx - sn * dy, wy = cs * dy + sn * dx;
        v[c][q] = make_float2(ex - wy, -(ey + wx));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const uint64_t j = t + q * T;
      float x[2 * CPT];
      load_resampled<2 * CPT>(in + src * g.in_tstride, in_pad + src * g.pad_tstride, static_cast<uint32_t>(n),
                              log2row, static_cast<uint32_t>(g.inpitch), af, size,
                              2u * (static_cast<uint32_t>(N1) * static_cast<uint32_t>(j) + static_cast<uint32_t>(c0)),
                              x);
#pragma unroll
      for (int c = 0; c < CPT; ++c) v[c][q] = make_float2(x[2 * c], x[2 * c + 1]);
    }
  }
  trace_event(1);
  fft_stages<L, CPT, C::CG, 1>(v, lds + grp * C::GROUP_FLOATS, t, tab + to.n2);
  const uint32_t mask = static_cast<uint32_t>(N1) * L - 1;
  float2* yk = Y + static_cast<uint64_t>(k) * g.ystride;
  // Four-step twiddles W^{(c0+c) k2}, k2 = t + qT: w0 = W^{c0 k2}, step =
  // W^{k2}.  kFft4UniformTw: both split into a per-thread factor (W^{c0 t},
  // W^t: one pair of table lookups) times a workgroup-uniform factor
  // (W^{c0 q T}, W^{q T}: computed in lanes 0..7, read back with readlane
  // into SGPRs) instead of four table lookups per q.
  const bool utw = flags & kFft4UniformTw;
  float2 bt0 = make_float2(1.f, 0.f), bts = make_float2(1.f, 0.f), u0 = bt0, us = bt0;
  if (utw) {
    bt0 = twiddle_M((static_cast<uint32_t>(c0) * static_cast<uint32_t>(t)) & mask, tab + to.lo, tab + to.hi);
    bts = twiddle_M(static_cast<uint32_t>(t), tab + to.lo, tab + to.hi);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t qT = (lane & 7u) * static_cast<uint32_t>(T);
    u0 = twiddle_M((static_cast<uint32_t>(c0) * qT) & mask, tab + to.lo, tab + to.hi);
    us = twiddle_M(qT & mask, tab + to.lo, tab + to.hi);
  }
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    const uint32_t k2 = t + q * T;
    float2 w, step;
    if (utw) {
      const float2 ua = make_float2(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(u0.x), q)),
                                    __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u0.y), q)));
      const float2 ub = make_float2(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(us.x), q)),
                                    __int_as_float(__builtin_amdgcn_readlane(__float_as_int(us.y), q)));
      w = cmul(bt0, ua);
      step = cmul(bts, ub);
    } else {
      w = twiddle_M((static_cast<uint32_t>(c0) * k2) & mask, tab + to.lo, tab + to.hi);
      step = twiddle_M(k2, tab + to.lo, tab + to.hi);
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      v[c][q] = cmul(v[c][q], w);
      w = cmul(w, step);
    }
    if constexpr (kPairY) {
      // lanes k2, k2 + 1 write 16 contiguous bytes; the 8 columns of a lane
      // fill one 128-byte line across the 8 stores (merged in L2)
      float2* dst = yk + static_cast<uint64_t>(k2 >> 1) * (2 * N1) + 2 * c0 + (k2 & 1);
#pragma unroll
      for (int c = 0; c < CPT; ++c) dst[2 * c] = v[c][q];
    } else if constexpr (kTileY) {
      float2* dst = yk + static_cast<uint64_t>(c0) * g.n2 + (k2 >> 3) * 64 + (k2 & 7);
#pragma unroll
      for (int c = 0; c < CPT; ++c) dst[c * 8] = v[c][q];
    } else if constexpr (!kBlocked && CPT == 8) {
      // natural Y[k2][i] (the external row FFT's input): the four lanes of a
      // quad hold rows k2 .. k2+3 (8 columns each); a 4 x 4 transpose of
      // their 16-byte pieces (two DPP xor exchanges) lets each store
      // instruction write 64 contiguous bytes per row through four lanes,
      // instead of 16 bytes in 64 different rows
      const int j = static_cast<int>(threadIdx.x & 3u);
      f4v a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = f4v{v[2 * u][q].x, v[2 * u][q].y, v[2 * u + 1][q].x, v[2 * u + 1][q].y};
      quad_transpose(a, j);
      const uint64_t kb = static_cast<uint64_t>(k2 - j);  // the quad's first row
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<f4v*>(yk + (kb + r) * g.ypitch + c0 + 2 * j) = a[r];
    } else {
      // blocked: Y_b[c0/8][k2][c] (each lane 64 contiguous bytes); else Y[k2][i] at pitch ypitch
      float2* dst = kBlocked ? yk + static_cast<uint64_t>(c0) * g.n2 + k2 * CPT
                             : yk + static_cast<uint64_t>(k2) * g.ypitch + c0;
      store_row<CPT>(dst, v, q);
    }
  }
  trace_event(11);
}

// ---------------------------------------------------------------------------
// One-exchange pass A (kFft4OneX).  Column length L = G * P: thread
// (cp = t & 3, g = t >> 2) owns columns c0 + 2cp and c0 + 2cp + 1 at rows
// g + G m (m < P): one 16-byte load per row, four lanes covering a row's
// 64-byte segment.  With n = G m + g and k = k1 + P k2,
//   X[k] = sum_g W_G^{g k2} [ W_L^{g k1} sum_m x[G m + g] W_P^{m k1} ],
// so each thread runs the P-point DFT over m of its two columns in registers
// (twiddles are compile-time constants), multiplies by W_L^{g k1}, and one
// LDS exchange (in g slices of at most 8192 complex) hands every thread
// (column, k1) pairs holding all G values of g, whose G-point DFTs again run
// in registers.  The Stockham kernel above needs log_8(L) - 1 exchanges (3 at
// L = 2048) and table twiddles in every stage.  Reader pairs are assigned so
// that every store instruction of a wave writes one contiguous 512-byte block
// of the tiled Y.


template <int L, int G, int R>
struct OneX {
  static constexpr int P = L / G;           // rows per thread and column: g + G m
  static constexpr int THREADS = 4 * G;     // (cp, g)
  static constexpr int NW = THREADS / 64;   // waves
  static constexpr int NPAIR = 2 * P / G;   // (column, k1) pairs per thread after the exchange
  static constexpr int ROUNDS = R;          // exchange rounds: g slices of GS values (one writer wave group each)
  static constexpr int GS = G / ROUNDS;
  // LDS element (c, k1, g') at c + SK k1 + SG g': ds_write_b128 of a thread's
  // two columns hits 8 distinct 16-byte slots per 8-lane group (SG = 8 mod
  // 16) and the pair reads 32 distinct dword pairs per 32-lane group (SK = 4
  // mod 32); 8 + SG (GS - 1) <= SK keeps the (c, g') blocks of every k1 apart.
  static constexpr int SG = 8;
  static constexpr int SK = (SG * GS + 27) / 32 * 32 + 4;
  static constexpr int BUF = SK * (P - 1) + SG * GS;   // complex elements per buffer
  static constexpr int NBUF = ROUNDS > 1 ? 2 : 1;      // double-buffered rounds: one barrier each
  static constexpr int TWS = 8 * (G + 1);              // W_M^{col P k2} rows of the 8 columns (padded: 4
                                                       // columns read by a 32-lane group on distinct banks)
  static_assert(P % 8 == 0 && G % 16 == 0 && NPAIR >= 1 && NPAIR * G == 2 * P, "one-exchange shape");
  static_assert(GS * ROUNDS == G && GS % 16 == 0 && 8 + SG * (GS - 1) <= SK, "one-exchange LDS layout");
  // two workgroups per CU (the whole 128 KiB exchange in one round, one
  // workgroup per CU, measured slower)
  static_assert((NBUF * BUF + TWS) * 8 <= kLdsBudget, "one-exchange LDS budget");
};

// The part both one-exchange passes share: P-point DFTs of the thread's two
// transforms, W_L^{g k1} (twL: the length-L table), the exchange, G-point
// DFTs of the thread's pairs (u[p][k2] = X[k1 + P k2] of pair p).
// W_L^{g k1}, k1 = 8 a + b, as (W_L^{8 g a}) (W_L^{g b}): the factors from the length-L table
template <int L, int P>
__device__ __forceinline__ void onex_wl(const float2* __restrict__ twL, int gg, float2 (&pb)[8], float2 (&pa)[P / 8]) {
  pb[0] = make_float2(1.f, 0.f);
#pragma unroll
  for (int b = 1; b < 8; ++b) pb[b] = twL[(gg * b) & (L - 1)];
  pa[0] = make_float2(1.f, 0.f);
#pragma unroll
  for (int a = 1; a < P / 8; ++a) pa[a] = twL[(gg * 8 * a) & (L - 1)];
}

// EARLY: pb / pa were loaded by the caller before the data loads (their
// round trip hidden behind the data's); else they are loaded here, after
// the DFTs, and the wave waits for them
template <int L, int G, int R, bool EARLY>
__device__ __forceinline__ void onex_core(float2 (&va)[L / G], float2 (&vb)[L / G], float2 (&u)[2 * (L / G) / G][G],
                                          float2* __restrict__ lds, const float2* __restrict__ twL, int t,
                                          float2 (&pb)[8], float2 (&pa)[L / G / 8]) {
  using C = OneX<L, G, R>;
  constexpr int P = C::P;
  const int lane = t & 63, w = t >> 6, cp = t & 3, gg = t >> 2, rc = (lane >> 3) & 7;
  dft<P>(va);
  dft<P>(vb);
  {
    if constexpr (!EARLY) onex_wl<L, P>(twL, gg, pb, pa);
#pragma unroll
    for (int a = 0; a < P / 8; ++a) {
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if (a == 0 && b == 0) continue;
        const float2 wv = a == 0 ? pb[b] : cmul(pa[a], pb[b]);
        va[8 * a + b] = cmul(va[8 * a + b], wv);
        vb[8 * a + b] = cmul(vb[8 * a + b], wv);
      }
    }
  }
  trace_event(2);
  // exchange: round r moves g in [r GS, (r + 1) GS); reader pair p of lane
  // (w, lane) is column c = lane >> 3, k1 = 8 (w + NW p) + (lane & 7)
#pragma unroll
  for (int r = 0; r < C::ROUNDS; ++r) {
    float2* buf = lds + (r & 1) * C::BUF;  // rounds alternate buffers: the barrier of round r also
                                           // retires every read of round r - 1
    if (gg / C::GS == r) {
      const int gq = gg - r * C::GS;
#pragma unroll
      for (int k1 = 0; k1 < P; ++k1) {
        float4* d = reinterpret_cast<float4*>(buf + 2 * cp + C::SK * k1 + C::SG * gq);
        *d = make_float4(va[k1].x, va[k1].y, vb[k1].x, vb[k1].y);
      }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < C::NPAIR; ++p) {
      const int k1 = 8 * (w + C::NW * p) + (lane & 7);
      const float2* s = buf + rc + C::SK * k1;
#pragma unroll
      for (int q = 0; q < C::GS; ++q) u[p][r * C::GS + q] = s[C::SG * q];
    }
  }
  trace_event(3);
#pragma unroll
  for (int p = 0; p < C::NPAIR; ++p) dft<G>(u[p]);
  trace_event(4);
}

template <int L, int G, int R, bool STRIPS, bool EARLY, bool WIDE = false>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, OneX<L, G, R>::THREADS), amdgpu_waves_per_eu(2)))
fft4_colpass_onex_kernel(const float* __restrict__ in, const float* __restrict__ in_pad, uint64_t n,
                         const double* __restrict__ afs, int K, float2* __restrict__ Y, Fft4Geom g,
                         const float2* __restrict__ tab, int flags) {
  using C = OneX<L, G, R>;
  constexpr int P = C::P;
  __shared__ __attribute__((aligned(16))) float2 lds[C::NBUF * C::BUF + C::TWS];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int cp = t & 3, gg = t >> 2;
  const int N1 = g.n1;
  trace_event(0);
  // block -> (trial k, first column c0): the Stockham kernel's order and XCD grouping
  const uint32_t lb = logical_block(gridDim.x, !(flags & kFft4NoRemap));
  int k = static_cast<int>(lb % static_cast<uint32_t>(K));
  int c0 = static_cast<int>(lb / static_cast<uint32_t>(K)) * 8;
  if ((flags & kFft4GroupXcd) && (K & 7) == 0) {
    const uint32_t b = blockIdx.x;
    const uint32_t Gp = ((b >> 7) << 3) | (b & 7u), wq = (b >> 3) & 15u;
    const uint32_t kg = static_cast<uint32_t>(K) >> 3;
    k = static_cast<int>(8 * (Gp % kg) + (wq & 7u));
    c0 = static_cast<int>(2 * (Gp / kg) + (wq >> 3)) * 8;
  } else if (flags & kFft4PairXcd) {
    const uint32_t b = blockIdx.x;
    const uint32_t s = (b >> 3) & 1u, u = ((b >> 4) << 3) | (b & 7u);
    k = static_cast<int>(u % static_cast<uint32_t>(K));
    c0 = static_cast<int>(2 * (u / static_cast<uint32_t>(K)) + s) * 8;
  }
  const int log2row = __builtin_ctz(static_cast<unsigned>(2 * N1));
  const TableOffsets to = table_offsets(N1, L);
  const double af = afs[k];
  // workgroup-uniform: readfirstlane keeps pointers built from it (and the
  // buffer resource of the one-exchange loads) in SGPRs -- a VGPR resource
  // wraps every buffer load in a waterfall loop
  const uint64_t src =
      __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g.tsrc ? g.tsrc[k] : static_cast<uint64_t>(k)));
  const float* ink = in + src * g.in_tstride;
  const float* padk = in_pad + src * g.pad_tstride;
  const uint32_t nn = static_cast<uint32_t>(n);
  float2* tws = lds + C::NBUF * C::BUF;
  static_assert(onex_g(L) == G, "one-exchange twiddle table shape");
  // rows c0 .. c0 + 7 of the ox table: loaded first, written to LDS only
  // after the input loads are issued (a store here would wait for its load --
  // a whole memory round trip -- before the first input load goes out);
  // visible to every thread after the exchange's first barrier
  static_assert((8 * G) % C::THREADS == 0, "ox rows per thread");
  constexpr int kTw = 8 * G / C::THREADS;
  const int rc = (lane >> 3) & 7;
  const uint32_t mask = static_cast<uint32_t>(N1) * L - 1;
  const uint32_t col = static_cast<uint32_t>(c0 + rc);
  float2 pb[8], pa[P / 8], om_hi = make_float2(1.f, 0.f), om_lo = om_hi;
  if constexpr (EARLY) {
    // every table value the thread needs after its data loads (the W_L
    // factors of the P-point DFT outputs, the two factors of the four-step
    // twiddle W_M^{col k1}), issued first: the data loads' round trip covers
    // theirs, and nothing waits on a dependent load after the exchange
    onex_wl<L, P>(tab + to.n2, gg, pb, pa);
    const uint32_t a0 = (col * static_cast<uint32_t>(8 * w + (lane & 7))) & mask;  // (NPAIR == 1: k1 of pair 0)
    om_hi = tab[to.hi + (a0 >> kSplit)];
    om_lo = tab[to.lo + (a0 & ((1u << kSplit) - 1))];
  }
  float2 twv[kTw];
#pragma unroll
  for (int q = 0; q < kTw; ++q) twv[q] = tab[to.ox + static_cast<uint64_t>(c0) * G + t + q * C::THREADS];
  const float afl = static_cast<float>(af), sizef = static_cast<float>(n);
  // fp32 shift estimate: |af p (p - n)| <= |af| n^2 / 4 with < 2.4e-7 relative
  // error; exact float positions need n <= 2^24.  The row's other three
  // samples p0 + e differ from it by |af e (2 p0 + e - n)| <= 3 |af| (n + 3)
  // (~1.3e-3 at 2^23 and 500 m/s^2): a first estimate that far inside its
  // rounding interval gives all four samples its shift -- one estimate per
  // row, not one at each end.
  const float band = n <= (1ull << 24) ? 6e-7f * fabsf(afl) * sizef * sizef * 0.25f + 1e-5f +
                                             3.0003f * fabsf(afl) * (sizef + 3.0f)
                                       : 1.0f;

  float2 va[P], vb[P];  // columns c0 + 2cp, c0 + 2cp + 1
  {
    // four consecutive resampled samples x[p0 .. p0+3] per row (resampleII):
    // the shift rint(af p (p - n)) is estimated in fp32 at p0; when the
    // estimate is further than `band` (the fp32 error bound plus the span's
    // change) from a rounding tie, the samples share that shift and are one
    // 16-byte load of the padded input (32-bit buffer offsets); other rows
    // (rare: a shift step inside the four samples, a near-tie, a series edge)
    // are redone below with every index evaluated exactly in double
    // (dev::accel_index_ii32, the reference's expression).
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(padk), 0, 0x7fffffff, 0x00020000);
    const uint32_t rowmask = (1u << log2row) - 1u, pitch = static_cast<uint32_t>(g.inpitch);
    constexpr bool strips = STRIPS;  // (the host pads in strips exactly when kFft4StripInput is set)
    const uint32_t nrows = static_cast<uint32_t>(L);
    uint32_t bad = 0;
    // Rows are loaded in the order dft<P> consumes them: its first radix-8
    // pass takes rows b, b + P/8, ..., b + 7 P/8 for b = 0, 1, ..., so the
    // compiler's vmcnt waits let the first groups' butterflies run while the
    // later groups' loads are still in flight.
#pragma unroll
    for (int ii = 0; ii < P; ++ii) {
      const int m = P >= 16 ? (P / 8) * (ii % 8) + ii / 8 : ii;
      const uint32_t j = static_cast<uint32_t>(gg + G * m);
      const uint32_t col = static_cast<uint32_t>(c0 + 2 * cp);
      const uint32_t p0 = 2u * (static_cast<uint32_t>(N1) * j + col);
      const float pa = static_cast<float>(p0);
      const float fa = afl * pa * (pa - sizef);
      const float sa = rintf(fa);
      // (32-bit: p0 < 2^24 where the fast path can hold, |shift| << 2^30)
      const int first = static_cast<int>(p0 + static_cast<uint32_t>(static_cast<int>(sa)));  // (wrapping add)
      // (& not &&: the compiler turned the short circuit into a branch per row)
      const bool ok = (fabsf(fa - sa) < 0.5f - band) & (first >= 0) & (first + 3 < static_cast<int>(nn));
      const uint32_t i = ok ? static_cast<uint32_t>(first) : p0;
      const uint32_t row = i >> log2row, ic = i & rowmask;
      const uint32_t off = strips ? ((ic >> 4) * nrows + row) * kStripW + (ic & 15u) : row * pitch + ic;
      const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, off * 4u, 0, 0));
      bad |= ok ? 0u : (1u << m);
      va[m] = make_float2(v.x, v.y);
      vb[m] = make_float2(v.z, v.w);
    }
    trace_event(1);
    if (bad != 0) {
      const double size = static_cast<double>(n);
#pragma unroll
      for (int m = 0; m < P; ++m) {
        if (bad & (1u << m)) {
          const uint32_t j = static_cast<uint32_t>(gg + G * m);
          const uint32_t p0 = 2u * (static_cast<uint32_t>(N1) * j + static_cast<uint32_t>(c0 + 2 * cp));
          float x[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = ink[dev::accel_index_ii32(af, size, p0 + static_cast<uint32_t>(e), nn - 1)];
          va[m] = make_float2(x[0], x[1]);
          vb[m] = make_float2(x[2], x[3]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kTw; ++q) {
    const int e = t + q * C::THREADS;
    tws[(e / G) * (G + 1) + (e % G)] = twv[q];
  }
  float2 u[C::NPAIR][G];
  onex_core<L, G, R, EARLY>(va, vb, u, lds, tab + to.n2, t, pb, pa);

  // four-step twiddle W_M^{col k}, k = k1 + P k2: W_M^{col k1} (table pair)
  // times W_M^{col P k2} (the staged ox rows); tiled store
  // Y_t[c0 / 8][k / 8][c][k % 8] (one 512-byte block per wave and k2)
  float2* yk = Y + static_cast<uint64_t>(k) * g.ystride + static_cast<uint64_t>(c0) * L;
  float2* yp = Y + static_cast<uint64_t>(k) * g.ystride + 2 * col;
  const float2* twr = tws + rc * (G + 1);
#pragma unroll
  for (int p = 0; p < C::NPAIR; ++p) {
    const uint32_t k1 = static_cast<uint32_t>(8 * (w + C::NW * p) + (lane & 7));
    const float2 om = EARLY && p == 0 ? cmul(om_hi, om_lo) : twiddle_M((col * k1) & mask, tab + to.lo, tab + to.hi);
    auto put = [&](int k2, float2 wv) {
      const uint32_t kk = k1 + static_cast<uint32_t>(P * k2);
      // (non-temporal: Y is read back only by the spectrum pass after the whole
      // batch, far beyond the caches; L2 and the Infinity Cache are left to the
      // input series every trial of a DM re-reads)
      const float2 yv = cmul(u[p][k2], wv);
      float2* dst = g.ypair ? yp + (kk >> 1) * (2 * static_cast<uint32_t>(N1)) + (kk & 1)  // Y_p[kk/2][col][kk%2]
                            : yk + (kk >> 3) * 64 + static_cast<uint32_t>(rc) * 8 + (kk & 7);
      __builtin_nontemporal_store(f2v{yv.x, yv.y}, reinterpret_cast<f2v*>(dst));
    };
    if constexpr (EARLY && WIDE) {
      // row-pair Y (g.ypair): lanes k1 (even) and k1 + 1 of a column write the
      // two halves of one 16-byte Y_p[kk/2][col] pair.  For each pair of k2
      // values (a, b) the even lane hands its b value to the odd lane and
      // takes the odd lane's a value (one DPP swap of adjacent lanes): the
      // even lane stores {own a, partner a}, the odd lane {partner b, own b}
      // -- one 16-byte store per lane per two k2, the same bytes and lines.
      const bool odd = lane & 1;
#pragma unroll
      for (int k0 = 0; k0 < G; k0 += 8) {
        float2 tw8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tw8[e] = twr[k0 + e];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const int a = k0 + e, b = a + 1;
          const float2 ya = cmul(u[p][a], a == 0 ? om : cmul(om, tw8[e]));
          const float2 yb = cmul(u[p][b], cmul(om, tw8[e + 1]));
          const float2 snd = odd ? ya : yb;
          // quad_perm [1, 0, 3, 2]: lane i reads lane i ^ 1
          const float2 rcv = make_float2(
              __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd.x), 0xB1, 0xF, 0xF, false)),
              __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd.y), 0xB1, 0xF, 0xF, false)));
          const float2 lo = odd ? rcv : ya, hi = odd ? yb : rcv;
          const uint32_t kk = (odd ? k1 - 1 : k1) + static_cast<uint32_t>(P * (odd ? b : a));  // even
          float2* dst = yp + (kk >> 1) * (2 * static_cast<uint32_t>(N1));
          __builtin_nontemporal_store(f4v{lo.x, lo.y, hi.x, hi.y}, reinterpret_cast<f4v*>(dst));
        }
      }
    } else if constexpr (EARLY) {
      // the staged ox values eight at a time: their LDS reads issued together,
      // one wait per eight stores instead of one per store
#pragma unroll
      for (int k0 = 0; k0 < G; k0 += 8) {
        float2 tw8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tw8[e] = twr[k0 + e];
#pragma unroll
        for (int e = 0; e < 8; ++e) put(k0 + e, k0 + e == 0 ? om : cmul(om, tw8[e]));
      }
    } else {
#pragma unroll
      for (int k2 = 0; k2 < G; ++k2) put(k2, k2 == 0 ? om : cmul(om, twr[k2]));
    }
  }
  trace_event(11);
}

// Pass B.  Logical block = row block * K + trial.
template <int L, int CPT, int SUB, int MODE>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, Cfg<L, CPT, SUB>::THREADS), amdgpu_waves_per_eu(2))) fft4_rowpass_kernel(
    const float2* __restrict__ Y, float2* __restrict__ X, int K, Fft4Geom g, const float2* __restrict__ tab,
    int flags, uint32_t keep_oct) {
  using C = Cfg<L, CPT, SUB>;
  constexpr bool kBlocked = MODE & kModeBlocked, kTileY = MODE & kModeTileY, kPairY = MODE & kModePairY;
  static_assert(!kTileY || (CPT == 8 && SUB == 1), "tiled Y: 8 transforms per thread");
  static_assert(!kPairY || kTileY, "row-pair Y: the tiled-Y kernel shape");
  __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];
  constexpr int T = C::T;
  const int grp = threadIdx.x / T;
  const int t = threadIdx.x - grp * T;
  const uint32_t lb = logical_block(gridDim.x, !(flags & kFft4NoRemap));
  trace_event(0);
  const int k = static_cast<int>(lb % static_cast<uint32_t>(K));
  const int r0 = static_cast<int>(lb / static_cast<uint32_t>(K)) * C::CH + grp * CPT;
  const TableOffsets to = table_offsets(L, g.n2);
  const float2* yk = Y + static_cast<uint64_t>(k) * g.ystride;
  Vec<CPT> v;
  if constexpr (kTileY) {
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const uint32_t i = t + q * T;
      const float4* src = reinterpret_cast<const float4*>(yk + static_cast<uint64_t>(i >> 3) * (8 * g.n2) +
                                                          (r0 >> 3) * 64 + (i & 7) * 8 + (r0 & 7));
#pragma unroll
      for (int c2 = 0; c2 < CPT / 2; ++c2) {
        const float4 w = src[c2];
        v[2 * c2][q] = make_float2(w.x, w.y);
        v[2 * c2 + 1][q] = make_float2(w.z, w.w);
      }
    }
  } else
#pragma unroll
  for (int c = 0; c < CPT; ++c)
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const uint32_t i = t + q * T;
      if (kBlocked)  // Y_b[i/8][r0 + c][i%8] (pass A always writes 8-wide blocks)
        v[c][q] = yk[static_cast<uint64_t>(i / 8) * (8 * g.n2) + (r0 + c) * 8 + (i % 8)];
      else
        v[c][q] = yk[static_cast<uint64_t>(r0 + c) * g.ypitch + i];
    }
  trace_event(1);
  fft_stages<L, CPT, C::CG, 1>(v, lds + grp * C::GROUP_FLOATS, t, tab + to.n1);
  float2* xk = X + static_cast<uint64_t>(k) * g.xstride;
  if constexpr ((MODE & kModeTileX) != 0) {
    // keep_oct > 0: only k1 octets [0, keep_oct) and [L/8 - keep_oct, L/8)
    // are ever read (bins below the search limit and their mirrors); a wave's
    // 64 lanes cover 8 whole octets, so the predicate is wave-uniform.
    const uint32_t hi_oct = L / 8 - keep_oct;
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const uint64_t k1 = t + q * T;
      const uint32_t oct = static_cast<uint32_t>(k1 >> 3);
      if (keep_oct != 0 && oct >= keep_oct && oct < hi_oct) continue;
      float2* dst = xk + static_cast<uint64_t>(r0 >> 3) * (8 * L) + (k1 >> 3) * 64 + (r0 & 7) * 8 + (k1 & 7);
#pragma unroll
      for (int c = 0; c < CPT; ++c) dst[c * 8] = v[c][q];
    }
    trace_event(11);
    return;
  }
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    const uint64_t k1 = t + q * T;
    // blocked: X_b[r0/8][k1][c] (8-wide blocks); else X[k1][k2] at pitch xpitch
    float2* dst = kBlocked ? xk + static_cast<uint64_t>(r0 / 8) * (8 * L) + k1 * 8 : xk + k1 * g.xpitch + r0;
    store_row<CPT>(dst, v, q);
  }
}

// ---------------------------------------------------------------------------
// Pass B fused with the search spectrum (fft4_rowpass_spectrum): row DFTs,
// real-FFT post-processing, interbinning, normalisation and the screening
// bytes in one pass.  The half-length spectrum Z never leaves the registers:
// the unfused search wrote it (8 bytes per bin) and read it back in the r2c
// pass; here each bin costs the 4 bytes of P and the 1 byte of Q.
//
// Bin k = r + n2 k1 (r = k2 < n2).  X[k] = r2c_combine(Z[k], Z[M-k], e^{-i pi k/M})
// (harmsum.hip) needs the mirror bin Z[M-k]: row n2-r at k1' = n1-1-k1 for
// r > 0, row 0 at -k1 for r = 0.  With W = e^{-2 pi i/n1} and Y_r the pass-A
// rows (the four-step twiddle W_M^{i r} applied), in both cases
//   Z[M-k] = sum_i W^{-i k1} u_r[i],  u_r[i] = W^{-i} Y_{n2-r}[i] (r > 0),  Y_0[i] (r = 0),
// = conj(FFT_n1(conj u_r))[k1]: the SAME k1 as Z[k] = FFT_n1(Y_r)[k1].  So a
// thread that transforms Y_r and conj(u_r) = W^{i} conj(Y_{n2-r}) holds Z[k]
// and Z[M-k] of the same bins in the same registers, with the forward FFT
// code for both ("pair-row" r).
//
// A workgroup transforms the pair-rows r = 4v .. 4v+4 (10 transforms per
// thread, v < n2/8) and forms
//   P[k]   for k = r + n2 k1, r = 4v+1 .. 4v+4   (interbin neighbour X[k-1]: pair-row r-1),
//   P[M-k] for k = r + n2 k1, r = 4v   .. 4v+3   (neighbour X[M-k-1] = X[M-(k+1)]: pair-row r+1),
// i.e. rows 1 .. n2/2 ascending and the rest as mirrors: every bin 1 .. M
// once; bin 0 (no left neighbour) by (v = 0, k1 = 0).  Pair-row 4v+4 is
// shared with the next workgroup (25% more row transforms; its Y is read
// again from L2: consecutive v run on one XCD, see the block order below).
//
// Outputs (kernels.hpp SpecOut): P in the workgroup-blocked layout
// spec_pblk_index (each lane stores 16 contiguous bytes per side and k1: whole
// lines per wave), Q in natural bin order shifted by kSpecQShift so that each
// lane's 4 bytes per side are one aligned dword; the 8 workgroups that share
// a 128-byte Q line run together on one XCD, so L2 merges the dwords.
// Reference: src/kernels.cu:231-252 (bin_interbin), :469-494 (normalise);
// the r2c step replaces cuFFT's R2C post-processing (pipeline_multi.cu:216-228).
constexpr int kSpecNp = 5;  // pair-rows per workgroup
// cos / sin of 2 pi q / 8 and of pi q / 8 = 2 pi q / 16, q < 8
__constant__ constexpr float kCos8[8] = {1.f, 0.70710678118654752f, 0.f, -0.70710678118654752f,
                                         -1.f, -0.70710678118654752f, 0.f, 0.70710678118654752f};
__constant__ constexpr float kSin8[8] = {0.f, 0.70710678118654752f, 1.f, 0.70710678118654752f,
                                         0.f, -0.70710678118654752f, -1.f, -0.70710678118654752f};
__constant__ constexpr float kCos16[8] = {1.f, 0.92387953251128676f, 0.70710678118654752f, 0.38268343236508977f,
                                          0.f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128676f};
__constant__ constexpr float kSin16[8] = {0.f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128676f,
                                          1.f, 0.92387953251128676f, 0.70710678118654752f, 0.38268343236508977f};

// EARLY (kFft4EarlyTw): the stage twiddles staged in LDS (TwLds) and the
// output phase's constants (statistics, r2c twiddle factors) loaded with the
// Y rows, so no dependent global round trip follows the loads.
template <int L>
struct SpecLds {
  static constexpr int EX = Cfg<L, 2 * kSpecNp, 1>::LDS_FLOATS;  // exchange buffer (floats)
  static constexpr int TW = 2 * TwLds<L>::N;                      // staged stage twiddles
  static constexpr int HT = 2 * (L / kPts);                       // e^{-i pi t / L}, one per thread
  // two workgroups per CU (163840 bytes): the per-thread factors join only where they fit
  static constexpr bool HT_LDS = (EX + TW + HT) * 4 * 2 <= 163840;
  static constexpr int TOTAL = EX + TW + (HT_LDS ? HT : 0);
  static_assert((EX + TW) * 4 * 2 <= 163840, "spectrum pass LDS: two workgroups per CU");
};

template <int L, bool PAIRY, bool EARLY>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, Cfg<L, 2 * kSpecNp, 1>::THREADS),
                               amdgpu_waves_per_eu(2)))
fft4_rowpass_spectrum_kernel(const float2* __restrict__ Y, int K, Fft4Geom g, const float2* __restrict__ tab,
                             SpecOut o) {
  constexpr int NP = kSpecNp, CPT = 2 * NP;
  using C = Cfg<L, CPT, 1>;
  using SL = SpecLds<L>;
  static_assert(!EARLY || TwLds<L>::covers(), "staged twiddles cover every stage");
  __shared__ __attribute__((aligned(16))) float lds[EARLY ? SL::TOTAL : C::LDS_FLOATS];
  constexpr int T = C::T;
  const int t = threadIdx.x;
  // block order: XCD x (blockIdx % 8) runs trials x, x+8, ..., each trial's
  // workgroups in increasing v (the writers of one Q line are consecutive)
  trace_event(0);
  const uint32_t n2 = static_cast<uint32_t>(g.n2), nv = n2 / 8;
  const uint32_t slot = blockIdx.x >> 3;
  // (readfirstlane: workgroup-uniform in SGPRs, with every address built from them)
  const int k = __builtin_amdgcn_readfirstlane(static_cast<int>(8 * (slot / nv) + (blockIdx.x & 7u)));
  if (k >= K) return;  // (the grid covers K rounded up to 8; workgroup-uniform)
  const uint32_t v = __builtin_amdgcn_readfirstlane(slot % nv);
  const TableOffsets to = table_offsets(L, static_cast<int>(n2));
  const float2* yk = Y + static_cast<uint64_t>(k) * g.ystride;
  const uint32_t fr = 4 * v;                     // forward rows fr .. fr+4 (channels 0..4)
  const uint32_t mg = n2 - 4 * v - 4;            // mirror rows mg .. mg+3 = pair-rows 4v+4 .. 4v+1 (channels 9..6)
  const uint32_t m0 = (n2 - 4 * v) & (n2 - 1);   // mirror row of pair-row 4v (channel 5; row 0 when v = 0)
  // W^{i} = W^{t} e^{-2 pi i q / 8} for i = t + q T (T = L / 8): one table
  // value per thread, the rest compile-time constants
  const float2 wt = tab[to.n1 + t];
  // EARLY: the staged table entries and this thread's e^{-i pi t / L} ahead
  // of the Y rows, the workgroup's statistics and r2c factors (scalar)
  // right behind them: all needed only after the FFT or its first exchange
  constexpr int kTwq = (TwLds<L>::N + T - 1) / T;
  float2 twq[EARLY ? kTwq : 1], ht_early = make_float2(1.f, 0.f);
  float mean_e = 0.f, sigma_e = 1.f;
  float2 hr_early[NP];
  if constexpr (EARLY) {
#pragma unroll
    for (int q = 0; q < kTwq; ++q) {
      const int e = t + q * T;
      twq[q] = e < TwLds<L>::N ? tab[to.n1 + TwLds<L>::index(e)] : make_float2(0.f, 0.f);
    }
    if constexpr (SL::HT_LDS) ht_early = tab[to.hk + t];
  }
  Vec<CPT> x;
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    const uint32_t i = t + q * T;
    float4 a0, a1, b0, b1;
    if constexpr (PAIRY) {
      // row pairs: Y_p[k2/2][i][k2%2] (fr, mg, m0 even)
      const float2* yi = yk + 2 * i;
      a0 = *reinterpret_cast<const float4*>(yi + (fr >> 1) * (2 * L));
      a1 = *reinterpret_cast<const float4*>(yi + ((fr >> 1) + 1) * (2 * L));
      b0 = *reinterpret_cast<const float4*>(yi + (mg >> 1) * (2 * L));
      b1 = *reinterpret_cast<const float4*>(yi + ((mg >> 1) + 1) * (2 * L));
      x[4][q] = yi[((fr >> 1) + 2) * (2 * L)];
      x[5][q] = yi[(m0 >> 1) * (2 * L)];
    } else {
      // tiled Y: Y_t[i/8][k2/8][i%8][k2%8]
      const float2* yi = yk + static_cast<uint64_t>(i >> 3) * (8 * n2) + (i & 7) * 8;
      const float4* a = reinterpret_cast<const float4*>(yi + (fr >> 3) * 64 + (fr & 7));
      const float4* b = reinterpret_cast<const float4*>(yi + (mg >> 3) * 64 + (mg & 7));
      a0 = a[0];
      a1 = a[1];
      b0 = b[0];
      b1 = b[1];
      x[4][q] = yi[((fr + 4) >> 3) * 64 + ((fr + 4) & 7)];
      x[5][q] = yi[(m0 >> 3) * 64 + (m0 & 7)];
    }
    x[0][q] = make_float2(a0.x, a0.y);
    x[1][q] = make_float2(a0.z, a0.w);
    x[2][q] = make_float2(a1.x, a1.y);
    x[3][q] = make_float2(a1.z, a1.w);
    x[9][q] = make_float2(b0.x, b0.y);
    x[8][q] = make_float2(b0.z, b0.w);
    x[7][q] = make_float2(b1.x, b1.y);
    x[6][q] = make_float2(b1.z, b1.w);
  }
  if constexpr (EARLY) {
    // (uniform values by scalar loads: in SGPRs, waited for by lgkmcnt)
    const uint32_t ts = o.tsrc ? dev::sload(o.tsrc, static_cast<uint64_t>(k)) : 0u;
    mean_e = dev::sload(o.stats, 4 * static_cast<uint64_t>(ts));
    sigma_e = dev::sload(o.stats, 4 * static_cast<uint64_t>(ts) + 2);
#pragma unroll
    for (int c = 0; c < NP; ++c) hr_early[c] = dev::sload2(tab, to.hr + fr + c);
  }
  // (every load is issued before the first use of a loaded value)
  __builtin_amdgcn_sched_barrier(0);
  float2* tw_lds = reinterpret_cast<float2*>(lds + C::LDS_FLOATS);
  float2* ht_lds = reinterpret_cast<float2*>(lds + C::LDS_FLOATS + SL::TW);
  if constexpr (EARLY) {
    // (visible to every thread after the first exchange's barrier; stage 0
    // reads no twiddle)
#pragma unroll
    for (int q = 0; q < kTwq; ++q)
      if (t + q * T < TwLds<L>::N) tw_lds[t + q * T] = twq[q];
    if constexpr (SL::HT_LDS) ht_lds[t] = ht_early;
  }
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    // mirror channels: conj(u_r) = W^{i} conj(Y_{n2-r}) (pair-row 0: conj(Y_0))
    const float2 w = q == 0 ? wt : cmul(wt, make_float2(kCos8[q], -kSin8[q]));
#pragma unroll
    for (int c = NP; c < CPT; ++c) {
      const float2 y = make_float2(x[c][q].x, -x[c][q].y);
      x[c][q] = (c == NP && v == 0) ? y : cmul(w, y);
    }
  }
  trace_event(1);
  if constexpr (EARLY)
    fft_stages<L, CPT, C::CG, 1>(x, lds, t, TwLds<L>{tw_lds});
  else
    fft_stages<L, CPT, C::CG, 1>(x, lds, t, tab + to.n1);
  trace_event(9);

  float mean, sigma;
  float2 hr[NP];  // e^{-i pi r / M}, r = 4v .. 4v+4 (workgroup-uniform)
  if constexpr (EARLY) {
    mean = mean_e * o.nscale;
    sigma = sigma_e * o.nscale;
#pragma unroll
    for (int c = 0; c < NP; ++c) hr[c] = hr_early[c];
  } else {
    const float* st = o.stats + (o.tsrc ? 4 * static_cast<uint64_t>(o.tsrc[k]) : 0);
    mean = st[0] * o.nscale;
    sigma = st[2] * o.nscale;
#pragma unroll
    for (int c = 0; c < NP; ++c) hr[c] = tab[to.hr + fr + c];
  }
  const float rsig = 1.0f / sigma;  // per bin dev::div_rn: IEEE division
  const uint32_t M = static_cast<uint32_t>(L) * n2;
  float4* pk = reinterpret_cast<float4*>(o.P + static_cast<uint64_t>(k) * o.pstride);
  uint8_t* qk = o.Q + static_cast<uint64_t>(k) * o.qstride + kSpecQShift;  // qk[b]: bin b
  // A fresh copy of t: without it the compiler keeps the load phase's per-q
  // indices alive across the FFT (spilled to scratch, and every reload then
  // waited behind the Q/P stores already in flight: one vmcnt queue).
  // The output phase issues no vector load at all.
  uint32_t tt = static_cast<uint32_t>(t);
  asm volatile("" : "+v"(tt));
  // e^{-i pi k1 / L} = e^{-i pi t / L} e^{-i pi q / 8} (k1 = t + q T), formed per q
  float2 ht = EARLY && SL::HT_LDS ? ht_lds[tt] : tab[to.hk + tt];
  asm volatile("" : "+v"(ht.x), "+v"(ht.y));
  // Scaled forms (all factors exact powers of two): with e = z + w and
  // d = z - w (w = conj Z[M-k], as the mirror channel holds it), 2 X[k] =
  // e + (A, B) and 2 X[M-k] = (e.x - A, B - e.y), A = c d.y + s d.x,
  // B = s d.y - c d.x ((c, s) = e^{-i pi k / M}); interbinning the doubled
  // values doubles the amplitude, so P = (amp2 - 2 mean) / (2 sigma) rounds
  // exactly as (amp - mean) / sigma.
  const float mean2 = 2.0f * mean, sigma2 = 2.0f * sigma, rsig2 = 0.5f * rsig;
  const uint32_t nb = o.nbins ? o.nbins : M + 1;  // bins the search reads
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    // (one iteration at a time: interleaving them raised the register peak into scratch spills)
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t k1 = tt + q * T;
    // forward bins n2 k1 + fr + 1 .. + 4, mirror bins M - n2 k1 - fr - 3 .. M - n2 k1 - fr:
    // formed and stored only below nb (lanes of a wave share k1's high bits:
    // whole waves skip)
    const bool wf = n2 * k1 + fr + 1 < nb, wm = M - n2 * k1 - fr - 3 < nb;
    if (!(wf | wm)) continue;
    const float2 hk = q == 0 ? ht : cmul(ht, make_float2(kCos16[q], -kSin16[q]));  // e^{-i pi k1 / L}
    float2 X[NP], Xm[NP];
#pragma unroll
    for (int c = 0; c < NP; ++c) {
      const float2 tw = cmul(hk, hr[c]);  // e^{-i pi (r + n2 k1) / M}
      const float2 z = x[c][q], w = x[NP + c][q];
      const float2 e = make_float2(z.x + w.x, z.y + w.y);
      const float2 d = make_float2(z.x - w.x, z.y - w.y);
      const float A = __builtin_fmaf(tw.x, d.y, tw.y * d.x);
      const float B = __builtin_fmaf(tw.y, d.y, -(tw.x * d.x));
      X[c] = make_float2(e.x + A, e.y + B);
      Xm[c] = make_float2(e.x - A, B - e.y);
    }
    // interbinned amplitude (bin_interbin: max(|X|^2, |X - X_left|^2 / 2)), hardware sqrt
    auto amp = [](float2 a, float2 l) {
      const float p2 = __builtin_fmaf(a.x, a.x, a.y * a.y);
      const float dx = a.x - l.x, dy = a.y - l.y;
      const float q2 = __builtin_fmaf(dx, dx, dy * dy) * 0.5f;
      return __builtin_amdgcn_sqrtf(fmaxf(p2, q2));
    };
    float pp[4], pm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pp[j] = dev::div_rn(amp(X[j + 1], X[j]) - mean2, sigma2, rsig2);
      pm[j] = dev::div_rn(amp(Xm[j], Xm[j + 1]) - mean2, sigma2, rsig2);
    }
    // (P streams out: only candidate bins are read back, much later; non-temporal
    // stores leave L2 to the Q lines still being assembled and the Y reads)
    if (wf) __builtin_nontemporal_store(f4v{pp[0], pp[1], pp[2], pp[3]}, reinterpret_cast<f4v*>(pk + 2 * v * L + k1));
    if (wm)
      __builtin_nontemporal_store(f4v{pm[0], pm[1], pm[2], pm[3]}, reinterpret_cast<f4v*>(pk + (2 * v + 1) * L + k1));
    // screening bytes (dev::q8): t = rint(4 p) + 127 -> t in [0, 253] as is,
    // >= 254 or NaN -> 254, <= -1 -> 255 (min first: NaN -> 254)
    auto qb = [](float p) {
      const float t = fmaxf(fminf(rintf(p * 4.0f) + 127.0f, 254.0f), -1.0f);
      return static_cast<uint32_t>(static_cast<int>(t)) & 0xffu;
    };
    const uint32_t qa = qb(pp[0]) | (qb(pp[1]) << 8) | (qb(pp[2]) << 16) | (qb(pp[3]) << 24);
    const uint32_t qm = qb(pm[3]) | (qb(pm[2]) << 8) | (qb(pm[1]) << 16) | (qb(pm[0]) << 24);
    if (wf) *reinterpret_cast<uint32_t*>(qk + fr + 1 + n2 * k1) = qa;        // bins fr+1 .. fr+4 (+ n2 k1)
    if (wm) *reinterpret_cast<uint32_t*>(qk + (M - n2 * k1 - fr - 3)) = qm;  // bins M - n2 k1 - (fr+3 .. fr)
    if (v == 0 && k1 == 0) {  // bin 0: X[-1] = 0 (bin_interbin)
      const float p0 = dev::div_rn(amp(X[0], make_float2(0.f, 0.f)) - mean2, sigma2, rsig2);
      o.P[static_cast<uint64_t>(k) * o.pstride + M] = p0;
      qk[0] = static_cast<uint8_t>(qb(p0));
    }
  }
  trace_event(11);
}

bool supported_len(int L) { return L >= 128 && L <= 4096 && (L & (L - 1)) == 0; }

}  // namespace

Fft4Geom fft4_geometry(uint64_t M) {
  Fft4Geom g;
  if (M == 0 || (M & (M - 1)) != 0) return g;
  int lg = 0;
  while ((uint64_t(1) << lg) < M) ++lg;
  const int a = lg / 2, b = lg - a;  // N2 = 2^a <= N1 = 2^b
  if (!supported_len(1 << a) || !supported_len(1 << b)) return g;
  g.n1 = 1 << b;
  g.n2 = 1 << a;
  g.ypitch = static_cast<uint64_t>(g.n1) + 8;
  g.ystride = g.ypitch * g.n2;
  g.xpitch = static_cast<uint64_t>(g.n2) + 8;
  g.xstride = g.xpitch * g.n1;
  g.log2_xrow = a;
  g.inpitch = 2 * static_cast<uint64_t>(g.n1) + 32;
  g.insize = std::max(g.inpitch * g.n2, strip_floats(g.n1, g.n2));
  g.ok = true;
  return g;
}

Fft4Geom fft4_geometry_rows(uint64_t M) {
  Fft4Geom g;
  constexpr int kCol = 4096;  // the longest column the Stockham pass A takes
  if (M == 0 || (M & (M - 1)) != 0 || M < uint64_t(2) * kCol * kCol || M >= (uint64_t(1) << 31)) return g;
  g.n2 = kCol;
  g.n1 = static_cast<int>(M / kCol);
  g.rows_ext = true;
  g.ypitch = static_cast<uint64_t>(g.n1) + 8;  // natural Y rows: the row FFT's input, pitch off a power of two
  g.ystride = g.ypitch * g.n2;
  g.xpitch = static_cast<uint64_t>(g.n1) + 8;  // the row FFT's output rows (r2c_interbin_normalise_rows)
  g.xstride = g.xpitch * g.n2;
  g.log2_xrow = __builtin_ctz(static_cast<unsigned>(kCol));
  g.inpitch = 2 * static_cast<uint64_t>(g.n1) + 32;
  g.insize = g.inpitch * g.n2;
  g.ok = true;
  return g;
}

std::vector<float2> fft4_tables(const Fft4Geom& g) {
  const TableOffsets o = table_offsets(g.n1, g.n2);
  const double M = static_cast<double>(g.n1) * g.n2;
  std::vector<float2> t(o.total);
  auto w = [](double num, double den) {
    const double a = -2.0 * M_PI * num / den;
    return make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a)));
  };
  for (int m = 0; m < g.n2; ++m) t[o.n2 + m] = w(m, g.n2);
  for (int m = 0; m < g.n1; ++m) t[o.n1 + m] = w(m, g.n1);
  for (uint64_t m = 0; m < (1u << kSplit); ++m) t[o.lo + m] = w(static_cast<double>(m), M);
  for (uint64_t m = 0; m < (o.ox - o.hi); ++m) t[o.hi + m] = w(static_cast<double>(m << kSplit), M);
  const uint64_t GX = static_cast<uint64_t>(onex_g(g.n2)), PX = static_cast<uint64_t>(g.n2) / GX;
  const uint64_t Mi = static_cast<uint64_t>(g.n1) * static_cast<uint64_t>(g.n2);
  for (uint64_t col = 0; col < static_cast<uint64_t>(g.n1); ++col)
    for (uint64_t k2 = 0; k2 < GX; ++k2) t[o.ox + col * GX + k2] = w(static_cast<double>((col * PX * k2) % Mi), M);
  for (int k1 = 0; k1 < g.n1; ++k1) t[o.hk + k1] = w(0.5 * k1, g.n1);
  for (int r = 0; r <= g.n2 / 2; ++r) t[o.hr + r] = w(0.5 * r, M);
  return t;
}

namespace {
// fastest measured (tools/kbench.py, bench A/B); the strip input: pass A 15.9 -> 13.9 us/trial alone,
// bench within noise (profiles/r3_strip)
int g_fft4_flags = kFft4Cpt8 | kFft4NoRemap | kFft4Blocked | kFft4TileY | kFft4TileX | kFft4PairXcd |
                   kFft4GroupXcd | kFft4UniformTw | kFft4OneX | kFft4StripInput | kFft4PairY | kFft4EarlyTw |
                   kFft4WideY | kFft4WhitenStrips | kFft4WhitenU8;
}  // namespace

void fft4_pad_input_u8(const uint8_t* in, uint64_t nvalid, uint64_t n, const unsigned long long* sum, float* in_pad,
                       const Fft4Geom& g, hipStream_t s, int count, uint64_t in_stride) {
  PSOUP_CHECK(count >= 1 && count <= 65535, "fft4_pad_input_u8: bad count");
  PSOUP_CHECK(strip_layout(g, g_fft4_flags) || fft4_direct_source(g), "fft4_pad_input_u8: strip layouts only");
  PSOUP_CHECK(n == 2ull * g.n1 * g.n2 && nvalid <= n, "fft4_pad_input_u8: length");
  const uint32_t rowlen = 2u * static_cast<uint32_t>(g.n1);
  PSOUP_CHECK(rowlen % 16 == 0 && rowlen <= static_cast<uint32_t>(kStripLdsBytes) && strip_floats(g.n1, g.n2) <= g.insize &&
                  g.insize % 4 == 0 && (reinterpret_cast<uintptr_t>(in_pad) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (count == 1 || in_stride % 16 == 0),
              "fft4_pad_input_u8: strip layout size / alignment");
  int log2_r = 0;  // rows per workgroup: the staged rows fill kStripLdsBytes, at most 16
  while (log2_r < 4 && (rowlen << (log2_r + 1)) <= static_cast<uint32_t>(kStripLdsBytes) &&
         (g.n2 >> (log2_r + 1)) >= 1)
    ++log2_r;
  PSOUP_CHECK(g.n2 % (1 << log2_r) == 0, "fft4_pad_input_u8: rows per workgroup");
  const dim3 grid(static_cast<unsigned>(g.n2 >> log2_r), static_cast<unsigned>(count));
  fft4_strips_u8_kernel<<<grid, 256, 0, s>>>(in, nvalid, n, sum, in_pad, rowlen, static_cast<uint32_t>(g.n2), log2_r,
                                             in_stride, g.insize);
  post_launch_check("fft4_strips_u8_kernel", s);
}

void fft4_pad_input(const float* in, uint64_t n, float* in_pad, const Fft4Geom& g, hipStream_t s, int count,
                    uint64_t in_stride) {
  PSOUP_CHECK(count >= 1 && count <= 65535, "fft4_pad_input: bad count");
  if (strip_layout(g, g_fft4_flags)) {
    const uint64_t rows = strip_floats(g.n1, g.n2) / kStripW;
    PSOUP_CHECK(rows < (1ull << 32) && rows * kStripW <= g.insize && g.insize % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(in_pad) & 15) == 0,
                "fft4_pad_input: strip layout size / alignment");
    const bool aligned = (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (count == 1 || in_stride % 4 == 0);
    const dim3 grid(dev::grid_for(rows, 256, count > 1 ? 1024 : 4096), static_cast<unsigned>(count));
    fft4_pad_strips_kernel<<<grid, 256, 0, s>>>(in, n, in_pad, 2u * static_cast<uint32_t>(g.n1),
                                                __builtin_ctz(static_cast<unsigned>(g.n2)), static_cast<uint32_t>(rows),
                                                in_stride, g.insize, aligned);
    post_launch_check("fft4_pad_strips_kernel", s);
    return;
  }
  const uint64_t total = g.inpitch * g.n2;
  const bool vec = n % 4 == 0 && g.inpitch % 4 == 0 && g.n1 % 2 == 0 && in_stride % 4 == 0 && g.insize % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (reinterpret_cast<uintptr_t>(in_pad) & 15) == 0 &&
                   total / 4 < (1ull << 32) && n / 4 < (1ull << 32);
  if (vec) {
    const dim3 grid(dev::grid_for(total / 4, 256, count > 1 ? 1024 : 4096), static_cast<unsigned>(count));
    fft4_pad_input_vec_kernel<<<grid, 256, 0, s>>>(
        reinterpret_cast<const float4*>(in), static_cast<uint32_t>(n / 4), reinterpret_cast<float4*>(in_pad),
        static_cast<uint32_t>(g.n1 / 2), static_cast<uint32_t>(g.inpitch / 4), static_cast<uint32_t>(total / 4),
        in_stride / 4, g.insize / 4);
    post_launch_check("fft4_pad_input_vec_kernel", s);
    return;
  }
  const dim3 grid(dev::grid_for(total, 256, count > 1 ? 1024 : 4096), static_cast<unsigned>(count));
  fft4_pad_input_kernel<<<grid, 256, 0, s>>>(in, n, in_pad, 2ull * g.n1, g.inpitch, total, in_stride, g.insize);
  post_launch_check("fft4_pad_input_kernel", s);
}

namespace {

template <int CPT, int SUB, int MODE, int SRC = kSrcPad>
void launch_colpass(const float* in, const float* in_pad, uint64_t n, const double* af, int K, float2* Y,
                    const Fft4Geom& g, const float2* tables, dim3 grid, int flags, hipStream_t s) {
  switch (g.n2) {
#define PS_CASE(LL)                                                                                         \
  case LL:                                                                                                  \
    fft4_colpass_kernel<LL, CPT, SUB, MODE, SRC><<<grid, Cfg<LL, CPT, SUB>::THREADS, 0, s>>>(in, in_pad, n, af, K, Y, \
                                                                                            g, tables, flags); \
    break;
    PS_CASE(128) PS_CASE(256) PS_CASE(512) PS_CASE(1024) PS_CASE(2048) PS_CASE(4096)
#undef PS_CASE
    default: PSOUP_THROW("fft4: unsupported column length " << g.n2);
  }
}

template <int CPT, int SUB, int MODE>
void launch_rowpass(const float2* Y, float2* X, int K, const Fft4Geom& g, const float2* tables, dim3 grid, int flags,
                    hipStream_t s, uint32_t keep_oct = 0) {
  switch (g.n1) {
#define PS_CASE(LL)                                                                                             \
  case LL:                                                                                                      \
    fft4_rowpass_kernel<LL, CPT, SUB, MODE><<<grid, Cfg<LL, CPT, SUB>::THREADS, 0, s>>>(Y, X, K, g, tables, flags, \
                                                                                        keep_oct);             \
    break;
    PS_CASE(128) PS_CASE(256) PS_CASE(512) PS_CASE(1024) PS_CASE(2048) PS_CASE(4096)
#undef PS_CASE
    default: PSOUP_THROW("fft4: unsupported row length " << g.n1);
  }
}

}  // namespace

void fft4_rowpass_spectrum(const float2* Y, int K, const Fft4Geom& g, const float2* tables, const SpecOut& o,
                           hipStream_t s) {
  PSOUP_CHECK(g.ok && K >= 1 && g.n2 >= 16 && g.n1 >= 128 && !g.rows_ext, "fft4 spectrum pass: bad geometry");
  const uint64_t M = static_cast<uint64_t>(g.n1) * g.n2;
  PSOUP_CHECK(M < (1ull << 31), "fft4 spectrum pass: spectrum too long for 32-bit bin indices");
  const int f = g_fft4_flags;
  PSOUP_CHECK((f & kFft4Blocked) && (f & kFft4TileY), "fft4 spectrum pass: needs the tiled Y layout");
  PSOUP_CHECK(o.P && o.Q && o.stats && o.pstride >= M + 1 && o.pstride % 4 == 0 && o.qstride >= M + 1 + kSpecQShift &&
                  o.qstride % 16 == 0 && (reinterpret_cast<uintptr_t>(o.P) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(o.Q) & 15) == 0 && (reinterpret_cast<uintptr_t>(Y) & 15) == 0,
              "fft4 spectrum pass: output layout");
  const uint64_t nblocks = static_cast<uint64_t>(g.n2 / 8) * ((static_cast<uint64_t>(K) + 7) / 8 * 8);
  PSOUP_CHECK(nblocks < (1ull << 31), "fft4 spectrum pass: grid");
  const dim3 grid(static_cast<unsigned>(nblocks));
  PSOUP_CHECK(!g.ypair || fft4_pair_y(g), "fft4 spectrum pass: pass A cannot write the row-pair Y layout");
  switch (g.n1) {
#define PS_CASE(LL)                                                                                         \
  case LL:                                                                                                  \
    if (g.ypair && (f & kFft4EarlyTw))                                                                      \
      fft4_rowpass_spectrum_kernel<LL, true, true><<<grid, Cfg<LL, 2 * kSpecNp, 1>::THREADS, 0, s>>>(Y, K, g, tables, \
                                                                                                  o);             \
    else if (g.ypair)                                                                                       \
      fft4_rowpass_spectrum_kernel<LL, true, false><<<grid, Cfg<LL, 2 * kSpecNp, 1>::THREADS, 0, s>>>(Y, K, g,       \
                                                                                                   tables, o);    \
    else                                                                                                    \
      fft4_rowpass_spectrum_kernel<LL, false, false><<<grid, Cfg<LL, 2 * kSpecNp, 1>::THREADS, 0, s>>>(Y, K, g,      \
                                                                                                    tables, o);   \
    break;
    PS_CASE(128) PS_CASE(256) PS_CASE(512) PS_CASE(1024) PS_CASE(2048) PS_CASE(4096)
#undef PS_CASE
    default: PSOUP_THROW("fft4 spectrum pass: unsupported row length " << g.n1);
  }
  post_launch_check("fft4_rowpass_spectrum_kernel", s);
}

bool fft4_pair_y(const Fft4Geom& g) { return g.ok && pair_y_layout(g.n2, g_fft4_flags); }
bool fft4_direct_source(const Fft4Geom& g) {
  const int f = g_fft4_flags;
  return g.ok && g.zero_shift && !g.ypair && !onex_colpass(g.n2, f) && (f & kFft4Blocked) && (f & kFft4TileY);
}
bool fft4_strip_layout(const Fft4Geom& g) { return g.ok && strip_layout(g, g_fft4_flags); }

void fft4_set_flags(int flags) {
  g_fft4_flags = flags;
  set_numerics_flag("fft4_flags", flags);
}
void fft4_set_trace(unsigned long long* d_events) {
  PSOUP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_fft4_trace), &d_events, sizeof(d_events)));
}

// The tiled spectrum needs 8 x 256 r2c tiles: n2 >= 256, n1 >= 16.
bool tiled_x(const Fft4Geom& g, int f) {
  return (f & kFft4Blocked) && (f & kFft4TileY) && (f & kFft4TileX) && g.n2 >= 256 && g.n1 >= 16;
}

Fft4XLayout fft4_x_layout(const Fft4Geom& g) {
  const int f = g_fft4_flags;
  if (tiled_x(g, f)) return {g.log2_xrow, 0, 0, 3, true};
  if ((f & kFft4Blocked) && (f & kFft4Cpt8)) return {g.log2_xrow, 8, 8ull * g.n1, 3, false};
  return {g.log2_xrow, g.xpitch, 8, 3, false};
}
int fft4_flags() { return g_fft4_flags; }

// Kernel shape per flag set (both passes):
//   Blocked + TileY (+ OneX at column length 2048): the production shapes;
//   Cpt8 + Blocked: 8 transforms per thread, blocked Y/X (small geometries);
//   Cpt8: natural Y/X, 8 transforms per thread; none: natural, 2 x 4.
void fft4_resample_colpass(const float* in, const float* in_pad, uint64_t n, const double* af, int K, float2* Y,
                           const Fft4Geom& g, const float2* tables, hipStream_t s) {
  PSOUP_CHECK(g.ok && K >= 1 && n == 2ull * g.n1 * g.n2, "fft4 colpass: bad geometry n=" << n << " K=" << K);
  PSOUP_CHECK(n < (1ull << 31) && g.insize < (1ull << 32), "fft4 colpass: series too long for 32-bit indices");
  PSOUP_CHECK((reinterpret_cast<uintptr_t>(Y) & 63) == 0, "fft4 colpass: Y alignment");
  const int f = g_fft4_flags;
  const uint64_t nblocks = static_cast<uint64_t>(g.n1 / 8) * K;
  PSOUP_CHECK(nblocks < (1ull << 31) && nblocks % 16 == 0, "fft4 colpass: grid");
  PSOUP_CHECK(!(f & kFft4GroupXcd) || (K & 7) != 0 || nblocks % 128 == 0, "fft4 colpass: group grid");
  const dim3 grid(static_cast<unsigned>(nblocks));
  PSOUP_CHECK(!g.ypair || pair_y_layout(g.n2, f), "fft4 colpass: this pass A cannot write the row-pair Y layout");
  PSOUP_CHECK(!g.rows_ext || !(g.u8 || g.c2r || g.f32_direct || g.strips_direct || g.ypair || g.zero_shift),
              "fft4 colpass: the external-row geometry takes the padded input and writes natural Y");
  if (g.u8 || g.c2r || g.f32_direct || g.strips_direct) {
    PSOUP_CHECK(fft4_direct_source(g) && (!!g.u8 + !!g.c2r + g.f32_direct + g.strips_direct) == 1,
                "fft4 colpass: direct sources need a zero-shift Stockham pass A");
    PSOUP_CHECK(!g.f32_direct || ((reinterpret_cast<uintptr_t>(in) & 15) == 0 && (K == 1 || g.in_tstride % 4 == 0)),
                "fft4 colpass: f32 source alignment");
    PSOUP_CHECK(!g.u8 || (g.u8sum && g.u8_nvalid <= n && (reinterpret_cast<uintptr_t>(g.u8) & 15) == 0 &&
                          (K == 1 || g.src_stride % 16 == 0)),
                "fft4 colpass: 8-bit source layout");
    PSOUP_CHECK(!g.c2r || (K == 1 || g.src_stride >= n / 2 + 1), "fft4 colpass: spectrum source layout");
  }
  if (g.rows_ext)  // natural Y rows for the external row FFT
    launch_colpass<8, 1, 0>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if (g.strips_direct)
    launch_colpass<8, 1, kModeBlocked | kModeTileY, kSrcStrips>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if (g.f32_direct)
    launch_colpass<8, 1, kModeBlocked | kModeTileY, kSrcF32>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if (g.u8)
    launch_colpass<8, 1, kModeBlocked | kModeTileY, kSrcU8>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if (g.c2r)
    launch_colpass<8, 1, kModeBlocked | kModeTileY, kSrcC2R>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if (onex_colpass(g.n2, f)) {
    constexpr int TH = OneX<2048, 64, 4>::THREADS;
    const bool strips = strip_layout(g, f);
    if (strips && (f & kFft4EarlyTw) && (f & kFft4WideY) && g.ypair)
      fft4_colpass_onex_kernel<2048, 64, 4, true, true, true><<<grid, TH, 0, s>>>(in, in_pad, n, af, K, Y, g, tables,
                                                                                  f);
    else if (strips && (f & kFft4EarlyTw))
      fft4_colpass_onex_kernel<2048, 64, 4, true, true><<<grid, TH, 0, s>>>(in, in_pad, n, af, K, Y, g, tables, f);
    else if (strips)
      fft4_colpass_onex_kernel<2048, 64, 4, true, false><<<grid, TH, 0, s>>>(in, in_pad, n, af, K, Y, g, tables, f);
    else
      fft4_colpass_onex_kernel<2048, 64, 4, false, false><<<grid, TH, 0, s>>>(in, in_pad, n, af, K, Y, g, tables, f);
  }
  else if (g.ypair)
    launch_colpass<8, 1, kModeBlocked | kModeTileY | kModePairY>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if ((f & kFft4Blocked) && (f & kFft4TileY))
    launch_colpass<8, 1, kModeBlocked | kModeTileY>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if ((f & kFft4Cpt8) && (f & kFft4Blocked))
    launch_colpass<8, 1, kModeBlocked>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else if (f & kFft4Cpt8)
    launch_colpass<8, 1, 0>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  else
    launch_colpass<4, 2, 0>(in, in_pad, n, af, K, Y, g, tables, grid, f, s);
  post_launch_check("fft4_colpass_kernel", s);
}

void fft4_rowpass(const float2* Y, float2* X, int K, const Fft4Geom& g, const float2* tables, hipStream_t s,
                  uint64_t nbins_out) {
  PSOUP_CHECK(g.ok && K >= 1 && !g.rows_ext, "fft4 rowpass: bad geometry");
  PSOUP_CHECK((reinterpret_cast<uintptr_t>(X) & 63) == 0, "fft4 rowpass: X alignment");
  const int f = g_fft4_flags;
  const uint64_t nblocks = static_cast<uint64_t>(g.n2 / 8) * K;
  PSOUP_CHECK(nblocks < (1ull << 31) && nblocks % 8 == 0, "fft4 rowpass: grid");
  const dim3 grid(static_cast<unsigned>(nblocks));
  const bool tiley = (f & kFft4Blocked) && (f & kFft4TileY);
  if (tiley && tiled_x(g, f)) {
    // rows r2c_interbin_normalise_tiled reads: octets [0, ny] and [n1/8 - ny, n1/8)
    uint32_t keep = 0;
    if (nbins_out > 0) {
      const uint32_t ny = r2c_tiled_row_blocks(nbins_out, g.n1, g.n2);
      if (2 * (ny + 1) < static_cast<uint32_t>(g.n1 / 8)) keep = ny + 1;
    }
    launch_rowpass<8, 1, kModeBlocked | kModeTileY | kModeTileX>(Y, X, K, g, tables, grid, f, s, keep);
  } else if (tiley)
    launch_rowpass<8, 1, kModeBlocked | kModeTileY>(Y, X, K, g, tables, grid, f, s);
  else if ((f & kFft4Cpt8) && (f & kFft4Blocked))
    launch_rowpass<8, 1, kModeBlocked>(Y, X, K, g, tables, grid, f, s);
  else if (f & kFft4Cpt8)
    launch_rowpass<8, 1, 0>(Y, X, K, g, tables, grid, f, s);
  else
    launch_rowpass<4, 2, 0>(Y, X, K, g, tables, grid, f, s);
  post_launch_check("fft4_rowpass_kernel", s);
}

}  // namespace kern
}  // namespace psoup
