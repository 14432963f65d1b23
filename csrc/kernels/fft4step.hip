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
// Each workgroup transforms 8 adjacent columns (pass A) or rows (pass B) at
// once, so every global access is one 64-byte vector per lane (8 complex
// values), and every thread owns the same 8 points of each of the 8
// transforms: 64 complex values in VGPRs.  The transforms are Stockham
// radix-8 (+ a final radix-4/2 stage) with LDS exchanges between stages, in
// channel groups sized to keep LDS at 72 KiB so two workgroups share a CU.
// Twiddles come from small host-built tables (double-precision), not
// per-thread transcendental evaluation.
#include "device_common.hpp"
#include "psoup/kernels.hpp"

#include <cmath>

namespace psoup {
namespace kern {

namespace {

constexpr int kCh = 8;   // transforms per workgroup -> 64-byte vectors per lane
constexpr int kPts = 8;  // points per thread per transform
constexpr int kSplit = 11;  // W_M^a = hi[a >> kSplit] * lo[a & (2^kSplit - 1)]

template <int L>
struct Cfg {
  static constexpr int T = L / kPts;                                // threads per workgroup
  static constexpr int CG = L >= 4096 ? 2 : (L >= 2048 ? 4 : 8);    // channels per LDS exchange
  static constexpr int PAD = L + L / 8;                             // padded floats per channel plane
  static constexpr int LDS_FLOATS = 2 * CG * PAD;
};

using Vec = float2[kCh][kPts];
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-byte load

__device__ __forceinline__ int lds_pad(int x) { return x + (x >> 3); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // * -i

__device__ __forceinline__ void fft2(float2& a, float2& b) {
  const float2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

// Forward 4-point DFT, natural order in and out.
__device__ __forceinline__ void fft4(float2& x0, float2& x1, float2& x2, float2& x3) {
  const float2 s0 = cadd(x0, x2), d0 = csub(x0, x2);
  const float2 s1 = cadd(x1, x3), d1 = mul_mi(csub(x1, x3));
  x0 = cadd(s0, s1);
  x2 = csub(s0, s1);
  x1 = cadd(d0, d1);
  x3 = csub(d0, d1);
}

// Forward 8-point DFT (decimation in frequency), natural order in and out.
__device__ __forceinline__ void fft8(float2& a0, float2& a1, float2& a2, float2& a3, float2& a4, float2& a5,
                                     float2& a6, float2& a7) {
  constexpr float r2 = 0.70710678118654752440f;
  float2 b0 = cadd(a0, a4), b1 = cadd(a1, a5), b2 = cadd(a2, a6), b3 = cadd(a3, a7);
  float2 c0 = csub(a0, a4), c1 = csub(a1, a5), c2 = csub(a2, a6), c3 = csub(a3, a7);
  c1 = make_float2(r2 * (c1.x + c1.y), r2 * (c1.y - c1.x));     // * W8
  c2 = mul_mi(c2);                                             // * W8^2
  c3 = make_float2(r2 * (c3.y - c3.x), -r2 * (c3.x + c3.y));    // * W8^3
  fft4(b0, b1, b2, b3);
  fft4(c0, c1, c2, c3);
  a0 = b0; a1 = c0; a2 = b1; a3 = c1; a4 = b2; a5 = c2; a6 = b3; a7 = c3;
}

// One Stockham iteration's arithmetic (Govindaraju et al. formulation): for
// virtual thread j' = t + b*T, points v[b + r*B] = data[j' + r*L/R] are
// twiddled by W_{Ns R}^{r (j' mod Ns)} and transformed in place.
template <int L, int Ns, int R>
__device__ __forceinline__ void stage_compute(Vec& v, int t, const float2* __restrict__ twL) {
  constexpr int T = L / kPts, B = kPts / R;
#pragma unroll
  for (int b = 0; b < B; ++b) {
    if constexpr (Ns > 1) {
      const int jm = (t + b * T) & (Ns - 1);
      constexpr int scale = L / (Ns * R);
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const float2 w = twL[r * jm * scale];
#pragma unroll
        for (int c = 0; c < kCh; ++c) v[c][b + r * B] = cmul(v[c][b + r * B], w);
      }
    }
#pragma unroll
    for (int c = 0; c < kCh; ++c) {
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
template <int L, int Ns, int R>
__device__ __forceinline__ void exchange(Vec& v, float* __restrict__ lds, int t) {
  constexpr int T = L / kPts, B = kPts / R, CG = Cfg<L>::CG, PAD = Cfg<L>::PAD;
  float* re = lds;
  float* im = lds + CG * PAD;
#pragma unroll
  for (int g = 0; g < kCh; g += CG) {
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int j = t + b * T;
      const int base = (j / Ns) * Ns * R + (j & (Ns - 1));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int idx = lds_pad(base + r * Ns);
#pragma unroll
        for (int cc = 0; cc < CG; ++cc) {
          re[cc * PAD + idx] = v[g + cc][b + r * B].x;
          im[cc * PAD + idx] = v[g + cc][b + r * B].y;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPts; ++q) {
      const int idx = lds_pad(t + q * T);
#pragma unroll
      for (int cc = 0; cc < CG; ++cc) v[g + cc][q] = make_float2(re[cc * PAD + idx], im[cc * PAD + idx]);
    }
    __syncthreads();
  }
}

// Full forward DFT of length L on the 8 channels; input and output both in
// the pattern v[c][q] <-> element t + q*T.
template <int L, int Ns>
__device__ __forceinline__ void fft_stages(Vec& v, float* __restrict__ lds, int t, const float2* __restrict__ twL) {
  constexpr int R = (L / Ns >= 8) ? 8 : L / Ns;
  stage_compute<L, Ns, R>(v, t, twL);
  if constexpr (Ns * R < L) {
    exchange<L, Ns, R>(v, lds, t);
    fft_stages<L, Ns * R>(v, lds, t, twL);
  }
}

// Sixteen consecutive resampled samples x[p0 .. p0+15].  The read index
// drifts by < 1 sample per 16 for any physical acceleration, so they come
// from one 20-float window (five dword-aligned 16-byte loads); lanes where
// that does not hold (series edges, extreme drift) gather per sample.
__device__ __forceinline__ void load_resampled16(const float* __restrict__ in, uint64_t n, double af, double size,
                                                 uint64_t p0, float (&x)[16]) {
  uint32_t e[16];
  const uint64_t i0 = dev::accel_index_ii(af, size, p0, n - 1);
  const int64_t w0 = static_cast<int64_t>(i0) - 1;
  bool fast = (w0 >= 0) && (static_cast<uint64_t>(w0) + 20 <= n);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t idx = i == 0 ? i0 : dev::accel_index_ii(af, size, p0 + i, n - 1);
    e[i] = static_cast<uint32_t>(static_cast<int64_t>(idx) - (w0 + i));
    fast = fast && (e[i] <= 2u);
  }
  if (fast) {
    float w[20];
    const f4u* src = reinterpret_cast<const f4u*>(in + w0);
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const f4u q = src[u];
      w[4 * u] = q.x;
      w[4 * u + 1] = q.y;
      w[4 * u + 2] = q.z;
      w[4 * u + 3] = q.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = e[i] == 0 ? w[i] : (e[i] == 1 ? w[i + 1] : w[i + 2]);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = in[w0 + i + static_cast<int64_t>(static_cast<int32_t>(e[i]))];
  }
}

// Table layout (float2): [tw_N2 (N2)] [tw_N1 (N1)] [lo (2^kSplit)] [hi (M >> kSplit)]
struct TableOffsets {
  uint64_t n2, n1, lo, hi, total;
};
__host__ __device__ inline TableOffsets table_offsets(int N1, int N2) {
  const uint64_t M = static_cast<uint64_t>(N1) * N2;
  TableOffsets o;
  o.n2 = 0;
  o.n1 = o.n2 + N2;
  o.lo = o.n1 + N1;
  o.hi = o.lo + (1u << kSplit);
  o.total = o.hi + (M >> kSplit);
  return o;
}

__device__ __forceinline__ float2 twiddle_M(uint32_t a, const float2* __restrict__ lo, const float2* __restrict__ hi) {
  return cmul(hi[a >> kSplit], lo[a & ((1u << kSplit) - 1)]);
}

// Pass A.  grid.x = (N1/8) * K, trial fastest so the K workgroups of one
// column block run together and share the input window in L2.
template <int L>
__global__ void __launch_bounds__(Cfg<L>::T) fft4_colpass_kernel(const float* __restrict__ in, uint64_t n,
                                                                  const double* __restrict__ afs, int K,
                                                                  float2* __restrict__ Y, uint64_t ystride, int N1,
                                                                  const float2* __restrict__ tab) {
  __shared__ float lds[Cfg<L>::LDS_FLOATS];
  constexpr int T = Cfg<L>::T;
  const int t = threadIdx.x;
  const int k = blockIdx.x % K;
  const int i0 = (blockIdx.x / K) * kCh;
  const TableOffsets to = table_offsets(N1, L);
  const double af = afs[k];
  const double size = static_cast<double>(n);
  Vec v;
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    const uint64_t j = t + q * T;
    float x[16];
    load_resampled16(in, n, af, size, 2 * (static_cast<uint64_t>(N1) * j + i0), x);
#pragma unroll
    for (int c = 0; c < kCh; ++c) v[c][q] = make_float2(x[2 * c], x[2 * c + 1]);
  }
  fft_stages<L, 1>(v, lds, t, tab + to.n2);
  const uint32_t mask = static_cast<uint32_t>(N1) * L - 1;
  float2* y = Y + static_cast<uint64_t>(k) * ystride + i0;
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    const uint32_t k2 = t + q * T;
    float2 w = twiddle_M((static_cast<uint32_t>(i0) * k2) & mask, tab + to.lo, tab + to.hi);
    const float2 step = twiddle_M(k2, tab + to.lo, tab + to.hi);
#pragma unroll
    for (int c = 0; c < kCh; ++c) {
      v[c][q] = cmul(v[c][q], w);
      w = cmul(w, step);
    }
    float4* dst = reinterpret_cast<float4*>(y + static_cast<uint64_t>(k2) * N1);
#pragma unroll
    for (int c = 0; c < kCh; c += 2) dst[c / 2] = make_float4(v[c][q].x, v[c][q].y, v[c + 1][q].x, v[c + 1][q].y);
  }
}

// Pass B.  grid.x = (N2/8) * K.
template <int L>
__global__ void __launch_bounds__(Cfg<L>::T) fft4_rowpass_kernel(const float2* __restrict__ Y, uint64_t ystride,
                                                                  float2* __restrict__ X, uint64_t xstride, int K,
                                                                  int N2, const float2* __restrict__ tab) {
  __shared__ float lds[Cfg<L>::LDS_FLOATS];
  constexpr int T = Cfg<L>::T;
  const int t = threadIdx.x;
  const int k = blockIdx.x % K;
  const int r0 = (blockIdx.x / K) * kCh;
  const TableOffsets to = table_offsets(L, N2);
  const float2* y = Y + static_cast<uint64_t>(k) * ystride + static_cast<uint64_t>(r0) * L;
  Vec v;
#pragma unroll
  for (int c = 0; c < kCh; ++c)
#pragma unroll
    for (int q = 0; q < kPts; ++q) v[c][q] = y[static_cast<uint64_t>(c) * L + t + q * T];
  fft_stages<L, 1>(v, lds, t, tab + to.n1);
  float2* x = X + static_cast<uint64_t>(k) * xstride + r0;
#pragma unroll
  for (int q = 0; q < kPts; ++q) {
    const uint64_t k1 = t + q * T;
    float4* dst = reinterpret_cast<float4*>(x + k1 * N2);
#pragma unroll
    for (int c = 0; c < kCh; c += 2) dst[c / 2] = make_float4(v[c][q].x, v[c][q].y, v[c + 1][q].x, v[c + 1][q].y);
  }
}

bool supported_len(int L) { return L >= 128 && L <= 4096 && (L & (L - 1)) == 0; }

}  // namespace

bool fft4_factor(uint64_t M, int* N1, int* N2) {
  if (M == 0 || (M & (M - 1)) != 0) return false;
  int lg = 0;
  while ((uint64_t(1) << lg) < M) ++lg;
  const int a = lg / 2, b = lg - a;  // N2 = 2^a <= N1 = 2^b
  if (!supported_len(1 << a) || !supported_len(1 << b)) return false;
  if (N1) *N1 = 1 << b;
  if (N2) *N2 = 1 << a;
  return true;
}

std::vector<float2> fft4_tables(int N1, int N2) {
  const TableOffsets o = table_offsets(N1, N2);
  const double M = static_cast<double>(N1) * N2;
  std::vector<float2> t(o.total);
  auto w = [](double num, double den) {
    const double a = -2.0 * M_PI * num / den;
    return make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a)));
  };
  for (int m = 0; m < N2; ++m) t[o.n2 + m] = w(m, N2);
  for (int m = 0; m < N1; ++m) t[o.n1 + m] = w(m, N1);
  for (uint64_t m = 0; m < (1u << kSplit); ++m) t[o.lo + m] = w(static_cast<double>(m), M);
  for (uint64_t m = 0; m < (o.total - o.hi); ++m) t[o.hi + m] = w(static_cast<double>(m << kSplit), M);
  return t;
}

void fft4_resample_colpass(const float* in, uint64_t n, const double* af, int K, float2* Y, uint64_t ystride, int N1,
                           int N2, const float2* tables, hipStream_t s) {
  PSOUP_CHECK(K >= 1 && n == 2ull * N1 * N2 && supported_len(N1) && supported_len(N2),
              "fft4 colpass: bad geometry n=" << n << " N1=" << N1 << " N2=" << N2 << " K=" << K);
  PSOUP_CHECK(ystride % 8 == 0 && ystride >= static_cast<uint64_t>(N1) * N2 &&
                  (reinterpret_cast<uintptr_t>(Y) & 63) == 0,
              "fft4 colpass: Y alignment/stride");
  const uint64_t nblocks = static_cast<uint64_t>(N1 / kCh) * K;
  PSOUP_CHECK(nblocks < (1ull << 31), "fft4 colpass: grid too large");
  const dim3 grid(static_cast<unsigned>(nblocks));
  switch (N2) {
    case 128: fft4_colpass_kernel<128><<<grid, Cfg<128>::T, 0, s>>>(in, n, af, K, Y, ystride, N1, tables); break;
    case 256: fft4_colpass_kernel<256><<<grid, Cfg<256>::T, 0, s>>>(in, n, af, K, Y, ystride, N1, tables); break;
    case 512: fft4_colpass_kernel<512><<<grid, Cfg<512>::T, 0, s>>>(in, n, af, K, Y, ystride, N1, tables); break;
    case 1024: fft4_colpass_kernel<1024><<<grid, Cfg<1024>::T, 0, s>>>(in, n, af, K, Y, ystride, N1, tables); break;
    case 2048: fft4_colpass_kernel<2048><<<grid, Cfg<2048>::T, 0, s>>>(in, n, af, K, Y, ystride, N1, tables); break;
    default: fft4_colpass_kernel<4096><<<grid, Cfg<4096>::T, 0, s>>>(in, n, af, K, Y, ystride, N1, tables); break;
  }
  post_launch_check("fft4_colpass_kernel", s);
}

void fft4_rowpass(const float2* Y, uint64_t ystride, float2* X, uint64_t xstride, int K, int N1, int N2,
                  const float2* tables, hipStream_t s) {
  PSOUP_CHECK(K >= 1 && supported_len(N1) && supported_len(N2), "fft4 rowpass: bad geometry");
  PSOUP_CHECK(xstride % 8 == 0 && xstride >= static_cast<uint64_t>(N1) * N2 &&
                  (reinterpret_cast<uintptr_t>(X) & 63) == 0,
              "fft4 rowpass: X alignment/stride");
  const dim3 grid(static_cast<unsigned>(static_cast<uint64_t>(N2 / kCh) * K));
  switch (N1) {
    case 128: fft4_rowpass_kernel<128><<<grid, Cfg<128>::T, 0, s>>>(Y, ystride, X, xstride, K, N2, tables); break;
    case 256: fft4_rowpass_kernel<256><<<grid, Cfg<256>::T, 0, s>>>(Y, ystride, X, xstride, K, N2, tables); break;
    case 512: fft4_rowpass_kernel<512><<<grid, Cfg<512>::T, 0, s>>>(Y, ystride, X, xstride, K, N2, tables); break;
    case 1024: fft4_rowpass_kernel<1024><<<grid, Cfg<1024>::T, 0, s>>>(Y, ystride, X, xstride, K, N2, tables); break;
    case 2048: fft4_rowpass_kernel<2048><<<grid, Cfg<2048>::T, 0, s>>>(Y, ystride, X, xstride, K, N2, tables); break;
    default: fft4_rowpass_kernel<4096><<<grid, Cfg<4096>::T, 0, s>>>(Y, ystride, X, xstride, K, N2, tables); break;
  }
  post_launch_check("fft4_rowpass_kernel", s);
}

}  // namespace kern
}  // namespace psoup
