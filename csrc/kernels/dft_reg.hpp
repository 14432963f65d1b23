// In-register complex DFT building blocks shared by the four-step FFT passes
// (fft4step.hip) and the fold optimiser (fold.hip): complex arithmetic on
// the packed-f32 VALU (cplx_pk.hpp), 2/4/8-point butterflies and dft<N>, a compile-time
// unrolled radix-8 DFT of up to 64 points whose twiddles are literals.
#pragma once

#include <hip/hip_runtime.h>

#include "cplx_pk.hpp"

namespace psoup {
namespace kern {
namespace dreg {

__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // * -i

// The butterflies and twiddle products run on the packed-f32 VALU
// (cplx_pk.hpp: half the VALU issue slots of the scalar forms).
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return pk::add(a, b); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return pk::sub(a, b); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return pk::mul(a, b); }
__device__ __forceinline__ float2 cadd_mi(float2 a, float2 b) { return pk::add_mi(a, b); }
__device__ __forceinline__ float2 csub_mi(float2 a, float2 b) { return pk::sub_mi(a, b); }
__device__ __forceinline__ float2 mul_w8(float2 c) { return pk::mul_w8(c); }
__device__ __forceinline__ float2 mul_w83(float2 c) { return pk::mul_w83(c); }

__device__ __forceinline__ void fft2(float2& a, float2& b) {
  const float2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

// Forward 4-point DFT, natural order in and out.
__device__ __forceinline__ void fft4(float2& x0, float2& x1, float2& x2, float2& x3) {
  const float2 s0 = cadd(x0, x2), d0 = csub(x0, x2);
  const float2 s1 = cadd(x1, x3), e1 = csub(x1, x3);
  x0 = cadd(s0, s1);
  x2 = csub(s0, s1);
  x1 = cadd_mi(d0, e1);  // d0 + (-i) e1
  x3 = csub_mi(d0, e1);
}

// Forward 8-point DFT (decimation in frequency), natural order in and out.
__device__ __forceinline__ void fft8(float2& a0, float2& a1, float2& a2, float2& a3, float2& a4, float2& a5,
                                     float2& a6, float2& a7) {
  float2 b0 = cadd(a0, a4), b1 = cadd(a1, a5), b2 = cadd(a2, a6), b3 = cadd(a3, a7);
  float2 c0 = csub(a0, a4), c1 = csub(a1, a5), c2 = csub(a2, a6), c3 = csub(a3, a7);
  c1 = mul_w8(c1);    // * W8
  c2 = mul_mi(c2);    // * W8^2
  c3 = mul_w83(c3);   // * W8^3
  fft4(b0, b1, b2, b3);
  fft4(c0, c1, c2, c3);
  a0 = b0; a1 = c0; a2 = b1; a3 = c1; a4 = b2; a5 = c2; a6 = b3; a7 = c3;
}

// compile-time twiddles: W_N^e = exp(-2 pi i e / N), octant-reduced Taylor series in double
struct ccf {
  float x, y;
};
constexpr double ct_sin(double x) {  // |x| <= pi/4
  double term = x, sum = x;
  for (int i = 1; i < 12; ++i) {
    term *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
    sum += term;
  }
  return sum;
}
constexpr double ct_cos(double x) {
  double term = 1.0, sum = 1.0;
  for (int i = 1; i < 12; ++i) {
    term *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
    sum += term;
  }
  return sum;
}
constexpr ccf wconst(int N, int e) {
  e = ((e % N) + N) % N;
  const int q = (4 * e) / N, rem = e - q * (N / 4);  // angle = q quarter turns + 2 pi rem / N
  constexpr double kTwoPi = 6.28318530717958647692;
  double c = 0.0, s = 0.0;
  if (8 * rem <= N) {
    const double th = kTwoPi * rem / N;
    c = ct_cos(th);
    s = ct_sin(th);
  } else {
    const double th = kTwoPi * (N / 4 - rem) / N;
    c = ct_sin(th);
    s = ct_cos(th);
  }
  double cq = c, sq = s;  // rotate by q quarter turns
  if (q == 1) { cq = -s; sq = c; }
  if (q == 2) { cq = -c; sq = -s; }
  if (q == 3) { cq = s; sq = -c; }
  return ccf{static_cast<float>(cq), static_cast<float>(-sq)};
}

template <int I>
struct ic {
  static constexpr int value = I;
};
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(ic<B>{});
    sfor<B + 1, E>(static_cast<F&&>(f));
  }
}

// v * W_N^E (compile-time exponent; trivial factors without multiplications)
template <int N, int E>
__device__ __forceinline__ float2 twc(float2 v) {
  constexpr int e = ((E % N) + N) % N;
  if constexpr (e == 0) {
    return v;
  } else if constexpr (2 * e == N) {
    return make_float2(-v.x, -v.y);
  } else if constexpr (4 * e == N) {
    return mul_mi(v);
  } else if constexpr (4 * e == 3 * N) {
    return make_float2(-v.y, v.x);
  } else if constexpr (8 * e == N) {
    return mul_w8(v);
  } else if constexpr (8 * e == 3 * N) {
    return mul_w83(v);
  } else {
    constexpr ccf w = wconst(N, e);
    return cmul(v, make_float2(w.x, w.y));
  }
}

// In-register forward DFT of length N (power of two <= 64), natural order in
// and out: N = 8 B, n = B a + b, k = ka + 8 kb.
template <int N>
__device__ __forceinline__ void dft(float2 (&x)[N]) {
  if constexpr (N == 2) {
    fft2(x[0], x[1]);
  } else if constexpr (N == 4) {
    fft4(x[0], x[1], x[2], x[3]);
  } else if constexpr (N == 8) {
    fft8(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
  } else {
    constexpr int A = 8, B = N / 8;
    float2 y[N];
    sfor<0, B>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      float2 t[A];
      sfor<0, A>([&](auto ac) { t[decltype(ac)::value] = x[B * decltype(ac)::value + b]; });
      dft<A>(t);
      sfor<0, A>([&](auto kc) {
        constexpr int ka = decltype(kc)::value;
        y[b * A + ka] = twc<N, b * ka>(t[ka]);
      });
    });
    sfor<0, A>([&](auto kc) {
      constexpr int ka = decltype(kc)::value;
      float2 t[B];
      sfor<0, B>([&](auto bc) { t[decltype(bc)::value] = y[decltype(bc)::value * A + ka]; });
      dft<B>(t);
      sfor<0, B>([&](auto jc) { x[ka + A * decltype(jc)::value] = t[decltype(jc)::value]; });
    });
  }
}

// Inverse DFT without the 1/N scale: conj(DFT(conj(x))).
template <int N>
__device__ __forceinline__ void idft(float2 (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) x[i].y = -x[i].y;
  dft<N>(x);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i].y = -x[i].y;
}

}  // namespace dreg
}  // namespace kern
}  // namespace psoup
