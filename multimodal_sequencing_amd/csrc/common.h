// Shared device helpers for the mmseq HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmseq.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

#define MMSEQ_LDS __attribute__((address_space(3)))

// --- bf16 <-> f32 (round-to-nearest-even; NaN kept NaN via the hardware cvt) ---
__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(unsigned short, b);
}

// Generic element load/store for the two storage types used on the path.
template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct Elem<unsigned short> {
  static __device__ __forceinline__ float ld(const unsigned short* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(unsigned short* p, float v) { *p = f2bf(v); }
};

// 4 contiguous elements <-> f32x4 (8-byte bf16 / 16-byte f32 accesses; caller guarantees alignment)
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static __device__ __forceinline__ f32x4 ld(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  static __device__ __forceinline__ void st(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
};
template <> struct Vec4<unsigned short> {
  static __device__ __forceinline__ f32x4 ld(const unsigned short* p) {
    u16x4 u = *reinterpret_cast<const u16x4*>(p);
    return (f32x4){bf2f(u[0]), bf2f(u[1]), bf2f(u[2]), bf2f(u[3])};
  }
  static __device__ __forceinline__ void st(unsigned short* p, f32x4 v) {
    u16x4 u = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    *reinterpret_cast<u16x4*>(p) = u;
  }
};

// --- wave64 reductions ---
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// --- activations (reference sites in include/mmseq.h) ---
__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case MMSEQ_ACT_GELU_ERF: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
    case MMSEQ_ACT_QUICKGELU: return x / (1.0f + __expf(-1.702f * x));
    case MMSEQ_ACT_TANH: return tanhf(x);
    case MMSEQ_ACT_GELU_TANH: {
      const float k = 0.79788456080286536f;  // sqrt(2/pi)
      return 0.5f * x * (1.0f + tanhf(k * (x + 0.044715f * x * x * x)));
    }
    default: return x;
  }
}
// d act / dx evaluated at the pre-activation x
__device__ __forceinline__ float act_bwd(int act, float x) {
  switch (act) {
    case MMSEQ_ACT_GELU_ERF: {
      float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
      float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
      return cdf + x * pdf;
    }
    case MMSEQ_ACT_QUICKGELU: {
      float s = 1.0f / (1.0f + __expf(-1.702f * x));
      return s + 1.702f * x * s * (1.0f - s);
    }
    case MMSEQ_ACT_TANH: {
      float t = tanhf(x);
      return 1.0f - t * t;
    }
    case MMSEQ_ACT_GELU_TANH: {
      const float k = 0.79788456080286536f;
      float u = k * (x + 0.044715f * x * x * x);
      float t = tanhf(u);
      return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k * (1.0f + 3.0f * 0.044715f * x * x);
    }
    default: return 1.0f;
  }
}

// --- fast activations for the bf16 GEMM epilogues (no divergent libm branches) ---------------
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16 resolution); the
// exp(-x^2) term is shared with the GELU derivative's pdf.
__device__ __forceinline__ void erf_and_gauss(float x, float& erf_x, float& e) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  e = __expf(-ax * ax);
  erf_x = copysignf(fmaf(-poly, e, 1.0f), x);
}
__device__ __forceinline__ float act_fwd_fast(int act, float x) {
  if (act == MMSEQ_ACT_GELU_ERF) {
    float er, e;
    erf_and_gauss(x * 0.70710678118654752f, er, e);
    return 0.5f * x * (1.0f + er);
  }
  if (act == MMSEQ_ACT_QUICKGELU) return x * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x));
  return act_fwd(act, x);
}
__device__ __forceinline__ float act_bwd_fast(int act, float x) {
  if (act == MMSEQ_ACT_GELU_ERF) {
    float er, e;  // e = exp(-x^2 / 2)
    erf_and_gauss(x * 0.70710678118654752f, er, e);
    return fmaf(0.39894228040143268f * x, e, 0.5f * (1.0f + er));
  }
  if (act == MMSEQ_ACT_QUICKGELU) {
    const float s = __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x));
    return s + 1.702f * x * s * (1.0f - s);
  }
  return act_bwd(act, x);
}

// GELU (erf form) for the bf16 GEMM epilogues without transcendentals: GELU(x) - x/2 and
// GELU'(x) - 1/2 are odd, so both are x * P(u) with u = 2 x^2 / 25 - 1 for x clamped to [-5, 5]
// and P a degree-12 Chebyshev fit (power basis in u). Max abs error over all x, evaluated in fp32:
// 7.6e-6 (GELU), 2.5e-5 (GELU'); the bf16 quantum near 1 is 3.9e-3. Evaluated on element pairs so
// the Horner chain issues as packed v_pk_fma_f32.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_poly_pair(f32x2 x, const float (&c)[13], f32x2& xc) {
  xc = (f32x2){__builtin_amdgcn_fmed3f(x[0], -5.f, 5.f), __builtin_amdgcn_fmed3f(x[1], -5.f, 5.f)};
  const f32x2 u = __builtin_elementwise_fma(xc * xc, (f32x2){0.08f, 0.08f}, (f32x2){-1.f, -1.f});
  f32x2 p = (f32x2){c[12], c[12]};
#pragma unroll
  for (int k = 11; k >= 0; --k) p = __builtin_elementwise_fma(p, u, (f32x2){c[k], c[k]});
  return __builtin_elementwise_fma(xc, p, (f32x2){0.5f, 0.5f});  // Phi(x) resp. GELU'(x)
}
// GELU (erf form) in the forward bf16 epilogues, cheaper than the degree-12 Horner chain: Phi(x)
// as a logistic of an odd quintic, GELU(x) ~= x * sigmoid(x (c0 + c1 x^2 + c2 x^4)) with x clamped
// to [-9, 9] inside the polynomial (its fitted range; Phi(9) = 1 - 1e-19). Minimax fit of the GELU
// error over all x: max abs error 2.5e-5 (the bf16 quantum near 1 is 3.9e-3). Cost per element:
// med3 + 4 FMA-class + exp2 + rcp (the Horner form: 14 packed FMAs per PAIR, 8-cycle issue each).
__device__ __forceinline__ float gelu_sig(float x) {
  constexpr float L2E = 1.4426950408889634f;
  constexpr float K0 = -1.59501577f * L2E, K1 = -7.40112921e-2f * L2E, K2 = 7.03033584e-4f * L2E;
  const float xc = __builtin_amdgcn_fmed3f(x, -9.f, 9.f);
  const float x2 = xc * xc;
  const float q = xc * fmaf(x2, fmaf(x2, K2, K1), K0);  // -log2(e) * x (c0 + c1 x^2 + c2 x^4)
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(q));
}
// gelu_sig on 8 values as packed fp32 pairs (v_pk_mul / v_pk_fma / v_pk_add_f32: the same fp32
// operations in the same order, so bit-identical to gelu_sig per element): for the GEMM epilogues,
// where no MFMA runs beside them (beside MFMAs packed fp32 costs more than two scalar ops,
// MI355X_MICROARCH.md, which is why the rest of the library builds with -fno-slp-vectorize)
__device__ __forceinline__ void gelu_sig8(float* v) {
  constexpr float L2E = 1.4426950408889634f;
  constexpr float K0 = -1.59501577f * L2E, K1 = -7.40112921e-2f * L2E, K2 = 7.03033584e-4f * L2E;
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    const f32x2 x = {v[r], v[r + 1]};
    const f32x2 xc = {__builtin_amdgcn_fmed3f(x[0], -9.f, 9.f), __builtin_amdgcn_fmed3f(x[1], -9.f, 9.f)};
    const f32x2 x2 = xc * xc;
    const f32x2 t = __builtin_elementwise_fma(x2, __builtin_elementwise_fma(x2, (f32x2){K2, K2}, (f32x2){K1, K1}),
                                              (f32x2){K0, K0});
    const f32x2 q = xc * t;
    const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(q[0]), __builtin_amdgcn_exp2f(q[1])} + (f32x2){1.0f, 1.0f};
    const f32x2 y = x * (f32x2){__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    v[r] = y[0];
    v[r + 1] = y[1];
  }
}
// bias + alpha for 8 accumulators as packed pairs: v = acc * alpha + bias (fmaf per element)
__device__ __forceinline__ void bias_alpha8(float* v, const f32x4& lo, const f32x4& hi, float alpha,
                                            const f32x4& b0, const f32x4& b1) {
  const f32x2 al = {alpha, alpha};
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    const f32x2 a = __builtin_elementwise_fma((f32x2){lo[r], lo[r + 1]}, al, (f32x2){b0[r], b0[r + 1]});
    const f32x2 c = __builtin_elementwise_fma((f32x2){hi[r], hi[r + 1]}, al, (f32x2){b1[r], b1[r + 1]});
    v[r] = a[0]; v[r + 1] = a[1];
    v[4 + r] = c[0]; v[4 + r + 1] = c[1];
  }
}
// derivative of gelu_sig's function (the backward of the forward actually computed): s + x s (1 - s)
// p'(x), p' = c0 + 3 c1 x^2 + 5 c2 x^4; max abs error vs the exact GELU' 1.1e-4
__device__ __forceinline__ float gelu_sig_grad(float x) {
  constexpr float L2E = 1.4426950408889634f;
  constexpr float C0 = 1.59501577f, C1 = 7.40112921e-2f, C2 = -7.03033584e-4f;
  const float xc = __builtin_amdgcn_fmed3f(x, -9.f, 9.f);
  const float x2 = xc * xc;
  const float q = xc * fmaf(x2, fmaf(x2, -C2 * L2E, -C1 * L2E), -C0 * L2E);
  const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(q));
  const float dp = fmaf(x2, fmaf(x2, 5.f * C2, 3.f * C1), C0);
  return fmaf(xc * fmaf(-sg, sg, sg), dp, sg);
}
__device__ __forceinline__ f32x2 gelu_bwd_pair(f32x2 x) {
  constexpr float c[13] = {1.421341449e-01f, -7.509786636e-02f, 6.654060632e-02f, -7.212746888e-02f,
                           8.076252043e-02f, -8.158523589e-02f, 7.798881084e-02f, -7.819437981e-02f,
                           5.708414689e-02f, -1.684123091e-02f, 1.213573292e-02f, -2.509075962e-02f,
                           1.229602005e-02f};
  f32x2 xc;
  return gelu_poly_pair(x, c, xc);
}

// --- dropout: counter-based mask (no stored masks; fwd and bwd regenerate the same bits) ---
// One 32-bit hash per element QUAD (idx >> 2) decides its four elements: elements 4q and 4q + 1
// use the low / high 16-bit half of h = lowbias32(key mix of q), elements 4q + 2 and 4q + 3 the
// halves of h2 = m ^ (m >> 16), m = h * 0x9E3779B1 (one multiply); an element is dropped iff its
// half < round(p * 2^16). The per-call key is derived on the host from (seed, stream) by
// splitmix64, so streams and seeds are independent. (Until round 4: one lowbias32 per element
// PAIR; the quad form halves the hashing with the same 16-bit threshold resolution. Rate, field
// and lag independence measured in DESIGN §4.2.)
struct Drop {
  uint32_t thr;     // drop iff half < thr; thr == 0 -> disabled
  uint32_t k0, k1;  // per-call key
  float scale;      // 1 / (1 - p)
};
__host__ inline uint64_t drop_splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__host__ inline Drop make_drop(const mmseq_dropout* d) {
  Drop r;
  r.thr = 0; r.k0 = 0; r.k1 = 0; r.scale = 1.f;
  if (d && d->p > 0.f) {
    uint32_t t = (uint32_t)(d->p * 65536.0f + 0.5f);
    r.thr = t < 1u ? 1u : t;
    const uint64_t key = drop_splitmix64(d->seed ^ drop_splitmix64(0x5bd1e995ull + d->stream));
    r.k0 = (uint32_t)key;
    r.k1 = (uint32_t)(key >> 32) | 1u;
    r.scale = 1.0f / (1.0f - d->p);
  }
  return r;
}
__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {  // Wellons' lowbias32
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// h of element quad `quad`
__device__ __forceinline__ uint32_t drop_hash(const Drop& d, uint64_t quad) {
  // high word enters by xor + add (no multiply: quad indices here stay below 2^32, and the
  // lowbias32 rounds provide the diffusion)
  return drop_mix(((uint32_t)quad ^ d.k0) + ((uint32_t)(quad >> 32) ^ d.k1));
}
// h2: the quad's second 32 bits (elements 4q + 2, 4q + 3)
__device__ __forceinline__ uint32_t drop_hash2(uint32_t h) {
  const uint32_t m = h * 0x9E3779B1u;
  return m ^ (m >> 16);
}
__device__ __forceinline__ float drop_sel(const Drop& d, uint32_t h, int hi) {
  const uint32_t u = hi ? (h >> 16) : (h & 0xFFFFu);
  return u < d.thr ? 0.f : d.scale;
}
// multiplier for element idx: 0 (dropped) or 1/(1-p); 1 when disabled
__device__ __forceinline__ float drop_mul(const Drop& d, uint64_t idx) {
  if (d.thr == 0) return 1.f;
  const uint32_t h = drop_hash(d, idx >> 2);
  return drop_sel(d, (idx & 2) ? drop_hash2(h) : h, (int)(idx & 1));
}
// multipliers for elements idx .. idx + 2n - 1 with idx EVEN (one hash per quad when idx % 4 == 0)
template <int NPAIR>
__device__ __forceinline__ void drop_mul_pairs(const Drop& d, uint64_t idx, float* m) {
  if ((NPAIR % 2) == 0 && (idx & 3) == 0) {
#pragma unroll
    for (int q = 0; q < NPAIR / 2; ++q) {
      const uint32_t h = drop_hash(d, (idx >> 2) + q), h2 = drop_hash2(h);
      m[4 * q] = drop_sel(d, h, 0);
      m[4 * q + 1] = drop_sel(d, h, 1);
      m[4 * q + 2] = drop_sel(d, h2, 0);
      m[4 * q + 3] = drop_sel(d, h2, 1);
    }
  } else {
#pragma unroll
    for (int q = 0; q < NPAIR; ++q) {
      const uint64_t j = (idx >> 1) + q;  // element pair j = elements 2j, 2j + 1
      const uint32_t h = drop_hash(d, j >> 1);
      const uint32_t w = (j & 1) ? drop_hash2(h) : h;
      m[2 * q] = drop_sel(d, w, 0);
      m[2 * q + 1] = drop_sel(d, w, 1);
    }
  }
}
// multipliers for the 4 elements idx .. idx + 3 (one hash when idx % 4 == 0)
__device__ __forceinline__ void drop_mul4(const Drop& d, uint64_t idx, float* m) {
  if (d.thr == 0) {
    m[0] = m[1] = m[2] = m[3] = 1.f;
  } else if ((idx & 1) == 0) {
    drop_mul_pairs<2>(d, idx, m);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = drop_mul(d, idx + e);
  }
}

// status plumbing shared by the ABI wrappers
mmseq_status mmseq_set_error(mmseq_status code, const char* fmt, ...);
mmseq_status mmseq_check_launch(const char* what);

#define MMSEQ_REQUIRE(cond, ...) \
  do { if (!(cond)) return mmseq_set_error(MMSEQ_EINVAL, __VA_ARGS__); } while (0)
