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

// --- dropout: counter-based mask (no stored masks; fwd and bwd regenerate the same bits) ---
struct Drop {
  uint32_t thr;     // drop iff (hash >> 8) < thr   (thr = p * 2^24); thr == 0 -> disabled
  uint32_t stream;
  uint64_t seed;
  float scale;      // 1 / (1 - p)
};
__host__ inline Drop make_drop(const mmseq_dropout* d) {
  Drop r;
  r.thr = 0; r.stream = 0; r.seed = 0; r.scale = 1.f;
  if (d && d->p > 0.f) {
    r.thr = (uint32_t)(d->p * 16777216.0f);
    r.stream = d->stream;
    r.seed = d->seed;
    r.scale = 1.0f / (1.0f - d->p);
  }
  return r;
}
__device__ __forceinline__ uint32_t drop_hash(const Drop& d, uint64_t idx) {
  uint32_t h = (uint32_t)idx ^ ((uint32_t)(idx >> 32) * 0x9e3779b1u) ^ (uint32_t)d.seed ^
               (d.stream * 0x85ebca77u);
  h *= 0xcc9e2d51u;
  h ^= (uint32_t)(d.seed >> 32) + 0x27d4eb2fu;
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;  // fmix32
  return h;
}
// multiplier for element idx: 0 (dropped) or 1/(1-p); 1 when disabled
__device__ __forceinline__ float drop_mul(const Drop& d, uint64_t idx) {
  if (d.thr == 0) return 1.f;
  return (drop_hash(d, idx) >> 8) < d.thr ? 0.f : d.scale;
}

// status plumbing shared by the ABI wrappers
mmseq_status mmseq_set_error(mmseq_status code, const char* fmt, ...);
mmseq_status mmseq_check_launch(const char* what);

#define MMSEQ_REQUIRE(cond, ...) \
  do { if (!(cond)) return mmseq_set_error(MMSEQ_EINVAL, __VA_ARGS__); } while (0)
