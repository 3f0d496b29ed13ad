// LayerNorm forward / backward with fp32 statistics (one wave64 per row, shuffle reductions).
// Reference sites: lxrt/modeling.py:353,432,486,577 (BertLayerNorm eps 1e-12);
// clip/model.py:190-196 (fp32 LayerNorm, eps 1e-5); berson/encoder.py:16,42, neural.py:25 (1e-6).
// Rows are addressed through mmseq_rows (two-level strides) so the kernels can read / write the
// text or the visual half of the joint [P][T][H] activation in place (the fused concat).
// Lane l owns columns j*256 + 4l .. +3 (j < 4): 8-byte (bf16) / 16-byte (f32) accesses when the
// row layout allows it (VEC), scalar otherwise; cols <= 256 * MJ (MJ = 4 up to 1024 columns, 8 up
// to 2048: the 2H-wide MRM head LayerNorm of the pretraining path).
#include "common.h"

namespace {

constexpr int RPB = 128;  // rows per workgroup in bwd (dgamma/dbeta partial granularity)

// 32-bit division (rows < 2^31): a 64-bit divide is a ~100-instruction branchy subroutine
__device__ __forceinline__ int64_t row_off(const mmseq_rows& l, int64_t r) {
  const uint32_t rr = (uint32_t)r, rpb = (uint32_t)l.rpb;
  const uint32_t q = rr / rpb, rem = rr - q * rpb;
  return (int64_t)q * l.bstride + (int64_t)rem * l.ld;
}

template <typename T, bool VEC>
__device__ __forceinline__ f32x4 ld4(const T* p, int c, int cols) {
  if (VEC) {
    if (c < cols) return Vec4<T>::ld(p + c);
    return (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = c + e < cols ? Elem<T>::ld(p + c + e) : 0.f;
  return v;
}
template <typename T, bool VEC>
__device__ __forceinline__ void st4(T* p, int c, int cols, f32x4 v) {
  if (VEC) {
    if (c < cols) Vec4<T>::st(p + c, v);
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (c + e < cols) Elem<T>::st(p + c + e, v[e]);
}
__device__ __forceinline__ f32x4 ldp(const float* p, int c, int cols) {
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = c + e < cols ? p[c + e] : 0.f;
  return v;
}

template <typename TX, typename TY, bool VEC, int MAXJ>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int cols, const TX* __restrict__ x,
                                                     mmseq_rows xl, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     TY* __restrict__ y, mmseq_rows yl,
                                                     float* __restrict__ mean,
                                                     float* __restrict__ rstd, Drop dy_) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const TX* xr = x + row_off(xl, r);
  f32x4 v[MAXJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    v[j] = ld4<TX, VEC>(xr, j * 256 + lane * 4, cols);
    s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  const float mu = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float d = (j * 256 + lane * 4 + e < cols) ? v[j][e] - mu : 0.f;
      q += d * d;
    }
  const float rs = rsqrtf(wave_sum(q) / cols + eps);
  TY* yr = y + row_off(yl, r);
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = j * 256 + lane * 4;
    if (c >= cols) continue;
    f32x4 g = ldp(gamma, c, cols), b = ldp(beta, c, cols), o;
    float dm[4];
    drop_mul4(dy_, (uint64_t)r * cols + c, dm);
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = ((v[j][e] - mu) * rs * g[e] + b[e]) * dm[e];
    st4<TY, VEC>(yr, c, cols, o);
  }
  if (lane == 0) {
    if (mean) mean[r] = mu;
    if (rstd) rstd[r] = rs;
  }
}

// dx = rstd * (g*dy - mean_c(g*dy) - xhat * mean_c(g*dy*xhat)) (+ dres)
// per-block partial dgamma / dbeta -> ws[block][2][cols]
template <typename T, bool VEC, int MAXJ>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int cols, const T* __restrict__ dy,
                                                     mmseq_rows dyl, const T* __restrict__ x,
                                                     mmseq_rows xl, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma,
                                                     T* __restrict__ dx, mmseq_rows dxl,
                                                     const T* __restrict__ dres, mmseq_rows dresl,
                                                     float* __restrict__ ws, Drop din,
                                                     T* __restrict__ dxd, mmseq_rows dxdl, Drop dout) {
  __shared__ float red[4][2][256 * MAXJ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 pg[MAXJ], pb[MAXJ], gm[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    pg[j] = pb[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    gm[j] = ldp(gamma, j * 256 + lane * 4, cols);
  }
  const int64_t rbeg = (int64_t)blockIdx.x * RPB;
  for (int64_t r = rbeg + wave; r < rbeg + RPB && r < rows; r += 4) {
    const T* xr = x + row_off(xl, r);
    const T* dyr = dy + row_off(dyl, r);
    const float mu = mean[r], rs = rstd[r];
    f32x4 xh[MAXJ], gdy[MAXJ];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = j * 256 + lane * 4;
      f32x4 xv = ld4<T, VEC>(xr, c, cols), d = ld4<T, VEC>(dyr, c, cols);
      if (din.thr) {
        float dm[4];
        drop_mul4(din, (uint64_t)r * cols + c, dm);
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] *= dm[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool in = c + e < cols;
        float xn = in ? (xv[e] - mu) * rs : 0.f;
        xh[j][e] = xn;
        gdy[j][e] = d[e] * gm[j][e];
        pg[j][e] += d[e] * xn;
        pb[j][e] += d[e];
        s1 += gdy[j][e];
        s2 += gdy[j][e] * xn;
      }
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
    T* dxr = dx + row_off(dxl, r);
    const T* drr = dres ? dres + row_off(dresl, r) : nullptr;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = j * 256 + lane * 4;
      if (c >= cols) continue;
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = rs * (gdy[j][e] - s1 - xh[j][e] * s2);
      if (dxd) {
        f32x4 od;
        float dm[4];
        drop_mul4(dout, (uint64_t)r * cols + c, dm);
#pragma unroll
        for (int e = 0; e < 4; ++e) od[e] = o[e] * dm[e];
        st4<T, VEC>(dxd + row_off(dxdl, r), c, cols, od);
      }
      if (drr) {
        f32x4 dr = ld4<T, VEC>(drr, c, cols);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += dr[e];
      }
      st4<T, VEC>(dxr, c, cols, o);
    }
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = j * 256 + lane * 4 + e;
      if (c < cols) {
        red[wave][0][c] = pg[j][e];
        red[wave][1][c] = pb[j][e];
      }
    }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    float g = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    float b = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    ws[((int64_t)blockIdx.x * 2 + 0) * cols + c] = g;
    ws[((int64_t)blockIdx.x * 2 + 1) * cols + c] = b;
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 fast path (cols % 256 == 0, cols <= 1024, 16-byte aligned rows): a HALF wave (32 lanes)
// per row, lane l owning the 8-column chunks j*32 + l (j < NJ = cols / 256), so every access is
// 16 bytes and a wave keeps two rows' loads in flight; reductions are 5 xor-shuffles.
// ---------------------------------------------------------------------------------------------
typedef unsigned short us;
__device__ __forceinline__ float hsum(float v) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ void unpack8(const u16x8& u, float* v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(u[e]);
}
__device__ __forceinline__ u16x8 pack8(const float* v) {
  u16x8 u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  return u;
}

template <int NJ>
__global__ __launch_bounds__(256) void ln_fwd16_kernel(int rows, int cols, const us* __restrict__ x,
                                                       mmseq_rows xl, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       us* __restrict__ y, mmseq_rows yl,
                                                       float* __restrict__ mean,
                                                       float* __restrict__ rstd, Drop dy_) {
  const int l = threadIdx.x & 31;
  const int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  if (r >= rows) return;
  const us* xr = x + row_off(xl, r);
  u16x8 raw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) raw[j] = *reinterpret_cast<const u16x8*>(xr + (j * 32 + l) * 8);
  float v[NJ][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    unpack8(raw[j], v[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[j][e];
  }
  const float mu = hsum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[j][e] - mu;
      q = fmaf(d, d, q);
    }
  const float rs = rsqrtf(hsum(q) / cols + eps);
  us* yr = y + row_off(yl, r);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (j * 32 + l) * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c), g1 = *reinterpret_cast<const f32x4*>(gamma + c + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c), b1 = *reinterpret_cast<const f32x4*>(beta + c + 4);
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = fmaf((v[j][e] - mu) * rs, g0[e], b0[e]);
      o[4 + e] = fmaf((v[j][4 + e] - mu) * rs, g1[e], b1[e]);
    }
    if (dy_.thr) {
      float dm[8];
      drop_mul_pairs<4>(dy_, (uint64_t)r * cols + c, dm);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= dm[e];
    }
    *reinterpret_cast<u16x8*>(yr + c) = pack8(o);
  }
  if (l == 0) {
    if (mean) mean[r] = mu;
    if (rstd) rstd[r] = rs;
  }
}

// LayerNorm forward (no dropout) whose output is also written as MX-fp8 for the next GEMM's A
// operand (fp8.hip layout: e4m3 [rows][ldq], E8M0 per 32 columns, packed scales), bit-identical to
// mmseq_quant_mxfp8 of the bf16 output: the bf16-rounded values are quantised. A 32-column block
// is 4 consecutive lanes' 8 columns, so its amax takes two lane swaps. y may be null (the GEMM is
// the only consumer). Blocks past the last row write the zero scales of the rows up to the next
// multiple of 64 (as the quantiser does).
template <int NJ>
__global__ __launch_bounds__(256) void ln_fwd16_q8_kernel(int rows, int cols,
                                                          const us* __restrict__ x, mmseq_rows xl,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          us* __restrict__ y, mmseq_rows yl,
                                                          float* __restrict__ mean,
                                                          float* __restrict__ rstd,
                                                          uint8_t* __restrict__ q, int64_t ldq,
                                                          uint8_t* __restrict__ qs) {
  const int l = threadIdx.x & 31;
  const int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int KB = cols >> 5;
  auto sidx = [&](int64_t row, int c) {
    return ((row >> 6) * KB + (c >> 5)) * 64 + (row & 15) * 4 + ((row >> 4) & 3);
  };
  if (r >= rows) {  // zero scales of the padding rows up to the next multiple of 64
    if (r < ((rows + 63) & ~63) && (l & 3) == 0) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) qs[sidx(r, (j * 32 + l) * 8)] = 0;
    }
    return;
  }
  const us* xr = x + row_off(xl, r);
  u16x8 raw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) raw[j] = *reinterpret_cast<const u16x8*>(xr + (j * 32 + l) * 8);
  float v[NJ][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    unpack8(raw[j], v[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[j][e];
  }
  const float mu = hsum(s) / cols;
  float qv = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[j][e] - mu;
      qv = fmaf(d, d, qv);
    }
  const float rs = rsqrtf(hsum(qv) / cols + eps);
  us* yr = y ? y + row_off(yl, r) : nullptr;
  uint8_t* qr = q + r * ldq;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (j * 32 + l) * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c), g1 = *reinterpret_cast<const f32x4*>(gamma + c + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c), b1 = *reinterpret_cast<const f32x4*>(beta + c + 4);
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = fmaf((v[j][e] - mu) * rs, g0[e], b0[e]);
      o[4 + e] = fmaf((v[j][4 + e] - mu) * rs, g1[e], b1[e]);
    }
    const u16x8 ob = pack8(o);
    if (yr) *reinterpret_cast<u16x8*>(yr + c) = ob;
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = bf2f(ob[e]);
      amax = fmaxf(amax, fabsf(o[e]));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    int ex = amax > 0.f ? (int)((__float_as_uint(amax) >> 23) & 0xff) - 127 : -127;
    ex = max(-127, min(127, ex - 8));
    const float inv = ldexpf(1.f, -ex);
    if ((l & 3) == 0) qs[sidx(r, c)] = (uint8_t)(ex + 127);
    uint32_t w[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float s0 = fminf(448.f, fmaxf(-448.f, o[4 * h] * inv));
      const float s1 = fminf(448.f, fmaxf(-448.f, o[4 * h + 1] * inv));
      const float s2 = fminf(448.f, fmaxf(-448.f, o[4 * h + 2] * inv));
      const float s3 = fminf(448.f, fmaxf(-448.f, o[4 * h + 3] * inv));
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(s0, s1, 0, false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(s2, s3, pk, true);
      w[h] = (uint32_t)pk;
    }
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
    *reinterpret_cast<u32x2*>(qr + c) = (u32x2){w[0], w[1]};
  }
  if (l == 0) {
    if (mean) mean[r] = mu;
    if (rstd) rstd[r] = rs;
  }
}

// dx = rstd * (g*dy - mean_c(g*dy) - xhat * mean_c(g*dy*xhat)) (+ dres); rpb rows per block,
// each half wave walks rows hw, hw + 8, ... with the next row's loads issued before the current
// row's math; per-block dgamma / dbeta partials -> ws[block][2][cols]
constexpr int RPB16 = 64;
// Q8 (config 5's fp8 dgrad): the gradient the next data-gradient GEMM reads (dxd when written, else
// dx with the residual) also leaves in MX-fp8 (mmseq_quant_mxfp8 of the bf16 values: q [rows][ldq],
// packed scales; the padding rows' scales are the caller's, zero-initialised)
// CS: also the column sums of the gradient it writes for the next GEMM (dx_drop when DXD, else dx
// with dres), as stored (bf16-rounded): the bias gradient of the Linear whose output gradient that
// is, instead of a pass in its weight-gradient GEMM; per-block partials -> ws[block][2][cols]
template <int NJ, bool DIN, bool DXD, bool Q8 = false, bool CS = false>
__global__ __launch_bounds__(256) void ln_bwd16_kernel(int rows, int cols, int rpb, const us* __restrict__ dy,
                                                       mmseq_rows dyl, const us* __restrict__ x,
                                                       mmseq_rows xl, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma,
                                                       us* __restrict__ dx, mmseq_rows dxl,
                                                       const us* __restrict__ dres, mmseq_rows dresl,
                                                       float* __restrict__ ws, Drop din,
                                                       us* __restrict__ dxd, mmseq_rows dxdl, Drop dout,
                                                       uint8_t* __restrict__ q8 = nullptr,
                                                       int64_t ldq = 0, uint8_t* __restrict__ q8s = nullptr) {
  constexpr int NA = CS ? 3 : 2;  // partial arrays: dgamma, dbeta (, the written gradient's sums)
  __shared__ float red[4][NA][NJ * 256];
  const int l = threadIdx.x & 31, hw = threadIdx.x >> 5;
  float pg[NJ][8], pb[NJ][8], pc[CS ? NJ : 1][8];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) pg[j][e] = pb[j][e] = 0.f;
#pragma unroll
  for (int j = 0; j < (CS ? NJ : 1); ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) pc[j][e] = 0.f;
  const int64_t rbeg = (int64_t)blockIdx.x * rpb;
  const int64_t rend = rbeg + rpb < rows ? rbeg + rpb : rows;
  auto load_g = [&](int c, float* g8) {
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c), g1 = *reinterpret_cast<const f32x4*>(gamma + c + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { g8[e] = g0[e]; g8[4 + e] = g1[e]; }
  };
  // x-hat and g*dy are recomputed in the second pass from the packed row (4 waves per SIMD)
#pragma unroll 1
  for (int64_t r = rbeg + hw; r < rend; r += 8) {
    u16x8 xc[NJ], dc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      xc[j] = *reinterpret_cast<const u16x8*>(x + row_off(xl, r) + (j * 32 + l) * 8);
      dc[j] = *reinterpret_cast<const u16x8*>(dy + row_off(dyl, r) + (j * 32 + l) * 8);
    }
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = (j * 32 + l) * 8;
      float xv[8], d[8], g8[8];
      unpack8(xc[j], xv);
      unpack8(dc[j], d);
      load_g(c, g8);
      if (DIN) {
        float dm[8];
        drop_mul_pairs<4>(din, (uint64_t)r * cols + c, dm);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] *= dm[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xx = (xv[e] - mu) * rs;
        const float gd = d[e] * g8[e];
        pg[j][e] = fmaf(d[e], xx, pg[j][e]);
        pb[j][e] += d[e];
        s1 += gd;
        s2 = fmaf(gd, xx, s2);
      }
    }
    s1 = hsum(s1) / cols;
    s2 = hsum(s2) / cols;
    us* dxr = dx + row_off(dxl, r);
    const us* drr = dres ? dres + row_off(dresl, r) : nullptr;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = (j * 32 + l) * 8;
      float xv[8], d[8], g8[8], o[8];
      unpack8(xc[j], xv);
      unpack8(dc[j], d);
      load_g(c, g8);
      float dm[8];
      if (DIN) drop_mul_pairs<4>(din, (uint64_t)r * cols + c, dm);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dd = DIN ? d[e] * dm[e] : d[e];
        o[e] = rs * (dd * g8[e] - s1 - (xv[e] - mu) * rs * s2);
      }
      u16x8 qsrc;
      if (DXD) {
        float od[8], dm2[8];
        drop_mul_pairs<4>(dout, (uint64_t)r * cols + c, dm2);
#pragma unroll
        for (int e = 0; e < 8; ++e) od[e] = o[e] * dm2[e];
        qsrc = pack8(od);
        *reinterpret_cast<u16x8*>(dxd + row_off(dxdl, r) + c) = qsrc;
      }
      if (drr) {
        float t[8];
        unpack8(*reinterpret_cast<const u16x8*>(drr + c), t);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += t[e];
      }
      const u16x8 ob = pack8(o);
      *reinterpret_cast<u16x8*>(dxr + c) = ob;
      if (CS) {
        float t8[8];
        unpack8(DXD ? qsrc : ob, t8);
#pragma unroll
        for (int e = 0; e < 8; ++e) pc[j][e] += t8[e];
      }
      if (Q8) {  // 32-column block = lanes l .. l + 3 (l & ~3): amax by two lane swaps
        if (!DXD) qsrc = ob;
        float qv[8], amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          qv[e] = bf2f(qsrc[e]);
          amax = fmaxf(amax, fabsf(qv[e]));
        }
        amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
        int ex = amax > 0.f ? (int)((__float_as_uint(amax) >> 23) & 0xff) - 127 : -127;
        ex = max(-127, min(127, ex - 8));
        const float inv = ldexpf(1.f, -ex);
        if ((l & 3) == 0)
          q8s[((r >> 6) * (cols >> 5) + (c >> 5)) * 64 + (r & 15) * 4 + ((r >> 4) & 3)] = (uint8_t)(ex + 127);
        uint32_t w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float s0 = fminf(448.f, fmaxf(-448.f, qv[4 * h] * inv));
          const float s1 = fminf(448.f, fmaxf(-448.f, qv[4 * h + 1] * inv));
          const float s2 = fminf(448.f, fmaxf(-448.f, qv[4 * h + 2] * inv));
          const float s3 = fminf(448.f, fmaxf(-448.f, qv[4 * h + 3] * inv));
          int pk = __builtin_amdgcn_cvt_pk_fp8_f32(s0, s1, 0, false);
          pk = __builtin_amdgcn_cvt_pk_fp8_f32(s2, s3, pk, true);
          w[h] = (uint32_t)pk;
        }
        typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
        *reinterpret_cast<u32x2*>(q8 + r * ldq + c) = (u32x2){w[0], w[1]};
      }
    }
  }
  // deterministic cross-half-wave reduction in two LDS rounds (keeps LDS at 8 KB per 256 columns)
  if (hw >= 4) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[hw - 4][0][(j * 32 + l) * 8 + e] = pg[j][e];
        red[hw - 4][1][(j * 32 + l) * 8 + e] = pb[j][e];
        if (CS) red[hw - 4][NA - 1][(j * 32 + l) * 8 + e] = pc[CS ? j : 0][e];
      }
  }
  __syncthreads();
  if (hw < 4) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[hw][0][(j * 32 + l) * 8 + e] += pg[j][e];
        red[hw][1][(j * 32 + l) * 8 + e] += pb[j][e];
        if (CS) red[hw][NA - 1][(j * 32 + l) * 8 + e] += pc[CS ? j : 0][e];
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
#pragma unroll
    for (int k = 0; k < NA; ++k)
      ws[((int64_t)blockIdx.x * NA + k) * cols + c] = (red[0][k][c] + red[1][k][c]) + (red[2][k][c] + red[3][k][c]);
  }
}

bool rows_vec16(const void* p, const mmseq_rows& l) {
  return ((uintptr_t)p % 16) == 0 && l.ld % 8 == 0 && l.bstride % 8 == 0;
}

bool rows_vec(const void* p, const mmseq_rows& l, int esz) {
  return ((uintptr_t)p % (4 * esz)) == 0 && l.ld % 4 == 0 && l.bstride % 4 == 0;
}

}  // namespace

int64_t mmseq_reduce_extra(int nb, int W);
mmseq_status mmseq_reduce_partials(int nb, int W, int split, const float* ws, float* ws2,
                                   float* outA, float* outB, int accumulate, hipStream_t s);

// ws must hold nb*2*cols partials followed by mmseq_reduce_extra(nb, 2*cols) scratch floats
mmseq_status ln_reduce_partials(int nb, int cols, const float* ws, float* dg, float* db,
                                hipStream_t s) {
  return mmseq_reduce_partials(nb, 2 * cols, cols, ws, const_cast<float*>(ws) + (int64_t)nb * 2 * cols,
                               dg, db, 1, s);
}

extern "C" mmseq_status mmseq_layernorm_fwd(int rows, int cols, const void* x, mmseq_rows xl,
                                            const float* gamma, const float* beta, float eps,
                                            void* y, mmseq_rows yl, float* mean, float* rstd,
                                            mmseq_dtype xd, mmseq_dtype yd,
                                            const mmseq_dropout* drop_y, mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && cols > 0 && cols <= 2048, "layernorm: cols must be in (0, 2048]");
  MMSEQ_REQUIRE(x && y && gamma && beta, "layernorm: null buffer");
  MMSEQ_REQUIRE(xl.rpb > 0 && yl.rpb > 0, "layernorm: rpb must be > 0");
  if (rows == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((rows + 3) / 4);
  const bool vec = cols % 4 == 0 && rows_vec(x, xl, xd == MMSEQ_BF16 ? 2 : 4) &&
                   rows_vec(y, yl, yd == MMSEQ_BF16 ? 2 : 4);
  const Drop dd = make_drop(drop_y);
  if (xd == MMSEQ_BF16 && yd == MMSEQ_BF16 && cols % 256 == 0 && cols <= 1024 && rows_vec16(x, xl) &&
      rows_vec16(y, yl) && ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0) {
    const dim3 g8((rows + 7) / 8);
    switch (cols / 256) {
#define LNF16(NJ) hipLaunchKernelGGL((ln_fwd16_kernel<NJ>), g8, dim3(256), 0, s, rows, cols, \
                    (const us*)x, xl, gamma, beta, eps, (us*)y, yl, mean, rstd, dd); break
      case 1: LNF16(1); case 2: LNF16(2); case 3: LNF16(3); case 4: LNF16(4);
#undef LNF16
    }
    return mmseq_check_launch("layernorm_fwd");
  }
#define LNF(TX, TY, V)                                                                            \
  if (cols <= 1024)                                                                               \
    hipLaunchKernelGGL((ln_fwd_kernel<TX, TY, V, 4>), grid, dim3(256), 0, s, rows, cols,           \
                       (const TX*)x, xl, gamma, beta, eps, (TY*)y, yl, mean, rstd, dd);            \
  else                                                                                            \
    hipLaunchKernelGGL((ln_fwd_kernel<TX, TY, V, 8>), grid, dim3(256), 0, s, rows, cols,           \
                       (const TX*)x, xl, gamma, beta, eps, (TY*)y, yl, mean, rstd, dd)
#define LNF2(TX, TY) \
  if (vec) { LNF(TX, TY, true); } else { LNF(TX, TY, false); }
  if (xd == MMSEQ_F32 && yd == MMSEQ_F32) { LNF2(float, float); }
  else if (xd == MMSEQ_F32 && yd == MMSEQ_BF16) { LNF2(float, unsigned short); }
  else if (xd == MMSEQ_BF16 && yd == MMSEQ_F32) { LNF2(unsigned short, float); }
  else { LNF2(unsigned short, unsigned short); }
#undef LNF2
#undef LNF
  return mmseq_check_launch("layernorm_fwd");
}

extern "C" int64_t mmseq_colsum_workspace(int rows, int cols);
mmseq_status mmseq_reduce_partials3(int nb, int W, int split, int split2, const float* ws, float* ws2,
                                    float* outA, float* outB, float* outC, int accumulate,
                                    hipStream_t s);
extern "C" mmseq_status mmseq_colsum(int rows, int cols, const void* x, int64_t ldx, float* out,
                                     int accumulate, float* ws, mmseq_dtype dt, mmseq_stream stream);

extern "C" int64_t mmseq_layernorm_bwd_workspace(int rows, int cols) {
  const int nb = (rows + RPB16 - 1) / RPB16;  // the bf16 fast path's block count (>= the generic)
  // three partial rows per block (dgamma, dbeta, the written gradient's column sums) or, where the
  // fast kernel does not take the column sums, the separate column-sum pass's workspace
  const int64_t w = (int64_t)nb * 3 * cols + mmseq_reduce_extra(nb, 3 * cols);
  const int64_t c = mmseq_colsum_workspace(rows, cols);
  return w > c ? w : c;
}

static mmseq_status layernorm_bwd_impl(int rows, int cols, const void* dy, mmseq_rows dyl,
                                       const void* x, mmseq_rows xl, const float* mean,
                                       const float* rstd, const float* gamma, void* dx,
                                       mmseq_rows dxl, const void* dres, mmseq_rows dresl,
                                       float* dgamma, float* dbeta, float* workspace,
                                       mmseq_dtype dtype, const mmseq_dropout* drop_dy,
                                       void* dx_drop, mmseq_rows dxdl, const mmseq_dropout* drop_dx,
                                       void* q, int64_t ldq, void* q_scales, float* dsum,
                                       mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && cols > 0 && cols <= 2048, "layernorm_bwd: cols must be in (0, 2048]");
  MMSEQ_REQUIRE(dy && x && mean && rstd && gamma && dx && workspace, "layernorm_bwd: null buffer");
  if (rows == 0) return MMSEQ_OK;
  // dsum (+)= column sums of the gradient written for the next GEMM: dx_drop if given, else dx
  const mmseq_rows gl = dx_drop ? dxdl : dxl;
  MMSEQ_REQUIRE(!dsum || gl.rpb >= rows || gl.bstride == gl.rpb * gl.ld,
                "layernorm_bwd: dsum needs the summed gradient in dense rows");
  if (!dres) dresl = dxl;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = (rows + RPB - 1) / RPB;
  const int esz = dtype == MMSEQ_BF16 ? 2 : 4;
  const bool vec = cols % 4 == 0 && rows_vec(dy, dyl, esz) && rows_vec(x, xl, esz) &&
                   rows_vec(dx, dxl, esz) && (!dres || rows_vec(dres, dresl, esz)) &&
                   (!dx_drop || rows_vec(dx_drop, dxdl, esz));
  const Drop din = make_drop(drop_dy), dout = make_drop(drop_dx);
  if (dtype == MMSEQ_BF16 && cols % 256 == 0 && cols <= 1024 && rows_vec16(dy, dyl) && rows_vec16(x, xl) &&
      rows_vec16(dx, dxl) && (!dres || rows_vec16(dres, dresl)) &&
      (!dx_drop || rows_vec16(dx_drop, dxdl)) && ((uintptr_t)gamma % 16) == 0) {
    // at most 512 blocks (two per CU at this kernel's ~190 VGPRs: one resident round), each over
    // rpb rows: 2.5-10x fewer dgamma / dbeta partial rows to write and reduce than 64-row blocks
    int rpb = RPB16, nb16 = (rows + RPB16 - 1) / RPB16;
    if (nb16 > 512) {
      rpb = ((rows + 511) / 512 + 7) / 8 * 8;
      nb16 = (rows + rpb - 1) / rpb;
    }
    const bool di = din.thr != 0, dd = dx_drop != nullptr;
    // the column sums ride in the kernel where it has the registers (no input dropout, bf16 out)
    const bool cs = dsum && !q && !di && cols <= 768;  // at cols 1024 it would spill
#define LNB16C(NJ, B) hipLaunchKernelGGL((ln_bwd16_kernel<NJ, false, B, false, true>), dim3(nb16), dim3(256), \
                    0, s, rows, cols, rpb, (const us*)dy, dyl, (const us*)x, xl, mean, rstd, gamma, (us*)dx,  \
                    dxl, (const us*)dres, dresl, workspace, din, (us*)dx_drop, dxdl, dout, nullptr, 0, nullptr)
#define LNB16K(NJ, A, B) hipLaunchKernelGGL((ln_bwd16_kernel<NJ, A, B>), dim3(nb16), dim3(256), 0, s, rows, \
                    cols, rpb, (const us*)dy, dyl, (const us*)x, xl, mean, rstd, gamma, (us*)dx, dxl,         \
                    (const us*)dres, dresl, workspace, din, (us*)dx_drop, dxdl, dout, nullptr, 0, nullptr)
#define LNB16Q(NJ, A, B) hipLaunchKernelGGL((ln_bwd16_kernel<NJ, A, B, true>), dim3(nb16), dim3(256), 0, s, \
                    rows, cols, rpb, (const us*)dy, dyl, (const us*)x, xl, mean, rstd, gamma, (us*)dx, dxl,   \
                    (const us*)dres, dresl, workspace, din, (us*)dx_drop, dxdl, dout, (uint8_t*)q, ldq, \
                    (uint8_t*)q_scales)
#define LNB16(NJ)                                           \
  if (cs) {                                                 \
    if (dd) LNB16C(NJ, true);                               \
    else LNB16C(NJ, false);                                 \
  } else LNB16N(NJ)
#define LNB16N(NJ)                                          \
  if (q) {                                                  \
    if (di && dd) LNB16Q(NJ, true, true);                   \
    else if (di) LNB16Q(NJ, true, false);                   \
    else if (dd) LNB16Q(NJ, false, true);                   \
    else LNB16Q(NJ, false, false);                          \
  } else if (di && dd) LNB16K(NJ, true, true);              \
  else if (di) LNB16K(NJ, true, false);                     \
  else if (dd) LNB16K(NJ, false, true);                     \
  else LNB16K(NJ, false, false);                            \
  break
    switch (cols / 256) {
      case 1: LNB16(1); case 2: LNB16(2); case 3: LNB16(3); case 4: LNB16N(4);
    }
#undef LNB16
#undef LNB16N
#undef LNB16Q
#undef LNB16K
#undef LNB16C
    mmseq_status st = mmseq_check_launch("layernorm_bwd");
    if (st) return st;
    if (cs)
      return mmseq_reduce_partials3(nb16, 3 * cols, cols, 2 * cols, workspace,
                                    workspace + (int64_t)nb16 * 3 * cols, dgamma, dbeta, dsum, 1, s);
    if (dgamma || dbeta) {
      st = ln_reduce_partials(nb16, cols, workspace, dgamma, dbeta, s);
      if (st) return st;
    }
    // column sums as their own pass over the written gradient (the workspace is free again)
    if (dsum) return mmseq_colsum(rows, cols, dx_drop ? dx_drop : dx, gl.ld, dsum, 1, workspace, dtype, stream);
    return MMSEQ_OK;
  }
  if (q) return mmseq_set_error(MMSEQ_EUNSUPPORTED, "layernorm_bwd_mxfp8: bf16, cols 256..1024 (x256), 16-byte rows");
#define LNBJ(T, V, J)                                                                             \
  hipLaunchKernelGGL((ln_bwd_kernel<T, V, J>), dim3(nb), dim3(256), 0, s, rows, cols, (const T*)dy, \
                     dyl, (const T*)x, xl, mean, rstd, gamma, (T*)dx, dxl, (const T*)dres, dresl,   \
                     workspace, din, (T*)dx_drop, dxdl, dout)
#define LNB(T, V) \
  if (cols <= 1024) { LNBJ(T, V, 4); } else { LNBJ(T, V, 8); }
  if (dtype == MMSEQ_F32) {
    if (vec) { LNB(float, true); } else { LNB(float, false); }
  } else {
    if (vec) { LNB(unsigned short, true); } else { LNB(unsigned short, false); }
  }
#undef LNBJ
#undef LNB
  mmseq_status st = mmseq_check_launch("layernorm_bwd");
  if (st) return st;
  if (dgamma || dbeta) {
    st = ln_reduce_partials(nb, cols, workspace, dgamma, dbeta, s);
    if (st) return st;
  }
  if (dsum) return mmseq_colsum(rows, cols, dx_drop ? dx_drop : dx, gl.ld, dsum, 1, workspace, dtype, stream);
  return MMSEQ_OK;
}

extern "C" mmseq_status mmseq_layernorm_bwd(int rows, int cols, const void* dy, mmseq_rows dyl,
                                            const void* x, mmseq_rows xl, const float* mean,
                                            const float* rstd, const float* gamma, void* dx,
                                            mmseq_rows dxl, const void* dres, mmseq_rows dresl,
                                            float* dgamma, float* dbeta, float* workspace,
                                            mmseq_dtype dtype, const mmseq_dropout* drop_dy,
                                            void* dx_drop, const mmseq_dropout* drop_dx,
                                            mmseq_stream stream) {
  return layernorm_bwd_impl(rows, cols, dy, dyl, x, xl, mean, rstd, gamma, dx, dxl, dres, dresl,
                            dgamma, dbeta, workspace, dtype, drop_dy, dx_drop, dxl, drop_dx, nullptr,
                            0, nullptr, nullptr, stream);
}

extern "C" mmseq_status mmseq_layernorm_bwd_ex(int rows, int cols, const void* dy, mmseq_rows dyl,
                                               const void* x, mmseq_rows xl, const float* mean,
                                               const float* rstd, const float* gamma, void* dx,
                                               mmseq_rows dxl, const void* dres, mmseq_rows dresl,
                                               float* dgamma, float* dbeta, float* workspace,
                                               mmseq_dtype dtype, const mmseq_dropout* drop_dy,
                                               void* dx_drop, mmseq_rows dx_dropl,
                                               const mmseq_dropout* drop_dx, float* dsum,
                                               mmseq_stream stream) {
  return layernorm_bwd_impl(rows, cols, dy, dyl, x, xl, mean, rstd, gamma, dx, dxl, dres, dresl,
                            dgamma, dbeta, workspace, dtype, drop_dy, dx_drop,
                            dx_drop ? dx_dropl : dxl, drop_dx, nullptr, 0, nullptr, dsum, stream);
}

extern "C" mmseq_status mmseq_layernorm_bwd_rows(int rows, int cols, const void* dy, mmseq_rows dyl,
                                                 const void* x, mmseq_rows xl, const float* mean,
                                                 const float* rstd, const float* gamma, void* dx,
                                                 mmseq_rows dxl, const void* dres, mmseq_rows dresl,
                                                 float* dgamma, float* dbeta, float* workspace,
                                                 mmseq_dtype dtype, const mmseq_dropout* drop_dy,
                                                 void* dx_drop, mmseq_rows dx_dropl,
                                                 const mmseq_dropout* drop_dx, mmseq_stream stream) {
  MMSEQ_REQUIRE(dx_drop, "layernorm_bwd_rows: dx_drop is required");
  return layernorm_bwd_impl(rows, cols, dy, dyl, x, xl, mean, rstd, gamma, dx, dxl, dres, dresl,
                            dgamma, dbeta, workspace, dtype, drop_dy, dx_drop, dx_dropl, drop_dx,
                            nullptr, 0, nullptr, nullptr, stream);
}

extern "C" mmseq_status mmseq_layernorm_bwd_mxfp8(int rows, int cols, const void* dy, mmseq_rows dyl,
                                                  const void* x, mmseq_rows xl, const float* mean,
                                                  const float* rstd, const float* gamma, void* dx,
                                                  mmseq_rows dxl, const void* dres, mmseq_rows dresl,
                                                  float* dgamma, float* dbeta, float* workspace,
                                                  const mmseq_dropout* drop_dy, void* dx_drop,
                                                  const mmseq_dropout* drop_dx, void* q, int64_t ldq,
                                                  void* q_scales, mmseq_stream stream) {
  MMSEQ_REQUIRE(q && q_scales && ldq >= cols && ldq % 16 == 0 && ((uintptr_t)q & 15) == 0,
                "layernorm_bwd_mxfp8: q / ldq");
  return layernorm_bwd_impl(rows, cols, dy, dyl, x, xl, mean, rstd, gamma, dx, dxl, dres, dresl,
                            dgamma, dbeta, workspace, MMSEQ_BF16, drop_dy, dx_drop, dxl, drop_dx, q,
                            ldq, q_scales, nullptr, stream);
}

extern "C" mmseq_status mmseq_layernorm_fwd_mxfp8(int rows, int cols, const void* x, mmseq_rows xl,
                                                  const float* gamma, const float* beta, float eps,
                                                  void* y, mmseq_rows yl, float* mean, float* rstd,
                                                  void* q, int64_t ldq, void* q_scales,
                                                  mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && cols % 256 == 0 && cols >= 256 && cols <= 1024,
                "layernorm_fwd_mxfp8: cols must be 256, 512, 768 or 1024");
  MMSEQ_REQUIRE(x && gamma && beta && q && q_scales && ldq >= cols && ldq % 16 == 0,
                "layernorm_fwd_mxfp8: null buffer / ldq");
  MMSEQ_REQUIRE(xl.rpb > 0 && (!y || yl.rpb > 0), "layernorm_fwd_mxfp8: rpb must be > 0");
  MMSEQ_REQUIRE(rows_vec16(x, xl) && (!y || rows_vec16(y, yl)) && ((uintptr_t)gamma % 16) == 0 &&
                    ((uintptr_t)beta % 16) == 0 && ((uintptr_t)q % 16) == 0,
                "layernorm_fwd_mxfp8: 16-byte aligned rows");
  if (rows == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 g8((((rows + 63) & ~63) + 7) / 8);
  switch (cols / 256) {
#define LNQ(NJ) hipLaunchKernelGGL((ln_fwd16_q8_kernel<NJ>), g8, dim3(256), 0, s, rows, cols,       \
                  (const us*)x, xl, gamma, beta, eps, (us*)y, yl, mean, rstd, (uint8_t*)q, ldq, \
                  (uint8_t*)q_scales); break
    case 1: LNQ(1); case 2: LNQ(2); case 3: LNQ(3); case 4: LNQ(4);
#undef LNQ
  }
  return mmseq_check_launch("layernorm_fwd_mxfp8");
}
