// CLIP ModifiedResNet (RN50) pieces on NHWC activations (clip/model.py:10-187,
// lxrt/modeling.py:621-705, 1014-1030). The convolutions themselves are GEMMs (1x1 directly,
// 3x3 through an NHWC im2col with K = 9 C padded); this file holds the im2col / col2im, the
// BatchNorm (batch statistics by Chan-merged Welford partials, deterministic), the 2x2 average
// pool, and the attention pool's token gather (with the reference's reshape quirk) and output
// expansion. Byte / HBM-bound kernels: coalesced along the channel dimension.
#include "common.h"

namespace {

template <typename T> struct Pack8;
template <> struct Pack8<unsigned short> {
  u16x8 v;
  __device__ __forceinline__ void ld(const unsigned short* p) { v = *reinterpret_cast<const u16x8*>(p); }
  __device__ __forceinline__ void st(unsigned short* p) const { *reinterpret_cast<u16x8*>(p) = v; }
  __device__ __forceinline__ void zero() { v = (u16x8){0, 0, 0, 0, 0, 0, 0, 0}; }
};
template <> struct Pack8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void ld(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ __forceinline__ void st(float* p) const {
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
  __device__ __forceinline__ void zero() { a = b = (f32x4){0.f, 0.f, 0.f, 0.f}; }
};

struct ConvGeom {
  int U, H, W, C, Ho, Wo, ks, stride, pad, Kp;
};

// cols[r][k], r = (u, oy, ox), k = (ky * ks + kx) * C + c; zero past ks*ks*C and in the padding.
// MODE 1: one thread per 8 columns of one tap (C % 8 == 0, 16-byte load and store); MODE 2: one
// thread per 8 columns gathered one by one (Kp % 8 == 0: the C = 3 stem), one 16-byte store;
// MODE 0: one thread per column.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void im2col_nhwc_kernel(ConvGeom g, const T* __restrict__ x,
                                                          T* __restrict__ cols) {
  const int per = MODE ? 8 : 1;
  const int kchunks = g.Kp / per;
  const int64_t rows = (int64_t)g.U * g.Ho * g.Wo;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * kchunks) return;
  const int64_t r = idx / kchunks;
  const int k = (int)(idx - r * kchunks) * per;
  const int u = (int)(r / (g.Ho * g.Wo));
  const int rem = (int)(r - (int64_t)u * g.Ho * g.Wo);
  const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
  T* dst = cols + r * g.Kp + k;
  if constexpr (MODE == 2) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = k + j, tap = kk / g.C, c = kk - tap * g.C;
      const int ky = tap / g.ks, kx = tap - ky * g.ks;
      const int iy = oy * g.stride + ky - g.pad, ix = ox * g.stride + kx - g.pad;
      const bool in = tap < g.ks * g.ks && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
      v[j] = in ? Elem<T>::ld(x + (((int64_t)u * g.H + iy) * g.W + ix) * g.C + c) : 0.f;
    }
    Vec4<T>::st(dst, (f32x4){v[0], v[1], v[2], v[3]});
    Vec4<T>::st(dst + 4, (f32x4){v[4], v[5], v[6], v[7]});
    return;
  }
  const int tap = k / g.C, c = k - tap * g.C;
  const int ky = tap / g.ks, kx = tap - ky * g.ks;
  const int iy = oy * g.stride + ky - g.pad, ix = ox * g.stride + kx - g.pad;
  const bool in = tap < g.ks * g.ks && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
  const T* src = x + (((int64_t)u * g.H + iy) * g.W + ix) * g.C + c;
  if constexpr (MODE == 1) {
    Pack8<T> p;
    if (in) p.ld(src); else p.zero();
    p.st(dst);
  } else {
    *dst = in ? *src : (T)0;
  }
}

// dx[u][iy][ix][c] = sum over taps of dcols at the output positions that read (iy, ix); PER
// channels per thread (8 with 16-byte accesses when C % 8 == 0)
template <typename T, int PER>
__global__ __launch_bounds__(256) void col2im_nhwc_kernel(ConvGeom g, const T* __restrict__ dcols,
                                                          T* __restrict__ dx) {
  const int cg = g.C / PER;
  const int64_t total = (int64_t)g.U * g.H * g.W * cg;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % cg) * PER;
  int64_t t = idx / cg;
  const int ix = (int)(t % g.W);
  t /= g.W;
  const int iy = (int)(t % g.H);
  const int u = (int)(t / g.H);
  float acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) acc[j] = 0.f;
  for (int ky = 0; ky < g.ks; ++ky) {
    const int yy = iy + g.pad - ky;
    if (yy < 0 || yy % g.stride) continue;
    const int oy = yy / g.stride;
    if (oy >= g.Ho) continue;
    for (int kx = 0; kx < g.ks; ++kx) {
      const int xx = ix + g.pad - kx;
      if (xx < 0 || xx % g.stride) continue;
      const int ox = xx / g.stride;
      if (ox >= g.Wo) continue;
      const int64_t r = ((int64_t)u * g.Ho + oy) * g.Wo + ox;
      const T* src = dcols + r * g.Kp + (ky * g.ks + kx) * g.C + c;
      if constexpr (PER == 8) {
        const f32x4 a = Vec4<T>::ld(src), b = Vec4<T>::ld(src + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] += a[j];
          acc[4 + j] += b[j];
        }
      } else {
        acc[0] += Elem<T>::ld(src);
      }
    }
  }
  T* dst = dx + (((int64_t)u * g.H + iy) * g.W + ix) * g.C + c;
  if constexpr (PER == 8) {
    Vec4<T>::st(dst, (f32x4){acc[0], acc[1], acc[2], acc[3]});
    Vec4<T>::st(dst + 4, (f32x4){acc[4], acc[5], acc[6], acc[7]});
  } else {
    Elem<T>::st(dst, acc[0]);
  }
}

// ---------------------------------------------------------------------------------------------
// BatchNorm over rows of [rows][C] (NHWC), HBM-bound: every thread moves 8 consecutive channels
// (16 B of bf16). A statistics block covers CW = min(C, 512) channels (CW / 8 lanes per row,
// 2048 / CW rows per block step) over a chunk of rows; the chunk length is chosen so the grid has
// ~1024 blocks. Per-thread sums are shifted by the chunk's first row (sum d, sum d^2 with
// d = x - x[r0]), added across the block in a fixed order, and turned into per-chunk partials
// (n, mean, M2) that the finalize kernel Chan-merges in chunk order: deterministic.
struct BnPlan {
  int cw, lpr, rpb, gx;  // channels per block, lanes per row, rows per block step, channel blocks
  int64_t chunk;         // rows per chunk (multiple of rpb)
  int nch;               // chunks
};

__host__ inline bool bn_shape_ok(int C) {
  return C % 8 == 0 && (C > 512 ? C % 512 == 0 : (256 % (C / 8)) == 0);
}

__host__ inline BnPlan bn_plan(int64_t rows, int C) {
  BnPlan p;
  p.cw = C < 512 ? C : 512;
  p.lpr = p.cw / 8;
  p.rpb = 256 / p.lpr;
  p.gx = C / p.cw;
  const int64_t want = (rows * p.gx + 1023) / 1024;  // rows per chunk for ~1024 blocks
  int64_t ch = want < 4 * p.rpb ? 4 * p.rpb : want;
  p.chunk = (ch + p.rpb - 1) / p.rpb * p.rpb;
  p.nch = rows > 0 ? (int)((rows + p.chunk - 1) / p.chunk) : 0;
  return p;
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* v) {
  const f32x4 a = Vec4<T>::ld(p), b = Vec4<T>::ld(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = a[j];
    v[4 + j] = b[j];
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* v) {
  Vec4<T>::st(p, (f32x4){v[0], v[1], v[2], v[3]});
  Vec4<T>::st(p + 4, (f32x4){v[4], v[5], v[6], v[7]});
}
__device__ __forceinline__ void ldf8(const float* p, float* v) { ld8<float>(p, v); }

// per-chunk partials part[k][C] (n), part[nch + k][C] (mean), part[2 nch + k][C] (M2)
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(int64_t rows, int C, BnPlan pl,
                                                               const T* __restrict__ x,
                                                               float* __restrict__ part) {
  __shared__ float sh[2][2048];
  const int lp = threadIdx.x % pl.lpr, rr = threadIdx.x / pl.lpr;
  const int c0 = blockIdx.x * pl.cw + lp * 8;
  const int64_t r0 = (int64_t)blockIdx.y * pl.chunk;
  const int64_t r1 = min(rows, r0 + pl.chunk);
  float k[8], s[8], q[8];
  ld8(x + r0 * C + c0, k);
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
#pragma unroll 2
  for (int64_t r = r0 + rr; r < r1; r += pl.rpb) {
    float v[8];
    ld8(x + r * C + c0, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[j] - k[j];
      s[j] += d;
      q[j] = fmaf(d, d, q[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][rr * pl.cw + lp * 8 + j] = s[j];
    sh[1][rr * pl.cw + lp * 8 + j] = q[j];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < pl.cw; t += 256) {
    float S = 0.f, Q = 0.f;
    for (int i = 0; i < pl.rpb; ++i) {
      S += sh[0][i * pl.cw + t];
      Q += sh[1][i * pl.cw + t];
    }
    const int c = blockIdx.x * pl.cw + t;
    const float n = (float)(r1 - r0), kk = Elem<T>::ld(x + r0 * C + c);
    const float m = S / n;
    const int64_t o = (int64_t)blockIdx.y * C + c, stride = (int64_t)pl.nch * C;
    part[o] = n;
    part[stride + o] = kk + m;
    part[2 * stride + o] = fmaxf(Q - S * m, 0.f);
  }
}

struct Welford {
  float n, mean, m2;
  __device__ __forceinline__ void merge(float nb, float mb, float m2b) {
    if (nb == 0.f) return;
    const float nn = n + nb, d = mb - mean;
    mean += d * (nb / nn);
    m2 += m2b + d * d * (n * nb / nn);
    n = nn;
  }
};

// mean / rstd from the partials; train-mode running-stat update (momentum, unbiased variance with
// the reference's element count n_ref, which counts each image as often as the reference's
// batch holds it). Block = 32 channels x 32 chunk lanes: lane j merges chunks j, j + 32, ... in
// order, then lane 0 merges the 32 lane results in order (deterministic).
__global__ __launch_bounds__(1024) void bn_stats_final_kernel(int C, int nch, const float* part,
                                                              float eps, float momentum,
                                                              double n_ref, float* mean,
                                                              float* rstd, float* run_mean,
                                                              float* run_var) {
  __shared__ float sh[3][32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + tx;
  Welford s{0.f, 0.f, 0.f};
  if (c < C)
    for (int k = ty; k < nch; k += 32)
      s.merge(part[(int64_t)k * C + c], part[((int64_t)nch + k) * C + c],
              part[(2 * (int64_t)nch + k) * C + c]);
  sh[0][ty][tx] = s.n;
  sh[1][ty][tx] = s.mean;
  sh[2][ty][tx] = s.m2;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  Welford t{0.f, 0.f, 0.f};
  for (int j = 0; j < 32; ++j) t.merge(sh[0][j][tx], sh[1][j][tx], sh[2][j][tx]);
  const float var = t.n > 0.f ? t.m2 / t.n : 0.f;
  mean[c] = t.mean;
  rstd[c] = rsqrtf(var + eps);
  if (run_mean) {
    const double unb = n_ref > 1.0 ? (double)var * n_ref / (n_ref - 1.0) : (double)var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * t.mean;
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
  }
}

__global__ __launch_bounds__(256) void bn_eval_stats_kernel(int C, float eps, const float* run_mean,
                                                            const float* run_var, float* mean,
                                                            float* rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = run_mean[c];
  rstd[c] = rsqrtf(run_var[c] + eps);
}

// y = act((x - mean) * rstd * gamma + beta + resid), 8 channels per thread
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(int64_t n8, int C, const T* __restrict__ x,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const T* __restrict__ resid, int relu,
                                                       T* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int64_t e = i * 8;
  const int c = (int)(e % C);
  float v[8], mu[8], rs[8], ga[8], be[8];
  ld8(x + e, v);
  ldf8(mean + c, mu);
  ldf8(rstd + c, rs);
  ldf8(gamma + c, ga);
  ldf8(beta + c, be);
  float r[8];
  if (resid) ld8(resid + e, r);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = fmaf((v[j] - mu[j]) * rs[j], ga[j], be[j]);
    if (resid) t += r[j];
    v[j] = relu ? fmaxf(t, 0.f) : t;
  }
  st8(y + e, v);
}

// backward partial sums per chunk: sum g, sum g * xhat with g = dy * (y > 0 when relu);
// part[k][C] = sum g, part[nch + k][C] = sum g xhat
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(int64_t rows, int C, BnPlan pl,
                                                             const T* __restrict__ dy,
                                                             const T* __restrict__ y,
                                                             const T* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             float* __restrict__ part) {
  __shared__ float sh[2][2048];
  const int lp = threadIdx.x % pl.lpr, rr = threadIdx.x / pl.lpr;
  const int c0 = blockIdx.x * pl.cw + lp * 8;
  const int64_t r0 = (int64_t)blockIdx.y * pl.chunk;
  const int64_t r1 = min(rows, r0 + pl.chunk);
  float mu[8], rs[8], sg[8], sgx[8];
  ldf8(mean + c0, mu);
  ldf8(rstd + c0, rs);
#pragma unroll
  for (int j = 0; j < 8; ++j) sg[j] = sgx[j] = 0.f;
#pragma unroll 2
  for (int64_t r = r0 + rr; r < r1; r += pl.rpb) {
    float g[8], xv[8];
    ld8(dy + r * C + c0, g);
    ld8(x + r * C + c0, xv);
    if (y) {
      float yv[8];
      ld8(y + r * C + c0, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sg[j] += g[j];
      sgx[j] = fmaf(g[j], (xv[j] - mu[j]) * rs[j], sgx[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][rr * pl.cw + lp * 8 + j] = sg[j];
    sh[1][rr * pl.cw + lp * 8 + j] = sgx[j];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < pl.cw; t += 256) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < pl.rpb; ++i) {
      a += sh[0][i * pl.cw + t];
      b += sh[1][i * pl.cw + t];
    }
    const int c = blockIdx.x * pl.cw + t;
    part[(int64_t)blockIdx.y * C + c] = a;
    part[((int64_t)pl.nch + blockIdx.y) * C + c] = b;
  }
}

__global__ __launch_bounds__(1024) void bn_bwd_final_kernel(int C, int nch, const float* part,
                                                            float* sums, float* dgamma,
                                                            float* dbeta) {
  __shared__ float sh[2][32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + tx;
  float sg = 0.f, sgx = 0.f;
  if (c < C)
    for (int k = ty; k < nch; k += 32) {
      sg += part[(int64_t)k * C + c];
      sgx += part[((int64_t)nch + k) * C + c];
    }
  sh[0][ty][tx] = sg;
  sh[1][ty][tx] = sgx;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  float a = 0.f, b = 0.f;
  for (int j = 0; j < 32; ++j) {
    a += sh[0][j][tx];
    b += sh[1][j][tx];
  }
  sums[c] = a;
  sums[C + c] = b;
  if (dgamma) dgamma[c] += b;
  if (dbeta) dbeta[c] += a;
}

// dx = gamma rstd (g - sum g / n - xhat sum(g xhat) / n)  (train; eval: gamma rstd g);
// dres = g (the residual branch's gradient) when requested; 8 channels per thread
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(int64_t n8, int C, int64_t rows,
                                                           const T* __restrict__ dy,
                                                           const T* __restrict__ y,
                                                           const T* __restrict__ x,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ sums,
                                                           int train, T* __restrict__ dx,
                                                           T* __restrict__ dres) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int64_t e = i * 8;
  const int c = (int)(e % C);
  float g[8], rs[8], ga[8];
  ld8(dy + e, g);
  if (y) {
    float yv[8];
    ld8(y + e, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
  }
  if (dres) st8(dres + e, g);
  ldf8(rstd + c, rs);
  ldf8(gamma + c, ga);
  float v[8];
  if (train) {
    const float inv = 1.f / (float)rows;
    float xv[8], mu[8], s1[8], s2[8];
    ld8(x + e, xv);
    ldf8(mean + c, mu);
    ldf8(sums + c, s1);
    ldf8(sums + C + c, s2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (xv[j] - mu[j]) * rs[j];
      v[j] = (g[j] - s1[j] * inv - xh * s2[j] * inv) * rs[j] * ga[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = g[j] * rs[j] * ga[j];
  }
  st8(dx + e, v);
}

// 2x2 average pool, NHWC
template <typename T>
__global__ __launch_bounds__(256) void avgpool2_fwd_kernel(int U, int H, int W, int C,
                                                           const T* __restrict__ x,
                                                           T* __restrict__ y) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t n = (int64_t)U * Ho * Wo * C;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  int64_t t = i / C;
  const int ox = (int)(t % Wo);
  t /= Wo;
  const int oy = (int)(t % Ho);
  const int u = (int)(t / Ho);
  const T* p = x + (((int64_t)u * H + 2 * oy) * W + 2 * ox) * C + c;
  const float s = Elem<T>::ld(p) + Elem<T>::ld(p + C) + Elem<T>::ld(p + (int64_t)W * C) +
                  Elem<T>::ld(p + (int64_t)W * C + C);
  Elem<T>::st(y + i, 0.25f * s);
}

template <typename T>
__global__ __launch_bounds__(256) void avgpool2_bwd_kernel(int U, int H, int W, int C,
                                                           const T* __restrict__ dy,
                                                           T* __restrict__ dx) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t n = (int64_t)U * H * W * C;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  int64_t t = i / C;
  const int ix = (int)(t % W);
  t /= W;
  const int iy = (int)(t % H);
  const int u = (int)(t / H);
  const int oy = iy / 2, ox = ix / 2;
  float v = 0.f;
  if (oy < Ho && ox < Wo) v = 0.25f * Elem<T>::ld(dy + (((int64_t)u * Ho + oy) * Wo + ox) * C + c);
  Elem<T>::st(dx + i, v);
}

// ---------------------------------------------------------------------------------------------
// Attention pool input (clip/model.py:77-84 with img_len = 2): the pair's two [C][7][7] maps are
// reshaped as [C][98] BEFORE the channel/spatial permute, so token tt (0..97), channel ch reads
// image (ch >= C/2), channel 2 (ch mod C/2) + (tt >= S), position tt mod S (S = 49); token 0 is the
// mean of the 98 tokens; positions add pos[t] for t <= S and pos[t - S - 1] after (the img_len
// positional quirk). feats NHWC [U][S][C]; pairimg [P][2] unique-image ids.
template <typename T>
__global__ __launch_bounds__(256) void pool_gather_fwd_kernel(int P, int S, int C,
                                                              const T* __restrict__ feats,
                                                              const int* __restrict__ pairimg,
                                                              const float* __restrict__ pos,
                                                              T* __restrict__ x) {
  const int p = blockIdx.y;
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= C) return;
  const int half = C / 2;
  const int img = pairimg[2 * p + (ch >= half ? 1 : 0)];
  const int cb = 2 * (ch % half);
  const T* f = feats + (int64_t)img * S * C;
  T* out = x + (int64_t)p * (2 * S + 1) * C;
  float sum = 0.f;
  for (int tt = 0; tt < 2 * S; ++tt) {
    const int src = cb + (tt >= S ? 1 : 0), s = tt % S;
    const float v = Elem<T>::ld(f + (int64_t)s * C + src);
    sum += v;
    const int t = tt + 1;
    Elem<T>::st(out + (int64_t)t * C + ch, v + pos[(int64_t)(t <= S ? t : t - S - 1) * C + ch]);
  }
  Elem<T>::st(out + ch, sum / (float)(2 * S) + pos[ch]);
}

// dfeats[u][s][src] = sum over the pairs holding image u in role r of (dx[p][1 + tt][ch] +
// dx[p][0][ch] / 2S), ch = src / 2 + r C/2, tt = s + S (src & 1). rolepairs[a][r][k]: the
// story-local pairs (N - 1 per role) holding image a in role r.
template <typename T>
__global__ __launch_bounds__(256) void pool_gather_bwd_kernel(int U, int N, int S, int C,
                                                              int npair,
                                                              const T* __restrict__ dx,
                                                              const int* __restrict__ rolepairs,
                                                              T* __restrict__ dfeats) {
  const int64_t n = (int64_t)U * S * C;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int src = (int)(i % C);
  const int64_t t = i / C;
  const int s = (int)(t % S);
  const int u = (int)(t / S);
  const int b = u / N, a = u - b * N;
  const int half = C / 2, T2 = 2 * S + 1;
  const int tt = s + (src & 1 ? S : 0);
  float acc = 0.f;
  for (int r = 0; r < 2; ++r) {
    const int ch = src / 2 + r * half;
    for (int k = 0; k < N - 1; ++k) {
      const int p = b * npair + rolepairs[(a * 2 + r) * (N - 1) + k];
      const T* d = dx + (int64_t)p * T2 * C;
      acc += Elem<T>::ld(d + (int64_t)(1 + tt) * C + ch) + Elem<T>::ld(d + ch) / (float)(2 * S);
    }
  }
  Elem<T>::st(dfeats + i, acc);
}

// attention-pool output (clip/model.py:99-101: cat([x, x], -1)) + visual position
// (lxrt:628-660: x_pos[w] + y_pos[h], 7 x 7 grid, repeated per image, token 0 = position 0) +
// token type (lxrt:670-705: image index of the token): y [P][T2][2 Ch], a [P][T2][Ch]
template <typename T>
__global__ __launch_bounds__(256) void pool_out_fwd_kernel(int64_t rows, int T2, int Ch, int G,
                                                           const T* __restrict__ a,
                                                           const float* __restrict__ xpos,
                                                           const float* __restrict__ ypos,
                                                           const float* __restrict__ ttype,
                                                           T* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int C2 = 2 * Ch;
  if (i >= rows * C2) return;
  const int c = (int)(i % C2);
  const int64_t r = i / C2;
  const int t = (int)(r % T2);
  const int S = G * G;
  const int q = t == 0 ? 0 : (t - 1) % S;  // grid position
  const int ty = t == 0 ? 0 : (t - 1) / S;  // image index = token type
  const float v = Elem<T>::ld(a + r * Ch + (c % Ch)) + xpos[(int64_t)(q / G) * C2 + c] +
                  ypos[(int64_t)(q % G) * C2 + c] + ttype[(int64_t)ty * C2 + c];
  Elem<T>::st(y + i, v);
}

// da[r][c] = dy[r][c] + dy[r][Ch + c]; colsum[t][c2] = sum_p dy[p][t][c2] (fixed order)
template <typename T>
__global__ __launch_bounds__(256) void pool_out_bwd_kernel(int64_t rows, int Ch,
                                                           const T* __restrict__ dy,
                                                           T* __restrict__ da) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * Ch) return;
  const int64_t r = i / Ch;
  const int c = (int)(i - r * Ch);
  const T* d = dy + r * 2 * Ch;
  Elem<T>::st(da + i, Elem<T>::ld(d + c) + Elem<T>::ld(d + Ch + c));
}

template <typename T>
__global__ __launch_bounds__(256) void token_colsum_kernel(int P, int T2, int C2,
                                                           const T* __restrict__ dy,
                                                           float* __restrict__ out) {
  const int t = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C2) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += Elem<T>::ld(dy + ((int64_t)p * T2 + t) * C2 + c);
  out[(int64_t)t * C2 + c] = s;
}

template <typename T>
inline unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

#define MMSEQ_DT_DISPATCH(dtype, KERNEL, ...)                                       \
  do {                                                                              \
    if ((dtype) == MMSEQ_BF16) { KERNEL(unsigned short, __VA_ARGS__); }             \
    else { KERNEL(float, __VA_ARGS__); }                                            \
  } while (0)

extern "C" mmseq_status mmseq_conv_im2col(int U, int H, int W, int C, int ks, int stride, int pad,
                                          int Kp, const void* x, void* cols, mmseq_dtype dtype,
                                          mmseq_stream stream) {
  MMSEQ_REQUIRE(U >= 0 && H > 0 && W > 0 && C > 0 && ks > 0 && stride > 0 && pad >= 0 &&
                    Kp >= ks * ks * C, "conv_im2col: bad sizes");
  MMSEQ_REQUIRE(x && cols, "conv_im2col: null buffer");
  if (U == 0) return MMSEQ_OK;
  ConvGeom g{U, H, W, C, (H + 2 * pad - ks) / stride + 1, (W + 2 * pad - ks) / stride + 1, ks,
             stride, pad, Kp};
  const int64_t rows = (int64_t)U * g.Ho * g.Wo;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool al = ((uintptr_t)cols & 15) == 0 && Kp % 8 == 0;
  const int mode = al && C % 8 == 0 && ((uintptr_t)x & 15) == 0 ? 1 : al ? 2 : 0;
  const dim3 grid((unsigned)((rows * (Kp / (mode ? 8 : 1)) + 255) / 256));
#define LAUNCH(T, M) hipLaunchKernelGGL((im2col_nhwc_kernel<T, M>), grid, dim3(256), 0, s, g, \
                                        (const T*)x, (T*)cols)
#define LAUNCH3(T, _) \
  if (mode == 1) LAUNCH(T, 1); else if (mode == 2) LAUNCH(T, 2); else LAUNCH(T, 0)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH3, 0);
#undef LAUNCH3
#undef LAUNCH
  return mmseq_check_launch("conv_im2col");
}

extern "C" mmseq_status mmseq_conv_col2im(int U, int H, int W, int C, int ks, int stride, int pad,
                                          int Kp, const void* dcols, void* dx, mmseq_dtype dtype,
                                          mmseq_stream stream) {
  MMSEQ_REQUIRE(U >= 0 && H > 0 && W > 0 && C > 0 && ks > 0 && stride > 0 && pad >= 0 &&
                    Kp >= ks * ks * C, "conv_col2im: bad sizes");
  MMSEQ_REQUIRE(dcols && dx, "conv_col2im: null buffer");
  if (U == 0) return MMSEQ_OK;
  ConvGeom g{U, H, W, C, (H + 2 * pad - ks) / stride + 1, (W + 2 * pad - ks) / stride + 1, ks,
             stride, pad, Kp};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool vec = C % 8 == 0 && Kp % 8 == 0 && (((uintptr_t)dcols | (uintptr_t)dx) & 15) == 0;
  const int64_t n = (int64_t)U * H * W * (vec ? C / 8 : C);
  const dim3 grid((unsigned)((n + 255) / 256));
#define LAUNCH(T, _)                                                                          \
  if (vec)                                                                                    \
    hipLaunchKernelGGL((col2im_nhwc_kernel<T, 8>), grid, dim3(256), 0, s, g, (const T*)dcols, \
                       (T*)dx);                                                               \
  else                                                                                        \
    hipLaunchKernelGGL((col2im_nhwc_kernel<T, 1>), grid, dim3(256), 0, s, g, (const T*)dcols, (T*)dx)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("conv_col2im");
}

extern "C" int64_t mmseq_bn_workspace(int64_t rows, int C) {
  if (rows < 0 || C <= 0 || !bn_shape_ok(C)) return 0;
  return (3 * (int64_t)bn_plan(rows, C).nch * C + 2 * (int64_t)C) * (int64_t)sizeof(float);
}

extern "C" mmseq_status mmseq_bn_fwd(int64_t rows, int C, const void* x, const float* gamma,
                                     const float* beta, const void* resid, int relu, int train,
                                     float eps, float momentum, double n_ref, float* mean,
                                     float* rstd, float* run_mean, float* run_var, void* y,
                                     float* workspace, int64_t workspace_bytes,
                                     mmseq_dtype dtype, mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && C > 0 && bn_shape_ok(C),
                "bn_fwd: C must be 8 x a power of two up to 512, or a multiple of 512");
  MMSEQ_REQUIRE(x && gamma && beta && mean && rstd && y, "bn_fwd: null buffer");
  MMSEQ_REQUIRE(train || (run_mean && run_var), "bn_fwd: eval needs running statistics");
  MMSEQ_REQUIRE((((uintptr_t)x | (uintptr_t)resid | (uintptr_t)y | (uintptr_t)mean |
                  (uintptr_t)rstd | (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0,
                "bn_fwd: buffers must be 16-byte aligned");
  if (rows == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (train) {
    MMSEQ_REQUIRE(workspace && workspace_bytes >= mmseq_bn_workspace(rows, C),
                  "bn_fwd: workspace too small");
    const BnPlan pl = bn_plan(rows, C);
#define LAUNCH(T, _) hipLaunchKernelGGL(bn_stats_partial_kernel<T>, dim3(pl.gx, pl.nch), dim3(256), 0, \
                                        s, rows, C, pl, (const T*)x, workspace)
    MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3((C + 31) / 32), dim3(1024), 0, s, C, pl.nch,
                       workspace, eps, momentum, n_ref, mean, rstd, run_mean, run_var);
  } else {
    // eval: the running statistics, as mean / rstd for the apply and the backward
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, eps,
                       run_mean, run_var, mean, rstd);
  }
  const int64_t n8 = rows * C / 8;
#define LAUNCH(T, _)                                                                        \
  hipLaunchKernelGGL(bn_apply_kernel<T>, dim3((n8 + 255) / 256), dim3(256), 0, s, n8, C,     \
                     (const T*)x, mean, rstd, gamma, beta, (const T*)resid, relu, (T*)y)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("bn_fwd");
}

extern "C" mmseq_status mmseq_bn_bwd(int64_t rows, int C, const void* dy, const void* y,
                                     const void* x, const float* mean, const float* rstd,
                                     const float* gamma, int train, float* dgamma, float* dbeta,
                                     void* dx, void* dres, float* workspace,
                                     int64_t workspace_bytes, mmseq_dtype dtype,
                                     mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && C > 0 && bn_shape_ok(C),
                "bn_bwd: C must be 8 x a power of two up to 512, or a multiple of 512");
  MMSEQ_REQUIRE(dy && x && mean && rstd && gamma && dx && workspace, "bn_bwd: null buffer");
  MMSEQ_REQUIRE(workspace_bytes >= mmseq_bn_workspace(rows, C), "bn_bwd: workspace too small");
  MMSEQ_REQUIRE((((uintptr_t)dy | (uintptr_t)y | (uintptr_t)x | (uintptr_t)dx | (uintptr_t)dres |
                  (uintptr_t)mean | (uintptr_t)rstd | (uintptr_t)gamma | (uintptr_t)workspace) &
                 15) == 0, "bn_bwd: buffers must be 16-byte aligned");
  if (rows == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const BnPlan pl = bn_plan(rows, C);
  float* sums = workspace + 3 * (int64_t)pl.nch * C;
#define LAUNCH(T, _) hipLaunchKernelGGL(bn_bwd_partial_kernel<T>, dim3(pl.gx, pl.nch), dim3(256), 0, \
                                        s, rows, C, pl, (const T*)dy, (const T*)y, (const T*)x, \
                                        mean, rstd, workspace)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3((C + 31) / 32), dim3(1024), 0, s, C, pl.nch,
                     workspace, sums, dgamma, dbeta);
  const int64_t n8 = rows * C / 8;
#define LAUNCH(T, _)                                                                          \
  hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3((n8 + 255) / 256), dim3(256), 0, s, n8, C, rows, \
                     (const T*)dy, (const T*)y, (const T*)x, mean, rstd, gamma, sums, train,   \
                     (T*)dx, (T*)dres)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("bn_bwd");
}

extern "C" mmseq_status mmseq_avgpool2(int U, int H, int W, int C, const void* x, void* y,
                                       int backward, mmseq_dtype dtype, mmseq_stream stream) {
  MMSEQ_REQUIRE(U >= 0 && H >= 2 && W >= 2 && C > 0, "avgpool2: bad sizes");
  MMSEQ_REQUIRE(x && y, "avgpool2: null buffer");
  if (U == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!backward) {
    const int64_t n = (int64_t)U * (H / 2) * (W / 2) * C;
#define LAUNCH(T, _) hipLaunchKernelGGL(avgpool2_fwd_kernel<T>, dim3(blocks<T>(n)), dim3(256), 0, s, \
                                        U, H, W, C, (const T*)x, (T*)y)
    MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  } else {
    const int64_t n = (int64_t)U * H * W * C;
#define LAUNCH(T, _) hipLaunchKernelGGL(avgpool2_bwd_kernel<T>, dim3(blocks<T>(n)), dim3(256), 0, s, \
                                        U, H, W, C, (const T*)x, (T*)y)
    MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  }
  return mmseq_check_launch("avgpool2");
}

extern "C" mmseq_status mmseq_attnpool_gather(int P, int S, int C, const void* feats,
                                              const int32_t* pairimg, const float* pos, void* x,
                                              mmseq_dtype dtype, mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && S > 0 && C > 0 && C % 2 == 0, "attnpool_gather: bad sizes");
  MMSEQ_REQUIRE(feats && pairimg && pos && x, "attnpool_gather: null buffer");
  if (P == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define LAUNCH(T, _) hipLaunchKernelGGL(pool_gather_fwd_kernel<T>, dim3((C + 255) / 256, P), dim3(256), \
                                        0, s, P, S, C, (const T*)feats, (const int*)pairimg, pos, (T*)x)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("attnpool_gather");
}

extern "C" mmseq_status mmseq_attnpool_gather_bwd(int U, int N, int S, int C, int npair,
                                                  const void* dx, const int32_t* rolepairs,
                                                  void* dfeats, mmseq_dtype dtype,
                                                  mmseq_stream stream) {
  MMSEQ_REQUIRE(U >= 0 && N >= 2 && S > 0 && C > 0 && C % 2 == 0 && npair == N * (N - 1),
                "attnpool_gather_bwd: bad sizes");
  MMSEQ_REQUIRE(dx && rolepairs && dfeats, "attnpool_gather_bwd: null buffer");
  if (U == 0) return MMSEQ_OK;
  const int64_t n = (int64_t)U * S * C;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define LAUNCH(T, _) hipLaunchKernelGGL(pool_gather_bwd_kernel<T>, dim3(blocks<T>(n)), dim3(256), 0, s, \
                                        U, N, S, C, npair, (const T*)dx, (const int*)rolepairs,  \
                                        (T*)dfeats)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("attnpool_gather_bwd");
}

extern "C" mmseq_status mmseq_attnpool_out(int64_t rows, int T2, int Ch, int G, const void* a,
                                           const float* xpos, const float* ypos,
                                           const float* ttype, void* y, mmseq_dtype dtype,
                                           mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && T2 == 2 * G * G + 1 && Ch > 0, "attnpool_out: bad sizes");
  MMSEQ_REQUIRE(a && xpos && ypos && ttype && y, "attnpool_out: null buffer");
  if (rows == 0) return MMSEQ_OK;
  const int64_t n = rows * 2 * Ch;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define LAUNCH(T, _) hipLaunchKernelGGL(pool_out_fwd_kernel<T>, dim3(blocks<T>(n)), dim3(256), 0, s, \
                                        rows, T2, Ch, G, (const T*)a, xpos, ypos, ttype, (T*)y)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("attnpool_out");
}

extern "C" mmseq_status mmseq_attnpool_out_bwd(int P, int T2, int Ch, const void* dy, void* da,
                                               float* token_colsum, mmseq_dtype dtype,
                                               mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && T2 > 0 && Ch > 0, "attnpool_out_bwd: bad sizes");
  MMSEQ_REQUIRE(dy && da && token_colsum, "attnpool_out_bwd: null buffer");
  if (P == 0) return MMSEQ_OK;
  const int64_t rows = (int64_t)P * T2;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define LAUNCH(T, _)                                                                           \
  hipLaunchKernelGGL(pool_out_bwd_kernel<T>, dim3(blocks<T>(rows * Ch)), dim3(256), 0, s, rows, \
                     Ch, (const T*)dy, (T*)da);                                                 \
  hipLaunchKernelGGL(token_colsum_kernel<T>, dim3((2 * Ch + 255) / 256, T2), dim3(256), 0, s, P, \
                     T2, 2 * Ch, (const T*)dy, token_colsum)
  MMSEQ_DT_DISPATCH(dtype, LAUNCH, 0);
#undef LAUNCH
  return mmseq_check_launch("attnpool_out_bwd");
}
