// Token-side and patch-side embedding kernels, writing straight into the activation buffers.
//   text:  BertEmbeddings (lxrt/modeling.py:342-370) fused with the image-text concat (:1093)
//   image: CLIP ViT patchify + class token + img_len=2 positional quirk + ln_pre
//          (clip/model.py:262-278), with the per-pair image gather of
//          process_images (process_inputs_for_berson.py:82-97) done on device.
#include "common.h"

mmseq_status ln_reduce_partials(int nb, int cols, const float* ws, float* dg, float* db,
                                hipStream_t s);
int64_t mmseq_reduce_extra(int nb, int W);

namespace {

constexpr int MAXV = 16;
constexpr int RPB = 64;

// ---------------------------------------------------------------------------------------------
// text embeddings
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(int P, int Lt, int H,
                                                        const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ tt,
                                                        const float* __restrict__ word,
                                                        const float* __restrict__ pos,
                                                        const float* __restrict__ type,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        T* __restrict__ joint, int64_t ld_pair,
                                                        float* __restrict__ mean,
                                                        float* __restrict__ rstd, Drop dr) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (int64_t)P * Lt) return;
  const int p = r / Lt, t = r % Lt;
  const float* wr = word + ids[r] * H;
  const float* pr = pos + (int64_t)t * H;
  const float* tr = type + (tt ? tt[r] : 0) * H;
  float v[MAXV], s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    v[j] = c < H ? wr[c] + pr[c] + tr[c] : 0.f;
    s += v[j];
  }
  const float mu = wave_sum(s) / H;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    float d = c < H ? v[j] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / H + eps);
  T* out = joint + (int64_t)p * ld_pair + (int64_t)t * H;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    if (c < H)
      Elem<T>::st(out + c, ((v[j] - mu) * rs * gamma[c] + beta[c]) * drop_mul(dr, (uint64_t)r * H + c));
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

// LN backward on recomputed e; de -> ws_de [P*Lt][H] (f32); word/type scatter with atomics
// (row 0 skipped: padding_idx = 0 on all three tables, lxrt/modeling.py:347-349).
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(int P, int Lt, int H,
                                                        const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ tt,
                                                        const float* __restrict__ word,
                                                        const float* __restrict__ pos,
                                                        const float* __restrict__ type,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const T* __restrict__ djoint,
                                                        int64_t ld_pair, float* __restrict__ dword,
                                                        float* __restrict__ dtype_tab,
                                                        float* __restrict__ ws_de,
                                                        float* __restrict__ ws_ln, Drop dr) {
  __shared__ float red[4][2][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t rows = (int64_t)P * Lt;
  float pg[MAXV], pb[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) pg[j] = pb[j] = 0.f;
  const int64_t rbeg = (int64_t)blockIdx.x * RPB;
  for (int64_t r = rbeg + wave; r < rbeg + RPB && r < rows; r += 4) {
    const int p = r / Lt, t = r % Lt;
    const int64_t id = ids[r];
    const int64_t ty = tt ? tt[r] : 0;
    const float* wr = word + id * H;
    const float* pr = pos + (int64_t)t * H;
    const float* tr = type + ty * H;
    const T* dyr = djoint + (int64_t)p * ld_pair + (int64_t)t * H;
    const float mu = mean[r], rs = rstd[r];
    float xh[MAXV], gdy[MAXV], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      int c = j * 64 + lane;
      if (c < H) {
        float xv = (wr[c] + pr[c] + tr[c] - mu) * rs;
        float d = Elem<T>::ld(dyr + c) * drop_mul(dr, (uint64_t)r * H + c);
        xh[j] = xv;
        gdy[j] = d * gamma[c];
        pg[j] += d * xv;
        pb[j] += d;
        s1 += gdy[j];
        s2 += gdy[j] * xv;
      } else {
        xh[j] = gdy[j] = 0.f;
      }
    }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      int c = j * 64 + lane;
      if (c < H) {
        float de = rs * (gdy[j] - s1 - xh[j] * s2);
        ws_de[r * H + c] = de;
        if (id != 0) atomicAdd(dword + id * H + c, de);
        if (ty != 0 && dtype_tab) atomicAdd(dtype_tab + ty * H + c, de);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    if (c < H) {
      red[wave][0][c] = pg[j];
      red[wave][1][c] = pb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256) {
    ws_ln[((int64_t)blockIdx.x * 2 + 0) * H + c] =
        red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    ws_ln[((int64_t)blockIdx.x * 2 + 1) * H + c] =
        red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
  }
}

// dpos[t][c] += sum_p de[p][t][c], t >= 1 (position ids are 0..Lt-1, lxrt:358; row 0 = padding)
__global__ __launch_bounds__(256) void embed_pos_kernel(int P, int Lt, int H,
                                                        const float* __restrict__ de,
                                                        float* __restrict__ dpos) {
  const int t = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (t == 0 || c >= H) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += de[((int64_t)p * Lt + t) * H + c];
  dpos[(int64_t)t * H + c] += s;
}

// ---------------------------------------------------------------------------------------------
// ViT patch path
// ---------------------------------------------------------------------------------------------
// Any patch size: one workgroup (64 lanes) per patch row; lane t < 3 ps copies the ps pixels of
// (channel t / ps, kernel row t % ps) — contiguous in the image — and the columns K .. ldk - 1 are
// zero-filled (K padded to the GEMM's K granularity, e.g. 588 -> 640 for ViT-L/14).
template <typename T>
__global__ __launch_bounds__(64) void im2col_kernel(int64_t rows, int N, int npair, int R, int ps,
                                                    int64_t ldk, const float* __restrict__ images,
                                                    const int64_t* __restrict__ pairs,
                                                    T* __restrict__ out) {
  const int g = R / ps, gg = g * g, K = 3 * ps * ps;
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const int patch = (int)(row % gg);
  const int64_t rest = row / gg;
  const int s = (int)(rest & 1);
  const int64_t pj = rest >> 1;
  const int b = (int)(pj / npair);
  const int img = (int)pairs[pj * 2 + s];
  const int py = patch / g, px = patch % g;
  const float* src_img = images + ((int64_t)b * N + img) * 3 * R * R;
  T* dst = out + row * ldk;
  for (int t = threadIdx.x; t < 3 * ps; t += 64) {
    const int c = t / ps, ky = t % ps;
    const float* src = src_img + ((int64_t)c * R + py * ps + ky) * R + px * ps;
    T* d = dst + (c * ps + ky) * ps;
    for (int kx = 0; kx < ps; ++kx) Elem<T>::st(d + kx, src[kx]);
  }
  for (int col = K + threadIdx.x; col < ldk; col += 64) Elem<T>::st(dst + col, 0.f);
}

// bf16 patches: one row per 96 threads, 8 consecutive pixels of one (channel, patch row) per
// thread (two 16-byte loads, one 16-byte store); the row's pair / image decode is done once
// per row instead of per element (64-bit divisions). Requires ps % 8 == 0 and ldk == K.
__global__ __launch_bounds__(192) void im2col_bf16_kernel(int64_t rows, int N, int npair, int R,
                                                         int ps, const float* __restrict__ images,
                                                         const int64_t* __restrict__ pairs,
                                                         unsigned short* __restrict__ out) {
  const int g = R / ps, gg = g * g, K = 3 * ps * ps;
  const int64_t row = (int64_t)blockIdx.x * 2 + threadIdx.x / 96;
  const int chunk = threadIdx.x % 96;
  if (row >= rows) return;
  const int patch = (int)(row % gg);
  const int64_t rest = row / gg;
  const int s = (int)(rest & 1);
  const int64_t pj = rest >> 1;
  const int b = (int)(pj / npair);
  const int img = (int)pairs[pj * 2 + s];
  const int py = patch / g, px = patch % g;
  const float* src_img = images + ((int64_t)b * N + img) * 3 * R * R;
  for (int c8 = chunk; c8 * 8 < K; c8 += 96) {
    const int col = c8 * 8;
    const int c = col / (ps * ps), ky = (col / ps) % ps, kx = col % ps;
    const float* src = src_img + ((int64_t)c * R + py * ps + ky) * R + px * ps + kx;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(src);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(src + 4);
    u16x8 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = f2bf(v0[r]);
      o[4 + r] = f2bf(v1[r]);
    }
    *reinterpret_cast<u16x8*>(out + row * K + col) = o;
  }
}

__device__ __forceinline__ int vit_pos_row(int t, int gg) {
  // clip/model.py:271-275 with img_len = 2: rows 0..gg for CLS + img0, rows 0..gg-1 for img1
  return t <= gg ? t : t - gg - 1;
}

template <typename T>
__global__ __launch_bounds__(256) void vit_embed_fwd_kernel(int P, int ntok, int W, int gg,
                                                            const T* __restrict__ patch_out,
                                                            const float* __restrict__ cls,
                                                            const float* __restrict__ pos,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            float eps, T* __restrict__ x,
                                                            T* __restrict__ y,
                                                            float* __restrict__ mean,
                                                            float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (int64_t)P * ntok) return;
  const int p = r / ntok, t = r % ntok;
  const float* pr = pos + (int64_t)vit_pos_row(t, gg) * W;
  const T* src = t > 0 ? patch_out + ((int64_t)p * (ntok - 1) + (t - 1)) * W : nullptr;
  float v[MAXV], s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    float a = 0.f;
    if (c < W) a = (t == 0 ? cls[c] : Elem<T>::ld(src + c)) + pr[c];
    v[j] = a;
    s += a;
  }
  T* xr = x + r * W;
  T* yr = y + r * W;
  // the stored pre-LN x is the rounded value; statistics use the same rounded values so that the
  // backward (which re-reads x) sees a consistent input
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    if (c < W) {
      Elem<T>::st(xr + c, v[j]);
      v[j] = Elem<T>::ld(xr + c);
    }
  }
  s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) s += (j * 64 + lane < W) ? v[j] : 0.f;
  const float mu = wave_sum(s) / W;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    float d = c < W ? v[j] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / W + eps);
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    if (c < W) Elem<T>::st(yr + c, (v[j] - mu) * rs * gamma[c] + beta[c]);
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void vit_embed_bwd_kernel(int P, int ntok, int W,
                                                            const T* __restrict__ dy,
                                                            const T* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ gamma,
                                                            T* __restrict__ dpatch,
                                                            float* __restrict__ dx0,
                                                            float* __restrict__ ws_ln) {
  __shared__ float red[4][2][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t rows = (int64_t)P * ntok;
  float pg[MAXV], pb[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) pg[j] = pb[j] = 0.f;
  const int64_t rbeg = (int64_t)blockIdx.x * RPB;
  for (int64_t r = rbeg + wave; r < rbeg + RPB && r < rows; r += 4) {
    const int p = r / ntok, t = r % ntok;
    const T* xr = x + r * W;
    const T* dyr = dy + r * W;
    const float mu = mean[r], rs = rstd[r];
    float xh[MAXV], gdy[MAXV], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      int c = j * 64 + lane;
      if (c < W) {
        float xv = (Elem<T>::ld(xr + c) - mu) * rs;
        float d = Elem<T>::ld(dyr + c);
        xh[j] = xv;
        gdy[j] = d * gamma[c];
        pg[j] += d * xv;
        pb[j] += d;
        s1 += gdy[j];
        s2 += gdy[j] * xv;
      } else {
        xh[j] = gdy[j] = 0.f;
      }
    }
    s1 = wave_sum(s1) / W;
    s2 = wave_sum(s2) / W;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      int c = j * 64 + lane;
      if (c < W) {
        float d = rs * (gdy[j] - s1 - xh[j] * s2);
        if (t == 0) dx0[(int64_t)p * W + c] = d;
        else Elem<T>::st(dpatch + ((int64_t)p * (ntok - 1) + t - 1) * W + c, d);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int c = j * 64 + lane;
    if (c < W) {
      red[wave][0][c] = pg[j];
      red[wave][1][c] = pb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < W; c += 256) {
    ws_ln[((int64_t)blockIdx.x * 2 + 0) * W + c] =
        red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    ws_ln[((int64_t)blockIdx.x * 2 + 1) * W + c] =
        red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
  }
}

// dpos / dcls reductions over pairs (deterministic, fixed order)
template <typename T>
__global__ __launch_bounds__(256) void vit_pos_kernel(int P, int ntok, int W, int gg,
                                                      const T* __restrict__ dpatch,
                                                      const float* __restrict__ dx0,
                                                      float* __restrict__ dcls,
                                                      float* __restrict__ dpos) {
  const int r = blockIdx.y;  // 0..gg  (gg+1 = cls row)
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= W) return;
  const int64_t ps = (int64_t)(ntok - 1) * W;
  float s = 0.f;
  if (r == gg + 1) {
    for (int p = 0; p < P; ++p) s += dx0[(int64_t)p * W + c];
    dcls[c] += s;
    return;
  }
  // tokens t with vit_pos_row(t) == r: t = r (if r <= gg) and t = r + gg + 1 (if r < gg)
  for (int p = 0; p < P; ++p) {
    const T* dp = dpatch + p * ps;
    if (r == 0) s += dx0[(int64_t)p * W + c];
    else s += Elem<T>::ld(dp + (int64_t)(r - 1) * W + c);
    if (r < gg && r + gg + 1 < ntok) s += Elem<T>::ld(dp + (int64_t)(r + gg) * W + c);
  }
  dpos[(int64_t)r * W + c] += s;
}

}  // namespace

extern "C" mmseq_status mmseq_embed_ln_fwd(int P, int Lt, int H, const int64_t* ids,
                                           const int64_t* tt, const float* word, const float* pos,
                                           const float* type, const float* gamma,
                                           const float* beta, float eps, void* joint,
                                           int64_t ld_pair, float* mean, float* rstd,
                                           mmseq_dtype dtype, const mmseq_dropout* drop,
                                           mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && Lt > 0 && H > 0 && H <= 1024, "embed: bad sizes");
  MMSEQ_REQUIRE(ids && word && pos && type && gamma && beta && joint && mean && rstd,
                "embed: null buffer");
  if (P == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)(((int64_t)P * Lt + 3) / 4));
  if (dtype == MMSEQ_F32)
    hipLaunchKernelGGL(embed_fwd_kernel<float>, grid, dim3(256), 0, s, P, Lt, H, ids, tt, word,
                       pos, type, gamma, beta, eps, (float*)joint, ld_pair, mean, rstd,
                       make_drop(drop));
  else
    hipLaunchKernelGGL(embed_fwd_kernel<unsigned short>, grid, dim3(256), 0, s, P, Lt, H, ids, tt,
                       word, pos, type, gamma, beta, eps, (unsigned short*)joint, ld_pair, mean,
                       rstd, make_drop(drop));
  return mmseq_check_launch("embed_ln_fwd");
}

extern "C" int64_t mmseq_embed_ln_bwd_workspace(int P, int Lt, int H) {
  const int64_t rows = (int64_t)P * Lt;
  const int nb = (int)((rows + RPB - 1) / RPB);
  return rows * H + (int64_t)nb * 2 * H + mmseq_reduce_extra(nb, 2 * H);
}

extern "C" mmseq_status mmseq_embed_ln_bwd(int P, int Lt, int H, const int64_t* ids,
                                           const int64_t* tt, const float* word, const float* pos,
                                           const float* type, const float* gamma,
                                           const float* mean, const float* rstd,
                                           const void* djoint, int64_t ld_pair, float* dword,
                                           float* dpos, float* dtype_tab, float* dgamma,
                                           float* dbeta, float* workspace, mmseq_dtype dtype,
                                           const mmseq_dropout* drop, mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && Lt > 0 && H > 0 && H <= 1024, "embed_bwd: bad sizes");
  MMSEQ_REQUIRE(workspace && djoint && dword && dpos, "embed_bwd: null buffer");
  if (P == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t rows = (int64_t)P * Lt;
  const int nb = (int)((rows + RPB - 1) / RPB);
  float* ws_de = workspace;
  float* ws_ln = workspace + rows * H;
  if (dtype == MMSEQ_F32)
    hipLaunchKernelGGL(embed_bwd_kernel<float>, dim3(nb), dim3(256), 0, s, P, Lt, H, ids, tt,
                       word, pos, type, gamma, mean, rstd, (const float*)djoint, ld_pair, dword,
                       dtype_tab, ws_de, ws_ln, make_drop(drop));
  else
    hipLaunchKernelGGL(embed_bwd_kernel<unsigned short>, dim3(nb), dim3(256), 0, s, P, Lt, H, ids,
                       tt, word, pos, type, gamma, mean, rstd, (const unsigned short*)djoint,
                       ld_pair, dword, dtype_tab, ws_de, ws_ln, make_drop(drop));
  hipLaunchKernelGGL(embed_pos_kernel, dim3((H + 255) / 256, Lt), dim3(256), 0, s, P, Lt, H,
                     ws_de, dpos);
  mmseq_status st = mmseq_check_launch("embed_ln_bwd");
  if (st) return st;
  return ln_reduce_partials(nb, H, ws_ln, dgamma, dbeta, s);
}

extern "C" mmseq_status mmseq_vit_im2col(int B, int N, int npair, int R, int ps,
                                         const float* images, const int64_t* pairs, void* patches,
                                         int64_t ld_patch, mmseq_dtype dtype, mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && N > 0 && npair > 0 && ps > 0 && R % ps == 0, "im2col: bad sizes");
  MMSEQ_REQUIRE(images && pairs && patches, "im2col: null buffer");
  MMSEQ_REQUIRE(ld_patch >= 3 * ps * ps, "im2col: ld_patch < 3 ps^2");
  if (B == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t rows = (int64_t)B * npair * 2 * (R / ps) * (R / ps);
  MMSEQ_REQUIRE(rows < (1ll << 31), "im2col: too many patches");
  if (dtype == MMSEQ_BF16 && ps % 8 == 0 && R % 4 == 0 && ld_patch == 3 * ps * ps &&
      (((uintptr_t)images) & 15) == 0 && (((uintptr_t)patches) & 15) == 0) {
    hipLaunchKernelGGL(im2col_bf16_kernel, dim3((unsigned)((rows + 1) / 2)), dim3(192), 0, s, rows, N,
                       npair, R, ps, images, pairs, (unsigned short*)patches);
  } else if (dtype == MMSEQ_F32) {
    hipLaunchKernelGGL(im2col_kernel<float>, dim3((unsigned)rows), dim3(64), 0, s, rows, N, npair,
                       R, ps, ld_patch, images, pairs, (float*)patches);
  } else {
    hipLaunchKernelGGL(im2col_kernel<unsigned short>, dim3((unsigned)rows), dim3(64), 0, s, rows, N,
                       npair, R, ps, ld_patch, images, pairs, (unsigned short*)patches);
  }
  return mmseq_check_launch("vit_im2col");
}

extern "C" mmseq_status mmseq_vit_embed_fwd(int P, int ntok, int W, int npatch_img,
                                            const void* patch_out, const float* cls,
                                            const float* pos, const float* gamma,
                                            const float* beta, float eps, void* x, void* y,
                                            float* mean, float* rstd, mmseq_dtype dtype,
                                            mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && W > 0 && W <= 1024 && ntok == 1 + 2 * npatch_img,
                "vit_embed: requires img_len = 2 (ntok = 1 + 2*npatch) and W <= 1024");
  if (P == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)(((int64_t)P * ntok + 3) / 4));
  if (dtype == MMSEQ_F32)
    hipLaunchKernelGGL(vit_embed_fwd_kernel<float>, grid, dim3(256), 0, s, P, ntok, W, npatch_img,
                       (const float*)patch_out, cls, pos, gamma, beta, eps, (float*)x, (float*)y,
                       mean, rstd);
  else
    hipLaunchKernelGGL(vit_embed_fwd_kernel<unsigned short>, grid, dim3(256), 0, s, P, ntok, W,
                       npatch_img, (const unsigned short*)patch_out, cls, pos, gamma, beta, eps,
                       (unsigned short*)x, (unsigned short*)y, mean, rstd);
  return mmseq_check_launch("vit_embed_fwd");
}

extern "C" int64_t mmseq_vit_embed_bwd_workspace(int P, int ntok, int W) {
  const int64_t rows = (int64_t)P * ntok;
  const int nb = (int)((rows + RPB - 1) / RPB);
  return (int64_t)P * W + (int64_t)nb * 2 * W + mmseq_reduce_extra(nb, 2 * W);
}

extern "C" mmseq_status mmseq_vit_embed_bwd(int P, int ntok, int W, int npatch_img,
                                            const void* dy, const void* x, const float* mean,
                                            const float* rstd, const float* gamma,
                                            void* dpatch_out, float* dcls, float* dpos,
                                            float* dgamma, float* dbeta, float* workspace,
                                            mmseq_dtype dtype, mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && W > 0 && W <= 1024 && ntok == 1 + 2 * npatch_img, "vit_embed_bwd: sizes");
  MMSEQ_REQUIRE(dy && x && dpatch_out && dcls && dpos && workspace, "vit_embed_bwd: null buffer");
  if (P == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t rows = (int64_t)P * ntok;
  const int nb = (int)((rows + RPB - 1) / RPB);
  float* dx0 = workspace;
  float* ws_ln = workspace + (int64_t)P * W;
  dim3 gpos((W + 255) / 256, npatch_img + 2);
  if (dtype == MMSEQ_F32) {
    hipLaunchKernelGGL(vit_embed_bwd_kernel<float>, dim3(nb), dim3(256), 0, s, P, ntok, W,
                       (const float*)dy, (const float*)x, mean, rstd, gamma, (float*)dpatch_out,
                       dx0, ws_ln);
    hipLaunchKernelGGL(vit_pos_kernel<float>, gpos, dim3(256), 0, s, P, ntok, W, npatch_img,
                       (const float*)dpatch_out, dx0, dcls, dpos);
  } else {
    hipLaunchKernelGGL(vit_embed_bwd_kernel<unsigned short>, dim3(nb), dim3(256), 0, s, P, ntok,
                       W, (const unsigned short*)dy, (const unsigned short*)x, mean, rstd, gamma,
                       (unsigned short*)dpatch_out, dx0, ws_ln);
    hipLaunchKernelGGL(vit_pos_kernel<unsigned short>, gpos, dim3(256), 0, s, P, ntok, W,
                       npatch_img, (const unsigned short*)dpatch_out, dx0, dcls, dpos);
  }
  mmseq_status st = mmseq_check_launch("vit_embed_bwd");
  if (st) return st;
  return ln_reduce_partials(nb, W, ws_ln, dgamma, dbeta, s);
}
