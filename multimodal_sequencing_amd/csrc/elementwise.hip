// HBM-bound utilities: casts / weight shadows, bias-gradient column sums, activations,
// sum of squares (clip_grad_norm_), fused AdamW over the flat parameter buffer.
#include <math.h>

#include "common.h"

namespace {

template <typename TS, typename TD>
__global__ __launch_bounds__(256) void cast_kernel(int64_t n, const TS* __restrict__ s,
                                                   TD* __restrict__ d) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    Elem<TD>::st(d + i, Elem<TS>::ld(s + i));
}

// 32x32 tiles through LDS (+1 pad: conflict-free column reads)
template <typename TD>
__global__ __launch_bounds__(256) void transpose_kernel(int rows, int cols, const float* __restrict__ s,
                                                        TD* __restrict__ d) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  for (int k = ty; k < 32; k += 8) {
    int r = r0 + k, c = c0 + tx;
    t[k][tx] = (r < rows && c < cols) ? s[(int64_t)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    int c = c0 + k, r = r0 + tx;
    if (c < cols && r < rows) Elem<TD>::st(d + (int64_t)c * rows + r, t[tx][k]);
  }
}

// Many fp32 [rows][cols] matrices -> their bf16 / fp32 transposes in one launch (the per-step
// refresh of a parameter store's transposed dgrad shadows): desc[m] = {rows, cols, src offset,
// dst offset, first tile} (elements; 64 x 64 tiles numbered matrix by matrix), one workgroup per
// tile, 16-byte fp32 reads along a source row, 8-byte writes along a destination row.
template <typename TD>
__global__ __launch_bounds__(256) void transpose_batch_kernel(int n, const int64_t* __restrict__ desc,
                                                              const float* __restrict__ src,
                                                              TD* __restrict__ dst) {
  __shared__ float t[64][65];
  const int64_t tile = blockIdx.x;
  int lo = 0, hi = n - 1;  // the last matrix whose first tile <= this tile (uniform)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * 5 + 4] <= tile) lo = mid; else hi = mid - 1;
  }
  const int rows = (int)desc[lo * 5], cols = (int)desc[lo * 5 + 1];
  const float* s = src + desc[lo * 5 + 2];
  TD* d = dst + desc[lo * 5 + 3];
  const int tc = (cols + 63) >> 6;
  const int64_t k = tile - desc[lo * 5 + 4];
  const int r0 = (int)(k / tc) * 64, c0 = (int)(k % tc) * 64;
  const int tid = threadIdx.x;
  const bool vec = (cols & 3) == 0 && (desc[lo * 5 + 2] & 3) == 0;  // 16-byte aligned source rows
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // 64 rows x 16 quads, 16 rows per pass
    const int rr = p * 16 + (tid >> 4), cq = (tid & 15) * 4;
    const int r = r0 + rr, c = c0 + cq;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < rows) {
      if (vec && c + 3 < cols) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(s + (int64_t)r * cols + c);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
      } else {
        for (int e = 0; e < 4; ++e)
          if (c + e < cols) v[e] = s[(int64_t)r * cols + c + e];
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) t[rr][cq + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // destination row = source column c0 + cc, 4 source rows per lane
    const int cc = p * 16 + (tid >> 4), rq = (tid & 15) * 4;
    const int c = c0 + cc, r = r0 + rq;
    if (c >= cols) continue;
    TD* o = d + (int64_t)c * rows + r;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (r + e < rows) Elem<TD>::st(o + e, t[rq + e][cc]);
  }
}

constexpr int CS_ROWS = 256;
// partial column sums over CS_ROWS rows: lane owns 8 columns (16-byte bf16 loads when VEC),
// the 4 waves of the block stride over the rows and are combined through LDS.
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void colsum_partial_kernel(int rows, int cols, const T* __restrict__ x,
                                                             int64_t ldx, float* __restrict__ ws) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(rows, r0 + CS_ROWS);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = r0 + wave; r < r1; r += 4) {
    const T* p = x + (int64_t)r * ldx + c0;
    if (VEC && c0 + 8 <= cols) {
      f32x4 a = Vec4<T>::ld(p), b = Vec4<T>::ld(p + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] += a[e];
        acc[4 + e] += b[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < cols) acc[e] += Elem<T>::ld(p + e);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[wave][lane * 8 + e] = acc[e];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.x * 512 + i;
    if (c < cols) ws[(int64_t)blockIdx.y * cols + c] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}
template <typename T>
__global__ __launch_bounds__(256) void act_kernel(int64_t n, int act, const T* __restrict__ x,
                                                  T* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    Elem<T>::st(y + i, act_fwd(act, Elem<T>::ld(x + i)));
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(int64_t n, const T* __restrict__ x,
                                                      T* __restrict__ y, Drop d) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    Elem<T>::st(y + i, Elem<T>::ld(x + i) * drop_mul(d, (uint64_t)i));
}

template <typename T>
__global__ __launch_bounds__(256) void act_bwd_kernel(int64_t n, int act, const T* __restrict__ z,
                                                      const T* __restrict__ dy, T* __restrict__ dz) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    Elem<T>::st(dz + i, Elem<T>::ld(dy + i) * act_bwd(act, Elem<T>::ld(z + i)));
}

constexpr int SQ_BLOCKS = 1024;
__global__ __launch_bounds__(256) void sumsq_partial_kernel(int64_t n, const float* __restrict__ x,
                                                            float* __restrict__ ws) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v = x[i];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ __launch_bounds__(256) void sumsq_final_kernel(int nb, const float* __restrict__ ws,
                                                          float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += ws[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void adamw_kernel(int64_t n, float* __restrict__ p,
                                                    const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const uint8_t* __restrict__ decay, float lr,
                                                    float b1, float b2, float eps, float wd,
                                                    float step_size, float max_norm,
                                                    const float* __restrict__ sumsq,
                                                    unsigned short* __restrict__ shadow) {
  float clip = 1.0f;
  if (max_norm > 0.f && sumsq) {
    float c = max_norm / (sqrtf(sumsq[0]) + 1e-6f);
    clip = c < 1.0f ? c : 1.0f;
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float gi = g[i] * clip;
    float mi = b1 * m[i] + (1.0f - b1) * gi;
    float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    float pi = p[i] - step_size * mi / (sqrtf(vi) + eps);
    if (wd > 0.f && (!decay || decay[i])) pi -= lr * wd * pi;
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

extern "C" mmseq_status mmseq_cast(int64_t n, const void* src, mmseq_dtype sd, void* dst,
                                   mmseq_dtype dd, mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && src && dst, "cast: bad args");
  if (n == 0) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(grid_for(n));
  if (sd == MMSEQ_F32 && dd == MMSEQ_BF16)
    hipLaunchKernelGGL((cast_kernel<float, unsigned short>), grid, dim3(256), 0, s, n,
                       (const float*)src, (unsigned short*)dst);
  else if (sd == MMSEQ_BF16 && dd == MMSEQ_F32)
    hipLaunchKernelGGL((cast_kernel<unsigned short, float>), grid, dim3(256), 0, s, n,
                       (const unsigned short*)src, (float*)dst);
  else if (sd == MMSEQ_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), grid, dim3(256), 0, s, n, (const float*)src,
                       (float*)dst);
  else
    hipLaunchKernelGGL((cast_kernel<unsigned short, unsigned short>), grid, dim3(256), 0, s, n,
                       (const unsigned short*)src, (unsigned short*)dst);
  return mmseq_check_launch("cast");
}

extern "C" mmseq_status mmseq_transpose_cast(int rows, int cols, const float* src, void* dst,
                                             mmseq_dtype dd, mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && cols >= 0 && src && dst, "transpose_cast: bad args");
  if (!rows || !cols) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  if (dd == MMSEQ_BF16)
    hipLaunchKernelGGL(transpose_kernel<unsigned short>, grid, dim3(256), 0, s, rows, cols, src,
                       (unsigned short*)dst);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, s, rows, cols, src,
                       (float*)dst);
  return mmseq_check_launch("transpose_cast");
}

extern "C" mmseq_status mmseq_transpose_cast_batch(int n, const int64_t* desc, int64_t tiles,
                                                   const float* src, void* dst, mmseq_dtype dd,
                                                   mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && tiles >= 0 && (n == 0 || (desc && src && dst)), "transpose_cast_batch: bad args");
  if (!n || !tiles) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dd == MMSEQ_BF16)
    hipLaunchKernelGGL(transpose_batch_kernel<unsigned short>, dim3((unsigned)tiles), dim3(256), 0, s, n,
                       desc, src, (unsigned short*)dst);
  else
    hipLaunchKernelGGL(transpose_batch_kernel<float>, dim3((unsigned)tiles), dim3(256), 0, s, n, desc,
                       src, (float*)dst);
  return mmseq_check_launch("transpose_cast_batch");
}

int64_t mmseq_reduce_extra(int nb, int W);
mmseq_status mmseq_reduce_partials(int nb, int W, int split, const float* ws, float* ws2,
                                   float* outA, float* outB, int accumulate, hipStream_t s);

extern "C" int64_t mmseq_colsum_workspace(int rows, int cols) {
  const int nb = (rows + CS_ROWS - 1) / CS_ROWS;
  return (int64_t)nb * cols + mmseq_reduce_extra(nb, cols);
}

extern "C" mmseq_status mmseq_colsum(int rows, int cols, const void* x, int64_t ldx, float* out,
                                     int accumulate, float* ws, mmseq_dtype dt,
                                     mmseq_stream stream) {
  MMSEQ_REQUIRE(rows >= 0 && cols > 0 && x && out && ws, "colsum: bad args");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = (rows + CS_ROWS - 1) / CS_ROWS;
  if (nb > 0) {
    dim3 grid((cols + 511) / 512, nb);
    const int esz = dt == MMSEQ_F32 ? 4 : 2;
    const bool vec = ((uintptr_t)x % 16) == 0 && ldx % 8 == 0 && (8 * esz) % 16 == 0;
    if (dt == MMSEQ_F32) {
      if (vec)
        hipLaunchKernelGGL((colsum_partial_kernel<float, true>), grid, dim3(256), 0, s, rows, cols,
                           (const float*)x, ldx, ws);
      else
        hipLaunchKernelGGL((colsum_partial_kernel<float, false>), grid, dim3(256), 0, s, rows,
                           cols, (const float*)x, ldx, ws);
    } else {
      if (vec)
        hipLaunchKernelGGL((colsum_partial_kernel<unsigned short, true>), grid, dim3(256), 0, s,
                           rows, cols, (const unsigned short*)x, ldx, ws);
      else
        hipLaunchKernelGGL((colsum_partial_kernel<unsigned short, false>), grid, dim3(256), 0, s,
                           rows, cols, (const unsigned short*)x, ldx, ws);
    }
  }
  mmseq_status st = mmseq_check_launch("colsum");
  if (st) return st;
  return mmseq_reduce_partials(nb, cols, cols, ws, ws + (int64_t)nb * cols, out, nullptr, accumulate,
                               s);
}

extern "C" mmseq_status mmseq_act_fwd(int64_t n, int act, const void* x, void* y, mmseq_dtype dt,
                                      mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && x && y, "act: bad args");
  if (!n) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dt == MMSEQ_F32)
    hipLaunchKernelGGL(act_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, n, act,
                       (const float*)x, (float*)y);
  else
    hipLaunchKernelGGL(act_kernel<unsigned short>, dim3(grid_for(n)), dim3(256), 0, s, n, act,
                       (const unsigned short*)x, (unsigned short*)y);
  return mmseq_check_launch("act_fwd");
}

extern "C" mmseq_status mmseq_dropout_apply(int64_t n, const void* x, void* y, mmseq_dtype dt,
                                            const mmseq_dropout* drop, mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && x && y, "dropout: bad args");
  if (!n) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const Drop d = make_drop(drop);
  if (dt == MMSEQ_F32)
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, n,
                       (const float*)x, (float*)y, d);
  else
    hipLaunchKernelGGL(dropout_kernel<unsigned short>, dim3(grid_for(n)), dim3(256), 0, s, n,
                       (const unsigned short*)x, (unsigned short*)y, d);
  return mmseq_check_launch("dropout_apply");
}

extern "C" mmseq_status mmseq_act_bwd(int64_t n, int act, const void* z, const void* dy, void* dz,
                                      mmseq_dtype dt, mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && z && dy && dz, "act_bwd: bad args");
  if (!n) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dt == MMSEQ_F32)
    hipLaunchKernelGGL(act_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, n, act,
                       (const float*)z, (const float*)dy, (float*)dz);
  else
    hipLaunchKernelGGL(act_bwd_kernel<unsigned short>, dim3(grid_for(n)), dim3(256), 0, s, n, act,
                       (const unsigned short*)z, (const unsigned short*)dy, (unsigned short*)dz);
  return mmseq_check_launch("act_bwd");
}

extern "C" int64_t mmseq_sumsq_workspace(int64_t n) { return SQ_BLOCKS; }

extern "C" mmseq_status mmseq_sumsq(int64_t n, const float* x, float* out, float* ws,
                                    mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && x && out && ws, "sumsq: bad args");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(SQ_BLOCKS), dim3(256), 0, s, n, x, ws);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, s, SQ_BLOCKS, ws, out);
  return mmseq_check_launch("sumsq");
}

extern "C" mmseq_status mmseq_adamw(int64_t n, float* p, const float* g, float* m, float* v,
                                    const uint8_t* decay_mask, float lr, float beta1, float beta2,
                                    float eps, float weight_decay, int step, float max_norm,
                                    const float* sumsq, void* shadow_bf16, mmseq_stream stream) {
  MMSEQ_REQUIRE(n >= 0 && p && g && m && v && step >= 1, "adamw: bad args");
  if (!n) return MMSEQ_OK;
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)(lr * sqrt(bc2) / bc1);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, s, n, p, g, m, v, decay_mask,
                     lr, beta1, beta2, eps, weight_decay, step_size, max_norm, sumsq,
                     (unsigned short*)shadow_bf16);
  return mmseq_check_launch("adamw");
}
