// Deterministic column reductions of per-workgroup partial rows (bias / LayerNorm-affine
// gradients): out[w] (+)= sum_b ws[b][w] for w < W, in a fixed order. Two levels so that the
// first level has ~(W/64) x (nb/64) workgroups in flight instead of W/64 serial loops.
#include "common.h"

namespace {

constexpr int RCH = 64;  // partial rows per level-1 workgroup

__global__ __launch_bounds__(256) void reduce_l1_kernel(int nb, int W, const float* __restrict__ ws,
                                                        float* __restrict__ ws2) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = blockIdx.x * 64 + lane;
  const int b0 = blockIdx.y * RCH;
  float s = 0.f;
  if (w < W)
    for (int b = b0 + wave; b < min(nb, b0 + RCH); b += 4) s += ws[(int64_t)b * W + w];
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && w < W)
    ws2[(int64_t)blockIdx.y * W + w] = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
}

__global__ __launch_bounds__(256) void reduce_l2_kernel(int nb2, int W, int split, int split2,
                                                        const float* __restrict__ ws2,
                                                        float* __restrict__ outA,
                                                        float* __restrict__ outB,
                                                        float* __restrict__ outC, int accumulate) {
  const int w = blockIdx.x * 256 + threadIdx.x;
  if (w >= W) return;
  float* dst = w < split ? (outA ? outA + w : nullptr)
                         : w < split2 ? (outB ? outB + (w - split) : nullptr)
                                      : (outC ? outC + (w - split2) : nullptr);
  if (!dst) return;
  float s = 0.f;
  for (int b = 0; b < nb2; ++b) s += ws2[(int64_t)b * W + w];
  *dst = accumulate ? *dst + s : s;
}

}  // namespace

int64_t mmseq_reduce_extra(int nb, int W) { return (int64_t)((nb + RCH - 1) / RCH) * W; }

// ws: [nb][W] partials; ws2: scratch of mmseq_reduce_extra(nb, W) floats.
// columns [0, split) go to outA, [split, W) to outB (either may be NULL).
mmseq_status mmseq_reduce_partials(int nb, int W, int split, const float* ws, float* ws2,
                                   float* outA, float* outB, int accumulate, hipStream_t s) {
  if (W <= 0) return MMSEQ_OK;
  const int nb2 = (nb + RCH - 1) / RCH;
  if (nb > 0)
    hipLaunchKernelGGL(reduce_l1_kernel, dim3((W + 63) / 64, nb2), dim3(256), 0, s, nb, W, ws, ws2);
  hipLaunchKernelGGL(reduce_l2_kernel, dim3((W + 255) / 256), dim3(256), 0, s, nb > 0 ? nb2 : 0, W,
                     split, W, ws2, outA, outB, nullptr, accumulate);
  return mmseq_check_launch("reduce_partials");
}

// three outputs: columns [0, split) to outA, [split, split2) to outB, [split2, W) to outC
mmseq_status mmseq_reduce_partials3(int nb, int W, int split, int split2, const float* ws, float* ws2,
                                    float* outA, float* outB, float* outC, int accumulate,
                                    hipStream_t s) {
  if (W <= 0) return MMSEQ_OK;
  const int nb2 = (nb + RCH - 1) / RCH;
  if (nb > 0)
    hipLaunchKernelGGL(reduce_l1_kernel, dim3((W + 63) / 64, nb2), dim3(256), 0, s, nb, W, ws, ws2);
  hipLaunchKernelGGL(reduce_l2_kernel, dim3((W + 255) / 256), dim3(256), 0, s, nb > 0 ? nb2 : 0, W,
                     split, split2, ws2, outA, outB, outC, accumulate);
  return mmseq_check_launch("reduce_partials");
}
