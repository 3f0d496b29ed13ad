// Image preprocessing on device: the reference's per-image host transform
// (trainers/multimodal_utils.py:195-208 -> datasets/img_utils.py:27-56, 85-100, 135-144):
//   uint8 HWC (RGB) -> float [0,1] -> skimage.transform.resize to out_h x out_w (scikit-image
//   0.17.2, requirements.txt:256: anti-aliasing Gaussian with sigma = max(0, (in/out - 1) / 2)
//   per axis, scipy 'mirror' boundary, truncate 4, then bilinear sampling at pixel-centre aligned
//   coordinates in / out * (o + 0.5) - 0.5 with 'reflect' (= mirror) boundary) -> CHW
//   -> Normalize(mean, std).
// Both steps are linear and separable per axis, so each axis is one small weight vector per
// output coordinate (bilinear taps x Gaussian taps, mirrored indices): pass 1 filters rows into
// a [H][3][out_w] f32 workspace, pass 2 filters columns and normalises straight into the
// [n][3][out_h][out_w] model input. Byte / HBM-bound work: uint8 in once, f32 out once.
#include "common.h"

namespace {

constexpr int kMaxTaps = 4096;  // sanity bound on 2 bilinear x (2r + 1) Gaussian taps

__device__ __forceinline__ int mirror_index(int i, int n) {  // scipy 'mirror' / numpy 'reflect'
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  i %= period;
  if (i < 0) i += period;
  return i < n ? i : period - i;
}

// scale factor, sigma and radius in double as skimage / scipy compute them (the radius is an
// int() of a double, so a float sigma could land on the other side of a rounding boundary)
struct AxisPlan {
  double f;      // in / out
  float inv2s2;  // 1 / (2 sigma^2), 0 without filter
  int radius;    // int(4 sigma + 0.5)
  float inv_norm;
};

__device__ __forceinline__ AxisPlan axis_plan(int n_in, int n_out) {
  AxisPlan a;
  a.f = (double)n_in / (double)n_out;
  const double sigma = fmax(0.0, (a.f - 1.0) * 0.5);
  a.radius = sigma > 0.0 ? (int)(4.0 * sigma + 0.5) : 0;
  a.inv2s2 = sigma > 0.0 ? (float)(0.5 / (sigma * sigma)) : 0.f;
  float s = 0.f;
  for (int j = -a.radius; j <= a.radius; ++j) s += __expf(-(float)(j * j) * a.inv2s2);
  a.inv_norm = 1.f / s;
  return a;
}

// Accumulate sum_k w_k * src(k) over the composed taps of output coordinate o on one axis.
template <typename F>
__device__ __forceinline__ void axis_apply(const AxisPlan& a, int o, int n_in, F&& take) {
  const double p = a.f * ((double)o + 0.5) - 0.5;
  const double fl = floor(p);
  const float t = (float)(p - fl);
  const int i0 = (int)fl;
  const float inv2s2 = a.inv2s2;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float wb = e ? t : 1.f - t;
    if (wb == 0.f) continue;
    const int k = mirror_index(i0 + e, n_in);  // the warp samples the filtered image (reflect)
    for (int j = -a.radius; j <= a.radius; ++j) {
      const float wg = __expf(-(float)(j * j) * inv2s2) * a.inv_norm;
      take(mirror_index(k + j, n_in), wb * wg);
    }
  }
}

// pass 1: rows. table[i] = (pixel offset, H, W, workspace offset)
__global__ void __launch_bounds__(256) resize_rows_kernel(const uint8_t* __restrict__ pixels,
                                                          const int64_t* __restrict__ table,
                                                          int out_w, float* __restrict__ ws) {
  const int img = blockIdx.y, y = blockIdx.x;
  const int64_t poff = table[4 * img], woff = table[4 * img + 3];
  const int H = (int)table[4 * img + 1], W = (int)table[4 * img + 2];
  if (y >= H) return;
  const AxisPlan a = axis_plan(W, out_w);
  const uint8_t* row = pixels + poff + (int64_t)y * W * 3;
  for (int x = threadIdx.x; x < out_w; x += blockDim.x) {
    float r = 0.f, g = 0.f, b = 0.f;
    axis_apply(a, x, W, [&](int xs, float w) {
      const uint8_t* px = row + 3 * xs;
      r += w * (float)px[0];
      g += w * (float)px[1];
      b += w * (float)px[2];
    });
    float* o = ws + woff + (int64_t)y * 3 * out_w + x;
    o[0] = r;
    o[out_w] = g;
    o[2 * out_w] = b;
  }
}

struct Norm {
  float scale[3], shift[3];  // v / 255 -> (v / 255 - mean) / std = v * scale + shift
};

// pass 2: columns + normalise into out[img][c][y][x]
__global__ void __launch_bounds__(256) resize_cols_kernel(const int64_t* __restrict__ table,
                                                          int out_h, int out_w,
                                                          const float* __restrict__ ws, Norm nm,
                                                          float* __restrict__ out) {
  const int img = blockIdx.y, y = blockIdx.x;
  const int64_t woff = table[4 * img + 3];
  const int H = (int)table[4 * img + 1];
  const AxisPlan a = axis_plan(H, out_h);
  const float* src = ws + woff;
  for (int q = threadIdx.x; q < 3 * out_w; q += blockDim.x) {
    const int c = q / out_w, x = q - c * out_w;
    float acc = 0.f;
    axis_apply(a, y, H, [&](int ys, float w) { acc += w * src[((int64_t)ys * 3 + c) * out_w + x]; });
    out[(((int64_t)img * 3 + c) * out_h + y) * out_w + x] = acc * nm.scale[c] + nm.shift[c];
  }
}

}  // namespace

extern "C" int64_t mmseq_image_resize_workspace(int n_images, const int32_t* heights, int out_w) {
  int64_t total = 0;
  for (int i = 0; i < n_images; ++i) total += (int64_t)heights[i] * 3 * out_w;
  return total * (int64_t)sizeof(float);
}

extern "C" mmseq_status mmseq_image_resize_normalize(
    int n_images, const uint8_t* pixels, const int64_t* table, int max_h, int max_w, int out_h,
    int out_w, const float* mean, const float* stdev, float* workspace, int64_t workspace_bytes,
    float* out, mmseq_stream stream) {
  // workspace_bytes: >= mmseq_image_resize_workspace(heights); the table lives on the device,
  // so the caller (which built it) is the one that can check it
  MMSEQ_REQUIRE(workspace_bytes >= (int64_t)3 * out_w * (int64_t)sizeof(float),
                "image_resize: workspace too small");
  MMSEQ_REQUIRE(n_images >= 0 && out_h > 0 && out_w > 0 && max_h > 0 && max_w > 0,
                "image_resize: bad sizes");
  MMSEQ_REQUIRE(pixels && table && mean && stdev && workspace && out, "image_resize: null buffer");
  MMSEQ_REQUIRE(max_h < 65536 && max_w < (1 << 20) && out_h < 65536, "image_resize: too large");
  // widest composed footprint: 2 bilinear taps x (2 r + 1), r = int(4 sigma + 0.5)
  const double sig = fmax(0.0, ((double)max_w / out_w - 1.0) * 0.5);
  const double sig_h = fmax(0.0, ((double)max_h / out_h - 1.0) * 0.5);
  MMSEQ_REQUIRE(2 * (2 * (int)(4.0 * fmax(sig, sig_h) + 0.5) + 1) <= kMaxTaps,
                "image_resize: downscale factor too large");
  if (n_images == 0) return MMSEQ_OK;
  Norm nm;
  for (int c = 0; c < 3; ++c) {
    MMSEQ_REQUIRE(stdev[c] != 0.f, "image_resize: zero std");
    nm.scale[c] = 1.f / (255.f * stdev[c]);
    nm.shift[c] = -mean[c] / stdev[c];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(resize_rows_kernel, dim3(max_h, n_images), dim3(256), 0, s, pixels, table,
                     out_w, workspace);
  hipLaunchKernelGGL(resize_cols_kernel, dim3(out_h, n_images), dim3(256), 0, s, table, out_h,
                     out_w, workspace, nm, out);
  return mmseq_check_launch("image_resize_normalize");
}
