// Measured dense bf16 MFMA peak on this MI355X (SURVEY §8(d) "measured GEMM peak"): every CU
// runs 4 waves (one per SIMD) of back-to-back v_mfma_f32_16x16x32_bf16 on random register
// operands, 8 independent accumulators per wave; FLOP/s from hipEvent time over 5 launches
// after 3 warm-up launches. Also the 32x32x16 form. Prints one JSON line.
//   build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form tools/mfma_peak.cpp -o tools/mfma_peak
//   (VGPR-form accumulators: in AGPR form hipcc shuffles the 8 accumulators through v_accvgpr
//   moves inside the loop and chains them, halving the measured 16x16x32 rate)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) int i32x8;

template <int SHAPE>
__global__ void __launch_bounds__(256) mfma_loop(const unsigned short* __restrict__ seed, int iters,
                                                 float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    unsigned short u = seed[(blockIdx.x * 256 + threadIdx.x) * 16 + j];
    unsigned short v = seed[(blockIdx.x * 256 + threadIdx.x) * 16 + 8 + j];
    a[j] = __builtin_bit_cast(__bf16, u);
    b[j] = __builtin_bit_cast(__bf16, v);
  }
  float out = 0.f;
  if constexpr (SHAPE == 8) {
    i32x8 fa, fb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // e4m3 bytes with the exponent's top bit clear: finite, no NaN
      fa[j] = (int)((((uint32_t)a[j % 8] << 16) | (uint32_t)b[j % 8]) & 0x37373737u);
      fb[j] = (int)((((uint32_t)b[j % 8] << 16) | (uint32_t)a[(j + 3) % 8]) & 0x37373737u);
    }
    f32x4 acc[8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        acc[k] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa, fb, acc[k], 0, 0, 0, 127, 0, 127);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  } else if constexpr (SHAPE == 16) {
    f32x4 acc[8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  } else {
    f32x16 acc[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[k], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      for (int r = 0; r < 16; ++r) out += acc[k][r];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = out;  // vector store, keeps the loop alive
  (void)lane;
}

template <int SHAPE>
static double run(int cus, int iters) {
  const int blocks = cus;  // 256 threads = 4 waves = one per SIMD
  const size_t n = (size_t)blocks * 256 * 16;
  unsigned short* h = (unsigned short*)malloc(n * 2);
  unsigned s = 12345u;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    float f = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;  // random in [-0.5, 0.5)
    unsigned bits;
    memcpy(&bits, &f, 4);
    h[i] = (unsigned short)(bits >> 16);
  }
  unsigned short* d;
  float* sink;
  hipMalloc(&d, n * 2);
  hipMalloc(&sink, (size_t)blocks * 256 * 4);
  hipMemcpy(d, h, n * 2, hipMemcpyHostToDevice);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(mfma_loop<SHAPE>, dim3(blocks), dim3(256), 0, 0, d, iters, sink);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mfma_loop<SHAPE>, dim3(blocks), dim3(256), 0, 0, d, iters, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double per_mfma = SHAPE == 8 ? 2.0 * 16 * 16 * 128 : SHAPE == 16 ? 2.0 * 16 * 16 * 32 : 2.0 * 32 * 32 * 16;
  const double per_wave_iter = SHAPE == 32 ? 4 : 8;
  const double flops = (double)reps * blocks * 4 * iters * per_wave_iter * per_mfma;
  hipFree(d);
  hipFree(sink);
  free(h);
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int iters = 40000;
  double t16 = run<16>(cus, iters);
  double t32 = run<32>(cus, iters);
  double t8 = run<8>(cus, iters / 2);
  printf("{\"device\": \"%s\", \"cus\": %d, \"iters_per_wave\": %d, \"bf16_16x16x32_tflops\": %.1f, "
         "\"bf16_32x32x16_tflops\": %.1f, \"mxfp8_16x16x128_tflops\": %.1f, \"spec_dense_bf16_tflops\": 2500.0, "
         "\"spec_dense_fp8_tflops\": 5000.0, \"operands\": \"random bf16 / e4m3 in registers\"}\n",
         p.gcnArchName, cus, iters, t16, t32, t8);
  return 0;
}
