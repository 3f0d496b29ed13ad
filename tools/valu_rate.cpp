// VALU issue-cost microbenchmark: cycles per wave-instruction for v_mul_lo_u32, v_mul_u32_u24,
// v_mul_hi_u32_u24, v_xor_b32, v_lshl_add_u32, v_exp_f32 (8 independent chains, one wave per
// SIMD so nothing hides the issue cost). Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.cpp
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
#define ITERS 4096

#define KERNEL(NAME, ASM)                                                                      \
  __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed, long long* cyc) {  \
    unsigned v[CHAINS];                                                                        \
    for (int c = 0; c < CHAINS; ++c) v[c] = seed + threadIdx.x * 7 + c;                        \
    const unsigned k = seed | 1u;                                                              \
    long long t0 = clock64();                                                                  \
    for (int i = 0; i < ITERS; ++i) {                                                          \
      _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) asm volatile(ASM : "+v"(v[c]) : "v"(k)); \
    }                                                                                          \
    long long t1 = clock64();                                                                  \
    unsigned s = 0;                                                                            \
    for (int c = 0; c < CHAINS; ++c) s ^= v[c];                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                            \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                           \
  }

KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mul24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_mulhi24, "v_mul_hi_u32_u24 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
KERNEL(k_exp, "v_exp_f32 %0, %0")
KERNEL(k_pk_sub_u16, "v_pk_sub_u16 %0, %0, %1 clamp")

template <typename F>
double run(F f, const char* name) {
  unsigned* out;
  long long* cyc;
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&cyc, 256 * 8);
  // 256 blocks x 4 waves: one wave per SIMD on every CU
  hipLaunchKernelGGL(f, dim3(256), dim3(256), 0, 0, out, 12345u, cyc);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(f, dim3(256), dim3(256), 0, 0, out, 12345u, cyc);
  long long h[256];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 256; ++i) s += (double)h[i];
  s /= 256;
  const double per = s / ((double)ITERS * CHAINS);
  printf("\"%s\": %.2f, ", name, per);
  (void)hipFree(out);
  (void)hipFree(cyc);
  return per;
}

int main() {
  printf("{\"clock64 cycles per wave instruction (one wave per SIMD, 8 chains)\": {");
  run(k_xor, "v_xor_b32");
  run(k_lshl_add, "v_lshl_add_u32");
  run(k_mul24, "v_mul_u32_u24");
  run(k_mulhi24, "v_mul_hi_u32_u24");
  run(k_mul_lo, "v_mul_lo_u32");
  run(k_pk_sub_u16, "v_pk_sub_u16_clamp");
  run(k_exp, "v_exp_f32");
  printf("\"_\": 0}}\n");
  return 0;
}
