// Store-shape microbenchmark: write a [M][N] bf16 matrix with 16-byte lane stores whose wave
// instruction covers R rows x (1024 / R) bytes (R = 16: the NT GEMM epilogue's 16 rows x 64 B;
// 8, 4, 1), optionally reading a residual of the same shape first. Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_shape tools/store_shape.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <int R, bool READ>
__global__ __launch_bounds__(256) void store_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                    int M, int N) {
  // a wave owns 64 rows x all N columns; a lane writes 8 bf16 (16 B)
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int r_base = wave * 64;
  if (r_base >= M) return;
  constexpr int LPR = 64 / R;           // lanes per row
  const int lr = lane / LPR, lc = lane % LPR;
  const int nv = N / 8;                 // 16-B vectors per row
  for (int r0 = 0; r0 < 64; r0 += R) {
    const int row = r_base + r0 + lr;
    if (row >= M) break;
    for (int c0 = 0; c0 < nv; c0 += LPR) {
      const int64_t o = (int64_t)row * nv + c0 + lc;
      u32x4 v = {(unsigned)row, (unsigned)c0, 7u, 9u};
      if (READ) v += in[o];
      out[o] = v;
    }
  }
}

template <int R, bool READ>
float run(const u32x4* in, u32x4* out, int M, int N) {
  const int waves = (M + 63) / 64;
  dim3 grid((waves + 3) / 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  store_kernel<R, READ><<<grid, 256>>>(in, out, M, N);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) store_kernel<R, READ><<<grid, 256>>>(in, out, M, N);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const int M = 164160;
  for (int N : {768, 3072}) {
    const size_t bytes = (size_t)M * N * 2;
    u32x4 *in, *out;
    hipMalloc(&in, bytes);
    hipMalloc(&out, bytes);
    hipMemset(in, 0, bytes);
    float t16 = run<16, false>(in, out, M, N), t8 = run<8, false>(in, out, M, N);
    float t4 = run<4, false>(in, out, M, N), t1 = run<1, false>(in, out, M, N);
    float r16 = run<16, true>(in, out, M, N), r8 = run<8, true>(in, out, M, N);
    float r4 = run<4, true>(in, out, M, N), r1 = run<1, true>(in, out, M, N);
    printf("{\"N\": %d, \"MB\": %.1f, \"store_TBps\": {\"16x64B\": %.2f, \"8x128B\": %.2f, \"4x256B\": %.2f, "
           "\"1x1KB\": %.2f}, \"load+store_TBps\": {\"16x64B\": %.2f, \"8x128B\": %.2f, \"4x256B\": %.2f, "
           "\"1x1KB\": %.2f}}\n",
           N, bytes / 1e6, bytes / t16 / 1e9, bytes / t8 / 1e9, bytes / t4 / 1e9, bytes / t1 / 1e9,
           2 * bytes / r16 / 1e9, 2 * bytes / r8 / 1e9, 2 * bytes / r4 / 1e9, 2 * bytes / r1 / 1e9);
    hipFree(in);
    hipFree(out);
  }
  return 0;
}
