// Experiment: is the persistent 256x256 NT GEMM's epilogue bound per CU (store issue) or chip-wide
// (all CUs storing at once)? Times the path's shapes without / with the plain and residual
// epilogues (a) on every CU, (b) on half the CUs, (c) on every CU with the blocks that have one
// tile fewer starting late by a fraction of a tile (mmseq_gemm256_nt `delay`).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gemm_desync.hip -o tools/gemm_desync
#include "../multimodal_sequencing_amd/csrc/gemm256.hip"

#include <cstdio>
#include <vector>

__global__ void init_bf16(unsigned short* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9e3779b1u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    const float v = ((float)(x >> 8) * (1.0f / 8388608.0f) - 1.0f) * scale;
    p[i] = (unsigned short)(__float_as_uint(v) >> 16);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const int R = 164160;
  int dev_cus = 0;
  CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int shapes[4][2] = {{2304, 768}, {768, 768}, {3072, 768}, {768, 3072}};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    const int N = sh[0], K = sh[1];
    unsigned short *A, *B, *C, *Res;
    float* bias;
    CK(hipMalloc(&A, (size_t)R * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)R * N * 2));
    CK(hipMalloc(&Res, (size_t)R * N * 2));
    CK(hipMalloc(&bias, (size_t)N * 4));
    CK(hipMemset(bias, 0, (size_t)N * 4));
    hipLaunchKernelGGL(init_bf16, dim3(4096), dim3(256), 0, s, A, (int64_t)R * K, 1u, 1.0f);
    hipLaunchKernelGGL(init_bf16, dim3(4096), dim3(256), 0, s, B, (int64_t)N * K, 2u, 0.05f);
    hipLaunchKernelGGL(init_bf16, dim3(4096), dim3(256), 0, s, Res, (int64_t)R * N, 3u, 1.0f);
    CK(hipStreamSynchronize(s));
    const double fl = 2.0 * R * N * K;
    const int est_tile = 73 * K;  // shader cycles per 256x256 tile at ~1.1 PFLOP/s (estimate)
    struct Cfg { const char* name; int epi; int cus; float frac; };
    // epi: 0 none, 1 plain, 2 residual. (A probe of 8 rows x 128 B per store instruction instead
    // of 16 x 64 B measured equal to plain: profiles/r2s2_gemm_store_shape.json.)
    std::vector<Cfg> cfgs = {{"noepi", 0, dev_cus, 0.f},      {"plain", 1, dev_cus, 0.f},
                             {"resid", 2, dev_cus, 0.f},      {"noepi_halfcu", 0, dev_cus / 2, 0.f},
                             {"plain_halfcu", 1, dev_cus / 2, 0.f}, {"resid_halfcu", 2, dev_cus / 2, 0.f},
                             {"plain_d25", 1, dev_cus, .25f}, {"plain_d50", 1, dev_cus, .5f},
                             {"resid_d25", 2, dev_cus, .25f}, {"resid_d50", 2, dev_cus, .5f},
                             // grid a multiple of the column-tile count (252 = 28 x 9 = 84 x 3 =
                             // 21 x 12): every block keeps its B panel from round to round
                             {"noepi_g252", 0, 252, 0.f}, {"plain_g252", 1, 252, 0.f},
                             {"resid_g252", 2, 252, 0.f}};
    printf("{\"N\": %d, \"K\": %d, \"tiles\": %d", N, K, ((R + 255) / 256) * (N / 256));
    for (auto& c : cfgs) {
      mmseq_gemm_detail::GemmArgs a{};
      a.M = R; a.N = N; a.K = K;
      a.A = A; a.lda = K; a.B = B; a.ldb = K; a.C = C; a.ldc = N;
      a.alpha = c.epi == 0 ? -12345.0f : 1.0f;
      a.bias = c.epi == 0 ? nullptr : bias;
      a.resid = c.epi == 2 ? Res : nullptr;
      a.ldr = N;
      a.splitk = 1;
      const int delay = (int)(c.frac * est_tile);
      hipError_t err;
      for (int w = 0; w < 2; ++w) mmseq_gemm256_nt(a, true, c.cus, s, &err, 0, delay);
      CK(hipEventRecord(e0, s));
      const int iters = 10;
      for (int it = 0; it < iters; ++it)
        if (!mmseq_gemm256_nt(a, true, c.cus, s, &err, 0, delay)) { fprintf(stderr, "rejected\n"); return 1; }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(err);
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf(", \"%s\": %.1f", c.name, fl / (ms / iters * 1e-3) / 1e12);
      fflush(stdout);
    }
    printf("}\n");
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(Res)); CK(hipFree(bias));
  }
  return 0;
}
