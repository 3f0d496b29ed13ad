// MX-fp8 (OCP e4m3 elements, E8M0 scale per 32 K-elements) NT GEMM and the bf16 -> MX-fp8
// quantiser, for the config-5 forward GEMMs (BASELINE config 5: ViT-L/14 + RoBERTa-large, fp8
// MFMA). The block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 runs twice the bf16 rate per clock
// (MI355X_MICROARCH.md, matrix-core table), and fp8 operands halve the staged bytes.
//
// Scale layout ("packed", chosen so one dword per lane per K-step carries the scales of the four
// 16-row blocks that lane multiplies, one byte each):
//   scale(m, kb) at byte ((m / 64) * (K / 32) + kb) * 64 + (m % 16) * 4 + (m % 64) / 16
// rows up to the next multiple of 64 exist (scale 0).
//
// GEMM: C[m][n] = act(alpha * sum_k A[m][k] B[n][k] + bias[n]) (+ resid[m][n]), bf16 out.
// 128 x 128 tiles, 4 waves (2 x 2, 64 x 64 each = 4 x 4 MFMA blocks), BK = 128 (one MFMA K),
// LDS ring of NSLOT slots filled by LDS-DMA (16-byte chunks XOR-swizzled by row), counted vmcnt
// + raw s_barrier as the bf16 ring kernel (gemm.hip).
#include "gemm_common.h"

using namespace mmseq_gemm_detail;

namespace {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

constexpr int kSlotBytes = 2 * 128 * 128 + 1024;  // A + B tiles + their scales
constexpr int kSlots = 2;

__device__ __forceinline__ void dma_chunk(rsrc_t r, uint8_t* lds, uint32_t voff) {
  dma16(r, reinterpret_cast<unsigned short*>(lds), voff);
}

// one operand tile [128 rows][128 B] of K-step kt: 16 DMA instructions, 4 per wave
__device__ __forceinline__ void stage_tile(rsrc_t r, int64_t ld, int k0, uint8_t* s, int wave,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int inst = wave * 4 + i;
    const int row = inst * 8 + (lane >> 3), cp = lane & 7;
    const int c = cp ^ (row & 7);
    dma_chunk(r, s + inst * 1024, (uint32_t)((int64_t)row * ld + k0 + c * 16));
  }
}

// Operand fragment of the 16x16x128 f8 MFMA: lane l holds row l & 15 and the K positions
// 16 g .. 16 g + 15 (registers 0-3) and 64 + 16 g .. 64 + 16 g + 15 (registers 4-7), g = l >> 4;
// the scale of K-block b (32 positions) is taken from lane group b (probed with
// tools/fp8_probe.py: with 32 contiguous positions per lane the blocks are mis-paired).
__device__ __forceinline__ i32x8 frag(const uint8_t* s, int rb, int lane) {
  const int rr = rb + (lane & 15), g = lane >> 4;
  const uint8_t* row = s + rr * 128;
  const i32x4 lo = *reinterpret_cast<const i32x4*>(row + ((g ^ (rr & 7)) << 4));
  const i32x4 hi = *reinterpret_cast<const i32x4*>(row + (((4 + g) ^ (rr & 7)) << 4));
  return (i32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ __launch_bounds__(256, 2) void gemm_mxfp8_nt_kernel(GemmArgs a, const uint8_t* sa,
                                                              const uint8_t* sb, int64_t sa_bytes,
                                                              int64_t sb_bytes, int tiles_n) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kSlots * kSlotBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int Lr = xcd_item(blockIdx.x, gridDim.x);
  const int tm = Lr / tiles_n, tn = Lr % tiles_n;
  const int m0 = tm * 128, n0 = tn * 128;
  const uint8_t* A = reinterpret_cast<const uint8_t*>(a.A);
  const uint8_t* B = reinterpret_cast<const uint8_t*>(a.B);
  const int KB = a.K / 32, nk = a.K / 128;
  const rsrc_t ra = make_rsrc(A + (int64_t)m0 * a.lda, (int64_t)(a.M - m0 - 1) * a.lda + a.K);
  const rsrc_t rb = make_rsrc(B + (int64_t)n0 * a.ldb, (int64_t)(a.N - n0 - 1) * a.ldb + a.K);
  const rsrc_t rsa = make_rsrc(sa, sa_bytes), rsb = make_rsrc(sb, sb_bytes);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // scale DMA: wave 0 lanes 0-31 the A scales (2 x 256 B), wave 1 lanes 0-31 the B scales
  auto issue = [&](int kt) {
    uint8_t* s = smem + (kt % kSlots) * kSlotBytes;
    stage_tile(ra, a.lda, kt * 128, s, wave, lane);
    stage_tile(rb, a.ldb, kt * 128, s + 16384, wave, lane);
    if (wave < 2 && lane < 32) {
      const int grp = ((wave == 0 ? m0 : n0) >> 6) + (lane >> 4);
      dma_chunk(wave == 0 ? rsa : rsb, s + 32768 + wave * 512,
                (uint32_t)(((int64_t)grp * KB + 4 * kt) * 64 + (lane & 15) * 16));
    }
  };

  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    // this wave's DMA for kt retired; the next step's (8 or 9 instructions) may stay in flight
    if (more) {
      issue(kt + 1);
      if (wave < 2) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* s = smem + (kt % kSlots) * kSlotBytes;
    i32x8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i] = frag(s, wr * 64 + i * 16, lane);
      fb[i] = frag(s + 16384, wc * 64 + i * 16, lane);
    }
    const int so = (lane >> 4) * 64 + (lane & 15) * 4;
    const int scA = *reinterpret_cast<const int*>(s + 32768 + wr * 256 + so);        // rows m
    const int scB = *reinterpret_cast<const int*>(s + 32768 + 512 + wc * 256 + so);  // rows n
    // the instruction reads the scale from byte 0 of its scale operand whatever OPSEL says
    // (noted in CK's amd_xdlops.hpp), so block i's byte is shifted down instead of selected
    int sA[4], sB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sA[i] = (int)((uint32_t)scA >> (8 * i));
      sB[i] = (int)((uint32_t)scB >> (8 * i));
    }
#define MX_MFMA(I, J)                                                                        \
  acc[I][J] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[J], fa[I], acc[I][J], 0, 0, \
                                                               0, sB[J], 0, sA[I])
    MX_MFMA(0, 0); MX_MFMA(0, 1); MX_MFMA(0, 2); MX_MFMA(0, 3);
    MX_MFMA(1, 0); MX_MFMA(1, 1); MX_MFMA(1, 2); MX_MFMA(1, 3);
    MX_MFMA(2, 0); MX_MFMA(2, 1); MX_MFMA(2, 2); MX_MFMA(2, 3);
    MX_MFMA(3, 0); MX_MFMA(3, 1); MX_MFMA(3, 2); MX_MFMA(3, 3);
#undef MX_MFMA
    // every wave done reading slot kt before the DMA of step kt + 2 (issued next iteration)
    // overwrites it: this wave's LDS reads retired, then the barrier (the compiler would
    // otherwise leave fragment reads in flight across it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  const int g = lane >> 4, ii = lane & 15;
  unsigned short* C = reinterpret_cast<unsigned short*>(a.C);
  const unsigned short* resid = reinterpret_cast<const unsigned short*>(a.resid);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wr * 64 + i * 16 + ii;
      const int n = n0 + wc * 64 + j * 16 + 4 * g;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epilogue4<unsigned short>(a, C, resid, nullptr, nullptr, m, n, v);
    }
}

template <int ROWS_PER_WAVE>  // rows of 128 B one wave stages: 8 per DMA instruction
__device__ __forceinline__ void stage_rows(rsrc_t r, int64_t ld, int k0, uint8_t* s, int wave,
                                           int lane) {
  constexpr int NI = ROWS_PER_WAVE / 8;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int inst = wave * NI + i;
    const int row = inst * 8 + (lane >> 3), cp = lane & 7;
    dma_chunk(r, s + inst * 1024, (uint32_t)((int64_t)row * ld + k0 + ((cp ^ (row & 7)) << 4)));
  }
}

// 256 x 256 tiles, 8 waves (4 x 2, 64 x 128 each), BK = 128, 2-slot LDS-DMA ring (2 x 66 KB).
// The main loop is bound by the latency of the operand DMA (PMC at the config-5 FC2 shape: MFMA
// busy 0.39, 43 % of wave time in memory waits, L2 hit 79 %): the bytes a CU can keep in flight
// are what LDS leaves beside the slot being computed, so the rate per CU goes with MFLOP per
// staged byte. 256 x 256 stages half the bytes per MFLOP of 128 x 128 (1.13x at FC2, 1.08x at
// QKV); a 256 x 128 tile with a 3-slot ring and register-double-buffered fragments measured no
// better than 128 x 128 (same bytes in flight per MFLOP). The B fragments of a step are read in
// two halves of four 16-column blocks to stay inside the register file (128 accumulators).
constexpr int kQ_A = 256 * 128, kQ_B = 256 * 128;
constexpr int kQSlot = kQ_A + kQ_B + 1024 + 1024;

__global__ __launch_bounds__(512, 1) void gemm_mxfp8_nt256x256_kernel(GemmArgs a, const uint8_t* sa,
                                                                     const uint8_t* sb,
                                                                     int64_t sa_bytes,
                                                                     int64_t sb_bytes, int tiles_n) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kQSlot];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int Lr = xcd_item(blockIdx.x, gridDim.x);
  const int tm = Lr / tiles_n, tn = Lr % tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const uint8_t* A = reinterpret_cast<const uint8_t*>(a.A);
  const uint8_t* B = reinterpret_cast<const uint8_t*>(a.B);
  const int KB = a.K / 32, nk = a.K / 128;
  const rsrc_t ra = make_rsrc(A + (int64_t)m0 * a.lda, (int64_t)(a.M - m0 - 1) * a.lda + a.K);
  const rsrc_t rb = make_rsrc(B + (int64_t)n0 * a.ldb, (int64_t)(a.N - n0 - 1) * a.ldb + a.K);
  const rsrc_t rsa = make_rsrc(sa, sa_bytes), rsb = make_rsrc(sb, sb_bytes);

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // per wave and step: 4 A + 4 B DMA instructions and one for the scales (waves 0-3 one A row
  // group of 64 rows each, waves 4-7 one B row group each; 16 lanes x 16 B)
  auto issue = [&](int kt) {
    uint8_t* s = smem + (kt & 1) * kQSlot;
    stage_rows<32>(ra, a.lda, kt * 128, s, wave, lane);
    stage_rows<32>(rb, a.ldb, kt * 128, s + kQ_A, wave, lane);
    if (lane < 16) {
      const bool isa = wave < 4;  // wave-uniform
      const int grp = ((isa ? m0 : n0) >> 6) + (wave & 3);
      dma_chunk(isa ? rsa : rsb, s + kQ_A + kQ_B + wave * 256,
                (uint32_t)(((int64_t)grp * KB + 4 * kt) * 64 + lane * 16));
    }
  };

  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's DMA of step kt retired and its reads of the other slot (step kt - 1) too; after
    // the barrier that slot takes the DMA of step kt + 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) issue(kt + 1);
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* s = smem + (kt & 1) * kQSlot;
    const int so = (lane >> 4) * 64 + (lane & 15) * 4;
    const int scA = *reinterpret_cast<const int*>(s + kQ_A + kQ_B + wr * 256 + so);
    i32x8 fa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(s, wr * 64 + i * 16, lane);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int scB = *reinterpret_cast<const int*>(s + kQ_A + kQ_B + 1024 + (wc * 2 + h) * 256 + so);
      i32x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag(s + kQ_A, wc * 128 + h * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][h * 4 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              fb[j], fa[i], acc[i][h * 4 + j], 0, 0, 0, (int)((uint32_t)scB >> (8 * j)), 0,
              (int)((uint32_t)scA >> (8 * i)));
    }
  }

  const int g = lane >> 4, ii = lane & 15;
  unsigned short* C = reinterpret_cast<unsigned short*>(a.C);
  const unsigned short* resid = reinterpret_cast<const unsigned short*>(a.resid);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + wr * 64 + i * 16 + ii;
      const int n = n0 + wc * 128 + j * 16 + 4 * g;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epilogue4<unsigned short>(a, C, resid, nullptr, nullptr, m, n, v);
    }
}

// bf16 / f32 [M][K] -> e4m3 [M][K] (row stride ldq) + packed E8M0 scales; one thread per
// (row, 32-element block), rows up to the next multiple of 64 get scale 0
template <typename TI>
__global__ __launch_bounds__(256) void quant_mxfp8_kernel(int M, int K, const TI* __restrict__ x,
                                                          int64_t ldx, uint8_t* __restrict__ q,
                                                          int64_t ldq,
                                                          uint8_t* __restrict__ scales) {
  const int KB = K / 32;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int Mp = (M + 63) & ~63;
  if (idx >= (int64_t)Mp * KB) return;
  const int m = (int)(idx / KB), kb = (int)(idx - (int64_t)m * KB);
  uint8_t* sp = scales + ((int64_t)(m >> 6) * KB + kb) * 64 + (m & 15) * 4 + ((m >> 4) & 3);
  if (m >= M) {
    *sp = 0;
    return;
  }
  const TI* xp = x + (int64_t)m * ldx + kb * 32;
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 32; j += 4) {
    const f32x4 t = Vec4<TI>::ld(xp + j);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[j + r] = t[r];
      amax = fmaxf(amax, fabsf(t[r]));
    }
  }
  // OCP MX: shared exponent floor(log2 amax) - emax(e4m3) = 8, as an E8M0 byte (bias 127)
  int e = amax > 0.f ? (int)((__float_as_uint(amax) >> 23) & 0xff) - 127 : -127;
  e = max(-127, min(127, e - 8));
  *sp = (uint8_t)(e + 127);
  const float inv = ldexpf(1.f, -e);
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s0 = fminf(448.f, fmaxf(-448.f, v[4 * j] * inv));
    float s1 = fminf(448.f, fmaxf(-448.f, v[4 * j + 1] * inv));
    float s2 = fminf(448.f, fmaxf(-448.f, v[4 * j + 2] * inv));
    float s3 = fminf(448.f, fmaxf(-448.f, v[4 * j + 3] * inv));
    int p = __builtin_amdgcn_cvt_pk_fp8_f32(s0, s1, 0, false);
    p = __builtin_amdgcn_cvt_pk_fp8_f32(s2, s3, p, true);
    w[j] = (uint32_t)p;
  }
  uint8_t* qp = q + (int64_t)m * ldq + kb * 32;
  *reinterpret_cast<i32x4*>(qp) = (i32x4){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
  *reinterpret_cast<i32x4*>(qp + 16) = (i32x4){(int)w[4], (int)w[5], (int)w[6], (int)w[7]};
}

}  // namespace

extern "C" int64_t mmseq_mxfp8_scale_bytes(int M, int K) {
  return (int64_t)((M + 63) / 64) * (K / 32) * 64;
}

extern "C" mmseq_status mmseq_quant_mxfp8(int M, int K, const void* x, int64_t ldx,
                                          mmseq_dtype dtype, void* q, int64_t ldq, void* scales,
                                          mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && K > 0 && K % 32 == 0 && ldx >= K && ldq >= K && ldq % 16 == 0,
                "quant_mxfp8: bad sizes (K % 32, ldq % 16)");
  MMSEQ_REQUIRE(x && q && scales, "quant_mxfp8: null buffer");
  MMSEQ_REQUIRE(((uintptr_t)q & 15) == 0 && (ldx * (dtype == MMSEQ_BF16 ? 2 : 4)) % 16 == 0 &&
                    ((uintptr_t)x & 15) == 0,
                "quant_mxfp8: 16-byte alignment");
  if (M == 0) return MMSEQ_OK;
  const int64_t n = (int64_t)((M + 63) & ~63) * (K / 32);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == MMSEQ_BF16)
    hipLaunchKernelGGL(quant_mxfp8_kernel<unsigned short>, grid, dim3(256), 0, s, M, K,
                       (const unsigned short*)x, ldx, (uint8_t*)q, ldq, (uint8_t*)scales);
  else
    hipLaunchKernelGGL(quant_mxfp8_kernel<float>, grid, dim3(256), 0, s, M, K, (const float*)x,
                       ldx, (uint8_t*)q, ldq, (uint8_t*)scales);
  return mmseq_check_launch("quant_mxfp8");
}

extern "C" mmseq_status mmseq_gemm_mxfp8(int M, int N, int K, const void* A, int64_t lda,
                                         const void* a_scales, const void* B, int64_t ldb,
                                         const void* b_scales, void* C, int64_t ldc,
                                         const float* bias, int act, const void* resid,
                                         int64_t ldr, float alpha, mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 128 == 0, "gemm_mxfp8: K must be a multiple of 128");
  MMSEQ_REQUIRE(lda >= K && ldb >= K && lda % 16 == 0 && ldb % 16 == 0 && ldc >= N && ldc % 4 == 0,
                "gemm_mxfp8: leading dimensions");
  MMSEQ_REQUIRE(A && B && C && a_scales && b_scales, "gemm_mxfp8: null buffer");
  MMSEQ_REQUIRE(!resid || (ldr >= N && ldr % 4 == 0), "gemm_mxfp8: ldr");
  MMSEQ_REQUIRE(((uintptr_t)C & 7) == 0 && (!resid || ((uintptr_t)resid & 7) == 0),
                "gemm_mxfp8: 8-byte aligned output");
  if (M == 0) return MMSEQ_OK;
#ifndef MMSEQ_F8_OLD
  {  // the 256 x 256 8-phase schedule (gemm256.hip, F8) when K % 256 == 0 and there are tiles for it
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
    g.bias = bias; g.act = act; g.resid = resid; g.ldr = ldr; g.alpha = alpha;
    g.splitk = 1; g.kchunk = K; g.drop = make_drop(nullptr);
    g.f8_sa = (const uint8_t*)a_scales; g.f8_sb = (const uint8_t*)b_scales;
    g.f8_sa_bytes = mmseq_mxfp8_scale_bytes(M, K); g.f8_sb_bytes = mmseq_mxfp8_scale_bytes(N, K);
    hipError_t e = hipSuccess;
    if (M >= 256 && N >= 256 &&
        mmseq_gemm256_nt_f8(g, mmseq_device_cus(), reinterpret_cast<hipStream_t>(stream), &e)) {
      if (e != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm_mxfp8 launch: %s", hipGetErrorString(e));
      return mmseq_check_launch("gemm_mxfp8");
    }
  }
#endif
  // 256 x 256 tiles once there are rows and columns for them, else 128 x 128
  const bool wide = M >= 512 && N >= 256;
  const int tile = wide ? 256 : 128;
  const int tiles_m = (M + tile - 1) / tile, tiles_n = (N + tile - 1) / tile;
  MMSEQ_REQUIRE((int64_t)tiles_m * tiles_n < (1ll << 31), "gemm_mxfp8: too many tiles");
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
  a.bias = bias; a.act = act; a.resid = resid; a.ldr = ldr; a.alpha = alpha;
  a.vec_c = 1;
  hipLaunchKernelGGL(wide ? gemm_mxfp8_nt256x256_kernel : gemm_mxfp8_nt_kernel,
                     dim3(tiles_m * tiles_n), dim3(wide ? 512 : 256), 0,
                     reinterpret_cast<hipStream_t>(stream), a, (const uint8_t*)a_scales,
                     (const uint8_t*)b_scales, mmseq_mxfp8_scale_bytes(M, K),
                     mmseq_mxfp8_scale_bytes(N, K), tiles_n);
  return mmseq_check_launch("gemm_mxfp8");
}

// Training GEMM on the fp8 MFMA (BASELINE config 5): C (bf16) = dropout(act(A B^T + bias)) + resid
// with aux = the pre-activation, or, with q, the MX-fp8 output q + q_scales (and C then its bf16
// copy, aux the pre-activation; no residual / dropout): the MLP's FC1 writes what the backward reads
// (bf16 GELU output and pre-activation) and FC2's fp8 operand in one epilogue; or, with dact, the
// dgrad form C = (A B^T) * act'(dact) (with q: its MX-fp8 copy for the next dgrad GEMM too, C then
// the bf16 copy the weight gradient reads). The 256 x 256 8-phase F8 schedule only (K % 256 == 0,
// M and N >= 256); otherwise MMSEQ_EUNSUPPORTED.
extern "C" mmseq_status mmseq_gemm_mxfp8_ex(int M, int N, int K, const void* A, int64_t lda,
                                            const void* a_scales, const void* B, int64_t ldb,
                                            const void* b_scales, void* C, int64_t ldc,
                                            const float* bias, int act, void* aux,
                                            const void* dact, const void* resid, int64_t ldr,
                                            const mmseq_dropout* drop, void* q, int64_t ldq,
                                            void* q_scales, mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && N > 0 && K > 0, "gemm_mxfp8_ex: sizes");
  MMSEQ_REQUIRE(A && B && a_scales && b_scales && (C || q), "gemm_mxfp8_ex: null buffer");
  MMSEQ_REQUIRE(!q == !q_scales, "gemm_mxfp8_ex: q and q_scales go together");
  MMSEQ_REQUIRE(!aux || act, "gemm_mxfp8_ex: aux needs an activation");
  MMSEQ_REQUIRE(!dact || (act && !aux && !resid && !bias && !(drop && drop->p > 0.f)),
                "gemm_mxfp8_ex: dact (dgrad) takes an activation and nothing else");
  MMSEQ_REQUIRE(act == 0 || act == MMSEQ_ACT_GELU_ERF || act == MMSEQ_ACT_QUICKGELU,
                "gemm_mxfp8_ex: act");
  if (M == 0) return MMSEQ_OK;
  if (K % 256 != 0 || M < 256 || N < 256)
    return mmseq_set_error(MMSEQ_EUNSUPPORTED, "gemm_mxfp8_ex: needs K %% 256 == 0 and M, N >= 256");
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = lda; g.B = B; g.ldb = ldb;
  g.bias = bias; g.act = act; g.aux = aux; g.dact = dact; g.resid = resid; g.ldr = resid ? ldr : 0;
  g.alpha = 1.f; g.splitk = 1; g.kchunk = K;
  g.drop = make_drop(drop);
  if (q) {
    g.C = q; g.ldc = ldq;
    g.q8_scales = reinterpret_cast<uint8_t*>(q_scales);
    g.cbf = C; g.ldcb = ldc;
  } else {
    g.C = C; g.ldc = ldc;
  }
  g.f8_sa = (const uint8_t*)a_scales; g.f8_sb = (const uint8_t*)b_scales;
  g.f8_sa_bytes = mmseq_mxfp8_scale_bytes(M, K); g.f8_sb_bytes = mmseq_mxfp8_scale_bytes(N, K);
  hipError_t e = hipSuccess;
  MMSEQ_REQUIRE(mmseq_gemm256_nt_f8(g, mmseq_device_cus(), reinterpret_cast<hipStream_t>(stream), &e),
                "gemm_mxfp8_ex: preconditions (leading dimensions, alignment, epilogue combination)");
  if (e != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm_mxfp8_ex launch: %s", hipGetErrorString(e));
  return mmseq_check_launch("gemm_mxfp8_ex");
}

extern "C" mmseq_status mmseq_gemm_mxfp8_out(int M, int N, int K, const void* A, int64_t lda,
                                             const void* B, int64_t ldb, const float* bias,
                                             int act, void* q, int64_t ldq, void* scales,
                                             mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 128 == 0 && N % 32 == 0,
                "gemm_mxfp8_out: K % 128 and N % 32 must be 0");
  MMSEQ_REQUIRE(lda >= K && ldb >= K && lda % 8 == 0 && ldb % 8 == 0 && ldq >= N && ldq % 16 == 0,
                "gemm_mxfp8_out: leading dimensions");
  MMSEQ_REQUIRE(A && B && q && scales, "gemm_mxfp8_out: null buffer");
  MMSEQ_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 && ((uintptr_t)q & 15) == 0,
                "gemm_mxfp8_out: 16-byte alignment");
  MMSEQ_REQUIRE(act == 0 || act == MMSEQ_ACT_GELU_ERF || act == MMSEQ_ACT_QUICKGELU,
                "gemm_mxfp8_out: act");
  if (M == 0) return MMSEQ_OK;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = q; a.ldc = ldq;
  a.bias = bias; a.act = act; a.alpha = 1.f; a.splitk = 1; a.kchunk = K;
  a.drop = make_drop(nullptr);
  a.q8_scales = reinterpret_cast<uint8_t*>(scales);
  hipError_t e = hipSuccess;
  MMSEQ_REQUIRE(mmseq_gemm256_nt_q8(a, mmseq_device_cus(), reinterpret_cast<hipStream_t>(stream), &e),
                "gemm_mxfp8_out: preconditions");
  if (e != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm_mxfp8_out launch: %s", hipGetErrorString(e));
  return mmseq_check_launch("gemm_mxfp8_out");
}

extern "C" mmseq_status mmseq_gemm_mxfp8_q8(int M, int N, int K, const void* A, int64_t lda,
                                            const void* a_scales, const void* B, int64_t ldb,
                                            const void* b_scales, const float* bias, int act,
                                            void* q, int64_t ldq, void* q_scales,
                                            mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 256 == 0 && N % 32 == 0,
                "gemm_mxfp8_q8: K % 256 and N % 32 must be 0");
  MMSEQ_REQUIRE(lda >= K && ldb >= K && lda % 16 == 0 && ldb % 16 == 0 && ldq >= N && ldq % 16 == 0,
                "gemm_mxfp8_q8: leading dimensions");
  MMSEQ_REQUIRE(A && B && a_scales && b_scales && q && q_scales, "gemm_mxfp8_q8: null buffer");
  MMSEQ_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 && ((uintptr_t)q & 15) == 0,
                "gemm_mxfp8_q8: 16-byte alignment");
  MMSEQ_REQUIRE(act == 0 || act == MMSEQ_ACT_GELU_ERF || act == MMSEQ_ACT_QUICKGELU,
                "gemm_mxfp8_q8: act");
  if (M == 0) return MMSEQ_OK;
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = q; g.ldc = ldq;
  g.bias = bias; g.act = act; g.alpha = 1.f; g.splitk = 1; g.kchunk = K;
  g.drop = make_drop(nullptr);
  g.q8_scales = reinterpret_cast<uint8_t*>(q_scales);
  g.f8_sa = (const uint8_t*)a_scales; g.f8_sb = (const uint8_t*)b_scales;
  g.f8_sa_bytes = mmseq_mxfp8_scale_bytes(M, K); g.f8_sb_bytes = mmseq_mxfp8_scale_bytes(N, K);
  hipError_t e = hipSuccess;
  MMSEQ_REQUIRE(mmseq_gemm256_nt_f8(g, mmseq_device_cus(), reinterpret_cast<hipStream_t>(stream), &e),
                "gemm_mxfp8_q8: preconditions");
  if (e != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm_mxfp8_q8 launch: %s", hipGetErrorString(e));
  return mmseq_check_launch("gemm_mxfp8_q8");
}
