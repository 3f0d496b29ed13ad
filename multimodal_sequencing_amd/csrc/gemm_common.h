// Shared pieces of the GEMM kernels (gemm.hip, gemm256.hip): argument block, fused epilogue,
// buffer-resource LDS-DMA helpers.
#pragma once
#include "common.h"

namespace mmseq_gemm_detail {

struct GemmArgs {
  int M, N, K;
  const void* A; int64_t lda, sA;
  const void* B; int64_t ldb, sB;
  void* C; int64_t ldc, sC;
  const float* bias; int act; void* aux; const void* dact; const void* resid; int64_t ldr, sR;
  float alpha; int accumulate; int vec_ok; int vec_c;
  int splitk; int kchunk; float* slab;  // split-K (TN wgrad): partial slabs [splitk][M][N] f32
  Drop drop;                            // dropout after the activation, before the residual
  float* cs;       // TN wgrad: fused bias gradient cs[m] += sum_k A[k][m] (nullptr: off)
  float* cs_slab;  // ... its partials [splitk][column tile][M] (nullptr: first column tile adds to cs)
  uint8_t* q8_scales;  // 256 NT kernel, MX-fp8 output: C is e4m3 [M][ldc] + these packed scales
  // 256 NT kernel, MX-fp8 operands (F8): A / B are e4m3 [rows][ld] with these packed E8M0 scales
  const uint8_t* f8_sa; const uint8_t* f8_sb; int64_t f8_sa_bytes, f8_sb_bytes;
  // MX-fp8 output (q8_scales) of a training forward: the bf16 output too (cbf [M][ldcb]) and the
  // pre-activation (aux, same layout) that the backward reads
  void* cbf; int64_t ldcb;
};

template <typename TO>
__device__ __forceinline__ void epilogue4(const GemmArgs& a, TO* __restrict__ C, const TO* resid,
                                          TO* aux, const TO* dact, int m, int n, const float* acc,
                                          int b = 0) {
  if (m >= a.M || n >= a.N) return;
  float v[4];
  bool full = (n + 3 < a.N);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[r] = acc[r] * a.alpha;
    if (a.bias && n + r < a.N) v[r] += a.bias[n + r];
  }
  TO* cp = C + (int64_t)m * a.ldc + n;
  if (dact) {
    const TO* dp = dact + (int64_t)m * a.ldc + n;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < a.N)
        v[r] *= sizeof(TO) == 2 ? act_bwd_fast(a.act, Elem<TO>::ld(dp + r))
                                : act_bwd(a.act, Elem<TO>::ld(dp + r));
  } else if (a.act) {
    TO* ap = aux ? aux + (int64_t)m * a.ldc + n : nullptr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (n + r < a.N) {
        if (ap) Elem<TO>::st(ap + r, v[r]);
        // bf16 out: branch-free erf (|error| <= 1.5e-7, far below bf16 resolution); the fp32
        // parity path keeps libm's erff
        v[r] = sizeof(TO) == 2 ? act_fwd_fast(a.act, v[r]) : act_fwd(a.act, v[r]);
      }
    }
  }
  if (a.drop.thr) {
    const int64_t di = ((int64_t)b * a.M + m) * a.N + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= drop_mul(a.drop, di + r);
  }
  if (resid) {
    const TO* rp = resid + (int64_t)m * a.ldr + n;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < a.N) v[r] += Elem<TO>::ld(rp + r);
  }
  if (a.accumulate) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < a.N) v[r] += Elem<TO>::ld(cp + r);
  }
  if (full && a.vec_c) {
    if (sizeof(TO) == 2) {
      u16x4 o = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
      *reinterpret_cast<u16x4*>(cp) = o;
    } else {
      f32x4 o = {v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(cp) = o;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < a.N) Elem<TO>::st(cp + r, v[r]);
  }
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, int64_t bytes) {
  uint32_t n = bytes <= 0 ? 0u : (bytes >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

// XCD-aware work index: workgroups are dispatched round-robin over the 8 XCDs (block b on XCD
// b & 7), so XCD x holds q + (x < r) of the G = 8q + r blocks; numbering each XCD's blocks
// consecutively gives the ones that share operand panels (same K-split / neighbouring tiles)
// one L2. A bijection on [0, G) for any G.
__device__ __forceinline__ int xcd_item(int b, int G) {
  const int q = G >> 3, r = G & 7, x = b & 7;
  return x * q + min(x, r) + (b >> 3);
}

// 16-byte-per-lane LDS-DMA (buffer_load_dwordx4 ... lds; destination M0 + 16 * lane), issued
// as inline asm on purpose: the compiler's waitcnt pass cannot tell an in-flight DMA into one LDS
// buffer from a ds_read_b64_tr_b16 of the other and puts a vmcnt(0) in front of every transposed
// read, which waits out the next tile's prefetch in the middle of the current one. Every reader of
// DMA'd data therefore waits explicitly (counted s_waitcnt vmcnt + s_barrier), which the kernels
// do anyway. m0 is a reserved register that the compiler only materialises right before its own
// m0 readers; none are left in these kernels (tests/test_structure.py audits the code object).
__device__ __forceinline__ void dma16(rsrc_t r, unsigned short* lds, uint32_t voff) {
  const uint32_t la = (uint32_t)(uintptr_t)lds;  // low 32 bits of an LDS-aperture address
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(la)), "v"(voff), "s"(r) : "memory");
}


}  // namespace mmseq_gemm_detail

// persistent 256 x 256 NT kernel (gemm256.hip); returns false when its preconditions fail
// variant 0: one 8-wave 256 x 256 block per CU; 1: two 4-wave 256 x 128 blocks per CU.
// delay: shader cycles by which the blocks with one tile fewer start late (0: none)
bool mmseq_gemm256_nt(const mmseq_gemm_detail::GemmArgs& a, bool out_bf16, int num_cu, hipStream_t s,
                      hipError_t* err, int variant, int delay);
// ... with the activations written as MX-fp8 (e4m3 + packed E8M0 per 32 columns, fp8.hip
// layout) instead of bf16: the consumer GEMM's A operand without a quantisation pass
bool mmseq_gemm256_nt_q8(const mmseq_gemm_detail::GemmArgs& a, int num_cu, hipStream_t s,
                         hipError_t* err);
bool mmseq_gemm256_nt_f8(const mmseq_gemm_detail::GemmArgs& a, int num_cu, hipStream_t s,
                         hipError_t* err);
// CU count of the current device (write-once per-device table, gemm.hip)
int mmseq_device_cus();
// 256 x 256 TN (wgrad) kernel, fp32 out: a.splitk / a.kchunk (multiple of 128) / a.slab set by the
// caller (slab [splitk][M][N] when splitk > 1); returns false when its preconditions fail
bool mmseq_gemm256_tn(const mmseq_gemm_detail::GemmArgs& a, hipStream_t s, hipError_t* err);
