// MFMA GEMM for every Linear on the path (see include/mmseq.h: mmseq_gemm).
//
// Design (gfx950): 256-thread workgroups (4 waves, 2x2), 128x128 output tile, each wave a 64x64
// sub-tile of 4x4 MFMA 16x16 tiles. bf16 operands use v_mfma_f32_16x16x32_bf16 (BK = 64),
// fp32 operands the exact-fp32 v_mfma_f32_16x16x4_f32 (BK = 32, parity mode).
// Two operand layouts only:
//   NT (forward  Y = X W^T, dgrad dX = dY W with the bf16 W^T shadow): both operands
//      K-contiguous -> LDS [rows][BK+pad], fragments by 16-byte ds_read_b128 row reads.
//   TN (wgrad  dW = dY^T X): both operands M/N-contiguous -> LDS [BK][rows+pad], fragments by
//      ds_read_b64_tr_b16 transposed reads; the k order inside a 32-step is permuted identically
//      for both operands ({4g..4g+3} U {16+4g..16+4g+3} for lane group g) so every 32-lane half of
//      a transposed read touches 8 distinct LDS rows spaced 72 dwords apart: conflict-free.
// The MFMA is issued with the operands swapped (B-fragment as "A"), so each accumulator holds
// C^T: lane (g = l>>4, i = l&15) owns C[m0+i][n0+4g .. n0+4g+3] -> 4 contiguous outputs per lane
// for the fused epilogue (bias, activation / activation-backward, residual, accumulate).
// Staging: global -> registers (16 B per lane per chunk, issued before the MFMA loop of the
// previous tile) -> LDS after the barrier (the async-STAGE split of the guide, T14).
#include <cstdlib>
#include "gemm_common.h"

#include <atomic>

// The ABI is stateless: kernel selection and the split-K slab workspace are per-call arguments.
// The only process-wide state is this lazily filled, per-device, write-once CU-count table.
static std::atomic<int> g_cu_table[64];

static int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = g_cu_table[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  // MMSEQ_GEMM_CUS: persistent-grid size override for measurement (tools/gemm_epi_bench.py),
  // read once per device
  if (const char* e = getenv("MMSEQ_GEMM_CUS")) {
    const int v = atoi(e);
    if (v > 0 && v <= n) n = v;
  }
  g_cu_table[dev].store(n, std::memory_order_relaxed);
  return n;
}
int mmseq_device_cus() { return device_cus(); }

// Per-call kernel selection (mmseq_gemm `variant`, include/mmseq.h)
struct GemmSel {
  bool disable_fast;  // generic register-staged kernel only
  int big;            // 256 x 256 NT / TN kernels: 1 for large problems, 2 always, 0 never
  bool ring;          // BK=32 four-slot ring kernel instead of the BK=64 double-buffer kernel
  int nt_variant;     // large NT: 0 = 256x256 one block/CU, 1 = 256x128 two blocks/CU
  int nt_delay;       // large NT: start delay (cycles) of the blocks with one tile fewer
  int num_cu;
};

static bool make_sel(int variant, GemmSel* s) {
  if (variant < 0 || variant > 6) return false;
  s->disable_fast = variant == 0;
  s->big = variant == 1 ? 1 : ((variant >= 4) ? 2 : 0);
  s->nt_variant = variant == 5 ? 1 : (variant == 6 ? 2 : 0);
  s->ring = variant == 3;
  s->nt_delay = 0;
  s->num_cu = device_cus();
  return true;
}

namespace {
using namespace mmseq_gemm_detail;

constexpr int BM = 128, BN = 128, NT_THREADS = 256;

template <typename TI> struct Cfg;
template <> struct Cfg<unsigned short> {  // bf16
  static constexpr int BK = 64, VE = 8;
  static constexpr int PADK = 16;  // NT row = 80 elems = 160 B (conflict-free b128 row reads)
  static constexpr int PADM = 16;  // TN row = 144 elems = 288 B = 72 dwords (== 8 mod 64)
};
template <> struct Cfg<float> {
  static constexpr int BK = 32, VE = 4;
  static constexpr int PADK = 4;   // NT row = 36 floats
  static constexpr int PADM = 4;   // TN row = 132 floats
};

template <typename TI, bool TRANS>
struct Tile {
  static constexpr int BK = Cfg<TI>::BK, VE = Cfg<TI>::VE;
  // NT: [rows][BK+PADK]; TN: [BK][rows+PADM]
  static constexpr int LD = TRANS ? (BM + Cfg<TI>::PADM) : (BK + Cfg<TI>::PADK);
  static constexpr int ELEMS = TRANS ? BK * LD : BM * LD;
  static constexpr int CHUNKS_PER_ROW = TRANS ? BM / VE : BK / VE;
  static constexpr int NCHUNK = (BM * BK / VE) / NT_THREADS;  // = 4
};

template <typename TI> struct Vec16;
template <> struct Vec16<unsigned short> { typedef u16x8 T; };
template <> struct Vec16<float> { typedef f32x4 T; };

// Load chunk `c` of this thread for one operand tile into registers (zero-fill out of range).
// rows_lim = M (or N) bound for the "row" (m/n) index; K bound for k.
template <typename TI, bool TRANS>
__device__ __forceinline__ typename Vec16<TI>::T load_chunk(const TI* __restrict__ base, int64_t ld,
                                                            int row0, int k0, int c, int tid,
                                                            int rows_lim, int K, bool vec_ok) {
  typedef Tile<TI, TRANS> Tl;
  typedef typename Vec16<TI>::T V;
  constexpr int VE = Tl::VE;
  int L = c * NT_THREADS + tid;
  int r = L / Tl::CHUNKS_PER_ROW, cc = L % Tl::CHUNKS_PER_ROW;
  V out;
  if (!TRANS) {
    int row = row0 + r, k = k0 + cc * VE;
    const TI* p = base + (int64_t)row * ld + k;
    if (row < rows_lim && vec_ok && k + VE <= K) {
      out = *reinterpret_cast<const V*>(p);
    } else {
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        TI v = 0;
        if (row < rows_lim && k + e < K) v = p[e];
        out[e] = v;
      }
    }
  } else {
    int k = k0 + r, col = row0 + cc * VE;
    const TI* p = base + (int64_t)k * ld + col;
    if (k < K && vec_ok && col + VE <= rows_lim) {
      out = *reinterpret_cast<const V*>(p);
    } else {
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        TI v = 0;
        if (k < K && col + e < rows_lim) v = p[e];
        out[e] = v;
      }
    }
  }
  return out;
}

template <typename TI, bool TRANS>
__device__ __forceinline__ void store_chunk(TI* __restrict__ s, typename Vec16<TI>::T v, int c,
                                            int tid) {
  typedef Tile<TI, TRANS> Tl;
  int L = c * NT_THREADS + tid;
  int r = L / Tl::CHUNKS_PER_ROW, cc = L % Tl::CHUNKS_PER_ROW;
  *reinterpret_cast<typename Vec16<TI>::T*>(s + r * Tl::LD + cc * Tl::VE) = v;
}

// ---- fragment reads ------------------------------------------------------------------------
// bf16 NT: lane (g, i) -> 8 contiguous k of row (rb + i) at k = ks*32 + 8g.
__device__ __forceinline__ bf16x8_t frag_nt_bf16(const unsigned short* s, int rb, int ks, int lane) {
  typedef Tile<unsigned short, false> Tl;
  const unsigned short* p = s + (rb + (lane & 15)) * Tl::LD + ks * 32 + (lane >> 4) * 8;
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8*>(p));
}
// bf16 TN: two ds_read_b64_tr_b16; lane (g, i=4q+p) supplies row (ks*32 + 4g + q [+16]),
// columns rb + 4p .. +3, and receives column rb + i of the 4 rows.
__device__ __forceinline__ bf16x8_t frag_tn_bf16(const unsigned short* s, int rb, int ks, int lane) {
  typedef Tile<unsigned short, true> Tl;
  int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const unsigned short* a0 = s + (ks * 32 + 4 * g + q) * Tl::LD + rb + 4 * p;
  const unsigned short* a1 = a0 + 16 * Tl::LD;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MMSEQ_LDS s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MMSEQ_LDS s16x4*)(a1));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <typename TI, typename TO, bool TRANS>
__global__ __launch_bounds__(NT_THREADS) void gemm_kernel(GemmArgs a) {
  typedef Tile<TI, TRANS> Tl;
  typedef typename Vec16<TI>::T V;
  constexpr int BK = Tl::BK;
  __shared__ __attribute__((aligned(16))) TI smem[2 * Tl::ELEMS];
  TI* sA = smem;
  TI* sB = smem + Tl::ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  // split-K (plain fp32 TN / NT with few tiles): blockIdx.z is the K slice, output a raw slab
  const int split = a.splitk > 1 ? blockIdx.z : 0, b = a.splitk > 1 ? 0 : blockIdx.z;
  const int kbeg = split * a.kchunk;
  const int kend = a.splitk > 1 ? min(a.K, kbeg + a.kchunk) : a.K;
  const TI* A = reinterpret_cast<const TI*>(a.A) + (int64_t)b * a.sA;
  const TI* B = reinterpret_cast<const TI*>(a.B) + (int64_t)b * a.sB;
  const bool vec = a.vec_ok;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  V ra[Tl::NCHUNK], rb[Tl::NCHUNK];
  const int nk = (kend - kbeg + BK - 1) / BK;
#pragma unroll
  for (int c = 0; c < Tl::NCHUNK; ++c) {
    ra[c] = load_chunk<TI, TRANS>(A, a.lda, m0, kbeg, c, tid, a.M, kend, vec);
    rb[c] = load_chunk<TI, TRANS>(B, a.ldb, n0, kbeg, c, tid, a.N, kend, vec);
  }
#pragma unroll
  for (int c = 0; c < Tl::NCHUNK; ++c) {
    store_chunk<TI, TRANS>(sA, ra[c], c, tid);
    store_chunk<TI, TRANS>(sB, rb[c], c, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
#pragma unroll
      for (int c = 0; c < Tl::NCHUNK; ++c) {
        ra[c] = load_chunk<TI, TRANS>(A, a.lda, m0, kbeg + (kt + 1) * BK, c, tid, a.M, kend, vec);
        rb[c] = load_chunk<TI, TRANS>(B, a.ldb, n0, kbeg + (kt + 1) * BK, c, tid, a.N, kend, vec);
      }
    }
    if constexpr (sizeof(TI) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8_t fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (TRANS) {
            fa[i] = frag_tn_bf16((const unsigned short*)sA, wr * 64 + i * 16, ks, lane);
            fb[i] = frag_tn_bf16((const unsigned short*)sB, wc * 64 + i * 16, ks, lane);
          } else {
            fa[i] = frag_nt_bf16((const unsigned short*)sA, wr * 64 + i * 16, ks, lane);
            fb[i] = frag_nt_bf16((const unsigned short*)sB, wc * 64 + i * 16, ks, lane);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    } else {
      const int g = lane >> 4, ii = lane & 15;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (TRANS) {
            fa[i] = ((const float*)sA)[(kk + g) * Tl::LD + wr * 64 + i * 16 + ii];
            fb[i] = ((const float*)sB)[(kk + g) * Tl::LD + wc * 64 + i * 16 + ii];
          } else {
            fa[i] = ((const float*)sA)[(wr * 64 + i * 16 + ii) * Tl::LD + kk + g];
            fb[i] = ((const float*)sB)[(wc * 64 + i * 16 + ii) * Tl::LD + kk + g];
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
#pragma unroll
      for (int c = 0; c < Tl::NCHUNK; ++c) {
        store_chunk<TI, TRANS>(sA, ra[c], c, tid);
        store_chunk<TI, TRANS>(sB, rb[c], c, tid);
      }
      __syncthreads();
    }
  }

  const int g = lane >> 4, ii = lane & 15;
  if (a.splitk > 1) {  // raw fp32 partial slab [split][M][N], reduced by splitk_reduce
    float* slab = a.slab + (int64_t)split * a.M * a.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wr * 64 + i * 16 + ii;
        const int n = n0 + wc * 64 + j * 16 + 4 * g;
        if (m < a.M) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < a.N) slab[(int64_t)m * a.N + n + r] = acc[i][j][r];
        }
      }
    return;
  }
  TO* C = reinterpret_cast<TO*>(a.C) + (int64_t)b * a.sC;
  const TO* resid = a.resid ? reinterpret_cast<const TO*>(a.resid) + (int64_t)b * a.sR : nullptr;
  TO* aux = a.aux ? reinterpret_cast<TO*>(a.aux) + (int64_t)b * a.sC : nullptr;
  const TO* dact = a.dact ? reinterpret_cast<const TO*>(a.dact) + (int64_t)b * a.sC : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int m = m0 + wr * 64 + i * 16 + ii;
      int n = n0 + wc * 64 + j * 16 + 4 * g;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epilogue4<TO>(a, C, resid, aux, dact, m, n, v, b);
    }
}

template <typename TI, typename TO>
hipError_t launch(int trans, const GemmArgs& a, int batch, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, batch);
  if (trans)
    hipLaunchKernelGGL((gemm_kernel<TI, TO, true>), grid, dim3(NT_THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_kernel<TI, TO, false>), grid, dim3(NT_THREADS), 0, s, a);
  return hipGetLastError();
}


// =============================================================================================
// Fast path (bf16, both layouts): LDS-DMA staging (buffer_load ... lds, 16 B per lane) into a
// two-stage double buffer, one barrier per 64-deep K-step, XOR-swizzled lane-linear LDS images
// (swizzle applied to the per-lane SOURCE offset, guide rule 21), XCD-aware block order (T1).
// Buffer resources give free zero-fill past the operand's last row (M/N edge for NT, K tail for
// TN). Preconditions (checked on the host): NT needs K % 64 == 0; TN needs M % 8 == 0 and
// N % 8 == 0; all leading dimensions multiples of 8, pointers 16-byte aligned.
//   NT image: [128 rows][64 k], 128-B rows, chunk' = chunk ^ ((row >> 1) & 7)  -> conflict-free
//             16-B row reads for the 16x16x32 operand (every 16-lane group hits 16 slots)
//   TN image: [64 k][128 m], 256-B rows, chunk' = chunk ^ ((row & 7) << 1)     -> conflict-free
//             ds_read_b64_tr_b16 (each 32-lane half reads 8 rows x 2 chunks = 16 slots)
// =============================================================================================
template <bool TRANS>
__device__ __forceinline__ bf16x8_t frag_swz(const unsigned short* s, int rb, int ks, int lane) {
  if (!TRANS) {
    const int rr = rb + (lane & 15), c = ks * 4 + (lane >> 4);
    const unsigned short* p = s + rr * 64 + ((c ^ ((rr >> 1) & 7)) << 3);
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8*>(p));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int r = ks * 32 + 4 * g + q, col = rb + 4 * pp;
    const unsigned short* a0 = s + r * 128 + (((col >> 3) ^ ((r & 7) << 1)) << 3) + (col & 7);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MMSEQ_LDS s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MMSEQ_LDS s16x4*)(a0 + 16 * 128));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

// issue this wave's 4 LDS-DMA pieces of one 128 x 64 operand tile
template <bool TRANS>
__device__ __forceinline__ void stage_operand(rsrc_t r, int64_t ld, int k0, unsigned short* s,
                                              int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int inst = wave * 4 + i;
    uint32_t voff;
    if (!TRANS) {
      const int row = inst * 8 + (lane >> 3), cp = lane & 7;
      const int c = cp ^ ((row >> 1) & 7);
      voff = (uint32_t)(((int64_t)row * ld + k0 + c * 8) * 2);
    } else {
      const int row = inst * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ ((row & 7) << 1);
      voff = (uint32_t)(((int64_t)row * ld + c * 8) * 2);  // base already advanced to k0
    }
    dma16(r, s + inst * 512, voff);
  }
}

template <typename TO, bool TRANS>
__global__ __launch_bounds__(256, 2) void gemm_fast_kernel(GemmArgs a, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * 2 * 128 * 64];  // 64 KB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  // XCD-aware bijective remap: blocks that share an A panel run on one XCD (one L2)
  const int nwg = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int Lr = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int tm = Lr / tiles_n, tn = Lr % tiles_n;
  const int m0 = tm * 128, n0 = tn * 128;
  const int split = a.splitk > 1 ? blockIdx.y : 0;
  const int b = a.splitk > 1 ? 0 : blockIdx.y;
  const int kbeg = split * a.kchunk;
  const int Kend = a.splitk > 1 ? min(a.K, kbeg + a.kchunk) : a.K;
  const unsigned short* A = reinterpret_cast<const unsigned short*>(a.A) + (int64_t)b * a.sA;
  const unsigned short* B = reinterpret_cast<const unsigned short*>(a.B) + (int64_t)b * a.sB;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (Kend - kbeg + 63) / 64;
  rsrc_t ra, rb;
  if (!TRANS) {
    ra = make_rsrc(A + (int64_t)m0 * a.lda, ((int64_t)(a.M - m0 - 1) * a.lda + a.K) * 2);
    rb = make_rsrc(B + (int64_t)n0 * a.ldb, ((int64_t)(a.N - n0 - 1) * a.ldb + a.K) * 2);
  }
  auto issue = [&](int kt, int stg) {
    unsigned short* sA = smem + stg * 16384;
    unsigned short* sB = sA + 8192;
    const int k0 = kbeg + kt * 64;
    if (!TRANS) {
      stage_operand<false>(ra, a.lda, k0, sA, wave, lane);
      stage_operand<false>(rb, a.ldb, k0, sB, wave, lane);
    } else {
      // rows k >= K fall outside the descriptor -> zero-filled
      rsrc_t ta = make_rsrc(A + (int64_t)k0 * a.lda + m0,
                            ((int64_t)(Kend - k0 - 1) * a.lda + (a.M - m0)) * 2);
      rsrc_t tb = make_rsrc(B + (int64_t)k0 * a.ldb + n0,
                            ((int64_t)(Kend - k0 - 1) * a.ldb + (a.N - n0)) * 2);
      stage_operand<true>(ta, a.lda, k0, sA, wave, lane);
      stage_operand<true>(tb, a.ldb, k0, sB, wave, lane);
    }
  };

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
    const unsigned short* sA = smem + cur * 16384;
    const unsigned short* sB = sA + 8192;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = frag_swz<TRANS>(sA, wr * 64 + i * 16, ks, lane);
        fb[i] = frag_swz<TRANS>(sB, wc * 64 + i * 16, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const int g = lane >> 4, ii = lane & 15;
  if (a.splitk > 1) {  // raw fp32 partial slab, reduced (deterministically) by splitk_reduce
    float* slab = a.slab + (int64_t)split * a.M * a.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int m = m0 + wr * 64 + i * 16 + ii;
        int n = n0 + wc * 64 + j * 16 + 4 * g;
        if (m < a.M && n < a.N)  // N % 8 == 0 on this path: n..n+3 all in range
          *reinterpret_cast<f32x4*>(slab + (int64_t)m * a.N + n) = acc[i][j];
      }
    return;
  }
  TO* C = reinterpret_cast<TO*>(a.C) + (int64_t)b * a.sC;
  const TO* resid = a.resid ? reinterpret_cast<const TO*>(a.resid) + (int64_t)b * a.sR : nullptr;
  TO* aux = a.aux ? reinterpret_cast<TO*>(a.aux) + (int64_t)b * a.sC : nullptr;
  const TO* dact = a.dact ? reinterpret_cast<const TO*>(a.dact) + (int64_t)b * a.sC : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int m = m0 + wr * 64 + i * 16 + ii;
      int n = n0 + wc * 64 + j * 16 + 4 * g;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epilogue4<TO>(a, C, resid, aux, dact, m, n, v, b);
    }
}


// ---------------------------------------------------------------------------------------------
// Ring variant: BK = 32, four-slot LDS ring (16 KB per slot), three K-steps in flight behind a
// COUNTED vmcnt and a raw s_barrier (guide §5 "Pipelining across barriers": __syncthreads()
// would drain every LDS-DMA with vmcnt(0)). 64 KB per workgroup -> 2 workgroups per CU.
//   NT image: [128 rows][32 k], 64-B rows, chunk' = chunk ^ (((row >> 3) & 1) << 1)
//   TN image: [32 k][128 m], 256-B rows, chunk' = chunk ^ ((row & 7) << 1)
// ---------------------------------------------------------------------------------------------
template <bool TRANS>
__device__ __forceinline__ void stage32(rsrc_t r, int64_t ld, int k0, unsigned short* s, int wave,
                                        int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = wave * 2 + i;
    uint32_t voff;
    if (!TRANS) {
      const int row = inst * 16 + (lane >> 2), cp = lane & 3;
      const int c = cp ^ (((row >> 3) & 1) << 1);
      voff = (uint32_t)(((int64_t)row * ld + k0 + c * 8) * 2);
    } else {
      const int row = inst * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ ((row & 7) << 1);
      voff = (uint32_t)(((int64_t)row * ld + c * 8) * 2);
    }
    dma16(r, s + inst * 512, voff);
  }
}

template <bool TRANS>
__device__ __forceinline__ bf16x8_t frag32(const unsigned short* s, int rb, int lane) {
  if (!TRANS) {
    const int rr = rb + (lane & 15), c = lane >> 4;
    const unsigned short* p = s + rr * 32 + ((c ^ (((rr >> 3) & 1) << 1)) << 3);
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8*>(p));
  }
  return frag_swz<true>(s, rb, 0, lane);
}

template <typename TO, bool TRANS>
__global__ __launch_bounds__(256, 2) void gemm_ring_kernel(GemmArgs a, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned short smem[4 * 2 * 128 * 32];  // 64 KB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nwg = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int Lr = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int tm = Lr / tiles_n, tn = Lr % tiles_n;
  const int m0 = tm * 128, n0 = tn * 128;
  const int split = a.splitk > 1 ? blockIdx.y : 0;
  const int b = a.splitk > 1 ? 0 : blockIdx.y;
  const int kbeg = split * a.kchunk;
  const int Kend = a.splitk > 1 ? min(a.K, kbeg + a.kchunk) : a.K;
  const unsigned short* A = reinterpret_cast<const unsigned short*>(a.A) + (int64_t)b * a.sA;
  const unsigned short* B = reinterpret_cast<const unsigned short*>(a.B) + (int64_t)b * a.sB;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (Kend - kbeg + 31) / 32;
  rsrc_t ra, rb;
  if (!TRANS) {
    ra = make_rsrc(A + (int64_t)m0 * a.lda, ((int64_t)(a.M - m0 - 1) * a.lda + a.K) * 2);
    rb = make_rsrc(B + (int64_t)n0 * a.ldb, ((int64_t)(a.N - n0 - 1) * a.ldb + a.K) * 2);
  }
  auto issue = [&](int kt) {
    unsigned short* sA = smem + (kt & 3) * 8192;
    unsigned short* sB = sA + 4096;
    const int k0 = kbeg + kt * 32;
    if (!TRANS) {
      stage32<false>(ra, a.lda, k0, sA, wave, lane);
      stage32<false>(rb, a.ldb, k0, sB, wave, lane);
    } else {
      rsrc_t ta = make_rsrc(A + (int64_t)k0 * a.lda + m0,
                            ((int64_t)(Kend - k0 - 1) * a.lda + (a.M - m0)) * 2);
      rsrc_t tb = make_rsrc(B + (int64_t)k0 * a.ldb + n0,
                            ((int64_t)(Kend - k0 - 1) * a.ldb + (a.N - n0)) * 2);
      stage32<true>(ta, a.lda, k0, sA, wave, lane);
      stage32<true>(tb, a.ldb, k0, sB, wave, lane);
    }
  };

  issue(0);
  if (nk > 1) issue(1);
  if (nk > 2) issue(2);
  for (int kt = 0; kt < nk; ++kt) {
    // retire this wave's DMA for step kt; later steps (4 instructions each) may stay in flight
    const int later = nk - 1 - kt;
    if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA for kt landed; slot (kt-1)&3 fully read
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 3 < nk) issue(kt + 3);
    const unsigned short* sA = smem + (kt & 3) * 8192;
    const unsigned short* sB = sA + 4096;
    bf16x8_t fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i] = frag32<TRANS>(sA, wr * 64 + i * 16, lane);
      fb[i] = frag32<TRANS>(sB, wc * 64 + i * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  }

  const int g = lane >> 4, ii = lane & 15;
  if (a.splitk > 1) {
    float* slab = a.slab + (int64_t)split * a.M * a.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int m = m0 + wr * 64 + i * 16 + ii;
        int n = n0 + wc * 64 + j * 16 + 4 * g;
        if (m < a.M && n < a.N)
          *reinterpret_cast<f32x4*>(slab + (int64_t)m * a.N + n) = acc[i][j];
      }
    return;
  }
  TO* C = reinterpret_cast<TO*>(a.C) + (int64_t)b * a.sC;
  const TO* resid = a.resid ? reinterpret_cast<const TO*>(a.resid) + (int64_t)b * a.sR : nullptr;
  TO* aux = a.aux ? reinterpret_cast<TO*>(a.aux) + (int64_t)b * a.sC : nullptr;
  const TO* dact = a.dact ? reinterpret_cast<const TO*>(a.dact) + (int64_t)b * a.sC : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int m = m0 + wr * 64 + i * 16 + ii;
      int n = n0 + wc * 64 + j * 16 + 4 * g;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epilogue4<TO>(a, C, resid, aux, dact, m, n, v, b);
    }
}

// C[m][n] (+)= sum_s slab[s][m][n], fixed order (bitwise reproducible)
// out[m] += sum_s slab[s][m] (fused bias-gradient partials of the split-K wgrad; fixed order).
// S = splits x column tiles runs to ~100 partials: a block takes 32 columns and spreads the
// partials over 8 slices (slice j sums s = j, j + 8, ...), then adds the 8 slice sums in order
__global__ __launch_bounds__(256) void cs_reduce_kernel(int M, int S, const float* __restrict__ slab,
                                                        float* __restrict__ out) {
  __shared__ float red[8][32];
  const int c = threadIdx.x & 31, j = threadIdx.x >> 5;
  const int m = blockIdx.x * 32 + c;
  float v = 0.f;
  if (m < M) {
#pragma unroll 4
    for (int s = j; s < S; s += 8) v += slab[(int64_t)s * M + m];
  }
  red[j][c] = v;
  __syncthreads();
  if (j == 0 && m < M)
    out[m] += ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) +
              ((red[4][c] + red[5][c]) + (red[6][c] + red[7][c]));
}

// out[m] += sum_k A[k][m] (fallback bias gradient when the fused path is not eligible)
template <typename TI>
__global__ __launch_bounds__(256) void colsum_simple_kernel(int M, int K, const TI* __restrict__ A,
                                                            int64_t lda, float* __restrict__ out) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  float v = 0.f;
  for (int k = 0; k < K; ++k) v += Elem<TI>::ld(A + (int64_t)k * lda + m);
  out[m] += v;
}

// fp32 split-K with the full epilogue: v = sum_s slab[s][m][n .. n+3] in split order, then the
// same epilogue4 the unsplit kernel applies (bias, activation / aux / act', dropout, residual,
// accumulate), so splitting changes only the summation grouping of the dot products
__global__ __launch_bounds__(256) void splitk_epi_kernel(GemmArgs a, int S, const float* __restrict__ slab) {
  const int n4 = (a.N + 3) >> 2;
  const int64_t total = (int64_t)a.M * n4, MN = (int64_t)a.M * a.N;
  float* C = reinterpret_cast<float*>(a.C);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / n4), n = (int)(i - (int64_t)m * n4) * 4;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t e = (int64_t)m * a.N + n + r;
      float x = 0.f;
      if (n + r < a.N) {
        x = slab[e];
        for (int q = 1; q < S; ++q) x += slab[q * MN + e];
      }
      v[r] = x;
    }
    epilogue4<float>(a, C, reinterpret_cast<const float*>(a.resid), reinterpret_cast<float*>(a.aux),
                     reinterpret_cast<const float*>(a.dact), m, n, v, 0);
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(int M, int N, int S, const float* __restrict__ slab,
                                                            float* __restrict__ C, int64_t ldc,
                                                            int accumulate) {
  const int64_t total4 = (int64_t)M * N / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 4;
    const int m = e / N, n = e % N;
    f32x4 v = *reinterpret_cast<const f32x4*>(slab + e);
    for (int s = 1; s < S; ++s) v += *reinterpret_cast<const f32x4*>(slab + (int64_t)s * M * N + e);
    float* cp = C + (int64_t)m * ldc + n;
    if (accumulate) v += *reinterpret_cast<const f32x4*>(cp);
    *reinterpret_cast<f32x4*>(cp) = v;
  }
}

template <typename TO>
hipError_t launch_fast(int trans, const GemmArgs& a, int batch, hipStream_t s, const GemmSel& sel) {
  if (!trans && sel.big && a.splitk == 1 && batch == 1 && a.K % 128 == 0 &&
      (sel.big == 2 || (int64_t)((a.M + 255) / 256) * ((a.N + 255) / 256) >= 256)) {
    hipError_t e;
    if (mmseq_gemm256_nt(a, sizeof(TO) == 2, sel.num_cu, s, &e, sel.nt_variant, sel.nt_delay)) return e;
  }
  const int tiles_m = (a.M + 127) / 128, tiles_n = (a.N + 127) / 128;
  dim3 grid(tiles_m * tiles_n, a.splitk > 1 ? a.splitk : batch);
  if (sel.ring) {
    if (trans)
      hipLaunchKernelGGL((gemm_ring_kernel<TO, true>), grid, dim3(256), 0, s, a, tiles_n);
    else
      hipLaunchKernelGGL((gemm_ring_kernel<TO, false>), grid, dim3(256), 0, s, a, tiles_n);
    return hipGetLastError();
  }
  if (trans)
    hipLaunchKernelGGL((gemm_fast_kernel<TO, true>), grid, dim3(256), 0, s, a, tiles_n);
  else
    hipLaunchKernelGGL((gemm_fast_kernel<TO, false>), grid, dim3(256), 0, s, a, tiles_n);
  return hipGetLastError();
}

inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

}  // namespace

extern "C" mmseq_status mmseq_gemm(int trans, int M, int N, int K, int batch, const void* A,
                                   int64_t lda, int64_t strideA, const void* B, int64_t ldb,
                                   int64_t strideB, void* C, int64_t ldc, int64_t strideC,
                                   const float* bias, int act, void* aux_out, const void* dact_aux,
                                   const void* resid, int64_t ldr, int64_t strideR, float alpha,
                                   int accumulate, mmseq_dtype in_dtype, mmseq_dtype out_dtype,
                                   const mmseq_dropout* drop, int variant, void* workspace,
                                   int64_t workspace_bytes, mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "gemm: bad sizes M=%d N=%d K=%d b=%d",
                M, N, K, batch);
  MMSEQ_REQUIRE(A && B && C, "gemm: null operand");
  MMSEQ_REQUIRE(act >= 0 && act <= 4, "gemm: bad act %d", act);
  MMSEQ_REQUIRE(!(aux_out && dact_aux), "gemm: aux_out and dact_aux are exclusive");
  MMSEQ_REQUIRE(in_dtype == MMSEQ_F32 || in_dtype == MMSEQ_BF16, "gemm: bad in dtype");
  MMSEQ_REQUIRE(out_dtype == MMSEQ_F32 || out_dtype == MMSEQ_BF16, "gemm: bad out dtype");
  if (!trans) {
    MMSEQ_REQUIRE(lda >= K && ldb >= K && ldc >= N, "gemm NT: ld too small");
  } else {
    MMSEQ_REQUIRE(lda >= M && ldb >= N && ldc >= N, "gemm TN: ld too small");
  }
  MMSEQ_REQUIRE(workspace_bytes >= 0 && (workspace || workspace_bytes == 0) &&
                    ((uintptr_t)workspace & 15) == 0,
                "gemm: workspace must be 16-byte aligned (or NULL with 0 bytes)");
  GemmSel sel;
  MMSEQ_REQUIRE(make_sel(variant, &sel), "gemm: bad variant %d", variant);
  if (M == 0 || N == 0) return MMSEQ_OK;
  float* const g_slab = reinterpret_cast<float*>(workspace);
  const int64_t g_slab_bytes = workspace ? workspace_bytes : 0;
  const int g_num_cu = sel.num_cu;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda; a.sA = strideA;
  a.B = B; a.ldb = ldb; a.sB = strideB;
  a.C = C; a.ldc = ldc; a.sC = strideC;
  a.bias = bias; a.act = act; a.aux = aux_out; a.dact = dact_aux;
  a.resid = resid; a.ldr = resid ? ldr : 0; a.sR = strideR;
  a.alpha = alpha; a.accumulate = accumulate;
  a.drop = make_drop(drop);
  const int ve = in_dtype == MMSEQ_BF16 ? 8 : 4;
  a.vec_ok = al16(A) && al16(B) && lda % ve == 0 && ldb % ve == 0 && strideA % ve == 0 &&
             strideB % ve == 0;
  const int vc = 4;
  const int esz = out_dtype == MMSEQ_BF16 ? 2 : 4;
  a.vec_c = ((uintptr_t)C % (vc * esz) == 0) && ldc % vc == 0 && strideC % vc == 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  const bool fast_ok = in_dtype == MMSEQ_BF16 && a.vec_ok && !sel.disable_fast &&
                       (trans ? (M % 8 == 0 && N % 8 == 0) : (K % 64 == 0)) &&
                       (int64_t)M * N >= 128 * 128;
  a.splitk = 1; a.kchunk = K; a.slab = nullptr;
  a.cs = nullptr; a.cs_slab = nullptr;
  if (fast_ok) {
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    const bool plain = !bias && !act && !aux_out && !dact_aux && !resid && alpha == 1.0f &&
                       !a.drop.thr &&
                       out_dtype == MMSEQ_F32 && batch == 1 && ldc % 4 == 0 && al16(C);
    // weight gradients: 256 x 256 TN kernel, K split so that (tiles x splits) fills the CUs
    if (trans && plain && sel.big) {
      const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
      int S2 = t256 < g_num_cu ? g_num_cu / t256 : 1;
      if (S2 > K / 1024) S2 = K / 1024 > 0 ? K / 1024 : 1;
      while (S2 > 1 && (!g_slab || (int64_t)S2 * M * N * 4 > g_slab_bytes)) --S2;
      GemmArgs t = a;
      t.splitk = S2;
      t.kchunk = ((K + S2 - 1) / S2 + 127) / 128 * 128;
      t.splitk = (K + t.kchunk - 1) / t.kchunk;
      t.slab = g_slab;
      hipError_t e2 = hipSuccess;
      if (t.splitk <= 1) { t.splitk = 1; t.kchunk = K; }
      if (mmseq_gemm256_tn(t, s, &e2)) {
        if (e2 == hipSuccess && t.splitk > 1) {
          int64_t t4 = (int64_t)M * N / 4;
          unsigned blocks = (unsigned)((t4 + 255) / 256 < 4096 ? (t4 + 255) / 256 : 4096);
          hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, M, N, t.splitk,
                             g_slab, (float*)C, ldc, accumulate);
          e2 = hipGetLastError();
        }
        if (e2 != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm launch: %s", hipGetErrorString(e2));
        return MMSEQ_OK;
      }
    }
    int S = 1;
    if (trans && plain && g_slab && tiles < 512) {
      S = (1024 + tiles - 1) / tiles;
      const int maxS = K / (64 * 16);  // keep >= 16 K-steps per split
      if (S > maxS) S = maxS;
      while (S > 1 && (int64_t)S * M * N * 4 > g_slab_bytes) --S;
    }
    if (S > 1) {
      a.splitk = S;
      a.kchunk = ((K + S - 1) / S + 63) / 64 * 64;
      S = (K + a.kchunk - 1) / a.kchunk;
      a.splitk = S;
      a.slab = g_slab;
      e = launch_fast<float>(trans, a, 1, s, sel);
      if (e == hipSuccess) {
        int64_t t4 = (int64_t)M * N / 4;
        unsigned blocks = (unsigned)((t4 + 255) / 256 < 4096 ? (t4 + 255) / 256 : 4096);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, M, N, S, g_slab,
                           (float*)C, ldc, accumulate);
        e = hipGetLastError();
      }
    } else {
      e = out_dtype == MMSEQ_BF16 ? launch_fast<unsigned short>(trans, a, batch, s, sel)
                                  : launch_fast<float>(trans, a, batch, s, sel);
    }
  } else if (in_dtype == MMSEQ_F32 && out_dtype == MMSEQ_F32 && batch == 1 && g_slab &&
             ((M + 127) / 128) * ((N + 127) / 128) < 128 && K >= 256) {
    // fp32 GEMMs with few output tiles (the BERSON head: M = 16-400 rows per story batch, and
    // its weight gradients over all tokens): split K over the CUs, fp32 partial slabs, a
    // fixed-order reduction that applies the epilogue (bitwise reproducible)
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    int S = (g_num_cu + tiles - 1) / tiles;
    if (S > K / 128) S = K / 128;
    while (S > 1 && (int64_t)S * M * N * 4 > g_slab_bytes) --S;
    a.splitk = S;
    a.kchunk = ((K + S - 1) / S + 31) / 32 * 32;
    a.splitk = (K + a.kchunk - 1) / a.kchunk;
    a.slab = g_slab;
    if (a.splitk > 1) {
      dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, a.splitk);
      if (trans)
        hipLaunchKernelGGL((gemm_kernel<float, float, true>), grid, dim3(NT_THREADS), 0, s, a);
      else
        hipLaunchKernelGGL((gemm_kernel<float, float, false>), grid, dim3(NT_THREADS), 0, s, a);
      e = hipGetLastError();
      if (e == hipSuccess) {
        const int64_t tot = (int64_t)M * ((N + 3) / 4);
        const unsigned blocks = (unsigned)((tot + 255) / 256 < 4096 ? (tot + 255) / 256 : 4096);
        hipLaunchKernelGGL(splitk_epi_kernel, dim3(blocks), dim3(256), 0, s, a, a.splitk, g_slab);
        e = hipGetLastError();
      }
    } else {
      a.splitk = 1; a.kchunk = K; a.slab = nullptr;
      e = launch<float, float>(trans, a, batch, s);
    }
  } else if (in_dtype == MMSEQ_BF16 && out_dtype == MMSEQ_BF16)
    e = launch<unsigned short, unsigned short>(trans, a, batch, s);
  else if (in_dtype == MMSEQ_BF16 && out_dtype == MMSEQ_F32)
    e = launch<unsigned short, float>(trans, a, batch, s);
  else if (in_dtype == MMSEQ_F32 && out_dtype == MMSEQ_F32)
    e = launch<float, float>(trans, a, batch, s);
  else
    e = launch<float, unsigned short>(trans, a, batch, s);
  if (e != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm launch: %s", hipGetErrorString(e));
  return MMSEQ_OK;
}

// Upper bound of the split-K slab bytes any path of mmseq_gemm / mmseq_gemm_wgrad picks for this
// shape on the current device (less workspace only lowers the split count).
extern "C" int64_t mmseq_gemm_workspace_size(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int64_t cus = device_cus(), MN = (int64_t)M * N;
  int64_t best = 0;
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  int64_t s2 = t256 < cus ? cus / t256 : 1;
  if (s2 > K / 1024) s2 = K / 1024 > 0 ? K / 1024 : 1;
  if (s2 > 1) best = s2 * ((int64_t)((N + 255) / 256) * M + MN) * 4;  // + bias partials per column tile
  const int64_t tiles = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (tiles < 512) {
    int64_t s = (1024 + tiles - 1) / tiles;
    if (s > K / 1024) s = K / 1024;
    if (s > 1 && s * MN * 4 > best) best = s * MN * 4;
  }
  if (tiles < 128 && K >= 256) {
    int64_t s = (cus + tiles - 1) / tiles;
    if (s > K / 128) s = K / 128;
    if (s > 1 && s * MN * 4 > best) best = s * MN * 4;
  }
  return best;
}

// Weight gradient with the fused bias gradient (include/mmseq.h): C[M][N] += A^T B and
// bias_grad[m] += sum_k A[k][m]. bf16 operands with an eligible shape take the 256 x 256 TN
// kernel (column sums of the A fragments on the VALU beside the MFMAs); anything else runs
// mmseq_gemm plus a separate column-sum kernel.
extern "C" mmseq_status mmseq_gemm_wgrad(int M, int N, int K, const void* A, int64_t lda,
                                         const void* B, int64_t ldb, float* C, int64_t ldc,
                                         float* bias_grad, mmseq_dtype in_dtype, int variant,
                                         void* workspace, int64_t workspace_bytes,
                                         mmseq_stream stream) {
  MMSEQ_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_wgrad: bad sizes");
  MMSEQ_REQUIRE(A && B && C, "gemm_wgrad: null operand");
  MMSEQ_REQUIRE(lda >= M && ldb >= N && ldc >= N, "gemm_wgrad: ld too small");
  MMSEQ_REQUIRE(in_dtype == MMSEQ_F32 || in_dtype == MMSEQ_BF16, "gemm_wgrad: bad dtype");
  MMSEQ_REQUIRE(workspace_bytes >= 0 && (workspace || workspace_bytes == 0) &&
                    ((uintptr_t)workspace & 15) == 0,
                "gemm_wgrad: workspace must be 16-byte aligned (or NULL with 0 bytes)");
  GemmSel sel;
  MMSEQ_REQUIRE(make_sel(variant, &sel), "gemm_wgrad: bad variant %d", variant);
  if (M == 0 || N == 0 || K == 0) return MMSEQ_OK;
  float* const g_slab = reinterpret_cast<float*>(workspace);
  const int64_t g_slab_bytes = workspace ? workspace_bytes : 0;
  const int g_num_cu = sel.num_cu;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // the split-K reduction does f32x4 read-modify-writes on C: 16-byte aligned rows only
  const bool c_vec = ((uintptr_t)C & 15) == 0 && ldc % 4 == 0;
  // bias-free wgrads (convolution weights) take the same split-K TN kernel, without the fused
  // column sums
  if (in_dtype == MMSEQ_BF16 && sel.big && c_vec) {
    GemmArgs t = {};
    t.M = M; t.N = N; t.K = K;
    t.A = A; t.lda = lda; t.B = B; t.ldb = ldb; t.C = C; t.ldc = ldc;
    t.alpha = 1.f; t.accumulate = 1;
    t.drop = make_drop(nullptr);
    const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
    int S2 = t256 < g_num_cu ? g_num_cu / t256 : 1;
    if (S2 > K / 1024) S2 = K / 1024 > 0 ? K / 1024 : 1;
    const int tn256 = (N + 255) / 256;
    const int64_t cs_rows = bias_grad ? (int64_t)tn256 * M : 0;  // one partial row per column tile
    while (S2 > 1 && (!g_slab || (int64_t)S2 * (cs_rows + (int64_t)M * N) * 4 > g_slab_bytes)) --S2;
    t.splitk = S2;
    t.kchunk = ((K + S2 - 1) / S2 + 127) / 128 * 128;
    t.splitk = (K + t.kchunk - 1) / t.kchunk;
    if (t.splitk <= 1) { t.splitk = 1; t.kchunk = K; }
    t.slab = g_slab;
    t.cs = bias_grad;
    // the bias gradient's partials [split][column tile][M] (balanced over the column tiles, summed
    // in fixed order by cs_reduce); without workspace room the first column tile adds them directly
    const int64_t slab_c = t.splitk > 1 ? (int64_t)t.splitk * M * N : 0;
    t.cs_slab = bias_grad && g_slab &&
                        (slab_c + (int64_t)t.splitk * tn256 * M) * 4 <= g_slab_bytes
                    ? g_slab + slab_c : nullptr;
    hipError_t e2 = hipSuccess;
    if (mmseq_gemm256_tn(t, s, &e2)) {
      if (e2 == hipSuccess && t.splitk > 1) {
        const int64_t t4 = (int64_t)M * N / 4;
        const unsigned blocks = (unsigned)((t4 + 255) / 256 < 4096 ? (t4 + 255) / 256 : 4096);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, M, N, t.splitk,
                           g_slab, C, ldc, 1);
        e2 = hipGetLastError();
      }
      if (e2 == hipSuccess && t.cs_slab) {
        hipLaunchKernelGGL(cs_reduce_kernel, dim3((M + 31) / 32), dim3(256), 0, s, M,
                           t.splitk * tn256, t.cs_slab, bias_grad);
        e2 = hipGetLastError();
      }
      if (e2 != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "gemm_wgrad: %s", hipGetErrorString(e2));
      return MMSEQ_OK;
    }
  }
  mmseq_status st = mmseq_gemm(1, M, N, K, 1, A, lda, 0, B, ldb, 0, C, ldc, 0, nullptr, 0, nullptr,
                               nullptr, nullptr, 0, 0, 1.0f, 1, in_dtype, MMSEQ_F32, nullptr,
                               variant, workspace, workspace_bytes, stream);
  if (st || !bias_grad) return st;
  if (in_dtype == MMSEQ_BF16)
    hipLaunchKernelGGL(colsum_simple_kernel<unsigned short>, dim3((M + 255) / 256), dim3(256), 0, s,
                       M, K, (const unsigned short*)A, lda, bias_grad);
  else
    hipLaunchKernelGGL(colsum_simple_kernel<float>, dim3((M + 255) / 256), dim3(256), 0, s, M, K,
                       (const float*)A, lda, bias_grad);
  return mmseq_check_launch("gemm_wgrad colsum");
}
