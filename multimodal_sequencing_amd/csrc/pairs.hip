// BERSON pair expansion on device (models/berson/process_inputs_for_berson.py:13-368; SURVEY §8f
// row 2): a story row of <s> ... </s> steps becomes N(N-1) ordered pair rows
// <s> step_a </s> <s> step_c </s> padded with pad_id to the batch's longest pair, plus the pair
// mask (padded with pad_id too: quirk C.7), token types, </s> positions and pairwise labels.
//
// Integer / byte work, HBM- and latency-bound (a few MB per step): no MFMA, one wave per story for
// the scan, coalesced int64 row writes for the expansion.
#include "common.h"

namespace {

constexpr int kMaxSteps = 64;  // N <= 64 (one wave holds a story's steps)

// ordered pair j of pairs_generator(N) (:246-261): combinations (a < c) in lexicographic order,
// then the same list reversed element-wise
__device__ __forceinline__ void pair_of(int j, int N, int& a, int& c) {
  const int half = N * (N - 1) / 2;
  int r = j < half ? j : j - half;
  int x = 0;
  while (r >= N - 1 - x) {
    r -= N - 1 - x;
    ++x;
  }
  const int y = x + 1 + r;
  if (j < half) { a = x; c = y; } else { a = y; c = x; }
}

// One wave per story: step boundaries by ballot over 64-token chunks, the stable argsort of the
// gold order, per-pair lengths / </s> positions / pairwise labels, and the batch max pair length.
// status[0] = max pair length (atomicMax), status[1] = malformed story count.
__global__ void __launch_bounds__(64) pair_scan_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ labels, int L, int N,
    int64_t cls_id, int64_t sep_id, int64_t* __restrict__ starts, int64_t* __restrict__ lens,
    int64_t* __restrict__ plab, int64_t* __restrict__ sep_pos, int* __restrict__ status) {
  __shared__ int s_start[kMaxSteps], s_end[kMaxSteps], s_rank[kMaxSteps];
  __shared__ int64_t s_lab[kMaxSteps];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int64_t* row = ids + (int64_t)b * L;
  const uint64_t below = (1ull << lane) - 1ull;
  int ns = 0, ne = 0;
  for (int base = 0; base < L; base += 64) {
    const int i = base + lane;
    const int64_t v = i < L ? row[i] : 0;
    const bool isc = i < L && v == cls_id, iss = i < L && v == sep_id;
    const uint64_t mc = __ballot(isc), ms = __ballot(iss);
    if (isc) {
      const int k = ns + __popcll(mc & below);
      if (k < N) s_start[k] = i;
    }
    if (iss) {
      const int k = ne + __popcll(ms & below);
      if (k < N) s_end[k] = i;
    }
    ns += __popcll(mc);
    ne += __popcll(ms);
  }
  if (lane < N) s_lab[lane] = labels[(int64_t)b * N + lane];
  __syncthreads();
  bool bad = ns != N || ne != N;
  if (!bad && lane < N) bad = s_end[lane] < s_start[lane];
  if (__ballot(bad) != 0ull) {  // parse_input_ids (:100-110) would not yield N steps
    if (lane == 0) atomicAdd(&status[1], 1);
    return;
  }
  if (lane < N) {
    starts[(int64_t)b * N + lane] = s_start[lane];
    lens[(int64_t)b * N + lane] = s_end[lane] - s_start[lane] + 1;
    // stable argsort: the sorted position of element `lane`, rank[position] = lane
    const int64_t me = s_lab[lane];
    int pos = 0;
    for (int j = 0; j < N; ++j) pos += (s_lab[j] < me) || (s_lab[j] == me && j < lane);
    s_rank[pos] = lane;
  }
  __syncthreads();
  const int npair = N * (N - 1);
  int best = 0;
  for (int j = lane; j < npair; j += 64) {
    int a, c;
    pair_of(j, N, a, c);
    const int l1 = s_end[a] - s_start[a] + 1, l2 = s_end[c] - s_start[c] + 1;
    const int64_t o = (int64_t)b * npair + j;
    sep_pos[2 * o] = l1 - 1;
    sep_pos[2 * o + 1] = l1 + l2 - 1;
    plab[o] = s_rank[a] < s_rank[c] ? 1 : 0;  // :162-174
    best = max(best, l1 + l2);
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) best = max(best, __shfl_xor(best, s, 64));
  if (lane == 0) atomicMax(&status[0], best);
}

// One workgroup per pair row: <s> a </s> <s> c </s> then pad_id; mask 1 / pad_id; token type 0,
// or 1 on the second step when cls_id != 0 (BERT-style ids).
__global__ void __launch_bounds__(256) pair_expand_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ starts,
    const int64_t* __restrict__ lens, int L, int N, int Lp, int64_t pad_id, int second_type,
    int64_t* __restrict__ out_ids, int64_t* __restrict__ out_mask, int64_t* __restrict__ out_tt) {
  const int npair = N * (N - 1);
  const int r = blockIdx.x;
  const int b = r / npair, j = r - b * npair;
  int a, c;
  pair_of(j, N, a, c);
  const int64_t s1 = starts[(int64_t)b * N + a], l1 = lens[(int64_t)b * N + a];
  const int64_t s2 = starts[(int64_t)b * N + c], l2 = lens[(int64_t)b * N + c];
  const int64_t* row = ids + (int64_t)b * L;
  const int64_t o = (int64_t)r * Lp;
  for (int t = threadIdx.x; t < Lp; t += blockDim.x) {
    const bool in1 = t < l1, in2 = !in1 && t < l1 + l2;
    int64_t src = in1 ? s1 + t : (in2 ? s2 + (t - l1) : 0);
    src = src < 0 ? 0 : (src >= L ? L - 1 : src);
    const bool valid = in1 || in2;
    out_ids[o + t] = valid ? row[src] : pad_id;
    out_mask[o + t] = valid ? 1 : pad_id;
    out_tt[o + t] = (second_type && in2) ? 1 : 0;
  }
}

}  // namespace

extern "C" mmseq_status mmseq_pair_scan(int B, int L, int N, const int64_t* input_ids,
                                        const int64_t* labels, int64_t cls_id, int64_t sep_id,
                                        int64_t* starts, int64_t* lens, int64_t* pairwise_labels,
                                        int64_t* sep_positions, int32_t* status,
                                        mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && L > 0 && N >= 2 && N <= kMaxSteps, "pair_scan: bad sizes");
  MMSEQ_REQUIRE(input_ids && labels && starts && lens && pairwise_labels && sep_positions && status,
                "pair_scan: null buffer");
  if (B == 0) return MMSEQ_OK;
  hipLaunchKernelGGL(pair_scan_kernel, dim3(B), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     input_ids, labels, L, N, cls_id, sep_id, starts, lens, pairwise_labels,
                     sep_positions, (int*)status);
  return mmseq_check_launch("pair_scan");
}

extern "C" mmseq_status mmseq_pair_expand(int B, int L, int N, int Lp, const int64_t* input_ids,
                                          const int64_t* starts, const int64_t* lens,
                                          int64_t pad_id, int second_type, int64_t* out_ids,
                                          int64_t* out_mask, int64_t* out_token_type,
                                          mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && L > 0 && N >= 2 && N <= kMaxSteps && Lp > 0 && Lp <= L,
                "pair_expand: bad sizes");
  MMSEQ_REQUIRE(input_ids && starts && lens && out_ids && out_mask && out_token_type,
                "pair_expand: null buffer");
  if (B == 0) return MMSEQ_OK;
  const int64_t rows = (int64_t)B * N * (N - 1);
  MMSEQ_REQUIRE(rows < (1ll << 31), "pair_expand: too many pairs");
  const int threads = Lp >= 256 ? 256 : (Lp >= 128 ? 128 : 64);
  hipLaunchKernelGGL(pair_expand_kernel, dim3((unsigned)rows), dim3(threads), 0,
                     reinterpret_cast<hipStream_t>(stream), input_ids, starts, lens, L, N, Lp,
                     pad_id, second_type, out_ids, out_mask, out_token_type);
  return mmseq_check_launch("pair_expand");
}
