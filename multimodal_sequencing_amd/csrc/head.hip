// BERSON head kernels (models/berson/modeling_bert.py, neural.py): span pooling of the pair
// encoder output, the pointer-network scoring + masked log-softmax + NLL, and the small
// multi-head attention of the inter-sentence encoder. All fp32 compute; no host loops, no
// device->host syncs (the reference does 2P .cpu() syncs + ~6P scalar index_put per step here).
#include "common.h"

namespace {

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  // 256 threads -> 4 waves
  v = is_max ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = is_max ? fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3])) : sh[0] + sh[1] + sh[2] + sh[3];
  return r;
}

// ---------------------------------------------------------------------------------------------
// pointer scoring (modeling_bert.py:1083-1142)
// ---------------------------------------------------------------------------------------------
constexpr int MAXN = 32;

__global__ __launch_bounds__(256) void pointer_fwd_kernel(int B, int N, int H,
                                                          const float* __restrict__ q,
                                                          const float* __restrict__ key,
                                                          const float* __restrict__ okey,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ wbias,
                                                          const uint8_t* __restrict__ pointed,
                                                          const int64_t* __restrict__ tgt_len,
                                                          const int64_t* __restrict__ target,
                                                          float* __restrict__ logp,
                                                          float* __restrict__ nll) {
  __shared__ float e[MAXN];
  const int b = blockIdx.x / N, t = blockIdx.x % N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* qr = q + ((int64_t)b * N + t) * H;
  const int L = (int)tgt_len[b];
  for (int j = wave; j < N; j += 4) {
    const float* kr = key + (((int64_t)b * N + t) * N + j) * H;
    const float* orow = okey + ((int64_t)b * N + j) * H;
    float s = 0.f;
    for (int h = lane; h < H; h += 64) s += w[h] * tanhf(qr[h] + kr[h] + orow[h]);
    s = wave_sum(s);
    if (lane == 0) {
      float v = s + (wbias ? wbias[0] : 0.f);
      if (pointed[((int64_t)b * N + t) * N + j] != 0 || j >= L) v = -1e9f;  // :1112-1113
      e[j] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float mx = -INFINITY;
    for (int j = 0; j < N; ++j) mx = fmaxf(mx, e[j]);
    float s = 0.f;
    for (int j = 0; j < N; ++j) s += expf(e[j] - mx);
    const float lse = mx + logf(s);
    for (int j = 0; j < N; ++j) logp[((int64_t)b * N + t) * N + j] = e[j] - lse;
    const int tg = (int)target[(int64_t)b * N + t];
    nll[(int64_t)b * N + t] = t < L ? -(e[tg] - lse) : 0.f;  // :1126-1135
  }
}

// One workgroup per story b, every sum in a fixed order (no float atomics: the backward is
// bit-stable run to run): dq / dkey per (t, j), dokey[b][j] summed over t, and the story's
// partials of dw (tanh_linear.weight) and dw_bias into ws[b][H + 1], which pointer_bwd_reduce
// sums over the stories in order.
__global__ __launch_bounds__(256) void pointer_bwd_kernel(int B, int N, int H,
                                                          const float* __restrict__ q,
                                                          const float* __restrict__ key,
                                                          const float* __restrict__ okey,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ logp,
                                                          const uint8_t* __restrict__ pointed,
                                                          const int64_t* __restrict__ tgt_len,
                                                          const int64_t* __restrict__ target,
                                                          const float* __restrict__ dnll,
                                                          float* __restrict__ dq,
                                                          float* __restrict__ dkey,
                                                          float* __restrict__ dokey,
                                                          float* __restrict__ ws) {
  __shared__ float de[MAXN * MAXN];
  const int b = blockIdx.x;
  const int L = (int)tgt_len[b];
  for (int e = threadIdx.x; e < N * N; e += 256) {
    const int t = e / N, j = e - t * N;
    const int64_t bt = (int64_t)b * N + t;
    const int tg = (int)target[bt];
    const float g = t < L ? dnll[bt] : 0.f;
    const float sm = expf(logp[bt * N + j]);
    // masked entries were overwritten with -1e9 (masked_fill_): no gradient flows through them
    const bool masked = pointed[bt * N + j] != 0 || j >= L;
    de[e] = masked ? 0.f : g * (sm - (j == tg ? 1.f : 0.f));
  }
  __syncthreads();
  float* wsb = ws + (int64_t)b * (H + 1);
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int e = 0; e < N * N; ++e) s += de[e];
    wsb[H] = s;
  }
  for (int h = threadIdx.x; h < H; h += 256) {
    const float wh = w[h];
    float dwh = 0.f;
    for (int j = 0; j < N; ++j) {
      const float okh = okey[((int64_t)b * N + j) * H + h];
      float dok = 0.f;
      for (int t = 0; t < N; ++t) {
        const int64_t bt = (int64_t)b * N + t;
        const int64_t kidx = (bt * N + j) * H + h;
        const float th = tanhf(q[bt * H + h] + key[kidx] + okh);
        const float dj = de[t * N + j];
        const float d = dj * wh * (1.f - th * th);
        dkey[kidx] = d;
        float* dqp = dq + bt * H + h;  // this thread's own element: summed over j in order
        *dqp = j == 0 ? d : *dqp + d;
        dok += d;
        dwh += dj * th;
      }
      dokey[((int64_t)b * N + j) * H + h] += dok;
    }
    wsb[h] = dwh;
  }
}

// dw[h] += sum_b ws[b][h], dw_bias += sum_b ws[b][H], stories in order
__global__ __launch_bounds__(256) void pointer_bwd_reduce(int B, int H, const float* __restrict__ ws,
                                                          float* __restrict__ dw,
                                                          float* __restrict__ dwb) {
  const int h = blockIdx.x * 256 + threadIdx.x;
  if (h > H) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += ws[(int64_t)b * (H + 1) + h];
  if (h < H) dw[h] += s;
  else dwb[0] += s;
}

// ---------------------------------------------------------------------------------------------
// HierarchicalAttention span pooling (modeling_bert.py:703-741)
// ---------------------------------------------------------------------------------------------
constexpr int MAXLT = 1024;

__device__ __forceinline__ bool in_span(int s, int t, int s0, int s1) {
  return s == 0 ? (t >= 1 && t <= s0) : (t > s0 && t <= s1);  // :711-712
}

template <typename T>
__global__ __launch_bounds__(256) void span_fwd_kernel(int P, int Lt, int H, const T* __restrict__ top,
                                                       int64_t ld_pair, const float* __restrict__ score,
                                                       const int64_t* __restrict__ sep,
                                                       float* __restrict__ probs,
                                                       float* __restrict__ mix, Drop drop) {
  __shared__ float pr[2][MAXLT];
  __shared__ float red[4];
  const int p = blockIdx.x;
  const int s0 = (int)sep[2 * p], s1 = (int)sep[2 * p + 1];
  for (int s = 0; s < 2; ++s) {
    float mx = -INFINITY;
    for (int t = threadIdx.x; t < Lt; t += 256) {
      // (1-m)*-10000 + m*score, exactly as :722-731
      float a = in_span(s, t, s0, s1) ? score[(int64_t)p * Lt + t] : -10000.0f;
      pr[s][t] = a;
      mx = fmaxf(mx, a);
    }
    mx = block_reduce(mx, red, true);
    float sum = 0.f;
    for (int t = threadIdx.x; t < Lt; t += 256) {
      float e = expf(pr[s][t] - mx);
      pr[s][t] = e;
      sum += e;
    }
    sum = block_reduce(sum, red, false);
    const float inv = 1.f / sum;
    for (int t = threadIdx.x; t < Lt; t += 256) {
      pr[s][t] *= inv;
      probs[((int64_t)p * 2 + s) * Lt + t] = pr[s][t];
      pr[s][t] *= drop_mul(drop, ((uint64_t)p * 2 + s) * Lt + t);  // :735 (after softmax)
    }
  }
  __syncthreads();
  const T* tp = top + (int64_t)p * ld_pair;
  for (int h = threadIdx.x; h < H; h += 256) {
    float a0 = 0.f, a1 = 0.f;
    for (int t = 0; t < Lt; ++t) {
      float v = Elem<T>::ld(tp + (int64_t)t * H + h);
      a0 += pr[0][t] * v;
      a1 += pr[1][t] * v;
    }
    mix[((int64_t)p * 2 + 0) * H + h] = a0;
    mix[((int64_t)p * 2 + 1) * H + h] = a1;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void span_bwd_kernel(int P, int Lt, int H, const T* __restrict__ top,
                                                       int64_t ld_pair, const float* __restrict__ probs,
                                                       const int64_t* __restrict__ sep,
                                                       const float* __restrict__ dmix,
                                                       float* __restrict__ dscore,
                                                       T* __restrict__ dtop, Drop drop) {
  __shared__ float dpr[2][MAXLT];
  __shared__ float red[4];
  const int p = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s0 = (int)sep[2 * p], s1 = (int)sep[2 * p + 1];
  const T* tp = top + (int64_t)p * ld_pair;
  const float* dm0 = dmix + ((int64_t)p * 2 + 0) * H;
  const float* dm1 = dmix + ((int64_t)p * 2 + 1) * H;
  for (int t = wave; t < Lt; t += 4) {
    float a0 = 0.f, a1 = 0.f;
    for (int h = lane; h < H; h += 64) {
      float v = Elem<T>::ld(tp + (int64_t)t * H + h);
      a0 += dm0[h] * v;
      a1 += dm1[h] * v;
    }
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    if (lane == 0) {  // gradient w.r.t. the undropped probabilities
      dpr[0][t] = a0 * drop_mul(drop, ((uint64_t)p * 2 + 0) * Lt + t);
      dpr[1][t] = a1 * drop_mul(drop, ((uint64_t)p * 2 + 1) * Lt + t);
    }
  }
  __syncthreads();
  const float* pr0 = probs + ((int64_t)p * 2 + 0) * Lt;
  const float* pr1 = probs + ((int64_t)p * 2 + 1) * Lt;
  float c0 = 0.f, c1 = 0.f;
  for (int t = threadIdx.x; t < Lt; t += 256) {
    c0 += pr0[t] * dpr[0][t];
    c1 += pr1[t] * dpr[1][t];
  }
  c0 = block_reduce(c0, red, false);
  c1 = block_reduce(c1, red, false);
  for (int t = threadIdx.x; t < Lt; t += 256) {
    float d = 0.f;
    if (in_span(0, t, s0, s1)) d += pr0[t] * (dpr[0][t] - c0);
    if (in_span(1, t, s0, s1)) d += pr1[t] * (dpr[1][t] - c1);
    dscore[(int64_t)p * Lt + t] = d;
  }
  T* dtp = dtop + (int64_t)p * ld_pair;
  for (int t = 0; t < Lt; ++t) {
    const float w0 = pr0[t] * drop_mul(drop, ((uint64_t)p * 2 + 0) * Lt + t);
    const float w1 = pr1[t] * drop_mul(drop, ((uint64_t)p * 2 + 1) * Lt + t);
    for (int h = threadIdx.x; h < H; h += 256) {
      T* d = dtp + (int64_t)t * H + h;
      Elem<T>::st(d, Elem<T>::ld(d) + w0 * dm0[h] + w1 * dm1[h]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// small MHA for the inter-sentence encoder (neural.py:98-235): one workgroup per (b, head)
// ---------------------------------------------------------------------------------------------
constexpr int SA_T = 64;

__global__ __launch_bounds__(256) void small_attn_fwd_kernel(int B, int T, int heads, int d,
                                                             const float* __restrict__ q,
                                                             const float* __restrict__ k,
                                                             const float* __restrict__ v,
                                                             const float* __restrict__ kbias,
                                                             float scale, float* __restrict__ out,
                                                             float* __restrict__ probs, Drop drop) {
  __shared__ float S[SA_T][SA_T + 1];
  const int b = blockIdx.x / heads, h = blockIdx.x % heads;
  const int D = heads * d;
  const float* qb = q + (int64_t)b * T * D + h * d;
  const float* kb = k + (int64_t)b * T * D + h * d;
  const float* vb = v + (int64_t)b * T * D + h * d;
  for (int e = threadIdx.x; e < T * T; e += 256) {
    int i = e / T, j = e % T;
    float s = 0.f;
    for (int c = 0; c < d; ++c) s += qb[(int64_t)i * D + c] * kb[(int64_t)j * D + c];
    // neural.py:208-213: query pre-scaled by 1/sqrt(d), mask added as (1-m)*-10000
    S[i][j] = s * scale + (kbias ? kbias[(int64_t)b * T + j] : 0.f);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < T; i += 256) {
    float mx = -INFINITY;
    for (int j = 0; j < T; ++j) mx = fmaxf(mx, S[i][j]);
    float sum = 0.f;
    for (int j = 0; j < T; ++j) {
      float e = expf(S[i][j] - mx);
      S[i][j] = e;
      sum += e;
    }
    float inv = 1.f / sum;
    for (int j = 0; j < T; ++j) {
      S[i][j] *= inv;
      const uint64_t idx = (((uint64_t)b * heads + h) * T + i) * T + j;
      probs[idx] = S[i][j];
      S[i][j] *= drop_mul(drop, idx);  // neural.py:228
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * d; e += 256) {
    int i = e / d, c = e % d;
    float s = 0.f;
    for (int j = 0; j < T; ++j) s += S[i][j] * vb[(int64_t)j * D + c];
    out[(int64_t)b * T * D + (int64_t)i * D + h * d + c] = s;
  }
}

__global__ __launch_bounds__(256) void small_attn_bwd_kernel(int B, int T, int heads, int d,
                                                             const float* __restrict__ q,
                                                             const float* __restrict__ k,
                                                             const float* __restrict__ v,
                                                             const float* __restrict__ probs,
                                                             const float* __restrict__ dout,
                                                             float scale, float* __restrict__ dq,
                                                             float* __restrict__ dk,
                                                             float* __restrict__ dv, Drop drop) {
  __shared__ float Pm[SA_T][SA_T + 1];
  __shared__ float Mk[SA_T][SA_T + 1];  // dropout multipliers
  __shared__ float dS[SA_T][SA_T + 1];
  const int b = blockIdx.x / heads, h = blockIdx.x % heads;
  const int D = heads * d;
  const int64_t off = (int64_t)b * T * D + h * d;
  for (int e = threadIdx.x; e < T * T; e += 256) {
    int i = e / T, j = e % T;
    const uint64_t idx = (((uint64_t)b * heads + h) * T + i) * T + j;
    Pm[i][j] = probs[idx];
    const float mk = drop_mul(drop, idx);
    Mk[i][j] = mk;
    float s = 0.f;
    for (int c = 0; c < d; ++c) s += dout[off + (int64_t)i * D + c] * v[off + (int64_t)j * D + c];
    dS[i][j] = s * mk;  // dP w.r.t. the undropped probabilities
  }
  __syncthreads();
  for (int i = threadIdx.x; i < T; i += 256) {
    float c = 0.f;
    for (int j = 0; j < T; ++j) c += Pm[i][j] * dS[i][j];
    for (int j = 0; j < T; ++j) dS[i][j] = Pm[i][j] * (dS[i][j] - c);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * d; e += 256) {
    int i = e / d, c = e % d;
    float aq = 0.f, ak = 0.f, av = 0.f;
    for (int j = 0; j < T; ++j) {
      aq += dS[i][j] * k[off + (int64_t)j * D + c];
      ak += dS[j][i] * q[off + (int64_t)j * D + c];
      av += Pm[j][i] * Mk[j][i] * dout[off + (int64_t)j * D + c];
    }
    dq[off + (int64_t)i * D + c] = aq * scale;
    dk[off + (int64_t)i * D + c] = ak * scale;
    dv[off + (int64_t)i * D + c] = av;
  }
}

}  // namespace


// ------------------------------------------------------------------------------------------------
// LSTM cell (modeling_bert.py:1027-1078 nn.LSTM decoder, gate order i, f, g, o), one thread per
// (row, unit): gates = gx + gh (both already include their biases); saves the four activations.
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(256) void lstm_fwd_kernel(int B, int H, const float* __restrict__ gx,
                                                       int64_t ldx, const float* __restrict__ gh,
                                                       const float* __restrict__ c,
                                                       float* __restrict__ h_out,
                                                       float* __restrict__ c_out,
                                                       float* __restrict__ act) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * H) return;
  const int b = (int)(idx / H), u = (int)(idx - (int64_t)b * H);
  const float* x = gx + b * ldx;
  const float* hh = gh + (int64_t)b * 4 * H;
  const float i = sigm(x[u] + hh[u]);
  const float f = sigm(x[H + u] + hh[H + u]);
  const float g = tanhf(x[2 * H + u] + hh[2 * H + u]);
  const float o = sigm(x[3 * H + u] + hh[3 * H + u]);
  const float c2 = f * c[idx] + i * g;
  c_out[idx] = c2;
  h_out[idx] = o * tanhf(c2);
  float* a = act + (int64_t)b * 4 * H;
  a[u] = i;
  a[H + u] = f;
  a[2 * H + u] = g;
  a[3 * H + u] = o;
}

// dh, dc_next (gradient flowing into c_out) -> dgates (pre-activation) and dc_prev
__global__ __launch_bounds__(256) void lstm_bwd_kernel(int B, int H, const float* __restrict__ act,
                                                       const float* __restrict__ c,
                                                       const float* __restrict__ c_out,
                                                       const float* __restrict__ dh,
                                                       const float* __restrict__ dc_next,
                                                       float* __restrict__ dgates,
                                                       float* __restrict__ dc_prev) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * H) return;
  const int b = (int)(idx / H), u = (int)(idx - (int64_t)b * H);
  const float* a = act + (int64_t)b * 4 * H;
  const float i = a[u], f = a[H + u], g = a[2 * H + u], o = a[3 * H + u];
  const float tc = tanhf(c_out[idx]);
  const float dhv = dh ? dh[idx] : 0.f;
  const float dc = (dc_next ? dc_next[idx] : 0.f) + dhv * o * (1.f - tc * tc);
  float* d = dgates + (int64_t)b * 4 * H;
  d[u] = dc * g * i * (1.f - i);
  d[H + u] = dc * c[idx] * f * (1.f - f);
  d[2 * H + u] = dc * i * (1.f - g * g);
  d[3 * H + u] = dhv * tc * o * (1.f - o);
  dc_prev[idx] = dc * f;
}

extern "C" mmseq_status mmseq_pointer_fwd(int B, int N, int H, const float* q, const float* key,
                                          const float* okey, const float* w, const float* w_bias,
                                          const uint8_t* pointed, const int64_t* tgt_len,
                                          const int64_t* target, float* logp, float* nll,
                                          mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && N > 0 && N <= MAXN && H > 0, "pointer: N must be in (0, %d]", MAXN);
  MMSEQ_REQUIRE(q && key && okey && w && pointed && tgt_len && target && logp && nll,
                "pointer_fwd: null buffer");
  if (!B) return MMSEQ_OK;
  hipLaunchKernelGGL(pointer_fwd_kernel, dim3(B * N), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), B, N, H, q, key, okey, w, w_bias,
                     pointed, tgt_len, target, logp, nll);
  return mmseq_check_launch("pointer_fwd");
}

extern "C" int64_t mmseq_pointer_bwd_workspace(int B, int N, int H) {
  (void)N;
  return (int64_t)B * (H + 1);
}

extern "C" mmseq_status mmseq_pointer_bwd(int B, int N, int H, const float* q, const float* key,
                                          const float* okey, const float* w, const float* logp,
                                          const uint8_t* pointed, const int64_t* tgt_len, const int64_t* target,
                                          const float* dnll, float* dq, float* dkey, float* dokey,
                                          float* dw, float* dw_bias, float* workspace,
                                          mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && N > 0 && N <= MAXN && H > 0, "pointer_bwd: bad sizes");
  MMSEQ_REQUIRE(q && key && okey && w && logp && pointed && tgt_len && target && dnll && dq &&
                    dkey && dokey && dw && dw_bias && workspace,
                "pointer_bwd: null buffer");
  if (!B) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(pointer_bwd_kernel, dim3(B), dim3(256), 0, s, B, N, H, q, key, okey, w, logp,
                     pointed, tgt_len, target, dnll, dq, dkey, dokey, workspace);
  hipLaunchKernelGGL(pointer_bwd_reduce, dim3((H + 1 + 255) / 256), dim3(256), 0, s, B, H, workspace,
                     dw, dw_bias);
  return mmseq_check_launch("pointer_bwd");
}

extern "C" mmseq_status mmseq_span_pool_fwd(int P, int Lt, int H, const void* top,
                                            int64_t ld_pair, const float* score,
                                            const int64_t* sep, float* probs, float* mix,
                                            mmseq_dtype dt, const mmseq_dropout* drop,
                                            mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && Lt > 0 && Lt <= MAXLT && H > 0, "span_pool: Lt must be <= %d", MAXLT);
  MMSEQ_REQUIRE(top && score && sep && probs && mix, "span_pool_fwd: null buffer");
  if (!P) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dt == MMSEQ_F32)
    hipLaunchKernelGGL(span_fwd_kernel<float>, dim3(P), dim3(256), 0, s, P, Lt, H,
                       (const float*)top, ld_pair, score, sep, probs, mix, make_drop(drop));
  else
    hipLaunchKernelGGL(span_fwd_kernel<unsigned short>, dim3(P), dim3(256), 0, s, P, Lt, H,
                       (const unsigned short*)top, ld_pair, score, sep, probs, mix,
                       make_drop(drop));
  return mmseq_check_launch("span_pool_fwd");
}

extern "C" mmseq_status mmseq_span_pool_bwd(int P, int Lt, int H, const void* top,
                                            int64_t ld_pair, const float* probs,
                                            const int64_t* sep, const float* dmix, float* dscore,
                                            void* dtop, mmseq_dtype dt, const mmseq_dropout* drop,
                                            mmseq_stream stream) {
  MMSEQ_REQUIRE(P >= 0 && Lt > 0 && Lt <= MAXLT && H > 0, "span_pool_bwd: bad sizes");
  MMSEQ_REQUIRE(top && probs && sep && dmix && dscore && dtop, "span_pool_bwd: null buffer");
  if (!P) return MMSEQ_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dt == MMSEQ_F32)
    hipLaunchKernelGGL(span_bwd_kernel<float>, dim3(P), dim3(256), 0, s, P, Lt, H,
                       (const float*)top, ld_pair, probs, sep, dmix, dscore, (float*)dtop,
                       make_drop(drop));
  else
    hipLaunchKernelGGL(span_bwd_kernel<unsigned short>, dim3(P), dim3(256), 0, s, P, Lt, H,
                       (const unsigned short*)top, ld_pair, probs, sep, dmix, dscore,
                       (unsigned short*)dtop, make_drop(drop));
  return mmseq_check_launch("span_pool_bwd");
}

extern "C" mmseq_status mmseq_small_attn_fwd(int B, int T, int heads, int d, const float* q,
                                             const float* k, const float* v,
                                             const float* key_bias, float scale, float* out,
                                             float* probs, const mmseq_dropout* drop,
                                             mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && T > 0 && T <= SA_T && heads > 0 && d > 0, "small_attn: T must be <= %d",
                SA_T);
  MMSEQ_REQUIRE(q && k && v && out && probs, "small_attn_fwd: null buffer");
  if (!B) return MMSEQ_OK;
  hipLaunchKernelGGL(small_attn_fwd_kernel, dim3(B * heads), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), B, T, heads, d, q, k, v, key_bias,
                     scale, out, probs, make_drop(drop));
  return mmseq_check_launch("small_attn_fwd");
}

extern "C" mmseq_status mmseq_small_attn_bwd(int B, int T, int heads, int d, const float* q,
                                             const float* k, const float* v, const float* probs,
                                             const float* dout, float scale, float* dq, float* dk,
                                             float* dv, const mmseq_dropout* drop,
                                             mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && T > 0 && T <= SA_T && heads > 0 && d > 0, "small_attn_bwd: bad sizes");
  MMSEQ_REQUIRE(q && k && v && probs && dout && dq && dk && dv, "small_attn_bwd: null buffer");
  if (!B) return MMSEQ_OK;
  hipLaunchKernelGGL(small_attn_bwd_kernel, dim3(B * heads), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), B, T, heads, d, q, k, v, probs, dout,
                     scale, dq, dk, dv, make_drop(drop));
  return mmseq_check_launch("small_attn_bwd");
}

extern "C" mmseq_status mmseq_lstm_cell_fwd(int B, int H, const float* gx, int64_t ld_gx,
                                            const float* gh, const float* c, float* h_out,
                                            float* c_out, float* act, mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && H > 0 && ld_gx >= 4 * (int64_t)H, "lstm_cell_fwd: bad sizes");
  MMSEQ_REQUIRE(gx && gh && c && h_out && c_out && act, "lstm_cell_fwd: null buffer");
  if (B == 0) return MMSEQ_OK;
  const int64_t n = (int64_t)B * H;
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), B, H, gx, ld_gx, gh, c, h_out, c_out,
                     act);
  return mmseq_check_launch("lstm_cell_fwd");
}

extern "C" mmseq_status mmseq_lstm_cell_bwd(int B, int H, const float* act, const float* c,
                                            const float* c_out, const float* dh,
                                            const float* dc_next, float* dgates, float* dc_prev,
                                            mmseq_stream stream) {
  MMSEQ_REQUIRE(B >= 0 && H > 0, "lstm_cell_bwd: bad sizes");
  MMSEQ_REQUIRE(act && c && c_out && dgates && dc_prev, "lstm_cell_bwd: null buffer");
  if (B == 0) return MMSEQ_OK;
  const int64_t n = (int64_t)B * H;
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), B, H, act, c, c_out, dh, dc_next,
                     dgates, dc_prev);
  return mmseq_check_launch("lstm_cell_bwd");
}
