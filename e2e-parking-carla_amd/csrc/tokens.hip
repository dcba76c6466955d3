// Token assembly of the two transformer stacks, fused with the positional embedding and the
// positional dropout, forward and backward:
//
//  * fusion encoder (reference model/feature_fusion.py:40-46): the BEV encoder output
//    (B, C, S) transposed to tokens, the motion MLP output (B, S) broadcast into the last
//    E - C token channels (expand + torch.cat), + pos_embed (S, E), then pos_drop:
//      t[b][s][e] = drop((e < C ? bev[b][e][s] : motion[b][s]) + pos[s][e])
//    PyTorch runs transpose copy, expand, cat, broadcast add and dropout (RNG fill + mask) as
//    separate launches, and the backward as narrow / sum-over-batch / mask launches.
//  * control decoder (reference model/control_predict.py:14-15,49-54): the token embedding
//    lookup + pos_embed (T, E), then pos_drop:
//      o[b][t][e] = drop(table[tok[b][t]][e] + pos[t][e])
//    backward: dtable[v] = sum over (b, t) with tok == v in (b, t) order, dpos[t] = sum over b
//    in b order (fixed order: deterministic, no atomics).
//
// Dropout: keep(i) = att_keep(seed, i) for the output element index i (dropout.h), scaled by
// 1 / (1 - p); p = 0 is the identity (eval, and the deterministic-train protocol).
#include "common.h"
#include "dropout.h"

namespace e2ep {

constexpr int TT = 32;  // transpose tile

__device__ __forceinline__ float tok_drop(float v, float p, uint32_t sm, uint32_t i, float sc) {
  return p > 0.f ? (att_keep(sm, i, p) ? v * sc : 0.f) : v;
}

// grid (ceil(E/32), ceil(S/32), B), block 32 x 8
__global__ void __launch_bounds__(256) k_fusion_tokens_fwd(
    const float *__restrict__ bev, const float *__restrict__ motion, const float *__restrict__ pos,
    int C, int S, int E, float p, const int *__restrict__ seed, float *__restrict__ out) {
  __shared__ float tile[TT][TT + 1];  // [e][s]
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int e0 = blockIdx.x * TT, s0 = blockIdx.y * TT, b = blockIdx.z;
  const int s = s0 + tx;
#pragma unroll
  for (int i = 0; i < TT / 8; ++i) {
    const int e = e0 + ty + 8 * i;
    float v = 0.f;
    if (s < S && e < E) v = e < C ? bev[((size_t)b * C + e) * S + s] : motion[(size_t)b * S + s];
    tile[ty + 8 * i][tx] = v;
  }
  __syncthreads();
  const uint32_t sm = att_seedmix(seed);
  const float sc = 1.f / (1.f - p);
  const int e = e0 + tx;
#pragma unroll
  for (int i = 0; i < TT / 8; ++i) {
    const int ss = s0 + ty + 8 * i;
    if (ss >= S || e >= E) continue;
    const size_t o = ((size_t)b * S + ss) * E + e;
    out[o] = tok_drop(tile[tx][ty + 8 * i] + pos[(size_t)ss * E + e], p, sm, (uint32_t)o, sc);
  }
}

// grid (ceil(E/32), ceil(S/32)), block 32 x 8; the block walks b in order (dpos = sum over b)
__global__ void __launch_bounds__(256) k_fusion_tokens_bwd(
    const float *__restrict__ g, int B, int C, int S, int E, float p, const int *__restrict__ seed,
    float *__restrict__ dbev, float *__restrict__ dmotion, float *__restrict__ dpos) {
  __shared__ float tile[TT][TT + 1];  // [s][e]
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int e0 = blockIdx.x * TT, s0 = blockIdx.y * TT;
  const uint32_t sm = att_seedmix(seed);
  const float sc = 1.f / (1.f - p);
  const int e = e0 + tx;
  float dp[TT / 8] = {0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
#pragma unroll
    for (int i = 0; i < TT / 8; ++i) {
      const int s = s0 + ty + 8 * i;
      float v = 0.f;
      if (s < S && e < E) {
        const size_t o = ((size_t)b * S + s) * E + e;
        v = tok_drop(g[o], p, sm, (uint32_t)o, sc);  // d(pre-dropout sum)
      }
      dp[i] += v;
      tile[ty + 8 * i][tx] = v;
    }
    __syncthreads();
    // dbev[b][e][s] (e < C): transposed write, coalesced along s
    const int s = s0 + tx;
#pragma unroll
    for (int i = 0; i < TT / 8; ++i) {
      const int ee = e0 + ty + 8 * i;
      if (s < S && ee < C) dbev[((size_t)b * C + ee) * S + s] = tile[tx][ty + 8 * i];
    }
    // dmotion[b][s] = sum of the token channels C .. E-1 in order (the broadcast columns)
    if (e0 <= C && C < e0 + TT && ty == 0 && s < S) {
      float m = 0.f;
      for (int ee = C; ee < E && ee < e0 + TT; ++ee) m += tile[tx][ee - e0];
      dmotion[(size_t)b * S + s] = m;
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TT / 8; ++i) {
    const int s = s0 + ty + 8 * i;
    if (s < S && e < E) dpos[(size_t)s * E + e] = dp[i];
  }
}

// grid (B*T), block 256
__global__ void __launch_bounds__(256) k_embed_tokens_fwd(
    const int64_t *__restrict__ tok, int tok_stride, const float *__restrict__ table, int V,
    const float *__restrict__ pos, int T, int E, float p, const int *__restrict__ seed,
    float *__restrict__ out) {
  const int bt = blockIdx.x, b = bt / T, t = bt - b * T;
  int64_t v = tok[(size_t)b * tok_stride + t];
  v = v < 0 ? 0 : (v >= V ? V - 1 : v);  // never read out of the table
  const uint32_t sm = att_seedmix(seed);
  const float sc = 1.f / (1.f - p);
  for (int e = threadIdx.x; e < E; e += 256) {
    const size_t o = (size_t)bt * E + e;
    out[o] = tok_drop(table[(size_t)v * E + e] + pos[(size_t)t * E + e], p, sm, (uint32_t)o, sc);
  }
}

// grid (V + T), block 256: blocks < V write dtable row v, the rest dpos row t
__global__ void __launch_bounds__(256) k_embed_tokens_bwd(
    const float *__restrict__ g, const int64_t *__restrict__ tok, int tok_stride, int V, int B,
    int T, int E, float p, const int *__restrict__ seed, float *__restrict__ dtable,
    float *__restrict__ dpos) {
  __shared__ int64_t st[1024];
  const int n = B * T;
  const uint32_t sm = att_seedmix(seed);
  const float sc = 1.f / (1.f - p);
  if ((int)blockIdx.x < V) {
    const int v = blockIdx.x;
    for (int i = threadIdx.x; i < n && i < 1024; i += 256) {
      const int64_t x = tok[(size_t)(i / T) * tok_stride + i % T];
      st[i] = x < 0 ? 0 : (x >= V ? V - 1 : x);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 256) {
      float acc = 0.f;
      for (int i = 0; i < n; ++i) {
        int64_t x = i < 1024 ? st[i] : tok[(size_t)(i / T) * tok_stride + i % T];
        x = x < 0 ? 0 : (x >= V ? V - 1 : x);
        if (x == v) {
          const size_t o = (size_t)i * E + e;
          acc += tok_drop(g[o], p, sm, (uint32_t)o, sc);
        }
      }
      dtable[(size_t)v * E + e] = acc;
    }
    return;
  }
  const int t = blockIdx.x - V;
  for (int e = threadIdx.x; e < E; e += 256) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) {
      const size_t o = ((size_t)b * T + t) * E + e;
      acc += tok_drop(g[o], p, sm, (uint32_t)o, sc);
    }
    dpos[(size_t)t * E + e] = acc;
  }
}

// Autoregressive decode step (reference model/control_predict.py:70-75): softmax of one
// logits row, argmax of the probabilities (torch.argmax: the first index of the largest
// value), the token written into column `pos` of the persistent sequence.  Block per row; the
// max and the sum reduce in a fixed order (deterministic).
__global__ void __launch_bounds__(256) k_token_argmax_append(const float *__restrict__ logits,
                                                             long long rstride, int V,
                                                             int64_t *__restrict__ seq,
                                                             int seq_stride, int pos) {
  __shared__ float sf[4];
  __shared__ int si[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float *row = logits + (size_t)b * rstride;
  float m = -INFINITY;
  for (int v = tid; v < V; v += 256) m = fmaxf(m, row[v]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) sf[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(sf[0], sf[1]), fmaxf(sf[2], sf[3]));
  __syncthreads();
  float s = 0.f;
  for (int v = tid; v < V; v += 256) s += expf(row[v] - m);
  s = wave_sum(s);
  if (lane == 0) sf[wv] = s;
  __syncthreads();
  s = (sf[0] + sf[1]) + (sf[2] + sf[3]);
  __syncthreads();
  float best = -1.f;
  int bi = 0x7fffffff;
  for (int v = tid; v < V; v += 256) {
    const float p = expf(row[v] - m) / s;
    if (p > best) {  // v ascends per thread: the first index of a tie is kept
      best = p;
      bi = v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) {
    sf[wv] = best;
    si[wv] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (sf[w] > best || (sf[w] == best && si[w] < bi)) {
        best = sf[w];
        bi = si[w];
      }
    seq[(size_t)b * seq_stride + pos] = bi;
  }
}

// seq[b][t] = t < L ? prefix[b][t] : pad   (grid B, block 64)
__global__ void k_tokens_init(const int64_t *__restrict__ prefix, int pstride, int L,
                              int64_t *__restrict__ seq, int T, int64_t pad) {
  const int b = blockIdx.x;
  for (int t = threadIdx.x; t < T; t += blockDim.x)
    seq[(size_t)b * T + t] = t < L ? prefix[(size_t)b * pstride + t] : pad;
}

static int tok_check(float p, const int32_t *seed, long long n, const char *who) {
  E2EP_REQUIRE(p >= 0.f && p < 1.f && (p == 0.f || seed), E2EP_EINVAL, "%s: bad dropout p / seed", who);
  E2EP_REQUIRE(n > 0 && n < 0xffffffffLL, E2EP_ERANGE, "%s: %lld elements (need 1 .. 2^32)", who, n);
  return 0;
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_fusion_tokens_fwd(const float *bev, const float *motion, const float *pos, int B, int C,
                           int S, int E, float p, const int32_t *seed, float *tokens,
                           void *stream) {
  E2EP_REQUIRE(bev && motion && pos && tokens && B > 0 && C > 0 && S > 0 && E >= C && B <= 65535,
               E2EP_EINVAL, "e2ep_fusion_tokens_fwd: bad arguments");
  if (int rc = tok_check(p, seed, (long long)B * S * E, "e2ep_fusion_tokens_fwd")) return rc;
  hipLaunchKernelGGL(k_fusion_tokens_fwd, dim3(cdiv(E, TT), cdiv(S, TT), B), dim3(256), 0,
                     as_stream(stream), bev, motion, pos, C, S, E, p, seed, tokens);
  return launch_status("e2ep_fusion_tokens_fwd");
}

int e2ep_fusion_tokens_bwd(const float *dtokens, int B, int C, int S, int E, float p,
                           const int32_t *seed, float *dbev, float *dmotion, float *dpos,
                           void *stream) {
  E2EP_REQUIRE(dtokens && dbev && dmotion && dpos && B > 0 && C > 0 && S > 0 && E > C &&
                   C % TT + (E - C) <= TT,
               E2EP_EINVAL, "e2ep_fusion_tokens_bwd: bad arguments (the E - C broadcast "
               "channels must lie in one 32-channel tile)");
  if (int rc = tok_check(p, seed, (long long)B * S * E, "e2ep_fusion_tokens_bwd")) return rc;
  hipLaunchKernelGGL(k_fusion_tokens_bwd, dim3(cdiv(E, TT), cdiv(S, TT)), dim3(256), 0,
                     as_stream(stream), dtokens, B, C, S, E, p, seed, dbev, dmotion, dpos);
  return launch_status("e2ep_fusion_tokens_bwd");
}

int e2ep_embed_tokens_fwd(const int64_t *tok, int tok_stride, const float *table, int V,
                          const float *pos, int B, int T, int E, float p, const int32_t *seed,
                          float *out, void *stream) {
  E2EP_REQUIRE(tok && table && pos && out && V > 0 && B > 0 && T > 0 && E > 0 && tok_stride >= T,
               E2EP_EINVAL, "e2ep_embed_tokens_fwd: bad arguments");
  if (int rc = tok_check(p, seed, (long long)B * T * E, "e2ep_embed_tokens_fwd")) return rc;
  hipLaunchKernelGGL(k_embed_tokens_fwd, dim3(B * T), dim3(256), 0, as_stream(stream), tok,
                     tok_stride, table, V, pos, T, E, p, seed, out);
  return launch_status("e2ep_embed_tokens_fwd");
}

int e2ep_tokens_init(const int64_t *prefix, int prefix_stride, int B, int L, int64_t *seq, int T,
                     int64_t pad, void *stream) {
  E2EP_REQUIRE(prefix && seq && B > 0 && L > 0 && T >= L && prefix_stride >= L, E2EP_EINVAL,
               "e2ep_tokens_init: bad arguments");
  hipLaunchKernelGGL(k_tokens_init, dim3(B), dim3(64), 0, as_stream(stream), prefix, prefix_stride,
                     L, seq, T, pad);
  return launch_status("e2ep_tokens_init");
}

int e2ep_token_argmax_append(const float *logits, long long row_stride, int B, int V,
                             int64_t *seq, int seq_stride, int pos, void *stream) {
  E2EP_REQUIRE(logits && seq && B > 0 && V > 0 && row_stride >= V && pos >= 0 &&
                   pos < seq_stride,
               E2EP_EINVAL, "e2ep_token_argmax_append: bad arguments");
  hipLaunchKernelGGL(k_token_argmax_append, dim3(B), dim3(256), 0, as_stream(stream), logits,
                     row_stride, V, seq, seq_stride, pos);
  return launch_status("e2ep_token_argmax_append");
}

int e2ep_embed_tokens_bwd(const float *dout, const int64_t *tok, int tok_stride, int V, int B,
                          int T, int E, float p, const int32_t *seed, float *dtable, float *dpos,
                          void *stream) {
  E2EP_REQUIRE(dout && tok && dtable && dpos && V > 0 && B > 0 && T > 0 && E > 0 && tok_stride >= T,
               E2EP_EINVAL, "e2ep_embed_tokens_bwd: bad arguments");
  if (int rc = tok_check(p, seed, (long long)B * T * E, "e2ep_embed_tokens_bwd")) return rc;
  hipLaunchKernelGGL(k_embed_tokens_bwd, dim3(V + T), dim3(256), 0, as_stream(stream), dout, tok,
                     tok_stride, V, B, T, E, p, seed, dtable, dpos);
  return launch_status("e2ep_embed_tokens_bwd");
}

}  // extern "C"
