// Squeeze-and-excitation of efficientnet-pytorch's MBConv as one fused op, NCHW fp32, gfx950
// (reference: efficientnet-pytorch 0.7.1 MBConvBlock, used through model/cam_encoder.py:69-73):
//   pooled = mean_hw(x);  h = swish(W1 pooled + b1);  a = W2 h + b2;  y = x * sigmoid(a)
// Forward: squeeze (wave per plane), the MLP on the 1x1 map as two small kernels (hidden
// units, wave per output; logits, LDS-staged W2 tile), excite (float4 stream).  Backward: da
// (wave per plane), MLP backward (dh partials over channel spans, then dhpre + dpooled), one
// weight-gradient kernel (sums over the batch in fixed order), and
// dx = dy * sigmoid(a) + dpooled / HW in a single stream — no separate avg-pool backward and
// no autograd add of the two input-gradient paths.
#include "common.h"
#include "handoff.h"

namespace e2ep {

constexpr int SE_MAXC = 4096, SE_MAXSQ = 256;
// float4 loads in flight per lane in the per-plane reductions (squeeze, da)
constexpr int SE_U = 4;

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + expf(-v)); }

// Optional input transform: when the SE input is the raw output of the depthwise conv, the
// block's _bn1 + swish is applied on load, x -> swish(x * sc[c] + sh[c]) (sc / sh from
// e2ep_bn_stats), so the activation tensor is never written.
struct SeIn {
  const float *sc, *sh;
  int C;
};
__device__ __forceinline__ float se_in(float v, float sc, float sh, bool t) {
  if (!t) return v;
  const float z = v * sc + sh;
  return z / (1.f + expf(-z));
}
__device__ __forceinline__ float4 se_in4(float4 v, float sc, float sh, bool t) {
  return make_float4(se_in(v.x, sc, sh, t), se_in(v.y, sc, sh, t), se_in(v.z, sc, sh, t),
                     se_in(v.w, sc, sh, t));
}

// sum over one plane (HW floats, float4 when HW % 4 == 0) by one wave
__device__ __forceinline__ float plane_sum(const float *__restrict__ p, int HW, int lane,
                                           float sc, float sh, bool t) {
  float s = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2;
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    // SE_U loads in flight per lane (clamped, unconditional); the lane still sums i, i + 64,
    // ... in ascending order
    for (int i0 = lane; i0 < HW4; i0 += 64 * SE_U) {
      float4 v[SE_U];
#pragma unroll
      for (int u = 0; u < SE_U; ++u) v[u] = p4[min(i0 + u * 64, HW4 - 1)];
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        if (i0 + u * 64 >= HW4) break;
        const float4 w = se_in4(v[u], sc, sh, t);
        s += (w.x + w.y) + (w.z + w.w);
      }
    }
  } else {
    for (int i = lane; i < HW; i += 64) s += se_in(p[i], sc, sh, t);
  }
  return wave_sum(s);
}

__global__ void __launch_bounds__(256) k_se_squeeze(const float *__restrict__ x, SeIn tf,
                                                    int planes, int HW,
                                                    float *__restrict__ pooled) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pl >= planes) return;
  const bool t = tf.sc != nullptr;
  const int c = pl % tf.C;
  const float s = plane_sum(x + (size_t)pl * HW, HW, threadIdx.x & 63, t ? tf.sc[c] : 1.f,
                            t ? tf.sh[c] : 0.f, t);
  if ((threadIdx.x & 63) == 0) pooled[pl] = s / (float)HW;
}

// hpre[n][k] = W1[k] . pooled[n] + b1[k]  (W1 [sq][C]): one wave per (n, k), lanes along
// the W1 row and pooled[n] (coalesced), fixed-order wave reduction.  grid (N, sq / 4).
__global__ void __launch_bounds__(256) k_se_hidden(const float *__restrict__ pooled,
                                                   const float *__restrict__ w1,
                                                   const float *__restrict__ b1, int C, int sq,
                                                   float *__restrict__ hpre) {
  const int n = blockIdx.x, k = blockIdx.y * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= sq) return;
  const float *pn = pooled + (size_t)n * C, *wr = w1 + (size_t)k * C;
  float s0 = 0.f, s1 = 0.f;
  int c = lane;
  for (; c + 64 < C; c += 128) {
    s0 += wr[c] * pn[c];
    s1 += wr[c + 64] * pn[c + 64];
  }
  if (c < C) s0 += wr[c] * pn[c];
  const float s = wave_sum(s0 + s1);
  if (lane == 0) hpre[(size_t)n * sq + k] = s + (b1 ? b1[k] : 0.f);
}

// a[n][c] = W2[c] . swish(hpre[n]) + b2[c]  (W2 [C][sq]).  A block owns SE_CT channels x
// SE_NT samples: the W2 rows of its channels (one contiguous span, loaded coalesced) and the
// samples' hidden vectors are staged in LDS; thread (c, n) then dots them.  grid
// (C / SE_CT, N / SE_NT), dynamic LDS (SE_CT * (sq + 1) + SE_NT * sq) floats.
constexpr int SE_CT = 32, SE_NT = 8;
__global__ void __launch_bounds__(256) k_se_logits(const float *__restrict__ hpre,
                                                   const float *__restrict__ w2,
                                                   const float *__restrict__ b2, int N, int C,
                                                   int sq, float *__restrict__ a) {
  extern __shared__ float lds[];
  const int ld = sq + 1;  // odd row stride: the 32 rows sit in distinct banks
  float *sw = lds, *sh = lds + SE_CT * ld;
  const int c0 = blockIdx.x * SE_CT, n0 = blockIdx.y * SE_NT;
  const int nc = min(SE_CT, C - c0), nn = min(SE_NT, N - n0);
  const float *src = w2 + (size_t)c0 * sq;
  for (int e = threadIdx.x; e < nc * sq; e += 256) {
    const int r = e / sq;
    sw[r * ld + (e - r * sq)] = src[e];
  }
  for (int e = threadIdx.x; e < nn * sq; e += 256) {
    const float z = hpre[(size_t)n0 * sq + e];
    sh[e] = z * sigm(z);
  }
  __syncthreads();
  const int ci = threadIdx.x % SE_CT, ni = threadIdx.x / SE_CT;
  if (ci >= nc || ni >= nn) return;
  const float *wr = sw + ci * ld, *hr = sh + ni * sq;
  float s = 0.f;
#pragma unroll 4
  for (int k = 0; k < sq; ++k) s += wr[k] * hr[k];
  a[(size_t)(n0 + ni) * C + c0 + ci] = s + (b2 ? b2[c0 + ci] : 0.f);
}

// y = x * sigmoid(a[plane]); float4 stream (HW % 4 == 0) or scalar
__global__ void __launch_bounds__(256) k_se_excite(const float *__restrict__ x, SeIn tf,
                                                   const float *__restrict__ a, int HW,
                                                   long long nvec, int vec,
                                                   float *__restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const bool t = tf.sc != nullptr;
  const long long pl = vec ? i / (HW >> 2) : i / HW;
  const int c = (int)(pl % tf.C);
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  const float s = sigm(a[pl]);
  if (vec) {
    float4 v = se_in4(reinterpret_cast<const float4 *>(x)[i], sc, sh, t);
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    reinterpret_cast<float4 *>(y)[i] = v;
  } else {
    y[i] = se_in(x[i], sc, sh, t) * s;
  }
}

// da[plane] = s (1 - s) sum_hw dy * x      (wave per plane)
__global__ void __launch_bounds__(256) k_se_da(const float *__restrict__ x, SeIn tf,
                                               const float *__restrict__ dy,
                                               const float *__restrict__ a, int planes, int HW,
                                               float *__restrict__ da) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (pl >= planes) return;
  const bool t = tf.sc != nullptr;
  const int c = pl % tf.C;
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  const float *xp = x + (size_t)pl * HW, *gp = dy + (size_t)pl * HW;
  float acc = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2;
    const float4 *x4 = reinterpret_cast<const float4 *>(xp), *g4 = reinterpret_cast<const float4 *>(gp);
    for (int i0 = lane; i0 < HW4; i0 += 64 * SE_U) {
      float4 xv[SE_U], gv[SE_U];
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        const int i = min(i0 + u * 64, HW4 - 1);
        xv[u] = x4[i];
        gv[u] = g4[i];
      }
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        if (i0 + u * 64 >= HW4) break;
        const float4 w = se_in4(xv[u], sc, sh, t), g = gv[u];
        acc += (w.x * g.x + w.y * g.y) + (w.z * g.z + w.w * g.w);
      }
    }
  } else {
    for (int i = lane; i < HW; i += 64) acc += se_in(xp[i], sc, sh, t) * gp[i];
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float s = sigm(a[pl]);
    da[pl] = acc * s * (1.f - s);
  }
}

// Partial dh over one span of SE_DH_SPAN channels: dhp[n][j][k] = sum_{c in span j} W2[c][k]
// da[n][c].  Threads form KT hidden-unit lanes (KT = sq rounded up to a power of two, <= 256)
// x 256/KT channel slices, so a row of W2 is read by consecutive threads; the slices are
// summed in fixed order through LDS.  grid (N, C / SE_DH_SPAN).
constexpr int SE_DH_SPAN = 256;
static_assert(SE_MAXC / SE_DH_SPAN == 16, "e2ep_se_bwd workspace (e2ep.h) holds 16 dh partials");
__global__ void __launch_bounds__(256) k_se_dh(const float *__restrict__ da,
                                               const float *__restrict__ w2, int C, int sq, int KT,
                                               float *__restrict__ dhp) {
  __shared__ float red[256];
  const int n = blockIdx.x, j = blockIdx.y;
  const int k = threadIdx.x % KT, sl = threadIdx.x / KT, nsl = 256 / KT;
  const int cb = j * SE_DH_SPAN, ce = min(C, cb + SE_DH_SPAN);
  const float *dn = da + (size_t)n * C;
  float s = 0.f;
  if (k < sq)
#pragma unroll 4
    for (int c = cb + sl; c < ce; c += nsl) s += w2[(size_t)c * sq + k] * dn[c];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < KT && k < sq) {
    float t = 0.f;
    for (int q = 0; q < nsl; ++q) t += red[q * KT + k];
    dhp[((size_t)n * gridDim.y + j) * sq + k] = t;
  }
}

// dhpre = (sum of the dh partials) * swish'(hpre);  dpooled[n][c] = sum_k W1[k][c] dhpre[n][k]
// (thread per c, coalesced W1 columns).  grid (N, C-chunks of 256).
__global__ void __launch_bounds__(256) k_se_dpooled(const float *__restrict__ dhp, int spans,
                                                    const float *__restrict__ hpre,
                                                    const float *__restrict__ w1, int C, int sq,
                                                    float *__restrict__ dhpre,
                                                    float *__restrict__ dpooled) {
  __shared__ float sd[SE_MAXSQ];
  const int n = blockIdx.x;
  for (int k = threadIdx.x; k < sq; k += 256) {
    float t = 0.f;
    for (int j = 0; j < spans; ++j) t += dhp[((size_t)n * spans + j) * sq + k];
    const float z = hpre[(size_t)n * sq + k], sg = sigm(z);
    const float g = t * (sg * (1.f + z * (1.f - sg)));
    if (blockIdx.y == 0) dhpre[(size_t)n * sq + k] = g;
    sd[k] = g;
  }
  __syncthreads();
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c < C) {
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < sq; ++k) s += w1[(size_t)k * C + c] * sd[k];
    dpooled[(size_t)n * C + c] = s;
  }
}

// weight gradients, sums over the batch in sample order (one thread per output):
//   dW1[k][c] = sum_n dhpre[n][k] pooled[n][c]     dW2[c][k] = sum_n da[n][c] swish(hpre[n][k])
//   db1[k]    = sum_n dhpre[n][k]                  db2[c]    = sum_n da[n][c]
__global__ void __launch_bounds__(256) k_se_wgrad(const float *__restrict__ pooled,
                                                  const float *__restrict__ hpre,
                                                  const float *__restrict__ da,
                                                  const float *__restrict__ dhpre, int N, int C,
                                                  int sq, float *__restrict__ dw1,
                                                  float *__restrict__ db1, float *__restrict__ dw2,
                                                  float *__restrict__ db2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n1 = sq * C, n2 = C * sq;
  float s = 0.f;
  if (i < n1) {
    const int k = i / C, c = i - k * C;
#pragma unroll 8
    for (int n = 0; n < N; ++n) s += dhpre[(size_t)n * sq + k] * pooled[(size_t)n * C + c];
    if (dw1) dw1[i] = s;
  } else if (i < n1 + n2) {
    const int j = i - n1, c = j / sq, k = j - c * sq;
#pragma unroll 8
    for (int n = 0; n < N; ++n) {
      const float z = hpre[(size_t)n * sq + k];
      s += da[(size_t)n * C + c] * (z * sigm(z));
    }
    if (dw2) dw2[j] = s;
  } else if (i < n1 + n2 + sq) {
    const int k = i - n1 - n2;
#pragma unroll 8
    for (int n = 0; n < N; ++n) s += dhpre[(size_t)n * sq + k];
    if (db1) db1[k] = s;
  } else if (i < n1 + n2 + sq + C) {
    const int c = i - n1 - n2 - sq;
#pragma unroll 8
    for (int n = 0; n < N; ++n) s += da[(size_t)n * C + c];
    if (db2) db2[c] = s;
  }
}

// dx = dy * sigmoid(a[plane]) + dpooled[plane] / HW
__global__ void __launch_bounds__(256) k_se_dx(const float *__restrict__ dy,
                                               const float *__restrict__ a,
                                               const float *__restrict__ dpooled, int HW,
                                               long long nvec, int vec, float *__restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const float inv = 1.f / (float)HW;
  if (vec) {
    const long long pl = i / (HW >> 2);
    const float s = sigm(a[pl]), d = dpooled[pl] * inv;
    float4 g = reinterpret_cast<const float4 *>(dy)[i];
    g.x = g.x * s + d; g.y = g.y * s + d; g.z = g.z * s + d; g.w = g.w * s + d;
    reinterpret_cast<float4 *>(dx)[i] = g;
  } else {
    const long long pl = i / HW;
    dx[i] = dy[i] * sigm(a[pl]) + dpooled[pl] * inv;
  }
}

// ------------------------------------------------------------------------------------------
// Fused forms (e2ep_tune key 27 = 2; OFF by default): the MLP on the 1x1 map runs inside the
// streaming kernels instead of as launches of its own.  Measured in the replayed C2 step
// (profiles/r04/se_fold_ab.txt): 25.7 vs 23.9 ms/step — k_se_squeeze_mlp 56 us against 13 + 5
// for squeeze + hidden, k_se_da_mlp 66 us against 20 + 8 + 6 — because every one of the
// thousands of small streaming workgroups (4 planes, 4 KB at 16x16) now ends in a
// write-through store drain and a returning device-scope atomic (several us each under
// load, paid once per residency round), which costs more than the launches it saves.
//  * k_se_squeeze_mlp: the squeeze; a sample's C/4 workgroups store their plane means
//    write-through and take an arrival ticket (handoff.h); the sample's last workgroup reads
//    the C means back (sc1) and computes hpre[n][k] = W1[k] . pooled[n] + b1[k] for every k.
//  * k_se_excite_logits: the excite; each workgroup first forms the logits a of the planes it
//    covers (a wave per plane: W2[c] . swish(hpre[n]) + b2[c]), the workgroup holding a
//    plane's first element stores it for the backward.
//  * k_se_da_mlp: da per plane as k_se_da; a sample's last workgroup then forms
//    dh = W2^T da[n], dhpre = dh * swish'(hpre), dpooled[n] = W1^T dhpre.
// Every sum runs in a fixed order, so results are run-to-run deterministic.  Needs C % 4 == 0
// (a workgroup's four planes belong to one sample).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_se_squeeze_mlp(const float *__restrict__ x, SeIn tf,
                                                        int HW, const float *__restrict__ w1,
                                                        const float *__restrict__ b1, int sq,
                                                        float *__restrict__ pooled,
                                                        float *__restrict__ hpre,
                                                        unsigned int *__restrict__ cnt) {
  __shared__ float sp[SE_MAXC];
  __shared__ int s_last;
  const int C = tf.C;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pl = blockIdx.x * 4 + wave;
  const int n = (blockIdx.x * 4) / C;
  const bool t = tf.sc != nullptr;
  const int c = pl - n * C;
  const float s = plane_sum(x + (size_t)pl * HW, HW, lane, t ? tf.sc[c] : 1.f, t ? tf.sh[c] : 0.f, t);
  if (lane == 0) st_sc1(pooled + pl, s / (float)HW);
  handoff_drain();
  if (!handoff_arrive(cnt + n, C / 4, &s_last)) return;
  for (int i = threadIdx.x; i < C; i += 256) sp[i] = ld_sc1(pooled + (size_t)n * C + i);
  __syncthreads();
  for (int k = wave; k < sq; k += 4) {  // k_se_hidden's dot, one wave per hidden unit
    const float *wr = w1 + (size_t)k * C;
    float s0 = 0.f, s1 = 0.f;
    int i = lane;
    for (; i + 64 < C; i += 128) {
      s0 += wr[i] * sp[i];
      s1 += wr[i + 64] * sp[i + 64];
    }
    if (i < C) s0 += wr[i] * sp[i];
    const float h = wave_sum(s0 + s1);
    if (lane == 0) hpre[(size_t)n * sq + k] = h + (b1 ? b1[k] : 0.f);
  }
}

constexpr int SE_XPL = 32;  // planes one excite workgroup may cover (>= 16 elements per plane)
__global__ void __launch_bounds__(256) k_se_excite_logits(const float *__restrict__ x, SeIn tf,
                                                          const float *__restrict__ hpre,
                                                          const float *__restrict__ w2,
                                                          const float *__restrict__ b2, int sq,
                                                          int HW, long long nvec, int vec,
                                                          float *__restrict__ a,
                                                          float *__restrict__ y) {
  __shared__ float sa[SE_XPL];
  const int C = tf.C;
  const int per = vec ? HW >> 2 : HW;  // vector elements per plane
  const long long i0 = (long long)blockIdx.x * 256;
  const long long i1 = min(nvec, i0 + 256) - 1;
  const long long pl0 = i0 / per;
  const int np = (int)(i1 / per - pl0) + 1;  // host guarantees <= SE_XPL
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int j = wave; j < np; j += 4) {
    const long long pl = pl0 + j;
    const int n = (int)(pl / C), c = (int)(pl - (long long)n * C);
    const float *wr = w2 + (size_t)c * sq, *hr = hpre + (size_t)n * sq;
    float s = 0.f;
    for (int k = lane; k < sq; k += 64) {
      const float z = hr[k];
      s += wr[k] * (z * sigm(z));
    }
    s = wave_sum(s) + (b2 ? b2[c] : 0.f);
    if (lane == 0) {
      sa[j] = s;
      if (pl * per >= i0) a[pl] = s;  // the workgroup holding the plane's first element
    }
  }
  __syncthreads();
  const long long i = i0 + threadIdx.x;
  if (i >= nvec) return;
  const bool t = tf.sc != nullptr;
  const long long pl = i / per;
  const int c = (int)(pl % C);
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  const float g = sigm(sa[pl - pl0]);
  if (vec) {
    float4 v = se_in4(reinterpret_cast<const float4 *>(x)[i], sc, sh, t);
    v.x *= g; v.y *= g; v.z *= g; v.w *= g;
    reinterpret_cast<float4 *>(y)[i] = v;
  } else {
    y[i] = se_in(x[i], sc, sh, t) * g;
  }
}

__global__ void __launch_bounds__(256) k_se_da_mlp(const float *__restrict__ x, SeIn tf,
                                                   const float *__restrict__ dy,
                                                   const float *__restrict__ a, int HW,
                                                   const float *__restrict__ w1,
                                                   const float *__restrict__ w2,
                                                   const float *__restrict__ hpre, int sq, int KT,
                                                   float *__restrict__ da,
                                                   float *__restrict__ dhpre,
                                                   float *__restrict__ dpooled,
                                                   unsigned int *__restrict__ cnt) {
  __shared__ float sda[SE_MAXC];
  __shared__ float red[256];
  __shared__ float sdh[SE_MAXSQ];
  __shared__ int s_last;
  const int C = tf.C;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pl = blockIdx.x * 4 + wave;
  const int n = (blockIdx.x * 4) / C;
  const bool t = tf.sc != nullptr;
  const int c = pl - n * C;
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  const float *xp = x + (size_t)pl * HW, *gp = dy + (size_t)pl * HW;
  float acc = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2;
    const float4 *x4 = reinterpret_cast<const float4 *>(xp), *g4 = reinterpret_cast<const float4 *>(gp);
    for (int i0 = lane; i0 < HW4; i0 += 64 * SE_U) {
      float4 xv[SE_U], gv[SE_U];
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        const int i = min(i0 + u * 64, HW4 - 1);
        xv[u] = x4[i];
        gv[u] = g4[i];
      }
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        if (i0 + u * 64 >= HW4) break;
        const float4 w = se_in4(xv[u], sc, sh, t), g = gv[u];
        acc += (w.x * g.x + w.y * g.y) + (w.z * g.z + w.w * g.w);
      }
    }
  } else {
    for (int i = lane; i < HW; i += 64) acc += se_in(xp[i], sc, sh, t) * gp[i];
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float s = sigm(a[pl]);
    st_sc1(da + pl, acc * s * (1.f - s));
  }
  handoff_drain();
  if (!handoff_arrive(cnt + n, C / 4, &s_last)) return;
  for (int i = threadIdx.x; i < C; i += 256) sda[i] = ld_sc1(da + (size_t)n * C + i);
  __syncthreads();
  // dh[k] = sum_c W2[c][k] da[n][c]: KT hidden-unit lanes x 256/KT channel slices (a W2 row
  // is read by consecutive threads), slices summed in order
  {
    const int k = threadIdx.x % KT, sl = threadIdx.x / KT, nsl = 256 / KT;
    float s = 0.f;
    if (k < sq)
#pragma unroll 4
      for (int i = sl; i < C; i += nsl) s += w2[(size_t)i * sq + k] * sda[i];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < KT && k < sq) {
      float tt = 0.f;
      for (int q = 0; q < nsl; ++q) tt += red[q * KT + k];
      const float z = hpre[(size_t)n * sq + k], sg = sigm(z);
      const float g = tt * (sg * (1.f + z * (1.f - sg)));
      dhpre[(size_t)n * sq + k] = g;
      sdh[k] = g;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += 256) {  // dpooled[n][c] = sum_k W1[k][c] dhpre[n][k]
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < sq; ++k) s += w1[(size_t)k * C + i] * sdh[k];
    dpooled[(size_t)n * C + i] = s;
  }
}

}  // namespace e2ep

using namespace e2ep;

// fused squeeze-excitation launches (e2ep_tune key 27 = 2): a workgroup's four planes in one
// sample; an excite workgroup of 256 vector elements covers at most 255 / 16 + 2 <= SE_XPL
// planes when a plane has >= 16 of them
static bool se_fused_ok(int C, int HW) {
  return g_tune[TUNE_SE_FUSED] == 2 && C % 4 == 0 && ((HW & 3) == 0 ? HW / 4 : HW) >= 16;
}

extern "C" {

int e2ep_se_fwd(const float *x, const float *x_scale, const float *x_shift, const float *w1,
                const float *b1, const float *w2, const float *b2, int N, int C, int HW, int sq,
                float *pooled, float *hpre, float *a, float *y, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0 && sq > 0, E2EP_EINVAL, "e2ep_se_fwd: bad shape");
  E2EP_REQUIRE(!x_scale == !x_shift, E2EP_EINVAL, "e2ep_se_fwd: x_scale / x_shift both or neither");
  const SeIn tf{x_scale, x_shift, C};
  E2EP_REQUIRE(C <= SE_MAXC && sq <= SE_MAXSQ, E2EP_ERANGE, "e2ep_se_fwd: C %d > %d or sq %d > %d",
               C, SE_MAXC, sq, SE_MAXSQ);
  hipStream_t s = as_stream(stream);
  const int planes = N * C;
  const int vec = (HW & 3) == 0;
  const long long nvec = (long long)planes * HW / (vec ? 4 : 1);
  unsigned int *cnt = se_fused_ok(C, HW) ? handoff_slots(N) : nullptr;
  if (cnt) {  // two launches: squeeze + hidden units, logits + excite
    hipLaunchKernelGGL(k_se_squeeze_mlp, dim3(planes / 4), dim3(256), 0, s, x, tf, HW, w1, b1, sq,
                       pooled, hpre, cnt);
    hipLaunchKernelGGL(k_se_excite_logits, dim3(cdiv(nvec, 256)), dim3(256), 0, s, x, tf, hpre,
                       w2, b2, sq, HW, nvec, vec, a, y);
    return launch_status("e2ep_se_fwd");
  }
  hipLaunchKernelGGL(k_se_squeeze, dim3(cdiv(planes, 4)), dim3(256), 0, s, x, tf, planes, HW,
                     pooled);
  hipLaunchKernelGGL(k_se_hidden, dim3(N, cdiv(sq, 4)), dim3(256), 0, s, pooled, w1, b1, C, sq,
                     hpre);
  hipLaunchKernelGGL(k_se_logits, dim3(cdiv(C, SE_CT), cdiv(N, SE_NT)), dim3(256),
                     (SE_CT * (sq + 1) + SE_NT * sq) * sizeof(float), s, hpre, w2, b2, N, C, sq, a);
  hipLaunchKernelGGL(k_se_excite, dim3(cdiv(nvec, 256)), dim3(256), 0, s, x, tf, a, HW, nvec, vec,
                     y);
  return launch_status("e2ep_se_fwd");
}

int e2ep_se_bwd(const float *x, const float *x_scale, const float *x_shift, const float *dy,
                const float *w1, const float *w2, const float *pooled, const float *hpre,
                const float *a, int N, int C, int HW, int sq, float *dx, float *dpooled_out,
                float *dw1, float *db1, float *dw2, float *db2, float *workspace, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0 && sq > 0, E2EP_EINVAL, "e2ep_se_bwd: bad shape");
  E2EP_REQUIRE(!x_scale == !x_shift, E2EP_EINVAL, "e2ep_se_bwd: x_scale / x_shift both or neither");
  E2EP_REQUIRE(!(x_scale && dx), E2EP_EINVAL,
               "e2ep_se_bwd: with an input transform dx is formed by e2ep_bn_bwd (gate_logit / "
               "gate_dpooled); pass dx = NULL");
  const SeIn tf{x_scale, x_shift, C};
  E2EP_REQUIRE(C <= SE_MAXC && sq <= SE_MAXSQ, E2EP_ERANGE, "e2ep_se_bwd: C %d > %d or sq %d > %d",
               C, SE_MAXC, sq, SE_MAXSQ);
  hipStream_t s = as_stream(stream);
  const int planes = N * C;
  float *da = workspace, *dhpre = workspace + 2 * planes;
  float *dpooled = dpooled_out ? dpooled_out : workspace + planes;
  float *dhp = workspace + 2 * planes + N * sq;
  const int spans = cdiv(C, SE_DH_SPAN);
  int KT = 1;
  while (KT < sq) KT *= 2;
  unsigned int *cnt = se_fused_ok(C, HW) ? handoff_slots(N) : nullptr;
  if (cnt) {  // da + the MLP backward in one launch
    hipLaunchKernelGGL(k_se_da_mlp, dim3(planes / 4), dim3(256), 0, s, x, tf, dy, a, HW, w1, w2,
                       hpre, sq, KT, da, dhpre, dpooled, cnt);
  } else {
    hipLaunchKernelGGL(k_se_da, dim3(cdiv(planes, 4)), dim3(256), 0, s, x, tf, dy, a, planes, HW, da);
    hipLaunchKernelGGL(k_se_dh, dim3(N, spans), dim3(256), 0, s, da, w2, C, sq, KT, dhp);
    hipLaunchKernelGGL(k_se_dpooled, dim3(N, cdiv(C, 256)), dim3(256), 0, s, dhp, spans, hpre, w1,
                       C, sq, dhpre, dpooled);
  }
  if (dw1 || db1 || dw2 || db2) {
    const int outs = 2 * sq * C + sq + C;
    hipLaunchKernelGGL(k_se_wgrad, dim3(cdiv(outs, 256)), dim3(256), 0, s, pooled, hpre, da, dhpre,
                       N, C, sq, dw1, db1, dw2, db2);
  }
  if (dx) {
    const int vec = (HW & 3) == 0;
    const long long nvec = (long long)planes * HW / (vec ? 4 : 1);
    hipLaunchKernelGGL(k_se_dx, dim3(cdiv(nvec, 256)), dim3(256), 0, s, dy, a, dpooled, HW, nvec, vec,
                       dx);
  }
  return launch_status("e2ep_se_bwd");
}

}  // extern "C"
