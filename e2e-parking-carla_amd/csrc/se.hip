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

// Contraction only within one expression (a*b + c -> fma): the fp32 and bf16-storage
// instantiations of a kernel (E2EP_IO_*) then fuse the same operations and round alike —
// under the default cross-statement contraction hipcc may pick a different multiply to fuse
// in each instantiation (tests/test_bf16_store_gpu.py holds them bitwise equal).
#pragma clang fp contract(on)

namespace e2ep {

constexpr int SE_MAXC = 4096, SE_MAXSQ = 256;
// float4 loads in flight per lane in the per-plane reductions (squeeze, da)
constexpr int SE_U = 4;

__device__ __forceinline__ float sigm(float v) { return sigmoid_f(v); }

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
  return swish_f(z);
}
__device__ __forceinline__ float4 se_in4(float4 v, float sc, float sh, bool t) {
  return make_float4(se_in(v.x, sc, sh, t), se_in(v.y, sc, sh, t), se_in(v.z, sc, sh, t),
                     se_in(v.w, sc, sh, t));
}

// sum over one plane (HW values, 4 at a time when HW % 4 == 0) by one wave; TX = float or
// bf16_t (bf16 activation storage, E2EP_IO_X_BF16)
template <typename TX>
__device__ __forceinline__ float plane_sum(const TX *__restrict__ p, int HW, int lane,
                                           float sc, float sh, bool t) {
  float s = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2;
    // SE_U loads in flight per lane (clamped, unconditional); the lane still sums i, i + 64,
    // ... in ascending order
    for (int i0 = lane; i0 < HW4; i0 += 64 * SE_U) {
      float4 v[SE_U];
#pragma unroll
      for (int u = 0; u < SE_U; ++u) v[u] = ld4(p + 4 * min(i0 + u * 64, HW4 - 1));
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        if (i0 + u * 64 >= HW4) break;
        const float4 w = se_in4(v[u], sc, sh, t);
        s += (w.x + w.y) + (w.z + w.w);
      }
    }
  } else {
    for (int i = lane; i < HW; i += 64) s += se_in(ld1(p + i), sc, sh, t);
  }
  return wave_sum(s);
}

template <typename TX>
__global__ void __launch_bounds__(256) k_se_squeeze(const TX *__restrict__ x, SeIn tf,
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
template <typename TX, typename TY = float>
__global__ void __launch_bounds__(256) k_se_excite(const TX *__restrict__ x, SeIn tf,
                                                   const float *__restrict__ a, int HW,
                                                   long long nvec, int vec,
                                                   TY *__restrict__ y) {
  // 32-bit indices (nvec < 2^29, checked by e2ep_se_fwd): a 64-bit division and remainder per
  // thread cost more than the float4's arithmetic
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= nvec) return;
  const bool t = tf.sc != nullptr;
  const int pl = vec ? i / (HW >> 2) : i / HW;
  const int c = pl % tf.C;
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  const float s = sigm(a[pl]);
  if (vec) {
    float4 v = se_in4(ld4(x + 4 * i), sc, sh, t);
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    st4(y + 4 * i, v);
  } else {
    st1(y + i, se_in(ld1(x + i), sc, sh, t) * s);
  }
}

// k_se_excite with k_se_logits folded in (e2ep_tune key 34 = 2): the block's planes [p0, p1]
// (at most SE_XP) get a[p] = W2[c] . swish(hpre[n]) + b2[c] first, one wave per plane (lanes
// over the hidden units, fixed-order wave reduction), their gates sigmoid(a) in LDS; the block
// holding a plane's first element also writes a[p] (the backward's input).  One launch and one
// dependent hop fewer per SE block, on the forward's critical path.
constexpr int SE_XP = 8;
template <typename TX, typename TY = float>
__global__ void __launch_bounds__(256) k_se_excite_mlp(const TX *__restrict__ x, SeIn tf,
                                                       const float *__restrict__ hpre,
                                                       const float *__restrict__ w2,
                                                       const float *__restrict__ b2, int sq,
                                                       float *__restrict__ a, int HW,
                                                       long long nvec, int vec,
                                                       TY *__restrict__ y) {
  __shared__ float sg[SE_XP];
  const int per = vec ? (HW >> 2) : HW;  // vectors per plane
  const int i0 = (int)(blockIdx.x * blockDim.x);
  const int last = (int)min((long long)i0 + (long long)blockDim.x, nvec) - 1;
  const int p0 = i0 / per, p1 = last / per;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int p = p0 + wv; p <= p1; p += 4) {  // wave-uniform
    const int n = p / tf.C, c = p - n * tf.C;
    const float *hr = hpre + (size_t)n * sq, *wr = w2 + (size_t)c * sq;
    float acc = 0.f;
    for (int k = lane; k < sq; k += 64) {
      const float z = hr[k];
      acc += wr[k] * (z * sigm(z));
    }
    acc = wave_sum(acc);
    const float av = acc + (b2 ? b2[c] : 0.f);
    if (lane == 0) {
      sg[p - p0] = sigm(av);
      if (p * per >= i0) a[p] = av;  // the plane starts in this block
    }
  }
  __syncthreads();
  const int i = i0 + (int)threadIdx.x;
  if (i >= nvec) return;
  const bool t = tf.sc != nullptr;
  const int pl = i / per;
  const int c = pl % tf.C;
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  const float g = sg[pl - p0];
  if (vec) {
    float4 v = se_in4(ld4(x + 4 * i), sc, sh, t);
    v.x *= g; v.y *= g; v.z *= g; v.w *= g;
    st4(y + 4 * i, v);
  } else {
    st1(y + i, se_in(ld1(x + i), sc, sh, t) * g);
  }
}

// The block's _bn1 backward sums, taken in the same pass (BNS, training BN with the SE input
// transform): with xhat = (x - mean) invstd, zb = xhat gamma + beta (the arithmetic of
// bn.hip's BnBwdElem) and sp = swish'(zb), the BN backward's channel sums of
// dzb = (dy sigmoid(a) + dpooled / HW) sp factor per plane into
//   A1 = sum dy sp,  A2 = sum sp,  A3 = sum dy sp xhat,  A4 = sum sp xhat
// (fp64 per plane), which e2ep_bn_bwd_planes combines with the gate once dpooled is known —
// the BN backward's own reduction pass over x and dy is not run.
struct SeBn {
  const float *mean, *invstd, *gamma, *beta;
  double *sums;  // [planes][4]
};

// da[plane] = s (1 - s) sum_hw dy * x      (wave per plane)
template <bool BNS, typename TX, typename TD = float>
__global__ void __launch_bounds__(256) k_se_da(const TX *__restrict__ x, SeIn tf,
                                               const TD *__restrict__ dy,
                                               const float *__restrict__ a, int planes, int HW,
                                               float *__restrict__ da, SeBn bn) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (pl >= planes) return;
  const bool t = tf.sc != nullptr;
  const int c = pl % tf.C;
  const float sc = t ? tf.sc[c] : 1.f, sh = t ? tf.sh[c] : 0.f;
  float mu = 0.f, is = 1.f, gm = 1.f, bt = 0.f;
  if constexpr (BNS) {
    mu = bn.mean[c];
    is = bn.invstd[c];
    gm = bn.gamma ? bn.gamma[c] : 1.f;
    bt = bn.beta ? bn.beta[c] : 0.f;
  }
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0;
  const TX *xp = x + (size_t)pl * HW;
  const TD *gp = dy + (size_t)pl * HW;
  float acc = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2;
    for (int i0 = lane; i0 < HW4; i0 += 64 * SE_U) {
      float4 xv[SE_U], gv[SE_U];
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        const int i = min(i0 + u * 64, HW4 - 1);
        xv[u] = ld4(xp + 4 * i);
        gv[u] = ld4(gp + 4 * i);
      }
#pragma unroll
      for (int u = 0; u < SE_U; ++u) {
        if (i0 + u * 64 >= HW4) break;
        const float4 g = gv[u];
        if constexpr (BNS) {
          // one sigmoid per element serves the SE input t = zb s and the BN's swish'(zb)
          // (zb = xhat gamma + beta: the BN backward's arithmetic; t equals the forward's
          // swish(x scale + shift) up to rounding)
          const float xv4[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
          const float gv4[4] = {g.x, g.y, g.z, g.w};
          float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float xh = (xv4[j] - mu) * is;
            const float zb = xh * gm + bt;
            const float sg = sigmoid_f(zb);
            const float sp = sg * (1.f + zb * (1.f - sg));
            a0 += (zb * sg) * gv4[j];
            a1 += gv4[j] * sp;
            a2 += sp;
            a3 += gv4[j] * sp * xh;
            a4 += sp * xh;
          }
          acc += a0;
          s1 += a1; s2 += a2; s3 += a3; s4 += a4;
        } else {
          const float4 w = se_in4(xv[u], sc, sh, t);
          acc += (w.x * g.x + w.y * g.y) + (w.z * g.z + w.w * g.w);
        }
      }
    }
  } else {
    for (int i = lane; i < HW; i += 64) {
      const float xv = ld1(xp + i), g = ld1(gp + i);
      if constexpr (BNS) {
        const float xh = (xv - mu) * is;
        const float zb = xh * gm + bt;
        const float sg = sigmoid_f(zb);
        const float sp = sg * (1.f + zb * (1.f - sg));
        acc += (zb * sg) * g;
        s1 += g * sp; s2 += sp; s3 += g * sp * xh; s4 += sp * xh;
      } else {
        acc += se_in(xv, sc, sh, t) * g;
      }
    }
  }
  acc = wave_sum(acc);
  if constexpr (BNS) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
      s3 += __shfl_xor(s3, o, 64);
      s4 += __shfl_xor(s4, o, 64);
    }
    if (lane == 0) {
      double *o = bn.sums + 4LL * pl;
      o[0] = s1; o[1] = s2; o[2] = s3; o[3] = s4;
    }
  }
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

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_se_fwd(const void *x, const float *x_scale, const float *x_shift, const float *w1,
                const float *b1, const float *w2, const float *b2, int N, int C, int HW, int sq,
                float *pooled, float *hpre, float *a, void *y, void *stream, int io) {
  E2EP_REQUIRE(io == 0 || ((io == E2EP_IO_X_BF16 || io == (E2EP_IO_X_BF16 | E2EP_IO_DX_BF16)) &&
                           HW % 4 == 0),
               E2EP_EINVAL, "e2ep_se_fwd: storage mask %d not supported (0, X or X|DX bf16, "
               "HW %% 4 == 0)", io);
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0 && sq > 0, E2EP_EINVAL, "e2ep_se_fwd: bad shape");
  E2EP_REQUIRE(!x_scale == !x_shift, E2EP_EINVAL, "e2ep_se_fwd: x_scale / x_shift both or neither");
  const SeIn tf{x_scale, x_shift, C};
  E2EP_REQUIRE(C <= SE_MAXC && sq <= SE_MAXSQ, E2EP_ERANGE, "e2ep_se_fwd: C %d > %d or sq %d > %d",
               C, SE_MAXC, sq, SE_MAXSQ);
  hipStream_t s = as_stream(stream);
  const int planes = N * C;
  const int vec = (HW & 3) == 0;
  const long long nvec = (long long)planes * HW / (vec ? 4 : 1);
  E2EP_REQUIRE(nvec < (1LL << 29), E2EP_ERANGE, "e2ep_se_fwd: %lld vectors >= 2^29", nvec);
  if (io)
    hipLaunchKernelGGL(k_se_squeeze<bf16_t>, dim3(cdiv(planes, 4)), dim3(256), 0, s,
                       static_cast<const bf16_t *>(x), tf, planes, HW, pooled);
  else
    hipLaunchKernelGGL(k_se_squeeze<float>, dim3(cdiv(planes, 4)), dim3(256), 0, s,
                       static_cast<const float *>(x), tf, planes, HW, pooled);
  hipLaunchKernelGGL(k_se_hidden, dim3(N, cdiv(sq, 4)), dim3(256), 0, s, pooled, w1, b1, C, sq,
                     hpre);
  // the logits inside the excite launch (key 34 = 2) when a 256-thread block spans at most
  // SE_XP planes
  const int per = vec ? HW / 4 : HW;
  if (g_tune[TUNE_SE_EXCITE_MLP] == 2 && cdiv(256, per) + 1 <= SE_XP) {
#define E2EP_SEX(TXV, TYV)                                                                      \
  hipLaunchKernelGGL((k_se_excite_mlp<TXV, TYV>), dim3(cdiv(nvec, 256)), dim3(256), 0, s,       \
                     static_cast<const TXV *>(x), tf, hpre, w2, b2, sq, a, HW, nvec, vec,        \
                     static_cast<TYV *>(y))
    if (io & E2EP_IO_DX_BF16) E2EP_SEX(bf16_t, bf16_t);
    else if (io) E2EP_SEX(bf16_t, float);
    else E2EP_SEX(float, float);
#undef E2EP_SEX
    return launch_status("e2ep_se_fwd");
  }
  hipLaunchKernelGGL(k_se_logits, dim3(cdiv(C, SE_CT), cdiv(N, SE_NT)), dim3(256),
                     (SE_CT * (sq + 1) + SE_NT * sq) * sizeof(float), s, hpre, w2, b2, N, C, sq, a);
  if (io & E2EP_IO_DX_BF16)
    hipLaunchKernelGGL((k_se_excite<bf16_t, bf16_t>), dim3(cdiv(nvec, 256)), dim3(256), 0, s,
                       static_cast<const bf16_t *>(x), tf, a, HW, nvec, vec, static_cast<bf16_t *>(y));
  else if (io)
    hipLaunchKernelGGL((k_se_excite<bf16_t, float>), dim3(cdiv(nvec, 256)), dim3(256), 0, s,
                       static_cast<const bf16_t *>(x), tf, a, HW, nvec, vec, static_cast<float *>(y));
  else
    hipLaunchKernelGGL((k_se_excite<float, float>), dim3(cdiv(nvec, 256)), dim3(256), 0, s,
                       static_cast<const float *>(x), tf, a, HW, nvec, vec, static_cast<float *>(y));
  return launch_status("e2ep_se_fwd");
}

static int se_bwd_impl(const void *x, int io, const float *x_scale, const float *x_shift,
                       const void *dy, const float *w1, const float *w2, const float *pooled,
                       const float *hpre, const float *a, int N, int C, int HW, int sq, float *dx,
                       float *dpooled_out, float *dw1, float *db1, float *dw2, float *db2,
                       float *workspace, const SeBn &bn, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0 && sq > 0, E2EP_EINVAL, "e2ep_se_bwd: bad shape");
  E2EP_REQUIRE(!x_scale == !x_shift, E2EP_EINVAL, "e2ep_se_bwd: x_scale / x_shift both or neither");
  E2EP_REQUIRE(io == 0 || ((io == E2EP_IO_X_BF16 || io == (E2EP_IO_X_BF16 | E2EP_IO_DY_BF16)) &&
                           HW % 4 == 0 && !dx),
               E2EP_EINVAL, "e2ep_se_bwd: storage mask %d not supported (0, X or X|DY bf16 with "
               "dx formed by the BN backward, HW %% 4 == 0)", io);
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
  const float *xf = static_cast<const float *>(x);
  const bf16_t *xh = static_cast<const bf16_t *>(x);
  const float *df = static_cast<const float *>(dy);
  const bf16_t *dh = static_cast<const bf16_t *>(dy);
  const dim3 gda(cdiv(planes, 4));
  const bool hx = io & E2EP_IO_X_BF16, hd = io & E2EP_IO_DY_BF16;
#define SE_DA(BNSV)                                                                                   \
  do {                                                                                                \
    if (hx && hd)                                                                                     \
      hipLaunchKernelGGL((k_se_da<BNSV, bf16_t, bf16_t>), gda, dim3(256), 0, s, xh, tf, dh, a, planes, \
                         HW, da, bn);                                                                 \
    else if (hx)                                                                                      \
      hipLaunchKernelGGL((k_se_da<BNSV, bf16_t, float>), gda, dim3(256), 0, s, xh, tf, df, a, planes, \
                         HW, da, bn);                                                                 \
    else                                                                                              \
      hipLaunchKernelGGL((k_se_da<BNSV, float, float>), gda, dim3(256), 0, s, xf, tf, df, a, planes,  \
                         HW, da, bn);                                                                 \
  } while (0)
  if (bn.sums) SE_DA(true);
  else SE_DA(false);
#undef SE_DA
  hipLaunchKernelGGL(k_se_dh, dim3(N, spans), dim3(256), 0, s, da, w2, C, sq, KT, dhp);
  hipLaunchKernelGGL(k_se_dpooled, dim3(N, cdiv(C, 256)), dim3(256), 0, s, dhp, spans, hpre, w1,
                     C, sq, dhpre, dpooled);
  if (dw1 || db1 || dw2 || db2) {
    const int outs = 2 * sq * C + sq + C;
    hipLaunchKernelGGL(k_se_wgrad, dim3(cdiv(outs, 256)), dim3(256), 0, s, pooled, hpre, da, dhpre,
                       N, C, sq, dw1, db1, dw2, db2);
  }
  if (dx) {
    const int vec = (HW & 3) == 0;
    const long long nvec = (long long)planes * HW / (vec ? 4 : 1);
    hipLaunchKernelGGL(k_se_dx, dim3(cdiv(nvec, 256)), dim3(256), 0, s, static_cast<const float *>(dy), a,
                       dpooled, HW, nvec, vec, dx);
  }
  return launch_status("e2ep_se_bwd");
}

int e2ep_se_bwd(const void *x, const float *x_scale, const float *x_shift, const void *dy,
                const float *w1, const float *w2, const float *pooled, const float *hpre,
                const float *a, int N, int C, int HW, int sq, float *dx, float *dpooled_out,
                float *dw1, float *db1, float *dw2, float *db2, float *workspace, void *stream,
                int io) {
  return se_bwd_impl(x, io, x_scale, x_shift, dy, w1, w2, pooled, hpre, a, N, C, HW, sq, dx,
                     dpooled_out, dw1, db1, dw2, db2, workspace, SeBn{}, stream);
}

int e2ep_se_bwd_bn(const void *x, const float *x_scale, const float *x_shift,
                   const float *bn_mean, const float *bn_invstd, const float *gamma,
                   const float *beta, const void *dy, const float *w1, const float *w2,
                   const float *pooled, const float *hpre, const float *a, int N, int C, int HW,
                   int sq, float *dpooled_out, float *dw1, float *db1, float *dw2, float *db2,
                   double *plane_sums, float *workspace, void *stream, int io) {
  E2EP_REQUIRE(x_scale && x_shift && bn_mean && bn_invstd && dpooled_out && plane_sums,
               E2EP_EINVAL, "e2ep_se_bwd_bn: the BN transform, its statistics, dpooled_out and "
               "plane_sums are required");
  return se_bwd_impl(x, io, x_scale, x_shift, dy, w1, w2, pooled, hpre, a, N, C, HW, sq, nullptr,
                     dpooled_out, dw1, db1, dw2, db2, workspace,
                     SeBn{bn_mean, bn_invstd, gamma, beta, plane_sums}, stream);
}

}  // extern "C"
