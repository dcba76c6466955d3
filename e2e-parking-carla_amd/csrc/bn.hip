// BatchNorm2d (training: batch statistics; eval: running statistics) fused with the
// following activation, forward and backward, NCHW fp32, for gfx950.
//
// Replaces torch BatchNorm2d + ReLU / swish pairs throughout the hot path
// (efficientnet-pytorch MBConv _bn0/_bn1/_bn2 + swish, reference
// model/bev_encoder.py:14-20 bn1/relu and torchvision BasicBlock, model/convolutions.py
// ASPP/DeepLab/UpsamplingConcat conv-BN-ReLU, model/segmentation_head.py:26-31).
//
// Statistics are accumulated in fp64 (sum, sum of squares) from fixed per-workgroup slices
// and combined in a fixed order: biased variance for normalisation, unbiased for the
// running-variance update (PyTorch semantics), deterministic run to run.
// Backward recomputes the pre-activation from x (no saved activation tensor).
#include <algorithm>

#include "common.h"

// Contraction only within one expression (a*b + c -> fma): the fp32 and bf16-storage
// instantiations of a kernel (E2EP_IO_*) then fuse the same operations and round alike —
// under the default cross-statement contraction hipcc may pick a different multiply to fuse
// in each instantiation (tests/test_bf16_store_gpu.py holds them bitwise equal).
#pragma clang fp contract(on)

namespace e2ep {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2 };

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == ACT_RELU) return fmaxf(z, 0.f);
  if (act == ACT_SWISH) return swish_f(z);
  return z;
}
// d act / dz
__device__ __forceinline__ float act_bwd(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_SWISH) {
    const float s = sigmoid_f(z);
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Channel-major iteration: channel c's data is N rows of HW floats at stride C*HW.  Kernels
// walk it as one sequence of N*HWv vectors (VEC = 4 when HW % 4 == 0, else 1); vector t is
// row n = t / HWv, column p = t % HWv.
template <int VEC>
struct Vec;
template <>
struct Vec<4> {
  typedef float4 T;
  static __device__ __forceinline__ float4 ld(const float *p) { return *reinterpret_cast<const float4 *>(p); }
  static __device__ __forceinline__ float4 ld(const bf16_t *p) { return ld4(p); }
  static __device__ __forceinline__ void st(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
  static __device__ __forceinline__ void st(bf16_t *p, float4 v) { st4(p, v); }
  static __device__ __forceinline__ float get(const float4 &v, int i) {
    return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
  }
  static __device__ __forceinline__ void set(float4 &v, int i, float f) {
    if (i == 0) v.x = f; else if (i == 1) v.y = f; else if (i == 2) v.z = f; else v.w = f;
  }
  static __device__ __forceinline__ float4 zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <>
struct Vec<1> {
  typedef float T;
  static __device__ __forceinline__ float ld(const float *p) { return *p; }
  static __device__ __forceinline__ float ld(const bf16_t *p) { return ld1(p); }
  static __device__ __forceinline__ void st(float *p, float v) { *p = v; }
  static __device__ __forceinline__ void st(bf16_t *p, float v) { st1(p, v); }
  static __device__ __forceinline__ float get(const float &v, int) { return v; }
  static __device__ __forceinline__ void set(float &v, int, float f) { v = f; }
  static __device__ __forceinline__ float zero() { return 0.f; }
};

// (n, p) = divmod(t, HWv) for t = t0, t0 + 256, t0 + 512, ... (a 256-thread block's strided
// walk over a channel's N x HWv vectors): one division up front, then a carry per step instead
// of an integer division (~25 instructions) per vector
struct PlaneWalk {
  int n, p, dq, dr, hw;
  __device__ __forceinline__ PlaneWalk(int t0, int hw_) : hw(hw_) {
    n = t0 / hw;
    p = t0 - n * hw;
    dq = 256 / hw;
    dr = 256 - dq * hw;
  }
  __device__ __forceinline__ void next() {
    p += dr;
    n += dq;
    if (p >= hw) {
      p -= hw;
      ++n;
    }
  }
};

// fixed-order fp64 block reduction of two values (256 threads); result valid in every thread
__device__ __forceinline__ void block_sum2(double &s, double &q) {
  __shared__ double rs[4], rq[4];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  __syncthreads();  // rs/rq may still be read by a previous call
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  s = (rs[0] + rs[1]) + (rs[2] + rs[3]);
  q = (rq[0] + rq[1]) + (rq[2] + rq[3]);
}

// sum of channel c's `splits` partial pairs, fixed order (thread k takes entries k, k+256, ...)
__device__ __forceinline__ void channel_partials(const double *__restrict__ part, int c,
                                                 int splits, double &s, double &q) {
  s = 0.0;
  q = 0.0;
  for (int k = threadIdx.x; k < splits; k += 256) {
    s += part[((long long)c * splits + k) * 2 + 0];
    q += part[((long long)c * splits + k) * 2 + 1];
  }
  block_sum2(s, q);
}

// drop-connect (efficientnet-pytorch, training): out = bn / keep * floor(keep + u[n])
__device__ __forceinline__ float dc_scale(const float *dc_rand, float keep, int n, float z) {
  return dc_rand ? __fmul_rn(__fdiv_rn(z, keep), floorf(__fadd_rn(keep, dc_rand[n]))) : z;
}

// partial sums over a slice of channel c: grid (C, splits); slice = `per` vectors
template <int VEC, typename TX = float>
__global__ void __launch_bounds__(256) k_bn_stats(const TX *__restrict__ x, int N, int C,
                                                  int HWv, int splits, int per,
                                                  double *__restrict__ part) {
  const int c = blockIdx.x, sp = blockIdx.y;
  const int tot = N * HWv;
  const int beg = sp * per, end = min(tot, beg + per);
  double s = 0.0, q = 0.0;
  PlaneWalk w(beg + (int)threadIdx.x, HWv);
  for (int t = beg + threadIdx.x; t < end; t += 256, w.next()) {
    const int n = w.n, p = w.p;
    const auto v = Vec<VEC>::ld(x + (((size_t)n * C + c) * HWv + p) * VEC);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const double d = Vec<VEC>::get(v, i);
      s += d;
      q += d * d;
    }
  }
  block_sum2(s, q);
  if (threadIdx.x == 0) {
    part[((long long)c * splits + sp) * 2 + 0] = s;
    part[((long long)c * splits + sp) * 2 + 1] = q;
  }
}

// y = act(dc(gamma * (x - mean) * invstd + beta) + res); grid (C, chunks of `per` vectors).
// Train: mean / invstd from the stats partials (fp64, biased variance); chunk 0 of each
// channel publishes them and updates the running stats (unbiased variance).  Eval: from the
// running stats.
template <int VEC>
__global__ void __launch_bounds__(256) k_bn_apply(
    const float *__restrict__ x, const double *__restrict__ part, int splits, long long cnt,
    float eps, float momentum, float *__restrict__ running_mean, float *__restrict__ running_var,
    float *__restrict__ mean_out, float *__restrict__ invstd_out, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ res,
    const float *__restrict__ dc_rand, float dc_keep, int N, int C, int HWv, int per, int act,
    float *__restrict__ y, const float *__restrict__ scale, const float *__restrict__ shift,
    int rev) {
  // rev: back-to-front sweep, starting on the rows the producing conv wrote last (e2ep_tune 33)
  const int c = rev ? C - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int j = rev ? (int)gridDim.y - 1 - (int)blockIdx.y : (int)blockIdx.y;
  float mu = 0.f, is = 0.f;
  if (scale) {
    // folded affine from e2ep_bn_finalize_part / e2ep_bn_stats (bn_finalize_channel: the same
    // sc / sh expressions as below)
  } else if (part) {
    double s, q;
    channel_partials(part, c, splits, s, q);
    const double m = s / (double)cnt;
    double var = q / (double)cnt - m * m;
    if (var < 0.0) var = 0.0;
    mu = (float)m;
    is = (float)(1.0 / sqrt(var + (double)eps));
    if (j == 0 && threadIdx.x == 0) {
      mean_out[c] = mu;
      invstd_out[c] = is;
      if (running_mean) {
        const double unb = cnt > 1 ? var * (double)cnt / (double)(cnt - 1) : var;
        running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * m);
        running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
      }
    }
  } else {
    mu = running_mean[c];
    is = (float)(1.0 / sqrt((double)running_var[c] + (double)eps));
    if (j == 0 && threadIdx.x == 0) {
      mean_out[c] = mu;
      invstd_out[c] = is;
    }
  }
  const float sc = scale ? scale[c] : is * (gamma ? gamma[c] : 1.f);
  const float sh = scale ? shift[c] : (beta ? beta[c] : 0.f) - mu * sc;
  const int tot = N * HWv;
  const int beg = j * per, end = min(tot, beg + per);
  PlaneWalk w(beg + (int)threadIdx.x, HWv);
  for (int t = beg + threadIdx.x; t < end; t += 256, w.next()) {
    const int n = w.n, p = w.p;
    const size_t off = (((size_t)n * C + c) * HWv + p) * VEC;
    auto v = Vec<VEC>::ld(x + off);
    const auto r = res ? Vec<VEC>::ld(res + off) : Vec<VEC>::zero();
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float z = dc_scale(dc_rand, dc_keep, n, Vec<VEC>::get(v, i) * sc + sh);
      Vec<VEC>::set(v, i, act_fwd(z + Vec<VEC>::get(r, i), act));
    }
    Vec<VEC>::st(y + off, v);
  }
}

// statistics only (for a consumer that applies the normalisation on load, e.g. the depthwise
// conv): mean / invstd, the folded scale / shift (sc = gamma * invstd, sh = beta - mean * sc,
// the same arithmetic as k_bn_apply) and the running-stat update of channel c; every thread
// of the block calls it (block-wide partial sum), thread 0 writes
__device__ __forceinline__ void bn_finalize_channel(
    int c, const double *__restrict__ part, int splits, long long cnt, float eps, float momentum,
    float *__restrict__ running_mean, float *__restrict__ running_var, float *__restrict__ mean_out,
    float *__restrict__ invstd_out, const float *__restrict__ gamma, const float *__restrict__ beta,
    float *__restrict__ scale, float *__restrict__ shift) {
  float mu, is;
  if (part) {
    double s, q;
    channel_partials(part, c, splits, s, q);
    if (threadIdx.x != 0) return;
    const double m = s / (double)cnt;
    double var = q / (double)cnt - m * m;
    if (var < 0.0) var = 0.0;
    mu = (float)m;
    is = (float)(1.0 / sqrt(var + (double)eps));
    if (running_mean) {
      const double unb = cnt > 1 ? var * (double)cnt / (double)(cnt - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * m);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
    }
  } else {
    if (threadIdx.x != 0) return;
    mu = running_mean[c];
    is = (float)(1.0 / sqrt((double)running_var[c] + (double)eps));
  }
  mean_out[c] = mu;
  invstd_out[c] = is;
  const float sc = is * (gamma ? gamma[c] : 1.f);
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - mu * sc;
}

// Finalize from a producer's tile-major partials (bnstats.h: part[(tile * C + c) * 2]):
// block = 8 channels x 128 tile groups (lane = tid % 8 -> channel c0 + lane, group = tid / 8):
// the 8 lanes of a group read one 128-B line per tile (channels c0 .. c0+7), group j sums tiles
// j, j + 128, ...; the group sums are added in group order through LDS, then the statistics
// as bn_finalize_channel computes them.  grid = C / 8.  Fixed order: deterministic.  (A
// two-level version that spread each channel's tiles over workgroups and handed the range
// sums to the last-arriving one spent 12.7 us per launch on the hand-off's uncached loads.)
constexpr int FT_CH = 8, FT_GROUPS = 128;  // 1024 threads: a few loads per thread, all in flight
__global__ void __launch_bounds__(FT_CH * FT_GROUPS) k_bn_finalize_tiles(
    const double *__restrict__ part, int tiles, int C, long long cnt, float eps, float momentum,
    float *__restrict__ running_mean, float *__restrict__ running_var,
    float *__restrict__ mean_out, float *__restrict__ invstd_out, const float *__restrict__ gamma,
    const float *__restrict__ beta, float *__restrict__ scale, float *__restrict__ shift) {
  __shared__ double rs[FT_GROUPS][FT_CH], rq[FT_GROUPS][FT_CH];
  const int lane = threadIdx.x % FT_CH, grp = threadIdx.x / FT_CH;
  const int c = blockIdx.x * FT_CH + lane;
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int k = grp; k < tiles; k += FT_GROUPS) {
      const double2 v = *reinterpret_cast<const double2 *>(part + ((size_t)k * C + c) * 2);
      s += v.x;
      q += v.y;
    }
  }
  rs[grp][lane] = s;
  rq[grp][lane] = q;
  __syncthreads();
  // fixed two-level order: groups j, j + 16, ..., j + 112 for j < 16, then the 16 in order
  double s2 = 0.0, q2 = 0.0;
  if (grp < 16) {
    s2 = rs[grp][lane];
    q2 = rq[grp][lane];
    for (int j = grp + 16; j < FT_GROUPS; j += 16) {
      s2 += rs[j][lane];
      q2 += rq[j][lane];
    }
  }
  __syncthreads();  // every thread: the first-level sums are read before they are overwritten
  if (grp < 16) {
    rs[grp][lane] = s2;
    rq[grp][lane] = q2;
  }
  __syncthreads();
  if (grp != 0 || c >= C) return;
  double S = rs[0][lane], Q = rq[0][lane];
  for (int j = 1; j < 16; ++j) {
    S += rs[j][lane];
    Q += rq[j][lane];
  }
  const double m = S / (double)cnt;
  double var = Q / (double)cnt - m * m;
  if (var < 0.0) var = 0.0;
  const float mu = (float)m;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) {
    const double unb = cnt > 1 ? var * (double)cnt / (double)(cnt - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * m);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
  mean_out[c] = mu;
  invstd_out[c] = is;
  const float sc = is * (gamma ? gamma[c] : 1.f);
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - mu * sc;
}

// Eval statistics of many BatchNorm layers in one launch (e2ep_bn_eval_multi): block = one
// table row {running_mean, running_var, gamma, beta, out, C, eps bits}; out = [mean | invstd |
// scale | shift] (4 x C), the arithmetic of bn_finalize_channel's eval branch.
__global__ void __launch_bounds__(256) k_bn_eval_multi(const long long *__restrict__ tab) {
  const long long *r = tab + 7LL * blockIdx.x;
  const float *rm = reinterpret_cast<const float *>(r[0]);
  const float *rv = reinterpret_cast<const float *>(r[1]);
  const float *gamma = reinterpret_cast<const float *>(r[2]);
  const float *beta = reinterpret_cast<const float *>(r[3]);
  float *out = reinterpret_cast<float *>(r[4]);
  const int C = (int)r[5];
  const float eps = __builtin_bit_cast(float, (int)r[6]);
  for (int c = threadIdx.x; c < C; c += 256) {
    const float mu = rm[c];
    const float is = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
    const float sc = is * (gamma ? gamma[c] : 1.f);
    out[c] = mu;
    out[C + c] = is;
    out[2 * C + c] = sc;
    out[3 * C + c] = (beta ? beta[c] : 0.f) - mu * sc;
  }
}

// grid (C): eval (part == null) or a separate finalize after k_bn_stats
__global__ void __launch_bounds__(256) k_bn_finalize(
    const double *__restrict__ part, int splits, long long cnt, float eps, float momentum,
    float *__restrict__ running_mean, float *__restrict__ running_var, float *__restrict__ mean_out,
    float *__restrict__ invstd_out, const float *__restrict__ gamma, const float *__restrict__ beta,
    float *__restrict__ scale, float *__restrict__ shift) {
  bn_finalize_channel(blockIdx.x, part, splits, cnt, eps, momentum, running_mean, running_var,
                      mean_out, invstd_out, gamma, beta, scale, shift);
}

// squeeze-excitation gate downstream of the activation (e2ep_bn_bwd gate_logit /
// gate_dpooled): the gradient at the activation output is dy * sigmoid(logit[n,c]) +
// dpooled[n,c] / HW (the SE op's dx, se.hip k_se_dx, formed here instead of stored)
struct BnGate {
  const float *logit, *dpooled;
  float inv_hw;
  __device__ __forceinline__ bool on() const { return logit != nullptr; }
  __device__ __forceinline__ void coef(int n, int C, int c, float &s, float &d) const {
    const int i = n * C + c;
    s = sigmoid_f(logit[i]);
    d = dpooled[i] * inv_hw;
  }
};
template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T gate_dy(typename Vec<VEC>::T dv, const BnGate &gt,
                                                        int n, int C, int c) {
  if (gt.on()) {
    float s, d;
    gt.coef(n, C, c, s, d);
#pragma unroll
    for (int i = 0; i < VEC; ++i) Vec<VEC>::set(dv, i, Vec<VEC>::get(dv, i) * s + d);
  }
  return dv;
}

// backward pieces shared by reduce and apply: from x, dy (and res / drop-connect), returns
// xhat, dz (gradient at the activation input = dres) and dzb (gradient at the BN output)
template <int VEC>
struct BnBwdElem {
  float mu, is, g, b;
  const float *dc_rand;
  float keep;
  int act;
  __device__ __forceinline__ void operator()(float xv, float dyv, float rv, int n, float &xh,
                                             float &dz, float &dzb) const {
    xh = (xv - mu) * is;
    const float zb = xh * g + b;
    dz = dyv * act_bwd(dc_scale(dc_rand, keep, n, zb) + rv, act);
    dzb = dc_rand ? __fdiv_rn(__fmul_rn(dz, floorf(__fadd_rn(keep, dc_rand[n]))), keep) : dz;
  }
  // the same with the sample's drop-connect factor floor(keep + u[n]) loaded beforehand
  __device__ __forceinline__ void with_factor(float xv, float dyv, float rv, float dcf, float &xh,
                                              float &dz, float &dzb) const {
    xh = (xv - mu) * is;
    const float zb = xh * g + b;
    const float zs = dc_rand ? __fmul_rn(__fdiv_rn(zb, keep), dcf) : zb;
    dz = dyv * act_bwd(zs + rv, act);
    dzb = dc_rand ? __fdiv_rn(__fmul_rn(dz, dcf), keep) : dz;
  }
};

// per-vector sample factors of the single-launch kernels, loaded before the channel data:
// a per-element `dc_rand[n]` / gate read inside the element loop made hipcc wait vmcnt(0)
// (the counters are in order) behind every x / dy load, one round trip per vector (the
// single-launch backward ran at 1.7 TB/s, round 3)
template <int T, int R>
__device__ __forceinline__ void bns_factors(int tot, int HWv, int C, int c, const float *dc_rand,
                                            float keep, const BnGate *gt, float (&dcf)[R],
                                            float (&gs)[R], float (&gd)[R]) {
  int n[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    n[u] = min((int)threadIdx.x + u * T, tot - 1) / HWv;
    dcf[u] = 1.f;
    gs[u] = 1.f;
    gd[u] = 0.f;
  }
  // raw loads only (uniform branches); bns_factors_finish does the arithmetic once the
  // caller has issued its channel loads too, so every load of the block is in flight at once
  if (dc_rand) {
#pragma unroll
    for (int u = 0; u < R; ++u) dcf[u] = dc_rand[n[u]];
  }
  if (gt && gt->on()) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      gs[u] = gt->logit[n[u] * C + c];
      gd[u] = gt->dpooled[n[u] * C + c];
    }
  }
}
template <int R>
__device__ __forceinline__ void bns_factors_finish(const float *dc_rand, float keep,
                                                   const BnGate *gt, float (&dcf)[R],
                                                   float (&gs)[R], float (&gd)[R]) {
  if (dc_rand) {
#pragma unroll
    for (int u = 0; u < R; ++u) dcf[u] = floorf(__fadd_rn(keep, dcf[u]));
  }
  if (gt && gt->on()) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      gs[u] = sigmoid_f(gs[u]);  // = BnGate::coef
      gd[u] = gd[u] * gt->inv_hw;
    }
  }
}

// backward reduction: per channel sums of dzb and dzb * xhat (fp64); grid (C, splits)
template <int VEC, typename TX = float, typename TD = float>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce(
    const TX *__restrict__ x, const TD *__restrict__ dy, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ res,
    const float *__restrict__ dc_rand, float dc_keep, BnGate gt, int N, int C, int HWv,
    int splits, int per, int act, double *__restrict__ part, int rev) {
  // rev: walk the tensor back to front (blocks are dispatched x fastest, so the forward order
  // sweeps memory front to back; e2ep_tune key 33)
  const int c = rev ? C - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int sp = rev ? (int)gridDim.y - 1 - (int)blockIdx.y : (int)blockIdx.y;
  const int tot = N * HWv;
  const int beg = sp * per, end = min(tot, beg + per);
  const BnBwdElem<VEC> el{mean[c], invstd[c], gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f,
                          dc_rand, dc_keep, act};
  double s = 0.0, q = 0.0;
  PlaneWalk w(beg + (int)threadIdx.x, HWv);
  for (int t = beg + threadIdx.x; t < end; t += 256, w.next()) {
    const int n = w.n, p = w.p;
    const size_t off = (((size_t)n * C + c) * HWv + p) * VEC;
    const auto xv = Vec<VEC>::ld(x + off);
    const auto dv = gate_dy<VEC>(Vec<VEC>::ld(dy + off), gt, n, C, c);
    const auto rv = res ? Vec<VEC>::ld(res + off) : Vec<VEC>::zero();
    // a vector's VEC terms summed in fp32 first, then into the fp64 sums (one fp64 add per
    // vector and sum instead of an add, a multiply and two conversions per element)
    float s4 = 0.f, q4 = 0.f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float xh, dz, dzb;
      el(Vec<VEC>::get(xv, i), Vec<VEC>::get(dv, i), Vec<VEC>::get(rv, i), n, xh, dz, dzb);
      s4 += dzb;
      q4 = __builtin_fmaf(dzb, xh, q4);
    }
    s += s4;
    q += q4;
  }
  block_sum2(s, q);
  if (threadIdx.x == 0) {
    part[((long long)c * splits + sp) * 2 + 0] = s;
    part[((long long)c * splits + sp) * 2 + 1] = q;
  }
}

// dbeta[c] = sum dzb, dgamma[c] = sum dzb*xhat: only when no dx / dres is wanted
__global__ void __launch_bounds__(256) k_bn_bwd_finalize(const double *__restrict__ part,
                                                         int splits, float *__restrict__ dgamma,
                                                         float *__restrict__ dbeta) {
  const int c = blockIdx.x;
  double s, q;
  channel_partials(part, c, splits, s, q);
  if (threadIdx.x == 0) {
    if (dbeta) dbeta[c] = (float)s;
    if (dgamma) dgamma[c] = (float)q;
  }
}

// dres = dz;  dx = gamma * invstd * (dzb - (sum_dzb + xhat * sum_dzbxhat) / M)   (train)
//             dx = gamma * invstd * dzb                                          (eval)
// grid (C, chunks); chunk 0 of each channel writes dgamma / dbeta.
template <int VEC, typename TX = float, typename TD = float, typename TO = float>
__global__ void __launch_bounds__(256) k_bn_bwd_apply(
    const TX *__restrict__ x, const TD *__restrict__ dy, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ res,
    const float *__restrict__ dc_rand, float dc_keep, BnGate gt, const double *__restrict__ part,
    int splits, long long cnt, int N, int C, int HWv, int per, int act, int train,
    TO *__restrict__ dx, float *__restrict__ dres, float *__restrict__ dgamma,
    float *__restrict__ dbeta, const double *__restrict__ planes, int rev) {
  // rev: back-to-front sweep, so the apply pass starts on the rows the reduction (or the
  // producer) touched last, while they may still sit in the 256 MB MALL (e2ep_tune key 33)
  const int c = rev ? C - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int j = rev ? (int)gridDim.y - 1 - (int)blockIdx.y : (int)blockIdx.y;
  double s, q;
  if (planes) {  // e2ep_bn_bwd_planes: the sums from the SE pass's per-plane factors
    s = 0.0;
    q = 0.0;
    for (int n = threadIdx.x; n < N; n += 256) {
      float gs, gd;
      gt.coef(n, C, c, gs, gd);
      const double *a = planes + 4LL * ((long long)n * C + c);
      s += (double)gs * a[0] + (double)gd * a[1];
      q += (double)gs * a[2] + (double)gd * a[3];
    }
    block_sum2(s, q);
  } else {
    channel_partials(part, c, splits, s, q);
  }
  if (j == 0 && threadIdx.x == 0) {
    if (dbeta) dbeta[c] = (float)s;
    if (dgamma) dgamma[c] = (float)q;
  }
  const float ms = (float)(s / (double)cnt), mq = (float)(q / (double)cnt);
  const BnBwdElem<VEC> el{mean[c], invstd[c], gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f,
                          dc_rand, dc_keep, act};
  const float gis = el.g * el.is;
  const int tot = N * HWv;
  const int beg = j * per, end = min(tot, beg + per);
  PlaneWalk w(beg + (int)threadIdx.x, HWv);
  for (int t = beg + threadIdx.x; t < end; t += 256, w.next()) {
    const int n = w.n, p = w.p;
    const size_t off = (((size_t)n * C + c) * HWv + p) * VEC;
    const auto xv = Vec<VEC>::ld(x + off);
    const auto dv = gate_dy<VEC>(Vec<VEC>::ld(dy + off), gt, n, C, c);
    const auto rv = res ? Vec<VEC>::ld(res + off) : Vec<VEC>::zero();
    auto ox = Vec<VEC>::zero(), orr = Vec<VEC>::zero();
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float xh, dz, dzb;
      el(Vec<VEC>::get(xv, i), Vec<VEC>::get(dv, i), Vec<VEC>::get(rv, i), n, xh, dz, dzb);
      Vec<VEC>::set(orr, i, dz);
      Vec<VEC>::set(ox, i, gis * (train ? dzb - (ms + xh * mq) : dzb));
    }
    if (dres) Vec<VEC>::st(dres + off, orr);
    if (dx) Vec<VEC>::st(dx + off, ox);
  }
}

// ------------------------------------------------------------------------------------------
// Single-launch BatchNorm for channels of at most BNS_T * 4 * BNS_R = 8192 elements (N * H * W:
// the 16x16 EfficientNet stages and the BEV encoder's deepest layers): one 256-thread block per
// channel holds the channel in registers from
// the statistics to the normalisation, so forward is one launch and one read of x (instead of
// stats + apply / finalize), backward one launch and one read of x, dy (instead of reduce +
// apply).  Same fp64 statistics and element arithmetic as the split kernels above; the
// summation is in a fixed order (thread t takes vectors t, t + 1024, ...), so deterministic.
// ------------------------------------------------------------------------------------------
constexpr int BNS_T = 256, BNS_R = 8;
static int g_bn_small = 1;  // e2ep_bn_small(0) routes every shape to the split kernels (tests, A/B)
// largest channel (in float4 vectors) the single-launch kernels take, forward / backward
// (e2ep_bn_small_limits, A/B timing; at most BNS_R * BNS_T).  In the replayed C2 step, blocks
// of 1024 threads for channels up to 32768 elements measured 0.25 ms/step slower than the
// split kernels there (25.45 vs 25.19 ms, profiles/r02/session6/wgrad_target_bn_limits_ab.txt),
// so only the 256-thread shapes take the single launch.
static int g_bns_fwd_max = BNS_R * BNS_T, g_bns_bwd_max = BNS_R * BNS_T;
static bool bn_small_enabled() { return g_bn_small != 0; }

template <int T>
__device__ __forceinline__ void block_sum2_t(double &s, double &q) {
  constexpr int NW = T / 64;
  __shared__ double rs[NW], rq[NW];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  s = 0.0;
  q = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    s += rs[i];
    q += rq[i];
  }
}

// float offset of float4 vector t of channel c (row n = t / HWv)
__device__ __forceinline__ size_t bns_off(int t, int HWv, int C, int c) {
  const int n = t / HWv, p = t - n * HWv;
  return (((size_t)n * C + c) * HWv + p) * 4;
}

// train-mode forward; y == null: statistics only (scale / shift for an apply-on-load consumer)
template <int T, int R, typename TX = float>
__global__ void __launch_bounds__(T) k_bn_fwd_small(
    const TX *__restrict__ x, long long cnt, float eps, float momentum,
    float *__restrict__ running_mean, float *__restrict__ running_var, float *__restrict__ mean_out,
    float *__restrict__ invstd_out, const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ res, const float *__restrict__ dc_rand, float dc_keep, int N, int C,
    int HWv, int act, float *__restrict__ y, float *__restrict__ scale, float *__restrict__ shift) {
  const int c = blockIdx.x, tot = N * HWv;
  float dcf[R], gs[R], gd[R];
  if (y) bns_factors<T, R>(tot, HWv, C, c, dc_rand, dc_keep, nullptr, dcf, gs, gd);
  float4 v[R];
#pragma unroll
  for (int u = 0; u < R; ++u) v[u] = Vec<4>::ld(x + bns_off(min((int)threadIdx.x + u * T, tot - 1), HWv, C, c));
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int u = 0; u < R; ++u) {
    if ((int)threadIdx.x + u * T >= tot) break;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double d = Vec<4>::get(v[u], i);
      s += d;
      q += d * d;
    }
  }
  block_sum2_t<T>(s, q);
  const double m = s / (double)cnt;
  double var = q / (double)cnt - m * m;
  if (var < 0.0) var = 0.0;
  const float mu = (float)m, is = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = is * (gamma ? gamma[c] : 1.f);
  const float sh = (beta ? beta[c] : 0.f) - mu * sc;
  if (threadIdx.x == 0) {
    mean_out[c] = mu;
    invstd_out[c] = is;
    if (scale) {
      scale[c] = sc;
      shift[c] = sh;
    }
    if (running_mean) {
      const double unb = cnt > 1 ? var * (double)cnt / (double)(cnt - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * m);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
    }
  }
  if (!y) return;
  float4 rr[R];
#pragma unroll
  for (int u = 0; u < R; ++u)
    rr[u] = res ? Vec<4>::ld(res + bns_off(min((int)threadIdx.x + u * T, tot - 1), HWv, C, c))
                : Vec<4>::zero();
  bns_factors_finish<R>(dc_rand, dc_keep, nullptr, dcf, gs, gd);
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int t = threadIdx.x + u * T;
    if (t >= tot) break;
    const size_t off = bns_off(t, HWv, C, c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float zb = Vec<4>::get(v[u], i) * sc + sh;
      const float z = dc_rand ? __fmul_rn(__fdiv_rn(zb, dc_keep), dcf[u]) : zb;  // = dc_scale
      Vec<4>::set(v[u], i, act_fwd(z + Vec<4>::get(rr[u], i), act));
    }
    Vec<4>::st(y + off, v[u]);
  }
}

template <int T, int R, typename TX = float, typename TD = float, typename TO = float>
__global__ void __launch_bounds__(T) k_bn_bwd_small(
    const TX *__restrict__ x, const TD *__restrict__ dy, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ res,
    const float *__restrict__ dc_rand, float dc_keep, BnGate gt, long long cnt, int N, int C,
    int HWv, int act, int train, TO *__restrict__ dx, float *__restrict__ dres,
    float *__restrict__ dgamma, float *__restrict__ dbeta) {
  const int c = blockIdx.x, tot = N * HWv;
  const BnBwdElem<4> el{mean[c], invstd[c], gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f,
                        dc_rand, dc_keep, act};
  float dcf[R], gs[R], gd[R];
  bns_factors<T, R>(tot, HWv, C, c, dc_rand, dc_keep, &gt, dcf, gs, gd);
  float4 xv[R], dv[R], rv[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const size_t off = bns_off(min((int)threadIdx.x + u * T, tot - 1), HWv, C, c);
    xv[u] = Vec<4>::ld(x + off);
    dv[u] = Vec<4>::ld(dy + off);
    rv[u] = res ? Vec<4>::ld(res + off) : Vec<4>::zero();
  }
  bns_factors_finish<R>(dc_rand, dc_keep, &gt, dcf, gs, gd);
  // one pass of the element math (act derivative: an exp and a divide for swish) whose results
  // stay in registers for the apply below (the block holds one channel: registers are free)
  float xh[R][4], dz[R][4], dzb[R][4];
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int t = threadIdx.x + u * T;
    float s4 = 0.f, q4 = 0.f;  // fp32 over the vector, then fp64 (as k_bn_bwd_reduce)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      el.with_factor(Vec<4>::get(xv[u], i), Vec<4>::get(dv[u], i) * gs[u] + gd[u],
                     Vec<4>::get(rv[u], i), dcf[u], xh[u][i], dz[u][i], dzb[u][i]);
      s4 += dzb[u][i];
      q4 = __builtin_fmaf(dzb[u][i], xh[u][i], q4);
    }
    if (t < tot) {
      s += s4;
      q += q4;
    }
  }
  block_sum2_t<T>(s, q);
  if (threadIdx.x == 0) {
    if (dbeta) dbeta[c] = (float)s;
    if (dgamma) dgamma[c] = (float)q;
  }
  if (!dx && !dres) return;
  const float ms = (float)(s / (double)cnt), mq = (float)(q / (double)cnt);
  const float gis = el.g * el.is;
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int t = threadIdx.x + u * T;
    if (t >= tot) break;
    const size_t off = bns_off(t, HWv, C, c);
    float4 ox, orr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Vec<4>::set(orr, i, dz[u][i]);
      Vec<4>::set(ox, i, gis * (train ? dzb[u][i] - (ms + xh[u][i] * mq) : dzb[u][i]));
    }
    if (dres) Vec<4>::st(dres + off, orr);
    if (dx) Vec<4>::st(dx + off, ox);
  }
}

// vectors per thread of the single-launch kernels (R = 0: the channel is too large); 256-thread
// blocks, every block of a step resident at once
static int bns_r(int totv, int &threads) {
  threads = BNS_T;
  const int per = cdiv(totv, threads);
  if (per <= 1) return 1;
  if (per <= 2) return 2;
  if (per <= 4) return 4;
  if (per <= BNS_R) return 8;
  return 0;
}
#define BNS_LAUNCH(KERNEL, R, TH, ...) BNS_LAUNCH_T(KERNEL, , R, TH, __VA_ARGS__)
// TYPES: the kernel's storage-type template arguments after <threads, R> (", bf16_t, float, ..."
// or empty)
#define BNS_LAUNCH_T(KERNEL, TYPES, R, TH, ...)                                                   \
  do {                                                                                            \
    (void)(TH);                                                                                   \
    if (R == 1) hipLaunchKernelGGL((KERNEL<BNS_T, 1 TYPES>), dim3(C), dim3(BNS_T), 0, s, __VA_ARGS__);  \
    else if (R == 2 && g_tune[TUNE_BNS_WIDE_LO] == 2)                                             \
      hipLaunchKernelGGL((KERNEL<2 * BNS_T, 1 TYPES>), dim3(C), dim3(2 * BNS_T), 0, s, __VA_ARGS__); \
    else if (R == 2) hipLaunchKernelGGL((KERNEL<BNS_T, 2 TYPES>), dim3(C), dim3(BNS_T), 0, s, __VA_ARGS__); \
    else if (R == 4 && g_tune[TUNE_BNS_WIDE_LO] == 2)                                             \
      hipLaunchKernelGGL((KERNEL<2 * BNS_T, 2 TYPES>), dim3(C), dim3(2 * BNS_T), 0, s, __VA_ARGS__); \
    else if (R == 4) hipLaunchKernelGGL((KERNEL<BNS_T, 4 TYPES>), dim3(C), dim3(BNS_T), 0, s, __VA_ARGS__); \
    else if (g_tune[TUNE_BNS_WIDE] == 2)                                                         \
      hipLaunchKernelGGL((KERNEL<2 * BNS_T, 4 TYPES>), dim3(C), dim3(2 * BNS_T), 0, s, __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<BNS_T, 8 TYPES>), dim3(C), dim3(BNS_T), 0, s, __VA_ARGS__);   \
  } while (0)
// (e2ep_tune key 25 = 2: channels that need 8 float4 per thread at 256 threads run 512-thread
// blocks of 4 per thread instead: half the registers per thread, twice the waves per channel;
// key 26 = 2 does the same for the 2- and 4-vector cases)

// elementwise activation forward/backward (for activations not fused into a BN)
__global__ void k_act_fwd(const float *__restrict__ x, long long n, int act, float *__restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = act_fwd(x[i], act);
}
__global__ void k_act_bwd(const float *__restrict__ x, const float *__restrict__ dy, long long n,
                          int act, float *__restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = dy[i] * act_bwd(x[i], act);
}

static int bn_splits(long long per_channel, int C) {
  // enough workgroups to fill the chip (e2ep_tune key 0) with >= key-1 elements each
  long long want = (g_tune[TUNE_BN_SPLIT_TARGET] + C - 1) / C;
  long long cap = per_channel / g_tune[TUNE_BN_SPLIT_MIN];
  long long s = want < cap ? want : cap;
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  return (int)s;
}

// vectors per apply workgroup (4 per thread)
#define APPLY_PER (g_tune[TUNE_BN_APPLY_PER])

// sweep direction of the split BN passes (e2ep_tune key 33 = 1 + mask): mask bit 0 backward
// apply back to front, bit 1 backward reduction back to front, bit 2 forward apply back to front
static int bn_rev_apply() { return ((g_tune[TUNE_BN_ORDER] - 1) >> 0) & 1; }
static int bn_rev_reduce() { return ((g_tune[TUNE_BN_ORDER] - 1) >> 1) & 1; }
static int bn_rev_fwd() { return ((g_tune[TUNE_BN_ORDER] - 1) >> 2) & 1; }

}  // namespace e2ep

using namespace e2ep;

extern "C" {

size_t e2ep_bn_workspace(int N, int C, int H, int W) {
  const int sp = bn_splits((long long)N * H * W, C);
  return (size_t)C * sp * 2 * sizeof(double);
}

int e2ep_bn_fwd(const float *x, const float *gamma, const float *beta, const float *res,
                const float *dc_rand, float dc_keep, float *running_mean, float *running_var,
                int N, int C, int H, int W, int train, float momentum, float eps, int act,
                float *mean, float *invstd, float *y, void *workspace, size_t workspace_bytes,
                void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && C <= 65535 && (long long)N * H * W < (1LL << 31),
               E2EP_EINVAL, "e2ep_bn_fwd: bad shape");
  E2EP_REQUIRE(!train || (workspace && workspace_bytes >= e2ep_bn_workspace(N, C, H, W)),
               E2EP_EINVAL, "%s: workspace %zu bytes < %zu (e2ep_bn_workspace)", "e2ep_bn_fwd",
               workspace_bytes, e2ep_bn_workspace(N, C, H, W));

  E2EP_REQUIRE(act >= 0 && act <= 2, E2EP_EINVAL, "e2ep_bn_fwd: act must be 0/1/2");
  E2EP_REQUIRE(train || (running_mean && running_var), E2EP_EINVAL,
               "e2ep_bn_fwd: eval needs running stats");
  E2EP_REQUIRE(!dc_rand || dc_keep > 0.f, E2EP_EINVAL, "e2ep_bn_fwd: drop-connect keep must be > 0");
  hipStream_t s = as_stream(stream);
  const int HW = H * W;
  const long long per_c = (long long)N * HW;
  const bool v4 = (HW & 3) == 0;
  const int HWv = v4 ? HW / 4 : HW;
  const int totv = N * HWv;
  const bool small_ok = bn_small_enabled();
  int th = 0;
  const int R = (train && v4 && small_ok && totv <= g_bns_fwd_max) ? bns_r(totv, th) : 0;
  if (R) {
    BNS_LAUNCH(k_bn_fwd_small, R, th, x, per_c, eps, momentum, running_mean, running_var, mean, invstd,
               gamma, beta, res, dc_rand, dc_keep, N, C, HWv, act, y, nullptr, nullptr);
    return launch_status("e2ep_bn_fwd");
  }
  double *part = nullptr;
  int sp = 1;
  if (train) {
    sp = bn_splits(per_c, C);
    const int per = cdiv(totv, sp);
    sp = cdiv(totv, per);
    part = static_cast<double *>(workspace);
    if (v4)
      hipLaunchKernelGGL(k_bn_stats<4>, dim3(C, sp), dim3(256), 0, s, x, N, C, HWv, sp, per, part);
    else
      hipLaunchKernelGGL(k_bn_stats<1>, dim3(C, sp), dim3(256), 0, s, x, N, C, HWv, sp, per, part);
  }
  const dim3 grid(C, cdiv(totv, APPLY_PER));
  if (v4)
    hipLaunchKernelGGL(k_bn_apply<4>, grid, dim3(256), 0, s, x, part, sp, per_c, eps, momentum,
                       running_mean, running_var, mean, invstd, gamma, beta, res, dc_rand, dc_keep,
                       N, C, HWv, APPLY_PER, act, y, nullptr, nullptr, bn_rev_fwd());
  else
    hipLaunchKernelGGL(k_bn_apply<1>, grid, dim3(256), 0, s, x, part, sp, per_c, eps, momentum,
                       running_mean, running_var, mean, invstd, gamma, beta, res, dc_rand, dc_keep,
                       N, C, HWv, APPLY_PER, act, y, nullptr, nullptr, bn_rev_fwd());
  return launch_status("e2ep_bn_fwd");
}

}  // extern "C"

template <typename TX>
static int bn_stats_impl(const TX *x, const float *gamma, const float *beta, float *running_mean,
                         float *running_var, int N, int C, int H, int W, int train, float momentum,
                         float eps, float *mean, float *invstd, float *scale, float *shift,
                         void *workspace, size_t workspace_bytes, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && C <= 65535 && (long long)N * H * W < (1LL << 31),
               E2EP_EINVAL, "e2ep_bn_stats: bad shape");
  E2EP_REQUIRE(!train || (workspace && workspace_bytes >= e2ep_bn_workspace(N, C, H, W)),
               E2EP_EINVAL, "%s: workspace %zu bytes < %zu (e2ep_bn_workspace)", "e2ep_bn_stats",
               workspace_bytes, e2ep_bn_workspace(N, C, H, W));

  E2EP_REQUIRE(train || (running_mean && running_var), E2EP_EINVAL,
               "e2ep_bn_stats: eval needs running stats");
  E2EP_REQUIRE(mean && invstd && scale && shift, E2EP_EINVAL, "e2ep_bn_stats: null output");
  hipStream_t s = as_stream(stream);
  const int HW = H * W;
  const long long per_c = (long long)N * HW;
  const bool v4 = (HW & 3) == 0;
  const int HWv = v4 ? HW / 4 : HW;
  const int totv = N * HWv;
  const bool small_ok = bn_small_enabled();
  int th = 0;
  const int R = (train && v4 && small_ok && totv <= g_bns_fwd_max) ? bns_r(totv, th) : 0;
  if (R) {
#define E2EP_BN_TYPES , TX
    BNS_LAUNCH_T(k_bn_fwd_small, E2EP_BN_TYPES, R, th, x, per_c, eps, momentum, running_mean, running_var,
                 mean, invstd, gamma, beta, nullptr, nullptr, 1.f, N, C, HWv, 0, nullptr, scale, shift);
#undef E2EP_BN_TYPES
    return launch_status("e2ep_bn_stats");
  }
  double *part = nullptr;
  int sp = 1;
  if (train) {
    sp = bn_splits(per_c, C);
    const int per = cdiv(totv, sp);
    sp = cdiv(totv, per);
    part = static_cast<double *>(workspace);
    if (v4)
      hipLaunchKernelGGL((k_bn_stats<4, TX>), dim3(C, sp), dim3(256), 0, s, x, N, C, HWv, sp, per, part);
    else
      hipLaunchKernelGGL((k_bn_stats<1, TX>), dim3(C, sp), dim3(256), 0, s, x, N, C, HWv, sp, per, part);
  }
  hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(256), 0, s, part, sp, per_c, eps, momentum,
                     running_mean, running_var, mean, invstd, gamma, beta, scale, shift);
  return launch_status("e2ep_bn_stats");
}

extern "C" {

int e2ep_bn_stats(const void *x, const float *gamma, const float *beta, float *running_mean,
                  float *running_var, int N, int C, int H, int W, int train, float momentum,
                  float eps, float *mean, float *invstd, float *scale, float *shift,
                  void *workspace, size_t workspace_bytes, void *stream, int io) {
  E2EP_REQUIRE(io == 0 || (io == E2EP_IO_X_BF16 && (H * W) % 4 == 0), E2EP_EINVAL,
               "e2ep_bn_stats: storage mask %d not supported (0 or X bf16, H*W %% 4 == 0)", io);
  if (io)
    return bn_stats_impl(static_cast<const bf16_t *>(x), gamma, beta, running_mean, running_var, N, C,
                         H, W, train, momentum, eps, mean, invstd, scale, shift, workspace,
                         workspace_bytes, stream);
  return bn_stats_impl(static_cast<const float *>(x), gamma, beta, running_mean, running_var, N, C, H,
                       W, train, momentum, eps, mean, invstd, scale, shift, workspace, workspace_bytes,
                       stream);
}

int e2ep_bn_fwd_split(int N, int C, int H, int W) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  const int HW = H * W;
  const bool v4 = (HW & 3) == 0;
  const int totv = N * (v4 ? HW / 4 : HW);
  int th = 0;
  return (v4 && bn_small_enabled() && totv <= g_bns_fwd_max && bns_r(totv, th)) ? 0 : 1;
}

size_t e2ep_bn_finalize_part_workspace(int C, int tiles) {
  (void)C;
  (void)tiles;
  return 0;  // one launch, no workspace (kept in the ABI for a future split plan)
}

int e2ep_bn_finalize_part(const double *part, int tiles, const float *gamma, const float *beta,
                          float *running_mean, float *running_var, int N, int C, int H, int W,
                          float momentum, float eps, float *mean, float *invstd, float *scale,
                          float *shift, void *workspace, size_t workspace_bytes, void *stream) {
  E2EP_REQUIRE(part && tiles > 0 && N > 0 && C > 0 && H > 0 && W > 0 && C <= 65535, E2EP_EINVAL,
               "e2ep_bn_finalize_part: bad arguments");
  E2EP_REQUIRE(mean && invstd && scale && shift, E2EP_EINVAL, "e2ep_bn_finalize_part: null output");
  E2EP_REQUIRE(!running_mean == !running_var, E2EP_EINVAL,
               "e2ep_bn_finalize_part: running_mean / running_var both or neither");
  (void)workspace;
  (void)workspace_bytes;
  hipLaunchKernelGGL(k_bn_finalize_tiles, dim3(cdiv(C, FT_CH)), dim3(FT_CH * FT_GROUPS), 0, as_stream(stream),
                     part, tiles, C, (long long)N * H * W, eps, momentum, running_mean, running_var,
                     mean, invstd, gamma, beta, scale, shift);
  return launch_status("e2ep_bn_finalize_part");
}

int e2ep_bn_apply(const float *x, const float *scale, const float *shift, const float *res,
                  const float *dc_rand, float dc_keep, int N, int C, int H, int W, int act,
                  float *y, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && C <= 65535 && (long long)N * H * W < (1LL << 31),
               E2EP_EINVAL, "e2ep_bn_apply: bad shape");
  E2EP_REQUIRE(x && y && scale && shift && act >= 0 && act <= 2, E2EP_EINVAL,
               "e2ep_bn_apply: bad arguments");
  E2EP_REQUIRE(!dc_rand || dc_keep > 0.f, E2EP_EINVAL, "e2ep_bn_apply: drop-connect keep must be > 0");
  const int HW = H * W;
  const bool v4 = (HW & 3) == 0 && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)res) & 15) == 0;
  const int HWv = v4 ? HW / 4 : HW;
  const int totv = N * HWv;
  const dim3 grid(C, cdiv(totv, APPLY_PER));
  hipStream_t s = as_stream(stream);
  if (v4)
    hipLaunchKernelGGL(k_bn_apply<4>, grid, dim3(256), 0, s, x, nullptr, 1, (long long)N * HW, 0.f,
                       0.f, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, res, dc_rand,
                       dc_keep, N, C, HWv, APPLY_PER, act, y, scale, shift, bn_rev_fwd());
  else
    hipLaunchKernelGGL(k_bn_apply<1>, grid, dim3(256), 0, s, x, nullptr, 1, (long long)N * HW, 0.f,
                       0.f, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, res, dc_rand,
                       dc_keep, N, C, HWv, APPLY_PER, act, y, scale, shift, bn_rev_fwd());
  return launch_status("e2ep_bn_apply");
}

}  // extern "C"

// storage types of (x, dy, dx) for an io mask (e2ep.h E2EP_IO_*): fp32, or the bf16
// combinations the step stores — the depthwise output's BN (_bn1: x and dx bf16, dy bf16 too
// when the squeeze-excitation output is stored bf16) and the expand output's BN (_bn0: the
// depthwise data gradient dy bf16)
enum BnIo {
  BNIO_F32 = 0,
  BNIO_XDX = E2EP_IO_X_BF16 | E2EP_IO_DX_BF16,
  BNIO_ALL = E2EP_IO_X_BF16 | E2EP_IO_DY_BF16 | E2EP_IO_DX_BF16,
  BNIO_DY = E2EP_IO_DY_BF16
};
static bool bn_io_ok(int io) {
  return io == BNIO_F32 || io == BNIO_XDX || io == BNIO_ALL || io == BNIO_DY;
}

template <typename TX, typename TD, typename TO>
static int bn_bwd_impl(const TX *x, const TD *dy, const float *mean, const float *invstd,
                       const float *gamma, const float *beta, const float *res,
                       const float *dc_rand, float dc_keep, const BnGate &gt, int N, int C, int H,
                       int W, int train, int act, TO *dx, float *dgamma, float *dbeta, float *dres,
                       void *workspace, size_t workspace_bytes, hipStream_t s) {
  const int HW = H * W;
  const long long per_c = (long long)N * HW;
  const bool v4 = (HW & 3) == 0;
  const int HWv = v4 ? HW / 4 : HW;
  const int totv = N * HWv;
  const bool small_ok = bn_small_enabled();
  int th = 0;
  const int R = (v4 && small_ok && totv <= g_bns_bwd_max) ? bns_r(totv, th) : 0;
  if (R) {
#define E2EP_BN_TYPES , TX, TD, TO
    BNS_LAUNCH_T(k_bn_bwd_small, E2EP_BN_TYPES, R, th, x, dy, mean, invstd, gamma, beta, res, dc_rand,
                 dc_keep, gt, per_c, N, C, HWv, act, train, dx, dres, dgamma, dbeta);
#undef E2EP_BN_TYPES
    return launch_status("e2ep_bn_bwd");
  }
  E2EP_REQUIRE(workspace && workspace_bytes >= e2ep_bn_workspace(N, C, H, W), E2EP_EINVAL,
               "e2ep_bn_bwd: workspace %zu bytes < %zu (e2ep_bn_workspace)", workspace_bytes,
               e2ep_bn_workspace(N, C, H, W));
  int sp = bn_splits(per_c, C);
  const int per = cdiv(totv, sp);
  sp = cdiv(totv, per);
  double *part = static_cast<double *>(workspace);
  if (v4)
    hipLaunchKernelGGL((k_bn_bwd_reduce<4, TX, TD>), dim3(C, sp), dim3(256), 0, s, x, dy, mean, invstd,
                       gamma, beta, res, dc_rand, dc_keep, gt, N, C, HWv, sp, per, act, part,
                       bn_rev_reduce());
  else
    hipLaunchKernelGGL((k_bn_bwd_reduce<1, TX, TD>), dim3(C, sp), dim3(256), 0, s, x, dy, mean, invstd,
                       gamma, beta, res, dc_rand, dc_keep, gt, N, C, HWv, sp, per, act, part,
                       bn_rev_reduce());
  if (dx || dres) {
    const dim3 grid(C, cdiv(totv, APPLY_PER));
    if (v4)
      hipLaunchKernelGGL((k_bn_bwd_apply<4, TX, TD, TO>), grid, dim3(256), 0, s, x, dy, mean, invstd,
                         gamma, beta, res, dc_rand, dc_keep, gt, part, sp, per_c, N, C, HWv, APPLY_PER,
                         act, train, dx, dres, dgamma, dbeta, nullptr, bn_rev_apply());
    else
      hipLaunchKernelGGL((k_bn_bwd_apply<1, TX, TD, TO>), grid, dim3(256), 0, s, x, dy, mean, invstd,
                         gamma, beta, res, dc_rand, dc_keep, gt, part, sp, per_c, N, C, HWv, APPLY_PER,
                         act, train, dx, dres, dgamma, dbeta, nullptr, bn_rev_apply());
  } else if (dgamma || dbeta) {
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(C), dim3(256), 0, s, part, sp, dgamma, dbeta);
  }
  return launch_status("e2ep_bn_bwd");
}

extern "C" {

int e2ep_bn_bwd(const void *x, const void *dy, const float *mean, const float *invstd,
                const float *gamma, const float *beta, const float *res, const float *dc_rand,
                float dc_keep, const float *gate_logit, const float *gate_dpooled, int N, int C,
                int H, int W, int train, int act, void *dx, float *dgamma, float *dbeta,
                float *dres, void *workspace, size_t workspace_bytes, void *stream, int io) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && C <= 65535 && (long long)N * H * W < (1LL << 31),
               E2EP_EINVAL, "e2ep_bn_bwd: bad shape");
  E2EP_REQUIRE(!gate_logit == !gate_dpooled, E2EP_EINVAL,
               "e2ep_bn_bwd: gate_logit / gate_dpooled both or neither");
  E2EP_REQUIRE(!dc_rand || dc_keep > 0.f, E2EP_EINVAL, "e2ep_bn_bwd: drop-connect keep must be > 0");
  E2EP_REQUIRE(bn_io_ok(io) && (io == 0 || (H * W) % 4 == 0), E2EP_EINVAL,
               "e2ep_bn_bwd: storage mask %d not supported (0, X|DX, X|DY|DX or DY bf16, "
               "H*W %% 4 == 0)", io);
  const BnGate gt{gate_logit, gate_dpooled, 1.f / (float)(H * W)};
  hipStream_t s = as_stream(stream);
  if (io == BNIO_XDX)
    return bn_bwd_impl(static_cast<const bf16_t *>(x), static_cast<const float *>(dy), mean, invstd,
                       gamma, beta, res, dc_rand, dc_keep, gt, N, C, H, W, train, act,
                       static_cast<bf16_t *>(dx), dgamma, dbeta, dres, workspace, workspace_bytes, s);
  if (io == BNIO_ALL)
    return bn_bwd_impl(static_cast<const bf16_t *>(x), static_cast<const bf16_t *>(dy), mean, invstd,
                       gamma, beta, res, dc_rand, dc_keep, gt, N, C, H, W, train, act,
                       static_cast<bf16_t *>(dx), dgamma, dbeta, dres, workspace, workspace_bytes, s);
  if (io == BNIO_DY)
    return bn_bwd_impl(static_cast<const float *>(x), static_cast<const bf16_t *>(dy), mean, invstd,
                       gamma, beta, res, dc_rand, dc_keep, gt, N, C, H, W, train, act,
                       static_cast<float *>(dx), dgamma, dbeta, dres, workspace, workspace_bytes, s);
  return bn_bwd_impl(static_cast<const float *>(x), static_cast<const float *>(dy), mean, invstd, gamma,
                     beta, res, dc_rand, dc_keep, gt, N, C, H, W, train, act, static_cast<float *>(dx),
                     dgamma, dbeta, dres, workspace, workspace_bytes, s);
}

int e2ep_bn_bwd_split(int N, int C, int H, int W) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  const int HW = H * W;
  const bool v4 = (HW & 3) == 0;
  const int totv = N * (v4 ? HW / 4 : HW);
  int th = 0;
  return (v4 && bn_small_enabled() && totv <= g_bns_bwd_max && bns_r(totv, th)) ? 0 : 1;
}

int e2ep_bn_bwd_planes(const void *x, const void *dy, const float *mean, const float *invstd,
                       const float *gamma, const float *beta, const float *gate_logit,
                       const float *gate_dpooled, const double *plane_sums, int N, int C, int H,
                       int W, int act, void *dx, float *dgamma, float *dbeta, void *stream, int io) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && C <= 65535 && (long long)N * H * W < (1LL << 31),
               E2EP_EINVAL, "e2ep_bn_bwd_planes: bad shape");
  E2EP_REQUIRE(x && dy && mean && invstd && gate_logit && gate_dpooled && plane_sums && dx,
               E2EP_EINVAL, "e2ep_bn_bwd_planes: null argument");
  E2EP_REQUIRE(act >= 0 && act <= 2, E2EP_EINVAL, "e2ep_bn_bwd_planes: act must be 0/1/2");
  E2EP_REQUIRE((io == BNIO_F32 || io == BNIO_XDX || io == BNIO_ALL) && (io == 0 || (H * W) % 4 == 0),
               E2EP_EINVAL, "e2ep_bn_bwd_planes: storage mask %d not supported (0, X|DX or X|DY|DX "
               "bf16, H*W %% 4 == 0)", io);
  const BnGate gt{gate_logit, gate_dpooled, 1.f / (float)(H * W)};
  const int HW = H * W;
  const long long per_c = (long long)N * HW;
  const bool v4 = (HW & 3) == 0;
  const int HWv = v4 ? HW / 4 : HW;
  const int totv = N * HWv;
  const dim3 grid(C, cdiv(totv, APPLY_PER));
  hipStream_t s = as_stream(stream);
  const float *dyf = static_cast<const float *>(dy);
  if (io == BNIO_ALL)
    hipLaunchKernelGGL((k_bn_bwd_apply<4, bf16_t, bf16_t, bf16_t>), grid, dim3(256), 0, s,
                       static_cast<const bf16_t *>(x), static_cast<const bf16_t *>(dy), mean, invstd,
                       gamma, beta, nullptr, nullptr, 1.f, gt, nullptr, 1, per_c, N, C, HWv, APPLY_PER,
                       act, 1, static_cast<bf16_t *>(dx), nullptr, dgamma, dbeta, plane_sums,
                       bn_rev_apply());
  else if (io == BNIO_XDX)
    hipLaunchKernelGGL((k_bn_bwd_apply<4, bf16_t, float, bf16_t>), grid, dim3(256), 0, s,
                       static_cast<const bf16_t *>(x), dyf, mean, invstd, gamma, beta, nullptr, nullptr,
                       1.f, gt, nullptr, 1, per_c, N, C, HWv, APPLY_PER, act, 1,
                       static_cast<bf16_t *>(dx), nullptr, dgamma, dbeta, plane_sums,
                       bn_rev_apply());
  else if (v4)
    hipLaunchKernelGGL(k_bn_bwd_apply<4>, grid, dim3(256), 0, s, static_cast<const float *>(x), dyf, mean,
                       invstd, gamma, beta, nullptr, nullptr, 1.f, gt, nullptr, 1, per_c, N, C, HWv,
                       APPLY_PER, act, 1, static_cast<float *>(dx), nullptr, dgamma, dbeta, plane_sums,
                       bn_rev_apply());
  else
    hipLaunchKernelGGL(k_bn_bwd_apply<1>, grid, dim3(256), 0, s, static_cast<const float *>(x), dyf, mean,
                       invstd, gamma, beta, nullptr, nullptr, 1.f, gt, nullptr, 1, per_c, N, C, HWv,
                       APPLY_PER, act, 1, static_cast<float *>(dx), nullptr, dgamma, dbeta, plane_sums,
                       bn_rev_apply());
  return launch_status("e2ep_bn_bwd_planes");
}

int e2ep_bn_eval_multi(const long long *table, int n, void *stream) {
  E2EP_REQUIRE(table && n > 0 && n <= 65535, E2EP_EINVAL, "e2ep_bn_eval_multi: bad table (n %d)", n);
  hipLaunchKernelGGL(k_bn_eval_multi, dim3(n), dim3(256), 0, as_stream(stream), table);
  return launch_status("e2ep_bn_eval_multi");
}

int e2ep_bn_small_limits(int fwd_max_vec, int bwd_max_vec) {
  if (fwd_max_vec >= 0) g_bns_fwd_max = std::min(fwd_max_vec, BNS_R * BNS_T);
  if (bwd_max_vec >= 0) g_bns_bwd_max = std::min(bwd_max_vec, BNS_R * BNS_T);
  return 0;
}

int e2ep_bn_small(int on) {
  const int prev = g_bn_small;
  if (on >= 0) g_bn_small = on ? 1 : 0;
  return prev;
}

int e2ep_act_fwd(const float *x, long long n, int act, float *y, void *stream) {
  E2EP_REQUIRE(n >= 0 && act >= 0 && act <= 2, E2EP_EINVAL, "e2ep_act_fwd: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_act_fwd, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), x, n, act, y);
  return launch_status("e2ep_act_fwd");
}

int e2ep_act_bwd(const float *x, const float *dy, long long n, int act, float *dx, void *stream) {
  E2EP_REQUIRE(n >= 0 && act >= 0 && act <= 2, E2EP_EINVAL, "e2ep_act_bwd: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_act_bwd, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), x, dy, n, act, dx);
  return launch_status("e2ep_act_bwd");
}

}  // extern "C"
