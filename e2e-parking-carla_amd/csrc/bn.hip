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
#include "common.h"

namespace e2ep {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2 };

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == ACT_RELU) return fmaxf(z, 0.f);
  if (act == ACT_SWISH) return z / (1.f + expf(-z));
  return z;
}
// d act / dz
__device__ __forceinline__ float act_bwd(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_SWISH) {
    const float s = 1.f / (1.f + expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// partial sums over a slice of the (n, hw) extent of channel c: grid (C, splits)
__global__ void __launch_bounds__(256) k_bn_stats(const float *__restrict__ x, int N, int C,
                                                  int HW, int splits, long long per,
                                                  double *__restrict__ part) {
  const int c = blockIdx.x, sp = blockIdx.y;
  const int tot = N * HW;
  const int beg = sp * (int)per, end = min(tot, beg + (int)per);
  double s = 0.0, q = 0.0;
  if ((HW & 3) == 0) {
    // vectorised: slices never straddle an image when per % 4 == 0 and HW % 4 == 0
    for (int i = beg + threadIdx.x * 4; i < end; i += 1024) {
      const int n = i / HW, p = i - n * HW;
      const float4 v = *reinterpret_cast<const float4 *>(x + ((size_t)n * C + c) * HW + p);
      s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
      q += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
  } else {
    for (int i = beg + threadIdx.x; i < end; i += 256) {
      const int n = i / HW, p = i - n * HW;
      const double v = x[((size_t)n * C + c) * HW + p];
      s += v;
      q += v * v;
    }
  }
  __shared__ double rs[4], rq[4];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((long long)c * splits + sp) * 2 + 0] = (rs[0] + rs[1]) + (rs[2] + rs[3]);
    part[((long long)c * splits + sp) * 2 + 1] = (rq[0] + rq[1]) + (rq[2] + rq[3]);
  }
}

// mean / invstd per channel; running-stat update (momentum m): r = (1-m) r + m * stat
__global__ void k_bn_finalize(const double *__restrict__ part, int C, int splits, long long cnt,
                              float eps, float momentum, float *__restrict__ running_mean,
                              float *__restrict__ running_var, float *__restrict__ mean,
                              float *__restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int k = 0; k < splits; ++k) {
    s += part[((long long)c * splits + k) * 2 + 0];
    q += part[((long long)c * splits + k) * 2 + 1];
  }
  const double mu = s / (double)cnt;
  double var = q / (double)cnt - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) {
    const double unb = cnt > 1 ? var * (double)cnt / (double)(cnt - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mu);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
}

// eval-mode statistics from the running buffers
__global__ void k_bn_eval_stats(const float *__restrict__ rm, const float *__restrict__ rv, int C,
                                float eps, float *__restrict__ mean, float *__restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
}

// y = act(gamma * (x - mean) * invstd + beta); grid covers N*C*HW/4 float4s (HW % 4 == 0)
// or scalars otherwise.
__global__ void __launch_bounds__(256) k_bn_apply(const float *__restrict__ x,
                                                  const float *__restrict__ mean,
                                                  const float *__restrict__ invstd,
                                                  const float *__restrict__ gamma,
                                                  const float *__restrict__ beta,
                                                  const float *__restrict__ res, int C, int HW,
                                                  int act, float *__restrict__ y) {
  const int q = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (q >= HW) return;
  const int c = blockIdx.y % C;
  const size_t i = (size_t)blockIdx.y * HW + q;
  if ((HW & 3) == 0) {
    const float sc = invstd[c] * (gamma ? gamma[c] : 1.f);
    const float sh = (beta ? beta[c] : 0.f) - mean[c] * sc;
    float4 v = *reinterpret_cast<const float4 *>(x + i);
    float4 r = res ? *reinterpret_cast<const float4 *>(res + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    v.x = act_fwd(v.x * sc + sh + r.x, act);
    v.y = act_fwd(v.y * sc + sh + r.y, act);
    v.z = act_fwd(v.z * sc + sh + r.z, act);
    v.w = act_fwd(v.w * sc + sh + r.w, act);
    *reinterpret_cast<float4 *>(y + i) = v;
  } else {
    for (int j = 0; j < 4 && q + j < HW; ++j) {
      const float sc = invstd[c] * (gamma ? gamma[c] : 1.f);
      const float sh = (beta ? beta[c] : 0.f) - mean[c] * sc;
      y[i + j] = act_fwd(x[i + j] * sc + sh + (res ? res[i + j] : 0.f), act);
    }
  }
}

// backward reduction: per channel, dz = dy * act'(z);  sums of dz and dz * xhat (fp64)
__global__ void __launch_bounds__(256) k_bn_bwd_reduce(
    const float *__restrict__ x, const float *__restrict__ dy, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ res, int N, int C, int HW,
    int splits, int act, double *__restrict__ part) {
  const int c = blockIdx.x, sp = blockIdx.y;
  const int tot = N * HW;
  const int per = (tot + splits - 1) / splits;
  const int beg = sp * per, end = min(tot, beg + per);
  const float mu = mean[c], is = invstd[c];
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  double s = 0.0, q = 0.0;
  for (int i = beg + threadIdx.x; i < end; i += 256) {
    const int n = i / HW, p = i - n * HW;
    const size_t off = ((size_t)n * C + c) * HW + p;
    const float xh = (x[off] - mu) * is;
    const float dz = dy[off] * act_bwd(xh * g + b + (res ? res[off] : 0.f), act);
    s += dz;
    q += (double)dz * xh;
  }
  __shared__ double rs[4], rq[4];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((long long)c * splits + sp) * 2 + 0] = (rs[0] + rs[1]) + (rs[2] + rs[3]);
    part[((long long)c * splits + sp) * 2 + 1] = (rq[0] + rq[1]) + (rq[2] + rq[3]);
  }
}

// dbeta[c] = sum dz, dgamma[c] = sum dz*xhat  (fixed-order combine of the slices)
__global__ void k_bn_bwd_finalize(const double *__restrict__ part, int C, int splits,
                                  float *__restrict__ dgamma, float *__restrict__ dbeta,
                                  double *__restrict__ sums) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int k = 0; k < splits; ++k) {
    s += part[((long long)c * splits + k) * 2 + 0];
    q += part[((long long)c * splits + k) * 2 + 1];
  }
  sums[2 * c] = s;
  sums[2 * c + 1] = q;
  if (dbeta) dbeta[c] = (float)s;
  if (dgamma) dgamma[c] = (float)q;
}

// dx = gamma * invstd * (dz - (sum_dz + xhat * sum_dzxhat) / M)        (train)
// dx = gamma * invstd * dz                                              (eval: train == 0)
__global__ void __launch_bounds__(256) k_bn_bwd_apply(
    const float *__restrict__ x, const float *__restrict__ dy, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ res, const double *__restrict__ sums,
    int C, int HW, long long cnt, int act, int train, float *__restrict__ dx,
    float *__restrict__ dres) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= HW) return;
  const int c = blockIdx.y % C;
  const size_t i = (size_t)blockIdx.y * HW + q;
  const float mu = mean[c], is = invstd[c];
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  const float xh = (x[i] - mu) * is;
  const float dz = dy[i] * act_bwd(xh * g + b + (res ? res[i] : 0.f), act);
  if (dres) dres[i] = dz;
  float v = dz;
  if (train) {
    const float ms = (float)(sums[2 * c] / (double)cnt);
    const float mq = (float)(sums[2 * c + 1] / (double)cnt);
    v = dz - (ms + xh * mq);
  }
  if (dx) dx[i] = g * is * v;
}

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
  // enough workgroups to fill the chip (~1024) with >= 4096 elements each
  long long want = (1024 + C - 1) / C;
  long long cap = per_channel / 4096;
  long long s = want < cap ? want : cap;
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  return (int)s;
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

size_t e2ep_bn_workspace(int N, int C, int H, int W) {
  const int sp = bn_splits((long long)N * H * W, C);
  return (size_t)C * sp * 2 * sizeof(double) + (size_t)C * 2 * sizeof(double);
}

int e2ep_bn_fwd(const float *x, const float *gamma, const float *beta, const float *res,
                float *running_mean, float *running_var, int N, int C, int H, int W, int train,
                float momentum, float eps, int act, float *mean, float *invstd, float *y,
                void *workspace, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && N * C <= 65535 &&
                   (long long)N * H * W < (1LL << 31), E2EP_EINVAL, "e2ep_bn_fwd: bad shape");
  E2EP_REQUIRE(act >= 0 && act <= 2, E2EP_EINVAL, "e2ep_bn_fwd: act must be 0/1/2");
  hipStream_t s = as_stream(stream);
  const int HW = H * W;
  const long long per = (long long)N * HW;
  if (train) {
    int sp = bn_splits(per, C);
    long long pp = (per + sp - 1) / sp;
    if ((HW & 3) == 0 && (pp & 3)) {  // keep vector slices aligned to whole float4s
      pp = (pp + 3) & ~3LL;
      sp = (int)((per + pp - 1) / pp);
    }
    double *part = static_cast<double *>(workspace);
    hipLaunchKernelGGL(k_bn_stats, dim3(C, sp), dim3(256), 0, s, x, N, C, HW, sp, pp, part);
    hipLaunchKernelGGL(k_bn_finalize, dim3(cdiv(C, 64)), dim3(64), 0, s, part, C, sp, per, eps,
                       momentum, running_mean, running_var, mean, invstd);
  } else {
    E2EP_REQUIRE(running_mean && running_var, E2EP_EINVAL, "e2ep_bn_fwd: eval needs running stats");
    hipLaunchKernelGGL(k_bn_eval_stats, dim3(cdiv(C, 64)), dim3(64), 0, s, running_mean, running_var,
                       C, eps, mean, invstd);
  }
  hipLaunchKernelGGL(k_bn_apply, dim3(cdiv(cdiv(HW, 4), 256), N * C), dim3(256), 0, s, x, mean,
                     invstd, gamma, beta, res, C, HW, act, y);
  return launch_status("e2ep_bn_fwd");
}

int e2ep_bn_bwd(const float *x, const float *dy, const float *mean, const float *invstd,
                const float *gamma, const float *beta, const float *res, int N, int C, int H, int W,
                int train, int act, float *dx, float *dgamma, float *dbeta, float *dres,
                void *workspace, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && N * C <= 65535 &&
                   (long long)N * H * W < (1LL << 31), E2EP_EINVAL, "e2ep_bn_bwd: bad shape");
  hipStream_t s = as_stream(stream);
  const int HW = H * W;
  const long long per = (long long)N * HW;
  const int sp = bn_splits(per, C);
  double *part = static_cast<double *>(workspace);
  double *sums = part + (size_t)C * sp * 2;
  hipLaunchKernelGGL(k_bn_bwd_reduce, dim3(C, sp), dim3(256), 0, s, x, dy, mean, invstd, gamma, beta,
                     res, N, C, HW, sp, act, part);
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(cdiv(C, 64)), dim3(64), 0, s, part, C, sp, dgamma, dbeta,
                     sums);
  if (dx || dres)
    hipLaunchKernelGGL(k_bn_bwd_apply, dim3(cdiv(HW, 256), N * C), dim3(256), 0, s, x, dy, mean,
                       invstd, gamma, beta, res, sums, C, HW, per, act, train, dx, dres);
  return launch_status("e2ep_bn_bwd");
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
