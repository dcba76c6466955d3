// Pooling / gating kernels of the hot path, NCHW fp32, gfx950:
//   max-pool 3x3/2 pad 1 (torchvision ResNet maxpool, reference model/bev_encoder.py:17,30):
//     forward stores the winning tap (first maximum in scan order, PyTorch semantics),
//     backward gathers (no atomics);
//   global average pool per plane (ASPPPooling, squeeze-excitation squeeze);
//   squeeze-excitation gate y = x * sigmoid(a[n,c]) with its two gradients.
#include "common.h"

namespace e2ep {

__global__ void __launch_bounds__(256) k_maxpool_fwd(const float *__restrict__ x, int planes, int H,
                                                     int W, int P, int Q, float *__restrict__ y,
                                                     int8_t *__restrict__ arg) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)planes * P * Q;
  if (i >= total) return;
  const int ox = (int)(i % Q);
  const long long r = i / Q;
  const int oy = (int)(r % P);
  const long long pl = r / P;
  const float *xp = x + pl * H * W;
  // PyTorch max_pool2d: strictly-greater keeps the first maximum; a NaN always wins
  float best = -INFINITY;
  int bt = -1;
  for (int a = 0; a < 3; ++a) {
    const int iy = oy * 2 - 1 + a;
    if ((unsigned)iy >= (unsigned)H) continue;
    for (int b = 0; b < 3; ++b) {
      const int ix = ox * 2 - 1 + b;
      if ((unsigned)ix >= (unsigned)W) continue;
      const float v = xp[iy * W + ix];
      if (bt < 0) bt = a * 3 + b;
      if (v > best || isnan(v)) {
        best = v;
        bt = a * 3 + b;
      }
    }
  }
  y[i] = best;
  arg[i] = (int8_t)bt;
}

__global__ void __launch_bounds__(256) k_maxpool_bwd(const float *__restrict__ gy,
                                                     const int8_t *__restrict__ arg, int planes,
                                                     int H, int W, int P, int Q,
                                                     float *__restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)planes * H * W;
  if (i >= total) return;
  const int ix = (int)(i % W);
  const long long r = i / W;
  const int iy = (int)(r % H);
  const long long pl = r / H;
  float s = 0.f;
  // outputs covering (iy, ix): oy*2-1 <= iy <= oy*2+1
  const int oy_lo = max(0, (iy + 1 - 2 + 1) / 2), oy_hi = min(P - 1, (iy + 1) / 2);
  const int ox_lo = max(0, (ix + 1 - 2 + 1) / 2), ox_hi = min(Q - 1, (ix + 1) / 2);
  for (int oy = oy_lo; oy <= oy_hi; ++oy)
    for (int ox = ox_lo; ox <= ox_hi; ++ox) {
      const int a = iy - (oy * 2 - 1), b = ix - (ox * 2 - 1);
      if (a < 0 || a > 2 || b < 0 || b > 2) continue;
      const long long o = (pl * P + oy) * Q + ox;
      if (arg[o] == a * 3 + b) s += gy[o];
    }
  dx[i] = s;
}

// mean over each plane: one wave per plane
__global__ void __launch_bounds__(256) k_avgpool_fwd(const float *__restrict__ x, int planes, int HW,
                                                     float *__restrict__ y) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pl >= planes) return;
  const float *p = x + (long long)pl * HW;
  float s = 0.f;
  for (int i = threadIdx.x & 63; i < HW; i += 64) s += p[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) y[pl] = s / (float)HW;
}

__global__ void k_avgpool_bwd(const float *__restrict__ gy, int planes, int HW,
                              float *__restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)planes * HW) return;
  dx[i] = gy[i / HW] / (float)HW;
}

// y = x * sigmoid(a[plane])
__global__ void k_se_gate_fwd(const float *__restrict__ x, const float *__restrict__ a, int HW,
                              long long total, float *__restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float s = sigmoid_f(a[i / HW]);
  y[i] = x[i] * s;
}

// dx = dy * sigmoid(a);  da[plane] = sum_hw dy * x * s * (1 - s)   (one wave per plane)
__global__ void __launch_bounds__(256) k_se_gate_bwd(const float *__restrict__ x,
                                                     const float *__restrict__ a,
                                                     const float *__restrict__ dy, int planes,
                                                     int HW, float *__restrict__ dx,
                                                     float *__restrict__ da) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pl >= planes) return;
  const float s = sigmoid_f(a[pl]);
  const long long base = (long long)pl * HW;
  float acc = 0.f;
  for (int i = threadIdx.x & 63; i < HW; i += 64) {
    const float g = dy[base + i];
    dx[base + i] = g * s;
    acc += g * x[base + i];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) da[pl] = acc * s * (1.f - s);
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_maxpool3s2_fwd(const float *x, int planes, int H, int W, float *y, int8_t *arg,
                        void *stream) {
  E2EP_REQUIRE(planes > 0 && H > 0 && W > 0, E2EP_EINVAL, "e2ep_maxpool3s2_fwd: bad shape");
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  const long long total = (long long)planes * P * Q;
  hipLaunchKernelGGL(k_maxpool_fwd, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), x, planes,
                     H, W, P, Q, y, arg);
  return launch_status("e2ep_maxpool3s2_fwd");
}

int e2ep_maxpool3s2_bwd(const float *gy, const int8_t *arg, int planes, int H, int W, float *dx,
                        void *stream) {
  E2EP_REQUIRE(planes > 0 && H > 0 && W > 0, E2EP_EINVAL, "e2ep_maxpool3s2_bwd: bad shape");
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  const long long total = (long long)planes * H * W;
  hipLaunchKernelGGL(k_maxpool_bwd, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), gy, arg,
                     planes, H, W, P, Q, dx);
  return launch_status("e2ep_maxpool3s2_bwd");
}

int e2ep_avgpool_fwd(const float *x, int planes, int HW, float *y, void *stream) {
  E2EP_REQUIRE(planes > 0 && HW > 0, E2EP_EINVAL, "e2ep_avgpool_fwd: bad shape");
  hipLaunchKernelGGL(k_avgpool_fwd, dim3(cdiv(planes, 4)), dim3(256), 0, as_stream(stream), x, planes,
                     HW, y);
  return launch_status("e2ep_avgpool_fwd");
}

int e2ep_avgpool_bwd(const float *gy, int planes, int HW, float *dx, void *stream) {
  E2EP_REQUIRE(planes > 0 && HW > 0, E2EP_EINVAL, "e2ep_avgpool_bwd: bad shape");
  hipLaunchKernelGGL(k_avgpool_bwd, dim3(cdiv((long long)planes * HW, 256)), dim3(256), 0,
                     as_stream(stream), gy, planes, HW, dx);
  return launch_status("e2ep_avgpool_bwd");
}

int e2ep_se_gate_fwd(const float *x, const float *a, int planes, int HW, float *y, void *stream) {
  E2EP_REQUIRE(planes > 0 && HW > 0, E2EP_EINVAL, "e2ep_se_gate_fwd: bad shape");
  const long long total = (long long)planes * HW;
  hipLaunchKernelGGL(k_se_gate_fwd, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), x, a, HW,
                     total, y);
  return launch_status("e2ep_se_gate_fwd");
}

int e2ep_se_gate_bwd(const float *x, const float *a, const float *dy, int planes, int HW, float *dx,
                     float *da, void *stream) {
  E2EP_REQUIRE(planes > 0 && HW > 0, E2EP_EINVAL, "e2ep_se_gate_bwd: bad shape");
  hipLaunchKernelGGL(k_se_gate_bwd, dim3(cdiv(planes, 4)), dim3(256), 0, as_stream(stream), x, a, dy,
                     planes, HW, dx, da);
  return launch_status("e2ep_se_gate_bwd");
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Softmax over the channel dim of NCHW (the depth distribution, reference
// model/bev_model.py:64 `depth.softmax(1)`): thread per pixel, channel loop, pixel-coalesced
// reads; backward dx = y (dy - sum_c y dy).  PyTorch runs this shape (C = 48, 32 x 32 planes)
// as a spatial softmax with few workgroups.
// ------------------------------------------------------------------------------------------
namespace e2ep {

// C <= SMC_MAX: a thread's channel column is loaded in one batch (all loads in flight) and
// kept in registers; 64-thread blocks spread the pixels over the whole chip.
constexpr int SMC_MAX = 64;
__global__ void __launch_bounds__(64) k_softmax_c_fwd(const float *__restrict__ x, int N, int C,
                                                      int HW, float *__restrict__ y) {
  const long long t = (long long)blockIdx.x * 64 + threadIdx.x;
  if (t >= (long long)N * HW) return;
  const long long n = t / HW, p = t - n * HW;
  const float *xs = x + n * C * HW + p;
  float *ys = y + n * C * HW + p;
  float v[SMC_MAX];
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c) v[c] = xs[(long long)min(c, C - 1) * HW];  // no branches
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c) v[c] = c < C ? v[c] : -INFINITY;
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c) m = fmaxf(m, v[c]);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c) {
    v[c] = expf(v[c] - m);  // padded channels: exp(-inf) = 0
    s += v[c];
  }
  const float r = 1.f / s;
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c)
    if (c < C) ys[(long long)c * HW] = v[c] * r;
}

__global__ void __launch_bounds__(64) k_softmax_c_bwd(const float *__restrict__ y,
                                                      const float *__restrict__ dy, int N, int C,
                                                      int HW, float *__restrict__ dx) {
  const long long t = (long long)blockIdx.x * 64 + threadIdx.x;
  if (t >= (long long)N * HW) return;
  const long long n = t / HW, p = t - n * HW;
  const long long base = n * C * HW + p;
  float yv[SMC_MAX], gv[SMC_MAX];
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c) {
    const float yy = y[base + (long long)min(c, C - 1) * HW];
    const float gg = dy[base + (long long)min(c, C - 1) * HW];
    yv[c] = c < C ? yy : 0.f;
    gv[c] = c < C ? gg : 0.f;
  }
  float d = 0.f;
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c) d = __builtin_fmaf(yv[c], gv[c], d);
#pragma unroll
  for (int c = 0; c < SMC_MAX; ++c)
    if (c < C) dx[base + (long long)c * HW] = yv[c] * (gv[c] - d);
}

}  // namespace e2ep

extern "C" {

int e2ep_softmax_c_fwd(const float *x, int N, int C, int HW, float *y, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && C <= e2ep::SMC_MAX && HW > 0, E2EP_EINVAL,
               "e2ep_softmax_c_fwd: bad shape (C <= %d)", e2ep::SMC_MAX);
  hipLaunchKernelGGL(e2ep::k_softmax_c_fwd, dim3(e2ep::cdiv((long long)N * HW, 64)), dim3(64), 0,
                     e2ep::as_stream(stream), x, N, C, HW, y);
  return e2ep::launch_status("e2ep_softmax_c_fwd");
}

int e2ep_softmax_c_bwd(const float *y, const float *dy, int N, int C, int HW, float *dx,
                       void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && C <= e2ep::SMC_MAX && HW > 0, E2EP_EINVAL,
               "e2ep_softmax_c_bwd: bad shape (C <= %d)", e2ep::SMC_MAX);
  hipLaunchKernelGGL(e2ep::k_softmax_c_bwd, dim3(e2ep::cdiv((long long)N * HW, 64)), dim3(64), 0,
                     e2ep::as_stream(stream), y, dy, N, C, HW, dx);
  return e2ep::launch_status("e2ep_softmax_c_bwd");
}

}  // extern "C"
