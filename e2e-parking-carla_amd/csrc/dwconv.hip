// Depthwise (groups == channels, multiplier 1) conv for EfficientNet's MBConv
// (efficientnet-pytorch 0.7.1 _depthwise_conv: k3/k5, stride 1/2, static SAME padding),
// forward, data gradient (gather, no atomics) and weight gradient (fixed-order split
// reduction), NCHW fp32, for gfx950.  Memory-bound: each kernel streams its input once.
#include "common.h"

namespace e2ep {

struct DwGeom {
  int N, C, H, W, K, P, Q, st, pt, pl;
};

// forward: one thread per output pixel; taps unrolled; branch-free guarded loads
template <int K, int ST>
__global__ void __launch_bounds__(256) k_dw_fwd(const float *__restrict__ x,
                                                const float *__restrict__ w, DwGeom g,
                                                float *__restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P * g.Q) return;
  const int nc = blockIdx.y;
  const int c = nc % g.C;
  const int oy = i / g.Q, ox = i - oy * g.Q;
  const int HW = g.H * g.W;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x + (size_t)nc * HW, 4LL * HW);
  const float *wp = w + c * K * K;
  const int y0 = oy * ST - g.pt, x0 = ox * ST - g.pl;
  float v[K * K];
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int iy = y0 + a;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int ix = x0 + b;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      v[a * K + b] = bload(rx, ok ? (iy * g.W + ix) * 4 : OOR);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < K * K; ++t) s += wp[t] * v[t];
  y[(size_t)nc * g.P * g.Q + i] = s;
}

// data gradient: one thread per input pixel, gather the outputs whose window covers it
// (branch-free: invalid taps read 0 through an out-of-range buffer offset)
template <int K, int ST>
__global__ void __launch_bounds__(256) k_dw_dgrad(const float *__restrict__ gy,
                                                  const float *__restrict__ w, DwGeom g,
                                                  float *__restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.H * g.W) return;
  const int nc = blockIdx.y;
  const int c = nc % g.C;
  const int iy = i / g.W, ix = i - iy * g.W;
  const int PQ = g.P * g.Q;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gy + (size_t)nc * PQ, 4LL * PQ);
  const float *wp = w + c * K * K;
  float v[K * K];
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int ny = iy + g.pt - a;
    const int oy = ny >= 0 ? ny / ST : -1;  // ST is a compile-time 1 or 2
    const bool oky = ny >= 0 && oy * ST == ny && oy < g.P;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int nx = ix + g.pl - b;
      const int ox = nx >= 0 ? nx / ST : -1;
      const bool ok = oky && nx >= 0 && ox * ST == nx && ox < g.Q;
      v[a * K + b] = bload(rg, ok ? (oy * g.Q + ox) * 4 : OOR);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < K * K; ++t) s += wp[t] * v[t];
  dx[(size_t)nc * g.H * g.W + i] = s;
}

// weight gradient partials: grid (C, splits); each slice of (n, oy, ox) accumulates K*K taps
template <int K, int ST>
__global__ void __launch_bounds__(256) k_dw_wgrad(const float *__restrict__ gy,
                                                  const float *__restrict__ x, DwGeom g,
                                                  int splits, float *__restrict__ part) {
  const int c = blockIdx.x, sp = blockIdx.y;
  const int PQ = g.P * g.Q;
  const int tot = g.N * PQ;
  const int per = (tot + splits - 1) / splits;
  const int beg = sp * per, end = min(tot, beg + per);
  float acc[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) acc[t] = 0.f;
  const int HW = g.H * g.W;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.C * HW);
  for (int i = beg + threadIdx.x; i < end; i += 256) {
    const int n = i / PQ;
    const int pix = i - n * PQ;
    const int oy = pix / g.Q, ox = pix - oy * g.Q;
    const float gv = gy[((size_t)n * g.C + c) * PQ + pix];
    const int xb = (n * g.C + c) * HW;
    const int y0 = oy * ST - g.pt, x0 = ox * ST - g.pl;
#pragma unroll
    for (int a = 0; a < K; ++a) {
      const int iy = y0 + a;
      const bool oky = (unsigned)iy < (unsigned)g.H;
#pragma unroll
      for (int b = 0; b < K; ++b) {
        const int ix = x0 + b;
        const bool ok = oky && (unsigned)ix < (unsigned)g.W;
        acc[a * K + b] += gv * bload(rx, ok ? (xb + iy * g.W + ix) * 4 : OOR);
      }
    }
  }
  __shared__ float red[4][K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float v = wave_sum(acc[t]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K) {
    const int t = threadIdx.x;
    part[((long long)c * splits + sp) * K * K + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  }
}

__global__ void k_dw_wgrad_finalize(const float *__restrict__ part, int C, int KK, int splits,
                                    float *__restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * KK) return;
  const int c = i / KK, t = i - c * KK;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[((long long)c * splits + k) * KK + t];
  dw[i] = s;
}

static int dw_splits(long long pixels, int C) {
  long long want = (1024 + C - 1) / C;
  long long cap = pixels / 2048;
  long long s = want < cap ? want : cap;
  return (int)(s < 1 ? 1 : (s > 128 ? 128 : s));
}

static DwGeom dw_geom(const int *d) {
  DwGeom g;
  g.N = d[0]; g.C = d[1]; g.H = d[2]; g.W = d[3]; g.K = d[4]; g.P = d[5]; g.Q = d[6];
  g.st = d[7]; g.pt = d[8]; g.pl = d[9];
  return g;
}

}  // namespace e2ep

using namespace e2ep;

#define DW_DISPATCH(KERNEL, GRID, ...)                                                        \
  do {                                                                                        \
    if (g.K == 3 && g.st == 1)                                                                \
      hipLaunchKernelGGL((KERNEL<3, 1>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else if (g.K == 3 && g.st == 2)                                                           \
      hipLaunchKernelGGL((KERNEL<3, 2>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else if (g.K == 5 && g.st == 1)                                                           \
      hipLaunchKernelGGL((KERNEL<5, 1>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else if (g.K == 5 && g.st == 2)                                                           \
      hipLaunchKernelGGL((KERNEL<5, 2>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else {                                                                                    \
      set_error("depthwise conv: kernel %d / stride %d unsupported (k 3|5, s 1|2)", g.K, g.st); \
      return E2EP_ERANGE;                                                                     \
    }                                                                                         \
  } while (0)

extern "C" {

// dims[10] = {N, C, H, W, K, P, Q, stride, pad_top, pad_left}
int e2ep_dwconv_fwd(const float *x, const float *w, const int *dims, float *y, void *stream) {
  DwGeom g = dw_geom(dims);
  E2EP_REQUIRE(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0, E2EP_EINVAL,
               "e2ep_dwconv_fwd: bad geometry");
  E2EP_REQUIRE(g.N * g.C <= 65535, E2EP_ERANGE, "e2ep_dwconv_fwd: N*C > 65535");
  DW_DISPATCH(k_dw_fwd, dim3(cdiv(g.P * g.Q, 256), g.N * g.C), x, w, g, y);
  return launch_status("e2ep_dwconv_fwd");
}

int e2ep_dwconv_dgrad(const float *gy, const float *w, const int *dims, float *dx, void *stream) {
  DwGeom g = dw_geom(dims);
  E2EP_REQUIRE(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0, E2EP_EINVAL,
               "e2ep_dwconv_dgrad: bad geometry");
  E2EP_REQUIRE(g.N * g.C <= 65535, E2EP_ERANGE, "e2ep_dwconv_dgrad: N*C > 65535");
  DW_DISPATCH(k_dw_dgrad, dim3(cdiv(g.H * g.W, 256), g.N * g.C), gy, w, g, dx);
  return launch_status("e2ep_dwconv_dgrad");
}

size_t e2ep_dwconv_wgrad_workspace(const int *dims) {
  DwGeom g = dw_geom(dims);
  return (size_t)g.C * dw_splits((long long)g.N * g.P * g.Q, g.C) * g.K * g.K * sizeof(float);
}

int e2ep_dwconv_wgrad(const float *gy, const float *x, const int *dims, void *workspace, float *dw,
                      void *stream) {
  DwGeom g = dw_geom(dims);
  E2EP_REQUIRE(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0, E2EP_EINVAL,
               "e2ep_dwconv_wgrad: bad geometry");
  const int sp = dw_splits((long long)g.N * g.P * g.Q, g.C);
  float *part = static_cast<float *>(workspace);
  DW_DISPATCH(k_dw_wgrad, dim3(g.C, sp), gy, x, g, sp, part);
  hipLaunchKernelGGL(k_dw_wgrad_finalize, dim3(cdiv(g.C * g.K * g.K, 256)), dim3(256), 0,
                     as_stream(stream), part, g.C, g.K * g.K, sp, dw);
  return launch_status("e2ep_dwconv_wgrad");
}

}  // extern "C"
