// Bilinear resize (align_corners=False, PyTorch upsample_bilinear2d semantics), NCHW fp32,
// forward and a deterministic separable gather backward, for gfx950.
//
// Used by the BEV encoder's 200->256 resize (reference model/bev_encoder.py:24), the
// segmentation head's x2 upsamplings and 128->200 resize (model/segmentation_head.py:35-38),
// UpsamplingConcat (model/convolutions.py:197) and ASPP pooling broadcast (:238-240).
//
// Source coordinate of destination index o: src = max(scale * (o + 0.5) - 0.5, 0),
// i0 = (int)src, i1 = i0 + (i0 < In - 1), l1 = src - i0, l0 = 1 - l1, with scale = 1/sf when
// a scale factor is given and In/Out otherwise (both passed in as `scale`).
#include <stdint.h>
#include <stdlib.h>

#include "common.h"

namespace e2ep {

struct Tap {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ Tap tap(int o, float scale, int In) {
  float src = scale * ((float)o + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  Tap t;
  t.i0 = (int)src;
  t.i1 = t.i0 + (t.i0 < In - 1 ? 1 : 0);
  t.l1 = src - (float)t.i0;
  t.l0 = 1.f - t.l1;
  return t;
}

// grid (ceil(Ho*Wo/256), planes); plane pl = n*C + c reads x + n*x_nstride + c*Hi*Wi and
// writes y + n*y_nstride + c*Ho*Wo (so channel slices of bigger tensors need no copy)
__global__ void __launch_bounds__(256) k_resize_fwd(const float *__restrict__ x, int C,
                                                    long long x_nstride, int Hi, int Wi, int Ho,
                                                    int Wo, float sh, float sw, float *__restrict__ y,
                                                    long long y_nstride) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Ho * Wo) return;
  const int pl = blockIdx.y;
  const int n = pl / C, c = pl - n * C;
  const int oh = i / Wo, ow = i - oh * Wo;
  const Tap th = tap(oh, sh, Hi), tw = tap(ow, sw, Wi);
  const float *p = x + n * x_nstride + (long long)c * Hi * Wi;
  const float v = th.l0 * (tw.l0 * p[th.i0 * Wi + tw.i0] + tw.l1 * p[th.i0 * Wi + tw.i1]) +
                  th.l1 * (tw.l0 * p[th.i1 * Wi + tw.i0] + tw.l1 * p[th.i1 * Wi + tw.i1]);
  y[n * y_nstride + (long long)c * Ho * Wo + i] = v;
}

// Four outputs of one row per thread (Wo % 4 == 0, y 16-B aligned): one vertical tap and one
// float4 store per four outputs, a quarter of the workgroups.  One output per thread ran the
// BEV encoder's 200 -> 256 resize (65 planes x 8, 33.5 M outputs) at 1.5 TB/s of writes, 89 us
// (profiles/r06/step_sequence_fp32_final.txt).  Each output is the same expression as
// k_resize_fwd's (this file is built without contraction): bitwise equal.
__global__ void __launch_bounds__(256) k_resize_fwd4(const float *__restrict__ x, int C,
                                                     long long x_nstride, int Hi, int Wi, int Ho,
                                                     int Wo, float sh, float sw, float *__restrict__ y,
                                                     long long y_nstride) {
  const int i = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= Ho * Wo) return;
  const int pl = blockIdx.y;
  const int n = pl / C, c = pl - n * C;
  const int oh = i / Wo, ow = i - oh * Wo;
  const Tap th = tap(oh, sh, Hi);
  const float *p = x + n * x_nstride + (long long)c * Hi * Wi;
  const float *r0 = p + th.i0 * Wi, *r1 = p + th.i1 * Wi;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const Tap tw = tap(ow + j, sw, Wi);
    v[j] = th.l0 * (tw.l0 * r0[tw.i0] + tw.l1 * r0[tw.i1]) + th.l1 * (tw.l0 * r1[tw.i0] + tw.l1 * r1[tw.i1]);
  }
  *reinterpret_cast<float4 *>(y + n * y_nstride + (long long)c * Ho * Wo + i) =
      make_float4(v[0], v[1], v[2], v[3]);
}

// backward pass 1 (along W): t[pl, oh, j] = sum_{ow} w(ow -> j) g[pl, oh, ow]
__global__ void __launch_bounds__(256) k_resize_bwd_w(const float *__restrict__ g, long long g_pstride,
                                                      int planes, int Ho, int Wo, int Wi, float sw,
                                                      float *__restrict__ t) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Ho * Wi) return;
  const int pl = blockIdx.y;
  const int oh = i / Wi, j = i - oh * Wi;
  const float *gr = g + pl * g_pstride + (long long)oh * Wo;
  // outputs touching source j lie in a window around j / sw; recompute each tap exactly
  const float inv = 1.f / sw;
  int lo = (int)floorf(((float)j - 0.5f) * inv - 0.5f) - 2;
  int hi = (int)ceilf(((float)j + 1.5f) * inv - 0.5f) + 2;
  lo = max(lo, 0);
  hi = min(hi, Wo - 1);
  float s = 0.f;
  for (int o = lo; o <= hi; ++o) {
    const Tap tw = tap(o, sw, Wi);
    const float gv = gr[o];
    s += (tw.i0 == j ? tw.l0 : 0.f) * gv + (tw.i1 == j ? tw.l1 : 0.f) * gv;
  }
  t[(long long)pl * Ho * Wi + i] = s;
}

// backward pass 2 (along H): gx[pl, i, j] = sum_{oh} w(oh -> i) t[pl, oh, j]
__global__ void __launch_bounds__(256) k_resize_bwd_h(const float *__restrict__ t, int planes, int Ho,
                                                      int Hi, int Wi, float sh,
                                                      float *__restrict__ gx, int accumulate) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Hi * Wi) return;
  const int pl = blockIdx.y;
  const int i = q / Wi, j = q - i * Wi;
  const long long idx = (long long)pl * Hi * Wi + q;
  const float *tp = t + (long long)pl * Ho * Wi + j;
  const float inv = 1.f / sh;
  int lo = (int)floorf(((float)i - 0.5f) * inv - 0.5f) - 2;
  int hi = (int)ceilf(((float)i + 1.5f) * inv - 0.5f) + 2;
  lo = max(lo, 0);
  hi = min(hi, Ho - 1);
  float s = 0.f;
  for (int o = lo; o <= hi; ++o) {
    const Tap th = tap(o, sh, Hi);
    const float tv = tp[(long long)o * Wi];
    s += (th.i0 == i ? th.l0 : 0.f) * tv + (th.i1 == i ? th.l1 : 0.f) * tv;
  }
  gx[idx] = accumulate ? gx[idx] + s : s;
}

// Destinations o along one axis whose bilinear taps touch source index i with a non-zero
// weight have sources in (i - 1, i + 1): a run of at most ceil(2 / scale) consecutive
// indices, <= 4 for scale >= 0.5.  axis_taps evaluates the six candidates from one before
// the estimated run start exactly (the estimate is within one of the true start) and keeps
// the four-wide window starting at the first non-zero weight; returns its first index.
constexpr int RB_T = 4;
__device__ __forceinline__ int axis_taps(int i, float scale, int In, int Out, float *w) {
  const float inv = 1.f / scale;
  const int c = max(0, (int)ceilf(((float)i - 0.5f) * inv - 0.5f)) - 1;
  float v[RB_T + 2];
#pragma unroll
  for (int k = 0; k < RB_T + 2; ++k) {
    const int o = c + k;
    float x = 0.f;
    if (o >= 0 && o < Out) {
      const Tap t = tap(o, scale, In);
      x = (t.i0 == i ? t.l0 : 0.f) + (t.i1 == i ? t.l1 : 0.f);
    }
    v[k] = x;
  }
  const int sh = v[0] != 0.f ? 0 : v[1] != 0.f ? 1 : 2;
#pragma unroll
  for (int k = 0; k < RB_T; ++k) w[k] = sh == 0 ? v[k] : sh == 1 ? v[k + 1] : v[k + 2];
  return c + sh;
}

// Single-pass backward for scales >= 0.5 (<= 2x upsampling): gx[pl, i, j] =
// sum_{a,b < 4} wh[i][a] ww[j][b] g[pl, oh_i + a, ow_j + b].  A block owns an 8 x 32 source
// tile of one plane; the per-row and per-column tap tables are built once in LDS, then
// every thread does 16 cached loads — no intermediate through HBM, no per-pixel tap math.
constexpr int RB_TH = 8, RB_TW = 32;
__global__ void __launch_bounds__(256) k_resize_bwd_2d(const float *__restrict__ g,
                                                       long long g_pstride, int Ho, int Wo,
                                                       int Hi, int Wi, float sh, float sw,
                                                       float *__restrict__ gx, int accumulate) {
  __shared__ int s_oh[RB_TH], s_ow[RB_TW];
  __shared__ float s_wh[RB_TH][RB_T], s_ww[RB_TW][RB_T];
  const int tid = threadIdx.x;
  const int i0 = blockIdx.y * RB_TH, j0 = blockIdx.x * RB_TW;
  if (tid < RB_TH) {
    float w[RB_T];
    s_oh[tid] = axis_taps(min(i0 + tid, Hi - 1), sh, Hi, Ho, w);
#pragma unroll
    for (int k = 0; k < RB_T; ++k) s_wh[tid][k] = w[k];
  } else if (tid >= 64 && tid < 64 + RB_TW) {
    float w[RB_T];
    const int c = tid - 64;
    s_ow[c] = axis_taps(min(j0 + c, Wi - 1), sw, Wi, Wo, w);
#pragma unroll
    for (int k = 0; k < RB_T; ++k) s_ww[c][k] = w[k];
  }
  __syncthreads();
  const int r = tid / RB_TW, c = tid % RB_TW;
  const int i = i0 + r, j = j0 + c;
  if (i >= Hi || j >= Wi) return;
  const float *gp = g + blockIdx.z * g_pstride;
  const int ow = s_ow[c], oh = s_oh[r];
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < RB_T; ++a) {
    const float *gr = gp + (long long)min(oh + a, Ho - 1) * Wo;
    float t = 0.f;
#pragma unroll
    for (int b = 0; b < RB_T; ++b) t += s_ww[c][b] * gr[min(ow + b, Wo - 1)];
    s += s_wh[r][a] * t;
  }
  const long long idx = ((long long)blockIdx.z * Hi + i) * Wi + j;
  gx[idx] = accumulate ? gx[idx] + s : s;
}

// Single-pass backward writing the source gradient pillar-major, gxT[n][i * Wi + j][c]
// (channels last) — the layout the lift-splat backward gathers rows of (k_lss_bwd reads one
// 256-B channel row per pillar), so the BEV gradient needs no transpose.  Block = one source
// row i x 32 source columns x 64 channels of one image: thread (column tid % 32, channel
// group tid / 32) sums the 4 x 4 taps of 8 channels from the NCHW gradient (lanes along the
// gradient rows), the 32 x 64 tile is transposed through LDS and stored as 32 contiguous
// 256-B rows.  Same per-element arithmetic (and order) as k_resize_bwd_2d.
constexpr int RBC_C = 64;
__global__ void __launch_bounds__(256) k_resize_bwd_2d_cl(const float *__restrict__ g,
                                                          long long g_pstride, int C, int Ho,
                                                          int Wo, int Hi, int Wi, float sh,
                                                          float sw, float *__restrict__ gxT) {
  __shared__ int s_ow[RB_TW];
  __shared__ float s_ww[RB_TW][RB_T], s_wh[RB_T];
  __shared__ int s_oh;
  __shared__ float tile[RB_TW][RBC_C + 1];
  const int tid = threadIdx.x;
  const int i = blockIdx.y, j0 = blockIdx.x * RB_TW;
  const int cchunks = (C + RBC_C - 1) / RBC_C;
  const int n = blockIdx.z / cchunks, c0 = (blockIdx.z - n * cchunks) * RBC_C;
  if (tid == 0) {
    float w[RB_T];
    s_oh = axis_taps(i, sh, Hi, Ho, w);
#pragma unroll
    for (int k = 0; k < RB_T; ++k) s_wh[k] = w[k];
  } else if (tid >= 64 && tid < 64 + RB_TW) {
    float w[RB_T];
    const int c = tid - 64;
    s_ow[c] = axis_taps(min(j0 + c, Wi - 1), sw, Wi, Wo, w);
#pragma unroll
    for (int k = 0; k < RB_T; ++k) s_ww[c][k] = w[k];
  }
  __syncthreads();
  const int jj = tid % RB_TW, cg = tid / RB_TW;
  const int ow = s_ow[jj], oh = s_oh;
#pragma unroll
  for (int q = 0; q < RBC_C / 8; ++q) {
    const int cl = cg + 8 * q, c = c0 + cl;
    float s = 0.f;
    if (c < C) {
      const float *gp = g + ((long long)n * C + c) * g_pstride;
#pragma unroll
      for (int a = 0; a < RB_T; ++a) {
        const float *gr = gp + (long long)min(oh + a, Ho - 1) * Wo;
        float t = 0.f;
#pragma unroll
        for (int b = 0; b < RB_T; ++b) t += s_ww[jj][b] * gr[min(ow + b, Wo - 1)];
        s += s_wh[a] * t;
      }
    }
    tile[jj][cl] = s;
  }
  __syncthreads();
  for (int e = tid; e < RB_TW * RBC_C; e += 256) {
    const int r = e / RBC_C, cl = e - r * RBC_C;
    const int j = j0 + r, c = c0 + cl;
    if (j < Wi && c < C) gxT[((long long)n * Hi * Wi + (long long)i * Wi + j) * C + c] = tile[r][cl];
  }
}


// k_resize_bwd_2d_cl with the gradient window staged in LDS: a block (one source row, 32
// source columns, 32 channels) loads the 4 destination rows x (window width) x 32 channels it
// reads ONCE, coalesced along the row, then forms each output from LDS with the same tap
// weights and the same operation order as k_resize_bwd_2d_cl (bitwise equal: this file is
// built without contraction).  k_resize_bwd_2d_cl's 16 cached gathers per output x 8 channels
// per thread ran the BEV stem's 256 -> 200 backward (B = 8, 64 channels) at 1.4 TB/s, 153 us
// (profiles/r06/step_kernels_fp32_final.txt).
constexpr int RBL_C = 32, RBL_W = 72;  // channels per block, widest window (scale >= 0.5: <= 70)
__global__ void __launch_bounds__(256) k_resize_bwd_2d_cl_lds(const float *__restrict__ g,
                                                              long long g_pstride, int C, int Ho,
                                                              int Wo, int Hi, int Wi, float sh,
                                                              float sw, float *__restrict__ gxT) {
  __shared__ int s_ow[RB_TW];
  __shared__ float s_ww[RB_TW][RB_T], s_wh[RB_T];
  __shared__ int s_oh;
  __shared__ float gs[RB_T][RBL_C][RBL_W];
  __shared__ float tile[RB_TW][RBL_C + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = blockIdx.y, j0 = blockIdx.x * RB_TW;
  const int cchunks = (C + RBL_C - 1) / RBL_C;
  const int n = blockIdx.z / cchunks, c0 = (blockIdx.z - n * cchunks) * RBL_C;
  if (tid == 0) {
    float w[RB_T];
    s_oh = axis_taps(i, sh, Hi, Ho, w);
#pragma unroll
    for (int k = 0; k < RB_T; ++k) s_wh[k] = w[k];
  } else if (tid >= 64 && tid < 64 + RB_TW) {
    float w[RB_T];
    const int c = tid - 64;
    s_ow[c] = axis_taps(min(j0 + c, Wi - 1), sw, Wi, Wo, w);
#pragma unroll
    for (int k = 0; k < RB_T; ++k) s_ww[c][k] = w[k];
  }
  __syncthreads();
  const int oh = s_oh, owlo = s_ow[0];
  const int wneed = min(s_ow[RB_TW - 1] - owlo + RB_T, RBL_W);  // host: always fits
  // window rows (tap row a, channel): a wave per row, lanes along the row (clamped as the
  // gathers of k_resize_bwd_2d_cl clamp); every load of the wave's 32 rows issued before the
  // first LDS store (one row per round trip took the kernel to 413 us)
  constexpr int RPW = RB_T * RBL_C / 4;  // rows per wave
  for (int w0 = 0; w0 < wneed; w0 += 64) {
    const int w = w0 + lane;
    const int col = min(owlo + min(w, wneed - 1), Wo - 1);
    float v[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int row = wave + 4 * k, a = row / RBL_C, cl = row - a * RBL_C;
      v[k] = g[((long long)n * C + min(c0 + cl, C - 1)) * g_pstride + (long long)min(oh + a, Ho - 1) * Wo + col];
    }
    if (w < wneed) {
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int row = wave + 4 * k, a = row / RBL_C, cl = row - a * RBL_C;
        gs[a][cl][w] = v[k];
      }
    }
  }
  __syncthreads();
  const int jj = tid % RB_TW, cg = tid / RB_TW;
  const int ow = s_ow[jj] - owlo;
#pragma unroll
  for (int q = 0; q < RBL_C / 8; ++q) {
    const int cl = cg + 8 * q, c = c0 + cl;
    float s = 0.f;
    if (c < C) {
#pragma unroll
      for (int a = 0; a < RB_T; ++a) {
        float t = 0.f;
#pragma unroll
        for (int b = 0; b < RB_T; ++b) t += s_ww[jj][b] * gs[a][cl][ow + b];
        s += s_wh[a] * t;
      }
    }
    tile[jj][cl] = s;
  }
  __syncthreads();
  for (int e = tid; e < RB_TW * RBL_C; e += 256) {
    const int r = e / RBL_C, cl = e - r * RBL_C;
    const int j = j0 + r, c = c0 + cl;
    if (j < Wi && c < C) gxT[((long long)n * Hi * Wi + (long long)i * Wi + j) * C + c] = tile[r][cl];
  }
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_resize_fwd(const float *x, int N, int C, long long x_nstride, int Hi, int Wi, int Ho,
                    int Wo, float scale_h, float scale_w, float *y, long long y_nstride,
                    void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && N * C <= 65535,
               E2EP_EINVAL, "e2ep_resize_fwd: bad shape");
  const bool v4 = Wo % 4 == 0 && y_nstride % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(k_resize_fwd4, dim3(cdiv(Ho * Wo / 4, 256), N * C), dim3(256), 0,
                       as_stream(stream), x, C, x_nstride, Hi, Wi, Ho, Wo, scale_h, scale_w, y, y_nstride);
  else
    hipLaunchKernelGGL(k_resize_fwd, dim3(cdiv(Ho * Wo, 256), N * C), dim3(256), 0, as_stream(stream),
                       x, C, x_nstride, Hi, Wi, Ho, Wo, scale_h, scale_w, y, y_nstride);
  return launch_status("e2ep_resize_fwd");
}

int e2ep_resize_bwd_cl(const float *g, long long g_pstride, int N, int C, int Hi, int Wi, int Ho,
                       int Wo, float scale_h, float scale_w, float *gxT, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && Hi <= 65535 &&
                   (long long)N * cdiv(C, RBC_C) <= 65535 && scale_h >= 0.5f && scale_w >= 0.5f,
               E2EP_EINVAL, "e2ep_resize_bwd_cl: bad shape or scale < 0.5");
  // the LDS-window kernel: 32 source columns read at most ceil(32 / scale) + 6 <= 70 <= RBL_W
  // destination columns for scale >= 0.5 (checked above); E2EP_RESIZE_CL_GATHER=1 keeps the
  // gather kernel (A/B)
  static const bool gather = getenv("E2EP_RESIZE_CL_GATHER") && getenv("E2EP_RESIZE_CL_GATHER")[0] == '1';
  if (!gather && (long long)N * cdiv(C, RBL_C) <= 65535)
    hipLaunchKernelGGL(k_resize_bwd_2d_cl_lds, dim3(cdiv(Wi, RB_TW), Hi, N * cdiv(C, RBL_C)), dim3(256),
                       0, as_stream(stream), g, g_pstride, C, Ho, Wo, Hi, Wi, scale_h, scale_w, gxT);
  else
    hipLaunchKernelGGL(k_resize_bwd_2d_cl, dim3(cdiv(Wi, RB_TW), Hi, N * cdiv(C, RBC_C)), dim3(256),
                       0, as_stream(stream), g, g_pstride, C, Ho, Wo, Hi, Wi, scale_h, scale_w, gxT);
  return launch_status("e2ep_resize_bwd_cl");
}

size_t e2ep_resize_bwd_workspace(int planes, int Ho, int Wi) {
  return (size_t)planes * Ho * Wi * sizeof(float);
}

int e2ep_resize_bwd(const float *g, long long g_pstride, int planes, int Hi, int Wi, int Ho, int Wo,
                    float scale_h, float scale_w, float *gx, int accumulate, void *workspace,
                    void *stream) {
  E2EP_REQUIRE(planes > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, E2EP_EINVAL,
               "e2ep_resize_bwd: bad shape");
  hipStream_t s = as_stream(stream);
  if (scale_h >= 0.5f && scale_w >= 0.5f && planes <= 65535) {
    hipLaunchKernelGGL(k_resize_bwd_2d, dim3(cdiv(Wi, RB_TW), cdiv(Hi, RB_TH), planes), dim3(256),
                       0, s, g, g_pstride, Ho, Wo, Hi, Wi, scale_h, scale_w, gx, accumulate);
    return launch_status("e2ep_resize_bwd");
  }
  float *t = static_cast<float *>(workspace);
  hipLaunchKernelGGL(k_resize_bwd_w, dim3(cdiv(Ho * Wi, 256), planes), dim3(256), 0, s, g, g_pstride,
                     planes, Ho, Wo, Wi, scale_w, t);
  hipLaunchKernelGGL(k_resize_bwd_h, dim3(cdiv(Hi * Wi, 256), planes), dim3(256), 0, s, t, planes, Ho,
                     Hi, Wi, scale_h, gx, accumulate);
  return launch_status("e2ep_resize_bwd");
}

}  // extern "C"
