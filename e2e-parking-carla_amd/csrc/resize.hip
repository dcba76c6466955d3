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

__global__ void __launch_bounds__(256) k_resize_fwd(const float *__restrict__ x, int planes, int Hi,
                                                    int Wi, int Ho, int Wo, float sh, float sw,
                                                    float *__restrict__ y, long long y_pstride) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)planes * Ho * Wo;
  if (i >= total) return;
  const int ow = (int)(i % Wo);
  const long long r = i / Wo;
  const int oh = (int)(r % Ho);
  const long long pl = r / Ho;
  const Tap th = tap(oh, sh, Hi), tw = tap(ow, sw, Wi);
  const float *p = x + pl * Hi * Wi;
  const float v = th.l0 * (tw.l0 * p[th.i0 * Wi + tw.i0] + tw.l1 * p[th.i0 * Wi + tw.i1]) +
                  th.l1 * (tw.l0 * p[th.i1 * Wi + tw.i0] + tw.l1 * p[th.i1 * Wi + tw.i1]);
  y[pl * y_pstride + (long long)oh * Wo + ow] = v;
}

// backward pass 1 (along W): t[pl, oh, j] = sum_{ow} w(ow -> j) g[pl, oh, ow]
__global__ void __launch_bounds__(256) k_resize_bwd_w(const float *__restrict__ g, long long g_pstride,
                                                      int planes, int Ho, int Wo, int Wi, float sw,
                                                      float *__restrict__ t) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)planes * Ho * Wi;
  if (i >= total) return;
  const int j = (int)(i % Wi);
  const long long r = i / Wi;  // pl * Ho + oh
  const long long pl = r / Ho;
  const int oh = (int)(r - pl * Ho);
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
    if (tw.i0 == j) s += tw.l0 * gr[o];
    if (tw.i1 == j) s += tw.l1 * gr[o];
  }
  t[i] = s;
}

// backward pass 2 (along H): gx[pl, i, j] = sum_{oh} w(oh -> i) t[pl, oh, j]
__global__ void __launch_bounds__(256) k_resize_bwd_h(const float *__restrict__ t, int planes, int Ho,
                                                      int Hi, int Wi, float sh,
                                                      float *__restrict__ gx, int accumulate) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)planes * Hi * Wi;
  if (idx >= total) return;
  const int j = (int)(idx % Wi);
  const long long r = idx / Wi;
  const long long pl = r / Hi;
  const int i = (int)(r - pl * Hi);
  const float *tp = t + pl * Ho * Wi + j;
  const float inv = 1.f / sh;
  int lo = (int)floorf(((float)i - 0.5f) * inv - 0.5f) - 2;
  int hi = (int)ceilf(((float)i + 1.5f) * inv - 0.5f) + 2;
  lo = max(lo, 0);
  hi = min(hi, Ho - 1);
  float s = 0.f;
  for (int o = lo; o <= hi; ++o) {
    const Tap th = tap(o, sh, Hi);
    if (th.i0 == i) s += th.l0 * tp[(long long)o * Wi];
    if (th.i1 == i) s += th.l1 * tp[(long long)o * Wi];
  }
  gx[idx] = accumulate ? gx[idx] + s : s;
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_resize_fwd(const float *x, int planes, int Hi, int Wi, int Ho, int Wo, float scale_h,
                    float scale_w, float *y, long long y_pstride, void *stream) {
  E2EP_REQUIRE(planes > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, E2EP_EINVAL,
               "e2ep_resize_fwd: bad shape");
  const long long total = (long long)planes * Ho * Wo;
  hipLaunchKernelGGL(k_resize_fwd, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), x, planes,
                     Hi, Wi, Ho, Wo, scale_h, scale_w, y, y_pstride);
  return launch_status("e2ep_resize_fwd");
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
  float *t = static_cast<float *>(workspace);
  const long long n1 = (long long)planes * Ho * Wi;
  hipLaunchKernelGGL(k_resize_bwd_w, dim3(cdiv(n1, 256)), dim3(256), 0, s, g, g_pstride, planes, Ho,
                     Wo, Wi, scale_w, t);
  const long long n2 = (long long)planes * Hi * Wi;
  hipLaunchKernelGGL(k_resize_bwd_h, dim3(cdiv(n2, 256)), dim3(256), 0, s, t, planes, Ho, Hi, Wi,
                     scale_h, gx, accumulate);
  return launch_status("e2ep_resize_bwd");
}

}  // extern "C"
