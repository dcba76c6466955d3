// Squeeze-and-excitation of efficientnet-pytorch's MBConv as one fused op, NCHW fp32, gfx950
// (reference: efficientnet-pytorch 0.7.1 MBConvBlock, used through model/cam_encoder.py:69-73):
//   pooled = mean_hw(x);  h = swish(W1 pooled + b1);  a = W2 h + b2;  y = x * sigmoid(a)
// Forward: squeeze (wave per plane), a per-sample MLP kernel (both 1x1 convs + swish on the
// 1x1 map), excite (float4 stream).  Backward: da (wave per plane), per-sample MLP backward
// (dh, dpooled), one weight-gradient kernel (sums over the batch in fixed order), and
// dx = dy * sigmoid(a) + dpooled / HW in a single stream — no separate avg-pool backward and
// no autograd add of the two input-gradient paths.
#include "common.h"

namespace e2ep {

constexpr int SE_MAXC = 4096, SE_MAXSQ = 256;

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + expf(-v)); }

// sum over one plane (HW floats, float4 when HW % 4 == 0) by one wave
__device__ __forceinline__ float plane_sum(const float *__restrict__ p, int HW, int lane) {
  float s = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2;
    for (int i = lane; i < HW4; i += 64) {
      const float4 v = reinterpret_cast<const float4 *>(p)[i];
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    for (int i = lane; i < HW; i += 64) s += p[i];
  }
  return wave_sum(s);
}

__global__ void __launch_bounds__(256) k_se_squeeze(const float *__restrict__ x, int planes,
                                                    int HW, float *__restrict__ pooled) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pl >= planes) return;
  const float s = plane_sum(x + (size_t)pl * HW, HW, threadIdx.x & 63);
  if ((threadIdx.x & 63) == 0) pooled[pl] = s / (float)HW;
}

// Block-wide sums of 16 per-thread values (fixed order: wave reduction, then waves 0..3).
// Valid in red[0..15] after the call.
__device__ __forceinline__ void block_sum16(float *v, float *red /* [4][16] */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = wave_sum(v[j]);
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < 16; ++j) red[wave * 16 + j] = v[j];
  __syncthreads();
  if (threadIdx.x < 16) {
    const int j = threadIdx.x;
    red[64 + j] = (red[j] + red[16 + j]) + (red[32 + j] + red[48 + j]);
  }
  __syncthreads();
}

// per sample n: hpre = W1 pooled + b1 (W1 [sq][C]);  a = W2 swish(hpre) + b2 (W2 [C][sq]).
// grid (N, C-chunks of 256).  Every block recomputes the hidden vector with all 256 threads
// (thread t takes channels t, t+256, ...; 16 hidden units at a time in registers, so its
// loads are independent and coalesced), then its chunk of a (thread per c).
__global__ void __launch_bounds__(256) k_se_mlp_fwd(const float *__restrict__ pooled,
                                                    const float *__restrict__ w1,
                                                    const float *__restrict__ b1,
                                                    const float *__restrict__ w2,
                                                    const float *__restrict__ b2, int C, int sq,
                                                    float *__restrict__ hpre,
                                                    float *__restrict__ a) {
  __shared__ float sh[SE_MAXSQ], red[80];
  const int n = blockIdx.x;
  const float *pn = pooled + (size_t)n * C;
  for (int k0 = 0; k0 < sq; k0 += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
      const float pv = pn[c];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (k0 + j < sq) v[j] += w1[(size_t)(k0 + j) * C + c] * pv;
    }
    block_sum16(v, red);
    if (threadIdx.x < 16 && k0 + threadIdx.x < sq) {
      const int k = k0 + threadIdx.x;
      const float z = red[64 + threadIdx.x] + (b1 ? b1[k] : 0.f);
      if (blockIdx.y == 0) hpre[(size_t)n * sq + k] = z;
      sh[k] = z * sigm(z);
    }
  }
  __syncthreads();
  // a[c] for this block's 256 channels: wave per channel, lanes along the W2 row (coalesced)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cend = min(C, (blockIdx.y + 1) * 256);
  for (int c = blockIdx.y * 256 + wave; c < cend; c += 4) {
    const float *wr = w2 + (size_t)c * sq;
    float s = 0.f;
    for (int k = lane; k < sq; k += 64) s += wr[k] * sh[k];
    s = wave_sum(s);
    if (lane == 0) a[(size_t)n * C + c] = s + (b2 ? b2[c] : 0.f);
  }
}

// y = x * sigmoid(a[plane]); float4 stream (HW % 4 == 0) or scalar
__global__ void __launch_bounds__(256) k_se_excite(const float *__restrict__ x,
                                                   const float *__restrict__ a, int HW,
                                                   long long nvec, int vec,
                                                   float *__restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  if (vec) {
    const int HW4 = HW >> 2;
    const float s = sigm(a[i / HW4]);
    float4 v = reinterpret_cast<const float4 *>(x)[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    reinterpret_cast<float4 *>(y)[i] = v;
  } else {
    y[i] = x[i] * sigm(a[i / HW]);
  }
}

// da[plane] = s (1 - s) sum_hw dy * x      (wave per plane)
__global__ void __launch_bounds__(256) k_se_da(const float *__restrict__ x,
                                               const float *__restrict__ dy,
                                               const float *__restrict__ a, int planes, int HW,
                                               float *__restrict__ da) {
  const int pl = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (pl >= planes) return;
  const float *xp = x + (size_t)pl * HW, *gp = dy + (size_t)pl * HW;
  float acc = 0.f;
  if ((HW & 3) == 0) {
    for (int i = lane; i < (HW >> 2); i += 64) {
      const float4 u = reinterpret_cast<const float4 *>(xp)[i];
      const float4 g = reinterpret_cast<const float4 *>(gp)[i];
      acc += (u.x * g.x + u.y * g.y) + (u.z * g.z + u.w * g.w);
    }
  } else {
    for (int i = lane; i < HW; i += 64) acc += xp[i] * gp[i];
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float s = sigm(a[pl]);
    da[pl] = acc * s * (1.f - s);
  }
}

// per sample n: dh = W2^T da;  dhpre = dh * swish'(hpre);  dpooled = W1^T dhpre.
// grid (N, C-chunks of 256); dh by all threads (channels strided over threads, 16 hidden
// units at a time), then the block's chunk of dpooled (thread per c, coalesced W1 columns).
__global__ void __launch_bounds__(256) k_se_mlp_bwd(const float *__restrict__ da,
                                                    const float *__restrict__ hpre,
                                                    const float *__restrict__ w1,
                                                    const float *__restrict__ w2, int C, int sq,
                                                    float *__restrict__ dhpre,
                                                    float *__restrict__ dpooled) {
  __shared__ float sd[SE_MAXSQ], red[80];
  const int n = blockIdx.x;
  const float *dn = da + (size_t)n * C;
  for (int k0 = 0; k0 < sq; k0 += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
      const float dv = dn[c];
      const float *wr = w2 + (size_t)c * sq + k0;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (k0 + j < sq) v[j] += wr[j] * dv;
    }
    block_sum16(v, red);
    if (threadIdx.x < 16 && k0 + threadIdx.x < sq) {
      const int k = k0 + threadIdx.x;
      const float z = hpre[(size_t)n * sq + k], sg = sigm(z);
      const float g = red[64 + threadIdx.x] * (sg * (1.f + z * (1.f - sg)));
      if (blockIdx.y == 0) dhpre[(size_t)n * sq + k] = g;
      sd[k] = g;
    }
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

int e2ep_se_fwd(const float *x, const float *w1, const float *b1, const float *w2,
                const float *b2, int N, int C, int HW, int sq, float *pooled, float *hpre,
                float *a, float *y, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0 && sq > 0, E2EP_EINVAL, "e2ep_se_fwd: bad shape");
  E2EP_REQUIRE(C <= SE_MAXC && sq <= SE_MAXSQ, E2EP_ERANGE, "e2ep_se_fwd: C %d > %d or sq %d > %d",
               C, SE_MAXC, sq, SE_MAXSQ);
  hipStream_t s = as_stream(stream);
  const int planes = N * C;
  hipLaunchKernelGGL(k_se_squeeze, dim3(cdiv(planes, 4)), dim3(256), 0, s, x, planes, HW, pooled);
  hipLaunchKernelGGL(k_se_mlp_fwd, dim3(N, cdiv(C, 256)), dim3(256), 0, s, pooled, w1, b1, w2, b2, C,
                     sq, hpre, a);
  const int vec = (HW & 3) == 0;
  const long long nvec = (long long)planes * HW / (vec ? 4 : 1);
  hipLaunchKernelGGL(k_se_excite, dim3(cdiv(nvec, 256)), dim3(256), 0, s, x, a, HW, nvec, vec, y);
  return launch_status("e2ep_se_fwd");
}

int e2ep_se_bwd(const float *x, const float *dy, const float *w1, const float *w2,
                const float *pooled, const float *hpre, const float *a, int N, int C, int HW,
                int sq, float *dx, float *dw1, float *db1, float *dw2, float *db2,
                float *workspace, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0 && sq > 0, E2EP_EINVAL, "e2ep_se_bwd: bad shape");
  E2EP_REQUIRE(C <= SE_MAXC && sq <= SE_MAXSQ, E2EP_ERANGE, "e2ep_se_bwd: C %d > %d or sq %d > %d",
               C, SE_MAXC, sq, SE_MAXSQ);
  hipStream_t s = as_stream(stream);
  const int planes = N * C;
  float *da = workspace, *dpooled = workspace + planes, *dhpre = workspace + 2 * planes;
  hipLaunchKernelGGL(k_se_da, dim3(cdiv(planes, 4)), dim3(256), 0, s, x, dy, a, planes, HW, da);
  hipLaunchKernelGGL(k_se_mlp_bwd, dim3(N, cdiv(C, 256)), dim3(256), 0, s, da, hpre, w1, w2, C, sq,
                     dhpre, dpooled);
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
