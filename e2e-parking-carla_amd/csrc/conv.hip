// NCHW fp32 convolution for gfx950 as implicit GEMM on the exact-f32 matrix cores
// (v_mfma_f32_32x32x2_f32: f32 in, f32 accumulate, bitwise an fmaf chain).
//
//   forward      y[n,co,p]  = sum_k W[co,k] * xcol[k,(n,p)]            M=Cout N=n*P*Q K=Cin*R*S
//   bwd-data     dx[n,ci,p] = sum_k W'[ci,k] * gcol[k,(n,p)]           M=Cin  N=n*H*W K=Cout*R*S
//   bwd-weight   dW[co,k]   = sum_(n,p) g[n,co,p] * xcol[k,(n,p)]      M=Cout N=Cin*R*S K=n*P*Q
//
// Every conv of the hot path uses these three kernels: BEV encoder (conv7x7/2 + ResNet-18
// layers 1-3), segmentation head, DeepLab/ASPP heads, UpsamplingConcat, EfficientNet 1x1
// expand/project/SE convs and the stem (reference model/bev_encoder.py:13-34,
// model/segmentation_head.py:19-31, model/convolutions.py:183-282, efficientnet-pytorch MBConv).
// Depthwise convs have their own memory-bound kernels (dwconv.hip).
//
// Tiling: 256 threads = 4 waves (2 x 2), block tile 64 (M) x 128 (N), K-step 16, each wave a
// 32 x 64 slab = two 32x32 accumulators sharing the A fragment.  A and B are staged
// global -> registers -> LDS (double buffered, one barrier per K-step).  The im2col gather is
// driven by a per-conv k-table (int4 {b_off, dh, dw, a_off}) built once on the device, so the
// inner loop has no integer division.  bwd-weight splits the pixel reduction over blocks and
// reduces the fp32 partial slabs in a fixed order: results are run-to-run deterministic.
#include "common.h"

namespace e2ep {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 128, BK = 16;
constexpr int PADA = 4, PADB = 4;

struct ConvGeom {
  int N;            // images
  int Cin, H, W;    // input
  int Cout, R, S;   // filter
  int P, Q;         // output spatial
  int sh, sw, ph, pw, dh, dw;
};

// ------------------------------------------------------------------------------------------
// k-tables
//   fwd / wgrad (gather from x): k=(ci,r,s): b_off = ci*H*W, dh = r*dh, dw = s*dw, a_off = k
//   dgrad       (gather from g): k=(co,r,s): b_off = co*P*Q, dh = r*dh, dw = s*dw,
//                                            a_off = co*Cin*R*S + r*S + s   (A row stride R*S)
// ------------------------------------------------------------------------------------------
__global__ void k_conv_table(ConvGeom g, int dgrad, int4 *__restrict__ tab, int Kg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Kg) return;
  const int RS = g.R * g.S;
  const int c = k / RS, rs = k - c * RS, r = rs / g.S, s = rs - r * g.S;
  int4 t;
  t.y = r * g.dh;
  t.z = s * g.dw;
  if (!dgrad) {
    t.x = c * g.H * g.W;
    t.w = k;
  } else {
    t.x = c * g.P * g.Q;
    t.w = c * g.Cin * RS + rs;
  }
  tab[k] = t;
}

// ------------------------------------------------------------------------------------------
// forward / bwd-data kernel
// ------------------------------------------------------------------------------------------
// MODE 0: forward (B gathered from x at output pixel (oh,ow): ih = oh*sh - ph + dh_k)
// MODE 1: bwd-data (B gathered from g at input pixel (ih,iw): oh = (ih + ph - dh_k) / sh)
template <int MODE, int ACT>
__global__ void __launch_bounds__(256, 2) k_conv_gemm(
    const float *__restrict__ A, int a_row_stride, const float *__restrict__ src,
    const int4 *__restrict__ tab, const float *__restrict__ bias, float *__restrict__ dst,
    ConvGeom g, int M, int Kg) {
  __shared__ float As[2][BK][BM + PADA];
  __shared__ float Bs[2][BK][BN + PADB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  // output-pixel geometry of this block's columns
  const int Hd = MODE == 0 ? g.P : g.H, Wd = MODE == 0 ? g.Q : g.W;  // dst spatial
  const int Hs = MODE == 0 ? g.H : g.P, Ws = MODE == 0 ? g.W : g.Q;  // src spatial
  const int Cs = MODE == 0 ? g.Cin : g.Cout;
  const int HWd = Hd * Wd;
  const long long Ntot = (long long)g.N * HWd;

  // this thread's B-load column
  const int bn = tid & (BN - 1);
  const int bk0 = tid >> 7;  // 0..1
  const long long ncol = (long long)n0 + bn;
  const bool col_ok = ncol < Ntot;
  int img = 0, od = 0;
  if (col_ok) {
    img = (int)(ncol / HWd);
    od = (int)(ncol - (long long)img * HWd);
  }
  const int oy = od / Wd, ox = od - oy * Wd;
  const float *sbase = src + (long long)img * Cs * Hs * Ws;
  // MODE 0: base coords in the source; MODE 1: numerators before subtracting dh_k
  const int y0 = MODE == 0 ? oy * g.sh - g.ph : oy + g.ph;
  const int x0 = MODE == 0 ? ox * g.sw - g.pw : ox + g.pw;

  // this thread's A-load coordinates
  const int am = tid & (BM - 1);
  const int ak0 = tid >> 6;  // 0..3
  const bool arow_ok = (m0 + am) < M;
  const float *abase = A + (long long)(m0 + am) * a_row_stride;

  float ra[4], rb[8];

  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + ak0 + 4 * j;
      float v = 0.f;
      if (arow_ok && k < Kg) v = abase[tab[k].w];
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + bk0 + 2 * j;
      float v = 0.f;
      if (col_ok && k < Kg) {
        const int4 t = tab[k];
        if (MODE == 0) {
          const int iy = y0 + t.y, ix = x0 + t.z;
          if ((unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws)
            v = sbase[t.x + iy * Ws + ix];
        } else {
          const int ny = y0 - t.y, nx = x0 - t.z;
          if (ny >= 0 && nx >= 0) {
            const int qy = ny / g.sh, qx = nx / g.sw;
            if (qy * g.sh == ny && qx * g.sw == nx && qy < Hs && qx < Ws)
              v = sbase[t.x + qy * Ws + qx];
          }
        }
      }
      rb[j] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) As[buf][ak0 + 4 * j][am] = ra[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) Bs[buf][bk0 + 2 * j][bn] = rb[j];
  };

  f32x16 acc0 = {0}, acc1 = {0};
  const int nk = (Kg + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_tiles((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[buf][kk + lk][32 * wm + li];
      const float b0 = Bs[buf][kk + lk][64 * wn + li];
      const float b1 = Bs[buf][kk + lk][64 * wn + 32 + li];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const long long n = (long long)n0 + 64 * wn + 32 * t + li;
    if (n >= Ntot) continue;
    const int im = (int)(n / HWd);
    const int p = (int)(n - (long long)im * HWd);
    float *dbase = dst + (long long)im * M * HWd + p;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
      if (m < M) {
        float v = t == 0 ? acc0[r] : acc1[r];
        if (bias) v += bias[m];
        if (ACT == 1) v = fmaxf(v, 0.f);
        dbase[(long long)m * HWd] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// bwd-weight: dW[co,k] = sum over pixels of g[n,co,p] * xcol[k,(n,p)]; split over pixels.
// Block tile 64 (co) x 128 (k), K-step = 16 pixels.  Partial slab per split.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 2) k_conv_wgrad(
    const float *__restrict__ gout, const float *__restrict__ x, const int4 *__restrict__ tab,
    float *__restrict__ part, ConvGeom g, int Kg, long long pix_per_split) {
  __shared__ float As[2][BK][BM + PADA];  // As[pixel][co]
  __shared__ float Bs[2][BK][BN + PADB];  // Bs[pixel][k]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int split = blockIdx.z;
  const int PQ = g.P * g.Q;
  const long long Ptot = (long long)g.N * PQ;
  const long long pbeg = (long long)split * pix_per_split;
  const long long pend = min(Ptot, pbeg + pix_per_split);

  // A loads: 64 co x 16 pixels; thread -> pixel = tid & 15, co = (tid >> 4) + 16 j
  const int ap = tid & 15, am0 = tid >> 4;
  // B loads: 16 pixels x 128 k; thread -> pixel = tid & 15, k = (tid >> 4) + 16 j
  const int bp = tid & 15, bkk0 = tid >> 4;
  int4 tk[8];
  bool kok[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = n0 + bkk0 + 16 * j;
    kok[j] = k < Kg;
    tk[j] = kok[j] ? tab[k] : make_int4(0, 0, 0, 0);
  }
  float ra[4], rb[8];

  auto load_tiles = [&](long long p0) {
    const long long p = p0 + ap;
    const bool pok = p < pend;
    int im = 0, od = 0;
    if (pok) {
      im = (int)(p / PQ);
      od = (int)(p - (long long)im * PQ);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = m0 + am0 + 16 * j;
      ra[j] = (pok && co < g.Cout) ? gout[((long long)im * g.Cout + co) * PQ + od] : 0.f;
    }
    const long long pb = p0 + bp;
    const bool pbok = pb < pend;
    int imb = 0, odb = 0;
    if (pbok) {
      imb = (int)(pb / PQ);
      odb = (int)(pb - (long long)imb * PQ);
    }
    const int oy = odb / g.Q, ox = odb - oy * g.Q;
    const int y0 = oy * g.sh - g.ph, x0 = ox * g.sw - g.pw;
    const float *xb = x + (long long)imb * g.Cin * g.H * g.W;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = 0.f;
      if (pbok && kok[j]) {
        const int iy = y0 + tk[j].y, ix = x0 + tk[j].z;
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          v = xb[tk[j].x + iy * g.W + ix];
      }
      rb[j] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) As[buf][ap][am0 + 16 * j] = ra[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) Bs[buf][bp][bkk0 + 16 * j] = rb[j];
  };

  f32x16 acc0 = {0}, acc1 = {0};
  const long long nk = (pend - pbeg + BK - 1) / BK;
  const int li = lane & 31, lk = lane >> 5;
  if (nk > 0) {
    load_tiles(pbeg);
    store_tiles(0);
  }
  __syncthreads();
  for (long long kt = 0; kt < nk; ++kt) {
    const int buf = (int)(kt & 1);
    if (kt + 1 < nk) load_tiles(pbeg + (kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[buf][kk + lk][32 * wm + li];
      const float b0 = Bs[buf][kk + lk][64 * wn + li];
      const float b1 = Bs[buf][kk + lk][64 * wn + 32 + li];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(buf ^ 1);
    __syncthreads();
  }
  float *pbase = part + (long long)split * g.Cout * Kg;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = n0 + 64 * wn + 32 * t + li;
    if (k >= Kg) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
      if (co < g.Cout) pbase[(long long)co * Kg + k] = t == 0 ? acc0[r] : acc1[r];
    }
  }
}

// fixed-order sum of the split slabs (+ optional accumulate into an existing gradient)
__global__ void k_reduce_splits(const float *__restrict__ part, int splits, long long n,
                                float *__restrict__ out, int accumulate) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = accumulate ? out[i] : 0.f;
  for (int k = 0; k < splits; ++k) s += part[(long long)k * n + i];
  out[i] = s;
}

// per-channel bias gradient: db[c] = sum over (n, p) of g[n, c, p]  (one block per channel)
__global__ void __launch_bounds__(256) k_bias_grad(const float *__restrict__ g, int N, int C,
                                                   int HW, float *__restrict__ db) {
  const int c = blockIdx.x;
  float s = 0.f;
  for (int n = 0; n < N; ++n) {
    const float *p = g + ((long long)n * C + c) * HW;
    for (int i = threadIdx.x; i < HW; i += 256) s += p[i];
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) db[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace e2ep

using namespace e2ep;

static ConvGeom make_geom(const int *d) {
  ConvGeom g;
  g.N = d[0]; g.Cin = d[1]; g.H = d[2]; g.W = d[3];
  g.Cout = d[4]; g.R = d[5]; g.S = d[6]; g.P = d[7]; g.Q = d[8];
  g.sh = d[9]; g.sw = d[10]; g.ph = d[11]; g.pw = d[12]; g.dh = d[13]; g.dw = d[14];
  return g;
}

static bool geom_ok(const ConvGeom &g) {
  return g.N > 0 && g.Cin > 0 && g.H > 0 && g.W > 0 && g.Cout > 0 && g.R > 0 && g.S > 0 &&
         g.P > 0 && g.Q > 0 && g.sh > 0 && g.sw > 0 && g.dh > 0 && g.dw > 0 && g.ph >= 0 &&
         g.pw >= 0;
}

extern "C" {

int e2ep_conv_table(const int *dims, int dgrad, void *table, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_table: bad geometry");
  const int Kg = (dgrad ? g.Cout : g.Cin) * g.R * g.S;
  hipLaunchKernelGGL(k_conv_table, dim3(cdiv(Kg, 256)), dim3(256), 0, as_stream(stream), g, dgrad,
                     static_cast<int4 *>(table), Kg);
  return launch_status("e2ep_conv_table");
}

int e2ep_conv_fwd(const float *x, const float *w, const float *bias, const void *table,
                  const int *dims, int act, float *y, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_fwd: bad geometry");
  E2EP_REQUIRE(act == 0 || act == 1, E2EP_EINVAL, "e2ep_conv_fwd: act must be 0 (none) or 1 (relu)");
  const int Kg = g.Cin * g.R * g.S;
  const long long Ncols = (long long)g.N * g.P * g.Q;
  dim3 grid(cdiv(Ncols, BN), cdiv(g.Cout, BM));
  const int4 *tab = static_cast<const int4 *>(table);
  if (act == 0)
    hipLaunchKernelGGL((k_conv_gemm<0, 0>), grid, dim3(256), 0, as_stream(stream), w, Kg, x, tab,
                       bias, y, g, g.Cout, Kg);
  else
    hipLaunchKernelGGL((k_conv_gemm<0, 1>), grid, dim3(256), 0, as_stream(stream), w, Kg, x, tab,
                       bias, y, g, g.Cout, Kg);
  return launch_status("e2ep_conv_fwd");
}

int e2ep_conv_dgrad(const float *gout, const float *w, const void *table, const int *dims,
                    float *dx, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_dgrad: bad geometry");
  const int Kg = g.Cout * g.R * g.S;
  const long long Ncols = (long long)g.N * g.H * g.W;
  dim3 grid(cdiv(Ncols, BN), cdiv(g.Cin, BM));
  hipLaunchKernelGGL((k_conv_gemm<1, 0>), grid, dim3(256), 0, as_stream(stream), w, g.R * g.S, gout,
                     static_cast<const int4 *>(table), (const float *)nullptr, dx, g, g.Cin, Kg);
  return launch_status("e2ep_conv_dgrad");
}

size_t e2ep_conv_wgrad_workspace(const int *dims, int splits) {
  ConvGeom g = make_geom(dims);
  return (size_t)splits * g.Cout * g.Cin * g.R * g.S * sizeof(float);
}

int e2ep_conv_wgrad(const float *gout, const float *x, const void *table, const int *dims,
                    int splits, void *workspace, float *dw, int accumulate, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g) && splits > 0, E2EP_EINVAL, "e2ep_conv_wgrad: bad geometry");
  const int Kg = g.Cin * g.R * g.S;
  const long long Ptot = (long long)g.N * g.P * g.Q;
  long long per = (Ptot + splits - 1) / splits;
  per = (per + BK - 1) / BK * BK;
  dim3 grid(cdiv(Kg, BN), cdiv(g.Cout, BM), splits);
  hipStream_t s = as_stream(stream);
  float *part = static_cast<float *>(workspace);
  hipLaunchKernelGGL(k_conv_wgrad, grid, dim3(256), 0, s, gout, x,
                     static_cast<const int4 *>(table), part, g, Kg, per);
  const long long n = (long long)g.Cout * Kg;
  hipLaunchKernelGGL(k_reduce_splits, dim3(cdiv(n, 256)), dim3(256), 0, s, part, splits, n, dw,
                     accumulate);
  return launch_status("e2ep_conv_wgrad");
}

int e2ep_bias_grad(const float *gout, int N, int C, int HW, float *db, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0, E2EP_EINVAL, "e2ep_bias_grad: bad shape");
  hipLaunchKernelGGL(k_bias_grad, dim3(C), dim3(256), 0, as_stream(stream), gout, N, C, HW, db);
  return launch_status("e2ep_bias_grad");
}

}  // extern "C"
