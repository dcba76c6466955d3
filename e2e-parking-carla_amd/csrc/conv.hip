// NCHW fp32 convolution for gfx950 as implicit GEMM on the exact-f32 matrix cores
// (v_mfma_f32_32x32x2_f32: f32 in, f32 accumulate, bitwise an fmaf chain).
//
//   forward      y[n,co,p]  = sum_k W[co,k] * xcol[k,(n,p)]            M=Cout N=n*P*Q K=Cin*R*S
//   bwd-data     dx[n,ci,p] = sum_k W'[ci,k] * gcol[k,(n,p)]           M=Cin  N=n*H*W K=Cout*R*S
//   bwd-weight   dW[co,k]   = sum_(n,p) g[n,co,p] * xcol[k,(n,p)]      M=Cout N=Cin*R*S K=n*P*Q
//
// Every conv of the hot path uses these kernels: BEV encoder (conv7x7/2 + ResNet-18 layers
// 1-3), segmentation head, DeepLab/ASPP heads, UpsamplingConcat, EfficientNet 1x1
// expand/project convs and the stem (reference model/bev_encoder.py:13-34,
// model/segmentation_head.py:19-31, model/convolutions.py:183-282, efficientnet-pytorch
// MBConv).  1x1 convs on 1x1 maps (squeeze-excitation) use the skinny-GEMM kernel at the end;
// depthwise convs have their own memory-bound kernels (dwconv.hip).
//
// Tiling: 256 threads = 4 waves (2 x 2); block tile 64 (M) x BNT (N, 64 or 128), K-step 16,
// each wave 32 x BNT/2 (one or two 32x32 accumulators sharing the A fragment).  A and B are
// staged global -> registers -> LDS (double buffered, one barrier per K-step).  The im2col
// gather is driven by per-conv k-tables (int4 {b_off, dy, dx, a_off}) built once on the
// device, so the inner loop has no integer division:
//   fwd:   iy = oy*sh - ph + dy,  ix = ox*sw - pw + dx
//   dgrad: split by input-pixel phase (iy % sh, ix % sw); only the taps whose output
//          coordinate is integral for that phase are in the phase's table, and
//          qy = u + dy, qx = v + dx  (iy = py + sh*u) -- no zero taps at stride 2.
// bwd-weight splits the pixel reduction over blocks and sums the fp32 partial slabs in a
// fixed order: results are run-to-run deterministic.
#include <algorithm>

#include "common.h"

namespace e2ep {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BK = 16;
constexpr int PADA = 4, PADB = 4;
constexpr int MAXPH = 4;

struct ConvGeom {
  int N;            // images
  int Cin, H, W;    // input
  int Cout, R, S;   // filter
  int P, Q;         // output spatial
  int sh, sw, ph, pw, dh, dw;
};

struct Phases {  // dgrad phase decomposition
  int n;
  int py[MAXPH], px[MAXPH];     // phase offsets
  int Hp[MAXPH], Wp[MAXPH];     // pixels of the phase
  int k0[MAXPH], kn[MAXPH];     // table slice
};

// ------------------------------------------------------------------------------------------
// k-tables
// ------------------------------------------------------------------------------------------
__global__ void k_conv_table_fwd(ConvGeom g, int4 *__restrict__ tab, int Kg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Kg) return;
  const int RS = g.R * g.S;
  const int c = k / RS, rs = k - c * RS, r = rs / g.S, s = rs - r * g.S;
  tab[k] = make_int4(c * g.H * g.W, r * g.dh, s * g.dw, k);
}

// dgrad table of one phase (py, px): taps whose output coordinate is integral
__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__global__ void k_conv_table_dgrad(ConvGeom g, int py, int px, int4 *__restrict__ tab) {
  // single thread: deterministic compaction (tables are tiny and built once per geometry)
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int n = 0;
  const int RS = g.R * g.S;
  for (int co = 0; co < g.Cout; ++co)
    for (int r = 0; r < g.R; ++r) {
      const int ny = py + g.ph - r * g.dh;
      if (((ny % g.sh) + g.sh) % g.sh) continue;
      for (int s = 0; s < g.S; ++s) {
        const int nx = px + g.pw - s * g.dw;
        if (((nx % g.sw) + g.sw) % g.sw) continue;
        tab[n++] = make_int4(co * g.P * g.Q, floordiv(ny, g.sh), floordiv(nx, g.sw),
                             co * g.Cin * RS + r * g.S + s);
      }
    }
}

// ------------------------------------------------------------------------------------------
// forward / bwd-data GEMM
// ------------------------------------------------------------------------------------------
template <int MODE, int ACT, int BNT>
__global__ void __launch_bounds__(256, 2) k_conv_gemm(
    const float *__restrict__ A, int a_row_stride, const float *__restrict__ src,
    const int4 *__restrict__ tab_all, const float *__restrict__ bias, float *__restrict__ dst,
    ConvGeom g, int M, int Kfwd, Phases ph) {
  constexpr int NACC = BNT / 64;
  __shared__ float As[2][BK][BM + PADA];
  __shared__ float Bs[2][BK][BNT + PADB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BNT;

  // phase (dgrad) or the single forward "phase"
  int py = 0, px = 0, Hc, Wc, Kg;
  const int4 *tab;
  if (MODE == 0) {
    Hc = g.P; Wc = g.Q; Kg = Kfwd; tab = tab_all;
  } else {
    const int z = blockIdx.z;
    py = ph.py[z]; px = ph.px[z]; Hc = ph.Hp[z]; Wc = ph.Wp[z];
    Kg = ph.kn[z]; tab = tab_all + ph.k0[z];
  }
  const int Hd = MODE == 0 ? g.P : g.H, Wd = MODE == 0 ? g.Q : g.W;  // dst spatial
  const int Hs = MODE == 0 ? g.H : g.P, Ws = MODE == 0 ? g.W : g.Q;  // src spatial
  const int Cs = MODE == 0 ? g.Cin : g.Cout;
  const int HWc = Hc * Wc;
  const int Ntot = g.N * HWc;
  if (n0 >= Ntot) return;

  // this thread's B-load column (constant over the K loop)
  constexpr int BROWS = 256 / BNT;          // rows loaded per pass (2 or 4)
  constexpr int BPER = BK / BROWS;          // loads per thread (8 or 4)
  const int bn = tid % BNT;
  const int bk0 = tid / BNT;
  const int ncol = n0 + bn;
  const bool col_ok = ncol < Ntot;
  int img = 0, cp = 0;
  if (col_ok) {
    img = ncol / HWc;
    cp = ncol - img * HWc;
  }
  const int cy = cp / Wc, cx = cp - cy * Wc;
  const float *sbase = src + (size_t)img * Cs * Hs * Ws;
  const int y0 = MODE == 0 ? cy * g.sh - g.ph : cy;
  const int x0 = MODE == 0 ? cx * g.sw - g.pw : cx;

  // this thread's A-load coordinates
  const int am = tid & (BM - 1);
  const int ak0 = tid >> 6;  // 0..3
  const bool arow_ok = (m0 + am) < M;
  const float *abase = A + (size_t)(m0 + am) * a_row_stride;

  float ra[4], rb[BPER];

  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + ak0 + 4 * j;
      ra[j] = (arow_ok && k < Kg) ? abase[tab[k].w] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < BPER; ++j) {
      const int k = k0 + bk0 + BROWS * j;
      float v = 0.f;
      if (col_ok && k < Kg) {
        const int4 t = tab[k];
        const int iy = y0 + t.y, ix = x0 + t.z;
        if ((unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws) v = sbase[t.x + iy * Ws + ix];
      }
      rb[j] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) As[buf][ak0 + 4 * j][am] = ra[j];
#pragma unroll
    for (int j = 0; j < BPER; ++j) Bs[buf][bk0 + BROWS * j][bn] = rb[j];
  };

  f32x16 acc[NACC];
#pragma unroll
  for (int t = 0; t < NACC; ++t) acc[t] = f32x16{0};
  const int nk = (Kg + BK - 1) / BK;
  if (nk > 0) {
    load_tiles(0);
    store_tiles(0);
  }
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_tiles((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[buf][kk + lk][32 * wm + li];
#pragma unroll
      for (int t = 0; t < NACC; ++t) {
        const float b = Bs[buf][kk + lk][(BNT / 2) * wn + 32 * t + li];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store_tiles(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int HWd = Hd * Wd;
#pragma unroll
  for (int t = 0; t < NACC; ++t) {
    const int n = n0 + (BNT / 2) * wn + 32 * t + li;
    if (n >= Ntot) continue;
    const int im = n / HWc;
    const int p = n - im * HWc;
    int dp = p;
    if (MODE == 1) {
      const int u = p / Wc, v = p - u * Wc;
      dp = (py + g.sh * u) * Wd + (px + g.sw * v);
    }
    float *dbase = dst + (size_t)im * M * HWd + dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
      if (m < M) {
        float v = acc[t][r];
        if (bias) v += bias[m];
        if (ACT == 1) v = fmaxf(v, 0.f);
        dbase[(size_t)m * HWd] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// bwd-weight: dW[co,k] = sum over pixels of g[n,co,p] * xcol[k,(n,p)]; split over pixels.
// Block tile 64 (co) x 128 (k), K-step = 16 pixels.  Partial slab per split.
// ------------------------------------------------------------------------------------------
constexpr int WBN = 128;

__global__ void __launch_bounds__(256, 2) k_conv_wgrad(
    const float *__restrict__ gout, const float *__restrict__ x, const int4 *__restrict__ tab,
    float *__restrict__ part, ConvGeom g, int Kg, int pix_per_split) {
  __shared__ float As[2][BK][BM + PADA];  // As[pixel][co]
  __shared__ float Bs[2][BK][WBN + PADB];  // Bs[pixel][k]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * WBN;
  const int split = blockIdx.z;
  const int PQ = g.P * g.Q;
  const int Ptot = g.N * PQ;
  const int pbeg = split * pix_per_split;
  const int pend = min(Ptot, pbeg + pix_per_split);

  // thread -> pixel = tid & 15 (same pixel for its A and B loads), co/k rows = tid >> 4
  const int tp = tid & 15, trow = tid >> 4;
  int4 tk[8];
  bool kok[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = n0 + trow + 16 * j;
    kok[j] = k < Kg;
    tk[j] = kok[j] ? tab[k] : make_int4(0, 0, 0, 0);
  }
  // running (image, pixel) of this thread's pixel, advanced by BK per K-step (no division)
  int p_cur = pbeg + tp;
  int im = p_cur / max(PQ, 1), od = p_cur - im * PQ;

  float ra[4], rb[8];
  auto load_tiles = [&]() {
    const bool pok = p_cur < pend;
    const int oy = od / g.Q, ox = od - oy * g.Q;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = m0 + trow + 16 * j;
      ra[j] = (pok && co < g.Cout) ? gout[((size_t)im * g.Cout + co) * PQ + od] : 0.f;
    }
    const int y0 = oy * g.sh - g.ph, x0 = ox * g.sw - g.pw;
    const float *xb = x + (size_t)im * g.Cin * g.H * g.W;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = 0.f;
      if (pok && kok[j]) {
        const int iy = y0 + tk[j].y, ix = x0 + tk[j].z;
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          v = xb[tk[j].x + iy * g.W + ix];
      }
      rb[j] = v;
    }
    p_cur += BK;
    od += BK;
    while (od >= PQ) {
      od -= PQ;
      ++im;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) As[buf][tp][trow + 16 * j] = ra[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) Bs[buf][tp][trow + 16 * j] = rb[j];
  };

  f32x16 acc0 = {0}, acc1 = {0};
  const int nk = (pend - pbeg + BK - 1) / BK;
  const int li = lane & 31, lk = lane >> 5;
  if (nk > 0) {
    load_tiles();
    store_tiles(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_tiles();
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
  float *pbase = part + (size_t)split * g.Cout * Kg;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = n0 + 64 * wn + 32 * t + li;
    if (k >= Kg) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
      if (co < g.Cout) pbase[(size_t)co * Kg + k] = t == 0 ? acc0[r] : acc1[r];
    }
  }
}

// fixed-order sum of the split slabs (+ optional accumulate into an existing gradient)
__global__ void k_reduce_splits(const float *__restrict__ part, int splits, int n,
                                float *__restrict__ out, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = accumulate ? out[i] : 0.f;
  for (int k = 0; k < splits; ++k) s += part[(size_t)k * n + i];
  out[i] = s;
}

// per-channel bias gradient: db[c] = sum over (n, p) of g[n, c, p]  (one block per channel)
__global__ void __launch_bounds__(256) k_bias_grad(const float *__restrict__ g, int N, int C,
                                                   int HW, float *__restrict__ db) {
  const int c = blockIdx.x;
  float s = 0.f;
  for (int n = 0; n < N; ++n) {
    const float *p = g + ((size_t)n * C + c) * HW;
    for (int i = threadIdx.x; i < HW; i += 256) s += p[i];
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) db[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------------------------------
// skinny GEMM (tiny M x N, any K): C[i,j] = sum_k A[i*ai + k*ak] * B[k*bk + j*bj] (+ bias[j]).
// One wave per output element, lanes stride K, wave reduction.  Used for the SE 1x1 convs
// on 1x1 maps (N*C <= a few thousand outputs) forward and backward.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_skinny_gemm(const float *__restrict__ A, int ai, int ak,
                                                     const float *__restrict__ B, int bk, int bj,
                                                     const float *__restrict__ bias, int Mi, int Nj,
                                                     int K, float *__restrict__ C) {
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= Mi * Nj) return;
  const int i = o / Nj, j = o - i * Nj;
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += A[(size_t)i * ai + (size_t)k * ak] * B[(size_t)k * bk + (size_t)j * bj];
  s = wave_sum(s);
  if (lane == 0) C[o] = s + (bias ? bias[j] : 0.f);
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
         g.pw >= 0 && (long long)g.N * g.Cin * g.H * g.W < (1LL << 31) &&
         (long long)g.N * g.Cout * g.P * g.Q < (1LL << 31);
}

// dgrad table layout: int4 entries of phase 0 .. phase n-1, each phase slice sized
// Cout*R*S (upper bound); the count of phase (py, px) is Cout * nr(py) * ns(px).
static int n_phases(const ConvGeom &g) { return g.sh * g.sw; }

static int valid_taps(int p, int pad, int K, int dil, int st) {
  int n = 0;
  for (int r = 0; r < K; ++r) {
    const int v = p + pad - r * dil;
    if (((v % st) + st) % st == 0) ++n;
  }
  return n;
}

static Phases make_phases(const ConvGeom &g, bool dgrad) {
  Phases p;
  p.n = n_phases(g);
  const int cap = g.Cout * g.R * g.S;
  for (int z = 0; z < p.n; ++z) {
    p.py[z] = z / g.sw;
    p.px[z] = z % g.sw;
    p.Hp[z] = p.py[z] < g.H ? (g.H - p.py[z] + g.sh - 1) / g.sh : 0;
    p.Wp[z] = p.px[z] < g.W ? (g.W - p.px[z] + g.sw - 1) / g.sw : 0;
    p.k0[z] = z * cap;
    p.kn[z] = dgrad ? g.Cout * valid_taps(p.py[z], g.ph, g.R, g.dh, g.sh) *
                          valid_taps(p.px[z], g.pw, g.S, g.dw, g.sw)
                    : 0;
  }
  return p;
}

extern "C" {

size_t e2ep_conv_table_bytes(const int *dims, int dgrad) {
  ConvGeom g = make_geom(dims);
  if (!dgrad) return (size_t)g.Cin * g.R * g.S * 16;
  return (size_t)n_phases(g) * g.Cout * g.R * g.S * 16;
}

int e2ep_conv_table(const int *dims, int dgrad, void *table, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_table: bad geometry");
  E2EP_REQUIRE(n_phases(g) <= MAXPH, E2EP_ERANGE, "e2ep_conv_table: stride product > %d", MAXPH);
  hipStream_t s = as_stream(stream);
  if (!dgrad) {
    const int Kg = g.Cin * g.R * g.S;
    hipLaunchKernelGGL(k_conv_table_fwd, dim3(cdiv(Kg, 256)), dim3(256), 0, s, g,
                       static_cast<int4 *>(table), Kg);
  } else {
    int4 *ent = static_cast<int4 *>(table);
    const int cap = g.Cout * g.R * g.S;
    for (int z = 0; z < n_phases(g); ++z)
      hipLaunchKernelGGL(k_conv_table_dgrad, dim3(1), dim3(64), 0, s, g, z / g.sw, z % g.sw,
                         ent + (size_t)z * cap);
  }
  return launch_status("e2ep_conv_table");
}

static int launch_gemm(int mode, int act, const float *A, int a_stride, const float *src,
                       const int4 *tab, const float *bias, float *dst, const ConvGeom &g, int M,
                       int Kfwd, const Phases &ph, hipStream_t s) {
  // columns of the largest phase / the forward output
  long long ncols = 0;
  if (mode == 0) {
    ncols = (long long)g.N * g.P * g.Q;
  } else {
    for (int z = 0; z < ph.n; ++z) ncols = std::max(ncols, (long long)g.N * ph.Hp[z] * ph.Wp[z]);
  }
  const int mblocks = cdiv(M, BM);
  // prefer the wide tile when it still yields >= 2 workgroups per CU
  const bool wide = cdiv(ncols, 128) * mblocks * (mode ? ph.n : 1) >= 512;
  const int bnt = wide ? 128 : 64;
  dim3 grid(cdiv(ncols, bnt), mblocks, mode ? ph.n : 1);
#define GEMM_LAUNCH(MD, AC, BT)                                                                   \
  hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT>), grid, dim3(256), 0, s, A, a_stride, src, tab, bias, \
                     dst, g, M, Kfwd, ph)
  if (mode == 0 && act == 0) { if (wide) GEMM_LAUNCH(0, 0, 128); else GEMM_LAUNCH(0, 0, 64); }
  else if (mode == 0) { if (wide) GEMM_LAUNCH(0, 1, 128); else GEMM_LAUNCH(0, 1, 64); }
  else { if (wide) GEMM_LAUNCH(1, 0, 128); else GEMM_LAUNCH(1, 0, 64); }
#undef GEMM_LAUNCH
  return 0;
}

int e2ep_conv_fwd(const float *x, const float *w, const float *bias, const void *table,
                  const int *dims, int act, float *y, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_fwd: bad geometry");
  E2EP_REQUIRE(act == 0 || act == 1, E2EP_EINVAL, "e2ep_conv_fwd: act must be 0 (none) or 1 (relu)");
  const int Kg = g.Cin * g.R * g.S;
  Phases ph = make_phases(g, false);
  launch_gemm(0, act, w, Kg, x, static_cast<const int4 *>(table), bias, y, g, g.Cout, Kg, ph,
              as_stream(stream));
  return launch_status("e2ep_conv_fwd");
}

int e2ep_conv_dgrad(const float *gout, const float *w, const void *table, const int *dims,
                    int m_channels, float *dx, void *stream) {
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_dgrad: bad geometry");
  E2EP_REQUIRE(m_channels > 0 && m_channels <= g.Cin, E2EP_EINVAL,
               "e2ep_conv_dgrad: m_channels must be in [1, Cin]");
  E2EP_REQUIRE(n_phases(g) <= MAXPH, E2EP_ERANGE, "e2ep_conv_dgrad: stride product > %d", MAXPH);
  Phases ph = make_phases(g, true);
  launch_gemm(1, 0, w, g.R * g.S, gout, static_cast<const int4 *>(table), nullptr, dx, g, m_channels, 0, ph, as_stream(stream));
  return launch_status("e2ep_conv_dgrad");
}

int e2ep_conv_wgrad_splits(const int *dims) {
  ConvGeom g = make_geom(dims);
  const int Kg = g.Cin * g.R * g.S;
  const long long base = (long long)cdiv(Kg, WBN) * cdiv(g.Cout, BM);
  const long long pix = (long long)g.N * g.P * g.Q;
  long long want = (1024 + base - 1) / base;
  long long cap = pix / 128;
  long long s = want < cap ? want : cap;
  if (s < 1) s = 1;
  if (s > 1024) s = 1024;
  return (int)s;
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
  const int Ptot = g.N * g.P * g.Q;
  int per = (Ptot + splits - 1) / splits;
  per = (per + BK - 1) / BK * BK;
  const int used = (Ptot + per - 1) / per;
  dim3 grid(cdiv(Kg, WBN), cdiv(g.Cout, BM), used);
  hipStream_t s = as_stream(stream);
  float *part = static_cast<float *>(workspace);
  hipLaunchKernelGGL(k_conv_wgrad, grid, dim3(256), 0, s, gout, x, static_cast<const int4 *>(table),
                     part, g, Kg, per);
  const int n = g.Cout * Kg;
  hipLaunchKernelGGL(k_reduce_splits, dim3(cdiv(n, 256)), dim3(256), 0, s, part, used, n, dw,
                     accumulate);
  return launch_status("e2ep_conv_wgrad");
}

int e2ep_bias_grad(const float *gout, int N, int C, int HW, float *db, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0, E2EP_EINVAL, "e2ep_bias_grad: bad shape");
  hipLaunchKernelGGL(k_bias_grad, dim3(C), dim3(256), 0, as_stream(stream), gout, N, C, HW, db);
  return launch_status("e2ep_bias_grad");
}

int e2ep_skinny_gemm(const float *A, int ai, int ak, const float *B, int bk, int bj,
                     const float *bias, int Mi, int Nj, int K, float *C, void *stream) {
  E2EP_REQUIRE(Mi > 0 && Nj > 0 && K > 0, E2EP_EINVAL, "e2ep_skinny_gemm: bad shape");
  hipLaunchKernelGGL(k_skinny_gemm, dim3(cdiv((long long)Mi * Nj, 4)), dim3(256), 0, as_stream(stream),
                     A, ai, ak, B, bk, bj, bias, Mi, Nj, K, C);
  return launch_status("e2ep_skinny_gemm");
}

}  // extern "C"
