// NCHW fp32 convolution for gfx950 as implicit GEMM on the exact-f32 matrix cores
// (v_mfma_f32_32x32x2_f32: f32 in, f32 accumulate, bitwise an fmaf chain).
//
//   forward      y[n,co,p]  = sum_(tap,ci) W[co,ci,tap] * x[n,ci,p+tap]       M=Cout  N=n*P*Q
//   bwd-data     dx[n,ci,p] = sum_(tap,co) W[co,ci,tap] * g[n,co,(p-tap)/s]   M=Cin   N=n*H*W
//   bwd-weight   dW[co,ci,tap] = sum_(n,p) g[n,co,p] * x[n,ci,p+tap]         M=Cout  N=taps*Cin
//
// Every conv of the hot path uses these kernels: BEV encoder (conv7x7/2 + ResNet-18 layers
// 1-3), segmentation head, DeepLab/ASPP heads, UpsamplingConcat, EfficientNet 1x1
// expand/project convs and the stem (reference model/bev_encoder.py:13-34,
// model/segmentation_head.py:19-31, model/convolutions.py:183-282, efficientnet-pytorch
// MBConv).  1x1 convs on 1x1 maps (squeeze-excitation) use the skinny-GEMM kernel at the end;
// depthwise convs have their own memory-bound kernels (dwconv.hip).
//
// K order is tap-outer / channel-inner: one K-step = one filter tap x 16 channels, so the
// im2col bounds test is done once per pixel per K-step (not per element), channel rows are
// a fixed stride apart, and no lookup table is needed.  The data gradient is split by
// input-pixel phase (iy % sh, ix % sw): each phase only visits the taps that land on an
// integral output coordinate (no zero taps at stride 2).
//
// Tiling: 256 threads = 4 waves (2 x 2); block tile 64 (M) x BNT (N, 64 or 128), each wave
// 32 x BNT/2 (one or two 32x32 accumulators sharing the A fragment).  A and B are staged
// global -> registers -> LDS (double buffered, one barrier per K-step) with branch-free
// buffer loads (out-of-range offset -> 0).  Small grids split K; partial slabs are reduced
// in a fixed order, so every result is run-to-run deterministic.
#include <algorithm>

#include "common.h"
#include "conv.h"
#include "gemm.h"
#include "bnstats.h"
#include "handoff.h"

// Contraction only within one expression (a*b + c -> fma): the fp32 and bf16-storage
// instantiations of a kernel (E2EP_IO_*) then fuse the same operations and round alike —
// under the default cross-statement contraction hipcc may pick a different multiply to fuse
// in each instantiation (tests/test_bf16_store_gpu.py holds them bitwise equal).
#pragma clang fp contract(on)

namespace e2ep {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 64, BK = 16;
constexpr int PADA = 4, PADB = 4;
constexpr int MAXPH = 4;
// ------------------------------------------------------------------------------------------
// forward (MODE 0) / data-gradient (MODE 1) implicit GEMM
// ------------------------------------------------------------------------------------------
// MODE 0: rows m = co, K channels c = ci, src = x [N,Cin,H,W], dst = y [N,Cout,P,Q];
//         column pixel (oy,ox); tap (r,s): iy = oy*sh - ph + r*dh, ix = ox*sw - pw + s*dw.
// MODE 1: rows m = ci, K channels c = co, src = g [N,Cout,P,Q], dst = dx [N,Cin,H,W];
//         phase z = (py, px), column pixel (u,v) -> (iy, ix) = (py + sh*u, px + sw*v);
//         tap (r,s) valid for the phase: qy = u + (py + ph - r*dh)/sh (exact), qx likewise.
// OP (0 fp32 / 1 bf16 / 2 fp16) as for k_conv_gemm2 below: for low precision one 16-deep MFMA
// per K-step takes lane half h's k = 8h .. 8h+7 (eight LDS reads per operand, as the eight
// fp32 MFMAs would do).
template <int BNT, int BMT>
constexpr int conv_gemm_lds_floats() { return 2 * BK * (BMT + PADA) + 2 * BK * (BNT + PADB); }

// The block body of k_conv_gemm for block (bx, by, bz) of a grid gx blocks wide; `lds` holds
// conv_gemm_lds_floats<BNT, BMT>() floats of the caller's __shared__ memory (so a kernel can run
// two problems in one grid: k_conv_bwd_pair).
// TS / TD: element types of src / dst (bf16_t: C3's bf16-stored activations, e2ep.h
// E2EP_IO_*; the weights and the MODE 1 residual gradient stay fp32)
template <int MODE, int ACT, int BNT, int BMT, bool AV, int OP, bool ST, typename TS = float,
          typename TD = float>
__device__ __forceinline__ void conv_gemm_block(
    const float *__restrict__ w, const TS *__restrict__ src, const float *__restrict__ bias,
    TD *__restrict__ dst, long long dst_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part, unsigned int *__restrict__ cnt, double *__restrict__ stats, int bx,
    int by, int bz, int gx, float *lds) {
  // block tile BMT x BNT: BMT = 64 -> 2 x 2 waves of 32 x BNT/2; BMT = 32 (small-M layers:
  // Cout or Cin 24..56) -> 1 x 4 waves of 32 x BNT/4, so no MFMA rows are padding
  constexpr int WC = BMT == 64 ? BNT / 2 : BNT / 4;  // columns per wave
  constexpr int NACC = WC / 32;
  constexpr int BROWS = 256 / BNT;  // B rows per pass (1, 2 or 4)
  constexpr int BPER = BK / BROWS;  // B loads per thread (16, 8 or 4)
  constexpr int NA = BK * BMT / 256;  // A loads per thread (4 or 2)
  float(*As)[BK][BMT + PADA] = reinterpret_cast<float(*)[BK][BMT + PADA]>(lds);
  float(*Bs)[BK][BNT + PADB] = reinterpret_cast<float(*)[BK][BNT + PADB]>(lds + 2 * BK * (BMT + PADA));
  __shared__ int s_tdy[MAXTAPS], s_tdx[MAXTAPS], s_trs[MAXTAPS];
  __shared__ int s_ntaps;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = BMT == 64 ? (wave & 1) : 0, wn = BMT == 64 ? (wave >> 1) : wave;
  const int m0 = by * BMT, n0 = bx * BNT;
  const int split = bz % splits, z = bz / splits;
  const int RS = g.R * g.S;

  // phase / pixel space of the columns
  int py = 0, px = 0, Hc, Wc;
  if (MODE == 0) {
    Hc = g.P; Wc = g.Q;
  } else {
    py = z / g.sw; px = z % g.sw;
    Hc = py < g.H ? (g.H - py + g.sh - 1) / g.sh : 0;
    Wc = px < g.W ? (g.W - px + g.sw - 1) / g.sw : 0;
  }
  const int HWc = Hc * Wc;
  const int Ntot = g.N * HWc;
  if (n0 >= Ntot) return;

  // tap table of this phase (tiny; built by one thread)
  if (tid == 0) {
    int n = 0;
    for (int r = 0; r < g.R; ++r) {
      int dy;
      if (MODE == 0) {
        dy = r * g.dh - g.ph;
      } else {
        const int ny = py + g.ph - r * g.dh;
        if (((ny % g.sh) + g.sh) % g.sh) continue;
        dy = floordiv(ny, g.sh);
      }
      for (int s = 0; s < g.S; ++s) {
        int dx;
        if (MODE == 0) {
          dx = s * g.dw - g.pw;
          if (!axis_live(dy, g.P, g.sh, g.H) || !axis_live(dx, g.Q, g.sw, g.W)) continue;
        } else {
          const int nx = px + g.pw - s * g.dw;
          if (((nx % g.sw) + g.sw) % g.sw) continue;
          dx = floordiv(nx, g.sw);
          if (!axis_live(dy, Hc, 1, g.P) || !axis_live(dx, Wc, 1, g.Q)) continue;
        }
        s_tdy[n] = dy;
        s_tdx[n] = dx;
        s_trs[n] = r * g.S + s;
        ++n;
      }
    }
    s_ntaps = n;
  }
  __syncthreads();
  const int ntaps = s_ntaps;
  const int Kc = MODE == 0 ? g.Cin : g.Cout;  // channels summed per tap
  const int csteps = (Kc + BK - 1) / BK;
  const int ksteps_all = ntaps * csteps;
  const int kbeg = split * kper;
  const int kend = min(ksteps_all, kbeg + kper);
  const int nk = max(0, kend - kbeg);

  const int Hs = MODE == 0 ? g.H : g.P, Ws = MODE == 0 ? g.W : g.Q;  // src spatial
  const int HWs = Hs * Ws;
  constexpr int ES = sizeof(TS);  // bytes per src element
  const __amdgpu_buffer_rsrc_t rw = rsrc(w, 4LL * g.Cout * g.Cin * RS);
  const __amdgpu_buffer_rsrc_t rx = rsrc(src, (long long)ES * g.N * Kc * HWs);

  // B-load column of this thread (fixed); its rows are wave-uniform
  const int bn = tid % BNT;
  const int bk0 = __builtin_amdgcn_readfirstlane(tid / BNT);  // BNT >= 64: wave-uniform
  const int ncol = n0 + bn;
  const bool col_ok = ncol < Ntot;
  int img = 0, cp = 0;
  if (col_ok) {
    img = ncol / HWc;
    cp = ncol - img * HWc;
  }
  const int cy = cp / Wc, cx = cp - cy * Wc;
  const int ybase = MODE == 0 ? cy * g.sh : cy;
  const int xbase = MODE == 0 ? cx * g.sw : cx;
  const int simg = img * Kc * HWs;

  // A-load row of this thread; its k rows (channels) are wave-uniform (dgrad).  Forward
  // loads run along the weight's channel axis instead (thread = row tid/4, channels
  // 4*(tid%4)..+3: float4 for 1x1 filters), so a wave touches 16 weight rows, not 64.
  const int am = MODE == 0 ? tid / (BK / NA) : (tid & (BMT - 1));
  const int ac = MODE == 0 ? NA * (tid % (BK / NA)) : 0;
  // dgrad: this thread's first k row (then every 256/BMT); wave-uniform for BMT = 64
  const int ak0 = BMT == 64 ? __builtin_amdgcn_readfirstlane(tid / BMT) : tid / BMT;
  const bool arow_ok = (m0 + am) < M;
  // weight layout 0 (PyTorch [Cout][Cin][RS]):
  //   fwd: W[m][c][rs] = w[m*Cin*RS + c*RS + rs];  dgrad: W[c][m][rs] = w[c*Cin*RS + m*RS + rs]
  // weight layout 1 (tap-major [RS][Cout][Cin], contiguous along Cin for every tap):
  //   fwd: w[rs*Cout*Cin + m*Cin + c];             dgrad: w[rs*Cout*Cin + c*Cin + m]
  const bool tm = g.wlayout == 1;
  const int a_mstride = MODE == 0 ? (tm ? g.Cin : g.Cin * RS) : (tm ? 1 : RS);
  const int a_cstride = MODE == 0 ? (tm ? 1 : RS) : (tm ? g.Cin : g.Cin * RS);
  const int a_tstride = tm ? g.Cout * g.Cin : 1;
  // AV (host-checked): forward, tap-major weights, Cin % 4 == 0 -> one 16-B A load per thread
  static_assert(!AV || (MODE == 0 && NA == 4), "AV: forward 64-row tiles only");
  const int arow = (m0 + am) * a_mstride;

  // Guards without per-element branches: a disabled operand gets an offset >= the buffer's
  // size (returns 0).  Per-thread conditions (pixel / row in range) pick the base offset once
  // per K-step; per-row channel conditions are wave-uniform and pick the row term on the
  // scalar unit; row terms are uniform strides, so each element costs one add.  Sums stay
  // below 2^32: the base is < 2^31 and so is every row term.
  const int nrw = (int)min(4LL * g.Cout * g.Cin * RS, 0x7fffffffLL);
  const int nrx = (int)min((long long)ES * g.N * Kc * HWs, 0x7fffffffLL);

  // global -> register loads run two K-steps ahead of the MFMAs (two register sets), LDS
  // is double buffered: one barrier per K-step, ~2 steps of MFMA work to cover a load.  (A
  // third register set, loads three steps ahead, measured 5-40 % slower per shape in round 3.)
  float ra0[NA], rb0[BPER], ra1[NA], rb1[BPER];
  // Every call issues the same loads (steps past the range read zeros), so the loop has no
  // branches around loads and the s_waitcnt before each LDS store waits only for the step
  // being stored, not for the prefetch issued after it.
  const int klast = kend - 1;
  auto load_tiles = [&](int ks_in, float(&ra)[NA], float(&rb)[BPER]) {
    const bool live = ks_in <= klast;                 // uniform
    const int ks = min(ks_in, klast);
    const int tap = g.korder ? ks % ntaps : ks / csteps;  // uniform
    const int c0 = (g.korder ? ks / ntaps : ks - tap * csteps) * BK;
    const int dy = s_tdy[tap], dx = s_tdx[tap], rs = s_trs[tap] * a_tstride;
    if (MODE == 0) {
      const int c = c0 + ac;
      if (AV) {
        const float4 v = bload4(rw, (live && arow_ok && c < Kc) ? (arow + c + rs) * 4 : OOR);
        ra[0] = v.x; ra[1] = v.y; ra[NA > 2 ? 2 : 0] = v.z; ra[NA > 3 ? 3 : 0] = v.w;
      } else {
        const int abase = (live && arow_ok) ? (arow + rs) * 4 : nrw;
#pragma unroll
        for (int j = 0; j < NA; ++j)
          ra[j] = bload(rw, c + j < Kc ? abase + (c + j) * a_cstride * 4 : OOR);
      }
    } else {
      // rows c0 + ak0 + (256/BMT) j: wave-uniform (ak0 = wave index for BMT = 64)
      const int abase = (live && arow_ok) ? (arow + rs) * 4 : nrw;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int c = c0 + ak0 + (256 / BMT) * j;
        const int rterm = c < Kc ? c * a_cstride * 4 : nrw;
        ra[j] = bload(rw, abase + rterm);
      }
    }
    const int iy = ybase + dy, ix = xbase + dx;
    const bool pix_ok = live && col_ok && (unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws;
    // rows c0 + bk0 + BROWS j: wave-uniform (bk0 = tid / BNT, BNT >= 64)
    const int bbase = pix_ok ? (simg + iy * Ws + ix) * ES : nrx;
#pragma unroll
    for (int j = 0; j < BPER; ++j) {
      const int c = c0 + bk0 + BROWS * j;
      const int rterm = c < Kc ? c * HWs * ES : nrx;
      rb[j] = bload_t(rx, bbase + rterm, src);
    }
  };
  auto store_tiles = [&](int buf, const float(&ra)[NA], const float(&rb)[BPER]) {
#pragma unroll
    for (int j = 0; j < NA; ++j) As[buf][MODE == 0 ? ac + j : ak0 + (256 / BMT) * j][am] = ra[j];
#pragma unroll
    for (int j = 0; j < BPER; ++j) Bs[buf][bk0 + BROWS * j][bn] = rb[j];
  };

  f32x16 acc[NACC];
#pragma unroll
  for (int t = 0; t < NACC; ++t) acc[t] = f32x16{0};
  const int li = lane & 31, lk = lane >> 5;
  auto compute = [&](int buf) {
    if (OP == 0) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const float a = As[buf][kk + lk][32 * wm + li];
#pragma unroll
        for (int t = 0; t < NACC; ++t) {
          const float b = Bs[buf][kk + lk][WC * wn + 32 * t + li];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
        }
      }
    } else {
      bf16x8 abf;
      f16x8 ah;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = As[buf][8 * lk + j][32 * wm + li];
        if (OP == 1) abf[j] = (__bf16)a; else ah[j] = (_Float16)a;
      }
#pragma unroll
      for (int t = 0; t < NACC; ++t) {
        bf16x8 bbf;
        f16x8 bh;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float b = Bs[buf][8 * lk + j][WC * wn + 32 * t + li];
          if (OP == 1) bbf[j] = (__bf16)b; else bh[j] = (_Float16)b;
        }
        if (OP == 1) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(abf, bbf, acc[t], 0, 0, 0);
        else acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
      }
    }
  };
  if (nk > 0) {
    load_tiles(kbeg, ra0, rb0);
    store_tiles(0, ra0, rb0);
    load_tiles(kbeg + 1, ra1, rb1);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      // buffer 0 holds step kt, registers 1 hold step kt+1
      load_tiles(kbeg + kt + 2, ra0, rb0);
      // the loads stay at the top of the step (hipcc otherwise sinks them behind the MFMAs)
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);  // the LDS write after all of the step's MFMAs
      store_tiles(1, ra1, rb1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      // buffer 1 holds step kt+1, registers 0 hold step kt+2
      load_tiles(kbeg + kt + 3, ra1, rb1);
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      store_tiles(0, ra0, rb0);
      __syncthreads();
    }
  }

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // splits == 1: final values (bias, act) into dst[img][m][pixel];
  // splits > 1:  raw partial sums into part[split][m][n]: with `cnt` (the in-launch fold)
  // write-through, and the tile's last-arriving split sums every slab in split order
  // (k_conv_reduce's order) and writes the final values; without, k_conv_reduce does.
  if (splits > 1) {
    __shared__ int s_last;
    const int MN = M * Ntot;
    const __amdgpu_buffer_rsrc_t rp = rsrc(part + (size_t)split * MN, 4LL * MN);
#pragma unroll
    for (int t = 0; t < NACC; ++t) {
      const int n = n0 + WC * wn + 32 * t + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
        const int off = (n < Ntot && m < M) ? (m * Ntot + n) * 4 : OOR;
        if (cnt) bstore_sc1(rp, off, acc[t][r]);
        else bstore(rp, off, acc[t][r]);
      }
    }
    if (!cnt) return;
    handoff_drain();
    if (!handoff_arrive(cnt + bx + gx * by, splits, &s_last)) return;
    const __amdgpu_buffer_rsrc_t rall = rsrc(part, 4LL * splits * MN);
#pragma unroll
    for (int t = 0; t < NACC; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    for (int k = 0; k < splits; ++k) {
#pragma unroll
      for (int t = 0; t < NACC; ++t) {
        const int n = n0 + WC * wn + 32 * t + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
          acc[t][r] += bload_sc1(rall, (n < Ntot && m < M) ? (k * MN + m * Ntot + n) * 4 : OOR);
        }
      }
    }
  }
  const __amdgpu_buffer_rsrc_t rd = rsrc(dst, dst_bytes);
  constexpr int ED = sizeof(TD);  // bytes per dst element (the fp32 residual: 4)
  // MODE 1: `bias` is an optional residual gradient in dst's layout, added to dx here (the
  // skip connection's gradient, so autograd needs no separate accumulation kernel)
  const __amdgpu_buffer_rsrc_t rres = rsrc(bias, MODE == 1 && bias ? dst_bytes / ED * 4 : 0);
  const int Hd = MODE == 0 ? g.P : g.H, Wd = MODE == 0 ? g.Q : g.W;
  const int HWd = Hd * Wd;
  // MODE 0 with `stats`: BatchNorm partial sums of the stored values (bnstats.h)
  constexpr bool want_stats = ST && MODE == 0;
  float fs[16], fq[16];  // this lane's NACC (<= 4) values per row; fp64 from the butterfly on
#pragma unroll
  for (int r = 0; r < 16; ++r) fs[r] = fq[r] = 0.f;
#pragma unroll
  for (int t = 0; t < NACC; ++t) {
    const int n = n0 + WC * wn + 32 * t + li;
    const bool nok = n < Ntot;
    int dbase, mstride;
    if (true) {
      const int im = n / HWc;
      const int p = n - im * HWc;
      int dp = p;
      if (MODE == 1) {
        const int u = p / Wc, v = p - u * Wc;
        dp = (py + g.sh * u) * Wd + (px + g.sw * v);
      }
      dbase = im * M * HWd + dp;
      mstride = HWd;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
      float v = acc[t][r];
      const bool in = nok && m < M;
      const int e = dbase + m * mstride;  // element offset (res: 4 B, dst: ED B)
      if (MODE == 0) {
        if (bias) v += bias[min(m, M - 1)];
        if (ACT == 1) v = fmaxf(v, 0.f);
      } else if (bias) {
        v += bload(rres, in ? e * 4 : OOR);
      }
      if (want_stats) {
        const float d = in ? stored<TD>(v) : 0.f;
        fs[r] += d;
        fq[r] = __builtin_fmaf(d, d, fq[r]);
      }
      bstore_t(rd, in ? e * ED : OOR, v, dst);
    }
  }
  if (want_stats) {
    __shared__ double s_bn[2 * 64 * 2];  // [wn][row][2]: 2 x 64 or 4 x 32 rows
    double bs[16], bq[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      bs[r] = fs[r];
      bq[r] = fq[r];
    }
    bns_store_tile(bs, bq, wm, wn, BMT == 64 ? 2 : 4, BMT, m0, M, bx, s_bn, stats);
  }
}

// ST (forward only): the epilogue also writes BatchNorm partial sums into `stats` (bnstats.h);
// a separate instantiation, so the plain forward keeps its register allocation.
template <int MODE, int ACT, int BNT, int BMT, bool AV, int OP = 0, bool ST = false,
          typename TS = float, typename TD = float>
__global__ void __launch_bounds__(256, 2) k_conv_gemm(
    const float *__restrict__ w, const TS *__restrict__ src, const float *__restrict__ bias,
    TD *__restrict__ dst, long long dst_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part, unsigned int *__restrict__ cnt, double *__restrict__ stats) {
  __shared__ __attribute__((aligned(16))) float lds[conv_gemm_lds_floats<BNT, BMT>()];
  conv_gemm_block<MODE, ACT, BNT, BMT, AV, OP, ST, TS, TD>(w, src, bias, dst, dst_bytes, g, M,
                                                           splits, kper, part, cnt, stats,
                                                           blockIdx.x, blockIdx.y, blockIdx.z,
                                                           gridDim.x, lds);
}

// split-K reduction (fixed order) + bias / relu epilogue:
// out[img][m][p] = act(sum_s part[s][m][img*HW + p] + bias[m])
__global__ void k_conv_reduce(const float *__restrict__ part, int splits, int M, int HW, int Ntot,
                              const float *__restrict__ bias, int act,
                              const float *__restrict__ res, float *__restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= Ntot) return;
  const int m = blockIdx.y;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[((size_t)k * M + m) * Ntot + n];
  if (bias) s += bias[m];
  if (act == 1) s = fmaxf(s, 0.f);
  const int im = n / HW, p = n - im * HW;
  const size_t o = ((size_t)im * M + m) * HW + p;
  if (res) s += res[o];
  out[o] = s;
}


// ------------------------------------------------------------------------------------------
// forward (MODE 0) / data-gradient (MODE 1) implicit GEMM, second generation (large shapes:
// the BEV stem 7x7/2, the segmentation head's 3x3 at 200x200, the ResNet layers).
//
// What changes against k_conv_gemm:
//  * LDS images are k-contiguous ([row][16 k + 4 pad], 80-B rows: conflict-free b128 reads
//    and writes), and the K index inside a K-step is permuted so lane half h of MFMA t
//    takes k = 8h + t: a lane's 8 A (or B) operands of the step are one 32-B run, read as
//    two ds_read_b128 instead of eight ds_read_b32.  The sum is over the same 16 k; its
//    order is fixed, so results are deterministic.
//  * wave tiles 32 x 32*WNT (WNT = 4: four accumulators share each A fragment); block tile
//    64 x 64*WNT, 32*WNT MFMAs per wave per barrier.
//  * no zero-padded channel steps: K = taps x floor(Kc/16) full steps + "tail" steps that
//    flatten the remaining (channel, tap) pairs 16 at a time (the BEV stem's 65th channel:
//    4 tail steps instead of 49 half-empty ones), each tail row with its own tap offset.
// ------------------------------------------------------------------------------------------
constexpr int V2_LDW = 20;    // LDS row stride in floats (16 k + 4 pad)
constexpr int V2_TAIL = 256;  // max flattened (remainder channel, tap) rows

// OP: MFMA operand precision — 0 fp32 (v_mfma_f32_32x32x2_f32, exact), 1 bf16 / 2 fp16
// (v_mfma_f32_32x32x16_{bf16,f16}: the fragments are rounded to nearest-even when read from
// LDS, products and sums stay fp32; the BASELINE C3 bf16 forward and C5 fp16 inference
// modes).  A lane's 8 fragment values are exactly the 8 k of its lane half that the 16-deep
// low-precision MFMA takes, so one MFMA replaces the eight fp32 ones per K-step.
template <int MODE, int ACT, int WNT, int OP = 0>
__global__ void __launch_bounds__(256) k_conv_gemm2(
    const float *__restrict__ w, const float *__restrict__ src, const float *__restrict__ bias,
    float *__restrict__ dst, long long dst_bytes, ConvGeom g, int M, int splits, int kper) {
  constexpr int BN = 64 * WNT;        // block columns (2 waves x 32*WNT)
  constexpr int KGRP = 256 / BN;      // B k-groups per pass (1 or 2)
  constexpr int RPT = BK / KGRP;      // B rows per thread (16 or 8)
  __shared__ __attribute__((aligned(16))) float As[2][64][V2_LDW];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][V2_LDW];
  __shared__ int s_tdy[MAXTAPS], s_tdx[MAXTAPS], s_trs[MAXTAPS];
  __shared__ int s_kc[V2_TAIL], s_kdy[V2_TAIL], s_kdx[V2_TAIL], s_krs[V2_TAIL];
  __shared__ int s_ntaps;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * BN;
  const int split = blockIdx.z % splits, z = blockIdx.z / splits;
  const int RS = g.R * g.S;

  int py = 0, px = 0, Hc, Wc;
  if (MODE == 0) {
    Hc = g.P; Wc = g.Q;
  } else {
    py = z / g.sw; px = z % g.sw;
    Hc = py < g.H ? (g.H - py + g.sh - 1) / g.sh : 0;
    Wc = px < g.W ? (g.W - px + g.sw - 1) / g.sw : 0;
  }
  const int HWc = Hc * Wc;
  const int Ntot = g.N * HWc;
  if (n0 >= Ntot) return;
  const int Kc = MODE == 0 ? g.Cin : g.Cout;   // channels summed per tap
  const int cfull = Kc / BK, crem = Kc - cfull * BK;

  // live tap table of this phase, then the tail table (remainder channel major, tap minor)
  if (tid == 0) {
    int n = 0;
    for (int r = 0; r < g.R; ++r) {
      int dy;
      if (MODE == 0) {
        dy = r * g.dh - g.ph;
      } else {
        const int ny = py + g.ph - r * g.dh;
        if (((ny % g.sh) + g.sh) % g.sh) continue;
        dy = floordiv(ny, g.sh);
      }
      for (int s = 0; s < g.S; ++s) {
        int dx;
        if (MODE == 0) {
          dx = s * g.dw - g.pw;
          if (!axis_live(dy, g.P, g.sh, g.H) || !axis_live(dx, g.Q, g.sw, g.W)) continue;
        } else {
          const int nx = px + g.pw - s * g.dw;
          if (((nx % g.sw) + g.sw) % g.sw) continue;
          dx = floordiv(nx, g.sw);
          if (!axis_live(dy, Hc, 1, g.P) || !axis_live(dx, Wc, 1, g.Q)) continue;
        }
        s_tdy[n] = dy;
        s_tdx[n] = dx;
        s_trs[n] = r * g.S + s;
        ++n;
      }
    }
    s_ntaps = n;
  }
  __syncthreads();
  const int ntaps = s_ntaps;
  const int ntail = crem * ntaps;  // host guarantees <= V2_TAIL
  for (int i = tid; i < ntail; i += 256) {
    const int c = i / ntaps, t = i - c * ntaps;
    s_kc[i] = cfull * BK + c;
    s_kdy[i] = s_tdy[t];
    s_kdx[i] = s_tdx[t];
    s_krs[i] = s_trs[t];
  }
  __syncthreads();
  const int kmain = ntaps * cfull;
  const int ksteps_all = kmain + (ntail + BK - 1) / BK;
  const int kbeg = split * kper;
  const int kend = min(ksteps_all, kbeg + kper);
  const int nk = max(0, kend - kbeg);

  const int Hs = MODE == 0 ? g.H : g.P, Ws = MODE == 0 ? g.W : g.Q;
  const int HWs = Hs * Ws;
  const __amdgpu_buffer_rsrc_t rw = rsrc(w, 4LL * g.Cout * g.Cin * RS);
  const __amdgpu_buffer_rsrc_t rx = rsrc(src, 4LL * g.N * Kc * HWs);
  const int nrw = (int)min(4LL * g.Cout * g.Cin * RS, 0x7fffffffLL);
  const int nrx = (int)min(4LL * g.N * Kc * HWs, 0x7fffffffLL);
  const int tapstride = g.Cout * g.Cin;   // tap-major weights [RS][Cout][Cin]

  // B: this thread's column and k-group
  const int bn = tid % BN, kg = tid / BN;
  const int ncol = n0 + bn;
  const bool col_ok = ncol < Ntot;
  int img = 0, cp = 0;
  if (col_ok) {
    img = ncol / HWc;
    cp = ncol - img * HWc;
  }
  const int cy = cp / Wc, cx = cp - cy * Wc;
  const int ybase = MODE == 0 ? cy * g.sh : cy;
  const int xbase = MODE == 0 ? cx * g.sw : cx;
  const int simg = img * Kc * HWs;
  // A: MODE 0 thread = (row tid/4, k quad tid%4), channels contiguous in memory (float4
  // when Cin % 4 == 0); MODE 1 thread = (row tid%64, k quad tid/64), rows contiguous in
  // memory (lanes coalesce along ci)
  const int am = MODE == 0 ? tid >> 2 : tid & 63;
  const int akq = MODE == 0 ? tid & 3 : tid >> 6;
  const bool arow_ok = m0 + am < M;
  const bool avec = MODE == 0 && (g.Cin & 3) == 0;

  float ra[4], rb[RPT];
  const int klast = kend - 1;
  auto load_tiles = [&](int ks_in) {
    const bool live = ks_in <= klast;
    const int ks = min(ks_in, klast);
    if (ks < kmain) {                                  // full step: one tap, 16 channels
      const int tap = g.korder ? ks % ntaps : ks / cfull;
      const int c0 = (g.korder ? ks / ntaps : ks - tap * cfull) * BK;
      const int dy = s_tdy[tap], dx = s_tdx[tap], rs = s_trs[tap] * tapstride;
      if (MODE == 0) {
        const int c = c0 + 4 * akq;
        const int base = (live && arow_ok) ? (rs + (m0 + am) * g.Cin + c) * 4 : nrw;
        if (avec) {
          const float4 v = bload4(rw, base);
          ra[0] = v.x; ra[1] = v.y; ra[2] = v.z; ra[3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) ra[j] = bload(rw, base + 4 * j);
        }
      } else {
        // A[m = ci][k = co]: w[rs][co][ci]
        const int base = (live && arow_ok) ? (rs + (c0 + 4 * akq) * g.Cin + m0 + am) * 4 : nrw;
#pragma unroll
        for (int j = 0; j < 4; ++j) ra[j] = bload(rw, base + j * g.Cin * 4);
      }
      const int iy = ybase + dy, ix = xbase + dx;
      const bool pix_ok = live && col_ok && (unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws;
      const int bbase = pix_ok ? (simg + (c0 + kg * RPT) * HWs + iy * Ws + ix) * 4 : nrx;
#pragma unroll
      for (int r = 0; r < RPT; ++r) rb[r] = bload(rx, bbase + r * HWs * 4);
    } else {                                           // tail step: 16 flattened rows
      const int t0 = (ks - kmain) * BK;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = t0 + 4 * akq + j;
        const bool ok = live && arow_ok && i < ntail;
        const int ii = ok ? i : 0;
        const int c = s_kc[ii], rs = s_krs[ii] * tapstride;
        ra[j] = bload(rw, ok ? (MODE == 0 ? (rs + (m0 + am) * g.Cin + c) : (rs + c * g.Cin + m0 + am)) * 4
                              : OOR);
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int i = t0 + kg * RPT + r;
        const int ii = i < ntail ? i : 0;
        const int iy = ybase + s_kdy[ii], ix = xbase + s_kdx[ii];
        const bool ok = live && col_ok && i < ntail && (unsigned)iy < (unsigned)Hs &&
                        (unsigned)ix < (unsigned)Ws;
        rb[r] = bload(rx, ok ? (simg + s_kc[ii] * HWs + iy * Ws + ix) * 4 : OOR);
      }
    }
  };
  auto store_tiles = [&](int buf) {
    *reinterpret_cast<float4 *>(&As[buf][am][4 * akq]) = make_float4(ra[0], ra[1], ra[2], ra[3]);
#pragma unroll
    for (int r = 0; r < RPT; r += 4)
      *reinterpret_cast<float4 *>(&Bs[buf][bn][kg * RPT + r]) =
          make_float4(rb[r], rb[r + 1], rb[r + 2], rb[r + 3]);
  };

  f32x16 acc[WNT];
#pragma unroll
  for (int t = 0; t < WNT; ++t) acc[t] = f32x16{0};
  const int li = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    const float4 a0 = *reinterpret_cast<const float4 *>(&As[buf][32 * wm + li][8 * lh]);
    const float4 a1 = *reinterpret_cast<const float4 *>(&As[buf][32 * wm + li][8 * lh + 4]);
    const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    bf16x8 abf;
    f16x8 ah;
    if (OP == 1) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) abf[kk] = (__bf16)a[kk];
    } else if (OP == 2) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) ah[kk] = (_Float16)a[kk];
    }
#pragma unroll
    for (int t = 0; t < WNT; ++t) {
      const int col = 32 * WNT * wn + 32 * t + li;
      const float4 b0 = *reinterpret_cast<const float4 *>(&Bs[buf][col][8 * lh]);
      const float4 b1 = *reinterpret_cast<const float4 *>(&Bs[buf][col][8 * lh + 4]);
      const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      if (OP == 0) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk], b[kk], acc[t], 0, 0, 0);
      } else if (OP == 1) {
        bf16x8 bb;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) bb[kk] = (__bf16)b[kk];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(abf, bb, acc[t], 0, 0, 0);
      } else {
        f16x8 bh;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) bh[kk] = (_Float16)b[kk];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
      }
    }
  };
  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      load_tiles(kbeg + kt + 1);  // past the range: reads zeros
      __builtin_amdgcn_sched_barrier(0);  // loads first, then the step's MFMAs
      compute(kt & 1);
      // all of the step's MFMAs before the LDS write (hipcc otherwise hoists the write, and
      // its wait on the loads, into the middle of them); unconditional (the last step's zeros
      // land in the idle buffer): a conditional store lets hipcc sink the loads into its branch
      __builtin_amdgcn_sched_barrier(0);
      store_tiles((kt + 1) & 1);
      __syncthreads();
    }
  }

  // epilogue (as k_conv_gemm): C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const __amdgpu_buffer_rsrc_t rd = rsrc(dst, dst_bytes);
  const __amdgpu_buffer_rsrc_t rres = rsrc(bias, MODE == 1 && bias ? dst_bytes : 0);
  const int Hd = MODE == 0 ? g.P : g.H, Wd = MODE == 0 ? g.Q : g.W;
  const int HWd = Hd * Wd;
#pragma unroll
  for (int t = 0; t < WNT; ++t) {
    const int n = n0 + 32 * WNT * wn + 32 * t + li;
    const bool nok = n < Ntot;
    int dbase, mstride;
    if (splits == 1) {
      const int im = n / HWc;
      const int p = n - im * HWc;
      int dp = p;
      if (MODE == 1) {
        const int u = p / Wc, v = p - u * Wc;
        dp = (py + g.sh * u) * Wd + (px + g.sw * v);
      }
      dbase = im * M * HWd + dp;
      mstride = HWd;
    } else {
      dbase = split * M * Ntot + n;
      mstride = Ntot;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * lh;
      float v = acc[t][r];
      const int off = (nok && m < M) ? (dbase + m * mstride) * 4 : OOR;
      if (splits == 1) {
        if (MODE == 0) {
          if (bias) v += bias[min(m, M - 1)];
          if (ACT == 1) v = fmaxf(v, 0.f);
        } else if (bias) {
          v += bload(rres, off);
        }
      }
      bstore(rd, off, v);
    }
  }
}

// ------------------------------------------------------------------------------------------
// bwd-weight: dW[co, col] = sum_(n,p) g[n,co,p] * x[n,ci,p+tap], col = ci*R*S + tap (the
// weight layout); pixels split over blocks.  Block tile 64 (co) x 64 (col), K-step = 16
// pixels; each thread's 4 columns keep (ci, dy, dx) in registers.  Partial slab per split,
// reduced in fixed order.
// ------------------------------------------------------------------------------------------
constexpr int WBN = 64;

template <int OP, int KB>
__global__ void __launch_bounds__(256, 2) k_conv_wgrad(
    const float *__restrict__ gout, const float *__restrict__ x, float *__restrict__ part,
    ConvGeom g, int pix_per_split, TapList tl) {
  constexpr int TPR = 256 / KB;  // co / col rows per load pass
  constexpr int NJ = 64 / TPR;   // loads per thread per operand per K-step
  __shared__ float As[2][KB][BM + PADA];   // As[pixel][co]
  __shared__ float Bs[2][KB][WBN + PADB];  // Bs[pixel][col]
  __shared__ int s_tap[MAXTAPS];
  if (threadIdx.x < MAXTAPS) s_tap[threadIdx.x] = threadIdx.x < tl.n ? tl.tap[threadIdx.x] : 0;
  __syncthreads();

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int RS = g.R * g.S;
  const int Kw = g.Cin * RS;       // columns of dW (ci-major, tap-minor)
  const int Kl = g.Cin * tl.n;     // live columns this GEMM computes: (ci, live tap index)
  const int n0 = blockIdx.x * WBN;
  const int m0 = blockIdx.y * BM;
  const int split = blockIdx.z;
  const int PQ = g.P * g.Q;
  const int Ptot = g.N * PQ;
  const int pbeg = split * pix_per_split;
  const int pend = min(Ptot, pbeg + pix_per_split);
  const int HW = g.H * g.W;

  // thread -> pixel = tid % KB (same pixel for its A and B loads), co / col rows = tid / KB.
  // Guards are branch-free: an invalid element gets an offset >= the buffer size (reads 0);
  // per-column constants (channel plane + tap displacement) are folded once.
  const int tp = tid % KB, trow = tid / KB;
  const int nrg = (int)min(4LL * g.N * g.Cout * PQ, 0x7fffffffLL);
  const int nrx = (int)min(4LL * g.N * g.Cin * HW, 0x7fffffffLL);
  int cconst[NJ], cdy[NJ], cdx[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + trow + TPR * j;
    const int cc = col < Kl ? col : 0;
    const int ci = cc / tl.n, tap = s_tap[cc - ci * tl.n];
    const int r = tap / g.S, s = tap - r * g.S;
    cdy[j] = r * g.dh - g.ph;
    cdx[j] = s * g.dw - g.pw;
    cconst[j] = ci * HW + cdy[j] * g.W + cdx[j];
    // an out-of-range column gets an impossible row displacement: never in bounds
    if (col >= Kl) cdy[j] = -(1 << 29);
  }
  const int arow = (m0 + trow) * PQ;  // gout row of this thread's first co
  int p_cur = pbeg + tp;
  int im = p_cur / max(PQ, 1), od = p_cur - im * PQ;

  const __amdgpu_buffer_rsrc_t rg = rsrc(gout, 4LL * g.N * g.Cout * PQ);
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.Cin * HW);
  float ra0[NJ], rb0[NJ], ra1[NJ], rb1[NJ];  // two register sets: loads run two K-steps ahead
  auto load_tiles = [&](float(&ra)[NJ], float(&rb)[NJ]) {
    const bool pok = p_cur < pend;
    const int oy = od / g.Q, ox = od - oy * g.Q;
    const int abase = pok ? (im * g.Cout * PQ + od + arow) * 4 : nrg;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int co = m0 + trow + TPR * j;
      ra[j] = bload(rg, co < g.Cout ? abase + j * TPR * PQ * 4 : OOR);
    }
    const int yb = oy * g.sh, xb0 = ox * g.sw;
    const int pbase = im * g.Cin * HW + yb * g.W + xb0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bool ok = pok && (unsigned)(yb + cdy[j]) < (unsigned)g.H &&
                      (unsigned)(xb0 + cdx[j]) < (unsigned)g.W;
      rb[j] = bload(rx, ok ? (pbase + cconst[j]) * 4 : nrx);
    }
    p_cur += KB;
    od += KB;
    while (od >= PQ) {
      od -= PQ;
      ++im;
    }
  };
  auto store_tiles = [&](int buf, const float(&ra)[NJ], const float(&rb)[NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) As[buf][tp][trow + TPR * j] = ra[j];
#pragma unroll
    for (int j = 0; j < NJ; ++j) Bs[buf][tp][trow + TPR * j] = rb[j];
  };

  f32x16 acc = {0};
  const int nk = (pend - pbeg + KB - 1) / KB;
  const int li = lane & 31, lk = lane >> 5;
  // OP 1 (bf16 mode, BASELINE C3): one 32x32x16 bf16 MFMA per 16 pixels, lane half h taking
  // pixels 8h .. 8h+7 of them (eight LDS reads per operand, as the eight fp32 MFMAs do)
  auto compute = [&](int buf) {
    if (OP == 0) {
#pragma unroll
      for (int kk = 0; kk < KB; kk += 2) {
        const float a = As[buf][kk + lk][32 * wm + li];
        const float b = Bs[buf][kk + lk][32 * wn + li];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; kb += 16) {
        bf16x8 a, b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] = (__bf16)As[buf][kb + 8 * lk + j][32 * wm + li];
          b[j] = (__bf16)Bs[buf][kb + 8 * lk + j][32 * wn + li];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      }
    }
  };
  // unconditional loads (past the range they read zeros): exact s_waitcnt, see k_conv_gemm
  if (nk > 0) {
    load_tiles(ra0, rb0);
    store_tiles(0, ra0, rb0);
    load_tiles(ra1, rb1);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      load_tiles(ra0, rb0);
      __builtin_amdgcn_sched_barrier(0);  // loads first, then the step's MFMAs
      compute(0);
      store_tiles(1, ra1, rb1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      load_tiles(ra1, rb1);
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      store_tiles(0, ra0, rb0);
      __syncthreads();
    }
  }
  const __amdgpu_buffer_rsrc_t rp = rsrc(part, 4LL * gridDim.z * g.Cout * Kw);
  const int lcol = n0 + 32 * wn + li;
  const int lci = lcol < Kl ? lcol / tl.n : 0;
  const int col = lci * RS + s_tap[lcol < Kl ? lcol - lci * tl.n : 0];  // dW column
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int co = m0 + 32 * wm + (rr & 3) + 8 * (rr >> 2) + 4 * lk;
    const bool ok = co < g.Cout && lcol < Kl;
    bstore(rp, ok ? ((split * g.Cout + co) * Kw + col) * 4 : OOR, acc[rr]);
  }
}


// ------------------------------------------------------------------------------------------
// bwd-weight, second generation (round 3).  The same GEMM as k_conv_wgrad (M = Cout, N =
// (ci, live tap), K = pixels split over blocks into fixed-order slabs), for maps whose pixel
// count per image is a multiple of the 32-pixel K-step (every hot-path map), so a K-step never
// straddles two images:
//  * the step's image and first pixel are wave-uniform.  (k_conv_wgrad advances a per-lane
//    pixel index through the images with a divergent loop, and hipcc drains the in-flight
//    loads around it: the ISA showed vmcnt(7..1) waits before every step's loads.)
//  * LDS rows are k-contiguous ([row][32 + 4 pad]); a lane's 16 MFMA operands per step are
//    four ds_read_b128 per operand (lane half h supplies k = 16h .. 16h+15), as in k_gemm.
//  * A = g rows load as float4 along the pixels; B = the im2col x columns load one pixel per
//    lane, lanes on consecutive pixels (coalesced along the image rows).
//  * the next step's loads are issued at the top of the step (one step of lookahead).
// OP 1 (bf16, BASELINE C3): two 32x32x16 bf16 MFMAs per step on the same operand registers.
// ------------------------------------------------------------------------------------------
constexpr int W2K = 32, W2LD = 36;

constexpr int W2_LDS_FLOATS = 2 * 2 * 64 * W2LD;  // As[2][64][W2LD] (co x pixel), Bs likewise

// The block body of k_conv_wgrad2 for block (bx, by, bz) of a grid with gz splits; `lds` holds
// W2_LDS_FLOATS floats (16-B aligned) of the caller's __shared__ memory (k_conv_bwd_pair).
template <int OP>
__device__ __forceinline__ void conv_wgrad2_block(
    const float *__restrict__ gout, const float *__restrict__ x, float *__restrict__ part,
    ConvGeom g, int pix_per_split, TapList tl, int bx, int by, int bz, int gz, float *lds) {
  float(*As)[64][W2LD] = reinterpret_cast<float(*)[64][W2LD]>(lds);                 // As[co][pixel]
  float(*Bs)[64][W2LD] = reinterpret_cast<float(*)[64][W2LD]>(lds + 2 * 64 * W2LD);  // Bs[column][pixel]
  __shared__ int s_tap[MAXTAPS];
  if (threadIdx.x < MAXTAPS) s_tap[threadIdx.x] = threadIdx.x < tl.n ? tl.tap[threadIdx.x] : 0;
  __syncthreads();

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int RS = g.R * g.S;
  const int Kw = g.Cin * RS;    // columns of dW (ci-major, tap-minor)
  const int Kl = g.Cin * tl.n;  // live columns (ci, live tap index)
  const int n0 = bx * 64, m0 = by * 64;
  const int split = bz;
  const int PQ = g.P * g.Q;
  const int Ptot = g.N * PQ;
  const int pbeg = split * pix_per_split;  // a multiple of W2K
  const int pend = min(Ptot, pbeg + pix_per_split);
  const int nk = max(0, (pend - pbeg) / W2K);  // Ptot % W2K == 0: whole steps only
  const int HW = g.H * g.W;

  // A: thread = (co row tid/8 and +32, pixel quad tid%8)
  const int ar = tid >> 3, aq = tid & 7;
  // B: thread = (pixel tid%32, column group tid/32): columns bcg + 8 j
  const int bp = tid & 31, bcg = tid >> 5;
  int cconst[8], cdy[8], cdx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = n0 + bcg + 8 * j;
    const int cc = col < Kl ? col : 0;
    const int ci = cc / tl.n, tap = s_tap[cc - ci * tl.n];
    const int r = tap / g.S, sx = tap - r * g.S;
    cdy[j] = r * g.dh - g.ph;
    cdx[j] = sx * g.dw - g.pw;
    cconst[j] = ci * HW + cdy[j] * g.W + cdx[j];
    if (col >= Kl) cdy[j] = -(1 << 29);  // never in bounds
  }
  const __amdgpu_buffer_rsrc_t rg = rsrc(gout, 4LL * g.N * g.Cout * PQ);
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.Cin * HW);
  const int nrx = (int)min(4LL * g.N * g.Cin * HW, 0x7fffffffLL);

  float4 ra[2];
  float rb[8];
  // the step's (image, first pixel) and this lane's output pixel (oy, ox), advanced by W2K
  // pixels per step with carries instead of a scalar and a per-lane division per step (a step
  // never straddles images: PQ % W2K == 0)
  int im = pbeg / PQ, od0 = pbeg - im * PQ;
  int oy = (od0 + bp) / g.Q, ox = od0 + bp - oy * g.Q;
  const int q32 = W2K / g.Q, r32 = W2K - q32 * g.Q;
  auto advance = [&]() {
    od0 += W2K;
    if (od0 >= PQ) {
      od0 -= PQ;
      ++im;
    }
    ox += r32;
    oy += q32;
    if (ox >= g.Q) {
      ox -= g.Q;
      ++oy;
    }
    if (oy >= g.P) oy -= g.P;
  };
  auto load_tiles = [&](int ks) {  // ks = 0, 1, ... in order; ks >= nk re-reads step nk - 1
    if (ks > 0 && ks < nk) advance();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = m0 + ar + 32 * i;
      ra[i] = bload4(rg, co < g.Cout ? ((im * g.Cout + co) * PQ + od0 + 4 * aq) * 4 : OOR);
    }
    const int yb = oy * g.sh, xb = ox * g.sw;
    const int pbase = im * g.Cin * HW + yb * g.W + xb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = (unsigned)(yb + cdy[j]) < (unsigned)g.H && (unsigned)(xb + cdx[j]) < (unsigned)g.W;
      rb[j] = bload(rx, ok ? (pbase + cconst[j]) * 4 : nrx);
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<float4 *>(&As[buf][ar + 32 * i][4 * aq]) = ra[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) Bs[buf][bcg + 8 * j][bp] = rb[j];
  };

  f32x16 acc = {0};
  const int li = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    float a[16], b[16];
    const float *pa = &As[buf][32 * wm + li][16 * lh];
    const float *pb = &Bs[buf][32 * wn + li][16 * lh];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 u = *reinterpret_cast<const float4 *>(pa + 4 * q);
      const float4 v = *reinterpret_cast<const float4 *>(pb + 4 * q);
      a[4 * q] = u.x; a[4 * q + 1] = u.y; a[4 * q + 2] = u.z; a[4 * q + 3] = u.w;
      b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
    }
    if (OP == 0) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk], b[kk], acc, 0, 0, 0);
    } else {
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        bf16x8 av, bv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          av[j] = (__bf16)a[8 * blk + j];
          bv[j] = (__bf16)b[8 * blk + j];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
      }
    }
  };
  if (nk > 0) {
    load_tiles(0);
    store_tiles(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      load_tiles(kt + 1);
      __builtin_amdgcn_sched_barrier(0);  // loads first, then the step's MFMAs
      compute(kt & 1);
      // all of the step's MFMAs before the LDS write (hipcc otherwise hoists the write, and its
      // wait on the loads, into the middle of them); unconditional (the last step's copy lands
      // in the idle buffer and is never read): a conditional store lets hipcc sink the B loads
      // into its branch, behind the MFMAs
      __builtin_amdgcn_sched_barrier(0);
      store_tiles((kt + 1) & 1);
      __syncthreads();
    }
  }
  const __amdgpu_buffer_rsrc_t rp = rsrc(part, 4LL * gz * g.Cout * Kw);
  const int lcol = n0 + 32 * wn + li;
  const int lci = lcol < Kl ? lcol / tl.n : 0;
  const int col = lci * RS + s_tap[lcol < Kl ? lcol - lci * tl.n : 0];  // dW column
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int co = m0 + 32 * wm + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
    const bool ok = co < g.Cout && lcol < Kl;
    bstore(rp, ok ? ((split * g.Cout + co) * Kw + col) * 4 : OOR, acc[rr]);
  }
}

template <int OP>
__global__ void __launch_bounds__(256) k_conv_wgrad2(
    const float *__restrict__ gout, const float *__restrict__ x, float *__restrict__ part,
    ConvGeom g, int pix_per_split, TapList tl) {
  __shared__ __attribute__((aligned(16))) float lds[W2_LDS_FLOATS];
  conv_wgrad2_block<OP>(gout, x, part, g, pix_per_split, tl, blockIdx.x, blockIdx.y, blockIdx.z,
                        gridDim.z, lds);
}

// A conv layer's data gradient (k_conv_gemm MODE 1, fp32) and spatial / small-map weight
// gradient (k_conv_wgrad2, fp32) in one grid: blocks [0, n1) run the data gradient, the rest
// the weight gradient's split slabs (reduced by k_reduce_splits after the launch).  One launch
// instead of two on forked streams (e2ep_conv_bwd): in a replayed graph a fork / join costs
// ~5 + ~10 us of idle GPU, and the 16 x 16 / 32 x 32 layers' gradients take 20 - 50 us each.
template <int BNT, int BMT>
__global__ void __launch_bounds__(256, 2) k_conv_bwd_pair(
    const float *__restrict__ w, const float *__restrict__ gout, const float *__restrict__ res,
    float *__restrict__ dx, long long dx_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part1, unsigned int *__restrict__ cnt, int gx1, int gy1, int gz1,
    const float *__restrict__ x, float *__restrict__ part2, int pix_per_split, TapList tl,
    int gx2, int gy2, int gz2) {
  constexpr int L1 = conv_gemm_lds_floats<BNT, BMT>();
  constexpr int L = L1 > W2_LDS_FLOATS ? L1 : W2_LDS_FLOATS;
  __shared__ __attribute__((aligned(16))) float lds[L];
  // data-gradient blocks [0, n1) first: the weight-gradient-first order measured 0.15 ms/step
  // slower in C2 and C3 (profiles/r04/conv_pair_order_ab.txt; the switch is retired)
  const int n1 = gx1 * gy1 * gz1;
  int id = blockIdx.x;
  if (id < n1) {
    conv_gemm_block<1, 0, BNT, BMT, false, 0, false>(w, gout, res, dx, dx_bytes, g, M, splits, kper,
                                                     part1, cnt, nullptr, id % gx1,
                                                     (id / gx1) % gy1, id / (gx1 * gy1), gx1, lds);
  } else {
    id -= n1;
    conv_wgrad2_block<0>(gout, x, part2, g, pix_per_split, tl, id % gx2, (id / gx2) % gy2,
                         id / (gx2 * gy2), gz2, lds);
  }
}

// ------------------------------------------------------------------------------------------
// bwd-weight of 1x1 / stride-1 / unpadded convs (the EfficientNet expand / project convs,
// the BEV heads' 1x1s): dW[co][ci] = sum_q g[co][q] x[ci][q] over all pixels q.  No LDS, no
// barrier in the main loop: each wave owns a 32 (co) x 32 (ci) tile and a pixel range, and
// loads its MFMA operands straight from memory as float4s along the pixel axis — lane l
// reads 4 consecutive pixels of row l%32 (g for A, x for B), and MFMA t of a group takes
// element t of every lane (the K axis is reordered within each 8-pixel group; the sum is the
// same and its order fixed).  The four waves of a block split the block's pixel range and
// are summed in LDS in wave order; slabs per split are reduced by k_reduce_splits.  Wave
// tiles are 32x32 or, when both channel counts fill them, 64x64 (four accumulators sharing
// each loaded operand: half the L1/L2 operand traffic per MFMA).
// ------------------------------------------------------------------------------------------
constexpr int W1_GROUPS = 4;  // 8-pixel groups per wave iteration (8 float4 loads in flight)

// Used for large pixel counts with few channel pairs (the early EfficientNet stages, the
// segmentation classifier); elsewhere the LDS-tiled k_conv_wgrad reads each operand row once
// per 64x64 tile instead of once per 32x32 wave tile and is faster (scripts/bench_conv.py).
static bool wgrad1x1_ok(const ConvGeom &g) {
  const long long pix = (long long)g.N * g.P * g.Q;
  return g.R == 1 && g.S == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0 &&
         g.P == g.H && g.Q == g.W && (g.P * g.Q) % 8 == 0 && pix >= 131072 &&
         (pix >= 200000 || (long long)g.Cout * g.Cin <= 6144);
}

static int wgrad1x1_splits_for(const ConvGeom &g, int to, int tc) {
  const long long tiles = (long long)cdiv(g.Cout, to) * cdiv(g.Cin, tc);
  const long long pix = (long long)g.N * g.P * g.Q;
  long long want = (g_tune[TUNE_WGRAD1X1_TARGET] + tiles - 1) / tiles;   // e2ep_tune key 3 / 5
  long long cap = pix / 2048;                    // >= 16 loop iterations per wave
  long long s = want < cap ? want : cap;
  if (s < 1) s = 1;
  if (s > 4096) s = 4096;
  return (int)s;
}

// Wave tile rows per channel axis (Cout, Cin): 64 where that pads the axis at most 1/8 beyond
// 32-row tiles, but only for large pixel counts whose 64-row grid still has >= 128 workgroups
// (smaller problems are latency-bound and want the wider grid; scripts/bench_conv.py).
static void wgrad1x1_tiles(const ConvGeom &g, int &to, int &tc) {
  auto wide = [](int c) { return 8LL * cdiv(c, 64) * 64 <= 9LL * cdiv(c, 32) * 32; };
  to = tc = 32;
  if ((long long)g.N * g.P * g.Q < 65536) return;
  const int wo = wide(g.Cout) ? 64 : 32, wc = wide(g.Cin) ? 64 : 32;
  if ((long long)cdiv(g.Cout, wo) * cdiv(g.Cin, wc) * wgrad1x1_splits_for(g, wo, wc) < 128) return;
  to = wo;
  tc = wc;
}

static int wgrad1x1_splits(const ConvGeom &g) {
  int to, tc;
  wgrad1x1_tiles(g, to, tc);
  return wgrad1x1_splits_for(g, to, tc);
}

// The block body for tile bt of split `split`, its wave-sum tile in the caller's LDS
// (red[TI * TJ * 16][64]): k_wgrad_1x1, and the weight-gradient half of k_conv_bwd_pair1x1.
template <int TI, int TJ, int OP>
__device__ __forceinline__ void wgrad1x1_block(const float *__restrict__ gout,
                                               const float *__restrict__ x,
                                               float *__restrict__ part, ConvGeom g, int splits,
                                               int groups_per_split, int bt, int split,
                                               float (*red)[64]) {
  // wave tile (32*TI co) x (32*TJ ci): TI*TJ accumulators share each loaded operand
  constexpr int NT = TI * TJ;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntj = (g.Cin + 32 * TJ - 1) / (32 * TJ);
  const int ti = bt / ntj, tj = bt - ti * ntj;
  const int PQ = g.P * g.Q;
  const int ngroups = g.N * PQ / 8;  // 8-pixel groups (never straddle an image: PQ % 8 == 0)
  const int gb = split * groups_per_split;
  const int ge = min(ngroups, gb + groups_per_split);
  const int row = lane & 31, h = lane >> 5;
  const int co0 = ti * 32 * TI + row, ci0 = tj * 32 * TJ + row;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gout, 4LL * g.N * g.Cout * PQ);
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.Cin * PQ);
  const int gpq = PQ / 8;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{0};
  // wave w takes groups gb + w*W1_GROUPS + 4*W1_GROUPS*i ...
  for (int g0 = gb + wave * W1_GROUPS; g0 < ge; g0 += 4 * W1_GROUPS) {
    float4 a[W1_GROUPS][TI], b[W1_GROUPS][TJ];
#pragma unroll
    for (int u = 0; u < W1_GROUPS; ++u) {
      const int grp = g0 + u;
      const bool ok = grp < ge;
      const int n = grp / gpq, p = (grp - n * gpq) * 8 + 4 * h;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + 32 * i;
        a[u][i] = bload4(rg, (ok && co < g.Cout) ? (((n * g.Cout + co) * PQ) + p) * 4 : OOR);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int ci = ci0 + 32 * j;
        b[u][j] = bload4(rx, (ok && ci < g.Cin) ? (((n * g.Cin + ci) * PQ) + p) * 4 : OOR);
      }
    }
    if (OP == 0) {
#pragma unroll
      for (int u = 0; u < W1_GROUPS; ++u)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            f32x16 &c = acc[i * TJ + j];
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i].x, b[u][j].x, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i].y, b[u][j].y, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i].z, b[u][j].z, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i].w, b[u][j].w, c, 0, 0, 0);
          }
    } else {
      // bf16 mode: groups u, u+1 (16 pixels) feed one 32x32x16 MFMA; lane half h holds
      // pixels 4h..4h+3 of each group, identically for both operands
#pragma unroll
      for (int u = 0; u < W1_GROUPS; u += 2)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            const bf16x8 av = {(__bf16)a[u][i].x, (__bf16)a[u][i].y, (__bf16)a[u][i].z,
                               (__bf16)a[u][i].w, (__bf16)a[u + 1][i].x, (__bf16)a[u + 1][i].y,
                               (__bf16)a[u + 1][i].z, (__bf16)a[u + 1][i].w};
            const bf16x8 bv = {(__bf16)b[u][j].x, (__bf16)b[u][j].y, (__bf16)b[u][j].z,
                               (__bf16)b[u][j].w, (__bf16)b[u + 1][j].x, (__bf16)b[u + 1][j].y,
                               (__bf16)b[u + 1][j].z, (__bf16)b[u + 1][j].w};
            acc[i * TJ + j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i * TJ + j], 0, 0, 0);
          }
    }
  }
  // the four waves' tiles are summed in wave order through one LDS tile
  for (int w = 0; w < 4; ++w) {
    if (wave == w)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          red[t * 16 + r][lane] = w == 0 ? acc[t][r] : red[t * 16 + r][lane] + acc[t][r];
    __syncthreads();
  }
  // C layout: element r of lane l is (i, j) = ((r&3) + 8*(r>>2) + 4*(l>>5), l&31)
  const int Kw = g.Cin;
  for (int e = threadIdx.x; e < NT * 16 * 64; e += 256) {
    const int tr = e >> 6, l = e & 63;
    const int t = tr >> 4, r = tr & 15;
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), j = l & 31;
    const int oc = ti * 32 * TI + 32 * (t / TJ) + i, ic = tj * 32 * TJ + 32 * (t % TJ) + j;
    if (oc < g.Cout && ic < g.Cin) {
      part[((long long)split * g.Cout + oc) * Kw + ic] = red[tr][l];
    }
  }
}

template <int TI, int TJ, int OP>
__global__ void __launch_bounds__(256) k_wgrad_1x1(const float *__restrict__ gout,
                                                   const float *__restrict__ x,
                                                   float *__restrict__ part, ConvGeom g,
                                                   int splits, int groups_per_split) {
  __shared__ float red[TI * TJ * 16][64];
  wgrad1x1_block<TI, TJ, OP>(gout, x, part, g, splits, groups_per_split, blockIdx.x, blockIdx.y,
                             red);
}

// A 1x1 conv layer's data gradient (k_conv_gemm MODE 1, fp32) and weight gradient (the
// LDS-free k_wgrad_1x1 wave tiles: the large-map EfficientNet expand / project convs) in one
// grid, as k_conv_bwd_pair; wfirst puts the weight-gradient blocks first (e2ep_tune key 30,
// the default: each walks a long pixel range, the long poles of the launch; C2 22.73 -> 22.50
// ms against data-gradient-first, profiles/r04/conv_pair1x1_ab.txt).
template <int BNT, int BMT, int TI, int TJ>
__global__ void __launch_bounds__(256, 2) k_conv_bwd_pair1x1(
    const float *__restrict__ w, const float *__restrict__ gout, const float *__restrict__ res,
    float *__restrict__ dx, long long dx_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part1, unsigned int *__restrict__ cnt, int gx1, int gy1, int gz1,
    const float *__restrict__ x, float *__restrict__ part2, int splits2, int gps, int nt2,
    int wfirst) {
  constexpr int L1 = conv_gemm_lds_floats<BNT, BMT>();
  constexpr int L2 = TI * TJ * 16 * 64;
  __shared__ __attribute__((aligned(16))) float lds[L1 > L2 ? L1 : L2];
  const int n1 = gx1 * gy1 * gz1, n2 = nt2 * splits2;
  const int id = wfirst ? ((int)blockIdx.x >= n2 ? (int)blockIdx.x - n2 : n1 + (int)blockIdx.x)
                        : (int)blockIdx.x;
  if (id < n1) {
    conv_gemm_block<1, 0, BNT, BMT, false, 0, false>(w, gout, res, dx, dx_bytes, g, M, splits, kper,
                                                     part1, cnt, nullptr, id % gx1,
                                                     (id / gx1) % gy1, id / (gx1 * gy1), gx1, lds);
  } else {
    const int j = id - n1;
    wgrad1x1_block<TI, TJ, 0>(gout, x, part2, g, splits2, gps, j % nt2, j / nt2,
                              reinterpret_cast<float(*)[64]>(lds));
  }
}

// fixed-order sum of the split slabs (+ optional accumulate into an existing gradient).
// Block = 64 outputs x 16 split lanes: thread (o, r) sums splits r, r+16, ... with 4
// independent chains, then the 16 lane sums are added in order through LDS.
// Entries i whose tap (i % RS) is not live in `mask` are never written by the GEMM: their
// result is 0 (a weight tap that only ever meets zero padding).
__global__ void __launch_bounds__(1024) k_reduce_splits(const float *__restrict__ part, int splits,
                                                        int n, float *__restrict__ out,
                                                        int accumulate, int RS,
                                                        unsigned long long mask) {
  __shared__ float red[16][64];
  const int o = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + o;
  const bool live = (mask >> (i % RS)) & 1ULL;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n && live) {
    int k = r;
    for (; k + 48 < splits; k += 64) {
      s0 += part[(size_t)(k + 0) * n + i];
      s1 += part[(size_t)(k + 16) * n + i];
      s2 += part[(size_t)(k + 32) * n + i];
      s3 += part[(size_t)(k + 48) * n + i];
    }
    for (; k < splits; k += 16) s0 += part[(size_t)k * n + i];
  }
  red[r][o] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (r == 0 && i < n) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += red[j][o];
    out[i] = accumulate ? out[i] + s : s;
  }
}

// The same reduction, four consecutive outputs per thread (n % 4 == 0): float4 loads of every
// slab in split order, summed in that order.  The 16-lane tree above runs ~1.4 loads per
// thread and left the launch latency-bound (15 us for the 13.5 MB of slabs of a 16x16 1x1
// conv's weight gradient, ~1 TB/s); here each thread keeps all its slab loads in flight.
__global__ void __launch_bounds__(256) k_reduce_splits4(const float *__restrict__ part, int splits,
                                                         int n, float *__restrict__ out,
                                                         int accumulate, int RS,
                                                         unsigned long long mask) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  float4 acc = *reinterpret_cast<const float4 *>(part + i);
#pragma unroll 8
  for (int k = 1; k < splits; ++k) {
    const float4 v = *reinterpret_cast<const float4 *>(part + (size_t)k * n + i);
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  float r[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (!((mask >> ((i + e) % RS)) & 1ULL)) r[e] = 0.f;  // dead tap: never written by the GEMM
  float4 o = make_float4(r[0], r[1], r[2], r[3]);
  if (accumulate) {
    const float4 a = *reinterpret_cast<const float4 *>(out + i);
    o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
  }
  *reinterpret_cast<float4 *>(out + i) = o;
}

// fixed-order split-K reduction of the weight-gradient slabs: the float4 kernel when it has
// enough threads to fill the chip (>= 32768: one per 4 outputs) and few slabs each; the split-
// lane kernel otherwise (small weights with hundreds of slabs, e.g. the 1x1 weight gradients
// of the 128x128 maps: one float4 thread per 4 outputs serialises those, 27 -> 39 us)
static void reduce_splits(const float *part, int splits, int n, float *out, int accumulate, int RS,
                          unsigned long long mask, hipStream_t s) {
  if (n % 4 == 0 && n >= 131072 && splits <= 64 && (reinterpret_cast<uintptr_t>(part) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 15) == 0)
    hipLaunchKernelGGL(k_reduce_splits4, dim3(cdiv(n / 4, 256)), dim3(256), 0, s, part, splits, n,
                       out, accumulate, RS, mask);
  else
    hipLaunchKernelGGL(k_reduce_splits, dim3(cdiv(n, 64)), dim3(1024), 0, s, part, splits, n, out,
                       accumulate, RS, mask);
}

// per-channel bias gradient: db[c] = sum over (n, p) of g[n, c, p]  (one block per channel)
// Column sums of a row-major [rows][C] matrix (Linear bias gradients, reference
// torch.nn.Linear backward inside the transformer layers): stage 1, block = 64 columns x 4
// row lanes over one row chunk, coalesced 256-B row reads, fixed-order LDS reduction into
// partial[chunk][C]; stage 2 sums the chunks in order.  Deterministic.
constexpr int COLSUM_ROWS = 128;  // rows per chunk
__global__ void __launch_bounds__(256) k_col_sum_partial(const float *__restrict__ g, int rows,
                                                         int C, float *__restrict__ part) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * COLSUM_ROWS, r1 = min(rows, r0 + COLSUM_ROWS);
  float s = 0.f;
  if (c < C) {
    float t[COLSUM_ROWS / 4];
#pragma unroll
    for (int u = 0; u < COLSUM_ROWS / 4; ++u) {
      const int r = r0 + ty + 4 * u;
      t[u] = r < r1 ? g[(long long)r * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < COLSUM_ROWS / 4; ++u) s += t[u];
  }
  __shared__ float red[4][64];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C)
    part[(long long)blockIdx.y * C + c] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

__global__ void k_col_sum_final(const float *__restrict__ part, int chunks, int C,
                                float *__restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k0 = 0; k0 < chunks; k0 += 16) {  // 16 independent loads in flight, summed in order
    float t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) t[u] = k0 + u < chunks ? part[(long long)(k0 + u) * C + c] : 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) s += t[u];
  }
  out[c] = s;
}

__global__ void __launch_bounds__(1024) k_bias_grad(const float *__restrict__ g, int N, int C,
                                                    int HW, float *__restrict__ db) {
  // one workgroup per channel; its N rows of HW are walked as one sequence (float4 when
  // HW % 4 == 0), fixed-order reduction
  const int c = blockIdx.x;
  float s = 0.f;
  if ((HW & 3) == 0) {
    const int HW4 = HW >> 2, tot = N * HW4;
    for (int t = threadIdx.x; t < tot; t += 1024) {
      const int n = t / HW4, p = t - n * HW4;
      const float4 v = *reinterpret_cast<const float4 *>(g + ((size_t)n * C + c) * HW + 4 * p);
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    const int tot = N * HW;
    for (int t = threadIdx.x; t < tot; t += 1024) {
      const int n = t / HW, p = t - n * HW;
      s += g[((size_t)n * C + c) * HW + p];
    }
  }
  __shared__ float red[16];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w];
    db[c] = t;
  }
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

// ------------------------------------------------------------------------------------------
// Direct forward convolution for tiny reduction depth (Cin*R*S <= 32, R*S > 1) and
// Cout <= 64: the EfficientNet stem (3 -> 48, 3x3/2).  As an implicit GEMM its K = 27 pads
// to a 16-channel step per tap (9 MFMA K-steps for 27 useful products); directly it is one
// pass over the input and the output (HBM-bound).
// ------------------------------------------------------------------------------------------
constexpr int DK = 32;  // max Cin*R*S

__device__ __forceinline__ int dk_w_index(const ConvGeom &g, int co, int k) {
  const int RS = g.R * g.S, ci = k / RS, rs = k - ci * RS;
  return g.wlayout == 1 ? (rs * g.Cout + co) * g.Cin + ci : (co * g.Cin + ci) * RS + rs;
}

// im2col row of output pixel (oy, ox) of image img: xin[k], k = ci*R*S + r*S + s (zero pad)
__device__ __forceinline__ void dk_gather(const ConvGeom &g, const __amdgpu_buffer_rsrc_t &rx,
                                          int img, int oy, int ox, bool ok, float (&xin)[DK]) {
  const int RS = g.R * g.S, K = g.Cin * RS;
#pragma unroll
  for (int k = 0; k < DK; ++k) {
    const int ci = k / RS, rs = k - ci * RS, r = rs / g.S, sx = rs - r * g.S;
    const int iy = oy * g.sh - g.ph + r * g.dh, ix = ox * g.sw - g.pw + sx * g.dw;
    const bool in = ok && k < K && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    xin[k] = bload(rx, in ? (((img * g.Cin + ci) * g.H + iy) * g.W + ix) * 4 : OOR);
  }
}

// forward: thread per output pixel, all Cout channels in chunks of 16; weights [k][co] in LDS
// (every lane reads the same word: broadcast)
constexpr int DCO = 64, DCH = 16;
__global__ void __launch_bounds__(256) k_conv_direct(const float *__restrict__ x,
                                                     const float *__restrict__ w,
                                                     const float *__restrict__ bias, ConvGeom g,
                                                     int act, float *__restrict__ y) {
  __shared__ float4 wl[DK][DCO / 4];
  __shared__ float xs[DK][256];  // this block's im2col rows, k-major (thread-contiguous)
  const int K = g.Cin * g.R * g.S;
  for (int e = threadIdx.x; e < DK * DCO; e += 256) {
    const int k = e / DCO, co = e - k * DCO;
    reinterpret_cast<float *>(wl)[e] = (k < K && co < g.Cout) ? w[dk_w_index(g, co, k)] : 0.f;
  }
  const int PQ = g.P * g.Q;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const bool ok = pix < g.N * PQ;
  const int img = ok ? pix / PQ : 0, pq = ok ? pix - img * PQ : 0;
  const int oy = pq / g.Q, ox = pq - oy * g.Q;
  {
    const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.Cin * g.H * g.W);
    float xin[DK];
    dk_gather(g, rx, img, oy, ox, ok, xin);
#pragma unroll
    for (int k = 0; k < DK; ++k) xs[k][threadIdx.x] = xin[k];
  }
  __syncthreads();
  float *yp = y + (size_t)img * g.Cout * PQ + pq;
#pragma unroll 1
  for (int c0 = 0; c0 < g.Cout; c0 += DCH) {
    float acc[DCH];
#pragma unroll
    for (int j = 0; j < DCH; ++j) acc[j] = 0.f;
#pragma unroll 4
    for (int k = 0; k < K; ++k) {
      const float xv = xs[k][threadIdx.x];
#pragma unroll
      for (int j4 = 0; j4 < DCH / 4; ++j4) {
        const float4 wv = wl[k][c0 / 4 + j4];
        acc[4 * j4 + 0] = __builtin_fmaf(xv, wv.x, acc[4 * j4 + 0]);
        acc[4 * j4 + 1] = __builtin_fmaf(xv, wv.y, acc[4 * j4 + 1]);
        acc[4 * j4 + 2] = __builtin_fmaf(xv, wv.z, acc[4 * j4 + 2]);
        acc[4 * j4 + 3] = __builtin_fmaf(xv, wv.w, acc[4 * j4 + 3]);
      }
    }
    if (ok) {
#pragma unroll
      for (int j = 0; j < DCH; ++j) {
        const int co = c0 + j;
        if (co < g.Cout) {
          float v = acc[j] + (bias ? bias[co] : 0.f);
          if (act == 1) v = fmaxf(v, 0.f);
          yp[(size_t)co * PQ] = v;
        }
      }
    }
  }
}

// forward only (the weight gradient stays on the split-K GEMM: measured faster), and only
// for R x S > 1 (a 1x1 with K <= 32 is already a plain GEMM with no tap padding)
static bool direct_ok(const ConvGeom &g) {
  return g.R * g.S > 1 && g.Cin * g.R * g.S <= DK && g.Cout <= DCO;
}

}  // namespace e2ep

using namespace e2ep;

static ConvGeom make_geom(const int *d) {
  ConvGeom g;
  g.N = d[0]; g.Cin = d[1]; g.H = d[2]; g.W = d[3];
  g.Cout = d[4]; g.R = d[5]; g.S = d[6]; g.P = d[7]; g.Q = d[8];
  g.sh = d[9]; g.sw = d[10]; g.ph = d[11]; g.pw = d[12]; g.dh = d[13]; g.dw = d[14];
  g.wlayout = 0;
  g.korder = 0;  // set by korder_of() at launch
  g.xcd = g_tune[TUNE_XCD] == 2;
  return g;
}

static bool geom_ok(const ConvGeom &g) {
  return g.N > 0 && g.Cin > 0 && g.H > 0 && g.W > 0 && g.Cout > 0 && g.R > 0 && g.S > 0 &&
         g.P > 0 && g.Q > 0 && g.sh > 0 && g.sw > 0 && g.dh > 0 && g.dw > 0 && g.ph >= 0 &&
         g.pw >= 0 && g.R * g.S <= MAXTAPS && g.sh * g.sw <= MAXPH &&
         4LL * g.N * g.Cin * g.H * g.W < (1LL << 31) && 4LL * g.N * g.Cout * g.P * g.Q < (1LL << 31);
}


// live taps of one axis (the kernels' tap tables apply the same rules): forward, or data-
// gradient phase p (stride-phase split, cols = the phase's column count)
static int live_taps_axis(int mode, int p, int pad, int K, int dil, int st, int n_in, int n_out,
                          int cols) {
  int n = 0;
  for (int r = 0; r < K; ++r) {
    if (mode == 0) {
      n += axis_live(r * dil - pad, n_out, st, n_in);
    } else {
      const int v = p + pad - r * dil;
      if (((v % st) + st) % st) continue;
      n += axis_live(floordiv(v, st), cols, 1, n_out);
    }
  }
  return n;
}

static TapList live_taps(const ConvGeom &g) {
  TapList t;
  t.n = 0;
  t.mask = 0;
  for (int r = 0; r < g.R; ++r)
    for (int c = 0; c < g.S; ++c)
      if (axis_live(r * g.dh - g.ph, g.P, g.sh, g.H) && axis_live(c * g.dw - g.pw, g.Q, g.sw, g.W)) {
        t.tap[t.n++] = r * g.S + c;
        t.mask |= 1ULL << (r * g.S + c);
      }
  return t;
}

struct GemmPlan {
  int bm, bnt, splits, kper, nph;
  long long ncols;  // columns of the largest phase
};

// Deterministic launch plan shared by the workspace query and the launch.
// split-K plan of the forward / data-gradient GEMMs (e2ep_conv_split_params, A/B timing)
static int g_split_target = 1024, g_split_thresh = 512;
static int g_wgrad_target = 1024;  // workgroups the spatial weight-gradient split aims at

static GemmPlan plan_gemm(int mode, const ConvGeom &g, int M) {
  GemmPlan p;
  const int Kc = mode == 0 ? g.Cin : g.Cout;
  const int csteps = cdiv(Kc, BK);
  int kmax;
  p.nph = mode ? g.sh * g.sw : 1;
  if (mode == 0) {
    p.ncols = (long long)g.N * g.P * g.Q;
    kmax = live_taps_axis(0, 0, g.ph, g.R, g.dh, g.sh, g.H, g.P, 0) *
           live_taps_axis(0, 0, g.pw, g.S, g.dw, g.sw, g.W, g.Q, 0) * csteps;
  } else {
    p.ncols = 0;
    kmax = 0;
    for (int z = 0; z < p.nph; ++z) {
      const int py = z / g.sw, px = z % g.sw;
      const long long Hp = py < g.H ? (g.H - py + g.sh - 1) / g.sh : 0;
      const long long Wp = px < g.W ? (g.W - px + g.sw - 1) / g.sw : 0;
      p.ncols = std::max(p.ncols, (long long)g.N * Hp * Wp);
      const int taps = live_taps_axis(1, py, g.ph, g.R, g.dh, g.sh, g.H, g.P, (int)Hp) *
                       live_taps_axis(1, px, g.pw, g.S, g.dw, g.sw, g.W, g.Q, (int)Wp);
      kmax = std::max(kmax, taps * csteps);
    }
  }
  // 32-row tiles when 64-row tiles would pad M by more than 25 % (M = 24, 32, 96; measured:
  // for smaller savings the wider tile's better reuse wins, scripts/bench_conv.py)
  p.bm = 5LL * cdiv(M, 32) * 32 <= 4LL * cdiv(M, 64) * 64 ? 32 : 64;
  const long long mblocks0 = cdiv(M, p.bm);
  const int wide_n = p.bm == 64 ? 128 : 256;
  p.bnt = cdiv(p.ncols, wide_n) * mblocks0 * p.nph >= g_tune[TUNE_CONV_WIDE_MIN] ? wide_n : wide_n / 2;
  // benchmarking override of the tile (e2ep_tune key 7 = bm * 1000 + bnt; 1 = automatic)
  const int ft = g_tune[TUNE_CONV_FORCE_TILE];
  if (ft > 1) {
    const int fbm = ft / 1000, fbn = ft % 1000;
    if ((fbm == 64 && (fbn == 64 || fbn == 128)) || (fbm == 32 && (fbn == 128 || fbn == 256))) {
      p.bm = fbm;
      p.bnt = fbn;
    }
  }
  const long long mblocks = cdiv(M, p.bm);
  const long long blocks = cdiv(p.ncols, p.bnt) * mblocks * p.nph;
  p.splits = 1;
  // split K when the grid cannot fill the chip twice over (measured best: aim at ~1024
  // workgroups below 512, scripts/bench_conv.py)
  const int target = g_split_target, thresh = g_split_thresh;
  if (blocks < thresh && p.nph == 1) {
    int s = (int)((target + blocks - 1) / blocks);
    s = std::min(s, std::max(1, kmax / 4));
    s = std::min(s, 32);
    p.splits = std::max(1, s);
  }
  // benchmarking override of the K split (e2ep_tune key 8 = splits + 1; 1 = automatic)
  if (g_tune[TUNE_CONV_FORCE_SPLITS] > 1 && p.nph == 1)
    p.splits = std::min(g_tune[TUNE_CONV_FORCE_SPLITS] - 1, std::max(1, kmax));
  p.kper = cdiv(std::max(kmax, 1), p.splits);
  if (p.splits > 1) p.splits = cdiv(kmax, p.kper);
  return p;
}

static size_t gemm_workspace(const GemmPlan &p, int M) {
  return p.splits > 1 ? (size_t)p.splits * M * p.ncols * sizeof(float) : 0;
}

// ---- second-generation GEMM plan (k_conv_gemm2) ------------------------------------------
static int g_conv_precision = 0;  // GEMM operand precision: 0 fp32, 1 bf16, 2 fp16
static int g_wgrad_kb = 16;       // k_conv_wgrad pixels per K-step (e2ep_conv_wgrad_kstep)
static int g_gemm_variant = 0;  // 0 auto, 1 always k_conv_gemm, 2 k_conv_gemm2 wherever it
                                // applies, 3 the same with 128-column tiles only, 4 auto with
                                // the 1x1 forward / data gradient on the batched k_gemm, 5 the
                                // same for maps of <= 1024 pixels only

// live taps of the largest phase and the column count (as plan_gemm)
static void gemm_extent(int mode, const ConvGeom &g, int &taps_max, long long &ncols, int &nph) {
  nph = mode ? g.sh * g.sw : 1;
  if (mode == 0) {
    ncols = (long long)g.N * g.P * g.Q;
    taps_max = live_taps_axis(0, 0, g.ph, g.R, g.dh, g.sh, g.H, g.P, 0) *
               live_taps_axis(0, 0, g.pw, g.S, g.dw, g.sw, g.W, g.Q, 0);
    return;
  }
  ncols = 0;
  taps_max = 0;
  for (int z = 0; z < nph; ++z) {
    const int py = z / g.sw, px = z % g.sw;
    const long long Hp = py < g.H ? (g.H - py + g.sh - 1) / g.sh : 0;
    const long long Wp = px < g.W ? (g.W - px + g.sw - 1) / g.sw : 0;
    ncols = std::max(ncols, (long long)g.N * Hp * Wp);
    taps_max = std::max(taps_max, live_taps_axis(1, py, g.ph, g.R, g.dh, g.sh, g.H, g.P, (int)Hp) *
                                      live_taps_axis(1, px, g.pw, g.S, g.dw, g.sw, g.W, g.Q, (int)Wp));
  }
}

// k_conv_gemm2 applies when the tail table fits (remainder channels x taps <= V2_TAIL).
// Automatic choice (scripts/bench_conv_variants.py, MI355X): spatial filters (R*S > 1) with
// M >= 40 on large maps — 64 x 256 tiles when their grid fills whole rounds of 2 blocks per CU
// (>= 95 % of the last round used: the BEV stem 7x7/2 fwd 0.80 -> 0.52 ms), else 64 x 128 tiles
// when there are >= 1024 of them (the segmentation 3x3 at 200x200); everything else (1x1
// convs, small maps, split-K grids) stays on k_conv_gemm, which is faster there.
static bool plan_gemm2(int mode, const ConvGeom &g, int M, GemmPlan &p, int &wnt) {
  if (g_gemm_variant == 1) return false;
  int taps;
  long long ncols;
  int nph;
  gemm_extent(mode, g, taps, ncols, nph);
  const int Kc = mode == 0 ? g.Cin : g.Cout;
  if ((Kc % BK) * taps > V2_TAIL || taps == 0) return false;
  const long long mblocks = cdiv(M, 64);
  const long long b256 = cdiv(ncols, 256) * mblocks * nph, b128 = cdiv(ncols, 128) * mblocks * nph;
  const long long slots = 2LL * 256;  // 64 x 256 tiles resident per round (2 per CU)
  const bool fill256 = b256 >= slots && 100 * b256 >= 95 * (cdiv(b256, slots) * slots);
  if (g_gemm_variant == 0 || g_gemm_variant >= 4) {
    if (g.R * g.S == 1 || M < 40) return false;
    if (!fill256 && b128 < 1024) return false;
    wnt = fill256 ? 4 : 2;
  } else {
    wnt = (g_gemm_variant == 2 && b256 >= 512) ? 4 : 2;
  }
  p.bm = 64;
  p.bnt = 64 * wnt;
  p.nph = nph;
  p.ncols = ncols;
  p.splits = 1;
  const int ksteps = taps * (Kc / BK) + cdiv((Kc % BK) * taps, BK);
  p.kper = std::max(ksteps, 1);
  return true;
}

// Variant 4: 1x1 / stride-1 / unpadded convolutions forward and data gradient as a column-
// batched GEMM on k_gemm (gemm.hip): columns = (image, pixel), the weight as the A operand
// (k-contiguous in the forward, row-contiguous in the data gradient), bias per output channel
// (row), the skip gradient in dx's layout.  In isolation 15-35 % faster than k_conv_gemm on
// the EfficientNet 1x1 shapes (scripts/bench_gemm.py --conv), but 0.33 ms/step SLOWER inside
// the replayed train step (rocprofv3 kernel stats, profiles/r02/session4), so it is opt-in.
// fp32 only.
static bool conv1x1_gemm_ok(int mode, const ConvGeom &g) {
  (void)mode;
  return (g_gemm_variant == 4 || (g_gemm_variant == 5 && g.H * g.W <= 1024)) &&
         g_conv_precision == 0 && g.R == 1 && g.S == 1 && g.sh == 1 &&
         g.sw == 1 && g.ph == 0 && g.pw == 0 && (g.H * g.W) % 32 == 0 &&
         4LL * g.N * std::max(g.Cin, g.Cout) * g.H * g.W < 0x7fffffffLL;
}

static size_t conv1x1_ws(int mode, const ConvGeom &g, int M) {
  return gemm_ws(M, g.N * g.H * g.W, mode == 0 ? g.Cin : g.Cout);
}

static int conv1x1_gemm(int mode, int act, const float *w, const float *src, const float *bias,
                        float *dst, long long dst_bytes, const ConvGeom &g, int M, void *workspace,
                        hipStream_t s) {
  const int HW = g.H * g.W;
  const int N = g.N * HW;
  const long long w_bytes = 4LL * g.Cout * g.Cin;
  if (mode == 0) {  // y[n][co][p] = sum_ci w[co][ci] x[n][ci][p] (+ bias[co]) (relu)
    return gemm_run(w, g.Cin, true, w_bytes, src, HW, false, 4LL * g.N * g.Cin * HW, bias, true,
                    nullptr, 0, dst, dst_bytes, HW, GemmCols{HW, (long long)g.Cin * HW, (long long)M * HW},
                    M, N, g.Cin, act == 1, workspace, s);
  }
  // dx[n][ci][p] = sum_co w[co][ci] gout[n][co][p] (+ res[n][ci][p])
  return gemm_run(w, g.Cin, false, w_bytes, src, HW, false, 4LL * g.N * g.Cout * HW, nullptr,
                  false, bias, HW, dst, dst_bytes, HW,
                  GemmCols{HW, (long long)g.Cout * HW, (long long)M * HW}, M, N, g.Cout, 0,
                  workspace, s);
}

// weight-gradient kernel family: k_wgrad_lp for C3 (bf16 operands; fp16 inference keeps the fp32
// weight gradient) unless e2ep_tune key 12 = 1, and for fp32 when key 15 = 2
static bool lp_wgrad_selected() {
  if (g_conv_precision == 1) return g_tune[TUNE_LP_WGRAD] != 1;
  return g_tune[TUNE_LP32W] == 2;
}

// K order of the forward / data-gradient GEMMs (e2ep_tune key 18; 1 = automatic): channel
// chunk outer and taps inner for 16-bit operands (a block reads the same input rows for every
// tap of a chunk while they are cache resident: bf16 BEV stem forward 416 -> 287 us, data
// gradient 230 -> 160 us, profiles/r03/lp/korder_ab_bf16.txt), tap outer for fp32 (MFMA-bound
// there: the channel-outer order measured 1 % slower); 2 forces channel outer, 3 tap outer
static int korder_of() {
  const int t = g_tune[TUNE_KORDER];
  if (t == 2) return 1;
  if (t == 3) return 0;
  return g_conv_precision != 0 ? 1 : 0;
}

// The kernel family launch_gemm runs for a geometry (host only; g with korder / xcd set).
enum ConvRoute { ROUTE_LP = 1, ROUTE_1X1 = 2, ROUTE_G2 = 3, ROUTE_LP32 = 4, ROUTE_GEMM = 5 };
static int conv_route(int mode, const ConvGeom &g, int M) {
  if (g_conv_precision != 0 && lp_ok(mode, g, M, g_conv_precision)) return ROUTE_LP;
  if (conv1x1_gemm_ok(mode, g)) return ROUTE_1X1;
  GemmPlan p2;
  int wnt;
  if (g.wlayout == 1 && plan_gemm2(mode, g, M, p2, wnt)) return ROUTE_G2;
  if (g_conv_precision == 0 && g_tune[TUNE_LP32] == 2 && lp_ok(mode, g, M, 0)) return ROUTE_LP32;
  return ROUTE_GEMM;
}

// Column tiles of the forward's BatchNorm partial statistics (e2ep_conv_fwd_stats), or 0 when
// the routed kernel does not take them (then the BN layer computes its own).
static int fwd_stats_tiles(const ConvGeom &g0) {
  ConvGeom g = g0;
  g.korder = korder_of();
  g.xcd = g_tune[TUNE_XCD] == 2;
  if (direct_ok(g)) return 0;
  const int route = conv_route(0, g, g.Cout);
  if (stem_direct_ok(0, g, g.Cout, g_conv_precision)) return 0;  // the direct stem takes no stats
  if (route == ROUTE_LP) return lp_stats_tiles(g, g_conv_precision);
  if (route == ROUTE_LP32) return lp_stats_tiles(g, 0);
  if (route != ROUTE_GEMM || g_conv_precision != 0) return 0;  // fp32 k_conv_gemm only
  const GemmPlan p = plan_gemm(0, g, g.Cout);
  if (p.splits > 1 && g_tune[TUNE_SPLITK_FOLD] != 2) return 0;  // final values in k_conv_reduce
  return (int)cdiv(p.ncols, p.bnt);
}

// io (e2ep.h E2EP_IO_*): bf16 storage of the forward input (mode 0, E2EP_IO_X_BF16) or of the
// data gradient (mode 1, E2EP_IO_DX_BF16), on the bf16-operand kernels (C3) only
static int launch_gemm(int mode, int act, const float *w, const void *srcv, const float *bias,
                       void *dstv, long long dst_bytes, const ConvGeom &g0, int M, void *workspace,
                       hipStream_t s, double *stats = nullptr, int io = 0) {
  ConvGeom g = g0;
  g.korder = korder_of();
  g.xcd = g_tune[TUNE_XCD] == 2;
  const int route = conv_route(mode, g, M);
  if (stats && (mode != 0 || route == ROUTE_1X1 || route == ROUTE_G2)) {
    set_error("conv: BatchNorm statistics requested from a kernel that does not take them");
    return E2EP_EINVAL;
  }
  // the BEV stem's direct-convolution kernels (conv_stem.hip) whatever the route
  if (!stats && !io && mode == 0 && stem_direct_ok(0, g, M, g_conv_precision))
    return stem_direct_launch(act, g_conv_precision, w, static_cast<const float *>(srcv), bias,
                              static_cast<float *>(dstv), dst_bytes, g, workspace, s);
  if (!io && mode == 1 && !bias && stem_direct_ok(1, g, M, g_conv_precision))
    return stem_dgrad_launch(g_conv_precision, w, static_cast<const float *>(srcv),
                             static_cast<float *>(dstv), dst_bytes, g, workspace, s);
  if (route == ROUTE_LP)
    return lp_launch(mode, act, g_conv_precision, w, srcv, bias, dstv, dst_bytes, g, M, workspace, s,
                     stats, io);
  const bool sb = io && mode == 0 && io == E2EP_IO_X_BF16;
  const bool db = io && mode == 1 && io == E2EP_IO_DX_BF16;
  if (io && (route != ROUTE_GEMM || g_conv_precision != 1 || !(sb || db))) {
    set_error("conv: storage mask %d not supported on this route (bf16 operands: the forward input "
              "or the data-gradient output on k_conv_lp / k_conv_gemm)", io);
    return E2EP_EINVAL;
  }
  const float *src = static_cast<const float *>(srcv);
  float *dst = static_cast<float *>(dstv);
  if (route == ROUTE_1X1)
    return conv1x1_gemm(mode, act, w, src, bias, dst, dst_bytes, g, M, workspace, s);
  if (route == ROUTE_G2) {
    GemmPlan p2;
    int wnt;
    if (plan_gemm2(mode, g, M, p2, wnt)) {
      dim3 grid(cdiv(p2.ncols, p2.bnt), cdiv(M, 64), p2.nph);
#define G2(MD, AC, W)                                                                         \
  do {                                                                                        \
    if (g_conv_precision == 1)                                                                \
      hipLaunchKernelGGL((k_conv_gemm2<MD, AC, W, 1>), grid, dim3(256), 0, s, w, src, bias, dst, \
                         dst_bytes, g, M, 1, p2.kper);                                        \
    else if (g_conv_precision == 2)                                                           \
      hipLaunchKernelGGL((k_conv_gemm2<MD, AC, W, 2>), grid, dim3(256), 0, s, w, src, bias, dst, \
                         dst_bytes, g, M, 1, p2.kper);                                        \
    else                                                                                      \
      hipLaunchKernelGGL((k_conv_gemm2<MD, AC, W, 0>), grid, dim3(256), 0, s, w, src, bias, dst, \
                         dst_bytes, g, M, 1, p2.kper);                                        \
  } while (0)
      if (mode == 0 && act == 0) { if (wnt == 4) G2(0, 0, 4); else G2(0, 0, 2); }
      else if (mode == 0) { if (wnt == 4) G2(0, 1, 4); else G2(0, 1, 2); }
      else { if (wnt == 4) G2(1, 0, 4); else G2(1, 0, 2); }
#undef G2
      return 0;
    }
  }
  if (route == ROUTE_LP32)
    return lp_launch(mode, act, 0, w, src, bias, dst, dst_bytes, g, M, workspace, s, stats);
  const GemmPlan p = plan_gemm(mode, g, M);
  dim3 grid(cdiv(p.ncols, p.bnt), cdiv(M, p.bm), p.nph * p.splits);
  float *part = nullptr;
  unsigned int *cnt = nullptr;
  if (p.splits > 1) {
    if (!workspace) {
      set_error("conv: split-K plan needs a workspace (query the *_workspace entry point)");
      return E2EP_EINVAL;
    }
    part = static_cast<float *>(workspace);
    // in-launch fold (e2ep_tune key 28 = 2): one arrival counter per output tile
    if (g_tune[TUNE_SPLITK_FOLD] == 2) cnt = handoff_slots((int)grid.x * (int)grid.y, s);
  }
  if (stats && p.splits > 1 && !cnt) {
    set_error("conv: BatchNorm statistics need the in-launch split-K fold (e2ep_tune key 28 = 2)");
    return E2EP_EINVAL;
  }
  if (db && p.splits > 1 && !cnt) {
    set_error("conv: a bf16 data gradient needs the in-launch split-K fold (e2ep_tune key 28 = 2)");
    return E2EP_EINVAL;
  }
  const bool av = mode == 0 && g.wlayout == 1 && (g.Cin & 3) == 0;
#define GEMM_LAUNCH1(MD, AC, BT, BMT, V)                                                          \
  do {                                                                                             \
    if (g_conv_precision == 1 && MD == 0 && sb)                                                    \
      hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT, BMT, V, 1, false, bf16_t, float>), grid, dim3(256), 0, s, \
                         w, static_cast<const bf16_t *>(srcv), bias, dst, dst_bytes, g, M, p.splits, \
                         p.kper, part, cnt, nullptr);                                              \
    else if (g_conv_precision == 1 && MD == 1 && db)                                               \
      hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT, BMT, V, 1, false, float, bf16_t>), grid, dim3(256), 0, s, \
                         w, src, bias, static_cast<bf16_t *>(dstv), dst_bytes, g, M, p.splits,     \
                         p.kper, part, cnt, nullptr);                                              \
    else if (g_conv_precision == 1)                                                                \
      hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT, BMT, V, 1>), grid, dim3(256), 0, s, w, src, bias, \
                         dst, dst_bytes, g, M, p.splits, p.kper, part, cnt, nullptr);             \
    else if (g_conv_precision == 2)                                                                \
      hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT, BMT, V, 2>), grid, dim3(256), 0, s, w, src, bias, \
                         dst, dst_bytes, g, M, p.splits, p.kper, part, cnt, nullptr);             \
    else if (MD == 0 && stats)                                                                     \
      hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT, BMT, V, 0, true>), grid, dim3(256), 0, s, w, src, \
                         bias, dst, dst_bytes, g, M, p.splits, p.kper, part, cnt, stats);         \
    else                                                                                           \
      hipLaunchKernelGGL((k_conv_gemm<MD, AC, BT, BMT, V, 0>), grid, dim3(256), 0, s, w, src, bias, \
                         dst, dst_bytes, g, M, p.splits, p.kper, part, cnt, nullptr);             \
  } while (0)
#define GEMM_LAUNCH(MD, AC, BT, BMT)                                  \
  do {                                                                \
    if (MD == 0 && BMT == 64 && av) GEMM_LAUNCH1(MD, AC, BT, BMT, MD == 0 && BMT == 64); \
    else GEMM_LAUNCH1(MD, AC, BT, BMT, false);                        \
  } while (0)
#define GEMM_TILES(MD, AC)                                             \
  do {                                                                 \
    if (p.bm == 64) {                                                  \
      if (p.bnt == 128) GEMM_LAUNCH(MD, AC, 128, 64);                  \
      else GEMM_LAUNCH(MD, AC, 64, 64);                                \
    } else {                                                           \
      if (p.bnt == 256) GEMM_LAUNCH(MD, AC, 256, 32);                  \
      else GEMM_LAUNCH(MD, AC, 128, 32);                               \
    }                                                                  \
  } while (0)
  if (mode == 0 && act == 0) GEMM_TILES(0, 0);
  else if (mode == 0) GEMM_TILES(0, 1);
  else GEMM_TILES(1, 0);
#undef GEMM_TILES
#undef GEMM_LAUNCH
#undef GEMM_LAUNCH1
  if (p.splits > 1 && !cnt) {
    const int HW = mode == 0 ? g.P * g.Q : g.H * g.W;
    hipLaunchKernelGGL(k_conv_reduce, dim3(cdiv(p.ncols, 256), M), dim3(256), 0, s,
                       static_cast<const float *>(workspace), p.splits, M, HW, (int)p.ncols,
                       mode == 0 ? bias : nullptr, act, mode == 1 ? bias : nullptr, dst);
  }
  return 0;
}

extern "C" {

// (sized for the k_conv_gemm plan; the k_conv_gemm2 path needs none, so a caller may pass a
// workspace sized by these queries whichever kernel runs)
static size_t conv_fwd_workspace(const int *dims);
size_t e2ep_conv_fwd_workspace(const int *dims) {
  ConvGeom g = make_geom(dims);
  g.wlayout = 1;  // w_layout unknown here: cover the direct stem's weight image
  const size_t ws = conv_fwd_workspace(dims);
  return stem_direct_ok(0, g, g.Cout, g_conv_precision)
             ? std::max(ws, stem_direct_workspace(g, 0, g_conv_precision)) : ws;
}
static size_t conv_fwd_workspace(const int *dims) {
  ConvGeom g = make_geom(dims);
  if (direct_ok(g)) return 0;
  if (g_conv_precision != 0 || g_tune[TUNE_LP32] == 2) {  // w_layout unknown here: cover all
    g.wlayout = 1;
    if (lp_ok(0, g, g.Cout, g_conv_precision)) {
      size_t ws = std::max(lp_workspace(0, g, g.Cout, g_conv_precision),
                           gemm_workspace(plan_gemm(0, g, g.Cout), g.Cout));
      return ws;
    }
  }
  if (conv1x1_gemm_ok(0, g)) return conv1x1_ws(0, g, g.Cout);
  return gemm_workspace(plan_gemm(0, g, g.Cout), g.Cout);
}

static size_t conv_dgrad_workspace(const int *dims, int m_channels);
size_t e2ep_conv_dgrad_workspace(const int *dims, int m_channels) {
  ConvGeom g = make_geom(dims);
  g.wlayout = 1;
  const size_t ws = conv_dgrad_workspace(dims, m_channels);
  return stem_direct_ok(1, g, m_channels, g_conv_precision)
             ? std::max(ws, stem_direct_workspace(g, 1, g_conv_precision)) : ws;
}
static size_t conv_dgrad_workspace(const int *dims, int m_channels) {
  ConvGeom g = make_geom(dims);
  if (g_conv_precision != 0 || g_tune[TUNE_LP32] == 2) {
    g.wlayout = 1;
    if (lp_ok(1, g, m_channels, g_conv_precision)) {
      size_t ws = std::max(lp_workspace(1, g, m_channels, g_conv_precision),
                           gemm_workspace(plan_gemm(1, g, m_channels), m_channels));
      return ws;
    }
  }
  if (conv1x1_gemm_ok(1, g)) return conv1x1_ws(1, g, m_channels);
  return gemm_workspace(plan_gemm(1, g, m_channels), m_channels);
}

int e2ep_conv_precision(int precision) {
  const int old = g_conv_precision;
  if (precision >= 0 && precision <= 2) g_conv_precision = precision;
  return old;
}

int e2ep_conv_wgrad_kstep(int pixels) {
  const int old = g_wgrad_kb;
  if (pixels == 16 || pixels == 32) g_wgrad_kb = pixels;
  return old;
}

int e2ep_conv_split_params(int target, int thresh, int wgrad_target) {
  if (target > 0) g_split_target = target;
  if (thresh >= 0) g_split_thresh = thresh;
  if (wgrad_target > 0) g_wgrad_target = wgrad_target;
  return 0;
}

int e2ep_conv_gemm_variant(int variant) {
  const int old = g_gemm_variant;
  if (variant >= 0 && variant <= 5) g_gemm_variant = variant;
  return old;
}

int e2ep_conv_fwd_stats_tiles(const int *dims, int w_layout) {
  ConvGeom g = make_geom(dims);
  g.wlayout = w_layout;
  if (!geom_ok(g) || (w_layout != 0 && w_layout != 1)) return 0;
  return fwd_stats_tiles(g);
}

int e2ep_conv_fwd(const void *x, const float *w, const float *bias, const int *dims, int act,
                  int w_layout, float *y, void *workspace, size_t workspace_bytes, void *stream,
                  int io) {
  return e2ep_conv_fwd_stats(x, w, bias, dims, act, w_layout, y, workspace, workspace_bytes,
                             nullptr, 0, stream, io);
}

int e2ep_conv_fwd_stats(const void *x, const float *w, const float *bias, const int *dims, int act,
                        int w_layout, float *y, void *workspace, size_t workspace_bytes,
                        double *stats, size_t stats_bytes, void *stream, int io) {
  ConvGeom g = make_geom(dims);
  {
    const size_t need = e2ep_conv_fwd_workspace(dims);
    E2EP_REQUIRE(!need || (workspace && workspace_bytes >= need), E2EP_EINVAL,
                 "e2ep_conv_fwd: workspace %zu bytes < %zu the launch plan needs (query "
                 "e2ep_conv_fwd_workspace after setting precision / tunables)", workspace_bytes, need);
  }
  E2EP_REQUIRE(w_layout == 0 || w_layout == 1, E2EP_EINVAL, "e2ep_conv_fwd: w_layout must be 0 or 1");
  g.wlayout = w_layout;
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_fwd: bad geometry");
  E2EP_REQUIRE(act == 0 || act == 1, E2EP_EINVAL, "e2ep_conv_fwd: act must be 0 (none) or 1 (relu)");
  if (stats) {  // BatchNorm partials [Cout][tiles][2] from the epilogue (bnstats.h)
    const int tiles = fwd_stats_tiles(g);
    E2EP_REQUIRE(tiles > 0, E2EP_EINVAL,
                 "e2ep_conv_fwd_stats: this geometry's kernel takes no statistics "
                 "(e2ep_conv_fwd_stats_tiles returned 0)");
    E2EP_REQUIRE(stats_bytes >= (size_t)g.Cout * tiles * 2 * sizeof(double), E2EP_EINVAL,
                 "e2ep_conv_fwd_stats: stats %zu bytes < %zu (Cout x tiles x 2 doubles)",
                 stats_bytes, (size_t)g.Cout * tiles * 2 * sizeof(double));
  }
  E2EP_REQUIRE(io == 0 || io == E2EP_IO_X_BF16, E2EP_EINVAL,
               "e2ep_conv_fwd: storage mask %d not supported (0 or X bf16)", io);
  if (direct_ok(g)) {
    E2EP_REQUIRE(io == 0, E2EP_EINVAL, "e2ep_conv_fwd: the direct kernel reads fp32 x only");
    hipLaunchKernelGGL(k_conv_direct, dim3(cdiv((long long)g.N * g.P * g.Q, 256)), dim3(256), 0,
                       as_stream(stream), static_cast<const float *>(x), w, bias, g, act, y);
    return launch_status("e2ep_conv_fwd");
  }
  const int rc = launch_gemm(0, act, w, x, bias, y, 4LL * g.N * g.Cout * g.P * g.Q, g, g.Cout,
                             workspace, as_stream(stream), stats, io);
  if (rc) return rc;
  return launch_status("e2ep_conv_fwd");
}

int e2ep_conv_dgrad_acc(const float *gout, const float *w, const int *dims, int m_channels,
                        int w_layout, const float *res, void *dx, void *workspace,
                        size_t workspace_bytes, void *stream, int io) {
  ConvGeom g = make_geom(dims);
  if (m_channels > 0 && m_channels <= g.Cin) {
    const size_t need = e2ep_conv_dgrad_workspace(dims, m_channels);
    E2EP_REQUIRE(!need || (workspace && workspace_bytes >= need), E2EP_EINVAL,
                 "e2ep_conv_dgrad: workspace %zu bytes < %zu the launch plan needs (query "
                 "e2ep_conv_dgrad_workspace after setting precision / tunables)", workspace_bytes, need);
  }
  E2EP_REQUIRE(w_layout == 0 || w_layout == 1, E2EP_EINVAL, "e2ep_conv_dgrad: w_layout must be 0 or 1");
  g.wlayout = w_layout;
  E2EP_REQUIRE(geom_ok(g), E2EP_EINVAL, "e2ep_conv_dgrad: bad geometry");
  E2EP_REQUIRE(m_channels > 0 && m_channels <= g.Cin, E2EP_EINVAL,
               "e2ep_conv_dgrad: m_channels must be in [1, Cin]");
  E2EP_REQUIRE(io == 0 || io == E2EP_IO_DX_BF16, E2EP_EINVAL,
               "e2ep_conv_dgrad: storage mask %d not supported (0 or DX bf16)", io);
  const long long esz = io ? 2 : 4;
  const int rc = launch_gemm(1, 0, w, gout, res, dx, esz * g.N * m_channels * g.H * g.W, g,
                             m_channels, workspace, as_stream(stream), nullptr, io);
  if (rc) return rc;
  return launch_status("e2ep_conv_dgrad");
}

int e2ep_conv_dgrad(const float *gout, const float *w, const int *dims, int m_channels,
                    int w_layout, float *dx, void *workspace, size_t workspace_bytes, void *stream) {
  return e2ep_conv_dgrad_acc(gout, w, dims, m_channels, w_layout, nullptr, dx, workspace,
                             workspace_bytes, stream, 0);
}

int e2ep_conv_wgrad_splits(const int *dims) {
  ConvGeom g = make_geom(dims);
  if (stem_direct_ok(2, g, g.Cout, g_conv_precision == 1 ? 1 : 0)) return stem_wgrad_splits(g);
  if (lp_wgrad_selected()) {  // k_wgrad_lp (conv_lp.hip): C3 bf16, or fp32 when selected
    const TapList tl = live_taps(g);
    if (lp_wgrad_ok(g, tl)) return lp_wgrad_splits(g, tl, g_conv_precision == 1 ? 1 : 0);
  }
  if (wgrad1x1_ok(g)) return wgrad1x1_splits(g);
  const int nl = std::max(1, live_taps(g).n);
  const long long base = (long long)cdiv(g.Cin * nl, WBN) * cdiv(g.Cout, BM);
  const long long pix = (long long)g.N * g.P * g.Q;
  long long want = (g_wgrad_target + base - 1) / base;
  long long cap = pix / 256;
  long long s = want < cap ? want : cap;
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  return (int)s;
}

size_t e2ep_conv_wgrad_workspace(const int *dims, int splits) {
  ConvGeom g = make_geom(dims);
  return (size_t)splits * g.Cout * g.Cin * g.R * g.S * sizeof(float);
}

int e2ep_conv_wgrad(const float *gout, const void *xv, const int *dims, int splits,
                    void *workspace, size_t workspace_bytes, float *dw, int accumulate,
                    void *stream, int io) {
  const float *x = static_cast<const float *>(xv);
  ConvGeom g = make_geom(dims);
  E2EP_REQUIRE(geom_ok(g) && splits > 0, E2EP_EINVAL, "e2ep_conv_wgrad: bad geometry");
  // the kernels write at most `splits` slabs of Cout * Cin * R * S floats
  E2EP_REQUIRE(workspace && workspace_bytes >= e2ep_conv_wgrad_workspace(dims, splits),
               E2EP_EINVAL, "e2ep_conv_wgrad: workspace %zu bytes < %zu for %d splits",
               workspace_bytes, e2ep_conv_wgrad_workspace(dims, splits), splits);
  E2EP_REQUIRE(io == 0 || io == E2EP_IO_X_BF16, E2EP_EINVAL,
               "e2ep_conv_wgrad: storage mask %d not supported (0 or X bf16)", io);
  // the weight gradient's operands: bf16 in C3, fp32 otherwise (C5's fp16 mode included)
  if (io == 0 && stem_direct_ok(2, g, g.Cout, g_conv_precision == 1 ? 1 : 0)) {
    hipStream_t s = as_stream(stream);
    float *part = static_cast<float *>(workspace);
    const int used = stem_wgrad_launch(gout, x, g, splits, part, s, g_conv_precision == 1 ? 1 : 0);
    E2EP_REQUIRE(used > 0, E2EP_EINVAL, "e2ep_conv_wgrad: direct stem weight gradient refused");
    reduce_splits(part, used, g.Cout * g.Cin * g.R * g.S, dw, accumulate, g.R * g.S, live_taps(g).mask, s);
    return launch_status("e2ep_conv_wgrad");
  }
  if (lp_wgrad_selected()) {
    const TapList tl = live_taps(g);
    if (lp_wgrad_ok(g, tl)) {
      E2EP_REQUIRE(io == 0 || g_conv_precision == 1, E2EP_EINVAL,
                   "e2ep_conv_wgrad: a bf16 x needs the bf16-operand weight gradient");
      hipStream_t s = as_stream(stream);
      float *part = static_cast<float *>(workspace);
      const int used = lp_wgrad_launch(gout, xv, g, tl, splits, part, s, g_conv_precision == 1 ? 1 : 0,
                                       io != 0);
      reduce_splits(part, used, g.Cout * g.Cin * g.R * g.S, dw, accumulate, g.R * g.S, tl.mask, s);
      return launch_status("e2ep_conv_wgrad");
    }
  }
  E2EP_REQUIRE(io == 0, E2EP_EINVAL,
               "e2ep_conv_wgrad: a bf16 x runs on the bf16-operand weight gradient (k_wgrad_lp) only");
  if (wgrad1x1_ok(g)) {
    const int groups = g.N * g.P * g.Q / 8;
    const int gps = cdiv(groups, splits);
    const int used = cdiv(groups, gps);
    hipStream_t s = as_stream(stream);
    float *part = static_cast<float *>(workspace);
    int to, tc;
    wgrad1x1_tiles(g, to, tc);
    const dim3 grid(cdiv(g.Cout, to) * cdiv(g.Cin, tc), used);
#define W1_LAUNCH(TI, TJ)                                                                      \
  do {                                                                                         \
    if (g_conv_precision == 1)                                                                 \
      hipLaunchKernelGGL((k_wgrad_1x1<TI, TJ, 1>), grid, dim3(256), 0, s, gout, x, part, g, used, \
                         gps);                                                                 \
    else                                                                                       \
      hipLaunchKernelGGL((k_wgrad_1x1<TI, TJ, 0>), grid, dim3(256), 0, s, gout, x, part, g, used, \
                         gps);                                                                 \
  } while (0)
    if (to == 64 && tc == 64) W1_LAUNCH(2, 2);
    else if (to == 64) W1_LAUNCH(2, 1);
    else if (tc == 64) W1_LAUNCH(1, 2);
    else W1_LAUNCH(1, 1);
#undef W1_LAUNCH
    const int n = g.Cout * g.Cin;
    reduce_splits(part, used, n, dw, accumulate, 1, 1ULL, s);
    return launch_status("e2ep_conv_wgrad");
  }
  const int Ptot = g.N * g.P * g.Q;
  // second generation when the K-step never straddles images (e2ep_tune key 9: 1 = always
  // the first generation, for A/B timing)
  const bool v2 = (g.P * g.Q) % W2K == 0 && g_tune[TUNE_WGRAD_GEN] != 1;
  const int kb = v2 ? W2K : g_wgrad_kb;
  int per = (Ptot + splits - 1) / splits;
  per = (per + kb - 1) / kb * kb;
  const int used = (Ptot + per - 1) / per;
  const TapList tl = live_taps(g);
  hipStream_t s = as_stream(stream);
  float *part = static_cast<float *>(workspace);
  if (tl.n > 0 && v2) {
    dim3 grid(cdiv(g.Cin * tl.n, 64), cdiv(g.Cout, 64), used);
    if (g_conv_precision == 1)
      hipLaunchKernelGGL((k_conv_wgrad2<1>), grid, dim3(256), 0, s, gout, x, part, g, per, tl);
    else
      hipLaunchKernelGGL((k_conv_wgrad2<0>), grid, dim3(256), 0, s, gout, x, part, g, per, tl);
  } else if (tl.n > 0) {
    dim3 grid(cdiv(g.Cin * tl.n, WBN), cdiv(g.Cout, BM), used);
#define WG_LAUNCH(OPV, KBV) \
  hipLaunchKernelGGL((k_conv_wgrad<OPV, KBV>), grid, dim3(256), 0, s, gout, x, part, g, per, tl)
    // bf16 operands in C3 (fp32 accumulate / gradient); pixel K-step 16 or 32
    if (g_conv_precision == 1) {
      if (kb == 32) WG_LAUNCH(1, 32); else WG_LAUNCH(1, 16);
    } else {
      if (kb == 32) WG_LAUNCH(0, 32); else WG_LAUNCH(0, 16);
    }
#undef WG_LAUNCH
  }
  const int n = g.Cout * g.Cin * g.R * g.S;
  reduce_splits(part, used, n, dw, accumulate, g.R * g.S, tl.mask, s);
  return launch_status("e2ep_conv_wgrad");
}

// The paired backward of e2ep_conv_bwd, where the two-launch path's kernels have a paired
// instantiation: PAIR_GEMM = fp32 k_conv_gemm data gradient (one split or folded splits) with
// k_conv_wgrad2 (k_conv_bwd_pair); PAIR_LP = k_conv_lp data gradient (fp32 where TUNE_LP32
// routes it, bf16 in C3) with the k_wgrad_lp / k_conv_wgrad2 weight gradient (k_lp_bwd_pair).
enum PairKind { PAIR_NONE = 0, PAIR_GEMM = 1, PAIR_LP = 2, PAIR_GEMM1X1 = 3 };
static int conv_bwd_pair_plan(ConvGeom &g, int m_channels, GemmPlan &p, TapList &tl) {
  g.wlayout = 1;
  g.korder = korder_of();
  g.xcd = g_tune[TUNE_XCD] == 2;
  if (!geom_ok(g) || m_channels <= 0 || m_channels > g.Cin) return PAIR_NONE;
  tl = live_taps(g);
  if (tl.n <= 0) return PAIR_NONE;
  // the BEV stem on the direct-convolution kernels (conv_stem.hip) runs its two gradients as
  // separate launches (both faster than the paired implicit GEMMs)
  if (stem_direct_ok(1, g, m_channels, g_conv_precision) || stem_direct_ok(2, g, g.Cout, g_conv_precision))
    return PAIR_NONE;
  // the weight-gradient kernel e2ep_conv_wgrad would run
  const bool wg_lp = lp_wgrad_selected() && lp_wgrad_ok(g, tl);
  const bool wg_2 = !wg_lp && !wgrad1x1_ok(g) && (g.P * g.Q) % W2K == 0 &&
                    g_tune[TUNE_WGRAD_GEN] != 1;
  const int route = conv_route(1, g, m_channels);
  const bool wg_1x1 = !wg_lp && wgrad1x1_ok(g);
  if (g_conv_precision == 0 && route == ROUTE_GEMM && (wg_2 || wg_1x1)) {
    p = plan_gemm(1, g, m_channels);
    if (p.splits > 1 && g_tune[TUNE_SPLITK_FOLD] != 2) return PAIR_NONE;
    const bool tile_ok = (p.bm == 64 && (p.bnt == 64 || p.bnt == 128)) ||
                         (p.bm == 32 && (p.bnt == 128 || p.bnt == 256));
    return tile_ok ? (wg_1x1 ? PAIR_GEMM1X1 : PAIR_GEMM) : PAIR_NONE;
  }
  if (g_conv_precision == 0 && route == ROUTE_LP32 && wg_2)
    return lp_bwd_pair_ok(g, m_channels, 0, tl) ? PAIR_LP : PAIR_NONE;
  if (g_conv_precision == 1 && route == ROUTE_LP && wg_lp)
    return lp_bwd_pair_ok(g, m_channels, 1, tl) ? PAIR_LP : PAIR_NONE;
  return PAIR_NONE;
}

int e2ep_conv_bwd_pair_ok(const int *dims, int m_channels) {
  ConvGeom g = make_geom(dims);
  GemmPlan p;
  TapList tl;
  return conv_bwd_pair_plan(g, m_channels, p, tl) != PAIR_NONE ? 1 : 0;
}

int e2ep_conv_bwd(const float *gout, const void *xv, const float *w, const int *dims,
                  int m_channels, const float *res, void *dxv, void *ws_dgrad,
                  size_t ws_dgrad_bytes, int wsplits, void *ws_wgrad, size_t ws_wgrad_bytes,
                  float *dw, void *stream, int io) {
  const float *x = static_cast<const float *>(xv);
  float *dx = static_cast<float *>(dxv);
  ConvGeom g = make_geom(dims);
  GemmPlan p;
  TapList tl;
  const int kind = conv_bwd_pair_plan(g, m_channels, p, tl);
  E2EP_REQUIRE(kind != PAIR_NONE, E2EP_EINVAL,
               "e2ep_conv_bwd: this geometry / setting has no paired backward "
               "(e2ep_conv_bwd_pair_ok returned 0)");
  E2EP_REQUIRE(gout && x && w && dx && dw && wsplits > 0, E2EP_EINVAL, "e2ep_conv_bwd: bad arguments");
  const size_t need_d = e2ep_conv_dgrad_workspace(dims, m_channels);
  E2EP_REQUIRE(!need_d || (ws_dgrad && ws_dgrad_bytes >= need_d), E2EP_EINVAL,
               "e2ep_conv_bwd: data-gradient workspace %zu bytes < %zu", ws_dgrad_bytes, need_d);
  E2EP_REQUIRE(ws_wgrad && ws_wgrad_bytes >= e2ep_conv_wgrad_workspace(dims, wsplits), E2EP_EINVAL,
               "e2ep_conv_bwd: weight-gradient workspace %zu bytes < %zu for %d splits",
               ws_wgrad_bytes, e2ep_conv_wgrad_workspace(dims, wsplits), wsplits);
  // bf16 storage (io = X|DX): x and dx bf16 on the bf16-operand pair (k_lp_bwd_pair) only
  const bool xb = io == (E2EP_IO_X_BF16 | E2EP_IO_DX_BF16);
  E2EP_REQUIRE(io == 0 || (xb && kind == PAIR_LP && g_conv_precision == 1 && !res), E2EP_EINVAL,
               "e2ep_conv_bwd: storage mask %d not supported (0, or X|DX bf16 on the bf16 k_lp_bwd_pair "
               "without a residual gradient)", io);
  hipStream_t s = as_stream(stream);
  const int M = m_channels;
  const long long dx_bytes = (xb ? 2LL : 4LL) * g.N * M * g.H * g.W;
  float *part2 = static_cast<float *>(ws_wgrad);
  int used;
  if (kind == PAIR_LP) {
    used = lp_bwd_pair_launch(w, gout, res, dxv, dx_bytes, g, M, g_conv_precision == 1 ? 1 : 0,
                              ws_dgrad, xv, tl, wsplits, part2, s, xb);
    E2EP_REQUIRE(used > 0, E2EP_EINVAL, "e2ep_conv_bwd: no paired k_conv_lp plan");
    reduce_splits(part2, used, g.Cout * g.Cin * g.R * g.S, dw, 0, g.R * g.S, tl.mask, s);
    return launch_status("e2ep_conv_bwd");
  }
  // k_conv_gemm data gradient: launch_gemm's grid and fold counters
  const dim3 g1(cdiv(p.ncols, p.bnt), cdiv(M, p.bm), p.nph * p.splits);
  float *part1 = p.splits > 1 ? static_cast<float *>(ws_dgrad) : nullptr;
  unsigned int *cnt = p.splits > 1 ? handoff_slots((int)g1.x * (int)g1.y, s) : nullptr;
  if (kind == PAIR_GEMM1X1) {
    // e2ep_conv_wgrad's k_wgrad_1x1 plan
    const int groups = g.N * g.P * g.Q / 8;
    const int gps = cdiv(groups, wsplits);
    used = cdiv(groups, gps);
    int to, tc;
    wgrad1x1_tiles(g, to, tc);
    const int nt2 = cdiv(g.Cout, to) * cdiv(g.Cin, tc);
    const dim3 grid(g1.x * g1.y * g1.z + nt2 * used);
    const int wfirst = g_tune[TUNE_PAIR1X1_ORDER] == 2 ? 1 : 0;
#define E2EP_PAIR1(BNTV, BMTV, TIV, TJV)                                                          \
  hipLaunchKernelGGL((k_conv_bwd_pair1x1<BNTV, BMTV, TIV, TJV>), grid, dim3(256), 0, s, w, gout,  \
                     res, dx, dx_bytes, g, M, p.splits, p.kper, part1, cnt, (int)g1.x, (int)g1.y,  \
                     (int)g1.z, x, part2, used, gps, nt2, wfirst)
#define E2EP_PAIR1_W(BNTV, BMTV)                                          \
  do {                                                                    \
    if (to == 64 && tc == 64) E2EP_PAIR1(BNTV, BMTV, 2, 2);               \
    else if (to == 64) E2EP_PAIR1(BNTV, BMTV, 2, 1);                      \
    else if (tc == 64) E2EP_PAIR1(BNTV, BMTV, 1, 2);                      \
    else E2EP_PAIR1(BNTV, BMTV, 1, 1);                                    \
  } while (0)
    if (p.bm == 64) {
      if (p.bnt == 128) E2EP_PAIR1_W(128, 64);
      else E2EP_PAIR1_W(64, 64);
    } else {
      if (p.bnt == 256) E2EP_PAIR1_W(256, 32);
      else E2EP_PAIR1_W(128, 32);
    }
#undef E2EP_PAIR1_W
#undef E2EP_PAIR1
    if (p.splits > 1 && !cnt)  // no fold counters: the data gradient's slabs reduced here
      hipLaunchKernelGGL(k_conv_reduce, dim3(cdiv(p.ncols, 256), M), dim3(256), 0, s, part1,
                         p.splits, M, g.H * g.W, (int)p.ncols, nullptr, 0, res, dx);
    reduce_splits(part2, used, g.Cout * g.Cin, dw, 0, 1, 1ULL, s);
    return launch_status("e2ep_conv_bwd");
  } else {
    // weight gradient grid (e2ep_conv_wgrad's k_conv_wgrad2 path)
    const int Ptot = g.N * g.P * g.Q;
    int per = (Ptot + wsplits - 1) / wsplits;
    per = (per + W2K - 1) / W2K * W2K;
    used = (Ptot + per - 1) / per;
    const dim3 g2(cdiv(g.Cin * tl.n, 64), cdiv(g.Cout, 64), used);
    const dim3 grid(g1.x * g1.y * g1.z + g2.x * g2.y * g2.z);
#define E2EP_PAIR(BNTV, BMTV)                                                                     \
  hipLaunchKernelGGL((k_conv_bwd_pair<BNTV, BMTV>), grid, dim3(256), 0, s, w, gout, res, dx,      \
                     dx_bytes, g, M, p.splits, p.kper, part1, cnt, (int)g1.x, (int)g1.y,           \
                     (int)g1.z, x, part2, per, tl, (int)g2.x, (int)g2.y, (int)g2.z)
    if (p.bm == 64) {
      if (p.bnt == 128) E2EP_PAIR(128, 64);
      else E2EP_PAIR(64, 64);
    } else {
      if (p.bnt == 256) E2EP_PAIR(256, 32);
      else E2EP_PAIR(128, 32);
    }
#undef E2EP_PAIR
  }
  if (p.splits > 1 && !cnt)  // no fold counters: the data gradient's slabs reduced here
    hipLaunchKernelGGL(k_conv_reduce, dim3(cdiv(p.ncols, 256), M), dim3(256), 0, s, part1,
                       p.splits, M, g.H * g.W, (int)p.ncols, nullptr, 0, res, dx);
  reduce_splits(part2, used, g.Cout * g.Cin * g.R * g.S, dw, 0, g.R * g.S, tl.mask, s);
  return launch_status("e2ep_conv_bwd");
}

size_t e2ep_col_sum_workspace(int rows, int C) {
  return (size_t)cdiv(rows, COLSUM_ROWS) * C * sizeof(float);
}

int e2ep_col_sum(const float *g, int rows, int C, float *out, void *workspace, void *stream) {
  E2EP_REQUIRE(rows > 0 && C > 0 && workspace, E2EP_EINVAL, "e2ep_col_sum: bad args");
  const int chunks = cdiv(rows, COLSUM_ROWS);
  // one chunk (e.g. the control decoder's 112 token rows): the partial sums are the result
  float *part = chunks == 1 ? out : static_cast<float *>(workspace);
  hipLaunchKernelGGL(k_col_sum_partial, dim3(cdiv(C, 64), chunks), dim3(256), 0,
                     as_stream(stream), g, rows, C, part);
  if (chunks > 1)
    hipLaunchKernelGGL(k_col_sum_final, dim3(cdiv(C, 256)), dim3(256), 0, as_stream(stream), part,
                       chunks, C, out);
  return launch_status("e2ep_col_sum");
}

int e2ep_bias_grad(const float *gout, int N, int C, int HW, float *db, void *stream) {
  E2EP_REQUIRE(N > 0 && C > 0 && HW > 0, E2EP_EINVAL, "e2ep_bias_grad: bad shape");
  hipLaunchKernelGGL(k_bias_grad, dim3(C), dim3(1024), 0, as_stream(stream), gout, N, C, HW, db);
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
