// Low-precision implicit-GEMM convolution (forward / data gradient) for gfx950: the BASELINE
// C3 bf16 training mode and the C5 fp16 inference mode (operands rounded to nearest-even as
// they are staged, fp32 accumulate, fp32 tensors in HBM).
//
// k_conv_gemm / k_conv_gemm2 (conv.hip) were shaped for the exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32, 64 cycles per 4096 FLOP): a 16-deep K-step feeds eight of them per
// accumulator.  Run with bf16 operands the same step is ONE v_mfma_f32_32x32x16_bf16 (32
// cycles for 32768 FLOP), so those kernels spend their time on per-step load issue, the fp32
// LDS round trip, per-fragment conversions and barriers (C3 conv family at 0.027 of the bf16
// peak, profiles/r02/bench_c3_bf16.json).  This kernel is built for the 16-bit MFMA instead:
//  * operands are converted ONCE, when written to LDS (packed 8 x 16-bit per ds_write_b128),
//    and the LDS images hold 16-bit values: half the LDS bytes, no conversion per fragment;
//  * a K-step is 32 deep (two 16-deep MFMAs per accumulator per barrier) and the block tile is
//    up to 128 x 256 (wave tiles up to 64 x 128: each A fragment feeds WN MFMAs, each B
//    fragment WM), so L2 -> LDS operand bytes per FLOP drop 2 - 4x against 64 x 64 tiles;
//  * LDS rows are k-contiguous, 32 values + 8 pad (80 B): the b128 fragment reads (a lane's 8
//    consecutive k of one row) and the b128 stores are bank-conflict free;
//  * K order as k_conv_gemm2: (live tap, 32-channel chunk) steps, then the remainder channels
//    flattened over the taps 32 (channel, tap) pairs per step (no zero-padded channel steps:
//    the BEV stem's 65 channels take 2 chunk steps per tap + 2 tail steps, not 3 per tap);
//  * the data gradient is split by input-pixel phase, as in conv.hip;
//  * one register set of lookahead: the next step's global loads are issued at the top of the
//    step, its LDS store follows all of the step's MFMAs (sched_barrier fences, as conv.hip).
// Small grids split K into fixed-order partial slabs (k_conv_lp_reduce): deterministic.
#include <algorithm>

#include "conv.h"
#include "bnstats.h"
#include "handoff.h"

// Contraction only within one expression (a*b + c -> fma): the fp32 and bf16-storage
// instantiations of a kernel (E2EP_IO_*) then fuse the same operations and round alike —
// under the default cross-statement contraction hipcc may pick a different multiply to fuse
// in each instantiation (tests/test_bf16_store_gpu.py holds them bitwise equal).
#pragma clang fp contract(on)

namespace e2ep {

constexpr int MAXPH_LP = 4;  // stride phases of the data gradient (sh * sw <= 4, conv.hip)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int LK = 32;   // default K per step (k_conv_lp: channels of one tap; k_wgrad_lp: pixels)
// LDS row stride in elements: 16-bit rows of lk k + 8 pad (32 k: 80 B, 64 k: 144 B), fp32
// rows of 32 k + 4 pad (144 B); 20- and 36-dword strides keep the b128 reads and writes
// bank-conflict free
constexpr int lld_of(int op, int lk) { return op == 0 ? lk + 4 : lk + 8; }
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OP> struct LpType;
template <> struct LpType<0> { typedef float T; typedef f32x4 T8; };
template <> struct LpType<1> { typedef __bf16 T; typedef bf16x8 T8; };
template <> struct LpType<2> { typedef _Float16 T; typedef f16x8 T8; };

template <int OP>
__device__ __forceinline__ typename LpType<OP>::T8 cvt8(const float *v) {
  static_assert(OP != 0, "fp32 rows are stored as float4");
  f32x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = v[j];
  return __builtin_convertvector(f, typename LpType<OP>::T8);
}

template <int OP>
__device__ __forceinline__ f32x16 mfma16(typename LpType<OP>::T8 a, typename LpType<OP>::T8 b,
                                         f32x16 c) {
  if constexpr (OP == 1) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// MODE 0 (forward): rows m = co, K = (tap, ci), src = x [N,Cin,H,W], dst = y [N,Cout,P,Q].
// MODE 1 (data gradient): rows m = ci, K = (tap, co), src = g [N,Cout,P,Q], dst = dx
//   [N,M,H,W]; phase z = (py, px) (blockIdx.z / splits) as in k_conv_gemm.
// Block tile (64 WM) x (64 WN), 2 x 2 waves of (32 WM) x (32 WN).
// The block body for block (bx, by, bz) of a grid gx blocks wide, its operand tiles in the
// caller's LDS (As[2][BMT][LD], Bs[2][BNT][LD]): k_conv_lp, and the data-gradient half of
// k_lp_bwd_pair.
// TS / TD: element types of src and dst (bf16_t: C3's bf16-stored squeeze-excitation output
// as the project conv's input, and its gradient as the project conv's data gradient; e2ep.h
// E2EP_IO_*); the MODE 1 residual gradient (`bias`) stays fp32.
template <int MODE, int ACT, int WM, int WN, int OP, int LKS, bool ST = false,
          typename TS = float, typename TD = float>
__device__ __forceinline__ void conv_lp_block(
    const float *__restrict__ w, const TS *__restrict__ src, const float *__restrict__ bias,
    TD *__restrict__ dst, long long dst_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part, unsigned int *__restrict__ cnt, double *__restrict__ stats, int bx,
    int by, int bz, int gx, typename LpType<OP>::T (*As)[64 * WM][lld_of(OP, LKS)],
    typename LpType<OP>::T (*Bs)[64 * WN][lld_of(OP, LKS)]) {
  typedef typename LpType<OP>::T8 T8;
  constexpr int BMT = 64 * WM, BNT = 64 * WN;
  constexpr int KGB = 256 / BNT;  // B k-groups (4, 2, 1)
  constexpr int RPB = LKS / KGB;   // B k rows per thread (8, 16, 32)
  constexpr int KGA = 256 / BMT;  // A k-groups (4, 2)
  constexpr int RPA = LKS / KGA;   // A k per thread (8, 16)
  static_assert(OP != 0 || (WN <= 2 && LKS == 32), "fp32: 32-deep steps, tiles up to 128 x 128");
  static_assert(LKS == 32 || LKS == 64, "K step 32 or 64");
  __shared__ int s_tdy[MAXTAPS], s_tdx[MAXTAPS], s_trs[MAXTAPS];
  __shared__ int s_ntaps;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = by * BMT, n0 = bx * BNT;
  const int split = bz % splits, z = bz / splits;

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

  // live tap table of this phase (the same rules as k_conv_gemm)
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
  const int cfull = Kc / LKS, crem = Kc - cfull * LKS;
  const int ntail = crem * ntaps;             // flattened (remainder channel, tap) rows
  const int kmain = ntaps * cfull;
  const int ksteps_all = kmain + (ntail + LKS - 1) / LKS;
  const int kbeg = split * kper;
  const int kend = min(ksteps_all, kbeg + kper);
  const int nk = max(0, kend - kbeg);

  const int Hs = MODE == 0 ? g.H : g.P, Ws = MODE == 0 ? g.W : g.Q;  // src spatial
  const int HWs = Hs * Ws;
  const int RS = g.R * g.S;
  const __amdgpu_buffer_rsrc_t rw = rsrc(w, 4LL * g.Cout * g.Cin * RS);
  constexpr int ES = sizeof(TS);  // bytes per src element
  const __amdgpu_buffer_rsrc_t rx = rsrc(src, (long long)ES * g.N * Kc * HWs);
  const int nrw = (int)min(4LL * g.Cout * g.Cin * RS, 0x7fffffffLL);
  const int nrx = (int)min((long long)ES * g.N * Kc * HWs, 0x7fffffffLL);
  const int tapstride = g.Cout * g.Cin;  // tap-major weights [RS][Cout][Cin]

  // B: this thread's column (fixed) and k group (rows kg*RPB .. +RPB-1 of each step)
  const int bn = tid % BNT, kg = tid / BNT;
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
  // A: MODE 0 thread = (row tid/KGA, k group tid%KGA): RPA channels contiguous in memory
  // (float4 loads when Cin % 4 == 0); MODE 1 thread = (row tid%BMT, k group tid/BMT): rows
  // contiguous in memory (lanes coalesce along ci), one load per k
  const int am = MODE == 0 ? tid / KGA : tid % BMT;
  const int akg = MODE == 0 ? tid % KGA : tid / BMT;
  const bool arow_ok = m0 + am < M;
  const bool avec = MODE == 0 && (g.Cin & 3) == 0;

  float ra[RPA], rb[RPB];
  const int klast = kend - 1;
  auto load_tiles = [&](int ks_in) {
    const bool live = ks_in <= klast;
    const int ks = min(ks_in, klast);
    if (ks < kmain) {  // one tap, 32 channels
      const int tap = g.korder ? ks % ntaps : ks / cfull;
      const int c0 = (g.korder ? ks / ntaps : ks - tap * cfull) * LKS;
      const int dy = s_tdy[tap], dx = s_tdx[tap], rs = s_trs[tap] * tapstride;
      if (MODE == 0) {
        const int base = (live && arow_ok) ? (rs + (m0 + am) * g.Cin + c0 + akg * RPA) * 4 : nrw;
        if (avec) {
#pragma unroll
          for (int q = 0; q < RPA / 4; ++q) {
            const float4 v = bload4(rw, base + 16 * q);
            ra[4 * q] = v.x; ra[4 * q + 1] = v.y; ra[4 * q + 2] = v.z; ra[4 * q + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int j = 0; j < RPA; ++j) ra[j] = bload(rw, base + 4 * j);
        }
      } else {
        // A[m = ci][k = co] = w[rs][co][ci]
        const int base = (live && arow_ok) ? (rs + (c0 + akg * RPA) * g.Cin + m0 + am) * 4 : nrw;
#pragma unroll
        for (int j = 0; j < RPA; ++j) ra[j] = bload(rw, base + j * g.Cin * 4);
      }
      const int iy = ybase + dy, ix = xbase + dx;
      const bool pix_ok = live && col_ok && (unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws;
      const int bbase = pix_ok ? (simg + (c0 + kg * RPB) * HWs + iy * Ws + ix) * ES : nrx;
#pragma unroll
      for (int r = 0; r < RPB; ++r) rb[r] = bload_t(rx, bbase + r * HWs * ES, src);
    } else {  // tail step: 32 flattened (remainder channel, tap) rows
      // a thread's rows are consecutive flattened indices: decode the first (one division),
      // then step the (channel, tap) pair
      const int t0 = (ks - kmain) * LKS;
      {
        const int i0 = t0 + akg * RPA;
        int cq = i0 / ntaps, t = i0 - cq * ntaps;
#pragma unroll
        for (int j = 0; j < RPA; ++j) {
          const bool ok = live && arow_ok && i0 + j < ntail;
          const int c = cfull * LKS + cq, rs = s_trs[ok ? t : 0] * tapstride;
          ra[j] = bload(rw, ok ? (MODE == 0 ? rs + (m0 + am) * g.Cin + c : rs + c * g.Cin + m0 + am) * 4 : OOR);
          const bool wrap = ++t == ntaps;
          t = wrap ? 0 : t;
          cq += wrap ? 1 : 0;
        }
      }
      {
        const int i0 = t0 + kg * RPB;
        int cq = i0 / ntaps, t = i0 - cq * ntaps;
#pragma unroll
        for (int r = 0; r < RPB; ++r) {
          const bool in = i0 + r < ntail;
          const int tt = in ? t : 0;
          const int iy = ybase + s_tdy[tt], ix = xbase + s_tdx[tt];
          const bool ok = live && col_ok && in && (unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws;
          rb[r] = bload_t(rx, ok ? (simg + (cfull * LKS + cq) * HWs + iy * Ws + ix) * ES : OOR, src);
          const bool wrap = ++t == ntaps;
          t = wrap ? 0 : t;
          cq += wrap ? 1 : 0;
        }
      }
    }
  };
  auto store_tiles = [&](int buf) {
    if constexpr (OP == 0) {
#pragma unroll
      for (int q = 0; q < RPA / 4; ++q)
        *reinterpret_cast<f32x4 *>(&As[buf][am][akg * RPA + 4 * q]) =
            f32x4{ra[4 * q], ra[4 * q + 1], ra[4 * q + 2], ra[4 * q + 3]};
#pragma unroll
      for (int q = 0; q < RPB / 4; ++q)
        *reinterpret_cast<f32x4 *>(&Bs[buf][bn][kg * RPB + 4 * q]) =
            f32x4{rb[4 * q], rb[4 * q + 1], rb[4 * q + 2], rb[4 * q + 3]};
    } else {
#pragma unroll
      for (int q = 0; q < RPA / 8; ++q)
        *reinterpret_cast<T8 *>(&As[buf][am][akg * RPA + 8 * q]) = cvt8<OP>(ra + 8 * q);
#pragma unroll
      for (int q = 0; q < RPB / 8; ++q)
        *reinterpret_cast<T8 *>(&Bs[buf][bn][kg * RPB + 8 * q]) = cvt8<OP>(rb + 8 * q);
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{0};
  const int li = lane & 31, lh = lane >> 5;
  // 16-bit: lane half h supplies k = 8h .. 8h+7 of each 16-deep MFMA (one b128 read per
  // fragment).  fp32 (v_mfma_f32_32x32x2_f32, exact): MFMA i of the step takes k = i from lane
  // half 0 and k = 16 + i from lane half 1, so a lane's 16 operands per row are one 64-B run
  // (four b128 reads); the 32 k are summed in that fixed order.
  auto compute = [&](int buf) {
    if constexpr (OP == 0) {
      float a[WM][16], b[WN][16];
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4 *>(&As[buf][32 * (WM * wm + i) + li][16 * lh + 4 * q]);
          a[i][4 * q] = v[0]; a[i][4 * q + 1] = v[1]; a[i][4 * q + 2] = v[2]; a[i][4 * q + 3] = v[3];
        }
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4 *>(&Bs[buf][32 * (WN * wn + j) + li][16 * lh + 4 * q]);
          b[j][4 * q] = v[0]; b[j][4 * q + 1] = v[1]; b[j][4 * q + 2] = v[2]; b[j][4 * q + 3] = v[3];
        }
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][kk], b[j][kk], acc[i][j], 0, 0, 0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < LKS / 16; ++kk) {
      T8 a[WM], b[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i)
        a[i] = *reinterpret_cast<const T8 *>(&As[buf][32 * (WM * wm + i) + li][16 * kk + 8 * lh]);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        b[j] = *reinterpret_cast<const T8 *>(&Bs[buf][32 * (WN * wn + j) + li][16 * kk + 8 * lh]);
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = mfma16<OP>(a[i], b[j], acc[i][j]);
    }
  };
  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      load_tiles(kbeg + kt + 1);          // past the range: re-reads, stored to the idle buffer
      __builtin_amdgcn_sched_barrier(0);  // loads first, then the step's MFMAs
      compute(kt & 1);
      __builtin_amdgcn_sched_barrier(0);  // the LDS write after all of the step's MFMAs
      store_tiles((kt + 1) & 1);
      __syncthreads();
    }
  }

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // splits == 1: final values (bias, act; MODE 1: + residual gradient) into dst;
  // splits > 1:  raw partial sums into part[split][m][n]: with `cnt` (the in-launch fold)
  // write-through, and the tile's last-arriving split sums every slab in split order
  // (k_conv_lp_reduce's order) and writes the final values; without, k_conv_lp_reduce does.
  if (splits > 1) {
    __shared__ int s_last;
    const int MN = M * Ntot;
    const __amdgpu_buffer_rsrc_t rp = rsrc(part + (size_t)split * MN, 4LL * MN);
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = n0 + 32 * (WN * wn + j) + li;
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * (WM * wm + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const int off = (n < Ntot && m < M) ? (m * Ntot + n) * 4 : OOR;
          if (cnt) bstore_sc1(rp, off, acc[i][j][r]);
          else bstore(rp, off, acc[i][j][r]);
        }
    }
    if (!cnt) return;
    handoff_drain();
    if (!handoff_arrive(cnt + bx + gx * by, splits, &s_last)) return;
    const __amdgpu_buffer_rsrc_t rall = rsrc(part, 4LL * splits * MN);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int k = 0; k < splits; ++k) {
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int n = n0 + 32 * (WN * wn + j) + li;
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + 32 * (WM * wm + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
            acc[i][j][r] += bload_sc1(rall, (n < Ntot && m < M) ? (k * MN + m * Ntot + n) * 4 : OOR);
          }
      }
    }
  }
  const __amdgpu_buffer_rsrc_t rd = rsrc(dst, dst_bytes);
  constexpr int ED = sizeof(TD);  // bytes per dst element (the fp32 residual: 4)
  const __amdgpu_buffer_rsrc_t rres = rsrc(bias, MODE == 1 && bias ? dst_bytes / ED * 4 : 0);
  const int Hd = MODE == 0 ? g.P : g.H, Wd = MODE == 0 ? g.Q : g.W;
  const int HWd = Hd * Wd;
  // MODE 0 with `stats`: BatchNorm partial sums of the stored values (bnstats.h)
  constexpr bool want_stats = ST && MODE == 0;  // BatchNorm partials: separate instantiation
  float fs[WM][16], fq[WM][16];  // this lane's WN values per row; fp64 from the butterfly on
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) fs[i][r] = fq[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int n = n0 + 32 * (WN * wn + j) + li;
    const bool nok = n < Ntot;
    int dbase, mstride;
    {
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
    for (int i = 0; i < WM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 32 * (WM * wm + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
        float v = acc[i][j][r];
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
          fs[i][r] += d;
          fq[i][r] = __builtin_fmaf(d, d, fq[i][r]);
        }
        bstore_t(rd, in ? e * ED : OOR, v, dst);
      }
    }
  }
  if (want_stats) {
    __shared__ double s_bn[2 * BMT * 2];  // [wn][row][2]
    double bs[WM][16], bq[WM][16];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        bs[i][r] = fs[i][r];
        bq[i][r] = fq[i][r];
      }
    bns_store_tile_n<WM>(bs, bq, 32 * WM * wm, wn, 2, BMT, m0, M, bx, s_bn, stats);
  }
}

template <int MODE, int ACT, int WM, int WN, int OP, int LKS, bool ST = false,
          typename TS = float, typename TD = float>
__global__ void __launch_bounds__(256) k_conv_lp(
    const float *__restrict__ w, const TS *__restrict__ src, const float *__restrict__ bias,
    TD *__restrict__ dst, long long dst_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part, unsigned int *__restrict__ cnt, double *__restrict__ stats) {
  typedef typename LpType<OP>::T T;
  constexpr int LD = lld_of(OP, LKS);
  __shared__ __attribute__((aligned(16))) T As[2][64 * WM][LD];
  __shared__ __attribute__((aligned(16))) T Bs[2][64 * WN][LD];
  int bx, by, bz;
  xcd_block(g.xcd != 0, bx, by, bz);
  conv_lp_block<MODE, ACT, WM, WN, OP, LKS, ST, TS, TD>(w, src, bias, dst, dst_bytes, g, M, splits,
                                                         kper, part, cnt, stats, bx, by, bz,
                                                         gridDim.x, As, Bs);
}

// split-K reduction (fixed order) + bias / relu / residual epilogue:
// out[img][m][p] = act(sum_s part[s][m][img*HW + p] + bias[m]) (+ res[img][m][p])
__global__ void __launch_bounds__(256) k_conv_lp_reduce(
    const float *__restrict__ part, int splits, int M, int HW, int Ntot,
    const float *__restrict__ bias, int act, const float *__restrict__ res,
    float *__restrict__ out) {
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

// ---- launch plan ---------------------------------------------------------------------------
struct LpPlan {
  int wm, wn, lk, splits, kper, nph;
  long long ncols;  // columns of the largest phase
};

static LpPlan lp_plan(int mode, const ConvGeom &g, int M, int op) {
  LpPlan p;
  const int Kc = mode == 0 ? g.Cin : g.Cout;
  p.nph = mode ? g.sh * g.sw : 1;
  p.ncols = 0;
  int taps_ph[MAXPH_LP];
  for (int z = 0; z < p.nph; ++z) {
    int taps = 0;
    long long cols;
    if (mode == 0) {
      cols = (long long)g.N * g.P * g.Q;
      int ty = 0, tx = 0;
      for (int r = 0; r < g.R; ++r) ty += axis_live(r * g.dh - g.ph, g.P, g.sh, g.H);
      for (int s = 0; s < g.S; ++s) tx += axis_live(s * g.dw - g.pw, g.Q, g.sw, g.W);
      taps = ty * tx;
    } else {
      const int py = z / g.sw, px = z % g.sw;
      const int Hp = py < g.H ? (g.H - py + g.sh - 1) / g.sh : 0;
      const int Wp = px < g.W ? (g.W - px + g.sw - 1) / g.sw : 0;
      cols = (long long)g.N * Hp * Wp;
      int ty = 0, tx = 0;
      for (int r = 0; r < g.R; ++r) {
        const int v = py + g.ph - r * g.dh;
        if (((v % g.sh) + g.sh) % g.sh == 0) ty += axis_live(floordiv(v, g.sh), Hp, 1, g.P);
      }
      for (int s = 0; s < g.S; ++s) {
        const int v = px + g.pw - s * g.dw;
        if (((v % g.sw) + g.sw) % g.sw == 0) tx += axis_live(floordiv(v, g.sw), Wp, 1, g.Q);
      }
      taps = ty * tx;
    }
    p.ncols = std::max(p.ncols, cols);
    taps_ph[z] = taps;
  }
  // rows: 128-row tiles when they pad M by at most 25 % (M = 112, 336, 672, 960 ...)
  const bool tall = cdiv(M, 128) * 128LL * 4 <= 5LL * M;
  p.wm = tall ? 2 : 1;
  const long long mb = cdiv(M, 64 * p.wm);
  // columns: the widest tile that still gives >= 2 workgroups per CU
  p.wn = 1;
  for (int wn = 4; wn >= 1; wn >>= 1) {
    if ((p.wm == 2 || op == 0) && wn == 4) continue;  // not instantiated
    if (cdiv(p.ncols, 64 * wn) * mb * p.nph >= 512 || wn == 1) {
      p.wn = wn;
      break;
    }
  }
  // fp32: 64 x 64 tiles (the larger fp32 tiles measured 1.3 - 2x slower: profiles/r03/lp/
  // conv_ab_fp32.txt)
  if (op == 0) p.wm = p.wn = 1;
  const int ft = g_tune[TUNE_LP_FORCE_TILE];  // benchmarking override: wm * 10 + wn
  if (ft > 1) {
    const int fwm = ft / 10, fwn = ft % 10;
    if ((fwm == 1 || fwm == 2) && (fwn == 1 || fwn == 2 || fwn == 4) && !((fwm == 2 || op == 0) && fwn == 4)) {
      p.wm = fwm;
      p.wn = fwn;
    }
  }
  // K-step depth: 32 (64-deep steps for the 16-bit operands, half the barriers and twice the
  // loads in flight per step, measured equal: 6.80 vs 6.79 ms for the bf16 conv set,
  // profiles/r03/lp/conv_ab_bf16_lk.txt; e2ep_tune key 16 forces 32 / 64 for A/B)
  p.lk = 32;
  if (op != 0 && (g_tune[TUNE_LP_LK] == 32 || (g_tune[TUNE_LP_LK] == 64 && p.wn <= 2)))
    p.lk = g_tune[TUNE_LP_LK];
  const int cfull = Kc / p.lk, crem = Kc - cfull * p.lk;
  int kmax = 0;
  for (int z = 0; z < p.nph; ++z)
    kmax = std::max(kmax, taps_ph[z] * cfull + cdiv((long long)crem * taps_ph[z], p.lk));
  const long long blocks = cdiv(p.ncols, 64 * p.wn) * cdiv(M, 64 * p.wm) * p.nph;
  p.splits = 1;
  if (blocks < 512 && p.nph == 1) {  // K split toward ~1024 workgroups, >= 4 steps each
    int s = (int)((1024 + blocks - 1) / blocks);
    s = std::min(s, std::max(1, kmax / 4));
    p.splits = std::max(1, std::min(s, 32));
  }
  p.kper = cdiv(std::max(kmax, 1), p.splits);
  if (p.splits > 1) p.splits = cdiv(kmax, p.kper);
  return p;
}

// Shapes left on k_conv_gemm (conv.hip), measured faster there (scripts/bench_conv.py --ab,
// profiles/r03/lp_ab.txt): M < 40 (it has 32-row tiles) and single-step K (Kc <= 32 on a 1x1:
// the 128x128-map expand / project convs, a streaming pass whose smaller tiles keep more
// workgroups in flight per CU).
bool lp_ok(int mode, const ConvGeom &g, int M, int op) {
  if (g_tune[TUNE_LP] == 1 || !(g.wlayout == 1 || g.R * g.S == 1)) return false;
  if (g_tune[TUNE_LP_FORCE_TILE] > 1) return true;  // benchmarking / tests: every shape
  const int Kc = mode == 0 ? g.Cin : g.Cout;
  // fp32 (e2ep_tune key 14): spatial filters with >= 64 rows and >= 64 channels per tap on
  // maps below k_conv_gemm2's range (3x3 layers of the BEV encoder / heads: -4..-6 us per launch
  // against k_conv_gemm; the 1x1s measured slower, profiles/r03/lp/conv_ab_fp32.txt)
  if (op == 0) return g.R * g.S > 1 && M >= 64 && Kc >= 64;
  return M >= 40 && (g.R * g.S > 1 || Kc > LK);
}

size_t lp_workspace(int mode, const ConvGeom &g, int M, int op) {
  const LpPlan p = lp_plan(mode, g, M, op);
  return p.splits > 1 ? (size_t)p.splits * M * p.ncols * sizeof(float) : 0;
}

template <int MODE, int ACT, int OP, typename TS = float, typename TD = float>
static void lp_tiles(const LpPlan &p, dim3 grid, hipStream_t s, const float *w, const TS *src,
                     const float *bias, TD *out, long long out_bytes, const ConvGeom &g, int M,
                     float *part, unsigned int *cnt, double *stats) {
#define LP_L(WMV, WNV)                                                                              \
  do {                                                                                              \
    if (OP != 0 && WNV <= 2 && p.lk == 64) {                                                        \
      if (MODE == 0 && stats)                                                                       \
        hipLaunchKernelGGL((k_conv_lp<MODE, ACT, WMV, WNV, OP, (OP != 0 && WNV <= 2) ? 64 : 32, true, TS, TD>), \
                           grid, dim3(256), 0, s, w, src, bias, out, out_bytes, g, M, p.splits,     \
                           p.kper, part, cnt, stats);                                               \
      else                                                                                          \
        hipLaunchKernelGGL((k_conv_lp<MODE, ACT, WMV, WNV, OP, (OP != 0 && WNV <= 2) ? 64 : 32, false, TS, TD>), \
                           grid, dim3(256), 0, s, w, src, bias, out, out_bytes, g, M, p.splits,     \
                           p.kper, part, cnt, nullptr);                                             \
    } else if (MODE == 0 && stats) {                                                                \
      hipLaunchKernelGGL((k_conv_lp<MODE, ACT, WMV, WNV, OP, 32, true, TS, TD>), grid, dim3(256), 0, s, \
                         w, src, bias, out, out_bytes, g, M, p.splits, p.kper, part, cnt, stats);   \
    } else {                                                                                        \
      hipLaunchKernelGGL((k_conv_lp<MODE, ACT, WMV, WNV, OP, 32, false, TS, TD>), grid, dim3(256), 0, s, \
                         w, src, bias, out, out_bytes, g, M, p.splits, p.kper, part, cnt, nullptr); \
    }                                                                                               \
  } while (0)
  if (p.wm == 2) {
    if (p.wn == 2) LP_L(2, 2);
    else LP_L(2, 1);
  } else {
    if constexpr (OP != 0) {
      if (p.wn == 4) {
        LP_L(1, 4);
        return;
      }
    }
    if (p.wn == 2) LP_L(1, 2);
    else LP_L(1, 1);
  }
#undef LP_L
}

int lp_stats_tiles(const ConvGeom &g, int op) {
  const LpPlan p = lp_plan(0, g, g.Cout, op);
  if (p.splits > 1 && g_tune[TUNE_SPLITK_FOLD] != 2) return 0;  // final values in the reduce
  return (int)cdiv(p.ncols, 64 * p.wn);
}

int lp_launch(int mode, int act, int op, const float *w, const void *src, const float *bias,
              void *dst, long long dst_bytes, const ConvGeom &g, int M, void *workspace,
              hipStream_t s, double *stats, int io) {
  const LpPlan p = lp_plan(mode, g, M, op);
  const dim3 grid(cdiv(p.ncols, 64 * p.wn), cdiv(M, 64 * p.wm), p.nph * p.splits);
  float *part = nullptr;
  unsigned int *cnt = nullptr;
  if (p.splits > 1) {
    if (!workspace) {
      set_error("conv (low precision): split-K plan needs a workspace (query the *_workspace entry point)");
      return E2EP_EINVAL;
    }
    part = static_cast<float *>(workspace);
    // in-launch fold (e2ep_tune key 28 = 2): one arrival counter per output tile
    if (g_tune[TUNE_SPLITK_FOLD] == 2) cnt = handoff_slots((int)grid.x * (int)grid.y, s);
  }
  if (stats && (mode != 0 || (p.splits > 1 && !cnt))) {
    set_error("conv (low precision): BatchNorm statistics need the forward with its final epilogue");
    return E2EP_EINVAL;
  }
  // bf16 storage: a bf16 forward input, or a bf16 data gradient written by the kernel's own
  // final epilogue (the separate split reduction writes fp32)
  const bool sb = mode == 0 && io == E2EP_IO_X_BF16, db = mode == 1 && io == E2EP_IO_DX_BF16;
  if (io && (op != 1 || !(sb || db) || (db && p.splits > 1 && !cnt))) {
    set_error("conv (low precision): storage mask %d not supported here (bf16 operands; forward "
              "input or data-gradient output; the in-launch split-K fold)", io);
    return E2EP_EINVAL;
  }
  // bias / residual: the kernel's final epilogue, or the separate reduction
  const float *kb = (p.splits > 1 && !cnt) ? nullptr : bias;
  const float *srcf = static_cast<const float *>(src);
  float *dstf = static_cast<float *>(dst);
#define LP_OPS(MD, AC)                                                     \
  do {                                                                     \
    if (op == 1 && sb)                                                     \
      lp_tiles<MD, AC, 1, bf16_t, float>(p, grid, s, w, static_cast<const bf16_t *>(src), kb, dstf, \
                                         dst_bytes, g, M, part, cnt, stats); \
    else if (op == 1 && db)                                                \
      lp_tiles<MD, AC, 1, float, bf16_t>(p, grid, s, w, srcf, kb, static_cast<bf16_t *>(dst), \
                                         dst_bytes, g, M, part, cnt, stats); \
    else if (op == 1) lp_tiles<MD, AC, 1>(p, grid, s, w, srcf, kb, dstf, dst_bytes, g, M, part, cnt, stats); \
    else if (op == 2) lp_tiles<MD, AC, 2>(p, grid, s, w, srcf, kb, dstf, dst_bytes, g, M, part, cnt, stats); \
    else lp_tiles<MD, AC, 0>(p, grid, s, w, srcf, kb, dstf, dst_bytes, g, M, part, cnt, stats); \
  } while (0)
  if (mode == 0 && act == 0) LP_OPS(0, 0);
  else if (mode == 0) LP_OPS(0, 1);
  else LP_OPS(1, 0);
#undef LP_OPS
  if (p.splits > 1 && !cnt) {
    const int HW = mode == 0 ? g.P * g.Q : g.H * g.W;
    hipLaunchKernelGGL(k_conv_lp_reduce, dim3(cdiv(p.ncols, 256), M), dim3(256), 0, s,
                       static_cast<const float *>(workspace), p.splits, M, HW, (int)p.ncols,
                       mode == 0 ? bias : nullptr, act, mode == 1 ? bias : nullptr, dstf);
  }
  return 0;
}

// ------------------------------------------------------------------------------------------
// bf16 weight gradient (BASELINE C3: bf16 operands, fp32 accumulate and gradient).
//   dW[co][ci*RS + tap] = sum_(n,p) g[n,co,p] x[n,ci,p+tap]: M = Cout, N = (ci, live tap)
//   columns, K = pixels, split over blocks into fixed-order partial slabs (k_reduce_splits).
// k_conv_wgrad2 (conv.hip) with bf16 operands runs two 16-deep MFMAs per 64 x 64 tile and
// 32-pixel step, converting every fragment from fp32 LDS rows.  Here, as in k_conv_lp, the
// operands are converted once into 16-bit LDS rows (32 pixels + 8 pad), tiles are up to
// 128 x 128 (wave tiles up to 64 x 64: 8 MFMAs per wave per step), and:
//  * A = g rows: a thread owns 8 consecutive pixels of a row (two float4 loads, one b128
//    LDS write);
//  * B = im2col x columns (16-bit operands, round 5): a thread owns (column, pixel octet)
//    pairs — 8 consecutive output pixels of one column, inside one output row (Q % 8 == 0) —
//    whose input window is read as 2 float4 (stride 1) or 4 float4 (stride 2, every other
//    value kept) when it lies inside the input row, value by value at the row ends, and
//    written as one bf16x8 (b128) LDS row segment: 2 (stride 1) / 4 (stride 2) loads and 1 LDS
//    write per 8 values where the pixel-pair form took 8 scalar loads and 4 b32 writes
//    (the fp32 form, OP 0, keeps the pixel pairs: a thread owns a pixel PAIR of BNT/16
//    columns, packed per column);
//  * a step never straddles two images (P*Q % 32 == 0, every hot-path map), so its image and
//    first pixel are block-uniform.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// OP 0: the same GEMM on the exact-f32 MFMA with fp32 LDS rows (k_conv_lp's fp32 K order).
// The block body for block (bx, by, bz) of a grid with gz pixel splits, its operand tiles in
// the caller's LDS: k_wgrad_lp, and the weight-gradient half of k_lp_bwd_pair.
template <int WM, int WN, int OP, int LKS, typename TX = float>
__device__ __forceinline__ void wgrad_lp_block(
    const float *__restrict__ gout, const TX *__restrict__ x, float *__restrict__ part,
    ConvGeom g, int pix_per_split, TapList tl, int bx, int by, int bz, int gz,
    typename LpType<OP == 0 ? 0 : 1>::T (*As)[64 * WM][lld_of(OP, LKS)],
    typename LpType<OP == 0 ? 0 : 1>::T (*Bs)[64 * WN][lld_of(OP, LKS)]) {
  constexpr int BMT = 64 * WM, BNT = 64 * WN;
  static_assert(OP != 0 || LKS == 32, "fp32: 32-pixel steps");
  constexpr int OPR = LKS / 8;             // A pixel octets per row
  constexpr int NA8 = BMT * OPR / 256;     // A octets per thread
  constexpr int PP = LKS / 2;              // B pixel pairs per step
  constexpr int CG = 256 / PP;             // B column groups
  constexpr int NBC = BNT / CG;            // B columns per thread
  // As[co][pixel], Bs[column][pixel]
  __shared__ int s_tap[MAXTAPS];
  if (threadIdx.x < MAXTAPS) s_tap[threadIdx.x] = threadIdx.x < tl.n ? tl.tap[threadIdx.x] : 0;
  __syncthreads();

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int RS = g.R * g.S;
  const int Kw = g.Cin * RS;    // columns of dW (ci-major, tap-minor)
  const int Kl = g.Cin * tl.n;  // live columns (ci, live tap index)
  const int n0 = bx * BNT, m0 = by * BMT;
  const int split = bz;
  const int PQ = g.P * g.Q;
  const int Ptot = g.N * PQ;
  const int pbeg = split * pix_per_split;  // a multiple of LKS
  const int pend = min(Ptot, pbeg + pix_per_split);
  const int nk = max(0, (pend - pbeg) / LKS);
  const int HW = g.H * g.W;

  // A: octet o = tid + 256 i -> (co row o / OPR, pixel octet o % OPR)
  // B (OP 0): thread = (pixel pair tid % PP, column group tid / PP): columns bcg + CG j
  // B (16-bit): thread = (pixel octet tid % OCT, column tid / OCT + (256 / OCT) j)
  constexpr int OCT = LKS / 8;                    // pixel octets per column per step
  constexpr int NOC = OP == 0 ? 1 : BNT * OCT / 256;  // (column, octet) pairs per thread
  static_assert(OP == 0 || (BNT * OCT) % 256 == 0, "whole (column, octet) pairs per thread");
  constexpr int NCOL = OP == 0 ? NBC : NOC;       // columns per thread
  const int bq = tid % PP, bcg = tid / PP;
  const int boc = tid % OCT, bcol = tid / OCT;
  int cconst[NCOL], cdy[NCOL], cdx[NCOL];
#pragma unroll
  for (int j = 0; j < NCOL; ++j) {
    const int col = n0 + (OP == 0 ? bcg + CG * j : bcol + (256 / OCT) * j);
    const int cc = col < Kl ? col : 0;
    const int ci = cc / tl.n, tap = s_tap[cc - ci * tl.n];
    const int r = tap / g.S, sx = tap - r * g.S;
    cdy[j] = r * g.dh - g.ph;
    cdx[j] = sx * g.dw - g.pw;
    cconst[j] = ci * HW + cdy[j] * g.W + cdx[j];
    if (col >= Kl) cdy[j] = -(1 << 29);  // never in bounds
  }
  const __amdgpu_buffer_rsrc_t rg = rsrc(gout, 4LL * g.N * g.Cout * PQ);
  constexpr int EX = sizeof(TX);  // bytes per x element (bf16: C3's stored SE output)
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, (long long)EX * g.N * g.Cin * HW);
  const int nrx = (int)min((long long)EX * g.N * g.Cin * HW, 0x7fffffffLL);

  float4 ra[NA8][2];
  float rb[NBC][2];
  float4 rv[NOC][4];  // 16-bit B: a pair's window (stride 1: [0..1]; stride 2: [0..3], .x / .z kept)
  auto load_tiles = [&](int ks) {
    const int p0 = pbeg + min(ks, nk - 1) * LKS;  // past the range: re-read, never stored
    const int im = p0 / PQ, od0 = p0 - im * PQ;    // block-uniform
#pragma unroll
    for (int i = 0; i < NA8; ++i) {
      const int o = tid + 256 * i, ar = o / OPR, ao = o % OPR;
      const int co = m0 + ar;
      const int base = co < g.Cout ? ((im * g.Cout + co) * PQ + od0 + 8 * ao) * 4 : OOR;
      ra[i][0] = bload4(rg, base);
      ra[i][1] = bload4(rg, base + 16);
    }
    if constexpr (OP == 0) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int od = od0 + 2 * bq + e;
        const int oy = od / g.Q, ox = od - oy * g.Q;
        const int yb = oy * g.sh, xb = ox * g.sw;
        const int pbase = im * g.Cin * HW + yb * g.W + xb;
#pragma unroll
        for (int j = 0; j < NBC; ++j) {
          const bool ok = (unsigned)(yb + cdy[j]) < (unsigned)g.H && (unsigned)(xb + cdx[j]) < (unsigned)g.W;
          rb[j][e] = bload_t(rx, ok ? (pbase + cconst[j]) * EX : nrx, x);
        }
      }
    } else {
      const int od = od0 + 8 * boc;  // the octet's first output pixel (one output row)
      const int oy = od / g.Q, ox = od - oy * g.Q;
      const int yb = oy * g.sh, xb = ox * g.sw;
      const int pbase = im * g.Cin * HW + yb * g.W + xb;
      const int last = 7 * g.sw;  // the window's last input column past its first
#pragma unroll
      for (int j = 0; j < NOC; ++j) {
        const int x0 = xb + cdx[j];
        const bool rowok = (unsigned)(yb + cdy[j]) < (unsigned)g.H;  // dead columns: never
        const int base = pbase + cconst[j];  // element offset of the window's first value
        if (rowok && x0 >= 0 && x0 + last < g.W) {  // inside the row: vector loads
          if constexpr (EX == 2) {  // bf16 x: 4 (stride 1) / 8 (stride 2) values per 8-B load
            rv[j][0] = bload4t(rx, base * 2, x);
            rv[j][1] = bload4t(rx, base * 2 + 8, x);
            if (g.sw == 2) {
              rv[j][2] = bload4t(rx, base * 2 + 16, x);
              rv[j][3] = bload4t(rx, base * 2 + 24, x);
            }
          } else {
            rv[j][0] = bload4(rx, base * 4);
            rv[j][1] = bload4(rx, base * 4 + 16);
            if (g.sw == 2) {
              rv[j][2] = bload4(rx, base * 4 + 32);
              rv[j][3] = bload4(rx, base * 4 + 48);
            }
          }
        } else {  // a row end (zero padding) or a dead column: value by value
          float t[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const bool ok = rowok && (unsigned)(x0 + q * g.sw) < (unsigned)g.W;
            t[q] = bload_t(rx, ok ? (base + q * g.sw) * EX : nrx, x);
          }
          if (g.sw == 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) rv[j][q] = make_float4(t[2 * q], 0.f, t[2 * q + 1], 0.f);
          } else {
            rv[j][0] = make_float4(t[0], t[1], t[2], t[3]);
            rv[j][1] = make_float4(t[4], t[5], t[6], t[7]);
          }
        }
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA8; ++i) {
      const int o = tid + 256 * i, ar = o / OPR, ao = o % OPR;
      if constexpr (OP == 0) {
        *reinterpret_cast<float4 *>(&As[buf][ar][8 * ao]) = ra[i][0];
        *reinterpret_cast<float4 *>(&As[buf][ar][8 * ao + 4]) = ra[i][1];
      } else {
        const float v[8] = {ra[i][0].x, ra[i][0].y, ra[i][0].z, ra[i][0].w,
                            ra[i][1].x, ra[i][1].y, ra[i][1].z, ra[i][1].w};
        *reinterpret_cast<bf16x8 *>(&As[buf][ar][8 * ao]) = cvt8<1>(v);
      }
    }
    if constexpr (OP == 0) {
#pragma unroll
      for (int j = 0; j < NBC; ++j) {
        const f32x2 f = {rb[j][0], rb[j][1]};
        *reinterpret_cast<f32x2 *>(&Bs[buf][bcg + CG * j][2 * bq]) = f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NOC; ++j) {
        float v[8];
        if (g.sw == 2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[2 * q] = rv[j][q].x;
            v[2 * q + 1] = rv[j][q].z;
          }
        } else {
          v[0] = rv[j][0].x; v[1] = rv[j][0].y; v[2] = rv[j][0].z; v[3] = rv[j][0].w;
          v[4] = rv[j][1].x; v[5] = rv[j][1].y; v[6] = rv[j][1].z; v[7] = rv[j][1].w;
        }
        *reinterpret_cast<bf16x8 *>(&Bs[buf][bcol + (256 / OCT) * j][8 * boc]) = cvt8<1>(v);
      }
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{0};
  const int li = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    if constexpr (OP == 0) {  // MFMA i: k = i (lane half 0) and 16 + i (lane half 1)
      float a[WM][16], b[WN][16];
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4 *>(&As[buf][32 * (WM * wm + i) + li][16 * lh + 4 * q]);
          a[i][4 * q] = v[0]; a[i][4 * q + 1] = v[1]; a[i][4 * q + 2] = v[2]; a[i][4 * q + 3] = v[3];
        }
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4 *>(&Bs[buf][32 * (WN * wn + j) + li][16 * lh + 4 * q]);
          b[j][4 * q] = v[0]; b[j][4 * q + 1] = v[1]; b[j][4 * q + 2] = v[2]; b[j][4 * q + 3] = v[3];
        }
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][kk], b[j][kk], acc[i][j], 0, 0, 0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < LKS / 16; ++kk) {
      bf16x8 a[WM], b[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i)
        a[i] = *reinterpret_cast<const bf16x8 *>(&As[buf][32 * (WM * wm + i) + li][16 * kk + 8 * lh]);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        b[j] = *reinterpret_cast<const bf16x8 *>(&Bs[buf][32 * (WN * wn + j) + li][16 * kk + 8 * lh]);
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
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
      __builtin_amdgcn_sched_barrier(0);  // the LDS write after all of the step's MFMAs
      store_tiles((kt + 1) & 1);
      __syncthreads();
    }
  }
  const __amdgpu_buffer_rsrc_t rp = rsrc(part, 4LL * gz * g.Cout * Kw);
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int lcol = n0 + 32 * (WN * wn + j) + li;
    const int lci = lcol < Kl ? lcol / tl.n : 0;
    const int col = lci * RS + s_tap[lcol < Kl ? lcol - lci * tl.n : 0];  // dW column
#pragma unroll
    for (int i = 0; i < WM; ++i) {
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int co = m0 + 32 * (WM * wm + i) + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
        const bool ok = co < g.Cout && lcol < Kl;
        bstore(rp, ok ? ((split * g.Cout + co) * Kw + col) * 4 : OOR, acc[i][j][rr]);
      }
    }
  }
}

template <int WM, int WN, int OP, int LKS, typename TX = float>
__global__ void __launch_bounds__(256) k_wgrad_lp(const float *__restrict__ gout,
                                                  const TX *__restrict__ x,
                                                  float *__restrict__ part, ConvGeom g,
                                                  int pix_per_split, TapList tl) {
  typedef typename LpType<OP == 0 ? 0 : 1>::T T;
  constexpr int LD = lld_of(OP, LKS);
  __shared__ __attribute__((aligned(16))) T As[2][64 * WM][LD];
  __shared__ __attribute__((aligned(16))) T Bs[2][64 * WN][LD];
  int bx, by, bz;
  xcd_block(g.xcd != 0, bx, by, bz);
  wgrad_lp_block<WM, WN, OP, LKS, TX>(gout, x, part, g, pix_per_split, tl, bx, by, bz, gridDim.z, As,
                                      Bs);
}

// A conv layer's data gradient (k_conv_lp MODE 1) and weight gradient (k_wgrad_lp slabs) in
// one grid: blocks [0, n1) run the data gradient, the rest the weight gradient (reduced by
// k_reduce_splits after the launch).  One launch instead of two on forked streams
// (e2ep_conv_bwd): in a replayed graph a fork / join idles the GPU ~15 us.  LDS: the larger
// of the two halves' operand tiles, one buffer.  fp32 (OP 0) pairs the 64 x 64 weight-gradient
// tile, whose K order and slabs are k_conv_wgrad2's (the kernel the two-launch fp32 path runs).
template <int DWM, int DWN, int OP, int WWM, int WWN, typename TX = float>
__global__ void __launch_bounds__(256) k_lp_bwd_pair(
    const float *__restrict__ w, const float *__restrict__ gout, const float *__restrict__ res,
    TX *__restrict__ dx, long long dx_bytes, ConvGeom g, int M, int splits, int kper,
    float *__restrict__ part1, unsigned int *__restrict__ cnt, int gx1, int gy1, int gz1,
    const TX *__restrict__ x, float *__restrict__ part2, int pix_per_split, TapList tl,
    int gx2, int gy2, int gz2) {
  typedef typename LpType<OP>::T T;
  constexpr int LD = lld_of(OP, LK);
  constexpr int L1 = 2 * 64 * (DWM + DWN) * LD, L2 = 2 * 64 * (WWM + WWN) * LD;
  __shared__ __attribute__((aligned(16))) T lds[L1 > L2 ? L1 : L2];
  const int n1 = gx1 * gy1 * gz1;  // data-gradient blocks first (as k_conv_bwd_pair)
  int id = (int)blockIdx.x;
  if (id < n1) {
    if (g.xcd) id = xcd_linear(id, n1);
    conv_lp_block<1, 0, DWM, DWN, OP, LK, false, float, TX>(
        w, gout, res, dx, dx_bytes, g, M, splits, kper, part1, cnt, nullptr, id % gx1,
        (id / gx1) % gy1, id / (gx1 * gy1), gx1, reinterpret_cast<T(*)[64 * DWM][LD]>(lds),
        reinterpret_cast<T(*)[64 * DWN][LD]>(lds + 2 * 64 * DWM * LD));
  } else {
    id -= n1;
    const int n2 = gx2 * gy2 * gz2;
    if (g.xcd) id = xcd_linear(id, n2);
    wgrad_lp_block<WWM, WWN, OP, LK, TX>(
        gout, x, part2, g, pix_per_split, tl, id % gx2, (id / gx2) % gy2, id / (gx2 * gy2), gz2,
        reinterpret_cast<T(*)[64 * WWM][LD]>(lds),
        reinterpret_cast<T(*)[64 * WWN][LD]>(lds + 2 * 64 * WWM * LD));
  }
}

// pixels per K-step of k_wgrad_lp: 32 (bf16 64-pixel steps measured equal, 128 slower: register
// pressure, removed in round 5; e2ep_tune key 17 forces 32 / 64 for A/B), fp32 32
static int lp_wgrad_lk(const ConvGeom &g, int op) {
  const int pq = g.P * g.Q, f = g_tune[TUNE_LPW_LK];
  if (op == 0) return 32;
  if ((f == 32 || f == 64) && pq % f == 0) return f;
  return 32;
}

static void lp_wgrad_tile(const ConvGeom &g, const TapList &tl, int &wm, int &wn) {
  const int Kl = g.Cin * tl.n;
  wm = cdiv(g.Cout, 128) * 128LL * 4 <= 5LL * g.Cout ? 2 : 1;
  wn = cdiv(Kl, 128) * 128LL * 4 <= 5LL * Kl ? 2 : 1;
  // few pixels (slabs of >= 8 steps): smaller tiles until the grid has >= 256 workgroups
  const long long cap = std::max(1LL, (long long)g.N * g.P * g.Q / 256);
  while (wm * wn > 1 && (long long)cdiv(Kl, 64 * wn) * cdiv(g.Cout, 64 * wm) * std::min(cap, 256LL) < 256) {
    if (wm >= wn) wm = 1;
    else wn = 1;
  }
  const int ft = g_tune[TUNE_LP_WGRAD_TILE];  // benchmarking override: wm * 10 + wn
  if (ft > 1 && (ft / 10 == 1 || ft / 10 == 2) && (ft % 10 == 1 || ft % 10 == 2)) {
    wm = ft / 10;
    wn = ft % 10;
  }
}

// Few (Cout, column) pairs over many pixels (the 128x128 maps' 24 / 48-channel 1x1s, the
// segmentation classifier) stay on k_wgrad_1x1 / k_conv_wgrad2, measured faster there.
bool lp_wgrad_ok(const ConvGeom &g, const TapList &tl) {
  // Q % 8 == 0 and stride 1 / 2 along x: the 16-bit B staging's pixel octets (one output row,
  // 2 or 4 float4 per input window); the fp32 form (OP 0) reads pixel pairs but shares the rule
  if (tl.n <= 0 || (g.P * g.Q) % LK != 0 || g.Q % 8 != 0 || (g.sw != 1 && g.sw != 2)) return false;
  return g_tune[TUNE_LP_WGRAD_TILE] > 1 || (long long)g.Cout * g.Cin * tl.n >= 2048;
}

int lp_wgrad_splits(const ConvGeom &g, const TapList &tl, int op) {
  int wm, wn;
  lp_wgrad_tile(g, tl, wm, wn);
  const int lk = lp_wgrad_lk(g, op);
  const long long tiles = (long long)cdiv(g.Cin * tl.n, 64 * wn) * cdiv(g.Cout, 64 * wm);
  const long long pix = (long long)g.N * g.P * g.Q;
  const long long target = g_tune[TUNE_LPW_TARGET];  // workgroups aimed at (e2ep_tune key 22)
  long long s = (target + tiles - 1) / tiles;
  s = std::min(s, std::max(1LL, pix / (std::max(256, 4 * lk))));  // >= 256 pixels per slab
  return (int)std::max(1LL, std::min(s, 256LL));
}

int lp_wgrad_launch(const float *gout, const void *xv, const ConvGeom &g, const TapList &tl,
                    int splits, float *part, hipStream_t s, int op, bool xb) {
  const float *x = static_cast<const float *>(xv);
  const bf16_t *xh = static_cast<const bf16_t *>(xv);
  int wm, wn;
  lp_wgrad_tile(g, tl, wm, wn);
  const int lk = lp_wgrad_lk(g, op);
  const int Ptot = g.N * g.P * g.Q;
  int per = (Ptot + splits - 1) / splits;
  per = (per + lk - 1) / lk * lk;
  const int used = (Ptot + per - 1) / per;
  const dim3 grid(cdiv(g.Cin * tl.n, 64 * wn), cdiv(g.Cout, 64 * wm), used);
#define WL(WMV, WNV)                                                                             \
  do {                                                                                           \
    if (op != 1)                                                                                 \
      hipLaunchKernelGGL((k_wgrad_lp<WMV, WNV, 0, 32>), grid, dim3(256), 0, s, gout, x, part, g, per, tl); \
    else if (xb && lk == 64)                                                                     \
      hipLaunchKernelGGL((k_wgrad_lp<WMV, WNV, 1, 64, bf16_t>), grid, dim3(256), 0, s, gout, xh, part, g, per, tl); \
    else if (xb)                                                                                 \
      hipLaunchKernelGGL((k_wgrad_lp<WMV, WNV, 1, 32, bf16_t>), grid, dim3(256), 0, s, gout, xh, part, g, per, tl); \
    else if (lk == 64)                                                                           \
      hipLaunchKernelGGL((k_wgrad_lp<WMV, WNV, 1, 64>), grid, dim3(256), 0, s, gout, x, part, g, per, tl); \
    else                                                                                         \
      hipLaunchKernelGGL((k_wgrad_lp<WMV, WNV, 1, 32>), grid, dim3(256), 0, s, gout, x, part, g, per, tl); \
  } while (0)
  if (wm == 2 && wn == 2) WL(2, 2);
  else if (wm == 2) WL(2, 1);
  else if (wn == 2) WL(1, 2);
  else WL(1, 1);
#undef WL
  return used;
}

// ---- paired backward (k_lp_bwd_pair) ------------------------------------------------------
// Instantiated pairs: fp32 (op 0) 64 x 64 data-gradient tiles with the 64 x 64 weight-gradient
// tile; bf16 (op 1) data-gradient tiles 64 x 64, 128 x 64 and 64 x 128 with weight-gradient
// tiles 64 / 128 x 64 / 128, 32-deep K-steps on both (the plans' defaults).
static bool lp_pair_tiles(const ConvGeom &g, int M, int op, const TapList &tl, LpPlan &p,
                          int &wwm, int &wwn) {
  p = lp_plan(1, g, M, op);
  if (p.lk != LK || (p.splits > 1 && g_tune[TUNE_SPLITK_FOLD] != 2)) return false;
  if (op == 0) {
    wwm = wwn = 1;
    return p.wm == 1 && p.wn == 1 && (g.P * g.Q) % LK == 0;
  }
  // not the 128 x 128 data-gradient tile: its ~200 VGPRs hold the whole paired grid to one
  // workgroup per SIMD, and the weight-gradient blocks then run at a third of their occupancy
  // (C3: 87 us paired against ~39 + 44 us overlapped on two streams).  Without a K split the
  // pair runs that data gradient on 128 x 64 tiles instead: every output's K order is the
  // same whatever the tile, so the results stay bitwise those of the two-launch path.
  if (op == 1 && p.wm == 2 && p.wn == 2 && p.splits == 1) p.wn = 1;
  if (op != 1 || p.wn > 2 || (p.wm == 2 && p.wn == 2) || !lp_wgrad_ok(g, tl) ||
      lp_wgrad_lk(g, op) != LK)
    return false;
  lp_wgrad_tile(g, tl, wwm, wwn);
  return true;
}

bool lp_bwd_pair_ok(const ConvGeom &g, int M, int op, const TapList &tl) {
  LpPlan p;
  int wwm, wwn;
  return lp_pair_tiles(g, M, op, tl, p, wwm, wwn);
}

int lp_bwd_pair_launch(const float *w, const float *gout, const float *res, void *dxv,
                       long long dx_bytes, const ConvGeom &g, int M, int op, void *ws_dgrad,
                       const void *xv, const TapList &tl, int wsplits, float *part2,
                       hipStream_t s, bool xb) {
  LpPlan p;
  int wwm, wwn;
  if (!lp_pair_tiles(g, M, op, tl, p, wwm, wwn)) return -1;
  if (xb && op != 1) return -1;
  float *dx = static_cast<float *>(dxv);
  const float *x = static_cast<const float *>(xv);
  bf16_t *dxh = static_cast<bf16_t *>(dxv);
  const bf16_t *xh = static_cast<const bf16_t *>(xv);
  const dim3 g1(cdiv(p.ncols, 64 * p.wn), cdiv(M, 64 * p.wm), p.nph * p.splits);
  float *part1 = p.splits > 1 ? static_cast<float *>(ws_dgrad) : nullptr;
  unsigned int *cnt = p.splits > 1 ? handoff_slots((int)g1.x * (int)g1.y, s) : nullptr;
  const int Ptot = g.N * g.P * g.Q;
  int per = (Ptot + wsplits - 1) / wsplits;
  per = (per + LK - 1) / LK * LK;
  const int used = (Ptot + per - 1) / per;
  const dim3 g2(cdiv(g.Cin * tl.n, 64 * wwn), cdiv(g.Cout, 64 * wwm), used);
  const dim3 grid(g1.x * g1.y * g1.z + g2.x * g2.y * g2.z);
#define PAIR_L(DM, DN, OPV, WMV, WNV)                                                           \
  do {                                                                                          \
    if (OPV == 1 && xb)                                                                         \
      hipLaunchKernelGGL((k_lp_bwd_pair<DM, DN, OPV, WMV, WNV, bf16_t>), grid, dim3(256), 0, s, w, \
                         gout, res, dxh, dx_bytes, g, M, p.splits, p.kper, part1, cnt, (int)g1.x, \
                         (int)g1.y, (int)g1.z, xh, part2, per, tl, (int)g2.x, (int)g2.y, (int)g2.z); \
    else                                                                                        \
      hipLaunchKernelGGL((k_lp_bwd_pair<DM, DN, OPV, WMV, WNV>), grid, dim3(256), 0, s, w, gout,  \
                         res, dx, dx_bytes, g, M, p.splits, p.kper, part1, cnt, (int)g1.x,       \
                         (int)g1.y, (int)g1.z, x, part2, per, tl, (int)g2.x, (int)g2.y, (int)g2.z); \
  } while (0)
#define PAIR_W(DM, DN)                                     \
  do {                                                     \
    if (wwm == 2 && wwn == 2) PAIR_L(DM, DN, 1, 2, 2);     \
    else if (wwm == 2) PAIR_L(DM, DN, 1, 2, 1);            \
    else if (wwn == 2) PAIR_L(DM, DN, 1, 1, 2);            \
    else PAIR_L(DM, DN, 1, 1, 1);                          \
  } while (0)
  if (op == 0) PAIR_L(1, 1, 0, 1, 1);
  else if (p.wm == 2) PAIR_W(2, 1);
  else if (p.wn == 2) PAIR_W(1, 2);
  else PAIR_W(1, 1);
#undef PAIR_W
#undef PAIR_L
  if (p.splits > 1 && !cnt)  // no fold counters: the data gradient's slabs reduced here
    hipLaunchKernelGGL(k_conv_lp_reduce, dim3(cdiv(p.ncols, 256), M), dim3(256), 0, s,
                       static_cast<const float *>(part1), p.splits, M, g.H * g.W, (int)p.ncols,
                       nullptr, 0, res, dx);
  return used;
}

}  // namespace e2ep
