// Internal interface shared by the convolution kernel files (conv.hip, conv_lp.hip).
#pragma once
#include "common.h"

namespace e2ep {

constexpr int MAXTAPS = 64;  // live filter taps per phase (R * S <= 64)

struct ConvGeom {
  int N;            // images
  int Cin, H, W;    // input
  int Cout, R, S;   // filter
  int P, Q;         // output spatial
  int sh, sw, ph, pw, dh, dw;
  int wlayout;      // 0: [Cout][Cin][R*S] (PyTorch), 1: [R*S][Cout][Cin] (tap-major)
  int korder;       // forward / data-gradient K order: 0 tap-outer, 1 channel-chunk-outer
  int xcd;          // conv_lp.hip kernels: 1 = XCD-contiguous block order (xcd_block)
};

// XCD-contiguous logical block index: hardware block i runs on XCD i % 8 (a placement used for
// speed only, never for correctness); logical = the i-th block of that XCD's contiguous share
// of the grid, so neighbouring tiles (shared input rows, shared gradient rows) meet in one XCD's
// L2.  A bijection for any grid size.
__device__ __forceinline__ int xcd_linear(int i, int total) {
  const int q = total >> 3, r = total & 7, x = i & 7, j = i >> 3;
  return x * q + min(x, r) + j;
}

__device__ __forceinline__ void xcd_block(bool on, int &bx, int &by, int &bz) {
  bx = blockIdx.x;
  by = blockIdx.y;
  bz = blockIdx.z;
  if (!on) return;
  const int gx = gridDim.x, gy = gridDim.y;
  const int total = gx * gy * gridDim.z;
  const int L = xcd_linear(bx + gx * (by + gy * bz), total);
  bx = L % gx;
  by = (L / gx) % gy;
  bz = L / (gx * gy);
}

__host__ __device__ __forceinline__ int floordiv(int a, int b) {
  return a >= 0 ? a / b : -((-a + b - 1) / b);
}

// Tap liveness: does any output position o in [0, n_out) read an input o*step + d inside
// [0, n_in)?  A filter tap that never does only multiplies zero padding (the DeepLab ASPP
// branches at dilation 24 / 36 on 16x16 maps, reference model/convolutions.py:218-225: 8 of
// their 9 taps), so the GEMMs skip it: the sums are unchanged (those products are exact
// zeros) and the weight gradient of such a tap is exactly 0.
__host__ __device__ __forceinline__ bool axis_live(int d, int n_out, int step, int n_in) {
  if (n_out <= 0) return false;
  const int o0 = d >= 0 ? 0 : (-d + step - 1) / step;
  return o0 < n_out && o0 * step + d < n_in;
}

// live filter taps (axis_live on both axes): the weight-gradient GEMMs run over the columns
// (ci, live tap) only; the dead taps' gradient is written as 0 by the split reduction
struct TapList {
  int n;
  unsigned long long mask;  // bit tap = live (R*S <= MAXTAPS = 64)
  int tap[MAXTAPS];
};

// Implicit-GEMM forward (mode 0) / data gradient (mode 1) with 32-deep K-steps and up to
// 128-row tiles, conv_lp.hip: bf16 / fp16 operands (op 1 / 2), and fp32 (op 0) where
// TUNE_LP32 selects it.  lp_workspace() bytes of split-K workspace (0: none); lp_launch() returns an
// E2EP status.  Tap-major weights ([R*S][Cout][Cin]) or 1x1 filters only.
bool lp_ok(int mode, const ConvGeom &g, int M, int op);
size_t lp_workspace(int mode, const ConvGeom &g, int M, int op);
// stats (forward only): BatchNorm partial sums of dst from the epilogue (bnstats.h), over
// lp_stats_tiles(g, op) column tiles (0 = the plan cannot produce them).
// io (e2ep.h E2EP_IO_*, op 1 only): mode 0 with E2EP_IO_X_BF16 reads a bf16 src, mode 1 with
// E2EP_IO_DX_BF16 writes a bf16 dst (dst_bytes: its size in bytes); E2EP_EINVAL otherwise.
int lp_launch(int mode, int act, int op, const float *w, const void *src, const float *bias,
              void *dst, long long dst_bytes, const ConvGeom &g, int M, void *workspace,
              hipStream_t s, double *stats = nullptr, int io = 0);
int lp_stats_tiles(const ConvGeom &g, int op);

// Weight gradient with 32-pixel K-steps and up to 128 x 128 tiles, conv_lp.hip: bf16 operands
// (op 1, C3) or fp32 (op 0, where TUNE_LP32W selects it).  Partial slabs
// part[split][Cout][Cin*R*S] for the fixed-order split reduction of conv.hip;
// lp_wgrad_launch returns the slabs written.
bool lp_wgrad_ok(const ConvGeom &g, const TapList &tl);
int lp_wgrad_splits(const ConvGeom &g, const TapList &tl, int op);
// xb: x is bf16 (op 1 only)
int lp_wgrad_launch(const float *gout, const void *x, const ConvGeom &g, const TapList &tl,
                    int splits, float *part, hipStream_t s, int op, bool xb = false);

// A conv layer's data gradient on k_conv_lp (route ROUTE_LP / ROUTE_LP32 of conv.hip) and
// weight gradient (op 1: k_wgrad_lp; op 0: the k_conv_wgrad2-equivalent 64 x 64 tile) in one
// k_lp_bwd_pair launch (e2ep_conv_bwd).  lp_bwd_pair_launch returns the weight-gradient slabs
// written to part2 (for the split reduction), -1 if the plan has no instantiated pair.
bool lp_bwd_pair_ok(const ConvGeom &g, int M, int op, const TapList &tl);
// xb: x and dx are bf16 (op 1 only; dx_bytes its size in bytes)
int lp_bwd_pair_launch(const float *w, const float *gout, const float *res, void *dx,
                       long long dx_bytes, const ConvGeom &g, int M, int op, void *ws_dgrad,
                       const void *x, const TapList &tl, int wsplits, float *part2,
                       hipStream_t s, bool xb = false);

// Direct convolution of a 7x7 / 2 conv with 64 output channels on 16-bit operands (op 1 / 2:
// the BEV stem in C3 / C5), conv_stem.hip: the forward (mode 0, k_conv_stem_lp) stages each
// output tile's input patch once per 16-channel chunk, the data gradient (mode 1, pad 3, 64
// gradient channels, k_conv_stem_dgrad_lp) each tile's gradient patch once.  Tap-major
// weights; e2ep_tune key 35 = 1 + mask (1 forward, 2 data gradient, 4 weight gradient; on fp32
// operands, op 0, also 8 for the gradients and 16 for the forward).  workspace: stem_direct_workspace(g, mode,
// op) bytes for the weight image (k_stem_wprep*).
bool stem_direct_ok(int mode, const ConvGeom &g, int M, int op);
size_t stem_direct_workspace(const ConvGeom &g, int mode, int op);
int stem_direct_launch(int act, int op, const float *w, const float *x, const float *bias, float *y,
                       long long y_bytes, const ConvGeom &g, void *workspace, hipStream_t s);
int stem_dgrad_launch(int op, const float *w, const float *gy, float *dx, long long dx_bytes,
                      const ConvGeom &g, void *workspace, hipStream_t s);
// mode 2: the weight gradient (k_conv_stem_wgrad_lp, op 1 bf16 / op 0 fp32 operands): split
// slabs part[split][64][Cin * 49] for the split reduction; returns the slabs written (-1: refused)
int stem_wgrad_splits(const ConvGeom &g);
int stem_wgrad_launch(const float *gy, const float *x, const ConvGeom &g, int splits, float *part,
                      hipStream_t s, int op);

}  // namespace e2ep
