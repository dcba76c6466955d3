/*
 * e2ep.h — C ABI of libe2ep_hip.so, the MI355X (gfx950) kernels behind the ParkingModel
 * hot path of qintonguav/e2e-parking-carla.
 *
 * Conventions (every entry point):
 *   - all array pointers are DEVICE pointers owned by the caller; nothing is allocated inside;
 *   - work is enqueued on the caller's hipStream_t (passed as void*), so every call can be
 *     captured into a hipGraph; no host synchronisation happens inside;
 *   - the return value is 0 on success, otherwise a hipError_t (>0) or an E2EP_E* code (<0);
 *     e2ep_last_error() returns a thread-local message for the last failure;
 *   - tensors are dense row-major fp32 unless stated; "stride" arguments are in elements.
 *
 * The reference is pure PyTorch (no native code), so each entry point
 * replaces a PyTorch op chain; the citation names the reference code it stands in for.
 */
#ifndef E2EP_H
#define E2EP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define E2EP_EINVAL (-1) /* bad shape / argument */
#define E2EP_ERANGE (-2) /* shape outside what the kernel supports */

int e2ep_abi_version(void);
const char *e2ep_last_error(void);

/* ABI 4 (round 6): e2ep_lss_plan takes workspace_bytes; new entry points
 * e2ep_capture_unjoined, e2ep_tokens_init / e2ep_token_argmax_append, e2ep_dwconv_bf16_ok. */

/* bf16 activation storage (ABI 3; BASELINE C3, the bf16 training mode): the entry points that
 * take an `io` mask read / write the named tensors as bf16 (torch.bfloat16 bits) instead of
 * fp32; their pointers are then void*.  The arithmetic stays fp32: a bf16 element is widened on
 * load, a stored value is rounded to nearest-even, and statistics / gradients of parameters /
 * partial sums stay fp32 / fp64.  io = 0 is the fp32 behaviour of ABI 2.  Each entry point
 * lists the masks it supports (others: E2EP_EINVAL); every bf16 tensor needs H*W % 4 == 0. */
#define E2EP_IO_X_BF16 1  /* the input activation x (a depthwise strip kernel's input plane) */
#define E2EP_IO_DY_BF16 2 /* the incoming gradient dy / gy */
#define E2EP_IO_DX_BF16 4 /* the produced tensor: y of a forward, dx of a backward */

/* ---------------------------------------------------------------------------------------
 * Lift-splat
 * ------------------------------------------------------------------------------------- */

/* Rig algebra (model/bev_model.py:46-53): combine [BN,3,3] = R(E^-1) K^-1, trans [BN,3] = t(E^-1)
 * from K [BN,3,3], E [BN,4,4].  fp64 Gauss-Jordan (partial pivoting), one rounding to fp32:
 * deterministic on every host, whereas the reference's fp32 CPU torch.inverse differs by host
 * ISA in the last ulp (tests/test_lss_gpu.py documents the effect on the pillar index). */
int e2ep_rig_transforms(const float *K, const float *E, int BN, float *combine, float *trans,
                        void *stream);

/* Ego-frame geometry + integer pillar index of every frustum point.
 * Replaces BevModel.get_geometry (model/bev_model.py:45-57) and the voxelisation / mask /
 * rank of proj_bev_feature (model/bev_model.py:85-95).
 *   frustum [D,h,w,3]  (the module's `frustum` parameter; u, v, depth)
 *   combine [B*N,3,3] = R(E^-1) K^-1,  trans [B*N,3] = t(E^-1)   (computed as the reference does)
 *   lo[3] = bev_start_pos - bev_res/2,  res[3] = bev_res  (HOST arrays, read at call time),
 *   X,Y,Z = bev_dim
 *   out pillar [B*N*D*h*w] int32: x*Y*Z + y*Z + z, or -1 where the point is masked.
 * Bit-exact with the reference's fp32 CPU path: sequential non-fused multiply/add, IEEE
 * division, truncation toward zero (Tensor.long()). */
int e2ep_geom_index(const float *frustum, const float *combine, const float *trans,
                    const float *lo, const float *res, int X, int Y, int Z,
                    int B, int N, int D, int h, int w, int32_t *pillar, void *stream);

/* Bytes of int32 workspace e2ep_lss_plan needs: B*X*Y*Z*4. */
size_t e2ep_lss_plan_workspace(int B, int XYZ);

/* Pillars per output tile of e2ep_lss_fwd, and the tile-schedule entries to allocate per
 * sample: 2 * ceil(XYZ / E2EP_LSS_TILE) + 16 (room for the lane schedule's padded lanes). */
#define E2EP_LSS_TILE 64
int e2ep_lss_tiles(int XYZ);

/* Counting sort of kept points by pillar (replaces the mask / argsort / cumsum-boundary
 * bookkeeping of model/bev_model.py:86-99 and tool/geometry.py:292-300).
 *   pillar [B*P] (P = N*D*h*w) from e2ep_geom_index
 *   offsets [B*(XYZ+1)]: points of pillar q of sample b are order[b*P + offsets[b*(XYZ+1)+q] ..
 *                        offsets[b*(XYZ+1)+q+1])
 *   order   [B*P] packed point codes (n<<24 | d<<16 | h*w index), ascending within a pillar,
 *           so every later sum has a fixed, run-to-run identical order.
 *   tiles   [B*e2ep_lss_tiles(XYZ)] or NULL: the forward's launch schedule (any order of the
 *           tiles is correct): B = 8 (or any B not dividing 8): per sample its tiles, heaviest
 *           first, block -> (sample id % B, rank id / B); B = 1, 2, 4: lane schedule — each
 *           sample's tiles cut into G = 8/B contiguous pillar ranges of balanced point counts (each
 *           at most L tiles, else the even cut), range g of sample s = lane g*B + s =
 *           tiles[lane * L .. +L) (L = ceil(1.5 * ceil(tiles / G))), heaviest first, -1
 *           padded, block -> (lane id % 8, entry id / 8): a lane's blocks share an XCD and its L2.
 * Limits: N < 128, D < 256, h*w < 65536; with tiles, ceil(XYZ / E2EP_LSS_TILE) <= 4096. */
int e2ep_lss_plan(const int32_t *pillar, int B, int N, int D, int h, int w, int XYZ,
                  int32_t *offsets, int32_t *order, int32_t *tiles, void *workspace,
                  size_t workspace_bytes, void *stream);

/* Fused depth-distribution x feature outer product + pillar sum-pooling, forward.
 * Replaces encoder_forward's outer product/permute (model/bev_model.py:64-71) and
 * proj_bev_feature's gather / VoxelsSumming / scatter (model/bev_model.py:74-107,
 * tool/geometry.py:289-305).  The (B,N,D,h,w,C) outer product is never materialised.
 *   prob  [B*N, D, h*w]   softmax depth distribution
 *   featT [B*N, h*w, C]   camera features, pixel-major (see e2ep_transpose), 16-B aligned
 *   offsets, order, tiles from e2ep_lss_plan (tiles may be NULL: natural tile order)
 *   bev   out: bev[b*bev_bstride + c*XYZ + q] for c < C, every q written (zeros included).
 * Each pillar is summed in a fixed order: deterministic, run to run. */
int e2ep_lss_fwd(const float *prob, const float *featT, const int32_t *offsets,
                 const int32_t *order, const int32_t *tiles, int B, int N, int D, int hw, int C,
                 int XYZ, float *bev, long long bev_bstride, void *stream);

/* Diagnostics only: when dev_buf != NULL every later e2ep_lss_fwd launch (C % 4 == 0 path)
 * records per block {start, end (s_memrealtime, 100 MHz), XCC/HW id, points} as 4 int64 at
 * dev_buf[4*block]; NULL turns it off (the round-2 per-block trace; the reading script is in
 * git history, commit a6dfde2). */
int e2ep_debug_fwd_trace(void *dev_buf);

/* Backward of e2ep_lss_fwd (replaces VoxelsSumming.backward, tool/geometry.py:307-317, and
 * the autograd of the outer product).  Gather formulation, no atomics, deterministic:
 *   grad_prob[p] = sum_c gT[q(p), c] * feat[pix(p), c]
 *   grad_feat[pix, c] = sum_d gT[q(pix,d), c] * prob[pix, d]
 *   gT    [B, XYZ, C]   grad of bev, pillar-major (see e2ep_transpose)
 *   featT [B*N, h*w, C]
 *   pillar [B*N*D*h*w] from e2ep_geom_index
 *   out grad_prob [B*N, D, h*w], grad_feat [B*N, C, h*w]
 * Limits: C <= 64, D <= 64. */
int e2ep_lss_bwd(const float *gT, const float *prob, const float *featT, const int32_t *pillar,
                 int B, int N, int D, int hw, int C, int XYZ, float *grad_prob,
                 float *grad_feat, void *stream);

/* Batched 2-D transpose: out[b][c][r] = in[b*in_bstride + r*cols + c], r < rows, c < cols;
 * out batch stride rows*cols.  Used to produce featT / gT above. */
int e2ep_transpose(const float *in, long long in_bstride, int batch, int rows, int cols,
                   float *out, void *stream);
/* Many transposes in one launch: `table` (device, n <= 256 entries of 6 int64) holds per
 * entry {src, dst, rows, cols, first tile, ceil(cols / 64)}, tiles counted in 64 x 64 blocks
 * in entry order; dst = src^T (rows x cols -> cols x rows).  Replaces the per-conv weight
 * transposes of one forward (every R x S > 1 conv weight [Cout,Cin,R,S] -> [R*S,Cout,Cin],
 * the kernels' w_layout 1; reference convs: model/cam_encoder.py, model/bev_encoder.py,
 * model/convolutions.py, model/segmentation_head.py) with a single launch. */
int e2ep_transpose_multi(const long long *table, int n, int tiles, void *stream);

/* Target-point channel (replaces ParkingModel.add_target_bev, model/parking_model.py:28-46).
 *   target_point [B,3] (x m, y m, yaw);  noise [B,2] uniform [0,1) (the rand_like draw)
 *   px = int(X/2 + x/res_x) + int(noise0*10-5), py likewise; out plane [X,Y] of sample b at
 *   out + b*out_bstride is zeroed and the 8x8 square [px-4,px+4) x [py-4,py+4) set to 1 with
 *   Python slice semantics (negative bounds wrap, then clamp). */
int e2ep_target_bev(const float *target_point, const float *noise, int B, int X, int Y,
                    float res_x, float res_y, float *out, long long out_bstride, void *stream);

/* ---------------------------------------------------------------------------------------
 * Convolution, NCHW fp32, implicit GEMM on the exact-f32 matrix cores (K order: filter tap
 * outer, 16-channel chunks inner; no im2col buffer, no lookup table) (SURVEY.md §8a rows
 * a8 (1x1/stem), a9, a11, a13).  Replaces torch.nn.Conv2d forward/backward in
 * model/bev_encoder.py:13-34, model/segmentation_head.py:19-31,
 * model/convolutions.py:183-282 and the efficientnet-pytorch 1x1 / stem convs.
 *
 * dims[15] = {N, Cin, H, W, Cout, R, S, P, Q, stride_h, stride_w, pad_top, pad_left,
 *             dil_h, dil_w}; P, Q are the output size (so asymmetric "SAME" padding is just
 * a bigger P/Q with implicit zero rows/cols at the bottom/right).  groups == 1.
 * ------------------------------------------------------------------------------------- */

/* y[N,Cout,P,Q] = conv(x[N,Cin,H,W], w) + bias (nullable); act 0 none, 1 relu.
 * w_layout 0: w[Cout,Cin,R,S] (PyTorch); 1: tap-major w[R*S,Cout,Cin] (see e2ep_transpose),
 * whose rows are contiguous along Cin for both the forward and the data gradient (16-B
 * weight loads); the two coincide for 1x1 filters.
 * Grids that cannot fill the chip split K; the partial sums then need a workspace of
 * e2ep_conv_fwd_workspace bytes (0 = none needed; pass NULL) and are reduced in fixed order. */
size_t e2ep_conv_fwd_workspace(const int *dims);
/* io: 0, or E2EP_IO_X_BF16 (x bf16: C3's bf16-stored squeeze-excitation output as the MBConv
 * project conv's input; the bf16-operand kernels only, precision 1). */
int e2ep_conv_fwd(const void *x, const float *w, const float *bias, const int *dims, int act,
                  int w_layout, float *y, void *workspace, size_t workspace_bytes, void *stream,
                  int io);
/* e2ep_conv_fwd plus the batch statistics of y for the BatchNorm that follows the conv
 * (MBConv _expand_conv -> _bn0, _project_conv -> _bn2; reference model/cam_encoder.py:69-82
 * via efficientnet-pytorch): the epilogue writes, per output channel c and column tile t
 * (tiles over the N*P*Q output pixels), the fp64 sum and sum of squares of the stored values
 * into stats[(t * Cout + c) * 2 + {0, 1}] — the partials e2ep_bn_finalize_part reduces, so
 * the BN layer never re-reads y for its statistics.  tiles = e2ep_conv_fwd_stats_tiles(dims,
 * w_layout), which is 0 when the geometry's kernel takes no statistics (then stats must be
 * NULL and the BN computes its own); stats_bytes >= Cout * tiles * 16.  Deterministic. */
int e2ep_conv_fwd_stats_tiles(const int *dims, int w_layout);
int e2ep_conv_fwd_stats(const void *x, const float *w, const float *bias, const int *dims, int act,
                        int w_layout, float *y, void *workspace, size_t workspace_bytes,
                        double *stats, size_t stats_bytes, void *stream, int io /* as e2ep_conv_fwd */);

/* dx[N,m_channels,H,W] = conv_transpose(gout[N,Cout,P,Q], w) restricted to the first
 * m_channels input channels; split by input-pixel stride phase, so no zero taps at stride 2.
 * w_layout as for e2ep_conv_fwd. */
size_t e2ep_conv_dgrad_workspace(const int *dims, int m_channels);
int e2ep_conv_dgrad(const float *gout, const float *w, const int *dims, int m_channels,
                    int w_layout, float *dx, void *workspace, size_t workspace_bytes, void *stream);
/* e2ep_conv_dgrad plus a residual gradient res (dx's layout, may be NULL) added in the
 * epilogue: dx = conv_transpose(gout, w) + res.  The skip connection around a block whose
 * first conv reads the block input (MBConv expand conv, ResNet BasicBlock conv1) gets its
 * input gradient in one pass instead of dgrad + an autograd accumulation add. */
/* io: 0, or E2EP_IO_DX_BF16 (dx written bf16 — the gradient at a bf16-stored input; the
 * bf16-operand kernels with the in-launch split-K fold; res stays fp32). */
int e2ep_conv_dgrad_acc(const float *gout, const float *w, const int *dims, int m_channels,
                        int w_layout, const float *res, void *dx, void *workspace,
                        size_t workspace_bytes, void *stream, int io);

/* A conv layer's backward in one launch: dx (e2ep_conv_dgrad_acc with res, w tap-major) and
 * dw (e2ep_conv_wgrad with `wsplits`, accumulate 0), their blocks sharing one grid instead of
 * two launches on forked streams (a fork / join of a replayed HIP graph idles the GPU
 * ~15 us; the small-map layers' gradients take 20 - 50 us each), then the weight gradient's
 * fixed-order split reduction.  Kernels: k_conv_bwd_pair (fp32 k_conv_gemm data gradient +
 * k_conv_wgrad2), k_conv_bwd_pair1x1 (+ the large-map k_wgrad_1x1), k_lp_bwd_pair (k_conv_lp
 * data gradient, fp32 or C3 bf16, + k_wgrad_lp).  Where e2ep_conv_bwd_pair_ok is 0 (fp16,
 * the large-map k_conv_gemm2 kernels, tiles without a paired instantiation) the caller
 * launches the two separately.  Workspaces: e2ep_conv_dgrad_workspace(dims, m_channels),
 * e2ep_conv_wgrad_workspace(dims, wsplits).  Results bitwise those of the two launches. */
int e2ep_conv_bwd_pair_ok(const int *dims, int m_channels);
int e2ep_conv_bwd(const float *gout, const void *x, const float *w, const int *dims,
                  int m_channels, const float *res, void *dx, void *ws_dgrad,
                  size_t ws_dgrad_bytes, int wsplits, void *ws_wgrad, size_t ws_wgrad_bytes,
                  float *dw, void *stream,
                  int io /* 0, or X|DX bf16 on the C3 k_lp_bwd_pair without res */);

/* dw[Cout,Cin,R,S] (=, or += when accumulate) = sum over pixels of gout x im2col(x).
 * The pixel reduction is split over `splits` workgroups; partial slabs (workspace of
 * e2ep_conv_wgrad_workspace bytes) are summed in a fixed order: deterministic. */
/* Forward / data-gradient GEMM selection (tests, benchmarks): 0 = automatic (default),
 * 1 = always the first-generation kernel, 2 = the second-generation kernel (k-contiguous LDS
 * fragments, no padded channel steps) wherever its limits allow, 3 = the same with 128-column
 * tiles only, 4 = automatic but the 1x1 forward / data gradient on the column-batched GEMM of
 * e2ep_gemm, 5 = the same for maps of at most 1024 pixels only.  Returns the previous value;
 * a value outside 0..5 only queries.  Process-global; not thread-safe against concurrent
 * launches. */
int e2ep_conv_gemm_variant(int variant);
/* Split-K plans: forward / data-gradient conv GEMM grids under `thresh` workgroups are split
 * toward `target` (defaults 1024 / 512; thresh 0 = never split); the spatial weight gradient
 * (e2ep_conv_wgrad_splits) aims at `wgrad_target` workgroups (default 1024).  Values <= 0
 * (thresh < 0) keep the current setting.  For A/B timing. */
int e2ep_conv_split_params(int target, int thresh, int wgrad_target);
/* Operand precision of the conv GEMMs: 0 = fp32 (default; exact-f32 MFMA), 1 = bf16, 2 = fp16
 * (operands rounded to nearest-even, fp32 products and accumulation, fp32 tensors in and
 * out) — BASELINE configs C3 (bf16 forward / fp32 gradients, AMP-style: bf16 operands in the
 * forward, data-gradient and weight-gradient GEMMs, gradients accumulated and stored fp32;
 * every other op, the optimizer and the all-reduce stay fp32) and C5 (fp16 inference: forward
 * and data-gradient GEMMs only).  Both GEMM generations take the setting; the direct tiny-K
 * stem conv and 1x1 convs on 1x1 maps (squeeze-excitation) stay fp32.
 * Returns the previous value; out-of-range values only query.  Process-global. */
int e2ep_conv_precision(int precision);
/* Pixels per K-step of the tiled weight-gradient kernel (benchmarking): 16 (default) or 32;
 * returns the previous value, other values only query.  Process-global. */
int e2ep_conv_wgrad_kstep(int pixels);
int e2ep_conv_wgrad_splits(const int *dims);
size_t e2ep_conv_wgrad_workspace(const int *dims, int splits);
int e2ep_conv_wgrad(const float *gout, const void *x, const int *dims, int splits,
                    void *workspace, size_t workspace_bytes, float *dw, int accumulate,
                    void *stream, int io /* 0, or E2EP_IO_X_BF16 on k_wgrad_lp (C3) */);

/* db[C] = sum over (n, p) of gout[N, C, HW]. */
int e2ep_bias_grad(const float *gout, int N, int C, int HW, float *db, void *stream);

/* out[C] = column sums of the row-major g[rows][C] (nn.Linear bias gradient), deterministic
 * two-stage reduction; workspace e2ep_col_sum_workspace bytes. */
size_t e2ep_col_sum_workspace(int rows, int C);
int e2ep_col_sum(const float *g, int rows, int C, float *out, void *workspace, void *stream);

/* Skinny GEMM for tiny outputs: C[i*Nj + j] = sum_k A[i*ai + k*ak] * B[k*bk + j*bj]
 * (+ bias[j]); one wave per output.  1x1 convs on 1x1 maps (squeeze-excitation) and small
 * linears, forward and backward, via strides. */
int e2ep_skinny_gemm(const float *A, int ai, int ak, const float *B, int bk, int bj,
                     const float *bias, int Mi, int Nj, int K, float *C, void *stream);

/* ---------------------------------------------------------------------------------------
 * BatchNorm2d + activation (+ residual), NCHW fp32.
 * Replaces BatchNorm2d(+ReLU / swish, + identity add) pairs of the reference model tree, and
 * efficientnet-pytorch's drop_connect + skip add of MBConv (reference model/cam_encoder.py:70-72).
 *   y = act(dc(gamma * (x - mean) * invstd + beta) + res)
 * act: 0 none, 1 relu, 2 swish (x * sigmoid(x)); res (nullable) is added before act;
 * dc(z) = z / dc_keep * floor(dc_keep + dc_rand[n]) when dc_rand [N] (uniform draws) is given,
 * else z.  train != 0: batch statistics (fp64 accumulation, fixed order), running stats
 * updated in place with `momentum` (unbiased variance); train == 0: running statistics.
 * mean / invstd [C] are outputs of fwd and inputs of bwd.  workspace: e2ep_bn_workspace.
 * Two launches each way (statistics / reduction, then the elementwise pass, which also
 * finishes the per-channel statistics): no separate finalize launch.
 * ------------------------------------------------------------------------------------- */
size_t e2ep_bn_workspace(int N, int C, int H, int W);
int e2ep_bn_fwd(const float *x, const float *gamma, const float *beta, const float *res,
                const float *dc_rand, float dc_keep, float *running_mean, float *running_var,
                int N, int C, int H, int W, int train, float momentum, float eps, int act,
                float *mean, float *invstd, float *y, void *workspace, size_t workspace_bytes,
                void *stream);
/* Statistics half of e2ep_bn_fwd (same fp64 reduction, same running-stat update) for a
 * consumer that applies the normalisation on load (e2ep_dwconv_fwd / _wgrad in_scale,
 * in_shift): writes mean / invstd [C] and the folded affine scale = gamma * invstd,
 * shift = beta - mean * scale [C].  The backward is e2ep_bn_bwd on the same x. */
int e2ep_bn_stats(const void *x, const float *gamma, const float *beta, float *running_mean,
                  float *running_var, int N, int C, int H, int W, int train, float momentum,
                  float eps, float *mean, float *invstd, float *scale, float *shift,
                  void *workspace, size_t workspace_bytes, void *stream,
                  int io /* 0 or E2EP_IO_X_BF16 */);
/* 1 when the training forward of this shape takes the split path (a statistics pass over x,
 * then the elementwise pass), 0 when it runs the single-launch kernel that keeps each channel
 * in registers — where a producer's partial sums (e2ep_conv_fwd_stats) save nothing. */
int e2ep_bn_fwd_split(int N, int C, int H, int W);
/* Training statistics from a producer's partial sums (e2ep_conv_fwd_stats /
 * e2ep_dwconv_fwd_stats): part[tiles][C][2] fp64 (sum, sum of squares) over the N*H*W elements
 * of each channel, reduced in fixed order; writes mean / invstd / scale / shift [C] and updates
 * the running stats as e2ep_bn_stats does.  One launch of C/8 workgroups reading whole
 * 128-B lines (8 channels of one tile); e2ep_bn_finalize_part_workspace returns 0 today (the
 * workspace arguments are kept for a split plan). */
size_t e2ep_bn_finalize_part_workspace(int C, int tiles);
int e2ep_bn_finalize_part(const double *part, int tiles, const float *gamma, const float *beta,
                          float *running_mean, float *running_var, int N, int C, int H, int W,
                          float momentum, float eps, float *mean, float *invstd, float *scale,
                          float *shift, void *workspace, size_t workspace_bytes, void *stream);
/* Elementwise half of e2ep_bn_fwd with the affine already folded: y = act(dc(x * scale[c] +
 * shift[c]) + res) (scale / shift from e2ep_bn_finalize_part or e2ep_bn_stats; res, dc_rand,
 * dc_keep, act as in e2ep_bn_fwd) — the same arithmetic as e2ep_bn_fwd's apply pass. */
int e2ep_bn_apply(const float *x, const float *scale, const float *shift, const float *res,
                  const float *dc_rand, float dc_keep, int N, int C, int H, int W, int act,
                  float *y, void *stream);
/* dx, dgamma, dbeta, dres (each nullable) from x, dy and the forward's mean/invstd; res and
 * dc_rand / dc_keep as in the forward (dres = gradient at the activation input).
 * gate_logit / gate_dpooled [N,C] (both or neither): the activation output fed a
 * squeeze-excitation gate (e2ep_se_fwd with x_scale / x_shift), so the gradient at it is
 * dy * sigmoid(gate_logit) + gate_dpooled / (H*W), formed on the fly from the gate's dy. */
int e2ep_bn_bwd(const void *x, const void *dy, const float *mean, const float *invstd,
                const float *gamma, const float *beta, const float *res, const float *dc_rand,
                float dc_keep, const float *gate_logit, const float *gate_dpooled, int N, int C,
                int H, int W, int train, int act, void *dx, float *dgamma, float *dbeta,
                float *dres, void *workspace, size_t workspace_bytes, void *stream,
                int io /* 0, X|DX or X|DY|DX (the depthwise output's _bn1) or DY (_bn0) */);
/* 1 when e2ep_bn_bwd runs this shape as the split reduce + apply pair (a channel of more
 * than 8192 elements, or the single-launch kernels switched off), 0 for the single launch. */
int e2ep_bn_bwd_split(int N, int C, int H, int W);
/* The apply half of e2ep_bn_bwd (training statistics, squeeze-excitation gate) whose channel
 * sums come from e2ep_se_bwd_bn's per-plane factors instead of a reduction pass over x and dy:
 * sum dzb = sum_n sigmoid(logit) A1 + dpooled / HW A2, sum dzb xhat = ... A3 / A4 (fp64).
 * Same arguments and element arithmetic as e2ep_bn_bwd; no workspace. */
int e2ep_bn_bwd_planes(const void *x, const void *dy, const float *mean, const float *invstd,
                       const float *gamma, const float *beta, const float *gate_logit,
                       const float *gate_dpooled, const double *plane_sums, int N, int C, int H,
                       int W, int act, void *dx, float *dgamma, float *dbeta, void *stream,
                       int io /* 0, X|DX or X|DY|DX */);
/* Eval-mode statistics of n BatchNorm layers in one launch (the per-layer e2ep_bn_stats calls
 * of an inference forward, 42 launches of C5 predict): table = DEVICE array of n rows of 7
 * int64 {running_mean, running_var, gamma (nullable), beta (nullable), out, C, eps as fp32
 * bits}; out [4][C] = mean, invstd, scale, shift, the same arithmetic as e2ep_bn_stats with
 * train = 0. */
int e2ep_bn_eval_multi(const long long *table, int n, void *stream);
/* Stand-alone activation (act as above) and its gradient w.r.t. the pre-activation x. */
int e2ep_act_fwd(const float *x, long long n, int act, float *y, void *stream);
int e2ep_act_bwd(const float *x, const float *dy, long long n, int act, float *dx, void *stream);

/* ---------------------------------------------------------------------------------------
 * Layout and bookkeeping (csrc/small.hip)
 * ------------------------------------------------------------------------------------- */
/* torch.cat(pieces, dim=1) of n <= 8 NCHW fp32 tensors [N][chans[j]][HW] into dst
 * [N][sum chans][HW] (ASPP branches, reference model/convolutions.py:262-263; UpsamplingConcat,
 * model/convolutions.py:281-282), and its backward: the split of dst-shaped `src` into n
 * contiguous pieces (torch's CatBackward slices + .contiguous() copies).  srcs / dsts / chans
 * are HOST arrays of device pointers / channel counts; HW % 4 == 0, pointers 16-B aligned. */
int e2ep_cat_channels(const float *const *srcs, const int *chans, int n, int N, long long HW,
                      float *dst, void *stream);
int e2ep_split_channels(const float *src, const int *chans, int n, int N, long long HW,
                        float *const *dsts, void *stream);
/* out[i] = a[i] + b[i], i < n (fp32): the gradient of an activation read by two consumers
 * (nn_ops.fork2), in place of autograd's accumulation. */
int e2ep_add_f32(const float *a, const float *b, long long n, float *out, void *stream);
/* out[0] = (a[0] + b[0]) + c[0] in fp32: the training loss (trainer/pl_trainer.py:57-59,
 * control + segmentation + depth) as one launch. */
int e2ep_sum3(const float *a, const float *b, const float *c, float *out, void *stream);
/* mask[b*T + t] = tok[b*rstride + t] == value (1 / 0): the decoder's PAD-key mask
 * (model/control_predict.py create_mask, tgt == pad_idx) on int64 tokens. */
int e2ep_eq_mask_i64(const int64_t *tok, long long rstride, int B, int T, int64_t value,
                     uint8_t *mask, void *stream);
/* One launch of the step's random draws: f[0..nf) uniform on [0, 1) (24-bit), iv[0..ni) uniform
 * on [0, 2^31), value i a splitmix64 hash of (state[0] = seed, state[1] = draw counter, i);
 * the kernel then advances state[1], so every launch or graph replay draws fresh values.
 * Replaces torch.rand / torch.randint draws of a training forward (the drop-connect uniforms
 * of efficientnet-pytorch's MBConv, the target noise of model/parking_model.py:36, the dropout
 * seed pool of e2ep_amd/rng.py).  nf + ni <= any; one workgroup. */
int e2ep_rng_draw(long long *state, int nf, float *f, int ni, int *iv, void *stream);
/* *(int64 *)table[i] += v for i < n (device table of device addresses): every BatchNorm's
 * num_batches_tracked increment of a forward (torch.nn.BatchNorm2d) in one launch. */
int e2ep_add_i64_multi(const long long *table, int n, long long v, void *stream);

/* ---------------------------------------------------------------------------------------
 * Squeeze-and-excitation of an MBConv block as one op (efficientnet-pytorch 0.7.1
 * MBConvBlock._se_reduce / _swish / _se_expand / sigmoid gate, reference
 * model/cam_encoder.py:69-73).  x, y [N,C,HW]; w1 [sq,C] b1 [sq] (_se_reduce), w2 [C,sq]
 * b2 [C] (_se_expand), biases nullable:
 *   pooled = mean_hw x; hpre = w1 pooled + b1; a = w2 swish(hpre) + b2; y = x * sigmoid(a)
 * pooled [N,C], hpre [N,sq], a [N,C] are forward outputs the backward reads.
 * Backward: dx = dy*sigmoid(a) + (w1^T (swish'(hpre) * (w2^T da))) / HW with
 * da = sigmoid'(a) * sum_hw dy*x, and the four parameter gradients (each nullable), batch sums
 * in sample order.  workspace: (2*N*C + 17*N*sq) floats.  Limits: C <= 4096, sq <= 256.
 * x_scale / x_shift [C] (both or neither): the SE input is swish(x * x_scale + x_shift),
 * i.e. the block's _bn1 + swish applied on load to the raw depthwise output x (e2ep_bn_stats);
 * then the backward leaves dx to e2ep_bn_bwd (pass dx = NULL, dpooled_out [N,C], and hand a
 * and dpooled_out to e2ep_bn_bwd as gate_logit / gate_dpooled).
 * ------------------------------------------------------------------------------------- */
int e2ep_se_fwd(const void *x, const float *x_scale, const float *x_shift, const float *w1,
                const float *b1, const float *w2, const float *b2, int N, int C, int HW, int sq,
                float *pooled, float *hpre, float *a, void *y, void *stream,
                int io /* 0, E2EP_IO_X_BF16 or X|DX (y bf16 too) */);
int e2ep_se_bwd(const void *x, const float *x_scale, const float *x_shift, const void *dy,
                const float *w1, const float *w2, const float *pooled, const float *hpre,
                const float *a, int N, int C, int HW, int sq, float *dx, float *dpooled_out,
                float *dw1, float *db1, float *dw2, float *db2, float *workspace, void *stream,
                int io /* 0, X or X|DY bf16 (dx = NULL: formed by the BN backward) */);
/* e2ep_se_bwd (x_scale / x_shift transform, dx left to the BN) that also takes the block's
 * _bn1 backward sums in its da pass over x and dy (MBConv _bn1 -> swish -> SE, reference
 * model/cam_encoder.py:69-73): with xhat = (x - bn_mean) bn_invstd and sp = swish'(xhat gamma +
 * beta), plane_sums [N*C][4] (fp64) = (sum dy sp, sum sp, sum dy sp xhat, sum sp xhat) per
 * (n, c) plane, for e2ep_bn_bwd_planes (which then skips e2ep_bn_bwd's reduction pass).
 * gamma / beta nullable (1 / 0). */
int e2ep_se_bwd_bn(const void *x, const float *x_scale, const float *x_shift,
                   const float *bn_mean, const float *bn_invstd, const float *gamma,
                   const float *beta, const void *dy, const float *w1, const float *w2,
                   const float *pooled, const float *hpre, const float *a, int N, int C, int HW,
                   int sq, float *dpooled_out, float *dw1, float *db1, float *dw2, float *db2,
                   double *plane_sums, float *workspace, void *stream,
                   int io /* 0, X or X|DY bf16 */);

/* ---------------------------------------------------------------------------------------
 * Residual add + dropout + LayerNorm of the post-norm transformer layers (torch
 * TransformerEncoderLayer / TransformerDecoderLayer norm1..3 with dropout1..3; reference
 * model/feature_fusion.py:13-14, model/control_predict.py:19-20), rows x E, E <= 512:
 *   x = a + drop(b),  drop(b) = b * [u >= p] / (1 - p)  (u nullable: no dropout; b nullable)
 *   y = (x - mean) * rstd * gamma + beta,  rstd = 1 / sqrt(biased var + eps)
 * x (nullable), mean, rstd [rows] are saved for the backward, which returns da = dL/dx,
 * db = da * [u >= p] / (1 - p) and gamma / beta gradients (fixed-order column sums;
 * workspace e2ep_add_drop_ln_bwd_workspace bytes).  The _seeded variants draw the mask from
 * the counter hash shared with the attention / feed-forward dropout (keep element
 * row * E + c iff hash(seed, row * E + c) >= p), keyed by the device int32 *seed: no uniform
 * tensor is read.
 * ------------------------------------------------------------------------------------- */
int e2ep_add_drop_ln_fwd_seeded(const float *a, const float *b, const int *seed, float p,
                                const float *gamma, const float *beta, int rows, int E, float eps,
                                float *x, float *y, float *mean, float *rstd, void *stream);
int e2ep_add_drop_ln_bwd_seeded(const float *dy, const float *x, const float *mean,
                                const float *rstd, const float *gamma, const int *seed, float p,
                                int rows, int E, float *da, float *db, float *dgamma,
                                float *dbeta, void *workspace, void *stream);
int e2ep_add_drop_ln_fwd(const float *a, const float *b, const float *u, float p,
                         const float *gamma, const float *beta, int rows, int E, float eps,
                         float *x, float *y, float *mean, float *rstd, void *stream);
size_t e2ep_add_drop_ln_bwd_workspace(int rows, int E);
int e2ep_add_drop_ln_bwd(const float *dy, const float *x, const float *mean, const float *rstd,
                         const float *gamma, const float *u, float p, int rows, int E,
                         float *da, float *db, float *dgamma, float *dbeta, void *workspace,
                         void *stream);

/* ---------------------------------------------------------------------------------------
 * Fused multi-head attention core, fp32: O = dropout_p(softmax(scale Q K^T + mask)) V per
 * (batch, head), replacing the bmm / mask / softmax / dropout / bmm chain inside
 * torch.nn.MultiheadAttention as the reference's transformer layers run it
 * (model/feature_fusion.py:13-14,48-50; model/control_predict.py:19-20,39-47).
 * Q, K, V, O are (S, B, E)-strided: row (s, b) of head h starts at
 * base + s*ss + b*sb + h*dh (so Q/K/V are read in place from the in-projection output).
 * Sq, Sk <= 256, dh <= 64.  causal masks key j > query i; key_pad (bool [B][Sk], may be NULL)
 * masks keys; a fully masked row yields O = 0.  Dropout keep(bh, i, j) is a hash of *seed
 * and the counter (bh*Sq + i)*Sk + j (seed: device int32, may be NULL when p == 0).
 * lse: [B*H][Sq] row log-sum-exp (log2 domain, internal) for the backward.
 * Backward writes dq (Q's layout) and dk, dv (K/V's layout); workspace
 * e2ep_attn_bwd_workspace bytes.  e2ep_attn_keep_mask materialises the keep mask
 * ([BH][Sq][Sk] bytes) for tests.
 * ------------------------------------------------------------------------------------- */
int e2ep_attn_fwd(const float *q, const float *k, const float *v, int B, int H, int Sq, int Sk,
                  int dh, int q_ss, int q_sb, int kv_ss, int kv_sb, int o_ss, int o_sb,
                  float scale, int causal, const uint8_t *key_pad, float p, const int32_t *seed,
                  float *o, float *lse, void *stream);
size_t e2ep_attn_bwd_workspace(int B, int H, int Sq);
int e2ep_attn_bwd(const float *q, const float *k, const float *v, const float *o, const float *dout,
                  const float *lse, int B, int H, int Sq, int Sk, int dh, int q_ss, int q_sb,
                  int kv_ss, int kv_sb, int o_ss, int o_sb, float scale, int causal,
                  const uint8_t *key_pad, float p, const int32_t *seed, float *dq, float *dk,
                  float *dv, void *workspace, void *stream);
/* The same backward in parts (part 0 = all of it, as e2ep_attn_bwd): 1 writes D = rowsum(dO * O)
 * into the workspace; after it, 2 (dq) and 3 (dk, dv) are independent and may run concurrently
 * on two streams (e2ep_amd.attention forks them). */
int e2ep_attn_bwd_part(const float *q, const float *k, const float *v, const float *o,
                       const float *dout, const float *lse, int B, int H, int Sq, int Sk, int dh,
                       int q_ss, int q_sb, int kv_ss, int kv_sb, int o_ss, int o_sb, float scale,
                       int causal, const uint8_t *key_pad, float p, const int32_t *seed, float *dq,
                       float *dk, float *dv, void *workspace, int part, void *stream);
int e2ep_attn_keep_mask(const int32_t *seed, int BH, int Sq, int Sk, float p, uint8_t *out,
                        void *stream);
/* Softmax over the channel dim of x [N, C, HW] (model/bev_model.py:64 depth.softmax(1)) and
 * its backward dx = y (dy - sum_c y dy).  C <= 64. */
int e2ep_softmax_c_fwd(const float *x, int N, int C, int HW, float *y, void *stream);
int e2ep_softmax_c_bwd(const float *y, const float *dy, int N, int C, int HW, float *dx,
                       void *stream);
/* Transformer feed-forward activation y = dropout_p(relu(x)) over n floats (n % 4 == 0,
 * 16-B aligned), and dx = dy * relu'(x) * keep / (1-p).  Keep bit of element c = the
 * attention hash of (*seed, c) (e2ep_attn_keep_mask with BH = Sq = 1, Sk = n shows it). */
int e2ep_relu_dropout_fwd(const float *x, long long n, float p, const int32_t *seed, float *y,
                          void *stream);
int e2ep_relu_dropout_bwd(const float *x, const float *dy, long long n, float p,
                          const int32_t *seed, float *dx, void *stream);

/* ---------------------------------------------------------------------------------------
 * Bilinear resize, align_corners=False (F.interpolate / nn.Upsample semantics) over
 * `planes` = N*C planes.  scale_* = 1/scale_factor when a factor is given, else In/Out.
 * Replaces model/bev_encoder.py:24, model/segmentation_head.py:35-38,
 * model/convolutions.py:197,238-240.  Backward is a deterministic two-pass gather.
 * ------------------------------------------------------------------------------------- */
/* forward over N*C planes; plane (n, c) reads x + n*x_nstride + c*Hi*Wi and writes
 * y + n*y_nstride + c*Ho*Wo, so channel slices of larger tensors are read/written in place. */
int e2ep_resize_fwd(const float *x, int N, int C, long long x_nstride, int Hi, int Wi, int Ho,
                    int Wo, float scale_h, float scale_w, float *y, long long y_nstride,
                    void *stream);
size_t e2ep_resize_bwd_workspace(int planes, int Ho, int Wi);
int e2ep_resize_bwd(const float *g, long long g_pstride, int planes, int Hi, int Wi, int Ho,
                    int Wo, float scale_h, float scale_w, float *gx, int accumulate,
                    void *workspace, void *stream);
/* Backward for scale_h, scale_w >= 0.5 (up to 2x upsampling) written channels-last:
 * gxT[n][i * Wi + j][c] from the NCHW gradient g (plane (n, c) at g + (n*C + c)*g_pstride).
 * The BEV encoder stem's 200 -> 256 resize (model/bev_encoder.py:24) hands the lift-splat
 * backward (tool/geometry.py:307-317, e2ep_lss_bwd) its pillar-major BEV gradient directly. */
int e2ep_resize_bwd_cl(const float *g, long long g_pstride, int N, int C, int Hi, int Wi, int Ho,
                       int Wo, float scale_h, float scale_w, float *gxT, void *stream);

/* ---------------------------------------------------------------------------------------
 * Depthwise conv (EfficientNet MBConv _depthwise_conv; k 3 or 5, stride 1 or 2, static
 * SAME padding).  dims[10] = {N, C, H, W, K, P, Q, stride, pad_top, pad_left}.
 * ------------------------------------------------------------------------------------- */
/* in_scale / in_shift [C] (both or neither) and in_act (0 none, 1 relu, 2 swish): the conv
 * input is act(x * in_scale + in_shift), i.e. the preceding BatchNorm + activation applied on
 * load (e2ep_bn_stats); the zero padding is in the transformed space.  dgrad returns the
 * gradient w.r.t. the transformed input (feed it to e2ep_bn_bwd with the same act). */
int e2ep_dwconv_fwd(const float *x, const float *w, const int *dims, const float *in_scale,
                    const float *in_shift, int in_act, float *y, void *stream);
/* e2ep_dwconv_fwd plus the batch statistics of y for the BatchNorm that follows (MBConv
 * _depthwise_conv -> _bn1): per channel c and tile t (t = n * units + the output-row block
 * of one wave), the fp64 sum and sum of squares of y into stats[(t * C + c) * 2 + {0, 1}]
 * (e2ep_bn_finalize_part's input).  tiles = e2ep_dwconv_fwd_stats_tiles(dims), 0 when the
 * geometry runs the generic kernel (then stats must be NULL); stats_bytes >= C * tiles * 16. */
int e2ep_dwconv_fwd_stats_tiles(const int *dims);
/* io: 0, or E2EP_IO_DX_BF16 (y stored bf16 — C3's depthwise output; x stays fp32; the statistics
 * are those of the stored bf16 values).  The bf16 forms run on the strip kernels only. */
int e2ep_dwconv_fwd_stats(const float *x, const float *w, const int *dims, const float *in_scale,
                          const float *in_shift, int in_act, void *y, double *stats,
                          size_t stats_bytes, void *stream, int io);
/* io: 0, or E2EP_IO_DY_BF16 | E2EP_IO_DX_BF16 (gy and dx bf16) */
int e2ep_dwconv_dgrad(const void *gy, const float *w, const int *dims, void *dx, void *stream,
                      int io);
/* A stride-1 depthwise layer's backward in one launch (k_dw_bwd_pair): dx as
 * e2ep_dwconv_dgrad, dw as e2ep_dwconv_wgrad (in_scale / in_shift / in_act: the input
 * transform of the weight gradient's x, as there), their blocks sharing one grid instead of
 * two launches on forked streams.  Where e2ep_dwconv_bwd_pair_ok is 0 the caller launches the
 * two separately.  Workspace: e2ep_dwconv_wgrad_workspace.  Results bitwise those of the two
 * separate launches. */
int e2ep_dwconv_bwd_pair_ok(const int *dims);
/* 1 when every kernel on either side of this depthwise conv takes the bf16 storage masks
 * (E2EP_IO_*): the forward strip kernel (y bf16), the data gradient (strip or stride-2 strip
 * kernel, gy / dx bf16), the weight-gradient strip kernel (gy bf16) and the BatchNorms on
 * its input and output planes (H*W and P*Q multiples of 4); else 0 — the caller keeps fp32
 * storage for that layer instead of failing partway through a step. */
int e2ep_dwconv_bf16_ok(const int *dims);
int e2ep_dwconv_bwd(const void *gy, const float *x, const float *w, const int *dims,
                    const float *in_scale, const float *in_shift, int in_act, void *dx,
                    void *workspace, size_t workspace_bytes, float *dw, void *stream,
                    int io /* 0 or E2EP_IO_DY_BF16 | E2EP_IO_DX_BF16 (x stays fp32) */);
size_t e2ep_dwconv_wgrad_workspace(const int *dims);
int e2ep_dwconv_wgrad(const void *gy, const float *x, const int *dims, const float *in_scale,
                      const float *in_shift, int in_act, void *workspace, size_t workspace_bytes,
                      float *dw, void *stream, int io /* 0 or E2EP_IO_DY_BF16 */);

/* ---------------------------------------------------------------------------------------
 * Pooling and squeeze-excitation gating.
 * max-pool 3x3 / stride 2 / pad 1 (ResNet stem, model/bev_encoder.py:17,30) stores the
 * winning tap index (int8) for its gather backward; global average pool per plane (ASPP
 * pooling, SE squeeze); SE gate y = x * sigmoid(a[plane]).
 * ------------------------------------------------------------------------------------- */
int e2ep_maxpool3s2_fwd(const float *x, int planes, int H, int W, float *y, int8_t *arg,
                        void *stream);
int e2ep_maxpool3s2_bwd(const float *gy, const int8_t *arg, int planes, int H, int W, float *dx,
                        void *stream);
int e2ep_avgpool_fwd(const float *x, int planes, int HW, float *y, void *stream);
int e2ep_avgpool_bwd(const float *gy, int planes, int HW, float *dx, void *stream);
int e2ep_se_gate_fwd(const float *x, const float *a, int planes, int HW, float *y, void *stream);
int e2ep_se_gate_bwd(const float *x, const float *a, const float *dy, int planes, int HW,
                     float *dx, float *da, void *stream);

/* ---------------------------------------------------------------------------------------
 * Transformer token assembly with the positional embedding and pos_drop, fwd and bwd
 * (dropout: keep bit = counter hash of the device seed and the output element index, scale
 * 1 / (1 - p); p = 0 is the identity and needs no seed):
 *  - fusion encoder (replaces model/feature_fusion.py:41-46: transpose, expand, torch.cat,
 *    + pos_embed, pos_drop): tokens [B][S][E] = drop(x + pos[S][E]) with x = bev[b][e][s]
 *    (bev [B][C][S], the BEV encoder output) for e < C and motion[b][s] (motion [B][S]) for
 *    C <= e < E.  bwd: dbev [B][C][S], dmotion [B][S] (sum over the E - C broadcast channels,
 *    which must lie in one 32-channel tile), dpos [S][E] (sum over b in order).
 *  - control decoder (replaces model/control_predict.py:53-54: embedding + pos_embed +
 *    pos_drop): out [B][T][E] = drop(table[tok[b*tok_stride + t]] + pos[T][E]) (int64 tokens,
 *    clamped into [0, V)); bwd: dtable [V][E] (every row written: sum over the (b, t) whose
 *    token is v, in (b, t) order), dpos [T][E] (sum over b in order).  No atomics.
 * ------------------------------------------------------------------------------------- */
int e2ep_fusion_tokens_fwd(const float *bev, const float *motion, const float *pos, int B, int C,
                           int S, int E, float p, const int32_t *seed, float *tokens,
                           void *stream);
int e2ep_fusion_tokens_bwd(const float *dtokens, int B, int C, int S, int E, float p,
                           const int32_t *seed, float *dbev, float *dmotion, float *dpos,
                           void *stream);
int e2ep_embed_tokens_fwd(const int64_t *tok, int tok_stride, const float *table, int V,
                          const float *pos, int B, int T, int E, float p, const int32_t *seed,
                          float *out, void *stream);
/* Autoregressive control decoding on a persistent token buffer (reference
 * model/parking_model.py:72-78 calling model/control_predict.py:60-75 three times: pad with
 * PAD, softmax, argmax, torch.cat — here two kernels, no host sync, capturable):
 *   e2ep_tokens_init: seq[b, t] = t < L ? prefix[b * prefix_stride + t] : pad   (B x T)
 *   e2ep_token_argmax_append: seq[b, pos] = argmax_v softmax(logits[b * row_stride + v])
 *     over v < V: the softmax values as exp(x - max) / sum, argmax = first index of the largest
 *     probability (torch.argmax's rule).  One workgroup per row. */
int e2ep_tokens_init(const int64_t *prefix, int prefix_stride, int B, int L, int64_t *seq, int T,
                     int64_t pad, void *stream);
int e2ep_token_argmax_append(const float *logits, long long row_stride, int B, int V,
                             int64_t *seq, int seq_stride, int pos, void *stream);
int e2ep_embed_tokens_bwd(const float *dout, const int64_t *tok, int tok_stride, int V, int B,
                          int T, int E, float p, const int32_t *seed, float *dtable, float *dpos,
                          void *stream);

/* ---------------------------------------------------------------------------------------
 * Optimizer: fused Adam over one flat parameter buffer (replaces torch.optim.Adam configured
 * at trainer/pl_trainer.py:116-121; torch Adam semantics: L2 weight decay added to the
 * gradient, bias-corrected step, no amsgrad).
 * chunks[4*n_chunks] = {tensor, start element, length (<= e2ep_adam_chunk_elems()), 0};
 * offsets[tensor] = element offset of the tensor in the flat
 * param / exp_avg / exp_avg_sq buffers (multiple of 4).  Gradients come from grad_ptrs
 * (device array of per-tensor device addresses; 0 = no gradient, tensor not stepped) or,
 * if grad_flat is non-null, from a flat buffer laid out like the parameters (grad_ptrs, when
 * also given, still marks the tensors without a gradient, which are skipped).  `step` is a
 * device fp32 counter incremented by the call and `lr` a device fp64 scalar read by it, so a
 * captured call follows an LR schedule (trainer/pl_trainer.py:120 CosineAnnealingLR) under
 * graph replay: no host scalar that changes between steps is baked into the launch.
 * `stepped` (optional, int32 per tensor) is set to 1 for every tensor the call steps, so the
 * caller can write torch.optim.Adam-format state for exactly the stepped tensors.
 * ------------------------------------------------------------------------------------- */
int e2ep_adam_chunk_elems(void);
int e2ep_adam_step(const int *chunks, int n_chunks, const long long *offsets,
                   const long long *grad_ptrs, const float *grad_flat, float *param, float *exp_avg,
                   float *exp_avg_sq, float *step, const double *lr, double beta1, double beta2,
                   double eps, double weight_decay, float grad_scale, int *stepped,
                   void *stream);
/* per-tensor gradients -> flat buffer (zeros for missing gradients), for the all-reduce;
 * a sub-range of the chunk table (chunks + 4*first, n) gathers one gradient bucket */
int e2ep_grad_gather(const int *chunks, int n_chunks, const long long *offsets,
                     const long long *grad_ptrs, float *grad_flat, void *stream);

/* ---------------------------------------------------------------------------------------
 * Training losses (fp32; fixed-order reductions; every scalar stays on the device):
 *  - control CE (loss/control_loss.py:15-19): logits [B*T, vocab], targets
 *    gt[b*gt_stride + gt_offset + t] (int64, the reference's gt_control[:, 1:]), rows whose
 *    target is `pad` ignored, mean over the rest.  fwd writes loss, lse [B*T] and count
 *    (non-ignored rows) for bwd; workspace e2ep_control_ce_workspace(B*T) bytes.
 *  - segmentation CE (loss/seg_loss.py:12-26): logits [images, C, HW], target [images, HW]
 *    int64, class weights [C]; per-pixel weighted CE, `ignore` pixels contribute 0, plain
 *    mean over all images*HW pixels; workspace e2ep_seg_ce_workspace(images, HW) bytes.
 *  - depth BCE (loss/depth_loss.py:18-48): prob [BN, D, H/down, W/down] softmax
 *    probabilities, gt [BN, H, W] metric depth; label of a cell = one-hot(D+1)[1:] of
 *    trunc((min non-zero depth of its down x down block - lo) / step) (bins outside [0, D+1)
 *    -> 0; lo = d_bound[0] - d_bound[2], step = d_bound[2]); BCE (log clamped at -100) over
 *    the cells with a label, summed / max(1, #such cells).  fwd writes loss, den (the
 *    normaliser) and cls [BN*h*w] (the class, 0 = background) for bwd; workspace
 *    e2ep_depth_bce_workspace(BN, H, W, down) bytes.  e2ep_depth_bce_fwd_f64 takes the
 *    float64 depth the reference dataset produces (dataset/carla_dataset.py:107-113) and
 *    computes the bins in float64, as torch does on that tensor.
 * Backward kernels read the upstream gradient `gloss` (a device scalar) and write the full
 * input gradient (zeros where the loss does not depend on the input).
 * ------------------------------------------------------------------------------------- */
size_t e2ep_control_ce_workspace(int rows);
int e2ep_control_ce_fwd(const float *logits, const long long *gt, int B, int T, int gt_stride,
                        int gt_offset, int vocab, int pad, float *loss, float *lse, float *count,
                        void *workspace, void *stream);
int e2ep_control_ce_bwd(const float *logits, const long long *gt, const float *lse,
                        const float *count, const float *gloss, int B, int T, int gt_stride,
                        int gt_offset, int vocab, int pad, float *dlogits, void *stream);
size_t e2ep_seg_ce_workspace(int images, int HW);
int e2ep_seg_ce_fwd(const float *logits, const long long *target, const float *weights, int images,
                    int C, int HW, int ignore, float *loss, void *workspace, void *stream);
int e2ep_seg_ce_bwd(const float *logits, const long long *target, const float *weights,
                    const float *gloss, int images, int C, int HW, int ignore, float *dlogits,
                    void *stream);
size_t e2ep_depth_bce_workspace(int BN, int H, int W, int down);
int e2ep_depth_bce_fwd(const float *prob, const float *gt, int BN, int D, int H, int W, int down,
                       float lo, float step, float *loss, float *den, int *cls, void *workspace,
                       void *stream);
int e2ep_depth_bce_fwd_f64(const float *prob, const double *gt, int BN, int D, int H, int W,
                           int down, double lo, double step, float *loss, float *den, int *cls,
                           void *workspace, void *stream);
int e2ep_depth_bce_bwd(const float *prob, const int *cls, const float *den, const float *gloss,
                       int BN, int D, int hw, float *dprob, void *stream);

/* ---------------------------------------------------------------------------------------
 * Strided fp32 GEMM for the transformer linears (nn.Linear forward and its two backward
 * GEMMs: model/feature_fusion.py:13-14,24-29,48-50, model/control_predict.py:18-24):
 *   C[m][n] = sum_k A(m,k) B(k,n) (+ bias[n]) (+ Cadd[m][n]), then ReLU when relu != 0;
 *   A(m,k) = a_kcontig ? A[m*lda + k] : A[k*lda + m];  B(k,n) = b_kcontig ? B[n*ldb + k]
 *   : B[k*ldb + n];  C row-major with leading dimension ldc.
 * v_mfma_f32_32x32x2_f32, fixed summation order (deterministic).  Small grids split K and
 * need e2ep_gemm_workspace(M, N, K) bytes of workspace (0 when no split).
 * ------------------------------------------------------------------------------------- */
size_t e2ep_gemm_workspace(int M, int N, int K);
/* Benchmarking override of the launch plan: block tile 1 = 64x64, 2 = 32x128, 3 = 128x128,
 * 4 = 64x128, 5 = 128x64, 6 = 64x256 (0 = the automatic plan), and the K split. */
int e2ep_gemm_force(int tile, int splits, int unused);
/* Few-row forward products (a_kcontig and b_kcontig, M <= max_rows, at most 128; default 16)
 * run on a block-per-output-column dot-product kernel instead of the MFMA tiles (the control
 * decoder's 14 rows at B = 1, C5 predict); 0 disables it, < 0 only queries.  Returns the
 * previous limit. */
int e2ep_gemm_skinny(int max_rows);
/* Operand precision of e2ep_gemm / e2ep_gemm_rowsum: 0 = fp32 (default, exact-f32 MFMA), 1 =
 * bf16 operands rounded as they enter the matrix cores (v_mfma_f32_32x32x16_bf16), fp32
 * products, sums and tensors (BASELINE C3); < 0 only queries.  Returns the previous value.
 * The few-row path (e2ep_gemm_skinny) stays fp32. */
int e2ep_gemm_precision(int precision);
/* Minimum K-steps (32 deep) per K split for grids under 64 blocks (default 8); <= 0 queries.
 * Returns the previous value. */
int e2ep_gemm_split_min(int ksteps);

/* BatchNorm single-launch switch: on = 1 (default) lets e2ep_bn_fwd / e2ep_bn_stats /
 * e2ep_bn_bwd run channels of N*H*W <= 8192 (H*W % 4 == 0, training statistics) as one
 * block-per-channel launch that keeps the channel in registers; 0 forces the split
 * statistics + apply kernels for every shape; < 0 only queries.  Returns the previous value. */
int e2ep_bn_small(int on);
/* Largest channel, in float4 vectors (N*H*W / 4), the single-launch BN kernels take in the
 * forward / backward (default and maximum 2048 each; < 0 keeps the setting).  For A/B timing. */
int e2ep_bn_small_limits(int fwd_max_vec, int bwd_max_vec);
/* Launch-plan tunables (read at every launch; value <= 0 only queries; returns the previous
 * value, -1 for an unknown key), defaults in parentheses: 0 split-BN target workgroups (2048),
 * 1 minimum elements per split-BN workgroup (4096), 2 float4 vectors per BN apply workgroup
 * (1024), 3 depthwise weight-gradient target workgroups (512), 4 K-split e2ep_gemm target
 * workgroups (768), 5 1x1 weight-gradient target workgroups (1024), 6 conv forward /
 * data-gradient grids of at least this many wide (128 / 256-column) tiles use them (512),
 * 7 k_conv_gemm block tile forced to bm * 1000 + bnt (64064, 64128, 32128, 32256; 1 =
 * automatic), 8 k_conv_gemm K splits forced to value - 1 (1 = automatic), 9 spatial
 * weight-gradient kernel (2 = k_conv_wgrad2 where it applies, 1 = k_conv_wgrad), 10 k_conv_lp
 * wave tile forced to wm * 10 + wn (1 = automatic), 11 16-bit conv forward / data gradient on
 * k_conv_lp (2) or the fp32-era kernels with rounded operands (1), 12 bf16 weight gradient on
 * k_wgrad_lp (2) or k_conv_wgrad2 / k_wgrad_1x1 (1), 13 k_wgrad_lp tile forced (wm * 10 + wn;
 * 1 = automatic), 14 fp32 3x3 layers on the fp32 k_conv_lp tile (2) or not (1), 15 fp32 weight
 * gradient on k_wgrad_lp (2) or not (1, default), 16 k_conv_lp K step (32 / 64; 1 = automatic
 * = 32), 17 k_wgrad_lp pixels per step (32 / 64 / 128; 1 = automatic = 32), 18 forward /
 * data-gradient K order (1 = automatic: channel chunk outer for 16-bit operands, tap outer for
 * fp32; 2 channel outer; 3 tap outer), 19 XCD-contiguous block order of the conv_lp.hip
 * kernels (2 = on, 1 = off, default), 20 attention lanes per query / key for sequences longer
 * than 16 (1 = automatic, 2, 4), 21 attention on the matrix-core kernels of attn_mf.hip where
 * they apply (2 = forward and dq, default; 3 = also dk / dv; 1 = off), 22 k_wgrad_lp K-split
 * target workgroups (1024), 23 depthwise strip kernels' LDS window reads (2 = 16-B vector
 * reads, default; 1 = scalar reads), 24 depthwise forward / stride-1 data-gradient grid cap in
 * blocks (2048; each wave walks units beyond it in a software-pipelined loop), 25 single-launch BN
 * blocks for channels of 1025..2048 float4 (2 = 512 threads x 4 float4, default; 1 = 256 x 8),
 * 26 the same for channels of 257..1024 float4 (2 = 512 threads; 1 = 256, default: equal),
 * 28 split-K reductions folded into the producing launch (2, default) or separate reduce
 * kernels (1), 30 1x1 paired backward block order (2 = weight-gradient blocks first, default;
 * 1 = data-gradient first).  Keys 27, 29 and 31 are retired (their A/B kept the default and the
 * alternative code is removed): they return -1 like an unknown key.
 * For A/B timing.
 * Contract for every plan override and tunable above (e2ep_conv_split_params,
 * e2ep_gemm_force, e2ep_gemm_split_min, e2ep_bn_small*, e2ep_tune): a launch recomputes its
 * plan from these process-wide settings, and the *_workspace() queries size the workspace
 * from the same plan, so set them before a caller queries workspace sizes (in practice:
 * before the first step is run or captured) and never change them between a caller's
 * workspace query and its launch.  Every entry point that takes a workspace also takes its
 * size in bytes (workspace_bytes) and returns E2EP_EINVAL, launching nothing, when the plan it
 * would run needs more (round 4: a plan changed after the query can no longer write past the
 * buffer). */
int e2ep_tune(int key, int value);
int e2ep_gemm(const float *A, int lda, int a_kcontig, const float *B, int ldb, int b_kcontig,
              const float *bias, const float *Cadd, int ldadd, float *C, int ldc, int M, int N,
              int K, int relu, void *workspace, size_t workspace_bytes, void *stream);
/* Weight gradient of a linear layer together with its bias gradient (replaces the
 * nn.Linear backward's grad_weight = dY^T X and grad_bias = dY.sum(0), model/feature_fusion.py
 * :13-14,24-29, model/control_predict.py:18-24): C = A(m,k) B(k,n) with A(m,k) = A[k*lda + m]
 * and B(k,n) = B[k*ldb + n] (the a_kcontig = b_kcontig = 0 case of e2ep_gemm), and
 * rowsum[m] = sum_k A(m,k) taken by the same launch as a column of ones appended to B.
 * Workspace: e2ep_gemm_rowsum_workspace(M, N, K) bytes (0 when no K split). */
size_t e2ep_gemm_rowsum_workspace(int M, int N, int K);
int e2ep_gemm_rowsum(const float *A, int lda, const float *B, int ldb, float *C, int ldc,
                     float *rowsum, int M, int N, int K, void *workspace,
                     size_t workspace_bytes, void *stream);
/* A linear layer's backward in one launch (k_gemm_pair): dx[M][K] = dy[M][N] w[N][K] (+ gskip,
 * nullable, a residual gradient in dx's layout) and dw[N][K] = dy^T x[M][K] with db[N] = the
 * row sums of dy^T (the bias gradient) — the two products of e2ep_gemm / e2ep_gemm_rowsum,
 * their blocks sharing one grid instead of two launches on forked streams (a fork / join of a
 * replayed HIP graph idles the GPU ~15 us, longer than either product of the control decoder).
 * Replaces nn.Linear's backward in the transformer layers (model/feature_fusion.py:13-14,
 * model/control_predict.py:19-20).  Workspaces: ws_dx of e2ep_gemm_workspace(M, K, N) bytes,
 * ws_dw of e2ep_gemm_rowsum_workspace(N, K, M) bytes (either may be NULL when that query is 0).
 * Results are bitwise those of the two separate launches. */
int e2ep_linear_bwd(const float *dy, int ldy, const float *x, int ldx, const float *w, int ldw,
                    const float *gskip, int ldskip, float *dx, int lddx, float *dw, int lddw,
                    float *db, int M, int N, int K, void *ws_dx, size_t ws_dx_bytes, void *ws_dw,
                    size_t ws_dw_bytes, void *stream);

/* ---------------------------------------------------------------------------------------
 * Frame decode (dataset/carla_dataset.py:114-131, :494-515, :404-406): the per-step
 * arithmetic of the reference data path on cached uint8 crops.
 *  - e2ep_decode_frames: rgb / depth_rgb [*][hw][3] uint8 (either may be NULL); output
 *    frame f reads source frame src_frame[f] (f when src_frame is NULL: a gather out of a
 *    resident cache and the decode in one pass) -> image [frames][3][hw] fp32 = (v / 255 - mean_c) / std_c with the ImageNet mean / std
 *    (torchvision ToTensor + Normalize, each step rounded to fp32), depth [frames][hw] fp64
 *    metres = 1000 * ((R + 256 G + 65536 B) / (2^24 - 1)).  hw % 4 == 0; inputs 4-byte and
 *    outputs 16-byte aligned.  Bit-identical to the reference's CPU arithmetic.
 *  - e2ep_widen_u8_i64: rows x row_len uint8 class ids -> int64, output row r reading
 *    source row src_row[r] (r when NULL); row_len % 4 == 0, src 4-byte and dst 16-byte
 *    aligned.
 * ------------------------------------------------------------------------------------- */
int e2ep_decode_frames(const void *rgb, const void *depth_rgb, const long long *src_frame,
                       long long frames, int hw, float *image, double *depth, void *stream);
int e2ep_widen_u8_i64(const void *src, const long long *src_row, long long rows, int row_len,
                      long long *dst, void *stream);

/* ---------------------------------------------------------------------------------------
 * HIP-graph surgery: replace every memset node of a captured (not yet instantiated)
 * hipGraph_t by an equivalent kernel node.  Memset nodes replay incorrectly after the first
 * launch on this ROCm stack; PyTorch's reductions capture them.  `replaced` (optional)
 * receives the number of nodes rewritten.
 * ------------------------------------------------------------------------------------- */
int e2ep_graph_replace_memsets(void *graph, int *replaced);
/* An executable of a (repaired) captured graph and its launch on a stream, bypassing
 * torch.cuda.CUDAGraph.replay(), whose prologue launches int64 fill kernels to refresh torch's
 * generator states (the step's random numbers come from e2ep_rng_draw). */
int e2ep_graph_exec_create(void *graph, void **exec);
/* Before ending a capture on `origin`: *unjoined = 1 when `side` is part of the same capture
 * and its last captured work is not an ancestor of origin's current capture frontier (a
 * forked stream that was never joined back; hipStreamEndCapture would fail or crash on it),
 * else 0.  Host-side graph inspection only (hipStreamGetCaptureInfo_v2). */
int e2ep_capture_unjoined(void *origin, void *side, int *unjoined);
int e2ep_graph_exec_launch(void *exec, void *stream);
int e2ep_graph_exec_destroy(void *exec);

#ifdef __cplusplus
}
#endif
#endif /* E2EP_H */
