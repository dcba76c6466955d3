// Launch-plan tunables shared by the kernel files (set through e2ep_tune, read at launch).
#pragma once

namespace e2ep {
enum Tune {
  TUNE_BN_SPLIT_TARGET = 0,   // workgroups the split BN statistics / reduction aim at
  TUNE_BN_SPLIT_MIN = 1,      // minimum elements per split-BN workgroup
  TUNE_BN_APPLY_PER = 2,      // float4 vectors per BN apply workgroup
  TUNE_DW_WGRAD_TARGET = 3,   // workgroups the depthwise weight gradient aims at
  TUNE_GEMM_SPLIT_TARGET = 4, // workgroups a K-split e2ep_gemm aims at
  TUNE_WGRAD1X1_TARGET = 5,   // workgroups the 1x1 weight gradient aims at
  TUNE_CONV_WIDE_MIN = 6,     // conv fwd / dgrad grids of at least this many wide tiles use them
  TUNE_CONV_FORCE_TILE = 7,   // benchmarking: k_conv_gemm tile bm * 1000 + bnt (1 = automatic)
  TUNE_CONV_FORCE_SPLITS = 8, // benchmarking: k_conv_gemm K splits + 1 (1 = automatic)
  TUNE_WGRAD_GEN = 9,         // spatial weight-gradient kernel: 2 = k_conv_wgrad2 where it applies, 1 = k_conv_wgrad
  TUNE_LP_FORCE_TILE = 10,    // benchmarking: k_conv_lp wave tile wm * 10 + wn (1 = automatic)
  TUNE_LP = 11,               // low-precision conv forward / data gradient: 2 = k_conv_lp, 1 = k_conv_gemm(2)
  TUNE_LP_WGRAD = 12,         // bf16 weight gradient: 2 = k_wgrad_lp, 1 = k_conv_wgrad2 / k_wgrad_1x1
  TUNE_LP_WGRAD_TILE = 13,    // benchmarking: k_wgrad_lp wave tile wm * 10 + wn (1 = automatic)
  TUNE_LP32 = 14,             // fp32 conv forward / data gradient: 2 = k_conv_lp<OP 0> where lp_ok, 1 = conv.hip kernels
  TUNE_LP32W = 15,            // fp32 weight gradient: 2 = k_wgrad_lp<OP 0> where lp_wgrad_ok, 1 = conv.hip kernels
  TUNE_LP_LK = 16,            // k_conv_lp K step (16-bit operands): 32 / 64 forced, 1 = automatic
  TUNE_LPW_LK = 17,           // k_wgrad_lp pixels per step (bf16): 32 / 64 forced, 1 = automatic
  TUNE_KORDER = 18,           // conv forward / data-gradient K order: 1 = automatic, 2 = channel chunk outer, 3 = tap outer
  TUNE_XCD = 19,              // conv_lp.hip kernels: 2 = XCD-contiguous block order, 1 = hardware order
  TUNE_ATT_LANES = 20,        // attention lanes per query / key for long sequences: 1 (automatic), 2, 4
  TUNE_ATT_MF = 21,           // attention on the matrix-core kernels where they apply: 2 = on, 1 = off
  TUNE_LPW_TARGET = 22,       // workgroups the k_wgrad_lp K split aims at
  TUNE_DW_VEC = 23,           // depthwise strip kernels' LDS rows: 2 = ds_read_b128 windows, 1 = scalar reads
  TUNE_DW_FWD_BLOCKS = 24,    // depthwise forward / stride-1 data-gradient strip kernel: grid cap (blocks)
  TUNE_BNS_WIDE = 25,         // single-launch BN, channels of 1025..2048 float4: 2 = 512 threads x 4, 1 = 256 x 8
  TUNE_BNS_WIDE_LO = 26,      // the same for channels of 257..1024 float4: 2 = 512 threads x 1 / 2, 1 = 256 x 2 / 4
  TUNE_RETIRED_27 = 27,       // retired (was the fused squeeze-excitation MLP: 1.8 ms/step slower, removed)
  TUNE_SPLITK_FOLD = 28,      // split-K reductions folded into the producing launch (last-arriving split sums): 2 = on, 1 = separate reduce kernels
  TUNE_RETIRED_29 = 29,       // retired (was the conv pair block order: data-gradient first kept)
  TUNE_PAIR1X1_ORDER = 30,    // 1x1 paired backward (k_conv_bwd_pair1x1): 2 = weight-gradient blocks first (default: C2 22.73 -> 22.50 ms), 1 = data-gradient blocks first
  TUNE_RETIRED_31 = 31,       // retired (was the linear pair block order: input-gradient first kept)
  TUNE_LSS_FWD = 32,          // k_lss_fwd shape: 1 = automatic (16 x 16 when a sample's featT > 4 MB, else 16 x 8), 2 = 32 groups x 8 rows in flight, 3 = 16 x 16, 4 = 32 x 16, 5 = 16 x 8
  TUNE_BN_ORDER = 33,         // split BN sweeps back to front: 1 + mask (1 bwd apply, 2 bwd reduction, 4 fwd apply); 1 = all front to back
  TUNE_SE_EXCITE_MLP = 34,    // squeeze-excitation logits inside the excite launch: 2 = on, 1 = k_se_logits + k_se_excite
  TUNE_STEM_DIRECT = 35,      // BEV stem (7x7/2, 64 out, 16-bit operands) on the direct-conv kernels: 1 + mask (1 forward k_conv_stem_lp, 2 data gradient k_conv_stem_dgrad_lp, 4 weight gradient k_conv_stem_wgrad_lp; fp32 operands also 8 the gradients, 16 the forward); 1 = the implicit GEMMs
  TUNE_N = 36
};
extern int g_tune[TUNE_N];
}  // namespace e2ep
