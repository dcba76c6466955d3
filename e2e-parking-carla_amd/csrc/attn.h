// Internal interface of the attention kernels (attn.hip: vector-FMA kernels for every shape;
// attn_mf.hip: matrix-core kernels for the fusion encoder's long sequences).
#pragma once
#include <stdint.h>

#include "common.h"

namespace e2ep {

struct AttnDims {
  int B, H, Sq, Sk, dh;
  int q_ss, q_sb, kv_ss, kv_sb, o_ss, o_sb;  // element strides (sequence, batch)
  float scale, p;
  int causal;
};

// attn_mf.hip: unmasked attention with Sq, Sk in {128, 256} and head dim <= 44 on
// v_mfma_f32_32x32x2_f32 (e2ep_tune key 21: 2 = forward and dq (default), 3 = also dk / dv,
// 1 = off).  The same
// log2-domain lse, dropout counters and D = dO . O as the attn.hip kernels, so either forward
// pairs with either backward.
bool attn_mf_ok(const AttnDims &a, const uint8_t *key_pad);
void attn_mf_fwd(const float *q, const float *k, const float *v, const int *seed,
                 const AttnDims &a, float *o, float *lse2, hipStream_t s);
// dq (and D into Dbuf), then, with e2ep_tune key 21 = 3, dk / dv (reading Dbuf); part as
// e2ep_attn_bwd_part (0 all, 2 dq only, 3 dk / dv only).  Returns whether dk / dv were done.
bool attn_mf_bwd(const float *q, const float *k, const float *v, const float *o,
                 const float *dout, const float *lse2, const int *seed, const AttnDims &a,
                 float *dq, float *dk, float *dv, float *Dbuf, int part, hipStream_t s);

}  // namespace e2ep
