// Fused multi-head attention (fp32) for the fusion encoder and the control decoder:
// softmax(scale * Q K^T + mask) -> dropout -> @ V, forward and backward, reading Q/K/V
// straight out of the in-projection output and writing O in the (S, B, E) layout the
// out-projection consumes.  Replaces the inner part of torch.nn.MultiheadAttention as called
// by the reference's TransformerEncoderLayer / TransformerDecoderLayer
// (model/feature_fusion.py:13-14,48-50; model/control_predict.py:19-20,39-47): PyTorch runs
// it there as bmm -> (mask add) -> safe softmax -> dropout -> bmm with the score tensor
// written and re-read by ~10 launches per direction.
//
// Shapes on the path: encoder Sq = Sk = 256, decoder self Sq = Sk = 14 (causal + key
// padding), decoder cross Sq = 14, Sk = 256; 6 heads x dh 43; B = 8.  Scores never leave the
// chip.  Work per (query, key) pair is a few dh-long dot products, so this is vector-FMA
// work on data held in LDS (a head's K/V is <= 90 KB), not MFMA: at dh = 43 and fp32 the
// 32x32x2 MFMA tile would waste a third of the K dimension and the whole problem is
// ~0.3 GFLOP per layer.
//
//   k_attn_fwd    block = (64-query tile, b*h); the head's K and V staged in LDS row-major
//                 [key][DHP]; lane = query (q row in registers), 4 waves split the keys and
//                 run an online softmax over 8-key groups; the 4 partial (max, sum, acc)
//                 triples are merged in fixed wave order through LDS; O goes out through an
//                 LDS tile as contiguous dh-float rows.  Also writes lse (log2 domain).
//   k_attn_bwd_q  same tiling; recomputes P from lse, D_i = dO_i . O_i, and
//                 dS = P (drop(dO V^T) - D); dQ = scale dS K (waves merged in fixed order).
//   k_attn_bwd_kv block = (64-key tile, b*h); Q, dO, lse, D of the head staged in LDS;
//                 lane = key (k, v, dk, dv rows in registers), 4 waves split the queries;
//                 dV = P_drop^T dO, dK = scale dS^T Q.
// Dropout: keep(b*h, i, j) = hash(seed, (bh*Sq + i)*Sk + j) >= p, scaled by 1/(1-p); the
// seed is read from device memory (drawn by the caller each call, graph-capturable), so the
// backward regenerates the same mask without storing it.
#include "attn.h"
#include "common.h"
#include "dropout.h"

namespace e2ep {

constexpr int ATT_SMAX = 256;  // max Sq / Sk (one head's K, V staged whole)
constexpr int ATT_WAVES = 4;
constexpr float LOG2E = 1.4426950408889634f;
#ifndef E2EP_ATT_KG
#define E2EP_ATT_KG 4
#endif
constexpr int FWD_KG = E2EP_ATT_KG;  // keys per online-softmax rescale in the forward
// lanes per query (forward, dq) / per key (dk, dv) for sequences longer than 16 (the encoder's
// 256): e2ep_tune key 20 (1 = automatic = 1, or 2 / 4 for A/B; more lanes per query = smaller
// query tiles, more workgroups)
static int att_lanes() {
  const int t = g_tune[TUNE_ATT_LANES];
  return t == 2 || t == 4 ? t : 1;
}

// 2^x on the hardware v_exp_f32 (arguments here are <= 0 or -inf; tiny results flush to 0)
__device__ __forceinline__ float att_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int DHP>
__device__ __forceinline__ float dot_lds(const float (&r)[DHP], const float *row) {
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int d = 0; d < DHP; d += 4) {
    const float4 k = *reinterpret_cast<const float4 *>(row + d);
    s0 = __builtin_fmaf(r[d], k.x, s0);
    s1 = __builtin_fmaf(r[d + 1], k.y, s1);
    s0 = __builtin_fmaf(r[d + 2], k.z, s0);
    s1 = __builtin_fmaf(r[d + 3], k.w, s1);
  }
  return s0 + s1;
}
template <int DHP>
__device__ __forceinline__ void axpy_lds(float (&acc)[DHP], float a, const float *row) {
#pragma unroll
  for (int d = 0; d < DHP; d += 4) {
    const float4 v = *reinterpret_cast<const float4 *>(row + d);
    acc[d] = __builtin_fmaf(a, v.x, acc[d]);
    acc[d + 1] = __builtin_fmaf(a, v.y, acc[d + 1]);
    acc[d + 2] = __builtin_fmaf(a, v.z, acc[d + 2]);
    acc[d + 3] = __builtin_fmaf(a, v.w, acc[d + 3]);
  }
}


// stage rows [0, n) of a head's (S, B, E)-strided matrix into LDS as [n][DHP] (zero padded).
// Loads go out STAGE_BATCH per thread before any LDS store (branch-free buffer loads; out of
// range -> 0), so a head's 90 KB arrives in a few memory round trips, not one per element.
constexpr int STAGE_BATCH = 32;
template <int DHP>
__device__ __forceinline__ void stage_rows(float *dst, const float *src, int n, int ss, int dh) {
  const int total = n * DHP;
  const __amdgpu_buffer_rsrc_t R = rsrc(src, 4LL * ((long long)(n - 1) * ss + dh));
  for (int e0 = 0; e0 < total; e0 += ATT_WAVES * 64 * STAGE_BATCH) {
    float t[STAGE_BATCH];
#pragma unroll
    for (int u = 0; u < STAGE_BATCH; ++u) {
      const int e = e0 + u * ATT_WAVES * 64 + (int)threadIdx.x;
      const int r = e / DHP, d = e - r * DHP;
      t[u] = bload(R, (e < total && d < dh) ? 4 * (r * ss + d) : OOR);
    }
#pragma unroll
    for (int u = 0; u < STAGE_BATCH; ++u) {
      const int e = e0 + u * ATT_WAVES * 64 + (int)threadIdx.x;
      if (e < total) dst[e] = t[u];
    }
  }
}

// one head row (dh floats at p) into registers, zero padded to DHP, times mul.  p differs per
// lane, so no buffer descriptor (that would waterfall): padded slots re-read element dh-1
// (always in bounds) and are zeroed by the multiplier, so the loads carry no branches.
template <int DHP>
__device__ __forceinline__ void load_row(float (&r)[DHP], const float *p, int dh, float mul) {
#pragma unroll
  for (int d = 0; d < DHP; ++d) r[d] = p[min(d, dh - 1)] * (d < dh ? mul : 0.f);
}

// lanes-per-row butterfly merges (rows = queries or keys spread over L consecutive lanes)
template <int L, int N>
__device__ __forceinline__ void lane_sum(float (&x)[N]) {
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1)
#pragma unroll
    for (int d = 0; d < N; ++d) x[d] += __shfl_xor(x[d], off, 64);
}

// write an LDS tile [ROWS][DHP] (rows r0.. of a head) to an (S, B, E)-strided matrix
template <int DHP, int ROWS>
__device__ __forceinline__ void store_rows(float *dst, const float *tile, int r0, int n, int ss,
                                           int dh) {
  const int nr = min(ROWS, n - r0);
  for (int e = threadIdx.x; e < nr * dh; e += ATT_WAVES * 64) {
    const int r = e / dh, d = e - r * dh;
    dst[(long long)(r0 + r) * ss + d] = tile[r * DHP + d];
  }
}

template <int DHP, int LPQ>
__global__ void __launch_bounds__(ATT_WAVES * 64) k_attn_fwd(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const uint8_t *__restrict__ kpad, const int *__restrict__ seed, AttnDims a,
    float *__restrict__ o, float *__restrict__ lse2) {
  __shared__ __attribute__((aligned(16))) float sm[2 * ATT_SMAX * DHP];
  __shared__ float smask[ATT_SMAX];
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  constexpr int QPW = 64 / LPQ;  // queries per block; LPQ lanes share a query's keys
  const int q0 = blockIdx.x * QPW;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane & (LPQ - 1);
  float *sK = sm, *sV = sm + ATT_SMAX * DHP;
  const long long kvoff = (long long)b * a.kv_sb + h * a.dh;
  stage_rows<DHP>(sK, k + kvoff, a.Sk, a.kv_ss, a.dh);
  stage_rows<DHP>(sV, v + kvoff, a.Sk, a.kv_ss, a.dh);
  for (int j = threadIdx.x; j < a.Sk; j += ATT_WAVES * 64)
    smask[j] = (kpad && kpad[(long long)b * a.Sk + j]) ? -INFINITY : 0.f;
  const int i = q0 + lane / LPQ;
  float qr[DHP];
  const float qmul = a.scale * LOG2E;  // scores in the log2 domain
  const float *qrow = q + (long long)b * a.q_sb + h * a.dh + (long long)min(i, a.Sq - 1) * a.q_ss;
  load_row<DHP>(qr, qrow, a.dh, qmul);
  __syncthreads();
  const uint32_t sm_ = att_seedmix(seed);
  const int chunk = (a.Sk + ATT_WAVES - 1) / ATT_WAVES;
  const int j0 = w * chunk, j1 = min(a.Sk, j0 + chunk);
  float m = -INFINITY, l = 0.f, acc[DHP];
#pragma unroll
  for (int d = 0; d < DHP; ++d) acc[d] = 0.f;
  const uint32_t cbase = ((uint32_t)bh * a.Sq + i) * a.Sk;
  for (int jb = j0 + sub; jb < j1; jb += FWD_KG * LPQ) {
    float s[FWD_KG];
    float bm = -INFINITY;
#pragma unroll
    for (int u = 0; u < FWD_KG; ++u) {
      const int j = jb + u * LPQ;
      const int jl = min(j, j1 - 1);
      const float x = dot_lds<DHP>(qr, sK + jl * DHP) + smask[jl];
      s[u] = (j < j1 && !(a.causal && j > i)) ? x : -INFINITY;
      bm = fmaxf(bm, s[u]);
    }
    const float mn = fmaxf(m, bm);
    const float ms = mn == -INFINITY ? 0.f : mn;
    const float corr = att_exp2(m - ms);
    m = mn;
    l *= corr;
#pragma unroll
    for (int d = 0; d < DHP; ++d) acc[d] *= corr;
#pragma unroll
    for (int u = 0; u < FWD_KG; ++u) {
      const float pu = att_exp2(s[u] - ms);
      l += pu;
      const int j = min(jb + u * LPQ, j1 - 1);
      const float pd = (a.p > 0.f && !att_keep(sm_, cbase + j, a.p)) ? 0.f : pu;
      axpy_lds<DHP>(acc, pd, sV + j * DHP);
    }
  }
  if (LPQ > 1) {  // merge the query's LPQ lane partials (same result in every lane)
#pragma unroll
    for (int off = LPQ / 2; off > 0; off >>= 1) {
      const float mo = __shfl_xor(m, off, 64);
      const float mn = fmaxf(m, mo);
      const float ms = mn == -INFINITY ? 0.f : mn;
      const float fs = att_exp2(m - ms), fo = att_exp2(mo - ms);
      l = l * fs + __shfl_xor(l, off, 64) * fo;
#pragma unroll
      for (int d = 0; d < DHP; ++d) acc[d] = acc[d] * fs + __shfl_xor(acc[d], off, 64) * fo;
      m = mn;
    }
  }
  __syncthreads();  // K/V no longer needed: reuse sm for the merge
  float *mrg = sm;  // [w][DHP + 2][64], column = query within the block
  constexpr int MS = (DHP + 2) * 64;
  if (sub == 0) {
    const int c = lane / LPQ;
    mrg[w * MS + c] = m;
    mrg[w * MS + 64 + c] = l;
#pragma unroll
    for (int d = 0; d < DHP; ++d) mrg[w * MS + (d + 2) * 64 + c] = acc[d];
  }
  __syncthreads();
  // wave w merges dims [w*DHP/4, (w+1)*DHP/4) of query `lane` in fixed wave order
  float M = -INFINITY;
#pragma unroll
  for (int x = 0; x < ATT_WAVES; ++x) M = fmaxf(M, mrg[x * MS + lane]);
  const float Ms = M == -INFINITY ? 0.f : M;
  float L = 0.f, f[ATT_WAVES];
#pragma unroll
  for (int x = 0; x < ATT_WAVES; ++x) {
    f[x] = att_exp2(mrg[x * MS + lane] - Ms);
    L = __builtin_fmaf(mrg[x * MS + 64 + lane], f[x], L);
  }
  const float rinv = L > 0.f ? 1.f / (L * (1.f - a.p)) : 0.f;
  constexpr int DPW = DHP / ATT_WAVES;
  float outv[DPW];
#pragma unroll
  for (int t = 0; t < DPW; ++t) {
    const int d = w * DPW + t;
    float sacc = 0.f;
#pragma unroll
    for (int x = 0; x < ATT_WAVES; ++x) sacc = __builtin_fmaf(mrg[x * MS + (d + 2) * 64 + lane], f[x], sacc);
    outv[t] = sacc * rinv;
  }
  if (w == 0 && lane < QPW && q0 + lane < a.Sq)
    lse2[(long long)bh * a.Sq + q0 + lane] = L > 0.f ? M + log2f(L) : INFINITY;
  __syncthreads();
  float *tile = sm + ATT_WAVES * MS;  // [64][DHP]
#pragma unroll
  for (int t = 0; t < DPW; ++t) tile[lane * DHP + w * DPW + t] = outv[t];
  __syncthreads();
  store_rows<DHP, QPW>(o + (long long)b * a.o_sb + h * a.dh, tile, q0, a.Sq, a.o_ss, a.dh);
}

template <int DHP, int LPQ>
__global__ void __launch_bounds__(ATT_WAVES * 64) k_attn_bwd_q(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const float *__restrict__ o, const float *__restrict__ dout, const float *__restrict__ lse2,
    const uint8_t *__restrict__ kpad, const int *__restrict__ seed, AttnDims a,
    float *__restrict__ dq, float *__restrict__ Dbuf) {
  __shared__ __attribute__((aligned(16))) float sm[2 * ATT_SMAX * DHP];
  __shared__ float smask[ATT_SMAX];
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  constexpr int QPW = 64 / LPQ;
  const int q0 = blockIdx.x * QPW;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane & (LPQ - 1);
  float *sK = sm, *sV = sm + ATT_SMAX * DHP;
  const long long kvoff = (long long)b * a.kv_sb + h * a.dh;
  stage_rows<DHP>(sK, k + kvoff, a.Sk, a.kv_ss, a.dh);
  stage_rows<DHP>(sV, v + kvoff, a.Sk, a.kv_ss, a.dh);
  for (int j = threadIdx.x; j < a.Sk; j += ATT_WAVES * 64)
    smask[j] = (kpad && kpad[(long long)b * a.Sk + j]) ? -INFINITY : 0.f;
  const int i = q0 + lane / LPQ, ic = min(i, a.Sq - 1);
  float qr[DHP], dor[DHP];
  const float qmul = a.scale * LOG2E;
  const float *qrow = q + (long long)b * a.q_sb + h * a.dh + (long long)ic * a.q_ss;
  const long long orow = (long long)b * a.o_sb + h * a.dh + (long long)ic * a.o_ss;
  float orr[DHP];
  load_row<DHP>(qr, qrow, a.dh, qmul);
  load_row<DHP>(dor, dout + orow, a.dh, 1.f);
  load_row<DHP>(orr, o + orow, a.dh, 1.f);
  float Di = 0.f;
#pragma unroll
  for (int d = 0; d < DHP; ++d) Di = __builtin_fmaf(dor[d], orr[d], Di);
  const float li = lse2[(long long)bh * a.Sq + ic];
  __syncthreads();
  const uint32_t sm_ = att_seedmix(seed);
  const float rkeep = 1.f / (1.f - a.p);
  const int chunk = (a.Sk + ATT_WAVES - 1) / ATT_WAVES;
  const int j0 = w * chunk, j1 = min(a.Sk, j0 + chunk);
  float acc[DHP];
#pragma unroll
  for (int d = 0; d < DHP; ++d) acc[d] = 0.f;
  const uint32_t cbase = ((uint32_t)bh * a.Sq + i) * a.Sk;
  for (int j = j0 + sub; j < j1; j += LPQ) {
    const float s = dot_lds<DHP>(qr, sK + j * DHP) + smask[j];
    const float pj = (a.causal && j > i) ? 0.f : att_exp2(s - li);
    const float dpd = dot_lds<DHP>(dor, sV + j * DHP);
    const float dp = (a.p > 0.f && !att_keep(sm_, cbase + j, a.p)) ? 0.f : dpd * rkeep;
    axpy_lds<DHP>(acc, pj * (dp - Di), sK + j * DHP);
  }
  if (LPQ > 1) lane_sum<LPQ, DHP>(acc);
  if (Dbuf && w == 0 && sub == 0 && i < a.Sq) Dbuf[(long long)bh * a.Sq + i] = Di;
  __syncthreads();
  constexpr int MS = DHP * 64;
  float *mrg = sm;  // [w][DHP][64], column = query within the block
  if (sub == 0) {
#pragma unroll
    for (int d = 0; d < DHP; ++d) mrg[w * MS + d * 64 + lane / LPQ] = acc[d];
  }
  __syncthreads();
  constexpr int DPW = DHP / ATT_WAVES;
  float outv[DPW];
#pragma unroll
  for (int t = 0; t < DPW; ++t) {
    const int d = w * DPW + t;
    float sacc = 0.f;
#pragma unroll
    for (int x = 0; x < ATT_WAVES; ++x) sacc += mrg[x * MS + d * 64 + lane];
    outv[t] = sacc * a.scale;
  }
  __syncthreads();
  float *tile = sm + ATT_WAVES * MS;
#pragma unroll
  for (int t = 0; t < DPW; ++t) tile[lane * DHP + w * DPW + t] = outv[t];
  __syncthreads();
  store_rows<DHP, QPW>(dq + (long long)b * a.q_sb + h * a.dh, tile, q0, a.Sq, a.q_ss, a.dh);
}

template <int DHP, int LPK>
__global__ void __launch_bounds__(ATT_WAVES * 64) k_attn_bwd_kv(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const float *__restrict__ dout, const float *__restrict__ lse2, const float *__restrict__ Dbuf,
    const uint8_t *__restrict__ kpad, const int *__restrict__ seed, AttnDims a,
    float *__restrict__ dk, float *__restrict__ dv) {
  // staging [Sq][DHP] x 2 and the merge [w][2*DHP][64] share one buffer
  constexpr int SMF = (2 * ATT_SMAX * DHP > ATT_WAVES * 128 * DHP) ? 2 * ATT_SMAX * DHP
                                                                   : ATT_WAVES * 128 * DHP;
  __shared__ __attribute__((aligned(16))) float sm[SMF];
  __shared__ float slse[ATT_SMAX], sD[ATT_SMAX];
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  constexpr int KPW = 64 / LPK;  // keys per block; LPK lanes share a key's queries
  const int k0 = blockIdx.x * KPW;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane & (LPK - 1);
  float *sQ = sm, *sO = sm + ATT_SMAX * DHP;
  stage_rows<DHP>(sQ, q + (long long)b * a.q_sb + h * a.dh, a.Sq, a.q_ss, a.dh);
  stage_rows<DHP>(sO, dout + (long long)b * a.o_sb + h * a.dh, a.Sq, a.o_ss, a.dh);
  for (int t = threadIdx.x; t < a.Sq; t += ATT_WAVES * 64) {
    slse[t] = lse2[(long long)bh * a.Sq + t];
    sD[t] = Dbuf[(long long)bh * a.Sq + t];
  }
  const int j = k0 + lane / LPK, jc = min(j, a.Sk - 1);
  const bool kmasked = kpad && kpad[(long long)b * a.Sk + jc];
  const long long krow = (long long)b * a.kv_sb + h * a.dh + (long long)jc * a.kv_ss;
  float kr[DHP], vr[DHP], adk[DHP], adv[DHP];
  const float kmul = a.scale * LOG2E;
  load_row<DHP>(kr, k + krow, a.dh, kmul);
  load_row<DHP>(vr, v + krow, a.dh, 1.f);
#pragma unroll
  for (int d = 0; d < DHP; ++d) {
    adk[d] = 0.f;
    adv[d] = 0.f;
  }
  __syncthreads();
  const uint32_t sm_ = att_seedmix(seed);
  const float rkeep = 1.f / (1.f - a.p);
  const int chunk = (a.Sq + ATT_WAVES - 1) / ATT_WAVES;
  const int i0 = w * chunk, i1 = min(a.Sq, i0 + chunk);
  for (int i = i0 + sub; i < i1; i += LPK) {
    const float s = dot_lds<DHP>(kr, sQ + i * DHP);
    const bool masked = kmasked || (a.causal && j > i);
    const float pj = masked ? 0.f : att_exp2(s - slse[i]);
    const bool keep = !(a.p > 0.f) || att_keep(sm_, ((uint32_t)bh * a.Sq + i) * a.Sk + j, a.p);
    const float pd = keep ? pj * rkeep : 0.f;
    const float dpd = dot_lds<DHP>(vr, sO + i * DHP);
    const float ds = pj * ((keep ? dpd * rkeep : 0.f) - sD[i]);
    axpy_lds<DHP>(adv, pd, sO + i * DHP);
    axpy_lds<DHP>(adk, ds, sQ + i * DHP);
  }
  if (LPK > 1) {
    lane_sum<LPK, DHP>(adk);
    lane_sum<LPK, DHP>(adv);
  }
  __syncthreads();
  constexpr int MS = 2 * DHP * 64;
  float *mrg = sm;  // [w][2*DHP][64], column = key within the block
  if (sub == 0) {
    const int c = lane / LPK;
#pragma unroll
    for (int d = 0; d < DHP; ++d) {
      mrg[w * MS + d * 64 + c] = adk[d];
      mrg[w * MS + (DHP + d) * 64 + c] = adv[d];
    }
  }
  __syncthreads();
  // wave w reduces columns [w*2*DHP/4, ...) of the 2*DHP (dk | dv) columns
  constexpr int CPW = 2 * DHP / ATT_WAVES;
  float outv[CPW];
#pragma unroll
  for (int t = 0; t < CPW; ++t) {
    const int c = w * CPW + t;
    float sacc = 0.f;
#pragma unroll
    for (int x = 0; x < ATT_WAVES; ++x) sacc += mrg[x * MS + c * 64 + lane];
    outv[t] = c < DHP ? sacc * a.scale : sacc;
  }
  __syncthreads();
  float *tile = sm;  // [64][2*DHP]: dk | dv
#pragma unroll
  for (int t = 0; t < CPW; ++t) tile[lane * 2 * DHP + w * CPW + t] = outv[t];
  __syncthreads();
  const int nr = min(KPW, a.Sk - k0);
  const long long base = (long long)b * a.kv_sb + h * a.dh;
  for (int e = threadIdx.x; e < nr * a.dh; e += ATT_WAVES * 64) {
    const int r = e / a.dh, d = e - r * a.dh;
    const long long off = base + (long long)(k0 + r) * a.kv_ss + d;
    dk[off] = tile[r * 2 * DHP + d];
    dv[off] = tile[r * 2 * DHP + DHP + d];
  }
}

// keep mask as bytes [BH][Sq][Sk] (test/diagnostic entry)
__global__ void k_attn_keep_mask(const int *seed, int BH, int Sq, int Sk, float p, uint8_t *out) {
  const long long n = (long long)BH * Sq * Sk;
  const uint32_t sm_ = att_seedmix(seed);
  for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < n;
       c += (long long)gridDim.x * blockDim.x)
    out[c] = att_keep(sm_, (uint32_t)c, p) ? 1 : 0;
}

static int attn_check(const AttnDims &a, const char *who) {
  E2EP_REQUIRE(a.B > 0 && a.H > 0 && a.Sq > 0 && a.Sk > 0 && a.dh > 0, E2EP_EINVAL, "%s: bad shape", who);
  E2EP_REQUIRE(a.Sq <= ATT_SMAX && a.Sk <= ATT_SMAX && a.dh <= 64, E2EP_ERANGE,
               "%s: Sq %d / Sk %d (max %d) or head dim %d (max 64) unsupported", who, a.Sq, a.Sk,
               ATT_SMAX, a.dh);
  E2EP_REQUIRE(a.p >= 0.f && a.p < 1.f, E2EP_EINVAL, "%s: dropout p %g outside [0, 1)", who, a.p);
  E2EP_REQUIRE((long long)a.B * a.H * a.Sq * a.Sk < 0xffffffffLL, E2EP_ERANGE,
               "%s: dropout counter space exceeds 32 bits", who);
  return 0;
}

static AttnDims make_dims(int B, int H, int Sq, int Sk, int dh, int q_ss, int q_sb, int kv_ss,
                          int kv_sb, int o_ss, int o_sb, float scale, int causal, float p) {
  AttnDims a;
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.dh = dh;
  a.q_ss = q_ss; a.q_sb = q_sb; a.kv_ss = kv_ss; a.kv_sb = kv_sb; a.o_ss = o_ss; a.o_sb = o_sb;
  a.scale = scale; a.p = p; a.causal = causal;
  return a;
}

// ------------------------------------------------------------------------------------------
// Feed-forward activation of the transformer layers: dropout_p(relu(x)) and its backward
// (reference: linear1 -> relu -> dropout inside TransformerEncoderLayer/DecoderLayer._ff_block,
// model/feature_fusion.py:13-14, model/control_predict.py:19-20).  One launch each way instead
// of clamp + RNG fill + dropout (fwd) and dropout-mask scale + threshold (bwd).  The keep bit
// of element c is att_keep(seed, c): the same hash as the attention dropout, regenerated in
// the backward.  float4 per thread.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_relu_drop_fwd(const float4 *__restrict__ x, long long n4,
                                                       float p, const int *__restrict__ seed,
                                                       float4 *__restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const uint32_t sm_ = att_seedmix(seed);
  const float sc = 1.f / (1.f - p);
  const float4 v = x[i];
  const uint32_t c = (uint32_t)(4 * i);
  float4 o;
  o.x = (p > 0.f && !att_keep(sm_, c, p)) ? 0.f : fmaxf(v.x, 0.f) * sc;
  o.y = (p > 0.f && !att_keep(sm_, c + 1, p)) ? 0.f : fmaxf(v.y, 0.f) * sc;
  o.z = (p > 0.f && !att_keep(sm_, c + 2, p)) ? 0.f : fmaxf(v.z, 0.f) * sc;
  o.w = (p > 0.f && !att_keep(sm_, c + 3, p)) ? 0.f : fmaxf(v.w, 0.f) * sc;
  y[i] = o;
}

__global__ void __launch_bounds__(256) k_relu_drop_bwd(const float4 *__restrict__ x,
                                                       const float4 *__restrict__ dy, long long n4,
                                                       float p, const int *__restrict__ seed,
                                                       float4 *__restrict__ dx) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const uint32_t sm_ = att_seedmix(seed);
  const float sc = 1.f / (1.f - p);
  const float4 v = x[i], g = dy[i];
  const uint32_t c = (uint32_t)(4 * i);
  float4 o;
  o.x = (v.x > 0.f && !(p > 0.f && !att_keep(sm_, c, p))) ? g.x * sc : 0.f;
  o.y = (v.y > 0.f && !(p > 0.f && !att_keep(sm_, c + 1, p))) ? g.y * sc : 0.f;
  o.z = (v.z > 0.f && !(p > 0.f && !att_keep(sm_, c + 2, p))) ? g.z * sc : 0.f;
  o.w = (v.w > 0.f && !(p > 0.f && !att_keep(sm_, c + 3, p))) ? g.w * sc : 0.f;
  dx[i] = o;
}

static int relu_drop_check(const void *x, long long n, float p, const int32_t *seed, const char *who) {
  E2EP_REQUIRE(n > 0 && n % 4 == 0 && n < 0xffffffffLL, E2EP_EINVAL,
               "%s: n = %lld must be a positive multiple of 4 below 2^32", who, n);
  E2EP_REQUIRE(((uintptr_t)x & 15) == 0, E2EP_EINVAL, "%s: tensors must be 16-B aligned", who);
  E2EP_REQUIRE(p >= 0.f && p < 1.f && (p == 0.f || seed), E2EP_EINVAL, "%s: bad dropout p / seed", who);
  return 0;
}

}  // namespace e2ep

using namespace e2ep;

// D_i = dO_i . O_i per (batch*head, query), the same fma chain as k_attn_bwd_q computes for
// its own rows, so k_attn_bwd_kv can start without waiting for k_attn_bwd_q
template <int DHP>
__global__ void __launch_bounds__(256) k_attn_bwd_d(const float *__restrict__ o,
                                                    const float *__restrict__ dout, AttnDims a,
                                                    float *__restrict__ Dbuf) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= a.B * a.H * a.Sq) return;
  const int bh = t / a.Sq, i = t - bh * a.Sq, b = bh / a.H, h = bh - b * a.H;
  const long long orow = (long long)b * a.o_sb + h * a.dh + (long long)i * a.o_ss;
  float dor[DHP], orr[DHP];
  load_row<DHP>(dor, dout + orow, a.dh, 1.f);
  load_row<DHP>(orr, o + orow, a.dh, 1.f);
  float Di = 0.f;
#pragma unroll
  for (int d = 0; d < DHP; ++d) Di = __builtin_fmaf(dor[d], orr[d], Di);
  Dbuf[t] = Di;
}

extern "C" {

int e2ep_attn_fwd(const float *q, const float *k, const float *v, int B, int H, int Sq, int Sk,
                  int dh, int q_ss, int q_sb, int kv_ss, int kv_sb, int o_ss, int o_sb,
                  float scale, int causal, const uint8_t *key_pad, float p, const int32_t *seed,
                  float *o, float *lse, void *stream) {
  const AttnDims a = make_dims(B, H, Sq, Sk, dh, q_ss, q_sb, kv_ss, kv_sb, o_ss, o_sb, scale, causal, p);
  if (int rc = attn_check(a, "e2ep_attn_fwd")) return rc;
  E2EP_REQUIRE(p == 0.f || seed, E2EP_EINVAL, "e2ep_attn_fwd: dropout needs a seed");
  hipStream_t st = as_stream(stream);
  if (attn_mf_ok(a, key_pad)) {  // the fusion encoder's 256-token self-attention (attn_mf.hip)
    attn_mf_fwd(q, k, v, seed, a, o, lse, st);
    return launch_status("e2ep_attn_fwd");
  }
  const dim3 blk(ATT_WAVES * 64);
  // short query sequences (the control decoder's 14 tokens): 4 lanes per query
#define E2EP_ATT_FWD(DHP, LPQ)                                                                   \
  hipLaunchKernelGGL((k_attn_fwd<DHP, LPQ>), dim3(cdiv(Sq, 64 / LPQ), B * H), blk, 0, st, q, k, v, \
                     key_pad, seed, a, o, lse)
  if (dh <= 44) {
    if (Sq <= 16 || att_lanes() == 4) E2EP_ATT_FWD(44, 4); else if (att_lanes() == 2) E2EP_ATT_FWD(44, 2); else E2EP_ATT_FWD(44, 1);
  } else {
    if (Sq <= 16 || att_lanes() == 4) E2EP_ATT_FWD(64, 4); else if (att_lanes() == 2) E2EP_ATT_FWD(64, 2); else E2EP_ATT_FWD(64, 1);
  }
#undef E2EP_ATT_FWD
  return launch_status("e2ep_attn_fwd");
}

size_t e2ep_attn_bwd_workspace(int B, int H, int Sq) { return (size_t)B * H * Sq * sizeof(float); }

int e2ep_attn_bwd_part(const float *q, const float *k, const float *v, const float *o,
                       const float *dout, const float *lse, int B, int H, int Sq, int Sk, int dh,
                       int q_ss, int q_sb, int kv_ss, int kv_sb, int o_ss, int o_sb, float scale,
                       int causal, const uint8_t *key_pad, float p, const int32_t *seed, float *dq,
                       float *dk, float *dv, void *workspace, int part, void *stream) {
  E2EP_REQUIRE(part >= 0 && part <= 3, E2EP_EINVAL, "e2ep_attn_bwd_part: part must be 0..3");
  const AttnDims a = make_dims(B, H, Sq, Sk, dh, q_ss, q_sb, kv_ss, kv_sb, o_ss, o_sb, scale, causal, p);
  if (int rc = attn_check(a, "e2ep_attn_bwd")) return rc;
  E2EP_REQUIRE(p == 0.f || seed, E2EP_EINVAL, "e2ep_attn_bwd: dropout needs a seed");
  float *D = static_cast<float *>(workspace);
  hipStream_t s = as_stream(stream);
  const dim3 blk(ATT_WAVES * 64);
#define E2EP_ATT_BQ(DHP, LPQ, DB)                                                                \
  hipLaunchKernelGGL((k_attn_bwd_q<DHP, LPQ>), dim3(cdiv(Sq, 64 / LPQ), B * H), blk, 0, s, q, k, v, \
                     o, dout, lse, key_pad, seed, a, dq, DB)
#define E2EP_ATT_BKV(DHP, LPK)                                                                   \
  hipLaunchKernelGGL((k_attn_bwd_kv<DHP, LPK>), dim3(cdiv(Sk, 64 / LPK), B * H), blk, 0, s, q, k, \
                     v, dout, lse, D, key_pad, seed, a, dk, dv)
  // part 0: everything in order; 1: D only; 2: dq only (D already in the workspace); 3: dk, dv
  // only (likewise) — parts 2 and 3 are independent and may run on two streams
  if (part == 1) {
    if (dh <= 44)
      hipLaunchKernelGGL(k_attn_bwd_d<44>, dim3(cdiv(B * H * Sq, 256)), dim3(256), 0, s, o, dout, a, D);
    else
      hipLaunchKernelGGL(k_attn_bwd_d<64>, dim3(cdiv(B * H * Sq, 256)), dim3(256), 0, s, o, dout, a, D);
    return launch_status("e2ep_attn_bwd");
  }
  float *Dq = part == 2 ? nullptr : D;  // dq pass alone: D is read by the other pass, not rewritten
  if (attn_mf_ok(a, key_pad)) {  // matrix-core dq (+ D) (attn_mf.hip); dk / dv below or there
    if (attn_mf_bwd(q, k, v, o, dout, lse, seed, a, dq, dk, dv, D, part, s) || part == 2)
      return launch_status("e2ep_attn_bwd");
    part = 3;  // dk / dv on the vector-FMA kernel (faster at this shape), reading D
  }
  if (part != 3) {
    if (dh <= 44) {
      if (Sq <= 16 || att_lanes() == 4) E2EP_ATT_BQ(44, 4, Dq); else if (att_lanes() == 2) E2EP_ATT_BQ(44, 2, Dq); else E2EP_ATT_BQ(44, 1, Dq);
    } else {
      if (Sq <= 16 || att_lanes() == 4) E2EP_ATT_BQ(64, 4, Dq); else if (att_lanes() == 2) E2EP_ATT_BQ(64, 2, Dq); else E2EP_ATT_BQ(64, 1, Dq);
    }
  }
  if (part != 2) {
    if (dh <= 44) {
      if (Sk <= 16 || att_lanes() == 4) E2EP_ATT_BKV(44, 4); else if (att_lanes() == 2) E2EP_ATT_BKV(44, 2); else E2EP_ATT_BKV(44, 1);
    } else {
      if (Sk <= 16 || att_lanes() == 4) E2EP_ATT_BKV(64, 4); else if (att_lanes() == 2) E2EP_ATT_BKV(64, 2); else E2EP_ATT_BKV(64, 1);
    }
  }
#undef E2EP_ATT_BQ
#undef E2EP_ATT_BKV
  return launch_status("e2ep_attn_bwd");
}

int e2ep_attn_bwd(const float *q, const float *k, const float *v, const float *o, const float *dout,
                  const float *lse, int B, int H, int Sq, int Sk, int dh, int q_ss, int q_sb,
                  int kv_ss, int kv_sb, int o_ss, int o_sb, float scale, int causal,
                  const uint8_t *key_pad, float p, const int32_t *seed, float *dq, float *dk,
                  float *dv, void *workspace, void *stream) {
  return e2ep_attn_bwd_part(q, k, v, o, dout, lse, B, H, Sq, Sk, dh, q_ss, q_sb, kv_ss, kv_sb, o_ss,
                            o_sb, scale, causal, key_pad, p, seed, dq, dk, dv, workspace, 0, stream);
}

int e2ep_attn_keep_mask(const int32_t *seed, int BH, int Sq, int Sk, float p, uint8_t *out,
                        void *stream) {
  E2EP_REQUIRE(seed && BH > 0 && Sq > 0 && Sk > 0, E2EP_EINVAL, "e2ep_attn_keep_mask: bad args");
  const long long n = (long long)BH * Sq * Sk;
  hipLaunchKernelGGL(k_attn_keep_mask, dim3(min(cdiv(n, 256), 4096)), dim3(256), 0, as_stream(stream),
                     seed, BH, Sq, Sk, p, out);
  return launch_status("e2ep_attn_keep_mask");
}

int e2ep_relu_dropout_fwd(const float *x, long long n, float p, const int32_t *seed, float *y,
                          void *stream) {
  if (int rc = relu_drop_check(x, n, p, seed, "e2ep_relu_dropout_fwd")) return rc;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_relu_drop_fwd, dim3(cdiv(n4, 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4 *>(x), n4, p, seed, reinterpret_cast<float4 *>(y));
  return launch_status("e2ep_relu_dropout_fwd");
}

int e2ep_relu_dropout_bwd(const float *x, const float *dy, long long n, float p,
                          const int32_t *seed, float *dx, void *stream) {
  if (int rc = relu_drop_check(x, n, p, seed, "e2ep_relu_dropout_bwd")) return rc;
  E2EP_REQUIRE((((uintptr_t)dy | (uintptr_t)dx) & 15) == 0, E2EP_EINVAL,
               "e2ep_relu_dropout_bwd: tensors must be 16-B aligned");
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_relu_drop_bwd, dim3(cdiv(n4, 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4 *>(x), reinterpret_cast<const float4 *>(dy), n4, p,
                     seed, reinterpret_cast<float4 *>(dx));
  return launch_status("e2ep_relu_dropout_bwd");
}

}  // extern "C"
