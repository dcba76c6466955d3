// Matrix-core attention for the fusion encoder (reference model/feature_fusion.py:13-14,48-50:
// nn.TransformerEncoder self-attention, Sq = Sk = 256 BEV tokens, 6 heads x dh 43, dropout),
// forward and backward on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32: products and sums in
// fp32, as the vector-FMA kernels of attn.hip).
//
// attn.hip's kernels put one query (or key) per lane and read every K / V row from LDS as a
// wave-wide broadcast: ~5 600 ds_read_b128 per wave for a 64-query tile, which, not the FMAs,
// bound them (42 us forward, 58 / 38 us for the two backward passes per encoder layer at B = 8).
// Here the dot products are 32 x 32 MFMA tiles:
//   S = Q K^T   (K dimension = the head dim, 22 MFMAs per 32 x 32 tile)
//   O = P V     (K dimension = keys; P goes through LDS from the C/D layout to the A layout)
// A lane's MFMA operands are runs of a row: MFMA t of a head-dim product takes d = t from lane
// half 0 and d = 22 + t from lane half 1 (dh <= 44), MFMA t of a key / query product takes
// index t and 32 + t of the wave's 64; every sum is in a fixed order (run-to-run deterministic).
//
//   k_attn_fwd_mf   block = (32 queries, b*h), 4 waves split the keys; per wave a row max /
//                   row sum over its keys, P (dropped) -> LDS -> P V; the 4 partial (m, l, O)
//                   merged in wave order; O and lse2 = m + log2(l) (log2 domain) as attn.hip
//   k_attn_bq_mf    block = (32 queries, b*h), waves split the keys: P = exp2(S - lse2),
//                   dP = dO V^T, dS = P (drop(dP) - D), dQ = scale dS K; D_i = dO_i . O_i with
//                   the d-ordered fma chain of attn.hip's k_attn_bwd_d (written to the workspace
//                   for the dk / dv pass)
//   k_attn_bkv_mf   block = (32 keys, b*h), waves split the queries: the transposed tiles
//                   S^T = K Q^T and dP^T = V dO^T, dV = drop(P)^T dO, dK = scale dS^T Q
// Dropout: keep(bh, i, j) = att_keep(seedmix, (bh*Sq + i)*Sk + j, p) (dropout.h), the counter
// space of attn.hip, so masks, lse and D are interchangeable between the two kernel families.
#include "attn.h"
#include "dropout.h"

namespace e2ep {

typedef float mf16 __attribute__((ext_vector_type(16)));
constexpr int MF_T = 22;          // head-dim MFMAs (dh <= 44)
constexpr int MF_LD = 68;         // LDS row stride of the 32 x 64 tiles (b128 reads conflict-free)
constexpr float MF_LOG2E = 1.4426950408889634f;

__device__ __forceinline__ mf16 mf_mma(float a, float b, mf16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// row of the C/D layout for register r of lane half h (column = lane & 31)
__device__ __forceinline__ int mf_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// lane half h's run of a head row: d = 22 h + t (zero beyond dh), times mul
__device__ __forceinline__ void mf_half(float (&x)[MF_T], const float *row, int dh, int h, float mul) {
#pragma unroll
  for (int t = 0; t < MF_T; ++t) {
    const int d = MF_T * h + t;
    x[t] = row[min(d, dh - 1)] * (d < dh ? mul : 0.f);
  }
}

// One wave stages a 32-row x dh tile of a (S, B, E)-strided head matrix into its LDS buffer
// [32][MF_RS] (coalesced: consecutive lanes on consecutive d), scaled and zero padded to 44;
// lanes then read their half-row runs from LDS (per-lane global row reads, 64 rows per
// instruction, measured slower).  MF_RS = 45: odd stride, the 32 rows' ds_read_b32 hit 32
// distinct banks.
constexpr int MF_RS = 45;
__device__ __forceinline__ void mf_wsync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void mf_stage32(float *tile, const float *row0, long long ss, int dh,
                                           float mul, int lane) {
  mf_wsync();  // the previous reads of the buffer are done
#pragma unroll 2
  for (int e = lane; e < 32 * 2 * MF_T; e += 64) {
    const int r = e / (2 * MF_T), d = e - r * (2 * MF_T);
    tile[r * MF_RS + d] = row0[(long long)r * ss + min(d, dh - 1)] * (d < dh ? mul : 0.f);
  }
  mf_wsync();
}
__device__ __forceinline__ void mf_half_lds(float (&x)[MF_T], const float *tile, int li, int h) {
#pragma unroll
  for (int t = 0; t < MF_T; ++t) x[t] = tile[li * MF_RS + MF_T * h + t];
}

// max / sum over the 32 lanes of a lane half (the 32 columns of a C/D tile)
__device__ __forceinline__ float mf_hmax(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ float mf_hsum(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// acc[dt] += A(32 rows x 64 k, LDS rows at `tile`, k-permuted: MFMA t takes k = t (half 0) and
// 32 + t (half 1)) x B(64 k x 32 cols): B(k, c) = rowsB[k][32 dt + c] from global rows
// `brow0 + k * bss` (columns >= dh read as 0).  nrows = 32: the A columns 32.. are zero and the
// B rows past the tile are not read (row index clamped).
__device__ __forceinline__ void mf_tile_times_rows(mf16 (&acc)[2], const float *tile, int li, int lh,
                                                   const float *brow0, long long bss, int dh,
                                                   int nrows) {
  float a[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = *reinterpret_cast<const float4 *>(tile + li * MF_LD + 32 * lh + 4 * q);
    a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const int d = 32 * dt + li;
    const float keep = d < dh ? 1.f : 0.f;
    const float *col = brow0 + min(d, dh - 1);
    float bv[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) bv[t] = col[(long long)min(t + 32 * lh, nrows - 1) * bss] * keep;
#pragma unroll
    for (int t = 0; t < 32; ++t) acc[dt] = mf_mma(a[t], bv[t], acc[dt]);
  }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <int NT>  // key tiles of 32 per wave: Sk = 128 NT
__global__ void __launch_bounds__(256) k_attn_fwd_mf(const float *__restrict__ q,
                                                     const float *__restrict__ k,
                                                     const float *__restrict__ v,
                                                     const int *__restrict__ seed, AttnDims a,
                                                     float *__restrict__ o,
                                                     float *__restrict__ lse2) {
  __shared__ __attribute__((aligned(16))) float sT[4][32][MF_LD];  // P tiles, then O partials
  __shared__ float sM[4][32], sL[4][32];
  __shared__ float sR[4][32 * MF_RS];  // per-wave row staging
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.x * 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const long long qoff = (long long)b * a.q_sb + h * a.dh, kvoff = (long long)b * a.kv_sb + h * a.dh;
  const int kw0 = w * 32 * NT;  // this wave's keys
  const uint32_t smx = att_seedmix(seed);
  float *stg = sR[w];

  float qa[MF_T];
  mf_stage32(stg, q + qoff + (long long)q0 * a.q_ss, a.q_ss, a.dh, a.scale * MF_LOG2E, lane);
  mf_half_lds(qa, stg, li, lh);
  mf16 s[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    float kb[MF_T];
    mf_stage32(stg, k + kvoff + (long long)(kw0 + 32 * kt) * a.kv_ss, a.kv_ss, a.dh, 1.f, lane);
    mf_half_lds(kb, stg, li, lh);
    s[kt] = mf16{0};
#pragma unroll
    for (int t = 0; t < MF_T; ++t) s[kt] = mf_mma(qa[t], kb[t], s[kt]);
  }
  // row max / sum over this wave's keys (rows = queries, spread over the 16 registers)
  float m[16], l[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float x = s[0][r];
#pragma unroll
    for (int kt = 1; kt < NT; ++kt) x = fmaxf(x, s[kt][r]);
    m[r] = mf_hmax(x);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = q0 + mf_row(r, lh);
    float x = 0.f;
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      const float pu = __builtin_amdgcn_exp2f(s[kt][r] - m[r]);
      x += pu;
      const int j = kw0 + 32 * kt + li;
      const bool kp = a.p <= 0.f || att_keep(smx, ((uint32_t)bh * a.Sq + i) * a.Sk + j, a.p);
      sT[w][mf_row(r, lh)][32 * kt + li] = kp ? pu : 0.f;
    }
    l[r] = mf_hsum(x);
  }
  if (NT == 1) {  // a single key tile: the second half of the 64-key row is zero
#pragma unroll
    for (int r = 0; r < 16; ++r) sT[w][mf_row(r, lh)][32 + li] = 0.f;
  }
  __syncthreads();
  mf16 oc[2] = {mf16{0}, mf16{0}};
  mf_tile_times_rows(oc, &sT[w][0][0], li, lh, v + kvoff + (long long)kw0 * a.kv_ss, a.kv_ss, a.dh,
                     32 * NT);
  __syncthreads();  // P tiles consumed: reuse sT for the O partials
  if (li == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sM[w][mf_row(r, lh)] = m[r];
      sL[w][mf_row(r, lh)] = l[r];
    }
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) sT[w][mf_row(r, lh)][32 * dt + li] = oc[dt][r];
  __syncthreads();
  // merge the 4 waves in order: element (query i, dim d)
  for (int e = threadIdx.x; e < 32 * a.dh; e += 256) {
    const int i = e / a.dh, d = e - i * a.dh;
    float M = sM[0][i];
#pragma unroll
    for (int x = 1; x < 4; ++x) M = fmaxf(M, sM[x][i]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const float f = __builtin_amdgcn_exp2f(sM[x][i] - M);
      L = __builtin_fmaf(sL[x][i], f, L);
      O = __builtin_fmaf(sT[x][i][d], f, O);
    }
    o[(long long)b * a.o_sb + h * a.dh + (long long)(q0 + i) * a.o_ss + d] = O / (L * (1.f - a.p));
    if (d == 0) lse2[(long long)bh * a.Sq + q0 + i] = M + log2f(L);
  }
}

// ------------------------------------------------------------------------------------------
// backward, dq (and D)
// ------------------------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(256) k_attn_bq_mf(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const float *__restrict__ o, const float *__restrict__ dout, const float *__restrict__ lse2,
    const int *__restrict__ seed, AttnDims a, float *__restrict__ dq, float *__restrict__ Dbuf) {
  __shared__ __attribute__((aligned(16))) float sT[4][32][MF_LD];  // dS tiles, then dQ partials
  __shared__ float sD[32];
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.x * 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const long long qoff = (long long)b * a.q_sb + h * a.dh, kvoff = (long long)b * a.kv_sb + h * a.dh;
  const long long ooff = (long long)b * a.o_sb + h * a.dh;
  const int kw0 = w * 32 * NT;
  const uint32_t smx = att_seedmix(seed);
  // D_i = dO_i . O_i, d-ordered fma chain (k_attn_bwd_d's), by wave 0's lane half 0
  if (w == 0 && lh == 0) {
    const float *dor = dout + ooff + (long long)(q0 + li) * a.o_ss;
    const float *orr = o + ooff + (long long)(q0 + li) * a.o_ss;
    float Di = 0.f;
    for (int d = 0; d < a.dh; ++d) Di = __builtin_fmaf(dor[d], orr[d], Di);
    sD[li] = Di;
    if (Dbuf) Dbuf[(long long)bh * a.Sq + q0 + li] = Di;
  }
  float qa[MF_T], da[MF_T];
  mf_half(qa, q + qoff + (long long)(q0 + li) * a.q_ss, a.dh, lh, a.scale * MF_LOG2E);
  mf_half(da, dout + ooff + (long long)(q0 + li) * a.o_ss, a.dh, lh, 1.f);
  float lse[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) lse[r] = lse2[(long long)bh * a.Sq + q0 + mf_row(r, lh)];
  __syncthreads();  // sD
  const float inv_keep = 1.f / (1.f - a.p);
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    const int j0 = kw0 + 32 * kt;
    float kb[MF_T], vb[MF_T];
    mf_half(kb, k + kvoff + (long long)(j0 + li) * a.kv_ss, a.dh, lh, 1.f);
    mf_half(vb, v + kvoff + (long long)(j0 + li) * a.kv_ss, a.dh, lh, 1.f);
    mf16 s = mf16{0}, dp = mf16{0};
#pragma unroll
    for (int t = 0; t < MF_T; ++t) {
      s = mf_mma(qa[t], kb[t], s);
      dp = mf_mma(da[t], vb[t], dp);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = q0 + mf_row(r, lh), j = j0 + li;
      const float P = __builtin_amdgcn_exp2f(s[r] - lse[r]);
      const bool kp = a.p <= 0.f || att_keep(smx, ((uint32_t)bh * a.Sq + i) * a.Sk + j, a.p);
      const float dpd = kp ? dp[r] * inv_keep : 0.f;
      sT[w][mf_row(r, lh)][32 * kt + li] = P * (dpd - sD[mf_row(r, lh)]);
    }
  }
  if (NT == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sT[w][mf_row(r, lh)][32 + li] = 0.f;
  }
  __syncthreads();
  mf16 acc[2] = {mf16{0}, mf16{0}};
  mf_tile_times_rows(acc, &sT[w][0][0], li, lh, k + kvoff + (long long)kw0 * a.kv_ss, a.kv_ss, a.dh,
                     32 * NT);
  __syncthreads();
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) sT[w][mf_row(r, lh)][32 * dt + li] = acc[dt][r];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * a.dh; e += 256) {
    const int i = e / a.dh, d = e - i * a.dh;
    const float g = (sT[0][i][d] + sT[1][i][d]) + (sT[2][i][d] + sT[3][i][d]);
    dq[qoff + (long long)(q0 + i) * a.q_ss + d] = g * a.scale;
  }
}

// ------------------------------------------------------------------------------------------
// backward, dk and dv
// ------------------------------------------------------------------------------------------
template <int NT>  // query tiles of 32 per wave: Sq = 128 NT
__global__ void __launch_bounds__(256) k_attn_bkv_mf(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const float *__restrict__ dout, const float *__restrict__ lse2, const float *__restrict__ Dbuf,
    const int *__restrict__ seed, AttnDims a, float *__restrict__ dk, float *__restrict__ dv) {
  __shared__ __attribute__((aligned(16))) float sP[4][32][MF_LD];  // drop(P)^T, then dV partials
  __shared__ __attribute__((aligned(16))) float sS[4][32][MF_LD];  // dS^T, then dK partials
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int k0 = blockIdx.x * 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const long long qoff = (long long)b * a.q_sb + h * a.dh, kvoff = (long long)b * a.kv_sb + h * a.dh;
  const long long ooff = (long long)b * a.o_sb + h * a.dh;
  const int iw0 = w * 32 * NT;  // this wave's queries
  const uint32_t smx = att_seedmix(seed);
  float ka[MF_T], va[MF_T];
  mf_half(ka, k + kvoff + (long long)(k0 + li) * a.kv_ss, a.dh, lh, a.scale * MF_LOG2E);
  mf_half(va, v + kvoff + (long long)(k0 + li) * a.kv_ss, a.dh, lh, 1.f);
  const float inv_keep = 1.f / (1.f - a.p);
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) {
    const int i0 = iw0 + 32 * qt, i = i0 + li;  // this lane's query (the tile's column)
    float qb[MF_T], db[MF_T];
    mf_half(qb, q + qoff + (long long)i * a.q_ss, a.dh, lh, 1.f);
    mf_half(db, dout + ooff + (long long)i * a.o_ss, a.dh, lh, 1.f);
    const float lse_i = lse2[(long long)bh * a.Sq + i], D_i = Dbuf[(long long)bh * a.Sq + i];
    mf16 st = mf16{0}, dpt = mf16{0};
#pragma unroll
    for (int t = 0; t < MF_T; ++t) {
      st = mf_mma(ka[t], qb[t], st);
      dpt = mf_mma(va[t], db[t], dpt);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = k0 + mf_row(r, lh);  // key (the tile's row)
      const float P = __builtin_amdgcn_exp2f(st[r] - lse_i);
      const bool kp = a.p <= 0.f || att_keep(smx, ((uint32_t)bh * a.Sq + i) * a.Sk + j, a.p);
      sP[w][mf_row(r, lh)][32 * qt + li] = kp ? P * inv_keep : 0.f;
      sS[w][mf_row(r, lh)][32 * qt + li] = P * ((kp ? dpt[r] * inv_keep : 0.f) - D_i);
    }
  }
  if (NT == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sP[w][mf_row(r, lh)][32 + li] = 0.f;
      sS[w][mf_row(r, lh)][32 + li] = 0.f;
    }
  }
  __syncthreads();
  mf16 gv[2] = {mf16{0}, mf16{0}}, gk[2] = {mf16{0}, mf16{0}};
  mf_tile_times_rows(gv, &sP[w][0][0], li, lh, dout + ooff + (long long)iw0 * a.o_ss, a.o_ss, a.dh,
                     32 * NT);
  mf_tile_times_rows(gk, &sS[w][0][0], li, lh, q + qoff + (long long)iw0 * a.q_ss, a.q_ss, a.dh,
                     32 * NT);
  __syncthreads();
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sP[w][mf_row(r, lh)][32 * dt + li] = gv[dt][r];
      sS[w][mf_row(r, lh)][32 * dt + li] = gk[dt][r];
    }
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * a.dh; e += 256) {
    const int j = e / a.dh, d = e - j * a.dh;
    const float gvs = (sP[0][j][d] + sP[1][j][d]) + (sP[2][j][d] + sP[3][j][d]);
    const float gks = (sS[0][j][d] + sS[1][j][d]) + (sS[2][j][d] + sS[3][j][d]);
    const long long off = kvoff + (long long)(k0 + j) * a.kv_ss + d;
    dv[off] = gvs;
    dk[off] = gks * a.scale;
  }
}

bool attn_mf_ok(const AttnDims &a, const uint8_t *key_pad) {
  if (g_tune[TUNE_ATT_MF] <= 1) return false;
  const bool s_ok = (a.Sq == 128 || a.Sq == 256) && (a.Sk == 128 || a.Sk == 256);
  return s_ok && a.dh <= 2 * MF_T && !a.causal && !key_pad;
}

void attn_mf_fwd(const float *q, const float *k, const float *v, const int *seed,
                 const AttnDims &a, float *o, float *lse2, hipStream_t s) {
  const dim3 grid(a.Sq / 32, a.B * a.H);
  if (a.Sk == 256)
    hipLaunchKernelGGL(k_attn_fwd_mf<2>, grid, dim3(256), 0, s, q, k, v, seed, a, o, lse2);
  else
    hipLaunchKernelGGL(k_attn_fwd_mf<1>, grid, dim3(256), 0, s, q, k, v, seed, a, o, lse2);
}

bool attn_mf_bwd(const float *q, const float *k, const float *v, const float *o,
                 const float *dout, const float *lse2, const int *seed, const AttnDims &a,
                 float *dq, float *dk, float *dv, float *Dbuf, int part, hipStream_t s) {
  if (part != 3) {
    const dim3 grid(a.Sq / 32, a.B * a.H);
    float *Dw = part == 0 ? Dbuf : nullptr;
    if (a.Sk == 256)
      hipLaunchKernelGGL(k_attn_bq_mf<2>, grid, dim3(256), 0, s, q, k, v, o, dout, lse2, seed, a, dq, Dw);
    else
      hipLaunchKernelGGL(k_attn_bq_mf<1>, grid, dim3(256), 0, s, q, k, v, o, dout, lse2, seed, a, dq, Dw);
  }
  if (part != 2 && g_tune[TUNE_ATT_MF] == 3) {  // dk / dv on the matrix cores only when asked
    const dim3 grid(a.Sk / 32, a.B * a.H);
    if (a.Sq == 256)
      hipLaunchKernelGGL(k_attn_bkv_mf<2>, grid, dim3(256), 0, s, q, k, v, dout, lse2, Dbuf, seed, a, dk, dv);
    else
      hipLaunchKernelGGL(k_attn_bkv_mf<1>, grid, dim3(256), 0, s, q, k, v, dout, lse2, Dbuf, seed, a, dk, dv);
  }
  return part != 2 && g_tune[TUNE_ATT_MF] == 3;
}

}  // namespace e2ep
