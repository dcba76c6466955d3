// Lift-splat kernels for gfx950: geometry + pillar index, counting-sort plan, fused
// outer-product/pillar-pool forward, gather backward, transpose, target channel.
//
// Reference behaviour (qintonguav/e2e-parking-carla):
//   model/bev_model.py:45-57   get_geometry        -> k_geom_index (bit-exact, fp32, no FMA)
//   model/bev_model.py:59-71   outer product       -> fused into k_lss_fwd (never materialised)
//   model/bev_model.py:74-107  proj_bev_feature    -> k_count/k_scan/k_fill/k_segsort + k_lss_fwd
//   tool/geometry.py:285-317   VoxelsSumming       -> k_lss_fwd (direct per-pillar sum) /
//                                                     k_lss_bwd (gather, no atomics)
//   model/parking_model.py:28-46 add_target_bev    -> k_target_bev
//
// HBM layout: prob [B*N][D][hw], featT [B*N][hw][C] (pixel-major, 256-B rows at C=64),
// bev [B][C..][X*Y] channel-major (the reference's output layout), gT [B][XY][C].
#include "common.h"

#pragma clang fp contract(off)

namespace e2ep {

// ------------------------------------------------------------------------------------------
// geometry + pillar index: one thread per frustum point
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_geom_index(
    const float *__restrict__ frustum, const float *__restrict__ combine,
    const float *__restrict__ trans, float lo0, float lo1, float lo2, float r0, float r1,
    float r2, int X, int Y, int Z, int DHW, long long total, int *__restrict__ pillar) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int bn = (int)(i / DHW);
  const int f = (int)(i - (long long)bn * DHW);
  const float u = frustum[3 * f + 0], v = frustum[3 * f + 1], d = frustum[3 * f + 2];
  // points = (u*d, v*d, d)                                   (bev_model.py:51-52)
  const float p0 = __fmul_rn(u, d), p1 = __fmul_rn(v, d), p2 = d;
  const float *c = combine + 9 * bn;
  const float *t = trans + 3 * bn;
  // combine @ p, accumulated in k order, then + translation  (bev_model.py:54-55)
  float xyz[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    float a = __fmul_rn(c[3 * r + 0], p0);
    a = __fadd_rn(a, __fmul_rn(c[3 * r + 1], p1));
    a = __fadd_rn(a, __fmul_rn(c[3 * r + 2], p2));
    xyz[r] = __fadd_rn(a, t[r]);
  }
  // ((xyz - lo) / res).long(), mask on all three dims      (bev_model.py:85-90)
  const float gx = truncf(__fdiv_rn(__fsub_rn(xyz[0], lo0), r0));
  const float gy = truncf(__fdiv_rn(__fsub_rn(xyz[1], lo1), r1));
  const float gz = truncf(__fdiv_rn(__fsub_rn(xyz[2], lo2), r2));
  const bool ok = gx >= 0.f && gx < (float)X && gy >= 0.f && gy < (float)Y && gz >= 0.f &&
                  gz < (float)Z;
  pillar[i] = ok ? ((int)gx * (Y * Z) + (int)gy * Z + (int)gz) : -1;
}

// ------------------------------------------------------------------------------------------
// plan: histogram -> exclusive scan -> fill -> per-pillar sort (deterministic order)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_count(const int *__restrict__ pillar, int P, int XYZ,
                                               long long total, int *__restrict__ counts) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int q = pillar[i];
  if (q >= 0) atomicAdd(&counts[(i / P) * XYZ + q], 1);
}

// one 1024-thread block per sample; offsets[b][0..XYZ] = exclusive scan of counts[b]
__global__ void __launch_bounds__(1024) k_scan(const int *__restrict__ counts, int XYZ,
                                               int *__restrict__ offsets,
                                               int *__restrict__ cursor) {
  __shared__ int part[1024];
  const int b = blockIdx.x, t = threadIdx.x;
  const int per = (XYZ + 1023) / 1024;
  const int beg = min(t * per, XYZ), end = min(beg + per, XYZ);
  const int *cnt = counts + (long long)b * XYZ;
  int s = 0;
  for (int i = beg; i < end; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - s;  // exclusive prefix of this thread's chunk
  int *off = offsets + (long long)b * (XYZ + 1);
  int *cur = cursor + (long long)b * XYZ;
  for (int i = beg; i < end; ++i) {
    off[i] = run;
    cur[i] = run;
    run += cnt[i];
  }
  if (t == 1023) off[XYZ] = part[1023];
}

__global__ void __launch_bounds__(256) k_fill(const int *__restrict__ pillar, int P, int DHW,
                                              int HW, int XYZ, long long total,
                                              int *__restrict__ cursor,
                                              int *__restrict__ order) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int q = pillar[i];
  if (q < 0) return;
  const long long b = i / P;
  const int local = (int)(i - b * P);
  const int n = local / DHW;
  const int rem = local - n * DHW;
  const int d = rem / HW;
  const int pix = rem - d * HW;
  const int slot = atomicAdd(&cursor[b * XYZ + q], 1);
  order[b * P + slot] = (n << 24) | (d << 16) | pix;
}

// insertion sort of each pillar's segment: fixes the (atomic, racy) fill order
__global__ void __launch_bounds__(256) k_segsort(const int *__restrict__ offsets, int P, int XYZ,
                                                 int B, int *__restrict__ order) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * XYZ) return;
  const long long b = i / XYZ;
  const int q = (int)(i - b * XYZ);
  const int *off = offsets + b * (XYZ + 1);
  int *seg = order + b * P;
  const int beg = off[q], end = off[q + 1];
  for (int k = beg + 1; k < end; ++k) {
    const int key = seg[k];
    int j = k - 1;
    while (j >= beg && seg[j] > key) {
      seg[j + 1] = seg[j];
      --j;
    }
    seg[j + 1] = key;
  }
}

// ------------------------------------------------------------------------------------------
// fused forward, general channel count (C % 4 != 0; the C = 64 product width uses
// k_lss_fwd below).  Block = 64 consecutive pillars of one sample x 64 channels; lane =
// channel, so every point costs one broadcast depth probability and one coalesced 256-B
// feature row (L2-resident: a sample's featT is 1 MB).  The block's points are contiguous
// in `order`; the 4 waves split them at pillar boundaries into ~equal point counts, walk
// them in sorted order (the same summation order as a sequential per-pillar sum), and
// stage per-pillar sums in an LDS [channel][pillar] tile that is written out channel-major
// with 256-B coalesced rows.  Codes and probabilities are gathered 64 points at a time
// (lane = point) and broadcast with shuffles; feature rows are fetched FWD_UNROLL at a time
// through a buffer descriptor (no per-load branch).  Block id -> (sample = id % B, tile =
// id / B), so at B = 8 each XCD works on one sample and its featT stays in that XCD's L2.
// ------------------------------------------------------------------------------------------
constexpr int FWD_TILE = 64;    // pillars per block
constexpr int FWD_UNROLL = 8;   // feature rows in flight per wave

__device__ __forceinline__ int first_ge(const int *O, int npil, int target, int lane) {
  const bool ge = lane <= npil && O[lane] >= target;
  const unsigned long long m = __ballot(ge);
  return m ? __ffsll((long long)m) - 1 : npil;
}

__global__ void __launch_bounds__(256) k_lss_fwd_narrow(
    const float *__restrict__ prob, const float *__restrict__ featT,
    const int *__restrict__ offsets, const int *__restrict__ order, int B, int N, int D, int HW,
    int C, int XYZ, int P, float *__restrict__ bev, long long bev_bstride) {
  __shared__ int O[FWD_TILE + 1];
  __shared__ float tile[64][FWD_TILE + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x % B, q0 = (blockIdx.x / B) * FWD_TILE;
  const int c0 = blockIdx.y * 64;
  const int npil = min(FWD_TILE, XYZ - q0);
  const int *off = offsets + (long long)b * (XYZ + 1);
  if ((int)threadIdx.x <= npil) O[threadIdx.x] = off[q0 + threadIdx.x];
  __syncthreads();
  const int base = O[0], T = O[npil] - base;
  const int ps = wave == 0 ? 0 : first_ge(O, npil, base + (int)(((long long)wave * T) >> 2), lane);
  const int pe = wave == 3 ? npil : first_ge(O, npil, base + (int)(((long long)(wave + 1) * T) >> 2), lane);
  const int cc = c0 + lane;
  const int *ord = order + (long long)b * P;
  const __amdgpu_buffer_rsrc_t rf = rsrc(featT, 4LL * B * N * HW * C);
  const int coff = cc < C ? cc * 4 : OOR;  // lanes past C read 0
  const int HWC = HW * C;
  int p = ps;
  float acc = 0.f;
  if (ps < pe) {
    const int ke = O[pe];
    int pend = O[p + 1];
    for (int k0 = O[ps]; k0 < ke; k0 += 64) {
      // lane-parallel gather of 64 point codes -> (feature row offset, probability)
      const int k = k0 + lane;
      int rowoff = 0;
      float pr = 0.f;
      if (k < ke) {
        const int code = ord[k];
        const int n = code >> 24, d = (code >> 16) & 255, pix = code & 65535;
        const int bn = b * N + n;
        pr = prob[((long long)bn * D + d) * HW + pix];
        rowoff = (bn * HWC + pix * C) * 4;
      }
      const int cnt = min(64, ke - k0);
      for (int j0 = 0; j0 < cnt; j0 += FWD_UNROLL) {
        float f[FWD_UNROLL], w[FWD_UNROLL];
#pragma unroll
        for (int u = 0; u < FWD_UNROLL; ++u) {
          const int ro = __shfl(rowoff, j0 + u, 64);
          w[u] = __shfl(pr, j0 + u, 64);
          f[u] = bload(rf, j0 + u < cnt ? ro + coff : OOR);
        }
#pragma unroll
        for (int u = 0; u < FWD_UNROLL; ++u) {
          if (j0 + u >= cnt) break;
          const int kk = k0 + j0 + u;
          while (kk >= pend) {  // pillar p complete (wave-uniform)
            tile[lane][p] = acc;
            acc = 0.f;
            ++p;
            pend = O[p + 1];
          }
          acc += w[u] * f[u];
        }
      }
    }
  }
  for (; p < pe; ++p) {  // the last pillar and any empty ones
    tile[lane][p] = acc;
    acc = 0.f;
  }
  __syncthreads();
  if (lane < npil) {
    float *o = bev + (long long)b * bev_bstride + q0 + lane;
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const int ch = wave * 16 + j;
      if (c0 + ch < C) o[(long long)(c0 + ch) * XYZ] = tile[ch][lane];
    }
  }
}

// ------------------------------------------------------------------------------------------
// fused forward, v2 (default).  Block = T consecutive pillars of one sample x 64 channels,
// 16 groups of 16 lanes; a lane owns 4 channels, so one point's 256-B feature row is one
// 16-B load per lane and a wave has 4 points' rows per load instruction (8 in flight per
// group = 32 rows per wave).  The block's points (contiguous in `order`) are cut into 16
// equal chunks at arbitrary positions, one per group, so every group does the same work
// whatever the pillar sizes.  A group walks its chunk in sorted order, keeping one running
// float4 sum (fma); on a pillar change it stores the sum into an LDS [channel][pillar] tile
// (zeroed first, so empty pillars read 0).  The chunk's first pillar may have started in the
// previous chunk: its partial sum goes to a per-group carry slot instead, and after a barrier
// the 16 carries are added in group order — a fixed summation order, so the result is
// deterministic.  Point codes are prefetched a batch ahead; codes and probabilities are
// gathered lane-parallel (16 per group) and broadcast inside the 16-lane row with DPP
// row_newbcast folded into the consuming instruction (no LDS traffic).  The tile is written
// out channel-major with 16-B stores.  Block id -> (sample = id % B, tile = tiles[b][id / B]):
// one sample per XCD at B = 8 (its 1 MB featT stays in that XCD's L2), heaviest tiles first.
// Measured (rocprofv3, B = 8, 4 cams): 37 us vs 61 us for v1; per-block traces
// (scripts/trace_lss_fwd.py) show a block lifetime of ~4 us fixed (offsets -> codes ->
// rows round trips, 16 KB write-out) + ~25 ns per point: latency-bound, not HBM-bound.
// ------------------------------------------------------------------------------------------

template <int J>
__device__ __forceinline__ int row_bcast(int v) {  // lane J of this lane's 16-lane row
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + J, 0xf, 0xf, true);
}
template <int J>
__device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(float, row_bcast<J>(__builtin_bit_cast(int, v)));
}

// One 8-point step of a group's walk: lanes J0..J0+7 of the 16-lane row hold the batch's row
// offsets / probabilities.  Slots past the chunk end carry probability 0 and row 0 (a valid
// row), and their position is clamped to the chunk's last point, so they add exactly 0 and
// never trigger a pillar change: no per-slot guards.
template <int J0, int UN>
__device__ __forceinline__ void fwd_step8(const __amdgpu_buffer_rsrc_t rf, int rowoff, float pr,
                                          int lane_off, int kbase, int klast, int &p, int &pend,
                                          const int *O, float4 &acc, bool &first, float *carry4,
                                          int *carry_pg, float *tile_l, int TP, int lg) {
  float4 f[UN];
  float w[UN];
#define E2EP_LD(U)                                               \
  f[U] = bload4(rf, row_bcast<J0 + U>(rowoff) + lane_off);      \
  w[U] = row_bcast<J0 + U>(pr);
  E2EP_LD(0) E2EP_LD(1) E2EP_LD(2) E2EP_LD(3) E2EP_LD(4) E2EP_LD(5) E2EP_LD(6) E2EP_LD(7)
  if constexpr (UN == 16) {
    E2EP_LD(8) E2EP_LD(9) E2EP_LD(10) E2EP_LD(11) E2EP_LD(12) E2EP_LD(13) E2EP_LD(14) E2EP_LD(15)
  }
#undef E2EP_LD
#pragma unroll
  for (int u = 0; u < UN; ++u) {
    if (min(kbase + J0 + u, klast) >= pend) {  // pillar p complete (group-uniform)
      if (first) {
        *reinterpret_cast<float4 *>(carry4) = acc;
        if (lg == 0) *carry_pg = p;
        first = false;
      } else {
        tile_l[0 * TP + p] = acc.x;
        tile_l[1 * TP + p] = acc.y;
        tile_l[2 * TP + p] = acc.z;
        tile_l[3 * TP + p] = acc.w;
      }
      acc = make_float4(0.f, 0.f, 0.f, 0.f);
      do {
        ++p;
        pend = O[p + 1];
      } while (pend <= kbase + J0 + u);
    }
    acc.x = __builtin_fmaf(w[u], f[u].x, acc.x);
    acc.y = __builtin_fmaf(w[u], f[u].y, acc.y);
    acc.z = __builtin_fmaf(w[u], f[u].z, acc.z);
    acc.w = __builtin_fmaf(w[u], f[u].w, acc.w);
  }
}

__device__ long long *g_fwd_trace;  // diagnostics: per-block (start, end, hw id, points)

template <int T, int NG, int UN>
__global__ void __launch_bounds__(NG * 16) k_lss_fwd(
    const float *__restrict__ prob, const float *__restrict__ featT,
    const int *__restrict__ offsets, const int *__restrict__ order,
    const int *__restrict__ tiles, int B, int N, int D, int HW, int C, int XYZ, int P,
    float *__restrict__ bev, long long bev_bstride, int vec_out, int lane_len) {
  constexpr int TP = T + 4;  // row pitch (16-B aligned rows)
  constexpr int NTHR = NG * 16;
  __shared__ int O[T + 1];
  __shared__ __attribute__((aligned(16))) float tile[64 * TP];
  __shared__ __attribute__((aligned(16))) float carry[NG][64];
  __shared__ int carry_p[NG];
  const int tid = threadIdx.x, g = tid >> 4, lg = tid & 15;
  const long long t_start = __builtin_amdgcn_s_memrealtime();
  int b, q0;
  if (lane_len) {  // lane schedule (k_tile_schedule): lane = block % 8, its j-th tile
    const int lane = blockIdx.x & 7, t = tiles[lane * lane_len + (blockIdx.x >> 3)];
    if (t < 0) return;  // a shorter lane's padding (whole block)
    b = lane % B;
    q0 = t * T;
  } else {
    b = blockIdx.x % B;
    const int rank = blockIdx.x / B, ntiles = (XYZ + T - 1) / T;
    q0 = (tiles && T == E2EP_LSS_TILE ? tiles[b * ntiles + rank] : rank) * T;
  }
  const int c0 = blockIdx.y * 64;
  const int npil = min(T, XYZ - q0);
  const int *off = offsets + (long long)b * (XYZ + 1);
  for (int i = tid; i <= npil; i += NTHR) O[i] = off[q0 + i];
  for (int i = tid; i < 16 * TP; i += NTHR)
    reinterpret_cast<float4 *>(tile)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lg == 0) carry_p[g] = -1;
  __syncthreads();
  const int base = O[0], tot = O[npil] - base;
  const int ks = base + (int)(((long long)g * tot) / NG);
  const int ke = base + (int)(((long long)(g + 1) * tot) / NG);
  if (ks < ke) {  // group-uniform
    // p = the pillar holding point ks = #{j in [1, npil] : O[j] <= ks}
    int cnt = 0;
    for (int j = lg + 1; j <= npil; j += 16) cnt += O[j] <= ks;
    cnt += __shfl_xor(cnt, 8, 64);
    cnt += __shfl_xor(cnt, 4, 64);
    cnt += __shfl_xor(cnt, 2, 64);
    cnt += __shfl_xor(cnt, 1, 64);
    int p = cnt, pend = O[p + 1];
    bool first = true;
    const int cc = c0 + 4 * lg;
    // this lane's 16 B of a feature row; lanes past C read 0 (offset beyond the buffer)
    const int lane_off = cc < C ? 4 * cc : 0x40000000;  // C % 4 == 0 (checked on the host)
    const __amdgpu_buffer_rsrc_t rf = rsrc(featT, 4LL * B * N * HW * C);
    const __amdgpu_buffer_rsrc_t rp = rsrc(prob, 4LL * B * N * D * HW);
    const int HWC = HW * C, DHW = D * HW;
    float *tile_l = tile + 4 * lg * TP;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // point codes are prefetched one 16-point batch ahead (branch-free loads, so the
    // compiler can leave the prefetch in flight).  (A deeper pipeline — codes two batches and
    // feature rows one 8-point step ahead — took 102 VGPRs: C4 111.6 -> 104.8 us but C2 37.7 ->
    // 49.4 us; the backward with all of a pixel's gathers issued together and the next pixel
    // prefetched, 117 VGPRs: 58 -> 63 us (C2), 153 -> 158 us (C4); profiles/r04/
    // lss_pipeline_ab.txt.  Fewer resident waves cost more than the deeper prefetch saved.)
    const __amdgpu_buffer_rsrc_t ro_ = rsrc(order + (long long)b * P, 4LL * P);
    int code_n = bload_i(ro_, ks + lg < ke ? (ks + lg) * 4 : OOR);
    for (int k0 = ks; k0 < ke; k0 += 16) {
      const int code = code_n;
      const bool valid = k0 + lg < ke;
      code_n = bload_i(ro_, k0 + 16 + lg < ke ? (k0 + 16 + lg) * 4 : OOR);
      const int n = code >> 24, d = (code >> 16) & 255, pix = code & 65535;
      const int bn = b * N + n;
      const float pr = bload(rp, valid ? (bn * DHW + d * HW + pix) * 4 : OOR);
      const int rowoff = valid ? (bn * HWC + pix * C) * 4 : 0;
      const int klast = ke - 1;
      if constexpr (UN == 16) {  // all 16 rows of the batch in flight together
        fwd_step8<0, 16>(rf, rowoff, pr, lane_off, k0, klast, p, pend, O, acc, first,
                         &carry[g][4 * lg], &carry_p[g], tile_l, TP, lg);
      } else {
        fwd_step8<0, 8>(rf, rowoff, pr, lane_off, k0, klast, p, pend, O, acc, first,
                        &carry[g][4 * lg], &carry_p[g], tile_l, TP, lg);
        if (k0 + 8 < ke)
          fwd_step8<8, 8>(rf, rowoff, pr, lane_off, k0, klast, p, pend, O, acc, first,
                          &carry[g][4 * lg], &carry_p[g], tile_l, TP, lg);
      }
    }
    if (first) {  // the chunk's last pillar
      *reinterpret_cast<float4 *>(&carry[g][4 * lg]) = acc;
      if (lg == 0) carry_p[g] = p;
    } else {
      tile_l[0 * TP + p] = acc.x;
      tile_l[1 * TP + p] = acc.y;
      tile_l[2 * TP + p] = acc.z;
      tile_l[3 * TP + p] = acc.w;
    }
  }
  __syncthreads();
  if (tid < 64) {  // carries, in chunk order
    for (int j = 0; j < NG; ++j) {
      const int pc = carry_p[j];
      if (pc >= 0) tile[tid * TP + pc] += carry[j][tid];
    }
  }
  __syncthreads();
  float *o = bev + (long long)b * bev_bstride + (long long)c0 * XYZ + q0;
  const int nch = min(64, C - c0);
  if (vec_out) {
    constexpr int R4 = T / 4;  // float4 per tile row
    for (int e = tid; e < 64 * R4; e += NTHR) {
      const int ch = e / R4, i4 = e - ch * R4;
      if (ch >= nch) break;
      const int i = 4 * i4;
      const float4 v = *reinterpret_cast<const float4 *>(&tile[ch * TP + i]);
      float *dst = o + (long long)ch * XYZ + i;
      if (i + 3 < npil) {
        *reinterpret_cast<float4 *>(dst) = v;
      } else {
        if (i < npil) dst[0] = v.x;
        if (i + 1 < npil) dst[1] = v.y;
        if (i + 2 < npil) dst[2] = v.z;
      }
    }
  } else {
    for (int e = tid; e < 64 * T; e += NTHR) {
      const int ch = e / T, i = e - ch * T;
      if (ch >= nch) break;
      if (i < npil) o[(long long)ch * XYZ + i] = tile[ch * TP + i];
    }
  }
  if (g_fwd_trace && tid == 0) {
    long long *r = g_fwd_trace + 4LL * (blockIdx.y * gridDim.x + blockIdx.x);
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    r[0] = t_start;
    r[1] = __builtin_amdgcn_s_memrealtime();
    r[2] = ((long long)xcc << 32) | hw;
    r[3] = tot;
  }
}

// ------------------------------------------------------------------------------------------
// backward: wave per pixel (lane = channel).  For one pixel of one camera, with q_d the
// pillar of depth bin d and G the gathered gT rows:
//   grad_feat[c] = sum_d prob[d] * G[d][c]      (register accumulation, d ascending)
//   grad_prob[d] = sum_c G[d][c] * feat[c]      (cross-lane reduction)
// The pixel's pillar indices and probabilities are loaded lane-parallel (lane = d) and
// broadcast with shuffles; the gT rows are gathered BWD_CHUNK at a time (one coalesced 256-B
// row per bin, all in flight together, masked bins read 0 through an out-of-range buffer
// offset); the 16 per-lane products of a chunk are reduced across the wave with a
// transposed halving (xor 8,4,2,1 keeps one value per lane, then xor 16,32), leaving
// grad_prob[d0 + u] in lanes 16*k + u.  Results go through LDS for coalesced stores.
// ------------------------------------------------------------------------------------------
constexpr int BWD_PIX_PER_WAVE = 4;
constexpr int BWD_WAVES = 4;
constexpr int BWD_PIX = BWD_PIX_PER_WAVE * BWD_WAVES;  // pixels per block
constexpr int BWD_CHUNK = 16;

template <int HALF>
__device__ __forceinline__ void halve(float *v, int lane) {
  const bool upper = (lane & HALF) != 0;
#pragma unroll
  for (int j = 0; j < HALF; ++j) {
    const float send = upper ? v[j] : v[j + HALF];
    const float keep = upper ? v[j + HALF] : v[j];
    v[j] = keep + __shfl_xor(send, HALF, 64);
  }
}

__global__ void __launch_bounds__(256) k_lss_bwd(
    const float *__restrict__ gT, const float *__restrict__ prob,
    const float *__restrict__ featT, const int *__restrict__ pillar, int B, int N, int D,
    int HW, int C, int XYZ, float *__restrict__ grad_prob, float *__restrict__ grad_feat) {
  __shared__ float s_gp[64][BWD_PIX + 1];
  __shared__ float s_gf[64][BWD_PIX + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // XCD-contiguous work order: workgroups are dealt round-robin to the 8 XCDs, so block L runs
  // on XCD L % 8; give XCD x the contiguous work range [x G/8, (x+1) G/8) — at B = 8 one
  // sample's 4 cameras, so an XCD's L2 holds the gT rows of one sample (a camera's rays
  // touch ~1/4 of its 10 MB) instead of every XCD streaming all eight samples' rows.
  const int chunks = (HW + BWD_PIX - 1) / BWD_PIX;
  const int G = gridDim.x, L = blockIdx.x;
  const int w = (G % 8 == 0) ? (L % 8) * (G / 8) + L / 8 : L;
  const int bn = w / chunks;  // b*N + n
  const int b = bn / N;
  const int pix0 = (w - bn * chunks) * BWD_PIX;
  const bool lane_ok = lane < C;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gT, 4LL * B * XYZ * C);
  const int rowbase = b * XYZ;
  for (int pp = 0; pp < BWD_PIX_PER_WAVE; ++pp) {
    const int lp = wave * BWD_PIX_PER_WAVE + pp;  // local pixel
    const int pix = pix0 + lp;
    if (pix >= HW) break;  // wave-uniform
    const float f = lane_ok ? featT[((long long)bn * HW + pix) * C + lane] : 0.f;
    int qd = -1;
    float pd = 0.f;
    if (lane < D) {
      const long long pidx = ((long long)bn * D + lane) * HW + pix;
      qd = pillar[pidx];
      pd = prob[pidx];
    }
    float gf = 0.f, gp = 0.f;
    for (int d0 = 0; d0 < D; d0 += BWD_CHUNK) {
      float g[BWD_CHUNK];
#pragma unroll
      for (int u = 0; u < BWD_CHUNK; ++u) {
        const int q = __shfl(qd, d0 + u, 64);  // -1 for d >= D (lanes past D hold -1)
        g[u] = bload(rg, (q >= 0 && lane_ok) ? ((rowbase + q) * C + lane) * 4 : OOR);
      }
#pragma unroll
      for (int u = 0; u < BWD_CHUNK; ++u) gf += __shfl(pd, d0 + u, 64) * g[u];
#pragma unroll
      for (int u = 0; u < BWD_CHUNK; ++u) g[u] *= f;
      halve<8>(g, lane);
      halve<4>(g, lane);
      halve<2>(g, lane);
      halve<1>(g, lane);
      float t = g[0];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      if ((lane >> 4) == d0 / BWD_CHUNK) gp = t;  // lane d now holds grad_prob[d] (D <= 64)
    }
    s_gp[lane][lp] = gp;
    s_gf[lane][lp] = gf;
  }
  __syncthreads();
  // coalesced write-back: rows d / c, columns = this block's pixels
  for (int e = threadIdx.x; e < 64 * BWD_PIX; e += 256) {
    const int r = e / BWD_PIX, lp = e - r * BWD_PIX;
    const int pix = pix0 + lp;
    if (pix >= HW) continue;
    if (r < D) grad_prob[((long long)bn * D + r) * HW + pix] = s_gp[r][lp];
    if (r < C) grad_feat[((long long)bn * C + r) * HW + pix] = s_gf[r][lp];
  }
}

// ------------------------------------------------------------------------------------------
// batched transpose through a padded 64x64 LDS tile
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_transpose(const float *__restrict__ in,
                                                   long long in_bstride, int rows, int cols,
                                                   float *__restrict__ out) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const float *src = in + (long long)b * in_bstride;
  float *dst = out + (long long)b * rows * cols;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int gr = r0 + r, gc = c0 + tx;
    if (gr < rows && gc < cols) tile[r][tx] = src[(long long)gr * cols + gc];
  }
  __syncthreads();
  for (int c = ty; c < 64; c += 4) {
    const int gc = c0 + c, gr = r0 + tx;
    if (gr < rows && gc < cols) dst[(long long)gc * rows + gr] = tile[tx][c];
  }
}

// many small transposes in one launch (the conv weights' tap-major copies, conv.py
// TapMajorBatch): entry e = {src, dst, rows, cols, first tile, column tiles} as int64;
// block = one 64 x 64 tile of one entry (found by a scan of the n <= 256 tile offsets)
__global__ void __launch_bounds__(256) k_transpose_multi(const long long *__restrict__ tab, int n) {
  __shared__ float tile[64][65];
  const int bid = blockIdx.x;
  int e = 0;
  while (e + 1 < n && tab[(e + 1) * 6 + 4] <= bid) ++e;
  const long long *t = tab + e * 6;
  const float *src = reinterpret_cast<const float *>(t[0]);
  float *dst = reinterpret_cast<float *>(t[1]);
  const int rows = (int)t[2], cols = (int)t[3], ct = (int)t[5];
  const int loc = bid - (int)t[4];
  const int r0 = (loc / ct) * 64, c0 = (loc % ct) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int gr = r0 + r, gc = c0 + tx;
    if (gr < rows && gc < cols) tile[r][tx] = src[(long long)gr * cols + gc];
  }
  __syncthreads();
  for (int c = ty; c < 64; c += 4) {
    const int gc = c0 + c, gr = r0 + tx;
    if (gr < rows && gc < cols) dst[(long long)gc * rows + gr] = tile[tx][c];
  }
}

// ------------------------------------------------------------------------------------------
// target channel: block per sample, zero the plane and set the 8x8 square
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void py_slice(int s, int e, int L, int &lo, int &hi) {
  if (s < 0) s += L;
  if (s < 0) s = 0;
  if (e < 0) e += L;
  if (e < 0) e = 0;
  lo = min(s, L);
  hi = min(e, L);
}

__global__ void __launch_bounds__(256) k_target_bev(const float *__restrict__ tp,
                                                    const float *__restrict__ noise, int X,
                                                    int Y, float res_x, float res_y,
                                                    float *__restrict__ out,
                                                    long long out_bstride) {
  const int b = blockIdx.x;
  // x_pixel = int(h/2 + x/res), + int(rand*10 - 5)            (parking_model.py:33-37)
  const float fx = __fadd_rn((float)X * 0.5f, __fdiv_rn(tp[3 * b + 0], res_x));
  const float fy = __fadd_rn((float)Y * 0.5f, __fdiv_rn(tp[3 * b + 1], res_y));
  const int nx = (int)truncf(__fsub_rn(__fmul_rn(noise[2 * b + 0], 10.f), 5.f));
  const int ny = (int)truncf(__fsub_rn(__fmul_rn(noise[2 * b + 1], 10.f), 5.f));
  const int px = (int)truncf(fx) + nx, py = (int)truncf(fy) + ny;
  int xlo, xhi, ylo, yhi;
  py_slice(px - 4, px + 4, X, xlo, xhi);
  py_slice(py - 4, py + 4, Y, ylo, yhi);
  float *o = out + (long long)b * out_bstride;
  for (int i = threadIdx.x; i < X * Y; i += blockDim.x) {
    const int x = i / Y, y = i - x * Y;
    o[i] = (x >= xlo && x < xhi && y >= ylo && y < yhi) ? 1.f : 0.f;
  }
}


// ------------------------------------------------------------------------------------------
// rig algebra on the device: combine = R(E^-1) K^-1, trans = t(E^-1)   (bev_model.py:46-53)
// fp64 Gauss-Jordan with partial pivoting, rounded once to fp32: deterministic on every host
// (the reference's fp32 LAPACK result varies by host CPU ISA in the last ulp).
// ------------------------------------------------------------------------------------------
template <int M>
__device__ void inv_gj(const double *a_in, double *inv) {
  double a[M][M], r[M][M];
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < M; ++j) {
      a[i][j] = a_in[i * M + j];
      r[i][j] = i == j ? 1.0 : 0.0;
    }
  for (int c = 0; c < M; ++c) {
    int piv = c;
    for (int i = c + 1; i < M; ++i)
      if (fabs(a[i][c]) > fabs(a[piv][c])) piv = i;
    if (piv != c)
      for (int j = 0; j < M; ++j) {
        double t = a[c][j]; a[c][j] = a[piv][j]; a[piv][j] = t;
        t = r[c][j]; r[c][j] = r[piv][j]; r[piv][j] = t;
      }
    const double d = a[c][c];
    for (int j = 0; j < M; ++j) { a[c][j] /= d; r[c][j] /= d; }
    for (int i = 0; i < M; ++i) {
      if (i == c) continue;
      const double f = a[i][c];
      if (f == 0.0) continue;
      for (int j = 0; j < M; ++j) { a[i][j] -= f * a[c][j]; r[i][j] -= f * r[c][j]; }
    }
  }
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < M; ++j) inv[i * M + j] = r[i][j];
}

__global__ void k_rig(const float *__restrict__ K, const float *__restrict__ E, int BN,
                      float *__restrict__ combine, float *__restrict__ trans) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= BN) return;
  double k[9], e[16], ki[9], ei[16];
  for (int j = 0; j < 9; ++j) k[j] = K[9 * i + j];
  for (int j = 0; j < 16; ++j) e[j] = E[16 * i + j];
  inv_gj<3>(k, ki);
  inv_gj<4>(e, ei);
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) {
      double acc = 0.0;
      for (int t = 0; t < 3; ++t) acc += ei[4 * r + t] * ki[3 * t + c];
      combine[9 * i + 3 * r + c] = (float)acc;
    }
    trans[3 * i + r] = (float)ei[4 * r + 3];
  }
}

// Tile schedule for k_lss_fwd: the T-pillar tiles ranked by point count, heaviest first (ties
// by index), so the few dense tiles next to the ego vehicle (up to 5x the mean) start at once
// instead of setting the kernel's tail.  One block per sample.
//  * B = 8 (or lane_len = 0): per sample, all of its tiles; block id -> (sample id % B, rank
//    id / B): one sample per XCD at B = 8, where its featT (1 MB) stays in that XCD's L2.
//  * B = 1, 2, 4 (lane schedule, G = 8 / B lanes per sample): each sample's tiles are cut into G
//    contiguous pillar ranges (x bands of the BEV grid, seen by a subset of the cameras), and
//    range g of sample s is the list of lane g * B + s: tiles[lane][0..lane_len), heaviest
//    first, padded with -1.  Block id -> (lane id % 8, entry id / 8): a lane's blocks share one
//    XCD (workgroups are dealt round-robin over the 8 XCDs — a placement used for speed only),
//    so an XCD's L2 holds the features of part of one sample's cameras instead of all of them
//    (C4, B = 4: 6.3 MB of featT per sample against a 4 MB L2; round 4 measured a 51 % L2 hit
//    rate for the per-sample order).  Round 6: the range boundaries balance POINTS, not tiles —
//    the C4 rig's front band holds 1.8x the rear band's points (554 k vs 305 k per sample), so
//    equal tile ranges left one XCD of each pair with 65 % of the sample's work.  A tile goes to
//    the range its point midpoint falls in; ranges stay within lane_len tiles (lss_lane_len:
//    1.5x the even share), else the even cut is kept.
constexpr int SCHED_MAX_TILES = 4096;
constexpr int SCHED_MAX_G = 8;
__global__ void __launch_bounds__(1024) k_tile_schedule(const int *__restrict__ offsets, int XYZ,
                                                        int T, int B, int lane_len,
                                                        int *__restrict__ tiles) {
  __shared__ int cnt[SCHED_MAX_TILES];
  __shared__ int bnd[SCHED_MAX_G + 1];
  const int b = blockIdx.x, nt = (XYZ + T - 1) / T;
  const int G = lane_len ? 8 / B : 1;
  const int *off = offsets + (long long)b * (XYZ + 1);
  for (int t = threadIdx.x; t < nt; t += blockDim.x)
    cnt[t] = off[min((t + 1) * T, XYZ)] - off[t * T];
  if ((int)threadIdx.x <= G) bnd[threadIdx.x] = 0;
  __syncthreads();
  if (G > 1) {
    // point-balanced cut: tile t belongs to range floor(G * mid(t) / total), mid(t) = the
    // points before it + half its own (offsets are the exclusive prefix of the counts);
    // bnd[g] = number of tiles of ranges < g
    const long long total = off[XYZ] - off[0];
    for (int t = threadIdx.x; t < nt; t += blockDim.x) {
      const long long mid2 = 2LL * (off[t * T] - off[0]) + cnt[t];  // 2 * midpoint
      const int g = total > 0 ? (int)min((long long)G - 1, (mid2 * G) / (2 * total)) : 0;
      for (int u = g + 1; u <= G; ++u) atomicAdd(&bnd[u], 1);
    }
    __syncthreads();
    bool fits = bnd[G] == nt;
    for (int g = 0; g < G; ++g) fits = fits && bnd[g + 1] - bnd[g] <= lane_len;
    __syncthreads();
    if (!fits && (int)threadIdx.x <= G)  // the even cut
      bnd[threadIdx.x] = (int)(((long long)threadIdx.x * nt + G - 1) / G);
    __syncthreads();
  } else if (threadIdx.x == 0) {
    bnd[1] = nt;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < nt; t += blockDim.x) {
    const int c = cnt[t];
    int g = 0;
    while (g + 1 < G && t >= bnd[g + 1]) ++g;
    const int lo = bnd[g], hi = bnd[g + 1];
    int r = 0;
    for (int u = lo; u < hi; ++u) r += cnt[u] > c || (cnt[u] == c && u < t);
    if (lane_len) tiles[(long long)(g * B + b) * lane_len + r] = t;
    else tiles[(long long)b * nt + r] = t;
  }
  if (lane_len)  // padding past each range's end
    for (int g = 0; g < G; ++g) {
      const int len = bnd[g + 1] - bnd[g];
      for (int r = len + threadIdx.x; r < lane_len; r += blockDim.x)
        tiles[(long long)(g * B + b) * lane_len + r] = -1;
    }
}

// lane-schedule length (0 = per-sample order): B divides 8 and B < 8.  1.5x the even share of
// tiles, so point-balanced ranges fit (k_tile_schedule)
static int lss_lane_len(int B, int XYZ) {
  const int nt = cdiv(XYZ, E2EP_LSS_TILE);
  if (B >= 8 || 8 % B != 0) return 0;
  return cdiv(3 * cdiv(nt, 8 / B), 2);
}

__global__ void k_zero_i32(int *p, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_geom_index(const float *frustum, const float *combine, const float *trans,
                    const float *lo, const float *res, int X, int Y, int Z, int B, int N, int D,
                    int h, int w, int32_t *pillar, void *stream) {
  E2EP_REQUIRE(B > 0 && N > 0 && D > 0 && h > 0 && w > 0 && X > 0 && Y > 0 && Z > 0, E2EP_EINVAL,
               "e2ep_geom_index: non-positive shape");
  E2EP_REQUIRE(lo && res, E2EP_EINVAL, "e2ep_geom_index: lo/res must be host arrays of 3");
  const long long total = (long long)B * N * D * h * w;
  hipLaunchKernelGGL(k_geom_index, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream),
                     frustum, combine, trans, lo[0], lo[1], lo[2], res[0], res[1], res[2], X, Y, Z,
                     D * h * w, total, pillar);
  return launch_status("e2ep_geom_index");
}

int e2ep_rig_transforms(const float *K, const float *E, int BN, float *combine, float *trans,
                        void *stream) {
  E2EP_REQUIRE(BN > 0, E2EP_EINVAL, "e2ep_rig_transforms: BN must be positive");
  hipLaunchKernelGGL(k_rig, dim3(cdiv(BN, 64)), dim3(64), 0, as_stream(stream), K, E, BN, combine,
                     trans);
  return launch_status("e2ep_rig_transforms");
}

size_t e2ep_lss_plan_workspace(int B, int XYZ) { return (size_t)B * XYZ * sizeof(int); }

int e2ep_debug_fwd_trace(void *dev_buf) {
  long long *p = static_cast<long long *>(dev_buf);
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_trace), &p, sizeof(p));
  return e == hipSuccess ? 0 : (int)e;
}

// per sample: room for the lane schedule's 8 * lss_lane_len(B, XYZ) entries at any B
int e2ep_lss_tiles(int XYZ) { return 2 * cdiv(XYZ, E2EP_LSS_TILE) + 16; }

int e2ep_lss_plan(const int32_t *pillar, int B, int N, int D, int h, int w, int XYZ,
                  int32_t *offsets, int32_t *order, int32_t *tiles, void *workspace,
                  size_t workspace_bytes, void *stream) {
  E2EP_REQUIRE(B > 0 && XYZ > 0, E2EP_EINVAL, "e2ep_lss_plan: bad shape");
  E2EP_REQUIRE(workspace && workspace_bytes >= e2ep_lss_plan_workspace(B, XYZ), E2EP_EINVAL,
               "e2ep_lss_plan: workspace %zu bytes < %zu (e2ep_lss_plan_workspace)",
               workspace_bytes, e2ep_lss_plan_workspace(B, XYZ));
  E2EP_REQUIRE(N < 128 && D < 256 && h * w < 65536, E2EP_ERANGE,
               "e2ep_lss_plan: packed point code needs N<128, D<256, h*w<65536 (got %d,%d,%d)", N,
               D, h * w);
  hipStream_t s = as_stream(stream);
  int *cnt = static_cast<int *>(workspace);
  const int P = N * D * h * w;
  const long long total = (long long)B * P;
  // zero the counters with a kernel, not hipMemsetAsync: memset nodes do not replay
  // correctly from captured HIP graphs on this stack (csrc/graph.hip)
  hipLaunchKernelGGL(k_zero_i32, dim3(cdiv((long long)B * XYZ, 256)), dim3(256), 0, s, cnt,
                     (long long)B * XYZ);
  hipLaunchKernelGGL(k_count, dim3(cdiv(total, 256)), dim3(256), 0, s, pillar, P, XYZ, total, cnt);
  // scan writes offsets and re-uses the count buffer as the fill cursor
  hipLaunchKernelGGL(k_scan, dim3(B), dim3(1024), 0, s, cnt, XYZ, offsets, cnt);
  hipLaunchKernelGGL(k_fill, dim3(cdiv(total, 256)), dim3(256), 0, s, pillar, P, D * h * w, h * w,
                     XYZ, total, cnt, order);
  hipLaunchKernelGGL(k_segsort, dim3(cdiv((long long)B * XYZ, 256)), dim3(256), 0, s, offsets, P,
                     XYZ, B, order);
  if (tiles) {
    E2EP_REQUIRE(cdiv(XYZ, E2EP_LSS_TILE) <= SCHED_MAX_TILES, E2EP_ERANGE,
                 "e2ep_lss_plan: %d tiles per sample exceed the scheduler's %d (pass tiles=NULL)",
                 cdiv(XYZ, E2EP_LSS_TILE), SCHED_MAX_TILES);
    E2EP_REQUIRE(8LL * lss_lane_len(B, XYZ) <= (long long)B * e2ep_lss_tiles(XYZ), E2EP_ERANGE,
                 "e2ep_lss_plan: lane schedule exceeds the tile buffer");
    hipLaunchKernelGGL(k_tile_schedule, dim3(B), dim3(1024), 0, s, offsets, XYZ, E2EP_LSS_TILE, B,
                       lss_lane_len(B, XYZ), tiles);
  }
  return launch_status("e2ep_lss_plan");
}

int e2ep_lss_fwd(const float *prob, const float *featT, const int32_t *offsets,
                 const int32_t *order, const int32_t *tiles, int B, int N, int D, int hw, int C,
                 int XYZ, float *bev, long long bev_bstride, void *stream) {
  E2EP_REQUIRE(B > 0 && N > 0 && D > 0 && hw > 0 && C > 0 && XYZ > 0, E2EP_EINVAL,
               "e2ep_lss_fwd: bad shape");
  E2EP_REQUIRE(((uintptr_t)featT & 15) == 0, E2EP_EINVAL, "e2ep_lss_fwd: featT must be 16-B aligned");
  E2EP_REQUIRE(4LL * B * N * hw * C < 0x7fffffffLL, E2EP_ERANGE,
               "e2ep_lss_fwd: featT over 2 GiB (32-bit buffer offsets)");
  if (C % 4 != 0) {  // general-width path: lane = channel
    dim3 grid(cdiv(XYZ, FWD_TILE) * B, cdiv(C, 64));
    hipLaunchKernelGGL(k_lss_fwd_narrow, grid, dim3(256), 0, as_stream(stream), prob, featT, offsets,
                       order, B, N, D, hw, C, XYZ, N * D * hw, bev, bev_bstride);
  } else {
    const int vec = ((uintptr_t)bev & 15) == 0 && XYZ % 4 == 0 && bev_bstride % 4 == 0;
    const int ll = tiles ? lss_lane_len(B, XYZ) : 0;
    const int gx = ll ? 8 * ll : cdiv(XYZ, E2EP_LSS_TILE) * B;
    // groups per block x feature rows in flight per group.  Automatic (e2ep_tune key 32 = 1):
    // 16 rows when a sample's featT exceeds an XCD's 4 MB L2 (C4: 6.3 MB, its rows come from
    // MALL / HBM: 89.8 -> 82.1 us, bitwise equal), else 8 (C2, 1 MB: 37.9 us against 44.8 us
    // with 16, the extra VGPRs cost occupancy); profiles/r05/lss_fwd_variants.txt
    int v = g_tune[TUNE_LSS_FWD];
    if (v == 1 && 4LL * N * hw * C > (4LL << 20)) v = 3;
#define E2EP_LSSF(NGV, UNV)                                                                      \
  hipLaunchKernelGGL((k_lss_fwd<E2EP_LSS_TILE, NGV, UNV>), dim3(gx, cdiv(C, 64)), dim3(NGV * 16), \
                     0, as_stream(stream), prob, featT, offsets, order, tiles, B, N, D, hw, C,    \
                     XYZ, N * D * hw, bev, bev_bstride, vec, ll)
    if (v == 2) E2EP_LSSF(32, 8);
    else if (v == 3) E2EP_LSSF(16, 16);
    else if (v == 4) E2EP_LSSF(32, 16);
    else if (v == 5) E2EP_LSSF(16, 8);
    else E2EP_LSSF(16, 8);
#undef E2EP_LSSF
  }
  return launch_status("e2ep_lss_fwd");
}

int e2ep_lss_bwd(const float *gT, const float *prob, const float *featT, const int32_t *pillar,
                 int B, int N, int D, int hw, int C, int XYZ, float *grad_prob, float *grad_feat,
                 void *stream) {
  E2EP_REQUIRE(B > 0 && N > 0 && D > 0 && hw > 0 && C > 0 && XYZ > 0, E2EP_EINVAL,
               "e2ep_lss_bwd: bad shape");
  E2EP_REQUIRE(C <= 64 && D <= 64, E2EP_ERANGE, "e2ep_lss_bwd: needs C<=64, D<=64 (got %d,%d)", C, D);
  dim3 grid(cdiv(hw, BWD_PIX) * B * N);  // 1-D: the kernel maps blocks to XCD-contiguous work
  E2EP_REQUIRE(4LL * B * XYZ * C < 0x7fffffffLL, E2EP_ERANGE,
               "e2ep_lss_bwd: gT over 2 GiB (32-bit buffer offsets)");
  hipLaunchKernelGGL(k_lss_bwd, grid, dim3(256), 0, as_stream(stream), gT, prob, featT, pillar, B,
                     N, D, hw, C, XYZ, grad_prob, grad_feat);
  return launch_status("e2ep_lss_bwd");
}

int e2ep_transpose(const float *in, long long in_bstride, int batch, int rows, int cols, float *out,
                   void *stream) {
  E2EP_REQUIRE(batch > 0 && rows > 0 && cols > 0 && batch < 65536, E2EP_EINVAL,
               "e2ep_transpose: bad shape");
  dim3 grid(cdiv(cols, 64), cdiv(rows, 64), batch);
  hipLaunchKernelGGL(k_transpose, grid, dim3(256), 0, as_stream(stream), in, in_bstride, rows, cols,
                     out);
  return launch_status("e2ep_transpose");
}

int e2ep_transpose_multi(const long long *table, int n, int tiles, void *stream) {
  E2EP_REQUIRE(table && n > 0 && n <= 256 && tiles > 0, E2EP_EINVAL,
               "e2ep_transpose_multi: bad table (n %d, tiles %d)", n, tiles);
  hipLaunchKernelGGL(k_transpose_multi, dim3(tiles), dim3(256), 0, as_stream(stream), table, n);
  return launch_status("e2ep_transpose_multi");
}

int e2ep_target_bev(const float *target_point, const float *noise, int B, int X, int Y, float res_x,
                    float res_y, float *out, long long out_bstride, void *stream) {
  E2EP_REQUIRE(B > 0 && X > 0 && Y > 0, E2EP_EINVAL, "e2ep_target_bev: bad shape");
  hipLaunchKernelGGL(k_target_bev, dim3(B), dim3(256), 0, as_stream(stream), target_point, noise, X,
                     Y, res_x, res_y, out, out_bstride);
  return launch_status("e2ep_target_bev");
}

}  // extern "C"
