// Depthwise (groups == channels, multiplier 1) conv for EfficientNet's MBConv
// (efficientnet-pytorch 0.7.1 _depthwise_conv: k3/k5, stride 1/2, static SAME padding),
// forward, data gradient (gather, no atomics) and weight gradient (fixed-order split
// reduction), NCHW fp32, for gfx950.  Memory-bound: each kernel streams its input once.
#include <type_traits>

#include "common.h"
#include "handoff.h"

// Contraction only within one expression (a*b + c -> fma): the fp32 and bf16-storage
// instantiations of a kernel (E2EP_IO_*) then fuse the same operations and round alike —
// under the default cross-statement contraction hipcc may pick a different multiply to fuse
// in each instantiation (tests/test_bf16_store_gpu.py holds them bitwise equal).
#pragma clang fp contract(on)

namespace e2ep {

// Weight-gradient output: per-split slabs part[c][split][K*K]; with one split the slab is the
// gradient and is written to dw directly; with several and `cnt` (the in-launch fold, e2ep_tune
// key 28 = 2) the slabs are stored write-through and the channel's last-arriving split sums
// them in split order (k_dw_wgrad_finalize's order) into dw; otherwise k_dw_wgrad_finalize does.
struct DwPart {
  float *part, *dw;
  unsigned int *cnt;
};

template <int KK>
__device__ __forceinline__ void dw_wgrad_out(DwPart o, int c, int sp, int splits, float v,
                                             int *s_last) {
  const int t = threadIdx.x;
  if (t < KK) {
    if (splits == 1) o.dw[(long long)c * KK + t] = v;
    else if (o.cnt) st_sc1(o.part + ((long long)c * splits + sp) * KK + t, v);
    else o.part[((long long)c * splits + sp) * KK + t] = v;
  }
  if (splits == 1 || !o.cnt) return;
  handoff_drain();
  if (!handoff_arrive(o.cnt + c, splits, s_last)) return;
  if (t < KK) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += ld_sc1(o.part + ((long long)c * splits + k) * KK + t);
    o.dw[(long long)c * KK + t] = s;
  }
}

struct DwGeom {
  int N, C, H, W, K, P, Q, st, pt, pl;
};

// Optional input transform of the forward / weight-gradient kernels: the input is the raw
// output of the preceding 1x1 conv and the kernel applies that layer's BatchNorm (per-channel
// scale / shift from e2ep_bn_stats) and activation on load, so the normalised tensor is never
// written (zero padding stays zero: it lives in the normalised space).
struct DwIn {
  const float *sc, *sh;  // [C] or null (identity)
  int act;               // 0 none, 1 relu, 2 swish
};
__device__ __forceinline__ float dw_in(float v, float sc, float sh, int act) {
  const float z = v * sc + sh;
  return act == 2 ? swish_f(z) : act == 1 ? fmaxf(z, 0.f) : z;
}

// forward: one thread per output pixel; taps unrolled; branch-free guarded loads
template <int K, int ST>
__global__ void __launch_bounds__(256) k_dw_fwd(const float *__restrict__ x,
                                                const float *__restrict__ w, DwGeom g,
                                                float *__restrict__ y, const float *__restrict__ tsc,
                                                const float *__restrict__ tsh, int tact) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P * g.Q) return;
  const int nc = blockIdx.y;
  const int c = nc % g.C;
  const int oy = i / g.Q, ox = i - oy * g.Q;
  const int HW = g.H * g.W;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x + (size_t)nc * HW, 4LL * HW);
  const float *wp = w + c * K * K;
  const int y0 = oy * ST - g.pt, x0 = ox * ST - g.pl;
  float v[K * K];
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int iy = y0 + a;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int ix = x0 + b;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      v[a * K + b] = bload(rx, ok ? (iy * g.W + ix) * 4 : OOR);
      if (tsc && ok) v[a * K + b] = dw_in(v[a * K + b], tsc[c], tsh[c], tact);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < K * K; ++t) s += wp[t] * v[t];
  y[(size_t)nc * g.P * g.Q + i] = s;
}

// data gradient: one thread per input pixel, gather the outputs whose window covers it
// (branch-free: invalid taps read 0 through an out-of-range buffer offset)
template <int K, int ST>
__global__ void __launch_bounds__(256) k_dw_dgrad(const float *__restrict__ gy,
                                                  const float *__restrict__ w, DwGeom g,
                                                  float *__restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.H * g.W) return;
  const int nc = blockIdx.y;
  const int c = nc % g.C;
  const int iy = i / g.W, ix = i - iy * g.W;
  const int PQ = g.P * g.Q;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gy + (size_t)nc * PQ, 4LL * PQ);
  const float *wp = w + c * K * K;
  float v[K * K];
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int ny = iy + g.pt - a;
    const int oy = ny >= 0 ? ny / ST : -1;  // ST is a compile-time 1 or 2
    const bool oky = ny >= 0 && oy * ST == ny && oy < g.P;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int nx = ix + g.pl - b;
      const int ox = nx >= 0 ? nx / ST : -1;
      const bool ok = oky && nx >= 0 && ox * ST == nx && ox < g.Q;
      v[a * K + b] = bload(rg, ok ? (oy * g.Q + ox) * 4 : OOR);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < K * K; ++t) s += wp[t] * v[t];
  dx[(size_t)nc * g.H * g.W + i] = s;
}

// weight gradient partials: grid (C, splits); each slice of (n, oy, ox) accumulates K*K taps
template <int K, int ST>
__global__ void __launch_bounds__(256) k_dw_wgrad(const float *__restrict__ gy,
                                                  const float *__restrict__ x, DwGeom g,
                                                  int splits, DwPart part,
                                                  const float *__restrict__ tsc,
                                                  const float *__restrict__ tsh, int tact) {
  const int c = blockIdx.x, sp = blockIdx.y;
  const int PQ = g.P * g.Q;
  const int tot = g.N * PQ;
  const int per = (tot + splits - 1) / splits;
  const int beg = sp * per, end = min(tot, beg + per);
  float acc[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) acc[t] = 0.f;
  const int HW = g.H * g.W;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.C * HW);
  for (int i = beg + threadIdx.x; i < end; i += 256) {
    const int n = i / PQ;
    const int pix = i - n * PQ;
    const int oy = pix / g.Q, ox = pix - oy * g.Q;
    const float gv = gy[((size_t)n * g.C + c) * PQ + pix];
    const int xb = (n * g.C + c) * HW;
    const int y0 = oy * ST - g.pt, x0 = ox * ST - g.pl;
#pragma unroll
    for (int a = 0; a < K; ++a) {
      const int iy = y0 + a;
      const bool oky = (unsigned)iy < (unsigned)g.H;
#pragma unroll
      for (int b = 0; b < K; ++b) {
        const int ix = x0 + b;
        const bool ok = oky && (unsigned)ix < (unsigned)g.W;
        float xv = bload(rx, ok ? (xb + iy * g.W + ix) * 4 : OOR);
        if (tsc && ok) xv = dw_in(xv, tsc[c], tsh[c], tact);
        acc[a * K + b] += gv * xv;
      }
    }
  }
  __shared__ float red[4][K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float v = wave_sum(acc[t]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v;
  }
  __syncthreads();
  const int t = threadIdx.x < K * K ? threadIdx.x : 0;
  // the last-arriver flag reuses red[0][0] (read above, before dw_wgrad_out's first barrier):
  // a static __shared__ int would leave the kernel's static LDS at 4 mod 16 bytes and shift the
  // strip kernels' dynamic LDS base off 16-B alignment (their b128 window reads then replay:
  // 1.5 - 2x slower; cdna_hip_programming.md Guideline 17)
  dw_wgrad_out<K * K>(part, c, sp, splits, (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]),
                      reinterpret_cast<int *>(&red[0][0]));
}

__global__ void k_dw_wgrad_finalize(const float *__restrict__ part, int C, int KK, int splits,
                                    float *__restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * KK) return;
  const int c = i / KK, t = i - c * KK;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[((long long)c * splits + k) * KK + t];
  dw[i] = s;
}

// ------------------------------------------------------------------------------------------
// Strip kernels (Q % 4 == 0, Q <= 256): each wave owns one unit = (plane n*C+c, RO = 256/Q
// consecutive output rows) and every lane 4 horizontally adjacent outputs, so a unit is
// exactly 64 x 4 outputs.  The unit's input rows ((RO-1)*ST + K of them) are staged once in
// LDS with float4 loads, zero-padded left/right (DW_PADL columns) and above/below, and each
// lane reads its (3*ST + K) x K window from LDS: per output K*(3*ST+K)/4 LDS reads instead of
// K*K global loads.  Weights are wave-uniform (scalar loads).  Forward; the stride-1 data
// gradient is the same correlation with the filter flipped and pads K-1-pad (FLIP).
// ------------------------------------------------------------------------------------------
constexpr int DW_PADL = 4;  // left halo columns in LDS (>= max left pad 2, keeps rows 16-B aligned)

struct DwStrip {
  int RO, IR, WP, units_per_plane;  // out rows / unit, staged input rows, LDS row pitch
};

static DwStrip dw_strip(int K, int st, int W, int P, int Q) {
  DwStrip d;
  d.RO = 64 / (Q / 4);  // lanes past RO * (Q / 4) idle
  d.IR = (d.RO - 1) * st + K;
  d.WP = W + 2 * DW_PADL;
  d.units_per_plane = (P + d.RO - 1) / d.RO;
  return d;
}

// Each wave of the strip kernels stages and reads only its own LDS region, so the staging
// needs a wave-level fence, not a block barrier: the wave's LDS writes complete (lgkmcnt(0))
// before any lane reads another lane's words, and the four waves of a block run decoupled.
__device__ __forceinline__ void dw_wave_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt unconstrained
  __builtin_amdgcn_wave_barrier();
}

// stage input rows [iy0, iy0 + IR) of plane `src` (H x W) into this wave's LDS buffer.  The
// loads are branch-free buffer loads (rows outside the plane read 0 through an out-of-range
// offset) issued before any is used: a guarded `if (row ok) v = load` made hipcc branch
// around each load and wait for it, one round trip per float4 (1.2-3 TB/s, round 3).
constexpr int DW_MAXV = 6;  // float4 per lane the unrolled staging covers (host-checked)
// the input transform resolved for one channel (read once per wave, not per staged row)
struct DwT {
  float sc, sh;
  int act;
  bool on;
};
__device__ __forceinline__ DwT dw_t(DwIn tf, int c) {
  const bool on = tf.sc != nullptr;
  return DwT{on ? tf.sc[c] : 1.f, on ? tf.sh[c] : 0.f, tf.act, on};
}
// transform of one staged float4; `in` = inside the plane (padding stays zero).  The act
// branches are wave-uniform; the padding test is a per-lane select, not a branch
__device__ __forceinline__ float4 dw_tf4(float4 v, const DwT &t, bool in) {
  if (!t.on) return v;
  float z[4] = {v.x * t.sc + t.sh, v.y * t.sc + t.sh, v.z * t.sc + t.sh, v.w * t.sc + t.sh};
  if (t.act == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = swish_f(z[i]);
  } else if (t.act == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = fmaxf(z[i], 0.f);
  }
  return make_float4(in ? z[0] : 0.f, in ? z[1] : 0.f, in ? z[2] : 0.f, in ? z[3] : 0.f);
}
// buffer descriptor of a wave-uniform plane: the base pointer and size go through
// readfirstlane so the descriptor lives in SGPRs (a VGPR descriptor makes hipcc wrap every
// buffer load in a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_u(const void *p, long long bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes >= 0x7fffffff ? 0x7fffffff : bytes));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void *>(((unsigned long long)hi << 32) | lo), (short)0, nb, 0x00020000);
}
template <typename TI>
__device__ __forceinline__ void dw_stage(const TI *__restrict__ src, int H, int W, int iy0,
                                         int IR, int WP, float *lds, int lane,
                                         DwIn tf = DwIn{nullptr, nullptr, 0}, int c = 0) {
  const int W4 = W >> 2;
  const DwT t = dw_t(tf, c);
  constexpr int EB = sizeof(TI);  // bytes per element (4 fp32, 2 bf16 storage)
  const __amdgpu_buffer_rsrc_t rs = rsrc_u(src, (long long)EB * H * W);
  float4 v[DW_MAXV];
  bool in[DW_MAXV];
#pragma unroll
  for (int i = 0; i < DW_MAXV; ++i) {
    const int e = lane + 64 * i;
    const int r = e / W4, j = e - r * W4;
    const int iy = iy0 + r;
    in[i] = e < IR * W4 && (unsigned)iy < (unsigned)H;
    v[i] = bload4t(rs, in[i] ? (iy * W + 4 * j) * EB : OOR, src);
  }
#pragma unroll
  for (int i = 0; i < DW_MAXV; ++i) {
    const int e = lane + 64 * i;
    if (e >= IR * W4) break;
    const int r = e / W4, j = e - r * W4;
    // padding rows stay zero (the padding lives in the normalised space)
    *reinterpret_cast<float4 *>(lds + r * WP + DW_PADL + 4 * j) = dw_tf4(v[i], t, in[i]);
  }
  // halo columns
  for (int e = lane; e < IR * 2 * DW_PADL; e += 64) {
    const int r = e / (2 * DW_PADL), j = e - r * (2 * DW_PADL);
    lds[r * WP + (j < DW_PADL ? j : W + j)] = 0.f;
  }
}

// The same staging split in two for software pipelining: dw_fetch issues a unit's row loads
// into registers (at most DW_MAXV float4 per lane), dw_put writes them (normalised) and the
// halo zeros into LDS once they have landed.
template <int V, typename TI>
__device__ __forceinline__ void dw_fetch(const TI *__restrict__ src, int H, int W, int iy0,
                                         int IR, int lane, float4 (&r)[V], bool active) {
  const int W4 = W >> 2;
  constexpr int EB = sizeof(TI);
  const __amdgpu_buffer_rsrc_t rs = rsrc_u(src, (long long)EB * H * W);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int e = lane + 64 * i;
    const int rr = e / W4, j = e - rr * W4;
    const int iy = iy0 + rr;
    const bool ok = active && e < IR * W4 && (unsigned)iy < (unsigned)H;
    r[i] = bload4t(rs, ok ? (iy * W + 4 * j) * EB : OOR, src);  // branch-free (see dw_stage)
  }
}
template <int V>
__device__ __forceinline__ void dw_put(const float4 (&r)[V], int H, int W, int iy0, int IR,
                                       int WP, float *lds, int lane, const DwT &t) {
  const int W4 = W >> 2;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int e = lane + 64 * i;
    if (e >= IR * W4) break;
    const int rr = e / W4, j = e - rr * W4;
    // padding rows stay zero
    *reinterpret_cast<float4 *>(lds + rr * WP + DW_PADL + 4 * j) =
        dw_tf4(r[i], t, (unsigned)(iy0 + rr) < (unsigned)H);
  }
  for (int e = lane; e < IR * 2 * DW_PADL; e += 64) {
    const int rr = e / (2 * DW_PADL), j = e - rr * (2 * DW_PADL);
    lds[rr * WP + (j < DW_PADL ? j : W + j)] = 0.f;
  }
}

// One lane's LDS window row v[0 .. NV) starting at `base`.  OFF >= 0: base sits OFF floats past a
// 16-B boundary (OFF = -pl mod 4: the staged rows start 16-B aligned, every lane's first
// output column is a multiple of 4), and the row is read as ceil((OFF + NV) / 4) ds_read_b128
// from that boundary: 4 lane groups of 16 consecutive 16-B words, conflict-free, where the
// scalar reads (OFF = -1, e2ep_tune key 23 = 1) land lanes 8 apart on one bank (4-way) at
// 1 or 2 floats per instruction.  The words read past the window stay inside the staged row
// (its right halo), since the row pitch is a multiple of 4.
template <int NV, int OFF>
__device__ __forceinline__ void dw_row(const float *base, float (&v)[NV]) {
  if constexpr (OFF < 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = base[j];
  } else {
    constexpr int NF = (OFF + NV + 3) / 4;
    const float4 *p = reinterpret_cast<const float4 *>(base - OFF);
    float f[4 * NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const float4 t = p[i];
      f[4 * i] = t.x;
      f[4 * i + 1] = t.y;
      f[4 * i + 2] = t.z;
      f[4 * i + 3] = t.w;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = f[OFF + j];
  }
}

// V: float4 per lane that hold a unit's staged rows (2 or DW_MAXV; the host picks the
// smallest that covers IR * W / 4, so short units keep fewer registers and more waves resident)
// BS: BatchNorm partial sums of y for the BN that follows (MBConv _bn1), one fp64 (sum, sum of
// squares) pair per unit (a lane's 4 outputs in fp32, the wave's 64 lanes in fp64), written by
// the unit's wave, tile-major like bnstats.h: tile = n * units_per_plane + row block,
// stats[(tile * C + c) * 2].
__device__ __forceinline__ double dw_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// bf16 activation storage (B, e2ep.h E2EP_IO_*): the forward's output y (the MBConv depthwise
// output, read by the squeeze-excitation and the _bn1 backward) and, in the backward, the
// incoming gradient gy and the data gradient dx are bf16; the forward's input (the raw expand
// conv output, normalised on load) stays fp32.  FLIP (the stride-1 data gradient) reads gy.
template <bool FLIP, bool B>
using dw_ti = std::conditional_t<FLIP && B, bf16_t, float>;
template <bool B>
using dw_to = std::conditional_t<B, bf16_t, float>;

// The block body for block blk of nblk (k_dw_fwd_strip, and the data-gradient half of
// k_dw_bwd_pair), over the kernel's dynamic LDS.  BS statistics are of the stored (rounded)
// values.
template <int K, int ST, bool FLIP, int OFF, int V, bool BS = false, bool B = false>
__device__ __forceinline__ void dw_fwd_strip_body(const dw_ti<FLIP, B> *__restrict__ x,
                                                  const float *__restrict__ w, DwGeom g, DwStrip d,
                                                  int units, dw_to<B> *__restrict__ y, DwIn tf,
                                                  double *__restrict__ stats, int blk, int nblk) {
  extern __shared__ float dw_lds[];
  // Grid-stride over units, software-pipelined like k_dw_wgrad_strip: the wave's next unit's
  // input rows are loaded into registers before the current unit's FMAs (one unit per wave
  // with stage / wait / compute in series ran at 1.7-3.5 TB/s).  The grid is capped at
  // e2ep_tune key 24 blocks, so each wave walks several units.
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR descriptors
  float *lds = dw_lds + wave * d.IR * d.WP;
  const int QL = g.Q >> 2;  // lanes per output row
  const int ro = lane / QL, ox0 = 4 * (lane - ro * QL);
  constexpr int NV = 3 * ST + K;
  const int step = nblk * 4;
  int u = blk * 4 + wave;  // wave-uniform
  int nc = 0, oy0 = 0;
  auto unit_of = [&](int un) {
    nc = un / d.units_per_plane;
    oy0 = (un - nc * d.units_per_plane) * d.RO;
  };
  float4 rx[V];
  if (u < units) unit_of(u);
  dw_fetch(x + (size_t)nc * g.H * g.W, g.H, g.W, oy0 * ST - g.pt, d.IR, lane, rx, u < units);
  for (; u < units; u += step) {
    const int c = nc % g.C;
    dw_put(rx, g.H, g.W, oy0 * ST - g.pt, d.IR, d.WP, lds, lane, dw_t(tf, c));
    const int cur_nc = nc, cur_oy0 = oy0;
    const bool nxt = u + step < units;
    if (nxt) unit_of(u + step);
    dw_fetch(x + (size_t)nc * g.H * g.W, g.H, g.W, oy0 * ST - g.pt, d.IR, lane, rx, nxt);
    float wr[K * K];
#pragma unroll
    for (int t = 0; t < K * K; ++t) wr[t] = w[c * K * K + (FLIP ? K * K - 1 - t : t)];
    dw_wave_sync();
    const int oy = cur_oy0 + ro;
    const bool live = ro < d.RO && oy < g.P;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    if (live) {
      const float *base = lds + (ro * ST) * d.WP + DW_PADL + ox0 * ST - g.pl;
#pragma unroll
      for (int a = 0; a < K; ++a) {
        float v[NV];
        dw_row<NV, OFF>(base + a * d.WP, v);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int b = 0; b < K; ++b) o[q] = __builtin_fmaf(wr[a * K + b], v[q * ST + b], o[q]);
      }
      st4(y + ((size_t)cur_nc * g.P + oy) * g.Q + ox0, make_float4(o[0], o[1], o[2], o[3]));
    }
    if (BS) {  // BatchNorm partials (separate instantiation)
      float f1 = 0.f, f2 = 0.f;
      if (live) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = stored<dw_to<B>>(o[q]);
          f1 += v;
          f2 = __builtin_fmaf(v, v, f2);
        }
      }
      const double s1 = dw_wave_sum((double)f1);
      const double s2 = dw_wave_sum((double)f2);
      if (lane == 0) {
        const int n = cur_nc / g.C, c = cur_nc - n * g.C;
        const size_t at = (((size_t)n * d.units_per_plane + cur_oy0 / d.RO) * g.C + c) * 2;
        stats[at] = s1;
        stats[at + 1] = s2;
      }
    }
    dw_wave_sync();  // LDS reuse
  }
}

template <int K, int ST, bool FLIP, int OFF, int V, bool BS = false, bool B = false>
__global__ void __launch_bounds__(256) k_dw_fwd_strip(const dw_ti<FLIP, B> *__restrict__ x,
                                                      const float *__restrict__ w, DwGeom g,
                                                      DwStrip d, int units, dw_to<B> *__restrict__ y,
                                                      DwIn tf, double *__restrict__ stats) {
  dw_fwd_strip_body<K, ST, FLIP, OFF, V, BS, B>(x, w, g, d, units, y, tf, stats, blockIdx.x,
                                                gridDim.x);
}

// stride-2 data gradient over strip units: a wave owns RO = 64/(W/4) rows of dx of one plane,
// each lane 4 adjacent dx pixels; the gy rows those rows read are staged in LDS.  For dx
// pixel ix only taps b with (ix + pl - b) even contribute; ix0 is a multiple of 4, so the
// parity of (u + pl - b) is compile-time given PLP = pl & 1.
// The block body for block blk (k_dw_dgrad_s2_strip, and the data-gradient half of
// k_dw_bwd_pair_s2), over the kernel's dynamic LDS.
template <int K, int PLP, bool B = false>
__device__ __forceinline__ void dw_dgrad_s2_body(const dw_to<B> *__restrict__ gy,
                                                 const float *__restrict__ w, DwGeom g, int RO,
                                                 int GR, int WPg, int units_per_plane, int units,
                                                 dw_to<B> *__restrict__ dx, int blk) {
  extern __shared__ float dw_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR descriptors
  const int unit = blk * 4 + wave;
  float *lds = dw_lds + wave * GR * WPg;
  const bool active = unit < units;
  int nc = 0, iy0 = 0, oyA = 0;
  if (active) {
    nc = unit / units_per_plane;
    iy0 = (unit - nc * units_per_plane) * RO;
    oyA = (iy0 + g.pt - (K - 1)) >> 1;  // floor division by 2
    dw_stage(gy + (size_t)nc * g.P * g.Q, g.P, g.Q, oyA, GR, WPg, lds, lane);
  }
  dw_wave_sync();
  if (!active) return;
  const int c = nc % g.C;
  float wr[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) wr[t] = w[c * K * K + t];
  const int WL = g.W >> 2;
  const int r = lane / WL, ix0 = 4 * (lane - r * WL);
  const int iy = iy0 + r;
  if (r >= RO || iy >= g.H) return;
  const int xoff = (ix0 >> 1) + ((g.pl - PLP) >> 1) + DW_PADL;
  float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int ny = iy + g.pt - a;
    if (ny & 1) continue;
    const float *row = lds + ((ny >> 1) - oyA) * WPg + xoff;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int b = 0; b < K; ++b)
        if (((u + PLP - b) & 1) == 0) o[u] = __builtin_fmaf(wr[a * K + b], row[(u + PLP - b) >> 1], o[u]);
  }
  st4(dx + ((size_t)nc * g.H + iy) * g.W + ix0, make_float4(o[0], o[1], o[2], o[3]));
}

template <int K, int PLP, bool B = false>
__global__ void __launch_bounds__(256) k_dw_dgrad_s2_strip(const dw_to<B> *__restrict__ gy,
                                                           const float *__restrict__ w, DwGeom g,
                                                           int RO, int GR, int WPg,
                                                           int units_per_plane, int units,
                                                           dw_to<B> *__restrict__ dx) {
  dw_dgrad_s2_body<K, PLP, B>(gy, w, g, RO, GR, WPg, units_per_plane, units, dx, blockIdx.x);
}

// weight gradient partials over strip units: grid (C, splits); the block's waves walk the
// channel's units (n, strip) of its slice; per lane K*K register accumulators, fixed-order
// wave + block reduction.
// The block body for channel c, split sp (k_dw_wgrad_strip, and the weight-gradient half of
// k_dw_bwd_pair), over the kernel's dynamic LDS.
template <int K, int ST, int OFF, int V, bool B = false>
__device__ __forceinline__ void dw_wgrad_strip_body(const dw_to<B> *__restrict__ gy,
                                                    const float *__restrict__ x, DwGeom g,
                                                    DwStrip d, int splits, DwPart part, DwIn tf,
                                                    int c, int sp) {
  extern __shared__ float dw_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR descriptors
  float *lds = dw_lds + wave * d.IR * d.WP;
  const int cunits = g.N * d.units_per_plane;  // units of this channel
  const int per = (cunits + splits - 1) / splits;
  const int beg = sp * per, end = min(cunits, beg + per);
  const int QL = g.Q >> 2;
  const int ro = lane / QL, ox0 = 4 * (lane - ro * QL);
  constexpr int NV = 3 * ST + K;
  float acc[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) acc[t] = 0.f;
  // Software-pipelined over the wave's units (u0 + wave, u0 + wave + 4, ...): the next unit's
  // input rows and gy row are loaded into registers before the current unit's FMAs, so the
  // load latency overlaps compute (the wave used to stage, wait, compute, one unit at a time:
  // 1.2-2.1 TB/s).  Up to DW_MAXV float4 per lane per unit (host-checked).
  auto unit_of = [&](int un, int &n, int &oy0) {
    n = un / d.units_per_plane;
    oy0 = (un - n * d.units_per_plane) * d.RO;
  };
  float4 rx[V];
  float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int GB = sizeof(dw_to<B>);  // bytes per gy element
  const __amdgpu_buffer_rsrc_t rgy = rsrc(gy, (long long)GB * g.N * g.C * g.P * g.Q);
  int n = 0, oy0 = 0;
  bool active = beg + wave < end;
  if (active) unit_of(beg + wave, n, oy0);
  auto fetch = [&](bool act, int nn, int yy0) {
    dw_fetch(x + ((size_t)nn * g.C + c) * g.H * g.W, g.H, g.W, yy0 * ST - g.pt, d.IR, lane, rx, act);
    const int oy = yy0 + ro;
    const bool ok = act && ro < d.RO && oy < g.P;
    gq = bload4t(rgy, ok ? (((nn * g.C + c) * g.P + oy) * g.Q + ox0) * GB : OOR, gy);
  };
  const DwT tfc = dw_t(tf, c);  // the block's channel: read once
  fetch(active, n, oy0);
  for (int u0 = beg; u0 < end; u0 += 4) {
    dw_put(rx, g.H, g.W, oy0 * ST - g.pt, d.IR, d.WP, lds, lane, tfc);
    const float gv[4] = {gq.x, gq.y, gq.z, gq.w};
    const bool cur_active = active;
    const int cur_oy0 = oy0;
    // next unit of this wave: its loads fly while this unit computes
    const bool nxt = u0 + 4 + wave < end;
    int nn = 0, noy0 = 0;
    if (nxt) unit_of(u0 + 4 + wave, nn, noy0);
    fetch(nxt, nn, noy0);
    active = nxt;
    n = nn;
    oy0 = noy0;
    dw_wave_sync();
    const int oy = cur_oy0 + ro;
    if (cur_active && ro < d.RO && oy < g.P) {
      const float *base = lds + (ro * ST) * d.WP + DW_PADL + ox0 * ST - g.pl;
#pragma unroll
      for (int a = 0; a < K; ++a) {
        float v[NV];
        dw_row<NV, OFF>(base + a * d.WP, v);
#pragma unroll
        for (int b = 0; b < K; ++b)
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[a * K + b] = __builtin_fmaf(gv[u], v[u * ST + b], acc[a * K + b]);
      }
    }
    dw_wave_sync();  // LDS reuse
  }
  __shared__ float red[4][K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float v = wave_sum(acc[t]);
    if (lane == 0) red[wave][t] = v;
  }
  __syncthreads();
  const int t = threadIdx.x < K * K ? threadIdx.x : 0;
  // the last-arriver flag reuses red[0][0] (read above, before dw_wgrad_out's first barrier):
  // a static __shared__ int would leave the kernel's static LDS at 4 mod 16 bytes and shift the
  // strip kernels' dynamic LDS base off 16-B alignment (their b128 window reads then replay:
  // 1.5 - 2x slower; cdna_hip_programming.md Guideline 17)
  dw_wgrad_out<K * K>(part, c, sp, splits, (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]),
                      reinterpret_cast<int *>(&red[0][0]));
}

template <int K, int ST, int OFF, int V, bool B = false>
__global__ void __launch_bounds__(256) k_dw_wgrad_strip(const dw_to<B> *__restrict__ gy,
                                                        const float *__restrict__ x, DwGeom g,
                                                        DwStrip d, int splits,
                                                        DwPart part, DwIn tf) {
  dw_wgrad_strip_body<K, ST, OFF, V, B>(gy, x, g, d, splits, part, tf, blockIdx.x, blockIdx.y);
}

// A stride-1 depthwise layer's data gradient (the flipped-filter strip forward over gy, gt /
// dt its geometry) and weight gradient (strip partials, g / d) in one grid: block c + C * sp
// (< nw = C * splits) the weight gradient of channel c, split sp, the nd blocks after them
// walk the data-gradient units grid-stride.  The weight-gradient blocks go first: each walks
// a channel's units of its split (tens per wave) and ends in a block reduction, the long
// poles of the launch; queued behind the data-gradient blocks they ran last and serial
// (67.5 us against 52 us for the weight gradient alone).  One launch instead of two on
// forked streams (e2ep_dwconv_bwd): in a replayed graph the fork / join idles the GPU ~17 us
// per layer.  Dynamic LDS: the larger of the two halves' per-wave row buffers.
template <int K, int OFF, int VD, int VW, bool B = false>
__global__ void __launch_bounds__(256) k_dw_bwd_pair(const dw_to<B> *__restrict__ gy,
                                                     const float *__restrict__ w, DwGeom gt,
                                                     DwStrip dt, int units, dw_to<B> *__restrict__ dx,
                                                     int nd, const float *__restrict__ x, DwGeom g,
                                                     DwStrip d, int splits, DwPart part, DwIn tf) {
  const int b = blockIdx.x, nw = g.C * splits;
  if (b < nw) {
    dw_wgrad_strip_body<K, 1, OFF, VW, B>(gy, x, g, d, splits, part, tf, b % g.C, b / g.C);
  } else {
    dw_fwd_strip_body<K, 1, true, OFF, VD, false, B>(gy, w, gt, dt, units, dx,
                                                     DwIn{nullptr, nullptr, 0}, nullptr, b - nw, nd);
  }
}

// The stride-2 form of k_dw_bwd_pair: weight-gradient blocks first (channel c, split sp), then
// the k_dw_dgrad_s2_strip blocks (one unit per wave).
template <int K, int PLP, int OFF, int VW, bool B = false>
__global__ void __launch_bounds__(256) k_dw_bwd_pair_s2(const dw_to<B> *__restrict__ gy,
                                                        const float *__restrict__ w, int RO, int GR,
                                                        int WPg, int upp2, int units2,
                                                        dw_to<B> *__restrict__ dx,
                                                        const float *__restrict__ x, DwGeom g,
                                                        DwStrip d, int splits, DwPart part, DwIn tf) {
  const int b = blockIdx.x, nw = g.C * splits;
  if (b < nw)
    dw_wgrad_strip_body<K, 2, OFF, VW, B>(gy, x, g, d, splits, part, tf, b % g.C, b / g.C);
  else
    dw_dgrad_s2_body<K, PLP, B>(gy, w, g, RO, GR, WPg, upp2, units2, dx, b - nw);
}

static int dw_splits(long long pixels, int C) {
  long long want = (1024 + C - 1) / C;
  long long cap = pixels / 2048;
  long long s = want < cap ? want : cap;
  return (int)(s < 1 ? 1 : (s > 128 ? 128 : s));
}

static DwGeom dw_geom(const int *d) {
  DwGeom g;
  g.N = d[0]; g.C = d[1]; g.H = d[2]; g.W = d[3]; g.K = d[4]; g.P = d[5]; g.Q = d[6];
  g.st = d[7]; g.pt = d[8]; g.pl = d[9];
  return g;
}

}  // namespace e2ep

using namespace e2ep;

#define DW_DISPATCH(KERNEL, GRID, ...)                                                        \
  do {                                                                                        \
    if (g.K == 3 && g.st == 1)                                                                \
      hipLaunchKernelGGL((KERNEL<3, 1>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else if (g.K == 3 && g.st == 2)                                                           \
      hipLaunchKernelGGL((KERNEL<3, 2>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else if (g.K == 5 && g.st == 1)                                                           \
      hipLaunchKernelGGL((KERNEL<5, 1>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else if (g.K == 5 && g.st == 2)                                                           \
      hipLaunchKernelGGL((KERNEL<5, 2>), GRID, dim3(256), 0, as_stream(stream), __VA_ARGS__); \
    else {                                                                                    \
      set_error("depthwise conv: kernel %d / stride %d unsupported (k 3|5, s 1|2)", g.K, g.st); \
      return E2EP_ERANGE;                                                                     \
    }                                                                                         \
  } while (0)

// the strip kernels' LDS row-read variant: dw_row's OFF for left pad pl, or -1 (scalar reads)
// grid of the forward strip kernel: one unit per wave up to e2ep_tune key 24 blocks
static int dw_fwd_blocks(int units) { return std::min(cdiv(units, 4), g_tune[TUNE_DW_FWD_BLOCKS]); }
static int dw_off(int pl) { return g_tune[TUNE_DW_VEC] == 1 ? -1 : ((-pl) & 3); }

// launch a strip kernel with the row-read variant `off` as its compile-time OFF and the
// staging registers V = 2 float4 per lane when `nv` (float4 per lane a unit needs) allows
// (the scalar-read variant, an A/B switch, always takes DW_MAXV)
template <int K, int ST, bool FLIP, int V, bool B>
static void dw_fwd_strip_v(int off, dim3 grid, size_t shm, hipStream_t st, const void *xv,
                           const float *w, DwGeom g, DwStrip d, int units, void *yv, DwIn tf,
                           double *stats) {
  const auto *x = static_cast<const dw_ti<FLIP, B> *>(xv);
  auto *y = static_cast<dw_to<B> *>(yv);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), shm, st, x, w, g, d, units, y, tf, stats);
  };
  if (stats && !FLIP) {
    switch (off) {
      case 0: go(k_dw_fwd_strip<K, ST, FLIP, 0, V, true, B>); break;
      case 1: go(k_dw_fwd_strip<K, ST, FLIP, 1, V, true, B>); break;
      case 2: go(k_dw_fwd_strip<K, ST, FLIP, 2, V, true, B>); break;
      default: go(k_dw_fwd_strip<K, ST, FLIP, 3, V, true, B>);
    }
    return;
  }
  switch (off) {
    case 0: go(k_dw_fwd_strip<K, ST, FLIP, 0, V, false, B>); break;
    case 1: go(k_dw_fwd_strip<K, ST, FLIP, 1, V, false, B>); break;
    case 2: go(k_dw_fwd_strip<K, ST, FLIP, 2, V, false, B>); break;
    default: go(k_dw_fwd_strip<K, ST, FLIP, 3, V, false, B>);
  }
}
template <int K, int ST, bool FLIP, bool B>
static void dw_fwd_strip(int off, int nv, dim3 grid, size_t shm, hipStream_t st, const void *xv,
                         const float *w, DwGeom g, DwStrip d, int units, void *yv, DwIn tf,
                         double *stats) {
  const auto *x = static_cast<const dw_ti<FLIP, B> *>(xv);
  auto *y = static_cast<dw_to<B> *>(yv);
  if (off < 0 && stats && !FLIP)
    hipLaunchKernelGGL((k_dw_fwd_strip<K, ST, FLIP, -1, DW_MAXV, true, B>), grid, dim3(256), shm, st,
                       x, w, g, d, units, y, tf, stats);
  else if (off < 0)
    hipLaunchKernelGGL((k_dw_fwd_strip<K, ST, FLIP, -1, DW_MAXV, false, B>), grid, dim3(256), shm, st,
                       x, w, g, d, units, y, tf, nullptr);
  else if (nv <= 2)
    dw_fwd_strip_v<K, ST, FLIP, 2, B>(off, grid, shm, st, xv, w, g, d, units, yv, tf, stats);
  else
    dw_fwd_strip_v<K, ST, FLIP, DW_MAXV, B>(off, grid, shm, st, xv, w, g, d, units, yv, tf, stats);
}
template <int K, int ST, int V, bool B>
static void dw_wgrad_strip_v(int off, dim3 grid, size_t shm, hipStream_t st, const void *gyv,
                             const float *x, DwGeom g, DwStrip d, int splits, DwPart part, DwIn tf) {
  const auto *gy = static_cast<const dw_to<B> *>(gyv);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(256), shm, st, gy, x, g, d, splits, part, tf); };
  switch (off) {
    case 0: go(k_dw_wgrad_strip<K, ST, 0, V, B>); break;
    case 1: go(k_dw_wgrad_strip<K, ST, 1, V, B>); break;
    case 2: go(k_dw_wgrad_strip<K, ST, 2, V, B>); break;
    default: go(k_dw_wgrad_strip<K, ST, 3, V, B>);
  }
}
template <int K, int ST, bool B>
static void dw_wgrad_strip(int off, int nv, dim3 grid, size_t shm, hipStream_t st, const void *gyv,
                           const float *x, DwGeom g, DwStrip d, int splits, DwPart part, DwIn tf) {
  if (off < 0)
    hipLaunchKernelGGL((k_dw_wgrad_strip<K, ST, -1, DW_MAXV, B>), grid, dim3(256), shm, st,
                       static_cast<const dw_to<B> *>(gyv), x, g, d, splits, part, tf);
  else if (nv <= 2)
    dw_wgrad_strip_v<K, ST, 2, B>(off, grid, shm, st, gyv, x, g, d, splits, part, tf);
  else
    dw_wgrad_strip_v<K, ST, DW_MAXV, B>(off, grid, shm, st, gyv, x, g, d, splits, part, tf);
}

extern "C" {

static bool dw_strip_ok(const DwGeom &g) {
  if (!(g.Q % 4 == 0 && g.Q <= 256 && g.W % 4 == 0 && (g.K == 3 || g.K == 5) &&
        (g.st == 1 || g.st == 2)))
    return false;
  const DwStrip d = dw_strip(g.K, g.st, g.W, g.P, g.Q);
  return d.IR * (g.W / 4) <= 64 * DW_MAXV;  // the unrolled staging's reach
}

#define DW_STRIP_DISPATCH(LAUNCHER, FLIPARG, GRID, SHMEM, ...)                                   \
  do {                                                                                         \
    const int off = dw_off(g.pl);                                                              \
    const int nv = cdiv(d.IR * (g.W / 4), 64);                                                 \
    if (g.K == 3 && g.st == 1)                                                                 \
      LAUNCHER<3, 1 FLIPARG>(off, nv, GRID, SHMEM, as_stream(stream), __VA_ARGS__);                \
    else if (g.K == 3 && g.st == 2)                                                            \
      LAUNCHER<3, 2 FLIPARG>(off, nv, GRID, SHMEM, as_stream(stream), __VA_ARGS__);                \
    else if (g.K == 5 && g.st == 1)                                                            \
      LAUNCHER<5, 1 FLIPARG>(off, nv, GRID, SHMEM, as_stream(stream), __VA_ARGS__);                \
    else                                                                                       \
      LAUNCHER<5, 2 FLIPARG>(off, nv, GRID, SHMEM, as_stream(stream), __VA_ARGS__);                \
  } while (0)
#define DW_NOFLIP , false, false
#define DW_NOFLIP_B16 , false, true
#define DW_NONE , false
#define DW_B16 , true

// dims[10] = {N, C, H, W, K, P, Q, stride, pad_top, pad_left}
int e2ep_dwconv_fwd_stats_tiles(const int *dims) {
  const DwGeom g = dw_geom(dims);
  if (!(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0) || !dw_strip_ok(g)) return 0;
  return g.N * dw_strip(g.K, g.st, g.W, g.P, g.Q).units_per_plane;
}

int e2ep_dwconv_fwd(const float *x, const float *w, const int *dims, const float *in_scale,
                    const float *in_shift, int in_act, float *y, void *stream) {
  return e2ep_dwconv_fwd_stats(x, w, dims, in_scale, in_shift, in_act, y, nullptr, 0, stream, 0);
}

int e2ep_dwconv_fwd_stats(const float *x, const float *w, const int *dims, const float *in_scale,
                          const float *in_shift, int in_act, void *y, double *stats,
                          size_t stats_bytes, void *stream, int io) {
  DwGeom g = dw_geom(dims);
  E2EP_REQUIRE(io == 0 || (io == E2EP_IO_DX_BF16 && dw_strip_ok(g)), E2EP_EINVAL,
               "e2ep_dwconv_fwd_stats: storage mask %d not supported (0, or y bf16 on the strip "
               "kernels)", io);
  if (stats) {
    const int tiles = e2ep_dwconv_fwd_stats_tiles(dims);
    E2EP_REQUIRE(tiles > 0, E2EP_EINVAL,
                 "e2ep_dwconv_fwd_stats: this geometry's kernel takes no statistics");
    E2EP_REQUIRE(stats_bytes >= (size_t)g.C * tiles * 2 * sizeof(double), E2EP_EINVAL,
                 "e2ep_dwconv_fwd_stats: stats %zu bytes < %zu (C x tiles x 2 doubles)",
                 stats_bytes, (size_t)g.C * tiles * 2 * sizeof(double));
  }
  E2EP_REQUIRE(!in_scale == !in_shift && in_act >= 0 && in_act <= 2, E2EP_EINVAL,
               "e2ep_dwconv_fwd: in_scale / in_shift both or neither, in_act 0..2");
  const DwIn tf{in_scale, in_shift, in_act};
  E2EP_REQUIRE(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0, E2EP_EINVAL,
               "e2ep_dwconv_fwd: bad geometry");
  if (dw_strip_ok(g)) {
    const DwStrip d = dw_strip(g.K, g.st, g.W, g.P, g.Q);
    const int units = g.N * g.C * d.units_per_plane;
    if (io)
      DW_STRIP_DISPATCH(dw_fwd_strip, DW_NOFLIP_B16, dim3(dw_fwd_blocks(units)), 4 * d.IR * d.WP * 4,
                        x, w, g, d, units, y, tf, stats);
    else
      DW_STRIP_DISPATCH(dw_fwd_strip, DW_NOFLIP, dim3(dw_fwd_blocks(units)), 4 * d.IR * d.WP * 4, x,
                        w, g, d, units, y, tf, stats);
    return launch_status("e2ep_dwconv_fwd");
  }
  E2EP_REQUIRE(g.N * g.C <= 65535, E2EP_ERANGE, "e2ep_dwconv_fwd: N*C > 65535");
  DW_DISPATCH(k_dw_fwd, dim3(cdiv(g.P * g.Q, 256), g.N * g.C), x, w, g, static_cast<float *>(y),
              in_scale, in_shift, in_act);
  return launch_status("e2ep_dwconv_fwd");
}

// The stride-2 data-gradient strip plan of e2ep_dwconv_dgrad (RO output rows per unit, GR gy
// rows staged); false where that entry point runs the generic kernel.
struct DwS2 {
  int RO, GR, WPg, upp, units;
};
static bool dw_s2_plan(const DwGeom &g, DwS2 &p) {
  if (!(g.st == 2 && g.W % 4 == 0 && g.W <= 256 && g.Q % 4 == 0 && (g.K == 3 || g.K == 5) &&
        g.pl <= 2 && g.pt <= 2))
    return false;
  p.RO = 64 / (g.W / 4);
  p.GR = ((p.RO - 1 + g.pt) >> 1) - ((g.pt - (g.K - 1)) >> 1) + 2;
  if (p.GR * (g.Q / 4) > 64 * DW_MAXV) return false;
  p.WPg = g.Q + 2 * DW_PADL;
  p.upp = (g.H + p.RO - 1) / p.RO;
  p.units = g.N * g.C * p.upp;
  return true;
}

int e2ep_dwconv_dgrad(const void *gy, const float *w, const int *dims, void *dx, void *stream,
                      int io) {
  DwGeom g = dw_geom(dims);
  E2EP_REQUIRE(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0, E2EP_EINVAL,
               "e2ep_dwconv_dgrad: bad geometry");
  E2EP_REQUIRE(io == 0 || io == (E2EP_IO_DY_BF16 | E2EP_IO_DX_BF16), E2EP_EINVAL,
               "e2ep_dwconv_dgrad: storage mask %d not supported (0 or DY|DX bf16)", io);
  if (g.st == 1) {
    // stride 1: dx = gy (P x Q) correlated with the flipped filter, pads K-1-pad, output H x W
    DwGeom t = g;
    t.H = g.P; t.W = g.Q; t.P = g.H; t.Q = g.W;
    t.pt = g.K - 1 - g.pt; t.pl = g.K - 1 - g.pl;
    if (dw_strip_ok(t) && t.pt >= 0 && t.pl >= 0 && t.pl <= DW_PADL) {
      const DwStrip d = dw_strip(t.K, 1, t.W, t.P, t.Q);
      const int units = t.N * t.C * d.units_per_plane;
      const size_t shm = 4 * d.IR * d.WP * 4;
      const DwIn none{nullptr, nullptr, 0};
      const int nv = cdiv(d.IR * (t.W / 4), 64);
      const dim3 grid(dw_fwd_blocks(units));
      hipStream_t s = as_stream(stream);
      if (t.K == 3 && io)
        dw_fwd_strip<3, 1, true, true>(dw_off(t.pl), nv, grid, shm, s, gy, w, t, d, units, dx, none, nullptr);
      else if (t.K == 3)
        dw_fwd_strip<3, 1, true, false>(dw_off(t.pl), nv, grid, shm, s, gy, w, t, d, units, dx, none, nullptr);
      else if (io)
        dw_fwd_strip<5, 1, true, true>(dw_off(t.pl), nv, grid, shm, s, gy, w, t, d, units, dx, none, nullptr);
      else
        dw_fwd_strip<5, 1, true, false>(dw_off(t.pl), nv, grid, shm, s, gy, w, t, d, units, dx, none, nullptr);
      return launch_status("e2ep_dwconv_dgrad");
    }
  }
  DwS2 p2;
  if (dw_s2_plan(g, p2)) {
    const int RO = p2.RO, GR = p2.GR, WPg = p2.WPg, upp = p2.upp, units = p2.units;
    const size_t shm = 4 * GR * WPg * sizeof(float);
    const dim3 grid(cdiv(units, 4));
    const bool odd = g.pl & 1;
#define DWS2(KV, PV, BV)                                                                           \
  hipLaunchKernelGGL((k_dw_dgrad_s2_strip<KV, PV, BV>), grid, dim3(256), shm, as_stream(stream),      \
                     static_cast<const dw_to<BV> *>(gy), w, g, RO, GR, WPg, upp, units,             \
                     static_cast<dw_to<BV> *>(dx))
    if (g.K == 3 && !odd) { if (io) DWS2(3, 0, true); else DWS2(3, 0, false); }
    else if (g.K == 3) { if (io) DWS2(3, 1, true); else DWS2(3, 1, false); }
    else if (!odd) { if (io) DWS2(5, 0, true); else DWS2(5, 0, false); }
    else { if (io) DWS2(5, 1, true); else DWS2(5, 1, false); }
#undef DWS2
    return launch_status("e2ep_dwconv_dgrad");
  }
  E2EP_REQUIRE(io == 0, E2EP_EINVAL, "e2ep_dwconv_dgrad: bf16 storage needs the strip kernels");
  E2EP_REQUIRE(g.N * g.C <= 65535, E2EP_ERANGE, "e2ep_dwconv_dgrad: N*C > 65535");
  DW_DISPATCH(k_dw_dgrad, dim3(cdiv(g.H * g.W, 256), g.N * g.C), static_cast<const float *>(gy), w, g,
              static_cast<float *>(dx));
  return launch_status("e2ep_dwconv_dgrad");
}

// the pipelined weight-gradient strip kernel holds a unit's input rows in registers
static bool dw_wgrad_strip_ok(const DwGeom &g) {
  if (!dw_strip_ok(g)) return false;
  const DwStrip d = dw_strip(g.K, g.st, g.W, g.P, g.Q);
  return d.IR * (g.W / 4) <= 64 * DW_MAXV;
}

static int dw_wgrad_splits(const DwGeom &g) {
  if (dw_wgrad_strip_ok(g)) {
    const DwStrip d = dw_strip(g.K, g.st, g.W, g.P, g.Q);
    const int cunits = g.N * d.units_per_plane;
    int want = (g_tune[TUNE_DW_WGRAD_TARGET] + g.C - 1) / g.C;  // e2ep_tune key 3 / 5
    int cap = (cunits + 7) / 8;                   // >= 8 units (2 per wave) each
    int s = want < cap ? want : cap;
    return s < 1 ? 1 : (s > 128 ? 128 : s);
  }
  return dw_splits((long long)g.N * g.P * g.Q, g.C);
}

// The stride-2 paired backward's plan: both strip kernels, weight-gradient row reads at an
// instantiated (K, pad_left): K = 3 pad 0 / 1, K = 5 pad 1 / 2.  Not for data gradients of
// more than DW_S2_PAIR_UNITS units: the 128 x 128-map layer (294 912 units) ran 220 us paired
// against ~183 us as two forked launches, while the 43 008- and 98 304-unit layers ran 37 / 87
// us paired against ~44 / ~86 us forked (step_sequence_fp32_final.txt against _r4z.txt).
constexpr int DW_S2_PAIR_UNITS = 131072;
static bool dw_bwd_pair_s2_plan(const DwGeom &g, DwS2 &p) {
  if (g.st != 2 || g_tune[TUNE_DW_VEC] == 1 || !dw_wgrad_strip_ok(g) || !dw_s2_plan(g, p) ||
      p.units > DW_S2_PAIR_UNITS)
    return false;
  return (g.K == 3 && (g.pl == 0 || g.pl == 1)) || (g.K == 5 && (g.pl == 1 || g.pl == 2));
}

// The paired backward's plan (stride 1, both strip kernels, vector row reads with one OFF for
// both halves: symmetric padding, K = 3 pad 1 -> 3, K = 5 pad 2 -> 2).
static bool dw_bwd_pair_plan(const DwGeom &g, DwGeom &t, int &off) {
  if (g.st != 1 || g_tune[TUNE_DW_VEC] == 1 || !dw_wgrad_strip_ok(g)) return false;
  t = g;
  t.H = g.P; t.W = g.Q; t.P = g.H; t.Q = g.W;
  t.pt = g.K - 1 - g.pt; t.pl = g.K - 1 - g.pl;
  if (!(dw_strip_ok(t) && t.pt >= 0 && t.pl >= 0 && t.pl <= DW_PADL)) return false;
  off = dw_off(g.pl);
  return off == dw_off(t.pl) && ((g.K == 3 && off == 3) || (g.K == 5 && off == 2));
}

int e2ep_dwconv_bwd_pair_ok(const int *dims) {
  const DwGeom g = dw_geom(dims);
  DwGeom t;
  int off;
  DwS2 p2;
  return (g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0 &&
          (dw_bwd_pair_plan(g, t, off) || dw_bwd_pair_s2_plan(g, p2))) ? 1 : 0;
}

int e2ep_dwconv_bf16_ok(const int *dims) {
  const DwGeom g = dw_geom(dims);
  if (!(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0)) return 0;
  if (!dw_strip_ok(g) || !dw_wgrad_strip_ok(g)) return 0;  // forward y, weight-gradient gy
  if ((g.H * g.W) % 4 != 0 || (g.P * g.Q) % 4 != 0) return 0;  // the BatchNorms beside it
  if (g.st == 1) {  // the stride-1 data gradient's strip path (e2ep_dwconv_dgrad)
    DwGeom t = g;
    t.H = g.P; t.W = g.Q; t.P = g.H; t.Q = g.W;
    t.pt = g.K - 1 - g.pt; t.pl = g.K - 1 - g.pl;
    return (dw_strip_ok(t) && t.pt >= 0 && t.pl >= 0 && t.pl <= DW_PADL) ? 1 : 0;
  }
  DwS2 p2;
  return dw_s2_plan(g, p2) ? 1 : 0;  // the stride-2 data gradient's strip path
}

size_t e2ep_dwconv_wgrad_workspace(const int *dims) {
  DwGeom g = dw_geom(dims);
  return (size_t)g.C * dw_wgrad_splits(g) * g.K * g.K * sizeof(float);
}

int e2ep_dwconv_wgrad(const void *gy, const float *x, const int *dims, const float *in_scale,
                      const float *in_shift, int in_act, void *workspace, size_t workspace_bytes,
                      float *dw, void *stream, int io) {
  DwGeom g = dw_geom(dims);
  E2EP_REQUIRE(io == 0 || (io == E2EP_IO_DY_BF16 && dw_wgrad_strip_ok(g)), E2EP_EINVAL,
               "e2ep_dwconv_wgrad: storage mask %d not supported (0, or gy bf16 on the strip "
               "kernels)", io);
  E2EP_REQUIRE(workspace && workspace_bytes >= e2ep_dwconv_wgrad_workspace(dims), E2EP_EINVAL,
               "e2ep_dwconv_wgrad: workspace %zu bytes < %zu (e2ep_dwconv_wgrad_workspace)",
               workspace_bytes, e2ep_dwconv_wgrad_workspace(dims));
  E2EP_REQUIRE(!in_scale == !in_shift && in_act >= 0 && in_act <= 2, E2EP_EINVAL,
               "e2ep_dwconv_wgrad: in_scale / in_shift both or neither, in_act 0..2");
  const DwIn tf{in_scale, in_shift, in_act};
  E2EP_REQUIRE(g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0, E2EP_EINVAL,
               "e2ep_dwconv_wgrad: bad geometry");
  const int sp = dw_wgrad_splits(g);
  // one split: the slab is the gradient; several: in-launch fold or k_dw_wgrad_finalize
  DwPart part{static_cast<float *>(workspace), dw,
              (sp > 1 && g_tune[TUNE_SPLITK_FOLD] == 2) ? handoff_slots(g.C, as_stream(stream)) : nullptr};
  if (dw_wgrad_strip_ok(g)) {
    const DwStrip d = dw_strip(g.K, g.st, g.W, g.P, g.Q);
    if (io)
      DW_STRIP_DISPATCH(dw_wgrad_strip, DW_B16, dim3(g.C, sp), 4 * d.IR * d.WP * 4, gy, x, g, d, sp,
                        part, tf);
    else
      DW_STRIP_DISPATCH(dw_wgrad_strip, DW_NONE, dim3(g.C, sp), 4 * d.IR * d.WP * 4, gy, x, g, d,
                        sp, part, tf);
  } else {
    DW_DISPATCH(k_dw_wgrad, dim3(g.C, sp), static_cast<const float *>(gy), x, g, sp, part, in_scale,
                in_shift, in_act);
  }
  if (sp > 1 && !part.cnt)
    hipLaunchKernelGGL(k_dw_wgrad_finalize, dim3(cdiv(g.C * g.K * g.K, 256)), dim3(256), 0,
                       as_stream(stream), part.part, g.C, g.K * g.K, sp, dw);
  return launch_status("e2ep_dwconv_wgrad");
}

int e2ep_dwconv_bwd(const void *gy, const float *x, const float *w, const int *dims,
                    const float *in_scale, const float *in_shift, int in_act, void *dx,
                    void *workspace, size_t workspace_bytes, float *dw, void *stream, int io) {
  E2EP_REQUIRE(io == 0 || io == (E2EP_IO_DY_BF16 | E2EP_IO_DX_BF16), E2EP_EINVAL,
               "e2ep_dwconv_bwd: storage mask %d not supported (0 or DY|DX bf16)", io);
  const bool hb = io != 0;
  const DwGeom g = dw_geom(dims);
  DwGeom t;
  int off;
  DwS2 p2;
  const bool geo = g.N > 0 && g.C > 0 && g.P > 0 && g.Q > 0 && g.st > 0;
  const bool s1 = geo && dw_bwd_pair_plan(g, t, off), s2 = geo && !s1 && dw_bwd_pair_s2_plan(g, p2);
  E2EP_REQUIRE(s1 || s2, E2EP_EINVAL, "e2ep_dwconv_bwd: no paired backward for this geometry "
               "(e2ep_dwconv_bwd_pair_ok returned 0)");
  E2EP_REQUIRE(workspace && workspace_bytes >= e2ep_dwconv_wgrad_workspace(dims), E2EP_EINVAL,
               "e2ep_dwconv_bwd: workspace %zu bytes < %zu (e2ep_dwconv_wgrad_workspace)",
               workspace_bytes, e2ep_dwconv_wgrad_workspace(dims));
  E2EP_REQUIRE(!in_scale == !in_shift && in_act >= 0 && in_act <= 2, E2EP_EINVAL,
               "e2ep_dwconv_bwd: in_scale / in_shift both or neither, in_act 0..2");
  E2EP_REQUIRE(gy && x && w && dx && dw, E2EP_EINVAL, "e2ep_dwconv_bwd: null tensor");
  const DwIn tf{in_scale, in_shift, in_act};
  hipStream_t s = as_stream(stream);
  if (s2) {
    const DwStrip d = dw_strip(g.K, 2, g.W, g.P, g.Q);
    const int vw = cdiv(d.IR * (g.W / 4), 64) <= 2 ? 2 : DW_MAXV;
    const int sp = dw_wgrad_splits(g);
    DwPart part{static_cast<float *>(workspace), dw,
                (sp > 1 && g_tune[TUNE_SPLITK_FOLD] == 2) ? handoff_slots(g.C, s) : nullptr};
    const size_t shm = 4 * (size_t)std::max(p2.GR * p2.WPg, d.IR * d.WP) * 4;
    const dim3 grid(g.C * sp + cdiv(p2.units, 4));
#define DWP2B(KV, PLPV, OFFV, VWV, BV)                                                             \
  hipLaunchKernelGGL((k_dw_bwd_pair_s2<KV, PLPV, OFFV, VWV, BV>), grid, dim3(256), shm, s,         \
                     static_cast<const dw_to<BV> *>(gy), w, p2.RO, p2.GR, p2.WPg, p2.upp, p2.units, \
                     static_cast<dw_to<BV> *>(dx), x, g, d, sp, part, tf)
#define DWP2(KV, PLPV, OFFV)                                                                       \
  do {                                                                                             \
    if (vw == 2 && hb) DWP2B(KV, PLPV, OFFV, 2, true);                                             \
    else if (vw == 2) DWP2B(KV, PLPV, OFFV, 2, false);                                             \
    else if (hb) DWP2B(KV, PLPV, OFFV, DW_MAXV, true);                                             \
    else DWP2B(KV, PLPV, OFFV, DW_MAXV, false);                                                    \
  } while (0)
    // PLP = pad_left & 1, OFF = -pad_left mod 4 (dw_off)
    if (g.K == 3 && g.pl == 0) DWP2(3, 0, 0);
    else if (g.K == 3) DWP2(3, 1, 3);
    else if (g.pl == 1) DWP2(5, 1, 3);
    else DWP2(5, 0, 2);
#undef DWP2
#undef DWP2B
    if (sp > 1 && !part.cnt)
      hipLaunchKernelGGL(k_dw_wgrad_finalize, dim3(cdiv(g.C * g.K * g.K, 256)), dim3(256), 0, s,
                         part.part, g.C, g.K * g.K, sp, dw);
    return launch_status("e2ep_dwconv_bwd");
  }
  const DwStrip dt = dw_strip(t.K, 1, t.W, t.P, t.Q);
  const int units = t.N * t.C * dt.units_per_plane;
  const int nd = dw_fwd_blocks(units);
  const int vd = cdiv(dt.IR * (t.W / 4), 64) <= 2 ? 2 : DW_MAXV;
  const DwStrip d = dw_strip(g.K, 1, g.W, g.P, g.Q);
  const int vw = cdiv(d.IR * (g.W / 4), 64) <= 2 ? 2 : DW_MAXV;
  const int sp = dw_wgrad_splits(g);
  DwPart part{static_cast<float *>(workspace), dw,
              (sp > 1 && g_tune[TUNE_SPLITK_FOLD] == 2) ? handoff_slots(g.C, s) : nullptr};
  const size_t shm = 4 * (size_t)std::max(dt.IR * dt.WP, d.IR * d.WP) * 4;
  const dim3 grid(nd + g.C * sp);
#define DWPB(KV, OFFV, VDV, VWV, BV)                                                              \
  hipLaunchKernelGGL((k_dw_bwd_pair<KV, OFFV, VDV, VWV, BV>), grid, dim3(256), shm, s,             \
                     static_cast<const dw_to<BV> *>(gy), w, t, dt, units, static_cast<dw_to<BV> *>(dx), \
                     nd, x, g, d, sp, part, tf)
#define DWP(KV, OFFV, VDV, VWV)                          \
  do {                                                   \
    if (hb) DWPB(KV, OFFV, VDV, VWV, true);              \
    else DWPB(KV, OFFV, VDV, VWV, false);                \
  } while (0)
#define DWP_V(KV, OFFV)                                  \
  do {                                                   \
    if (vd == 2 && vw == 2) DWP(KV, OFFV, 2, 2);         \
    else if (vd == 2) DWP(KV, OFFV, 2, DW_MAXV);         \
    else if (vw == 2) DWP(KV, OFFV, DW_MAXV, 2);         \
    else DWP(KV, OFFV, DW_MAXV, DW_MAXV);                \
  } while (0)
  if (g.K == 3) DWP_V(3, 3);
  else DWP_V(5, 2);
#undef DWP_V
#undef DWP
#undef DWPB
  if (sp > 1 && !part.cnt)
    hipLaunchKernelGGL(k_dw_wgrad_finalize, dim3(cdiv(g.C * g.K * g.K, 256)), dim3(256), 0, s,
                       part.part, g.C, g.K * g.K, sp, dw);
  return launch_status("e2ep_dwconv_bwd");
}

}  // extern "C"
