// Strided fp32 GEMM on MFMA for the transformer linears (nn.Linear forward and both
// backward GEMMs of model/feature_fusion.py:13-14,24-29,48-50 and model/control_predict.py:
// 18-24: d = 258 / 774 / 2048 at 2048 encoder rows and 112 decoder rows).
//
//   C[m][n] = sum_k A(m, k) * B(k, n)  (+ bias[n])  (+ Cadd[m][n])  (then ReLU if asked)
//   A(m, k) = AK ? A[m * lda + k] : A[k * lda + m]
//   B(k, n) = BKC ? B[n * ldb + k] : B[k * ldb + n]
//
// Forward y = x W^T + b is (AK, BKC); dX = dY W is (AK, !BKC); dW = dY^T X is (!AK, !BKC).
// Design (the k_conv_gemm2 scheme, CDNA4 fp32 MFMA v_mfma_f32_32x32x2_f32):
//  * block (64 TM) x (64 TN), 4 waves as 2 x 2, wave tile 32 TM x 32 TN (each A fragment
//    feeds TN MFMAs, each B fragment TM); K-step 32;
//  * LDS rows are k-contiguous ([row][32 + 4 pad]) whatever the global layout, so a lane's
//    16 fragment values are four ds_read_b128 (lane half h supplies k = 16h..16h+15 to the 16
//    MFMAs of a step — the sum over the 32 k is the same, its order fixed);
//  * global loads are raw buffer loads with out-of-range offsets for the M / N / K edges
//    (returns 0: no padding copies, K = 258 needs no special case); the next step's tile is
//    loaded into registers while the current one feeds the MFMAs;
//  * small grids split K (fixed-order reduction in k_gemm_reduce, so results are
//    deterministic run to run), large ones write C directly with the fused epilogue.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "gemm.h"
#include "handoff.h"

namespace e2ep {

typedef float g_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 g_bf16x8 __attribute__((ext_vector_type(8)));

// bload2 (8-B buffer load): common.h

// v & (ok ? ~0 : 0) as one v_and_b32 the compiler cannot turn back into a branch
__device__ __forceinline__ float kmask(float v, bool ok) {
  const unsigned m = ok ? 0xffffffffu : 0u;
  unsigned r;
  asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(__builtin_bit_cast(unsigned, v)), "v"(m));
  return __builtin_bit_cast(float, r);
}
constexpr int G_BK = 32;
constexpr int G_LDW = 36;  // LDS row stride in floats (32 k + 4 pad)

// OP: MFMA operand precision, 0 = fp32 (v_mfma_f32_32x32x2_f32, exact), 1 = bf16 (BASELINE
// C3: the fragments are rounded to bf16 when read from LDS, two v_mfma_f32_32x32x16_bf16 per
// 32-deep step, products and sums fp32; HBM tensors stay fp32)
// One GEMM problem of a launch: operands, epilogue inputs, its tile grid (gx column tiles x gy
// row tiles x gz K splits) and split-K fold state.
struct GemmArgs {
  const float *A;
  int lda;
  long long a_bytes;
  const float *B;
  int ldb;
  long long b_bytes;
  const float *bias;
  int bias_rows;
  const float *Cadd;
  int ldadd;
  float *C;
  long long c_bytes;
  int ldc;
  GemmCols cols;
  int M, N, K, kper, relu;
  float *rs, *part;
  unsigned int *cnt;
  int gx, gy, gz;
};

template <bool AK_, bool BKC_, int WM_, int TM_, int TN_, int AVEC_, int BVEC_, int OP_>
struct GemmCfg {
  static constexpr bool AK = AK_, BKC = BKC_;
  static constexpr int WM = WM_, TM = TM_, TN = TN_, AVEC = AVEC_, BVEC = BVEC_, OP = OP_;
  static constexpr int BM = 32 * TM * WM, BN = 32 * TN * (4 / WM);
  static constexpr int LDS_FLOATS = 2 * (BM + BN) * G_LDW;  // As[2][BM][G_LDW], Bs[2][BN][G_LDW]
};

// The block body of k_gemm for block (bx, by, bz) of problem g; `lds` holds CFG::LDS_FLOATS
// floats (16-B aligned) and s_last one int, both __shared__ of the calling kernel (so a kernel
// running two problems, k_gemm_pair, shares one LDS allocation between them).
template <class CFG>
__device__ __forceinline__ void gemm_block(const GemmArgs &g, int bx, int by, int bz, float *lds,
                                           int *s_last) {
  constexpr bool AK = CFG::AK, BKC = CFG::BKC;
  constexpr int WM = CFG::WM, TM = CFG::TM, TN = CFG::TN, AVEC = CFG::AVEC, BVEC = CFG::BVEC,
                OP = CFG::OP;
  const float *__restrict__ A = g.A;
  const int lda = g.lda;
  const long long a_bytes = g.a_bytes;
  const float *__restrict__ B = g.B;
  const int ldb = g.ldb;
  const long long b_bytes = g.b_bytes;
  const float *__restrict__ bias = g.bias;
  const int bias_rows = g.bias_rows;
  const float *__restrict__ Cadd = g.Cadd;
  const int ldadd = g.ldadd;
  float *__restrict__ C = g.C;
  const long long c_bytes = g.c_bytes;
  const int ldc = g.ldc;
  const GemmCols cols = g.cols;
  const int M = g.M, N = g.N, K = g.K, kper = g.kper, relu = g.relu;
  float *__restrict__ rs = g.rs;
  float *__restrict__ part = g.part;
  unsigned int *__restrict__ cnt = g.cnt;
  // rs != null (only !AK, !BKC, unbatched): B gets a logical column N of ones, so column N of
  // the product is the row sum of A over k — rs[m] = sum_k A(m, k), the bias gradient of a
  // linear layer taken by its weight-gradient GEMM (no separate column-sum launches)
  constexpr int BM = CFG::BM, BN = CFG::BN;
  constexpr int GA = BM / 32, GB = BN / 32;       // 32-row load groups per operand tile
  float(*As)[BM][G_LDW] = reinterpret_cast<float(*)[BM][G_LDW]>(lds);
  float(*Bs)[BN][G_LDW] = reinterpret_cast<float(*)[BN][G_LDW]>(lds + 2 * BM * G_LDW);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = by * BM, n0 = bx * BN;
  const int split = bz;
  const int ksteps = (K + G_BK - 1) / G_BK;
  const int kbeg = split * kper;
  const int kend = min(ksteps, kbeg + kper);
  const int nk = max(0, kend - kbeg);
  const __amdgpu_buffer_rsrc_t ra_ = rsrc(A, a_bytes), rb_ = rsrc(B, b_bytes);

  // An operand tile is groups of 32 rows x 32 k; per group a thread loads 4 values:
  // k-contiguous -> (row tid/8, k quad tid%8), one float4 / two float2 when aligned;
  // row-contiguous -> (row tid%32, k quad tid/32), lanes coalesced along the row.
  const int ar = AK ? tid >> 3 : tid & 31, aq = AK ? tid & 7 : tid >> 5;
  const int br = BKC ? tid >> 3 : tid & 31, bq = BKC ? tid & 7 : tid >> 5;

  // column-batched B: this thread's load column is fixed, so its image offset is too
  long long bcol_off[GB];
  bool bone[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int n = min(n0 + 32 * i + br, N - 1);
    bcol_off[i] = cols.hw ? (long long)(n / cols.hw) * cols.b_img + n % cols.hw : n;
    bone[i] = !BKC && rs && n0 + 32 * i + br == N;
  }

  // One step of register lookahead: the next K-step's loads are issued before this step's
  // MFMAs and written to the other LDS buffer after them.  (Deeper register pipelines, 2 and
  // 3 steps, measured 4-5 % slower: the extra registers cost a wave per SIMD.)
  float ra[GA][4], rb[GB][4];
  // Loads are unconditional and branch-free: the row index is clamped into the matrix (rows
  // past M / N only feed outputs that are never stored) and k into the buffer; values at
  // k >= K are zeroed with an integer mask when the registers are written to LDS (after the
  // step's MFMAs, so the loads stay in flight).  The vector width is a template parameter: a
  // run-time width / K-tail switch made hipcc branch around every load group and wait
  // vmcnt(0) before the next one, serialising each K-step's loads (round 3, from the ISA).
  // A vector load at the K tail may read past the row (masked) or the buffer (reads 0).
  auto load_k = [&](float *regs, const __amdgpu_buffer_rsrc_t &rs, auto vec_c, long long base,
                    int k) {  // 4 k-contiguous values at base + k
    constexpr int vec = decltype(vec_c)::value;
    if constexpr (vec == 2) {
      const float4 v = bload4(rs, (int)((base + k) * 4));
      regs[0] = v.x; regs[1] = v.y; regs[2] = v.z; regs[3] = v.w;
    } else if constexpr (vec == 1) {
      const float2 v0 = bload2(rs, (int)((base + k) * 4)), v1 = bload2(rs, (int)((base + k + 2) * 4));
      regs[0] = v0.x; regs[1] = v0.y; regs[2] = v1.x; regs[3] = v1.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) regs[j] = bload(rs, (int)((base + min(k + j, K - 1)) * 4));
    }
  };
  auto load_tiles = [&](float (&xa)[GA][4], float (&xb)[GB][4], int ks_in) {
    const int k0 = min(ks_in, kend - 1) * G_BK;  // past the range: re-read, never stored
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int row = min(m0 + 32 * i + ar, M - 1);
      const int k = k0 + 4 * aq;
      if (AK) {
        load_k(xa[i], ra_, std::integral_constant<int, AVEC>{}, (long long)row * lda, k);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          xa[i][j] = bload(ra_, (int)(((long long)min(k + j, K - 1) * lda + row) * 4));
      }
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int k = k0 + 4 * bq;
      if (BKC) {
        const int row = min(n0 + 32 * i + br, N - 1);
        load_k(xb[i], rb_, std::integral_constant<int, BVEC>{}, (long long)row * ldb, k);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = bload(rb_, (int)(((long long)min(k + j, K - 1) * ldb + bcol_off[i]) * 4));
          xb[i][j] = bone[i] ? 1.f : v;
        }
      }
    }
  };
  // LDS writes: regs -> k-contiguous rows; the zero mask for k >= K applied here
  auto store_tiles = [&](float (&xa)[GA][4], float (&xb)[GB][4], int buf, int ks) {
    const int k0 = ks * G_BK;
    const bool full = k0 + G_BK <= K;  // uniform
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      if (!full)
#pragma unroll
        for (int j = 0; j < 4; ++j) xa[i][j] = kmask(xa[i][j], k0 + 4 * aq + j < K);
      *reinterpret_cast<float4 *>(&As[buf][32 * i + ar][4 * aq]) =
          make_float4(xa[i][0], xa[i][1], xa[i][2], xa[i][3]);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      if (!full)
#pragma unroll
        for (int j = 0; j < 4; ++j) xb[i][j] = kmask(xb[i][j], k0 + 4 * bq + j < K);
      *reinterpret_cast<float4 *>(&Bs[buf][32 * i + br][4 * bq]) =
          make_float4(xb[i][0], xb[i][1], xb[i][2], xb[i][3]);
    }
  };

  // wave (wm, wn) owns rows 32 TM wm + 32 u and columns 32 TN wn + 32 t
  g_f32x16 acc[TM][TN];
#pragma unroll
  for (int u = 0; u < TM; ++u)
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[u][t] = g_f32x16{0};
  const int li = lane & 31, lh = lane >> 5;
  // lane half h supplies k = 16h .. 16h+15 to the 16 MFMAs of a step
  auto compute = [&](int buf) {
    float a[TM][16], b[TN][16];
#pragma unroll
    for (int u = 0; u < TM; ++u) {
      const float *p = &As[buf][32 * TM * wm + 32 * u + li][16 * lh];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4 *>(p + 4 * q);
        a[u][4 * q] = x.x; a[u][4 * q + 1] = x.y; a[u][4 * q + 2] = x.z; a[u][4 * q + 3] = x.w;
      }
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const float *p = &Bs[buf][32 * TN * wn + 32 * t + li][16 * lh];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4 *>(p + 4 * q);
        b[t][4 * q] = x.x; b[t][4 * q + 1] = x.y; b[t][4 * q + 2] = x.z; b[t][4 * q + 3] = x.w;
      }
    }
    if (OP == 0) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int u = 0; u < TM; ++u)
#pragma unroll
          for (int t = 0; t < TN; ++t)
            acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][kk], b[t][kk], acc[u][t], 0, 0, 0);
    } else {
      // lane half h supplies k = 16h + 8 blk + j to MFMA blk (element j): one consistent
      // permutation of the step's 32 k for both operands
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        g_bf16x8 ab[TM], bb[TN];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int u = 0; u < TM; ++u) ab[u][j] = (__bf16)a[u][8 * blk + j];
#pragma unroll
          for (int t = 0; t < TN; ++t) bb[t][j] = (__bf16)b[t][8 * blk + j];
        }
#pragma unroll
        for (int u = 0; u < TM; ++u)
#pragma unroll
          for (int t = 0; t < TN; ++t)
            acc[u][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab[u], bb[t], acc[u][t], 0, 0, 0);
      }
    }
  };
  if (nk > 0) {
    load_tiles(ra, rb, kbeg);
    store_tiles(ra, rb, 0, kbeg);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      load_tiles(ra, rb, kbeg + kt + 1);  // past the range: re-read, never stored
      // keep the loads at the top of the step: hipcc otherwise sinks them behind half the
      // MFMAs, leaving half a step to cover their latency before the LDS write waits on them
      __builtin_amdgcn_sched_barrier(0);
      compute(kt & 1);
      // all of the step's MFMAs before the LDS write (hipcc otherwise hoists the write, and its
      // wait on the loads, into the middle of them); unconditional: the last step's copy lands
      // in the idle buffer and is never read (a conditional store lets hipcc sink loads into
      // its branch, behind the MFMAs)
      __builtin_amdgcn_sched_barrier(0);
      store_tiles(ra, rb, (kt + 1) & 1, min(kbeg + kt + 1, kend - 1));
      __syncthreads();
    }
  }

  // epilogue: C/D layout col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
  // gridDim.z > 1: raw partial sums into part[split][M][Nw] (dense, unbatched); with `cnt`
  // (the in-launch fold) they are stored write-through, the tile's last-arriving split sums
  // every slab in split order (k_gemm_reduce's order) and runs the final epilogue below; with
  // no `cnt` k_gemm_reduce does that in a launch of its own.
  const int Nw = rs ? N + 1 : N;  // split-K partials carry the row-sum column
  if (g.gz > 1) {
    const long long MNw = (long long)M * Nw;
    const __amdgpu_buffer_rsrc_t rp = rsrc(part + split * MNw, 4LL * MNw);
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int n = n0 + 32 * TN * wn + 32 * t + li;
      const bool nok = n < N || (rs && n == N);
#pragma unroll
      for (int u = 0; u < TM; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * TM * wm + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const int off = (nok && m < M) ? (m * Nw + n) * 4 : OOR;
          if (cnt) bstore_sc1(rp, off, acc[u][t][r]);
          else bstore(rp, off, acc[u][t][r]);
        }
    }
    if (!cnt) return;
    handoff_drain();
    if (!handoff_arrive(cnt + bx + g.gx * by, g.gz, s_last)) return;
    const __amdgpu_buffer_rsrc_t rall = rsrc(part, 4LL * g.gz * MNw);
    for (int k = 0; k < g.gz; ++k) {
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int n = n0 + 32 * TN * wn + 32 * t + li;
        const bool nok = n < N || (rs && n == N);
#pragma unroll
        for (int u = 0; u < TM; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + 32 * TM * wm + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * lh;
            const float v = bload_sc1(rall, (nok && m < M) ? (int)((k * MNw + m * Nw + n) * 4) : OOR);
            acc[u][t][r] = k == 0 ? v : acc[u][t][r] + v;
          }
      }
    }
  }
  const bool final_ = true;
  float *dst = C;
  const int ldd = ldc;
  const bool batched = cols.hw > 0;
  // edges: buffer stores with out-of-range offsets are dropped; the epilogue's optional
  // inputs are behind uniform branches, and the 16 Cadd values of a tile are loaded together
  const __amdgpu_buffer_rsrc_t rd = rsrc(dst, c_bytes);
  const __amdgpu_buffer_rsrc_t rrs = rsrc(rs, rs ? 4LL * M : 0);
  const __amdgpu_buffer_rsrc_t rc =
      rsrc(Cadd, Cadd ? (batched ? c_bytes : 4LL * ((long long)(M - 1) * ldadd + N)) : 0);
  const bool add_c = final_ && Cadd != nullptr, add_b = final_ && bias != nullptr;
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = n0 + 32 * TN * wn + 32 * t + li;
    const bool nok = n < N;
    const bool rsc = rs && n == N;
    const long long cbase = batched ? (long long)(n / cols.hw) * cols.c_img + n % cols.hw : n;
    const float bn_ = (add_b && !bias_rows) ? bias[min(n, N - 1)] : 0.f;
#pragma unroll
    for (int u = 0; u < TM; ++u) {
      float cv[16];
      if (add_c) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * TM * wm + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const long long off = batched ? cbase + (long long)m * ldd : (long long)m * ldadd + n;
          cv[r] = bload(rc, (nok && m < M) ? (int)(off * 4) : OOR);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 32 * TM * wm + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * lh;
        float v = acc[u][t][r];
        if (add_b) v += bias_rows ? bias[min(m, M - 1)] : bn_;
        if (add_c) v += cv[r];
        if (final_ && relu) v = fmaxf(v, 0.f);
        bstore(rd, (nok && m < M) ? (int)((cbase + (long long)m * ldd) * 4) : OOR, v);
        if (rs) bstore(rrs, (rsc && m < M) ? m * 4 : OOR, v);
      }
    }
  }
}

template <bool AK, bool BKC, int WM, int TM, int TN, int AVEC, int BVEC, int OP = 0>
__global__ void __launch_bounds__(256) k_gemm(GemmArgs g) {
  typedef GemmCfg<AK, BKC, WM, TM, TN, AVEC, BVEC, OP> CFG;
  __shared__ __attribute__((aligned(16))) float lds[CFG::LDS_FLOATS];
  __shared__ int s_last;
  gemm_block<CFG>(g, blockIdx.x, blockIdx.y, blockIdx.z, lds, &s_last);
}

// Two independent GEMM problems in one launch (a linear layer's input gradient and its
// weight + bias gradient, e2ep_linear_bwd): blocks [0, n1) run problem 1, the rest problem 2,
// each with its own tile grid, splits and fold counters.  One launch instead of two on forked
// streams: in a replayed graph a fork / join costs ~5 + ~10 us of idle GPU (scripts/
// step_sequence.py), more than either product of the control decoder takes.
template <class C1, class C2>
__global__ void __launch_bounds__(256) k_gemm_pair(GemmArgs g1, GemmArgs g2) {
  constexpr int L = C1::LDS_FLOATS > C2::LDS_FLOATS ? C1::LDS_FLOATS : C2::LDS_FLOATS;
  __shared__ __attribute__((aligned(16))) float lds[L];
  __shared__ int s_last;
  // the first problem's blocks first (the reverse order was within noise,
  // profiles/r04/linear_pair_order_ab.txt; the switch is retired)
  const int n1 = g1.gx * g1.gy * g1.gz;
  int id = (int)blockIdx.x;
  if (id < n1) {
    gemm_block<C1>(g1, id % g1.gx, (id / g1.gx) % g1.gy, id / (g1.gx * g1.gy), lds, &s_last);
  } else {
    id -= n1;
    gemm_block<C2>(g2, id % g2.gx, (id / g2.gx) % g2.gy, id / (g2.gx * g2.gy), lds, &s_last);
  }
}

// C[m][n] = sum over splits in order (+ bias) (+ Cadd) (ReLU).  V = 4: four consecutive
// elements per thread with 16-byte loads / stores (plain dense C, column bias, M*N % 4 == 0);
// V = 1 handles column-batched C (Cadd in C's layout) and row bias.
template <int V>
__global__ void __launch_bounds__(256)
    k_gemm_reduce(const float *__restrict__ part, int splits, int M, int N,
                  const float *__restrict__ bias, int bias_rows, const float *__restrict__ Cadd,
                  int ldadd, float *__restrict__ C, int ldc, GemmCols cols, int relu,
                  float *__restrict__ rs) {
  // rs: the partials are M x (N + 1), column N = row sums of A (V = 1 only)
  const int Nw = rs ? N + 1 : N;
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * V;
  const long long MN = (long long)M * Nw;
  if (i >= MN) return;
  float s[V];
  if (V == 4) {
    float4 a = *reinterpret_cast<const float4 *>(part + i);
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
    for (int k = 1; k < splits; ++k) {
      a = *reinterpret_cast<const float4 *>(part + k * MN + i);
      s[0] += a.x; s[1] += a.y; s[2] += a.z; s[3] += a.w;
    }
  } else {
    s[0] = part[i];
    for (int k = 1; k < splits; ++k) s[0] += part[k * MN + i];
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const long long e = i + v;
    const int m = (int)(e / Nw), n = (int)(e - (long long)m * Nw);
    if (V == 1 && rs && n == N) {
      rs[m] = s[v];
      return;
    }
    const long long off = cols.hw ? (long long)(n / cols.hw) * cols.c_img + n % cols.hw +
                                        (long long)m * ldc
                                  : (long long)m * ldc + n;
    if (bias) s[v] += bias[bias_rows ? m : n];
    if (Cadd) s[v] += Cadd[cols.hw ? off : (long long)m * ldadd + n];
    if (relu) s[v] = fmaxf(s[v], 0.f);
    if (V == 1) C[off] = s[v];
  }
  if (V == 4) *reinterpret_cast<float4 *>(C + i) = make_float4(s[0], s[1], s[2], s[3]);
}

// Skinny GEMM for the forward layout with few rows (M <= g_skinny_rows, at most SK_ROWS: the
// control decoder's 14 token rows in C5 predict): C[m][n] = sum_k A[m*lda + k]
// B[n*ldb + k] (+ bias[n]) (+ Cadd) (ReLU).  One block per (output column n, chunk of
// SK_MAXM rows); lanes stride k (float2 when lda, ldb are even and the bases 8-byte aligned),
// each lane keeps SK_MAXM partial dot products; fixed-order wave, then block, reductions.  The
// MFMA tiles (32 x 128 at the least) left those launches a chain of K-steps on a dozen blocks
// (15 us for a 14 x 2048 x 258 product).
constexpr int SK_MAXM = 16, SK_ROWS = 128;
template <int V>
__global__ void __launch_bounds__(256) k_gemm_skinny(
    const float *__restrict__ A, int lda, const float *__restrict__ B, int ldb,
    const float *__restrict__ bias, const float *__restrict__ Cadd, int ldadd,
    float *__restrict__ C, int ldc, int M, int N, int K, int relu) {
  __shared__ float red[4][SK_MAXM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = blockIdx.x;
  const int m0 = blockIdx.y * SK_MAXM;
  A += (size_t)m0 * lda;
  C += (size_t)m0 * ldc;
  if (Cadd) Cadd += (size_t)m0 * ldadd;
  M = min(M - m0, SK_MAXM);
  float acc[SK_MAXM];
#pragma unroll
  for (int m = 0; m < SK_MAXM; ++m) acc[m] = 0.f;
  const float *brow = B + (size_t)n * ldb;
  for (int k = (wave * 64 + lane) * V; k < K; k += 256 * V) {
    if (V == 2 && k + 1 < K) {
      const float2 b = *reinterpret_cast<const float2 *>(brow + k);
      float2 a[SK_MAXM];
#pragma unroll
      for (int m = 0; m < SK_MAXM; ++m)
        a[m] = *reinterpret_cast<const float2 *>(A + (size_t)min(m, M - 1) * lda + k);
#pragma unroll
      for (int m = 0; m < SK_MAXM; ++m) {
        acc[m] = fmaf(a[m].x, b.x, acc[m]);
        acc[m] = fmaf(a[m].y, b.y, acc[m]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (k + j >= K) break;
        const float b = brow[k + j];
#pragma unroll
        for (int m = 0; m < SK_MAXM; ++m)
          acc[m] = fmaf(A[(size_t)min(m, M - 1) * lda + k + j], b, acc[m]);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < SK_MAXM; ++m) {
    const float v = wave_sum(acc[m]);
    if (lane == 0) red[wave][m] = v;
  }
  __syncthreads();
  if ((int)threadIdx.x < M) {
    const int m = threadIdx.x;
    float v = (red[0][m] + red[1][m]) + (red[2][m] + red[3][m]);
    if (bias) v += bias[n];
    if (Cadd) v += Cadd[(size_t)m * ldadd + n];
    if (relu) v = fmaxf(v, 0.f);
    C[(size_t)m * ldc + n] = v;
  }
}

struct GemmLaunch {
  int tile, splits, kper;
};

// Block tiles (wm waves along M, wave tile 32 tm x 32 tn):
//   1: 64 x 64 (2 x 2 waves, 32 x 32)     2: 32 x 128 (1 x 4, 32 x 32)
//   3: 128 x 128 (2 x 2, 64 x 64)         4: 64 x 128 (2 x 2, 32 x 64)
//   5: 128 x 64 (2 x 2, 64 x 32)          6: 64 x 256 (1 x 4, 64 x 64)
// (the larger tiles measured no faster on the C2 shapes, scripts/bench_gemm.py --sweep:
// profiles/r02/gemm_sweep_tiles.json; they stay selectable for other shapes)
struct GemmTile {
  int bm, bn;
};
static GemmTile tile_dims(int tile) {
  switch (tile) {
    case 2: return {32, 128};
    case 3: return {128, 128};
    case 4: return {64, 128};
    case 5: return {128, 64};
    case 6: return {64, 256};
    default: return {64, 64};
  }
}

// Automatic plan (scripts/bench_gemm.py --sweep / --conv): 64 x 64, or 32 x 128 when M is not
// a multiple of 64 and 32-row tiles pad it less (M = 32, 112, 144, 160, 336 ...); K split
// toward ~768 workgroups (3 per CU), at most 8 ways and >= 8 K-steps each.
static int g_force_tile = 0, g_force_splits = 0;  // 0: automatic
// K-steps per split for grids under 64 blocks (e2ep_gemm_split_min).  8, 4 and 2 measured
// the same C2 step within noise (25.52 / 25.49 / 25.44 ms, profiles/r02/session6/
// gemm_split_min_ab.txt): the default stays 8.
static int g_split_min_small = 8;
// e2ep_gemm_skinny: few-row forward products up to this M.  16 (the decoder at B = 1): C5
// predict fp16 4.84 -> 4.28 ms p50; the C2 step's 112-row decoder measured slower on it (25.66
// vs 25.39 ms/step, profiles/r02/session6/skinny_ab.txt), so it stays on the MFMA tiles.
static int g_skinny_rows = 16;
// operand precision of k_gemm (e2ep_gemm_precision): 0 fp32, 1 bf16 (C3)
static int g_gemm_precision = 0;

static GemmLaunch gemm_plan(int M, int N, int K) {
  GemmLaunch p{1, 1, 1};
  const int ksteps = cdiv(K, G_BK);
  if (g_force_tile > 0) {  // benchmarking override (e2ep_gemm_force)
    p.tile = g_force_tile;
    p.splits = std::max(1, std::min(g_force_splits, ksteps));
  } else {
    if (cdiv(M, 32) * 32 < cdiv(M, 64) * 64) p.tile = 2;
    const GemmTile t = tile_dims(p.tile);
    const long long blocks = (long long)cdiv(M, t.bm) * cdiv(N, t.bn);
    // tiny grids (the decoder's 112-row products: a dozen blocks) are a chain of K-steps, so
    // they may split down to g_split_min_small steps per split (e2ep_gemm_split_min)
    const long long nb = (long long)cdiv(M, t.bm) * cdiv(N, t.bn);
    const int smin = nb < 64 ? g_split_min_small : 8;
    const int cap = std::min(nb < 64 ? 16 : 8, std::max(1, ksteps / smin));
    p.splits = (int)std::min<long long>(cap, std::max(1LL, (long long)cdiv(g_tune[TUNE_GEMM_SPLIT_TARGET], blocks)));
  }
  p.kper = cdiv(ksteps, p.splits);
  p.splits = cdiv(ksteps, p.kper);
  return p;
}

size_t gemm_ws(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const GemmLaunch p = gemm_plan(M, N, K);
  return p.splits > 1 ? (size_t)p.splits * M * N * sizeof(float) : 0;
}

// vector loads along k for k-contiguous operands: 2 = float4 (rows 16-byte aligned), 1 =
// float2 (8-byte aligned: the d = 258 rows).  Row-contiguous operands stay on dword loads
// (lanes consecutive along the row): a float2 row-pair variant measured 1.2 - 1.5x slower on
// the weight-gradient shapes.
static int vec_of(bool kc, int ld, const void *ptr) {
  if (!kc) return 0;
  if (ld % 4 == 0 && ((uintptr_t)ptr & 15) == 0) return 2;
  return ld % 2 == 0 && ((uintptr_t)ptr & 7) == 0 ? 1 : 0;
}

static bool skinny_ok(bool ak, bool bk, bool bias_rows, GemmCols cols, int M, float *rs) {
  return ak && bk && !bias_rows && cols.hw == 0 && !rs && M <= g_skinny_rows && g_force_tile == 0;
}

int gemm_run(const float *A, int lda, bool ak, long long a_bytes, const float *B, int ldb,
             bool bk, long long b_bytes, const float *bias, bool bias_rows, const float *Cadd,
             int ldadd, float *C, long long c_bytes, int ldc, GemmCols cols, int M, int N, int K,
             int relu, void *workspace, hipStream_t s, float *rs) {
  if (rs && (ak || bk || cols.hw)) {
    set_error("gemm: the row sum of A needs a k-major A, a row-contiguous B, unbatched C");
    return E2EP_EINVAL;
  }
  if (skinny_ok(ak, bk, bias_rows, cols, M, rs)) {
    const bool v2 = lda % 2 == 0 && ldb % 2 == 0 && ((uintptr_t)A & 7) == 0 && ((uintptr_t)B & 7) == 0;
    const dim3 grid(N, cdiv(M, SK_MAXM));
    if (v2)
      hipLaunchKernelGGL(k_gemm_skinny<2>, grid, dim3(256), 0, s, A, lda, B, ldb, bias, Cadd, ldadd,
                         C, ldc, M, N, K, relu);
    else
      hipLaunchKernelGGL(k_gemm_skinny<1>, grid, dim3(256), 0, s, A, lda, B, ldb, bias, Cadd, ldadd,
                         C, ldc, M, N, K, relu);
    return 0;
  }
  const int Nx = rs ? N + 1 : N;  // logical columns including the ones column
  GemmLaunch p = gemm_plan(M, Nx, K);
  if (g_gemm_precision == 1 && p.tile != 1 && p.tile != 2) p.tile = 1;  // bf16: tiles 1 / 2 only
  if (p.splits > 1 && !workspace) {
    set_error("gemm: workspace of e2ep_gemm_workspace() bytes required");
    return E2EP_EINVAL;
  }
  float *part = p.splits > 1 ? static_cast<float *>(workspace) : nullptr;
  const GemmTile td = tile_dims(p.tile);
  // in-launch split-K fold (e2ep_tune key 28 = 2): one arrival counter per output tile
  unsigned int *cnt = (p.splits > 1 && g_tune[TUNE_SPLITK_FOLD] == 2)
                          ? handoff_slots(cdiv(Nx, td.bn) * cdiv(M, td.bm), s) : nullptr;
  dim3 grid(cdiv(Nx, td.bn), cdiv(M, td.bm), p.splits);
  const int avec = vec_of(ak, lda, A), bvec = vec_of(bk, ldb, B);
  const int br = bias_rows ? 1 : 0;
  const GemmArgs ga{A, lda, a_bytes, B, ldb, b_bytes, bias, br, Cadd, ldadd, C, c_bytes, ldc,
                    cols, M, N, K, p.kper, relu, rs, part, cnt, (int)grid.x, (int)grid.y,
                    (int)grid.z};
#define E2EP_GEMM_LAUNCH(AKV, BKV, WMV, TMV, TNV, AVV, BVV)                                     \
  hipLaunchKernelGGL((k_gemm<AKV, BKV, WMV, TMV, TNV, AVV, BVV>), grid, dim3(256), 0, s, ga)
#define E2EP_GEMM_T(AKV, BKV, AVV, BVV)                                     \
  do {                                                                      \
    if (g_gemm_precision == 1) { /* bf16: the automatic tiles */            \
      if (p.tile == 2)                                                      \
        hipLaunchKernelGGL((k_gemm<AKV, BKV, 1, 1, 1, AVV, BVV, 1>), grid, dim3(256), 0, s, ga); \
      else                                                                  \
        hipLaunchKernelGGL((k_gemm<AKV, BKV, 2, 1, 1, AVV, BVV, 1>), grid, dim3(256), 0, s, ga); \
      break;                                                                \
    }                                                                       \
    switch (p.tile) {                                                       \
      case 2: E2EP_GEMM_LAUNCH(AKV, BKV, 1, 1, 1, AVV, BVV); break;          \
      case 3: E2EP_GEMM_LAUNCH(AKV, BKV, 2, 2, 2, AVV, BVV); break;          \
      case 4: E2EP_GEMM_LAUNCH(AKV, BKV, 2, 1, 2, AVV, BVV); break;          \
      case 5: E2EP_GEMM_LAUNCH(AKV, BKV, 2, 2, 1, AVV, BVV); break;          \
      case 6: E2EP_GEMM_LAUNCH(AKV, BKV, 1, 2, 2, AVV, BVV); break;          \
      default: E2EP_GEMM_LAUNCH(AKV, BKV, 2, 1, 1, AVV, BVV); break;         \
    }                                                                       \
  } while (0)
  // vector widths along k of the k-contiguous operands (template: no run-time switch)
#define E2EP_GEMM_BV(AKV, BKV, AVV)                 \
  do {                                              \
    if (bvec == 2) E2EP_GEMM_T(AKV, BKV, AVV, 2);    \
    else if (bvec == 1) E2EP_GEMM_T(AKV, BKV, AVV, 1); \
    else E2EP_GEMM_T(AKV, BKV, AVV, 0);              \
  } while (0)
  if (ak && bk) {
    if (avec == 2) E2EP_GEMM_BV(true, true, 2);
    else if (avec == 1) E2EP_GEMM_BV(true, true, 1);
    else E2EP_GEMM_BV(true, true, 0);
  } else if (ak) {
    if (avec == 2) E2EP_GEMM_T(true, false, 2, 0);
    else if (avec == 1) E2EP_GEMM_T(true, false, 1, 0);
    else E2EP_GEMM_T(true, false, 0, 0);
  } else if (bk) {
    E2EP_GEMM_BV(false, true, 0);
  } else {
    E2EP_GEMM_T(false, false, 0, 0);
  }
#undef E2EP_GEMM_BV
#undef E2EP_GEMM_T
#undef E2EP_GEMM_LAUNCH
  if (p.splits > 1 && !cnt) {
    const long long MN = (long long)M * Nx;
    const bool v4 = !rs && MN % 4 == 0 && ldc == N && cols.hw == 0 && !bias_rows &&
                    (!Cadd || ldadd == N) && ((uintptr_t)C & 15) == 0;
    if (v4)
      hipLaunchKernelGGL(k_gemm_reduce<4>, dim3(cdiv(MN / 4, 256)), dim3(256), 0, s,
                         static_cast<const float *>(workspace), p.splits, M, N, bias, br, Cadd,
                         ldadd, C, ldc, cols, relu, nullptr);
    else
      hipLaunchKernelGGL(k_gemm_reduce<1>, dim3(cdiv(MN, 256)), dim3(256), 0, s,
                         static_cast<const float *>(workspace), p.splits, M, N, bias, br, Cadd,
                         ldadd, C, ldc, cols, relu, rs);
  }
  return 0;
}

// One problem of a k_gemm_pair launch: its plan, fold counters and arguments; false when the
// pair kernel cannot take it (benchmark-forced tiles, or K splits without the in-launch fold).
static bool gemm_prepare(const float *A, int lda, bool ak, long long a_bytes, const float *B,
                         int ldb, bool bk, long long b_bytes, const float *Cadd, int ldadd,
                         float *C, long long c_bytes, int ldc, int M, int N, int K,
                         void *workspace, float *rs, hipStream_t s, GemmArgs &ga, int &wm,
                         int &avec) {
  const int Nx = rs ? N + 1 : N;
  GemmLaunch p = gemm_plan(M, Nx, K);
  if (g_gemm_precision == 1 && p.tile != 1 && p.tile != 2) p.tile = 1;
  if (p.tile != 1 && p.tile != 2) return false;
  if (p.splits > 1 && (!workspace || g_tune[TUNE_SPLITK_FOLD] != 2)) return false;
  const GemmTile td = tile_dims(p.tile);
  const int gx = cdiv(Nx, td.bn), gy = cdiv(M, td.bm);
  unsigned int *cnt = p.splits > 1 ? handoff_slots(gx * gy, s) : nullptr;
  if (p.splits > 1 && !cnt) return false;  // no counters: the two-launch path reduces
  ga = GemmArgs{A, lda, a_bytes, B, ldb, b_bytes, nullptr, 0, Cadd, ldadd, C, c_bytes, ldc,
                GemmCols{0, 0, 0}, M, N, K, p.kper, 0, rs,
                p.splits > 1 ? static_cast<float *>(workspace) : nullptr, cnt, gx, gy, p.splits};
  wm = p.tile == 2 ? 1 : 2;  // tile 1: 64 x 64 (2 x 2 waves); tile 2: 32 x 128 (1 x 4)
  avec = vec_of(ak, lda, A);
  (void)bk;
  return true;
}

// k_gemm_pair for (input gradient: A k-contiguous, B row-contiguous) + (weight gradient with
// the row-sum column: both row-contiguous), dispatched over the tiles / vector width / precision
template <int OP, int WM1, int AV1, int WM2>
static void pair4(dim3 grid, hipStream_t s, const GemmArgs &g1, const GemmArgs &g2) {
  hipLaunchKernelGGL((k_gemm_pair<GemmCfg<true, false, WM1, 1, 1, AV1, 0, OP>,
                                  GemmCfg<false, false, WM2, 1, 1, 0, 0, OP>>),
                     grid, dim3(256), 0, s, g1, g2);
}
template <int OP, int WM1, int AV1>
static void pair3(int wm2, dim3 grid, hipStream_t s, const GemmArgs &g1, const GemmArgs &g2) {
  if (wm2 == 2) pair4<OP, WM1, AV1, 2>(grid, s, g1, g2);
  else pair4<OP, WM1, AV1, 1>(grid, s, g1, g2);
}
template <int OP, int WM1>
static void pair2(int av1, int wm2, dim3 grid, hipStream_t s, const GemmArgs &g1, const GemmArgs &g2) {
  if (av1 == 2) pair3<OP, WM1, 2>(wm2, grid, s, g1, g2);
  else if (av1 == 1) pair3<OP, WM1, 1>(wm2, grid, s, g1, g2);
  else pair3<OP, WM1, 0>(wm2, grid, s, g1, g2);
}
template <int OP>
static void pair1(int wm1, int av1, int wm2, dim3 grid, hipStream_t s, const GemmArgs &g1,
                  const GemmArgs &g2) {
  if (wm1 == 2) pair2<OP, 2>(av1, wm2, grid, s, g1, g2);
  else pair2<OP, 1>(av1, wm2, grid, s, g1, g2);
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_linear_bwd(const float *dy, int ldy, const float *x, int ldx, const float *w, int ldw,
                    const float *gskip, int ldskip, float *dx, int lddx, float *dw, int lddw,
                    float *db, int M, int N, int K, void *ws_dx, size_t ws_dx_bytes, void *ws_dw,
                    size_t ws_dw_bytes, void *stream) {
  E2EP_REQUIRE(dy && x && w && dx && dw && db && M > 0 && N > 0 && K > 0, E2EP_EINVAL,
               "e2ep_linear_bwd: bad arguments M=%d N=%d K=%d", M, N, K);
  E2EP_REQUIRE(ldy >= N && ldx >= K && ldw >= K && lddx >= K && lddw >= K &&
                   (!gskip || ldskip >= K),
               E2EP_EINVAL, "e2ep_linear_bwd: leading dimension too small");
  const size_t need_dx = gemm_ws(M, K, N), need_dw = gemm_ws(N, K + 1, M);
  E2EP_REQUIRE((!need_dx || (ws_dx && ws_dx_bytes >= need_dx)) &&
                   (!need_dw || (ws_dw && ws_dw_bytes >= need_dw)),
               E2EP_EINVAL, "e2ep_linear_bwd: workspaces %zu / %zu bytes < %zu / %zu "
               "(e2ep_gemm_workspace(M, K, N) / e2ep_gemm_rowsum_workspace(N, K, M))",
               ws_dx_bytes, ws_dw_bytes, need_dx, need_dw);
  const long long y_bytes = 4LL * ((long long)(M - 1) * ldy + N);
  const long long x_bytes = 4LL * ((long long)(M - 1) * ldx + K);
  const long long w_bytes = 4LL * ((long long)(N - 1) * ldw + K);
  const long long dx_bytes = 4LL * ((long long)(M - 1) * lddx + K);
  const long long dw_bytes = 4LL * ((long long)(N - 1) * lddw + K);
  E2EP_REQUIRE(y_bytes < 0x7fffffffLL && x_bytes < 0x7fffffffLL && w_bytes < 0x7fffffffLL &&
                   dx_bytes < 0x7fffffffLL && dw_bytes < 0x7fffffffLL &&
                   4LL * N * (K + 1) * 8 < 0x7fffffffLL,
               E2EP_ERANGE, "e2ep_linear_bwd: operand larger than 2 GB");
  hipStream_t s = as_stream(stream);
  // dX[M][K] = dY[M][N] W[N][K] (+ gskip);  dW[N][K] = dY^T X with db[N] = row sums of dY^T
  GemmArgs g1, g2;
  int wm1, av1, wm2, av2;
  if (g_force_tile == 0 &&
      gemm_prepare(dy, ldy, true, y_bytes, w, ldw, false, w_bytes, gskip, ldskip, dx, dx_bytes,
                   lddx, M, K, N, ws_dx, nullptr, s, g1, wm1, av1) &&
      gemm_prepare(dy, ldy, false, y_bytes, x, ldx, false, x_bytes, nullptr, 0, dw, dw_bytes,
                   lddw, N, K, M, ws_dw, db, s, g2, wm2, av2)) {
    const dim3 grid(g1.gx * g1.gy * g1.gz + g2.gx * g2.gy * g2.gz);
    if (g_gemm_precision == 1) pair1<1>(wm1, av1, wm2, grid, s, g1, g2);
    else pair1<0>(wm1, av1, wm2, grid, s, g1, g2);
    return launch_status("e2ep_linear_bwd");
  }
  // fallback (benchmark-forced tiles, folds off): the two launches in order on one stream
  int rc = gemm_run(dy, ldy, true, y_bytes, w, ldw, false, w_bytes, nullptr, false, gskip, ldskip,
                    dx, dx_bytes, lddx, GemmCols{0, 0, 0}, M, K, N, 0, ws_dx, s, nullptr);
  if (rc) return rc;
  rc = gemm_run(dy, ldy, false, y_bytes, x, ldx, false, x_bytes, nullptr, false, nullptr, 0, dw,
                dw_bytes, lddw, GemmCols{0, 0, 0}, N, K, M, 0, ws_dw, s, db);
  if (rc) return rc;
  return launch_status("e2ep_linear_bwd");
}

int e2ep_gemm_force(int tile, int splits, int unused) {
  (void)unused;
  E2EP_REQUIRE(tile >= 0 && tile <= 6 && splits >= 0, E2EP_EINVAL,
               "e2ep_gemm_force: tile in 1..6 (0 = automatic), splits >= 0");
  g_force_tile = tile;
  g_force_splits = splits;
  return 0;
}

size_t e2ep_gemm_workspace(int M, int N, int K) { return gemm_ws(M, N, K); }

int e2ep_gemm_split_min(int ksteps) {
  const int prev = g_split_min_small;
  if (ksteps > 0) g_split_min_small = ksteps;
  return prev;
}

int e2ep_gemm_precision(int precision) {
  const int prev = g_gemm_precision;
  if (precision == 0 || precision == 1) g_gemm_precision = precision;
  return prev;
}

int e2ep_gemm_skinny(int max_rows) {
  const int prev = g_skinny_rows;
  if (max_rows >= 0) g_skinny_rows = std::min(max_rows, SK_ROWS);
  return prev;
}
size_t e2ep_gemm_rowsum_workspace(int M, int N, int K) { return gemm_ws(M, N + 1, K); }

int e2ep_gemm(const float *A, int lda, int a_kcontig, const float *B, int ldb, int b_kcontig,
              const float *bias, const float *Cadd, int ldadd, float *C, int ldc, int M, int N,
              int K, int relu, void *workspace, size_t workspace_bytes, void *stream) {
  E2EP_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0, E2EP_EINVAL,
               "e2ep_gemm: bad arguments M=%d N=%d K=%d", M, N, K);
  E2EP_REQUIRE(!gemm_ws(M, N, K) || (workspace && workspace_bytes >= gemm_ws(M, N, K)),
               E2EP_EINVAL, "e2ep_gemm: workspace %zu bytes < %zu the launch plan needs (query "
               "e2ep_gemm_workspace after setting precision / tunables)", workspace_bytes,
               gemm_ws(M, N, K));
  E2EP_REQUIRE(lda >= (a_kcontig ? K : M) && ldb >= (b_kcontig ? K : N) && ldc >= N &&
                   (!Cadd || ldadd >= N),
               E2EP_EINVAL, "e2ep_gemm: leading dimension too small");
  const long long a_bytes = 4LL * (a_kcontig ? (long long)(M - 1) * lda + K : (long long)(K - 1) * lda + M);
  const long long b_bytes = 4LL * (b_kcontig ? (long long)(N - 1) * ldb + K : (long long)(K - 1) * ldb + N);
  const long long c_bytes = 4LL * ((long long)(M - 1) * ldc + N);
  E2EP_REQUIRE(a_bytes < 0x7fffffffLL && b_bytes < 0x7fffffffLL && c_bytes < 0x7fffffffLL &&
                   (!Cadd || 4LL * ((long long)(M - 1) * ldadd + N) < 0x7fffffffLL),
               E2EP_ERANGE, "e2ep_gemm: operand larger than 2 GB");
  const int rc = gemm_run(A, lda, a_kcontig, a_bytes, B, ldb, b_kcontig, b_bytes, bias, false,
                          Cadd, ldadd, C, c_bytes, ldc, GemmCols{0, 0, 0}, M, N, K, relu,
                          workspace, as_stream(stream), nullptr);
  if (rc) return rc;
  return launch_status("e2ep_gemm");
}

int e2ep_gemm_rowsum(const float *A, int lda, const float *B, int ldb, float *C, int ldc,
                     float *rowsum, int M, int N, int K, void *workspace,
                     size_t workspace_bytes, void *stream) {
  E2EP_REQUIRE(A && B && C && rowsum && M > 0 && N > 0 && K > 0, E2EP_EINVAL,
               "e2ep_gemm_rowsum: bad arguments M=%d N=%d K=%d", M, N, K);
  E2EP_REQUIRE(!gemm_ws(M, N + 1, K) || (workspace && workspace_bytes >= gemm_ws(M, N + 1, K)),
               E2EP_EINVAL, "e2ep_gemm_rowsum: workspace %zu bytes < %zu the launch plan needs",
               workspace_bytes, gemm_ws(M, N + 1, K));
  E2EP_REQUIRE(lda >= M && ldb >= N && ldc >= N, E2EP_EINVAL,
               "e2ep_gemm_rowsum: leading dimension too small");
  const long long a_bytes = 4LL * ((long long)(K - 1) * lda + M);
  const long long b_bytes = 4LL * ((long long)(K - 1) * ldb + N);
  const long long c_bytes = 4LL * ((long long)(M - 1) * ldc + N);
  E2EP_REQUIRE(a_bytes < 0x7fffffffLL && b_bytes < 0x7fffffffLL && c_bytes < 0x7fffffffLL &&
                   4LL * M * (N + 1) * 8 < 0x7fffffffLL,
               E2EP_ERANGE, "e2ep_gemm_rowsum: operand larger than 2 GB");
  const int rc = gemm_run(A, lda, false, a_bytes, B, ldb, false, b_bytes, nullptr, false, nullptr,
                          0, C, c_bytes, ldc, GemmCols{0, 0, 0}, M, N, K, 0, workspace,
                          as_stream(stream), rowsum);
  if (rc) return rc;
  return launch_status("e2ep_gemm_rowsum");
}

}  // extern "C"
