// Direct-convolution forward of the BEV stem with 16-bit operands: conv 7x7 / 2, pad 3,
// 65 -> 64 channels, 256^2 -> 128^2 (reference model/bev_encoder.py:13,26) in the C3 bf16
// training mode and the C5 fp16 inference mode (operands rounded to nearest-even as they are
// staged, fp32 accumulate, fp32 tensors in HBM — the k_conv_lp semantics).
//
// The implicit GEMM (k_conv_lp) re-gathers the im2col operand for every (tap, channel chunk)
// K-step: the 7x7/2 stem read each input value ~12 times through L2 and spent its time on
// load issue (k_conv_lp<0,0,1,4,1,32> 290 us, 0.07 of the bf16 peak,
// profiles/r06/step_sequence_bf16_final.txt).  Here a block owns an output tile of
// 64 channels x 8 rows x 32 columns of one image and stages its input patch ONCE per
// 16-channel chunk:
//  * patch = 21 x 69 input positions x 16 channels, 16-bit, laid out [row][channel half]
//    [column parity][column / 2][8 channels]: for tap (r, s) lane i of a wave reads output
//    column i's 8 channels as one ds_read_b128, and the 32 lanes of a half read 32
//    consecutive 16-B slots (the stride-2 columns de-interleaved by parity) — conflict free;
//  * weights: k_stem_wprep first writes them once per launch as a 16-bit image in the order
//    the blocks read them ([chunk][filter row][s][channel half][co][8], then the tail's
//    [step][half][co][8]: 408 KB for the stem); a block copies one (chunk, filter row) —
//    14 KB, 3.5 coalesced b128 loads per thread — into a double-buffered LDS slot, the next
//    row's loads in flight during the current row's MFMAs (gathering them from the fp32
//    tap-major weights, 8 scalar loads per lane 260 B apart, took the kernel to 159 us);
//  * each wave computes 64 co x 2 output rows x 32 columns: per tap two A fragments (co
//    0-31, 32-63) x two B fragments (its rows) = 4 v_mfma_f32_32x32x16 per 4 b128 LDS reads;
//  * the Cin % 16 remainder channels (the stem's 65th, the target plane) run as flattened
//    (channel, tap) K-steps over a scalar patch image: 4 steps for 1 x 49 rows, not a
//    zero-padded 16-channel chunk (13 % of the MFMAs);
//  * LDS 75.7 KB per block: two blocks per CU, one staging while the other computes.
// Sum order per output: chunks in order, filter rows, filter columns, then the remainder rows
// in (channel, tap) order — fixed, so results are deterministic run to run.
#include <algorithm>
#include <type_traits>

#include "conv.h"

#pragma clang fp contract(on)

namespace e2ep {

namespace {

typedef float sd_f32x16 __attribute__((ext_vector_type(16)));
typedef float sd_f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 sd_bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 sd_f16x8 __attribute__((ext_vector_type(8)));

template <int OP> struct SdType;
template <> struct SdType<0> { typedef float T; typedef sd_f32x8 T8; };  // exact-f32 MFMA (C2)
template <> struct SdType<1> { typedef __bf16 T; typedef sd_bf16x8 T8; };
template <> struct SdType<2> { typedef _Float16 T; typedef sd_f16x8 T8; };

constexpr int SD_K = 7;                        // filter rows = columns
constexpr int SD_TH = 8, SD_TW = 32;           // output tile rows x columns (4 waves x 2 rows)
constexpr int SD_PR = 2 * (SD_TH - 1) + SD_K;  // 21 patch rows
constexpr int SD_PC = 2 * (SD_TW - 1) + SD_K;  // 69 patch columns
constexpr int SD_PCH = (SD_PC + 1) / 2;        // 35 columns per parity
constexpr int SD_PATCH8 = SD_PR * 2 * 2 * SD_PCH;  // 8-channel groups of the patch image
constexpr int SD_PTASKS = 2 * SD_PR * SD_PC;       // (channel half, row, column) staging tasks
constexpr int SD_WROW8 = SD_K * 2 * 64;            // 8-channel weight groups per filter row
constexpr int SD_TAILMAX = 4;                      // remainder channels (14 flattened steps)

template <int OP>
__device__ __forceinline__ typename SdType<OP>::T8 sd_cvt8(const float *v) {
  sd_f32x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = v[j];
  return __builtin_convertvector(f, typename SdType<OP>::T8);
}

// One 16-deep K-step of a 32 x 32 tile: one v_mfma_f32_32x32x16_{bf16,f16}; for fp32 operands
// (OP 0, v_mfma_f32_32x32x2_f32) eight, MFMA t taking element t of each lane half's 8 values
// (k = t and 8 + t: the same 16 k, as k_conv_gemm2 permutes them)
template <int OP>
__device__ __forceinline__ sd_f32x16 sd_mfma(typename SdType<OP>::T8 a, typename SdType<OP>::T8 b,
                                             sd_f32x16 c) {
  if constexpr (OP == 1) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  } else if constexpr (OP == 2) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  } else {
#pragma unroll
    for (int t = 0; t < 8; ++t) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], c, 0, 0, 0);
    return c;
  }
}

// group `i` (8 values: 16 B, or 32 B for fp32) of a weight image; zeros when !ok
template <int OP>
__device__ __forceinline__ typename SdType<OP>::T8 sd_gload(__amdgpu_buffer_rsrc_t r, int i, bool ok) {
  typedef typename SdType<OP>::T8 T8;
  if constexpr (OP == 0) {
    const float4 u = bload4(r, ok ? i * 32 : OOR), v = bload4(r, ok ? i * 32 + 16 : OOR);
    T8 o;
    o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w;
    o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = v.w;
    return o;
  } else {
    return __builtin_bit_cast(T8, bload4(r, ok ? i * 16 : OOR));
  }
}

}  // namespace

// x [N][Cin][H][W] fp32, wimg the k_stem_wprep weight image, y [N][64][P][Q] fp32 (+ bias, relu).
// Grid (ceil(Q / 32), ceil(P / 8), N), 256 threads; the host gate stem_direct_ok holds the
// shape assumptions (64 output channels, 7x7, stride 2, Cin % 16 <= 4, byte offsets < 2^31).
template <int OP, int ACT>
__global__ void __launch_bounds__(256) k_conv_stem_lp(const float *__restrict__ x,
                                                      const void *__restrict__ wimg,
                                                      const float *__restrict__ bias,
                                                      float *__restrict__ y, long long y_bytes,
                                                      ConvGeom g) {
  typedef typename SdType<OP>::T T;
  typedef typename SdType<OP>::T8 T8;
  __shared__ T8 patch[SD_PATCH8];   // [row][half][parity][column / 2]; the tail's scalar image
  __shared__ T8 wl[2][SD_WROW8];    // [buffer][s][half][co]; the tail's [step][half][co]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int n = blockIdx.z, oy0 = blockIdx.y * SD_TH, ox0 = blockIdx.x * SD_TW;
  const int iy0 = 2 * oy0 - g.ph, ix0 = 2 * ox0 - g.pw;
  const int HW = g.H * g.W;
  const int nch = g.Cin >> 4, crem = g.Cin - 16 * nch;
  const int xbase = n * g.Cin * HW;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.Cin * HW);
  const int kt = crem * SD_K * SD_K;
  const int tsteps = (kt + 15) >> 4;
  const __amdgpu_buffer_rsrc_t rw = rsrc(wimg, (long long)sizeof(T8) * (nch * SD_K * SD_WROW8 + tsteps * 128));

  // one 16-channel chunk's patch: task = (half, row, column), 8 channel loads (lanes on
  // consecutive columns: coalesced) -> one b128 LDS write
  auto stage_patch = [&](int c) {
    for (int t0 = 0; t0 < SD_PTASKS; t0 += 4 * 256) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + 256 * u + tid;
        const int pc = t % SD_PC, rest = t / SD_PC;
        const int pr = rest % SD_PR, h = rest / SD_PR;
        const int iy = iy0 + pr, ix = ix0 + pc;
        const bool ok = t < SD_PTASKS && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
        const int base = xbase + (16 * c + 8 * h) * HW + iy * g.W + ix;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = bload(rx, ok ? (base + e * HW) * 4 : OOR);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + 256 * u + tid;
        const int pc = t % SD_PC, rest = t / SD_PC;
        const int pr = rest % SD_PR, h = rest / SD_PR;
        if (t < SD_PTASKS) patch[((pr * 2 + h) * 2 + (pc & 1)) * SD_PCH + (pc >> 1)] = sd_cvt8<OP>(v[u]);
      }
    }
  };
  // one (chunk, filter row) of the weight image: 896 consecutive 16-B groups
  T8 wv[4];
  auto load_w = [&](int c, int r) {
    const int g0 = (c * SD_K + r) * SD_WROW8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int task = tid + 256 * u;
      wv[u] = sd_gload<OP>(rw, g0 + task, task < SD_WROW8);
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int task = tid + 256 * u;
      if (task < SD_WROW8) wl[buf][task] = wv[u];
    }
  };

  sd_f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[a][j] = sd_f32x16{0};

  auto compute_row = [&](int r, int buf) {
#pragma unroll
    for (int s = 0; s < SD_K; ++s) {
      const T8 a0 = wl[buf][(s * 2 + lh) * 64 + li];
      const T8 a1 = wl[buf][(s * 2 + lh) * 64 + 32 + li];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pr = 2 * (2 * wave + j) + r;
        const T8 b = patch[((pr * 2 + lh) * 2 + (s & 1)) * SD_PCH + li + (s >> 1)];
        acc[0][j] = sd_mfma<OP>(a0, b, acc[0][j]);
        acc[1][j] = sd_mfma<OP>(a1, b, acc[1][j]);
      }
    }
  };

  const int nsteps = nch * SD_K;  // (chunk, filter row) steps
  if (nsteps > 0) {
    stage_patch(0);
    load_w(0, 0);
    store_w(0);
    __syncthreads();
    for (int k = 0; k < nsteps; ++k) {
      const int c = k / SD_K, r = k - SD_K * c;
      const int kn = min(k + 1, nsteps - 1);  // the last step re-reads itself into the idle buffer
      load_w(kn / SD_K, kn % SD_K);
      __builtin_amdgcn_sched_barrier(0);  // weight loads first, then the row's MFMAs
      compute_row(r, k & 1);
      __builtin_amdgcn_sched_barrier(0);
      store_w((k + 1) & 1);
      if (r == SD_K - 1 && k + 1 < nsteps) {  // chunk done by every wave: restage the patch
        __syncthreads();
        stage_patch(c + 1);
      }
      __syncthreads();
    }
  }

  if (crem > 0) {  // remainder channels: flattened (channel, tap) rows, 16 per K-step
    T *tp = reinterpret_cast<T *>(patch);  // [channel][row][column]
    T8 *tw = &wl[0][0];                    // [step][half][co]
    for (int t = tid; t < crem * SD_PR * SD_PC; t += 256) {
      const int pc = t % SD_PC, rest = t / SD_PC;
      const int pr = rest % SD_PR, cc = rest / SD_PR;
      const int iy = iy0 + pr, ix = ix0 + pc;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      tp[t] = (T)bload(rx, ok ? (xbase + (16 * nch + cc) * HW + iy * g.W + ix) * 4 : OOR);
    }
    for (int t = tid; t < tsteps * 128; t += 256)
      tw[t] = sd_gload<OP>(rw, nch * SD_K * SD_WROW8 + t, true);
    __syncthreads();
    for (int step = 0; step < tsteps; ++step) {
      const T8 a0 = tw[(step * 2 + lh) * 64 + li];
      const T8 a1 = tw[(step * 2 + lh) * 64 + 32 + li];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        T8 b;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // rows past kt carry zero weights; clamp them onto a staged (finite) value
          const int k = min(16 * step + 8 * lh + e, kt - 1);
          const int cc = k / (SD_K * SD_K), tap = k - SD_K * SD_K * cc;
          const int r = tap / SD_K, s = tap - SD_K * r;
          b[e] = tp[(cc * SD_PR + 2 * (2 * wave + j) + r) * SD_PC + 2 * li + s];
        }
        acc[0][j] = sd_mfma<OP>(a0, b, acc[0][j]);
        acc[1][j] = sd_mfma<OP>(a1, b, acc[1][j]);
      }
    }
  }

  // epilogue: C/D layout col = lane & 31 (output column), row = (r&3) + 8(r>>2) + 4(lane>>5)
  const __amdgpu_buffer_rsrc_t ry = rsrc(y, y_bytes);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int oy = oy0 + 2 * wave + j, ox = ox0 + li;
    const bool ok = oy < g.P && ox < g.Q;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int co = 32 * a + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
        float v = acc[a][j][rr];
        if (bias) v += bias[co];
        if (ACT == 1) v = fmaxf(v, 0.f);
        bstore(ry, ok ? (((n * 64 + co) * g.P + oy) * g.Q + ox) * 4 : OOR, v);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Data gradient of the same conv (C3: the BEV stem's gradient into the 64 BEV channels,
// bf16 operands gy and W, fp32 accumulate): dx[ci][y][x] = sum_(co, r, s) W[co][ci][r][s]
// gy[co][(y + 3 - r) / 2][(x + 3 - s) / 2] over the taps whose parity matches (stride 2, pad 3).
// Written per output phase (py, px) = (y & 1, x & 1), y = 2u + py: phase py takes the filter
// rows r with r + py odd, at gradient row u + (py + 3 - r) / 2 (offset -1 .. +2).  A block
// owns 64 ci x all four phases of a coarse 4 x 32 (u, v) tile — a 8 x 64 pixel dx tile — and
// stages the gradient patch (7 x 35 positions x all 64 co, 31 KB) ONCE; wave w takes coarse
// row u0 + w, all four phases (8 accumulators of 32 v x 32 ci): per tap two b128 weight
// fragments (ci halves, the (chunk, filter row) double-buffered from a prepped
// [chunk][r][s][co half][ci][8 co] image) and one b128 patch fragment, 2 MFMAs.  Every wave
// runs every tap once (no phase imbalance).  Sum order: co chunk, r, s — deterministic.
// ------------------------------------------------------------------------------------------
constexpr int SG_TU = 4, SG_TV = 32;                  // coarse tile: 4 waves x 32 columns
constexpr int SG_PU = SG_TU + 3, SG_PV = SG_TV + 3;   // patch rows / columns (offsets -1 .. +2)
constexpr int SG_CH = 4;                              // 16-channel chunks of the 64 co
constexpr int SG_PATCH8 = SG_CH * SG_PU * 2 * SG_PV;  // 8-channel groups of the patch (1960)

template <int OP>
__global__ void __launch_bounds__(256, OP == 0 ? 1 : 2) k_conv_stem_dgrad_lp(const float *__restrict__ gy,
                                                            const void *__restrict__ wimg,
                                                            float *__restrict__ dx,
                                                            long long dx_bytes, ConvGeom g) {
  typedef typename SdType<OP>::T8 T8;
  __shared__ T8 patch[SG_PATCH8];  // [chunk][row][half][column]
  __shared__ T8 wl[2][SD_WROW8];   // [buffer][s][half][ci]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int n = blockIdx.z, u0 = blockIdx.y * SG_TU, v0 = blockIdx.x * SG_TV;
  const int PQ = g.P * g.Q;
  const int gbase = n * 64 * PQ;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gy, 4LL * g.N * 64 * PQ);
  const __amdgpu_buffer_rsrc_t rw = rsrc(wimg, (long long)sizeof(T8) * SG_CH * SD_K * SD_WROW8);

  // the whole gradient patch: task = (chunk, row, half, column), 8 channel loads (lanes on
  // consecutive columns) -> one b128 LDS write
  for (int t0 = 0; t0 < SG_PATCH8; t0 += 4 * 256) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 256 * u + tid;
      const int pv = t % SG_PV, rest = t / SG_PV;
      const int h = rest & 1, pu = (rest >> 1) % SG_PU, c = (rest >> 1) / SG_PU;
      const int oy = u0 - 1 + pu, ox = v0 - 1 + pv;
      const bool ok = t < SG_PATCH8 && (unsigned)oy < (unsigned)g.P && (unsigned)ox < (unsigned)g.Q;
      const int base = gbase + (16 * c + 8 * h) * PQ + oy * g.Q + ox;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[u][e] = bload(rg, ok ? (base + e * PQ) * 4 : OOR);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 256 * u + tid;
      if (t < SG_PATCH8) patch[t] = sd_cvt8<OP>(v[u]);
    }
  }
  T8 wv[4];
  auto load_w = [&](int c, int r) {
    const int g0 = (c * SD_K + r) * SD_WROW8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int task = tid + 256 * u;
      wv[u] = sd_gload<OP>(rw, g0 + task, task < SD_WROW8);
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int task = tid + 256 * u;
      if (task < SD_WROW8) wl[buf][task] = wv[u];
    }
  };

  sd_f32x16 acc[2][2][2];  // [py][px][ci half]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc[i][j][0] = sd_f32x16{0};
      acc[i][j][1] = sd_f32x16{0};
    }
  // filter row r of chunk c: phase py = (r + 1) & 1 (compile time in each branch)
  auto compute = [&](auto py_c, int c, int r, int buf) {
    constexpr int PY = decltype(py_c)::value;
    const int dr = (PY + 3 - r) >> 1;
    const int prow = ((c * SG_PU + wave + dr + 1) * 2 + lh) * SG_PV + li;
#pragma unroll
    for (int s = 0; s < SD_K; ++s) {
      const int px = (s + 1) & 1, ds = (px + 3 - s) >> 1;
      const T8 a0 = wl[buf][(s * 2 + lh) * 64 + li];
      const T8 a1 = wl[buf][(s * 2 + lh) * 64 + 32 + li];
      const T8 b = patch[prow + ds + 1];
      if (px == 0) {
        acc[PY][0][0] = sd_mfma<OP>(a0, b, acc[PY][0][0]);
        acc[PY][0][1] = sd_mfma<OP>(a1, b, acc[PY][0][1]);
      } else {
        acc[PY][1][0] = sd_mfma<OP>(a0, b, acc[PY][1][0]);
        acc[PY][1][1] = sd_mfma<OP>(a1, b, acc[PY][1][1]);
      }
      // one tap's fragments live at a time: hoisting all seven taps' LDS reads ahead of the
      // MFMAs (hipcc's choice) needs 84 more VGPRs than 2 waves / SIMD leave next to the 128
      // accumulator registers
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  load_w(0, 0);
  store_w(0);
  __syncthreads();
  constexpr int nsteps = SG_CH * SD_K;
  for (int k = 0; k < nsteps; ++k) {
    const int c = k / SD_K, r = k - SD_K * c;
    const int kn = min(k + 1, nsteps - 1);
    load_w(kn / SD_K, kn % SD_K);
    __builtin_amdgcn_sched_barrier(0);
    if (r & 1) compute(std::integral_constant<int, 0>{}, c, r, k & 1);
    else compute(std::integral_constant<int, 1>{}, c, r, k & 1);
    __builtin_amdgcn_sched_barrier(0);
    store_w((k + 1) & 1);
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t rd = rsrc(dx, dx_bytes);
#pragma unroll
  for (int py = 0; py < 2; ++py)
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      const int y = 2 * (u0 + wave) + py, xx = 2 * (v0 + li) + px;
      const bool ok = y < g.H && xx < g.W;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int ci = 32 * a + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
          bstore(rd, ok ? (((n * 64 + ci) * g.H + y) * g.W + xx) * 4 : OOR, acc[py][px][a][rr]);
        }
    }
}

// k_conv_stem_dgrad_lp's weight image: group (c, r, s, half, ci) = W[16c + 8 half + e][ci][r][s],
// e = 0..7, for the 64 gradient channels ci; wt tap-major fp32 [49][64][Cin].
template <int OP>
__global__ void __launch_bounds__(256) k_stem_wprep_dgrad(const float *__restrict__ wt, int Cin,
                                                          typename SdType<OP>::T8 *__restrict__ img) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= SG_CH * SD_K * SD_WROW8) return;
  const int c = i / (SD_K * SD_WROW8), rem = i - c * SD_K * SD_WROW8;
  const int r = rem / SD_WROW8, task = rem - r * SD_WROW8;
  const int s = task >> 7, h = (task >> 6) & 1, ci = task & 63;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = wt[((r * SD_K + s) * 64 + 16 * c + 8 * h + e) * Cin + ci];
  img[i] = sd_cvt8<OP>(v);
}

// ------------------------------------------------------------------------------------------
// Weight gradient of the same conv on bf16 operands (C3): dW[co][ci][r][s] = sum over pixels of
// gy[co][oy][ox] x[ci][2oy + r - 3][2ox + s - 3].  GEMM rows m = co (64), columns n = (ci, r, s)
// of an 8-channel chunk (392 = 13 tiles of 32), K = output pixels.  k_wgrad_lp gathers the
// im2col column of every (ci, tap) from L2 on its own (each x value fetched ~49 times, stride-2
// float4 windows half discarded: 492 us for the stem in the C3 step).  Here a block walks its
// share of 4 x 16 output-pixel tiles for one channel chunk and stages per tile
//  * gy: 64 co x 64 pixels, 16-bit rows of 64 + 8 (144 B: conflict-free b128 reads);
//  * x: the tile's 13 x 37 input window of the 8 channels, written once per filter column s
//    as the stride-2 sample row X[ci][row][s][ox] = x[..][2 ox + s - 3] (16-bit rows of 16 + 8,
//    48 B): the B fragment of column (ci, r, s) and pixel octet (oy, ox..ox+7) is then ONE
//    aligned b128 read at row 2 oy + r — each x value loaded once (coalesced), stored 3-4 times;
//  * wave w: rows co 32 (w & 1) .., column tiles of parity w >> 1 (7 or 6 accumulators).
// Every block writes its chunk's columns of its split slab part[split][co][ci * 49 + tap]
// (k_reduce_splits sums the slabs in split order: deterministic).
// ------------------------------------------------------------------------------------------
constexpr int SW_TH = 4, SW_TW = 16;             // output pixel tile (64 pixels: 4 K-steps)
constexpr int SW_CC = 8;                         // channels per chunk
constexpr int SW_NCOL = SW_CC * SD_K * SD_K;     // 392 columns (ci, r, s)
constexpr int SW_NT = (SW_NCOL + 31) / 32;       // 13 column tiles: 7 + 6 over the two wave pairs
static_assert(SW_NT == 13, "column tiles split 7 + 6");
constexpr int SW_XR = 2 * SW_TH + SD_K - 2;      // 13 input rows (2 (TH - 1) + 7)
constexpr int SW_XC = 2 * SW_TW + SD_K - 2;      // 37 input columns
constexpr int SW_XLD = SW_TW + 8;                // X row stride (elements): 48 B, conflict-free b128
constexpr int SW_GLD = SW_TH * SW_TW + 8;        // G row stride (elements): 144 B
constexpr int SW_OCT = SW_TW / 8;                // pixel octets per tile row
constexpr int SW_GG = 64 * SW_TH * SW_OCT / 256;  // gy octets per thread

template <int OP>
__global__ void __launch_bounds__(256, OP == 0 ? 1 : 2) k_conv_stem_wgrad_lp(const float *__restrict__ gy,
                                                               const float *__restrict__ x,
                                                               float *__restrict__ part,
                                                               int tiles_per_split, ConvGeom g) {
  typedef typename SdType<OP>::T T;
  typedef typename SdType<OP>::T8 T8;
  __shared__ __attribute__((aligned(16))) T Gs[64 * SW_GLD];                   // [co][pixel]
  __shared__ __attribute__((aligned(16))) T Xs[SW_CC * SW_XR * SD_K * SW_XLD];  // [ci][row][s][ox]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int mt = wave & 1, np = wave >> 1;  // co half, column-tile parity
  const int cb = blockIdx.x, sp = blockIdx.y;
  const int tq = (g.Q + SW_TW - 1) / SW_TW, tp = (g.P + SW_TH - 1) / SW_TH;
  const int ntiles = g.N * tp * tq;
  const int t_beg = sp * tiles_per_split, t_end = min(ntiles, t_beg + tiles_per_split);
  const int PQ = g.P * g.Q, HW = g.H * g.W;
  const __amdgpu_buffer_rsrc_t rg = rsrc(gy, 4LL * g.N * 64 * PQ);
  const __amdgpu_buffer_rsrc_t rx = rsrc(x, 4LL * g.N * g.Cin * HW);

  // this lane's B column per tile j (n = 32 (2 j + np) + li): X offset of (ci, r, s)
  int boff[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int n = min(32 * (2 * j + np) + li, SW_NCOL - 1);
    const int ci = n / (SD_K * SD_K), tap = n - SD_K * SD_K * ci;
    const int r = tap / SD_K, s = tap - SD_K * r;
    boff[j] = ((ci * SW_XR + r) * SD_K + s) * SW_XLD + 8 * lh;
  }
  const int njt = np == 0 ? 7 : 6;  // column tiles of this wave (13 = 7 + 6)
  sd_f32x16 acc[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) acc[j] = sd_f32x16{0};

  // per-tile staging through registers, one tile ahead: the next tile's loads are in flight
  // during this tile's MFMAs (staging in dependent rounds of loads left ~12 k cycles of
  // latency per tile; with 4 x 32 tiles the prefetch registers spilled: 343 us)
  constexpr int XT = SW_CC * SW_XR * SW_XC;  // 3848 window values
  constexpr int XU = (XT + 255) / 256;       // 16 per thread
  float4 ga[SW_GG], gb[SW_GG];
  float xv[XU];
  auto load_tile = [&](int t) {
    const int img = t / (tp * tq), rem = t - img * tp * tq;
    const int oy0 = (rem / tq) * SW_TH, ox0 = (rem % tq) * SW_TW;
#pragma unroll
    for (int u = 0; u < SW_GG; ++u) {  // gy: group (co, row, octet)
      const int gi = tid + 256 * u;
      const int j = gi % SW_OCT, oyl = (gi / SW_OCT) % SW_TH, co = gi / (SW_OCT * SW_TH);
      const int oy = oy0 + oyl, ox = ox0 + 8 * j;
      const bool ok = oy < g.P && ox < g.Q;  // Q % 8 == 0: an octet is all in or all out
      const int off = ((img * 64 + co) * g.P + oy) * g.Q + ox;
      ga[u] = bload4(rg, ok ? off * 4 : OOR);
      gb[u] = bload4(rg, ok ? (off + 4) * 4 : OOR);
    }
    const int iy0 = 2 * oy0 - g.ph, ix0 = 2 * ox0 - g.pw;
#pragma unroll
    for (int u = 0; u < XU; ++u) {  // x window: task (ci, row, column), lanes on columns
      const int k = 256 * u + tid;
      const int col = k % SW_XC, rest = k / SW_XC;
      const int row = rest % SW_XR, cl = rest / SW_XR;
      const int ci = SW_CC * cb + cl, iy = iy0 + row, ix = ix0 + col;
      const bool ok = k < XT && ci < g.Cin && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      xv[u] = bload(rx, ok ? (((img * g.Cin + ci) * g.H + iy) * g.W + ix) * 4 : OOR);
    }
  };
  auto store_tile = [&]() {
    // an opaque copy of tid: without it hipcc keeps every slot's store address (computed with
    // the load's) live across the MFMAs and spills
    int tid2 = tid;
    asm volatile("" : "+v"(tid2));
#pragma unroll
    for (int u = 0; u < SW_GG; ++u) {
      const int gi = tid2 + 256 * u;
      const int j = gi % SW_OCT, oyl = (gi / SW_OCT) % SW_TH, co = gi / (SW_OCT * SW_TH);
      const float v[8] = {ga[u].x, ga[u].y, ga[u].z, ga[u].w, gb[u].x, gb[u].y, gb[u].z, gb[u].w};
      *reinterpret_cast<T8 *>(&Gs[co * SW_GLD + oyl * SW_TW + 8 * j]) = sd_cvt8<OP>(v);
    }
    // each window value into its 3-4 stride-2 sample rows (filter columns s = column mod 2,
    // + 2, ..; ox = (column - s) / 2 in range)
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int k = 256 * u + tid2;
      if (k < XT) {
        const int col = k % SW_XC, rest = k / SW_XC;
        const int row = rest % SW_XR, cl = rest / SW_XR;
        const T h = (T)xv[u];
        T *dst = &Xs[(cl * SW_XR + row) * SD_K * SW_XLD];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int s = (col & 1) + 2 * q;
          const int ox2 = col - s;
          if (s < SD_K && ox2 >= 0 && ox2 <= 2 * (SW_TW - 1)) dst[s * SW_XLD + (ox2 >> 1)] = h;
        }
      }
    }
  };

  if (t_beg < t_end) load_tile(t_beg);
  for (int t = t_beg; t < t_end; ++t) {
    __syncthreads();  // the previous tile's fragments are read
    store_tile();
    __syncthreads();
    load_tile(min(t + 1, t_end - 1));  // next tile's loads in flight during the MFMAs
    __builtin_amdgcn_sched_barrier(0);
    // K-steps: (output row, 16-pixel half); A = gy octet of co, B = sample-row octet
#pragma unroll
    for (int ks = 0; ks < SW_TH * SW_TW / 16; ++ks) {
      const int oyl = ks / (SW_TW / 16), hx = ks % (SW_TW / 16);
      const T8 a = *reinterpret_cast<const T8 *>(&Gs[(32 * mt + li) * SW_GLD + oyl * SW_TW + 16 * hx + 8 * lh]);
      const int kofs = 2 * oyl * SD_K * SW_XLD + 16 * hx;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        if (j < njt) {
          const T8 b = *reinterpret_cast<const T8 *>(&Xs[boff[j] + kofs]);
          acc[j] = sd_mfma<OP>(a, b, acc[j]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one K-step's fragments live at a time
    }
  }

  // slab columns of this chunk: n = ci_l * 49 + tap -> column (8 cb + ci_l) * 49 + tap
  const int ncols = g.Cin * SD_K * SD_K;
  const __amdgpu_buffer_rsrc_t rp = rsrc(part, 4LL * gridDim.y * 64 * ncols);
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    if (j >= njt) break;
    const int n = 32 * (2 * j + np) + li;
    const int col = SW_CC * cb * SD_K * SD_K + n;
    const bool nok = n < SW_NCOL && col < ncols;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int co = 32 * mt + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
      bstore(rp, nok ? ((sp * 64 + co) * ncols + col) * 4 : OOR, acc[j][rr]);
    }
  }
}

// The 16-bit weight image k_conv_stem_lp reads: group i (8 values) of the full chunks is
// (c, r, s, half, co) = the 8 input channels 16c + 8 half .. of tap (r, s), output channel co;
// past them the tail's flattened rows k = (remainder channel, tap), 16 per step.  One thread
// per group; wt is tap-major fp32 [49][64][Cin].
template <int OP>
__global__ void __launch_bounds__(256) k_stem_wprep(const float *__restrict__ wt, int Cin,
                                                    typename SdType<OP>::T8 *__restrict__ img) {
  const int nch = Cin >> 4, crem = Cin - 16 * nch;
  const int kt = crem * SD_K * SD_K;
  const int nmain = nch * SD_K * SD_WROW8, total = nmain + ((kt + 15) >> 4) * 128;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  float v[8];
  if (i < nmain) {
    const int c = i / (SD_K * SD_WROW8), rem = i - c * SD_K * SD_WROW8;
    const int r = rem / SD_WROW8, task = rem - r * SD_WROW8;
    const int s = task >> 7, h = (task >> 6) & 1, co = task & 63;
    const float *p = wt + ((r * SD_K + s) * 64 + co) * Cin + 16 * c + 8 * h;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p[e];
  } else {
    const int t = i - nmain, step = t >> 7, h = (t >> 6) & 1, co = t & 63;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 16 * step + 8 * h + e;
      const int cc = k / (SD_K * SD_K), tap = k - SD_K * SD_K * cc;
      v[e] = k < kt ? wt[(tap * 64 + co) * Cin + 16 * nch + cc] : 0.f;
    }
  }
  img[i] = sd_cvt8<OP>(v);
}

static int stem_groups(const ConvGeom &g) {
  const int nch = g.Cin >> 4, kt = (g.Cin - 16 * nch) * SD_K * SD_K;
  return nch * SD_K * SD_WROW8 + ((kt + 15) >> 4) * 128;
}

size_t stem_direct_workspace(const ConvGeom &g, int mode, int op) {
  return (op == 0 ? 32 : 16) * (size_t)(mode == 0 ? stem_groups(g) : SG_CH * SD_K * SD_WROW8);
}

// e2ep_tune key 35 = 1 + mask: 1 the forward, 2 the data gradient, 4 the weight gradient; on fp32
// operands (exact-f32 MFMA: C2, and C5's fp32 weight gradient) also 8 for the gradients and 16
// for the forward
bool stem_direct_ok(int mode, const ConvGeom &g, int M, int op) {
  const int mask = g_tune[TUNE_STEM_DIRECT] - 1;
  if (mode == 0 ? !(mask & 1) : mode == 1 ? !(mask & 2) : mode == 2 ? !(mask & 4) : true) return false;
  if (op < 0 || op > 2 || (op == 0 && !(mask & (mode == 0 ? 16 : 8))) || (mode == 2 && op == 2) ||
      (mode != 2 && g.wlayout != 1))
    return false;
  if (g.R != SD_K || g.S != SD_K || g.sh != 2 || g.sw != 2 || g.dh != 1 || g.dw != 1) return false;
  if (g.Cout != 64 || M != 64 || g.ph < 0 || g.pw < 0) return false;
  if (mode == 0 && g.Cin % 16 > SD_TAILMAX) return false;
  if (mode == 1 && (g.ph != 3 || g.pw != 3 || g.Cin < 64)) return false;
  if (mode == 2 && (g.Q % 8 != 0 || g.Cin > 4096)) return false;
  if (g.P != (g.H + 2 * g.ph - SD_K) / 2 + 1 || g.Q != (g.W + 2 * g.pw - SD_K) / 2 + 1) return false;
  const long long lim = 0x7fffffffLL - 16;
  return 4LL * g.N * g.Cin * g.H * g.W < lim && 4LL * g.N * 64 * g.P * g.Q < lim &&
         4LL * SD_K * SD_K * 64 * g.Cin < lim && g.N <= 65535;
}

int stem_direct_launch(int act, int op, const float *w, const float *x, const float *bias, float *y,
                       long long y_bytes, const ConvGeom &g, void *workspace, hipStream_t s) {
  if (!stem_direct_ok(0, g, 64, op) || (act != 0 && act != 1) || !workspace) {
    set_error("conv: the direct stem kernel does not take this geometry / needs its weight-image "
              "workspace (stem_direct_ok, e2ep_conv_fwd_workspace)");
    return E2EP_EINVAL;
  }
  const int groups = stem_groups(g);
  const dim3 grid(cdiv(g.Q, SD_TW), cdiv(g.P, SD_TH), g.N);
#define SD_LAUNCH(OPV, ACTV)                                                                       \
  do {                                                                                             \
    hipLaunchKernelGGL((k_stem_wprep<OPV>), dim3(cdiv(groups, 256)), dim3(256), 0, s, w, g.Cin,    \
                       static_cast<typename SdType<OPV>::T8 *>(workspace));                        \
    hipLaunchKernelGGL((k_conv_stem_lp<OPV, ACTV>), grid, dim3(256), 0, s, x, workspace, bias, y,  \
                       y_bytes, g);                                                                \
  } while (0)
  if (op == 1) {
    if (act) SD_LAUNCH(1, 1);
    else SD_LAUNCH(1, 0);
  } else if (op == 2) {
    if (act) SD_LAUNCH(2, 1);
    else SD_LAUNCH(2, 0);
  } else {
    if (act) SD_LAUNCH(0, 1);
    else SD_LAUNCH(0, 0);
  }
#undef SD_LAUNCH
  return 0;
}

int stem_dgrad_launch(int op, const float *w, const float *gy, float *dx, long long dx_bytes,
                      const ConvGeom &g, void *workspace, hipStream_t s) {
  if (!stem_direct_ok(1, g, 64, op) || !workspace) {
    set_error("conv: the direct stem data gradient does not take this geometry / needs its "
              "weight-image workspace (stem_direct_ok, e2ep_conv_dgrad_workspace)");
    return E2EP_EINVAL;
  }
  const int groups = SG_CH * SD_K * SD_WROW8;
  const dim3 grid(cdiv((g.W + 1) / 2, SG_TV), cdiv((g.H + 1) / 2, SG_TU), g.N);
#define SG_LAUNCH(OPV)                                                                           \
  do {                                                                                           \
    hipLaunchKernelGGL((k_stem_wprep_dgrad<OPV>), dim3(cdiv(groups, 256)), dim3(256), 0, s, w,   \
                       g.Cin, static_cast<typename SdType<OPV>::T8 *>(workspace));               \
    hipLaunchKernelGGL((k_conv_stem_dgrad_lp<OPV>), grid, dim3(256), 0, s, gy, workspace, dx,    \
                       dx_bytes, g);                                                             \
  } while (0)
  if (op == 1) SG_LAUNCH(1);
  else if (op == 2) SG_LAUNCH(2);
  else SG_LAUNCH(0);
#undef SG_LAUNCH
  return 0;
}

// slabs of the direct weight gradient: ~2 blocks per CU over the channel chunks
int stem_wgrad_splits(const ConvGeom &g) {
  const int chunks = (g.Cin + SW_CC - 1) / SW_CC;
  const int ntiles = g.N * ((g.P + SW_TH - 1) / SW_TH) * ((g.Q + SW_TW - 1) / SW_TW);
  return std::max(1, std::min(ntiles, 512 / chunks));
}

int stem_wgrad_launch(const float *gy, const float *x, const ConvGeom &g, int splits, float *part,
                      hipStream_t s, int op) {
  if (!stem_direct_ok(2, g, 64, op) || splits < 1) {
    set_error("conv: the direct stem weight gradient does not take this geometry (stem_direct_ok)");
    return -1;
  }
  const int ntiles = g.N * ((g.P + SW_TH - 1) / SW_TH) * ((g.Q + SW_TW - 1) / SW_TW);
  const int tps = cdiv(ntiles, splits);
  const int used = cdiv(ntiles, tps);
  const dim3 grid(cdiv(g.Cin, SW_CC), used);
  if (op == 1) hipLaunchKernelGGL((k_conv_stem_wgrad_lp<1>), grid, dim3(256), 0, s, gy, x, part, tps, g);
  else hipLaunchKernelGGL((k_conv_stem_wgrad_lp<0>), grid, dim3(256), 0, s, gy, x, part, tps, g);
  return used;
}

}  // namespace e2ep
