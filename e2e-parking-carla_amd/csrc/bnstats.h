// BatchNorm batch statistics taken in a producer's epilogue (e2ep_conv_fwd_stats): per output
// channel (GEMM row) and per column tile, the fp64 sum and sum of squares of the values the
// epilogue stores, written as partial pairs in the layout the BN kernels reduce
// tile-major: part[(tile * C + c) * 2 + {0, 1}], so a block's partials are one contiguous run
// of whole cache lines (a channel-major layout scattered 16-B writes over the lines of 8
// blocks and cost the 128 x 128 expand conv 53 us of its 125).  The BN layer that follows
// reduces them (bn.hip k_bn_finalize_tiles) instead of re-reading its input (k_bn_stats).
//
// Accumulator layout (v_mfma_f32_32x32x*): lane half h = lane >> 5 holds rows
// (r & 3) + 8 (r >> 2) + 4 h of its 32-row wave tile in element r, lanes li = lane & 31 the
// columns.  A butterfly reduce-scatter over the 32 lanes of a half (steps 16, 8, 4, 2 halve
// the rows each lane carries, step 1 completes the sum) leaves row (li >> 1) & 15 in lanes li
// and li ^ 1: 2 x 16 shuffles per statistic instead of 16 x 5.  Every sum has a fixed tree,
// so the statistics are deterministic run to run.
#pragma once
#include "common.h"

namespace e2ep {

template <int N>
__device__ __forceinline__ void bns_bfly(const double *in, double *out, int lane, int off) {
  const bool hi = (lane & off) != 0;
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    const double send = hi ? in[j] : in[j + N / 2];
    const double keep = hi ? in[j + N / 2] : in[j];
    out[j] = keep + __shfl_xor(send, off, 64);
  }
}

// sum over the 32 lanes of this lane's half of row (lane >> 1) & 15 of v
__device__ __forceinline__ double bns_half_rowsum(const double (&v)[16], int lane) {
  double a8[8], a4[4], a2[2], a1[1];
  bns_bfly<16>(v, a8, lane, 16);
  bns_bfly<8>(a8, a4, lane, 8);
  bns_bfly<4>(a4, a2, lane, 4);
  bns_bfly<2>(a2, a1, lane, 2);
  return a1[0] + __shfl_xor(a1[0], 1, 64);
}

// Block epilogue: bs[i] / bq[i] = this lane's sums for row r of the wave's i-th 32-row block
// (elements of columns outside the output already zero), the blocks starting at block-local
// row row0 + 32 i; waves wn = 0 .. nwn-1 share rows and are summed in wn order through `red`
// (__shared__ of the caller: nwn x bmt x 2 doubles, [wn][row][2]).  Every thread of the block
// must call it (one barrier).  Writes stats[(tile * M + m) * 2 + {0, 1}] for the bmt rows.
template <int NI>
__device__ __forceinline__ void bns_store_tile_n(const double (&bs)[NI][16],
                                                 const double (&bq)[NI][16], int row0, int wn,
                                                 int nwn, int bmt, int m0, int M, int tile,
                                                 double *red, double *__restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 31, r = (li >> 1) & 15;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const double s = bns_half_rowsum(bs[i], lane);
    const double q = bns_half_rowsum(bq[i], lane);
    if ((li & 1) == 0) {
      const int row = row0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      red[(wn * bmt + row) * 2] = s;
      red[(wn * bmt + row) * 2 + 1] = q;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < bmt && m0 + t < M) {
    double S = red[t * 2], Q = red[t * 2 + 1];
    for (int w = 1; w < nwn; ++w) {
      S += red[(w * bmt + t) * 2];
      Q += red[(w * bmt + t) * 2 + 1];
    }
    const size_t o = ((size_t)tile * M + m0 + t) * 2;
    stats[o] = S;
    stats[o + 1] = Q;
  }
}

// one 32-row block per wave (k_conv_gemm)
__device__ __forceinline__ void bns_store_tile(const double (&bs)[16], const double (&bq)[16],
                                               int wm, int wn, int nwn, int bmt, int m0, int M,
                                               int tile, double *red, double *__restrict__ stats) {
  const double(&b1)[1][16] = reinterpret_cast<const double(&)[1][16]>(bs);
  const double(&q1)[1][16] = reinterpret_cast<const double(&)[1][16]>(bq);
  bns_store_tile_n<1>(b1, q1, 32 * wm, wn, nwn, bmt, m0, M, tile, red, stats);
}

}  // namespace e2ep
