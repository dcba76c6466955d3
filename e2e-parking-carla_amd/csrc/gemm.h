// Internal interface of the strided / column-batched MFMA GEMM (gemm.hip), shared with the
// 1x1-convolution path of conv.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace e2ep {

// Column batching (1x1 convolutions, NCHW): with hw > 0, column n = (image n / hw, pixel
// n % hw); B(k, n) = B[img * b_img + k * ldb + p] and C(m, n) = C[img * c_img + m * ldc + p]
// (Cadd in C's layout).  hw must be a multiple of 32.
struct GemmCols {
  int hw;  // 0: plain matrix
  long long b_img, c_img;
};

// C = A B (+ bias: per column, or per row when bias_rows) (+ Cadd) (ReLU); see gemm.hip.
int gemm_run(const float *A, int lda, bool ak, long long a_bytes, const float *B, int ldb,
             bool bk, long long b_bytes, const float *bias, bool bias_rows, const float *Cadd,
             int ldadd, float *C, long long c_bytes, int ldc, GemmCols cols, int M, int N, int K,
             int relu, void *workspace, hipStream_t s, float *rs = nullptr);
size_t gemm_ws(int M, int N, int K);

}  // namespace e2ep
