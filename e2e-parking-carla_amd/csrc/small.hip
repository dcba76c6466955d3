// Step bookkeeping and layout kernels that replaced the last PyTorch-native launches of the
// train step: channel concatenation / split (torch.cat of the ASPP branches and the
// UpsamplingConcat inputs, and its backward's slice copies), the sum of the three losses,
// the decoder's PAD-key mask, the BatchNorm num_batches_tracked counters, the gradient sum of
// a two-consumer activation and the step's random draws (dropout seeds, drop-connect, target
// noise) in one launch.
#include "common.h"

namespace e2ep {

constexpr int CAT_MAX = 8;
struct CatPlan {
  const float *src[CAT_MAX];
  float *dst[CAT_MAX];
  int c0[CAT_MAX + 1];  // first channel of piece j in the concatenation; c0[n] = total
  int n;
};

// one float4 of the concatenated tensor [N][Ctot][HW] per thread; split = 0: gather the
// pieces into `cat`, split = 1: scatter `cat` into the pieces.  Coalesced on both sides (a
// piece's channel block is contiguous per image in both layouts).
__global__ void k_cat_channels(CatPlan pl, int N, long long HW4, float4 *cat, int split) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int C = pl.c0[pl.n];
  const long long per_n = (long long)C * HW4;
  if (i >= (long long)N * per_n) return;
  const int n = (int)(i / per_n);
  const long long r = i - n * per_n;
  const int c = (int)(r / HW4);
  const long long p = r - (long long)c * HW4;
  int j = 0;
#pragma unroll
  for (int t = 1; t < CAT_MAX; ++t)
    if (t < pl.n && c >= pl.c0[t]) j = t;
  const int cj = pl.c0[j + 1] - pl.c0[j];
  const long long off = ((long long)n * cj + (c - pl.c0[j])) * HW4 + p;
  if (split)
    reinterpret_cast<float4 *>(pl.dst[j])[off] = cat[i];
  else
    cat[i] = reinterpret_cast<const float4 *>(pl.src[j])[off];
}

// out = a + b elementwise (the gradient of a tensor read by two consumers, nn_ops.fork2)
__global__ void k_add_f32x4(const float4 *a, const float4 *b, long long n4, float4 *out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 x = a[i], y = b[i];
  out[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}
__global__ void k_add_f32(const float *a, const float *b, long long n, float *out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

__global__ void k_sum3(const float *a, const float *b, const float *c, float *out) {
  if (threadIdx.x == 0) out[0] = __fadd_rn(__fadd_rn(a[0], b[0]), c[0]);  // (a + b) + c
}

__global__ void k_eq_mask_i64(const int64_t *tok, long long rstride, int B, int T, int64_t value,
                              uint8_t *mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T) return;
  const int b = i / T, t = i - b * T;
  mask[i] = tok[b * rstride + t] == value ? 1 : 0;
}

__global__ void k_add_i64_multi(const long long *table, int n, long long v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *reinterpret_cast<long long *>(table[i]) += v;
}

// Counter-based step draws: value i of draw number `state[1]` is a splitmix64 hash of
// (state[0], state[1], i); floats take the top 24 bits (uniform on [0, 1)), ints the top 31.
// One block: every thread reads the counter before thread 0 advances it, so each launch (or
// graph replay) draws fresh values.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void __launch_bounds__(1024) k_rng_draw(long long *state, int nf, float *f, int ni,
                                                   int *iv) {
  const unsigned long long seed = (unsigned long long)state[0];
  const unsigned long long ctr = (unsigned long long)state[1];
  const unsigned long long base = mix64(seed ^ mix64(ctr));
  for (int i = threadIdx.x; i < nf + ni; i += blockDim.x) {
    const unsigned long long h = mix64(base + (unsigned long long)i);
    if (i < nf)
      f[i] = (float)(h >> 40) * 0x1p-24f;
    else
      iv[i - nf] = (int)(h >> 33);
  }
  __syncthreads();
  if (threadIdx.x == 0) state[1] = (long long)(ctr + 1);
}

static int cat_plan(const int *chans, int n, int N, long long HW, CatPlan &pl, const char *who) {
  E2EP_REQUIRE(n >= 1 && n <= CAT_MAX && N > 0 && HW > 0 && HW % 4 == 0, E2EP_EINVAL,
               "%s: 1..8 pieces, N > 0, HW > 0 and a multiple of 4", who);
  pl.n = n;
  pl.c0[0] = 0;
  for (int j = 0; j < n; ++j) {
    E2EP_REQUIRE(chans[j] > 0, E2EP_EINVAL, "%s: piece %d has no channels", who, j);
    pl.c0[j + 1] = pl.c0[j] + chans[j];
  }
  for (int j = n + 1; j <= CAT_MAX; ++j) pl.c0[j] = pl.c0[n];
  return 0;
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_cat_channels(const float *const *srcs, const int *chans, int n, int N, long long HW,
                      float *dst, void *stream) {
  CatPlan pl{};
  if (int rc = cat_plan(chans, n, N, HW, pl, "e2ep_cat_channels")) return rc;
  for (int j = 0; j < n; ++j) {
    E2EP_REQUIRE(((uintptr_t)srcs[j] & 15) == 0, E2EP_EINVAL, "e2ep_cat_channels: 16-B aligned pieces");
    pl.src[j] = srcs[j];
  }
  E2EP_REQUIRE(((uintptr_t)dst & 15) == 0, E2EP_EINVAL, "e2ep_cat_channels: 16-B aligned output");
  const long long tot = (long long)N * pl.c0[n] * (HW / 4);
  hipLaunchKernelGGL(k_cat_channels, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0,
                     as_stream(stream), pl, N, HW / 4, reinterpret_cast<float4 *>(dst), 0);
  return launch_status("e2ep_cat_channels");
}

int e2ep_split_channels(const float *src, const int *chans, int n, int N, long long HW,
                        float *const *dsts, void *stream) {
  CatPlan pl{};
  if (int rc = cat_plan(chans, n, N, HW, pl, "e2ep_split_channels")) return rc;
  for (int j = 0; j < n; ++j) {
    E2EP_REQUIRE(((uintptr_t)dsts[j] & 15) == 0, E2EP_EINVAL, "e2ep_split_channels: 16-B aligned pieces");
    pl.dst[j] = dsts[j];
  }
  E2EP_REQUIRE(((uintptr_t)src & 15) == 0, E2EP_EINVAL, "e2ep_split_channels: 16-B aligned input");
  const long long tot = (long long)N * pl.c0[n] * (HW / 4);
  hipLaunchKernelGGL(k_cat_channels, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0,
                     as_stream(stream), pl, N, HW / 4,
                     reinterpret_cast<float4 *>(const_cast<float *>(src)), 1);
  return launch_status("e2ep_split_channels");
}

int e2ep_add_f32(const float *a, const float *b, long long n, float *out, void *stream) {
  E2EP_REQUIRE(n >= 0, E2EP_EINVAL, "e2ep_add_f32: n < 0");
  if (n == 0) return 0;
  if (n % 4 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) & 15) == 0)
    hipLaunchKernelGGL(k_add_f32x4, dim3(cdiv(n / 4, 256)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4 *>(a), reinterpret_cast<const float4 *>(b),
                       n / 4, reinterpret_cast<float4 *>(out));
  else
    hipLaunchKernelGGL(k_add_f32, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), a, b, n, out);
  return launch_status("e2ep_add_f32");
}

int e2ep_sum3(const float *a, const float *b, const float *c, float *out, void *stream) {
  hipLaunchKernelGGL(k_sum3, dim3(1), dim3(64), 0, as_stream(stream), a, b, c, out);
  return launch_status("e2ep_sum3");
}

int e2ep_eq_mask_i64(const int64_t *tok, long long rstride, int B, int T, int64_t value,
                     uint8_t *mask, void *stream) {
  E2EP_REQUIRE(B >= 0 && T >= 0, E2EP_EINVAL, "e2ep_eq_mask_i64: bad shape");
  if (B * T == 0) return 0;
  hipLaunchKernelGGL(k_eq_mask_i64, dim3(cdiv(B * T, 256)), dim3(256), 0, as_stream(stream), tok,
                     rstride, B, T, value, mask);
  return launch_status("e2ep_eq_mask_i64");
}

int e2ep_rng_draw(long long *state, int nf, float *f, int ni, int *iv, void *stream) {
  E2EP_REQUIRE(nf >= 0 && ni >= 0 && (nf == 0 || f) && (ni == 0 || iv), E2EP_EINVAL,
               "e2ep_rng_draw: bad arguments");
  hipLaunchKernelGGL(k_rng_draw, dim3(1), dim3(1024), 0, as_stream(stream), state, nf, f, ni, iv);
  return launch_status("e2ep_rng_draw");
}

int e2ep_add_i64_multi(const long long *table, int n, long long v, void *stream) {
  E2EP_REQUIRE(n >= 0, E2EP_EINVAL, "e2ep_add_i64_multi: n < 0");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_add_i64_multi, dim3(cdiv(n, 256)), dim3(256), 0, as_stream(stream), table,
                     n, v);
  return launch_status("e2ep_add_i64_multi");
}

}  // extern "C"
