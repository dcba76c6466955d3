// Residual add + dropout + LayerNorm, fused, for the post-norm transformer layers of the
// feature fusion encoder and the control decoder (torch.nn.TransformerEncoderLayer /
// TransformerDecoderLayer, reference model/feature_fusion.py:13-14,48-50 and
// model/control_predict.py:19-20,39-47):  y = LayerNorm(a + dropout(b))  with
// dropout(b) = b * [u >= p] / (1 - p)  (u: uniform draws, one per element; p = 0: identity),
// or, without u, the counter hash of dropout.h keyed by a per-call device seed (element index
// row * E + c as the counter) — no uniform tensor is drawn, written or read.
// Forward: one wave per row (E = d_model columns, lanes stride the row).  Backward: one wave
// per row for the input gradients (da = dx, db = dx * mask / (1 - p)); gamma / beta gradients
// as per-block column partials over fixed row ranges, summed in block order by a second
// kernel — deterministic.
#include "common.h"
#include "dropout.h"

namespace e2ep {

constexpr int LN_MAXV = 8;  // up to 512 columns per row (8 per lane)

__global__ void __launch_bounds__(256) k_add_drop_ln_fwd(
    const float *__restrict__ a, const float *__restrict__ b, const float *__restrict__ u,
    const int *__restrict__ seed, float p, float scale, const float *__restrict__ gamma,
    const float *__restrict__ beta, int rows, int E, float eps, float *__restrict__ x,
    float *__restrict__ y, float *__restrict__ mean, float *__restrict__ rstd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const size_t base = (size_t)row * E;
  const bool hashed = !u && seed && p > 0.f;
  const uint32_t sm_ = hashed ? att_seedmix(seed) : 0u;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    const int c = lane + 64 * j;
    v[j] = 0.f;
    if (c < E) {
      float bv = b ? b[base + c] : 0.f;
      if (u) bv = u[base + c] >= p ? bv * scale : 0.f;
      else if (hashed) bv = att_keep(sm_, (uint32_t)(base + c), p) ? bv * scale : 0.f;
      v[j] = a[base + c] + bv;
      s += v[j];
    }
  }
  const float mu = wave_sum(s) / (float)E;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    const int c = lane + 64 * j;
    if (c < E) {
      const float d = v[j] - mu;
      q += d * d;
    }
  }
  const float r = rsqrtf(wave_sum(q) / (float)E + eps);
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    const int c = lane + 64 * j;
    if (c < E) {
      if (x) x[base + c] = v[j];
      y[base + c] = (v[j] - mu) * r * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = r;
  }
}

// input gradients (wave per row) + gamma/beta partials per block: block = 4 waves x
// LN_ROWS_PER_WAVE rows; partial[blk][c] (dgamma) and partial[nblk + blk][c] (dbeta)
constexpr int LN_ROWS_PER_WAVE = 1;

__global__ void __launch_bounds__(256) k_add_drop_ln_bwd(
    const float *__restrict__ dy, const float *__restrict__ x, const float *__restrict__ mean,
    const float *__restrict__ rstd, const float *__restrict__ gamma, const float *__restrict__ u,
    const int *__restrict__ seed, float p, float scale, int rows, int E, float *__restrict__ da,
    float *__restrict__ db, float *__restrict__ part) {
  const bool hashed = !u && seed && p > 0.f;
  const uint32_t sm_ = hashed ? att_seedmix(seed) : 0u;
  __shared__ float sg[4][LN_MAXV * 64], sb[4][LN_MAXV * 64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float pg[LN_MAXV], pb[LN_MAXV];
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) pg[j] = pb[j] = 0.f;
  const int r0 = (blockIdx.x * 4 + wave) * LN_ROWS_PER_WAVE;
  for (int i = 0; i < LN_ROWS_PER_WAVE; ++i) {
    const int row = r0 + i;
    if (row >= rows) break;  // wave-uniform
    const size_t base = (size_t)row * E;
    const float mu = mean[row], rs = rstd[row];
    float xh[LN_MAXV], gy[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      const int c = lane + 64 * j;
      xh[j] = gy[j] = 0.f;
      if (c < E) {
        const float g = dy[base + c];
        xh[j] = (x[base + c] - mu) * rs;
        gy[j] = g * (gamma ? gamma[c] : 1.f);
        pg[j] += g * xh[j];
        pb[j] += g;
        s1 += gy[j];
        s2 += gy[j] * xh[j];
      }
    }
    const float c1 = wave_sum(s1) / (float)E, c2 = wave_sum(s2) / (float)E;
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      const int c = lane + 64 * j;
      if (c < E) {
        const float dx = rs * (gy[j] - c1 - xh[j] * c2);
        if (da) da[base + c] = dx;
        if (db)
          db[base + c] = u        ? (u[base + c] >= p ? dx * scale : 0.f)
                         : hashed ? (att_keep(sm_, (uint32_t)(base + c), p) ? dx * scale : 0.f)
                                  : dx;
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    sg[wave][lane + 64 * j] = pg[j];
    sb[wave][lane + 64 * j] = pb[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < E; c += 256) {
    part[(size_t)blockIdx.x * E + c] = (sg[0][c] + sg[1][c]) + (sg[2][c] + sg[3][c]);
    part[((size_t)gridDim.x + blockIdx.x) * E + c] = (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]);
  }
}

// dgamma / dbeta = fixed-order sums of the per-block partials: block = 64 columns x 16
// partial lanes (thread (c, r) takes blocks r, r+16, ...), lanes added in order via LDS;
// grid (columns / 64, 2): y = 0 gamma, 1 beta
__global__ void __launch_bounds__(1024) k_ln_param_grads(const float *__restrict__ part, int nblk,
                                                         int E, float *__restrict__ dgamma,
                                                         float *__restrict__ dbeta) {
  __shared__ float red[16][64];
  const int o = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + o;
  const float *pp = part + (size_t)blockIdx.y * nblk * E;
  float s = 0.f;
  if (c < E)
    for (int k = r; k < nblk; k += 16) s += pp[(size_t)k * E + c];
  red[r][o] = s;
  __syncthreads();
  if (r == 0 && c < E) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][o];
    float *out = blockIdx.y == 0 ? dgamma : dbeta;
    if (out) out[c] = t;
  }
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

static int add_drop_ln_fwd(const float *a, const float *b, const float *u, const int *seed,
                           float p, const float *gamma, const float *beta, int rows, int E,
                           float eps, float *x, float *y, float *mean, float *rstd,
                           hipStream_t stream) {
  E2EP_REQUIRE(rows > 0 && E > 0, E2EP_EINVAL, "e2ep_add_drop_ln_fwd: bad shape");
  E2EP_REQUIRE(E <= 64 * LN_MAXV, E2EP_ERANGE, "e2ep_add_drop_ln_fwd: E %d > %d", E, 64 * LN_MAXV);
  E2EP_REQUIRE(p >= 0.f && p < 1.f, E2EP_EINVAL, "e2ep_add_drop_ln_fwd: p must be in [0, 1)");
  E2EP_REQUIRE((long long)rows * E < 0xffffffffLL, E2EP_ERANGE, "e2ep_add_drop_ln_fwd: too large");
  const float scale = 1.f / (1.f - p);
  hipLaunchKernelGGL(k_add_drop_ln_fwd, dim3(cdiv(rows, 4)), dim3(256), 0, stream, a, b, u, seed,
                     p, scale, gamma, beta, rows, E, eps, x, y, mean, rstd);
  return launch_status("e2ep_add_drop_ln_fwd");
}

int e2ep_add_drop_ln_fwd(const float *a, const float *b, const float *u, float p,
                         const float *gamma, const float *beta, int rows, int E, float eps,
                         float *x, float *y, float *mean, float *rstd, void *stream) {
  return add_drop_ln_fwd(a, b, u, nullptr, p, gamma, beta, rows, E, eps, x, y, mean, rstd,
                         as_stream(stream));
}

int e2ep_add_drop_ln_fwd_seeded(const float *a, const float *b, const int *seed, float p,
                                const float *gamma, const float *beta, int rows, int E, float eps,
                                float *x, float *y, float *mean, float *rstd, void *stream) {
  E2EP_REQUIRE(seed || p == 0.f, E2EP_EINVAL, "e2ep_add_drop_ln_fwd_seeded: seed required for p > 0");
  return add_drop_ln_fwd(a, b, nullptr, seed, p, gamma, beta, rows, E, eps, x, y, mean, rstd,
                         as_stream(stream));
}

size_t e2ep_add_drop_ln_bwd_workspace(int rows, int E) {
  return (size_t)2 * cdiv(rows, 4 * LN_ROWS_PER_WAVE) * E * sizeof(float);
}

static int add_drop_ln_bwd(const float *dy, const float *x, const float *mean, const float *rstd,
                           const float *gamma, const float *u, const int *seed, float p, int rows,
                           int E, float *da, float *db, float *dgamma, float *dbeta,
                           void *workspace, hipStream_t stream) {
  E2EP_REQUIRE(rows > 0 && E > 0, E2EP_EINVAL, "e2ep_add_drop_ln_bwd: bad shape");
  E2EP_REQUIRE(E <= 64 * LN_MAXV, E2EP_ERANGE, "e2ep_add_drop_ln_bwd: E %d > %d", E, 64 * LN_MAXV);
  const float scale = 1.f / (1.f - p);
  const int nblk = cdiv(rows, 4 * LN_ROWS_PER_WAVE);
  float *part = (dgamma || dbeta) ? static_cast<float *>(workspace) : nullptr;
  E2EP_REQUIRE(!(dgamma || dbeta) || workspace, E2EP_EINVAL, "e2ep_add_drop_ln_bwd: workspace needed");
  hipLaunchKernelGGL(k_add_drop_ln_bwd, dim3(nblk), dim3(256), 0, stream, dy, x, mean, rstd,
                     gamma, u, seed, p, scale, rows, E, da, db, part);
  if (part)
    hipLaunchKernelGGL(k_ln_param_grads, dim3(cdiv(E, 64), 2), dim3(1024), 0, stream, part, nblk,
                       E, dgamma, dbeta);
  return launch_status("e2ep_add_drop_ln_bwd");
}

int e2ep_add_drop_ln_bwd(const float *dy, const float *x, const float *mean, const float *rstd,
                         const float *gamma, const float *u, float p, int rows, int E,
                         float *da, float *db, float *dgamma, float *dbeta, void *workspace,
                         void *stream) {
  return add_drop_ln_bwd(dy, x, mean, rstd, gamma, u, nullptr, p, rows, E, da, db, dgamma, dbeta,
                         workspace, as_stream(stream));
}

int e2ep_add_drop_ln_bwd_seeded(const float *dy, const float *x, const float *mean,
                                const float *rstd, const float *gamma, const int *seed, float p,
                                int rows, int E, float *da, float *db, float *dgamma,
                                float *dbeta, void *workspace, void *stream) {
  E2EP_REQUIRE(seed || p == 0.f, E2EP_EINVAL, "e2ep_add_drop_ln_bwd_seeded: seed required for p > 0");
  return add_drop_ln_bwd(dy, x, mean, rstd, gamma, nullptr, seed, p, rows, E, da, db, dgamma,
                         dbeta, workspace, as_stream(stream));
}

}  // extern "C"
