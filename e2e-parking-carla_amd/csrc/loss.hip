// The three training losses of the ParkingModel step as fused HIP kernels (fp32), forward and
// backward, replacing the reference's PyTorch op chains:
//   control  loss/control_loss.py:15-19  cross entropy over (B*T, vocab) logits vs gt[:, 1:],
//            ignore_index = PAD, mean over the non-ignored rows;
//   segment. loss/seg_loss.py:12-26      per-pixel class-weighted cross entropy
//            (reduction='none', ignore_index=255), then a plain mean over ALL pixels;
//   depth    loss/depth_loss.py:18-48    ground-truth depth -> min non-zero depth of each
//            down x down cell -> depth bin -> one-hot(D+1)[1:] labels, BCE on the cells with
//            a label (foreground), summed / max(1, #foreground).
// Every reduction runs in a fixed order (per-row / per-block partials, then one block sums
// the partials by index), so the losses are bitwise run-to-run deterministic.  Nothing is
// copied to the host: the reference's boolean foreground indexing (a data-dependent shape)
// becomes a per-cell mask, and the backward kernels read the upstream gradient and the
// normaliser from device memory, so all six launches are graph-capturable.
#include "common.h"

namespace e2ep {

constexpr int LOSS_THREADS = 256;

// fixed-order block sum of one value per thread; returns the total in every thread
__device__ __forceinline__ float block_sum(float v, float *red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---- control cross entropy ----------------------------------------------------------------
// row r = b*T + t: logits x[r, :V], target gt[b*gstride + goff + t]
__global__ void __launch_bounds__(LOSS_THREADS)
    k_ctrl_ce_rows(const float *__restrict__ x, const long long *__restrict__ gt, int R, int T,
                   int gstride, int goff, int V, int pad, float *__restrict__ row_loss,
                   float *__restrict__ row_valid, float *__restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (LOSS_THREADS / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  const float *xr = x + (long long)r * V;
  float m = -INFINITY;
  for (int v = lane; v < V; v += 64) m = fmaxf(m, xr[v]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float s = 0.f;
  for (int v = lane; v < V; v += 64) s += expf(xr[v] - m);
  s = wave_sum(s);
  const float l = m + logf(s);  // logsumexp
  const long long t = gt[(long long)(r / T) * gstride + goff + (r % T)];
  if (lane == 0) {
    const bool ok = t != pad && t >= 0 && t < V;
    row_loss[r] = ok ? l - xr[t] : 0.f;
    row_valid[r] = ok ? 1.f : 0.f;
    lse[r] = l;
  }
}

// one block: loss = sum(row_loss) / sum(row_valid), count = sum(row_valid)
__global__ void __launch_bounds__(LOSS_THREADS)
    k_ctrl_ce_final(const float *__restrict__ row_loss, const float *__restrict__ row_valid, int R,
                    float *__restrict__ loss, float *__restrict__ count) {
  __shared__ float red[LOSS_THREADS / 64];
  float a = 0.f, c = 0.f;
  for (int r = threadIdx.x; r < R; r += LOSS_THREADS) {
    a += row_loss[r];
    c += row_valid[r];
  }
  const float sa = block_sum(a, red);
  const float sc = block_sum(c, red);
  if (threadIdx.x == 0) {
    loss[0] = sc > 0.f ? sa / sc : NAN;  // torch: mean over zero rows is nan
    count[0] = sc;
  }
}

__global__ void __launch_bounds__(LOSS_THREADS)
    k_ctrl_ce_bwd(const float *__restrict__ x, const long long *__restrict__ gt,
                  const float *__restrict__ lse, const float *__restrict__ count,
                  const float *__restrict__ gloss, int R, int T, int gstride, int goff, int V,
                  int pad, float *__restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (LOSS_THREADS / 64) + (threadIdx.x >> 6);
  if (r >= R) return;
  const long long t = gt[(long long)(r / T) * gstride + goff + (r % T)];
  const bool ok = t != pad && t >= 0 && t < V;
  const float scale = ok ? gloss[0] / count[0] : 0.f;
  const float l = lse[r];
  const float *xr = x + (long long)r * V;
  float *dr = dx + (long long)r * V;
  for (int v = lane; v < V; v += 64) {
    const float p = expf(xr[v] - l);
    dr[v] = scale * (p - (v == t ? 1.f : 0.f));
  }
}

// ---- segmentation weighted cross entropy ---------------------------------------------------
// logits x[n][c][hw], target tg[n][hw] (int64), class weights w[C]
__global__ void __launch_bounds__(LOSS_THREADS)
    k_seg_ce_fwd(const float *__restrict__ x, const long long *__restrict__ tg,
                 const float *__restrict__ w, int Nimg, int C, int HW, int ignore,
                 float *__restrict__ part) {
  __shared__ float red[LOSS_THREADS / 64];
  const long long i = (long long)blockIdx.x * LOSS_THREADS + threadIdx.x;
  float v = 0.f;
  if (i < (long long)Nimg * HW) {
    const long long n = i / HW, p = i - n * HW;
    const float *xp = x + n * C * HW + p;
    const long long t = tg[i];
    if (t != ignore && t >= 0 && t < C) {
      float m = -INFINITY;
      for (int c = 0; c < C; ++c) m = fmaxf(m, xp[(long long)c * HW]);
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += expf(xp[(long long)c * HW] - m);
      v = w[t] * (m + logf(s) - xp[t * HW]);
    }
  }
  const float b = block_sum(v, red);
  if (threadIdx.x == 0) part[blockIdx.x] = b;
}

// one block: out = scale_num * sum(part[0:n]) / den, den = max(den_min, sum(cnt)) or den_fixed
__global__ void __launch_bounds__(LOSS_THREADS)
    k_loss_final(const float *__restrict__ part, const float *__restrict__ cnt, int n,
                 float den_fixed, float *__restrict__ loss, float *__restrict__ den_out) {
  __shared__ float red[LOSS_THREADS / 64];
  float a = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < n; i += LOSS_THREADS) {
    a += part[i];
    if (cnt) c += cnt[i];
  }
  const float sa = block_sum(a, red);
  const float sc = cnt ? block_sum(c, red) : 0.f;
  if (threadIdx.x == 0) {
    const float den = cnt ? fmaxf(1.f, sc) : den_fixed;
    loss[0] = sa / den;
    if (den_out) den_out[0] = den;
  }
}

__global__ void __launch_bounds__(LOSS_THREADS)
    k_seg_ce_bwd(const float *__restrict__ x, const long long *__restrict__ tg,
                 const float *__restrict__ w, const float *__restrict__ gloss, int Nimg, int C,
                 int HW, int ignore, float *__restrict__ dx) {
  const long long i = (long long)blockIdx.x * LOSS_THREADS + threadIdx.x;
  if (i >= (long long)Nimg * HW) return;
  const long long n = i / HW, p = i - n * HW;
  const float *xp = x + n * C * HW + p;
  float *dp = dx + n * C * HW + p;
  const long long t = tg[i];
  if (t == ignore || t < 0 || t >= C) {
    for (int c = 0; c < C; ++c) dp[(long long)c * HW] = 0.f;
    return;
  }
  const float scale = gloss[0] / (float)((long long)Nimg * HW) * w[t];
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, xp[(long long)c * HW]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += expf(xp[(long long)c * HW] - m);
  const float l = m + logf(s);
  for (int c = 0; c < C; ++c)
    dp[(long long)c * HW] = scale * (expf(xp[(long long)c * HW] - l) - (c == t ? 1.f : 0.f));
}

// ---- depth BCE ------------------------------------------------------------------------------
// gt [BN][H][W] metres, prob [BN][D][h][w] (h = H/down, w = W/down); one thread per cell.
// cls[cell] = the one-hot class (1..D foreground, 0 background), kept for the backward.
__device__ __forceinline__ float bce_term(float p, float l) {
  // torch binary_cross_entropy: (l - 1) * max(log1p(-p), -100) - l * max(log(p), -100)
  return (l - 1.f) * fmaxf(log1pf(-p), -100.f) - l * fmaxf(logf(p), -100.f);
}

// T is the ground-truth type: fp32, or fp64 as the reference dataset delivers it
// (dataset/carla_dataset.py:107-113 returns float64 metres); the bin arithmetic runs in T, as
// torch does on a T tensor.
template <typename T>
__global__ void __launch_bounds__(LOSS_THREADS)
    k_depth_bce_fwd(const float *__restrict__ prob, const T *__restrict__ gt, int BN, int D,
                    int H, int W, int down, T lo, T step, int *__restrict__ cls,
                    float *__restrict__ part, float *__restrict__ part_fg) {
  __shared__ float red[LOSS_THREADS / 64];
  const int h = H / down, w = W / down;
  const long long cells = (long long)BN * h * w;
  const long long i = (long long)blockIdx.x * LOSS_THREADS + threadIdx.x;
  float v = 0.f, fg = 0.f;
  if (i < cells) {
    const long long bn = i / (h * w);
    const int pix = (int)(i - bn * h * w), ci = pix / w, cj = pix - ci * w;
    const T *g = gt + (bn * H + (long long)ci * down) * W + (long long)cj * down;
    T mn = T(1e5);
    for (int r = 0; r < down; ++r)
      for (int c = 0; c < down; ++c) {
        const T d = g[(long long)r * W + c];
        const T e = d == T(0) ? T(1e5) : d;
        mn = e < mn ? e : mn;
      }
    // (d - (d0 - step)) / step, kept in [0, D+1) else 0, truncated: the bin; one-hot[1:]
    const T b = (mn - lo) / step;
    const int k = (b < T(D + 1) && b >= T(0)) ? (int)b : 0;
    cls[i] = k;
    if (k >= 1) {
      fg = 1.f;
      const float *pp = prob + bn * D * h * w + pix;
      for (int d = 0; d < D; ++d) v += bce_term(pp[(long long)d * h * w], d + 1 == k ? 1.f : 0.f);
    }
  }
  const float s = block_sum(v, red);
  const float f = block_sum(fg, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s;
    part_fg[blockIdx.x] = f;
  }
}

__global__ void __launch_bounds__(LOSS_THREADS)
    k_depth_bce_bwd(const float *__restrict__ prob, const int *__restrict__ cls,
                    const float *__restrict__ den, const float *__restrict__ gloss, int BN, int D,
                    int hw, float *__restrict__ dprob) {
  const long long i = (long long)blockIdx.x * LOSS_THREADS + threadIdx.x;
  if (i >= (long long)BN * hw) return;
  const long long bn = i / hw;
  const int pix = (int)(i - bn * hw);
  const int k = cls[i];
  const float *pp = prob + bn * D * hw + pix;
  float *dp = dprob + bn * D * hw + pix;
  const float scale = k >= 1 ? gloss[0] / den[0] : 0.f;
  for (int d = 0; d < D; ++d) {
    // torch BCE backward: g * (p - l) / max((1 - p) * p, 1e-12)
    const float p = pp[(long long)d * hw];
    const float l = d + 1 == k ? 1.f : 0.f;
    dp[(long long)d * hw] = k >= 1 ? scale * (p - l) / fmaxf((1.f - p) * p, 1e-12f) : 0.f;
  }
}

}  // namespace e2ep

using namespace e2ep;

template <typename T>
static int depth_bce_fwd(const char *name, const float *prob, const T *gt, int BN, int D, int H,
                         int W, int down, T lo, T step, float *loss, float *den, int *cls,
                         void *workspace, void *stream) {
  E2EP_REQUIRE(prob && gt && loss && den && cls && workspace, E2EP_EINVAL, "%s: null argument",
               name);
  E2EP_REQUIRE(BN > 0 && D > 0 && down > 0 && H % down == 0 && W % down == 0, E2EP_EINVAL,
               "%s: bad shape H=%d W=%d down=%d", name, H, W, down);
  const int nb = cdiv((long long)BN * (H / down) * (W / down), LOSS_THREADS);
  float *part = static_cast<float *>(workspace), *part_fg = part + nb;
  hipLaunchKernelGGL(k_depth_bce_fwd<T>, dim3(nb), dim3(LOSS_THREADS), 0, as_stream(stream), prob,
                     gt, BN, D, H, W, down, lo, step, cls, part, part_fg);
  hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(LOSS_THREADS), 0, as_stream(stream), part,
                     part_fg, nb, 0.f, loss, den);
  return launch_status(name);
}

extern "C" {

size_t e2ep_control_ce_workspace(int rows) { return (size_t)rows * 2 * sizeof(float); }

int e2ep_control_ce_fwd(const float *logits, const long long *gt, int B, int T, int gt_stride,
                        int gt_offset, int vocab, int pad, float *loss, float *lse, float *count,
                        void *workspace, void *stream) {
  E2EP_REQUIRE(logits && gt && loss && lse && count && workspace, E2EP_EINVAL,
               "e2ep_control_ce_fwd: null argument");
  E2EP_REQUIRE(B > 0 && T > 0 && vocab > 0 && gt_offset + T <= gt_stride, E2EP_EINVAL,
               "e2ep_control_ce_fwd: bad shape B=%d T=%d stride=%d offset=%d", B, T, gt_stride,
               gt_offset);
  const int R = B * T;
  float *row_loss = static_cast<float *>(workspace), *row_valid = row_loss + R;
  hipLaunchKernelGGL(k_ctrl_ce_rows, dim3(cdiv(R, LOSS_THREADS / 64)), dim3(LOSS_THREADS), 0,
                     as_stream(stream), logits, gt, R, T, gt_stride, gt_offset, vocab, pad, row_loss,
                     row_valid, lse);
  hipLaunchKernelGGL(k_ctrl_ce_final, dim3(1), dim3(LOSS_THREADS), 0, as_stream(stream), row_loss,
                     row_valid, R, loss, count);
  return launch_status("e2ep_control_ce_fwd");
}

int e2ep_control_ce_bwd(const float *logits, const long long *gt, const float *lse,
                        const float *count, const float *gloss, int B, int T, int gt_stride,
                        int gt_offset, int vocab, int pad, float *dlogits, void *stream) {
  E2EP_REQUIRE(logits && gt && lse && count && gloss && dlogits, E2EP_EINVAL,
               "e2ep_control_ce_bwd: null argument");
  const int R = B * T;
  hipLaunchKernelGGL(k_ctrl_ce_bwd, dim3(cdiv(R, LOSS_THREADS / 64)), dim3(LOSS_THREADS), 0,
                     as_stream(stream), logits, gt, lse, count, gloss, R, T, gt_stride, gt_offset,
                     vocab, pad, dlogits);
  return launch_status("e2ep_control_ce_bwd");
}

size_t e2ep_seg_ce_workspace(int images, int HW) {
  return (size_t)cdiv((long long)images * HW, LOSS_THREADS) * sizeof(float);
}

int e2ep_seg_ce_fwd(const float *logits, const long long *target, const float *weights, int images,
                    int C, int HW, int ignore, float *loss, void *workspace, void *stream) {
  E2EP_REQUIRE(logits && target && weights && loss && workspace, E2EP_EINVAL,
               "e2ep_seg_ce_fwd: null argument");
  E2EP_REQUIRE(images > 0 && C > 0 && HW > 0, E2EP_EINVAL, "e2ep_seg_ce_fwd: bad shape");
  const int nb = cdiv((long long)images * HW, LOSS_THREADS);
  float *part = static_cast<float *>(workspace);
  hipLaunchKernelGGL(k_seg_ce_fwd, dim3(nb), dim3(LOSS_THREADS), 0, as_stream(stream), logits,
                     target, weights, images, C, HW, ignore, part);
  hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(LOSS_THREADS), 0, as_stream(stream), part,
                     (const float *)nullptr, nb, (float)((long long)images * HW), loss,
                     (float *)nullptr);
  return launch_status("e2ep_seg_ce_fwd");
}

int e2ep_seg_ce_bwd(const float *logits, const long long *target, const float *weights,
                    const float *gloss, int images, int C, int HW, int ignore, float *dlogits,
                    void *stream) {
  E2EP_REQUIRE(logits && target && weights && gloss && dlogits, E2EP_EINVAL,
               "e2ep_seg_ce_bwd: null argument");
  hipLaunchKernelGGL(k_seg_ce_bwd, dim3(cdiv((long long)images * HW, LOSS_THREADS)),
                     dim3(LOSS_THREADS), 0, as_stream(stream), logits, target, weights, gloss,
                     images, C, HW, ignore, dlogits);
  return launch_status("e2ep_seg_ce_bwd");
}

size_t e2ep_depth_bce_workspace(int BN, int H, int W, int down) {
  return (size_t)2 * cdiv((long long)BN * (H / down) * (W / down), LOSS_THREADS) * sizeof(float);
}

int e2ep_depth_bce_fwd(const float *prob, const float *gt, int BN, int D, int H, int W, int down,
                       float lo, float step, float *loss, float *den, int *cls, void *workspace,
                       void *stream) {
  return depth_bce_fwd("e2ep_depth_bce_fwd", prob, gt, BN, D, H, W, down, lo, step, loss, den,
                       cls, workspace, stream);
}

int e2ep_depth_bce_fwd_f64(const float *prob, const double *gt, int BN, int D, int H, int W,
                           int down, double lo, double step, float *loss, float *den, int *cls,
                           void *workspace, void *stream) {
  return depth_bce_fwd("e2ep_depth_bce_fwd_f64", prob, gt, BN, D, H, W, down, lo, step, loss, den,
                       cls, workspace, stream);
}

int e2ep_depth_bce_bwd(const float *prob, const int *cls, const float *den, const float *gloss,
                       int BN, int D, int hw, float *dprob, void *stream) {
  E2EP_REQUIRE(prob && cls && den && gloss && dprob, E2EP_EINVAL,
               "e2ep_depth_bce_bwd: null argument");
  hipLaunchKernelGGL(k_depth_bce_bwd, dim3(cdiv((long long)BN * hw, LOSS_THREADS)),
                     dim3(LOSS_THREADS), 0, as_stream(stream), prob, cls, den, gloss, BN, D, hw,
                     dprob);
  return launch_status("e2ep_depth_bce_bwd");
}

}  // extern "C"
