// Fused Adam (torch.optim.Adam semantics, L2 weight decay, no amsgrad) over ONE flat fp32
// parameter buffer — the optimizer the reference configures at trainer/pl_trainer.py:116-121.
//
// Parameters, exp_avg and exp_avg_sq are flat, every tensor 16-byte aligned inside them; the
// gradients are either the per-tensor buffers autograd produced (a device table of pointers,
// so no accumulate-into-flat copy is needed) or one flat buffer (data-parallel: gathered and
// all-reduced).  One launch updates all ~28M weights: 7 x 4 bytes per weight of HBM traffic.
#include "common.h"

namespace e2ep {

// torch.optim.Adam evaluates its scalars in double on the host and hands them to fp32
// kernels: beta**step and lr/bc1 in double, (1 - beta) in double then rounded to fp32.
// The learning rate is read from device memory (a double written by the host when an LR
// scheduler changes it), so a captured step follows CosineAnnealingLR under graph replay.
struct AdamHyper {
  double beta1, beta2;
  float b1f, b2f, w1, w2, eps, wd, grad_scale;
};

constexpr int ADAM_THREADS = 256;
constexpr int ADAM_VEC = 4;
constexpr int ADAM_ITERS = 4;

__global__ void k_adam_count(float *step) { step[0] += 1.f; }

// chunk table row: {tensor, start element within tensor, length, unused}
__global__ void __launch_bounds__(ADAM_THREADS)
    k_adam(const int4 *__restrict__ chunks, const long long *__restrict__ offs,
           const long long *__restrict__ gptrs, const float *__restrict__ gflat,
           float *__restrict__ p, float *__restrict__ m, float *__restrict__ v,
           const float *__restrict__ step, const double *__restrict__ lr, AdamHyper h,
           int *__restrict__ stepped) {
  const int4 c = chunks[blockIdx.x];
  const long long off = offs[c.x] + c.y;
  // a parameter without a gradient this step is not stepped (as torch.optim.Adam); on the
  // flat (all-reduced) path the table still says which parameters had one, so the result
  // does not depend on the world size
  const float *gt = gptrs ? reinterpret_cast<const float *>(gptrs[c.x]) : nullptr;
  if (gptrs && gt == nullptr) return;
  // per-tensor "stepped at least once" flag (torch.optim.Adam keeps state only for those)
  if (stepped && c.y == 0 && threadIdx.x == 0) stepped[c.x] = 1;
  const float *g = gflat ? gflat + off : gt + c.y;
  // torch: bias_correction = 1 - beta**step (python double), step_size = lr / bc1,
  // denom = sqrt(v) / sqrt(bc2) + eps, p -= step_size * m / denom
  const double t = (double)step[0];
  const double bc1 = 1.0 - pow(h.beta1, t);
  const double bc2 = 1.0 - pow(h.beta2, t);
  const float step_size = (float)(lr[0] / bc1);
  const float bc2s = (float)sqrt(bc2);
  const float w1 = h.w1, w2 = h.w2;
  float *pp = p + off, *mp = m + off, *vp = v + off;
  const bool vec = (reinterpret_cast<uintptr_t>(g) & 15) == 0;  // wave-uniform
  auto upd = [&](float &pv, float &mv, float &vv, float gv) {
    gv = gv * h.grad_scale;
    gv = gv + h.wd * pv;
    mv = mv + w1 * (gv - mv);  // exp_avg.lerp_(grad, 1 - beta1)
    vv = vv * h.b2f + w2 * gv * gv;
    const float den = sqrtf(vv) / bc2s + h.eps;
    pv = pv - step_size * (mv / den);
  };
  if (vec) {
#pragma unroll
    for (int it = 0; it < ADAM_ITERS; ++it) {
      const int i = (it * ADAM_THREADS + threadIdx.x) * ADAM_VEC;
      if (i >= c.z) break;
      if (i + ADAM_VEC <= c.z) {
        float4 P = *reinterpret_cast<const float4 *>(pp + i);
        float4 M = *reinterpret_cast<const float4 *>(mp + i);
        float4 V = *reinterpret_cast<const float4 *>(vp + i);
        const float4 G = *reinterpret_cast<const float4 *>(g + i);
        upd(P.x, M.x, V.x, G.x);
        upd(P.y, M.y, V.y, G.y);
        upd(P.z, M.z, V.z, G.z);
        upd(P.w, M.w, V.w, G.w);
        *reinterpret_cast<float4 *>(pp + i) = P;
        *reinterpret_cast<float4 *>(mp + i) = M;
        *reinterpret_cast<float4 *>(vp + i) = V;
      } else {
        for (int j = i; j < c.z; ++j) upd(pp[j], mp[j], vp[j], g[j]);
      }
    }
  } else {
    for (int j = threadIdx.x; j < c.z; j += ADAM_THREADS) upd(pp[j], mp[j], vp[j], g[j]);
  }
}

// gather per-tensor gradients into the flat (aligned, zero-padded) buffer for all-reduce
__global__ void __launch_bounds__(ADAM_THREADS)
    k_grad_gather(const int4 *__restrict__ chunks, const long long *__restrict__ offs,
                  const long long *__restrict__ gptrs, float *__restrict__ flat) {
  const int4 c = chunks[blockIdx.x];
  const float *g = reinterpret_cast<const float *>(gptrs[c.x]);
  float *o = flat + offs[c.x] + c.y;
  for (int j = threadIdx.x; j < c.z; j += ADAM_THREADS) o[j] = g ? g[c.y + j] : 0.f;
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_adam_chunk_elems(void) { return ADAM_THREADS * ADAM_VEC * ADAM_ITERS; }

int e2ep_adam_step(const int *chunks, int n_chunks, const long long *offsets,
                   const long long *grad_ptrs, const float *grad_flat, float *param, float *exp_avg,
                   float *exp_avg_sq, float *step, const double *lr, double beta1, double beta2,
                   double eps, double weight_decay, float grad_scale, int *stepped,
                   void *stream) {
  E2EP_REQUIRE(n_chunks > 0 && chunks && offsets && param && exp_avg && exp_avg_sq && step && lr,
               E2EP_EINVAL, "e2ep_adam_step: null argument");
  E2EP_REQUIRE(grad_ptrs || grad_flat, E2EP_EINVAL, "e2ep_adam_step: no gradients");
  AdamHyper h{beta1, beta2, (float)beta1, (float)beta2, (float)(1.0 - beta1),
              (float)(1.0 - beta2), (float)eps, (float)weight_decay, grad_scale};
  hipLaunchKernelGGL(k_adam_count, dim3(1), dim3(1), 0, as_stream(stream), step);
  hipLaunchKernelGGL(k_adam, dim3(n_chunks), dim3(ADAM_THREADS), 0, as_stream(stream),
                     reinterpret_cast<const int4 *>(chunks), offsets, grad_ptrs, grad_flat, param,
                     exp_avg, exp_avg_sq, step, lr, h, stepped);
  return launch_status("e2ep_adam_step");
}

int e2ep_grad_gather(const int *chunks, int n_chunks, const long long *offsets,
                     const long long *grad_ptrs, float *grad_flat, void *stream) {
  E2EP_REQUIRE(n_chunks > 0 && chunks && offsets && grad_ptrs && grad_flat, E2EP_EINVAL,
               "e2ep_grad_gather: null argument");
  hipLaunchKernelGGL(k_grad_gather, dim3(n_chunks), dim3(ADAM_THREADS), 0, as_stream(stream),
                     reinterpret_cast<const int4 *>(chunks), offsets, grad_ptrs, grad_flat);
  return launch_status("e2ep_grad_gather");
}

}  // extern "C"
