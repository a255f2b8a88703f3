// adam.hip — the training step's optimizer update over every parameter in
// one launch (torch.optim.Adam semantics, the optimizer RecBole's trainer
// builds for RecBLR: run.py / RecBole's Trainer, learner 'adam').
//
// torch's fused Adam walks its tensor lists in 64K-element chunks, one
// workgroup each: the encoder's ~2.1 M parameters make a few dozen
// workgroups on 256 CUs (48 us per step at ~1 TB/s, profiles/r03_v12_
// kernel_stats.csv).  Here every parameter is a job of a job table; each
// job gets blocks in proportion to its size (float4 per thread, a tail of
// n % 4 scalars), so the launch spans the chip.  Per element:
//   g' = g + wd p;  m += (1 - b1)(g' - m);  v = b2 v + (1 - b2) g'^2
//   p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)
// with bc1 = 1 - b1^t, bc2 = 1 - b2^t computed on the host for step t.
#include "common.h"

#include <cmath>

namespace rb {
namespace {

constexpr int kAdamThreads = 256;
constexpr int kAdamPerBlock = kAdamThreads * 4;   // float4 per thread

struct AdamJobs {
  float* p[RB_MAX_ADAM_JOBS];
  const float* g[RB_MAX_ADAM_JOBS];
  float* m[RB_MAX_ADAM_JOBS];
  float* v[RB_MAX_ADAM_JOBS];
  int64_t n[RB_MAX_ADAM_JOBS];
  int bstart[RB_MAX_ADAM_JOBS + 1];
  int njobs;
};

struct AdamHyper {
  float step_size, one_m_b1, b2, one_m_b2, eps, wd, sqrt_bc2;
};

// torch's single-tensor order: m.lerp_(g, 1 - b1), v.mul_(b2).addcmul_(g, g,
// 1 - b2), denom = sqrt(v) / sqrt(bc2) + eps, p.addcdiv_(m, denom, -lr / bc1)
__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamHyper& h) {
  if (h.wd != 0.0f) g = g + h.wd * p;
  m = m + h.one_m_b1 * (g - m);
  v = v * h.b2 + h.one_m_b2 * g * g;
  const float denom = sqrtf(v) / h.sqrt_bc2 + h.eps;
  p = p + h.step_size * (m / denom);
}

__global__ void __launch_bounds__(kAdamThreads) k_adam(const AdamJobs jobs, const AdamHyper h) {
  int j = 0;
  while (j + 1 < jobs.njobs && (int)blockIdx.x >= jobs.bstart[j + 1]) ++j;   // <= 48 jobs
  const int64_t n = jobs.n[j];
  const int64_t base = (int64_t)((int)blockIdx.x - jobs.bstart[j]) * kAdamPerBlock;
  const int64_t e = base + 4 * (int64_t)threadIdx.x;
  float* P = jobs.p[j];
  const float* G = jobs.g[j];
  float* Mm = jobs.m[j];
  float* V = jobs.v[j];
  if (e + 4 <= n) {
    float4 p = *reinterpret_cast<const float4*>(P + e);
    const float4 g = *reinterpret_cast<const float4*>(G + e);
    float4 m = *reinterpret_cast<const float4*>(Mm + e);
    float4 v = *reinterpret_cast<const float4*>(V + e);
    adam_one(p.x, g.x, m.x, v.x, h);
    adam_one(p.y, g.y, m.y, v.y, h);
    adam_one(p.z, g.z, m.z, v.z, h);
    adam_one(p.w, g.w, m.w, v.w, h);
    *reinterpret_cast<float4*>(P + e) = p;
    *reinterpret_cast<float4*>(Mm + e) = m;
    *reinterpret_cast<float4*>(V + e) = v;
  } else {
    for (int64_t k = e; k < n && k < e + 4; ++k) {
      float p = P[k], m = Mm[k], v = V[k];
      adam_one(p, G[k], m, v, h);
      P[k] = p;
      Mm[k] = m;
      V[k] = v;
    }
  }
}

}  // namespace

int launch_adam(const rb_adam_job* jobs, int n, double lr, double beta1, double beta2, double eps,
                double weight_decay, double bc1, double bc2, hipStream_t st) {
  AdamJobs aj{};
  aj.njobs = n;
  int blocks = 0;
  for (int j = 0; j < n; ++j) {
    aj.p[j] = jobs[j].param;
    aj.g[j] = jobs[j].grad;
    aj.m[j] = jobs[j].exp_avg;
    aj.v[j] = jobs[j].exp_avg_sq;
    aj.n[j] = jobs[j].n;
    aj.bstart[j] = blocks;
    blocks += (int)((jobs[j].n + kAdamPerBlock - 1) / kAdamPerBlock);
  }
  aj.bstart[n] = blocks;
  // formed in double, rounded to fp32 once (torch passes its Python-float
  // scalars to the kernels the same way)
  const AdamHyper h{(float)(-lr / bc1), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                    (float)eps, (float)weight_decay, (float)std::sqrt(bc2)};
  k_adam<<<(unsigned)blocks, kAdamThreads, 0, st>>>(aj, h);
  return launch_status("rb_adam_step");
}

}  // namespace rb
