// The element-wise optimizer updates shared by the flat-shard apply kernels (optim.hip) and the
// parameter-server data plane (ps_plane.hip): 4 elements per call, fp32 math, TF / torch.optim
// semantics (SGD with (Nesterov) momentum and L2 weight decay; Adam / AdamW with bias correction).
#pragma once
#include "common.h"

namespace tony {

// v = mu v + (g gs + wd w);  w -= lr (nesterov ? g' + mu v : v)
__device__ __forceinline__ void sgd_update4(float* wf, float* vf, const float* gf, float lr, float mu, float wd,
                                            float gs, bool nesterov) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gk = fmaf(gf[k], gs, wd * wf[k]);
    vf[k] = fmaf(mu, vf[k], gk);
    const float upd = nesterov ? fmaf(mu, vf[k], gk) : vf[k];
    wf[k] = fmaf(-lr, upd, wf[k]);
  }
}

// m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  w -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
// (decoupled: w *= 1 - lr wd first, AdamW; else g += wd w)
__device__ __forceinline__ void adam_update4(float* wf, float* mf, float* vf, const float* gf, float lr, float b1,
                                             float b2, float eps, float wd, float gs, float step_size,
                                             float inv_sqrt_bc2, bool decoupled) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float gk = gf[k] * gs;
    if (decoupled)
      wf[k] *= (1.f - lr * wd);
    else
      gk = fmaf(wd, wf[k], gk);
    mf[k] = fmaf(b1, mf[k], (1.f - b1) * gk);
    vf[k] = fmaf(b2, vf[k], (1.f - b2) * gk * gk);
    const float denom = sqrtf(vf[k]) * inv_sqrt_bc2 + eps;
    wf[k] = fmaf(-step_size, mf[k] / denom, wf[k]);
  }
}

}  // namespace tony
