// charpt: AdamW element arithmetic (torch.optim.AdamW, GPT1.py:218,233), shared by the AdamW kernels
// (ce_adamw.hip) and the AdamW jobs the persistent GEMM's free blocks run (gemm_common.h red_tail).
#pragma once
#include <math.h>

#include "common.h"

namespace cg {
// Same fp32 operation order as torch/optim/adam.py _single_tensor_adam (decoupled decay):
//   p *= 1 - lr*wd ; m = m + (1-b1)*(g - m) [lerp, w<0.5] ; v = v*b2 + (1-b2)*g*g ;
//   denom = sqrt(v)/sqrt(bc2) + eps ; p += (-lr/bc1)*m / denom
// Explicit _rn intrinsics keep the compiler from contracting into FMAs.
struct AdamScalars {
    float decay, w1, b2, omb2, eps, neg_step, bc2_sqrt;
};

__device__ __forceinline__ float adam_one(float p, float g, float& m, float& v, const AdamScalars& s) {
    p = __fmul_rn(p, s.decay);
    m = __fadd_rn(m, __fmul_rn(s.w1, __fsub_rn(g, m)));
    v = __fadd_rn(__fmul_rn(v, s.b2), __fmul_rn(__fmul_rn(s.omb2, g), g));
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), s.bc2_sqrt), s.eps);
    return __fadd_rn(p, __fdiv_rn(__fmul_rn(s.neg_step, m), denom));
}


__device__ __forceinline__ AdamScalars adam_scalars(double lr, double beta1, double beta2, double eps, double wd,
                                                    const int64_t* step_ptr) {
    const double t = (double)*step_ptr;
    AdamScalars s;
    s.decay = (float)(1.0 - lr * wd);
    s.w1 = (float)(1.0 - beta1);
    s.b2 = (float)beta2;
    s.omb2 = (float)(1.0 - beta2);
    s.eps = (float)eps;
    const double bc1 = 1.0 - pow(beta1, t);
    const double bc2 = 1.0 - pow(beta2, t);
    s.neg_step = (float)(-(lr / bc1));
    s.bc2_sqrt = (float)sqrt(bc2);
    return s;
}
}  // namespace cg
