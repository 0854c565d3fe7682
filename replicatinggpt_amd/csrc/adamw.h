// charpt: AdamW element arithmetic (torch.optim.AdamW, GPT1.py:218,233), shared by the AdamW kernels
// (ce_adamw.hip) and the AdamW jobs the persistent GEMM's free blocks run (gemm_common.h red_tail).
#pragma once
#include <math.h>

#include "common.h"

namespace cg {
// The fp32 arithmetic of torch/optim/adam.py _single_tensor_adam (decoupled decay) as torch's CPU
// kernels round it:
//   p *= 1 - lr*wd ; m = fma(1-b1, g - m, m) [lerp, w < 0.5: the vectorised CPU lerp fuses] ;
//   v = fma((1-b2)*g, g, v*b2) [mul_ + addcmul_, fused] ; denom = sqrt(v)/sqrt(bc2) + eps ;
//   p += (-lr/bc1)*m / denom
// Every rounding is explicit: contraction is OFF in this function and the two fused steps are
// __builtin_fmaf.  (Round 4's form relied on __fmul_rn / __fadd_rn to keep the compiler from
// contracting; it does not -- hipcc's default -ffp-contract=fast fused mul/add pairs, and WHICH pairs
// depended on the surrounding code: the GEMM-hosted one-chunk loop happened to fuse like k_adamw, a
// four-chunks-in-flight loop did not, and rounded ~1 ulp differently (profiles/r5_early_adamw_cause.txt);
// and __fsqrt_rn was not a correctly rounded square root.)
struct AdamScalars {
    float decay, w1, b2, omb2, eps, neg_step, bc2_sqrt;
};

__device__ __forceinline__ float adam_one(float p, float g, float& m, float& v, const AdamScalars& s) {
#pragma clang fp contract(off)
    p = p * s.decay;
    m = __builtin_fmaf(s.w1, g - m, m);
    v = __builtin_fmaf(s.omb2 * g, g, v * s.b2);
    // __builtin_sqrtf is the correctly rounded sequence (v_sqrt_f32 + an fma-residual ulp fix);
    // __fsqrt_rn lowers to the bare 1-ulp v_sqrt_f32 on gfx950 / ROCm 7.2
    const float denom = __fdiv_rn(__builtin_sqrtf(v), s.bc2_sqrt) + s.eps;
    return p + __fdiv_rn(s.neg_step * m, denom);
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
