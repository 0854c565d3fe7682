// charpt: the LayerNorm forward's row body (nn.LayerNorm, GPT1.py:159-160,173), shared by
// layernorm.hip's k_ln_fwd and the LayerNorm + attention keep-bit launch (attention_generic.hip
// k_ln_fwd_dropmask).
#pragma once
#include "common.h"

namespace {
using namespace cg;

template <int VEC>
struct VecIO;
template <>
struct VecIO<1> {
    static __device__ __forceinline__ void ld(const float* p, float* v) { v[0] = *p; }
    static __device__ __forceinline__ void st(float* p, const float* v) { *p = v[0]; }
    static __device__ __forceinline__ void st(bf16_t* p, const float* v) { *p = f2bf(v[0]); }
};
template <>
struct VecIO<2> {
    static __device__ __forceinline__ void ld(const float* p, float* v) {
        float2 t = *(const float2*)p;
        v[0] = t.x;
        v[1] = t.y;
    }
    static __device__ __forceinline__ void st(float* p, const float* v) { *(float2*)p = make_float2(v[0], v[1]); }
    static __device__ __forceinline__ void st(bf16_t* p, const float* v) { *(uint32_t*)p = pack_bf2(v[0], v[1]); }
};
template <>
struct VecIO<4> {
    static __device__ __forceinline__ void ld(const float* p, float* v) {
        float4 t = *(const float4*)p;
        v[0] = t.x;
        v[1] = t.y;
        v[2] = t.z;
        v[3] = t.w;
    }
    static __device__ __forceinline__ void st(float* p, const float* v) {
        *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    }
    static __device__ __forceinline__ void st(bf16_t* p, const float* v) {
        *(uint2*)p = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
};

// One row in the lane layout below (lane l holds elements (j*64 + l)*VEC + q): mean, variance (two
// passes over the registers, wave_sum_dpp), rstd and the affine output.  Shared by ln_fwd_rows and
// the residual GEMM + LayerNorm epilogue (gemm_ln.hip), so both give the same bits.
template <int VEC, int NJ, typename TY, bool FULL>
__device__ __forceinline__ void ln_fwd_row(const float (&v)[NJ][VEC], const float (&wv)[NJ][VEC],
                                           const float (&bv)[NJ][VEC], int C, float invC, float eps, int lane,
                                           TY* __restrict__ yr, float& mu_out, float& rs_out) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < VEC; ++q) s += v[j][q];
    const float mu = wave_sum_dpp(s) * invC;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int e = (j * 64 + lane) * VEC;
        if (FULL || e < C) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                const float d = v[j][q] - mu;
                ss += d * d;
            }
        }
    }
    const float var = wave_sum_dpp(ss) * invC;
    const float rs = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int e = (j * 64 + lane) * VEC;
        if (FULL || e < C) {
            float o[VEC];
#pragma unroll
            for (int q = 0; q < VEC; ++q) o[q] = (v[j][q] - mu) * rs * wv[j][q] + bv[j][q];
            VecIO<VEC>::st(yr + e, o);
        }
    }
    mu_out = mu;
    rs_out = rs;
}

// One wave per row, RPW rows per wave: every load of the wave's rows is issued before the first
// reduction, and gamma/beta are held in registers for all of them (they were re-read after each
// row's reductions, on the critical path).
// Block `bid` of `nblk` (256 threads): rows bid*4 + wave, then a stride of nblk*4 rows.
template <int VEC, int NJ, typename TY, int RPW, bool FULL = false>
__device__ __forceinline__ void ln_fwd_rows(const float* __restrict__ x, const float* __restrict__ w,
                                            const float* __restrict__ b, TY* __restrict__ y,
                                            float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                            int64_t rows, int C, float eps, int bid, int nblk) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const float invC = 1.0f / (float)C;
    float wv[NJ][VEC], bv[NJ][VEC];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int e = (j * 64 + lane) * VEC;
        if (FULL || e < C) {
            VecIO<VEC>::ld(w + e, wv[j]);
            VecIO<VEC>::ld(b + e, bv[j]);
        }
    }
    const int64_t stride = (int64_t)nblk * 4;
    for (int64_t r0 = (int64_t)bid * 4 + wave; r0 < rows; r0 += stride * RPW) {
        float v[RPW][NJ][VEC];
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int64_t r = r0 + i * stride < rows ? r0 + i * stride : r0;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int e = (j * 64 + lane) * VEC;
                if (FULL || e < C) {
                    VecIO<VEC>::ld(x + r * C + e, v[i][j]);
                } else {
#pragma unroll
                    for (int q = 0; q < VEC; ++q) v[i][j][q] = 0.f;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int64_t r = r0 + i * stride;
            if (r >= rows) break;
            float mu, rs;
            ln_fwd_row<VEC, NJ, TY, FULL>(v[i], wv, bv, C, invC, eps, lane, y + r * C, mu, rs);
            if (lane == 0) {
                mean_out[r] = mu;
                rstd_out[r] = rs;
            }
        }
    }
}

}  // namespace
