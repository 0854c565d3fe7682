// charpt attention internals shared by attention_generic.hip (generic kernels, dropout mask,
// C ABI) and attention_d64.hip (bf16 MFMA kernels for head_size 64).
#pragma once
#include "common.h"

namespace cg {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct DropArgs {
    uint32_t thr;
    float dscale;
    uint64_t seed;
    const uint64_t* rng_call;
    int site;
    const uint64_t* mask;  // fast kernels: precomputed keep bits (k_attn_dropmask), NULL = no dropout
};

// Keep-bit image for the MFMA kernels, per (b*H + h) and 16x16 (query tile, key tile):
// 4 uint64 words, bit l of word w = keep(query = 16*qt + (l & 15), key = 16*kt + 4*(l >> 4) + w).
// Generated once per forward from the canonical Philox stream (same bits as keep_elem), read by
// the forward, dQ and dK/dV kernels instead of re-running Philox in their inner loops.
__device__ __forceinline__ const uint64_t* mask_tile(const uint64_t* mask, int bh, int NT, int qt, int kt) {
    return mask + ((((int64_t)bh * NT + qt) * NT + kt) << 2);
}


namespace attn {
// bf16 MFMA kernels, head_size 64, T % 64 == 0 (attention_d64.hip)
void launch_fwd_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st);
// also computes delta = rowsum(dO * O) for its queries and writes it (read by launch_dkdv_d64 next)
void launch_dq_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                   const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, float* delta,
                   bf16_t* dq, int64_t lddq, float scale, const DropArgs& d, hipStream_t st);
void launch_dkdv_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                     const bf16_t* dout, int64_t ldd, const float* lse, const float* delta, bf16_t* dk, bf16_t* dv,
                     int64_t lddkv, float scale, const DropArgs& d, hipStream_t st);
// whole-(b, h)-resident kernels for T % 64 == 0, T <= 256 (attention_res.hip), opt-in with
// attn_variant bit 8
bool res_ok(int64_t T);
void launch_fwd_res(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st);
void launch_bwd_res(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, bf16_t* dq,
                    bf16_t* dk, bf16_t* dv, int64_t lddqkv, float scale, const DropArgs& d, hipStream_t st);
}  // namespace attn
extern int g_attn_variant;

}  // namespace cg
