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
    const uint64_t* mask;      // fast kernels: precomputed keep bits, FWD orientation; NULL = no dropout
    const uint64_t* mask_bwd;  // the same bits, BWD orientation (mask + B*H*mask_tri_blocks(T)*16)
};

// Keep-bit image of the MFMA kernels, generated once per forward (k_attn_dropmask) from the
// canonical Philox stream (same bits as keep_of on element ((b*H + h)*T + q)*T + k) and read by the
// forward, dQ and dK/dV kernels.  Per (b*H + h) and per 32x32 block (query block qb, key block
// kb <= qb, lower-triangle order), 16 uint64 words in each of two orientations -- exactly the
// 32x32x16 MFMA accumulator layout (column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
// for register r), so word r is the lane mask of accumulator register r (one v_cndmask each):
//   FWD (forward, dQ: swapped products, lane = query):
//        bit l of word r = keep(q = 32 qb + (l & 31), k = 32 kb + (r & 3) + 8 (r >> 2) + 4 (l >> 5))
//   BWD (dK/dV: lane = key):
//        bit l of word r = keep(q = 32 qb + (r & 3) + 8 (r >> 2) + 4 (l >> 5), k = 32 kb + (l & 31))
__host__ __device__ __forceinline__ int64_t mask_tri_blocks(int64_t T) {
    const int64_t n = T / 32;
    return n * (n + 1) / 2;
}
__device__ __forceinline__ const uint64_t* mask_block(const uint64_t* mask, int64_t bh, int64_t ntri, int qb, int kb) {
    return mask + (bh * ntri + (int64_t)qb * (qb + 1) / 2 + kb) * 16;
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
}  // namespace attn
extern int g_attn_variant;

}  // namespace cg
