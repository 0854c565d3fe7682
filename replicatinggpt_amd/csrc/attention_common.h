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
    const uint32_t* mask;      // fast kernels: precomputed keep bits, FWD tiles; NULL = no dropout
    const uint32_t* mask_bwd;  // the same bits, BWD tiles (mask + B*H*mask_tiles(T)*64)
};

// Keep-bit image of the MFMA kernels, generated once per forward (k_attn_dropmask) from the
// canonical Philox stream (same bits as keep_of on element ((b*H + h)*T + q)*T + k) and read by the
// forward, dQ and dK/dV kernels with one coalesced 32-bit load per lane per 64-row tile, prefetched
// a tile ahead (a VGPR: no scalar-load latency in the inner loop, one v_bfe_i32 + v_and per use).
// T % 64 == 0; NB = T/32 blocks of 32, NP = T/64 tiles of 64.  Accumulator register r of 32x32
// sub-block s (32x32x16 MFMA layout: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
// =: row(r, l)) is bit f(s, r) = 8 s + (r >> 1) + 16 (r & 1) of a FWD word -- the two registers the
// forward packs into one bf16 pair at bits j and j + 16, so one shift + v_perm_b32 makes the pair's
// mask -- and bit 16 s + r of a BWD word:
//   FWD (forward, dQ: swapped products, lane = query), tile (qb, kt) for kt <= qb/2:
//        bit f(s, r) of lane l = keep(q = 32 qb + (l & 31), k = 64 kt + 32 s + row(r, l))
//   BWD (dK/dV: lane = key), tile (kb, qt) for qt >= kb/2:
//        bit 16 s + r of lane l = keep(q = 64 qt + 32 s + row(r, l), k = 32 kb + (l & 31))
// Sub-blocks wholly above the diagonal are 0; diagonal sub-blocks are stored whole (the kernels
// apply the causal mask themselves).  Per (b*H + h): mask_tiles(T) tiles of 64 words each, FWD
// row-major over qb, BWD column-major over kb.
__host__ __device__ __forceinline__ int64_t mask_tiles(int64_t T) {
    const int64_t nb = T / 32;
    return nb + (nb - 1) * (nb - 1) / 4;
}
__device__ __forceinline__ int64_t mask_fwd_tile(int qb, int kt) { return qb + (qb ? (qb - 1) * (qb - 1) / 4 : 0) + kt; }
__device__ __forceinline__ int64_t mask_bwd_tile(int kb, int qt, int np) {
    return (int64_t)kb * np - (kb ? (kb - 1) * (kb - 1) / 4 : 0) + qt - kb / 2;
}
// all-ones where bit `bit` of a lane's mask word is set (one v_bfe_i32)
__device__ __forceinline__ uint32_t keep_lanes(uint32_t w, int bit) { return (uint32_t)((int32_t)(w << (31 - bit)) >> 31); }

namespace attn {
// bf16 MFMA kernels, head_size 64, T % 64 == 0 (attention_d64.hip)
void launch_fwd_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st);
// also computes delta = rowsum(dO * O) for its queries and writes it (read by launch_dkdv_d64 next)
void launch_dq_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                   const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, float* delta,
                   bf16_t* dq, int64_t lddq, float scale, const DropArgs& d, hipStream_t st);
// dQ then dK/dV (T <= 256: one merged launch, bwd_merged(T)); delta_ready (merged launch only):
// `delta` already holds rowsum(dO * O) and is read, not computed
bool bwd_merged(int64_t T);
void launch_bwd_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, float* delta,
                    bool delta_ready, bf16_t* dq, int64_t lddq, bf16_t* dk, bf16_t* dv, int64_t lddkv, float scale, const DropArgs& d,
                    hipStream_t st);
void launch_dkdv_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                     const bf16_t* dout, int64_t ldd, const float* lse, const float* delta, bf16_t* dk, bf16_t* dv,
                     int64_t lddkv, float scale, const DropArgs& d, hipStream_t st);
}  // namespace attn
extern int g_attn_variant;

}  // namespace cg
