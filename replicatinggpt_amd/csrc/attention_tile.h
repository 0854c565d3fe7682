// charpt attention tile helpers shared by the streaming MFMA kernels (attention_d64.hip) and the
// resident-(b,h) kernels (attention_res.hip): swizzled [rows][64] bf16 LDS images, MFMA fragment
// reads (row and transposed), accumulator packing, keep-bit words.
#pragma once
#include "attention_common.h"

namespace cg {
namespace atile {

typedef __attribute__((address_space(3))) sv4 lds_sv4;

__device__ __forceinline__ fv4 mfma16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

// [rows][64] bf16 images, 128-B rows, 16-B chunk c (0..7).
// ROW: conflict-free for ds_read_b128 row reads; TR: conflict-free for ds_read_b64_tr_b16.
__device__ __forceinline__ int off_row(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ int off_tr(int r, int c) { return r * 128 + ((c ^ (((r >> 1) & 3) << 1)) << 4); }
template <bool TRSWZ>
__device__ __forceinline__ int img_off(int r, int c) {
    return TRSWZ ? off_tr(r, c) : off_row(r, c);
}

// a [64][64] bf16 tile as 2 x 16 B per thread (256 threads)
struct Tile2 {
    uint4 a, b;
};
__device__ __forceinline__ Tile2 tile_load(const bf16_t* base, int64_t ld, int64_t row0, int tid) {
    const int r = tid >> 3, c = tid & 7;
    Tile2 t;
    t.a = *(const uint4*)(base + (row0 + r) * ld + c * 8);
    t.b = *(const uint4*)(base + (row0 + r + 32) * ld + c * 8);
    return t;
}
template <bool TRSWZ>
__device__ __forceinline__ void tile_store(const Tile2& t, char* img, int tid) {
    const int r = tid >> 3, c = tid & 7;
    *(uint4*)(img + img_off<TRSWZ>(r, c)) = t.a;
    *(uint4*)(img + img_off<TRSWZ>(r + 32, c)) = t.b;
}

template <bool TRSWZ>
__device__ __forceinline__ sv8 frag_rows(const char* img, int rb, int s, int lane) {
    return *(const sv8*)(img + img_off<TRSWZ>(rb + (lane & 15), s * 4 + (lane >> 4)));
}

// transposed fragment: X(m = e0 + (lane&15), k = kappa), kappa = 8g + j <-> image row
// rbase + 16*(j>>2) + 4g + (j&3)  (the accumulator-as-operand key order of pack8)
template <bool TRSWZ>
__device__ __forceinline__ sv8 frag_tr(const char* img, int rbase, int e0, int lane) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
    const int chunk = (e0 >> 3) + (p >> 1), byte = 8 * (p & 1);
    const sv4 lo =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_off<TRSWZ>(rbase + 4 * g + qq, chunk) + byte));
    const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_sv4*)(img + img_off<TRSWZ>(rbase + 16 + 4 * g + qq, chunk) + byte));
    return sv8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ sv8 pack8(const fv4& a, const fv4& b) {
    const uint32_t w0 = pack_bf2(a[0], a[1]), w1 = pack_bf2(a[2], a[3]), w2 = pack_bf2(b[0], b[1]),
                   w3 = pack_bf2(b[2], b[3]);
    sv8 r;
    r[0] = (short)(w0 & 0xffff); r[1] = (short)(w0 >> 16);
    r[2] = (short)(w1 & 0xffff); r[3] = (short)(w1 >> 16);
    r[4] = (short)(w2 & 0xffff); r[5] = (short)(w2 >> 16);
    r[6] = (short)(w3 & 0xffff); r[7] = (short)(w3 >> 16);
    return r;
}

struct Words4 {
    uint64_t w[4];
};
__device__ __forceinline__ Words4 lds_words(const char* p) {
    const uint4 x = *(const uint4*)p, y = *(const uint4*)(p + 16);
    Words4 o;
    o.w[0] = ((uint64_t)x.y << 32) | x.x;
    o.w[1] = ((uint64_t)x.w << 32) | x.z;
    o.w[2] = ((uint64_t)y.y << 32) | y.x;
    o.w[3] = ((uint64_t)y.w << 32) | y.z;
    return o;
}

// The keep words are wave-uniform 64-bit lane masks (bit i <-> lane i, k_attn_dropmask's ballots):
// move them to SGPRs once and select with ONE v_cndmask_b32 per element, whose condition operand
// is exactly such a lane mask -- instead of a per-lane 64-bit shift, and, compare and select.
__device__ __forceinline__ float keep_sel(uint64_t word, float v) {
    const uint64_t lanemask = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(word >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)word);
    return __builtin_amdgcn_inverse_ballot_w64(lanemask) ? v : 0.f;
}

constexpr int TILE = 8192;  // [64][64] bf16

// XCD-aware block order for a (row blocks, B*H) grid.  The dispatcher deals linear block ids to
// the 8 XCDs round-robin, and each XCD has its own L2: left alone, the row blocks of one (b,h) --
// which all stream the same K/V (or Q/dO) -- land on 8 different L2s (measured: 35 % L2 hits, the
// C4 forward fetching 4.5x its algorithmic bytes).  The bijective remap gives every XCD a
// contiguous run of logical ids, i.e. whole (b,h) groups; REV runs a group's blocks last-first
// (the causal forward / dQ blocks with the longest key prefix start first).
template <bool REV>
__device__ __forceinline__ void block_coords(int& blk, int& bh) {
    const int nx = (int)gridDim.x, n = nx * (int)gridDim.y;
    const int id = (int)blockIdx.y * nx + (int)blockIdx.x;
    const int q = n >> 3, r = n & 7, xcd = id & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
    bh = lid / nx;
    blk = lid - bh * nx;
    if (REV) blk = nx - 1 - blk;
}

}  // namespace atile
}  // namespace cg
