// charpt: the head_size-64 attention kernels (attention_d64.hip: the launchers) -- shared by the
// product translation unit and the A/B-only one (ab/attention_ab.hip, `make ab`).  See the
// structure notes below.
#pragma once
// charpt: bf16 MFMA causal attention for head_size 64 (the C2/C4 perf path of Head.forward x
// n_head, GPT1.py:109-123,134-135) -- forward, dQ and dK/dV kernels on v_mfma_f32_32x32x16_bf16.
//
// Structure (CDNA4: 64-wide waves, 32x32 MFMA tiles):
//  * forward / dQ: a block of 4 waves owns 256 queries; each wave two 32-query groups, g and 7-g
//    of the block, so every wave walks the same number of causal key tiles (1+4, 1+4, 2+3, 2+3 at
//    the first block: the causal triangle is balanced inside the block).  Products are swapped --
//    S^T = K Q^T, dP^T = V dO^T -- so the query is the accumulator column (lane & 31): softmax
//    statistics are lane-local plus one lane^32 exchange, and the accumulator, packed to bf16, is
//    directly the B operand of O^T = V^T P^T / dQ^T = K^T dS^T (V / K read transposed).
//  * dK/dV: a block of 4 waves owns 128 keys (32 per wave); S = Q K^T, dP = dO V^T with the key
//    as the column, Z = dropped P and dS feed dV^T = dO^T Z and dK^T = Q^T dS as B operands.
//  * 64-row K/V (or Q/dO) tiles, register-staged into a double-buffered LDS ring (next tile's
//    global loads issued before the current tile's MFMAs, written after them, one barrier per
//    tile).  One XOR swizzle serves both the row reads (ds_read_b128) and the transposed reads
//    (ds_read_b64_tr_b16) conflict-free.
//  * Forward: lazy rescaling -- the running max is only moved (and O, l rescaled) when a tile's max
//    exceeds it by 2^8, so the O-wide multiply is off the common path; probabilities stay <= 256.
//  * Dropout keep bits (k_attn_dropmask, attention_common.h): one 32-bit word per lane per 64-row
//    tile, loaded a tile ahead with the K/V (or Q/dO) staging loads and applied as v_bfe_i32 +
//    v_and_b32 per element; the 1/(1-p) is applied once at the end.
#include <float.h>
#include <type_traits>

#include "attention_common.h"

namespace cg {
extern int g_attn_variant;
extern int g_attn_bwd_lpt;

#ifdef CG_ATTN_STAMPS
// Diagnostic build only (make attnstamps; tools/attn_stamps.py): per workgroup of the resident
// kernels, {start, operands landed (the prologue's wait), end} in s_memrealtime ticks (100 MHz) and
// {kind << 48 | XCC << 40 | HW_ID} -- written by lane 0 of wave 0 with a plain vector store into a
// buffer no other code reads.  Never in the product library.
constexpr int ATTN_STAMP_WG = 4096;
__device__ unsigned long long g_attn_stamps[ATTN_STAMP_WG * 4];
extern "C" int cg_debug_attn_stamps(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), (size_t)n * 4 * sizeof(unsigned long long)) ==
                   hipSuccess ? 0 : 1;
}
__device__ __forceinline__ void attn_stamp(int slot, unsigned long long v) {
    const int wg = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    if (threadIdx.x == 0 && wg < ATTN_STAMP_WG) {
        volatile unsigned long long* p = g_attn_stamps + 4 * wg + slot + (threadIdx.x & 63);
        *p = v;
    }
}
__device__ __forceinline__ unsigned long long attn_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ unsigned long long attn_where(int kind) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return ((unsigned long long)kind << 48) | ((unsigned long long)(xcc & 0xff) << 40) | hw;
}
#define ATTN_STAMP(slot, v) attn_stamp(slot, v)
#else
#define ATTN_STAMP(slot, v)
#endif

namespace {

typedef float fv16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) sv4 lds_sv4;

constexpr int TILE = 8192;             // [64 rows][64 bf16] image
constexpr float RESCALE_THR = 8.0f;    // log2 units (forward lazy rescale)

__device__ __forceinline__ fv16 mfma32(sv8 a, sv8 b, fv16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

// Forward row sums on the matrix core.  A 32x32x16 B-operand fragment of P^T (lane l: keys 8 (l>>5) + j,
// query l & 31) read as the B operand of v_mfma_f32_16x16x32_bf16 (lane l: k' = 8 (l>>4) + j, column
// l & 15) mixes two queries per column; the A operand below is 1 exactly where the k' group's query
// half ((k'>>3) & 1 = (l>>4) & 1 of the source lane) equals the output row's ((m>>2) & 1), so output
// row m, column n sums the 16 keys of query n + 16 ((m>>2) & 1), and lane l's four accumulator
// registers (rows 4 (l>>4) + i) all hold the running sum of query l & 31.  One 16-cycle MFMA per
// 16 keys replaces 16 v_add_f32 per lane (the sum is over the bf16-rounded P that O^T also sums).
typedef float fv4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ fv4 mfma16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}
__device__ __forceinline__ sv8 rowsum_ones(int lane) {
    const short o = (((lane >> 4) ^ (lane >> 2)) & 1) ? (short)0 : (short)0x3F80;   // bf16 1.0
    return sv8{o, o, o, o, o, o, o, o};
}

// [64][64] bf16 image, 128-B rows; 16-B chunk c of row r at r*128 + ((c ^ X(r)) << 4) with
// X(r) = ((r>>1)&1)<<2 | (r>>2)&3.  Row reads of the 32x32x16 operand (16-lane groups of
// ds_read_b128 over rows {0-3,12-15,20-27} / {4-11,16-19,28-31}) land on 16 distinct 16-B slots;
// transposed reads (a 32-lane half reads rows r0..r0+3, 64 bytes each) on 64 distinct banks.
__device__ __forceinline__ int aoff(int r, int c) { return r * 128 + ((c ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))) << 4); }

// A operand, tile rows rb..rb+31: lane l holds X(rb + (l&31), 16 ks + 8 (l>>5) + j), j = 0..7
__device__ __forceinline__ sv8 frag_row(const char* img, int rb, int ks, int lane) {
    return *(const sv8*)(img + aoff(rb + (lane & 31), 2 * ks + (lane >> 5)));
}

// A operand = tile^T, tile columns cb..cb+31 as rows: lane l, element j <-> tile row
// rb + 16 ks + 8 (j>>2) + 4 (l>>5) + (j&3), column cb + (l&31) -- the k order of an accumulator
// packed as the B operand (pack16 below).  Two ds_read_b64_tr_b16: each 16-lane group reads a
// 4-row x 16-column block, lane 4q+p addressing row q, columns 4p..4p+3.
__device__ __forceinline__ sv8 frag_tr(const char* img, int rb, int ks, int cb, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int col = cb + 16 * (g & 1) + 4 * p;
    const int r0 = rb + 16 * ks + 4 * (g >> 1) + q;
    const int chunk = col >> 3, byte = (col & 7) * 2;
    const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + aoff(r0, chunk) + byte));
    const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + aoff(r0 + 8, chunk) + byte));
    return sv8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// FWD keep-word bit of accumulator register r of 32-key subtile kt (attention_common.h: the two
// registers packed into one bf16 pair sit at bits j and j + 16, j = 8 kt + (r >> 1))
__device__ __forceinline__ constexpr int fwd_bit(int kt, int r) { return 8 * kt + (r >> 1) + 16 * (r & 1); }

// accumulator registers 8s..8s+7 -> bf16 B-operand fragment of k-step s
__device__ __forceinline__ sv8 pack16(const fv16& x, int s) {
    const uint32_t w0 = pack_bf2(x[8 * s + 0], x[8 * s + 1]), w1 = pack_bf2(x[8 * s + 2], x[8 * s + 3]);
    const uint32_t w2 = pack_bf2(x[8 * s + 4], x[8 * s + 5]), w3 = pack_bf2(x[8 * s + 6], x[8 * s + 7]);
    sv8 r;
    r[0] = (short)(w0 & 0xffff); r[1] = (short)(w0 >> 16);
    r[2] = (short)(w1 & 0xffff); r[3] = (short)(w1 >> 16);
    r[4] = (short)(w2 & 0xffff); r[5] = (short)(w2 >> 16);
    r[6] = (short)(w3 & 0xffff); r[7] = (short)(w3 >> 16);
    return r;
}

// accumulator row of register r (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// all-ones / zero lane mask from bit `bit` of this lane's keep word (one v_bfe_i32).  The empty asm
// hides that the value is a sign-extended bit: hipcc otherwise rewrites `x & mask` as a select,
// v_and + v_cmp + v_cndmask, sunk past the bf16 packing (+v_lshr / v_perm): 4-5 instructions per
// element instead of v_bfe_i32 + v_and_b32.  (No real instruction in asm here: an asm consumer of a
// v_exp result would bypass the transcendental-use hazard padding.)
__device__ __forceinline__ uint32_t keep_mask(uint32_t w, int bit) {
    uint32_t m = keep_lanes(w, bit);
    asm("" : "+v"(m));
    return m;
}
// kept ? a : b through the keep mask: one gfx950 v_bitop3_b32 (truth table 0xe4 = s2 ? s0 : s1,
// bitwise); the plain C form became v_and, v_xor, v_and, v_or once the mask had a second use
__device__ __forceinline__ float keep_sel2(uint32_t m, float a, float b) {
    return __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(a), __float_as_uint(b), m, 0xe4));
}
__device__ __forceinline__ float keep_and(uint32_t w, int bit, float x) {
    return __uint_as_float(__float_as_uint(x) & keep_mask(w, bit));
}

// causal mask of one 32x32 accumulator tile whose key rows start at key0 (column = query qa):
// rows acc_row(r) > qa - key0 become -inf.  Called under a wave-uniform branch (diagonal tiles only).
__device__ __forceinline__ void mask_upper(fv16& x, int qa, int key0, int lane, float fill) {
    const int rel = qa - key0 - 4 * (lane >> 5);
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if ((r & 3) + 8 * (r >> 2) > rel) x[r] = fill;
}

// two [64][64] bf16 tiles (rows row0..row0+63 of X and Y) staged through registers: 4 x 16 B per thread
struct Stage2 {
    uint4 a0, a1, b0, b1;
};
__device__ __forceinline__ Stage2 stage_load(const bf16_t* X, int64_t ldx, const bf16_t* Y, int64_t ldy, int64_t row0,
                                             int tid) {
    const int r = tid >> 3, c = tid & 7;
    Stage2 s;
    s.a0 = *(const uint4*)(X + (row0 + r) * ldx + c * 8);
    s.a1 = *(const uint4*)(X + (row0 + r + 32) * ldx + c * 8);
    s.b0 = *(const uint4*)(Y + (row0 + r) * ldy + c * 8);
    s.b1 = *(const uint4*)(Y + (row0 + r + 32) * ldy + c * 8);
    return s;
}
__device__ __forceinline__ void stage_store(const Stage2& s, char* img, int tid) {
    const int r = tid >> 3, c = tid & 7;
    *(uint4*)(img + aoff(r, c)) = s.a0;
    *(uint4*)(img + aoff(r + 32, c)) = s.a1;
    *(uint4*)(img + TILE + aoff(r, c)) = s.b0;
    *(uint4*)(img + TILE + aoff(r + 32, c)) = s.b1;
}

// one [64][64] bf16 tile staged through registers: 2 x 16 B per thread
struct Stage1 {
    uint4 a0, a1;
};
__device__ __forceinline__ Stage1 stage_load1(const bf16_t* X, int64_t ldx, int64_t row0, int tid) {
    const int r = tid >> 3, c = tid & 7;
    return Stage1{*(const uint4*)(X + (row0 + r) * ldx + c * 8), *(const uint4*)(X + (row0 + r + 32) * ldx + c * 8)};
}
__device__ __forceinline__ void stage_store1(const Stage1& s, char* img, int tid) {
    const int r = tid >> 3, c = tid & 7;
    *(uint4*)(img + aoff(r, c)) = s.a0;
    *(uint4*)(img + aoff(r + 32, c)) = s.a1;
}

// XCD-aware block order for a (row blocks, B*H) grid: the dispatcher deals linear block ids to the
// 8 XCDs round-robin and each XCD has its own L2; the bijective remap hands every XCD a contiguous
// run of logical ids (whole (b, h) groups, which stream the same K/V or Q/dO), measured 35 -> 81 %
// L2 hits at C4.  REV runs a group's blocks last-first (longest causal prefix first).
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

// 16-B fragment of row `row` of a row-major bf16 matrix, columns 16 ks + 8 (lane>>5) .. +7
__device__ __forceinline__ sv8 ld_frag(const bf16_t* base, int64_t ld, int64_t row, int ks, int lane) {
    return *(const sv8*)(base + row * ld + 16 * ks + 8 * (lane >> 5));
}

// store an O^T-layout accumulator pair (dims 32 dt + acc_row, one row per lane) as bf16, x mult
__device__ __forceinline__ void store_rows(bf16_t* row, const fv16 (&acc)[2], float mult, int lane) {
    const int h = lane >> 5;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float* x = &((const float*)&acc[dt])[4 * i];
            *(uint2*)(row + 32 * dt + 8 * i + 4 * h) =
                make_uint2(pack_bf2(x[0] * mult, x[1] * mult), pack_bf2(x[2] * mult, x[3] * mult));
        }
}

// LDS-DMA (global_load_lds_dwordx4, common.h dma16) of one [64][64] bf16 tile -- rows row0..row0+63 of a row-major
// matrix -- into an aoff-swizzled image: 8 wave-instructions of 1 KB, two per wave.  LDS slot s of
// image row r holds global chunk s ^ X(r), so each lane fetches that chunk.
// img: 32-bit LDS byte address (lds_base of the __shared__ array + an offset), wave wave-uniform; the
// source as a wave-uniform base + per-lane byte offset (saddr form, common.h dma16sl)
__device__ __forceinline__ void dma_tile(const bf16_t* X, int64_t ldx, int64_t row0, uint32_t img, int wave, int lane) {
    const bf16_t* base = X + row0 * ldx;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ins = 2 * wave + i, r = 8 * ins + (lane >> 3), c = (lane & 7) ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3));
        dma16sl(base, (uint32_t)((r * ldx + 8 * c) * 2), img + 1024u * ins);
    }
}

// Tell hipcc that registers loaded by compiler-counted loads before a loop are ready here (after a
// hidden wait that drained them): otherwise its wait-count pass puts the s_waitcnt for them at their
// first use INSIDE the loop, where it runs every iteration -- vmcnt(0), which also waits for the
// next tile's DMAs issued at the iteration head (no prefetch left).
template <typename R>
__device__ __forceinline__ void ready1(const R& r) {
    asm volatile("" ::"v"(r));
}
template <typename... R>
__device__ __forceinline__ void mark_ready(const R&... r) {
    (ready1(r), ...);
}

// Resident kernels: wait for every vector-memory operation of this wave (the LDS-DMA tiles with
// it), then a workgroup barrier: every wave's DMAs have landed.  One asm statement, so no LDS read
// can be scheduled between the two.
__device__ __forceinline__ void wait_all_barrier() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// end of a ring tile: this wave's vector-memory operations older than the N DMA instructions just
// requested have landed, then every wave's (LDS reads drained too: the slot read now is rewritten
// after a later barrier)
template <int N>
__device__ __forceinline__ void ring_wait(bool pf) {
    if (pf) asm volatile("s_waitcnt vmcnt(%c0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


// =====================================================================================
// forward
// =====================================================================================
// S^T (64 keys x 32 queries) of one query group (rows qr..qr+31 of the block's Q image) against a
// K image: two independent MFMA chains, Q fragments read from LDS (not held in registers)
__device__ __forceinline__ void qk_tile(fv16 (&s)[2], const char* Ki, const char* Qimg, int qr, int lane) {
    s[0] = fv16{};
    s[1] = fv16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const sv8 qf = frag_row(Qimg, qr, ks, lane);
        s[0] = mfma32(frag_row(Ki, 0, ks, lane), qf, s[0]);
        s[1] = mfma32(frag_row(Ki, 32, ks, lane), qf, s[1]);
    }
}

// max over this lane's 32 scores (two interleaved v_max3 chains: a 2-input fmaxf of raw MFMA
// results would be preceded by canonicalising v_max x, x on each input), then over the lane^32
// partner (v_permlane32_swap: no LDS round trip)
template <int NSUB = 2>
__device__ __forceinline__ float tile_max(const fv16 (&s)[2]) {
    float m;
    if (NSUB == 2) {
        float m0 = fmaxf(fmaxf(s[0][0], s[0][1]), s[0][2]), m1 = fmaxf(fmaxf(s[1][0], s[1][1]), s[1][2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) {
            m0 = fmaxf(fmaxf(m0, s[0][r]), s[0][r + 1]);
            m1 = fmaxf(fmaxf(m1, s[1][r]), s[1][r + 1]);
        }
        m0 = fmaxf(fmaxf(m0, s[0][15]), s[1][15]);
        m = fmaxf(m0, m1);
    } else {
        float m0 = fmaxf(fmaxf(s[0][0], s[0][1]), s[0][2]), m1 = fmaxf(fmaxf(s[0][3], s[0][4]), s[0][5]);
#pragma unroll
        for (int r = 6; r < 14; r += 4) {
            m0 = fmaxf(fmaxf(m0, s[0][r]), s[0][r + 1]);
            m1 = fmaxf(fmaxf(m1, s[0][r + 2]), s[0][r + 3]);
        }
        m = fmaxf(fmaxf(m0, s[0][14]), fmaxf(m1, s[0][15]));
    }
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return __builtin_amdgcn_fmed3f(__uint_as_float(sw[0]), __uint_as_float(sw[1]), INFINITY);   // max, no re-canonicalising
}

// lazy online-softmax rescale (threshold RESCALE_THR in log2 units): called after the group's
// previous tiles are all in O and l, before this tile is exponentiated
__device__ __forceinline__ void rescale_if(float mt, float& m_run, fv4& l_run, fv16 (&o)[2]) {
    if (__any(mt > m_run + RESCALE_THR)) {   // rare after the first tiles
        const float mn = fmaxf(m_run, mt);
        const float alpha = __builtin_amdgcn_exp2f(m_run - mn);
        o[0] *= alpha;
        o[1] *= alpha;
        l_run *= alpha;
        m_run = mn;
    }
}

// low / high 16 bits all-ones where bit j / j + 16 of a FWD keep word is set: v_lshlrev_b32 puts them
// at bits 15 / 31, v_perm_b32 selectors 8 / 9 replicate those bits over bytes 0-1 / 2-3
__device__ __forceinline__ uint32_t pair_mask(uint32_t w, int j) {
    const uint32_t x = w << (15 - j), sel = 0x09090808u;
    uint32_t m;
    // (the builtin form made hipcc emit an illegal v_cmp against src_shared_base in the forward ring kernel)
    asm("v_perm_b32 %0, %1, %1, %2" : "=v"(m) : "v"(x), "s"(sel));
    return m;
}

// P = exp2(S scale_log2 - m) of a tile's NSUB subtiles, packed to the bf16 B operands of
// O^T += V^T P^T; the row sums of the packed (undropped) P go to the matrix core (rowsum_ones), then
// the dropout keep bits are applied to the packed pairs: the pair j = 8 kt + 4 sk + i of fragment
// (kt, sk) has its keep bits at j and j + 16 of the FWD word, so w << (15 - j) puts them at bits 15
// and 31, v_perm_b32 selectors 8 / 9 replicate those into the low / high 16 bits, and one v_and_b32
// drops the pair's halves -- 3 instructions per pair instead of v_bfe_i32 + v_and_b32 per element
template <bool DROP, int NSUB = 2>
__device__ __forceinline__ void softmax_pack(fv16 (&s)[2], float scale_log2, float m_run, fv4& l_run, uint32_t mw,
                                             sv8 (&pf)[2][2], const sv8& ones) {
    const float mneg = -m_run;
#pragma unroll
    for (int kt = 0; kt < NSUB; ++kt) {
#pragma unroll
        for (int r = 0; r < 16; ++r)   // raw v_exp_f32: weights below 2^-126 of the stale max flush to 0
            s[kt][r] = __builtin_amdgcn_exp2f(fmaf(s[kt][r], scale_log2, mneg));
#pragma unroll
        for (int sk = 0; sk < 2; ++sk) {
            sv8 u = pack16(s[kt], sk);
            l_run = mfma16(ones, u, l_run);
            if (DROP) {
                const int j = 8 * kt + 4 * sk;
                uint4 w = __builtin_bit_cast(uint4, u);
                w.x &= pair_mask(mw, j);
                w.y &= pair_mask(mw, j + 1);
                w.z &= pair_mask(mw, j + 2);
                w.w &= pair_mask(mw, j + 3);
                u = __builtin_bit_cast(sv8, w);
            }
            pf[kt][sk] = u;
        }
    }
}

// O^T += V^T P^T over a 64-key tile's NSUB live subtiles (two independent chains, one per 32-dim half)
template <int NSUB = 2>
__device__ __forceinline__ void pv_tile(fv16 (&o)[2], const char* Vi, const sv8 (&pf)[2][2], int lane) {
#pragma unroll
    for (int kt = 0; kt < NSUB; ++kt)
#pragma unroll
        for (int sk = 0; sk < 2; ++sk) {
            o[0] = mfma32(frag_tr(Vi, 32 * kt, sk, 0, lane), pf[kt][sk], o[0]);
            o[1] = mfma32(frag_tr(Vi, 32 * kt, sk, 32, lane), pf[kt][sk], o[1]);
        }
}

// One query group's 64-key tile outside the pipeline: NSUB live 32-key subtiles (1 when the second
// lies wholly above the diagonal); DIAG = the subtile holding the diagonal (-1: none) -- the only
// one masked.  Straight-line code per case (the merged form copied accumulators between paths).
// QREG: the group's Q fragments come from registers (qreg[4]) instead of the Q image.
template <bool DROP, int NSUB, int DIAG, bool QREG = false>
__device__ __forceinline__ void fwd_group_tile(const char* Ki, const char* Vi, const char* Qimg, int qr, int lane,
                                               float scale_log2, float& m_run, fv4& l_run, fv16 (&o)[2],
                                               uint32_t mw, const sv8& ones, const sv8* qreg = nullptr) {
    fv16 s[2];
    s[0] = fv16{};
    s[1] = fv16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const sv8 qf = QREG ? qreg[ks] : frag_row(Qimg, qr, ks, lane);
        s[0] = mfma32(frag_row(Ki, 0, ks, lane), qf, s[0]);
        if (NSUB == 2) s[1] = mfma32(frag_row(Ki, 32, ks, lane), qf, s[1]);
    }
    if (DIAG >= 0) mask_upper(s[DIAG], lane & 31, 0, lane, -INFINITY);   // key0 = the group's first query
    rescale_if(tile_max<NSUB>(s) * scale_log2, m_run, l_run, o);
    sv8 pf[2][2];
    softmax_pack<DROP, NSUB>(s, scale_log2, m_run, l_run, mw, pf, ones);
    pv_tile<NSUB>(o, Vi, pf, lane);
}

// Forward.  Tiles where both of a wave's query groups (A = 7 - w, B = w) are full (before B's
// diagonal tile) run software-pipelined, B one phase behind A, so every MFMA phase has the other
// group's softmax VALU work beside it:
//   [1] S_A(kv)      || P_B(kv-1) = softmax of B's previous tile
//   [2] O_B += P_B V(kv-1) || max_A(kv), A's rescale decision
//   [3] S_B(kv)      || P_A(kv)
//   [4] O_A += P_A V(kv)   || max_B(kv), B's rescale decision
// (each group's decision precedes its exponentials and follows its previous P V).  K/V tiles go
// through a 3-slot LDS ring (B still reads V(kv-1) while kv+1 is written), one barrier per tile.
// The diagonal and later tiles run unpipelined.  The block's 256 Q rows live in LDS (32 KB, same
// swizzle) rather than in registers: 48 + 32 KB per block, two blocks per CU.
constexpr int FWD_SLOT = 2 * TILE;
constexpr int FWD_LDS = 3 * FWD_SLOT + 4 * TILE;   // K/V ring + Q image: 80 KB


// =====================================================================================
// dQ: S^T = K Q^T, dP^T = V dO^T, dS^T = P^T (keep/(1-p) dP^T - delta), dQ^T += K^T dS^T.
// The 1/(1-p) is factored out of dS (dS = 1/(1-p) P (keep dP - (1-p) delta), applied with scale in
// the epilogue), so an element costs dP - delta', one v_bfi_b32 select (dropped: -delta') and P x.
// =====================================================================================
// query-side operands of one dQ group (query qa = qg + (lane & 31)): Q and dO fragments, lse in
// log2 units and -delta' = -(1-p) delta, where delta = rowsum(dO * O) (dropout-invariant: O already
// holds the dropped P) is also written for the dK/dV kernel.  Bases are the (b, h) row-0 pointers.
__device__ __forceinline__ void dq_group_setup(bool act, int64_t qa, const bf16_t* qb, int64_t ld, const bf16_t* ob,
                                               int64_t ldo, const bf16_t* db, int64_t ldd, const float* lse_bh,
                                               float* delta_bh, float dscale, int lane, sv8 (&qf)[4], sv8 (&df)[4],
                                               float& lse2, float& dl) {
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        qf[ks] = act ? ld_frag(qb, ld, qa, ks, lane) : sv8{};
        df[ks] = act ? ld_frag(db, ldd, qa, ks, lane) : sv8{};
        if (act) {
            const sv8 of = ld_frag(ob, ldo, qa, ks, lane);
#pragma unroll
            for (int j = 0; j < 8; ++j) dsum += bf2f((bf16_t)of[j]) * bf2f((bf16_t)df[ks][j]);
        }
    }
    dsum += __shfl_xor(dsum, 32, 64);
    dl = -dsum / dscale;   // -delta' = -(1-p) delta
    lse2 = act ? lse_bh[qa] * LOG2E : 0.f;
    if (act && lane < 32) delta_bh[qa] = dsum;
}

// one 64-key tile (K / V images, first key k0) of a dQ query group starting at query qg: its 32-key
// subtiles up to the diagonal; only the subtile whose first key is qg holds the diagonal
template <bool DROP>
__device__ __forceinline__ void dq_group_tile(const char* Ki, const char* Vi, int k0, int qg, const sv8 (&qf)[4],
                                              const sv8 (&df)[4], float lse2, float dl, uint32_t mw, float c2,
                                              fv16 (&dqa)[2], int lane) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        if (k0 + 32 * kt > qg + 31) break;   // subtile fully masked
        const bool diag = __builtin_amdgcn_readfirstlane(k0 + 32 * kt == qg);
        // dP^T starts from -delta' (its column's, lane-uniform), so the chain leaves dP - delta'
        fv16 s = fv16{}, dp = fv16{} + dl;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            s = mfma32(frag_row(Ki, 32 * kt, ks, lane), qf[ks], s);
            dp = mfma32(frag_row(Vi, 32 * kt, ks, lane), df[ks], dp);
        }
        if (diag) mask_upper(s, lane & 31, 0, lane, -INFINITY);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lse2));
            float d = dp[r];
            if (DROP) d = keep_sel2(keep_mask(mw, fwd_bit(kt, r)), d, dl);
            s[r] = p * d;
        }
        const sv8 d0 = pack16(s, 0), d1 = pack16(s, 1);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            dqa[dt] = mfma32(frag_tr(Ki, 32 * kt, 0, 32 * dt, lane), d0, dqa[dt]);
            dqa[dt] = mfma32(frag_tr(Ki, 32 * kt, 1, 32 * dt, lane), d1, dqa[dt]);
        }
    }
}

// K/V tiles by LDS-DMA (common.h dma16) into a 2-slot ring, the next tile's DMAs issued before the
// current tile's products (round 2: register staging measured 706 -> 686 us for the C4 backward)
template <bool DROP, int NS>
__device__ __forceinline__ void dq_qblock(int qblk, int bh, char* smem, int64_t T_, int H, const bf16_t* __restrict__ q,
                                          const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, int64_t ld,
                                          const bf16_t* __restrict__ o, int64_t ldo, const bf16_t* __restrict__ dout,
                                          int64_t ldd, const float* __restrict__ lse, float* __restrict__ delta,
                                          bf16_t* __restrict__ dq, int64_t lddq, float scale,
                                          const uint32_t* __restrict__ mask, float dscale) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = (int)T_, b = bh / H, hh = bh % H;
    const int Q0 = qblk * 256;
    const int64_t boff = (int64_t)b * T_, ntile = mask_tiles(T_);
    const float c2 = scale * LOG2E;
    const bf16_t* kb_ = k + boff * ld + hh * 64;
    const bf16_t* vb_ = v + boff * ld + hh * 64;
    const int qg[2] = {Q0 + 32 * (7 - wave), Q0 + 32 * wave};
    const bool act[2] = {qg[0] < T, qg[1] < T};
    const uint32_t* mrow[2];
    uint32_t mw[2] = {0u, 0u};
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        mrow[g] = DROP ? mask + ((int64_t)bh * ntile + mask_fwd_tile(qg[g] >> 5, 0)) * 64 + lane : nullptr;
        if (DROP && act[g]) mw[g] = mrow[g][0];
    }
    sv8 qf[2][4], df[2][4];
    float lse2[2], dl[2];
#pragma unroll
    for (int g = 0; g < 2; ++g)
        dq_group_setup(act[g], qg[g] + (lane & 31), q + boff * ld + hh * 64, ld, o + boff * ldo + hh * 64, ldo,
                       dout + boff * ldd + hh * 64, ldd, lse + (int64_t)bh * T_, delta + (int64_t)bh * T_, dscale, lane,
                       qf[g], df[g], lse2[g], dl[g]);
    fv16 dqa[2][2];
#pragma unroll
    for (int g = 0; g < 2; ++g) dqa[g][0] = dqa[g][1] = fv16{};
    const int qlast = (Q0 + 255 < T - 1) ? Q0 + 255 : T - 1;
    const int nkv = qlast / 64 + 1;
    const int wave_ = __builtin_amdgcn_readfirstlane(tid >> 6);
    // K/V ring of NS slots, tile kv + AH requested at the head of tile kv into the slot of tile
    // kv + AH - NS (read before an earlier barrier); NS = 4: two tiles of compute to land
    constexpr int AH = NS / 2;
    auto slot = [&](int t) { return smem + (t & (NS - 1)) * 2 * TILE; };
    const uint32_t l0 = lds_base(smem);
    auto lslot = [&](int t) { return l0 + (uint32_t)((t & (NS - 1)) * 2 * TILE); };
#pragma unroll
    for (int t = 0; t < AH; ++t) {
        if (t < nkv) {
            dma_tile(kb_, ld, (int64_t)t * 64, lslot(t), wave_, lane);
            dma_tile(vb_, ld, (int64_t)t * 64, lslot(t) + TILE, wave_, lane);
        }
    }
    ring_wait<AH == 2 ? 4 : 0>(AH == 2 && nkv > 1);   // operands and tile 0 have landed
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) mark_ready(qf[g][ks], df[g][ks]);
    mark_ready(mw[0], mw[1], lse2[0], lse2[1], dl[0], dl[1]);
    for (int kv = 0; kv < nkv; ++kv) {
        const int nxt = kv + 1 < nkv ? kv + 1 : kv;
        // the next tile's keep words by hidden loads, issued before the DMAs so that the counted wait
        // at the tile's end retires them (a compiler-counted load issued after the DMAs made hipcc
        // wait vmcnt(0) -- for the DMAs too -- at the head of the tile)
        uint32_t mn[2] = {0u, 0u};
        if constexpr (DROP) {
#pragma unroll
            for (int g = 0; g < 2; ++g)
                if (act[g] && nxt * 64 <= qg[g] + 31) gload4(mn[g], mrow[g] + nxt * 64);
        }
        const bool pf = kv + AH < nkv;
        if (pf) {
            dma_tile(kb_, ld, (int64_t)(kv + AH) * 64, lslot(kv + AH), wave_, lane);
            dma_tile(vb_, ld, (int64_t)(kv + AH) * 64, lslot(kv + AH) + TILE, wave_, lane);
        }
        const char* Ki = slot(kv);
        const int k0 = kv * 64;
#pragma unroll
        for (int g = 0; g < 2; ++g)
            if (act[g] && k0 <= qg[g] + 31)
                dq_group_tile<DROP>(Ki, Ki + TILE, k0, qg[g], qf[g], df[g], lse2[g], dl[g], mw[g], c2, dqa[g], lane);
        ring_wait<AH == 2 ? 4 : 0>(pf);   // tile kv + 1 (and the keep words) have landed for every wave
        asm volatile("" : "+v"(mn[0]), "+v"(mn[1]));
        mw[0] = mn[0];
        mw[1] = mn[1];
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (!act[g]) continue;
        const int64_t qa = qg[g] + (lane & 31);
        store_rows(dq + (boff + qa) * lddq + hh * 64, dqa[g], scale * dscale, lane);
    }
}

// pairs of query blocks per workgroup, as the forward
template <bool DROP, int NS>
__global__ __launch_bounds__(256, 2) void k_attn_dq_d64(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                        const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                        int64_t ld, const bf16_t* __restrict__ o, int64_t ldo,
                                                        const bf16_t* __restrict__ dout, int64_t ldd,
                                                        const float* __restrict__ lse, float* __restrict__ delta,
                                                        bf16_t* __restrict__ dq, int64_t lddq, float scale,
                                                        const uint32_t* __restrict__ mask, float dscale) {
    __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TILE];
    int x, bh;
    block_coords<false>(x, bh);
    const int nq = (int)((T_ + 255) / 256), first = nq - 1 - x;
    const int npass = x == first ? 1 : 2;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
        if (pass) __syncthreads();
        dq_qblock<DROP, NS>(pass ? x : first, bh, smem, T_, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale,
                        mask, dscale);
    }
}

// =====================================================================================
// dK / dV: block = 4 waves x 32 keys; stream 64-query tiles (Q, dO, lse, delta)
// =====================================================================================
constexpr int KV_STAGE = 2 * TILE + 512;   // Q image, dO image, lse*log2e [64], delta [64]

// one 64-query tile (Q / dO images, their lse*log2e and -delta' rows) of a dK/dV key group starting
// at key kq (key = kq + (lane & 31)): the 32-query subtiles that reach the group's keys
template <bool DROP>
__device__ __forceinline__ void dkdv_tile(const char* Qi, const char* Oi, const float* st_lse, const float* st_del,
                                          int q0, int kq, int key, const sv8 (&kf)[4], const sv8 (&vf)[4], uint32_t mw,
                                          float c2, fv16 (&dka)[2], fv16 (&dva)[2], int lane) {
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
        const int q0s = q0 + 32 * qs;
        if (q0s + 31 < kq) continue;   // every query of the subtile precedes every key
        // dP starts from -delta' of its rows (the accumulator's initial value), so the MFMA
        // chain leaves dP - delta'; dS = 1/(1-p) P (keep dP - delta'), the 1/(1-p) in the epilogue
        fv16 s = fv16{}, dp;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 d4 = *(const float4*)(st_del + 32 * qs + 8 * i + 4 * (lane >> 5));
            dp[4 * i] = d4.x;
            dp[4 * i + 1] = d4.y;
            dp[4 * i + 2] = d4.z;
            dp[4 * i + 3] = d4.w;
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            s = mfma32(frag_row(Qi, 32 * qs, ks, lane), kf[ks], s);
            dp = mfma32(frag_row(Oi, 32 * qs, ks, lane), vf[ks], dp);
        }
        if (__builtin_amdgcn_readfirstlane(q0s < kq + 31)) {
            // diagonal subtile: queries (rows) before the key (column) are masked
            const int rel = key - q0s - 4 * (lane >> 5);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if ((r & 3) + 8 * (r >> 2) < rel) s[r] = -INFINITY;
        }
        fv16 z;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // rows 8i + 4(lane>>5) + 0..3 of the subtile: one 16-B LDS read each (broadcast)
            const int row = 32 * qs + 8 * i + 4 * (lane >> 5);
            const float4 l4 = *(const float4*)(st_lse + row);
            const float4 d4 = *(const float4*)(st_del + row);
            const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dvv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * i + e;
                const float p = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lv[e]));
                float d = dp[r];   // dP - delta'
                if (DROP) {
                    const uint32_t kp = keep_mask(mw, 16 * qs + r);   // 1/(1-p) of dV: epilogue
                    z[r] = __uint_as_float(__float_as_uint(p) & kp);
                    d = keep_sel2(kp, d, dvv[e]);                     // dropped: -delta'
                } else {
                    z[r] = p;
                }
                s[r] = p * d;
            }
        }
        const sv8 z0 = pack16(z, 0), z1 = pack16(z, 1), s0 = pack16(s, 0), s1 = pack16(s, 1);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            dva[dt] = mfma32(frag_tr(Oi, 32 * qs, 0, 32 * dt, lane), z0, dva[dt]);
            dva[dt] = mfma32(frag_tr(Oi, 32 * qs, 1, 32 * dt, lane), z1, dva[dt]);
            dka[dt] = mfma32(frag_tr(Qi, 32 * qs, 0, 32 * dt, lane), s0, dka[dt]);
            dka[dt] = mfma32(frag_tr(Qi, 32 * qs, 1, 32 * dt, lane), s1, dka[dt]);
        }
    }
}

template <bool DROP, int NS>
__device__ __forceinline__ void dkdv_kblock(int kblk, int bh, char* smem, int64_t T_, int H,
                                            const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                            const bf16_t* __restrict__ v, int64_t ld, const bf16_t* __restrict__ dout,
                                            int64_t ldd, const float* __restrict__ lse,
                                            const float* __restrict__ delta, bf16_t* __restrict__ dk,
                                            bf16_t* __restrict__ dv, int64_t lddkv, float scale,
                                            const uint32_t* __restrict__ mask, float dscale) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = (int)T_, b = bh / H, hh = bh % H;
    const int K0 = kblk * 128, kq = K0 + 32 * wave;
    const bool act = kq < T;
    const int64_t boff = (int64_t)b * T_, ntile = mask_tiles(T_);
    const float c2 = scale * LOG2E;
    const int key = kq + (lane & 31);
    sv8 kf[4], vf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        kf[ks] = act ? ld_frag(k + boff * ld + hh * 64, ld, key, ks, lane) : sv8{};
        vf[ks] = act ? ld_frag(v + boff * ld + hh * 64, ld, key, ks, lane) : sv8{};
    }
    fv16 dka[2] = {fv16{}, fv16{}}, dva[2] = {fv16{}, fv16{}};
    const bf16_t* qb_ = q + boff * ld + hh * 64;
    const bf16_t* ob_ = dout + boff * ldd + hh * 64;
    const float* lse_b = lse + (int64_t)bh * T_;
    const float* del_b = delta + (int64_t)bh * T_;
    const int nq = T / 64, qt0 = K0 / 64;
    // keep words: BWD tiles (key block kq/32, query tile qt >= kq/64), prefetched one tile ahead
    const int kbw = kq >> 5, qtm = kbw >> 1;
    const uint32_t* mcol =
        DROP && act ? mask + ((int64_t)bh * ntile + mask_bwd_tile(kbw, qtm, nq)) * 64 + lane : nullptr;
    uint32_t mw = (DROP && act && qt0 >= qtm) ? mcol[(qt0 - qtm) * 64] : 0u;
    auto stat_load = [&](int qt) {
        float s = 0.f;
        if (tid < 64) s = lse_b[qt * 64 + tid] * LOG2E;
        else if (tid < 128) s = -del_b[qt * 64 + tid - 64] / dscale;   // -delta' = -(1-p) delta
        return s;
    };
    const int wave_ = __builtin_amdgcn_readfirstlane(tid >> 6);
    // Q/dO ring of NS slots (images + row statistics), tile qt + AH requested at the head of tile qt
    // into the slot of tile qt + AH - NS (read before an earlier barrier); NS = 4: two tiles of
    // compute to land.  A slot's statistics are written from hidden loads issued with its DMA.
    constexpr int AH = NS / 2;
    auto slot = [&](int it_) { return smem + (it_ & (NS - 1)) * KV_STAGE; };
    const uint32_t l0 = lds_base(smem);
    auto lslot = [&](int it_) { return l0 + (uint32_t)((it_ & (NS - 1)) * KV_STAGE); };
    {
        const float s0 = stat_load(qt0);
        const float s1 = (AH == 2 && qt0 + 1 < nq) ? stat_load(qt0 + 1) : 0.f;
#pragma unroll
        for (int t = 0; t < AH; ++t) {
            if (qt0 + t < nq) {
                dma_tile(qb_, ld, (int64_t)(qt0 + t) * 64, lslot(t), wave_, lane);
                dma_tile(ob_, ldd, (int64_t)(qt0 + t) * 64, lslot(t) + TILE, wave_, lane);
                if (tid < 128) ((float*)(slot(t) + 2 * TILE))[tid] = t ? s1 : s0;
            }
        }
    }
    ring_wait<AH == 2 ? 4 : 0>(AH == 2 && qt0 + 1 < nq);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) mark_ready(kf[ks], vf[ks]);
    mark_ready(mw);
    for (int qt = qt0; qt < nq; ++qt) {
        const int it = qt - qt0;
        const int nxt = qt + 1 < nq ? qt + 1 : qt;
        const bool pf = qt + AH < nq;
        // tile qt + AH's row statistics and tile qt + 1's keep word by hidden loads issued before the
        // DMAs, so the counted wait at the tile's end retires them (compiler-counted loads issued
        // after the DMAs made hipcc wait vmcnt(0) -- for the DMAs too -- inside this tile's products)
        uint32_t sw = 0u, mn = 0u;
        if (pf) {
            if (tid < 64) gload4(sw, lse_b + (qt + AH) * 64 + tid);
            else if (tid < 128) gload4(sw, del_b + (qt + AH) * 64 + tid - 64);
        }
        if (DROP && act && nxt >= qtm) gload4(mn, mcol + (nxt - qtm) * 64);
        if (pf) {
            dma_tile(qb_, ld, (int64_t)(qt + AH) * 64, lslot(it + AH), wave_, lane);
            dma_tile(ob_, ldd, (int64_t)(qt + AH) * 64, lslot(it + AH) + TILE, wave_, lane);
        }
        const char* S0 = slot(it);
        const char* Qi = S0;
        const char* Oi = S0 + TILE;
        const float* st_lse = (const float*)(S0 + 2 * TILE);
        const float* st_del = st_lse + 64;
        const int q0 = qt * 64;
        if (act && q0 + 63 >= kq) dkdv_tile<DROP>(Qi, Oi, st_lse, st_del, q0, kq, key, kf, vf, mw, c2, dka, dva, lane);
        // tile qt + 1, the statistics and the keep word have landed (tile qt + AH's DMAs may not)
        if (AH == 2 && pf) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(sw), "+v"(mn));
        if (pf) {   // stat_load's arithmetic on the loaded word
            char* D = slot(it + AH);
            if (tid < 64) ((float*)(D + 2 * TILE))[tid] = __uint_as_float(sw) * LOG2E;
            else if (tid < 128) ((float*)(D + 2 * TILE))[tid] = -__uint_as_float(sw) / dscale;
        }
        mw = mn;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (!act) return;
    store_rows(dk + (boff + key) * lddkv + hh * 64, dka, scale * dscale, lane);
    store_rows(dv + (boff + key) * lddkv + hh * 64, dva, DROP ? dscale : 1.f, lane);
}

// pairs of 128-key blocks per workgroup (x, then nk - 1 - x): uniform causal work per workgroup
template <bool DROP, int NS>
__global__ __launch_bounds__(256, 2) void k_attn_dkdv_d64(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                          const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                          int64_t ld, const bf16_t* __restrict__ dout, int64_t ldd,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta, bf16_t* __restrict__ dk,
                                                          bf16_t* __restrict__ dv, int64_t lddkv, float scale,
                                                          const uint32_t* __restrict__ mask, float dscale) {
    __shared__ __attribute__((aligned(16))) char smem[NS * KV_STAGE];
    int x, bh;
    block_coords<false>(x, bh);
    const int nk = (int)((T_ + 127) / 128), second = nk - 1 - x;
    const int npass = x == second ? 1 : 2;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
        if (pass) __syncthreads();
        dkdv_kblock<DROP, NS>(pass ? second : x, bh, smem, T_, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale,
                          mask, dscale);
    }
}

// =====================================================================================
// T <= 256: sequence-resident kernels (the C2 shape, T = 256)
// =====================================================================================
// At T = 256 the ring kernels above are latency-bound: a workgroup per (b, h) stages one 16-KB tile
// at a time through registers (one tile in flight per 256 threads), and 384 workgroups fill 1.5 of
// the 2 slots per CU (forward 23 us for 52.7 MB, 2.3 TB/s).  Here every K/V (or Q/dO) tile of the
// (b, h) is requested at once by LDS-DMA (64 KB per workgroup), the query-side (key-side) operands
// are loaded to registers right behind them, and after one wait + barrier the tile loop runs with
// no staging barriers.  Same wave/group assignment, per-tile arithmetic and keep-bit words as the
// ring kernels, so the results are bitwise the same.  (The register loads follow the DMAs: vmcnt
// retires in order, so waiting for them covers the tiles too -- see common.h dma16.)
// O^T accumulator pair of one query (lane & 31; dims 32 dt + acc_row) as bf16, x mult, in 16-B
// row segments: lanes l and l + 32 hold the two 4-dim halves of each 8-dim group, so for each
// pair of groups (i, i + 1) one v_permlane32_swap per dword leaves lanes 0-31 with dims 8i..8i+7
// and lanes 32-63 with 8(i+1)..8(i+1)+7 (cdna_hip_programming.md T21): 4 dwordx4 stores per lane
// instead of 8 dwordx2.  Same bytes as store_rows.
__device__ __forceinline__ void store_rows_wide(bf16_t* row, const fv16 (&acc)[2], float mult, int lane) {
    const int h = lane >> 5;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            const float* x = &((const float*)&acc[dt])[4 * i];
            const float* y = &((const float*)&acc[dt])[4 * i + 4];
            const uint32_t a0 = pack_bf2(x[0] * mult, x[1] * mult), a1 = pack_bf2(x[2] * mult, x[3] * mult);
            const uint32_t b0 = pack_bf2(y[0] * mult, y[1] * mult), b1 = pack_bf2(y[2] * mult, y[3] * mult);
            const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
            *(uint4*)(row + 32 * dt + 8 * (i + h)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
}

// Resident forward (T = 64 NT <= 256).  Every load is issued up front -- the query-side operands
// first (Q fragments and keep words: hidden register loads, common.h gload16/gload4), then the
// K/V tiles in tile order by LDS-DMA -- and tile t waits only for what it reads: the register
// loads and tiles 0..t (vmcnt counts them in issue order), so the first tile's MFMAs start while
// the later tiles are still in flight.  Same per-tile arithmetic and keep words as the ring kernel.
template <bool DROP, int NT>
__global__ __launch_bounds__(256, 2) void k_attn_fwd_d64r(int H, const bf16_t* __restrict__ q,
                                                          const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                          int64_t ld, bf16_t* __restrict__ o, int64_t ldo,
                                                          float* __restrict__ lse, float scale_log2,
                                                          const uint32_t* __restrict__ mask, float dscale) {
    constexpr int T = 64 * NT;
    __shared__ __attribute__((aligned(16))) char smem[NT * 2 * TILE];   // K, V images of tile t at 2 t TILE
    ATTN_STAMP(0, attn_now());
    int x, bh;
    block_coords<false>(x, bh);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = bh / H, hh = bh % H;
    const int64_t boff = (int64_t)b * T, ntile = mask_tiles(T);
    const int qg[2] = {32 * (7 - wave), 32 * wave};   // A = 7 - w (longer causal prefix), B = w
    const bool act[2] = {qg[0] < T, qg[1] < T};
    sv8 qv[2][4];
    uint32_t mw[2][NT];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const int qa = (act[g] ? qg[g] : 0) + (lane & 31);   // inactive groups load a valid row, unused
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) gload16(qv[g][ks], q + (boff + qa) * ld + hh * 64 + 16 * ks + 8 * (lane >> 5));
        if constexpr (DROP) {
            const int qb = act[g] ? qg[g] >> 5 : 0;
#pragma unroll
            for (int t = 0; t < NT; ++t) {   // tiles past the group's diagonal re-read tile 0 (unused)
                const int tt = 64 * t <= 32 * qb + 31 ? t : 0;
                gload4(mw[g][t], mask + ((int64_t)bh * ntile + mask_fwd_tile(qb, tt)) * 64 + lane);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        dma_tile(k + boff * ld + hh * 64, ld, 64 * t, lds_base(smem) + 2u * t * TILE, wave, lane);
        dma_tile(v + boff * ld + hh * 64, ld, 64 * t, lds_base(smem) + (2u * t + 1) * TILE, wave, lane);
    }
    // the register loads and tile 0 have landed (4 DMA instructions per tile per wave stay younger)
    if constexpr (!DROP) {
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int t = 0; t < NT; ++t) mw[g][t] = 0u;
    }
    // then every destination is named "+v" by an (ordered, volatile) empty statement after the wait,
    // so nothing reads it earlier
    asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(4 * (NT - 1)) : "memory");
    ATTN_STAMP(1, attn_now());
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(qv[g][ks]));
#pragma unroll
        for (int t = 0; t < NT; ++t) asm volatile("" : "+v"(mw[g][t]));
    }
    const sv8 (&qf)[2][4] = qv;
    fv16 oacc[2][2];
#pragma unroll
    for (int g = 0; g < 2; ++g) oacc[g][0] = oacc[g][1] = fv16{};
    float m_run[2] = {-FLT_MAX, -FLT_MAX};
    fv4 l_run[2] = {fv4{}, fv4{}};
    const sv8 ones = rowsum_ones(lane);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t) {   // tile t's DMAs (every wave's) have landed
            if constexpr (NT >= 2) {
                if (t == 1) asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(4 * (NT > 1 ? NT - 2 : 0)) : "memory");
            }
            if constexpr (NT >= 3) {
                if (t == 2) asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(4 * (NT > 2 ? NT - 3 : 0)) : "memory");
            }
            if constexpr (NT >= 4) {
                if (t == 3) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            }
        }
        const char* Ki = smem + 2 * t * TILE;
        const char* Vi = Ki + TILE;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (!act[g] || 64 * t > qg[g] + 31) continue;
            const int rel = __builtin_amdgcn_readfirstlane(qg[g] - 64 * t);
            if (rel >= 64)
                fwd_group_tile<DROP, 2, -1, true>(Ki, Vi, nullptr, 0, lane, scale_log2, m_run[g], l_run[g], oacc[g],
                                                  mw[g][t], ones, qf[g]);
            else if (rel == 32)
                fwd_group_tile<DROP, 2, 1, true>(Ki, Vi, nullptr, 0, lane, scale_log2, m_run[g], l_run[g], oacc[g],
                                                 mw[g][t], ones, qf[g]);
            else
                fwd_group_tile<DROP, 1, 0, true>(Ki, Vi, nullptr, 0, lane, scale_log2, m_run[g], l_run[g], oacc[g],
                                                 mw[g][t], ones, qf[g]);
        }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (!act[g]) continue;
        const float lt = l_run[g][0];   // every accumulator register holds query lane & 31's sum
        const int64_t qa = qg[g] + (lane & 31);
        store_rows_wide(o + (boff + qa) * ldo + hh * 64, oacc[g], dscale / lt, lane);
        if (lane < 32) lse[(int64_t)bh * T + qa] = (m_run[g] + __log2f(lt)) * LN2;
    }
    ATTN_STAMP(2, attn_now());
    ATTN_STAMP(3, attn_where(2));
}

// tile t > 0 of a resident kernel: this wave's DMAs of tiles 0..t have landed (4 DMA instructions per
// tile per wave, issued in tile order after the first register loads; X hidden loads issued after the
// DMAs stay in flight too), then every wave's (barrier)
template <int NT, int X = 0>
__device__ __forceinline__ void res_tile_wait(int t) {
    if constexpr (NT >= 2) {
        if (t == 1) asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(4 * (NT > 1 ? NT - 2 : 0) + X) : "memory");
    }
    if constexpr (NT >= 3) {
        if (t == 2) asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(4 * (NT > 2 ? NT - 3 : 0) + X) : "memory");
    }
    if constexpr (NT >= 4) {
        if (t == 3) asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(X) : "memory");
    }
}

// Resident dQ (T = 64 NT <= 256): the query-side operands (Q, dO and O fragments, lse, keep words)
// by hidden register loads first, then the K/V tiles by LDS-DMA in tile order; tile t waits only
// for tiles 0..t (as k_attn_fwd_d64r).  Per-group setup (delta in dq_group_setup's summation order)
// and per-tile arithmetic as the ring kernel.
template <bool DROP, int NT, bool DIN = false>
__device__ __forceinline__ void dq_res(int bh, char* smem, int H, const bf16_t* __restrict__ q,
                                       const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, int64_t ld,
                                       const bf16_t* __restrict__ o, int64_t ldo, const bf16_t* __restrict__ dout,
                                       int64_t ldd, const float* __restrict__ lse, float* __restrict__ delta,
                                       bf16_t* __restrict__ dq, int64_t lddq, float scale,
                                       const uint32_t* __restrict__ mask, float dscale) {
    constexpr int T = 64 * NT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = bh / H, hh = bh % H;
    const int64_t boff = (int64_t)b * T, ntile = mask_tiles(T);
    const float c2 = scale * LOG2E;
    const int qg[2] = {32 * (7 - wave), 32 * wave};
    const bool act[2] = {qg[0] < T, qg[1] < T};
    sv8 qf[2][4], df[2][4], of[2][4];
    uint32_t lsew[2], delw[2] = {0u, 0u}, mw[2][NT];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const int64_t qa = (act[g] ? qg[g] : 0) + (lane & 31);   // inactive groups: a valid row, unused
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int col = hh * 64 + 16 * ks + 8 * (lane >> 5);
            gload16(qf[g][ks], q + (boff + qa) * ld + col);
            gload16(df[g][ks], dout + (boff + qa) * ldd + col);
            if constexpr (!DIN) gload16(of[g][ks], o + (boff + qa) * ldo + col);
        }
        gload4(lsew[g], lse + (int64_t)bh * T + qa);
        if constexpr (DIN) gload4(delw[g], delta + (int64_t)bh * T + qa);
        if constexpr (DROP) {
            const int qb = act[g] ? qg[g] >> 5 : 0;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int tt = 64 * t <= 32 * qb + 31 ? t : 0;
                gload4(mw[g][t], mask + ((int64_t)bh * ntile + mask_fwd_tile(qb, tt)) * 64 + lane);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        dma_tile(k + boff * ld + hh * 64, ld, 64 * t, lds_base(smem) + 2u * t * TILE, wave, lane);
        dma_tile(v + boff * ld + hh * 64, ld, 64 * t, lds_base(smem) + (2u * t + 1) * TILE, wave, lane);
    }
    if constexpr (!DROP) {
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int t = 0; t < NT; ++t) mw[g][t] = 0u;
    }
    asm volatile("s_waitcnt vmcnt(%c0)\n\ts_barrier" ::"i"(4 * (NT - 1)) : "memory");
    ATTN_STAMP(1, attn_now());
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            asm volatile("" : "+v"(qf[g][ks]));
            asm volatile("" : "+v"(df[g][ks]));
            if constexpr (!DIN) asm volatile("" : "+v"(of[g][ks]));
        }
        asm volatile("" : "+v"(lsew[g]), "+v"(delw[g]));
#pragma unroll
        for (int t = 0; t < NT; ++t) asm volatile("" : "+v"(mw[g][t]));
    }
    float lse2[2], dl[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {   // dq_group_setup's arithmetic on the loaded fragments
        float dsum = 0.f;
        if constexpr (DIN) {
            dsum = act[g] ? __uint_as_float(delw[g]) : 0.f;
        } else {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                for (int j = 0; j < 8; ++j) dsum += bf2f((bf16_t)of[g][ks][j]) * bf2f((bf16_t)df[g][ks][j]);
            if (!act[g]) dsum = 0.f;
            dsum += __shfl_xor(dsum, 32, 64);
        }
        dl[g] = -dsum / dscale;
        lse2[g] = act[g] ? __uint_as_float(lsew[g]) * LOG2E : 0.f;
        if (!DIN && act[g] && lane < 32) delta[(int64_t)bh * T + qg[g] + (lane & 31)] = dsum;
    }
    fv16 dqa[2][2];
#pragma unroll
    for (int g = 0; g < 2; ++g) dqa[g][0] = dqa[g][1] = fv16{};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        res_tile_wait<NT>(t);
        const char* Ki = smem + 2 * t * TILE;
#pragma unroll
        for (int g = 0; g < 2; ++g)
            if (act[g] && 64 * t <= qg[g] + 31)
                dq_group_tile<DROP>(Ki, Ki + TILE, 64 * t, qg[g], qf[g], df[g], lse2[g], dl[g], mw[g][t], c2, dqa[g],
                                    lane);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (!act[g]) continue;
        const int64_t qa = qg[g] + (lane & 31);
        store_rows_wide(dq + (boff + qa) * lddq + hh * 64, dqa[g], scale * dscale, lane);
    }
}

template <bool DROP, int NT>
__global__ __launch_bounds__(256, 2) void k_attn_dq_d64r(int H, const bf16_t* __restrict__ q,
                                                         const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                         int64_t ld, const bf16_t* __restrict__ o, int64_t ldo,
                                                         const bf16_t* __restrict__ dout, int64_t ldd,
                                                         const float* __restrict__ lse, float* __restrict__ delta,
                                                         bf16_t* __restrict__ dq, int64_t lddq, float scale,
                                                         const uint32_t* __restrict__ mask, float dscale) {
    __shared__ __attribute__((aligned(16))) char smem[NT * 2 * TILE];
    int x, bh;
    block_coords<false>(x, bh);
    dq_res<DROP, NT>(bh, smem, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, mask, dscale);
}

// dK/dV: one workgroup per (b, h); wave w takes key group w, then key group 7 - w (equal causal
// work per wave: 8 + 1, 7 + 2, ... 32-query subtiles at T = 256), Q / dO / lse / delta resident.
// o != NULL: delta = rowsum(dO * O) is computed here (in dq_group_setup's summation order, so
// bitwise the dQ kernel's value) instead of read from `delta` -- the merged backward launch.
// Register operands (row statistics, the first key group's K / V fragments, keep words) by hidden
// loads first, then the Q / dO tiles by LDS-DMA; the first key group's tile t waits only for tiles
// 0..t.  OD: delta from O and dO (o != NULL), else read from `delta`.
template <bool DROP, int NT, bool OD>
__device__ __forceinline__ void dkdv_res(int bh, char* smem, int H, const bf16_t* __restrict__ q,
                                         const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, int64_t ld,
                                         const bf16_t* __restrict__ dout, int64_t ldd, const float* __restrict__ lse,
                                         const float* __restrict__ delta, const bf16_t* __restrict__ o, int64_t ldo,
                                         bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int64_t lddkv, float scale,
                                         const uint32_t* __restrict__ mask, float dscale) {
    constexpr int T = 64 * NT;
    float* st_lse = (float*)(smem + NT * 2 * TILE);
    float* st_del = st_lse + T;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = bh / H, hh = bh % H;
    const int64_t boff = (int64_t)b * T, ntile = mask_tiles(T);
    const float c2 = scale * LOG2E;
    const int kqs[2] = {32 * wave, 32 * (7 - wave)};
    const bf16_t* kb_ = k + boff * ld + hh * 64;
    const bf16_t* vb_ = v + boff * ld + hh * 64;
    const bool srow = tid < T;   // whole waves (T % 64 == 0)
    const int64_t sr = srow ? tid : 0;
    uint32_t lsew = 0u, delw = 0u;
    sv8 ov[2][4], dv_[2][4];   // O / dO row of query tid: halves h, columns 16 ks + 8 h .. +7
    if (srow) {
        gload4(lsew, lse + (int64_t)bh * T + sr);
        if constexpr (OD) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    gload16(ov[h][ks], o + (boff + sr) * ldo + hh * 64 + 16 * ks + 8 * h);
                    gload16(dv_[h][ks], dout + (boff + sr) * ldd + hh * 64 + 16 * ks + 8 * h);
                }
        } else {
            gload4(delw, delta + (int64_t)bh * T + sr);
        }
    }
    uint32_t mw[2][NT];
    if constexpr (DROP) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int kbw = kqs[p] >> 5, qtm = kbw >> 1;
            const bool ok = kqs[p] < T;
#pragma unroll
            for (int t = 0; t < NT; ++t) {   // tiles before the key group's first query tile re-read its first
                const int tt = ok && t >= qtm ? t - qtm : 0;
                gload4(mw[p][t], mask + ((int64_t)bh * ntile + mask_bwd_tile(ok ? kbw : 0, ok ? qtm : 0, NT)) * 64 +
                                     lane + tt * 64);
            }
        }
    }
    sv8 kf[4], vf[4];
    {
        const int key0 = (kqs[0] < T ? kqs[0] : 0) + (lane & 31);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            gload16(kf[ks], kb_ + (int64_t)key0 * ld + 16 * ks + 8 * (lane >> 5));
            gload16(vf[ks], vb_ + (int64_t)key0 * ld + 16 * ks + 8 * (lane >> 5));
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        dma_tile(q + boff * ld + hh * 64, ld, 64 * t, lds_base(smem) + 2u * t * TILE, wave, lane);
        dma_tile(dout + boff * ldd + hh * 64, ldd, 64 * t, lds_base(smem) + (2u * t + 1) * TILE, wave, lane);
    }
    // the second key group's K / V fragments behind the tiles (in flight until that group starts)
    sv8 kf1[4], vf1[4];
    {
        const int key1 = (kqs[1] < T ? kqs[1] : 0) + (lane & 31);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            gload16(kf1[ks], kb_ + (int64_t)key1 * ld + 16 * ks + 8 * (lane >> 5));
            gload16(vf1[ks], vb_ + (int64_t)key1 * ld + 16 * ks + 8 * (lane >> 5));
        }
    }
    asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(4 * (NT - 1) + 8) : "memory");
    asm volatile("" : "+v"(lsew), "+v"(delw));
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            asm volatile("" : "+v"(ov[h][ks]));
            asm volatile("" : "+v"(dv_[h][ks]));
        }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        asm volatile("" : "+v"(kf[ks]));
        asm volatile("" : "+v"(vf[ks]));
    }
    if constexpr (DROP) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int t = 0; t < NT; ++t) asm volatile("" : "+v"(mw[p][t]));
    } else {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int t = 0; t < NT; ++t) mw[p][t] = 0u;
    }
    if (srow) {
        st_lse[tid] = __uint_as_float(lsew) * LOG2E;
        float dsum;
        if constexpr (OD) {   // query tid: halves h = 0, 1 (columns 16 ks + 8 h + j) summed as dq_group_setup's lanes
            float sh[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float acc = 0.f;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc += bf2f((bf16_t)ov[h][ks][j]) * bf2f((bf16_t)dv_[h][ks][j]);
                sh[h] = acc;
            }
            dsum = sh[0] + sh[1];
        } else {
            dsum = __uint_as_float(delw);
        }
        st_del[tid] = -dsum / dscale;   // -delta' = -(1-p) delta
    }
    // the row statistics are visible to every wave, and tile 0 has landed for every wave
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    ATTN_STAMP(1, attn_now());
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int kq = kqs[p], key = kq + (lane & 31);
        const bool act = kq < T;
        if (p) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                asm volatile("" : "+v"(kf1[ks]));
                asm volatile("" : "+v"(vf1[ks]));
                kf[ks] = kf1[ks];
                vf[ks] = vf1[ks];
            }
        }
        fv16 dka[2] = {fv16{}, fv16{}}, dva[2] = {fv16{}, fv16{}};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (!p) res_tile_wait<NT, 8>(t);
            if (act && 64 * t + 63 >= kq)
                dkdv_tile<DROP>(smem + 2 * t * TILE, smem + (2 * t + 1) * TILE, st_lse + 64 * t, st_del + 64 * t,
                                64 * t, kq, key, kf, vf, mw[p][t], c2, dka, dva, lane);
        }
        if (act) {
            store_rows_wide(dk + (boff + key) * lddkv + hh * 64, dka, scale * dscale, lane);
            store_rows_wide(dv + (boff + key) * lddkv + hh * 64, dva, DROP ? dscale : 1.f, lane);
        }
    }
}

template <bool DROP, int NT>
__global__ __launch_bounds__(256, 2) void k_attn_dkdv_d64r(int H, const bf16_t* __restrict__ q,
                                                           const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                           int64_t ld, const bf16_t* __restrict__ dout, int64_t ldd,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, bf16_t* __restrict__ dk,
                                                           bf16_t* __restrict__ dv, int64_t lddkv, float scale,
                                                           const uint32_t* __restrict__ mask, float dscale) {
    __shared__ __attribute__((aligned(16))) char smem[NT * 2 * TILE + 2 * 64 * NT * 4];
    int x, bh;
    block_coords<false>(x, bh);
    dkdv_res<DROP, NT, false>(bh, smem, H, q, k, v, ld, dout, ldd, lse, delta, nullptr, 0, dk, dv, lddkv, scale, mask,
                       dscale);
}

// The whole T <= 256 backward in one launch: workgroup 2i computes dQ of (b, h) = i, 2i + 1 its
// dK/dV (with delta from O and dO itself, so the two do not depend on each other; DIN: both read
// delta, precomputed by the dO GEMM's epilogue, and neither loads O).  768
// workgroups fill the 512 slots and the second wave of them starts as slots free up, where the
// two separate 384-workgroup launches each ran 3/4 full and back to back.  The pair of one (b, h)
// stays on one XCD (block_coords: consecutive logical ids), sharing its K/V/Q/dO lines in L2.
template <bool DROP, int NT, bool DIN>
__global__ __launch_bounds__(256, 2) void k_attn_bwd_d64r(int H, const bf16_t* __restrict__ q,
                                                          const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                          int64_t ld, const bf16_t* __restrict__ o, int64_t ldo,
                                                          const bf16_t* __restrict__ dout, int64_t ldd,
                                                          const float* __restrict__ lse, float* __restrict__ delta,
                                                          bf16_t* __restrict__ dq, int64_t lddq, bf16_t* __restrict__ dk,
                                                          bf16_t* __restrict__ dv, int64_t lddkv, float scale,
                                                          const uint32_t* __restrict__ mask_fwd,
                                                          const uint32_t* __restrict__ mask_bwd, float dscale,
                                                          int lpt) {
    __shared__ __attribute__((aligned(16))) char smem[NT * 2 * TILE + 2 * 64 * NT * 4];
    ATTN_STAMP(0, attn_now());
    int x, id;
    const int n = (int)gridDim.y, w = (int)blockIdx.y;
    if (lpt && (n & 15) == 0) {
        // longest first within each XCD: the dispatcher deals workgroup w to XCD w & 7, in order of
        // w >> 3 there; each XCD owns n/16 consecutive (b, h) and runs all their dK/dV workgroups (22 us
        // at C2) before their dQ workgroups (16 us), so the 1.5-round grid's second round is dQ only
        const int half = n >> 4, xcd = w & 7, j = w >> 3, bh0 = xcd * half;
        id = j < half ? 2 * (bh0 + j) + 1 : 2 * (bh0 + j - half);
    } else {
        block_coords<false>(x, id);
    }
    if (id & 1)
        dkdv_res<DROP, NT, !DIN>(id >> 1, smem, H, q, k, v, ld, dout, ldd, lse, delta, o, ldo, dk, dv, lddkv, scale,
                                 mask_bwd, dscale);
    else
        dq_res<DROP, NT, DIN>(id >> 1, smem, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, mask_fwd,
                              dscale);
    ATTN_STAMP(2, attn_now());
    ATTN_STAMP(3, attn_where(id & 1));
}

// =====================================================================================
// Forward at T > 256 with an LDS-DMA K/V ring.  Same two-group software pipeline and per-tile
// arithmetic as fwd_qblock (identical bits), but K/V tiles arrive by LDS-DMA requested at the head
// of a tile (no staging VGPRs or ds_writes in the loop), so a tile has a whole tile of compute (QR:
// two) to land instead of the half tile the register staging gave it.  The keep words of tile kv + 1
// are hidden register loads issued just before the DMA, retired by the same counted wait.
//   QR = false: Q image in LDS (32 KB) + 3-slot ring (48 KB), tile kv + 1 requested at tile kv into
//               the slot tile kv - 2 used (B read V(kv - 2) during tile kv - 1);
//   QR = true:  the groups' Q fragments in registers (hidden loads) + 4-slot ring (64 KB), tile kv + 2
//               requested at tile kv.
// Both fit two blocks per CU.
// =====================================================================================
template <bool QR>
struct FwdRing {
    static constexpr int NSLOT = QR ? 4 : 3, AHEAD = QR ? 2 : 1;
    static constexpr int LDS = NSLOT * 2 * TILE + (QR ? 0 : 4 * TILE);
    static __device__ __forceinline__ int slot_of(int t) { return QR ? (t & 3) : (t + 3) % 3; }
};

// dma_tile with a uniform tile base and the per-lane byte offsets precomputed (dma_lane_offs): the
// same 8 wave-instructions, 2 per wave
__device__ __forceinline__ void dma_lane_offs(int64_t ldx, int wave, int lane, uint32_t (&off)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ins = 2 * wave + i, r = 8 * ins + (lane >> 3), c = (lane & 7) ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3));
        off[i] = (uint32_t)((r * ldx + 8 * c) * 2);
    }
}
// img as a 32-bit LDS byte address (lds_base of the kernel's __shared__ array + an integer offset):
// casting a generic slot pointer back to LDS per call made hipcc emit a null-pointer select -- and,
// once the forward ring kernel ran out of SGPRs, an illegal v_cmp on src_shared_base for it
__device__ __forceinline__ void dma_tile_s(const bf16_t* X, int64_t ldx, int64_t row0, const uint32_t (&off)[2],
                                           uint32_t img, int wave) {
    const bf16_t* base = X + row0 * ldx;
#pragma unroll
    for (int i = 0; i < 2; ++i) dma16sl(base, off[i], img + 1024 * (2 * wave + i));
}

__device__ __forceinline__ void qk_tile_reg(fv16 (&s)[2], const char* Ki, const sv8 (&qf)[4], int lane) {
    s[0] = fv16{};
    s[1] = fv16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        s[0] = mfma32(frag_row(Ki, 0, ks, lane), qf[ks], s[0]);
        s[1] = mfma32(frag_row(Ki, 32, ks, lane), qf[ks], s[1]);
    }
}

template <bool DROP, bool QR>
__device__ __forceinline__ void fwd_qblock_dma(int qblk, int bh, char* smem, int64_t T_, int H,
                                               const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                               const bf16_t* __restrict__ v, int64_t ld, bf16_t* __restrict__ o,
                                               int64_t ldo, float* __restrict__ lse, float scale_log2,
                                               const uint32_t* __restrict__ mask, float dscale) {
    using R = FwdRing<QR>;
    constexpr int AH = R::AHEAD;
    // tile kv + AH is requested at tile kv: 4 DMA instructions per wave stay in flight at its end
    // when AH = 2 (tile kv + 1 must have landed), none when AH = 1
    constexpr int NWAIT = AH == 2 ? 4 : 0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = (int)T_, b = bh / H, hh = bh % H;
    const int Q0 = qblk * 256;
    const int64_t boff = (int64_t)b * T_, ntile = mask_tiles(T_);
    const bf16_t* kb_ = k + boff * ld + hh * 64;
    const bf16_t* vb_ = v + boff * ld + hh * 64;
    const bf16_t* qb_ = q + boff * ld + hh * 64;
    char* const Qimg = smem + R::NSLOT * 2 * TILE;   // !QR only
    const int qg[2] = {Q0 + 32 * (7 - wave), Q0 + 32 * wave};   // g = 0 (A): the longer causal prefix
    const int qr[2] = {32 * (7 - wave), 32 * wave};             // the groups' rows in the Q image
    const bool act[2] = {qg[0] < T, qg[1] < T};
    uint32_t doff[2];   // per-lane DMA byte offsets (K, V and Q share ld and the image layout)
    dma_lane_offs(ld, wave, lane, doff);
    auto slot = [&](int t) { return smem + R::slot_of(t) * 2 * TILE; };
    const uint32_t lds0 = lds_base(smem);
    auto lslot = [&](int t) { return lds0 + (uint32_t)(R::slot_of(t) * 2 * TILE); };
    // keep words of (group, key tile t) at mrow[g] + 64 t + lane (uniform bases, one lane offset); an
    // inactive group reads block 0's (unused)
    const uint32_t* mrow[2];
    const uint32_t loff = 4u * lane;
    sv8 qf[2][4];
    uint32_t mw[2] = {0u, 0u};
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        mrow[g] = mask + ((int64_t)bh * ntile + mask_fwd_tile(act[g] ? qg[g] >> 5 : 0, 0)) * 64;
        if constexpr (QR) {
            const int qa = (act[g] ? qg[g] : 0) + (lane & 31);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) gload16(qf[g][ks], qb_ + (int64_t)qa * ld + 16 * ks + 8 * (lane >> 5));
        }
        if constexpr (DROP) gload4s(mw[g], mrow[g], loff);
    }
    const int qlast = (Q0 + 255 < T - 1) ? Q0 + 255 : T - 1;
    const int nkv = qlast / 64 + 1;
    const int npipe = act[1] ? (qg[1] + 31) / 64 : 0;   // B's diagonal tile: first unpipelined tile
    {   // the V half of tile -1's slot is the pipeline head's "previous tile": zeros
        const int r = tid >> 3, c = tid & 7;
        *(uint4*)(slot(-1) + TILE + aoff(r, c)) = make_uint4(0, 0, 0, 0);
        *(uint4*)(slot(-1) + TILE + aoff(r + 32, c)) = make_uint4(0, 0, 0, 0);
    }
    if constexpr (!QR) {   // Q image: the block's 64-row tiles by LDS-DMA, rows past T zero
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (Q0 + 64 * t < T) {
                dma_tile_s(qb_, ld, Q0 + 64 * t, doff, lds0 + (uint32_t)(R::NSLOT * 2 * TILE + t * TILE), wave);
            } else {
                const int r = tid >> 3, c = tid & 7;
                *(uint4*)(Qimg + t * TILE + aoff(r, c)) = make_uint4(0, 0, 0, 0);
                *(uint4*)(Qimg + t * TILE + aoff(r + 32, c)) = make_uint4(0, 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < AH; ++t) {
        if (t < nkv) {
            dma_tile_s(kb_, ld, (int64_t)t * 64, doff, lslot(t), wave);
            dma_tile_s(vb_, ld, (int64_t)t * 64, doff, lslot(t) + TILE, wave);
        }
    }
    ring_wait<NWAIT>(AH == 2 && nkv > 1);   // the register loads, Q and tile 0 have landed
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if constexpr (QR) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(qf[g][ks]));
        }
        asm volatile("" : "+v"(mw[g]));
    }
    if constexpr (!DROP) mw[0] = mw[1] = 0u;
    auto qk = [&](fv16 (&s)[2], const char* Ki, int g) {
        if constexpr (QR) qk_tile_reg(s, Ki, qf[g], lane);
        else qk_tile(s, Ki, Qimg, qr[g], lane);
    };
    fv16 oacc[2][2];
#pragma unroll
    for (int g = 0; g < 2; ++g) oacc[g][0] = oacc[g][1] = fv16{};
    float m_run[2] = {-FLT_MAX, -FLT_MAX};
    fv4 l_run[2] = {fv4{}, fv4{}};
    const sv8 ones = rowsum_ones(lane);
    fv16 sA[2], sB[2] = {fv16{} - INFINITY, fv16{} - INFINITY};
    sv8 pfA[2][2], pfB[2][2];
    uint32_t mwBp = 0u;   // B's keep word of the previous tile
    int kv = 0;
    for (; kv < npipe; ++kv) {
        uint32_t mn[2] = {0u, 0u};   // tile kv + 1 <= npipe: both groups full through it
        if constexpr (DROP) {
            gload4s(mn[0], mrow[0] + (kv + 1) * 64, loff);
            gload4s(mn[1], mrow[1] + (kv + 1) * 64, loff);
        }
        const bool pf = kv + AH < nkv;
        if (pf) {
            dma_tile_s(kb_, ld, (int64_t)(kv + AH) * 64, doff, lslot(kv + AH), wave);
            dma_tile_s(vb_, ld, (int64_t)(kv + AH) * 64, doff, lslot(kv + AH) + TILE, wave);
        }
        const char* Ki = slot(kv);
        const char* Vi = Ki + TILE;
        const char* Vp = slot(kv - 1) + TILE;
        // at kv = 0, B's "previous tile" is sB = -inf against the zeroed V slot: it adds exactly 0
        qk(sA, Ki, 0);
        softmax_pack<DROP>(sB, scale_log2, m_run[1], l_run[1], mwBp, pfB, ones);
        pv_tile(oacc[1], Vp, pfB, lane);
        rescale_if(tile_max(sA) * scale_log2, m_run[0], l_run[0], oacc[0]);
        qk(sB, Ki, 1);
        softmax_pack<DROP>(sA, scale_log2, m_run[0], l_run[0], mw[0], pfA, ones);
        pv_tile(oacc[0], Vi, pfA, lane);
        rescale_if(tile_max(sB) * scale_log2, m_run[1], l_run[1], oacc[1]);
        ring_wait<NWAIT>(pf);
        if constexpr (DROP) asm volatile("" : "+v"(mn[0]), "+v"(mn[1]));
        mwBp = mw[1];
        mw[0] = mn[0];
        mw[1] = mn[1];
    }
    if (npipe > 0) {   // pipeline tail: B's pending tile npipe - 1 (its V still in that tile's slot)
        softmax_pack<DROP>(sB, scale_log2, m_run[1], l_run[1], mwBp, pfB, ones);
        pv_tile(oacc[1], slot(npipe - 1) + TILE, pfB, lane);   // the tail requests kv + AH: another slot
    }
    for (; kv < nkv; ++kv) {
        uint32_t mn[2] = {0u, 0u};
        const int nxt = kv + 1 < nkv ? kv + 1 : kv;
        if constexpr (DROP) {
#pragma unroll
            for (int g = 0; g < 2; ++g)   // past a group's diagonal: re-read its tile 0 (unused)
                gload4s(mn[g], mrow[g] + (act[g] && nxt * 64 <= qg[g] + 31 ? nxt : 0) * 64, loff);
        }
        const bool pf = kv + AH < nkv;
        if (pf) {
            dma_tile_s(kb_, ld, (int64_t)(kv + AH) * 64, doff, lslot(kv + AH), wave);
            dma_tile_s(vb_, ld, (int64_t)(kv + AH) * 64, doff, lslot(kv + AH) + TILE, wave);
        }
        const char* Ki = slot(kv);
        const char* Vi = Ki + TILE;
        const int k0 = kv * 64;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (!act[g] || k0 > qg[g] + 31) continue;
            const int rel = __builtin_amdgcn_readfirstlane(qg[g] - k0);
            if constexpr (QR) {
                if (rel >= 64)
                    fwd_group_tile<DROP, 2, -1, true>(Ki, Vi, nullptr, 0, lane, scale_log2, m_run[g], l_run[g],
                                                      oacc[g], mw[g], ones, qf[g]);
                else if (rel == 32)
                    fwd_group_tile<DROP, 2, 1, true>(Ki, Vi, nullptr, 0, lane, scale_log2, m_run[g], l_run[g],
                                                     oacc[g], mw[g], ones, qf[g]);
                else
                    fwd_group_tile<DROP, 1, 0, true>(Ki, Vi, nullptr, 0, lane, scale_log2, m_run[g], l_run[g],
                                                     oacc[g], mw[g], ones, qf[g]);
            } else {
                if (rel >= 64)
                    fwd_group_tile<DROP, 2, -1>(Ki, Vi, Qimg, qr[g], lane, scale_log2, m_run[g], l_run[g], oacc[g],
                                                mw[g], ones);
                else if (rel == 32)
                    fwd_group_tile<DROP, 2, 1>(Ki, Vi, Qimg, qr[g], lane, scale_log2, m_run[g], l_run[g], oacc[g],
                                               mw[g], ones);
                else
                    fwd_group_tile<DROP, 1, 0>(Ki, Vi, Qimg, qr[g], lane, scale_log2, m_run[g], l_run[g], oacc[g],
                                               mw[g], ones);
            }
        }
        ring_wait<NWAIT>(pf);
        if constexpr (DROP) asm volatile("" : "+v"(mn[0]), "+v"(mn[1]));
        mw[0] = mn[0];
        mw[1] = mn[1];
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (!act[g]) continue;
        const float lt = l_run[g][0];   // every accumulator register holds query lane & 31's sum
        const int64_t qa = qg[g] + (lane & 31);
        store_rows_wide(o + (boff + qa) * ldo + hh * 64, oacc[g], dscale / lt, lane);
        if (lane < 32) lse[(int64_t)bh * T_ + qa] = (m_run[g] + __log2f(lt)) * LN2;
    }
}

template <bool DROP, bool QR>
__global__ __launch_bounds__(256, 2) void k_attn_fwd_d64d(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                          const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                          int64_t ld, bf16_t* __restrict__ o, int64_t ldo,
                                                          float* __restrict__ lse, float scale_log2,
                                                          const uint32_t* __restrict__ mask, float dscale) {
    __shared__ __attribute__((aligned(16))) char smem[FwdRing<QR>::LDS];
    int x, bh;
    block_coords<false>(x, bh);
    const int nq = (int)((T_ + 255) / 256), first = nq - 1 - x;
    const int npass = x == first ? 1 : 2;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
        if (pass) __syncthreads();
        fwd_qblock_dma<DROP, QR>(pass ? x : first, bh, smem, T_, H, q, k, v, ld, o, ldo, lse, scale_log2, mask,
                                 dscale);
    }
}

}  // namespace

#ifdef CG_AB_VARIANTS
namespace attn_ab {
// ab/attention_ab.hip: the measured-slower attention variants, selected by cg_set_tuning("attn_variant");
// each returns false when the variant does not apply (the product kernel then runs)
bool launch_fwd(int variant, dim3 grid, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v,
                int64_t ld, bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st);
bool launch_dq(int variant, dim3 grid, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v,
               int64_t ld, const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse,
               float* delta, bf16_t* dq, int64_t lddq, float scale, const DropArgs& d, hipStream_t st);
bool launch_dkdv(int variant, dim3 grid, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v,
                 int64_t ld, const bf16_t* dout, int64_t ldd, const float* lse, const float* delta, bf16_t* dk,
                 bf16_t* dv, int64_t lddkv, float scale, const DropArgs& d, hipStream_t st);
}  // namespace attn_ab
#endif

}  // namespace cg
