// charpt: persistent LDS-DMA bf16 MFMA GEMM (gfx950) -- the default kernel behind cg_gemm for the
// nn.Linear forward / dgrad / wgrad products of GPT1.py:111-112,121,136,143,145.
//
// Measured on MI355X (tools/gemm_diag.hip): with one 128x128 tile per block, a K=384 launch spends
// ~0.7 us waiting for its first K-tile and ~2.5 us in an LDS-staged epilogue against ~3 us of
// MFMA loop.  This kernel removes both:
//  * persistent blocks (grid = resident slots) walk a flattened (item, K-tile) sequence; the
//    LDS-DMA stream (global_load_lds_dwordx4, NBUF stages, NBUF-1 tiles in flight) runs straight
//    across item boundaries, so the next item's first tiles land while this item finishes;
//  * the MFMA operands are swapped (D = B_tile x A_tile^T), so each lane's accumulator holds four
//    consecutive output COLUMNS of one row: bias / ReLU / Philox dropout (exactly one Philox group
//    per 4 columns) / residual / ReLU-backward are applied in registers and stored as one 8-B
//    (bf16) or 16-B (fp32) store -- no LDS staging, no epilogue barriers.
// An item is one BM x BN output tile of one K-split; items are ordered split-major and remapped
// so that consecutive items (same row panel / same split) share an XCD's L2.
#include "gemm_tile.h"

#ifdef CG_PK_STAMPS
// Diagnostic build only (tools/gemm_stamps.py, make stamps): per-wave s_memtime cycle sums of the
// K-step segments of k_gemm_pk -- [0] the head wait (vmcnt + barrier), [1] fragment reads + MFMA
// and DMA issue, [2] item epilogues, [3] K-steps, [4] whole wave, [5] s_memrealtime ticks of the
// wave (100 MHz) -- summed over all waves.  Never in the product library.
__device__ unsigned long long g_pk_stamps[8];
__device__ __forceinline__ uint64_t pk_clk() { return __builtin_amdgcn_s_memtime(); }
extern "C" int cg_debug_pk_stamps(unsigned long long* host8) {
    return hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_pk_stamps), 8 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
extern "C" int cg_debug_pk_stamps_reset() {
    unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pk_stamps), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
#define PK_STAMP(v) const uint64_t v = pk_clk()
#else
#define PK_STAMP(v)
#endif

#ifdef CG_PK_BOUNDS
// Diagnostic build only (make bounds; tools/gemm_bounds.py): every LDS-DMA source chunk of k_gemm_pk
// (the past-the-end reloads included) is checked against its operand's extent, every item's output
// tile / split-K slab against the problem, and -- check-only, nothing issued -- the address stream of
// round 3's L2-prefetch trial (commit db80795: one 128-B line per lane of K-tile g + 1 + PF, bytes 0
// and 64), for PF = 1..3.  Counts: [0] A DMA, [1] B DMA, [2] item tile / slab, [3..5] prefetch PF = 1..3.
// Violations are added by the offending lanes (vector atomics); never in the product library.
__device__ unsigned long long g_pk_bounds[8];
extern "C" int cg_debug_pk_bounds(unsigned long long* host8) {
    return hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_pk_bounds), 8 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
extern "C" int cg_debug_pk_bounds_reset() {
    unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pk_bounds), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
__device__ __forceinline__ void bounds_chk(const void* p, int bytes, const void* lo, const void* hi, int slot) {
    if ((const char*)p < (const char*)lo || (const char*)p + bytes > (const char*)hi) atomicAdd(&g_pk_bounds[slot], 1ull);
}
#endif

namespace cg {
int g_pk_flags = 0;  // cg_set_tuning("pk_flags"): bit 0 = drain epilogue stores each step, bit 1 = per-fragment epilogue
namespace {
using namespace gt;

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// per-lane part of one operand's LDS-DMA sources: R rows (K-contiguous) or R columns (TR) x BK k
template <bool TR, int R, int WAVES, int BK>
struct DmaP {
    static constexpr int INSTR = R * BK * 2 / 1024;  // 1-KB wave instructions per K-tile
    static constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(PER_WAVE * WAVES == INSTR, "tile/wave mismatch");
    static_assert(!TR || R >= 128, "transposed image swizzle needs >= 16 chunks per row");
    uint32_t off[PER_WAVE];  // byte offset of this lane's 16-B chunk from the tile origin
    int64_t kstep;
#ifdef CG_PK_BOUNDS
    const void* lo = nullptr;
    const void* hi = nullptr;
    int slot = 0;
#endif

    __device__ __forceinline__ void init(int64_t ld, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) {
            const int pos = (wave * PER_WAVE + i) * 1024 + lane * 16;
            if (!TR) {
                const int r = BK == 64 ? pos >> 7 : pos >> 6;
                const int c = BK == 64 ? ((pos >> 4) & 7) ^ row_swz(r) : ((pos >> 4) & 3) ^ row_swz32(r);
                off[i] = 2u * (uint32_t)((int)(r * ld) + c * 8);
            } else {
                const int k = pos / (2 * R), c = ((pos % (2 * R)) >> 4) ^ col_swz(k);
                off[i] = 2u * (uint32_t)((int)(k * ld) + c * 8);
            }
        }
        kstep = TR ? (int64_t)BK * ld : (int64_t)BK;
    }
    // instruction i (0..PER_WAVE-1) of one K-tile, from that K-tile's (wave-uniform) base address into
    // the image at 32-bit LDS address img: the saddr form (SGPR base + per-lane byte offset) and an
    // SGPR LDS address.  With a generic image pointer and a 64-bit lane address hipcc spent ~6
    // instructions per DMA (two 64-bit VALU adds, two v_readfirstlane, a null-pointer select) on a
    // VALU -> SGPR -> m0 dependency chain.
    __device__ __forceinline__ void issue1(const bf16_t* base, int i, uint32_t img, int wave) const {
#ifdef CG_PK_BOUNDS
        bounds_chk((const char*)base + off[i], 16, lo, hi, slot);
#endif
        dma16sl(base, off[i], img + (uint32_t)((wave * PER_WAVE + i) * 1024));
    }
};

__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

__device__ __forceinline__ void store4_plain(const fv4& v, int64_t m, int64_t n, void* Cv, int c_dtype, int64_t ldc) {
    if (c_dtype == CG_BF16)
        *(uint2*)((bf16_t*)Cv + m * ldc + n) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    else
        st_out16((float4*)((float*)Cv + m * ldc + n), make_float4(v[0], v[1], v[2], v[3]));
}

// Dropout keep bits of a wave's 64x64 item fragment, 4 per (i, j) -- bit q <-> column
// nc + 16 j + q of row mr + 16 i.  Lanes l and l ^ 16 hold the two 4-column halves of the same
// 8-element Philox group (same row, columns 8k..8k+7), so each evaluates 8 of the 16 groups (j in
// {0,1} or {2,3}) and the pair trades bytes with one lane swap per j half: half the Philox calls
// of one keep4_bits per fragment, same bits.
__device__ __forceinline__ void drop_nibbles(const EpiArgs& epi, uint64_t stream, int64_t mr, int64_t nc, int64_t N,
                                             uint32_t (&nib)[4][4]) {
    const int lane = threadIdx.x & 63;
    const uint32_t odd = (lane >> 4) & 1;
    const int64_t c8 = nc & ~(int64_t)7;
    uint32_t mine[2] = {0u, 0u};
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t idx = (uint64_t)(mr + 16 * i) * (uint64_t)N + (uint64_t)(c8 + 16 * (2 * odd + jj));
            mine[jj] |= keep8_bits(philox_group(epi.seed, stream, idx >> 3), epi.thr) << (8 * i);
        }
    uint32_t other[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) other[jj] = (uint32_t)__shfl_xor((int)mine[jj], 16, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t w = ((uint32_t)(j >> 1) == odd) ? mine[j & 1] : other[j & 1];
            nib[i][j] = (w >> (8 * i + 4 * odd)) & 0xfu;
        }
}

// The item's 16 output fragments.  WIDE with a bf16 output: 16-B row segments instead of 8-B ones --
// for each fragment pair (j, j+1) lanes of rows 1 and 3 (lane >> 4 odd) trade their fragment-j
// quarter for the other row's fragment-(j+1) quarter (v_permlane16_swap: odd 16-lane rows of vdst
// <-> even rows of src), so lane quarter q then holds 8 contiguous columns: 8 dwordx4 stores, each
// writing 64 contiguous bytes of 16 rows, instead of 16 dwordx2 (cdna_hip_programming.md T21).
template <bool WIDE>
__device__ __forceinline__ void store_item(const fv4 (&v)[4][4], int64_t mr, int64_t nc, void* Cv, int c_dtype,
                                           int64_t ldc) {
    if (WIDE && c_dtype == CG_BF16) {   // 16-B row segments (gemm_tile.h store_bf16_wide): 8 stores
        store_bf16_wide<4>(v, (bf16_t*)Cv, ldc, mr, nc);
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) store4_plain(v[i][j], mr + 16 * i, nc + 16 * j, Cv, c_dtype, ldc);
}

// The whole 64x64 epilogue of one wave: every operand it reads (bias, residual, ReLU output) is
// loaded for all 16 fragments before the first store.  Per-fragment load -> use made hipcc wait
// vmcnt(0) 16 times per item, each time also for the previous fragments' stores and the next
// K-tile's DMA (measured: +10 us on the C2 FFN1 bias+ReLU forward, +14 us on the ReLU-backward
// dgrad).  Arithmetic and order are exactly epi_store4's; beta != 0 keeps the per-fragment form.
// EK >= 0: the epilogue kind fixed at compile time (CG_EPI_*; dispatch guarantees beta == 0 and the
// kind's bias / residual pointers non-NULL), EK < 0: every kind at run time.
template <int EK>
__device__ __forceinline__ void epi_item(fv4 (&acc)[4][4], int64_t mr, int64_t nc, int64_t N, void* Cv, int c_dtype,
                                         int64_t ldc, const EpiArgs& epi, uint64_t stream) {
    const int kind = EK >= 0 ? EK : epi.kind;
    // the fixed kinds' output dtype (launch_ek dispatches them only with it): no per-fragment branch
    constexpr int OUT = (EK == CG_EPI_BIAS_RESID || EK == CG_EPI_BIAS_DROP_RESID) ? CG_F32
                        : (EK == CG_EPI_BIAS_RELU || EK == CG_EPI_RELU_BWD)   ? CG_BF16
                                                                              : -1;
    if constexpr (OUT >= 0) c_dtype = OUT;
    constexpr bool WIDE = EK == CG_EPI_STORE || EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_RELU_BWD;
    if constexpr (EK == CG_EPI_STORE_ROWDOT) {
        // bf16(acc) stored, and per row the dot of those rounded values with O's row over this wave's
        // 64 columns (one head): lane l holds columns 16j + 4(l >> 4) + q of rows 16i + (l & 15), so
        // 16 products per lane, then the 4 lane quarters (xor 16, 32); quarter 0 writes 4 rows' delta.
        // These 4 stores precede the item's 8 output stores (EPI_OPS = 12).
        const int lane = threadIdx.x & 63;
        uint2 o[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) o[i][j] = *(const uint2*)((const bf16_t*)epi.aux + (mr + 16 * i) * epi.ld_aux + nc + 16 * j);
        float dsum[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const fv4& v = acc[i][j];
                s += rbf(v[0]) * __uint_as_float(o[i][j].x << 16);
                s += rbf(v[1]) * __uint_as_float(o[i][j].x & 0xffff0000u);
                s += rbf(v[2]) * __uint_as_float(o[i][j].y << 16);
                s += rbf(v[3]) * __uint_as_float(o[i][j].y & 0xffff0000u);
            }
            s += __shfl_xor(s, 16, 64);
            s += __shfl_xor(s, 32, 64);
            dsum[i] = s;
        }
        const int64_t T = epi.ld_resid, H = N >> 6, h = (nc - 4 * (lane >> 4)) >> 6;
        if (lane < 16) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t m = mr + 16 * i, b = m / T;
                epi.colpart[(b * H + h) * T + (m - b * T)] = dsum[i];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        store_item<true>(acc, mr, nc, Cv, CG_BF16, ldc);
        return;
    }
    if (EK < 0 && epi.beta != 0.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) epi_store4(acc[i][j], mr + 16 * i, nc + 16 * j, N, Cv, c_dtype, ldc, epi, stream);
        return;
    }
    if (kind == CG_EPI_RELU_BWD) {
        if (epi.aux_dtype == CG_BF16 || epi.aux_dtype == CG_BITS) {
            if (epi.aux_dtype == CG_BITS) {   // keep bits: one 8-B word pair per row instead of 4 x 8 B of bf16
                const int lane = threadIdx.x & 63;
                uint2 w[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    w[i] = *(const uint2*)((const uint32_t*)epi.aux + (mr + 16 * i) * epi.ld_aux + ((nc - 4 * (lane >> 4)) >> 5));
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t kb = relu_nib(w[i], j, lane);
                        fv4& v = acc[i][j];
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = ((kb >> q) & 1u) ? v[q] : 0.f;
                    }
            } else {
                uint2 h[4][4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        h[i][j] = *(const uint2*)((const bf16_t*)epi.aux + (mr + 16 * i) * epi.ld_aux + nc + 16 * j);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        fv4& v = acc[i][j];
                        v[0] = __uint_as_float(h[i][j].x << 16) > 0.f ? v[0] : 0.f;
                        v[1] = __uint_as_float(h[i][j].x & 0xffff0000u) > 0.f ? v[1] : 0.f;
                        v[2] = __uint_as_float(h[i][j].y << 16) > 0.f ? v[2] : 0.f;
                        v[3] = __uint_as_float(h[i][j].y & 0xffff0000u) > 0.f ? v[3] : 0.f;
                    }
            }
            if (epi.colpart) {
                // the consumer's bias gradient, fused: column sums of this wave's 64 rows (rows
                // 16i + lane&15 of each column 16j + 4(lane>>4) + q: 4 rows per lane, then a
                // DPP row sum over the 16 lanes of the column group), lane r = 0 of each group writes.
                // These stores precede the item's 16 output stores, which stay the youngest
                // EPI_OPS vector-memory operations the main loop's wait counts assume.
                const int lane = threadIdx.x & 63;
                float* cp = epi.colpart + ((mr - (lane & 15)) >> 6) * N + nc;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    fv4 t;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        // the bf16-rounded values the stores below write (the precision cg_colsum
                        // and the W1 weight gradient see), summed in fp32
                        const float s = ((rbf(acc[0][j][q]) + rbf(acc[1][j][q])) + rbf(acc[2][j][q])) + rbf(acc[3][j][q]);
                        t[q] = row16_sum_dpp(s);   // the 16 lanes of the column group = one DPP row
                    }
                    if ((lane & 15) == 0) *(fv4*)(cp + 16 * j) = t;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            store_item<WIDE>(acc, mr, nc, Cv, c_dtype, ldc);
        } else {
            float4 h[4][4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    h[i][j] = *(const float4*)((const float*)epi.aux + (mr + 16 * i) * epi.ld_aux + nc + 16 * j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    fv4 v = acc[i][j];
                    v[0] = h[i][j].x > 0.f ? v[0] : 0.f;
                    v[1] = h[i][j].y > 0.f ? v[1] : 0.f;
                    v[2] = h[i][j].z > 0.f ? v[2] : 0.f;
                    v[3] = h[i][j].w > 0.f ? v[3] : 0.f;
                    store4_plain(v, mr + 16 * i, nc + 16 * j, Cv, c_dtype, ldc);
                }
        }
        return;
    }
    const bool has_bias = EK >= 0 ? (EK >= CG_EPI_BIAS && EK <= CG_EPI_BIAS_DROP_RESID) : (kind != CG_EPI_STORE && epi.bias);
    float4 bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = has_bias ? *(const float4*)(epi.bias + nc + 16 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
    const bool has_resid = (kind == CG_EPI_BIAS_RESID || kind == CG_EPI_BIAS_DROP_RESID) && (EK >= 0 || epi.resid);
    if (has_resid) {
        float4 r[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) r[i][j] = *(const float4*)(epi.resid + (mr + 16 * i) * epi.ld_resid + nc + 16 * j);
        const bool drop = kind == CG_EPI_BIAS_DROP_RESID && (EK == CG_EPI_BIAS_DROP_RESID || epi.thr);
        uint32_t nib[4][4];
        if (drop) drop_nibbles(epi, stream, mr, nc, N, nib);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t m = mr + 16 * i, n = nc + 16 * j;
                fv4 v = acc[i][j];
                if (has_bias) {
                    v[0] += bv[j].x; v[1] += bv[j].y; v[2] += bv[j].z; v[3] += bv[j].w;
                }
                if (drop) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = ((nib[i][j] >> q) & 1u) ? v[q] * epi.dscale : 0.f;
                }
                v[0] = r[i][j].x + v[0]; v[1] = r[i][j].y + v[1]; v[2] = r[i][j].z + v[2]; v[3] = r[i][j].w + v[3];
                store4_plain(v, m, n, Cv, c_dtype, ldc);
            }
        return;
    }
    if (kind == CG_EPI_BIAS_RELU && epi.aux_dtype == CG_BITS) {   // bf16 output + its ReLU keep bits
        const int lane = threadIdx.x & 63;
        uint32_t kb[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                fv4& v = acc[i][j];
                v[0] = fmaxf(v[0] + bv[j].x, 0.f); v[1] = fmaxf(v[1] + bv[j].y, 0.f);
                v[2] = fmaxf(v[2] + bv[j].z, 0.f); v[3] = fmaxf(v[3] + bv[j].w, 0.f);
                kb[i][j] = nz4_bf16(make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])));
            }
        store_item<WIDE>(acc, mr, nc, Cv, CG_BF16, ldc);
        relu_bits_store<4>(kb, (uint32_t*)epi.aux, epi.ld_aux, mr, nc - 4 * (lane >> 4), lane);
        return;
    }
    const bool drop = kind == CG_EPI_BIAS_DROP_RESID && epi.thr;
    uint32_t nib[4][4];
    if (drop) drop_nibbles(epi, stream, mr, nc, N, nib);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            fv4& v = acc[i][j];
            if (has_bias) {
                v[0] += bv[j].x; v[1] += bv[j].y; v[2] += bv[j].z; v[3] += bv[j].w;
            }
            if (kind == CG_EPI_BIAS_RELU) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
            } else if (drop) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = ((nib[i][j] >> q) & 1u) ? v[q] * epi.dscale : 0.f;
            }
        }
    store_item<WIDE>(acc, mr, nc, Cv, c_dtype, ldc);
}

// The fp32 residual epilogues (CG_EPI_BIAS_RESID, CG_EPI_BIAS_DROP_RESID) of a 64 x 16NJ wave tile:
// epi_item's arithmetic and order (bias, dropout, residual), operands loaded before the first store.
template <int EK, int NJ>
__device__ __forceinline__ void epi_resid_nj(fv4 (&acc)[4][NJ], int64_t mr, int64_t nc, int64_t N, float* C, int64_t ldc,
                                             const EpiArgs& epi, uint64_t stream) {
    static_assert(EK == CG_EPI_BIAS_RESID || EK == CG_EPI_BIAS_DROP_RESID, "residual kinds only");
    float4 bv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bv[j] = *(const float4*)(epi.bias + nc + 16 * j);
    float4 r[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) r[i][j] = *(const float4*)(epi.resid + (mr + 16 * i) * epi.ld_resid + nc + 16 * j);
    uint32_t nib[4][NJ];
    if constexpr (EK == CG_EPI_BIAS_DROP_RESID) drop_nibbles_rows<NJ>(epi, stream, mr, nc, N, nib);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            fv4 v = acc[i][j];
            v[0] += bv[j].x; v[1] += bv[j].y; v[2] += bv[j].z; v[3] += bv[j].w;
            if constexpr (EK == CG_EPI_BIAS_DROP_RESID) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = ((nib[i][j] >> q) & 1u) ? v[q] * epi.dscale : 0.f;
            }
            v[0] = r[i][j].x + v[0]; v[1] = r[i][j].y + v[1]; v[2] = r[i][j].z + v[2]; v[3] = r[i][j].w + v[3];
            st_out16((float4*)(C + (mr + 16 * i) * ldc + nc + 16 * j), make_float4(v[0], v[1], v[2], v[3]));
        }
}

// Wave grid: 64 x 64 wave tiles, except BN = 96 (two 64 x 48 wave tiles per 64-row band: NJ = 3
// fragments of 16 columns instead of 4).
template <int BM, int BN, int NBUF, int BK = FBK>
struct GeoP {
    static constexpr int WM = BM / 64, WN = BN == 96 ? 2 : BN / 64, WAVES = WM * WN, THREADS = WAVES * 64;
    static constexpr int WTN = BN / WN, NJ = WTN / 16;   // wave tile columns, 16-column fragments per wave
    static_assert(WTN == 64 || WTN == 48, "wave tile");
    static constexpr int IMG_A = BM * BK * 2, IMG_B = BN * BK * 2, STAGE = IMG_A + IMG_B;
    static constexpr int LDS = NBUF * STAGE;
    static constexpr int OCC_LDS = (160 * 1024) / LDS;
    static constexpr int OCC = OCC_LDS > 4 ? 4 : (OCC_LDS < 1 ? 1 : OCC_LDS);  // resident blocks per CU (LDS-bound)
    static constexpr int WPE = (WAVES * OCC + 3) / 4;   // waves per SIMD
};

// EK: the item epilogue.  EK_SLAB = split-K (split_k > 1, fp32 slab stores only), 0..5 = one
// CG_EPI_* kind fixed at compile time, EK_ANY = every kind, beta and the per-fragment form at run
// time.  The run-time epilogue's conditional loads (bias present or not, residual, ReLU-backward aux,
// beta) leave the compiler's wait-count state with a load it cannot retire at the loop head, and it
// puts s_waitcnt vmcnt(0) before every K-tile's fragment reads -- waiting for the item's output
// stores and, with the DMAs hidden from it (common.h dma16), for the prefetched stages too.  The
// fixed-kind and slab instantiations have no such wait.
#ifndef CG_PK_DPG
#define CG_PK_DPG 1   // next-stage DMA instructions issued per group of 4 MFMAs
#endif
constexpr int EK_ANY = -1, EK_SLAB = 6, EK_SLAB16 = 8;   // 7: CG_EPI_STORE_ROWDOT
// BK: K depth of one LDS stage, 64 or 32 (32: the same 64 KB per block holds 4 stages, 3 K-tiles in
// flight at two blocks per CU; same bits -- kchunk stays a multiple of 64, same k order.  Measured
// 10-15 % slower on every C2 shape: 64-B row segments double the TA/TCP requests,
// profiles/r3_gemm_bk32.txt -- no launcher instantiates it)
// amdgpu_waves_per_eu: LDS caps residency at OCC blocks, so tell the scheduler the real occupancy;
// left at its default it schedules for 8+ waves/SIMD, keeps ONE A fragment register and waits
// lgkmcnt(0) before every 4 MFMAs (LDS latency exposed 8x per K-tile)
template <bool AT, bool BT, int BM, int BN, int NBUF, int EK, int BK>
__global__ __launch_bounds__((GeoP<BM, BN, NBUF, BK>::THREADS), (GeoP<BM, BN, NBUF, BK>::OCC))
__attribute__((amdgpu_waves_per_eu(1, GeoP<BM, BN, NBUF, BK>::WPE)))
void k_gemm_pk(int64_t M, int64_t N, int64_t K, const bf16_t* __restrict__ A, int64_t lda,
               const bf16_t* __restrict__ B, int64_t ldb, void* __restrict__ Cv, int c_dtype, int64_t ldc,
               EpiArgs epi, int split_k, int64_t kchunk, float* __restrict__ ws, int flags, RedJobs red) {
    static_assert(BK == 64 || BK == 32, "BK");
    constexpr int NS = BK / 32;   // 32-deep MFMA slices per K-tile
    using G = GeoP<BM, BN, NBUF, BK>;
    constexpr int NJ = G::NJ, WTN = G::WTN;
    static_assert(NJ == 4 || (!BT && (EK == CG_EPI_BIAS_RESID || EK == CG_EPI_BIAS_DROP_RESID)),
                  "48-column wave tiles: the fp32 residual kinds with a K-contiguous B only");
    using DA = DmaP<AT, BM, G::WAVES, BK>;
    using DB = DmaP<BT, BN, G::WAVES, BK>;
    constexpr int LPT = DA::PER_WAVE + DB::PER_WAVE;  // DMA instructions per thread per K-tile
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / G::WN, wn = wave % G::WN;
    const int tilesN = (int)(N / BN);
    const int ntiles = (int)(M / BM) * tilesN;
    const int nitems = ntiles * split_k;
    // split s covers K-tiles [s*nkc, min((s+1)*nkc, nkt)): the last split may be shorter (uneven
    // split-K: any split count, not only divisors of the K-tile count)
    const int nkt = (int)(K / BK), nkc = (int)(kchunk / BK);
    const int P = gridDim.x, b = blockIdx.x;
    const int my_items = b < nitems ? (nitems - 1 - b) / P + 1 : 0;
    auto split_nk = [&](int sp) { return nkt - sp * nkc < nkc ? nkt - sp * nkc : nkc; };
    const uint64_t stream =
        (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr && split_k == 1) ? dropout_stream(epi.rng_call, epi.site) : 0;

    DA da;
    DB db;
    const uint32_t lds0 = lds_base(smem);
#ifdef CG_PK_WHATIF
    // diagnostic build only (make whatif; tools/gemm_whatif.py): pk_flags bit 4 skips the in-loop
    // DMAs, bit 5 the MFMAs, bit 6 the item epilogues -- wrong results, timing only
    // bit 3: only each block's LAST item stores (what the stores at the earlier item ends cost)
    const bool WI_NODMA = flags & 16, WI_NOMFMA = flags & 32, WI_NOEPI = flags & 64, WI_LASTONLY = flags & 8;
#else
    constexpr bool WI_NODMA = false, WI_NOMFMA = false, WI_NOEPI = false, WI_LASTONLY = false;
#endif
    da.init(lda, wave, lane);
    db.init(ldb, wave, lane);

    auto decode = [&](int j, int64_t& m0, int64_t& n0, int& split) {
        const int it = xcd_remap(b + j * P, nitems);
        int tm, tn;
        split = it / ntiles;
        tile_rc(it - split * ntiles, ntiles / tilesN, tilesN, flags >> 8, tm, tn);
        m0 = (int64_t)tm * BM;
        n0 = (int64_t)tn * BN;
    };
    int total = 0;
    for (int j = 0; j < my_items; ++j) {
        int64_t m0, n0;
        int sp;
        decode(j, m0, n0, sp);
        total += split_nk(sp);
    }
#ifdef CG_PK_BOUNDS
    da.lo = A;
    da.hi = A + (AT ? K * lda : M * lda);
    da.slot = 0;
    db.lo = B;
    db.hi = B + (BT ? K * ldb : N * ldb);
    db.slot = 1;
    if (flags & 128) {   // positive control (tools/gemm_bounds.py): windows 1 KB short, so in-range chunks count
        da.hi = (const char*)da.hi - 1024;
        db.hi = (const char*)db.hi - 1024;
    }
    // the L2-prefetch trial's cursors (db80795), one per distance PF = 1..3: tile j + PF of this
    // block's K-tile sequence when the DMA cursor is at tile j (clamped to the last tile)
    int pij[3] = {0, 0, 0}, pikt[3] = {0, 0, 0}, pink[3] = {0, 0, 0}, pkt[3] = {0, 0, 0};
    const bf16_t* poa[3] = {A, A, A};
    const bf16_t* pob[3] = {B, B, B};
    auto pf_adv = [&](int q) {
        if (pij[q] < my_items) {
            if (pikt[q] == 0) {
                int64_t m0, n0;
                int sp;
                decode(pij[q], m0, n0, sp);
                pink[q] = split_nk(sp);
                const int64_t kb = sp * kchunk;
                poa[q] = AT ? A + kb * lda + m0 : A + m0 * lda + kb;
                pob[q] = BT ? B + kb * ldb + n0 : B + n0 * ldb + kb;
            }
            pkt[q] = pikt[q];
            if (++pikt[q] == pink[q]) {
                pikt[q] = 0;
                ++pij[q];
            }
        }
    };
    auto pf_check = [&](int q) {   // lines 0..127 of the A (waves 0-1) or B (waves 2-3) K-tile
        const bool opb = wave >= 2;
        const bool tr = opb ? BT : AT;
        const int64_t ldx = opb ? ldb : lda;
        const int i = (wave & 1) * 64 + lane;
        const uint32_t off = tr ? 2u * (uint32_t)((i >> 1) * ldx) + 128u * (uint32_t)(i & 1) : 2u * (uint32_t)(i * ldx);
        const char* t = opb ? (const char*)(pob[q] + pkt[q] * db.kstep) : (const char*)(poa[q] + pkt[q] * da.kstep);
        bounds_chk(t + off, 4, opb ? db.lo : da.lo, opb ? db.hi : da.hi, 3 + q);
        bounds_chk(t + off + 64, 4, opb ? db.lo : da.lo, opb ? db.hi : da.hi, 3 + q);
    };
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        pf_adv(q);
        for (int t = 1; t <= q + 1; ++t) {
            pf_adv(q);
            pf_check(q);
        }
    }
#endif

    // DMA issue cursor (item ij, K-tile ikt) and its operand origins
    int ij = 0, ikt = 0, ink = 0;   // ink: K-tiles of the DMA cursor's item
    const bf16_t* oa = A;
    const bf16_t* ob = B;
    // The in-loop DMA is split from its address bookkeeping: prep_next() (branchy: item decode at
    // item boundaries) runs before the fragment reads and yields the K-tile's base addresses; the
    // LPT wave-instructions themselves are then issued one per 4 MFMAs (each costs ~60 issue
    // cycles -- MI355X_MICROARCH.md -- which now overlap the MFMAs instead of preceding them).
    // Past the last K-tile the same (valid) addresses are loaded again into the free stage, which
    // nothing reads; the loop drains them before the wave exits.
    const bf16_t* na = A;
    const bf16_t* nbp = B;
    auto prep_next = [&](bool real) {
        if (real) {
            if (ikt == 0) {
                int64_t m0, n0;
                int sp;
                decode(ij, m0, n0, sp);
                ink = split_nk(sp);
                const int64_t kb = sp * kchunk;
                oa = AT ? A + kb * lda + m0 : A + m0 * lda + kb;
                ob = BT ? B + kb * ldb + n0 : B + n0 * ldb + kb;
            }
            na = oa + ikt * da.kstep;
            nbp = ob + ikt * db.kstep;
            if (++ikt == ink) {
                ikt = 0;
                ++ij;
            }
        }
    };

    fv4 acc[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s)
        if (s < total) {
            prep_next(true);
            const uint32_t img = lds0 + (uint32_t)(s * G::STAGE);
#pragma unroll
            for (int i = 0; i < DA::PER_WAVE; ++i) da.issue1(na, i, img, wave);
#pragma unroll
            for (int i = 0; i < DB::PER_WAVE; ++i) db.issue1(nbp, i, img + G::IMG_A, wave);
        }

    // An item's epilogue issues exactly EPI_OPS vector stores (one per 16x16 fragment: dwordx2 bf16,
    // dwordx4 fp32 or split-K slab; checked in the ISA).  They are the youngest VMEM operations at
    // the next step's wait, so the count below lets them drain under the next MFMAs instead of
    // stalling the next K-tile on the store latency (vmcnt counts loads, LDS-DMA and stores in
    // issue order).
    // (8 for the fixed kinds whose bf16 output goes out as 16-B row segments -- store_item: with an
    // fp32 output they issue 16, more than counted, which only makes the wait conservative)
    // (4 NJ = 12 for the 48-column wave tiles, whose residual kinds store each fragment on its own;
    // 4 + 8 for STORE_ROWDOT: its delta stores, then the 16-B row segments)
    constexpr int EPI_OPS =
        NJ != 4 ? 4 * NJ
        : EK == CG_EPI_STORE_ROWDOT ? 12
        : EK == EK_SLAB16 ? 8
        : (EK == CG_EPI_STORE || EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_RELU_BWD) ? 8 : 16;
    int cur = 0, cj = 0, ckt = 0;
    int cnk;   // K-tiles of the compute cursor's item
    {
        int64_t m0, n0;
        int sp;
        decode(0, m0, n0, sp);
        cnk = my_items ? split_nk(sp) : 0;
    }
    bool stored = false;
#ifdef CG_PK_STAMPS
    uint64_t sw = 0, sm = 0, se = 0;
    const uint64_t w0 = pk_clk(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    for (int g = 0; g < total; ++g) {
        PK_STAMP(ta);
        const int ahead = total - 1 - g;  // steps issued after g that may stay in flight: min(NBUF-2, ahead)
        if (stored && !(flags & 1)) {
            if constexpr (NBUF >= 4) {
                if (ahead >= 2) wait_vm<2 * LPT + EPI_OPS>();
                else if (ahead == 1) wait_vm<LPT + EPI_OPS>();
                else wait_vm<EPI_OPS>();
            } else if constexpr (NBUF == 3) {
                if (ahead >= 1) wait_vm<LPT + EPI_OPS>();
                else wait_vm<EPI_OPS>();
            } else {
                wait_vm<EPI_OPS>();
            }
        } else if constexpr (NBUF >= 4) {
            if (ahead >= 2) wait_vm<2 * LPT>();
            else if (ahead == 1) wait_vm<LPT>();
            else wait_vm<0>();
        } else if constexpr (NBUF == 3) {
            if (ahead >= 1) wait_vm<LPT>();
            else wait_vm<0>();
        } else {
            wait_vm<0>();
        }
        stored = false;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        PK_STAMP(tb);
        int nb = cur + NBUF - 1;
        if (nb >= NBUF) nb -= NBUF;
        prep_next(g + NBUF - 1 < total);
#ifdef CG_PK_BOUNDS
#pragma unroll
        for (int q = 0; q < 3; ++q) {   // the trial issued tile g + 1 + PF after this step's DMAs
            pf_adv(q);
            pf_check(q);
        }
#endif
        const uint32_t dimg = lds0 + (uint32_t)(nb * G::STAGE);
        const char* imgA = smem + cur * G::STAGE;
        const char* imgB = imgA + G::IMG_A;
        // both 32-deep halves' fragments are read before the first MFMA (sched_barrier pins it):
        // otherwise the scheduler sinks each A read next to its 4 MFMAs and waits lgkmcnt(0) on it
        sv8 af[NS][4], bf[NS][NJ];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if constexpr (BK == 64) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) bf[s][j] = frag<BT, BN>(imgB, wn * WTN + j * 16, s, lane);
#pragma unroll
                for (int i = 0; i < 4; ++i) af[s][i] = frag<AT, BM>(imgA, wm * 64 + i * 16, s, lane);
            } else {
#pragma unroll
                for (int j = 0; j < NJ; ++j) bf[s][j] = frag32<BT, BN>(imgB, wn * WTN + j * 16, lane);
#pragma unroll
                for (int i = 0; i < 4; ++i) af[s][i] = frag32<AT, BM>(imgA, wm * 64 + i * 16, lane);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // 8 groups of 4 MFMAs (half s, A fragment i); the next stage's DMA instructions in between,
        // CG_PK_DPG of them after each group (1: spread over the whole step)
        auto issue_dma = [&](int t) {
            if (WI_NODMA) return;
            if (t < DA::PER_WAVE) {
                da.issue1(na, t, dimg, wave);
            } else {
                db.issue1(nbp, t - DA::PER_WAVE, dimg + G::IMG_A, wave);
            }
        };
#pragma unroll
        for (int t = 0; t < 4 * NS; ++t) {
            const int s = t >> 2, i = t & 3;
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                if (!WI_NOMFMA) acc[i][j] = mfma_bf16(bf[s][j], af[s][i], acc[i][j]);
#pragma unroll
            for (int d = 0; d < CG_PK_DPG; ++d)
                if (t * CG_PK_DPG + d < LPT) issue_dma(t * CG_PK_DPG + d);
        }
#pragma unroll
        for (int t = 4 * NS * CG_PK_DPG; t < LPT; ++t) issue_dma(t);
#pragma unroll
        for (int t = 0; t < 4 * NS; ++t) {
            __builtin_amdgcn_sched_group_barrier(0x008, NJ, 0);
#pragma unroll
            for (int d = 0; d < CG_PK_DPG; ++d)
                if (t * CG_PK_DPG + d < LPT) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        cur = cur + 1 == NBUF ? 0 : cur + 1;
        PK_STAMP(tc);
#ifdef CG_PK_STAMPS
        sw += tb - ta;
        sm += tc - tb;
#endif
        if (++ckt == cnk) {
            // item done: acc[i][j][r] = C[mw + 16i + (lane&15)][nw + 16j + 4(lane>>4) + r]
            int64_t m0, n0;
            int sp;
            decode(cj, m0, n0, sp);
            const int64_t mr = m0 + wm * 64 + (lane & 15), nc = n0 + wn * WTN + 4 * (lane >> 4);
#ifdef CG_PK_BOUNDS
            if (m0 < 0 || m0 + BM > M || n0 < 0 || n0 + BN > N || sp < 0 || sp >= split_k)
                atomicAdd(&g_pk_bounds[2], 1ull);
#endif
            if (WI_NOEPI || (WI_LASTONLY && cj + 1 < my_items)) {
            } else if constexpr (EK == EK_SLAB16) {   // bf16 slab: 16-B row segments, as a bf16 output
                store_item<true>(acc, mr, nc, (bf16_t*)ws + (int64_t)sp * M * N, CG_BF16, N);
            } else if (EK == EK_SLAB || split_k > 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) *(fv4*)(ws + ((int64_t)sp * M + mr + 16 * i) * N + nc + 16 * j) = acc[i][j];
            } else if constexpr (EK == EK_SLAB) {
            } else if (EK < 0 && (flags & 2)) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        epi_store4(acc[i][j], mr + 16 * i, nc + 16 * j, N, Cv, c_dtype, ldc, epi, stream);
            } else if constexpr (NJ == 4) {
                epi_item<EK < 0 ? EK_ANY : EK>(acc, mr, nc, N, Cv, c_dtype, ldc, epi, stream);
            } else {
                epi_resid_nj<EK, NJ>(acc, mr, nc, N, (float*)Cv, ldc, epi, stream);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
            ckt = 0;
            ++cj;
            if (cj < my_items) {
                int64_t m1, n1;
                int sp1;
                decode(cj, m1, n1, sp1);
                cnk = split_nk(sp1);
            }
            stored = true;
#ifdef CG_PK_STAMPS
            se += pk_clk() - tc;
#endif
        }
    }
#ifdef CG_PK_STAMPS
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&g_pk_stamps[0], (unsigned long long)sw);
        atomicAdd(&g_pk_stamps[1], (unsigned long long)sm);
        atomicAdd(&g_pk_stamps[2], (unsigned long long)se);
        atomicAdd(&g_pk_stamps[3], (unsigned long long)total);
        atomicAdd(&g_pk_stamps[4], (unsigned long long)(pk_clk() - w0));
        atomicAdd(&g_pk_stamps[5], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - r0));
        atomicAdd(&g_pk_stamps[6], 1ull);
    }
#endif
    wait_vm<0>();  // the dummy DMAs past the last K-tile land before the workgroup's LDS is released
    // a deferred split-K reduce of an earlier launch (gemm_common.h): on the blocks beyond the items
    // when the launch has them (launch_p), else in every block's tail
    if (red.n || red.na) red_tail(red, P > nitems ? nitems : 0);
}


int cu_count() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <bool AT_, bool BT_, int BM, int BN, int NBUF, int EK, int BK>
void launch_1(unsigned grid, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
              void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, int64_t kchunk, float* ws,
              hipStream_t st) {
    using G = GeoP<BM, BN, NBUF, BK>;
    // tile order (gemm_tile.h tile_rc): row-major -- consecutive items, which run on one XCD, share
    // the A row panel and walk the B panels -- unless there are more B panels than A panels (the FFN2
    // weight gradient dW2 = dz2^T h: 6 x 24 tiles at C4), where column-major makes them share the
    // B panel (h, 403 MB at C4: read by one XCD instead of up to all eight) and walk the few A panels.
    // cg_set_tuning("gemm_group_pk", g): g row panels per group (1 = row-major); 0 = this choice.
    const int64_t tM = M / BM, tN = N / BN;
    const int gm = g_gemm_group_pk > 0 ? g_gemm_group_pk : (tN > tM ? (int)tM : 0);
    // AdamW jobs only to a launch with >= SIDE_MIN blocks beyond its items (launch_p gives a
    // part-filling launch its free slots when work is pending)
    const bool side_ok = (int64_t)grid - tM * tN * split_k >= SIDE_MIN;
    k_gemm_pk<AT_, BT_, BM, BN, NBUF, EK, BK><<<grid, G::THREADS, G::LDS, st>>>(M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e,
                                                                         split_k, kchunk, ws, g_pk_flags | (gm << 8),
                                                                         take_pending_reduces(st, side_ok));
}

// epilogue instantiation: slab for split-K; a fixed kind for the default 128x128 2-stage kernel's
// non-transposed-A products (forward / dgrad) when the call allows it; otherwise the run-time one
template <bool AT_, bool BT_, int BM, int BN, int NBUF, int BK>
void launch_ek(unsigned grid, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
               int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, int64_t kchunk, float* ws,
               hipStream_t st) {
#define L1(EK_) launch_1<AT_, BT_, BM, BN, NBUF, EK_, BK>(grid, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, kchunk, ws, st)
    if (split_k > 1) {
        if (e.slab_bf16) L1(EK_SLAB16);
        else L1(EK_SLAB);
        return;
    }
    if constexpr (!AT_ && BM == 128 && BN == 128) {
        const bool needs_bias = e.kind >= CG_EPI_BIAS && e.kind <= CG_EPI_BIAS_DROP_RESID;
        const bool needs_resid = e.kind == CG_EPI_BIAS_RESID || e.kind == CG_EPI_BIAS_DROP_RESID;
        // the residual kinds write fp32, BIAS_RELU / RELU_BWD bf16 (epi_item's OUT); other dtypes take
        // the run-time epilogue.  Dropout at p = 0 is the bias + residual epilogue (same arithmetic).
        const bool f32 = c_dtype == CG_F32, b16 = c_dtype == CG_BF16;
        if (!(g_pk_flags & 2) && e.beta == 0.f && (!needs_bias || e.bias) && (!needs_resid || e.resid)) {
            switch (e.kind) {
                case CG_EPI_STORE: L1(CG_EPI_STORE); return;
                case CG_EPI_BIAS: L1(CG_EPI_BIAS); return;
                case CG_EPI_BIAS_RELU:
                    if (b16) { L1(CG_EPI_BIAS_RELU); return; }
                    break;
                case CG_EPI_BIAS_RESID:
                    if (f32) { L1(CG_EPI_BIAS_RESID); return; }
                    break;
                case CG_EPI_BIAS_DROP_RESID:
                    if (f32 && e.thr) { L1(CG_EPI_BIAS_DROP_RESID); return; }
                    if (f32) { L1(CG_EPI_BIAS_RESID); return; }
                    break;
                case CG_EPI_RELU_BWD:
                    if (b16) { L1(CG_EPI_RELU_BWD); return; }
                    break;
                case CG_EPI_STORE_ROWDOT:   // fast_gemm_launch admits it only here (rowdot_ok)
                    L1(CG_EPI_STORE_ROWDOT);
                    return;
                default: break;
            }
        }
    }
    L1(EK_ANY);
#undef L1
}

template <int BM, int BN, int NBUF, int BK = FBK>
bool launch_p(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
              int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
              hipStream_t st) {
    using G = GeoP<BM, BN, NBUF, BK>;
    const int64_t kchunk = (K / FBK + split_k - 1) / split_k * FBK;   // K-tiles per split, last one short
    const int64_t nitems = (M / BM) * (N / BN) * split_k;
    int64_t slots = (int64_t)cu_count() * G::OCC;
    if (g_gemm_max_grid > 0 && g_gemm_max_grid < slots) slots = g_gemm_max_grid;
    // a part-filling launch with >= SIDE_MIN free slots that will take pending work gets the free
    // slots too: those blocks have no items and run the reduce / AdamW jobs beside the items
    // (red_tail's `first`).  With fewer free slots the launch keeps grid = items and every block
    // takes its share of a reduce after its item (a few free blocks must not carry a whole reduce).
    const bool side = g_red_side && slots - nitems >= SIDE_MIN && has_pending_reduces(st, true);
    const unsigned grid = (unsigned)(nitems < slots && !side ? nitems : slots);
#define FG(AT_, BT_) launch_ek<AT_, BT_, BM, BN, NBUF, BK>(grid, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, kchunk, ws, st)
    // transposed LDS images need a multiple of 128 rows (DmaP, col_swz): other tiles serve only the
    // layouts they can; false = not launched
    if (!at && !bt) {
        FG(false, false);
        return true;
    } else if (!at && bt) {
        if constexpr (BN % 128 == 0) {
            FG(false, true);
            return true;
        }
    } else if (at && !bt) {
        if constexpr (BM % 128 == 0) {
            FG(true, false);
            return true;
        }
    } else {
        if constexpr (BM % 128 == 0 && BN % 128 == 0) {
            FG(true, true);
            return true;
        }
    }
    return false;
#undef FG
}

// 128 x 96 tiles for the fp32 residual forwards (projection + residual, FFN2 + dropout + residual)
// where they shorten the busiest resident slot's work (rounds of items x tile width): at C2
// (M = 16384, N = 384) 384 tiles of 128 x 128 fill 3/4 of the 512 two-per-CU slots -- half the CUs
// run two, half one, and the launch waits for the former -- while 512 tiles of 128 x 96 put two on
// every CU: a quarter fewer MFMAs and an eighth fewer operand bytes on the busiest CU (proj 19.4 ->
// 16.6 us, FFN2 36.7 -> 31.5 us).  Same K order per output element as 128 x 128: bitwise equal.  The
// plain-store products measured no gain or a loss (QKV forward, transposed-B input gradients:
// profiles/r4_gemm_n96_ab.txt).  cg_set_tuning("gemm_n96", 0) turns it off (A/B).
bool launch_n96(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
                int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, hipStream_t st) {
    if (!g_gemm_n96 || at || bt || split_k != 1 || e.beta != 0.f || e.colpart || (g_pk_flags & 2)) return false;
    if ((e.kind != CG_EPI_BIAS_RESID && e.kind != CG_EPI_BIAS_DROP_RESID) || !e.bias || !e.resid || c_dtype != CG_F32)
        return false;
    if (M % 128 || N % 96 || K % FBK) return false;
    using G = GeoP<128, 96, 2>;
    int64_t slots = (int64_t)cu_count() * G::OCC;
    if (g_gemm_max_grid > 0 && g_gemm_max_grid < slots) slots = g_gemm_max_grid;
    // the busiest slot's output columns: rounds of items x tile width
    const int64_t t96 = (M / 128) * (N / 96), t128 = (M / 128) * (N / 128);
    const int64_t crit96 = (t96 + slots - 1) / slots * 96, crit128 = N % 128 ? INT64_MAX : (t128 + slots - 1) / slots * 128;
    if (crit96 >= crit128) return false;
    const unsigned grid = (unsigned)(t96 < slots ? t96 : slots);
#define L96(EK_) launch_1<false, false, 128, 96, 2, EK_, FBK>(grid, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, 1, K, nullptr, st)
    if (e.kind == CG_EPI_BIAS_DROP_RESID && e.thr) L96(CG_EPI_BIAS_DROP_RESID);
    else L96(CG_EPI_BIAS_RESID);   // dropout at p = 0 is the bias + residual epilogue
#undef L96
    return true;
}

}  // namespace

int gemm_cu_count() { return cu_count(); }

bool pk_gemm_launch(int v, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                    const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                    float* ws, hipStream_t st) {
    switch (v) {
        case 9:
            if (launch_n96(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, st)) return true;
            return launch_p<128, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
#ifdef CG_AB_VARIANTS   // measured-slower A/B tiles (profiles/r1_gemm_scan*.txt, r2_gemm_ring_depth_scan.txt)
        case 10: launch_p<128, 128, 3>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        case 11:
            if (M % 256) return false;
            launch_p<256, 128, 3>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
            return true;
        case 12: launch_p<128, 128, 4>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        // narrow tiles for N = 384 outputs (384 128x128 tiles fill only 3/4 of 512 resident slots)
        case 13:
            if (at) return false;
            launch_p<64, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
            return true;
        case 14:
            if (at) return false;
            launch_p<64, 128, 3>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
            return true;
        case 15:
            if (at || bt) return false;
            launch_p<128, 64, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
            return true;
        case 16:
            if (at) return false;
            launch_p<64, 128, 4>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
            return true;
#endif
        default: return false;
    }
}

}  // namespace cg
