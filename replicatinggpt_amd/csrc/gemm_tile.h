// charpt bf16 MFMA GEMM tile helpers shared by the register-staged kernel (gemm_bf16.hip) and the
// LDS-DMA kernel (gemm_glds.hip): swizzled LDS images, MFMA fragments, XCD remap and the fused
// LDS-staged epilogue.
#pragma once
#include "gemm_common.h"

namespace cg {
namespace gt {

constexpr int FBK = 64;  // K depth of one staged tile

typedef __attribute__((address_space(3))) sv4 lds_sv4;

// K-contiguous image of R rows: [R][64] bf16, 128-B rows, chunk c (16 B, 0..7) at c ^ ((r>>1)&7)
__device__ __forceinline__ int img_row_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ int row_swz(int r) { return (r >> 1) & 7; }
// M/N-contiguous image of R columns: [64 k][R] bf16, rows of 2R bytes, chunk c (0..R/8-1); the low
// 4 chunk bits are XORed with ((k&3)<<2 | (k>>2)&3)  (cdna guide T10, layout (b))
__device__ __forceinline__ int col_swz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
template <int R>
__device__ __forceinline__ int img_col_off(int k, int c) {
    return k * (2 * R) + ((c ^ col_swz(k)) << 4);
}

// MFMA 16x16x32 operand fragment: tile rows rb..rb+15, k = 32s..32s+31.
// lane l holds X(rb + (l&15), 32s + 8(l>>4) + j), j = 0..7
template <bool TR, int R>
__device__ __forceinline__ sv8 frag(const char* img, int rb, int s, int lane) {
    if (!TR) {
        return *(const sv8*)(img + img_row_off(rb + (lane & 15), s * 4 + (lane >> 4)));
    } else {
        const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
        const int ka = 32 * s + 8 * g;
        const int chunk = (rb >> 3) + (p >> 1), byte = 8 * (p & 1);
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_col_off<R>(ka + q, chunk) + byte));
        const sv4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_col_off<R>(ka + 4 + q, chunk) + byte));
        return sv8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
}

// 32-deep K-tiles (k_gemm_pk BK = 32): K-contiguous image [R][32] bf16, 64-B rows, chunk c (0..3) at
// c ^ ((r>>2)&2).  A 16x16x32 fragment read (ds_read_b128, lane l: row rb + (l&15), chunk l>>4) then
// puts each 16-lane group of the instruction on 16 distinct 16-B slots of the 256-B bank row
// (lanes {0-3,12-15,20-27}: rows j, 12+j, 4+j, 8+j of chunks 0,0,1,1 -> slots 4j + {0,2,1,3}).  The
// M/N-contiguous image is the 64-deep one cut to 32 k-rows (same col_swz).
__device__ __forceinline__ int row_swz32(int r) { return (r >> 2) & 2; }
__device__ __forceinline__ int img_row_off32(int r, int c) { return r * 64 + ((c ^ row_swz32(r)) << 4); }
template <bool TR, int R>
__device__ __forceinline__ sv8 frag32(const char* img, int rb, int lane) {
    if (!TR) return *(const sv8*)(img + img_row_off32(rb + (lane & 15), lane >> 4));
    return frag<true, R>(img, rb, 0, lane);
}

__device__ __forceinline__ fv4 mfma_bf16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

// bijective XCD-aware remap (cdna guide §5 "XCD swizzle must be bijective"): consecutive remapped
// ids run on one XCD (shared L2)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// output tile (tm, tn) of flattened tile index t.  gm <= 1: row-major.  gm > 1: grouped order --
// gm row panels walked column by column (the last group may be shorter), so the items one XCD runs
// at once (consecutive after xcd_remap) share fewer A and B panels in its L2.  Bijective.
__device__ __forceinline__ void tile_rc(int t, int tilesM, int tilesN, int gm, int& tm, int& tn) {
    if (gm <= 1) {
        tm = t / tilesN;
        tn = t - tm * tilesN;
        return;
    }
    const int per = gm * tilesN, g = t / per, first = g * gm;
    const int rows = tilesM - first < gm ? tilesM - first : gm;
    const int r = t - g * per;
    tn = r / rows;
    tm = first + (r - tn * rows);
}

// 8 consecutive output columns of one row: bias / relu / dropout / relu-bwd / residual / beta, store
__device__ __forceinline__ void epi_store8(float (&v)[8], int64_t m, int64_t n, int64_t N, void* Cv, int c_dtype,
                                           int64_t ldc, const EpiArgs& epi, uint64_t stream) {
    const int kind = epi.kind;
    if (kind != CG_EPI_STORE && kind != CG_EPI_RELU_BWD && epi.bias) {
        const float4 b0 = *(const float4*)(epi.bias + n), b1 = *(const float4*)(epi.bias + n + 4);
        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
        v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (kind == CG_EPI_BIAS_RELU) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
    } else if (kind == CG_EPI_BIAS_DROP_RESID && epi.thr) {
        const uint64_t idx = (uint64_t)m * (uint64_t)N + (uint64_t)n;  // n % 8 == 0, N % 8 == 0
        const uint32_t kb = keep4_bits(epi.seed, stream, idx, epi.thr) | (keep4_bits(epi.seed, stream, idx + 4, epi.thr) << 4);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = ((kb >> q) & 1u) ? v[q] * epi.dscale : 0.f;
    } else if (kind == CG_EPI_RELU_BWD) {
        if (epi.aux_dtype == CG_BF16) {
            const uint4 h = *(const uint4*)((const bf16_t*)epi.aux + m * epi.ld_aux + n);
            const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[2 * q] = __uint_as_float(hw[q] << 16) > 0.f ? v[2 * q] : 0.f;
                v[2 * q + 1] = __uint_as_float(hw[q] & 0xffff0000u) > 0.f ? v[2 * q + 1] : 0.f;
            }
        } else {
            const float* h = (const float*)epi.aux + m * epi.ld_aux + n;
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = h[q] > 0.f ? v[q] : 0.f;
        }
    }
    if ((kind == CG_EPI_BIAS_RESID || kind == CG_EPI_BIAS_DROP_RESID) && epi.resid) {
        const float* rp = epi.resid + m * epi.ld_resid + n;
        const float4 r0 = *(const float4*)rp, r1 = *(const float4*)(rp + 4);
        v[0] = r0.x + v[0]; v[1] = r0.y + v[1]; v[2] = r0.z + v[2]; v[3] = r0.w + v[3];
        v[4] = r1.x + v[4]; v[5] = r1.y + v[5]; v[6] = r1.z + v[6]; v[7] = r1.w + v[7];
    }
    if (c_dtype == CG_BF16) {
        bf16_t* o = (bf16_t*)Cv + m * ldc + n;
        if (epi.beta != 0.f) {
            const uint4 old = *(const uint4*)o;
            const uint32_t ow[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[2 * q] += epi.beta * __uint_as_float(ow[q] << 16);
                v[2 * q + 1] += epi.beta * __uint_as_float(ow[q] & 0xffff0000u);
            }
        }
        *(uint4*)o = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
    } else {
        float* o = (float*)Cv + m * ldc + n;
        if (epi.beta != 0.f) {
            const float4 o0 = *(const float4*)o, o1 = *(const float4*)(o + 4);
            v[0] += epi.beta * o0.x; v[1] += epi.beta * o0.y; v[2] += epi.beta * o0.z; v[3] += epi.beta * o0.w;
            v[4] += epi.beta * o1.x; v[5] += epi.beta * o1.y; v[6] += epi.beta * o1.z; v[7] += epi.beta * o1.w;
        }
        *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}

// 4 consecutive output columns n..n+3 (n % 4 == 0) of row m, straight from the accumulator of a
// swapped-operand MFMA (lane holds C[m][n..n+3]): the same fused epilogues as epi_store8; the
// dropout word group idx>>2 = (m*N+n)/4 is exactly one Philox call.
__device__ __forceinline__ void epi_store4(fv4 v, int64_t m, int64_t n, int64_t N, void* Cv, int c_dtype,
                                           int64_t ldc, const EpiArgs& epi, uint64_t stream) {
    const int kind = epi.kind;
    if (kind != CG_EPI_STORE && kind != CG_EPI_RELU_BWD && epi.bias) {
        const float4 b = *(const float4*)(epi.bias + n);
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    if (kind == CG_EPI_BIAS_RELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
    } else if (kind == CG_EPI_BIAS_DROP_RESID && epi.thr) {
        const uint32_t kb = keep4_bits(epi.seed, stream, (uint64_t)m * (uint64_t)N + (uint64_t)n, epi.thr);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ((kb >> q) & 1u) ? v[q] * epi.dscale : 0.f;
    } else if (kind == CG_EPI_RELU_BWD) {
        if (epi.aux_dtype == CG_BF16) {
            const uint2 h = *(const uint2*)((const bf16_t*)epi.aux + m * epi.ld_aux + n);
            v[0] = __uint_as_float(h.x << 16) > 0.f ? v[0] : 0.f;
            v[1] = __uint_as_float(h.x & 0xffff0000u) > 0.f ? v[1] : 0.f;
            v[2] = __uint_as_float(h.y << 16) > 0.f ? v[2] : 0.f;
            v[3] = __uint_as_float(h.y & 0xffff0000u) > 0.f ? v[3] : 0.f;
        } else {
            const float4 h = *(const float4*)((const float*)epi.aux + m * epi.ld_aux + n);
            v[0] = h.x > 0.f ? v[0] : 0.f;
            v[1] = h.y > 0.f ? v[1] : 0.f;
            v[2] = h.z > 0.f ? v[2] : 0.f;
            v[3] = h.w > 0.f ? v[3] : 0.f;
        }
    }
    if ((kind == CG_EPI_BIAS_RESID || kind == CG_EPI_BIAS_DROP_RESID) && epi.resid) {
        const float4 r = *(const float4*)(epi.resid + m * epi.ld_resid + n);
        v[0] = r.x + v[0]; v[1] = r.y + v[1]; v[2] = r.z + v[2]; v[3] = r.w + v[3];
    }
    if (c_dtype == CG_BF16) {
        bf16_t* o = (bf16_t*)Cv + m * ldc + n;
        if (epi.beta != 0.f) {
            const uint2 old = *(const uint2*)o;
            v[0] += epi.beta * __uint_as_float(old.x << 16);
            v[1] += epi.beta * __uint_as_float(old.x & 0xffff0000u);
            v[2] += epi.beta * __uint_as_float(old.y << 16);
            v[3] += epi.beta * __uint_as_float(old.y & 0xffff0000u);
        }
        *(uint2*)o = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    } else {
        float* o = (float*)Cv + m * ldc + n;
        if (epi.beta != 0.f) {
            const float4 old = *(const float4*)o;
            v[0] += epi.beta * old.x; v[1] += epi.beta * old.y; v[2] += epi.beta * old.z; v[3] += epi.beta * old.w;
        }
        *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// Dropout keep nibbles of a wave's 64 x 16NJ item fragment for any NJ (k_gemm_pk and k_gemm_p8 residual
// epilogues): as gemm_pk.hip's drop_nibbles, lanes l and
// l ^ 16 hold the two 4-column halves of one 8-column Philox group, but the pair splits the work by
// rows -- lane half odd = (lane >> 4) & 1 evaluates rows i = 2 odd, 2 odd + 1 for every j -- and
// trades one word per j.  Same bits.
template <int NJ>
__device__ __forceinline__ void drop_nibbles_rows(const EpiArgs& epi, uint64_t stream, int64_t mr, int64_t nc, int64_t N,
                                                  uint32_t (&nib)[4][NJ]) {
    const int lane = threadIdx.x & 63;
    const uint32_t odd = (lane >> 4) & 1;
    const int64_t c8 = nc & ~(int64_t)7;
    uint32_t mine[NJ], other[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        mine[j] = 0u;
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
            const uint64_t idx = (uint64_t)(mr + 16 * (2 * odd + ii)) * (uint64_t)N + (uint64_t)(c8 + 16 * j);
            mine[j] |= keep8_bits(philox_group(epi.seed, stream, idx >> 3), epi.thr) << (8 * ii);
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) other[j] = (uint32_t)__shfl_xor((int)mine[j], 16, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint32_t w = ((uint32_t)(i >> 1) == odd) ? mine[j] : other[j];
            nib[i][j] = (w >> (8 * (i & 1) + 4 * odd)) & 0xfu;
        }
}

// LDS bytes the epilogue needs for a BM x BN block: 128-row rounds of fp32 rows padded by 4
template <int BN>
constexpr int epi_lds_bytes() {
    return 128 * (BN + 4) * 4;
}

// accumulators of a WM x WN grid of 64x64 wave tiles -> LDS (fp32, 128-row rounds) -> 8 consecutive
// columns per lane -> epi_store8 (or the fp32 split-K slab).  Caller has finished all LDS reads of
// the staging buffers (a barrier precedes the first LDS write here).
template <int BM, int BN>
__device__ __forceinline__ void epilogue(fv4 (&acc)[4][4], char* smem, int tid, int64_t M, int64_t N, int64_t m0,
                                         int64_t n0, void* Cv, int c_dtype, int64_t ldc, const EpiArgs& epi,
                                         int split_k, int split, float* ws) {
    constexpr int WN = BN / 64, THREADS = (BM / 64) * WN * 64;
    constexpr int CS_LD = BN + 4, EPI_ROWS = 128;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    float* Cs = (float*)smem;
    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
#pragma unroll
    for (int round = 0; round < BM / EPI_ROWS; ++round) {
        if (wm / 2 == round) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        Cs[((wm & 1) * 64 + i * 16 + 4 * (lane >> 4) + r) * CS_LD + wn * 64 + j * 16 + (lane & 15)] =
                            acc[i][j][r];
        }
        __syncthreads();
        constexpr int CPR = BN / 8;  // 8-column groups per row
#pragma unroll 1
        for (int idx = tid; idx < EPI_ROWS * CPR; idx += THREADS) {
            const int row = idx / CPR, col = (idx % CPR) * 8;
            const int64_t m = m0 + round * EPI_ROWS + row, n = n0 + col;
            float v[8];
            const float4 x0 = *(const float4*)(Cs + row * CS_LD + col);
            const float4 x1 = *(const float4*)(Cs + row * CS_LD + col + 4);
            v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
            v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
            if (split_k > 1) {
                float* o = ws + ((int64_t)split * M + m) * N + n;
                *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
                *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
            } else {
                epi_store8(v, m, n, N, Cv, c_dtype, ldc, epi, stream);
            }
        }
        if (round + 1 < BM / EPI_ROWS) __syncthreads();
    }
}

}  // namespace gt

// ReLU keep bits (CG_BITS) of a wave's FM x 4 fragments of 16x16 (64 columns from the wave's column
// base cb = nc - 4 (lane >> 4)); nib[i][j] bit q <-> (row rb + 16 i, column cb + 16 j + 4 (lane >> 4)
// + q), rb = this lane's row.  Word jp of a row = columns cb + 32 jp .. + 31 (bit = column - base).
// Lanes l, l^16, l^32, l^48 hold the four column quarters of each fragment row: OR-reduced across
// them, then lane group g = lane >> 4 stores the two words of rows i = g (mod 4) as one 8-B store.
template <int FM>
__device__ __forceinline__ void relu_bits_store(const uint32_t (&nib)[FM][4], uint32_t* bits, int64_t ldw, int64_t rb,
                                                int64_t cb, int lane) {
    const int g = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        uint32_t w0 = (nib[i][0] << (4 * g)) | (nib[i][1] << (16 + 4 * g));
        uint32_t w1 = (nib[i][2] << (4 * g)) | (nib[i][3] << (16 + 4 * g));
        w0 |= (uint32_t)__shfl_xor((int)w0, 16, 64);
        w1 |= (uint32_t)__shfl_xor((int)w1, 16, 64);
        w0 |= (uint32_t)__shfl_xor((int)w0, 32, 64);
        w1 |= (uint32_t)__shfl_xor((int)w1, 32, 64);
        if ((i & 3) == g) *(uint2*)(bits + (rb + 16 * i) * ldw + (cb >> 5)) = make_uint2(w0, w1);
    }
}
// nonzero-ness of the 4 bf16 values of a packed fragment (bit q <-> value q): the ReLU keep bits
__device__ __forceinline__ uint32_t nz4_bf16(uint2 pk) {
    return (uint32_t)((pk.x & 0x7fffu) != 0) | ((uint32_t)((pk.x & 0x7fff0000u) != 0) << 1) |
           ((uint32_t)((pk.y & 0x7fffu) != 0) << 2) | ((uint32_t)((pk.y & 0x7fff0000u) != 0) << 3);
}
// the keep nibble of fragment (i, j) from its row's two words (uint2 at column base cb)
__device__ __forceinline__ uint32_t relu_nib(uint2 w, int j, int lane) {
    return (((j >> 1) ? w.y : w.x) >> (16 * (j & 1) + 4 * (lane >> 4))) & 0xfu;
}
// bf16 stores of a wave's FM x 4 output fragments (16x16, lane: row rb = mr + 16 i, columns
// nc + 16 j .. +3 with nc = cb + 4 (lane >> 4)) as 16-B row segments: for each fragment pair
// (j, j+1) the lanes of odd 16-lane rows trade their fragment-j quarter for the even row's
// fragment-(j+1) quarter (v_permlane16_swap), so lane quarter q holds 8 contiguous columns: FM x 2
// dwordx4 stores, each 64 contiguous bytes of 16 rows, instead of FM x 4 dwordx2
// (cdna_hip_programming.md T21).  The callers' wait counts know it is FM x 2 stores.
template <int FM>
__device__ __forceinline__ void store_bf16_wide(const fv4 (&v)[FM][4], bf16_t* C, int64_t ldc, int64_t mr, int64_t nc) {
    const int q = (threadIdx.x & 63) >> 4;
    const int64_t col = nc - 4 * q + ((q & 1) ? 16 : 0) + ((q >> 1) ? 8 : 0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
            const uint32_t ax = pack_bf2(v[i][jp][0], v[i][jp][1]), ay = pack_bf2(v[i][jp][2], v[i][jp][3]);
            const uint32_t bx = pack_bf2(v[i][jp + 1][0], v[i][jp + 1][1]), by = pack_bf2(v[i][jp + 1][2], v[i][jp + 1][3]);
            const auto sx = __builtin_amdgcn_permlane16_swap(ax, bx, false, false);
            const auto sy = __builtin_amdgcn_permlane16_swap(ay, by, false, false);
            st_out16((uint4*)(C + (mr + 16 * i) * ldc + col + 16 * jp), make_uint4(sx[0], sy[0], sx[1], sy[1]));
        }
}
}  // namespace cg
