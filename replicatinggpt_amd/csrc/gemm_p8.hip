// charpt: persistent 8-wave LDS-DMA bf16 MFMA GEMM (gfx950) -- the default kernel behind cg_gemm
// for the nn.Linear forward / dgrad / wgrad products of GPT1.py:111-112,121,136,143,145.
//
// Why this shape (measured with tools/gemm_diag.hip on MI355X):
//  * a 128x128 block tile needs (BM+BN)*BK*2 B of operands per 2*BM*BN*BK FLOP = 64 FLOP/B, i.e.
//    ~31 TB/s of L2->LDS traffic at the MFMA peak -- the chip's whole L2 bandwidth.  256x128 tiles
//    halve that per FLOP (85 FLOP/B), 256x256 tiles quarter it (128 FLOP/B);
//  * with one tile per block every CU runs load -> MFMA -> store in lockstep with every other CU,
//    so a short-K launch (K = 384: 6 K-tiles) pays the HBM-bound first load and the HBM-bound
//    output store in series with the MFMA loop.  Here blocks are persistent (one per CU, 8 waves =
//    2 per SIMD) and walk a flattened (item, K-tile) sequence; the LDS-DMA ring
//    (global_load_lds_dwordx4, NBUF stages, NBUF-1 K-tiles in flight, counted vmcnt, raw
//    s_barrier) runs straight across item boundaries, and the epilogue is register-direct
//    (swapped MFMA operands: each lane holds 4 consecutive output columns of one row), so the
//    output stores of item j drain while item j+1's MFMAs run.
// An item is one BM x BN output tile of one K-split; items are ordered split-major and remapped so
// that consecutive items (same row panel) share an XCD's L2.
#include "gemm_tile.h"

namespace cg {
namespace {
using namespace gt;

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int P8_WAVES = 8, P8_THREADS = 512;

// per-lane LDS-DMA sources of one operand image: R rows (K-contiguous) or R columns (TR) x 64 k.
// Wave-instruction i writes LDS bytes [1024 i, 1024 i + 1024) lane-linearly; the XOR swizzle of
// gemm_tile.h is applied to the SOURCE address (cdna guide §5.4 rule 21).
template <bool TR, int R>
struct Dma8 {
    static constexpr int INSTR = R * FBK * 2 / 1024;
    static constexpr int PER_WAVE = INSTR / P8_WAVES;
    static_assert(PER_WAVE * P8_WAVES == INSTR, "tile/wave mismatch");
    static_assert(!TR || R >= 128, "transposed image swizzle needs >= 16 chunks per row");
    uint32_t off[PER_WAVE];   // byte offsets (saddr form, gemm_pk.hip DmaP)
    int64_t kstep;

    __device__ __forceinline__ void init(int64_t ld, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) {
            const int pos = (wave * PER_WAVE + i) * 1024 + lane * 16;
            if (!TR) {
                const int r = pos >> 7, c = ((pos >> 4) & 7) ^ row_swz(r);
                off[i] = 2u * (uint32_t)((int)(r * ld) + c * 8);
            } else {
                const int k = pos / (2 * R), c = ((pos % (2 * R)) >> 4) ^ col_swz(k);
                off[i] = 2u * (uint32_t)((int)(k * ld) + c * 8);
            }
        }
        kstep = TR ? (int64_t)FBK * ld : (int64_t)FBK;
    }
    __device__ __forceinline__ void issue(const bf16_t* origin, int kt, uint32_t img, int wave) const {
        const bf16_t* base = origin + kt * kstep;
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) dma16sl(base, off[i], img + (uint32_t)((wave * PER_WAVE + i) * 1024));
    }
};

// half-depth pieces (32 k) of the same images for the staggered schedule: an R-row K-contiguous
// image [R][32] with 64-B rows (gemm_tile.h img_row_off32) or the first / second 32 k-rows of the
// transposed one; k-half h of K-tile kt starts 32 h k past the K-tile's origin
template <bool TR, int R>
struct Dma8h {
    static constexpr int INSTR = R * 32 * 2 / 1024;
    static constexpr int PER_WAVE = INSTR / P8_WAVES;
    static_assert(PER_WAVE * P8_WAVES == INSTR, "tile/wave mismatch");
    static_assert(!TR || R >= 128, "transposed image swizzle needs >= 16 chunks per row");
    uint32_t off[PER_WAVE];
    int64_t kstep, hstep;

    __device__ __forceinline__ void init(int64_t ld, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) {
            const int pos = (wave * PER_WAVE + i) * 1024 + lane * 16;
            if (!TR) {
                const int r = pos >> 6, c = ((pos >> 4) & 3) ^ row_swz32(r);
                off[i] = 2u * (uint32_t)((int)(r * ld) + c * 8);
            } else {
                const int k = pos / (2 * R), c = ((pos % (2 * R)) >> 4) ^ col_swz(k);
                off[i] = 2u * (uint32_t)((int)(k * ld) + c * 8);
            }
        }
        kstep = TR ? (int64_t)FBK * ld : (int64_t)FBK;
        hstep = TR ? (int64_t)32 * ld : (int64_t)32;
    }
    __device__ __forceinline__ void issue(const bf16_t* origin, int kt, int h, uint32_t img, int wave) const {
        const bf16_t* base = origin + kt * kstep + h * hstep;
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) dma16sl(base, off[i], img + (uint32_t)((wave * PER_WAVE + i) * 1024));
    }
};

template <int BM, int BN, int NBUF>
struct Geo8 {
    static constexpr int IMG_A = BM * FBK * 2, IMG_B = BN * FBK * 2, STAGE = IMG_A + IMG_B;
    static constexpr int LDS = NBUF * STAGE;
    static constexpr int OCC = LDS <= 80 * 1024 ? 2 : 1;  // resident blocks per CU (LDS-bound)
};

// WM = waves along M (8 / WM along N); per-wave tile (BM/WM) x (BN/(8/WM)) in 16x16 fragments.
// EP: the item epilogue, one per instantiation (each path alone keeps the 256x256 tile's 128
// accumulators out of scratch; both colpart mask forms in one kernel spilled 228 B/lane and ran the
// C4 FFN2 dgrad at 1.04 ms instead of 0.36):
//   P8_GENERIC    per-fragment epi_store4 (any kind) or split-K slabs
//   P8_CP_BF16    ReLU backward + fused bias-gradient column partials, mask from the bf16 ReLU output
//   P8_CP_BITS    the same with the mask from CG_BITS keep bits
//   P8_RELU_BITS  bias + ReLU, bf16 output and its CG_BITS keep bits
//   P8_BWD_BITS   ReLU backward from CG_BITS keep bits, no column partials
//   P8_BF16       STORE / BIAS / BIAS_RELU with a bf16 output (beta 0, split 1)
//   P8_RESID      BIAS_RESID / BIAS_DROP_RESID with an fp32 output (beta 0, split 1, bias and residual
//                 present): the residual of a 64-row band loaded before the band's first store (the
//                 generic path's per-fragment load -> store order, with C and the residual possibly
//                 the same array, was 32 dependent HBM round trips per item), the dropout bits from
//                 one Philox call per 8 columns shared by lane pairs (drop_nibbles_rows)
// Every path but P8_GENERIC writes its bf16 output as 16-B row segments (store_bf16_wide: FM x 2
// stores per item), so their EPI_OPS is half the generic path's FM x FN.
enum { P8_GENERIC = 0, P8_CP_BF16 = 1, P8_CP_BITS = 2, P8_RELU_BITS = 3, P8_BWD_BITS = 4, P8_BF16 = 5, P8_RESID = 6 };
// SCH: 0 = one barrier per K-tile, both wave groups in step; 1 = the staggered 8-phase schedule
template <bool AT, bool BT, int BM, int BN, int WM, int NBUF, int EP, int SCH>
__global__ __launch_bounds__(P8_THREADS, (Geo8<BM, BN, NBUF>::OCC))
void k_gemm_p8(int64_t M, int64_t N, int64_t K, const bf16_t* __restrict__ A, int64_t lda,
               const bf16_t* __restrict__ B, int64_t ldb, void* __restrict__ Cv, int c_dtype, int64_t ldc,
               EpiArgs epi, int split_k, int64_t kchunk, float* __restrict__ ws, int gm, RedJobs red) {
    using G = Geo8<BM, BN, NBUF>;
    using DA = Dma8<AT, BM>;
    using DB = Dma8<BT, BN>;
    constexpr int WN = P8_WAVES / WM, FM = BM / WM / 16, FN = BN / WN / 16;
    constexpr int LPT = DA::PER_WAVE + DB::PER_WAVE;  // DMA instructions per lane per K-tile
    // vector-memory output stores per lane per item (the youngest VMEM operations at the next wait)
    constexpr int EPI_OPS = (EP == P8_GENERIC || FN != 4) ? FM * FN : FM * 2;
    static_assert(NBUF >= 2 && NBUF <= 4, "ring depth");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int tilesN = (int)(N / BN);
    const int ntiles = (int)(M / BM) * tilesN;
    const int nitems = ntiles * split_k;
    const int nk = (int)(kchunk / FBK);
    const int P = gridDim.x, b = blockIdx.x;
    const int my_items = b < nitems ? (nitems - 1 - b) / P + 1 : 0;
    const int total = my_items * nk;
    const uint64_t stream =
        (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr && split_k == 1) ? dropout_stream(epi.rng_call, epi.site) : 0;

    DA da;
    DB db;
    da.init(lda, wave, lane);
    db.init(ldb, wave, lane);

    auto decode = [&](int j, int64_t& m0, int64_t& n0, int& split) {
        const int it = xcd_remap(b + j * P, nitems);
        split = it / ntiles;
        int tm, tn;
        tile_rc(it - split * ntiles, ntiles / tilesN, tilesN, gm, tm, tn);
        m0 = (int64_t)tm * BM;
        n0 = (int64_t)tn * BN;
    };

    // DMA issue cursor (item ij, K-tile ikt) and its operand origins
    int ij = 0, ikt = 0;
    const bf16_t* oa = A;
    const bf16_t* ob = B;
    auto issue_next = [&](int buf) {
        if (ikt == 0) {
            int64_t m0, n0;
            int sp;
            decode(ij, m0, n0, sp);
            const int64_t kb = sp * kchunk;
            oa = AT ? A + kb * lda + m0 : A + m0 * lda + kb;
            ob = BT ? B + kb * ldb + n0 : B + n0 * ldb + kb;
        }
        const uint32_t img = lds_base(smem) + (uint32_t)(buf * G::STAGE);
        da.issue(oa, ikt, img, wave);
        db.issue(ob, ikt, img + G::IMG_A, wave);
        if (++ikt == nk) {
            ikt = 0;
            ++ij;
        }
    };

    fv4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    int cj = 0;   // items finished by this block
    // the item epilogue, after the item's last K-tile (both schedules)
    auto finish_item = [&]() {
        // item done: acc[i][j][r] = C[mw + 16i + (lane&15)][nw + 16j + 4(lane>>4) + r]
        int64_t m0, n0;
        int sp;
        decode(cj, m0, n0, sp);
        const int64_t mr = m0 + wm * (BM / WM) + (lane & 15), nc = n0 + wn * (BN / WN) + 4 * (lane >> 4);
        constexpr bool COLPART = EP == P8_CP_BF16 || EP == P8_CP_BITS;
        if constexpr (COLPART) {
            // ReLU backward (bf16 ReLU output as the mask, beta 0: checked on the host) with the
            // consumer's bias gradient fused: column sums of the bf16-rounded outputs per 64-row
            // block (the layout of k_gemm_pk's colpart), 4 rows per lane then a DPP row sum over the
            // column group's 16 lanes.  The partial stores go before the item's FM x FN output
            // stores, which stay the youngest EPI_OPS vector-memory operations.
            if constexpr (EP == P8_CP_BITS) {   // ReLU keep bits: one word pair per row (FN == 4)
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    const uint2 w =
                        *(const uint2*)((const uint32_t*)epi.aux + (mr + 16 * i) * epi.ld_aux + ((nc - 4 * (lane >> 4)) >> 5));
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const uint32_t kb = relu_nib(w, j, lane);
                        fv4& v = acc[i][j];
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = bf2f(f2bf(((kb >> q) & 1u) ? v[q] : 0.f));
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const uint2 h = *(const uint2*)((const bf16_t*)epi.aux + (mr + 16 * i) * epi.ld_aux + nc + 16 * j);
                        fv4& v = acc[i][j];
                        v[0] = bf2f(f2bf(__uint_as_float(h.x << 16) > 0.f ? v[0] : 0.f));
                        v[1] = bf2f(f2bf(__uint_as_float(h.x & 0xffff0000u) > 0.f ? v[1] : 0.f));
                        v[2] = bf2f(f2bf(__uint_as_float(h.y << 16) > 0.f ? v[2] : 0.f));
                        v[3] = bf2f(f2bf(__uint_as_float(h.y & 0xffff0000u) > 0.f ? v[3] : 0.f));
                    }
            }
#pragma unroll
            for (int ib = 0; ib < FM / 4; ++ib) {
                float* cp = epi.colpart + ((mr - (lane & 15) + 64 * ib) >> 6) * N + nc;
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    fv4 t;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float sum = ((acc[4 * ib][j][q] + acc[4 * ib + 1][j][q]) + acc[4 * ib + 2][j][q]) +
                                          acc[4 * ib + 3][j][q];
                        t[q] = row16_sum_dpp(sum);   // the 16 lanes of the column group = one DPP row
                    }
                    if ((lane & 15) == 0) *(fv4*)(cp + 16 * j) = t;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (FN == 4) {
                store_bf16_wide<FM>(acc, (bf16_t*)Cv, ldc, mr, nc);
            } else {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const fv4& v = acc[i][j];
                        *(uint2*)((bf16_t*)Cv + (mr + 16 * i) * ldc + nc + 16 * j) =
                            make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
                    }
            }
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
        } else if constexpr (EP == P8_BWD_BITS) {
            // ReLU backward from keep bits (bf16 output, beta 0: checked on the host)
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const uint2 w =
                    *(const uint2*)((const uint32_t*)epi.aux + (mr + 16 * i) * epi.ld_aux + ((nc - 4 * (lane >> 4)) >> 5));
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const uint32_t kb = relu_nib(w, j, lane);
                    fv4& v = acc[i][j];
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = ((kb >> q) & 1u) ? v[q] : 0.f;
                }
            }
            store_bf16_wide<FM>(acc, (bf16_t*)Cv, ldc, mr, nc);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
        } else if constexpr (EP == P8_RELU_BITS) {
            // bias + ReLU, bf16 output and its ReLU keep bits (checked on the host: bias, bf16, beta 0)
            uint32_t kb[FM][4];
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const float4 b = *(const float4*)(epi.bias + nc + 16 * j);
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    fv4& v = acc[i][j];
                    v[0] = fmaxf(v[0] + b.x, 0.f); v[1] = fmaxf(v[1] + b.y, 0.f);
                    v[2] = fmaxf(v[2] + b.z, 0.f); v[3] = fmaxf(v[3] + b.w, 0.f);
                    kb[i][j & 3] = nz4_bf16(make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])));
                }
            }
            store_bf16_wide<FM>(acc, (bf16_t*)Cv, ldc, mr, nc);
            relu_bits_store<FM>(kb, (uint32_t*)epi.aux, epi.ld_aux, mr, nc - 4 * (lane >> 4), lane);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
        } else if constexpr (EP == P8_BF16) {
            // STORE / BIAS / BIAS_RELU, bf16 output (host-checked: beta 0, split 1, bias present
            // for the bias kinds)
            const bool bias = epi.kind != CG_EPI_STORE, relu = epi.kind == CG_EPI_BIAS_RELU;
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const float4 b = bias ? *(const float4*)(epi.bias + nc + 16 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    fv4& v = acc[i][j];
                    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
                    if (relu) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
                    }
                }
            }
#ifdef CG_P8_WHATIF
            if (ldc < 0)   // what-if build: the item's stores skipped (a host-never-true test keeps the math)
#endif
            store_bf16_wide<FM>(acc, (bf16_t*)Cv, ldc, mr, nc);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
        } else if constexpr (EP == P8_RESID) {
            // x + dropout(acc + b) in fp32 (epi_store4's arithmetic and order), per 32-row half band:
            // its residual loaded before its first store (the item issues 8 FN loads and 2 FM FN stores
            // after the pieces in flight, so the loop's EPI_OPS = 2 FM allowance stays a lower bound)
            // the bias goes in first, for the whole item, so its registers are free before the
            // band's residual (64) and keep bits are live next to the 128 accumulators
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const float4 b = *(const float4*)(epi.bias + nc + 16 * j);
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    fv4& v = acc[i][j];
                    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
                }
            }
            const bool drop = epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr;
            // 32-row half bands t = (band t / 2, half t % 2), each half's residual loaded before the
            // previous half's stores: vmcnt counts loads and stores together, so a load issued after
            // them would wait for every earlier store of the item first (different rows, so an
            // in-place residual is read before any store can reach it)
            float4 r[2][FN];
            uint32_t nib[4][FN];
            auto load_half = [&](int t) {
                const int64_t mh = mr + 64 * (t >> 1) + 32 * (t & 1);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        r[i][j] = *(const float4*)(epi.resid + (mh + 16 * i) * epi.ld_resid + nc + 16 * j);
            };
            load_half(0);
#pragma unroll
            for (int t = 0; t < 2 * (FM / 4); ++t) {
                const int hb = t >> 1, hh = t & 1;
                const int64_t mb = mr + 64 * hb;
                if (hh == 0 && drop) drop_nibbles_rows<FN>(epi, stream, mb, nc, N, nib);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const int ii = 2 * hh + i;
                        fv4& v = acc[4 * hb + ii][j];
                        if (drop) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) v[q] = ((nib[ii][j] >> q) & 1u) ? v[q] * epi.dscale : 0.f;
                        }
                        v[0] = r[i][j].x + v[0]; v[1] = r[i][j].y + v[1]; v[2] = r[i][j].z + v[2]; v[3] = r[i][j].w + v[3];
                    }
                if (t + 1 < 2 * (FM / 4)) load_half(t + 1);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const int ii = 2 * hh + i;
                        fv4& v = acc[4 * hb + ii][j];
                        st_out16((float4*)((float*)Cv + (mb + 16 * ii) * ldc + nc + 16 * j),
                                 make_float4(v[0], v[1], v[2], v[3]));
                        v = fv4{0.f, 0.f, 0.f, 0.f};
                    }
            }
        } else {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int64_t m = mr + 16 * i, n = nc + 16 * j;
                    if (split_k > 1)
                        *(fv4*)(ws + ((int64_t)sp * M + m) * N + n) = acc[i][j];
                    else
                        epi_store4(acc[i][j], m, n, N, Cv, c_dtype, ldc, epi, stream);
                    acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
                }
        }
        ++cj;
    };

    if constexpr (SCH == 0) {
#pragma unroll
        for (int s = 0; s < NBUF - 1; ++s)
            if (s < total) issue_next(s);

        int cur = 0, ckt = 0;
        bool stored = false;  // the previous step ended an item: EPI_OPS stores are the youngest VMEM ops
        for (int g = 0; g < total; ++g) {
            // DMA steps issued after step g (they may stay in flight): min(NBUF-2, total-1-g)
            const int ahead = total - 1 - g;
            if (stored) {
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
            } else {
                if constexpr (NBUF >= 4) {
                    if (ahead >= 2) wait_vm<2 * LPT>();
                    else if (ahead == 1) wait_vm<LPT>();
                    else wait_vm<0>();
                } else if constexpr (NBUF == 3) {
                    if (ahead >= 1) wait_vm<LPT>();
                    else wait_vm<0>();
                } else {
                    wait_vm<0>();
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (g + NBUF - 1 < total) {
                int nb = cur + NBUF - 1;
                if (nb >= NBUF) nb -= NBUF;
                issue_next(nb);
            }
            const char* imgA = smem + cur * G::STAGE;
            const char* imgB = imgA + G::IMG_A;
            // LDS reads run one group ahead of the MFMAs that consume them (sched_barrier pins the order;
            // left alone the scheduler sinks each A read next to its MFMAs and waits lgkmcnt(0) on it):
            // [B0 A0] | [B1 A1(lo)] mfma0(lo) | [A1(hi)] mfma0(hi) | mfma1 -- A1(hi) reuses A0(lo)'s
            // registers, so a 128x64 wave tile stays inside 256 VGPRs at two waves per SIMD
            constexpr int FH = FM / 2;
            sv8 af0[FM], bf0[FN], af1[FM], bf1[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bf0[j] = frag<BT, BN>(imgB, wn * (BN / WN) + j * 16, 0, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i) af0[i] = frag<AT, BM>(imgA, wm * (BM / WM) + i * 16, 0, lane);
#pragma unroll
            for (int j = 0; j < FN; ++j) bf1[j] = frag<BT, BN>(imgB, wn * (BN / WN) + j * 16, 1, lane);
#pragma unroll
            for (int i = 0; i < FH; ++i) af1[i] = frag<AT, BM>(imgA, wm * (BM / WM) + i * 16, 1, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < FH; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma_bf16(bf0[j], af0[i], acc[i][j]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = FH; i < FM; ++i) af1[i] = frag<AT, BM>(imgA, wm * (BM / WM) + i * 16, 1, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = FH; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma_bf16(bf0[j], af0[i], acc[i][j]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma_bf16(bf1[j], af1[i], acc[i][j]);
            __builtin_amdgcn_sched_barrier(0);
            cur = cur + 1 == NBUF ? 0 : cur + 1;
            stored = false;
            if (++ckt == nk) {
                finish_item();
                ckt = 0;
                stored = true;
            }
        }
    } else {
        // Staggered 8-phase schedule (cdna guide §5 "The 256² 8-phase template"; MI355X_MICROARCH
        // "Two waves per SIMD").  A K-tile is 4 phases of 16 MFMAs, phase p = (k-half p>>1, row half
        // p&1) of the wave's 128x64 tile; each phase is a load section (this phase's fragments, the
        // DMA pieces due) and an MFMA section, each closed by a workgroup s_barrier.  Group 1 (waves
        // 4-7, wm = 1) runs one section behind group 0, so the two waves of every SIMD alternate
        // MFMA and LDS/DMA work.  A stage holds two k-halves (32-deep images, gemm_tile.h
        // img_row_off32 / the transposed image's first 32 k-rows); piece (t, h) = k-half h of K-tile
        // t, 4 DMA instructions per wave.  Piece order: ks0(0) ks1(0) ks0(1) | per tile t: ks1(t+1)
        // in phase 0, ks0(t+2) in phase 2 (each into a half whose last reader, group 1, finished
        // a section earlier).  Waits: ks1(t) before the barrier closing phase 1 of tile t, ks0(t+1)
        // before the one closing phase 3 -- in group 0's MFMA section and group 1's load section of
        // that phase, so every wave's pieces have landed before the first reader's load section.
        static_assert(WM == 2 && FM % 2 == 0, "staggered schedule: two wave groups along M");
        using DAh = Dma8h<AT, BM>;
        using DBh = Dma8h<BT, BN>;
        constexpr int LPH = DAh::PER_WAVE + DBh::PER_WAVE;   // DMA instructions per lane per piece
        constexpr int IMG_AH = BM * 64, HALF = IMG_AH + BN * 64;
        static_assert(2 * HALF == G::STAGE, "stage = two k-halves");
        constexpr int FH = FM / 2;
        DAh dah;
        DBh dbh;
        dah.init(lda, wave, lane);
        dbh.init(ldb, wave, lane);
        const bool grp = wm != 0;   // wave-uniform
        int pj = 0, pkt = 0;        // piece cursor: item, K-tile within it
        const bf16_t* pa = A;
        const bf16_t* pb = B;
        auto issue_piece = [&](int t, int h) {   // called in piece order
            if (pkt == 0 && h == 0) {
                int64_t m0, n0;
                int sp;
                decode(pj, m0, n0, sp);
                const int64_t kb = sp * kchunk;
                pa = AT ? A + kb * lda + m0 : A + m0 * lda + kb;
                pb = BT ? B + kb * ldb + n0 : B + n0 * ldb + kb;
            }
            const uint32_t img = lds_base(smem) + (uint32_t)((t & 1) * G::STAGE + h * HALF);
            dah.issue(pa, pkt, h, img, wave);
            dbh.issue(pb, pkt, h, img + IMG_AH, wave);
            if (h == 1 && ++pkt == nk) {
                pkt = 0;
                ++pj;
            }
        };
        // this wave's older pieces landed, `pieces` younger pieces (and the last item's output stores
        // when `stored`) may stay in flight
        auto wait_pieces = [&](int pieces, bool stored) {
            if (stored) {
                if (pieces >= 2) wait_vm<2 * LPH + EPI_OPS>();
                else if (pieces == 1) wait_vm<LPH + EPI_OPS>();
                else wait_vm<EPI_OPS>();
            } else {
                if (pieces >= 2) wait_vm<2 * LPH>();
                else if (pieces == 1) wait_vm<LPH>();
                else wait_vm<0>();
            }
        };
        if (total > 0) {
            issue_piece(0, 0);
            issue_piece(0, 1);
            if (total > 1) issue_piece(1, 0);
            wait_pieces(total > 1 ? 2 : 1, false);   // ks0(0)
            __builtin_amdgcn_s_barrier();
            if (grp) __builtin_amdgcn_s_barrier();
        }
        int ckt = 0;
        bool stored = false;   // tile g-1 ended an item: its EPI_OPS output stores are younger than the pieces waited in tile g
        for (int g = 0; g < total; ++g) {
            const char* stg = smem + (g & 1) * G::STAGE;
            sv8 bf[FN], af[FH];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int h = p >> 1, ih = p & 1;
                const char* imgA = stg + h * HALF;
                const char* imgB = imgA + IMG_AH;
                // the piece waited in this phase (odd phases) and how many younger ones this wave issued
                const bool wt = p == 1 || (p == 3 && g + 1 < total);
                const int younger = p == 1 ? (g + 1 < total ? 2 : 0) : 1 + (g + 2 < total ? 1 : 0);
                // ---- load section
                if (p == 0 && g + 1 < total) issue_piece(g + 1, 1);
                if (p == 2 && g + 2 < total) issue_piece(g + 2, 0);
                if (ih == 0) {
#pragma unroll
                    for (int j = 0; j < FN; ++j) bf[j] = frag32<BT, BN>(imgB, wn * (BN / WN) + j * 16, lane);
                }
#pragma unroll
                for (int i = 0; i < FH; ++i) af[i] = frag32<AT, BM>(imgA, wm * (BM / WM) + (ih * FH + i) * 16, lane);
                if (grp && wt) wait_pieces(younger, stored);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                // ---- MFMA section
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < FH; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[ih * FH + i][j] = mfma_bf16(bf[j], af[i], acc[ih * FH + i][j]);
                __builtin_amdgcn_s_setprio(0);
                if (!grp && wt) wait_pieces(younger, stored);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
            }
            stored = false;
            if (++ckt == nk) {
                finish_item();
                ckt = 0;
                stored = true;
            }
        }
        if (total > 0 && !grp) __builtin_amdgcn_s_barrier();   // group 1's extra barrier at the start
    }
    if (red.n) red_tail(red);   // a deferred split-K reduce of an earlier launch (gemm_common.h)
}

int cu_count8() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <int BM, int BN, int WM, int NBUF, int SCH = 0>
bool launch8(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
             int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
             hipStream_t st) {
    using G = Geo8<BM, BN, NBUF>;
    const int64_t kchunk = K / split_k;
    const int64_t nitems = (M / BM) * (N / BN) * split_k;
    const int occ = G::OCC;
    int64_t slots = (int64_t)cu_count8() * occ;
    if (g_gemm_max_grid > 0 && g_gemm_max_grid < slots) slots = g_gemm_max_grid;
    const unsigned grid = (unsigned)(nitems < slots ? nitems : slots);
#define FG(AT_, BT_, EP_)                                                                                \
    k_gemm_p8<AT_, BT_, BM, BN, WM, NBUF, EP_, SCH><<<grid, P8_THREADS, G::LDS, st>>>(M, N, K, A, lda, B, ldb, C,     \
                                                                                 c_dtype, ldc, e, split_k, kchunk, ws, \
                                                                                 g_gemm_group_p8, take_pending_reduces(st))
    // keep bits (host-checked: split 1, bf16 output, beta 0) need 64-column wave fragments (FN == 4)
    const bool bits = e.aux_dtype == CG_BITS;
    constexpr bool FN4 = BN / (8 / WM) == 64;
    if (bits) {
        if constexpr (FN4) {
            if (e.colpart && !at && bt) FG(false, true, P8_CP_BITS);
            else if (e.colpart && !at) FG(false, false, P8_CP_BITS);
            else if (e.kind == CG_EPI_BIAS_RELU && !at && !bt) FG(false, false, P8_RELU_BITS);
            else if (e.kind == CG_EPI_RELU_BWD && !at && bt) FG(false, true, P8_BWD_BITS);
            else return false;
            return true;
        }
        return false;
    }
    if (e.colpart) {   // non-transposed A, split 1, RELU_BWD with bf16 aux, bf16 output (host-checked)
        if (!bt) FG(false, false, P8_CP_BF16);
        else FG(false, true, P8_CP_BF16);
        return true;
    }
    if constexpr (FN4) {
        const bool plain = e.kind == CG_EPI_STORE || ((e.kind == CG_EPI_BIAS || e.kind == CG_EPI_BIAS_RELU) && e.bias);
        if (plain && !at && split_k == 1 && c_dtype == CG_BF16 && e.beta == 0.f) {
            if (!bt) FG(false, false, P8_BF16);
            else FG(false, true, P8_BF16);
            return true;
        }
    }
    if constexpr (FN4) {
        const bool resid = (e.kind == CG_EPI_BIAS_RESID || e.kind == CG_EPI_BIAS_DROP_RESID) && e.bias && e.resid;
        if (resid && !at && split_k == 1 && c_dtype == CG_F32 && e.beta == 0.f) {
            if (!bt) FG(false, false, P8_RESID);
            else FG(false, true, P8_RESID);
            return true;
        }
    }
    if (!at && !bt) FG(false, false, P8_GENERIC);
    else if (!at && bt) FG(false, true, P8_GENERIC);
    else if (at && !bt) FG(true, false, P8_GENERIC);
    else FG(true, true, P8_GENERIC);
#undef FG
    return true;
}

}  // namespace

// variants: 20 = automatic tile choice; 21 = 256x128 (NBUF 3); 22 = 128x256 (NBUF 3);
// 23 = 128x128 (NBUF 4); 24 = 256x256 (NBUF 2); 25 = 256x128 (NBUF 2)
// Returns false (nothing launched) if the chosen tile does not divide the problem.
bool p8_gemm_launch(int v, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                    const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                    float* ws, hipStream_t st) {
    if (K % (FBK * split_k)) return false;
#ifndef CG_AB_VARIANTS   // the default build has the 256x256 tile only (the others: `make ab`)
    if (v != 24) return false;
#endif
    if (v == 20) {
        // largest tile that divides the problem and still yields >= ~3/4 of a block per CU
        const int64_t cus = cu_count8();
        auto items = [&](int bm, int bn) { return (M / bm) * (N / bn) * split_k; };
        if (M % 256 == 0 && N % 128 == 0 && items(256, 128) >= (cus * 3) / 4) v = 21;
        else if (M % 128 == 0 && N % 256 == 0 && items(128, 256) >= (cus * 3) / 4) v = 22;
        else if (M % 128 == 0 && N % 128 == 0) v = 23;
        else return false;
    }
    switch (v) {
#ifdef CG_AB_VARIANTS
        case 21:
            if (M % 256 || N % 128) return false;
            return launch8<256, 128, 4, 3>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
        case 22:
            if (M % 128 || N % 256) return false;
            return launch8<128, 256, 2, 3>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
        case 23:
            if (M % 128 || N % 128) return false;
            return launch8<128, 128, 2, 4>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
        case 25:
            if (M % 256 || N % 128) return false;
            return launch8<256, 128, 4, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
#endif
        case 24:
            if (M % 256 || N % 256) return false;
            return launch8<256, 256, 2, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
#ifdef CG_AB_VARIANTS
        case 26:   // A/B: the same tile on the staggered 8-phase schedule (profiles/r5_gemm_p8_staggered_ab.txt)
            if (M % 256 || N % 256) return false;
            return launch8<256, 256, 2, 2, 1>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
#endif
        default:
            return false;
    }
}

}  // namespace cg
