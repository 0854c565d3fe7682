// charpt: bf16 MFMA GEMM for gfx950 -- the perf path of every nn.Linear forward, dgrad and wgrad
// (GPT1.py:111-112,121,136,143,145).
//
//   C[m,n] = epilogue( sum_k A(m,k) * B(n,k) ),  A(m,k) = A[m*lda+k] | A[k*lda+m] (AT),
//                                                B(n,k) = B[n*ldb+k] | B[k*ldb+n] (BT).
//
// Block tile BM x BN x 64, one wave per 64x64 sub-tile (4x4 MFMA 16x16x32 bf16 tiles, fp32
// accumulators).  Global -> registers -> LDS staging, PREF K-tiles in flight, double-buffered LDS,
// one barrier per K-tile.  LDS images are XOR-swizzled: K-contiguous operands are read with
// ds_read_b128, M/N-contiguous operands ("transposed": dgrad weights, both wgrad operands) with the
// gfx950 transpose read ds_read_b64_tr_b16, so NT / NN / TN products share the kernel.
// Epilogue staged through LDS, 8 consecutive columns per lane (16-B stores), fused bias / ReLU /
// Philox dropout / residual / ReLU-backward.  Blocks are remapped so that the column tiles of one
// row panel run on one XCD (shared L2).
#include "gemm_common.h"

namespace cg {
namespace {

constexpr int FBK = 64;

typedef __attribute__((address_space(3))) sv4 lds_sv4;

// ---- LDS images -------------------------------------------------------------------------
// K-contiguous image of R rows: [R][64] bf16, 128-B rows, chunk c (16 B, 0..7) at c ^ ((r>>1)&7)
__device__ __forceinline__ int img_row_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// M/N-contiguous image of R columns: [64 k][R] bf16, rows of 2R bytes, chunk c (0..R/8-1); the low
// 4 chunk bits are XORed with ((k&3)<<2 | (k>>2)&3)  (cdna guide T10, layout (b))
template <int R>
__device__ __forceinline__ int img_col_off(int k, int c) {
    return k * (2 * R) + ((c ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 4);
}

template <bool TR, int R, int THREADS>
struct Operand {
    static constexpr int BYTES = R * FBK * 2;
    static constexpr int NCH = BYTES / (THREADS * 16);  // 16-B chunks per thread per K-tile
    static_assert(NCH >= 1 && NCH * THREADS * 16 == BYTES, "tile/thread mismatch");
    struct Stage {
        uint4 v[NCH];
    };
    static __device__ __forceinline__ Stage load(const bf16_t* __restrict__ X, int64_t ld, int64_t r0, int64_t k0,
                                                 int tid) {
        Stage s;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int lin = tid + i * THREADS;
            if (!TR) {
                const int r = lin >> 3, c = lin & 7;
                s.v[i] = *(const uint4*)(X + (r0 + r) * ld + k0 + c * 8);
            } else {
                constexpr int CPR = R / 8;
                const int k = lin / CPR, c = lin % CPR;
                s.v[i] = *(const uint4*)(X + (k0 + k) * ld + r0 + c * 8);
            }
        }
        return s;
    }
    static __device__ __forceinline__ void store(const Stage& s, char* img, int tid) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int lin = tid + i * THREADS;
            if (!TR) {
                const int r = lin >> 3, c = lin & 7;
                *(uint4*)(img + img_row_off(r, c)) = s.v[i];
            } else {
                constexpr int CPR = R / 8;
                const int k = lin / CPR, c = lin % CPR;
                *(uint4*)(img + img_col_off<R>(k, c)) = s.v[i];
            }
        }
    }
    // MFMA 16x16x32 operand fragment: tile rows rb..rb+15, k = 32s..32s+31.
    // lane l holds X(rb + (l&15), 32s + 8(l>>4) + j), j = 0..7
    static __device__ __forceinline__ sv8 frag(const char* img, int rb, int s, int lane) {
        if (!TR) {
            return *(const sv8*)(img + img_row_off(rb + (lane & 15), s * 4 + (lane >> 4)));
        } else {
            const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
            const int ka = 32 * s + 8 * g;
            const int chunk = (rb >> 3) + (p >> 1), byte = 8 * (p & 1);
            const sv4 lo =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_col_off<R>(ka + q, chunk) + byte));
            const sv4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_col_off<R>(ka + 4 + q, chunk) + byte));
            return sv8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
    }
};

__device__ __forceinline__ fv4 mfma_bf16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

// bijective XCD-aware remap (cdna guide §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int BM, int BN>
struct Geo {
    static constexpr int WM = BM / 64, WN = BN / 64, WAVES = WM * WN, THREADS = WAVES * 64;
    static constexpr int IMG_A = BM * FBK * 2, IMG_B = BN * FBK * 2, STAGE = IMG_A + IMG_B;
    static constexpr int CS_LD = BN + 4;                       // epilogue staging row stride (floats)
    static constexpr int EPI_ROWS = 128;                        // rows staged per epilogue round
    static constexpr int EPI_BYTES = EPI_ROWS * CS_LD * 4;
    static constexpr int LDS = (2 * STAGE) > EPI_BYTES ? (2 * STAGE) : EPI_BYTES;
};

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
        const uint64_t idx = (uint64_t)m * (uint64_t)N + (uint64_t)n;
        const u32x4 r0 = philox_group(epi.seed, stream, idx >> 2);
        const u32x4 r1 = philox_group(epi.seed, stream, (idx >> 2) + 1);
        const uint32_t w[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = w[q] >= epi.thr ? v[q] * epi.dscale : 0.f;
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

template <bool AT, bool BT, int BM, int BN, int PREF>
__global__ __launch_bounds__((BM / 64) * (BN / 64) * 64, 2)
void k_gemm_bf16(int64_t M, int64_t N, int64_t K, const bf16_t* __restrict__ A, int64_t lda,
                 const bf16_t* __restrict__ B, int64_t ldb, void* __restrict__ Cv, int c_dtype, int64_t ldc,
                 EpiArgs epi, int split_k, int64_t kchunk, float* __restrict__ ws) {
    using G = Geo<BM, BN>;
    using OA = Operand<AT, BM, G::THREADS>;
    using OB = Operand<BT, BN, G::THREADS>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / G::WN, wn = wave % G::WN;
    const int tilesN = (int)(N / BN);
    const int ntiles = (int)(M / BM) * tilesN;
    const int t = xcd_remap(blockIdx.x, ntiles);
    const int64_t m0 = (int64_t)(t / tilesN) * BM, n0 = (int64_t)(t % tilesN) * BN;
    const int split = blockIdx.y;
    const int64_t kb = split * kchunk;
    const int nk = (int)(kchunk / FBK);

    fv4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    auto kaddr = [&](int kt) { return kb + (int64_t)(kt < nk ? kt : nk - 1) * FBK; };
    auto compute = [&](const char* img) {
        const char* imgA = img;
        const char* imgB = img + G::IMG_A;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            sv8 af[4], bf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = OA::frag(imgA, wm * 64 + i * 16, s, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = OB::frag(imgB, wn * 64 + j * 16, s, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma_bf16(af[i], bf[j], acc[i][j]);
        }
    };

    if constexpr (PREF == 1) {
        {
            const auto ga = OA::load(A, lda, m0, kaddr(0), tid);
            const auto gb = OB::load(B, ldb, n0, kaddr(0), tid);
            OA::store(ga, smem, tid);
            OB::store(gb, smem + G::IMG_A, tid);
        }
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const auto ga = OA::load(A, lda, m0, kaddr(kt + 1), tid);
            const auto gb = OB::load(B, ldb, n0, kaddr(kt + 1), tid);
            compute(smem + (kt & 1) * G::STAGE);
            char* nxt = smem + ((kt + 1) & 1) * G::STAGE;
            OA::store(ga, nxt, tid);
            OB::store(gb, nxt + G::IMG_A, tid);
            __syncthreads();
        }
    } else {
        // two K-tiles in flight: register sets P (even tiles) and Q (odd tiles)
        auto pa = OA::load(A, lda, m0, kaddr(0), tid);
        auto pb = OB::load(B, ldb, n0, kaddr(0), tid);
        auto qa = OA::load(A, lda, m0, kaddr(1), tid);
        auto qb = OB::load(B, ldb, n0, kaddr(1), tid);
        OA::store(pa, smem, tid);
        OB::store(pb, smem + G::IMG_A, tid);
        __syncthreads();
        for (int kt = 0; kt < nk; kt += 2) {
            // even: LDS[0] holds tile kt, Q holds kt+1
            pa = OA::load(A, lda, m0, kaddr(kt + 2), tid);
            pb = OB::load(B, ldb, n0, kaddr(kt + 2), tid);
            compute(smem);
            OA::store(qa, smem + G::STAGE, tid);
            OB::store(qb, smem + G::STAGE + G::IMG_A, tid);
            __syncthreads();
            if (kt + 1 >= nk) break;
            // odd: LDS[1] holds tile kt+1, P holds kt+2
            qa = OA::load(A, lda, m0, kaddr(kt + 3), tid);
            qb = OB::load(B, ldb, n0, kaddr(kt + 3), tid);
            compute(smem + G::STAGE);
            OA::store(pa, smem, tid);
            OB::store(pb, smem + G::IMG_A, tid);
            __syncthreads();
        }
    }

    // ---- epilogue: accumulators -> LDS (fp32, 128-row rounds) -> 8 consecutive columns per lane
    float* Cs = (float*)smem;
    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
#pragma unroll
    for (int round = 0; round < BM / G::EPI_ROWS; ++round) {
        if (wm / 2 == round) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        Cs[((wm & 1) * 64 + i * 16 + 4 * (lane >> 4) + r) * G::CS_LD + wn * 64 + j * 16 + (lane & 15)] =
                            acc[i][j][r];
        }
        __syncthreads();
        constexpr int CPR = BN / 8;  // 8-column groups per row
#pragma unroll 1
        for (int idx = tid; idx < G::EPI_ROWS * CPR; idx += G::THREADS) {
            const int row = idx / CPR, col = (idx % CPR) * 8;
            const int64_t m = m0 + round * G::EPI_ROWS + row, n = n0 + col;
            float v[8];
            const float4 x0 = *(const float4*)(Cs + row * G::CS_LD + col);
            const float4 x1 = *(const float4*)(Cs + row * G::CS_LD + col + 4);
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
        if (round + 1 < BM / G::EPI_ROWS) __syncthreads();
    }
}

template <int BM, int BN, int PREF>
void launch(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
            int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
            hipStream_t st) {
    using G = Geo<BM, BN>;
    const int64_t kchunk = K / split_k;
    dim3 grid((unsigned)((M / BM) * (N / BN)), (unsigned)split_k);
#define FG(AT_, BT_)                                                                                              \
    k_gemm_bf16<AT_, BT_, BM, BN, PREF><<<grid, G::THREADS, G::LDS, st>>>(M, N, K, A, lda, B, ldb, C, c_dtype, ldc, \
                                                                        e, split_k, kchunk, ws)
    if (!at && !bt) FG(false, false);
    else if (!at && bt) FG(false, true);
    else if (at && !bt) FG(true, false);
    else FG(true, true);
#undef FG
}

}  // namespace

bool fast_gemm_launch(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
                      int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
                      hipStream_t st) {
    if (N % 128 || K % (FBK * split_k) || M % 128) return false;
    if (lda % 8 || ldb % 8 || ldc % 8) return false;
    if ((((uintptr_t)A) | ((uintptr_t)B) | ((uintptr_t)C)) & 15) return false;
    if (e.bias && (((uintptr_t)e.bias) & 15)) return false;
    if (e.resid && ((((uintptr_t)e.resid) & 15) || e.ld_resid % 4)) return false;
    if (e.aux && ((((uintptr_t)e.aux) & 15) || e.ld_aux % 8)) return false;
    int v = g_gemm_variant;
    if (v == 0) v = 2;  // measured best on MI355X for every C2/C4 shape (tools/gemm_tune.py)
    if ((v == 3 || v == 4) && M % 256) v = 1;
    switch (v) {
        case 2: launch<128, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); break;
        case 3: launch<256, 128, 1>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); break;
        case 4: launch<256, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); break;
        default: launch<128, 128, 1>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); break;
    }
    return true;
}

}  // namespace cg
