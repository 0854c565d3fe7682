// charpt: bf16 MFMA GEMM for gfx950 -- the perf path of every nn.Linear forward, dgrad and wgrad
// (GPT1.py:111-112,121,136,143,145).  Register-staged variant + the variant dispatcher.
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
// row panel run on one XCD (shared L2).  The LDS-DMA variant lives in gemm_glds.hip.
#include "gemm_tile.h"

namespace cg {
namespace {
using namespace gt;

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
};

template <int BM, int BN>
struct Geo {
    static constexpr int WM = BM / 64, WN = BN / 64, WAVES = WM * WN, THREADS = WAVES * 64;
    static constexpr int IMG_A = BM * FBK * 2, IMG_B = BN * FBK * 2, STAGE = IMG_A + IMG_B;
    static constexpr int LDS = (2 * STAGE) > epi_lds_bytes<BN>() ? (2 * STAGE) : epi_lds_bytes<BN>();
};

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
            for (int i = 0; i < 4; ++i) af[i] = frag<AT, BM>(imgA, wm * 64 + i * 16, s, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = frag<BT, BN>(imgB, wn * 64 + j * 16, s, lane);
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
    epilogue<BM, BN>(acc, smem, tid, M, N, m0, n0, Cv, c_dtype, ldc, epi, split_k, split, ws);
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

// the kernel variant cg_gemm's bf16 dispatch runs for this problem (before any fallback)
static int pick_variant(int at, int bt, int64_t M, int64_t N, int split_k) {
    int v = g_gemm_variant;
    if (v == 0) {
        // persistent 128x128 LDS-DMA: measured best on the C2 shapes (profiles/r1_gemm_scan.txt); the
        // 8-wave 256x256 tile once there are >= 2 tiles per CU (C4 forward/dgrad: profiles/r1_gemm_scan_c4_v24.txt)
        // (the one-block-per-CU 128x192 tile, A/B variant 18, measured slower on the C2 N = 384
        // forwards than 128x128 tiles part-filling the two-per-CU slots: profiles/r3_gemm_128x192_ab.txt)
        (void)bt;
        const int64_t t256 = (M / 256) * (N / 256);
        v = (!at && split_k == 1 && M % 256 == 0 && N % 256 == 0 && t256 >= 2 * (int64_t)gemm_cu_count()) ? 24 : 9;
    }
    return v;
}

static bool fast_shape_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int split_k) {
    return N % 128 == 0 && K % FBK == 0 && K / FBK >= split_k && M % 128 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
           ldc % 8 == 0;
}

// the 128x128 persistent kernel (gemm_pk.hip); the A/B build also its 3- and 4-stage rings
#ifdef CG_AB_VARIANTS
static bool pk128(int v) { return v == 9 || v == 10 || v == 12; }
#else
static bool pk128(int v) { return v == 9; }
#endif

// column partials come from the 128x128 persistent kernel's per-item ReLU-backward epilogue (not its
// pk_flags bit-1 per-fragment form) and from the 8-wave 256x256 persistent kernel
static bool colpart_ok(int v, int at, int split_k) {
    return (v == 24 || v == 26 || (pk128(v) && !(g_pk_flags & 2))) && split_k == 1 && !at;
}

bool gemm_colpart_supported(int at, int bt, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
    return fast_shape_ok(M, N, K, lda, ldb, ldc, 1) && colpart_ok(pick_variant(at, bt, M, N, 1), at, 1);
}

// CG_BITS ReLU keep bits are written / read by the same two kernels' item epilogues (64-column
// wave fragments: k_gemm_pk 128x128, k_gemm_p8 256x256)
static bool relu_bits_ok(int v, int at, int split_k, int64_t N) {
    return colpart_ok(v, at, split_k) && N % 64 == 0;
}

bool gemm_relu_bits_supported(int at, int bt, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
    return fast_shape_ok(M, N, K, lda, ldb, ldc, 1) && relu_bits_ok(pick_variant(at, bt, M, N, 1), at, 1, N);
}

// the attention-delta epilogue (CG_EPI_STORE_ROWDOT) is the 128x128 persistent kernel's fixed kind:
// one wave's 64 output columns are one head
static bool rowdot_ok(int v, int at, int split_k, int64_t N) {
    return pk128(v) && !(g_pk_flags & 2) && split_k == 1 && !at && N % 64 == 0;
}

bool gemm_rowdot_supported(int at, int bt, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
    return fast_shape_ok(M, N, K, lda, ldb, ldc, 1) && rowdot_ok(pick_variant(at, bt, M, N, 1), at, 1, N);
}

bool fast_gemm_launch(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
                      int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
                      hipStream_t st) {
    if (!fast_shape_ok(M, N, K, lda, ldb, ldc, split_k)) return false;
    if ((((uintptr_t)A) | ((uintptr_t)B) | ((uintptr_t)C)) & 15) return false;
    if (e.bias && (((uintptr_t)e.bias) & 15)) return false;
    if (e.resid && ((((uintptr_t)e.resid) & 15) || e.ld_resid % 4)) return false;
    if (e.aux && ((((uintptr_t)e.aux) & 15) || e.ld_aux % 8)) return false;
    int v = pick_variant(at, bt, M, N, split_k);
    if (e.slab_bf16 && (!pk128(v) || split_k < 2 || e.kind != CG_EPI_STORE)) return false;
    if (K % (FBK * split_k)) {
        // uneven split-K (the last split shorter): only the 128x128 persistent kernel, and only when
        // every split is non-empty; otherwise the generic kernels (ceil-sized chunks) take it
        const int64_t nkt = K / FBK, nkc = (nkt + split_k - 1) / split_k;
        if (!pk128(v) || (split_k - 1) * nkc >= nkt) return false;
    }
    if (e.kind == CG_EPI_STORE_ROWDOT &&
        (!rowdot_ok(v, at, split_k, N) || !e.aux || e.aux_dtype != CG_BF16 || !e.colpart || e.ld_resid <= 0 ||
         M % e.ld_resid || e.beta != 0.f || c_dtype != CG_BF16 || (((uintptr_t)e.colpart) & 3)))
        return false;
    if (e.colpart && e.kind != CG_EPI_STORE_ROWDOT && (!colpart_ok(v, at, split_k) || e.kind != CG_EPI_RELU_BWD ||
                      (e.aux_dtype != CG_BF16 && e.aux_dtype != CG_BITS) || e.beta != 0.f || c_dtype != CG_BF16))
        return false;
    if (e.aux_dtype == CG_BITS &&
        (!relu_bits_ok(v, at, split_k, N) || (e.kind != CG_EPI_RELU_BWD && e.kind != CG_EPI_BIAS_RELU) ||
         (e.kind == CG_EPI_BIAS_RELU && !e.bias) || !e.aux || e.beta != 0.f || c_dtype != CG_BF16))
        return false;
    if (v >= 20 && p8_gemm_launch(v, at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st))
        return true;
    if (e.aux_dtype == CG_BITS && !pk128(v)) return false;   // only the two persistent kernels read / write keep bits
    if (v >= 20) v = 2;
#ifdef CG_AB_VARIANTS   // the LDS-DMA variants 5-8 (ab/gemm_glds.hip), else the persistent kernels
    if (v >= 5 && glds_gemm_launch(v, at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st))
        return true;
#else
    if (v >= 5 && pk_gemm_launch(v, at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st))
        return true;
#endif
#ifdef CG_AB_VARIANTS
    if ((v == 3 || v == 4) && M % 256) v = 1;
    switch (v) {
        case 3: launch<256, 128, 1>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        case 4: launch<256, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        case 1: launch<128, 128, 1>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        default: break;
    }
#endif
    // the register-staged 128x128 kernel: the fallback when the persistent tile cannot take the call
    launch<128, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
    return true;
}

}  // namespace cg
