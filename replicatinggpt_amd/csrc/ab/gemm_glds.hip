// charpt: bf16 MFMA GEMM, LDS-DMA staged (gfx950 global_load_lds_dwordx4) -- same contract and
// epilogues as gemm_bf16.hip (GPT1.py:111-112,121,136,143,145 nn.Linear forward/dgrad/wgrad).
//
// Operand tiles go HBM/L2 -> LDS directly (no register staging), NBUF LDS stages deep: NBUF-1
// K-tiles stay in flight while the block computes on the current one.  Per K-tile: counted
// `s_waitcnt vmcnt` (own DMA of this tile done) -> raw s_barrier (everyone's DMA done, everyone
// finished the previous tile) -> issue the DMA for tile kt+NBUF-1 into the stage just freed ->
// MFMAs.  The LDS-DMA destination is linear per wave instruction (base + 16*lane), so the XOR
// swizzle of the images (gemm_tile.h) is applied to the per-lane GLOBAL source address instead
// (the source permutation and the read permutation are the same involution).
// A/B-only (never the product library: `make ab`, CG_AB_VARIANTS): measured slower than gemm_pk.hip.
#include "../gemm_tile.h"

namespace cg {
namespace {
using namespace gt;

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA loader for one operand tile: R rows (K-contiguous) or R columns (TR, M/N-contiguous) x 64 k
template <bool TR, int R, int WAVES>
struct Dma {
    static constexpr int INSTR = R * FBK * 2 / 1024;  // 1-KB wave instructions per tile
    static constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(PER_WAVE * WAVES == INSTR, "tile/wave mismatch");
    static_assert(!TR || R >= 128, "transposed image swizzle needs >= 16 chunks per row");
    const bf16_t* src[PER_WAVE];  // per-lane source of K-tile 0
    int64_t kstep;                // elements between consecutive K-tiles

    __device__ __forceinline__ void init(const bf16_t* X, int64_t ld, int64_t r0, int64_t kb, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) {
            const int pos = (wave * PER_WAVE + i) * 1024 + lane * 16;
            if (!TR) {
                const int r = pos >> 7, c = ((pos >> 4) & 7) ^ row_swz(r);
                src[i] = X + (r0 + r) * ld + kb + c * 8;
            } else {
                const int k = pos / (2 * R), c = ((pos % (2 * R)) >> 4) ^ col_swz(k);
                src[i] = X + (kb + k) * ld + r0 + c * 8;
            }
        }
        kstep = TR ? (int64_t)FBK * ld : (int64_t)FBK;
    }
    __device__ __forceinline__ void issue(int kt, char* img, int wave) const {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * kstep),
                                             (lds_void*)(img + (wave * PER_WAVE + i) * 1024), 16, 0, 0);
    }
};

template <int BM, int BN, int NBUF>
struct GeoD {
    static constexpr int WM = BM / 64, WN = BN / 64, WAVES = WM * WN, THREADS = WAVES * 64;
    static constexpr int IMG_A = BM * FBK * 2, IMG_B = BN * FBK * 2, STAGE = IMG_A + IMG_B;
    static constexpr int LDS = (NBUF * STAGE) > epi_lds_bytes<BN>() ? (NBUF * STAGE) : epi_lds_bytes<BN>();
    static constexpr int OCC = LDS <= 80 * 1024 ? 2 : 1;
};

template <bool AT, bool BT, int BM, int BN, int NBUF>
__global__ __launch_bounds__((BM / 64) * (BN / 64) * 64, ((BM + BN) * 128 * NBUF <= 80 * 1024 ? 2 : 1))
void k_gemm_glds(int64_t M, int64_t N, int64_t K, const bf16_t* __restrict__ A, int64_t lda,
                 const bf16_t* __restrict__ B, int64_t ldb, void* __restrict__ Cv, int c_dtype, int64_t ldc,
                 EpiArgs epi, int split_k, int64_t kchunk, float* __restrict__ ws) {
    using G = GeoD<BM, BN, NBUF>;
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

    Dma<AT, BM, G::WAVES> da;
    Dma<BT, BN, G::WAVES> db;
    da.init(A, lda, m0, kb, wave, lane);
    db.init(B, ldb, n0, kb, wave, lane);
    constexpr int LPT = Dma<AT, BM, G::WAVES>::PER_WAVE + Dma<BT, BN, G::WAVES>::PER_WAVE;

    fv4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int kt, int buf) {
        char* img = smem + buf * G::STAGE;
        da.issue(kt, img, wave);
        db.issue(kt, img + G::IMG_A, wave);
    };
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

#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s)
        if (s < nk) issue(s, s);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
        // tiles issued after kt that may stay in flight: min(NBUF-2, nk-1-kt)
        const int ahead = nk - 1 - kt;
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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + NBUF - 1 < nk) {
            int nb = cur + NBUF - 1;
            if (nb >= NBUF) nb -= NBUF;
            issue(kt + NBUF - 1, nb);
        }
        compute(smem + cur * G::STAGE);
        cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
    __syncthreads();
    epilogue<BM, BN>(acc, smem, tid, M, N, m0, n0, Cv, c_dtype, ldc, epi, split_k, split, ws);
}

template <int BM, int BN, int NBUF>
void launch_d(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
              int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
              hipStream_t st) {
    using G = GeoD<BM, BN, NBUF>;
    const int64_t kchunk = K / split_k;
    dim3 grid((unsigned)((M / BM) * (N / BN)), (unsigned)split_k);
#define FG(AT_, BT_)                                                                                               \
    k_gemm_glds<AT_, BT_, BM, BN, NBUF><<<grid, G::THREADS, G::LDS, st>>>(M, N, K, A, lda, B, ldb, C, c_dtype, ldc, \
                                                                        e, split_k, kchunk, ws)
    if (!at && !bt) FG(false, false);
    else if (!at && bt) FG(false, true);
    else if (at && !bt) FG(true, false);
    else FG(true, true);
#undef FG
}

}  // namespace

bool glds_gemm_launch(int v, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                      const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                      float* ws, hipStream_t st) {
    switch (v) {
        case 5: launch_d<128, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        case 6: launch_d<128, 128, 3>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        case 7:
            if (M % 256) return false;
            launch_d<256, 128, 2>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
            return true;
        case 8: launch_d<128, 128, 4>(at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st); return true;
        default: return pk_gemm_launch(v, at, bt, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k, ws, st);
    }
}

}  // namespace cg
