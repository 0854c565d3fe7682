// charpt: GEMMs for every nn.Linear in the hot path (GPT1.py:111-112,121,136,143,145,184),
// their dgrad/wgrad in the backward, and bias-gradient column sums.
//
//   C[m,n] = epilogue( sum_k A(m,k) * B(n,k) ),  A(m,k) = A[m*lda+k] | A[k*lda+m] (a_trans),
//                                                B(n,k) = B[n*ldb+k] | B[k*ldb+n] (b_trans).
//
// Two kernels:
//   * k_gemm_bf16  -- the perf path: 128x128x64 tiles, 4 waves (2x2, 64x64 each), bf16 MFMA
//     16x16x32 with fp32 accumulation, register-staged double-buffered LDS (one barrier per
//     K-tile), XOR-swizzled LDS images: K-contiguous operands are read with ds_read_b128,
//     M/N-contiguous ("transposed") operands with the gfx950 transpose read ds_read_b64_tr_b16,
//     so forward (NT), dgrad (NN) and wgrad (TN) share one kernel.  Epilogue staged through LDS
//     and stored 16 B per lane.  Needs M%128 = N%128 = K%64 = 0, 16-B aligned rows.
//   * k_gemm_generic -- exact-f32 MFMA (16x16x4 f32) on 64x64x16 tiles with bounds checks:
//     any shape/stride/dtype; the fp32 parity path and odd shapes (n_embd=126, V=65).
// Both support deterministic split-K through fp32 slabs reduced in a fixed order.
#include <map>

#include "defer.h"
#include "gemm_common.h"
#include "ln_fwd.h"

using namespace cg;

namespace {

// =====================================================================================
// generic exact-f32 GEMM
// =====================================================================================
constexpr int GBM = 64, GBN = 64, GBK = 16;

template <typename TA, typename TB, typename TC>
__global__ __launch_bounds__(256) void k_gemm_generic(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K,
                                                      const TA* __restrict__ A, int64_t lda,
                                                      const TB* __restrict__ B, int64_t ldb, TC* __restrict__ C,
                                                      int64_t ldc, EpiArgs epi, int split_k, int64_t kchunk,
                                                      float* __restrict__ ws) {
    __shared__ float As[GBK][GBM + 4];
    __shared__ float Bs[GBK][GBN + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t tilesN = (N + GBN - 1) / GBN;
    const int64_t m0 = (int64_t)(blockIdx.x / tilesN) * GBM;
    const int64_t n0 = (int64_t)(blockIdx.x % tilesN) * GBN;
    const int split = blockIdx.y;
    const int64_t kb = split * kchunk;
    const int64_t ke = kb + kchunk < K ? kb + kchunk : K;

    fv4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    for (int64_t k0 = kb; k0 < ke; k0 += GBK) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int mm, kk;
            if (!a_trans) {
                kk = tid & 15;
                mm = (tid >> 4) + 16 * i;
            } else {
                mm = tid & 63;
                kk = (tid >> 6) + 4 * i;
            }
            const int64_t gm = m0 + mm, gk = k0 + kk;
            float v = 0.f;
            if (gm < M && gk < ke) v = ld_as_f32<TA>(A + (a_trans ? gk * lda + gm : gm * lda + gk));
            As[kk][mm] = v;
            int nn;
            if (!b_trans) {
                kk = tid & 15;
                nn = (tid >> 4) + 16 * i;
            } else {
                nn = tid & 63;
                kk = (tid >> 6) + 4 * i;
            }
            const int64_t gn = n0 + nn, gk2 = k0 + kk;
            float w = 0.f;
            if (gn < N && gk2 < ke) w = ld_as_f32<TB>(B + (b_trans ? gk2 * ldb + gn : gn * ldb + gk2));
            Bs[kk][nn] = w;
        }
        __syncthreads();
#pragma unroll
        for (int k4 = 0; k4 < GBK / 4; ++k4) {
            const int kr = k4 * 4 + (lane >> 4);
            float a0 = As[kr][wm * 32 + (lane & 15)];
            float a1 = As[kr][wm * 32 + 16 + (lane & 15)];
            float b0 = Bs[kr][wn * 32 + (lane & 15)];
            float b1 = Bs[kr][wn * 32 + 16 + (lane & 15)];
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }

    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + wm * 32 + mt * 16 + 4 * (lane >> 4) + r;
                const int64_t n = n0 + wn * 32 + nt * 16 + (lane & 15);
                if (m < M && n < N) {
                    if (split_k > 1) {
                        ws[((int64_t)split * M + m) * N + n] = acc[mt][nt][r];
                    } else {
                        store_out<TC>(C, m * ldc + n, epi_scalar(epi, acc[mt][nt][r], m, n, N, stream), epi.beta);
                    }
                }
            }
}

// ---------------------------------------------------------------------------------------
// fp32 MFMA GEMM (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation) -- the exact
// (dtype="fp32") model path: parity runs, the as-shipped fp32 training and generate() on
// model.pth.  128 x 64 block tile, BK = 16, 4 waves of 64 x 32; operand tiles staged k-major in
// LDS ([k][rows], so a fragment read is 16 consecutive floats) with the next K-tile prefetched
// into registers during the MFMAs; any M / N / K (masked), all four layouts, split-K slabs.
// ---------------------------------------------------------------------------------------
constexpr int FBM = 128, FBN = 64, FBKK = 16;

template <bool TR, int R>
struct F32Tile {
    static constexpr int PER = R * FBKK / 256;  // elements per thread
    float v[PER];
    __device__ __forceinline__ void load(const float* __restrict__ X, int64_t ld, int64_t r0, int64_t rmax,
                                         int64_t k0, int64_t kmax, int tid) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int lin = tid + 256 * i;
            int r, kk;
            if (!TR) { kk = lin % FBKK; r = lin / FBKK; }
            else { r = lin % R; kk = lin / R; }
            const int64_t gr = r0 + r, gk = k0 + kk;
            v[i] = (gr < rmax && gk < kmax) ? (TR ? X[gk * ld + gr] : X[gr * ld + gk]) : 0.f;
        }
    }
    __device__ __forceinline__ void store(float* Xs, int tid) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int lin = tid + 256 * i;
            int r, kk;
            if (!TR) { kk = lin % FBKK; r = lin / FBKK; }
            else { r = lin % R; kk = lin / R; }
            Xs[kk * (R + 4) + r] = v[i];
        }
    }
};

template <bool AT, bool BT>
__global__ __launch_bounds__(256, 2) void k_gemm_f32(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                     int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                     float* __restrict__ C, int64_t ldc, EpiArgs epi, int split_k,
                                                     int64_t kchunk, float* __restrict__ ws) {
    __shared__ float As[FBKK * (FBM + 4)];
    __shared__ float Bs[FBKK * (FBN + 4)];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, g = lane >> 4, li = lane & 15;
    const int64_t tilesN = (N + FBN - 1) / FBN;
    const int64_t m0 = (int64_t)(blockIdx.x / tilesN) * FBM, n0 = (int64_t)(blockIdx.x % tilesN) * FBN;
    const int split = blockIdx.y;
    const int64_t kb = split * kchunk, ke = kb + kchunk < K ? kb + kchunk : K;
    fv4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = fv4{0.f, 0.f, 0.f, 0.f};
    F32Tile<AT, FBM> ta;
    F32Tile<BT, FBN> tb;
    ta.load(A, lda, m0, M, kb, ke, tid);
    tb.load(B, ldb, n0, N, kb, ke, tid);
    for (int64_t k0 = kb; k0 < ke; k0 += FBKK) {
        __syncthreads();
        ta.store(As, tid);
        tb.store(Bs, tid);
        __syncthreads();
        if (k0 + FBKK < ke) {
            ta.load(A, lda, m0, M, k0 + FBKK, ke, tid);
            tb.load(B, ldb, n0, N, k0 + FBKK, ke, tid);
        }
#pragma unroll
        for (int k4 = 0; k4 < FBKK / 4; ++k4) {
            const int kr = 4 * k4 + g;
            float a[4], b[2];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[kr * (FBM + 4) + wm * 64 + 16 * i + li];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[kr * (FBN + 4) + wn * 32 + 16 * j + li];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    }
    const int kind = epi.kind;
    if (split_k == 1 && epi.beta == 0.f &&
        (kind == CG_EPI_STORE || kind == CG_EPI_BIAS || kind == CG_EPI_BIAS_RELU || kind == CG_EPI_BIAS_RESID)) {
        // every operand of the tile's epilogue (bias, residual) loaded before its first store: loaded
        // per element (epi_scalar + store_out), each load waited for every earlier store too (vmcnt
        // counts both), one HBM round trip per output element of the lane.  Same arithmetic and
        // order as epi_scalar: bias added only when present, ReLU, then resid + v.
        const bool hb = kind != CG_EPI_STORE && epi.bias, hr = kind == CG_EPI_BIAS_RESID && epi.resid;
        float bv[2] = {0.f, 0.f}, rv[2][2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t n = n0 + wn * 32 + 16 * j + li;
            if (hb && n < N) bv[j] = epi.bias[n];
        }
        // row fragments in two halves (i = 0-1, 2-3): each half's residuals loaded before the previous
        // half's stores, one half's registers live at a time
        auto load_half = [&](int hf) {
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t m = m0 + wm * 64 + 16 * (2 * hf + ii) + 4 * g + r;
                        const int64_t n = n0 + wn * 32 + 16 * j + li;
                        rv[ii][j][r] = (hr && m < M && n < N) ? epi.resid[m * epi.ld_resid + n] : 0.f;
                    }
        };
        load_half(0);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 2 * hf + ii;
                        float v = acc[i][j][r];
                        if (hb) v += bv[j];
                        if (kind == CG_EPI_BIAS_RELU) v = fmaxf(v, 0.f);
                        if (hr) v = rv[ii][j][r] + v;
                        acc[i][j][r] = v;
                    }
            if (hf == 0) load_half(1);
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 2 * hf + ii;
                        const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
                        const int64_t n = n0 + wn * 32 + 16 * j + li;
                        if (m < M && n < N) C[m * ldc + n] = acc[i][j][r];
                    }
        }
        return;
    }
    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
                const int64_t n = n0 + wn * 32 + 16 * j + li;
                if (m < M && n < N) {
                    if (split_k > 1)
                        ws[((int64_t)split * M + m) * N + n] = acc[i][j][r];
                    else
                        store_out<float>(C, m * ldc + n, epi_scalar(epi, acc[i][j][r], m, n, N, stream), epi.beta);
                }
            }
}

// ---------------------------------------------------------------------------------------
// fp32 forward (NT) products with few rows (M <= 2048: generate()'s per-token steps, 256 rows) --
// k_gemm_f32's 128 x 64 tiles leave most CUs idle there and pay a global-load round trip per 16-deep
// K-step.  One wave per 32 x 32 tile: each 128-deep K chunk's operands (a lane's A / B values for 32
// k4-steps) are loaded straight to registers, all in flight together, then its MFMAs.  The same
// v_mfma_f32_16x16x4_f32 lane / k assignment, k order and zero-padded K (to a multiple of 16) as
// k_gemm_f32, and its epilogue arithmetic with the operands loaded before the stores: bitwise its
// result.
template <int EK>
__global__ __launch_bounds__(64) void k_gemm_f32s(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                  int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                  float* __restrict__ C, int64_t ldc, EpiArgs epi) {
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int64_t m0 = (int64_t)blockIdx.x * 32, n0 = (int64_t)blockIdx.y * 32;
    const int64_t kpad = (K + 15) / 16 * 16;   // k_gemm_f32's padded depth
    fv4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = fv4{0.f, 0.f, 0.f, 0.f};
    const int64_t ra0 = m0 + li, ra1 = m0 + 16 + li, rb0 = n0 + li, rb1 = n0 + 16 + li;
    for (int64_t kc = 0; kc < kpad; kc += 128) {
        float a[2][32], b[2][32];
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int64_t k = kc + 4 * t + g;
            const bool kin = k < K;
            a[0][t] = (kin && ra0 < M) ? A[ra0 * lda + k] : 0.f;
            a[1][t] = (kin && ra1 < M) ? A[ra1 * lda + k] : 0.f;
            b[0][t] = (kin && rb0 < N) ? B[rb0 * ldb + k] : 0.f;
            b[1][t] = (kin && rb1 < N) ? B[rb1 * ldb + k] : 0.f;
        }
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            if (kc + 4 * t < kpad) {   // wave-uniform: k_gemm_f32's k4-steps only
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
            }
        }
    }
    constexpr bool BIAS = EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_BIAS_RESID;
    const bool hb = BIAS && epi.bias, hr = EK == CG_EPI_BIAS_RESID && epi.resid;
    float bv[2] = {0.f, 0.f}, rv[2][2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int64_t n = n0 + 16 * j + li;
        if (hb && n < N) bv[j] = epi.bias[n];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + 16 * i + 4 * g + r, n = n0 + 16 * j + li;
                rv[i][j][r] = (hr && m < M && n < N) ? epi.resid[m * epi.ld_resid + n] : 0.f;
            }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + 16 * i + 4 * g + r, n = n0 + 16 * j + li;
                float v = acc[i][j][r];
                if (hb) v += bv[j];
                if (EK == CG_EPI_BIAS_RELU) v = fmaxf(v, 0.f);
                if (hr) v = rv[i][j][r] + v;
                if (m < M && n < N) C[m * ldc + n] = v;
            }
}

// The same products with the whole K slab resident (K <= 624, even; 8-B aligned rows): one 4-wave block per
// 32 x 32 tile loads its 32 A rows and 32 B rows once (every float2 of the slab in flight together,
// coalesced along K) into LDS, then each wave runs its 16 x 16 fragment's MFMA chain from LDS.  k_gemm_f32s
// walked K in 128-deep register chunks, one load round trip each, on 32 waves for the C5 FFN2 (19 us).
// Same lane / k order, padded depth and epilogue as k_gemm_f32: bitwise its result.
// Every global load is unconditional at a clamped address (row M - 1, column K - 2), the zero selected
// after it: a guarded load compiles to an exec-masked branch that waits for its own load (64 dependent
// round trips per thread at K = 504).  The chain reads its operands from LDS one 4-step group ahead of
// the MFMAs (a wait every 2 MFMAs before).
// LN (U == 1, K <= 128): A' = LayerNorm(A; ln_w, ln_b, eps) in the launch -- wave rr holds rows rr + 4 s
// with lane l on columns 2l, 2l + 1, k_ln_fwd's own row layout, so each row goes through its row body
// (ln_fwd.h ln_fwd_row, cg_layernorm_fwd's choice for C <= 128 even) into the LDS slab: the same bits
// as cg_layernorm_fwd then this GEMM (generate()'s per-token ln1 + QKV, ln2 + FFN1, lnf + lm_head).
// KV (generate()'s per-token QKV product): columns C..3C-1 of each row also go to the layer's K / V
// caches [rows][H][Tmax][D] at position *len - 1 -- the same values cg_decode_kv_append copies.
struct KvAppend {
    float* kc;
    float* vc;
    const int64_t* len;
    int64_t C, H, D, Tmax;
};
template <int EK, int U, bool LN = false, bool KV = false>   // U = ceil(kpad / 128): float2 columns per thread and row
__global__ __launch_bounds__(256, 1) void k_gemm_f32r(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                      int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ C, int64_t ldc, EpiArgs epi,
                                                      const float* __restrict__ ln_w = nullptr,
                                                      const float* __restrict__ ln_b = nullptr, float eps = 0.f,
                                                      KvAppend kva = KvAppend{}) {
    static_assert(!LN || U == 1, "k_gemm_f32r: the LayerNorm form needs K <= 128");
    static_assert(!KV || EK == CG_EPI_STORE, "k_gemm_f32r: the K / V append goes with the plain store");
    extern __shared__ __attribute__((aligned(16))) float smr[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
    const int kpad = (int)((K + 15) / 16 * 16);   // k_gemm_f32's padded depth
    const int KS = kpad + 4;                       // LDS row stride (floats)
    float* As = smr;
    float* Bs = smr + 32 * KS;
    const int64_t mb = (int64_t)blockIdx.x * 32, nb = (int64_t)blockIdx.y * 32;
    const int rr = tid >> 6, c = tid & 63;      // rows rr + 4 s, float2 columns c + 64 u
    const int Ki = (int)K;
    float2 av[8][U], bv[8][U];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int r = rr + 4 * s;
        const int64_t ra = mb + r < M ? mb + r : M - 1, rb = nb + r < N ? nb + r : N - 1;
        const float* ap = A + ra * lda;
        const float* bp = B + rb * ldb;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = 2 * (c + 64 * u), kc = k < Ki ? k : Ki - 2;   // K even: k + 1 < K as well
            av[s][u] = *(const float2*)(ap + kc);
            bv[s][u] = *(const float2*)(bp + kc);
        }
    }
    if constexpr (LN) {
        // rows past M normalise row M - 1 (their outputs are not stored); columns K..kpad-1 zero
        const int k = 2 * c;
        const float invC = 1.0f / (float)Ki;
        float wl[1][2] = {{0.f, 0.f}}, bl[1][2] = {{0.f, 0.f}};
        if (k < Ki) {
            wl[0][0] = ln_w[k], wl[0][1] = ln_w[k + 1];
            bl[0][0] = ln_b[k], bl[0][1] = ln_b[k + 1];
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int r = rr + 4 * s;
            float v[1][2] = {{k < Ki ? av[s][0].x : 0.f, k < Ki ? av[s][0].y : 0.f}};
            float mu, rs;
            ln_fwd_row<2, 1, float, false>(v, wl, bl, Ki, invC, eps, c, As + r * KS, mu, rs);
            if (k >= Ki && k < kpad) *(float2*)(As + r * KS + k) = make_float2(0.f, 0.f);
            if (k < kpad) *(float2*)(Bs + r * KS + k) = (k < Ki && nb + r < N) ? bv[s][0] : make_float2(0.f, 0.f);
        }
    } else {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = rr + 4 * s, k = 2 * (c + 64 * u);
                if (k < kpad) {
                    const float2 z = make_float2(0.f, 0.f);
                    *(float2*)(As + r * KS + k) = (k < Ki && mb + r < M) ? av[s][u] : z;
                    *(float2*)(Bs + r * KS + k) = (k < Ki && nb + r < N) ? bv[s][u] : z;
                }
            }
    }
    constexpr bool BIAS = EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_BIAS_RESID;
    const bool hb = BIAS && epi.bias, hr = EK == CG_EPI_BIAS_RESID && epi.resid;
    const int i = w >> 1, j = w & 1;
    const int64_t m0 = mb + 16 * i, n = nb + 16 * j + li, nc = n < N ? n : N - 1;
    // the epilogue's operands in flight under the chain
    float bb = 0.f, rv[4] = {0.f, 0.f, 0.f, 0.f};
    if (hb) bb = epi.bias[nc];
    if (hr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t m = m0 + 4 * g + r, mc = m < M ? m : M - 1;
            rv[r] = epi.resid[mc * epi.ld_resid + nc];
        }
    }
    __syncthreads();
    const float* ar = As + (16 * i + li) * KS + g;
    const float* br = Bs + (16 * j + li) * KS + g;
    fv4 acc = fv4{0.f, 0.f, 0.f, 0.f};
    const int nt = kpad / 4;   // a multiple of 4
    float pa[4], pb[4], qa[4], qb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        pa[u] = ar[4 * u];
        pb[u] = br[4 * u];
    }
    // the look-ahead reads are unconditional (clamped to the last group: no LDS op under a branch, so
    // each wait counts only the group the MFMAs need)
    for (int t0 = 0;; t0 += 8) {
        const int t1 = t0 + 4 < nt ? t0 + 4 : nt - 4, t2 = t0 + 8 < nt ? t0 + 8 : nt - 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            qa[u] = ar[4 * (t1 + u)];
            qb[u] = br[4 * (t1 + u)];
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[u], pb[u], acc, 0, 0, 0);
        if (t0 + 4 >= nt) break;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pa[u] = ar[4 * (t2 + u)];
            pb[u] = br[4 * (t2 + u)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[u], qb[u], acc, 0, 0, 0);
        if (t0 + 8 >= nt) break;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + 4 * g + r;
        float v = acc[r];
        if (hb) v += (n < N ? bb : 0.f);
        if (EK == CG_EPI_BIAS_RELU) v = fmaxf(v, 0.f);
        if (hr) v = ((m < M && n < N) ? rv[r] : 0.f) + v;
        if (m < M && n < N) C[m * ldc + n] = v;
        if constexpr (KV) {
            const int64_t pos = *kva.len - 1;   // a position outside the cache writes nothing
            if (m < M && n < N && n >= kva.C && pos >= 0 && pos < kva.Tmax) {
                const bool isv = n >= 2 * kva.C;
                const int64_t t = n - (isv ? 2 * kva.C : kva.C), h = t / kva.D, e = t - h * kva.D;
                (isv ? kva.vc : kva.kc)[((m * kva.H + h) * kva.Tmax + pos) * kva.D + e] = v;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Persistent fp32 forward (NT) GEMM for many rows (M > 2048: generate()'s sliding-window products,
// M = 65536, N = 126-504, K = 126 / 504).  k_gemm_f32's 128 x 64 grid runs 2.4-3.2 rounds of
// 5 blocks per CU there (1024-4096 blocks), each block's 8-16 K-steps behind two barriers and its
// own prologue load, at ~55 % of the f32 MFMA rate (profiles/r5_gemm_f32_pmc.txt).  Here 2 blocks
// per CU own equal contiguous runs of 128 x 128 tiles (row-band-major: a run's tiles share the A row
// panel, read once into the XCD's L2), K in 32-deep steps through a 2-stage [k][row] LDS ring with
// one barrier per step, the next K-tile (or the next tile's first one) loaded to registers as float2
// along K during the current step's MFMAs, so the ring never drains at a tile seam.  4 waves of
// 64 x 64 = 2 x 2 v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation, 4 independent
// chains per wave).  An f32 MFMA accumulates as a k-ordered fma chain (cdna guide §3 'FP32-input
// MFMA'), so the 32x32x2 chain over k = 0..kpad-1 (kpad = K rounded up to 16, zero padding, the
// 32-deep step's second half skipped past kpad) is k_gemm_f32's 16x16x4 chain, and the epilogue is
// its beta-0 arithmetic: bitwise k_gemm_f32 (test_gemm_f32_persistent_matches_128x64_bitwise).
// Needs K even, lda / ldb even and 8-B aligned A / B (float2 loads).
typedef float fv16f __attribute__((ext_vector_type(16)));
constexpr int PBM = 128, PBN = 128, PBK = 32, PLD = PBM + 4;   // LDS row stride over k (floats)

template <int EK>
__global__ __launch_bounds__(256, 2) void k_gemm_f32p(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                      int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ C, int64_t ldc, EpiArgs epi,
                                                      int wflags) {
    __shared__ __attribute__((aligned(16))) float sm[2][2][PBK * PLD];   // [stage][A | B][k][row]: 66 KB
#ifdef CG_F32P_WHATIF
    // diagnostic build only (make whatif; tools/f32p_whatif.py): pk_flags bit 4 skips the in-loop loads
    // after each tile's first K-step, bit 5 the MFMAs, bit 6 the epilogue stores -- timing only
    // bit 8: fragment reads only in each tile's first K-step (MFMAs on stale registers after it),
    // bit 9: LDS store + barrier only in each tile's first K-step
    const bool WI_NOLOAD = wflags & 16, WI_NOMFMA = wflags & 32, WI_NOEPI = wflags & 64, WI_NOREAD = wflags & 256,
               WI_NOSYNC = wflags & 512;
#else
    constexpr bool WI_NOLOAD = false, WI_NOMFMA = false, WI_NOEPI = false, WI_NOREAD = false, WI_NOSYNC = false;
#endif
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
    const int wm = w >> 1, wn = w & 1;
    const int64_t tilesN = (N + PBN - 1) / PBN, ntiles = (M + PBM - 1) / PBM * tilesN;
    const int kpad = (int)((K + 15) / 16 * 16);
    const int nks = (kpad + PBK - 1) / PBK;
    const int64_t G = gridDim.x, bid = blockIdx.x;
    const int64_t t_begin = bid * ntiles / G, t_end = (bid + 1) * ntiles / G;
    // loads: rows lr + 16 i (i = 0..7) of the A and B tiles, k pair lc (a wave: 4 rows x 128 B).  Rows
    // past M / N read row M-1 / N-1 instead (they only reach outputs that are not stored), k past K reads
    // k = K-2 and is zeroed (the padded depth must add exact zeros) -- no branches around the loads.
    const int lr = tid >> 4, lc = tid & 15;
    const char* ta = nullptr;   // the tile's row m0 / n0 (wave-uniform), 32-bit byte offsets per lane
    const char* tb = nullptr;
    uint32_t oa[8], ob[8];
    auto rows_of = [&](int64_t m0, int64_t n0) {
        ta = (const char*)(A + m0 * lda);
        tb = (const char*)(B + n0 * ldb);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int64_t ma = m0 + lr + 16 * i < M ? lr + 16 * i : M - 1 - m0;
            const int64_t nb = n0 + lr + 16 * i < N ? lr + 16 * i : N - 1 - n0;
            oa[i] = (uint32_t)(ma * lda * 4);
            ob[i] = (uint32_t)(nb * ldb * 4);
        }
    };
    float2 ra[8], rb[8];
    bool rk = true;   // the loaded k pair is inside K (else it is stored as zeros: a select at the LDS
                      // write, not a write to the load's registers, which would wait for the load)
    auto load = [&](int ks) {
        const int k = ks * PBK + 2 * lc;
        rk = k < (int)K;
        const uint32_t kc = 4u * (uint32_t)(rk ? k : (int)K - 2);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            ra[i] = *(const float2*)(ta + (oa[i] + kc));
            rb[i] = *(const float2*)(tb + (ob[i] + kc));
        }
    };
    auto store = [&](int st) {
        float* As = sm[st][0];
        float* Bs = sm[st][1];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = lr + 16 * i;
            As[2 * lc * PLD + r] = rk ? ra[i].x : 0.f;
            As[(2 * lc + 1) * PLD + r] = rk ? ra[i].y : 0.f;
            Bs[2 * lc * PLD + r] = rk ? rb[i].x : 0.f;
            Bs[(2 * lc + 1) * PLD + r] = rk ? rb[i].y : 0.f;
        }
    };
    constexpr bool BIAS = EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_BIAS_RESID;
    const bool hb = BIAS && epi.bias, hr = EK == CG_EPI_BIAS_RESID && epi.resid;
    // tile coordinates advance without division: a block's tiles are consecutive in row-band-major order
    int64_t tm = t_begin / tilesN, tn = t_begin - tm * tilesN;
    int stc = 0;
    if (t_begin < t_end) {
        rows_of(tm * PBM, tn * PBN);
        load(0);
    }
#pragma unroll 1
    for (int64_t t = t_begin; t < t_end; ++t) {
        const int64_t m0t = tm * PBM, n0t = tn * PBN;
        if (++tn == tilesN) {
            tn = 0;
            ++tm;
        }
        fv16f acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = fv16f{};
#pragma unroll 1
        for (int ks = 0; ks < nks; ++ks) {
            const int st = stc & 1;
            ++stc;
            if (!WI_NOSYNC || ks == 0) {
                store(st);   // stage st was last read two steps ago, before the previous step's barrier
                __syncthreads();
            }
            if (ks + 1 < nks) {
                if (!WI_NOLOAD) load(ks + 1);
            } else if (t + 1 < t_end) {
                rows_of(tm * PBM, tn * PBN);
                load(0);
            }
            const float* As = sm[st][0] + h * PLD + 64 * wm + l32;
            const float* Bs = sm[st][1] + h * PLD + 64 * wn + l32;
            const bool full = kpad - ks * PBK > 16;   // wave-uniform: the step's second 16 k are inside kpad
            // a half step's fragments (8 k2-steps, 32 registers) read before its MFMAs: one LDS round
            // trip per 32 MFMAs instead of one per 4
            float fa[8][2], fb[8][2];
#pragma unroll
            for (int hs = 0; hs < 2; ++hs) {
                if ((hs == 1 && !full) || WI_NOMFMA) break;
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    if (WI_NOREAD && (ks > 0 || hs > 0)) break;
                    const int o = 2 * (8 * hs + s) * PLD;
                    fa[s][0] = As[o];
                    fa[s][1] = As[o + 32];
                    fb[s][0] = Bs[o];
                    fb[s][1] = Bs[o + 32];
                }
                __builtin_amdgcn_sched_barrier(0);   // keep the batch together (hipcc sinks each read to its MFMAs)
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s][0], fb[s][0], acc[0][0], 0, 0, 0);
                    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s][0], fb[s][1], acc[0][1], 0, 0, 0);
                    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s][1], fb[s][0], acc[1][0], 0, 0, 0);
                    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s][1], fb[s][1], acc[1][1], 0, 0, 0);
                }
            }
        }
        // epilogue (k_gemm_f32's beta-0 arithmetic): bias, ReLU, resid + v, per 32-row half i, the
        // half's residuals loaded before its stores.  Lane column
        // n = l32; register r holds row (r & 3) + 8 (r >> 2) + 4 h of the 32 x 32 fragment.
        const int64_t m0 = m0t + 64 * wm + 4 * h, n0 = n0t + 64 * wn + l32;
        float bv[2] = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (hb && n0 + 32 * j < N) bv[j] = epi.bias[n0 + 32 * j];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            float rv[2][16];
            if (hr) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int64_t m = m0 + 32 * i + (r & 3) + 8 * (r >> 2), n = n0 + 32 * j;
                        rv[j][r] = (m < M && n < N) ? epi.resid[m * epi.ld_resid + n] : 0.f;
                    }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t m = m0 + 32 * i + (r & 3) + 8 * (r >> 2), n = n0 + 32 * j;
                    float v = acc[i][j][r];
                    if (hb) v += bv[j];
                    if (EK == CG_EPI_BIAS_RELU) v = fmaxf(v, 0.f);
                    if (hr) v = rv[j][r] + v;
                    if (m < M && n < N && !WI_NOEPI) C[m * ldc + n] = v;
                }
        }
    }
}

bool launch_f32p(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                 int64_t ldc, const EpiArgs& e, hipStream_t st) {
    // 96 forces this kernel at any M (tests); 98 / 97 leave the fp32 products to k_gemm_f32 / the small-M kernels
    if (g_gemm_variant == 98 || g_gemm_variant == 97 || e.beta != 0.f || (M <= 2048 && g_gemm_variant != 96) ||
        M <= 0 || N <= 0 || K <= 0 || K % 2 || lda % 2 || ldb % 2 || (((uintptr_t)A | (uintptr_t)B) & 7))
        return false;
    if (e.kind != CG_EPI_STORE && e.kind != CG_EPI_BIAS && e.kind != CG_EPI_BIAS_RELU && e.kind != CG_EPI_BIAS_RESID)
        return false;
    // the kernel's 32-bit lane offsets within a 128-row tile (rows_of): 128 rows of lda floats under 4 GB
    if (lda >= ((int64_t)1 << 22) || ldb >= ((int64_t)1 << 22) || K >= ((int64_t)1 << 22)) return false;
    const int64_t ntiles = (M + PBM - 1) / PBM * ((N + PBN - 1) / PBN);
    const int64_t slots = 2 * (int64_t)gemm_cu_count();
    const unsigned grid = (unsigned)(ntiles < slots ? ntiles : slots);
#define KP(EK_) k_gemm_f32p<EK_><<<grid, 256, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, g_pk_flags)
    switch (e.kind) {
        case CG_EPI_STORE: KP(CG_EPI_STORE); break;
        case CG_EPI_BIAS: KP(CG_EPI_BIAS); break;
        case CG_EPI_BIAS_RELU: KP(CG_EPI_BIAS_RELU); break;
        default: KP(CG_EPI_BIAS_RESID); break;
    }
#undef KP
    return true;
}

// ---------------------------------------------------------------------------------------
// Fused fp32 FFN forward for inference (FeedForward GPT1.py:142-147 in eval: no dropout) --
// generate()'s sliding-window blocks, M = 65536 rows of C = 126:
//     out = resid + (relu(a W1^T + b1) W2^T + b2),   a [M][C], W1 [H][C], W2 [C][H]
// without writing h (M x H fp32: 132 MB per launch at C5) to HBM and reading it back.  A block owns
// 128 rows, each wave 32 of them, and walks the hidden units in chunks of 32:
//   * GEMM 1 transposed, D[unit][row] = W1 a^T: its "B" operand is the wave's a rows, held in 64
//     registers for the whole block (xr[s] = a[row][2s + h] after one v_permlane32_swap per float2),
//     its "A" operand the chunk's 32 W1 rows (all of k) staged in LDS;
//   * D's accumulator layout puts the row on the lane and the hidden unit on the register, which is
//     GEMM 2's A-operand layout up to a pairing of k: two v_permlane32_swap per 8 hidden units
//     (below) make lane half 0 hold the even and half 1 the odd units, so h = relu(D + b1) feeds
//     out += h W2^T straight from registers; the chunk's 32 W2 columns are staged in LDS.
// Each chunk is two 64-MFMA slices per wave (W1, then W2) through a 2-stage LDS ring -- the next
// slice loaded to registers during the current one's MFMAs, one barrier per slice; biases in LDS.
// Bitwise the two-GEMM path (k_gemm_f32 / k_gemm_f32p BIAS_RELU then BIAS_RESID): every h element
// is the same k-ordered f32 fma chain over k < ceil16(C) plus b1 then max(., 0), every output the
// chain over hidden units < ceil16(H) (zero-padded h and W2 past H) plus b2 then resid + v
// (test_ffn_f32_fused_matches_two_gemms).  C <= 128 even, H <= 2048 even, lda / ldw1 / ldw2 even.
// The B operand of a transposed row GEMM held in registers for a whole block (k_ffn_f32 GEMM 1,
// k_linear_f32t): the wave's 32 rows of a [M][C] (C <= 128 even), xr[s] = a'[row mw + l32][2s + h]
// with a' = a or (LN) LayerNorm(a; ln_w, ln_b, eps) computed with k_ln_fwd's own row body --
// cg_layernorm_fwd's choice for C <= 128 even and 8-B aligned pointers, so the same bits -- through
// a per-wave scratch at the start of the caller's LDS ring (>= 4 x 16 x 130 floats; the LN form ends
// in a block barrier).
template <bool LN>
__device__ __forceinline__ void rows_b_operand(float (&xr)[64], float* ring, const float* __restrict__ a, int64_t lda,
                                               int64_t M, int C, int64_t mw, const float* __restrict__ ln_w,
                                               const float* __restrict__ ln_b, float eps, int lane, int w) {
    const int h = lane >> 5, l32 = lane & 31;
    if constexpr (LN) {
        // a = LayerNorm(x; ln_w, ln_b) of the wave's rows, with k_ln_fwd's own row body (ln_fwd.h
        // ln_fwd_row: one wave per row, lane l holding elements 2l, 2l+1) -- the same bits -- into a
        // per-wave LDS scratch in the ring (16 rows per pass, row stride 130 floats), read back in
        // GEMM 1's B-operand layout: xr[s] = a[row][2s + h]
        constexpr int LDR = 130;
        float* scr = ring + w * 16 * LDR;
        const float invC = 1.0f / (float)C;
        float wv[1][2] = {{0.f, 0.f}}, bv[1][2] = {{0.f, 0.f}};
        if (2 * lane < C) {
            wv[0][0] = ln_w[2 * lane], wv[0][1] = ln_w[2 * lane + 1];
            bv[0][0] = ln_b[2 * lane], bv[0][1] = ln_b[2 * lane + 1];
        }
        float v[32][1][2];   // all 32 rows in flight at once (one load latency, not two)
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int64_t row = mw + i < M ? mw + i : M - 1;
            const float2 t = *(const float2*)(a + row * lda + (2 * lane < C ? 2 * lane : 0));
            v[i][0][0] = 2 * lane < C ? t.x : 0.f;
            v[i][0][1] = 2 * lane < C ? t.y : 0.f;
        }
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float mu, rs;
                ln_fwd_row<2, 1, float, false>(v[16 * pass + i], wv, bv, C, invC, eps, lane, scr + i * LDR, mu, rs);
            }
            if ((l32 >> 4) == pass) {
#pragma unroll
                for (int s = 0; s < 64; ++s) {
                    const int k = 2 * s + h;
                    xr[s] = k < C ? scr[(l32 & 15) * LDR + k] : 0.f;
                }
            }
        }
        __syncthreads();   // the scratch is the caller's LDS ring
    } else {
        // the wave's a rows in GEMM 1's B-operand layout: lane (l32, h) loads a[row][4t + 2h, +1]; one
        // swap of h1's .x with h0's .y leaves xr[2t] = a[row][4t + h], xr[2t + 1] = a[row][4t + 2 + h]
        const int64_t row = mw + l32 < M ? mw + l32 : M - 1;
        const float* ar = a + row * lda;
        float2 v[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int k = 4 * t + 2 * h;
            v[t] = *(const float2*)(ar + (k < C ? k : C - 2));
            if (k >= C) v[t] = make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[t].x), __float_as_uint(v[t].y), false,
                                                            false);
            xr[2 * t] = __uint_as_float(r[0]);
            xr[2 * t + 1] = __uint_as_float(r[1]);
        }
    }

}

constexpr int FFN_LD1 = 33, FFN_LD2 = 132, FFN_STAGE = 32 * FFN_LD2;   // W1 [128 k][32 + 1], W2 [32 unit][128 + 4]

template <bool LN>
__global__ __launch_bounds__(256, 2) void k_ffn_f32(int64_t M, int C, int H, const float* __restrict__ a, int64_t lda,
                                                    const float* __restrict__ w1, int64_t ldw1,
                                                    const float* __restrict__ b1, const float* __restrict__ w2,
                                                    int64_t ldw2, const float* __restrict__ b2,
                                                    const float* resid, int64_t ldr, float* out, int64_t ldo,
                                                    const float* __restrict__ ln_w, const float* __restrict__ ln_b,
                                                    float eps) {
    __shared__ __attribute__((aligned(16))) float sm[2][FFN_STAGE];   // 33.8 KB
    __shared__ float sb1[2048], sb2[128];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
    const int64_t mw = (int64_t)blockIdx.x * 128 + 32 * w;   // the wave's first row
    const int kpad1 = (C + 15) / 16 * 16, kpad2 = (H + 15) / 16 * 16;
    const int nc = (H + 31) / 32;
    for (int i = tid; i < H; i += 256) sb1[i] = b1[i];
    for (int i = tid; i < C; i += 256) sb2[i] = b2[i];

    // slice staging, 8 float2 per thread.  kind 0: W1 rows 32 c + (tid >> 6) + 4 i at k = 2 (tid & 63)
    // (a wave reads one 512-B row), stored [k][unit] with row stride FFN_LD1; kind 1: W2 rows
    // (tid >> 4) + 16 i at unit 32 c + 2 (tid & 15), stored [unit][column] with row stride FFN_LD2
    float2 ra[8];
    bool rk = true;
    auto load = [&](int c, int kind) {
        const float* base;
        int ld, rmax, k, kmax, r0, rs;
        if (kind == 0) {
            base = w1, ld = (int)ldw1, rmax = H, kmax = C, k = 2 * (tid & 63), r0 = 32 * c + (tid >> 6), rs = 4;
        } else {
            base = w2, ld = (int)ldw2, rmax = C, kmax = H, k = 32 * c + 2 * (tid & 15), r0 = tid >> 4, rs = 16;
        }
        rk = k < kmax;
        const int kc = rk ? k : kmax - 2;
#pragma unroll
        for (int i = 0; i < 8; ++i) {   // cg_ffn_fwd_f32 checks: rows * ld under 2^31
            const int r = r0 + rs * i < rmax ? r0 + rs * i : rmax - 1;
            ra[i] = *(const float2*)(base + (uint32_t)(r * ld + kc));
        }
    };
    auto store = [&](int st, int kind) {   // kind: the staged slice's (that of the step storing it)
        float* S = sm[st];
        const int LD = kind == 0 ? FFN_LD1 : FFN_LD2;
        const int kk = kind == 0 ? 2 * (tid & 63) : 2 * (tid & 15);
        const int r0 = kind == 0 ? tid >> 6 : tid >> 4, rs = kind == 0 ? 4 : 16;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = r0 + rs * i;
            S[kk * LD + r] = rk ? ra[i].x : 0.f;
            S[(kk + 1) * LD + r] = rk ? ra[i].y : 0.f;
        }
    };
    load(0, 0);   // the first W1 slice in flight under the a / LayerNorm prologue

    float xr[64];
    rows_b_operand<LN>(xr, &sm[0][0], a, lda, M, C, mw, ln_w, ln_b, eps, lane, w);

    int stc = 0;
    // one ring step: the staged slice (chunk c, kind) to LDS, barrier, the following slice's load;
    // returns the stage to compute from
    auto step = [&](int c, int kind) {
        const int st = stc & 1;
        ++stc;
        store(st, kind);
        __syncthreads();
        if (kind == 0) load(c, 1);
        else if (c + 1 < nc) load(c + 1, 0);
        return st;
    };

    fv16f acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = fv16f{};
    const int nst1 = kpad1 / 2;   // GEMM 1 k2-steps (<= 64)
#pragma unroll 1
    for (int c = 0; c < nc; ++c) {
        // GEMM 1: D (hidden units 32 c.., the wave's rows) over k: one accumulator chain
        fv16f D = fv16f{};
        {
            const float* S = sm[step(c, 0)] + h * FFN_LD1 + l32;
#pragma unroll
            for (int b = 0; b < 16; ++b) {   // 4 k2-steps per fragment batch
                if (4 * b >= nst1) break;
                float fa[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) fa[u] = S[2 * (4 * b + u) * FFN_LD1];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; ++u) D = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[u], xr[4 * b + u], D, 0, 0, 0);
            }
        }
        // h = relu(D + b1), zero past H; then lane half 0 takes the even, half 1 the odd hidden units:
        // register 4q + t holds unit 8q + t + 4h; swapping h1's 4q+0 with h0's 4q+1 and h1's 4q+2 with
        // h0's 4q+3 leaves h0 {8q+0, 8q+4, 8q+2, 8q+6}, h1 {8q+1, 8q+5, 8q+3, 8q+7}
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int hc = 32 * c + (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = D[r];
            v += sb1[hc < H ? hc : 0];
            v = fmaxf(v, 0.f);
            D[r] = hc < H ? v : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            auto r0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(D[4 * q]), __float_as_uint(D[4 * q + 1]), false,
                                                       false);
            auto r1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(D[4 * q + 2]), __float_as_uint(D[4 * q + 3]),
                                                       false, false);
            D[4 * q] = __uint_as_float(r0[0]);
            D[4 * q + 1] = __uint_as_float(r0[1]);
            D[4 * q + 2] = __uint_as_float(r1[0]);
            D[4 * q + 3] = __uint_as_float(r1[1]);
        }
        // GEMM 2: acc[j] (output columns 32 j.., the wave's rows) over the chunk's units; k2-step s
        // reads register 4 (s >> 2) + {0, 2, 1, 3}[s & 3]
        {
            const float* S = sm[step(c, 1)] + h * FFN_LD2 + l32;
            const int nst = kpad2 - 32 * c >= 32 ? 16 : 8;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if (2 * b >= nst) break;
                float fb[2][4];
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int j = 0; j < 4; ++j) fb[u][j] = S[2 * (2 * b + u) * FFN_LD2 + 32 * j];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    constexpr int perm[4] = {0, 2, 1, 3};
                    const int sstep = 2 * b + u;
                    const float ha = D[4 * (sstep >> 2) + perm[sstep & 3]];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ha, fb[u][j], acc[j], 0, 0, 0);
                }
            }
        }
    }
    // out = resid + (acc + b2): lane column n = 32 j + l32, register r row (r & 3) + 8 (r >> 2) + 4 h;
    // every residual loaded before the first store (out may alias resid); residual rows / columns
    // clamped, not branched around, so the loads stay in flight together
    const int64_t mr = M - 1 - mw;   // the wave's last valid row offset
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = 32 * j + l32 < C ? 32 * j + l32 : C - 1;
        const float bb = sb2[n];
        float rv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t dm = (r & 3) + 8 * (r >> 2) + 4 * h;
            rv[r] = resid[(mw + (dm < mr ? dm : mr)) * ldr + n];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = acc[j][r];
            v += bb;
            acc[j][r] = rv[r] + v;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t m = mw + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int n = 32 * j + l32;
            if (m < M && n < C) out[m * ldo + n] = acc[j][r];
        }
}

// ---------------------------------------------------------------------------------------
// Row-resident fp32 forward for K <= 128 (generate()'s window: the QKV product with its ln1
// inside, GPT1.py:111-112,163; the projection with its residual, :136): out[m][n] =
// epi(a'[m] . W[n]) with a' = a or LayerNorm(a) (rows_b_operand: the wave's 32 rows in 64 registers
// for the whole block, the LayerNorm with k_ln_fwd's row body).  Computed transposed, D[n][m] =
// W a'^T, 32 output columns per slice: the W slice (32 rows x all of K) through a 2-stage LDS ring,
// 64 MFMAs per wave per slice in one accumulator chain, then the slice's epilogue -- each lane holds
// 4 consecutive columns of its row per 8 (registers 4q..4q+3 = columns 8q + 4h + 0..3), stored as two
// float2 -- with its residuals loaded under the slice's MFMAs.  Same k-ordered f32 fma chain over
// ceil16(K) and the same beta-0 epilogue as k_gemm_f32 / k_gemm_f32p: bitwise
// (test_linear_rows_f32_matches_gemm).  K even <= 128, N even <= 2048.
template <bool LN, int EK, int NB>   // NB: 32-column blocks per slice (independent accumulator chains)
__global__ __launch_bounds__(256, 2) void k_linear_f32t(int64_t M, int C, int N, const float* __restrict__ a,
                                                        int64_t lda, const float* __restrict__ w, int64_t ldw,
                                                        const float* __restrict__ bias, const float* resid,
                                                        int64_t ldr, float* out, int64_t ldo,
                                                        const float* __restrict__ ln_w,
                                                        const float* __restrict__ ln_b, float eps) {
    constexpr int LDW = 32 * NB + 1;   // [128 k][32 NB + 1] per stage
    __shared__ __attribute__((aligned(16))) float sm[2][128 * LDW];
    __shared__ float sbias[2048];
    constexpr bool BIAS = EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_BIAS_RESID;
    const bool hb = BIAS && bias, hr = EK == CG_EPI_BIAS_RESID && resid;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l32 = lane & 31;
    const int64_t mw = (int64_t)blockIdx.x * 128 + 32 * wv;   // the wave's first row
    const int nst = (C + 15) / 16 * 8;                          // k2-steps over ceil16(K) (<= 64)
    const int nc = (N + 32 * NB - 1) / (32 * NB);
    if (hb)
        for (int i = tid; i < N; i += 256) sbias[i] = bias[i];
    // W slice c: rows 32 NB c + (tid >> 6) + 4 i, k = 2 (tid & 63) (a wave reads one row), stored [k][row]
    float2 ra[8 * NB];
    bool rk = true;
    auto load = [&](int c) {
        const int k = 2 * (tid & 63), r0 = 32 * NB * c + (tid >> 6);
        rk = k < C;
        const int kc = rk ? k : C - 2;
#pragma unroll
        for (int i = 0; i < 8 * NB; ++i) {   // cg_linear_rows_f32 checks: rows * ldw under 2^31
            const int r = r0 + 4 * i < N ? r0 + 4 * i : N - 1;
            ra[i] = *(const float2*)(w + (uint32_t)(r * (int)ldw + kc));
        }
    };
    auto store = [&](int st) {
        float* S = sm[st];
        const int kk = 2 * (tid & 63), r0 = tid >> 6;
#pragma unroll
        for (int i = 0; i < 8 * NB; ++i) {
            S[kk * LDW + r0 + 4 * i] = rk ? ra[i].x : 0.f;
            S[(kk + 1) * LDW + r0 + 4 * i] = rk ? ra[i].y : 0.f;
        }
    };
    load(0);   // in flight under the row / LayerNorm prologue
    float xr[64];
    rows_b_operand<LN>(xr, &sm[0][0], a, lda, M, C, mw, ln_w, ln_b, eps, lane, wv);
    const int64_t m = mw + l32;
    const int64_t mc = m < M ? m : M - 1;   // residual row, clamped (not branched around)
    int stc = 0;
#pragma unroll 1
    for (int c = 0; c < nc; ++c) {
        const int st = stc & 1;
        ++stc;
        store(st);   // stage st was last read two slices ago, before the previous slice's barrier
        __syncthreads();
        if (c + 1 < nc) load(c + 1);
        float2 rv[NB][4][2];
        if (hr) {
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int n = 32 * (NB * c + j) + 8 * q + 4 * h + 2 * e;
                        rv[j][q][e] = *(const float2*)(resid + mc * ldr + (n < N ? n : N - 2));
                    }
        }
        fv16f D[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) D[j] = fv16f{};
        const float* S = sm[st] + h * LDW + l32;
#pragma unroll
        for (int b = 0; b < 16; ++b) {   // 4 k2-steps per fragment batch
            if (4 * b >= nst) break;
            float fa[4][NB];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < NB; ++j) fa[u][j] = S[2 * (4 * b + u) * LDW + 32 * j];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < NB; ++j)
                    D[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[u][j], xr[4 * b + u], D[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int n = 32 * (NB * c + j) + 8 * q + 4 * h + 2 * e;
                    float v0 = D[j][4 * q + 2 * e], v1 = D[j][4 * q + 2 * e + 1];
                    if (hb) {
                        v0 += sbias[n < N ? n : 0];
                        v1 += sbias[n + 1 < N ? n + 1 : 0];
                    }
                    if (EK == CG_EPI_BIAS_RELU) {
                        v0 = fmaxf(v0, 0.f);
                        v1 = fmaxf(v1, 0.f);
                    }
                    if (hr) {
                        v0 = rv[j][q][e].x + v0;
                        v1 = rv[j][q][e].y + v1;
                    }
                    if (m < M && n < N) *(float2*)(out + m * ldo + n) = make_float2(v0, v1);
                }
    }
}

// 16-row form of rows_b_operand (v_mfma_f32_16x16x4_f32's B operand): the wave's rows mw..mw+15 of
// a [M][C] (C <= 128 even), lane l loading elements 2l, 2l+1 of each (k_ln_fwd's layout), LayerNorm in
// that layout where asked (k_ln_fwd's row body: the same bits), through a per-wave scratch [16][130]
// at the start of the caller's LDS ring, read back as xr[t] = a'[row mw + (l & 15)][4t + (l >> 4)];
// ends in a block barrier.
template <bool LN>
__device__ __forceinline__ void rows16_b_operand(float (&xr)[32], float* ring, const float* __restrict__ a,
                                                 int64_t lda, int64_t M, int C, int64_t mw,
                                                 const float* __restrict__ ln_w, const float* __restrict__ ln_b,
                                                 float eps, int lane, int wv) {
    const int li = lane & 15, g = lane >> 4;
    {
        constexpr int LDR = 130;
        float* scr = ring + wv * 16 * LDR;
        float v[16][1][2];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t row = mw + i < M ? mw + i : M - 1;
            const float2 t = *(const float2*)(a + row * lda + (2 * lane < C ? 2 * lane : 0));
            v[i][0][0] = 2 * lane < C ? t.x : 0.f;
            v[i][0][1] = 2 * lane < C ? t.y : 0.f;
        }
        if constexpr (LN) {
            const float invC = 1.0f / (float)C;
            float wl[1][2] = {{0.f, 0.f}}, bl[1][2] = {{0.f, 0.f}};
            if (2 * lane < C) {
                wl[0][0] = ln_w[2 * lane], wl[0][1] = ln_w[2 * lane + 1];
                bl[0][0] = ln_b[2 * lane], bl[0][1] = ln_b[2 * lane + 1];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float mu, rs;
                ln_fwd_row<2, 1, float, false>(v[i], wl, bl, C, invC, eps, lane, scr + i * LDR, mu, rs);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (2 * lane < C) *(float2*)(scr + i * LDR + 2 * lane) = make_float2(v[i][0][0], v[i][0][1]);
        }
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int k = 4 * t + g;
            xr[t] = k < C ? scr[li * LDR + k] : 0.f;
        }
        __syncthreads();   // the scratch is the ring's first stage
    }
}

// The same Linear with 16-row waves on v_mfma_f32_16x16x4_f32 (k_gemm_f32's own instruction):
// 64-row blocks, 1,024 workgroups at C5 and four per CU (34 KB of LDS, <= 128 VGPRs), so four waves
// per SIMD instead of two, and two independent 16 x 16 accumulator chains per 32-column slice.  The
// wave's rows go through an LDS scratch (coalesced row loads, the LayerNorm with k_ln_fwd's row body
// where asked) and come back as the B operand xr[t] = a'[row li][4t + g] (lane li + 16 g).  D[j] holds
// output columns 32 c + 16 j + 4 g + r of row li: one float4 of consecutive columns per tile.  Same
// k-ordered fma chain over ceil16(K) and epilogue as k_gemm_f32: bitwise.
template <bool LN, int EK>
__global__ __launch_bounds__(256, 4) void k_linear_f32q(int64_t M, int C, int N, const float* __restrict__ a,
                                                        int64_t lda, const float* __restrict__ w, int64_t ldw,
                                                        const float* __restrict__ bias, const float* resid,
                                                        int64_t ldr, float* out, int64_t ldo,
                                                        const float* __restrict__ ln_w,
                                                        const float* __restrict__ ln_b, float eps) {
    __shared__ __attribute__((aligned(16))) float sm[2][FFN_STAGE];   // W slices [128 k][32 + 1]
    constexpr bool BIAS = EK == CG_EPI_BIAS || EK == CG_EPI_BIAS_RELU || EK == CG_EPI_BIAS_RESID;
    const bool hb = BIAS && bias, hr = EK == CG_EPI_BIAS_RESID && resid;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, g = lane >> 4;
    const int64_t mw = (int64_t)blockIdx.x * 64 + 16 * wv;   // the wave's first row
    const int nk4 = (C + 15) / 16 * 4;                         // k4-steps over ceil16(K) (<= 32)
    const int nc = (N + 31) / 32;
    float2 ra[8];
    bool rk = true;
    auto load = [&](int c) {
        const int k = 2 * (tid & 63), r0 = 32 * c + (tid >> 6);
        rk = k < C;
        const int kc = rk ? k : C - 2;
#pragma unroll
        for (int i = 0; i < 8; ++i) {   // cg_linear_rows_f32 checks: rows * ldw under 2^31
            const int r = r0 + 4 * i < N ? r0 + 4 * i : N - 1;
            ra[i] = *(const float2*)(w + (uint32_t)(r * (int)ldw + kc));
        }
    };
    auto store = [&](int st) {
        float* S = sm[st];
        const int kk = 2 * (tid & 63), r0 = tid >> 6;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            S[kk * FFN_LD1 + r0 + 4 * i] = rk ? ra[i].x : 0.f;
            S[(kk + 1) * FFN_LD1 + r0 + 4 * i] = rk ? ra[i].y : 0.f;
        }
    };
    load(0);
    float xr[32];
    rows16_b_operand<LN>(xr, &sm[0][0], a, lda, M, C, mw, ln_w, ln_b, eps, lane, wv);
    const int64_t m = mw + li;
    const int64_t mc = m < M ? m : M - 1;   // residual row, clamped (not branched around)
    int stc = 0;
#pragma unroll 1
    for (int c = 0; c < nc; ++c) {
        const int st = stc & 1;
        ++stc;
        store(st);   // stage st was last read two slices ago, before the previous slice's barrier
        __syncthreads();
        if (c + 1 < nc) load(c + 1);
        float2 rv[2][2];
        float2 bv[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int n = 32 * c + 16 * j + 4 * g + 2 * e, nn = n < N ? n : N - 2;
                if (hr) rv[j][e] = *(const float2*)(resid + mc * ldr + nn);
                if (hb) bv[j][e] = make_float2(bias[nn], bias[nn + 1]);
            }
        fv4 D[2] = {fv4{0.f, 0.f, 0.f, 0.f}, fv4{0.f, 0.f, 0.f, 0.f}};
        const float* S = sm[st] + g * FFN_LD1 + li;
#pragma unroll
        for (int b = 0; b < 8; ++b) {   // 4 k4-steps per fragment batch
            if (4 * b >= nk4) break;
            float fa[4][2];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 2; ++j) fa[u][j] = S[4 * (4 * b + u) * FFN_LD1 + 16 * j];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    D[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[u][j], xr[4 * b + u], D[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int n = 32 * c + 16 * j + 4 * g + 2 * e;
                float v0 = D[j][2 * e], v1 = D[j][2 * e + 1];
                if (hb) {
                    v0 += bv[j][e].x;
                    v1 += bv[j][e].y;
                }
                if (EK == CG_EPI_BIAS_RELU) {
                    v0 = fmaxf(v0, 0.f);
                    v1 = fmaxf(v1, 0.f);
                }
                if (hr) {
                    v0 = rv[j][e].x + v0;
                    v1 = rv[j][e].y + v1;
                }
                if (m < M && n < N) *(float2*)(out + m * ldo + n) = make_float2(v0, v1);
            }
    }
}

// M <= 2048: k_gemm_f32r (32 x 32 tiles, any N); above: k_linear_f32q / k_linear_f32t (N <= 2048 even)
bool linear_rows_f32_supported(int64_t M, int64_t N, int64_t K) {
    return M > 0 && K >= 2 && K <= 128 && K % 2 == 0 && N >= 1 &&
           (M <= 2048 || (N >= 2 && N <= 2048 && N % 2 == 0));
}

bool ffn_f32_supported(int64_t M, int64_t C, int64_t H) {
    return M > 0 && C >= 2 && C <= 128 && C % 2 == 0 && H >= 2 && H <= 2048 && H % 2 == 0;
}

// the small-M kernel's conditions (else k_gemm_f32); gemm_variant 98 forces k_gemm_f32,
// 97 k_gemm_f32s (A/B, tests)
bool launch_f32s(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                 int64_t ldc, const EpiArgs& e, hipStream_t st) {
    if (g_gemm_variant == 98 || e.beta != 0.f || M > 2048) return false;
    const dim3 grid((unsigned)((M + 31) / 32), (unsigned)((N + 31) / 32));
    const int64_t kpad = (K + 15) / 16 * 16;
    if (g_gemm_variant != 97 && K >= 2 && K % 2 == 0 && kpad <= 624 && lda % 2 == 0 && ldb % 2 == 0 &&
        (((uintptr_t)A | (uintptr_t)B) & 7) == 0 &&
        (e.kind == CG_EPI_STORE || e.kind == CG_EPI_BIAS || e.kind == CG_EPI_BIAS_RELU || e.kind == CG_EPI_BIAS_RESID)) {
        const int U = (int)((kpad + 127) / 128);
        const size_t lds = (size_t)2 * 32 * (kpad + 4) * sizeof(float);
#define KR(EK_, U_) k_gemm_f32r<EK_, U_><<<grid, 256, lds, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e)
#define KRU(EK_)                  \
    switch (U) {                  \
        case 1: KR(EK_, 1); break; \
        case 2: KR(EK_, 2); break; \
        case 3: KR(EK_, 3); break; \
        case 4: KR(EK_, 4); break; \
        default: KR(EK_, 5); break; \
    }
        switch (e.kind) {
            case CG_EPI_STORE: KRU(CG_EPI_STORE); break;
            case CG_EPI_BIAS: KRU(CG_EPI_BIAS); break;
            case CG_EPI_BIAS_RELU: KRU(CG_EPI_BIAS_RELU); break;
            default: KRU(CG_EPI_BIAS_RESID); break;
        }
#undef KRU
#undef KR
        return true;
    }
#define KS(EK_) k_gemm_f32s<EK_><<<grid, 64, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e)
    switch (e.kind) {
        case CG_EPI_STORE: KS(CG_EPI_STORE); return true;
        case CG_EPI_BIAS: KS(CG_EPI_BIAS); return true;
        case CG_EPI_BIAS_RELU: KS(CG_EPI_BIAS_RELU); return true;
        case CG_EPI_BIAS_RESID: KS(CG_EPI_BIAS_RESID); return true;
        default: return false;
    }
#undef KS
}

void launch_f32(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                const float* B, int64_t ldb, float* C, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
                hipStream_t st) {
    if (!a_trans && !b_trans && split_k == 1 &&
        (launch_f32p(M, N, K, A, lda, B, ldb, C, ldc, e, st) || launch_f32s(M, N, K, A, lda, B, ldb, C, ldc, e, st)))
        return;
    int64_t kchunk = (K + split_k - 1) / split_k;
    kchunk = (kchunk + FBKK - 1) / FBKK * FBKK;
    dim3 grid((unsigned)(((M + FBM - 1) / FBM) * ((N + FBN - 1) / FBN)), (unsigned)split_k);
#define KF(at_, bt_) k_gemm_f32<at_, bt_><<<grid, 256, 0, st>>>(M, N, K, A, lda, B, ldb, C, ldc, e, split_k, kchunk, ws)
    if (!a_trans && !b_trans) KF(false, false);
    else if (!a_trans && b_trans) KF(false, true);
    else if (a_trans && !b_trans) KF(true, false);
    else KF(true, true);
#undef KF
}

template <typename TC>
__global__ void k_splitk_reduce(const float* __restrict__ ws, int split_k, int64_t M, int64_t N, TC* __restrict__ C,
                                int64_t ldc, EpiArgs epi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int64_t m = i / N, n = i % N;
    float s = 0.f;
    for (int k = 0; k < split_k; ++k) s += ws[(int64_t)k * M * N + i];
    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
    store_out<TC>(C, m * ldc + n, epi_scalar(epi, s, m, n, N, stream), epi.beta);
}

// Vectorised form for the MFMA path's slabs (N % 4 == 0, 16-B aligned rows): four consecutive
// columns per thread, every slab load issued before the sum, 32-bit index math (the scalar form
// above spent its time in 64-bit division; measured 12.8 us for the C2 FFN weight gradient, split 8).
// Same summation order (k = 0..split-1) and epilogue arithmetic as epi_scalar, so results are
// bitwise those of the scalar form.
// S > 0: compile-time split, every slab's float4 loaded before the first add (S loads in flight per
// thread instead of 4); the adds still run k = 0..S-1 in order.
// bf16 slabs of an fp32 STORE output (cg_set_tuning "slab_bf16"): 8 outputs per thread
__global__ __launch_bounds__(256) void k_slab16_reduce8(const void* __restrict__ ws, int S, int64_t n8,
                                                        float* __restrict__ out, float beta) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n8) slab16_chunk8(ws, S, 8 * n8, i, out, beta);
}

template <typename TC, int S>
__global__ __launch_bounds__(256) void k_splitk_reduce4(const float* __restrict__ ws, int split_k, int M, int N,
                                                        TC* __restrict__ C, int64_t ldc, EpiArgs epi) {
    const int n4 = N >> 2;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= M * n4) return;
    const int m = i / n4, n = (i - m * n4) * 4;
    const int64_t slab = (int64_t)M * N, p = (int64_t)m * N + n;
    const bool sb = epi.slab_bf16;   // bf16 slabs (cg_set_tuning "slab_bf16"): same order, widened exactly
    fv4 s;
    int k = 1;
    if constexpr (S > 0) {
        fv4 a[S];
#pragma unroll
        for (int j = 0; j < S; ++j) a[j] = ld_slab4(ws, p + j * slab, sb);   // slabs are read once
        s = a[0];
#pragma unroll
        for (int j = 1; j < S; ++j) s += a[j];
        k = split_k;
    } else {
        s = ld_slab4(ws, p, sb);
    }
    for (; k + 4 <= split_k; k += 4) {
        const fv4 a = ld_slab4(ws, p + k * slab, sb), b = ld_slab4(ws, p + (k + 1) * slab, sb);
        const fv4 c = ld_slab4(ws, p + (k + 2) * slab, sb), d = ld_slab4(ws, p + (k + 3) * slab, sb);
        s += a;
        s += b;
        s += c;
        s += d;
    }
    for (; k < split_k; ++k) s += ld_slab4(ws, p + k * slab, sb);
    float v[4] = {s[0], s[1], s[2], s[3]};
    if (epi.kind != CG_EPI_STORE && epi.bias) {
        const float4 b = *(const float4*)(epi.bias + n);
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    if (epi.kind == CG_EPI_BIAS_RESID && epi.resid) {
        const float4 r = *(const float4*)(epi.resid + (int64_t)m * epi.ld_resid + n);
        v[0] = r.x + v[0]; v[1] = r.y + v[1]; v[2] = r.z + v[2]; v[3] = r.w + v[3];
    }
    TC* o = C + (int64_t)m * ldc + n;
#pragma unroll
    for (int q = 0; q < 4; ++q) store_out<TC>(o, q, v[q], epi.beta);
}

// =====================================================================================
// column sums (bias gradients): out[n] (=|+=) sum_m X[m,n]
// =====================================================================================
constexpr int CS_ROWS = 256;

// per 256-row chunk column partials: 64 columns x 4 row-lanes, 8 loads in flight per thread
template <typename TX>
__global__ __launch_bounds__(256) void k_colsum_partial(const TX* __restrict__ X, int64_t rows, int64_t N,
                                                        int64_t ldx, float* __restrict__ part) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
    const int64_t n = (int64_t)blockIdx.x * 64 + c;
    const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS;
    float s = 0.f;
    if (n < N) {
        if (r0 + CS_ROWS <= rows) {
#pragma unroll
            for (int j0 = 0; j0 < CS_ROWS / 4; j0 += 16) {
                float v[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = ld_as_f32<TX>(X + (r0 + rl + 4 * (j0 + j)) * ldx + n);
#pragma unroll
                for (int j = 0; j < 16; ++j) s += v[j];
            }
        } else {
            for (int64_t r = r0 + rl; r < rows; r += 4) s += ld_as_f32<TX>(X + r * ldx + n);
        }
    }
    red[rl][c] = s;
    __syncthreads();
    if (rl == 0 && n < N) part[(int64_t)blockIdx.y * N + n] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

EpiArgs make_epi(const cg_epilogue_t* e) {
    EpiArgs a;
    memset(&a, 0, sizeof(a));
    a.kind = CG_EPI_STORE;
    a.dscale = 1.f;
    if (!e) return a;
    a.kind = e->kind;
    a.bias = e->bias;
    a.resid = e->resid;
    a.ld_resid = e->ld_resid;
    a.aux = e->aux;
    a.aux_dtype = e->aux_dtype;
    a.ld_aux = e->ld_aux;
    a.thr = e->dropout_p > 0 ? dropout_threshold(e->dropout_p) : 0u;
    a.dscale = e->dropout_p > 0 ? dropout_scale(e->dropout_p) : 1.f;
    a.seed = e->seed;
    a.rng_call = e->rng_call;
    a.site = e->site;
    a.beta = e->beta;
    a.colpart = e->colpart;
    return a;
}

template <typename TA, typename TB>
int launch_generic(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                   const void* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                   void* ws, hipStream_t st) {
    int64_t kchunk = (K + split_k - 1) / split_k;
    kchunk = (kchunk + GBK - 1) / GBK * GBK;
    const int64_t tiles = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
    dim3 grid((unsigned)tiles, (unsigned)split_k);
    if (c_dtype == CG_BF16)
        k_gemm_generic<TA, TB, bf16_t><<<grid, 256, 0, st>>>(a_trans, b_trans, M, N, K, (const TA*)A, lda,
                                                             (const TB*)B, ldb, (bf16_t*)C, ldc, e, split_k, kchunk,
                                                             (float*)ws);
    else
        k_gemm_generic<TA, TB, float><<<grid, 256, 0, st>>>(a_trans, b_trans, M, N, K, (const TA*)A, lda,
                                                            (const TB*)B, ldb, (float*)C, ldc, e, split_k, kchunk,
                                                            (float*)ws);
    return CG_OK;
}

}  // namespace

namespace cg {
int g_gemm_variant = 0;
int g_linear_rows_nb = 0;   // cg_set_tuning("linear_rows_nb"): 0 k_linear_f32q (16-row waves), 1 / 2 k_linear_f32t
int g_gemm_max_grid = 0;
int g_gemm_group_p8 = 0;   // persistent-kernel tile order (gemm_tile.h tile_rc), cg_set_tuning knobs
int g_gemm_group_pk = 0;
int g_gemm_n96 = 1;       // cg_set_tuning("gemm_n96"): 128x96 tiles for the part-filling fp32 residual forwards (gemm_pk.hip launch_n96)
int g_adam_per_launch = 0;   // cg_set_tuning("adam_per_launch"): AdamW jobs one launch's free blocks take (0 = MAX_ADAM)
int g_red_side = 1;       // cg_set_tuning("red_side"): a part-filling persistent launch takes a pending reduce on extra blocks
int g_adam_batch = 1;     // cg_set_tuning("adam_batch"), A/B build only: the side blocks' AdamW chunks in flight per thread

static int current_device() {
    int d = -1;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
}

// the device a stream belongs to: hipStreamGetDevice for a created stream, the current device for
// the null stream.  The queue key must not depend on the calling thread's current device: the
// autograd device thread queues work with the tensor's device current, while the flush may come
// from a thread whose current device is another one.
static int stream_device(hipStream_t st) {
    if (st) {
        hipDevice_t d = -1;
        if (hipStreamGetDevice(st, &d) == hipSuccess && d >= 0) return (int)d;
    }
    return current_device();
}

// the deferral registry (defer.h): one queue per (device, stream)
std::mutex& defer_mutex() {
    static std::mutex m;
    return m;
}

static std::map<std::pair<int, hipStream_t>, DeferQueue>& defer_registry() {
    static std::map<std::pair<int, hipStream_t>, DeferQueue> reg;
    return reg;
}

DeferQueue* defer_queue(hipStream_t st, bool create) {
    auto& reg = defer_registry();
    const auto key = std::make_pair(stream_device(st), st);
    auto it = reg.find(key);
    if (it != reg.end()) return &it->second;
    if (!create) return nullptr;
    DeferQueue& q = reg[key];
    q.stream = st;
    q.device = key.first;
    return &q;
}

// an emptied queue leaves the registry: a stream destroyed after its flush / discard leaves no queue
// behind for a new stream that reuses its handle
void defer_queue_drop(DeferQueue* q) {
    if (q && !q->nred && !q->nadam && !q->parts.n) defer_registry().erase(std::make_pair(q->device, q->stream));
}

// launches of a queue's flush run with the queue's device current (a kernel goes to the stream's
// device), the caller's device restored after
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        const int cur = current_device();
        if (dev >= 0 && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// pending jobs for a launch on stream st of the current device: the stream's split-K reduces, and
// with side_ok (the launch has >= SIDE_MIN free blocks) up to MAX_ADAM of its AdamW jobs, oldest first
RedJobs take_pending_reduces(hipStream_t st, bool side_ok) {
    RedJobs r = {};
    std::lock_guard<std::mutex> lk(defer_mutex());
    DeferQueue* q = defer_queue(st, false);
    if (!q) return r;
    r.n = q->nred;
    for (int i = 0; i < r.n; ++i) r.j[i] = q->red[i];
    q->nred = 0;
    if (side_ok && q->nadam) {
        const int cap = g_adam_per_launch > 0 && g_adam_per_launch < MAX_ADAM ? g_adam_per_launch : MAX_ADAM;
        r.na = q->nadam < cap ? q->nadam : cap;
        for (int i = 0; i < r.na; ++i) r.a[i] = q->adam[i];
        for (int i = r.na; i < q->nadam; ++i) q->adam[i - r.na] = q->adam[i];
        q->nadam -= r.na;
        q->adam_taken += r.na;
    }
#ifdef CG_AB_VARIANTS
    r.adam_batch = g_adam_batch;
#endif
    return r;
}

bool has_pending_reduces(hipStream_t st, bool side_ok) {
    std::lock_guard<std::mutex> lk(defer_mutex());
    const DeferQueue* q = defer_queue(st, false);
    return q && (q->nred || (side_ok && q->nadam));
}

int adamw_job_launch(const AdamJob& j, hipStream_t st);   // ce_adamw.hip
int adamw_segments_launch(float* p, const float* g, float* m, float* v, bf16_t* pb, const int64_t* segs, int nseg,
                          double lr, double beta1, double beta2, double eps, double wd, const int64_t* step,
                          hipStream_t st);   // ce_adamw.hip

// the stream's pending AdamW jobs: slices of one set of flat buffers with one set of hyperparameters
// (the training step's weight matrices) as ONE segmented launch, anything else job by job
void flush_adam_locked(DeferQueue& q) {
    if (!q.nadam) return;
    const int n = q.nadam;
    q.nadam = 0;
    q.adam_taken += n;   // launched: cg_discard_deferred reports them (cg_flush_deferred resets the count)
    const AdamJob* J = q.adam;
    int b = 0;   // the job with the lowest address is the segments' base
    for (int i = 1; i < n; ++i)
        if (J[i].p < J[b].p) b = i;
    bool one = n > 1 && n <= 64;
    int64_t segs[2 * MAX_ADAM_PENDING];
    for (int i = 0; i < n && one; ++i) {
        const int64_t d = J[i].p - J[b].p;
        one = J[i].g - J[b].g == d && J[i].m - J[b].m == d && J[i].v - J[b].v == d && J[i].pb - J[b].pb == d &&
              J[i].lr == J[b].lr && J[i].beta1 == J[b].beta1 && J[i].beta2 == J[b].beta2 && J[i].eps == J[b].eps &&
              J[i].wd == J[b].wd && J[i].step == J[b].step;
        segs[2 * i] = d;
        segs[2 * i + 1] = 4 * J[i].n4;
    }
    if (one)
        (void)adamw_segments_launch(J[b].p, J[b].g, J[b].m, J[b].v, J[b].pb, segs, n, J[b].lr, J[b].beta1, J[b].beta2,
                                    J[b].eps, J[b].wd, J[b].step, q.stream);
    else
        for (int i = 0; i < n; ++i) (void)adamw_job_launch(J[i], q.stream);
}

static void launch_splitk_reduce_job(const RedJob& j, hipStream_t st);

// the stream's pending split-K reduces as standalone reduce kernels (cg_flush_deferred, a full queue,
// or an AdamW job whose gradient one of them writes)
void flush_red_locked(DeferQueue& q) {
    const int n = q.nred;
    q.nred = 0;
    for (int i = 0; i < n; ++i) launch_splitk_reduce_job(q.red[i], q.stream);
}

int g_skip_splitk_reduce = 0;  // measurement knob (WRONG results): time a step without the split-K reduce
extern int g_attn_variant;  // attention_d64.hip
extern int g_attn_bwd_lpt;  // attention_d64.hip
extern int g_decode_attn_rows;  // decode.hip
extern int g_ln_rpb;  // layernorm.hip
extern int g_adamw_mode;  // ce_adamw.hip
extern int g_ln_waves;  // layernorm.hip
extern int g_ln_pf;     // layernorm.hip
extern int g_ln_rl;     // layernorm.hip
extern int g_ln_nt;     // layernorm.hip
}

extern "C" int cg_timing_event_create(void** event) {
    CG_REQUIRE(event, "cg_timing_event_create: null");
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {
        cg::set_error("cg_timing_event_create: hipEventCreate failed");
        return CG_EHIP;
    }
    *event = (void*)e;
    return CG_OK;
}

extern "C" int cg_timing_event_record(void* event, void* stream) {
    CG_REQUIRE(event, "cg_timing_event_record: null event");
    hipStream_t st = (hipStream_t)stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    hipError_t r = hipStreamGetCaptureInfo_v2(st, &cs, &id, &g, &deps, &nd);
    if (r == hipSuccess && cs == hipStreamCaptureStatusActive) {
        // an event-record node appended to the capture by hand (hipEventRecordWithFlags with
        // hipEventRecordExternal is refused during capture on this runtime): it depends on the
        // stream's current capture frontier and becomes the new frontier
        hipGraphNode_t node = nullptr;
        r = hipGraphAddEventRecordNode(&node, g, deps, nd, (hipEvent_t)event);
        if (r == hipSuccess) r = hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies);
    } else if (r == hipSuccess) {
        r = hipEventRecord((hipEvent_t)event, st);
    }
    if (r != hipSuccess) {
        (void)hipGetLastError();   // leave no sticky error for the caller's next launch check
        cg::set_error("cg_timing_event_record: %s", hipGetErrorString(r));
        return CG_EHIP;
    }
    return CG_OK;
}

extern "C" int cg_timing_event_elapsed(void* start, void* end, float* ms) {
    CG_REQUIRE(start && end && ms, "cg_timing_event_elapsed: null");
    const hipError_t r = hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end);
    if (r != hipSuccess) {
        cg::set_error("cg_timing_event_elapsed: %s", hipGetErrorString(r));
        return CG_EHIP;
    }
    return CG_OK;
}

extern "C" int cg_timing_event_destroy(void* event) {
    if (event) (void)hipEventDestroy((hipEvent_t)event);
    return CG_OK;
}

extern "C" int cg_set_tuning(const char* key, int value) {
    CG_REQUIRE(key, "cg_set_tuning: null key");
    if (!strcmp(key, "gemm_variant")) {
        // default build: automatic (0), the register-staged fallback (2), the persistent 128x128 (9)
        // and 256x256 (24) tiles, k_gemm_f32 for every fp32 product (98: not the small-M or
        // persistent kernels; 97: k_gemm_f32s, not the K-resident one; 96: the persistent
        // k_gemm_f32p at any M), the generic kernels (99); the
        // measured-slower A/B tiles (among
        // them 26, the 256x256 tile on the staggered 8-phase schedule) only in
        // libcharpt_hip_ab.so (`make ab`, CG_AB_VARIANTS)
#ifndef CG_AB_VARIANTS
        CG_REQUIRE(value == 0 || value == 2 || value == 9 || value == 24 || value == 96 || value == 97 || value == 98 || value == 99,
                   "cg_set_tuning: gemm_variant %d is an A/B variant, not in this build (make ab)", value);
#endif
        g_gemm_variant = value;
        return CG_OK;
    }
    if (!strcmp(key, "linear_rows_nb")) {
        CG_REQUIRE(value >= 0 && value <= 2, "cg_set_tuning: linear_rows_nb must be 0 (16-row waves), 1 or 2");
        g_linear_rows_nb = value;
        return CG_OK;
    }
    if (!strcmp(key, "gemm_max_grid")) {
        g_gemm_max_grid = value;
        return CG_OK;
    }
    if (!strcmp(key, "gemm_group_p8")) {   // gemm_tile.h tile_rc row panels per group (0/1: row-major)
        CG_REQUIRE(value >= 0 && value < 256, "cg_set_tuning: gemm_group_p8 out of range");
        g_gemm_group_p8 = value;
        return CG_OK;
    }
    if (!strcmp(key, "gemm_group_pk")) {
        CG_REQUIRE(value >= 0 && value < 256, "cg_set_tuning: gemm_group_pk out of range");
        g_gemm_group_pk = value;
        return CG_OK;
    }
    if (!strcmp(key, "gemm_n96")) {
        g_gemm_n96 = value;
        return CG_OK;
    }
    if (!strcmp(key, "pk_flags")) {
        g_pk_flags = value;
        return CG_OK;
    }
    if (!strcmp(key, "ln_rl")) {   // A/B: the LayerNorm backward rows' next loads before the current stores
        CG_REQUIRE(value >= 0 && value <= 2, "cg_set_tuning: ln_rl must be 0, 1 or 2 (2: also at C = 768)");
        g_ln_rl = value;
        return CG_OK;
    }
    if (!strcmp(key, "decode_attn_rows")) {   // A/B: the coalesced-chunk phase-1 decode attention (decode.hip)
        CG_REQUIRE(value == 0 || value == 1, "cg_set_tuning: decode_attn_rows must be 0 or 1");
        g_decode_attn_rows = value;
        return CG_OK;
    }
    if (!strcmp(key, "attn_bwd_lpt")) {   // A/B: merged resident backward workgroup order (1 = dK/dV first)
        CG_REQUIRE(value == 0 || value == 1, "cg_set_tuning: attn_bwd_lpt must be 0 or 1");
        g_attn_bwd_lpt = value;
        return CG_OK;
    }
    if (!strcmp(key, "attn_variant")) {
#ifndef CG_AB_VARIANTS
        // 0 automatic, 1 ring kernels at T <= 256 (and the 64-query-block fp32 forward instead of the
        // sequence-resident one), 2 separate resident dQ / dK-dV launches (A/B build
        // also 4: the 8-wave ping-pong forward at T % 256 == 0, 512..1024)
        CG_REQUIRE(value >= 0 && value <= 2, "cg_set_tuning: attn_variant %d is an A/B variant, not in this build (make ab)",
                   value);
#endif
        g_attn_variant = value;
        return CG_OK;
    }
    if (!strcmp(key, "skip_splitk_reduce")) {
        g_skip_splitk_reduce = value;
        return CG_OK;
    }
    if (!strcmp(key, "adam_per_launch")) {
        g_adam_per_launch = value;
        return CG_OK;
    }
    if (!strcmp(key, "adam_batch")) {
#ifndef CG_AB_VARIANTS
        CG_REQUIRE(value == 1, "cg_set_tuning: adam_batch %d is an A/B variant, not in this build (make ab)", value);
#endif
        g_adam_batch = value;
        return CG_OK;
    }
    if (!strcmp(key, "red_side")) {
        g_red_side = value;
        return CG_OK;
    }
    if (!strcmp(key, "defer_splitk") || !strcmp(key, "slab_bf16") || !strcmp(key, "defer_partials")) {
        set_error("cg_set_tuning: %s is a per-call flag since round 5 (cg_epilogue_t.flags CG_GEMM_DEFER_REDUCE / "
                  "CG_GEMM_SLAB_BF16, the CG_DEFER flag of the _ex reduces)", key);
        return CG_EINVAL;
    }
    if (!strcmp(key, "ln_waves")) {   // takes effect for workspaces sized after the call
        g_ln_waves = value;
        return CG_OK;
    }
    if (!strcmp(key, "adamw_mode")) {
        CG_REQUIRE(value >= 0 && value <= 5, "cg_set_tuning: adamw_mode out of range");
        g_adamw_mode = value;
        return CG_OK;
    }
    if (!strcmp(key, "ln_nt")) {   // the LayerNorm backward's non-temporal streams (-1 automatic, 0..3)
        g_ln_nt = value;
        return CG_OK;
    }
    if (!strcmp(key, "ln_pf")) {
        g_ln_pf = value;
        return CG_OK;
    }
    if (!strcmp(key, "ln_rpb")) {   // takes effect for workspaces sized after the call
        g_ln_rpb = value;
        return CG_OK;
    }
    set_error("cg_set_tuning: unknown key %s", key);
    return CG_EINVAL;
}

extern "C" int cg_gemm_colpart_supported(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, int64_t lda,
                                         int64_t ldb, int64_t ldc) {
    return gemm_colpart_supported(a_trans, b_trans, M, N, K, lda, ldb, ldc) ? 1 : 0;
}

extern "C" int cg_gemm_relu_bits_supported(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, int64_t lda,
                                           int64_t ldb, int64_t ldc) {
    return gemm_relu_bits_supported(a_trans, b_trans, M, N, K, lda, ldb, ldc) ? 1 : 0;
}

extern "C" int cg_gemm_rowdot_supported(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, int64_t lda,
                                        int64_t ldb, int64_t ldc) {
    return gemm_rowdot_supported(a_trans, b_trans, M, N, K, lda, ldb, ldc) ? 1 : 0;
}

extern "C" int64_t cg_gemm_workspace(int64_t M, int64_t N, int split_k) {
    return split_k > 1 ? (int64_t)split_k * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int cg_linear_rows_f32_supported(int64_t M, int64_t N, int64_t K) {
    return linear_rows_f32_supported(M, N, K) ? 1 : 0;
}

extern "C" int cg_linear_rows_f32(int64_t M, int64_t N, int64_t K, const float* a, int64_t lda, const float* ln_w,
                                  const float* ln_b, float eps, const float* w, int64_t ldw, const float* bias, int relu,
                                  const float* resid, int64_t ldr, float* out, int64_t ldo, void* stream) {
    CG_REQUIRE(linear_rows_f32_supported(M, N, K),
               "cg_linear_rows_f32: unsupported shape M=%lld N=%lld K=%lld (K <= 128 even; above 2048 rows N <= 2048 even)",
               (long long)M, (long long)N, (long long)K);
    CG_REQUIRE(a && w && out, "cg_linear_rows_f32: null pointer");
    CG_REQUIRE(!relu || (bias && !resid), "cg_linear_rows_f32: relu needs a bias and no residual");
    CG_REQUIRE(!ln_w == !ln_b, "cg_linear_rows_f32: ln_w and ln_b both or neither");
    hipStream_t st = (hipStream_t)stream;
    if (M <= 2048) {
        // generate()'s per-token rows: k_gemm_f32r (the kernel cg_gemm runs there), the LayerNorm in its
        // prologue -- the bits of [cg_layernorm_fwd +] cg_gemm at any N
        CG_REQUIRE(lda >= K && lda % 2 == 0 && ldw >= K && ldw % 2 == 0 && ldo >= N && (!resid || ldr >= N),
                   "cg_linear_rows_f32: bad leading dimensions");
        CG_REQUIRE((((uintptr_t)a | (uintptr_t)w) & 7) == 0, "cg_linear_rows_f32: a, w must be 8-B aligned");
        EpiArgs e{};
        e.kind = resid ? CG_EPI_BIAS_RESID : relu ? CG_EPI_BIAS_RELU : bias ? CG_EPI_BIAS : CG_EPI_STORE;
        e.bias = bias;
        e.resid = resid;
        e.ld_resid = ldr;
        const dim3 grid((unsigned)((M + 31) / 32), (unsigned)((N + 31) / 32));
        const size_t lds = (size_t)2 * 32 * ((K + 15) / 16 * 16 + 4) * sizeof(float);
#define KR(EK_, LN_) \
    k_gemm_f32r<EK_, 1, LN_><<<grid, 256, lds, st>>>(M, N, K, a, lda, w, ldw, out, ldo, e, ln_w, ln_b, eps)
#define KRL(EK_)                  \
    do {                          \
        if (ln_w) KR(EK_, true);  \
        else KR(EK_, false);      \
    } while (0)
        switch (e.kind) {
            case CG_EPI_STORE: KRL(CG_EPI_STORE); break;
            case CG_EPI_BIAS: KRL(CG_EPI_BIAS); break;
            case CG_EPI_BIAS_RELU: KRL(CG_EPI_BIAS_RELU); break;
            default: KRL(CG_EPI_BIAS_RESID); break;
        }
#undef KRL
#undef KR
        CG_LAUNCH_CHECK("cg_linear_rows_f32");
        return CG_OK;
    }
    CG_REQUIRE(lda >= K && lda % 2 == 0 && ldw >= K && ldw % 2 == 0 && ldo >= N && ldo % 2 == 0 &&
                   (!resid || (ldr >= N && ldr % 2 == 0)) && N * ldw < ((int64_t)1 << 31),
               "cg_linear_rows_f32: bad leading dimensions");
    CG_REQUIRE((((uintptr_t)a | (uintptr_t)w | (uintptr_t)out | (uintptr_t)(resid ? resid : out)) & 7) == 0,
               "cg_linear_rows_f32: a, w, out, resid must be 8-B aligned");
    CG_REQUIRE(!ln_w || ((((uintptr_t)ln_w | (uintptr_t)ln_b) & 7) == 0 && lda == K),
               "cg_linear_rows_f32: ln_w / ln_b must be 8-B aligned and a dense (lda == K) with the LayerNorm");
    const dim3 grid((unsigned)((M + 127) / 128));
    // 16-row waves (k_linear_f32q: four waves per SIMD) by default; cg_set_tuning("linear_rows_nb", 1 / 2):
    // 32-row waves with one / two 32-column chains per slice -- 3.3 % / 5.4 % slower in generate
    // (profiles/r6_linear_rows_gen.txt)
#define KL(LN_, EK_)                                                                                              \
    do {                                                                                                          \
        if (g_linear_rows_nb == 0)                                                                                \
            k_linear_f32q<LN_, EK_><<<dim3((unsigned)((M + 63) / 64)), 256, 0, st>>>(                             \
                M, (int)K, (int)N, a, lda, w, ldw, bias, resid, ldr, out, ldo, ln_w, ln_b, eps);                  \
        else if (g_linear_rows_nb == 1)                                                                           \
            k_linear_f32t<LN_, EK_, 1><<<grid, 256, 0, st>>>(M, (int)K, (int)N, a, lda, w, ldw, bias, resid, ldr, \
                                                             out, ldo, ln_w, ln_b, eps);                          \
        else                                                                                                      \
            k_linear_f32t<LN_, EK_, 2><<<grid, 256, 0, st>>>(M, (int)K, (int)N, a, lda, w, ldw, bias, resid, ldr, \
                                                             out, ldo, ln_w, ln_b, eps);                          \
    } while (0)
    const bool ln = ln_w != nullptr;
    if (resid) {
        if (ln) KL(true, CG_EPI_BIAS_RESID); else KL(false, CG_EPI_BIAS_RESID);
    } else if (relu) {
        if (ln) KL(true, CG_EPI_BIAS_RELU); else KL(false, CG_EPI_BIAS_RELU);
    } else if (bias) {
        if (ln) KL(true, CG_EPI_BIAS); else KL(false, CG_EPI_BIAS);
    } else {
        if (ln) KL(true, CG_EPI_STORE); else KL(false, CG_EPI_STORE);
    }
#undef KL
    CG_LAUNCH_CHECK("cg_linear_rows_f32");
    return CG_OK;
}

extern "C" int cg_decode_qkv_f32(int64_t B, int64_t C, int64_t H, const float* x, int64_t ldx, const float* ln_w,
                                 const float* ln_b, float eps, const float* w, int64_t ldw, float* qkv, int64_t ldq,
                                 const int64_t* len_dev, int64_t Tmax, float* kcache, float* vcache, void* stream) {
    CG_REQUIRE(B > 0 && B <= 2048 && C >= 2 && C <= 128 && C % 2 == 0 && H > 0 && C % H == 0 && Tmax > 0,
               "cg_decode_qkv_f32: needs 0 < B <= 2048, C <= 128 even, H | C (B=%lld C=%lld H=%lld)", (long long)B,
               (long long)C, (long long)H);
    CG_REQUIRE(x && ln_w && ln_b && w && qkv && len_dev && kcache && vcache, "cg_decode_qkv_f32: null pointer");
    CG_REQUIRE(ldx >= C && ldx % 2 == 0 && ldw >= C && ldw % 2 == 0 && ldq >= 3 * C,
               "cg_decode_qkv_f32: bad leading dimensions");
    CG_REQUIRE((((uintptr_t)x | (uintptr_t)w) & 7) == 0, "cg_decode_qkv_f32: x, w must be 8-B aligned");
    EpiArgs e{};
    e.kind = CG_EPI_STORE;
    const KvAppend kva{kcache, vcache, len_dev, C, H, C / H, Tmax};
    const int64_t N = 3 * C;
    const dim3 grid((unsigned)((B + 31) / 32), (unsigned)((N + 31) / 32));
    const size_t lds = (size_t)2 * 32 * ((C + 15) / 16 * 16 + 4) * sizeof(float);
    k_gemm_f32r<CG_EPI_STORE, 1, true, true><<<grid, 256, lds, (hipStream_t)stream>>>(B, N, C, x, ldx, w, ldw, qkv, ldq,
                                                                                     e, ln_w, ln_b, eps, kva);
    CG_LAUNCH_CHECK("cg_decode_qkv_f32");
    return CG_OK;
}

extern "C" int cg_ffn_fwd_f32_supported(int64_t M, int64_t C, int64_t H) { return ffn_f32_supported(M, C, H) ? 1 : 0; }

extern "C" int cg_ffn_fwd_f32(int64_t M, int64_t C, int64_t H, const float* a, int64_t lda, const float* ln_w,
                              const float* ln_b, float eps, const float* w1, int64_t ldw1, const float* b1,
                              const float* w2, int64_t ldw2, const float* b2, const float* resid, int64_t ldr,
                              float* out, int64_t ldo, void* stream) {
    CG_REQUIRE(ffn_f32_supported(M, C, H),
               "cg_ffn_fwd_f32: unsupported shape M=%lld C=%lld H=%lld (C <= 128 even, H <= 2048 even)", (long long)M,
               (long long)C, (long long)H);
    CG_REQUIRE(a && w1 && b1 && w2 && b2 && resid && out, "cg_ffn_fwd_f32: null pointer");
    CG_REQUIRE(lda >= C && lda % 2 == 0 && ldw1 >= C && ldw1 % 2 == 0 && ldw2 >= H && ldw2 % 2 == 0 && ldr >= C &&
                   ldo >= C && (int64_t)H * ldw1 < ((int64_t)1 << 31) && C * ldw2 < ((int64_t)1 << 31),
               "cg_ffn_fwd_f32: bad leading dimensions");
    CG_REQUIRE((((uintptr_t)a | (uintptr_t)w1 | (uintptr_t)w2) & 7) == 0, "cg_ffn_fwd_f32: a, w1, w2 must be 8-B aligned");
    CG_REQUIRE(!ln_w == !ln_b, "cg_ffn_fwd_f32: ln_w and ln_b both or neither");
    // (k_ln_fwd's narrow-row body -- the one the in-launch LayerNorm repeats -- is cg_layernorm_fwd's
    // choice for C <= 128 even with 8-B aligned x / w / b)
    CG_REQUIRE(!ln_w || ((((uintptr_t)ln_w | (uintptr_t)ln_b) & 7) == 0 && lda == C),
               "cg_ffn_fwd_f32: ln_w / ln_b must be 8-B aligned and a dense (lda == C) with the LayerNorm");
    const dim3 grid((unsigned)((M + 127) / 128));
    if (ln_w)
        k_ffn_f32<true><<<grid, 256, 0, (hipStream_t)stream>>>(M, (int)C, (int)H, a, lda, w1, ldw1, b1, w2, ldw2, b2,
                                                                resid, ldr, out, ldo, ln_w, ln_b, eps);
    else
        k_ffn_f32<false><<<grid, 256, 0, (hipStream_t)stream>>>(M, (int)C, (int)H, a, lda, w1, ldw1, b1, w2, ldw2, b2,
                                                                 resid, ldr, out, ldo, nullptr, nullptr, 0.f);
    CG_LAUNCH_CHECK("cg_ffn_fwd_f32");
    return CG_OK;
}

extern "C" int cg_gemm_resid_layernorm_supported(int64_t M, int64_t N, int64_t K) {
    return gemm_resid_ln_supported(M, N, K) ? 1 : 0;
}

extern "C" int cg_gemm_resid_layernorm(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* W,
                                       int64_t ldw, float* out, int64_t ldc, const cg_epilogue_t* epi,
                                       const float* ln_w, const float* ln_b, void* y, float* mean, float* rstd,
                                       float eps, void* stream) {
    CG_REQUIRE(gemm_resid_ln_supported(M, N, K),
               "cg_gemm_resid_layernorm: unsupported shape M=%lld N=%lld K=%lld (N == 384, M %% 64 == 0, K %% 64 == 0)",
               (long long)M, (long long)N, (long long)K);
    CG_REQUIRE(epi && (epi->kind == CG_EPI_BIAS_RESID || epi->kind == CG_EPI_BIAS_DROP_RESID) && epi->bias &&
                   epi->resid && epi->beta == 0.f && epi->flags == 0 && !epi->colpart,
               "cg_gemm_resid_layernorm: needs a BIAS_RESID / BIAS_DROP_RESID epilogue with bias and residual, beta 0");
    CG_REQUIRE(A && W && out && ln_w && ln_b && y && mean && rstd, "cg_gemm_resid_layernorm: null pointer");
    CG_REQUIRE(lda >= K && ldw >= K && lda % 8 == 0 && ldw % 8 == 0 && ldc >= N && ldc % 4 == 0 &&
                   epi->ld_resid >= N && epi->ld_resid % 4 == 0,
               "cg_gemm_resid_layernorm: bad leading dimensions");
    CG_REQUIRE((((uintptr_t)A | (uintptr_t)W | (uintptr_t)out | (uintptr_t)epi->resid | (uintptr_t)epi->bias |
                 (uintptr_t)ln_w | (uintptr_t)ln_b | (uintptr_t)y) & 15) == 0,
               "cg_gemm_resid_layernorm: operands must be 16-B aligned");
    const EpiArgs e = make_epi(epi);
    gemm_resid_ln_launch(M, K, (const bf16_t*)A, lda, (const bf16_t*)W, ldw, out, ldc, e, ln_w, ln_b, (bf16_t*)y, mean,
                         rstd, eps, (hipStream_t)stream);
    CG_LAUNCH_CHECK("cg_gemm_resid_layernorm");
    return CG_OK;
}

extern "C" int cg_gemm(int op_dtype, int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, const void* A,
                       int64_t lda, const void* B, int64_t ldb, void* C, int c_dtype, int64_t ldc,
                       const cg_epilogue_t* epi, int split_k, void* workspace, void* stream) {
    CG_REQUIRE(M > 0 && N > 0 && K > 0, "cg_gemm: empty problem M=%lld N=%lld K=%lld", (long long)M, (long long)N,
               (long long)K);
    CG_REQUIRE(split_k >= 1 && split_k <= 64, "cg_gemm: split_k out of range");
    CG_REQUIRE(split_k == 1 || workspace, "cg_gemm: split_k > 1 needs a workspace");
    CG_REQUIRE(op_dtype == CG_BF16 || op_dtype == CG_F32, "cg_gemm: bad op dtype");
    hipStream_t st = (hipStream_t)stream;
    EpiArgs e = make_epi(epi);
    CG_REQUIRE(split_k == 1 || e.kind == CG_EPI_STORE || e.kind == CG_EPI_BIAS || e.kind == CG_EPI_BIAS_RESID,
               "cg_gemm: split-K supports STORE/BIAS/BIAS_RESID epilogues only");
    const bool vec4 = N % 4 == 0 && ldc % 4 == 0 && M * N < (int64_t)1 << 31 &&
                      (((uintptr_t)C | (uintptr_t)workspace | (uintptr_t)(e.bias ? e.bias : (const float*)C) |
                        (uintptr_t)(e.resid ? e.resid : (const float*)C)) & 15) == 0 &&
                      (!e.resid || e.ld_resid % 4 == 0);
    bool fast = false;
    const int flags = epi ? epi->flags : 0;
    CG_REQUIRE((flags & ~(CG_GEMM_SLAB_BF16 | CG_GEMM_DEFER_REDUCE)) == 0, "cg_gemm: unknown epilogue flags %#x", flags);
    // bf16 slabs (CG_GEMM_SLAB_BF16): only the 128x128 persistent kernel writes them (fast_gemm_launch
    // declines otherwise, nothing launched) and only the vectorised reduces read them
    e.slab_bf16 = (flags & CG_GEMM_SLAB_BF16) && split_k > 1 && op_dtype == CG_BF16 && e.kind == CG_EPI_STORE &&
                  c_dtype == CG_F32 && vec4 && ldc == N && (M * N) % 8 == 0 && !g_skip_splitk_reduce;
    if (e.slab_bf16) {
        fast = fast_gemm_launch(a_trans, b_trans, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, c_dtype,
                                ldc, e, split_k, (float*)workspace, st);
        if (!fast) e.slab_bf16 = 0;
    }
    if (fast) {
    } else if (op_dtype == CG_BF16 && fast_gemm_launch(a_trans, b_trans, M, N, K, (const bf16_t*)A, lda,
                                                       (const bf16_t*)B, ldb, C, c_dtype, ldc, e, split_k,
                                                       (float*)workspace, st)) {
        fast = true;
    } else if (e.aux_dtype == CG_BITS) {
        set_error("cg_gemm: CG_BITS ReLU keep bits need a persistent bf16 kernel (cg_gemm_relu_bits_supported)");
        return CG_EINVAL;
    } else if (e.kind == CG_EPI_STORE_ROWDOT) {
        set_error("cg_gemm: CG_EPI_STORE_ROWDOT needs the 128x128 persistent bf16 kernel (cg_gemm_rowdot_supported; "
                  "bf16 aux, colpart, ld_resid = T dividing M)");
        return CG_EINVAL;
    } else if (e.colpart) {
        set_error("cg_gemm: colpart needs a persistent bf16 kernel (bf16 operands and output, NT/NN, beta 0, "
                  "split 1, M %% 128 == 0, default dispatch)");
        return CG_EINVAL;
    } else if (op_dtype == CG_BF16) {
        launch_generic<bf16_t, bf16_t>(a_trans, b_trans, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k,
                                       workspace, st);
    } else if (c_dtype == CG_F32 && g_gemm_variant != 99) {  // 99: force the generic kernel (tests)
        launch_f32(a_trans, b_trans, M, N, K, (const float*)A, lda, (const float*)B, ldb, (float*)C, ldc, e, split_k,
                   (float*)workspace, st);
    } else {
        launch_generic<float, float>(a_trans, b_trans, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k,
                                     workspace, st);
    }
    // (slab sets above 40 MB -- the C4 FFN / QKV weight gradients -- keep their own reduce kernel: in
    // the next 256x256 GEMM's tail they measured no gain, C4 58.2 vs 57.9 ms/step)
    if (split_k > 1 && vec4 && !g_skip_splitk_reduce && (flags & CG_GEMM_DEFER_REDUCE) && fast &&
        e.kind == CG_EPI_STORE && c_dtype == CG_F32 && ldc == N &&
        (int64_t)split_k * M * N * 4 <= ((int64_t)40 << 20)) {
        // deferred: summed in the tail of the next persistent GEMM launch on this stream of this
        // device (or cg_flush_deferred(st) there) -- the queue key holds the device, so the null
        // stream, whose handle names a different queue on every device, is fine too
        std::lock_guard<std::mutex> lk(defer_mutex());
        DeferQueue& q = *defer_queue(st, true);
        if (q.nred == MAX_RED) flush_red_locked(q);
        q.red[q.nred++] = RedJob{(const float*)workspace, (float*)C, M * N / 4, split_k, e.beta, e.slab_bf16};
    } else if (split_k > 1 && e.slab_bf16) {
        const int64_t n8 = M * N / 8;
        k_slab16_reduce8<<<ceil_div(n8, 256), 256, 0, st>>>(workspace, split_k, n8, (float*)C, e.beta);
    } else if (split_k > 1 && vec4 && !g_skip_splitk_reduce) {
        const int n4 = (int)(M * N / 4);
#define SKR(TC_, S_)                                                                                  \
    k_splitk_reduce4<TC_, S_><<<ceil_div(n4, 256), 256, 0, st>>>((const float*)workspace, split_k, (int)M, \
                                                                 (int)N, (TC_*)C, ldc, e)
#define SKR_ANY(TC_)                        \
    switch (split_k) {                      \
        case 2: SKR(TC_, 2); break;         \
        case 4: SKR(TC_, 4); break;         \
        case 8: SKR(TC_, 8); break;         \
        case 12: SKR(TC_, 12); break;       \
        case 14: SKR(TC_, 14); break;       \
        case 16: SKR(TC_, 16); break;       \
        case 32: SKR(TC_, 32); break;       \
        default: SKR(TC_, 0); break;        \
    }
        if (c_dtype == CG_BF16) {
            SKR_ANY(bf16_t)
        } else {
            SKR_ANY(float)
        }
#undef SKR_ANY
#undef SKR
    } else if (split_k > 1) {
        const int64_t n = M * N;
        if (c_dtype == CG_BF16)
            k_splitk_reduce<bf16_t><<<ceil_div(n, 256), 256, 0, st>>>((const float*)workspace, split_k, M, N,
                                                                      (bf16_t*)C, ldc, e);
        else
            k_splitk_reduce<float><<<ceil_div(n, 256), 256, 0, st>>>((const float*)workspace, split_k, M, N,
                                                                     (float*)C, ldc, e);
    }
    CG_LAUNCH_CHECK("cg_gemm");
    return CG_OK;
}

extern "C" int cg_reduce_rows_ex(const float* part, int64_t rows, int64_t N, float* out, int accumulate, int flags,
                                 void* stream) {
    CG_REQUIRE(part && out && rows > 0 && N > 0, "cg_reduce_rows: bad arguments");
    CG_REQUIRE((flags & ~CG_DEFER) == 0, "cg_reduce_rows_ex: unknown flags %#x", flags);
    reduce_partials_deferrable(part, rows, N, out, nullptr, nullptr, N, accumulate, 0, flags & CG_DEFER,
                               (hipStream_t)stream);
    CG_LAUNCH_CHECK("cg_reduce_rows");
    return CG_OK;
}

extern "C" int cg_reduce_rows(const float* part, int64_t rows, int64_t N, float* out, int accumulate, void* stream) {
    return cg_reduce_rows_ex(part, rows, N, out, accumulate, 0, stream);
}

extern "C" int64_t cg_colsum_workspace(int64_t rows, int64_t N) {
    return ((rows + CS_ROWS - 1) / CS_ROWS) * N * (int64_t)sizeof(float);
}

extern "C" int cg_colsum(const void* X, int x_dtype, int64_t rows, int64_t N, int64_t ldx, float* out, int accumulate,
                         void* workspace, void* stream) {
    CG_REQUIRE(rows > 0 && N > 0, "cg_colsum: empty");
    hipStream_t st = (hipStream_t)stream;
    const int64_t nchunk = (rows + CS_ROWS - 1) / CS_ROWS;
    dim3 grid(ceil_div(N, 64), (unsigned)nchunk);
    if (x_dtype == CG_BF16)
        k_colsum_partial<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)X, rows, N, ldx, (float*)workspace);
    else
        k_colsum_partial<float><<<grid, 256, 0, st>>>((const float*)X, rows, N, ldx, (float*)workspace);
    launch_reduce_partials((const float*)workspace, nchunk, N, out, nullptr, N, accumulate, st);
    CG_LAUNCH_CHECK("cg_colsum");
    return CG_OK;
}

namespace cg {
static void launch_splitk_reduce_job(const RedJob& j, hipStream_t st) {
    if (j.bf16 && (j.n4 & 1) == 0) {   // red_tail's bf16 form, standalone
        k_slab16_reduce8<<<ceil_div(j.n4 / 2, 256), 256, 0, st>>>(j.ws, j.S, j.n4 / 2, j.out, j.beta);
        return;
    }
    EpiArgs e = make_epi(nullptr);
    e.beta = j.beta;
    e.slab_bf16 = j.bf16;
    const int64_t n = 4 * j.n4;
    const int n4 = (int)j.n4;
    // one row of n elements: the same kernel and summation order as the in-line reduce
    switch (j.S) {
#define SKJ(S_) k_splitk_reduce4<float, S_><<<ceil_div(n4, 256), 256, 0, st>>>(j.ws, j.S, 1, (int)n, j.out, n, e)
        case 8: SKJ(8); break;
        case 14: SKJ(14); break;
        case 16: SKJ(16); break;
        case 32: SKJ(32); break;
        default: SKJ(0); break;
#undef SKJ
    }
}
}  // namespace cg

extern "C" int cg_adamw_defer(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, double lr,
                              double beta1, double beta2, double eps, double weight_decay, const int64_t* step_ptr,
                              void* stream) {
    using namespace cg;
    CG_REQUIRE(p && g && m && v && p_bf16 && step_ptr && n > 0 && n % 4 == 0,
               "cg_adamw_defer: bad arguments (n must be a positive multiple of 4)");
    CG_REQUIRE(((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                   (((uintptr_t)p_bf16) & 7) == 0,
               "cg_adamw_defer: p, g, m, v must be 16-B aligned, p_bf16 8-B aligned");
    hipStream_t st = (hipStream_t)stream;
    {
        std::lock_guard<std::mutex> lk(defer_mutex());
        DeferQueue& q = *defer_queue(st, true);
        DeviceScope ds(q.device);
        // the region's gradient must be final first: a pending split-K reduce or column-sum reduce
        // writing into it goes out now
        for (int i = 0; i < q.nred; ++i)
            if (q.red[i].out < g + n && g < q.red[i].out + 4 * q.red[i].n4) {
                flush_red_locked(q);
                break;
            }
        flush_parts_touching_locked(&q, g, n);
        if (q.nadam == MAX_ADAM_PENDING) flush_adam_locked(q);
        q.adam[q.nadam++] = AdamJob{p, g, m, v, (bf16_t*)p_bf16, n / 4, lr, beta1, beta2, eps, weight_decay, step_ptr};
    }
    CG_LAUNCH_CHECK("cg_adamw_defer");
    return CG_OK;
}

extern "C" int cg_flush_deferred(void* stream) {
    using namespace cg;
    {
        std::lock_guard<std::mutex> lk(defer_mutex());
        DeferQueue* q = defer_queue((hipStream_t)stream, false);
        if (q) {
            DeviceScope ds(q->device);
            flush_red_locked(*q);
            flush_adam_locked(*q);
            flush_parts_locked(*q);
            q->adam_taken = 0;
            defer_queue_drop(q);
        }
    }
    CG_LAUNCH_CHECK("cg_flush_deferred");
    return CG_OK;
}

extern "C" int cg_discard_deferred(void* stream, int* adam_jobs_taken) {
    using namespace cg;
    int taken = 0;
    {
        std::lock_guard<std::mutex> lk(defer_mutex());
        DeferQueue* q = defer_queue((hipStream_t)stream, false);
        if (q) {
            taken = q->adam_taken;
            q->nred = q->nadam = q->parts.n = q->adam_taken = 0;
            defer_queue_drop(q);
        }
    }
    if (adam_jobs_taken) *adam_jobs_taken = taken;
    return CG_OK;
}
