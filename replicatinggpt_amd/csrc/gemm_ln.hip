// charpt: a residual-stream GEMM fused with the LayerNorm that reads its output -- the attention
// projection (GPT1.py:136, x + sa(ln1(x)) at :163) followed by ln2 (:160, 164), and the FFN's second
// Linear + dropout (:145-147, x + ffwd(ln2(x)) at :164) followed by the next block's ln1 (:159) or
// ln_f (:173).  cg_gemm's fp32 residual epilogue writes x = resid + [dropout](A W^T + bias) and the
// next launch reads x back for LayerNorm(x); here one workgroup owns whole rows (a 64 x 384 row
// panel: N = n_embd = 384, C2), so the same epilogue also keeps the panel's x in LDS and normalises
// it there: y = LN(x) (bf16), mean, rstd -- the x re-read (25 MB per launch at C2) and one launch
// per LayerNorm are gone.  Bits: the GEMM arithmetic (K order, fp32 accumulation, bias -> dropout ->
// residual, Philox keep bits from drop_nibbles_rows) is k_gemm_pk's residual epilogue's, and the row
// math is ln_fwd_row, shared with k_ln_fwd (test_gemm_resid_layernorm_matches_two_launches).
//
// Layout: 8 waves (2 per SIMD), one 64-row panel per workgroup (M / 64 workgroups, one per CU at C2).
// Wave w owns output columns 48 w .. 48 w + 47 (3 fragments of 16) of all 64 rows (4 fragments);
// swapped MFMA operands, so lane l holds row 16 i + (l & 15), columns 16 j + 4 (l >> 4) .. +3.
// K-loop: LDS-DMA rings (gemm_tile.h swizzled images), one barrier per K-tile: W (384 x 64 = 48 KB,
// L2-resident, shared by every workgroup) 2 stages, requested one K-tile ahead; A (64 x 64 = 8 KB,
// streamed from HBM) 4 stages, requested three ahead.
// Epilogue: x fp32 to HBM and to an LDS tile [64][388] (reusing the ring), barrier, then wave w
// normalises rows 8 w .. 8 w + 7 in ln_fwd_row's lane layout (VEC 2, NJ 3).
#include "gemm_tile.h"
#include "ln_fwd.h"

namespace cg {
namespace {
using namespace gt;

constexpr int RL_BM = 64, RL_N = 384, RL_WAVES = 8, RL_THREADS = 64 * RL_WAVES, RL_NJ = 3;
constexpr int RL_IMG_A = RL_BM * FBK * 2, RL_IMG_B = RL_N * FBK * 2;
constexpr int RL_AOFF = 2 * RL_IMG_B;                 // W stages [0, 96 KB), A stages [96 KB, 128 KB)
constexpr int RL_LDS = RL_AOFF + 4 * RL_IMG_A;        // 128 KB: one workgroup per CU
constexpr int RL_XLD = RL_N + 4;       // x tile row pitch (floats): 16 lanes of a column write 16 banks apart
static_assert(RL_BM * RL_XLD * 4 <= RL_LDS, "x tile fits the ring");

template <int N>
__device__ __forceinline__ void rl_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA of R rows x 64 k (K-contiguous rows, gemm_tile.h img_row_off image), PER_WAVE 1-KB
// wave-instructions per wave
template <int R>
struct RlDma {
    static constexpr int PER_WAVE = R * FBK * 2 / 1024 / RL_WAVES;
    static_assert(PER_WAVE * RL_WAVES * 1024 == R * FBK * 2, "tile/wave mismatch");
    uint32_t off[PER_WAVE];
    __device__ __forceinline__ void init(int64_t ld, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) {
            const int pos = (wave * PER_WAVE + i) * 1024 + lane * 16;
            const int r = pos >> 7, c = ((pos >> 4) & 7) ^ row_swz(r);
            off[i] = 2u * (uint32_t)((int)(r * ld) + c * 8);
        }
    }
    __device__ __forceinline__ void issue(const bf16_t* base, uint32_t img, int wave) const {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) dma16sl(base, off[i], img + (uint32_t)((wave * PER_WAVE + i) * 1024));
    }
};

template <bool DROP>
__global__ __launch_bounds__(RL_THREADS, 1) void k_gemm_resid_ln(int64_t K, const bf16_t* __restrict__ A, int64_t lda,
                                                                const bf16_t* __restrict__ W, int64_t ldw,
                                                                float* __restrict__ X, int64_t ldx, EpiArgs epi,
                                                                const float* __restrict__ lnw,
                                                                const float* __restrict__ lnb, bf16_t* __restrict__ Y,
                                                                float* __restrict__ mean, float* __restrict__ rstd,
                                                                float eps) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t m0 = (int64_t)blockIdx.x * RL_BM;
    const int nk = (int)(K / FBK);
    RlDma<RL_BM> da;
    RlDma<RL_N> db;
    da.init(lda, wave, lane);
    db.init(ldw, wave, lane);
    const bf16_t* a0 = A + m0 * lda;
    const uint32_t lds0 = lds_base(smem);
    auto issue_w = [&](int kt) { db.issue(W + (int64_t)kt * FBK, lds0 + (uint32_t)((kt & 1) * RL_IMG_B), wave); };
    auto issue_a = [&](int kt) {
        da.issue(a0 + (int64_t)kt * FBK, lds0 + (uint32_t)(RL_AOFF + (kt & 3) * RL_IMG_A), wave);
    };
    fv4 acc[4][RL_NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < RL_NJ; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    // issue order: W0 A0 A1 A2 | head kt: W(kt+1) A(kt+3).  At head kt, W(kt) and everything older
    // (A(kt) among it) must have landed; only A(kt+2) (and, at kt = 0, A1 A2) is younger
    issue_w(0);
#pragma unroll
    for (int t = 0; t < 3; ++t)
        if (t < nk) issue_a(t);
    for (int kt = 0; kt < nk; ++kt) {
        const int younger = kt == 0 ? (nk - 1 < 2 ? nk - 1 : 2) : (kt + 2 < nk ? 1 : 0);
        if (younger == 2) rl_wait_vm<2>();
        else if (younger == 1) rl_wait_vm<1>();
        else rl_wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // ... for every wave; everyone is done with K-tile kt - 1's stages
        if (kt + 1 < nk) issue_w(kt + 1);
        if (kt + 3 < nk) issue_a(kt + 3);
        const char* imgB = smem + (kt & 1) * RL_IMG_B;
        const char* imgA = smem + RL_AOFF + (kt & 3) * RL_IMG_A;
        sv8 af[2][4], bf[2][RL_NJ];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int j = 0; j < RL_NJ; ++j) bf[s][j] = frag<false, RL_N>(imgB, 48 * wave + 16 * j, s, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i) af[s][i] = frag<false, RL_BM>(imgA, 16 * i, s, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < RL_NJ; ++j) acc[i][j] = mfma_bf16(bf[s][j], af[s][i], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
    }
    // ---- residual epilogue (k_gemm_pk epi_resid_nj's arithmetic and order): x = resid + [drop](acc + b)
    const int64_t mr = m0 + (lane & 15);
    const int ncl = 48 * wave + 4 * (lane >> 4);   // the lane's first column
    float4 bv[RL_NJ];
#pragma unroll
    for (int j = 0; j < RL_NJ; ++j) bv[j] = *(const float4*)(epi.bias + ncl + 16 * j);
    float4 r[4][RL_NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < RL_NJ; ++j) r[i][j] = *(const float4*)(epi.resid + (mr + 16 * i) * epi.ld_resid + ncl + 16 * j);
    uint32_t nib[4][RL_NJ];
    if constexpr (DROP) drop_nibbles_rows<RL_NJ>(epi, dropout_stream(epi.rng_call, epi.site), mr, ncl, RL_N, nib);
    rl_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave's last fragment reads are done: the rings become the x tile
    float* xs = (float*)smem;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < RL_NJ; ++j) {
            fv4 v = acc[i][j];
            v[0] += bv[j].x; v[1] += bv[j].y; v[2] += bv[j].z; v[3] += bv[j].w;
            if constexpr (DROP) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = ((nib[i][j] >> q) & 1u) ? v[q] * epi.dscale : 0.f;
            }
            v[0] = r[i][j].x + v[0]; v[1] = r[i][j].y + v[1]; v[2] = r[i][j].z + v[2]; v[3] = r[i][j].w + v[3];
            const float4 o = make_float4(v[0], v[1], v[2], v[3]);
            *(float4*)(X + (mr + 16 * i) * ldx + ncl + 16 * j) = o;
            *(float4*)(xs + (16 * i + (lane & 15)) * RL_XLD + ncl + 16 * j) = o;
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- LayerNorm of the panel's rows (k_ln_fwd's row math, VEC 2, NJ 3)
    constexpr float invC = 1.0f / (float)RL_N;
    float wv[3][2], bw[3][2];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int e = (j * 64 + lane) * 2;
        VecIO<2>::ld(lnw + e, wv[j]);
        VecIO<2>::ld(lnb + e, bw[j]);
    }
#pragma unroll 2
    for (int rr = 0; rr < RL_BM / RL_WAVES; ++rr) {
        const int row = RL_WAVES * rr + wave;
        float v[3][2];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float2 t = *(const float2*)(xs + row * RL_XLD + (j * 64 + lane) * 2);
            v[j][0] = t.x;
            v[j][1] = t.y;
        }
        float mu, rs;
        ln_fwd_row<2, 3, bf16_t, true>(v, wv, bw, RL_N, invC, eps, lane, Y + (m0 + row) * RL_N, mu, rs);
        if (lane == 0) {
            mean[m0 + row] = mu;
            rstd[m0 + row] = rs;
        }
    }
}

}  // namespace

bool gemm_resid_ln_supported(int64_t M, int64_t N, int64_t K) {
    return N == RL_N && M > 0 && M % RL_BM == 0 && K > 0 && K % FBK == 0 && M / RL_BM < (1LL << 31);
}

// host-checked by cg_gemm_resid_layernorm: shape, kinds, alignment
void gemm_resid_ln_launch(int64_t M, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, float* X,
                          int64_t ldx, const EpiArgs& e, const float* lnw, const float* lnb, bf16_t* Y, float* mean,
                          float* rstd, float eps, hipStream_t st) {
    const unsigned grid = (unsigned)(M / RL_BM);
    if (e.kind == CG_EPI_BIAS_DROP_RESID && e.thr)
        k_gemm_resid_ln<true><<<grid, RL_THREADS, RL_LDS, st>>>(K, A, lda, W, ldw, X, ldx, e, lnw, lnb, Y, mean, rstd, eps);
    else
        k_gemm_resid_ln<false><<<grid, RL_THREADS, RL_LDS, st>>>(K, A, lda, W, ldw, X, ldx, e, lnw, lnb, Y, mean, rstd,
                                                                eps);
}

}  // namespace cg
