// charpt GEMM internals shared by gemm.hip (generic path, dispatch) and gemm_bf16.hip (MFMA path).
#pragma once
#include "common.h"

namespace cg {

struct EpiArgs {
    int kind;
    const float* bias;
    const float* resid;
    int64_t ld_resid;
    const void* aux;
    int aux_dtype;
    int64_t ld_aux;
    uint32_t thr;
    float dscale;
    uint64_t seed;
    const uint64_t* rng_call;
    int site;
    float beta;
    float* colpart;  // RELU_BWD: per-64-row-block column sums; STORE_ROWDOT: per-head row dots (k_gemm_pk only)
};

__device__ __forceinline__ float aux_at(const EpiArgs& e, int64_t m, int64_t n) {
    return e.aux_dtype == CG_BF16 ? bf2f(((const bf16_t*)e.aux)[m * e.ld_aux + n])
                                  : ((const float*)e.aux)[m * e.ld_aux + n];
}

// scalar epilogue (generic path and split-K reduce); idx for dropout = m*N + n
__device__ __forceinline__ float epi_scalar(const EpiArgs& e, float v, int64_t m, int64_t n, int64_t N,
                                            uint64_t stream) {
    switch (e.kind) {
        case CG_EPI_BIAS:
            if (e.bias) v += e.bias[n];
            break;
        case CG_EPI_BIAS_RELU:
            if (e.bias) v += e.bias[n];
            v = fmaxf(v, 0.f);
            break;
        case CG_EPI_BIAS_RESID:
            if (e.bias) v += e.bias[n];
            if (e.resid) v = e.resid[m * e.ld_resid + n] + v;
            break;
        case CG_EPI_BIAS_DROP_RESID: {
            if (e.bias) v += e.bias[n];
            const uint64_t idx = (uint64_t)m * (uint64_t)N + (uint64_t)n;
            if (e.thr) v = keep_of(philox_of(e.seed, stream, idx), idx, e.thr) ? v * e.dscale : 0.f;
            if (e.resid) v = e.resid[m * e.ld_resid + n] + v;
            break;
        }
        case CG_EPI_RELU_BWD:
            v = aux_at(e, m, n) > 0.f ? v : 0.f;
            break;
        default:
            break;
    }
    return v;
}

template <typename TC>
__device__ __forceinline__ void store_out(TC* C, int64_t off, float v, float beta) {
    if (beta != 0.f) v += beta * ld_as_f32<TC>(C + off);
    st_from_f32<TC>(C + off, v);
}


// A split-K reduce deferred out of its own cg_gemm call (cg_set_tuning("defer_splitk", 1), the
// training backward): out[i] = sum_{s < S} ws[s n + i] (+ beta out[i]) over n = 4 n4 fp32 elements,
// run in the tail of the next persistent GEMM launch on the stream (each thread takes float4
// chunks once its block's own items are done) or by cg_flush_deferred.  Slab 0 first, then 1, ...:
// k_splitk_reduce4's order, so the same bits.
struct RedJob {
    const float* ws;
    float* out;
    int64_t n4;
    int S;
    float beta;
};
constexpr int MAX_RED = 2;
struct RedJobs {
    RedJob j[MAX_RED];
    int n;
};
RedJobs take_pending_reduces(hipStream_t st);   // gemm.hip: pending jobs (cleared) for a launch on st

// thread t sums float4 chunks t, t + threads, ... of every job
__device__ __forceinline__ void red_tail(const RedJobs& r) {
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int q = 0; q < r.n; ++q) {
        const RedJob& J = r.j[q];
        const int64_t slab = 4 * J.n4;
        for (int64_t i = t0; i < J.n4; i += nthr) {
            const float* p = J.ws + 4 * i;
            fv4 s = __builtin_nontemporal_load((const fv4*)p);
#pragma unroll 8
            for (int k = 1; k < J.S; ++k) s += __builtin_nontemporal_load((const fv4*)(p + k * slab));
            fv4* o = (fv4*)(J.out + 4 * i);
            if (J.beta != 0.f) s += J.beta * *o;
            *o = s;
        }
    }
}

// tuning knob (cg_set_tuning("gemm_variant", v)); 0 = automatic choice
extern int g_gemm_variant;
// test knob (cg_set_tuning("gemm_max_grid", n)): cap on persistent-kernel blocks; 0 = resident slots
extern int g_gemm_max_grid;
extern int g_gemm_group_p8;
extern int g_gemm_group_pk;
extern int g_gemm_n96;
// test knob (cg_set_tuning("pk_flags", f)) for the persistent kernel's epilogue (gemm_pk.hip)
extern int g_pk_flags;
int gemm_cu_count();  // compute units of the current device (cached; gemm_pk.hip)

// launches the bf16 MFMA kernel if the problem qualifies; returns false (nothing launched) if not
bool fast_gemm_launch(int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* B,
                      int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k, float* ws,
                      hipStream_t st);
// whether cg_gemm (bf16, split 1, CG_EPI_RELU_BWD with bf16 aux, beta 0) can write column partials
bool gemm_colpart_supported(int at, int bt, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
// whether cg_gemm can write / read CG_BITS ReLU keep bits for this problem (bf16, split 1, beta 0)
bool gemm_rowdot_supported(int at, int bt, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
bool gemm_relu_bits_supported(int at, int bt, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
// LDS-DMA (global_load_lds) kernels, variant >= 5 (gemm_glds.hip); false if the variant/shape does not apply
bool glds_gemm_launch(int variant, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                      const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                      float* ws, hipStream_t st);
// persistent LDS-DMA kernels with register epilogues, variant >= 9 (gemm_pk.hip)
bool pk_gemm_launch(int variant, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                    const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                    float* ws, hipStream_t st);

// persistent 8-wave LDS-DMA kernels (gemm_p8.hip), variant >= 20 (20 = automatic tile choice)
bool p8_gemm_launch(int variant, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                    const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                    float* ws, hipStream_t st);

}  // namespace cg
