// charpt GEMM internals shared by gemm.hip (generic path, dispatch) and gemm_bf16.hip (MFMA path).
#pragma once
#include "adamw.h"
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
    int slab_bf16;   // split-K: the per-split partial sums stored as bf16 slabs (cg_epilogue_t.flags CG_GEMM_SLAB_BF16)
};

// four consecutive slab elements as fp32 (bf16 slabs: one 8-B load, exact widening)
typedef unsigned slab_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fv4 ld_slab4(const void* ws, int64_t idx, bool bf16) {
    if (bf16) {
        const slab_u2 w = __builtin_nontemporal_load((const slab_u2*)((const bf16_t*)ws + idx));
        return fv4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                   __uint_as_float(w.y & 0xffff0000u)};
    }
    return __builtin_nontemporal_load((const fv4*)((const float*)ws + idx));
}

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


// A split-K reduce deferred out of its own cg_gemm call (CG_GEMM_DEFER_REDUCE, the training
// backward; queued per stream, defer.h): out[i] = sum_{s < S} ws[s n + i] (+ beta out[i]) over n = 4 n4 fp32 elements,
// run in the tail of the next persistent GEMM launch on the stream (each thread takes float4
// chunks once its block's own items are done) or by cg_flush_deferred.  Slab 0 first, then 1, ...:
// k_splitk_reduce4's order, so the same bits.
struct RedJob {
    const float* ws;   // fp32 slabs, or bf16 ones (bf16 != 0)
    float* out;
    int64_t n4;
    int S;
    float beta;
    int bf16;
};
constexpr int MAX_RED = 2;
// An AdamW update of one weight region deferred onto the free blocks of a later part-filling
// persistent GEMM launch (cg_adamw_defer; the training step's weight matrices once their gradient
// is final and the backward no longer reads their bf16 shadow): adam_one per element, so the bits
// of the AdamW kernel.  n4 float4 chunks; p, g, m, v 16-B aligned, pb 8-B aligned.
struct AdamJob {
    float* p;
    const float* g;
    float* m;
    float* v;
    bf16_t* pb;
    int64_t n4;
    double lr, beta1, beta2, eps, wd;
    const int64_t* step;
};
constexpr int MAX_ADAM = 4;
struct RedJobs {
    RedJob j[MAX_RED];
    int n;
    AdamJob a[MAX_ADAM];
    int na;   // AdamW jobs: only a launch with free blocks (red_tail `first` > 0) is given any
    int adam_batch;   // A/B build only (cg_set_tuning "adam_batch"): chunks in flight per thread (1 = product loop)
};
// gemm.hip: pending jobs (cleared) for a launch on st -- the split-K reduces, and with side_ok (the
// launch has >= SIDE_MIN free blocks) the AdamW jobs; has_pending_reduces: whether it would take any
constexpr int SIDE_MIN = 64;
RedJobs take_pending_reduces(hipStream_t st, bool side_ok = false);
bool has_pending_reduces(hipStream_t st, bool side_ok = false);

// out[8i .. 8i+7] = sum over slabs k = 0..S-1 (in order, fp32) of bf16 slab elements (one 16-B load
// per slab), (+ beta out): the deferred tail and the standalone reduce of bf16 slabs (same bits)
__device__ __forceinline__ void slab16_chunk8(const void* ws, int S, int64_t slab, int64_t i, float* out, float beta) {
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    fv4 lo = fv4{0.f, 0.f, 0.f, 0.f}, hi = lo;
#pragma unroll 8
    for (int k = 0; k < S; ++k) {
        const u4v w = __builtin_nontemporal_load((const u4v*)((const bf16_t*)ws + 8 * i + k * slab));
        const fv4 a = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                       __uint_as_float(w.y & 0xffff0000u)};
        const fv4 b = {__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u), __uint_as_float(w.w << 16),
                       __uint_as_float(w.w & 0xffff0000u)};
        if (k == 0) {
            lo = a;
            hi = b;
        } else {
            lo += a;
            hi += b;
        }
    }
    fv4* o = (fv4*)(out + 8 * i);
    if (beta != 0.f) {
        lo += beta * o[0];
        hi += beta * o[1];
    }
    o[0] = lo;
    o[1] = hi;
}

// thread t sums float4 chunks t, t + threads, ... of every job.  first > 0: only blocks first ..
// grid - 1 take part -- the blocks a part-filling GEMM launch was given beyond its items, which run
// the reduce beside the items instead of after them
__device__ __forceinline__ void red_tail(const RedJobs& r, int first = 0) {
    if ((int)blockIdx.x < first) return;
    const int64_t nthr = (int64_t)(gridDim.x - first) * blockDim.x;
    const int64_t t0 = (int64_t)(blockIdx.x - first) * blockDim.x + threadIdx.x;
    for (int q = 0; q < r.n; ++q) {
        const RedJob& J = r.j[q];
        const int64_t slab = 4 * J.n4;
        if (J.bf16 && (J.n4 & 1) == 0) {   // bf16 slabs: 8 elements (one 16-B load) per slab per chunk
            for (int64_t i = t0; i < J.n4 / 2; i += nthr) slab16_chunk8(J.ws, J.S, slab, i, J.out, J.beta);
            continue;
        }
        for (int64_t i = t0; i < J.n4; i += nthr) {
            fv4 s = ld_slab4(J.ws, 4 * i, J.bf16);
#pragma unroll 8
            for (int k = 1; k < J.S; ++k) s += ld_slab4(J.ws, 4 * i + k * slab, J.bf16);
            fv4* o = (fv4*)(J.out + 4 * i);
            if (J.beta != 0.f) s += J.beta * *o;
            *o = s;
        }
    }
#ifdef CG_AB_VARIANTS
    // A/B: four float4 chunks in flight per thread, all loads first.  Batch b of
    // thread t holds chunks t + (4 b + s) nthr, s = 0..3 -- disjoint batches (stride 4 nthr), so every
    // chunk is updated exactly once, as in the product loop below.
    // adam_batch 5: the same loop with batches stepping by nthr (overlapping: chunk t + k nthr is
    // re-processed by up to four batches of thread t) -- the candidate cause of round 4's failure
    if (r.adam_batch == 4 || r.adam_batch == 5) {
        const int64_t stride = r.adam_batch == 4 ? 4 * nthr : nthr;
        for (int q = 0; q < r.na; ++q) {
            const AdamJob& J = r.a[q];
            const AdamScalars sc = adam_scalars(J.lr, J.beta1, J.beta2, J.eps, J.wd, J.step);
            for (int64_t i0 = t0; i0 < J.n4; i0 += stride) {
                fv4 pv[4], gv[4], mv[4], vv[4];
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int64_t i = i0 + s * nthr;
                    if (i < J.n4) {
                        pv[s] = *(const fv4*)(J.p + 4 * i);
                        gv[s] = *(const fv4*)(J.g + 4 * i);
                        mv[s] = *(const fv4*)(J.m + 4 * i);
                        vv[s] = *(const fv4*)(J.v + 4 * i);
                    }
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int64_t i = i0 + s * nthr;
                    if (i < J.n4) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float me = mv[s][e], ve = vv[s][e];
                            pv[s][e] = adam_one(pv[s][e], gv[s][e], me, ve, sc);
                            mv[s][e] = me;
                            vv[s][e] = ve;
                        }
                        *(fv4*)(J.p + 4 * i) = pv[s];
                        *(fv4*)(J.m + 4 * i) = mv[s];
                        *(fv4*)(J.v + 4 * i) = vv[s];
                        *(uint2*)(J.pb + 4 * i) = make_uint2(pack_bf2(pv[s][0], pv[s][1]), pack_bf2(pv[s][2], pv[s][3]));
                    }
                }
            }
        }
        return;
    }
#endif
    // AdamW jobs (free blocks only: first > 0): float4 chunk per thread per step, adam_one per element.
    // Thread t of the nthr side threads owns chunks t, t + nthr, t + 2 nthr, ...: each chunk exactly
    // once (a bijection chunk -> (thread, step)), so no chunk's update can read another's store.
    for (int q = 0; q < r.na; ++q) {
        const AdamJob& J = r.a[q];
        const AdamScalars sc = adam_scalars(J.lr, J.beta1, J.beta2, J.eps, J.wd, J.step);
        for (int64_t i = t0; i < J.n4; i += nthr) {
            fv4 pv = *(const fv4*)(J.p + 4 * i);
            const fv4 gv = *(const fv4*)(J.g + 4 * i);
            fv4 mv = *(const fv4*)(J.m + 4 * i), vv = *(const fv4*)(J.v + 4 * i);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float me = mv[e], ve = vv[e];
                pv[e] = adam_one(pv[e], gv[e], me, ve, sc);
                mv[e] = me;
                vv[e] = ve;
            }
            *(fv4*)(J.p + 4 * i) = pv;
            *(fv4*)(J.m + 4 * i) = mv;
            *(fv4*)(J.v + 4 * i) = vv;
            *(uint2*)(J.pb + 4 * i) = make_uint2(pack_bf2(pv[0], pv[1]), pack_bf2(pv[2], pv[3]));
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
extern int g_red_side;
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
// gemm_ln.hip: the residual GEMM + next LayerNorm kernel (N = 384 row panels)
bool gemm_resid_ln_supported(int64_t M, int64_t N, int64_t K);
void gemm_resid_ln_launch(int64_t M, int64_t K, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, float* X,
                          int64_t ldx, const EpiArgs& e, const float* lnw, const float* lnb, bf16_t* Y, float* mean,
                          float* rstd, float eps, hipStream_t st);
bool p8_gemm_launch(int variant, int at, int bt, int64_t M, int64_t N, int64_t K, const bf16_t* A, int64_t lda,
                    const bf16_t* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                    float* ws, hipStream_t st);

}  // namespace cg
