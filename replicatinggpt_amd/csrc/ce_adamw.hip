// charpt: cross entropy over the character vocabulary (F.cross_entropy, GPT1.py:189-192) and
// the fused AdamW step over flat fp32 buffers (torch.optim.AdamW, GPT1.py:218,233).
#include <math.h>

#include "adamw.h"
#include "common.h"
#include "gemm_common.h"

using namespace cg;

// ---- cross entropy: one wave per row, V <= 64*16 ------------------------------------------
__global__ __launch_bounds__(256) void k_ce_fwd(const float* __restrict__ logits, int64_t rows, int V, int64_t ld,
                                                const int64_t* __restrict__ targets, float* __restrict__ loss_rows,
                                                float* __restrict__ lse) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* x = logits + r * ld;
    float mx = -INFINITY;
    for (int v = lane; v < V; v += 64) mx = fmaxf(mx, x[v]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int v = lane; v < V; v += 64) s += expf(x[v] - mx);
    s = wave_sum(s);
    const float l = mx + logf(s);
    if (lane == 0) {
        lse[r] = l;
        if (targets && loss_rows) {
            // F.cross_entropy raises on a target outside [0, V) (ignore_index is never produced by
            // GPT1.py): the row loss turns NaN instead, so a bad label cannot pass silently
            const int64_t t = targets[r];
            loss_rows[r] = (t < 0 || t >= V) ? __builtin_nanf("") : l - x[t];
        }
    }
}

extern "C" int cg_ce_fwd(const float* logits, int64_t rows, int64_t V, int64_t ld, const int64_t* targets,
                         float* loss_rows, float* lse, void* stream) {
    CG_REQUIRE(rows > 0 && V > 0 && V <= 1024, "cg_ce_fwd: bad shape");
    k_ce_fwd<<<ceil_div(rows, 4), 256, 0, (hipStream_t)stream>>>(logits, rows, (int)V, ld, targets, loss_rows, lse);
    CG_LAUNCH_CHECK("cg_ce_fwd");
    return CG_OK;
}

__global__ void k_ce_bwd(const float* __restrict__ logits, int64_t rows, int V, int64_t ld,
                         const int64_t* __restrict__ targets, const float* __restrict__ lse,
                         const float* __restrict__ gp, float g_mult, float* __restrict__ dlogits, int64_t ldd,
                         bf16_t* __restrict__ dlp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * V) return;
    const int64_t r = i / V;
    const int v = (int)(i % V);
    const float g = *gp * g_mult;
    const int64_t t = targets[r];
    const float p = expf(logits[r * ld + v] - lse[r]);
    const float d = (t < 0 || t >= V) ? __builtin_nanf("") : g * (p - (v == t ? 1.f : 0.f));
    if (dlogits) dlogits[r * ldd + v] = d;
    if (dlp) dlp[r * ldd + v] = f2bf(d);
}

extern "C" int cg_ce_bwd(const float* logits, int64_t rows, int64_t V, int64_t ld, const int64_t* targets,
                         const float* lse, const float* g, float g_mult, float* dlogits, int64_t ld_d,
                         void* dst_lp, void* stream) {
    CG_REQUIRE(rows > 0 && V > 0, "cg_ce_bwd: bad shape");
    k_ce_bwd<<<ceil_div(rows * V, 256), 256, 0, (hipStream_t)stream>>>(logits, rows, (int)V, ld, targets, lse, g, g_mult,
                                                                       dlogits, ld_d, (bf16_t*)dst_lp);
    CG_LAUNCH_CHECK("cg_ce_bwd");
    return CG_OK;
}

// ---- AdamW ------------------------------------------------------------------------------
// element arithmetic and the per-launch scalars: adamw.h (shared with the GEMM side blocks)
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned nu2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* p) {
    if constexpr (NT) {
        const nf4 x = __builtin_nontemporal_load((const nf4*)p);
        return make_float4(x[0], x[1], x[2], x[3]);
    } else {
        return *(const float4*)p;
    }
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, float4 x) {
    if constexpr (NT) __builtin_nontemporal_store(nf4{x.x, x.y, x.z, x.w}, (nf4*)p);
    else *(float4*)p = x;
}


// U float4 groups per thread per iteration (all loads issued before any arithmetic); NT: the
// 30 B/param stream bypasses the caches (non-temporal loads and stores) -- every byte is touched once
template <bool VEC, bool NT, int U>
__global__ __launch_bounds__(256) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ m, float* __restrict__ v, bf16_t* __restrict__ pb,
                                               int64_t n, double lr, double beta1, double beta2, double eps,
                                               double wd, const int64_t* __restrict__ step_ptr) {
    const AdamScalars s = adam_scalars(lr, beta1, beta2, eps, wd, step_ptr);
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    int64_t i = i0;
    if (VEC) {
        for (; i + (U - 1) * stride + 3 < n; i += U * stride) {
            float4 pv[U], gv[U], mv[U], vv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t j = i + u * stride;
                pv[u] = ld4<NT>(p + j);
                gv[u] = ld4<NT>(g + j);
                mv[u] = ld4<NT>(m + j);
                vv[u] = ld4<NT>(v + j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t j = i + u * stride;
                pv[u].x = adam_one(pv[u].x, gv[u].x, mv[u].x, vv[u].x, s);
                pv[u].y = adam_one(pv[u].y, gv[u].y, mv[u].y, vv[u].y, s);
                pv[u].z = adam_one(pv[u].z, gv[u].z, mv[u].z, vv[u].z, s);
                pv[u].w = adam_one(pv[u].w, gv[u].w, mv[u].w, vv[u].w, s);
                st4<NT>(p + j, pv[u]);
                st4<NT>(m + j, mv[u]);
                st4<NT>(v + j, vv[u]);
                if (pb) {
                    const uint2 w = make_uint2(pack_bf2(pv[u].x, pv[u].y), pack_bf2(pv[u].z, pv[u].w));
                    if constexpr (NT) __builtin_nontemporal_store(nu2{w.x, w.y}, (nu2*)(pb + j));
                    else *(uint2*)(pb + j) = w;
                }
            }
        }
    }
    for (; i < n; i += stride) {
        if (VEC && i + 3 < n) {
            float4 pv = ld4<NT>(p + i), gv = ld4<NT>(g + i), mv = ld4<NT>(m + i), vv = ld4<NT>(v + i);
            pv.x = adam_one(pv.x, gv.x, mv.x, vv.x, s);
            pv.y = adam_one(pv.y, gv.y, mv.y, vv.y, s);
            pv.z = adam_one(pv.z, gv.z, mv.z, vv.z, s);
            pv.w = adam_one(pv.w, gv.w, mv.w, vv.w, s);
            st4<NT>(p + i, pv);
            st4<NT>(m + i, mv);
            st4<NT>(v + i, vv);
            if (pb) *(uint2*)(pb + i) = make_uint2(pack_bf2(pv.x, pv.y), pack_bf2(pv.z, pv.w));
        } else {
            for (int64_t j = i; j < n && j < i + 4; ++j) {
                float mm = m[j], vv = v[j];
                const float np = adam_one(p[j], g[j], mm, vv, s);
                p[j] = np;
                m[j] = mm;
                v[j] = vv;
                if (pb) pb[j] = f2bf(np);
            }
        }
    }
}

namespace cg {
// cg_set_tuning("adamw_mode"): 0 automatic -- non-temporal loads/stores with two float4 groups per
// thread in flight once the 30 B/param stream is far past the 256 MB Infinity Cache (n >= 32 M: C4
// 86 M params, -2.4 % same-box interleaved A/B), plain loads/stores below (C2 10.8 M: the NT form is
// 16 % slower there, the gradients just written by the backward are still partly cache-resident);
// 1 plain, 2 NT + 2 groups, 3 plain + 2 groups (A/B: profiles/r3_adamw_ab.txt), 4 NT + 4 groups,
// 5 plain + 4 groups
int g_adamw_mode = 0;
}

static int adamw_launch(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, double lr,
                        double beta1, double beta2, double eps, double weight_decay, const int64_t* step_ptr,
                        void* stream) {
    CG_REQUIRE(n >= 0, "cg_adamw: n < 0");
    if (n == 0) return CG_OK;
    // the flat buffers are 16-B aligned; a single parameter's slice (torch-AdamW-style skipping of
    // grad-None parameters, optim.py) may not be: element-wise path
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 &&
                     (((uintptr_t)p_bf16) & 7) == 0;
    int grid = ceil_div((n + 3) / 4, 256);
    grid = grid > 8192 ? 8192 : grid;
    hipStream_t st = (hipStream_t)stream;
#define ADAMW(VEC_, NT_, U_)                                                                                \
    k_adamw<VEC_, NT_, U_><<<grid, 256, 0, st>>>(p, g, m, v, (bf16_t*)p_bf16, n, lr, beta1, beta2, eps, \
                                                 weight_decay, step_ptr)
    const int mode = g_adamw_mode ? g_adamw_mode : (n >= (int64_t)1 << 25 ? 2 : 1);
    if (!vec) ADAMW(false, false, 1);
    else if (mode == 2) ADAMW(true, true, 2);
    else if (mode == 3) ADAMW(true, false, 2);
    else if (mode == 4) ADAMW(true, true, 4);    // A/B: four groups in flight per thread
    else if (mode == 5) ADAMW(true, false, 4);
    else ADAMW(true, false, 1);
#undef ADAMW
    CG_LAUNCH_CHECK("cg_adamw");
    return CG_OK;
}

// AdamW over a list of flat segments (the training step's remaining parameters once its weight
// matrices were updated early by cg_adamw_defer jobs): float4 chunk c of the concatenation ->
// segment s by binary search over the chunk prefix counts; adam_one per element, so the bits of
// the one-launch form
constexpr int ADAM_MAX_SEGS = 64;
struct AdamSegs {
    int64_t start[ADAM_MAX_SEGS];      // element offsets (multiples of 4)
    int64_t pre[ADAM_MAX_SEGS + 1];    // float4 chunks before segment s
    int n;
};

__global__ __launch_bounds__(256) void k_adamw_segs(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16_t* __restrict__ pb, AdamSegs sg, double lr, double beta1,
                                                    double beta2, double eps, double wd,
                                                    const int64_t* __restrict__ step_ptr) {
    const AdamScalars s = adam_scalars(lr, beta1, beta2, eps, wd, step_ptr);
    const int64_t total = sg.pre[sg.n], stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total; c += stride) {
        int lo = 0, hi = sg.n - 1;
        while (lo < hi) {   // last segment with pre[seg] <= c
            const int mid = (lo + hi + 1) >> 1;
            if (sg.pre[mid] <= c) lo = mid;
            else hi = mid - 1;
        }
        const int64_t i = sg.start[lo] + 4 * (c - sg.pre[lo]);
        float4 pv = *(const float4*)(p + i);
        const float4 gv = *(const float4*)(g + i);
        float4 mv = *(const float4*)(m + i), vv = *(const float4*)(v + i);
        pv.x = adam_one(pv.x, gv.x, mv.x, vv.x, s);
        pv.y = adam_one(pv.y, gv.y, mv.y, vv.y, s);
        pv.z = adam_one(pv.z, gv.z, mv.z, vv.z, s);
        pv.w = adam_one(pv.w, gv.w, mv.w, vv.w, s);
        *(float4*)(p + i) = pv;
        *(float4*)(m + i) = mv;
        *(float4*)(v + i) = vv;
        if (pb) *(uint2*)(pb + i) = make_uint2(pack_bf2(pv.x, pv.y), pack_bf2(pv.z, pv.w));
    }
}

namespace cg {
int adamw_segments_launch(float* p, const float* g, float* m, float* v, bf16_t* pb, const int64_t* segs, int nseg,
                          double lr, double beta1, double beta2, double eps, double wd, const int64_t* step,
                          hipStream_t st);
}

extern "C" int cg_adamw_segments(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, const int64_t* segs,
                                 int nseg, double lr, double beta1, double beta2, double eps, double weight_decay,
                                 const int64_t* step_ptr, void* stream) {
    return cg::adamw_segments_launch(p, g, m, v, (bf16_t*)p_bf16, segs, nseg, lr, beta1, beta2, eps, weight_decay,
                                     step_ptr, (hipStream_t)stream);
}

int cg::adamw_segments_launch(float* p, const float* g, float* m, float* v, bf16_t* p_bf16, const int64_t* segs,
                              int nseg, double lr, double beta1, double beta2, double eps, double weight_decay,
                              const int64_t* step_ptr, hipStream_t stream) {
    CG_REQUIRE(p && g && m && v && segs && nseg >= 0 && nseg <= ADAM_MAX_SEGS,
               "cg_adamw_segments: bad arguments (at most %d segments)", ADAM_MAX_SEGS);
    CG_REQUIRE(((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                   (((uintptr_t)p_bf16) & 7) == 0,
               "cg_adamw_segments: p, g, m, v must be 16-B aligned, p_bf16 8-B aligned");
    AdamSegs sg = {};
    int k = 0;
    for (int q = 0; q < nseg; ++q) {
        const int64_t st = segs[2 * q], len = segs[2 * q + 1];
        CG_REQUIRE(st >= 0 && len >= 0 && st % 4 == 0 && len % 4 == 0,
                   "cg_adamw_segments: segment starts and lengths must be multiples of 4");
        if (!len) continue;
        sg.start[k] = st;
        sg.pre[k + 1] = sg.pre[k] + len / 4;
        ++k;
    }
    sg.n = k;
    if (!k) return CG_OK;
    int grid = ceil_div(sg.pre[k], 256);
    grid = grid > 8192 ? 8192 : grid;
    k_adamw_segs<<<grid, 256, 0, (hipStream_t)stream>>>(p, g, m, v, (bf16_t*)p_bf16, sg, lr, beta1, beta2, eps,
                                                        weight_decay, step_ptr);
    CG_LAUNCH_CHECK("cg_adamw_segments");
    return CG_OK;
}

namespace cg {
int adamw_job_launch(const AdamJob& j, hipStream_t st) {
    return adamw_launch(j.p, j.g, j.m, j.v, (uint16_t*)j.pb, 4 * j.n4, j.lr, j.beta1, j.beta2, j.eps, j.wd, j.step, st);
}
}  // namespace cg

extern "C" int cg_adamw(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, double lr,
                        double beta1, double beta2, double eps, double weight_decay, const int64_t* step_ptr,
                        void* stream) {
    return adamw_launch(p, g, m, v, p_bf16, n, lr, beta1, beta2, eps, weight_decay, step_ptr, stream);
}
