// charpt: token + position embeddings (GPT1.py:179-181) forward and deterministic backward.
#include "common.h"

using namespace cg;

// x[b,t,:] = wte[idx[b,t],:] + wpe[t,:]   -- one block per (b,t) row, coalesced over C
__global__ void k_embed_fwd(const int64_t* __restrict__ idx, const float* __restrict__ wte,
                            const float* __restrict__ wpe, float* __restrict__ x, int64_t T, int64_t C, int64_t V) {
    const int64_t row = blockIdx.x;
    const int64_t t = row % T;
    int64_t tok = idx[row];
    tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);  // out-of-range ids are a caller error (torch raises)
    const float* a = wte + tok * C;
    const float* p = wpe + t * C;
    float* o = x + row * C;
    if ((C & 3) == 0) {
        for (int64_t c = threadIdx.x * 4; c < C; c += blockDim.x * 4) {
            float4 u = *(const float4*)(a + c), w = *(const float4*)(p + c);
            *(float4*)(o + c) = make_float4(u.x + w.x, u.y + w.y, u.z + w.z, u.w + w.w);
        }
    } else {
        for (int64_t c = threadIdx.x; c < C; c += blockDim.x) o[c] = a[c] + p[c];
    }
}

// C % 4 == 0: 8 rows per 256-thread block, 32 lanes per row, each lane's NV float4 columns of wte
// and wpe loaded before any store (all of a row's loads in flight).  The one-row blocks above ran
// 16384 blocks of 96 active lanes at C2: 9.5 us for a 25 MB write.
template <int NV>
__global__ __launch_bounds__(256) void k_embed_fwd_rows(const int64_t* __restrict__ idx, const float* __restrict__ wte,
                                                        const float* __restrict__ wpe, float* __restrict__ x,
                                                        int64_t rows, int64_t T, int64_t C, int64_t V) {
    const int64_t row = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    const int l = threadIdx.x & 31;
    if (row >= rows) return;
    const int64_t t = row % T;
    int64_t tok = idx[row];
    tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);  // out-of-range ids are a caller error (torch raises)
    const float4* a = (const float4*)(wte + tok * C);
    const float4* p = (const float4*)(wpe + t * C);
    float4* o = (float4*)(x + row * C);
    const int c4 = (int)(C >> 2);
    float4 u[NV], w[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i)
        if (l + 32 * i < c4) {
            u[i] = a[l + 32 * i];
            w[i] = p[l + 32 * i];
        }
#pragma unroll
    for (int i = 0; i < NV; ++i)
        if (l + 32 * i < c4) o[l + 32 * i] = make_float4(u[i].x + w[i].x, u[i].y + w[i].y, u[i].z + w[i].z, u[i].w + w[i].w);
}

// Even C not a multiple of 4 (C1 / C5: C = 126, 8-B aligned rows): one float2 per thread over the flat
// output, so every wave stores 512 contiguous bytes.  The one-row blocks ran 65536 blocks of 126 active
// lanes for generate()'s window (22.6 us for a 33 MB write).
__global__ __launch_bounds__(256) void k_embed_fwd_pairs(const int64_t* __restrict__ idx, const float* __restrict__ wte,
                                                         const float* __restrict__ wpe, float* __restrict__ x,
                                                         int64_t n2, int64_t T, int64_t C, int64_t V) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n2) return;
    // 32-bit index arithmetic (the host keeps n2 < 2^31): a 64-bit division is a long software sequence
    const uint32_t c2 = (uint32_t)(C >> 1), rw = (uint32_t)j / c2;
    const int64_t row = rw, c = 2 * (int64_t)((uint32_t)j - rw * c2);
    const int64_t t = (int64_t)(rw % (uint32_t)T);
    int64_t tok = idx[row];
    tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);  // out-of-range ids are a caller error (torch raises)
    const float2 u = *(const float2*)(wte + tok * C + c), w = *(const float2*)(wpe + t * C + c);
    *(float2*)(x + row * C + c) = make_float2(u.x + w.x, u.y + w.y);
}

extern "C" int cg_embed_fwd(const int64_t* idx, const float* wte, const float* wpe, float* x, int64_t B, int64_t T,
                            int64_t C, int64_t V, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && C > 0 && V > 0, "cg_embed_fwd: bad shape");
    hipStream_t st = (hipStream_t)stream;
    const int64_t rows = B * T;
    const bool al16 = ((((uintptr_t)wte) | ((uintptr_t)wpe) | ((uintptr_t)x)) & 15) == 0;
    if (C % 4 == 0 && C <= 1024 && al16) {
        const unsigned grid = (unsigned)((rows + 7) / 8);
        switch ((int)((C / 4 + 31) / 32)) {
#define EF(NV_) \
    case NV_: k_embed_fwd_rows<NV_><<<grid, 256, 0, st>>>(idx, wte, wpe, x, rows, T, C, V); break;
            EF(1) EF(2) EF(3) EF(4) EF(5) EF(6) EF(7) EF(8)
#undef EF
            default: break;
        }
        CG_LAUNCH_CHECK("cg_embed_fwd");
        return CG_OK;
    }
    const bool al8 = ((((uintptr_t)wte) | ((uintptr_t)wpe) | ((uintptr_t)x)) & 7) == 0;
    if (C % 2 == 0 && al8 && rows * (C / 2) < ((int64_t)1 << 31)) {
        const int64_t n2 = rows * (C / 2);
        k_embed_fwd_pairs<<<(unsigned)((n2 + 255) / 256), 256, 0, st>>>(idx, wte, wpe, x, n2, T, C, V);
        CG_LAUNCH_CHECK("cg_embed_fwd");
        return CG_OK;
    }
    k_embed_fwd<<<(unsigned)(B * T), 128, 0, st>>>(idx, wte, wpe, x, T, C, V);
    CG_LAUNCH_CHECK("cg_embed_fwd");
    return CG_OK;
}

// ---- backward -------------------------------------------------------------------------
// dwpe[t,c] = sum_b dx[b,t,c]   (fixed b order).  4 columns per thread, 8 batch rows of loads in
// flight (the sum order is still b = 0, 1, 2, ...); 64-thread blocks so a T*C = 98K-element
// table still spreads over every CU.
__global__ __launch_bounds__(64) void k_embed_bwd_pos4(const float* __restrict__ dx, float* __restrict__ dwpe,
                                                     int64_t B, int64_t TC, int accumulate) {
    const int64_t i = ((int64_t)blockIdx.x * 64 + threadIdx.x) * 4;
    if (i >= TC) return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t b = 0;
    for (; b + 8 <= B; b += 8) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const float4*)(dx + (b + j) * TC + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s.x += v[j].x;
            s.y += v[j].y;
            s.z += v[j].z;
            s.w += v[j].w;
        }
    }
    for (; b < B; ++b) {
        const float4 v = *(const float4*)(dx + b * TC + i);
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
    }
    float4* o = (float4*)(dwpe + i);
    if (accumulate) {
        const float4 p = *o;
        s = make_float4(p.x + s.x, p.y + s.y, p.z + s.z, p.w + s.w);
    }
    *o = s;
}

__global__ void k_embed_bwd_pos(const float* __restrict__ dx, float* __restrict__ dwpe, int64_t B, int64_t T,
                                int64_t C, int accumulate) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T * C) return;
    float s = 0.f;
    for (int64_t b = 0; b < B; ++b) s += dx[b * T * C + i];
    dwpe[i] = accumulate ? dwpe[i] + s : s;
}

// per row-chunk partial histogram-sum: part[chunk][v][c] = sum_{rows in chunk, idx=v} dx[row][c].
// A block takes 64 columns of a 128-row chunk; its EMB_WAVES waves walk rows 128/W w .. of the chunk
// in order into their own LDS histograms (lane = column: deterministic, no atomics), which are then
// added in wave order.  4 waves (the 65-character vocabulary: 66.5 KB of histograms; the former
// 2-wave blocks walked twice the rows per lane, 20 us per C2 step against 14.6) while
// 4 V 64 4 B fits the LDS, then 2 (V <= 320) and 1 (V <= 640): fewer waves, same per-V bits for
// a given wave count.
constexpr int EMB_CHUNK = 128;
constexpr int EMB_COLS = 64;

template <int EMB_WAVES>
__global__ __launch_bounds__(64 * EMB_WAVES) void k_embed_bwd_tok_partial(const int64_t* __restrict__ idx,
                                                                          const float* __restrict__ dx,
                                                                          float* __restrict__ part, int64_t rows,
                                                                          int64_t C, int64_t V) {
    constexpr int EMB_RPW = EMB_CHUNK / EMB_WAVES;
    extern __shared__ __attribute__((aligned(16))) float acc[];  // [EMB_WAVES][V][EMB_COLS]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.x * EMB_COLS + lane;
    const int64_t chunk = blockIdx.y;
    float* my = acc + (int64_t)wave * V * EMB_COLS;
    for (int64_t v = 0; v < V; ++v) my[v * EMB_COLS + lane] = 0.f;
    const int64_t r0 = chunk * EMB_CHUNK + wave * EMB_RPW;
    const int64_t r1 = r0 + EMB_RPW < rows ? r0 + EMB_RPW : rows;
    if (c < C) {
        int64_t r = r0;
        for (; r + 8 <= r1; r += 8) {   // 8 rows of loads in flight; accumulation stays in row order
            int64_t tk[8];
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t t = idx[r + j];
                tk[j] = t < 0 ? 0 : (t >= V ? V - 1 : t);
                v[j] = dx[(r + j) * C + c];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) my[tk[j] * EMB_COLS + lane] += v[j];
        }
        for (; r < r1; ++r) {
            int64_t tok = idx[r];
            tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);
            my[tok * EMB_COLS + lane] += dx[r * C + c];
        }
    }
    __syncthreads();
    // the chunk's partial: ((w0 + w1) + w2) + w3 per (v, column), all threads over V x 64 entries
    const int64_t n = V * EMB_COLS;
    float* out = part + chunk * V * C;
    for (int64_t i = threadIdx.x; i < n; i += 64 * EMB_WAVES) {
        const int64_t v = i / EMB_COLS, cc = (int64_t)blockIdx.x * EMB_COLS + (i % EMB_COLS);
        if (cc < C) {
            float t = acc[i];
#pragma unroll
            for (int w = 1; w < EMB_WAVES; ++w) t += acc[(int64_t)w * n + i];
            out[v * C + cc] = t;
        }
    }
}

// Both gradients from one read of dx (the C2 step: B 64, T 256): block (column block, chunk) takes
// the TS = 128 / B positions t0 .. t0 + TS - 1 of every sequence -- wave w the sequences
// [w B / 4, (w + 1) B / 4), rows in (t, b) order -- into its LDS token histogram (as
// k_embed_bwd_tok_partial, the chunk's partial in wave order) and, per position, a register sum
// over its sequences; dwpe[t] = ((s0 + s1) + s2) + s3 over the waves.  Replaces the separate
// position kernel's second 25 MB read of dx.  Deterministic (fixed orders), not the separate
// kernels' bits.
template <int TS>
__global__ __launch_bounds__(256) void k_embed_bwd_fused(const int64_t* __restrict__ idx, const float* __restrict__ dx,
                                                         float* __restrict__ part, float* __restrict__ dwpe,
                                                         int64_t B, int64_t T, int64_t C, int64_t V, int accumulate) {
    extern __shared__ __attribute__((aligned(16))) float acc[];  // [4][V][EMB_COLS], then pos [4][TS][EMB_COLS]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t c = (int64_t)blockIdx.x * EMB_COLS + lane;
    const int64_t chunk = blockIdx.y, t0 = chunk * TS;
    float* my = acc + (int64_t)wave * V * EMB_COLS;
    float* pos = acc + 4 * V * EMB_COLS;
    for (int64_t v = 0; v < V; ++v) my[v * EMB_COLS + lane] = 0.f;
    const int64_t nb = B / 4, b0 = wave * nb;
    if (c < C) {
#pragma unroll
        for (int ti = 0; ti < TS; ++ti) {
            const int64_t t = t0 + ti;
            float ps = 0.f;
            int64_t b = b0;
            for (; b + 8 <= b0 + nb; b += 8) {   // 8 rows of loads in flight; sums stay in b order
                int64_t tk[8];
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int64_t r = (b + j) * T + t;
                    const int64_t tt = idx[r];
                    tk[j] = tt < 0 ? 0 : (tt >= V ? V - 1 : tt);
                    v[j] = dx[r * C + c];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    my[tk[j] * EMB_COLS + lane] += v[j];
                    ps += v[j];
                }
            }
            for (; b < b0 + nb; ++b) {
                const int64_t r = b * T + t;
                int64_t tok = idx[r];
                tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);
                const float v = dx[r * C + c];
                my[tok * EMB_COLS + lane] += v;
                ps += v;
            }
            pos[(wave * TS + ti) * EMB_COLS + lane] = ps;
        }
    }
    __syncthreads();
    const int64_t n = V * EMB_COLS;
    float* out = part + chunk * V * C;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const int64_t v = i / EMB_COLS, cc = (int64_t)blockIdx.x * EMB_COLS + (i % EMB_COLS);
        if (cc < C) out[v * C + cc] = ((acc[i] + acc[n + i]) + acc[2 * n + i]) + acc[3 * n + i];
    }
    for (int i = threadIdx.x; i < TS * EMB_COLS; i += 256) {
        const int ti = i / EMB_COLS, l = i % EMB_COLS;
        const int64_t cc = (int64_t)blockIdx.x * EMB_COLS + l;
        if (cc < C) {
            const float s = ((pos[ti * EMB_COLS + l] + pos[(TS + ti) * EMB_COLS + l]) + pos[(2 * TS + ti) * EMB_COLS + l]) +
                            pos[(3 * TS + ti) * EMB_COLS + l];
            float* o = dwpe + (t0 + ti) * C + cc;
            *o = accumulate ? *o + s : s;
        }
    }
}

__global__ void k_embed_bwd_tok_reduce(const float* __restrict__ part, float* __restrict__ dwte, int64_t nchunk,
                                       int64_t VC, int accumulate) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= VC) return;
    float s = 0.f;
    int64_t k = 0;
    for (; k + 8 <= nchunk; k += 8) {   // 8 partials in flight, summed in chunk order
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = part[(k + j) * VC + i];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < nchunk; ++k) s += part[k * VC + i];
    dwte[i] = accumulate ? dwte[i] + s : s;
}

extern "C" int64_t cg_embed_bwd_workspace(int64_t B, int64_t T, int64_t C, int64_t V) {
    int64_t nchunk = (B * T + EMB_CHUNK - 1) / EMB_CHUNK;
    return nchunk * V * C * (int64_t)sizeof(float);
}

extern "C" int cg_embed_bwd(const int64_t* idx, const float* dx, float* dwte, float* dwpe, int64_t B, int64_t T,
                            int64_t C, int64_t V, int accumulate, void* workspace, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && C > 0 && V > 0, "cg_embed_bwd: bad shape");
    CG_REQUIRE(V * EMB_COLS * 4 <= 160 * 1024, "cg_embed_bwd: vocab %lld too large for the LDS histogram",
               (long long)V);
    const int waves = 4 * V * EMB_COLS * 4 <= 160 * 1024 ? 4 : (2 * V * EMB_COLS * 4 <= 160 * 1024 ? 2 : 1);
    hipStream_t st = (hipStream_t)stream;
    const int64_t rows = B * T;
    // both gradients, one accumulate flag, a 4-wave histogram and B a divisor or multiple of 128
    // (TS = 128 / B positions per chunk -- the same chunk count as the row chunks): the fused kernel
    const int64_t ts = B >= 128 ? 1 : 128 / B;
    const bool fused = dwte && dwpe && waves == 4 && B % 4 == 0 && (B >= 128 ? B % 128 == 0 : 128 % B == 0) &&
                       T % ts == 0 && (ts == 1 || ts == 2 || ts == 4 || ts == 8) &&
                       (4 * V + 4 * ts) * EMB_COLS * 4 <= 160 * 1024;
    if (fused) {
        const int64_t nchunk = T / ts;
        dim3 grid(ceil_div(C, EMB_COLS), (unsigned)nchunk);
        const size_t lds = (size_t)(4 * V + 4 * ts) * EMB_COLS * sizeof(float);
#define EBF(TS_) k_embed_bwd_fused<TS_><<<grid, 256, lds, st>>>(idx, dx, (float*)workspace, dwpe, B, T, C, V, accumulate)
        if (ts == 1) EBF(1);
        else if (ts == 2) EBF(2);
        else if (ts == 4) EBF(4);
        else EBF(8);
#undef EBF
        k_embed_bwd_tok_reduce<<<ceil_div(V * C, 64), 64, 0, st>>>((const float*)workspace, dwte, nchunk, V * C,
                                                                    accumulate);
        CG_LAUNCH_CHECK("cg_embed_bwd");
        return CG_OK;
    }
    if (dwpe) {
        if ((T * C) % 4 == 0 && ((((uintptr_t)dx) | ((uintptr_t)dwpe)) & 15) == 0)
            k_embed_bwd_pos4<<<ceil_div(T * C / 4, 64), 64, 0, st>>>(dx, dwpe, B, T * C, accumulate);
        else
            k_embed_bwd_pos<<<ceil_div(T * C, 256), 256, 0, st>>>(dx, dwpe, B, T, C, accumulate);
    }
    if (dwte) {
        const int64_t nchunk = (rows + EMB_CHUNK - 1) / EMB_CHUNK;
        dim3 grid(ceil_div(C, EMB_COLS), (unsigned)nchunk);
        const size_t lds = (size_t)waves * V * EMB_COLS * sizeof(float);
        if (waves == 4)
            k_embed_bwd_tok_partial<4><<<grid, 256, lds, st>>>(idx, dx, (float*)workspace, rows, C, V);
        else if (waves == 2)
            k_embed_bwd_tok_partial<2><<<grid, 128, lds, st>>>(idx, dx, (float*)workspace, rows, C, V);
        else
            k_embed_bwd_tok_partial<1><<<grid, 64, lds, st>>>(idx, dx, (float*)workspace, rows, C, V);
        k_embed_bwd_tok_reduce<<<ceil_div(V * C, 64), 64, 0, st>>>((const float*)workspace, dwte, nchunk, V * C,
                                                                    accumulate);
    }
    CG_LAUNCH_CHECK("cg_embed_bwd");
    return CG_OK;
}
