// charpt: batched autoregressive decode kernels for generate() (GPT1.py:196-212).
//
// The reference crops the context to the last block_size tokens and re-runs the full forward
// every step (positions are re-indexed from 0 after the crop, so once the window slides no K/V can
// be reused -- SURVEY Q7).  The decode engine (replicatinggpt_amd/decode.py) therefore runs
//   phase 1 (length <= block_size): one new token per step against a per-layer K/V cache
//            (cg_decode_kv_append + cg_decode_attn), positions identical to the full recompute;
//   phase 2 (sliding window): the full window forward (cg_decode_window gathers it), last row only
//            through ln_f / lm_head;
// and samples on the device (cg_decode_sample: argmax, or inverse-CDF sampling from a Philox
// stream).  Every step's shapes are static and the current length lives in device memory, so each
// phase is captured once as a hipGraph and replayed per token.
#include "common.h"

namespace cg {
int g_decode_attn_rows = 1;   // cg_set_tuning("decode_attn_rows"): 0 = k_decode_attn for every layout (A/B, tests)
}
namespace {
using namespace cg;

// out[b, j] = idx[b, start + j], start = max(0, len - T)  (len = *len_dev; idx row stride ld)
__global__ void k_decode_window(const int64_t* __restrict__ idx, int64_t ld, int64_t B, int64_t T,
                                const int64_t* __restrict__ len_dev, int64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * T) return;
    const int64_t b = i / T, j = i % T;
    const int64_t len = *len_dev;
    const int64_t start = len > T ? len - T : 0;
    out[i] = start + j < ld ? idx[b * ld + start + j] : 0;   // rows shorter than T: zero padding
}

// x[b, :] = wte[idx[b, pos]] + wpe[pos]   (pos = *len_dev - 1: the newest token)
__global__ void k_decode_embed(const int64_t* __restrict__ idx, int64_t ld, const float* __restrict__ wte,
                               const float* __restrict__ wpe, int64_t C, const int64_t* __restrict__ len_dev,
                               float* __restrict__ x, int64_t B) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * C) return;
    const int64_t b = i / C, c = i % C;
    const int64_t pos = *len_dev - 1;
    x[i] = wte[idx[b * ld + pos] * C + c] + wpe[pos * C + c];
}

// K/V cache [B, H, Tmax, D]: row pos = *len_dev - 1 from the qkv rows (k at k_off, v at v_off)
__global__ void k_decode_kv_append(const float* __restrict__ qkv, int64_t ld, int64_t k_off, int64_t v_off,
                                   int64_t B, int64_t H, int64_t D, int64_t Tmax,
                                   const int64_t* __restrict__ len_dev, float* __restrict__ kc,
                                   float* __restrict__ vc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * H * D) return;
    const int64_t b = i / (H * D), r = i % (H * D), h = r / D, e = r % D;
    const int64_t pos = *len_dev - 1;
    const int64_t dst = ((b * H + h) * Tmax + pos) * D + e;
    kc[dst] = qkv[b * ld + k_off + h * D + e];
    vc[dst] = qkv[b * ld + v_off + h * D + e];
}

// one wave per (b, h): the newest query against cached keys 0..n-1 (causal by construction),
// scale = n_embd^-0.5.  Keys are spread over the lanes -- chunk c holds key 64 c + lane
// -- and each lane keeps its key's whole dot product and its own partial output row acc[0..D) (D
// padded to DP at compile time): a chunk's softmax statistics are two wave reductions (online over
// chunks), every K / V element load of a chunk is independent, and the output row is one DPP wave
// sum per dimension at the end.  (The previous form put 4 lanes on a key and accumulated V with a
// serial 16-step __shfl + dependent-load loop per chunk, and its vector loads needed D == 64: 73 us
// per call for the C5 model's head size 21, 10 % of generate().)
// K/V element (b, h, key j, e) at base + b*sb + h*sh + j*sj + e: the [B, H, Tmax, D] cache
// (sb = H*Tmax*D, sh = Tmax*D, sj = D) or the rows of a window's qkv buffer (sb = T*ld, sh = D, sj = ld).
template <int DP>
__global__ __launch_bounds__(256) void k_decode_attn(const float* __restrict__ q, int64_t ldq,
                                                     const float* __restrict__ kc, const float* __restrict__ vc,
                                                     int64_t sb, int64_t sh, int64_t sj, int64_t B, int64_t H,
                                                     int64_t D, const int64_t* __restrict__ len_dev, int64_t nfix,
                                                     float scale, float* __restrict__ o, int64_t ldo) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t bh = (int64_t)blockIdx.x * 4 + w;
    if (bh >= B * H) return;
    const int64_t b = bh / H, h = bh % H;
    const int64_t n = len_dev ? *len_dev : nfix;  // keys 0..n-1
    const float* K = kc + b * sb + h * sh;
    const float* V = vc + b * sb + h * sh;
    float qv[DP], acc[DP];
#pragma unroll
    for (int e = 0; e < DP; ++e) {
        qv[e] = e < D ? q[b * ldq + h * D + e] : 0.f;
        acc[e] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int64_t c0 = 0; c0 < n; c0 += 64) {
        const int64_t j = c0 + lane;
        const bool ok = j < n;
        const float* kr = K + (ok ? j : 0) * sj;
        const float* vr = V + (ok ? j : 0) * sj;
        float kv[DP], vv[DP];
#pragma unroll
        for (int e = 0; e < DP; ++e) {   // every load of the chunk in flight together
            kv[e] = e < D ? kr[e] : 0.f;
            vv[e] = e < D ? vr[e] : 0.f;
        }
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < DP; ++e) s = fmaf(qv[e], kv[e], s);
        s = ok ? s * scale : -INFINITY;
        const float m_new = fmaxf(m, wave_max(s));
        const float alpha = __expf(m - m_new);
        const float p = ok ? __expf(s - m_new) : 0.f;
        l = l * alpha + wave_sum(p);
        m = m_new;
#pragma unroll
        for (int e = 0; e < DP; ++e) acc[e] = fmaf(p, vv[e], acc[e] * alpha);
    }
    const float inv = 1.f / l;
    float out = 0.f;
#pragma unroll
    for (int e = 0; e < DP; ++e) {
        if (e < D) {   // wave-uniform
            const float t = wave_sum_dpp(acc[e]);
            out = lane == e ? t * inv : out;
        }
    }
    if (lane < D) o[b * ldo + h * D + lane] = out;
}

// k_decode_attn for the phase-1 cache ([B, H, Tmax, D], key rows contiguous, 16-B aligned chunks): one
// 64-thread block per (b, h).  A lane-per-key load reads one float of each of 64 rows per instruction --
// D instructions per chunk and operand, each touching ~D/1.5 cache lines -- and the rows of 6 waves a CU
// holds do not stay in its L1 between those instructions: the kernel ran at 1.4 TB/s of K / V at 256 keys
// and its time grew with the line count per instruction (row stride 32 floats: 0.75 TB/s;
// tools/decode_attn_probe.py).  Here a chunk's 64 K and V rows (64 D contiguous floats each) are read as
// float4s, lane l taking float4 l + 64 r, the next chunk's loads issued before the current chunk's
// arithmetic, and staged through LDS so that each lane then reads its key's row (stride D: conflict-free
// for odd D).  Per lane the arithmetic is k_decode_attn's, value for value (a lane past the last key
// reads zero rows instead of key 0's: its p is 0 either way), so the output is bitwise the same.
// SJ: key rows sj floats apart (phase 2's last layer: the window's qkv rows, sj = 3 C) -- the chunk's
// floats read as dwords, lane l taking float l + 64 r of the chunk's 64 D (row (l + 64 r) / D), so an
// instruction spans ~64 / D rows instead of 64.
template <int DP, bool SJ = false>
__global__ __launch_bounds__(64) void k_decode_attn_rows(const float* __restrict__ q, int64_t ldq,
                                                         const float* __restrict__ kc, const float* __restrict__ vc,
                                                         int64_t sb, int64_t sh, int64_t sj, int64_t B, int64_t H,
                                                         int64_t D,
                                                         const int64_t* __restrict__ len_dev, int64_t nfix, float scale,
                                                         float* __restrict__ o, int64_t ldo) {
    constexpr int R4 = DP;   // float4s per lane per operand: 64 rows x DP floats / 4 / 64 lanes
    __shared__ float4 ks4[16 * DP], vs4[16 * DP];
    const float* ks = (const float*)ks4;
    const float* vs = (const float*)vs4;
    const int lane = threadIdx.x;
    // XCD-contiguous (b, h) (block i runs on XCD i % 8): a sequence's heads share one L2 -- with the
    // window's row-strided K / V (SJ) each head reads 84 B of every 1 KB row
    const int nblk = (int)gridDim.x, id = (int)blockIdx.x, nq = nblk >> 3, nr = nblk & 7, xcd = id & 7;
    const int64_t bh = (xcd < nr ? xcd * (nq + 1) : nr * (nq + 1) + (xcd - nr) * nq) + (id >> 3);
    const int64_t b = bh / H, h = bh % H;
    const int64_t n = len_dev ? *len_dev : nfix;  // keys 0..n-1
    const float4* K4 = (const float4*)(kc + b * sb + h * sh);
    const float4* V4 = (const float4*)(vc + b * sb + h * sh);
    const int64_t f4 = 16 * D;   // float4s per 64-row chunk
    float qv[DP], acc[DP];
#pragma unroll
    for (int e = 0; e < DP; ++e) {
        qv[e] = e < D ? q[b * ldq + h * D + e] : 0.f;
        acc[e] = 0.f;
    }
    float4 kr[R4 / 4], vr[R4 / 4];
    float kr1[SJ ? DP : 1], vr1[SJ ? DP : 1];
    const float* Kb = kc + b * sb + h * sh;
    const float* Vb = vc + b * sb + h * sh;
    int off[SJ ? DP : 1];   // SJ: float l + 64 r of a chunk at row * sj + e (INT_MAX: past the chunk)
    if constexpr (SJ) {
        int row = lane / (int)D, e = lane - row * (int)D;
        const int drow = 64 / (int)D, de = 64 - drow * (int)D;
#pragma unroll
        for (int r = 0; r < DP; ++r) {
            off[r] = lane + 64 * r < 64 * D ? row * (int)sj + e : INT_MAX;
            row += drow;
            e += de;
            if (e >= D) e -= (int)D, ++row;
        }
    }
    auto load = [&](int64_t c0) {
        if constexpr (SJ) {
            const int64_t rows = n - c0 < 64 ? n - c0 : 64;
            const int lim = (int)(rows * sj);   // offsets of the chunk's keys (e < D <= sj)
            const float* kb = Kb + c0 * sj;
            const float* vb = Vb + c0 * sj;
#pragma unroll
            for (int r = 0; r < DP; ++r) {
                const bool in = off[r] < lim;
                kr1[r] = in ? kb[off[r]] : 0.f;
                vr1[r] = in ? vb[off[r]] : 0.f;
            }
            return;
        }
        const int64_t lim = ((n - c0 < 64 ? n - c0 : 64) * D + 3) / 4;   // float4s holding the chunk's keys
#pragma unroll
        for (int r = 0; r < R4 / 4; ++r) {
            const int64_t i = lane + 64 * r;
            const bool in = i < f4 && i < lim;
            kr[r] = in ? K4[c0 / 4 * D + i] : float4{0.f, 0.f, 0.f, 0.f};
            vr[r] = in ? V4[c0 / 4 * D + i] : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    float m = -INFINITY, l = 0.f;
    load(0);
    for (int64_t c0 = 0; c0 < n; c0 += 64) {
        const int64_t cnt = (n - c0 < 64 ? n - c0 : 64) * D;   // floats of the chunk's keys
        __syncthreads();   // the previous chunk's rows are read (one wave: no wait for other waves)
        if constexpr (SJ) {
#pragma unroll
            for (int r = 0; r < DP; ++r) {
                const int64_t i = lane + 64 * r;
                if (i < 64 * D) {
                    ((float*)ks4)[i] = kr1[r];
                    ((float*)vs4)[i] = vr1[r];
                }
            }
        }
#pragma unroll
        for (int r = 0; r < (SJ ? 0 : R4 / 4); ++r) {
            const int64_t i = lane + 64 * r;
            if (i < f4) {
                float4 kx = kr[r], vx = vr[r];
                // a float4 straddling the last key: floats past it zero (key 0's floats in k_decode_attn
                // never reach a valid lane's row either way)
                const int64_t f = 4 * i;
                if (f + 4 > cnt) {
                    if (f + 0 >= cnt) kx.x = vx.x = 0.f;
                    if (f + 1 >= cnt) kx.y = vx.y = 0.f;
                    if (f + 2 >= cnt) kx.z = vx.z = 0.f;
                    if (f + 3 >= cnt) kx.w = vx.w = 0.f;
                }
                ks4[i] = kx;
                vs4[i] = vx;
            }
        }
        __syncthreads();
        if (c0 + 64 < n) load(c0 + 64);
        const int64_t j = c0 + lane;
        const bool ok = j < n;
        float kv[DP], vv[DP];
#pragma unroll
        for (int e = 0; e < DP; ++e) {
            kv[e] = e < D ? ks[lane * D + e] : 0.f;
            vv[e] = e < D ? vs[lane * D + e] : 0.f;
        }
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < DP; ++e) s = fmaf(qv[e], kv[e], s);
        s = ok ? s * scale : -INFINITY;
        const float m_new = fmaxf(m, wave_max(s));
        const float alpha = __expf(m - m_new);
        const float p = ok ? __expf(s - m_new) : 0.f;
        l = l * alpha + wave_sum(p);
        m = m_new;
#pragma unroll
        for (int e = 0; e < DP; ++e) acc[e] = fmaf(p, vv[e], acc[e] * alpha);
    }
    const float inv = 1.f / l;
    float out = 0.f;
#pragma unroll
    for (int e = 0; e < DP; ++e) {
        if (e < D) {   // wave-uniform
            const float t = wave_sum_dpp(acc[e]);
            out = lane == e ? t * inv : out;
        }
    }
    if (lane < D) o[b * ldo + h * D + lane] = out;
}

// next token per row from logits [B, V]: greedy = first argmax (torch.argmax tie rule); else
// inverse-CDF sampling of softmax(logits) with u = Philox(seed, stream = step)[b] / 2^32.
// Writes idx[b, len] (len = *len_dev) -- the caller then advances *len_dev.
__global__ __launch_bounds__(64) void k_decode_sample(const float* __restrict__ logits, int64_t ldl, int64_t V,
                                                      int64_t B, int greedy, const uint64_t* __restrict__ seed_dev,
                                                      const int64_t* __restrict__ len_dev,
                                                      int64_t* __restrict__ idx, int64_t ld) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int lane = threadIdx.x;
    const float* row = logits + b * ldl;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = lane; v < V; v += 64) {
        const float x = row[v];
        if (x > best || (x == best && v < bi)) { best = x; bi = v; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float ob = __shfl_xor(best, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    const int64_t len = *len_dev;
    int64_t tok = bi;
    if (!greedy) {
        float s = 0.f;
        for (int v = lane; v < V; v += 64) s += __expf(row[v] - best);
        s = wave_sum(s);
        const u32x4 r = philox_group(seed_dev ? *seed_dev : 0ull, (uint64_t)len, (uint64_t)b);
        const float u = (float)(r.x >> 8) * (1.0f / 16777216.0f) * s;  // 24-bit uniform in [0, s)
        // sequential inverse CDF in vocabulary order (lane 0; V is the 65-char vocabulary)
        if (lane == 0) {
            float c = 0.f;
            tok = V - 1;
            for (int v = 0; v < V; ++v) {
                c += __expf(row[v] - best);
                if (u < c) { tok = v; break; }
            }
        }
    }
    if (lane == 0) idx[b * ld + len] = tok;
}

}  // namespace

extern "C" int cg_decode_window(const int64_t* idx, int64_t ld, int64_t B, int64_t T, const int64_t* len_dev,
                                int64_t* out, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && ld > 0, "cg_decode_window: bad sizes");
    k_decode_window<<<ceil_div(B * T, 256), 256, 0, (hipStream_t)stream>>>(idx, ld, B, T, len_dev, out);
    CG_LAUNCH_CHECK("cg_decode_window");
    return CG_OK;
}

extern "C" int cg_decode_embed(const int64_t* idx, int64_t ld, const float* wte, const float* wpe, int64_t C,
                               const int64_t* len_dev, float* x, int64_t B, void* stream) {
    CG_REQUIRE(B > 0 && C > 0, "cg_decode_embed: bad sizes");
    k_decode_embed<<<ceil_div(B * C, 256), 256, 0, (hipStream_t)stream>>>(idx, ld, wte, wpe, C, len_dev, x, B);
    CG_LAUNCH_CHECK("cg_decode_embed");
    return CG_OK;
}

extern "C" int cg_decode_kv_append(const float* qkv, int64_t ld, int64_t k_off, int64_t v_off, int64_t B, int64_t H,
                                   int64_t D, int64_t Tmax, const int64_t* len_dev, float* kcache, float* vcache,
                                   void* stream) {
    CG_REQUIRE(B > 0 && H > 0 && D > 0 && Tmax > 0, "cg_decode_kv_append: bad sizes");
    k_decode_kv_append<<<ceil_div(B * H * D, 256), 256, 0, (hipStream_t)stream>>>(qkv, ld, k_off, v_off, B, H, D,
                                                                                  Tmax, len_dev, kcache, vcache);
    CG_LAUNCH_CHECK("cg_decode_kv_append");
    return CG_OK;
}

extern "C" int cg_decode_attn(const float* q, int64_t ldq, const float* k, const float* v, int64_t sb, int64_t sh,
                              int64_t sj, int64_t B, int64_t H, int64_t D, const int64_t* len_dev, int64_t nkeys,
                              float scale, float* o, int64_t ldo, void* stream) {
    CG_REQUIRE(B > 0 && H > 0 && D > 0 && D <= 64, "cg_decode_attn: needs D <= 64");
    CG_REQUIRE(len_dev || nkeys > 0, "cg_decode_attn: needs at least one key");
    // contiguous, 16-B aligned key rows (the phase-1 cache): the coalesced-chunk kernel
    const bool rows = g_decode_attn_rows && D <= 24 && sj == D && sh % 4 == 0 && sb % 4 == 0 &&
                      ((uintptr_t)k & 15) == 0 && ((uintptr_t)v & 15) == 0;
    if (rows)
        k_decode_attn_rows<24><<<(unsigned)(B * H), 64, 0, (hipStream_t)stream>>>(q, ldq, k, v, sb, sh, sj, B, H, D,
                                                                                  len_dev, nkeys, scale, o, ldo);
    else if (g_decode_attn_rows && D <= 24 && sj >= D && sj < (1 << 24))   // key rows sj floats apart (a window's qkv rows)
        k_decode_attn_rows<24, true><<<(unsigned)(B * H), 64, 0, (hipStream_t)stream>>>(
            q, ldq, k, v, sb, sh, sj, B, H, D, len_dev, nkeys, scale, o, ldo);
    else if (D <= 24)
        k_decode_attn<24><<<ceil_div(B * H, 4), 256, 0, (hipStream_t)stream>>>(q, ldq, k, v, sb, sh, sj, B, H, D,
                                                                               len_dev, nkeys, scale, o, ldo);
    else
        k_decode_attn<64><<<ceil_div(B * H, 4), 256, 0, (hipStream_t)stream>>>(q, ldq, k, v, sb, sh, sj, B, H, D,
                                                                               len_dev, nkeys, scale, o, ldo);
    CG_LAUNCH_CHECK("cg_decode_attn");
    return CG_OK;
}

extern "C" int cg_decode_sample(const float* logits, int64_t ldl, int64_t V, int64_t B, int greedy,
                                const uint64_t* seed_dev, const int64_t* len_dev, int64_t* idx, int64_t ld,
                                void* stream) {
    CG_REQUIRE(B > 0 && V > 0, "cg_decode_sample: bad sizes");
    k_decode_sample<<<(unsigned)B, 64, 0, (hipStream_t)stream>>>(logits, ldl, V, B, greedy, seed_dev, len_dev, idx,
                                                                 ld);
    CG_LAUNCH_CHECK("cg_decode_sample");
    return CG_OK;
}
