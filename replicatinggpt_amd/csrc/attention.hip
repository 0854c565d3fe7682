// charpt: fused causal self-attention over all heads -- Head.forward (GPT1.py:109-123) run for
// every head of MultiHeadAttention (GPT1.py:134-135) without materialising the T x T scores.
//
//   S = q k^T * scale (scale = n_embd^-0.5); S[j > i] = -inf (tril, GPT1.py:115);
//   P = softmax(S) (GPT1.py:116); P = dropout(P) (GPT1.py:117); out = P v (GPT1.py:122).
//
// Online softmax, logsumexp saved for the backward, dropout regenerated from the Philox
// counter (element idx = ((b*H + h)*T + i)*T + j).  Backward = FlashAttention-2 style
// recompute split in two deterministic kernels (dK/dV per key block, dQ per query block), so no
// float atomics are needed.
//
// Kernels:
//   *_generic : fp32 math, any head size D <= 128 and any T; the fp32 parity path and the
//               as-shipped head_size 21.  32x32 blocks, VALU dot products.
//   *_d64     : bf16 MFMA (16x16x32), D = 64, T % 64 == 0 -- the C2/C4 perf path.
#include <math.h>

#include "common.h"

using namespace cg;

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct DropArgs {
    uint32_t thr;
    float dscale;
    uint64_t seed;
    const uint64_t* rng_call;
    int site;
    const uint64_t* mask;  // fast kernels: precomputed keep bits (k_attn_dropmask), NULL = no dropout
};

// Keep-bit image for the MFMA kernels, per (b*H + h) and 16x16 (query tile, key tile):
// 4 uint64 words, bit l of word w = keep(query = 16*qt + (l & 15), key = 16*kt + 4*(l >> 4) + w).
// Generated once per forward from the canonical Philox stream (same bits as keep_elem), read by
// the forward, dQ and dK/dV kernels instead of re-running Philox in their inner loops.
__device__ __forceinline__ const uint64_t* mask_tile(const uint64_t* mask, int bh, int NT, int qt, int kt) {
    return mask + ((((int64_t)bh * NT + qt) * NT + kt) << 2);
}

__global__ __launch_bounds__(256) void k_attn_dropmask(int64_t T_, uint64_t* __restrict__ mask, DropArgs d) {
    const int NT = (int)(T_ >> 4);
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= NT * NT) return;
    const int qt = tile / NT, kt = tile % NT;
    if (kt > qt) return;  // strictly above the diagonal: fully causal-masked, never read
    const int lane = threadIdx.x & 63;
    const uint64_t bh = blockIdx.y;
    const uint64_t stream = dropout_stream(d.rng_call, d.site);
    const uint64_t q = (uint64_t)qt * 16 + (lane & 15), key0 = (uint64_t)kt * 16 + 4 * (lane >> 4);
    const u32x4 r = philox_group(d.seed, stream, ((bh * T_ + q) * T_ + key0) >> 2);
    const uint64_t b0 = __ballot(r.x >= d.thr), b1 = __ballot(r.y >= d.thr);
    const uint64_t b2 = __ballot(r.z >= d.thr), b3 = __ballot(r.w >= d.thr);
    if (lane == 0) {
        uint64_t* o = mask + (((bh * NT + qt) * NT + kt) << 2);
        o[0] = b0;
        o[1] = b1;
        o[2] = b2;
        o[3] = b3;
    }
}

__device__ __forceinline__ bool keep_elem(const DropArgs& d, uint64_t stream, uint64_t idx) {
    const u32x4 r = philox_group(d.seed, stream, idx >> 2);
    return philox_word(r, (int)(idx & 3)) >= d.thr;
}

// =====================================================================================
// generic fp32 kernels
// =====================================================================================
constexpr int GB = 32;  // rows per block (queries or keys)

template <typename T>
__device__ __forceinline__ void load_rows(float* dst, int DP, const T* base, int64_t ld, int64_t row0, int64_t T_,
                                          int D, int tid) {
    for (int i = tid; i < GB * D; i += 256) {
        const int r = i / D, e = i % D;
        const int64_t t = row0 + r;
        dst[r * DP + e] = t < T_ ? ld_as_f32<T>(base + t * ld + e) : 0.f;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_attn_fwd_generic(int64_t T_, int H, int D, const T* __restrict__ q,
                                                          const T* __restrict__ k, const T* __restrict__ v, int64_t ld,
                                                          T* __restrict__ o, int64_t ldo, float* __restrict__ lse,
                                                          float scale, DropArgs drop) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int DP = D + 1;
    float* Qs = sm;
    float* Ks = Qs + GB * DP;
    float* Vs = Ks + GB * DP;
    float* Ps = Vs + GB * DP;  // [GB][GB+1]
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int qb = blockIdx.x;
    const int64_t q0 = (int64_t)qb * GB;
    const int tid = threadIdx.x, qi = tid >> 3, sub = tid & 7;
    const int64_t qa = q0 + qi;
    const T* qbase = q + (int64_t)b * T_ * ld + h * D;
    const T* kbase = k + (int64_t)b * T_ * ld + h * D;
    const T* vbase = v + (int64_t)b * T_ * ld + h * D;
    load_rows<T>(Qs, DP, qbase, ld, q0, T_, D, tid);
    const uint64_t stream = drop.thr ? dropout_stream(drop.rng_call, drop.site) : 0;
    float m_run = -INFINITY, l_run = 0.f;
    float oacc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) oacc[j] = 0.f;
    for (int kb = 0; kb <= qb; ++kb) {
        const int64_t k0 = (int64_t)kb * GB;
        __syncthreads();
        load_rows<T>(Ks, DP, kbase, ld, k0, T_, D, tid);
        load_rows<T>(Vs, DP, vbase, ld, k0, T_, D, tid);
        __syncthreads();
        float s[4], mx = -INFINITY;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = sub + 8 * jj;
            const int64_t key = k0 + j;
            float acc = 0.f;
            for (int e = 0; e < D; ++e) acc += Qs[qi * DP + e] * Ks[j * DP + e];
            acc *= scale;
            if (key > qa || key >= T_) acc = -INFINITY;
            s[jj] = acc;
            mx = fmaxf(mx, acc);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
        const float m_new = fmaxf(m_run, mx);
        const float alpha = m_new == -INFINITY ? 1.f : expf(m_run - m_new);
        float psum = 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = sub + 8 * jj;
            const float p = s[jj] == -INFINITY ? 0.f : expf(s[jj] - m_new);
            psum += p;
            float pd = p;
            if (drop.thr && p != 0.f) {
                const uint64_t idx = (((uint64_t)bh * T_ + qa) * T_ + (k0 + j));
                pd = keep_elem(drop, stream, idx) ? p * drop.dscale : 0.f;
            }
            Ps[qi * (GB + 1) + j] = pd;
        }
        psum += __shfl_xor(psum, 1, 64);
        psum += __shfl_xor(psum, 2, 64);
        psum += __shfl_xor(psum, 4, 64);
        l_run = l_run * alpha + psum;
        m_run = m_new;
        __syncthreads();
#pragma unroll
        for (int j8 = 0; j8 < 16; ++j8) {
            const int e = sub + 8 * j8;
            if (e < D) {
                float a = oacc[j8] * alpha;
                for (int j = 0; j < GB; ++j) a += Ps[qi * (GB + 1) + j] * Vs[j * DP + e];
                oacc[j8] = a;
            }
        }
    }
    if (qa < T_) {
        const float inv = 1.f / l_run;
        T* orow = o + ((int64_t)b * T_ + qa) * ldo + h * D;
#pragma unroll
        for (int j8 = 0; j8 < 16; ++j8) {
            const int e = sub + 8 * j8;
            if (e < D) st_from_f32<T>(orow + e, oacc[j8] * inv);
        }
        if (sub == 0) lse[(int64_t)bh * T_ + qa] = m_run + logf(l_run);
    }
}

// delta[bh, t] = sum_e dO * O  -- one thread per (b, t, h) row
template <typename T>
__global__ void k_attn_delta(int64_t B, int64_t T_, int H, int D, const T* __restrict__ o, int64_t ldo,
                             const T* __restrict__ dout, int64_t ldd, float* __restrict__ delta) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (b*T + t)*H + h
    if (row >= B * T_ * H) return;
    const int64_t bt = row / H;
    const int h = (int)(row % H);
    const int64_t b = bt / T_, t = bt % T_;
    const T* op = o + bt * ldo + h * D;
    const T* dp = dout + bt * ldd + h * D;
    float s = 0.f;
    if (sizeof(T) == 2 && D % 8 == 0 && ((((uintptr_t)op) | ((uintptr_t)dp)) & 15) == 0) {
        for (int e = 0; e < D; e += 8) {
            const uint4 a = *(const uint4*)(op + e), c = *(const uint4*)(dp + e);
            const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s += __uint_as_float(aw[q] << 16) * __uint_as_float(cw[q] << 16);
                s += __uint_as_float(aw[q] & 0xffff0000u) * __uint_as_float(cw[q] & 0xffff0000u);
            }
        }
    } else {
        for (int e = 0; e < D; ++e) s += ld_as_f32<T>(op + e) * ld_as_f32<T>(dp + e);
    }
    delta[(b * H + h) * T_ + t] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void k_attn_dq_generic(int64_t T_, int H, int D, const T* __restrict__ q,
                                                         const T* __restrict__ k, const T* __restrict__ v, int64_t ld,
                                                         const T* __restrict__ dout, int64_t ldd,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta, T* __restrict__ dq,
                                                         int64_t lddq, float scale, DropArgs drop) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int DP = D + 1;
    float* Qs = sm;
    float* Os = Qs + GB * DP;  // dO rows
    float* Ks = Os + GB * DP;
    float* Vs = Ks + GB * DP;
    float* Ss = Vs + GB * DP;  // dS [GB][GB+1]
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int qb = blockIdx.x;
    const int64_t q0 = (int64_t)qb * GB;
    const int tid = threadIdx.x, qi = tid >> 3, sub = tid & 7;
    const int64_t qa = q0 + qi;
    const int64_t boff = (int64_t)b * T_;
    load_rows<T>(Qs, DP, q + boff * ld + h * D, ld, q0, T_, D, tid);
    load_rows<T>(Os, DP, dout + boff * ldd + h * D, ldd, q0, T_, D, tid);
    const bool valid_q = qa < T_;
    const float lq = valid_q ? lse[(int64_t)bh * T_ + qa] : 0.f;
    const float dq_ = valid_q ? delta[(int64_t)bh * T_ + qa] : 0.f;
    const uint64_t stream = drop.thr ? dropout_stream(drop.rng_call, drop.site) : 0;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    for (int kb = 0; kb <= qb; ++kb) {
        const int64_t k0 = (int64_t)kb * GB;
        __syncthreads();
        load_rows<T>(Ks, DP, k + boff * ld + h * D, ld, k0, T_, D, tid);
        load_rows<T>(Vs, DP, v + boff * ld + h * D, ld, k0, T_, D, tid);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = sub + 8 * jj;
            const int64_t key = k0 + j;
            float ds = 0.f;
            if (valid_q && key <= qa) {
                float s = 0.f, dp = 0.f;
                for (int e = 0; e < D; ++e) {
                    s += Qs[qi * DP + e] * Ks[j * DP + e];
                    dp += Os[qi * DP + e] * Vs[j * DP + e];
                }
                const float p = expf(s * scale - lq);
                if (drop.thr) {
                    const uint64_t idx = (((uint64_t)bh * T_ + qa) * T_ + key);
                    dp = keep_elem(drop, stream, idx) ? dp * drop.dscale : 0.f;
                }
                ds = p * (dp - dq_);
            }
            Ss[qi * (GB + 1) + j] = ds;
        }
        __syncthreads();
#pragma unroll
        for (int j8 = 0; j8 < 16; ++j8) {
            const int e = sub + 8 * j8;
            if (e < D) {
                float a = acc[j8];
                for (int j = 0; j < GB; ++j) a += Ss[qi * (GB + 1) + j] * Ks[j * DP + e];
                acc[j8] = a;
            }
        }
    }
    if (valid_q) {
        T* row = dq + (boff + qa) * lddq + h * D;
#pragma unroll
        for (int j8 = 0; j8 < 16; ++j8) {
            const int e = sub + 8 * j8;
            if (e < D) st_from_f32<T>(row + e, acc[j8] * scale);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_attn_dkdv_generic(int64_t T_, int H, int D, const T* __restrict__ q,
                                                           const T* __restrict__ k, const T* __restrict__ v,
                                                           int64_t ld, const T* __restrict__ dout, int64_t ldd,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, T* __restrict__ dk,
                                                           T* __restrict__ dv, int64_t lddkv, float scale,
                                                           DropArgs drop) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int DP = D + 1;
    float* Ks = sm;
    float* Vs = Ks + GB * DP;
    float* Qs = Vs + GB * DP;
    float* Os = Qs + GB * DP;
    float* Zs = Os + GB * DP;        // [key][q]
    float* Ds = Zs + GB * (GB + 1);  // [key][q]
    float* Ls = Ds + GB * (GB + 1);  // lse[GB], delta[GB]
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int kb = blockIdx.x;
    const int64_t k0 = (int64_t)kb * GB;
    const int tid = threadIdx.x, kj = tid >> 3, sub = tid & 7;
    const int64_t ka = k0 + kj;
    const int64_t boff = (int64_t)b * T_;
    load_rows<T>(Ks, DP, k + boff * ld + h * D, ld, k0, T_, D, tid);
    load_rows<T>(Vs, DP, v + boff * ld + h * D, ld, k0, T_, D, tid);
    const uint64_t stream = drop.thr ? dropout_stream(drop.rng_call, drop.site) : 0;
    float adk[16], adv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) adk[j] = adv[j] = 0.f;
    const int nqb = (int)((T_ + GB - 1) / GB);
    for (int qb = kb; qb < nqb; ++qb) {
        const int64_t q0 = (int64_t)qb * GB;
        __syncthreads();
        load_rows<T>(Qs, DP, q + boff * ld + h * D, ld, q0, T_, D, tid);
        load_rows<T>(Os, DP, dout + boff * ldd + h * D, ldd, q0, T_, D, tid);
        if (tid < GB) {
            const int64_t t = q0 + tid;
            Ls[tid] = t < T_ ? lse[(int64_t)bh * T_ + t] : 0.f;
            Ls[GB + tid] = t < T_ ? delta[(int64_t)bh * T_ + t] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const int qi = sub + 8 * ii;
            const int64_t qa = q0 + qi;
            float z = 0.f, ds = 0.f;
            if (ka < T_ && qa < T_ && ka <= qa) {
                float s = 0.f, dp = 0.f;
                for (int e = 0; e < D; ++e) {
                    s += Ks[kj * DP + e] * Qs[qi * DP + e];
                    dp += Vs[kj * DP + e] * Os[qi * DP + e];
                }
                const float p = expf(s * scale - Ls[qi]);
                z = p;
                if (drop.thr) {
                    const uint64_t idx = (((uint64_t)bh * T_ + qa) * T_ + ka);
                    const bool kp = keep_elem(drop, stream, idx);
                    z = kp ? p * drop.dscale : 0.f;
                    dp = kp ? dp * drop.dscale : 0.f;
                }
                ds = p * (dp - Ls[GB + qi]);
            }
            Zs[kj * (GB + 1) + qi] = z;
            Ds[kj * (GB + 1) + qi] = ds;
        }
        __syncthreads();
#pragma unroll 1
        for (int i = 0; i < GB; ++i) {
            const float zi = Zs[kj * (GB + 1) + i], di = Ds[kj * (GB + 1) + i];
#pragma unroll
            for (int j8 = 0; j8 < 16; ++j8) {
                const int e = sub + 8 * j8;
                if (e < D) {
                    adv[j8] += zi * Os[i * DP + e];
                    adk[j8] += di * Qs[i * DP + e];
                }
            }
        }
    }
    if (ka < T_) {
        T* krow = dk + (boff + ka) * lddkv + h * D;
        T* vrow = dv + (boff + ka) * lddkv + h * D;
#pragma unroll
        for (int j8 = 0; j8 < 16; ++j8) {
            const int e = sub + 8 * j8;
            if (e < D) {
                st_from_f32<T>(krow + e, adk[j8] * scale);
                st_from_f32<T>(vrow + e, adv[j8]);
            }
        }
    }
}

// =====================================================================================
// bf16 MFMA kernels for head_size 64
// =====================================================================================
typedef __attribute__((address_space(3))) sv4 lds_sv4;

__device__ __forceinline__ fv4 mfma16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

// [rows][64] bf16 images with 128-B rows; chunk (16 B) c in 0..7.
// f_row: conflict-free for ds_read_b128 row reads; f_tr: conflict-free for ds_read_b64_tr_b16.
__device__ __forceinline__ int off_row(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ int off_tr(int r, int c) { return r * 128 + ((c ^ (((r >> 1) & 3) << 1)) << 4); }

template <bool TRSWZ>
__device__ __forceinline__ int img_off(int r, int c) {
    return TRSWZ ? off_tr(r, c) : off_row(r, c);
}

// stage a [64 rows][64] bf16 tile (rows row0.. of a (b*T+t)*ld + h*64 tensor) into an image
template <bool TRSWZ>
__device__ __forceinline__ void stage_tile(char* img, const bf16_t* base, int64_t ld, int64_t row0, int tid) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (tid >> 3) + 32 * i, c = tid & 7;
        const uint4 g = *(const uint4*)(base + (row0 + r) * ld + c * 8);
        *(uint4*)(img + img_off<TRSWZ>(r, c)) = g;
    }
}

// A/B fragment from rows rb..rb+15, k = 32s..32s+31 (K-contiguous read)
template <bool TRSWZ>
__device__ __forceinline__ sv8 frag_rows(const char* img, int rb, int s, int lane) {
    return *(const sv8*)(img + img_off<TRSWZ>(rb + (lane & 15), s * 4 + (lane >> 4)));
}

// transposed fragment: operand X(m = col e0 + (lane&15), k = kappa) where kappa = 8g + j maps to
// image row rbase + 16*(j>>2) + 4g + (j&3)  (the accumulator-as-operand key order)
template <bool TRSWZ>
__device__ __forceinline__ sv8 frag_tr(const char* img, int rbase, int e0, int lane) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
    const int chunk = (e0 >> 3) + (p >> 1), byte = 8 * (p & 1);
    const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_off<TRSWZ>(rbase + 4 * g + qq, chunk) + byte));
    const sv4 hi =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_off<TRSWZ>(rbase + 16 + 4 * g + qq, chunk) + byte));
    return sv8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ sv8 pack8(const fv4& a, const fv4& b) {
    const uint32_t w0 = pack_bf2(a[0], a[1]), w1 = pack_bf2(a[2], a[3]), w2 = pack_bf2(b[0], b[1]),
                   w3 = pack_bf2(b[2], b[3]);
    sv8 r;
    r[0] = (short)(w0 & 0xffff); r[1] = (short)(w0 >> 16);
    r[2] = (short)(w1 & 0xffff); r[3] = (short)(w1 >> 16);
    r[4] = (short)(w2 & 0xffff); r[5] = (short)(w2 >> 16);
    r[6] = (short)(w3 & 0xffff); r[7] = (short)(w3 >> 16);
    return r;
}

// ---------------------------------------------------------------------------------------
// forward, D = 64: block = 4 waves x 32 queries; KV tiles of 64 keys double-buffered in LDS.
// Swapped product S^T = K Q^T keeps one query per lane column, so softmax statistics are
// lane-local (+2 cross-group shuffles) and P^T feeds O^T = V^T P^T with no data movement.
// ---------------------------------------------------------------------------------------
constexpr int FQ = 128;  // queries per block

__global__ __launch_bounds__(256) void k_attn_fwd_d64(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                      const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                      int64_t ld, bf16_t* __restrict__ o, int64_t ldo,
                                                      float* __restrict__ lse, float scale_log2, DropArgs drop) {
    __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][K,V]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int64_t qblk0 = (int64_t)blockIdx.x * FQ;
    const int64_t qw0 = qblk0 + wave * 32;  // this wave's first query
    const int64_t boff = (int64_t)b * T_;
    const bf16_t* kb_ = k + boff * ld + h * 64;
    const bf16_t* vb_ = v + boff * ld + h * 64;
    const bool wave_active = qw0 < T_;

    // Q^T fragments (B operand): lane holds Q[q = qw0 + 16qt + li][e = 32s + 8g ..+7]
    sv8 qf[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int64_t qrow = qw0 + 16 * qt + li;
            qf[qt][s] = wave_active ? *(const sv8*)(q + (boff + qrow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
        }

    fv4 oacc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) oacc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
    const int NT = (int)(T_ >> 4);

    const int64_t qlast = (qblk0 + FQ - 1) < (T_ - 1) ? (qblk0 + FQ - 1) : (T_ - 1);
    const int nkv = (int)(qlast / 64) + 1;
    stage_tile<false>(smem[0][0], kb_, ld, 0, tid);
    stage_tile<true>(smem[0][1], vb_, ld, 0, tid);
    __syncthreads();
    for (int kv = 0; kv < nkv; ++kv) {
        const int st = kv & 1;
        if (kv + 1 < nkv) {  // prefetch next tile into the other stage (read last iteration, barrier passed)
            stage_tile<false>(smem[st ^ 1][0], kb_, ld, (int64_t)(kv + 1) * 64, tid);
            stage_tile<true>(smem[st ^ 1][1], vb_, ld, (int64_t)(kv + 1) * 64, tid);
        }
        const int64_t k0 = (int64_t)kv * 64;
        if (wave_active && k0 <= qw0 + 31) {
            const char* Ki = smem[st][0];
            const char* Vi = smem[st][1];
            fv4 sacc[4][2];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                const sv8 a0 = frag_rows<false>(Ki, 16 * kt, 0, lane);
                const sv8 a1 = frag_rows<false>(Ki, 16 * kt, 1, lane);
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) {
                    fv4 c = {0.f, 0.f, 0.f, 0.f};
                    c = mfma16(a0, qf[qt][0], c);
                    sacc[kt][qt] = mfma16(a1, qf[qt][1], c);
                }
            }
            const bool diag = k0 + 63 > qw0;  // some key may exceed some query of this wave
            float alpha[2];
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
                const int64_t qa = qw0 + 16 * qt + li;
                float mx = -INFINITY;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float x = sacc[kt][qt][r] * scale_log2;
                        if (diag && k0 + 16 * kt + 4 * g + r > qa) x = -INFINITY;
                        sacc[kt][qt][r] = x;
                        mx = fmaxf(mx, x);
                    }
                mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
                mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
                const float m_new = fmaxf(m_run[qt], mx);
                alpha[qt] = exp2f(m_run[qt] - m_new);
                float ls = 0.f;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    const uint64_t* mw = nullptr;
                    if (drop.mask) mw = mask_tile(drop.mask, bh, NT, (int)((qw0 + 16 * qt) >> 4), (int)((k0 + 16 * kt) >> 4));
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float p = exp2f(sacc[kt][qt][r] - m_new);
                        ls += p;
                        float pd = p;
                        if (drop.mask) pd = ((mw[r] >> lane) & 1ull) ? p * drop.dscale : 0.f;
                        sacc[kt][qt][r] = pd;
                    }
                }
                ls += __shfl_xor(ls, 16, 64);
                ls += __shfl_xor(ls, 32, 64);
                l_run[qt] = l_run[qt] * alpha[qt] + ls;
                m_run[qt] = m_new;
            }
            // P^T as B operand: k-step u covers key tiles 2u, 2u+1
            sv8 pf[2][2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) pf[u][qt] = pack8(sacc[2 * u][qt], sacc[2 * u + 1][qt]);
#pragma unroll
            for (int et = 0; et < 4; ++et) {
                const sv8 v0 = frag_tr<true>(Vi, 0, 16 * et, lane);
                const sv8 v1 = frag_tr<true>(Vi, 32, 16 * et, lane);
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) {
                    fv4 c = oacc[et][qt] * alpha[qt];
                    c = mfma16(v0, pf[0][qt], c);
                    oacc[et][qt] = mfma16(v1, pf[1][qt], c);
                }
            }
        }
        __syncthreads();
    }
    if (!wave_active) return;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int64_t qa = qw0 + 16 * qt + li;
        if (qa >= T_) continue;
        const float inv = 1.f / l_run[qt];
        bf16_t* orow = o + (boff + qa) * ldo + h * 64;
#pragma unroll
        for (int et = 0; et < 4; ++et) {
            const fv4 x = oacc[et][qt] * inv;
            *(uint2*)(orow + 16 * et + 4 * g) = make_uint2(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]));
        }
        if (g == 0) lse[(int64_t)bh * T_ + qa] = (m_run[qt] + log2f(l_run[qt])) * LN2;
    }
}

// ---------------------------------------------------------------------------------------
// dQ, D = 64: swapped orientation as the forward.  Per 64-key tile:
//   S^T = K Q^T, dP^T = V dO^T, dS^T = P^T (dP^T keep/(1-p) - delta), dQ^T += K^T dS^T.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_attn_dq_d64(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                     const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                     int64_t ld, const bf16_t* __restrict__ dout, int64_t ldd,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     bf16_t* __restrict__ dq, int64_t lddq, float scale,
                                                     DropArgs drop) {
    __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][K,V]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int64_t qblk0 = (int64_t)blockIdx.x * FQ;
    const int64_t qw0 = qblk0 + wave * 32;
    const int64_t boff = (int64_t)b * T_;
    const bool wave_active = qw0 < T_;
    const float scale_log2 = scale * LOG2E;

    sv8 qf[2][2], of[2][2];
    float lq[2], dl[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int64_t qrow = qw0 + 16 * qt + li;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            qf[qt][s] = wave_active ? *(const sv8*)(q + (boff + qrow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
            of[qt][s] = wave_active ? *(const sv8*)(dout + (boff + qrow) * ldd + h * 64 + 32 * s + 8 * g) : sv8{};
        }
        lq[qt] = wave_active ? lse[(int64_t)bh * T_ + qrow] * LOG2E : 0.f;
        dl[qt] = wave_active ? delta[(int64_t)bh * T_ + qrow] : 0.f;
    }
    fv4 dqacc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) dqacc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    const int NT = (int)(T_ >> 4);
    const bf16_t* kb_ = k + boff * ld + h * 64;
    const bf16_t* vb_ = v + boff * ld + h * 64;
    const int64_t qlast = (qblk0 + FQ - 1) < (T_ - 1) ? (qblk0 + FQ - 1) : (T_ - 1);
    const int nkv = (int)(qlast / 64) + 1;
    stage_tile<false>(smem[0][0], kb_, ld, 0, tid);
    stage_tile<false>(smem[0][1], vb_, ld, 0, tid);
    __syncthreads();
    for (int kv = 0; kv < nkv; ++kv) {
        const int st = kv & 1;
        if (kv + 1 < nkv) {
            stage_tile<false>(smem[st ^ 1][0], kb_, ld, (int64_t)(kv + 1) * 64, tid);
            stage_tile<false>(smem[st ^ 1][1], vb_, ld, (int64_t)(kv + 1) * 64, tid);
        }
        const int64_t k0 = (int64_t)kv * 64;
        if (wave_active && k0 <= qw0 + 31) {
            const char* Ki = smem[st][0];
            const char* Vi = smem[st][1];
            fv4 sa[4][2], pa[4][2];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                const sv8 k0f = frag_rows<false>(Ki, 16 * kt, 0, lane), k1f = frag_rows<false>(Ki, 16 * kt, 1, lane);
                const sv8 v0f = frag_rows<false>(Vi, 16 * kt, 0, lane), v1f = frag_rows<false>(Vi, 16 * kt, 1, lane);
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) {
                    fv4 c = {0.f, 0.f, 0.f, 0.f};
                    c = mfma16(k0f, qf[qt][0], c);
                    sa[kt][qt] = mfma16(k1f, qf[qt][1], c);
                    fv4 d = {0.f, 0.f, 0.f, 0.f};
                    d = mfma16(v0f, of[qt][0], d);
                    pa[kt][qt] = mfma16(v1f, of[qt][1], d);
                }
            }
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
                const int64_t qa = qw0 + 16 * qt + li;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    const uint64_t* mw = nullptr;
                    if (drop.mask) mw = mask_tile(drop.mask, bh, NT, (int)((qw0 + 16 * qt) >> 4), (int)((k0 + 16 * kt) >> 4));
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t key = k0 + 16 * kt + 4 * g + r;
                        float p = key > qa ? 0.f : exp2f(sa[kt][qt][r] * scale_log2 - lq[qt]);
                        float dp = pa[kt][qt][r];
                        if (drop.mask) dp = ((mw[r] >> lane) & 1ull) ? dp * drop.dscale : 0.f;
                        sa[kt][qt][r] = p * (dp - dl[qt]);
                    }
                }
            }
            // dQ^T[e][q] += sum_key K^T[e][key] dS^T[key][q]
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                sv8 dsf[2];
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) dsf[qt] = pack8(sa[2 * u][qt], sa[2 * u + 1][qt]);
#pragma unroll
                for (int et = 0; et < 4; ++et) {
                    const sv8 kf = frag_tr<false>(Ki, 32 * u, 16 * et, lane);
#pragma unroll
                    for (int qt = 0; qt < 2; ++qt) dqacc[et][qt] = mfma16(kf, dsf[qt], dqacc[et][qt]);
                }
            }
        }
        __syncthreads();
    }
    if (!wave_active) return;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const int64_t qa = qw0 + 16 * qt + li;
        if (qa >= T_) continue;
        bf16_t* row = dq + (boff + qa) * lddq + h * 64;
#pragma unroll
        for (int et = 0; et < 4; ++et) {
            const fv4 x = dqacc[et][qt] * scale;
            *(uint2*)(row + 16 * et + 4 * g) = make_uint2(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]));
        }
    }
}

// ---------------------------------------------------------------------------------------
// dK/dV, D = 64: block = 4 waves x 32 keys (128 keys); loop over 64-query tiles (staged Q,
// dO, lse, delta).  Unswapped S = Q K^T puts the key on the lane so that Z (= dropped P) and
// dS feed dV^T = dO^T Z and dK^T = Q^T dS as B operands directly.  Dropout bits are made in
// the forward's (query-on-lane) grouping and redistributed with 4 ballots.
// ---------------------------------------------------------------------------------------
constexpr int FK = 128;  // keys per block

__global__ __launch_bounds__(256) void k_attn_dkdv_d64(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                       const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                       int64_t ld, const bf16_t* __restrict__ dout, int64_t ldd,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ delta, bf16_t* __restrict__ dk,
                                                       bf16_t* __restrict__ dv, int64_t lddkv, float scale,
                                                       DropArgs drop) {
    __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][Q,dO]
    __shared__ float stat[2][2][64];                                  // [stage][lse*log2e, delta]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int64_t kblk0 = (int64_t)blockIdx.x * FK;
    const int64_t kw0 = kblk0 + wave * 32;  // this wave's first key
    const int64_t boff = (int64_t)b * T_;
    const bool wave_active = kw0 < T_;
    const float scale_log2 = scale * LOG2E;

    // K, V fragments as B operands of S = Q K^T and dP = dO V^T: lane holds X[key = kw0+16kt+li][e = 32s+8g..]
    sv8 kf[2][2], vf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int64_t krow = kw0 + 16 * kt + li;
            kf[kt][s] = wave_active ? *(const sv8*)(k + (boff + krow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
            vf[kt][s] = wave_active ? *(const sv8*)(v + (boff + krow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
        }
    fv4 dka[4][2], dva[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) dka[i][j] = dva[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    const int NT = (int)(T_ >> 4);
    const bf16_t* qb_ = q + boff * ld + h * 64;
    const bf16_t* ob_ = dout + boff * ldd + h * 64;
    const int nq = (int)(T_ / 64);
    const int q_start = (int)(kblk0 / 64);

    auto stage = [&](int st, int qtile) {
        stage_tile<false>(smem[st][0], qb_, ld, (int64_t)qtile * 64, tid);
        stage_tile<false>(smem[st][1], ob_, ldd, (int64_t)qtile * 64, tid);
        if (tid < 64) {
            stat[st][0][tid] = lse[(int64_t)bh * T_ + (int64_t)qtile * 64 + tid] * LOG2E;
            stat[st][1][tid] = delta[(int64_t)bh * T_ + (int64_t)qtile * 64 + tid];
        }
    };
    stage(0, q_start);
    __syncthreads();
    for (int qtile = q_start; qtile < nq; ++qtile) {
        const int st = (qtile - q_start) & 1;
        if (qtile + 1 < nq) stage(st ^ 1, qtile + 1);
        const int64_t q0 = (int64_t)qtile * 64;
        if (wave_active && q0 + 63 >= kw0) {
            const char* Qi = smem[st][0];
            const char* Oi = smem[st][1];
#pragma unroll
            for (int half = 0; half < 2; ++half) {  // 32 queries at a time: qt = 2*half + {0,1}
                const int qr0 = 32 * half;
                if (q0 + qr0 + 31 < kw0) continue;  // all these queries precede all this wave's keys
                fv4 sa[2][2], pa[2][2];             // [qt][kt]
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) {
                    const sv8 q0f = frag_rows<false>(Qi, qr0 + 16 * qt, 0, lane), q1f = frag_rows<false>(Qi, qr0 + 16 * qt, 1, lane);
                    const sv8 o0f = frag_rows<false>(Oi, qr0 + 16 * qt, 0, lane), o1f = frag_rows<false>(Oi, qr0 + 16 * qt, 1, lane);
#pragma unroll
                    for (int kt = 0; kt < 2; ++kt) {
                        fv4 c = {0.f, 0.f, 0.f, 0.f};
                        c = mfma16(q0f, kf[kt][0], c);
                        sa[qt][kt] = mfma16(q1f, kf[kt][1], c);
                        fv4 d = {0.f, 0.f, 0.f, 0.f};
                        d = mfma16(o0f, vf[kt][0], d);
                        pa[qt][kt] = mfma16(o1f, vf[kt][1], d);
                    }
                }
                // probabilities, dropout, dS.  lane: key = kw0 + 16kt + li, query = q0 + qr0 + 16qt + 4g + r
                sv8 zf[2], dsf[2];
                fv4 z[2][2], ds[2][2];
#pragma unroll
                for (int qt = 0; qt < 2; ++qt)
#pragma unroll
                    for (int kt = 0; kt < 2; ++kt) {
                        const int64_t key = kw0 + 16 * kt + li;
                        uint64_t keepbits = ~0ull;  // bit r set -> keep (query 4g + r)
                        if (drop.mask) {
                            // tile words are in the forward's (query-on-lane) order: word w, bit l =
                            // keep(query l&15, key 4(l>>4) + w); transpose through the bit index
                            const uint64_t* mw =
                                mask_tile(drop.mask, bh, NT, (int)((q0 + qr0 + 16 * qt) >> 4), (int)((kw0 + 16 * kt) >> 4));
                            const int w = li & 3;  // my key's word within its group
                            const uint64_t bw = w == 0 ? mw[0] : (w == 1 ? mw[1] : (w == 2 ? mw[2] : mw[3]));
                            // source lane for (query 4g + r, key li): (4g + r) + 16 * (li >> 2)
                            keepbits = 0;
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                keepbits |= ((bw >> ((4 * g + r) + 16 * (li >> 2))) & 1ull) << r;
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int qrel = qr0 + 16 * qt + 4 * g + r;
                            const int64_t qa = q0 + qrel;
                            const float p =
                                key > qa ? 0.f : exp2f(sa[qt][kt][r] * scale_log2 - stat[st][0][qrel]);
                            float dp = pa[qt][kt][r];
                            float zz = p;
                            if (drop.mask) {
                                const bool kp = (keepbits >> r) & 1ull;
                                dp = kp ? dp * drop.dscale : 0.f;
                                zz = kp ? p * drop.dscale : 0.f;
                            }
                            z[qt][kt][r] = zz;
                            ds[qt][kt][r] = p * (dp - stat[st][1][qrel]);
                        }
                    }
#pragma unroll
                for (int kt = 0; kt < 2; ++kt) {
                    zf[kt] = pack8(z[0][kt], z[1][kt]);
                    dsf[kt] = pack8(ds[0][kt], ds[1][kt]);
                }
                // dV^T[e][key] += dO^T[e][q] Z[q][key];  dK^T[e][key] += Q^T[e][q] dS[q][key]
#pragma unroll
                for (int et = 0; et < 4; ++et) {
                    const sv8 oft = frag_tr<false>(Oi, qr0, 16 * et, lane);
                    const sv8 qft = frag_tr<false>(Qi, qr0, 16 * et, lane);
#pragma unroll
                    for (int kt = 0; kt < 2; ++kt) {
                        dva[et][kt] = mfma16(oft, zf[kt], dva[et][kt]);
                        dka[et][kt] = mfma16(qft, dsf[kt], dka[et][kt]);
                    }
                }
            }
        }
        __syncthreads();
    }
    if (!wave_active) return;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        const int64_t key = kw0 + 16 * kt + li;
        if (key >= T_) continue;
        bf16_t* krow = dk + (boff + key) * lddkv + h * 64;
        bf16_t* vrow = dv + (boff + key) * lddkv + h * 64;
#pragma unroll
        for (int et = 0; et < 4; ++et) {
            const fv4 x = dka[et][kt] * scale;
            const fv4 y = dva[et][kt];
            *(uint2*)(krow + 16 * et + 4 * g) = make_uint2(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]));
            *(uint2*)(vrow + 16 * et + 4 * g) = make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
        }
    }
}

DropArgs make_drop(double p, uint64_t seed, const uint64_t* rng_call, int site) {
    DropArgs d;
    d.thr = p > 0 ? dropout_threshold(p) : 0u;
    d.dscale = p > 0 ? dropout_scale(p) : 1.f;
    d.seed = seed;
    d.rng_call = rng_call;
    d.site = site;
    d.mask = nullptr;
    return d;
}

int64_t mask_bytes(int64_t B, int64_t H, int64_t T) { return B * H * (T / 16) * (T / 16) * 32; }

void launch_dropmask(int64_t B, int64_t H, int64_t T, uint64_t* mask, const DropArgs& d, hipStream_t st) {
    const int64_t NT = T / 16;
    dim3 grid(ceil_div(NT * NT, 4), (unsigned)(B * H));
    k_attn_dropmask<<<grid, 256, 0, st>>>(T, mask, d);
}

bool fast_attn_ok(int dtype, int64_t T, int64_t D, const void* a, const void* b, const void* c, int64_t ld1,
                  int64_t ld2) {
    return dtype == CG_BF16 && D == 64 && T % 64 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) == 0 &&
           ld1 % 8 == 0 && ld2 % 8 == 0;
}

template <typename T>
size_t generic_lds(int D, int nrows_blocks, int nsq) {
    return (size_t)(nrows_blocks * GB * (D + 1) + nsq * GB * (GB + 1) + 2 * GB) * sizeof(float);
}

}  // namespace

extern "C" int cg_attn_fwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                           const void* v, int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale,
                           double dropout_p, uint64_t seed, const uint64_t* rng_call, int site, uint64_t* mask,
                           void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && H > 0 && D > 0 && D <= 128, "cg_attn_fwd: bad shape (D must be <= 128)");
    CG_REQUIRE(dropout_p >= 0 && dropout_p < 1, "cg_attn_fwd: dropout_p must be in [0,1)");
    hipStream_t st = (hipStream_t)stream;
    DropArgs d = make_drop(dropout_p, seed, rng_call, site);
    if (fast_attn_ok(dtype, T, D, q, k, o, ld_qkv, ld_o)) {
        if (d.thr) {
            CG_REQUIRE(mask, "cg_attn_fwd: dropout on the MFMA path needs a mask buffer (cg_attn_mask_bytes)");
            launch_dropmask(B, H, T, mask, d, st);
            d.mask = mask;
        }
        dim3 grid(ceil_div(T, FQ), (unsigned)(B * H));
        k_attn_fwd_d64<<<grid, 256, 0, st>>>(T, (int)H, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ld_qkv,
                                             (bf16_t*)o, ld_o, lse, scale * LOG2E, d);
    } else {
        dim3 grid(ceil_div(T, GB), (unsigned)(B * H));
        const size_t lds = generic_lds<float>((int)D, 3, 1);
        if (dtype == CG_BF16)
            k_attn_fwd_generic<bf16_t><<<grid, 256, lds, st>>>(T, (int)H, (int)D, (const bf16_t*)q, (const bf16_t*)k,
                                                               (const bf16_t*)v, ld_qkv, (bf16_t*)o, ld_o, lse, scale, d);
        else
            k_attn_fwd_generic<float><<<grid, 256, lds, st>>>(T, (int)H, (int)D, (const float*)q, (const float*)k,
                                                              (const float*)v, ld_qkv, (float*)o, ld_o, lse, scale, d);
    }
    CG_LAUNCH_CHECK("cg_attn_fwd");
    return CG_OK;
}

extern "C" int64_t cg_attn_mask_bytes(int64_t B, int64_t H, int64_t T) { return mask_bytes(B, H, T); }

extern "C" int64_t cg_attn_bwd_workspace(int64_t B, int64_t T, int64_t H, int64_t D) {
    (void)D;
    const int64_t delta = (B * H * T * (int64_t)sizeof(float) + 255) / 256 * 256;
    return delta + mask_bytes(B, H, T);
}

extern "C" int cg_attn_bwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                           const void* v, int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout, int64_t ld_do,
                           const float* lse, void* dq, void* dk, void* dv, int64_t ld_dqkv, float scale,
                           double dropout_p, uint64_t seed, const uint64_t* rng_call, int site, const uint64_t* mask,
                           void* workspace, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && H > 0 && D > 0 && D <= 128, "cg_attn_bwd: bad shape (D must be <= 128)");
    CG_REQUIRE(workspace, "cg_attn_bwd: workspace required");
    hipStream_t st = (hipStream_t)stream;
    DropArgs d = make_drop(dropout_p, seed, rng_call, site);
    float* delta = (float*)workspace;
    const int64_t nrows = B * T * H;
    if (dtype == CG_BF16)
        k_attn_delta<bf16_t><<<ceil_div(nrows, 256), 256, 0, st>>>(B, T, (int)H, (int)D, (const bf16_t*)o, ld_o,
                                                                 (const bf16_t*)dout, ld_do, delta);
    else
        k_attn_delta<float><<<ceil_div(nrows, 256), 256, 0, st>>>(B, T, (int)H, (int)D, (const float*)o, ld_o,
                                                                (const float*)dout, ld_do, delta);
    const bool fast = fast_attn_ok(dtype, T, D, q, dout, dq, ld_qkv, ld_do) && ld_dqkv % 8 == 0 &&
                      ((((uintptr_t)dk) | ((uintptr_t)dv)) & 15) == 0;
    if (fast) {
        if (d.thr) {
            if (!mask) {  // regenerate the forward's keep bits (identical Philox stream)
                uint64_t* m = (uint64_t*)((char*)workspace + (B * H * T * (int64_t)sizeof(float) + 255) / 256 * 256);
                launch_dropmask(B, H, T, m, d, st);
                mask = m;
            }
            d.mask = mask;
        }
        const bf16_t *Q = (const bf16_t*)q, *K = (const bf16_t*)k, *V = (const bf16_t*)v, *DO = (const bf16_t*)dout;
        k_attn_dq_d64<<<dim3(ceil_div(T, FQ), (unsigned)(B * H)), 256, 0, st>>>(T, (int)H, Q, K, V, ld_qkv, DO, ld_do, lse,
                                                                               delta, (bf16_t*)dq, ld_dqkv, scale, d);
        k_attn_dkdv_d64<<<dim3(ceil_div(T, FK), (unsigned)(B * H)), 256, 0, st>>>(
            T, (int)H, Q, K, V, ld_qkv, DO, ld_do, lse, delta, (bf16_t*)dk, (bf16_t*)dv, ld_dqkv, scale, d);
    } else {
        dim3 grid(ceil_div(T, GB), (unsigned)(B * H));
        const size_t lds_dq = generic_lds<float>((int)D, 4, 1);
        const size_t lds_kv = generic_lds<float>((int)D, 4, 2);
        if (dtype == CG_BF16) {
            k_attn_dq_generic<bf16_t><<<grid, 256, lds_dq, st>>>(T, (int)H, (int)D, (const bf16_t*)q, (const bf16_t*)k,
                                                                 (const bf16_t*)v, ld_qkv, (const bf16_t*)dout, ld_do,
                                                                 lse, delta, (bf16_t*)dq, ld_dqkv, scale, d);
            k_attn_dkdv_generic<bf16_t><<<grid, 256, lds_kv, st>>>(T, (int)H, (int)D, (const bf16_t*)q,
                                                                   (const bf16_t*)k, (const bf16_t*)v, ld_qkv,
                                                                   (const bf16_t*)dout, ld_do, lse, delta,
                                                                   (bf16_t*)dk, (bf16_t*)dv, ld_dqkv, scale, d);
        } else {
            k_attn_dq_generic<float><<<grid, 256, lds_dq, st>>>(T, (int)H, (int)D, (const float*)q, (const float*)k,
                                                                (const float*)v, ld_qkv, (const float*)dout, ld_do,
                                                                lse, delta, (float*)dq, ld_dqkv, scale, d);
            k_attn_dkdv_generic<float><<<grid, 256, lds_kv, st>>>(T, (int)H, (int)D, (const float*)q, (const float*)k,
                                                                  (const float*)v, ld_qkv, (const float*)dout, ld_do,
                                                                  lse, delta, (float*)dk, (float*)dv, ld_dqkv, scale,
                                                                  d);
        }
    }
    CG_LAUNCH_CHECK("cg_attn_bwd");
    return CG_OK;
}
