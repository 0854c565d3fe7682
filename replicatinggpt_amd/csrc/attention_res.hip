// charpt: bf16 MFMA causal attention with the whole (batch, head) resident in LDS -- the C2 path
// (block_size 256, head_size 64) of Head.forward x n_head (GPT1.py:109-123,134-135).
//
// Measured on MI355X (profiles/r1_c2_pmc_step.txt): the streaming kernels of attention_d64.hip
// spend most of their time waiting on one 64-row K/V (or Q/dO) tile after another -- at T = 256 a
// query block sees at most 4 tiles, so every tile is a full global-load latency with little MFMA
// work to hide it.  Here one 512-thread block owns one (b, h):
//   forward : K, V (T x 64 bf16 each) and the (b, h)'s dropout keep bits are loaded ONCE into LDS
//             (all loads in flight together, one barrier); 8 waves x 32 queries then run the
//             online-softmax loop of attention_d64.hip's forward over the resident tiles.
//   backward: Q, K, V, dO, lse and the keep bits resident (138 KB), delta = rowsum(dO * O)
//             computed in the prologue; each wave then computes dK/dV for 32 keys (key-owned,
//             query tiles >= key) and dQ for 32 queries (query-owned, key tiles <= query) -- the
//             two causal loops have opposite per-wave lengths, so every wave does the same work,
//             and one launch replaces delta + dQ + dK/dV.
// Same math, layouts and key orders as attention_d64.hip (S^T = K Q^T for forward / dQ, S = Q K^T
// for dK / dV); no float atomics.  Requires T % 64 == 0, T <= 256, D = 64.
//
// Status: opt-in (attn_variant bit 8).  Measured at C2 (B 64, H 6, T 256) these run SLOWER than the
// streaming kernels (forward 43 vs 35 us, backward 86 vs 83 us): 384 blocks of 8 waves leave half
// the CUs with one block and the causal loop makes waves within a block uneven (1..4 tiles), so
// per-CU parallelism, not tile-load latency, bounds this size (profiles/r1_attention_res.txt).
#include "attention_tile.h"

namespace cg {
namespace {
using namespace atile;

constexpr int RT = 256;                   // max resident sequence length
constexpr int IMG = RT * 128;             // [256][64] bf16 image
constexpr int MSKB = (RT / 16) * (RT / 16) * 32;  // keep bits of one (b, h)

// copy R rows x 64 bf16 (row stride ld) into an image (row / transposed-read swizzle), 512 threads
template <bool TRSWZ>
__device__ __forceinline__ void load_image(const bf16_t* __restrict__ base, int64_t ld, int R, char* img, int tid) {
    constexpr int N = RT * 8 / 512;
    uint4 v0, v1, v2, v3;   // named (not an array): a conditionally written array goes to scratch
    static_assert(N == 4, "image load is unrolled for 4 chunks per thread");
    auto ld16 = [&](int i) {
        const int c = tid + 512 * i, r = min(c >> 3, R - 1), cc = c & 7;
        return *(const uint4*)(base + (int64_t)r * ld + cc * 8);
    };
    auto st16 = [&](int i, const uint4& x) {
        const int c = tid + 512 * i, r = c >> 3, cc = c & 7;
        if (r < R) *(uint4*)(img + img_off<TRSWZ>(r, cc)) = x;
    };
    v0 = ld16(0);
    v1 = ld16(1);
    v2 = ld16(2);
    v3 = ld16(3);
    st16(0, v0);
    st16(1, v1);
    st16(2, v2);
    st16(3, v3);
}

__device__ __forceinline__ void load_mask(const uint64_t* __restrict__ mask, int bh, int NT, char* dst, int tid) {
    const int bytes = NT * NT * 32;
    const char* src = (const char*)mask_tile(mask, bh, NT, 0, 0);
    for (int o = tid * 16; o < bytes; o += 512 * 16) *(uint4*)(dst + o) = *(const uint4*)(src + o);
}

// =====================================================================================
// forward: 8 waves x 32 queries over resident K / V
// =====================================================================================
__global__ __launch_bounds__(512, 2) void k_attn_fwd_res(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                        const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                        int64_t ld, bf16_t* __restrict__ o, int64_t ldo,
                                                        float* __restrict__ lse, float scale_log2,
                                                        const uint64_t* __restrict__ mask, float dscale) {
    constexpr int QW = 32, QT = 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ki = smem;
    char* Vi = smem + IMG;
    char* Mi = smem + 2 * IMG;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int bh = blockIdx.x, b = bh / H, h = bh % H;
    const int T = (int)T_, NT = T >> 4;
    const int64_t boff = (int64_t)b * T_;
    const int qw0 = wave * QW;
    const bool active = qw0 < T;
    sv8 qf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
            qf[qt][s] = active ? *(const sv8*)(q + (boff + qw0 + 16 * qt + li) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
    load_image<false>(k + boff * ld + h * 64, ld, T, Ki, tid);
    load_image<true>(v + boff * ld + h * 64, ld, T, Vi, tid);
    if (mask) load_mask(mask, bh, NT, Mi, tid);
    __syncthreads();
    if (!active) return;

    fv4 oacc[4][QT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < QT; ++j) oacc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    float m_run[QT], l_run[QT];
#pragma unroll
    for (int j = 0; j < QT; ++j) {
        m_run[j] = -INFINITY;
        l_run[j] = 0.f;
    }
    const int nkv = (qw0 + QW - 1) / 64 + 1;
    for (int kv = 0; kv < nkv; ++kv) {
        const int k0 = kv * 64;
        fv4 sacc[4][QT];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const sv8 a0 = frag_rows<false>(Ki, k0 + 16 * kt, 0, lane), a1 = frag_rows<false>(Ki, k0 + 16 * kt, 1, lane);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                fv4 c = {0.f, 0.f, 0.f, 0.f};
                c = mfma16(a0, qf[qt][0], c);
                sacc[kt][qt] = mfma16(a1, qf[qt][1], c);
            }
        }
        const bool diag = k0 + 63 > qw0;
        float alpha[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const int qa = qw0 + 16 * qt + li;
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
            const int q16 = (qw0 >> 4) + qt;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                Words4 mw;
                if (mask) mw = lds_words(Mi + (q16 * NT + kv * 4 + kt) * 32);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float p = exp2f(sacc[kt][qt][r] - m_new);
                    ls += p;
                    sacc[kt][qt][r] = (!mask || ((mw.w[r] >> lane) & 1ull)) ? p * dscale : 0.f;
                }
            }
            ls += __shfl_xor(ls, 16, 64);
            ls += __shfl_xor(ls, 32, 64);
            l_run[qt] = l_run[qt] * alpha[qt] + ls;
            m_run[qt] = m_new;
        }
        sv8 pf[2][QT];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) pf[u][qt] = pack8(sacc[2 * u][qt], sacc[2 * u + 1][qt]);
#pragma unroll
        for (int et = 0; et < 4; ++et) {
            const sv8 v0 = frag_tr<true>(Vi, k0, 16 * et, lane), v1 = frag_tr<true>(Vi, k0 + 32, 16 * et, lane);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                fv4 c = oacc[et][qt] * alpha[qt];
                c = mfma16(v0, pf[0][qt], c);
                oacc[et][qt] = mfma16(v1, pf[1][qt], c);
            }
        }
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int qa = qw0 + 16 * qt + li;
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

// =====================================================================================
// backward: delta, dK/dV (key-owned) and dQ (query-owned) over resident Q, K, V, dO
// =====================================================================================
constexpr int BW_STAT = 4 * IMG;              // lse * log2e [256] then delta [256] (fp32)
constexpr int BW_MSK = BW_STAT + 2 * RT * 4;  // keep bits
constexpr int BW_LDS = BW_MSK + MSKB;

// dK / dV for keys kw0 .. kw0 + 15 (one 16-key group): attention_d64.hip k_attn_dkdv_d64<16> body
__device__ __forceinline__ void res_dkdv16(int kw0, int T, int NT, const char* Qi, const char* Ki, const char* Vi,
                                           const char* Oi, const float* st_lse, const float* st_del, const char* Mi,
                                           bool has_mask, float scale_log2, float dscale, float scale, int lane,
                                           bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int64_t lddkv,
                                           int64_t boff, int h) {
    const int g = lane >> 4, li = lane & 15;
    sv8 kf[2], vf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        kf[s] = frag_rows<false>(Ki, kw0, s, lane);
        vf[s] = frag_rows<false>(Vi, kw0, s, lane);
    }
    fv4 dka[4], dva[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dka[i] = dva[i] = fv4{0.f, 0.f, 0.f, 0.f};
    const int key = kw0 + li;
    for (int q0 = (kw0 / 64) * 64; q0 < T; q0 += 64) {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int qr0 = q0 + 32 * half;
            if (qr0 + 31 < kw0) continue;
            fv4 z[2], ds[2];
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
                const int qb = qr0 + 16 * qt;
                const sv8 q0f = frag_rows<false>(Qi, qb, 0, lane), q1f = frag_rows<false>(Qi, qb, 1, lane);
                const sv8 o0f = frag_rows<false>(Oi, qb, 0, lane), o1f = frag_rows<false>(Oi, qb, 1, lane);
                fv4 sa = {0.f, 0.f, 0.f, 0.f}, pa = {0.f, 0.f, 0.f, 0.f};
                sa = mfma16(q0f, kf[0], sa);
                sa = mfma16(q1f, kf[1], sa);
                pa = mfma16(o0f, vf[0], pa);
                pa = mfma16(o1f, vf[1], pa);
                uint64_t keepbits = 0xFull;  // bit r -> keep(query qb + 4g + r, key kw0 + li)
                if (has_mask) {
                    const Words4 mw = lds_words(Mi + ((qb >> 4) * NT + (kw0 >> 4)) * 32);
                    const int w = li & 3;
                    const uint64_t bw = w == 0 ? mw.w[0] : (w == 1 ? mw.w[1] : (w == 2 ? mw.w[2] : mw.w[3]));
                    keepbits = 0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) keepbits |= ((bw >> ((4 * g + r) + 16 * (li >> 2))) & 1ull) << r;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int qa = qb + 4 * g + r;
                    const float p = key > qa ? 0.f : exp2f(sa[r] * scale_log2 - st_lse[qa]);
                    const bool kp = (keepbits >> r) & 1ull;
                    const float dp = kp ? pa[r] * dscale : 0.f;
                    z[qt][r] = kp ? p * dscale : 0.f;
                    ds[qt][r] = p * (dp - st_del[qa]);
                }
            }
            const sv8 zf = pack8(z[0], z[1]), dsf = pack8(ds[0], ds[1]);
#pragma unroll
            for (int et = 0; et < 4; ++et) {
                const sv8 oft = frag_tr<false>(Oi, qr0, 16 * et, lane);
                const sv8 qft = frag_tr<false>(Qi, qr0, 16 * et, lane);
                dva[et] = mfma16(oft, zf, dva[et]);
                dka[et] = mfma16(qft, dsf, dka[et]);
            }
        }
    }
    bf16_t* krow = dk + (boff + key) * lddkv + h * 64;
    bf16_t* vrow = dv + (boff + key) * lddkv + h * 64;
#pragma unroll
    for (int et = 0; et < 4; ++et) {
        const fv4 x = dka[et] * scale;
        const fv4 y = dva[et];
        *(uint2*)(krow + 16 * et + 4 * g) = make_uint2(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]));
        *(uint2*)(vrow + 16 * et + 4 * g) = make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
    }
}

// dQ for queries qw0 .. qw0 + 15: attention_d64.hip k_attn_dq_d64<16> body
__device__ __forceinline__ void res_dq16(int qw0, int NT, const char* Qi, const char* Ki, const char* Vi,
                                         const char* Oi, const float* st_lse, const float* st_del, const char* Mi,
                                         bool has_mask, float scale_log2, float dscale, float scale, int lane,
                                         bf16_t* __restrict__ dq, int64_t lddq, int64_t boff, int h) {
    const int g = lane >> 4, li = lane & 15;
    const sv8 qf0 = frag_rows<false>(Qi, qw0, 0, lane), qf1 = frag_rows<false>(Qi, qw0, 1, lane);
    const sv8 of0 = frag_rows<false>(Oi, qw0, 0, lane), of1 = frag_rows<false>(Oi, qw0, 1, lane);
    const int qa = qw0 + li;
    const float lq = st_lse[qa], dl = st_del[qa];
    fv4 dqacc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dqacc[i] = fv4{0.f, 0.f, 0.f, 0.f};
    const int nkv = (qw0 + 15) / 64 + 1;
    for (int kv = 0; kv < nkv; ++kv) {
        const int k0 = kv * 64;
        fv4 sa[4], pa[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const sv8 k0f = frag_rows<false>(Ki, k0 + 16 * kt, 0, lane), k1f = frag_rows<false>(Ki, k0 + 16 * kt, 1, lane);
            const sv8 v0f = frag_rows<false>(Vi, k0 + 16 * kt, 0, lane), v1f = frag_rows<false>(Vi, k0 + 16 * kt, 1, lane);
            fv4 c = {0.f, 0.f, 0.f, 0.f};
            c = mfma16(k0f, qf0, c);
            sa[kt] = mfma16(k1f, qf1, c);
            fv4 d = {0.f, 0.f, 0.f, 0.f};
            d = mfma16(v0f, of0, d);
            pa[kt] = mfma16(v1f, of1, d);
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            Words4 mw;
            if (has_mask) mw = lds_words(Mi + ((qw0 >> 4) * NT + kv * 4 + kt) * 32);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = k0 + 16 * kt + 4 * g + r;
                const float p = key > qa ? 0.f : exp2f(sa[kt][r] * scale_log2 - lq);
                float dp = pa[kt][r];
                if (has_mask) dp = ((mw.w[r] >> lane) & 1ull) ? dp * dscale : 0.f;
                sa[kt][r] = p * (dp - dl);
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const sv8 dsf = pack8(sa[2 * u], sa[2 * u + 1]);
#pragma unroll
            for (int et = 0; et < 4; ++et) {
                const sv8 kf = frag_tr<false>(Ki, k0 + 32 * u, 16 * et, lane);
                dqacc[et] = mfma16(kf, dsf, dqacc[et]);
            }
        }
    }
    bf16_t* row = dq + (boff + qa) * lddq + h * 64;
#pragma unroll
    for (int et = 0; et < 4; ++et) {
        const fv4 x = dqacc[et] * scale;
        *(uint2*)(row + 16 * et + 4 * g) = make_uint2(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]));
    }
}

__global__ __launch_bounds__(512, 2) void k_attn_bwd_res(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                        const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                        int64_t ld, const bf16_t* __restrict__ o, int64_t ldo,
                                                        const bf16_t* __restrict__ dout, int64_t ldd,
                                                        const float* __restrict__ lse, bf16_t* __restrict__ dq,
                                                        bf16_t* __restrict__ dk, bf16_t* __restrict__ dv,
                                                        int64_t lddqkv, float scale,
                                                        const uint64_t* __restrict__ mask, float dscale) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qi = smem;
    char* Ki = smem + IMG;
    char* Vi = smem + 2 * IMG;
    char* Oi = smem + 3 * IMG;                      // dO image
    float* st_lse = (float*)(smem + BW_STAT);
    float* st_del = st_lse + RT;
    char* Mi = smem + BW_MSK;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bh = blockIdx.x, b = bh / H, h = bh % H;
    const int T = (int)T_, NT = T >> 4;
    const int64_t boff = (int64_t)b * T_;
    const float scale_log2 = scale * LOG2E;
    load_image<false>(q + boff * ld + h * 64, ld, T, Qi, tid);
    load_image<false>(k + boff * ld + h * 64, ld, T, Ki, tid);
    load_image<false>(v + boff * ld + h * 64, ld, T, Vi, tid);
    load_image<false>(dout + boff * ldd + h * 64, ldd, T, Oi, tid);
    if (mask) load_mask(mask, bh, NT, Mi, tid);
    // lse (log2 domain) and delta = rowsum(dO * O): 2 threads per row, 32 elements each
    if (tid < 2 * T) {
        const int r = tid >> 1, hf = tid & 1;
        const bf16_t* orow = o + (boff + r) * ldo + h * 64 + 32 * hf;
        const bf16_t* drow = dout + (boff + r) * ldd + h * 64 + 32 * hf;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint4 a = *(const uint4*)(orow + 8 * c), d = *(const uint4*)(drow + 8 * c);
            const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                s += __uint_as_float(aw[e] << 16) * __uint_as_float(dw[e] << 16);
                s += __uint_as_float(aw[e] & 0xffff0000u) * __uint_as_float(dw[e] & 0xffff0000u);
            }
        }
        s += __shfl_xor(s, 1, 64);
        if (hf == 0) {
            st_del[r] = s;
            st_lse[r] = lse[(int64_t)bh * T_ + r] * LOG2E;
        }
    }
    __syncthreads();
    const bool has_mask = mask != nullptr;
    // key-owned dK/dV for keys [32 wave, +32), then query-owned dQ for queries [32 wave, +32)
    if (32 * wave < T) {
#pragma unroll 1
        for (int g16 = 0; g16 < 2; ++g16)
            res_dkdv16(32 * wave + 16 * g16, T, NT, Qi, Ki, Vi, Oi, st_lse, st_del, Mi, has_mask, scale_log2, dscale,
                       scale, lane, dk, dv, lddqkv, boff, h);
#pragma unroll 1
        for (int g16 = 0; g16 < 2; ++g16)
            res_dq16(32 * wave + 16 * g16, NT, Qi, Ki, Vi, Oi, st_lse, st_del, Mi, has_mask, scale_log2, dscale, scale,
                     lane, dq, lddqkv, boff, h);
    }
}

}  // namespace

namespace attn {
bool res_ok(int64_t T) { return T % 64 == 0 && T <= RT && (g_attn_variant & 8); }

void launch_fwd_res(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st) {
    const float ds = d.mask ? d.dscale : 1.f;
    k_attn_fwd_res<<<(unsigned)(B * H), 512, 2 * IMG + MSKB, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E,
                                                                  d.mask, ds);
}

void launch_bwd_res(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, bf16_t* dq,
                    bf16_t* dk, bf16_t* dv, int64_t lddqkv, float scale, const DropArgs& d, hipStream_t st) {
    const float ds = d.mask ? d.dscale : 1.f;
    k_attn_bwd_res<<<(unsigned)(B * H), 512, BW_LDS, st>>>(T, H, q, k, v, ld, o, ldo, dout, ldd, lse, dq, dk, dv,
                                                          lddqkv, scale, d.mask, ds);
}
}  // namespace attn

}  // namespace cg
