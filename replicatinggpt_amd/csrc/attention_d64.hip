// charpt: bf16 MFMA causal attention for head_size 64 (the C2/C4 perf path of Head.forward x
// n_head, GPT1.py:109-123,134-135) -- forward, dQ and dK/dV kernels.
//
// All three kernels stream 64-row tiles (K/V for the query-block kernels, Q/dO for dK/dV)
// through a double-buffered LDS ring: the next tile's global loads are issued into registers
// before the current tile's MFMAs and written to the other LDS stage after them (one barrier per
// tile), so load latency hides under compute.  Dropout keep bits (k_attn_dropmask) are staged
// with each tile and read from LDS with uniform-address loads.
//
// Layouts (16x16x32 bf16 MFMA, lane l: A/B fragment rows l&15, k = 8(l>>4)..+7; C col = l&15,
// row = 4(l>>4) + r):
//  * forward / dQ: swapped S^T = K Q^T -- the query is the C column, so softmax statistics are
//    lane-local; P^T (bf16) is directly the B operand of O^T = V^T P^T, and dS^T of dQ^T = K^T dS^T
//    (V / K read with ds_read_b64_tr_b16 in the matching key order).
//  * dK/dV: S = Q K^T -- the key is the C column; Z (= dropped P) and dS are the B operands of
//    dV^T = dO^T Z and dK^T = Q^T dS.
// QW / KW (queries / keys per wave, 16 or 32) trade registers (occupancy) for reuse.
#include "attention_tile.h"

namespace cg {
int g_attn_variant = 0;

namespace {
using namespace atile;

// keep-bit rows for a (QROWS*16)-query block x 64-key tile: [QROWS q16][4 k16][32 B], 16 B per thread
template <int QROWS>
__device__ __forceinline__ uint4 qmask_load(const uint64_t* mask, int bh, int NT, int q16_0, int k16_0, int tid) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (mask && tid < QROWS * 8) {
        const int row = tid >> 3, c = tid & 7;
        if (q16_0 + row < NT) v = *(const uint4*)((const char*)mask_tile(mask, bh, NT, q16_0 + row, k16_0) + c * 16);
    }
    return v;
}

// =====================================================================================
// forward: block = 4 waves x QW queries, KV tiles of 64 keys
// =====================================================================================
template <int QW>
__global__ __launch_bounds__(256, QW == 16 ? 3 : 2) void k_attn_fwd_d64(
    int64_t T_, int H, const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    int64_t ld, bf16_t* __restrict__ o, int64_t ldo, float* __restrict__ lse, float scale_log2,
    const uint64_t* __restrict__ mask, float dscale) {
    constexpr int QT = QW / 16, FQ = 4 * QW, QROWS = FQ / 16;
    constexpr int MB = QROWS * 128;  // keep-bit bytes per stage
    constexpr int STG = 2 * TILE + MB;
    __shared__ __attribute__((aligned(16))) char smem[2 * STG];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    int xblk, bh;
    block_coords<true>(xblk, bh);
    const int b = bh / H, h = bh % H;
    const int NT = (int)(T_ >> 4);
    const int64_t qblk0 = (int64_t)xblk * FQ;
    const int64_t qw0 = qblk0 + wave * QW;
    const int64_t boff = (int64_t)b * T_;
    const bf16_t* kb_ = k + boff * ld + h * 64;
    const bf16_t* vb_ = v + boff * ld + h * 64;
    const bool wave_active = qw0 < T_;

    sv8 qf[QT][2];  // Q^T as B operand: lane holds Q[qw0 + 16qt + li][32s + 8g ..]
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
            qf[qt][s] = wave_active ? *(const sv8*)(q + (boff + qw0 + 16 * qt + li) * ld + h * 64 + 32 * s + 8 * g) : sv8{};

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

    const int64_t qlast = (qblk0 + FQ - 1) < (T_ - 1) ? (qblk0 + FQ - 1) : (T_ - 1);
    const int nkv = (int)(qlast / 64) + 1;
    const int q16_0 = (int)(qblk0 >> 4);
    {
        const Tile2 kt = tile_load(kb_, ld, 0, tid), vt = tile_load(vb_, ld, 0, tid);
        const uint4 mt = qmask_load<QROWS>(mask, bh, NT, q16_0, 0, tid);
        tile_store<false>(kt, smem, tid);
        tile_store<true>(vt, smem + TILE, tid);
        if (tid < QROWS * 8) *(uint4*)(smem + 2 * TILE + tid * 16) = mt;
    }
    __syncthreads();
    for (int kv = 0; kv < nkv; ++kv) {
        const int nxt = kv + 1 < nkv ? kv + 1 : kv;
        const Tile2 kn = tile_load(kb_, ld, (int64_t)nxt * 64, tid), vn = tile_load(vb_, ld, (int64_t)nxt * 64, tid);
        const uint4 mn = qmask_load<QROWS>(mask, bh, NT, q16_0, nxt * 4, tid);
        const char* S = smem + (kv & 1) * STG;
        const int64_t k0 = (int64_t)kv * 64;
        if (wave_active && k0 <= qw0 + QW - 1) {
            const char* Ki = S;
            const char* Vi = S + TILE;
            fv4 sacc[4][QT];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                const sv8 a0 = frag_rows<false>(Ki, 16 * kt, 0, lane), a1 = frag_rows<false>(Ki, 16 * kt, 1, lane);
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
                // raw scores; the scale is applied inside the exponent's fma (max commutes with
                // the positive scale, and the rounding is monotone: same max as scaling first)
                const int qa = (int)(qw0 + 16 * qt) + li, kb = (int)k0 + 4 * g;
                float mx = -INFINITY;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float x = sacc[kt][qt][r];
                        if (diag && kb + 16 * kt + r > qa) x = -INFINITY;
                        sacc[kt][qt][r] = x;
                        mx = fmaxf(mx, x);
                    }
                mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
                mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
                const float m_new = fmaxf(m_run[qt], mx * scale_log2);
                alpha[qt] = __builtin_amdgcn_exp2f(m_run[qt] - m_new);
                float ls = 0.f;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    Words4 mw = {{~0ull, ~0ull, ~0ull, ~0ull}};  // no dropout: keep everything, no branch
                    if (mask) mw = lds_words(S + 2 * TILE + ((wave * QT + qt) * 4 + kt) * 32);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        // exp2 of the raw hardware instruction: results below 2^-126 (weights that
                        // vanish against the row max) flush to 0 instead of going denormal
                        const float p = __builtin_amdgcn_exp2f(fmaf(sacc[kt][qt][r], scale_log2, -m_new));
                        ls += p;
                        // 1/(1-p) of the kept weights is applied once, in the epilogue
                        sacc[kt][qt][r] = keep_sel(mw.w[r], p);
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
                const sv8 v0 = frag_tr<true>(Vi, 0, 16 * et, lane), v1 = frag_tr<true>(Vi, 32, 16 * et, lane);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    fv4 c = oacc[et][qt] * alpha[qt];
                    c = mfma16(v0, pf[0][qt], c);
                    oacc[et][qt] = mfma16(v1, pf[1][qt], c);
                }
            }
        }
        char* D = smem + ((kv + 1) & 1) * STG;
        tile_store<false>(kn, D, tid);
        tile_store<true>(vn, D + TILE, tid);
        if (tid < QROWS * 8) *(uint4*)(D + 2 * TILE + tid * 16) = mn;
        __syncthreads();
    }
    if (!wave_active) return;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int64_t qa = qw0 + 16 * qt + li;
        if (qa >= T_) continue;
        const float inv = dscale / l_run[qt];
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
// dQ: S^T = K Q^T, dP^T = V dO^T, dS^T = P^T (keep/(1-p) dP^T - delta), dQ^T += K^T dS^T
// =====================================================================================
template <int QW>
__global__ __launch_bounds__(256, QW == 16 ? 3 : 2) void k_attn_dq_d64(
    int64_t T_, int H, const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    int64_t ld, const bf16_t* __restrict__ o, int64_t ldo, const bf16_t* __restrict__ dout, int64_t ldd,
    const float* __restrict__ lse, float* __restrict__ delta, bf16_t* __restrict__ dq, int64_t lddq, float scale,
    const uint64_t* __restrict__ mask, float dscale) {
    constexpr int QT = QW / 16, FQ = 4 * QW, QROWS = FQ / 16;
    constexpr int MB = QROWS * 128;
    constexpr int STG = 2 * TILE + MB;
    __shared__ __attribute__((aligned(16))) char smem[2 * STG];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    int xblk, bh;
    block_coords<true>(xblk, bh);
    const int b = bh / H, h = bh % H;
    const int NT = (int)(T_ >> 4);
    const int64_t qblk0 = (int64_t)xblk * FQ;
    const int64_t qw0 = qblk0 + wave * QW;
    const int64_t boff = (int64_t)b * T_;
    const bool wave_active = qw0 < T_;
    const float scale_log2 = scale * LOG2E;

    sv8 qf[QT][2], of[QT][2];
    float lq[QT], dl[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int64_t qrow = qw0 + 16 * qt + li;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            qf[qt][s] = wave_active ? *(const sv8*)(q + (boff + qrow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
            of[qt][s] = wave_active ? *(const sv8*)(dout + (boff + qrow) * ldd + h * 64 + 32 * s + 8 * g) : sv8{};
        }
        lq[qt] = wave_active ? lse[(int64_t)bh * T_ + qrow] * LOG2E : 0.f;
        // delta = rowsum(dO * O) (dropout-invariant: O already holds the dropped P); lane group g
        // holds elements 32s + 8g .. +7 of the row: reduce over s in-lane, then across g
        float dsum = 0.f;
        if (wave_active) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const uint4 ov = *(const uint4*)(o + (boff + qrow) * ldo + h * 64 + 32 * s + 8 * g);
                const sv8 dv8 = of[qt][s];
                const uint32_t ow[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    dsum += __uint_as_float(ow[e] << 16) * __uint_as_float(((uint32_t)(uint16_t)dv8[2 * e]) << 16);
                    dsum += __uint_as_float(ow[e] & 0xffff0000u) *
                            __uint_as_float(((uint32_t)(uint16_t)dv8[2 * e + 1]) << 16);
                }
            }
        }
        dsum += __shfl_xor(dsum, 16, 64);
        dsum += __shfl_xor(dsum, 32, 64);
        dl[qt] = dsum;
        if (wave_active && g == 0) delta[(int64_t)bh * T_ + qrow] = dsum;
    }
    fv4 dqacc[4][QT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < QT; ++j) dqacc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* kb_ = k + boff * ld + h * 64;
    const bf16_t* vb_ = v + boff * ld + h * 64;
    const int64_t qlast = (qblk0 + FQ - 1) < (T_ - 1) ? (qblk0 + FQ - 1) : (T_ - 1);
    const int nkv = (int)(qlast / 64) + 1;
    const int q16_0 = (int)(qblk0 >> 4);
    {
        const Tile2 kt = tile_load(kb_, ld, 0, tid), vt = tile_load(vb_, ld, 0, tid);
        const uint4 mt = qmask_load<QROWS>(mask, bh, NT, q16_0, 0, tid);
        tile_store<false>(kt, smem, tid);
        tile_store<false>(vt, smem + TILE, tid);
        if (tid < QROWS * 8) *(uint4*)(smem + 2 * TILE + tid * 16) = mt;
    }
    __syncthreads();
    for (int kv = 0; kv < nkv; ++kv) {
        const int nxt = kv + 1 < nkv ? kv + 1 : kv;
        const Tile2 kn = tile_load(kb_, ld, (int64_t)nxt * 64, tid), vn = tile_load(vb_, ld, (int64_t)nxt * 64, tid);
        const uint4 mn = qmask_load<QROWS>(mask, bh, NT, q16_0, nxt * 4, tid);
        const char* S = smem + (kv & 1) * STG;
        const int64_t k0 = (int64_t)kv * 64;
        if (wave_active && k0 <= qw0 + QW - 1) {
            const char* Ki = S;
            const char* Vi = S + TILE;
            fv4 sa[4][QT], pa[4][QT];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                const sv8 k0f = frag_rows<false>(Ki, 16 * kt, 0, lane), k1f = frag_rows<false>(Ki, 16 * kt, 1, lane);
                const sv8 v0f = frag_rows<false>(Vi, 16 * kt, 0, lane), v1f = frag_rows<false>(Vi, 16 * kt, 1, lane);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    fv4 c = {0.f, 0.f, 0.f, 0.f};
                    c = mfma16(k0f, qf[qt][0], c);
                    sa[kt][qt] = mfma16(k1f, qf[qt][1], c);
                    fv4 d = {0.f, 0.f, 0.f, 0.f};
                    d = mfma16(v0f, of[qt][0], d);
                    pa[kt][qt] = mfma16(v1f, of[qt][1], d);
                }
            }
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int qa = (int)(qw0 + 16 * qt) + li, kb = (int)k0 + 4 * g;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    Words4 mw = {{~0ull, ~0ull, ~0ull, ~0ull}};  // no dropout: keep everything, no branch
                    if (mask) mw = lds_words(S + 2 * TILE + ((wave * QT + qt) * 4 + kt) * 32);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float p = kb + 16 * kt + r > qa
                                            ? 0.f
                                            : __builtin_amdgcn_exp2f(fmaf(sa[kt][qt][r], scale_log2, -lq[qt]));
                        float dp = pa[kt][qt][r];
                        dp = keep_sel(mw.w[r], dp * dscale);  // dscale is 1 without dropout
                        sa[kt][qt][r] = p * (dp - dl[qt]);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                sv8 dsf[QT];
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) dsf[qt] = pack8(sa[2 * u][qt], sa[2 * u + 1][qt]);
#pragma unroll
                for (int et = 0; et < 4; ++et) {
                    const sv8 kf = frag_tr<false>(Ki, 32 * u, 16 * et, lane);
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) dqacc[et][qt] = mfma16(kf, dsf[qt], dqacc[et][qt]);
                }
            }
        }
        char* D = smem + ((kv + 1) & 1) * STG;
        tile_store<false>(kn, D, tid);
        tile_store<false>(vn, D + TILE, tid);
        if (tid < QROWS * 8) *(uint4*)(D + 2 * TILE + tid * 16) = mn;
        __syncthreads();
    }
    if (!wave_active) return;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
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

// =====================================================================================
// dK / dV: block = 4 waves x KW keys; stream 64-query tiles (Q, dO, lse, delta, keep bits)
// =====================================================================================
template <int KW>
__global__ __launch_bounds__(256, KW == 16 ? 2 : 1) void k_attn_dkdv_d64(
    int64_t T_, int H, const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    int64_t ld, const bf16_t* __restrict__ dout, int64_t ldd, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int64_t lddkv, float scale,
    const uint64_t* __restrict__ mask, float dscale) {
    constexpr int KT = KW / 16, FK = 4 * KW, K16 = FK / 16;  // key tiles per block
    constexpr int CPR = K16 * 2;                             // 16-B keep-bit chunks per q16 row
    constexpr int STAT = 2 * TILE;                           // lse*log2e [64] then delta [64]
    constexpr int MSK = 2 * TILE + 512;                      // keep bits [4 q16][K16][32 B]
    constexpr int STG = MSK + 4 * K16 * 32;
    __shared__ __attribute__((aligned(16))) char smem[2 * STG];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    int xblk, bh;
    block_coords<false>(xblk, bh);
    const int b = bh / H, h = bh % H;
    const int NT = (int)(T_ >> 4);
    const int64_t kblk0 = (int64_t)xblk * FK;
    const int64_t kw0 = kblk0 + wave * KW;
    const int64_t boff = (int64_t)b * T_;
    const bool wave_active = kw0 < T_;
    const float scale_log2 = scale * LOG2E;
    const int k16_0 = (int)(kblk0 >> 4);

    sv8 kf[KT][2], vf[KT][2];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int64_t krow = kw0 + 16 * kt + li;
            kf[kt][s] = wave_active ? *(const sv8*)(k + (boff + krow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
            vf[kt][s] = wave_active ? *(const sv8*)(v + (boff + krow) * ld + h * 64 + 32 * s + 8 * g) : sv8{};
        }
    fv4 dka[4][KT], dva[4][KT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < KT; ++j) dka[i][j] = dva[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* qb_ = q + boff * ld + h * 64;
    const bf16_t* ob_ = dout + boff * ldd + h * 64;
    const int nq = (int)(T_ / 64);
    const int q_start = (int)(kblk0 / 64);

    struct QStage {
        Tile2 qt, ot;
        float stat;
        uint4 msk;
    };
    auto qload = [&](int qtile) {
        QStage s;
        s.qt = tile_load(qb_, ld, (int64_t)qtile * 64, tid);
        s.ot = tile_load(ob_, ldd, (int64_t)qtile * 64, tid);
        s.stat = 0.f;
        if (tid < 64) s.stat = lse[(int64_t)bh * T_ + (int64_t)qtile * 64 + tid] * LOG2E;
        else if (tid < 128) s.stat = delta[(int64_t)bh * T_ + (int64_t)qtile * 64 + tid - 64];
        s.msk = make_uint4(0, 0, 0, 0);
        if (mask && tid >= 128 && tid < 128 + 4 * CPR) {
            const int row = (tid - 128) / CPR, c = (tid - 128) % CPR;
            if (k16_0 + (c >> 1) < NT)
                s.msk = *(const uint4*)((const char*)mask_tile(mask, bh, NT, qtile * 4 + row, k16_0) + c * 16);
        }
        return s;
    };
    auto qstore = [&](const QStage& s, char* D) {
        tile_store<false>(s.qt, D, tid);
        tile_store<false>(s.ot, D + TILE, tid);
        if (tid < 128) ((float*)(D + STAT))[tid] = s.stat;
        else if (tid < 128 + 4 * CPR) *(uint4*)(D + MSK + (tid - 128) * 16) = s.msk;
    };
    qstore(qload(q_start), smem);
    __syncthreads();
    for (int qtile = q_start; qtile < nq; ++qtile) {
        const int it = qtile - q_start;
        const QStage nxt = qload(qtile + 1 < nq ? qtile + 1 : qtile);
        const char* S = smem + (it & 1) * STG;
        const int64_t q0 = (int64_t)qtile * 64;
        if (wave_active && q0 + 63 >= kw0) {
            const char* Qi = S;
            const char* Oi = S + TILE;
            const float* st_lse = (const float*)(S + STAT);
            const float* st_del = st_lse + 64;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int qr0 = 32 * half;
                if (q0 + qr0 + 31 < kw0) continue;
                sv8 zf[KT], dsf[KT];
#pragma unroll
                for (int kt = 0; kt < KT; ++kt) {
                    const int key = (int)kw0 + 16 * kt + li;
                    fv4 z[2], ds[2];
#pragma unroll
                    for (int qt = 0; qt < 2; ++qt) {
                        const sv8 q0f = frag_rows<false>(Qi, qr0 + 16 * qt, 0, lane);
                        const sv8 q1f = frag_rows<false>(Qi, qr0 + 16 * qt, 1, lane);
                        const sv8 o0f = frag_rows<false>(Oi, qr0 + 16 * qt, 0, lane);
                        const sv8 o1f = frag_rows<false>(Oi, qr0 + 16 * qt, 1, lane);
                        fv4 sa = {0.f, 0.f, 0.f, 0.f}, pa = {0.f, 0.f, 0.f, 0.f};
                        sa = mfma16(q0f, kf[kt][0], sa);
                        sa = mfma16(q1f, kf[kt][1], sa);
                        pa = mfma16(o0f, vf[kt][0], pa);
                        pa = mfma16(o1f, vf[kt][1], pa);
                        uint64_t keepbits = 0xFull;  // bit r -> keep(query 4g + r, key li)
                        if (mask) {
                            const Words4 mw = lds_words(S + MSK + ((half * 2 + qt) * K16 + wave * KT + kt) * 32);
                            const int w = li & 3;
                            const uint64_t bw = w == 0 ? mw.w[0] : (w == 1 ? mw.w[1] : (w == 2 ? mw.w[2] : mw.w[3]));
                            keepbits = 0;
#pragma unroll
                            for (int r = 0; r < 4; ++r) keepbits |= ((bw >> ((4 * g + r) + 16 * (li >> 2))) & 1ull) << r;
                        }
                        const int qb = (int)q0 + qr0 + 16 * qt + 4 * g;
                        const float4 lse4 = *(const float4*)(st_lse + qr0 + 16 * qt + 4 * g);
                        const float4 del4 = *(const float4*)(st_del + qr0 + 16 * qt + 4 * g);
                        const float lsev[4] = {lse4.x, lse4.y, lse4.z, lse4.w};
                        const float delv[4] = {del4.x, del4.y, del4.z, del4.w};
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float p = key > qb + r ? 0.f : __builtin_amdgcn_exp2f(fmaf(sa[r], scale_log2, -lsev[r]));
                            const bool kp = (keepbits >> r) & 1ull;
                            const float dp = kp ? pa[r] * dscale : 0.f;
                            z[qt][r] = kp ? p : 0.f;   // 1/(1-p) of dV applied in the epilogue
                            ds[qt][r] = p * (dp - delv[r]);
                        }
                    }
                    zf[kt] = pack8(z[0], z[1]);
                    dsf[kt] = pack8(ds[0], ds[1]);
                }
#pragma unroll
                for (int et = 0; et < 4; ++et) {
                    const sv8 oft = frag_tr<false>(Oi, qr0, 16 * et, lane);
                    const sv8 qft = frag_tr<false>(Qi, qr0, 16 * et, lane);
#pragma unroll
                    for (int kt = 0; kt < KT; ++kt) {
                        dva[et][kt] = mfma16(oft, zf[kt], dva[et][kt]);
                        dka[et][kt] = mfma16(qft, dsf[kt], dka[et][kt]);
                    }
                }
            }
        }
        qstore(nxt, smem + ((it + 1) & 1) * STG);
        __syncthreads();
    }
    if (!wave_active) return;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
        const int64_t key = kw0 + 16 * kt + li;
        if (key >= T_) continue;
        bf16_t* krow = dk + (boff + key) * lddkv + h * 64;
        bf16_t* vrow = dv + (boff + key) * lddkv + h * 64;
#pragma unroll
        for (int et = 0; et < 4; ++et) {
            const fv4 x = dka[et][kt] * scale;
            const fv4 y = dva[et][kt] * dscale;
            *(uint2*)(krow + 16 * et + 4 * g) = make_uint2(pack_bf2(x[0], x[1]), pack_bf2(x[2], x[3]));
            *(uint2*)(vrow + 16 * et + 4 * g) = make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
        }
    }
}

// variant bits: 1 -> forward/dQ with 32 queries per wave; 2 -> dK/dV with 32 keys per wave;
// 8 -> the whole-(b, h)-resident kernels where they apply (attention_res.hip)
inline int qw_of() { return (g_attn_variant & 1) ? 32 : 16; }
inline int kw_of() { return (g_attn_variant & 2) ? 32 : 16; }

}  // namespace

namespace attn {
void launch_fwd_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st) {
    const float ds = d.mask ? d.dscale : 1.f;
    if (qw_of() == 32)
        k_attn_fwd_d64<32><<<dim3(ceil_div(T, 128), (unsigned)(B * H)), 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse,
                                                                                     scale * LOG2E, d.mask, ds);
    else
        k_attn_fwd_d64<16><<<dim3(ceil_div(T, 64), (unsigned)(B * H)), 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse,
                                                                                    scale * LOG2E, d.mask, ds);
}
void launch_dq_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                   const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, float* delta,
                   bf16_t* dq, int64_t lddq, float scale, const DropArgs& d, hipStream_t st) {
    const float ds = d.mask ? d.dscale : 1.f;
    if (qw_of() == 32)
        k_attn_dq_d64<32><<<dim3(ceil_div(T, 128), (unsigned)(B * H)), 256, 0, st>>>(
            T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, d.mask, ds);
    else
        k_attn_dq_d64<16><<<dim3(ceil_div(T, 64), (unsigned)(B * H)), 256, 0, st>>>(
            T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, d.mask, ds);
}
void launch_dkdv_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                     const bf16_t* dout, int64_t ldd, const float* lse, const float* delta, bf16_t* dk, bf16_t* dv,
                     int64_t lddkv, float scale, const DropArgs& d, hipStream_t st) {
    const float ds = d.mask ? d.dscale : 1.f;
    if (kw_of() == 32)
        k_attn_dkdv_d64<32><<<dim3(ceil_div(T, 128), (unsigned)(B * H)), 256, 0, st>>>(
            T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale, d.mask, ds);
    else
        k_attn_dkdv_d64<16><<<dim3(ceil_div(T, 64), (unsigned)(B * H)), 256, 0, st>>>(
            T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale, d.mask, ds);
}
}  // namespace attn

}  // namespace cg
