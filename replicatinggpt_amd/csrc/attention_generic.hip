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

#include <type_traits>

#include "attention_common.h"
#include "ln_fwd.h"

using namespace cg;

namespace {


// Keep bits of the MFMA kernels (attention_common.h: FWD and BWD tiles).  One wave per 64x64
// (query tile QT, key tile KT <= QT) region, DM_TPW regions per wave: its four 32x32 sub-blocks
// (qs, ks) give FWD tiles (2 QT + qs, KT) and BWD tiles (2 KT + ks, QT) whole.  Per sub-block, lane
// l = 32 h + i takes query 32 qs + sig(i) -- sig(i) = (i & 3) + 8 ((i >> 2) & 3) + 4 (i >> 4), a lane
// order chosen for the BWD words below -- and keys 32 ks + 16 h .. +15: two Philox calls, 16
// decisions, each made by one packed saturating u16 add (or subtract, thr > 2^15) whose top bit is
// the decision and one packed shift.  A lane gathers its 32 decisions of sub-block row qs into one
// word R (bit 8 ks + 4 (w >> 1) + 2 c + (w & 1) + 16 e for call c, Philox word w, half e), an order in
// which
//   FWD: the lane's own decisions already sit at their FWD bits and its lane^32 partner's sit 4 bits
//        off: one v_permlane32_swap, one rotate and one v_bfi_b32 make the FWD word (stored at the
//        lane of query sig(i));
//   BWD: a 32x32 bit transpose inside each half-wave (five butterfly stages: one lane exchange, one
//        rotate, one v_bfi_b32 each) gives lane 32 h + j the column j of R over the 32 queries in
//        sig order, which makes every BWD lane's 16 query bits contiguous: one ds_bpermute and one
//        v_bfe_u32 per (qs, ks).
// (The round-2 form spent ~880 of its ~1200 instructions per region on keep8_bits compares, nibble
// assembly and an LDS transpose; Philox itself -- 19 v_mad_u64_u32 per call -- is what remains.)
constexpr int DM_TPW = 2;
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// keep decisions of the two u16 halves of a Philox word as bits 0 and 16: u >= thr <=> the top bit of
// sat(u + (2^15 - thr)) (thr <= 2^15) or of sat(u - (thr - 2^15)) (thr > 2^15)
template <bool SUBF>
__device__ __forceinline__ uint32_t keep2(uint32_t w, us2 k) {
    const us2 u = __builtin_bit_cast(us2, w);
    const us2 t = SUBF ? __builtin_elementwise_sub_sat(u, k) : __builtin_elementwise_add_sat(u, k);
    return __builtin_bit_cast(uint32_t, (us2)(t >> (us2)15));
}

// block `bid` (256 threads) of the keep-bit generation: regions (bid * 4 + wave) * DM_TPW ..
template <bool SUBF>
__device__ __forceinline__ void dropmask_block(int64_t T_, int64_t nbh, uint32_t* __restrict__ mask_f,
                                               uint32_t* __restrict__ mask_b, const DropArgs& d, int bid) {
    const int NB = (int)(T_ >> 5), NP = NB >> 1;
    const int64_t nreg = (int64_t)NP * (NP + 1) / 2, ntile = mask_tiles(T_);
    const int64_t total = nbh * nreg;
    const int lane = threadIdx.x & 63, h = lane >> 5, lq = lane & 31, w = threadIdx.x >> 6;
    const int qsig = (lq & 3) + 8 * ((lq >> 2) & 3) + 4 * (lq >> 4);
    const uint64_t stream = dropout_stream(d.rng_call, d.site);
    const uint16_t kc = (uint16_t)(SUBF ? d.thr - 0x8000u : 0x8000u - d.thr);
    const us2 K = us2{kc, kc};
    const int64_t first = ((int64_t)bid * 4 + w) * DM_TPW;
    if (first >= total) return;
    // butterfly stage j = 16 >> t: lanes with bit j clear keep the low blocks (mask m_j) and take their
    // partner's low blocks into the high ones (rotate right by 32 - j), the others the reverse
    uint32_t bmask[5], brot[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int j = 16 >> t;
        const uint32_t m = t == 0 ? 0x0000FFFFu : t == 1 ? 0x00FF00FFu : t == 2 ? 0x0F0F0F0Fu : t == 3 ? 0x33333333u : 0x55555555u;
        const bool lo = (lane & j) == 0;
        bmask[t] = lo ? m : ~m;
        brot[t] = lo ? (uint32_t)(32 - j) : (uint32_t)j;
    }
    // BWD gather source: column j of R (key lq of the sub-block) in half-wave lq >> 4
    const int kk = lq;
    const int jcol = 16 * (kk & 1) + 4 * ((kk >> 2) & 1) + 2 * ((kk >> 3) & 1) + ((kk >> 1) & 1);
    const int src0 = 32 * (kk >> 4) + jcol;   // + 8 ks
    const uint32_t fmask = h ? 0xF0F0F0F0u : 0x0F0F0F0Fu, frot = h ? 4u : 28u;
    uint64_t bh = (uint64_t)(first / nreg);
    const int r0 = (int)(first - (int64_t)bh * nreg);
    int QT = (int)((sqrtf(8.f * r0 + 1.f) - 1.f) * 0.5f);
    while ((QT + 1) * (QT + 2) / 2 <= r0) ++QT;
    while (QT * (QT + 1) / 2 > r0) --QT;
    int KT = r0 - QT * (QT + 1) / 2;
#pragma unroll 1
    for (int i = 0; i < DM_TPW; ++i) {
        if (first + i >= total) return;
        if (i && ++KT > QT) {
            KT = 0;
            if (++QT == NP) {
                QT = 0;
                ++bh;
            }
        }
        uint32_t R[2] = {0u, 0u};
        // Philox group of (query 64 QT + 32 qs + sig, keys 64 KT + 32 ks + 16 h + 8 c ..): g0 + 4 T qs + 4 ks + c
        const uint64_t g0 = ((bh * (uint64_t)T_ + (uint64_t)(64 * QT + qsig)) * (uint64_t)T_ + (uint64_t)(64 * KT + 16 * h)) >> 3;
#pragma unroll
        for (int qs = 0; qs < 2; ++qs)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const uint64_t grp = g0 + (uint64_t)(4 * T_ * qs + 4 * ks);
                // (the sub-block above the diagonal is computed too -- branch-free -- and zeroed below)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const u32x4 r = philox_group(d.seed, stream, grp + c);
                    const int b0 = 8 * ks + 2 * c;
                    R[qs] |= keep2<SUBF>(r.x, K) << b0;
                    R[qs] |= keep2<SUBF>(r.y, K) << (b0 + 1);
                    R[qs] |= keep2<SUBF>(r.z, K) << (b0 + 4);
                    R[qs] |= keep2<SUBF>(r.w, K) << (b0 + 5);
                }
            }
        if (QT == KT) R[0] &= 0x00FF00FFu;   // sub-block (0, 1) wholly above the diagonal: zero bits
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) {
            const auto sw = __builtin_amdgcn_permlane32_swap(R[qs], R[qs], false, false);
            const uint32_t part = h ? sw[0] : sw[1];
            const uint32_t rp = __builtin_amdgcn_alignbit(part, part, frot);
            mask_f[((int64_t)bh * ntile + mask_fwd_tile(2 * QT + qs, KT)) * 64 + 32 * h + qsig] =
                (R[qs] & fmask) | (rp & ~fmask);
        }
        uint32_t W[2];
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) {
            uint32_t x = R[qs];
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                const uint32_t y = (uint32_t)__shfl_xor((int)x, 16 >> t, 64);
                const uint32_t ry = __builtin_amdgcn_alignbit(y, y, brot[t]);
                x = (x & bmask[t]) | (ry & ~bmask[t]);
            }
            W[qs] = x;
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const uint32_t a = (uint32_t)__shfl((int)W[0], src0 + 8 * ks, 64);
            const uint32_t b = (uint32_t)__shfl((int)W[1], src0 + 8 * ks, 64);
            mask_b[((int64_t)bh * ntile + mask_bwd_tile(2 * KT + ks, QT, NP)) * 64 + lane] =
                __builtin_amdgcn_ubfe(a, 16 * h, 16) | (__builtin_amdgcn_ubfe(b, 16 * h, 16) << 16);
        }
    }
}

template <bool SUBF>
__global__ __launch_bounds__(256) void k_attn_dropmask(int64_t T_, int64_t nbh, uint32_t* __restrict__ mask_f,
                                                       uint32_t* __restrict__ mask_b, DropArgs d) {
    dropmask_block<SUBF>(T_, nbh, mask_f, mask_b, d, (int)blockIdx.x);
}

// One launch for a sublayer's LayerNorm forward and its attention's keep bits (the two are
// independent: LN1 feeds the QKV GEMM, the bits the attention after it).  Blocks 0..n_dm-1 generate
// keep bits (Philox: VALU-bound), the rest run LayerNorm rows (HBM-bound) -- co-resident on the CUs,
// so the Philox arithmetic hides under the LayerNorm's memory time instead of running as its own
// 7.8 us launch at C2.  Bits and rows are exactly those of k_attn_dropmask and k_ln_fwd.
template <bool SUBF, int VEC, int NJ>
__global__ __launch_bounds__(256) void k_ln_fwd_dropmask(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, bf16_t* __restrict__ y,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                         int64_t rows, int C, float eps, int n_ln, int64_t T_,
                                                         int64_t nbh, uint32_t* __restrict__ mask_f,
                                                         uint32_t* __restrict__ mask_b, DropArgs d, int n_dm) {
    const int bid = (int)blockIdx.x;
    if (bid < n_dm)
        dropmask_block<SUBF>(T_, nbh, mask_f, mask_b, d, bid);
    else
        ln_fwd_rows<VEC, NJ, bf16_t, 2, true>(x, w, b, y, mean_out, rstd_out, rows, C, eps, bid - n_dm, n_ln);
}

__device__ __forceinline__ bool keep_elem(const DropArgs& d, uint64_t stream, uint64_t idx) {
    return keep_of(philox_of(d.seed, stream, idx), idx, d.thr);
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

// =====================================================================================
// fp32 MFMA forward for small heads (D <= 32, e.g. the as-shipped head_size 21), no dropout:
// the eval / generate path of the fp32 model.  v_mfma_f32_16x16x4_f32 (exact f32 products, f32
// accumulation).  Block = 4 waves x 16 queries; 64-key K/V tiles in LDS (zero-padded to DP4 / 32
// columns).  S^T = K Q^T puts the query on the lane column (softmax statistics lane-local + two
// shuffles); P^T is consumed straight from the S^T accumulator as the B operand of O^T = V^T P^T in
// the permuted key order {4g + s} (k-step s, lane group g), V read in the same order.
// =====================================================================================
__device__ __forceinline__ fv4 mfma_f32x4(float a, float b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int DP4>  // D padded to a multiple of 4 (<= 32)
__global__ __launch_bounds__(256) void k_attn_fwd_f32mfma(int64_t T_, int H, int D, const float* __restrict__ q,
                                                          const float* __restrict__ k, const float* __restrict__ v,
                                                          int64_t ld, float* __restrict__ o, int64_t ldo,
                                                          float* __restrict__ lse, float scale) {
    constexpr int KS = DP4 / 4;           // k-steps of S^T
    constexpr int KLD = DP4 + 1, VLD = 33;
    __shared__ float Ks[64 * KLD];
    __shared__ float Vs[64 * VLD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int64_t qblk0 = (int64_t)blockIdx.x * 64;
    const int64_t qw0 = qblk0 + wave * 16;
    const int64_t qa = qw0 + li;                       // this lane's query (S^T column)
    const float* qb = q + (int64_t)b * T_ * ld + h * D;
    const float* kb = k + (int64_t)b * T_ * ld + h * D;
    const float* vb = v + (int64_t)b * T_ * ld + h * D;
    float qf[KS];                                      // Q^T B operand: Q[qa][4t + g]
#pragma unroll
    for (int t = 0; t < KS; ++t) {
        const int e = 4 * t + g;
        qf[t] = (qa < T_ && e < D) ? qb[qa * ld + e] : 0.f;
    }
    fv4 oacc[2] = {fv4{0.f, 0.f, 0.f, 0.f}, fv4{0.f, 0.f, 0.f, 0.f}};
    float m_run = -INFINITY, l_run = 0.f;
    const int64_t qlast = (qblk0 + 63) < (T_ - 1) ? (qblk0 + 63) : (T_ - 1);
    const int nkv = (int)(qlast / 64) + 1;
    for (int kv = 0; kv < nkv; ++kv) {
        const int64_t k0 = (int64_t)kv * 64;
        __syncthreads();
        for (int i = tid; i < 64 * 32; i += 256) {
            const int r = i >> 5, e = i & 31;
            const int64_t key = k0 + r;
            const bool ok = key < T_ && e < D;
            if (e < DP4) Ks[r * KLD + e] = ok ? kb[key * ld + e] : 0.f;
            Vs[r * VLD + e] = ok ? vb[key * ld + e] : 0.f;
        }
        __syncthreads();
        if (qw0 >= T_ || k0 > qw0 + 15) continue;      // wave past the end / tile fully masked
        fv4 st[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            fv4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < KS; ++t) c = mfma_f32x4(Ks[(16 * kt + li) * KLD + 4 * t + g], qf[t], c);
            st[kt] = c;
        }
        // lane: query qa, keys k0 + 16kt + 4g + r
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t key = k0 + 16 * kt + 4 * g + r;
                float x = st[kt][r] * scale;
                if (key > qa || key >= T_) x = -INFINITY;
                st[kt][r] = x;
                mx = fmaxf(mx, x);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx);
        const float alpha = m_new == -INFINITY ? 1.f : expf(m_run - m_new);
        float ps = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = st[kt][r] == -INFINITY ? 0.f : expf(st[kt][r] - m_new);
                st[kt][r] = p;
                ps += p;
            }
        ps += __shfl_xor(ps, 16, 64);
        ps += __shfl_xor(ps, 32, 64);
        l_run = l_run * alpha + ps;
        m_run = m_new;
        oacc[0] *= alpha;
        oacc[1] *= alpha;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int key = 16 * kt + 4 * g + s;   // permuted order: k-step s, lane group g
#pragma unroll
                for (int et = 0; et < 2; ++et)
                    oacc[et] = mfma_f32x4(Vs[key * VLD + 16 * et + li], st[kt][s], oacc[et]);
            }
    }
    if (qa >= T_) return;
    // O^T accumulator: lane holds e = 16 et + 4g + r for query qa
    const float inv = 1.f / l_run;
    float* orow = o + ((int64_t)b * T_ + qa) * ldo + h * D;
#pragma unroll
    for (int et = 0; et < 2; ++et)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = 16 * et + 4 * g + r;
            if (e < D) orow[e] = oacc[et][r] * inv;
        }
    if (g == 0) lse[(int64_t)bh * T_ + qa] = m_run + logf(l_run);
}

// Sequence-resident form of k_attn_fwd_f32mfma for T <= 256 (the generate() window and the fp32
// model's eval forward): one 8-wave block per (b, h) stages every K / V row of the sequence in LDS
// once (the 64-query blocks above re-load the causal prefix: 10 tile loads per (b, h) at T = 256
// instead of 4, each behind its own barrier), then wave w runs 16-query groups w and 15 - w (equal
// causal work per wave) with the per-group arithmetic of k_attn_fwd_f32mfma unchanged -- the same
// MFMAs in the same order, the same online softmax over the same 64-key tiles -- so the outputs
// are bitwise those of the 64-query-block kernel.
#ifdef CG_F32RES_FASTEXP   // what-if build only (make fastexp): the hardware exp2 path, not bitwise
#define F32RES_EXP(x) __expf(x)
#else
#define F32RES_EXP(x) expf(x)
#endif
template <int DP4>
__global__ __launch_bounds__(512, 4) void k_attn_fwd_f32res(int64_t T_, int H, int D, const float* __restrict__ q,
                                                         const float* __restrict__ k, const float* __restrict__ v,
                                                         int64_t ld, float* __restrict__ o, int64_t ldo,
                                                         float* __restrict__ lse, float scale) {
    constexpr int KS = DP4 / 4;
    // V rows hold only the DP4 padded dimensions (the O^T MFMAs' dims DP4..31 read zeros): 51 KB of
    // LDS at DP4 = 24; the operand look-ahead's 93 VGPRs make it two blocks per CU
    constexpr int KLD = DP4 + 1, VLD = DP4 + 1;
    __shared__ float Ks[256 * KLD];
    __shared__ float Vs[256 * VLD];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    // XCD-contiguous (b, h): the dispatcher deals block i to XCD i % 8, so XCD x runs the x-th eighth of
    // the (b, h) range in order and a sequence's heads share its L2 -- each head reads 84 of a row's
    // 1512 B, so with the heads spread over 6 XCDs every row's lines came from HBM ~6 times (234 MB read
    // per launch against the 99 MB of q / k / v)
    const int nblk = (int)gridDim.x, id = (int)blockIdx.x, nq = nblk >> 3, nr = nblk & 7, xcd = id & 7;
    const int bh = (xcd < nr ? xcd * (nq + 1) : nr * (nq + 1) + (xcd - nr) * nq) + (id >> 3);
    const int b = bh / H, h = bh % H;
    const float* qb = q + (int64_t)b * T_ * ld + h * D;
    const float* kb = k + (int64_t)b * T_ * ld + h * D;
    const float* vb = v + (int64_t)b * T_ * ld + h * D;
    // every K / V element of the thread loaded before the first LDS write (a load-write loop waits
    // for each load in turn: 32 dependent round trips per thread before any MFMA)
    constexpr int NL = 256 * DP4 / 512;
    float kx[NL], vx[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int i = tid + 512 * u, r = i / DP4, e = i - r * DP4;
        const bool ok = r < T_ && e < D;
        kx[u] = ok ? kb[(int64_t)r * ld + e] : 0.f;
        vx[u] = ok ? vb[(int64_t)r * ld + e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int i = tid + 512 * u, r = i / DP4, e = i - r * DP4;
        Ks[r * KLD + e] = kx[u];
        Vs[r * VLD + e] = vx[u];
    }
    __syncthreads();
#pragma unroll 1
    for (int gi = 0; gi < 2; ++gi) {
        const int64_t qw0 = 16 * (gi == 0 ? wave : 15 - wave);
        if (qw0 >= T_) continue;
        const int64_t qa = qw0 + li;
        float qf[KS];
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const int e = 4 * t + g;
            qf[t] = (qa < T_ && e < D) ? qb[qa * ld + e] : 0.f;
        }
        fv4 oacc[2] = {fv4{0.f, 0.f, 0.f, 0.f}, fv4{0.f, 0.f, 0.f, 0.f}};
        float m_run = -INFINITY, l_run = 0.f;
        const int nkv = (int)((qw0 + 15) / 64) + 1;   // the 64-key tiles with k0 <= qw0 + 15, in order
        // one 64-key tile.  FULL: every key of the tile precedes the group's first query (and T) -- no
        // causal mask, no -inf scores, all four 16-key sub-tiles: the same arithmetic with the masking
        // compares, the -inf tests and the sub-tile guards compiled out (int32 indices), bitwise equal
        auto tile = [&](int kv, auto fullc) {
            constexpr bool FULL = decltype(fullc)::value;
            const int k0 = kv * 64;
            const float* Kt = Ks + k0 * KLD;
            const float* Vt = Vs + k0 * VLD;
            // 16-key sub-tiles past the group's last query (k0 + 16 kt > qw0 + 15) are fully masked: their
            // scores are -inf, their p exact zeros, so their S and O MFMAs and softmax terms change
            // nothing (max with -inf, + 0, MFMA products all 0) -- skipped, the result bitwise the same
            const int nkt = FULL ? 4 : ((int)qw0 + 15 - k0) / 16 + 1 < 4 ? ((int)qw0 + 15 - k0) / 16 + 1 : 4;
            // operands read one 16-key sub-tile ahead of their MFMAs, unconditionally (rows < 256 of the
            // staged sequence): K for the S products, then V's first sub-tile under the softmax and
            // each next one under the current one's O MFMAs -- not one LDS round trip per MFMA
            auto rdk = [&](float (&kr)[KS], int kt) {
#pragma unroll
                for (int t = 0; t < KS; ++t) kr[t] = Kt[(16 * kt + li) * KLD + 4 * t + g];
            };
            auto rdv = [&](float (&vr)[4][2], int kt) {
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int et = 0; et < 2; ++et) {
                        const int e = 16 * et + li;
                        vr[s][et] = e < DP4 ? Vt[(16 * kt + 4 * g + s) * VLD + e] : 0.f;
                    }
            };
            fv4 st[4];
            float kr[2][KS];
            rdk(kr[0], 0);
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                if (kt < 3) rdk(kr[(kt + 1) & 1], kt + 1);
                __builtin_amdgcn_sched_barrier(0);
                fv4 c = {0.f, 0.f, 0.f, 0.f};
                if (kt < nkt) {
#pragma unroll
                    for (int t = 0; t < KS; ++t) c = mfma_f32x4(kr[kt & 1][t], qf[t], c);
                }
                st[kt] = c;
            }
            float mx = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = k0 + 16 * kt + 4 * g + r;
                    float x = st[kt][r] * scale;
                    if constexpr (FULL) asm("" : "+v"(x));   // keep x * scale rounded: the masked path's
                    else if (key > (int)qa || key >= (int)T_) x = -INFINITY;   // select stops its fma with - m_new
                    st[kt][r] = x;
                    if (kt < nkt) mx = fmaxf(mx, x);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float m_new = fmaxf(m_run, mx);
            const float alpha = m_new == -INFINITY ? 1.f : F32RES_EXP(m_run - m_new);
            float ps = 0.f;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (kt < nkt) {
                        const float p = (!FULL && st[kt][r] == -INFINITY) ? 0.f : F32RES_EXP(st[kt][r] - m_new);
                        st[kt][r] = p;
                        ps += p;
                    }
                }
            ps += __shfl_xor(ps, 16, 64);
            ps += __shfl_xor(ps, 32, 64);
            l_run = l_run * alpha + ps;
            m_run = m_new;
            oacc[0] *= alpha;
            oacc[1] *= alpha;
            float vr[2][4][2];
            rdv(vr[0], 0);
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                if (kt >= nkt) break;
                if (kt < 3) rdv(vr[(kt + 1) & 1], kt + 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int et = 0; et < 2; ++et) oacc[et] = mfma_f32x4(vr[kt & 1][s][et], st[kt][s], oacc[et]);
            }
        };
        for (int kv = 0; kv < nkv; ++kv) {
            if (kv * 64 + 63 <= (int)qw0 && kv * 64 + 63 < (int)T_) tile(kv, std::true_type{});
            else tile(kv, std::false_type{});
        }
        if (qa >= T_) continue;
        const float inv = 1.f / l_run;
        float* orow = o + ((int64_t)b * T_ + qa) * ldo + h * D;
#pragma unroll
        for (int et = 0; et < 2; ++et)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = 16 * et + 4 * g + r;
                if (e < D) orow[e] = oacc[et][r] * inv;
            }
        if (g == 0) lse[(int64_t)bh * T_ + qa] = m_run + logf(l_run);
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

DropArgs make_drop(double p, uint64_t seed, const uint64_t* rng_call, int site) {
    DropArgs d;
    d.thr = p > 0 ? dropout_threshold(p) : 0u;
    d.dscale = p > 0 ? dropout_scale(p) : 1.f;
    d.seed = seed;
    d.rng_call = rng_call;
    d.site = site;
    d.mask = nullptr;
    d.mask_bwd = nullptr;
    return d;
}

// FWD and BWD tiles, 256 B each
int64_t mask_bytes(int64_t B, int64_t H, int64_t T) { return 2 * B * H * mask_tiles(T) * 256; }

void set_masks(DropArgs& d, const uint64_t* mask, int64_t B, int64_t H, int64_t T) {
    d.mask = (const uint32_t*)mask;
    d.mask_bwd = (const uint32_t*)mask + B * H * mask_tiles(T) * 64;
}

void launch_dropmask(int64_t B, int64_t H, int64_t T, uint64_t* mask, const DropArgs& d, hipStream_t st) {
    const int64_t np = T / 64, regions = B * H * np * (np + 1) / 2;
    uint32_t* m = (uint32_t*)mask;
    if (d.thr > 0x8000u)
        k_attn_dropmask<true><<<ceil_div(regions, 4 * DM_TPW), 256, 0, st>>>(T, B * H, m, m + B * H * mask_tiles(T) * 64, d);
    else
        k_attn_dropmask<false><<<ceil_div(regions, 4 * DM_TPW), 256, 0, st>>>(T, B * H, m, m + B * H * mask_tiles(T) * 64, d);
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

namespace {
int attn_fwd_impl(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k, const void* v,
                  int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale, double dropout_p, uint64_t seed,
                  const uint64_t* rng_call, int site, uint64_t* mask, bool mask_ready, void* stream);
}

extern "C" int cg_attn_fwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                           const void* v, int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale,
                           double dropout_p, uint64_t seed, const uint64_t* rng_call, int site, uint64_t* mask,
                           void* stream) {
    return attn_fwd_impl(dtype, B, T, H, D, q, k, v, ld_qkv, o, ld_o, lse, scale, dropout_p, seed, rng_call, site,
                         mask, false, stream);
}

extern "C" int cg_attn_fwd_premasked(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q,
                                     const void* k, const void* v, int64_t ld_qkv, void* o, int64_t ld_o, float* lse,
                                     float scale, double dropout_p, uint64_t seed, const uint64_t* rng_call, int site,
                                     uint64_t* mask, void* stream) {
    return attn_fwd_impl(dtype, B, T, H, D, q, k, v, ld_qkv, o, ld_o, lse, scale, dropout_p, seed, rng_call, site,
                         mask, true, stream);
}

extern "C" int cg_attn_dropmask(int64_t B, int64_t H, int64_t T, double dropout_p, uint64_t seed,
                                const uint64_t* rng_call, int site, uint64_t* mask, void* stream) {
    CG_REQUIRE(B > 0 && H > 0 && T > 0 && T % 64 == 0, "cg_attn_dropmask: bad shape (T %% 64 == 0 required)");
    CG_REQUIRE(dropout_p > 0 && dropout_p < 1 && mask, "cg_attn_dropmask: needs 0 < p < 1 and a mask buffer");
    DropArgs d = make_drop(dropout_p, seed, rng_call, site);
    launch_dropmask(B, H, T, mask, d, (hipStream_t)stream);
    CG_LAUNCH_CHECK("cg_attn_dropmask");
    return CG_OK;
}

extern "C" int cg_layernorm_fwd_attn_dropmask(const float* x, const float* w, const float* b, void* y, int y_dtype,
                                              float* mean, float* rstd, int64_t rows, int64_t C, float eps, int64_t B,
                                              int64_t H, int64_t T, double dropout_p, uint64_t seed,
                                              const uint64_t* rng_call, int site, uint64_t* mask, void* stream) {
    CG_REQUIRE(B > 0 && H > 0 && T > 0 && T % 64 == 0, "cg_layernorm_fwd_attn_dropmask: bad shape (T %% 64 == 0 required)");
    CG_REQUIRE(dropout_p > 0 && dropout_p < 1 && mask, "cg_layernorm_fwd_attn_dropmask: needs 0 < p < 1 and a mask buffer");
    CG_REQUIRE(rows > 0 && C > 0 && C <= 2048, "cg_layernorm_fwd_attn_dropmask: need 0 < C <= 2048");
    hipStream_t st = (hipStream_t)stream;
    const DropArgs d = make_drop(dropout_p, seed, rng_call, site);
    const bool al16 = (((uintptr_t)x | (uintptr_t)w | (uintptr_t)b) & 15) == 0;
    if (y_dtype != CG_BF16 || !al16 || (C != 384 && C != 768)) {   // the shapes without a fused form: two launches
        const int rc = cg_layernorm_fwd(x, w, b, y, y_dtype, mean, rstd, rows, C, eps, stream);
        if (rc != CG_OK) return rc;
        launch_dropmask(B, H, T, mask, d, st);
        CG_LAUNCH_CHECK("cg_layernorm_fwd_attn_dropmask");
        return CG_OK;
    }
    const int64_t np = T / 64, regions = B * H * np * (np + 1) / 2;
    const int n_dm = (int)ceil_div(regions, 4 * DM_TPW);
    int n_ln = (int)ceil_div(rows, 8);   // k_ln_fwd's grid: 4 waves x 2 rows per block
    n_ln = n_ln > 4096 ? 4096 : n_ln;
    uint32_t* mf = (uint32_t*)mask;
    uint32_t* mb = mf + B * H * mask_tiles(T) * 64;
#define LDM(SUBF_, V_)                                                                                                \
    k_ln_fwd_dropmask<SUBF_, V_, 3><<<n_dm + n_ln, 256, 0, st>>>(x, w, b, (bf16_t*)y, mean, rstd, rows, (int)C, eps, \
                                                               n_ln, T, B * H, mf, mb, d, n_dm)
    if (d.thr > 0x8000u) {
        if (C == 384) LDM(true, 2);
        else LDM(true, 4);
    } else {
        if (C == 384) LDM(false, 2);
        else LDM(false, 4);
    }
#undef LDM
    CG_LAUNCH_CHECK("cg_layernorm_fwd_attn_dropmask");
    return CG_OK;
}

namespace {
int attn_fwd_impl(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k, const void* v,
                  int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale, double dropout_p, uint64_t seed,
                  const uint64_t* rng_call, int site, uint64_t* mask, bool mask_ready, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && H > 0 && D > 0 && D <= 128, "cg_attn_fwd: bad shape (D must be <= 128)");
    CG_REQUIRE(dropout_p >= 0 && dropout_p < 1, "cg_attn_fwd: dropout_p must be in [0,1)");
    hipStream_t st = (hipStream_t)stream;
    DropArgs d = make_drop(dropout_p, seed, rng_call, site);
    if (fast_attn_ok(dtype, T, D, q, k, o, ld_qkv, ld_o)) {
        if (d.thr) {
            CG_REQUIRE(mask, "cg_attn_fwd: dropout on the MFMA path needs a mask buffer (cg_attn_mask_bytes)");
            if (!mask_ready) launch_dropmask(B, H, T, mask, d, st);
            set_masks(d, mask, B, H, T);
        }
        attn::launch_fwd_d64(B, T, (int)H, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ld_qkv, (bf16_t*)o,
                             ld_o, lse, scale, d, st);
    } else {
        dim3 grid(ceil_div(T, GB), (unsigned)(B * H));
        const size_t lds = generic_lds<float>((int)D, 3, 1);
        if (dtype == CG_F32 && !d.thr && D <= 32 && T <= 256 && g_attn_variant != 1) {
            // attn_variant 1 (A/B, tests): the 64-query-block kernel below
#define AR(dp) k_attn_fwd_f32res<dp><<<(unsigned)(B * H), 512, 0, st>>>(T, (int)H, (int)D, (const float*)q, \
                                                                     (const float*)k, (const float*)v, ld_qkv, \
                                                                     (float*)o, ld_o, lse, scale)
            const int dp4 = (int)((D + 3) / 4) * 4;
            if (dp4 <= 8) AR(8);
            else if (dp4 <= 16) AR(16);
            else if (dp4 <= 24) AR(24);
            else AR(32);
#undef AR
        } else if (dtype == CG_F32 && !d.thr && D <= 32) {
            dim3 g2(ceil_div(T, 64), (unsigned)(B * H));
#define AF(dp)                                                                                                  \
    k_attn_fwd_f32mfma<dp><<<g2, 256, 0, st>>>(T, (int)H, (int)D, (const float*)q, (const float*)k, (const float*)v, \
                                               ld_qkv, (float*)o, ld_o, lse, scale)
            const int dp4 = (int)((D + 3) / 4) * 4;
            if (dp4 <= 8) AF(8);
            else if (dp4 <= 16) AF(16);
            else if (dp4 <= 24) AF(24);
            else AF(32);
#undef AF
        } else if (dtype == CG_BF16)
            k_attn_fwd_generic<bf16_t><<<grid, 256, lds, st>>>(T, (int)H, (int)D, (const bf16_t*)q, (const bf16_t*)k,
                                                               (const bf16_t*)v, ld_qkv, (bf16_t*)o, ld_o, lse, scale, d);
        else
            k_attn_fwd_generic<float><<<grid, 256, lds, st>>>(T, (int)H, (int)D, (const float*)q, (const float*)k,
                                                              (const float*)v, ld_qkv, (float*)o, ld_o, lse, scale, d);
    }
    CG_LAUNCH_CHECK("cg_attn_fwd");
    return CG_OK;
}
}  // namespace

extern "C" int64_t cg_attn_mask_bytes(int64_t B, int64_t H, int64_t T) { return mask_bytes(B, H, T); }

extern "C" int64_t cg_attn_bwd_workspace(int64_t B, int64_t T, int64_t H, int64_t D) {
    (void)D;
    const int64_t delta = (B * H * T * (int64_t)sizeof(float) + 255) / 256 * 256;
    return delta + mask_bytes(B, H, T);
}

namespace {
// delta_in: rowsum(dO * O) precomputed (cg_attn_bwd_delta), read only by the merged resident kernel
int attn_bwd_impl(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                  const void* v, int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout, int64_t ld_do,
                  const float* lse, const float* delta_in, void* dq, void* dk, void* dv, int64_t ld_dqkv, float scale,
                  double dropout_p, uint64_t seed, const uint64_t* rng_call, int site, const uint64_t* mask,
                  void* workspace, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && H > 0 && D > 0 && D <= 128, "cg_attn_bwd: bad shape (D must be <= 128)");
    CG_REQUIRE(workspace, "cg_attn_bwd: workspace required");
    hipStream_t st = (hipStream_t)stream;
    DropArgs d = make_drop(dropout_p, seed, rng_call, site);
    float* delta = (float*)workspace;
    const int64_t nrows = B * T * H;
    const bool fast = fast_attn_ok(dtype, T, D, q, dout, dq, ld_qkv, ld_do) && ld_dqkv % 8 == 0 &&
                      ((((uintptr_t)dk) | ((uintptr_t)dv) | ((uintptr_t)o)) & 15) == 0 && ld_o % 8 == 0;
    if (fast) {
        // delta = rowsum(dO * O) is computed inside the dQ kernel (which runs before dK/dV)
    } else if (dtype == CG_BF16)
        k_attn_delta<bf16_t><<<ceil_div(nrows, 256), 256, 0, st>>>(B, T, (int)H, (int)D, (const bf16_t*)o, ld_o,
                                                                 (const bf16_t*)dout, ld_do, delta);
    else
        k_attn_delta<float><<<ceil_div(nrows, 256), 256, 0, st>>>(B, T, (int)H, (int)D, (const float*)o, ld_o,
                                                                (const float*)dout, ld_do, delta);
    if (fast) {
        if (d.thr) {
            if (!mask) {  // regenerate the forward's keep bits (identical Philox stream)
                uint64_t* m = (uint64_t*)((char*)workspace + (B * H * T * (int64_t)sizeof(float) + 255) / 256 * 256);
                launch_dropmask(B, H, T, m, d, st);
                mask = m;
            }
            set_masks(d, mask, B, H, T);
        }
        const bf16_t *Q = (const bf16_t*)q, *K = (const bf16_t*)k, *V = (const bf16_t*)v, *DO = (const bf16_t*)dout;
        const bool din = delta_in && attn::bwd_merged(T);
        attn::launch_bwd_d64(B, T, (int)H, Q, K, V, ld_qkv, (const bf16_t*)o, ld_o, DO, ld_do, lse,
                             din ? (float*)delta_in : delta, din, (bf16_t*)dq, ld_dqkv, (bf16_t*)dk, (bf16_t*)dv,
                             ld_dqkv, scale, d, st);
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
}  // namespace

extern "C" int cg_attn_bwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                           const void* v, int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout, int64_t ld_do,
                           const float* lse, void* dq, void* dk, void* dv, int64_t ld_dqkv, float scale,
                           double dropout_p, uint64_t seed, const uint64_t* rng_call, int site, const uint64_t* mask,
                           void* workspace, void* stream) {
    return attn_bwd_impl(dtype, B, T, H, D, q, k, v, ld_qkv, o, ld_o, dout, ld_do, lse, nullptr, dq, dk, dv, ld_dqkv,
                         scale, dropout_p, seed, rng_call, site, mask, workspace, stream);
}

extern "C" int cg_attn_bwd_delta(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                                 const void* v, int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout,
                                 int64_t ld_do, const float* lse, const float* delta, void* dq, void* dk, void* dv,
                                 int64_t ld_dqkv, float scale, double dropout_p, uint64_t seed,
                                 const uint64_t* rng_call, int site, const uint64_t* mask, void* workspace,
                                 void* stream) {
    CG_REQUIRE(!delta || (((uintptr_t)delta) & 3) == 0, "cg_attn_bwd_delta: delta must be 4-byte aligned");
    return attn_bwd_impl(dtype, B, T, H, D, q, k, v, ld_qkv, o, ld_o, dout, ld_do, lse, delta, dq, dk, dv, ld_dqkv,
                         scale, dropout_p, seed, rng_call, site, mask, workspace, stream);
}
