// charpt A/B-only attention variants (never the product library: `make ab`, CG_AB_VARIANTS):
// measured slower than the product kernels of attention_d64.h, kept for the interleaved A/B tools.
#include "../attention_d64.h"

namespace cg {
namespace {
template <bool DROP>
__device__ __forceinline__ void fwd_qblock(int qblk, int bh, char* smem, int64_t T_, int H, const bf16_t* __restrict__ q,
                                           const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, int64_t ld,
                                           bf16_t* __restrict__ o, int64_t ldo, float* __restrict__ lse,
                                           float scale_log2, const uint32_t* __restrict__ mask, float dscale) {
    constexpr int SLOT = FWD_SLOT;
    char* const Qimg = smem + 3 * SLOT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = (int)T_, b = bh / H, hh = bh % H;
    const int Q0 = qblk * 256;
    const int64_t boff = (int64_t)b * T_, ntile = mask_tiles(T_);
    const bf16_t* kb_ = k + boff * ld + hh * 64;
    const bf16_t* vb_ = v + boff * ld + hh * 64;
    const int qg[2] = {Q0 + 32 * (7 - wave), Q0 + 32 * wave};   // g = 0 (A): the longer causal prefix
    const bool act[2] = {qg[0] < T, qg[1] < T};
    // keep words: FWD tile (query block, key tile kv) of each group, prefetched one tile ahead
    const uint32_t* mrow[2];
    uint32_t mw[2] = {0u, 0u};
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        mrow[g] = DROP ? mask + ((int64_t)bh * ntile + mask_fwd_tile(qg[g] >> 5, 0)) * 64 + lane : nullptr;
        if (DROP && act[g]) mw[g] = mrow[g][0];
    }
    {   // Q image: rows Q0 .. Q0 + 255 (zero past T)
        const bf16_t* qb_ = q + boff * ld + hh * 64;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = (tid >> 3) + 32 * i, c = tid & 7;
            const uint4 x = Q0 + r < T ? *(const uint4*)(qb_ + (int64_t)(Q0 + r) * ld + c * 8) : make_uint4(0, 0, 0, 0);
            *(uint4*)(Qimg + aoff(r, c)) = x;
        }
    }
    const int qr[2] = {32 * (7 - wave), 32 * wave};   // the groups' rows in the Q image
    fv16 oacc[2][2];
#pragma unroll
    for (int g = 0; g < 2; ++g) oacc[g][0] = oacc[g][1] = fv16{};
    // running max starts at -FLT_MAX, not -inf: a -inf score then exponentiates to 0, never NaN,
    // and the first tile still always moves the max (its decision compares against -FLT_MAX + THR)
    float m_run[2] = {-FLT_MAX, -FLT_MAX};
    fv4 l_run[2] = {fv4{}, fv4{}};
    const sv8 ones = rowsum_ones(lane);
    const int qlast = (Q0 + 255 < T - 1) ? Q0 + 255 : T - 1;
    const int nkv = qlast / 64 + 1;
    const int npipe = act[1] ? (qg[1] + 31) / 64 : 0;   // B's diagonal tile: first unpipelined tile
    fv16 sA[2], sB[2] = {fv16{} - INFINITY, fv16{} - INFINITY};
    sv8 pfA[2][2], pfB[2][2];
    uint32_t mwBp = 0u;   // B's keep word of the previous tile
    int cs = 0, ps = 2, ns = 1;   // ring slots of tiles kv, kv - 1, kv + 1
    stage_store(stage_load(kb_, ld, vb_, ld, 0, tid), smem, tid);
    {   // the V half of slot 2 is tile -1 of the pipeline head: zeros
        const int r = tid >> 3, c = tid & 7;
        *(uint4*)(smem + 2 * SLOT + TILE + aoff(r, c)) = make_uint4(0, 0, 0, 0);
        *(uint4*)(smem + 2 * SLOT + TILE + aoff(r + 32, c)) = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    // per tile: issue the next tile's loads first, write them to the ring after the compute
    auto next_loads = [&](int kv, uint32_t (&mn)[2]) {
        const int nxt = kv + 1 < nkv ? kv + 1 : kv;
#pragma unroll
        for (int g = 0; g < 2; ++g)
            mn[g] = (DROP && act[g] && nxt * 64 <= qg[g] + 31) ? mrow[g][nxt * 64] : 0u;
        return stage_load(kb_, ld, vb_, ld, (int64_t)nxt * 64, tid);
    };
    auto advance = [&](const Stage2& st, const uint32_t (&mn)[2]) {
        stage_store(st, smem + ns * SLOT, tid);
        mwBp = mw[1];
        mw[0] = mn[0];
        mw[1] = mn[1];
        ps = cs;
        cs = ns;
        ns = ns == 2 ? 0 : ns + 1;
        __syncthreads();
    };
    int kv = 0;
    for (; kv < npipe; ++kv) {
        // next K tile loaded now and written to its (free) slot mid-tile, next V tile loaded then
        // and written at the end: 8 staging VGPRs live at a time instead of 16
        const int nxt = kv + 1;   // < nkv: B's diagonal tile is still ahead
        uint32_t mn[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) mn[g] = DROP ? mrow[g][nxt * 64] : 0u;   // both groups full through nxt
        const Stage1 stk = stage_load1(kb_, ld, (int64_t)nxt * 64, tid);
        const char* Ki = smem + cs * SLOT;
        const char* Vi = Ki + TILE;
        const char* Vp = smem + ps * SLOT + TILE;
        // at kv = 0, B's "previous tile" is sB = -inf against a zeroed V slot: it adds exactly 0
        qk_tile(sA, Ki, Qimg, qr[0], lane);
        softmax_pack<DROP>(sB, scale_log2, m_run[1], l_run[1], mwBp, pfB, ones);
        pv_tile(oacc[1], Vp, pfB, lane);
        rescale_if(tile_max(sA) * scale_log2, m_run[0], l_run[0], oacc[0]);
        stage_store1(stk, smem + ns * SLOT, tid);
        const Stage1 stv = stage_load1(vb_, ld, (int64_t)nxt * 64, tid);
        qk_tile(sB, Ki, Qimg, qr[1], lane);
        softmax_pack<DROP>(sA, scale_log2, m_run[0], l_run[0], mw[0], pfA, ones);
        pv_tile(oacc[0], Vi, pfA, lane);
        rescale_if(tile_max(sB) * scale_log2, m_run[1], l_run[1], oacc[1]);
        stage_store1(stv, smem + ns * SLOT + TILE, tid);
        mwBp = mw[1];
        mw[0] = mn[0];
        mw[1] = mn[1];
        ps = cs;
        cs = ns;
        ns = ns == 2 ? 0 : ns + 1;
        __syncthreads();
    }
    if (npipe > 0) {   // pipeline tail: B's pending tile npipe - 1 (its V still in the previous slot)
        softmax_pack<DROP>(sB, scale_log2, m_run[1], l_run[1], mwBp, pfB, ones);
        pv_tile(oacc[1], smem + ps * SLOT + TILE, pfB, lane);
    }
    for (; kv < nkv; ++kv) {
        uint32_t mn[2];
        const Stage2 st = next_loads(kv, mn);
        const char* Ki = smem + cs * SLOT;
        const char* Vi = Ki + TILE;
        const int k0 = kv * 64;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (!act[g] || k0 > qg[g] + 31) continue;
            // qg is a multiple of 32: the tile is full (k0 + 63 < qg), has the diagonal in its second
            // subtile (qg = k0 + 32) or in its first with the second wholly masked (qg = k0)
            const int rel = __builtin_amdgcn_readfirstlane(qg[g] - k0);
            if (rel >= 64)
                fwd_group_tile<DROP, 2, -1>(Ki, Vi, Qimg, qr[g], lane, scale_log2, m_run[g], l_run[g], oacc[g], mw[g], ones);
            else if (rel == 32)
                fwd_group_tile<DROP, 2, 1>(Ki, Vi, Qimg, qr[g], lane, scale_log2, m_run[g], l_run[g], oacc[g], mw[g], ones);
            else
                fwd_group_tile<DROP, 1, 0>(Ki, Vi, Qimg, qr[g], lane, scale_log2, m_run[g], l_run[g], oacc[g], mw[g], ones);
        }
        advance(st, mn);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (!act[g]) continue;
        const float lt = l_run[g][0];   // every accumulator register holds query lane & 31's sum
        const int64_t qa = qg[g] + (lane & 31);
        store_rows(o + (boff + qa) * ldo + hh * 64, oacc[g], dscale / lt, lane);
        if (lane < 32) lse[(int64_t)bh * T_ + qa] = (m_run[g] + __log2f(lt)) * LN2;
    }
}

// One workgroup per (b, h) and PAIR of 256-query blocks (nq - 1 - x, then x): the causal work of a
// pair is the same for every x, so the grid has no long-block tail (measured occupancy of the
// one-block-per-workgroup grid at C4: 63 %).  K/V reuse stays inside the workgroup and its L2.
template <bool DROP>
__global__ __launch_bounds__(256, 2) void k_attn_fwd_d64(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                         const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                         int64_t ld, bf16_t* __restrict__ o, int64_t ldo,
                                                         float* __restrict__ lse, float scale_log2,
                                                         const uint32_t* __restrict__ mask, float dscale) {
    __shared__ __attribute__((aligned(16))) char smem[FWD_LDS];
    int x, bh;
    block_coords<false>(x, bh);
    const int nq = (int)((T_ + 255) / 256), first = nq - 1 - x;
    const int npass = x == first ? 1 : 2;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
        if (pass) __syncthreads();
        fwd_qblock<DROP>(pass ? x : first, bh, smem, T_, H, q, k, v, ld, o, ldo, lse, scale_log2, mask, dscale);
    }
}
// =====================================================================================
// Forward at T % 256 == 0, T >= 512: two waves per SIMD in ping-pong (MI355X_MICROARCH.md "Two
// waves per SIMD"; cdna guide "Fused attention prefill").  One 512-thread workgroup per CU; wave w
// owns query group g = 2 (w & 3) + (w >> 2) of the 256-query block (team w >> 2: the even / odd
// groups, so both teams have the same diagonal tail).  A group's key tile t is two items, each one
// barrier-delimited segment:
//   M(t) = O^T += V^T P^T of tile t - 1, then S^T = K Q^T of tile t   (16 MFMAs, LDS reads)
//   V(t) = causal mask, row max, lazy rescale, exp2 / pack / row sums, keep bits   (VALU)
// and team 1 runs one segment behind team 0, so on every SIMD one wave's MFMA segment sits beside
// the other's softmax.  Per group the arithmetic and its order are fwd_group_tile's (S, mask,
// rescale, P, then P V before the next rescale): the same bits as the ring kernel.
// K/V tiles: 4-slot LDS ring (16 KB each), tile u + 2 requested by LDS-DMA at segment 2u (its slot's
// previous tile u - 2 was last read, by team 1's P V, in segment 2u - 1), every wave's DMAs of tile
// u retired by the counted wait + barrier opening segment 2u.  Keep words: the group's FWD tiles
// 0..ng-1 are contiguous in the mask image, copied once per block into a per-wave LDS region.
// =====================================================================================
constexpr int PP_SLOTS = 4, PP_KW_TILES = 16;   // T <= 1024: a group spans <= 16 key tiles
constexpr int PP_LDS = PP_SLOTS * 2 * TILE + 8 * PP_KW_TILES * 256;   // 64 KB ring + 32 KB keep words

template <bool DROP>
__device__ __forceinline__ void fwd_pp_block(int qblk, int bh, char* smem, int64_t T_, int H,
                                             const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                             const bf16_t* __restrict__ v, int64_t ld, bf16_t* __restrict__ o,
                                             int64_t ldo, float* __restrict__ lse, float scale_log2,
                                             const uint32_t* __restrict__ mask, float dscale) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), team = wave >> 2, wq = wave & 3;
    const int g = 2 * wq + team;
    const int b = bh / H, hh = bh % H;
    const int Q0 = qblk * 256, q0 = Q0 + 32 * g;
    const int64_t boff = (int64_t)b * T_, ntile = mask_tiles(T_);
    const bf16_t* kb_ = k + boff * ld + hh * 64;
    const bf16_t* vb_ = v + boff * ld + hh * 64;
    const bf16_t* qb_ = q + boff * ld + hh * 64;
    const int ng = (q0 + 31) / 64 + 1;          // this group's key tiles
    const int nmax = (Q0 + 255) / 64 + 1;       // the block's (group 7)
    const uint32_t lds0 = lds_base(smem);
    const uint32_t kw_lds = lds0 + (uint32_t)(PP_SLOTS * 2 * TILE + wave * PP_KW_TILES * 256);
    const char* kw = smem + PP_SLOTS * 2 * TILE + wave * PP_KW_TILES * 256;
    uint32_t doff[2];
    dma_lane_offs(ld, wq, lane, doff);
    // tile t: K by team 0's waves, V by team 1's, 2 DMA instructions per wave
    auto issue_tile = [&](int t) {
        dma_tile_s(team ? vb_ : kb_, ld, (int64_t)t * 64, doff,
                   lds0 + (uint32_t)((t & 3) * 2 * TILE + (team ? TILE : 0)), wq);
    };
    sv8 qf[4];
    {
        const int64_t qa = q0 + (lane & 31);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) gload16(qf[ks], qb_ + qa * ld + 16 * ks + 8 * (lane >> 5));
    }
    if constexpr (DROP) {   // keep words of tiles 0..ng-1: 4 tiles (1 KB) per wave-instruction
        const uint32_t* mrow = mask + ((int64_t)bh * ntile + mask_fwd_tile(q0 >> 5, 0)) * 64;
        const int nw = ng * 64;
        for (int i = 0; i < (ng + 3) / 4; ++i) {
            const int w = i * 256 + lane * 4;
            dma16sl(mrow, (uint32_t)((w + 4 <= nw ? w : nw - 4) * 4), kw_lds + 1024u * i);   // past ng: unused
        }
    }
    issue_tile(0);
    if (nmax > 1) issue_tile(1);
    // Q, keep words and tile 0 landed for every wave (tile 1 may stay in flight)
    if (nmax > 1) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(qf[ks]));
    fv16 oacc[2] = {fv16{}, fv16{}}, s[2] = {fv16{}, fv16{}};
    sv8 pf[2][2] = {};
    float m_run = -FLT_MAX;
    fv4 l_run = fv4{};
    const sv8 ones = rowsum_ones(lane);
    // M(t): P V of tile t - 1 (PV), then S of tile t (S); every LDS fragment is read before the first
    // MFMA.  Both subtiles always: on a diagonal tile whose second subtile lies wholly above the
    // diagonal, V(t) sets it to -inf, so its P is 0 and it adds exact zeros to l and O (the bits of
    // fwd_group_tile<.., 1, 0>).
    auto m_item = [&](int t, auto PV, auto S) {
        const char* Vi = smem + ((t - 1) & 3) * 2 * TILE + TILE;
        const char* Ki = smem + (t & 3) * 2 * TILE;
        sv8 vf[2][2][2], kf[2][4];
        if constexpr (decltype(PV)::value) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int sk = 0; sk < 2; ++sk)
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt) vf[kt][sk][dt] = frag_tr(Vi, 32 * kt, sk, 32 * dt, lane);
        }
        if constexpr (decltype(S)::value) {
#pragma unroll
            for (int sb = 0; sb < 2; ++sb)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) kf[sb][ks] = frag_row(Ki, 32 * sb, ks, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (decltype(PV)::value) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int sk = 0; sk < 2; ++sk) {
                    oacc[0] = mfma32(vf[kt][sk][0], pf[kt][sk], oacc[0]);
                    oacc[1] = mfma32(vf[kt][sk][1], pf[kt][sk], oacc[1]);
                }
        }
        if constexpr (decltype(S)::value) {
            s[0] = fv16{};
            s[1] = fv16{};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                s[0] = mfma32(kf[0][ks], qf[ks], s[0]);
                s[1] = mfma32(kf[1][ks], qf[ks], s[1]);
            }
        }
    };
    // V(t): causal mask, row max, lazy rescale, P (fwd_group_tile's order)
    auto v_item = [&](int t) {
        const int rel = q0 - 64 * t;   // this group's first query against the tile's first key
        uint32_t mw = 0u;
        if constexpr (DROP) mw = *(const uint32_t*)(kw + t * 256 + lane * 4);
        if (rel == 32) {
            mask_upper(s[1], lane & 31, 0, lane, -INFINITY);
        } else if (rel == 0) {
            mask_upper(s[0], lane & 31, 0, lane, -INFINITY);
            s[1] = fv16{} - INFINITY;
        }
        rescale_if(tile_max<2>(s) * scale_log2, m_run, l_run, oacc);
        softmax_pack<DROP, 2>(s, scale_log2, m_run, l_run, mw, pf, ones);
    };
    // segment k opens with a barrier; at k = 2u every wave's DMAs of tile u have landed first (tile
    // u + 1 may stay in flight) and tile u + 2 is requested after it
    const int nseg = 2 * nmax + 2;
    auto seg = [&](int kseg) {
        if (kseg > 0) {
            if (kseg & 1) {
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            } else if ((kseg >> 1) + 1 < nmax) {
                asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            }
        }
        if (!(kseg & 1) && (kseg >> 1) + 2 < nmax) issue_tile((kseg >> 1) + 2);
    };
    using Y = std::true_type;
    using N_ = std::false_type;
    // team 0 runs item i in segment i, team 1 in segment i + 1 (items: M(0) V(0) M(1) V(1) .. M(ng));
    // straight-line bodies per team, so the loop-carried registers need no copies between paths
    if (team == 0) {
        seg(0);
        m_item(0, N_{}, Y{});
        seg(1);
        v_item(0);
#pragma unroll 1
        for (int t = 1; t < ng; ++t) {
            seg(2 * t);
            m_item(t, Y{}, Y{});
            seg(2 * t + 1);
            v_item(t);
        }
        seg(2 * ng);
        m_item(ng, Y{}, N_{});
#pragma unroll 1
        for (int kseg = 2 * ng + 1; kseg < nseg; ++kseg) seg(kseg);
    } else {
        seg(0);
        seg(1);
        m_item(0, N_{}, Y{});
        seg(2);
        v_item(0);
#pragma unroll 1
        for (int t = 1; t < ng; ++t) {
            seg(2 * t + 1);
            m_item(t, Y{}, Y{});
            seg(2 * t + 2);
            v_item(t);
        }
        seg(2 * ng + 1);
        m_item(ng, Y{}, N_{});
#pragma unroll 1
        for (int kseg = 2 * ng + 2; kseg < nseg; ++kseg) seg(kseg);
    }
    const float lt = l_run[0];   // every accumulator register holds query lane & 31's sum
    const int64_t qa = q0 + (lane & 31);
    store_rows_wide(o + (boff + qa) * ldo + hh * 64, oacc, dscale / lt, lane);
    if (lane < 32) lse[(int64_t)bh * T_ + qa] = (m_run + __log2f(lt)) * LN2;
}

template <bool DROP>
__global__ __launch_bounds__(512, 1) void k_attn_fwd_pp(int64_t T_, int H, const bf16_t* __restrict__ q,
                                                        const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                        int64_t ld, bf16_t* __restrict__ o, int64_t ldo,
                                                        float* __restrict__ lse, float scale_log2,
                                                        const uint32_t* __restrict__ mask, float dscale) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int x, bh;
    block_coords<false>(x, bh);
    const int nq = (int)(T_ / 256), first = nq - 1 - x;
    const int npass = x == first ? 1 : 2;
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);   // the younger team
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
        if (pass) __syncthreads();
        fwd_pp_block<DROP>(pass ? x : first, bh, smem, T_, H, q, k, v, ld, o, ldo, lse, scale_log2, mask, dscale);
    }
}

}  // namespace
namespace attn_ab {
bool launch_fwd(int variant, dim3 grid, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v,
                int64_t ld, bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st) {
    if (variant == 5) {   // the register-staged ring with the Q image in LDS
        if (d.mask)
            k_attn_fwd_d64<true><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, d.mask, d.dscale);
        else
            k_attn_fwd_d64<false><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, nullptr, 1.f);
        return true;
    }
    if (variant == 6) {   // Q image in LDS, 3-slot DMA ring one tile ahead
        if (d.mask)
            k_attn_fwd_d64d<true, false><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, d.mask,
                                                               d.dscale);
        else
            k_attn_fwd_d64d<false, false><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E,
                                                                nullptr, 1.f);
        return true;
    }
    if (variant == 4 && T % 256 == 0 && T >= 512 && T <= 64 * PP_KW_TILES) {   // the 8-wave ping-pong forward
        if (d.mask)
            k_attn_fwd_pp<true><<<grid, 512, PP_LDS, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, d.mask,
                                                          d.dscale);
        else
            k_attn_fwd_pp<false><<<grid, 512, PP_LDS, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, nullptr,
                                                           1.f);
        return true;
    }
    return false;
}

bool launch_dq(int variant, dim3 grid, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v,
               int64_t ld, const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse,
               float* delta, bf16_t* dq, int64_t lddq, float scale, const DropArgs& d, hipStream_t st) {
    if (variant != 7) return false;   // the 2-slot ring one tile ahead
    if (d.mask)
        k_attn_dq_d64<true, 2><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale,
                                                     d.mask, d.dscale);
    else
        k_attn_dq_d64<false, 2><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale,
                                                      nullptr, 1.f);
    return true;
}

bool launch_dkdv(int variant, dim3 grid, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v,
                 int64_t ld, const bf16_t* dout, int64_t ldd, const float* lse, const float* delta, bf16_t* dk,
                 bf16_t* dv, int64_t lddkv, float scale, const DropArgs& d, hipStream_t st) {
    if (variant != 7) return false;   // the 2-slot ring one tile ahead
    if (d.mask)
        k_attn_dkdv_d64<true, 2><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale,
                                                       d.mask_bwd, d.dscale);
    else
        k_attn_dkdv_d64<false, 2><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv,
                                                        scale, nullptr, 1.f);
    return true;
}
}  // namespace attn_ab

}  // namespace cg
