// charpt: LayerNorm forward/backward (nn.LayerNorm, GPT1.py:159-160,173), fp32 statistics.
// One wave64 per row; the row lives in registers: lane owns NJ chunks of VEC consecutive
// floats at e = (j*64 + lane)*VEC.  Specialised shapes: C = 384 (VEC 2, NJ 3), 768 (4, 3),
// 512 (4, 2), 1024 (4, 4), even C <= 128 (2, 1; forward); any other C <= 2048 uses (1, 32) with
// bounds checks.
#include <type_traits>

#include "common.h"
#include "ln_fwd.h"

using namespace cg;

namespace {

// non-temporal VEC-float load / store (VEC 2 or 4): the stream bypasses the caches' allocation
template <int VEC>
__device__ __forceinline__ void ld_nt(const float* p, float* v) {
    typedef float nfv __attribute__((ext_vector_type(VEC)));
    const nfv t = __builtin_nontemporal_load((const nfv*)p);
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = t[q];
}
template <int VEC>
__device__ __forceinline__ void st_nt(float* p, const float* v) {
    typedef float nfv __attribute__((ext_vector_type(VEC)));
    nfv t;
#pragma unroll
    for (int q = 0; q < VEC; ++q) t[q] = v[q];
    __builtin_nontemporal_store(t, (nfv*)p);
}

template <typename T>
__device__ __forceinline__ void ld_vec_any(const T* p, float* v, int n);
template <>
__device__ __forceinline__ void ld_vec_any<float>(const float* p, float* v, int n) {
    if (n == 4) VecIO<4>::ld(p, v);
    else if (n == 2) VecIO<2>::ld(p, v);
    else VecIO<1>::ld(p, v);
}
template <>
__device__ __forceinline__ void ld_vec_any<bf16_t>(const bf16_t* p, float* v, int n) {
    for (int i = 0; i < n; ++i) v[i] = bf2f(p[i]);
}

}  // namespace

template <int VEC, int NJ, typename TY, int RPW, bool FULL = false>
__global__ __launch_bounds__(256) void k_ln_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                                const float* __restrict__ b, TY* __restrict__ y,
                                                float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                int64_t rows, int C, float eps) {
    ln_fwd_rows<VEC, NJ, TY, RPW, FULL>(x, w, b, y, mean_out, rstd_out, rows, C, eps, (int)blockIdx.x, (int)gridDim.x);
}

// Backward rows per block: sized so the grid has ~512 blocks (2 per CU) at any token count, 8..256,
// a multiple of the 8 waves.  The per-block column partials (dgamma, dbeta, consumer bias) are
// [nblk][NP*C]: 512 x 2304 floats at C4.
namespace cg {
int g_ln_rpb = 0;     // cg_set_tuning("ln_rpb"): rows per backward block (0 = automatic)
int g_ln_waves = 0;   // cg_set_tuning("ln_waves"): waves per backward block, 4 or 8 (0 = automatic)
int g_ln_pf = 0;      // cg_set_tuning("ln_pf"): 1 = next row's loads before the current row (FULL shapes)
// cg_set_tuning("ln_rl"): 1 (default) = the NT backward rows at C = 384 issue the next row's loads after
// computing the current row's outputs and before storing them (0: load, compute, store per row -- each
// row's loads then wait for the previous row's stores, vmcnt counting both).  Not at C = 768: there the
// held outputs cost the 4-wave blocks a wave per SIMD (158 -> 184 VGPRs; 2 = there too, A/B: C4 step
// 50.85 -> 51.05 ms, profiles/r5_ln_bwd_row_order_ab.txt)
int g_ln_rl = 1;
// cg_set_tuning("ln_nt"): the backward's non-temporal streams (k_ln_bwd NTM) for the FULL C = 384 / 768
// rows; -1 (default) = 3: the residual gradient and x read and dx written non-temporally.  dx is read
// again only by the next LayerNorm backward, after the sublayer's GEMMs and attention, so caching it
// only evicts their operands: C4 rows kernel 172 -> 133 us (4.7 -> 6.0 TB/s), C4 step 54.0 -> 53.6 ms,
// C2 step 3.045 -> 3.038 ms (the C2 kernel alone 18.0 -> 18.4 us) -- profiles/r4_ln_nt_ab.txt
int g_ln_nt = -1;
}  // namespace cg
// Waves per backward block: 8, or 4 where the row kernel's registers cap a SIMD at 3 waves (the
// VEC 4 variants, C = 512..1024: 166 VGPRs at C = 768) -- 8-wave blocks then fit once per CU (8 of
// 12 wave slots), 4-wave blocks three times.  Blocks target one round over the CUs' slots.
static int ln_bwd_waves(int64_t C) {
    if (g_ln_waves == 4 || g_ln_waves == 8) return g_ln_waves;
    return (C >= 512 && C <= 1024 && C % 4 == 0) ? 4 : 8;
}
static int ln_bwd_rpb(int64_t rows, int64_t C) {
    const int W = ln_bwd_waves(C);
    if (g_ln_rpb > 0) return (g_ln_rpb + W - 1) / W * W;
    int64_t r = rows / (W == 8 ? 512 : 768);
    r = r < W ? W : (r > 256 ? 256 : r);
    return (int)((r + W - 1) / W * W);
}
static int64_t ln_bwd_blocks(int64_t rows, int64_t C) {
    const int rpb = ln_bwd_rpb(rows, C);
    return (rows + rpb - 1) / rpb;
}

// The consumer-side extras of the backward (the residual-stream gradient dx feeds the previous
// sublayer's backward, GPT1.py:163-164): a bf16 copy of it with that sublayer's dropout applied
// (FeedForward's nn.Dropout, GPT1.py:146 -- keep(idx = r*C + c) from the Philox stream, scaled), or
// a plain bf16 copy (the attention projection's input gradient), and the column sums of that
// tensor (the consumer's bias gradient, fp32 before rounding) -- fused here so the consumer needs
// neither a dropout / cast pass nor a column-sum pass over it.
struct LnLp {
    bf16_t* out;             // NULL: no copy
    uint32_t thr;            // dropout threshold (0: none)
    float dscale;
    uint64_t seed;
    const uint64_t* rng_call;
    int site;
    int csum;                // 1: column sums of the copy into part columns [2C, 3C)
};

template <int VEC, int NJ>
struct LnRow {
    float x[NJ][VEC], d[NJ][VEC], rv[NJ][VEC];
    float mu, rs;
};

// One wave per row, row in registers as in the forward; 8 waves per block, each walking rpb/8
// consecutive rows (rpb: ln_bwd_rpb).  Partials [block][NP*C]: dgamma, dbeta (+ consumer bias
// column sums), summed over the 8 waves in a fixed order.  Measured (tools/ln_bench.py): issuing
// the next row's loads before reducing the current one (double-buffered rows) gained nothing at
// C4 and lost 15-25 % at C2 (occupancy); ~4.8 TB/s at C4, 5.2 TB/s at C2 without dropout.
// NTM (VEC 2 / 4): 1 the residual gradient read non-temporally, 2 also x, 3 also the dx store
template <int VEC, int NJ, typename TDY, int WAVES, bool FULL = false, bool PF = false, int NTM = 0, bool RL = false>
__global__ __launch_bounds__(64 * WAVES) void k_ln_bwd(const TDY* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ w, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ dres, float* __restrict__ dx,
                                                           LnLp lp, float* __restrict__ part, int64_t rows, int C,
                                                           int rpb) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [4][NP*C]
    const int NP = lp.csum ? 3 : 2;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const float invC = 1.0f / (float)C;
    const uint64_t stream = lp.thr ? dropout_stream(lp.rng_call, lp.site) : 0;
    const int rpw = rpb / WAVES;
    float adw[NJ][VEC], adb[NJ][VEC], acs[NJ][VEC], wv[NJ][VEC];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int e = (j * 64 + lane) * VEC;
#pragma unroll
        for (int q = 0; q < VEC; ++q) adw[j][q] = adb[j][q] = acs[j][q] = 0.f;
        if (FULL || e < C) VecIO<VEC>::ld(w + e, wv[j]);
        else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) wv[j][q] = 0.f;
        }
    }
    auto load = [&](int64_t r, LnRow<VEC, NJ>& b, auto hr) {
        constexpr bool HR = decltype(hr)::value;
        b.mu = mean[r];
        b.rs = rstd[r];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int e = (j * 64 + lane) * VEC;
            if (FULL || e < C) {
                if constexpr (NTM >= 2 && VEC >= 2) ld_nt<VEC>(x + r * C + e, b.x[j]);
                else VecIO<VEC>::ld(x + r * C + e, b.x[j]);
                ld_vec_any<TDY>(dy + r * C + e, b.d[j], VEC);
                if constexpr (HR && NTM >= 1 && VEC >= 2) ld_nt<VEC>(dres + r * C + e, b.rv[j]);
                else if (HR) VecIO<VEC>::ld(dres + r * C + e, b.rv[j]);
            }
        }
    };
    // Dropout keep bits of a row with C % 8 == 0: lane l evaluates Philox group l (+ 64 c) of the
    // row -- one call per 64 groups instead of one per lane and 8 / VEC lanes per group -- and each
    // lane fetches the byte of its own group with ds_bpermute (__shfl).  The group index c of
    // element e = (64 j + lane) VEC is (j VEC) >> 3 for every lane (no carry: 8 VEC <= 64).
    constexpr int NCALL = (NJ * VEC + 7) / 8;
    const bool row_groups = (C & 7) == 0;
    // ST: store the row's outputs here; else leave them in oo / zz for store_row (RL)
    auto process = [&](int64_t r, const LnRow<VEC, NJ>& b, auto hr, auto stc, float (&oo)[NJ][VEC],
                       float (&zz)[NJ][VEC]) {
        constexpr bool HR = decltype(hr)::value;
        constexpr bool ST = decltype(stc)::value;
        uint32_t kbyte[NJ];   // keep bits of the 8-group holding this lane's element e, per j
        if (lp.out && lp.thr && row_groups) {
            uint32_t kb[NCALL];
#pragma unroll
            for (int c = 0; c < NCALL; ++c) {
                const int gr = 64 * c + lane;
                kb[c] = 8 * gr < C ? keep8_bits(philox_group(lp.seed, stream, (uint64_t)r * (uint64_t)(C >> 3) + gr), lp.thr)
                                   : 0u;
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j)   // all lanes active (a bpermute source must be)
                kbyte[j] = (uint32_t)__shfl((int)kb[(j * VEC) >> 3], (((j * 64 + lane) * VEC) >> 3) & 63, 64);
        }
        float xh[NJ][VEC], g[NJ][VEC];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int e = (j * 64 + lane) * VEC;
            if (FULL || e < C) {
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    xh[j][q] = (b.x[j][q] - b.mu) * b.rs;
                    g[j][q] = b.d[j][q] * wv[j][q];
                    s1 += g[j][q];
                    s2 += g[j][q] * xh[j][q];
                    adw[j][q] += b.d[j][q] * xh[j][q];
                    adb[j][q] += b.d[j][q];
                }
            }
        }
        const float c1 = wave_sum_dpp(s1) * invC;
        const float c2 = wave_sum_dpp(s2) * invC;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int e = (j * 64 + lane) * VEC;
            if (FULL || e < C) {
                float o[VEC];
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    o[q] = b.rs * (g[j][q] - c1 - xh[j][q] * c2);
                    if (HR) o[q] += b.rv[j][q];
                }
                if constexpr (ST) {
                    if constexpr (NTM >= 3 && VEC >= 2) st_nt<VEC>(dx + r * C + e, o);
                    else VecIO<VEC>::st(dx + r * C + e, o);
                } else {
#pragma unroll
                    for (int q = 0; q < VEC; ++q) oo[j][q] = o[q];
                }
                if (lp.out) {
                    float z[VEC];
                    if (lp.thr && row_groups) {
#pragma unroll
                        for (int q = 0; q < VEC; ++q) z[q] = ((kbyte[j] >> ((e & 7) + q)) & 1u) ? o[q] * lp.dscale : 0.f;
                    } else if (lp.thr) {
                        const uint64_t idx = (uint64_t)r * (uint64_t)C + (uint64_t)e;
                        u32x4 ph = philox_of(lp.seed, stream, idx);
#pragma unroll
                        for (int q = 0; q < VEC; ++q) {
                            const uint64_t iq = idx + q;
                            if (q > 0 && (iq & 7) == 0) ph = philox_of(lp.seed, stream, iq);
                            z[q] = keep_of(ph, iq, lp.thr) ? o[q] * lp.dscale : 0.f;
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < VEC; ++q) z[q] = o[q];
                    }
                    if constexpr (ST) {
                        VecIO<VEC>::st(lp.out + r * C + e, z);
                    } else {
#pragma unroll
                        for (int q = 0; q < VEC; ++q) zz[j][q] = z[q];
                    }
#pragma unroll
                    for (int q = 0; q < VEC; ++q) acs[j][q] += z[q];
                }
            }
        }
    };
    auto store_row = [&](int64_t r, const float (&oo)[NJ][VEC], const float (&zz)[NJ][VEC]) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int e = (j * 64 + lane) * VEC;
            if (FULL || e < C) {
                if constexpr (NTM >= 3 && VEC >= 2) st_nt<VEC>(dx + r * C + e, oo[j]);
                else VecIO<VEC>::st(dx + r * C + e, oo[j]);
                if (lp.out) VecIO<VEC>::st(lp.out + r * C + e, zz[j]);
            }
        }
    };
    const int64_t r0 = (int64_t)blockIdx.x * rpb + (int64_t)wave * rpw;
    const int n = (int)(r0 < rows ? (rows - r0 < rpw ? rows - r0 : rpw) : 0);
    // the residual-gradient presence as a compile-time branch of the row loop: with FULL rows (C =
    // 64 VEC NJ, no lane guards) a row's loads are then one basic block, issued back to back
    // PF: the next row's loads are issued before the current row is processed (two rows in flight per
    // wave; more VGPRs -- cg_set_tuning("ln_pf"))
    // RL: the next row's loads are issued after the current row's outputs are computed and before
    // they are stored, so they do not wait for those stores (one row of loads in flight, as before)
    float oo[NJ][VEC], zz[NJ][VEC];
    auto row_loop = [&](auto hr) {
        if constexpr (PF) {
            if (n > 0) {
                LnRow<VEC, NJ> A;
                load(r0, A, hr);
#pragma unroll 1
                for (int i = 0; i < n; ++i) {
                    LnRow<VEC, NJ> Bn;
                    if (i + 1 < n) load(r0 + i + 1, Bn, hr);
                    process(r0 + i, A, hr, std::true_type{}, oo, zz);
                    A = Bn;
                }
            }
        } else if constexpr (RL) {
            if (n > 0) {
                LnRow<VEC, NJ> A;
                load(r0, A, hr);
#pragma unroll 1
                for (int i = 0; i < n; ++i) {
                    process(r0 + i, A, hr, std::false_type{}, oo, zz);
                    if (i + 1 < n) load(r0 + i + 1, A, hr);
                    __builtin_amdgcn_sched_barrier(0);
                    store_row(r0 + i, oo, zz);
                }
            }
        } else {
#pragma unroll 1
            for (int i = 0; i < n; ++i) {
                LnRow<VEC, NJ> A;
                load(r0 + i, A, hr);
                process(r0 + i, A, hr, std::true_type{}, oo, zz);
            }
        }
    };
    if (dres) row_loop(std::true_type{});
    else row_loop(std::false_type{});
    // column partials of the block: waves w and w + 4 pairwise, then waves 0..3 in order
    const int NC = NP * C;
    auto put = [&](bool add) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int e = (j * 64 + lane) * VEC;
            if (FULL || e < C) {
                float* dst = red + (wave & 3) * NC + e;
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    dst[q] = add ? dst[q] + adw[j][q] : adw[j][q];
                    dst[C + q] = add ? dst[C + q] + adb[j][q] : adb[j][q];
                    if (NP == 3) dst[2 * C + q] = add ? dst[2 * C + q] + acs[j][q] : acs[j][q];
                }
            }
        }
    };
    if (WAVES == 8) {
        if (wave >= 4) put(false);
        __syncthreads();
        if (wave < 4) put(true);
    } else {
        put(false);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NC; c += blockDim.x)
        part[(int64_t)blockIdx.x * NC + c] = ((red[c] + red[NC + c]) + red[2 * NC + c]) + red[3 * NC + c];
}

namespace {
template <typename TY>
int launch_ln_fwd(const float* x, const float* w, const float* b, TY* y, float* mean, float* rstd, int64_t rows,
                  int C, float eps, hipStream_t st) {
    const bool al16 = (((uintptr_t)x | (uintptr_t)w | (uintptr_t)b) & 15) == 0;
    const bool al8 = (((uintptr_t)x | (uintptr_t)w | (uintptr_t)b) & 7) == 0;
    if (C <= 128 && C % 2 == 0 && al8) {
        // narrow rows (C1 / C5: C = 126, 504 B): one 8-B chunk per lane and 8 rows per wave in flight --
        // the generic (1, 32) form issued 4-B loads through 32 bounds-checked chunks, 2 rows per wave
        // (28 us for the [65536, 126] decode window: 2.4 TB/s)
        if (rows < 8192) {   // generate()'s 256-row steps: one row per wave, every CU's share in flight at once
            k_ln_fwd<2, 1, TY, 1><<<ceil_div(rows, 4), 256, 0, st>>>(x, w, b, y, mean, rstd, rows, C, eps);
            return CG_OK;
        }
        constexpr int RPW8 = 8;
        int grid8 = ceil_div(rows, 4 * RPW8);
        grid8 = grid8 > 4096 ? 4096 : grid8;
        k_ln_fwd<2, 1, TY, RPW8><<<grid8, 256, 0, st>>>(x, w, b, y, mean, rstd, rows, C, eps);
        return CG_OK;
    }
    constexpr int RPW = 2;
    int grid = ceil_div(rows, 4 * RPW);
    grid = grid > 4096 ? 4096 : grid;
#define LNF(V, N, F) k_ln_fwd<V, N, TY, RPW, F><<<grid, 256, 0, st>>>(x, w, b, y, mean, rstd, rows, C, eps)
    if (C == 384 && al16) LNF(2, 3, true);   // FULL rows: C = 64 V N, no per-lane column guards
    else if (C == 768 && al16) LNF(4, 3, true);
    else if (C == 512 && al16) LNF(4, 2, true);
    else if (C == 1024 && al16) LNF(4, 4, true);
    else LNF(1, 32, false);
#undef LNF
    return CG_OK;
}

template <typename TDY>
int launch_ln_bwd(const TDY* dy, const float* x, const float* w, const float* mean, const float* rstd,
                  const float* dres, float* dx, const LnLp& lp, float* dw, float* db, float* dbias, int accumulate,
                  int dbias_accumulate, float* part, int64_t rows, int C, int defer, hipStream_t st) {
    const bool al16 = (((uintptr_t)x | (uintptr_t)w | (uintptr_t)dx | (uintptr_t)(dres ? dres : x)) & 15) == 0 &&
                      (((uintptr_t)dy) & 7) == 0 && (((uintptr_t)(lp.out ? lp.out : (bf16_t*)x)) & 7) == 0;
    const int64_t nblk = ln_bwd_blocks(rows, C);
    const int NP = lp.csum ? 3 : 2;
    const size_t lds = (size_t)4 * NP * C * sizeof(float);
    const int rpb = ln_bwd_rpb(rows, C);
    const int waves = ln_bwd_waves(C);
#define LNB_(V, N, F, P)                                                                                       \
    do {                                                                                                       \
        if (waves == 4)                                                                                        \
            k_ln_bwd<V, N, TDY, 4, F, P><<<(unsigned)nblk, 256, lds, st>>>(dy, x, w, mean, rstd, dres, dx, lp, part,    \
                                                                           rows, C, rpb);                      \
        else                                                                                                   \
            k_ln_bwd<V, N, TDY, 8, F, P><<<(unsigned)nblk, 512, lds, st>>>(dy, x, w, mean, rstd, dres, dx, lp, part,    \
                                                                           rows, C, rpb);                      \
    } while (0)
#define LNB_NT_(V, N, M_, RL_)                                                                                 \
    do {                                                                                                       \
        if (waves == 4)                                                                                        \
            k_ln_bwd<V, N, TDY, 4, true, false, M_, RL_><<<(unsigned)nblk, 256, lds, st>>>(                      \
                dy, x, w, mean, rstd, dres, dx, lp, part, rows, C, rpb);                                         \
        else                                                                                                   \
            k_ln_bwd<V, N, TDY, 8, true, false, M_, RL_><<<(unsigned)nblk, 512, lds, st>>>(                      \
                dy, x, w, mean, rstd, dres, dx, lp, part, rows, C, rpb);                                         \
    } while (0)
#define LNB_NT(V, N, M_)                  \
    do {                                  \
        if (g_ln_rl == 2 || (g_ln_rl && V == 2)) LNB_NT_(V, N, M_, true); \
        else LNB_NT_(V, N, M_, false);    \
    } while (0)
#define LNB(V, N, F)                        \
    do {                                    \
        if (F && g_ln_pf) LNB_(V, N, F, F); \
        else LNB_(V, N, F, false);          \
    } while (0)
    // the exact shapes run FULL rows (C = 64 V N: no per-lane column guards)
    const int ntm = g_ln_nt >= 0 ? g_ln_nt : 3;
    const bool nt_ok = al16 && !g_ln_pf && (C == 384 || C == 768);
    if (nt_ok && ntm == 1 && C == 384) LNB_NT(2, 3, 1);
    else if (nt_ok && ntm == 2 && C == 384) LNB_NT(2, 3, 2);
    else if (nt_ok && ntm == 3 && C == 384) LNB_NT(2, 3, 3);
    else if (nt_ok && ntm == 1 && C == 768) LNB_NT(4, 3, 1);
    else if (nt_ok && ntm == 2 && C == 768) LNB_NT(4, 3, 2);
    else if (nt_ok && ntm == 3 && C == 768) LNB_NT(4, 3, 3);
    else if (C == 384 && al16) LNB(2, 3, true);
    else if (C == 768 && al16) LNB(4, 3, true);
    else if (C == 512 && al16) LNB(4, 2, true);
    else if (C == 1024 && al16) LNB(4, 4, true);
    else LNB(1, 16, false);   // C <= 1024
#undef LNB
#undef LNB_
#undef LNB_NT
#undef LNB_NT_
    if (!defer && (dw || db || dbias))
        launch_reduce_partials3(part, nblk, NP * C, dw, db, dbias, C, accumulate, dbias_accumulate, st);
    return CG_OK;
}
}  // namespace

extern "C" int cg_layernorm_fwd(const float* x, const float* w, const float* b, void* y, int y_dtype, float* mean,
                                float* rstd, int64_t rows, int64_t C, float eps, void* stream) {
    CG_REQUIRE(rows > 0 && C > 0 && C <= 2048, "cg_layernorm_fwd: need 0 < C <= 2048 (got %lld)", (long long)C);
    hipStream_t st = (hipStream_t)stream;
    if (y_dtype == CG_BF16) launch_ln_fwd<bf16_t>(x, w, b, (bf16_t*)y, mean, rstd, rows, (int)C, eps, st);
    else launch_ln_fwd<float>(x, w, b, (float*)y, mean, rstd, rows, (int)C, eps, st);
    CG_LAUNCH_CHECK("cg_layernorm_fwd");
    return CG_OK;
}

extern "C" int64_t cg_layernorm_bwd_workspace(int64_t rows, int64_t C) {
    return ln_bwd_blocks(rows, C) * 3 * C * (int64_t)sizeof(float);
}

static int layernorm_bwd_impl(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                                   const float* rstd, const float* dres, float* dx, uint16_t* lp_out,
                                   double lp_dropout_p, uint64_t lp_seed, const uint64_t* lp_rng_call, int lp_site,
                                   float* dw, float* db, float* lp_colsum, int accumulate, int colsum_accumulate,
                                   void* workspace, int64_t rows, int64_t C, int defer, void* stream) {
    CG_REQUIRE(rows > 0 && C > 0 && C <= 1024, "cg_layernorm_bwd: need 0 < C <= 1024");
    CG_REQUIRE(lp_dropout_p >= 0 && lp_dropout_p < 1, "cg_layernorm_bwd_ex: dropout p must be in [0, 1)");
    CG_REQUIRE(!lp_colsum || lp_out, "cg_layernorm_bwd_ex: lp_colsum needs lp_out");
    hipStream_t st = (hipStream_t)stream;
    LnLp lp;
    lp.out = (bf16_t*)lp_out;
    lp.thr = lp_dropout_p > 0 ? dropout_threshold(lp_dropout_p) : 0u;
    lp.dscale = lp_dropout_p > 0 ? dropout_scale(lp_dropout_p) : 1.f;
    lp.seed = lp_seed;
    lp.rng_call = lp_rng_call;
    lp.site = lp_site;
    lp.csum = lp_colsum != nullptr;
    if (dy_dtype == CG_BF16)
        launch_ln_bwd<bf16_t>((const bf16_t*)dy, x, w, mean, rstd, dres, dx, lp, dw, db, lp_colsum, accumulate,
                              colsum_accumulate, (float*)workspace, rows, (int)C, defer, st);
    else
        launch_ln_bwd<float>((const float*)dy, x, w, mean, rstd, dres, dx, lp, dw, db, lp_colsum, accumulate,
                             colsum_accumulate, (float*)workspace, rows, (int)C, defer, st);
    CG_LAUNCH_CHECK("cg_layernorm_bwd");
    return CG_OK;
}

extern "C" int cg_layernorm_bwd_ex(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                                   const float* rstd, const float* dres, float* dx, uint16_t* lp_out,
                                   double lp_dropout_p, uint64_t lp_seed, const uint64_t* lp_rng_call, int lp_site,
                                   float* dw, float* db, float* lp_colsum, int accumulate, int colsum_accumulate,
                                   void* workspace, int64_t rows, int64_t C, void* stream) {
    return layernorm_bwd_impl(dy, dy_dtype, x, w, mean, rstd, dres, dx, lp_out, lp_dropout_p, lp_seed, lp_rng_call,
                              lp_site, dw, db, lp_colsum, accumulate, colsum_accumulate, workspace, rows, C, 0, stream);
}

// The row kernel alone: its per-block column partials stay in the workspace for
// cg_layernorm_bwd_reduce (which the caller may launch on another stream, after this one).
extern "C" int cg_layernorm_bwd_rows(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                                     const float* rstd, const float* dres, float* dx, uint16_t* lp_out,
                                     double lp_dropout_p, uint64_t lp_seed, const uint64_t* lp_rng_call, int lp_site,
                                     int lp_colsum, void* workspace, int64_t rows, int64_t C, void* stream) {
    // dw/db only gate the (deferred) reduce; lp_colsum needs a non-null marker to select 3 partials
    float* marker = lp_colsum ? (float*)workspace : nullptr;
    return layernorm_bwd_impl(dy, dy_dtype, x, w, mean, rstd, dres, dx, lp_out, lp_dropout_p, lp_seed, lp_rng_call,
                              lp_site, nullptr, nullptr, marker, 0, 0, workspace, rows, C, 1, stream);
}

extern "C" int cg_layernorm_bwd_reduce_ex(const void* workspace, int64_t rows, int64_t C, int lp_colsum_partials,
                                          float* dw, float* db, float* lp_colsum, int accumulate,
                                          int colsum_accumulate, int flags, void* stream) {
    CG_REQUIRE(rows > 0 && C > 0 && C <= 1024, "cg_layernorm_bwd_reduce: need 0 < C <= 1024");
    CG_REQUIRE((flags & ~CG_DEFER) == 0, "cg_layernorm_bwd_reduce_ex: unknown flags %#x", flags);
    CG_REQUIRE(!lp_colsum || lp_colsum_partials, "cg_layernorm_bwd_reduce: lp_colsum needs the colsum partials");
    if (!dw && !db && !lp_colsum) return CG_OK;
    const int64_t nblk = ln_bwd_blocks(rows, C);
    const int NP = lp_colsum_partials ? 3 : 2;
    reduce_partials_deferrable((const float*)workspace, nblk, NP * C, dw, db, lp_colsum, C, accumulate,
                               colsum_accumulate, flags & CG_DEFER, (hipStream_t)stream);
    CG_LAUNCH_CHECK("cg_layernorm_bwd_reduce");
    return CG_OK;
}

extern "C" int cg_layernorm_bwd_reduce(const void* workspace, int64_t rows, int64_t C, int lp_colsum_partials,
                                       float* dw, float* db, float* lp_colsum, int accumulate, int colsum_accumulate,
                                       void* stream) {
    return cg_layernorm_bwd_reduce_ex(workspace, rows, C, lp_colsum_partials, dw, db, lp_colsum, accumulate,
                                      colsum_accumulate, 0, stream);
}

extern "C" int cg_layernorm_bwd(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                                const float* rstd, const float* dres, float* dx, uint16_t* dx_bf16, float* dw,
                                float* db, int accumulate, void* workspace, int64_t rows, int64_t C, void* stream) {
    return cg_layernorm_bwd_ex(dy, dy_dtype, x, w, mean, rstd, dres, dx, dx_bf16, 0.0, 0, nullptr, 0, dw, db, nullptr,
                               accumulate, 0, workspace, rows, C, stream);
}
