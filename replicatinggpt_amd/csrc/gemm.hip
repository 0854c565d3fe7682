// charpt: GEMMs for every nn.Linear in the hot path (GPT1.py:111-112,121,136,143,145,184),
// their dgrad/wgrad in the backward, and bias-gradient column sums.
//
//   C[m,n] = epilogue( sum_k A(m,k) * B(n,k) ),  A(m,k) = A[m*lda+k] | A[k*lda+m] (a_trans),
//                                                B(n,k) = B[n*ldb+k] | B[k*ldb+n] (b_trans).
//
// Two kernels:
//   * k_gemm_bf16  -- the perf path: 128x128x64 tiles, 4 waves (2x2, 64x64 each), bf16 MFMA
//     16x16x32 with fp32 accumulation, register-staged double-buffered LDS (one barrier per
//     K-tile), XOR-swizzled LDS images: K-contiguous operands are read with ds_read_b128,
//     M/N-contiguous ("transposed") operands with the gfx950 transpose read ds_read_b64_tr_b16,
//     so forward (NT), dgrad (NN) and wgrad (TN) share one kernel.  Epilogue staged through LDS
//     and stored 16 B per lane.  Needs M%128 = N%128 = K%64 = 0, 16-B aligned rows.
//   * k_gemm_generic -- exact-f32 MFMA (16x16x4 f32) on 64x64x16 tiles with bounds checks:
//     any shape/stride/dtype; the fp32 parity path and odd shapes (n_embd=126, V=65).
// Both support deterministic split-K through fp32 slabs reduced in a fixed order.
#include "common.h"

using namespace cg;

namespace {

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
};

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
            const u32x4 r = philox_group(e.seed, stream, idx >> 2);
            if (e.thr) v = philox_word(r, (int)(idx & 3)) >= e.thr ? v * e.dscale : 0.f;
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

// =====================================================================================
// generic exact-f32 GEMM
// =====================================================================================
constexpr int GBM = 64, GBN = 64, GBK = 16;

template <typename TA, typename TB, typename TC>
__global__ __launch_bounds__(256) void k_gemm_generic(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K,
                                                      const TA* __restrict__ A, int64_t lda,
                                                      const TB* __restrict__ B, int64_t ldb, TC* __restrict__ C,
                                                      int64_t ldc, EpiArgs epi, int split_k, int64_t kchunk,
                                                      float* __restrict__ ws) {
    __shared__ float As[GBK][GBM + 4];
    __shared__ float Bs[GBK][GBN + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t tilesN = (N + GBN - 1) / GBN;
    const int64_t m0 = (int64_t)(blockIdx.x / tilesN) * GBM;
    const int64_t n0 = (int64_t)(blockIdx.x % tilesN) * GBN;
    const int split = blockIdx.y;
    const int64_t kb = split * kchunk;
    const int64_t ke = kb + kchunk < K ? kb + kchunk : K;

    fv4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    for (int64_t k0 = kb; k0 < ke; k0 += GBK) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int mm, kk;
            if (!a_trans) {
                kk = tid & 15;
                mm = (tid >> 4) + 16 * i;
            } else {
                mm = tid & 63;
                kk = (tid >> 6) + 4 * i;
            }
            const int64_t gm = m0 + mm, gk = k0 + kk;
            float v = 0.f;
            if (gm < M && gk < ke) v = ld_as_f32<TA>(A + (a_trans ? gk * lda + gm : gm * lda + gk));
            As[kk][mm] = v;
            int nn;
            if (!b_trans) {
                kk = tid & 15;
                nn = (tid >> 4) + 16 * i;
            } else {
                nn = tid & 63;
                kk = (tid >> 6) + 4 * i;
            }
            const int64_t gn = n0 + nn, gk2 = k0 + kk;
            float w = 0.f;
            if (gn < N && gk2 < ke) w = ld_as_f32<TB>(B + (b_trans ? gk2 * ldb + gn : gn * ldb + gk2));
            Bs[kk][nn] = w;
        }
        __syncthreads();
#pragma unroll
        for (int k4 = 0; k4 < GBK / 4; ++k4) {
            const int kr = k4 * 4 + (lane >> 4);
            float a0 = As[kr][wm * 32 + (lane & 15)];
            float a1 = As[kr][wm * 32 + 16 + (lane & 15)];
            float b0 = Bs[kr][wn * 32 + (lane & 15)];
            float b1 = Bs[kr][wn * 32 + 16 + (lane & 15)];
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }

    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + wm * 32 + mt * 16 + 4 * (lane >> 4) + r;
                const int64_t n = n0 + wn * 32 + nt * 16 + (lane & 15);
                if (m < M && n < N) {
                    if (split_k > 1) {
                        ws[((int64_t)split * M + m) * N + n] = acc[mt][nt][r];
                    } else {
                        store_out<TC>(C, m * ldc + n, epi_scalar(epi, acc[mt][nt][r], m, n, N, stream), epi.beta);
                    }
                }
            }
}

template <typename TC>
__global__ void k_splitk_reduce(const float* __restrict__ ws, int split_k, int64_t M, int64_t N, TC* __restrict__ C,
                                int64_t ldc, EpiArgs epi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int64_t m = i / N, n = i % N;
    float s = 0.f;
    for (int k = 0; k < split_k; ++k) s += ws[(int64_t)k * M * N + i];
    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
    store_out<TC>(C, m * ldc + n, epi_scalar(epi, s, m, n, N, stream), epi.beta);
}

// =====================================================================================
// fast bf16 MFMA GEMM
// =====================================================================================
constexpr int FBM = 128, FBN = 128, FBK = 64;
constexpr int F_STAGE_BYTES = 2 * 16384;  // A + B image per stage
constexpr int F_CS_LD = FBN + 4;          // epilogue staging row stride (floats)
constexpr int F_LDS_BYTES = (FBM * F_CS_LD * 4) > (2 * F_STAGE_BYTES) ? (FBM * F_CS_LD * 4) : (2 * F_STAGE_BYTES);

typedef __attribute__((address_space(3))) sv4 lds_sv4;

// K-contiguous image: [128 rows][64 k] bf16, 128-B rows, 16-B chunk c (0..7) swizzled by (r>>1)&7
__device__ __forceinline__ int img_row_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// M/N-contiguous image: [64 k][128 rows] bf16, 256-B rows, chunk c (0..15) swizzled (cdna guide T10 (b))
__device__ __forceinline__ int img_col_off(int k, int c) {
    return k * 256 + ((c ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 4);
}

template <bool TR>
struct Operand {
    // global -> registers for the tile whose first row (m or n) is r0 and first k is k0
    static __device__ __forceinline__ void load(uint4 (&g)[4], const bf16_t* __restrict__ X, int64_t ld, int64_t r0,
                                                int64_t k0, int tid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!TR) {
                const int r = (tid >> 3) + 32 * i, c = tid & 7;
                g[i] = *(const uint4*)(X + (r0 + r) * ld + k0 + c * 8);
            } else {
                const int k = (tid >> 4) + 16 * i, c = tid & 15;
                g[i] = *(const uint4*)(X + (k0 + k) * ld + r0 + c * 8);
            }
        }
    }
    static __device__ __forceinline__ void store(const uint4 (&g)[4], char* img, int tid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!TR) {
                const int r = (tid >> 3) + 32 * i, c = tid & 7;
                *(uint4*)(img + img_row_off(r, c)) = g[i];
            } else {
                const int k = (tid >> 4) + 16 * i, c = tid & 15;
                *(uint4*)(img + img_col_off(k, c)) = g[i];
            }
        }
    }
    // MFMA 16x16x32 operand fragment: rows rb..rb+15 of the tile, k-step s (k = 32s .. 32s+31)
    static __device__ __forceinline__ sv8 frag(const char* img, int rb, int s, int lane) {
        if (!TR) {
            const int r = rb + (lane & 15), c = s * 4 + (lane >> 4);
            return *(const sv8*)(img + img_row_off(r, c));
        } else {
            const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
            const int ka = 32 * s + 8 * g;
            const int chunk = (rb >> 3) + (p >> 1), byte = 8 * (p & 1);
            const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_col_off(ka + q, chunk) + byte));
            const sv4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_sv4*)(img + img_col_off(ka + 4 + q, chunk) + byte));
            return sv8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
    }
};

__device__ __forceinline__ fv4 mfma_bf16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

// bijective XCD-aware remap (cdna guide §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <bool AT, bool BT>
__global__ __launch_bounds__(256, 2) void k_gemm_bf16(int64_t M, int64_t N, int64_t K, const bf16_t* __restrict__ A,
                                                      int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
                                                      void* __restrict__ Cv, int c_dtype, int64_t ldc, EpiArgs epi,
                                                      int split_k, int64_t kchunk, float* __restrict__ ws) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tilesN = (int)(N / FBN);
    const int ntiles = (int)(M / FBM) * tilesN;
    const int t = xcd_remap(blockIdx.x, ntiles);
    const int64_t m0 = (int64_t)(t / tilesN) * FBM, n0 = (int64_t)(t % tilesN) * FBN;
    const int split = blockIdx.y;
    const int64_t kb = split * kchunk;
    const int nk = (int)(kchunk / FBK);

    fv4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    uint4 ga[4], gb[4];
    Operand<AT>::load(ga, A, lda, m0, kb, tid);
    Operand<BT>::load(gb, B, ldb, n0, kb, tid);
    Operand<AT>::store(ga, smem, tid);
    Operand<BT>::store(gb, smem + 16384, tid);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const char* imgA = smem + (kt & 1) * F_STAGE_BYTES;
        const char* imgB = imgA + 16384;
        const bool more = kt + 1 < nk;
        if (more) {
            Operand<AT>::load(ga, A, lda, m0, kb + (int64_t)(kt + 1) * FBK, tid);
            Operand<BT>::load(gb, B, ldb, n0, kb + (int64_t)(kt + 1) * FBK, tid);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            sv8 af[4], bf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = Operand<AT>::frag(imgA, wm * 64 + i * 16, s, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = Operand<BT>::frag(imgB, wn * 64 + j * 16, s, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma_bf16(af[i], bf[j], acc[i][j]);
        }
        if (more) {
            char* nxt = smem + ((kt + 1) & 1) * F_STAGE_BYTES;
            Operand<AT>::store(ga, nxt, tid);
            Operand<BT>::store(gb, nxt + 16384, tid);
        }
        __syncthreads();
    }

    // ---- epilogue: accumulators -> LDS (fp32, stride 132) -> 8 consecutive columns per lane
    float* Cs = (float*)smem;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                Cs[(wm * 64 + i * 16 + 4 * (lane >> 4) + r) * F_CS_LD + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();

    const uint64_t stream = (epi.kind == CG_EPI_BIAS_DROP_RESID && epi.thr) ? dropout_stream(epi.rng_call, epi.site) : 0;
#pragma unroll 1
    for (int pass = 0; pass < 8; ++pass) {
        const int row = pass * 16 + (tid >> 4), col = (tid & 15) * 8;
        const int64_t m = m0 + row, n = n0 + col;
        float v[8];
        {
            const float4 x0 = *(const float4*)(Cs + row * F_CS_LD + col);
            const float4 x1 = *(const float4*)(Cs + row * F_CS_LD + col + 4);
            v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
            v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
        }
        if (split_k > 1) {
            float* o = ws + ((int64_t)split * M + m) * N + n;
            *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
            *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
            continue;
        }
        const int kind = epi.kind;
        if (kind != CG_EPI_STORE && kind != CG_EPI_RELU_BWD && epi.bias) {
            const float4 b0 = *(const float4*)(epi.bias + n), b1 = *(const float4*)(epi.bias + n + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if (kind == CG_EPI_BIAS_RELU) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
        } else if (kind == CG_EPI_BIAS_DROP_RESID && epi.thr) {
            const uint64_t idx = (uint64_t)m * (uint64_t)N + (uint64_t)n;
            const u32x4 r0 = philox_group(epi.seed, stream, idx >> 2);
            const u32x4 r1 = philox_group(epi.seed, stream, (idx >> 2) + 1);
            const uint32_t w[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = w[q] >= epi.thr ? v[q] * epi.dscale : 0.f;
        } else if (kind == CG_EPI_RELU_BWD) {
            if (epi.aux_dtype == CG_BF16) {
                const uint4 h = *(const uint4*)((const bf16_t*)epi.aux + m * epi.ld_aux + n);
                const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    v[2 * q] = __uint_as_float(hw[q] << 16) > 0.f ? v[2 * q] : 0.f;
                    v[2 * q + 1] = __uint_as_float(hw[q] & 0xffff0000u) > 0.f ? v[2 * q + 1] : 0.f;
                }
            } else {
                const float* h = (const float*)epi.aux + m * epi.ld_aux + n;
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = h[q] > 0.f ? v[q] : 0.f;
            }
        }
        if ((kind == CG_EPI_BIAS_RESID || kind == CG_EPI_BIAS_DROP_RESID) && epi.resid) {
            const float* rp = epi.resid + m * epi.ld_resid + n;
            const float4 r0 = *(const float4*)rp, r1 = *(const float4*)(rp + 4);
            v[0] = r0.x + v[0]; v[1] = r0.y + v[1]; v[2] = r0.z + v[2]; v[3] = r0.w + v[3];
            v[4] = r1.x + v[4]; v[5] = r1.y + v[5]; v[6] = r1.z + v[6]; v[7] = r1.w + v[7];
        }
        if (c_dtype == CG_BF16) {
            bf16_t* o = (bf16_t*)Cv + m * ldc + n;
            if (epi.beta != 0.f) {
                const uint4 old = *(const uint4*)o;
                const uint32_t ow[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    v[2 * q] += epi.beta * __uint_as_float(ow[q] << 16);
                    v[2 * q + 1] += epi.beta * __uint_as_float(ow[q] & 0xffff0000u);
                }
            }
            *(uint4*)o = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                                    pack_bf2(v[6], v[7]));
        } else {
            float* o = (float*)Cv + m * ldc + n;
            if (epi.beta != 0.f) {
                const float4 o0 = *(const float4*)o, o1 = *(const float4*)(o + 4);
                v[0] += epi.beta * o0.x; v[1] += epi.beta * o0.y; v[2] += epi.beta * o0.z; v[3] += epi.beta * o0.w;
                v[4] += epi.beta * o1.x; v[5] += epi.beta * o1.y; v[6] += epi.beta * o1.z; v[7] += epi.beta * o1.w;
            }
            *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
            *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
}

// =====================================================================================
// column sums (bias gradients): out[n] (=|+=) sum_m X[m,n]
// =====================================================================================
constexpr int CS_ROWS = 256;

template <typename TX>
__global__ __launch_bounds__(256) void k_colsum_partial(const TX* __restrict__ X, int64_t rows, int64_t N,
                                                        int64_t ldx, float* __restrict__ part) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
    const int64_t n = (int64_t)blockIdx.x * 64 + c;
    const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS;
    float s = 0.f;
    if (n < N)
        for (int64_t r = r0 + rl; r < r0 + CS_ROWS && r < rows; r += 4) s += ld_as_f32<TX>(X + r * ldx + n);
    red[rl][c] = s;
    __syncthreads();
    if (rl == 0 && n < N) part[(int64_t)blockIdx.y * N + n] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

__global__ void k_colsum_final(const float* __restrict__ part, int64_t nchunk, int64_t N, float* __restrict__ out,
                               int accumulate) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    float s = 0.f;
    for (int64_t k = 0; k < nchunk; ++k) s += part[k * N + n];
    out[n] = accumulate ? out[n] + s : s;
}

EpiArgs make_epi(const cg_epilogue_t* e) {
    EpiArgs a;
    memset(&a, 0, sizeof(a));
    a.kind = CG_EPI_STORE;
    a.dscale = 1.f;
    if (!e) return a;
    a.kind = e->kind;
    a.bias = e->bias;
    a.resid = e->resid;
    a.ld_resid = e->ld_resid;
    a.aux = e->aux;
    a.aux_dtype = e->aux_dtype;
    a.ld_aux = e->ld_aux;
    a.thr = e->dropout_p > 0 ? dropout_threshold(e->dropout_p) : 0u;
    a.dscale = e->dropout_p > 0 ? dropout_scale(e->dropout_p) : 1.f;
    a.seed = e->seed;
    a.rng_call = e->rng_call;
    a.site = e->site;
    a.beta = e->beta;
    return a;
}

template <typename TA, typename TB>
int launch_generic(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                   const void* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const EpiArgs& e, int split_k,
                   void* ws, hipStream_t st) {
    int64_t kchunk = (K + split_k - 1) / split_k;
    kchunk = (kchunk + GBK - 1) / GBK * GBK;
    const int64_t tiles = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
    dim3 grid((unsigned)tiles, (unsigned)split_k);
    if (c_dtype == CG_BF16)
        k_gemm_generic<TA, TB, bf16_t><<<grid, 256, 0, st>>>(a_trans, b_trans, M, N, K, (const TA*)A, lda,
                                                             (const TB*)B, ldb, (bf16_t*)C, ldc, e, split_k, kchunk,
                                                             (float*)ws);
    else
        k_gemm_generic<TA, TB, float><<<grid, 256, 0, st>>>(a_trans, b_trans, M, N, K, (const TA*)A, lda,
                                                            (const TB*)B, ldb, (float*)C, ldc, e, split_k, kchunk,
                                                            (float*)ws);
    return CG_OK;
}

bool fast_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb, const void* C,
             int64_t ldc, int c_dtype, const EpiArgs& e, int split_k) {
    if (M % FBM || N % FBN || K % (FBK * split_k)) return false;
    if (lda % 8 || ldb % 8 || ldc % 8) return false;
    if ((((uintptr_t)A) | ((uintptr_t)B) | ((uintptr_t)C)) & 15) return false;
    if (e.bias && (((uintptr_t)e.bias) & 15)) return false;
    if (e.resid && ((((uintptr_t)e.resid) & 15) || e.ld_resid % 4)) return false;
    if (e.aux && ((((uintptr_t)e.aux) & 15) || e.ld_aux % 8)) return false;
    return true;
}

}  // namespace

extern "C" int64_t cg_gemm_workspace(int64_t M, int64_t N, int split_k) {
    return split_k > 1 ? (int64_t)split_k * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int cg_gemm(int op_dtype, int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, const void* A,
                       int64_t lda, const void* B, int64_t ldb, void* C, int c_dtype, int64_t ldc,
                       const cg_epilogue_t* epi, int split_k, void* workspace, void* stream) {
    CG_REQUIRE(M > 0 && N > 0 && K > 0, "cg_gemm: empty problem M=%lld N=%lld K=%lld", (long long)M, (long long)N,
               (long long)K);
    CG_REQUIRE(split_k >= 1 && split_k <= 64, "cg_gemm: split_k out of range");
    CG_REQUIRE(split_k == 1 || workspace, "cg_gemm: split_k > 1 needs a workspace");
    CG_REQUIRE(op_dtype == CG_BF16 || op_dtype == CG_F32, "cg_gemm: bad op dtype");
    hipStream_t st = (hipStream_t)stream;
    EpiArgs e = make_epi(epi);
    CG_REQUIRE(split_k == 1 || e.kind == CG_EPI_STORE || e.kind == CG_EPI_BIAS || e.kind == CG_EPI_BIAS_RESID,
               "cg_gemm: split-K supports STORE/BIAS/BIAS_RESID epilogues only");
    if (op_dtype == CG_BF16 && fast_ok(M, N, K, A, lda, B, ldb, C, ldc, c_dtype, e, split_k)) {
        const int64_t kchunk = K / split_k;
        dim3 grid((unsigned)((M / FBM) * (N / FBN)), (unsigned)split_k);
#define FG(AT, BT)                                                                                            \
    k_gemm_bf16<AT, BT><<<grid, 256, F_LDS_BYTES, st>>>(M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, \
                                                       c_dtype, ldc, e, split_k, kchunk, (float*)workspace)
        if (!a_trans && !b_trans) FG(false, false);
        else if (!a_trans && b_trans) FG(false, true);
        else if (a_trans && !b_trans) FG(true, false);
        else FG(true, true);
#undef FG
    } else if (op_dtype == CG_BF16) {
        launch_generic<bf16_t, bf16_t>(a_trans, b_trans, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k,
                                       workspace, st);
    } else {
        launch_generic<float, float>(a_trans, b_trans, M, N, K, A, lda, B, ldb, C, c_dtype, ldc, e, split_k,
                                     workspace, st);
    }
    if (split_k > 1) {
        const int64_t n = M * N;
        if (c_dtype == CG_BF16)
            k_splitk_reduce<bf16_t><<<ceil_div(n, 256), 256, 0, st>>>((const float*)workspace, split_k, M, N,
                                                                      (bf16_t*)C, ldc, e);
        else
            k_splitk_reduce<float><<<ceil_div(n, 256), 256, 0, st>>>((const float*)workspace, split_k, M, N,
                                                                     (float*)C, ldc, e);
    }
    CG_LAUNCH_CHECK("cg_gemm");
    return CG_OK;
}

extern "C" int64_t cg_colsum_workspace(int64_t rows, int64_t N) {
    return ((rows + CS_ROWS - 1) / CS_ROWS) * N * (int64_t)sizeof(float);
}

extern "C" int cg_colsum(const void* X, int x_dtype, int64_t rows, int64_t N, int64_t ldx, float* out, int accumulate,
                         void* workspace, void* stream) {
    CG_REQUIRE(rows > 0 && N > 0, "cg_colsum: empty");
    hipStream_t st = (hipStream_t)stream;
    const int64_t nchunk = (rows + CS_ROWS - 1) / CS_ROWS;
    dim3 grid(ceil_div(N, 64), (unsigned)nchunk);
    if (x_dtype == CG_BF16)
        k_colsum_partial<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)X, rows, N, ldx, (float*)workspace);
    else
        k_colsum_partial<float><<<grid, 256, 0, st>>>((const float*)X, rows, N, ldx, (float*)workspace);
    k_colsum_final<<<ceil_div(N, 256), 256, 0, st>>>((const float*)workspace, nchunk, N, out, accumulate);
    CG_LAUNCH_CHECK("cg_colsum");
    return CG_OK;
}
