// charpt: fused language-model head for the bf16 training path (GPT1.py:174,183-192):
//   logits = ln_f(x) @ lm_head.W^T + b   (V = 65 columns: never a GEMM-shaped problem on its own),
//   lse, cross entropy per row and the mean loss -- one kernel + one 1-block finish;
//   backward: dlogits = g/M (softmax - onehot) [+ g_logits] written as a zero-padded bf16 [M, KP]
//   operand for the dgrad / wgrad MFMA GEMMs, plus the deterministic bias-gradient partials.
//
// Forward layout: one wave per 16 rows; MFMA 16x16x32 with swapped operands (D = W_pad . a^T), so
// lane l holds row m = l & 15 and columns 16t + 4(l >> 4) + r: the row softmax reduces over 4VT
// registers and two cross-lane shuffles (xor 16, 32).  W_pad ([16 VT, C] bf16, rows >= V zero) and
// the row panel are read straight from global as MFMA fragments (W_pad is L2-resident: 50 KB).
#include "common.h"

namespace {
using namespace cg;

__device__ __forceinline__ fv4 mfma16(sv8 a, sv8 b, fv4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0,
                                                   0);
}

constexpr int HEAD_ROWS = 64;  // rows per 256-thread block (4 waves x 16)

// KS = C / 32 when known at compile time (all A fragments of the row panel loaded up front, so the
// wave has every global load in flight at once); KS = 0: runtime loop over K
template <int VT, int KS>
__global__ __launch_bounds__(256) void k_head_fwd(const bf16_t* __restrict__ a, int64_t C,
                                                  const bf16_t* __restrict__ wpad, const float* __restrict__ bias,
                                                  int V, const int64_t* __restrict__ tgt, float* __restrict__ logits,
                                                  float* __restrict__ lse, float* __restrict__ loss_part, int64_t M) {
    __shared__ float red[4];
    // the wave's 16 logit rows staged in LDS in their [row][V] memory order, then written as one
    // contiguous 16 V-float run with float4 stores (lane-per-row scalar stores touched 16 rows per
    // instruction: 16.6 us per C2 step for a 4.3 MB write)
    __shared__ __attribute__((aligned(16))) float stage[4][16 * 16 * VT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t m0 = (int64_t)blockIdx.x * HEAD_ROWS + wave * 16;
    float my_loss = 0.f;
    if (m0 < M) {
        const int64_t row = m0 + (lane & 15);
        const int kq = 8 * (lane >> 4);
        fv4 acc[VT];
#pragma unroll
        for (int t = 0; t < VT; ++t) acc[t] = fv4{0.f, 0.f, 0.f, 0.f};
        const bf16_t* ap = a + row * C + kq;
        const bf16_t* wp = wpad + (int64_t)(lane & 15) * C + kq;
        if constexpr (KS > 0) {
            sv8 af[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) af[ks] = *(const sv8*)(ap + 32 * ks);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                sv8 bf[VT];
#pragma unroll
                for (int t = 0; t < VT; ++t) bf[t] = *(const sv8*)(wp + (int64_t)16 * t * C + 32 * ks);
#pragma unroll
                for (int t = 0; t < VT; ++t) acc[t] = mfma16(bf[t], af[ks], acc[t]);
            }
        } else {
#pragma unroll 2
            for (int64_t k0 = 0; k0 < C; k0 += 32) {
                const sv8 af = *(const sv8*)(ap + k0);
#pragma unroll
                for (int t = 0; t < VT; ++t) {
                    const sv8 bf = *(const sv8*)(wp + (int64_t)16 * t * C + k0);
                    acc[t] = mfma16(bf, af, acc[t]);
                }
            }
        }
        // lane: row, columns n = 16t + 4(lane>>4) + r
        const int nb = 4 * (lane >> 4);
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < VT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * t + nb + r;
                const float x = n < V ? acc[t][r] + bias[n] : -INFINITY;
                acc[t][r] = x;
                mx = fmaxf(mx, x);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float s = 0.f;
        const int64_t tr = tgt ? tgt[row] : -1;
        float xt = 0.f;
#pragma unroll
        for (int t = 0; t < VT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * t + nb + r;
                if (n < V) {
                    s += __expf(acc[t][r] - mx);
                    stage[wave][(lane & 15) * V + n] = acc[t][r];
                    if (n == tr) xt = acc[t][r];
                }
            }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        xt += __shfl_xor(xt, 16, 64);
        xt += __shfl_xor(xt, 32, 64);
        // every lane's stage writes land before any lane of the wave reads them back
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        {
            const int64_t nrow = M - m0 < 16 ? M - m0 : 16;
            const int64_t cnt = nrow * V;           // floats of rows m0 .. m0 + nrow - 1, contiguous
            float* dst = logits + m0 * V;
            const float* src = stage[wave];
            if ((((uintptr_t)dst) & 15) == 0) {
                const int64_t c4 = cnt >> 2;
                for (int64_t i = lane; i < c4; i += 64) ((float4*)dst)[i] = ((const float4*)src)[i];
                for (int64_t i = 4 * c4 + lane; i < cnt; i += 64) dst[i] = src[i];
            } else {
                for (int64_t i = lane; i < cnt; i += 64) dst[i] = src[i];
            }
        }
        const float l = mx + __logf(s);
        if (lane < 16) {
            lse[row] = l;
            // F.cross_entropy raises on a target outside [0, V): here the loss turns NaN instead
            my_loss = (tgt && (tr < 0 || tr >= V)) ? __builtin_nanf("") : l - xt;
        }
    }
    // block partial of the loss sum (fixed order: lanes 0-15 of each wave, then waves)
    float w = my_loss;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
    if (lane == 0) red[wave] = w;
    __syncthreads();
    if (tid == 0 && loss_part) loss_part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(256) void k_head_loss_final(const float* __restrict__ part, int np, float scale,
                                                         float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < np; i += 256) s += part[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) *out = (((red[0] + red[1]) + red[2]) + red[3]) * scale;
}

// dl[m, c] (bf16, c < KP; zero for c >= V) and per-block column partials of the fp32 dl (c < V).
// 16 threads per row x 8 columns each; 16 rows per pass, HEAD_ROWS rows per block.
__global__ __launch_bounds__(256) void k_head_bwd(const float* __restrict__ logits, const float* __restrict__ lse,
                                                  const int64_t* __restrict__ tgt, const float* __restrict__ g_loss,
                                                  float g_mult, const float* __restrict__ g_logits, int V,
                                                  int64_t M, bf16_t* __restrict__ dl, int KP,
                                                  float* __restrict__ part) {
    __shared__ float red[16][129];
    const int tid = threadIdx.x, cg8 = tid & 15, rl = tid >> 4;
    const float gs = g_loss ? *g_loss * g_mult : 0.f;
    float colsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int c0 = 8 * cg8;
    for (int pass = 0; pass < HEAD_ROWS / 16; ++pass) {
        const int64_t m = (int64_t)blockIdx.x * HEAD_ROWS + pass * 16 + rl;
        if (m >= M) break;
        const float l = lse[m];
        const int64_t t = tgt ? tgt[m] : -1;
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int c = c0 + q;
            float d = 0.f;
            if (c < V) {
                const float x = logits[m * V + c];
                if (tgt) d = (t < 0 || t >= V) ? __builtin_nanf("") : gs * (__expf(x - l) - (c == t ? 1.f : 0.f));
                if (g_logits) d += g_logits[m * V + c];
            }
            v[q] = d;
            colsum[q] += d;
        }
        if (c0 < KP)
            *(uint4*)(dl + m * KP + c0) =
                make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) red[rl][c0 + q] = colsum[q];
    __syncthreads();
    if (tid < V) {
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) s += red[r][tid];
        part[(int64_t)blockIdx.x * V + tid] = s;
    }
}

}  // namespace

extern "C" int64_t cg_head_workspace(int64_t M, int64_t V) {
    const int64_t nb = (M + HEAD_ROWS - 1) / HEAD_ROWS;
    return (nb * (V > 1 ? V : 1) + 64) * (int64_t)sizeof(float);
}

extern "C" int cg_head_fwd(const void* a, const void* wpad, int64_t wpad_rows, const float* bias,
                           const int64_t* targets, float* logits, float* lse, float* loss, void* workspace,
                           int64_t M, int64_t C, int64_t V, void* stream) {
    CG_REQUIRE(M > 0 && C > 0 && V > 0, "cg_head_fwd: empty problem");
    CG_REQUIRE(M % 16 == 0 && C % 32 == 0, "cg_head_fwd: needs M %% 16 == 0 and C %% 32 == 0 (M=%lld C=%lld)",
               (long long)M, (long long)C);
    CG_REQUIRE(V <= 128 && wpad_rows >= ((V + 15) / 16) * 16, "cg_head_fwd: V=%lld needs wpad_rows >= %lld (<=128)",
               (long long)V, (long long)(((V + 15) / 16) * 16));
    CG_REQUIRE(((uintptr_t)a & 15) == 0 && ((uintptr_t)wpad & 15) == 0, "cg_head_fwd: operands must be 16-B aligned");
    CG_REQUIRE(!targets || (loss && workspace), "cg_head_fwd: targets need loss and workspace");
    hipStream_t st = (hipStream_t)stream;
    const int nb = ceil_div(M, HEAD_ROWS);
    float* part = targets ? (float*)workspace : nullptr;
    const int VT = (int)((V + 15) / 16);
#define HFK(vt, ks)                                                                                          \
    k_head_fwd<vt, ks><<<nb, 256, 0, st>>>((const bf16_t*)a, C, (const bf16_t*)wpad, bias, (int)V, targets, \
                                           logits, lse, part, M)
#define HF(vt)                          \
    if (C == 128) HFK(vt, 4);           \
    else if (C == 384) HFK(vt, 12);     \
    else if (C == 768) HFK(vt, 24);     \
    else HFK(vt, 0)
    switch (VT) {
        case 1: HF(1); break;
        case 2: HF(2); break;
        case 3: HF(3); break;
        case 4: HF(4); break;
        case 5: HF(5); break;
        case 6: HF(6); break;
        case 7: HF(7); break;
        default: HF(8); break;
    }
#undef HF
#undef HFK
    if (targets) k_head_loss_final<<<1, 256, 0, st>>>(part, nb, 1.f / (float)M, loss);
    CG_LAUNCH_CHECK("cg_head_fwd");
    return CG_OK;
}

extern "C" int cg_head_bwd_ex(const float* logits, const float* lse, const int64_t* targets, const float* g_loss,
                              float g_mult, const float* g_logits, void* dl, int64_t ld_dl, float* db,
                              int db_accumulate, void* workspace, int64_t M, int64_t V, int flags, void* stream) {
    CG_REQUIRE(M > 0 && V > 0 && V <= 128, "cg_head_bwd: bad sizes");
    CG_REQUIRE((flags & ~CG_DEFER) == 0, "cg_head_bwd_ex: unknown flags %#x", flags);
    CG_REQUIRE(ld_dl % 8 == 0 && ld_dl >= V && ld_dl <= 128, "cg_head_bwd: ld_dl must be a multiple of 8 in [V, 128]");
    CG_REQUIRE(!targets || g_loss, "cg_head_bwd: targets need g_loss");
    hipStream_t st = (hipStream_t)stream;
    const int nb = ceil_div(M, HEAD_ROWS);
    k_head_bwd<<<nb, 256, 0, st>>>(logits, lse, targets, g_loss, g_mult, g_logits, (int)V, M, (bf16_t*)dl, (int)ld_dl,
                                   (float*)workspace);
    if (db)   // CG_DEFER: queued on the stream's deferral queue (functional.DEFER, db a flat gradient slot)
        reduce_partials_deferrable((const float*)workspace, nb, V, db, nullptr, nullptr, V, db_accumulate, 0,
                                   flags & CG_DEFER, st);
    CG_LAUNCH_CHECK("cg_head_bwd");
    return CG_OK;
}

extern "C" int cg_head_bwd(const float* logits, const float* lse, const int64_t* targets, const float* g_loss,
                           float g_mult, const float* g_logits, void* dl, int64_t ld_dl, float* db, int db_accumulate,
                           void* workspace, int64_t M, int64_t V, void* stream) {
    return cg_head_bwd_ex(logits, lse, targets, g_loss, g_mult, g_logits, dl, ld_dl, db, db_accumulate, workspace, M,
                          V, 0, stream);
}
