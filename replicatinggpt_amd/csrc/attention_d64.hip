// charpt: bf16 MFMA causal attention for head_size 64 -- the launchers (kernels: attention_d64.h;
// the A/B-only variants: ab/attention_ab.hip).  GPT1.py:109-123,134-135.
#include "attention_d64.h"

namespace cg {
int g_attn_variant = 0;
int g_attn_bwd_lpt = 1;   // merged resident backward: dK/dV workgroups first per XCD (0: interleaved, A/B)


namespace attn {
// sequence-resident kernels for T <= 256 unless cg_set_tuning("attn_variant", 1) selects the ring
// kernels (A/B and tests); attn_variant 2: resident dQ and dK/dV as two launches instead of one
static bool resident(int64_t T) { return T <= 256 && g_attn_variant != 1; }
#define RES_SWITCH(T, ...)                  \
    switch ((int)((T) / 64)) {              \
        case 1: { constexpr int NT_ = 1; __VA_ARGS__; } break; \
        case 2: { constexpr int NT_ = 2; __VA_ARGS__; } break; \
        case 3: { constexpr int NT_ = 3; __VA_ARGS__; } break; \
        default: { constexpr int NT_ = 4; __VA_ARGS__; } break; \
    }

void launch_fwd_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    bf16_t* o, int64_t ldo, float* lse, float scale, const DropArgs& d, hipStream_t st) {
    if (resident(T)) {
        const float sl2 = scale * LOG2E;
        RES_SWITCH(T, if (d.mask) k_attn_fwd_d64r<true, NT_><<<dim3(1, (unsigned)(B * H)), 256, 0, st>>>(
                              H, q, k, v, ld, o, ldo, lse, sl2, d.mask, d.dscale);
                   else k_attn_fwd_d64r<false, NT_><<<dim3(1, (unsigned)(B * H)), 256, 0, st>>>(
                              H, q, k, v, ld, o, ldo, lse, sl2, nullptr, 1.f));
        return;
    }
    const dim3 grid((unsigned)((ceil_div(T, 256) + 1) / 2), (unsigned)(B * H));   // pairs of query blocks
#ifdef CG_AB_VARIANTS   // attn_variant 4 / 5 / 6: ab/attention_ab.hip
    if (attn_ab::launch_fwd(g_attn_variant, grid, T, H, q, k, v, ld, o, ldo, lse, scale, d, st)) return;
#endif
    // Q fragments in registers, 4-slot LDS-DMA ring two tiles ahead: C4 forward 248 -> 223 us against
    // the register-staged ring, 244 us for the one-tile-ahead DMA ring with the Q image in LDS
    // (same-process interleaved A/B, profiles/r3_attn_fwd_ring_ab.txt)
    if (d.mask)
        k_attn_fwd_d64d<true, true><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, d.mask,
                                                          d.dscale);
    else
        k_attn_fwd_d64d<false, true><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, lse, scale * LOG2E, nullptr,
                                                           1.f);
}

void launch_dq_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                   const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, float* delta,
                   bf16_t* dq, int64_t lddq, float scale, const DropArgs& d, hipStream_t st) {
    if (resident(T)) {
        RES_SWITCH(T, if (d.mask) k_attn_dq_d64r<true, NT_><<<dim3(1, (unsigned)(B * H)), 256, 0, st>>>(
                              H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, d.mask, d.dscale);
                   else k_attn_dq_d64r<false, NT_><<<dim3(1, (unsigned)(B * H)), 256, 0, st>>>(
                              H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, nullptr, 1.f));
        return;
    }
    const dim3 grid((unsigned)((ceil_div(T, 256) + 1) / 2), (unsigned)(B * H));
#define DQ(NS_)                                                                                                    \
    do {                                                                                                           \
        if (d.mask)                                                                                                \
            k_attn_dq_d64<true, NS_><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, \
                                                           scale, d.mask, d.dscale);                               \
        else                                                                                                       \
            k_attn_dq_d64<false, NS_><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq,      \
                                                            lddq, scale, nullptr, 1.f);                            \
    } while (0)
#ifdef CG_AB_VARIANTS   // attn_variant 7: ab/attention_ab.hip
    if (attn_ab::launch_dq(g_attn_variant, grid, T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, d, st))
        return;
#endif
    DQ(4);
#undef DQ
}
bool bwd_merged(int64_t T) { return resident(T) && g_attn_variant != 2; }   // 2: the two resident kernels (A/B)

void launch_bwd_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                    const bf16_t* o, int64_t ldo, const bf16_t* dout, int64_t ldd, const float* lse, float* delta,
                    bool delta_ready, bf16_t* dq, int64_t lddq, bf16_t* dk, bf16_t* dv, int64_t lddkv, float scale,
                    const DropArgs& d, hipStream_t st) {
    if (bwd_merged(T)) {
        const dim3 grid(1, (unsigned)(2 * B * H));
#define BWDR(DIN_)                                                                                                 \
    RES_SWITCH(T, if (d.mask) k_attn_bwd_d64r<true, NT_, DIN_><<<grid, 256, 0, st>>>(                            \
                          H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, dk, dv, lddkv, scale, d.mask,    \
                          d.mask_bwd, d.dscale, g_attn_bwd_lpt);                                                    \
               else k_attn_bwd_d64r<false, NT_, DIN_><<<grid, 256, 0, st>>>(                                     \
                          H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, dk, dv, lddkv, scale, nullptr,   \
                          nullptr, 1.f, g_attn_bwd_lpt))
        if (delta_ready) {
            BWDR(true);
        } else {
            BWDR(false);
        }
#undef BWDR
        return;
    }
    launch_dq_d64(B, T, H, q, k, v, ld, o, ldo, dout, ldd, lse, delta, dq, lddq, scale, d, st);
    launch_dkdv_d64(B, T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale, d, st);
}

void launch_dkdv_d64(int64_t B, int64_t T, int H, const bf16_t* q, const bf16_t* k, const bf16_t* v, int64_t ld,
                     const bf16_t* dout, int64_t ldd, const float* lse, const float* delta, bf16_t* dk, bf16_t* dv,
                     int64_t lddkv, float scale, const DropArgs& d, hipStream_t st) {
    if (resident(T)) {
        RES_SWITCH(T, if (d.mask) k_attn_dkdv_d64r<true, NT_><<<dim3(1, (unsigned)(B * H)), 256, 0, st>>>(
                              H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale, d.mask_bwd, d.dscale);
                   else k_attn_dkdv_d64r<false, NT_><<<dim3(1, (unsigned)(B * H)), 256, 0, st>>>(
                              H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale, nullptr, 1.f));
        return;
    }
    const dim3 grid((unsigned)((ceil_div(T, 128) + 1) / 2), (unsigned)(B * H));
#define DKDV(NS_)                                                                                                  \
    do {                                                                                                           \
        if (d.mask)                                                                                                \
            k_attn_dkdv_d64<true, NS_><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, \
                                                             scale, d.mask_bwd, d.dscale);                         \
        else                                                                                                       \
            k_attn_dkdv_d64<false, NS_><<<grid, 256, 0, st>>>(T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv,      \
                                                              lddkv, scale, nullptr, 1.f);                         \
    } while (0)
#ifdef CG_AB_VARIANTS   // attn_variant 7: ab/attention_ab.hip
    if (attn_ab::launch_dkdv(g_attn_variant, grid, T, H, q, k, v, ld, dout, ldd, lse, delta, dk, dv, lddkv, scale, d, st))
        return;
#endif
    DKDV(4);
#undef DKDV
}
}  // namespace attn

}  // namespace cg
