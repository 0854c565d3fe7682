// charpt HIP library -- shared device/host helpers (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/charpt.h"

// ---------------------------------------------------------------------------------------
// error convention: every entry point returns CG_OK or an error code and records a message
// retrievable through cg_last_error_string() (thread-local).
// ---------------------------------------------------------------------------------------
namespace cg {
void set_error(const char* fmt, ...);
// out[n] (=|+=) sum_k part[k*N + n] in a fixed order (deterministic); columns n >= S go to
// out_b[n - S] (either output may be NULL to drop it).  Defined in util.hip.
void launch_reduce_partials(const float* part, int64_t K, int64_t N, float* out_a, float* out_b, int64_t S,
                            int accumulate, hipStream_t st);
// three segments of S columns: out_a, out_b (accumulate), out_c (accumulate_c)
void launch_reduce_partials3(const float* part, int64_t K, int64_t N, float* out_a, float* out_b, float* out_c,
                             int64_t S, int accumulate, int accumulate_c, hipStream_t st);
// the same, queued on stream st's deferral queue when defer (CG_DEFER; one multi-job launch at
// cg_flush_deferred(st), defer.h); an immediate reduce into a queued job's outputs flushes them first
void reduce_partials_deferrable(const float* part, int64_t K, int64_t N, float* out_a, float* out_b, float* out_c,
                                int64_t S, int accumulate, int accumulate_c, int defer, hipStream_t st);
}  // namespace cg

namespace cg {
// One 16-B-per-lane LDS-DMA (global_load_lds_dwordx4: lane l's 16 bytes from g land at LDS byte
// lds + 16 l; lds must be wave-uniform) issued from inline asm, so the compiler does not see an LDS
// DMA.  Seen (the __builtin_amdgcn_global_load_lds form), it makes every later LDS read it cannot
// prove disjoint wait for ALL outstanding DMAs (s_waitcnt vmcnt(0) before the ds_read): a ring's
// in-flight prefetch stages are then waited for before the current stage is read, i.e. no
// pipelining beyond one stage.  Callers wait for these DMAs with their own s_waitcnt vmcnt(N).
// vmcnt retires in issue order, so the compiler's own waits stay correct but count only the loads
// it knows: a compiler-visible load issued BEFORE hidden DMAs is waited for as if the DMAs had
// landed too -- issue register loads after the DMAs they should not wait for.  The "memory"
// clobber keeps loads/stores from being scheduled across the DMA.  m0 is clobbered; nothing else
// in these kernels uses it (gfx9+ LDS access does not).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const void* g, const void* lds) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
}
// the same with a wave-uniform base in an SGPR pair and a per-lane 32-bit byte offset (saddr form):
// one VGPR per lane instead of a 64-bit address, and loop-invariant lane offsets
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, const void* lds) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l)
                 : "memory", "m0");
}
// the same with the LDS destination already a 32-bit LDS byte address (wave-uniform)
__device__ __forceinline__ void dma16sl(const void* sbase, uint32_t voff, uint32_t lds) {
    const uint32_t l = __builtin_amdgcn_readfirstlane(lds);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l)
                 : "memory", "m0");
}
// LDS byte address of a pointer into a __shared__ array (fold the cast once per kernel)
__device__ __forceinline__ uint32_t lds_base(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
#pragma clang diagnostic pop
}  // namespace cg

#define CG_REQUIRE(cond, ...)                \
    do {                                     \
        if (!(cond)) {                       \
            cg::set_error(__VA_ARGS__);      \
            return CG_EINVAL;                \
        }                                    \
    } while (0)

#define CG_LAUNCH_CHECK(name)                                                        \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess) {                                                      \
            cg::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));      \
            return CG_EHIP;                                                          \
        }                                                                            \
    } while (0)

namespace cg {

typedef unsigned short bf16_t;  // raw bf16 bits in memory
typedef short sv8 __attribute__((ext_vector_type(8)));
typedef short sv4 __attribute__((ext_vector_type(4)));
// Register loads hidden from hipcc's wait-count model, like dma16: a kernel that issues them ahead of
// its DMAs counts them in its own vmcnt and must name every destination "+v" in the statement that
// waits for them (cdna_hip_programming.md 5.7 item 1 (ii)) before anything reads them.
__device__ __forceinline__ void gload16(sv8& dst, const void* g) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(g) : "memory");
}
__device__ __forceinline__ void gload4(uint32_t& dst, const void* g) {
    asm volatile("global_load_dword %0, %1, off" : "=v"(dst) : "v"(g) : "memory");
}
// saddr forms: wave-uniform base in an SGPR pair + per-lane 32-bit byte offset
__device__ __forceinline__ void gload4s(uint32_t& dst, const void* sbase, uint32_t voff) {
    asm volatile("global_load_dword %0, %1, %2" : "=v"(dst) : "v"(voff), "s"(sbase) : "memory");
}
typedef float fv4 __attribute__((ext_vector_type(4)));

// A GEMM output's 16-B store.  CG_STORE_SC1 (A/B build, make sc1): global_store_dwordx4 ... sc1 -- the
// line leaves the XCD's L2 (MI355X_MICROARCH.md store flavours) instead of staying there dirty, so the
// output stream neither evicts the operand panels the LDS-DMA reads nor is written back at the kernel
// boundary.  The s_nop: the store reads its 128-bit data after issue, and hipcc's hazard recognizer
// does not see inside the asm (it reused the data registers as the next store's address at once).
template <typename T>
__device__ __forceinline__ void st_out16(T* p, const T& v) {
    static_assert(sizeof(T) == 16, "16-B stores");
#ifdef CG_STORE_SC1
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 d = __builtin_bit_cast(u32x4, v);
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
#else
    *p = v;
#endif
}
typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even f32 -> bf16: a plain __bf16 conversion compiles to gfx950's
// v_cvt_pk_bf16_f32 (one instruction for two values; the integer RNE sequence it replaces cost
// ~5 VALU per value in every bf16-writing epilogue).  NaN stays NaN.
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    const bf2v v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

template <typename T>
__device__ __forceinline__ float ld_as_f32(const T* p);
template <>
__device__ __forceinline__ float ld_as_f32<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld_as_f32<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <typename T>
__device__ __forceinline__ void st_from_f32(T* p, float v);
template <>
__device__ __forceinline__ void st_from_f32<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st_from_f32<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// ---------------------------------------------------------------------------------------
// wave64 reductions
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// wave64 sum through DPP (no LDS round trips): quad butterflies, row rotations, then the
// row_bcast:15 / row_bcast:31 steps carry the row sums into row 3; lane 63 holds the total and
// is broadcast with readlane.  Fixed association order (deterministic).  Every lane of the wave
// must be active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf,
                                                                 false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_f<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x124, 0xf>(v);  // row_ror:4
    v += dpp_f<0x128, 0xf>(v);  // row_ror:8   -> every lane holds its row's sum
    v += dpp_f<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3 add rows 0, 2
    v += dpp_f<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3 add row 1 (= rows 0 + 1)
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// sum over the 16 lanes of each DPP row (lanes 16r .. 16r + 15) with no LDS round trip: the quad
// butterflies and two row rotations of wave_sum_dpp.  Every lane ends with its row's sum; the
// association depends on the lane's quad (fixed run to run), so read one fixed lane per row.  Every
// lane of the wave must be active.  (__shfl_xor over 1, 2, 4, 8 compiled to four ds_bpermute_b32:
// LDS-pipe instructions with LDS latency in a dependent chain.)
__device__ __forceinline__ float row16_sum_dpp(float v) {
    v += dpp_f<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x124, 0xf>(v);  // row_ror:4
    v += dpp_f<0x128, 0xf>(v);  // row_ror:8
    return v;
}

// ---------------------------------------------------------------------------------------
// Philox4x32-10 counter-based dropout RNG (spec: oracle/philox.py; DESIGN.md "Dropout").
// 16-bit keep decisions, 8 consecutive elements per Philox call:
//   element idx -> ctr = (idx>>3 lo, idx>>3 hi, stream lo, stream hi), key = seed,
//   u16 = half (idx&1) of word ((idx>>1)&3);  keep = u16 >= thr (thr = round(p * 2^16))
// ---------------------------------------------------------------------------------------
struct u32x4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one v_mad_u64_u32 per product (hi and lo together) instead of v_mul_lo_u32 + v_mul_hi_u32
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        // three-input XORs as one gfx950 v_bitop3_b32 each (truth table 0x96): 20 VALU per call saved
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    return {c0, c1, c2, c3};
}

// Philox output of one counter group (elements [8*group, 8*group+8) of a dropout stream)
__device__ __forceinline__ u32x4 philox_group(uint64_t seed, uint64_t stream, uint64_t group) {
    return philox4x32_10((uint32_t)group, (uint32_t)(group >> 32), (uint32_t)stream, (uint32_t)(stream >> 32),
                         (uint32_t)seed, (uint32_t)(seed >> 32));
}

__device__ __forceinline__ uint32_t philox_word(const u32x4& r, int w) {
    return w == 0 ? r.x : (w == 1 ? r.y : (w == 2 ? r.z : r.w));
}

// Philox of the group holding element idx
__device__ __forceinline__ u32x4 philox_of(uint64_t seed, uint64_t stream, uint64_t idx) {
    return philox_group(seed, stream, idx >> 3);
}

// keep decision of element idx from its group's Philox output r
__device__ __forceinline__ bool keep_of(const u32x4& r, uint64_t idx, uint32_t thr) {
    const uint32_t w = philox_word(r, (int)((idx >> 1) & 3));
    return ((idx & 1) ? (w >> 16) : (w & 0xffffu)) >= thr;
}

// keep bits (bit q <-> element idx + q) of the 4 consecutive elements idx..idx+3, idx % 4 == 0:
// one Philox call, half of its output
__device__ __forceinline__ uint32_t keep4_bits(uint64_t seed, uint64_t stream, uint64_t idx, uint32_t thr) {
    const u32x4 r = philox_group(seed, stream, idx >> 3);
    const bool hi = (idx >> 2) & 1;
    const uint32_t a = hi ? r.z : r.x, b = hi ? r.w : r.y;
    return (uint32_t)((a & 0xffffu) >= thr) | ((uint32_t)((a >> 16) >= thr) << 1) |
           ((uint32_t)((b & 0xffffu) >= thr) << 2) | ((uint32_t)((b >> 16) >= thr) << 3);
}

// keep bits of 8 consecutive elements 8*group .. 8*group+7 (bit e <-> element 8*group + e)
__device__ __forceinline__ uint32_t keep8_bits(const u32x4& r, uint32_t thr) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
    uint32_t bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const uint32_t u = (e & 1) ? (w[e >> 1] >> 16) : (w[e >> 1] & 0xffffu);
        bits |= (uint32_t)(u >= thr) << e;
    }
    return bits;
}

__device__ __forceinline__ uint64_t dropout_stream(const uint64_t* rng_call, int site) {
    return (rng_call ? (*rng_call << 8) : 0ull) | (uint64_t)(site & 0xff);
}

// 16-bit threshold: drop iff u16 < thr.  Any p > 0 gives thr >= 1, so thr != 0 <=> dropout on.
inline uint32_t dropout_threshold(double p) {
    if (!(p > 0)) return 0u;
    const double r = __builtin_nearbyint(p * 65536.0);
    return r < 1.0 ? 1u : (r >= 65535.0 ? 65535u : (uint32_t)r);
}

inline float dropout_scale(double p) { return (float)(1.0 / (1.0 - p)); }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace cg
