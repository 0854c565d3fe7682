// charpt: error plumbing, counters, RNG helpers, reductions, batch gather.
#include <stdarg.h>

#include "common.h"
#include "defer.h"

namespace cg {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace cg

using namespace cg;

extern "C" const char* cg_last_error_string(void) { return g_err; }
extern "C" int cg_version(void) { return 1; }

extern "C" int cg_device_info(int* n_cu, int* major, int* minor) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) {
        set_error("cg_device_info: no HIP device");
        return CG_EHIP;
    }
    *n_cu = prop.multiProcessorCount;
    *major = prop.major;
    *minor = prop.minor;
    return CG_OK;
}

// --------------------------------------------------------------------------------------
__global__ void k_counter_add(int64_t* c, int64_t d) { *c += d; }
__global__ void k_rng_snapshot(uint64_t* c, uint64_t* s) {
    uint64_t v = *c;
    *s = v;
    *c = v + 1;
}

extern "C" int cg_counter_add(int64_t* counter, int64_t delta, void* stream) {
    k_counter_add<<<1, 1, 0, (hipStream_t)stream>>>(counter, delta);
    CG_LAUNCH_CHECK("cg_counter_add");
    return CG_OK;
}

extern "C" int cg_rng_snapshot(uint64_t* counter, uint64_t* snap, void* stream) {
    k_rng_snapshot<<<1, 1, 0, (hipStream_t)stream>>>(counter, snap);
    CG_LAUNCH_CHECK("cg_rng_snapshot");
    return CG_OK;
}

__global__ void k_dropout_mask(float* dst, int64_t n, uint32_t thr, uint64_t seed, const uint64_t* rng_call,
                               int site) {
    const uint64_t stream = dropout_stream(rng_call, site);
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // group of 8 consecutive elements
    const int64_t i0 = g * 8;
    if (i0 >= n) return;
    const uint32_t kb = keep8_bits(philox_group(seed, stream, (uint64_t)g), thr);
    for (int j = 0; j < 8 && i0 + j < n; ++j) dst[i0 + j] = ((kb >> j) & 1u) ? 1.f : 0.f;
}

extern "C" int cg_dropout_mask(float* dst, int64_t n, double p, uint64_t seed, const uint64_t* rng_call, int site,
                               void* stream) {
    CG_REQUIRE(n >= 0, "cg_dropout_mask: n < 0");
    if (n == 0) return CG_OK;
    const int64_t groups = (n + 7) / 8;
    k_dropout_mask<<<ceil_div(groups, 256), 256, 0, (hipStream_t)stream>>>(dst, n, dropout_threshold(p),
                                                                                 seed, rng_call, site);
    CG_LAUNCH_CHECK("cg_dropout_mask");
    return CG_OK;
}

// y = x * keep * 1/(1-p), element index r*C + c (FFN dropout backward, GPT1.py:146)
template <typename TY>
__global__ void k_dropout_apply(const float* __restrict__ x, int64_t rows, int64_t C, int64_t ldx, TY* __restrict__ y,
                                uint32_t thr, float dscale, uint64_t seed, const uint64_t* rng_call, int site) {
    const uint64_t stream = thr ? dropout_stream(rng_call, site) : 0;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // group of 8 consecutive elements
    const int64_t n = rows * C;
    const int64_t i0 = g * 8;
    if (i0 >= n) return;
    const uint32_t kb = thr ? keep8_bits(philox_group(seed, stream, (uint64_t)g), thr) : 0xffu;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + j;
        if (i < n) {
            const int64_t row = i / C, col = i % C;
            float v = x[row * ldx + col];
            if (thr) v = ((kb >> j) & 1u) ? v * dscale : 0.f;
            st_from_f32<TY>(y + i, v);
        }
    }
}

extern "C" int cg_dropout_apply(const float* x, int64_t rows, int64_t C, int64_t ldx, void* y, int y_dtype, double p,
                                uint64_t seed, const uint64_t* rng_call, int site, void* stream) {
    CG_REQUIRE(rows >= 0 && C > 0 && p >= 0 && p < 1, "cg_dropout_apply: bad args");
    const int64_t n = rows * C;
    if (n == 0) return CG_OK;
    const uint32_t thr = p > 0 ? dropout_threshold(p) : 0u;
    const float ds = p > 0 ? dropout_scale(p) : 1.f;
    const int grid = ceil_div((n + 7) / 8, 256);
    if (y_dtype == CG_BF16)
        k_dropout_apply<bf16_t><<<grid, 256, 0, (hipStream_t)stream>>>(x, rows, C, ldx, (bf16_t*)y, thr, ds, seed,
                                                                        rng_call, site);
    else
        k_dropout_apply<float><<<grid, 256, 0, (hipStream_t)stream>>>(x, rows, C, ldx, (float*)y, thr, ds, seed,
                                                                       rng_call, site);
    CG_LAUNCH_CHECK("cg_dropout_apply");
    return CG_OK;
}

// --------------------------------------------------------------------------------------
// column reduction of per-block partials [K][N] (LayerNorm dgamma/dbeta, bias column sums):
// 16 columns x 64 row-lanes per block, float4 loads, all of a lane's rows (8 at K = 512) in flight,
// then the 64 row-lane sums added in a fixed order (deterministic).  The former 32-column blocks
// (72 blocks at C4, 8 loads in flight per lane) ran 130 us for 9.4 MB.
// Column n goes to out_a[n] (n < S), out_b[n - S] (n < 2S) or out_c[n - 2S]; NULL drops it.
// One block's work (block blk of the job's ceil(N / 16)): shared by the single-job kernel and the
// deferred multi-job one, so both give the same bits.
__device__ __forceinline__ void reduce_partials_block(const float* __restrict__ part, int64_t K, int64_t N,
                                                      float* __restrict__ out_a, float* __restrict__ out_b,
                                                      float* __restrict__ out_c, int64_t S, int accumulate,
                                                      int accumulate_c, int64_t blk, float (*red)[17]) {
    const int cq = threadIdx.x & 3, rl = threadIdx.x >> 2;
    const int64_t n0 = blk * 16 + 4 * cq;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if ((N & 3) == 0 && (((uintptr_t)part) & 15) == 0) {
        if (n0 < N) {
            int64_t k = rl;
            for (; k + 7 * 64 < K; k += 8 * 64) {
                float4 v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = *(const float4*)(part + (k + 64 * j) * N + n0);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    a[0] += v[j].x;
                    a[1] += v[j].y;
                    a[2] += v[j].z;
                    a[3] += v[j].w;
                }
            }
            for (; k < K; k += 64) {
                const float4 v = *(const float4*)(part + k * N + n0);
                a[0] += v.x;
                a[1] += v.y;
                a[2] += v.z;
                a[3] += v.w;
            }
        }
    } else {
        for (int64_t k = rl; k < K; k += 64)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (n0 + q < N) a[q] += part[k * N + n0 + q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) red[rl][4 * cq + q] = a[q];
    __syncthreads();
    if (threadIdx.x < 16) {
        const int c = threadIdx.x;
        const int64_t n = blk * 16 + c;
        if (n < N) {
            float t = 0.f;
            for (int j = 0; j < 64; ++j) t += red[j][c];
            float* dst;
            int acc = accumulate;
            if (n < S) dst = out_a ? out_a + n : nullptr;
            else if (n < 2 * S) dst = out_b ? out_b + (n - S) : nullptr;
            else {
                dst = out_c ? out_c + (n - 2 * S) : nullptr;
                acc = accumulate_c;
            }
            if (dst) *dst = acc ? *dst + t : t;
        }
    }
}

__global__ __launch_bounds__(256) void k_reduce_partials(const float* __restrict__ part, int64_t K, int64_t N,
                                                         float* __restrict__ out_a, float* __restrict__ out_b,
                                                         float* __restrict__ out_c, int64_t S, int accumulate,
                                                         int accumulate_c) {
    __shared__ float red[64][17];
    reduce_partials_block(part, K, N, out_a, out_b, out_c, S, accumulate, accumulate_c, blockIdx.x, red);
}

__global__ __launch_bounds__(256) void k_reduce_partials_multi(cg::PartJobs jobs) {
    __shared__ float red[64][17];
    const int b = blockIdx.x;
    int q = 0;
    while (q + 1 < jobs.n && b >= jobs.start[q + 1]) ++q;
    const cg::PartJob& j = jobs.j[q];
    reduce_partials_block(j.part, j.K, j.N, j.a, j.b, j.c, j.S, j.acc, j.acc_c, b - jobs.start[q], red);
}

namespace cg {
// Deferred column-sum reduces (the CG_DEFER calls: cg_layernorm_bwd_reduce_ex, cg_reduce_rows_ex,
// cg_head_bwd_ex; the caller keeps every queued job's partials allocated and reads no output before
// cg_flush_deferred on that stream).  The training backward queues its ~20 LayerNorm / bias-gradient
// reduces and the flush launches them as ONE kernel: on one hardware queue each was a ~5 us launch
// for ~1 us of work.  The queue is the stream's DeferQueue (defer.h).
void flush_parts_locked(DeferQueue& q) {
    if (!q.parts.n) return;
    const PartJobs jobs = q.parts;
    q.parts.n = 0;
    k_reduce_partials_multi<<<jobs.start[jobs.n], 256, 0, q.stream>>>(jobs);
}

// [p, p + n) of job j's outputs
static bool overlaps(const float* p, int64_t n, const float* q, int64_t m) {
    return p && q && n > 0 && m > 0 && p < q + m && q < p + n;
}
static bool job_outputs_overlap(const PartJob& x, const float* p, int64_t n) {
    return overlaps(x.a, x.S, p, n) || overlaps(x.b, x.S, p, n) || overlaps(x.c, x.N - 2 * x.S, p, n);
}
// an immediate reduce / write into [p, p + n) on stream st: that stream's queued jobs that target it
// go first (caller holds the registry lock)
void flush_parts_touching_locked(DeferQueue* q, const float* p, int64_t n) {
    if (!q) return;
    for (int i = 0; i < q->parts.n; ++i)
        if (job_outputs_overlap(q->parts.j[i], p, n)) {
            flush_parts_locked(*q);
            return;
        }
}

static void enqueue_partials(const PartJob& j, hipStream_t st) {
    std::lock_guard<std::mutex> lk(defer_mutex());
    DeferQueue& q = *defer_queue(st, true);
    PartJobs& P = q.parts;
    bool clash = P.n == MAX_PART_JOBS;
    for (int i = 0; i < P.n && !clash; ++i) {
        const PartJob& x = P.j[i];
        clash = job_outputs_overlap(x, j.a, j.S) || job_outputs_overlap(x, j.b, j.S) ||
                job_outputs_overlap(x, j.c, j.N - 2 * j.S);
    }
    if (clash) flush_parts_locked(q);
    if (!P.n) P.start[0] = 0;
    P.j[P.n] = j;
    P.start[P.n + 1] = P.start[P.n] + (int)ceil_div(j.N, 16);
    ++P.n;
}

void launch_reduce_partials(const float* part, int64_t K, int64_t N, float* out_a, float* out_b, int64_t S,
                            int accumulate, hipStream_t st) {
    {
        std::lock_guard<std::mutex> lk(defer_mutex());
        DeferQueue* q = defer_queue(st, false);
        flush_parts_touching_locked(q, out_a, S);
        flush_parts_touching_locked(q, out_b, N - S);
    }
    k_reduce_partials<<<ceil_div(N, 16), 256, 0, st>>>(part, K, N, out_a, out_b, nullptr, S, accumulate, 0);
}
void launch_reduce_partials3(const float* part, int64_t K, int64_t N, float* out_a, float* out_b, float* out_c,
                             int64_t S, int accumulate, int accumulate_c, hipStream_t st) {
    {
        std::lock_guard<std::mutex> lk(defer_mutex());
        DeferQueue* q = defer_queue(st, false);
        flush_parts_touching_locked(q, out_a, S);
        flush_parts_touching_locked(q, out_b, S);
        flush_parts_touching_locked(q, out_c, N - 2 * S);
    }
    k_reduce_partials<<<ceil_div(N, 16), 256, 0, st>>>(part, K, N, out_a, out_b, out_c, S, accumulate, accumulate_c);
}
// the deferrable forms (cg_layernorm_bwd_reduce_ex, cg_reduce_rows_ex, cg_head_bwd_ex): queued on the
// stream's DeferQueue with CG_DEFER, else launched now
void reduce_partials_deferrable(const float* part, int64_t K, int64_t N, float* out_a, float* out_b, float* out_c,
                                int64_t S, int accumulate, int accumulate_c, int defer, hipStream_t st) {
    if (defer) {
        enqueue_partials(PartJob{part, K, N, S, out_a, out_b, out_c, accumulate, accumulate_c}, st);
        return;
    }
    launch_reduce_partials3(part, K, N, out_a, out_b, out_c, S, accumulate, accumulate_c, st);
}
}  // namespace cg

// deterministic two-pass sum: pass 1 -> one partial per block (fixed order), pass 2 one block
__global__ void k_sum_partial(const float* x, int64_t n, float* part) {
    __shared__ float red[16];
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        s += x[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        part[blockIdx.x] = t;
    }
}
__global__ void k_sum_final(const float* part, int np, float scale, float* out) {
    __shared__ float red[16];
    float s = 0.f;
    for (int i = threadIdx.x; i < np; i += blockDim.x) s += part[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        *out = t * scale;
    }
}

extern "C" int cg_sum_f32(const float* x, int64_t n, float scale, float* out, float* ws, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    int nb = (int)(n / 4096);
    nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
    k_sum_partial<<<nb, 256, 0, st>>>(x, n, ws);
    k_sum_final<<<1, 256, 0, st>>>(ws, nb, scale, out);
    CG_LAUNCH_CHECK("cg_sum_f32");
    return CG_OK;
}

__global__ void k_cast_f32_bf16(const float* x, bf16_t* y, int64_t n) {
    int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i + 3 < n) {
        float4 v = *(const float4*)(x + i);
        uint2 o;
        o.x = pack_bf2(v.x, v.y);
        o.y = pack_bf2(v.z, v.w);
        *(uint2*)(y + i) = o;
    } else {
        for (; i < n; ++i) y[i] = f2bf(x[i]);
    }
}

extern "C" int cg_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, void* stream) {
    if (n == 0) return CG_OK;
    CG_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0, "cg_cast_f32_bf16: misaligned");
    k_cast_f32_bf16<<<ceil_div((n + 3) / 4, 256), 256, 0, (hipStream_t)stream>>>(x, (bf16_t*)y, n);
    CG_LAUNCH_CHECK("cg_cast_f32_bf16");
    return CG_OK;
}

// --------------------------------------------------------------------------------------
// get_batch windows on device (GPT1.py:79-80)
template <typename D>
__global__ void k_gather_batch(const D* data, const int64_t* ix, int64_t* x, int64_t* y, int64_t B, int64_t T) {
    int64_t b = blockIdx.y;
    int64_t base = ix[b];
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (int64_t)gridDim.x * blockDim.x) {
        x[b * T + t] = (int64_t)data[base + t];
        y[b * T + t] = (int64_t)data[base + t + 1];
    }
}

extern "C" int cg_gather_batch(const void* data, int data_is_u8, const int64_t* ix, int64_t* x, int64_t* y,
                               int64_t B, int64_t T, void* stream) {
    CG_REQUIRE(B > 0 && T > 0 && B < 65536, "cg_gather_batch: bad shape");
    dim3 grid(ceil_div(T, 256), (unsigned)B);
    if (data_is_u8)
        k_gather_batch<uint8_t><<<grid, 256, 0, (hipStream_t)stream>>>((const uint8_t*)data, ix, x, y, B, T);
    else
        k_gather_batch<int64_t><<<grid, 256, 0, (hipStream_t)stream>>>((const int64_t*)data, ix, x, y, B, T);
    CG_LAUNCH_CHECK("cg_gather_batch");
    return CG_OK;
}
