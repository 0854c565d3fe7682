// Diagnostic build (not part of the library): the LDS-DMA GEMM body with s_memrealtime stamps per
// block at start / after the first tile landed / after the K loop / at the end, to see where a
// short-K launch spends its time.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_diag.hip -o /tmp/gemm_diag
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../replicatinggpt_amd/csrc/gemm_tile.h"

using namespace cg;
using namespace cg::gt;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int BM = 128, BN = 128, WAVES = 4, IMG = BM * 128, STAGE = 2 * IMG;

__global__ __launch_bounds__(256, 2) void k_diag(int64_t M, int64_t N, int64_t K, const bf16_t* A, const bf16_t* B,
                                                 bf16_t* C, uint64_t* st, int mode) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t t0 = stamp();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / 2, wn = wave % 2;
    const int tilesN = (int)(N / BN);
    const int ntiles = (int)(M / BM) * tilesN;
    const int t = xcd_remap(blockIdx.x, ntiles);
    const int64_t m0 = (int64_t)(t / tilesN) * BM, n0 = (int64_t)(t % tilesN) * BN;
    const int nk = (int)(K / 64);
    const bf16_t* sa[4];
    const bf16_t* sb[4];
    for (int i = 0; i < 4; ++i) {
        const int pos = (wave * 4 + i) * 1024 + lane * 16;
        const int r = pos >> 7, c = ((pos >> 4) & 7) ^ row_swz(r);
        sa[i] = A + (m0 + r) * K + c * 8;
        sb[i] = B + (n0 + r) * K + c * 8;
    }
    auto issue = [&](int kt, int buf) {
        char* img = smem + buf * STAGE;
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(sa[i] + kt * 64), (lds_void*)(img + (wave * 4 + i) * 1024),
                                             16, 0, 0);
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(sb[i] + kt * 64),
                                             (lds_void*)(img + IMG + (wave * 4 + i) * 1024), 16, 0, 0);
    };
    fv4 acc[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    issue(0, 0);
    uint64_t t1 = 0;
    for (int kt = 0; kt < nk; ++kt) {
        wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt == 0) t1 = stamp();
        if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
        const char* img = smem + (kt & 1) * STAGE;
        for (int s = 0; s < 2; ++s) {
            sv8 af[4], bf[4];
            for (int i = 0; i < 4; ++i) af[i] = frag<false, BM>(img, wm * 64 + i * 16, s, lane);
            for (int j = 0; j < 4; ++j) bf[j] = frag<false, BN>(img + IMG, wn * 64 + j * 16, s, lane);
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma_bf16(af[i], bf[j], acc[i][j]);
        }
    }
    __syncthreads();
    uint64_t t2 = stamp();
    if (mode == 0) {
        EpiArgs e{};
        e.kind = CG_EPI_STORE;
        epilogue<BM, BN>(acc, smem, tid, M, N, m0, n0, C, CG_BF16, N, e, 1, 0, nullptr);
    } else {
        // direct register stores (no LDS staging): 2-byte scattered
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int r = 0; r < 4; ++r) {
                    const int64_t m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r, n = n0 + wn * 64 + j * 16 + (lane & 15);
                    C[m * N + n] = f2bf(acc[i][j][r]);
                }
    }
    __syncthreads();
    uint64_t t3 = stamp();
    if (tid == 0) {
        st[blockIdx.x * 4 + 0] = t0;
        st[blockIdx.x * 4 + 1] = t1;
        st[blockIdx.x * 4 + 2] = t2;
        st[blockIdx.x * 4 + 3] = t3;
    }
}

__global__ void k_empty(uint64_t* st) {
    if (threadIdx.x == 0) st[blockIdx.x] = stamp();
}

int main() {
    const int64_t N = 384;
    for (int64_t M : {2048, 16384}) {
        for (int64_t K : {64, 384, 1536}) {
            for (int mode = 0; mode < 2; ++mode) {
                bf16_t *A, *B, *C;
                uint64_t* st;
                hipMalloc(&A, M * K * 2);
                hipMalloc(&B, N * K * 2);
                hipMalloc(&C, M * N * 2);
                hipMemset(A, 0x3c, M * K * 2);
                hipMemset(B, 0x3c, N * K * 2);
                const int nb = (int)((M / BM) * (N / BN));
                hipMalloc(&st, nb * 4 * 8);
                const int lds = std::max(2 * STAGE, epi_lds_bytes<BN>());
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                for (int w = 0; w < 3; ++w) k_diag<<<nb, 256, lds>>>(M, N, K, A, B, C, st, mode);
                hipEventRecord(e0);
                const int R = 20;
                for (int w = 0; w < R; ++w) k_diag<<<nb, 256, lds>>>(M, N, K, A, B, C, st, mode);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                std::vector<uint64_t> h(nb * 4);
                hipMemcpy(h.data(), st, nb * 32, hipMemcpyDeviceToHost);
                uint64_t tmin = ~0ull, tmax = 0;
                double d01 = 0, d12 = 0, d23 = 0, mx01 = 0, mx12 = 0, mx23 = 0;
                for (int b = 0; b < nb; ++b) {
                    tmin = std::min(tmin, h[b * 4]);
                    tmax = std::max(tmax, h[b * 4 + 3]);
                    const double a = (h[b * 4 + 1] - h[b * 4]) * 0.01, c = (h[b * 4 + 2] - h[b * 4 + 1]) * 0.01,
                                 d = (h[b * 4 + 3] - h[b * 4 + 2]) * 0.01;
                    d01 += a; d12 += c; d23 += d;
                    mx01 = std::max(mx01, a); mx12 = std::max(mx12, c); mx23 = std::max(mx23, d);
                }
                uint64_t smax = 0;
                for (int b = 0; b < nb; ++b) smax = std::max(smax, h[b * 4]);
                printf("M=%6ld K=%5ld epi=%s blocks=%4d  event %6.1f us/launch | span(first start->last end) %6.1f us, "
                       "last start +%5.1f us | per block avg(max) us: first tile %5.2f(%5.2f) loop %5.2f(%5.2f) epi %5.2f(%5.2f)\n",
                       (long)M, (long)K, mode ? "direct" : "lds", nb, ms * 1000 / R, (tmax - tmin) * 0.01,
                       (smax - tmin) * 0.01, d01 / nb, mx01, d12 / nb, mx12, d23 / nb, mx23);
                hipFree(A); hipFree(B); hipFree(C); hipFree(st);
            }
        }
    }
    // launch overhead of an empty kernel
    uint64_t* st;
    hipMalloc(&st, 4096 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_empty<<<384, 256>>>(st);
    hipEventRecord(e0);
    for (int w = 0; w < 100; ++w) k_empty<<<384, 256>>>(st);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel (384 blocks): %.2f us/launch\n", ms * 10);
    return 0;
}
