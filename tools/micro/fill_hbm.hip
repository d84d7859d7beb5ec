// Microbenchmark: the 1M-node heartbeat stream (1M x 1072-byte records, 1.07 GB,
// far past the 256 MiB Infinity Cache) by store flavour, waves per CU and grid.
// The 4-slot-group layout of k_tick's hb_fill_groups: every lane keeps its 5
// template units in registers.  usage: fill_hbm [n_hb]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int NT>
__global__ void k_fill_reg(u32x4* dst, uint64_t n_hb) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    u32x4 r[5];
#pragma unroll
    for (int k = 0; k < 5; k++) r[k] = u32x4{(uint32_t)((64 * k + l) % 67), 1u, 2u, 3u};
    const uint64_t ng = n_hb / 4, g0 = ng * blockIdx.x / gridDim.x, g1 = ng * (blockIdx.x + 1) / gridDim.x;
    for (uint64_t g = g0 + w; g < g1; g += nw) {
        u32x4* p = dst + g * 268 + l;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (NT) __builtin_nontemporal_store(r[k], p + 64 * k);
            else p[64 * k] = r[k];
        }
        if (l < 12) {
            if (NT) __builtin_nontemporal_store(r[4], p + 256);
            else p[256] = r[4];
        }
    }
}
// contiguous per-wave pieces: wave q of the grid writes groups [q*G/W, (q+1)*G/W)
template <int NT>
__global__ void k_fill_wave(u32x4* dst, uint64_t n_hb) {
    const int l = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6), q = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    u32x4 r[5];
#pragma unroll
    for (int k = 0; k < 5; k++) r[k] = u32x4{(uint32_t)((64 * k + l) % 67), 1u, 2u, 3u};
    const uint64_t ng = n_hb / 4, g0 = ng * q / W, g1 = ng * (q + 1) / W;
    for (uint64_t g = g0; g < g1; g++) {
        u32x4* p = dst + g * 268 + l;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (NT) __builtin_nontemporal_store(r[k], p + 64 * k);
            else p[64 * k] = r[k];
        }
        if (l < 12) {
            if (NT) __builtin_nontemporal_store(r[4], p + 256);
            else p[256] = r[4];
        }
    }
}
int main(int argc, char** argv) {
    const uint64_t n_hb = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000;
    u32x4* dst;
    if (hipMalloc(&dst, n_hb * 1072 + 4096) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("n_hb %llu (%.1f MB), %d CUs\n", (unsigned long long)n_hb, n_hb * 1072 / 1e6, cus);
    for (int kind = 0; kind < 4; kind++)
        for (int threads : {256, 512, 1024})
            for (int bpc : {1, 2, 4}) {
                const int grid = cus * bpc;
                if (threads * bpc > 2048) continue;
                auto launch = [&] {
                    switch (kind) {
                        case 0: hipLaunchKernelGGL(k_fill_reg<0>, dim3(grid), dim3(threads), 0, 0, dst, n_hb); break;
                        case 1: hipLaunchKernelGGL(k_fill_reg<1>, dim3(grid), dim3(threads), 0, 0, dst, n_hb); break;
                        case 2: hipLaunchKernelGGL(k_fill_wave<0>, dim3(grid), dim3(threads), 0, 0, dst, n_hb); break;
                        default: hipLaunchKernelGGL(k_fill_wave<1>, dim3(grid), dim3(threads), 0, 0, dst, n_hb); break;
                    }
                };
                for (int w = 0; w < 3; w++) launch();
                (void)hipDeviceSynchronize();
                float best = 1e9, sum = 0;
                for (int r = 0; r < 10; r++) {
                    (void)hipEventRecord(e0);
                    launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    best = std::min(best, ms);
                    sum += ms;
                }
                static const char* nm[4] = {"grp-plain", "grp-nt", "wave-plain", "wave-nt"};
                printf("%-10s threads %4d blocks/CU %d: best %7.1f us mean %7.1f us -> %.2f TB/s (best)\n", nm[kind],
                       threads, bpc, best * 1e3, sum * 1e2, n_hb * 1072 / (best * 1e-3) / 1e12);
            }
    return 0;
}
