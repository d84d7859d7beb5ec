// Microbenchmark: how much a small read stream mixed into a write stream costs.
// The initial tick's emission writes 7.2 GB of patch bytes while its classification
// reads a few percent of that (pod state, node flags, tables).  Each wave writes a
// contiguous piece of a 7.2 GB buffer (1 KiB per store instruction, plain stores)
// and, every `every` stores, reads one 16-byte word per lane from its own piece of a
// second buffer (the read share = 1 / every).  The reads cycle over `rmb` MB (small:
// Infinity-Cache resident), the stores plain or non-temporal.  Mode "tab" instead loads,
// per store, one uint4 + one u32 per lane from a 256 KB table at a per-lane index (cache
// hits, as the emission's unit-table loads).  usage: fill_mix [mb_written] [tab]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// per store: a 16-byte table row + a 4-byte descriptor per lane, L2 / L1 hits (2 x 4096 x 20 B)
template <int NT>
__global__ void k_tab(u32x4* dst, uint64_t n16, const u32x4* tab, const uint32_t* desc, u32x4* sink) {
    const int l = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6), q = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nrow = n16 / 64, r0 = nrow * q / W, r1 = nrow * (q + 1) / W;
    u32x4 acc = u32x4{0u, 0u, 0u, 0u};
    uint32_t u = (uint32_t)(q * 45u + l) & 4095u;
    for (uint64_t r = r0; r < r1; r++) {
        const u32x4 t = tab[u];
        const uint32_t d = desc[u];
        const u32x4 v = u32x4{t.x | d, t.y, t.z, t.w ^ (uint32_t)r};
        if (NT) __builtin_nontemporal_store(v, dst + r * 64 + l);
        else dst[r * 64 + l] = v;
        u = (u + 64u) & 4095u;
        acc += t;
    }
    if (acc.x == 0xFFFFFFFFu) sink[l] = acc;
}
template <int NT>
__global__ void k_mix(u32x4* dst, uint64_t n16, const u32x4* src, uint64_t s16, int every, u32x4* sink) {
    const int l = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6), q = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nrow = n16 / 64, r0 = nrow * q / W, r1 = nrow * (q + 1) / W;
    const uint64_t srow = s16 / 64, sr0 = srow * q / W, sr1 = srow * (q + 1) / W;
    u32x4 acc = u32x4{0u, 0u, 0u, 0u}, v = u32x4{(uint32_t)l, 1u, 2u, 3u};
    uint64_t sr = sr0;
    int k = 0;
    for (uint64_t r = r0; r < r1; r++) {
        if (NT) __builtin_nontemporal_store(v, dst + r * 64 + l);
        else dst[r * 64 + l] = v;
        if (every && ++k == every) {
            k = 0;
            const u32x4 x = src[sr * 64 + l];
            acc += x;
            v.y ^= x.x;  // the stores depend on the reads (as the emission's do)
            if (++sr >= sr1) sr = sr0;
        }
    }
    if (acc.x == 0xFFFFFFFFu) sink[l] = acc;
}
int main(int argc, char** argv) {
    const uint64_t mb = argc > 1 ? strtoull(argv[1], 0, 10) : 7240;
    const uint64_t n16 = mb * 1000000ull / 16;
    u32x4 *dst, *src, *sink;
    const uint64_t s16 = n16 / 8;  // up to 1/8 of the written bytes read
    if (hipMalloc(&dst, n16 * 16) != hipSuccess || hipMalloc(&src, s16 * 16) != hipSuccess ||
        hipMalloc(&sink, 64 * 16) != hipSuccess)
        return 1;
    (void)hipMemset(src, 1, s16 * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("%llu MB written, %d CUs\n", (unsigned long long)mb, cus);
    if (argc > 2) {  // "tab": table loads per store
        u32x4* tab;
        uint32_t* desc;
        if (hipMalloc(&tab, 4096 * 16) != hipSuccess || hipMalloc(&desc, 4096 * 4) != hipSuccess) return 1;
        (void)hipMemset(tab, 0, 4096 * 16);
        (void)hipMemset(desc, 0, 4096 * 4);
        for (int nt = 0; nt < 2; nt++)
            for (int wpc : {4, 12}) {
                const int grid = cus * wpc / 4;
                auto launch = [&] {
                    if (nt) hipLaunchKernelGGL(k_tab<1>, dim3(grid), dim3(256), 0, 0, dst, n16, tab, desc, sink);
                    else hipLaunchKernelGGL(k_tab<0>, dim3(grid), dim3(256), 0, 0, dst, n16, tab, desc, sink);
                };
                for (int w = 0; w < 2; w++) launch();
                (void)hipDeviceSynchronize();
                float best = 1e9, sum = 0;
                for (int r = 0; r < 8; r++) {
                    (void)hipEventRecord(e0);
                    launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    best = std::min(best, ms);
                    sum += ms;
                }
                printf("%s stores + table loads per store, waves/CU %2d: best %7.1f us mean %7.1f us -> write %.2f TB/s (best)\n",
                       nt ? "nt   " : "plain", wpc, best * 1e3, sum / 8 * 1e3, n16 * 16 / (best * 1e-3) / 1e12);
            }
        return 0;
    }
    for (int nt = 0; nt < 2; nt++)
        for (uint64_t rmb : {(uint64_t)0, (uint64_t)64, (uint64_t)800})
            for (int every : {0, 32}) {
                if ((every == 0) != (rmb == 0)) continue;
                const uint64_t r16 = rmb ? rmb * 1000000ull / 16 : s16;
                const int threads = 256, grid = cus * 3;
                auto launch = [&] {
                    if (nt) hipLaunchKernelGGL(k_mix<1>, dim3(grid), dim3(threads), 0, 0, dst, n16, src, r16, every, sink);
                    else hipLaunchKernelGGL(k_mix<0>, dim3(grid), dim3(threads), 0, 0, dst, n16, src, r16, every, sink);
                };
                for (int w = 0; w < 2; w++) launch();
                (void)hipDeviceSynchronize();
                float best = 1e9, sum = 0;
                for (int r = 0; r < 8; r++) {
                    (void)hipEventRecord(e0);
                    launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    best = std::min(best, ms);
                    sum += ms;
                }
                printf("%s stores, read 1/%-2d over %4llu MB: best %7.1f us mean %7.1f us -> write %.2f TB/s (best)\n",
                       nt ? "nt   " : "plain", every, (unsigned long long)rmb, best * 1e3, sum / 8 * 1e3,
                       n16 * 16 / (best * 1e-3) / 1e12);
            }
    return 0;
}
