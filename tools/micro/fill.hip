// Microbenchmark: 107 MB heartbeat-style fill (1072-byte records from a 67 x 16 B
// LDS template), by store flavour and grid size.  In-kernel span via s_memrealtime.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ void k_fill(u32x4* dst, uint64_t n_hb, unsigned long long* clk) {
    __shared__ uint4 tmpl[67];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 67) tmpl[threadIdx.x] = make_uint4(threadIdx.x, 1, 2, 3);
    __syncthreads();
    const uint64_t nchunks = n_hb * 67, lo = nchunks * blockIdx.x / gridDim.x, hi = nchunks * (blockIdx.x + 1) / gridDim.x;
    uint64_t i = lo + threadIdx.x;
    uint32_t m = (uint32_t)(i % 67);
    const uint32_t dm = blockDim.x % 67;
    for (; i < hi; i += blockDim.x) {
        const uint4 v = tmpl[m];
        u32x4 w = {v.x, v.y, v.z, v.w};
        if (MODE == 0) __builtin_nontemporal_store(w, &dst[i]);
        else if (MODE == 1) dst[i] = w;
        else __hip_atomic_store(reinterpret_cast<uint64_t*>(&dst[i]), (uint64_t)v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m += dm;
        if (m >= 67) m -= 67;
    }
    __syncthreads();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime(); }
}
int main() {
    const uint64_t n_hb = 100000;
    u32x4* dst; (void)hipMalloc(&dst, n_hb * 1072);
    unsigned long long* clk; (void)hipMalloc(&clk, 16 * 4096);
    std::vector<unsigned long long> hc(2 * 4096);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const char* names[3] = {"nt", "plain", "sc1(8B)"};
    for (int mode = 0; mode < 2; mode++)
        for (int threads : {256, 512, 1024})
            for (int grid : {256, 512, 1024, 2048}) {
                auto launch = [&] {
                    if (mode == 0) hipLaunchKernelGGL(k_fill<0>, dim3(grid), dim3(threads), 0, 0, dst, n_hb, clk);
                    else hipLaunchKernelGGL(k_fill<1>, dim3(grid), dim3(threads), 0, 0, dst, n_hb, clk);
                };
                for (int w = 0; w < 5; w++) launch();
                (void)hipDeviceSynchronize();
                float best = 1e9; double span_best = 1e9;
                for (int r = 0; r < 20; r++) {
                    (void)hipEventRecord(e0); launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
                    float ms; (void)hipEventElapsedTime(&ms, e0, e1); best = std::min(best, ms);
                    (void)hipMemcpy(hc.data(), clk, 16 * grid, hipMemcpyDeviceToHost);
                    unsigned long long mn = ~0ull, mx = 0;
                    for (int b = 0; b < grid; b++) { mn = std::min(mn, hc[2 * b]); mx = std::max(mx, hc[2 * b + 1]); }
                    span_best = std::min(span_best, (mx - mn) * 0.01);
                }
                printf("%-6s threads %4d grid %5d: event %.2f us  span %.2f us  -> %.2f TB/s (span)\n", names[mode], threads, grid,
                       best * 1e3, span_best, n_hb * 1072 / (span_best * 1e-6) / 1e12);
            }
    return 0;
}
