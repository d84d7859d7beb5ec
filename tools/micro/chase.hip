// Microbenchmark: launch-relative latency of D dependent global loads per thread
// (256 blocks x 256 threads, each thread its own index chain), on arrays of a
// given size, each level a DIFFERENT array (as in the tick kernel).  Reports
// the best-of-50 event time per launch for D = 0..4 and array sizes 1 MB / 64 MB.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
__global__ void k_chase(const uint32_t* const* arr, int depth, uint32_t mask, uint32_t* out, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t idx = (blockIdx.x * 256 + threadIdx.x) * 4 & mask;
    for (int d = 0; d < depth; d++) idx = (arr[d][idx] + threadIdx.x * 4) & mask;
    out[blockIdx.x * 256 + threadIdx.x] = idx;
    __syncthreads();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime(); }
}
int main() {
    uint32_t* out; (void)hipMalloc(&out, 4 * 65536);
    unsigned long long* clk; (void)hipMalloc(&clk, 16 * 256);
    std::vector<unsigned long long> hc(512);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (size_t mb : {1, 64}) {
        size_t n = mb << 18;  // u32 elements
        std::vector<uint32_t*> a(4);
        std::vector<uint32_t> h(n);
        for (size_t i = 0; i < n; i++) h[i] = (uint32_t)((i * 2654435761u) & (n - 1)) & ~3u;
        for (auto& p : a) { (void)hipMalloc(&p, n * 4); (void)hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice); }
        uint32_t** d_a; (void)hipMalloc(&d_a, sizeof(uint32_t*) * 4);
        (void)hipMemcpy(d_a, a.data(), sizeof(uint32_t*) * 4, hipMemcpyHostToDevice);
        printf("array %zu MB:", mb);
        for (int depth = 0; depth <= 4; depth++) {
            auto launch = [&] { hipLaunchKernelGGL(k_chase, dim3(256), dim3(256), 0, 0, (const uint32_t* const*)d_a, depth, (uint32_t)(n - 1), out, clk); };
            for (int w = 0; w < 10; w++) launch();
            (void)hipDeviceSynchronize();
            float best = 1e9, sum = 0;
            for (int r = 0; r < 50; r++) {
                (void)hipEventRecord(e0); launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
                float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms; sum += ms;
            }
            (void)hipMemcpy(hc.data(), clk, 16 * 256, hipMemcpyDeviceToHost);
            unsigned long long mn = ~0ull, mx = 0; double med = 0;
            std::vector<double> d(256);
            for (int b = 0; b < 256; b++) { mn = std::min(mn, hc[2 * b]); mx = std::max(mx, hc[2 * b + 1]); d[b] = (hc[2 * b + 1] - hc[2 * b]) * 0.01; }
            std::sort(d.begin(), d.end()); med = d[128];
            printf("  D=%d ev %.2f us, block median %.2f us, span %.2f us\n", depth, best * 1e3, med, (mx - mn) * 0.01);
        }
        printf("\n");
    }
    return 0;
}
