// Microbenchmark: cost of the chain blocks' end-of-classification reduction.
// G blocks each add F per-block values into F device accumulators (one 128-byte
// line each) with returning atomics (the k_tick arrival scheme), vs variants.
// Reports, per variant, the span from the earliest block start to the latest
// block's completion of its adds (s_memrealtime, 100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
template <int MODE>
__global__ void k_acc(unsigned long long* acc, int F, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int t = threadIdx.x;
    unsigned long long r = 0;
    if (MODE == 0) {  // F returning adds, one lane each
        if (t < F) r = __hip_atomic_fetch_add(&acc[t * 16], (1ull << 54) | 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (MODE == 1) {  // F non-returning adds, then one returning arrival
        if (t < F) __hip_atomic_fetch_add(&acc[t * 16], 7ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (t == 0) r = __hip_atomic_fetch_add(&acc[16 * 16], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (MODE == 2) {  // F returning adds spread over 8 copies (block % 8): 8x less contention
        if (t < F) r = __hip_atomic_fetch_add(&acc[(t * 8 + (blockIdx.x & 7)) * 16], (1ull << 54) | 7, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    } else if (MODE == 3) {  // a single returning add (arrival only)
        if (t == 0) r = __hip_atomic_fetch_add(&acc[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {  // plain dependent-free load of one line per lane (round-trip reference)
        if (t < F) r = __hip_atomic_load(&acc[t * 16 + 4096], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (t == 0 || r == 12345) {
        clk[2 * blockIdx.x] = t0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}
int main() {
    unsigned long long *acc, *clk;
    (void)hipMalloc(&acc, 8 * 16 * 8192);
    (void)hipMemset(acc, 0, 8 * 16 * 8192);
    (void)hipMalloc(&clk, 16 * 4096);
    std::vector<unsigned long long> hc(2 * 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[5] = {"F returning", "F plain + arrival", "F returning /8 copies", "1 returning", "F loads"};
    for (int mode = 0; mode < 5; mode++)
        for (int G : {256, 512})
            for (int F : {1, 8, 15}) {
                if (mode == 3 && F != 1) continue;
                auto launch = [&] {
                    switch (mode) {
                        case 0: hipLaunchKernelGGL(k_acc<0>, dim3(G), dim3(256), 0, 0, acc, F, clk); break;
                        case 1: hipLaunchKernelGGL(k_acc<1>, dim3(G), dim3(256), 0, 0, acc, F, clk); break;
                        case 2: hipLaunchKernelGGL(k_acc<2>, dim3(G), dim3(256), 0, 0, acc, F, clk); break;
                        case 3: hipLaunchKernelGGL(k_acc<3>, dim3(G), dim3(256), 0, 0, acc, F, clk); break;
                        default: hipLaunchKernelGGL(k_acc<4>, dim3(G), dim3(256), 0, 0, acc, F, clk); break;
                    }
                };
                for (int w = 0; w < 5; w++) launch();
                (void)hipDeviceSynchronize();
                std::vector<double> spans, evs, meds;
                for (int r = 0; r < 30; r++) {
                    (void)hipEventRecord(e0);
                    launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    (void)hipMemcpy(hc.data(), clk, 16 * G, hipMemcpyDeviceToHost);
                    unsigned long long mn = ~0ull, mx = 0;
                    std::vector<double> d;
                    for (int b = 0; b < G; b++) {
                        mn = std::min(mn, hc[2 * b]);
                        mx = std::max(mx, hc[2 * b + 1]);
                        d.push_back((hc[2 * b + 1] - hc[2 * b]) * 0.01);
                    }
                    std::sort(d.begin(), d.end());
                    spans.push_back((mx - mn) * 0.01);
                    evs.push_back(ms * 1e3);
                    meds.push_back(d[d.size() / 2]);
                }
                std::sort(spans.begin(), spans.end());
                std::sort(evs.begin(), evs.end());
                std::sort(meds.begin(), meds.end());
                printf("%-22s G %4d F %2d: span %6.2f us  per-block median %5.2f us  event %6.2f us\n", names[mode], G, F,
                       spans[15], meds[15], evs[15]);
            }
    return 0;
}
