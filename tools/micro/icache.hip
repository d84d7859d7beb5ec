// Microbenchmark: is straight-line code fetched cold at every kernel launch?
// A: N unrolled dependent-free VALU ops (large code); B: the same op count in a loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int N>
__global__ void k_unrolled(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = a * 3u, c = a + 7u, d = a ^ 0x55u;
#pragma unroll
    for (int i = 0; i < N; i++) {
        a = a * 1664525u + (uint32_t)i; b ^= a >> 3; c += b * (uint32_t)(i | 1); d = (d << 1) ^ c;
    }
    if ((a ^ b ^ c ^ d) == 0x12345u) out[0] = a;
}
__global__ void k_loop(uint32_t* out, uint32_t seed, int n) {
    uint32_t a = threadIdx.x ^ seed, b = a * 3u, c = a + 7u, d = a ^ 0x55u;
#pragma unroll 1
    for (int i = 0; i < n; i++) {
        a = a * 1664525u + (uint32_t)i; b ^= a >> 3; c += b * (uint32_t)(i | 1); d = (d << 1) ^ c;
    }
    if ((a ^ b ^ c ^ d) == 0x12345u) out[0] = a;
}
int main() {
    uint32_t* out; hipMalloc(&out, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto time = [&](auto launch) {
        for (int w = 0; w < 10; w++) launch();
        hipDeviceSynchronize();
        float best = 1e9;
        for (int r = 0; r < 50; r++) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        return best * 1000.f;
    };
    float a1 = time([&] { hipLaunchKernelGGL(k_unrolled<256>, dim3(512), dim3(256), 0, 0, out, 1u); });
    float a2 = time([&] { hipLaunchKernelGGL(k_unrolled<2048>, dim3(512), dim3(256), 0, 0, out, 1u); });
    float b1 = time([&] { hipLaunchKernelGGL(k_loop, dim3(512), dim3(256), 0, 0, out, 1u, 256); });
    float b2 = time([&] { hipLaunchKernelGGL(k_loop, dim3(512), dim3(256), 0, 0, out, 1u, 2048); });
    printf("unrolled 256: %.2f us   unrolled 2048: %.2f us   loop 256: %.2f us   loop 2048: %.2f us\n", a1, a2, b1, b2);
    return 0;
}
