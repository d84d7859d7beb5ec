// Microbenchmark: per-tick fixed cost of (a) launch + stream sync of a trivial
// 512-block kernel, vs (b) a resident kernel that ping-pongs with the host
// through pinned memory (block 0 polls the host mailbox and relays through
// device memory; the last block to finish a round writes the host's done word).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>
__global__ void k_empty(int* p) { if (threadIdx.x == 0 && blockIdx.x == 100000) p[0] = 1; }
__global__ void k_server(volatile unsigned* mbox, volatile unsigned* done, unsigned* relay, unsigned* cnt, int rounds) {
    __shared__ unsigned seq;
    for (unsigned r = 1; r <= (unsigned)rounds; r++) {
        if (threadIdx.x == 0) {
            if (blockIdx.x == 0) {
                unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load((unsigned*)mbox, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < r)
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
                __hip_atomic_store(relay, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < r) {
                    __builtin_amdgcn_s_sleep(1);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
                }
            }
            seq = r;
        }
        __syncthreads();
        // (the tick would run here)
        if (threadIdx.x == 0) {
            unsigned old = atomicAdd(cnt, 1u);
            if (old + 1 == r * gridDim.x) __hip_atomic_store((unsigned*)done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
    }
}
int main() {
    int* p; (void)hipMalloc(&p, 4);
    hipStream_t st; (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int i = 0; i < 100; i++) { hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, st, p); (void)hipStreamSynchronize(st); }
    auto t0 = std::chrono::steady_clock::now();
    const int N = 2000;
    for (int i = 0; i < N; i++) { hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, st, p); (void)hipStreamSynchronize(st); }
    auto t1 = std::chrono::steady_clock::now();
    printf("launch+sync of an empty 512-block kernel: %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    unsigned *mbox, *done, *relay, *cnt;
    (void)hipHostMalloc((void**)&mbox, 64, hipHostMallocDefault);
    (void)hipHostMalloc((void**)&done, 64, hipHostMallocDefault);
    (void)hipMalloc(&relay, 64); (void)hipMalloc(&cnt, 64);
    (void)hipMemset(relay, 0, 64); (void)hipMemset(cnt, 0, 64);
    *mbox = 0; *done = 0;
    const int R = 2000;
    hipLaunchKernelGGL(k_server, dim3(512), dim3(256), 0, st, mbox, done, relay, cnt, R);
    // warm
    for (unsigned r = 1; r <= 100; r++) { __atomic_store_n(mbox, r, __ATOMIC_RELEASE); while (__atomic_load_n(done, __ATOMIC_ACQUIRE) < r) {} }
    t0 = std::chrono::steady_clock::now();
    for (unsigned r = 101; r <= (unsigned)R; r++) { __atomic_store_n(mbox, r, __ATOMIC_RELEASE); while (__atomic_load_n(done, __ATOMIC_ACQUIRE) < r) {} }
    t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    printf("resident kernel ping-pong round: %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / (R - 100));
    return 0;
}
