// Microbenchmark: per-kernel cost of back-to-back launches on one stream (the
// queued-tick case): 512 blocks x 256 threads doing nothing / writing one word to
// pinned host memory, with and without an event record after each launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>
__global__ void k_nop(unsigned* p) { if (threadIdx.x == 0 && blockIdx.x == 100000) p[0] = 1; }
__global__ void k_host(unsigned* h) { if (threadIdx.x == 0 && blockIdx.x == 0) h[0] = h[0] + 1; }
__global__ void k_spin(unsigned* p, unsigned ns100) {  // each block busy for ~ns100 x 10 ns
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ns100) {}
    if (threadIdx.x == 0 && blockIdx.x == 100000) p[0] = 1;
}
int main() {
    unsigned *d, *h;
    (void)hipMalloc(&d, 64);
    (void)hipHostMalloc(&h, 64, hipHostMallocDefault);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t ev, ev_nf;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ev_nf, hipEventDisableTiming | hipEventDisableSystemFence);
    const int N = 200;
    const char* recn[4] = {"", "+event", "+ev-nofence", "+writeval"};
    unsigned seq = 0;
    for (int kind = 0; kind < 3; kind++)
        for (int rec = 0; rec < 4; rec++)
            for (int blocks : {256, 512}) {
                auto one = [&] {
                    if (kind == 0) hipLaunchKernelGGL(k_nop, dim3(blocks), dim3(256), 0, st, d);
                    else if (kind == 1) hipLaunchKernelGGL(k_host, dim3(blocks), dim3(256), 0, st, h);
                    else hipLaunchKernelGGL(k_spin, dim3(blocks), dim3(256), 0, st, d, 2000u);
                    if (rec == 1) (void)hipEventRecord(ev, st);
                    if (rec == 2) (void)hipEventRecord(ev_nf, st);
                    if (rec == 3) (void)hipStreamWriteValue32(st, h + 8, ++seq, 0);
                };
                for (int w = 0; w < 20; w++) one();
                (void)hipStreamSynchronize(st);
                double best = 1e9;
                for (int r = 0; r < 5; r++) {
                    auto t0 = std::chrono::steady_clock::now();
                    for (int i = 0; i < N; i++) one();
                    (void)hipStreamSynchronize(st);
                    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
                    best = std::min(best, us);
                }
                printf("%-10s %-8s blocks %3d: %.2f us per launch\n", kind == 0 ? "nop" : kind == 1 ? "host-store" : "spin-20us",
                       recn[rec], blocks, best);
            }
    // host-observed latency: launch one spin kernel, then wait for completion by
    // (a) spinning on an event, (b) spinning on a stream-written value
    for (int mode = 0; mode < 4; mode++) {
        double tot = 0;
        for (int r = 0; r < 50; r++) {
            auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_spin, dim3(512), dim3(256), 0, st, d, 2000u);
            if (mode == 0 || mode == 2) {
                hipEvent_t e = mode == 0 ? ev : ev_nf;
                (void)hipEventRecord(e, st);
                while (hipEventQuery(e) == hipErrorNotReady) {}
            } else if (mode == 3) {
                (void)hipStreamSynchronize(st);
            } else {
                const unsigned want = ++seq;
                (void)hipStreamWriteValue32(st, h + 8, want, 0);
                while (__atomic_load_n((volatile unsigned*)(h + 8), __ATOMIC_ACQUIRE) != want) {}
            }
            tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
        const char* wn[4] = {"event spin", "write-value spin", "no-fence event spin", "stream sync"};
        printf("launch + wait (%s): %.2f us (kernel ~20 us)\n", wn[mode], tot / 50);
    }
    return 0;
}
