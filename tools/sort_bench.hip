// Timing harness of the ingest's bucket sort (kwok_amd/csrc/ingest.hip,
// bucket_sort): n keys (argv[1], 1M) over nb buckets (argv[2], 4096; +5% "nothing
// to apply"), sorted 20 times; run under rocprofv3 --kernel-trace --stats for
// per-kernel times (tools/gpu_s40.sh).  Checks the result against a host stable sort.
#include "../kwok_amd/csrc/ingest.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u, nb = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096u,
                   nk = nb + 1;
    std::vector<uint32_t> keys(n);
    std::mt19937 rng(7);
    for (auto& k : keys) k = (rng() % 20 == 0) ? nb : rng() % nb;
    uint32_t *dk, *dks, *dix, *dbeg, *dend;
    void* tmp;
    const size_t tb = kwok::bucket_sort_bytes(n, kwok::BS_MAX_KEYS);
    if (hipMalloc(&dk, n * 4) || hipMalloc(&dks, n * 4) || hipMalloc(&dix, n * 4) || hipMalloc(&dbeg, nb * 4) ||
        hipMalloc(&dend, nb * 4) || hipMalloc(&tmp, tb))
        return 2;
    (void)hipMemcpy(dk, keys.data(), n * 4, hipMemcpyHostToDevice);
    for (int it = 0; it < 20; it++)
        if (!kwok::bucket_sort(dk, n, nk, dks, dix, dbeg, dend, tmp, tb, nullptr)) return 3;
    (void)hipDeviceSynchronize();
    std::vector<uint32_t> ix(n), beg(nb), end(nb);
    (void)hipMemcpy(ix.data(), dix, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(beg.data(), dbeg, nb * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(end.data(), dend, nb * 4, hipMemcpyDeviceToHost);
    std::vector<uint32_t> ref(n);
    for (uint32_t i = 0; i < n; i++) ref[i] = i;
    std::stable_sort(ref.begin(), ref.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; i++) bad += ix[i] != ref[i];
    printf("n=%u mismatches=%u beg[7]=%u end[7]=%u\n", n, bad, beg[7], end[7]);
    return 0;
}
