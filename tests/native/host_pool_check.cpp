// Host-only stress check of sng_api.cpp's HostPool / parallel_ranges (the pool that draws the
// Python-stream PV ratios and seeds the streams): many parallel sections, every item visited exactly
// once per section, no deadlock.  tests/test_host_pool.py extracts the pool's source text into
// host_pool.inc and builds this file with g++ (with -fsanitize=thread when available).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
static int g_threads = 8;
int host_threads() { return g_threads; }
#include "host_pool.inc"
int main() {
    std::vector<long> v(100003, 0);
    int reps = 0;
    for (int t : {1, 2, 3, 8, 16}) {
        g_threads = t;
        for (int rep = 0; rep < 300; ++rep, ++reps) {
            std::atomic<long> sum{0};
            const int64_t n = (int64_t)v.size() - rep;   // ragged sizes
            parallel_ranges(n, 1024, [&](int64_t b, int64_t e) {
                for (int64_t i = b; i < e; ++i) v[i] += 1;
                sum += e - b;
            });
            if (sum != n) {
                std::printf("FAIL: %ld of %ld items\n", (long)sum.load(), (long)n);
                return 1;
            }
        }
    }
    for (size_t i = 0; i < v.size(); ++i) {
        long want = 0;
        for (int t = 0; t < 5; ++t)
            for (int rep = 0; rep < 300; ++rep) want += (int64_t)i < (int64_t)v.size() - rep ? 1 : 0;
        if (v[i] != want) {
            std::printf("FAIL: item %zu visited %ld times, want %ld\n", i, v[i], want);
            return 1;
        }
    }
    std::printf("pool ok: %d sections\n", reps);
    return 0;
}
