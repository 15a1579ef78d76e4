// CPU check of the HBM layout helpers in sng_layout.h (tests/test_layout_cpu.py): soc_index (charger pairs)
// and rec_index (charger quads) map every (charger, env) of a plane to a distinct element of [0, N * E),
// and code_soc maps the 8,192 arrival-SoC codes to strictly increasing float32 values inside (0.1, 0.9).
#include <cstdio>
#include <vector>

#include "sng_layout.h"

using namespace sng;

int main() {
    const int ns[] = {1, 2, 3, 4, 5, 7, 10, 16, 33, 50, 128};
    const int64_t es[] = {1, 7, 64, 257};
    for (int n : ns)
        for (int64_t E : es) {
            std::vector<int> seen_s((size_t)n * E, 0), seen_r((size_t)n * E, 0);
            for (int c = 0; c < n; ++c)
                for (int64_t e = 0; e < E; ++e) {
                    const size_t i = soc_index(c, e, n, E), j = rec_index(c, e, n, E);
                    if (i >= (size_t)n * E || j >= (size_t)n * E) {
                        printf("out of range n=%d E=%lld c=%d e=%lld\n", n, (long long)E, c, (long long)e);
                        return 1;
                    }
                    ++seen_s[i];
                    ++seen_r[j];
                    // a pair's or quad's members are adjacent elements of one env
                    if ((c & 1) && (c & ~1) + 2 <= n && soc_index(c, e, n, E) != soc_index(c - 1, e, n, E) + 1) return 2;
                    if ((c & 3) && rec_index(c, e, n, E) != rec_index(c - 1, e, n, E) + 1) return 3;
                }
            for (size_t k = 0; k < seen_s.size(); ++k)
                if (seen_s[k] != 1 || seen_r[k] != 1) {
                    printf("not a bijection n=%d E=%lld at %zu\n", n, (long long)E, k);
                    return 4;
                }
        }
    float prev = 0.1f;
    for (uint32_t k = 0; k < (1u << kSocCodeBits); ++k) {
        const float v = code_soc(k);
        if (!(v > prev && v < 0.9f)) {
            printf("code_soc(%u) = %.9g after %.9g\n", k, v, prev);
            return 5;
        }
        // an empty record carrying code k decodes to the same value
        if (rec_soc(rec_carry(true, k)) != v || rec_soc(rec_carry(false, k)) != v) return 6;
        prev = v;
    }
    // the packed record's fields round-trip
    for (uint32_t cap = 0; cap < 128; ++cap)
        for (uint32_t dep = 0; dep < 64; ++dep) {
            const uint32_t r = W_OCC | W_PEN | (cap << P_CAP_SHIFT) | (dep << P_DEP_SHIFT);
            if (r > 0xffffu || rec_cap(r) != cap || rec_dep(r) != dep) return 7;
        }
    printf("layout ok\n");
    return 0;
}
