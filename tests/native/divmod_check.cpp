// kg_divmod64_fp (kg_common.h: the device's int64 quotient / remainder for the finalize ratios) must
// equal C int64 division on random and boundary operands over its range |n| < 2^57, 0 < d < 2^41.
// Built and run by tests/test_qdiv_cpu.py.
#include "kg_common.h"
#include <cstdio>
#include <cstdlib>
#include <random>
int main(int argc, char **argv) {
    std::mt19937_64 g(7);
    const long iters = argc > 1 ? atol(argv[1]) : 2000000;
    long bad = 0;
    for (long it = 0; it < iters; it++) {
        int64_t d = (int64_t)(g() % (1ULL << (1 + g() % 41))) + 1;
        if (d >= (1LL << 41)) d = (1LL << 41) - 1;
        const int mode = (int)(g() % 5);
        const int64_t lim = (1LL << 57) - 1;
        int64_t n;
        if (mode == 4) {
            n = (int64_t)(g() % (uint64_t)lim);
        } else {
            const int64_t k = (int64_t)(g() % (uint64_t)(lim / d));
            n = k * d + (mode == 1 ? -1 : mode == 2 ? 1 : 0);
        }
        if (g() & 1) n = -n;
        if (n >= lim || n <= -lim) continue;
        int64_t q, r;
        kg_divmod64_fp(n, d, q, r);
        if (q != n / d || r != n % d) {
            if (bad < 5) printf("bad n=%lld d=%lld got %lld %lld want %lld %lld\n", (long long)n, (long long)d,
                                (long long)q, (long long)r, (long long)(n / d), (long long)(n % d));
            bad++;
        }
    }
    printf("checked %ld bad %ld\n", iters, bad);
    return bad != 0;
}
