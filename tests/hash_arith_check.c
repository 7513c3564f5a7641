/* Host check of the integer shortcuts in the MinMax query's hashes (skml_sparse.hip: div1000,
 * bkdr3, bkdr_chunks, java_hash_fm's 32-bit branch), with the GPU's 24-bit multiply emulated as
 * the low 32 bits of the product of the operands' low 24 bits.  Exits non-zero on the first
 * mismatch.  Built and run by tests/test_hash_arith.py. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint32_t mul24(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)(a & 0xFFFFFFu) * (b & 0xFFFFFFu)); }
static uint32_t div1000(uint32_t k) { return (uint32_t)((double)k * 0.001); }
static uint32_t bkdr3(uint32_t s, uint32_t r) {
    const uint32_t t = mul24(r, 205u) >> 11, h = mul24(r, 41u) >> 12;
    return mul24(mul24(r - 10u * t, s) + (t - 10u * h), s) + h;
}
static uint32_t bkdr_fast(uint32_t s, uint32_t k) {
    const uint32_t s2 = s * s, s3 = s2 * s;
    uint32_t c = 0;
    while (k >= 1000u) {
        const uint32_t q = div1000(k);
        if (q >= (1u << 24)) return 0xDEADBEEFu;
        c = c * s3 + bkdr3(s, k - mul24(q, 1000u));
        k = q;
    }
    if (k >= 100u) {
        c = c * s3 + bkdr3(s, k);
    } else if (k >= 10u) {
        const uint32_t t = mul24(k, 205u) >> 11;
        c = c * s2 + mul24(k - 10u * t, s) + t;
    } else if (k) {
        c = c * s + k;
    }
    return c;
}
/* BKDRHash.java's loop on a non-negative key */
static uint32_t bkdr_ref(uint32_t s, int32_t key) {
    uint32_t c = 0;
    while (key != 0) {
        c = s * c + (uint32_t)(key % 10);
        key /= 10;
    }
    return c;
}
static int32_t mod_fast(int32_t r, int32_t size) {
    const double inv = 1.0 / (double)size;
    const int32_t q = (int32_t)floor((double)r * inv);
    int32_t m = (int32_t)((uint32_t)r - (uint32_t)q * (uint32_t)size);
    if (m < 0) m += size;
    else if (m >= size) m -= size;
    return m;
}
static int32_t mod_ref(int32_t r, int32_t size) {
    const int32_t m = r % size;
    return m >= 0 ? m : m + size;
}
static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 16);
}

int main(void) {
    static const uint32_t seeds[5] = {31u, 131u, 267u, 1313u, 13131u};
    for (uint64_t k = 0; k < (1ull << 32); k++)
        if (div1000((uint32_t)k) != (uint32_t)k / 1000u) {
            printf("div1000 %llu\n", (unsigned long long)k);
            return 1;
        }
    for (int si = 0; si < 5; si++) {
        const uint32_t s = seeds[si];
        for (uint32_t r = 0; r < 1000; r++) {
            const uint32_t d0 = r % 10, d1 = r / 10 % 10, d2 = r / 100;
            if (bkdr3(s, r) != (d0 * s + d1) * s + d2) {
                printf("bkdr3 seed %u r %u\n", s, r);
                return 1;
            }
        }
        for (uint32_t k = 0; k < (1u << 24); k++)
            if (bkdr_fast(s, k) != bkdr_ref(s, (int32_t)k)) {
                printf("bkdr seed %u key %u\n", s, k);
                return 1;
            }
        for (int i = 0; i < (1 << 22); i++) {
            const int32_t k = (int32_t)(next32() & 0x7FFFFFFFu);
            if (bkdr_fast(s, (uint32_t)k) != bkdr_ref(s, k)) {
                printf("bkdr seed %u key %d\n", s, k);
                return 1;
            }
        }
        if (bkdr_fast(s, 0x7FFFFFFFu) != bkdr_ref(s, 0x7FFFFFFF)) return 1;
    }
    static const int32_t sizes[] = {1, 2, 3, 7, 10, 1000, 65521, 1 << 20, (1 << 21) + 1, 99999989, (1 << 29) + 3,
                                    0x3FFFFFFF, 0x40000000};
    for (unsigned z = 0; z < sizeof sizes / sizeof sizes[0]; z++) {
        const int32_t size = sizes[z];
        static const int32_t edge[] = {0, 1, -1, 0x7FFFFFFF, (int32_t)0x80000000, 0x7FFFFFFE, (int32_t)0x80000001};
        for (unsigned e = 0; e < sizeof edge / sizeof edge[0]; e++)
            for (int64_t d = -3; d <= 3; d++) {
                const int64_t r = (int64_t)edge[e] + d * size;
                if (r < INT32_MIN || r > INT32_MAX) continue;
                for (int64_t o = -2; o <= 2; o++) {
                    const int64_t x = r + o;
                    if (x < INT32_MIN || x > INT32_MAX) continue;
                    if (mod_fast((int32_t)x, size) != mod_ref((int32_t)x, size)) {
                        printf("mod %lld %d\n", (long long)x, size);
                        return 1;
                    }
                }
            }
        for (int i = 0; i < (1 << 22); i++) {
            const int32_t r = (int32_t)next32();
            if (mod_fast(r, size) != mod_ref(r, size)) {
                printf("mod %d %d\n", r, size);
                return 1;
            }
        }
    }
    for (int i = 0; i < (1 << 24); i++) {
        const int32_t r = (int32_t)next32(), size = (int32_t)(1 + next32() % 0x40000000u);
        if (mod_fast(r, size) != mod_ref(r, size)) {
            printf("mod %d %d\n", r, size);
            return 1;
        }
    }
    printf("ok\n");
    return 0;
}
