// asan_driver.cpp -- AddressSanitizer / UBSan run of the oracle and the CPU baseline
// (TEST INFRASTRUCTURE ONLY; built and run by `make -C oracle asan-run`, tests/test_oracle_asan.py).
// Exercises every oracle entry point and cpu_baseline.cpp on seeded inputs, including the edge
// shapes (empty, 1 value, < 256, ragged multi-level, duplicates, signed zeros, NaN), and checks
// the round trips the reference guarantees (readObject(writeObject), Delta/Huffman decode(encode),
// restore keys) so a sanitizer report or a mismatch fails the run.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "skml_oracle.h"

extern "C" {
struct cpb_header {
    int32_t bin_num, zero_idx, status, pad;
    double min, max;
};
int cpb_encode(const float* x, int32_t n, int32_t bins, int64_t seed, int32_t threads, uint8_t* codes,
               cpb_header* hdr, double* splits_out);
}

static int fails = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                   \
        }                                                              \
    } while (0)

static std::vector<double> data(int n, int kind, unsigned seed) {
    std::mt19937_64 g(seed);
    std::normal_distribution<double> nd;
    std::vector<double> v(n);
    for (int i = 0; i < n; i++) {
        double x = (double)(float)nd(g);
        if (kind == 1 && (g() % 10) == 0) x = 0.0;
        if (kind == 2) x = (double)(int)(g() % 11) - 5.0;
        if (kind == 3 && (g() % 5) == 0) x = (g() & 1) ? 0.0 : -0.0;
        v[i] = x;
    }
    return v;
}

int main() {
    orc_quant_header* h = (orc_quant_header*)std::malloc(sizeof(orc_quant_header));
    orc_quant_header* h2 = (orc_quant_header*)std::malloc(sizeof(orc_quant_header));
    const int sizes[] = {0, 1, 255, 256, 257, 4096 + 17, 70001, 300000};
    for (int n : sizes)
        for (int kind = 0; kind < 4; kind++)
            for (int bins : {2, 4, 256, 1000}) {
                std::vector<double> v = data(n, kind, (unsigned)(n * 7 + kind * 3 + bins));
                std::vector<int32_t> b(n > 0 ? n : 1), b2(n > 0 ? n : 1);
                CHECK(orc_quantize(v.data(), n, bins, 5, h, b.data()) == ORC_OK);
                if (n > 0) {
                    std::vector<double> vals(h->bin_num);
                    orc_get_values(h, vals.data());
                    const int64_t need = orc_write_ref(h, b.data(), nullptr, 0);
                    std::vector<uint8_t> buf(need);
                    CHECK(orc_write_ref(h, b.data(), buf.data(), need) == need);
                    CHECK(orc_read_ref(buf.data(), need, h2, b2.data(), n) == ORC_OK);
                    CHECK(h2->bin_num == h->bin_num && std::memcmp(b.data(), b2.data(), 4 * (size_t)n) == 0);
                    // the CPU baseline computes the same bins
                    std::vector<float> f(v.begin(), v.end());
                    std::vector<uint8_t> codes(n);
                    std::vector<double> sp(bins);
                    cpb_header ch;
                    CHECK(cpb_encode(f.data(), n, bins, 5, 1, codes.data(), &ch, sp.data()) == 0);
                    CHECK(ch.bin_num == h->bin_num && ch.zero_idx == h->zero_idx);
                    for (int i = 0; i < n; i++) CHECK(codes[i] == (uint8_t)(b[i] - 128));
                    CHECK(orc_parallel_quantize(v.data(), n, bins, 3, 5, h2, b2.data()) == ORC_OK);
                    CHECK(cpb_encode(f.data(), n, bins, 5, 3, codes.data(), &ch, sp.data()) == 0);
                    for (int i = 0; i < n; i++) CHECK(codes[i] == (uint8_t)(b2[i] - 128));
                    orc_times_by(h, 0.5);
                }
                CHECK(orc_uniform_quantize(v.data(), n, bins, h2, b2.data()) == ORC_OK);
            }
    {  // NaN is rejected by the quantile path, binned by the uniform one
        std::vector<double> v = data(1000, 0, 1);
        v[17] = NAN;
        std::vector<int32_t> b(1000);
        CHECK(orc_quantize(v.data(), 1000, 256, 1, h, b.data()) == ORC_E_NAN);
        CHECK(orc_uniform_quantize(v.data(), 1000, 256, h, b.data()) == ORC_OK);
    }
    for (int n : {1, 2, 300, 40000}) {  // sparse: compact, compress, restore; Delta + Huffman
        std::vector<double> dense = data(n * 4, 1, (unsigned)n);
        std::vector<int32_t> keys(dense.size());
        std::vector<double> vals(dense.size());
        const int64_t nnz = orc_to_sparse(dense.data(), (int64_t)dense.size(), keys.data(), vals.data());
        CHECK(nnz == orc_count_nnz(dense.data(), (int64_t)dense.size()));
        if (nnz == 0) continue;
        for (int groups : {2, 8}) {
            orc_sparse s;
            std::memset(&s, 0, sizeof(s));
            std::vector<int32_t> bins(nnz), rk(nnz), rb(nnz);
            const int st = orc_sparse_compress(keys.data(), vals.data(), (int32_t)nnz, 256, groups, 2, 0.3, 1, 2, &s,
                                               bins.data());
            if (st == ORC_E_ARG && s.q.bin_num < groups) {  // calGroupEdges' / by zero, as in Java
                orc_sparse_free(&s);
                continue;
            }
            CHECK(st == ORC_OK);
            CHECK(orc_sparse_restore(&s, rk.data(), rb.data()) == nnz);
            CHECK(std::memcmp(rk.data(), keys.data(), 4 * (size_t)nnz) == 0);
            orc_sparse_free(&s);
        }
        orc_delta d;
        CHECK(orc_delta_encode(keys.data(), (int32_t)nnz, &d) == ORC_OK);
        std::vector<int32_t> back(nnz);
        CHECK(orc_delta_decode(&d, back.data()) == ORC_OK);
        CHECK(std::memcmp(back.data(), keys.data(), 4 * (size_t)nnz) == 0);
        orc_delta_free(&d);
        std::vector<int32_t> tab(nnz);
        for (int64_t i = 0; i < nnz; i++) tab[i] = keys[i] % 37;
        orc_huffman hf;
        CHECK(orc_huffman_encode(tab.data(), (int32_t)nnz, &hf) == ORC_OK);
        std::vector<int32_t> tb(nnz);
        CHECK(orc_huffman_decode(&hf, tb.data()) == ORC_OK);
        CHECK(std::memcmp(tb.data(), tab.data(), 4 * (size_t)nnz) == 0);
        orc_huffman_free(&hf);
    }
    {
        int32_t keys[3] = {5, 5, 7};  // not strictly increasing: "Log for 0"
        orc_delta d;
        CHECK(orc_delta_encode(keys, 3, &d) == ORC_E_ORDER);
    }
    std::free(h);
    std::free(h2);
    std::printf("asan driver: %d check failures\n", fails);
    return fails ? 1 : 0;
}
