// cpu_baseline.cpp -- the reference's dense encode on host cores, for bench.py's cpu_baseline leg.
//
// TEST / MEASUREMENT INFRASTRUCTURE ONLY (like skml_oracle.c): bench.py times it as the CPU
// baseline and tests/ check it against the oracle; the product library never links it.
//
// It restates the reference Java path the way the JVM runs it, in optimised C++ (-O3):
//   QuantileQuantizer.quantize            (quantization/QuantileQuantizer.java:27-50), 1 thread
//   QuantileQuantizer.parallelQuantize    (QuantileQuantizer.java:53-92): T slice sketches on
//                                          T threads, merged in slice order, no Maths.unique
//   Quantizer.quantizeToBins / parallelQuantizeToBins (base/Quantizer.java:87-117): indexOf per
//                                          value, the T-thread variant over the same slicing
// with the sketch of HeapQuantileSketch.java:74-250 / QSketchUtils.java:45-141.  Arrays.sort of
// each 256-value base buffer is std::sort over total-order keys (the JDK sorts doubles with a
// dual-pivot quicksort on `<` and then orders -0.0 before 0.0: the same order).  Values are the
// fp32 gradient widened to double, as the Java double[] would hold them.
//
// RNG: java.util.Random(seed); slice t's sketch draws after the draws of slices 0..t-1 (a sketch
// of m values makes 2C - popcount(C) draws, C = m / 256), the merges after all of them -- the
// schedule the oracle's orc_parallel_quantize runs sequentially, so the results are identical.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kMult = 0x5DEECE66DULL, kAdd = 0xBULL, kMask = (1ULL << 48) - 1;
constexpr int kK = 128, kBase = 256, kLv = 32;

struct JRandom {
    uint64_t s;
    explicit JRandom(int64_t seed) : s(((uint64_t)seed ^ kMult) & kMask) {}
    bool next_boolean() {  // next(1) != 0
        s = (s * kMult + kAdd) & kMask;
        return (s >> 47) != 0;
    }
    void skip(uint64_t k) {  // affine jump-ahead by squaring
        uint64_t a = kMult, c = kAdd;
        while (k) {
            if (k & 1) s = (a * s + c) & kMask;
            c = (a * c + c) & kMask;
            a = (a * a) & kMask;
            k >>= 1;
        }
    }
};

inline uint64_t bits_of(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}
inline double of_bits(uint64_t u) {
    double d;
    std::memcpy(&d, &u, 8);
    return d;
}
// Arrays.sort total order as an unsigned key and back
inline uint64_t tkey(double d) {
    const uint64_t u = bits_of(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
inline double untkey(uint64_t k) { return of_bits((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k); }
// Math.max / Math.min for non-NaN doubles (-0.0 < 0.0)
inline double jmax(double a, double b) {
    if (a == 0.0 && b == 0.0) return (bits_of(a) >> 63) ? b : a;
    return a >= b ? a : b;
}
inline double jmin(double a, double b) {
    if (a == 0.0 && b == 0.0) return (bits_of(b) >> 63) ? b : a;
    return a <= b ? a : b;
}

uint64_t sketch_draws(int64_t n) {
    const uint64_t C = (uint64_t)(n / kBase);
    return 2 * C - (uint64_t)__builtin_popcountll(C);
}

struct Sketch {
    int64_t n = 0;
    double base[kBase];
    int bc = 0;
    uint64_t pattern = 0;
    double lv[kLv][kK];
    double minv = 1.7976931348623157e308, maxv = 4.9e-324;  // HeapQuantileSketch.java:67-68
    bool nan = false;
    JRandom* rng = nullptr;

    // QSketchUtils.compactBuffer: one RNG bit picks the odd or even positions
    void halve(const double* src, double* dst) {
        const int odd = rng->next_boolean() ? 1 : 0;
        for (int j = 0; j < kK; j++) dst[j] = src[odd + 2 * j];
    }
    // mergeArrays: IEEE `<`, a tie emits the newer run first; then compaction
    void carry(int from, int dest) {
        double tmp[2 * kK];
        for (int l = from; l < dest; l++) {
            const double* a = lv[l];
            const double* b = lv[dest];
            int i = 0, j = 0, o = 0;
            while (i < kK && j < kK) tmp[o++] = a[i] < b[j] ? a[i++] : b[j++];
            while (i < kK) tmp[o++] = a[i++];
            while (j < kK) tmp[o++] = b[j++];
            halve(tmp, lv[dest]);
        }
    }
    int first_free(int from) const {
        int l = from;
        while ((pattern >> l) & 1ULL) l++;
        return l;
    }
    // fullBaseBufferPropagation: Arrays.sort, compact, carry
    void flush() {
        uint64_t k[kBase];
        for (int i = 0; i < bc; i++) k[i] = tkey(base[i]);
        std::sort(k, k + bc);
        for (int i = 0; i < bc; i++) base[i] = untkey(k[i]);
        const int dest = first_free(0);
        halve(base, lv[dest]);
        carry(0, dest);
        pattern += 1;
        bc = 0;
    }
    // HeapQuantileSketch.update
    inline void update(double v) {
        if (v != v) {
            nan = true;
            return;
        }
        maxv = jmax(maxv, v);
        minv = jmin(minv, v);
        base[bc++] = v;
        n++;
        if (bc == kBase) flush();
    }
    // HeapQuantileSketch.merge / inPlacePropagationMerge
    void merge(const Sketch& o) {
        if (o.n == 0) return;
        if (n == 0) {
            JRandom* keep = rng;
            *this = o;
            rng = keep;
            return;
        }
        const int64_t total = n + o.n;
        for (int i = 0; i < o.bc; i++) update(o.base[i]);
        for (int l = 0; l < kLv; l++) {
            if (!((o.pattern >> l) & 1ULL)) continue;
            const int dest = first_free(l);
            std::memcpy(lv[dest], o.lv[l], sizeof(lv[dest]));
            carry(l, dest);
            pattern += 1ULL << l;
        }
        n = total;
        maxv = jmax(maxv, o.maxv);
        minv = jmin(minv, o.minv);
        nan = nan || o.nan;
    }
};

// makeSummary + blockyMergeSort + getQuantiles(parts) (HeapQuantileSketch.java:126-174,293-323)
void quantiles(const Sketch& q, int parts, std::vector<double>& splits) {
    std::vector<double> s;
    std::vector<int64_t> w;
    int64_t wt = 1;
    for (int l = 0; l < kLv; l++) {
        wt *= 2;
        if ((q.pattern >> l) & 1ULL)
            for (int i = 0; i < kK; i++) {
                s.push_back(q.lv[l][i]);
                w.push_back(wt);
            }
    }
    const size_t b0 = s.size();
    for (int i = 0; i < q.bc; i++) {
        s.push_back(q.base[i]);
        w.push_back(1);
    }
    {  // the base buffer is sorted (copyBuf2Arr, Arrays.sort)
        std::vector<uint64_t> k(q.bc);
        for (int i = 0; i < q.bc; i++) k[i] = tkey(s[b0 + i]);
        std::sort(k.begin(), k.end());
        for (int i = 0; i < q.bc; i++) s[b0 + i] = untkey(k[i]);
    }
    // blockyMergeSort: a stable merge of sorted runs under `<=`, left run first on ties
    const size_t ns = s.size();
    std::vector<size_t> idx(ns);
    for (size_t i = 0; i < ns; i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return s[a] < s[b]; });
    std::vector<double> ss(ns);
    std::vector<int64_t> cut(ns + 1);
    int64_t acc = 0;
    for (size_t i = 0; i < ns; i++) {
        ss[i] = s[idx[i]];
        cut[i] = acc;
        acc += w[idx[i]];
    }
    cut[ns] = acc;
    splits.assign((size_t)parts - 1, NAN);
    if (ns == 0) return;
    int64_t lo = 0;
    double frac = 1.0 / parts;
    const double step = 1.0 / parts;
    for (int i = 0; i + 1 < parts; i++) {
        int64_t rank = (int64_t)((double)q.n * frac);
        if (rank > q.n - 1) rank = q.n - 1;
        int64_t l = lo, r = (int64_t)ns;
        while (l + 1 < r) {
            const int64_t mid = l + ((r - l) >> 1);
            if (cut[mid] <= rank) l = mid;
            else r = mid;
        }
        splits[i] = ss[l];
        lo = l;
        frac += step;
    }
}

struct Quant {
    std::vector<double> splits;
    int bin_num = 0, zero_idx = 0;
    double mn = 0, mx = 0;
    // Quantizer.indexOf (Quantizer.java:49-72)
    inline int index_of(double x) const {
        const double* s = splits.data();
        const int last = bin_num - 2;
        if (x < s[0]) return 0;
        if (x >= s[last]) return bin_num - 1;
        int l = zero_idx, r = zero_idx;
        if (x < 0.0) l = 0;
        else r = last;
        while (l + 1 < r) {
            const int mid = (l + r) >> 1;
            if (s[mid] > x) {
                if (mid == 0 || s[mid - 1] <= x) return mid;
                r = mid;
            } else {
                l = mid;
            }
        }
        const int mid = (l + r) >> 1;
        return s[mid] <= x ? mid + 1 : mid;
    }
    void find_zero() {  // Quantizer.findZeroIdx
        if (mn > 0.0) zero_idx = 0;
        else if (mx < 0.0) zero_idx = bin_num - 1;
        else {
            int t = 0;
            while (t < bin_num - 1 && splits[t] < 0.0) t++;
            zero_idx = t;
        }
    }
};

// quantizeToBins over [from, to): bins written as the 1-byte (bin - 128) wire values
void bins_range(const Quant& q, const float* x, int64_t from, int64_t to, uint8_t* codes) {
    for (int64_t i = from; i < to; i++) codes[i] = (uint8_t)(q.index_of((double)x[i]) - 128);
}

}  // namespace

extern "C" {

struct cpb_header {
    int32_t bin_num, zero_idx, status, pad;
    double min, max;
};

// One encode of x[0, n) with T threads (T = 1: quantize with Maths.unique; T > 1: parallelQuantize
// + parallelQuantizeToBins).  splits_out: bin_num - 1 doubles (capacity bins - 1).  Returns 0, or
// 2 when the input holds a NaN ("Encounter NaN value").
int cpb_encode(const float* x, int32_t n, int32_t bins, int64_t seed, int32_t threads, uint8_t* codes,
               cpb_header* hdr, double* splits_out) {
    if (bins < 2 || bins > 65536 || threads < 1 || n < 0) return 1;
    Quant q;
    if (threads == 1) {
        JRandom rng(seed);
        Sketch* sk = new Sketch();
        sk->rng = &rng;
        for (int32_t i = 0; i < n; i++) sk->update((double)x[i]);
        if (sk->nan) {
            delete sk;
            return 2;
        }
        quantiles(*sk, bins, q.splits);
        q.mn = sk->minv;
        q.mx = sk->maxv;
        delete sk;
        // QuantileQuantizer.java:38-43: Maths.unique, binNum shrinks
        int o = bins > 1 ? 1 : 0;
        for (int i = 1; i < bins - 1; i++)
            if (q.splits[i] != q.splits[i - 1]) q.splits[o++] = q.splits[i];
        q.splits.resize((size_t)o);
        q.bin_num = o + 1;
        q.find_zero();
        bins_range(q, x, 0, n, codes);
    } else {
        const int32_t per = n / threads;
        std::vector<Sketch*> sk((size_t)threads);
        std::vector<JRandom> rng((size_t)threads, JRandom(seed));
        uint64_t skip = 0;
        for (int t = 0; t < threads; t++) {
            const int32_t from = t * per, to = (t + 1 == threads) ? n : from + per;
            rng[t].skip(skip);
            skip += sketch_draws(to - from);
            sk[t] = new Sketch();
            sk[t]->rng = &rng[t];
        }
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++)
            th.emplace_back([&, t] {
                const int32_t from = t * per, to = (t + 1 == threads) ? n : from + per;
                for (int32_t i = from; i < to; i++) sk[t]->update((double)x[i]);
            });
        for (auto& h : th) h.join();
        th.clear();
        JRandom mrng(seed);  // the merges draw after every slice's draws
        mrng.skip(skip);
        sk[0]->rng = &mrng;
        for (int t = 1; t < threads; t++) sk[0]->merge(*sk[t]);
        const bool nan = sk[0]->nan;
        if (!nan) {
            quantiles(*sk[0], bins, q.splits);
            q.mn = sk[0]->minv;
            q.mx = sk[0]->maxv;
        }
        for (auto* s : sk) delete s;
        if (nan) return 2;
        q.bin_num = bins;  // no Maths.unique (QuantileQuantizer.java:85)
        q.find_zero();
        for (int t = 0; t < threads; t++)
            th.emplace_back([&, t] {
                const int64_t from = (int64_t)t * per, to = (t + 1 == threads) ? n : from + per;
                bins_range(q, x, from, to, codes);
            });
        for (auto& h : th) h.join();
    }
    if (hdr) {
        hdr->bin_num = q.bin_num;
        hdr->zero_idx = q.zero_idx;
        hdr->status = 0;
        hdr->min = q.mn;
        hdr->max = q.mx;
    }
    if (splits_out) std::copy(q.splits.begin(), q.splits.end(), splits_out);
    return 0;
}

// Wall seconds of `reps` encodes (seeds seed, seed+1, ...).
double cpb_bench(const float* x, int32_t n, int32_t bins, int64_t seed, int32_t threads, int32_t reps,
                 uint8_t* codes) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) cpb_encode(x, n, bins, seed + r, threads, codes, nullptr, nullptr);
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // extern "C"
