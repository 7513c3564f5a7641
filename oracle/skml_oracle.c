/*
 * skml_oracle.c -- CPU restatement of the reference SketchML codec.  TEST INFRASTRUCTURE ONLY:
 * the parity checker for the HIP product path (see skml_oracle.h for status, pinning and the
 * RNG model).  Compiled with -ffp-contract=off so double arithmetic rounds like the JVM.
 *
 * Citations: sketch/src/main/java/org/dma/sketchml/sketch/<file>:<line> unless "ml/".
 */
#include "skml_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ======================================================================================
 * java.util.Random -- JDK 8 public spec (48-bit LCG).  Used by QSketchUtils.java:9,47,
 * HashFactory.java:15, Maths.java:42-44.
 * ====================================================================================== */
#define JR_MULT 0x5DEECE66DULL
#define JR_ADD 0xBULL
#define JR_MASK ((1ULL << 48) - 1)

void orc_jr_seed(orc_jrandom* r, int64_t seed) {
    r->s = ((uint64_t)seed ^ JR_MULT) & JR_MASK;
    r->have_gauss = 0;
    r->gauss = 0.0;
}

int32_t orc_jr_next(orc_jrandom* r, int bits) {
    r->s = (r->s * JR_MULT + JR_ADD) & JR_MASK;
    return (int32_t)(uint32_t)(r->s >> (48 - bits));
}

int32_t orc_jr_next_int(orc_jrandom* r) { return orc_jr_next(r, 32); }

int orc_jr_next_boolean(orc_jrandom* r) { return orc_jr_next(r, 1) != 0; }

int32_t orc_jr_next_int_bound(orc_jrandom* r, int32_t bound) {
    int32_t v = orc_jr_next(r, 31);
    int32_t m = bound - 1;
    if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)v) >> 31);
    /* rejection loop with Java int wrap-around in `u - v + m < 0` */
    for (int32_t u = v;; u = orc_jr_next(r, 31)) {
        v = u % bound;
        if ((int32_t)((uint32_t)u - (uint32_t)v + (uint32_t)m) >= 0) break;
    }
    return v;
}

double orc_jr_next_double(orc_jrandom* r) {
    int64_t hi = (int64_t)orc_jr_next(r, 26);
    int64_t lo = (int64_t)orc_jr_next(r, 27);
    return (double)((hi << 27) + lo) * (1.0 / (double)(1ULL << 53));
}

/* polar method; StrictMath.log is fdlibm -- libm log may differ in the last ulp, so this is
 * only used to synthesise App-like data, never as a parity anchor. */
double orc_jr_next_gaussian(orc_jrandom* r) {
    if (r->have_gauss) {
        r->have_gauss = 0;
        return r->gauss;
    }
    double v1, v2, s;
    do {
        v1 = 2 * orc_jr_next_double(r) - 1;
        v2 = 2 * orc_jr_next_double(r) - 1;
        s = v1 * v1 + v2 * v2;
    } while (s >= 1 || s == 0);
    double mul = sqrt(-2 * log(s) / s);
    r->gauss = v2 * mul;
    r->have_gauss = 1;
    return v1 * mul;
}

int orc_jr_bit_at(int64_t seed, int64_t idx) {
    orc_jrandom r;
    orc_jr_seed(&r, seed);
    int b = 0;
    for (int64_t i = 0; i <= idx; i++) b = orc_jr_next_boolean(&r);
    return b;
}

/* ======================================================================================
 * Java double helpers
 * ====================================================================================== */
static uint64_t dbits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}

/* Math.max / Math.min for non-NaN doubles (JDK spec: -0.0 < +0.0) */
static double jmax(double a, double b) {
    if (a == 0.0 && b == 0.0) return (dbits(a) >> 63) ? b : a;
    return a >= b ? a : b;
}
static double jmin(double a, double b) {
    if (a == 0.0 && b == 0.0) return (dbits(b) >> 63) ? b : a;
    return a <= b ? a : b;
}

/* Arrays.sort(double[]) order: total order, -0.0 before 0.0 (NaN never reaches it here). */
static uint64_t total_key(double x) {
    uint64_t u = dbits(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
static int cmp_total(const void* a, const void* b) {
    uint64_t ka = total_key(*(const double*)a), kb = total_key(*(const double*)b);
    return ka < kb ? -1 : (ka > kb ? 1 : 0);
}
static void java_sort(double* a, int64_t len) {
    if (len > 1) qsort(a, (size_t)len, sizeof(double), cmp_total);
}

/* ======================================================================================
 * HeapQuantileSketch (sketch/quantile/HeapQuantileSketch.java) with k = 128.
 * State: a 2k base buffer plus per-level k-sample nodes; `pattern` is the binary counter
 * n / 2k whose set bits say which levels hold a node (HeapQuantileSketch.java:24-27).
 * ====================================================================================== */
#define QS_K 128
#define QS_MAXLV 64

typedef struct {
    int64_t n;
    double base[2 * QS_K];
    int base_count;
    uint64_t pattern;
    double level[QS_MAXLV][QS_K];
    double minv, maxv;
    orc_jrandom* rng;
} qsk;

static void qsk_init(qsk* q, orc_jrandom* rng) {
    q->n = 0;
    q->base_count = 0;
    q->pattern = 0;
    q->minv = 1.7976931348623157e308;  /* Double.MAX_VALUE (HeapQuantileSketch.java:67) */
    q->maxv = 4.9e-324;                /* Double.MIN_VALUE (HeapQuantileSketch.java:68) */
    q->rng = rng;
}

/* QSketchUtils.compactBuffer (QSketchUtils.java:45-51): one RNG bit picks odd/even positions */
static void qsk_halve(qsk* q, const double* src, double* dst) {
    int odd = orc_jr_next_boolean(q->rng);
    for (int j = 0; j < QS_K; j++) dst[j] = src[odd + 2 * j];
}

/* QSketchUtils.mergeArrays (QSketchUtils.java:53-69): IEEE `<`, a tie emits the NEWER run */
static void qsk_merge_runs(const double* older, const double* newer, double* out) {
    int i = 0, j = 0, o = 0;
    while (i < QS_K && j < QS_K) out[o++] = (older[i] < newer[j]) ? older[i++] : newer[j++];
    while (i < QS_K) out[o++] = older[i++];
    while (j < QS_K) out[o++] = newer[j++];
}

/* Carry a fresh node (already compacted into level[dest]) through the occupied levels
 * [from, dest): QSketchUtils.levelwisePropagation (QSketchUtils.java:71-82). */
static void qsk_carry(qsk* q, int from, int dest) {
    double scratch[2 * QS_K];
    for (int lv = from; lv < dest; lv++) {
        qsk_merge_runs(q->level[lv], q->level[dest], scratch);
        qsk_halve(q, scratch, q->level[dest]);
    }
}

static int first_free_level(uint64_t pattern, int from) {
    int lv = from;
    while ((pattern >> lv) & 1ULL) lv++;
    return lv;
}

/* fullBaseBufferPropagation + inPlacePropagationUpdate (HeapQuantileSketch.java:107-124) */
static void qsk_flush_base(qsk* q) {
    java_sort(q->base, q->base_count);
    int dest = first_free_level(q->pattern, 0);
    qsk_halve(q, q->base, q->level[dest]);
    qsk_carry(q, 0, dest);
    q->pattern += 1ULL;
    q->base_count = 0;
}

/* HeapQuantileSketch.update (HeapQuantileSketch.java:74-86) */
static int qsk_update(qsk* q, double v) {
    if (v != v) return ORC_E_NAN; /* "Encounter NaN value" (:75-76) */
    q->maxv = jmax(q->maxv, v);
    q->minv = jmin(q->minv, v);
    q->base[q->base_count++] = v;
    q->n++;
    if (q->base_count == 2 * QS_K) qsk_flush_base(q);
    return ORC_OK;
}

/* HeapQuantileSketch.merge / inPlacePropagationMerge / copy (HeapQuantileSketch.java:186-250) */
static int qsk_merge(qsk* q, const qsk* o) {
    if (o->n == 0) return ORC_OK;
    if (q->n == 0) {
        orc_jrandom* keep = q->rng;
        *q = *o;
        q->rng = keep;
        return ORC_OK;
    }
    int64_t total = q->n + o->n;
    for (int i = 0; i < o->base_count; i++) {
        int st = qsk_update(q, o->base[i]);
        if (st) return st;
    }
    for (int lv = 0; lv < QS_MAXLV; lv++) {
        if (!((o->pattern >> lv) & 1ULL)) continue;
        int dest = first_free_level(q->pattern, lv);
        memcpy(q->level[dest], o->level[lv], sizeof(q->level[dest]));
        qsk_carry(q, lv, dest);
        q->pattern += 1ULL << lv;
    }
    q->n = total;
    q->maxv = jmax(q->maxv, o->maxv);
    q->minv = jmin(q->minv, o->minv);
    return ORC_OK;
}

/* QSketchUtils.blockyMerge (QSketchUtils.java:113-140): `<=`, ties emit the LEFT run */
static void blocky_merge(const double* ks, const int64_t* vs, int64_t a0, int64_t alen, int64_t b0,
                         int64_t blen, double* kd, int64_t* vd, int64_t d0) {
    int64_t i = a0, j = b0, o = d0, ae = a0 + alen, be = b0 + blen;
    while (i < ae && j < be) {
        if (ks[i] <= ks[j]) {
            kd[o] = ks[i];
            vd[o++] = vs[i++];
        } else {
            kd[o] = ks[j];
            vd[o++] = vs[j++];
        }
    }
    while (i < ae) { kd[o] = ks[i]; vd[o++] = vs[i++]; }
    while (j < be) { kd[o] = ks[j]; vd[o++] = vs[j++]; }
}

/* recursiveBlockyMergeSort (QSketchUtils.java:91-111): src/dst swap roles per recursion level */
static void blocky_sort_rec(double* ksrc, int64_t* vsrc, double* kdst, int64_t* vdst, int64_t blk0,
                            int64_t nblk, int64_t bs, int64_t limit) {
    if (nblk == 1) return;
    int64_t n1 = nblk >> 1, n2 = nblk - n1;
    blocky_sort_rec(kdst, vdst, ksrc, vsrc, blk0, n1, bs, limit);
    blocky_sort_rec(kdst, vdst, ksrc, vsrc, blk0 + n1, n2, bs, limit);
    int64_t a0 = blk0 * bs, b0 = (blk0 + n1) * bs, alen = n1 * bs, blen = n2 * bs;
    if (b0 + blen > limit) blen = limit - b0;
    blocky_merge(ksrc, vsrc, a0, alen, b0, blen, kdst, vdst, a0);
}

static void blocky_sort(double* keys, int64_t* vals, int64_t len, int64_t bs) {
    if (len <= bs) return;
    int64_t nblk = (len + bs - 1) / bs;
    double* tk = (double*)malloc(sizeof(double) * (size_t)len);
    int64_t* tv = (int64_t*)malloc(sizeof(int64_t) * (size_t)len);
    memcpy(tk, keys, sizeof(double) * (size_t)len);
    memcpy(tv, vals, sizeof(int64_t) * (size_t)len);
    blocky_sort_rec(tk, tv, keys, vals, 0, nblk, bs, len);
    free(tk);
    free(tv);
}

/* makeSummary + copyBuf2Arr (HeapQuantileSketch.java:126-174).  samples/weights sized by caller
 * (numSamples <= 64*k + 2k).  weights gets the exclusive prefix, numSamples+1 entries. */
static int64_t qsk_summary(const qsk* q, double* samples, int64_t* weights) {
    int64_t cur = 0, w = 1;
    for (int lv = 0; lv < QS_MAXLV; lv++) {
        w *= 2;
        if ((q->pattern >> lv) & 1ULL) {
            for (int i = 0; i < QS_K; i++) {
                samples[cur] = q->level[lv][i];
                weights[cur++] = w;
            }
        }
        if ((q->pattern >> lv) == 0) break;
    }
    int64_t base0 = cur;
    for (int i = 0; i < q->base_count; i++) {
        samples[cur] = q->base[i];
        weights[cur++] = 1;
    }
    weights[cur] = 0;
    java_sort(samples + base0, cur - base0);
    blocky_sort(samples, weights, cur, QS_K);
    int64_t acc = 0;
    for (int64_t i = 0; i <= cur; i++) {
        int64_t nx = acc + weights[i];
        weights[i] = acc;
        acc = nx;
    }
    return cur;
}

/* getQuantiles(int evenPartition) (HeapQuantileSketch.java:293-323) */
static int qsk_quantiles(const qsk* q, int32_t parts, double* splits) {
    if (parts <= 1) return ORC_E_ARG; /* "Invalid partition number" (QSketchUtils.java:40-43) */
    int64_t cap = 2 * QS_K + (int64_t)QS_K * QS_MAXLV + 1;
    double* samples = (double*)malloc(sizeof(double) * (size_t)cap);
    int64_t* weights = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t ns = qsk_summary(q, samples, weights);
    if (ns == 0) {
        for (int i = 0; i + 1 < parts; i++) splits[i] = NAN;
    } else {
        int64_t lo = 0;
        double frac = 1.0 / parts, step = 1.0 / parts;
        for (int i = 0; i + 1 < parts; i++) {
            int64_t rank = (int64_t)((double)q->n * frac);
            if (rank > q->n - 1) rank = q->n - 1;
            /* largest index with weights[idx] <= rank, searched upward from the last answer */
            int64_t l = lo, r = ns;
            while (l + 1 < r) {
                int64_t mid = l + ((r - l) >> 1);
                if (weights[mid] <= rank) l = mid;
                else r = mid;
            }
            splits[i] = samples[l];
            lo = l;
            frac += step;
        }
    }
    free(samples);
    free(weights);
    return ORC_OK;
}

int64_t orc_sketch_summary(const double* values, int64_t n, int64_t seed, double* samples,
                           int64_t* weights, int64_t cap, double* min_out, double* max_out) {
    orc_jrandom rng;
    orc_jr_seed(&rng, seed);
    qsk* q = (qsk*)malloc(sizeof(qsk));
    qsk_init(q, &rng);
    for (int64_t i = 0; i < n; i++)
        if (qsk_update(q, values[i])) { free(q); return -ORC_E_NAN; }
    int64_t need = (int64_t)__builtin_popcountll(q->pattern) * QS_K + q->base_count + 1;
    if (need > cap) { free(q); return -ORC_E_ARG; }
    int64_t ns = qsk_summary(q, samples, weights);
    if (min_out) *min_out = q->minv;
    if (max_out) *max_out = q->maxv;
    free(q);
    return ns;
}

int orc_sketch_quantiles(const double* values, int64_t n, int64_t seed, int32_t parts,
                         double* splits) {
    orc_jrandom rng;
    orc_jr_seed(&rng, seed);
    qsk* q = (qsk*)malloc(sizeof(qsk));
    qsk_init(q, &rng);
    for (int64_t i = 0; i < n; i++)
        if (qsk_update(q, values[i])) { free(q); return ORC_E_NAN; }
    int st = qsk_quantiles(q, parts, splits);
    free(q);
    return st;
}

/* ======================================================================================
 * Quantizer / QuantileQuantizer
 * ====================================================================================== */

/* Maths.unique (util/Maths.java:51-67): drop a split equal (IEEE ==) to its predecessor */
static int32_t java_unique(double* s, int32_t len) {
    if (len == 0) return 0;
    int32_t o = 1;
    for (int32_t i = 1; i < len; i++)
        if (s[i] != s[i - 1]) s[o++] = s[i];
    return o;
}

/* Quantizer.findZeroIdx (Quantizer.java:74-85) */
static void find_zero_idx(orc_quant_header* h) {
    if (h->min > 0.0) h->zero_idx = 0;
    else if (h->max < 0.0) h->zero_idx = h->bin_num - 1;
    else {
        int32_t t = 0;
        while (t < h->bin_num - 1 && h->splits[t] < 0.0) t++;
        h->zero_idx = t;
    }
}

/* Quantizer.indexOf (Quantizer.java:49-72), restated with the same zero-seeded bisection */
int32_t orc_index_of(const orc_quant_header* h, double x) {
    const double* s = h->splits;
    int32_t last = h->bin_num - 2;
    if (x < s[0]) return 0;
    if (x >= s[last]) return h->bin_num - 1;
    int32_t lo = h->zero_idx, hi = h->zero_idx;
    if (x < 0.0) lo = 0;
    else hi = last;
    while (lo + 1 < hi) {
        int32_t mid = (lo + hi) >> 1;
        if (s[mid] > x) {
            if (mid == 0 || s[mid - 1] <= x) return mid;
            hi = mid;
        } else {
            lo = mid;
        }
    }
    int32_t mid = (lo + hi) >> 1;
    return s[mid] <= x ? mid + 1 : mid;
}

int orc_quantize(const double* values, int32_t n, int32_t bin_num, int64_t seed,
                 orc_quant_header* hdr, int32_t* bins) {
    if (bin_num <= 1 || bin_num > 65536) return ORC_E_ARG;
    orc_jrandom rng;
    orc_jr_seed(&rng, seed);
    qsk* q = (qsk*)malloc(sizeof(qsk));
    if (!q) return ORC_E_OOM;
    qsk_init(q, &rng);
    for (int32_t i = 0; i < n; i++)
        if (qsk_update(q, values[i])) { free(q); return ORC_E_NAN; }
    hdr->n = n;
    hdr->min = q->minv;
    hdr->max = q->maxv;
    int st = qsk_quantiles(q, bin_num, hdr->splits);
    free(q);
    if (st) return st;
    /* QuantileQuantizer.java:38-43: dedup, shrink binNum (WARN in Java) */
    hdr->bin_num = java_unique(hdr->splits, bin_num - 1) + 1;
    find_zero_idx(hdr);
    if (bins)
        for (int32_t i = 0; i < n; i++) bins[i] = orc_index_of(hdr, values[i]);
    return ORC_OK;
}

/* QuantileQuantizer.quantize (QuantileQuantizer.java:27-43) up to findZeroIdx on float input
 * widened to double; n may exceed a Java int only in the sense that hdr->n is then meaningless
 * (the tests stay at or below 2^30). */
int orc_quantize_header_f32(const float* values, int64_t n, int32_t bin_num, int64_t seed, orc_quant_header* hdr) {
    if (bin_num <= 1 || bin_num > 65536) return ORC_E_ARG;
    orc_jrandom rng;
    orc_jr_seed(&rng, seed);
    qsk* q = (qsk*)malloc(sizeof(qsk));
    if (!q) return ORC_E_OOM;
    qsk_init(q, &rng);
    for (int64_t i = 0; i < n; i++)
        if (qsk_update(q, (double)values[i])) { free(q); return ORC_E_NAN; }
    hdr->n = (int32_t)n;
    hdr->min = q->minv;
    hdr->max = q->maxv;
    int st = qsk_quantiles(q, bin_num, hdr->splits);
    free(q);
    if (st) return st;
    hdr->bin_num = java_unique(hdr->splits, bin_num - 1) + 1;
    find_zero_idx(hdr);
    return ORC_OK;
}

void orc_index_of_many_f32(const orc_quant_header* h, const float* x, int64_t n, int32_t* bins) {
    for (int64_t i = 0; i < n; i++) bins[i] = orc_index_of(h, (double)x[i]);
}

int orc_parallel_quantize(const double* values, int32_t n, int32_t bin_num, int32_t threads,
                          int64_t seed, orc_quant_header* hdr, int32_t* bins) {
    if (bin_num <= 1 || bin_num > 65536 || threads < 1) return ORC_E_ARG;
    /* One schedule the reference can run: the T slice sketches one after another, then the
     * merges, all drawing from the one static Random (QSketchUtils.java:9) seeded with `seed`. */
    orc_jrandom rng;
    orc_jr_seed(&rng, seed);
    qsk* sk = (qsk*)malloc(sizeof(qsk) * (size_t)threads);
    int st = ORC_OK;
    int32_t per = n / threads;
    for (int32_t t = 0; t < threads && !st; t++) {
        qsk_init(&sk[t], &rng);
        int32_t from = t * per, to = (t + 1 == threads) ? n : from + per;
        for (int32_t i = from; i < to && !st; i++) st = qsk_update(&sk[t], values[i]);
    }
    for (int32_t t = 1; t < threads && !st; t++) st = qsk_merge(&sk[0], &sk[t]);
    if (!st) {
        hdr->n = n;
        hdr->min = sk[0].minv;
        hdr->max = sk[0].maxv;
        st = qsk_quantiles(&sk[0], bin_num, hdr->splits);
        hdr->bin_num = bin_num; /* no Maths.unique here (QuantileQuantizer.java:85) */
        find_zero_idx(hdr);
        if (bins && !st)
            for (int32_t i = 0; i < n; i++) bins[i] = orc_index_of(hdr, values[i]);
    }
    free(sk);
    return st;
}

int orc_uniform_quantize(const double* values, int32_t n, int32_t bin_num, orc_quant_header* hdr,
                         int32_t* bins) {
    if (bin_num <= 1 || bin_num > 65536) return ORC_E_ARG;
    /* UniformQuantizer.java:24-29 */
    double mn = 1.7976931348623157e308, mx = 4.9e-324;
    for (int32_t i = 0; i < n; i++) {
        const double v = values[i];
        if (v < mn) mn = v;
        if (v > mx) mx = v;
    }
    /* UniformQuantizer.java:31-36: sequential accumulation, every add rounded */
    const double step = (mx - mn) / bin_num;
    const int32_t ns = bin_num - 1;
    hdr->n = n;
    hdr->min = mn;
    hdr->max = mx;
    hdr->bin_num = bin_num;
    if (ns > 0) hdr->splits[0] = mn + step;
    for (int32_t i = 1; i < ns; i++) hdr->splits[i] = hdr->splits[i - 1] + step;
    find_zero_idx(hdr); /* UniformQuantizer.java:38 */
    if (bins)
        for (int32_t i = 0; i < n; i++) bins[i] = orc_index_of(hdr, values[i]);
    return ORC_OK;
}

void orc_get_values(const orc_quant_header* h, double* out) {
    int32_t ns = h->bin_num - 1;
    out[0] = 0.5 * (h->min + h->splits[0]);
    for (int32_t i = 1; i < ns; i++) out[i] = 0.5 * (h->splits[i - 1] + h->splits[i]);
    out[ns] = 0.5 * (h->splits[ns - 1] + h->max);
}

void orc_times_by(orc_quant_header* h, double x) {
    h->min *= x;
    h->max *= x;
    for (int32_t i = 0; i + 1 < h->bin_num; i++) h->splits[i] *= x;
}

/* ---- DataOutput big-endian primitives ---- */
static void put_be(uint8_t* p, uint64_t v, int nbytes) {
    for (int i = nbytes - 1; i >= 0; i--) {
        p[i] = (uint8_t)(v & 0xFF);
        v >>= 8;
    }
}
static uint64_t get_be(const uint8_t* p, int nbytes) {
    uint64_t v = 0;
    for (int i = 0; i < nbytes; i++) v = (v << 8) | p[i];
    return v;
}

int64_t orc_write_ref(const orc_quant_header* h, const int32_t* bins, uint8_t* buf, int64_t cap) {
    int32_t ns = h->bin_num - 1;
    int w = h->bin_num <= 256 ? 1 : (h->bin_num <= 65536 ? 2 : 4);
    int64_t need = 4 + 4 + 8LL * ns + 4 + 8 + 8 + 4 + (int64_t)w * h->n;
    if (!buf) return need;
    if (cap < need) return -ORC_E_ARG;
    uint8_t* p = buf;
    put_be(p, (uint32_t)h->bin_num, 4); p += 4;
    put_be(p, (uint32_t)h->n, 4); p += 4;
    for (int32_t i = 0; i < ns; i++) { put_be(p, dbits(h->splits[i]), 8); p += 8; }
    put_be(p, (uint32_t)h->zero_idx, 4); p += 4;
    put_be(p, dbits(h->min), 8); p += 8;
    put_be(p, dbits(h->max), 8); p += 8;
    put_be(p, (uint32_t)h->n, 4); p += 4;
    for (int32_t i = 0; i < h->n; i++) {
        if (w == 1) *p++ = (uint8_t)(bins[i] - 128);
        else if (w == 2) { put_be(p, (uint16_t)(bins[i] - 32768), 2); p += 2; }
        else { put_be(p, (uint32_t)bins[i], 4); p += 4; }
    }
    return need;
}

int orc_read_ref(const uint8_t* buf, int64_t len, orc_quant_header* h, int32_t* bins,
                 int32_t bins_cap) {
    const uint8_t* p = buf;
    if (len < 8) return ORC_E_ARG;
    h->bin_num = (int32_t)get_be(p, 4); p += 4;
    h->n = (int32_t)get_be(p, 4); p += 4;
    int32_t ns = h->bin_num - 1;
    if (ns < 0 || ns > 65535) return ORC_E_ARG;
    for (int32_t i = 0; i < ns; i++) {
        uint64_t u = get_be(p, 8);
        memcpy(&h->splits[i], &u, 8);
        p += 8;
    }
    h->zero_idx = (int32_t)get_be(p, 4); p += 4;
    uint64_t u = get_be(p, 8); memcpy(&h->min, &u, 8); p += 8;
    u = get_be(p, 8); memcpy(&h->max, &u, 8); p += 8;
    int32_t nb = (int32_t)get_be(p, 4); p += 4;
    if (nb > bins_cap) return ORC_E_ARG;
    int w = h->bin_num <= 256 ? 1 : (h->bin_num <= 65536 ? 2 : 4);
    for (int32_t i = 0; i < nb; i++) {
        if (w == 1) bins[i] = (int32_t)(int8_t)p[0] + 128, p += 1;
        else if (w == 2) bins[i] = (int32_t)(int16_t)get_be(p, 2) + 32768, p += 2;
        else bins[i] = (int32_t)get_be(p, 4), p += 4;
    }
    return ORC_OK;
}

/* ======================================================================================
 * Sparse path
 * ====================================================================================== */
int64_t orc_count_nnz(const double* dense, int64_t dim) {
    int64_t c = 0;
    for (int64_t i = 0; i < dim; i++) c += fabs(dense[i]) > 1e-8; /* ml/util/Maths.scala:8 EPS */
    return c;
}

int64_t orc_to_sparse(const double* dense, int64_t dim, int32_t* keys, double* vals) {
    int64_t j = 0;
    for (int64_t i = 0; i < dim; i++)
        if (fabs(dense[i]) > 1e-8) { keys[j] = (int32_t)i; vals[j++] = dense[i]; }
    return j;
}

/* Java int helpers: wrap-around add/mul/shl, arithmetic >>, truncating % */
static inline int32_t ji_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t ji_mul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t ji_shl(int32_t a, int s) { return (int32_t)((uint32_t)a << (s & 31)); }
static inline int32_t ji_sar(int32_t a, int s) { return a >> (s & 31); }
static inline int32_t fold_mod(int32_t code, int32_t size) {
    code %= size;
    return code >= 0 ? code : code + size;
}

/* hash/BJHash.java:10-20 */
static int32_t h_bj(int32_t c, int32_t size) {
    c = ji_add(ji_add(c, 0x7ed55d16), ji_shl(c, 12));
    c = (c ^ (int32_t)0xc761c23c) ^ ji_sar(c, 19);
    c = ji_add(ji_add(c, 0x165667b1), ji_shl(c, 5));
    c = ji_add(c, (int32_t)0xd3a2646c) ^ ji_shl(c, 9);
    c = ji_add(ji_add(c, (int32_t)0xfd7046c5), ji_shl(c, 3));
    c = (c ^ (int32_t)0xb55a4f09) ^ ji_sar(c, 16);
    return fold_mod(c, size);
}
/* hash/Mix64Hash.java:10-21 */
static int32_t h_mix64(int32_t c, int32_t size) {
    c = ji_add(~c, ji_shl(c, 21));
    c = c ^ ji_sar(c, 24);
    c = ji_add(ji_add(c, ji_shl(c, 3)), ji_shl(c, 8));
    c = c ^ ji_sar(c, 14);
    c = ji_add(ji_add(c, ji_shl(c, 2)), ji_shl(c, 4));
    c = c ^ ji_sar(c, 28);
    c = ji_add(c, ji_shl(c, 31));
    return fold_mod(c, size);
}
/* hash/TWHash.java:10-20 */
static int32_t h_tw(int32_t c, int32_t size) {
    c = ji_add(~c, ji_shl(c, 15));
    c = c ^ ji_sar(c, 12);
    c = ji_add(c, ji_shl(c, 2));
    c = c ^ ji_sar(c, 4);
    c = ji_mul(c, 2057);
    c = c ^ ji_sar(c, 16);
    return fold_mod(c, size);
}
/* hash/BKDRHash.java:13-21 */
static int32_t h_bkdr(int32_t key, int32_t seed, int32_t size) {
    int32_t c = 0;
    while (key != 0) {
        c = ji_add(ji_mul(seed, c), key % 10);
        key /= 10;
    }
    return fold_mod(c, size);
}

int32_t orc_hash(int32_t id, int32_t key, int32_t size) {
    static const int32_t bkdr_seed[8] = {0, 0, 0, 31, 131, 267, 1313, 13131};
    switch (id) {
        case 0: return h_bj(key, size);
        case 1: return h_mix64(key, size);
        case 2: return h_tw(key, size);
        default: return h_bkdr(key, bkdr_seed[id & 7], size);
    }
}

/* HashFactory.getRandomInt2IntHashes + Maths.shuffle (HashFactory.java:23-38, Maths.java:41-49) */
void orc_pick_hashes(int64_t seed, int32_t rows, int32_t* ids) {
    int32_t idx[8];
    for (int i = 0; i < 8; i++) idx[i] = i;
    orc_jrandom r;
    orc_jr_seed(&r, seed);
    for (int i = 7; i > 0; i--) {
        int32_t j = orc_jr_next_int_bound(&r, i + 1);
        int32_t t = idx[j];
        idx[j] = idx[i];
        idx[i] = t;
    }
    for (int i = 0; i < rows; i++) ids[i] = idx[i];
}

/* FSketchUtils.calGroupEdges (frequency/FSketchUtils.java:9-28).  Returns ORC_E_ARG where Java's
 * `zeroIdx % bpg` throws ArithmeticException (bin_num < group_num and zeroIdx >= 0 = bpg). */
int orc_group_edges(int32_t zero_idx, int32_t bin_num, int32_t group_num, int32_t* edges) {
    if (group_num == 2) {
        edges[0] = zero_idx;
        edges[1] = bin_num;
        return ORC_OK;
    }
    int32_t bpg = bin_num / group_num;
    if (zero_idx < bpg) edges[0] = zero_idx;
    else if (bpg == 0) return ORC_E_ARG;
    else if ((zero_idx % bpg) < (bpg / 2)) edges[0] = bpg + zero_idx % bpg;
    else edges[0] = zero_idx % bpg;
    for (int32_t i = 1; i < group_num - 1; i++) edges[i] = edges[i - 1] + bpg;
    edges[group_num - 1] = bin_num;
    return ORC_OK;
}

/* ---- BitSet as little-endian uint64 words; BinaryUtils.setBits writes MSB first ---- */
typedef struct {
    uint64_t* w;
    int64_t cap_words;
} bitbuf;

static void bb_reserve(bitbuf* b, int64_t nbits) {
    int64_t need = (nbits + 63) / 64 + 1;
    if (need <= b->cap_words) return;
    int64_t nc = b->cap_words ? b->cap_words * 2 : 64;
    while (nc < need) nc *= 2;
    b->w = (uint64_t*)realloc(b->w, sizeof(uint64_t) * (size_t)nc);
    memset(b->w + b->cap_words, 0, sizeof(uint64_t) * (size_t)(nc - b->cap_words));
    b->cap_words = nc;
}
/* BinaryUtils.setBits (binary/BinaryUtils.java:6-14) */
static void bb_put(bitbuf* b, int64_t off, uint32_t value, int nbits) {
    bb_reserve(b, off + nbits);
    for (int i = 0; i < nbits; i++) {
        int sh = nbits - 1 - i;
        int bit = sh < 32 ? (int)((value >> sh) & 1u) : 0;
        if (bit) b->w[(off + i) >> 6] |= 1ULL << ((off + i) & 63);
    }
}
static int bb_get1(const uint64_t* w, int64_t nwords, int64_t pos) {
    int64_t wi = pos >> 6;
    if (wi >= nwords) return 0;
    return (int)((w[wi] >> (pos & 63)) & 1ULL);
}
/* BinaryUtils.getBits (binary/BinaryUtils.java:16-25) */
static int32_t bb_getn(const uint64_t* w, int64_t nwords, int64_t off, int nbits) {
    uint32_t r = 0;
    for (int i = 0; i < nbits; i++) r = (r << 1) | (uint32_t)bb_get1(w, nwords, off + i);
    return (int32_t)r;
}
/* BitSet.toLongArray: words up to the last non-zero word */
static int32_t bb_trim(const bitbuf* b) {
    int64_t n = b->cap_words;
    while (n > 0 && b->w[n - 1] == 0) n--;
    return (int32_t)n;
}

static int32_t log2nlz(int32_t k) { return 31 - __builtin_clz((uint32_t)k); }

/* DeltaAdaptiveEncoder.calOptimalIntervals (binary/DeltaAdaptiveEncoder.java:23-51) */
static void delta_choose(const double* prob, int32_t* m_out, int32_t* kind_out) {
    double best = 32.0;
    int32_t bm = 1, bk = 0;
    for (int32_t m = 2; m <= 16; m *= 2) {
        double iprob[16] = {0};
        int32_t b = 32 / m;
        double sum = 0.0;
        for (int32_t i = 0; i < m; i++) {
            for (int32_t j = 0; j < b; j++) iprob[i] += prob[i * b + j];
            sum += (i + 1) * iprob[i];
        }
        double t1 = sum * b + log2nlz(m);
        if (t1 < best) { best = t1; bm = m; bk = 0; }
        double t2 = sum * (b + 1) + 1;
        if (t2 < best) { best = t2; bm = m; bk = 1; }
    }
    *m_out = bm;
    *kind_out = bk;
}

int orc_delta_encode(const int32_t* keys, int32_t n, orc_delta* out) {
    memset(out, 0, sizeof(*out));
    if (n <= 0) return ORC_E_ARG;
    int32_t* delta = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    int8_t* need = (int8_t*)malloc((size_t)n);
    double prob[32] = {0};
    for (int32_t i = 0; i < n; i++) {
        delta[i] = i == 0 ? keys[0] : (int32_t)((uint32_t)keys[i] - (uint32_t)keys[i - 1]);
        if (i == 0 && delta[0] == 0) need[0] = 1;
        else {
            if (delta[i] <= 0) { free(delta); free(need); return ORC_E_ORDER; } /* "Log for" */
            need[i] = (int8_t)(log2nlz(delta[i]) + 1);
        }
        prob[need[i]] += 1.0;
    }
    for (int i = 0; i < 32; i++) prob[i] /= n;
    int32_t m, kind;
    delta_choose(prob, &m, &kind);
    int32_t bpi = 32 / m, shift = log2nlz(bpi);
    bitbuf fb = {0}, db = {0};
    int64_t fo = 0, dof = 0;
    for (int32_t i = 0; i < n; i++) {
        int32_t iv = (need[i] + bpi - 1) >> shift;
        if (!kind) {
            int32_t nf = log2nlz(m);
            bb_put(&fb, fo, (uint32_t)(iv - 1), nf);
            fo += nf;
        } else {
            bb_put(&fb, fo, (uint32_t)((1u << (iv + 1)) - 2u), iv + 1);
            fo += iv + 1;
        }
        bb_put(&db, dof, (uint32_t)delta[i], bpi * iv);
        dof += (int64_t)bpi * iv;
    }
    bb_reserve(&fb, 1);
    bb_reserve(&db, 1);
    out->size = n;
    out->num_intervals = m;
    out->flag_kind = kind;
    out->n_flag_bits = fo;
    out->n_delta_bits = dof;
    out->flag_words = fb.w;
    out->delta_words = db.w;
    out->n_flag_longs = bb_trim(&fb);
    out->n_delta_longs = bb_trim(&db);
    free(delta);
    free(need);
    return ORC_OK;
}

int orc_delta_decode(const orc_delta* d, int32_t* res) {
    int32_t bpi = 32 / d->num_intervals;
    int64_t fo = 0, dof = 0;
    int32_t prev = 0;
    for (int32_t i = 0; i < d->size; i++) {
        int32_t iv;
        if (!d->flag_kind) {
            int32_t nf = log2nlz(d->num_intervals);
            iv = bb_getn(d->flag_words, d->n_flag_longs, fo, nf) + 1;
            fo += nf;
        } else {
            iv = 0;
            while (bb_get1(d->flag_words, d->n_flag_longs, fo++)) iv++;
        }
        int32_t dl = bb_getn(d->delta_words, d->n_delta_longs, dof, bpi * iv);
        dof += (int64_t)bpi * iv;
        res[i] = (int32_t)((uint32_t)prev + (uint32_t)dl);
        prev = res[i];
    }
    return ORC_OK;
}

void orc_delta_free(orc_delta* d) {
    free(d->flag_words);
    free(d->delta_words);
    d->flag_words = d->delta_words = NULL;
}

/* ---- HuffmanEncoder (binary/HuffmanEncoder.java:88-166).  The tree is built with a
 * restatement of JDK 8 java.util.PriorityQueue (binary heap, siftUp/siftDown with the
 * occurrence comparator), fed in ascending value order (Int2ObjectRBTreeMap iteration). ---- */
typedef struct hnode {
    int32_t value, occ, leaf;
    int32_t left, right; /* indices into node pool */
} hnode;

static void pq_sift_up(int32_t* q, int32_t k, int32_t x, const hnode* pool) {
    while (k > 0) {
        int32_t parent = (k - 1) >> 1;
        int32_t e = q[parent];
        if (pool[x].occ >= pool[e].occ) break;
        q[k] = e;
        k = parent;
    }
    q[k] = x;
}
static void pq_sift_down(int32_t* q, int32_t size, int32_t k, int32_t x, const hnode* pool) {
    int32_t half = size >> 1;
    while (k < half) {
        int32_t child = (k << 1) + 1;
        int32_t c = q[child];
        int32_t right = child + 1;
        if (right < size && pool[c].occ > pool[q[right]].occ) c = q[child = right];
        if (pool[x].occ <= pool[c].occ) break;
        q[k] = c;
        k = child;
    }
    q[k] = x;
}
static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return x < y ? -1 : (x > y);
}
typedef struct { int32_t value, bits, nbits; } hitem;
static void h_traverse(const hnode* pool, int32_t nd, int32_t bits, int32_t depth, hitem* items,
                       int32_t* ni) {
    if (pool[nd].leaf) {
        items[*ni].value = pool[nd].value;
        items[*ni].bits = bits;
        items[*ni].nbits = depth == 0 ? 1 : depth;
        (*ni)++;
    } else {
        h_traverse(pool, pool[nd].left, (int32_t)((uint32_t)bits << 1), depth + 1, items, ni);
        h_traverse(pool, pool[nd].right, (int32_t)(((uint32_t)bits << 1) | 1u), depth + 1, items, ni);
    }
}
static int cmp_item(const void* a, const void* b) {
    return cmp_i32(&((const hitem*)a)->value, &((const hitem*)b)->value);
}

int orc_huffman_encode(const int32_t* values, int32_t n, orc_huffman* out) {
    memset(out, 0, sizeof(*out));
    out->size = n;
    if (n == 0) return ORC_OK;
    int32_t* sorted = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    memcpy(sorted, values, sizeof(int32_t) * (size_t)n);
    qsort(sorted, (size_t)n, sizeof(int32_t), cmp_i32);
    int32_t nd = 0;
    for (int32_t i = 0; i < n; i++) nd += (i == 0 || sorted[i] != sorted[i - 1]);
    hnode* pool = (hnode*)calloc((size_t)(2 * nd), sizeof(hnode));
    int32_t np = 0;
    for (int32_t i = 0; i < n; i++) {
        if (i == 0 || sorted[i] != sorted[i - 1]) {
            pool[np].value = sorted[i];
            pool[np].occ = 0;
            pool[np].leaf = 1;
            np++;
        }
        pool[np - 1].occ++;
    }
    int32_t* q = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * nd));
    int32_t qs = 0;
    for (int32_t i = 0; i < nd; i++) pq_sift_up(q, qs++, i, pool); /* addAll = add in order */
    while (qs > 1) {
        int32_t x = q[0];
        int32_t last = q[--qs];
        if (qs > 0) pq_sift_down(q, qs, 0, last, pool);
        int32_t y = q[0];
        last = q[--qs];
        if (qs > 0) pq_sift_down(q, qs, 0, last, pool);
        pool[np].value = -1;
        pool[np].occ = pool[x].occ + pool[y].occ;
        pool[np].leaf = 0;
        pool[np].left = x;
        pool[np].right = y;
        pq_sift_up(q, qs++, np, pool);
        np++;
    }
    hitem* items = (hitem*)malloc(sizeof(hitem) * (size_t)nd);
    int32_t ni = 0;
    h_traverse(pool, q[0], 0, 0, items, &ni);
    qsort(items, (size_t)ni, sizeof(hitem), cmp_item); /* mapping is an RB-tree by value */
    out->n_items = ni;
    out->item_value = (int32_t*)malloc(sizeof(int32_t) * (size_t)ni);
    out->item_bits = (int32_t*)malloc(sizeof(int32_t) * (size_t)ni);
    out->item_nbits = (int32_t*)malloc(sizeof(int32_t) * (size_t)ni);
    for (int32_t i = 0; i < ni; i++) {
        out->item_value[i] = items[i].value;
        out->item_bits[i] = items[i].bits;
        out->item_nbits[i] = items[i].nbits;
    }
    bitbuf bb = {0};
    int64_t off = 0;
    for (int32_t i = 0; i < n; i++) {
        hitem key = {values[i], 0, 0};
        hitem* it = (hitem*)bsearch(&key, items, (size_t)ni, sizeof(hitem), cmp_item);
        bb_put(&bb, off, (uint32_t)it->bits, it->nbits);
        off += it->nbits;
    }
    bb_reserve(&bb, 1);
    out->words = bb.w;
    out->n_bits = off;
    out->n_longs = bb_trim(&bb);
    free(items);
    free(q);
    free(pool);
    free(sorted);
    return ORC_OK;
}

int orc_huffman_decode(const orc_huffman* h, int32_t* out) {
    if (h->size == 0) return ORC_OK;
    /* rebuild the code tree from the item table (HuffmanEncoder.java:131-152) */
    int32_t cap = 1;
    for (int32_t i = 0; i < h->n_items; i++) cap += h->item_nbits[i];
    int32_t* lc = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int32_t* rc = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int32_t* val = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int8_t* leaf = (int8_t*)calloc((size_t)cap, 1);
    for (int32_t i = 0; i < cap; i++) lc[i] = rc[i] = -1;
    int32_t nn = 1;
    for (int32_t i = 0; i < h->n_items; i++) {
        int32_t cur = 0, nb = h->item_nbits[i];
        for (int32_t b = nb - 1; b >= 0; b--) {
            int right = (int)(((uint32_t)h->item_bits[i] >> b) & 1u);
            int32_t* slot = right ? &rc[cur] : &lc[cur];
            if (*slot < 0) *slot = nn++;
            cur = *slot;
        }
        val[cur] = h->item_value[i];
        leaf[cur] = 1;
    }
    int32_t cnt = 0, cur = 0;
    int64_t idx = 0;
    while (cnt < h->size) {
        cur = bb_get1(h->words, h->n_longs, idx++) ? rc[cur] : lc[cur];
        if (cur < 0) break;
        if (leaf[cur]) {
            out[cnt++] = val[cur];
            cur = 0;
        }
    }
    free(lc); free(rc); free(val); free(leaf);
    return cnt == h->size ? ORC_OK : ORC_E_ARG;
}

void orc_huffman_free(orc_huffman* h) {
    free(h->item_value); free(h->item_bits); free(h->item_nbits); free(h->words);
    memset(h, 0, sizeof(*h));
}

/* MinMaxSketch.compare (frequency/MinMaxSketch.java:80-86) with Java int wrap */
static int32_t mm_dist(int32_t v, int32_t zero) {
    int32_t d = (int32_t)((uint32_t)v - (uint32_t)zero);
    return d < 0 ? (int32_t)(0u - (uint32_t)d) : d;
}
static int32_t mm_cmp(int32_t a, int32_t b, int32_t zero) {
    return (int32_t)((uint32_t)mm_dist(a, zero) - (uint32_t)mm_dist(b, zero));
}

int orc_sparse_compress(const int32_t* keys, const double* vals, int32_t nnz, int32_t bin_num,
                        int32_t group_num, int32_t row_num, double col_ratio, int64_t seed,
                        int64_t hash_seed, orc_sparse* s, int32_t* bins_out) {
    return orc_sparse_compress_q(keys, vals, nnz, bin_num, group_num, row_num, col_ratio, seed, hash_seed, 0, s,
                                 bins_out);
}

int orc_sparse_compress_q(const int32_t* keys, const double* vals, int32_t nnz, int32_t bin_num,
                          int32_t group_num, int32_t row_num, double col_ratio, int64_t seed,
                          int64_t hash_seed, int32_t quant_type, orc_sparse* s, int32_t* bins_out) {
    memset(s, 0, sizeof(*s));
    if (group_num < 2 || group_num > 64 || row_num < 1 || row_num > 8) return ORC_E_ARG;
    int32_t* bins = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    /* SparseVectorCompressor.java:60-62: Quantizer.newQuantizer(quantType, ...).quantize(values) */
    int st = quant_type == 1 ? orc_uniform_quantize(vals, nnz, bin_num, &s->q, bins)
                             : orc_quantize(vals, nnz, bin_num, seed, &s->q, bins);
    if (st) { free(bins); return st; }
    if (bins_out) memcpy(bins_out, bins, sizeof(int32_t) * (size_t)nnz);
    s->group_num = group_num;
    s->row_num = row_num;
    s->col_ratio = col_ratio;
    if (orc_group_edges(s->q.zero_idx, s->q.bin_num, group_num, s->edges)) {
        free(bins);
        return ORC_E_ARG;
    }
    /* FSketchUtils.partition (FSketchUtils.java:30-47): first group whose edge > bin, stable */
    int32_t* gid = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    for (int32_t i = 0; i < nnz; i++) {
        int32_t g = 0;
        while (s->edges[g] <= bins[i]) g++;
        gid[i] = g;
        s->group_size[g]++;
    }
    int32_t* gk = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    int32_t* gb = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    for (int32_t g = 0; g < group_num && !st; g++) {
        int32_t m = 0;
        for (int32_t i = 0; i < nnz; i++)
            if (gid[i] == g) { gk[m] = keys[i]; gb[m++] = bins[i]; }
        if (m == 0) continue; /* GroupedMinMaxSketch.java:105-109: empty group -> nulls */
        /* GroupedMinMaxSketch.compOneGroup (:103-121) */
        int32_t cols = (int32_t)ceil((double)m * col_ratio);
        s->col_num[g] = cols;
        orc_pick_hashes(hash_seed + g, row_num, s->hash_ids[g]);
        int32_t* t = (int32_t*)malloc(sizeof(int32_t) * (size_t)row_num * (size_t)cols);
        /* sentinel: compare(MIN, MAX) <= 0 ? MIN : MAX (MinMaxSketch.java:30-33) */
        int32_t fill = mm_cmp(INT32_MIN, INT32_MAX, s->q.zero_idx) <= 0 ? INT32_MIN : INT32_MAX;
        for (int64_t i = 0; i < (int64_t)row_num * cols; i++) t[i] = fill;
        for (int32_t j = 0; j < m; j++) /* MinMaxSketch.insert (:48-55) */
            for (int32_t r = 0; r < row_num; r++) {
                int32_t idx = r * cols + orc_hash(s->hash_ids[g][r], gk[j], cols);
                if (mm_cmp(gb[j], t[idx], s->q.zero_idx) < 0) t[idx] = gb[j];
            }
        s->tables[g] = t;
        st = orc_delta_encode(gk, m, &s->deltas[g]);
    }
    free(gk); free(gb); free(gid); free(bins);
    return st;
}

int32_t orc_sparse_restore(const orc_sparse* s, int32_t* keys_out, int32_t* bins_out) {
    int32_t* gkeys[64] = {0};
    int32_t* gbins[64] = {0};
    int32_t glen[64] = {0};
    int32_t total = 0;
    for (int32_t g = 0; g < s->group_num; g++) {
        if (!s->tables[g]) continue;
        int32_t m = s->deltas[g].size;
        gkeys[g] = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
        gbins[g] = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
        orc_delta_decode(&s->deltas[g], gkeys[g]);
        for (int32_t j = 0; j < m; j++) { /* MinMaxSketch.query (:64-73) */
            int32_t res = s->q.zero_idx;
            for (int32_t r = 0; r < s->row_num; r++) {
                int32_t v = s->tables[g][r * s->col_num[g] +
                                         orc_hash(s->hash_ids[g][r], gkeys[g][j], s->col_num[g])];
                if (mm_cmp(v, res, s->q.zero_idx) > 0) res = v;
            }
            gbins[g][j] = res;
        }
        glen[g] = m;
        total += m;
    }
    /* Sort.merge(int[][], int[][], ...) (util/Sort.java:362-379): strict `<` => lower list wins */
    int32_t pos[64] = {0};
    for (int32_t c = 0; c < total; c++) {
        int32_t arg = -1, mn = INT32_MAX;
        for (int32_t g = 0; g < s->group_num; g++)
            if (pos[g] < glen[g] && gkeys[g][pos[g]] < mn) { arg = g; mn = gkeys[g][pos[g]]; }
        if (arg < 0) { /* every head == INT32_MAX: Java would index [-1]; take first live */
            for (int32_t g = 0; g < s->group_num; g++) if (pos[g] < glen[g]) { arg = g; break; }
        }
        keys_out[c] = gkeys[arg][pos[arg]];
        bins_out[c] = gbins[arg][pos[arg]];
        pos[arg]++;
    }
    for (int32_t g = 0; g < 64; g++) { free(gkeys[g]); free(gbins[g]); }
    return total;
}

void orc_sparse_free(orc_sparse* s) {
    for (int32_t g = 0; g < 64; g++) {
        free(s->tables[g]);
        s->tables[g] = NULL;
        if (s->deltas[g].flag_words || s->deltas[g].delta_words) orc_delta_free(&s->deltas[g]);
    }
}

/* ======================================================================================
 * CPU baseline timing: QuantileQuantizer.quantize over fp32 input widened to double, then
 * the 1-byte code write of Quantizer.writeObject (Quantizer.java:193-195).
 * ====================================================================================== */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double orc_bench_dense_encode(const float* x, int32_t n, int32_t bin_num, int64_t seed, int reps,
                              uint8_t* codes_out) {
    double* v = (double*)malloc(sizeof(double) * (size_t)n);
    int32_t* bins = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    orc_quant_header* h = (orc_quant_header*)malloc(sizeof(orc_quant_header));
    double t0 = now_s();
    for (int r = 0; r < reps; r++) {
        for (int32_t i = 0; i < n; i++) v[i] = (double)x[i];
        orc_quantize(v, n, bin_num, seed + r, h, bins);
        for (int32_t i = 0; i < n; i++) codes_out[i] = (uint8_t)(bins[i] - 128);
    }
    double t = now_s() - t0;
    free(v); free(bins); free(h);
    return t;
}
