/*
 * skml_oracle.h -- CPU restatement of the reference SketchML codec (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity CHECKER for the HIP product path in sketchml_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product library
 * (libskml.so) never links or calls it.
 *
 * Parity status: the reference (Java 8 + Scala/Spark) cannot be compiled or run in this container
 * (no JDK / javac / mvn) and ships no tests or golden vectors (§4).  This
 * restatement is therefore pinned only by known-answer tests derived by hand from the Java sources
 * and the public JDK specifications (java.util.Random LCG, Arrays.sort total order, BitSet word
 * layout, DataOutput big-endian) -- see tests/test_oracle.py (K1-K8) -- and cross-checked against an
 * independent numpy restatement (oracle/np_oracle.py).  No output of the reference itself pins it:
 * "parity unpinned" against a live reference run.
 *
 * All file:line citations are relative to
 *   /root/reference/sketch/src/main/java/org/dma/sketchml/sketch/
 * unless prefixed with ml/ (= /root/reference/ml/src/main/scala/org/dma/sketchml/ml/).
 *
 * RNG model (the reference draws from unseeded JVM-global Randoms, QSketchUtils.java:9,
 * HashFactory.java:15, Maths.java:42): every entry point here takes an explicit seed and draws
 * from java.util.Random(seed) exactly as the Java code would draw from its static Random.
 */
#ifndef SKML_ORACLE_H
#define SKML_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (mirror include/skml.h) */
#define ORC_OK 0
#define ORC_E_ARG 1
#define ORC_E_NAN 2
#define ORC_E_ORDER 3
#define ORC_E_OOM 6

/* ---- java.util.Random (JDK 8 spec) ---- */
typedef struct {
    uint64_t s;
    int have_gauss;
    double gauss;
} orc_jrandom;

void orc_jr_seed(orc_jrandom* r, int64_t seed);
int32_t orc_jr_next(orc_jrandom* r, int bits);
int32_t orc_jr_next_int(orc_jrandom* r);
int32_t orc_jr_next_int_bound(orc_jrandom* r, int32_t bound);
int orc_jr_next_boolean(orc_jrandom* r);
double orc_jr_next_double(orc_jrandom* r);
double orc_jr_next_gaussian(orc_jrandom* r);
/* the value next(1) would return as the idx-th call (0-based) on Random(seed) */
int orc_jr_bit_at(int64_t seed, int64_t idx);

/* ---- Dense quantile quantizer (QuantileQuantizer + Quantizer) ---- */
typedef struct {
    int32_t bin_num;      /* effective after Maths.unique */
    int32_t n;
    int32_t zero_idx;
    double min, max;
    double splits[65536]; /* bin_num - 1 used */
} orc_quant_header;

/* QuantileQuantizer.quantize (QuantileQuantizer.java:27-50).  bins may be NULL. */
int orc_quantize(const double* values, int32_t n, int32_t bin_num, int64_t seed,
                 orc_quant_header* hdr, int32_t* bins);
/* QuantileQuantizer.parallelQuantize (QuantileQuantizer.java:53-92) with T slices, in the
 * schedule where the slice sketches run one after another and then merge in slice order, all
 * drawing from the one Random(seed) (the reference's static Random, QSketchUtils.java:9). */
int orc_parallel_quantize(const double* values, int32_t n, int32_t bin_num, int32_t threads,
                          int64_t seed, orc_quant_header* hdr, int32_t* bins);
/* UniformQuantizer.quantize (quantization/UniformQuantizer.java:21-45): min / max by IEEE `<` / `>`
 * from Double.MAX_VALUE / Double.MIN_VALUE (NaN values skipped, the first zero wins the min),
 * splits by repeated `+= step` in double, no Maths.unique.  NaN values are accepted and binned
 * by indexOf.  bins may be NULL. */
int orc_uniform_quantize(const double* values, int32_t n, int32_t bin_num, orc_quant_header* hdr,
                         int32_t* bins);
/* The same on float values (each widened to double, exactly as a float[] copied into the
 * reference's double[] would be): the header only, for the full-size parity tests, whose bins
 * come from orc_index_of_many_f32 in slices.  No bins argument. */
int orc_quantize_header_f32(const float* values, int64_t n, int32_t bin_num, int64_t seed, orc_quant_header* hdr);
/* Quantizer.indexOf (Quantizer.java:49-72) */
int32_t orc_index_of(const orc_quant_header* h, double x);
/* Quantizer.quantizeToBins (Quantizer.java:94-101) over a slice of float values: bins[i] =
 * indexOf((double) x[i]).  Elementwise, so callers may run slices on several threads. */
void orc_index_of_many_f32(const orc_quant_header* h, const float* x, int64_t n, int32_t* bins);
/* Quantizer.getValues (Quantizer.java:39-47) */
void orc_get_values(const orc_quant_header* h, double* out);
/* Quantizer.timesBy (Quantizer.java:119-124) */
void orc_times_by(orc_quant_header* h, double x);
/* Quantizer.writeObject field stream (Quantizer.java:184-203), big-endian DataOutput. */
int64_t orc_write_ref(const orc_quant_header* h, const int32_t* bins, uint8_t* buf, int64_t cap);
int orc_read_ref(const uint8_t* buf, int64_t len, orc_quant_header* h, int32_t* bins, int32_t bins_cap);

/* ---- Raw sketch access (HeapQuantileSketch) for tests ---- */
/* Build a sketch over values with Random(seed) and return its summary: samples / weights
 * (exclusive prefix, numSamples+1 entries), min, max.  Returns numSamples or <0 on error. */
int64_t orc_sketch_summary(const double* values, int64_t n, int64_t seed, double* samples,
                           int64_t* weights, int64_t cap, double* min_out, double* max_out);
/* HeapQuantileSketch.getQuantiles(int) on a freshly built sketch. */
int orc_sketch_quantiles(const double* values, int64_t n, int64_t seed, int32_t parts,
                         double* splits);

/* ---- Sparse path ---- */
/* DenseDoubleGradient.countNNZ / toSparse (ml/gradient/DenseDoubleGradient.scala:64-89) */
int64_t orc_count_nnz(const double* dense, int64_t dim);
int64_t orc_to_sparse(const double* dense, int64_t dim, int32_t* keys, double* vals);

/* the 8 Int2IntHash functions, ids in HashFactory.java:12-14 list order:
 * 0 BJ, 1 Mix64, 2 TW, 3 BKDR(31), 4 BKDR(131), 5 BKDR(267), 6 BKDR(1313), 7 BKDR(13131) */
int32_t orc_hash(int32_t id, int32_t key, int32_t size);
/* HashFactory.getRandomInt2IntHashes's Maths.shuffle draw, on Random(seed) */
void orc_pick_hashes(int64_t seed, int32_t rows, int32_t* ids);

/* FSketchUtils.calGroupEdges; ORC_E_ARG where Java divides by zero (bin_num < group_num) */
int orc_group_edges(int32_t zero_idx, int32_t bin_num, int32_t group_num, int32_t* edges);

/* DeltaAdaptiveEncoder (binary/DeltaAdaptiveEncoder.java) */
typedef struct {
    int32_t size;
    int32_t num_intervals;
    int32_t flag_kind;
    int64_t n_flag_bits, n_delta_bits;  /* logical bit lengths written */
    int32_t n_flag_longs, n_delta_longs; /* BitSet.toLongArray lengths (trailing zeros trimmed) */
    uint64_t* flag_words;
    uint64_t* delta_words;
} orc_delta;
int orc_delta_encode(const int32_t* keys, int32_t n, orc_delta* out); /* allocates words */
int orc_delta_decode(const orc_delta* d, int32_t* keys_out);
void orc_delta_free(orc_delta* d);

/* HuffmanEncoder (binary/HuffmanEncoder.java) over an int table */
typedef struct {
    int32_t n_items;
    int32_t* item_value;
    int32_t* item_bits;
    int32_t* item_nbits;
    int64_t n_bits;
    int32_t n_longs;
    uint64_t* words;
    int32_t size;
} orc_huffman;
int orc_huffman_encode(const int32_t* values, int32_t n, orc_huffman* out);
int orc_huffman_decode(const orc_huffman* h, int32_t* out);
void orc_huffman_free(orc_huffman* h);

/* GroupedMinMaxSketch + quantizer: SparseVectorCompressor.compressSparse
 * (sample/SparseVectorCompressor.java:52-67).  Group g's hash permutation is drawn from
 * Random(hash_seed + g). */
typedef struct {
    orc_quant_header q;
    int32_t group_num, row_num;
    double col_ratio;
    int32_t edges[64];
    int32_t group_size[64];
    int32_t col_num[64];
    int32_t hash_ids[64][8];
    int32_t* tables[64];     /* row_num * col_num ints, or NULL for empty groups */
    orc_delta deltas[64];
} orc_sparse;
int orc_sparse_compress(const int32_t* keys, const double* vals, int32_t nnz, int32_t bin_num,
                        int32_t group_num, int32_t row_num, double col_ratio, int64_t seed,
                        int64_t hash_seed, orc_sparse* out, int32_t* bins_out /*nullable*/);
/* The same with the values' quantizer chosen by quant_type (0 QUANTILE, 1 UNIFORM;
 * SparseVectorCompressor.java:60-62 Quantizer.newQuantizer). */
int orc_sparse_compress_q(const int32_t* keys, const double* vals, int32_t nnz, int32_t bin_num,
                          int32_t group_num, int32_t row_num, double col_ratio, int64_t seed,
                          int64_t hash_seed, int32_t quant_type, orc_sparse* s, int32_t* bins_out);
/* GroupedMinMaxSketch.restore + Sort.merge; returns nnz */
int32_t orc_sparse_restore(const orc_sparse* s, int32_t* keys_out, int32_t* bins_out);
void orc_sparse_free(orc_sparse* s);

/* Timing helper for bench.py's cpu_baseline: quantize + 1-byte code write, returns seconds. */
double orc_bench_dense_encode(const float* x, int32_t n, int32_t bin_num, int64_t seed, int reps,
                              uint8_t* codes_out);

#ifdef __cplusplus
}
#endif
#endif
