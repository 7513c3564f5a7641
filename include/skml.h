/*
 * skml.h -- C ABI of the MI355X SketchML gradient codec (libskml.so, sketchml_amd/lib/).
 *
 * This is the drop-in boundary for the reference's `sketch` module hot path.  Every entry point
 * takes plain pointers and sizes (no torch / no C++ types) so the reference's Java host can bind
 * it through JNI.  Each function below names the reference interface it
 * replaces; paths are relative to
 *   /root/reference/sketch/src/main/java/org/dma/sketchml/sketch/
 *
 * Execution model: a context owns one HIP stream on one device.  Encode / decode calls enqueue
 * device work and return without synchronising; errors detected on the device (NaN input, as
 * HeapQuantileSketch.update throws, HeapQuantileSketch.java:75-76) are recorded in the payload
 * header and reported by skml_dense_info() / skml_ctx_sync().
 *
 * RNG model: the reference draws compaction bits from an unseeded JVM-global java.util.Random
 * (QSketchUtils.java:9,47).  Here the stream is java.util.Random(params.seed), consumed in exactly
 * the order the sequential Java sketch would consume it, so results are reproducible and equal
 * to the reference algorithm driven by that stream.
 */
#ifndef SKML_H
#define SKML_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes; the JNI shim maps them to the reference's exceptions ---- */
#define SKML_OK 0
#define SKML_E_ARG 1   /* SketchMLException / QuantileSketchException (argument checks) */
#define SKML_E_NAN 2   /* QuantileSketchException("Encounter NaN value") */
#define SKML_E_ORDER 3 /* SketchMLException("Log for ...") on non-increasing keys */
#define SKML_E_HIP 4
#define SKML_E_RCCL 5
#define SKML_E_OOM 6
#define SKML_E_STATE 7

#define SKML_DENSE_MAGIC 0x444D4B53u /* "SKMD" */
#define SKML_MAX_BINS 65536          /* Quantizer.writeObject's short-code limit */

typedef struct skml_ctx skml_ctx;

/* Codec knobs (ml/conf/MLConf.scala:35-42; Quantizer.java:29; GroupedMinMaxSketch.java:35-36;
 * MinMaxSketch.java:25).  The sketch's k is fixed at 128 (HeapQuantileSketch.java:13). */
typedef struct skml_params {
    int32_t bin_num;   /* requested bins, 2..65536, default 256 */
    int32_t group_num; /* sparse: MinMax groups, default 8 */
    int32_t row_num;   /* sparse: MinMax rows, default 2 */
    int32_t dedup;     /* 1: QuantileQuantizer.quantize (Maths.unique); 0: parallelQuantize */
    double col_ratio;  /* sparse: MinMax columns / group size, default 0.3 */
    int64_t seed;      /* java.util.Random seed of the sketch's compaction stream */
    int64_t hash_seed; /* sparse: group g's hashes are drawn from Random(hash_seed + g) */
    int32_t quant_type; /* sparse: the values' quantizer, SKML_QUANTILE (default) or SKML_UNIFORM
                           (Quantizer.newQuantizer, base/Quantizer.java:126-136); the dense path
                           has separate entry points per quantizer */
    int32_t parallelism; /* sparse path: slice sketches of the values' parallelQuantize when > 1
                            (Constants.Parallel, SparseVectorCompressor.java:90-91); 0 or 1: one.
                            The dense path takes T as an argument
                            (skml_dense_encode_parallel_f32) */
} skml_params;
#define SKML_QUANTILE 0
#define SKML_UNIFORM 1

/* Device payload header (little-endian, 64 bytes) followed by double splits[req_bins-1],
 * padded to 256 bytes, then the packed codes (code_bits per element, LSB-first). */
typedef struct skml_dense_header {
    uint32_t magic;
    int32_t status;    /* SKML_OK or SKML_E_NAN */
    int64_t n;
    int32_t bin_num;   /* effective bins (after Maths.unique), Quantizer.binNum */
    int32_t zero_idx;  /* Quantizer.zeroIdx */
    int32_t code_bits; /* 1, 2, 4, 8 or 16 */
    int32_t req_bins;  /* capacity of the splits array + 1 */
    double min;        /* Quantizer.min (Double.MAX_VALUE-initialised quirk kept) */
    double max;        /* Quantizer.max (Double.MIN_VALUE-initialised quirk kept) */
    int64_t codes_offset;
    int64_t reserved;
} skml_dense_header;

void skml_params_default(skml_params* p);
const char* skml_last_error(void); /* thread-local message of the last failing call */
const char* skml_version(void);

/* Context: one HIP stream on one device.  `hip_stream` is an existing hipStream_t (e.g.
 * torch.cuda.current_stream().cuda_stream; NULL is the device's default stream) or
 * SKML_STREAM_OWN, in which case the library creates and owns a non-blocking stream. */
#define SKML_STREAM_OWN ((void*)(intptr_t)-1)
int skml_ctx_create(int device, void* hip_stream, skml_ctx** out);
int skml_ctx_destroy(skml_ctx* ctx);
int skml_ctx_sync(skml_ctx* ctx);
int skml_ctx_set_stream(skml_ctx* ctx, void* hip_stream);

/* Per-kernel timing with HIP events recorded on the context stream around the launches of the
 * selected kernels (profiling aid for bench.py's roofline; off by default).  `mask`: bit k
 * times kernel id k; SKML_TIMING_ALL times every kernel; 0 turns timing off. */
#define SKML_K_LEAF 0
#define SKML_K_MERGE 1
#define SKML_K_SUMMARY 2
#define SKML_K_QUANTIZE 3
#define SKML_K_DECODE 4
#define SKML_K_DECODE_SUM 5
#define SKML_K_SPARSE 6
#define SKML_K_COUNT 7
#define SKML_TIMING_ALL (-1)
int skml_ctx_set_timing(skml_ctx* ctx, int mask);
/* Synchronises; total device milliseconds and launch count of kernel `kid` since the reset. */
int skml_ctx_kernel_stats(skml_ctx* ctx, int kid, int64_t* launches, double* total_ms);
int skml_ctx_reset_stats(skml_ctx* ctx);
/* Profiling ablation of the sketch leaf kernel (stage 0 load, 1 + leaf sort, 2 + in-wave merges,
 * 3 full): average device ms over `iters` launches on n values.  Not part of the codec. */
int skml_debug_leaf_stage(skml_ctx* ctx, const float* x_dev, int64_t n, int stage, int iters,
                          double* avg_ms);
/* Test hook: while `on` is non-zero, the sparse encode treats its two MinMax staging scratch
 * buffers (the hashed cells and the per-(tile, bucket) reservations) as failed allocations, so
 * the fallback path (key-carrying pairs, rehashing scatter) is exercised.  Not part of the codec. */
int skml_debug_sparse_scratch_fail(int on);

/* Test hook: how the calling thread's last restore / decode merged the groups' runs (Sort.merge):
 * 0 none (fewer than two groups or no keys), 1 the one-pass key-range merge, 2 the pairwise merge
 * rounds (forced by SKML_FORM_RS_ROUNDS), 3 the one-pass merge found the input irregular (a run
 * that does not ascend, a repeated key, a key outside [0, INT32_MAX)) and the rounds ran instead. */
int skml_debug_sparse_merge_path(void);

/* Test hook: force one of the library's alternative kernel forms, process-wide.  Every form gives
 * the same results (the tests run each one against the oracle); 0 is the library's own choice.
 * Returns the previous value, -1 for an unknown id, or -2 (nothing changed) for a form whose
 * kernels only the A/B build carries (built with -DSKML_AB into sketchml_amd/lib_ab/: the forms
 * measured slower than the default, kept for A/B runs).  Not part of the codec. */
#define SKML_FORM_LEAF_SPLIT 0      /* 2: the split leaf always (the default at every size); A/B build: 1 one wave per 64-chunk tile, 3 / 4 / 5 the last 25 / 12.5 / 50 % split */
#define SKML_FORM_DECODE_SUM 1      /* 1: the per-payload kernel (the form for > 8 payloads, mixed widths or wide tables); A/B build: 2 the occupancy form without prefetch */
#define SKML_FORM_PART_BALLOT 2     /* 1: the ballot-ranked partition scatter */
#define SKML_FORM_RS_ROUNDS 3       /* 1: Sort.merge by the pairwise merge rounds always (the fallback for irregular runs); A/B build: 2 the one-pass merge without prefetch */
#define SKML_FORM_DEC_ROWS_SERIAL 4 /* 1: the generic MinMax query (rows one by one; the form for edge tiles and rows != 2) for every tile; A/B build: 2 persistent workgroups */
#define SKML_FORM_AGG_TILES 5       /* 0: Gradient.sum's sum tile in LDS (the default), 1: the 4,096-key wave-per-payload tiles (the form for > 8 groups or > 256 quantValues); A/B build: 2 / 3 staged tiles four / two per round, 4 staged tiles with the next tile prefetched, 5 staged tiles without */
#define SKML_FORM_AGG_ONE_LANE 6    /* 1: Gradient.sum restores every payload on the caller's stream */
#define SKML_FORM_RUN_BOUNDS 7      /* A/B build: 1 the runs' tile / key-range bounds (Gradient.sum, the one-pass Sort.merge) in passes of their own (k_agg_bounds, k_rs_bounds) instead of by the key query */
#define SKML_FORM_DEC_LOOKBACK 8    /* A/B build: 1 the restore's bit lengths and deltas in one pass with decoupled look-backs for the bit offsets and the deltas' prefixes, 2 the same pass with the deltas' tile scan after it */
#define SKML_FORM_COUNT 9
int skml_debug_form(int id, int value);
/* Build flags of the loaded library: SKML_BUILD_AB when it carries the A/B-only forms. */
#define SKML_BUILD_AB 1
int skml_build_flags(void);

/* ---- Dense path: QuantileQuantizer.quantize + Quantizer.getBins/getValues ---- */

/* Bytes of a device payload able to hold n codes for `bin_num` requested bins. */
size_t skml_dense_payload_bytes(int64_t n, int32_t bin_num);

/* QuantileQuantizer.quantize(double[]) (quantization/QuantileQuantizer.java:27-50) on fp32
 * input: k=128 quantile sketch (HeapQuantileSketch.update), getQuantiles(bin_num), Maths.unique,
 * findZeroIdx, then bins[i] = indexOf(x[i]) (Quantizer.java:49-92), packed into the payload.
 * params->dedup = 0 gives parallelQuantize's no-dedup split table (QuantileQuantizer.java:85).
 * x_dev and payload_dev are device pointers.  Asynchronous. */
int skml_dense_encode_f32(skml_ctx* ctx, const float* x_dev, int64_t n, const skml_params* params,
                          void* payload_dev, size_t payload_cap);

/* The same on fp64 input (the reference's own double[] path): the sketch
 * sorts and merges 64-bit keys, indexOf compares in double.  Asynchronous. */
int skml_dense_encode_f64(skml_ctx* ctx, const double* x_dev, int64_t n, const skml_params* params,
                          void* payload_dev, size_t payload_cap);

/* UniformQuantizer.quantize(double[]) (quantization/UniformQuantizer.java:21-45): min / max
 * (Double.MAX_VALUE / Double.MIN_VALUE initialised, NaN values skipped), bin_num-1 splits by
 * repeated `+= (max-min)/bin_num`, findZeroIdx, bins[i] = indexOf(x[i]).  No Maths.unique; NaN
 * values are binned, not rejected.  parallelQuantize is the same computation
 * (UniformQuantizer.java:48-70).  params->seed / dedup are ignored.  Asynchronous. */
int skml_dense_encode_uniform_f32(skml_ctx* ctx, const float* x_dev, int64_t n,
                                  const skml_params* params, void* payload_dev, size_t payload_cap);
int skml_dense_encode_uniform_f64(skml_ctx* ctx, const double* x_dev, int64_t n,
                                  const skml_params* params, void* payload_dev, size_t payload_cap);

/* Several independent buckets (QuantileQuantizer.quantize of each, e.g. the gradient buckets of
 * one DDP step): results identical to skml_dense_encode_f32 per bucket.  The buckets run on two
 * internal streams so that one bucket's sketch (VALU-bound) overlaps the previous bucket's
 * quantize pass (HBM-bound).  xs / ns / payloads / caps: host arrays of nbuckets entries
 * (device pointers).  Ordered after, and waited for by, the context's stream.  Asynchronous. */
int skml_dense_encode_batch_f32(skml_ctx* ctx, int32_t nbuckets, const float* const* xs_dev, const int64_t* ns,
                                const skml_params* params, void* const* payloads_dev, const size_t* payload_caps);

/* QuantileQuantizer.parallelQuantize (QuantileQuantizer.java:53-92) with `threads` slices
 * (Constants.Parallel.getParallelism): slice t = [t*(n/T), ...), the last slice takes the
 * remainder; each slice is sketched, the sketches merged in slice order (HeapQuantileSketch.merge,
 * HeapQuantileSketch.java:186-228), no Maths.unique unless params->dedup (default params: 0).
 * The reference draws every compaction bit from one static Random (QSketchUtils.java:9) in a
 * thread-interleaved order; this is the schedule that runs the slice sketches one after another
 * and then the merges, with Random(params->seed).  threads = 1 equals skml_dense_encode_f32 with
 * dedup = 0.  Asynchronous. */
int skml_dense_encode_parallel_f32(skml_ctx* ctx, const float* x_dev, int64_t n, int32_t threads,
                                   const skml_params* params, void* payload_dev, size_t payload_cap);

/* The same split table over P devices (SURVEY §8e single-split-table mode): shard s holds
 * shard_n[s] consecutive values of one logical gradient.  Each rank sketches its shard into a
 * fixed-size device record (skml_sketch_record_bytes(0)), the records are all-gathered in shard
 * order (skml_allgather), and every rank merges them identically and quantises its own shard.
 * The result equals skml_dense_encode_parallel_f32 over the concatenation when the shards follow
 * its slicing; any shard sizes are accepted (merge order = shard order).  The payload header
 * carries the global splits / min / max / zeroIdx and n = shard_n[shard]. */
size_t skml_sketch_record_bytes(int32_t fp64);
int skml_dense_sketch_shard_f32(skml_ctx* ctx, const float* x_dev, int64_t n, const int64_t* shard_n,
                                int32_t nshards, int32_t shard, int64_t seed, void* record_dev);
int skml_dense_encode_sharded_f32(skml_ctx* ctx, const float* x_dev, int64_t n, const int64_t* shard_n,
                                  int32_t nshards, int32_t shard, const void* records_dev,
                                  const skml_params* params, void* payload_dev, size_t payload_cap);
/* fp64 input (the reference's double[] itself): records of skml_sketch_record_bytes(1) bytes. */
int skml_dense_encode_parallel_f64(skml_ctx* ctx, const double* x_dev, int64_t n, int32_t threads,
                                   const skml_params* params, void* payload_dev, size_t payload_cap);
int skml_dense_sketch_shard_f64(skml_ctx* ctx, const double* x_dev, int64_t n, const int64_t* shard_n,
                                int32_t nshards, int32_t shard, int64_t seed, void* record_dev);
int skml_dense_encode_sharded_f64(skml_ctx* ctx, const double* x_dev, int64_t n, const int64_t* shard_n,
                                  int32_t nshards, int32_t shard, const void* records_dev,
                                  const skml_params* params, void* payload_dev, size_t payload_cap);

/* Split-injected parity mode: quantise against a caller-given split table (host doubles,
 * sorted ascending), min and max, exactly as Quantizer.quantizeToBins would.  Asynchronous. */
int skml_dense_encode_with_splits_f32(skml_ctx* ctx, const float* x_dev, int64_t n,
                                      const double* splits_host, int32_t nsplits, double min,
                                      double max, void* payload_dev, size_t payload_cap);

/* DenseVectorCompressor.decompressDense (sample/DenseVectorCompressor.java:84-91):
 * out[i] = (float) Quantizer.getValues()[bin[i]].  Asynchronous. */
int skml_dense_decode_f32(skml_ctx* ctx, const void* payload_dev, float* out_dev, int64_t n);

/* decompressDense into double[] (the reference's return type): out[i] = getValues()[bin[i]]
 * without the float rounding.  Asynchronous. */
int skml_dense_decode_f64(skml_ctx* ctx, const void* payload_dev, double* out_dev, int64_t n);

/* Fused decode of P payloads into one sum: out[i] = scale * sum_p values_p[bin_p[i]], the
 * decode half of Gradient.sum + timesBy(1/P) (ml/gradient/Gradient.scala:44-49,
 * ml/algorithm/GeneralizedLinearModel.scala:145-150).  payloads_dev points to P payloads laid
 * out `stride` bytes apart.  Asynchronous. */
int skml_dense_decode_sum_f32(skml_ctx* ctx, const void* payloads_dev, int32_t P, size_t stride,
                              float* out_dev, int64_t n, double scale);

/* Quantizer.getBins() (Quantizer.java:168-170): materialise int32 bins on the device. */
int skml_dense_bins_i32(skml_ctx* ctx, const void* payload_dev, int32_t* bins_dev, int64_t n);

/* Synchronise and read the header + splits (Quantizer.getBinNum/getSplits/getZeroIdx/getMin/
 * getMax/getN).  splits_host may be NULL; otherwise it receives bin_num-1 doubles.  Returns the
 * header's status (SKML_E_NAN if the input held a NaN). */
int skml_dense_info(skml_ctx* ctx, const void* payload_dev, skml_dense_header* hdr_host,
                    double* splits_host, int32_t splits_cap);

/* Quantizer.timesBy (Quantizer.java:119-124): scale min, max and splits in place. */
int skml_dense_times_by(skml_ctx* ctx, void* payload_dev, double x);

/* Quantizer.writeObject field stream (Quantizer.java:184-203): big-endian binNum, n,
 * splits[binNum-1], zeroIdx, min, max, bins.length, then bins as (bin-128) bytes / (bin-32768)
 * shorts / ints.  Synchronising.  *written receives the byte count (also when buf is NULL). */
int skml_dense_serialize_ref(skml_ctx* ctx, const void* payload_dev, uint8_t* buf_host,
                             size_t cap, size_t* written);
/* Quantizer.readObject (Quantizer.java:205-226) into a device payload.  Synchronising. */
int skml_dense_deserialize_ref(skml_ctx* ctx, const uint8_t* buf_host, size_t len,
                               void* payload_dev, size_t payload_cap);

/* ---- Host memory in and out (the JNI path: a JVM float[] on its way to a socket) ---- */

/* Pinned host memory (hipHostMalloc): a Java direct ByteBuffer over it (JNI NewDirectByteBuffer)
 * lets the host entry points DMA the gradient without the staging copy. */
int skml_host_alloc(size_t bytes, void** out);
int skml_host_free(void* p);

/* DenseVectorCompressor.compressDense (sample/DenseVectorCompressor.java:34-41) from host memory:
 * x_host (pageable or pinned) -> device -> QuantileQuantizer.quantize (as skml_dense_encode_f32)
 * -> the payload (header, splits, packed codes) back in payload_host.  Pageable input is staged
 * through library-owned pinned buffers, the host copy of one piece overlapping the DMA of the
 * previous one.  payload_host NULL: *written = an upper bound of the payload size.  Otherwise
 * *written = the bytes written (codes_offset + ceil(n * code_bits / 8)).  params->parallelism > 1
 * selects parallelQuantize (QuantileQuantizer.java:53-92) with that many slices, as on the sparse
 * path (params->dedup then applies as given); params->quant_type = SKML_UNIFORM selects
 * UniformQuantizer instead (skml_dense_encode_uniform_f32/_f64).  Synchronising. */
int skml_dense_encode_host_f32(skml_ctx* ctx, const float* x_host, int64_t n, const skml_params* params,
                               void* payload_host, size_t payload_cap, size_t* written);
/* The reference's own double[] input (QuantileQuantizer.quantize(double[]), no fp32 rounding):
 * as skml_dense_encode_host_f32 over skml_dense_encode_f64. */
int skml_dense_encode_host_f64(skml_ctx* ctx, const double* x_host, int64_t n, const skml_params* params,
                               void* payload_host, size_t payload_cap, size_t* written);
/* DenseVectorCompressor.decompressDense (DenseVectorCompressor.java:84-91) from a host payload
 * (as written above) into a host float[n] / double[n].  Synchronising. */
int skml_dense_decode_host_f32(skml_ctx* ctx, const void* payload_host, size_t payload_len, float* out_host,
                               int64_t n);
int skml_dense_decode_host_f64(skml_ctx* ctx, const void* payload_host, size_t payload_len, double* out_host,
                               int64_t n);
/* Host payloads without a device (pure host code):
 *   skml_dense_info_host     Quantizer.getBinNum/getSplits/getZeroIdx/getMin/getMax/getN
 *   skml_dense_bins_host     Quantizer.getBins() (Quantizer.java:163-165): unpacked int32 bins
 *   skml_dense_times_by_host Quantizer.timesBy (Quantizer.java:119-124), in place */
int skml_dense_info_host(const void* payload_host, size_t payload_len, skml_dense_header* hdr, double* splits_host,
                         int32_t splits_cap);
int skml_dense_bins_host(const void* payload_host, size_t payload_len, int32_t* bins_host, int64_t n);
int skml_dense_times_by_host(void* payload_host, size_t payload_len, double x);

/* ---- Sparse path: SketchGradient.fromSparse / SparseVectorCompressor ---- */

typedef struct skml_sparse skml_sparse; /* library-owned; free with skml_sparse_free */

/* DenseDoubleGradient.countNNZ + toSparse (ml/gradient/DenseDoubleGradient.scala:64-89):
 * keep |x| > 1e-8 with ascending int32 keys.  keys_dev / vals_dev need dim capacity.
 * Synchronising (returns nnz through *nnz_out). */
int skml_sparse_compact_f32(skml_ctx* ctx, const float* dense_dev, int64_t dim, int32_t* keys_dev,
                            float* vals_dev, int64_t* nnz_out);
/* The same over the reference's own double[] (DenseDoubleGradient.values): |x| > 1e-8 in double. */
int skml_sparse_compact_f64(skml_ctx* ctx, const double* dense_dev, int64_t dim, int32_t* keys_dev,
                            double* vals_dev, int64_t* nnz_out);

/* SparseVectorCompressor.compressSparse (sample/SparseVectorCompressor.java:52-67):
 * QuantileQuantizer.quantize(values) then GroupedMinMaxSketch.create(keys, bins)
 * (frequency/GroupedMinMaxSketch.java:51-70): group partition, MinMax insert, DeltaAdaptive key
 * encoding (binary/DeltaAdaptiveEncoder.java:54-112).  Synchronising. */
int skml_sparse_encode_kv_f32(skml_ctx* ctx, const int32_t* keys_dev, const float* vals_dev,
                              int64_t nnz, const skml_params* params, skml_sparse** out);
/* SparseVectorCompressor.compressSparse(int[], double[]) / SketchGradient.fromSparse on the
 * reference's own double values (SketchGradient.scala:35-48, SparseVectorCompressor.java:52-67):
 * the values' quantizer sketches and bins the doubles themselves (skml_dense_encode_f64, or the
 * uniform / parallel f64 forms), so split samples and bins equal the Java double[] path even for
 * values that are not fp32-representable.  Synchronising. */
int skml_sparse_encode_kv_f64(skml_ctx* ctx, const int32_t* keys_dev, const double* vals_dev,
                              int64_t nnz, const skml_params* params, skml_sparse** out);
/* SketchGradient.fromSparse after toAuto's compaction: compact + encode_kv. */
int skml_sparse_encode_f32(skml_ctx* ctx, const float* dense_dev, int64_t dim,
                           const skml_params* params, skml_sparse** out);
/* The ml path itself: DenseDoubleGradient.toAuto / toSparse (DenseDoubleGradient.scala:64-95) of a
 * double[] gradient, then SketchGradient.fromSparse on the double values. */
int skml_sparse_encode_f64(skml_ctx* ctx, const double* dense_dev, int64_t dim,
                           const skml_params* params, skml_sparse** out);
/* GroupedMinMaxSketch.restore + Sort.merge (GroupedMinMaxSketch.java:123-146,
 * util/Sort.java:362-379) and SparseVectorCompressor.decompressSparse's value lookup
 * (SparseVectorCompressor.java:118-126).  keys/vals device buffers of nnz capacity.  A restored
 * bin outside quantValues returns SKML_E_ARG (Java: ArrayIndexOutOfBoundsException). */
int skml_sparse_decode_f32(skml_ctx* ctx, const skml_sparse* s, int32_t* keys_dev,
                           float* vals_dev);
/* The same with the values as the reference's doubles (quantValues[bin], no fp32 rounding). */
int skml_sparse_decode_f64(skml_ctx* ctx, const skml_sparse* s, int32_t* keys_dev,
                           double* vals_dev);
int skml_sparse_nnz(const skml_sparse* s, int64_t* nnz);
/* SparseVectorCompressor.timesBy (sample/SparseVectorCompressor.java:128-134): scales the
 * double quantValues table in place (the scaled values are what decode returns, as fp32). */
int skml_sparse_times_by(skml_sparse* s, double x);
/* quantValues (Quantizer.getValues times every timesBy factor): min(bin_num, cap) doubles. */
int skml_sparse_values(const skml_sparse* s, double* out, int32_t cap);
/* Header of the quantizer inside the sparse payload (bins, zero index, splits). */
int skml_sparse_quant_info(const skml_sparse* s, skml_dense_header* hdr, double* splits_host,
                           int32_t splits_cap);
/* Per-group view for parity checks: size, colNum, hash ids, DeltaAdaptive choice and bit
 * lengths; tables/words are copied to host buffers when non-NULL. */
typedef struct skml_sparse_group {
    int32_t size;
    int32_t col_num;
    int32_t hash_ids[8];
    int32_t num_intervals;
    int32_t flag_kind;
    int64_t n_flag_bits;
    int64_t n_delta_bits;
} skml_sparse_group;
int skml_sparse_group_info(skml_ctx* ctx, const skml_sparse* s, int32_t g, skml_sparse_group* info,
                           int32_t* table_host, uint64_t* flag_words_host,
                           uint64_t* delta_words_host);
/* GroupedMinMaxSketch.writeObject-ordered field stream (GroupedMinMaxSketch.java:148-158),
 * without Java object-stream framing; see DESIGN.md for the exact layout. */
int skml_sparse_serialize(skml_ctx* ctx, const skml_sparse* s, uint8_t* buf_host, size_t cap,
                          size_t* written);
/* GroupedMinMaxSketch.readObject (GroupedMinMaxSketch.java:161-172) with its MinMaxSketch,
 * HuffmanEncoder and DeltaAdaptiveEncoder readObjects: parses the stream skml_sparse_serialize
 * writes and rebuilds a device payload (the Huffman tables are decoded on the device).
 * quant_values (SparseVectorCompressor.quantValues, may be NULL with nvalues 0) enable
 * skml_sparse_decode_f32; without them only skml_sparse_restore_bins applies.  Synchronising. */
int skml_sparse_deserialize(skml_ctx* ctx, const uint8_t* buf_host, size_t len, const double* quant_values,
                            int32_t nvalues, skml_sparse** out);
/* GroupedMinMaxSketch.restore (GroupedMinMaxSketch.java:123-146): keys in Sort.merge order and
 * their int32 bins, on the device.  Synchronising. */
int skml_sparse_restore_bins(skml_ctx* ctx, const skml_sparse* s, int32_t* keys_dev, int32_t* bins_dev);
int skml_sparse_free(skml_sparse* s);

/* ---- Sparse payloads between GPUs (the ml path's exchange) ----
 * A payload exported as one contiguous, relocatable device blob: a 256-byte header (magic "SKSP",
 * section offsets), the group table, the quantizer header + splits, quantValues (doubles, timesBy
 * applied), the MinMaxSketch tables and the two DeltaAdaptive word streams.  It is what the RCCL
 * all-gather moves (sizes first, then the blobs padded to the largest: skml_allgather), with no
 * host round trip.  The blob replaces the Java-serialised SketchGradient that Spark's collect /
 * broadcast ship (ml/algorithm/GeneralizedLinearModel.scala:145-156). */
int skml_sparse_export_bytes(const skml_sparse* s, size_t* bytes);
/* dst_dev: 256-byte aligned device memory of at least export_bytes.  Asynchronous. */
int skml_sparse_export(skml_ctx* ctx, const skml_sparse* s, void* dst_dev, size_t cap);
/* A library-owned copy of the blob at blob_dev (len bytes available there); the blob is checked
 * (magic, section offsets, group-table invariants) before anything runs on it.  Synchronising. */
int skml_sparse_import(skml_ctx* ctx, const void* blob_dev, size_t len, skml_sparse** out);
/* Gradient.sum (ml/gradient/Gradient.scala:44-49) of P blobs laid out `stride` bytes apart (the
 * all-gather output): out[0, dim) = +0.0, then payload by payload, in order,
 * DenseDoubleGradient.plusBy(SketchGradient.toAuto) (DenseDoubleGradient.scala:38) -- every restored
 * key adds quantValues[bin] in double (the live values only, plus the dense form's +0.0, when the
 * payload's live count exceeds dim * 2 / 3: SparseDoubleGradient.toAuto); then out *= scale when
 * scale != 1 (the 1/P average, one double multiply per element).  A key outside [0, dim) fails
 * with SKML_E_ARG (SparseDoubleGradient's bound check), and so do a key repeated across one
 * payload's groups (its constructor requires strictly increasing keys) and a payload that restores
 * no keys (its constructor reads indices.head).  Synchronising. */
int skml_sparse_decode_sum_f64(skml_ctx* ctx, const void* blobs_dev, int32_t P, size_t stride, int64_t dim,
                               double scale, double* out_dev);
/* Host-memory forms of encode_kv / decode (int[] keys and float[] values in JVM arrays). */
int skml_sparse_encode_kv_host_f32(skml_ctx* ctx, const int32_t* keys_host, const float* vals_host, int64_t nnz,
                                   const skml_params* params, skml_sparse** out);
/* int[] keys and double[] values (SparseVectorCompressor.compressSparse(int[], double[])). */
int skml_sparse_encode_kv_host_f64(skml_ctx* ctx, const int32_t* keys_host, const double* vals_host, int64_t nnz,
                                   const skml_params* params, skml_sparse** out);
int skml_sparse_decode_host_f32(skml_ctx* ctx, const skml_sparse* s, int32_t* keys_host, float* vals_host);
/* keys into an int[] and quantValues[bin] into a double[] (SparseVectorCompressor.decompressSparse). */
int skml_sparse_decode_host_f64(skml_ctx* ctx, const skml_sparse* s, int32_t* keys_host, double* vals_host);

/* ---- DeltaAdaptiveEncoder as a standalone BinaryEncoder (base/BinaryEncoder.java:6-11) ---- */
/* encode(int[]): keys strictly increasing (keys[0] >= 0).  Outputs the choice and the two
 * BitSet word streams (BitSet.toLongArray layout).  Synchronising. */
int skml_delta_encode(skml_ctx* ctx, const int32_t* keys_dev, int64_t n, int32_t* num_intervals,
                      int32_t* flag_kind, int64_t* n_flag_bits, int64_t* n_delta_bits,
                      uint64_t* flag_words_dev, uint64_t* delta_words_dev, int64_t words_cap);
/* decode(): keys_dev receives n keys.  Asynchronous. */
int skml_delta_decode(skml_ctx* ctx, int64_t n, int32_t num_intervals, int32_t flag_kind,
                      const uint64_t* flag_words_dev, int64_t n_flag_words,
                      const uint64_t* delta_words_dev, int64_t n_delta_words, int32_t* keys_dev);

/* Host-memory forms (a JVM int[] in, BitSet.toLongArray long[]s out, and back): words_cap is the
 * capacity of each word array; NULL word arrays query the bit counts only. */
int skml_delta_encode_host(skml_ctx* ctx, const int32_t* keys_host, int64_t n, int32_t* num_intervals,
                           int32_t* flag_kind, int64_t* n_flag_bits, int64_t* n_delta_bits, uint64_t* flag_words_host,
                           uint64_t* delta_words_host, int64_t words_cap);
int skml_delta_decode_host(skml_ctx* ctx, int64_t n, int32_t num_intervals, int32_t flag_kind,
                           const uint64_t* flag_words_host, int64_t n_flag_words, const uint64_t* delta_words_host,
                           int64_t n_delta_words, int32_t* keys_host);

/* ---- Multi-GPU: RCCL all-gather of payloads over xGMI ---- */
typedef struct skml_comm skml_comm;
#define SKML_UNIQUE_ID_BYTES 128
int skml_comm_unique_id(uint8_t id_out[SKML_UNIQUE_ID_BYTES]);
int skml_comm_init_rank(skml_ctx* ctx, const uint8_t id[SKML_UNIQUE_ID_BYTES], int32_t nranks,
                        int32_t rank, skml_comm** out);
int skml_comm_destroy(skml_comm* comm);
/* ncclAllGather of `bytes` from each rank's payload into all_dev (nranks * bytes). Async. */
int skml_allgather(skml_ctx* ctx, skml_comm* comm, const void* payload_dev, size_t bytes,
                   void* all_dev);

#ifdef __cplusplus
}
#endif
#endif /* SKML_H */
