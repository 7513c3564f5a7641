// skml_internal.h -- constants and launch interfaces shared by skml_api.cpp and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/skml.h"

namespace skml {

// The kernel form selected by skml_debug_form (SKML_FORM_*): 0 = the library's own choice.
int form(int id);

constexpr uint64_t kLcgMult = 0x5DEECE66DULL;  // java.util.Random
constexpr uint64_t kLcgAdd = 0xBULL;
constexpr uint64_t kLcgMask = (1ULL << 48) - 1;

constexpr int kK = 128;                 // HeapQuantileSketch.DEFAULT_K (HeapQuantileSketch.java:13)
constexpr int kChunk = 2 * kK;          // base buffer size: 256 values per leaf
constexpr int kLeafWaves = 8;           // waves per leaf workgroup
constexpr int kChunksPerWave = 8;       // 32 keys per lane, 8 lanes per chunk
constexpr int kLeafChunks = kLeafWaves * kChunksPerWave;  // 64 chunks -> one level-6 node
constexpr int kLeafTopLevel = 6;
constexpr int kMergeGroupLog = 6;       // upper merge: 64 nodes per workgroup
constexpr int kMaxLevels = 24;     // n < 2^31 -> fewer than 2^23 chunks
constexpr int kHeaderBytes = 64;
// Quantize bucket LUT: the top kLutBits of a value's total-order key select a bucket whose entry
// is the number of splits below the bucket; at most `cmax` splits fall inside any bucket.
constexpr int kLutBits = 14;
constexpr int kLutSize = 1 << kLutBits;
constexpr int kLutMaxNeed = 15;    // <= 4 bisection steps after the lookup; else Eytzinger
constexpr int kLutMaxSplits = 4096;  // split table must fit the quantize kernel's LDS
constexpr int kLutPad = 16;          // NaN padding after the last split (2^4 bisection reach)
struct QuantLut {
    uint16_t base[kLutSize];
    int32_t cmax;  // -1: LUT unusable (too many splits per bucket); kLutJavaMode: see below
    int32_t pad[15];
};
// cmax value asking the quantize pass for Quantizer.indexOf literally (a degenerate uniform split
// table: NaN or descending splits, on which indexOf is not an upper bound).
constexpr int32_t kLutJavaMode = -2;

// fp64 leaf partials (one per 64-chunk tile): min / max total-order key, flags (bit0 NaN).
struct LeafPartial64 {
    uint64_t min_key;
    uint64_t max_key;
    uint32_t flags;
    uint32_t pad;
};
// Uniform quantizer partials (one per workgroup): IEEE min / max of the non-NaN values and the
// index of the first zero.
struct UniPartial {
    double mn, mx;
    int64_t zidx;
    int64_t pad;
};
constexpr int kUniMaxParts = 1024;

// Per leaf workgroup partial results: min key, max key, flags (bit0 NaN, bit1 -0, bit2 +0).
struct LeafPartial {
    uint32_t min_key;
    uint32_t max_key;
    uint32_t flags;
    uint32_t pad;
};

// One HeapQuantileSketch's state (a parallelQuantize slice sketch, QuantileQuantizer.java:63-75),
// fixed size so that P of them all-gather as one buffer.  Levels are the bits of n / 256.
struct SketchRecord {
    int64_t n;
    LeafPartial mm;               // min / max total-order keys, flags (bit0 NaN)
    int64_t pad;
    float tail[kChunk];           // base buffer in insertion order (n % 256 used)
    float level[kMaxLevels][kK];  // level l: 128 samples, IEEE-sorted
};

// fp64 counterpart of SketchRecord.
struct SketchRecord64 {
    int64_t n;
    LeafPartial64 mm;
    double tail[kChunk];
    double level[kMaxLevels][kK];
};
// fp64 leaf in the fp32 leaf's layout (8 lanes x 32 values per chunk), skml_sketch.hip
hipError_t launch_leaf2_f64(hipStream_t st, const double* x, int64_t chunks, uint64_t s0, const uint64_t* jump_tab,
                            LeafPartial64* part, double* nodes6, double* roots, uint8_t* ubits);
hipError_t launch_sketch_record64(hipStream_t st, const double* x, int64_t n, const LeafPartial64* part,
                                  int64_t nparts, const double* roots, SketchRecord64* rec);
// Merge of fp64 records into (roots, tail, part) for launch_summary64 (tail, sharded = 1).
hipError_t launch_sketch_merge64(hipStream_t st, const SketchRecord64* recs, int nrec, uint64_t s0, uint64_t bit0,
                                 const uint64_t* jump_tab, double* roots, double* tail, LeafPartial64* part);

struct MergeJob {
    int64_t src_node;      // first input node index (in src buffer)
    int64_t dst_node;      // first output node index (in dst buffer), or -1 -> root slot
    int64_t chunk_base;    // first chunk covered by the job's first input node
    int32_t level_in;      // level of the input nodes
    int32_t group_log;     // each workgroup merges 2^group_log consecutive nodes
    int32_t groups;        // number of workgroups for this job
    int32_t root_level;    // >= 0: the single output is the tree root of this level
};
constexpr int kMaxJobs = 24;
struct MergePass {
    MergeJob job[kMaxJobs];
    int32_t njobs;
    int32_t fuse_summary;  // last pass: its last workgroup also runs the summary
    int32_t wg_prefix[kMaxJobs + 1];
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
// Packed code width: smallest of 1, 2, 4, 8, 16 bits holding bin_num codes.
__host__ __device__ inline int code_bits_for(int bins) {
    int b = 1;
    while ((1LL << b) < bins) b <<= 1;
    return b;
}
__host__ __device__ inline size_t dense_codes_offset(int req_bins) {
    return align_up(kHeaderBytes + 8 * (size_t)(req_bins - 1), 256);
}

// Upper merge nodes (tree levels >= kLeafTopLevel + 1) of the fixed merge tree over C chunks,
// numbered level by level: node i of level L covers chunks [i 2^L, (i+1) 2^L), and its number is
// upper_level_offset(C, L) + i.  The leaf kernel draws their compaction bits (one per wave) into
// a byte array so the merge passes look them up instead of jumping the LCG themselves.
__host__ __device__ inline int64_t upper_level_offset(int64_t C, int L) {
    int64_t o = 0;
    for (int l = kLeafTopLevel + 1; l < L; l++) o += C >> l;
    return o;
}
__host__ __device__ inline int64_t upper_node_count(int64_t C) { return upper_level_offset(C, kMaxLevels); }

// ---- kernel launchers (skml_sketch.hip) ----
// ubits: upper_node_count(full tiles * 64) bytes; the leaf draws the upper merge tree's bits into it
hipError_t launch_leaf(hipStream_t st, const float* x, int64_t chunks, uint64_t s0,
                       const uint64_t* jump_tab, LeafPartial* part, float* nodes6, float* roots, uint8_t* ubits);
hipError_t launch_leaf_stage(hipStream_t st, int stage, const float* x, int64_t chunks, uint64_t s0,
                             const uint64_t* jump_tab, LeafPartial* part, float* scratch, float* roots);
// fp64 merge pass over double nodes (no summary; `next` as in launch_merge_pass).
hipError_t launch_merge_pass64(hipStream_t st, const MergePass& pass, const MergePass* next, const double* src,
                               double* dst, double* next_dst, double* roots, uint64_t s0, const uint64_t* jump_tab,
                               unsigned* done, const uint8_t* ubits, int64_t uchunks);
// Slice sketch -> record (after the leaf and the merge passes without a summary).
hipError_t launch_sketch_record(hipStream_t st, const float* x, int64_t n, const LeafPartial* part, int64_t nparts,
                                const float* roots, SketchRecord* rec);
// HeapQuantileSketch.merge of recs[0..nrec) in order (compaction bits from stream index bit0
// on), then the summary of the merged sketch (n_total values) into payload's header, splits and
// the quantize LUT; the header's n is n_local.  scratch: kMaxLevels*kK + kChunk floats and nrec
// LeafPartials (device).
hipError_t launch_sketch_merge(hipStream_t st, const SketchRecord* recs, int nrec, uint64_t s0, uint64_t bit0,
                               const uint64_t* jump_tab, int64_t n_total, int64_t n_local, const int64_t* ranks,
                               int req_bins, int dedup, void* payload, double* scratch_raw, QuantLut* lut,
                               float* scratch_roots, float* scratch_tail, LeafPartial* scratch_part);
// `next` (may be null): a one-workgroup pass run by this pass's last workgroup (its src is `dst`,
// its output `next_dst`), saving a launch.
hipError_t launch_merge_pass(hipStream_t st, const MergePass& pass, const MergePass* next, const float* src,
                             float* dst, float* next_dst, float* roots, uint64_t s0, const uint64_t* jump_tab,
                             unsigned* done, const float* x, int64_t n, const LeafPartial* part, int64_t nparts,
                             const int64_t* ranks, int req_bins, int dedup, void* payload,
                             double* scratch_raw, QuantLut* lut, const uint8_t* ubits, LeafPartial* part_red,
                             int64_t nred, int64_t part_from);
hipError_t launch_summary(hipStream_t st, const float* x, int64_t n, const LeafPartial* part,
                          int64_t nparts, const float* roots, const int64_t* ranks, int req_bins,
                          int dedup, void* payload, double* scratch_raw, QuantLut* lut);
// getQuantiles' rank table for (n, bins) written on the device (bins - 1 int64)
hipError_t launch_set_ranks(hipStream_t st, int64_t n, int bins, int64_t* ranks);
hipError_t launch_set_splits(hipStream_t st, void* payload, int64_t n, const double* splits_dev,
                             int nsplits, double mn, double mx, int req_bins, QuantLut* lut);
// ---- kernel launchers (skml_dense.hip) ----
// `lut` may be null (Eytzinger / global search); req_bins sizes the kernel's LDS split table.
hipError_t launch_quantize(hipStream_t st, const float* x, int64_t n, void* payload, const QuantLut* lut,
                           int req_bins);
hipError_t launch_decode(hipStream_t st, const void* payload, float* out, int64_t n);
hipError_t launch_decode_sum(hipStream_t st, const void* payloads, int P, size_t stride, float* out,
                             int64_t n, double scale, int common_bits,
                             int max_bins);  // common_bits 0: mixed widths
hipError_t launch_bins(hipStream_t st, const void* payload, int32_t* bins, int64_t n);
hipError_t launch_ref_body(hipStream_t st, const void* payload, uint8_t* out, int64_t n, int width);
hipError_t launch_times_by(hipStream_t st, void* payload, double x);
// ---- kernel launchers (skml_f64.hip) ----
hipError_t launch_summary64(hipStream_t st, const double* x, int64_t n, const LeafPartial64* part, int64_t nparts,
                            const double* roots, const int64_t* ranks, int req_bins, int dedup, void* payload,
                            double* g_raw, QuantLut* lut,
                            const double* tail = nullptr, int sharded = 0, int64_t n_local = 0);
// `lut` may be null; fp64 values are looked up by their round-down fp32 image, then corrected
// by exact double compares.
hipError_t launch_quantize64(hipStream_t st, const double* x, int64_t n, void* payload, const QuantLut* lut,
                             const int* qflags, int req_bins);
hipError_t launch_decode64(hipStream_t st, const void* payload, double* out, int64_t n);
int uniform_partials(int64_t n);
hipError_t launch_uniform(hipStream_t st, const float* x, int64_t n, int bin_num, UniPartial* part, void* payload,
                          QuantLut* lut, int* qflags);
hipError_t launch_uniform64(hipStream_t st, const double* x, int64_t n, int bin_num, UniPartial* part,
                            void* payload, QuantLut* lut, int* qflags);
// *bad (device int, zeroed by the caller) counts waves that met a bin outside [0, binNum)
hipError_t launch_pack_ref(hipStream_t st, const uint8_t* body, int width, int64_t n, void* payload, int* bad);

}  // namespace skml
