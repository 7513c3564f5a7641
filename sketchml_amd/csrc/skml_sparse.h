// skml_sparse.h -- sparse-path device structures and launchers shared by skml_sparse_api.cpp and
// skml_sparse.hip (SparseVectorCompressor / GroupedMinMaxSketch / DeltaAdaptiveEncoder).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/skml.h"

namespace skml {

constexpr int kMaxGroups = 64;  // GroupedMinMaxSketch groups (Java: any int; 8 by default)
constexpr int kMaxRows = 8;     // MinMaxSketch rows <= the 8 hash functions (HashFactory.java:24-27)

// Group table in device memory.  The encode fills it on the device (k_sp_plan_*: edges from the
// quantizer header, shapes from the partition counts, interval choice from the bitsNeeded
// histogram) and the host reads it back once at the end; decode-side payloads fill it on the host.
// Group g holds grouped elements [gstart[g], gstart[g+1]).
enum : int32_t { kSpNan = 1, kSpEdges = 2, kSpOrder = 4 };  // SpGroups.status bits
struct SpGroups {
    int32_t G, rows, zero, bin_num;
    int32_t fill;    // MinMaxSketch table sentinel (MinMaxSketch.java:30-33)
    int32_t status;  // kSp* of a failed encode: the encode's later kernels return at once
    int32_t edges[kMaxGroups];  // FSketchUtils.calGroupEdges
    int64_t gstart[kMaxGroups + 1];
    int32_t cols[kMaxGroups];
    int64_t tab_off[kMaxGroups];  // first cell of group g's rows*cols table
    int32_t hash_ids[kMaxGroups][kMaxRows];
    int32_t m[kMaxGroups];     // DeltaAdaptiveEncoder.numIntervals
    int32_t kind[kMaxGroups];  // DeltaAdaptiveEncoder.flagKind (0 fixed, 1 unary)
    int64_t fb[kMaxGroups + 1];  // first flag bit of group g in the concatenated flag stream
    int64_t db[kMaxGroups + 1];  // first delta bit of group g in the concatenated delta stream
    int32_t kind1_before[kMaxGroups];  // elements of unary-flag groups before g (decode select)
    double inv_cols[kMaxGroups];       // 1.0 / cols[g]: the hash's `% size` as a multiply (set on upload)
    double col_ratio;                  // GroupedMinMaxSketch colRatio
    int64_t ncells;                    // all groups' table cells
    // 1 when the MinMax insert runs on 4-byte pairs: every group's bins lie on one side of zeroIdx
    // (so a cell's minimum distance fixes its value and no insert order is needed) and the staged
    // scatter runs (init.narrow_ok); 0 = 8-byte pairs that carry the key for the tie rule
    int32_t mm_narrow;
    int32_t pad_;
};

// What the host knows before an encode starts: the shape parameters and every group's hash
// choice (HashFactory.getRandomInt2IntHashes(seed + g) depends on g only); passed by value.
struct SpInit {
    int32_t G, rows;
    int32_t narrow_ok;  // the host runs the staged scatter (cells kept, ranges reserved)
    double col_ratio;
    int32_t hash_ids[kMaxGroups][kMaxRows];
};

constexpr int kSpThreads = 256;
constexpr int kSpTile = 2048;             // elements per workgroup tile (8 per thread)
constexpr int kCompactTile = 16384;       // dense elements per compaction tile (64 per thread)
constexpr int kDeltaHist = 33;            // bitsNeeded in 1..32

__host__ __device__ inline int64_t sp_tiles(int64_t n, int64_t tile) { return (n + tile - 1) / tile; }

// ---- launchers (skml_sparse.hip) ----
// Device-side encode plan (one workgroup each, no host round trip):
//   edges: the table from `init`, then calGroupEdges / fill from the quantizer header (status on NaN / error);
//   groups: gstart, cols, tab_off, ncells from the partition totals sizes[G];
//   delta: calOptimalIntervals per group from hist, the order-check flag, kind1_before;
//   finalize: fb / db of empty groups and the stream totals (tot = the scanned tile sums' total row).
hipError_t launch_sp_plan_edges(hipStream_t st, const void* qpayload, const SpInit& init, SpGroups* gp);
hipError_t launch_sp_plan_groups(hipStream_t st, SpGroups* gp, const uint64_t* sizes, int64_t stride);
hipError_t launch_sp_plan_delta(hipStream_t st, SpGroups* gp, const uint32_t* hist, const uint32_t* err);
hipError_t launch_sp_finalize(hipStream_t st, SpGroups* gp, const uint64_t* tot);
// Zero the stream words the writer ORs into (every tile's first and last word, and the word
// after the end) from the scanned [tiles + 1][2] tile sums.
hipError_t launch_sp_zero_edges(hipStream_t st, const uint64_t* tile_base, int64_t tiles, const SpGroups* gp,
                                uint64_t* flag_words, uint64_t* delta_words);
// DenseDoubleGradient.toSparse: keys/vals of |x| > 1e-8 in index order.  status/ticket zeroed.
hipError_t launch_compact(hipStream_t st, const float* x, int64_t dim, int32_t* keys, float* vals,
                          uint64_t* status, unsigned* ticket, int64_t* nnz_out);
// the same over doubles (DenseDoubleGradient's own values); tiles of kCompactTile / 2
hipError_t launch_compact64(hipStream_t st, const double* x, int64_t dim, int32_t* keys, double* vals,
                            uint64_t* status, unsigned* ticket, int64_t* nnz_out);
// Exclusive scan, in place, of each of K columns of a [tiles][K] u64 table; totals -> row `tiles`.
hipError_t launch_scan_cols(hipStream_t st, uint64_t* sums, int64_t tiles, int K);
// launch_scan_cols on 256-thread workgroups (a kernel queued beside a full chip)
hipError_t launch_scan_cols_small(hipStream_t st, uint64_t* sums, int64_t tiles, int K);
// The same over K columns of tiles + 1 entries each, column k at sums + k * (tiles + 1).
hipError_t launch_scan_cols_major(hipStream_t st, uint64_t* sums, int64_t tiles, int K);
// FSketchUtils.partition: per-tile group counts (column-major: group g's column of tiles + 1 at
// tile_counts + g * (tiles + 1)), then the stable scatter into group order.
// The grid also zeroes z32[0, n32) and z64[0, n64) (the next passes' counters: no memset launches).
hipError_t launch_part_count(hipStream_t st, const void* qpayload, int64_t n, const SpGroups* gp,
                             uint64_t* tile_counts, uint32_t* z32, int64_t n32, uint64_t* z64, int64_t n64);
// gbins: u16 (bins < SKML_MAX_BINS = 65536)
hipError_t launch_part_scatter(hipStream_t st, const int32_t* keys, const void* qpayload, int64_t n,
                               const SpGroups* gp, const uint64_t* tile_base, int32_t* gkeys,
                               uint16_t* gbins);
// Deltas, bitsNeeded histogram, order check, and the per-bucket pair counts of the bucketed
// MinMaxSketch.insert (bucket_count: nbuckets u64, zeroed; unused when rows == 0).
#ifndef SKML_MM_BUCKET_BITS
#define SKML_MM_BUCKET_BITS 15
#endif
// MinMax cells per bucket: 128 KB of u32 minima in LDS (narrow pairs); key-carrying pairs take
// the bucket in sub-ranges of 8192 cells (64 KB of u64 minima each)
constexpr int kMmCellsPerBucket = 1 << SKML_MM_BUCKET_BITS;
// cells (rows x n int32, may be null): each (element, row) pair's table cell, kept for the scatter.
// tile_off ([tiles of kMmChunk][nbuckets] u32, may be null): each tile's reserved offset inside
// each bucket, taken while counting, so the scatter needs neither a count pass nor atomics.
hipError_t launch_group_prep(hipStream_t st, const int32_t* gkeys, int64_t n, const SpGroups* gp, uint8_t* need,
                             uint32_t* hist, uint32_t* err, uint64_t* bucket_count, int nbuckets, int32_t* cells,
                             uint32_t* tile_off);
// pairs in bucket order (bucket_base: exclusive scan of the counts; cursor: nbuckets u64, zeroed).
// Pairs are u64, or u32 when gp->mm_narrow (only with the staged scatter: mm_scatter_staged).
bool mm_scatter_staged(bool cells, bool reserved, int nbuckets);
hipError_t launch_mm_scatter(hipStream_t st, const int32_t* gkeys, const uint16_t* gbins, int64_t n,
                             const SpGroups* gp, const uint64_t* bucket_base, uint64_t* cursor, int nbuckets,
                             void* pairs, const int32_t* cells, const uint32_t* tile_off);
#ifndef SKML_MM_CHUNK
#define SKML_MM_CHUNK 32768
#endif
constexpr int64_t kMmChunkElems = SKML_MM_CHUNK;  // elements per workgroup tile of the count / scatter passes
// The tile actually used for n grouped keys: a function of n alone, so the count pass, the
// scatter and the per-(tile, bucket) reservations agree.  kMmChunkElems while the tiles fit one
// round of k_group_prep's workgroups (two per CU, 256 CUs); above that the multiple of 4,096 in
// [16,384, kMmChunkElems] whose tile count best fills its last round, ties to the larger tile
// (C3's 26.8 M keys: 820 tiles of 32,768 fill 2 rounds to 80 %, 937 of 28,672 to 92 %;
// k_group_prep 173 -> 159 us, the staged scatter 173 -> 160 us).
constexpr int64_t kMmRoundSlots = 512;
inline int64_t mm_chunk(int64_t n) {
    const auto tiles = [n](int64_t c) { return (n + c - 1) / c; };
    if (tiles(kMmChunkElems) <= kMmRoundSlots) return kMmChunkElems;
    int64_t best = kMmChunkElems;
    double best_fill = 0.0;
    for (int64_t c = kMmChunkElems; c >= 16384; c -= 4096) {
        const int64_t t = tiles(c), rounds = (t + kMmRoundSlots - 1) / kMmRoundSlots;
        const double fill = (double)t / (double)(rounds * kMmRoundSlots);
        if (fill > best_fill + 0.02) {
            best_fill = fill;
            best = c;
        }
    }
    return best;
}
// The exact narrow image of MinMax tables whose cells hold bins in [0, bin_num) or the fill: a bin
// in 8 bits when bin_num <= 255, in 16 bits when bin_num <= 65,535 (0: no narrow image), the fill
// as the top code 2^W - 1.  The encoder writes it beside the int32 cells, the restore gathers from
// it, and the exchange blob carries it instead of the int32 cells.
__host__ __device__ inline int tnar_width_for(int32_t bin_num) {
    return bin_num <= 255 ? 8 : bin_num <= 65535 ? 16 : 0;
}
// per-bucket minimum -> int32 MinMaxSketch tables (empty cells get the fill value) and, when tnar is
// not nullptr, their exact narrow image (tnar_width_for(gp->bin_num) bits a cell); nbuckets may
// exceed the table's (gp->ncells) buckets: the extra workgroups exit
hipError_t launch_mm_bucket(hipStream_t st, const void* pairs, const uint64_t* bucket_base, int nbuckets,
                            const SpGroups* gp, int32_t* table, void* tnar);
// quantValues (Quantizer.getValues) of a dense quantizer payload into qv[bin_num] on the device
hipError_t launch_sp_qvalues(hipStream_t st, const void* qpayload, double* qv);
// int32 cells from an exact narrow image of tw (8 or 16) bits: the top code becomes `fill`
hipError_t launch_widen_cells(hipStream_t st, const void* tn, int tw, int64_t ncells, int32_t fill, int32_t* t32);
// DeltaAdaptiveEncoder bit streams: tile sums of (flag bits, delta bits), then the writer.
hipError_t launch_delta_lens(hipStream_t st, const uint8_t* need, int64_t n, const SpGroups* gp,
                             uint64_t* tile_sums);
hipError_t launch_delta_write(hipStream_t st, const int32_t* gkeys, const uint8_t* need, int64_t n,
                              SpGroups* gp, const uint64_t* tile_base, uint64_t* flag_words,
                              uint64_t* delta_words);
// ---- decode (GroupedMinMaxSketch.restore) ----
hipError_t launch_unary_count(hipStream_t st, const uint64_t* flag_words, int64_t nwords,
                              const SpGroups* gp, uint64_t* tile_sums);
hipError_t launch_unary_select(hipStream_t st, const uint64_t* flag_words, int64_t nwords,
                               const SpGroups* gp, const uint64_t* tile_base, int64_t* end_pos);
// the narrow table image k_dec_keys gathers from (launch_narrow_table's job), built by extra blocks
// of the k_dec_lens launch beside the lengths; tn == nullptr: none
struct NarrowJob {
    const int32_t* t32;
    int64_t ncells;
    void* tn;
    int width;
};
hipError_t launch_dec_lens(hipStream_t st, const uint64_t* flag_words, int64_t n_flag_words,
                           const int64_t* end_pos, int64_t n, const SpGroups* gp, uint8_t* dlen,
                           uint64_t* tile_sums, NarrowJob nj = NarrowJob{nullptr, 0, nullptr, 0});
hipError_t launch_dec_deltas(hipStream_t st, const uint64_t* delta_words, int64_t n_delta_words,
                             const uint8_t* dlen, int64_t n, const SpGroups* gp,
                             const uint64_t* tile_base, uint32_t* delta, uint64_t* tile_sums);
// lengths and deltas in one pass (decoupled look-back over the tiles' bit totals; status: 2 tiles
// + 2 u64 of scratch, zeroed by the launch); tile_sums: the tiles' delta sums as launch_dec_deltas
// writes them, or with scan_sums their exclusive scan and total (a second look-back), as
// scan_tiles leaves them
#ifdef SKML_AB
hipError_t launch_dec_lens_deltas(hipStream_t st, const uint64_t* flag_words, int64_t n_flag_words,
                                  const int64_t* end_pos, int64_t n, const SpGroups* gp,
                                  const uint64_t* delta_words, int64_t n_delta_words, uint32_t* delta,
                                  uint64_t* tile_sums, uint64_t* status, NarrowJob nj, bool scan_sums);
#endif
hipError_t launch_group_prefix(hipStream_t st, const uint32_t* delta, int64_t n, const SpGroups* gp, int G,
                               const uint64_t* tile_base, uint64_t* gpre);
// keys and MinMax bins; gh: the host copy of *gp (the grid follows the group sizes).  width 8 / 16:
// tnar is launch_narrow_table's image of `table` (int32 cells outside [0, 2^width - 1) read back
// from `table`), or with table == nullptr an exact image (tnar_width_for: the top code is the
// fill); width 32: `table` alone (nullptr with gp->rows == 0: keys only).  gbins may be
// null; gvals (optional) receives quantValues[bin] from qv[nq], a bin outside it sets *err
// The runs' bounds written by the key query itself.  info == nullptr: Gradient.sum's tiles
// (k_agg_bounds' job): bounds[g * (ntiles + 1) + t] = the first element of run g with key >= t <<
// tile_bits (the run's end past its last key); a key outside [0, dim) or not ascending inside its
// run sets *err bit 0.  info != nullptr: the one-pass Sort.merge's key ranges (k_rs_bounds' job,
// kRsRanges + 1 per run, RsInfo's last ranges and irregular flag; *info zeroed before).
// bounds == nullptr: not written.
struct RsInfo;
struct RunBoundsOut {
    int32_t* bounds;
    int64_t ntiles, dim;
    int tile_bits;
    RsInfo* info = nullptr;
};
hipError_t launch_dec_keys(hipStream_t st, const uint32_t* delta, int64_t n, const SpGroups* gp, const SpGroups& gh,
                           const uint64_t* tile_base, const uint64_t* gpre, const int32_t* table, const void* tnar,
                           int width, int32_t* gkeys, int32_t* gbins, int nq, void* gbn, int bn_width,
                           unsigned* err, RunBoundsOut rb = RunBoundsOut{nullptr, 0, 0, 0});
// the narrow (width 8 or 16) image of int32 MinMax tables for k_dec_keys; t32 16-byte aligned
hipError_t launch_narrow_table(hipStream_t st, const int32_t* t32, int64_t ncells, int width, void* tn);
// live entries of a restored payload (skml_sparse_decode_sum_f64's toAuto choice)
// live entries (|quantValues[bin]| > 1e-8) among n narrow bins (bw = 1 or 2 bytes each)
hipError_t launch_count_live(hipStream_t st, const void* bins, int bw, int64_t n, const double* qv, uint64_t* count);
// the tiled Gradient.sum: per-payload run bounds per dense tile, then the tiles built in LDS
constexpr int kAggTile = 4096;  // dense keys per tile (32 KB of doubles in LDS)
struct AggPayload {
    const int32_t* gk;      // restored keys, grouped order
    const void* gb;         // their bins, bw bytes each (1: bin_num <= 256, else 2)
    const double* qv;       // quantValues (timesBy applied), nq of them
    const int32_t* bounds;  // [G][ntiles + 1]
    int32_t G, dense_form;
    int32_t bw, nq;
    // gk - keys base and gb - bins base (elements / bytes) of launch_agg_tiles' bases: the staged
    // tiles index both with 32-bit offsets from one base each
    int32_t gk_off, gb_off;
};
static_assert(sizeof(AggPayload) % 8 == 0, "copied as u64 words");
// tile_bits: log2 of the keys per tile the bounds are taken at (agg_tile_bits of the chosen form)
#ifdef SKML_AB
hipError_t launch_agg_bounds(hipStream_t st, const int32_t* gk, int64_t n, const SpGroups* gp, int64_t ntiles,
                             int64_t dim, int32_t* bounds, unsigned* err, int tile_bits);
#endif
// vtiles: the staged wave-tile form (agg_vtiles_ok: payloads of at most 8 groups and 256
// quantValues, launched 8 at a time); else the 4,096-key wave-per-payload tiles (any P, G, nq).
// Both set err bit 1 for a key outside its tile and bit 2 for a key repeated inside one payload.
constexpr int kAggVPayloads = 8;
bool agg_vtiles_ok(int max_groups, int max_nq);
int agg_tile_bits(bool vtiles);
// kbase / bbase: the buffers every payload's gk / gb lie in (AggPayload::gk_off / gb_off);
// any_dense: a payload of the launch takes the dense form (AggPayload::dense_form)
hipError_t launch_agg_tiles(hipStream_t st, const AggPayload* pays, int P, int64_t ntiles, int64_t dim, double* out,
                            int from_out, double scale, unsigned* err, bool vtiles, const int32_t* kbase,
                            const uint8_t* bbase, bool any_dense);

// Exported sparse payload: one contiguous device blob (skml_sparse_export / _import, the unit the
// RCCL all-gather moves).  Offsets are from the blob start, every section 256-byte aligned.
constexpr uint32_t kSpBlobMagic = 0x50534B53u;  // "SKSP"
struct SpBlobHeader {
    uint32_t magic;
    int32_t version;
    int64_t total_bytes;
    int64_t nnz;
    int64_t ncells;
    int64_t n_flag_words, n_delta_words;  // stored words (bit streams + one trailing zero word)
    int64_t flag_bits, delta_bits;
    int32_t nvalues;                      // quantValues doubles
    int32_t quant_bytes;                  // dense header + splits
    int64_t off_groups, off_quant, off_values, off_tables, off_flags, off_deltas;
    skml_params params;
    int32_t table_width;                  // version 2: bits a MinMax cell (8 / 16: the exact narrow
    int32_t pad0;                         // image, tnar_width_for; 32: int32 cells); version 1: 32
    int64_t reserved[7];
};
static_assert(sizeof(SpBlobHeader) <= 256, "blob header fits its 256-byte section");
// One round of pairwise stable merges of sorted runs (Sort.merge order: lower run first on ties).
// run_start: nruns + 1 device offsets; total = run_start[nruns].
// run_start: nruns + 1 HOST offsets (passed to the kernels by value); split: (total / 2048 + 2)
// int64 device scratch (the tile boundaries' merge-path split points)
// Sort.merge in one pass (the regular case: runs ascend strictly, keys distinct and in [0, INT32_MAX)):
// bounds = G x (kRsRanges + 1) int32 scratch; info->irregular != 0 after the launches means the
// input was not regular and the caller must run the merge rounds instead.  vkind 0: out = int32
// bins; 1: float quantValues[bin]; 2: double quantValues[bin] (qv: nq doubles).  *info must be
// zeroed by the caller before the launch.
constexpr int kRsBits = 13, kRsRange = 1 << kRsBits, kRsWords = kRsRange / 32;
constexpr int64_t kRsRanges = (int64_t)1 << (31 - kRsBits);  // key ranges of [0, 2^31)
struct RsInfo {
    unsigned irregular;          // 1: a run does not ascend / key out of range, 2: a repeated key or bad bin
    int32_t tmax1;               // 1 + the last key range holding a key
    int32_t tlast1[kMaxGroups];  // 1 + run g's last key range (0: empty run)
};
hipError_t launch_rs_merge(hipStream_t st, const int32_t* gk, const int32_t* gb, int64_t n, const SpGroups* gp,
                           int32_t* bounds, RsInfo* info, int32_t* keys_out, void* out, int vkind, const double* qv,
                           int nq, bool bounds_ready);  // bounds_ready: the key query wrote bounds and *info
hipError_t launch_merge_round(hipStream_t st, const int32_t* kin, const int32_t* bin_in, int32_t* kout,
                              int32_t* bout, const int64_t* run_start, int nruns, int64_t total, int64_t* split);
// values[bins[i]] from the double quantValues LUT (SparseVectorCompressor.java:118-126); a bin
// outside [0, B) writes 0 and sets *err.
hipError_t launch_bin_values(hipStream_t st, const int32_t* bins, int64_t n, const double* qvalues, int B,
                             float* vals, unsigned* err);
hipError_t launch_bin_values64(hipStream_t st, const int32_t* bins, int64_t n, const double* qvalues, int B,
                               double* vals, unsigned* err);

// HuffmanEncoder of the MinMaxSketch tables (serialisation): per-group histograms [G][B+1]
// (symbol B = the fill value), code lengths per tile, and the MSB-first code stream writer
// (gbit[g] = first bit of group g's stream).  lut[g*(B+1)+sym] = (numBits << 32) | bits.
hipError_t launch_huff_hist(hipStream_t st, const int32_t* table, const SpGroups* gp, int G, int B,
                            int64_t max_cells, uint32_t* hist);
hipError_t launch_huff_lens(hipStream_t st, const int32_t* table, int64_t ncells, const SpGroups* gp, int B,
                            const uint64_t* lut, uint64_t* tile_sums);
hipError_t launch_huff_write(hipStream_t st, const int32_t* table, int64_t ncells, const SpGroups* gp, int B,
                             const uint64_t* lut, const uint64_t* tile_base, uint64_t* words, int64_t* gbit);

// HuffmanEncoder.decode (readObject side): speculative parallel decoding of the per-group code
// streams (see skml_sparse.hip).  lut: kHuffLutSize int2 per group row, {value, length} or
// {tree node, -1}; nodes: int4 {left, right, value, 0}, left < 0 for a leaf.
constexpr int kHuffLutBits = 12;
constexpr int kHuffLutSize = 1 << kHuffLutBits;
#ifndef SKML_HUFF_SEG
#define SKML_HUFF_SEG 2048
#endif
constexpr int64_t kHuffSeg = SKML_HUFF_SEG;  // bits per speculative segment
struct HuffDecGroup {
    int64_t word0;   // first word of the group's stream in the concatenated words
    int64_t nwords;  // stored words (BitSet.toLongArray); bits beyond read as 0
    int64_t tab_off; // first table cell
    int64_t size;    // symbols (rows * cols)
    int32_t lut_row;
    int32_t seg0;    // first segment of the group
};
struct HuffSeg {
    int64_t lim;  // nominal end: the next segment's nominal start
    int32_t g;
    int16_t first, last;
};
hipError_t launch_huff_spec(hipStream_t st, int nseg, const HuffSeg* segs, const HuffDecGroup* grp,
                            const uint64_t* words, const int2* lut, const int4* nodes, int64_t* start, int64_t* end,
                            uint64_t* cnt);
hipError_t launch_huff_sync(hipStream_t st, int nseg, const HuffSeg* segs, const HuffDecGroup* grp,
                            const uint64_t* words, const int2* lut, const int4* nodes, int64_t* start,
                            const int64_t* end_in, int64_t* end_out, uint64_t* cnt, unsigned* changed);
hipError_t launch_huff_decode_write(hipStream_t st, int nseg, const HuffSeg* segs, const HuffDecGroup* grp,
                                    const uint64_t* words, const int2* lut, const int4* nodes, const int64_t* start,
                                    const uint64_t* off, int32_t* table, unsigned* err);
hipError_t launch_fill_i32(hipStream_t st, int32_t* dst, int64_t n, int32_t v);

// ---- the GroupedMinMaxSketch field stream on the device (skml_wire.hip) ----
struct WireSrc {
    const uint64_t* flags;   // concatenated DeltaAdaptive flag bits
    const uint64_t* deltas;  // concatenated DeltaAdaptive delta bits
    const uint64_t* huff;    // concatenated HuffmanEncoder code bits of the tables
};
struct WireSec {          // one long array of the stream
    int64_t dst;          // byte offset of its first long in the stream
    int64_t bit0, nbits;  // its bit range in the source stream
    int64_t nwords;       // longs written (BitSet.toLongArray: trailing zero words trimmed)
    int32_t src;          // 0 flags, 1 deltas, 2 Huffman
    int32_t pad;
};
constexpr int kWireMaxSec = 3 * kMaxGroups;
hipError_t launch_wire_lastnz(hipStream_t st, const WireSrc& src, const WireSec* secs, int nsec, uint64_t* nz);
hipError_t launch_wire_longs(hipStream_t st, const WireSrc& src, const WireSec* secs, const int64_t* npre, int nsec,
                             int64_t total_words, uint8_t* wire);
hipError_t launch_wire_pieces(hipStream_t st, const uint8_t* small, const int64_t* pieces, int npieces, uint8_t* wire);
struct RdFlagSec {   // one group's stored flag long array in the device copy of the stream
    int64_t pos;     // byte offset of its first long
    int64_t nstored; // longs stored
    int64_t nbits;   // fixed flags: size * nf (the bits that hold fields)
    int64_t size;    // keys of the group
    int32_t nf;      // fixed flags: bits per field
    int32_t pad;
};
struct RdBitSec {
    int64_t pos, nstored;
};
hipError_t launch_rd_fixed_sum(hipStream_t st, const uint8_t* stream, const RdFlagSec* secs, const int64_t* wpre, int nsec,
                               int64_t total_words, uint64_t* sums);
constexpr int64_t kRdTileWords = 2048;  // k_rd_unary_tiles' words per tile
// tpre: per-section prefix of ceil(nstored / kRdTileWords) tiles; flen[s] = bit length of its `size` unary flags
hipError_t launch_rd_unary(hipStream_t st, const uint8_t* stream, const RdFlagSec* secs, const int64_t* tpre, int nsec,
                           int64_t total_tiles, uint32_t* tile_zeros, int64_t* flen);
hipError_t launch_rd_stream(hipStream_t st, const uint8_t* stream, const RdBitSec* secs, const int64_t* off, int G,
                            int64_t nwords, uint64_t* out);
hipError_t launch_rd_words(hipStream_t st, const uint8_t* stream, const int64_t* pos, const int64_t* wpre, int nsec,
                           int64_t total_words, uint64_t* words);

// ---- context services (skml_api.cpp) ----
hipStream_t ctx_stream(skml_ctx* c);
// the context's side stream (a high-priority child context) and two events for a fork / join
int ctx_side_fork(skml_ctx* c, hipStream_t* side, hipEvent_t* fork, hipEvent_t* join);
// the side context itself (its stream is ctx_side_fork's `side`; nullptr before the first fork)
skml_ctx* ctx_side_ctx(skml_ctx* c);
int ctx_device(skml_ctx* c);
// grow-only device scratch buffer `slot` (< kScratchSlots) of at least `bytes`; null on failure
constexpr int kScratchSlots = 24;
void* ctx_scratch(skml_ctx* c, int slot, size_t bytes);
// pinned host staging of at least `bytes`
void* ctx_pinned(skml_ctx* c, size_t bytes);
// the context's coherent, device-mapped host word (nullptr if it cannot be allocated)
int64_t* ctx_host_word(skml_ctx* c);
int set_error(int code, const char* msg);
bool ctx_timing(skml_ctx* c);

}  // namespace skml
