// skml_sparse_api.cpp -- host side of the sparse C ABI (include/skml.h, "Sparse path"):
// SparseVectorCompressor.compressSparse / decompressSparse (sample/SparseVectorCompressor.java:
// 52-67,118-126) over GroupedMinMaxSketch (frequency/GroupedMinMaxSketch.java:51-146) and the
// standalone DeltaAdaptiveEncoder (binary/DeltaAdaptiveEncoder.java).  All element work runs in
// skml_sparse.hip; the host plans launches, owns the per-group table and the tiny decisions
// the reference makes on whole-group statistics (colNum, hash choice, interval choice).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "skml_internal.h"
#include "skml_sparse.h"

using namespace skml;

namespace {

int sfail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return set_error(code, buf);
}

#define SP_HIP(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return sfail(SKML_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                         __FILE__, __LINE__);                                                \
    } while (0)

// scratch slots (device)
enum {
    kSlotTiles = 0,
    kSlotGKeys,
    kSlotGBins,
    kSlotNeed,
    kSlotCells,
    kSlotSmall,  // hist + err + gpre + run offsets
    kSlotEndPos,
    kSlotDelta,
    kSlotK1,
    kSlotB1,
    kSlotStatus,
    kSlotCellIdx,
    kSlotTileOff,
    kSlotCKeys,     // toSparse output of skml_sparse_encode_f32
    kSlotCVals,
    kSlotDeltaEnc,  // standalone DeltaAdaptiveEncoder: group table + stream words
    kSlotWire,      // readObject: the device copy of the field stream
    kSlotWireMeta,  // the wire kernels' section tables and small results
    kSlotNarrowTab, // the MinMax query's narrow table image
    kSlotRsMerge,   // one-pass Sort.merge: RsInfo + the runs' key-range bounds
    kSlotLookback,  // the restore's look-back statuses (lengths + deltas in one pass)
    kSlotCount_,
};
static_assert(kSlotCount_ <= kScratchSlots, "scratch slots");

// java.util.Random (JDK 8 spec): seed scramble, next(bits), nextInt(bound).
struct JavaRandom {
    uint64_t s;
    explicit JavaRandom(int64_t seed) : s(((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1)) {}
    int32_t next(int bits) {
        s = (s * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return (int32_t)(s >> (48 - bits));
    }
    int32_t next_int(int32_t bound) {
        if ((bound & -bound) == bound) return (int32_t)(((int64_t)bound * (int64_t)next(31)) >> 31);
        int32_t bits, val;
        do {
            bits = next(31);
            val = bits % bound;
        } while ((int32_t)((uint32_t)bits - (uint32_t)val + (uint32_t)(bound - 1)) < 0);  // int overflow test
        return val;
    }
};

// HashFactory.getRandomInt2IntHashes (hash/HashFactory.java:23-38) with Maths.shuffle
// (util/Maths.java:41-49): Fisher-Yates from the end over the 8 hash ids; rows take the first.
void pick_hashes(int64_t seed, int rows, int32_t* ids) {
    int32_t idx[8];
    for (int i = 0; i < 8; i++) idx[i] = i;
    JavaRandom r(seed);
    for (int i = 7; i > 0; i--) {
        const int32_t j = r.next_int(i + 1);
        std::swap(idx[i], idx[j]);
    }
    for (int i = 0; i < rows; i++) ids[i] = idx[i];
}

// FSketchUtils.calGroupEdges (frequency/FSketchUtils.java:9-28)
int group_edges(int32_t zero, int32_t bins, int32_t G, int32_t* edges) {
    if (G == 2) {
        edges[0] = zero;
        edges[1] = bins;
        return SKML_OK;
    }
    const int32_t bpg = bins / G;
    if (zero < bpg) edges[0] = zero;
    else if (bpg == 0) return sfail(SKML_E_ARG, "calGroupEdges: / by zero (bin_num %d < group_num %d)", bins, G);
    else if ((zero % bpg) < (bpg / 2)) edges[0] = bpg + zero % bpg;
    else edges[0] = zero % bpg;
    for (int32_t i = 1; i < G - 1; i++) edges[i] = edges[i - 1] + bpg;
    edges[G - 1] = bins;
    return SKML_OK;
}

int32_t log2nlz(int32_t k) { return 31 - __builtin_clz((uint32_t)k); }

// MinMaxSketch.compare with Java int wrap (MinMaxSketch.java:80-86)
int32_t mm_dist(int32_t v, int32_t zero) {
    const int32_t d = (int32_t)((uint32_t)v - (uint32_t)zero);
    return d < 0 ? (int32_t)(0u - (uint32_t)d) : d;
}
int32_t mm_cmp(int32_t a, int32_t b, int32_t zero) {
    return (int32_t)((uint32_t)mm_dist(a, zero) - (uint32_t)mm_dist(b, zero));
}

// HuffmanEncoder.encode's tree (binary/HuffmanEncoder.java:88-111): leaves fed in ascending
// value order (Int2ObjectRBTreeMap) into a JDK 8 java.util.PriorityQueue ordered by occurrence
// (binary heap, siftUp / siftDown as in the JDK), two polls per merge, the merged node offered
// back; codes from the traversal (left 0, right 1; a lone leaf gets one bit).
struct HuffItem {
    int32_t value, bits, nbits;
};
struct HuffBuilder {
    struct Node {
        int32_t value;
        int64_t occ;
        int32_t left, right;
        bool leaf;
    };
    std::vector<Node> pool;
    std::vector<int32_t> heap;
    bool less_than(int32_t a, int32_t b) const { return pool[(size_t)a].occ < pool[(size_t)b].occ; }
    void sift_up(size_t k, int32_t x) {
        while (k > 0) {
            const size_t parent = (k - 1) >> 1;
            const int32_t e = heap[parent];
            if (!less_than(x, e)) break;  // comparator(x, e) >= 0
            heap[k] = e;
            k = parent;
        }
        heap[k] = x;
    }
    void sift_down(size_t k, int32_t x) {
        const size_t n = heap.size(), half = n >> 1;
        while (k < half) {
            size_t child = 2 * k + 1;
            int32_t c = heap[child];
            const size_t right = child + 1;
            if (right < n && less_than(heap[right], c)) c = heap[child = right];  // cmp(c, right) > 0
            if (!less_than(c, x)) break;                                          // cmp(x, c) <= 0
            heap[k] = c;
            k = child;
        }
        heap[k] = x;
    }
    void offer(int32_t x) {
        heap.push_back(x);
        sift_up(heap.size() - 1, x);
    }
    int32_t poll() {
        const int32_t res = heap[0];
        const int32_t x = heap.back();
        heap.pop_back();
        if (!heap.empty()) sift_down(0, x);
        return res;
    }
    // symbols: (value, count) in ascending signed value order, counts > 0
    bool build(const std::vector<std::pair<int32_t, int64_t>>& syms, std::vector<HuffItem>& items) {
        pool.clear();
        heap.clear();
        for (const auto& sv : syms) {
            pool.push_back(Node{sv.first, sv.second, -1, -1, true});
            offer((int32_t)pool.size() - 1);
        }
        while (heap.size() > 1) {
            const int32_t x = poll(), y = poll();
            pool.push_back(Node{-1, pool[(size_t)x].occ + pool[(size_t)y].occ, x, y, false});
            offer((int32_t)pool.size() - 1);
        }
        items.clear();
        if (heap.empty()) return true;
        bool ok = true;
        // iterative traversal (left first), collecting leaves
        std::vector<std::tuple<int32_t, uint32_t, int>> st{{heap[0], 0u, 0}};
        while (!st.empty()) {
            auto [nd, bits, depth] = st.back();
            st.pop_back();
            const Node& n = pool[(size_t)nd];
            if (n.leaf) {
                items.push_back(HuffItem{n.value, (int32_t)bits, depth == 0 ? 1 : depth});
                if (depth > 32) ok = false;
            } else {
                st.emplace_back(n.right, (bits << 1) | 1u, depth + 1);
                st.emplace_back(n.left, bits << 1, depth + 1);
            }
        }
        std::sort(items.begin(), items.end(), [](const HuffItem& a, const HuffItem& b) { return a.value < b.value; });
        return ok;
    }
};

template <class T>
T* scratch(skml_ctx* c, int slot, size_t count) {
    return reinterpret_cast<T*>(ctx_scratch(c, slot, sizeof(T) * (count ? count : 1)));
}

}  // namespace

// =============================================================================================
// library-owned sparse payload
// =============================================================================================
struct skml_sparse {
    int device = 0;
    int64_t nnz = 0;
    skml_params params{};
    void* qpayload = nullptr;  // dense payload of the values' quantizer (header, splits, codes)
    size_t qbytes = 0;
    skml_dense_header hdr{};
    std::vector<double> splits;
    std::vector<double> qvalues;  // SparseVectorCompressor.quantValues (getValues, timesBy'd)
    SpGroups g{};               // host copy (complete after encode)
    void* block = nullptr;      // encode: one pooled device block holding everything below
    size_t block_cap = 0;
    SpGroups* g_dev = nullptr;  // device copy
    int32_t* tables = nullptr;  // all groups' MinMaxSketch tables, rows x cols each
    int64_t ncells = 0;
    void* tnar = nullptr;       // their exact narrow image (tnar_width_for), or nullptr; in the block
    int tnar_width = 0;         // 8 or 16 bits a cell
    double* qv_dev = nullptr;   // quantValues on the device (in the block), valid while qv_dev_ok:
    bool qv_dev_ok = false;     // written by the encode / import, stale after timesBy until re-uploaded
    uint64_t* flag_words = nullptr;  // concatenated DeltaAdaptive flag streams
    uint64_t* delta_words = nullptr;
    int64_t flag_bits = 0, delta_bits = 0;
    int64_t n_flag_words = 0, n_delta_words = 0;
    // MinMaxSketch tables' HuffmanEncoder (built on the first serialisation)
    bool huff_done = false;
    std::vector<std::vector<HuffItem>> huff_items;  // per group, ascending value
    std::vector<int64_t> huff_bit0, huff_bits;      // per group stream range
    uint64_t* huff_words = nullptr;
    int64_t n_huff_words = 0;
    void* wire_dev = nullptr;   // the serialised field stream on the device (built once; the
    size_t wire_bytes = 0;      // encoded state is immutable: timesBy scales quantValues only)
};

namespace {

// Device blocks of encoded payloads, recycled across encodes: a hipMalloc / hipFree pair per
// payload cost more than all the rest of an encode's host work (hipFree also waits for the
// device).  Every sparse call completes its device work before it returns (a failing encode
// synchronises before releasing), so a freed payload's block has no pending users.
struct BlockPool {
    struct Blk {
        int dev;
        void* p;
        size_t cap;
    };
    std::mutex mu;
    std::vector<Blk> free;
};
constexpr size_t kPoolMaxBlocks = 8;
BlockPool& block_pool() {
    static BlockPool* bp = new BlockPool();  // never destroyed: payloads may be freed during exit
    return *bp;
}
void pool_drop(std::vector<BlockPool::Blk>& v, int cur_dev) {
    for (const auto& b : v) {
        (void)hipSetDevice(b.dev);
        (void)hipFree(b.p);
    }
    if (!v.empty()) (void)hipSetDevice(cur_dev);
}
// smallest pooled block of `dev` holding `bytes` without wasting more than bytes + 64 MiB
void* block_get(int dev, size_t bytes, size_t* cap) {
    BlockPool& bp = block_pool();
    {
        std::lock_guard<std::mutex> lk(bp.mu);
        size_t best = bp.free.size();
        for (size_t i = 0; i < bp.free.size(); i++) {
            const BlockPool::Blk& b = bp.free[i];
            if (b.dev == dev && b.cap >= bytes && b.cap <= 2 * bytes + ((size_t)64 << 20) &&
                (best == bp.free.size() || b.cap < bp.free[best].cap))
                best = i;
        }
        if (best < bp.free.size()) {
            void* p = bp.free[best].p;
            *cap = bp.free[best].cap;
            bp.free.erase(bp.free.begin() + (ptrdiff_t)best);
            return p;
        }
    }
    const size_t c = align_up(std::max<size_t>(bytes, 1), (size_t)2 << 20);
    void* p = nullptr;
    if (hipMalloc(&p, c) != hipSuccess) {  // out of memory: return this device's pooled blocks, retry once
        (void)hipGetLastError();
        std::vector<BlockPool::Blk> drop;
        {
            std::lock_guard<std::mutex> lk(bp.mu);
            for (size_t i = 0; i < bp.free.size();)
                if (bp.free[i].dev == dev) {
                    drop.push_back(bp.free[i]);
                    bp.free.erase(bp.free.begin() + (ptrdiff_t)i);
                } else {
                    i++;
                }
        }
        pool_drop(drop, dev);
        if (hipMalloc(&p, c) != hipSuccess) return nullptr;
    }
    *cap = c;
    return p;
}
void block_put(int dev, void* p, size_t cap) {
    BlockPool& bp = block_pool();
    std::vector<BlockPool::Blk> drop;
    {
        std::lock_guard<std::mutex> lk(bp.mu);
        bp.free.push_back(BlockPool::Blk{dev, p, cap});
        while (bp.free.size() > kPoolMaxBlocks) {
            drop.push_back(bp.free.front());
            bp.free.erase(bp.free.begin());
        }
    }
    pool_drop(drop, dev);
}

void sparse_release(skml_sparse* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->block) {
        block_put(s->device, s->block, s->block_cap);
    } else {
        if (s->qpayload) (void)hipFree(s->qpayload);
        if (s->g_dev) (void)hipFree(s->g_dev);
        if (s->tables) (void)hipFree(s->tables);
        if (s->flag_words) (void)hipFree(s->flag_words);
        if (s->delta_words) (void)hipFree(s->delta_words);
    }
    if (s->huff_words) (void)hipFree(s->huff_words);
    if (s->wire_dev) (void)hipFree(s->wire_dev);
    delete s;
}

// The host table is edited between uploads, so each upload completes before returning.
int upload_groups(skml_ctx* c, skml_sparse* s) {
    for (int g = 0; g < kMaxGroups; g++) s->g.inv_cols[g] = s->g.cols[g] > 0 ? 1.0 / (double)s->g.cols[g] : 0.0;
    SP_HIP(hipMemcpyAsync(s->g_dev, &s->g, sizeof(SpGroups), hipMemcpyHostToDevice, ctx_stream(c)));
    SP_HIP(hipStreamSynchronize(ctx_stream(c)));
    return SKML_OK;
}

int sync_to_host(skml_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!bytes) return SKML_OK;
    void* pin = ctx_pinned(c, bytes);
    if (!pin) return sfail(SKML_E_OOM, "pinned staging of %zu bytes", bytes);
    SP_HIP(hipMemcpyAsync(pin, src, bytes, hipMemcpyDeviceToHost, ctx_stream(c)));
    SP_HIP(hipStreamSynchronize(ctx_stream(c)));
    std::memcpy(dst, pin, bytes);
    return SKML_OK;
}

// Spin on the context's coherent host word until a kernel of this stream publishes a count >= 0
// there.  The stream is checked every few thousand polls, so a failed launch cannot hang the caller.
int wait_host_count(skml_ctx* c, const int64_t* word, int64_t* out) {
    const volatile int64_t* w = word;
    hipStream_t st = ctx_stream(c);
    for (uint64_t k = 1;; k++) {
        const int64_t v = *w;
        if (v >= 0) {
            *out = v;
            return SKML_OK;
        }
        if ((k & 4095) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {  // the stream has drained: the publishing store is visible now
                const int64_t v2 = *w;
                if (v2 < 0) return sfail(SKML_E_HIP, "the compaction did not publish its count");
                *out = v2;
                return SKML_OK;
            }
            if (e != hipErrorNotReady) return sfail(SKML_E_HIP, "stream failed: %s", hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
}

// Exclusive column scans of a [tiles][K] table; column totals copied to `totals` (host).
int scan_tiles(skml_ctx* c, uint64_t* sums, int64_t tiles, int K, uint64_t* totals) {
    SP_HIP(launch_scan_cols(ctx_stream(c), sums, tiles, K));
    if (totals) return sync_to_host(c, totals, sums + tiles * K, sizeof(uint64_t) * (size_t)K);
    return SKML_OK;
}

// Worst-case stream words of n keys: 17 flag bits (unary, 16 intervals) and 32 delta bits each,
// the trailing word, and the edge words' slack.
inline int64_t flag_words_max(int64_t n) { return (17 * n + 63) / 64 + 3; }
inline int64_t delta_words_max(int64_t n) { return (32 * n + 63) / 64 + 3; }

// DeltaAdaptiveEncoder.encode (binary/DeltaAdaptiveEncoder.java:54-109) of every group of g_dev
// over the grouped keys gk (n of them), all on the stream: interval choice from the bitsNeeded
// histogram, bit lengths, their scan, the edge words, the writer, the group bases.
int encode_delta_device(skml_ctx* c, hipStream_t st, SpGroups* g_dev, const int32_t* gk, const uint8_t* need,
                        int64_t n, const uint32_t* hist, const uint32_t* err, uint64_t* fw, uint64_t* dw) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    uint64_t* ts = scratch<uint64_t>(c, kSlotTiles, (size_t)(tiles + 1) * 2);
    if (!ts) return sfail(SKML_E_OOM, "tile sums");
    SP_HIP(launch_sp_plan_delta(st, g_dev, hist, err));
    SP_HIP(launch_delta_lens(st, need, n, g_dev, ts));
    SP_HIP(launch_scan_cols_small(st, ts, tiles, 2));
    SP_HIP(launch_sp_zero_edges(st, ts, tiles, g_dev, fw, dw));
    SP_HIP(launch_delta_write(st, gk, need, n, g_dev, ts, fw, dw));
    SP_HIP(launch_sp_finalize(st, g_dev, ts + tiles * 2));
    return SKML_OK;
}

int check_params(const skml_params* p) {
    if (!p) return sfail(SKML_E_ARG, "params is NULL");
    if (p->bin_num < 2 || p->bin_num > SKML_MAX_BINS)
        return sfail(SKML_E_ARG, "bin_num %d outside [2, %d]", p->bin_num, SKML_MAX_BINS);
    if (p->group_num < 2 || p->group_num > kMaxGroups)
        return sfail(SKML_E_ARG, "group_num %d outside [2, %d]", p->group_num, kMaxGroups);
    if (p->row_num < 1 || p->row_num > kMaxRows)
        return sfail(SKML_E_ARG, "Currently only %d hash functions are available", kMaxRows);
    if (!(p->col_ratio > 0.0)) return sfail(SKML_E_ARG, "col_ratio must be positive");
    if (p->quant_type != SKML_QUANTILE && p->quant_type != SKML_UNIFORM)
        return sfail(SKML_E_ARG, "Unrecognizable quantization type: %d", p->quant_type);
    if (p->parallelism < 0 || p->parallelism > 65536)
        return sfail(SKML_E_ARG, "Invalid parallelism: %d", p->parallelism);
    return SKML_OK;
}

// SparseVectorCompressor.compressSparse (sample/SparseVectorCompressor.java:52-67) over
// GroupedMinMaxSketch.insert (frequency/GroupedMinMaxSketch.java:51-121).  Everything is queued
// on the stream without a host round trip -- the per-group decisions are made on the device
// (k_sp_plan_*) -- and the host reads the quantizer header, splits and group table back once.
// vals: nnz floats, or nnz doubles when f64 (the reference's own double[] values: the quantizer
// sketches and bins the doubles themselves, QuantileQuantizer.quantize(double[])).
// skml_debug_sparse_scratch_fail: simulate failed MinMax staging allocations (tests only)
static std::atomic<int> g_fail_cellbuf{0};

int encode_kv(skml_ctx* c, const int32_t* keys, const void* vals, bool f64, int64_t nnz, const skml_params* p,
              skml_sparse** out) {
    hipStream_t st = ctx_stream(c);
    skml_sparse* s = new skml_sparse();
    s->device = ctx_device(c);
    s->nnz = nnz;
    s->params = *p;
    hipStream_t side = nullptr;  // the DeltaAdaptive chain's stream, once forked
    auto bail = [&](int code) {
        (void)hipStreamSynchronize(st);  // the block returns to the pool: nothing may still use it
        if (side) (void)hipStreamSynchronize(side);
        sparse_release(s);
        return code;
    };
#define SP_TRY(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return bail(sfail(SKML_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_))); \
    } while (0)
    const int G = p->group_num, rows = p->row_num;
    // ---- the payload's device block, sized for the worst case (no count has to come back first) ----
    const double cols_all = std::ceil((double)nnz * p->col_ratio);
    if (cols_all * rows > 4.0e12) return bail(sfail(SKML_E_OOM, "MinMaxSketch tables of colRatio %g", p->col_ratio));
    const int64_t cells_max = nnz > 0 ? (int64_t)rows * ((int64_t)cols_all + 2 * G + 2) : 0;
    const int64_t fwn = flag_words_max(nnz), dwn = delta_words_max(nnz);
    s->qbytes = skml_dense_payload_bytes(nnz, p->bin_num);
    const size_t o_g = align_up(s->qbytes, 256);
    const size_t o_tab = o_g + align_up(sizeof(SpGroups), 256);
    // the tables' exact narrow image: 16 bits a cell reserved (the effective bin count, which picks
    // 8 or 16, is known on the device only)
    const bool want_tn = tnar_width_for(p->bin_num) != 0;
    const size_t o_tn = o_tab + align_up(sizeof(int32_t) * (size_t)std::max<int64_t>(cells_max, 1), 256);
    const size_t o_fw = o_tn + (want_tn ? align_up(sizeof(uint16_t) * (size_t)std::max<int64_t>(cells_max, 1), 256) : 0);
    const size_t o_dw = o_fw + align_up(sizeof(uint64_t) * (size_t)fwn, 256);
    const size_t o_qv = o_dw + align_up(sizeof(uint64_t) * (size_t)dwn, 256);
    const size_t total = o_qv + sizeof(double) * (size_t)p->bin_num;
    char* blk = static_cast<char*>(block_get(s->device, total, &s->block_cap));
    if (!blk) return bail(sfail(SKML_E_OOM, "sparse payload of %zu bytes", total));
    s->block = blk;
    s->qpayload = blk;
    s->qv_dev = reinterpret_cast<double*>(blk + o_qv);
    s->g_dev = reinterpret_cast<SpGroups*>(blk + o_g);
    s->tables = reinterpret_cast<int32_t*>(blk + o_tab);
    s->tnar = want_tn ? blk + o_tn : nullptr;
    s->flag_words = reinterpret_cast<uint64_t*>(blk + o_fw);
    s->delta_words = reinterpret_cast<uint64_t*>(blk + o_dw);
    // ---- 1. the values' quantizer (Quantizer.newQuantizer(quantType), SparseVectorCompressor.java:60-62) ----
    skml_params qp = *p;
    int qe;
    if (f64) {
        const double* v = static_cast<const double*>(vals);
        qe = p->quant_type == SKML_UNIFORM ? skml_dense_encode_uniform_f64(c, v, nnz, &qp, s->qpayload, s->qbytes)
             : p->parallelism > 1 ? skml_dense_encode_parallel_f64(c, v, nnz, p->parallelism, &qp, s->qpayload, s->qbytes)
                                  : skml_dense_encode_f64(c, v, nnz, &qp, s->qpayload, s->qbytes);
    } else {
        const float* v = static_cast<const float*>(vals);
        qe = p->quant_type == SKML_UNIFORM ? skml_dense_encode_uniform_f32(c, v, nnz, &qp, s->qpayload, s->qbytes)
             : p->parallelism > 1 ? skml_dense_encode_parallel_f32(c, v, nnz, p->parallelism, &qp, s->qpayload, s->qbytes)
                                  : skml_dense_encode_f32(c, v, nnz, &qp, s->qpayload, s->qbytes);
    }
    if (qe) return bail(qe);
    // ---- 2. group edges (device), partition counts, per-group MinMaxSketch shapes ----
    SpInit init{};
    init.G = G;
    init.rows = rows;
    // The staged scatter needs the pairs' hashed cells (int32, under 2^31 cells) and the per-(tile,
    // bucket) reservations (under 2^31 pairs).  Both scratch buffers are taken here, before
    // k_sp_plan_edges chooses narrow pairs, so narrow_ok follows what was actually allocated: when
    // either allocation fails the encode takes the rehashing, key-carrying scatter instead of failing.
    const int nbuckets = (int)((cells_max + kMmCellsPerBucket - 1) / kMmCellsPerBucket);
    const bool reserve = (uint64_t)rows * (uint64_t)nnz < (1ull << 31);
    const int64_t mm_tiles = sp_tiles(nnz, mm_chunk(nnz));  // the tiles k_group_prep / the scatter use
    const bool staging = !g_fail_cellbuf.load();
    uint32_t* tile_off =
        reserve && staging ? scratch<uint32_t>(c, kSlotTileOff, (size_t)mm_tiles * (size_t)nbuckets) : nullptr;
    int32_t* cellbuf =
        cells_max < INT32_MAX && staging ? scratch<int32_t>(c, kSlotCellIdx, (size_t)rows * (size_t)nnz) : nullptr;
    init.narrow_ok = mm_scatter_staged(cellbuf != nullptr, tile_off != nullptr, nbuckets) ? 1 : 0;
    init.col_ratio = p->col_ratio;
    for (int g = 0; g < G; g++) pick_hashes(p->hash_seed + g, rows, init.hash_ids[g]);
    SP_TRY(launch_sp_plan_edges(st, s->qpayload, init, s->g_dev));
    const int64_t tiles = sp_tiles(nnz, kSpTile);
    uint64_t* tc = scratch<uint64_t>(c, kSlotTiles, (size_t)(tiles + 1) * G);
    if (!tc) return bail(sfail(SKML_E_OOM, "tile counts"));
    // partition counts; the grid also zeroes the histogram, error flag and bucket counters below
    uint64_t* bucket = scratch<uint64_t>(c, kSlotCells, (size_t)2 * nbuckets + 2);  // counts->bases, cursors
    uint32_t* small = scratch<uint32_t>(c, kSlotSmall, (size_t)kMaxGroups * kDeltaHist + 64);
    if (!bucket || !small) return bail(sfail(SKML_E_OOM, "sparse scratch"));
    SP_TRY(launch_part_count(st, s->qpayload, nnz, s->g_dev, tc, small, (int64_t)kMaxGroups * kDeltaHist + 64, bucket,
                             (int64_t)2 * nbuckets + 2));
    SP_TRY(launch_scan_cols_major(st, tc, tiles, G));
    SP_TRY(launch_sp_plan_groups(st, s->g_dev, tc + tiles, tiles + 1));
    // ---- 3. partition, deltas / histogram / order check, bucketed MinMax insert ----
    int32_t* gk = scratch<int32_t>(c, kSlotGKeys, (size_t)nnz);
    uint16_t* gb = scratch<uint16_t>(c, kSlotGBins, (size_t)nnz);  // grouped bins (< 65536)
    uint8_t* need = scratch<uint8_t>(c, kSlotNeed, (size_t)nnz);
    // reserved ranges are padded to 16 wide (u64) or 32 narrow (u32) pairs
    const size_t npairs = (size_t)rows * (size_t)nnz + (tile_off ? (size_t)15 * mm_tiles * nbuckets : 0);
    const size_t npairs32 = (size_t)rows * (size_t)nnz + (tile_off ? (size_t)31 * mm_tiles * nbuckets : 0);
    uint64_t* pairs = scratch<uint64_t>(c, kSlotDelta, std::max(npairs, (npairs32 + 1) / 2));
    if (!gk || !gb || !need || !pairs) return bail(sfail(SKML_E_OOM, "sparse scratch"));
    uint64_t* cursor = bucket + nbuckets + 1;
    uint32_t* hist = small;
    uint32_t* err = small + kMaxGroups * kDeltaHist;
    SP_TRY(launch_part_scatter(st, keys, s->qpayload, nnz, s->g_dev, tc, gk, gb));
    SP_TRY(launch_group_prep(st, gk, nnz, s->g_dev, need, hist, err, bucket, nbuckets, cellbuf, tile_off));
    // ---- 4. DeltaAdaptive key streams on the side stream, beside the MinMax scatter and minima:
    // the VALU-bound stream writer runs while the scatter waits on memory.  The two chains touch
    // disjoint fields of the group table and disjoint buffers; the main stream joins before the
    // read-back.  (Forking before the count pass instead, with the deltas and histogram computed
    // on the side, overlapped the two VALU-bound passes and was slower.) ----
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipStream_t ds = st;
    if (nnz > 0 && ctx_side_fork(c, &side, &ev_fork, &ev_join) == SKML_OK) {
        SP_TRY(hipEventRecord(ev_fork, st));
        SP_TRY(hipStreamWaitEvent(side, ev_fork, 0));
        ds = side;
    } else {
        side = nullptr;
    }
    if (int e = encode_delta_device(c, ds, s->g_dev, gk, need, nnz, hist, err, s->flag_words, s->delta_words))
        return bail(e);
    // quantValues on the device (only restores read them): on the side chain, off the critical path
    SP_TRY(launch_sp_qvalues(ds, s->qpayload, s->qv_dev));
    if (side) SP_TRY(hipEventRecord(ev_join, side));
    SP_TRY(launch_scan_cols(st, bucket, nbuckets, 1));
    SP_TRY(launch_mm_scatter(st, gk, gb, nnz, s->g_dev, bucket, cursor, nbuckets, pairs, cellbuf, tile_off));
    SP_TRY(launch_mm_bucket(st, pairs, bucket, nbuckets, s->g_dev, s->tables, s->tnar));
    if (side) SP_TRY(hipStreamWaitEvent(st, ev_join, 0));
    // ---- 5. the one read-back: quantizer header and splits, group table ----
    const size_t qh = kHeaderBytes + sizeof(double) * (size_t)(p->bin_num - 1);
    const size_t o_pg = align_up(qh, 256);
    uint8_t* pin = static_cast<uint8_t*>(ctx_pinned(c, o_pg + sizeof(SpGroups)));
    if (!pin) return bail(sfail(SKML_E_OOM, "pinned staging"));
    SP_TRY(hipMemcpyAsync(pin, s->qpayload, qh, hipMemcpyDeviceToHost, st));
    SP_TRY(hipMemcpyAsync(pin + o_pg, s->g_dev, sizeof(SpGroups), hipMemcpyDeviceToHost, st));
    SP_TRY(hipStreamSynchronize(st));
#undef SP_TRY
    std::memcpy(&s->hdr, pin, sizeof(skml_dense_header));
    std::memcpy(&s->g, pin + o_pg, sizeof(SpGroups));
    if (s->hdr.status == SKML_E_NAN || (s->g.status & kSpNan)) return bail(sfail(SKML_E_NAN, "Encounter NaN value"));
    if (s->g.status & kSpEdges) {
        int32_t e_host[kMaxGroups];
        const int e = group_edges(s->hdr.zero_idx, s->hdr.bin_num, G, e_host);
        return bail(e ? e : sfail(SKML_E_HIP, "group plan disagrees with calGroupEdges"));
    }
    if (s->g.status & kSpOrder)
        return bail(sfail(SKML_E_ORDER, "Log for a non-positive key delta (keys must ascend strictly)"));
    {  // Quantizer.getValues (base/Quantizer.java:39-47)
        const int B = s->hdr.bin_num, ns = B - 1;
        const double* sp = reinterpret_cast<const double*>(pin + kHeaderBytes);
        s->splits.assign(sp, sp + std::max(ns, 0));
        s->qvalues.resize((size_t)B);
        for (int b = 0; b < B; b++) {
            double v;
            if (b == 0) v = 0.5 * (s->hdr.min + s->splits[0]);
            else if (b == ns) v = 0.5 * (s->splits[ns - 1] + s->hdr.max);
            else v = 0.5 * (s->splits[b - 1] + s->splits[b]);
            s->qvalues[(size_t)b] = v;
        }
    }
    s->qv_dev_ok = true;
    s->ncells = s->g.ncells;
    s->tnar_width = s->tnar ? tnar_width_for(s->g.bin_num) : 0;
    if (!s->tnar_width) s->tnar = nullptr;
    s->flag_bits = s->g.fb[G];
    s->delta_bits = s->g.db[G];
    s->n_flag_words = (s->flag_bits + 63) / 64 + 1;
    s->n_delta_words = (s->delta_bits + 63) / 64 + 1;
    *out = s;
    return SKML_OK;
}

// DeltaAdaptive decode of all groups + MinMax query: grouped keys/bins into gk/gb.
// DecodeValues: Gradient.sum's restore writes narrow bins (bw bytes: 1 for bin_num <= 256, else 2)
// into gb for the tiled sum, which looks quantValues up itself; a bin outside the nq values sets *err.
// rb: the tiles' run bounds, written by the query too (rb.bounds nullptr: not).
struct DecodeValues {
    int nq;
    void* gb;
    int bw;
    unsigned* err;
    RunBoundsOut rb;
};
int decode_groups(skml_ctx* c, const skml_sparse* s, int32_t* gk, int32_t* gb, bool query,
                  const DecodeValues* dv = nullptr, const RunBoundsOut* rbo = nullptr) {
    hipStream_t st = ctx_stream(c);
    const SpGroups& G = s->g;
    const int64_t n = s->nnz;
    bool any_unary = false;
    for (int g = 0; g < G.G; g++) any_unary |= G.kind[g] && G.gstart[g + 1] > G.gstart[g];
    int64_t* end_pos = nullptr;
    if (any_unary) {
        end_pos = scratch<int64_t>(c, kSlotEndPos, (size_t)n);
        const int64_t wt = sp_tiles(s->n_flag_words, kSpTile);
        uint64_t* ts = scratch<uint64_t>(c, kSlotTiles, (size_t)(wt + 1));
        if (!end_pos || !ts) return sfail(SKML_E_OOM, "decode scratch");
        SP_HIP(launch_unary_count(st, s->flag_words, s->n_flag_words, s->g_dev, ts));
        if (int e = scan_tiles(c, ts, wt, 1, nullptr)) return e;
        SP_HIP(launch_unary_select(st, s->flag_words, s->n_flag_words, s->g_dev, ts, end_pos));
    }
    const int64_t tiles = sp_tiles(n, kSpTile);
    uint64_t* ts = scratch<uint64_t>(c, kSlotTiles, (size_t)(tiles + 1) * 2);
    uint64_t* gpre = scratch<uint64_t>(c, kSlotSmall, kMaxGroups + 8);
    if (!ts || !gpre) return sfail(SKML_E_OOM, "decode scratch");
    uint64_t* ts2 = ts + (tiles + 1);
    uint8_t* dlen = scratch<uint8_t>(c, kSlotNeed, (size_t)n);
    uint32_t* delta = scratch<uint32_t>(c, kSlotDelta, (size_t)n);
    if (!dlen || !delta) return sfail(SKML_E_OOM, "decode scratch");
    // the query gathers from a byte (binNum <= 256) or 16-bit image of the tables, built by extra
    // blocks of the lengths' launch
    const int32_t* tab = query ? s->tables : nullptr;
    int width = 32;
    void* tnar = nullptr;
    if (query && s->tnar && s->ncells > 0) {  // the payload's exact image (encoder or blob): gathered as is
        tab = nullptr;
        width = s->tnar_width;
        tnar = s->tnar;
    } else if (tab && s->ncells > 0 && (reinterpret_cast<uintptr_t>(tab) & 15) == 0) {
        width = G.bin_num <= 256 ? 8 : 16;  // any width gives the same bins (the sentinel reads back)
        tnar = ctx_scratch(c, kSlotNarrowTab, (size_t)s->ncells * (size_t)(width / 8));
        if (!tnar) return sfail(SKML_E_OOM, "decode scratch (table image)");
    }
    // three passes (lengths, their tile scan, deltas); SKML_FORM_DEC_LOOKBACK = 1: one pass with
    // decoupled look-backs for the bit offsets and the deltas' prefixes, 2: the same pass with the
    // deltas' tile scan after it (A/B forms, measured slower: the look-back chain across 13 K tiles
    // ran 230 us against 107 us for the three passes, profiles/ab/r05_dec_lookback.txt)
#ifdef SKML_AB
    const int lb = form(SKML_FORM_DEC_LOOKBACK);
    const int split = lb == 1 ? 0 : lb == 2 ? 2 : 1;
#else
    constexpr int split = 1;
#endif
    if (split == 1) {
        SP_HIP(launch_dec_lens(st, s->flag_words, s->n_flag_words, end_pos, n, s->g_dev, dlen, ts,
                               NarrowJob{tab, s->ncells, tab ? tnar : nullptr, width}));
        if (int e = scan_tiles(c, ts, tiles, 1, nullptr)) return e;
        SP_HIP(launch_dec_deltas(st, s->delta_words, s->n_delta_words, dlen, n, s->g_dev, ts, delta, ts2));
    } else {
#ifdef SKML_AB
        uint64_t* status = scratch<uint64_t>(c, kSlotLookback, 2 * (size_t)tiles + 8);
        if (!status) return sfail(SKML_E_OOM, "decode scratch (look-back)");
        SP_HIP(launch_dec_lens_deltas(st, s->flag_words, s->n_flag_words, end_pos, n, s->g_dev, s->delta_words,
                                      s->n_delta_words, delta, ts2, status, NarrowJob{tab, s->ncells, tab ? tnar : nullptr, width},
                                      split == 0));
#endif
    }
    if (split != 0)
        if (int e = scan_tiles(c, ts2, tiles, 1, nullptr)) return e;
    SP_HIP(launch_group_prefix(st, delta, n, s->g_dev, G.G, ts2, gpre));
    SP_HIP(launch_dec_keys(st, delta, n, s->g_dev, G, ts2, gpre, tab, tnar, width, gk, gb, dv ? dv->nq : 0,
                           dv ? dv->gb : nullptr, dv ? dv->bw : 0, dv ? dv->err : nullptr,
                           dv ? dv->rb : rbo ? *rbo : RunBoundsOut{nullptr, 0, 0, 0}));
    return SKML_OK;
}

// Sort.merge (util/Sort.java:362-379) of the groups' (key, bin) runs: rounds of pairwise stable
// merges on the device; keys and bins land in keys_out / bins_out.
int merge_groups(skml_ctx* c, const skml_sparse* s, int32_t* gk, int32_t* gb, int32_t* keys_out,
                 int32_t* bins_out) {
    hipStream_t st = ctx_stream(c);
    const int64_t n = s->nnz;
    const SpGroups& G = s->g;
    int32_t* k1 = scratch<int32_t>(c, kSlotK1, (size_t)n);
    int32_t* b1 = scratch<int32_t>(c, kSlotB1, (size_t)n);
    if (!k1 || !b1) return sfail(SKML_E_OOM, "merge scratch");
    // every round's run offsets (the rounds halve the run count) go to the kernels by value
    std::vector<int64_t> rs(G.gstart, G.gstart + G.G + 1);
    int64_t* split = rs.size() > 2 ? scratch<int64_t>(c, kSlotEndPos, (size_t)sp_tiles(n, kSpTile) + 2) : nullptr;
    if (rs.size() > 2 && !split) return sfail(SKML_E_OOM, "merge split points");
    int32_t *kin = gk, *bin = gb, *kout = k1, *bout = b1;
    // the last round writes straight into the outputs (bins too unless bins_out is a scratch buffer)
    const bool bins_direct = bins_out && bins_out != gb && bins_out != b1;
    bool keys_done = false, bins_done = false;
    while (rs.size() > 2) {
        const bool last = rs.size() <= 3;
        int32_t* ko = last ? keys_out : kout;
        int32_t* bo = last && bins_direct ? bins_out : bout;
        SP_HIP(launch_merge_round(st, kin, bin, ko, bo, rs.data(), (int)rs.size() - 1, n, split));
        std::vector<int64_t> nx;
        for (size_t i = 0; i < rs.size(); i += 2) nx.push_back(rs[i]);
        if (nx.back() != rs.back()) nx.push_back(rs.back());
        rs.swap(nx);
        keys_done = last;
        bins_done = last && bins_direct;
        kin = ko;
        bin = bo;
        kout = kin == k1 ? gk : k1;
        bout = bin == b1 ? gb : b1;
    }
    if (!keys_done) SP_HIP(hipMemcpyAsync(keys_out, kin, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToDevice, st));
    if (!bins_done && bins_out && bins_out != bin)
        SP_HIP(hipMemcpyAsync(bins_out, bin, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToDevice, st));
    return SKML_OK;
}

thread_local int t_merge_path = 0;  // skml_debug_sparse_merge_path

// Sort.merge's one-pass form: its scratch (RsInfo + the runs' key-range bounds) taken and RsInfo
// zeroed up front, so the fill runs while the restore's first kernels are still being queued;
// m->info stays nullptr when the one-pass form will not run (one run, or the rounds forced through
// skml_debug_form).
struct RsMerge {
    RsInfo* info = nullptr;
    int32_t* bounds = nullptr;
    bool by_query = false;  // the key query writes the bounds (query_bounds); else k_rs_bounds
    RunBoundsOut query_bounds() {
        by_query = info && form(SKML_FORM_RUN_BOUNDS) != 1;
        return RunBoundsOut{by_query ? bounds : nullptr, 0, 0, kRsBits, info};
    }
};
int rs_merge_prepare(skml_ctx* c, const skml_sparse* s, RsMerge* m) {
    *m = RsMerge{};
    if (s->g.G < 2 || form(SKML_FORM_RS_ROUNDS) == 1) return SKML_OK;
    const size_t o_b = align_up(sizeof(RsInfo), 256);
    char* blk = static_cast<char*>(
        ctx_scratch(c, kSlotRsMerge, o_b + sizeof(int32_t) * (size_t)s->g.G * (size_t)(kRsRanges + 1)));
    if (!blk) return sfail(SKML_E_OOM, "merge scratch");
    SP_HIP(hipMemsetAsync(blk, 0, o_b, ctx_stream(c)));  // whole 256-byte units: one fill
    m->info = reinterpret_cast<RsInfo*>(blk);
    m->bounds = reinterpret_cast<int32_t*>(blk + o_b);
    return SKML_OK;
}
// The one-pass merge (launch_rs_merge) into keys_out and out (vkind: 0 int32 bins, 1 float / 2
// double quantValues[bin]).  *pending: a pinned word that is non-zero after the stream
// synchronises if the input was not regular (or held a bin outside quantValues) and merge_groups
// must run instead; nullptr when the one-pass form did not run.
int rs_merge_start(skml_ctx* c, const skml_sparse* s, const RsMerge& m, const int32_t* gk, const int32_t* gb,
                   int32_t* keys_out, void* out, int vkind, const double* qv, int nq, volatile unsigned** pending) {
    *pending = nullptr;
    if (!m.info) return SKML_OK;
    hipStream_t st = ctx_stream(c);
    unsigned* pin = static_cast<unsigned*>(ctx_pinned(c, 64));
    if (!pin) return sfail(SKML_E_OOM, "merge scratch");
    SP_HIP(launch_rs_merge(st, gk, gb, s->nnz, s->g_dev, m.bounds, m.info, keys_out, out, vkind, qv, nq, m.by_query));
    SP_HIP(hipMemcpyAsync(pin, &m.info->irregular, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    *pending = pin;
    return SKML_OK;
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {
// poll: the count goes to the context's host word and the call returns as soon as it is there,
// with the kernel's last stores possibly still in flight -- only for callers whose next work
// runs on the same stream (skml_sparse_encode_*); the public compaction synchronises.
template <typename T>
int compact_any(skml_ctx* c, const T* dense, int64_t dim, int32_t* keys, T* vals, int64_t* nnz_out,
                bool poll = false) {
    if (!c || !nnz_out || dim < 0 || (dim > 0 && (!dense || !keys || !vals)))
        return sfail(SKML_E_ARG, "bad compaction arguments");
    if (dim > (int64_t)INT32_MAX) return sfail(SKML_E_ARG, "dim %lld exceeds Java int keys", (long long)dim);
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    const int64_t tiles = sp_tiles(dim, sizeof(T) == 8 ? kCompactTile / 2 : kCompactTile);
    uint64_t* status = scratch<uint64_t>(c, kSlotStatus, (size_t)tiles + 8);
    if (!status) return sfail(SKML_E_OOM, "compaction status");
    unsigned* ticket = reinterpret_cast<unsigned*>(status + tiles);
    int64_t* nnz_dev = reinterpret_cast<int64_t*>(status + tiles + 1);
    int64_t* hw = poll && tiles > 0 ? ctx_host_word(c) : nullptr;
    if (hw) *reinterpret_cast<volatile int64_t*>(hw) = -1;
    SP_HIP(hipMemsetAsync(status, 0, sizeof(uint64_t) * ((size_t)tiles + 8), st));
    int64_t* dst = hw ? hw : nnz_dev;
    if constexpr (sizeof(T) == 8) SP_HIP(launch_compact64(st, dense, dim, keys, vals, status, ticket, dst));
    else SP_HIP(launch_compact(st, dense, dim, keys, vals, status, ticket, dst));
    if (hw) return wait_host_count(c, hw, nnz_out);
    return sync_to_host(c, nnz_out, nnz_dev, sizeof(int64_t));
}
}  // namespace

extern "C" {

int skml_sparse_compact_f32(skml_ctx* c, const float* dense, int64_t dim, int32_t* keys, float* vals,
                            int64_t* nnz_out) {
    return compact_any<float>(c, dense, dim, keys, vals, nnz_out);
}

int skml_sparse_compact_f64(skml_ctx* c, const double* dense, int64_t dim, int32_t* keys, double* vals,
                            int64_t* nnz_out) {
    return compact_any<double>(c, dense, dim, keys, vals, nnz_out);
}

int skml_sparse_encode_kv_f32(skml_ctx* c, const int32_t* keys, const float* vals, int64_t nnz,
                              const skml_params* p, skml_sparse** out) {
    if (!c || !out || nnz < 0 || (nnz > 0 && (!keys || !vals))) return sfail(SKML_E_ARG, "bad sparse arguments");
    if (nnz > (int64_t)INT32_MAX) return sfail(SKML_E_ARG, "nnz exceeds Java int");
    if (int e = check_params(p)) return e;
    SP_HIP(hipSetDevice(ctx_device(c)));
    *out = nullptr;
    return encode_kv(c, keys, vals, false, nnz, p, out);
}

int skml_sparse_encode_kv_f64(skml_ctx* c, const int32_t* keys, const double* vals, int64_t nnz,
                              const skml_params* p, skml_sparse** out) {
    if (!c || !out || nnz < 0 || (nnz > 0 && (!keys || !vals))) return sfail(SKML_E_ARG, "bad sparse arguments");
    if (nnz > (int64_t)INT32_MAX) return sfail(SKML_E_ARG, "nnz exceeds Java int");
    if (int e = check_params(p)) return e;
    SP_HIP(hipSetDevice(ctx_device(c)));
    *out = nullptr;
    return encode_kv(c, keys, vals, true, nnz, p, out);
}

int skml_sparse_encode_f32(skml_ctx* c, const float* dense, int64_t dim, const skml_params* p,
                           skml_sparse** out) {
    if (!c || !out || dim < 0) return sfail(SKML_E_ARG, "bad sparse arguments");
    if (int e = check_params(p)) return e;
    SP_HIP(hipSetDevice(ctx_device(c)));
    const size_t cap = (size_t)std::max<int64_t>(dim, 1);
    int32_t* keys = scratch<int32_t>(c, kSlotCKeys, cap);
    float* vals = scratch<float>(c, kSlotCVals, cap);
    if (!keys || !vals) return sfail(SKML_E_OOM, "compaction output");
    int64_t nnz = 0;
    if (int e = compact_any<float>(c, dense, dim, keys, vals, &nnz, true)) return e;
    return encode_kv(c, keys, vals, false, nnz, p, out);
}

int skml_sparse_encode_f64(skml_ctx* c, const double* dense, int64_t dim, const skml_params* p,
                           skml_sparse** out) {
    if (!c || !out || dim < 0) return sfail(SKML_E_ARG, "bad sparse arguments");
    if (int e = check_params(p)) return e;
    SP_HIP(hipSetDevice(ctx_device(c)));
    const size_t cap = (size_t)std::max<int64_t>(dim, 1);
    int32_t* keys = scratch<int32_t>(c, kSlotCKeys, cap);
    double* vals = scratch<double>(c, kSlotCVals, cap);
    if (!keys || !vals) return sfail(SKML_E_OOM, "compaction output");
    int64_t nnz = 0;
    if (int e = compact_any<double>(c, dense, dim, keys, vals, &nnz, true)) return e;
    return encode_kv(c, keys, vals, true, nnz, p, out);
}

}  // extern "C"

namespace {
// restore + Sort.merge + quantValues[bin] (SparseVectorCompressor.decompressSparse,
// SparseVectorCompressor.java:118-126) as fp32 or as the reference's doubles
template <typename T>
int decode_values(skml_ctx* c, const skml_sparse* s, int32_t* keys_dev, T* vals_dev) {
    if (!c || !s) return sfail(SKML_E_ARG, "bad decode arguments");
    const int64_t n = s->nnz;
    if (n == 0) return SKML_OK;
    if (!keys_dev || !vals_dev) return sfail(SKML_E_ARG, "keys/vals are NULL");
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    if (s->qvalues.empty()) return sfail(SKML_E_STATE, "quantValues are not set (deserialised without them)");
    int32_t* gk = scratch<int32_t>(c, kSlotGKeys, (size_t)n);
    int32_t* gb = scratch<int32_t>(c, kSlotGBins, (size_t)n);
    int32_t* b1 = scratch<int32_t>(c, kSlotB1, (size_t)n);
    if (!gk || !gb || !b1) return sfail(SKML_E_OOM, "decode scratch");
    // the value table's upload and the merge's RsInfo fill go first: the GPU runs them while the
    // decode's kernels are still being queued
    const int nq = (int)s->qvalues.size();
    double* qv = s->qv_dev;  // the payload's device copy (encode / import), or the host table uploaded
    if (!qv || !s->qv_dev_ok) {
        if (!qv) qv = reinterpret_cast<double*>(ctx_scratch(c, kSlotCells, sizeof(double) * s->qvalues.size()));
        if (!qv) return sfail(SKML_E_OOM, "value table");
        SP_HIP(hipMemcpyAsync(qv, s->qvalues.data(), sizeof(double) * s->qvalues.size(), hipMemcpyHostToDevice, st));
        if (qv == s->qv_dev) const_cast<skml_sparse*>(s)->qv_dev_ok = true;  // ordered before later restores
    }
    RsMerge rm;
    if (int e = rs_merge_prepare(c, s, &rm)) return e;
    const RunBoundsOut rbo = rm.query_bounds();  // the merge's key-range bounds from the query
    if (int e = decode_groups(c, s, gk, gb, true, nullptr, &rbo)) return e;
    // pairwise merge rounds, then quantValues[bin]; a bin outside the nq values (Java: index out
    // of bounds) fails the decode (the one-pass merge sends such input here too)
    auto rounds = [&]() -> int {
        unsigned* err = scratch<unsigned>(c, kSlotStatus, 64);
        if (!err) return sfail(SKML_E_OOM, "decode scratch");
        SP_HIP(hipMemsetAsync(err, 0, sizeof(unsigned), st));
        if (int e = merge_groups(c, s, gk, gb, keys_dev, b1)) return e;
        if constexpr (sizeof(T) == 8) SP_HIP(launch_bin_values64(st, b1, n, qv, nq, vals_dev, err));
        else SP_HIP(launch_bin_values(st, b1, n, qv, nq, vals_dev, err));
        unsigned bad = 0;
        if (int e = sync_to_host(c, &bad, err, sizeof(bad))) return e;
        return bad ? sfail(SKML_E_ARG, "a restored bin lies outside the %d quantValues", nq) : SKML_OK;
    };
    volatile unsigned* pending = nullptr;
    if (int e = rs_merge_start(c, s, rm, gk, gb, keys_dev, vals_dev, sizeof(T) == 8 ? 2 : 1, qv, nq, &pending))
        return e;
    if (!pending) {
        t_merge_path = s->g.G < 2 ? 0 : 2;
        return rounds();
    }
    SP_HIP(hipStreamSynchronize(st));
    t_merge_path = 1;
    if (*pending) {  // not regular, or a bin outside quantValues: the rounds decide
        t_merge_path = 3;
        return rounds();
    }
    return SKML_OK;
}
}  // namespace

extern "C" {

int skml_sparse_decode_f32(skml_ctx* c, const skml_sparse* s, int32_t* keys_dev, float* vals_dev) {
    return decode_values<float>(c, s, keys_dev, vals_dev);
}

int skml_sparse_decode_f64(skml_ctx* c, const skml_sparse* s, int32_t* keys_dev, double* vals_dev) {
    return decode_values<double>(c, s, keys_dev, vals_dev);
}

int skml_sparse_times_by(skml_sparse* s, double x) {
    if (!s) return sfail(SKML_E_ARG, "NULL argument");
    for (double& v : s->qvalues) v *= x;  // SparseVectorCompressor.timesBy (:128-134)
    s->qv_dev_ok = false;  // the device copy is re-uploaded by the next restore
    return SKML_OK;
}

int skml_sparse_values(const skml_sparse* s, double* out, int32_t cap) {
    if (!s || !out) return sfail(SKML_E_ARG, "NULL argument");
    const size_t k = std::min<size_t>(s->qvalues.size(), (size_t)std::max(cap, 0));
    std::memcpy(out, s->qvalues.data(), sizeof(double) * k);
    return SKML_OK;
}

int skml_sparse_nnz(const skml_sparse* s, int64_t* nnz) {
    if (!s || !nnz) return sfail(SKML_E_ARG, "NULL argument");
    *nnz = s->nnz;
    return SKML_OK;
}

int skml_sparse_quant_info(const skml_sparse* s, skml_dense_header* hdr, double* splits_host, int32_t cap) {
    if (!s || !hdr) return sfail(SKML_E_ARG, "NULL argument");
    *hdr = s->hdr;
    if (splits_host) {
        const size_t k = std::min<size_t>(s->splits.size(), (size_t)std::max(cap, 0));
        std::memcpy(splits_host, s->splits.data(), sizeof(double) * k);
    }
    return SKML_OK;
}

// Copy bits [b0, b0 + nbits) of a device word stream into host words starting at bit 0.
static int extract_bits(skml_ctx* c, const uint64_t* words, int64_t b0, int64_t nbits, uint64_t* out) {
    const int64_t nw = (nbits + 63) / 64;
    if (nw == 0) return SKML_OK;
    const int64_t w0 = b0 >> 6, w1 = (b0 + nbits - 1) >> 6;
    std::vector<uint64_t> buf((size_t)(w1 - w0 + 2), 0);
    if (int e = sync_to_host(c, buf.data(), words + w0, sizeof(uint64_t) * (size_t)(w1 - w0 + 1))) return e;
    const int sh = (int)(b0 & 63);
    for (int64_t i = 0; i < nw; i++) {
        uint64_t v = buf[(size_t)i] >> sh;
        if (sh) v |= buf[(size_t)i + 1] << (64 - sh);
        out[i] = v;
    }
    const int tail = (int)(nbits & 63);
    if (tail) out[nw - 1] &= (1ULL << tail) - 1ULL;
    return SKML_OK;
}

int skml_sparse_group_info(skml_ctx* c, const skml_sparse* s, int32_t g, skml_sparse_group* info,
                           int32_t* table_host, uint64_t* flag_words_host, uint64_t* delta_words_host) {
    if (!c || !s || !info || g < 0 || g >= s->g.G) return sfail(SKML_E_ARG, "bad group query");
    SP_HIP(hipSetDevice(ctx_device(c)));
    const SpGroups& G = s->g;
    std::memset(info, 0, sizeof(*info));
    info->size = (int32_t)(G.gstart[g + 1] - G.gstart[g]);
    if (info->size == 0) return SKML_OK;  // null sketch / encoder (GroupedMinMaxSketch.java:105-109)
    info->col_num = G.cols[g];
    for (int r = 0; r < G.rows; r++) info->hash_ids[r] = G.hash_ids[g][r];
    info->num_intervals = G.m[g];
    info->flag_kind = G.kind[g];
    info->n_flag_bits = G.fb[g + 1] - G.fb[g];
    info->n_delta_bits = G.db[g + 1] - G.db[g];
    if (table_host)
        if (int e = sync_to_host(c, table_host, s->tables + G.tab_off[g], sizeof(int32_t) * (size_t)G.rows * G.cols[g]))
            return e;
    if (flag_words_host)
        if (int e = extract_bits(c, s->flag_words, G.fb[g], info->n_flag_bits, flag_words_host)) return e;
    if (delta_words_host)
        if (int e = extract_bits(c, s->delta_words, G.db[g], info->n_delta_bits, delta_words_host)) return e;
    return SKML_OK;
}

// Per-group HuffmanEncoder of the MinMaxSketch tables: device histograms, host trees, device
// code stream (cached in the payload).
static int build_huffman(skml_ctx* c, skml_sparse* s) {
    if (s->huff_done) return SKML_OK;
    hipStream_t st = ctx_stream(c);
    const SpGroups& G = s->g;
    const int B = G.bin_num;
    const size_t nsym = (size_t)B + 1;
    s->huff_items.assign((size_t)G.G, {});
    s->huff_bit0.assign((size_t)G.G + 1, 0);
    s->huff_bits.assign((size_t)G.G, 0);
    if (s->ncells > 0) {
        int64_t max_cells = 0;
        for (int g = 0; g < G.G; g++)
            if (G.gstart[g + 1] > G.gstart[g]) max_cells = std::max<int64_t>(max_cells, (int64_t)G.rows * G.cols[g]);
        uint32_t* hist = scratch<uint32_t>(c, kSlotDelta, (size_t)G.G * nsym);
        uint64_t* lut = scratch<uint64_t>(c, kSlotCells, (size_t)G.G * nsym);
        if (!hist || !lut) return sfail(SKML_E_OOM, "huffman scratch");
        SP_HIP(hipMemsetAsync(hist, 0, sizeof(uint32_t) * (size_t)G.G * nsym, st));
        SP_HIP(launch_huff_hist(st, s->tables, s->g_dev, G.G, B, max_cells, hist));
        std::vector<uint32_t> hh((size_t)G.G * nsym);
        if (int e = sync_to_host(c, hh.data(), hist, sizeof(uint32_t) * hh.size())) return e;
        std::vector<uint64_t> lh((size_t)G.G * nsym, 0);
        HuffBuilder hb;
        int64_t bit = 0;
        for (int g = 0; g < G.G; g++) {
            s->huff_bit0[(size_t)g] = bit;
            if (G.gstart[g + 1] == G.gstart[g]) continue;
            std::vector<std::pair<int32_t, int64_t>> syms;
            const uint32_t* h = hh.data() + (size_t)g * nsym;
            if (G.fill < 0 && h[B]) syms.emplace_back(G.fill, h[B]);  // ascending signed order
            for (int v = 0; v < B; v++)
                if (h[v]) syms.emplace_back(v, h[v]);
            if (G.fill >= 0 && h[B]) syms.emplace_back(G.fill, h[B]);
            if (!hb.build(syms, s->huff_items[(size_t)g]))
                return sfail(SKML_E_STATE, "Huffman code longer than 32 bits (group %d)", g);
            for (const HuffItem& it : s->huff_items[(size_t)g]) {
                const int sym = (it.value >= 0 && it.value < B) ? it.value : B;
                lh[(size_t)g * nsym + sym] = ((uint64_t)it.nbits << 32) | (uint32_t)it.bits;
                s->huff_bits[(size_t)g] += (int64_t)it.nbits * h[sym];
            }
            bit += s->huff_bits[(size_t)g];
        }
        s->huff_bit0[(size_t)G.G] = bit;
        SP_HIP(hipMemcpyAsync(lut, lh.data(), sizeof(uint64_t) * lh.size(), hipMemcpyHostToDevice, st));
        const int64_t tiles = sp_tiles(s->ncells, kSpTile);
        uint64_t* ts = scratch<uint64_t>(c, kSlotTiles, (size_t)tiles + 1);
        int64_t* gbit = scratch<int64_t>(c, kSlotSmall, kMaxGroups + 1);
        if (!ts || !gbit) return sfail(SKML_E_OOM, "huffman scratch");
        SP_HIP(launch_huff_lens(st, s->tables, s->ncells, s->g_dev, B, lut, ts));
        uint64_t total = 0;
        if (int e = scan_tiles(c, ts, tiles, 1, &total)) return e;
        if ((int64_t)total != bit) return sfail(SKML_E_STATE, "huffman bit count mismatch");
        s->n_huff_words = (bit + 63) / 64 + 1;
        SP_HIP(hipMalloc(&s->huff_words, sizeof(uint64_t) * (size_t)s->n_huff_words));
        SP_HIP(hipMemsetAsync(s->huff_words, 0, sizeof(uint64_t) * (size_t)s->n_huff_words, st));
        SP_HIP(launch_huff_write(st, s->tables, s->ncells, s->g_dev, B, lut, ts, s->huff_words, gbit));
        SP_HIP(hipStreamSynchronize(st));
    }
    s->huff_done = true;
    return SKML_OK;
}

namespace {
// Host layout of the field stream: small fields are appended to `small` and form pieces of the
// stream; a long array leaves a gap of 8 * nwords bytes that k_wire_longs fills on the device.
struct WireBuilder {
    std::vector<uint8_t> small;
    std::vector<int64_t> pieces;  // {small offset, stream offset, length} triples
    int64_t total = 0;
    bool open = false;
    void put(uint64_t v, int n) {
        if (!open) {
            pieces.push_back((int64_t)small.size());
            pieces.push_back(total);
            pieces.push_back(0);
            open = true;
        }
        for (int i = n - 1; i >= 0; i--) small.push_back((uint8_t)(v >> (8 * i)));
        pieces.back() += n;
        total += n;
    }
    void i32(int32_t v) { put((uint32_t)v, 4); }
    void f64(double d) {
        uint64_t x;
        std::memcpy(&x, &d, 8);
        put(x, 8);
    }
    void byte(int v) { put((uint8_t)v, 1); }
    int64_t gap(int64_t bytes) {  // returns the gap's stream offset
        open = false;
        const int64_t at = total;
        total += bytes;
        return at;
    }
};

// The device field stream of a payload (cached in s->wire_dev): Huffman codes of the tables,
// the trims of every long array (one small read-back), the layout on the host, then two kernels.
int build_wire(skml_ctx* c, skml_sparse* s) {
    if (int e = build_huffman(c, s)) return e;
    hipStream_t st = ctx_stream(c);
    const SpGroups& G = s->g;
    static const int32_t kBkdrSeed[8] = {0, 0, 0, 31, 131, 267, 1313, 13131};
    // the long arrays in stream order: every present sketch's Huffman words, then every present
    // encoder's flag and delta words
    std::vector<WireSec> secs;
    std::vector<int> present;
    for (int g = 0; g < G.G; g++)
        if (G.gstart[g + 1] > G.gstart[g]) present.push_back(g);
    for (int g : present) secs.push_back(WireSec{0, s->huff_bit0[(size_t)g], s->huff_bits[(size_t)g], 0, 2, 0});
    for (int g : present) {
        secs.push_back(WireSec{0, G.fb[g], G.fb[g + 1] - G.fb[g], 0, 0, 0});
        secs.push_back(WireSec{0, G.db[g], G.db[g + 1] - G.db[g], 0, 1, 0});
    }
    const int nsec = (int)secs.size();
    std::vector<int64_t> wpre((size_t)nsec + 1, 0);
    for (int k = 0; k < nsec; k++) wpre[(size_t)k + 1] = wpre[(size_t)k] + (secs[(size_t)k].nbits + 63) / 64;
    const WireSrc src{s->flag_words, s->delta_words, s->huff_words};
    // section tables and the trims in one scratch block: secs | wpre | nz | npre
    const size_t o_pre = align_up(sizeof(WireSec) * (size_t)std::max(nsec, 1), 256);
    const size_t o_nz = o_pre + align_up(sizeof(int64_t) * ((size_t)nsec + 1), 256);
    const size_t o_npre = o_nz + align_up(sizeof(uint64_t) * (size_t)std::max(nsec, 1), 256);
    const size_t meta_bytes = o_npre + sizeof(int64_t) * ((size_t)nsec + 1);
    uint8_t* meta = scratch<uint8_t>(c, kSlotWireMeta, meta_bytes);
    if (!meta) return sfail(SKML_E_OOM, "wire scratch");
    WireSec* d_secs = reinterpret_cast<WireSec*>(meta);
    int64_t* d_pre = reinterpret_cast<int64_t*>(meta + o_pre);
    uint64_t* d_nz = reinterpret_cast<uint64_t*>(meta + o_nz);
    int64_t* d_npre = reinterpret_cast<int64_t*>(meta + o_npre);
    std::vector<uint64_t> nz((size_t)nsec, 0);
    if (nsec > 0) {
        SP_HIP(hipMemcpyAsync(d_secs, secs.data(), sizeof(WireSec) * (size_t)nsec, hipMemcpyHostToDevice, st));
        SP_HIP(hipMemcpyAsync(d_pre, wpre.data(), sizeof(int64_t) * wpre.size(), hipMemcpyHostToDevice, st));
        SP_HIP(hipMemsetAsync(d_nz, 0, sizeof(uint64_t) * (size_t)nsec, st));
        SP_HIP(launch_wire_lastnz(st, src, d_secs, nsec, d_nz));
        if (int e = sync_to_host(c, nz.data(), d_nz, sizeof(uint64_t) * (size_t)nsec)) return e;
    }
    // the layout (GroupedMinMaxSketch.writeObject field order, see skml_sparse_serialize)
    WireBuilder w;
    w.i32(G.G);
    w.i32(G.rows);
    w.f64(s->params.col_ratio);
    w.i32(G.bin_num);
    w.i32(G.zero);
    int k = 0;
    for (int g = 0; g < G.G; g++) {  // sketches
        const bool pres = G.gstart[g + 1] > G.gstart[g];
        w.byte(pres ? 1 : 0);
        if (!pres) continue;
        w.i32(G.rows);
        w.i32(G.cols[g]);
        w.i32(G.zero);
        for (int r = 0; r < G.rows; r++) {
            w.i32(G.hash_ids[g][r]);
            w.i32(G.cols[g]);
            w.i32(kBkdrSeed[G.hash_ids[g][r] & 7]);
        }
        const auto& items = s->huff_items[(size_t)g];
        w.i32((int32_t)items.size());
        for (const HuffItem& it : items) {
            w.i32(it.value);
            w.i32(it.bits);
            w.i32(it.nbits);
        }
        WireSec& sc = secs[(size_t)k++];
        sc.nwords = (int64_t)nz[(size_t)(&sc - secs.data())];
        w.i32((int32_t)sc.nwords);
        sc.dst = w.gap(8 * sc.nwords);
        w.i32(G.rows * G.cols[g]);
    }
    for (int g = 0; g < G.G; g++) {  // encoders
        const bool pres = G.gstart[g + 1] > G.gstart[g];
        w.byte(pres ? 1 : 0);
        if (!pres) continue;
        w.i32((int32_t)(G.gstart[g + 1] - G.gstart[g]));
        w.i32(G.m[g]);
        w.byte(G.kind[g] ? 1 : 0);
        for (int t = 0; t < 2; t++) {
            WireSec& sc = secs[(size_t)k];
            sc.nwords = (int64_t)nz[(size_t)k];
            k++;
            w.i32((int32_t)sc.nwords);
            sc.dst = w.gap(8 * sc.nwords);
        }
    }
    std::vector<int64_t> npre((size_t)nsec + 1, 0);
    for (int q = 0; q < nsec; q++) npre[(size_t)q + 1] = npre[(size_t)q] + secs[(size_t)q].nwords;
    // the stream: the small fields' pieces, then the long arrays
    void* wire = nullptr;
    SP_HIP(hipMalloc(&wire, (size_t)std::max<int64_t>(w.total, 1)));
    const int npieces = (int)(w.pieces.size() / 3);
    const size_t o_pcs = align_up(w.small.size(), 256);
    uint8_t* sm = scratch<uint8_t>(c, kSlotSmall, o_pcs + sizeof(int64_t) * w.pieces.size() + 8);
    if (!sm) {
        (void)hipFree(wire);
        return sfail(SKML_E_OOM, "wire scratch");
    }
    auto fail_free = [&](int e) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(wire);
        return e;
    };
#define W_HIP(expr)                                                                                         \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess) return fail_free(sfail(SKML_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_))); \
    } while (0)
    if (!w.small.empty()) W_HIP(hipMemcpyAsync(sm, w.small.data(), w.small.size(), hipMemcpyHostToDevice, st));
    if (npieces > 0)
        W_HIP(hipMemcpyAsync(sm + o_pcs, w.pieces.data(), sizeof(int64_t) * w.pieces.size(), hipMemcpyHostToDevice, st));
    if (nsec > 0) {
        W_HIP(hipMemcpyAsync(d_secs, secs.data(), sizeof(WireSec) * (size_t)nsec, hipMemcpyHostToDevice, st));
        W_HIP(hipMemcpyAsync(d_npre, npre.data(), sizeof(int64_t) * npre.size(), hipMemcpyHostToDevice, st));
    }
    W_HIP(launch_wire_pieces(st, sm, reinterpret_cast<const int64_t*>(sm + o_pcs), npieces, static_cast<uint8_t*>(wire)));
    if (nsec > 0) W_HIP(launch_wire_longs(st, src, d_secs, d_npre, nsec, npre.back(), static_cast<uint8_t*>(wire)));
    W_HIP(hipStreamSynchronize(st));  // the host vectors above are the copies' sources
#undef W_HIP
    s->wire_dev = wire;
    s->wire_bytes = (size_t)w.total;
    return SKML_OK;
}
}  // namespace

// GroupedMinMaxSketch.writeObject field order (GroupedMinMaxSketch.java:148-158) with
// MinMaxSketch.writeObject (MinMaxSketch.java:88-97), HuffmanEncoder.writeObject
// (HuffmanEncoder.java:168-190) and DeltaAdaptiveEncoder.writeObject (:148-170); big-endian
// DataOutput primitives; a 1-byte presence flag stands where Java writes a null object, and each
// Int2IntHash object is (int HashFactory index, int size, int BKDR seed or 0).  Assembled on the
// device (skml_wire.hip) and copied out once.
int skml_sparse_serialize(skml_ctx* c, const skml_sparse* cs, uint8_t* buf, size_t cap, size_t* written) {
    if (!c || !cs) return sfail(SKML_E_ARG, "bad serialise arguments");
    SP_HIP(hipSetDevice(ctx_device(c)));
    skml_sparse* s = const_cast<skml_sparse*>(cs);  // the Huffman streams and the wire are lazily built caches
    if (!s->wire_dev)
        if (int e = build_wire(c, s)) return e;
    if (written) *written = s->wire_bytes;
    if (!buf) return SKML_OK;
    if (cap < s->wire_bytes) return sfail(SKML_E_ARG, "buffer capacity %zu < %zu", cap, s->wire_bytes);
    SP_HIP(hipMemcpyAsync(buf, s->wire_dev, s->wire_bytes, hipMemcpyDeviceToHost, ctx_stream(c)));
    SP_HIP(hipStreamSynchronize(ctx_stream(c)));
    return SKML_OK;
}

namespace {
struct BeReader {
    const uint8_t* p;
    size_t n, i = 0;
    bool bad = false;
    uint64_t u(int k) {
        if (i + (size_t)k > n) {
            bad = true;
            i = n;
            return 0;
        }
        uint64_t v = 0;
        for (int j = 0; j < k; j++) v = (v << 8) | p[i++];
        return v;
    }
    int32_t i32() { return (int32_t)(uint32_t)u(4); }
    int64_t i64() { return (int64_t)u(8); }
    double f64() {
        const uint64_t x = u(8);
        double d;
        std::memcpy(&d, &x, 8);
        return d;
    }
    int byte() { return (int)u(1); }
    // a long[] body: its byte position, the contents stay in the stream (read on the device)
    bool skip_longs(size_t count, int64_t* pos) {
        if (count > (n - i) / 8) {
            bad = true;
            i = n;
            return false;
        }
        *pos = (int64_t)i;
        i += 8 * count;
        return true;
    }
};

struct HuffGroupIn {
    std::vector<HuffItem> items;
    int64_t pos = 0, nlongs = 0;  // the HuffmanEncoder's long[] in the stream
    int64_t size = 0;
};

// Decode tables of one group's HuffmanEncoder items (HuffmanEncoder.java:131-152 builds the same
// tree): codes of <= kHuffLutBits bits fill their LUT ranges, longer codes end in tree nodes.
int huff_tables(const std::vector<HuffItem>& items, int node_base, std::vector<int2>& lut,
                std::vector<int4>& nodes) {
    struct N {
        int left = -1, right = -1, value = 0;
        bool leaf = false;
    };
    const size_t l0 = lut.size();
    lut.resize(l0 + kHuffLutSize, int2{0, 0});
    std::vector<char> set(kHuffLutSize, 0);
    std::vector<int> prefix_node(kHuffLutSize, -1);  // subtree root of a long-code prefix
    std::vector<N> t;
    for (const HuffItem& it : items) {
        if (it.nbits <= 0 || it.nbits > 31) return sfail(SKML_E_ARG, "Huffman code of %d bits", it.nbits);
        const uint32_t code = (uint32_t)it.bits;
        if (it.nbits <= kHuffLutBits) {
            const uint32_t lo = code << (kHuffLutBits - it.nbits), hi = (code + 1) << (kHuffLutBits - it.nbits);
            if (hi > (uint32_t)kHuffLutSize) return sfail(SKML_E_ARG, "Huffman code wider than its length");
            for (uint32_t k = lo; k < hi; k++) {
                if (set[k]) return sfail(SKML_E_ARG, "Huffman codes are not prefix-free");
                set[k] = 1;
                lut[l0 + k] = int2{it.value, it.nbits};
            }
            continue;
        }
        const uint32_t pre = code >> (it.nbits - kHuffLutBits);
        if (pre >= (uint32_t)kHuffLutSize) return sfail(SKML_E_ARG, "Huffman code wider than its length");
        int node = prefix_node[pre];
        if (node < 0) {
            if (set[pre]) return sfail(SKML_E_ARG, "Huffman codes are not prefix-free");
            node = (int)t.size();
            t.push_back(N());
            prefix_node[pre] = node;
            set[pre] = 1;
            lut[l0 + pre] = int2{node_base + node, -1};
        }
        for (int b = it.nbits - kHuffLutBits - 1; b >= 0; b--) {
            if (t[(size_t)node].leaf) return sfail(SKML_E_ARG, "Huffman codes are not prefix-free");
            const bool one = (code >> b) & 1u;
            int child = one ? t[(size_t)node].right : t[(size_t)node].left;
            if (child < 0) {
                child = (int)t.size();
                t.push_back(N());
                if (one) t[(size_t)node].right = child;
                else t[(size_t)node].left = child;
            }
            node = child;
        }
        N& leaf = t[(size_t)node];
        if (leaf.leaf || leaf.left >= 0 || leaf.right >= 0) return sfail(SKML_E_ARG, "Huffman codes are not prefix-free");
        leaf.leaf = true;
        leaf.value = it.value;
    }
    for (int k = 0; k < kHuffLutSize; k++)
        if (!set[k]) return sfail(SKML_E_ARG, "Huffman tree is not full");
    for (const N& nd : t) {
        if (nd.leaf) {
            nodes.push_back(int4{-1, -1, nd.value, 0});
        } else {
            if (nd.left < 0 || nd.right < 0) return sfail(SKML_E_ARG, "Huffman tree is not full");
            nodes.push_back(int4{node_base + nd.left, node_base + nd.right, 0, 0});
        }
    }
    return SKML_OK;
}
}  // namespace

// GroupedMinMaxSketch.readObject (GroupedMinMaxSketch.java:161-172), MinMaxSketch.readObject
// (MinMaxSketch.java:99-108), HuffmanEncoder.readObject + decode (HuffmanEncoder.java:127-166,
// 193-207) and DeltaAdaptiveEncoder.readObject (DeltaAdaptiveEncoder.java:172-188): the stream
// skml_sparse_serialize writes, back into a device payload that restore/decode accept.
int skml_sparse_deserialize(skml_ctx* c, const uint8_t* buf, size_t len, const double* qvalues, int32_t nvalues,
                            skml_sparse** out) {
    if (!c || !buf || !out || nvalues < 0 || (nvalues > 0 && !qvalues))
        return sfail(SKML_E_ARG, "bad deserialise arguments");
    *out = nullptr;
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    BeReader r{buf, len};
    skml_sparse* s = new skml_sparse();
    s->device = ctx_device(c);
    auto bail = [&](int e) {
        sparse_release(s);
        return e;
    };
    SpGroups& G = s->g;
    G.G = r.i32();
    G.rows = r.i32();
    s->params.col_ratio = r.f64();
    G.bin_num = r.i32();
    G.zero = r.i32();
    if (r.bad || G.G < 1 || G.G > kMaxGroups || G.rows < 0 || G.rows > kMaxRows || G.bin_num < 1)
        return bail(sfail(SKML_E_ARG, "malformed GroupedMinMaxSketch stream (groups %d rows %d bins %d)", G.G, G.rows,
                          G.bin_num));
    s->params.group_num = G.G;
    s->params.row_num = G.rows;
    s->params.bin_num = G.bin_num;
    G.fill = mm_cmp(INT32_MIN, INT32_MAX, G.zero) <= 0 ? INT32_MIN : INT32_MAX;
    std::vector<HuffGroupIn> hg((size_t)G.G);
    std::vector<char> present((size_t)G.G, 0);
    int64_t cells = 0;
    for (int g = 0; g < G.G; g++) {  // MinMaxSketch objects
        present[(size_t)g] = (char)r.byte();
        if (!present[(size_t)g]) continue;
        const int32_t rows = r.i32(), cols = r.i32(), zero = r.i32();
        if (rows != G.rows || cols < 0 || zero != G.zero) return bail(sfail(SKML_E_ARG, "malformed MinMaxSketch %d", g));
        G.cols[g] = cols;
        for (int k = 0; k < rows; k++) {
            G.hash_ids[g][k] = r.i32();
            (void)r.i32();  // hash size (= cols)
            (void)r.i32();  // BKDR seed (a function of the hash id)
            if (G.hash_ids[g][k] < 0 || G.hash_ids[g][k] > 7) return bail(sfail(SKML_E_ARG, "bad hash id"));
        }
        HuffGroupIn& h = hg[(size_t)g];
        const int32_t ni = r.i32();
        if (ni < 0 || (size_t)ni * 12 > len) return bail(sfail(SKML_E_ARG, "malformed Huffman items"));
        h.items.resize((size_t)ni);
        for (auto& it : h.items) {
            it.value = r.i32();
            it.bits = r.i32();
            it.nbits = r.i32();
        }
        const int32_t nl = r.i32();
        if (nl < 0 || !r.skip_longs((size_t)nl, &h.pos)) return bail(sfail(SKML_E_ARG, "malformed Huffman bit set"));
        h.nlongs = nl;
        h.size = r.i32();
        if (h.size != (int64_t)rows * cols) return bail(sfail(SKML_E_ARG, "Huffman size %lld != rows*cols", (long long)h.size));
        G.tab_off[g] = cells;
        cells += h.size;
    }
    // DeltaAdaptiveEncoder objects: the small fields here, the BitSets' positions in the stream.
    // toLongArray dropped each BitSet's trailing zero words, but the decode kernels index one
    // contiguous stream per kind, so every group's exact bit lengths are recovered on the device
    // (fixed-width flags: size * nf bits, and the deltas take bpi * (size + the flags' field sum);
    // unary flags end at the size-th zero, the deltas take bpi * (that length - size)).
    struct EncIn {
        int32_t size = 0, nf = 0, bpi = 0;
        int64_t fpos = 0, fn = 0, dpos = 0, dn = 0;
    };
    std::vector<EncIn> enc((size_t)G.G);
    int64_t n = 0;
    int32_t k1 = 0;
    for (int g = 0; g < G.G; g++) {
        G.gstart[g] = n;
        G.kind1_before[g] = k1;
        const int pres = r.byte();
        if (pres != present[(size_t)g]) return bail(sfail(SKML_E_ARG, "sketch / encoder presence mismatch in group %d", g));
        if (!pres) {
            G.m[g] = 1;
            G.kind[g] = 0;
            continue;
        }
        EncIn& e = enc[(size_t)g];
        e.size = r.i32();
        const int32_t m = r.i32();
        G.m[g] = m;
        G.kind[g] = r.byte() ? 1 : 0;
        if (e.size < 0 || (m != 1 && m != 2 && m != 4 && m != 8 && m != 16))
            return bail(sfail(SKML_E_ARG, "malformed DeltaAdaptiveEncoder %d (numIntervals %d)", g, m));
        const int32_t nfl = r.i32();
        if (nfl < 0 || !r.skip_longs((size_t)nfl, &e.fpos)) return bail(sfail(SKML_E_ARG, "malformed BitSet"));
        const int32_t ndl = r.i32();
        if (ndl < 0 || !r.skip_longs((size_t)ndl, &e.dpos)) return bail(sfail(SKML_E_ARG, "malformed BitSet"));
        e.fn = nfl;
        e.dn = ndl;
        e.bpi = 32 / m;
        while ((1 << (e.nf + 1)) <= m) e.nf++;  // floor(log2 m)
        if (G.kind[g]) k1 += e.size;
        n += e.size;
    }
    G.gstart[G.G] = n;
    if (r.bad) return bail(sfail(SKML_E_ARG, "truncated GroupedMinMaxSketch stream"));
    // the stream on the device, once
    // 16 bytes of slack: be64_at reads the aligned word after an unaligned long
    uint8_t* dstream = scratch<uint8_t>(c, kSlotWire, std::max<size_t>(len + 16, 64));
    if (!dstream) return bail(sfail(SKML_E_OOM, "device copy of the stream"));
    SP_HIP(hipMemcpyAsync(dstream, buf, len, hipMemcpyHostToDevice, st));
    // the flags' lengths: field sums of the fixed groups, zero selects of the unary ones
    std::vector<RdFlagSec> fx, un;
    std::vector<int> fx_g, un_g;
    for (int g = 0; g < G.G; g++) {
        if (!present[(size_t)g]) continue;
        const EncIn& e = enc[(size_t)g];
        RdFlagSec sc{e.fpos, e.fn, (int64_t)e.size * e.nf, e.size, e.nf, 0};
        if (G.kind[g]) {
            un.push_back(sc);
            un_g.push_back(g);
        } else if (e.nf > 0) {
            fx.push_back(sc);
            fx_g.push_back(g);
        }
    }
    std::vector<int64_t> fx_pre(fx.size() + 1, 0), un_pre(un.size() + 1, 0);
    for (size_t q = 0; q < fx.size(); q++) fx_pre[q + 1] = fx_pre[q] + (fx[q].nbits + 63) / 64;
    for (size_t q = 0; q < un.size(); q++) un_pre[q + 1] = un_pre[q] + (un[q].nstored + kRdTileWords - 1) / kRdTileWords;
    const size_t nfx = fx.size(), nun = un.size();
    const size_t o_un = align_up(sizeof(RdFlagSec) * std::max<size_t>(nfx, 1), 256);
    const size_t o_fxp = o_un + align_up(sizeof(RdFlagSec) * std::max<size_t>(nun, 1), 256);
    const size_t o_unp = o_fxp + align_up(sizeof(int64_t) * (nfx + 1), 256);
    const size_t o_res = o_unp + align_up(sizeof(int64_t) * (nun + 1), 256);  // sums[nfx] | flen[nun]
    const size_t o_tz = o_res + align_up(sizeof(int64_t) * (nfx + nun + 1), 256);
    uint8_t* meta = scratch<uint8_t>(c, kSlotWireMeta, o_tz + sizeof(uint32_t) * (size_t)std::max<int64_t>(un_pre.back(), 1));
    if (!meta) return bail(sfail(SKML_E_OOM, "readObject scratch"));
    int64_t* d_res = reinterpret_cast<int64_t*>(meta + o_res);
    std::vector<int64_t> res(nfx + nun, 0);
    if (nfx + nun > 0) {
        if (nfx) SP_HIP(hipMemcpyAsync(meta, fx.data(), sizeof(RdFlagSec) * nfx, hipMemcpyHostToDevice, st));
        if (nun) SP_HIP(hipMemcpyAsync(meta + o_un, un.data(), sizeof(RdFlagSec) * nun, hipMemcpyHostToDevice, st));
        SP_HIP(hipMemcpyAsync(meta + o_fxp, fx_pre.data(), sizeof(int64_t) * fx_pre.size(), hipMemcpyHostToDevice, st));
        SP_HIP(hipMemcpyAsync(meta + o_unp, un_pre.data(), sizeof(int64_t) * un_pre.size(), hipMemcpyHostToDevice, st));
        SP_HIP(hipMemsetAsync(d_res, 0, sizeof(int64_t) * (nfx + nun), st));
        SP_HIP(launch_rd_fixed_sum(st, dstream, reinterpret_cast<const RdFlagSec*>(meta),
                                   reinterpret_cast<const int64_t*>(meta + o_fxp), (int)nfx, fx_pre.back(),
                                   reinterpret_cast<uint64_t*>(d_res)));
        SP_HIP(launch_rd_unary(st, dstream, reinterpret_cast<const RdFlagSec*>(meta + o_un),
                               reinterpret_cast<const int64_t*>(meta + o_unp), (int)nun, un_pre.back(),
                               reinterpret_cast<uint32_t*>(meta + o_tz), d_res + nfx));
        if (int e = sync_to_host(c, res.data(), d_res, sizeof(int64_t) * res.size())) return bail(e);
    }
    std::vector<int64_t> flen((size_t)G.G, 0), dlen((size_t)G.G, 0);
    for (size_t q = 0; q < nfx; q++) {
        const int g = fx_g[q];
        flen[(size_t)g] = fx[q].nbits;
        dlen[(size_t)g] = (int64_t)enc[(size_t)g].bpi * ((int64_t)enc[(size_t)g].size + res[q]);
    }
    for (size_t q = 0; q < nun; q++) {
        const int g = un_g[q];
        flen[(size_t)g] = res[nfx + q];
        if (flen[(size_t)g] < enc[(size_t)g].size) return bail(sfail(SKML_E_ARG, "unary flags of group %d do not end", g));
        dlen[(size_t)g] = (int64_t)enc[(size_t)g].bpi * (flen[(size_t)g] - enc[(size_t)g].size);
    }
    int64_t fbits = 0, dbits = 0;
    for (int g = 0; g < G.G; g++) {
        G.fb[g] = fbits;
        G.db[g] = dbits;
        if (!present[(size_t)g]) continue;
        const EncIn& e = enc[(size_t)g];
        if (!G.kind[g] && e.nf == 0) {  // one interval per key: no flag bits, 32-bit deltas
            flen[(size_t)g] = 0;
            dlen[(size_t)g] = (int64_t)e.bpi * e.size;
        }
        if (e.fn > (flen[(size_t)g] + 63) / 64 || e.dn > (dlen[(size_t)g] + 63) / 64)
            return bail(sfail(SKML_E_ARG, "DeltaAdaptiveEncoder %d holds bits past its stream", g));
        fbits += flen[(size_t)g];
        dbits += dlen[(size_t)g];
    }
    G.fb[G.G] = fbits;
    G.db[G.G] = dbits;
    s->nnz = n;
    s->ncells = cells;
    G.ncells = cells;  // the group table's total as the encoder's plan leaves it (exported blobs check it)
    s->flag_bits = fbits;
    s->delta_bits = dbits;
    s->n_flag_words = (fbits + 63) / 64 + 1;
    s->n_delta_words = (dbits + 63) / 64 + 1;
    s->hdr.magic = SKML_DENSE_MAGIC;
    s->hdr.status = SKML_OK;
    s->hdr.n = n;
    s->hdr.bin_num = G.bin_num;
    s->hdr.zero_idx = G.zero;
    s->hdr.req_bins = G.bin_num;
    s->hdr.code_bits = code_bits_for(G.bin_num);
    s->qvalues.assign(qvalues, qvalues + nvalues);
    // device: group table, the contiguous DeltaAdaptive streams, MinMax tables
    if (hipMalloc(&s->g_dev, sizeof(SpGroups)) != hipSuccess ||
        hipMalloc(&s->flag_words, sizeof(uint64_t) * (size_t)s->n_flag_words) != hipSuccess ||
        hipMalloc(&s->delta_words, sizeof(uint64_t) * (size_t)s->n_delta_words) != hipSuccess ||
        hipMalloc(&s->tables, sizeof(int32_t) * (size_t)std::max<int64_t>(cells, 1)) != hipSuccess)
        return bail(sfail(SKML_E_OOM, "deserialised payload"));
    {
        std::vector<RdBitSec> fsec((size_t)G.G), dsec((size_t)G.G);
        for (int g = 0; g < G.G; g++) {
            fsec[(size_t)g] = RdBitSec{enc[(size_t)g].fpos, enc[(size_t)g].fn};
            dsec[(size_t)g] = RdBitSec{enc[(size_t)g].dpos, enc[(size_t)g].dn};
        }
        const size_t o_d = align_up(sizeof(RdBitSec) * (size_t)G.G, 256);
        const size_t o_fo = 2 * o_d, o_do = o_fo + align_up(sizeof(int64_t) * (size_t)(G.G + 1), 256);
        uint8_t* m2 = scratch<uint8_t>(c, kSlotStatus, o_do + sizeof(int64_t) * (size_t)(G.G + 1));
        if (!m2) return bail(sfail(SKML_E_OOM, "readObject scratch"));
        SP_HIP(hipMemcpyAsync(m2, fsec.data(), sizeof(RdBitSec) * fsec.size(), hipMemcpyHostToDevice, st));
        SP_HIP(hipMemcpyAsync(m2 + o_d, dsec.data(), sizeof(RdBitSec) * dsec.size(), hipMemcpyHostToDevice, st));
        SP_HIP(hipMemcpyAsync(m2 + o_fo, G.fb, sizeof(int64_t) * (size_t)(G.G + 1), hipMemcpyHostToDevice, st));
        SP_HIP(hipMemcpyAsync(m2 + o_do, G.db, sizeof(int64_t) * (size_t)(G.G + 1), hipMemcpyHostToDevice, st));
        SP_HIP(launch_rd_stream(st, dstream, reinterpret_cast<const RdBitSec*>(m2),
                                reinterpret_cast<const int64_t*>(m2 + o_fo), G.G, s->n_flag_words, s->flag_words));
        SP_HIP(launch_rd_stream(st, dstream, reinterpret_cast<const RdBitSec*>(m2 + o_d),
                                reinterpret_cast<const int64_t*>(m2 + o_do), G.G, s->n_delta_words, s->delta_words));
        SP_HIP(hipStreamSynchronize(st));  // the host tables above are the copies' sources
    }
    if (int e = upload_groups(c, s)) return bail(e);
    // HuffmanEncoder.decode of every group's table
    std::vector<HuffDecGroup> dg;
    std::vector<HuffSeg> segs;
    std::vector<int64_t> starts;
    std::vector<int2> lut;
    std::vector<int4> nodes;
    std::vector<int64_t> wpos, wpre{0};  // the groups' Huffman long[]s: stream positions, word prefix
    for (int g = 0; g < G.G; g++) {
        const HuffGroupIn& h = hg[(size_t)g];
        if (!present[(size_t)g] || h.size == 0) continue;
        if (h.items.empty()) return bail(sfail(SKML_E_ARG, "Huffman items missing in group %d", g));
        if (h.items.size() == 1) {  // a one-symbol tree: zero-bit codes
            SP_HIP(launch_fill_i32(st, s->tables + G.tab_off[g], h.size, h.items[0].value));
            continue;
        }
        HuffDecGroup d;
        d.word0 = wpre.back();
        d.nwords = h.nlongs;
        d.tab_off = G.tab_off[g];
        d.size = h.size;
        d.lut_row = (int32_t)(lut.size() / kHuffLutSize);
        d.seg0 = (int32_t)segs.size();
        std::vector<int4> gn;
        if (int e = huff_tables(h.items, (int)nodes.size(), lut, gn)) return bail(e);
        nodes.insert(nodes.end(), gn.begin(), gn.end());
        wpos.push_back(h.pos);
        wpre.push_back(wpre.back() + h.nlongs);
        const int64_t bits = d.nwords * 64;
        const int64_t nseg = std::max<int64_t>(1, (bits + kHuffSeg - 1) / kHuffSeg);
        for (int64_t k = 0; k < nseg; k++) {
            HuffSeg sg;
            sg.g = (int32_t)dg.size();
            sg.first = k == 0;
            sg.last = k == nseg - 1;
            sg.lim = (k + 1) * kHuffSeg;
            segs.push_back(sg);
            starts.push_back(k * kHuffSeg);
        }
        dg.push_back(d);
    }
    const int ns = (int)segs.size();
    if (ns > 0) {
        if (nodes.empty()) nodes.push_back(int4{-1, -1, 0, 0});
        const size_t nwords_all = (size_t)wpre.back() + 1;  // + a zero word read past the last one
        // one device block: groups, segments, starts, 2 x ends, counts (+1 for the scan total),
        // flags, LUT, nodes, words
        const size_t b_grp = align_up(sizeof(HuffDecGroup) * dg.size(), 256);
        const size_t b_seg = align_up(sizeof(HuffSeg) * (size_t)ns, 256);
        const size_t b_i64 = align_up(sizeof(int64_t) * (size_t)ns, 256);
        const size_t b_cnt = align_up(sizeof(uint64_t) * (size_t)(ns + 1), 256);
        const size_t b_lut = align_up(sizeof(int2) * lut.size(), 256);
        const size_t b_nod = align_up(sizeof(int4) * nodes.size(), 256);
        const size_t b_wrd = align_up(sizeof(uint64_t) * nwords_all, 256);
        const size_t b_wp = align_up(sizeof(int64_t) * (wpos.size() + wpre.size()), 256);
        const size_t total = b_grp + b_seg + 3 * b_i64 + b_cnt + 256 + b_lut + b_nod + b_wrd + b_wp;
        char* blk = nullptr;
        SP_HIP(hipMalloc(&blk, total));
        auto run = [&]() -> int {
            char* q = blk;
            auto* d_grp = (HuffDecGroup*)q; q += b_grp;
            auto* d_seg = (HuffSeg*)q; q += b_seg;
            auto* d_start = (int64_t*)q; q += b_i64;
            auto* d_ea = (int64_t*)q; q += b_i64;
            auto* d_eb = (int64_t*)q; q += b_i64;
            auto* d_cnt = (uint64_t*)q; q += b_cnt;
            auto* d_flag = (unsigned*)q; q += 256;
            auto* d_lut = (int2*)q; q += b_lut;
            auto* d_nod = (int4*)q; q += b_nod;
            auto* d_wrd = (uint64_t*)q; q += b_wrd;
            auto* d_wp = (int64_t*)q;
            SP_HIP(hipMemcpyAsync(d_wp, wpos.data(), sizeof(int64_t) * wpos.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemcpyAsync(d_wp + wpos.size(), wpre.data(), sizeof(int64_t) * wpre.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemsetAsync(d_wrd + wpre.back(), 0, sizeof(uint64_t), st));
            SP_HIP(launch_rd_words(st, dstream, d_wp, d_wp + wpos.size(), (int)wpos.size(), wpre.back(), d_wrd));
            SP_HIP(hipMemcpyAsync(d_grp, dg.data(), sizeof(HuffDecGroup) * dg.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemcpyAsync(d_seg, segs.data(), sizeof(HuffSeg) * segs.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemcpyAsync(d_start, starts.data(), sizeof(int64_t) * starts.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemcpyAsync(d_lut, lut.data(), sizeof(int2) * lut.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemcpyAsync(d_nod, nodes.data(), sizeof(int4) * nodes.size(), hipMemcpyHostToDevice, st));
            SP_HIP(hipMemsetAsync(d_cnt, 0, b_cnt, st));
            SP_HIP(launch_huff_spec(st, ns, d_seg, d_grp, d_wrd, d_lut, d_nod, d_start, d_ea, d_cnt));
            // resynchronise until every segment starts where its predecessor ends
            for (int round = 0;; round++) {
                if (round > ns + 1) return sfail(SKML_E_ARG, "Huffman stream does not resynchronise");
                SP_HIP(hipMemsetAsync(d_flag, 0, sizeof(unsigned), st));
                SP_HIP(launch_huff_sync(st, ns, d_seg, d_grp, d_wrd, d_lut, d_nod, d_start, d_ea, d_eb, d_cnt, d_flag));
                unsigned changed = 0;
                if (int e = sync_to_host(c, &changed, d_flag, sizeof(unsigned))) return e;
                std::swap(d_ea, d_eb);
                if (!changed) break;
            }
            SP_HIP(launch_scan_cols(st, d_cnt, ns, 1));  // exclusive scan: symbol offsets
            SP_HIP(hipMemsetAsync(d_flag, 0, sizeof(unsigned), st));
            SP_HIP(launch_huff_decode_write(st, ns, d_seg, d_grp, d_wrd, d_lut, d_nod, d_start, d_cnt, s->tables,
                                            d_flag));
            unsigned err = 0;
            if (int e = sync_to_host(c, &err, d_flag, sizeof(unsigned))) return e;
            if (err) return sfail(SKML_E_ARG, "Huffman stream holds a different number of symbols than size");
            return SKML_OK;
        };
        const int e = run();
        (void)hipStreamSynchronize(st);
        (void)hipFree(blk);
        if (e) return bail(e);
    }
    SP_HIP(hipStreamSynchronize(st));
    *out = s;
    return SKML_OK;
}

// GroupedMinMaxSketch.restore (GroupedMinMaxSketch.java:123-146) + Sort.merge: keys and int32 bins.
int skml_sparse_restore_bins(skml_ctx* c, const skml_sparse* s, int32_t* keys_dev, int32_t* bins_dev) {
    if (!c || !s) return sfail(SKML_E_ARG, "bad restore arguments");
    const int64_t n = s->nnz;
    if (n == 0) return SKML_OK;
    if (!keys_dev || !bins_dev) return sfail(SKML_E_ARG, "keys/bins are NULL");
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    int32_t* gk = scratch<int32_t>(c, kSlotGKeys, (size_t)n);
    int32_t* gb = scratch<int32_t>(c, kSlotGBins, (size_t)n);
    if (!gk || !gb) return sfail(SKML_E_OOM, "restore scratch");
    RsMerge rm;
    if (int e = rs_merge_prepare(c, s, &rm)) return e;
    const RunBoundsOut rbo = rm.query_bounds();  // the merge's key-range bounds from the query
    if (int e = decode_groups(c, s, gk, gb, true, nullptr, &rbo)) return e;
    volatile unsigned* pending = nullptr;
    if (int e = rs_merge_start(c, s, rm, gk, gb, keys_dev, bins_dev, 0, nullptr, 0, &pending)) return e;
    if (!pending)
        if (int e = merge_groups(c, s, gk, gb, keys_dev, bins_dev)) return e;
    SP_HIP(hipStreamSynchronize(st));
    t_merge_path = s->g.G < 2 ? 0 : pending ? 1 : 2;
    if (pending && *pending) {  // not regular: the merge rounds decide
        t_merge_path = 3;
        if (int e = merge_groups(c, s, gk, gb, keys_dev, bins_dev)) return e;
        SP_HIP(hipStreamSynchronize(st));
    }
    return SKML_OK;
}

// ---- exchange: one contiguous device blob per payload (SpBlobHeader, skml_sparse.h) ----
}  // extern "C"

namespace {
struct BlobLayout {
    size_t off_groups, off_quant, off_values, off_tables, off_flags, off_deltas, total;
    int32_t quant_bytes;
    int table_width;  // the MinMax cells: the payload's exact narrow image (8 / 16 bits) when it has one
};
BlobLayout blob_layout(const skml_sparse* s) {
    BlobLayout L;
    L.quant_bytes = (int32_t)(kHeaderBytes + sizeof(double) * (size_t)std::max(s->hdr.bin_num - 1, 0));
    L.table_width = s->tnar ? s->tnar_width : 32;
    L.off_groups = 256;
    L.off_quant = L.off_groups + align_up(sizeof(SpGroups), 256);
    L.off_values = L.off_quant + align_up((size_t)L.quant_bytes, 256);
    L.off_tables = L.off_values + align_up(sizeof(double) * std::max<size_t>(s->qvalues.size(), 1), 256);
    L.off_flags = L.off_tables + align_up((size_t)L.table_width / 8 * (size_t)std::max<int64_t>(s->ncells, 1), 256);
    L.off_deltas = L.off_flags + align_up(sizeof(uint64_t) * (size_t)s->n_flag_words, 256);
    L.total = L.off_deltas + align_up(sizeof(uint64_t) * (size_t)s->n_delta_words, 256);
    return L;
}

// A blob's group table, checked for the invariants the decode kernels index by (a corrupt or
// foreign blob must fail here, not fault on the device).
int check_blob_groups(const SpBlobHeader& h, const SpGroups& G) {
    auto bad = [](const char* what) { return sfail(SKML_E_ARG, "sparse blob: inconsistent %s", what); };
    if (G.G < 1 || G.G > kMaxGroups || G.rows < 0 || G.rows > kMaxRows) return bad("group / row count");
    if (G.bin_num < 1 || G.bin_num > h.nvalues || G.zero < 0 || G.zero >= G.bin_num) return bad("bins");
    if (h.version >= 2 && h.table_width != 32 && h.table_width != tnar_width_for(G.bin_num)) return bad("cell width");
    if (G.gstart[0] != 0 || G.gstart[G.G] != h.nnz || G.fb[0] != 0 || G.db[0] != 0) return bad("stream starts");
    if (G.fb[G.G] != h.flag_bits || G.db[G.G] != h.delta_bits || G.ncells != h.ncells) return bad("stream totals");
    if (h.n_flag_words < (h.flag_bits + 63) / 64 + 1 || h.n_delta_words < (h.delta_bits + 63) / 64 + 1)
        return bad("word counts");
    int32_t k1 = 0;
    for (int g = 0; g < G.G; g++) {
        if (G.gstart[g + 1] < G.gstart[g] || G.fb[g + 1] < G.fb[g] || G.db[g + 1] < G.db[g]) return bad("offsets");
        const int64_t size = G.gstart[g + 1] - G.gstart[g];
        const int32_t m = G.m[g];
        if (m != 1 && m != 2 && m != 4 && m != 8 && m != 16) return bad("numIntervals");
        if (G.kind[g] != 0 && G.kind[g] != 1) return bad("flagKind");
        if (G.kind1_before[g] != k1) return bad("unary counts");
        if (G.kind[g]) k1 += (int32_t)size;
        if (size == 0) continue;
        if (G.cols[g] < 1 || G.tab_off[g] < 0 || G.tab_off[g] + (int64_t)G.rows * G.cols[g] > G.ncells)
            return bad("table shape");
        if (G.inv_cols[g] != 1.0 / (double)G.cols[g]) return bad("column reciprocal");
        for (int r = 0; r < G.rows; r++)
            if (G.hash_ids[g][r] < 0 || G.hash_ids[g][r] > 7) return bad("hash id");
    }
    return SKML_OK;
}

// A blob's header, checked against the `len` bytes it may span.
int blob_table_width(const SpBlobHeader* h) { return h->version >= 2 ? h->table_width : 32; }
int blob_check_header(const SpBlobHeader* h, size_t len) {
    if (h->magic != kSpBlobMagic || h->version < 1 || h->version > 2) return sfail(SKML_E_STATE, "not a sparse blob");
    const int tw = blob_table_width(h);
    if (tw != 8 && tw != 16 && tw != 32) return sfail(SKML_E_ARG, "sparse blob: cell width %d", tw);
    if (h->total_bytes < 256 || (size_t)h->total_bytes > len || h->nnz < 0 || h->nnz > INT32_MAX || h->ncells < 0 ||
        h->nvalues < 1 || h->nvalues > SKML_MAX_BINS || h->quant_bytes < kHeaderBytes ||
        h->off_groups != 256 || h->off_quant < h->off_groups + (int64_t)sizeof(SpGroups) ||
        h->off_values < h->off_quant + h->quant_bytes || h->off_tables < h->off_values + 8 * (int64_t)h->nvalues ||
        h->off_flags < h->off_tables + tw / 8 * h->ncells || h->off_deltas < h->off_flags + 8 * h->n_flag_words ||
        h->total_bytes < h->off_deltas + 8 * h->n_delta_words || (h->off_tables | h->off_flags | h->off_deltas) & 255)
        return sfail(SKML_E_ARG, "sparse blob: inconsistent section offsets");
    return SKML_OK;
}

// A non-owning skml_sparse view of the blob at `dev`, from its host meta `meta` (header, group
// table, quantizer header + splits, values: the blob's bytes up to off_tables).
int blob_view(skml_ctx* c, const uint8_t* dev, const SpBlobHeader& h, const uint8_t* meta, skml_sparse* view) {
    std::memcpy(&view->g, meta + h.off_groups, sizeof(SpGroups));
    if (int e = check_blob_groups(h, view->g)) return e;
    std::memcpy(&view->hdr, meta + h.off_quant, sizeof(skml_dense_header));
    const double* sp = reinterpret_cast<const double*>(meta + h.off_quant + kHeaderBytes);
    const int ns = (h.quant_bytes - kHeaderBytes) / 8;
    view->splits.assign(sp, sp + ns);
    const double* qv = reinterpret_cast<const double*>(meta + h.off_values);
    view->qvalues.assign(qv, qv + h.nvalues);
    view->device = ctx_device(c);
    view->nnz = h.nnz;
    view->params = h.params;
    view->ncells = h.ncells;
    view->flag_bits = h.flag_bits;
    view->delta_bits = h.delta_bits;
    view->n_flag_words = h.n_flag_words;
    view->n_delta_words = h.n_delta_words;
    view->g_dev = reinterpret_cast<SpGroups*>(const_cast<uint8_t*>(dev) + h.off_groups);
    uint8_t* tab = const_cast<uint8_t*>(dev) + h.off_tables;
    const int tw = blob_table_width(&h);
    view->tables = tw == 32 ? reinterpret_cast<int32_t*>(tab) : nullptr;
    view->tnar = tw == 32 ? nullptr : tab;
    view->tnar_width = tw == 32 ? 0 : tw;
    view->flag_words = reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(dev) + h.off_flags);
    view->delta_words = reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(dev) + h.off_deltas);
    return SKML_OK;
}

// The host meta of P blobs at `dev` + p * stride and their views: the first 16 KB of every blob
// (header, group table, quantizer and values of up to ~1,000 bins) in one strided device-to-host
// copy, and only if some blob's meta runs past that, every blob's meta in a second (a read-back
// per blob and section cost ~20 us of host round trip each, 16 of them for 8 payloads).
int blob_metas(skml_ctx* c, const uint8_t* dev, int P, size_t stride, SpBlobHeader* hs, skml_sparse* views) {
    if (!dev || P < 1 || stride < 256 || (stride & 255) || (reinterpret_cast<uintptr_t>(dev) & 255))
        return sfail(SKML_E_ARG, "sparse blob: NULL, shorter than its header or not 256-byte aligned");
    hipStream_t st = ctx_stream(c);
    size_t w = std::min<size_t>(stride, 16384);
    uint8_t* pin = static_cast<uint8_t*>(ctx_pinned(c, w * (size_t)P));
    if (!pin) return sfail(SKML_E_OOM, "pinned staging of %zu bytes", w * (size_t)P);
    SP_HIP(hipMemcpy2DAsync(pin, w, dev, stride, w, (size_t)P, hipMemcpyDeviceToHost, st));
    SP_HIP(hipStreamSynchronize(st));
    size_t meta_max = 0;
    for (int p = 0; p < P; p++) {
        std::memcpy(&hs[p], pin + (size_t)p * w, sizeof(SpBlobHeader));
        if (int e = blob_check_header(&hs[p], stride)) return sfail(e, "payload %d: %s", p, skml_last_error());
        meta_max = std::max(meta_max, (size_t)hs[p].off_tables);
    }
    if (meta_max > w) {  // off_tables is a multiple of 256 below total_bytes <= stride
        w = meta_max;
        pin = static_cast<uint8_t*>(ctx_pinned(c, w * (size_t)P));
        if (!pin) return sfail(SKML_E_OOM, "pinned staging of %zu bytes", w * (size_t)P);
        SP_HIP(hipMemcpy2DAsync(pin, w, dev, stride, w, (size_t)P, hipMemcpyDeviceToHost, st));
        SP_HIP(hipStreamSynchronize(st));
    }
    for (int p = 0; p < P; p++)
        if (int e = blob_view(c, dev + (size_t)p * stride, hs[p], pin + (size_t)p * w, &views[p]))
            return sfail(e, "payload %d: %s", p, skml_last_error());
    return SKML_OK;
}

// The host meta of a blob at `dev` (header, group table, quantizer header + splits, values) and a
// non-owning skml_sparse view of its device sections.
int blob_meta(skml_ctx* c, const uint8_t* dev, size_t len, SpBlobHeader* h, skml_sparse* view) {
    if (!dev || len < 256 || (reinterpret_cast<uintptr_t>(dev) & 255))
        return sfail(SKML_E_ARG, "sparse blob: NULL, shorter than its header or not 256-byte aligned");
    if (int e = sync_to_host(c, h, dev, sizeof(*h))) return e;
    if (int e = blob_check_header(h, len)) return e;
    std::vector<uint8_t> meta((size_t)h->off_tables);
    if (int e = sync_to_host(c, meta.data(), dev, meta.size())) return e;
    return blob_view(c, dev, *h, meta.data(), view);
}

// a view points into memory it does not own: cleared before it goes out of scope, so no later
// change to skml_sparse's destruction can free the caller's blob
struct ViewGuard {
    skml_sparse* v;
    ~ViewGuard() {
        v->g_dev = nullptr;
        v->tables = nullptr;
        v->tnar = nullptr;
        v->flag_words = v->delta_words = nullptr;
        v->qpayload = nullptr;
    }
};
}  // namespace

extern "C" {

int skml_sparse_export_bytes(const skml_sparse* s, size_t* bytes) {
    if (!s || !bytes) return sfail(SKML_E_ARG, "NULL argument");
    *bytes = blob_layout(s).total;
    return SKML_OK;
}

int skml_sparse_export(skml_ctx* c, const skml_sparse* s, void* dst, size_t cap) {
    if (!c || !s || !dst || (reinterpret_cast<uintptr_t>(dst) & 255)) return sfail(SKML_E_ARG, "bad export arguments");
    const BlobLayout L = blob_layout(s);
    if (cap < L.total) return sfail(SKML_E_ARG, "export capacity %zu < %zu", cap, L.total);
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    // the host-side sections go through the context's pinned staging in one copy
    const size_t host_bytes = L.off_tables;
    uint8_t* pin = static_cast<uint8_t*>(ctx_pinned(c, host_bytes));
    if (!pin) return sfail(SKML_E_OOM, "pinned staging");
    SP_HIP(hipStreamSynchronize(st));  // the staging buffer may still feed an earlier copy
    std::memset(pin, 0, host_bytes);
    SpBlobHeader h{};
    h.magic = kSpBlobMagic;
    h.version = 2;
    h.table_width = L.table_width;
    h.total_bytes = (int64_t)L.total;
    h.nnz = s->nnz;
    h.ncells = s->ncells;
    h.n_flag_words = s->n_flag_words;
    h.n_delta_words = s->n_delta_words;
    h.flag_bits = s->flag_bits;
    h.delta_bits = s->delta_bits;
    h.nvalues = (int32_t)s->qvalues.size();
    h.quant_bytes = L.quant_bytes;
    h.off_groups = (int64_t)L.off_groups;
    h.off_quant = (int64_t)L.off_quant;
    h.off_values = (int64_t)L.off_values;
    h.off_tables = (int64_t)L.off_tables;
    h.off_flags = (int64_t)L.off_flags;
    h.off_deltas = (int64_t)L.off_deltas;
    h.params = s->params;
    std::memcpy(pin, &h, sizeof(h));
    SpGroups g = s->g;
    for (int k = 0; k < kMaxGroups; k++) g.inv_cols[k] = g.cols[k] > 0 ? 1.0 / (double)g.cols[k] : 0.0;
    std::memcpy(pin + L.off_groups, &g, sizeof(g));
    std::memcpy(pin + L.off_quant, &s->hdr, sizeof(skml_dense_header));
    if (!s->splits.empty())
        std::memcpy(pin + L.off_quant + kHeaderBytes, s->splits.data(), sizeof(double) * s->splits.size());
    if (!s->qvalues.empty()) std::memcpy(pin + L.off_values, s->qvalues.data(), sizeof(double) * s->qvalues.size());
    uint8_t* d = static_cast<uint8_t*>(dst);
    SP_HIP(hipMemcpyAsync(d, pin, host_bytes, hipMemcpyHostToDevice, st));
    if (s->ncells > 0)  // the exact narrow image when the payload has one, else the int32 cells
        SP_HIP(hipMemcpyAsync(d + L.off_tables, s->tnar ? s->tnar : static_cast<const void*>(s->tables),
                              (size_t)L.table_width / 8 * (size_t)s->ncells, hipMemcpyDeviceToDevice, st));
    if (s->n_flag_words > 0)
        SP_HIP(hipMemcpyAsync(d + L.off_flags, s->flag_words, sizeof(uint64_t) * (size_t)s->n_flag_words,
                              hipMemcpyDeviceToDevice, st));
    if (s->n_delta_words > 0)
        SP_HIP(hipMemcpyAsync(d + L.off_deltas, s->delta_words, sizeof(uint64_t) * (size_t)s->n_delta_words,
                              hipMemcpyDeviceToDevice, st));
    return SKML_OK;
}

int skml_sparse_import(skml_ctx* c, const void* blob, size_t len, skml_sparse** out) {
    if (!c || !out) return sfail(SKML_E_ARG, "bad import arguments");
    *out = nullptr;
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    SpBlobHeader h;
    skml_sparse view;
    ViewGuard vg{&view};
    if (int e = blob_meta(c, static_cast<const uint8_t*>(blob), len, &h, &view)) return e;
    // an owned copy: the caller's gathered buffer may be reused by the next exchange
    skml_sparse* s = new skml_sparse();
    s->device = view.device;
    s->nnz = view.nnz;
    s->params = view.params;
    s->hdr = view.hdr;
    s->splits = view.splits;
    s->qvalues = view.qvalues;
    s->g = view.g;
    s->ncells = view.ncells;
    s->flag_bits = view.flag_bits;
    s->delta_bits = view.delta_bits;
    s->n_flag_words = view.n_flag_words;
    s->n_delta_words = view.n_delta_words;
    // a narrow blob keeps its exact image (the restore gathers from it) and gets its int32 cells
    // back (serialisation, group info)
    const int tw = view.tnar ? view.tnar_width : 0;
    const size_t o_tab = align_up(sizeof(SpGroups), 256);
    const size_t o_tn = o_tab + align_up(sizeof(int32_t) * (size_t)std::max<int64_t>(s->ncells, 1), 256);
    const size_t o_fw = o_tn + (tw ? align_up((size_t)tw / 8 * (size_t)std::max<int64_t>(s->ncells, 1), 256) : 0);
    const size_t o_dw = o_fw + align_up(sizeof(uint64_t) * (size_t)s->n_flag_words, 256);
    const size_t o_qv = o_dw + align_up(sizeof(uint64_t) * (size_t)s->n_delta_words, 256);
    const size_t total = o_qv + sizeof(double) * std::max<size_t>(s->qvalues.size(), 1);
    char* blk = static_cast<char*>(block_get(s->device, total, &s->block_cap));
    if (!blk) {
        sparse_release(s);
        return sfail(SKML_E_OOM, "imported sparse payload of %zu bytes", total);
    }
    s->qv_dev = reinterpret_cast<double*>(blk + o_qv);
    s->block = blk;
    s->g_dev = reinterpret_cast<SpGroups*>(blk);
    s->tables = reinterpret_cast<int32_t*>(blk + o_tab);
    s->tnar = tw ? blk + o_tn : nullptr;
    s->tnar_width = tw;
    s->flag_words = reinterpret_cast<uint64_t*>(blk + o_fw);
    s->delta_words = reinterpret_cast<uint64_t*>(blk + o_dw);
    auto fail_rel = [&](int e) {
        (void)hipStreamSynchronize(st);
        sparse_release(s);
        return e;
    };
#define IMP_HIP(expr)                                                                                        \
    do {                                                                                                     \
        hipError_t e_ = (expr);                                                                              \
        if (e_ != hipSuccess) return fail_rel(sfail(SKML_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_))); \
    } while (0)
    IMP_HIP(hipMemcpyAsync(s->g_dev, view.g_dev, sizeof(SpGroups), hipMemcpyDeviceToDevice, st));
    if (!s->qvalues.empty())  // the blob's values section: the device copy of quantValues
        IMP_HIP(hipMemcpyAsync(s->qv_dev, static_cast<const uint8_t*>(blob) + h.off_values,
                               sizeof(double) * s->qvalues.size(), hipMemcpyDeviceToDevice, st));
    s->qv_dev_ok = !s->qvalues.empty();
    if (s->ncells > 0 && tw) {
        IMP_HIP(hipMemcpyAsync(s->tnar, view.tnar, (size_t)tw / 8 * (size_t)s->ncells, hipMemcpyDeviceToDevice, st));
        IMP_HIP(launch_widen_cells(st, s->tnar, tw, s->ncells, s->g.fill, s->tables));
    } else if (s->ncells > 0) {
        IMP_HIP(hipMemcpyAsync(s->tables, view.tables, sizeof(int32_t) * (size_t)s->ncells, hipMemcpyDeviceToDevice, st));
    }
    if (s->n_flag_words > 0)
        IMP_HIP(hipMemcpyAsync(s->flag_words, view.flag_words, sizeof(uint64_t) * (size_t)s->n_flag_words,
                               hipMemcpyDeviceToDevice, st));
    if (s->n_delta_words > 0)
        IMP_HIP(hipMemcpyAsync(s->delta_words, view.delta_words, sizeof(uint64_t) * (size_t)s->n_delta_words,
                               hipMemcpyDeviceToDevice, st));
    IMP_HIP(hipStreamSynchronize(st));
#undef IMP_HIP
    *out = s;
    return SKML_OK;
}

// Gradient.sum over P exported sparse payloads (ml/gradient/Gradient.scala:44-49): out = +0.0,
// then for p = 0..P-1 in order DenseDoubleGradient.plusBy(payload p .toAuto)
// (DenseDoubleGradient.scala:38; SketchGradient.toSparse -> SparseDoubleGradient.toAuto), then
// out *= scale unless scale == 1.  A payload whose live count (|v| > 1e-8) exceeds dim * 2 / 3 (Java
// int arithmetic) reaches plusBy in dense form: only its live values are added, and every entry
// takes the dense form's + 0.0.  SketchGradient.toSparse builds a SparseDoubleGradient from the
// restored keys, whose constructor requires them strictly increasing and inside [0, dim)
// (SparseDoubleGradient.scala:9-14): a key repeated across a payload's groups, a run that does not
// ascend or a key out of range fails the whole sum with SKML_E_ARG.
int skml_sparse_decode_sum_f64(skml_ctx* c, const void* blobs, int32_t P, size_t stride, int64_t dim, double scale,
                               double* out) {
    if (!c || !blobs || P < 1 || dim < 0 || dim > (int64_t)INT32_MAX || (dim > 0 && !out) || stride % 256)
        return sfail(SKML_E_ARG, "bad sparse decode_sum arguments (P >= 1, 256-byte stride, dim in Java int)");
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    std::vector<SpBlobHeader> hs((size_t)P);
    std::vector<skml_sparse> views((size_t)P);  // non-owning: skml_sparse frees nothing on destruction
    if (int e = blob_metas(c, static_cast<const uint8_t*>(blobs), P, stride, hs.data(), views.data())) return e;
    const int64_t lim = (int64_t)(int32_t)((uint32_t)dim * 2u) / 3;  // dim * 2 / 3 with Java int wrap
    // run bounds are taken per tile of the tile kernel: 512 keys for the wave-tile form, else 4,096
    const int64_t ntiles_max = sp_tiles(dim, (int64_t)1 << agg_tile_bits(true));
    auto bin_width = [&](int p) { return views[(size_t)p].qvalues.size() <= 256 ? 1 : 2; };
    // a payload's restored keys and bins, each 16-byte aligned in its scratch buffer
    auto key_words = [&](int p) { return (views[(size_t)p].nnz + 3) & ~int64_t{3}; };
    auto bin_bytes = [&](int p) { return (views[(size_t)p].nnz * bin_width(p) + 15) & ~int64_t{15}; };
    // payloads in batches whose restored keys + bins + run bounds fit the scratch budget; the first
    // batch starts the sum at +0.0, later ones continue from it, the last one applies the scale
    constexpr size_t kBudget = (size_t)3 << 30;
    auto need_of = [&](int p) {
        return (size_t)key_words(p) * 4 + (size_t)bin_bytes(p) +
               (size_t)views[(size_t)p].g.G * (size_t)(ntiles_max + 1) * 4 + 1024;
    };
    // SketchGradient.toSparse of an empty restore builds SparseDoubleGradient(dim, [], []), whose
    // constructor reads indices.head (SparseDoubleGradient.scala:11) and throws: so does the sum
    for (int p = 0; p < P; p++)
        if (views[(size_t)p].nnz == 0)
            return sfail(SKML_E_ARG, "payload %d restores no keys: head of empty list (SparseDoubleGradient.scala:11)", p);
    std::vector<int> todo;
    for (int p = 0; p < P; p++) todo.push_back(p);
    uint8_t* small = scratch<uint8_t>(c, kSlotStatus, 1024 + sizeof(AggPayload) * (size_t)P);
    if (!small) return sfail(SKML_E_OOM, "decode_sum scratch");
    unsigned* err = reinterpret_cast<unsigned*>(small);
    uint64_t* live = reinterpret_cast<uint64_t*>(small + 256);
    AggPayload* d_pays = reinterpret_cast<AggPayload*>(small + 1024);
    SP_HIP(hipMemsetAsync(err, 0, sizeof(unsigned), st));
    size_t at = 0;
    bool first = true;
    while (at < todo.size()) {
        size_t end = at, bytes = 0;
        while (end < todo.size() && (end == at || bytes + need_of(todo[end]) <= kBudget)) bytes += need_of(todo[end++]);
        int max_g = 0, max_nq = 0;
        for (size_t q = at; q < end; q++) {
            max_g = std::max(max_g, (int)views[(size_t)todo[q]].g.G);
            max_nq = std::max(max_nq, (int)views[(size_t)todo[q]].qvalues.size());
        }
        const bool vt = agg_vtiles_ok(max_g, max_nq);
        const int tile_bits = agg_tile_bits(vt);
        const int64_t ntiles = sp_tiles(dim, (int64_t)1 << tile_bits);
        int64_t nk = 0, nbb = 0, nb = 0;
        for (size_t q = at; q < end; q++) {
            nk += key_words(todo[q]);
            nbb += bin_bytes(todo[q]);
            nb += (int64_t)views[(size_t)todo[q]].g.G * (ntiles + 1);
        }
        int32_t* gk = scratch<int32_t>(c, kSlotCKeys, (size_t)nk);
        uint8_t* gbn = scratch<uint8_t>(c, kSlotCVals, (size_t)nbb);  // 1 or 2 bytes per bin
        int32_t* bounds = scratch<int32_t>(c, kSlotCells, (size_t)nb);
        if (!gk || !gbn || !bounds) return sfail(SKML_E_OOM, "decode_sum scratch (%lld keys)", (long long)nk);
        SP_HIP(hipMemsetAsync(bounds, 0, sizeof(int32_t) * (size_t)nb, st));  // empty groups: every bound 0
        // two lanes: payloads alternate between the caller's stream and the side context's (each
        // restore is a chain of small latency-bound kernels; two chains fill the chip better),
        // joined before the tiles; SKML_SERIAL, SKML_FORM_AGG_ONE_LANE or a single payload keep one
        skml_ctx* lanes[2] = {c, nullptr};
        hipStream_t side_st = nullptr;
        hipEvent_t ev_fork = nullptr, ev_join = nullptr;
        if (end - at > 1 && form(SKML_FORM_AGG_ONE_LANE) != 1 && ctx_side_fork(c, &side_st, &ev_fork, &ev_join) == SKML_OK) {
            lanes[1] = ctx_side_ctx(c);
            SP_HIP(hipEventRecord(ev_fork, st));
            SP_HIP(hipStreamWaitEvent(side_st, ev_fork, 0));
        }
        std::vector<AggPayload> pays;
        int64_t ko = 0, bbo = 0, bo = 0;
        for (size_t q = at; q < end; q++) {
            const int p = todo[q];
            const int li = lanes[1] && ((q - at) & 1) ? 1 : 0;
            skml_ctx* lc = lanes[li];
            hipStream_t ls = ctx_stream(lc);
            uint64_t* llive = live + li;
            const skml_sparse& v = views[(size_t)p];
            AggPayload a{};
            a.gk = gk + ko;
            a.nq = (int)v.qvalues.size();
            a.bw = bin_width(p);
            a.gb = gbn + bbo;
            a.qv = reinterpret_cast<const double*>(static_cast<const uint8_t*>(blobs) + (size_t)p * stride +
                                                   hs[(size_t)p].off_values);
            a.bounds = bounds + bo;
            a.G = v.g.G;
            a.gk_off = (int32_t)ko;   // < 2^31: the batch's keys fit the 3 GB scratch budget
            a.gb_off = (int32_t)bbo;
            // the run bounds come from the key query unless SKML_FORM_RUN_BOUNDS = 1 asks for the
            // separate k_agg_bounds pass (A/B)
#ifdef SKML_AB
            const bool own_pass = form(SKML_FORM_RUN_BOUNDS) == 1;
#else
            constexpr bool own_pass = false;
#endif
            const DecodeValues dv{a.nq, const_cast<void*>(a.gb), a.bw, err,
                                  own_pass ? RunBoundsOut{nullptr, 0, 0, 0}
                                           : RunBoundsOut{const_cast<int32_t*>(a.bounds), ntiles, dim, tile_bits}};
            auto join = [&](int e) {  // an error after the fork: the caller's stream still waits for the side
                if (lanes[1]) {
                    (void)hipEventRecord(ev_join, side_st);
                    (void)hipStreamWaitEvent(st, ev_join, 0);
                }
                return e;
            };
            if (int e = decode_groups(lc, &v, gk + ko, nullptr, true, &dv)) return join(e);
            if (v.nnz > lim) {  // live <= nnz: only then can toAuto pick the dense form
                if (launch_count_live(ls, a.gb, a.bw, v.nnz, a.qv, llive) != hipSuccess)
                    return join(sfail(SKML_E_HIP, "count_live launch failed"));
                uint64_t nlive = 0;
                if (int e = sync_to_host(lc, &nlive, llive, sizeof(nlive))) return join(e);
                a.dense_form = (int64_t)nlive > lim ? 1 : 0;
            }
#ifdef SKML_AB
            if (own_pass && launch_agg_bounds(ls, a.gk, v.nnz, v.g_dev, ntiles, dim, const_cast<int32_t*>(a.bounds), err,
                                              tile_bits) != hipSuccess)
                return join(sfail(SKML_E_HIP, "agg_bounds launch failed"));
#endif
            pays.push_back(a);
            ko += key_words(p);
            bbo += bin_bytes(p);
            bo += (int64_t)v.g.G * (ntiles + 1);
        }
        if (lanes[1]) {
            SP_HIP(hipEventRecord(ev_join, side_st));
            SP_HIP(hipStreamWaitEvent(st, ev_join, 0));
        }
        const bool last = end == todo.size();
        SP_HIP(hipMemcpyAsync(d_pays, pays.data(), sizeof(AggPayload) * pays.size(), hipMemcpyHostToDevice, st));
        // the wave-tile form takes 8 payloads per launch (a lane per (payload, group)); later
        // launches continue the sum in payload order
        const size_t chunk = vt ? (size_t)kAggVPayloads : pays.size();
        for (size_t c0 = 0; c0 < pays.size(); c0 += chunk) {
            const size_t nc = std::min(chunk, pays.size() - c0);
            bool any_dense = false;
            for (size_t q = c0; q < c0 + nc; q++) any_dense |= pays[q].dense_form != 0;
            SP_HIP(launch_agg_tiles(st, d_pays + c0, (int)nc, ntiles, dim, out, first && c0 == 0 ? 0 : 1,
                                    last && c0 + nc == pays.size() ? scale : 1.0, err, vt, gk, gbn, any_dense));
        }
        SP_HIP(hipStreamSynchronize(st));  // `pays` (host) and the scratch are reused by the next batch
        first = false;
        at = end;
    }
    unsigned bad = 0;
    if (int e = sync_to_host(c, &bad, err, sizeof(bad))) return e;
    if (bad & 1u)
        return sfail(SKML_E_ARG, "a payload holds a key outside [0, %lld), a non-ascending run or a bin outside its "
                                 "values (SparseDoubleGradient requires ascending indices in range)", (long long)dim);
    if (bad & 2u)
        return sfail(SKML_E_ARG, "requirement failed: Indices are not strictly increasing (a key repeated across a "
                                 "payload's groups; SparseDoubleGradient.scala:12)");
    return SKML_OK;
}

int skml_debug_sparse_merge_path(void) { return t_merge_path; }

int skml_debug_sparse_scratch_fail(int on) {
    g_fail_cellbuf.store(on ? 1 : 0);
    return SKML_OK;
}

int skml_sparse_free(skml_sparse* s) {
    sparse_release(s);
    return SKML_OK;
}

// ---- standalone DeltaAdaptiveEncoder: one group, no MinMax ----
int skml_delta_encode(skml_ctx* c, const int32_t* keys, int64_t n, int32_t* num_intervals, int32_t* flag_kind,
                      int64_t* n_flag_bits, int64_t* n_delta_bits, uint64_t* flag_words_dev,
                      uint64_t* delta_words_dev, int64_t words_cap) {
    if (!c || !keys || n <= 0 || !num_intervals || !flag_kind || !n_flag_bits || !n_delta_bits)
        return sfail(SKML_E_ARG, "bad delta arguments");
    if (n > (int64_t)INT32_MAX) return sfail(SKML_E_ARG, "n exceeds Java int");
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    skml_sparse tmp;
    tmp.device = ctx_device(c);
    tmp.nnz = n;
    SpGroups& G = tmp.g;
    G.G = 1;
    G.rows = 0;
    G.gstart[0] = 0;
    G.gstart[1] = n;
    G.cols[0] = 1;
    uint8_t* need = scratch<uint8_t>(c, kSlotNeed, (size_t)n);
    uint32_t* small = scratch<uint32_t>(c, kSlotSmall, (size_t)kMaxGroups * kDeltaHist + 64);
    const int64_t fwn = flag_words_max(n), dwn = delta_words_max(n);
    const size_t o_w = align_up(sizeof(SpGroups), 256);
    char* blk = static_cast<char*>(ctx_scratch(c, kSlotDeltaEnc, o_w + sizeof(uint64_t) * (size_t)(fwn + dwn)));
    if (!need || !small || !blk) return sfail(SKML_E_OOM, "delta scratch");
    tmp.g_dev = reinterpret_cast<SpGroups*>(blk);
    uint64_t* fwd = reinterpret_cast<uint64_t*>(blk + o_w);
    uint64_t* dwd = fwd + fwn;
    int rc = upload_groups(c, &tmp);
    tmp.g_dev = nullptr;  // scratch-owned
    if (rc) return rc;
    SpGroups* g_dev = reinterpret_cast<SpGroups*>(blk);
    SP_HIP(hipMemsetAsync(small, 0, sizeof(uint32_t) * ((size_t)kMaxGroups * kDeltaHist + 1), st));
    SP_HIP(launch_group_prep(st, keys, n, g_dev, need, small, small + kMaxGroups * kDeltaHist, nullptr, 0, nullptr,
                             nullptr));
    if (int e = encode_delta_device(c, st, g_dev, keys, need, n, small, small + kMaxGroups * kDeltaHist, fwd, dwd))
        return e;
    if (int e = sync_to_host(c, &G, g_dev, sizeof(SpGroups))) return e;
    if (G.status & kSpOrder) return sfail(SKML_E_ORDER, "Log for a non-positive key delta (keys must ascend strictly)");
    *num_intervals = G.m[0];
    *flag_kind = G.kind[0];
    *n_flag_bits = G.fb[1];
    *n_delta_bits = G.db[1];
    const int64_t fw = (G.fb[1] + 63) / 64, dw = (G.db[1] + 63) / 64;
    if (flag_words_dev || delta_words_dev) {
        if (fw > words_cap || dw > words_cap)
            return sfail(SKML_E_ARG, "words_cap %lld < needed %lld", (long long)words_cap, (long long)std::max(fw, dw));
        if (flag_words_dev && fw)
            SP_HIP(hipMemcpyAsync(flag_words_dev, fwd, sizeof(uint64_t) * fw, hipMemcpyDeviceToDevice, st));
        if (delta_words_dev && dw)
            SP_HIP(hipMemcpyAsync(delta_words_dev, dwd, sizeof(uint64_t) * dw, hipMemcpyDeviceToDevice, st));
        SP_HIP(hipStreamSynchronize(st));
    }
    return SKML_OK;
}

int skml_delta_decode(skml_ctx* c, int64_t n, int32_t num_intervals, int32_t flag_kind, const uint64_t* flag_words,
                      int64_t n_flag_words, const uint64_t* delta_words, int64_t n_delta_words, int32_t* keys_dev) {
    if (!c || n <= 0 || !keys_dev || !(num_intervals == 1 || num_intervals == 2 || num_intervals == 4 ||
                                       num_intervals == 8 || num_intervals == 16))
        return sfail(SKML_E_ARG, "bad delta decode arguments");
    SP_HIP(hipSetDevice(ctx_device(c)));
    hipStream_t st = ctx_stream(c);
    skml_sparse tmp;
    tmp.device = ctx_device(c);
    tmp.nnz = n;
    SpGroups& G = tmp.g;
    G.G = 1;
    G.gstart[0] = 0;
    G.gstart[1] = n;
    G.m[0] = num_intervals;
    G.kind[0] = flag_kind ? 1 : 0;
    G.fb[0] = 0;
    G.fb[1] = n_flag_words * 64;  // trailing zero words were trimmed by toLongArray
    G.db[0] = 0;
    G.db[1] = n_delta_words * 64;
    // toLongArray may trim to zero words; keep readable (zero) words behind the caller's streams
    const int64_t nfw = std::max<int64_t>(n_flag_words, 0), ndw = std::max<int64_t>(n_delta_words, 0);
    tmp.flag_words = const_cast<uint64_t*>(flag_words);
    tmp.delta_words = const_cast<uint64_t*>(delta_words);
    tmp.n_flag_words = nfw;
    tmp.n_delta_words = ndw;
    int32_t* gb = scratch<int32_t>(c, kSlotGBins, (size_t)n);
    if (!gb) return sfail(SKML_E_OOM, "delta scratch");
    if (hipMalloc(&tmp.g_dev, sizeof(SpGroups)) != hipSuccess) return sfail(SKML_E_OOM, "group table");
    int rc = upload_groups(c, &tmp);
    if (!rc) rc = decode_groups(c, &tmp, keys_dev, gb, false);
    (void)hipStreamSynchronize(st);
    (void)hipFree(tmp.g_dev);
    tmp.g_dev = nullptr;
    tmp.flag_words = tmp.delta_words = nullptr;  // caller-owned
    return rc;
}

}  // extern "C"
