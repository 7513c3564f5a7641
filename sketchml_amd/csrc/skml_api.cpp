// skml_api.cpp -- host side of the C ABI (include/skml.h): contexts, workspace, launch planning
// for the dense codec, Java-layout (de)serialisation, RCCL all-gather.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "skml_internal.h"
#include "skml_sparse.h"

using namespace skml;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(SKML_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                                \
    } while (0)

}  // namespace

// =============================================================================================
// context
// =============================================================================================
struct skml_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint64_t* jump_tab = nullptr;  // device, 4 x 256 x (A^m, C_m)
    // dense workspace (grow-only)
    void* ws = nullptr;
    size_t ws_cap = 0;
    // fp64 sketch workspace (grow-only)
    void* ws64 = nullptr;
    size_t ws64_cap = 0;
    // rank table cache for (n, bin_num): HeapQuantileSketch.getQuantiles' curFrac ranks
    int64_t* ranks = nullptr;
    size_t ranks_cap = 0;
    int64_t ranks_n = -1;
    int ranks_bins = -1;
    // batched encode: a child context (own high-priority stream and workspace) and its events
    skml_ctx* side = nullptr;
    hipEvent_t ev_join = nullptr, ev_leaf = nullptr;
    hipEvent_t ev_fork2 = nullptr, ev_join2 = nullptr;  // sparse encode: its side-stream chain
    hipEvent_t after_leaf = nullptr;  // when set, recorded right after the next leaf launch
    hipEvent_t ev_switch = nullptr;   // skml_ctx_set_stream: orders the new stream after the old one
    // parallelQuantize: slice records + the merged sketch's export (grow-only)
    void* sk = nullptr;
    size_t sk_cap = 0;
    // staging
    void* stage = nullptr;
    size_t stage_cap = 0;
    // sparse path: grow-only device scratch slots and pinned host staging
    void* scratch[kScratchSlots] = {};
    size_t scratch_cap[kScratchSlots] = {};
    void* pinned = nullptr;
    size_t pinned_cap = 0;
    // one coherent, device-mapped host word: a kernel publishes a count there (the compaction's
    // nnz) and the host polls it instead of a copy + stream synchronisation
    int64_t* hword = nullptr;
    // host-memory entry points (skml_dense_encode_host_f32 / _decode_host_f32): device copies of
    // the input / payload, two pinned staging buffers and a pool of host copy threads
    void* hx = nullptr;
    size_t hx_cap = 0;
    void* hp = nullptr;
    size_t hp_cap = 0;
    void* hk = nullptr;
    size_t hk_cap = 0;
    void* hpin[2] = {nullptr, nullptr};
    size_t hpin_cap = 0;
    hipEvent_t hev[2] = {nullptr, nullptr};
    struct CopyPool* pool = nullptr;
    // per-kernel event timing (skml_ctx_set_timing)
    int timing = 0;  // bit k: time kernel id k
    std::vector<hipEvent_t> ev[SKML_K_COUNT];  // start/stop pairs
    size_t ev_used[SKML_K_COUNT] = {};
};

namespace skml {
// Records a start event on construction and a stop event on destruction when timing is on.
struct KernelTimer {
    skml_ctx* c;
    int kid;
    bool on;
    KernelTimer(skml_ctx* ctx, int k) : c(ctx), kid(k), on((ctx->timing >> k) & 1) {
        if (!on) return;
        auto& v = c->ev[kid];
        if (c->ev_used[kid] + 2 > v.size()) {
            hipEvent_t a, b;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
                on = false;
                return;
            }
            v.push_back(a);
            v.push_back(b);
        }
        (void)hipEventRecord(v[c->ev_used[kid]], c->stream);
    }
    ~KernelTimer() {
        if (!on) return;
        (void)hipEventRecord(c->ev[kid][c->ev_used[kid] + 1], c->stream);
        c->ev_used[kid] += 2;
    }
};
KernelTimer* make_timer(skml_ctx* c, int kid) { return new KernelTimer(c, kid); }
void end_timer(KernelTimer* t) { delete t; }

// skml_debug_form's process-wide selections (read once per launch decision, no environment)
static std::atomic<int> g_form[SKML_FORM_COUNT];
int form(int id) { return id >= 0 && id < SKML_FORM_COUNT ? g_form[id].load(std::memory_order_relaxed) : 0; }
}  // namespace skml

// The forms whose kernels only the A/B build (-DSKML_AB, sketchml_amd/lib_ab) carries: measured
// slower than the default, kept for the A/B tools and the tests that load that build.
static bool ab_only_form(int id, int v) {
    switch (id) {
        case SKML_FORM_LEAF_SPLIT: return v == 1 || v >= 3;
        case SKML_FORM_DECODE_SUM: return v == 2;
        case SKML_FORM_RS_ROUNDS: return v == 2;
        case SKML_FORM_DEC_ROWS_SERIAL: return v == 2;
        case SKML_FORM_AGG_TILES: return v >= 2;
        case SKML_FORM_RUN_BOUNDS: return v != 0;
        case SKML_FORM_DEC_LOOKBACK: return v != 0;
        default: return false;
    }
}

extern "C" int skml_debug_form(int id, int value) {
    if (id < 0 || id >= SKML_FORM_COUNT) return -1;
#ifndef SKML_AB
    if (ab_only_form(id, value)) return -2;
#else
    (void)ab_only_form;
#endif
    return g_form[id].exchange(value);
}

extern "C" int skml_build_flags(void) {
#ifdef SKML_AB
    return SKML_BUILD_AB;
#else
    return 0;
#endif
}

namespace {

struct Workspace {
    unsigned* done;  // arrival counter of the fused summary (always at offset 0, self-resetting)
    LeafPartial* part;
    float* nodes6;
    float* roots;
    float* upA;
    float* upB;
    double* raw;
    QuantLut* lut;  // quantize bucket LUT, written by the summary / set-splits kernel
    UniPartial* uni;  // uniform quantizer partials
    int* qflags;      // fp64 quantize flags (bit 0: literal Quantizer.indexOf)
    uint8_t* ubits;   // compaction bits of the upper merge tree, drawn by the leaf
    LeafPartial* part_red;  // leaf partials reduced per first-pass merge workgroup
};

size_t ws_layout(int64_t chunks, Workspace* w, char* base) {
    const int64_t nwg = (chunks + kLeafChunks - 1) / kLeafChunks;
    const int64_t full = chunks / kLeafChunks;
    const int64_t up = (full >> kMergeGroupLog) + 2 * kMaxLevels + 8;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes, 256);
        return base ? (void*)(base + o) : nullptr;
    };
    Workspace t;
    t.done = (unsigned*)take(256);
    t.part = (LeafPartial*)take(sizeof(LeafPartial) * (size_t)(nwg + 1));
    t.nodes6 = (float*)take(sizeof(float) * kK * (size_t)(full + 1));
    t.roots = (float*)take(sizeof(float) * kK * kMaxLevels);
    t.upA = (float*)take(sizeof(float) * kK * (size_t)up);
    t.upB = (float*)take(sizeof(float) * kK * (size_t)up);
    t.raw = (double*)take(sizeof(double) * SKML_MAX_BINS);
    t.lut = (QuantLut*)take(sizeof(QuantLut));
    t.uni = (UniPartial*)take(sizeof(UniPartial) * kUniMaxParts);
    t.qflags = (int*)take(sizeof(int) * 4);
    t.ubits = (uint8_t*)take((size_t)upper_node_count(full * kLeafChunks) + 64);
    t.part_red = (LeafPartial*)take(sizeof(LeafPartial) * (size_t)(full + 8));
    if (w) *w = t;
    return off;
}

int ensure_ws(skml_ctx* ctx, int64_t chunks, Workspace* w) {
    const size_t need = ws_layout(chunks, nullptr, nullptr);
    if (need > ctx->ws_cap) {
        if (ctx->ws) HIP_TRY(hipFree(ctx->ws));
        ctx->ws = nullptr;
        size_t cap = need + need / 4;
        HIP_TRY(hipMalloc(&ctx->ws, cap));
        // the fused summary's arrival counter starts at 0; zeroed on the context's own stream: a
        // hipMemset goes to the null stream, which a non-blocking stream (the batch encode's side
        // lane) does not wait for, so a fresh side workspace could be counted on before it was
        // zeroed and the summary skipped (a payload without a header, tests/test_gpu_configs.py C4)
        HIP_TRY(hipMemsetAsync(ctx->ws, 0, 256, ctx->stream));
        ctx->ws_cap = cap;
    }
    ws_layout(chunks, w, (char*)ctx->ws);
    return SKML_OK;
}

struct Workspace64 {
    LeafPartial64* part;
    double* nodes6;
    double* roots;
    double* upA;
    double* upB;
    double* raw;
    uint8_t* ubits;
};

size_t ws64_layout(int64_t chunks, Workspace64* w, char* base) {
    const int64_t tiles = (chunks + kLeafChunks - 1) / kLeafChunks;
    const int64_t up = (tiles >> 3) + 8;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes, 256);
        return base ? (void*)(base + o) : nullptr;
    };
    Workspace64 t;
    t.part = (LeafPartial64*)take(sizeof(LeafPartial64) * (size_t)(tiles + 1));
    t.nodes6 = (double*)take(sizeof(double) * kK * (size_t)(tiles + 1));
    t.roots = (double*)take(sizeof(double) * kK * kMaxLevels);
    t.upA = (double*)take(sizeof(double) * kK * (size_t)up);
    t.upB = (double*)take(sizeof(double) * kK * (size_t)up);
    t.raw = (double*)take(sizeof(double) * SKML_MAX_BINS);
    t.ubits = (uint8_t*)take((size_t)upper_node_count(tiles * kLeafChunks) + 64);
    if (w) *w = t;
    return off;
}

int ensure_ws64(skml_ctx* ctx, int64_t chunks, Workspace64* w) {
    const size_t need = ws64_layout(chunks, nullptr, nullptr);
    if (need > ctx->ws64_cap) {
        if (ctx->ws64) HIP_TRY(hipFree(ctx->ws64));
        ctx->ws64 = nullptr;
        size_t cap = need + need / 4;
        HIP_TRY(hipMalloc(&ctx->ws64, cap));
        ctx->ws64_cap = cap;
    }
    ws64_layout(chunks, w, (char*)ctx->ws64);
    return SKML_OK;
}

int ensure_stage(skml_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->stage_cap) return SKML_OK;
    if (ctx->stage) HIP_TRY(hipFree(ctx->stage));
    ctx->stage = nullptr;
    HIP_TRY(hipMalloc(&ctx->stage, bytes));
    ctx->stage_cap = bytes;
    return SKML_OK;
}

// getQuantiles(int) ranks: curFrac accumulated by repeated `+= 1/B` in double
// (HeapQuantileSketch.java:304-321); depends only on (n, B) so it is planned on the host.
int ensure_ranks(skml_ctx* ctx, int64_t n, int bins) {
    if (ctx->ranks_n == n && ctx->ranks_bins == bins) return SKML_OK;
    const size_t cnt = (size_t)(bins - 1);
    if (cnt > ctx->ranks_cap) {
        if (ctx->ranks) HIP_TRY(hipFree(ctx->ranks));
        ctx->ranks = nullptr;
        HIP_TRY(hipMalloc(&ctx->ranks, sizeof(int64_t) * (cnt + 1)));
        ctx->ranks_cap = cnt;
    }
    // written on the stream ahead of the sketch (no host table, no synchronisation); the kernels
    // reading it follow on the same stream
    HIP_TRY(launch_set_ranks(ctx->stream, n, bins, ctx->ranks));
    ctx->ranks_n = n;
    ctx->ranks_bins = bins;
    return SKML_OK;
}

void build_jump_table(std::vector<uint64_t>& tab) {
    tab.assign(4 * 256 * 2, 0);
    uint64_t base_a = kLcgMult, base_c = kLcgAdd;  // J_1
    for (int lvl = 0; lvl < 4; lvl++) {
        uint64_t a = 1, c = 0;  // J_0
        for (int b = 0; b < 256; b++) {
            tab[(lvl * 256 + b) * 2] = a;
            tab[(lvl * 256 + b) * 2 + 1] = c;
            // J_{(b+1) * 256^lvl} = J_base o J_{b * 256^lvl}
            c = (base_a * c + base_c) & kLcgMask;
            a = (base_a * a) & kLcgMask;
        }
        // next base = J_base^256
        uint64_t na = 1, nc = 0;
        for (int i = 0; i < 256; i++) {
            nc = (base_a * nc + base_c) & kLcgMask;
            na = (base_a * na) & kLcgMask;
        }
        base_a = na;
        base_c = nc;
    }
}

// Plan the upper merge passes for the trees of bits >= 6 of the chunk count.
struct Tree {
    int level;           // tree level l (bit of chunks)
    int m;               // remaining log2 node count
    int cur_level;       // level of its current nodes
    int64_t src;         // first node index in the current src buffer
    int64_t chunk_base;  // first chunk
};

bool valid_payload_ptr(const void* p) { return p && (((uintptr_t)p) % 256 == 0); }

void destroy_host_path(skml_ctx* c);

}  // namespace

extern "C" {

void skml_params_default(skml_params* p) {
    p->bin_num = 256;
    p->group_num = 8;
    p->row_num = 2;
    p->dedup = 1;
    p->col_ratio = 0.3;
    p->seed = 0;
    p->hash_seed = 0;
    p->quant_type = SKML_QUANTILE;
    p->parallelism = 1;
}

const char* skml_last_error(void) { return g_err.c_str(); }
const char* skml_version(void) { return "skml-mi355x 0.1 (gfx950)"; }

int skml_ctx_create(int device, void* hip_stream, skml_ctx** out) {
    if (!out) return fail(SKML_E_ARG, "out is NULL");
    *out = nullptr;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SKML_E_ARG, "device %d of %d", device, ndev);
    HIP_TRY(hipSetDevice(device));
    skml_ctx* c = new skml_ctx();
    c->device = device;
    if (hip_stream != SKML_STREAM_OWN) {
        c->stream = (hipStream_t)hip_stream;
    } else {
        hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete c;
            return fail(SKML_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
        }
        c->own_stream = true;
    }
    std::vector<uint64_t> tab;
    build_jump_table(tab);
    hipError_t e = hipMalloc(&c->jump_tab, tab.size() * sizeof(uint64_t));
    if (e == hipSuccess)
        e = hipMemcpy(c->jump_tab, tab.data(), tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        skml_ctx_destroy(c);
        return fail(SKML_E_HIP, "jump table: %s", hipGetErrorString(e));
    }
    *out = c;
    return SKML_OK;
}

int skml_ctx_destroy(skml_ctx* c) {
    if (!c) return SKML_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->jump_tab) (void)hipFree(c->jump_tab);
    if (c->ws) (void)hipFree(c->ws);
    if (c->ws64) (void)hipFree(c->ws64);
    if (c->ranks) (void)hipFree(c->ranks);
    if (c->stage) (void)hipFree(c->stage);
    if (c->side) skml_ctx_destroy(c->side);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_leaf) (void)hipEventDestroy(c->ev_leaf);
    if (c->ev_fork2) (void)hipEventDestroy(c->ev_fork2);
    if (c->ev_join2) (void)hipEventDestroy(c->ev_join2);
    if (c->ev_switch) (void)hipEventDestroy(c->ev_switch);
    if (c->sk) (void)hipFree(c->sk);
    for (int k = 0; k < SKML_K_COUNT; k++)
        for (hipEvent_t e : c->ev[k]) (void)hipEventDestroy(e);
    for (int i = 0; i < kScratchSlots; i++)
        if (c->scratch[i]) (void)hipFree(c->scratch[i]);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->hword) (void)hipHostFree(c->hword);
    destroy_host_path(c);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return SKML_OK;
}

int skml_ctx_sync(skml_ctx* c) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SKML_OK;
}

int skml_ctx_set_timing(skml_ctx* c, int mask) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    c->timing = mask;
    return SKML_OK;
}

int skml_ctx_reset_stats(skml_ctx* c) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int k = 0; k < SKML_K_COUNT; k++) c->ev_used[k] = 0;
    return SKML_OK;
}

int skml_ctx_kernel_stats(skml_ctx* c, int kid, int64_t* launches, double* total_ms) {
    if (!c || kid < 0 || kid >= SKML_K_COUNT) return fail(SKML_E_ARG, "bad kernel id");
    HIP_TRY(hipStreamSynchronize(c->stream));
    double tot = 0.0;
    for (size_t i = 0; i + 1 < c->ev_used[kid]; i += 2) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[kid][i], c->ev[kid][i + 1]));
        tot += ms;
    }
    if (launches) *launches = (int64_t)(c->ev_used[kid] / 2);
    if (total_ms) *total_ms = tot;
    return SKML_OK;
}

int skml_debug_leaf_stage(skml_ctx* c, const float* x, int64_t n, int stage, int iters,
                          double* avg_ms) {
    if (!c || !x || n < kChunk || iters < 1 || !avg_ms) return fail(SKML_E_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t chunks = n / kChunk;
    Workspace w;
    int st = ensure_ws(c, chunks, &w);
    if (st) return st;
    const int64_t nwg = (chunks + kLeafChunks - 1) / kLeafChunks;
    if ((st = ensure_stage(c, sizeof(float) * 512 * (size_t)nwg))) return st;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(launch_leaf_stage(c->stream, stage, x, chunks, 12345, c->jump_tab, w.part,
                              (float*)c->stage, w.roots));
    HIP_TRY(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; i++)
        HIP_TRY(launch_leaf_stage(c->stream, stage, x, chunks, 12345, c->jump_tab, w.part,
                                  (float*)c->stage, w.roots));
    HIP_TRY(hipEventRecord(b, c->stream));
    HIP_TRY(hipEventSynchronize(b));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *avg_ms = ms / iters;
    return SKML_OK;
}

int skml_ctx_set_stream(skml_ctx* c, void* hip_stream) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    if (hip_stream == SKML_STREAM_OWN) return fail(SKML_E_ARG, "SKML_STREAM_OWN is only valid at creation");
    hipStream_t next = (hipStream_t)hip_stream;
    if (next == c->stream) return SKML_OK;
    HIP_TRY(hipSetDevice(c->device));
    if (c->own_stream) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipStreamDestroy(c->stream));
        c->own_stream = false;
    } else {
        // the context's workspace (merge arrival counter, LUT, stage, scratch) is reused by the next
        // call: order the new stream after everything still queued on the old one
        if (!c->ev_switch) HIP_TRY(hipEventCreateWithFlags(&c->ev_switch, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(c->ev_switch, c->stream));
        HIP_TRY(hipStreamWaitEvent(next, c->ev_switch, 0));
    }
    c->stream = next;
    return SKML_OK;
}

size_t skml_dense_payload_bytes(int64_t n, int32_t bin_num) {
    if (n < 0 || bin_num < 2 || bin_num > SKML_MAX_BINS) return 0;
    const size_t rounded = align_up((size_t)n, 1024);
    return dense_codes_offset(bin_num) + align_up(rounded * (size_t)code_bits_for(bin_num) / 8, 256);
}

static int check_dense_args(skml_ctx* c, const void* x, int64_t n, int bins, const void* payload,
                            size_t cap) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    if (n < 0 || n > 0x7FFFFFFFLL) return fail(SKML_E_ARG, "n=%lld outside Java int range", (long long)n);
    if (bins < 2 || bins > SKML_MAX_BINS)
        return fail(SKML_E_ARG, "Invalid partition number: %d", bins);  // QSketchUtils.java:40-43
    if (n > 0 && (!x || ((uintptr_t)x) % 16 != 0))
        return fail(SKML_E_ARG, "input must be a 16-byte aligned device pointer");
    if (!valid_payload_ptr(payload)) return fail(SKML_E_ARG, "payload must be 256-byte aligned");
    if (cap < skml_dense_payload_bytes(n, bins))
        return fail(SKML_E_ARG, "payload capacity %zu < %zu", cap, skml_dense_payload_bytes(n, bins));
    return SKML_OK;
}

}  // extern "C"

namespace {
// Upper merge passes for the trees of bits l >= 7 of the chunk count (bit 6 is a single leaf
// node): each pass merges up to 2^kMergeGroupLog nodes of a tree per workgroup.
std::vector<MergePass> plan_merge_passes(int64_t chunks) {
    std::vector<Tree> trees;
    for (int l = kMaxLevels - 1; l > kLeafTopLevel; l--) {
        if (!((chunks >> l) & 1)) continue;
        Tree t;
        t.level = l;
        t.m = l - kLeafTopLevel;
        t.cur_level = kLeafTopLevel;
        t.chunk_base = (chunks >> (l + 1)) << (l + 1);
        t.src = t.chunk_base >> kLeafTopLevel;
        trees.push_back(t);
    }
    std::vector<MergePass> passes;
    while (true) {
        MergePass pass;
        std::memset(&pass, 0, sizeof(pass));
        int64_t dst_off = 0;
        int wg = 0;
        for (auto& t : trees) {
            if (t.m == 0) continue;
            const int g = t.m < kMergeGroupLog ? t.m : kMergeGroupLog;
            MergeJob& j = pass.job[pass.njobs];
            j.src_node = t.src;
            j.dst_node = dst_off;
            j.chunk_base = t.chunk_base;
            j.level_in = t.cur_level;
            j.group_log = g;
            j.groups = 1 << (t.m - g);
            j.root_level = (t.m - g == 0) ? t.level : -1;
            pass.wg_prefix[pass.njobs] = wg;
            wg += j.groups;
            pass.njobs++;
            t.src = dst_off;
            dst_off += j.groups;
            t.m -= g;
            t.cur_level += g;
        }
        if (pass.njobs == 0) break;
        pass.wg_prefix[pass.njobs] = wg;
        passes.push_back(pass);
    }
    return passes;
}
// a final pass of at most kFuseMaxWg workgroup-merges runs inside the previous pass's last
// workgroup, one merge after another (sizes that are not 64^k chunks end with a few small trees:
// C3's 26.8 M values leave 2, which otherwise cost a launch of their own)
constexpr int kFuseMaxWg = 4;
bool fuse_next_pass(const std::vector<MergePass>& passes, size_t i) {
    return i + 2 == passes.size() && passes[i + 1].wg_prefix[passes[i + 1].njobs] <= kFuseMaxWg;
}
}  // namespace

namespace {
// The sketch of x[0, n): leaf + upper merge passes.  summary: the last pass's last workgroup
// also runs the summary into `payload` (returns *fused = true); otherwise the levels stay in
// w.roots and the partials in w.part for a caller-side summary or a SketchRecord.
int run_sketch_f32(skml_ctx* c, const float* x, int64_t n, uint64_t s0, const Workspace& w, const skml_params* p,
                   void* payload, bool summary, bool* fused_out) {
    const int64_t chunks = n / kChunk;
    const int64_t nwg = (chunks + kLeafChunks - 1) / kLeafChunks;  // leaf partials (one per wave tile)
    bool fused = false;
    if (chunks > 0) {
        {
            KernelTimer kt(c, SKML_K_LEAF);
            HIP_TRY(launch_leaf(c->stream, x, chunks, s0, c->jump_tab, w.part, w.nodes6, w.roots, w.ubits));
        }
        if (c->after_leaf) {
            HIP_TRY(hipEventRecord(c->after_leaf, c->stream));
            c->after_leaf = nullptr;
        }
        std::vector<MergePass> passes = plan_merge_passes(chunks);
        if (summary && !passes.empty()) passes.back().fuse_summary = 1;
        // the first pass reduces the leaf partials of the tiles it merges (every tile of the
        // trees of level >= 7: [0, 2 * (chunks >> 7))) for the summary, one per workgroup
        const int64_t nred = passes.empty() ? 0 : passes[0].wg_prefix[passes[0].njobs];
        const int64_t part_from = passes.empty() ? 0 : (chunks >> 7) << 1;
        const float* src = w.nodes6;
        float* dst = w.upA;
        for (size_t i = 0; i < passes.size(); i++) {
            const bool fuse_next = fuse_next_pass(passes, i);
            float* next_dst = (dst == w.upA) ? w.upB : w.upA;
            KernelTimer kt(c, SKML_K_MERGE);
            HIP_TRY(launch_merge_pass(c->stream, passes[i], fuse_next ? &passes[i + 1] : nullptr, src, dst, next_dst,
                                      w.roots, s0, c->jump_tab, w.done, x, n, w.part, nwg, c->ranks, p->bin_num,
                                      p->dedup ? 1 : 0, payload, w.raw, w.lut, w.ubits,
                                      summary ? w.part_red : nullptr, summary ? nred : 0, summary ? part_from : 0));
            src = dst;
            dst = next_dst;
            if (fuse_next) break;
        }
        fused = summary && !passes.empty();
    }
    *fused_out = fused;
    return SKML_OK;
}

// java.util.Random state after k more draws (affine jump-ahead by squaring)
uint64_t lcg_skip(uint64_t s, uint64_t k) {
    uint64_t a = kLcgMult, c = kLcgAdd;
    while (k) {
        if (k & 1) s = (a * s + c) & kLcgMask;
        c = (a * c + c) & kLcgMask;
        a = (a * a) & kLcgMask;
        k >>= 1;
    }
    return s;
}
// Random draws of one sketch over n updates: chunk c's leaf compaction plus its carries,
// sum over c < C of (1 + trailing_ones(c)) = 2C - popcount(C).
uint64_t sketch_draws(int64_t n) {
    const uint64_t C = (uint64_t)(n / kChunk);
    return 2 * C - (uint64_t)__builtin_popcountll(C);
}
}  // namespace

extern "C" {

int skml_dense_encode_f32(skml_ctx* c, const float* x, int64_t n, const skml_params* p,
                          void* payload, size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    HIP_TRY(hipSetDevice(c->device));
    const int64_t chunks = n / kChunk;
    Workspace w;
    if ((st = ensure_ws(c, chunks, &w))) return st;
    if ((st = ensure_ranks(c, n, p->bin_num))) return st;
    const uint64_t s0 = ((uint64_t)p->seed ^ kLcgMult) & kLcgMask;
    const int64_t nwg = (chunks + kLeafChunks - 1) / kLeafChunks;
    bool fused = false;
    if ((st = run_sketch_f32(c, x, n, s0, w, p, payload, true, &fused))) return st;
    if (!fused) {
        KernelTimer kt(c, SKML_K_SUMMARY);
        HIP_TRY(launch_summary(c->stream, x, n, w.part, nwg, w.roots, c->ranks, p->bin_num,
                               p->dedup ? 1 : 0, payload, w.raw, w.lut));
    }
    {
        KernelTimer kt(c, SKML_K_QUANTIZE);
        HIP_TRY(launch_quantize(c->stream, x, n, payload, w.lut, p->bin_num));
    }
    return SKML_OK;
}

}  // extern "C"

namespace {
struct SkScratch {
    SketchRecord* recs;  // own records (parallel path)
    float* roots;
    float* tail;
    LeafPartial* part;
};
int ensure_sk(skml_ctx* c, int nrec_own, int nrec, SkScratch* out) {
    const size_t rec_bytes = align_up(sizeof(SketchRecord) * (size_t)nrec_own, 256);
    const size_t roots_bytes = align_up(sizeof(float) * kMaxLevels * kK, 256);
    const size_t tail_bytes = align_up(sizeof(float) * kChunk, 256);
    const size_t need = rec_bytes + roots_bytes + tail_bytes + sizeof(LeafPartial) * (size_t)nrec;
    if (need > c->sk_cap) {
        if (c->sk) {
            HIP_TRY(hipStreamSynchronize(c->stream));
            HIP_TRY(hipFree(c->sk));
            c->sk = nullptr;
            c->sk_cap = 0;
        }
        if (hipMalloc(&c->sk, need) != hipSuccess) return fail(SKML_E_OOM, "sketch scratch %zu B", need);
        c->sk_cap = need;
    }
    uint8_t* b = static_cast<uint8_t*>(c->sk);
    out->recs = reinterpret_cast<SketchRecord*>(b);
    out->roots = reinterpret_cast<float*>(b + rec_bytes);
    out->tail = reinterpret_cast<float*>(b + rec_bytes + roots_bytes);
    out->part = reinterpret_cast<LeafPartial*>(b + rec_bytes + roots_bytes + tail_bytes);
    return SKML_OK;
}

int check_shards(const int64_t* shard_n, int32_t nshards, int32_t shard, int64_t n, int64_t* total,
                 uint64_t* draws_before, uint64_t* draws_all) {
    if (!shard_n || nshards < 1 || shard < 0 || shard >= nshards)
        return fail(SKML_E_ARG, "bad shard table (nshards=%d shard=%d)", nshards, shard);
    int64_t tot = 0;
    uint64_t before = 0, all = 0;
    for (int i = 0; i < nshards; i++) {
        if (shard_n[i] < 0) return fail(SKML_E_ARG, "shard %d has %lld values", i, (long long)shard_n[i]);
        tot += shard_n[i];
        if (tot > 0x7FFFFFFFLL) return fail(SKML_E_ARG, "total n=%lld outside Java int range", (long long)tot);
        if (i < shard) before += sketch_draws(shard_n[i]);
        all += sketch_draws(shard_n[i]);
    }
    if (shard_n[shard] != n)
        return fail(SKML_E_ARG, "shard %d: n=%lld but the table says %lld", shard, (long long)n,
                    (long long)shard_n[shard]);
    *total = tot;
    *draws_before = before;
    *draws_all = all;
    return SKML_OK;
}

// Sketch x[0, n) with draws starting after `skip` draws of Random(seed) into rec.
int sketch_into_record(skml_ctx* c, const float* x, int64_t n, int64_t seed, uint64_t skip, SketchRecord* rec) {
    const int64_t chunks = n / kChunk;
    Workspace w;
    int st = ensure_ws(c, chunks, &w);
    if (st) return st;
    skml_params p;
    skml_params_default(&p);
    const uint64_t s0 = lcg_skip(((uint64_t)seed ^ kLcgMult) & kLcgMask, skip);
    bool fused = false;
    if ((st = run_sketch_f32(c, x, n, s0, w, &p, nullptr, false, &fused))) return st;
    KernelTimer kt(c, SKML_K_SUMMARY);
    HIP_TRY(launch_sketch_record(c->stream, x, n, w.part, (chunks + kLeafChunks - 1) / kLeafChunks, w.roots, rec));
    return SKML_OK;
}

// Merge nrec records, summary of n_total values, quantize x[0, n).
int merge_and_quantize(skml_ctx* c, const float* x, int64_t n, const SketchRecord* recs, int nrec, int64_t n_total,
                       uint64_t draws_all, const skml_params* p, void* payload, const SkScratch& sk) {
    Workspace w;
    int st = ensure_ws(c, n / kChunk, &w);
    if (st) return st;
    if ((st = ensure_ranks(c, n_total, p->bin_num))) return st;
    const uint64_t s0 = ((uint64_t)p->seed ^ kLcgMult) & kLcgMask;
    {
        KernelTimer kt(c, SKML_K_SUMMARY);
        HIP_TRY(launch_sketch_merge(c->stream, recs, nrec, s0, draws_all, c->jump_tab, n_total, n, c->ranks,
                                    p->bin_num, p->dedup ? 1 : 0, payload, w.raw, w.lut, sk.roots, sk.tail, sk.part));
    }
    KernelTimer kt(c, SKML_K_QUANTIZE);
    HIP_TRY(launch_quantize(c->stream, x, n, payload, w.lut, p->bin_num));
    return SKML_OK;
}
}  // namespace

extern "C" {

size_t skml_sketch_record_bytes(int32_t fp64) { return fp64 ? sizeof(SketchRecord64) : sizeof(SketchRecord); }

int skml_dense_sketch_shard_f32(skml_ctx* c, const float* x, int64_t n, const int64_t* shard_n, int32_t nshards,
                                int32_t shard, int64_t seed, void* record_dev) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    if (n > 0 && (!x || ((uintptr_t)x) % 16 != 0))
        return fail(SKML_E_ARG, "input must be a 16-byte aligned device pointer");
    if (!record_dev || ((uintptr_t)record_dev) % 16 != 0)
        return fail(SKML_E_ARG, "record must be a 16-byte aligned device pointer");
    int64_t total;
    uint64_t before, all;
    int st = check_shards(shard_n, nshards, shard, n, &total, &before, &all);
    if (st) return st;
    HIP_TRY(hipSetDevice(c->device));
    return sketch_into_record(c, x, n, seed, before, static_cast<SketchRecord*>(record_dev));
}

int skml_dense_encode_sharded_f32(skml_ctx* c, const float* x, int64_t n, const int64_t* shard_n, int32_t nshards,
                                  int32_t shard, const void* records_dev, const skml_params* p, void* payload,
                                  size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        def.dedup = 0;
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    if (!records_dev || ((uintptr_t)records_dev) % 16 != 0)
        return fail(SKML_E_ARG, "records must be a 16-byte aligned device pointer");
    int64_t total;
    uint64_t before, all;
    if ((st = check_shards(shard_n, nshards, shard, n, &total, &before, &all))) return st;
    HIP_TRY(hipSetDevice(c->device));
    SkScratch sk;
    if ((st = ensure_sk(c, 0, nshards, &sk))) return st;
    return merge_and_quantize(c, x, n, static_cast<const SketchRecord*>(records_dev), nshards, total, all, p, payload,
                              sk);
}

int skml_dense_encode_parallel_f32(skml_ctx* c, const float* x, int64_t n, int32_t threads, const skml_params* p,
                                   void* payload, size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        def.dedup = 0;
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    if (threads < 1 || threads > 65536) return fail(SKML_E_ARG, "Invalid parallelism: %d", threads);
    HIP_TRY(hipSetDevice(c->device));
    // QuantileQuantizer.java:66-68: thread t takes [t*(n/T), ...), the last one the remainder
    std::vector<int64_t> shard_n((size_t)threads, n / threads);
    shard_n.back() = n - (int64_t)(threads - 1) * (n / threads);
    SkScratch sk;
    if ((st = ensure_sk(c, threads, threads, &sk))) return st;
    uint64_t skip = 0;
    for (int t = 0; t < threads; t++) {
        const float* xt = x + (int64_t)t * (n / threads);
        if ((st = sketch_into_record(c, xt, shard_n[t], p->seed, skip, sk.recs + t))) return st;
        skip += sketch_draws(shard_n[t]);
    }
    return merge_and_quantize(c, x, n, sk.recs, threads, n, skip, p, payload, sk);
}


// Independent buckets, alternately on the caller's stream and a side stream: bucket i+1's
// VALU-bound leaf runs beside bucket i's HBM-bound quantize pass (and its latency-bound merge),
// which a single stream serialises.  Ordered after earlier work on ctx's stream; ctx's stream
// waits for all buckets.  (Forking both lanes off the caller's stream with events measured no
// overlap at all when that stream is the legacy null stream.)
}  // extern "C"

// The side context: a child context on its own stream, created at high priority (HIP keeps
// hardware queues per priority, so the two never share a queue; with GPU_MAX_HW_QUEUES = 4, a
// normal-priority stream created after the framework's own streams was measured to share one and
// serialise the lanes).  Used by the batched encode and the sparse encode's DeltaAdaptive chain.
static int ensure_side(skml_ctx* c) {
    if (c->side) return SKML_OK;
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    int st = skml_ctx_create(c->device, s, &c->side);
    if (st) {
        (void)hipStreamDestroy(s);
        return st;
    }
    c->side->own_stream = true;
    HIP_TRY(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    return SKML_OK;
}

extern "C" {

int skml_dense_encode_batch_f32(skml_ctx* c, int32_t nbuckets, const float* const* xs, const int64_t* ns,
                                const skml_params* p, void* const* payloads, const size_t* caps) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    if (nbuckets < 0 || (nbuckets > 0 && (!xs || !ns || !payloads || !caps)))
        return fail(SKML_E_ARG, "bad bucket arrays (nbuckets=%d)", nbuckets);
    if (nbuckets == 0) return SKML_OK;
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        p = &def;
    }
    for (int i = 0; i < nbuckets; i++) {
        int st = check_dense_args(c, xs[i], ns[i], p->bin_num, payloads[i], caps[i]);
        if (st) return st;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (nbuckets == 1) return skml_dense_encode_f32(c, xs[0], ns[0], p, payloads[0], caps[0]);
    // Lane 0 is the caller's stream itself; lane 1 is the side context (ensure_side).
    if (int st = ensure_side(c)) return st;
    if (!c->ev_leaf) HIP_TRY(hipEventCreateWithFlags(&c->ev_leaf, hipEventDisableTiming));
    skml_ctx* lane[2] = {c, c->side};
    // lane 1 starts when bucket 0's sketch pass is done (which also orders it after earlier work
    // on the caller's stream), so the lanes stay half a bucket apart: each lane's leaf runs
    // beside the other lane's merge and quantize
    c->after_leaf = c->ev_leaf;
    for (int i = 0; i < nbuckets; i++) {
        if (i == 1) HIP_TRY(hipStreamWaitEvent(lane[1]->stream, c->ev_leaf, 0));
        int st = skml_dense_encode_f32(lane[i & 1], xs[i], ns[i], p, payloads[i], caps[i]);
        if (st) {
            c->after_leaf = nullptr;
            if (i >= 1) {  // lane 1 holds queued buckets: the caller's stream must still wait for them
                (void)hipEventRecord(c->ev_join, c->side->stream);
                (void)hipStreamWaitEvent(c->stream, c->ev_join, 0);
            }
            return st;
        }
        if (i == 0 && c->after_leaf) {  // bucket 0 had no leaf (n < 256): order lane 1 after it
            c->after_leaf = nullptr;
            HIP_TRY(hipEventRecord(c->ev_leaf, c->stream));
        }
    }
    HIP_TRY(hipEventRecord(c->ev_join, c->side->stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_join, 0));
    return SKML_OK;
}

int skml_dense_encode_with_splits_f32(skml_ctx* c, const float* x, int64_t n, const double* splits,
                                      int32_t nsplits, double mn, double mx, void* payload,
                                      size_t cap) {
    int st = check_dense_args(c, x, n, nsplits + 1, payload, cap);
    if (st) return st;
    if (!splits) return fail(SKML_E_ARG, "splits is NULL");
    for (int i = 1; i < nsplits; i++)
        if (!(splits[i - 1] <= splits[i])) return fail(SKML_E_ARG, "splits must be ascending");
    HIP_TRY(hipSetDevice(c->device));
    if ((st = ensure_stage(c, sizeof(double) * (size_t)nsplits))) return st;
    HIP_TRY(hipMemcpyAsync(c->stage, splits, sizeof(double) * (size_t)nsplits, hipMemcpyHostToDevice,
                           c->stream));
    Workspace w;
    if ((st = ensure_ws(c, 0, &w))) return st;
    HIP_TRY(launch_set_splits(c->stream, payload, n, (const double*)c->stage, nsplits, mn, mx, nsplits + 1,
                              w.lut));
    HIP_TRY(launch_quantize(c->stream, x, n, payload, w.lut, nsplits + 1));
    HIP_TRY(hipStreamSynchronize(c->stream));  // the staged splits are reused by later calls
    return SKML_OK;
}

}  // extern "C"

namespace {
// fp64 sketch of x[0, n): leaf + per-tree merge passes; levels in w.roots, partials in w.part.
int run_sketch_f64(skml_ctx* c, const double* x, int64_t n, uint64_t s0, const Workspace64& w) {
    const int64_t chunks = n / kChunk;
    {
        KernelTimer kt(c, SKML_K_LEAF);
        HIP_TRY(launch_leaf2_f64(c->stream, x, chunks, s0, c->jump_tab, w.part, w.nodes6, w.roots, w.ubits));
    }
    // upper trees: the fp32 pass plan over double nodes (k_merge64)
    const std::vector<MergePass> passes = plan_merge_passes(chunks);
    Workspace wq;  // for its self-resetting arrival counter
    if (int st = ensure_ws(c, 0, &wq)) return st;
    const double* src = w.nodes6;
    double* dst = w.upA;
    for (size_t i = 0; i < passes.size(); i++) {
        const bool fuse_next = fuse_next_pass(passes, i);
        double* next_dst = (dst == w.upA) ? w.upB : w.upA;
        KernelTimer kt(c, SKML_K_MERGE);
        HIP_TRY(launch_merge_pass64(c->stream, passes[i], fuse_next ? &passes[i + 1] : nullptr, src, dst, next_dst,
                                    w.roots, s0, c->jump_tab, wq.done, w.ubits,
                                    (chunks / kLeafChunks) * kLeafChunks));
        src = dst;
        dst = next_dst;
        if (fuse_next) break;
    }
    return SKML_OK;
}

struct SkScratch64 {
    SketchRecord64* recs;
    double* roots;
    double* tail;
    LeafPartial64* part;
};
int ensure_sk64(skml_ctx* c, int nrec_own, int nrec, SkScratch64* out) {
    const size_t rec_bytes = align_up(sizeof(SketchRecord64) * (size_t)nrec_own, 256);
    const size_t roots_bytes = align_up(sizeof(double) * kMaxLevels * kK, 256);
    const size_t tail_bytes = align_up(sizeof(double) * kChunk, 256);
    const size_t need = rec_bytes + roots_bytes + tail_bytes + sizeof(LeafPartial64) * (size_t)nrec;
    if (need > c->sk_cap) {
        if (c->sk) {
            HIP_TRY(hipStreamSynchronize(c->stream));
            HIP_TRY(hipFree(c->sk));
            c->sk = nullptr;
            c->sk_cap = 0;
        }
        if (hipMalloc(&c->sk, need) != hipSuccess) return fail(SKML_E_OOM, "sketch scratch %zu B", need);
        c->sk_cap = need;
    }
    uint8_t* b = static_cast<uint8_t*>(c->sk);
    out->recs = reinterpret_cast<SketchRecord64*>(b);
    out->roots = reinterpret_cast<double*>(b + rec_bytes);
    out->tail = reinterpret_cast<double*>(b + rec_bytes + roots_bytes);
    out->part = reinterpret_cast<LeafPartial64*>(b + rec_bytes + roots_bytes + tail_bytes);
    return SKML_OK;
}

int sketch_into_record64(skml_ctx* c, const double* x, int64_t n, int64_t seed, uint64_t skip, SketchRecord64* rec) {
    const int64_t chunks = n / kChunk;
    Workspace64 w;
    int st = ensure_ws64(c, chunks, &w);
    if (st) return st;
    const uint64_t s0 = lcg_skip(((uint64_t)seed ^ kLcgMult) & kLcgMask, skip);
    if ((st = run_sketch_f64(c, x, n, s0, w))) return st;
    KernelTimer kt(c, SKML_K_SUMMARY);
    HIP_TRY(launch_sketch_record64(c->stream, x, n, w.part, (chunks + kLeafChunks - 1) / kLeafChunks, w.roots, rec));
    return SKML_OK;
}

int merge_and_quantize64(skml_ctx* c, const double* x, int64_t n, const SketchRecord64* recs, int nrec,
                         int64_t n_total, uint64_t draws_all, const skml_params* p, void* payload,
                         const SkScratch64& sk) {
    Workspace64 w;
    int st = ensure_ws64(c, n / kChunk, &w);
    if (st) return st;
    Workspace wq;  // the quantize LUT lives in the fp32 workspace
    if ((st = ensure_ws(c, 0, &wq))) return st;
    if ((st = ensure_ranks(c, n_total, p->bin_num))) return st;
    const uint64_t s0 = ((uint64_t)p->seed ^ kLcgMult) & kLcgMask;
    {
        KernelTimer kt(c, SKML_K_SUMMARY);
        HIP_TRY(launch_sketch_merge64(c->stream, recs, nrec, s0, draws_all, c->jump_tab, sk.roots, sk.tail, sk.part));
        HIP_TRY(launch_summary64(c->stream, nullptr, n_total, sk.part, nrec, sk.roots, c->ranks, p->bin_num,
                                 p->dedup ? 1 : 0, payload, w.raw, wq.lut, sk.tail, 1, n));
    }
    KernelTimer kt(c, SKML_K_QUANTIZE);
    HIP_TRY(launch_quantize64(c->stream, x, n, payload, wq.lut, nullptr, p->bin_num));
    return SKML_OK;
}
}  // namespace

extern "C" {

int skml_dense_encode_f64(skml_ctx* c, const double* x, int64_t n, const skml_params* p, void* payload,
                          size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    HIP_TRY(hipSetDevice(c->device));
    const int64_t chunks = n / kChunk;
    Workspace64 w;
    if ((st = ensure_ws64(c, chunks, &w))) return st;
    if ((st = ensure_ranks(c, n, p->bin_num))) return st;
    const uint64_t s0 = ((uint64_t)p->seed ^ kLcgMult) & kLcgMask;
    const int64_t tiles = (chunks + kLeafChunks - 1) / kLeafChunks;
    if ((st = run_sketch_f64(c, x, n, s0, w))) return st;
    Workspace wq;  // the quantize LUT lives in the fp32 workspace
    if ((st = ensure_ws(c, 0, &wq))) return st;
    {
        KernelTimer kt(c, SKML_K_SUMMARY);
        HIP_TRY(launch_summary64(c->stream, x, n, w.part, tiles, w.roots, c->ranks, p->bin_num,
                                 p->dedup ? 1 : 0, payload, w.raw, wq.lut));
    }
    {
        KernelTimer kt(c, SKML_K_QUANTIZE);
        HIP_TRY(launch_quantize64(c->stream, x, n, payload, wq.lut, nullptr, p->bin_num));
    }
    return SKML_OK;
}

int skml_dense_sketch_shard_f64(skml_ctx* c, const double* x, int64_t n, const int64_t* shard_n, int32_t nshards,
                                int32_t shard, int64_t seed, void* record_dev) {
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    if (n > 0 && (!x || ((uintptr_t)x) % 16 != 0))
        return fail(SKML_E_ARG, "input must be a 16-byte aligned device pointer");
    if (!record_dev || ((uintptr_t)record_dev) % 16 != 0)
        return fail(SKML_E_ARG, "record must be a 16-byte aligned device pointer");
    int64_t total;
    uint64_t before, all;
    int st = check_shards(shard_n, nshards, shard, n, &total, &before, &all);
    if (st) return st;
    HIP_TRY(hipSetDevice(c->device));
    return sketch_into_record64(c, x, n, seed, before, static_cast<SketchRecord64*>(record_dev));
}

int skml_dense_encode_sharded_f64(skml_ctx* c, const double* x, int64_t n, const int64_t* shard_n, int32_t nshards,
                                  int32_t shard, const void* records_dev, const skml_params* p, void* payload,
                                  size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        def.dedup = 0;
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    if (!records_dev || ((uintptr_t)records_dev) % 16 != 0)
        return fail(SKML_E_ARG, "records must be a 16-byte aligned device pointer");
    int64_t total;
    uint64_t before, all;
    if ((st = check_shards(shard_n, nshards, shard, n, &total, &before, &all))) return st;
    HIP_TRY(hipSetDevice(c->device));
    SkScratch64 sk;
    if ((st = ensure_sk64(c, 0, nshards, &sk))) return st;
    return merge_and_quantize64(c, x, n, static_cast<const SketchRecord64*>(records_dev), nshards, total, all, p,
                                payload, sk);
}

int skml_dense_encode_parallel_f64(skml_ctx* c, const double* x, int64_t n, int32_t threads, const skml_params* p,
                                   void* payload, size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        def.dedup = 0;
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    if (threads < 1 || threads > 65536) return fail(SKML_E_ARG, "Invalid parallelism: %d", threads);
    HIP_TRY(hipSetDevice(c->device));
    std::vector<int64_t> shard_n((size_t)threads, n / threads);
    shard_n.back() = n - (int64_t)(threads - 1) * (n / threads);
    SkScratch64 sk;
    if ((st = ensure_sk64(c, threads, threads, &sk))) return st;
    uint64_t skip = 0;
    for (int t = 0; t < threads; t++) {
        const double* xt = x + (int64_t)t * (n / threads);
        if ((st = sketch_into_record64(c, xt, shard_n[t], p->seed, skip, sk.recs + t))) return st;
        skip += sketch_draws(shard_n[t]);
    }
    return merge_and_quantize64(c, x, n, sk.recs, threads, n, skip, p, payload, sk);
}

int skml_dense_encode_uniform_f32(skml_ctx* c, const float* x, int64_t n, const skml_params* p, void* payload,
                                  size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    HIP_TRY(hipSetDevice(c->device));
    Workspace w;
    if ((st = ensure_ws(c, 0, &w))) return st;
    {
        KernelTimer kt(c, SKML_K_SUMMARY);
        HIP_TRY(launch_uniform(c->stream, x, n, p->bin_num, w.uni, payload, w.lut, w.qflags));
    }
    {
        KernelTimer kt(c, SKML_K_QUANTIZE);
        HIP_TRY(launch_quantize(c->stream, x, n, payload, w.lut, p->bin_num));
    }
    return SKML_OK;
}

int skml_dense_encode_uniform_f64(skml_ctx* c, const double* x, int64_t n, const skml_params* p, void* payload,
                                  size_t cap) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        p = &def;
    }
    int st = check_dense_args(c, x, n, p->bin_num, payload, cap);
    if (st) return st;
    HIP_TRY(hipSetDevice(c->device));
    Workspace w;
    if ((st = ensure_ws(c, 0, &w))) return st;
    {
        KernelTimer kt(c, SKML_K_SUMMARY);
        HIP_TRY(launch_uniform64(c->stream, x, n, p->bin_num, w.uni, payload, w.lut, w.qflags));
    }
    {
        KernelTimer kt(c, SKML_K_QUANTIZE);
        HIP_TRY(launch_quantize64(c->stream, x, n, payload, w.lut, w.qflags, p->bin_num));
    }
    return SKML_OK;
}

int skml_dense_decode_f64(skml_ctx* c, const void* payload, double* out, int64_t n) {
    if (!c || !valid_payload_ptr(payload) || (n > 0 && (!out || ((uintptr_t)out) % 16)))
        return fail(SKML_E_ARG, "bad decode arguments");
    HIP_TRY(hipSetDevice(c->device));
    KernelTimer kt(c, SKML_K_DECODE);
    HIP_TRY(launch_decode64(c->stream, payload, out, n));
    return SKML_OK;
}

int skml_dense_decode_f32(skml_ctx* c, const void* payload, float* out, int64_t n) {
    if (!c || !valid_payload_ptr(payload) || (n > 0 && (!out || ((uintptr_t)out) % 16)))
        return fail(SKML_E_ARG, "bad decode arguments");
    HIP_TRY(hipSetDevice(c->device));
    KernelTimer kt(c, SKML_K_DECODE);
    HIP_TRY(launch_decode(c->stream, payload, out, n));
    return SKML_OK;
}

int skml_dense_decode_sum_f32(skml_ctx* c, const void* payloads, int32_t P, size_t stride, float* out,
                              int64_t n, double scale) {
    if (!c || !valid_payload_ptr(payloads) || stride % 256 || P < 1 || P > 16 ||
        (n > 0 && (!out || ((uintptr_t)out) % 16)))
        return fail(SKML_E_ARG, "bad decode_sum arguments (P in [1,16], 256-B aligned payloads)");
    HIP_TRY(hipSetDevice(c->device));
    // Gradient.sum adds gradients of one dimension (ml/gradient/Gradient.scala:44-49): every
    // payload must be a finished dense payload of exactly n codes that fits its stride.
    skml_dense_header h[16];
    HIP_TRY(hipMemcpy2DAsync(h, sizeof(skml_dense_header), payloads, stride, sizeof(skml_dense_header), (size_t)P,
                             hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int p = 0; p < P; p++) {
        if (h[p].magic != SKML_DENSE_MAGIC) return fail(SKML_E_STATE, "payload %d is not a dense payload", p);
        if (h[p].status == SKML_E_NAN) return fail(SKML_E_NAN, "payload %d: Encounter NaN value", p);
        if (h[p].status != SKML_OK) return fail(SKML_E_STATE, "payload %d has status %d", p, h[p].status);
        if (h[p].n != n)
            return fail(SKML_E_ARG, "payload %d holds %lld values, the sum %lld", p, (long long)h[p].n, (long long)n);
        if (h[p].bin_num < 2 || h[p].bin_num > SKML_MAX_BINS || h[p].code_bits != code_bits_for(h[p].bin_num) ||
            h[p].bin_num > h[p].req_bins || h[p].codes_offset != (int64_t)dense_codes_offset(h[p].req_bins) ||
            skml_dense_payload_bytes(n, h[p].req_bins) > stride)
            return fail(SKML_E_ARG, "payload %d: inconsistent header or larger than the stride %zu", p, stride);
    }
    int common_bits = h[0].code_bits, max_bins = h[0].bin_num;
    for (int p = 1; p < P; p++) {
        if (h[p].code_bits != common_bits) common_bits = 0;
        max_bins = std::max(max_bins, (int)h[p].bin_num);
    }
    KernelTimer kt(c, SKML_K_DECODE_SUM);
    HIP_TRY(launch_decode_sum(c->stream, payloads, P, stride, out, n, scale, common_bits, max_bins));
    return SKML_OK;
}

int skml_dense_bins_i32(skml_ctx* c, const void* payload, int32_t* bins, int64_t n) {
    if (!c || !valid_payload_ptr(payload) || (n > 0 && !bins)) return fail(SKML_E_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(launch_bins(c->stream, payload, bins, n));
    return SKML_OK;
}

int skml_dense_info(skml_ctx* c, const void* payload, skml_dense_header* hdr, double* splits,
                    int32_t splits_cap) {
    if (!c || !valid_payload_ptr(payload) || !hdr) return fail(SKML_E_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(hdr, payload, sizeof(*hdr), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (hdr->magic != SKML_DENSE_MAGIC) return fail(SKML_E_STATE, "not a dense payload");
    if (splits && hdr->status == SKML_OK) {
        const int ns = hdr->bin_num - 1;
        if (ns > splits_cap) return fail(SKML_E_ARG, "splits capacity %d < %d", splits_cap, ns);
        HIP_TRY(hipMemcpyAsync(splits, (const char*)payload + kHeaderBytes, sizeof(double) * ns,
                               hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    if (hdr->status == SKML_E_NAN) return fail(SKML_E_NAN, "Encounter NaN value");
    return hdr->status;
}

int skml_dense_times_by(skml_ctx* c, void* payload, double x) {
    if (!c || !valid_payload_ptr(payload)) return fail(SKML_E_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(launch_times_by(c->stream, payload, x));
    return SKML_OK;
}

static void put_be(uint8_t* p, uint64_t v, int nb) {
    for (int i = nb - 1; i >= 0; i--) {
        p[i] = (uint8_t)(v & 0xFF);
        v >>= 8;
    }
}
static uint64_t get_be(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
    return v;
}
static uint64_t dbl_bits(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}

int skml_dense_serialize_ref(skml_ctx* c, const void* payload, uint8_t* buf, size_t cap, size_t* written) {
    skml_dense_header h;
    std::vector<double> sp(SKML_MAX_BINS);
    int st = skml_dense_info(c, payload, &h, sp.data(), SKML_MAX_BINS);
    if (st) return st;
    const int B = h.bin_num, ns = B - 1;
    const int width = B <= 256 ? 1 : (B <= 65536 ? 2 : 4);
    const size_t head = 4 + 4 + 8 * (size_t)ns + 4 + 8 + 8 + 4;
    const size_t total = head + (size_t)width * (size_t)h.n;
    if (written) *written = total;
    if (!buf) return SKML_OK;
    if (cap < total) return fail(SKML_E_ARG, "buffer capacity %zu < %zu", cap, total);
    uint8_t* p = buf;
    put_be(p, (uint32_t)B, 4); p += 4;
    put_be(p, (uint32_t)h.n, 4); p += 4;
    for (int i = 0; i < ns; i++) { put_be(p, dbl_bits(sp[i]), 8); p += 8; }
    put_be(p, (uint32_t)h.zero_idx, 4); p += 4;
    put_be(p, dbl_bits(h.min), 8); p += 8;
    put_be(p, dbl_bits(h.max), 8); p += 8;
    put_be(p, (uint32_t)h.n, 4); p += 4;
    if (h.n > 0) {
        if ((st = ensure_stage(c, (size_t)width * (size_t)h.n))) return st;
        HIP_TRY(launch_ref_body(c->stream, payload, (uint8_t*)c->stage, h.n, width));
        HIP_TRY(hipMemcpyAsync(p, c->stage, (size_t)width * (size_t)h.n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return SKML_OK;
}

int skml_dense_deserialize_ref(skml_ctx* c, const uint8_t* buf, size_t len, void* payload, size_t cap) {
    if (!c || !buf || !valid_payload_ptr(payload)) return fail(SKML_E_ARG, "bad arguments");
    if (len < 8) return fail(SKML_E_ARG, "truncated stream");
    const uint8_t* p = buf;
    const int32_t B = (int32_t)get_be(p, 4);
    const int32_t n = (int32_t)get_be(p + 4, 4);
    if (B < 2 || B > SKML_MAX_BINS || n < 0) return fail(SKML_E_ARG, "bad binNum %d / n %d", B, n);
    const int ns = B - 1;
    const int width = B <= 256 ? 1 : (B <= 65536 ? 2 : 4);
    const size_t head = 4 + 4 + 8 * (size_t)ns + 4 + 8 + 8 + 4;
    if (len < head) return fail(SKML_E_ARG, "truncated stream");
    p += 8;
    std::vector<double> sp(ns);
    for (int i = 0; i < ns; i++) {
        uint64_t u = get_be(p, 8);
        std::memcpy(&sp[i], &u, 8);
        p += 8;
    }
    skml_dense_header h;
    std::memset(&h, 0, sizeof(h));
    h.magic = SKML_DENSE_MAGIC;
    h.status = SKML_OK;
    h.zero_idx = (int32_t)get_be(p, 4); p += 4;
    uint64_t u = get_be(p, 8); std::memcpy(&h.min, &u, 8); p += 8;
    u = get_be(p, 8); std::memcpy(&h.max, &u, 8); p += 8;
    const int32_t nb = (int32_t)get_be(p, 4); p += 4;
    if (nb != n || len < head + (size_t)width * (size_t)n) return fail(SKML_E_ARG, "truncated bins");
    if (cap < skml_dense_payload_bytes(n, B)) return fail(SKML_E_ARG, "payload too small");
    // Quantizer.findZeroIdx only yields indices of bins (Quantizer.java:74-85)
    if (h.zero_idx < 0 || h.zero_idx >= B) return fail(SKML_E_ARG, "zeroIdx %d outside [0, %d)", h.zero_idx, B);
    h.n = n;
    h.bin_num = B;
    h.code_bits = code_bits_for(B);
    h.req_bins = B;
    h.codes_offset = (int64_t)dense_codes_offset(B);
    HIP_TRY(hipSetDevice(c->device));
    const size_t body = align_up((size_t)width * (size_t)n, 16);
    int st = ensure_stage(c, body + 16);
    if (st) return st;
    int* bad = reinterpret_cast<int*>((char*)c->stage + body);
    HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int), c->stream));
    HIP_TRY(hipMemcpyAsync(payload, &h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    if (ns) HIP_TRY(hipMemcpyAsync((char*)payload + kHeaderBytes, sp.data(), sizeof(double) * ns,
                                   hipMemcpyHostToDevice, c->stream));
    if (n) {
        HIP_TRY(hipMemcpyAsync(c->stage, p, (size_t)width * (size_t)n, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(launch_pack_ref(c->stream, (const uint8_t*)c->stage, width, n, payload, bad));
    }
    int nbad = 0;
    HIP_TRY(hipMemcpyAsync(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (nbad) {
        // leave no usable payload behind
        const uint32_t zero = 0;
        HIP_TRY(hipMemcpy(payload, &zero, sizeof(zero), hipMemcpyHostToDevice));
        return fail(SKML_E_ARG, "bin outside [0, %d) in the stream", B);
    }
    return SKML_OK;
}

// =============================================================================================
// RCCL all-gather of payloads over xGMI
// =============================================================================================
struct skml_comm {
    ncclComm_t comm;
    int nranks, rank;
};

int skml_comm_unique_id(uint8_t id_out[SKML_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) <= SKML_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(SKML_E_RCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    std::memset(id_out, 0, SKML_UNIQUE_ID_BYTES);
    std::memcpy(id_out, &id, sizeof(id));
    return SKML_OK;
}

int skml_comm_init_rank(skml_ctx* c, const uint8_t id_in[SKML_UNIQUE_ID_BYTES], int32_t nranks,
                        int32_t rank, skml_comm** out) {
    if (!c || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(SKML_E_ARG, "bad comm args");
    HIP_TRY(hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, id_in, sizeof(id));
    skml_comm* cm = new skml_comm();
    ncclResult_t r = ncclCommInitRank(&cm->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        delete cm;
        return fail(SKML_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    cm->nranks = nranks;
    cm->rank = rank;
    *out = cm;
    return SKML_OK;
}

int skml_comm_destroy(skml_comm* cm) {
    if (!cm) return SKML_OK;
    ncclCommDestroy(cm->comm);
    delete cm;
    return SKML_OK;
}

int skml_allgather(skml_ctx* c, skml_comm* cm, const void* payload, size_t bytes, void* all) {
    if (!c || !cm || !payload || !all) return fail(SKML_E_ARG, "bad allgather arguments");
    HIP_TRY(hipSetDevice(c->device));
    ncclResult_t r = ncclAllGather(payload, all, bytes, ncclUint8, cm->comm, c->stream);
    if (r != ncclSuccess) return fail(SKML_E_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
    return SKML_OK;
}

}  // extern "C"

// =============================================================================================
// Host-memory entry points: the path starts and ends in a JVM float[] / byte[] (north star).
// Pageable host memory is staged through two library-owned pinned buffers: host threads copy
// piece i+1 into one while the DMA engine moves piece i out of the other, so the pageable copy
// runs beside the PCIe transfer instead of before it.  Pinned caller memory (skml_host_alloc,
// e.g. behind a Java direct ByteBuffer) is transferred directly.
// =============================================================================================
struct CopyPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::function<void(int)> job;
    int parts = 0, next = 0, done = 0;
    uint64_t gen = 0;
    bool stop = false;
    explicit CopyPool(int n) {
        for (int i = 0; i < n; i++) th.emplace_back([this] { run(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
    void run() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(m);
        while (true) {
            cv.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            while (next < parts) {
                const int k = next++;
                lk.unlock();
                job(k);
                lk.lock();
                if (++done == parts) done_cv.notify_all();
            }
        }
    }
    // f(0..parts-1) on the pool plus the calling thread; returns when all are done
    void parallel(int nparts, const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> lk(m);
        job = f;
        parts = nparts;
        next = 0;
        done = 0;
        gen++;
        cv.notify_all();
        while (next < parts) {
            const int k = next++;
            lk.unlock();
            f(k);
            lk.lock();
            if (++done == parts) done_cv.notify_all();
        }
        done_cv.wait(lk, [&] { return done == parts; });
        parts = 0;
    }
};

namespace {

constexpr size_t kHostPiece = 8u << 20;  // bytes per staged piece

void destroy_host_path(skml_ctx* c) {
    delete c->pool;
    c->pool = nullptr;
    for (int b = 0; b < 2; b++) {
        if (c->hpin[b]) (void)hipHostFree(c->hpin[b]);
        if (c->hev[b]) (void)hipEventDestroy(c->hev[b]);
        c->hpin[b] = nullptr;
        c->hev[b] = nullptr;
    }
    if (c->hx) (void)hipFree(c->hx);
    if (c->hp) (void)hipFree(c->hp);
    if (c->hk) (void)hipFree(c->hk);
    c->hx = c->hp = c->hk = nullptr;
}

int ensure_dev_buf(void** p, size_t* cap, size_t bytes, hipStream_t st) {
    if (bytes <= *cap) return SKML_OK;
    if (*p) {
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipFree(*p));
        *p = nullptr;
        *cap = 0;
    }
    const size_t want = align_up(bytes, 1u << 20);
    if (hipMalloc(p, want) != hipSuccess) {
        (void)hipGetLastError();
        return fail(SKML_E_OOM, "device buffer of %zu B", want);
    }
    *cap = want;
    return SKML_OK;
}

int ensure_host_path(skml_ctx* c) {
    if (!c->hpin[0] || !c->hpin[1] || !c->hev[0] || !c->hev[1]) {
        // all four or nothing: a partial setup is freed so the next call starts over
        auto undo = [c]() {
            for (int b = 0; b < 2; b++) {
                if (c->hpin[b]) (void)hipHostFree(c->hpin[b]);
                if (c->hev[b]) (void)hipEventDestroy(c->hev[b]);
                c->hpin[b] = nullptr;
                c->hev[b] = nullptr;
            }
            c->hpin_cap = 0;
            (void)hipGetLastError();
        };
        undo();
        for (int b = 0; b < 2; b++) {
            if (hipHostMalloc(&c->hpin[b], kHostPiece, hipHostMallocDefault) != hipSuccess) {
                c->hpin[b] = nullptr;
                undo();
                return fail(SKML_E_OOM, "pinned staging of %zu B", kHostPiece);
            }
            if (hipEventCreateWithFlags(&c->hev[b], hipEventDisableTiming) != hipSuccess) {
                c->hev[b] = nullptr;
                undo();
                return fail(SKML_E_HIP, "staging event");
            }
        }
        c->hpin_cap = kHostPiece;
    }
    if (!c->pool) {
        int n = 4;  // host copy threads besides the caller (SKML_HOST_THREADS overrides)
        if (const char* e = std::getenv("SKML_HOST_THREADS")) n = std::max(0, std::min(64, std::atoi(e)));
        c->pool = new CopyPool(n);
    }
    return SKML_OK;
}

// memcpy on the pool, split into cache-friendly slices
void pool_copy(skml_ctx* c, void* dst, const void* src, size_t bytes) {
    const size_t slice = 1u << 20;
    const int parts = (int)((bytes + slice - 1) / slice);
    if (parts <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    c->pool->parallel(parts, [&](int k) {
        const size_t o = (size_t)k * slice, len = std::min(slice, bytes - o);
        std::memcpy((char*)dst + o, (const char*)src + o, len);
    });
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // a plain pageable pointer: not an error for us
        return false;
    }
    return a.type == hipMemoryTypeHost && a.hostPointer != nullptr;
}

// host -> device, staged through the pinned pair unless the source is pinned itself
int upload(skml_ctx* c, void* dev, const void* host, size_t bytes) {
    if (!bytes) return SKML_OK;
    if (is_pinned(host)) {
        HIP_TRY(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, c->stream));
        return SKML_OK;
    }
    size_t off = 0;
    for (int i = 0; off < bytes; i++) {
        const int b = i & 1;
        const size_t len = std::min(kHostPiece, bytes - off);
        // the DMA out of buffer b (this call's piece i-2, or an earlier call's last pieces) is done
        HIP_TRY(hipEventSynchronize(c->hev[b]));
        pool_copy(c, c->hpin[b], (const char*)host + off, len);
        HIP_TRY(hipMemcpyAsync((char*)dev + off, c->hpin[b], len, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->hev[b], c->stream));
        off += len;
    }
    return SKML_OK;
}

// device -> host (synchronous: returns with the bytes in `host`)
int download(skml_ctx* c, void* host, const void* dev, size_t bytes) {
    if (!bytes) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        return SKML_OK;
    }
    if (is_pinned(host)) {
        HIP_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return SKML_OK;
    }
    const size_t pieces = (bytes + kHostPiece - 1) / kHostPiece;
    auto issue = [&](size_t i) -> int {
        const int b = (int)(i & 1);
        const size_t off = i * kHostPiece, len = std::min(kHostPiece, bytes - off);
        HIP_TRY(hipMemcpyAsync(c->hpin[b], (const char*)dev + off, len, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipEventRecord(c->hev[b], c->stream));
        return SKML_OK;
    };
    int st = issue(0);
    if (!st && pieces > 1) st = issue(1);
    for (size_t i = 0; i < pieces && !st; i++) {
        const int b = (int)(i & 1);
        const size_t off = i * kHostPiece, len = std::min(kHostPiece, bytes - off);
        HIP_TRY(hipEventSynchronize(c->hev[b]));
        pool_copy(c, (char*)host + off, c->hpin[b], len);
        if (i + 2 < pieces) st = issue(i + 2);
    }
    return st;
}

}  // namespace

extern "C" {

int skml_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(SKML_E_ARG, "out is NULL");
    *out = nullptr;
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(SKML_E_OOM, "pinned host allocation of %zu B", bytes);
    }
    return SKML_OK;
}

int skml_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return SKML_OK;
}

}  // extern "C"

namespace {

// the device payload written by an encode on device buffers -> bytes in use (header, splits, codes)
size_t payload_used(const skml_dense_header& h) {
    return (size_t)h.codes_offset + ((size_t)h.n * (size_t)h.code_bits + 7) / 8;
}

// A host payload's header, checked for self-consistency against its length.
int host_header(const void* payload, size_t len, skml_dense_header* h, bool need_ok = true) {
    if (!payload || len < sizeof(skml_dense_header)) return fail(SKML_E_ARG, "payload too short");
    std::memcpy(h, payload, sizeof(*h));
    if (h->magic != SKML_DENSE_MAGIC) return fail(SKML_E_STATE, "not a dense payload");
    if (need_ok && h->status == SKML_E_NAN) return fail(SKML_E_NAN, "Encounter NaN value");
    if (need_ok && h->status != SKML_OK) return fail(SKML_E_STATE, "payload status %d", h->status);
    if (h->n < 0 || h->n > 0x7FFFFFFFLL || h->bin_num < 2 || h->bin_num > h->req_bins || h->req_bins > SKML_MAX_BINS ||
        h->code_bits != code_bits_for(h->bin_num) || h->codes_offset != (int64_t)dense_codes_offset(h->req_bins) ||
        h->zero_idx < 0 || h->zero_idx >= h->bin_num)
        return fail(SKML_E_ARG, "inconsistent payload header");
    if (h->status == SKML_OK && len < payload_used(*h))
        return fail(SKML_E_ARG, "payload of %zu B, header needs %zu", len, payload_used(*h));
    return SKML_OK;
}

template <typename T, typename Encode>
int encode_host(skml_ctx* c, const T* x, int64_t n, const skml_params* p, void* payload, size_t cap, size_t* written,
                Encode encode) {
    skml_params def;
    if (!p) {
        skml_params_default(&def);
        p = &def;
    }
    if (!c) return fail(SKML_E_ARG, "ctx is NULL");
    if (n < 0 || n > 0x7FFFFFFFLL) return fail(SKML_E_ARG, "n=%lld outside Java int range", (long long)n);
    if (p->bin_num < 2 || p->bin_num > SKML_MAX_BINS) return fail(SKML_E_ARG, "Invalid partition number: %d", p->bin_num);
    const size_t nb = skml_dense_payload_bytes(n, p->bin_num);
    if (!payload) {  // size query: an upper bound of the bytes written
        if (written) *written = nb;
        return SKML_OK;
    }
    if (n > 0 && !x) return fail(SKML_E_ARG, "x is NULL");
    HIP_TRY(hipSetDevice(c->device));
    int st;
    if ((st = ensure_host_path(c))) return st;
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, std::max<size_t>(16, sizeof(T) * (size_t)n), c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hp, &c->hp_cap, nb, c->stream))) return st;
    if ((st = upload(c, c->hx, x, sizeof(T) * (size_t)n))) return st;
    if ((st = encode(c, (const T*)c->hx, n, p, c->hp, c->hp_cap))) return st;
    skml_dense_header h;
    HIP_TRY(hipMemcpyAsync(&h, c->hp, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (h.status == SKML_E_NAN) return fail(SKML_E_NAN, "Encounter NaN value");
    const size_t used = payload_used(h);
    if (written) *written = used;
    if (cap < used) return fail(SKML_E_ARG, "payload capacity %zu < %zu", cap, used);
    return download(c, payload, c->hp, used);
}

template <typename T, typename Decode>
int decode_host(skml_ctx* c, const void* payload, size_t len, T* out, int64_t n, Decode decode) {
    if (!c || (n > 0 && !out)) return fail(SKML_E_ARG, "bad arguments");
    skml_dense_header h;
    int st = host_header(payload, len, &h);
    if (st) return st;
    if (h.n != n) return fail(SKML_E_ARG, "payload holds %lld values, asked for %lld", (long long)h.n, (long long)n);
    HIP_TRY(hipSetDevice(c->device));
    if ((st = ensure_host_path(c))) return st;
    if ((st = ensure_dev_buf(&c->hp, &c->hp_cap, skml_dense_payload_bytes(n, h.req_bins), c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, std::max<size_t>(16, sizeof(T) * (size_t)n), c->stream))) return st;
    if ((st = upload(c, c->hp, payload, payload_used(h)))) return st;
    if ((st = decode(c, c->hp, (T*)c->hx, n))) return st;
    return download(c, out, c->hx, sizeof(T) * (size_t)n);
}

}  // namespace

extern "C" {

// params->quant_type = SKML_UNIFORM selects UniformQuantizer (Quantizer.newQuantizer's switch,
// base/Quantizer.java:126-136, as on the sparse path); otherwise params->parallelism > 1 selects
// QuantileQuantizer.parallelQuantize with that many slices, else quantize.
int skml_dense_encode_host_f32(skml_ctx* c, const float* x, int64_t n, const skml_params* p, void* payload,
                               size_t cap, size_t* written) {
    return encode_host<float>(c, x, n, p, payload, cap, written,
                              [](skml_ctx* c2, const float* xd, int64_t m, const skml_params* q, void* pl, size_t cp) {
                                  return q->quant_type == SKML_UNIFORM ? skml_dense_encode_uniform_f32(c2, xd, m, q, pl, cp)
                                         : q->parallelism > 1
                                             ? skml_dense_encode_parallel_f32(c2, xd, m, q->parallelism, q, pl, cp)
                                             : skml_dense_encode_f32(c2, xd, m, q, pl, cp);
                              });
}

int skml_dense_encode_host_f64(skml_ctx* c, const double* x, int64_t n, const skml_params* p, void* payload,
                               size_t cap, size_t* written) {
    return encode_host<double>(c, x, n, p, payload, cap, written,
                               [](skml_ctx* c2, const double* xd, int64_t m, const skml_params* q, void* pl, size_t cp) {
                                   return q->quant_type == SKML_UNIFORM ? skml_dense_encode_uniform_f64(c2, xd, m, q, pl, cp)
                                          : q->parallelism > 1
                                              ? skml_dense_encode_parallel_f64(c2, xd, m, q->parallelism, q, pl, cp)
                                              : skml_dense_encode_f64(c2, xd, m, q, pl, cp);
                               });
}

int skml_dense_decode_host_f32(skml_ctx* c, const void* payload, size_t len, float* out, int64_t n) {
    return decode_host<float>(c, payload, len, out, n, skml_dense_decode_f32);
}

int skml_dense_decode_host_f64(skml_ctx* c, const void* payload, size_t len, double* out, int64_t n) {
    return decode_host<double>(c, payload, len, out, n, skml_dense_decode_f64);
}

int skml_dense_info_host(const void* payload, size_t len, skml_dense_header* hdr, double* splits, int32_t cap) {
    if (!hdr) return fail(SKML_E_ARG, "hdr is NULL");
    int st = host_header(payload, len, hdr, false);
    if (st) return st;
    if (hdr->status == SKML_E_NAN) return fail(SKML_E_NAN, "Encounter NaN value");
    if (splits) {
        const int ns = hdr->bin_num - 1;
        if (ns > cap) return fail(SKML_E_ARG, "splits capacity %d < %d", cap, ns);
        std::memcpy(splits, (const char*)payload + kHeaderBytes, sizeof(double) * (size_t)ns);
    }
    return hdr->status;
}

int skml_dense_bins_host(const void* payload, size_t len, int32_t* bins, int64_t n) {
    skml_dense_header h;
    int st = host_header(payload, len, &h);
    if (st) return st;
    if (h.n != n || (n > 0 && !bins)) return fail(SKML_E_ARG, "bins of %lld values, payload holds %lld", (long long)n,
                                                  (long long)h.n);
    const uint8_t* codes = (const uint8_t*)payload + h.codes_offset;
    const int b = h.code_bits;
    for (int64_t e = 0; e < n; e++) {  // LSB-first packed codes (include/skml.h)
        const uint64_t bit = (uint64_t)e * (uint64_t)b;
        uint32_t v;
        if (b == 16) v = (uint32_t)codes[2 * e] | ((uint32_t)codes[2 * e + 1] << 8);
        else v = (codes[bit >> 3] >> (bit & 7)) & ((1u << b) - 1u);
        bins[e] = (int32_t)v;
    }
    return SKML_OK;
}

int skml_dense_times_by_host(void* payload, size_t len, double x) {
    skml_dense_header h;
    int st = host_header(payload, len, &h);
    if (st) return st;
    double* sp = reinterpret_cast<double*>((char*)payload + kHeaderBytes);  // Quantizer.timesBy (:119-124)
    for (int i = 0; i < h.bin_num - 1; i++) sp[i] *= x;
    h.min *= x;
    h.max *= x;
    std::memcpy(payload, &h, sizeof(h));
    return SKML_OK;
}

int skml_sparse_encode_kv_host_f32(skml_ctx* c, const int32_t* keys, const float* vals, int64_t nnz,
                                   const skml_params* p, skml_sparse** out) {
    if (!c || !out || nnz < 0 || (nnz > 0 && (!keys || !vals))) return fail(SKML_E_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    int st;
    const size_t bytes = std::max<size_t>(16, 4 * (size_t)nnz);
    if ((st = ensure_host_path(c))) return st;
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, bytes, c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hk, &c->hk_cap, bytes, c->stream))) return st;
    if ((st = upload(c, c->hk, keys, 4 * (size_t)nnz))) return st;
    if ((st = upload(c, c->hx, vals, 4 * (size_t)nnz))) return st;
    return skml_sparse_encode_kv_f32(c, (const int32_t*)c->hk, (const float*)c->hx, nnz, p, out);
}

int skml_sparse_encode_kv_host_f64(skml_ctx* c, const int32_t* keys, const double* vals, int64_t nnz,
                                   const skml_params* p, skml_sparse** out) {
    if (!c || !out || nnz < 0 || (nnz > 0 && (!keys || !vals))) return fail(SKML_E_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    int st;
    if ((st = ensure_host_path(c))) return st;
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, std::max<size_t>(16, 8 * (size_t)nnz), c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hk, &c->hk_cap, std::max<size_t>(16, 4 * (size_t)nnz), c->stream))) return st;
    if ((st = upload(c, c->hk, keys, 4 * (size_t)nnz))) return st;
    if ((st = upload(c, c->hx, vals, 8 * (size_t)nnz))) return st;
    return skml_sparse_encode_kv_f64(c, (const int32_t*)c->hk, (const double*)c->hx, nnz, p, out);
}

}  // extern "C"

namespace {
template <typename T, typename Dec>
int sparse_decode_host(skml_ctx* c, const skml_sparse* s, int32_t* keys, T* vals, Dec dec) {
    int64_t n = 0;
    if (!c || !s || skml_sparse_nnz(s, &n)) return fail(SKML_E_ARG, "bad arguments");
    if (n > 0 && (!keys || !vals)) return fail(SKML_E_ARG, "keys/vals are NULL");
    HIP_TRY(hipSetDevice(c->device));
    int st;
    if ((st = ensure_host_path(c))) return st;
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, std::max<size_t>(16, sizeof(T) * (size_t)n), c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hk, &c->hk_cap, std::max<size_t>(16, 4 * (size_t)n), c->stream))) return st;
    if ((st = dec(c, s, (int32_t*)c->hk, (T*)c->hx))) return st;
    if ((st = download(c, keys, c->hk, 4 * (size_t)n))) return st;
    return download(c, vals, c->hx, sizeof(T) * (size_t)n);
}
}  // namespace

extern "C" {

int skml_sparse_decode_host_f32(skml_ctx* c, const skml_sparse* s, int32_t* keys, float* vals) {
    return sparse_decode_host<float>(c, s, keys, vals, skml_sparse_decode_f32);
}

int skml_sparse_decode_host_f64(skml_ctx* c, const skml_sparse* s, int32_t* keys, double* vals) {
    return sparse_decode_host<double>(c, s, keys, vals, skml_sparse_decode_f64);
}

int skml_delta_encode_host(skml_ctx* c, const int32_t* keys, int64_t n, int32_t* num_intervals, int32_t* flag_kind,
                           int64_t* n_flag_bits, int64_t* n_delta_bits, uint64_t* flag_words, uint64_t* delta_words,
                           int64_t words_cap) {
    if (!c || n <= 0 || !keys) return fail(SKML_E_ARG, "bad delta arguments");
    HIP_TRY(hipSetDevice(c->device));
    int st;
    if ((st = ensure_host_path(c))) return st;
    // a stream never exceeds 33 bits per key (16-bit flags are at most 4 bits, deltas at most 32)
    const size_t wcap = ((size_t)n * 33 + 63) / 64 + 1;
    if ((st = ensure_dev_buf(&c->hk, &c->hk_cap, 4 * (size_t)n, c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, 8 * wcap, c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hp, &c->hp_cap, 8 * wcap, c->stream))) return st;
    if ((st = upload(c, c->hk, keys, 4 * (size_t)n))) return st;
    int64_t nfb = 0, ndb = 0;
    if ((st = skml_delta_encode(c, (const int32_t*)c->hk, n, num_intervals, flag_kind, &nfb, &ndb, (uint64_t*)c->hx,
                                (uint64_t*)c->hp, (int64_t)wcap)))
        return st;
    if (n_flag_bits) *n_flag_bits = nfb;
    if (n_delta_bits) *n_delta_bits = ndb;
    const int64_t fw = (nfb + 63) / 64, dw = (ndb + 63) / 64;
    if (!flag_words && !delta_words) return SKML_OK;
    if (fw > words_cap || dw > words_cap)
        return fail(SKML_E_ARG, "words_cap %lld < needed %lld", (long long)words_cap, (long long)std::max(fw, dw));
    if (flag_words && (st = download(c, flag_words, c->hx, 8 * (size_t)fw))) return st;
    if (delta_words && (st = download(c, delta_words, c->hp, 8 * (size_t)dw))) return st;
    return SKML_OK;
}

int skml_delta_decode_host(skml_ctx* c, int64_t n, int32_t num_intervals, int32_t flag_kind, const uint64_t* flag_words,
                           int64_t n_flag_words, const uint64_t* delta_words, int64_t n_delta_words, int32_t* keys) {
    if (!c || n <= 0 || !keys || n_flag_words < 0 || n_delta_words < 0 || (n_flag_words && !flag_words) ||
        (n_delta_words && !delta_words))
        return fail(SKML_E_ARG, "bad delta decode arguments");
    HIP_TRY(hipSetDevice(c->device));
    int st;
    if ((st = ensure_host_path(c))) return st;
    // zero words past the trimmed streams (BitSet.toLongArray drops trailing zero words)
    const size_t fpad = 8 * ((size_t)n_flag_words + 64), dpad = 8 * ((size_t)n_delta_words + 64);
    if ((st = ensure_dev_buf(&c->hx, &c->hx_cap, fpad, c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hp, &c->hp_cap, dpad, c->stream))) return st;
    if ((st = ensure_dev_buf(&c->hk, &c->hk_cap, 4 * (size_t)n, c->stream))) return st;
    HIP_TRY(hipMemsetAsync(c->hx, 0, fpad, c->stream));
    HIP_TRY(hipMemsetAsync(c->hp, 0, dpad, c->stream));
    if ((st = upload(c, c->hx, flag_words, 8 * (size_t)n_flag_words))) return st;
    if ((st = upload(c, c->hp, delta_words, 8 * (size_t)n_delta_words))) return st;
    if ((st = skml_delta_decode(c, n, num_intervals, flag_kind, (const uint64_t*)c->hx, n_flag_words,
                                (const uint64_t*)c->hp, n_delta_words, (int32_t*)c->hk)))
        return st;
    return download(c, keys, c->hk, 4 * (size_t)n);
}

}  // extern "C"

// ---- accessors used by the sparse translation unit ----
namespace skml {
hipStream_t ctx_stream(skml_ctx* c) { return c->stream; }
int ctx_side_fork(skml_ctx* c, hipStream_t* side, hipEvent_t* fork, hipEvent_t* join) {
    // SKML_SERIAL=1 (profiling): no fork, every kernel runs alone on the caller's stream
    static const bool serial = [] {
        const char* e = std::getenv("SKML_SERIAL");
        return e && e[0] == '1';
    }();
    if (serial) return SKML_E_STATE;
    if (int st = ensure_side(c)) return st;
    if (!c->ev_fork2) HIP_TRY(hipEventCreateWithFlags(&c->ev_fork2, hipEventDisableTiming));
    if (!c->ev_join2) HIP_TRY(hipEventCreateWithFlags(&c->ev_join2, hipEventDisableTiming));
    *side = c->side->stream;
    *fork = c->ev_fork2;
    *join = c->ev_join2;
    return SKML_OK;
}
skml_ctx* ctx_side_ctx(skml_ctx* c) { return c->side; }
int ctx_device(skml_ctx* c) { return c->device; }
int set_error(int code, const char* msg) { return fail(code, "%s", msg); }
bool ctx_timing(skml_ctx* c) { return c->timing != 0; }
void* ctx_scratch(skml_ctx* c, int slot, size_t bytes) {
    if (slot < 0 || slot >= kScratchSlots) return nullptr;
    if (bytes == 0) bytes = 256;
    if (bytes > c->scratch_cap[slot]) {
        if (c->scratch[slot]) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(c->scratch[slot]);
        }
        c->scratch[slot] = nullptr;
        c->scratch_cap[slot] = 0;
        const size_t cap = align_up(bytes + bytes / 8, 256);
        if (hipMalloc(&c->scratch[slot], cap) != hipSuccess) return nullptr;
        c->scratch_cap[slot] = cap;
    }
    return c->scratch[slot];
}
int64_t* ctx_host_word(skml_ctx* c) {
    if (!c->hword) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        c->hword = static_cast<int64_t*>(p);
    }
    return c->hword;
}
void* ctx_pinned(skml_ctx* c, size_t bytes) {
    if (bytes > c->pinned_cap) {
        if (c->pinned) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipHostFree(c->pinned);
        }
        c->pinned = nullptr;
        c->pinned_cap = 0;
        const size_t cap = align_up(bytes + bytes / 8 + 4096, 4096);
        if (hipHostMalloc(&c->pinned, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        c->pinned_cap = cap;
    }
    return c->pinned;
}
}  // namespace skml
