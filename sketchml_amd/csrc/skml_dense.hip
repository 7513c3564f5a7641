// skml_dense.hip -- CDNA4 (gfx950) kernels of the dense gradient codec.
//
//   k_leaf       one pass over the fp32 gradient: per 256-value chunk an in-register bitonic sort
//                + RNG compaction (HeapQuantileSketch.fullBaseBufferPropagation,
//                HeapQuantileSketch.java:107-124), then the first six levels of the fixed merge
//                tree (QSketchUtils.levelwisePropagation, QSketchUtils.java:71-82) in registers /
//                LDS; min/max/NaN partials.  HBM-bound: reads 4 B per value, writes 1/128 of it.
//   k_merge      upper tree levels, 64 nodes per workgroup, exact reference tie rule.
//   k_summary    one workgroup: makeSummary + getQuantiles(int) + Maths.unique + findZeroIdx
//                (HeapQuantileSketch.java:126-174,293-323; Maths.java:51-67; Quantizer.java:74-85)
//   k_quantize   bins = indexOf(x) (Quantizer.java:49-92) as a branchless Eytzinger search over an
//                LDS split table, packed codes.  HBM-bound: 4 B in + code_bits/8 out per value.
//   k_decode     values[bins[i]] (DenseVectorCompressor.java:84-91), LUT in LDS.
#include "skml_device.hpp"

namespace skml {

// =============================================================================================
// Leaf kernel: 512 threads = 8 waves; wave w owns chunks [c0 + 8w, c0 + 8w + 8); lane group
// g = lane/8 holds chunk g as 32 keys per lane.  Output: the level-6 node of the 64 chunks (or,
// in the last partial workgroup, the roots of the small trees of chunks mod 64).
// =============================================================================================
struct LeafShared {
    float fb[kLeafWaves][1024];     // per-wave exact-merge area (rare path: mixed +/-0)
    float wn[kLeafWaves][kK];       // level-3 nodes of the waves
    float l4[4][kK];
    float l5[2][kK];
    float l6[kK];
    uint64_t mask[kLeafWaves];      // RNG bits [start, start+64) of each wave's chunk range
    uint64_t start[kLeafWaves];
    uint32_t min_key, max_key, flags;
};

// Exact path for one in-wave merge level: runs in registers (R keys / lane, G = 256/R lanes per
// merge group) -> LDS -> reference-rule merge + compaction -> registers (R/2 keys / lane).
template <int R>
__device__ __forceinline__ void wave_exact_level(uint32_t (&v)[R], uint32_t (&w)[R / 2], int lane,
                                                 uint32_t odd, float* fb) {
    constexpr int G = 256 / R;
    const int grp = lane / G, li = lane % G;
    float* run = fb + grp * 256;
#pragma unroll
    for (int r = 0; r < R; r++) run[li * R + r] = __uint_as_float(key2f(v[r]));
    int pos[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int p = li * R + r;
        const float x = __uint_as_float(key2f(v[r]));
        pos[r] = p < 128 ? p + count_le(run + 128, x) : (p - 128) + count_lt(run, x);
    }
    float* out = fb + grp * 128;  // in place: every read of this wave precedes every write
#pragma unroll
    for (int r = 0; r < R; r++)
        if (((uint32_t)pos[r] & 1u) == odd) out[pos[r] >> 1] = __uint_as_float(key2f(v[r]));
#pragma unroll
    for (int j = 0; j < R / 2; j++) w[j] = f2key(__float_as_uint(out[li * (R / 2) + j]));
}

// Export the node held in registers (G lanes x R keys, positions li*R + r) if it is the root
// of one of the small trees of the last partial workgroup.
template <int R>
__device__ __forceinline__ void export_wave_root(const uint32_t (&w)[R], int lane, int level,
                                                 int64_t wave_c0, int64_t wg_c0, int rem,
                                                 float* roots) {
    if (!rem || !((rem >> level) & 1)) return;
    constexpr int G = kK / R;
    const int64_t cs = wg_c0 + (((int64_t)rem >> (level + 1)) << (level + 1));
    const int64_t my_cs = wave_c0 + (int64_t)(lane / G) * ((int64_t)1 << level);
    if (my_cs != cs) return;
    float* dst = roots + (size_t)level * kK;
    const int li = lane % G;
#pragma unroll
    for (int r = 0; r < R; r++) dst[li * R + r] = __uint_as_float(key2f(w[r]));
}

// STAGE < 3 are truncated variants used only by skml_debug_leaf (profiling ablation).
template <int STAGE>
__global__ __launch_bounds__(512) void k_leaf(const float* __restrict__ x, int64_t chunks,
                                              uint64_t s0, const uint64_t* __restrict__ tab,
                                              LeafPartial* __restrict__ part,
                                              float* __restrict__ nodes6,
                                              float* __restrict__ roots) {
    __shared__ LeafShared sh;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int64_t wg_c0 = (int64_t)blockIdx.x * kLeafChunks;
    const int64_t wave_c0 = wg_c0 + wave * kChunksPerWave;
    const int64_t chunk = wave_c0 + (lane >> 3);
    const int rem = (wg_c0 + kLeafChunks > chunks) ? (int)(chunks - wg_c0) : 0;
    const bool valid = chunk < chunks;

    if (tid == 0) {
        sh.min_key = 0xFFFFFFFFu;
        sh.max_key = 0u;
        sh.flags = 0u;
    }
    __syncthreads();

    // ---- load 32 values: 8 x float4, each 8-lane group reads a full 128-B line per load ----
    uint32_t v[32];
    uint32_t mn = 0xFFFFFFFFu, mx = 0u, fl = 0u;
    {
        const float4* src = reinterpret_cast<const float4*>(x + (valid ? chunk : 0) * kChunk);
        float4 f[8];
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = src[j * 8 + (lane & 7)];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t b[4] = {__float_as_uint(f[j].x), __float_as_uint(f[j].y),
                                   __float_as_uint(f[j].z), __float_as_uint(f[j].w)};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                fl |= is_nan_bits(b[e]) ? 1u : 0u;
                fl |= (b[e] == 0x80000000u) ? 2u : 0u;
                fl |= (b[e] == 0u) ? 4u : 0u;
                const uint32_t k = f2key(b[e]);
                mn = k < mn ? k : mn;
                mx = k > mx ? k : mx;
                v[j * 4 + e] = k;
            }
        }
        if (!valid) fl = 0u;
    }

    // ---- compaction bits for the wave's chunk range: lane l computes draw #(start + l) ----
    const uint64_t start = node_bit_index((uint64_t)wave_c0, 0);
    uint64_t mask;
    {
        const uint64_t s_start = lcg_jump(tab, s0, start + 1);
        const uint64_t a = tab[lane * 2], c = tab[lane * 2 + 1];  // level-0 table: A^lane, C_lane
        const uint64_t s = (lane == 0) ? s_start : ((a * s_start + c) & kLcgMask);
        mask = __ballot((s >> 47) & 1ull);
    }
    if (lane == 0) {
        sh.mask[wave] = mask;
        sh.start[wave] = start;
    }
    if constexpr (STAGE == 0) {
        uint32_t acc = mn ^ mx ^ fl ^ (uint32_t)mask;
#pragma unroll
        for (int r = 0; r < 32; r++) acc ^= v[r];
        nodes6[(size_t)blockIdx.x * 512 + tid] = __uint_as_float(acc);
        return;
    }

    // ---- leaf: sort the chunk (Arrays.sort total order) and keep every other sample ----
    sort_group256<32>(v, lane);
    uint32_t w1[16];
    {
        const uint32_t odd = (uint32_t)(mask >> (node_bit_index((uint64_t)chunk, 0) - start)) & 1u;
        compact_regs<32>(v, w1, odd);
    }
    export_wave_root<16>(w1, lane, 0, wave_c0, wg_c0, rem, roots);
    if constexpr (STAGE == 1) {
        uint32_t acc = mn ^ mx ^ fl;
#pragma unroll
        for (int r = 0; r < 16; r++) acc ^= w1[r];
        nodes6[(size_t)blockIdx.x * 512 + tid] = __uint_as_float(acc);
        return;
    }

    // In-register bitonic merges equal the reference merge (IEEE `<`, ties -> newer run) unless
    // the wave's values contain both -0.0 and +0.0; then take the exact LDS path.
    const bool neg0 = __ballot((fl & 2u) != 0) != 0, pos0 = __ballot((fl & 4u) != 0) != 0;
    const bool exact = neg0 && pos0;
    float* fb = sh.fb[wave];

    uint32_t w2[8], w3[4], w4[2];
    {  // level 1: 16-lane groups
        const uint64_t c = (uint64_t)wave_c0 + (uint64_t)((lane >> 4) + 1) * 2 - 1;
        const uint32_t odd = (uint32_t)(mask >> (node_bit_index(c, 1) - start)) & 1u;
        if (!exact) {
            merge_group<16>(w1, lane);
            compact_regs<16>(w1, w2, odd);
        } else {
            wave_exact_level<16>(w1, w2, lane, odd, fb);
        }
    }
    export_wave_root<8>(w2, lane, 1, wave_c0, wg_c0, rem, roots);
    {  // level 2: 32-lane groups
        const uint64_t c = (uint64_t)wave_c0 + (uint64_t)((lane >> 5) + 1) * 4 - 1;
        const uint32_t odd = (uint32_t)(mask >> (node_bit_index(c, 2) - start)) & 1u;
        if (!exact) {
            merge_group<8>(w2, lane);
            compact_regs<8>(w2, w3, odd);
        } else {
            wave_exact_level<8>(w2, w3, lane, odd, fb);
        }
    }
    export_wave_root<4>(w3, lane, 2, wave_c0, wg_c0, rem, roots);
    {  // level 3: the whole wave
        const uint64_t c = (uint64_t)wave_c0 + 7;
        const uint32_t odd = (uint32_t)(mask >> (node_bit_index(c, 3) - start)) & 1u;
        if (!exact) {
            merge_group<4>(w3, lane);
            compact_regs<4>(w3, w4, odd);
        } else {
            wave_exact_level<4>(w3, w4, lane, odd, fb);
        }
    }
    if constexpr (STAGE == 2) {
        nodes6[(size_t)blockIdx.x * 512 + tid] = __uint_as_float(w4[0] ^ w4[1] ^ mn ^ mx ^ fl);
        return;
    }
    sh.wn[wave][lane * 2] = __uint_as_float(key2f(w4[0]));
    sh.wn[wave][lane * 2 + 1] = __uint_as_float(key2f(w4[1]));

    // ---- partial min / max / flags ----
    if (valid) {
        atomicMin(&sh.min_key, mn);
        atomicMax(&sh.max_key, mx);
        if (fl) atomicOr(&sh.flags, fl);
    }
    __syncthreads();

    // ---- levels 4..6 across waves (exact reference merge in LDS) ----
    auto wg_bit = [&](int level, int node) -> uint32_t {
        const int64_t last = wg_c0 + ((int64_t)(node + 1) << level) - 1;
        const int wv = (int)((last - wg_c0) >> 3);
        return (uint32_t)(sh.mask[wv] >> (node_bit_index((uint64_t)last, level) - sh.start[wv])) & 1u;
    };
    for (int task = tid; task < 4 * 256; task += 512) {
        const int m = task >> 8;
        exact_merge_task(sh.wn[2 * m], sh.wn[2 * m + 1], sh.l4[m], task & 255, wg_bit(4, m));
    }
    __syncthreads();
    {
        const int m = tid >> 8;
        exact_merge_task(sh.l4[2 * m], sh.l4[2 * m + 1], sh.l5[m], tid & 255, wg_bit(5, m));
    }
    __syncthreads();
    if (tid < 256) exact_merge_task(sh.l5[0], sh.l5[1], sh.l6, tid, wg_bit(6, 0));
    __syncthreads();

    if (!rem) {
        if (tid < kK) {
            nodes6[(size_t)blockIdx.x * kK + tid] = sh.l6[tid];
            // a level-6 tree (bit 6 of the chunk count) is this single node
            if (((chunks >> 6) & 1) && (int64_t)blockIdx.x == ((chunks >> 7) << 1))
                roots[(size_t)6 * kK + tid] = sh.l6[tid];
        }
    } else if (tid < kK) {
        // roots of levels 3..5 live in LDS
        for (int level = 3; level <= 5; level++) {
            if (!((rem >> level) & 1)) continue;
            const int cs = (rem >> (level + 1)) << (level + 1);  // chunk offset in workgroup
            const float* src = level == 3 ? sh.wn[cs >> 3] : (level == 4 ? sh.l4[cs >> 4] : sh.l5[cs >> 5]);
            roots[(size_t)level * kK + tid] = src[tid];
        }
    }
    if (tid == 0) {
        LeafPartial p;
        p.min_key = sh.min_key;
        p.max_key = sh.max_key;
        p.flags = sh.flags;
        p.pad = 0;
        part[blockIdx.x] = p;
    }
}

hipError_t launch_leaf(hipStream_t st, const float* x, int64_t chunks, uint64_t s0,
                       const uint64_t* jump_tab, LeafPartial* part, float* nodes6, float* roots) {
    const int64_t nwg = (chunks + kLeafChunks - 1) / kLeafChunks;
    if (nwg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_leaf<3>, dim3((unsigned)nwg), dim3(512), 0, st, x, chunks, s0, jump_tab,
                       part, nodes6, roots);
    return hipGetLastError();
}

// Profiling ablation: stage 0 = load + keys, 1 = + leaf sort/compaction, 2 = + in-wave merges,
// 3 = full kernel.  `scratch` must hold nwg * 512 floats.
hipError_t launch_leaf_stage(hipStream_t st, int stage, const float* x, int64_t chunks, uint64_t s0,
                             const uint64_t* jump_tab, LeafPartial* part, float* scratch, float* roots) {
    const int64_t nwg = (chunks + kLeafChunks - 1) / kLeafChunks;
    if (nwg <= 0) return hipSuccess;
    dim3 g((unsigned)nwg), b(512);
    switch (stage) {
        case 0: hipLaunchKernelGGL(k_leaf<0>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        case 1: hipLaunchKernelGGL(k_leaf<1>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        case 2: hipLaunchKernelGGL(k_leaf<2>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        default: hipLaunchKernelGGL(k_leaf<3>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
    }
    return hipGetLastError();
}

// =============================================================================================
// Upper merge levels: each workgroup merges 2^g consecutive nodes of one tree (g <= 6) with
// the exact reference merge, RNG bit per node by jump-ahead.
// =============================================================================================
__global__ __launch_bounds__(256) void k_merge(MergePass pass, const float* __restrict__ src,
                                               float* __restrict__ dst, float* __restrict__ roots,
                                               uint64_t s0, const uint64_t* __restrict__ tab) {
    __shared__ float bufA[64 * kK];
    __shared__ float bufB[32 * kK];
    int j = 0;
    while (j + 1 < pass.njobs && (int)blockIdx.x >= pass.wg_prefix[j + 1]) j++;
    const MergeJob job = pass.job[j];
    const int grp = (int)blockIdx.x - pass.wg_prefix[j];
    const int cnt = 1 << job.group_log;
    const float* in = src + (size_t)(job.src_node + (int64_t)grp * cnt) * kK;
    for (int i = threadIdx.x; i < cnt * kK; i += 256) bufA[i] = in[i];
    __syncthreads();
    const int64_t chunk0 = job.chunk_base + (((int64_t)grp * cnt) << job.level_in);
    float* a = bufA;
    float* b = bufB;
    for (int step = 1; step <= job.group_log; step++) {
        const int nm = cnt >> step;
        const int lvl = job.level_in + step;
        for (int task = threadIdx.x; task < nm * 256; task += 256) {
            const int m = task >> 8;
            const int64_t last = chunk0 + ((int64_t)(m + 1) << lvl) - 1;
            const uint32_t odd = lcg_bit(tab, s0, node_bit_index((uint64_t)last, lvl));
            exact_merge_task(a + (2 * m) * kK, a + (2 * m + 1) * kK, b + m * kK, task & 255, odd);
        }
        __syncthreads();
        float* t = a;
        a = b;
        b = t;
    }
    float* out = job.root_level >= 0 ? roots + (size_t)job.root_level * kK
                                     : dst + (size_t)(job.dst_node + grp) * kK;
    if (threadIdx.x < kK) out[threadIdx.x] = a[threadIdx.x];
}

hipError_t launch_merge_pass(hipStream_t st, const MergePass& pass, const float* src, float* dst,
                             float* roots, uint64_t s0, const uint64_t* jump_tab) {
    const int nwg = pass.wg_prefix[pass.njobs];
    if (nwg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_merge, dim3(nwg), dim3(256), 0, st, pass, src, dst, roots, s0, jump_tab);
    return hipGetLastError();
}

// =============================================================================================
// Summary: one workgroup of 1024 threads.
// =============================================================================================
constexpr int kSumThreads = 1024;
constexpr int kMaxSamples = kMaxLevels * kK + kChunk;

__device__ __forceinline__ int run_count_le(const float* r, int len, float x) {
    int lo = 0, hi = len;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (r[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int run_count_lt(const float* r, int len, float x) {
    int lo = 0, hi = len;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (r[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Block-wide exclusive scan of one int64 per thread.
__device__ int64_t block_exclusive_scan(int64_t v, int64_t* tmp, int64_t* total) {
    const int t = threadIdx.x;
    tmp[t] = v;
    __syncthreads();
    for (int off = 1; off < kSumThreads; off <<= 1) {
        int64_t add = t >= off ? tmp[t - off] : 0;
        __syncthreads();
        tmp[t] += add;
        __syncthreads();
    }
    const int64_t incl = tmp[t];
    if (total) *total = tmp[kSumThreads - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(kSumThreads) void k_summary(
    const float* __restrict__ x, int64_t n, const LeafPartial* __restrict__ part, int64_t nparts,
    const float* __restrict__ roots, const int64_t* __restrict__ ranks, int req_bins, int dedup,
    uint8_t* __restrict__ payload, double* __restrict__ g_raw) {
    __shared__ float s_smp[kMaxSamples];     // gathered runs
    __shared__ float g_samples[kMaxSamples]; // samplesArr after blockyMergeSort
    __shared__ int64_t g_w[kMaxSamples + 1]; // weightsArr -> cut points
    __shared__ int64_t s_scan[kSumThreads];
    __shared__ uint32_t s_min, s_max, s_flags;
    __shared__ int s_zero;
    __shared__ int64_t s_total;
    __shared__ int s_run_off[kMaxLevels + 2];
    __shared__ int s_run_lvl[kMaxLevels + 2];
    __shared__ int s_nruns;

    skml_dense_header* hdr = reinterpret_cast<skml_dense_header*>(payload);
    double* splits = reinterpret_cast<double*>(payload + kHeaderBytes);
    const int t = threadIdx.x;
    const int64_t chunks = n / kChunk;
    const int tail = (int)(n - chunks * kChunk);
    const float* xt = x + chunks * kChunk;

    if (t == 0) {
        s_min = 0xFFFFFFFFu;
        s_max = 0u;
        s_flags = 0u;
        s_zero = 0x7FFFFFFF;
    }
    __syncthreads();
    // ---- min / max / NaN ----
    {
        uint32_t mn = 0xFFFFFFFFu, mx = 0u, fl = 0u;
        for (int64_t i = t; i < nparts; i += kSumThreads) {
            const LeafPartial p = part[i];
            mn = p.min_key < mn ? p.min_key : mn;
            mx = p.max_key > mx ? p.max_key : mx;
            fl |= p.flags;
        }
        for (int i = t; i < tail; i += kSumThreads) {
            const uint32_t b = __float_as_uint(xt[i]);
            fl |= is_nan_bits(b) ? 1u : 0u;
            const uint32_t k = f2key(b);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
        atomicMin(&s_min, mn);
        atomicMax(&s_max, mx);
        atomicOr(&s_flags, fl);
    }
    // ---- run table: level roots (lowest level first, HeapQuantileSketch.copyBuf2Arr), tail ----
    if (t == 0) {
        int nr = 0, off = 0;
        for (int l = 0; l < kMaxLevels; l++)
            if ((chunks >> l) & 1) {
                s_run_off[nr] = off;
                s_run_lvl[nr] = l;
                nr++;
                off += kK;
            }
        s_run_off[nr] = off;       // tail run
        s_run_lvl[nr] = -1;
        s_run_off[nr + 1] = off + tail;
        s_nruns = nr + 1;
    }
    __syncthreads();
    const int nruns = s_nruns;
    const int ns = s_run_off[nruns];
    const uint32_t flags = s_flags;

    double vmin = 1.7976931348623157e308, vmax = 4.9e-324;  // HeapQuantileSketch.java:67-68
    if (n > 0) {
        const double fmin = (double)__uint_as_float(key2f(s_min));
        const double fmax = (double)__uint_as_float(key2f(s_max));
        if (fmin <= vmin) vmin = fmin;  // Math.min(Double.MAX_VALUE, x)
        if (fmax > vmax) vmax = fmax;   // Math.max(Double.MIN_VALUE, x): ties keep MIN_VALUE
    }
    if (flags & 1u) {  // NaN: QuantileSketchException("Encounter NaN value")
        if (t == 0) {
            hdr->magic = SKML_DENSE_MAGIC;
            hdr->status = SKML_E_NAN;
            hdr->n = n;
            hdr->bin_num = req_bins;
            hdr->zero_idx = 0;
            hdr->code_bits = code_bits_for(req_bins);
            hdr->req_bins = req_bins;
            hdr->min = vmin;
            hdr->max = vmax;
            hdr->codes_offset = (int64_t)dense_codes_offset(req_bins);
            hdr->reserved = 0;
        }
        return;
    }

    // ---- gather runs; the tail is sorted in Arrays.sort total order by rank counting ----
    for (int r = 0; r + 1 < nruns; r++) {
        const float* src = roots + (size_t)s_run_lvl[r] * kK;
        for (int i = t; i < kK; i += kSumThreads) s_smp[s_run_off[r] + i] = src[i];
    }
    {
        const int toff = s_run_off[nruns - 1];
        for (int i = t; i < tail; i += kSumThreads) {
            const uint32_t ki = f2key(__float_as_uint(xt[i]));
            int rank = 0;
            for (int j = 0; j < tail; j++) {
                const uint32_t kj = f2key(__float_as_uint(xt[j]));
                rank += (kj < ki) || (kj == ki && j < i);
            }
            s_smp[toff + rank] = xt[i];
        }
    }
    __syncthreads();

    // ---- blockyMergeSort == stable sort under IEEE `<=` (left wins): rank across runs ----
    for (int i = t; i < ns; i += kSumThreads) {
        int r = 0;
        while (s_run_off[r + 1] <= i) r++;
        const float v = s_smp[i];
        int rank = i - s_run_off[r];
        for (int q = 0; q < nruns; q++) {
            if (q == r) continue;
            const float* run = s_smp + s_run_off[q];
            const int len = s_run_off[q + 1] - s_run_off[q];
            rank += q < r ? run_count_le(run, len, v) : run_count_lt(run, len, v);
        }
        g_samples[rank] = v;
        g_w[rank] = s_run_lvl[r] < 0 ? 1 : ((int64_t)2 << s_run_lvl[r]);
    }
    __syncthreads();

    // ---- exclusive prefix of weights (weightsArr cut points, HeapQuantileSketch.java:137-142) ----
    {
        const int per = (ns + kSumThreads - 1) / kSumThreads;
        const int b0 = t * per, b1 = min(ns, b0 + per);
        int64_t loc = 0;
        for (int i = b0; i < b1; i++) loc += g_w[i];
        const int64_t base = block_exclusive_scan(loc, s_scan, &s_total);
        int64_t acc = base;
        for (int i = b0; i < b1; i++) {
            const int64_t wv = g_w[i];
            g_w[i] = acc;
            acc += wv;
        }
        if (t == 0) g_w[ns] = s_total;
        __syncthreads();
    }

    // ---- getQuantiles(int): split_i = samples[max idx with prefix[idx] <= rank_i] ----
    const int nsplit_req = req_bins - 1;
    for (int i = t; i < nsplit_req; i += kSumThreads) {
        double sp;
        if (ns == 0) {
            sp = __longlong_as_double(0x7FF8000000000000LL);  // NaN (HeapQuantileSketch.java:299-301)
        } else {
            const int64_t rank = ranks[i];
            int lo = 0, hi = ns;  // largest lo in [0, ns) with w[lo] <= rank
            while (lo + 1 < hi) {
                const int mid = (lo + hi) >> 1;
                if (g_w[mid] <= rank) lo = mid;
                else hi = mid;
            }
            sp = (double)g_samples[lo];
        }
        g_raw[i] = sp;
    }
    __threadfence();
    __syncthreads();

    // ---- Maths.unique (IEEE !=, keep first) + findZeroIdx ----
    int bin_num;
    {
        const int per = (nsplit_req + kSumThreads - 1) / kSumThreads;
        const int b0 = t * per, b1 = min(nsplit_req, b0 + per);
        int64_t loc = 0;
        for (int i = b0; i < b1; i++) loc += (!dedup || i == 0 || g_raw[i] != g_raw[i - 1]) ? 1 : 0;
        const int64_t base = block_exclusive_scan(loc, s_scan, &s_total);
        int64_t o = base;
        for (int i = b0; i < b1; i++) {
            if (!dedup || i == 0 || g_raw[i] != g_raw[i - 1]) {
                const double sp = g_raw[i];
                splits[o] = sp;
                if (!(sp < 0.0)) atomicMin(&s_zero, (int)o);
                o++;
            }
        }
        bin_num = (int)s_total + 1;
    }
    __syncthreads();
    if (t == 0) {
        int zero;
        if (vmin > 0.0) zero = 0;
        else if (vmax < 0.0) zero = bin_num - 1;
        else zero = s_zero < bin_num - 1 ? s_zero : bin_num - 1;
        hdr->magic = SKML_DENSE_MAGIC;
        hdr->status = SKML_OK;
        hdr->n = n;
        hdr->bin_num = bin_num;
        hdr->zero_idx = zero;
        hdr->code_bits = code_bits_for(bin_num);
        hdr->req_bins = req_bins;
        hdr->min = vmin;
        hdr->max = vmax;
        hdr->codes_offset = (int64_t)dense_codes_offset(req_bins);
        hdr->reserved = 0;
    }
}

hipError_t launch_summary(hipStream_t st, const float* x, int64_t n, const LeafPartial* part,
                          int64_t nparts, const float* roots, const int64_t* ranks, int req_bins,
                          int dedup, void* payload, double* scratch_raw) {
    hipLaunchKernelGGL(k_summary, dim3(1), dim3(kSumThreads), 0, st, x, n, part, nparts, roots,
                       ranks, req_bins, dedup, reinterpret_cast<uint8_t*>(payload), scratch_raw);
    return hipGetLastError();
}

// Split-injected parity mode: header from caller splits (Quantizer.findZeroIdx rule).
__global__ void k_set_splits(uint8_t* payload, int64_t n, const double* __restrict__ sp, int nsplits,
                             double mn, double mx, int req_bins) {
    skml_dense_header* hdr = reinterpret_cast<skml_dense_header*>(payload);
    double* splits = reinterpret_cast<double*>(payload + kHeaderBytes);
    __shared__ int s_zero;
    if (threadIdx.x == 0) s_zero = 0x7FFFFFFF;
    __syncthreads();
    for (int i = threadIdx.x; i < nsplits; i += blockDim.x) {
        splits[i] = sp[i];
        if (!(sp[i] < 0.0)) atomicMin(&s_zero, i);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int bins = nsplits + 1;
        hdr->magic = SKML_DENSE_MAGIC;
        hdr->status = SKML_OK;
        hdr->n = n;
        hdr->bin_num = bins;
        hdr->zero_idx = mn > 0.0 ? 0 : (mx < 0.0 ? bins - 1 : (s_zero < bins - 1 ? s_zero : bins - 1));
        hdr->code_bits = code_bits_for(bins);
        hdr->req_bins = req_bins;
        hdr->min = mn;
        hdr->max = mx;
        hdr->codes_offset = (int64_t)dense_codes_offset(req_bins);
        hdr->reserved = 0;
    }
}

hipError_t launch_set_splits(hipStream_t st, void* payload, int64_t n, const double* splits_dev,
                             int nsplits, double mn, double mx, int req_bins) {
    hipLaunchKernelGGL(k_set_splits, dim3(1), dim3(256), 0, st, reinterpret_cast<uint8_t*>(payload),
                       n, splits_dev, nsplits, mn, mx, req_bins);
    return hipGetLastError();
}

// =============================================================================================
// Quantize: Eytzinger search over the LDS split table; codes packed LSB-first.
// =============================================================================================
constexpr int kQThreads = 256;
constexpr int kEytzMax = 4096;

__device__ __forceinline__ void store_codes4(uint8_t* codes, int64_t e0, uint32_t c0, uint32_t c1,
                                             uint32_t c2, uint32_t c3, int bits, int lane) {
    // e0 is a multiple of 4; lanes l and l^1 cover adjacent 4-element groups
    switch (bits) {
        case 8:
            *reinterpret_cast<uint32_t*>(codes + e0) = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
            break;
        case 16:
            *reinterpret_cast<uint2*>(codes + e0 * 2) = make_uint2(c0 | (c1 << 16), c2 | (c3 << 16));
            break;
        case 4:
            *reinterpret_cast<uint16_t*>(codes + e0 / 2) = (uint16_t)(c0 | (c1 << 4) | (c2 << 8) | (c3 << 12));
            break;
        case 2:
            codes[e0 / 4] = (uint8_t)(c0 | (c1 << 2) | (c2 << 4) | (c3 << 6));
            break;
        default: {  // 1 bit: pair with the neighbour lane into one byte
            const uint32_t nib = c0 | (c1 << 1) | (c2 << 2) | (c3 << 3);
            const uint32_t other = lane_xor<1>(nib);
            if ((lane & 1) == 0) codes[e0 / 8] = (uint8_t)(nib | (other << 4));
            break;
        }
    }
}

__device__ __forceinline__ uint32_t eytz_bin(const float* E, int levels, uint32_t P, float xv) {
    uint32_t i = 1;
    for (int s = 0; s < levels; s++) i = 2 * i + (E[i] <= xv ? 1u : 0u);
    return i - P;
}

__device__ __forceinline__ uint32_t global_bin(const double* sp, int nsplit, float xv) {
    int lo = 0, hi = nsplit;
    const double xd = (double)xv;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (sp[mid] <= xd) lo = mid + 1;
        else hi = mid;
    }
    return (uint32_t)lo;
}

__global__ __launch_bounds__(kQThreads) void k_quantize(const float* __restrict__ x, int64_t n,
                                                        uint8_t* __restrict__ payload) {
    __shared__ float E[kEytzMax];
    const skml_dense_header* hdr = reinterpret_cast<const skml_dense_header*>(payload);
    if (hdr->status != SKML_OK) return;
    const int bins = hdr->bin_num, bits = hdr->code_bits, nsplit = bins - 1;
    const double* sp = reinterpret_cast<const double*>(payload + kHeaderBytes);
    uint8_t* codes = payload + hdr->codes_offset;
    uint32_t P = 1;
    int levels = 0;
    while (P < (uint32_t)bins) {
        P <<= 1;
        levels++;
    }
    const bool lds = P <= kEytzMax;
    if (lds) {
        for (uint32_t i = threadIdx.x + 1; i < P; i += kQThreads) {
            const int d = 31 - __clz(i);
            const uint32_t idx = ((2u * (i - (1u << d)) + 1u) << (levels - 1 - d)) - 1u;
            E[i] = idx < (uint32_t)nsplit ? (float)sp[idx] : __uint_as_float(0x7FC00000u);
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int64_t nwaves_total = (int64_t)gridDim.x * (kQThreads / 64);
    const int64_t wave_id = (int64_t)blockIdx.x * (kQThreads / 64) + (threadIdx.x >> 6);
    const int64_t full_tiles = n / 1024;
    for (int64_t tile = wave_id; tile < full_tiles; tile += nwaves_total) {
        const float4* src = reinterpret_cast<const float4*>(x + tile * 1024);
        float4 f[4];
#pragma unroll
        for (int j = 0; j < 4; j++) f[j] = src[j * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t c0, c1, c2, c3;
            if (lds) {
                c0 = eytz_bin(E, levels, P, f[j].x);
                c1 = eytz_bin(E, levels, P, f[j].y);
                c2 = eytz_bin(E, levels, P, f[j].z);
                c3 = eytz_bin(E, levels, P, f[j].w);
            } else {
                c0 = global_bin(sp, nsplit, f[j].x);
                c1 = global_bin(sp, nsplit, f[j].y);
                c2 = global_bin(sp, nsplit, f[j].z);
                c3 = global_bin(sp, nsplit, f[j].w);
            }
            store_codes4(codes, tile * 1024 + j * 256 + lane * 4, c0, c1, c2, c3, bits, lane);
        }
    }
    // tail tile (n % 1024 values), one wave, guarded element loads
    if (wave_id == full_tiles % nwaves_total && n % 1024) {
        const int64_t base = full_tiles * 1024;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e0 = base + j * 256 + lane * 4;
            uint32_t c[4] = {0, 0, 0, 0};
            for (int e = 0; e < 4; e++)
                if (e0 + e < n) {
                    const float xv = x[e0 + e];
                    c[e] = lds ? eytz_bin(E, levels, P, xv) : global_bin(sp, nsplit, xv);
                }
            const bool any = e0 < n;
            if (bits == 1) {
                const int64_t pair0 = base + j * 256 + (lane & ~1) * 4;
                const uint32_t nib = c[0] | (c[1] << 1) | (c[2] << 2) | (c[3] << 3);
                const uint32_t other = lane_xor<1>(nib);
                if ((lane & 1) == 0 && pair0 < n) codes[pair0 / 8] = (uint8_t)(nib | (other << 4));
            } else if (any) {
                store_codes4(codes, e0, c[0], c[1], c[2], c[3], bits, lane);
            }
        }
    }
}

static int quant_grid(int64_t n) {
    const int64_t tiles = (n + 1023) / 1024;
    int64_t wg = (tiles + 3) / 4;
    if (wg > 4096) wg = 4096;
    if (wg < 1) wg = 1;
    return (int)wg;
}

hipError_t launch_quantize(hipStream_t st, const float* x, int64_t n, void* payload) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_quantize, dim3(quant_grid(n)), dim3(kQThreads), 0, st, x, n,
                       reinterpret_cast<uint8_t*>(payload));
    return hipGetLastError();
}

// =============================================================================================
// Decode: LUT of Quantizer.getValues() midpoints (computed in double, Quantizer.java:39-47).
// =============================================================================================
__device__ __forceinline__ uint32_t read_code(const uint8_t* codes, int64_t e, int bits) {
    switch (bits) {
        case 8: return codes[e];
        case 16: return reinterpret_cast<const uint16_t*>(codes)[e];
        case 4: return (codes[e >> 1] >> ((e & 1) * 4)) & 15u;
        case 2: return (codes[e >> 2] >> ((e & 3) * 2)) & 3u;
        default: return (codes[e >> 3] >> (e & 7)) & 1u;
    }
}

// Four consecutive codes starting at e0 (multiple of 4).
__device__ __forceinline__ void read_codes4(const uint8_t* codes, int64_t e0, int bits, uint32_t (&c)[4]) {
    switch (bits) {
        case 8: {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(codes + e0);
            c[0] = w & 255u; c[1] = (w >> 8) & 255u; c[2] = (w >> 16) & 255u; c[3] = w >> 24;
            break;
        }
        case 16: {
            const uint2 w = *reinterpret_cast<const uint2*>(codes + e0 * 2);
            c[0] = w.x & 0xFFFFu; c[1] = w.x >> 16; c[2] = w.y & 0xFFFFu; c[3] = w.y >> 16;
            break;
        }
        case 4: {
            const uint32_t w = *reinterpret_cast<const uint16_t*>(codes + e0 / 2);
            c[0] = w & 15u; c[1] = (w >> 4) & 15u; c[2] = (w >> 8) & 15u; c[3] = (w >> 12) & 15u;
            break;
        }
        case 2: {
            const uint32_t w = codes[e0 / 4];
            c[0] = w & 3u; c[1] = (w >> 2) & 3u; c[2] = (w >> 4) & 3u; c[3] = (w >> 6) & 3u;
            break;
        }
        default: {
            const uint32_t w = (codes[e0 / 8] >> (e0 & 4)) & 15u;
            c[0] = w & 1u; c[1] = (w >> 1) & 1u; c[2] = (w >> 2) & 1u; c[3] = (w >> 3) & 1u;
            break;
        }
    }
}

__device__ __forceinline__ double lut_value(const skml_dense_header* h, const double* sp, int b) {
    const int ns = h->bin_num - 1;
    if (b == 0) return 0.5 * (h->min + sp[0]);
    if (b == ns) return 0.5 * (sp[ns - 1] + h->max);
    return 0.5 * (sp[b - 1] + sp[b]);
}

constexpr int kLutMax = 4096;

__global__ __launch_bounds__(256) void k_decode(const uint8_t* __restrict__ payload,
                                                float* __restrict__ out, int64_t n) {
    __shared__ float lut[kLutMax];
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(payload);
    const double* sp = reinterpret_cast<const double*>(payload + kHeaderBytes);
    const uint8_t* codes = payload + h->codes_offset;
    const int bins = h->bin_num, bits = h->code_bits;
    const bool lds = bins <= kLutMax;
    if (lds) {
        for (int b = threadIdx.x; b < bins; b += 256) lut[b] = (float)lut_value(h, sp, b);
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4, wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t full = n / 1024;
    for (int64_t tile = wid; tile < full; tile += nw) {
        float4* dst = reinterpret_cast<float4*>(out + tile * 1024);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t c[4];
            read_codes4(codes, tile * 1024 + j * 256 + lane * 4, bits, c);
            float4 o;
            if (lds) o = make_float4(lut[c[0]], lut[c[1]], lut[c[2]], lut[c[3]]);
            else o = make_float4((float)lut_value(h, sp, c[0]), (float)lut_value(h, sp, c[1]),
                                 (float)lut_value(h, sp, c[2]), (float)lut_value(h, sp, c[3]));
            dst[j * 64 + lane] = o;
        }
    }
    if (wid == full % nw) {
        for (int64_t e = full * 1024 + lane; e < n; e += 64) {
            const uint32_t c = read_code(codes, e, bits);
            out[e] = lds ? lut[c] : (float)lut_value(h, sp, c);
        }
    }
}

hipError_t launch_decode(hipStream_t st, const void* payload, float* out, int64_t n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode, dim3(quant_grid(n)), dim3(256), 0, st,
                       reinterpret_cast<const uint8_t*>(payload), out, n);
    return hipGetLastError();
}

// Fused decode of P payloads + sum in double (Gradient.sum adds doubles) + scale.
constexpr int kMaxSumPayloads = 16;
constexpr int kSumLutBins = 256;
__global__ __launch_bounds__(256) void k_decode_sum(const uint8_t* __restrict__ payloads, int P,
                                                    size_t stride, float* __restrict__ out, int64_t n,
                                                    double scale) {
    __shared__ double lut[kMaxSumPayloads][kSumLutBins];
    for (int p = 0; p < P; p++) {
        const uint8_t* pl = payloads + (size_t)p * stride;
        const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(pl);
        const double* sp = reinterpret_cast<const double*>(pl + kHeaderBytes);
        for (int b = threadIdx.x; b < h->bin_num && b < kSumLutBins; b += 256) lut[p][b] = lut_value(h, sp, b);
    }
    __syncthreads();
    const int64_t stride_e = (int64_t)gridDim.x * 256;
    for (int64_t e0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; e0 < n; e0 += stride_e * 4) {
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        for (int p = 0; p < P; p++) {
            const uint8_t* pl = payloads + (size_t)p * stride;
            const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(pl);
            const uint8_t* codes = pl + h->codes_offset;
            uint32_t c[4];
            if (e0 + 4 <= n) read_codes4(codes, e0, h->code_bits, c);
            else
                for (int e = 0; e < 4; e++) c[e] = e0 + e < n ? read_code(codes, e0 + e, h->code_bits) : 0;
            for (int e = 0; e < 4; e++) acc[e] += lut[p][c[e]];
        }
        if (e0 + 4 <= n) {
            *reinterpret_cast<float4*>(out + e0) = make_float4((float)(acc[0] * scale), (float)(acc[1] * scale),
                                                               (float)(acc[2] * scale), (float)(acc[3] * scale));
        } else {
            for (int e = 0; e < 4; e++)
                if (e0 + e < n) out[e0 + e] = (float)(acc[e] * scale);
        }
    }
}

hipError_t launch_decode_sum(hipStream_t st, const void* payloads, int P, size_t stride, float* out,
                             int64_t n, double scale) {
    if (n <= 0) return hipSuccess;
    if (P < 1 || P > kMaxSumPayloads) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_decode_sum, dim3(quant_grid(n)), dim3(256), 0, st,
                       reinterpret_cast<const uint8_t*>(payloads), P, stride, out, n, scale);
    return hipGetLastError();
}

// getBins(): int32 bins
__global__ void k_bins(const uint8_t* __restrict__ payload, int32_t* __restrict__ bins, int64_t n) {
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(payload);
    const uint8_t* codes = payload + h->codes_offset;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
        bins[e] = (int32_t)read_code(codes, e, h->code_bits);
}

hipError_t launch_bins(hipStream_t st, const void* payload, int32_t* bins, int64_t n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bins, dim3(quant_grid(n)), dim3(256), 0, st,
                       reinterpret_cast<const uint8_t*>(payload), bins, n);
    return hipGetLastError();
}

// Quantizer.writeObject bin stream (Quantizer.java:193-202): width 1 (bin-128), 2 (bin-32768, BE)
__global__ void k_ref_body(const uint8_t* __restrict__ payload, uint8_t* __restrict__ out, int64_t n,
                           int width) {
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(payload);
    const uint8_t* codes = payload + h->codes_offset;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t b = read_code(codes, e, h->code_bits);
        if (width == 1) out[e] = (uint8_t)(b - 128u);
        else if (width == 2) {
            const uint32_t s = (b - 32768u) & 0xFFFFu;
            out[2 * e] = (uint8_t)(s >> 8);
            out[2 * e + 1] = (uint8_t)s;
        } else {
            out[4 * e] = (uint8_t)(b >> 24);
            out[4 * e + 1] = (uint8_t)(b >> 16);
            out[4 * e + 2] = (uint8_t)(b >> 8);
            out[4 * e + 3] = (uint8_t)b;
        }
    }
}

hipError_t launch_ref_body(hipStream_t st, const void* payload, uint8_t* out, int64_t n, int width) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ref_body, dim3(quant_grid(n)), dim3(256), 0, st,
                       reinterpret_cast<const uint8_t*>(payload), out, n, width);
    return hipGetLastError();
}

__global__ void k_times_by(uint8_t* payload, double x) {
    skml_dense_header* h = reinterpret_cast<skml_dense_header*>(payload);
    double* sp = reinterpret_cast<double*>(payload + kHeaderBytes);
    for (int i = threadIdx.x; i < h->bin_num - 1; i += blockDim.x) sp[i] *= x;
    if (threadIdx.x == 0) {
        h->min *= x;
        h->max *= x;
    }
}

hipError_t launch_times_by(hipStream_t st, void* payload, double x) {
    hipLaunchKernelGGL(k_times_by, dim3(1), dim3(256), 0, st, reinterpret_cast<uint8_t*>(payload), x);
    return hipGetLastError();
}

}  // namespace skml

namespace skml {
// Quantizer.readObject bin stream (Quantizer.java:216-225) -> packed codes of the payload.
__global__ void k_pack_ref(const uint8_t* __restrict__ body, int width, int64_t n,
                           uint8_t* __restrict__ payload) {
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(payload);
    uint8_t* codes = payload + h->codes_offset;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t e0 = g * 4;
    uint32_t c[4] = {0, 0, 0, 0};
    for (int e = 0; e < 4; e++) {
        const int64_t i = e0 + e;
        if (i >= n) break;
        if (width == 1) c[e] = (uint32_t)((int32_t)(int8_t)body[i] + 128);
        else if (width == 2)
            c[e] = (uint32_t)((int32_t)(int16_t)(((uint32_t)body[2 * i] << 8) | body[2 * i + 1]) + 32768);
        else
            c[e] = ((uint32_t)body[4 * i] << 24) | ((uint32_t)body[4 * i + 1] << 16) |
                   ((uint32_t)body[4 * i + 2] << 8) | body[4 * i + 3];
    }
    const int lane = threadIdx.x & 63;
    if (h->code_bits == 1) {
        const uint32_t nib = c[0] | (c[1] << 1) | (c[2] << 2) | (c[3] << 3);
        const uint32_t other = lane_xor<1>(nib);
        if ((lane & 1) == 0 && e0 < n) codes[e0 / 8] = (uint8_t)(nib | (other << 4));
    } else if (e0 < n) {
        store_codes4(codes, e0, c[0], c[1], c[2], c[3], h->code_bits, lane);
    }
}

hipError_t launch_pack_ref(hipStream_t st, const uint8_t* body, int width, int64_t n, void* payload) {
    if (n <= 0) return hipSuccess;
    const int64_t groups = (n + 3) / 4;
    hipLaunchKernelGGL(k_pack_ref, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st, body,
                       width, n, reinterpret_cast<uint8_t*>(payload));
    return hipGetLastError();
}
}  // namespace skml
