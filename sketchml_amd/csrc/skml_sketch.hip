// skml_sketch.hip -- CDNA4 (gfx950) kernels building the k=128 quantile sketch of an fp32 bucket.
//
// The reference sketch (HeapQuantileSketch.java) is a fixed binary merge tree over 256-value
// chunks: each chunk is sorted (Arrays.sort total order) and compacted to 128 samples with one
// RNG bit (fullBaseBufferPropagation, HeapQuantileSketch.java:107-124; compactBuffer,
// QSketchUtils.java:45-51); node (level L+1) = compact(merge(older level-L node, newer one))
// (levelwisePropagation / mergeArrays, QSketchUtils.java:53-82).  The bit used by the node at
// `level` whose last chunk is c is draw #(2c - popcount(c) + level) of java.util.Random(seed).
//
//   k_leaf64  the fp32 pass over the bucket's full 64-chunk tiles (the hot kernel).  One wave owns
//             one tile: 4 rounds of 16 chunks, 64 values per lane (4 lanes per chunk).  In
//             registers: Batcher's odd-even network over the lane's 64 values (543 comparators,
//             v_min/v_max_f32), 3 cross-lane merge stages (DPP move + v_med3_f32) fused with the
//             compaction, then tree levels 1..4; levels 5..6 through a carry stack in LDS.  No
//             workgroup barriers.  Output: one level-6 node per 64 chunks, the tile's min / max /
//             NaN / zero-sign flags, and the upper tree's compaction bit of this tile.
//   k_leaf2   the same tree with 32 values per lane (8 lanes per chunk): the partial tile (run in
//             workgroup 0 of the k_leaf64 launch) and the fp64 leaf.
//   k_merge   64 nodes of level L -> one node of level L+6 with the same machinery; the last
//             workgroup of the last pass also runs the summary (makeSummary + getQuantiles +
//             Maths.unique + findZeroIdx, HeapQuantileSketch.java:126-174,293-323,
//             Maths.java:51-67, Quantizer.java:74-85) and writes the payload header.
//   k_summary the summary alone (buckets with < 128 chunks).
//
// Values are sorted as floats: gfx950's v_min/v_max/v_med3_f32 order -0.0 before +0.0, which is
// Arrays.sort's order for everything but NaN (flagged at load).  The merges equal the reference
// merge (IEEE `<`, ties emit the newer run) unless a merge sees both -0.0 and +0.0; a wave that
// has seen both takes the exact LDS path (count-based merge positions with the reference tie rule).
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "skml_device.hpp"

namespace skml {

// Phase timestamps of the fused merge + summary workgroup (profiling builds only:
// make EXTRA=-DSKML_PROF_SUMMARY); read back with skml_debug_prof.
__device__ unsigned long long g_prof[32];
#ifdef SKML_PROF_LEAF
// per-wave (start, end, hw_id, xcc_id) of the hot leaf kernel (profiling builds only)
__device__ unsigned long long g_leafprof[4 * 65536];
#endif
#ifdef SKML_PROF_SUMMARY
#define SKML_PROF(k)                                      \
    do {                                                  \
        if (threadIdx.x == 0) g_prof[(k)] = wall_clock64(); \
    } while (0)
#else
#define SKML_PROF(k) \
    do {             \
    } while (0)
#endif

// =============================================================================================
// shared memory
// =============================================================================================
constexpr int kWaveFb = 1536;  // per-wave exact-merge area, elements
template <typename S>
struct TileSharedT {
    S fb[kLeafWaves][kWaveFb];  // per-wave exact-merge area (mixed +/-0 only)
    S wn[kLeafWaves][kK];       // level L0+3 node of each wave
    S l4[4][kK];
    S l5[2][kK];
    S l6[kK];
    uint64_t mask[kLeafWaves];   // leaf: RNG draws [start, start+64) of each wave's chunks
    uint64_t start[kLeafWaves];
    uint32_t wgbits;             // bits of the 7 cross-wave merges
    uint32_t min_key, max_key, flags;
    int is_last;
};
using TileShared = TileSharedT<float>;

constexpr int kSumMaxRaw = 1024;  // raw splits kept in LDS up to this many
constexpr int kMaxSamples = kMaxLevels * kK + kChunk;
struct SummaryShared {
    float smp[kMaxSamples];      // gathered runs
    float sorted[kMaxSamples];   // samplesArr after blockyMergeSort
    int64_t w[kMaxSamples + 1];  // weightsArr -> cut points
    double raw[kSumMaxRaw];      // getQuantiles output before Maths.unique
    int64_t wsum[16];
    int run_off[kMaxLevels + 2];
    int run_lvl[kMaxLevels + 2];
    int nruns;
    uint32_t min_key, max_key, flags;
    int zero;
    int64_t total;
};

static_assert(sizeof(float) * kMaxSamples + sizeof(int64_t) * (kMaxSamples + 1) >= sizeof(uint16_t) * kLutSize,
              "LUT staging must fit in sorted[] + w[]");
static_assert(offsetof(SummaryShared, w) == offsetof(SummaryShared, sorted) + sizeof(float) * kMaxSamples,
              "sorted[] and w[] must be contiguous");

union MergeShared {
    TileShared t;
    SummaryShared s;
};

// =============================================================================================
// in-wave tree levels (input: 8 nodes of 128 keys, 8 lanes x 16 keys per node)
// =============================================================================================

// Exact path for one in-wave merge level (R keys / lane, G = 256/R lanes per merge group).
// fb holds 1536 floats: runs in [0, 1024), merged nodes in [1024, 1536).  The element loop is
// kept rolled and reads back from LDS so this rare path adds no register pressure.
// More than 4 merge groups per wave (R = 32: 8 groups) take the area in passes of 4 groups.
template <int R, typename T, typename S = typename Elem<T>::S>
__device__ __forceinline__ void wave_exact_level(T (&v)[R], T (&w)[R / 2], int lane, uint32_t odd, S* fb) {
    constexpr int G = 256 / R, kGroups = 64 / G, kPasses = kGroups > 4 ? kGroups / 4 : 1;
    const int grp = lane / G, li = lane % G;
    S* run = fb + (grp & 3) * 256;
    S* out = fb + 1024 + (grp & 3) * 128;
#pragma unroll 1
    for (int h = 0; h < kPasses; h++) {
        if ((grp >> 2) != h) continue;
#pragma unroll
        for (int r = 0; r < R; r++) run[li * R + r] = Elem<T>::to_s(v[r]);
#pragma unroll 1
        for (int r = 0; r < R; r++) {
            const int p = li * R + r;
            const S x = run[p];
            const int pos = p < 128 ? p + count_le(run + 128, x) : (p - 128) + count_lt(run, x);
            if (((uint32_t)pos & 1u) == odd) out[pos >> 1] = x;
        }
#pragma unroll
        for (int j = 0; j < R / 2; j++) w[j] = Elem<T>::from_s(out[li * (R / 2) + j]);
    }
}

template <int R, typename T, typename S>
__device__ __forceinline__ void wave_level(T (&v)[R], T (&w)[R / 2], int lane, uint32_t odd, bool exact, S* fb) {
    if (!exact) {
        merge_group_compact<R>(v, w, lane, odd != 0);
    } else {
        wave_exact_level<R>(v, w, lane, odd, fb);
    }
}

// Write the node held by lanes [g*G, g*G+G) (R keys per lane) as 128 floats.
template <int R, typename T>
__device__ __forceinline__ void store_node(const T (&w)[R], int lane, typename Elem<T>::S* dst) {
    constexpr int G = kK / R;
    const int li = lane % G;
    if constexpr (std::is_same<T, double>::value) {
        double2* d = reinterpret_cast<double2*>(dst + li * R);
#pragma unroll
        for (int q = 0; q < R / 2; q++) d[q] = make_double2(w[2 * q], w[2 * q + 1]);
    } else if constexpr (R >= 4) {  // vector stores: few address registers
        float4* d = reinterpret_cast<float4*>(dst + li * R);
#pragma unroll
        for (int q = 0; q < R / 4; q++)
            d[q] = make_float4(Elem<T>::to_s(w[4 * q]), Elem<T>::to_s(w[4 * q + 1]), Elem<T>::to_s(w[4 * q + 2]),
                               Elem<T>::to_s(w[4 * q + 3]));
    } else {
        reinterpret_cast<float2*>(dst + li * R)[0] = make_float2(Elem<T>::to_s(w[0]), Elem<T>::to_s(w[1]));
    }
}

// Levels +1..+3 inside a wave.  bits: 0..3 -> level+1 nodes, 4..5 -> level+2, 6 -> level+3.
// Exp(level_offset, node_in_wave, regs...) is called after each level for root exports.
template <typename T, typename S, class Exp>
__device__ __forceinline__ void inwave_levels(T (&w1)[16], T (&w4)[2], int lane, uint32_t bits, bool exact, S* fb,
                                              Exp&& exp, bool stamp = false) {
    T w2[8], w3[4];
    wave_level<16>(w1, w2, lane, (bits >> (lane >> 4)) & 1u, exact, fb);
#ifdef SKML_PROF_SUMMARY
    if (stamp && threadIdx.x == 0) g_prof[23] = wall_clock64();
#endif
    exp.template at<8>(1, lane >> 4, w2);
    wave_level<8>(w2, w3, lane, (bits >> (4 + (lane >> 5))) & 1u, exact, fb);
#ifdef SKML_PROF_SUMMARY
    if (stamp && threadIdx.x == 0) g_prof[24] = wall_clock64();
#endif
    exp.template at<4>(2, lane >> 5, w3);
    wave_level<4>(w3, w4, lane, (bits >> 6) & 1u, exact, fb);
#ifdef SKML_PROF_SUMMARY
    if (stamp && threadIdx.x == 0) g_prof[25] = wall_clock64();
#endif
    (void)stamp;
    exp.template at<2>(3, 0, w4);
}

// One wave merges two 128-float nodes from LDS into `out` (bitonic, 64 lanes x 4 keys).
template <typename T = uint32_t, typename S = typename Elem<T>::S>
__device__ __forceinline__ void wave_pair_merge(const S* A, const S* B, S* out, int lane, uint32_t odd) {
    const S* src = lane < 32 ? A + 4 * lane : B + 4 * (lane - 32);
    T v[4], o[2];
    if constexpr (std::is_same<S, double>::value) {
        const double2 p = reinterpret_cast<const double2*>(src)[0], q = reinterpret_cast<const double2*>(src)[1];
        v[0] = p.x, v[1] = p.y, v[2] = q.x, v[3] = q.y;
        merge_group_compact<4>(v, o, lane, odd != 0);
        reinterpret_cast<double2*>(out)[lane] = make_double2(o[0], o[1]);
    } else {
        const float4 f = reinterpret_cast<const float4*>(src)[0];
        v[0] = Elem<T>::from_s(f.x), v[1] = Elem<T>::from_s(f.y), v[2] = Elem<T>::from_s(f.z),
        v[3] = Elem<T>::from_s(f.w);
        merge_group_compact<4>(v, o, lane, odd != 0);
        reinterpret_cast<float2*>(out)[lane] = make_float2(Elem<T>::to_s(o[0]), Elem<T>::to_s(o[1]));
    }
}

// Levels +4..+6 across the 8 waves.  bits: 0..3 level+4, 4..5 level+5, 6 level+6.
template <typename T = uint32_t, typename S = typename Elem<T>::S>
__device__ __forceinline__ void crosswave_levels(TileSharedT<S>& sh, int tid, uint32_t bits, bool exact) {
    const int wave = tid >> 6, lane = tid & 63;
    if (!exact) {
        if (wave < 4) wave_pair_merge<T>(sh.wn[2 * wave], sh.wn[2 * wave + 1], sh.l4[wave], lane, (bits >> wave) & 1u);
    } else {
        for (int task = tid; task < 4 * 256; task += 512) {
            const int m = task >> 8;
            exact_merge_task(sh.wn[2 * m], sh.wn[2 * m + 1], sh.l4[m], task & 255, (bits >> m) & 1u);
        }
    }
    __syncthreads();
    if (!exact) {
        if (wave < 2) wave_pair_merge<T>(sh.l4[2 * wave], sh.l4[2 * wave + 1], sh.l5[wave], lane, (bits >> (4 + wave)) & 1u);
    } else {
        const int m = tid >> 8;
        exact_merge_task(sh.l4[2 * m], sh.l4[2 * m + 1], sh.l5[m], tid & 255, (bits >> (4 + m)) & 1u);
    }
    __syncthreads();
    if (!exact) {
        if (wave == 0) wave_pair_merge<T>(sh.l5[0], sh.l5[1], sh.l6, lane, (bits >> 6) & 1u);
    } else if (tid < 256) {
        exact_merge_task(sh.l5[0], sh.l5[1], sh.l6, tid, (bits >> 6) & 1u);
    }
    __syncthreads();
}

// =============================================================================================
// Leaf kernel
// =============================================================================================
struct NoExport {
    template <int R, typename T>
    __device__ void at(int, int, const T (&)[R]) const {}
};

// Roots of the small trees (chunks mod 64) in the last, partial leaf workgroup.
struct LeafExport {
    int lane, rem;
    int64_t wave_off;  // first chunk of the wave, relative to the workgroup
    float* roots;
    template <int R, typename T>
    __device__ __forceinline__ void at(int level, int node, const T (&w)[R]) const {
        if (!rem || !((rem >> level) & 1)) return;
        const int64_t cs = ((int64_t)rem >> (level + 1)) << (level + 1);
        if (wave_off + ((int64_t)node << level) != cs) return;
        store_node<R>(w, lane, roots + (size_t)level * kK);
    }
};

// ---------------------------------------------------------------------------------------------
// Wave-persistent leaf: every wave owns 64 consecutive chunks (one level-6 node) and walks them in
// 8 rounds of 8 chunks.  Round nodes (level 3) are carried through a register stack of levels
// 3..5 exactly like HeapQuantileSketch's binary counter (inPlacePropagationUpdate,
// HeapQuantileSketch.java:116-124), so no workgroup barrier is ever needed.
// ---------------------------------------------------------------------------------------------
// s_setprio 3..0 by the fraction of the wave's rounds already done (wave-uniform).
__device__ __forceinline__ void set_prio_by_progress(int round, int nrounds) {
    switch ((4 * round) / nrounds) {
        case 0: __builtin_amdgcn_s_setprio(3); break;
        case 1: __builtin_amdgcn_s_setprio(2); break;
        case 2: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
    }
}

constexpr int kLeafWaveChunks = 64;
constexpr int kLeaf2Waves = 4;

// Merge two register-resident nodes (64 lanes x 2 keys, positions lane*2 + r): older A, newer B.
template <typename T, typename S>
__device__ __forceinline__ void wave_node_merge(const T (&A)[2], const T (&B)[2], T (&out)[2], int lane, uint32_t odd,
                                                bool exact, S* buf) {
    S* a = buf;
    S* b = buf + kK;
    S* o = buf + 2 * kK;
    using S2 = typename std::conditional<std::is_same<S, double>::value, double2, float2>::type;
    reinterpret_cast<S2*>(a)[lane] = S2{Elem<T>::to_s(A[0]), Elem<T>::to_s(A[1])};
    reinterpret_cast<S2*>(b)[lane] = S2{Elem<T>::to_s(B[0]), Elem<T>::to_s(B[1])};
    if (!exact) {
        wave_pair_merge<T>(a, b, o, lane, odd);
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) exact_merge_task(a, b, o, lane + 64 * k, odd);
    }
    const S2 r = reinterpret_cast<const S2*>(o)[lane];
    out[0] = Elem<T>::from_s(r.x);
    out[1] = Elem<T>::from_s(r.y);
}

// Roots of the small trees inside the partial 64-chunk tile (compiled only into the PARTIAL
// variant: a divergent export in the hot kernel costs ~50 VGPRs).
template <bool PARTIAL, typename S = float>
struct WaveExport {
    int lane, rem;
    int64_t round_off;  // first chunk of the round relative to the tile
    S* roots;
    template <int R, typename T>
    __device__ __forceinline__ void at(int level, int node, const T (&w)[R]) const {
        if constexpr (PARTIAL) {
            if (!((rem >> level) & 1)) return;
            const int64_t cs = ((int64_t)rem >> (level + 1)) << (level + 1);
            if (round_off + ((int64_t)node << level) != cs) return;
            store_node<R>(w, lane, roots + (size_t)level * kK);
        }
    }
};

// E = float (fp32 input) or double (the reference's double[] itself: 2 registers per value,
// hence at least 2 waves per SIMD instead of 4).
template <typename E>
struct LeafTypes {
    using Key = uint32_t;
    using Part = LeafPartial;
    static constexpr int kMinWaves = 4;
};
template <>
struct LeafTypes<double> {
    using Key = uint64_t;
    using Part = LeafPartial64;
    static constexpr int kMinWaves = 2;
};
__device__ __forceinline__ uint32_t total_key(float f) { return f2key(__float_as_uint(f)); }
__device__ __forceinline__ uint64_t total_key(double d) {
    const uint64_t b = (uint64_t)__double_as_longlong(d);
    return b ^ ((uint64_t)((int64_t)b >> 63) | 0x8000000000000000ull);
}
__device__ __forceinline__ bool is_class(float f, int mask) { return __builtin_amdgcn_classf(f, mask); }
__device__ __forceinline__ bool is_class(double d, int mask) { return __builtin_amdgcn_class(d, mask); }
__device__ __forceinline__ uint32_t fold32(float f) { return __float_as_uint(f); }
__device__ __forceinline__ uint32_t fold32(double d) {
    const uint64_t b = (uint64_t)__double_as_longlong(d);
    return (uint32_t)b ^ (uint32_t)(b >> 32);
}

template <int STAGE, bool PARTIAL = false, typename E = float>
__device__ __forceinline__ void leaf2_wave(const E* __restrict__ x, int64_t chunks, uint64_t s0,
                                           const uint64_t* __restrict__ tab,
                                           typename LeafTypes<E>::Part* __restrict__ part, E* __restrict__ nodes6,
                                           E* __restrict__ roots, int64_t tile, uint8_t* __restrict__ ubits,
                                           E* wfb) {
    using Key = typename LeafTypes<E>::Key;
    const int lane = threadIdx.x & 63;
    const int64_t c_tile = tile * kLeafWaveChunks;
    if (c_tile >= chunks) return;  // wave-uniform; no block barriers in this kernel
    const int64_t left = chunks - c_tile;
    const int rem = left < kLeafWaveChunks ? (int)left : 0;
    const int nrounds = rem ? (rem + kChunksPerWave - 1) / kChunksPerWave : kLeafWaveChunks / kChunksPerWave;
    const uint64_t ta = tab[lane * 2], tc = tab[lane * 2 + 1];  // A^lane, C_lane
#ifdef SKML_PROF_LEAF
    const unsigned long long prof_t0 = wall_clock64();
#endif

    Key mn = ~(Key)0, mx = 0;
    uint32_t fl = 0u;
    bool neg_any = false, pos_any = false;
    E st3[2], st4[2], st5[2], top[2];
    uint32_t acc = 0;
#pragma unroll 1
    for (int round = 0; round < nrounds; round++) {
        // Issue priority falls as the wave progresses: the SIMD's arbiter favours the oldest
        // wave, so without this the 4 waves of a SIMD finish one after another (~50/72/95/118 us
        // at 2^26) and the last quarter of the kernel runs with too few waves to hide latency.
        set_prio_by_progress(round, nrounds);
        const int64_t c0 = c_tile + round * kChunksPerWave;
        const int64_t chunk = c0 + (lane >> 3);
        const bool valid = PARTIAL ? chunk < chunks : true;
        // The values are sorted as floats (v_min/v_max/v_med3_f32, no key conversion): on gfx950
        // these order -0.0 before 0.0 (tools/ubench/zero_minmax.hip), i.e. Arrays.sort's total
        // order, for every value but NaN, which they drop.  One class test per element flags
        // zeros and NaN into a wave mask; NaN is reported from it.
        E v[32];
        uint64_t zmask = 0;
        if constexpr (std::is_same<E, double>::value) {
            const double2* src = reinterpret_cast<const double2*>(x + (valid ? chunk : c0) * kChunk);
            double2 f[16];
#pragma unroll
            for (int j = 0; j < 16; j++) f[j] = src[j * 8 + (lane & 7)];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                zmask |= __ballot(is_class(f[j].x, 0x63) || is_class(f[j].y, 0x63));  // -0.0 | +0.0 | NaN
                v[2 * j] = f[j].x;
                v[2 * j + 1] = f[j].y;
            }
        } else {
            const float4* src = reinterpret_cast<const float4*>(x + (valid ? chunk : c0) * kChunk);
            float4 f[8];
#pragma unroll
            for (int j = 0; j < 8; j++) f[j] = src[j * 8 + (lane & 7)];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float e4[4] = {f[j].x, f[j].y, f[j].z, f[j].w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    zmask |= __ballot(is_class(e4[e], 0x63));  // -0.0 | +0.0 | NaN
                    v[j * 4 + e] = e4[e];
                }
            }
        }
        if (PARTIAL) zmask &= __ballot(valid);
        uint32_t rfl = 0;
        if (zmask) {  // wave-uniform: which zero signs, and NaN
            uint64_t nz = 0, pz = 0, nan = 0;
#pragma unroll
            for (int r = 0; r < 32; r++) {
                nz |= __ballot(is_class(v[r], 0x20));
                pz |= __ballot(is_class(v[r], 0x40));
                nan |= __ballot(is_class(v[r], 0x03));
            }
            if (PARTIAL) {
                nz &= __ballot(valid);
                pz &= __ballot(valid);
                nan &= __ballot(valid);
            }
            rfl = (nz ? 2u : 0u) | (pz ? 4u : 0u) | (nan ? 1u : 0u);
            fl |= rfl;
        }
        // compaction bits of this round's chunks (and their carries): draws [start, start+64)
        const uint64_t start = node_bit_index((uint64_t)c0, 0);
        uint64_t mask;
        {
            const uint64_t s_start = lcg_jump(tab, s0, start + 1);
            const uint64_t s = lane == 0 ? s_start : ((ta * s_start + tc) & kLcgMask);
            mask = __ballot((s >> 47) & 1ull);
        }
        if constexpr (STAGE == 0) {
#pragma unroll
            for (int r = 0; r < 32; r++) acc ^= fold32(v[r]);
            acc ^= (uint32_t)mask;
            continue;
        }
        neg_any = neg_any || (rfl & 2u);
        pos_any = pos_any || (rfl & 4u);
        const bool exact = STAGE == 2 ? false : (neg_any && pos_any);
        auto bit = [&](int level, int64_t last_chunk) -> uint32_t {
            return (uint32_t)(mask >> (node_bit_index((uint64_t)last_chunk, level) - start)) & 1u;
        };

        E w1[16];
        {
            sort_regs_oddeven<32>(v);
            sort_lanes_upto128<32, 64>(v, lane);
            // the chunk's two sorted 128-runs: its extremes are the chunk min / max (min at
            // register 0 of one lane, max at register 31 of another)
            if (valid) {
                const Key k0 = total_key(v[0]), k31 = total_key(v[31]);
                mn = k0 < mn ? k0 : mn;
                mx = k31 > mx ? k31 : mx;
            }
            merge_group_compact<32>(v, w1, lane, bit(0, chunk) != 0);
        }
        const WaveExport<PARTIAL, E> exp{lane, rem, round * kChunksPerWave, roots};
        exp.template at<16>(0, lane >> 3, w1);
        if constexpr (STAGE == 1) {
#pragma unroll
            for (int r = 0; r < 16; r++) acc ^= fold32(w1[r]);
            continue;
        }
        uint32_t ibits = 0;
        for (int j = 0; j < 4; j++) ibits |= bit(1, c0 + 2 * j + 1) << j;
        ibits |= bit(2, c0 + 3) << 4 | bit(2, c0 + 7) << 5 | bit(3, c0 + 7) << 6;
        E node[2];
        inwave_levels(w1, node, lane, ibits, exact, wfb, exp);
        if constexpr (STAGE == 2) {
            acc ^= fold32(node[0]) ^ fold32(node[1]);
            continue;
        }

        // carry through the stack (older node first), levels 4..6
        if (!(round & 1)) {
            st3[0] = node[0];
            st3[1] = node[1];
            continue;
        }
        E n4[2];
        wave_node_merge(st3, node, n4, lane, bit(4, c0 + 7), exact, wfb);
        if constexpr (PARTIAL)
            if (((rem >> 4) & 1) && (int64_t)(round - 1) * kChunksPerWave == ((int64_t)(rem >> 5) << 5))
                store_node<2>(n4, lane, roots + (size_t)4 * kK);
        if (!(round & 2)) {
            st4[0] = n4[0];
            st4[1] = n4[1];
            continue;
        }
        E n5[2];
        wave_node_merge(st4, n4, n5, lane, bit(5, c0 + 7), exact, wfb);
        if constexpr (PARTIAL)
            if (((rem >> 5) & 1) && round == 3) store_node<2>(n5, lane, roots + (size_t)5 * kK);
        if (!(round & 4)) {
            st5[0] = n5[0];
            st5[1] = n5[1];
            continue;
        }
        wave_node_merge(st5, n5, top, lane, bit(6, c0 + 7), exact, wfb);
    }
    if constexpr (STAGE <= 2) {
        nodes6[(size_t)tile * 64 + lane] = (E)(acc ^ (uint32_t)mn ^ (uint32_t)mx ^ fl);
        return;
    }
    if constexpr (!PARTIAL) {
        // one compaction bit of the upper merge tree per wave (upper_level_offset numbering);
        // `chunks` here counts the full 64-chunk tiles, which hold every node of level >= 7
        if (ubits && tile < upper_node_count(chunks)) {
            int L = kLeafTopLevel + 1;
            int64_t i = tile;
            while (i >= (chunks >> L)) i -= chunks >> L++;
            const uint64_t c = ((uint64_t)(i + 1) << L) - 1;
            if (lane == 0) ubits[tile] = (uint8_t)lcg_bit(tab, s0, node_bit_index(c, L));
        }
    }
    if constexpr (!PARTIAL) {
        store_node<2>(top, lane, nodes6 + (size_t)tile * kK);
        // a level-6 tree (bit 6 of the chunk count) is this single node
        if (((chunks >> 6) & 1) && tile == ((chunks >> 7) << 1)) store_node<2>(top, lane, roots + (size_t)6 * kK);
    }
    // per-wave partial: min / max / flags (NaN keys lie outside [key(-inf), key(+inf)])
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Key omn = __shfl_xor(mn, off, 64);
        const Key omx = __shfl_xor(mx, off, 64);
        const uint32_t ofl = (uint32_t)__shfl_xor((int)fl, off, 64);
        mn = omn < mn ? omn : mn;
        mx = omx > mx ? omx : mx;
        fl |= ofl;
    }
    if (lane == 0) {
        typename LeafTypes<E>::Part p;
        p.min_key = mn;
        p.max_key = mx;
        p.flags = fl;
        if constexpr (std::is_same<E, float>::value) p.flags |= (mn < 0x007FFFFFu || mx > 0xFF800000u) ? 1u : 0u;
        p.pad = 0;
        part[tile] = p;  // (a single atomic accumulator instead costs ~40 us of contention)
#ifdef SKML_PROF_LEAF
        if (!PARTIAL && tile < 65536) {
            g_leafprof[4 * tile] = prof_t0;
            g_leafprof[4 * tile + 1] = wall_clock64();
            g_leafprof[4 * tile + 2] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
            g_leafprof[4 * tile + 3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
        }
#endif
    }
}

template <int STAGE, bool PARTIAL = false, typename E = float>
__global__ __launch_bounds__(256, LeafTypes<E>::kMinWaves) void k_leaf2(
    const E* __restrict__ x, int64_t chunks, uint64_t s0, const uint64_t* __restrict__ tab,
    typename LeafTypes<E>::Part* __restrict__ part, E* __restrict__ nodes6, E* __restrict__ roots, int64_t tile0,
    uint8_t* __restrict__ ubits = nullptr) {
    __shared__ E fb[kLeaf2Waves][kWaveFb];
    const int wave = threadIdx.x >> 6;
    leaf2_wave<STAGE, PARTIAL, E>(x, chunks, s0, tab, part, nodes6, roots,
                                  tile0 + (int64_t)blockIdx.x * kLeaf2Waves + wave, ubits, fb[wave]);
}

// ---------------------------------------------------------------------------------------------
// 64-keys-per-lane leaf (fp32, full 64-chunk tiles): 4 lanes per chunk, 16 chunks per round, 4
// rounds per wave.  The chunk sort is Batcher's odd-even network over 64 registers (543
// comparators) plus 3 cross-lane stages (6 with 32 keys per lane), and tree levels 1..4 run in
// registers (levels 5 and 6 through LDS).  Same outputs as k_leaf2<3, false, float>.
// ---------------------------------------------------------------------------------------------
constexpr int kL64Lanes = 4;                         // lanes per chunk
constexpr int kL64Chunks = 64 / kL64Lanes;           // chunks per round
constexpr int kL64Rounds = kLeafWaveChunks / kL64Chunks;

#ifndef SKML_LEAF64_WAVES
#define SKML_LEAF64_WAVES 4
#endif
#ifndef SKML_LEAF_MIN3DET
#define SKML_LEAF_MIN3DET 1
#endif
#ifndef SKML_LEAF_SPLIT_BELOW
#define SKML_LEAF_SPLIT_BELOW 3072  // full tiles under which the split leaf runs alone
#endif
// `chunks` counts the full tiles' chunks; when total_chunks holds a partial tile as well, that
// tile's small trees (k_leaf2's PARTIAL path, one wave) run in workgroup 0, which is dispatched
// first, so they overlap the full tiles instead of following them.
// SPLIT (buckets with fewer tiles than the chip has wave slots): the workgroup's 4 waves share one
// tile, wave w running round w to its level-4 node; waves 1 and 3 merge the pairs to level 5 and
// wave 3 the level-6 node (exact merges there when the waves' zero signs differ), so a small
// bucket runs 4x the waves with the same outputs.
struct Leaf64Shared {
    float fb[kLeaf2Waves][kWaveFb];
    float2 stk[kLeaf2Waves][2][64];  // the carry stack (levels 4, 5) in LDS, not registers
    uint32_t wpart[kLeaf2Waves][4];  // SPLIT: each wave's min / max / flags / zero signs
};
template <bool SPLIT>
__device__ __forceinline__ void leaf64_tile(const float* __restrict__ x, int64_t chunks, uint64_t s0,
                                            const uint64_t* __restrict__ tab, LeafPartial* __restrict__ part,
                                            float* __restrict__ nodes6, float* __restrict__ roots,
                                            uint8_t* __restrict__ ubits, int64_t tile, Leaf64Shared& L) {
    auto& fb = L.fb;
    auto& stk = L.stk;
    auto& wpart = L.wpart;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t c_tile = tile * kLeafWaveChunks;
    if (c_tile >= chunks) return;  // workgroup-uniform under SPLIT, wave-uniform otherwise
#ifdef SKML_PROF_LEAF
    const unsigned long long prof_t0 = wall_clock64();
#endif
    float* wfb = fb[wave];
    uint32_t mn = ~0u, mx = 0, fl = 0u;
    bool neg_any = false, pos_any = false;
    float top[2];
    uint64_t split_mask = 0;  // SPLIT: this wave's round draws (levels 5 and 6 read from them)
    // A round either runs fast (no merge can meet both zero signs) or exact; once the wave has
    // seen -0.0 and +0.0 it redoes the round and the rest on the exact loop, a separate code
    // region so its LDS merge paths do not take registers from the fast one.
    auto run_round = [&](auto ex, int round) -> bool {
        constexpr bool EX = decltype(ex)::value;
        // lane-derived values (selectors, draw offsets, addresses) are recomputed each round: held
        // across the loop they push the fast path past 128 registers
        int ln = lane;
        asm volatile("" : "+v"(ln));
        if constexpr (!SPLIT) set_prio_by_progress(round, kL64Rounds);
            const int64_t c0 = c_tile + round * kL64Chunks;
            const int64_t chunk = c0 + (ln >> 2);
            float v[64];
            uint64_t zmask = 0;
            {
                const float4* src = reinterpret_cast<const float4*>(x + chunk * kChunk);
                float4 f[16];
#pragma unroll
                for (int j = 0; j < 16; j++) f[j] = src[j * kL64Lanes + (ln & 3)];
#if SKML_LEAF_MIN3DET
                // zero / NaN detector: v_minimum3_f32 over |x| two values per op (NaN propagates,
                // min |x| is 0 iff a zero is present), two chains, one ballot per round
                float za = __builtin_inff(), zb = __builtin_inff();
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    asm("v_minimum3_f32 %0, |%1|, |%2|, %3" : "=v"(za) : "v"(f[j].x), "v"(f[j].y), "v"(za));
                    asm("v_minimum3_f32 %0, |%1|, |%2|, %3" : "=v"(zb) : "v"(f[j].z), "v"(f[j].w), "v"(zb));
                    v[j * 4 + 0] = f[j].x, v[j * 4 + 1] = f[j].y, v[j * 4 + 2] = f[j].z, v[j * 4 + 3] = f[j].w;
                }
                float zm;
                asm("v_minimum3_f32 %0, %1, %2, %2" : "=v"(zm) : "v"(za), "v"(zb));
                zmask = __ballot(!(zm > 0.0f));  // -0.0 | +0.0 | NaN somewhere in the lane
#else
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const float e4[4] = {f[j].x, f[j].y, f[j].z, f[j].w};
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        zmask |= __ballot(is_class(e4[e], 0x63));  // -0.0 | +0.0 | NaN
                        v[j * 4 + e] = e4[e];
                    }
                }
#endif
            }
            uint32_t rfl = 0;
            if (zmask) {  // wave-uniform: which zero signs, and NaN
                uint64_t nz = 0, pz = 0, nan = 0;
#pragma unroll
                for (int r = 0; r < 64; r++) {
                    nz |= __ballot(is_class(v[r], 0x20));
                    pz |= __ballot(is_class(v[r], 0x40));
                    nan |= __ballot(is_class(v[r], 0x03));
                }
                rfl = (nz ? 2u : 0u) | (pz ? 4u : 0u) | (nan ? 1u : 0u);
                fl |= rfl;
            }
            // compaction bits of this round's 16 chunks and their carries: draws [start, start+64)
            const uint64_t start = node_bit_index((uint64_t)c0, 0);
            uint64_t mask;
            {
                // A^ln, C_lane reloaded each round (L2-resident) rather than held in 4 registers
                const uint64_t ta = tab[ln * 2], tc = tab[ln * 2 + 1];
                const uint64_t s_start = lcg_jump(tab, s0, start + 1);
                const uint64_t s = ln == 0 ? s_start : ((ta * s_start + tc) & kLcgMask);
                mask = __ballot((s >> 47) & 1ull);
            }
            neg_any = neg_any || (rfl & 2u);
            pos_any = pos_any || (rfl & 4u);
            if constexpr (!EX) {
                if (neg_any && pos_any) return false;  // mixed zero signs from here on: the exact loop
            }
            const bool exact = EX;
            // c0 is a multiple of 16, so the draw of the level-L node ending at chunk c0 + d sits at
            // offset 2d - popcount(d) + L from `start`: a per-ln constant
            auto bit = [&](int level, int d) -> uint32_t {
                return (uint32_t)(mask >> (2 * d - __popc((unsigned)d) + level)) & 1u;
            };
            float w1[32];
            sort_regs_oddeven<64>(v);
            sort_lanes_upto128<64, 128>(v, ln);  // two sorted 128-runs per chunk
            {
                const uint32_t k0 = total_key(v[0]), k63 = total_key(v[63]);
                mn = k0 < mn ? k0 : mn;
                mx = k63 > mx ? k63 : mx;
            }
            merge_group_compact<64>(v, w1, ln, bit(0, ln >> 2) != 0);
            // levels 1..4 in registers: 8, 16, 32, 64 lanes per merge
            float w2[16], w3[8], w4[4], n4[2];
#ifdef SKML_LEAF_ABLATE_TREE  // profiling ablation: levels 1..4 replaced by a fold (wrong results)
            for (int q = 0; q < 16; q++) w2[q] = fminf(w1[2 * q], w1[2 * q + 1]);
            for (int q = 0; q < 8; q++) w3[q] = w2[2 * q];
            for (int q = 0; q < 4; q++) w4[q] = w3[2 * q];
            n4[0] = w4[0];
            n4[1] = w4[2];
#else
            wave_level<32>(w1, w2, ln, bit(1, 2 * (ln >> 3) + 1), exact, wfb);
            wave_level<16>(w2, w3, ln, bit(2, 4 * (ln >> 4) + 3), exact, wfb);
            wave_level<8>(w3, w4, ln, bit(3, 8 * (ln >> 5) + 7), exact, wfb);
            wave_level<4>(w4, n4, ln, bit(4, 15), exact, wfb);
#endif
            if constexpr (SPLIT) {  // the cross-wave levels follow the round loops
                stk[wave][0][ln] = make_float2(n4[0], n4[1]);
                split_mask = mask;
                return true;
            }
            // levels 5 and 6: the binary-counter carry over rounds (older node first)
            if (!(round & 1)) {
                stk[wave][0][ln] = make_float2(n4[0], n4[1]);
                return true;
            }
            float n5[2];
            {
                const float2 o = stk[wave][0][ln];
                const float st4[2] = {o.x, o.y};
                wave_node_merge(st4, n4, n5, ln, bit(5, 15), exact, wfb);
            }
            if (!(round & 2)) {
                stk[wave][1][ln] = make_float2(n5[0], n5[1]);
                return true;
            }
            const float2 o = stk[wave][1][ln];
            const float st5[2] = {o.x, o.y};
            wave_node_merge(st5, n5, top, ln, bit(6, 15), exact, wfb);
            return true;
    };
    if constexpr (SPLIT) {
        if (!run_round(std::false_type{}, wave)) run_round(std::true_type{}, wave);
        // per-wave partial, then levels 5 and 6 across the waves
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t omn = __shfl_xor(mn, off, 64);
            const uint32_t omx = __shfl_xor(mx, off, 64);
            const uint32_t ofl = (uint32_t)__shfl_xor((int)fl, off, 64);
            mn = omn < mn ? omn : mn;
            mx = omx > mx ? omx : mx;
            fl |= ofl;
        }
        if (lane == 0) {
            wpart[wave][0] = mn;
            wpart[wave][1] = mx;
            wpart[wave][2] = fl;
        }
        __syncthreads();
        // the reference's zero signs seen by a merge: a node carries its chunks' values
        auto zs = [&](int w) { return wpart[w][2] & 6u; };
        // draw offsets inside round 1's / 3's mask: 2 * 15 - popcount(15) + level
        const uint32_t b5 = (uint32_t)(split_mask >> 31) & 1u, b6 = (uint32_t)(split_mask >> 32) & 1u;
        if (wave & 1) {
            const uint32_t z = zs(wave - 1) | zs(wave);
            const float2 o = stk[wave - 1][0][lane], m = stk[wave][0][lane];
            const float A[2] = {o.x, o.y}, B[2] = {m.x, m.y};
            float n5[2];
            wave_node_merge(A, B, n5, lane, b5, z == 6u, wfb);
            stk[wave][1][lane] = make_float2(n5[0], n5[1]);
        }
        __syncthreads();
        if (wave != 3) return;
        {
            const uint32_t z = zs(0) | zs(1) | zs(2) | zs(3);
            const float2 o = stk[1][1][lane], m = stk[3][1][lane];
            const float A[2] = {o.x, o.y}, B[2] = {m.x, m.y};
            wave_node_merge(A, B, top, lane, b6, z == 6u, wfb);
        }
        mn = min(min(wpart[0][0], wpart[1][0]), min(wpart[2][0], wpart[3][0]));
        mx = max(max(wpart[0][1], wpart[1][1]), max(wpart[2][1], wpart[3][1]));
        fl = wpart[0][2] | wpart[1][2] | wpart[2][2] | wpart[3][2];
    } else {
        int round = 0;
#pragma unroll 1
        for (; round < kL64Rounds; round++)
            if (!run_round(std::false_type{}, round)) break;
#pragma unroll 1
        for (; round < kL64Rounds; round++) run_round(std::true_type{}, round);
    }
    // one compaction bit of the upper merge tree per wave (upper_level_offset numbering)
    if (ubits && tile < upper_node_count(chunks)) {
        int L = kLeafTopLevel + 1;
        int64_t i = tile;
        while (i >= (chunks >> L)) i -= chunks >> L++;
        const uint64_t c = ((uint64_t)(i + 1) << L) - 1;
        if (lane == 0) ubits[tile] = (uint8_t)lcg_bit(tab, s0, node_bit_index(c, L));
    }
    store_node<2>(top, lane, nodes6 + (size_t)tile * kK);
    if (((chunks >> 6) & 1) && tile == ((chunks >> 7) << 1)) store_node<2>(top, lane, roots + (size_t)6 * kK);
    if constexpr (!SPLIT) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t omn = __shfl_xor(mn, off, 64);
            const uint32_t omx = __shfl_xor(mx, off, 64);
            const uint32_t ofl = (uint32_t)__shfl_xor((int)fl, off, 64);
            mn = omn < mn ? omn : mn;
            mx = omx > mx ? omx : mx;
            fl |= ofl;
        }
    }
    if (lane == 0) {
        LeafPartial p;
        p.min_key = mn;
        p.max_key = mx;
        p.flags = fl | ((mn < 0x007FFFFFu || mx > 0xFF800000u) ? 1u : 0u);
        p.pad = 0;
        part[tile] = p;
#ifdef SKML_PROF_LEAF
        if (!SPLIT && tile < 65536) {
            g_leafprof[4 * tile] = prof_t0;
            g_leafprof[4 * tile + 1] = wall_clock64();
            g_leafprof[4 * tile + 2] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
            g_leafprof[4 * tile + 3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
        }
#endif
    }
}

// MODE 0: one wave per 64-chunk tile; MODE 1: the split form (four waves per tile); MODE 2: tiles
// below split_from one per wave, the rest split.  The split tiles come last in dispatch order, so
// the end of a large bucket runs in quarter-size units: one wave per tile left a tail in which
// the chip ran short of waves (2^28: wave-slot use 0.82 over the span, tools/prof_leaf_waves.py,
// profiles/r05d_leaf_waves.txt).
template <int MODE>
__global__ __launch_bounds__(256, SKML_LEAF64_WAVES) void k_leaf64(const float* __restrict__ x, int64_t chunks, uint64_t s0,
                                                   const uint64_t* __restrict__ tab, LeafPartial* __restrict__ part,
                                                   float* __restrict__ nodes6, float* __restrict__ roots,
                                                   uint8_t* __restrict__ ubits, int64_t total_chunks,
                                                   int64_t split_from) {
    __shared__ Leaf64Shared L;
    const int wave = threadIdx.x >> 6;
    int64_t blk = blockIdx.x;
    if (total_chunks > chunks) {
        if (blk == 0) {
            if (wave == 0)
                leaf2_wave<3, true, float>(x, total_chunks, s0, tab, part, nodes6, roots, chunks / kLeafWaveChunks,
                                           nullptr, L.fb[0]);
            return;
        }
        blk -= 1;
    }
    if constexpr (MODE == 0) {
        leaf64_tile<false>(x, chunks, s0, tab, part, nodes6, roots, ubits, blk * kLeaf2Waves + wave, L);
    } else if constexpr (MODE == 1) {
        leaf64_tile<true>(x, chunks, s0, tab, part, nodes6, roots, ubits, blk, L);
    } else {
        const int64_t nwg = split_from / kLeaf2Waves;  // split_from: a multiple of 4
        if (blk < nwg) leaf64_tile<false>(x, chunks, s0, tab, part, nodes6, roots, ubits, blk * kLeaf2Waves + wave, L);
        else leaf64_tile<true>(x, chunks, s0, tab, part, nodes6, roots, ubits, split_from + (blk - nwg), L);
    }
}

template <int STAGE, int MINW = 1>
__global__ __launch_bounds__(512, MINW) void k_leaf(const float* __restrict__ x, int64_t chunks,
                                              uint64_t s0, const uint64_t* __restrict__ tab,
                                              LeafPartial* __restrict__ part,
                                              float* __restrict__ nodes6,
                                              float* __restrict__ roots) {
    __shared__ TileShared sh;
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
        if constexpr (STAGE == 4) {  // ablation: no HBM traffic, synthetic values
            uint32_t h = (uint32_t)(blockIdx.x * 512 + tid) * 2654435761u;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                h ^= h << 13; h ^= h >> 17; h ^= h << 5;
                f[j] = make_float4(__uint_as_float(h & 0xBF7FFFFFu), __uint_as_float((h * 3u) & 0xBF7FFFFFu),
                                   __uint_as_float((h * 5u) & 0xBF7FFFFFu), __uint_as_float((h * 7u) & 0xBF7FFFFFu));
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) f[j] = src[j * 8 + (lane & 7)];
        }
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

    // ---- compaction bits for the wave's chunks: lane l computes draw #(start + l) ----
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
    if constexpr (STAGE == 5) {  // ablation: in-register stages only
        sort_regs<32>(v);
        uint32_t acc = mn ^ mx ^ fl;
#pragma unroll
        for (int r = 0; r < 32; r++) acc ^= v[r] * (r + 1);
        nodes6[(size_t)blockIdx.x * 512 + tid] = __uint_as_float(acc);
        return;
    }
    sort_group256<32>(v, lane);
    uint32_t w1[16];
    compact_regs<32>(v, w1, (uint32_t)(mask >> (node_bit_index((uint64_t)chunk, 0) - start)) & 1u);
    const LeafExport exp{lane, rem, wave * kChunksPerWave, roots};
    exp.at<16>(0, lane >> 3, w1);
    if constexpr (STAGE == 1 || STAGE == 4) {
        uint32_t acc = mn ^ mx ^ fl;
#pragma unroll
        for (int r = 0; r < 16; r++) acc ^= w1[r];
        nodes6[(size_t)blockIdx.x * 512 + tid] = __uint_as_float(acc);
        return;
    }

    // ---- tree levels 1..3 in the wave ----
    uint32_t ibits = 0;
    {
        auto bit = [&](int level, int node) -> uint32_t {
            const uint64_t c = (uint64_t)wave_c0 + ((uint64_t)(node + 1) << level) - 1;
            return (uint32_t)(mask >> (node_bit_index(c, level) - start)) & 1u;
        };
        for (int j = 0; j < 4; j++) ibits |= bit(1, j) << j;
        ibits |= bit(2, 0) << 4 | bit(2, 1) << 5 | bit(3, 0) << 6;
    }
    const bool wexact = (__ballot((fl & 2u) != 0) != 0) && (__ballot((fl & 4u) != 0) != 0);
    uint32_t w4[2];
    inwave_levels(w1, w4, lane, ibits, wexact, sh.fb[wave], exp);
    if constexpr (STAGE == 2) {
        nodes6[(size_t)blockIdx.x * 512 + tid] = __uint_as_float(w4[0] ^ w4[1] ^ mn ^ mx ^ fl);
        return;
    }
    store_node<2>(w4, lane, sh.wn[wave]);
    if (valid) {
        atomicMin(&sh.min_key, mn);
        atomicMax(&sh.max_key, mx);
        if (fl) atomicOr(&sh.flags, fl);
    }
    __syncthreads();

    // ---- tree levels 4..6 across waves ----
    uint32_t wbits = 0;
    {
        auto bit = [&](int level, int node) -> uint32_t {
            const int64_t last = wg_c0 + ((int64_t)(node + 1) << level) - 1;
            const int wv = (int)((last - wg_c0) >> 3);
            return (uint32_t)(sh.mask[wv] >> (node_bit_index((uint64_t)last, level) - sh.start[wv])) & 1u;
        };
        for (int m = 0; m < 4; m++) wbits |= bit(4, m) << m;
        wbits |= bit(5, 0) << 4 | bit(5, 1) << 5 | bit(6, 0) << 6;
    }
    const bool gexact = (sh.flags & 6u) == 6u;
    crosswave_levels(sh, tid, wbits, gexact);

    if (!rem) {
        if (tid < kK) {
            nodes6[(size_t)blockIdx.x * kK + tid] = sh.l6[tid];
            // a level-6 tree (bit 6 of the chunk count) is this single node
            if (((chunks >> 6) & 1) && (int64_t)blockIdx.x == ((chunks >> 7) << 1))
                roots[(size_t)6 * kK + tid] = sh.l6[tid];
        }
    } else if (tid < kK) {
        for (int level = 4; level <= 5; level++) {  // roots of levels 4..5 live in LDS
            if (!((rem >> level) & 1)) continue;
            const int cs = (rem >> (level + 1)) << (level + 1);
            const float* src = level == 4 ? sh.l4[cs >> 4] : sh.l5[cs >> 5];
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

// One wave per tile fills the chip from 4,096 tiles (2^26 values) up; below that the split form
// (four waves per tile) keeps more waves in flight.  Larger buckets end with split tiles (the
// hybrid MODE 2), so the last wave generation runs in quarter-size units.  Returns the first
// split tile (0: all split, full: none).  SKML_FORM_LEAF_SPLIT forces a form (tests, A/B):
// 1 none, 2 all, 3 / 4 / 5 the last 25 / 12.5 / 50 % of the tiles.
// The split leaf runs every size by default: at 2^28 it takes 326 us against 342 us for one wave
// per tile (the tail: wave-slot use 0.80 over the span, profiles/r05e_leaf_waves_normal_form.txt),
// at 2^26 the two are level (0.1618 / 0.1625 ms per encode), at 2^24 it is faster (0.069 / 0.079),
// and the hybrid tails measured between (profiles/ab/r05_split*.txt, r05_hybrid.txt).
#ifndef SKML_LEAF_SPLIT_TAIL_PCT
#define SKML_LEAF_SPLIT_TAIL_PCT 100
#endif
static int64_t leaf_split_from(int64_t full_tiles) {
    [[maybe_unused]] auto tail = [&](int pct_x2) {  // the first split tile for the last pct_x2 / 2 % of the tiles
        const int64_t s = full_tiles - full_tiles * pct_x2 / 200;
        return std::max<int64_t>(0, s / kLeaf2Waves * kLeaf2Waves);
    };
#ifdef SKML_AB  // one wave per tile (1) and the hybrid tails (3 / 4 / 5): measured slower at 2^28
    switch (form(SKML_FORM_LEAF_SPLIT)) {
        case 1: return full_tiles;
        case 2: return 0;
        case 3: return tail(50);
        case 4: return tail(25);
        case 5: return tail(100);
        default: break;
    }
#endif
#if SKML_LEAF_SPLIT_TAIL_PCT >= 100
    return 0;
#else
    if (full_tiles < SKML_LEAF_SPLIT_BELOW) return 0;
    return tail(2 * SKML_LEAF_SPLIT_TAIL_PCT);
#endif
}

hipError_t launch_leaf(hipStream_t st, const float* x, int64_t chunks, uint64_t s0,
                       const uint64_t* jump_tab, LeafPartial* part, float* nodes6, float* roots, uint8_t* ubits) {
    const int64_t full = chunks / kLeafWaveChunks;
#ifndef SKML_LEAF64
#define SKML_LEAF64 1
#endif
    if (full > 0 && SKML_LEAF64) {  // the partial tile, if any, rides in the same launch
        const int extra = chunks % kLeafWaveChunks ? 1 : 0;
        const int64_t split_from = leaf_split_from(full);
        if (split_from == 0) {
            hipLaunchKernelGGL(k_leaf64<1>, dim3((unsigned)(full + extra)), dim3(64 * kLeaf2Waves), 0, st, x,
                               full * kLeafWaveChunks, s0, jump_tab, part, nodes6, roots, ubits, chunks, (int64_t)0);
            return hipGetLastError();
        }
#if defined(SKML_AB) || SKML_LEAF_SPLIT_TAIL_PCT < 100
        if (split_from >= full) {
            const unsigned grid = (unsigned)((full + kLeaf2Waves - 1) / kLeaf2Waves + extra);
            hipLaunchKernelGGL(k_leaf64<0>, dim3(grid), dim3(64 * kLeaf2Waves), 0, st, x, full * kLeafWaveChunks, s0,
                               jump_tab, part, nodes6, roots, ubits, chunks, full);
            return hipGetLastError();
        }
        const unsigned grid = (unsigned)(split_from / kLeaf2Waves + (full - split_from) + extra);
        hipLaunchKernelGGL(k_leaf64<2>, dim3(grid), dim3(64 * kLeaf2Waves), 0, st, x, full * kLeafWaveChunks, s0,
                           jump_tab, part, nodes6, roots, ubits, chunks, split_from);
        return hipGetLastError();
#else
        return hipErrorInvalidValue;  // (unreachable: split_from is 0)
#endif
    } else if (full > 0)
        hipLaunchKernelGGL((k_leaf2<3, false>), dim3((unsigned)((full + kLeaf2Waves - 1) / kLeaf2Waves)),
                           dim3(64 * kLeaf2Waves), 0, st, x, full * kLeafWaveChunks, s0, jump_tab, part,
                           nodes6, roots, (int64_t)0, ubits);
    if (chunks % kLeafWaveChunks)  // the small trees of the last chunks: one wave
        hipLaunchKernelGGL((k_leaf2<3, true>), dim3(1), dim3(64), 0, st, x, chunks, s0, jump_tab, part,
                           nodes6, roots, full);
    return hipGetLastError();
}

// fp64 leaf: the same wave-persistent kernel over doubles (level-6 nodes and roots as doubles).
hipError_t launch_leaf2_f64(hipStream_t st, const double* x, int64_t chunks, uint64_t s0, const uint64_t* jump_tab,
                            LeafPartial64* part, double* nodes6, double* roots, uint8_t* ubits) {
    const int64_t full = chunks / kLeafWaveChunks;
    if (full > 0)
        hipLaunchKernelGGL((k_leaf2<3, false, double>), dim3((unsigned)((full + kLeaf2Waves - 1) / kLeaf2Waves)),
                           dim3(64 * kLeaf2Waves), 0, st, x, full * kLeafWaveChunks, s0, jump_tab, part, nodes6, roots,
                           (int64_t)0, ubits);
    if (chunks % kLeafWaveChunks)
        hipLaunchKernelGGL((k_leaf2<3, true, double>), dim3(1), dim3(64), 0, st, x, chunks, s0, jump_tab, part, nodes6,
                           roots, full);
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
        case 3: hipLaunchKernelGGL(k_leaf<3>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        case 4: hipLaunchKernelGGL(k_leaf<4>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        // wave-persistent leaf: 20 = load only, 21 = + leaf sort, 23 = full
        case 20: case 21: case 22: case 23: {
            const int64_t tiles = (chunks + kLeafWaveChunks - 1) / kLeafWaveChunks;
            dim3 g2((unsigned)((tiles + kLeaf2Waves - 1) / kLeaf2Waves)), b2(64 * kLeaf2Waves);
            const int64_t z = 0;
            if (stage == 20) hipLaunchKernelGGL((k_leaf2<0>), g2, b2, 0, st, x, chunks, s0, jump_tab, part, scratch, roots, z);
            else if (stage == 21) hipLaunchKernelGGL((k_leaf2<1>), g2, b2, 0, st, x, chunks, s0, jump_tab, part, scratch, roots, z);
            else if (stage == 22) hipLaunchKernelGGL((k_leaf2<2>), g2, b2, 0, st, x, chunks, s0, jump_tab, part, scratch, roots, z);
            else hipLaunchKernelGGL((k_leaf2<3>), g2, b2, 0, st, x, chunks, s0, jump_tab, part, scratch, roots, z);
            break;
        }
        case 5: hipLaunchKernelGGL(k_leaf<5>, g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        // occupancy variants: 10 + stage with >= 6 waves / SIMD (<= 80 VGPRs)
        case 11: hipLaunchKernelGGL((k_leaf<1, 6>), g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        case 13: hipLaunchKernelGGL((k_leaf<3, 6>), g, b, 0, st, x, chunks, s0, jump_tab, part, scratch, roots); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// =============================================================================================
// Summary (one workgroup, any multiple of 64 threads up to 1024)
// =============================================================================================
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

// Exclusive block scan of one non-negative value per thread whose block total stays below 2^32
// (the summary's weights sum to n < 2^31, its split counts to < 2^16): DPP wave scans + one LDS
// round.
__device__ int64_t block_scan_excl(int64_t v, int64_t* wsum, int64_t* total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, nw = blockDim.x >> 6;
    const int64_t x = (int64_t)wave_incl_scan_u32((uint32_t)v);
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
        const int64_t s = (int64_t)wave_incl_scan_u32(lane < nw ? (uint32_t)wsum[lane] : 0u);
        if (lane < nw) wsum[lane] = s;
    }
    __syncthreads();
    const int64_t base = w > 0 ? wsum[w - 1] : 0;
    *total = wsum[nw - 1];
    __syncthreads();
    return base + x - v;
}

struct SummaryArgs {
    const float* x;
    int64_t n;
    const LeafPartial* part;
    int64_t nparts;
    const float* roots;
    const int64_t* ranks;
    uint8_t* payload;
    double* g_raw;
    QuantLut* lut;
    int req_bins;
    int dedup;
    const float* tail;  // base buffer (n % 256 values); null: the input's last n % 256 values
    int sharded;        // 1: the header's n is n_local (a parallelQuantize shard's codes)
    int64_t n_local;
    // min / max / flags pre-reduced by the first merge pass (one per workgroup), which covered
    // leaf tiles [0, part_from); tiles [part_from, nparts) are read from `part` itself
    const LeafPartial* part_red = nullptr;
    int64_t nred = 0;
    int64_t part_from = 0;
};

// pre: this thread's min / max / flags of the leaf partials, already loaded by the caller (the
// fused merge workgroup fetches them before its merge so the load latency hides there); null:
// load them here.
// has_pre: `pre` holds this thread's share of the leaf partials, loaded ahead by the caller (by
// value: a pointer to the caller's local put it in scratch memory, a store and a reload away).
__device__ void summary_block(const SummaryArgs& a, SummaryShared& S, bool has_pre = false,
                              LeafPartial pre = LeafPartial{0xFFFFFFFFu, 0u, 0u, 0u}) {
    const int t = threadIdx.x, T = blockDim.x;
    skml_dense_header* hdr = reinterpret_cast<skml_dense_header*>(a.payload);
    double* splits = reinterpret_cast<double*>(a.payload + kHeaderBytes);
    const int64_t n = a.n;
    const int64_t chunks = n / kChunk;
    const int tail = (int)(n - chunks * kChunk);
    const float* xt = a.tail ? a.tail : a.x + chunks * kChunk;
    const int req_bins = a.req_bins;
    SKML_PROF(2);

    if (t == 0) {
        S.min_key = 0xFFFFFFFFu;
        S.max_key = 0u;
        S.flags = 0u;
        S.zero = 0x7FFFFFFF;
        int nr = 0, off = 0;
        for (int l = 0; l < kMaxLevels; l++)
            if ((chunks >> l) & 1) {  // copyBuf2Arr: lowest level first (HeapQuantileSketch.java:151-161)
                S.run_off[nr] = off;
                S.run_lvl[nr] = l;
                nr++;
                off += kK;
            }
        S.run_off[nr] = off;  // tail = base buffer (weight 1)
        S.run_lvl[nr] = -1;
        S.run_off[nr + 1] = off + tail;
        S.nruns = nr + 1;
    }
    __syncthreads();
    // ---- min / max / NaN ----
    {
        uint32_t mn = 0xFFFFFFFFu, mx = 0u, fl = 0u;
        if (has_pre) {
            mn = pre.min_key;
            mx = pre.max_key;
            fl = pre.flags;
        }
        // the pre-reduced partials first, then the uncovered tiles: batches of 8 independent loads
        // per thread (one memory latency per batch, not per load)
        const int64_t ntot = has_pre ? 0 : a.nred + (a.nparts - a.part_from);
        for (int64_t i0 = t; i0 < ntot; i0 += 8 * (int64_t)T) {
            LeafPartial p[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int64_t i = i0 + (int64_t)k * T;
                p[k] = i < a.nred ? a.part_red[i]
                                  : (i < ntot ? a.part[a.part_from + (i - a.nred)] : LeafPartial{0xFFFFFFFFu, 0u, 0u, 0u});
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                mn = p[k].min_key < mn ? p[k].min_key : mn;
                mx = p[k].max_key > mx ? p[k].max_key : mx;
                fl |= p[k].flags;
            }
        }
        for (int i = t; i < tail; i += T) {
            const uint32_t b = __float_as_uint(xt[i]);
            fl |= is_nan_bits(b) ? 1u : 0u;
            const uint32_t k = f2key(b);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
        // wave reduction (DPP, result in lane 63): one LDS atomic per wave
        mn = wave_reduce_u32_lane63<0>(mn);
        mx = wave_reduce_u32_lane63<1>(mx);
        fl = wave_reduce_u32_lane63<2>(fl);
        if ((t & 63) == 63) {
            atomicMin(&S.min_key, mn);
            atomicMax(&S.max_key, mx);
            if (fl) atomicOr(&S.flags, fl);
        }
    }
    SKML_PROF(3);
    // ---- gather runs; the tail is sorted in Arrays.sort total order by rank counting ----
    const int nruns = S.nruns;
    const int ns = S.run_off[nruns];
    // all level runs in one flat pass (independent loads), the raw tail staged in LDS
    for (int idx = t; idx < (nruns - 1) * kK; idx += T) {
        const int r = idx / kK, i = idx % kK;
        S.smp[S.run_off[r] + i] = a.roots[(size_t)S.run_lvl[r] * kK + i];
    }
    for (int i = t; i < tail; i += T) S.sorted[i] = xt[i];
    __syncthreads();
    {
        const int toff = S.run_off[nruns - 1];
        for (int i = t; i < tail; i += T) {
            const float xi = S.sorted[i];
            const uint32_t ki = f2key(__float_as_uint(xi));
            int rank = 0;
            for (int j = 0; j < tail; j++) {
                const uint32_t kj = f2key(__float_as_uint(S.sorted[j]));
                rank += (kj < ki) || (kj == ki && j < i);
            }
            S.smp[toff + rank] = xi;
        }
    }
    __syncthreads();
    SKML_PROF(4);

    double vmin = 1.7976931348623157e308, vmax = 4.9e-324;  // HeapQuantileSketch.java:67-68
    if (n > 0) {
        const double fmin = (double)__uint_as_float(key2f(S.min_key));
        const double fmax = (double)__uint_as_float(key2f(S.max_key));
        if (fmin <= vmin) vmin = fmin;  // Math.min(Double.MAX_VALUE, x)
        if (fmax > vmax) vmax = fmax;   // Math.max(Double.MIN_VALUE, x)
    }
    if (S.flags & 1u) {  // NaN: QuantileSketchException("Encounter NaN value")
        payload_zero_tail(a.payload, 0, req_bins);
        if (t == 0) {
            hdr->magic = SKML_DENSE_MAGIC;
            hdr->status = SKML_E_NAN;
            hdr->n = a.sharded ? a.n_local : n;
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

    // ---- blockyMergeSort == stable sort under IEEE `<=` (left run wins ties): rank across runs ----
    // The level runs hold kK samples each at q * kK (the base buffer last).
    {
        const int nfull = nruns - 1;
        const float* tail_run = S.smp + S.run_off[nfull];
        for (int i = t; i < ns; i += T) {
            const int r = i < nfull * kK ? i / kK : nfull;
            const float v = S.smp[i];
            int rank = i - S.run_off[r];
            // two level runs at a time: two independent 7-step searches per loop trip, with the
            // IEEE `<=` / `<` choice as a branch-free predicate (a divergent le/lt branch ran
            // both sides); a run paired with itself or the sample's own run counts 0
            for (int q0 = 0; q0 < nfull; q0 += 2) {
                const int q1 = q0 + 1 < nfull ? q0 + 1 : q0;
                const uint32_t use_a = (uint32_t)(q0 != r), use_b = (uint32_t)(q1 != r) & (uint32_t)(q1 != q0);
                if (!(use_a | use_b)) continue;  // e.g. a single level run: nothing to search
                rank += rank_in_run_pair(S.smp + q0 * kK, S.smp + q1 * kK, v, (uint32_t)(q0 < r),
                                         (uint32_t)(q1 < r), use_a, use_b);
            }
            if (r < nfull) rank += run_count_lt(tail_run, tail, v);  // the base buffer comes last
            S.sorted[rank] = v;
            S.w[rank] = S.run_lvl[r] < 0 ? 1 : ((int64_t)2 << S.run_lvl[r]);
        }
    }
    __syncthreads();
    SKML_PROF(5);

    // ---- exclusive prefix of weights (HeapQuantileSketch.java:137-142) ----
    {
        const int per = (ns + T - 1) / T;
        const int b0 = min(ns, t * per), b1 = min(ns, b0 + per);
        int64_t loc = 0;
        for (int i = b0; i < b1; i++) loc += S.w[i];
        const int64_t base = block_scan_excl(loc, S.wsum, &S.total);
        int64_t acc = base;
        for (int i = b0; i < b1; i++) {
            const int64_t wv = S.w[i];
            S.w[i] = acc;
            acc += wv;
        }
        if (t == 0) S.w[ns] = S.total;
    }
    __syncthreads();
    SKML_PROF(6);

    // ---- getQuantiles(int): split_i = samples[max idx with cut[idx] <= rank_i] ----
    const int nsplit_req = req_bins - 1;
    const bool lds_raw = nsplit_req <= kSumMaxRaw;
    double* raw = lds_raw ? S.raw : a.g_raw;
    for (int i = t; i < nsplit_req; i += T) {
        double sp;
        if (ns == 0) {
            sp = __longlong_as_double(0x7FF8000000000000LL);  // NaN (HeapQuantileSketch.java:299-301)
        } else {
            const int64_t rank = a.ranks[i];
            int lo = 0, hi = ns;
            while (lo + 1 < hi) {
                const int mid = (lo + hi) >> 1;
                if (S.w[mid] <= rank) lo = mid;
                else hi = mid;
            }
            sp = (double)S.sorted[lo];
        }
        raw[i] = sp;
    }
    if (!lds_raw) __threadfence();
    __syncthreads();
    SKML_PROF(7);

    // ---- Maths.unique (IEEE !=, keep first) + findZeroIdx ----
    int bin_num;
    {
        const int per = (nsplit_req + T - 1) / T;
        const int b0 = min(nsplit_req, t * per), b1 = min(nsplit_req, b0 + per);
        int64_t loc = 0;
        for (int i = b0; i < b1; i++) loc += (!a.dedup || i == 0 || raw[i] != raw[i - 1]) ? 1 : 0;
        const int64_t base = block_scan_excl(loc, S.wsum, &S.total);
        int64_t o = base;
        int zmin = 0x7FFFFFFF;
        for (int i = b0; i < b1; i++) {
            if (!a.dedup || i == 0 || raw[i] != raw[i - 1]) {
                const double sp = raw[i];
                splits[o] = sp;
                if (o < kMaxSamples) S.smp[o] = (float)sp;  // LDS copy for the quantize LUT
                if (!(sp < 0.0)) zmin = min(zmin, (int)o);
                o++;
            }
        }
        zmin = (int)wave_reduce_u32_lane63<0>((uint32_t)zmin);  // indices >= 0: unsigned min
        if ((t & 63) == 63 && zmin != 0x7FFFFFFF) atomicMin(&S.zero, zmin);  // one LDS atomic per wave
        bin_num = (int)S.total + 1;
    }
    __syncthreads();
    payload_zero_tail(a.payload, bin_num - 1, req_bins);
    SKML_PROF(8);
    if (t == 0) {
        int zero;
        if (vmin > 0.0) zero = 0;
        else if (vmax < 0.0) zero = bin_num - 1;
        else zero = S.zero < bin_num - 1 ? S.zero : bin_num - 1;
        hdr->magic = SKML_DENSE_MAGIC;
        hdr->status = SKML_OK;
        hdr->n = a.sharded ? a.n_local : n;
        hdr->bin_num = bin_num;
        hdr->zero_idx = zero;
        hdr->code_bits = code_bits_for(bin_num);
        hdr->req_bins = req_bins;
        hdr->min = vmin;
        hdr->max = vmax;
        hdr->codes_offset = (int64_t)dense_codes_offset(req_bins);
        hdr->reserved = 0;
    }
    // ---- quantize bucket LUT over the final split table ----
    const int nsplit = bin_num - 1;
    if (nsplit <= kMaxSamples && nsplit <= kLutMaxSplits && n > 0) {
        SKML_PROF(9);
#ifdef SKML_PROF_SUMMARY
        if (threadIdx.x == 0) g_prof[28] = __builtin_amdgcn_s_memtime();
#endif
        // LDS staging of the table aliases sorted[] + w[] (both dead after getQuantiles)
#ifdef SKML_PROF_SUMMARY
        unsigned long long* lprof = g_prof + 30;
#else
        unsigned long long* lprof = nullptr;
#endif
        build_quant_lut(S.smp, nsplit, a.lut, reinterpret_cast<int*>(S.wsum), reinterpret_cast<uint32_t*>(S.sorted),
                        lprof);
    } else if (t == 0) {
        a.lut->cmax = -1;
    }
    SKML_PROF(10);
#ifdef SKML_PROF_SUMMARY
    if (threadIdx.x == 0) g_prof[29] = __builtin_amdgcn_s_memtime();
#endif
}

__global__ __launch_bounds__(512) void k_summary(SummaryArgs a) {
    __shared__ SummaryShared S;
    summary_block(a, S);
}

hipError_t launch_summary(hipStream_t st, const float* x, int64_t n, const LeafPartial* part,
                          int64_t nparts, const float* roots, const int64_t* ranks, int req_bins,
                          int dedup, void* payload, double* scratch_raw, QuantLut* lut) {
    SummaryArgs a{x, n, part, nparts, roots, ranks, reinterpret_cast<uint8_t*>(payload), scratch_raw,
                  lut, req_bins, dedup};
    hipLaunchKernelGGL(k_summary, dim3(1), dim3(512), 0, st, a);
    return hipGetLastError();
}

// =============================================================================================
// Upper merge levels: each workgroup merges 2^g (g <= 6) consecutive level-L nodes of one tree.
// Input nodes are placed like leaf chunks (8 per wave, 8 lanes x 16 keys per node); missing
// nodes (g < 6) are padding whose merges are never exported.
// =============================================================================================
template <typename S = float>
struct MergeExport {
    int lane, wave, g;
    S* out;
    template <int R, typename T>
    __device__ __forceinline__ void at(int level, int node, const T (&w)[R]) const {
        if (level == g && wave == 0 && node == 0) store_node<R>(w, lane, out);
    }
};

// One workgroup's share of a merge pass: 2^g consecutive level-L nodes of one tree -> one node.
// E = float: nodes sorted as total-order keys; E = double: as doubles (v_min/v_max_f64).
template <typename E = float>
__device__ __forceinline__ void merge_group_wg(const MergePass& pass, int wg, const E* __restrict__ src,
                                               E* __restrict__ dst, E* __restrict__ roots, uint64_t s0,
                                               const uint64_t* __restrict__ tab, TileSharedT<E>& sh,
                                               const uint8_t* __restrict__ ubits, int64_t uchunks,
                                               const LeafPartial* __restrict__ part_in = nullptr,
                                               LeafPartial* __restrict__ part_red = nullptr, int prof = -1) {
#ifdef SKML_PROF_SUMMARY
#define SKML_PROF_AT(k)                                                  \
    do {                                                                 \
        if (prof >= 0 && threadIdx.x == 0) g_prof[prof + (k)] = wall_clock64(); \
    } while (0)
#else
#define SKML_PROF_AT(k) \
    do {                \
    } while (0)
#endif
    SKML_PROF_AT(0);
    using T = typename std::conditional<std::is_same<E, double>::value, double, uint32_t>::type;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int j = 0;
    while (j + 1 < pass.njobs && wg >= pass.wg_prefix[j + 1]) j++;
    const MergeJob job = pass.job[j];
    const int grp = wg - pass.wg_prefix[j];
    const int g = job.group_log, L = job.level_in;
    const int nodes = 1 << g;
    const int64_t node0 = job.src_node + ((int64_t)grp << g);
    const int64_t chunk0 = job.chunk_base + ((int64_t)grp << (g + L));
    E* out = job.root_level >= 0 ? roots + (size_t)job.root_level * kK : dst + (size_t)(job.dst_node + grp) * kK;
    if (tid == 0) sh.flags = 0u;
    // this lane's compaction bit, drawn by the leaf (k_leaf2, upper_level_offset numbering); the
    // load is issued first so its latency hides behind the node loads.  Padding merges (g < 6)
    // read a clamped index: their bits are never used.
    uint32_t bsel = 0;
    {
        int lo = -1, last_node = 0;
        if (lane < 4) lo = 1, last_node = wave * 8 + 2 * lane + 1;
        else if (lane < 6) lo = 2, last_node = wave * 8 + 4 * (lane - 4) + 3;
        else if (lane == 6) lo = 3, last_node = wave * 8 + 7;
        else if (wave == 0 && lane >= 8 && lane < 12) lo = 4, last_node = 16 * (lane - 8) + 15;
        else if (wave == 0 && lane >= 12 && lane < 14) lo = 5, last_node = 32 * (lane - 12) + 31;
        else if (wave == 0 && lane == 14) lo = 6, last_node = 63;
        if (lo > 0) {
            const int lvl = L + lo;
            const int64_t i = ((chunk0 + ((int64_t)(last_node + 1) << L)) >> lvl) - 1;
            const int64_t cnt = upper_node_count(uchunks);
            int64_t idx = upper_level_offset(uchunks, lvl) + i;
            idx = idx < cnt ? idx : cnt - 1;
            bsel = ubits[idx < 0 ? 0 : idx];
        }
    }
    (void)tab;
    (void)s0;
    // first pass (level-6 input nodes = leaf tiles): wave 0 reduces the tiles' min / max / flags
    // for the summary (SummaryArgs::part_red); the load hides behind the node loads too
    const bool reduce_parts = part_red && L == kLeafTopLevel && wave == 0;
    LeafPartial tp{0xFFFFFFFFu, 0u, 0u, 0u};
    if (reduce_parts && lane < nodes) tp = part_in[node0 + lane];
    __syncthreads();

    // ---- load: node nd = 8*wave + lane/8, 16 floats per lane ----
    const int nd = wave * 8 + (lane >> 3);
    const bool valid = nd < nodes;
    T w1[16];
    uint32_t fl = 0;
    if constexpr (std::is_same<E, double>::value) {
        const double2* p = reinterpret_cast<const double2*>(src + (size_t)(node0 + (valid ? nd : 0)) * kK) + (lane & 7) * 8;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const double2 f = p[q];
            const double e2[2] = {f.x, f.y};
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const uint64_t b = (uint64_t)__double_as_longlong(e2[e]);
                fl |= (b == 0x8000000000000000ull) ? 2u : 0u;
                fl |= (b == 0ull) ? 4u : 0u;
                w1[q * 2 + e] = e2[e];  // padding nodes (g < 6) never meet a real node
            }
        }
    } else {
        const float4* p = reinterpret_cast<const float4*>(src + (size_t)(node0 + (valid ? nd : 0)) * kK) + (lane & 7) * 4;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float4 f = p[q];
            const uint32_t b[4] = {__float_as_uint(f.x), __float_as_uint(f.y), __float_as_uint(f.z),
                                   __float_as_uint(f.w)};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                fl |= (b[e] == 0x80000000u) ? 2u : 0u;
                fl |= (b[e] == 0u) ? 4u : 0u;
                w1[q * 4 + e] = valid ? f2key(b[e]) : 0xFFFFFFFFu;
            }
        }
    }
    if (!valid) fl = 0;
    SKML_PROF_AT(1);
    if (reduce_parts) {
        uint32_t mn = tp.min_key, mx = tp.max_key, f = tp.flags;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t omn = (uint32_t)__shfl_xor((int)mn, off, 64), omx = (uint32_t)__shfl_xor((int)mx, off, 64);
            mn = omn < mn ? omn : mn;
            mx = omx > mx ? omx : mx;
            f |= (uint32_t)__shfl_xor((int)f, off, 64);
        }
        if (lane == 0) part_red[wg] = LeafPartial{mn, mx, f, 0u};
    }
    // ---- the RNG bits fetched at the top (lane k < 7: an in-wave merge; wave 0 lanes 8..14: the
    // cross-wave ones) ----
    uint32_t ibits;
    {
        const uint64_t m = __ballot(bsel != 0);
        ibits = (uint32_t)m & 0x7Fu;
        if (wave == 0 && lane == 0) sh.wgbits = (uint32_t)(m >> 8) & 0x7Fu;
    }
#ifdef SKML_PROF_SUMMARY
    if (prof == 16 && threadIdx.x == 0) g_prof[22] = wall_clock64();
#endif
    if (fl) atomicOr(&sh.flags, fl);
    const bool wexact = (__ballot((fl & 2u) != 0) != 0) && (__ballot((fl & 4u) != 0) != 0);
    const MergeExport<E> exp{lane, wave, g, out};
    T w4[2];
    inwave_levels(w1, w4, lane, ibits, wexact, sh.fb[wave], exp, prof == 16);
    store_node<2>(w4, lane, sh.wn[wave]);
    __syncthreads();
    SKML_PROF_AT(2);
    if (g >= 4) {
        crosswave_levels<T>(sh, tid, sh.wgbits, (sh.flags & 6u) == 6u);
        if (tid < kK) out[tid] = g == 4 ? sh.l4[0][tid] : (g == 5 ? sh.l5[0][tid] : sh.l6[tid]);
    }
    SKML_PROF_AT(3);
}

// A merge pass.  `next` (njobs > 0) is a one-workgroup pass that the pass's last workgroup runs
// itself once every output of this pass is written (the last-arriver protocol below), so the
// two passes need one launch; the summary then follows in the same workgroup.
__global__ __launch_bounds__(512) void k_merge(MergePass pass, MergePass next, const float* __restrict__ src,
                                               float* __restrict__ dst, float* __restrict__ next_dst,
                                               float* __restrict__ roots, uint64_t s0,
                                               const uint64_t* __restrict__ tab, unsigned* __restrict__ done,
                                               SummaryArgs sa, const uint8_t* __restrict__ ubits, int64_t uchunks) {
    __shared__ MergeShared U;
    const int tid = threadIdx.x;
    if (pass.fuse_summary && gridDim.x == 1) SKML_PROF(0);
    merge_group_wg(pass, (int)blockIdx.x, src, dst, roots, s0, tab, U.t, ubits, uchunks, sa.part,
                   const_cast<LeafPartial*>(sa.part_red), blockIdx.x == 0 ? 12 : -1);
    const bool has_next = next.njobs > 0;
    if (!pass.fuse_summary && !has_next) return;

    // ---- last workgroup: the trailing pass and / or the summary (release/acquire per Guideline 16) ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = atomicAdd(done, 1u);
        const int last = old == (unsigned)(pass.wg_prefix[pass.njobs] - 1);
        if (last) {
#ifdef SKML_PROF_SUMMARY
            g_prof[20] = wall_clock64();
#endif
            *done = 0u;  // reset for the next encode
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef SKML_PROF_SUMMARY
            g_prof[21] = wall_clock64();
#endif
        }
        U.t.is_last = last;
    }
    __syncthreads();
    if (!U.t.is_last) return;
    __syncthreads();
    // the summary's leaf partials, fetched now so their latency hides behind the merge below
    LeafPartial pre{0xFFFFFFFFu, 0u, 0u, 0u};
    const int64_t npre = sa.nred + (sa.nparts - sa.part_from);
    const bool prefetch = pass.fuse_summary || next.fuse_summary ? npre <= (int64_t)blockDim.x : false;
    if (prefetch && tid < npre) pre = tid < sa.nred ? sa.part_red[tid] : sa.part[sa.part_from + (tid - sa.nred)];
    if (has_next) {
        SKML_PROF(0);
        // the trailing pass's merges (independent trees), one after another in this workgroup
        const int nnext = next.wg_prefix[next.njobs];
        for (int w = 0; w < nnext; w++) {
            if (w) __syncthreads();
            merge_group_wg(next, w, dst, next_dst, roots, s0, tab, U.t, ubits, uchunks, nullptr, nullptr,
                           w == 0 ? 16 : -1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        if (!next.fuse_summary) return;
    }
    SKML_PROF(1);
    summary_block(sa, U.s, prefetch, pre);
#ifdef SKML_PROF_WARM
    // diagnostic build: the summary again with warm instruction / data caches (phases 2..10 then
    // hold the second run; 26 / 27 bracket it)
    __syncthreads();
    if (threadIdx.x == 0) g_prof[26] = wall_clock64();
    summary_block(sa, U.s);
    __syncthreads();
    if (threadIdx.x == 0) g_prof[27] = wall_clock64();
#endif
}

hipError_t launch_merge_pass(hipStream_t st, const MergePass& pass, const MergePass* next, const float* src,
                             float* dst, float* next_dst, float* roots, uint64_t s0, const uint64_t* jump_tab,
                             unsigned* done, const float* x, int64_t n, const LeafPartial* part, int64_t nparts,
                             const int64_t* ranks, int req_bins, int dedup, void* payload,
                             double* scratch_raw, QuantLut* lut, const uint8_t* ubits, LeafPartial* part_red,
                             int64_t nred, int64_t part_from) {
    const int nwg = pass.wg_prefix[pass.njobs];
    if (nwg <= 0) return hipSuccess;
    SummaryArgs a{x, n, part, nparts, roots, ranks, reinterpret_cast<uint8_t*>(payload), scratch_raw,
                  lut, req_bins, dedup};
    a.part_red = part_red;  // written by the first pass (this launch or an earlier one)
    a.nred = nred;
    a.part_from = part_from;
    MergePass none;
    if (!next) {
        std::memset(&none, 0, sizeof(none));
        next = &none;
    }
    const int64_t uchunks = (n / kChunk / kLeafWaveChunks) * kLeafWaveChunks;
    hipLaunchKernelGGL(k_merge, dim3(nwg), dim3(512), 0, st, pass, *next, src, dst, next_dst, roots, s0, jump_tab,
                       done, a, ubits, uchunks);
    return hipGetLastError();
}

// fp64 merge pass (no fused summary: k_summary64 follows); `next` as in k_merge.
__global__ __launch_bounds__(512) void k_merge64(MergePass pass, MergePass next, const double* __restrict__ src,
                                                 double* __restrict__ dst, double* __restrict__ next_dst,
                                                 double* __restrict__ roots, uint64_t s0,
                                                 const uint64_t* __restrict__ tab, unsigned* __restrict__ done,
                                                 const uint8_t* __restrict__ ubits, int64_t uchunks) {
    __shared__ TileSharedT<double> T64;
    const int tid = threadIdx.x;
    merge_group_wg<double>(pass, (int)blockIdx.x, src, dst, roots, s0, tab, T64, ubits, uchunks);
    if (next.njobs == 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = atomicAdd(done, 1u);
        const int last = old == (unsigned)(pass.wg_prefix[pass.njobs] - 1);
        if (last) {
            *done = 0u;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        T64.is_last = last;
    }
    __syncthreads();
    if (!T64.is_last) return;
    __syncthreads();
    const int nnext = next.wg_prefix[next.njobs];
    for (int w = 0; w < nnext; w++) {
        if (w) __syncthreads();
        merge_group_wg<double>(next, w, dst, next_dst, roots, s0, tab, T64, ubits, uchunks);
    }
}

hipError_t launch_merge_pass64(hipStream_t st, const MergePass& pass, const MergePass* next, const double* src,
                               double* dst, double* next_dst, double* roots, uint64_t s0, const uint64_t* jump_tab,
                               unsigned* done, const uint8_t* ubits, int64_t uchunks) {
    const int nwg = pass.wg_prefix[pass.njobs];
    if (nwg <= 0) return hipSuccess;
    MergePass none;
    if (!next) {
        std::memset(&none, 0, sizeof(none));
        next = &none;
    }
    hipLaunchKernelGGL(k_merge64, dim3(nwg), dim3(512), 0, st, pass, *next, src, dst, next_dst, roots, s0, jump_tab,
                       done, ubits, uchunks);
    return hipGetLastError();
}

// Split-injected parity mode: header from caller splits (Quantizer.findZeroIdx rule).
__global__ __launch_bounds__(256) void k_set_splits(uint8_t* payload, int64_t n, const double* __restrict__ sp,
                                                    int nsplits, double mn, double mx, int req_bins,
                                                    QuantLut* lut) {
    skml_dense_header* hdr = reinterpret_cast<skml_dense_header*>(payload);
    double* splits = reinterpret_cast<double*>(payload + kHeaderBytes);
    __shared__ int s_zero;
    __shared__ int s_misc[20];
    __shared__ float s_sp[kLutMaxSplits];
    __shared__ __align__(16) uint32_t s_lbuf[kLutSize / 2];
    if (threadIdx.x == 0) s_zero = 0x7FFFFFFF;
    __syncthreads();
    for (int i = threadIdx.x; i < nsplits; i += blockDim.x) {
        splits[i] = sp[i];
        if (i < kLutMaxSplits) s_sp[i] = __double2float_ru(sp[i]);
        if (!(sp[i] < 0.0)) atomicMin(&s_zero, i);
    }
    payload_zero_tail(payload, nsplits, req_bins);
    __syncthreads();
    if (nsplits <= kLutMaxSplits) build_quant_lut(s_sp, nsplits, lut, s_misc, s_lbuf);
    else if (threadIdx.x == 0) lut->cmax = -1;
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

// HeapQuantileSketch.getQuantiles' ranks (HeapQuantileSketch.java:305-320): rank_i = min((long)(n *
// curFrac), n - 1) with curFrac += 1/bins accumulated in double, in order (one lane), the same
// IEEE double sequence as the JVM (built with -ffp-contract=off).  On the device so that a new n
// (every sparse payload's nnz) costs no host upload and no synchronisation.
__global__ __launch_bounds__(64) void k_set_ranks(int64_t n, int bins, int64_t* __restrict__ ranks) {
    // lane 0 runs the dependent chain of additions (one v_add_f64 each) into LDS, 1,024 at a time;
    // the wave then converts them in parallel (the double -> int64 conversion is the long part)
    constexpr int kChunk = 1024;
    __shared__ double fr[kChunk];
    const int lane = threadIdx.x;
    const double step = 1.0 / bins;
    double frac = step;
    for (int i0 = 0; i0 < bins - 1; i0 += kChunk) {
        const int m = min(kChunk, bins - 1 - i0);
        if (lane == 0)
            for (int j = 0; j < m; j++) {
                fr[j] = frac;
                frac = frac + step;
            }
        __syncthreads();
        for (int j = lane; j < m; j += 64) {
            int64_t r = (int64_t)((double)n * fr[j]);
            if (r > n - 1) r = n - 1;
            ranks[i0 + j] = r;
        }
        __syncthreads();
    }
}

hipError_t launch_set_ranks(hipStream_t st, int64_t n, int bins, int64_t* ranks) {
    hipLaunchKernelGGL(k_set_ranks, dim3(1), dim3(64), 0, st, n, bins, ranks);
    return hipGetLastError();
}

hipError_t launch_set_splits(hipStream_t st, void* payload, int64_t n, const double* splits_dev,
                             int nsplits, double mn, double mx, int req_bins, QuantLut* lut) {
    hipLaunchKernelGGL(k_set_splits, dim3(1), dim3(256), 0, st, reinterpret_cast<uint8_t*>(payload),
                       n, splits_dev, nsplits, mn, mx, req_bins, lut);
    return hipGetLastError();
}

// =============================================================================================
// QuantileQuantizer.parallelQuantize with T slices (QuantileQuantizer.java:53-92): each slice is
// sketched by the normal leaf + merge passes (its compaction bits from its own offset into the
// one Random stream), exported as a SketchRecord, and the records are merged in slice order by
// one workgroup replaying HeapQuantileSketch.merge (HeapQuantileSketch.java:186-228): the other
// sketch's base items go through update() (a full base buffer is sorted, compacted and carried),
// then each of its levels is carried up from its own level (inPlacePropagationMerge).  The
// merged state feeds summary_block unchanged.
// =============================================================================================
__global__ __launch_bounds__(512) void k_sketch_record(const float* __restrict__ x, int64_t n,
                                                       const LeafPartial* __restrict__ part, int64_t nparts,
                                                       const float* __restrict__ roots, SketchRecord* rec) {
    __shared__ uint32_t s_mn, s_mx, s_fl;
    const int t = threadIdx.x, T = blockDim.x;
    const int64_t chunks = n / kChunk;
    const int tail = (int)(n - chunks * kChunk);
    const float* xt = x + chunks * kChunk;
    if (t == 0) {
        s_mn = 0xFFFFFFFFu;
        s_mx = 0u;
        s_fl = 0u;
    }
    __syncthreads();
    uint32_t mn = 0xFFFFFFFFu, mx = 0u, fl = 0u;
    for (int64_t i = t; i < nparts; i += T) {
        const LeafPartial p = part[i];
        mn = p.min_key < mn ? p.min_key : mn;
        mx = p.max_key > mx ? p.max_key : mx;
        fl |= p.flags;
    }
    for (int i = t; i < tail; i += T) {
        const uint32_t b = __float_as_uint(xt[i]);
        fl |= is_nan_bits(b) ? 1u : 0u;
        const uint32_t k = f2key(b);
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
        rec->tail[i] = xt[i];
    }
    atomicMin(&s_mn, mn);
    atomicMax(&s_mx, mx);
    if (fl) atomicOr(&s_fl, fl);
    for (int l = 0; l < kMaxLevels; l++)
        if ((chunks >> l) & 1)
            for (int i = t; i < kK; i += T) rec->level[l][i] = roots[(size_t)l * kK + i];
    __syncthreads();
    if (t == 0) {
        rec->n = n;
        rec->mm = LeafPartial{s_mn, s_mx, s_fl, 0u};
        rec->pad = 0;
    }
}

hipError_t launch_sketch_record(hipStream_t st, const float* x, int64_t n, const LeafPartial* part, int64_t nparts,
                                const float* roots, SketchRecord* rec) {
    hipLaunchKernelGGL(k_sketch_record, dim3(1), dim3(512), 0, st, x, n, part, nparts, roots, rec);
    return hipGetLastError();
}

struct SkMergeShared {
    float lv[kMaxLevels][kK];
    float base[kChunk];
    float tmp[kChunk];
};
union SkMergeUnion {
    SkMergeShared m;
    SummaryShared s;
};

__global__ __launch_bounds__(512) void k_sketch_merge(const SketchRecord* __restrict__ recs, int nrec, uint64_t s0,
                                                      uint64_t bit0, const uint64_t* __restrict__ tab,
                                                      SummaryArgs a, float* g_roots, float* g_tail,
                                                      LeafPartial* g_part) {
    __shared__ SkMergeUnion U;
    SkMergeShared& M = U.m;
    const int t = threadIdx.x;
    // control state is uniform: every thread keeps its own identical copy
    uint64_t pattern = 0, bit = bit0;
    int64_t nacc = 0;
    int base_cnt = 0;

    auto first_free = [&](int from) {
        int l = from;
        while ((pattern >> l) & 1ull) l++;
        return l;
    };
    // levelwisePropagation (QSketchUtils.java:71-82): carry lv[dest] through levels [from, dest)
    auto carry = [&](int from, int dest) {
        for (int l = from; l < dest; l++) {
            const uint32_t odd = lcg_bit(tab, s0, bit++);
            if (t < kChunk) exact_merge_task(M.lv[l], M.lv[dest], M.tmp, t, odd);
            __syncthreads();
            if (t < kK) M.lv[dest][t] = M.tmp[t];
            __syncthreads();
        }
    };
    // fullBaseBufferPropagation (HeapQuantileSketch.java:107-124): Arrays.sort, compact, carry
    auto flush_base = [&]() {
        if (t < kChunk) {
            const float v = M.base[t];
            const uint32_t kv = f2key(__float_as_uint(v));
            int rank = 0;
            for (int j = 0; j < kChunk; j++) {
                const uint32_t kj = f2key(__float_as_uint(M.base[j]));
                rank += (kj < kv) || (kj == kv && j < t);
            }
            M.tmp[rank] = v;
        }
        __syncthreads();
        const int dest = first_free(0);
        const uint32_t odd = lcg_bit(tab, s0, bit++);
        if (t < kK) M.lv[dest][t] = M.tmp[2 * t + odd];
        __syncthreads();
        carry(0, dest);
        pattern += 1;
        base_cnt = 0;
    };

    for (int r = 0; r < nrec; r++) {
        const SketchRecord* R = recs + r;
        const int64_t rn = R->n;
        if (rn <= 0) continue;  // other.isEmpty()
        const uint64_t rpat = (uint64_t)(rn / kChunk);
        const int rtail = (int)(rn % kChunk);
        if (nacc == 0) {  // this.isEmpty(): copy(other), no compaction
            for (int l = 0; l < kMaxLevels; l++)
                if ((rpat >> l) & 1ull)
                    if (t < kK) M.lv[l][t] = R->level[l][t];
            if (t < rtail) M.base[t] = R->tail[t];
            __syncthreads();
            pattern = rpat;
            base_cnt = rtail;
            nacc = rn;
            continue;
        }
        // other's base items through update()
        for (int i = 0; i < rtail;) {
            const int take = min(rtail - i, kChunk - base_cnt);
            if (t < take) M.base[base_cnt + t] = R->tail[i + t];
            __syncthreads();
            base_cnt += take;
            i += take;
            if (base_cnt == kChunk) flush_base();
        }
        // other's levels, bottom-up (inPlacePropagationMerge)
        for (int l = 0; l < kMaxLevels; l++) {
            if (!((rpat >> l) & 1ull)) continue;
            const int dest = first_free(l);
            if (t < kK) M.lv[dest][t] = R->level[l][t];
            __syncthreads();
            carry(l, dest);
            pattern += 1ull << l;
        }
        nacc += rn;
    }
    // export the merged sketch in the summary's layout (levels by index, base buffer, partials)
    for (int l = 0; l < kMaxLevels; l++)
        if ((pattern >> l) & 1ull)
            if (t < kK) g_roots[(size_t)l * kK + t] = M.lv[l][t];
    if (t < base_cnt) g_tail[t] = M.base[t];
    for (int r = t; r < nrec; r += blockDim.x) g_part[r] = recs[r].mm;
    __threadfence();
    __syncthreads();
    summary_block(a, U.s);
}

hipError_t launch_sketch_merge(hipStream_t st, const SketchRecord* recs, int nrec, uint64_t s0, uint64_t bit0,
                               const uint64_t* jump_tab, int64_t n_total, int64_t n_local, const int64_t* ranks,
                               int req_bins, int dedup, void* payload, double* scratch_raw, QuantLut* lut,
                               float* scratch_roots, float* scratch_tail, LeafPartial* scratch_part) {
    SummaryArgs a{nullptr, n_total, scratch_part, nrec, scratch_roots, ranks, reinterpret_cast<uint8_t*>(payload),
                  scratch_raw, lut, req_bins, dedup, scratch_tail, 1, n_local};
    hipLaunchKernelGGL(k_sketch_merge, dim3(1), dim3(512), 0, st, recs, nrec, s0, bit0, jump_tab, a, scratch_roots,
                       scratch_tail, scratch_part);
    return hipGetLastError();
}

}  // namespace skml

#ifdef SKML_PROF_LEAF
extern "C" int skml_debug_leafprof(unsigned long long* out, int cap) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(skml::g_leafprof), sizeof(unsigned long long) * (size_t)cap) ==
                   hipSuccess ? SKML_OK : SKML_E_HIP;
}
#endif
extern "C" int skml_debug_prof(unsigned long long* out, int cap) {
    if (!out || cap <= 0) return SKML_E_ARG;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(skml::g_prof), sizeof(unsigned long long) * (size_t)(cap < 32 ? cap : 32)) ==
                   hipSuccess
               ? SKML_OK
               : SKML_E_HIP;
}
