// skml_sparse.hip -- CDNA4 (gfx950) kernels of the sparse codec (SketchGradient.fromSparse /
// SparseVectorCompressor.compressSparse and restore):
//   k_compact        DenseDoubleGradient.toSparse (ml/gradient/DenseDoubleGradient.scala:64-89):
//                    single-pass stream compaction with decoupled look-back (ticketed tiles).
//   k_part_*         FSketchUtils.partition (frequency/FSketchUtils.java:30-47): stable counting
//                    sort of (key, bin) by group, group = #{edges <= bin}.
//   k_group_prep     DeltaAdaptiveEncoder.encode step 1 (binary/DeltaAdaptiveEncoder.java:54-71)
//                    and MinMaxSketch.insert (frequency/MinMaxSketch.java:48-55) as a 64-bit
//                    atomicMin on (|bin-zero|, key, bin): the smaller distance wins, ties keep the
//                    earlier (= smaller key, keys ascend within a group) insert.
//   k_delta_*        DeltaAdaptiveEncoder.encode step 3 (:72-109): per-element bit lengths, a
//                    tile scan, and a writer that packs MSB-first fields (BinaryUtils.setBits) into
//                    an LDS window of 64-bit BitSet words, flushing boundary words atomically.
//   k_unary_* / k_dec_*  DeltaAdaptiveEncoder.decode (:114-146) in parallel: unary flags are
//                    resolved by selecting zero bits, delta offsets and keys by scans.
//   k_merge_round    Sort.merge (util/Sort.java:362-379) as rounds of stable merge-path merges.
#include <algorithm>
#include <type_traits>

#include "skml_device.hpp"
#include "skml_sparse.h"

namespace skml {

constexpr uint64_t kStAgg = 1ULL << 62, kStPre = 2ULL << 62, kStMask = (1ULL << 62) - 1;
constexpr uint32_t kEpsBelowBits = 0x322BCC77u;  // the largest float <= 1e-8 (Maths.scala:8 EPS)

// ---------------------------------------------------------------------------------------------
// block scan helpers (256 threads)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(v, off, 64);
        if (lane >= off) v += y;
    }
    return v;
}

// v[k] -> exclusive prefix over the block; total[k] = block sum.  sh: 4*K u64 of LDS.
template <int K>
__device__ __forceinline__ void block_excl_scan(uint64_t (&v)[K], uint64_t (&total)[K], uint64_t* sh) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t inc[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        inc[k] = wave_incl_u64(v[k], lane);
        if (lane == 63) sh[w * K + k] = inc[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        uint64_t base = 0, tot = 0;
#pragma unroll
        for (int j = 0; j < kSpThreads / 64; j++) {
            const uint64_t s = sh[j * K + k];
            base += j < w ? s : 0;
            tot += s;
        }
        v[k] = base + inc[k] - v[k];
        total[k] = tot;
    }
    __syncthreads();
}

// Look-back status words carry their payload (flag | count) in the word itself, so relaxed
// agent-scope atomics suffice: no release / acquire fences (an agent release writes back the
// whole L2 -- per tile, that was 30x slower).
__device__ __forceinline__ uint64_t ld_status(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A count the host may be polling in coherent host memory (ctx_host_word): a system-scope store,
// so it is not held in L2.  No release: the host only reads the value, and everything that reads
// the compaction's output runs later on the same stream.
__device__ __forceinline__ void put_count(int64_t* p, int64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifndef SKML_LOOKBACK_ROWS
#define SKML_LOOKBACK_ROWS 1  // predecessors per look-back step = 64 x this (A/B builds vary it)
#endif
// Decoupled look-back of one wave: the sum of the counts of the tiles before `tile` (every lane
// gets it).  One step loads 64 x K predecessors' status words at once (K per lane, all in flight),
// then walks them nearest first, in rows of 64, to the nearest inclusive prefix.  The tiles in
// flight finish at about the same time, so the nearest prefix sits several hundred tiles back: at
// 64 per step that took a dozen dependent L2 round trips per tile.
template <int K>
__device__ __forceinline__ uint64_t lookback_excl(const uint64_t* status, int64_t tile, int lane) {
    uint64_t acc = 0;
    int64_t p = tile - 1;
    bool done = false;
    while (!done) {
        uint64_t sv[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int64_t idx = p - (int64_t)(k * 64 + lane);
            sv[k] = idx >= 0 ? ld_status(&status[idx]) : kStPre;  // before tile 0: prefix 0
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (!done) {  // (no break: sv stays in registers only while every index is static)
                const int64_t idx = p - (int64_t)(k * 64 + lane);
                while (__ballot((sv[k] & ~kStMask) == 0)) {
                    __builtin_amdgcn_s_sleep(1);
                    if ((sv[k] & ~kStMask) == 0) sv[k] = ld_status(&status[idx]);
                }
                const uint64_t pre = __ballot((sv[k] & ~kStMask) == kStPre);
                const int stop = pre ? __ffsll((unsigned long long)pre) - 1 : 63;
                acc += lane <= stop ? (sv[k] & kStMask) : 0;
                done = pre != 0;
            }
        }
        p -= 64 * K;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    return acc;
}

// packed code of element e (LSB-first codes, code_bits in {1,2,4,8,16})
__device__ __forceinline__ int32_t code_at(const uint8_t* codes, int64_t e, int bits) {
    switch (bits) {
        case 8: return codes[e];
        case 16: return reinterpret_cast<const uint16_t*>(codes)[e];
        case 4: return (codes[e >> 1] >> ((e & 1) * 4)) & 15;
        case 2: return (codes[e >> 2] >> ((e & 3) * 2)) & 3;
        default: return (codes[e >> 3] >> (e & 7)) & 1;
    }
}

// #{edges[j] <= bin} over a sorted 64-entry LDS table padded with INT32_MAX
__device__ __forceinline__ int group_of_bin(const int32_t* E, int32_t bin) {
    int g = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
        if (E[g + step - 1] <= bin) g += step;
    return g;
}
// group g with gstart[g] <= i < gstart[g+1] (S: G+1 offsets in LDS, padded to 65 with INT64_MAX)
__device__ __forceinline__ int group_of_elem(const int64_t* S, int64_t i) {
    int g = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
        if (S[g + step] <= i) g += step;
    return g;
}

__device__ __forceinline__ void load_edges(const SpGroups* gp, int32_t* E) {
    for (int j = threadIdx.x; j < kMaxGroups; j += blockDim.x) E[j] = j < gp->G ? gp->edges[j] : INT32_MAX;
}
__device__ __forceinline__ void load_starts(const SpGroups* gp, int64_t* S) {
    for (int j = threadIdx.x; j <= kMaxGroups; j += blockDim.x) S[j] = j <= gp->G ? gp->gstart[j] : INT64_MAX;
}

// ---------------------------------------------------------------------------------------------
// Java Int2IntHash family (hash/BJHash.java:10-20, Mix64Hash.java:10-21, TWHash.java:10-20,
// BKDRHash.java:13-21), int32 wrap-around arithmetic; code % size folded non-negative.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sar(uint32_t c, int s) { return (uint32_t)((int32_t)c >> s); }

// BKDRHash's digit loop over a non-negative key, three decimal digits per step: a full chunk r
// (digits d0 d1 d2, d0 the lowest) advances the code to code * s^3 + (d0 s + d1) s + d2, the last
// chunk by as many digits as it has.  Every product but code * s^k has both operands below 2^24
// (r < 1000, d < 10, s <= 13131, k / 1000 < 2^23, (d0 s + d1) s < 2^31), so it is a full-rate
// 24-bit multiply instead of a quarter-rate 32-bit one; k / 1000 as the truncated double product
// with RN(1/1000), which lies above 1/1000: never below the quotient, and below the next integer
// by more than the product's rounding for every 32-bit k.  Checked exhaustively against the digit
// loop on the host (tests/test_hash_arith.py).
__device__ __forceinline__ uint32_t div1000(uint32_t k) { return (uint32_t)((double)k * 0.001); }
__device__ __forceinline__ uint32_t bkdr3(uint32_t seed, uint32_t r) {  // r < 1000: d0 s^2 + d1 s + d2
    const uint32_t t = __umul24(r, 205u) >> 11, h = __umul24(r, 41u) >> 12;  // r / 10, r / 100
    return __umul24(__umul24(r - 10u * t, seed) + (t - 10u * h), seed) + h;
}
__device__ __forceinline__ uint32_t bkdr_chunks(uint32_t seed, uint32_t k) {
    const uint32_t s2 = seed * seed, s3 = s2 * seed;
    uint32_t c = 0;
    while (k >= 1000u) {
        const uint32_t q = div1000(k);
        c = c * s3 + bkdr3(seed, k - __umul24(q, 1000u));
        k = q;
    }
    if (k >= 100u) {
        c = c * s3 + bkdr3(seed, k);
    } else if (k >= 10u) {
        const uint32_t t = __umul24(k, 205u) >> 11;
        c = c * s2 + __umul24(k - 10u * t, seed) + t;
    } else if (k) {
        c = c * seed + k;
    }
    return c;
}

__device__ __forceinline__ uint32_t java_hash_mix(int id, int32_t key) {
    uint32_t c = (uint32_t)key;
    if (id == 0) {
        c = (c + 0x7ed55d16u) + (c << 12);
        c = (c ^ 0xc761c23cu) ^ sar(c, 19);
        c = (c + 0x165667b1u) + (c << 5);
        c = (c + 0xd3a2646cu) ^ (c << 9);
        c = (c + 0xfd7046c5u) + (c << 3);
        c = (c ^ 0xb55a4f09u) ^ sar(c, 16);
    } else if (id == 1) {
        c = ~c + (c << 21);
        c = c ^ sar(c, 24);
        c = (c + (c << 3)) + (c << 8);
        c = c ^ sar(c, 14);
        c = (c + (c << 2)) + (c << 4);
        c = c ^ sar(c, 28);
        c = c + (c << 31);
    } else if (id == 2) {
        c = ~c + (c << 15);
        c = c ^ sar(c, 12);
        c = c + (c << 2);
        c = c ^ sar(c, 4);
        c = c * 2057u;
        c = c ^ sar(c, 16);
    } else {
        const uint32_t seed = id == 3 ? 31u : id == 4 ? 131u : id == 5 ? 267u : id == 6 ? 1313u : 13131u;
        c = 0;
        if (key >= 0) {  // every valid key: Java's int % and / are the unsigned ones
            c = bkdr_chunks(seed, (uint32_t)key);
        } else {
            int32_t k = key;
            while (k != 0) {
                c = seed * c + (uint32_t)(k % 10);
                k /= 10;
            }
        }
    }
    return c;
}
__device__ __forceinline__ int32_t java_hash(int id, int32_t key, int32_t size) {
    const int32_t r = (int32_t)java_hash_mix(id, key) % size;
    return r >= 0 ? r : r + size;
}
// The same with `% size` folded non-negative as r - floor(r * (1/size)) * size: the double
// product is within one of the true quotient and one correction step makes the result exact (an
// integer division by a run-time divisor is a long instruction sequence on the GPU).
// For size <= 2^30, in 32 bits: the quotient is off by at most one, so the uncorrected remainder
// lies in [-size, 2 size) (tests/test_hash_arith.py).
__device__ __forceinline__ int32_t java_hash_fm32(int id, int32_t key, int32_t size, double inv) {
    const int32_t r = (int32_t)java_hash_mix(id, key);
    const int32_t q = (int32_t)floor((double)r * inv);
    int32_t m = (int32_t)((uint32_t)r - (uint32_t)q * (uint32_t)size);
    if (m < 0) m += size;
    else if (m >= size) m -= size;
    return m;
}
__device__ __forceinline__ int32_t java_hash_fm(int id, int32_t key, int32_t size, double inv) {
    if (size <= 0x40000000) return java_hash_fm32(id, key, size, inv);
    const int32_t r = (int32_t)java_hash_mix(id, key);
    const int64_t q = (int64_t)floor((double)r * inv);
    int64_t m = (int64_t)r - q * (int64_t)size;
    if (m < 0) m += size;
    else if (m >= size) m -= size;
    return (int32_t)m;
}

// 4 elements' cells of one MinMax row with the hash fixed at compile time, as 32-bit offsets
// (row0: the row's first cell, relative): for a k_dec_keys tile inside one group, whose lanes all
// use the same hash id, java_hash_mix folds to the one hash instead of computing every variant.
// SKML_DEC_INTMOD (A/B builds): 1 = the modulus by a 32-bit magic-number division (java_mod, as the
// encode's MinMax insert does) instead of the double-precision quotient.
#ifndef SKML_DEC_INTMOD
#define SKML_DEC_INTMOD 0
#endif
template <int ID, typename DV>
__device__ __forceinline__ void dec_row_cells(const int32_t (&key)[4], int64_t i0, int64_t n, int64_t row0,
                                              int32_t cols, double inv, const DV& dv, uint32_t (&rel)[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
#ifdef SKML_ABLATE_DEC_HASH  // timing ablation only (wrong cells): the hashes priced
        rel[j] = (uint32_t)(row0 + ((uint32_t)key[j] & 0xFFFFu));
        continue;
#endif
        // every element is hashed, those past n too (their keys are whatever the prefix left and
        // their cells lie inside the row; nothing of theirs is stored): no exec-mask branches
        // around the digit loops and the gathers
        (void)i0, (void)n;
        if constexpr (SKML_DEC_INTMOD)
            rel[j] = (uint32_t)(row0 + dv(java_hash_mix(ID, key[j])));
        else
            rel[j] = (uint32_t)(row0 + java_hash_fm32(ID, key[j], cols, inv));
    }
}

// |v - zero| with Java int wrap (MinMaxSketch.compare, MinMaxSketch.java:80-86)
__device__ __forceinline__ int32_t mm_dist(int32_t v, int32_t zero) {
    const int32_t d = (int32_t)((uint32_t)v - (uint32_t)zero);
    return d < 0 ? (int32_t)(0u - (uint32_t)d) : d;
}

// =============================================================================================
// Compaction (decoupled look-back)
// =============================================================================================
// Each workgroup compacts one tile of values, all of it held in registers (fp32: 16,384 values,
// 16 float4 per thread, slab j of the tile = float4 j * 256 + t; fp64: 8,192 values, two double2
// per slab), so a tile keeps 64 KiB of loads in flight and takes one look-back.  Ranks follow index order: slab by slab, and within a slab
// by float4, from wave-level scans of 16-bit packed per-slab counts plus the waves' slab totals.
constexpr int kCompactStage = 4096;  // kept elements staged in LDS; denser tiles store directly

// Element traits: fp32 tiles of 16,384 (64 per thread, 16 float4 slabs), fp64 tiles of 8,192 (32
// per thread, 8 slabs of two double2): 64 KiB of loads in flight per tile either way.
template <typename T> struct CompactT;
template <> struct CompactT<float> {
    static constexpr int kTile = kCompactTile;
    typedef float v2 __attribute__((ext_vector_type(4)));  // one slab = one 16-byte load
    // Maths.scala:8 EPS: |x| > 1e-8 in double; for a float x that is |x| > RD_f32(1e-8) on the
    // magnitude bits, NaN excluded (abs bits above +inf's).
    static __device__ __forceinline__ bool keep(float v) {
        const uint32_t a = __float_as_uint(v) & 0x7FFFFFFFu;
        return a > kEpsBelowBits && a <= 0x7F800000u;
    }
};
template <> struct CompactT<double> {
    static constexpr int kTile = kCompactTile / 2;
    typedef double v2 __attribute__((ext_vector_type(2)));  // one slab = two 16-byte loads
    static __device__ __forceinline__ bool keep(double v) {  // |x| > 1e-8, NaN excluded
        const uint64_t a = (uint64_t)__double_as_longlong(v) & 0x7FFFFFFFFFFFFFFFull;
        return a > 0x3E45798EE2308C3Aull && a <= 0x7FF0000000000000ull;
    }
};
template <typename T>
constexpr int compact_tile() { return CompactT<T>::kTile; }

template <typename T>
__global__ __launch_bounds__(kSpThreads) void k_compact(const T* __restrict__ x, int64_t dim,
                                                        int32_t* __restrict__ keys, T* __restrict__ vals,
                                                        uint64_t* status, unsigned* ticket, int64_t ntiles,
                                                        int64_t* nnz_out) {
    constexpr int kTile = CompactT<T>::kTile;
    constexpr int kSlabs = kTile / (4 * kSpThreads);  // 4 elements per thread per slab
    static_assert(kSlabs % 4 == 0 && kSlabs <= 16, "16-bit slab counts, 4 per u64, 64-bit keep mask");
    typedef typename CompactT<T>::v2 vec;
    __shared__ uint32_t wtot[kSpThreads / 64][kSlabs];  // per-wave kept counts of each slab
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_excl;
    __shared__ int32_t stage_k[kCompactStage];
    __shared__ T stage_v[kCompactStage];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t base = tile * kTile;
    const int64_t lim = dim - base;
    T f[kSlabs][4];  // slab j of the tile = elements 4 * (j * 256 + t) .. + 3
    if (lim >= kTile && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        const vec* src = reinterpret_cast<const vec*>(x + base);
        constexpr int kVec = 4 / (16 / (int)sizeof(T) >= 4 ? 4 : 16 / (int)sizeof(T));  // loads per slab
        constexpr int kPer = 4 / kVec;                                                 // elements per load
#pragma unroll
        for (int j = 0; j < kSlabs; j++)
#pragma unroll
            for (int u = 0; u < kVec; u++) {
                const vec v = __builtin_nontemporal_load(src + ((int64_t)j * kSpThreads + t) * kVec + u);
#pragma unroll
                for (int e = 0; e < kPer; e++) f[j][u * kPer + e] = v[e];
            }
    } else {
#pragma unroll
        for (int j = 0; j < kSlabs; j++) {
            const int64_t e0 = 4 * ((int64_t)j * kSpThreads + t);
#pragma unroll
            for (int e = 0; e < 4; e++) f[j][e] = e0 + e < lim ? x[base + e0 + e] : (T)0;
        }
    }
    uint64_t keep = 0;
#pragma unroll
    for (int j = 0; j < kSlabs; j++)
#pragma unroll
        for (int e = 0; e < 4; e++) keep |= CompactT<T>::keep(f[j][e]) ? (1ull << (4 * j + e)) : 0ull;
    // wave-inclusive scans of the per-slab counts, four 16-bit lanes per u64
    uint64_t P[kSlabs / 4];
#pragma unroll
    for (int k = 0; k < kSlabs / 4; k++) {
        uint64_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) v |= (uint64_t)__popcll((keep >> (16 * k + 4 * q)) & 15ull) << (16 * q);
        P[k] = v;
    }
    uint64_t own[kSlabs / 4];
#pragma unroll
    for (int k = 0; k < kSlabs / 4; k++) own[k] = P[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
        for (int k = 0; k < kSlabs / 4; k++) {
            const uint64_t y = __shfl_up(P[k], off, 64);
            if (lane >= off) P[k] += y;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int j = 0; j < kSlabs; j++) wtot[w][j] = (uint32_t)(P[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
    }
    __syncthreads();
    // slab totals, this wave's offset inside each slab, and the tile total
    uint32_t slab_pre[kSlabs];
    uint32_t tile_total = 0;
#pragma unroll
    for (int j = 0; j < kSlabs; j++) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int u = 0; u < kSpThreads / 64; u++) {
            const uint32_t c = wtot[u][j];
            before += u < w ? c : 0u;
            tot += c;
        }
        slab_pre[j] = tile_total + before;
        tile_total += tot;
    }
    if (t < 64) {  // wave 0: publish the aggregate, then look back
        uint64_t excl = 0;
        if (tile == 0) {
            if (lane == 0) st_status(&status[0], kStPre | tile_total);
        } else {
            if (lane == 0) st_status(&status[tile], kStAgg | tile_total);
            excl = lookback_excl<sizeof(T) == 8 ? 1 : 4>(status, tile, lane);  // rows the register budget allows
            if (lane == 0) st_status(&status[tile], kStPre | (excl + tile_total));
        }
        if (lane == 0) {
            s_excl = excl;
            if (tile == ntiles - 1) put_count(nnz_out, (int64_t)(excl + tile_total));
        }
    }
    __syncthreads();
    const int64_t out0 = (int64_t)s_excl;
    if (tile_total <= (uint32_t)kCompactStage) {  // the tile's output through LDS: coalesced stores
#pragma unroll
        for (int j = 0; j < kSlabs; j++) {
            const uint32_t incl = (uint32_t)(P[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
            const uint32_t mine = (uint32_t)(own[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
            uint32_t pos = slab_pre[j] + incl - mine;
            const int32_t e0 = (int32_t)(base + 4 * ((int64_t)j * kSpThreads + t));
#pragma unroll
            for (int e = 0; e < 4; e++)
                if ((keep >> (4 * j + e)) & 1ull) {
                    stage_k[pos] = e0 + e;
                    stage_v[pos] = f[j][e];
                    pos++;
                }
        }
        __syncthreads();
        for (uint32_t q = t; q < tile_total; q += kSpThreads) {
            keys[out0 + q] = stage_k[q];
            vals[out0 + q] = stage_v[q];
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < kSlabs; j++) {
        const uint64_t incl = (P[j >> 2] >> (16 * (j & 3))) & 0xFFFFull;
        const uint64_t mine = (own[j >> 2] >> (16 * (j & 3))) & 0xFFFFull;
        int64_t pos = out0 + slab_pre[j] + (int64_t)(incl - mine);
        const int32_t e0 = (int32_t)(base + 4 * ((int64_t)j * kSpThreads + t));
#pragma unroll
        for (int e = 0; e < 4; e++)
            if ((keep >> (4 * j + e)) & 1ull) {
                keys[pos] = e0 + e;
                vals[pos] = f[j][e];
                pos++;
            }
    }
}

// fp32 compaction over big tiles: kCbSub sub-tiles of 8,192 values per workgroup, processed in
// turn (the next sub-tile's 32 KiB of loads in flight while the current one is ranked), their kept
// values and in-sub-tile offsets staged in LDS; one decoupled look-back per 65,536 values (a
// quarter of k_compact's: its prefix frontier, 64 tiles per look-back step, no longer trails the
// tiles' arrival), then coalesced stores.  A tile keeping more than kCbCap values re-reads its
// input and stores directly.
constexpr int kCbSlabs = 8;                              // float4 slabs per thread per sub-tile
constexpr int kCbSubElems = kCbSlabs * 4 * kSpThreads;  // 8,192 values
constexpr int kCbSub = 8, kCbTile = kCbSub * kCbSubElems, kCbCap = 8192;
static_assert(kCbSlabs % 4 == 0, "16-bit slab counts, 4 per u64");

// keep mask and in-sub-tile ranks of one sub-tile held as f[kCbSlabs][4] (slab j = float4 j * 256 + t)
struct CbRanks {
    uint32_t keep;
    uint32_t slab_pre[kCbSlabs];  // exclusive start of this thread's kept values of slab j in the sub-tile
    uint32_t total;               // kept values in the sub-tile
};
__device__ __forceinline__ void cb_rank(const float (&f)[kCbSlabs][4], uint32_t (*wtot)[kCbSlabs], CbRanks& R) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < kCbSlabs; j++)
#pragma unroll
        for (int e = 0; e < 4; e++) keep |= CompactT<float>::keep(f[j][e]) ? (1u << (4 * j + e)) : 0u;
    constexpr int kW = kCbSlabs / 4;
    uint64_t P[kW], own[kW];
#pragma unroll
    for (int k = 0; k < kW; k++) {
        uint64_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) v |= (uint64_t)__popc((keep >> (16 * k + 4 * q)) & 15u) << (16 * q);
        P[k] = own[k] = v;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
        for (int k = 0; k < kW; k++) {
            const uint64_t y = __shfl_up(P[k], off, 64);
            if (lane >= off) P[k] += y;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int j = 0; j < kCbSlabs; j++) wtot[w][j] = (uint32_t)(P[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
    }
    __syncthreads();
    uint32_t total = 0;
#pragma unroll
    for (int j = 0; j < kCbSlabs; j++) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int u = 0; u < kSpThreads / 64; u++) {
            const uint32_t c = wtot[u][j];
            before += u < w ? c : 0u;
            tot += c;
        }
        const uint32_t incl = (uint32_t)(P[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
        const uint32_t mine = (uint32_t)(own[j >> 2] >> (16 * (j & 3))) & 0xFFFFu;
        R.slab_pre[j] = total + before + incl - mine;
        total += tot;
    }
    R.keep = keep;
    R.total = total;
    __syncthreads();  // wtot is reused by the next sub-tile
}

__device__ __forceinline__ void cb_load(const float* __restrict__ x, int64_t base, int64_t dim,
                                        float (&f)[kCbSlabs][4]) {
    const int t = threadIdx.x;
    if (base + kCbSubElems <= dim) {
        typedef float vec4 __attribute__((ext_vector_type(4)));
        const vec4* src = reinterpret_cast<const vec4*>(x + base);
#pragma unroll
        for (int j = 0; j < kCbSlabs; j++) {
            const vec4 v = __builtin_nontemporal_load(src + j * kSpThreads + t);
            f[j][0] = v[0], f[j][1] = v[1], f[j][2] = v[2], f[j][3] = v[3];
        }
    } else {
#pragma unroll
        for (int j = 0; j < kCbSlabs; j++) {
            const int64_t e0 = base + 4 * ((int64_t)j * kSpThreads + t);
#pragma unroll
            for (int e = 0; e < 4; e++) f[j][e] = e0 + e < dim ? x[e0 + e] : 0.0f;
        }
    }
}

// workgroups of `kern` (`threads` each) resident at once on the device; 0 if the query fails
template <typename K>
static int resident_blocks(K kern, int threads) {
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    int r = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0) == hipSuccess)
        r = std::max(1, per_cu) * prop.multiProcessorCount;
    (void)hipGetLastError();
    return r;
}

#ifndef SKML_COMPACT_PERSIST
#define SKML_COMPACT_PERSIST 0  // 1: the persistent form (A/B builds)
#endif
// One tile per workgroup.  The persistent form (SKML_COMPACT_PERSIST 1, A/B builds) takes the next
// tile's ticket before its look-back and loads that tile's first sub-tile while its stores drain,
// with the grid at what the CUs hold at once (tickets are taken in order by running workgroups and
// a workgroup waits only on lower tickets, so the look-back always progresses); it measured 10-20
// us slower per C3 encode (profiles/ab/r06_compact_persist.txt).
__global__ __launch_bounds__(kSpThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_compact_big(const float* __restrict__ x, int64_t dim,
                                                            int32_t* __restrict__ keys, float* __restrict__ vals,
                                                            uint64_t* status, unsigned* ticket, int64_t ntiles,
                                                            int64_t* nnz_out) {
    __shared__ float st_v[kCbCap];
    __shared__ uint16_t st_k[kCbCap];  // offset inside the sub-tile (< 2^14)
    __shared__ uint32_t wtot[kSpThreads / 64][kCbSlabs];
    __shared__ uint32_t sub_pre[kCbSub + 1];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_excl;
    const int t = threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(x) & 15) != 0) __builtin_trap();  // the launcher checks alignment
    if (t == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
    __syncthreads();
    int64_t tile = s_tile;
    if (tile >= ntiles) return;  // workgroup-uniform
    float f[kCbSlabs][4], g[kCbSlabs][4];
    cb_load(x, tile * kCbTile, dim, f);
#pragma unroll 1
    while (true) {
        const int64_t base = tile * kCbTile;
        uint32_t run = 0;
#pragma unroll 1
        for (int sb = 0; sb < kCbSub; sb++) {
            float (&cur)[kCbSlabs][4] = f;
            if (sb + 1 < kCbSub) cb_load(x, base + (int64_t)(sb + 1) * kCbSubElems, dim, g);
            CbRanks R;
            cb_rank(cur, wtot, R);
            if (t == 0) sub_pre[sb] = run;
            if (run + R.total <= (uint32_t)kCbCap) {
#pragma unroll
                for (int j = 0; j < kCbSlabs; j++) {
                    uint32_t pos = run + R.slab_pre[j];
                    const int off0 = 4 * (j * kSpThreads + t);
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if ((R.keep >> (4 * j + e)) & 1u) {
                            st_v[pos] = cur[j][e];
                            st_k[pos] = (uint16_t)(off0 + e);
                            pos++;
                        }
                }
            }
            run += R.total;
#pragma unroll
            for (int j = 0; j < kCbSlabs; j++)
#pragma unroll
                for (int e = 0; e < 4; e++) f[j][e] = g[j][e];
        }
        const uint32_t tile_total = run;
        // every thread read s_tile before cb_rank's barriers: the next ticket may land there now
        if (SKML_COMPACT_PERSIST && t == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
        if (t < 64) {  // wave 0: publish the aggregate, then look back
            const int lane = t;
            uint64_t excl = 0;
            if (tile == 0) {
                if (lane == 0) st_status(&status[0], kStPre | tile_total);
            } else {
                if (lane == 0) st_status(&status[tile], kStAgg | tile_total);
                excl = lookback_excl<SKML_LOOKBACK_ROWS>(status, tile, lane);
                if (lane == 0) st_status(&status[tile], kStPre | (excl + tile_total));
            }
            if (lane == 0) {
                s_excl = excl;
                sub_pre[kCbSub] = tile_total;
                if (tile == ntiles - 1) put_count(nnz_out, (int64_t)(excl + tile_total));
            }
        }
        __syncthreads();
        const int64_t out0 = (int64_t)s_excl;
        const int64_t next = SKML_COMPACT_PERSIST ? s_tile : ntiles;
        if (tile_total <= (uint32_t)kCbCap) {
            if (next < ntiles) cb_load(x, next * kCbTile, dim, f);  // in flight while this tile's stores drain
            for (uint32_t q = t; q < tile_total; q += kSpThreads) {
                int sb = 0;
#pragma unroll
                for (int k = 1; k < kCbSub; k++) sb += q >= sub_pre[k] ? 1 : 0;
                keys[out0 + q] = (int32_t)(base + (int64_t)sb * kCbSubElems + st_k[q]);
                vals[out0 + q] = st_v[q];
            }
        } else {
            // more kept values than the stage holds: read each sub-tile again and store directly
            for (int sb = 0; sb < kCbSub; sb++) {
                const int64_t sbase = base + (int64_t)sb * kCbSubElems;
                cb_load(x, sbase, dim, f);
                CbRanks R;
                cb_rank(f, wtot, R);
#pragma unroll
                for (int j = 0; j < kCbSlabs; j++) {
                    int64_t pos = out0 + sub_pre[sb] + R.slab_pre[j];
                    const int64_t e0 = sbase + 4 * ((int64_t)j * kSpThreads + t);
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if ((R.keep >> (4 * j + e)) & 1u) {
                            keys[pos] = (int32_t)(e0 + e);
                            vals[pos] = f[j][e];
                            pos++;
                        }
                }
            }
            if (next < ntiles) cb_load(x, next * kCbTile, dim, f);
        }
        if (next >= ntiles) break;
        __syncthreads();  // the stage, sub_pre and s_excl are the next tile's
        tile = next;
    }
}

template <typename T>
hipError_t launch_compact_t(hipStream_t st, const T* x, int64_t dim, int32_t* keys, T* vals, uint64_t* status,
                            unsigned* ticket, int64_t* nnz_out) {
    const int64_t tiles = sp_tiles(dim, compact_tile<T>());
    if (tiles <= 0) return hipMemsetAsync(nnz_out, 0, sizeof(int64_t), st);
    hipLaunchKernelGGL(k_compact<T>, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, x, dim, keys, vals, status,
                       ticket, tiles, nnz_out);
    return hipGetLastError();
}
hipError_t launch_compact(hipStream_t st, const float* x, int64_t dim, int32_t* keys, float* vals,
                          uint64_t* status, unsigned* ticket, int64_t* nnz_out) {
    if ((reinterpret_cast<uintptr_t>(x) & 15) != 0 || dim < kCbTile)  // small or unaligned: the one-tile kernel
        return launch_compact_t<float>(st, x, dim, keys, vals, status, ticket, nnz_out);
    const int64_t tiles = sp_tiles(dim, kCbTile);
    int64_t grid = tiles;
    if (SKML_COMPACT_PERSIST) {  // the workgroups the CUs hold at once
        static const int resident = resident_blocks(k_compact_big, kSpThreads);
        if (resident > 0) grid = std::min<int64_t>(tiles, resident);
    }
    hipLaunchKernelGGL(k_compact_big, dim3((unsigned)grid), dim3(kSpThreads), 0, st, x, dim, keys, vals, status,
                       ticket, tiles, nnz_out);
    return hipGetLastError();
}
hipError_t launch_compact64(hipStream_t st, const double* x, int64_t dim, int32_t* keys, double* vals,
                            uint64_t* status, unsigned* ticket, int64_t* nnz_out) {
    return launch_compact_t<double>(st, x, dim, keys, vals, status, ticket, nnz_out);
}

// =============================================================================================
// Column scan of [tiles][K] u64 tile sums (one workgroup per column)
// =============================================================================================
// One workgroup of 1,024 threads per column, 8K entries per pass.  A 1,024-thread workgroup needs
// 16 wave slots of one CU at once, and in Gradient.sum it waits for a CU beside the other
// restore's k_dec_keys (profiles/r06c_aggregate_timeline.txt); 256-thread one-pass scans remove
// that wait but ran slower end to end (restore +13 us, Gradient.sum +80 us: the two restores'
// key queries then overlap each other, profiles/ab/r06_scan_threads.txt).
#ifndef SKML_SCAN_THREADS
#define SKML_SCAN_THREADS 1024  // A/B builds: 256 (with SKML_SCAN_PER 64)
#endif
#ifndef SKML_SCAN_PER
#define SKML_SCAN_PER 8
#endif
constexpr int kScanThreads = SKML_SCAN_THREADS, kScanPer = SKML_SCAN_PER;
static_assert(kScanPer % 2 == 0, "16-byte loads of two entries");
// Entry (i, k) at sums[k * ld + i * es]: [tiles][K] row-major (ld 1, es K) or one column of
// tiles + 1 entries per k (ld tiles + 1, es 1: contiguous column reads).
// THREADS x PER entries per pass (kScanThreads x kScanPer by default; the sparse encode's side
// chain takes 256-thread workgroups, launch_scan_cols_small)
template <int THREADS = kScanThreads, int PER = kScanPer>
__global__ __launch_bounds__(THREADS) void k_scan_cols(uint64_t* sums, int64_t tiles, int64_t ld, int64_t es) {
    constexpr int kScanThreads = THREADS, kScanPer = PER;
    __shared__ uint64_t sh[kScanThreads / 64];
    const int k = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t carry = 0;
    for (int64_t c0 = 0; c0 < tiles; c0 += kScanThreads * kScanPer) {
        uint64_t loc[kScanPer], s = 0;
        const int64_t i0 = c0 + t * kScanPer;
        if (es == 1 && i0 + kScanPer <= tiles && ((k * ld + i0) & 1) == 0) {  // 16-byte loads
            typedef uint64_t u64x2_t __attribute__((ext_vector_type(2)));
            const u64x2_t* src = reinterpret_cast<const u64x2_t*>(sums + k * ld + i0);
#pragma unroll
            for (int j = 0; j < kScanPer / 2; j++) {
                const u64x2_t v = src[j];
                loc[2 * j] = v.x;
                loc[2 * j + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kScanPer; j++) {
                const int64_t i = i0 + j;
                loc[j] = i < tiles ? sums[k * ld + i * es] : 0;
            }
        }
#pragma unroll
        for (int j = 0; j < kScanPer; j++) s += loc[j];
        const uint64_t inc = wave_incl_u64(s, lane);
        if (lane == 63) sh[w] = inc;
        __syncthreads();
        uint64_t before = 0, tot = 0;
#pragma unroll
        for (int j = 0; j < kScanThreads / 64; j++) {
            const uint64_t x = sh[j];
            before += j < w ? x : 0;
            tot += x;
        }
        __syncthreads();
        uint64_t run = carry + before + inc - s;
#pragma unroll
        for (int j = 0; j < kScanPer; j++) {
            const int64_t i = c0 + t * kScanPer + j;
            if (i < tiles) sums[k * ld + i * es] = run;
            run += loc[j];
        }
        carry += tot;
    }
    if (t == 0) sums[k * ld + tiles * es] = carry;
}

hipError_t launch_scan_cols(hipStream_t st, uint64_t* sums, int64_t tiles, int K) {
    hipLaunchKernelGGL(k_scan_cols<>, dim3(K), dim3(kScanThreads), 0, st, sums, tiles, (int64_t)1, (int64_t)K);
    return hipGetLastError();
}
hipError_t launch_scan_cols_major(hipStream_t st, uint64_t* sums, int64_t tiles, int K) {
    hipLaunchKernelGGL(k_scan_cols<>, dim3(K), dim3(kScanThreads), 0, st, sums, tiles, tiles + 1, (int64_t)1);
    return hipGetLastError();
}
// The same scan on 256-thread workgroups: in the sparse encode's side chain a 1,024-thread
// workgroup waits for a whole CU's wave slots beside the MinMax scatter (4-5 us alone, 57-70 us
// there), which pushed the DeltaAdaptive writer onto the bucket minima.
hipError_t launch_scan_cols_small(hipStream_t st, uint64_t* sums, int64_t tiles, int K) {
    hipLaunchKernelGGL((k_scan_cols<256, 32>), dim3(K), dim3(256), 0, st, sums, tiles, (int64_t)1, (int64_t)K);
    return hipGetLastError();
}

// =============================================================================================
// Partition by group (stable)
// =============================================================================================
// Up to kFewGroups groups (the default is 8): the edges sit in registers, the group of a bin is a
// sum of compares, and the per-group counts are 8-bit fields of one u64 per lane (at most 8
// elements per lane and step), reduced across the wave as two u64 of 16-bit fields.
constexpr int kFewGroups = 8;
struct FewEdges {
    int32_t e[kFewGroups - 1];  // edges[0 .. G-2], INT32_MAX beyond (edges[G-1] = binNum is above every bin)
};
__device__ __forceinline__ FewEdges few_edges(const SpGroups* gp, int G) {
    FewEdges f;
#pragma unroll
    for (int j = 0; j < kFewGroups - 1; j++) f.e[j] = j < G - 1 ? gp->edges[j] : INT32_MAX;
    return f;
}
__device__ __forceinline__ int few_group(const FewEdges& f, int32_t bin) {
    int g = 0;
#pragma unroll
    for (int j = 0; j < kFewGroups - 1; j++) g += f.e[j] <= bin ? 1 : 0;
    return g;
}
// wave sums of the 8-bit fields of acc, as 16-bit fields: groups 0,2,4,6 in lo and 1,3,5,7 in hi
__device__ __forceinline__ void few_wave_sum(uint64_t acc, uint64_t& lo, uint64_t& hi) {
    lo = acc & 0x00FF00FF00FF00FFull;
    hi = (acc >> 8) & 0x00FF00FF00FF00FFull;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        lo += __shfl_xor(lo, off, 64);
        hi += __shfl_xor(hi, off, 64);
    }
}
__device__ __forceinline__ uint32_t few_field(uint64_t lo, uint64_t hi, int g) {
    return (uint32_t)(((g & 1) ? hi : lo) >> (16 * (g >> 1))) & 0xFFFFu;
}

// kPartTiles consecutive tiles per workgroup, their code loads issued together (one tile per
// workgroup left the 2 KB-per-workgroup pass bound by workgroup dispatch: 26 us at C3).
constexpr int kPartTiles = 4;
__global__ __launch_bounds__(kSpThreads) void k_part_count(const uint8_t* __restrict__ qpayload, int64_t n,
                                                           const SpGroups* __restrict__ gp,
                                                           uint64_t* __restrict__ tile_counts,
                                                           uint32_t* __restrict__ z32, int64_t n32,
                                                           uint64_t* __restrict__ z64, int64_t n64) {
    for (int64_t z = (int64_t)blockIdx.x * kSpThreads + threadIdx.x, step = (int64_t)gridDim.x * kSpThreads;
         z < n32 || z < n64; z += step) {
        if (z < n32) z32[z] = 0;
        if (z < n64) z64[z] = 0;
    }
    if (gp->status) return;
    __shared__ int32_t E[kMaxGroups];
    __shared__ uint32_t cnt[kPartTiles][kMaxGroups];
    __shared__ uint64_t wsum[kPartTiles][kSpThreads / 64][2];
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(qpayload);
    const uint8_t* codes = qpayload + h->codes_offset;
    const int bits = h->code_bits, G = gp->G;
    const int64_t tiles = (n + kSpTile - 1) / kSpTile;
    const int64_t tile0 = (int64_t)blockIdx.x * kPartTiles;
    const int t = threadIdx.x;
    if (G <= kFewGroups) {  // 8 consecutive elements per lane, counted in registers
        static_assert(kSpTile == 8 * kSpThreads, "one 8-element run per lane");
        const FewEdges fe = few_edges(gp, G);
        const bool fast = bits == 8 && ((reinterpret_cast<uintptr_t>(codes) & 7) == 0);
        uint64_t w8[kPartTiles];
#pragma unroll
        for (int k = 0; k < kPartTiles; k++) {
            const int64_t i0 = (tile0 + k) * kSpTile + 8 * t;
            w8[k] = fast && i0 + 8 <= n ? *reinterpret_cast<const uint64_t*>(codes + i0) : 0ull;
        }
#pragma unroll
        for (int k = 0; k < kPartTiles; k++) {
            const int64_t i0 = (tile0 + k) * kSpTile + 8 * t;
            uint64_t acc = 0;
            if (fast && i0 + 8 <= n) {
#pragma unroll
                for (int e = 0; e < 8; e++) acc += 1ull << (8 * few_group(fe, (int32_t)((w8[k] >> (8 * e)) & 255u)));
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++)
                    if (i0 + e < n) acc += 1ull << (8 * few_group(fe, code_at(codes, i0 + e, bits)));
            }
            uint64_t lo, hi;
            few_wave_sum(acc, lo, hi);
            if ((t & 63) == 0) {
                wsum[k][t >> 6][0] = lo;
                wsum[k][t >> 6][1] = hi;
            }
        }
        __syncthreads();
        if (t < kPartTiles * G) {
            const int k = t / G, g = t - k * G;
            if (tile0 + k < tiles) {
                uint32_t c = 0;
#pragma unroll
                for (int w = 0; w < kSpThreads / 64; w++) c += few_field(wsum[k][w][0], wsum[k][w][1], g);
                tile_counts[(int64_t)g * (tiles + 1) + tile0 + k] = c;
            }
        }
        return;
    }
    load_edges(gp, E);
    for (int j = t; j < kPartTiles * kMaxGroups; j += kSpThreads) cnt[j / kMaxGroups][j % kMaxGroups] = 0;
    __syncthreads();
    for (int k = 0; k < kPartTiles; k++)
        for (int j = t; j < kSpTile; j += kSpThreads) {
            const int64_t i = (tile0 + k) * kSpTile + j;
            if (i < n) atomicAdd(&cnt[k][group_of_bin(E, code_at(codes, i, bits))], 1u);
        }
    __syncthreads();
    for (int j = t; j < kPartTiles * G; j += kSpThreads) {
        const int k = j / G, g = j - k * G;
        if (tile0 + k < tiles) tile_counts[(int64_t)g * (tiles + 1) + tile0 + k] = cnt[k][g];
    }
}

hipError_t launch_part_count(hipStream_t st, const void* qpayload, int64_t n, const SpGroups* gp,
                             uint64_t* tile_counts, uint32_t* z32, int64_t n32, uint64_t* z64, int64_t n64) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) {
        if (n32 > 0) {
            hipError_t e = hipMemsetAsync(z32, 0, sizeof(uint32_t) * (size_t)n32, st);
            if (e != hipSuccess) return e;
        }
        return n64 > 0 ? hipMemsetAsync(z64, 0, sizeof(uint64_t) * (size_t)n64, st) : hipSuccess;
    }
    hipLaunchKernelGGL(k_part_count, dim3((unsigned)((tiles + kPartTiles - 1) / kPartTiles)), dim3(kSpThreads), 0, st,
                       reinterpret_cast<const uint8_t*>(qpayload), n, gp, tile_counts, z32, n32, z64, n64);
    return hipGetLastError();
}

// Wave w of the tile owns elements [w*512, (w+1)*512), 64 per step in order; lanes with the same
// group are ranked by lane (peer mask from log2(G) ballots), so the scatter is stable.  The tile
// is first laid out in group order in LDS, then each group's run is stored with consecutive lanes
// on consecutive output indices (direct per-lane stores split every step into G short segments).
__global__ __launch_bounds__(kSpThreads) void k_part_scatter(const int32_t* __restrict__ keys,
                                                             const uint8_t* __restrict__ qpayload, int64_t n,
                                                             const SpGroups* __restrict__ gp,
                                                             const uint64_t* __restrict__ tile_base,
                                                             int32_t* __restrict__ gkeys, uint16_t* __restrict__ gbins,
                                                             int runs) {
    if (gp->status) return;
    constexpr int kWaves = kSpThreads / 64, kSteps = kSpTile / kSpThreads;
    __shared__ int32_t E[kMaxGroups];
    __shared__ int64_t wb[kWaves][kMaxGroups];  // counts, then running LDS slot per (wave, group)
    __shared__ int64_t gdst[kMaxGroups];        // output index of a group's slot 0 in the tile
    __shared__ int32_t sk[kSpTile], sb[kSpTile];
    __shared__ uint8_t sg[kSpTile];
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(qpayload);
    const uint8_t* codes = qpayload + h->codes_offset;
    const int bits = h->code_bits, G = gp->G;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const bool few = G <= kFewGroups;
    // the output base of group t's run in this tile, read before the counting (no round trip later)
    int64_t gbase = 0;
    if (t < G) gbase = gp->gstart[t] + (int64_t)tile_base[(int64_t)t * ((int64_t)gridDim.x + 1) + blockIdx.x];
    if (few && runs) {
        // Thread t owns the tile's elements [8t, 8t + 8): one 32-byte key load and one 8-byte code
        // load per thread.  Stable ranks without ballots: the thread's per-group counts packed as
        // 16-bit fields (groups 0,2,4,6 in lo, 1,3,5,7 in hi), a wave scan of the packed words,
        // the waves' totals through LDS.
        const FewEdges fe = few_edges(gp, G);
        const int64_t i0 = (int64_t)blockIdx.x * kSpTile + 8 * t;
        int32_t kk[8], bb[8], gg[8];
        const bool full = i0 + 8 <= n;
        if (full && (reinterpret_cast<uintptr_t>(keys + i0) & 15) == 0) {
            const int4 a = *reinterpret_cast<const int4*>(keys + i0), b = *reinterpret_cast<const int4*>(keys + i0 + 4);
            kk[0] = a.x, kk[1] = a.y, kk[2] = a.z, kk[3] = a.w, kk[4] = b.x, kk[5] = b.y, kk[6] = b.z, kk[7] = b.w;
        } else {
#pragma unroll
            for (int s = 0; s < 8; s++) kk[s] = i0 + s < n ? keys[i0 + s] : 0;
        }
        if (full && bits == 8 && (reinterpret_cast<uintptr_t>(codes + i0) & 7) == 0) {
            const uint64_t w8 = *reinterpret_cast<const uint64_t*>(codes + i0);
#pragma unroll
            for (int s = 0; s < 8; s++) bb[s] = (int32_t)((w8 >> (8 * s)) & 255u);
        } else {
#pragma unroll
            for (int s = 0; s < 8; s++) bb[s] = i0 + s < n ? code_at(codes, i0 + s, bits) : 0;
        }
        uint64_t lo = 0, hi = 0;  // this thread's per-group counts
#pragma unroll
        for (int s = 0; s < 8; s++) {
            gg[s] = i0 + s < n ? few_group(fe, bb[s]) : -1;
            if (gg[s] >= 0) {
                const uint64_t one = 1ull << (16 * (gg[s] >> 1));
                if (gg[s] & 1) hi += one;
                else lo += one;
            }
        }
        uint64_t li = lo, hi_i = hi;  // inclusive wave scans
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t yl = __shfl_up(li, off, 64), yh = __shfl_up(hi_i, off, 64);
            if (lane >= off) {
                li += yl;
                hi_i += yh;
            }
        }
        __shared__ uint64_t wt[kWaves][2];
        __shared__ int32_t wbase[kWaves][kFewGroups];  // LDS slot of (wave, group)'s first element
        if (lane == 63) {
            wt[w][0] = li;
            wt[w][1] = hi_i;
        }
        __syncthreads();
        if (t < 64) {  // lane g < G: the tile's group g totals, the LDS layout in group order
            uint32_t c = 0;
            if (lane < G)
                for (int j = 0; j < kWaves; j++) c += few_field(wt[j][0], wt[j][1], lane);
            uint32_t x = c;  // inclusive scan over the groups
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            if (lane < G) {
                uint32_t run = x - c;
                gdst[lane] = gbase - (int64_t)run;
                for (int j = 0; j < kWaves; j++) {
                    wbase[j][lane] = (int32_t)run;
                    run += few_field(wt[j][0], wt[j][1], lane);
                }
            }
        }
        __syncthreads();
        const uint64_t le = li - lo, he = hi_i - hi;  // exclusive: earlier lanes of this wave
        uint64_t seen_l = 0, seen_h = 0;              // this thread's earlier elements
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const int g = gg[s];
            if (g < 0) continue;
            const int pos = wbase[w][g] + (int)few_field(le, he, g) + (int)few_field(seen_l, seen_h, g);
            sk[pos] = kk[s];
            sb[pos] = bb[s];
            sg[pos] = (uint8_t)g;
            const uint64_t one = 1ull << (16 * (g >> 1));
            if (g & 1) seen_h += one;
            else seen_l += one;
        }
        __syncthreads();
        const int tile_n = (int)std::min<int64_t>(kSpTile, n - (int64_t)blockIdx.x * kSpTile);
        for (int q = t; q < tile_n; q += kSpThreads) {
            const int64_t dst = gdst[sg[q]] + q;
            gkeys[dst] = sk[q];
            gbins[dst] = (uint16_t)sb[q];
        }
        return;
    }
    if (!few) {
        load_edges(gp, E);
        for (int j = t; j < kWaves * kMaxGroups; j += kSpThreads) wb[j / kMaxGroups][j % kMaxGroups] = 0;
        __syncthreads();
    }
    const int64_t base = (int64_t)blockIdx.x * kSpTile + (int64_t)w * (kSpTile / kWaves);
    int32_t kk[kSteps], gg[kSteps], bb[kSteps];
    if (few) {  // the wave's group counts from register fields (see k_part_count)
        static_assert(kSteps <= 8, "8-bit count fields");
        const FewEdges fe = few_edges(gp, G);
        uint64_t acc = 0;
#pragma unroll
        for (int s = 0; s < kSteps; s++) {
            const int64_t i = base + s * 64 + lane;
            gg[s] = -1;
            if (i < n) {
                kk[s] = keys[i];
                bb[s] = code_at(codes, i, bits);
                gg[s] = few_group(fe, bb[s]);
                acc += 1ull << (8 * gg[s]);
            }
        }
        uint64_t lo, hi;
        few_wave_sum(acc, lo, hi);
        if (lane < G) wb[w][lane] = few_field(lo, hi, lane);
    } else {
#pragma unroll
        for (int s = 0; s < kSteps; s++) {
            const int64_t i = base + s * 64 + lane;
            gg[s] = -1;
            if (i < n) {
                kk[s] = keys[i];
                bb[s] = code_at(codes, i, bits);
                gg[s] = group_of_bin(E, bb[s]);
                atomicAdd(reinterpret_cast<unsigned long long*>(&wb[w][gg[s]]), 1ull);
            }
        }
    }
    __syncthreads();
    // the tile in group order in LDS: wave w's elements of group g at loc[g] + (earlier waves' g)
    if (t < 64) {
        uint32_t c = 0;
        if (lane < G)
            for (int j = 0; j < kWaves; j++) c += (uint32_t)wb[j][lane];
        uint32_t x = c;  // inclusive scan over the groups
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane < G) {
            uint32_t run = x - c;
            gdst[lane] = gbase - (int64_t)run;
            for (int j = 0; j < kWaves; j++) {
                const uint32_t cj = (uint32_t)wb[j][lane];
                wb[j][lane] = run;
                run += cj;
            }
        }
    }
    __syncthreads();
    int nb = 0;
    while ((1 << nb) < G) nb++;
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int s = 0; s < kSteps; s++) {
        const bool valid = gg[s] >= 0;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < nb; b++) {
            const uint64_t bal = __ballot(valid && ((gg[s] >> b) & 1));
            peers &= ((gg[s] >> b) & 1) ? bal : ~bal;
        }
        if (valid) {
            const int pos = (int)wb[w][gg[s]] + __popcll(peers & lt);
            sk[pos] = kk[s];
            sb[pos] = bb[s];
            sg[pos] = (uint8_t)gg[s];
        }
        // every lane has read its base; the leader of each peer set advances it
        __builtin_amdgcn_wave_barrier();
        if (valid && (peers & lt) == 0) wb[w][gg[s]] += __popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // each group's run of the tile goes out with consecutive lanes on consecutive addresses
    const int tile_n = (int)std::min<int64_t>(kSpTile, n - (int64_t)blockIdx.x * kSpTile);
    for (int q = t; q < tile_n; q += kSpThreads) {
        const int64_t dst = gdst[sg[q]] + q;
        gkeys[dst] = sk[q];
        gbins[dst] = (uint16_t)sb[q];
    }
}

hipError_t launch_part_scatter(hipStream_t st, const int32_t* keys, const void* qpayload, int64_t n,
                               const SpGroups* gp, const uint64_t* tile_base, int32_t* gkeys,
                               uint16_t* gbins) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) return hipSuccess;
    const int runs = form(SKML_FORM_PART_BALLOT) == 1 ? 0 : 1;  // (0: the ballot-ranked form)
    hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, keys,
                       reinterpret_cast<const uint8_t*>(qpayload), n, gp, tile_base, gkeys, gbins, runs);
    return hipGetLastError();
}

// =============================================================================================
// Group prep: deltas / bitsNeeded / order check / MinMax insert
// =============================================================================================
// MinMaxSketch.insert, bucketed: every (element, row) pair targets table cell c; pairs are
// counted per bucket of kMmBucketCells cells, scattered into bucket order, and each bucket's minimum is
// taken with LDS atomics by one workgroup (random global 64-bit atomics were HBM-latency bound).
// Pair word: |bin - zero| [63:48], key [47:17], bin < zero [16], cell % kMmBucketCells [14:0]; its
// value with the cell bits cleared orders by (distance, key): the smaller distance wins and ties
// keep the earlier insert (keys ascend within a group).
constexpr int kMmBucketBits = SKML_MM_BUCKET_BITS;
static_assert(kMmBucketBits >= 13 && kMmBucketBits <= 15, "pair layouts hold 13..15 cell bits");
constexpr int kMmSubBits = 13;  // key-carrying pairs: u64 LDS minima over 8192-cell sub-ranges
constexpr int kMmSubCells = 1 << kMmSubBits;
constexpr int kMmBucketCells = kMmCellsPerBucket;
static_assert(kMmBucketCells == 1 << kMmBucketBits, "bucket size");
constexpr int kMmLdsBuckets = 8192;  // per-workgroup bucket tables in LDS up to this many (96 KB in the scatter)
constexpr int kMmThreads = 1024;  // count / scatter workgroups: big tiles, long per-bucket runs
#ifndef SKML_MM_BATCH
#define SKML_MM_BATCH 4
#endif
constexpr int kMmBatch = SKML_MM_BATCH;  // elements per thread in flight (count, scatter)
#ifndef SKML_BUCKET_BATCH
#define SKML_BUCKET_BATCH 8
#endif
constexpr int kBucketBatch = SKML_BUCKET_BATCH;  // pairs per thread in flight in the bucket minima

// a group's MinMaxSketch shape, staged in LDS by the count pass
// Unsigned division by a run-time d through a multiplier (the round-up method: exact for every
// 32-bit dividend); sh < 0 marks d == 1.
struct DivU32 {
    uint32_t m;
    int32_t sh;
};
__device__ __forceinline__ DivU32 divu32_make(uint32_t d) {
    if (d <= 1) return DivU32{0u, -1};
    const int l = 32 - __clz(d - 1);  // ceil(log2 d)
    return DivU32{(uint32_t)(((((uint64_t)1 << l) - d) << 32) / d + 1), l - 1};
}
__device__ __forceinline__ uint32_t divu32(uint32_t n, DivU32 v) {
    const uint32_t t = __umulhi(n, v.m);
    return (t + ((n - t) >> 1)) >> v.sh;
}
// Int2IntHash's `code %= size; return code >= 0 ? code : code + size` (the floor modulus)
__device__ __forceinline__ int32_t java_mod(int32_t code, int32_t d, DivU32 v) {
    if (v.sh < 0) return 0;
    const uint32_t u = code < 0 ? 0u - (uint32_t)code : (uint32_t)code;
    const uint32_t rem = u - divu32(u, v) * (uint32_t)d;
    return (code < 0 && rem) ? d - (int32_t)rem : (int32_t)rem;
}

// a group's MinMaxSketch shape, staged in LDS by the count pass
struct MmGroup {
    int64_t tab_off;
    double inv;
    int32_t cols;
    DivU32 div;
    int32_t hid[kMaxRows];
};
__device__ __forceinline__ void load_mm_groups(const SpGroups* gp, MmGroup* GP) {
    for (int g = threadIdx.x; g < gp->G; g += blockDim.x) {
        GP[g].tab_off = gp->tab_off[g];
        GP[g].inv = gp->inv_cols[g];
        GP[g].cols = gp->cols[g];
        GP[g].div = divu32_make((uint32_t)gp->cols[g]);
        for (int r = 0; r < kMaxRows; r++) GP[g].hid[r] = gp->hash_ids[g][r];
    }
}
// reserved pair slots of a (tile, bucket) range: whole 128-byte lines (16 wide or 32 narrow
// pairs), padding = kMmNoPair / kMmNoPair32
__device__ __forceinline__ uint32_t mm_pad(uint32_t c) { return (c + 15u) & ~15u; }
__device__ __forceinline__ uint32_t mm_pad(uint32_t c, bool narrow) {
    return narrow ? (c + 31u) & ~31u : (c + 15u) & ~15u;
}
constexpr uint64_t kMmNoPair = ~0ull;
constexpr uint32_t kMmNoPair32 = ~0u;
// Narrow pair word (SpGroups.mm_narrow): |bin - zero| [31:B+1], bin < zero [B], cell % 2^B
// [B-1:0] with B = kMmBucketBits (|bin - zero| < 65536 fits 31 - B >= 16 bits).  In a one-sided
// group the sign bit is constant, so the minimum over a cell is the nearest bin.
__device__ __forceinline__ uint32_t mm_pair32(int32_t bin, int32_t zero, int64_t cell) {
    return ((uint32_t)mm_dist(bin, zero) << (kMmBucketBits + 1)) | ((bin < zero ? 1u : 0u) << kMmBucketBits) |
           (uint32_t)(cell & (kMmBucketCells - 1));
}
__device__ __forceinline__ int64_t mm_cell(const SpGroups* gp, int g, int r, int32_t key) {
    const int32_t cols = gp->cols[g];
    return gp->tab_off[g] + (int64_t)r * cols + java_hash_fm(gp->hash_ids[g][r], key, cols, gp->inv_cols[g]);
}
__device__ __forceinline__ uint64_t mm_pair(int32_t key, int32_t bin, int32_t zero, int64_t cell) {
    return ((uint64_t)mm_dist(bin, zero) << 48) | ((uint64_t)(uint32_t)key << 17) |
           ((uint64_t)(bin < zero ? 1u : 0u) << 16) | (uint64_t)(cell & (kMmBucketCells - 1));
}

// BKDRHash over 3-digit chunks (hash/BKDRHash.java:13-21).  The loop consumes a key's decimal
// digits least significant first, code = code * seed + digit, so a full 3-digit chunk c (digits
// d0 d1 d2, d0 the lowest) advances the code to code * seed^3 + (d0 seed^2 + d1 seed + d2), and
// the last chunk v (1..3 digits) to code * seed^len(v) + BKDR(v).  LDS tables per seed:
// f3[c] for full chunks, b3[v] = BKDR(v); one quarter-rate multiply per chunk instead of two per
// digit.  Keys are >= 0 here (a negative key fails the order check; java_hash_mix keeps the
// reference's signed digits for it).
constexpr int kBkSeeds = 5;  // hash ids 3..7
struct BkdrTables {
    uint32_t f3[kBkSeeds][1000];
    uint32_t b3[kBkSeeds][1000];
};
__device__ __forceinline__ uint32_t bkdr_seed(int id) {
    return id == 3 ? 31u : id == 4 ? 131u : id == 5 ? 267u : id == 6 ? 1313u : 13131u;
}
__device__ __forceinline__ void load_bkdr_tables(BkdrTables* T) {
    for (int e = threadIdx.x; e < kBkSeeds * 1000; e += blockDim.x) {
        const int si = e / 1000, v = e % 1000;
        const uint32_t sd = bkdr_seed(si + 3);
        const uint32_t d0 = (uint32_t)v % 10u, d1 = (uint32_t)v / 10u % 10u, d2 = (uint32_t)v / 100u;
        T->f3[si][v] = (d0 * sd + d1) * sd + d2;
        uint32_t c = 0, k = (uint32_t)v;
        while (k) {
            c = c * sd + k % 10u;
            k /= 10u;
        }
        T->b3[si][v] = c;
    }
}
template <int ID>
__device__ __forceinline__ uint32_t bkdr_fast(uint32_t k, const BkdrTables* T) {
    constexpr uint32_t sd = ID == 3 ? 31u : ID == 4 ? 131u : ID == 5 ? 267u : ID == 6 ? 1313u : 13131u;
    constexpr uint32_t s2 = sd * sd, s3 = s2 * sd;
    uint32_t c = 0;
    while (k >= 1000u) {
        const uint32_t q = k / 1000u;
        c = c * s3 + T->f3[ID - 3][k - q * 1000u];
        k = q;
    }
    const uint32_t pw = k >= 100u ? s3 : k >= 10u ? s2 : sd;
    return k ? c * pw + T->b3[ID - 3][k] : c;
}

// One row's cells of a batch whose group (and so hash) is uniform: the hash specialised at
// compile time, the modulus by multiplication.  Same cells as java_hash_fm.
template <int ID>
__device__ __forceinline__ void mm_cells(const int32_t (&key)[kMmBatch], int64_t base, int64_t c1, int64_t n, int r,
                                         int64_t row0, const MmGroup& q, const BkdrTables* BK,
                                         int32_t* __restrict__ cells_out, bool lds_b, uint32_t* BH,
                                         unsigned long long* __restrict__ bucket_count) {
    const int32_t cols = q.cols;
    const DivU32 dv = q.div;
#pragma unroll
    for (int u = 0; u < kMmBatch; u++) {
        const int64_t i = base + u * kMmThreads + threadIdx.x;
        if (i >= c1) continue;
        uint32_t h;
#ifdef SKML_ABLATE_GP_HASH  // timing ablation only (wrong cells): the insert's hashes priced
        h = (uint32_t)key[u] * 2654435761u;
#else
        if constexpr (ID >= 3) h = key[u] >= 0 ? bkdr_fast<ID>((uint32_t)key[u], BK) : java_hash_mix(ID, key[u]);
        else h = java_hash_mix(ID, key[u]);
#endif
        const int64_t cell = row0 + java_mod((int32_t)h, cols, dv);
        if (cells_out) cells_out[(int64_t)r * n + i] = (int32_t)cell;  // hashed once, reused by the scatter
        const int b = (int)(cell >> kMmBucketBits);
        if (lds_b) atomicAdd(&BH[b], 1u);
        else atomicAdd(&bucket_count[b], 1ull);
    }
}

// Deltas, bitsNeeded histogram and order check (DeltaAdaptiveEncoder.encode step 1) plus the
// per-bucket pair counts of the MinMax insert.
// 8 waves per SIMD (64 VGPRs, with kMmBatch = 4): two 1,024-thread workgroups per CU instead of
// one at 103 VGPRs and 8 elements in flight (C3: 195 -> 176 us; at 8 elements the cap spills)
#ifndef SKML_GP_WAVES
#define SKML_GP_WAVES 8
#endif
__global__ __launch_bounds__(kMmThreads, SKML_GP_WAVES) void k_group_prep(const int32_t* __restrict__ gkeys, int64_t n,
                                                           const SpGroups* __restrict__ gp,
                                                           uint8_t* __restrict__ need, uint32_t* __restrict__ hist,
                                                           uint32_t* __restrict__ err,
                                                           unsigned long long* __restrict__ bucket_count,
                                                           int nbuckets, int32_t* __restrict__ cells_out,
                                                           uint32_t* __restrict__ tile_off, int64_t chunk) {
    if (gp->status) return;
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint32_t H[kMaxGroups * kDeltaHist];
    __shared__ MmGroup GP[kMaxGroups];
    __shared__ BkdrTables BKs;
    extern __shared__ uint32_t BH[];  // nbuckets counters (dynamic: occupancy follows the table size)
    // need == nullptr: the MinMax part only; bucket_count == nullptr: the DeltaAdaptive part only
    const bool do_delta = need != nullptr, do_mm = bucket_count != nullptr;
    const int G = gp->G, rows = do_mm ? gp->rows : 0;
    const bool lds_b = nbuckets <= kMmLdsBuckets;
    const BkdrTables* BK = &BKs;
    load_starts(gp, S);
    load_mm_groups(gp, GP);
    if (rows > 0) load_bkdr_tables(&BKs);
    for (int j = threadIdx.x; j < G * kDeltaHist; j += kMmThreads) H[j] = 0;
    if (lds_b)
        for (int j = threadIdx.x; j < nbuckets; j += kMmThreads) BH[j] = 0;
    __syncthreads();
    uint32_t bad = 0;
    const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = std::min<int64_t>(n, c0 + chunk);
    // kMmBatch elements per thread in flight: their keys and predecessors load together
    for (int64_t base = c0; base < c1; base += kMmBatch * kMmThreads) {
        int32_t key[kMmBatch], prv[kMmBatch];
#pragma unroll
        for (int u = 0; u < kMmBatch; u++) {
            const int64_t i = base + u * kMmThreads + threadIdx.x;
            const int64_t j = i < c1 ? i : c1 - 1;
            key[u] = gkeys[j];
            prv[u] = do_delta && j > 0 ? gkeys[j - 1] : 0;
        }
        // almost every batch lies inside one group: then its hash ids are workgroup-uniform and
        // each row's cells come from a loop specialised for that hash
        const int64_t last = std::min<int64_t>(c1, base + kMmBatch * kMmThreads) - 1;
        const int g_lo = group_of_elem(S, base), g_hi = group_of_elem(S, last);
        const bool one = g_lo == g_hi;
        int gg[kMmBatch];
#pragma unroll
        for (int u = 0; u < kMmBatch; u++) {
            const int64_t i = base + u * kMmThreads + threadIdx.x;
            gg[u] = 0;
            if (i >= c1) continue;
            const int g = one ? g_lo : group_of_elem(S, i);
            gg[u] = g;
            if (!do_delta) continue;
            const bool first = i == S[g];
            const int32_t d = first ? key[u] : (int32_t)((uint32_t)key[u] - (uint32_t)prv[u]);
            int nb;
            if (first && d == 0) nb = 1;
            else {
                if (d <= 0) bad = 1;  // Maths.log2nlz: "Log for <d>" (util/Maths.java:16-21)
                nb = d > 0 ? 32 - __clz(d) : 1;
            }
            need[i] = (uint8_t)nb;
#ifndef SKML_ABLATE_GP_HIST  // timing ablation only (wrong histogram)
            atomicAdd(&H[g * kDeltaHist + nb], 1u);
#endif
        }
        if (one) {
            const MmGroup& q = GP[g_lo];
            for (int r = 0; r < rows; r++) {
                const int id = __builtin_amdgcn_readfirstlane(q.hid[r]);
                const int64_t row0 = q.tab_off + (int64_t)r * q.cols;
                switch (id) {
                    case 0: mm_cells<0>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    case 1: mm_cells<1>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    case 2: mm_cells<2>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    case 3: mm_cells<3>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    case 4: mm_cells<4>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    case 5: mm_cells<5>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    case 6: mm_cells<6>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                    default: mm_cells<7>(key, base, c1, n, r, row0, q, BK, cells_out, lds_b, BH, bucket_count); break;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < kMmBatch; u++) {
                const int64_t i = base + u * kMmThreads + threadIdx.x;
                if (i >= c1) continue;
                const MmGroup& q = GP[gg[u]];
                for (int r = 0; r < rows; r++) {
                    const int64_t cell =
                        q.tab_off + (int64_t)r * q.cols + java_hash_fm(q.hid[r], key[u], q.cols, q.inv);
                    if (cells_out) cells_out[(int64_t)r * n + i] = (int32_t)cell;
                    const int b = (int)(cell >> kMmBucketBits);
                    if (lds_b) atomicAdd(&BH[b], 1u);
                    else atomicAdd(&bucket_count[b], 1ull);
                }
            }
        }
    }
    if (bad) atomicOr(err, 1u);
    __syncthreads();
    if (do_delta)
        for (int j = threadIdx.x; j < G * kDeltaHist; j += kMmThreads)
            if (H[j]) atomicAdd(&hist[j], H[j]);
    if (lds_b && rows > 0) {
        if (tile_off) {  // reserve this tile's range in every bucket: 8 independent atomics in flight
            const bool narrow = gp->mm_narrow != 0;
            // Ranges are padded to whole 128-byte lines, so every line of the pair array is written by
            // one workgroup only (no partial-line write-backs from two XCDs' L2s).
            uint32_t* row = tile_off + (int64_t)blockIdx.x * nbuckets;
            for (int j0 = threadIdx.x; j0 < nbuckets; j0 += 8 * kMmThreads) {
                unsigned long long o[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + u * kMmThreads;
                    o[u] = (j < nbuckets && BH[j]) ? atomicAdd(&bucket_count[j], (unsigned long long)mm_pad(BH[j], narrow))
                                                   : 0ull;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + u * kMmThreads;
                    if (j < nbuckets) row[j] = (uint32_t)o[u];
                }
            }
        } else {
            for (int j = threadIdx.x; j < nbuckets; j += kMmThreads)
                if (BH[j]) atomicAdd(&bucket_count[j], (unsigned long long)BH[j]);
        }
    }
}

hipError_t launch_group_prep(hipStream_t st, const int32_t* gkeys, int64_t n, const SpGroups* gp, uint8_t* need,
                             uint32_t* hist, uint32_t* err, uint64_t* bucket_count, int nbuckets, int32_t* cells,
                             uint32_t* tile_off) {
    if (n <= 0) return hipSuccess;
    const size_t lds = nbuckets <= kMmLdsBuckets ? sizeof(uint32_t) * (size_t)(nbuckets > 0 ? nbuckets : 1) : 0;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_group_prep),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(sizeof(uint32_t) * kMmLdsBuckets));
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int64_t chunk = mm_chunk(n);
    hipLaunchKernelGGL(k_group_prep, dim3((unsigned)sp_tiles(n, chunk)), dim3(kMmThreads), lds, st, gkeys, n, gp,
                       need, hist, err, reinterpret_cast<unsigned long long*>(bucket_count), nbuckets, cells,
                       nbuckets <= kMmLdsBuckets ? tile_off : nullptr, chunk);
    return hipGetLastError();
}

// Scatter the pairs into bucket order: per-workgroup bucket counts reserve one range per bucket
// (one global atomic per workgroup and bucket), lanes take slots with LDS atomics.  Each thread
// handles 4 elements per step (4 independent load -> LDS atomic -> store chains), and the
// reserved 64-bit destinations sit in LDS, so the scatter never waits on a global load.
constexpr int kMmUnroll = 4;
__global__ __launch_bounds__(kMmThreads) void k_mm_scatter(const int32_t* __restrict__ gkeys,
                                                           const uint16_t* __restrict__ gbins, int64_t n,
                                                           const SpGroups* __restrict__ gp,
                                                           const uint64_t* __restrict__ bucket_base,
                                                           unsigned long long* __restrict__ cursor, int nbuckets,
                                                           uint64_t* __restrict__ pairs,
                                                           const int32_t* __restrict__ cells_in,
                                                           const uint32_t* __restrict__ tile_off, int64_t chunk) {
    if (gp->status) return;
    __shared__ int64_t S[kMaxGroups + 1];
    extern __shared__ uint64_t dyn64[];  // dst[nbuckets] (u64), cnt[nbuckets] (u32): dynamic, see launch
    uint64_t* dstb = dyn64;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(dyn64 + nbuckets);
    const int rows = gp->rows, zero = gp->zero;
    const bool lds_b = nbuckets <= kMmLdsBuckets;
    load_starts(gp, S);
    if (lds_b)
        for (int j = threadIdx.x; j < nbuckets; j += kMmThreads) cnt[j] = 0;
    __syncthreads();
    const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = std::min<int64_t>(n, c0 + chunk);
    // cell of (element i, row r): from k_group_prep's table when it kept one, else hashed again
    auto cell_of = [&](int g, int r, int64_t i, int32_t key) -> int64_t {
        return cells_in ? (int64_t)cells_in[(int64_t)r * n + i] : mm_cell(gp, g, r, key);
    };
    if (lds_b && tile_off) {  // ranges reserved by k_group_prep
        const uint32_t* row = tile_off + (int64_t)blockIdx.x * nbuckets;
        for (int j = threadIdx.x; j < nbuckets; j += kMmThreads) dstb[j] = bucket_base[j] + row[j];
        __syncthreads();
    } else if (lds_b) {
        for (int64_t base = c0; base < c1; base += kMmUnroll * kMmThreads) {
#pragma unroll
            for (int u = 0; u < kMmUnroll; u++) {
                const int64_t i = base + u * kMmThreads + threadIdx.x;
                if (i >= c1) break;
                const int g = cells_in ? 0 : group_of_elem(S, i);
                const int32_t key = cells_in ? 0 : gkeys[i];
                for (int r = 0; r < rows; r++) atomicAdd(&cnt[(int)(cell_of(g, r, i, key) >> kMmBucketBits)], 1u);
            }
        }
        __syncthreads();
        for (int j = threadIdx.x; j < nbuckets; j += kMmThreads) {
            dstb[j] = cnt[j] ? bucket_base[j] + atomicAdd(&cursor[j], (unsigned long long)cnt[j]) : 0ull;
            cnt[j] = 0;
        }
        __syncthreads();
    }
    if (lds_b && tile_off && cells_in) {
        // The common path, batched for memory-level parallelism: kMmBatch elements' keys, bins and
        // cells are loaded together (indices clamped into the tile), then ranked and stored.
        for (int64_t base = c0; base < c1; base += kMmBatch * kMmThreads) {
            int32_t key[kMmBatch], bin[kMmBatch];
            int64_t idx[kMmBatch];
#pragma unroll
            for (int u = 0; u < kMmBatch; u++) {
                const int64_t i = base + u * kMmThreads + threadIdx.x;
                idx[u] = i < c1 ? i : c1 - 1;
                key[u] = gkeys[idx[u]];
                bin[u] = gbins[idx[u]];
            }
            for (int r = 0; r < rows; r++) {
                int32_t cell[kMmBatch];
#pragma unroll
                for (int u = 0; u < kMmBatch; u++) cell[u] = cells_in[(int64_t)r * n + idx[u]];
#pragma unroll
                for (int u = 0; u < kMmBatch; u++) {
                    if (base + u * kMmThreads + threadIdx.x >= c1) continue;
                    const int b = cell[u] >> kMmBucketBits;
                    pairs[dstb[b] + atomicAdd(&cnt[b], 1u)] = mm_pair(key[u], bin[u], zero, cell[u]);
                }
            }
        }
    } else {
        for (int64_t base = c0; base < c1; base += kMmUnroll * kMmThreads) {
#pragma unroll
            for (int u = 0; u < kMmUnroll; u++) {
                const int64_t i = base + u * kMmThreads + threadIdx.x;
                if (i >= c1) break;
                const int g = cells_in ? 0 : group_of_elem(S, i);
                const int32_t key = gkeys[i], bin = gbins[i];
                for (int r = 0; r < rows; r++) {
                    const int64_t cell = cell_of(g, r, i, key);
                    const int b = (int)(cell >> kMmBucketBits);
                    const uint64_t dst = lds_b ? dstb[b] + atomicAdd(&cnt[b], 1u)
                                               : bucket_base[b] + (uint64_t)atomicAdd(&cursor[b], 1ull);
                    pairs[dst] = mm_pair(key, bin, zero, cell);
                }
            }
        }
    }
    if (lds_b && tile_off) {  // fill each range's padding (k_group_prep reserved mm_pad(count) slots)
        __syncthreads();
        for (int j = threadIdx.x; j < nbuckets * 16; j += kMmThreads) {
            const uint32_t c = cnt[j >> 4], slot = c + (uint32_t)(j & 15);
            if (c && slot < mm_pad(c)) pairs[dstb[j >> 4] + slot] = kMmNoPair;
        }
    }
}


// LDS-staged scatter (the common case: cells kept by k_group_prep, reserved ranges, at most
// kStageBuckets buckets).  The tile is cut into chunks of up to 8 pairs per thread; each chunk is
// ranked per bucket (LDS atomics), counting-sorted by bucket into LDS and stored bucket run by
// bucket run, so the pair stores go out as runs of consecutive addresses instead of one random
// 8-byte store per lane.  The next chunk's loads are issued before the current chunk's LDS phases.
constexpr int kStageBuckets = 4096;

template <int T>
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* sh, uint32_t& total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < T / 64; j++) {
        const uint32_t x = sh[j];
        before += j < w ? x : 0u;
        tot += x;
    }
    total = tot;
    return before + inc - v;
}

// PAIR: uint64_t (key-carrying pairs) or uint32_t (narrow pairs, SpGroups.mm_narrow).
template <int T, typename PAIR>
__device__ __forceinline__ void mm_scatter_staged_body(const int32_t* __restrict__ gkeys,
                                                       const uint16_t* __restrict__ gbins, int64_t n,
                                                       const SpGroups* __restrict__ gp,
                                                       const uint64_t* __restrict__ bucket_base, int nbuckets,
                                                       PAIR* __restrict__ pairs, const int32_t* __restrict__ cells_in,
                                                       const uint32_t* __restrict__ tile_off, uint64_t* dyn64,
                                                       uint32_t* scan_sh, int64_t chunk) {
    constexpr bool kNarrow = sizeof(PAIR) == 4;
    constexpr int kStage = 8 * T;
    // LDS: dstb[nb] u64 | stage[kStage] PAIR | lc[nb] u32 | lofs[nb + 1] u32 | sb[kStage] u16
    uint64_t* dstb = dyn64;
    PAIR* stage = reinterpret_cast<PAIR*>(dstb + nbuckets);
    uint32_t* lc = reinterpret_cast<uint32_t*>(stage + kStage);
    uint32_t* lofs = lc + nbuckets;
    uint16_t* sb = reinterpret_cast<uint16_t*>(lofs + nbuckets + 1);
    const int t = threadIdx.x, rows = gp->rows, zero = gp->zero;
    const uint32_t* row = tile_off + (int64_t)blockIdx.x * nbuckets;
    for (int j = t; j < nbuckets; j += T) {
        dstb[j] = bucket_base[j] + row[j];
        lc[j] = 0;
    }
    const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = std::min<int64_t>(n, c0 + chunk);
    const int et = 8 / rows;  // elements per thread per chunk: et * rows <= 8 pairs each
    const int np = et * rows;
    const int64_t step = (int64_t)et * T;
    constexpr int kPer = (kStageBuckets + T - 1) / T;
    int32_t nk[8], nbn[8], nc[8];  // the next chunk's loads
    auto load = [&](int64_t base) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int u = k / rows, r = k - u * rows;
            const int64_t i = base + (int64_t)u * T + t;
            nc[k] = -1;
            if (k < np && i < c1) {
                nc[k] = cells_in[(int64_t)r * n + i];
                if constexpr (!kNarrow) nk[k] = gkeys[i];
                nbn[k] = gbins[i];
            }
        }
    };
    load(c0);
    __syncthreads();
    for (int64_t base = c0; base < c1; base += step) {
        PAIR pv[8];
        int32_t bk[8];
        uint32_t rk[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            bk[k] = nc[k] >= 0 ? nc[k] >> kMmBucketBits : -1;
            if (bk[k] >= 0) {
                if constexpr (kNarrow) pv[k] = mm_pair32(nbn[k], zero, nc[k]);
                else pv[k] = mm_pair(nk[k], nbn[k], zero, nc[k]);
            }
        }
        if (base + step < c1) load(base + step);
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (bk[k] >= 0) rk[k] = atomicAdd(&lc[bk[k]], 1u);
        __syncthreads();
        // exclusive scan of the chunk's bucket counts
        uint32_t loc[kPer], sum = 0;
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const int j = t * kPer + q;
            loc[q] = j < nbuckets ? lc[j] : 0u;
            sum += loc[q];
        }
        uint32_t total;
        uint32_t run = block_excl_scan_u32<T>(sum, scan_sh, total);
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const int j = t * kPer + q;
            if (j < nbuckets) lofs[j] = run;
            run += loc[q];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (bk[k] >= 0) {
                const uint32_t q = lofs[bk[k]] + rk[k];
                stage[q] = pv[k];
                sb[q] = (uint16_t)bk[k];
            }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t q = (uint32_t)(u * T + t);
            if (q < total) {
                const int b = sb[q];
                pairs[dstb[b] + (q - lofs[b])] = stage[q];
            }
        }
        __syncthreads();
        for (int j = t; j < nbuckets; j += T)
            if (lc[j]) {
                dstb[j] += lc[j];
                lc[j] = 0;
            }
        __syncthreads();
    }
    // padding of each reserved range (mm_pad(count) slots): from the range's end up to the pad
    constexpr int kPadMax = kNarrow ? 32 : 16;
    for (int j = t; j < nbuckets * kPadMax; j += T) {
        const int bb = j / kPadMax;
        const uint64_t b0 = bucket_base[bb] + row[bb], e = dstb[bb];
        const uint64_t c = e - b0, slot = e + (uint64_t)(j % kPadMax);
        if (c && slot < b0 + mm_pad((uint32_t)c, kNarrow)) pairs[slot] = kNarrow ? (PAIR)kMmNoPair32 : (PAIR)kMmNoPair;
    }
}

template <int T>
__global__ __launch_bounds__(T) void k_mm_scatter_staged(const int32_t* __restrict__ gkeys,
                                                         const uint16_t* __restrict__ gbins, int64_t n,
                                                         const SpGroups* __restrict__ gp,
                                                         const uint64_t* __restrict__ bucket_base, int nbuckets,
                                                         void* __restrict__ pairs,
                                                         const int32_t* __restrict__ cells_in,
                                                         const uint32_t* __restrict__ tile_off, int64_t chunk) {
    if (gp->status) return;
    extern __shared__ uint64_t dyn64[];
    __shared__ uint32_t scan_sh[T / 64];
    if (gp->mm_narrow)
        mm_scatter_staged_body<T, uint32_t>(gkeys, gbins, n, gp, bucket_base, nbuckets,
                                            static_cast<uint32_t*>(pairs), cells_in, tile_off, dyn64, scan_sh, chunk);
    else
        mm_scatter_staged_body<T, uint64_t>(gkeys, gbins, n, gp, bucket_base, nbuckets,
                                            static_cast<uint64_t*>(pairs), cells_in, tile_off, dyn64, scan_sh, chunk);
}
#ifndef SKML_STAGE_THREADS
#define SKML_STAGE_THREADS 512
#endif
constexpr int kStageThreads = SKML_STAGE_THREADS;
inline size_t staged_lds(int nbuckets) {
    return (sizeof(uint64_t) + sizeof(uint16_t)) * 8 * kStageThreads + 16 * (size_t)nbuckets + 4;
}

bool mm_scatter_staged(bool cells, bool reserved, int nbuckets) {
    return cells && reserved && nbuckets <= kStageBuckets;
}

hipError_t launch_mm_scatter(hipStream_t st, const int32_t* gkeys, const uint16_t* gbins, int64_t n,
                             const SpGroups* gp, const uint64_t* bucket_base, uint64_t* cursor, int nbuckets,
                             void* pairs_v, const int32_t* cells, const uint32_t* tile_off) {
    uint64_t* pairs = static_cast<uint64_t*>(pairs_v);  // the unstaged scatter: key-carrying pairs only
    if (n <= 0) return hipSuccess;
    const int64_t chunk = mm_chunk(n);
    if (mm_scatter_staged(cells != nullptr, tile_off != nullptr, nbuckets)) {
        static bool attr_s = false;
        if (!attr_s) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mm_scatter_staged<kStageThreads>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)staged_lds(kStageBuckets));
            if (e != hipSuccess) return e;
            attr_s = true;
        }
        hipLaunchKernelGGL(k_mm_scatter_staged<kStageThreads>, dim3((unsigned)sp_tiles(n, chunk)),
                           dim3(kStageThreads), staged_lds(nbuckets), st, gkeys, gbins, n, gp, bucket_base, nbuckets,
                           pairs_v, cells, tile_off, chunk);
        return hipGetLastError();
    }
    constexpr size_t kPer = sizeof(uint64_t) + sizeof(uint32_t);
    const size_t lds = nbuckets <= kMmLdsBuckets ? kPer * (size_t)(nbuckets > 0 ? nbuckets : 1) : 0;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mm_scatter),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kPer * kMmLdsBuckets));
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(k_mm_scatter, dim3((unsigned)sp_tiles(n, chunk)), dim3(kMmThreads), lds, st, gkeys, gbins, n,
                       gp, bucket_base, reinterpret_cast<unsigned long long*>(cursor), nbuckets, pairs, cells,
                       nbuckets <= kMmLdsBuckets ? tile_off : nullptr, chunk);
    return hipGetLastError();
}

// One workgroup per bucket: LDS minimum per cell, then the int32 table cells (empty -> fill).
// Narrow pairs (SpGroups.mm_narrow) take 32-bit LDS minima over (distance, sign) for the whole
// bucket; key-carrying pairs take 64-bit minima, one 8192-cell sub-range after the other (each
// sub-range re-reads the bucket's pairs; this path only runs for groups on both sides of zeroIdx).
// tnar (may be nullptr): the exact narrow image of the table as well -- a cell's bin in 8 bits when
// the group table's bin_num <= 255, else in 16 bits when <= 65,535, the fill as the top code
// (2^W - 1); the payload's restore gathers from it and the exchange blob carries it
// (tnar_width_for).
__global__ __launch_bounds__(kMmThreads) void k_mm_bucket(const void* __restrict__ pairs_v,
                                                          const uint64_t* __restrict__ bucket_base,
                                                          const SpGroups* __restrict__ gp,
                                                          int32_t* __restrict__ table, void* __restrict__ tnar) {
    constexpr int kWords = kMmBucketCells / 2 > kMmSubCells ? kMmBucketCells / 2 : kMmSubCells;
    __shared__ unsigned long long cm64[kWords];  // u32 minima of the bucket, or u64 of a sub-range
    uint32_t* cm = reinterpret_cast<uint32_t*>(cm64);
    const int b = blockIdx.x;
    const int64_t ncells = gp->ncells;
    if (gp->status || ((int64_t)b << kMmBucketBits) >= ncells) return;
    const int32_t zero = gp->zero, fill = gp->fill;
    const uint64_t p0 = bucket_base[b], p1 = bucket_base[b + 1];
    const int64_t cell0 = (int64_t)b << kMmBucketBits;
    const int tw = tnar ? tnar_width_for(gp->bin_num) : 0;
    auto put = [&](int64_t cell, int32_t out) {
        table[cell] = out;
        if (tw == 8) static_cast<uint8_t*>(tnar)[cell] = out == fill ? (uint8_t)0xFF : (uint8_t)out;
        else if (tw == 16) static_cast<uint16_t*>(tnar)[cell] = out == fill ? (uint16_t)0xFFFF : (uint16_t)out;
    };
    if (gp->mm_narrow) {
        const uint32_t* pairs = static_cast<const uint32_t*>(pairs_v);
        for (int j = threadIdx.x; j < kMmBucketCells; j += kMmThreads) cm[j] = ~0u;
        __syncthreads();
        constexpr uint32_t kLo = (uint32_t)(kMmBucketCells - 1);
        constexpr int kB = 2 * kBucketBatch;  // half the bytes per pair: twice the pairs in flight
        for (uint64_t p = p0 + threadIdx.x; p < p1; p += kB * kMmThreads) {
            uint32_t v[kB];
#pragma unroll
            for (int u = 0; u < kB; u++) v[u] = p + u * kMmThreads < p1 ? pairs[p + u * kMmThreads] : kMmNoPair32;
#pragma unroll
            for (int u = 0; u < kB; u++)
                if (v[u] != kMmNoPair32) atomicMin(&cm[v[u] & kLo], v[u] >> kMmBucketBits);
        }
        __syncthreads();
        for (int j = threadIdx.x; j < kMmBucketCells && cell0 + j < ncells; j += kMmThreads) {
            const uint32_t v = cm[j];
            int32_t out = fill;
            if (v != ~0u) {
                const int32_t dist = (int32_t)(v >> 1);
                out = (v & 1u) ? zero - dist : zero + dist;
            }
            put(cell0 + j, out);
        }
        return;
    }
    const uint64_t* pairs = static_cast<const uint64_t*>(pairs_v);
    unsigned long long* cmin = cm64;
    constexpr uint64_t kLo = (uint64_t)(kMmBucketCells - 1), kSubLo = (uint64_t)(kMmSubCells - 1);
    for (int sub = 0; sub < kMmBucketCells / kMmSubCells; sub++) {
        const int64_t s0 = cell0 + (int64_t)sub * kMmSubCells;
        if (s0 >= ncells) break;
        if (sub) __syncthreads();  // the previous sub-range's cells are written
        for (int j = threadIdx.x; j < kMmSubCells; j += kMmThreads) cmin[j] = ~0ull;
        __syncthreads();
        for (uint64_t p = p0 + threadIdx.x; p < p1; p += kBucketBatch * kMmThreads) {
            uint64_t v[kBucketBatch];
#pragma unroll
            for (int u = 0; u < kBucketBatch; u++) v[u] = p + u * kMmThreads < p1 ? pairs[p + u * kMmThreads] : kMmNoPair;
#pragma unroll
            for (int u = 0; u < kBucketBatch; u++)
                if (v[u] != kMmNoPair && (int)((v[u] & kLo) >> kMmSubBits) == sub)
                    atomicMin(&cmin[v[u] & kSubLo], (unsigned long long)(v[u] & ~kLo));
        }
        __syncthreads();
        for (int j = threadIdx.x; j < kMmSubCells && s0 + j < ncells; j += kMmThreads) {
            const uint64_t v = cmin[j];
            int32_t out = fill;
            if (v != ~0ull) {
                const int32_t dist = (int32_t)(v >> 48);
                out = ((v >> 16) & 1u) ? zero - dist : zero + dist;
            }
            put(s0 + j, out);
        }
    }
}

hipError_t launch_mm_bucket(hipStream_t st, const void* pairs, const uint64_t* bucket_base, int nbuckets,
                            const SpGroups* gp, int32_t* table, void* tnar) {
    if (nbuckets <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mm_bucket, dim3((unsigned)nbuckets), dim3(kMmThreads), 0, st, pairs, bucket_base, gp,
                       table, tnar);
    return hipGetLastError();
}

// SparseVectorCompressor.quantValues = Quantizer.getValues() (base/Quantizer.java:39-47) of the
// values' quantizer payload, on the device: the same double expressions the host evaluates after
// the encode's read-back, so the restore needs no upload of the table.
__global__ __launch_bounds__(256) void k_sp_qvalues(const uint8_t* __restrict__ qpayload, double* __restrict__ qv) {
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(qpayload);
    if (h->status != SKML_OK) return;
    const double* sp = reinterpret_cast<const double*>(qpayload + kHeaderBytes);
    const int B = h->bin_num, ns = B - 1;
    for (int b = (int)threadIdx.x; b < B && ns > 0; b += 256) {
        double v;
        if (b == 0) v = 0.5 * (h->min + sp[0]);
        else if (b == ns) v = 0.5 * (sp[ns - 1] + h->max);
        else v = 0.5 * (sp[b - 1] + sp[b]);
        qv[b] = v;
    }
}

hipError_t launch_sp_qvalues(hipStream_t st, const void* qpayload, double* qv) {
    hipLaunchKernelGGL(k_sp_qvalues, dim3(1), dim3(256), 0, st, static_cast<const uint8_t*>(qpayload), qv);
    return hipGetLastError();
}

// int32 cells from an exact narrow image (tnar_width_for): the top code back to the fill
__global__ __launch_bounds__(256) void k_widen_cells(const void* __restrict__ tn, int tw, int64_t ncells, int32_t fill,
                                                     int32_t* __restrict__ t32) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ncells; i += (int64_t)gridDim.x * 256) {
        const uint32_t v = tw == 8 ? static_cast<const uint8_t*>(tn)[i] : static_cast<const uint16_t*>(tn)[i];
        t32[i] = v == (tw == 8 ? 0xFFu : 0xFFFFu) ? fill : (int32_t)v;
    }
}

hipError_t launch_widen_cells(hipStream_t st, const void* tn, int tw, int64_t ncells, int32_t fill, int32_t* t32) {
    if (ncells <= 0) return hipSuccess;
    if (tw != 8 && tw != 16) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<int64_t>(sp_tiles(ncells, 256 * 4), 4096);
    hipLaunchKernelGGL(k_widen_cells, dim3(grid), dim3(256), 0, st, tn, tw, ncells, fill, t32);
    return hipGetLastError();
}

// =============================================================================================
// DeltaAdaptive bit streams
// =============================================================================================
struct DeltaShape {
    int bpi, shift, nf, kind;
};
__device__ __forceinline__ DeltaShape delta_shape(const SpGroups* gp, int g) {
    DeltaShape s;
    const int m = gp->m[g];
    s.bpi = 32 / m;
    s.shift = 31 - __clz(s.bpi);
    s.nf = 31 - __clz(m);
    s.kind = gp->kind[g];
    return s;
}
// interval count, flag length, delta length of one element
__device__ __forceinline__ void delta_lens(const DeltaShape& s, int nb, int& iv, int& fl, int& dl) {
    iv = (nb + s.bpi - 1) >> s.shift;
    fl = s.kind ? iv + 1 : s.nf;
    dl = s.bpi * iv;
}

// need[i0, i0 + 8) (one 8-byte load when the run is whole; i0 is a multiple of 8)
__device__ __forceinline__ void load8_need(const uint8_t* __restrict__ need, int64_t i0, int64_t n, uint8_t (&nb)[8]) {
    if (i0 + 8 <= n) {
        const uint2 w = *reinterpret_cast<const uint2*>(need + i0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            nb[j] = (uint8_t)(w.x >> (8 * j));
            nb[4 + j] = (uint8_t)(w.y >> (8 * j));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) nb[j] = i0 + j < n ? need[i0 + j] : (uint8_t)0;
    }
}
// gkeys[i0, i0 + 8) (two 16-byte loads when the run is whole)
__device__ __forceinline__ void load8_keys(const int32_t* __restrict__ k, int64_t i0, int64_t n, int32_t (&key)[8]) {
    if (i0 + 8 <= n) {
        const int4 a = *reinterpret_cast<const int4*>(k + i0), b = *reinterpret_cast<const int4*>(k + i0 + 4);
        key[0] = a.x, key[1] = a.y, key[2] = a.z, key[3] = a.w;
        key[4] = b.x, key[5] = b.y, key[6] = b.z, key[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) key[j] = i0 + j < n ? k[i0 + j] : 0;
    }
}

__global__ __launch_bounds__(kSpThreads) void k_delta_lens(const uint8_t* __restrict__ need, int64_t n,
                                                           const SpGroups* __restrict__ gp,
                                                           uint64_t* __restrict__ tile_sums) {
    if (gp->status) return;
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint64_t sh[8];
    load_starts(gp, S);
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint64_t fsum = 0, dsum = 0;
    if (i0 < n) {
        uint8_t nb[8];
        load8_need(need, i0, n, nb);
        int g = group_of_elem(S, i0);
        DeltaShape s = delta_shape(gp, g);
        for (int j = 0; j < 8 && i0 + j < n; j++) {
            const int64_t i = i0 + j;
            while (i >= S[g + 1]) s = delta_shape(gp, ++g);
            int iv, fl, dl;
            delta_lens(s, nb[j], iv, fl, dl);
            fsum += fl;
            dsum += dl;
        }
    }
    uint64_t v[2] = {fsum, dsum}, tot[2];
    block_excl_scan<2>(v, tot, sh);
    if (threadIdx.x == 0) {
        tile_sums[blockIdx.x * 2] = tot[0];
        tile_sums[blockIdx.x * 2 + 1] = tot[1];
    }
}

hipError_t launch_delta_lens(hipStream_t st, const uint8_t* need, int64_t n, const SpGroups* gp,
                             uint64_t* tile_sums) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_delta_lens, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, need, n, gp, tile_sums);
    return hipGetLastError();
}

// BinaryUtils.setBits (binary/BinaryUtils.java:6-14): value's MSB at the lowest bit position.
__device__ __forceinline__ void lds_put_bits(uint64_t* win, int64_t rel, uint32_t value, int nbits) {
    if (nbits <= 0) return;
    const uint64_t rev = (uint64_t)(__brev(value) >> (32 - nbits));
    const int64_t w = rel >> 6;
    const int sh = (int)(rel & 63);
    atomicOr(reinterpret_cast<unsigned long long*>(&win[w]), (unsigned long long)(rev << sh));
    if (sh + nbits > 64) atomicOr(reinterpret_cast<unsigned long long*>(&win[w + 1]), (unsigned long long)(rev >> (64 - sh)));
}

constexpr int kFlagWin = (kSpTile * 17 + 63) / 64 + 2;
constexpr int kDeltaWin = (kSpTile * 32 + 63) / 64 + 2;

__device__ __forceinline__ void flush_window(const uint64_t* win, int64_t bit0, uint64_t nbits, uint64_t* out) {
    if (nbits == 0) return;
    const int64_t w0 = bit0 >> 6, w1 = (bit0 + (int64_t)nbits - 1) >> 6;
    for (int64_t w = w0 + threadIdx.x; w <= w1; w += kSpThreads) {
        const uint64_t v = win[w - w0];
        if (w == w0 || w == w1) {
            if (v) atomicOr(reinterpret_cast<unsigned long long*>(&out[w]), (unsigned long long)v);
        } else {
            out[w] = v;
        }
    }
}

__global__ __launch_bounds__(kSpThreads) void k_delta_write(const int32_t* __restrict__ gkeys,
                                                            const uint8_t* __restrict__ need, int64_t n,
                                                            SpGroups* __restrict__ gp,
                                                            const uint64_t* __restrict__ tile_base,
                                                            uint64_t* __restrict__ flag_words,
                                                            uint64_t* __restrict__ delta_words) {
    if (gp->status) return;
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint64_t sh[8];
    __shared__ uint64_t fwin[kFlagWin];
    __shared__ uint64_t dwin[kDeltaWin];
    load_starts(gp, S);
    for (int j = threadIdx.x; j < kFlagWin; j += kSpThreads) fwin[j] = 0;
    for (int j = threadIdx.x; j < kDeltaWin; j += kSpThreads) dwin[j] = 0;
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    int32_t key[8];
    uint8_t nb[8];
    uint64_t fsum = 0, dsum = 0;
    int g0 = 0;
    // every global read is issued here, before the scan: the tile's bases, the run's keys and
    // lengths, and the key before the run (used when the run does not start its group)
    const uint64_t fbase = tile_base[blockIdx.x * 2], dbase = tile_base[blockIdx.x * 2 + 1];
    int32_t prev0 = 0;
    if (i0 < n) {
        load8_keys(gkeys, i0, n, key);
        load8_need(need, i0, n, nb);
        prev0 = i0 > 0 ? gkeys[i0 - 1] : 0;
        g0 = group_of_elem(S, i0);
        int g = g0;
        DeltaShape s = delta_shape(gp, g);
        for (int j = 0; j < 8; j++) {
            const int64_t i = i0 + j;
            if (i >= n) break;
            while (i >= S[g + 1]) s = delta_shape(gp, ++g);
            int iv, fl, dl;
            delta_lens(s, nb[j], iv, fl, dl);
            fsum += fl;
            dsum += dl;
        }
    }
    uint64_t v[2] = {fsum, dsum}, tot[2];
    block_excl_scan<2>(v, tot, sh);
    const int64_t fw0 = (int64_t)(fbase >> 6) << 6, dw0 = (int64_t)(dbase >> 6) << 6;
    if (i0 < n) {
        int g = g0;
        DeltaShape s = delta_shape(gp, g);
        uint64_t fo = fbase + v[0], dof = dbase + v[1];
        int32_t prev = i0 > S[g] ? prev0 : 0;
        for (int j = 0; j < 8; j++) {
            const int64_t i = i0 + j;
            if (i >= n) break;
            while (i >= S[g + 1]) s = delta_shape(gp, ++g);
            const bool first = i == S[g];
            if (first) {
                gp->fb[g] = (int64_t)fo;
                gp->db[g] = (int64_t)dof;
            }
            const uint32_t d = first ? (uint32_t)key[j] : (uint32_t)key[j] - (uint32_t)prev;
            prev = key[j];
            int iv, fl, dl;
            delta_lens(s, nb[j], iv, fl, dl);
            const uint32_t fv = s.kind ? (uint32_t)((1u << (iv + 1)) - 2u) : (uint32_t)(iv - 1);
            lds_put_bits(fwin, (int64_t)fo - fw0, fv, fl);
            // bitsPerInterval * intervalNeeded <= 32; a 32-bit field holds d itself
            lds_put_bits(dwin, (int64_t)dof - dw0, d, dl);
            fo += fl;
            dof += dl;
        }
    }
    __syncthreads();
    flush_window(fwin, (int64_t)fbase, tot[0], flag_words);
    flush_window(dwin, (int64_t)dbase, tot[1], delta_words);
}

hipError_t launch_delta_write(hipStream_t st, const int32_t* gkeys, const uint8_t* need, int64_t n,
                              SpGroups* gp, const uint64_t* tile_base, uint64_t* flag_words,
                              uint64_t* delta_words) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_delta_write, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, gkeys, need, n, gp,
                       tile_base, flag_words, delta_words);
    return hipGetLastError();
}

// =============================================================================================
// Device-side encode plan: the per-group decisions the reference takes on whole-group
// statistics, made where the statistics are, so an encode never waits on a host round trip.
// =============================================================================================
// MinMaxSketch.compare with Java int wrap (MinMaxSketch.java:80-86)
__device__ __forceinline__ int32_t mm_cmp(int32_t a, int32_t b, int32_t zero) {
    return (int32_t)((uint32_t)mm_dist(a, zero) - (uint32_t)mm_dist(b, zero));
}

// 4-byte MinMax pairs when no group holds bins on both sides of zeroIdx (FSketchUtils.partition:
// group g takes the bins in [edges[g-1], edges[g])).  calGroupEdges puts zeroIdx on an edge
// unless it falls in the last group or two, so this is the common case.
__device__ void mm_plan_narrow(SpGroups* gp, const SpInit& init) {
    int32_t lo = 0, narrow = init.narrow_ok ? 1 : 0;
    for (int g = 0; g < gp->G; g++) {
        const int32_t hi = gp->edges[g];
        if (lo < gp->zero && gp->zero < hi - 1) narrow = 0;  // a bin below zero and one above
        lo = hi > lo ? hi : lo;
    }
    gp->mm_narrow = narrow;
}

// Table from `init` (every field of the reused device struct rewritten), then
// FSketchUtils.calGroupEdges (frequency/FSketchUtils.java:9-28) on the quantizer's zeroIdx and
// binNum, and the MinMaxSketch fill (MinMaxSketch.java:30-33).
__global__ __launch_bounds__(64) void k_sp_plan_edges(const skml_dense_header* __restrict__ h, SpInit init,
                                                      SpGroups* __restrict__ gp) {
    uint32_t* w = reinterpret_cast<uint32_t*>(gp);
    for (int j = threadIdx.x; j < (int)(sizeof(SpGroups) / 4); j += 64) w[j] = 0u;
    __syncthreads();
    for (int j = threadIdx.x; j < kMaxGroups * kMaxRows; j += 64)
        gp->hash_ids[j / kMaxRows][j % kMaxRows] = init.hash_ids[j / kMaxRows][j % kMaxRows];
    if (threadIdx.x) return;
    const int32_t G = init.G;
    gp->G = G;
    gp->rows = init.rows;
    gp->col_ratio = init.col_ratio;
    if (h->status != SKML_OK) {  // "Encounter NaN value": nothing else runs
        gp->status = kSpNan;
        return;
    }
    const int32_t zero = h->zero_idx, bins = h->bin_num;
    gp->zero = zero;
    gp->bin_num = bins;
    gp->fill = mm_cmp(INT32_MIN, INT32_MAX, zero) <= 0 ? INT32_MIN : INT32_MAX;
    if (G == 2) {
        gp->edges[0] = zero;
        gp->edges[1] = bins;
        mm_plan_narrow(gp, init);
        return;
    }
    const int32_t bpg = bins / G;
    int32_t e;
    if (zero < bpg) e = zero;
    else if (bpg == 0) {  // Java: ArithmeticException "/ by zero"
        gp->status = kSpEdges;
        return;
    } else if ((zero % bpg) < (bpg / 2)) e = bpg + zero % bpg;
    else e = zero % bpg;
    for (int32_t i = 0; i < G - 1; i++, e += bpg) gp->edges[i] = e;
    gp->edges[G - 1] = bins;
    mm_plan_narrow(gp, init);
}

// GroupedMinMaxSketch.compOneGroup's shapes (GroupedMinMaxSketch.java:103-121): colNum =
// ceil(size * colRatio) (no multiply-add contraction: the product rounds as in Java).
__global__ __launch_bounds__(64) void k_sp_plan_groups(SpGroups* __restrict__ gp, const uint64_t* __restrict__ sizes,
                                                       int64_t stride) {
    if (gp->status || threadIdx.x) return;
    const int G = gp->G, rows = gp->rows;
    const double ratio = gp->col_ratio;
    int64_t start = 0, cells = 0;
    for (int g = 0; g < G; g++) {
        const int64_t m = (int64_t)sizes[g * stride];
        gp->gstart[g] = start;
        start += m;
        const int32_t cols = m > 0 ? (int32_t)ceil(__dmul_rn((double)m, ratio)) : 1;
        gp->cols[g] = cols;
        gp->inv_cols[g] = __ddiv_rn(1.0, (double)cols);
        gp->tab_off[g] = cells;
        if (m > 0) cells += (int64_t)rows * cols;
        else
            for (int r = 0; r < kMaxRows; r++) gp->hash_ids[g][r] = 0;  // an empty group picks no hashes
    }
    gp->gstart[G] = start;
    gp->ncells = cells;
}

// DeltaAdaptiveEncoder.calOptimalIntervals (binary/DeltaAdaptiveEncoder.java:23-51) in the
// reference's double summation order, every operation rounded on its own.
__device__ void delta_choose(const uint32_t* __restrict__ count, int64_t size, int32_t& bm, int32_t& bk) {
    double prob[32];
    for (int i = 0; i < 32; i++) prob[i] = __ddiv_rn((double)count[i], (double)size);
    double best = 32.0;
    bm = 1;
    bk = 0;
    for (int32_t m = 2, lg = 1; m <= 16; m *= 2, lg++) {
        const int32_t b = 32 / m;
        double sum = 0.0;
        for (int32_t i = 0; i < m; i++) {
            double ip = 0.0;
            for (int32_t j = 0; j < b; j++) ip = __dadd_rn(ip, prob[i * b + j]);
            sum = __dadd_rn(sum, __dmul_rn((double)(i + 1), ip));
        }
        const double t1 = __dadd_rn(__dmul_rn(sum, (double)b), (double)lg);
        if (t1 < best) {
            best = t1;
            bm = m;
            bk = 0;
        }
        const double t2 = __dadd_rn(__dmul_rn(sum, (double)(b + 1)), 1.0);
        if (t2 < best) {
            best = t2;
            bm = m;
            bk = 1;
        }
    }
}

// One lane per group: its interval choice; lane 0 then the order check and kind1_before.
__global__ __launch_bounds__(64) void k_sp_plan_delta(SpGroups* __restrict__ gp, const uint32_t* __restrict__ hist,
                                                      const uint32_t* __restrict__ err) {
    if (gp->status) return;
    const int G = gp->G, g = threadIdx.x;
    if (g < G) {
        const int64_t m = gp->gstart[g + 1] - gp->gstart[g];
        int32_t bm = 1, bk = 0;
        if (m > 0) {
            uint32_t cnt[32];
            for (int i = 0; i < 32; i++) cnt[i] = hist[g * kDeltaHist + i];
            cnt[31] += hist[g * kDeltaHist + 32];  // bitsNeeded 32 cannot occur for positive deltas
            delta_choose(cnt, m, bm, bk);
        }
        gp->m[g] = bm;
        gp->kind[g] = bk;
    }
    __syncthreads();
    if (g) return;
    if (*err) {  // Maths.log2nlz: "Log for <d>" (util/Maths.java:16-21)
        gp->status = kSpOrder;
        return;
    }
    int32_t k1 = 0;
    for (int j = 0; j < G; j++) {
        gp->kind1_before[j] = k1;
        if (gp->kind[j]) k1 += (int32_t)(gp->gstart[j + 1] - gp->gstart[j]);
    }
}

__global__ __launch_bounds__(kSpThreads) void k_sp_zero_edges(const uint64_t* __restrict__ ts, int64_t tiles,
                                                              const SpGroups* __restrict__ gp,
                                                              uint64_t* __restrict__ fw, uint64_t* __restrict__ dw) {
    if (gp->status) return;
    const int64_t i = (int64_t)blockIdx.x * kSpThreads + threadIdx.x;
    if (i > tiles) return;
    const uint64_t f0 = ts[2 * i], d0 = ts[2 * i + 1];
    fw[f0 >> 6] = 0;
    dw[d0 >> 6] = 0;
    if (i < tiles) {
        const uint64_t f1 = ts[2 * i + 2], d1 = ts[2 * i + 3];
        if (f1 > f0) fw[(f1 - 1) >> 6] = 0;
        if (d1 > d0) dw[(d1 - 1) >> 6] = 0;
    } else {  // the trailing word of each stream (n_words = ceil(bits / 64) + 1)
        fw[(f0 >> 6) + 1] = 0;
        dw[(d0 >> 6) + 1] = 0;
    }
}

__global__ __launch_bounds__(64) void k_sp_finalize(SpGroups* __restrict__ gp, const uint64_t* __restrict__ tot) {
    if (gp->status || threadIdx.x) return;
    const int G = gp->G;
    gp->fb[G] = (int64_t)tot[0];
    gp->db[G] = (int64_t)tot[1];
    for (int g = G - 1; g >= 0; g--)  // k_delta_write set the non-empty groups' bases
        if (gp->gstart[g + 1] == gp->gstart[g]) {
            gp->fb[g] = gp->fb[g + 1];
            gp->db[g] = gp->db[g + 1];
        }
}

hipError_t launch_sp_plan_edges(hipStream_t st, const void* qpayload, const SpInit& init, SpGroups* gp) {
    hipLaunchKernelGGL(k_sp_plan_edges, dim3(1), dim3(64), 0, st,
                       reinterpret_cast<const skml_dense_header*>(qpayload), init, gp);
    return hipGetLastError();
}
hipError_t launch_sp_plan_groups(hipStream_t st, SpGroups* gp, const uint64_t* sizes, int64_t stride) {
    hipLaunchKernelGGL(k_sp_plan_groups, dim3(1), dim3(64), 0, st, gp, sizes, stride);
    return hipGetLastError();
}
hipError_t launch_sp_plan_delta(hipStream_t st, SpGroups* gp, const uint32_t* hist, const uint32_t* err) {
    hipLaunchKernelGGL(k_sp_plan_delta, dim3(1), dim3(64), 0, st, gp, hist, err);
    return hipGetLastError();
}
hipError_t launch_sp_finalize(hipStream_t st, SpGroups* gp, const uint64_t* tot) {
    hipLaunchKernelGGL(k_sp_finalize, dim3(1), dim3(64), 0, st, gp, tot);
    return hipGetLastError();
}
hipError_t launch_sp_zero_edges(hipStream_t st, const uint64_t* tile_base, int64_t tiles, const SpGroups* gp,
                                uint64_t* flag_words, uint64_t* delta_words) {
    const unsigned grid = (unsigned)((tiles + 1 + kSpThreads - 1) / kSpThreads);
    hipLaunchKernelGGL(k_sp_zero_edges, dim3(grid), dim3(kSpThreads), 0, st, tile_base, tiles, gp, flag_words,
                       delta_words);
    return hipGetLastError();
}

// =============================================================================================
// Decode
// =============================================================================================
// Mask of the bits of word w that lie in unary-flag groups' flag ranges.
__device__ __forceinline__ uint64_t unary_mask(const SpGroups* gp, int64_t w) {
    const int64_t lo = w * 64, hi = lo + 64;
    uint64_t m = 0;
    for (int g = 0; g < gp->G; g++) {
        if (!gp->kind[g]) continue;
        const int64_t a = std::max(lo, gp->fb[g]), b = std::min(hi, gp->fb[g + 1]);
        if (a >= b) continue;
        const int la = (int)(a - lo), lb = (int)(b - lo);
        const uint64_t upto_b = lb >= 64 ? ~0ull : ((1ull << lb) - 1ull);
        m |= upto_b & ~((1ull << la) - 1ull);
    }
    return m;
}

__global__ __launch_bounds__(kSpThreads) void k_unary_count(const uint64_t* __restrict__ words, int64_t nwords,
                                                            const SpGroups* __restrict__ gp,
                                                            uint64_t* __restrict__ tile_sums) {
    __shared__ uint64_t sh[4];
    const int64_t w0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint64_t c = 0;
    for (int j = 0; j < 8; j++) {
        const int64_t w = w0 + j;
        if (w < nwords) c += __popcll(~words[w] & unary_mask(gp, w));
    }
    uint64_t v[1] = {c}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot[0];
}

hipError_t launch_unary_count(hipStream_t st, const uint64_t* flag_words, int64_t nwords,
                              const SpGroups* gp, uint64_t* tile_sums) {
    const int64_t tiles = sp_tiles(nwords, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_unary_count, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, flag_words, nwords, gp,
                       tile_sums);
    return hipGetLastError();
}

// Zero bit #r (over unary groups, in stream order) ends the flag of element
// gstart[g] + r - kind1_before[g]; its position is recorded in end_pos.
__global__ __launch_bounds__(kSpThreads) void k_unary_select(const uint64_t* __restrict__ words, int64_t nwords,
                                                             const SpGroups* __restrict__ gp,
                                                             const uint64_t* __restrict__ tile_base,
                                                             int64_t* __restrict__ end_pos) {
    __shared__ uint64_t sh[4];
    const int64_t w0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint64_t z[8], c = 0;
    for (int j = 0; j < 8; j++) {
        const int64_t w = w0 + j;
        z[j] = w < nwords ? (~words[w] & unary_mask(gp, w)) : 0;
        c += __popcll(z[j]);
    }
    uint64_t v[1] = {c}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    uint64_t r = tile_base[blockIdx.x] + v[0];
    int g = 0;
    for (int j = 0; j < 8; j++) {
        uint64_t m = z[j];
        while (m) {
            const int b = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const int64_t p = (w0 + j) * 64 + b;
            while (g + 1 < gp->G && gp->fb[g + 1] <= p) g++;
            const int64_t e = gp->gstart[g] + (int64_t)r - gp->kind1_before[g];
            if (e < gp->gstart[g + 1]) end_pos[e] = p;  // zeros past the last flag are padding
            r++;
        }
    }
}

hipError_t launch_unary_select(hipStream_t st, const uint64_t* flag_words, int64_t nwords,
                               const SpGroups* gp, const uint64_t* tile_base, int64_t* end_pos) {
    const int64_t tiles = sp_tiles(nwords, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_unary_select, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, flag_words, nwords, gp,
                       tile_base, end_pos);
    return hipGetLastError();
}

// BinaryUtils.getBits (binary/BinaryUtils.java:16-25): nbits (<= 32) read MSB-first.
__device__ __forceinline__ uint32_t get_bits(const uint64_t* words, int64_t nwords, int64_t off, int nbits) {
    if (nbits <= 0) return 0;
    const int64_t w = off >> 6;
    const int sh = (int)(off & 63);
    uint64_t lo = w < nwords ? words[w] : 0;
    uint64_t v = lo >> sh;
    if (sh + nbits > 64) {
        const uint64_t hi = (w + 1) < nwords ? words[w + 1] : 0;
        v |= hi << (64 - sh);
    }
    const uint32_t field = (uint32_t)(v & (nbits == 64 ? ~0ull : ((1ull << nbits) - 1ull)));
    return __brev(field) >> (32 - nbits);
}

// The same read from two words already in registers: off in [0, 64) is relative to w0 and
// off + nbits <= 128.
__device__ __forceinline__ uint32_t bits_of_window(uint64_t w0, uint64_t w1, int off, int nbits) {
    if (nbits <= 0) return 0;
    const uint64_t v = off ? (w0 >> off) | (w1 << (64 - off)) : w0;
    const uint32_t field = (uint32_t)(v & ((1ull << nbits) - 1ull));
    return __brev(field) >> (32 - nbits);
}
__device__ __forceinline__ uint64_t word_or_zero(const uint64_t* __restrict__ words, int64_t nwords, int64_t w) {
    return w < nwords ? words[w] : 0ull;
}

template <typename TN>
__device__ __forceinline__ void narrow_cells(const int32_t* __restrict__ t32, int64_t ncells, TN* __restrict__ tn,
                                             int64_t blk) {
    constexpr uint32_t kTop = (uint32_t)(TN)~(TN)0;
    const int64_t i0 = (blk * kSpThreads + threadIdx.x) * 4;
    if (i0 + 4 <= ncells) {
        const int4 v = *reinterpret_cast<const int4*>(t32 + i0);
        const int32_t e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) tn[i0 + j] = (TN)((uint32_t)e[j] < kTop ? (uint32_t)e[j] : kTop);
    } else {
        for (int64_t i = i0; i < ncells; i++) tn[i] = (TN)((uint32_t)t32[i] < kTop ? (uint32_t)t32[i] : kTop);
    }
}
// The DeltaAdaptive bit lengths of elements i0 .. i0 + 7 (flag stream -> interval -> bits per
// delta) into l[], 0 past n; returns their sum.
__device__ __forceinline__ uint64_t dec_lens8(const uint64_t* __restrict__ fw, int64_t nfw,
                                              const int64_t* __restrict__ end_pos, int64_t n,
                                              const SpGroups* __restrict__ gp, const int64_t* S, int64_t i0,
                                              uint8_t (&l)[8]) {
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) l[j] = 0;
    int gf = i0 < n ? group_of_elem(S, i0) : 0;
    if (i0 + 8 <= n && i0 + 8 <= S[gf + 1] && !gp->kind[gf]) {
        // the common case: 8 fixed-width flags of one group, at most 40 contiguous bits: two word
        // loads instead of one or two per element
        const DeltaShape s = delta_shape(gp, gf);
        const int64_t b0 = gp->fb[gf] + (i0 - S[gf]) * s.nf;
        const int64_t w = b0 >> 6;
        const int sh = (int)(b0 & 63);
        const uint64_t w0 = word_or_zero(fw, nfw, w), w1 = word_or_zero(fw, nfw, w + 1);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int off = sh + j * s.nf;  // < 64 + 40
            const uint32_t f = off < 64 ? bits_of_window(w0, w1, off, s.nf) : bits_of_window(w1, 0ull, off - 64, s.nf);
            const int dl = s.bpi * ((int)f + 1);
            l[j] = (uint8_t)dl;
            sum += dl;
        }
    } else if (i0 < n) {
        int g = gf;
        DeltaShape s = delta_shape(gp, g);
        for (int j = 0; j < 8; j++) {
            const int64_t i = i0 + j;
            if (i >= n) break;
            while (i >= S[g + 1]) s = delta_shape(gp, ++g);
            int iv;
            if (!s.kind) {
                iv = (int)get_bits(fw, nfw, gp->fb[g] + (i - S[g]) * s.nf, s.nf) + 1;
            } else {
                const int64_t start = i == S[g] ? gp->fb[g] : end_pos[i - 1] + 1;
                iv = (int)(end_pos[i] - start);
            }
            const int dl = s.bpi * iv;
            l[j] = (uint8_t)dl;
            sum += dl;
        }
    }
    return sum;
}

__global__ __launch_bounds__(kSpThreads) void k_dec_lens(const uint64_t* __restrict__ fw, int64_t nfw,
                                                         const int64_t* __restrict__ end_pos, int64_t n,
                                                         const SpGroups* __restrict__ gp, uint8_t* __restrict__ dlen,
                                                         uint64_t* __restrict__ tile_sums, int64_t nlens,
                                                         NarrowJob nj) {
    if ((int64_t)blockIdx.x >= nlens) {  // the blocks past the lengths' tiles build the narrow table
        const int64_t b = (int64_t)blockIdx.x - nlens;
        if (nj.width == 8) narrow_cells<uint8_t>(nj.t32, nj.ncells, static_cast<uint8_t*>(nj.tn), b);
        else narrow_cells<uint16_t>(nj.t32, nj.ncells, static_cast<uint16_t*>(nj.tn), b);
        return;
    }
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint64_t sh[4];
    load_starts(gp, S);
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint8_t l[8];
    const uint64_t sum = dec_lens8(fw, nfw, end_pos, n, gp, S, i0, l);
    if (i0 + 8 <= n) {  // one 8-byte store of the lengths
        uint64_t packed = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) packed |= (uint64_t)l[j] << (8 * j);
        *reinterpret_cast<uint64_t*>(dlen + i0) = packed;
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (i0 + j < n) dlen[i0 + j] = l[j];
    }
    uint64_t v[1] = {sum}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot[0];
}

hipError_t launch_dec_lens(hipStream_t st, const uint64_t* flag_words, int64_t n_flag_words,
                           const int64_t* end_pos, int64_t n, const SpGroups* gp, uint8_t* dlen,
                           uint64_t* tile_sums, NarrowJob nj) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) return nj.tn ? launch_narrow_table(st, nj.t32, nj.ncells, nj.width, nj.tn) : hipSuccess;
    if (nj.tn && (reinterpret_cast<uintptr_t>(nj.t32) & 15) != 0) return hipErrorInvalidValue;
    const int64_t nn = nj.tn && nj.ncells > 0 ? sp_tiles(nj.ncells, (int64_t)kSpThreads * 4) : 0;
    hipLaunchKernelGGL(k_dec_lens, dim3((unsigned)(tiles + nn)), dim3(kSpThreads), 0, st, flag_words, n_flag_words,
                       end_pos, n, gp, dlen, tile_sums, tiles, nj);
    return hipGetLastError();
}

// The deltas of elements i0 .. i0 + 7 from their lengths l[] and the first one's bit offset
// `off` in the delta stream, stored to delta[]; returns their sum.
__device__ __forceinline__ uint64_t dec_deltas8(const uint64_t* __restrict__ dw, int64_t ndw, int64_t n, int64_t i0,
                                                int64_t off, const uint8_t (&l)[8], uint32_t* __restrict__ delta) {
    uint64_t dsum = 0;
    if (i0 + 8 <= n) {
        // the thread's 8 deltas are contiguous, at most 256 bits: five words loaded up front, each
        // field taken from the two words it straddles
        const int64_t w = off >> 6;
        uint64_t W[5];
#pragma unroll
        for (int q = 0; q < 5; q++) W[q] = word_or_zero(dw, ndw, w + q);
        int r = (int)(off & 63);
        uint32_t d[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int q = r >> 6, o = r & 63;
            const uint64_t lo = q == 0 ? W[0] : q == 1 ? W[1] : q == 2 ? W[2] : q == 3 ? W[3] : W[4];
            const uint64_t hi = q == 0 ? W[1] : q == 1 ? W[2] : q == 2 ? W[3] : q == 3 ? W[4] : 0ull;
            d[j] = bits_of_window(lo, hi, o, l[j]);
            dsum += d[j];
            r += l[j];
        }
        *reinterpret_cast<uint4*>(delta + i0) = make_uint4(d[0], d[1], d[2], d[3]);
        *reinterpret_cast<uint4*>(delta + i0 + 4) = make_uint4(d[4], d[5], d[6], d[7]);
    } else {
        for (int j = 0; j < 8; j++) {
            if (i0 + j >= n) break;
            const uint32_t d = get_bits(dw, ndw, off, l[j]);
            delta[i0 + j] = d;
            dsum += d;
            off += l[j];
        }
    }
    return dsum;
}

__global__ __launch_bounds__(kSpThreads) void k_dec_deltas(const uint64_t* __restrict__ dw, int64_t ndw,
                                                           const uint8_t* __restrict__ dlen, int64_t n,
                                                           const uint64_t* __restrict__ tile_base,
                                                           uint32_t* __restrict__ delta, uint64_t* __restrict__ tile_sums) {
    __shared__ uint64_t sh[4];
    const int64_t i0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint8_t l[8];
    uint64_t sum = 0;
    if (i0 + 8 <= n) {  // one 8-byte load of the lengths
        const uint64_t pk = *reinterpret_cast<const uint64_t*>(dlen + i0);
#pragma unroll
        for (int j = 0; j < 8; j++) l[j] = (uint8_t)(pk >> (8 * j));
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) l[j] = i0 + j < n ? dlen[i0 + j] : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) sum += l[j];
    uint64_t v[1] = {sum}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    const uint64_t dsum = dec_deltas8(dw, ndw, n, i0, (int64_t)(tile_base[blockIdx.x] + v[0]), l, delta);
    uint64_t v2[1] = {dsum}, tot2[1];
    block_excl_scan<1>(v2, tot2, sh);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot2[0];
}

#ifdef SKML_AB  // A/B form, measured slower (profiles/ab/r05_dec_lookback.txt)
// Lengths and deltas in one pass: each tile (taken in ticket order) computes its lengths in
// registers, takes its first bit offset in the delta stream by a decoupled look-back over the
// tiles' bit totals (the compaction's scheme), and extracts its deltas -- no length array written
// and read back, no tile scan in between.  Extra blocks past the tiles build the narrow table.
__device__ __forceinline__ uint64_t lookback_excl(uint64_t* status, int64_t tile, uint64_t total, int lane) {
    uint64_t excl = 0;
    if (tile == 0) {
        if (lane == 0) st_status(&status[0], kStPre | total);
        return 0;
    }
    if (lane == 0) st_status(&status[tile], kStAgg | total);
    int64_t p = tile - 1;
    while (true) {
        const int64_t idx = p - lane;
        uint64_t sv = idx >= 0 ? ld_status(&status[idx]) : kStPre;  // before tile 0: prefix 0
        while (__ballot((sv & ~kStMask) == 0)) {
            __builtin_amdgcn_s_sleep(1);
            if ((sv & ~kStMask) == 0) sv = ld_status(&status[idx]);
        }
        const uint64_t pre = __ballot((sv & ~kStMask) == kStPre);
        const int stop = pre ? __ffsll((unsigned long long)pre) - 1 : 63;  // nearest prefix
        uint64_t contrib = lane <= stop ? (sv & kStMask) : 0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) contrib += __shfl_xor(contrib, off, 64);
        excl += contrib;
        if (pre) break;
        p -= 64;
    }
    if (lane == 0) st_status(&status[tile], kStPre | (excl + total));
    return excl;
}
__global__ __launch_bounds__(kSpThreads) void k_dec_lens_deltas(const uint64_t* __restrict__ fw, int64_t nfw,
                                                                const int64_t* __restrict__ end_pos, int64_t n,
                                                                const SpGroups* __restrict__ gp,
                                                                const uint64_t* __restrict__ dw, int64_t ndw,
                                                                uint32_t* __restrict__ delta,
                                                                uint64_t* __restrict__ tile_sums, uint64_t* status,
                                                                uint64_t* status2, unsigned* ticket, int64_t nlens,
                                                                NarrowJob nj) {
    if ((int64_t)blockIdx.x >= nlens) {  // the blocks past the tiles build the narrow table
        const int64_t b = (int64_t)blockIdx.x - nlens;
        if (nj.width == 8) narrow_cells<uint8_t>(nj.t32, nj.ncells, static_cast<uint8_t*>(nj.tn), b);
        else narrow_cells<uint16_t>(nj.t32, nj.ncells, static_cast<uint16_t*>(nj.tn), b);
        return;
    }
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint64_t sh[4];
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_excl;
    load_starts(gp, S);
    if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);  // tiles in arrival order
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t i0 = tile * kSpTile + threadIdx.x * 8;
    uint8_t l[8];
    const uint64_t sum = dec_lens8(fw, nfw, end_pos, n, gp, S, i0, l);
    uint64_t v[1] = {sum}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    if (threadIdx.x < 64) {
        const uint64_t excl = lookback_excl(status, tile, tot[0], (int)threadIdx.x);
        if (threadIdx.x == 0) s_excl = excl;
    }
    __syncthreads();
    const uint64_t dsum = dec_deltas8(dw, ndw, n, i0, (int64_t)(s_excl + v[0]), l, delta);
    uint64_t v2[1] = {dsum}, tot2[1];
    block_excl_scan<1>(v2, tot2, sh);
    if (status2) {  // the tiles' delta prefixes too (a second look-back): tile_sums = the exclusive scan
        if (threadIdx.x < 64) {
            const uint64_t excl2 = lookback_excl(status2, tile, tot2[0], (int)threadIdx.x);
            if (threadIdx.x == 0) {
                tile_sums[tile] = excl2;
                if (tile == nlens - 1) tile_sums[nlens] = excl2 + tot2[0];
            }
        }
    } else if (threadIdx.x == 0) {
        tile_sums[tile] = tot2[0];
    }
}

hipError_t launch_dec_lens_deltas(hipStream_t st, const uint64_t* flag_words, int64_t n_flag_words,
                                  const int64_t* end_pos, int64_t n, const SpGroups* gp,
                                  const uint64_t* delta_words, int64_t n_delta_words, uint32_t* delta,
                                  uint64_t* tile_sums, uint64_t* status, NarrowJob nj, bool scan_sums) {
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) return nj.tn ? launch_narrow_table(st, nj.t32, nj.ncells, nj.width, nj.tn) : hipSuccess;
    if (nj.tn && (reinterpret_cast<uintptr_t>(nj.t32) & 15) != 0) return hipErrorInvalidValue;
    // statuses of the bit offsets, the ticket, statuses of the delta prefixes
    hipError_t e = hipMemsetAsync(status, 0, sizeof(uint64_t) * (size_t)(2 * tiles + 2), st);
    if (e != hipSuccess) return e;
    const int64_t nn = nj.tn && nj.ncells > 0 ? sp_tiles(nj.ncells, (int64_t)kSpThreads * 4) : 0;
    hipLaunchKernelGGL(k_dec_lens_deltas, dim3((unsigned)(tiles + nn)), dim3(kSpThreads), 0, st, flag_words,
                       n_flag_words, end_pos, n, gp, delta_words, n_delta_words, delta, tile_sums, status,
                       scan_sums ? status + tiles + 2 : nullptr, reinterpret_cast<unsigned*>(status + tiles), tiles,
                       nj);
    return hipGetLastError();
}
#endif  // SKML_AB


hipError_t launch_dec_deltas(hipStream_t st, const uint64_t* delta_words, int64_t n_delta_words,
                             const uint8_t* dlen, int64_t n, const SpGroups* gp,
                             const uint64_t* tile_base, uint32_t* delta, uint64_t* tile_sums) {
    (void)gp;
    const int64_t tiles = sp_tiles(n, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dec_deltas, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, delta_words, n_delta_words,
                       dlen, n, tile_base, delta, tile_sums);
    return hipGetLastError();
}

// Exclusive delta prefix at each group's first element: tile base + the in-tile partial sum.
__global__ __launch_bounds__(kSpThreads) void k_group_prefix(const uint32_t* __restrict__ delta, int64_t n,
                                                             const SpGroups* __restrict__ gp,
                                                             const uint64_t* __restrict__ tile_base,
                                                             uint64_t* __restrict__ gpre) {
    __shared__ uint64_t sh[4];
    const int g = blockIdx.x;
    const int64_t s0 = gp->gstart[g];
    const int64_t tile = s0 / kSpTile, lo = tile * kSpTile;
    uint64_t sum = 0;
    for (int64_t i = lo + threadIdx.x; i < s0 && i < n; i += kSpThreads) sum += delta[i];
    uint64_t v[1] = {sum}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    if (threadIdx.x == 0) gpre[g] = (s0 < n ? tile_base[tile] : 0) + tot[0];
}

hipError_t launch_group_prefix(hipStream_t st, const uint32_t* delta, int64_t n, const SpGroups* gp, int G,
                               const uint64_t* tile_base, uint64_t* gpre) {
    hipLaunchKernelGGL(k_group_prefix, dim3(G), dim3(kSpThreads), 0, st, delta, n, gp, tile_base, gpre);
    return hipGetLastError();
}

// A narrow image of the int32 MinMax tables for the query: values in [0, 2^W - 1) exactly, the
// rest (the fill of empty cells, and the top code itself) as the sentinel 2^W - 1, which sends the
// query back to the int32 cell.  A valid payload only queries inserted cells, so at W = 8 (binNum
// <= 256) the int32 table is read for bin 255 alone.  At C3 a group's two rows are 2 MB of bytes:
// with each group's tiles on one XCD (k_dec_keys) the gathers hit that XCD's 4 MB L2.
template <typename TN>
__global__ __launch_bounds__(kSpThreads) void k_narrow_table(const int32_t* __restrict__ t32, int64_t ncells,
                                                             TN* __restrict__ tn) {
    narrow_cells<TN>(t32, ncells, tn, blockIdx.x);
}

hipError_t launch_narrow_table(hipStream_t st, const int32_t* t32, int64_t ncells, int width, void* tn) {
    if (ncells <= 0) return hipSuccess;
    if ((reinterpret_cast<uintptr_t>(t32) & 15) != 0) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)sp_tiles(ncells, (int64_t)kSpThreads * 4);
    if (width == 8)
        hipLaunchKernelGGL(k_narrow_table<uint8_t>, dim3(grid), dim3(kSpThreads), 0, st, t32, ncells,
                           static_cast<uint8_t*>(tn));
    else
        hipLaunchKernelGGL(k_narrow_table<uint16_t>, dim3(grid), dim3(kSpThreads), 0, st, t32, ncells,
                           static_cast<uint16_t*>(tn));
    return hipGetLastError();
}

// Workgroup -> tile of k_dec_keys: each tile belongs to the group holding its first element, and
// the tiles of group g go to workgroups b with b % 8 == g % 8, which the dispatcher deals to one XCD
// (speed only: any placement gives the same result).  -1: an idle workgroup.
__device__ __forceinline__ int64_t dec_tile_of_block(const int64_t* S, int G, int64_t b) {
    const int x = (int)(b & 7);
    int64_t j = b >> 3;
    for (int g = x; g < G; g += 8) {
        const int64_t t0 = sp_tiles(S[g], kSpTile), t1 = sp_tiles(S[g + 1], kSpTile);
        if (j < t1 - t0) return t0 + j;
        j -= t1 > t0 ? t1 - t0 : 0;
    }
    return -1;
}

// keys: group-restarted prefix sums of the deltas (Java int wrap); bins: MinMaxSketch.query
// (MinMaxSketch.java:64-73): the row value farthest from zero, the first row on ties.  TN: the
// narrow table's cell type (int32_t: the int32 table itself).  512 threads per 2,048-element tile,
// 4 consecutive elements per thread (16-byte delta loads and key stores).
constexpr int kDecThreads = 512;
static_assert(kDecThreads * 4 == kSpTile, "dec_keys tile");
// MODE 1: the default shape (2 rows), tiles inside one group only (a tile across a group edge
// returns at once): both rows' hashes fixed at compile time by a switch on the group's hash ids,
// 8 gathers in flight per thread, cells as 32-bit offsets.  MODE 0: any shape and any tile, one
// row at a time with a per-lane hash id; it runs the whole grid for other shapes, or only the
// edge tiles (`edges`, at most one per group edge) after a MODE 1 launch.  Keeping the two apart
// keeps MODE 1's registers at what its own code needs.
struct DecEdgeTiles {
    int64_t t[kMaxGroups];
    int n;  // 0: every tile (dec_tile_of_block)
};
// NT: the delta stream and the key / bin stores nontemporal, so they pass L2 without evicting the
// table the gathers read.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));
// One tile of k_dec_keys from its preloaded deltas `d` and base `tb` (tile_base[tile]).  sh: one
// u64 per wave of LDS (the cross-wave prefix); a persistent caller alternates two of them.
template <typename TN, int MODE, bool NT>
__device__ __forceinline__ void dec_keys_tile(int64_t n, const SpGroups* __restrict__ gp,
                                              const uint64_t* __restrict__ gpre, const int32_t* __restrict__ table,
                                              const TN* __restrict__ tnar, int32_t* __restrict__ gkeys,
                                              int32_t* __restrict__ gbins, int nq, void* __restrict__ gbn,
                                              int bn_width, unsigned* __restrict__ err, const int64_t* S,
                                              uint64_t* sh, int64_t tile, const uint32_t (&d)[4], uint64_t tb,
                                              int tid, const RunBoundsOut& rb) {
    const int t = tid, lane = t & 63, w = t >> 6;
    const int64_t i0 = tile * kSpTile + t * 4;
    // the tile's exclusive prefix of the deltas (64-bit: a tile's deltas may pass 2^32)
    const uint64_t own = (uint64_t)d[0] + d[1] + d[2] + d[3];
    const uint64_t inc = wave_incl_u64(own, lane);
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    uint64_t p = tb + inc - own;
#pragma unroll
    for (int j = 0; j < kDecThreads / 64; j++) p += j < w ? sh[j] : 0ull;
    if (i0 >= n) return;
    const uint64_t p_before = p;  // the deltas' prefix through element i0 - 1
    const int zero = gp->zero, rows = gp->rows;
    int32_t key[4], res[4];
    int grp[4];
    if constexpr (MODE == 1) {  // the tile's one group, workgroup-uniform
        const int g = __builtin_amdgcn_readfirstlane(group_of_elem(S, tile * kSpTile));
        const uint64_t gb = gpre[g];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            p += d[j];
            grp[j] = g;
            key[j] = (int32_t)(uint32_t)(p - gb);
            res[j] = zero;
        }
    } else {
        int g = group_of_elem(S, i0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t i = i0 + j;
            if (i < n)
                while (i >= S[g + 1]) g++;
            p += d[j];
            grp[j] = g;
            key[j] = (int32_t)(uint32_t)(p - gpre[g]);
            res[j] = zero;
        }
    }
    if (rb.bounds) {  // the runs' bounds (run_bounds16's rules), from the keys in hand
        const bool rs = rb.info != nullptr;  // Sort.merge's key ranges, else Gradient.sum's tiles
        const int64_t ld = rs ? kRsRanges + 1 : rb.ntiles + 1;
        bool bad = false;
        auto tile_of = [&](int32_t k) -> int64_t {
            if (rs) return (int64_t)(k >> kRsBits);
            return k < 0 ? 0 : std::min<int64_t>((int64_t)(k >> rb.tile_bits), rb.ntiles);
        };
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t i = i0 + j;
            if (i >= n) break;
            const int g = grp[j];
            const int64_t lo = S[g], hi = S[g + 1];
            const int32_t k = key[j];
            const bool first = i == lo;
            // the element before, inside the same run when this one is not its first
            const int32_t prev = j > 0 ? key[j - 1] : (int32_t)(uint32_t)(p_before - gpre[g]);
            bool ok = true;
            if (rs) {  // the one-pass merge's regular input (else the merge rounds run)
                ok = !(k < 0 || k == INT32_MAX || (!first && k <= prev));
                bad |= !ok;
            } else {
                if (k < 0 || (int64_t)k >= rb.dim) bad = true;  // SparseDoubleGradient's bound check
                if (!first && k <= prev) bad = true;            // keys ascend strictly inside a run
            }
            if (ok) {
                const int64_t ti = tile_of(k), pt = first || (rs && prev < 0) ? -1 : tile_of(prev);
                int32_t* b = rb.bounds + (int64_t)g * ld;
                for (int64_t t = pt + 1; t <= ti; t++) b[t] = (int32_t)i;
                if (i == hi - 1) {
                    if (rs) {  // the run's last range ends at the run's end
                        b[ti + 1] = (int32_t)hi;
                        rb.info->tlast1[g] = (int32_t)ti + 1;
                        atomicMax(&rb.info->tmax1, (int32_t)ti + 1);
                    } else {
                        for (int64_t t = ti + 1; t <= rb.ntiles; t++) b[t] = (int32_t)hi;
                    }
                }
            }
        }
        if (bad) atomicOr(rs ? &rb.info->irregular : err, 1u);
    }
    constexpr uint32_t kTop = sizeof(TN) == 4 ? 0u : (uint32_t)(TN)~(TN)0;
    auto cell_of = [&](int j, int r) -> int64_t {
        const int gj = grp[j];
        const int32_t cols = gp->cols[gj];
        return i0 + j < n ? gp->tab_off[gj] + (int64_t)r * cols +
                                java_hash_fm(gp->hash_ids[gj][r], key[j], cols, gp->inv_cols[gj])
                          : -1;
    };
    auto gather = [&](int64_t idx) -> int32_t {
        if constexpr (sizeof(TN) == 4) return idx >= 0 ? table[idx] : zero;
        else return idx >= 0 ? (int32_t)tnar[idx] : zero;
    };
    // MinMaxSketch.query: the strictly farther value wins, ties keep the earlier row
    auto take = [&](int j, int32_t tv) {
        if ((int32_t)((uint32_t)mm_dist(tv, zero) - (uint32_t)mm_dist(res[j], zero)) > 0) res[j] = tv;
    };
    if constexpr (MODE == 1) {
        // both rows' 8 cells hashed, all 8 gathers in flight at once (the query is bound by the
        // gathers' L2 latency); the host runs this form only while every cell index is below
        // 2^32 - 1
        const int g0 = grp[0];  // the tile's one group
        const int64_t tb = gp->tab_off[g0];
        const int32_t cols = gp->cols[g0];
        const double inv = gp->inv_cols[g0];
        const DivU32 dvc = divu32_make((uint32_t)cols);
        const auto dv = [&](uint32_t h) { return java_mod((int32_t)h, cols, dvc); };
        const TN* tnb = tnar + tb;
        const int32_t* t32b = table ? table + tb : nullptr;  // nullptr: tnar is exact (top code = fill)
        uint32_t rel[2][4];
        int32_t tv[2][4];
#pragma unroll
        for (int r = 0; r < 2; r++) {  // a row's 4 gathers leave before the next row is hashed
            const int id = __builtin_amdgcn_readfirstlane(gp->hash_ids[g0][r]);
            const int64_t row0 = (int64_t)r * cols;
            switch (id) {
                case 0: dec_row_cells<0>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                case 1: dec_row_cells<1>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                case 2: dec_row_cells<2>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                case 3: dec_row_cells<3>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                case 4: dec_row_cells<4>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                case 5: dec_row_cells<5>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                case 6: dec_row_cells<6>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
                default: dec_row_cells<7>(key, i0, n, row0, cols, inv, dv, rel[r]); break;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
#ifdef SKML_ABLATE_DEC_GATHER  // timing ablation only (wrong bins): the table gathers priced
                tv[r][j] = (int32_t)(rel[r][j] & 0x3Fu);
                continue;
#endif
                if constexpr (sizeof(TN) == 4) tv[r][j] = t32b[rel[r][j]];
                else tv[r][j] = (int32_t)tnb[rel[r][j]];
            }
        }
        if constexpr (sizeof(TN) < 4) {
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int j = 0; j < 4; j++)  // the top code: the cell's int32 value, or the fill
                    if ((uint32_t)tv[r][j] == kTop) tv[r][j] = t32b ? t32b[rel[r][j]] : gp->fill;
        }
#ifdef SKML_ABLATE_DEC_HASH  // (the wrong cells may be empty ones: keep the bins inside quantValues)
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int j = 0; j < 4; j++) tv[r][j] &= 0x3F;
#endif
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int j = 0; j < 4; j++) take(j, tv[r][j]);
    } else {
        for (int r = 0; r < rows; r++) {
            int64_t idx[4];
            int32_t tv[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                idx[j] = cell_of(j, r);
                tv[j] = gather(idx[j]);
            }
            if constexpr (sizeof(TN) < 4) {
#pragma unroll
                for (int j = 0; j < 4; j++)  // the top code: the cell's int32 value, or the fill
                    if (idx[j] >= 0 && (uint32_t)tv[j] == kTop) tv[j] = table ? table[idx[j]] : gp->fill;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) take(j, tv[j]);
        }
    }
    const bool full = i0 + 4 <= n;
    if (gbn) {  // Gradient.sum's restore: narrow bins (the values come from quantValues in LDS later);
                // a bin outside the values is an error
        bool bad = false;
        uint32_t b[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool ok = res[j] >= 0 && res[j] < nq;
            bad |= !ok && i0 + j < n;
            b[j] = ok ? (uint32_t)res[j] : 0u;
        }
        if (bad) atomicOr(err, 1u);
        if (bn_width == 1) {
            uint8_t* o = static_cast<uint8_t*>(gbn) + i0;
            if (full && (reinterpret_cast<uintptr_t>(o) & 3) == 0) {
                const uint32_t w4 = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
                if constexpr (NT) __builtin_nontemporal_store(w4, reinterpret_cast<uint32_t*>(o));
                else *reinterpret_cast<uint32_t*>(o) = w4;
            } else
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (i0 + j < n) o[j] = (uint8_t)b[j];
        } else {
            uint16_t* o = static_cast<uint16_t*>(gbn) + i0;
            if (full && (reinterpret_cast<uintptr_t>(o) & 7) == 0)
                *reinterpret_cast<uint2*>(o) = make_uint2(b[0] | (b[1] << 16), b[2] | (b[3] << 16));
            else
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (i0 + j < n) o[j] = (uint16_t)b[j];
        }
    }
    if (full && (reinterpret_cast<uintptr_t>(gkeys + i0) & 15) == 0) {
        if constexpr (NT) {
            const i32x4_t kv = {key[0], key[1], key[2], key[3]};
            __builtin_nontemporal_store(kv, reinterpret_cast<i32x4_t*>(gkeys + i0));
        } else {
            *reinterpret_cast<int4*>(gkeys + i0) = make_int4(key[0], key[1], key[2], key[3]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (i0 + j < n) gkeys[i0 + j] = key[j];
    }
    if (gbins) {
        if (full && (reinterpret_cast<uintptr_t>(gbins + i0) & 15) == 0) {
            *reinterpret_cast<int4*>(gbins + i0) = make_int4(res[0], res[1], res[2], res[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (i0 + j < n) gbins[i0 + j] = res[j];
        }
    }
}


template <typename TN, int MODE, bool NT = false>
__global__ __launch_bounds__(kDecThreads) void k_dec_keys(const uint32_t* __restrict__ delta, int64_t n,
                                                          const SpGroups* __restrict__ gp,
                                                          const uint64_t* __restrict__ tile_base,
                                                          const uint64_t* __restrict__ gpre,
                                                          const int32_t* __restrict__ table, const TN* __restrict__ tnar,
                                                          int32_t* __restrict__ gkeys, int32_t* __restrict__ gbins,
                                                          int nq, void* __restrict__ gbn, int bn_width,
                                                          unsigned* __restrict__ err, DecEdgeTiles edges,
                                                          RunBoundsOut rb) {
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint64_t sh[kDecThreads / 64];
    load_starts(gp, S);
    __syncthreads();
    const int64_t tile = edges.n > 0 ? edges.t[blockIdx.x] : dec_tile_of_block(S, gp->G, blockIdx.x);
    if (tile < 0) return;  // workgroup-uniform
    if constexpr (MODE == 1) {
        const int64_t tf = tile * kSpTile, tl = std::min<int64_t>(n, tf + kSpTile) - 1;
        if (group_of_elem(S, tf) != group_of_elem(S, tl)) return;  // an edge tile: the MODE 0 launch
    }
    const int t = threadIdx.x;
    const int64_t i0 = tile * kSpTile + t * 4;
    uint32_t d[4];
    if (i0 + 4 <= n) {
        if constexpr (NT) {
            const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(delta + i0));
            d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        } else {
            const uint4 v = *reinterpret_cast<const uint4*>(delta + i0);
            d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) d[j] = i0 + j < n ? delta[i0 + j] : 0u;
    }
    dec_keys_tile<TN, MODE, NT>(n, gp, gpre, table, tnar, gkeys, gbins, nq, gbn, bn_width, err, S, sh, tile, d,
                                tile_base[tile], (int)threadIdx.x, rb);
}

#ifdef SKML_AB  // A/B form, measured slower (profiles/ab/r05_decp.txt)
// MODE 1 over every inner tile with persistent workgroups: workgroup b walks the tiles that
// dec_tile_of_block deals to its XCD slot (b % 8), and loads the next tile's deltas and base
// while it hashes, gathers and stores the current one.  Same output as k_dec_keys<TN, 1, NT>.
template <typename TN, bool NT>
__global__ __launch_bounds__(kDecThreads) void k_dec_keys_p(const uint32_t* __restrict__ delta, int64_t n,
                                                            const SpGroups* __restrict__ gp,
                                                            const uint64_t* __restrict__ tile_base,
                                                            const uint64_t* __restrict__ gpre,
                                                            const int32_t* __restrict__ table,
                                                            const TN* __restrict__ tnar, int32_t* __restrict__ gkeys,
                                                            int32_t* __restrict__ gbins, int nq, void* __restrict__ gbn,
                                                            int bn_width, unsigned* __restrict__ err, int64_t per_slot,
                                                            RunBoundsOut rb) {
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ uint64_t sh[2][kDecThreads / 64];
    load_starts(gp, S);
    __syncthreads();
    const int64_t slot = blockIdx.x & 7, stride = gridDim.x >> 3;  // gridDim.x: a multiple of 8
    // the j-th tile of this XCD slot's list (-1: past it); edge tiles are skipped (the MODE 0 launch)
    auto tile_at = [&](int64_t j) -> int64_t {
        while (j < per_slot) {
            const int64_t tt = dec_tile_of_block(S, gp->G, j * 8 + slot);
            if (tt < 0) return -1;
            const int64_t tf = tt * kSpTile, tl = std::min<int64_t>(n, tf + kSpTile) - 1;
            if (group_of_elem(S, tf) == group_of_elem(S, tl)) return tt;
            j += stride;  // an edge tile: the next one of this workgroup's walk
        }
        return -1;
    };
    auto load = [&](int64_t tt, uint32_t (&d)[4], uint64_t& tb) {
        const int64_t i0 = tt * kSpTile + threadIdx.x * 4;
        if (i0 + 4 <= n) {
            const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(delta + i0));
            d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) d[j] = i0 + j < n ? delta[i0 + j] : 0u;
        }
        tb = tile_base[tt];
    };
    int64_t j = blockIdx.x >> 3;
    int64_t tile = tile_at(j);
    uint32_t d[4] = {0, 0, 0, 0}, dn[4] = {0, 0, 0, 0};
    uint64_t tb = 0, tbn = 0;
    if (tile >= 0) load(tile, d, tb);
    int par = 0;
    while (tile >= 0) {
        j += stride;
        const int64_t next = tile_at(j);
        if (next >= 0) load(next, dn, tbn);  // in flight while this tile is decoded
        int tid = threadIdx.x;  // thread-derived values rematerialised per tile (hoisted, they cost registers)
        asm volatile("" : "+v"(tid));
        dec_keys_tile<TN, 1, NT>(n, gp, gpre, table, tnar, gkeys, gbins, nq, gbn, bn_width, err, S, sh[par], tile, d,
                                 tb, tid, rb);
        // (dec_keys_tile returns early past n, after its barrier; every thread of the workgroup
        // still runs the same iterations)
        tile = next;
        par ^= 1;
#pragma unroll
        for (int q = 0; q < 4; q++) d[q] = dn[q];
        tb = tbn;
    }
}
#endif  // SKML_AB


hipError_t launch_dec_keys(hipStream_t st, const uint32_t* delta, int64_t n, const SpGroups* gp, const SpGroups& gh,
                           const uint64_t* tile_base, const uint64_t* gpre, const int32_t* table, const void* tnar,
                           int width, int32_t* gkeys, int32_t* gbins, int nq, void* gbn, int bn_width,
                           unsigned* err, RunBoundsOut rb) {
    if (sp_tiles(n, kSpTile) <= 0) return hipSuccess;
    int64_t per[8] = {};  // tiles per XCD slot (dec_tile_of_block)
    for (int g = 0; g < gh.G; g++) {
        const int64_t t0 = sp_tiles(gh.gstart[g], kSpTile), t1 = sp_tiles(gh.gstart[g + 1], kSpTile);
        if (t1 > t0) per[g & 7] += t1 - t0;
    }
    int64_t most = 0;
    for (int x = 0; x < 8; x++) most = std::max(most, per[x]);
    const unsigned grid = (unsigned)(8 * most);
    // MODE 1 over every tile, then MODE 0 over the edge tiles; MODE 0 alone for other shapes, for
    // tables past 2^31 cells (MODE 1's cells are 32-bit offsets and its modulus takes cols <=
    // 2^30), and under SKML_FORM_DEC_ROWS_SERIAL (tests)
    const bool batched = gh.rows == 2 && (table != nullptr || (tnar != nullptr && width < 32)) &&
                         form(SKML_FORM_DEC_ROWS_SERIAL) != 1 &&
                         gh.ncells <= ((int64_t)1 << 31);
    DecEdgeTiles all{}, edges{};
    all.n = 0;
    if (batched) {  // tiles holding a group edge that is not a tile edge
        for (int g = 1; g < gh.G; g++) {
            const int64_t e = gh.gstart[g];
            if (e <= 0 || e >= n || e % kSpTile == 0 || gh.gstart[g + 1] == e) continue;
            const int64_t t = e / kSpTile;
            if (edges.n == 0 || edges.t[edges.n - 1] != t) edges.t[edges.n++] = t;
        }
    }
    // nontemporal streams (decode 0.73 -> 0.71 ms, profiles/ab/r04_sparse_restore_aggregate.txt)
#define SKML_DEC_LAUNCH(TNT, MODE, GRID, TILES, TNPTR)                                                            \
    hipLaunchKernelGGL((k_dec_keys<TNT, MODE>), dim3(GRID), dim3(kDecThreads), 0, st, delta, n, gp, tile_base, gpre, \
                       table, TNPTR, gkeys, gbins, nq, gbn, bn_width, err, TILES, rb)
    // MODE 1 with one workgroup per tile; SKML_FORM_DEC_ROWS_SERIAL = 2 selects persistent
    // workgroups with the next tile's deltas in flight (measured slower at 2^28: restore 0.767
    // vs 0.707 ms, profiles/ab/r05_decp.txt; kept as an A/B form)
#ifdef SKML_AB
    const bool persistent = form(SKML_FORM_DEC_ROWS_SERIAL) == 2;
#define SKML_DEC_PERSISTENT(TNT, TNPTR)                                                          \
        if (batched && persistent) {                                                      \
            static const int res = resident_blocks(k_dec_keys_p<TNT, true>, kDecThreads); \
            const int64_t ps = res > 0 ? std::max<int64_t>(1, std::min<int64_t>(most, res / 8)) : most; \
            hipLaunchKernelGGL((k_dec_keys_p<TNT, true>), dim3((unsigned)(8 * ps)), dim3(kDecThreads), 0, st, delta, \
                               n, gp, tile_base, gpre, table, TNPTR, gkeys, gbins, nq, gbn, bn_width, err, most, rb); \
            if (edges.n > 0) SKML_DEC_LAUNCH(TNT, 0, (unsigned)edges.n, edges, TNPTR);    \
        } else
#else
#define SKML_DEC_PERSISTENT(TNT, TNPTR)
#endif
#define SKML_DEC_WIDTH(TNT, TNPTR)                                                          \
    do {                                                                                  \
        SKML_DEC_PERSISTENT(TNT, TNPTR)                                                   \
        if (batched) {                                                                    \
            hipLaunchKernelGGL((k_dec_keys<TNT, 1, true>), dim3(grid), dim3(kDecThreads), 0, st, delta, n, gp,    \
                               tile_base, gpre, table, TNPTR, gkeys, gbins, nq, gbn, bn_width, err, all, rb); \
            if (edges.n > 0) SKML_DEC_LAUNCH(TNT, 0, (unsigned)edges.n, edges, TNPTR);    \
        } else {                                                                          \
            SKML_DEC_LAUNCH(TNT, 0, grid, all, TNPTR);                                    \
        }                                                                                 \
    } while (0)
    if (width == 8) SKML_DEC_WIDTH(uint8_t, static_cast<const uint8_t*>(tnar));
    else if (width == 16) SKML_DEC_WIDTH(uint16_t, static_cast<const uint16_t*>(tnar));
    else SKML_DEC_WIDTH(int32_t, static_cast<const int32_t*>(nullptr));
#undef SKML_DEC_WIDTH
#undef SKML_DEC_PERSISTENT
#undef SKML_DEC_LAUNCH
    return hipGetLastError();
}

// ---- Gradient.sum of P restored payloads, tiled over the dense sum (skml_sparse_decode_sum_f64) ----
// Each payload is restored (DeltaAdaptive keys + MinMax bins, grouped order, no Sort.merge) into
// scratch; k_agg_bounds records where every (payload, group) run enters each dense tile of
// kAggTile keys; k_agg_tiles then builds each tile of the double sum in LDS, payload after payload
// in payload order (keys are unique within a payload: no atomics), and writes it once.  The dense
// sum is read and written once instead of one random read-modify-write per restored key.
// bounds[g * (ntiles + 1) + t] = first element (payload index) of group g's run with key >=
// t * kAggTile; 0 throughout for an empty group.
#ifdef SKML_AB  // the runs' bounds in passes of their own (SKML_FORM_RUN_BOUNDS = 1); the key query writes them
// Run bounds over 16 consecutive restored keys per thread (four 16-byte loads and the key before
// them; the group's ends in registers): for each element, the ranges between its predecessor's
// range and its own get the element's index, and a run's last element closes its run.
// AGG: Gradient.sum's tiles of kAggTile keys (clamped to ntiles, tail filled to ntiles, keys
// checked against [0, dim)); else Sort.merge's ranges of kRsRange keys (last range + 1 and the
// range maxima into info, INT32_MAX and negative keys flagged irregular).  Both flag a key that
// does not ascend inside its run.
template <bool AGG>
__device__ __forceinline__ void run_bounds16(const int32_t* __restrict__ gk, int64_t n, const int64_t* S,
                                             int32_t* __restrict__ bounds, int64_t ld, int64_t ntiles, int64_t dim,
                                             RsInfo* __restrict__ info, unsigned& bad, int tile_bits = 12) {
    constexpr int kPer = 16;
    const int64_t i0 = ((int64_t)blockIdx.x * kSpThreads + threadIdx.x) * kPer;
    if (i0 >= n) return;
    int32_t key[kPer];
    if (i0 + kPer <= n && (reinterpret_cast<uintptr_t>(gk) & 15) == 0) {
#pragma unroll
        for (int q = 0; q < kPer / 4; q++) {
            const int4 v = *reinterpret_cast<const int4*>(gk + i0 + 4 * q);
            key[4 * q] = v.x, key[4 * q + 1] = v.y, key[4 * q + 2] = v.z, key[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < kPer; e++) key[e] = i0 + e < n ? gk[i0 + e] : 0;
    }
    int32_t prev = i0 > 0 ? gk[i0 - 1] : 0;
    int g = group_of_elem(S, i0);
    int64_t lo = S[g], hi = S[g + 1];
    auto tile_of = [&](int32_t k) -> int64_t {
        if constexpr (AGG) return k < 0 ? 0 : std::min<int64_t>((int64_t)(k >> tile_bits), ntiles);
        else return (int64_t)(k >> kRsBits);
    };
#pragma unroll
    for (int e = 0; e < kPer; e++) {
        const int64_t i = i0 + e;
        if (i >= n) break;
        while (i >= hi) {  // the next non-empty run (rare: at most G - 1 times over all threads)
            g++;
            lo = S[g];
            hi = S[g + 1];
        }
        const int32_t k = key[e];
        const bool first = i == lo;
        bool ok;
        if constexpr (AGG) {
            if (k < 0 || (int64_t)k >= dim) bad = 1;  // SparseDoubleGradient's bound check
            // keys ascend strictly inside a group (the tiles add without atomics)
            if (!first && k <= prev) bad = 1;
            ok = true;
        } else {
            ok = !(k < 0 || k == INT32_MAX || (!first && k <= prev));
            if (!ok) bad = 1;
        }
        if (ok) {
            const int64_t ti = tile_of(k);
            const int64_t pt = first || (!AGG && prev < 0) ? -1 : tile_of(prev);
            int32_t* b = bounds + (int64_t)g * ld;
            for (int64_t t = pt + 1; t <= ti; t++) b[t] = (int32_t)i;
            if (i == hi - 1) {
                if constexpr (AGG) {
                    for (int64_t t = ti + 1; t <= ntiles; t++) b[t] = (int32_t)hi;
                } else {  // the run's last range ends at the run's end
                    b[ti + 1] = (int32_t)hi;
                    info->tlast1[g] = (int32_t)ti + 1;
                    atomicMax(&info->tmax1, (int32_t)ti + 1);
                }
            }
        }
        prev = k;
    }
}

__global__ __launch_bounds__(kSpThreads) void k_agg_bounds(const int32_t* __restrict__ gk, int64_t n,
                                                           const SpGroups* __restrict__ gp, int64_t ntiles, int64_t dim,
                                                           int32_t* __restrict__ bounds, unsigned* __restrict__ err,
                                                           int tile_bits) {
    __shared__ int64_t S[kMaxGroups + 1];
    load_starts(gp, S);
    __syncthreads();
    unsigned bad = 0;
    run_bounds16<true>(gk, n, S, bounds, ntiles + 1, ntiles, dim, nullptr, bad, tile_bits);
    if (bad) atomicOr(err, 1u);
}
hipError_t launch_agg_bounds(hipStream_t st, const int32_t* gk, int64_t n, const SpGroups* gp, int64_t ntiles,
                             int64_t dim, int32_t* bounds, unsigned* err, int tile_bits) {
    if (n <= 0) return hipSuccess;
    const int64_t grid = sp_tiles(sp_tiles(n, 16), kSpThreads);  // 16 keys per thread
    hipLaunchKernelGGL(k_agg_bounds, dim3((unsigned)grid), dim3(kSpThreads), 0, st, gk, n, gp, ntiles, dim, bounds, err,
                       tile_bits);
    return hipGetLastError();
}
#endif  // SKML_AB

// Loads through AggPayload's pointers as global (address space 1) loads.  The pointers come from
// memory (the payload table, copied to LDS or registers), so the compiler would emit flat loads,
// which count on lgkmcnt as well: every later LDS wait would then wait for them too, one memory
// round trip per element batch instead of one per tile.
template <typename T>
__device__ __forceinline__ T gload(const void* p, int64_t i) {
    return ((const __attribute__((address_space(1))) T*)p)[i];
}
constexpr int kAggPB = 8, kAggThreads = 512, kAggLdsValues = 256;
static_assert(kAggPB == kAggVPayloads, "eight payloads per batch in both tile forms");
__device__ __forceinline__ int agg_search32(const int32_t* pre, int n, int j) {  // largest i < n: pre[i] <= j
    int i = 0;
    for (int step = 32; step >= 1; step >>= 1)
        if (i + step < n && pre[i + step] <= j) i += step;
    return i;
}

// Gradient.sum over tiles of kAggTile keys, one wave per payload of a batch (8 waves, 8
// payloads): the wave walks its payload's group runs in this tile (run bounds from k_agg_bounds),
// one lane per element; every wave loads its elements' keys and bins first, then the waves add
// into the LDS tile one after the other in payload order (one barrier per payload).  Up to
// kAggWPer elements per lane are held in registers, a longer payload (a dense form, or a tile far
// denser than the mean) adds the rest in further rounds of its turn.  Each wave marks its
// payload's keys in a presence bitmap of the tile as it adds them (an LDS atomic OR with return):
// a bit already set is a key repeated across the payload's groups, which the reference's
// SparseDoubleGradient constructor rejects (err bit 2).  The general form: any P, G and nq.
constexpr int kAggWPer = 8;
// A persistent grid walks the tiles strided: unit u = b * units-per-workgroup + sub takes tiles
// u, u + units, ..., so all units sweep the sum together (one write front).  Measured and dropped
// (round 4, profiles/ab/r04_sparse_aggregate_tiles.txt): an XCD-aware renumbering (equal: 1,826
// against 1,822 us) and a contiguous share per unit (5.87-5.92 -> 6.60-6.62 ms end to end: 4,096
// separate write fronts).
struct TileWalk {
    int64_t t0, t1, step;
};
__device__ __forceinline__ TileWalk tile_walk(int64_t blk, int64_t nblk, int sub, int nsub, int64_t ntiles) {
    return {blk * nsub + sub, ntiles, nblk * nsub};
}
// The same sweep with each round's tiles dealt to the XCDs in contiguous segments: workgroup b runs
// on XCD b % 8, so within a round XCD x takes tiles [x, x + 1) * (nblk / 8) * nsub and its
// workgroups take consecutive nsub-tile groups of that segment.  Neighbouring tiles share the
// cache lines of the payloads' run pieces (a 128-byte line of keys spans ~5 tiles of a C3 piece,
// of bins ~20): dealt round-robin, each line was fetched into several XCDs' L2 (the sum-tile kernel
// read 3.96 GB per 1.1 GB of elements, profiles/r05m_agg_pmc.json).  One write front per XCD.
__device__ __forceinline__ TileWalk tile_walk_xcd(int64_t blk, int64_t nblk, int sub, int nsub, int64_t ntiles) {
    if (nblk % 8 != 0) return tile_walk(blk, nblk, sub, nsub, ntiles);
    return {(blk % 8) * (nblk / 8) * nsub + (blk / 8) * nsub + sub, ntiles, nblk * nsub};
}
__global__ __launch_bounds__(kAggThreads) void k_agg_tiles_w(const AggPayload* __restrict__ pays, int P,
                                                            int64_t ntiles, int64_t dim, double* __restrict__ out,
                                                            int from_out, double scale, unsigned* __restrict__ err) {
    static_assert(kAggThreads / 64 == kAggPB, "one wave per payload of a batch");
    __shared__ double acc[kAggTile];
    __shared__ uint32_t here[kAggPB][kAggTile / 32];  // presence bits, one bitmap per wave
    __shared__ double qt[kAggPB][kAggLdsValues];
    __shared__ int32_t rb[kAggPB][kMaxGroups + 1];  // run prefix (elements) per group, this tile
    __shared__ int32_t rs[kAggPB][kMaxGroups];      // run start (element index in the payload)
    __shared__ int32_t dfs[kAggPB];                 // dense_form of the batch's payloads
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // a persistent grid: with one batch (P <= kAggPB) the payloads and their quantValues are read
    // once per workgroup instead of once per tile
    const bool one_batch = P <= kAggPB;
    AggPayload a{};
    auto load_batch = [&](int p0, int np) {
        if (wave < np) {
            a = pays[p0 + wave];
            for (int b = lane; b < kAggLdsValues; b += 64)
                if (a.nq <= kAggLdsValues && b < a.nq) qt[wave][b] = gload<double>(a.qv, b);
            if (lane == 0) dfs[wave] = a.dense_form;
        }
    };
    if (one_batch) load_batch(0, P);
    // with one batch, lane g of wave p holds the next tile's run bounds of payload p, group g:
    // loaded one tile ahead, so a tile's element loads wait on one memory round trip, not two
    int32_t nb0 = 0, nb1 = 0;
    auto fetch_bounds = [&](int64_t tt) {
        if (one_batch && wave < P && lane < a.G && tt < ntiles) {
            const int32_t* bd = a.bounds + (int64_t)lane * (ntiles + 1);
            nb0 = gload<int32_t>(bd, tt);
            nb1 = gload<int32_t>(bd, tt + 1);
        }
    };
    const TileWalk tw = tile_walk(blockIdx.x, gridDim.x, 0, 1, ntiles);
    fetch_bounds(tw.t0);
    unsigned bad = 0;
    // The store of tile t - 1 is deferred until tile t's element loads are in flight, and the
    // zeroing of the LDS sum follows it, so both overlap those loads' latency.
    int64_t prev_k0 = -1, prev_nk = 0;
    auto store_prev = [&]() {
        if (prev_k0 >= 0)
            for (int x = threadIdx.x; x < prev_nk; x += kAggThreads)
                out[prev_k0 + x] = scale == 1.0 ? acc[x] : __dmul_rn(acc[x], scale);
    };
    for (int64_t t = tw.t0; t < tw.t1; t += tw.step) {
        const int64_t k0 = t * kAggTile, nk = std::min<int64_t>(kAggTile, dim - k0);
        const int32_t cb0 = nb0, cb1 = nb1;  // this tile's bounds (one batch)
        fetch_bounds(t + tw.step);
        for (int p0 = 0; p0 < P; p0 += kAggPB) {
            const int np = std::min(kAggPB, P - p0);
            __syncthreads();  // the previous batch / tile is done with qt / rb / rs / acc's adds
            if (!one_batch) load_batch(p0, np);
            const bool mine = wave < np;
            if (mine) {
                int32_t len = 0;
                if (lane < a.G) {
                    int32_t b0 = cb0, b1 = cb1;
                    if (!one_batch) {
                        const int32_t* bd = a.bounds + (int64_t)lane * (ntiles + 1);
                        b0 = gload<int32_t>(bd, t);
                        b1 = gload<int32_t>(bd, t + 1);
                    }
                    len = b1 > b0 ? b1 - b0 : 0;
                    rs[wave][lane] = b0;
                }
                int32_t x = len;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int32_t y = __shfl_up(x, off, 64);
                    if (lane >= off) x += y;
                }
                if (lane < kMaxGroups) rb[wave][lane + 1] = x;
                if (lane == 0) rb[wave][0] = 0;
                reinterpret_cast<uint64_t*>(here[wave])[lane] = 0;  // 128 words: two per lane
            }
            __syncthreads();
            // this wave's elements: compact index j = lane + 64 u over the concatenated runs; the run
            // holding j by a walk over the (few) run prefixes
            const int total = mine ? rb[wave][a.G] : 0;
            const bool lds_q = a.nq <= kAggLdsValues;
            // the run holding j: with at most 8 groups, a count of the run ends (held in registers)
            // at or below j; else a binary search of the 65 prefix entries
            int32_t re[8];
#pragma unroll
            for (int q = 0; q < 8; q++) re[q] = rb[wave][q + 1];
            const bool few_g = a.G <= 8;
            auto run_of = [&](int j) -> int {
                if (few_g) {
                    int g = 0;
#pragma unroll
                    for (int q = 0; q < 8; q++) g += re[q] <= j ? 1 : 0;
                    return g;
                }
                return agg_search32(rb[wave], kMaxGroups + 1, j);
            };
            int32_t kk[kAggWPer];
            double vv[kAggWPer];
#pragma unroll
            for (int u = 0; u < kAggWPer; u++) {
                const int j = lane + 64 * u;
                kk[u] = 0;
                vv[u] = 0.0;
                if (j < total) {
                    const int g = run_of(j);
                    const int64_t i = (int64_t)rs[wave][g] + (j - rb[wave][g]);
                    kk[u] = gload<int32_t>(a.gk, i);
                    const uint32_t b = a.bw == 1 ? gload<uint8_t>(a.gb, i) : gload<uint16_t>(a.gb, i);
                    vv[u] = lds_q ? qt[wave][b] : gload<double>(a.qv, b);
                }
            }
            if (p0 == 0) {  // the previous tile leaves, this tile's sum starts (loads in flight)
                store_prev();
                __syncthreads();
                for (int x = threadIdx.x; x < kAggTile; x += kAggThreads)
                    acc[x] = (from_out && x < nk) ? out[k0 + x] : 0.0;
                __syncthreads();
                prev_k0 = k0;
                prev_nk = nk;
            }
            for (int pl = 0; pl < np; pl++) {
                if (wave == pl) {
                    const bool dform = a.dense_form != 0;
                    // a key outside this tile is an error (k_agg_bounds placed it here), and so is a
                    // key already marked in this payload's bitmap: then two lanes of one instruction
                    // may have added it racily, but the sum is refused anyway.  The dense form keeps
                    // |v| > EPS only (SparseDoubleGradient.toDense).
#define SKML_AGG_ADD(K, V)                                                        \
    do {                                                                          \
        const int32_t k_ = (K);                                                   \
        const double v_ = (V);                                                    \
        if (k_ < k0 || (int64_t)k_ >= k0 + nk) {                                  \
            bad |= 1u;                                                            \
        } else {                                                                  \
            const int x_ = (int)(k_ - k0);                                        \
            const uint32_t bit_ = 1u << (x_ & 31);                                \
            if (atomicOr(&here[wave][x_ >> 5], bit_) & bit_) bad |= 2u;           \
            if (!dform || fabs(v_) > 1e-8) acc[x_] += v_;                         \
        }                                                                         \
    } while (0)
#pragma unroll
                    for (int u = 0; u < kAggWPer; u++)
                        if (lane + 64 * u < total) SKML_AGG_ADD(kk[u], vv[u]);
                    for (int j = lane + 64 * kAggWPer; j < total; j += 64) {  // the rest of a long payload
                        const int g = run_of(j);
                        const int64_t i = (int64_t)rs[wave][g] + (j - rb[wave][g]);
                        const uint32_t b = a.bw == 1 ? gload<uint8_t>(a.gb, i) : gload<uint16_t>(a.gb, i);
                        SKML_AGG_ADD(gload<int32_t>(a.gk, i), lds_q ? qt[wave][b] : gload<double>(a.qv, b));
                    }
#undef SKML_AGG_ADD
                }
                __syncthreads();
                if (dfs[pl]) {  // the dense form adds +0.0 elsewhere: -0.0 sums become +0.0
                    for (int x = threadIdx.x; x < kAggTile; x += kAggThreads)
                        if (__double_as_longlong(acc[x]) == (long long)0x8000000000000000ull) acc[x] = 0.0;
                    __syncthreads();
                }
            }
        }
    }
    __syncthreads();
    store_prev();
    if (bad) atomicOr(err, bad);
}

// One wave per tile of kAggVTile keys, staged: lane 8p + g of the wave holds the run piece of
// payload p, group g (P <= 8, G <= 8), the pieces are concatenated payload by payload and each lane
// loads up to kAggWPer * SUB elements of the concatenation.  The wave then writes every element's
// bin to its slot of the wave's stage (one byte per (payload, key)) and sets the slot's presence
// bit; a bit already set is a key repeated inside one payload (err bit 2).  Last, lane l owns keys
// 8l .. 8l + 7 and sums them in registers payload after payload, which is Gradient.sum's order for
// every key, without a read-modify-write of an LDS sum per element.  Persistent waves: each wave
// loads its next tile's run bounds one tile ahead, and stores a tile's sums after the next tile's
// element loads are in flight.  bw == 1 and nq <= 256 for every payload (agg_vtiles_ok).
// SUB > 1: a wave takes SUB consecutive tiles at once (one bounds pair and one round of element
// loads for all of them: run pieces SUB times longer, so fewer L2 requests per element), then
// stages and sums them one tile after the other through the same 4 KB stage.
constexpr int kAggVBits = 9, kAggVTile = 1 << kAggVBits;
static_assert(kAggVTile == 8 * 64, "eight keys per lane");
#ifdef SKML_AB  // A/B forms of the sum tile (SKML_FORM_AGG_TILES 2..5), measured slower than k_agg_rmw
template <int SUB>
__global__ __launch_bounds__(kAggThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_agg_vtiles(
    const AggPayload* __restrict__ pays, int P, int64_t ntiles, int64_t dim, double* __restrict__ out, int from_out,
    double scale, unsigned* __restrict__ err, const int32_t* __restrict__ kbase, const uint8_t* __restrict__ bbase) {
    constexpr int kWaves = kAggThreads / 64;
    constexpr int kPer = kAggWPer * SUB;  // elements per lane held in registers
    // the stage: a bin per (payload, key); between tiles, the transpose of the stored sums
    __shared__ __attribute__((aligned(16))) uint8_t bins[kWaves][kAggPB][kAggVTile];
    static_assert(kAggPB * kAggVTile == kAggVTile * sizeof(double), "a tile of sums fits the stage");
    __shared__ uint32_t here[kWaves][kAggPB][kAggVTile / 32];  // presence bits
    __shared__ double qt[kAggPB][kAggLdsValues];
    __shared__ int32_t pre[kWaves][65];  // the wave's 64 run pieces, scanned
    __shared__ int32_t pk0[kWaves][64];  // each piece's first key (index from kbase)
    __shared__ int32_t pn0[kWaves][64];  // and its first bin (byte from bbase)
    __shared__ AggPayload pl[kAggPB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (threadIdx.x < P * (int)(sizeof(AggPayload) / 8))
        reinterpret_cast<uint64_t*>(pl)[threadIdx.x] = reinterpret_cast<const uint64_t*>(pays)[threadIdx.x];
    __syncthreads();
    if (wave < P)
        for (int b = lane; b < pl[wave].nq; b += 64) qt[wave][b] = gload<double>(pl[wave].qv, b);
    __syncthreads();
    const int pl_l = lane >> 3, g_l = lane & 7;
    const bool lane_on = pl_l < P && g_l < pl[pl_l].G;
    const int32_t* bd = lane_on ? pl[pl_l].bounds + (int64_t)g_l * (ntiles + 1) : nullptr;
    uint8_t(*B)[kAggVTile] = bins[wave];
    uint32_t(*H)[kAggVTile / 32] = here[wave];
    unsigned bad = 0;
    const int64_t nsup = (ntiles + SUB - 1) / SUB;  // super-tiles of SUB tiles
    int32_t nb0 = 0, nb1 = 0;
    auto fetch = [&](int64_t tt) {
        if (lane_on && tt < nsup) {
            nb0 = gload<int32_t>(bd, tt * SUB);
            nb1 = gload<int32_t>(bd, std::min<int64_t>(tt * SUB + SUB, ntiles));
        }
    };
    int64_t prev_k0 = -1, prev_nk = 0;
    // a tile's sums (lane l: keys 8l .. 8l + 7) wait in the stage until the next loads are in
    // flight (the last tile of a super-tile) or the next tile is staged, and leave transposed, so
    // each 16-byte store instruction covers 1 KB of the sum
    double* T = reinterpret_cast<double*>(&B[0][0]);
    auto store_prev = [&](int l) {
        if (prev_k0 < 0) return;
        double* o = out + prev_k0;
        const bool whole = prev_nk == kAggVTile && (reinterpret_cast<uintptr_t>(o) & 15) == 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int x = 128 * q + 2 * l;
            const double2 v = *reinterpret_cast<const double2*>(T + x);
            if (whole) {
                *reinterpret_cast<double2*>(o + x) = v;
            } else {
                if (x < prev_nk) o[x] = v.x;
                if (x + 1 < prev_nk) o[x + 1] = v.y;
            }
        }
        __builtin_amdgcn_wave_barrier();
        prev_k0 = -1;
    };
    const TileWalk tw = tile_walk(blockIdx.x, gridDim.x, wave, kWaves, nsup);
    fetch(tw.t0);
    for (int64_t t = tw.t0; t < tw.t1; t += tw.step) {
        // lane-derived values are recomputed each tile behind an empty asm barrier: hoisted out of
        // the loop (32 element indices, shuffle addresses) they were spilled to scratch
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int64_t K0 = t * SUB << kAggVBits, NK = std::min<int64_t>((int64_t)SUB << kAggVBits, dim - K0);
        const int32_t b0 = nb0, b1 = nb1;
        fetch(t + tw.step);
        const int32_t len = lane_on && b1 > b0 ? b1 - b0 : 0;
        const int32_t x = (int32_t)wave_incl_scan_u32((uint32_t)len);  // DPP scan: no lane-id addresses
        pre[wave][ln + 1] = x;
        if (ln == 0) pre[wave][0] = 0;
        pk0[wave][ln] = lane_on ? pl[pl_l].gk_off + b0 : 0;
        pn0[wave][ln] = lane_on ? pl[pl_l].gb_off + b0 : 0;
        const int total = __builtin_amdgcn_readlane(x, 63);
        __builtin_amdgcn_wave_barrier();
        auto piece_of = [&](int j) -> int {  // largest s < 64 with pre[s] <= j
            int s_ = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1)
                if (pre[wave][s_ + step] <= j) s_ += step;
            return s_;
        };
        // eight elements' pieces first (independent LDS searches), then their loads
        int32_t kk[kPer];
        uint32_t bb[kPer];
#pragma unroll
        for (int u0 = 0; u0 < kPer; u0 += kAggWPer) {
            int spc[kAggWPer];
#pragma unroll
            for (int u = 0; u < kAggWPer; u++) {
                const int j = ln + 64 * (u0 + u);
                spc[u] = piece_of(j < total ? j : 0);
            }
#pragma unroll
            for (int u = 0; u < kAggWPer; u++) {
                const int j = ln + 64 * (u0 + u);
                kk[u0 + u] = INT32_MIN;
                bb[u0 + u] = 0;
                if (j < total) {
                    const int sp = spc[u], p = sp >> 3, d = j - pre[wave][sp];
                    kk[u0 + u] = gload<int32_t>(kbase, (uint32_t)(pk0[wave][sp] + d));
                    bb[u0 + u] = gload<uint8_t>(bbase, (uint32_t)(pn0[wave][sp] + d)) | ((uint32_t)p << 8);
                }
            }
        }
        // one word per element: key offset in the super-tile (bits 0..12), bin (13..20), payload
        // (21..23); ~0u: no element.  A key outside the super-tile is an error (k_agg_bounds placed
        // it here).
        uint32_t ew[kPer];
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            const int64_t off = (int64_t)kk[u] - K0;
            ew[u] = ~0u;
            if (ln + 64 * u < total) {
                if (off < 0 || off >= NK) bad |= 1u;
                else ew[u] = (uint32_t)off | ((bb[u] & 0xFFu) << 13) | ((bb[u] >> 8) << 21);
            }
        }
        store_prev(ln);  // after this super-tile's loads are issued
#pragma unroll 1
        for (int sub = 0; sub < SUB; sub++) {
            const int64_t k0 = K0 + ((int64_t)sub << kAggVBits);
            const int64_t nk = std::min<int64_t>(kAggVTile, dim - k0);
            if (nk <= 0) break;
            int ls = ln;  // (rematerialised per tile, like ln)
            asm volatile("" : "+v"(ls));
            if (sub > 0) store_prev(ls);  // the previous tile's sums leave the stage before it is reused
            reinterpret_cast<uint64_t*>(H)[ls] = 0;  // 8 x 16 words: two per ls
            __builtin_amdgcn_wave_barrier();
            const uint32_t sub_lo = (uint32_t)sub << kAggVBits;
            auto stage = [&](uint32_t w) {  // w: an element word of this tile
                const int p = (int)(w >> 21), xk = (int)((w & 0x1FFFu) - sub_lo);
                B[p][xk] = (uint8_t)(w >> 13);
                const uint32_t bit = 1u << (xk & 31);
                if (atomicOr(&H[p][xk >> 5], bit) & bit) bad |= 2u;  // a key twice in one payload
            };
#pragma unroll
            for (int u = 0; u < kPer; u++)
                if (ew[u] != ~0u && ((ew[u] & 0x1FFFu) >> kAggVBits) == (uint32_t)sub) stage(ew[u]);
            for (int j = 64 * kPer + ls; j < total; j += 64) {  // elements past the registers
                const int sp = piece_of(j), p = sp >> 3, d = j - pre[wave][sp];
                const int64_t off = (int64_t)gload<int32_t>(kbase, (uint32_t)(pk0[wave][sp] + d)) - K0;
                if (off < 0 || off >= NK) {
                    bad |= 1u;
                    continue;
                }
                if ((off >> kAggVBits) == sub)
                    stage((uint32_t)off | ((uint32_t)gload<uint8_t>(bbase, (uint32_t)(pn0[wave][sp] + d)) << 13) |
                          ((uint32_t)p << 21));
            }
            __builtin_amdgcn_wave_barrier();
            // ls l: keys 8l .. 8l + 7, payload after payload
            double acc[8];
#pragma unroll
            for (int i = 0; i < 8; i++)  // a later batch continues the sum
                acc[i] = from_out && 8 * ls + i < nk ? out[k0 + 8 * ls + i] : 0.0;
            for (int p = 0; p < P; p++) {
                const uint32_t m = reinterpret_cast<const uint8_t*>(H[p])[ls];
                const uint2 bw8 = *reinterpret_cast<const uint2*>(&B[p][8 * ls]);
                const bool dform = pl[p].dense_form != 0;
                double v[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const uint32_t b = ((i < 4 ? bw8.x : bw8.y) >> (8 * (i & 3))) & 0xFFu;
                    v[i] = 0.0;
                    if (m & (1u << i)) v[i] = qt[p][b];
                }
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    // the dense form keeps |v| > EPS only (SparseDoubleGradient.toDense), and adds +0.0
                    // elsewhere: a -0.0 sum becomes +0.0
                    if ((m & (1u << i)) && (!dform || fabs(v[i]) > 1e-8)) acc[i] += v[i];
                    if (dform && __double_as_longlong(acc[i]) == (long long)0x8000000000000000ull) acc[i] = 0.0;
                }
            }
            if (scale != 1.0)
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] = __dmul_rn(acc[i], scale);
            __builtin_amdgcn_wave_barrier();  // the stage is read before the sums replace it
#pragma unroll
            for (int q = 0; q < 4; q++)
                *reinterpret_cast<double2*>(T + 8 * ls + 2 * q) = make_double2(acc[2 * q], acc[2 * q + 1]);
            __builtin_amdgcn_wave_barrier();
            prev_k0 = k0;
            prev_nk = nk;
        }
    }
    store_prev(lane);
    if (bad) atomicOr(err, bad);
}

// The staged tiles with the next tile's element loads in flight while this tile is staged and
// summed (software pipelined: run bounds two tiles ahead, elements one tile ahead, the piece tables
// double-buffered in LDS).  Same sums as k_agg_vtiles<1>.
__global__ __launch_bounds__(kAggThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_agg_vtiles_pf(
    const AggPayload* __restrict__ pays, int P, int64_t ntiles, int64_t dim, double* __restrict__ out, int from_out,
    double scale, unsigned* __restrict__ err, const int32_t* __restrict__ kbase, const uint8_t* __restrict__ bbase) {
    constexpr int kWaves = kAggThreads / 64;
    __shared__ __attribute__((aligned(16))) uint8_t bins[kWaves][kAggPB][kAggVTile];
    __shared__ uint32_t here[kWaves][kAggPB][kAggVTile / 32];
    __shared__ double qt[kAggPB][kAggLdsValues];
    __shared__ int32_t pre[2][kWaves][65];
    __shared__ int32_t pk0[2][kWaves][64];
    __shared__ int32_t pn0[2][kWaves][64];
    __shared__ AggPayload pl[kAggPB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (threadIdx.x < P * (int)(sizeof(AggPayload) / 8))
        reinterpret_cast<uint64_t*>(pl)[threadIdx.x] = reinterpret_cast<const uint64_t*>(pays)[threadIdx.x];
    __syncthreads();
    if (wave < P)
        for (int b = lane; b < pl[wave].nq; b += 64) qt[wave][b] = gload<double>(pl[wave].qv, b);
    __syncthreads();
    const int pl_l = lane >> 3, g_l = lane & 7;
    const bool lane_on = pl_l < P && g_l < pl[pl_l].G;
    const int32_t* bd = lane_on ? pl[pl_l].bounds + (int64_t)g_l * (ntiles + 1) : nullptr;
    const int32_t gk_off = lane_on ? pl[pl_l].gk_off : 0, gb_off = lane_on ? pl[pl_l].gb_off : 0;
    uint8_t(*B)[kAggVTile] = bins[wave];
    uint32_t(*H)[kAggVTile / 32] = here[wave];
    unsigned bad = 0;
    int32_t nb0 = 0, nb1 = 0;
    auto fetch = [&](int64_t tt) {
        if (lane_on && tt < ntiles) {
            nb0 = gload<int32_t>(bd, tt);
            nb1 = gload<int32_t>(bd, tt + 1);
        }
    };
    // a tile's piece tables into buffer `buf`; returns its element count
    auto plan = [&](int buf, int32_t b0, int32_t b1, int ln) -> int {
        const int32_t len = lane_on && b1 > b0 ? b1 - b0 : 0;
        const int32_t x = (int32_t)wave_incl_scan_u32((uint32_t)len);
        pre[buf][wave][ln + 1] = x;
        if (ln == 0) pre[buf][wave][0] = 0;
        pk0[buf][wave][ln] = gk_off + b0;
        pn0[buf][wave][ln] = gb_off + b0;
        __builtin_amdgcn_wave_barrier();
        return __builtin_amdgcn_readlane(x, 63);
    };
    auto piece_of = [&](int buf, int j) -> int {  // largest s < 64 with pre[s] <= j
        int s_ = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (pre[buf][wave][s_ + step] <= j) s_ += step;
        return s_;
    };
    auto load = [&](int buf, int total, int ln, int32_t (&kk)[kAggWPer], uint32_t (&bb)[kAggWPer]) {
        int spc[kAggWPer];
#pragma unroll
        for (int u = 0; u < kAggWPer; u++) {
            const int j = ln + 64 * u;
            spc[u] = piece_of(buf, j < total ? j : 0);
        }
#pragma unroll
        for (int u = 0; u < kAggWPer; u++) {
            const int j = ln + 64 * u;
            kk[u] = INT32_MIN;
            bb[u] = 0;
            if (j < total) {
                const int sp = spc[u], d = j - pre[buf][wave][sp];
                kk[u] = gload<int32_t>(kbase, (uint32_t)(pk0[buf][wave][sp] + d));
                bb[u] = gload<uint8_t>(bbase, (uint32_t)(pn0[buf][wave][sp] + d)) | ((uint32_t)(sp >> 3) << 8);
            }
        }
    };
    int64_t prev_k0 = -1, prev_nk = 0;
    double* T = reinterpret_cast<double*>(&B[0][0]);
    auto store_prev = [&](int l) {
        if (prev_k0 < 0) return;
        double* o = out + prev_k0;
        const bool whole = prev_nk == kAggVTile && (reinterpret_cast<uintptr_t>(o) & 15) == 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int x = 128 * q + 2 * l;
            const double2 v = *reinterpret_cast<const double2*>(T + x);
            if (whole) {
                *reinterpret_cast<double2*>(o + x) = v;
            } else {
                if (x < prev_nk) o[x] = v.x;
                if (x + 1 < prev_nk) o[x + 1] = v.y;
            }
        }
        __builtin_amdgcn_wave_barrier();
        prev_k0 = -1;
    };
    const TileWalk tw = tile_walk(blockIdx.x, gridDim.x, wave, kWaves, ntiles);
    int buf = 0, total = 0;
    int32_t kk[kAggWPer], kn[kAggWPer];
    uint32_t bb[kAggWPer], bn[kAggWPer];
    if (tw.t0 < tw.t1) {
        fetch(tw.t0);
        total = plan(0, nb0, nb1, lane);
        load(0, total, lane, kk, bb);
        fetch(tw.t0 + tw.step);
    }
    for (int64_t t = tw.t0; t < tw.t1; t += tw.step) {
        int ln = lane;  // lane-derived values rematerialised per tile (hoisted, they spill)
        asm volatile("" : "+v"(ln));
        const int64_t k0 = t << kAggVBits, nk = std::min<int64_t>(kAggVTile, dim - k0);
        // the next tile: its piece tables and its element loads, in flight while this one is summed
        int total_n = 0;
        const bool more = t + tw.step < tw.t1;
        if (more) {
            total_n = plan(buf ^ 1, nb0, nb1, ln);
            load(buf ^ 1, total_n, ln, kn, bn);
            fetch(t + 2 * tw.step);
        }
        store_prev(ln);
        reinterpret_cast<uint64_t*>(H)[ln] = 0;
        __builtin_amdgcn_wave_barrier();
        auto stage = [&](int p, int32_t k, uint32_t b) {
            if (k < k0 || (int64_t)k >= k0 + nk) {  // k_agg_bounds placed it here: an error
                bad |= 1u;
                return;
            }
            const int xk = (int)(k - k0);
            B[p][xk] = (uint8_t)b;
            const uint32_t bit = 1u << (xk & 31);
            if (atomicOr(&H[p][xk >> 5], bit) & bit) bad |= 2u;  // a key twice in one payload
        };
#pragma unroll
        for (int u = 0; u < kAggWPer; u++)
            if (ln + 64 * u < total) stage((int)(bb[u] >> 8), kk[u], bb[u] & 0xFFu);
        for (int j = 64 * kAggWPer + ln; j < total; j += 64) {  // elements past the registers
            const int sp = piece_of(buf, j), d = j - pre[buf][wave][sp];
            stage(sp >> 3, gload<int32_t>(kbase, (uint32_t)(pk0[buf][wave][sp] + d)),
                  gload<uint8_t>(bbase, (uint32_t)(pn0[buf][wave][sp] + d)));
        }
        __builtin_amdgcn_wave_barrier();
        double acc[8];
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] = from_out && 8 * ln + i < nk ? out[k0 + 8 * ln + i] : 0.0;
        for (int p = 0; p < P; p++) {
            const uint32_t m = reinterpret_cast<const uint8_t*>(H[p])[ln];
            const uint2 bw8 = *reinterpret_cast<const uint2*>(&B[p][8 * ln]);
            const bool dform = pl[p].dense_form != 0;
            double v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t b = ((i < 4 ? bw8.x : bw8.y) >> (8 * (i & 3))) & 0xFFu;
                v[i] = 0.0;
                if (m & (1u << i)) v[i] = qt[p][b];
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if ((m & (1u << i)) && (!dform || fabs(v[i]) > 1e-8)) acc[i] += v[i];
                if (dform && __double_as_longlong(acc[i]) == (long long)0x8000000000000000ull) acc[i] = 0.0;
            }
        }
        if (scale != 1.0)
#pragma unroll
            for (int i = 0; i < 8; i++) acc[i] = __dmul_rn(acc[i], scale);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<double2*>(T + 8 * ln + 2 * q) = make_double2(acc[2 * q], acc[2 * q + 1]);
        __builtin_amdgcn_wave_barrier();
        prev_k0 = k0;
        prev_nk = nk;
        buf ^= 1;
        total = total_n;
#pragma unroll
        for (int u = 0; u < kAggWPer; u++) {
            kk[u] = kn[u];
            bb[u] = bn[u];
        }
    }
    store_prev(lane);
    if (bad) atomicOr(err, bad);
}

#endif  // SKML_AB

// The sum tile itself in LDS: the waves, run pieces and prefetch of k_agg_vtiles_pf, but each
// element is added straight into the wave's tile of doubles (read, add, write back) instead of
// being staged as a bin and summed by a sweep over every (payload, key) slot, which looked up
// quantValues once per (payload, key) for ~10 % present.  The elements of a tile are concatenated
// payload by payload, so each element row (one load instruction) holds ascending payloads by lane
// and later rows never hold an earlier payload; a row is added payload by payload (one masked pass
// per payload present in it, usually one or two), and since a payload holds a key at most once, no
// two lanes of a pass touch the same slot and every key receives its payloads' values in payload
// order -- Gradient.sum's order, with the staged form's roundings.  A key repeated inside a
// payload (presence bit already set) is not added and sets err bit 2.  Dense-form payloads
// (DenseDoubleGradient.plusBy: only |v| > 1e-8 added, and every key's -0.0 sum turned into +0.0)
// sweep the tile once their payload is complete, before any later payload's add.
// BITS: 2^BITS keys per tile (512; 1,024-key tiles on four waves per workgroup, with run pieces
// twice as long, ran 5.7 against 5.0 ms for 8 C3 payloads: 247 VGPRs and half the waves per CU,
// profiles/ab/r05_agg_rmw1k.txt), PER: elements per lane held in registers (a longer tile takes
// the rest row by row).  DENSE: some payload of the launch takes the dense form.
template <int BITS, int WAVES, int PER, bool DENSE>
__global__ __launch_bounds__(64 * WAVES) void k_agg_rmw(
    const AggPayload* __restrict__ pays, int P, int64_t ntiles, int64_t dim, double* __restrict__ out, int from_out,
    double scale, unsigned* __restrict__ err, const int32_t* __restrict__ kbase, const uint8_t* __restrict__ bbase) {
    constexpr int kTile = 1 << BITS, kKeys = kTile / 64;  // keys per lane in the stores
    static_assert(PER == 8 || PER == 16, "piece bytes written as 8 or 16");
    static_assert(kTile / 64 <= 16, "presence bits: 64 words of 16 bits at most");
    __shared__ __attribute__((aligned(16))) double tsum[WAVES][kTile];
    // presence bits of the payload being added: key x at word x % 64, bit x / 64, cleared at each
    // payload (a pass's random keys spread over 64 words: few lanes share a word's atomic)
    __shared__ uint32_t here[WAVES][64];
    __shared__ double qt[kAggPB][kAggLdsValues];
    __shared__ int32_t pre[2][WAVES][65];
    __shared__ int2 pkn[2][WAVES][64];  // piece s's key / bin element bases minus its first index pre[s]
    __shared__ __attribute__((aligned(16))) uint8_t pcs[WAVES][64 * PER];  // piece of element j
    __shared__ AggPayload pl[kAggPB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (threadIdx.x < P * (int)(sizeof(AggPayload) / 8))
        reinterpret_cast<uint64_t*>(pl)[threadIdx.x] = reinterpret_cast<const uint64_t*>(pays)[threadIdx.x];
    __syncthreads();
    for (int q = wave; q < P; q += WAVES)
        for (int b = lane; b < pl[q].nq; b += 64) qt[q][b] = gload<double>(pl[q].qv, b);
    __syncthreads();
    uint32_t dmask = 0;  // dense-form payloads
    if constexpr (DENSE) {
        for (int q = 0; q < P; q++) dmask |= pl[q].dense_form ? 1u << q : 0u;
        dmask = __builtin_amdgcn_readfirstlane(dmask);
    }
    const int pl_l = lane >> 3, g_l = lane & 7;
    const bool lane_on = pl_l < P && g_l < pl[pl_l].G;
    const int32_t* bd = lane_on ? pl[pl_l].bounds + (int64_t)g_l * (ntiles + 1) : nullptr;
    const int32_t gk_off = lane_on ? pl[pl_l].gk_off : 0, gb_off = lane_on ? pl[pl_l].gb_off : 0;
    double* T = tsum[wave];
    uint32_t* H = here[wave];
    unsigned bad = 0;
    int32_t nb0 = 0, nb1 = 0;
    auto fetch = [&](int64_t tt) {
        if (lane_on && tt < ntiles) {
            nb0 = gload<int32_t>(bd, tt);
            nb1 = gload<int32_t>(bd, tt + 1);
        }
    };
    auto plan = [&](int buf, int32_t b0, int32_t b1, int ln) -> int {
        const int32_t len = lane_on && b1 > b0 ? b1 - b0 : 0;
        const int32_t x = (int32_t)wave_incl_scan_u32((uint32_t)len);
        pre[buf][wave][ln + 1] = x;
        if (ln == 0) pre[buf][wave][0] = 0;
        pkn[buf][wave][ln] = make_int2(gk_off + b0 - (x - len), gb_off + b0 - (x - len));
        __builtin_amdgcn_wave_barrier();
        return __builtin_amdgcn_readlane(x, 63);
    };
    auto piece_of = [&](int buf, int j) -> int {  // largest s < 64 with pre[s] <= j
        int s_ = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (pre[buf][wave][s_ + step] <= j) s_ += step;
        return s_;
    };
    // the pieces of the elements held in registers: lane l writes its own piece's number over the
    // piece's elements in pcs (a piece holds ~6-13 elements of a C3 tile: stores, no dependent
    // LDS reads); the loads then read the piece of j = l + 64 u back
    auto load = [&](int buf, int total, int ln, int32_t (&kk)[PER], uint32_t (&bb)[PER]) {
        {
            const int e0 = pre[buf][wave][ln], e1 = min(pre[buf][wave][ln + 1], 64 * PER);
            for (int e = e0; e < e1; e++) pcs[wave][e] = (uint8_t)ln;
            __builtin_amdgcn_wave_barrier();
        }
        int spc[PER];
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int j = ln + 64 * u;
            spc[u] = j < total ? (int)pcs[wave][j] : 0;
        }
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int j = ln + 64 * u;
            kk[u] = INT32_MIN;
            bb[u] = 0;
            if (j < total) {
                const int sp = spc[u];
                const int2 kb = pkn[buf][wave][sp];
                kk[u] = gload<int32_t>(kbase, (uint32_t)(kb.x + j));
                bb[u] = gload<uint8_t>(bbase, (uint32_t)(kb.y + j)) | ((uint32_t)(sp >> 3) << 8);
            }
        }
    };
    int64_t prev_k0 = -1, prev_nk = 0;
    auto store_prev = [&](int l) {  // the previous tile's sums, x scale, 1 KB per store instruction
        if (prev_k0 < 0) return;
        double* o = out + prev_k0;
        const bool whole = prev_nk == kTile && (reinterpret_cast<uintptr_t>(o) & 15) == 0;
#pragma unroll
        for (int q = 0; q < kTile / 128; q++) {
            const int x = 128 * q + 2 * l;
            double2 v = *reinterpret_cast<const double2*>(T + x);
            if (scale != 1.0) {
                v.x = __dmul_rn(v.x, scale);
                v.y = __dmul_rn(v.y, scale);
            }
#ifdef SKML_ABLATE_AGG_STORE  // timing ablation only (no sums written): the sum's stores priced
            if (v.x == 12345.678) o[x] = v.y;
            continue;
#endif
            if (whole) {
                *reinterpret_cast<double2*>(o + x) = v;
            } else {
                if (x < prev_nk) o[x] = v.x;
                if (x + 1 < prev_nk) o[x + 1] = v.y;
            }
        }
        __builtin_amdgcn_wave_barrier();
        prev_k0 = -1;
    };
    // payloads [a, b) complete: a dense-form one among them turns every -0.0 sum of the tile into +0.0
    auto finish = [&](int a, int b, int ln) {
        if constexpr (!DENSE) return;
        if (b <= a || !((dmask >> a) & ((1u << (b - a)) - 1u))) return;  // wave-uniform
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kKeys; i++) {
            double& t = T[kKeys * ln + i];
            if (__double_as_longlong(t) == (long long)0x8000000000000000ull) t = 0.0;
        }
        __builtin_amdgcn_wave_barrier();
    };
    const TileWalk tw = tile_walk_xcd(blockIdx.x, gridDim.x, wave, WAVES, ntiles);
    int buf = 0, total = 0;
    int32_t kk[PER], kn[PER];
    uint32_t bb[PER], bn[PER];
    if (tw.t0 < tw.t1) {
        fetch(tw.t0);
        total = plan(0, nb0, nb1, lane);
        load(0, total, lane, kk, bb);
        fetch(tw.t0 + tw.step);
    }
    for (int64_t t = tw.t0; t < tw.t1; t += tw.step) {
        int ln = lane;  // lane-derived values rematerialised per tile (hoisted, they spill)
        asm volatile("" : "+v"(ln));
        const int64_t k0 = t << BITS, nk = std::min<int64_t>(kTile, dim - k0);
        int total_n = 0;
        const bool more = t + tw.step < tw.t1;
        if (more) {
            total_n = plan(buf ^ 1, nb0, nb1, ln);
            load(buf ^ 1, total_n, ln, kn, bn);
            fetch(t + 2 * tw.step);
        }
        store_prev(ln);
        // the tile's starting sums (a later batch of payloads continues them)
#pragma unroll
        for (int q = 0; q < kKeys / 2; q++) {
            double2 v = make_double2(0.0, 0.0);
            if (from_out) {
                const int x = kKeys * ln + 2 * q;
                if (x < nk) v.x = out[k0 + x];
                if (x + 1 < nk) v.y = out[k0 + x + 1];
            }
            *reinterpret_cast<double2*>(T + kKeys * ln + 2 * q) = v;
        }
        __builtin_amdgcn_wave_barrier();
        int h_for = -1, p_act = 0;  // H's payload; payloads below p_act are complete (wave-uniform)
        const int32_t k0i = (int32_t)k0;  // dim <= 2^31: tile starts fit int32
        // one row of elements (lane l: element j = l + 64 u), payload by payload
        auto add_row = [&](bool act, int p_el, int32_t k, uint32_t b) {
            uint64_t rem = __ballot(act);
            while (rem) {
                const int first = __ffsll((unsigned long long)rem) - 1;
                const int pcur = __builtin_amdgcn_readlane(p_el, first);
                if (pcur != h_for) {  // a new payload: the ones before it are complete
                    finish(p_act, pcur, ln);
                    p_act = pcur;
                    H[ln] = 0u;
                    __builtin_amdgcn_wave_barrier();
                    h_for = pcur;
                }
                const bool mine = act && p_el == pcur;
#ifdef SKML_ABLATE_AGG_RMW  // timing ablation only (wrong sums): the adds into the tile priced
                if (mine && k == INT32_MIN) bad |= 4u;
                rem &= ~__ballot(mine);
                continue;
#endif
                if (mine) {
                    const int32_t xk = k - k0i;
                    if ((uint32_t)xk >= (uint32_t)nk) {  // outside the tile its bounds placed it in: an error
                        bad |= 1u;
                    } else {
                        const uint32_t bit = 1u << (xk >> 6);
                        if (atomicOr(&H[xk & 63], bit) & bit) {
                            bad |= 2u;  // a key twice in one payload
                        } else {
                            const double v = qt[pcur][b];
                            if (!DENSE || !((dmask >> pcur) & 1u) || fabs(v) > 1e-8) T[xk] = T[xk] + v;
                        }
                    }
                }
                rem &= ~__ballot(mine);
            }
        };
#pragma unroll
        for (int u = 0; u < PER; u++)
            add_row(ln + 64 * u < total, (int)(bb[u] >> 8), kk[u], bb[u] & 0xFFu);
        for (int j0 = 64 * PER; j0 < total; j0 += 64) {  // rows past the registers
            const int j = j0 + ln;
            const bool act = j < total;
            int sp = 0;
            int2 kb = make_int2(0, 0);
            if (act) {
                sp = piece_of(buf, j);
                kb = pkn[buf][wave][sp];
            }
            const int32_t k = act ? gload<int32_t>(kbase, (uint32_t)(kb.x + j)) : 0;
            const uint32_t b = act ? gload<uint8_t>(bbase, (uint32_t)(kb.y + j)) : 0u;
            add_row(act, sp >> 3, k, b);
        }
        finish(p_act, P, ln);  // the payloads from the last one seen on
        __builtin_amdgcn_wave_barrier();
        prev_k0 = k0;
        prev_nk = nk;
        buf ^= 1;
        total = total_n;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            kk[u] = kn[u];
            bb[u] = bn[u];
        }
    }
    store_prev(lane);
    if (bad) atomicOr(err, bad);
}

// The staged wave-tile form is the default for payloads of at most 8 groups and 256 quantValues
// (the caller launches it 8 payloads at a time); the wave-per-payload tiles take every other shape
// (SKML_FORM_AGG_TILES forces them for tests).
bool agg_vtiles_ok(int max_groups, int max_nq) {
    return max_groups <= 8 && max_nq <= kAggLdsValues && form(SKML_FORM_AGG_TILES) != 1;
}
int agg_tile_bits(bool vtiles) { return vtiles ? kAggVBits : 12; }

// workgroups of `kern` resident at once on the device (0 if the query fails: one per tile)
template <typename K>
static int resident_workgroups(K kern) {
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    int r = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kAggThreads, 0) == hipSuccess)
        r = std::max(1, per_cu) * prop.multiProcessorCount;
    (void)hipGetLastError();
    return r;
}

hipError_t launch_agg_tiles(hipStream_t st, const AggPayload* pays, int P, int64_t ntiles, int64_t dim, double* out,
                            int from_out, double scale, unsigned* err, bool vtiles, const int32_t* kbase,
                            const uint8_t* bbase, bool any_dense) {
    if (ntiles <= 0) return hipSuccess;
    if (vtiles) {
        if (P < 1 || P > kAggVPayloads) return hipErrorInvalidValue;  // one lane per (payload, group)
        // the default: the sum tile in LDS (k_agg_rmw); the A/B build adds SKML_FORM_AGG_TILES 4 / 5
        // (the staged tiles with and without the next tile's prefetch; 5.57-5.64 against 5.63-5.66
        // ms for 8 C3 payloads, profiles/ab/r05_pf.txt, both slower than k_agg_rmw) and 2 / 3 (four /
        // two staged tiles per wave round)
#ifdef SKML_AB
        const int f = form(SKML_FORM_AGG_TILES);
        if (f >= 2 && f <= 5) {
            if (f == 4) {
                static const int resident_pf = resident_workgroups(k_agg_vtiles_pf);
                const int64_t all = sp_tiles(ntiles, kAggThreads / 64);
                const unsigned grid = (unsigned)(resident_pf <= 0 ? all : std::min<int64_t>(all, resident_pf));
                hipLaunchKernelGGL(k_agg_vtiles_pf, dim3(grid), dim3(kAggThreads), 0, st, pays, P, ntiles, dim, out,
                                   from_out, scale, err, kbase, bbase);
                return hipGetLastError();
            }
#define SKML_VT_LAUNCH(SUB)                                                                                  \
    do {                                                                                                     \
        static const int res = resident_workgroups(k_agg_vtiles<SUB>);                                        \
        const int64_t all = sp_tiles(sp_tiles(ntiles, SUB), kAggThreads / 64);                               \
        const unsigned grid = (unsigned)(res <= 0 ? all : std::min<int64_t>(all, res));                      \
        hipLaunchKernelGGL(k_agg_vtiles<SUB>, dim3(grid), dim3(kAggThreads), 0, st, pays, P, ntiles, dim, out, \
                           from_out, scale, err, kbase, bbase);                                              \
    } while (0)
            if (f == 2) SKML_VT_LAUNCH(4);
            else if (f == 3) SKML_VT_LAUNCH(2);
            else SKML_VT_LAUNCH(1);
#undef SKML_VT_LAUNCH
            return hipGetLastError();
        }
#endif
#define SKML_RMW_LAUNCH(DENSE)                                                                                   \
    do {                                                                                                         \
        static const int res = resident_blocks(k_agg_rmw<kAggVBits, 8, 8, DENSE>, kAggThreads);                   \
        const int64_t all = sp_tiles(ntiles, 8);                                                                 \
        const unsigned grid = (unsigned)(res <= 0 ? all : std::min<int64_t>(all, res));                          \
        hipLaunchKernelGGL((k_agg_rmw<kAggVBits, 8, 8, DENSE>), dim3(grid), dim3(kAggThreads), 0, st, pays, P,   \
                           ntiles, dim, out, from_out, scale, err, kbase, bbase);                                \
    } while (0)
        if (any_dense) SKML_RMW_LAUNCH(true);
        else SKML_RMW_LAUNCH(false);
#undef SKML_RMW_LAUNCH
        return hipGetLastError();
    }
    // persistent: as many workgroups as are resident at once
    static const int resident = resident_workgroups(k_agg_tiles_w);
    const unsigned grid = (unsigned)(resident <= 0 ? ntiles : std::min<int64_t>(ntiles, resident));
    hipLaunchKernelGGL(k_agg_tiles_w, dim3(grid), dim3(kAggThreads), 0, st, pays, P, ntiles, dim, out, from_out, scale,
                       err);
    return hipGetLastError();
}

// live entries (|quantValues[bin]| > 1e-8) of a restored payload, for toAuto's dense / sparse choice
template <typename B>
__global__ __launch_bounds__(kSpThreads) void k_count_live(const B* __restrict__ bins, int64_t n,
                                                           const double* __restrict__ qv,
                                                           unsigned long long* __restrict__ count) {
    uint64_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * kSpThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kSpThreads)
        c += fabs(qv[bins[i]]) > 1e-8 ? 1u : 0u;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, (unsigned long long)c);
}
hipError_t launch_count_live(hipStream_t st, const void* bins, int bw, int64_t n, const double* qv, uint64_t* count) {
    hipError_t e = hipMemsetAsync(count, 0, sizeof(uint64_t), st);
    if (e != hipSuccess || n <= 0) return e;
    const int64_t grid = std::min<int64_t>(sp_tiles(n, kSpThreads * 8), 4096);
    if (bw == 1)
        hipLaunchKernelGGL(k_count_live<uint8_t>, dim3((unsigned)grid), dim3(kSpThreads), 0, st,
                           static_cast<const uint8_t*>(bins), n, qv, reinterpret_cast<unsigned long long*>(count));
    else
        hipLaunchKernelGGL(k_count_live<uint16_t>, dim3((unsigned)grid), dim3(kSpThreads), 0, st,
                           static_cast<const uint16_t*>(bins), n, qv, reinterpret_cast<unsigned long long*>(count));
    return hipGetLastError();
}

// =============================================================================================
// Merge rounds: runs r = [rs[r], rs[r+1]); pairs (2q, 2q+1) merge into the same range, ties
// take the lower run first (Sort.merge scans heads in list order with a strict `<`).
// Each thread produces kMergePer outputs found by a merge-path search.
// =============================================================================================
constexpr int kMergePer = 8;

__device__ __forceinline__ int64_t merge_path(const int32_t* A, int64_t na, const int32_t* B, int64_t nb, int64_t d) {
    int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (A[mid] <= B[d - mid - 1]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// merge_path by one wave: each step probes 64 evenly spaced points of the remaining range (the
// predicate A[i] <= B[d-i-1] is true then false along i), so a run of 13 M keys takes 4 dependent
// global reads instead of 24.
__device__ __forceinline__ int64_t merge_path_wave(const int32_t* A, int64_t na, const int32_t* B, int64_t nb,
                                                   int64_t d, int lane) {
    int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (hi - lo > 64) {
        const int64_t step = (hi - lo + 63) / 64;
        const int64_t i = lo + (int64_t)lane * step;
        const bool p = i < hi && A[i] <= B[d - i - 1];
        const int c = __popcll(__ballot(p));
        if (c == 0) return lo;
        const int64_t nlo = lo + (int64_t)(c - 1) * step + 1, nhi = lo + (int64_t)c * step;
        lo = nlo;
        hi = nhi < hi ? nhi : hi;
    }
    const int64_t i = lo + lane;
    const bool p = i < hi && A[i] <= B[d - i - 1];
    return lo + __popcll(__ballot(p));
}

// The round's run offsets by value (kernel arguments: no dependent loads before the searches).
struct MergeRuns {
    int64_t r[kMaxGroups + 1];
};
constexpr int kMergeTile = 4096, kMergeThreads = 512;  // outputs and threads per merge workgroup
static_assert(kMergeTile == kMergePer * kMergeThreads, "8 outputs per thread");

// Split points of the merge paths at every tile boundary (outputs b * kMergeTile, b in [0, tiles]),
// one wave per boundary: split[b] = how many of the boundary's pair's lower run precede it.
__global__ __launch_bounds__(256) void k_merge_splits(const int32_t* __restrict__ kin, MergeRuns rs, int nruns,
                                                      int64_t total, int64_t nb_bounds, int64_t* __restrict__ split) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nb_bounds) return;
    const int64_t pos = std::min<int64_t>(b * kMergeTile, total);
    int q = 0;  // the pair holding pos: the last even run start <= pos (runs [rs[2q], rs[2q+2]))
    while (2 * q + 2 < nruns && rs.r[2 * q + 2] <= pos) q++;
    const int64_t a0 = rs.r[2 * q], a1 = rs.r[std::min(2 * q + 1, nruns)], b1 = rs.r[std::min(2 * q + 2, nruns)];
    int64_t ia = 0;
    if (pos > a0) ia = pos >= b1 ? a1 - a0 : merge_path_wave(kin + a0, a1 - a0, kin + a1, b1 - a1, pos - a0, lane);
    if (lane == 0) split[b] = ia;
}

// One workgroup per kMergeTile outputs: the tile's end points on its pairs' merge paths come from
// k_merge_splits (or are a pair's ends), the tile's A and B pieces are staged in LDS (coalesced),
// every thread merges 8 outputs from its LDS merge-path split into an LDS output tile, and the tile
// is stored coalesced.
__global__ __launch_bounds__(kMergeThreads) void k_merge_round(const int32_t* __restrict__ kin,
                                                               const int32_t* __restrict__ bin_in,
                                                               int32_t* __restrict__ kout, int32_t* __restrict__ bout,
                                                               MergeRuns rs, int nruns, int64_t total,
                                                               const int64_t* __restrict__ split) {
    __shared__ int32_t sk[kMergeTile], sb[kMergeTile], ok[kMergeTile], ob[kMergeTile];
    const int t = threadIdx.x;
    const int64_t o0 = (int64_t)blockIdx.x * kMergeTile;
    const int64_t o1 = std::min<int64_t>(o0 + kMergeTile, total);
    const int64_t sp0 = split[blockIdx.x], sp1 = split[blockIdx.x + 1];
    int q = 0;
    for (int64_t out = o0; out < o1;) {
        while (2 * q + 2 <= nruns && rs.r[2 * q + 2] <= out) q++;
        const int64_t a0 = rs.r[2 * q];
        const int64_t a1 = rs.r[std::min(2 * q + 1, nruns)];
        const int64_t b1 = rs.r[std::min(2 * q + 2, nruns)];
        const int64_t na = a1 - a0;
        const int64_t end = std::min(o1, b1);
        // a segment starts at the tile start or at a pair start, and ends at the tile end or a pair end
        const int64_t ia0 = out == a0 ? 0 : sp0;
        const int64_t ia1 = end == b1 ? na : sp1;
        const int64_t ib0 = (out - a0) - ia0, ib1 = (end - a0) - ia1;
        const int la = (int)(ia1 - ia0), lb = (int)(ib1 - ib0);
        for (int k = t; k < la + lb; k += kMergeThreads) {
            const int64_t src = k < la ? a0 + ia0 + k : a1 + ib0 + (k - la);
            sk[k] = kin[src];
            sb[k] = bin_in[src];
        }
        __syncthreads();
        const int d = t * kMergePer;
        if (d < la + lb) {
            int ia = (int)merge_path(sk, la, sk + la, lb, d), ib = d - ia;
            const int cnt = std::min(kMergePer, la + lb - d);
            for (int j = 0; j < cnt; j++) {
                const bool takeA = ib >= lb || (ia < la && sk[ia] <= sk[la + ib]);
                const int k = takeA ? ia++ : la + ib++;
                ok[d + j] = sk[k];
                ob[d + j] = sb[k];
            }
        }
        __syncthreads();
        // the merged segment leaves with consecutive lanes on consecutive addresses (a thread's
        // own 8 outputs would be 32-byte strided stores)
        for (int k = t; k < la + lb; k += kMergeThreads) {
            kout[out + k] = ok[k];
            bout[out + k] = ob[k];
        }
        __syncthreads();
        out = end;
    }
}

hipError_t launch_merge_round(hipStream_t st, const int32_t* kin, const int32_t* bin_in, int32_t* kout,
                              int32_t* bout, const int64_t* run_start, int nruns, int64_t total, int64_t* split) {
    if (total <= 0) return hipSuccess;
    if (nruns > kMaxGroups) return hipErrorInvalidValue;
    MergeRuns rs{};
    for (int i = 0; i <= nruns; i++) rs.r[i] = run_start[i];
    const int64_t tiles = sp_tiles(total, kMergeTile), nb = tiles + 1;
    hipLaunchKernelGGL(k_merge_splits, dim3((unsigned)sp_tiles(nb, 4)), dim3(256), 0, st, kin, rs, nruns, total, nb,
                       split);
    hipLaunchKernelGGL(k_merge_round, dim3((unsigned)tiles), dim3(kMergeThreads), 0, st, kin, bin_in, kout, bout, rs,
                       nruns, total, split);
    return hipGetLastError();
}

// ---- Sort.merge in one pass over key ranges (the regular case) ----
// Sort.merge (util/Sort.java:362-379) takes the smallest head of the G runs each step (ties to the
// lower run).  When every run ascends strictly, no key repeats across runs and every key lies in
// [0, INT32_MAX), that is the ascending order of all keys, so an element's output index is the
// number of keys smaller than its own.  k_rs_bounds records where each run enters every range of
// kRsRange keys (and flags a run that does not ascend or a key outside the range); k_rs_merge marks
// one range's keys in an LDS bitmap, scans the bitmap's popcounts, and sends each element to the
// range's base + its rank among the set bits, with its bin or quantValues[bin].  A repeated key
// (a bit already set) flags the input too, and the host then runs the pairwise merge rounds,
// which follow Sort.merge for any input.  Regular C3 payloads: one pass instead of three rounds.
#ifdef SKML_AB  // the ranges' bounds in a pass of their own (SKML_FORM_RUN_BOUNDS = 1); the key query writes them
__global__ __launch_bounds__(kSpThreads) void k_rs_bounds(const int32_t* __restrict__ gk, int64_t n,
                                                          const SpGroups* __restrict__ gp, int32_t* __restrict__ bounds,
                                                          RsInfo* __restrict__ info) {
    __shared__ int64_t S[kMaxGroups + 1];
    load_starts(gp, S);
    __syncthreads();
    unsigned bad = 0;
    run_bounds16<false>(gk, n, S, bounds, kRsRanges + 1, 0, 0, info, bad);
    if (bad) atomicOr(&info->irregular, 1u);
}

#endif  // SKML_AB

template <typename V>
__device__ __forceinline__ V rs_value(int32_t b, const V* lut, const double* qv, int nq, bool lds, unsigned& bad) {
    if constexpr (std::is_same<V, int32_t>::value) {
        return b;
    } else {
        if (b < 0 || b >= nq) {
            bad = 1;
            return (V)0;
        }
        return lds ? lut[b] : (V)qv[b];
    }
}

constexpr int kRsThreads = 256, kRsBatch = 4, kRsLut = 1024;
static_assert(kRsWords == kRsThreads, "one bitmap word per thread");
#ifdef SKML_AB  // the one-pass merge without the pipelining (SKML_FORM_RS_ROUNDS = 2), measured slower
template <typename V>
__global__ __launch_bounds__(kRsThreads) void k_rs_merge(const int32_t* __restrict__ gk, const int32_t* __restrict__ gb,
                                                         const SpGroups* __restrict__ gp,
                                                         const int32_t* __restrict__ bounds, RsInfo* __restrict__ info,
                                                         int32_t* __restrict__ keys_out, V* __restrict__ out,
                                                         const double* __restrict__ qv, int nq) {
    constexpr int kLut = std::is_same<V, int32_t>::value ? 1 : kRsLut;
    __shared__ uint32_t bm[kRsWords];
    __shared__ int32_t slot[kRsRange];  // the bin of the key at each offset of the range
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ int64_t lo_s[kMaxGroups];
    __shared__ int32_t pre[kMaxGroups + 1];
    __shared__ int64_t obase;
    __shared__ uint32_t wsum[kRsThreads / 64];
    __shared__ V lut[kLut];
    if (info->irregular) return;  // workgroup-uniform: the merge rounds run instead
    const int tmax = info->tmax1 - 1;
    const int G = gp->G, t_ = threadIdx.x, lane = t_ & 63, w = t_ >> 6;
    load_starts(gp, S);
    const bool lds = !std::is_same<V, int32_t>::value && nq <= kLut;
    if (lds)
        for (int b = t_; b < nq; b += kRsThreads) lut[b] = (V)qv[b];
    constexpr int64_t ld = kRsRanges + 1;
    unsigned bad = 0;
    // wave 0, lane g < G: run g's last range, and the bounds of this workgroup's next range,
    // loaded one range ahead so a range waits on one memory round trip (its elements), not two
    const int tl = (w == 0 && lane < G) ? info->tlast1[lane] - 1 : -1;  // -1: an empty run
    int32_t nlo = 0, nhi = 0;
    auto fetch = [&](int64_t tt) {
        if (tl >= 0 && tt <= tl) {
            nlo = bounds[(int64_t)lane * ld + tt];
            nhi = bounds[(int64_t)lane * ld + tt + 1];
        }
    };
    if (w == 0 && lane < G) fetch(blockIdx.x);
    for (int64_t t = blockIdx.x; t <= tmax; t += gridDim.x) {
        const int32_t clo = nlo, chi = nhi;
        if (w == 0 && lane < G) fetch(t + gridDim.x);
        __syncthreads();  // S / lut loaded; the previous range is done with bm / slot / pre
        if (w == 0) {  // lane g: run g's piece of this range
            int64_t lo = 0, len = 0, before = 0;
            if (lane < G) {
                const int64_t s0 = S[lane], s1 = S[lane + 1];
                lo = s1;
                int64_t hi = s1;
                if (tl >= 0 && t <= tl) {
                    lo = clo;
                    hi = chi;
                }
                before = lo - s0;
                len = hi - lo;
                lo_s[lane] = lo;
            }
            int64_t x = len;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            if (lane < kMaxGroups) pre[lane + 1] = (int32_t)x;
            if (lane == 0) pre[0] = 0;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) before += __shfl_xor(before, off, 64);
            if (lane == 0) obase = before;
        }
        bm[t_] = 0;
        __syncthreads();
        const int cnt = pre[G];
        if (cnt == 0) continue;  // workgroup-uniform
        // the run holding j: with at most 8 runs a count of the run ends (in registers) at or below
        // j, else a binary search of the prefix
        int32_t re[8];
#pragma unroll
        for (int q = 0; q < 8; q++) re[q] = q + 1 <= G ? pre[q + 1] : INT32_MAX;
        auto run_of = [&](int j) -> int {
            if (G <= 8) {
                int g = 0;
#pragma unroll
                for (int q = 0; q < 8; q++) g += re[q] <= j ? 1 : 0;
                return g;
            }
            return agg_search32(pre, G, j);
        };
        // pass 1: the range's keys into the bitmap, their bins into the offset slots (4 loads of
        // each in flight per thread)
        for (int j0 = 0; j0 < cnt; j0 += kRsThreads * kRsBatch) {
            int32_t kk[kRsBatch], bb[kRsBatch];
#pragma unroll
            for (int u = 0; u < kRsBatch; u++) {
                const int j = j0 + u * kRsThreads + t_;
                kk[u] = -1;
                if (j < cnt) {
                    const int g = run_of(j);
                    const int64_t i = lo_s[g] + (j - pre[g]);
                    kk[u] = gk[i];
                    bb[u] = gb[i];
                }
            }
#pragma unroll
            for (int u = 0; u < kRsBatch; u++) {
                if (kk[u] < 0) continue;
                const uint32_t off = (uint32_t)kk[u] & (kRsRange - 1), bit = 1u << (off & 31);
                if (atomicOr(&bm[off >> 5], bit) & bit) bad = 1;  // a repeated key
                slot[off] = bb[u];
            }
        }
        __syncthreads();
        // pass 2: thread t_ owns bitmap word t_, i.e. the keys t * kRsRange + 32 t_ + [0, 32): its
        // set bits go out in key order from its exclusive popcount prefix
        const uint32_t word = bm[t_];
        const uint32_t own = __popc(word);
        uint32_t inc = own;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if (lane >= off) inc += y;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t run = inc - own;
        for (int q = 0; q < w; q++) run += wsum[q];
        int64_t o = obase + run;
        const int32_t kbase = (int32_t)(t * kRsRange) + 32 * t_;
        for (uint32_t m = word; m; m &= m - 1, o++) {
            const int b = __ffs(m) - 1;
            keys_out[o] = kbase + b;
            out[o] = rs_value<V>(slot[32 * t_ + b], lut, qv, nq, lds, bad);
        }
    }
    if (bad) atomicOr(&info->irregular, 2u);
}

#endif  // SKML_AB

// Sort.merge in one pass, software pipelined: while range t is marked, scanned and emitted, the
// element loads of the workgroup's next range are in flight (its piece table computed one range
// ahead into the other half of a double buffer, its run bounds fetched two ranges ahead).  The
// emission is coalesced: each thread lists its word's set offsets at their ranks in `ord`, and
// output j of the range is written by thread j % 256 (the per-bit stores of k_rs_merge write 64
// scattered words per instruction).  Values restores hold the bins as 16-bit slots (checked
// against nq on load: a bin outside quantValues flags the input, as rs_value does), so `ord` fits
// in the LDS the int32 slots took.  Same output and irregular-input flags as k_rs_merge.
// NARROW (values restores with at most 256 quantValues): byte slots and a 256-entry table, 26-27 KB
// of LDS instead of 37-41 KB, so 5-6 workgroups per CU hold ranges in flight instead of 3-4.
template <typename V, bool NARROW = false>
__global__ __launch_bounds__(kRsThreads) void k_rs_merge_pf(const int32_t* __restrict__ gk,
                                                            const int32_t* __restrict__ gb,
                                                            const SpGroups* __restrict__ gp,
                                                            const int32_t* __restrict__ bounds,
                                                            RsInfo* __restrict__ info, int32_t* __restrict__ keys_out,
                                                            V* __restrict__ out, const double* __restrict__ qv, int nq) {
    constexpr bool kBins = std::is_same<V, int32_t>::value;  // int32 bins out: any table value
    static_assert(!(kBins && NARROW), "narrow slots hold quantValues indices only");
    constexpr int kLut = kBins ? 1 : NARROW ? 256 : kRsLut;
    using ST = typename std::conditional<kBins, int32_t, typename std::conditional<NARROW, uint8_t, uint16_t>::type>::type;
    __shared__ uint32_t bm[kRsWords];
    __shared__ ST slot[kRsRange];
    __shared__ uint16_t ord[kRsRange];  // the range's set offsets in key order
    __shared__ int64_t S[kMaxGroups + 1];
    __shared__ int64_t lo_s[3][kMaxGroups];
    __shared__ int32_t pre[3][kMaxGroups + 1];
    __shared__ int64_t obase[3];
    __shared__ uint32_t wsum[kRsThreads / 64];
    __shared__ V lut[kLut];
    if (info->irregular) return;  // workgroup-uniform: the merge rounds run instead
    const int tmax = info->tmax1 - 1;
    const int G = gp->G, t_ = threadIdx.x, lane = t_ & 63, w = t_ >> 6;
    load_starts(gp, S);
    const bool lds = !std::is_same<V, int32_t>::value && nq <= kLut;
    if (lds)
        for (int b = t_; b < nq; b += kRsThreads) lut[b] = (V)qv[b];
    constexpr int64_t ld = kRsRanges + 1;
    unsigned bad = 0;
    const int tl = (w == 0 && lane < G) ? info->tlast1[lane] - 1 : -1;  // -1: an empty run
    int32_t nlo = 0, nhi = 0;
    auto fetch = [&](int64_t tt) {
        if (tl >= 0 && tt <= tl) {
            nlo = bounds[(int64_t)lane * ld + tt];
            nhi = bounds[(int64_t)lane * ld + tt + 1];
        }
    };
    // wave 0: range tt's run pieces into buffer b (lane g < G: run g), from bounds (clo, chi)
    auto plan = [&](int b, int64_t tt, int32_t clo, int32_t chi) {
        int64_t lo = 0, len = 0, before = 0;
        if (lane < G) {
            const int64_t s0 = S[lane], s1 = S[lane + 1];
            lo = s1;
            int64_t hi = s1;
            if (tl >= 0 && tt <= tl) {
                lo = clo;
                hi = chi;
            }
            before = lo - s0;
            len = hi - lo;
            lo_s[b][lane] = lo;
        }
        int64_t x = len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane < kMaxGroups) pre[b][lane + 1] = (int32_t)x;
        if (lane == 0) pre[b][0] = 0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) before += __shfl_xor(before, off, 64);
        if (lane == 0) obase[b] = before;
    };
    auto run_of = [&](int b, int j) -> int {
        if (G <= 8) {
            int g = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) g += (q + 1 <= G && pre[b][q + 1] <= j) ? 1 : 0;
            return g;
        }
        return agg_search32(pre[b], G, j);
    };
    auto load = [&](int b, int32_t (&kk)[kRsBatch], int32_t (&bb)[kRsBatch]) {
        const int cnt = pre[b][G];
        // the run ends in registers once per range (at most 8 runs), not one LDS read per run and element
        int32_t re[8];
#pragma unroll
        for (int q = 0; q < 8; q++) re[q] = q + 1 <= G ? pre[b][q + 1] : INT32_MAX;
#pragma unroll
        for (int u = 0; u < kRsBatch; u++) {
            const int j = u * kRsThreads + t_;
            kk[u] = -1;
            bb[u] = 0;
            if (j < cnt) {
                int g = 0;
                if (G <= 8) {
#pragma unroll
                    for (int q = 0; q < 8; q++) g += re[q] <= j ? 1 : 0;
                } else {
                    g = run_of(b, j);
                }
                const int64_t i = lo_s[b][g] + (j - pre[b][g]);
                kk[u] = gk[i];
                bb[u] = gb[i];
            }
        }
    };
    int32_t kc[kRsBatch], bc[kRsBatch], kn[kRsBatch], bn[kRsBatch];
    int buf = 0;
    const int64_t t0 = blockIdx.x;
    if (t0 <= tmax) {
        if (w == 0) {
            fetch(t0);
            plan(0, t0, nlo, nhi);
            fetch(t0 + gridDim.x);
        }
        __syncthreads();
        load(0, kc, bc);
    }
    for (int64_t t = t0; t <= tmax; t += gridDim.x) {
        const bool more = t + gridDim.x <= tmax;
        const int nbuf = buf == 2 ? 0 : buf + 1;
        if (w == 0 && more) {  // the next range's piece table, from the bounds fetched one range ago
            plan(nbuf, t + gridDim.x, nlo, nhi);
            fetch(t + 2 * (int64_t)gridDim.x);
        }
        bm[t_] = 0;
        __syncthreads();  // bm zeroed, the next plan visible, the previous emit done with bm / slot
        if (more) load(nbuf, kn, bn);  // in flight while this range is marked and emitted
        const int cnt = pre[buf][G];
        // pass 1: this range's keys into the bitmap, their bins into the offset slots
        auto to_slot = [&](int32_t b) -> ST {
            if constexpr (kBins) {
                return b;
            } else {
                if (b < 0 || b >= nq) {  // quantValues[bin] out of bounds: the rounds report it
                    bad = 1;
                    return 0;
                }
                return (ST)b;
            }
        };
#pragma unroll
        for (int u = 0; u < kRsBatch; u++) {
            if (kc[u] < 0) continue;
            const uint32_t off = (uint32_t)kc[u] & (kRsRange - 1), bit = 1u << (off & 31);
            if (atomicOr(&bm[off >> 5], bit) & bit) bad = 1;  // a repeated key
            slot[off] = to_slot(bc[u]);
        }
        for (int j = kRsThreads * kRsBatch + t_; j < cnt; j += kRsThreads) {  // past the registers
            const int g = run_of(buf, j);
            const int64_t i = lo_s[buf][g] + (j - pre[buf][g]);
            const int32_t k = gk[i];
            const uint32_t off = (uint32_t)k & (kRsRange - 1), bit = 1u << (off & 31);
            if (atomicOr(&bm[off >> 5], bit) & bit) bad = 1;
            slot[off] = to_slot(gb[i]);
        }
        __syncthreads();
        if (cnt > 0) {  // workgroup-uniform
            // pass 2: thread t_ owns bitmap word t_: its set bits go out in key order from its
            // exclusive popcount prefix
            const uint32_t word = bm[t_];
            const uint32_t own = __popc(word);
            uint32_t inc = own;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if (lane >= off) inc += y;
            }
            if (lane == 63) wsum[w] = inc;
            __syncthreads();
            uint32_t run = inc - own;
            for (int q = 0; q < w; q++) run += wsum[q];
            for (uint32_t m = word; m; m &= m - 1, run++) ord[run] = (uint16_t)(32 * t_ + __ffs(m) - 1);
            __syncthreads();
            const int64_t ob = obase[buf];
            const int32_t kbase = (int32_t)(t * kRsRange);
            for (int j = t_; j < cnt; j += kRsThreads) {
                const int off = ord[j];
                keys_out[ob + j] = kbase + off;
                out[ob + j] = rs_value<V>((int32_t)slot[off], lut, qv, nq, lds, bad);
            }
        }
        buf = nbuf;
#pragma unroll
        for (int u = 0; u < kRsBatch; u++) {
            kc[u] = kn[u];
            bc[u] = bn[u];
        }
    }
    if (bad) atomicOr(&info->irregular, 2u);
}

hipError_t launch_rs_merge(hipStream_t st, const int32_t* gk, const int32_t* gb, int64_t n, const SpGroups* gp,
                           int32_t* bounds, RsInfo* info, int32_t* keys_out, void* out, int vkind, const double* qv,
                           int nq, bool bounds_ready) {
    if (n <= 0) return hipSuccess;
    const int64_t bgrid = sp_tiles(sp_tiles(n, 16), kSpThreads);
#ifdef SKML_AB
    if (!bounds_ready)
        hipLaunchKernelGGL(k_rs_bounds, dim3((unsigned)bgrid), dim3(kSpThreads), 0, st, gk, n, gp, bounds, info);
#else
    (void)bgrid;
    if (!bounds_ready) return hipErrorInvalidValue;  // the key query writes the ranges' bounds
#endif
    // persistent workgroups over the key ranges up to the largest key (read on the device): as many
    // as are resident at once (4 per CU), fewer for small inputs
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(sp_tiles(n, 4096), 1), 1024);
    // the pipelined form unless SKML_FORM_RS_ROUNDS = 2 asks for the plain one-pass kernel
#define SKML_RS_LAUNCH(K)                                                                                         \
    do {                                                                                                          \
        if (vkind == 0)                                                                                           \
            hipLaunchKernelGGL(K<int32_t>, dim3(grid), dim3(kRsThreads), 0, st, gk, gb, gp, bounds, info, keys_out, \
                               static_cast<int32_t*>(out), qv, nq);                                              \
        else if (vkind == 1)                                                                                      \
            hipLaunchKernelGGL(K<float>, dim3(grid), dim3(kRsThreads), 0, st, gk, gb, gp, bounds, info, keys_out,  \
                               static_cast<float*>(out), qv, nq);                                                \
        else                                                                                                      \
            hipLaunchKernelGGL(K<double>, dim3(grid), dim3(kRsThreads), 0, st, gk, gb, gp, bounds, info, keys_out, \
                               static_cast<double*>(out), qv, nq);                                               \
    } while (0)
#ifdef SKML_AB
    if (form(SKML_FORM_RS_ROUNDS) == 2) SKML_RS_LAUNCH(k_rs_merge);
    else
#endif
#ifndef SKML_RS_NARROW
#define SKML_RS_NARROW 1  // A/B builds: 0 keeps 16-bit slots for every values restore
#endif
    if (SKML_RS_NARROW && vkind != 0 && nq >= 1 && nq <= 256) {
        // the grid is what the CUs hold of the narrow form (5-6 per CU), fewer for small inputs
        static const int res_f = resident_blocks(k_rs_merge_pf<float, true>, kRsThreads);
        static const int res_d = resident_blocks(k_rs_merge_pf<double, true>, kRsThreads);
        const int res = vkind == 1 ? res_f : res_d;
        const unsigned g2 = (unsigned)std::min<int64_t>(std::max<int64_t>(sp_tiles(n, 4096), 1), res > 0 ? res : 1024);
        if (vkind == 1)
            hipLaunchKernelGGL((k_rs_merge_pf<float, true>), dim3(g2), dim3(kRsThreads), 0, st, gk, gb, gp, bounds, info,
                               keys_out, static_cast<float*>(out), qv, nq);
        else
            hipLaunchKernelGGL((k_rs_merge_pf<double, true>), dim3(g2), dim3(kRsThreads), 0, st, gk, gb, gp, bounds, info,
                               keys_out, static_cast<double*>(out), qv, nq);
    } else {
        SKML_RS_LAUNCH(k_rs_merge_pf);
    }
#undef SKML_RS_LAUNCH
    return hipGetLastError();
}

// values[bins[i]] (SparseVectorCompressor.java:118-126) from the double quantValues LUT
// (Quantizer.getValues, times any timesBy factors): as fp32, or the doubles themselves.
template <typename T>
__global__ __launch_bounds__(kSpThreads) void k_bin_values(const int32_t* __restrict__ bins, int64_t n,
                                                           const double* __restrict__ qv, int B,
                                                           T* __restrict__ vals, unsigned* __restrict__ err) {
    __shared__ T lut[4096];
    const bool lds = B <= 4096;
    if (lds) {
        for (int b = threadIdx.x; b < B; b += kSpThreads) lut[b] = (T)qv[b];
        __syncthreads();
    }
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * kSpThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kSpThreads) {
        const int b = bins[i];
        const bool ok = b >= 0 && b < B;  // Java: quantValues[bin] out of bounds throws
        bad |= !ok;
        vals[i] = !ok ? (T)0 : lds ? lut[b] : (T)qv[b];
    }
    if (bad) atomicOr(err, 1u);
}

template <typename T>
hipError_t launch_bin_values_t(hipStream_t st, const int32_t* bins, int64_t n, const double* qvalues, int B, T* vals,
                               unsigned* err) {
    if (n <= 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>(sp_tiles(n, kSpThreads * 4), 4096);
    hipLaunchKernelGGL(k_bin_values<T>, dim3((unsigned)grid), dim3(kSpThreads), 0, st, bins, n, qvalues, B, vals, err);
    return hipGetLastError();
}
hipError_t launch_bin_values(hipStream_t st, const int32_t* bins, int64_t n, const double* qvalues, int B,
                             float* vals, unsigned* err) {
    return launch_bin_values_t<float>(st, bins, n, qvalues, B, vals, err);
}
hipError_t launch_bin_values64(hipStream_t st, const int32_t* bins, int64_t n, const double* qvalues, int B,
                               double* vals, unsigned* err) {
    return launch_bin_values_t<double>(st, bins, n, qvalues, B, vals, err);
}

// =============================================================================================
// HuffmanEncoder of each MinMaxSketch table (binary/HuffmanEncoder.java:88-124, used by
// MinMaxSketch.writeObject, MinMaxSketch.java:88-97): per-group value histograms, then the
// MSB-first code stream of all tables (codes from the host-built tree, one LUT per group).
// Symbol index: the value itself for bins in [0, B), B for the table's fill value.
// =============================================================================================
constexpr int kHuffLdsBins = 4097;

__device__ __forceinline__ int huff_sym(int32_t v, int B) { return (v >= 0 && v < B) ? v : B; }

__global__ __launch_bounds__(kSpThreads) void k_huff_hist(const int32_t* __restrict__ table,
                                                          const SpGroups* __restrict__ gp, int B,
                                                          uint32_t* __restrict__ hist) {
    __shared__ uint32_t H[kHuffLdsBins];
    const int g = blockIdx.y;
    if (gp->gstart[g + 1] == gp->gstart[g]) return;  // empty group: null sketch
    const int64_t cells = (int64_t)gp->rows * gp->cols[g], base = gp->tab_off[g];
    const bool lds = B + 1 <= kHuffLdsBins;
    uint32_t* gh = hist + (size_t)g * (B + 1);
    if (lds) {
        for (int j = threadIdx.x; j <= B; j += kSpThreads) H[j] = 0;
        __syncthreads();
    }
    for (int64_t i = (int64_t)blockIdx.x * kSpThreads + threadIdx.x; i < cells; i += (int64_t)gridDim.x * kSpThreads) {
        const int sidx = huff_sym(table[base + i], B);
        if (lds) atomicAdd(&H[sidx], 1u);
        else atomicAdd(&gh[sidx], 1u);
    }
    if (lds) {
        __syncthreads();
        for (int j = threadIdx.x; j <= B; j += kSpThreads)
            if (H[j]) atomicAdd(&gh[j], H[j]);
    }
}

hipError_t launch_huff_hist(hipStream_t st, const int32_t* table, const SpGroups* gp, int G, int B,
                            int64_t max_cells, uint32_t* hist) {
    const int64_t gx = std::max<int64_t>(1, std::min<int64_t>(sp_tiles(max_cells, kSpThreads * 8), 256));
    hipLaunchKernelGGL(k_huff_hist, dim3((unsigned)gx, (unsigned)G), dim3(kSpThreads), 0, st, table, gp, B, hist);
    return hipGetLastError();
}

// group owning table cell i: the last g with tab_off[g] <= i (empty groups share the next offset)
__device__ __forceinline__ void load_tab_offs(const SpGroups* gp, int64_t* T) {
    for (int j = threadIdx.x; j <= kMaxGroups; j += blockDim.x) T[j] = j < gp->G ? gp->tab_off[j] : INT64_MAX;
}
__device__ __forceinline__ int group_of_cell(const int64_t* T, int64_t i) {
    int g = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
        if (T[g + step] <= i) g += step;
    return g;
}

// lut[g * (B+1) + sym] = (numBits << 32) | bits
__global__ __launch_bounds__(kSpThreads) void k_huff_lens(const int32_t* __restrict__ table, int64_t ncells,
                                                          const SpGroups* __restrict__ gp, int B,
                                                          const uint64_t* __restrict__ lut,
                                                          uint64_t* __restrict__ tile_sums) {
    __shared__ int64_t T[kMaxGroups + 1];
    __shared__ uint64_t sh[4];
    load_tab_offs(gp, T);
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint64_t sum = 0;
    for (int j = 0; j < 8; j++) {
        const int64_t i = i0 + j;
        if (i >= ncells) break;
        const int g = group_of_cell(T, i);
        sum += lut[(size_t)g * (B + 1) + huff_sym(table[i], B)] >> 32;
    }
    uint64_t v[1] = {sum}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot[0];
}

hipError_t launch_huff_lens(hipStream_t st, const int32_t* table, int64_t ncells, const SpGroups* gp, int B,
                            const uint64_t* lut, uint64_t* tile_sums) {
    const int64_t tiles = sp_tiles(ncells, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_huff_lens, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, table, ncells, gp, B, lut,
                       tile_sums);
    return hipGetLastError();
}

constexpr int kHuffWin = (kSpTile * 32 + 63) / 64 + 2;

__global__ __launch_bounds__(kSpThreads) void k_huff_write(const int32_t* __restrict__ table, int64_t ncells,
                                                           const SpGroups* __restrict__ gp, int B,
                                                           const uint64_t* __restrict__ lut,
                                                           const uint64_t* __restrict__ tile_base,
                                                           uint64_t* __restrict__ words, int64_t* __restrict__ gbit) {
    __shared__ int64_t T[kMaxGroups + 1];
    __shared__ uint64_t sh[4];
    __shared__ uint64_t win[kHuffWin];
    load_tab_offs(gp, T);
    for (int j = threadIdx.x; j < kHuffWin; j += kSpThreads) win[j] = 0;
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kSpTile + threadIdx.x * 8;
    uint64_t code[8];
    uint64_t sum = 0;
    for (int j = 0; j < 8; j++) {
        const int64_t i = i0 + j;
        code[j] = 0;
        if (i >= ncells) continue;
        const int g = group_of_cell(T, i);
        code[j] = lut[(size_t)g * (B + 1) + huff_sym(table[i], B)];
        sum += code[j] >> 32;
    }
    uint64_t v[1] = {sum}, tot[1];
    block_excl_scan<1>(v, tot, sh);
    const uint64_t base = tile_base[blockIdx.x];
    const int64_t w0 = (int64_t)(base >> 6) << 6;
    uint64_t off = base + v[0];
    for (int j = 0; j < 8; j++) {
        const int64_t i = i0 + j;
        if (i >= ncells) break;
        const int g = group_of_cell(T, i);
        if (i == T[g]) gbit[g] = (int64_t)off;  // first cell of group g
        const int nb = (int)(code[j] >> 32);
        lds_put_bits(win, (int64_t)off - w0, (uint32_t)code[j], nb);
        off += nb;
    }
    __syncthreads();
    flush_window(win, (int64_t)base, tot[0], words);
}

hipError_t launch_huff_write(hipStream_t st, const int32_t* table, int64_t ncells, const SpGroups* gp, int B,
                             const uint64_t* lut, const uint64_t* tile_base, uint64_t* words, int64_t* gbit) {
    const int64_t tiles = sp_tiles(ncells, kSpTile);
    if (tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_huff_write, dim3((unsigned)tiles), dim3(kSpThreads), 0, st, table, ncells, gp, B, lut,
                       tile_base, words, gbit);
    return hipGetLastError();
}

// =============================================================================================
// HuffmanEncoder.decode (binary/HuffmanEncoder.java:127-166) of MinMaxSketch tables, the read
// side of GroupedMinMaxSketch.readObject.  The stream has no sync points, so it is decoded
// speculatively in parallel: every segment of kHuffSeg bits starts decoding at its nominal
// boundary; rounds of k_huff_sync then restart each segment at the true end of its predecessor
// until no start changes (prefix codes resynchronise within a few codewords); the per-segment
// symbol counts are scanned into table offsets and k_huff_write decodes again, writing cells.
// Codes are read MSB-first from BitSet words (bit i = word[i >> 6] >> (i & 63)), looked up in a
// 2^12-entry table per group, and codes longer than 12 bits finish with a walk over tree nodes.
// =============================================================================================
__device__ __forceinline__ uint32_t huff_peek32(const uint64_t* __restrict__ w, int64_t nwords, int64_t pos) {
    const int64_t wi = pos >> 6;
    const int sh = (int)(pos & 63);
    const uint64_t w0 = wi < nwords ? w[wi] : 0ull;  // BitSet.toLongArray trimmed zero words: read 0
    const uint64_t w1 = wi + 1 < nwords ? w[wi + 1] : 0ull;
    const uint64_t lo = sh ? ((w0 >> sh) | (w1 << (64 - sh))) : w0;
    return __brev((uint32_t)lo);  // stream bit `pos` becomes bit 31
}

__device__ __forceinline__ int32_t huff_symbol(const HuffDecGroup& gr, const uint64_t* __restrict__ words,
                                               const int2* __restrict__ lut, const int4* __restrict__ nodes,
                                               int64_t& pos) {
    const uint64_t* w = words + gr.word0;
    const uint32_t u = huff_peek32(w, gr.nwords, pos);
    const int2 e = lut[(size_t)gr.lut_row * kHuffLutSize + (u >> (32 - kHuffLutBits))];
    if (e.y > 0) {
        pos += e.y;
        return e.x;
    }
    int node = e.x;  // a code longer than the table: walk the tree from depth kHuffLutBits
    int64_t p = pos + kHuffLutBits;
    int4 nd = nodes[node];
    while (nd.x >= 0) {
        const uint32_t b = huff_peek32(w, gr.nwords, p) >> 31;
        p++;
        node = b ? nd.y : nd.x;
        nd = nodes[node];
    }
    pos = p;
    return nd.z;
}

__global__ __launch_bounds__(256) void k_huff_spec(int nseg, const HuffSeg* __restrict__ segs,
                                                   const HuffDecGroup* __restrict__ grp,
                                                   const uint64_t* __restrict__ words, const int2* __restrict__ lut,
                                                   const int4* __restrict__ nodes, int64_t* __restrict__ start,
                                                   int64_t* __restrict__ end, uint64_t* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    const HuffSeg sg = segs[i];
    int64_t pos = start[i];
    uint64_t c = 0;
    if (!sg.last) {
        const HuffDecGroup gr = grp[sg.g];
        while (pos < sg.lim) {
            (void)huff_symbol(gr, words, lut, nodes, pos);
            c++;
        }
    }
    end[i] = pos;
    cnt[i] = c;
}

__global__ __launch_bounds__(256) void k_huff_sync(int nseg, const HuffSeg* __restrict__ segs,
                                                   const HuffDecGroup* __restrict__ grp,
                                                   const uint64_t* __restrict__ words, const int2* __restrict__ lut,
                                                   const int4* __restrict__ nodes, int64_t* __restrict__ start,
                                                   const int64_t* __restrict__ end_in, int64_t* __restrict__ end_out,
                                                   uint64_t* __restrict__ cnt, unsigned* __restrict__ changed) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    const HuffSeg sg = segs[i];
    const int64_t ns = sg.first ? start[i] : end_in[i - 1];
    if (ns == start[i]) {
        end_out[i] = end_in[i];
        return;
    }
    start[i] = ns;
    int64_t pos = ns;
    uint64_t c = 0;
    if (!sg.last) {
        const HuffDecGroup gr = grp[sg.g];
        while (pos < sg.lim) {
            (void)huff_symbol(gr, words, lut, nodes, pos);
            c++;
        }
    }
    end_out[i] = pos;
    cnt[i] = c;
    atomicOr(changed, 1u);
}

// off: exclusive scan of cnt (global); a group's cells start at its first segment's offset.
__global__ __launch_bounds__(256) void k_huff_write(int nseg, const HuffSeg* __restrict__ segs,
                                                    const HuffDecGroup* __restrict__ grp,
                                                    const uint64_t* __restrict__ words, const int2* __restrict__ lut,
                                                    const int4* __restrict__ nodes, const int64_t* __restrict__ start,
                                                    const uint64_t* __restrict__ off, int32_t* __restrict__ table,
                                                    unsigned* __restrict__ err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    const HuffSeg sg = segs[i];
    const HuffDecGroup gr = grp[sg.g];
    const int64_t o = (int64_t)(off[i] - off[gr.seg0]);
    const int64_t m = sg.last ? gr.size - o : (int64_t)(off[i + 1] - off[i]);
    if (o < 0 || m < 0 || o + m > gr.size) {
        atomicOr(err, 1u);
        return;
    }
    int32_t* dst = table + gr.tab_off + o;
    int64_t pos = start[i];
    for (int64_t k = 0; k < m; k++) dst[k] = huff_symbol(gr, words, lut, nodes, pos);
}

__global__ __launch_bounds__(256) void k_fill_i32(int32_t* __restrict__ dst, int64_t n, int32_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = v;
}

hipError_t launch_huff_spec(hipStream_t st, int nseg, const HuffSeg* segs, const HuffDecGroup* grp,
                            const uint64_t* words, const int2* lut, const int4* nodes, int64_t* start, int64_t* end,
                            uint64_t* cnt) {
    if (nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_huff_spec, dim3((nseg + 255) / 256), dim3(256), 0, st, nseg, segs, grp, words, lut, nodes,
                       start, end, cnt);
    return hipGetLastError();
}
hipError_t launch_huff_sync(hipStream_t st, int nseg, const HuffSeg* segs, const HuffDecGroup* grp,
                            const uint64_t* words, const int2* lut, const int4* nodes, int64_t* start,
                            const int64_t* end_in, int64_t* end_out, uint64_t* cnt, unsigned* changed) {
    if (nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_huff_sync, dim3((nseg + 255) / 256), dim3(256), 0, st, nseg, segs, grp, words, lut, nodes,
                       start, end_in, end_out, cnt, changed);
    return hipGetLastError();
}
hipError_t launch_huff_decode_write(hipStream_t st, int nseg, const HuffSeg* segs, const HuffDecGroup* grp,
                                    const uint64_t* words, const int2* lut, const int4* nodes, const int64_t* start,
                                    const uint64_t* off, int32_t* table, unsigned* err) {
    if (nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_huff_write, dim3((nseg + 255) / 256), dim3(256), 0, st, nseg, segs, grp, words, lut, nodes,
                       start, off, table, err);
    return hipGetLastError();
}
hipError_t launch_fill_i32(hipStream_t st, int32_t* dst, int64_t n, int32_t v) {
    if (n <= 0) return hipSuccess;
    const int64_t g = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill_i32, dim3((unsigned)g), dim3(256), 0, st, dst, n, v);
    return hipGetLastError();
}

}  // namespace skml
