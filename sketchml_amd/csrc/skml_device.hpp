// skml_device.hpp -- device helpers shared by the CDNA4 kernels (gfx950, wave64).
//
// Keys: fp32 values are sorted as "total-order keys" (sign-magnitude -> unsigned), which is
// exactly the order java.util.Arrays.sort(double[]) uses (-0.0 before 0.0; NaN never sorted:
// HeapQuantileSketch.update rejects it, HeapQuantileSketch.java:75-76).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "skml_internal.h"

namespace skml {

__device__ __forceinline__ uint32_t f2key(uint32_t b) {
    return b ^ ((uint32_t)((int32_t)b >> 31) | 0x80000000u);
}
__device__ __forceinline__ uint32_t key2f(uint32_t k) {
    return k ^ ((k >> 31) ? 0x80000000u : 0xFFFFFFFFu);
}
__device__ __forceinline__ bool is_nan_bits(uint32_t b) { return (b & 0x7FFFFFFFu) > 0x7F800000u; }

// ------------------------------------------------------------------------------------------
// Cross-lane exchange: value held by lane ^ M.  Picks the cheapest gfx950 primitive per mask:
// DPP quad_perm / row_mirror / row_half_mirror / row_ror:8 when the pattern stays inside a
// 16-lane row, ds_swizzle (bit mode) inside 32 lanes, ds_bpermute otherwise.
// ------------------------------------------------------------------------------------------
// SKML_XLANE_SWIZZLE (A/B builds): every exchange inside 32 lanes through ds_swizzle, i.e. the
// LDS pipe, instead of a DPP move on the VALU (the leaf is VALU-issue bound); SKML_XLANE_SWZ: the
// same for the masks M whose bit is set (bit M), DPP for the rest.
#ifdef SKML_XLANE_SWIZZLE
#define SKML_XLANE_SWZ 0xFFFFFFFFu
#endif
#ifndef SKML_XLANE_SWZ
#define SKML_XLANE_SWZ 0u
#endif
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    int x = (int)v;
    if constexpr (M < 32 && ((SKML_XLANE_SWZ >> M) & 1u))
        return (uint32_t)__builtin_amdgcn_ds_swizzle(x, (M << 10) | 0x1F);
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);
    else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x1B, 0xF, 0xF, true);
    else if constexpr (M == 7) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true);
    else if constexpr (M == 15) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, true);
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true);
    else if constexpr (M < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle(x, (M << 10) | 0x1F);
    else {
        int lane = (int)__lane_id();
        return (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ M) << 2, x);
    }
}
template <int M>
__device__ __forceinline__ float lane_xor(float v) {
    return __uint_as_float(lane_xor<M>(__float_as_uint(v)));
}
template <int M>
__device__ __forceinline__ double lane_xor(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = lane_xor<M>((uint32_t)b), hi = lane_xor<M>((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Inclusive wave-64 prefix sum of 32-bit values in 6 DPP adds (row shifts 1, 2, 4, 8 inside each
// 16-lane row, then row_bcast:15 / row_bcast:31 carry the row totals): a dependent chain of VALU
// ops instead of six LDS-pipe shuffles (ds_bpermute, ~100+ cycles each).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1 (row edge reads 0)
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
    return (uint32_t)x;
}

// Wave-64 reductions (min / max / or of uint32) with the same DPP steps: the result is valid in
// lane 63, which the callers use for their one LDS atomic per wave.
template <int OP>  // 0 min, 1 max, 2 or
__device__ __forceinline__ uint32_t dpp_op(uint32_t a, uint32_t b) {
    return OP == 0 ? (a < b ? a : b) : OP == 1 ? (a > b ? a : b) : (a | b);
}
template <int OP>
__device__ __forceinline__ uint32_t wave_reduce_u32_lane63(uint32_t v) {
    constexpr int id = OP == 0 ? -1 : 0;  // identity in the lanes a shift leaves without a source
    int x = (int)v;
    x = (int)dpp_op<OP>((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(id, x, 0x111, 0xF, 0xF, false));
    x = (int)dpp_op<OP>((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(id, x, 0x112, 0xF, 0xF, false));
    x = (int)dpp_op<OP>((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(id, x, 0x114, 0xF, 0xF, false));
    x = (int)dpp_op<OP>((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(id, x, 0x118, 0xF, 0xF, false));
    x = (int)dpp_op<OP>((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(id, x, 0x142, 0xA, 0xF, false));
    x = (int)dpp_op<OP>((uint32_t)x, (uint32_t)__builtin_amdgcn_update_dpp(id, x, 0x143, 0xC, 0xF, false));
    return (uint32_t)x;
}

// Sort elements are uint32 total-order keys, raw floats or raw doubles.  Floats and doubles
// compare with v_min/v_max(/v_med3)_f32/f64, which on gfx950 order -0.0 before 0.0 like
// Arrays.sort (tools/ubench/zero_minmax.hip) and drop NaN, so the leaf flags NaN from a class
// test at load (k_leaf2).  fbits: the float's bit pattern.
__device__ __forceinline__ uint32_t elem_fbits(uint32_t k) { return key2f(k); }
__device__ __forceinline__ uint32_t elem_fbits(float f) { return __float_as_uint(f); }
template <typename T>
__device__ __forceinline__ T elem_of_fbits(uint32_t b);
template <>
__device__ __forceinline__ uint32_t elem_of_fbits<uint32_t>(uint32_t b) { return f2key(b); }
template <>
__device__ __forceinline__ float elem_of_fbits<float>(uint32_t b) { return __uint_as_float(b); }
// compare-exchange selector: med3(a, b, sel_of(false)) = min, med3(a, b, sel_of(true)) = max
template <typename T>
__device__ __forceinline__ T sel_of(bool upper);
template <>
__device__ __forceinline__ uint32_t sel_of<uint32_t>(bool upper) { return upper ? 0xFFFFFFFFu : 0u; }
template <>
__device__ __forceinline__ float sel_of<float>(bool upper) {
    return __uint_as_float(upper ? 0x7F800000u : 0xFF800000u);
}
template <>
__device__ __forceinline__ double sel_of<double>(bool upper) {
    return __longlong_as_double(upper ? 0x7FF0000000000000LL : (long long)0xFFF0000000000000ULL);
}

// How each element type is held in LDS / global node buffers (float for keys and floats,
// double for doubles) and converted.
template <typename T>
struct Elem {  // uint32 total-order keys
    using S = float;
    __device__ static __forceinline__ S to_s(uint32_t k) { return __uint_as_float(key2f(k)); }
    __device__ static __forceinline__ uint32_t from_s(S f) { return f2key(__float_as_uint(f)); }
};
template <>
struct Elem<float> {
    using S = float;
    __device__ static __forceinline__ S to_s(float f) { return f; }
    __device__ static __forceinline__ float from_s(S f) { return f; }
};
template <>
struct Elem<double> {
    using S = double;
    __device__ static __forceinline__ S to_s(double d) { return d; }
    __device__ static __forceinline__ double from_s(S d) { return d; }
};

__device__ __forceinline__ void ce(uint32_t& a, uint32_t& b) {
    uint32_t lo = a < b ? a : b;
    uint32_t hi = a < b ? b : a;
    a = lo;
    b = hi;
}
// Float compare-exchange as bare v_min_f32 / v_max_f32: the compiler's minnum lowering would
// first canonicalize every operand that comes from memory or a DPP move (one more VALU op each).
__device__ __forceinline__ void ce(float& a, float& b) {
    float lo, hi;
    asm("v_min_f32 %0, %1, %2" : "=v"(lo) : "v"(a), "v"(b));
    asm("v_max_f32 %0, %1, %2" : "=v"(hi) : "v"(a), "v"(b));
    a = lo;
    b = hi;
}
__device__ __forceinline__ void ce(double& a, double& b) {
    double lo, hi;
    asm("v_min_f64 %0, %1, %2" : "=v"(lo) : "v"(a), "v"(b));
    asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(a), "v"(b));
    a = lo;
    b = hi;
}

// Batcher's odd-even merge sort network for N = 2^m inputs ((m^2 - m + 4) 2^(m-2) - 1
// comparators: 191 for 32 against bitonic's 240), built at compile time so every register
// index is static.
template <int N>
struct OddEvenNet {
    static constexpr int count() {
        int c = 0;
        for (int p = 1; p < N; p *= 2)
            for (int k = p; k >= 1; k /= 2)
                for (int j = k % p; j < N - k; j += 2 * k)
                    for (int i = 0; i < (k < N - j - k ? k : N - j - k); i++)
                        if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) c++;
        return c;
    }
    static constexpr int kCount = count();
    // the first n comparators all join registers of one aligned block of 4
    static constexpr bool first_within_fours(int n) {
        auto t = table();
        for (int c = 0; c < n; c++)
            if (t.a[c] / 4 != t.b[c] / 4) return false;
        return true;
    }
    struct Table {
        unsigned char a[kCount], b[kCount];
    };
    static constexpr Table table() {
        Table t{};
        int c = 0;
        for (int p = 1; p < N; p *= 2)
            for (int k = p; k >= 1; k /= 2)
                for (int j = k % p; j < N - k; j += 2 * k)
                    for (int i = 0; i < (k < N - j - k ? k : N - j - k); i++)
                        if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                            t.a[c] = (unsigned char)(i + j);
                            t.b[c] = (unsigned char)(i + j + k);
                            c++;
                        }
        return t;
    }
};

// A 4-sorter of 8 VALU ops from gfx950's 3-input min / med3 / max (a comparator network needs 5
// comparators = 10 ops): p = min(a,b), q = max(a,b); the smallest is min3(p,c,d), the largest
// max3(q,c,d), the second smallest min(med3(p,c,d), q), the second largest max(med3(q,c,d), p).
// v_min3 / v_med3 / v_max3_f32 order -0.0 before +0.0 like v_min / v_max (tools/ubench/min3_probe.hip
// checks every operand order and every 4-tuple over {-inf,-2,-1,-0,+0,1,2,+inf}).
__device__ __forceinline__ void sort4_3in(float& a, float& b, float& c, float& d) {
    float p, q, lo, hi, m1, m2, o1, o2;
    asm("v_min_f32 %0, %1, %2" : "=v"(p) : "v"(a), "v"(b));
    asm("v_max_f32 %0, %1, %2" : "=v"(q) : "v"(a), "v"(b));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(lo) : "v"(p), "v"(c), "v"(d));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(hi) : "v"(q), "v"(c), "v"(d));
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(m1) : "v"(p), "v"(c), "v"(d));
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(m2) : "v"(q), "v"(c), "v"(d));
    asm("v_min_f32 %0, %1, %2" : "=v"(o1) : "v"(m1), "v"(q));
    asm("v_max_f32 %0, %1, %2" : "=v"(o2) : "v"(m2), "v"(p));
    a = lo;
    b = o1;
    c = o2;
    d = hi;
}
#ifndef SKML_SORT4_3IN
#define SKML_SORT4_3IN 1
#endif

template <int R, typename T>
__device__ __forceinline__ void sort_regs_oddeven(T (&v)[R]) {
    constexpr int C = OddEvenNet<R>::kCount;
    constexpr auto net = OddEvenNet<R>::table();
    // Batcher's first two merge levels (5 R / 4 comparators) sort each block of 4 registers
    constexpr bool k4 = SKML_SORT4_3IN && std::is_same<T, float>::value && R >= 8;
    constexpr int c0 = k4 ? 5 * (R / 4) : 0;
    static_assert(!k4 || OddEvenNet<R>::first_within_fours(c0), "network prefix is not the 4-sorters");
    if constexpr (k4) {
#pragma unroll
        for (int b = 0; b < R / 4; b++) sort4_3in(v[4 * b], v[4 * b + 1], v[4 * b + 2], v[4 * b + 3]);
    }
#pragma unroll
    for (int c = c0; c < C; c++) {
        ce(v[net.a[c]], v[net.b[c]]);
        // 64 keys per lane: keep the scheduler from stretching live ranges past the register budget
        if (R >= 64 && (c & 31) == 31) __builtin_amdgcn_sched_barrier(0);
    }
}

// In-register bitonic sort of R keys, ascending, all comparators in "flip" form.
template <int R, typename T>
__device__ __forceinline__ void sort_regs(T (&v)[R]) {
#pragma unroll
    for (int k = 2; k <= R; k <<= 1) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            int j = i ^ (k - 1);
            if (j > i) ce(v[i], v[j]);
        }
#pragma unroll
        for (int d = k >> 2; d >= 1; d >>= 1) {
#pragma unroll
            for (int i = 0; i < R; i++) {
                int j = i ^ d;
                if (j > i) ce(v[i], v[j]);
            }
        }
    }
}

template <int R, typename T>
__device__ __forceinline__ void halfclean_regs(T (&v)[R]) {
#pragma unroll
    for (int d = R >> 1; d >= 1; d >>= 1) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            int j = i ^ d;
            if (j > i) ce(v[i], v[j]);
        }
    }
}

// Cross-lane compare-exchange in one VALU op: the lower lane of a pair keeps min(a, b), the
// upper lane max(a, b), i.e. med3(a, b, sel) with sel = 0 (lower) or ~0 (upper).  The pattern
// below compiles to a single v_med3_u32.
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    return min(max(a, b), max(min(a, b), c));
}
__device__ __forceinline__ uint32_t med3(uint32_t a, uint32_t b, uint32_t c) { return umed3(a, b, c); }
__device__ __forceinline__ float med3(float a, float b, float c) { return __builtin_amdgcn_fmed3f(a, b, c); }
// no v_med3_f64: c is +inf (keep the max) or -inf (keep the min)
__device__ __forceinline__ double med3(double a, double b, double c) {
    double lo, hi;
    asm("v_min_f64 %0, %1, %2" : "=v"(lo) : "v"(a), "v"(b));
    asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(a), "v"(b));
    return __double_as_longlong(c) > 0 ? hi : lo;
}

#ifndef SKML_FLIP_GROUP
#define SKML_FLIP_GROUP 4  // pairs of a flip stage between scheduling barriers
#endif
#ifndef SKML_HALF_GROUP
#define SKML_HALF_GROUP 8  // registers of a cross-lane half-clean stage between scheduling barriers
#endif
// Flip stage across a block of (M+1) lanes: element (lane, r) meets (lane^M, R-1-r).
template <int R, int M, typename T>
__device__ __forceinline__ void flip_lanes(T (&v)[R], int lane) {
    const T sel = sel_of<T>((lane & ((M + 1) >> 1)) != 0);
#pragma unroll
    for (int r = 0; r < R / 2; r++) {
        const T pa = lane_xor<M>(v[R - 1 - r]);
        const T pb = lane_xor<M>(v[r]);
        v[r] = med3(v[r], pa, sel);
        v[R - 1 - r] = med3(v[R - 1 - r], pb, sel);
        // keep the scheduler from hoisting every exchange of the stage (register pressure)
        if ((r & (SKML_FLIP_GROUP - 1)) == SKML_FLIP_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R, int D, typename T>
__device__ __forceinline__ void halfclean_lanes(T (&v)[R], int lane) {
    const T sel = sel_of<T>((lane & D) != 0);
#pragma unroll
    for (int r = 0; r < R; r++) {
        v[r] = med3(v[r], lane_xor<D>(v[r]), sel);
        if ((r & (SKML_HALF_GROUP - 1)) == SKML_HALF_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R, int D, typename T>
__device__ __forceinline__ void halfclean_lanes_down(T (&v)[R], int lane) {
    if constexpr (D >= 1) {
        halfclean_lanes<R, D>(v, lane);
        halfclean_lanes_down<R, D / 2>(v, lane);
    }
}

// Bitonic merge of a group of G = 256/R lanes holding two sorted 128-runs (lower G/2 lanes and
// upper G/2 lanes, positions lane_in_group*R + r) into one sorted 256-run.
template <int R, typename T>
__device__ __forceinline__ void merge_group(T (&v)[R], int lane) {
    constexpr int G = 256 / R;
    flip_lanes<R, G - 1>(v, lane);
    halfclean_lanes_down<R, G / 4>(v, lane);
    halfclean_regs<R>(v);
}

// Sort 256 keys held by a group of G = 256/R lanes (any initial placement).
template <int R, int S, typename T>
__device__ __forceinline__ void sort_lanes_from(T (&v)[R], int lane) {
    if constexpr (S <= 256) {
        constexpr int M = S / R - 1;
        flip_lanes<R, M>(v, lane);
        halfclean_lanes_down<R, S / R / 4>(v, lane);
        halfclean_regs<R>(v);
        sort_lanes_from<R, S * 2>(v, lane);
    }
}
template <int R, typename T>
__device__ __forceinline__ void sort_group256(T (&v)[R], int lane) {
    sort_regs<R>(v);
    sort_lanes_from<R, 2 * R>(v, lane);
}

// Keep every other sorted position: parity `odd` is the compaction RNG bit
// (QSketchUtils.compactBuffer, QSketchUtils.java:45-51).
// (Written as a bit-select: `odd ? v[2j+1] : v[2j]` is turned into a dynamically indexed
// private array -- i.e. scratch memory -- by hipcc.)
template <int R>
__device__ __forceinline__ void compact_regs(const uint32_t (&v)[R], uint32_t (&w)[R / 2], bool odd) {
    const uint32_t m = odd ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int j = 0; j < R / 2; j++) w[j] = (v[2 * j + 1] & m) | (v[2 * j] & ~m);
}

// The last in-register stage of a bitonic merge compares positions (2j, 2j+1) and the
// compaction that follows keeps one of them: fused into one v_med3 per pair, selecting
// min (even position kept) or max (odd position kept).
template <int R, typename T>
__device__ __forceinline__ void halfclean_regs_compact(T (&v)[R], T (&w)[R / 2], bool odd) {
#pragma unroll
    for (int d = R >> 1; d >= 2; d >>= 1) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            int j = i ^ d;
            if (j > i) ce(v[i], v[j]);
        }
    }
    const T sel = sel_of<T>(odd);
#pragma unroll
    for (int j = 0; j < R / 2; j++) w[j] = med3(v[2 * j], v[2 * j + 1], sel);
}

// merge_group + compaction
template <int R, typename T>
__device__ __forceinline__ void merge_group_compact(T (&v)[R], T (&w)[R / 2], int lane, bool odd) {
    constexpr int G = 256 / R;
    flip_lanes<R, G - 1>(v, lane);
    halfclean_lanes_down<R, G / 4>(v, lane);
    halfclean_regs_compact<R>(v, w, odd);
}

// sort_group256 + compaction (the last merge's final stage fused with the selection)
template <int R, int S, typename T>
__device__ __forceinline__ void sort_lanes_upto128(T (&v)[R], int lane) {
    if constexpr (S <= 128) {
        constexpr int M = S / R - 1;
        flip_lanes<R, M>(v, lane);
        halfclean_lanes_down<R, S / R / 4>(v, lane);
        halfclean_regs<R>(v);
        sort_lanes_upto128<R, S * 2>(v, lane);
    }
}
template <int R, typename T>
__device__ __forceinline__ void sort_group256_compact(T (&v)[R], T (&w)[R / 2], int lane, bool odd) {
    sort_regs<R>(v);
    sort_lanes_upto128<R, 2 * R>(v, lane);  // two sorted 128-runs per group
    merge_group_compact<R>(v, w, lane, odd);  // the final 256 merge + selection
}

// ------------------------------------------------------------------------------------------
// java.util.Random jump-ahead: state after `steps` LCG steps = A^steps * s + C_steps (mod 2^48),
// from a 4-level byte-indexed table of (A^m, C_m) (built on the host, skml_api.cpp).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lcg_jump(const uint64_t* __restrict__ tab, uint64_t s,
                                             uint64_t steps) {
#pragma unroll
    for (int lvl = 0; lvl < 4; lvl++) {
        uint32_t b = (uint32_t)(steps >> (8 * lvl)) & 255u;
        if (b) {
            const uint64_t a = tab[(lvl * 256 + b) * 2];
            const uint64_t c = tab[(lvl * 256 + b) * 2 + 1];
            s = (a * s + c) & kLcgMask;
        }
    }
    return s;
}
// next(1) of the idx-th draw (0-based) from Random(seed) whose scrambled state is s0.
__device__ __forceinline__ uint32_t lcg_bit(const uint64_t* __restrict__ tab, uint64_t s0,
                                            uint64_t idx) {
    return (uint32_t)(lcg_jump(tab, s0, idx + 1) >> 47) & 1u;
}
// Bit-stream index of the compaction that forms the node at `level` whose last chunk is c:
// chunk c's leaf bit is #(2c - popcount(c)), followed by its carry compactions.
__device__ __forceinline__ uint64_t node_bit_index(uint64_t c, int level) {
    return 2 * c - (uint64_t)__popcll(c) + (uint64_t)level;
}

// ------------------------------------------------------------------------------------------
// Exact merge of two sorted 128-runs with the reference tie rule (QSketchUtils.mergeArrays,
// QSketchUtils.java:53-69: IEEE `<`, a tie emits the NEWER run first) followed by compaction.
// Task t in [0,256): element t of older (t<128) or newer.  Writes kept elements to out.
// ------------------------------------------------------------------------------------------
template <typename S>
__device__ __forceinline__ int count_le(const S* run, S x) {  // #{run[i] <= x}
    int lo = 0;
#pragma unroll
    for (int step = 64; step >= 1; step >>= 1)
        if (run[lo + step - 1] <= x) lo += step;
    return lo + (run[lo] <= x ? 1 : 0) * (lo == 127 ? 1 : 0);
}
template <typename S>
__device__ __forceinline__ int count_lt(const S* run, S x) {  // #{run[i] < x}
    int lo = 0;
#pragma unroll
    for (int step = 64; step >= 1; step >>= 1)
        if (run[lo + step - 1] < x) lo += step;
    return lo + (run[lo] < x ? 1 : 0) * (lo == 127 ? 1 : 0);
}
// blockyMergeSort rank contribution of two sorted kK-sample runs a, b for a sample v: #{s < v},
// plus the ties s == v where `tie` (the run precedes v's own run: IEEE `<=`).  The two binary
// searches are independent chains (their LDS reads overlap) and branch-free; `use_a` / `use_b`
// mask a run out (v's own run, or b repeating a).
__device__ __forceinline__ uint32_t tie_pred(float s, float v, uint32_t tie) {
    return (uint32_t)(s < v) | ((uint32_t)(s == v) & tie);
}
__device__ __forceinline__ uint32_t tie_pred(double s, double v, uint32_t tie) {
    return (uint32_t)(s < v) | ((uint32_t)(s == v) & tie);
}
template <typename S>
__device__ __forceinline__ int rank_in_run_pair(const S* a, const S* b, S v, uint32_t tie_a, uint32_t tie_b,
                                                uint32_t use_a, uint32_t use_b) {
    int la = 0, lb = 0;
#pragma unroll
    for (int step = kK / 2; step >= 1; step >>= 1) {
        const S sa = a[la + step - 1], sb = b[lb + step - 1];
        la += (int)tie_pred(sa, v, tie_a) * step;
        lb += (int)tie_pred(sb, v, tie_b) * step;
    }
    const S ea = a[la], eb = b[lb];
    la += (int)(tie_pred(ea, v, tie_a) & (uint32_t)(la == kK - 1));
    lb += (int)(tie_pred(eb, v, tie_b) & (uint32_t)(lb == kK - 1));
    return (int)use_a * la + (int)use_b * lb;
}

template <typename S>
__device__ __forceinline__ void exact_merge_task(const S* older, const S* newer, S* out, int t, uint32_t odd) {
    S v;
    int pos;
    if (t < 128) {
        v = older[t];
        pos = t + count_le(newer, v);
    } else {
        v = newer[t - 128];
        pos = (t - 128) + count_lt(older, v);
    }
    if (((uint32_t)pos & 1u) == odd) out[pos >> 1] = v;
}

// ------------------------------------------------------------------------------------------
// Bucket LUT for the quantize pass (built by one workgroup; `sp` = splits in LDS as floats
// rounded toward +inf, IEEE-sorted; `lut` in global memory).  For a non-NaN float x and a
// double split s, s <= x  <=>  RU(s) <= x, so the float table gives the exact indexOf.
//
// Bucket of a value = top kLutBits of its total-order key, with -0.0 counted in +0.0's bucket.
// base[b] = #{splits in buckets < b} (a histogram + exclusive scan) is a lower bound of indexOf
// for every x in bucket b, and indexOf(x) - base[b] <= need(b) = #{splits in bucket b}, plus all
// zero splits for the bucket holding -0.0 (IEEE -0.0 == +0.0); cmax = max need.  Quantize then
// starts at base[b] and bisects over the next 2^ceil(log2(cmax+1)) splits.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lut_bucket_of(float f) {
    uint32_t u = __float_as_uint(f);
    if (u == 0x80000000u) u = 0u;  // -0.0 -> +0.0's bucket
    return f2key(u) >> (32 - kLutBits);
}

// s_misc: 20 ints of LDS; lbuf: kLutSize / 2 uint32 of LDS (u16 counts, then u16 bases in place).
__device__ __forceinline__ void build_quant_lut(const float* sp, int nsplit, QuantLut* lut, int* s_misc,
                                                uint32_t* lbuf, unsigned long long* prof = nullptr) {
    const int T = blockDim.x, t = threadIdx.x, lane = t & 63, w = t >> 6, nw = T >> 6;
    constexpr uint32_t kNegZeroBucket = 0x7FFFFFFFu >> (32 - kLutBits);
    uint16_t* cnt = reinterpret_cast<uint16_t*>(lbuf);
    for (int i = t; i < kLutSize / 2; i += T) lbuf[i] = 0u;
    if (t < 20) s_misc[t] = 0;
    __syncthreads();
    for (int i = t; i < nsplit; i += T) {  // histogram (u16 halves of u32 words)
        const uint32_t b = lut_bucket_of(sp[i]);
        atomicAdd(&lbuf[b >> 1], 1u << (16 * (b & 1)));
        if ((__float_as_uint(sp[i]) & 0x7FFFFFFFu) == 0u) atomicAdd(&s_misc[0], 1);
    }
    __syncthreads();
    if (prof && t == 0) prof[0] = wall_clock64();  // profiling builds: histogram done
    // exclusive scan: each thread owns kLutSize / T consecutive buckets
    const int per = kLutSize / T, b0 = t * per;  // per >= 16, a multiple of 8
    const uint4* c4 = reinterpret_cast<const uint4*>(cnt + b0);
    int sum = 0, cmax = 0;
    for (int k = 0; k < per / 8; k++) {  // 8 u16 counts per 16-byte LDS read
        const uint4 q = c4[k];
        const uint32_t wds[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int lo = (int)(wds[e] & 0xFFFFu), hi = (int)(wds[e] >> 16);
            sum += lo + hi;
            cmax = max(cmax, max(lo, hi));
        }
    }
    if (b0 <= (int)kNegZeroBucket && (int)kNegZeroBucket < b0 + per) cmax = max(cmax, cnt[kNegZeroBucket] + s_misc[0]);
    const int inc = (int)wave_incl_scan_u32((uint32_t)sum);
    if (lane == 63) s_misc[4 + w] = inc;
    // one LDS atomic per wave (512 same-address atomics serialise: ~2 us)
    cmax = (int)wave_reduce_u32_lane63<1>((uint32_t)cmax);  // counts are >= 0
    if (lane == 63) atomicMax(&s_misc[1], cmax);
    __syncthreads();
    int run = inc - sum;
    for (int j = 0; j < w; j++) run += s_misc[4 + j];
    (void)nw;
    uint4* o4 = reinterpret_cast<uint4*>(cnt + b0);
    for (int k = 0; k < per / 8; k++) {  // counts -> bases in place, 8 per 16-byte access
        const uint4 q = o4[k];
        uint32_t wds[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint32_t lo = wds[e] & 0xFFFFu, hi = wds[e] >> 16;
            const uint32_t blo = (uint32_t)run;
            run += (int)lo;
            wds[e] = blo | ((uint32_t)run << 16);
            run += (int)hi;
        }
        o4[k] = make_uint4(wds[0], wds[1], wds[2], wds[3]);
    }
    __syncthreads();
    if (prof && t == 0) prof[1] = wall_clock64();  // profiling builds: scan done
    const uint4* src = reinterpret_cast<const uint4*>(lbuf);
    uint4* dst = reinterpret_cast<uint4*>(lut->base);
    for (int i = t; i < (int)(sizeof(lut->base) / (sizeof(uint4))); i += T) dst[i] = src[i];
    if (t == 0) lut->cmax = (s_misc[1] <= kLutMaxNeed && nsplit <= kLutMaxSplits) ? s_misc[1] : -1;
}

// Zero the payload bytes between the last written split and the codes (unused split slots after
// Maths.unique, and the 256-B alignment pad), so an encode's payload bytes are a pure function of
// its input and seed (determinism, and byte-equal payloads from any buffer).  Block-strided.
__device__ __forceinline__ void payload_zero_tail(uint8_t* payload, int nsplit_written, int req_bins) {
    double* sp = reinterpret_cast<double*>(payload + kHeaderBytes);
    const int end = (int)((dense_codes_offset(req_bins) - kHeaderBytes) / sizeof(double));
    for (int i = (nsplit_written > 0 ? nsplit_written : 0) + (int)threadIdx.x; i < end; i += (int)blockDim.x)
        sp[i] = 0.0;
}

// ------------------------------------------------------------------------------------------
// Quantizer.indexOf (Quantizer.java:49-72), literally: used for split tables on which it is not
// an upper bound (NaN or descending splits of a degenerate uniform range) and for NaN values.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t java_index_of(const double* s, int bin_num, int zero_idx, double x) {
    const int last = bin_num - 2;
    if (x < s[0]) return 0;
    if (x >= s[last]) return (uint32_t)(bin_num - 1);
    int l = zero_idx, r = zero_idx;
    if (x < 0.0) l = 0;
    else r = last;
    while (l + 1 < r) {
        const int mid = (l + r) >> 1;
        if (s[mid] > x) {
            if (mid == 0 || s[mid - 1] <= x) return (uint32_t)mid;
            r = mid;
        } else {
            l = mid;
        }
    }
    const int mid = (l + r) >> 1;
    return s[mid] <= x ? (uint32_t)(mid + 1) : (uint32_t)mid;
}

// Quantizer.indexOf (Quantizer.java:49-92) on a NaN value: the probe never succeeds, so the
// search runs from zeroIdx up to the last split and returns its final midpoint.
__host__ __device__ inline int nan_bin_for(int bin_num, int zero_idx) {
    const int last = bin_num - 2;
    if (last < 0) return 0;
    return zero_idx + 1 < last ? last - 1 : (zero_idx + last) >> 1;
}

}  // namespace skml
