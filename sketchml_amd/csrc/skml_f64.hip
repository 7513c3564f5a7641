// skml_f64.hip -- CDNA4 (gfx950) kernels for double-precision input and the uniform quantizer.
//
// The reference codec takes double[] (QuantileQuantizer.quantize(double[]),
// DenseVectorCompressor.compressDense(double[])).  This file builds the
// same k=128 sketch over fp64 values:
//
//   leaf / merge  k_leaf2<.., double> and k_merge64 in skml_sketch.hip: the fp32 leaf's layout
//                 (8 lanes x 32 values per chunk) and merge passes over doubles, compared with
//                 v_min/v_max_f64 (Arrays.sort order incl. -0.0 < 0.0 on gfx950).
//   k_summary64   makeSummary + getQuantiles + Maths.unique + findZeroIdx + header
//                 (HeapQuantileSketch.java:126-174,293-323; Maths.java:51-67; Quantizer.java:74-85).
//   k_quantize64  Quantizer.indexOf over an LDS split table (double compares), packed codes.
//   k_decode64    getValues()[bin] in double (DenseVectorCompressor.decompressDense).
//
// Uniform quantizer (quantization/UniformQuantizer.java:21-45), fp32 and fp64 input:
//   k_uni_minmax  per-workgroup IEEE min / max (NaN skipped) and the first zero's index
//   k_uni_finish  Java min / max (MAX_VALUE / MIN_VALUE initialised, the first zero wins the
//                 min), splits by repeated `+= step`, findZeroIdx, header, quantize LUT.
#include <algorithm>

#include "skml_device.hpp"

namespace skml {

__device__ __forceinline__ uint64_t d2key(uint64_t b) {
    return b ^ ((uint64_t)((int64_t)b >> 63) | 0x8000000000000000ull);
}
__device__ __forceinline__ uint64_t key2d(uint64_t k) {
    return k ^ ((k >> 63) ? 0x8000000000000000ull : ~0ull);
}
__device__ __forceinline__ double kd(uint64_t k) { return __longlong_as_double((long long)key2d(k)); }
__device__ __forceinline__ uint64_t dk(double d) { return d2key((uint64_t)__double_as_longlong(d)); }
__device__ __forceinline__ bool is_nan64(uint64_t b) {
    return (b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// #{run[i] <= x} / #{run[i] < x} over a sorted 128-run (the record merge, k_sketch_merge64)
__device__ __forceinline__ int count_le64(const double* run, double x) {  // #{run[i] <= x}
    int lo = 0;
#pragma unroll
    for (int step = 64; step >= 1; step >>= 1)
        if (run[lo + step - 1] <= x) lo += step;
    return lo + ((lo == 127 && run[127] <= x) ? 1 : 0);
}
__device__ __forceinline__ int count_lt64(const double* run, double x) {  // #{run[i] < x}
    int lo = 0;
#pragma unroll
    for (int step = 64; step >= 1; step >>= 1)
        if (run[lo + step - 1] < x) lo += step;
    return lo + ((lo == 127 && run[127] < x) ? 1 : 0);
}
// ---------------------------------------------------------------------------------------------
// Summary (one workgroup of 512 threads, dynamic LDS).
// ---------------------------------------------------------------------------------------------
constexpr int kMaxSamples64 = kMaxLevels * kK + kChunk;
constexpr int kSum64Raw = 1024;
struct Summary64Shared {
    double smp[kMaxSamples64];
    double sorted[kMaxSamples64];
    int64_t w[kMaxSamples64 + 1];
    double raw[kSum64Raw];
    int64_t wsum[16];
    int run_off[kMaxLevels + 2];
    int run_lvl[kMaxLevels + 2];
    int nruns;
    unsigned long long min_key, max_key;
    uint32_t flags;
    int zero;
    int64_t total;
};

__device__ int64_t block_scan_excl64(int64_t v, int64_t* wsum, int64_t* total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, nw = blockDim.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
        int64_t s = lane < nw ? wsum[lane] : 0;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const int64_t y = __shfl_up(s, off, 64);
            if (lane >= off) s += y;
        }
        if (lane < nw) wsum[lane] = s;
    }
    __syncthreads();
    const int64_t base = w > 0 ? wsum[w - 1] : 0;
    *total = wsum[nw - 1];
    __syncthreads();
    return base + x - v;
}

__device__ __forceinline__ int run_count_le64(const double* r, int len, double x) {
    int lo = 0, hi = len;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (r[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int run_count_lt64(const double* r, int len, double x) {
    int lo = 0, hi = len;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (r[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ void write_header(skml_dense_header* hdr, int status, int64_t n, int bin_num, int zero,
                             int req_bins, double vmin, double vmax) {
    hdr->magic = SKML_DENSE_MAGIC;
    hdr->status = status;
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

__global__ __launch_bounds__(512) void k_summary64(const double* __restrict__ x, int64_t n,
                                                   const LeafPartial64* __restrict__ part, int64_t nparts,
                                                   const double* __restrict__ roots,
                                                   const int64_t* __restrict__ ranks, int req_bins, int dedup,
                                                   uint8_t* __restrict__ payload, double* __restrict__ g_raw,
                                                   QuantLut* __restrict__ lut, const double* __restrict__ tail_in,
                                                   int sharded, int64_t n_local) {
    extern __shared__ __align__(16) uint8_t smem64[];
    Summary64Shared& S = *reinterpret_cast<Summary64Shared*>(smem64);
    const int t = threadIdx.x, T = blockDim.x;
    skml_dense_header* hdr = reinterpret_cast<skml_dense_header*>(payload);
    double* splits = reinterpret_cast<double*>(payload + kHeaderBytes);
    const int64_t chunks = n / kChunk;
    const int tail = (int)(n - chunks * kChunk);
    const double* xt = tail_in ? tail_in : x + chunks * kChunk;
    const int64_t n_hdr = sharded ? n_local : n;

    if (t == 0) {
        S.min_key = ~0ull;
        S.max_key = 0ull;
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
    {
        uint64_t mn = ~0ull, mx = 0ull;
        uint32_t fl = 0u;
        for (int64_t i = t; i < nparts; i += T) {
            const LeafPartial64 p = part[i];
            mn = p.min_key < mn ? p.min_key : mn;
            mx = p.max_key > mx ? p.max_key : mx;
            fl |= p.flags;
        }
        for (int i = t; i < tail; i += T) {
            const uint64_t b = (uint64_t)__double_as_longlong(xt[i]);
            fl |= is_nan64(b) ? 1u : 0u;
            const uint64_t k = d2key(b);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint64_t omn = __shfl_xor(mn, off, 64), omx = __shfl_xor(mx, off, 64);
            mn = omn < mn ? omn : mn;
            mx = omx > mx ? omx : mx;
            fl |= (uint32_t)__shfl_xor((int)fl, off, 64);
        }
        if ((t & 63) == 0) {
            atomicMin(&S.min_key, (unsigned long long)mn);
            atomicMax(&S.max_key, (unsigned long long)mx);
            if (fl) atomicOr(&S.flags, fl);
        }
    }
    const int nruns = S.nruns;
    const int ns = S.run_off[nruns];
    for (int idx = t; idx < (nruns - 1) * kK; idx += T) {
        const int r = idx / kK, i = idx % kK;
        S.smp[S.run_off[r] + i] = roots[(size_t)S.run_lvl[r] * kK + i];
    }
    for (int i = t; i < tail; i += T) S.sorted[i] = xt[i];
    __syncthreads();
    {  // the base buffer, sorted in Arrays.sort total order by rank counting (ties by position)
        const int toff = S.run_off[nruns - 1];
        for (int i = t; i < tail; i += T) {
            const double xi = S.sorted[i];
            const uint64_t ki = dk(xi);
            int rank = 0;
            for (int j = 0; j < tail; j++) {
                const uint64_t kj = dk(S.sorted[j]);
                rank += (kj < ki) || (kj == ki && j < i);
            }
            S.smp[toff + rank] = xi;
        }
    }
    __syncthreads();

    double vmin = 1.7976931348623157e308, vmax = 4.9e-324;  // HeapQuantileSketch.java:67-68
    if (n > 0) {
        const double fmin = kd(S.min_key), fmax = kd(S.max_key);
        if (fmin <= vmin) vmin = fmin;  // Math.min(Double.MAX_VALUE, x)
        if (fmax > vmax) vmax = fmax;   // Math.max(Double.MIN_VALUE, x)
    }
    if (S.flags & 1u) {  // NaN: QuantileSketchException("Encounter NaN value")
        payload_zero_tail(reinterpret_cast<uint8_t*>(hdr), 0, req_bins);
        if (t == 0) write_header(hdr, SKML_E_NAN, n_hdr, req_bins, 0, req_bins, vmin, vmax);
        return;
    }
    // blockyMergeSort == stable sort under IEEE `<=` (left run wins ties): rank across runs.  The
    // level runs hold kK samples each at q * kK (the base buffer last).
    {
        const int nfull = nruns - 1;
        const double* tail_run = S.smp + S.run_off[nfull];
        for (int i = t; i < ns; i += T) {
            const int r = i < nfull * kK ? i / kK : nfull;
            const double v = S.smp[i];
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
            if (r < nfull) rank += run_count_lt64(tail_run, tail, v);  // the base buffer comes last
            S.sorted[rank] = v;
            S.w[rank] = S.run_lvl[r] < 0 ? 1 : ((int64_t)2 << S.run_lvl[r]);
        }
    }
    __syncthreads();
    {  // exclusive prefix of weights (HeapQuantileSketch.java:137-142)
        const int per = (ns + T - 1) / T;
        const int b0 = min(ns, t * per), b1 = min(ns, b0 + per);
        int64_t loc = 0;
        for (int i = b0; i < b1; i++) loc += S.w[i];
        const int64_t base = block_scan_excl64(loc, S.wsum, &S.total);
        int64_t acc = base;
        for (int i = b0; i < b1; i++) {
            const int64_t wv = S.w[i];
            S.w[i] = acc;
            acc += wv;
        }
        if (t == 0) S.w[ns] = S.total;
    }
    __syncthreads();
    const int nsplit_req = req_bins - 1;
    const bool lds_raw = nsplit_req <= kSum64Raw;
    double* raw = lds_raw ? S.raw : g_raw;
    for (int i = t; i < nsplit_req; i += T) {  // getQuantiles(int)
        double sp;
        if (ns == 0) {
            sp = __longlong_as_double(0x7FF8000000000000LL);  // NaN (HeapQuantileSketch.java:299-301)
        } else {
            const int64_t rank = ranks[i];
            int lo = 0, hi = ns;
            while (lo + 1 < hi) {
                const int mid = (lo + hi) >> 1;
                if (S.w[mid] <= rank) lo = mid;
                else hi = mid;
            }
            sp = S.sorted[lo];
        }
        raw[i] = sp;
    }
    if (!lds_raw) __threadfence();
    __syncthreads();
    int bin_num;
    {  // Maths.unique (IEEE !=, keep first) + findZeroIdx
        const int per = (nsplit_req + T - 1) / T;
        const int b0 = min(nsplit_req, t * per), b1 = min(nsplit_req, b0 + per);
        int64_t loc = 0;
        for (int i = b0; i < b1; i++) loc += (!dedup || i == 0 || raw[i] != raw[i - 1]) ? 1 : 0;
        const int64_t base = block_scan_excl64(loc, S.wsum, &S.total);
        int64_t o = base;
        int zmin = 0x7FFFFFFF;
        for (int i = b0; i < b1; i++) {
            if (!dedup || i == 0 || raw[i] != raw[i - 1]) {
                const double sp = raw[i];
                splits[o] = sp;
                if (o < kLutMaxSplits) reinterpret_cast<float*>(S.smp)[o] = __double2float_ru(sp);  // LUT input
                if (!(sp < 0.0)) zmin = min(zmin, (int)o);
                o++;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) zmin = min(zmin, __shfl_xor(zmin, off, 64));
        if ((t & 63) == 0 && zmin != 0x7FFFFFFF) atomicMin(&S.zero, zmin);
        bin_num = (int)S.total + 1;
    }
    __syncthreads();
    payload_zero_tail(reinterpret_cast<uint8_t*>(hdr), bin_num - 1, req_bins);
    if (t == 0) {
        int zero;
        if (vmin > 0.0) zero = 0;
        else if (vmax < 0.0) zero = bin_num - 1;
        else zero = S.zero < bin_num - 1 ? S.zero : bin_num - 1;
        write_header(hdr, SKML_OK, n_hdr, bin_num, zero, req_bins, vmin, vmax);
    }
    // quantize bucket LUT over the RU(fp32) images of the splits (staging aliases sorted[] + w[])
    const int nsplit = bin_num - 1;
    if (nsplit <= kLutMaxSplits && n > 0) {
        build_quant_lut(reinterpret_cast<const float*>(S.smp), nsplit, lut, reinterpret_cast<int*>(S.wsum),
                        reinterpret_cast<uint32_t*>(S.sorted));
    } else if (t == 0) {
        lut->cmax = -1;
    }
}

// ---------------------------------------------------------------------------------------------
// Quantize (fp64 input): Eytzinger upper_bound over the LDS split table in double.
// `flags` bit 0: literal Java indexOf (degenerate split table).
// ---------------------------------------------------------------------------------------------
constexpr int kEytz64Max = 4096;

__device__ __forceinline__ void pack_store4(uint8_t* codes, int64_t e0, const uint32_t (&c)[4], int bits,
                                            int lane) {
    switch (bits) {
        case 8:
            *reinterpret_cast<uint32_t*>(codes + e0) = c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24);
            break;
        case 16:
            *reinterpret_cast<uint2*>(codes + e0 * 2) = make_uint2(c[0] | (c[1] << 16), c[2] | (c[3] << 16));
            break;
        case 4:
            *reinterpret_cast<uint16_t*>(codes + e0 / 2) = (uint16_t)(c[0] | (c[1] << 4) | (c[2] << 8) | (c[3] << 12));
            break;
        case 2:
            codes[e0 / 4] = (uint8_t)(c[0] | (c[1] << 2) | (c[2] << 4) | (c[3] << 6));
            break;
        default: {
            const uint32_t nib = c[0] | (c[1] << 1) | (c[2] << 2) | (c[3] << 3);
            const uint32_t other = lane_xor<1>(nib);
            if ((lane & 1) == 0) codes[e0 / 8] = (uint8_t)(nib | (other << 4));
            break;
        }
    }
}

// Modes: 0..4 = bucket LUT + that many float bisection steps; kQ64Eytz / kQ64Global / kQ64Java.
//
// LUT mode: y = RD(x), x rounded toward -inf to fp32, is <= x and lies in the same float-bounded
// interval as x, and the fp32 machinery counts #{s <= y} exactly (s <= y <=> RU(s) <= y for a
// float y, see build_quant_lut).  The splits in (y, x] -- within one fp32 ulp of x, almost
// always none -- are then added by exact double compares.
constexpr int kQ64Eytz = 8, kQ64Global = 9, kQ64Java = 10;

struct Q64Tables {
    const uint16_t* base;
    const float* S;
    const double* E;
    const double* sp;
    int nsplit, levels, zero, bins;
    uint32_t P, nan_bin;
};

template <int MODE>
__device__ __forceinline__ uint32_t q64_bin(const Q64Tables& q, double v) {
    if constexpr (MODE == kQ64Java) {
        return java_index_of(q.sp, q.bins, q.zero, v);
    } else {
        if (v != v) return q.nan_bin;
        uint32_t bin;
        if constexpr (MODE <= 4) {
            const float y = __double2float_rd(v);
            bin = q.base[f2key(__float_as_uint(y)) >> (32 - kLutBits)];
#pragma unroll
            for (int h = (1 << MODE) >> 1; h > 0; h >>= 1) bin += q.S[bin + h - 1] <= y ? (uint32_t)h : 0u;
            // a split in (y, x] has RU(split) <= RU(x): only then compare in double
            if (q.S[bin] <= __double2float_ru(v))
                while (bin < (uint32_t)q.nsplit && q.sp[bin] <= v) bin++;
        } else if constexpr (MODE == kQ64Eytz) {
            uint32_t i = 1;
            for (int s = 0; s < q.levels; s++) i = 2 * i + (q.E[i] <= v ? 1u : 0u);
            bin = i - q.P;  // +inf padding: v == +inf passes every pad; clamp to the split count
            bin = bin > (uint32_t)q.nsplit ? (uint32_t)q.nsplit : bin;
        } else {
            int lo = 0, hi = q.nsplit;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (q.sp[mid] <= v) lo = mid + 1;
                else hi = mid;
            }
            bin = (uint32_t)lo;
        }
        return bin;
    }
}

template <int MODE>
__device__ __forceinline__ void q64_tiles(const Q64Tables& q, const double* __restrict__ x, int64_t n,
                                          uint8_t* __restrict__ codes, int bits) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4, wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t full = n / 1024;
    for (int64_t tile = wid; tile < full; tile += nw) {
        const f64x2* src = reinterpret_cast<const f64x2*>(x + tile * 1024);
        f64x2 a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            a[j] = __builtin_nontemporal_load(src + j * 128 + 2 * lane);
            b[j] = __builtin_nontemporal_load(src + j * 128 + 2 * lane + 1);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t c[4] = {q64_bin<MODE>(q, a[j].x), q64_bin<MODE>(q, a[j].y), q64_bin<MODE>(q, b[j].x),
                                   q64_bin<MODE>(q, b[j].y)};
            pack_store4(codes, tile * 1024 + j * 256 + lane * 4, c, bits, lane);
        }
    }
    if (wid == full % nw && n % 1024) {
        const int64_t base = full * 1024;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e0 = base + j * 256 + lane * 4;
            uint32_t c[4] = {0, 0, 0, 0};
            for (int e = 0; e < 4; e++)
                if (e0 + e < n) c[e] = q64_bin<MODE>(q, x[e0 + e]);
            if (bits == 1) {
                const int64_t pair0 = base + j * 256 + (lane & ~1) * 4;
                const uint32_t nib = c[0] | (c[1] << 1) | (c[2] << 2) | (c[3] << 3);
                const uint32_t other = lane_xor<1>(nib);
                if ((lane & 1) == 0 && pair0 < n) codes[pair0 / 8] = (uint8_t)(nib | (other << 4));
            } else if (e0 < n) {
                pack_store4(codes, e0, c, bits, lane);
            }
        }
    }
}

// Dynamic LDS: LUT mode [0, 32 KB) bucket bases then `lds_splits` floats; Eytzinger mode reuses
// it as up to 4096 doubles.
__global__ __launch_bounds__(256) void k_quantize64(const double* __restrict__ x, int64_t n,
                                                    uint8_t* __restrict__ payload, const QuantLut* __restrict__ lut,
                                                    const int* __restrict__ qflags, int lds_splits) {
    extern __shared__ __align__(16) uint8_t q64sm[];
    const skml_dense_header* hdr = reinterpret_cast<const skml_dense_header*>(payload);
    if (hdr->status != SKML_OK) return;
    Q64Tables q;
    q.bins = hdr->bin_num;
    q.nsplit = q.bins - 1;
    q.zero = hdr->zero_idx;
    q.sp = reinterpret_cast<const double*>(payload + kHeaderBytes);
    q.nan_bin = (uint32_t)nan_bin_for(q.bins, q.zero);
    q.P = 1;
    q.levels = 0;
    while (q.P < (uint32_t)q.bins) {
        q.P <<= 1;
        q.levels++;
    }
    const int bits = hdr->code_bits;
    uint8_t* codes = payload + hdr->codes_offset;
    const int cmax = lut ? lut->cmax : -1;
    int mode;
    if ((qflags && (*qflags & 1)) || cmax == kLutJavaMode) {
        mode = kQ64Java;
    } else if (cmax >= 0 && q.nsplit + kLutPad <= lds_splits) {
        mode = cmax == 0 ? 0 : 32 - __clz((uint32_t)cmax);
        uint16_t* base = reinterpret_cast<uint16_t*>(q64sm);
        float* S = reinterpret_cast<float*>(q64sm + sizeof(lut->base));
        const uint4* src = reinterpret_cast<const uint4*>(lut->base);
        for (int i = threadIdx.x; i < (int)(sizeof(lut->base) / 16); i += blockDim.x)
            reinterpret_cast<uint4*>(base)[i] = src[i];
        for (int i = threadIdx.x; i < q.nsplit + kLutPad; i += blockDim.x)
            S[i] = i < q.nsplit ? __double2float_ru(q.sp[i]) : __uint_as_float(0x7FC00000u);
        q.base = base;
        q.S = S;
    } else if (q.P <= kEytz64Max && (size_t)q.P * sizeof(double) <= sizeof(lut->base) + lds_splits * sizeof(float)) {
        mode = kQ64Eytz;
        double* E = reinterpret_cast<double*>(q64sm);
        for (uint32_t i = threadIdx.x + 1; i < q.P; i += blockDim.x) {
            const int d = 31 - __clz(i);
            const uint32_t idx = ((2u * (i - (1u << d)) + 1u) << (q.levels - 1 - d)) - 1u;
            E[i] = idx < (uint32_t)q.nsplit ? q.sp[idx] : __longlong_as_double(0x7FF0000000000000LL);
        }
        q.E = E;
    } else {
        mode = kQ64Global;
    }
    __syncthreads();
    switch (mode) {
        case 0: q64_tiles<0>(q, x, n, codes, bits); break;
        case 1: q64_tiles<1>(q, x, n, codes, bits); break;
        case 2: q64_tiles<2>(q, x, n, codes, bits); break;
        case 3: q64_tiles<3>(q, x, n, codes, bits); break;
        case 4: q64_tiles<4>(q, x, n, codes, bits); break;
        case kQ64Eytz: q64_tiles<kQ64Eytz>(q, x, n, codes, bits); break;
        case kQ64Java: q64_tiles<kQ64Java>(q, x, n, codes, bits); break;
        default: q64_tiles<kQ64Global>(q, x, n, codes, bits); break;
    }
}

// ---------------------------------------------------------------------------------------------
// Decode to double: getValues()[bin] (Quantizer.java:39-47), LUT in LDS.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double lut_value64(const skml_dense_header* h, const double* sp, int b) {
    const int ns = h->bin_num - 1;
    if (b == 0) return 0.5 * (h->min + sp[0]);
    if (b == ns) return 0.5 * (sp[ns - 1] + h->max);
    return 0.5 * (sp[b - 1] + sp[b]);
}

__device__ __forceinline__ uint32_t code_at(const uint8_t* codes, int64_t e, int bits) {
    switch (bits) {
        case 8: return codes[e];
        case 16: return reinterpret_cast<const uint16_t*>(codes)[e];
        case 4: return (codes[e >> 1] >> ((e & 1) * 4)) & 15u;
        case 2: return (codes[e >> 2] >> ((e & 3) * 2)) & 3u;
        default: return (codes[e >> 3] >> (e & 7)) & 1u;
    }
}

// Four consecutive codes starting at e0 (a multiple of 4) from one load.
__device__ __forceinline__ void codes4(const uint8_t* codes, int64_t e0, int bits, uint32_t (&c)[4]) {
    uint32_t w;
    switch (bits) {
        case 16: {
            const uint2 q = *reinterpret_cast<const uint2*>(codes + e0 * 2);
            c[0] = q.x & 0xFFFFu; c[1] = q.x >> 16; c[2] = q.y & 0xFFFFu; c[3] = q.y >> 16;
            return;
        }
        case 8: w = *reinterpret_cast<const uint32_t*>(codes + e0); break;
        case 4: w = *reinterpret_cast<const uint16_t*>(codes + e0 / 2); break;
        case 2: w = codes[e0 / 4]; break;
        default: w = (uint32_t)(codes[e0 / 8] >> (e0 & 4)); break;
    }
    const uint32_t m = (1u << bits) - 1u;
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = (w >> (k * bits)) & m;
}

__global__ __launch_bounds__(256) void k_decode64(const uint8_t* __restrict__ payload, double* __restrict__ out,
                                                  int64_t n) {
    __shared__ double lut[kEytz64Max];
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(payload);
    const double* sp = reinterpret_cast<const double*>(payload + kHeaderBytes);
    const uint8_t* codes = payload + h->codes_offset;
    const int bins = h->bin_num, bits = h->code_bits;
    const bool lds = bins <= kEytz64Max;
    if (lds)
        for (int b = threadIdx.x; b < bins; b += blockDim.x) lut[b] = lut_value64(h, sp, b);
    __syncthreads();
    auto val = [&](uint32_t c) { return lds ? lut[c] : lut_value64(h, sp, (int)c); };
    // 1024-value tiles per wave: each lane reads 4 codes and writes two double2 per step
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4, wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t full = n / 1024;
    for (int64_t tile = wid; tile < full; tile += nw) {
        f64x2* dst = reinterpret_cast<f64x2*>(out + tile * 1024);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e0 = tile * 1024 + j * 256 + lane * 4;
            uint32_t c[4];
            codes4(codes, e0, bits, c);
            dst[j * 128 + 2 * lane] = f64x2{val(c[0]), val(c[1])};
            dst[j * 128 + 2 * lane + 1] = f64x2{val(c[2]), val(c[3])};
        }
    }
    if (wid == full % nw)
        for (int64_t e = full * 1024 + lane; e < n; e += 64) out[e] = val(code_at(codes, e, bits));
}

// ---------------------------------------------------------------------------------------------
// Uniform quantizer: per-workgroup min / max / first zero, then one finishing workgroup.
// ---------------------------------------------------------------------------------------------
template <typename T>
struct Vec16;  // 16-byte vector of T
template <>
struct Vec16<float> {
    typedef f32x4 type;
    static constexpr int N = 4;
    __device__ static void get(const f32x4& v, float (&o)[4]) {
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
};
template <>
struct Vec16<double> {
    typedef f64x2 type;
    static constexpr int N = 2;
    __device__ static void get(const f64x2& v, double (&o)[2]) {
        o[0] = v.x; o[1] = v.y;
    }
};

// Streaming min / max / first zero over 16-byte loads (8 in flight per thread), compared in the
// input type (IEEE order is the same as in double); the zero index is a Java int.
template <typename T>
__global__ __launch_bounds__(256) void k_uni_minmax(const T* __restrict__ x, int64_t n, UniPartial* __restrict__ part) {
    using V = Vec16<T>;
    typedef typename V::type VT;
    constexpr int U = 8;
    T mn = (T)__builtin_inf(), mx = -(T)__builtin_inf();
    int32_t z = INT32_MAX;
    const int64_t nv = n / V::N;
    const VT* xv = reinterpret_cast<const VT*>(x);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < nv; i += U * stride) {
        VT v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(xv + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; u++) {
            T e[V::N];
            V::get(v[u], e);
#pragma unroll
            for (int k = 0; k < V::N; k++) {
                mn = e[k] < mn ? e[k] : mn;  // NaN never compares: skipped, as `if (v < min)`
                mx = e[k] > mx ? e[k] : mx;
                const int32_t idx = (int32_t)((i + u * stride) * V::N + k);
                z = (e[k] == (T)0 && idx < z) ? idx : z;
            }
        }
    }
    for (; i < nv; i += stride) {
        T e[V::N];
        V::get(xv[i], e);
#pragma unroll
        for (int k = 0; k < V::N; k++) {
            mn = e[k] < mn ? e[k] : mn;
            mx = e[k] > mx ? e[k] : mx;
            const int32_t idx = (int32_t)(i * V::N + k);
            z = (e[k] == (T)0 && idx < z) ? idx : z;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < n - nv * V::N) {  // ragged tail
        const int64_t idx = nv * V::N + threadIdx.x;
        const T e = x[idx];
        mn = e < mn ? e : mn;
        mx = e > mx ? e : mx;
        z = (e == (T)0 && (int32_t)idx < z) ? (int32_t)idx : z;
    }
    __shared__ T smn[4], smx[4];
    __shared__ int32_t sz[4];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const T omn = __shfl_xor(mn, off, 64), omx = __shfl_xor(mx, off, 64);
        const int32_t oz = __shfl_xor(z, off, 64);
        mn = omn < mn ? omn : mn;
        mx = omx > mx ? omx : mx;
        z = oz < z ? oz : z;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smn[w] = mn;
        smx[w] = mx;
        sz[w] = z;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); k++) {
            mn = smn[k] < mn ? smn[k] : mn;
            mx = smx[k] > mx ? smx[k] : mx;
            z = sz[k] < z ? sz[k] : z;
        }
        part[blockIdx.x] = UniPartial{(double)mn, (double)mx, z == INT32_MAX ? INT64_MAX : (int64_t)z, 0};
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_uni_finish(const T* __restrict__ x, int64_t n,
                                                    const UniPartial* __restrict__ part, int nparts, int bin_num,
                                                    uint8_t* __restrict__ payload, QuantLut* __restrict__ lut,
                                                    int* __restrict__ qflags) {
    skml_dense_header* hdr = reinterpret_cast<skml_dense_header*>(payload);
    double* splits = reinterpret_cast<double*>(payload + kHeaderBytes);
    __shared__ double s_mn, s_mx;
    __shared__ double s_rmn[4], s_rmx[4];
    __shared__ int64_t s_rz[4];
    __shared__ int s_bad;
    __shared__ int s_zero;
    __shared__ int s_misc[20];
    __shared__ float s_sp[kLutMaxSplits];
    __shared__ __align__(16) uint32_t s_lbuf[kLutSize / 2];
    {  // reduce the partials (one per thread, then waves, then thread 0)
        double mn = __longlong_as_double(0x7FF0000000000000LL), mx = -mn;
        int64_t z = INT64_MAX;
        for (int k = threadIdx.x; k < nparts; k += blockDim.x) {
            const UniPartial p = part[k];
            mn = p.mn < mn ? p.mn : mn;
            mx = p.mx > mx ? p.mx : mx;
            z = p.zidx < z ? p.zidx : z;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double omn = __shfl_xor(mn, off, 64), omx = __shfl_xor(mx, off, 64);
            const int64_t oz = __shfl_xor(z, off, 64);
            mn = omn < mn ? omn : mn;
            mx = omx > mx ? omx : mx;
            z = oz < z ? oz : z;
        }
        if ((threadIdx.x & 63) == 0) {
            s_rmn[threadIdx.x >> 6] = mn;
            s_rmx[threadIdx.x >> 6] = mx;
            s_rz[threadIdx.x >> 6] = z;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double mn = s_rmn[0], mx = s_rmx[0];
        int64_t z = s_rz[0];
        for (int k = 1; k < (int)(blockDim.x >> 6); k++) {
            mn = s_rmn[k] < mn ? s_rmn[k] : mn;
            mx = s_rmx[k] > mx ? s_rmx[k] : mx;
            z = s_rz[k] < z ? s_rz[k] : z;
        }
        // UniformQuantizer.java:24-29: min from Double.MAX_VALUE by `<`, max from Double.MIN_VALUE
        // by `>`; among equal minima the first wins, which only shows for a zero minimum
        double jmin = 1.7976931348623157e308, jmax = 4.9e-324;
        if (mn < jmin) jmin = (mn == 0.0) ? (double)x[z] : mn;
        if (mx > jmax) jmax = mx;
        s_mn = jmin;
        s_mx = jmax;
        // UniformQuantizer.java:31-36: split i is min + step followed by i more `+= step`, a
        // serial chain of rounded adds; only the adds stay on one thread (the conversions and
        // checks below run on the whole workgroup: one thread doing all of it took ~30 us)
        const double step = (jmax - jmin) / bin_num;
        const int ns = bin_num - 1;
        double cur = jmin + step;
        for (int i = 0; i < ns; i++) {
            if (i > 0) cur = cur + step;
            splits[i] = cur;
        }
        s_bad = 0;
        s_zero = ns;
    }
    __threadfence_block();
    __syncthreads();
    const int ns = bin_num - 1;
    {
        int bad = 0, zero = ns;
        for (int i = threadIdx.x; i < ns; i += blockDim.x) {
            const double cur = splits[i], prev = i > 0 ? splits[i - 1] : cur;
            if (i < kLutMaxSplits) s_sp[i] = __double2float_ru(cur);
            bad |= (!(cur == cur) || !(prev <= cur)) ? 1 : 0;
            zero = (zero == ns && !(cur < 0.0)) ? i : zero;  // ascending i per thread: its first
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            bad |= __shfl_xor(bad, off, 64);
            zero = min(zero, __shfl_xor(zero, off, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            if (bad) atomicOr(&s_bad, 1);
            atomicMin(&s_zero, zero);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *qflags = s_bad;
    const double jmin = s_mn, jmax = s_mx;
    const bool lut_ok = !s_bad && ns <= kLutMaxSplits;
    payload_zero_tail(reinterpret_cast<uint8_t*>(hdr), ns, bin_num);
    if (lut_ok) build_quant_lut(s_sp, ns, lut, s_misc, s_lbuf);
    if (threadIdx.x == 0) {
        if (s_bad) lut->cmax = kLutJavaMode;
        else if (!lut_ok) lut->cmax = -1;
        int zero;  // Quantizer.findZeroIdx (Quantizer.java:74-85)
        if (jmin > 0.0) zero = 0;
        else if (jmax < 0.0) zero = bin_num - 1;
        else zero = s_zero;
        write_header(hdr, SKML_OK, n, bin_num, zero, bin_num, jmin, jmax);
    }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
hipError_t launch_summary64(hipStream_t st, const double* x, int64_t n, const LeafPartial64* part, int64_t nparts,
                            const double* roots, const int64_t* ranks, int req_bins, int dedup, void* payload,
                            double* g_raw, QuantLut* lut, const double* tail, int sharded, int64_t n_local) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_summary64),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)sizeof(Summary64Shared));
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(k_summary64, dim3(1), dim3(512), sizeof(Summary64Shared), st, x, n, part, nparts, roots,
                       ranks, req_bins, dedup, reinterpret_cast<uint8_t*>(payload), g_raw, lut, tail, sharded,
                       n_local);
    return hipGetLastError();
}

static int grid_for(int64_t n, int per_wg, int cap) {
    int64_t g = (n + per_wg - 1) / per_wg;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

hipError_t launch_quantize64(hipStream_t st, const double* x, int64_t n, void* payload, const QuantLut* lut,
                             const int* qflags, int req_bins) {
    if (n <= 0) return hipSuccess;
    // LDS sized for this request's split table (LUT mode), at least the 32 KB Eytzinger table
    const int lds_splits = std::min(std::max(req_bins - 1, 1), kLutMaxSplits) + kLutPad;
    const size_t lds = std::max(sizeof(QuantLut::base) + (size_t)lds_splits * sizeof(float),
                                (size_t)kEytz64Max * sizeof(double));
    hipLaunchKernelGGL(k_quantize64, dim3(grid_for(n, 4096, 1024)), dim3(256), lds, st, x, n,
                       reinterpret_cast<uint8_t*>(payload), lut, qflags, lds_splits);
    return hipGetLastError();
}

hipError_t launch_decode64(hipStream_t st, const void* payload, double* out, int64_t n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode64, dim3(grid_for(n, 4096, 2048)), dim3(256), 0, st,
                       reinterpret_cast<const uint8_t*>(payload), out, n);
    return hipGetLastError();
}

int uniform_partials(int64_t n) { return grid_for(n, 1 << 16, kUniMaxParts); }

template <typename T>
static hipError_t launch_uniform_t(hipStream_t st, const T* x, int64_t n, int bin_num, UniPartial* part,
                                   void* payload, QuantLut* lut, int* qflags) {
    const int np = uniform_partials(n);
    hipLaunchKernelGGL(k_uni_minmax<T>, dim3(np), dim3(256), 0, st, x, n, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_uni_finish<T>, dim3(1), dim3(256), 0, st, x, n, part, np, bin_num,
                       reinterpret_cast<uint8_t*>(payload), lut, qflags);
    return hipGetLastError();
}

hipError_t launch_uniform(hipStream_t st, const float* x, int64_t n, int bin_num, UniPartial* part, void* payload,
                          QuantLut* lut, int* qflags) {
    return launch_uniform_t<float>(st, x, n, bin_num, part, payload, lut, qflags);
}
hipError_t launch_uniform64(hipStream_t st, const double* x, int64_t n, int bin_num, UniPartial* part,
                            void* payload, QuantLut* lut, int* qflags) {
    return launch_uniform_t<double>(st, x, n, bin_num, part, payload, lut, qflags);
}

// =============================================================================================
// parallelQuantize over fp64 slices: record export and the in-order HeapQuantileSketch.merge
// (see k_sketch_merge in skml_sketch.hip; HeapQuantileSketch.java:186-228).  The merged state is
// written in the summary's layout and k_summary64 runs on it.
// =============================================================================================
__global__ __launch_bounds__(512) void k_sketch_record64(const double* __restrict__ x, int64_t n,
                                                         const LeafPartial64* __restrict__ part, int64_t nparts,
                                                         const double* __restrict__ roots, SketchRecord64* rec) {
    __shared__ unsigned long long s_mn, s_mx;
    __shared__ uint32_t s_fl;
    const int t = threadIdx.x, T = blockDim.x;
    const int64_t chunks = n / kChunk;
    const int tail = (int)(n - chunks * kChunk);
    const double* xt = x + chunks * kChunk;
    if (t == 0) {
        s_mn = ~0ull;
        s_mx = 0ull;
        s_fl = 0u;
    }
    __syncthreads();
    uint64_t mn = ~0ull, mx = 0ull;
    uint32_t fl = 0u;
    for (int64_t i = t; i < nparts; i += T) {
        const LeafPartial64 p = part[i];
        mn = p.min_key < mn ? p.min_key : mn;
        mx = p.max_key > mx ? p.max_key : mx;
        fl |= p.flags;
    }
    for (int i = t; i < tail; i += T) {
        const uint64_t b = (uint64_t)__double_as_longlong(xt[i]);
        fl |= is_nan64(b) ? 1u : 0u;
        const uint64_t k = d2key(b);
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
        rec->tail[i] = xt[i];
    }
    atomicMin(&s_mn, (unsigned long long)mn);
    atomicMax(&s_mx, (unsigned long long)mx);
    if (fl) atomicOr(&s_fl, fl);
    for (int l = 0; l < kMaxLevels; l++)
        if ((chunks >> l) & 1)
            for (int i = t; i < kK; i += T) rec->level[l][i] = roots[(size_t)l * kK + i];
    __syncthreads();
    if (t == 0) {
        rec->n = n;
        rec->mm = LeafPartial64{s_mn, s_mx, s_fl, 0u};
    }
}

hipError_t launch_sketch_record64(hipStream_t st, const double* x, int64_t n, const LeafPartial64* part,
                                  int64_t nparts, const double* roots, SketchRecord64* rec) {
    hipLaunchKernelGGL(k_sketch_record64, dim3(1), dim3(512), 0, st, x, n, part, nparts, roots, rec);
    return hipGetLastError();
}

__global__ __launch_bounds__(512) void k_sketch_merge64(const SketchRecord64* __restrict__ recs, int nrec,
                                                        uint64_t s0, uint64_t bit0,
                                                        const uint64_t* __restrict__ tab, double* g_roots,
                                                        double* g_tail, LeafPartial64* g_part) {
    __shared__ double lv[kMaxLevels][kK];
    __shared__ double base[kChunk];
    __shared__ double tmp[kChunk];
    const int t = threadIdx.x;
    uint64_t pattern = 0, bit = bit0;
    int64_t nacc = 0;
    int base_cnt = 0;
    auto first_free = [&](int from) {
        int l = from;
        while ((pattern >> l) & 1ull) l++;
        return l;
    };
    // levelwisePropagation: mergeArrays (IEEE `<`, a tie emits the carried node first) + compact
    auto carry = [&](int from, int dest) {
        for (int l = from; l < dest; l++) {
            const uint32_t odd = lcg_bit(tab, s0, bit++);
            if (t < kChunk) {
                double v;
                int pos;
                if (t < kK) {
                    v = lv[l][t];
                    pos = t + count_le64(lv[dest], v);
                } else {
                    v = lv[dest][t - kK];
                    pos = (t - kK) + count_lt64(lv[l], v);
                }
                if (((uint32_t)pos & 1u) == odd) tmp[pos >> 1] = v;
            }
            __syncthreads();
            if (t < kK) lv[dest][t] = tmp[t];
            __syncthreads();
        }
    };
    auto flush_base = [&]() {
        if (t < kChunk) {
            const double v = base[t];
            const uint64_t kv = dk(v);
            int rank = 0;
            for (int j = 0; j < kChunk; j++) {
                const uint64_t kj = dk(base[j]);
                rank += (kj < kv) || (kj == kv && j < t);
            }
            tmp[rank] = v;
        }
        __syncthreads();
        const int dest = first_free(0);
        const uint32_t odd = lcg_bit(tab, s0, bit++);
        if (t < kK) lv[dest][t] = tmp[2 * t + odd];
        __syncthreads();
        carry(0, dest);
        pattern += 1;
        base_cnt = 0;
    };
    for (int r = 0; r < nrec; r++) {
        const SketchRecord64* R = recs + r;
        const int64_t rn = R->n;
        if (rn <= 0) continue;
        const uint64_t rpat = (uint64_t)(rn / kChunk);
        const int rtail = (int)(rn % kChunk);
        if (nacc == 0) {
            for (int l = 0; l < kMaxLevels; l++)
                if ((rpat >> l) & 1ull)
                    if (t < kK) lv[l][t] = R->level[l][t];
            if (t < rtail) base[t] = R->tail[t];
            __syncthreads();
            pattern = rpat;
            base_cnt = rtail;
            nacc = rn;
            continue;
        }
        for (int i = 0; i < rtail;) {
            const int take = min(rtail - i, kChunk - base_cnt);
            if (t < take) base[base_cnt + t] = R->tail[i + t];
            __syncthreads();
            base_cnt += take;
            i += take;
            if (base_cnt == kChunk) flush_base();
        }
        for (int l = 0; l < kMaxLevels; l++) {
            if (!((rpat >> l) & 1ull)) continue;
            const int dest = first_free(l);
            if (t < kK) lv[dest][t] = R->level[l][t];
            __syncthreads();
            carry(l, dest);
            pattern += 1ull << l;
        }
        nacc += rn;
    }
    for (int l = 0; l < kMaxLevels; l++)
        if ((pattern >> l) & 1ull)
            if (t < kK) g_roots[(size_t)l * kK + t] = lv[l][t];
    if (t < base_cnt) g_tail[t] = base[t];
    for (int r = t; r < nrec; r += blockDim.x) g_part[r] = recs[r].mm;
}

hipError_t launch_sketch_merge64(hipStream_t st, const SketchRecord64* recs, int nrec, uint64_t s0, uint64_t bit0,
                                 const uint64_t* jump_tab, double* roots, double* tail, LeafPartial64* part) {
    hipLaunchKernelGGL(k_sketch_merge64, dim3(1), dim3(512), 0, st, recs, nrec, s0, bit0, jump_tab, roots, tail,
                       part);
    return hipGetLastError();
}

}  // namespace skml
