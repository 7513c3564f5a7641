// skml_dense.hip -- CDNA4 (gfx950) kernels of the dense codec's memory-bound passes:
//   k_quantize   bins = indexOf(x) (Quantizer.java:49-92) as a branchless Eytzinger search over an
//                LDS split table, packed codes.  HBM-bound: 4 B in + code_bits/8 out per value.
//   k_decode     values[bins[i]] (DenseVectorCompressor.java:84-91), LUT in LDS; k_decode_sum,
//                k_bins, k_ref_body / k_pack_ref (Quantizer.writeObject/readObject), k_times_by.
// The sketch build (leaf / merge / summary) lives in skml_sketch.hip.
#include <algorithm>

#include "skml_device.hpp"

namespace skml {

// =============================================================================================
// Quantize: Eytzinger search over the LDS split table; codes packed LSB-first.
// =============================================================================================
#ifndef SKML_Q_THREADS
#define SKML_Q_THREADS 256
#endif
#ifndef SKML_Q_GRID
#define SKML_Q_GRID 1024
#endif
constexpr int kQThreads = SKML_Q_THREADS;
constexpr int kEytzMax = 4096;

__device__ __forceinline__ void store_codes4(uint8_t* codes, int64_t e0, uint32_t c0, uint32_t c1,
                                             uint32_t c2, uint32_t c3, int bits, int lane) {
    // e0 is a multiple of 4; lanes l and l^1 cover adjacent 4-element groups
    switch (bits) {
        case 8:  // codes are written once and read by the next pass at the earliest: stream past L2
            __builtin_nontemporal_store(c0 | (c1 << 8) | (c2 << 16) | (c3 << 24),
                                        reinterpret_cast<uint32_t*>(codes + e0));
            break;
        case 16:
            *reinterpret_cast<uint2*>(codes + e0 * 2) = make_uint2(c0 | (c1 << 16), c2 | (c3 << 16));
            break;
        case 4:
            *reinterpret_cast<uint16_t*>(codes + e0 / 2) = (uint16_t)(c0 | (c1 << 4) | (c2 << 8) | (c3 << 12));
            break;
        case 2:
            __builtin_nontemporal_store((uint8_t)(c0 | (c1 << 2) | (c2 << 4) | (c3 << 6)), codes + e0 / 4);
            break;
        default: {  // 1 bit: pair with the neighbour lane into one byte
            const uint32_t nib = c0 | (c1 << 1) | (c2 << 2) | (c3 << 3);
            const uint32_t other = lane_xor<1>(nib);
            if ((lane & 1) == 0) codes[e0 / 8] = (uint8_t)(nib | (other << 4));
            break;
        }
    }
}

// Search modes of the quantize pass, chosen per launch from the header and the bucket LUT:
//   kModeLut<S>  bin = base[key >> 18] then S bisection steps over the LDS split table
//   kModeEytz    branchless Eytzinger descent over the LDS split table (cmax too large)
//   kModeGlobal  binary search over the payload's double splits (> 4095 splits)
// All compare the float value against splits rounded toward +inf, which is exact (see
// build_quant_lut); NaN values take Quantizer.indexOf's NaN bin.
constexpr int kModeEytz = 8, kModeGlobal = 9, kModeJava = 10;

struct QuantTables {
    const uint16_t* base;  // LDS bucket bases
    const float* S;        // LDS splits (+NaN padding), or Eytzinger array
    const double* sp;      // payload splits (global / Java mode)
    int nsplit, levels, zero;
    uint32_t P, nan_bin;
};

template <int MODE>
__device__ __forceinline__ uint32_t quant_bin(const QuantTables& q, float xv) {
    uint32_t bin;
    if constexpr (MODE <= 4) {
        bin = q.base[f2key(__float_as_uint(xv)) >> (32 - kLutBits)];
#pragma unroll
        for (int h = (1 << MODE) >> 1; h > 0; h >>= 1) bin += q.S[bin + h - 1] <= xv ? (uint32_t)h : 0u;
    } else if constexpr (MODE == kModeJava) {
        return java_index_of(q.sp, q.nsplit + 1, q.zero, (double)xv);
    } else if constexpr (MODE == kModeEytz) {
        uint32_t i = 1;
        for (int s = 0; s < q.levels; s++) i = 2 * i + (q.S[i] <= xv ? 1u : 0u);
        bin = i - q.P;
    } else {
        int lo = 0, hi = q.nsplit;
        const double xd = (double)xv;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (q.sp[mid] <= xd) lo = mid + 1;
            else hi = mid;
        }
        bin = (uint32_t)lo;
    }
    return xv == xv ? bin : q.nan_bin;
}

// Code store forms for 8-bit codes (SKML_Q_STORE, A/B builds): 0 (default) a 4-byte nontemporal
// store per lane and group of 4 codes; 1 / 2 the wave's 1,024 codes of a tile transposed through
// 1 KB of LDS (lane l then holds codes 16 l .. 16 l + 15) and stored as one 16-byte nontemporal (1)
// or write-through sc1 (2) store per lane.  Write-through leaves no dirty lines in the XCD's L2 for
// the end-of-kernel write-back (the ~10 us idle gap before the next encode's leaf, tools/trace_gaps.py),
// but the form measured 224 -> 246 us per 2^28 quantize (profiles/r05c_bench.json).
#ifndef SKML_Q_STORE
#define SKML_Q_STORE 0
#endif
constexpr int kQStageWords = 256;  // per wave: 1,024 one-byte codes

template <int MODE>
__device__ __forceinline__ void quant_tiles(const QuantTables& q, const float* __restrict__ x, int64_t n,
                                            uint8_t* __restrict__ codes, int bits, uint32_t* __restrict__ stage) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves_total = (int64_t)gridDim.x * (kQThreads / 64);
    const int64_t wave_id = (int64_t)blockIdx.x * (kQThreads / 64) + (threadIdx.x >> 6);
    const int64_t full_tiles = n / 1024;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    // software-pipelined: the next tile's 4 KiB is in flight while this one is binned
    f32x4 f[4];
    if (wave_id < full_tiles) {
        const f32x4* src = reinterpret_cast<const f32x4*>(x + wave_id * 1024);
#pragma unroll
        for (int j = 0; j < 4; j++) f[j] = __builtin_nontemporal_load(src + j * 64 + lane);
    }
    // codes are < 4 GB past `codes` (n < 2^31): one buffer descriptor, 32-bit offsets
    const bool wt = SKML_Q_STORE != 0 && bits == 8 && (reinterpret_cast<uintptr_t>(codes) & 15) == 0;
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        codes, 0, (int)std::min<int64_t>(full_tiles * 1024, (int64_t)0x7FFFFC00), 0x00020000);
    for (int64_t tile = wave_id; tile < full_tiles; tile += nwaves_total) {
        f32x4 g[4];
        const int64_t next = tile + nwaves_total;
        if (next < full_tiles) {
            const f32x4* src = reinterpret_cast<const f32x4*>(x + next * 1024);
#pragma unroll
            for (int j = 0; j < 4; j++) g[j] = __builtin_nontemporal_load(src + j * 64 + lane);
        }
        if (wt) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c0 = quant_bin<MODE>(q, f[j].x), c1 = quant_bin<MODE>(q, f[j].y);
                const uint32_t c2 = quant_bin<MODE>(q, f[j].z), c3 = quant_bin<MODE>(q, f[j].w);
                stage[j * 64 + lane] = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
            }
            __builtin_amdgcn_wave_barrier();
            const uint4 w = reinterpret_cast<const uint4*>(stage)[lane];
            __builtin_amdgcn_wave_barrier();  // the stage is read before the next tile overwrites it
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{w.x, w.y, w.z, w.w}, crs, (int)(tile * 1024 + lane * 16), 0,
                                                   SKML_Q_STORE == 2 ? 16 /* sc1: write-through */ : 2 /* nt */);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c0 = quant_bin<MODE>(q, f[j].x), c1 = quant_bin<MODE>(q, f[j].y);
                const uint32_t c2 = quant_bin<MODE>(q, f[j].z), c3 = quant_bin<MODE>(q, f[j].w);
                store_codes4(codes, tile * 1024 + j * 256 + lane * 4, c0, c1, c2, c3, bits, lane);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) f[j] = g[j];
    }
    // tail tile (n % 1024 values), one wave, guarded element loads
    if (wave_id == full_tiles % nwaves_total && n % 1024) {
        const int64_t base = full_tiles * 1024;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t e0 = base + j * 256 + lane * 4;
            uint32_t c[4] = {0, 0, 0, 0};
            for (int e = 0; e < 4; e++)
                if (e0 + e < n) c[e] = quant_bin<MODE>(q, x[e0 + e]);
            if (bits == 1) {
                const int64_t pair0 = base + j * 256 + (lane & ~1) * 4;
                const uint32_t nib = c[0] | (c[1] << 1) | (c[2] << 2) | (c[3] << 3);
                const uint32_t other = lane_xor<1>(nib);
                if ((lane & 1) == 0 && pair0 < n) codes[pair0 / 8] = (uint8_t)(nib | (other << 4));
            } else if (e0 < n) {
                store_codes4(codes, e0, c[0], c[1], c[2], c[3], bits, lane);
            }
        }
    }
}

// Dynamic LDS: [0, 32 KB) bucket bases, then `lds_splits` floats (LUT mode); Eytzinger mode
// reuses the start of the same buffer (P <= 4096 floats).
__global__ __launch_bounds__(kQThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_quantize(const float* __restrict__ x, int64_t n,
                                                        uint8_t* __restrict__ payload,
                                                        const QuantLut* __restrict__ lut, int lds_splits) {
    extern __shared__ __align__(16) uint8_t qsm[];
    __shared__ __align__(16) uint32_t qstage[kQThreads / 64][kQStageWords];
    const skml_dense_header* hdr = reinterpret_cast<const skml_dense_header*>(payload);
    if (hdr->status != SKML_OK) return;
    const int bins = hdr->bin_num, bits = hdr->code_bits, nsplit = bins - 1;
    const double* sp = reinterpret_cast<const double*>(payload + kHeaderBytes);
    uint8_t* codes = payload + hdr->codes_offset;
    QuantTables q;
    q.sp = sp;
    q.nsplit = nsplit;
    q.nan_bin = (uint32_t)nan_bin_for(bins, hdr->zero_idx);
    q.zero = hdr->zero_idx;
    q.P = 1;
    q.levels = 0;
    while (q.P < (uint32_t)bins) {
        q.P <<= 1;
        q.levels++;
    }
    const int cmax = lut ? lut->cmax : -1;
    int mode;
    if (cmax == kLutJavaMode) {
        mode = kModeJava;
    } else if (cmax >= 0 && nsplit + kLutPad <= lds_splits) {
        mode = cmax == 0 ? 0 : 32 - __clz((uint32_t)cmax);  // bisection steps: ceil(log2(cmax+1))
        uint16_t* base = reinterpret_cast<uint16_t*>(qsm);
        float* S = reinterpret_cast<float*>(qsm + sizeof(lut->base));
        const uint4* src = reinterpret_cast<const uint4*>(lut->base);
        for (int i = threadIdx.x; i < (int)(sizeof(lut->base) / 16); i += kQThreads)
            reinterpret_cast<uint4*>(base)[i] = src[i];
        for (int i = threadIdx.x; i < nsplit + kLutPad; i += kQThreads)
            S[i] = i < nsplit ? __double2float_ru(sp[i]) : __uint_as_float(0x7FC00000u);
        q.base = base;
        q.S = S;
    } else if (q.P <= kEytzMax) {
        mode = kModeEytz;
        float* E = reinterpret_cast<float*>(qsm);
        for (uint32_t i = threadIdx.x + 1; i < q.P; i += kQThreads) {
            const int d = 31 - __clz(i);
            const uint32_t idx = ((2u * (i - (1u << d)) + 1u) << (q.levels - 1 - d)) - 1u;
            E[i] = idx < (uint32_t)nsplit ? __double2float_ru(sp[idx]) : __uint_as_float(0x7FC00000u);
        }
        q.S = E;
    } else {
        mode = kModeGlobal;
    }
    __syncthreads();
    switch (mode) {
        case 0: quant_tiles<0>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        case 1: quant_tiles<1>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        case 2: quant_tiles<2>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        case 3: quant_tiles<3>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        case 4: quant_tiles<4>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        case kModeEytz: quant_tiles<kModeEytz>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        case kModeJava: quant_tiles<kModeJava>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
        default: quant_tiles<kModeGlobal>(q, x, n, codes, bits, qstage[threadIdx.x >> 6]); break;
    }
}

static int quant_grid(int64_t n) {
    const int64_t tiles = (n + 1023) / 1024;
    int64_t wg = (tiles + 3) / 4;
    if (wg > 4096) wg = 4096;
    if (wg < 1) wg = 1;
    return (int)wg;
}

hipError_t launch_quantize(hipStream_t st, const float* x, int64_t n, void* payload, const QuantLut* lut,
                           int req_bins) {
    if (n <= 0) return hipSuccess;
    // LDS sized for this request's split table; persistent-style grid (the LUT is loaded once per WG)
    const int lds_splits = std::min(std::max(req_bins - 1, 1), kLutMaxSplits) + kLutPad;
    const size_t lds = sizeof(QuantLut::base) + (size_t)lds_splits * sizeof(float);
    const int64_t tiles = (n + 1023) / 1024;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((tiles + 3) / 4, SKML_Q_GRID));
    hipLaunchKernelGGL(k_quantize, dim3(grid), dim3(kQThreads), lds, st, x, n,
                       reinterpret_cast<uint8_t*>(payload), lut, lds_splits);
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
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    for (int64_t tile = wid; tile < full; tile += nw) {
        f32x4* dst = reinterpret_cast<f32x4*>(out + tile * 1024);
        uint32_t c[4][4];
#pragma unroll
        for (int j = 0; j < 4; j++) read_codes4(codes, tile * 1024 + j * 256 + lane * 4, bits, c[j]);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            f32x4 o;
            if (lds) o = f32x4{lut[c[j][0]], lut[c[j][1]], lut[c[j][2]], lut[c[j][3]]};
            else o = f32x4{(float)lut_value(h, sp, c[j][0]), (float)lut_value(h, sp, c[j][1]),
                           (float)lut_value(h, sp, c[j][2]), (float)lut_value(h, sp, c[j][3])};
            // the decoded gradient is written once and not re-read by this pass: stream it past L2
            __builtin_nontemporal_store(o, dst + j * 64 + lane);
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

// Fused decode of P payloads + sum in double (Gradient.sum adds doubles) + scale.  Payloads of at
// most kSumLutBins bins look their values up in an LDS table; wider ones (16-bit codes) compute
// the midpoint from the payload's splits, as k_decode does above kLutMax.
constexpr int kMaxSumPayloads = 16;
constexpr int kSumLutBins = 256;
// 16 consecutive codes of one payload starting at e0 (a multiple of 16): one load of 2..32 bytes.
__device__ __forceinline__ void load_codes16(const uint8_t* codes, int64_t e0, int bits, uint32_t (&w)[8]) {
    switch (bits) {
        case 8: {
            const uint4 v = *reinterpret_cast<const uint4*>(codes + e0);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            break;
        }
        case 16: {
            const uint4 a = *reinterpret_cast<const uint4*>(codes + 2 * e0);
            const uint4 b = *reinterpret_cast<const uint4*>(codes + 2 * e0 + 16);
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
            break;
        }
        case 4: {
            const uint2 v = *reinterpret_cast<const uint2*>(codes + e0 / 2);
            w[0] = v.x; w[1] = v.y;
            break;
        }
        case 2: w[0] = *reinterpret_cast<const uint32_t*>(codes + e0 / 4); break;
        default: w[0] = *reinterpret_cast<const uint16_t*>(codes + e0 / 8); break;
    }
}
__device__ __forceinline__ uint32_t code16_at(const uint32_t (&w)[8], int e, int bits) {
    switch (bits) {
        case 8: return (w[e >> 2] >> (8 * (e & 3))) & 255u;
        case 16: return (w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
        case 4: return (w[e >> 3] >> (4 * (e & 7))) & 15u;
        case 2: return (w[0] >> (2 * e)) & 3u;
        default: return (w[0] >> e) & 1u;
    }
}

// The payload headers are read once per workgroup into LDS (codes pointer, code width, LUT row).
// Each lane owns 16 consecutive elements per step: it issues the code loads of up to 8 payloads
// first (one 16-byte load per payload at 8 bits), then adds their LUT values in payload order
// into 16 double accumulators (Gradient.sum adds doubles in gradient order), the next 8 payloads
// likewise, and stores 64 contiguous bytes of fp32 (nontemporal).  BITS: the code width when all
// payloads share it (the common case: one bin count), 0 = per payload.
constexpr int kSumChunk = 8;
template <int BITS>
__global__ __launch_bounds__(256) void k_decode_sum(const uint8_t* __restrict__ payloads, int P,
                                                    size_t stride, float* __restrict__ out, int64_t n,
                                                    double scale) {
    __shared__ double lut[kMaxSumPayloads][kSumLutBins];
    __shared__ const uint8_t* s_codes[kMaxSumPayloads];
    __shared__ int s_bits[kMaxSumPayloads], s_lds[kMaxSumPayloads];
    for (int p = 0; p < P; p++) {
        const uint8_t* pl = payloads + (size_t)p * stride;
        const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(pl);
        const double* sp = reinterpret_cast<const double*>(pl + kHeaderBytes);
        const bool in_lds = h->bin_num <= kSumLutBins;
        if (threadIdx.x == 0) {
            s_codes[p] = pl + h->codes_offset;
            s_bits[p] = h->code_bits;
            s_lds[p] = in_lds ? 1 : 0;
        }
        if (in_lds)
            for (int b = threadIdx.x; b < h->bin_num; b += 256) lut[p][b] = lut_value(h, sp, b);
    }
    __syncthreads();
    bool all_lds = true;
    for (int p = 0; p < P; p++) all_lds &= s_lds[p] != 0;
    auto value = [&](int p, uint32_t c) -> double {
        if (all_lds || s_lds[p]) return lut[p][c];
        const uint8_t* pl = payloads + (size_t)p * stride;
        return lut_value(reinterpret_cast<const skml_dense_header*>(pl),
                         reinterpret_cast<const double*>(pl + kHeaderBytes), (int)c);
    };
    const int64_t full = n / 16;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const int64_t gstep = (int64_t)gridDim.x * 256;
    if (BITS && P <= kSumChunk) {
        // software-pipelined: the next step's code loads are issued before this step's lookups, so
        // a wave waits on HBM once per kernel instead of once per step
        uint32_t wn[kSumChunk][8];
        int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
#pragma unroll
        for (int q = 0; q < kSumChunk; q++)
            if (q < P && g < full) load_codes16(s_codes[q], g * 16, BITS, wn[q]);
        for (; g < full; g += gstep) {
            constexpr int kW = BITS >= 2 ? BITS / 2 : 1;  // code words per payload per step
            uint32_t w[kSumChunk][8];
#pragma unroll
            for (int q = 0; q < kSumChunk; q++)
#pragma unroll
                for (int k = 0; k < kW; k++) w[q][k] = wn[q][k];
            if (g + gstep < full) {
#pragma unroll
                for (int q = 0; q < kSumChunk; q++)
                    if (q < P) load_codes16(s_codes[q], (g + gstep) * 16, BITS, wn[q]);
            }
            double acc[16];
#pragma unroll
            for (int e = 0; e < 16; e++) acc[e] = 0.0;
#pragma unroll
            for (int q = 0; q < kSumChunk; q++) {
                if (q >= P) break;
#pragma unroll
                for (int e = 0; e < 16; e++) acc[e] += value(q, code16_at(w[q], e, BITS));
            }
            f32x4* dst = reinterpret_cast<f32x4*>(out + g * 16);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const f32x4 o = {(float)(acc[4 * j] * scale), (float)(acc[4 * j + 1] * scale),
                                 (float)(acc[4 * j + 2] * scale), (float)(acc[4 * j + 3] * scale)};
                __builtin_nontemporal_store(o, dst + j);
            }
        }
    } else
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < full; g += gstep) {
        const int64_t e0 = g * 16;
        double acc[16];
#pragma unroll
        for (int e = 0; e < 16; e++) acc[e] = 0.0;
        for (int p0 = 0; p0 < P; p0 += kSumChunk) {
            uint32_t w[kSumChunk][8];
#pragma unroll
            for (int q = 0; q < kSumChunk; q++)
                if (p0 + q < P)
                    load_codes16(s_codes[p0 + q], e0, BITS ? BITS : __builtin_amdgcn_readfirstlane(s_bits[p0 + q]),
                                 w[q]);
#pragma unroll
            for (int q = 0; q < kSumChunk; q++) {
                if (p0 + q >= P) break;
                const int bits = BITS ? BITS : __builtin_amdgcn_readfirstlane(s_bits[p0 + q]);
#pragma unroll
                for (int e = 0; e < 16; e++) acc[e] += value(p0 + q, code16_at(w[q], e, bits));
            }
        }
        f32x4* dst = reinterpret_cast<f32x4*>(out + e0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const f32x4 o = {(float)(acc[4 * j] * scale), (float)(acc[4 * j + 1] * scale),
                             (float)(acc[4 * j + 2] * scale), (float)(acc[4 * j + 3] * scale)};
            __builtin_nontemporal_store(o, dst + j);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 16) {  // the last n % 16 elements
        const int64_t e = full * 16 + threadIdx.x;
        if (e < n) {
            double a = 0.0;
            for (int p = 0; p < P; p++) a += value(p, read_code(s_codes[p], e, s_bits[p]));
            out[e] = (float)(a * scale);
        }
    }
}

// Occupancy form (one code width, at most 8 payloads of at most 256 bins): each lookup is a random
// ds_read_b64, and a wave keeps at most 15 LDS reads in flight (lgkmcnt), so the sum runs at the
// rate the resident waves can keep lookups in flight (r04 counters: LDS array busy 22 % of the
// time, VALU 14 %).  Bank-replicated tables (16 interleaved copies, one workgroup per CU) halved
// the bank conflicts and ran slower (412 against 355 us at C4) for the same reason.  Here a lane
// owns 8 elements (half the registers of k_decode_sum: 8 waves per SIMD), the tables take
// P x bins doubles of dynamic LDS instead of a 32 KB array, and the next step's codes are loaded
// before this step's lookups.
#ifndef SKML_OCC_WAVES
#define SKML_OCC_WAVES 4  // waves per SIMD of the prefetching form, 8- and 16-bit codes (4 against 6 and 8: profiles/ab/r06_occ_waves.txt)
#endif
#ifndef SKML_OCC_WAVES_NARROW
// the same for 1-, 2- and 4-bit codes: a step then loads 1-4 bytes per payload and lane, so the
// codes need more waves in flight (C5's 2-bit sum ran 154 us at 6 and 253 us at 4, profiles/ab/r06_occ_narrow.txt)
#define SKML_OCC_WAVES_NARROW 6
#endif
#ifndef SKML_OCC_PER
#define SKML_OCC_PER 8  // elements per lane and step (A/B builds: 16)
#endif
constexpr int kOccPer = SKML_OCC_PER, kOccMaxP = 8;
static_assert(kOccPer == 8 || kOccPer == 16, "8 or 16 elements per lane");
// dynamic LDS of the P tables: what is left of the 64 KB a launch may take without opting in
// after the kernel's static array of code pointers
constexpr size_t kOccLdsMax = 64 * 1024 - sizeof(const uint8_t*) * kOccMaxP;
// code words one lane holds per payload and step
template <int BITS>
constexpr int occ_words() { return kOccPer * BITS >= 32 ? kOccPer * BITS / 32 : 1; }
// The code loads go through a global (address space 1) pointer: the payloads' code pointers sit in
// LDS, and loads through a generic pointer would be flat loads, which count on lgkmcnt too, so the
// table lookups' LDS waits would also wait for the next step's prefetched codes.
#define SKML_G(T) const __attribute__((address_space(1))) T*
template <int BITS>
__device__ __forceinline__ void load_codes_occ(const uint8_t* codes_any, int64_t e0, uint32_t (&w)[occ_words<BITS>()]) {
    SKML_G(uint8_t) codes = (SKML_G(uint8_t))codes_any;
    constexpr int kBytes = kOccPer * BITS / 8;  // e0 is a multiple of kOccPer: aligned to kBytes
    const int64_t b0 = e0 * BITS / 8;
    typedef uint32_t u32x4_g __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2_g __attribute__((ext_vector_type(2)));
    if constexpr (kBytes >= 16) {
#pragma unroll
        for (int q = 0; q < kBytes / 16; q++) {
            const u32x4_g v = *(SKML_G(u32x4_g))(codes + b0 + 16 * q);
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
    } else if constexpr (kBytes == 8) {
        const u32x2_g v = *(SKML_G(u32x2_g))(codes + b0);
        w[0] = v.x; w[1] = v.y;
    } else if constexpr (kBytes == 4) {
        w[0] = *(SKML_G(uint32_t))(codes + b0);
    } else if constexpr (kBytes == 2) {
        w[0] = *(SKML_G(uint16_t))(codes + b0);
    } else {
        w[0] = codes[b0];
    }
}
#undef SKML_G
template <int BITS>
__device__ __forceinline__ uint32_t code_occ_at(const uint32_t (&w)[occ_words<BITS>()], int e) {
    return (w[(e * BITS) >> 5] >> ((e * BITS) & 31)) & ((1u << BITS) - 1u);
}
template <int BITS, bool PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PF ? (BITS >= 8 ? SKML_OCC_WAVES : SKML_OCC_WAVES_NARROW) : 8))) void k_decode_sum_occ(
    const uint8_t* __restrict__ payloads, int P, size_t stride, float* __restrict__ out, int64_t n, double scale,
    int tab) {
    extern __shared__ double lt[];  // P tables of `tab` doubles
    __shared__ const uint8_t* s_codes[kOccMaxP];
    for (int p = 0; p < P; p++) {
        const uint8_t* pl = payloads + (size_t)p * stride;
        const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(pl);
        const double* sp = reinterpret_cast<const double*>(pl + kHeaderBytes);
        if (threadIdx.x == 0) s_codes[p] = pl + h->codes_offset;
        for (int b = threadIdx.x; b < h->bin_num; b += 256) lt[p * tab + b] = lut_value(h, sp, b);
    }
    __syncthreads();
    constexpr int kW = occ_words<BITS>();  // code words per payload per step
    const int64_t full = n / kOccPer, gstep = (int64_t)gridDim.x * 256;
    int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t wn[kOccMaxP][kW];
    if (PF) {
#pragma unroll
        for (int q = 0; q < kOccMaxP; q++)
            if (q < P && g < full) load_codes_occ<BITS>(s_codes[q], g * kOccPer, wn[q]);
    }
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    for (; g < full; g += gstep) {
        uint32_t w[kOccMaxP][kW];
        if (PF) {
#pragma unroll
            for (int q = 0; q < kOccMaxP; q++)
#pragma unroll
                for (int k = 0; k < kW; k++) w[q][k] = wn[q][k];
            if (g + gstep < full) {
#pragma unroll
                for (int q = 0; q < kOccMaxP; q++)
                    if (q < P) load_codes_occ<BITS>(s_codes[q], (g + gstep) * kOccPer, wn[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < kOccMaxP; q++)
                if (q < P) load_codes_occ<BITS>(s_codes[q], g * kOccPer, w[q]);
        }
        double acc[kOccPer];
#pragma unroll
        for (int e = 0; e < kOccPer; e++) acc[e] = 0.0;
#pragma unroll
        for (int q = 0; q < kOccMaxP; q++) {
            if (q >= P) break;
            const double* t = lt + q * tab;
#pragma unroll
            for (int e = 0; e < kOccPer; e++) acc[e] += t[code_occ_at<BITS>(w[q], e)];
        }
        f32x4* dst = reinterpret_cast<f32x4*>(out + g * kOccPer);
#pragma unroll
        for (int j = 0; j < kOccPer / 4; j++) {
            const f32x4 o = {(float)(acc[4 * j] * scale), (float)(acc[4 * j + 1] * scale),
                             (float)(acc[4 * j + 2] * scale), (float)(acc[4 * j + 3] * scale)};
            __builtin_nontemporal_store(o, dst + j);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < kOccPer) {  // the last n % kOccPer elements
        const int64_t e = full * kOccPer + threadIdx.x;
        if (e < n) {
            double a = 0.0;
            for (int p = 0; p < P; p++) a += lt[p * tab + read_code(s_codes[p], e, BITS)];
            out[e] = (float)(a * scale);
        }
    }
}

template <int BITS>
hipError_t launch_occ(hipStream_t st, const uint8_t* pl, int P, size_t stride, float* out, int64_t n, double scale,
                      int max_bins) {
    const size_t lds = sizeof(double) * (size_t)max_bins * (size_t)P;
    const int64_t groups = n / kOccPer;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((groups + 255) / 256, 4096));
#ifdef SKML_AB
    if (form(SKML_FORM_DECODE_SUM) == 2) {  // A/B: without the next step's prefetch (slower)
        hipLaunchKernelGGL((k_decode_sum_occ<BITS, false>), dim3(grid), dim3(256), lds, st, pl, P, stride, out, n, scale,
                           max_bins);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL((k_decode_sum_occ<BITS, true>), dim3(grid), dim3(256), lds, st, pl, P, stride, out, n, scale,
                       max_bins);
    return hipGetLastError();
}

hipError_t launch_decode_sum(hipStream_t st, const void* payloads, int P, size_t stride, float* out,
                             int64_t n, double scale, int common_bits, int max_bins) {
    if (n <= 0) return hipSuccess;
    if (P < 1 || P > kMaxSumPayloads) return hipErrorInvalidValue;
    // the occupancy form whenever the P tables fit beside its static LDS: every 1..8-bit shape
    // (<= 256 bins), and 16-bit codes up to 8 x 1,023 or 7 x 1,024 bins (8 x 1,024 take k_decode_sum)
    if ((size_t)max_bins * (size_t)P * sizeof(double) <= kOccLdsMax && P <= kOccMaxP && form(SKML_FORM_DECODE_SUM) != 1) {
        const uint8_t* pl = reinterpret_cast<const uint8_t*>(payloads);
        switch (common_bits) {
            case 16: return launch_occ<16>(st, pl, P, stride, out, n, scale, max_bins);
            case 8: return launch_occ<8>(st, pl, P, stride, out, n, scale, max_bins);
            case 4: return launch_occ<4>(st, pl, P, stride, out, n, scale, max_bins);
            case 2: return launch_occ<2>(st, pl, P, stride, out, n, scale, max_bins);
            case 1: return launch_occ<1>(st, pl, P, stride, out, n, scale, max_bins);
            default: break;  // mixed widths: the per-payload kernel below
        }
    }
    const int64_t groups = n / 16;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((groups + 255) / 256, 2048));
    const uint8_t* pl = reinterpret_cast<const uint8_t*>(payloads);
    switch (common_bits) {
        case 8: hipLaunchKernelGGL(k_decode_sum<8>, dim3(grid), dim3(256), 0, st, pl, P, stride, out, n, scale); break;
        case 2: hipLaunchKernelGGL(k_decode_sum<2>, dim3(grid), dim3(256), 0, st, pl, P, stride, out, n, scale); break;
        case 4: hipLaunchKernelGGL(k_decode_sum<4>, dim3(grid), dim3(256), 0, st, pl, P, stride, out, n, scale); break;
        case 1: hipLaunchKernelGGL(k_decode_sum<1>, dim3(grid), dim3(256), 0, st, pl, P, stride, out, n, scale); break;
        default: hipLaunchKernelGGL(k_decode_sum<0>, dim3(grid), dim3(256), 0, st, pl, P, stride, out, n, scale); break;
    }
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
// Quantizer.readObject bin stream (Quantizer.java:216-225) -> packed codes of the payload.  A bin
// outside [0, binNum) (a malformed stream; Java fails on it with ArrayIndexOutOfBounds in
// getValues) is counted in *bad and stored as 0, so no code field overflows into its neighbour.
__global__ void k_pack_ref(const uint8_t* __restrict__ body, int width, int64_t n,
                           uint8_t* __restrict__ payload, int* __restrict__ bad) {
    const skml_dense_header* h = reinterpret_cast<const skml_dense_header*>(payload);
    uint8_t* codes = payload + h->codes_offset;
    const uint32_t bins = (uint32_t)h->bin_num;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t e0 = g * 4;
    uint32_t c[4] = {0, 0, 0, 0};
    bool out_of_range = false;
    for (int e = 0; e < 4; e++) {
        const int64_t i = e0 + e;
        if (i >= n) break;
        if (width == 1) c[e] = (uint32_t)((int32_t)(int8_t)body[i] + 128);
        else if (width == 2)
            c[e] = (uint32_t)((int32_t)(int16_t)(((uint32_t)body[2 * i] << 8) | body[2 * i + 1]) + 32768);
        else
            c[e] = ((uint32_t)body[4 * i] << 24) | ((uint32_t)body[4 * i + 1] << 16) |
                   ((uint32_t)body[4 * i + 2] << 8) | body[4 * i + 3];
        if (c[e] >= bins) {
            out_of_range = true;
            c[e] = 0;
        }
    }
    if (__ballot(out_of_range) != 0 && (threadIdx.x & 63) == 0) atomicAdd(bad, 1);
    const int lane = threadIdx.x & 63;
    if (h->code_bits == 1) {
        const uint32_t nib = c[0] | (c[1] << 1) | (c[2] << 2) | (c[3] << 3);
        const uint32_t other = lane_xor<1>(nib);
        if ((lane & 1) == 0 && e0 < n) codes[e0 / 8] = (uint8_t)(nib | (other << 4));
    } else if (e0 < n) {
        store_codes4(codes, e0, c[0], c[1], c[2], c[3], h->code_bits, lane);
    }
}

hipError_t launch_pack_ref(hipStream_t st, const uint8_t* body, int width, int64_t n, void* payload, int* bad) {
    if (n <= 0) return hipSuccess;
    const int64_t groups = (n + 3) / 4;
    hipLaunchKernelGGL(k_pack_ref, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st, body,
                       width, n, reinterpret_cast<uint8_t*>(payload), bad);
    return hipGetLastError();
}
}  // namespace skml
