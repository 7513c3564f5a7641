// skml_wire.hip -- the GroupedMinMaxSketch field stream assembled and parsed on the device
// (GroupedMinMaxSketch.writeObject / readObject, GroupedMinMaxSketch.java:148-172, with
// MinMaxSketch.java:88-108, HuffmanEncoder.java:168-207 and DeltaAdaptiveEncoder.java:148-188).
//
// The stream is small fields (ints, doubles, presence bytes, Huffman items) around long arrays:
// each group's HuffmanEncoder words and its two DeltaAdaptive BitSets, written by
// ObjectOutputStream.writeLong (big-endian), each BitSet.toLongArray-trimmed of trailing zero words.
// The long arrays are >99 % of the bytes, and device-shaped work: a bit-range extraction from the
// concatenated device streams, a byte swap, and (read side) the inverse.  The host only walks the
// small fields.
//
// Write side: k_wire_lastnz finds each long array's last non-zero word (the trim), the host lays the
// stream out, k_wire_pieces copies the host-built small fields into place and k_wire_longs writes
// every long array, so the stream leaves the device with one copy.
// Read side: the stream arrives with one copy; k_rd_fixed_sum / k_rd_unary_* recover each group's
// exact DeltaAdaptive bit lengths (the trimmed BitSets do not carry them), k_rd_stream lays the
// groups' flag and delta bits out contiguously at their bit offsets and k_rd_words copies the
// Huffman words out for the device Huffman decoder.
#include <algorithm>

#include "skml_device.hpp"
#include "skml_sparse.h"

namespace skml {

// bits [b, b + 64) of a little-endian word stream (bit i = word[i >> 6] >> (i & 63)), bits at
// or beyond `avail` (relative to b) cleared.  Reads word (b >> 6) + 1 only when the range crosses it.
__device__ __forceinline__ uint64_t stream_bits(const uint64_t* __restrict__ w, int64_t b, int64_t avail) {
    const int64_t i = b >> 6;
    const int sh = (int)(b & 63);
    uint64_t v = w[i] >> sh;
    if (sh && avail > 64 - sh) v |= w[i + 1] << (64 - sh);
    if (avail < 64) v &= avail > 0 ? ((1ull << avail) - 1ull) : 0ull;
    return v;
}

// section of global word id `g` among `n` sections with word prefix `pre` (LDS, n + 1 entries)
__device__ __forceinline__ int find_section(const int64_t* pre, int n, int64_t g) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ const uint64_t* wire_src(const WireSrc& s, int which) {
    return which == 0 ? s.flags : which == 1 ? s.deltas : s.huff;
}

// ---------------------------------------------------------------- write side
// One workgroup per section, scanning back from its last word: the trim is the last non-zero
// word + 1, which a BitSet stream almost always has in its final 256 words (a per-word atomic max
// over the whole stream serialised millions of same-address atomics).
__global__ __launch_bounds__(256) void k_wire_lastnz(WireSrc src, const WireSec* __restrict__ secs,
                                                     unsigned long long* __restrict__ nz) {
    __shared__ int64_t found;
    const WireSec sc = secs[blockIdx.x];
    const uint64_t* w = wire_src(src, sc.src);
    const int64_t nw = (sc.nbits + 63) / 64;
    if (threadIdx.x == 0) found = 0;
    __syncthreads();
    for (int64_t hi = nw; hi > 0; hi -= 256) {
        const int64_t i = hi - 1 - threadIdx.x;
        int64_t mine = 0;
        if (i >= 0 && stream_bits(w, sc.bit0 + 64 * i, sc.nbits - 64 * i) != 0) mine = i + 1;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) mine = max(mine, (int64_t)__shfl_xor(mine, off, 64));
        if ((threadIdx.x & 63) == 0 && mine) atomicMax(reinterpret_cast<unsigned long long*>(&found), (unsigned long long)mine);
        __syncthreads();
        if (found) break;
        __syncthreads();
    }
    if (threadIdx.x == 0) nz[blockIdx.x] = (unsigned long long)found;
}

__global__ __launch_bounds__(256) void k_wire_longs(WireSrc src, const WireSec* __restrict__ secs,
                                                    const int64_t* __restrict__ npre, int nsec,
                                                    uint8_t* __restrict__ wire) {
    __shared__ int64_t pre[kWireMaxSec + 1];
    for (int j = threadIdx.x; j <= nsec; j += 256) pre[j] = npre[j];
    __syncthreads();
    const int64_t total = pre[nsec];
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (int64_t)gridDim.x * 256) {
        const int s = find_section(pre, nsec, g);
        const int64_t i = g - pre[s];
        const WireSec sc = secs[s];
        const uint64_t v = stream_bits(wire_src(src, sc.src), sc.bit0 + 64 * i, sc.nbits - 64 * i);
        uint8_t* d = wire + sc.dst + 8 * i;  // DataOutput.writeLong: big-endian, any byte offset
#pragma unroll
        for (int k = 0; k < 8; k++) d[k] = (uint8_t)(v >> (56 - 8 * k));
    }
}

// pieces: {src offset in `small`, dst offset in the wire, length} triples
__global__ __launch_bounds__(256) void k_wire_pieces(const uint8_t* __restrict__ small, const int64_t* __restrict__ pieces,
                                                     uint8_t* __restrict__ wire) {
    const int64_t so = pieces[3 * blockIdx.x], d = pieces[3 * blockIdx.x + 1], len = pieces[3 * blockIdx.x + 2];
    for (int64_t k = threadIdx.x; k < len; k += 256) wire[d + k] = small[so + k];
}

hipError_t launch_wire_lastnz(hipStream_t st, const WireSrc& src, const WireSec* secs, int nsec, uint64_t* nz) {
    if (nsec <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_wire_lastnz, dim3((unsigned)nsec), dim3(256), 0, st, src, secs,
                       reinterpret_cast<unsigned long long*>(nz));
    return hipGetLastError();
}
hipError_t launch_wire_longs(hipStream_t st, const WireSrc& src, const WireSec* secs, const int64_t* npre, int nsec,
                             int64_t total_words, uint8_t* wire) {
    if (total_words <= 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>((total_words + 255) / 256, 8192);
    hipLaunchKernelGGL(k_wire_longs, dim3((unsigned)grid), dim3(256), 0, st, src, secs, npre, nsec, wire);
    return hipGetLastError();
}
hipError_t launch_wire_pieces(hipStream_t st, const uint8_t* small, const int64_t* pieces, int npieces, uint8_t* wire) {
    if (npieces <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_wire_pieces, dim3((unsigned)npieces), dim3(256), 0, st, small, pieces, wire);
    return hipGetLastError();
}

// ---------------------------------------------------------------- read side
// ObjectInputStream.readLong of the word at byte p (any alignment): the big-endian long from the
// aligned words around it (two 8-byte loads and a funnel shift instead of eight byte loads).  The device copy of the stream is allocated with 16 bytes of
// slack, so the second word never lies outside it.
__device__ __forceinline__ uint64_t be64_at(const uint8_t* __restrict__ p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(a & ~static_cast<uintptr_t>(7));
    const int sh = (int)(a & 7) * 8;
    uint64_t v = q[0];
    if (sh) v = (v >> sh) | (q[1] << (64 - sh));
    return __builtin_bswap64(v);
}
// bits [q, q + 64) of a stored long array (ns words at byte pos; words past ns read as 0)
__device__ __forceinline__ uint64_t stored_bits(const uint8_t* __restrict__ stream, int64_t pos, int64_t ns, int64_t q) {
    const int64_t i = q >> 6;
    const int sh = (int)(q & 63);
    const uint64_t lo = i < ns ? be64_at(stream + pos + 8 * i) : 0ull;
    uint64_t v = lo >> sh;
    if (sh) {
        const uint64_t hi = i + 1 < ns ? be64_at(stream + pos + 8 * (i + 1)) : 0ull;
        v |= hi << (64 - sh);
    }
    return v;
}

// Fixed-width flags (flagKind false): sum over the size nf-bit fields (BinaryUtils.getBits order:
// a field's MSB at its lowest position) of the first size * nf bits: sum over residues k of
// 2^(nf-1-k) * popcount(bits at positions = k mod nf).
__device__ __forceinline__ uint64_t residue_mask(int nf, int r) {
    switch (nf) {
        case 1: return ~0ull;
        case 2: return r == 0 ? 0x5555555555555555ull : 0xAAAAAAAAAAAAAAAAull;
        case 3: return r == 0 ? 0x9249249249249249ull : r == 1 ? 0x2492492492492492ull : 0x4924924924924924ull;
        default: return 0x1111111111111111ull << r;
    }
}
__global__ __launch_bounds__(256) void k_rd_fixed_sum(const uint8_t* __restrict__ stream, const RdFlagSec* __restrict__ secs,
                                                      const int64_t* __restrict__ wpre, int nsec,
                                                      unsigned long long* __restrict__ sums) {
    __shared__ int64_t pre[kMaxGroups + 1];
    __shared__ unsigned long long ssum[kMaxGroups];  // the workgroup's per-section sums
    for (int j = threadIdx.x; j <= nsec; j += 256) pre[j] = wpre[j];
    for (int j = threadIdx.x; j < kMaxGroups; j += 256) ssum[j] = 0ull;
    __syncthreads();
    const int64_t total = pre[nsec];
    // every lane takes part in every trip (the wave reduction below)
    for (int64_t g0 = (int64_t)blockIdx.x * 256; g0 < total; g0 += (int64_t)gridDim.x * 256) {
        const int64_t g = std::min<int64_t>(g0 + threadIdx.x, total - 1);
        const bool live = g0 + threadIdx.x < total;
        const int s = find_section(pre, nsec, g);
        const int64_t i = g - pre[s];
        const RdFlagSec sc = secs[s];
        uint64_t v = (live && i < sc.nstored) ? be64_at(stream + sc.pos + 8 * i) : 0ull;
        const int64_t rem = sc.nbits - 64 * i;
        if (rem < 64) v &= rem > 0 ? ((1ull << rem) - 1ull) : 0ull;
        const int nf = sc.nf;
        // position 64 i + b has residue (ph + b) mod nf (i < 2^32: a section's word index)
        const int ph = nf > 0 ? (int)(((uint32_t)i % (uint32_t)nf) * (64u % (uint32_t)nf) % (uint32_t)nf) : 0;
        uint64_t sum = 0;
        for (int k = 0; k < nf; k++)
            sum += (uint64_t)__popcll(v & residue_mask(nf, (k - ph + nf) % nf)) << (nf - 1 - k);
        // one LDS atomic per wave when the wave's words lie in one section (all but a few waves)
        const int s0 = __builtin_amdgcn_readfirstlane(s);
        if (__all(s == s0)) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) sum += __shfl_xor(sum, off, 64);
            if ((threadIdx.x & 63) == 0 && sum) atomicAdd(&ssum[s0], (unsigned long long)sum);
        } else if (sum) {
            atomicAdd(&ssum[s], (unsigned long long)sum);
        }
    }
    // one global atomic per (workgroup, section): thousands of same-address global atomics (one
    // per wave) serialised at the memory side
    __syncthreads();
    for (int j = threadIdx.x; j < nsec; j += 256)
        if (ssum[j]) atomicAdd(&sums[j], ssum[j]);
}

// Unary flags (flagKind true): the bit length of `size` flags is the position of the size-th zero
// + 1.  Pass 1: zero counts of the stored words per tile of kRdTile words.  Pass 2 (one workgroup
// per group): the tile holding the crossing, then the word, then the bit; zeros past the stored
// words (the trimmed tail) count too.
constexpr int64_t kRdTile = kRdTileWords;
__global__ __launch_bounds__(256) void k_rd_unary_tiles(const uint8_t* __restrict__ stream, const RdFlagSec* __restrict__ secs,
                                                        const int64_t* __restrict__ tpre, int nsec,
                                                        uint32_t* __restrict__ tile_zeros) {
    __shared__ int64_t pre[kMaxGroups + 1];
    __shared__ uint32_t red[4];
    for (int j = threadIdx.x; j <= nsec; j += 256) pre[j] = tpre[j];
    __syncthreads();
    const int64_t t = blockIdx.x;  // one workgroup per tile
    const int s = find_section(pre, nsec, t);
    const RdFlagSec sc = secs[s];
    const int64_t w0 = (t - pre[s]) * kRdTile;
    uint32_t z = 0;
    for (int64_t i = w0 + threadIdx.x; i < std::min<int64_t>(w0 + kRdTile, sc.nstored); i += 256)
        z += 64u - (uint32_t)__popcll(be64_at(stream + sc.pos + 8 * i));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) z += __shfl_xor(z, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = z;
    __syncthreads();
    if (threadIdx.x == 0) tile_zeros[t] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void k_rd_unary_select(const uint8_t* __restrict__ stream,
                                                         const RdFlagSec* __restrict__ secs,
                                                         const int64_t* __restrict__ tpre,
                                                         const uint32_t* __restrict__ tile_zeros,
                                                         int64_t* __restrict__ flen) {
    __shared__ int64_t s_tile, s_before;
    __shared__ uint32_t wz[256];
    const int s = blockIdx.x;
    const RdFlagSec sc = secs[s];
    const int64_t need = sc.size;  // the size-th zero (1-based) ends the last flag
    if (threadIdx.x == 0) {
        int64_t acc = 0, tile = -1;
        for (int64_t t = tpre[s]; t < tpre[s + 1]; t++) {
            if (acc + tile_zeros[t] >= (uint64_t)need) {
                tile = t - tpre[s];
                break;
            }
            acc += tile_zeros[t];
        }
        s_tile = tile;
        s_before = acc;
    }
    __syncthreads();
    if (s_tile < 0) {  // the crossing lies in the trimmed zero tail
        if (threadIdx.x == 0) flen[s] = sc.nstored * 64 + (need - s_before);
        return;
    }
    // the tile's words, 8 per thread in order: per-thread zero counts, block scan, the crossing
    const int64_t w0 = s_tile * kRdTile;
    uint32_t cnt = 0;
    for (int k = 0; k < kRdTile / 256; k++) {
        const int64_t i = w0 + threadIdx.x * (kRdTile / 256) + k;
        if (i < sc.nstored) cnt += 64u - (uint32_t)__popcll(be64_at(stream + sc.pos + 8 * i));
    }
    wz[threadIdx.x] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t acc = s_before;
        for (int j = 0; j < 256; j++) {
            if (acc + wz[j] >= need) {
                for (int k = 0; k < kRdTile / 256; k++) {
                    const int64_t i = w0 + j * (kRdTile / 256) + k;
                    const uint64_t inv = ~be64_at(stream + sc.pos + 8 * i);
                    const int z = __popcll(inv);
                    if (acc + z >= need) {
                        uint64_t m = inv;
                        for (int64_t r = acc + 1; r < need; r++) m &= m - 1;  // drop the zeros before it
                        flen[s] = i * 64 + __ffsll((unsigned long long)m);  // position + 1
                        return;
                    }
                    acc += z;
                }
            }
            acc += wz[j];
        }
        flen[s] = -1;  // unreachable for a consistent tile count
    }
}

// Contiguous stream of every group's bits: dest bits [off[g], off[g+1]) = group g's bits [0, len),
// read from its stored long array.  One thread per destination word gathers from the groups that
// overlap it (no atomics).
__global__ __launch_bounds__(256) void k_rd_stream(const uint8_t* __restrict__ stream, const RdBitSec* __restrict__ secs,
                                                   const int64_t* __restrict__ off, int G, int64_t nwords,
                                                   uint64_t* __restrict__ out) {
    __shared__ int64_t O[kMaxGroups + 1];
    for (int j = threadIdx.x; j <= G; j += 256) O[j] = off[j];
    __syncthreads();
    for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * 256) {
        const int64_t lo = 64 * w, hi = lo + 64;
        int g = 0;
        {  // the first group with off[g + 1] > lo
            int a = 0, b = G;
            while (a < b) {
                const int mid = (a + b) >> 1;
                if (O[mid + 1] > lo) b = mid;
                else a = mid + 1;
            }
            g = a;
        }
        uint64_t v = 0;
        for (; g < G && O[g] < hi; g++) {
            const int64_t a = std::max(lo, O[g]), b = std::min(hi, O[g + 1]);
            if (a >= b) continue;
            const RdBitSec sc = secs[g];
            const uint64_t bits = stored_bits(stream, sc.pos, sc.nstored, a - O[g]);
            const int len = (int)(b - a);
            const uint64_t m = len >= 64 ? ~0ull : ((1ull << len) - 1ull);
            v |= (bits & m) << (a - lo);
        }
        out[w] = v;
    }
}

// words[word0 + i] = stored long i of section s (the Huffman streams, no bit shift)
__global__ __launch_bounds__(256) void k_rd_words(const uint8_t* __restrict__ stream, const int64_t* __restrict__ pos,
                                                  const int64_t* __restrict__ wpre, int nsec, uint64_t* __restrict__ words) {
    __shared__ int64_t pre[kMaxGroups + 1];
    for (int j = threadIdx.x; j <= nsec; j += 256) pre[j] = wpre[j];
    __syncthreads();
    const int64_t total = pre[nsec];
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (int64_t)gridDim.x * 256) {
        const int s = find_section(pre, nsec, g);
        words[g] = be64_at(stream + pos[s] + 8 * (g - pre[s]));
    }
}

hipError_t launch_rd_fixed_sum(hipStream_t st, const uint8_t* stream, const RdFlagSec* secs, const int64_t* wpre, int nsec,
                               int64_t total_words, uint64_t* sums) {
    if (total_words <= 0 || nsec <= 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>((total_words + 255) / 256, 1024);
    hipLaunchKernelGGL(k_rd_fixed_sum, dim3((unsigned)grid), dim3(256), 0, st, stream, secs, wpre, nsec,
                       reinterpret_cast<unsigned long long*>(sums));
    return hipGetLastError();
}
hipError_t launch_rd_unary(hipStream_t st, const uint8_t* stream, const RdFlagSec* secs, const int64_t* tpre, int nsec,
                           int64_t total_tiles, uint32_t* tile_zeros, int64_t* flen) {
    if (nsec <= 0) return hipSuccess;
    if (total_tiles > 0) {
        hipLaunchKernelGGL(k_rd_unary_tiles, dim3((unsigned)total_tiles), dim3(256), 0, st, stream, secs, tpre, nsec,
                           tile_zeros);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_rd_unary_select, dim3((unsigned)nsec), dim3(256), 0, st, stream, secs, tpre, tile_zeros, flen);
    return hipGetLastError();
}
hipError_t launch_rd_stream(hipStream_t st, const uint8_t* stream, const RdBitSec* secs, const int64_t* off, int G,
                            int64_t nwords, uint64_t* out) {
    if (nwords <= 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>((nwords + 255) / 256, 8192);
    hipLaunchKernelGGL(k_rd_stream, dim3((unsigned)grid), dim3(256), 0, st, stream, secs, off, G, nwords, out);
    return hipGetLastError();
}
hipError_t launch_rd_words(hipStream_t st, const uint8_t* stream, const int64_t* pos, const int64_t* wpre, int nsec,
                           int64_t total_words, uint64_t* words) {
    if (total_words <= 0 || nsec <= 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>((total_words + 255) / 256, 8192);
    hipLaunchKernelGGL(k_rd_words, dim3((unsigned)grid), dim3(256), 0, st, stream, pos, wpre, nsec, words);
    return hipGetLastError();
}

}  // namespace skml
