// sydelta_kernels.hip — hand-written gfx950 kernels for sy's delta hot path.
//
//   K1 k_sig_fast     signature of aligned full blocks (block_size % 64 == 0, >= 256):
//                     one wave64 per block, lane l owns bytes [16l + 1024j, +16) of
//                     every 1 KiB piece j -> coalesced 1 KiB per wave-instruction.
//                     Replaces compute_checksums' per-block loop (checksum.rs:46-76).
//   K1' k_sig_wave    same for any size > 240 at any alignment (odd block sizes such as
//                     calculate_block_size's sqrt rule, the partial last block).
//   K1" k_sig_scalar  one thread per block of <= 240 bytes (XXH3 short paths).
//   K3 k_idx_*        device hash table over the basis weak values (generator.rs:75-81).
//   K2 k_scan         rolling weak hash for every window start of the source + probe of the
//                     table (generator.rs:116-124, rolling.rs:66-79): Adler state rolled per
//                     position in closed form, filter bit then exact key probe.
//   K4 k_verify       XXH3 of each weak-hit window and first-in-index-order strong match
//                     (generator.rs:127-153).
//   k_tail            the partial-block tail rule (generator.rs:156-184).
//   k_synth_*         deterministic synthetic inputs for the bench.
//
// Launch wrappers at the bottom are the only symbols the host API uses.
#include "sydelta_device.hpp"
#include "sydelta_internal.hpp"

#include <hipcub/hipcub.hpp>

namespace sydelta {

// ===========================================================================
// K1: signature
// ===========================================================================
__global__ __launch_bounds__(256) void k_sig_fast(const uint8_t* __restrict__ buf, uint64_t nfull, uint32_t bs,
                                                  uint32_t* __restrict__ weak, uint64_t* __restrict__ strong) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t blk = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (blk >= nfull) return;
    const uint8_t* base = buf + blk * (uint64_t)bs;
    const uint32_t q = lane & 3, sl = lane >> 2;
    const uint32_t npieces = (bs + 1023) >> 10;
    const uint32_t ns = bs >> 6;
    uint64_t acc_lo = c_tab.init[2 * q], acc_hi = c_tab.init[2 * q + 1];
    const uint64_t k0n = c_tab.w[sl + 2 * q], k1n = c_tab.w[sl + 2 * q + 1];
    const uint64_t k0l = c_tab.last[2 * q], k1l = c_tab.last[2 * q + 1];
    const uint64_t sk0 = c_tab.w[16 + 2 * q], sk1 = c_tab.w[16 + 2 * q + 1];
    uint32_t asum = 0, vsum = 0;
    uint64_t bpos = 0;
    for (uint32_t j = 0; j < npieces; ++j) {
        const uint32_t off = (j << 10) + (lane << 4);
        const bool valid = off < bs;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (valid) v = *(const uint4*)(base + off);
        uint32_t s = udot4(v.x, 0x01010101u, 0);
        s = udot4(v.y, 0x01010101u, s);
        s = udot4(v.z, 0x01010101u, s);
        s = udot4(v.w, 0x01010101u, s);
        uint32_t u = udot4(v.x, 0x03020100u, 0);
        u = udot4(v.y, 0x07060504u, u);
        u = udot4(v.z, 0x0B0A0908u, u);
        u = udot4(v.w, 0x0F0E0D0Cu, u);
        asum += s;
        vsum += u;
        bpos += (uint64_t)(bs - off) * s;  // s == 0 when !valid
        const uint32_t st = (j << 4) + sl;
        const bool last = (st == ns - 1);
        const uint64_t k0 = last ? k0l : k0n, k1 = last ? k1l : k1n;
        const uint64_t w0 = (uint64_t)v.x | ((uint64_t)v.y << 32);
        const uint64_t w1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
        uint64_t c_lo = mul32x32(w0 ^ k0) + w1;  // acc[2q]   += mul(word 2q) + data(word 2q+1)
        uint64_t c_hi = mul32x32(w1 ^ k1) + w0;  // acc[2q+1] += mul(word 2q+1) + data(word 2q)
        if (!valid) { c_lo = 0; c_hi = 0; }
        c_lo += shfl_xor64(c_lo, 4);  c_hi += shfl_xor64(c_hi, 4);
        c_lo += shfl_xor64(c_lo, 8);  c_hi += shfl_xor64(c_hi, 8);
        c_lo += shfl_xor64(c_lo, 16); c_hi += shfl_xor64(c_hi, 16);
        c_lo += shfl_xor64(c_lo, 32); c_hi += shfl_xor64(c_hi, 32);
        acc_lo += c_lo;
        acc_hi += c_hi;
        if (j + 1 < npieces) { acc_lo = scramble1(acc_lo, sk0); acc_hi = scramble1(acc_hi, sk1); }
    }
    uint64_t f = fold64(acc_lo ^ c_tab.merge[2 * q], acc_hi ^ c_tab.merge[2 * q + 1]);
    f += shfl_xor64(f, 1);
    f += shfl_xor64(f, 2);
    const uint64_t h = xxh3_aval((uint64_t)bs * P64_1 + f);
    asum = wave_sum32(asum);
    vsum = wave_sum32(vsum);
    bpos = wave_sum64(bpos);
    const uint32_t A = (1u + asum) % kMod;
    const uint32_t B = (uint32_t)(((uint64_t)bs + bpos - vsum) % kMod);
    if (lane == 0) {
        weak[blk] = (B << 16) | A;
        strong[blk] = h;
    }
}

// One wave per segment: segment i = [seg_off(i), +seg_len(i)), seg_len > 240.
// Segments are blocks first..first+n of one file (bs stride, last one clipped at len).
__global__ __launch_bounds__(256) void k_sig_wave(const uint8_t* __restrict__ buf, uint64_t len, uint64_t bs,
                                                  uint64_t first, uint64_t nseg, uint32_t* __restrict__ weak,
                                                  uint64_t* __restrict__ strong) {
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nseg) return;
    const uint64_t blk = first + w;
    const uint64_t off = blk * bs;
    const uint64_t sz = (len - off) < bs ? (len - off) : bs;
    uint32_t wk;
    uint64_t st;
    wave_hash_long(buf + off, sz, wk, st);
    if ((threadIdx.x & 63) == 0) {
        weak[blk] = wk;
        strong[blk] = st;
    }
}

// One thread per block whose size is <= 240 bytes.
__global__ __launch_bounds__(256) void k_sig_scalar(const uint8_t* __restrict__ buf, uint64_t len, uint64_t bs,
                                                    uint64_t first, uint64_t nseg, uint32_t* __restrict__ weak,
                                                    uint64_t* __restrict__ strong) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg) return;
    const uint64_t blk = first + t;
    const uint64_t off = blk * bs;
    const uint64_t sz = (len - off) < bs ? (len - off) : bs;
    weak[blk] = adler_scalar(buf + off, sz);
    strong[blk] = xxh3_short(buf + off, sz);
}

// Batched signature (many files, shared block size): one wave per block via a
// block -> file map built on the host side of the launch (file start block prefix).
__global__ __launch_bounds__(256) void k_sig_batch(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ foff,
                                                   const uint64_t* __restrict__ flen,
                                                   const uint64_t* __restrict__ fblk,  // prefix of block counts, nfiles+1
                                                   uint64_t nfiles, uint64_t bs, uint64_t total_blocks,
                                                   uint32_t* __restrict__ weak, uint64_t* __restrict__ strong) {
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= total_blocks) return;
    // binary search the file holding global block w (uniform per wave)
    uint64_t lo = 0, hi = nfiles;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (fblk[mid] <= w) lo = mid; else hi = mid;
    }
    const uint64_t b = w - fblk[lo];
    const uint64_t off = b * bs;
    const uint64_t L = flen[lo];
    const uint64_t sz = (L - off) < bs ? (L - off) : bs;
    const uint8_t* p = buf + foff[lo] + off;
    uint32_t wk;
    uint64_t st;
    if (sz > 240) {
        wave_hash_long(p, sz, wk, st);
    } else {
        wk = 0; st = 0;
        if ((threadIdx.x & 63) == 0) { wk = adler_scalar(p, sz); st = xxh3_short(p, sz); }
    }
    if ((threadIdx.x & 63) == 0) {
        weak[w] = wk;
        strong[w] = st;
    }
}

// ===========================================================================
// K3: index (probe structure) over basis weak values
// ===========================================================================
// Blocked Bloom filter: one 64-bit word per key, 4 bits set, ~16 bits/key
// (FP ~0.6% on Adler values of random blocks; sized to stay L2-resident at 1 Mi
// keys).  Exact set: bucketised open addressing, 4 keys per 16-byte bucket,
// load <= 0.5, so a lookup is almost always one dwordx4 load.  Hash inputs are
// the two 16-bit Adler halves (A = weak & 0xFFFF, B = weak >> 16), mixed with
// 24-bit multiplies (full-rate v_mad_u32_u24).
struct BloomProbe {
    uint32_t word;
    uint32_t bits;  // four 6-bit bit positions
};
__device__ __forceinline__ uint64_t bloom_mask(uint32_t bits) {
    return (1ull << (bits & 63)) | (1ull << ((bits >> 6) & 63)) | (1ull << ((bits >> 12) & 63)) |
           (1ull << ((bits >> 18) & 63));
}
__device__ __forceinline__ BloomProbe bloom_of(uint32_t am, uint32_t bm, uint32_t fwshift) {
    const uint32_t h1 = am * 0x2F0B35u + bm * 0x9E3779u;
    const uint32_t g = am * 0x6B43A9u + bm * 0x1B8735u;
    const uint32_t g2 = am * 0x1F3D5Bu + bm * 0x5A17C3u;
    BloomProbe p;
    p.word = h1 >> fwshift;
    p.bits = (g >> 26) | (((g >> 20) & 63) << 6) | ((g2 >> 26) << 12) | (((g2 >> 20) & 63) << 18);
    return p;
}
__device__ __forceinline__ uint32_t bucket_hash(uint32_t w) {
    uint32_t h = w ^ (w >> 15);
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

__global__ void k_idx_insert(const uint32_t* __restrict__ weak, uint64_t n, unsigned long long* __restrict__ filt,
                             uint32_t fwshift, uint32_t* __restrict__ keys, uint32_t* __restrict__ cnt,
                             uint32_t bmask, uint32_t* __restrict__ slot_of) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t w = weak[i];
    const BloomProbe bp = bloom_of(w & 0xFFFF, w >> 16, fwshift);
    atomicOr(&filt[bp.word], (unsigned long long)bloom_mask(bp.bits));
    uint32_t b = bucket_hash(w) & bmask;
    for (;;) {
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t s = 4 * b + j;
            const uint32_t old = atomicCAS(&keys[s], kEmptyKey, w);
            if (old == kEmptyKey || old == w) {
                atomicAdd(&cnt[s], 1u);
                slot_of[i] = s;
                return;
            }
        }
        b = (b + 1) & bmask;
    }
}

__global__ void k_idx_scatter(uint64_t n, const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ start,
                              uint32_t* __restrict__ fill, uint32_t* __restrict__ order) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    const uint32_t k = atomicAdd(&fill[s], 1u);
    order[start[s] + k] = (uint32_t)i;
}

// Exact lookup: slot of weak value w, or -1.
__device__ __forceinline__ int64_t table_find(const uint32_t* __restrict__ keys, uint32_t bmask, uint32_t w) {
    uint32_t b = bucket_hash(w) & bmask;
    for (;;) {
        const uint4 k = *(const uint4*)(keys + 4 * b);
        if (k.x == w) return 4 * b;
        if (k.y == w) return 4 * b + 1;
        if (k.z == w) return 4 * b + 2;
        if (k.w == w) return 4 * b + 3;
        if (k.w == kEmptyKey) return -1;  // buckets fill in order: a free last slot ends the chain
        b = (b + 1) & bmask;
    }
}

// ===========================================================================
// K2+K4: rolling scan with in-kernel verification
// ===========================================================================
// Tile = kScanThreads threads x kScanRun positions.  Thread k rolls positions
// [p0, p0+kScanRun), p0 = tile_start + k*kScanRun.  The initial window of every
// thread comes from 64-byte chunk prefix sums over the tile (LDS):
//   A(p0) = 1 + sum x,  B(p0) = n + sum_i (n-i) x_{p0+i}
// then per position (rolling.rs:66-79 in closed form, u32, one mod each):
//   a_ex += in - out;  A = a_ex mod M
//   B'   = B + a_ex + nm*(255-out) + C0  (mod M),  nm = n mod M, C0 = 2M-1-(255 nm mod M)
// which is congruent to B - n*out + A' - 1.
// Per position the Bloom word is loaded (kBatch loads in flight per lane);
// positions that pass go to a per-wave LDS queue (fq).  Draining fq does the
// exact table lookups 64 at a time; weak hits (generator.rs:124 `get(&weak)` is
// Some) go to a second per-wave queue (wq).  Draining wq verifies each weak hit
// with a wave-cooperative XXH3 of its window (the bytes were just streamed by
// this workgroup, so they come from L2) and the first candidate in index order
// with equal strong (generator.rs:127-153) becomes a verified hit.
constexpr int kScanThreads = 256;
constexpr int kScanRun = 256;                         // positions per thread
constexpr int kScanTile = kScanThreads * kScanRun;    // 65536 positions per workgroup
constexpr int kBatch = 16;                            // Bloom loads in flight per lane
constexpr int kFQ = 64 * kBatch + 64;                 // filter-pass queue entries per wave
constexpr int kWQ = 128;                              // weak-hit queue entries per wave

struct ScanArgs {
    const uint8_t* src;
    uint64_t len;        // source length L
    uint64_t pos_begin;  // first position of this segment (multiple of kScanTile)
    uint64_t pos_end;    // one past the last full-window position of this segment
    uint32_t n;          // block size
    uint32_t nm;         // n mod M
    uint32_t c0;         // 2M - 1 - (255*nm mod M)
    uint32_t fwshift;    // 32 - log2(filter words)
    const unsigned long long* filt;
    const uint32_t* keys;
    uint32_t bmask;
    uint32_t nchunks;    // LDS chunk slots per tile
    const uint32_t* start;
    const uint32_t* cnt;
    const uint32_t* order;
    const uint64_t* strong;
    HitRec* out;         // verified hits (unordered): rel pos + block index
    uint64_t out_cap;
    unsigned long long* counters;  // [0] verified hits, [1] weak hits, [2] filter passes
};

// 64-byte chunk [c0, c0+64) of src, bytes at or beyond len read as 0.
__device__ __forceinline__ void load_chunk(const uint8_t* src, uint64_t len, uint64_t c0, uint32_t x[16]) {
    if (c0 + 64 <= len) {
        const uint4* q = (const uint4*)(src + c0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = q[i];
            x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint64_t o = c0 + 4 * i;
            uint32_t v = 0;
            if (o + 4 <= len) v = *(const uint32_t*)(src + o);
            else if (o < len) {
                for (uint64_t b = o; b < len; ++b) v |= (uint32_t)src[b] << (8 * (b - o));
            }
            x[i] = v;
        }
    }
}

// 64 bytes starting at an arbitrary address q (dword-granular loads + alignbyte);
// bytes at or beyond len read as 0.
__device__ __forceinline__ void load64_at(const uint8_t* src, uint64_t len, uint64_t q, uint32_t x[16]) {
    const uint32_t sh = (uint32_t)(q & 3);
    const uint64_t qa = q & ~3ull;
    uint32_t d[17];
    if (qa + 68 <= len) {
        const uint32_t* p = (const uint32_t*)(src + qa);
#pragma unroll
        for (int i = 0; i < 17; ++i) d[i] = p[i];
    } else {
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            const uint64_t o = qa + 4 * i;
            uint32_t v = 0;
            if (o + 4 <= len) v = *(const uint32_t*)(src + o);
            else if (o < len) {
                for (uint64_t b = o; b < len; ++b) v |= (uint32_t)src[b] << (8 * (b - o));
            }
            d[i] = v;
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Verify every queued weak hit of this wave (wave-uniform loop).
__device__ __forceinline__ void drain_wq(const ScanArgs& a, const uint2* wq, uint32_t nwq, uint64_t tile_start) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = 0; i < nwq; ++i) {
        const uint2 e = wq[i];  // {rel pos in tile, table slot}
        const uint64_t p = tile_start + e.x;
        const uint8_t* win = a.src + p;
        uint64_t st;
        if (a.n > 240) {
            uint32_t wk;
            wave_hash_long(win, a.n, wk, st);
        } else {
            st = 0;
            if (lane == 0) st = xxh3_short(win, a.n);
            st = shfl64(st, 0);
        }
        const uint32_t s0 = a.start[e.y], c = a.cnt[e.y];
        uint32_t best = 0xFFFFFFFFu;
        for (uint32_t j = lane; j < c; j += 64) {
            const uint32_t bi = a.order[s0 + j];
            if (a.strong[bi] == st) best = min(best, bi);
        }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) best = min(best, (uint32_t)__shfl_xor((int)best, m, 64));
        if (lane == 0 && best != 0xFFFFFFFFu) {
            const unsigned long long k = atomicAdd(&a.counters[0], 1ull);
            if (k < a.out_cap) {
                HitRec r;
                r.pos = (uint32_t)(p - a.pos_begin);
                r.slot = best;
                a.out[k] = r;
            }
        }
    }
}

// Exact lookups for the queued Bloom passes, 64 per round; weak hits go to wq.
__device__ __forceinline__ uint32_t drain_fq(const ScanArgs& a, const uint2* fq, uint32_t nfq, uint2* wq, uint32_t nwq,
                                          uint64_t tile_start) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = 0; base < nfq; base += 64) {
        const uint32_t i = base + lane;
        int64_t slot = -1;
        uint2 e = make_uint2(0, 0);
        if (i < nfq) {
            e = fq[i];  // {rel pos in tile, packed weak}
            slot = table_find(a.keys, a.bmask, e.y);
        }
        const bool hit = slot >= 0;
        const uint64_t m = __ballot(hit);
        const uint32_t cnt = __popcll(m);
        if (cnt && lane == 0) atomicAdd(&a.counters[1], (unsigned long long)cnt);
        if (cnt) {
            if (nwq + cnt > (uint32_t)kWQ) {  // keep room: verify what is queued
                lds_fence();
                drain_wq(a, wq, nwq, tile_start);
                nwq = 0;
            }
            if (hit) {
                const uint32_t off = nwq + __popcll(m & ((1ull << lane) - 1));
                wq[off] = make_uint2(e.x, (uint32_t)slot);
            }
            nwq += cnt;
            lds_fence();
        }
    }
    return nwq;
}

__global__ __launch_bounds__(kScanThreads) void k_scan(ScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nch = a.nchunks;
    uint32_t* PS = (uint32_t*)smem;                 // nch+1 prefix of chunk byte sums
    uint32_t* PV = PS + (nch + 1);                  // nch+1 prefix of in-chunk weighted sums
    const size_t pj_off = (((size_t)(2 * (nch + 1)) * 4 + 15) & ~(size_t)15);
    uint64_t* PJ = (uint64_t*)(smem + pj_off);      // prefix of c*S_c
    const size_t q_off = (pj_off + (size_t)(nch + 1) * 8 + 15) & ~(size_t)15;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    uint2* fq = (uint2*)(smem + q_off) + (size_t)wid * (kFQ + kWQ);
    uint2* wq = fq + kFQ;
    __shared__ uint32_t red_s[kScanThreads / 64], red_v[kScanThreads / 64];
    __shared__ uint64_t red_j[kScanThreads / 64];

    const uint64_t tile_start = a.pos_begin + (uint64_t)blockIdx.x * kScanTile;
    if (tile_start >= a.pos_end) return;
    const uint32_t n = a.n;

    // ---- phase 1: chunk sums (coalesced: thread t takes chunks t, t+256, ...)
    for (uint32_t c = tid; c < nch; c += kScanThreads) {
        uint32_t x[16];
        load_chunk(a.src, a.len, tile_start + 64ull * c, x);
        uint32_t S = 0, V = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) { S = udot4(x[i], 0x01010101u, S); V = udot4(x[i], offw(i), V); }
        PS[c] = S;
        PV[c] = V;
    }
    __syncthreads();
    // ---- phase 2: exclusive prefix over chunks (each thread a contiguous run)
    const uint32_t per = (nch + kScanThreads - 1) / kScanThreads;
    const uint32_t c_lo = tid * per, c_hi = min(nch, c_lo + per);
    uint32_t ts = 0, tv = 0;
    uint64_t tj = 0;
    for (uint32_t c = c_lo; c < c_hi; ++c) { ts += PS[c]; tv += PV[c]; tj += (uint64_t)c * PS[c]; }
    uint32_t is = ts, iv = tv;
    uint64_t ij = tj;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint32_t os = (uint32_t)__shfl_up((int)is, m, 64);
        const uint32_t ov = (uint32_t)__shfl_up((int)iv, m, 64);
        const uint32_t ojl = (uint32_t)__shfl_up((int)(uint32_t)ij, m, 64);
        const uint32_t ojh = (uint32_t)__shfl_up((int)(uint32_t)(ij >> 32), m, 64);
        if (lane >= (uint32_t)m) { is += os; iv += ov; ij += ((uint64_t)ojh << 32) | ojl; }
    }
    if (lane == 63) { red_s[wid] = is; red_v[wid] = iv; red_j[wid] = ij; }
    __syncthreads();
    uint32_t bs_ = 0, bv_ = 0;
    uint64_t bj_ = 0;
    for (uint32_t w = 0; w < wid; ++w) { bs_ += red_s[w]; bv_ += red_v[w]; bj_ += red_j[w]; }
    uint32_t es = bs_ + is - ts, ev = bv_ + iv - tv;
    uint64_t ej = bj_ + ij - tj;
    for (uint32_t c = c_lo; c < c_hi; ++c) {
        const uint32_t s = PS[c], v = PV[c];
        PS[c] = es; PV[c] = ev; PJ[c] = ej;
        es += s; ev += v; ej += (uint64_t)c * s;
    }
    if (tid == kScanThreads - 1) { PS[nch] = bs_ + is; PV[nch] = bv_ + iv; PJ[nch] = bj_ + ij; }
    __syncthreads();

    // ---- phase 3: initial window of this thread
    const uint64_t p0 = tile_start + (uint64_t)tid * kScanRun;
    const uint32_t c0 = tid * (kScanRun / 64);
    const uint32_t m = n >> 6, rem = n & 63;
    uint32_t a_ex = 0, bm = 0;
    const bool live = p0 < a.pos_end;
    if (live) {
        const uint64_t dS = PS[c0 + m] - PS[c0];
        const uint64_t dV = PV[c0 + m] - PV[c0];
        const uint64_t dJ = PJ[c0 + m] - PJ[c0];
        uint64_t A = dS;
        uint64_t B = (uint64_t)n * dS - 64ull * (dJ - (uint64_t)c0 * dS) - dV;
        if (rem) {
            uint32_t x[16];
            load_chunk(a.src, a.len, p0 + 64ull * m, x);
            for (uint32_t r = 0; r < rem; ++r) {
                const uint32_t xb = (x[r >> 2] >> (8 * (r & 3))) & 0xFF;
                A += xb;
                B += (uint64_t)(rem - r) * xb;
            }
        }
        a_ex = (uint32_t)(1 + A);
        bm = (uint32_t)((n + B) % kMod);
    }
    const uint32_t nm = a.nm, cc = a.c0;
    const uint64_t pend = live ? min(a.pos_end, p0 + (uint64_t)kScanRun) : p0;
    const uint32_t npos = (uint32_t)(pend - p0);
    const uint32_t rel0 = tid * kScanRun;  // position of p0 relative to the tile
    // wave-uniform trip count so the queue ballots see every lane
    uint32_t wave_npos = npos;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) wave_npos = max(wave_npos, (uint32_t)__shfl_xor((int)wave_npos, k, 64));
    uint32_t nfq = 0, nwq = 0;
    unsigned long long passes = 0;

    // ---- phase 4: roll
    for (uint32_t g = 0; g < wave_npos; g += 64) {
        uint32_t xo[16], xi[16];
        if (g < npos) {
            load_chunk(a.src, a.len, p0 + g, xo);
            load64_at(a.src, a.len, p0 + g + n, xi);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) { xo[i] = 0; xi[i] = 0; }
        }
#pragma unroll
        for (int hb = 0; hb < 64; hb += kBatch) {
            uint32_t wv[kBatch];
            uint64_t fw[kBatch];
            uint32_t fb[kBatch];
#pragma unroll
            for (int t = 0; t < kBatch; ++t) {
                const int i = hb + t;
                const uint32_t am = a_ex % kMod;
                wv[t] = (bm << 16) | am;
                const BloomProbe bp = bloom_of(am, bm, a.fwshift);
                fw[t] = a.filt[bp.word];
                fb[t] = bp.bits;
                const uint32_t out = (xo[i >> 2] >> (8 * (i & 3))) & 0xFF;
                const uint32_t in = (xi[i >> 2] >> (8 * (i & 3))) & 0xFF;
                a_ex = a_ex + in - out;
                bm = (bm + a_ex + nm * (out ^ 255u) + cc) % kMod;
            }
#pragma unroll
            for (int t = 0; t < kBatch; ++t) {
                const uint32_t rel = g + hb + t;
                const uint64_t fmask = bloom_mask(fb[t]);
                const bool pass = ((fw[t] & fmask) == fmask) && rel < npos;
                const uint64_t mk = __ballot(pass);
                if (mk) {
                    if (pass) fq[nfq + __popcll(mk & ((1ull << lane) - 1))] = make_uint2(rel0 + rel, wv[t]);
                    nfq += __popcll(mk);
                }
            }
            if (nfq > (uint32_t)(kFQ - 64 * kBatch)) {
                lds_fence();
                passes += nfq;
                nwq = drain_fq(a, fq, nfq, wq, nwq, tile_start);
                nfq = 0;
                lds_fence();
            }
        }
    }
    lds_fence();
    passes += nfq;
    nwq = drain_fq(a, fq, nfq, wq, nwq, tile_start);
    lds_fence();
    drain_wq(a, wq, nwq, tile_start);
    if (lane == 0 && passes) atomicAdd(&a.counters[2], passes);
}

// Tail rule (generator.rs:156-184): at p* = len - last_size (last_size < n), the
// suffix matches the last basis block iff weak and strong equal.  One wave.
__global__ void k_tail(const uint8_t* __restrict__ src, uint64_t len, uint64_t last_size, uint32_t want_weak,
                       uint64_t want_strong, int* __restrict__ flag) {
    const uint8_t* p = src + (len - last_size);
    uint32_t wk;
    uint64_t st;
    if (last_size > 240) {
        wave_hash_long(p, last_size, wk, st);
    } else {
        wk = 0; st = 0;
        if ((threadIdx.x & 63) == 0) { wk = adler_scalar(p, last_size); st = xxh3_short(p, last_size); }
    }
    if (threadIdx.x == 0) *flag = (wk == want_weak && st == want_strong) ? 1 : 0;
}

// ===========================================================================
// Synthetic inputs (bench)
// ===========================================================================
__global__ void k_synth_fill(uint8_t* __restrict__ buf, uint64_t len, uint64_t seed) {
    const uint64_t nw = (len + 7) / 8;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t z = splitmix_word(seed, i);
        if (8 * i + 8 <= len) {
            *(uint64_t*)(buf + 8 * i) = z;
        } else {
            for (uint64_t b = 8 * i; b < len; ++b) buf[b] = (uint8_t)(z >> (8 * (b - 8 * i)));
        }
    }
}

// Per byte: r = splitmix(seed, i); if (r & 0xFFFFFFFF) < rate * 2^32 / 1e6: byte ^= 1 + (r >> 32) % 255.
__global__ void k_synth_mutate(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t len, uint64_t seed,
                               uint64_t thresh) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = splitmix_word(seed, i);
        uint8_t v = src[i];
        if ((r & 0xFFFFFFFFull) < thresh) v ^= (uint8_t)(1 + (r >> 32) % 255);
        dst[i] = v;
    }
}

// ===========================================================================
// Launch wrappers
// ===========================================================================
static inline unsigned grid_for(uint64_t threads, unsigned block) { return (unsigned)((threads + block - 1) / block); }

hipError_t launch_signature(const uint8_t* d_buf, uint64_t len, uint64_t bs, uint32_t* d_weak, uint64_t* d_strong,
                            hipStream_t s, Profiler* prof) {
    if (len == 0) return hipSuccess;
    const uint64_t nblocks = (len + bs - 1) / bs;
    const uint64_t nfull = len / bs;
    const bool aligned = (((uintptr_t)d_buf) & 15) == 0;
    uint64_t done = 0;
    if (nfull && aligned && bs % 64 == 0 && bs >= 256 && bs <= (1u << 31)) {
        ProfScope ps(prof, s, "k_sig_fast");
        hipLaunchKernelGGL(k_sig_fast, dim3(grid_for(nfull * 64, 256)), dim3(256), 0, s, d_buf, nfull, (uint32_t)bs,
                           d_weak, d_strong);
        done = nfull;
    } else if (nfull && bs > 240) {
        ProfScope ps(prof, s, "k_sig_wave");
        hipLaunchKernelGGL(k_sig_wave, dim3(grid_for(nfull * 64, 256)), dim3(256), 0, s, d_buf, len, bs, (uint64_t)0,
                           nfull, d_weak, d_strong);
        done = nfull;
    } else if (nfull) {
        ProfScope ps(prof, s, "k_sig_scalar");
        hipLaunchKernelGGL(k_sig_scalar, dim3(grid_for(nfull, 256)), dim3(256), 0, s, d_buf, len, bs, (uint64_t)0,
                           nfull, d_weak, d_strong);
        done = nfull;
    }
    if (done < nblocks) {  // partial last block
        const uint64_t last = len - done * bs;
        if (last > 240)
            hipLaunchKernelGGL(k_sig_wave, dim3(1), dim3(64), 0, s, d_buf, len, bs, done, (uint64_t)1, d_weak, d_strong);
        else
            hipLaunchKernelGGL(k_sig_scalar, dim3(1), dim3(64), 0, s, d_buf, len, bs, done, (uint64_t)1, d_weak,
                               d_strong);
    }
    return hipGetLastError();
}

hipError_t launch_signature_batch(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len,
                                  const uint64_t* d_fblk, uint64_t nfiles, uint64_t bs, uint64_t total_blocks,
                                  uint32_t* d_weak, uint64_t* d_strong, hipStream_t s, Profiler* prof) {
    if (!total_blocks) return hipSuccess;
    ProfScope ps(prof, s, "k_sig_batch");
    hipLaunchKernelGGL(k_sig_batch, dim3(grid_for(total_blocks * 64, 256)), dim3(256), 0, s, d_buf, d_off, d_len,
                       d_fblk, nfiles, bs, total_blocks, d_weak, d_strong);
    return hipGetLastError();
}

hipError_t launch_index_build(const uint32_t* d_weak, uint64_t n, DeviceIndex& ix, hipStream_t s, Profiler* prof) {
    hipError_t e;
    const size_t nslots = (size_t)(ix.bmask + 1) * 4;
    if ((e = hipMemsetAsync(ix.filt, 0, ((size_t)1 << ix.fwbits) * 8, s))) return e;
    if ((e = hipMemsetAsync(ix.keys, 0xFF, nslots * 4, s))) return e;
    if ((e = hipMemsetAsync(ix.cnt, 0, nslots * 4, s))) return e;
    if ((e = hipMemsetAsync(ix.fill, 0, nslots * 4, s))) return e;
    if (n == 0) return hipSuccess;
    {
        ProfScope ps(prof, s, "k_idx_insert");
        hipLaunchKernelGGL(k_idx_insert, dim3(grid_for(n, 256)), dim3(256), 0, s, d_weak, n, ix.filt, 32 - ix.fwbits,
                           ix.keys, ix.cnt, ix.bmask, ix.slot_of);
    }
    size_t tmp = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, ix.cnt, ix.start, (int)nslots, s))) return e;
    void* d_tmp = nullptr;
    if ((e = hipMallocAsync(&d_tmp, tmp ? tmp : 16, s))) return e;
    e = hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp, ix.cnt, ix.start, (int)nslots, s);
    (void)hipFreeAsync(d_tmp, s);
    if (e) return e;
    {
        ProfScope ps(prof, s, "k_idx_scatter");
        hipLaunchKernelGGL(k_idx_scatter, dim3(grid_for(n, 256)), dim3(256), 0, s, n, ix.slot_of, ix.start, ix.fill,
                           ix.order);
    }
    return hipGetLastError();
}

size_t scan_lds_bytes(uint32_t n, uint32_t* nchunks_out) {
    const uint32_t nch = (uint32_t)((kScanTile + (uint64_t)n + 63) / 64) + 1;
    *nchunks_out = nch;
    const size_t pj_off = (((size_t)2 * (nch + 1) * 4) + 15) & ~(size_t)15;
    const size_t q_off = (pj_off + (size_t)(nch + 1) * 8 + 15) & ~(size_t)15;
    return q_off + (size_t)(kScanThreads / 64) * (kFQ + kWQ) * sizeof(uint2);
}

uint64_t scan_tile_positions() { return kScanTile; }

hipError_t launch_scan(const uint8_t* d_src, uint64_t len, uint64_t pos_begin, uint64_t pos_end, uint32_t n,
                       const DeviceIndex& ix, const uint64_t* d_strong, HitRec* d_out, uint64_t out_cap,
                       unsigned long long* d_counters, hipStream_t s, Profiler* prof) {
    ScanArgs a;
    a.src = d_src;
    a.len = len;
    a.pos_begin = pos_begin;
    a.pos_end = pos_end;
    a.n = n;
    a.nm = n % kMod;
    a.c0 = 2 * kMod - 1 - (uint32_t)((255ull * a.nm) % kMod);
    a.fwshift = 32 - ix.fwbits;
    a.filt = ix.filt;
    a.keys = ix.keys;
    a.bmask = ix.bmask;
    const size_t lds = scan_lds_bytes(n, &a.nchunks);
    a.start = ix.start;
    a.cnt = ix.cnt;
    a.order = ix.order;
    a.strong = d_strong;
    a.out = d_out;
    a.out_cap = out_cap;
    a.counters = d_counters;
    const uint64_t tiles = (pos_end - pos_begin + kScanTile - 1) / kScanTile;
    ProfScope ps(prof, s, "k_scan");
    hipLaunchKernelGGL(k_scan, dim3((unsigned)tiles), dim3(kScanThreads), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_sort_hits(HitRec* d_in, HitRec* d_tmp_out, uint64_t nhits, hipStream_t s, HitRec** sorted) {
    // Sort (pos, block) records by pos: view each record as a u64 key (pos in low word).
    // Radix sort on the low 32 bits only (pos); block index rides along in the high word.
    *sorted = d_in;
    if (nhits <= 1) return hipSuccess;
    size_t tmp = 0;
    hipError_t e;
    uint64_t* kin = (uint64_t*)d_in;
    uint64_t* kout = (uint64_t*)d_tmp_out;
    if ((e = hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, kin, kout, (int)nhits, 0, 32, s))) return e;
    void* d_t = nullptr;
    if ((e = hipMallocAsync(&d_t, tmp ? tmp : 16, s))) return e;
    e = hipcub::DeviceRadixSort::SortKeys(d_t, tmp, kin, kout, (int)nhits, 0, 32, s);
    (void)hipFreeAsync(d_t, s);
    *sorted = d_tmp_out;
    return e;
}

hipError_t launch_tail(const uint8_t* d_src, uint64_t len, uint64_t last_size, uint32_t want_weak, uint64_t want_strong,
                       int* d_flag, hipStream_t s) {
    hipLaunchKernelGGL(k_tail, dim3(1), dim3(64), 0, s, d_src, len, last_size, want_weak, want_strong, d_flag);
    return hipGetLastError();
}

hipError_t launch_synth_fill(uint8_t* d_buf, uint64_t len, uint64_t seed, hipStream_t s) {
    if (!len) return hipSuccess;
    hipLaunchKernelGGL(k_synth_fill, dim3(4096), dim3(256), 0, s, d_buf, len, seed);
    return hipGetLastError();
}

hipError_t launch_synth_mutate(uint8_t* d_dst, const uint8_t* d_src, uint64_t len, uint64_t seed, uint32_t rate_ppm,
                               hipStream_t s) {
    if (!len) return hipSuccess;
    const uint64_t thresh = (uint64_t)(((unsigned __int128)rate_ppm << 32) / 1000000u);
    hipLaunchKernelGGL(k_synth_mutate, dim3(4096), dim3(256), 0, s, d_dst, d_src, len, seed, thresh);
    return hipGetLastError();
}

}  // namespace sydelta
