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

#include <algorithm>
#include <chrono>
#include <mutex>

namespace sydelta {

#include "sydelta_kcommon.hpp"


// ===========================================================================
// K1: signature
// ===========================================================================
// K1: four blocks per wave, one per row.
__global__ __launch_bounds__(256) void k_sig_fast(const uint8_t* __restrict__ buf, uint64_t nfull, uint32_t bs,
                                                  uint32_t* __restrict__ weak, uint64_t* __restrict__ strong) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t blk = ((((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) << 2) + (lane >> 4);
    if ((blk & ~3ull) >= nfull) return;  // wave-uniform
    const bool live = blk < nfull;
    uint32_t wk;
    uint64_t st;
    row_hash(buf + (live ? blk : (nfull - 1)) * (uint64_t)bs, bs, wk, st);
    if ((lane & 15) == 0 && live) {
        weak[blk] = wk;
        strong[blk] = st;
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

// Batched signature, full blocks of 16-byte aligned files with bs % 64 == 0: the K1
// row layout (one 16-lane row per block, 4 blocks per wave) over a list of files with
// >= 1 full block: file j starts at aoff[j], its blocks are global blocks agb[j] + k,
// apfx = prefix of full-block counts (apfx[nact] = nfull).  The wave finds its first
// block's file by a 64-way search; its four blocks span at most four listed files.
__global__ __launch_bounds__(256) void k_sig_fast_batch(const uint8_t* __restrict__ buf,
                                                        const uint64_t* __restrict__ aoff,
                                                        const uint64_t* __restrict__ agb,
                                                        const uint64_t* __restrict__ apfx, uint64_t nact,
                                                        uint64_t nfull, uint32_t bs, uint32_t* __restrict__ weak,
                                                        uint64_t* __restrict__ strong) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) << 2;
    if (w0 >= nfull) return;  // wave-uniform
    const uint64_t e = min(w0 + (lane >> 4), nfull - 1);
    uint64_t lo = 0, hi = nact;
    while (hi - lo > 1) {
        const uint64_t step = (hi - lo + 63) >> 6;
        const uint64_t c = lo + lane * step;
        const uint64_t m = __ballot(c < hi && apfx[c] <= w0);
        const uint64_t nlo = lo + (63 - __builtin_clzll(m)) * step;
        hi = min(hi, nlo + step);
        lo = nlo;
    }
    while (apfx[lo + 1] <= e) ++lo;
    const uint64_t k = e - apfx[lo];
    uint32_t wk;
    uint64_t st;
    row_hash(buf + aoff[lo] + k * (uint64_t)bs, bs, wk, st);
    if ((lane & 15) == 0 && w0 + (lane >> 4) < nfull) {
        weak[agb[lo] + k] = wk;
        strong[agb[lo] + k] = st;
    }
}

// Signature of listed segments (partial last blocks): segment i = [loff[i], +llen[i]),
// output slot lidx[i]; one wave per segment.
__global__ __launch_bounds__(256) void k_sig_list(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ loff,
                                                  const uint64_t* __restrict__ llen, const uint64_t* __restrict__ lidx,
                                                  uint64_t n, uint32_t* __restrict__ weak,
                                                  uint64_t* __restrict__ strong) {
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= n) return;
    const uint8_t* p = buf + loff[w];
    const uint64_t sz = llen[w];
    uint32_t wk;
    uint64_t st;
    if (sz > 240) {
        wave_hash_long(p, sz, wk, st);
    } else {
        wk = 0; st = 0;
        if ((threadIdx.x & 63) == 0) { wk = adler_scalar(p, sz); st = xxh3_short(p, sz); }
    }
    if ((threadIdx.x & 63) == 0) {
        weak[lidx[w]] = wk;
        strong[lidx[w]] = st;
    }
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
// Block i of the concatenated signature -> its file (fblk = block prefix, nf+1 entries).
__device__ __forceinline__ uint32_t file_of_block(const uint64_t* __restrict__ fblk, uint32_t nf, uint64_t i) {
    uint32_t lo = 0, hi = nf;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (fblk[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// k_scan_r's ribbon level-1 filter (sydelta_internal.hpp)
// ---------------------------------------------------------------------------
// A key's equation: shard q >> 22, columns [start, start + 32) of the shard, start =
// floor((r >> 8) * (kRibBits - 31) / 2^24), coefficients (q ^ rotl(r, 16)) | 1 (bit 0:
// the column `start`).  The scan tests the same parity over its position's window.
__host__ __device__ __forceinline__ uint32_t rib_bit(uint32_t q, uint32_t r) {
    const uint32_t start = (uint32_t)(((uint64_t)(r >> 8) * ((kRibBits - 31) << 8)) >> 32);
    return (q >> 22) * kRibBits + start;  // global column of the window's first bit
}
__host__ __device__ __forceinline__ uint32_t rib_coef(uint32_t q, uint32_t r) {
    return (q ^ ((r << 16) | (r >> 16))) | 1u;
}
static_assert(((kRibBits - 31) << 8) < (1u << 24), "rib_bit's constant is a 24-bit operand");

__global__ void k_idx_insert(const uint32_t* __restrict__ weak, uint64_t n, const uint64_t* __restrict__ fblk,
                             uint32_t nf, const FileIx* __restrict__ files, uint32_t* __restrict__ filt,
                             uint32_t* __restrict__ l1, uint32_t l1_wshift, uint32_t* __restrict__ keys,
                             uint32_t* __restrict__ cnt, uint32_t* __restrict__ slot_of) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const FileIx F = files[file_of_block(fblk, nf, i)];
    const uint32_t w = weak[i];
    const ProbeHash h = probe_hash(w);
    atomicOr(filt + F.filt_off + (h.r >> F.fwshift), filt_mask(h.q));
    if (l1)  // single-file index only (l1_test)
        atomicOr(l1 + (l1_wshift == 1 ? (size_t)l1r_word(h.q) : (size_t)(h.q >> l1_wshift)), 1u << (h.q & 31));
    // The bucket's four slots are read first (one 16-byte load) and only a slot read empty is
    // claimed: a slot goes from empty to its key once during the build, so a key read is
    // final, and an empty read that is stale loses its CAS and moves on.  (One CAS per key
    // instead of one per slot tried before the free one.)
    uint32_t b = bucket_hash(w) & F.bmask;
    for (;;) {
        const uint64_t s0 = F.slot_off + 4ull * b;
        const uint4 v = *(const uint4*)(keys + s0);
        const uint32_t cur[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t j = 0; j < 4; ++j) {
            uint32_t old = cur[j];
            if (old == kEmptyKey) old = atomicCAS(&keys[s0 + j], kEmptyKey, w);
            if (old == kEmptyKey || old == w) {  // (the slot's count and start: k_idx_runs, after the sort)
                slot_of[i] = (uint32_t)(s0 + j);
                return;
            }
        }
        b = (b + 1) & F.bmask;
    }
}

// Insert equation (start column s, coefficients c with bit 0 set) into a shard's echelon
// rows (rows[j]: the row whose pivot is column j, bit k = column j + k; 0 = none).  Rows
// are written once (CAS from 0) and never change, so the lanes of a wave insert their keys
// concurrently: a lane xors a row it reads (final once set) or claims an empty one; a
// claim lost to another lane is re-read.  An equation that reduces to 0 is a combination of
// earlier ones (homogeneous: always consistent).
__device__ __forceinline__ void rib_insert(uint32_t* rows, uint32_t s, uint32_t c) {
    for (;;) {
        uint32_t v = __hip_atomic_load(&rows[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (!v) {
            v = atomicCAS(&rows[s], 0u, c);
            if (!v) return;
        }
        c ^= v;
        if (!c) return;
        const uint32_t t = __builtin_ctz(c);
        s += t;
        c >>= t;
    }
}

// Free columns of the back-substitution take pseudo-random bits (any values satisfy the
// equations; random ones make a non-key's parity a fair coin).
__device__ __forceinline__ uint32_t rib_free_bit(uint32_t col) {
    uint32_t h = col * 0x9E3779B9u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 13;
    return h >> 31;
}

// One workgroup (one wave) per shard: the shard's listed keys (and the overflow list's
// keys of this shard) inserted into LDS rows 64 at a time, then back-substitution from the
// last column to the first -- z[j] = parity(rows[j] >> 1 & z[j+1 .. j+31]) for a pivot
// column, a free bit otherwise -- carried in a 32-bit window; each finished word of z goes
// to l1[shard * 37 + word].
__global__ __launch_bounds__(64) void k_ribbon_build(const uint32_t* __restrict__ rib_keys,
                                                     const uint32_t* __restrict__ rib_cnt,
                                                     const uint32_t* __restrict__ rib_over, uint32_t* __restrict__ l1) {
    __shared__ uint32_t rows[kRibBits];
    const uint32_t sh = blockIdx.x, lane = threadIdx.x;
    for (uint32_t i = lane; i < kRibBits; i += 64) rows[i] = 0;
    __syncthreads();
    const uint32_t nk = min(rib_cnt[sh], kRibCap);
    for (uint32_t i = lane; i < nk; i += 64) {
        const ProbeHash h = probe_hash(rib_keys[(size_t)sh * kRibCap + i]);
        rib_insert(rows, rib_bit(h.q, h.r) - sh * kRibBits, rib_coef(h.q, h.r));
    }
    const uint32_t no = rib_cnt[kRibShards];
    for (uint32_t i = lane; i < no; i += 64) {
        const ProbeHash h = probe_hash(rib_over[i]);
        if ((h.q >> 22) == sh) rib_insert(rows, rib_bit(h.q, h.r) - sh * kRibBits, rib_coef(h.q, h.r));
    }
    __syncthreads();
    uint32_t zwin = 0;  // bit k: z[j + 1 + k] while column j is solved
    for (int wd = (int)(kRibBits / 32) - 1; wd >= 0; --wd) {
        const uint32_t rv = lane < 32 ? rows[wd * 32 + lane] : 0u;
#pragma unroll
        for (int j = 31; j >= 0; --j) {
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rv, j);
            const uint32_t col = sh * kRibBits + (uint32_t)(wd * 32 + j);
            const uint32_t z = r ? (__builtin_popcount((r >> 1) & zwin) & 1u) : rib_free_bit(col);
            zwin = (zwin << 1) | z;
        }
        if (lane == 0) l1[sh * (kRibBits / 32) + wd] = zwin;
    }
}

// The ribbon's key lists: every distinct key of the (single-file) exact table in its
// shard's list (q >> 22), past kRibCap in the overflow list.  Each workgroup takes `per`
// slots: it counts its keys per shard in LDS, reserves each shard's range with one
// global atomic, then places its keys (one global atomic per key on 1024 counters took
// 0.25 ms at 1 Mi keys).
constexpr uint32_t kRibListT = 256;
__global__ __launch_bounds__(kRibListT) void k_ribbon_list(const uint32_t* __restrict__ keys, uint64_t nslots,
                                                           uint64_t per, uint32_t* __restrict__ rib_keys,
                                                           uint32_t* __restrict__ rib_cnt,
                                                           uint32_t* __restrict__ rib_over) {
    __shared__ uint32_t cnt[kRibShards], base[kRibShards];
    const uint32_t tid = threadIdx.x;
    const uint64_t j0 = (uint64_t)blockIdx.x * per, j1 = min(nslots, j0 + per);
    for (uint32_t i = tid; i < kRibShards; i += kRibListT) cnt[i] = 0;
    __syncthreads();
    for (uint64_t j = j0 + tid; j < j1; j += kRibListT) {
        const uint32_t w = keys[j];
        if (w != kEmptyKey) atomicAdd(&cnt[probe_hash(w).q >> 22], 1u);
    }
    __syncthreads();
    for (uint32_t i = tid; i < kRibShards; i += kRibListT) {
        base[i] = cnt[i] ? atomicAdd(&rib_cnt[i], cnt[i]) : 0u;
        cnt[i] = 0;
    }
    __syncthreads();
    for (uint64_t j = j0 + tid; j < j1; j += kRibListT) {
        const uint32_t w = keys[j];
        if (w == kEmptyKey) continue;
        const uint32_t sh = probe_hash(w).q >> 22;
        const uint32_t rank = base[sh] + atomicAdd(&cnt[sh], 1u);
        if (rank < kRibCap) rib_keys[(size_t)sh * kRibCap + rank] = w;
        else rib_over[atomicAdd(&rib_cnt[kRibShards], 1u)] = w;  // at most nblocks distinct keys
    }
}

// A slot's candidates from the sorted (slot, block) pairs: the run of a slot starts at start
// (its first entry's position) and has cnt entries (set by its last entry); only slots that
// hold a key are ever read.  Replaces an atomic count per key and a scan over every slot.
__global__ void k_idx_runs(const uint32_t* __restrict__ sorted, uint64_t n, uint32_t* __restrict__ start) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t sl = sorted[j];
    if (j == 0 || sorted[j - 1] != sl) start[sl] = (uint32_t)j;
}
__global__ void k_idx_counts(const uint32_t* __restrict__ sorted, uint64_t n, const uint32_t* __restrict__ start,
                             uint32_t* __restrict__ cnt) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t sl = sorted[j];
    if (j + 1 == n || sorted[j + 1] != sl) cnt[sl] = (uint32_t)(j + 1 - start[sl]);
}

// Candidates grouped by slot in index order: order = block indices stably sorted
// by slot (launch_index_build), so the first candidate of a sweep whose strong
// matches is generator.rs:127-133's choice.  cstrong mirrors order with the
// candidates' strong hashes so a verification reads both in one round trip.
__global__ void k_iota(uint32_t* __restrict__ v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

__global__ void k_idx_cstrong(uint64_t n, const uint32_t* __restrict__ order, const uint64_t* __restrict__ strong,
                              uint64_t* __restrict__ cstrong) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    cstrong[j] = strong[order[j]];
}

// Fat table of an index with a level-1 filter (k_scan_r / k_scan_g): per slot {key, first candidate in index
// order (or kMulti | slot when the slot has more than one), that candidate's strong}, so
// one bucket read answers a lookup (the 4 slots of a bucket are one 64-byte line).
__global__ void k_idx_fat(uint64_t nslots, const uint32_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
                          const uint32_t* __restrict__ start, const uint32_t* __restrict__ order,
                          const uint64_t* __restrict__ cstrong, uint4* __restrict__ fat) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nslots) return;
    const uint32_t k = keys[j];
    uint4 r = make_uint4(k, 0, 0, 0);
    if (k != kEmptyKey) {
        const uint32_t s0 = start[j];
        const uint64_t st = cstrong[s0];
        r.y = cnt[j] > 1 ? (0x80000000u | (uint32_t)j) : order[s0];
        r.z = (uint32_t)st;
        r.w = (uint32_t)(st >> 32);
    }
    fat[j] = r;
}

// Candidates of one slot are stored in index order (launch_index_build sorts them),
// so generator.rs:127-133's "first candidate whose strong matches" is the first hit
// of an in-order sweep: 64 candidates per step, stop at the first step with a match.
// Wave-uniform arguments; every lane returns the block (or kNoBlock).
__device__ __forceinline__ uint32_t first_strong_match(const uint32_t* __restrict__ order,
                                                       const uint64_t* __restrict__ cstrong, uint32_t s0, uint32_t cn,
                                                       uint64_t st) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = 0; base < cn; base += 64) {
        const uint32_t j = base + lane;
        const uint64_t m = __ballot(j < cn && cstrong[s0 + j] == st);
        if (m) return order[s0 + base + (uint32_t)__builtin_ctzll(m)];
    }
    return 0xFFFFFFFFu;
}

// ===========================================================================
// K5: aligned-window probe (block-aligned positions k*n of a source)
// ===========================================================================
// The greedy walk (generator.rs:116-197) over a source that shares most blocks with
// the basis moves from one block-aligned hit to the next: positions strictly inside
// a block whose aligned window hits are never visited unless an unaligned hit jumps
// there.  k_probe classifies the aligned positions exactly like the scan does
// (weak -> candidates -> first candidate in index order with equal strong,
// generator.rs:121-155), one wave per window, so the host scans only the other
// blocks' windows (sydelta_api.cpp, Classifier).  out[w] = global block index of
// the hit, or kNoBlock.

__device__ __forceinline__ uint32_t probe_job(const ProbeJob* __restrict__ jobs, uint32_t njobs, uint64_t w) {
    uint32_t lo = 0, hi = njobs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (jobs[mid].pfx <= w) lo = mid; else hi = mid;
    }
    return lo;
}

// Pass 1, general windows: weak + strong, one wave per window, into pw / pst.
__global__ __launch_bounds__(256) void k_probe(const uint8_t* __restrict__ base, const ProbeJob* __restrict__ jobs,
                                               uint32_t njobs, uint64_t nprobes, uint32_t stride, uint32_t n,
                                               uint32_t* __restrict__ pw, uint64_t* __restrict__ pst) {
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nprobes) return;
    const ProbeJob J = jobs[probe_job(jobs, njobs, w)];
    const uint64_t k = J.k0 + (w - J.pfx) * stride;
    const uint8_t* p = base + J.src + k * n;
    uint32_t wk;
    uint64_t st;
    if (n > 240) {
        wave_hash_long(p, n, wk, st);
    } else {
        wk = 0; st = 0;
        if ((threadIdx.x & 63) == 0) { wk = adler_scalar(p, n); st = xxh3_short(p, n); }
    }
    if ((threadIdx.x & 63) == 0) {
        pw[w] = wk;
        pst[w] = st;
    }
}

// Pass 1, aligned windows (n % 64 == 0, n >= 256, 16-byte aligned): four windows
// per wave, one per row (row_hash, the signature kernel's layout).
template <bool kAligned>
__global__ __launch_bounds__(256) void k_probe_rows(const uint8_t* __restrict__ base,
                                                    const ProbeJob* __restrict__ jobs, uint32_t njobs,
                                                    uint64_t nprobes, uint32_t stride, uint32_t n,
                                                    uint32_t* __restrict__ pw, uint64_t* __restrict__ pst) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = ((((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) << 2) + (lane >> 4);
    if ((w & ~3ull) >= nprobes) return;  // wave-uniform
    const bool live = w < nprobes;
    const uint64_t wl = live ? w : nprobes - 1;
    const ProbeJob J = jobs[probe_job(jobs, njobs, wl)];
    const uint64_t k = J.k0 + (wl - J.pfx) * stride;
    uint32_t wk;
    uint64_t st;
    row_hash<kAligned>(base + J.src + k * n, n, wk, st);
    if ((lane & 15) == 0 && live) {
        pw[w] = wk;
        pst[w] = st;
    }
}

// Pass 2: one thread per window: filter, exact table, first candidate in index
// order with equal strong (generator.rs:121-155).
__global__ __launch_bounds__(256) void k_probe_lookup(const ProbeJob* __restrict__ jobs, uint32_t njobs,
                                                      uint64_t nprobes, const FileIx* __restrict__ files,
                                                      const uint32_t* __restrict__ filt,
                                                      const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ start,
                                                      const uint32_t* __restrict__ cnt,
                                                      const uint32_t* __restrict__ order,
                                                      const uint64_t* __restrict__ cstrong,
                                                      const uint32_t* __restrict__ pw, const uint64_t* __restrict__ pst,
                                                      uint32_t* __restrict__ out) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nprobes) return;
    const FileIx F = files[jobs[probe_job(jobs, njobs, w)].file];
    const uint32_t wk = pw[w];
    uint32_t best = kNoBlock;
    const ProbeHash h = probe_hash(wk);
    if (filt_pass(filt[F.filt_off + (h.r >> F.fwshift)], h.q)) {
        const int64_t slot = table_find(keys + F.slot_off, F.bmask, wk);
        if (slot >= 0) {
            const uint64_t gs = F.slot_off + (uint64_t)slot;
            const uint32_t s0 = start[gs], c = cnt[gs];
            const uint64_t st = pst[w];
            for (uint32_t j = 0; j < c; ++j)
                if (cstrong[s0 + j] == st) { best = order[s0 + j]; break; }
        }
    }
    out[w] = best;
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
    const uint8_t* src;  // scanned buffer (sources at segs[].src)
    uint32_t n;          // block size
    uint32_t nm;         // n mod M
    uint32_t c0;         // 2M - 1 - (255*nm mod M)    (k_scan)
    uint32_t timing;     // accumulate per-phase s_memtime cycles of wave 0 into counters[4..8)
                         // skips the drains, bit 1 the level-2 loads; bit 3 the hashing of weak
                         // hits, bit 4 the fat-table lookups
    // k_scan_lds: segment table and per-file probe offsets
    const ScanSeg* segs;
    uint32_t nsegs;
    uint32_t ntiles;
    const FileIx* files;
    // k_scan (one segment of file 0)
    uint64_t len;        // source length
    uint64_t pos_begin;  // first position of the segment (multiple of kScanTile)
    uint64_t pos_end;    // one past its last full-window position
    uint32_t seg_id;
    uint32_t fwshift;    // file 0's filter
    uint32_t bmask;      // file 0's table
    uint32_t nchunks;    // LDS chunk slots per tile (k_scan)
    // probe structures (concatenated over files)
    const uint32_t* filt;
    const uint32_t* l1;       // level-1 filter (k_scan_r / k_scan_g: kL1WordsR words)
    const uint4* fat;         // k_scan_r / k_scan_g: {key, first candidate | kMulti+slot, strong} per slot
    const uint32_t* keys;
    const uint32_t* start;
    const uint32_t* cnt;
    const uint32_t* order;
    const uint64_t* cstrong;  // strong hash of order[j]
    // outputs
    uint64_t* hit_key;   // (segment << 32) | position - segment start
    uint32_t* hit_val;   // global block index
    uint64_t out_cap;
    unsigned long long* counters;  // [0] verified hits, [1] weak hits, [2] filter passes, [4..8) phase cycles
    uint2* gfq;          // k_scan_lds: per-wave filter-pass queues in HBM/L2, kGFQ entries each
    struct WDef* wdef;   // k_scan_g: weak hits whose verification k_verify_w does (count: counters[10])
    uint64_t wdef_cap;
    // k_scan_r: each wave's level-2 passes of one wave tile {position in run, weak}
    uint2* rrec;
    // k_scan_r / k_scan_g / k_verify_w: each wave's staged outputs (WaveOut), kHStage
    // verified hits and kDStage deferred weak hits per wave
    uint4* hstage;
    struct WDef* dstage;
};

// A weak hit of k_scan_g, verified after the scan by k_verify_w.
struct WDef {
    uint64_t at;      // byte offset of the window in ScanArgs::src
    uint64_t key;     // its hit key: (segment << kSegShift) | position - segment start
    uint32_t cand;    // fat record: first candidate, or kMulti + slot
    uint32_t pad;
    uint64_t strong;  // the first candidate's strong hash (single-candidate records)
};

// The segment a tile belongs to, as the drains see it.
struct SegCtx {
    const uint8_t* base;  // first byte of the source
    uint64_t pos_begin;   // segment range, positions relative to the source
    uint64_t pos_end;
    const uint32_t* keys; // this file's exact table (slot_off applied)
    uint64_t slot_off;
    uint32_t bmask;
    uint32_t seg_id;
    // k_scan_r / k_scan_g
    const uint4* fat;     // this file's fat table (slot_off applied)
    const uint32_t* filt; // this file's level-2 filter
    uint32_t fwshift, fwords;
};

// 64-byte chunk [c0, c0+64) of src, bytes at or beyond len read as 0.  Past the
// end only whole 16-byte granules that hold a byte of [0, len) are loaded (the
// buffer is readable to the end of its last granule, sydelta.h) and masked.
__device__ __forceinline__ void load_chunk(const uint8_t* src, uint64_t len, uint64_t c0, uint32_t x[16]) {
    const uint4* q = (const uint4*)(src + c0);
    if (c0 + 64 <= len) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = q[i];
            x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (c0 + 16 * i < len) v = q[i];
        x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint64_t o = c0 + 4 * i;
        const uint32_t keep = o >= len ? 0u : (o + 4 <= len ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (o + 4 - len))));
        x[i] &= keep;
    }
}

// The register scans' row loads.  Non-temporal loads (meant to keep the rows from evicting
// the level-2 filter from L2) measured 9.82 ms at C3 against 9.59 ms with plain ones
// (profiles/r04h_ab_*), so the rows are loaded as any chunk.
__device__ __forceinline__ void load_chunk_nt(const uint8_t* src, uint64_t len, uint64_t c0, uint32_t x[16]) {
    load_chunk(src, len, c0, x);
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

// Verify every queued weak hit of this wave (wave-uniform loop): XXH3 of the
// window, first candidate in index order with equal strong (generator.rs:127-153).
// rows != nullptr: the tile's bytes are staged in LDS (k_scan_lds) and the window
// is hashed from there.
__device__ __forceinline__ void drain_wq(const ScanArgs& a, const SegCtx& c, uint2* wq, uint32_t nwq,
                                         uint64_t tile_start, const uint32_t* rows = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = 0; i < nwq; ++i) {
        const uint2 e = wq[i];  // {rel pos in tile, global table slot}
        const uint64_t p = tile_start + e.x;
        const uint8_t* win = c.base + p;
        uint64_t st;
        if (a.n > 240) {
            uint32_t wk;
            if (rows)
                wave_hash_src(LdsRowBytes{rows, e.x}, a.n, wk, st);
            else
                wave_hash_long(win, a.n, wk, st);
        } else {
            st = 0;
            if (lane == 0) st = xxh3_short(win, a.n);
            st = shfl64(st, 0);
        }
        const uint32_t best = first_strong_match(a.order, a.cstrong, a.start[e.y], a.cnt[e.y], st);
        if (lane == 0) wq[i].y = best;  // verified block, or none
    }
    // one output reservation per wave: the counter is shared by the whole chip
    lds_fence();
    uint32_t nver = 0;
    for (uint32_t base = 0; base < nwq; base += 64) {
        const bool v = base + lane < nwq && wq[base + lane].y != 0xFFFFFFFFu;
        nver += __popcll(__ballot(v));
    }
    if (!nver) return;
    unsigned long long k0 = 0;
    if (lane == 0) k0 = atomicAdd(&a.counters[0], (unsigned long long)nver);
    k0 = shfl64(k0, 0);
    for (uint32_t base = 0; base < nwq; base += 64) {
        const uint32_t i = base + lane;
        const uint2 e = i < nwq ? wq[i] : make_uint2(0, 0xFFFFFFFFu);
        const bool v = e.y != 0xFFFFFFFFu;
        const uint64_t m = __ballot(v);
        const unsigned long long k = k0 + __popcll(m & ((1ull << lane) - 1));
        if (v && k < a.out_cap) {
            const uint64_t p = tile_start + e.x;
            a.hit_key[k] = ((uint64_t)c.seg_id << kSegShift) | (uint64_t)(uint32_t)(p - c.pos_begin);
            a.hit_val[k] = e.y;
        }
        k0 += __popcll(m);
    }
}

// Exact lookups for the queued Bloom passes, 64 per round; weak hits go to wq
// (capacity WQ entries, verified in place when full).
template <int WQ>
__device__ __forceinline__ uint32_t drain_fq(const ScanArgs& a, const SegCtx& c, const uint2* fq, uint32_t nfq,
                                             uint2* wq, uint32_t nwq, uint64_t tile_start,
                                             unsigned long long& weak_hits) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = 0; base < nfq; base += 64) {
        const uint32_t i = base + lane;
        int64_t slot = -1;
        uint2 e = make_uint2(0, 0);
        if (i < nfq) {
            e = fq[i];  // {rel pos in tile, packed weak}
            if (tile_start + e.x < c.pos_end) slot = table_find(c.keys, c.bmask, e.y);
        }
        const bool hit = slot >= 0;
        const uint64_t m = __ballot(hit);
        const uint32_t cnt = __popcll(m);
        weak_hits += cnt;
        if (cnt) {
            if (nwq + cnt > (uint32_t)WQ) {  // keep room: verify what is queued
                lds_fence();
                drain_wq(a, c, wq, nwq, tile_start);
                nwq = 0;
            }
            if (hit) {
                const uint32_t off = nwq + __popcll(m & ((1ull << lane) - 1));
                wq[off] = make_uint2(e.x, (uint32_t)(c.slot_off + slot));
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
    SegCtx sc;
    sc.base = a.src;
    sc.pos_begin = a.pos_begin;
    sc.pos_end = a.pos_end;
    sc.keys = a.keys;
    sc.slot_off = 0;
    sc.bmask = a.bmask;
    sc.seg_id = a.seg_id;

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
    unsigned long long passes = 0, weak_hits = 0;

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
            uint32_t fw[kBatch];
            uint32_t fh[kBatch];
#pragma unroll
            for (int t = 0; t < kBatch; ++t) {
                const int i = hb + t;
                const uint32_t am = a_ex % kMod;
                wv[t] = (bm << 16) | am;
                const ProbeHash h = probe_hash(am, bm);
                fh[t] = h.q;
                fw[t] = a.filt[h.r >> a.fwshift];
                const uint32_t out = (xo[i >> 2] >> (8 * (i & 3))) & 0xFF;
                const uint32_t in = (xi[i >> 2] >> (8 * (i & 3))) & 0xFF;
                a_ex = a_ex + in - out;
                bm = (bm + a_ex + nm * (out ^ 255u) + cc) % kMod;
            }
#pragma unroll
            for (int t = 0; t < kBatch; ++t) {
                const uint32_t rel = g + hb + t;
                const bool pass = filt_pass(fw[t], fh[t]) && rel < npos;
                const uint64_t mk = __ballot(pass);
                if (mk) {
                    if (pass) fq[nfq + __popcll(mk & ((1ull << lane) - 1))] = make_uint2(rel0 + rel, wv[t]);
                    nfq += __popcll(mk);
                }
            }
            if (nfq > (uint32_t)(kFQ - 64 * kBatch)) {
                lds_fence();
                passes += nfq;
                nwq = drain_fq<kWQ>(a, sc, fq, nfq, wq, nwq, tile_start, weak_hits);
                nfq = 0;
                lds_fence();
            }
        }
    }
    lds_fence();
    passes += nfq;
    nwq = drain_fq<kWQ>(a, sc, fq, nfq, wq, nwq, tile_start, weak_hits);
    lds_fence();
    drain_wq(a, sc, wq, nwq, tile_start);
    if (lane == 0 && passes) atomicAdd(&a.counters[2], passes);
    if (lane == 0 && weak_hits) atomicAdd(&a.counters[1], weak_hits);
}

// ===========================================================================
// K2+K4, LDS-staged: k_scan_lds (window n <= kMaxN2)
// ===========================================================================
// Same classification as k_scan, reorganised so that every source byte leaves
// HBM once per tile and every per-position access is an LDS access:
//   phase 1  the tile's bytes [T0, T0 + kTile2 + n) are loaded with 16-byte
//            non-temporal loads into LDS rows of 64 bytes (row stride 68 B, so
//            the per-thread runs below hit distinct banks), chunk sums on the way;
//   phase 2  exclusive prefix of the chunk sums;
//   phase 3  thread t's first window [T0+64t, +n) in closed form;
//   phase 4  thread t rolls its 64 positions with both Adler halves kept
//            reduced (rolling.rs:66-79: a' = a+new-old, b' = b-n*old+a'-1, each
//            brought back to [0, M) with two unsigned min-subtracts), reads one
//            filter word per position (LDS copy of the filter when the index is
//            small, else HBM/L2), and only when some lane of the wave has a pass
//            in the batch queues the passes; exact table lookup and strong
//            verification (drain2) run from one inlined site.
// Persistent: workgroup b rolls tiles [b*per, (b+1)*per), contiguous, so a tile's
// halo (the next tile's first n bytes) is re-read from this XCD's L2; the filter
// copy and the n*x table are built once per workgroup.  Two workgroups per CU:
// one's staging (HBM latency) overlaps the other's roll.
constexpr int kT2 = 256;                 // threads per workgroup (4 waves)
constexpr int kR2 = 64;                  // positions per thread = one 64-byte row
constexpr int kTile2 = kT2 * kR2;        // 16384 positions per tile
constexpr int kB2 = 8;                   // positions per batch (filter reads in flight per lane)
constexpr int kGFQ = 2048;               // filter-pass queue entries per wave (global memory)
constexpr int kWQ2 = 128;                // weak-hit queue entries per wave (LDS)
constexpr uint32_t kMaxN2 = 8192;        // largest window the LDS layout holds
constexpr int kRowDw = 17;               // LDS row = 16 data dwords + 1 pad
constexpr int kWgPerCuMax2 = 4;          // up to 4 workgroups per CU when the LDS layout fits

struct Lds2 {
    uint32_t nch;
    uint32_t ps, pv, pj, ntab, filt, q, total;  // byte offsets
};
__host__ __device__ __forceinline__ Lds2 lds2_layout(uint32_t n, uint32_t filt_words) {
    Lds2 L;
    L.nch = (kTile2 + n + 63) / 64 + 1;
    uint32_t o = L.nch * kRowDw * 4;
    o = (o + 15) & ~15u; L.ps = o; o += (L.nch + 1) * 4;
    L.pv = o; o += (L.nch + 1) * 4;
    o = (o + 15) & ~15u; L.pj = o; o += (L.nch + 1) * 8;
    L.ntab = o; o += 256 * 4;
    o = (o + 15) & ~15u; L.filt = o; o += filt_words * 4;
    o = (o + 15) & ~15u; L.q = o; o += (kT2 / 64) * kWQ2 * 16;
    L.total = o;
    return L;
}

// k_scan_lds queues.  Filter passes (HBM, kGFQ per wave): {(tile - t_begin) << 14 |
// position in tile, weak}; weak hits (LDS, kWQ2 per wave): {segment, position in
// segment, global table slot, 0}.  Both are drained only when nearly full and at
// the end of the workgroup's tiles, so no tile waits on the latency chain of a
// lookup + verification; windows are hashed from global memory (L2-warm).
static_assert(kTile2 == (1 << 14), "queue entries pack the position in 14 bits");

// Segment holding tile t (tiles of a launch are laid out segment after segment).
__device__ __forceinline__ uint32_t seg_of_tile(const ScanArgs& a, uint32_t t) {
    uint32_t lo = 0, hi = a.nsegs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.segs[mid].tile_base <= t) lo = mid; else hi = mid;
    }
    return lo;
}

// XXH3-64 of the window at tile offset o (LDS rows, 17-dword stride) for this lane's
// row, n % 64 == 0 and n >= 256 (row_hash's layout, strong part only: the weak is
// already known equal).  Valid in every lane of the row.  Keys per lane in K.
struct RowKeys {
    uint64_t k0[4], k1[4];  // stripe keys of this lane's stripes slot + 4k, words 2q / 2q+1
    uint64_t l0, l1;        // last-stripe keys
    uint64_t s0, s1;        // scramble keys
};
__device__ __forceinline__ void row_keys(RowKeys& K) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t q = lane & 3, slot = (lane >> 2) & 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        K.k0[k] = c_tab.w[slot + 4 * k + 2 * q];
        K.k1[k] = c_tab.w[slot + 4 * k + 2 * q + 1];
    }
    K.l0 = c_tab.last[2 * q];
    K.l1 = c_tab.last[2 * q + 1];
    K.s0 = c_tab.w[16 + 2 * q];
    K.s1 = c_tab.w[16 + 2 * q + 1];
}
__device__ __forceinline__ uint64_t row_strong_lds(const uint32_t* rows, uint32_t o, uint32_t n, const RowKeys& K) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t q = lane & 3, slot = (lane >> 2) & 3;
    const uint32_t npieces = (n + 1023) >> 10;
    const uint32_t ls = (n >> 6) - 1 - ((npieces - 1) << 4);
    const uint32_t last_k = ls >> 2, last_slot = ls & 3;
    const uint32_t sh = o & 3;
    uint64_t acc_lo = c_tab.init[2 * q], acc_hi = c_tab.init[2 * q + 1];
    for (uint32_t j = 0; j < npieces; ++j) {
        uint64_t c_lo = 0, c_hi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t u = (j << 10) + ((slot + 4 * k) << 6) + (q << 4);
            // dword d of the tile sits at row d>>4, column d&15 (17-dword rows): the 5
            // dwords from d0 are at base + i, plus one past a row end
            const uint32_t d0 = (o + u) >> 2, c0 = d0 & 15;
            const uint32_t* p = rows + (d0 >> 4) * kRowDw + c0;
            uint32_t x[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) x[i] = p[i + ((c0 + i) >> 4)];
            const uint32_t v0 = __builtin_amdgcn_alignbyte(x[1], x[0], sh);
            const uint32_t v1 = __builtin_amdgcn_alignbyte(x[2], x[1], sh);
            const uint32_t v2 = __builtin_amdgcn_alignbyte(x[3], x[2], sh);
            const uint32_t v3 = __builtin_amdgcn_alignbyte(x[4], x[3], sh);
            const bool lastk = (j + 1 == npieces) && k == (int)last_k && slot == last_slot;
            const uint64_t k0 = lastk ? K.l0 : K.k0[k];
            const uint64_t k1 = lastk ? K.l1 : K.k1[k];
            const uint64_t w0 = (uint64_t)v0 | ((uint64_t)v1 << 32);
            const uint64_t w1 = (uint64_t)v2 | ((uint64_t)v3 << 32);
            uint64_t p_lo = mul32x32(w0 ^ k0) + w1;
            uint64_t p_hi = mul32x32(w1 ^ k1) + w0;
            if (u >= n) { p_lo = 0; p_hi = 0; }
            c_lo += p_lo;
            c_hi += p_hi;
        }
        c_lo = dpp_add64<kDppRowRor4>(c_lo);
        c_lo = dpp_add64<kDppRowRor8>(c_lo);
        c_hi = dpp_add64<kDppRowRor4>(c_hi);
        c_hi = dpp_add64<kDppRowRor8>(c_hi);
        acc_lo += c_lo;
        acc_hi += c_hi;
        if (j + 1 < npieces) {
            acc_lo = scramble1(acc_lo, K.s0);
            acc_hi = scramble1(acc_hi, K.s1);
        }
    }
    const uint64_t f = sum_quad64(fold64(acc_lo ^ c_tab.merge[2 * q], acc_hi ^ c_tab.merge[2 * q + 1]));
    return xxh3_aval((uint64_t)n * P64_1 + f);
}

// Tile-flush verification with the windows in LDS, four hits per wave (one per
// row); candidates in index order (first_strong_match's rule).
__device__ __forceinline__ void verify_rows_lds(const ScanArgs& a, uint4* wq, uint32_t nwq, const uint32_t* rows,
                                                uint64_t tile_start, const SegCtx* cur) {
    const uint32_t lane = threadIdx.x & 63, row = lane >> 4, rl = lane & 15;
    RowKeys K;
    row_keys(K);
    for (uint32_t t = 0; t < nwq; t += 4) {
        const uint32_t h = t + row;
        const bool live = h < nwq;
        const uint4 e = wq[live ? h : t];
        const uint32_t s0 = a.start[e.z], cn = a.cnt[e.z];  // in flight while hashing
        const uint32_t o = (uint32_t)(cur->pos_begin + e.y - tile_start);
        const uint64_t st = row_strong_lds(rows, o, a.n, K);
        if (!live) continue;
        uint32_t best = 0xFFFFFFFFu;
        for (uint32_t b = 0; b < cn; b += 16) {  // in index order, 16 candidates per step
            const uint32_t j = b + rl;
            const uint64_t m = (__ballot(j < cn && a.cstrong[s0 + j] == st) >> (row << 4)) & 0xFFFFull;
            if (m) {
                best = a.order[s0 + b + (uint32_t)__builtin_ctzll(m)];
                break;
            }
        }
        if (rl == 0) wq[h].w = best;
    }
}

// Verify the queued weak hits: XXH3 of each window, first candidate in index
// order with equal strong (generator.rs:127-153); one output reservation per wave.
// rows != nullptr (tile-flush mode): every queued hit lies in the current tile,
// whose bytes are staged in LDS and whose segment is *cur; hash from LDS and take
// the segment from registers.  Otherwise windows are hashed from global memory.
// The candidate group of up to 64 hits is fetched with one round trip of
// start/cnt and one of (order, cstrong), lane i serving hit i.
template <bool kRowVerify>
__device__ __forceinline__ void verify3(const ScanArgs& a, uint4* wq, uint32_t nwq, const uint32_t* rows,
                                        uint64_t tile_start, const SegCtx* cur) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = 0; base < nwq; base += 64) {
        const uint32_t cnt_here = min(64u, nwq - base);
        if (kRowVerify && rows && a.n % 64 == 0 && a.n >= 256) {
            verify_rows_lds(a, wq + base, cnt_here, rows, tile_start, cur);
            continue;
        }
        // lane i: candidate group of hit base+i, first candidate
        uint32_t s0 = 0, cn = 0, b0 = 0xFFFFFFFFu;
        uint64_t st0 = 0;
        if (lane < cnt_here) {
            const uint32_t slot = wq[base + lane].z;
            s0 = a.start[slot];
            cn = a.cnt[slot];
            b0 = a.order[s0];
            st0 = a.cstrong[s0];
        }
        for (uint32_t k = 0; k < cnt_here; ++k) {
            const uint4 e = wq[base + k];  // {segment, position in segment, global slot, -}
            uint64_t st;
            if (a.n > 240) {
                uint32_t wk;
                if (rows) {
                    wave_hash_src(LdsRowBytes{rows, (uint32_t)(cur->pos_begin + e.y - tile_start)}, a.n, wk, st);
                } else {
                    const ScanSeg S = a.segs[e.x];
                    wave_hash_long(a.src + S.src + S.pos_begin + e.y, a.n, wk, st);
                }
            } else {
                const uint8_t* win = rows ? cur->base + cur->pos_begin + e.y
                                          : a.src + a.segs[e.x].src + a.segs[e.x].pos_begin + e.y;
                st = 0;
                if (lane == 0) st = xxh3_short(win, a.n);
                st = shfl64(st, 0);
            }
            const uint32_t kcn = (uint32_t)__shfl((int)cn, k, 64);
            uint32_t best = 0xFFFFFFFFu;
            if (kcn == 1) {  // the usual case: the one candidate was fetched above
                if (shfl64(st0, k) == st) best = (uint32_t)__shfl((int)b0, k, 64);
            } else {
                best = first_strong_match(a.order, a.cstrong, (uint32_t)__shfl((int)s0, k, 64), kcn, st);
            }
            if (lane == 0) wq[base + k].w = best;  // verified block, or none
        }
    }
    lds_fence();
    uint32_t nver = 0;
    for (uint32_t base = 0; base < nwq; base += 64) {
        const bool v = base + lane < nwq && wq[base + lane].w != 0xFFFFFFFFu;
        nver += __popcll(__ballot(v));
    }
    if (!nver) return;
    unsigned long long k0 = 0;
    if (lane == 0) k0 = atomicAdd(&a.counters[0], (unsigned long long)nver);
    k0 = shfl64(k0, 0);
    for (uint32_t base = 0; base < nwq; base += 64) {
        const uint32_t i = base + lane;
        const uint4 e = i < nwq ? wq[i] : make_uint4(0, 0, 0, 0xFFFFFFFFu);
        const bool v = e.w != 0xFFFFFFFFu;
        const uint64_t m = __ballot(v);
        const unsigned long long k = k0 + __popcll(m & ((1ull << lane) - 1));
        if (v && k < a.out_cap) {
            a.hit_key[k] = ((uint64_t)e.x << kSegShift) | e.y;
            a.hit_val[k] = e.w;
        }
        k0 += __popcll(m);
    }
}

// Exact lookups of the queued filter passes, 64 per round (positions at or past
// the segment end are dropped here); weak hits go to wq and are verified when it
// cannot take another round, and at the end.
template <bool kRowVerify>
__device__ __forceinline__ void drain3(const ScanArgs& a, const uint2* fq, uint32_t nfq, uint4* wq, uint32_t t_begin,
                                       unsigned long long& weak_hits, const uint32_t* rows = nullptr,
                                       uint64_t tile_start = 0, const SegCtx* cur = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's queue stores have reached L2
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const bool tw = a.timing && threadIdx.x == 0;
    unsigned long long t_lk = 0, t_vf = 0, t0 = tw ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t nwq = 0;
    for (uint32_t base = 0; base < nfq; base += 64) {
        const uint32_t i = base + lane;
        int64_t slot = -1;
        uint32_t si = 0, rp = 0, fslot = 0;
        if (i < nfq) {
            const uint32_t ex = __builtin_nontemporal_load(&fq[i].x);
            const uint32_t ew = __builtin_nontemporal_load(&fq[i].y);
            if (cur) {  // tile-flush mode: every entry is from the current tile
                const uint64_t p = tile_start + (ex & (kTile2 - 1));
                si = cur->seg_id;
                if (p < cur->pos_end) {
                    slot = table_find(cur->keys, cur->bmask, ew);
                    fslot = (uint32_t)cur->slot_off;
                }
                rp = (uint32_t)(p - cur->pos_begin);
            } else {
                const uint32_t t = t_begin + (ex >> 14);
                si = seg_of_tile(a, t);
                const ScanSeg S = a.segs[si];
                const uint64_t p = S.pos_begin + (uint64_t)(t - S.tile_base) * kTile2 + (ex & (kTile2 - 1));
                if (p < S.pos_end) {
                    const FileIx F = a.files[S.file];
                    slot = table_find(a.keys + F.slot_off, F.bmask, ew);
                    fslot = (uint32_t)F.slot_off;
                }
                rp = (uint32_t)(p - S.pos_begin);
            }
        }
        const bool hit = slot >= 0;
        const uint64_t m = __ballot(hit);
        if (!m) continue;
        const uint32_t cnt = __popcll(m);
        weak_hits += cnt;
        if (nwq + cnt > (uint32_t)kWQ2) {
            lds_fence();
            verify3<kRowVerify>(a, wq, nwq, rows, tile_start, cur);
            nwq = 0;
        }
        if (hit) wq[nwq + __popcll(m & ((1ull << lane) - 1))] = make_uint4(si, rp, fslot + (uint32_t)slot, 0);
        nwq += cnt;
    }
    lds_fence();
    if (tw) { const unsigned long long t1 = __builtin_amdgcn_s_memtime(); t_lk += t1 - t0; t0 = t1; }
    verify3<kRowVerify>(a, wq, nwq, rows, tile_start, cur);
    lds_fence();
    if (tw) {
        t_vf += __builtin_amdgcn_s_memtime() - t0;
        atomicAdd(&a.counters[8], t_lk);
        atomicAdd(&a.counters[9], t_vf);
    }
}

template <bool kLdsFilter, int kWgPerCu = kLdsFilter ? 3 : 4, bool kRowVerify = false>
__global__ __launch_bounds__(kT2, kWgPerCu) void k_scan_lds(ScanArgs a, uint32_t per, uint32_t lds_fwords) {
    // Large indexes (filter in HBM/L2) come with dense Adler false hits (C3: ~1 per
    // 1000 positions): their verification runs at the end of every tile, hashing the
    // windows from LDS.  Small indexes have rare hits: queue across tiles, verify
    // from global memory when the queue fills and at the end.
    constexpr bool kTileFlush = !kLdsFilter;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t n = a.n;
    const Lds2 L = lds2_layout(n, kLdsFilter ? lds_fwords : 0u);
    uint32_t* rows = (uint32_t*)smem;
    uint32_t* PS = (uint32_t*)(smem + L.ps);
    uint32_t* PV = (uint32_t*)(smem + L.pv);
    uint64_t* PJ = (uint64_t*)(smem + L.pj);
    uint32_t* ntab = (uint32_t*)(smem + L.ntab);
    uint32_t* lfilt = (uint32_t*)(smem + L.filt);
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    uint4* wq = (uint4*)(smem + L.q) + (size_t)wid * kWQ2;
    uint2* fq = a.gfq + ((size_t)blockIdx.x * (kT2 / 64) + wid) * kGFQ;
    __shared__ uint32_t red_s[kT2 / 64], red_v[kT2 / 64];
    __shared__ uint64_t red_j[kT2 / 64];

    const uint32_t t_begin = blockIdx.x * per;
    const uint32_t t_end = min(a.ntiles, t_begin + per);
    if (t_begin >= t_end) return;
    const uint32_t nch = L.nch;

    for (uint32_t i = tid; i < 256; i += kT2) ntab[i] = kMod - 1 - (a.nm * i) % kMod;
    const uint32_t sh = n & 3;
    const uint32_t rel0 = tid * kR2;
    unsigned long long passes = 0, weak_hits = 0;
    uint32_t nfq = 0;
    uint32_t cur_file = 0xFFFFFFFFu;
    uint32_t fwshift = 0;
    const uint32_t* gfilt = a.filt;
    SegCtx sc;

    unsigned long long tm[4] = {0, 0, 0, 0};
    unsigned long long tprev = a.timing ? __builtin_amdgcn_s_memtime() : 0;
#define PHASE_MARK(k)                                                  \
    if (a.timing) {                                                    \
        const unsigned long long tnow = __builtin_amdgcn_s_memtime(); \
        tm[k] += tnow - tprev;                                         \
        tprev = tnow;                                                  \
    }
    uint32_t si = 0;  // segment of the current tile (tiles are visited in increasing order)
#pragma unroll 1
    for (uint32_t tile = t_begin; tile < t_end; ++tile) {
        // ---- segment of this tile (uniform): first one with tile_base > tile, minus one
        if (tile == t_begin || (si + 1 < a.nsegs && a.segs[si + 1].tile_base <= tile)) {
            uint32_t lo = si, hi = a.nsegs;
            if (tile == t_begin) lo = 0;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (a.segs[mid].tile_base <= tile) lo = mid; else hi = mid;
            }
            si = lo;
            const ScanSeg S = a.segs[si];
            const FileIx F = a.files[S.file];
            sc.base = a.src + S.src;
            sc.pos_begin = S.pos_begin;
            sc.pos_end = S.pos_end;
            sc.keys = a.keys + F.slot_off;
            sc.slot_off = F.slot_off;
            sc.bmask = F.bmask;
            sc.seg_id = si;
            fwshift = F.fwshift;
            gfilt = a.filt + F.filt_off;
            if (kLdsFilter && S.file != cur_file) {
                // the previous tile ended with a barrier; phase 1's barrier publishes the copy
                const uint4* src4 = (const uint4*)gfilt;
                uint4* dst4 = (uint4*)lfilt;
                const uint32_t fwords = 1u << (32 - fwshift);
#pragma unroll 4
                for (uint32_t i = tid; i < fwords / 4; i += kT2) dst4[i] = src4[i];
            }
            cur_file = S.file;
        }
        const uint64_t seg_len = a.segs[si].len;
        const uint64_t tile_start = sc.pos_begin + (uint64_t)(tile - a.segs[si].tile_base) * kTile2;

        // ---- phase 1: tile bytes -> LDS rows, chunk sums (chunks tid, tid + kT2)
#pragma unroll 1
        for (uint32_t c = tid; c < nch; c += kT2) {
            uint32_t x[16];
            load_chunk_nt(sc.base, seg_len, tile_start + 64ull * c, x);
            uint32_t S = 0, V = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                S = udot4(x[i], 0x01010101u, S);
                V = udot4(x[i], offw(i), V);
                rows[c * kRowDw + i] = x[i];
            }
            PS[c] = S;
            PV[c] = V;
        }
        __syncthreads();
        PHASE_MARK(0)

        // ---- phase 2: exclusive prefix over chunks
        {
            const uint32_t per_t = (nch + kT2 - 1) / kT2;
            const uint32_t c_lo = min(nch, tid * per_t), c_hi = min(nch, c_lo + per_t);
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
                const uint32_t s0 = PS[c], v0 = PV[c];
                PS[c] = es; PV[c] = ev; PJ[c] = ej;
                es += s0; ev += v0; ej += (uint64_t)c * s0;
            }
            if (tid == kT2 - 1) { PS[nch] = bs_ + is; PV[nch] = bv_ + iv; PJ[nch] = bj_ + ij; }
            __syncthreads();
        }

        // ---- phase 3: first window of this thread (tile offset 64*tid = start of row tid)
        uint32_t am, bm;
        {
            const uint32_t c0 = tid, m = n >> 6, rem = n & 63;
            const uint64_t dS = PS[c0 + m] - PS[c0];
            const uint64_t dV = PV[c0 + m] - PV[c0];
            const uint64_t dJ = PJ[c0 + m] - PJ[c0];
            uint64_t A = dS;
            uint64_t B = (uint64_t)n * dS - 64ull * (dJ - (uint64_t)c0 * dS) - dV;
            for (uint32_t r = 0; r < rem; ++r) {
                const uint32_t xr = (rows[(c0 + m) * kRowDw + (r >> 2)] >> (8 * (r & 3))) & 0xFF;
                A += xr;
                B += (uint64_t)(rem - r) * xr;
            }
            am = (uint32_t)((1 + A) % kMod);
            bm = (uint32_t)((n + B) % kMod);
        }
        PHASE_MARK(1)

        // ---- phase 4: roll 64 positions in batches of kB2.  Positions at or past
        // pos_end (last tile of a segment) are rolled like the others and dropped by
        // drain3's bound check, so the hot loop carries no bound test.  The pass queue
        // is drained at the top of a batch when it could not take a full batch.
        const uint32_t qtile = (tile - t_begin) << 14;
#pragma unroll 1
        for (uint32_t g = 0; g < (uint32_t)kR2; g += kB2) {
            if (nfq > (uint32_t)(kGFQ - 64 * kB2)) {
                passes += nfq;
                drain3<kRowVerify>(a, fq, nfq, wq, t_begin, weak_hits, kTileFlush ? rows : nullptr, tile_start,
                       kTileFlush ? &sc : nullptr);
                nfq = 0;
            }
            uint32_t xo[4], xi[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) xo[j] = rows[tid * kRowDw + (g >> 2) + j];
            {
                const uint32_t d0 = (rel0 + g + n) >> 2;
                uint32_t dw[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const uint32_t d = d0 + j;
                    dw[j] = rows[(d >> 4) * kRowDw + (d & 15)];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) xi[j] = __builtin_amdgcn_alignbyte(dw[j + 1], dw[j], sh);
            }
            uint32_t ct[kB2];
#pragma unroll
            for (int t = 0; t < kB2; ++t) ct[t] = ntab[(xo[t >> 2] >> (8 * (t & 3))) & 0xFF];
            uint32_t wv[kB2], fh[kB2], fw[kB2];
#pragma unroll
            for (int t = 0; t < kB2; ++t) {
                const uint32_t out = (xo[t >> 2] >> (8 * (t & 3))) & 0xFF;
                const uint32_t in = (xi[t >> 2] >> (8 * (t & 3))) & 0xFF;
                wv[t] = (bm << 16) | am;
                const ProbeHash h = probe_hash(am, bm);
                fh[t] = h.q;
                fw[t] = kLdsFilter ? lfilt[h.r >> fwshift] : gfilt[h.r >> fwshift];
                uint32_t u = am + in - out;  // (-255, M+255), wrapped when negative
                u = min(u, u + kMod);
                am = min(u, u - kMod);
                uint32_t v = bm + am + ct[t];  // [0, 3M)
                v = min(v, v - kMod);
                bm = min(v, v - kMod);
            }
#pragma unroll
            for (int t = 0; t < kB2; ++t) {
                const bool pass = filt_pass(fw[t], fh[t]);
                const uint64_t mk = __ballot(pass);
                if (mk) {
                    if (pass) fq[nfq + __popcll(mk & ((1ull << lane) - 1))] = make_uint2(qtile | (rel0 + g + t), wv[t]);
                    nfq += __popcll(mk);
                }
            }
        }
        PHASE_MARK(2)
        if (kTileFlush && nfq) {  // dense weak hits: verify while the tile is in LDS
            passes += nfq;
            drain3<kRowVerify>(a, fq, nfq, wq, t_begin, weak_hits, rows, tile_start, &sc);
            nfq = 0;
        }
        __syncthreads();  // rows / prefix arrays are rewritten by the next tile
        PHASE_MARK(3)
    }
    passes += nfq;
    drain3<kRowVerify>(a, fq, nfq, wq, t_begin, weak_hits);
#undef PHASE_MARK
    if (lane == 0 && passes) atomicAdd(&a.counters[2], passes);
    if (lane == 0 && weak_hits) atomicAdd(&a.counters[1], weak_hits);
    if (a.timing && tid == 0)
        for (int k = 0; k < 4; ++k) atomicAdd(&a.counters[4 + k], tm[k]);
}

// ===========================================================================
// Shared by the level-1-filter scans (k_scan_r, k_scan_g)
// ===========================================================================
// The BASELINE C3 shape: 2^32 window starts against 2^20 basis keys, every one a
// literal.  Each position must test its weak value against the key set.  With the
// level-2 filter (2 MiB, 16 bits per key) in L2 that is one random L2 request per
// position, and the chip serves ~265 G of those per second whatever their width or
// cache policy (profiles/r02_micro_gather2.txt): >= 16 ms per 4 GiB.  So each
// workgroup keeps a level-1 filter in LDS, and only the positions it passes cost an L2
// request.  Round 2's k_scan_l1 (128 KiB level-1, tile bytes staged in LDS rows, 16.8
// ms at C3) and round 3's k_scan_l2 (32 Ki-position tiles, 14.8 ms) and k_scan_s (a
// stripe per thread, 28.7 ms) were superseded by k_scan_r and removed in round 4; their
// measurements are in DESIGN.md section 6.
constexpr int kB3 = 8;             // positions per batch
constexpr uint32_t kMaxN3 = 4096;  // k_scan_r's window: a wave tile's in rows are the next tile's out rows
constexpr uint32_t kMulti = 0x80000000u;  // fat record: more than one candidate (info = slot)

// Fat-table lookup through the keys-only table: one 16-byte request for the bucket's four
// keys (ScanArgs::keys, 4 B per slot) and the 16-byte record only on a hit (reading the
// bucket's 64-byte line of records for every lookup cost more: round 3).
__device__ __forceinline__ bool fat_find_k(const uint32_t* __restrict__ keys, const uint4* __restrict__ fat,
                                           uint32_t bmask, uint32_t w, uint4& rec) {
    uint32_t b = bucket_hash(w) & bmask;
    for (;;) {
        const uint4 k = *(const uint4*)(keys + 4 * (size_t)b);
        const int j = k.x == w ? 0 : k.y == w ? 1 : k.z == w ? 2 : k.w == w ? 3 : -1;
        if (j >= 0) {
            rec = fat[4 * (size_t)b + j];
            return true;
        }
        if (k.w == kEmptyKey) return false;  // buckets fill in order
        b = (b + 1) & bmask;
    }
}


// One batch of kB3 positions in flight: the level-2 words (buffer loads issued),
// probe hashes and weak values, tested one batch later.
struct L1Batch {
    uint32_t w2[kB3], hq[kB3], wv[kB3];
};

// 16 bytes at src + c0 (16-byte aligned; bytes at or beyond len read as 0).
__device__ __forceinline__ void load16_nt(const uint8_t* src, uint64_t len, uint64_t c0, uint32_t x[4]) {
    if (c0 + 16 <= len) {
        const uint4* q = (const uint4*)(src + c0);
        x[0] = __builtin_nontemporal_load(&q->x);
        x[1] = __builtin_nontemporal_load(&q->y);
        x[2] = __builtin_nontemporal_load(&q->z);
        x[3] = __builtin_nontemporal_load(&q->w);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) {
                const uint64_t p = c0 + 4 * i + b;
                if (p < len) v |= (uint32_t)src[p] << (8 * b);
            }
            x[i] = v;
        }
    }
}

// ===========================================================================
// k_scan_r: the tile's bytes in registers, no workgroup barriers
// ===========================================================================
// Measured on k_scan_l2 (round 3, SYDELTA_ABLATE, C3, profiles/r03p_*): of its 14.8 ms,
// 6.0 ms go away without the level-2 loads (2.9e9 L2 requests, 0.68 per position: the
// chip's L2 request rate bounds the kernel), 1.6 ms without the verification and 0.85 ms
// without the fat-table lookups; the roll alone runs in 6.5 ms.  Fewer L2 requests need
// a larger level-1 filter, and k_scan_l2's LDS is full (36 KiB of staged rows beside the
// 112 KiB filter).  Here no byte is staged in LDS.  Each wave owns wave tiles of 4096
// positions: lane l rolls the 64 positions of row l, whose bytes leave the windows (out
// row [P + 64l, +64)) and enter them (in row [P + n + 64l, +64), n = 4096) from
// registers.  A wave walks a run of consecutive wave tiles, so tile k's in rows are tile
// k+1's out rows and each row is loaded once; the next tile's in rows are loaded while
// the current tile rolls.  First windows come from the two rows' sums by wave scans
// (k_scan_l2's closed form).  Waves never wait for each other: runs of two host tiles
// are handed out by an LDS counter.  The LDS holds the level-1 filter (150 KiB, passing
// 1 - e^(-keys/1228800) of the positions: 0.57 at 1 Mi keys) and ntab.
// Each wave appends its level-2 passes of a wave tile to its own region of HBM (no
// atomics) and, at the tile's end, looks them up (keys-only bucket reads) and verifies
// the weak hits from its registers (wave_strong_regs).  Round 3 measured the other forms
// (DESIGN.md section 6.4): the drains inline from global memory 14.43 ms at C3, the
// records verified by a second kernel from LDS-staged rows 9.88 + 2.81 ms, from the
// registers 11.17 ms.
constexpr int kTR = 512;          // threads per workgroup (8 waves)
constexpr int kWTR = 4096;        // positions per wave tile (64 per lane)
constexpr int kNBR = 64 / kB3;    // batches per lane per wave tile
static_assert(kMaxN3 == 4096 && kWTR % kMaxN3 == 0, "k_scan_r: a lane's in row is row l of the next wave tile");

struct LdsR {
    uint32_t l1, ntab, kt, ctr, total;  // byte offsets
};
__host__ __device__ constexpr LdsR ldsr_layout() {
    LdsR L{};
    uint32_t o = 0;
    L.l1 = o; o += kL1WordsR * 4;
    L.ntab = o; o += 256 * 4;
    L.kt = o; o += 48 * 8;  // wave_strong_regs' key table (kKtWords)
    L.ctr = o; o += 16;
    L.total = o;
    return L;
}
static_assert(ldsr_layout().total <= 160 * 1024 - 256, "k_scan_r's LDS");

// ---------------------------------------------------------------------------
// XXH3-64 of a 4096-byte window held in a wave's registers (k_scan_r, inline verification)
// ---------------------------------------------------------------------------
// The window starts at wave-tile offset o = 64 lp + c of the rows xo (rows 0..63: lane L
// holds row L) and xi (rows 64..127: lane L holds row 64 + L).  Lane s takes stripe s:
// bytes [64 s + c, +64) of rows lp + s and lp + s + 1, gathered with ds_bpermute from the
// owning lanes (the source register index q + j is uniform: v_movrels), aligned by c & 3.
// Stripes 0..62 use keys w[(s & 15) + i], stripe 63 -- the last stripe of a 4096-byte
// input -- the last-stripe keys; the four 16-lane rows are the four 1 KiB blocks, each
// reduced in its row (reduce-scatter: accumulator (L >> 1) & 7 ends in lane L), blocks
// 0..2 followed by a scramble, block 3 (stripes 48..62 and the last stripe) not.  Keys,
// initial accumulators and merge keys come from an LDS table (kt: w[0..23], last[0..7],
// init[0..7], merge[0..7]).  Every lane returns the hash.
constexpr int kKtW = 0, kKtLast = 24, kKtInit = 32, kKtMerge = 40, kKtWords = 48;
typedef uint32_t v16u32 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint64_t dpp64_ctrl_shr4(uint64_t v) {
    return ((uint64_t)dpp32<0x114>((uint32_t)(v >> 32)) << 32) | dpp32<0x114>((uint32_t)v);
}
__device__ __forceinline__ uint64_t dpp64_ctrl_shl4(uint64_t v) {
    return ((uint64_t)dpp32<0x104>((uint32_t)(v >> 32)) << 32) | dpp32<0x104>((uint32_t)v);
}
template <int kCtrl>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    return ((uint64_t)dpp32<kCtrl>((uint32_t)(v >> 32)) << 32) | dpp32<kCtrl>((uint32_t)v);
}

__device__ __forceinline__ uint64_t wave_strong_regs(const uint32_t (&xo)[16], const uint32_t (&xi)[16], uint32_t o,
                                                  const uint64_t* kt) {
    const uint32_t lane = threadIdx.x & 63;
    o = __builtin_amdgcn_readfirstlane(o);
    const uint32_t lp = o >> 6, c = o & 63, q = c >> 2, sh = c & 3;
    v16u32 S0, S1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        S0[r] = lane >= lp ? xo[r] : xi[r];  // global row lp + s for the lane that owns it
        S1[r] = lane > lp ? xo[r] : xi[r];   // global row lp + s + 1 (row lp + 64: xi of lane lp)
    }
    const int addrA = (int)(((lp + lane) & 63) << 2), addrB = (int)(((lp + lane + 1) & 63) << 2);
    uint32_t raw[17];
#pragma unroll
    for (int j = 0; j < 17; ++j) {
        const uint32_t r = q + j;  // uniform
        const uint32_t v = r < 16 ? S0[r & 15] : S1[r & 15];
        raw[j] = (uint32_t)__builtin_amdgcn_ds_bpermute(r < 16 ? addrA : addrB, (int)v);
    }
    const uint32_t kb = lane == 63 ? (uint32_t)kKtLast : (lane & 15);
    uint64_t cc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) cc[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t w0 = __builtin_amdgcn_alignbyte(raw[2 * i + 1], raw[2 * i], sh);
        const uint32_t w1 = __builtin_amdgcn_alignbyte(raw[2 * i + 2], raw[2 * i + 1], sh);
        const uint64_t v = (uint64_t)w0 | ((uint64_t)w1 << 32);
        const uint64_t dk = v ^ kt[kb + i];
        cc[i ^ 1] += v;
        cc[i] += mul32x32(dk);
    }
    // reduce-scatter inside each 16-lane row: lane L ends with accumulator (L >> 1) & 7
    uint64_t f;
    const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
    uint64_t d[4], e[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t send = b3 ? cc[k] : cc[4 + k], keep = b3 ? cc[4 + k] : cc[k];
        d[k] = keep + dpp64<kDppRowRor8>(send);  // row_ror:8 = xor 8
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint64_t send = b2 ? d[k] : d[2 + k], keep = b2 ? d[2 + k] : d[k];
        // both shifts in every lane, then the select: a DPP inside the conditional would run
        // with the partner lanes masked off and read 0 from them
        const uint64_t from_lo = dpp64_ctrl_shr4(send), from_hi = dpp64_ctrl_shl4(send);
        e[k] = keep + (b2 ? from_lo : from_hi);  // lane L ^ 4
    }
    {
        const uint64_t send = b1 ? e[0] : e[1], keep = b1 ? e[1] : e[0];
        f = keep + dpp64<kDppQuadXor2>(send);
    }
    f += dpp64<kDppQuadXor1>(f);
    // blocks 1..3 from the rows below; lanes 0..15 carry the chain
    const uint64_t p1 = shfl64(f, (int)((lane + 16) & 63));
    const uint64_t p2 = shfl64(f, (int)((lane + 32) & 63));
    const uint64_t p3 = shfl64(f, (int)((lane + 48) & 63));
    const uint32_t ai = (lane >> 1) & 7;
    const uint64_t skey = kt[kKtW + 16 + ai];
    uint64_t acc = kt[kKtInit + ai] + f;
    acc = scramble1(acc, skey) + p1;
    acc = scramble1(acc, skey) + p2;
    acc = scramble1(acc, skey) + p3;
    // merge: accumulators 2k, 2k+1 sit in lanes L, L ^ 2 (L % 4 == 0 holds 2k)
    const uint64_t z = acc ^ kt[kKtMerge + ai];
    const uint64_t zp = dpp64<kDppQuadXor2>(z);
    uint64_t m = (lane & 3) == 0 ? fold64(z, zp) : 0ull;
    m += dpp64<kDppRowRor4>(m);
    m += dpp64<kDppRowRor8>(m);
    const uint64_t h = xxh3_aval((uint64_t)4096 * P64_1 + m);
    return ((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(h >> 32), 0) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)h, 0);
}

// ---------------------------------------------------------------------------
// Per-wave staging of appended outputs (WaveOut)
// ---------------------------------------------------------------------------
// The register-fed scans and k_verify_w append verified hits (and k_scan_g its deferred
// weak hits) to lists shared by the whole launch.  Taking list slots with a returning
// atomicAdd per wave round costs one device-scope atomic on ONE word per round with a
// hit, and one word serves about 88 of those per microsecond chip-wide
// (MI355X_MICROARCH.md, dequeue): C3b's 1 M verified hits (one per wave tile) queued
// behind it, +4.7 ms of k_scan_r (profiles/r04c_c3b_bench.json).  So each wave writes its
// outputs to its own region (ScanArgs::hstage / dstage, no atomics) and moves them to the
// shared list with one atomicAdd per flush (a full region, or the wave's end).  The
// list's order changes, not its contents: the host sorts the hits by key.
constexpr uint32_t kHStage = 256;  // verified hits staged per wave {key lo, key hi, block, 0}
constexpr uint32_t kDStage = 64;   // deferred weak hits staged per wave

struct WaveOut {
    uint4* h;     // this wave's hit region
    WDef* d;      // this wave's deferred region (k_scan_g)
    uint32_t nh;  // staged hits (wave-uniform)
    uint32_t nd;  // staged deferred hits (wave-uniform)
};

// gwave: the wave's index in the launch (regions are kHStage / kDStage entries apart)
__device__ __forceinline__ WaveOut wave_out(const ScanArgs& a, uint64_t gwave) {
    WaveOut o;
    o.h = a.hstage + gwave * kHStage;
    o.d = a.dstage ? a.dstage + gwave * kDStage : nullptr;
    o.nh = 0;
    o.nd = 0;
    return o;
}

// Move the staged hits to the output list [counters[0], +nh) (slots past out_cap are
// counted, not written: the host grows the list and scans again).
__device__ __forceinline__ void flush_hits(const ScanArgs& a, WaveOut& o) {
    if (!o.nh) return;
    const uint32_t lane = threadIdx.x & 63;
    __threadfence_block();  // this wave's staging stores before its loads
    unsigned long long k0 = 0;
    if (lane == 0) k0 = atomicAdd(&a.counters[0], (unsigned long long)o.nh);
    k0 = shfl64(k0, 0);
    for (uint32_t i = lane; i < o.nh; i += 64) {
        const volatile uint4* g = o.h + i;  // rewritten by later flushes: not from a stale L1 line
        const uint32_t lo = g->x, hi = g->y, blk = g->z;
        const unsigned long long k = k0 + i;
        if (k < a.out_cap) {
            a.hit_key[k] = ((uint64_t)hi << 32) | lo;
            a.hit_val[k] = blk;
        }
    }
    o.nh = 0;
}

// Stage the hits of the lanes with v (key, block): wave-uniform call.
__device__ __forceinline__ void stage_hits(const ScanArgs& a, WaveOut& o, bool v, uint64_t key, uint32_t blk) {
    const uint64_t m = __ballot(v);
    if (!m) return;
    const uint32_t c = __popcll(m);
    if (o.nh + c > kHStage) flush_hits(a, o);
    const uint32_t lane = threadIdx.x & 63;
    if (v) o.h[o.nh + __popcll(m & ((1ull << lane) - 1))] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), blk, 0);
    o.nh += c;
}

// One deferred weak hit verified by the whole wave from global memory (the window at
// d.at): XXH3 of the window, then the first candidate in index order with equal strong
// (generator.rs:127-133).  Every lane returns the block or kNoBlock.
__device__ __forceinline__ uint32_t verify_def(const ScanArgs& a, const WDef& d) {
    uint64_t st;
    if (a.n > 240) {
        uint32_t wk;
        wave_hash_long(a.src + d.at, a.n, wk, st);
    } else {  // XXH3's short paths
        st = 0;
        if ((threadIdx.x & 63) == 0) st = xxh3_short(a.src + d.at, a.n);
        st = shfl64(st, 0);
    }
    if (!(d.cand & kMulti)) return st == d.strong ? d.cand : kNoBlock;
    return first_strong_match(a.order, a.cstrong, a.start[d.cand & ~kMulti], a.cnt[d.cand & ~kMulti], st);
}

// Move the staged deferred weak hits to a.wdef [counters[10], +nd); the ones past
// wdef_cap are verified here, one window per wave step (their hits staged).
__device__ __forceinline__ void flush_defs(const ScanArgs& a, WaveOut& o) {
    if (!o.nd) return;
    const uint32_t lane = threadIdx.x & 63;
    __threadfence_block();
    unsigned long long k0 = 0;
    if (lane == 0) k0 = atomicAdd(&a.counters[10], (unsigned long long)o.nd);
    k0 = shfl64(k0, 0);
    for (uint32_t i = lane; i < o.nd; i += 64) {
        const unsigned long long k = k0 + i;
        if (k < a.wdef_cap) {
            const volatile uint64_t* g = (const volatile uint64_t*)(o.d + i);
            WDef d;
            d.at = g[0];
            d.key = g[1];
            const uint64_t cp = g[2];
            d.cand = (uint32_t)cp;
            d.pad = 0;
            d.strong = g[3];
            a.wdef[k] = d;
        }
    }
    if (k0 + o.nd > a.wdef_cap) {  // the list is full: verify the rest here
        const uint32_t first = k0 >= a.wdef_cap ? 0u : (uint32_t)(a.wdef_cap - k0);
        for (uint32_t i = first; i < o.nd; ++i) {  // wave-uniform
            const volatile uint64_t* g = (const volatile uint64_t*)(o.d + i);
            WDef d;
            d.at = g[0];
            d.key = g[1];
            d.cand = (uint32_t)g[2];
            d.pad = 0;
            d.strong = g[3];
            const uint32_t best = verify_def(a, d);
            stage_hits(a, o, lane == 0 && best != kNoBlock, d.key, best);
        }
    }
    o.nd = 0;
}

// Stage the deferred weak hits of the lanes with v: wave-uniform call.
__device__ __forceinline__ void stage_defs(const ScanArgs& a, WaveOut& o, bool v, const WDef& d) {
    const uint64_t m = __ballot(v);
    if (!m) return;
    const uint32_t c = __popcll(m);
    if (o.nd + c > kDStage) flush_defs(a, o);
    const uint32_t lane = threadIdx.x & 63;
    if (v) o.d[o.nd + __popcll(m & ((1ull << lane) - 1))] = d;
    o.nd += c;
}

// Inline drain of one wave tile's level-2 pass records [0, nr) (just written by this wave
// to its region): keys-only lookups, 64 per round; each weak hit's window is hashed from
// the registers (wave_strong_regs, one window at a time for the whole wave), the first
// candidate in index order with equal strong taken (generator.rs:127-133); verified hits
// to the output.  tile_rel: the run position of the tile's first window.
// kSmall: the index has no fat table (small files): the exact table's slot is looked up and
// its candidates swept in index order (first_strong_match).
template <bool kSmall = false>
__device__ __forceinline__ void drain_regs(const ScanArgs& a, const uint2* recs, uint32_t nr, uint32_t tile_rel,
                                           const uint32_t (&xo)[16], const uint32_t (&xi)[16], const uint64_t* kt,
                                           unsigned long long& weak_hits, uint64_t run_start, const SegCtx& cur,
                                           WaveOut& o) {
    const uint32_t lane = threadIdx.x & 63;
    __threadfence_block();  // this wave's record stores before its loads
    for (uint32_t base = 0; base < nr; base += 64) {
        const uint32_t i = base + lane;
        bool hit = false;
        uint4 rec = make_uint4(0, 0, 0, 0);
        uint32_t pos = 0;
        if (i < nr) {
            const volatile uint2* g = recs + i;  // rewritten by later tiles: not from a stale L1 line
            pos = g->x;
            const uint32_t w = g->y;
            if (run_start + pos < cur.pos_end) {
                if (kSmall) {
                    const int64_t sl = table_find(cur.keys, cur.bmask, w);
                    hit = sl >= 0;
                    rec.y = kMulti | (uint32_t)(cur.slot_off + (uint64_t)(sl < 0 ? 0 : sl));
                } else {
                    hit = fat_find_k(cur.keys, cur.fat, cur.bmask, w, rec);
                }
            }
        }
        uint64_t m = __ballot(hit);
        weak_hits += __popcll(m);
        uint32_t best_mine = kNoBlock;
        while (m) {  // wave-uniform
            const int h = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t hp = __builtin_amdgcn_readlane((int)pos, h);
            const uint32_t hy = __builtin_amdgcn_readlane((int)rec.y, h);
            const uint64_t hs = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rec.w, h) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)rec.z, h);
            const uint64_t st = wave_strong_regs(xo, xi, hp - tile_rel, kt);
            uint32_t best = kNoBlock;
            if (!(hy & kMulti)) {
                if (st == hs) best = hy;
            } else {
                best = first_strong_match(a.order, a.cstrong, a.start[hy & ~kMulti], a.cnt[hy & ~kMulti], st);
            }
            if ((int)lane == h) best_mine = best;
        }
        stage_hits(a, o, best_mine != kNoBlock,
                   ((uint64_t)cur.seg_id << kSegShift) | (uint64_t)(run_start + pos - cur.pos_begin), best_mine);
    }
}

// Each wave tile's passes are looked up and verified at the tile's end (drain_regs: the
// windows hashed from the registers).
// kRib: the level-1 words hold the ribbon (rib_bit / rib_coef: a position passes when the
// parity of its coefficients over its window is even), else the one-hash Bloom (l1r_word).
// kWaves: waves per workgroup (one workgroup per CU: the level-1 filter fills the LDS);
// 12 = three per SIMD, which caps the kernel at 168 VGPRs.
// kSmall: small indexes (each file's Bloom filter <= kSmallWordsR words): no level-1 /
// level-2; each wave copies the filter of the file it scans into its own LDS slot and
// tests every position there (k_scan_g's small mode, with the windows verified from the
// registers).
template <bool kRib, int kWaves, bool kSmall = false>
__global__ __launch_bounds__(kWaves * 64, 1) void k_scan_r(ScanArgs a, uint32_t per, uint32_t small_words) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr LdsR L = ldsr_layout();
    constexpr uint32_t kT = kWaves * 64;
    const uint32_t n = a.n;  // kMaxN3 (launch_scan)
    const uint32_t* l1 = (const uint32_t*)(smem + L.l1);
    uint32_t* ntab = (uint32_t*)(smem + L.ntab);
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    uint32_t* ctr = (uint32_t*)(smem + L.ctr);
    const uint32_t gwave = blockIdx.x * kWaves + wid;
    uint2* rec = a.rrec + (size_t)gwave * kWTR;  // this wave's pass records (one wave tile)
    uint32_t* fslot = (uint32_t*)(smem + L.l1) + (size_t)wid * small_words;  // kSmall: this wave's filter
    uint32_t slot_file = 0xFFFFFFFFu;
    WaveOut wo = wave_out(a, gwave);

    const uint32_t t_begin = blockIdx.x * per;
    const uint32_t t_end = min(a.ntiles, t_begin + per);
    if (t_begin >= t_end) return;
    if (!kSmall) {
        const uint4* g = (const uint4*)a.l1;
        uint4* d = (uint4*)(smem + L.l1);
#pragma unroll 4
        for (uint32_t i = tid; i < kL1WordsR / 4; i += kT) d[i] = g[i];
    }
    for (uint32_t i = tid; i < 256; i += kT) ntab[i] = kMod - 1 - (a.nm * i) % kMod;
    uint64_t* kt = (uint64_t*)(smem + L.kt);
    if (tid < 48)
        kt[tid] = tid < 24 ? c_tab.w[tid] : tid < 32 ? c_tab.last[tid - 24] : tid < 40 ? c_tab.init[tid - 32]
                                                                                       : c_tab.merge[tid - 40];
    if (tid == 0) *ctr = 0;
    __syncthreads();  // the only barrier: the waves run independently from here

    unsigned long long passes = 0, weak_hits = 0;
    uint32_t nrec = 0, si_hint = 0;
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll 1
    for (;;) {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(ctr, 1u);
        c = __builtin_amdgcn_readfirstlane(c);
        const uint32_t t0 = t_begin + 2 * c;
        if (t0 >= t_end) break;
        const uint32_t tz = min(t_end, t0 + 2);
#pragma unroll 1
        for (uint32_t t = t0; t < tz;) {
            // the run: host tiles t (and t+1 when in the same segment)
            uint32_t lo = si_hint, hi = a.nsegs;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (a.segs[mid].tile_base <= t) lo = mid; else hi = mid;
            }
            const uint32_t si = lo;
            si_hint = si;
            const ScanSeg S = a.segs[si];
            const FileIx F = a.files[S.file];
            SegCtx sc;
            sc.base = a.src + S.src;
            sc.pos_begin = S.pos_begin;
            sc.keys = a.keys + F.slot_off;
            sc.fat = a.fat + F.slot_off;
            sc.slot_off = F.slot_off;
            sc.bmask = F.bmask;
            sc.seg_id = si;
            sc.fwshift = F.fwshift;
            sc.filt = a.filt + F.filt_off;
            sc.fwords = 1u << (32 - F.fwshift);
            const uint32_t span = (t + 1 < tz && !(si + 1 < a.nsegs && a.segs[si + 1].tile_base <= t + 1)) ? 2u : 1u;
            const uint64_t run_start = S.pos_begin + (uint64_t)(t - S.tile_base) * kTile2;
            sc.pos_end = min(S.pos_end, run_start + (uint64_t)span * kTile2);
            const uint64_t seg_len = S.len;
            const uint32_t nwt = span * (kTile2 / kWTR);  // wave tiles of the run
            t += span;

            const uint64_t fptr = (uint64_t)(uintptr_t)sc.filt;
            const uint32_t fp_lo = __builtin_amdgcn_readfirstlane((uint32_t)fptr);
            const uint32_t fp_hi = __builtin_amdgcn_readfirstlane((uint32_t)(fptr >> 32));
            const __amdgpu_buffer_rsrc_t frsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(uintptr_t)(((uint64_t)fp_hi << 32) | fp_lo), (short)0,
                (int)__builtin_amdgcn_readfirstlane(sc.fwords * 4), 0x00020000);
            const uint32_t fwshift = __builtin_amdgcn_readfirstlane(sc.fwshift);
            if (kSmall && S.file != slot_file) {  // this file's filter into the wave's slot
                slot_file = S.file;
                lds_fence();
                const uint4* g = (const uint4*)sc.filt;
                uint4* d = (uint4*)fslot;
                for (uint32_t i = lane; i < sc.fwords / 4; i += 64) d[i] = g[i];
                lds_fence();
            }

            uint32_t xo[16], xi[16], xn[16];
            load_chunk_nt(sc.base, seg_len, run_start + 64ull * lane, xo);  // read once: not kept in L2
            load_chunk_nt(sc.base, seg_len, run_start + n + 64ull * lane, xi);
#pragma unroll 1
            for (uint32_t k = 0; k < nwt; ++k) {
                const uint64_t P = run_start + (uint64_t)k * kWTR;
                const uint32_t rel0 = k * kWTR + lane * 64;  // position in run of this lane's first window
                // ---- window: lane l's window [P + 64l, +n) = out rows l..63 + in rows 0..l-1
                uint32_t am, bm;
                {
                    uint32_t Sx[2], Vx[2], Jx[2], TS[2], TV[2], TJ[2];
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        uint32_t s = 0, v = 0;
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const uint32_t d = j ? xi[i] : xo[i];
                            s = udot4(d, 0x01010101u, s);
                            v = udot4(d, offw(i), v);
                        }
                        Sx[j] = wave_scan_excl(s, TS[j]);
                        Vx[j] = wave_scan_excl(v, TV[j]);
                        Jx[j] = wave_scan_excl((uint32_t)(64 * j + lane) * s, TJ[j]);
                    }
                    const uint64_t dS = TS[0] + Sx[1] - Sx[0];
                    const uint64_t dV = TV[0] + Vx[1] - Vx[0];
                    const uint64_t dJ = TJ[0] + Jx[1] - Jx[0];
                    const uint32_t A = (uint32_t)dS;
                    const uint32_t B = (uint32_t)((uint64_t)n * dS - 64ull * (dJ - (uint64_t)lane * dS) - dV);
                    am = (1 + A) % kMod;
                    bm = (n + B) % kMod;
                }
                // ---- roll: k_scan_l2's trimmed roll, bytes from the registers
                auto compute = [&](const int g, L1Batch& Bt) {
                    const uint32_t xo0 = xo[g >> 2], xo1 = xo[(g >> 2) + 1];
                    const uint32_t xi0 = xi[g >> 2], xi1 = xi[(g >> 2) + 1];
                    uint32_t ct[kB3], rr[kB3], w1[kB3], w1b[kB3], bo[kB3];
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) ct[t2] = ntab[((t2 < 4 ? xo0 : xo1) >> (8 * (t2 & 3))) & 0xFF];
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) {
                        const uint32_t out = ((t2 < 4 ? xo0 : xo1) >> (8 * (t2 & 3))) & 0xFF;
                        const uint32_t in = ((t2 < 4 ? xi0 : xi1) >> (8 * (t2 & 3))) & 0xFF;
                        __builtin_assume(am < kMod);
                        __builtin_assume(bm < kMod);
                        Bt.wv[t2] = (bm << 16) | am;
                        const ProbeHash h = probe_hash(am, bm);
                        Bt.hq[t2] = h.q;
                        rr[t2] = h.r;
                        if (kSmall) {
                            Bt.w2[t2] = fslot[h.r >> fwshift];  // the file's whole filter, tested in finish
                        } else if (kRib) {  // the window's two words (ds_read2_b32)
                            bo[t2] = rib_bit(h.q, h.r);
                            w1[t2] = l1[bo[t2] >> 5];
                            w1b[t2] = l1[(bo[t2] >> 5) + 1];
                        } else {
                            w1[t2] = l1[l1r_word(h.q)];
                        }
                        const uint32_t u = am + in + (kMod - out);  // [M-255, 2M+255)
                        am = min(u, min(u - kMod, u - 2 * kMod));
                        const uint32_t v = bm + am + ct[t2];          // [0, 3M)
                        bm = min(v, min(v - kMod, v - 2 * kMod));
                    }
#pragma unroll
                    for (int t2 = 0; t2 < kB3 && !kSmall; ++t2) {
                        uint32_t p1;
                        if (kRib) {
                            const uint32_t win = __builtin_amdgcn_alignbit(w1b[t2], w1[t2], bo[t2]);
                            p1 = ~__builtin_popcount(win & rib_coef(Bt.hq[t2], rr[t2])) & 1u;
                        } else {
                            p1 = l1_test(w1[t2], Bt.hq[t2]);
                        }
                        // a level-1 miss asks for an offset past the buffer: no request, reads 0
                        Bt.w2[t2] = __builtin_amdgcn_raw_buffer_load_b32(frsrc, (int)(((rr[t2] >> fwshift) << 2) | (p1 - 1u)),
                                                                         0, 0);
                    }
                };
                auto finish = [&](const int g, L1Batch& Bt) {
                    uint32_t pbits = 0;
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) pbits |= filt_bit(Bt.w2[t2], Bt.hq[t2]) << t2;
                    asm volatile("" : "+v"(pbits));
                    if (!__ballot(pbits != 0)) return;
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) {  // appended in position order per batch
                        const uint64_t mk = __ballot((pbits >> t2) & 1);
                        if (!mk) continue;
                        if ((pbits >> t2) & 1) rec[nrec + __popcll(mk & below)] = make_uint2(rel0 + g + t2, Bt.wv[t2]);
                        nrec += __popcll(mk);
                    }
                };
                // batch b+2's level-2 loads are issued before batch b is tested; the next
                // wave tile's in rows after batch 4's (so that a wait on batches 0..4's
                // loads never waits on them, and they land before the tile ends)
                const uint32_t tile_rec = nrec;
                L1Batch b0, b1;
                compute(0, b0);
                compute(8, b1);
#pragma unroll
                for (int bi = 0; bi < kNBR; ++bi) {
                    L1Batch& Bt = (bi & 1) ? b1 : b0;
                    finish(kB3 * bi, Bt);
                    if (bi + 2 < kNBR) compute(kB3 * (bi + 2), Bt);
                    if (bi == 2 && k + 1 < nwt)
                        load_chunk_nt(sc.base, seg_len, P + n + kWTR + 64ull * lane, xn);
                }
                passes += nrec - tile_rec;
                if (nrec > tile_rec)
                    drain_regs<kSmall>(a, rec + tile_rec, nrec - tile_rec, k * kWTR, xo, xi, kt, weak_hits, run_start, sc,
                                       wo);
                nrec = tile_rec;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    xo[i] = xi[i];
                    xi[i] = xn[i];
                }
            }
        }
    }
    flush_hits(a, wo);
    if (lane == 0 && passes) atomicAdd(&a.counters[2], passes);
    if (lane == 0 && weak_hits) atomicAdd(&a.counters[1], weak_hits);
}

// ===========================================================================
// k_scan_g: k_scan_r's register-fed roll for any window n (one large file)
// ===========================================================================
// k_scan_r needs n = 4096: a wave tile's in rows are then the next tile's out rows, and
// lane l's first window is out rows l..63 + in rows 0..l-1.  For any other n the out
// rows [P + 64l, +64) and the in rows [P + n + 64l, +64) are loaded separately (the in
// rows at any alignment: load64_u), and the first windows follow from the window at the
// tile's start, (A0, B0), in closed form (rolling.rs:66-79 applied d = 64l times):
//   A(d) = A0 + In(d) - Out(d)
//   B(d) = B0 + d (A0 - 1) + sum_{j<d} (d - j) in_j - sum_{j<d} (d - j) out_j - n Out(d)
// from exclusive wave scans of the rows' sums; (A0, B0) of the next tile is lane 63's
// window after its 64 rolls.  A run's first window is summed from global memory
// (window_at).  The level-1 filter (Bloom or ribbon), level-2 loads and the keys-only
// lookups are k_scan_r's; a weak hit's window is not in the registers, so it goes to the
// deferred list (WDef) that k_verify_w hashes after the scan (hits the list cannot take
// are verified inline from global memory).  Replaces round 3's k_scan_w (windows above 8 KiB:
// 8.63 + 1.29 ms per 4 GiB at bs 65536) and
// k_scan_lds in global-filter mode for single-file indexes.

// 64 bytes at byte offset q of src (any alignment) through 16-byte granule loads and
// alignbyte; bytes at or beyond len read as 0 (only granules holding a byte of [0, len)
// are loaded).
__device__ __forceinline__ void load64_u(const uint8_t* src, uint64_t len, uint64_t q, uint32_t x[16]) {
    const uint32_t sh = (uint32_t)q & 15u;
    if (!sh) {
        load_chunk(src, len, q, x);
        return;
    }
    const uint64_t qa = q - sh;
    const uint4* g = (const uint4*)(src + qa);
    uint32_t d[20];
    if (qa + 80 <= len) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint4 v = g[i];
            d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (qa + 16 * i < len) v = g[i];
            d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 20; ++i) {
            const uint64_t o = qa + 4 * i;
            d[i] &= o >= len ? 0u : (o + 4 <= len ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (o + 4 - len))));
        }
    }
    const uint32_t ds = sh >> 2, bs = sh & 3;
    uint32_t e[17];
#pragma unroll
    for (int i = 0; i < 17; ++i) e[i] = ds == 0 ? d[i] : ds == 1 ? d[i + 1] : ds == 2 ? d[i + 2] : d[i + 3];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(e[i + 1], e[i], bs);
}

// Adler-32 state (A, B) of the window [P, P + n) of src (rolling.rs:35-45: A = 1 + sum x,
// B = n + sum (n - i) x_i, mod M), summed by the whole wave; every lane returns it.
__device__ __forceinline__ void window_at(const uint8_t* src, uint64_t len, uint64_t P, uint32_t n, uint32_t& am,
                                          uint32_t& bm) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t s = 0, t = 0;  // sum x, sum i x_i (i from the window start)
    for (uint32_t c = 64 * lane; c < n; c += 64 * 64) {
        uint32_t x[16];
        load64_u(src, len, P + c, x);
        uint32_t cs = 0, cv = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t j = c + 4 * i;
            const uint32_t keep = j >= n ? 0u : (j + 4 <= n ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (j + 4 - n))));
            const uint32_t v = x[i] & keep;
            cs = udot4(v, 0x01010101u, cs);
            cv = udot4(v, offw(i), cv);
        }
        s += cs;
        t += (uint64_t)c * cs + cv;
    }
    s = wave_sum64(s);
    t = wave_sum64(t);
    am = (uint32_t)((1 + s) % kMod);
    bm = (uint32_t)((n + (uint64_t)n * s - t) % kMod);
}

// Lookups of one wave tile's level-2 pass records (keys-only bucket reads, 64 per round);
// weak hits are staged for the deferred list a.wdef (flush_defs), which k_verify_w hashes
// after the scan.
__device__ __forceinline__ void drain_g(const ScanArgs& a, const uint2* recs, uint32_t nr, unsigned long long& weak_hits,
                                        uint64_t run_start, const SegCtx& cur, WaveOut& o) {
    const uint32_t lane = threadIdx.x & 63;
    __threadfence_block();  // this wave's record stores before its loads
    for (uint32_t base = 0; base < nr; base += 64) {
        const uint32_t i = base + lane;
        bool hit = false;
        uint4 rec = make_uint4(0, 0, 0, 0);
        uint32_t pos = 0;
        if (i < nr) {
            const volatile uint2* g = recs + i;  // rewritten by later tiles: not from a stale L1 line
            pos = g->x;
            const uint32_t w = g->y;
            if (run_start + pos < cur.pos_end) hit = fat_find_k(cur.keys, cur.fat, cur.bmask, w, rec);
        }
        const uint64_t m = __ballot(hit);
        if (!m) continue;
        weak_hits += __popcll(m);
        const uint64_t p = run_start + pos;
        WDef d;
        d.at = (uint64_t)(cur.base - a.src) + p;
        d.key = ((uint64_t)cur.seg_id << kSegShift) | (p - cur.pos_begin);
        d.cand = rec.y;
        d.pad = 0;
        d.strong = ((uint64_t)rec.w << 32) | rec.z;
        stage_defs(a, o, hit, d);
    }
}

// kSmall's drain: exact-table lookups (table_find; small indexes carry no fat table), 64
// per round; each weak hit is staged for the deferred list as {window, key, kMulti |
// global slot} (k_verify_w looks its candidates up in index order).
__device__ __forceinline__ void drain_gs(const ScanArgs& a, const uint2* recs, uint32_t nr,
                                         unsigned long long& weak_hits, uint64_t run_start, const SegCtx& cur,
                                         WaveOut& o) {
    const uint32_t lane = threadIdx.x & 63;
    __threadfence_block();  // this wave's record stores before its loads
    for (uint32_t base = 0; base < nr; base += 64) {
        const uint32_t i = base + lane;
        bool hit = false;
        uint32_t pos = 0, gslot = 0;
        if (i < nr) {
            const volatile uint2* g = recs + i;
            pos = g->x;
            const uint32_t w = g->y;
            if (run_start + pos < cur.pos_end) {
                const int64_t sl = table_find(cur.keys, cur.bmask, w);
                hit = sl >= 0;
                gslot = (uint32_t)(cur.slot_off + (uint64_t)(sl < 0 ? 0 : sl));
            }
        }
        const uint64_t m = __ballot(hit);
        if (!m) continue;
        weak_hits += __popcll(m);
        const uint64_t p = run_start + pos;
        WDef d;
        d.at = (uint64_t)(cur.base - a.src) + p;
        d.key = ((uint64_t)cur.seg_id << kSegShift) | (p - cur.pos_begin);
        d.cand = kMulti | gslot;
        d.pad = 0;
        d.strong = 0;
        stage_defs(a, o, hit, d);
    }
}

struct LdsG {
    uint32_t l1, ntab, ctr, total;  // byte offsets
};
// small_words: kSmall's per-wave filter slot (the largest file filter of the index), else 0
__host__ __device__ constexpr LdsG ldsg_layout(uint32_t small_words = 0) {
    LdsG L{};
    uint32_t o = 0;
    L.l1 = o; o += small_words ? (kTR / 64) * small_words * 4 : kL1WordsR * 4;
    L.ntab = o; o += 256 * 4;
    L.ctr = o; o += 16;
    L.total = o;
    return L;
}
static_assert(ldsg_layout().total <= 160 * 1024 - 256, "k_scan_g's LDS");

// per: host tiles per workgroup (a multiple of rt); rt: host tiles per run (the unit a wave
// takes from the workgroup's counter, sized so the run's first window, summed from global
// memory, is a small part of the run's reads).
// kSmall: small indexes (one or many files, each with its Bloom filter of <= kSmallWords
// words): no level-1 filter and no level-2 loads; each wave copies the filter of the file
// it scans into its own LDS slot (small_words words) and tests every position there;
// passes are looked up in the exact table (drain_gs).  Replaces k_scan_lds for them.
template <bool kRib, bool kSmall>
__global__ __launch_bounds__(kTR, 2) void k_scan_g(ScanArgs a, uint32_t per, uint32_t rt, uint32_t small_words) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const LdsG L = ldsg_layout(kSmall ? small_words : 0u);
    const uint32_t n = a.n;
    const uint32_t* l1 = (const uint32_t*)(smem + L.l1);
    uint32_t* ntab = (uint32_t*)(smem + L.ntab);
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    uint32_t* ctr = (uint32_t*)(smem + L.ctr);
    const uint32_t gwave = blockIdx.x * (kTR / 64) + wid;
    uint2* rec = a.rrec + (size_t)gwave * kWTR;  // this wave's pass records (one wave tile)
    WaveOut wo = wave_out(a, gwave);
    uint32_t* fslot = (uint32_t*)(smem + L.l1) + (size_t)wid * small_words;  // kSmall: this wave's filter

    const uint32_t t_begin = blockIdx.x * per;
    const uint32_t t_end = min(a.ntiles, t_begin + per);
    if (t_begin >= t_end) return;
    if (!kSmall) {
        const uint4* g = (const uint4*)a.l1;
        uint4* d = (uint4*)(smem + L.l1);
#pragma unroll 4
        for (uint32_t i = tid; i < kL1WordsR / 4; i += kTR) d[i] = g[i];
    }
    for (uint32_t i = tid; i < 256; i += kTR) ntab[i] = kMod - 1 - (a.nm * i) % kMod;
    if (tid == 0) *ctr = 0;
    __syncthreads();  // the only barrier: the waves run independently from here

    unsigned long long passes = 0, weak_hits = 0;
    uint32_t nrec = 0, si_hint = 0, slot_file = 0xFFFFFFFFu;
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll 1
    for (;;) {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(ctr, 1u);
        c = __builtin_amdgcn_readfirstlane(c);
        const uint32_t t0 = t_begin + rt * c;
        if (t0 >= t_end) break;
        const uint32_t tz = min(t_end, t0 + rt);
#pragma unroll 1
        for (uint32_t t = t0; t < tz;) {
            // the part of the run in one segment: host tiles [t, t + span)
            uint32_t lo = si_hint, hi = a.nsegs;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (a.segs[mid].tile_base <= t) lo = mid; else hi = mid;
            }
            const uint32_t si = lo;
            si_hint = si;
            const ScanSeg S = a.segs[si];
            const FileIx F = a.files[S.file];
            SegCtx sc;
            sc.base = a.src + S.src;
            sc.pos_begin = S.pos_begin;
            sc.keys = a.keys + F.slot_off;
            sc.fat = a.fat + F.slot_off;
            sc.slot_off = F.slot_off;
            sc.bmask = F.bmask;
            sc.seg_id = si;
            sc.fwshift = F.fwshift;
            sc.filt = a.filt + F.filt_off;
            sc.fwords = 1u << (32 - F.fwshift);
            const uint32_t seg_tend = si + 1 < a.nsegs ? a.segs[si + 1].tile_base : a.ntiles;
            const uint32_t span = min(tz, seg_tend) - t;
            const uint64_t run_start = S.pos_begin + (uint64_t)(t - S.tile_base) * kTile2;
            sc.pos_end = min(S.pos_end, run_start + (uint64_t)span * kTile2);
            const uint64_t seg_len = S.len;
            const uint32_t nwt = (uint32_t)((sc.pos_end - run_start + kWTR - 1) / kWTR);  // wave tiles with positions
            t += span;

            const uint64_t fptr = (uint64_t)(uintptr_t)sc.filt;
            const uint32_t fp_lo = __builtin_amdgcn_readfirstlane((uint32_t)fptr);
            const uint32_t fp_hi = __builtin_amdgcn_readfirstlane((uint32_t)(fptr >> 32));
            const __amdgpu_buffer_rsrc_t frsrc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(uintptr_t)(((uint64_t)fp_hi << 32) | fp_lo), (short)0,
                (int)__builtin_amdgcn_readfirstlane(sc.fwords * 4), 0x00020000);
            const uint32_t fwshift = __builtin_amdgcn_readfirstlane(sc.fwshift);
            if (kSmall && S.file != slot_file) {  // this file's filter into the wave's slot
                slot_file = S.file;
                lds_fence();  // the previous file's words are no longer read
                const uint4* g = (const uint4*)sc.filt;
                uint4* d = (uint4*)fslot;
                for (uint32_t i = lane; i < sc.fwords / 4; i += 64) d[i] = g[i];
                lds_fence();
            }

            uint32_t A0, B0;  // the window at the current wave tile's start
            window_at(sc.base, seg_len, run_start, n, A0, B0);
            uint32_t xo[16], xi[16], no_[16], ni_[16];
            load_chunk_nt(sc.base, seg_len, run_start + 64ull * lane, xo);  // the bytes' last read
            load64_u(sc.base, seg_len, run_start + n + 64ull * lane, xi);
#pragma unroll 1
            for (uint32_t k = 0; k < nwt; ++k) {
                const uint64_t P = run_start + (uint64_t)k * kWTR;
                const uint32_t rel0 = k * kWTR + lane * 64;  // position in run of this lane's first window
                // ---- window: lane l's window [P + 64l, +n) from (A0, B0) and the rows before l
                uint32_t am, bm;
                {
                    uint32_t so = 0, vo = 0, si_ = 0, vi = 0;
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        so = udot4(xo[i], 0x01010101u, so);
                        vo = udot4(xo[i], offw(i), vo);
                        si_ = udot4(xi[i], 0x01010101u, si_);
                        vi = udot4(xi[i], offw(i), vi);
                    }
                    uint32_t tot;
                    const uint32_t Ox = wave_scan_excl(so, tot), Ix = wave_scan_excl(si_, tot);
                    const uint32_t ROx = wave_scan_excl(lane * so, tot), RIx = wave_scan_excl(lane * si_, tot);
                    const uint32_t VOx = wave_scan_excl(vo, tot), VIx = wave_scan_excl(vi, tot);
                    const uint64_t d = 64ull * lane;
                    // sum_{j<d} (d - j) x_j over a row stream = 64 (l X - R) - V (every term >= 0)
                    const uint64_t pin = 64ull * ((uint64_t)lane * Ix - RIx) - VIx;
                    const uint64_t pout = 64ull * ((uint64_t)lane * Ox - ROx) - VOx;
                    am = (uint32_t)(((uint64_t)A0 + Ix + 16ull * kMod - Ox) % kMod);
                    const uint64_t bpos = (uint64_t)B0 + d * (A0 + kMod - 1) + pin;
                    const uint64_t bneg = (pout + (uint64_t)a.nm * Ox) % kMod;
                    bm = (uint32_t)((bpos % kMod + kMod - bneg) % kMod);
                }
                auto compute = [&](const int g, L1Batch& Bt) {
                    const uint32_t xo0 = xo[g >> 2], xo1 = xo[(g >> 2) + 1];
                    const uint32_t xi0 = xi[g >> 2], xi1 = xi[(g >> 2) + 1];
                    uint32_t ct[kB3], rr[kB3], w1[kB3], w1b[kB3], bo[kB3];
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) ct[t2] = ntab[((t2 < 4 ? xo0 : xo1) >> (8 * (t2 & 3))) & 0xFF];
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) {
                        const uint32_t out = ((t2 < 4 ? xo0 : xo1) >> (8 * (t2 & 3))) & 0xFF;
                        const uint32_t in = ((t2 < 4 ? xi0 : xi1) >> (8 * (t2 & 3))) & 0xFF;
                        __builtin_assume(am < kMod);
                        __builtin_assume(bm < kMod);
                        Bt.wv[t2] = (bm << 16) | am;
                        const ProbeHash h = probe_hash(am, bm);
                        Bt.hq[t2] = h.q;
                        rr[t2] = h.r;
                        if (kSmall) {
                            Bt.w2[t2] = fslot[h.r >> fwshift];  // the file's whole filter, tested in finish
                        } else if (kRib) {
                            bo[t2] = rib_bit(h.q, h.r);
                            w1[t2] = l1[bo[t2] >> 5];
                            w1b[t2] = l1[(bo[t2] >> 5) + 1];
                        } else {
                            w1[t2] = l1[l1r_word(h.q)];
                        }
                        const uint32_t u = am + in + (kMod - out);  // [M-255, 2M+255)
                        am = min(u, min(u - kMod, u - 2 * kMod));
                        const uint32_t v = bm + am + ct[t2];          // [0, 3M)
                        bm = min(v, min(v - kMod, v - 2 * kMod));
                    }
#pragma unroll
                    for (int t2 = 0; t2 < kB3 && !kSmall; ++t2) {
                        uint32_t p1;
                        if (kRib) {
                            const uint32_t win = __builtin_amdgcn_alignbit(w1b[t2], w1[t2], bo[t2]);
                            p1 = ~__builtin_popcount(win & rib_coef(Bt.hq[t2], rr[t2])) & 1u;
                        } else {
                            p1 = l1_test(w1[t2], Bt.hq[t2]);
                        }
                        Bt.w2[t2] = __builtin_amdgcn_raw_buffer_load_b32(frsrc, (int)(((rr[t2] >> fwshift) << 2) | (p1 - 1u)),
                                                                         0, 0);
                    }
                };
                auto finish = [&](const int g, L1Batch& Bt) {
                    uint32_t pbits = 0;
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) pbits |= filt_bit(Bt.w2[t2], Bt.hq[t2]) << t2;
                    asm volatile("" : "+v"(pbits));
                    if (!__ballot(pbits != 0)) return;
#pragma unroll
                    for (int t2 = 0; t2 < kB3; ++t2) {
                        const uint64_t mk = __ballot((pbits >> t2) & 1);
                        if (!mk) continue;
                        if ((pbits >> t2) & 1) rec[nrec + __popcll(mk & below)] = make_uint2(rel0 + g + t2, Bt.wv[t2]);
                        nrec += __popcll(mk);
                    }
                };
                const uint32_t tile_rec = nrec;
                L1Batch b0, b1;
                compute(0, b0);
                compute(8, b1);
#pragma unroll
                for (int bi = 0; bi < kNBR; ++bi) {
                    L1Batch& Bt = (bi & 1) ? b1 : b0;
                    finish(kB3 * bi, Bt);
                    if (bi + 2 < kNBR) compute(kB3 * (bi + 2), Bt);
                    if (bi == 2 && k + 1 < nwt) {
                        load_chunk_nt(sc.base, seg_len, P + kWTR + 64ull * lane, no_);
                        load64_u(sc.base, seg_len, P + kWTR + n + 64ull * lane, ni_);
                    }
                }
                // the next tile's first window: lane 63's after its 64 rolls
                A0 = __builtin_amdgcn_readlane(am, 63);
                B0 = __builtin_amdgcn_readlane(bm, 63);
                passes += nrec - tile_rec;
                if (nrec > tile_rec) {
                    if (kSmall) drain_gs(a, rec + tile_rec, nrec - tile_rec, weak_hits, run_start, sc, wo);
                    else drain_g(a, rec + tile_rec, nrec - tile_rec, weak_hits, run_start, sc, wo);
                }
                nrec = tile_rec;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    xo[i] = no_[i];
                    xi[i] = ni_[i];
                }
            }
        }
    }
    flush_defs(a, wo);  // may stage hits (verified past the list's capacity)
    flush_hits(a, wo);
    if (lane == 0 && passes) atomicAdd(&a.counters[2], passes);
    if (lane == 0 && weak_hits) atomicAdd(&a.counters[1], weak_hits);
}

// ===========================================================================
// Deferred verification of weak hits (k_scan_g)
// ===========================================================================
// The deferred weak hits of a k_scan_g launch (counters[10] of them, at most wdef_cap):
// XXH3 of each window (four windows per wave, one per 16-lane row, when n % 64 == 0;
// else one per wave), then the first candidate in index order with equal strong
// (generator.rs:127-133); verified hits to the output like verify_l1.
__global__ __launch_bounds__(256) void k_verify_w(ScanArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t row = lane >> 4, rl = lane & 15;
    const uint64_t total = min((uint64_t)a.counters[10], a.wdef_cap);
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    WaveOut wo = wave_out(a, wave);
    const bool rows = a.n % 64 == 0 && a.n >= 256;  // row_hash: the long path, whole stripes
    const uint32_t per = rows ? 4u : 1u;
    for (uint64_t r0 = wave * per; r0 < total; r0 += nwaves * per) {  // wave-uniform
        const uint64_t ri = rows ? r0 + row : r0;
        const bool live = ri < total;
        const WDef d = a.wdef[live ? ri : r0];
        uint32_t wk;
        uint64_t st;
        uint32_t best = kNoBlock;
        if (rows) {
            row_hash<false>(a.src + d.at, a.n, wk, st);  // valid in the row's first lane
            st = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(st >> 32), (int)(lane & 48)) << 32) |
                 (uint32_t)__shfl((int)(uint32_t)st, (int)(lane & 48));
            if (!(d.cand & kMulti)) {
                if (st == d.strong) best = d.cand;
            } else {
                const uint32_t s0 = a.start[d.cand & ~kMulti], cn = a.cnt[d.cand & ~kMulti];
                for (uint32_t b = 0; b < cn; b += 16) {  // in index order, 16 candidates per step
                    const uint32_t j = b + rl;
                    const uint64_t m = (__ballot(j < cn && a.cstrong[s0 + j] == st) >> (row << 4)) & 0xFFFFull;
                    if (m) {
                        best = a.order[s0 + b + (uint32_t)__builtin_ctzll(m)];
                        break;
                    }
                }
            }
        } else {
            if (a.n > 240) {
                wave_hash_long(a.src + d.at, a.n, wk, st);
            } else {  // XXH3's short paths (k_scan_g takes any window)
                st = 0;
                if (lane == 0) st = xxh3_short(a.src + d.at, a.n);
                st = shfl64(st, 0);
            }
            if (!(d.cand & kMulti)) {
                if (st == d.strong) best = d.cand;
            } else {
                best = first_strong_match(a.order, a.cstrong, a.start[d.cand & ~kMulti], a.cnt[d.cand & ~kMulti], st);
            }
        }
        stage_hits(a, wo, live && (rows ? rl == 0 : lane == 0) && best != kNoBlock, d.key, best);
    }
    flush_hits(a, wo);
}

// Tail rule (generator.rs:156-184): at p* = len - last_size (last_size < n), the
// suffix matches the last basis block iff weak and strong are equal.  One wave per
// job (file).
__global__ void k_tail(const uint8_t* __restrict__ buf, const TailJob* __restrict__ jobs, uint32_t njobs,
                       const uint32_t* __restrict__ weak, const uint64_t* __restrict__ strong, int* __restrict__ flag) {
    const uint32_t j = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (j >= njobs) return;
    const TailJob J = jobs[j];
    const uint8_t* p = buf + J.src;
    uint32_t wk;
    uint64_t st;
    if (J.last_size > 240) {
        wave_hash_long(p, J.last_size, wk, st);
    } else {
        wk = 0; st = 0;
        if ((threadIdx.x & 63) == 0) { wk = adler_scalar(p, J.last_size); st = xxh3_short(p, J.last_size); }
    }
    if ((threadIdx.x & 63) == 0) flag[j] = (wk == weak[J.blk] && st == strong[J.blk]) ? 1 : 0;
}

// ===========================================================================
// K5b: the greedy walk resolved on the device (sydelta_chain.hpp)
// ===========================================================================
// One thread per block / hit / forest node; the bodies live in sydelta_chain.hpp so the
// host emulation of the device layer runs the same code.  Every kernel is a plain
// gather/scatter over arrays of a few MiB (HBM- and launch-bound).
__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }

__global__ __launch_bounds__(256) void k_chain_flag(chain::ChainArgs a) {
    const uint64_t i = gtid();
    if (i <= a.nblk) chain::chain_flag(a, i);
}
__global__ __launch_bounds__(256) void k_chain_place_aligned(chain::ChainArgs a) {
    const uint64_t i = gtid();
    if (i < a.nblk) chain::chain_place_aligned(a, i);
}
__global__ __launch_bounds__(256) void k_chain_place_scan(chain::ChainArgs a) {
    const uint64_t i = gtid();
    if (i < a.H) chain::chain_place_scan(a, i);
}
__global__ __launch_bounds__(256) void k_chain_succ(chain::ChainArgs a) {
    const uint64_t i = gtid();
    if (i < a.M + 2) chain::chain_succ(a, i);
}
__global__ __launch_bounds__(256) void k_chain_lift(chain::ChainArgs a, uint32_t l) {
    const uint64_t i = gtid();
    if (i < a.M + 2) chain::chain_lift(a, l, i);
}
__global__ void k_chain_entry(chain::ChainArgs a) {
    if (gtid() == 0) chain::chain_entry(a);
}
__global__ __launch_bounds__(256) void k_chain_mark(chain::ChainArgs a, uint32_t l) {
    const uint64_t i = gtid();
    if (i < a.M + 2) chain::chain_mark(a, l, i);
}
__global__ __launch_bounds__(256) void k_chain_count(chain::ChainArgs a) {
    const uint64_t i = gtid();
    if (i < a.M + 1) chain::chain_count(a, i);
}
// The ops of the marked hits; per wave one atomic for the Data-op count and bytes.
__global__ __launch_bounds__(256) void k_chain_emit(chain::ChainArgs a) {
    const uint64_t i = gtid();
    const uint64_t lit = i < a.M ? chain::chain_emit(a, i) : 0;
    const uint64_t nd = wave_sum64(lit ? 1ull : 0ull);
    const uint64_t nb = wave_sum64(lit);
    if ((threadIdx.x & 63) == 0 && nd) {
        atomicAdd((unsigned long long*)&a.res->data_ops, (unsigned long long)nd);
        atomicAdd((unsigned long long*)&a.res->lit_bytes, (unsigned long long)nb);
    }
}
__global__ void k_chain_finish(chain::ChainArgs a) {
    if (gtid() == 0) chain::chain_finish(a);
}

// ===========================================================================
// K7z: zstd frame of a text in HBM (sydelta_zstd.hpp; ssh.rs:1009-1017)
// ===========================================================================
// One workgroup per 128 KiB block.  Entropy-only content: a byte histogram (per-wave LDS
// sub-histograms), the Huffman code by one thread (huf_build, scratch in LDS), then per
// literal stream a parallel bit scatter: thread t encodes a contiguous run of the
// stream's symbols, its first bit at the sum of the later runs' bits (the stream is
// written last symbol first), OR-ing whole 32-bit words into an LDS stream buffer; the
// stream leaves for the block's slot with its closing 1 bit.  Literals + sequences: the
// '{' distances, the sampled repeat distances and every position's best candidate match in
// parallel, then (when enough
// positions match) one thread parses, codes the literals and FSE-codes the sequences with
// the shared sequential functions (tables from the block's counts, in HBM scratch); the
// smaller content stays in the slot.  k_zstd_frame
// then lays the blocks out behind their headers.
constexpr int kZT = 256;

// SYDELTA_PHASE_TIMING: k_zstd_block's thread 0 adds its phases' wall-clock ticks (100 MHz)
// here: histogram + code, entropy-only streams, candidate distances, candidate matches,
// hash rounds, literals + sequences content, the rest; inside the content: the segment
// walks, the chaining, the gather, the repeat history, the literals section, the
// sequences section.
__device__ unsigned long long g_zstd_phase[16];
__device__ __forceinline__ void z_phase(uint32_t timing, uint64_t& tph, int k) {
    if (timing && threadIdx.x == 0) {
        const uint64_t t = wall_clock64();
        atomicAdd(&g_zstd_phase[k], (unsigned long long)(t - tph));
        tph = t;
    }
}
constexpr uint32_t kZRun = 144;  // bytes of a stream per thread: 256 runs cover 32 KiB + the 16-byte phase
static_assert(kZRun * kZT >= zstd::kBlockMax / 4 + 16, "one run per thread covers a stream");
// The LDS words: the hash rounds' table, then the parse's path bitmap (the literal streams
// are scattered into the block's global scratch, so the workgroup fits 40 KB of LDS).
constexpr uint32_t kZWords = (1u << zstd::kHashBits) > zstd::kBlockMax / 32 ? (1u << zstd::kHashBits) : zstd::kBlockMax / 32;
static_assert((zstd::kStreamBytesMax + 3) / 4 + 2 <= zstd::kStreamBytesMax, "a stream's words fit sc.streams (4 x kStreamBytesMax bytes)");

struct ZLds {
    // The words (hash table, path bitmap) share their space with what is dead whenever
    // they are live: the histograms and the Huffman build's work area, the sequences' FSE
    // tables (built after the literals section is out).  ~38 KB in all: four workgroups
    // per CU.
    union {
        uint32_t words[kZWords];
        struct {
            uint32_t hist[4][256];
            zstd::HufWork work;
        };
        struct {
            zstd::FseCT fse[3];  // the sequences' FSE tables (the coder's state lookups stay in LDS)
            zstd::FseWork fw;    // and their build's work arrays
        };
    };
    uint32_t part[kZT];
    zstd::HufCode code;
    uint32_t gaps[256];
    uint32_t reps[256];
    uint32_t cand[zstd::kCands];
    uint32_t ssize[4];
    uint32_t state[8];  // [0] type, [1] write offset, [2] abort, [3] entropy-only size, [4] nc, [5] nbest, [6] lz size
    uint32_t pstate[12];    // [2] literals section size, [3] raw, [4] write offset,
                            // [5] sequences header size, [8..10] the final FSE states (OF, ML, LL)
    uint32_t ccnt[36 + 53 + 32];  // the sequences' LL / ML / OF code counts
};
static_assert(sizeof(ZLds) <= 160 * 1024 / 4, "k_zstd_block's static LDS: four workgroups per CU");

typedef __attribute__((address_space(3))) uint8_t lds_u8;  // an LDS pointer kept as one

// Whether a word holds a '{' byte (exact: the zero-byte test of w ^ '{'s).
__device__ __forceinline__ bool z_has_brace(uint32_t w) {
    const uint32_t x = w ^ 0x7B7B7B7Bu;
    return ((x - 0x01010101u) & ~x & 0x80808080u) != 0;
}
// zstd::gap_count from the text in global memory (L1/L2: the 255 bytes behind p), four
// bytes a load; the first 259 positions byte by byte.
__device__ __forceinline__ void z_gap_count(const uint8_t* __restrict__ in, uint32_t p, uint32_t* gaps) {
    if (p < 259) {
        zstd::gap_count(in, p, gaps);
        return;
    }
    uint32_t seen = 0;
    for (uint32_t d0 = 1; d0 < 256 && seen < 3; d0 += 4) {
        const uint32_t w = zstd::ld32u(in + p - d0 - 3);  // byte 3 is at p - d0
        if (!z_has_brace(w)) continue;
        for (int k = 3; k >= 0; --k) {
            const uint32_t d = d0 + 3 - (uint32_t)k;
            if (d < 256 && seen < 3 && ((w >> (8 * k)) & 0xFF) == '{') {
                atomicAdd(&gaps[d], 1u);
                ++seen;
            }
        }
    }
}
// zstd::repeat_dist from the text in global memory.  p is a multiple of 4 (kRepStep), so
// the 32 distances of a chunk, D0 .. D0 + 31, start at bytes A + 3 .. A + 34 with A =
// p - D0 - 34 4-byte aligned: ten aligned loads and byte shifts by constants.
static_assert(zstd::kRepStep % 4 == 0, "repeat samples at 4-byte aligned positions");
__device__ __forceinline__ uint32_t z_repeat_dist(const uint8_t* __restrict__ in, uint32_t n, uint32_t p) {
    if (p < 260) return zstd::repeat_dist(in, n, p);
    if (p + 4 > n) return 0;
    const uint32_t v = *(const uint32_t*)(in + p);
    if (in[p - 1] == (v & 0xFF) && v == (v & 0xFF) * 0x01010101u) return 0;  // the 4 bytes continue a run
    for (uint32_t D0 = 2; D0 < 256; D0 += 32) {
        const uint32_t* A = (const uint32_t*)(in + (p - D0 - 34));  // the text is 16-byte aligned
        uint32_t w[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) w[i] = A[i];
        uint32_t hit = 0;
#pragma unroll
        for (uint32_t t = 0; t < 32; ++t) {  // start A + 3 + t is distance D0 + 31 - t
            const uint32_t o = 3 + t;
            const uint32_t x = (o & 3) ? __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], o & 3) : w[o >> 2];
            hit |= (uint32_t)(x == v) << (31 - t);
        }
        if (D0 + 31 > 255) hit &= (1u << (256 - D0)) - 1u;  // distances <= 255
        if (hit) return D0 + (uint32_t)__builtin_ctz(hit);
    }
    return 0;
}

// Block-wide: the sum of v over the threads after this one (returned) and over all of
// them (*total), by a wave suffix scan and the four wave sums in L.part[0..4).  Starts and
// ends with a barrier.
__device__ __forceinline__ uint32_t z_suffix(ZLds& L, uint32_t v, uint32_t& total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_down(x, o);
        if (lane + o < 64) x += y;
    }
    __syncthreads();
    if (lane == 0) L.part[wid] = x;
    __syncthreads();
    uint32_t later = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kZT / 64; ++w) {
        const uint32_t t = L.part[w];
        all += t;
        later += w > wid ? t : 0u;
    }
    total = all;
    __syncthreads();
    return later + x - v;
}

// Bits of symbols src[first, first + count) coded with L.code, written as one literal
// stream (last symbol first, LSB-first) into gw (global, the block's scratch) with its
// closing 1 bit by a parallel bit scatter: thread t encodes the run [A + kZRun t, +kZRun)
// (A = first rounded down to 16; src 16-byte aligned and readable to the end of its last
// granule), its first bit at the sum of the later runs' bits; the words wholly inside
// its bits are stored, the two it may share ORed.  Returns the stream's bits without the
// closing bit (every thread).
__device__ __forceinline__ uint32_t z_stream_scatter(ZLds& L, const uint8_t* __restrict__ src, uint32_t first,
                                                     uint32_t count, uint32_t* __restrict__ gw) {
    const uint32_t tid = threadIdx.x;
    const uint32_t nw = (count * zstd::kMaxBits + 1 + 31) / 32 + 1;
    for (uint32_t i = tid; i < nw; i += kZT) gw[i] = 0;
    const uint32_t A = first & ~15u, r0 = A + kZRun * tid, lim = first + count;
    // one 16-byte granule at a time (the run held whole in registers, fully unrolled, took
    // ~250 VGPRs: one workgroup per CU); the second pass reads the granules again (L1/L2)
    auto granule = [&](uint32_t j) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (r0 + 16 * j < lim) v = *(const uint4*)(src + r0 + 16 * j);
        return v;
    };
    uint32_t bits = 0;
#pragma unroll 1
    for (uint32_t j = 0; j < kZRun / 16; ++j) {
        const uint4 v = granule(j);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t p = r0 + 16 * j + k;
            if (p >= first && p < lim) bits += L.code.len[(w4[k >> 2] >> (8 * (k & 3))) & 0xFF];
        }
    }
    uint32_t total;
    const uint32_t off = z_suffix(L, bits, total);
    uint32_t word = off >> 5, fill = off & 31;
    uint64_t acc = 0;
    bool lead = true;
#pragma unroll 1
    for (uint32_t j = kZRun / 16; j-- > 0;) {
        const uint4 v = granule(j);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t kk = 16; kk-- > 0;) {
            const uint32_t p = r0 + 16 * j + kk;
            if (p >= first && p < lim) {
                const uint32_t sym = (w4[kk >> 2] >> (8 * (kk & 3))) & 0xFF;
                acc |= (uint64_t)L.code.code[sym] << fill;
                fill += L.code.len[sym];
                if (fill >= 32) {
                    if (lead) atomicOr(&gw[word], (uint32_t)acc);
                    else gw[word] = (uint32_t)acc;
                    lead = false;
                    acc >>= 32;
                    fill -= 32;
                    ++word;
                }
            }
        }
    }
    if (fill) atomicOr(&gw[word], (uint32_t)acc);
    __threadfence_block();
    __syncthreads();
    if (tid == 0) atomicOr(&gw[total >> 5], 1u << (total & 31));  // the closing bit
    __threadfence_block();
    __syncthreads();
    return total;
}

// The literals section of lit[0, nl) into out (global), as zstd::lit_section_seq writes
// it: Huffman-coded with the streams scattered in parallel (z_stream_scatter), or Raw
// when that is impossible or not smaller.  Returns its size (every thread).
__device__ __forceinline__ uint32_t z_lit_section(ZLds& L, const uint8_t* __restrict__ lit, uint32_t nl, uint8_t* __restrict__ out,
                                                  uint32_t* __restrict__ gw) {
    const uint32_t tid = threadIdx.x, wid = tid >> 6;
    for (uint32_t i = tid; i < 4 * 256; i += kZT) (&L.hist[0][0])[i] = 0;
    __syncthreads();
    for (uint32_t c = tid; 16 * c < nl; c += kZT) {
        const uint4 v = *(const uint4*)(lit + 16 * c);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (16 * c + k < nl) atomicAdd(&L.hist[wid][(w4[k >> 2] >> (8 * (k & 3))) & 0xFF], 1u);
    }
    __syncthreads();
    for (uint32_t sy = tid; sy < 256; sy += kZT) L.hist[0][sy] += L.hist[1][sy] + L.hist[2][sy] + L.hist[3][sy];
    __syncthreads();
    const bool four = nl > zstd::kSingleStreamMax;
    const uint32_t hs = four ? 5u : 3u;
    const uint32_t raw_size = nl + (nl < 32 ? 1u : nl < 4096 ? 2u : 3u);
    if (tid == 0) {
        uint32_t distinct = 0, hi = 0;
        for (uint32_t sy = 0; sy < 256; ++sy)
            if (L.hist[0][sy]) { ++distinct; hi = sy; }
        L.pstate[3] = (distinct < 2 || hi >= zstd::kSymbols) ? 1u : 0u;
        if (!L.pstate[3]) {
            zstd::huf_build(L.hist[0], L.code, L.work);
            const uint32_t tsz = zstd::huf_tree_desc(L.code, out + hs);
            L.pstate[4] = hs + tsz + (four ? 6u : 0u);
        }
    }
    __syncthreads();
    if (!L.pstate[3]) {
        for (uint32_t st = 0; st < (four ? 4u : 1u); ++st) {
            uint32_t first, count;
            zstd::stream_range(nl, four, st, first, count);
            const uint32_t total = z_stream_scatter(L, lit, first, count, gw);
            const uint32_t bytes = total / 8 + 1;
            const uint32_t o = L.pstate[4];
            if (o + bytes >= raw_size || (!four && o + bytes - hs > zstd::kSingleStreamMax)) {
                __syncthreads();
                if (tid == 0) L.pstate[3] = 1;
                __syncthreads();
                break;
            }
            const uint8_t* wb = (const uint8_t*)gw;
            for (uint32_t i = tid; i < bytes; i += kZT) out[o + i] = wb[i];
            __syncthreads();
            if (tid == 0) {
                L.ssize[st] = bytes;
                L.pstate[4] = o + bytes;
            }
            __syncthreads();
        }
    }
    if (L.pstate[3]) {  // Raw literals
        const uint32_t rh = nl < 32 ? 1u : nl < 4096 ? 2u : 3u;
        if (tid == 0) zstd::raw_lit_header(out, nl);
        for (uint32_t i = tid; i < nl; i += kZT) out[rh + i] = lit[i];
        __syncthreads();
        return rh + nl;
    }
    const uint32_t o = L.pstate[4];
    if (tid == 0) {
        zstd::lit_header(out, four, nl, o - hs);
        if (four) {
            const uint32_t tsz = 1 + (L.code.last + 1) / 2;
            for (uint32_t k = 0; k < 3; ++k) {
                out[hs + tsz + 2 * k] = (uint8_t)L.ssize[k];
                out[hs + tsz + 2 * k + 1] = (uint8_t)(L.ssize[k] >> 8);
            }
        }
    }
    __syncthreads();
    return o;
}

// The sequences' bitstream of zstd::seq_section_counted (after its header), in parallel:
// (1) every sequence's codes; (2) the three FSE state chains (OF, ML, LL: lanes 0-2 of
// wave 0 in lockstep, one sequence per step, last to first, the codes read 64 at a time),
// each step's state bits recorded; (3) every sequence's bit count and, by a block-wide
// suffix sum (the stream holds the last sequence first), its offset; (4) the fields ORed
// into a zeroed word buffer (sc.streams), the final states and the closing bit after
// them; (5) the bytes copied out.  Byte-identical to the sequential writer (BitW: bits
// LSB-first from byte 0).  Returns the stream's bytes (every thread).
__device__ __forceinline__ uint32_t z_seq_bits(ZLds& L, const zstd::SeqScratch& sc, uint32_t ns, uint8_t* __restrict__ out) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (!ns) return 0;  // uniform
    uint32_t* cw = sc.best;                // packed codes: lc | mc << 6 | oc << 12 | lb << 17 | mb << 22
    uint32_t* rec = sc.best + ns;          // 3 x ns state records: nbo << 16 | bits (OF, ML, LL)
    uint32_t* wb = (uint32_t*)sc.streams;  // the bit buffer
    for (uint32_t k = tid; k < ns; k += kZT) {
        uint32_t lc, lb, mc, mb, oc, ov;
        zstd::seq_codes(sc.seq[k], lc, lb, mc, mb, oc, ov);
        cw[k] = lc | (mc << 6) | (oc << 12) | (lb << 17) | (mb << 22);
    }
    __threadfence_block();
    __syncthreads();
    if (tid < 64) {
        const zstd::FseCT& T = lane == 0 ? L.fse[2] : lane == 1 ? L.fse[1] : L.fse[0];  // OF, ML, LL
        auto code_of = [&](uint32_t w) { return lane == 0 ? (w >> 12) & 31u : lane == 1 ? (w >> 6) & 63u : w & 63u; };
        const bool on = lane < 3 && T.log != 0;
        uint32_t st = 0;
        if (on) st = zstd::fse_init(T, code_of(cw[ns - 1]));
        for (uint32_t hi = ns - 1; hi > 0;) {  // sequences [lo, hi), last first
            const uint32_t lo = hi > 64 ? hi - 64 : 0;
            // each lane looks up its sequence's three code transforms (no dependence on the
            // states): the chains' steps then wait on one LDS read each, the state table's
            int32_t nb3[3] = {0, 0, 0}, fd3[3] = {0, 0, 0};
            if (lo + lane < hi) {
                const uint32_t w = cw[lo + lane];
                const uint32_t c3[3] = {(w >> 12) & 31u, (w >> 6) & 63u, w & 63u};  // OF, ML, LL
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const zstd::FseCT& U = L.fse[2 - t];
                    nb3[t] = U.delta_nb[c3[t]];
                    fd3[t] = U.delta_find[c3[t]];
                }
            }
            for (uint32_t j = hi - lo; j-- > 0;) {
                const int32_t n0 = __builtin_amdgcn_readlane(nb3[0], j), n1 = __builtin_amdgcn_readlane(nb3[1], j);
                const int32_t n2 = __builtin_amdgcn_readlane(nb3[2], j), f0 = __builtin_amdgcn_readlane(fd3[0], j);
                const int32_t f1 = __builtin_amdgcn_readlane(fd3[1], j), f2 = __builtin_amdgcn_readlane(fd3[2], j);
                if (lane < 3) {
                    uint32_t r = 0;
                    if (on) {
                        const int32_t dnb = lane == 0 ? n0 : lane == 1 ? n1 : n2;
                        const int32_t dfd = lane == 0 ? f0 : lane == 1 ? f1 : f2;
                        const uint32_t nbo = (uint32_t)((int32_t)st + dnb) >> 16;
                        r = (nbo << 16) | (st & ((1u << nbo) - 1u));
                        st = T.state[(st >> nbo) + dfd];
                    }
                    rec[lane * ns + lo + j] = r;
                }
            }
            hi = lo;
        }
        if (lane < 3) L.pstate[8 + lane] = st;  // final states: OF, ML, LL
    }
    __threadfence_block();
    __syncthreads();
    // bits per sequence, per thread range [t*per, +per), emitted from the top
    const uint32_t per = (ns + kZT - 1) / kZT;
    const uint32_t k0 = min(ns, tid * per), k1 = min(ns, k0 + per);
    auto bits_of = [&](uint32_t k) -> uint32_t {
        const uint32_t w = cw[k];
        uint32_t b = ((w >> 17) & 31u) + ((w >> 22) & 31u) + ((w >> 12) & 31u);
        if (k + 1 < ns) b += (rec[k] >> 16) + (rec[ns + k] >> 16) + (rec[2 * ns + k] >> 16);
        return b;
    };
    uint32_t mine = 0;
    for (uint32_t k = k0; k < k1; ++k) mine += bits_of(k);
    uint32_t total;
    const uint32_t off = z_suffix(L, mine, total);
    const uint32_t fb = L.fse[1].log + L.fse[2].log + L.fse[0].log;  // final states ML, OF, LL
    const uint32_t nw = (total + fb + 1 + 31) / 32 + 1;
    // <= 57 bits per sequence of >= 6 bytes: ~156 KiB at most; past the buffer the content
    // is reported too large (the block keeps its entropy-only content)
    if (nw > zstd::kStreamBytesMax) return 1u << 30;  // uniform
    for (uint32_t i = tid; i < nw; i += kZT) wb[i] = 0;
    __threadfence_block();
    __syncthreads();
    auto put = [&](uint32_t at, uint32_t v, uint32_t n) {
        if (!n) return;
        const uint64_t x = (uint64_t)(v & (n >= 32 ? 0xFFFFFFFFu : (1u << n) - 1u)) << (at & 31);
        atomicOr(&wb[at >> 5], (uint32_t)x);
        if (x >> 32) atomicOr(&wb[(at >> 5) + 1], (uint32_t)(x >> 32));
    };
    {
        // this thread's bits [off, off + mine) accumulated in a register: the words wholly
        // inside are stored, the two it may share with its neighbours ORed
        uint32_t word = off >> 5, fill = off & 31;
        uint64_t acc = 0;
        bool first = true;
        auto emit = [&](uint32_t v, uint32_t nb) {
            acc |= (uint64_t)(v & ((1u << nb) - 1u)) << fill;  // nb <= 31
            fill += nb;
            if (fill >= 32) {
                if (first) atomicOr(&wb[word], (uint32_t)acc);
                else wb[word] = (uint32_t)acc;
                first = false;
                acc >>= 32;
                fill -= 32;
                ++word;
            }
        };
        for (uint32_t k = k1; k-- > k0;) {
            const uint32_t w = cw[k];
            const zstd::Seq q = sc.seq[k];
            if (k + 1 < ns) {
                const uint32_t ro = rec[k], rm = rec[ns + k], rl = rec[2 * ns + k];
                emit(ro & 0xFFFFu, ro >> 16);
                emit(rm & 0xFFFFu, rm >> 16);
                emit(rl & 0xFFFFu, rl >> 16);
            }
            emit(q.ll, (w >> 17) & 31u);
            emit(q.ml - 3, (w >> 22) & 31u);
            emit(q.ov, (w >> 12) & 31u);
        }
        if (fill) atomicOr(&wb[word], (uint32_t)acc);
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) {  // the final states (ML, OF, LL) and the closing bit
        uint32_t a = total;
        put(a, L.pstate[9], L.fse[1].log); a += L.fse[1].log;
        put(a, L.pstate[8], L.fse[2].log); a += L.fse[2].log;
        put(a, L.pstate[10], L.fse[0].log); a += L.fse[0].log;
        put(a, 1u, 1u);
    }
    __threadfence_block();
    __syncthreads();
    const uint32_t bytes = (total + fb + 1 + 7) / 8;
    const uint8_t* src = (const uint8_t*)wb;
    for (uint32_t i = tid; i < bytes; i += kZT) out[i] = src[i];
    __syncthreads();
    return bytes;
}

// The literals + sequences content of a block (zstd::lz_content's bytes) with the parse in
// parallel.  The parse's path from position 0 is a function of the position alone
// (zstd::parse_take / match_len), so each thread walks its own 512 positions from their
// start, marking the positions it steps on in an LDS bitmap (L.words), and thread 0
// chains the segments: where the true entry of a segment differs from its start, it walks
// from the entry, clearing the speculative marks it jumps over, until it steps on a marked
// position (the two walks agree from there on).  The marked positions are the literals
// and the sequence starts: counted per thread, ranked, gathered (literals into sc.lit,
// starts into sc.seq).  Wave 0 then resolves the repeat history (zstd::seq_dist,
// rep_code) 64 sequences at a time by a wave scan, the literals section follows
// (z_lit_section), then the sequences section: its header by thread 0
// (seq_section_head), its bitstream in parallel (z_seq_bits).  Returns its size, 0 when
// the block has no sequence (every thread).
__device__ __forceinline__ uint32_t z_lz_content(ZLds& L, const uint8_t* __restrict__ in, uint32_t n, const zstd::SeqScratch& sc,
                                 uint32_t timing, uint64_t& tph) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    constexpr uint32_t kSeg = zstd::kBlockMax / kZT;  // 512 positions per thread
    static_assert(kSeg % 32 == 0 && 2 * (zstd::kBlockMax / 32) <= kZWords, "the path and take bitmaps fit the LDS words");
    uint32_t* bm = L.words;                          // the positions the path steps on
    uint32_t* tk = L.words + zstd::kBlockMax / 32;   // zstd::parse_take of every position
    const uint32_t s0 = tid * kSeg, s1 = min(n, s0 + kSeg);
    for (uint32_t w = tid * (kSeg / 32); w < (tid + 1) * (kSeg / 32); ++w) bm[w] = 0;
    {  // the take bitmap, 64 positions per wave step (coalesced bests, one ballot)
        const uint32_t wid = tid >> 6;
        for (uint32_t b = 64 * wid; b < zstd::kBlockMax; b += kZT) {
            const uint32_t q = b + lane;
            const uint32_t cur = q < n ? sc.best[q] : 0u;
            uint32_t nxt = __shfl_down(cur, 1);
            if (lane == 63) nxt = q + 1 < n ? sc.best[q + 1] : 0u;
            const bool take = cur && !(q + 1 < n && (nxt >> 24) > (cur >> 24));  // zstd::parse_take
            const uint64_t m = __ballot(take);
            if (lane == 0) {
                tk[b >> 5] = (uint32_t)m;
                tk[(b >> 5) + 1] = (uint32_t)(m >> 32);
            }
        }
    }
    __syncthreads();
    auto take_at = [&](uint32_t x) { return (tk[x >> 5] >> (x & 31)) & 1u; };
    auto step = [&](uint32_t x) -> uint32_t {
        return take_at(x) ? x + zstd::match_len(in, n, x, sc.best[x]) : x + 1;
    };
    // speculative walk of this thread's segment: a run of literals is skipped to the next
    // take position through the bitmap, marked whole words at a time
    uint32_t p = s0;
    while (p < s1) {
        uint32_t w = p >> 5, t = tk[w] & (~0u << (p & 31));
        while (!t && 32 * (w + 1) < s1) t = tk[++w];
        const uint32_t nt = t ? min(s1, 32 * w + (uint32_t)__builtin_ctz(t)) : s1;  // literals [p, nt)
        for (uint32_t x = p; x < nt;) {
            const uint32_t xe = min(nt, (x | 31) + 1);
            bm[x >> 5] |= (xe - x == 32 ? ~0u : ((1u << (xe - x)) - 1u)) << (x & 31);
            x = xe;
        }
        p = nt;
        if (p >= s1) break;
        bm[p >> 5] |= 1u << (p & 31);
        p += zstd::match_len(in, n, p, sc.best[p]);
    }
    L.part[tid] = s0 < n ? p : s0;  // the segment's exit
    __syncthreads();
    z_phase(timing, tph, 7);
    if (tid == 0) {
        auto bit = [&](uint32_t x) { return (bm[x >> 5] >> (x & 31)) & 1u; };
        auto clear = [&](uint32_t a, uint32_t b) {  // marks in [a, b)
            for (uint32_t x = a; x < b;) {
                if ((x & 31) == 0 && x + 32 <= b) { bm[x >> 5] = 0; x += 32; }
                else { bm[x >> 5] &= ~(1u << (x & 31)); ++x; }
            }
        };
        uint32_t e = L.part[0];
        for (uint32_t t = 1; t < kZT && t * kSeg < n; ++t) {
            const uint32_t a = t * kSeg, b = min(n, a + kSeg);
            if (e == a) { e = L.part[t]; continue; }
            if (e >= b) { clear(a, b); continue; }  // the path jumps over the whole segment
            clear(a, e);
            uint32_t x = e;
            bool met = false;
            while (x < b) {
                if (bit(x)) { met = true; break; }
                bm[x >> 5] |= 1u << (x & 31);
                const uint32_t y = step(x);
                clear(x + 1, min(y, b));
                x = y;
            }
            e = met ? L.part[t] : x;
        }
    }
    __syncthreads();
    z_phase(timing, tph, 8);
    // The marked positions are the path: a mark followed by a mark is a literal, any other
    // mark starts a sequence that runs to the next mark (position n counts as marked; a
    // match is >= kMinMatch bytes).  So the counts are popcounts and a sequence's length
    // is a bitmap search: no reread of the bests or the text.
    auto word = [&](uint32_t w) -> uint32_t {
        return (32 * w < n ? bm[w] : 0u) | ((n >> 5) == w ? 1u << (n & 31) : 0u);
    };
    auto lit_mask = [&](uint32_t w, uint32_t m) {  // literals among the marks m of word w
        return m & ((word(w) >> 1) | (word(w + 1) << 31));
    };
    uint32_t nlit = 0, nseq = 0;
    for (uint32_t w = s0 >> 5; 32 * w < s1; ++w) {
        const uint32_t m = bm[w], lit = lit_mask(w, m);
        nlit += __builtin_popcount(lit);
        nseq += __builtin_popcount(m & ~lit);
    }
    uint32_t nl, ns;  // block totals; a thread's ranks are what the earlier threads hold
    const uint32_t lat = z_suffix(L, nlit, nl), sat = z_suffix(L, nseq, ns);
    const uint32_t lrank = nl - lat - nlit, srank = ns - sat - nseq;
    if (ns == 0) return 0;  // uniform
    // gather: literals into sc.lit (the word's 32 text bytes loaded once), sequence starts
    // into sc.seq as {p, length, -, -}
    {
        uint32_t lr = lrank, sr = srank;
        for (uint32_t w = s0 >> 5; 32 * w < s1; ++w) {
            const uint32_t m = bm[w];
            if (!m) continue;
            const uint32_t lit = lit_mask(w, m);
            uint32_t sq = m & ~lit;
            if (lit) {  // the text is readable to the end of its last 16-byte granule
                const uint4 v0 = *(const uint4*)(in + 32 * w);
                uint4 v1 = make_uint4(0, 0, 0, 0);
                if (32 * w + 16 < n) v1 = *(const uint4*)(in + 32 * w + 16);
                const uint32_t t8[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                for (uint32_t k = 0; k < 32; ++k)
                    if ((lit >> k) & 1u) sc.lit[lr++] = (uint8_t)(t8[k >> 2] >> (8 * (k & 3)));
            }
            while (sq) {
                const uint32_t k = (uint32_t)__builtin_ctz(sq);
                sq &= sq - 1;
                uint32_t nw = w, t = word(w) & ~((2u << k) - 1u);  // marks after x
                while (!t) t = word(++nw);
                sc.seq[sr++] = zstd::Seq{32 * w + k, 32 * nw + (uint32_t)__builtin_ctz(t) - (32 * w + k), 0, 0};
            }
        }
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t k = tid; k < ns; k += kZT) sc.seq[k].off = sc.best[sc.seq[k].ll] & 0xFFFFFFu;  // best distances
    __threadfence_block();
    __syncthreads();
    z_phase(timing, tph, 9);
    // After a sequence the history's rep[0] is the distance it used, which is the best
    // distance of the last sequence that did not take the repeat: one of the few before.
    // So for every k at once: bit b-1 = sequence k also matches (all its l bytes) at the
    // best distance of sequence k - b, b = 1..8; the bytes in sc.streams (free on the
    // device path).
    uint8_t* okp = sc.streams;
    for (uint32_t k = tid; k < ns; k += kZT) {
        uint32_t ok = 0;
        const zstd::Seq q = sc.seq[k];
        const uint32_t x = q.ll, l = q.ml;
        for (uint32_t b = 1; b <= 8 && b <= k; ++b) {
            const uint32_t d = sc.seq[k - b].off;
            if (d > x || d == q.off) continue;  // unused: seq_dist needs rep[0] <= x and != the own best
            ok |= (uint32_t)(zstd::common_len(in, x, x - d, l) >= l) << (b - 1);
        }
        okp[k] = (uint8_t)ok;
    }
    __threadfence_block();
    __syncthreads();
    z_phase(timing, tph, 14);
    // The repeat history (wave 0), 64 sequences at a time.  Sequence k takes the repeat
    // distance when flag j-1 of its record is set, j = k - owner (the last sequence that
    // coded its own best): per lane that is a map of j in {0 (no history), 1..8, 9 (far)},
    // and a wave scan of the maps gives every lane its j.  Without a repeat coded after a
    // zero literal length at the same distance (the one case that puts a value twice in
    // zstd's history), the history entering a sequence is the three latest distinct
    // distances before it (move to front), which each lane finds by walking back over the
    // batch's distances, then the carried history.  A batch with a far j, such a repeat or
    // a carried history holding a value twice runs the sequential loop instead.
    if (tid < 64) {
        uint32_t* dl = L.part;  // the batch's distances (free here)
        uint32_t rp0 = 0, rp1 = 0, rp2 = 0, end = 0, owner = 0;  // the history; rp0 is the best distance of sequence `owner`
        uint32_t prev_off = 0;                                    // the previous batch's best distances
        for (uint32_t k0 = 0; k0 < ns; k0 += 64) {
            const uint32_t m = min(64u, ns - k0);
            zstd::Seq q{0, 0, 0, 0};
            uint32_t ok = 0;
            if (lane < m) {
                q = sc.seq[k0 + lane];
                ok = okp[k0 + lane];
            }
            // literal lengths in parallel: a sequence's start less the previous one's end
            const uint32_t pend = __shfl_up(q.ll + q.ml, 1);
            const uint32_t llv = q.ll - (lane ? pend : end);
            end = __builtin_amdgcn_readlane(q.ll + q.ml, m - 1);
            // (1) j per lane: maps of 10 states x 4 bits, composed by a wave scan
            const uint32_t jin = k0 == 0 ? 0u : min(k0 - owner, 9u);
            uint64_t f = 0x9876543210ull;  // identity (lanes past m)
            if (lane < m) {
                f = 0x9ull << 36 | 1ull;  // j = 9 stays far, j = 0 -> 1
#pragma unroll
                for (uint32_t j = 1; j <= 8; ++j) f |= (uint64_t)(((ok >> (j - 1)) & 1u) ? j + 1 : 1u) << (4 * j);
            }
            auto compose = [](uint64_t P, uint64_t Q) {  // P after Q
                uint64_t r = 0;
#pragma unroll
                for (uint32_t j = 0; j < 10; ++j) r |= ((P >> (4 * ((Q >> (4 * j)) & 15))) & 15) << (4 * j);
                return r;
            };
#pragma unroll
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint64_t Q = __shfl_up(f, o);
                if (lane >= o) f = compose(f, Q);
            }
            const uint64_t E = __shfl_up(f, 1);
            const uint32_t js = lane ? (uint32_t)(E >> (4 * jin)) & 15u : jin;
            const bool take = js >= 1 && js <= 8 && ((ok >> (js - 1)) & 1u);
            const uint32_t a0 = __shfl(q.off, (lane - js) & 63), a1 = __shfl(prev_off, (lane - js) & 63);
            const uint32_t dv = take ? (lane >= js ? a0 : a1) : q.off;
            // (2) the history entering each lane
            dl[lane] = dv;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t h0 = 0, h1 = 0, h2 = 0, nf = 0;
            auto add = [&](uint32_t v) {
                if (!v || nf >= 3 || v == h0 || v == h1) return;
                if (nf == 0) h0 = v; else if (nf == 1) h1 = v; else h2 = v;
                ++nf;
            };
            for (uint32_t o = 1; o <= 64; ++o) {
                const bool need = lane < m && nf < 3 && o <= lane;
                if (!__ballot(need)) break;
                if (need) add(dl[lane - o]);
            }
            add(rp0);
            add(rp1);
            add(rp2);
            const bool carried_ok = !(rp0 && (rp0 == rp1 || rp0 == rp2)) && !(rp1 && rp1 == rp2);
            const bool bad = lane < m && (js == 9 || (llv == 0 && dv == h0 && h0 != 0));
            if (carried_ok && !__ballot(bad)) {
                uint32_t t0 = h0, t1 = h1, t2 = h2;
                const uint32_t ov = zstd::rep_code3(t0, t1, t2, llv, dv);
                if (lane < m) sc.seq[k0 + lane] = zstd::Seq{llv, q.ml, dv, ov};
                rp0 = __builtin_amdgcn_readlane(t0, m - 1);
                rp1 = __builtin_amdgcn_readlane(t1, m - 1);
                rp2 = __builtin_amdgcn_readlane(t2, m - 1);
                const uint32_t jl = __builtin_amdgcn_readlane(js, m - 1);
                const bool tl = __builtin_amdgcn_readlane((uint32_t)take, m - 1) != 0;
                owner = k0 + m - (tl ? jl + 1 : 1u);
            } else {  // the sequential form of the batch
                uint32_t rd = 0, rov = 0;
                for (uint32_t j = 0; j < m; ++j) {
                    const uint32_t d0 = __builtin_amdgcn_readlane(q.off, j), okj = __builtin_amdgcn_readlane(ok, j);
                    const uint32_t ll = __builtin_amdgcn_readlane(llv, j);
                    uint32_t d = d0;
                    const uint32_t k = k0 + j;
                    if (rp0 && rp0 != d0) {  // zstd::seq_dist
                        bool good;
                        if (k - owner <= 8) {  // the flags hold rp0 <= x too
                            good = (okj >> (k - owner - 1)) & 1u;
                        } else {
                            const uint32_t x = __builtin_amdgcn_readlane(q.ll, j), l = __builtin_amdgcn_readlane(q.ml, j);
                            bool bd = rp0 > x;
                            if (!bd)
                                for (uint32_t i = lane; i < l; i += 64) bd |= in[x + i] != in[x + i - rp0];
                            good = !__ballot(bd);
                        }
                        if (good) d = rp0;
                    }
                    const uint32_t ov = zstd::rep_code3(rp0, rp1, rp2, ll, d);
                    if (lane == j) { rd = d; rov = ov; }
                    if (d == d0) owner = k;
                }
                if (lane < m) sc.seq[k0 + lane] = zstd::Seq{llv, q.ml, rd, rov};
            }
            prev_off = q.off;
            __builtin_amdgcn_wave_barrier();  // dl is rewritten by the next batch
        }
    }
    __threadfence_block();
    __syncthreads();
    z_phase(timing, tph, 10);
    // code counts in parallel (LDS atomics)
    for (uint32_t i = tid; i < 36 + 53 + 32; i += kZT) L.ccnt[i] = 0;
    __syncthreads();
    for (uint32_t k = tid; k < ns; k += kZT) {
        uint32_t lc, lb, mc, mb, oc, ov;
        zstd::seq_codes(sc.seq[k], lc, lb, mc, mb, oc, ov);
        atomicAdd(&L.ccnt[lc], 1u);
        atomicAdd(&L.ccnt[36 + mc], 1u);
        atomicAdd(&L.ccnt[36 + 53 + oc], 1u);
    }
    const uint32_t z = z_lit_section(L, sc.lit, nl, sc.body, (uint32_t*)sc.streams);  // starts with a barrier
    z_phase(timing, tph, 11);
    uint8_t* sp = sc.body + z;
    if (tid == 0)
        L.pstate[5] = zstd::seq_section_head(ns, sp, L.ccnt, L.ccnt + 36, L.ccnt + 36 + 53, L.fse[0], L.fse[1], L.fse[2],
                                               L.fw);
    __syncthreads();
    z_phase(timing, tph, 13);
    if (timing && tid == 0) atomicAdd(&g_zstd_phase[15], (unsigned long long)ns);
    const uint32_t ho = L.pstate[5];
    const uint32_t nb = z_seq_bits(L, sc, ns, sp + ho);
    z_phase(timing, tph, 12);
    return z + ho + nb;
}


__global__ __launch_bounds__(kZT) void k_zstd_block(const uint8_t* __restrict__ text, uint64_t len, uint64_t b0,
                                                    uint8_t* __restrict__ slots, uint8_t* __restrict__ lz, uint64_t nlz,
                                                    uint32_t* __restrict__ size_out, uint32_t* __restrict__ type_out,
                                                    uint64_t* __restrict__ len64, uint32_t timing) {
    __shared__ ZLds L;
    uint64_t tph = timing ? wall_clock64() : 0;
    auto phase = [&](int k) { z_phase(timing, tph, k); };
    const uint32_t tid = threadIdx.x, wid = tid >> 6;
    const uint64_t gb = b0 + blockIdx.x;
    const uint8_t* in = text + gb * zstd::kBlockMax;
    const uint32_t n = (uint32_t)min<uint64_t>(zstd::kBlockMax, len - gb * zstd::kBlockMax);
    uint8_t* slot = slots + (uint64_t)blockIdx.x * zstd::kBlockMax;
    const zstd::SeqScratch sc = zstd::seq_scratch_at(lz, nlz, blockIdx.x);
    for (uint32_t i = tid; i < 4 * 256; i += kZT) (&L.hist[0][0])[i] = 0;
    for (uint32_t i = tid; i < 256; i += kZT) {
        L.gaps[i] = 0;
        L.reps[i] = 0;
    }
    if (tid == 0) L.state[5] = 0;
    __syncthreads();
    // histogram, 16 bytes per load (the text is 16-byte aligned and readable to the end
    // of its last granule); bytes past n are not counted
    for (uint32_t c = tid; 16 * c < n; c += kZT) {
        const uint4 v = *(const uint4*)(in + 16 * c);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (16 * c + k < n) atomicAdd(&L.hist[wid][(w4[k >> 2] >> (8 * (k & 3))) & 0xFF], 1u);
    }
    __syncthreads();
    for (uint32_t s = tid; s < 256; s += kZT) L.hist[0][s] += L.hist[1][s] + L.hist[2][s] + L.hist[3][s];
    __syncthreads();
    phase(0);
    const bool four = n > zstd::kSingleStreamMax;
    const uint32_t hs = four ? 5u : 3u;  // literals header
    if (tid == 0) {
        uint32_t distinct = 0, hi = 0;
        for (uint32_t s = 0; s < 256; ++s)
            if (L.hist[0][s]) { ++distinct; hi = s; }
        uint32_t type = 0;  // Raw until a content smaller than n turns up
        if (distinct == 1 && n > 1) type = 1;
        L.state[0] = type;
        L.state[2] = (distinct >= 2 && hi < zstd::kSymbols) ? 0u : 1u;  // entropy-only coding possible?
        L.state[3] = 0xFFFFFFFFu;
        if (!L.state[2] && type == 0) {
            zstd::huf_build(L.hist[0], L.code, L.work);
            const uint32_t tsz = zstd::huf_tree_desc(L.code, slot + hs);
            L.state[1] = hs + tsz + (four ? 6u : 0u);  // the first stream's offset
        }
    }
    __syncthreads();
    const uint32_t rle = L.state[0];
    if (!rle && !L.state[2]) {
        const uint32_t ns = four ? 4u : 1u;
        for (uint32_t st = 0; st < ns; ++st) {
            uint32_t first, count;
            zstd::stream_range(n, four, st, first, count);
            const uint32_t total = z_stream_scatter(L, in, first, count, (uint32_t*)sc.streams);
            const uint32_t bytes = total / 8 + 1;
            const uint32_t o = L.state[1];
            // a stream that would not fit the block's own size: no entropy-only content
            const bool fits = o + bytes + 1 < n && (four || o + bytes - hs <= zstd::kSingleStreamMax);
            if (fits) {
                const uint8_t* wb = sc.streams;
                for (uint32_t i = tid; i < bytes; i += kZT) slot[o + i] = wb[i];
            }
            __syncthreads();
            if (tid == 0) {
                if (!fits) L.state[2] = 1;
                L.ssize[st] = bytes;
                L.state[1] = o + bytes;
            }
            __syncthreads();
            if (L.state[2]) break;
        }
        if (tid == 0 && !L.state[2]) {  // the entropy-only content is complete
            const uint32_t end = L.state[1];
            zstd::lit_header(slot, four, n, end - hs);
            if (four) {
                const uint32_t tsz = 1 + (L.code.last + 1) / 2;
                for (uint32_t k = 0; k < 3; ++k) {
                    slot[hs + tsz + 2 * k] = (uint8_t)L.ssize[k];
                    slot[hs + tsz + 2 * k + 1] = (uint8_t)(L.ssize[k] >> 8);
                }
            }
            slot[end] = 0;  // Sequences_Section: Number_of_Sequences = 0
            L.state[3] = end + 1;
        }
    }
    __syncthreads();
    phase(1);
    // literals + sequences
    if (!rle && n >= 2) {
        // the '{' gaps (zstd::gap_count) and the sampled repeat distances (zstd::repeat_dist)
        // straight from the text, four bytes a load, counted with LDS atomics
        for (uint32_t c = tid; 16 * c < n; c += kZT) {
            const uint4 v = *(const uint4*)(in + 16 * c);
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (!z_has_brace(w4[q])) continue;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t p = 16 * c + 4 * q + k;
                    if (p < n && ((w4[q] >> (8 * k)) & 0xFF) == '{') z_gap_count(in, p, L.gaps);
                }
            }
        }
        for (uint32_t p = zstd::kRepStep * tid; p < n; p += zstd::kRepStep * kZT)
            if (const uint32_t d = z_repeat_dist(in, n, p)) atomicAdd(&L.reps[d], 1u);
        __syncthreads();
        if (tid == 0) {
            L.state[4] = zstd::pick_cands(L.gaps, L.reps, L.cand);
        }
        __syncthreads();
        const uint32_t nc = L.state[4];
        phase(2);
        for (uint32_t p = tid; p < n; p += kZT) sc.best[p] = zstd::best_at(in, n, p, L.cand, nc);
        __syncthreads();
        phase(3);
        // hash candidates in rounds of kHashRound positions (zstd::hash_look), the table in
        // the stream words (free after the entropy-only streams); position p stays with
        // thread p % kZT, so its best is read back by the thread that wrote it
        static_assert(zstd::kHashRound % kZT == 0 && (1u << zstd::kHashBits) <= kZWords, "hash rounds");
        uint32_t* tab = L.words;
        for (uint32_t i = tid; i < (1u << zstd::kHashBits); i += kZT) tab[i] = 0;
        __syncthreads();
        // zstd::hash_look / hash_put, a thread's kPer positions of a round at once (their
        // loads in flight together; the hashes kept for the puts)
        constexpr uint32_t kPer = zstd::kHashRound / kZT;
        for (uint32_t r0 = 0; r0 < n; r0 += zstd::kHashRound) {
            uint32_t h[kPer], wp[kPer], e[kPer];
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                const uint32_t p = r0 + tid + i * kZT;
                wp[i] = p + 4 <= n ? zstd::ld32u(in + p) : 0u;
                h[i] = p + 4 <= n ? (wp[i] * 2654435761u) >> (32 - zstd::kHashBits) : 0xFFFFFFFFu;  // zstd::hash4
            }
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) e[i] = h[i] != 0xFFFFFFFFu ? tab[h[i]] : 0u;
            uint32_t wq[kPer], bp[kPer];
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                const uint32_t p = r0 + tid + i * kZT;
                wq[i] = e[i] ? zstd::ld32u(in + e[i] - 1) : ~wp[i];
                bp[i] = e[i] ? sc.best[p] : 0u;
            }
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                if (!e[i]) continue;
                const uint32_t p = r0 + tid + i * kZT, q = e[i] - 1, d = p - q;
                const uint32_t lim = min(n - p, zstd::kProbe);
                const uint32_t x = wp[i] ^ wq[i];
                const uint32_t l = x ? (uint32_t)__builtin_ctz(x) >> 3 : 4 + zstd::common_len(in, p + 4, q + 4, lim - 4);
                if (l >= (d < zstd::kHashNear ? zstd::kHashMinNear : zstd::kHashMinFar) && l > (bp[i] >> 24))
                    sc.best[p] = (l << 24) | d;
            }
            __syncthreads();
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i)
                if (h[i] != 0xFFFFFFFFu) atomicMax(&tab[h[i]], r0 + tid + i * kZT + 1);
            __syncthreads();
        }
        uint32_t mine = 0;
        for (uint32_t p = tid; p < n; p += kZT) mine += sc.best[p] != 0;
        if (mine) atomicAdd(&L.state[5], mine);
        __syncthreads();
        phase(4);
        if (zstd::lz_worth(L.state[5], n)) {
            const uint32_t zc = z_lz_content(L, in, n, sc, timing, tph);
            // zc < n keeps the copy inside this block's slot (the body may reach 2n + 64
            // when no entropy-only content was possible), as block_content_seq does
            if (tid == 0) L.state[6] = (zc && zc < L.state[3] && zc < n) ? zc : 0u;
            __syncthreads();
            phase(5);
            const uint32_t z = L.state[6];
            for (uint32_t i = tid; i < z; i += kZT) slot[i] = sc.body[i];
            if (tid == 0 && z) L.state[3] = z;
        }
    }
    phase(6);
    if (tid == 0) {
        uint32_t t = rle ? 1u : 0u, size = rle ? 1u : n;
        if (!rle && L.state[3] < n) {
            t = 2;
            size = L.state[3];
        }
        type_out[blockIdx.x] = t;
        size_out[blockIdx.x] = size;
        len64[blockIdx.x] = 3ull + size;
    }
}

// Blocks [b0, b0 + nb) behind their headers at base + off[i]; block 0 of the frame also
// writes the frame header.  Raw blocks come from the text, RLE blocks are one byte,
// Compressed blocks come from their slots.
__global__ __launch_bounds__(kZT) void k_zstd_frame(const uint8_t* __restrict__ text, uint64_t len, uint64_t b0,
                                                    uint64_t nblocks, const uint8_t* __restrict__ slots,
                                                    const uint32_t* __restrict__ size_in,
                                                    const uint32_t* __restrict__ type_in,
                                                    const uint64_t* __restrict__ off, uint64_t base,
                                                    uint8_t* __restrict__ out) {
    const uint64_t gb = b0 + blockIdx.x;
    const uint32_t t = type_in[blockIdx.x], size = size_in[blockIdx.x];
    const uint32_t n = (uint32_t)min<uint64_t>(zstd::kBlockMax, len - gb * zstd::kBlockMax);
    uint8_t* o = out + base + off[blockIdx.x];
    if (threadIdx.x == 0) {
        if (gb == 0) zstd::frame_header(out, len);
        zstd::block_header(o, gb + 1 == nblocks, t, t == 2 ? size : n);
    }
    const uint8_t* src = t == 2 ? slots + (uint64_t)blockIdx.x * zstd::kBlockMax : text + gb * zstd::kBlockMax;
    for (uint32_t i = threadIdx.x; i < size; i += kZT) o[3 + i] = src[i];
}

// ===========================================================================
// K6: apply_delta on the device (applier.rs:22-56 as a gather-copy)
// ===========================================================================
// One workgroup per piece (an op, or a <= 64 KiB slice of one).  Thread t writes the
// 16-byte-aligned destination chunks t, t+256, ... (aligned in absolute addresses, so
// any buffer offsets work); a chunk wholly inside the piece is assembled from two
// aligned 16-byte source loads with alignbyte (the source address of destination
// address x is x + delta, uniform per piece, so the misalignment delta & 15 is too);
// the partial chunks at the two ends of a piece are written byte by byte, so adjacent
// pieces never race.
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t r) {
    return __builtin_amdgcn_alignbyte(hi, lo, r);
}

__global__ __launch_bounds__(256) void k_apply(const ApplyPiece* __restrict__ pieces, const uint8_t* __restrict__ basis,
                                               const uint8_t* __restrict__ lit, uint8_t* __restrict__ out) {
    const ApplyPiece P = pieces[blockIdx.x];
    const uintptr_t a0 = (uintptr_t)(out + P.dst), a1 = a0 + P.len;  // absolute destination range
    const uintptr_t delta = (uintptr_t)((P.from_basis ? basis : lit) + P.src) - a0;  // mod 2^64
    const uintptr_t c_first = a0 & ~(uintptr_t)15, c_end = (a1 + 15) & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(delta & 15);
    const uint32_t dq = sh >> 2, r = sh & 3;
    for (uintptr_t c = c_first + 16ull * threadIdx.x; c < c_end; c += 16ull * blockDim.x) {
        if (c >= a0 && c + 16 <= a1) {
            const uint4* sa = (const uint4*)((c + delta) & ~(uintptr_t)15);
            const uint4 A = sa[0];
            uint4 B = make_uint4(0, 0, 0, 0);
            if (sh) B = sa[1];
            const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
            uint4 o;
            // dword k of the output = bytes [sh + 4k, +4) of A|B
            switch (dq) {
                case 0: o = make_uint4(funnel(w[1], w[0], r), funnel(w[2], w[1], r), funnel(w[3], w[2], r), funnel(w[4], w[3], r)); break;
                case 1: o = make_uint4(funnel(w[2], w[1], r), funnel(w[3], w[2], r), funnel(w[4], w[3], r), funnel(w[5], w[4], r)); break;
                case 2: o = make_uint4(funnel(w[3], w[2], r), funnel(w[4], w[3], r), funnel(w[5], w[4], r), funnel(w[6], w[5], r)); break;
                default: o = make_uint4(funnel(w[4], w[3], r), funnel(w[5], w[4], r), funnel(w[6], w[5], r), funnel(w[7], w[6], r)); break;
            }
            *(uint4*)c = o;
        } else {
            const uintptr_t lo = c < a0 ? a0 : c, hi = (c + 16 < a1) ? c + 16 : a1;
            for (uintptr_t x = lo; x < hi; ++x) *(uint8_t*)x = *(const uint8_t*)(x + delta);
        }
    }
}

// ===========================================================================
// K7: serde_json text of a Delta on the device (wire format, sydelta_wire.cpp)
// ===========================================================================
// Pieces in op order: a Copy op, or a <= 4 KiB chunk of a Data op's literal bytes.
// Pass 1 sizes every piece's text, an exclusive scan places them, pass 2 writes them.
// A Data chunk is formatted into LDS (<= 4 characters per byte) at the 16-byte phase of
// its destination, then leaves with aligned 16-byte stores; the partial granules at its
// two ends are written byte by byte, so neighbouring pieces never race.
__device__ __forceinline__ uint32_t dec_digits(uint64_t v) {
    uint32_t n = 1;
    while (v >= 10) { v /= 10; ++n; }
    return n;
}
__device__ __forceinline__ uint32_t byte_digits(uint32_t v) { return v >= 100 ? 3u : (v >= 10 ? 2u : 1u); }

__device__ __forceinline__ uint32_t json_copy_len(const JsonPiece& P) {
    return (P.flags & kJsonSep ? 1u : 0u) + 28u + dec_digits(P.a) + dec_digits(P.b);  // {"Copy":{"offset":,"size":}}
}

// K7s: serde_json text of a device-resident signature (sydelta_sigjson.hpp).  Per tile of
// kTile entries: the summed text length, then the text composed in LDS and stored with
// 16-byte stores (byte stores on the two edge chunks shared with the neighbours).
__global__ __launch_bounds__(sigjson::kTile) void k_sigjson_len(sigjson::SigArgs a, uint64_t* __restrict__ tile_len) {
    typedef hipcub::BlockReduce<uint32_t, sigjson::kTile> Reduce;
    __shared__ typename Reduce::TempStorage tmp;
    const uint64_t i = (uint64_t)blockIdx.x * sigjson::kTile + threadIdx.x;
    const uint32_t len = i < a.n ? sigjson::entry_len(a, i) : 0u;
    const uint32_t tot = Reduce(tmp).Sum(len);
    if (threadIdx.x == 0) tile_len[blockIdx.x] = tot;
}

__global__ __launch_bounds__(sigjson::kTile) void k_sigjson_write(sigjson::SigArgs a,
                                                                  const uint64_t* __restrict__ tile_off,
                                                                  uint8_t* __restrict__ out) {
    typedef hipcub::BlockScan<uint32_t, sigjson::kTile> Scan;
    __shared__ typename Scan::TempStorage tmp;
    __shared__ __attribute__((aligned(16))) uint8_t stage[sigjson::kStage];
    const uint64_t i = (uint64_t)blockIdx.x * sigjson::kTile + threadIdx.x;
    const uint32_t len = i < a.n ? sigjson::entry_len(a, i) : 0u;
    uint32_t off = 0, tot = 0;
    Scan(tmp).ExclusiveSum(len, off, tot);
    if (i < a.n) sigjson::entry_write(a, i, stage + off);
    __syncthreads();
    uint8_t* dst = out + tile_off[blockIdx.x];
    const uintptr_t c0 = (uintptr_t)dst & ~(uintptr_t)15, c1 = ((uintptr_t)dst + tot + 15) & ~(uintptr_t)15;
    for (uintptr_t c = c0 + 16ull * threadIdx.x; c < c1; c += 16ull * sigjson::kTile)
        sigjson::store_chunk(stage, tot, dst, c);
}

// K7p: the compact signature text parsed on the device (sydelta_sigjson.hpp chunk_parse).
__global__ __launch_bounds__(256) void k_sigparse_count(const uint8_t* __restrict__ t, uint64_t len,
                                                        uint64_t* __restrict__ count) {
    const uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (c * sigjson::kParseChunk < len) count[c] = sigjson::chunk_entries(t, len, c);
}

__global__ __launch_bounds__(256) void k_sigparse(const uint8_t* __restrict__ t, uint64_t len,
                                                  const uint64_t* __restrict__ rank, sydelta_block_checksum* out,
                                                  uint64_t cap, unsigned long long* bad) {
    const uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (c * sigjson::kParseChunk >= len) return;
    const uint64_t b = sigjson::chunk_parse(t, len, c, rank[c], out, cap);
    if (b != UINT64_MAX) atomicMin(bad, (unsigned long long)b);
}

// K7d: the compact Delta JSON parsed on the device (sydelta_dparse.hpp).  Each wave
// takes 64 consecutive chunks (4 KiB of text) and first stages them, with 8 bytes before
// and 136 after, in LDS (64-byte rows padded to 68 bytes, so the 64 lanes reading row l at
// the same column hit different banks); the per-chunk bodies then read their bytes from
// there (LdsText) and anything outside the staged span from global memory.  Round 3 ran
// the same bodies on global memory, one byte load per character per thread with the
// lanes 64 bytes apart: 113 GB/s of text over the three kernels.
constexpr uint32_t kDpRow = 68;                          // LDS bytes per staged 64-byte row
constexpr uint32_t kDpBefore = 8;                        // bytes staged before the wave's first chunk
constexpr uint32_t kDpSpan = 64 * 64 + kDpBefore + 136;  // staged bytes per wave
constexpr uint32_t kDpRows = (kDpSpan + 63) / 64;

// The text outside the staged span (not reached by well-formed text: every token and its
// look-ahead ends inside the 136-byte halo).  Not inlined, so that the compiler cannot
// turn the accessor's branch into a select that issues this global load for every byte.
__device__ __noinline__ uint8_t dp_gload(const uint8_t* g, uint64_t p) { return g[p]; }
struct LdsText {
    const uint8_t* g;   // the text
    const lds_u8* l;    // the wave's staged rows
    uint64_t p0, n;     // staged text [p0, p0 + n)
    __device__ __forceinline__ uint8_t operator[](uint64_t p) const {
        const uint64_t d = p - p0;
        if (__builtin_expect(d < n, 1)) return l[(d >> 6) * kDpRow + (d & 63)];
        return dp_gload(g, p);
    }
};

// The fast path of the three kernels: a chunk of 64 digits and commas (inside a Data
// op's literal run: almost all of a literal-heavy delta's text) is classified with SWAR
// masks from 18 dwords of the staged rows instead of byte by byte.  DpFast.ok: the chunk
// is such a chunk, every literal starting in it is 1-3 digits without a leading zero,
// <= 255, followed by ',' and a digit (all checked here, with 8 bytes of look-ahead), so
// chunk_count / chunk_parse would find exactly these literals and nothing else; any other
// chunk (ops, the end of a run, a bad byte) takes the bodies.
struct DpFast {
    bool ok;
    uint64_t lits;  // bit i: a literal starts at byte i of the chunk
    uint32_t x[18]; // the chunk's 64 bytes and 8 bytes of look-ahead
};
__device__ __forceinline__ uint32_t dp_bits4(uint32_t m) {  // bit 7 of each byte -> bits 0..3
    return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}
__device__ __forceinline__ uint32_t dp_digits4(uint32_t x) {
    const uint32_t t = x ^ 0x30303030u;
    return dp_bits4(~(((t & 0x7F7F7F7Fu) + 0x76767676u) | t) & 0x80808080u);
}
__device__ __forceinline__ uint32_t dp_eq4(uint32_t x, uint32_t pat) {
    const uint32_t y = x ^ pat;
    return dp_bits4(~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u);
}
__device__ __forceinline__ void dp_fast(const dparse::DArgs& a, const LdsText& t, uint64_t c, DpFast& f) {
    f.ok = false;
    f.lits = 0;
    const uint64_t lo = dparse::chunk_lo(a, c);
    if (c == 0 || lo + 72 > a.e) return;  // the first chunk, the tail: the bodies
    const uint32_t d0 = (uint32_t)(lo - t.p0);  // 8 + 64 * lane: dword-aligned, inside one row each
    if (d0 + 72 > t.n) return;
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
#pragma unroll
    for (int k = 0; k < 18; ++k) {
        const uint32_t dd = d0 + 4 * k;
        f.x[k] = *(lds_u32*)(t.l + (dd >> 6) * kDpRow + (dd & 63));
    }
    const uint32_t dp = d0 - 4;
    const uint32_t prevw = *(lds_u32*)(t.l + (dp >> 6) * kDpRow + (dp & 63));
    uint64_t D = 0, C = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        D |= (uint64_t)dp_digits4(f.x[k]) << (4 * k);
        C |= (uint64_t)dp_eq4(f.x[k], 0x2C2C2C2Cu) << (4 * k);
    }
    if ((D | C) != ~0ull) return;
    const uint32_t DL = dp_digits4(f.x[16]) | (dp_digits4(f.x[17]) << 4);  // look-ahead bytes 64..71
    const uint32_t CL = dp_eq4(f.x[16], 0x2C2C2C2Cu) | (dp_eq4(f.x[17], 0x2C2C2C2Cu) << 4);
    const uint32_t pb = prevw >> 24;
    const uint64_t L = D & ((C << 1) | (uint64_t)(pb == ',' || pb == '['));
    // digits / commas at i+1, i+2, i+3 (with the look-ahead)
    const uint64_t D1 = (D >> 1) | ((uint64_t)DL << 63), D2 = (D >> 2) | ((uint64_t)DL << 62),
                   D3 = (D >> 3) | ((uint64_t)DL << 61), D4 = (D >> 4) | ((uint64_t)DL << 60);
    const uint64_t C1 = (C >> 1) | ((uint64_t)CL << 63), C2 = (C >> 2) | ((uint64_t)CL << 62),
                   C3 = (C >> 3) | ((uint64_t)CL << 61);
    // 1 digit: ',' then a digit; 2: digit, ',', digit; 3: digit, digit, ',', digit; 4+: bad
    const uint64_t len1 = ~D1, len2 = D1 & ~D2, len3 = D1 & D2 & ~D3;
    const uint64_t follow = (len1 & C1 & D2) | (len2 & C2 & D3) | (len3 & C3 & D4);
    if (L & ~follow) return;
    f.lits = L;
    f.ok = true;  // values (<= 255, no leading zero) are checked while they are written
}
// Byte i of the fast chunk (constant i after unrolling).
__device__ __forceinline__ uint32_t dp_byte(const DpFast& f, int i) { return (f.x[i >> 2] >> (8 * (i & 3))) & 0xFFu; }

// Stage this wave's span (chunks c0 .. c0 + 63) and return its accessor.
__device__ __forceinline__ LdsText dp_stage(const dparse::DArgs& a, uint64_t c0, uint8_t* rows) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t p0 = dparse::chunk_lo(a, c0) - kDpBefore;  // >= 0: chunk 0 starts at kHead = 8
    const uint64_t hi = p0 + kDpSpan < a.e ? p0 + kDpSpan : a.e;
    const uint32_t n = (uint32_t)(hi - p0);
    const uint8_t* g = a.t + p0;
    if (((uintptr_t)g & 3) == 0) {
        for (uint32_t i = 4 * lane; i < n; i += 256) {
            if (i + 4 <= n) {
                *(uint32_t*)(rows + (i >> 6) * kDpRow + (i & 63)) = *(const uint32_t*)(g + i);
            } else {
                for (uint32_t j = i; j < n; ++j) rows[(j >> 6) * kDpRow + (j & 63)] = g[j];
            }
        }
    } else {
        for (uint32_t i = lane; i < n; i += 64) rows[(i >> 6) * kDpRow + (i & 63)] = g[i];
    }
    lds_fence();
    return LdsText{a.t, (const lds_u8*)rows, p0, n};
}

__global__ __launch_bounds__(256) void k_dparse_count(dparse::DArgs a, uint64_t* __restrict__ ocnt,
                                                      uint64_t* __restrict__ lcnt) {
    __shared__ uint8_t st[4][kDpRows * kDpRow];
    const uint64_t c0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) & ~63ull;  // the wave's first chunk
    if (c0 >= a.nc) return;  // whole waves only
    const LdsText t = dp_stage(a, c0, st[threadIdx.x >> 6]);
    const uint64_t c = c0 + (threadIdx.x & 63);
    if (c >= a.nc) return;
    uint64_t no, nl;
    DpFast f;
    dp_fast(a, t, c, f);
    if (f.ok) {
        no = 0;
        nl = __popcll(f.lits);
    } else {
        dparse::chunk_count(a, t, c, no, nl);
    }
    ocnt[c] = no;
    lcnt[c] = nl;
}

__global__ __launch_bounds__(256) void k_dparse_place(dparse::DArgs a, const uint64_t* __restrict__ orank,
                                                      uint64_t* __restrict__ pos) {
    __shared__ uint8_t st[4][kDpRows * kDpRow];
    const uint64_t c0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) & ~63ull;
    if (c0 >= a.nc) return;
    // a wave whose chunks start no op (a literal run's) has nothing to place: orank has nc + 1 entries
    if (orank[c0 + 64 < a.nc ? c0 + 64 : a.nc] == orank[c0]) return;  // wave-uniform
    const LdsText t = dp_stage(a, c0, st[threadIdx.x >> 6]);
    const uint64_t c = c0 + (threadIdx.x & 63);
    if (c >= a.nc) return;
    DpFast f;
    dp_fast(a, t, c, f);
    if (!f.ok) dparse::chunk_place(a, t, c, orank[c], pos);
}

// The literal bytes of a wave's chunks are one contiguous range of the output, [lrank[c0],
// lrank[c0 + 64]) (a 64-byte chunk starts at most 32 literals): the lanes write them into
// the wave's LDS staging (LdsLit) and the wave stores the range with whole dwords, the
// partial dwords at its two ends byte by byte (they may be shared with the neighbouring
// waves' ranges).  Byte stores from 64 lanes 18 bytes apart made the round-3 kernel's
// literal output the bulk of its time.
constexpr uint32_t kDpLitMax = 64 * (dparse::kChunk / 2);
struct LdsLit {
    __attribute__((address_space(3))) uint8_t* l;
    uint64_t base;  // output index of l[0]
    __device__ __forceinline__ explicit operator bool() const { return true; }
    __device__ __forceinline__ __attribute__((address_space(3))) uint8_t& operator[](uint64_t i) const {
        return l[i - base];
    }
};

__global__ __launch_bounds__(256) void k_dparse(dparse::DArgs a, const uint64_t* __restrict__ orank,
                                                const uint64_t* __restrict__ lrank, const uint64_t* __restrict__ pos,
                                                uint64_t nops, sydelta_op* __restrict__ ops, uint8_t* lit,
                                                unsigned long long* bad) {
    __shared__ uint8_t st[4][kDpRows * kDpRow];
    __shared__ uint8_t lo[4][kDpLitMax];
    const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t c0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) & ~63ull;
    if (c0 >= a.nc) return;
    const LdsText t = dp_stage(a, c0, st[wid]);
    const uint64_t c = c0 + lane;
    const uint64_t l0 = lrank[c0], l1 = lrank[c0 + 64 < a.nc ? c0 + 64 : a.nc];
    if (c < a.nc) {
        const bool staged = lit && l1 - l0 <= kDpLitMax;
        DpFast f;
        dp_fast(a, t, c, f);
        if (f.ok) {  // each literal's value; a leading zero or a value > 255 sends the chunk to the body
            const uint64_t r0 = lrank[c];
            bool good = true;
#pragma unroll
            for (int i = 0; i < 64; ++i) {
                if (!((f.lits >> i) & 1)) continue;
                const uint32_t b0 = dp_byte(f, i) - '0', b1 = dp_byte(f, i + 1) - '0', b2 = dp_byte(f, i + 2) - '0';
                const bool two = b1 < 10, three = two && b2 < 10;
                const uint32_t v = three ? b0 * 100 + b1 * 10 + b2 : two ? b0 * 10 + b1 : b0;
                good &= v <= 255 && !(two && b0 == 0);
                const uint64_t r = r0 + __popcll(f.lits & ((1ull << i) - 1));
                if (lit) {
                    if (staged) lo[wid][r - l0] = (uint8_t)v;
                    else lit[r] = (uint8_t)v;
                }
            }
            f.ok = good;
        }
        if (!f.ok) {
            uint64_t b;
            if (staged)
                b = dparse::chunk_parse(a, t, c, orank, lrank, pos, nops, ops,
                                        LdsLit{(__attribute__((address_space(3))) uint8_t*)lo[wid], l0});
            else
                b = dparse::chunk_parse(a, t, c, orank, lrank, pos, nops, ops, lit);
            if (b != dparse::kNoBad) atomicMin(bad, (unsigned long long)b);
        }
    }
    if (!lit || l1 - l0 > kDpLitMax || l1 == l0) return;  // wave-uniform
    lds_fence();
    // [l0, l1): head bytes up to a dword boundary (of the absolute address), whole dwords,
    // tail bytes
    const uint8_t* src = lo[wid];
    const int64_t ph = (int64_t)((uintptr_t)lit & 3);
    const uint64_t a0 = (uint64_t)((((int64_t)l0 + ph + 3) & ~3ll) - ph);
    const int64_t a1s = (((int64_t)l1 + ph) & ~3ll) - ph;
    const uint64_t a1 = a1s < (int64_t)a0 ? a0 : (uint64_t)a1s;
    if (a0 >= a1) {
        for (uint64_t i = l0 + lane; i < l1; i += 64) lit[i] = src[i - l0];
        return;
    }
    if (lane < a0 - l0) lit[l0 + lane] = src[lane];
    if (lane < l1 - a1) lit[a1 + lane] = src[a1 - l0 + lane];
    for (uint64_t i = a0 + 4ull * lane; i < a1; i += 256) {
        const uint64_t k = i - l0;
        const uint32_t v = (uint32_t)src[k] | ((uint32_t)src[k + 1] << 8) | ((uint32_t)src[k + 2] << 16) |
                           ((uint32_t)src[k + 3] << 24);
        *(uint32_t*)(lit + i) = v;
    }
}

__global__ __launch_bounds__(256) void k_json_len(const JsonPiece* __restrict__ pieces, uint64_t npieces,
                                                  const uint8_t* __restrict__ lit, uint64_t* __restrict__ len) {
    // one wave per piece (lane l sizes literal bytes [64l, 64l + 64) of a Data chunk);
    // Copy pieces are sized by lane 0
    const uint64_t pi = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (pi >= npieces) return;
    const JsonPiece P = pieces[pi];
    if (!(P.flags & kJsonData)) {
        if (lane == 0) len[pi] = json_copy_len(P);
        return;
    }
    static_assert(kJsonChunk == 64 * 64, "one lane per 64 literal bytes");
    const uint32_t b0 = 64 * lane;
    const uint32_t cnt = b0 < P.len ? min(64u, P.len - b0) : 0u;
    const uint8_t* lp = lit + P.src + b0;
    uint32_t c = 0;
    if (cnt == 64 && ((uintptr_t)lp & 15) == 0) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = ((const uint4*)lp)[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int j = 0; j < 16; ++j) c += byte_digits((w[j >> 2] >> (8 * (j & 3))) & 0xFF);
        }
    } else if (cnt == 64) {  // unaligned: the 17 dwords holding the 64 bytes
        const uintptr_t u = (uintptr_t)lp;
        const uint32_t sh = (uint32_t)(u & 3);
        const uint32_t* q = (const uint32_t*)(u & ~(uintptr_t)3);
        uint32_t d[17];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = q[k];
        d[16] = sh ? q[16] : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t x = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
#pragma unroll
            for (int j = 0; j < 4; ++j) c += byte_digits((x >> (8 * j)) & 0xFF);
        }
    } else {
        for (uint32_t j = 0; j < cnt; ++j) c += byte_digits(lp[j]);
    }
    c = wave_sum32_dpp(c);
    if (lane == 0) {
        uint32_t t = c;
        t += P.len ? P.len - 1 : 0;                     // commas between bytes of the chunk
        if (!(P.flags & kJsonLast) && P.len) t += 1;    // comma before the next chunk's first byte
        if (P.flags & kJsonFirst) t += 9;               // {"Data":[
        if (P.flags & kJsonLast) t += 2;                // ]}
        if (P.flags & kJsonSep) t += 1;                 // , before the op
        len[pi] = t;
    }
}

// Decimal digits of v at p (no terminator); returns their count.
__device__ __forceinline__ uint32_t put_dec(uint8_t* p, uint64_t v) {
    const uint32_t n = dec_digits(v);
    for (uint32_t i = n; i-- > 0;) {
        p[i] = (uint8_t)('0' + v % 10);
        v /= 10;
    }
    return n;
}

__global__ __launch_bounds__(256) void k_json_write(const JsonPiece* __restrict__ pieces,
                                                    const uint8_t* __restrict__ lit, const uint64_t* __restrict__ off,
                                                    uint64_t base, uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char js[];  // text staging, kJsonStage bytes
    __shared__ uint32_t wsum[4];
    const JsonPiece P = pieces[blockIdx.x];
    const uint64_t dst = base + off[blockIdx.x];
    if (!(P.flags & kJsonData)) {
        if (threadIdx.x == 0) {  // {"Copy":{"offset":A,"size":B}} straight to global memory
            uint8_t* o = out + dst;
            uint32_t k = 0;
            if (P.flags & kJsonSep) o[k++] = ',';
            const char* h = "{\"Copy\":{\"offset\":";
            for (uint32_t i = 0; h[i]; ++i) o[k++] = h[i];
            k += put_dec(o + k, P.a);
            const char* m = ",\"size\":";
            for (uint32_t i = 0; m[i]; ++i) o[k++] = m[i];
            k += put_dec(o + k, P.b);
            o[k++] = '}';
            o[k++] = '}';
        }
        return;
    }
    // thread t formats bytes [16t, 16t + 16) of the chunk (kJsonChunk = 16 * 256)
    const uint32_t b0 = 16 * threadIdx.x;
    const uint32_t cnt = b0 < P.len ? min(16u, P.len - b0) : 0u;
    const uint8_t* lp = lit + P.src + b0;
    uint32_t w[4] = {0, 0, 0, 0};
    if (cnt == 16) {
        const uintptr_t u = (uintptr_t)lp;
        if ((u & 15) == 0) {
            const uint4 v = *(const uint4*)lp;
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {  // dwords holding the 16 bytes (never past the granule of a valid byte)
            const uint32_t sh = (uint32_t)(u & 3);
            const uint32_t* q = (const uint32_t*)(u & ~(uintptr_t)3);
            const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = sh ? q[4] : 0u;
            w[0] = __builtin_amdgcn_alignbyte(d1, d0, sh); w[1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
            w[2] = __builtin_amdgcn_alignbyte(d3, d2, sh); w[3] = __builtin_amdgcn_alignbyte(d4, d3, sh);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < (int)cnt) w[j >> 2] |= (uint32_t)lp[j] << (8 * (j & 3));
    }
    // text of each byte + its comma: 2-4 characters, branch-free
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t v = (w[j >> 2] >> (8 * (j & 3))) & 0xFF;
        mine += (j < (int)cnt) ? 2u + (v >= 10) + (v >= 100) : 0u;
    }
    // exclusive scan of `mine` over the workgroup
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t inc = mine;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)inc, m, 64);
        if (lane >= (uint32_t)m) inc += o;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = inc - mine;
    for (uint32_t q = 0; q < wid; ++q) pre += wsum[q];
    const uint32_t ph = (uint32_t)(dst & 15);  // LDS byte k <-> global byte (dst & ~15) + k
    uint32_t head = ph;
    if (P.flags & kJsonSep) head += 1;
    if (P.flags & kJsonFirst) head += 9;
    if (threadIdx.x == 0) {
        uint32_t k = ph;
        if (P.flags & kJsonSep) js[k++] = ',';
        if (P.flags & kJsonFirst) {
            const char* h = "{\"Data\":[";
            for (uint32_t i = 0; h[i]; ++i) js[k++] = h[i];
        }
    }
    uint32_t k = head + pre;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t v = (w[j >> 2] >> (8 * (j & 3))) & 0xFF;
        const uint32_t h = v / 100, t = (v / 10) % 10, o = v % 10;
        const uint32_t nd = 1 + (v >= 10) + (v >= 100);
        // characters: [h] [t] o ','  (leading digits only when present)
        const uint32_t c0 = nd == 3 ? '0' + h : (nd == 2 ? '0' + t : '0' + o);
        const uint32_t c1 = nd == 3 ? '0' + t : (nd == 2 ? '0' + o : ',');
        const uint32_t c2 = nd == 3 ? '0' + o : ',';
        if (j < (int)cnt) {
            js[k] = (unsigned char)c0;
            js[k + 1] = (unsigned char)c1;
            if (nd >= 2) js[k + 2] = (unsigned char)c2;
            if (nd == 3) js[k + 3] = ',';
            k += nd + 1;
        }
    }
    const uint32_t body = wsum[0] + wsum[1] + wsum[2] + wsum[3];  // every byte with a comma
    static_assert(kJsonChunk == 16 * 256, "one thread per 16 literal bytes");
    uint32_t end = head + body;
    if ((P.flags & kJsonLast) && P.len) end -= 1;  // no comma after the op's last byte
    if (P.flags & kJsonLast) {
        __syncthreads();
        if (threadIdx.x == 0) { js[end] = ']'; js[end + 1] = '}'; }
        end += 2;
    }
    __syncthreads();
    // LDS [ph, end) -> out [dst, dst + end - ph)
    uint8_t* g = out + (dst & ~15ull);
    for (uint32_t c = 16 * threadIdx.x; c < end; c += 16 * blockDim.x) {
        if (c >= ph && c + 16 <= end) {
            *(uint4*)(g + c) = *(const uint4*)(js + c);
        } else {
            const uint32_t lo = max(c, ph), hi = min(c + 16, end);
            for (uint32_t x = lo; x < hi; ++x) g[x] = js[x];
        }
    }
}

// ===========================================================================
// K8: local-path block compare and change-ratio sampling (local.rs, ratio.rs)
// ===========================================================================
// Block k of the source against block k of the destination (local.rs:549-570): the
// reads match iff their lengths are equal and the bytes are equal.  One workgroup per
// block; 16-byte loads when both blocks are 16-byte aligned.
__global__ __launch_bounds__(256) void k_block_cmp(const uint8_t* __restrict__ src, uint64_t slen,
                                                   const uint8_t* __restrict__ dst, uint64_t dlen, uint64_t bs,
                                                   uint64_t nblocks, uint8_t* __restrict__ changed) {
    for (uint64_t k = blockIdx.x; k < nblocks; k += gridDim.x) {
        const uint64_t off = k * bs;
        const uint64_t sl = min(bs, slen - off);
        const uint64_t dl = dlen > off ? min(bs, dlen - off) : 0;
        int diff = sl != dl;
        if (!diff) {
            const uint8_t* a = src + off;
            const uint8_t* b = dst + off;
            if ((((uintptr_t)a | (uintptr_t)b) & 15) == 0) {
                // 16-byte nontemporal loads, 4 per buffer in flight per lane
                const u32x4* A = (const u32x4*)a;
                const u32x4* B = (const u32x4*)b;
                const uint64_t nv = sl >> 4, st = blockDim.x;
                uint32_t acc = 0;
                uint64_t i = threadIdx.x;
                for (; i + 3 * st < nv; i += 4 * st) {
                    u32x4 x[4], y[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(A + i + u * st);
#pragma unroll
                    for (int u = 0; u < 4; ++u) y[u] = __builtin_nontemporal_load(B + i + u * st);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const u32x4 d = x[u] ^ y[u];
                        acc |= d.x | d.y | d.z | d.w;
                    }
                }
                for (; i < nv; i += st) {
                    const u32x4 d = A[i] ^ B[i];
                    acc |= d.x | d.y | d.z | d.w;
                }
                diff = acc != 0;
                for (uint64_t j = (nv << 4) + threadIdx.x; j < sl && !diff; j += st) diff = a[j] != b[j];
            } else {
                for (uint64_t i = threadIdx.x; i < sl && !diff; i += blockDim.x) diff = a[i] != b[i];
            }
        }
        diff = __syncthreads_or(diff);
        if (threadIdx.x == 0) changed[k] = diff ? 1 : 0;
    }
}

// XXH3-64 of block pos[i] of buf (length min(bs, len - off), 0 past the end): one
// wave per sampled block (ratio.rs:160-165).
__global__ __launch_bounds__(256) void k_hash_blocks(const uint8_t* __restrict__ buf, uint64_t len, uint64_t bs,
                                                     const uint64_t* __restrict__ pos, uint32_t count,
                                                     uint64_t* __restrict__ out) {
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= count) return;
    const uint64_t off = pos[w] * bs;
    const uint64_t n = len > off ? min(bs, len - off) : 0;
    uint32_t wk;
    uint64_t st;
    if (n > 240) {
        wave_hash_long(buf + off, n, wk, st);
    } else {
        st = 0;
        if ((threadIdx.x & 63) == 0) st = xxh3_short(buf + off, n);
    }
    if ((threadIdx.x & 63) == 0) out[w] = st;
}

// ===========================================================================
// K9: whole-file XXH3-64 (integrity/xxhash3.rs:17-40, XxHash3Hasher::hash_file)
// ===========================================================================
// XXH3's long path is acc <- scramble(acc + C_k) over the 1 KiB blocks k of the file,
// where C_k (the 16 stripes' accumulator increments) does not depend on acc.  Phase A
// computes every C_k in parallel (HBM-bound); phase B runs the serial scramble chain,
// eight lanes per file and eight files per wave, then the tail stripes and the merge.

// 16 bytes at an arbitrary address, as two little-endian u64 (bytes [a, a+16) valid).
__device__ __forceinline__ void load16u(const uint8_t* a, uint64_t& w0, uint64_t& w1) {
    const uintptr_t u = (uintptr_t)a;
    if ((u & 15) == 0) {
        const u32x4 x = __builtin_nontemporal_load((const u32x4*)a);
        w0 = (uint64_t)x.x | ((uint64_t)x.y << 32);
        w1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
        return;
    }
    const uint32_t sh = (uint32_t)(u & 3);
    const uint32_t* q = (const uint32_t*)(u & ~(uintptr_t)3);
    const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = sh ? q[4] : 0u;
    const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh), x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    const uint32_t x2 = __builtin_amdgcn_alignbyte(d3, d2, sh), x3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
    w0 = (uint64_t)x0 | ((uint64_t)x1 << 32);
    w1 = (uint64_t)x2 | ((uint64_t)x3 << 32);
}

// Phase A: one 16-lane row per kPieceRows consecutive full 1 KiB blocks (global block e
// of file f is block e - fpfx[f] of the file); lane (slot, q) takes stripes slot + 4k
// and accumulator pair (2q, 2q+1).  The file table here lists only files with at
// least one full block.  C is SoA, C[i * cstride + e] = increment of acc[i] by block e,
// so a chain lane's addends are contiguous (16-byte loads cover two steps).
constexpr int kPieceRows = 4;
__global__ __launch_bounds__(256) void k_xxh_pieces(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ foff,
                                                    const uint64_t* __restrict__ fpfx, uint64_t nfiles,
                                                    uint64_t npieces, uint64_t cstride, uint64_t* __restrict__ C) {
    const uint32_t lane = threadIdx.x & 63, q = lane & 3, slot = (lane >> 2) & 3;
    const uint64_t row = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const uint64_t ebase = row * kPieceRows;
    // File of the wave's first block by a 64-way search (fpfx[nfiles] = npieces), then
    // each block steps forward: every listed file has >= 1 block, so the wave's
    // 4 * kPieceRows consecutive blocks span at most that many files.
    const uint64_t e0 = min(__shfl(ebase, 0), npieces - 1);
    uint64_t lo = 0, hi = nfiles;
    while (hi - lo > 1) {
        const uint64_t step = (hi - lo + 63) >> 6;
        const uint64_t c = lo + lane * step;
        const uint64_t m = __ballot(c < hi && fpfx[c] <= e0);
        const uint64_t nlo = lo + (63 - __builtin_clzll(m)) * step;
        hi = min(hi, nlo + step);
        lo = nlo;
    }
    uint64_t w0[kPieceRows][4], w1[kPieceRows][4];
#pragma unroll
    for (int r = 0; r < kPieceRows; ++r) {
        const uint64_t e = min(ebase + r, npieces - 1);
        while (fpfx[lo + 1] <= e) ++lo;
        const uint8_t* p = buf + foff[lo] + ((e - fpfx[lo]) << 10);
#pragma unroll
        for (int k = 0; k < 4; ++k) load16u(p + ((slot + 4 * k) << 6) + (q << 4), w0[r][k], w1[r][k]);
    }
#pragma unroll
    for (int r = 0; r < kPieceRows; ++r) {
        uint64_t c_lo = 0, c_hi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t st = slot + 4 * k;
            c_lo += mul32x32(w0[r][k] ^ c_tab.w[st + 2 * q]) + w1[r][k];
            c_hi += mul32x32(w1[r][k] ^ c_tab.w[st + 2 * q + 1]) + w0[r][k];
        }
        c_lo = dpp_add64<kDppRowRor4>(c_lo);
        c_lo = dpp_add64<kDppRowRor8>(c_lo);
        c_hi = dpp_add64<kDppRowRor4>(c_hi);
        c_hi = dpp_add64<kDppRowRor8>(c_hi);
        const uint64_t e = ebase + r;
        if (e < npieces && slot == 0) {
            C[(uint64_t)(2 * q) * cstride + e] = c_lo;
            C[(uint64_t)(2 * q + 1) * cstride + e] = c_hi;
        }
    }
}

// The chain is carried as y_k = acc_k + C_k (the value block k's scramble sees):
// y_{k+1} = scramble(y_k) + C_{k+1}, acc after the last block = scramble(y_{nb-1}).
// scramble(y) = (y ^ (y >> 47) ^ key) * PRIME32_1: y >> 47 touches only the low word,
// and "* P + c" is one 32x32+64 mad on the low word plus a 32-bit add on the high word,
// so the dependent path per block is shift -> xor3 -> mad -> add.
// (Inline asm pins that shape; left alone the compiler folds the high-word product into
// a second mad behind the first.)  The chain value is kept as two words.
struct Y2 {
    uint32_t lo, hi;
};
__device__ __forceinline__ Y2 chain_step(Y2 y, uint64_t c, uint32_t klo, uint32_t khi) {
    uint32_t t;  // y.lo ^ key.lo does not wait for the high word
    asm("v_xor_b32 %0, %1, %2" : "=v"(t) : "v"(y.lo), "v"(klo));
    const uint32_t tl = t ^ (y.hi >> 15);
    uint32_t th;
    asm("v_mul_lo_u32 %0, %1, %2" : "=v"(th) : "v"(y.hi ^ khi), "s"((uint32_t)P32_1));
    uint64_t m, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(m), "=s"(cc) : "v"(tl), "s"((uint32_t)P32_1), "v"(c));
    Y2 r;
    r.lo = (uint32_t)m;
    asm("v_add_u32 %0, %1, %2" : "=v"(r.hi) : "v"((uint32_t)(m >> 32)), "v"(th));
    return r;
}

constexpr int kChainBatch = 32;
static_assert(xxh_chain_records(0) == 3 * kChainBatch, "C row slack must cover the batch prefetch");

// Phase B: lanes 8g..8g+7 of a wave hash file order[8 * blockIdx.x + g]; lane i keeps
// acc[i].  Files are ordered by size so the eight chains of a wave have similar lengths.
__global__ __launch_bounds__(64) void k_xxh_chain(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ foff,
                                                  const uint64_t* __restrict__ flen, const uint64_t* __restrict__ fpfx,
                                                  const uint32_t* __restrict__ order, uint64_t nfiles,
                                                  uint64_t cstride, const uint64_t* __restrict__ C,
                                                  uint64_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63, g = lane >> 3, i = lane & 7;
    const uint64_t slot = (uint64_t)blockIdx.x * 8 + g;
    const bool act = slot < nfiles;
    const uint32_t f = act ? order[slot] : 0;
    const uint64_t len = act ? flen[f] : 0;
    const uint8_t* p = buf + foff[f];
    const uint64_t nb = len > 240 ? (len - 1) >> 10 : 0;
    const uint64_t steps = nb ? nb - 1 : 0;  // y -> y transitions
    const uint64_t* Ci = C + (uint64_t)i * cstride + (act ? fpfx[f] : 0);
    // step range over the wave
    uint64_t nmin = act ? steps : ~0ull, nmax = steps;
    for (int m = 8; m < 64; m <<= 1) {
        nmin = min(nmin, (uint64_t)__shfl_xor((unsigned long long)nmin, m));
        nmax = max(nmax, (uint64_t)__shfl_xor((unsigned long long)nmax, m));
    }
    const uint64_t key = c_tab.w[16 + i];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    const uint64_t y0 = c_tab.init[i] + Ci[0];  // another file's record (or slack) when nb == 0: unused
    Y2 y{(uint32_t)y0, (uint32_t)(y0 >> 32)};
    const uint64_t* Cn = Ci + 1;          // the addend of step k is C_{k+1}
    // Two register batches: the chain consumes one while the other is in flight.  C rows
    // have 3 * kChainBatch entries of slack, so batch loads never need a bound check.
    uint64_t ba[kChainBatch], bb[kChainBatch];
#pragma unroll
    for (int j = 0; j < kChainBatch; ++j) ba[j] = Cn[j];
    uint64_t k = 0;
    for (; k + 2 * kChainBatch <= nmin; k += 2 * kChainBatch) {  // every chain of the wave runs
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j) bb[j] = Cn[k + kChainBatch + j];
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j) y = chain_step(y, ba[j], klo, khi);
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j) ba[j] = Cn[k + 2 * kChainBatch + j];
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j) y = chain_step(y, bb[j], klo, khi);
    }
    for (; k < nmax; k += 2 * kChainBatch) {  // ragged ends
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j) bb[j] = Cn[k + kChainBatch + j];
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j)
            if (k + j < steps) y = chain_step(y, ba[j], klo, khi);
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j) ba[j] = Cn[k + 2 * kChainBatch + j];
#pragma unroll
        for (int j = 0; j < kChainBatch; ++j)
            if (k + kChainBatch + j < steps) y = chain_step(y, bb[j], klo, khi);
    }
    y = chain_step(y, 0, klo, khi);
    uint64_t acc = nb ? ((uint64_t)y.hi << 32 | y.lo) : c_tab.init[i];
    if (!act) return;
    if (len <= 240) {
        if (i == 0) out[f] = xxh3_short(p, len);
        return;
    }
    // stripes of the last (partial) block, then the last stripe (keys at secret + 121)
    const uint64_t tb = nb << 10;
    const uint64_t ns = ((len - 1) - tb) >> 6;
    for (uint64_t s = 0; s < ns; ++s) {
        const uint8_t* st = p + tb + (s << 6);
        const uint64_t v = ld64u(st + 8 * i), vx = ld64u(st + 8 * (i ^ 1));
        acc += vx + mul32x32(v ^ c_tab.w[s + i]);
    }
    {
        const uint8_t* st = p + len - 64;
        const uint64_t v = ld64u(st + 8 * i), vx = ld64u(st + 8 * (i ^ 1));
        acc += vx + mul32x32(v ^ c_tab.last[i]);
    }
    const uint64_t partner = shfl_xor64(acc, 1);
    uint64_t r = (i & 1) ? 0 : fold64(acc ^ c_tab.merge[i], partner ^ c_tab.merge[i + 1]);
    r += shfl_xor64(r, 2);
    r += shfl_xor64(r, 4);
    if (i == 0) out[f] = xxh3_aval(len * P64_1 + r);
}

// ===========================================================================
// Synthetic inputs (bench)
// ===========================================================================
// bytes [8*w0, 8*w0 + len) of the stream
__global__ void k_synth_fill(uint8_t* __restrict__ buf, uint64_t len, uint64_t seed, uint64_t w0) {
    const uint64_t nw = (len + 7) / 8;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t z = splitmix_word(seed, w0 + i);
        if (8 * i + 8 <= len) {
            *(uint64_t*)(buf + 8 * i) = z;
        } else {
            for (uint64_t b = 8 * i; b < len; ++b) buf[b] = (uint8_t)(z >> (8 * (b - 8 * i)));
        }
    }
}

// Block edits (BASELINE C5): block k (global) is edited iff (r & 0xFFFFFFFF) < thresh,
// r = splitmix(seed, k); byte (r >> 32) % bs of the block ^= 1 + (splitmix(~seed, k) % 255).
// One thread per block of [k0, k0 + nb); the copy of the unedited bytes is done by the caller.
__global__ void k_synth_edit_blocks(uint8_t* __restrict__ dst, uint64_t len, uint64_t bs, uint64_t k0, uint64_t nb,
                                    uint64_t seed, uint64_t thresh) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nb) return;
    const uint64_t r = splitmix_word(seed, k0 + t);
    if ((r & 0xFFFFFFFFull) >= thresh) return;
    const uint64_t o = t * bs + (r >> 32) % bs;
    if (o < len) dst[o] ^= (uint8_t)(1 + splitmix_word(~seed, k0 + t) % 255);
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

int scan_wide_mode() {
    const char* e = getenv("SYDELTA_SCAN_WIDE");
    return (e && e[0] == '0') ? 0 : (e && e[0] == '2') ? 2 : 1;
}

hipError_t launch_signature(const uint8_t* d_buf, uint64_t len, uint64_t bs, uint32_t* d_weak, uint64_t* d_strong,
                            hipStream_t s, Profiler* prof) {
    if (len == 0) return hipSuccess;
    const uint64_t nblocks = (len + bs - 1) / bs;
    const uint64_t nfull = len / bs;
    const bool aligned = (((uintptr_t)d_buf) & 15) == 0;
    uint64_t done = 0;
    if (nfull && aligned && bs % 64 == 0 && bs >= 256 && bs <= (1u << 31)) {
        ProfScope ps(prof, s, "k_sig_fast");
        hipLaunchKernelGGL(k_sig_fast, dim3(grid_for((nfull + 3) / 4 * 64, 256)), dim3(256), 0, s, d_buf, nfull,
                           (uint32_t)bs, d_weak, d_strong);
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

hipError_t launch_signature_batch_fast(const uint8_t* d_buf, const uint64_t* d_aoff, const uint64_t* d_agb,
                                       const uint64_t* d_apfx, uint64_t nact, uint64_t nfull, const uint64_t* d_loff,
                                       const uint64_t* d_llen, const uint64_t* d_lidx, uint64_t npart, uint64_t bs,
                                       uint32_t* d_weak, uint64_t* d_strong, hipStream_t s, Profiler* prof) {
    if (nfull) {
        ProfScope ps(prof, s, "k_sig_fast_batch");
        hipLaunchKernelGGL(k_sig_fast_batch, dim3(grid_for((nfull + 3) / 4 * 64, 256)), dim3(256), 0, s, d_buf, d_aoff,
                           d_agb, d_apfx, nact, nfull, (uint32_t)bs, d_weak, d_strong);
        if (hipError_t e = hipGetLastError()) return e;
    }
    if (npart) {
        ProfScope ps(prof, s, "k_sig_list");
        hipLaunchKernelGGL(k_sig_list, dim3(grid_for(npart * 64, 256)), dim3(256), 0, s, d_buf, d_loff, d_llen, d_lidx,
                           npart, d_weak, d_strong);
    }
    return hipGetLastError();
}

hipError_t launch_ribbon_build(const DeviceIndex& ix, hipStream_t s, Profiler* prof, const uint32_t* keys,
                               uint64_t nkeys) {
    if (!ix.rib_l1 || !ix.rib_keys || ix.nfiles != 1) return hipErrorInvalidValue;
    if (!keys) {  // the exact table's slots (kEmptyKey: free)
        keys = ix.keys;
        nkeys = ix.nslots;
    }
    hipError_t e;
    if ((e = hipMemsetAsync(ix.rib_cnt, 0, 4 * (kRibShards + 1), s))) return e;
    if ((e = hipMemsetAsync(ix.rib_l1, 0, 4 * (size_t)kL1WordsR, s))) return e;
    ProfScope ps(prof, s, "k_ribbon_build");  // listing + solving
    const uint64_t per = std::max<uint64_t>(4096, (nkeys + 127) / 128);  // 128 workgroups
    hipLaunchKernelGGL(k_ribbon_list, dim3((uint32_t)((nkeys + per - 1) / per)), dim3(kRibListT), 0, s, keys, nkeys,
                       per, ix.rib_keys, ix.rib_cnt, ix.rib_over);
    if ((e = hipGetLastError())) return e;
    hipLaunchKernelGGL(k_ribbon_build, dim3(kRibShards), dim3(64), 0, s, ix.rib_keys, ix.rib_cnt, ix.rib_over,
                       ix.rib_l1);
    return hipGetLastError();
}

// The level-1 filter's bits (as k_idx_insert sets them), for an index built without its extras
__global__ void k_idx_l1(const uint32_t* __restrict__ weak, uint64_t n, uint32_t* __restrict__ l1, uint32_t l1_wshift) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ProbeHash h = probe_hash(weak[i]);
    atomicOr(l1 + (l1_wshift == 1 ? (size_t)l1r_word(h.q) : (size_t)(h.q >> l1_wshift)), 1u << (h.q & 31));
}

hipError_t launch_index_extras(const uint32_t* d_weak, const DeviceIndex& ix, hipStream_t s, Profiler* prof) {
    hipError_t e;
    if (!ix.l1 || !ix.nblocks) return hipSuccess;
    ProfScope ps(prof, s, "k_idx_extras");
    if ((e = hipMemsetAsync(ix.l1, 0, l1_total_words(ix.l1_wshift) * 4, s))) return e;
    hipLaunchKernelGGL(k_idx_l1, dim3(grid_for(ix.nblocks, 256)), dim3(256), 0, s, d_weak, ix.nblocks, ix.l1,
                       ix.l1_wshift);
    if ((e = hipGetLastError())) return e;
    if (ix.fat)
        hipLaunchKernelGGL(k_idx_fat, dim3(grid_for(ix.nslots, 256)), dim3(256), 0, s, (uint64_t)ix.nslots, ix.keys,
                           ix.cnt, ix.start, ix.order, ix.cstrong, ix.fat);
    return hipGetLastError();
}

hipError_t launch_index_build(const uint32_t* d_weak, const uint64_t* d_strong, DeviceIndex& ix, hipStream_t s,
                              Profiler* prof, bool extras) {
    hipError_t e;
    if ((e = hipMemsetAsync(ix.filt, 0, ix.fwords * 4, s))) return e;
    if (extras && ix.l1 && (e = hipMemsetAsync(ix.l1, 0, l1_total_words(ix.l1_wshift) * 4, s))) return e;
    if ((e = hipMemsetAsync(ix.keys, 0xFF, ix.nslots * 4, s))) return e;
    const uint64_t n = ix.nblocks;
    if (n == 0) return hipSuccess;
    {
        ProfScope ps(prof, s, "k_idx_insert");
        hipLaunchKernelGGL(k_idx_insert, dim3(grid_for(n, 256)), dim3(256), 0, s, d_weak, n, ix.d_fblk,
                           (uint32_t)ix.nfiles, ix.d_files, ix.filt, extras ? ix.l1 : nullptr, ix.l1_wshift, ix.keys,
                           ix.cnt, ix.slot_of);
    }
    {
        // order = block indices stably sorted by slot (keys slot_of, scratch: fill / cstrong)
        ProfScope ps(prof, s, "k_idx_order");
        uint32_t* iota = (uint32_t*)ix.cstrong;              // n u32 (cstrong holds n u64)
        uint32_t* keys_out = ix.fill;                        // nslots >= n u32
        hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256)), dim3(256), 0, s, iota, n);
        if ((e = hipGetLastError())) return e;
        int end_bit = 1;
        while (end_bit < 32 && (1ull << end_bit) < ix.nslots) ++end_bit;
        size_t tmp2 = 0;
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp2, ix.slot_of, keys_out, iota, ix.order, (int)n, 0,
                                                    end_bit, s)))
            return e;
        void* d_t2 = nullptr;
        if ((e = dev_malloc_async(&d_t2, tmp2 ? tmp2 : 16, s))) return e;
        e = hipcub::DeviceRadixSort::SortPairs(d_t2, tmp2, ix.slot_of, keys_out, iota, ix.order, (int)n, 0, end_bit,
                                               s);
        (void)hipFreeAsync(d_t2, s);
        if (e) return e;
        hipLaunchKernelGGL(k_idx_runs, dim3(grid_for(n, 256)), dim3(256), 0, s, keys_out, n, ix.start);
        hipLaunchKernelGGL(k_idx_counts, dim3(grid_for(n, 256)), dim3(256), 0, s, keys_out, n, ix.start, ix.cnt);
        if ((e = hipGetLastError())) return e;
    }
    hipLaunchKernelGGL(k_idx_cstrong, dim3(grid_for(n, 256)), dim3(256), 0, s, n, ix.order, d_strong, ix.cstrong);
    if ((e = hipGetLastError())) return e;
    if (extras && ix.fat)
        hipLaunchKernelGGL(k_idx_fat, dim3(grid_for(ix.nslots, 256)), dim3(256), 0, s, (uint64_t)ix.nslots, ix.keys,
                           ix.cnt, ix.start, ix.order, ix.cstrong, ix.fat);
    return hipGetLastError();
}

hipError_t launch_probe(const uint8_t* d_base, const ProbeJob* d_jobs, uint32_t njobs, uint64_t nprobes,
                        uint32_t stride, uint32_t n, bool fast, const DeviceIndex& ix, uint32_t* d_pw,
                        uint64_t* d_pst, uint32_t* d_out, hipStream_t s, Profiler* prof, int phases) {
    if (!nprobes) return hipSuccess;
    if (fast && (n % 64 != 0 || n < 256)) return hipErrorInvalidValue;
    if (phases & 1) {
        ProfScope ps(prof, s, stride > 1 ? "k_probe_sample" : "k_probe");
        if (fast)
            hipLaunchKernelGGL(k_probe_rows<true>, dim3(grid_for((nprobes + 3) / 4 * 64, 256)), dim3(256), 0, s,
                               d_base, d_jobs, njobs, nprobes, stride, n, d_pw, d_pst);
        else if (n % 64 == 0 && n >= 256)  // any alignment: funnel-shifted row loads
            hipLaunchKernelGGL(k_probe_rows<false>, dim3(grid_for((nprobes + 3) / 4 * 64, 256)), dim3(256), 0, s,
                               d_base, d_jobs, njobs, nprobes, stride, n, d_pw, d_pst);
        else
            hipLaunchKernelGGL(k_probe, dim3(grid_for(nprobes * 64, 256)), dim3(256), 0, s, d_base, d_jobs, njobs,
                               nprobes, stride, n, d_pw, d_pst);
    }
    if (hipError_t e = hipGetLastError()) return e;
    if (!(phases & 2)) return hipSuccess;
    ProfScope ps(prof, s, "k_probe_lookup");
    hipLaunchKernelGGL(k_probe_lookup, dim3(grid_for(nprobes, 256)), dim3(256), 0, s, d_jobs, njobs, nprobes,
                       ix.d_files, ix.filt, ix.keys, ix.start, ix.cnt, ix.order, ix.cstrong, d_pw, d_pst, d_out);
    return hipGetLastError();
}

size_t scan_lds_bytes(uint32_t n, uint32_t* nchunks_out) {
    const uint32_t nch = (uint32_t)((kScanTile + (uint64_t)n + 63) / 64) + 1;
    *nchunks_out = nch;
    const size_t pj_off = (((size_t)2 * (nch + 1) * 4) + 15) & ~(size_t)15;
    const size_t q_off = (pj_off + (size_t)(nch + 1) * 8 + 15) & ~(size_t)15;
    return q_off + (size_t)(kScanThreads / 64) * (kFQ + kWQ) * sizeof(uint2);
}

uint64_t scan_tile_positions() { return kTile2; }
uint32_t scan_max_window() { return kMaxN2; }
size_t scan_queue_entries() { return (size_t)kWgPerCuMax2 * 256 * (kT2 / 64) * kGFQ; }

hipError_t launch_scan(const uint8_t* d_buf, const ScanSeg* d_segs, uint32_t nsegs, uint32_t ntiles, uint32_t n,
                       const DeviceIndex& ix, const uint64_t* d_strong, uint64_t* d_hit_key, uint32_t* d_hit_val,
                       uint64_t out_cap, unsigned long long* d_counters, uint2* gfq, size_t gfq_cap, hipStream_t s,
                       Profiler* prof, DevScratch* scratch) {
    if (n == 0) return hipErrorInvalidValue;
    // the register-fed scans' scratch: the caller's kept buffer (grown here), else one
    // allocation per call (freeing ~100-200 MB per call blocked the host 0.3-0.6 ms, round 3)
    auto scratch_get = [&](size_t bytes, void** p) -> hipError_t {
        if (!scratch) return dev_malloc_async(p, bytes, s);
        if (scratch->bytes < bytes) {
            if (scratch->p) (void)hipFreeAsync(scratch->p, s);
            scratch->p = nullptr;
            scratch->bytes = 0;
            const size_t b = bytes + bytes / 4;
            if (hipError_t e = dev_malloc_async(&scratch->p, b, s)) return e;
            scratch->bytes = b;
        }
        *p = scratch->p;
        return hipSuccess;
    };
    auto scratch_put = [&](void* p) -> hipError_t { return scratch ? hipSuccess : hipFreeAsync(p, s); };
    if (n > kMaxN2 && !(ix.l1 && ix.l1_wshift == 1 && ix.fat && ix.nfiles == 1)) return hipErrorInvalidValue;
    if (ntiles == 0) return hipSuccess;
    ScanArgs a{};
    a.src = d_buf;
    a.n = n;
    a.nm = n % kMod;
    static const bool timing = getenv("SYDELTA_PHASE_TIMING") != nullptr;
    a.timing = timing ? 1u : 0u;
    a.segs = d_segs;
    a.nsegs = nsegs;
    a.ntiles = ntiles;
    a.files = ix.d_files;
    a.filt = ix.filt;
    a.keys = ix.keys;
    a.start = ix.start;
    a.cnt = ix.cnt;
    a.order = ix.order;
    a.cstrong = ix.cstrong;
    a.hit_key = d_hit_key;
    a.hit_val = d_hit_val;
    a.out_cap = out_cap;
    a.counters = d_counters;
    a.l1 = ix.l1;
    a.fat = ix.fat;
    // k_scan_g: one file with a level-1 filter (more than kLdsFilterKeys blocks, or windows
    // above the LDS-staged layouts) at any n but 4096, or (kSmall) indexes whose file
    // filters are <= kSmallWords words at any n <= kMaxN2; weak hits verified by k_verify_w
    const bool small_off = getenv("SYDELTA_SCAN_SMALL") && getenv("SYDELTA_SCAN_SMALL")[0] == '0';  // (per call)
    const bool small = !ix.l1 && ix.max_fwords <= kSmallWords && n <= kMaxN2 && !small_off;
    // small indexes at n = 4096 with filters <= kSmallWordsR words: k_scan_r's small mode
    // (windows verified from the registers, no deferred list)
    const bool small_r = small && n == kMaxN3 && ix.max_fwords <= kSmallWordsR;
    if ((ix.l1 && ix.l1_wshift == 1 && ix.fat && ix.nfiles == 1 && n != kMaxN3) || (small && !small_r)) {
        static std::once_flag g_once;
        static hipError_t g_err = hipSuccess;
        static int g_cus = 256;
        std::call_once(g_once, [] {
            for (const void* f : {(const void*)k_scan_g<false, false>, (const void*)k_scan_g<true, false>,
                                  (const void*)k_scan_g<false, true>})
                if (g_err == hipSuccess)
                    g_err = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
            int dev = 0, cus = 0;
            if (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
                g_cus = cus;
        });
        if (g_err != hipSuccess) return g_err;
        const uint32_t small_words = small ? std::max<uint32_t>(ix.max_fwords, 64u) : 0u;
        const LdsG LG = ldsg_layout(small_words);
        // runs of rt host tiles: the run's first window (n bytes from global memory) <= 1/8 of
        // its reads; each workgroup a contiguous range of whole runs
        uint32_t rt = 2;
        while ((uint64_t)rt * kTile2 < 8ull * n) rt *= 2;
        uint32_t per = (uint32_t)((ntiles + (uint64_t)g_cus - 1) / (uint64_t)g_cus);
        per = (per + rt - 1) / rt * rt;
        const uint32_t grid = (uint32_t)((ntiles + (uint64_t)per - 1) / per);
        // the deferred list: one entry per 256 scanned positions, 64 Ki to 4 Mi (weak hits
        // past it are verified inside the scan); SYDELTA_WDEF_CAP overrides (tests)
        const char* we = getenv("SYDELTA_WDEF_CAP");  // (per call)
        const uint64_t wdef_env = we ? std::min<uint64_t>(strtoull(we, nullptr, 10), 1u << 22) : 0;
        a.wdef_cap = wdef_env ? wdef_env
                              : std::min<uint64_t>(1u << 22, std::max<uint64_t>(1u << 16, (uint64_t)ntiles * kTile2 / 256));
        const uint32_t verify_grid = 4 * (uint32_t)g_cus;  // k_verify_w: 4 waves per workgroup
        const size_t scan_waves = (size_t)grid * (kTR / 64);
        const size_t stage_waves = std::max(scan_waves, (size_t)verify_grid * 4);
        const size_t rec_bytes = (scan_waves * kWTR * sizeof(uint2) + 255) & ~(size_t)255;
        const size_t hst_bytes = stage_waves * kHStage * sizeof(uint4);
        const size_t dst_bytes = scan_waves * kDStage * sizeof(WDef);
        void* buf = nullptr;
        hipError_t e = scratch_get(rec_bytes + hst_bytes + dst_bytes + a.wdef_cap * sizeof(WDef), &buf);
        if (e != hipSuccess) return e;
        a.rrec = (uint2*)buf;
        a.hstage = (uint4*)((uint8_t*)buf + rec_bytes);
        a.dstage = (WDef*)((uint8_t*)buf + rec_bytes + hst_bytes);
        a.wdef = (WDef*)((uint8_t*)buf + rec_bytes + hst_bytes + dst_bytes);
        {
            ProfScope ps(prof, s, "k_scan_g");
            const dim3 gd(grid), bd(kTR);
#define LAUNCH_G(RB, SM) hipLaunchKernelGGL((k_scan_g<RB, SM>), gd, bd, LG.total, s, a, per, rt, small_words)
            if (small) LAUNCH_G(false, true);
            else if (ix.l1_ribbon) LAUNCH_G(true, false);
            else LAUNCH_G(false, false);
#undef LAUNCH_G
        }
        e = hipGetLastError();
        if (e == hipSuccess) {
            ProfScope ps(prof, s, "k_verify_w");
            hipLaunchKernelGGL(k_verify_w, dim3(verify_grid), dim3(256), 0, s, a);
            e = hipGetLastError();
        }
        const hipError_t fe = scratch_put(buf);
        return e != hipSuccess ? e : fe;
    }
    // k_scan_r: one large file at n = 4096
    if ((ix.l1 && ix.l1_wshift == 1 && n == kMaxN3) || small_r) {
        static std::once_flag r_once;
        static hipError_t r_err = hipSuccess;
        static int r_cus = 256;
        std::call_once(r_once, [] {
            for (const void* f : {(const void*)k_scan_r<false, 12>, (const void*)k_scan_r<true, 12>,
                                  (const void*)k_scan_r<false, 12, true>})
                if (r_err == hipSuccess)
                    r_err = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
            int dev = 0, cus = 0;
            if (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
                r_cus = cus;
        });
        if (r_err != hipSuccess) return r_err;
        if (!ix.fat && !small_r) return hipErrorInvalidValue;
        // 12 waves (three per SIMD, 168 VGPRs): 9.72 ms at C3 against 10.37 with 8 (round 4)
        const int waves = 12;
        const uint32_t small_words = small_r ? std::max<uint32_t>(ix.max_fwords, 64u) : 0u;
        constexpr LdsR LR = ldsr_layout();
        // one workgroup per CU over contiguous host tiles, an even number each (runs are pairs)
        uint32_t per = (uint32_t)((ntiles + (uint64_t)r_cus - 1) / (uint64_t)r_cus);
        per += per & 1;
        const uint32_t grid = (uint32_t)((ntiles + (uint64_t)per - 1) / per);
        // pass records: one wave tile per wave; then each wave's staged hits
        const size_t rec_bytes = ((size_t)grid * waves * kWTR * sizeof(uint2) + 255) & ~(size_t)255;
        void* rbuf = nullptr;
        hipError_t e = scratch_get(rec_bytes + (size_t)grid * waves * kHStage * sizeof(uint4), &rbuf);
        if (e != hipSuccess) return e;
        a.rrec = (uint2*)rbuf;
        a.hstage = (uint4*)((uint8_t*)rbuf + rec_bytes);
        {
            ProfScope ps(prof, s, "k_scan_r");
            const dim3 g(grid), b(64 * waves);
#define LAUNCH_R(RB, W) hipLaunchKernelGGL((k_scan_r<RB, W>), g, b, LR.total, s, a, per, 0u)
            if (small_r)
                hipLaunchKernelGGL((k_scan_r<false, 12, true>), g, b, LR.total, s, a, per, small_words);
            else if (ix.l1_ribbon)
                LAUNCH_R(true, 12);
            else
                LAUNCH_R(false, 12);
#undef LAUNCH_R
        }
        e = hipGetLastError();
        const hipError_t fe = scratch_put(rbuf);
        return e != hipSuccess ? e : fe;
    }
    const bool lds_filter = ix.max_fwords <= kLdsFilterWordsMax;
    const uint32_t lds_fwords = lds_filter ? std::max<uint32_t>(ix.max_fwords, 4u) : 0u;
    const Lds2 L = lds2_layout(n, lds_fwords);
    // dynamic LDS above 64 KiB must be opted into
    static std::once_flag attr_once;
    static hipError_t attr_err = hipSuccess;
    static int num_cus = 256;
    std::call_once(attr_once, [] {
        const int cap = 160 * 1024 / 2 - 512;
        attr_err = hipFuncSetAttribute((const void*)k_scan_lds<true>, hipFuncAttributeMaxDynamicSharedMemorySize, cap);
        if (attr_err == hipSuccess)
            attr_err = hipFuncSetAttribute((const void*)k_scan_lds<false, 3, true>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, cap);
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            num_cus = cus;
    });
    if (attr_err != hipSuccess) return attr_err;
    if (L.total > 160u * 1024 / 2 - 512) return hipErrorInvalidValue;
    // persistent: 2-4 workgroups per CU, as many as the LDS layout allows (launch
    // bounds hold the LDS-filter kernel to 3 waves per SIMD, the other to 4), each on a
    // contiguous range of tiles
    // global-filter mode: 3 workgroups per CU (the row-parallel LDS verification
    // needs ~160 VGPRs; 4 per CU spills); LDS-filter mode: as many as the LDS fits
    const uint32_t wg_per_cu = !lds_filter ? 3u
                               : L.total <= 160u * 1024 / 3 - 512           ? 3u
                                                                            : 2u;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)num_cus * wg_per_cu);
    const uint32_t per = (ntiles + grid - 1) / grid;
    if (per >= (1u << 18)) return hipErrorInvalidValue;  // queue entries pack (tile - t_begin) in 18 bits
    // the filter-pass queues: the caller's, else from the scratch
    const size_t gfq_need = (size_t)grid * (kT2 / 64) * kGFQ;
    void* qbuf = nullptr;
    if (!gfq) {
        if (hipError_t e = scratch_get(gfq_need * sizeof(uint2), &qbuf)) return e;
        gfq = (uint2*)qbuf;
        gfq_cap = gfq_need;
    }
    if (gfq_cap < gfq_need) return hipErrorInvalidValue;
    a.gfq = gfq;
    {
        ProfScope ps(prof, s, "k_scan_lds");
        if (lds_filter)
            hipLaunchKernelGGL(k_scan_lds<true>, dim3(grid), dim3(kT2), L.total, s, a, per, lds_fwords);
        else
            hipLaunchKernelGGL((k_scan_lds<false, 3, true>), dim3(grid), dim3(kT2), L.total, s, a, per, 0u);
    }
    const hipError_t e = hipGetLastError();
    const hipError_t fe = qbuf ? scratch_put(qbuf) : hipSuccess;
    return e != hipSuccess ? e : fe;
}

hipError_t launch_scan_wide(const uint8_t* d_src, uint64_t len, uint64_t pos_begin, uint64_t pos_end, uint32_t seg_id,
                            uint32_t n, const DeviceIndex& ix, const uint64_t* d_strong, uint64_t* d_hit_key,
                            uint32_t* d_hit_val, uint64_t out_cap, unsigned long long* d_counters, hipStream_t s,
                            Profiler* prof) {
    if (ix.nfiles != 1) return hipErrorInvalidValue;
    ScanArgs a{};
    a.src = d_src;
    a.len = len;
    a.pos_begin = pos_begin;
    a.pos_end = pos_end;
    a.seg_id = seg_id;
    a.n = n;
    a.nm = n % kMod;
    a.c0 = 2 * kMod - 1 - (uint32_t)((255ull * a.nm) % kMod);
    a.fwshift = ix.files[0].fwshift;
    a.bmask = ix.files[0].bmask;
    a.filt = ix.filt;
    a.keys = ix.keys;
    const size_t lds = scan_lds_bytes(n, &a.nchunks);
    a.start = ix.start;
    a.cnt = ix.cnt;
    a.order = ix.order;
    a.cstrong = ix.cstrong;
    a.hit_key = d_hit_key;
    a.hit_val = d_hit_val;
    a.out_cap = out_cap;
    a.counters = d_counters;
    const uint64_t tiles = (pos_end - pos_begin + kScanTile - 1) / kScanTile;
    ProfScope ps(prof, s, "k_scan");
    hipLaunchKernelGGL(k_scan, dim3((unsigned)tiles), dim3(kScanThreads), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_sort_hits(uint64_t* key, uint32_t* val, uint64_t* key_tmp, uint32_t* val_tmp, uint64_t nhits,
                            int end_bit, hipStream_t s, uint64_t** key_out, uint32_t** val_out) {
    *key_out = key;
    *val_out = val;
    if (nhits <= 1) return hipSuccess;
    size_t tmp = 0;
    hipError_t e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, key, key_tmp, val, val_tmp, (int)nhits, 0, end_bit, s)))
        return e;
    void* d_t = nullptr;
    if ((e = dev_malloc_async(&d_t, tmp ? tmp : 16, s))) return e;
    e = hipcub::DeviceRadixSort::SortPairs(d_t, tmp, key, key_tmp, val, val_tmp, (int)nhits, 0, end_bit, s);
    (void)hipFreeAsync(d_t, s);
    *key_out = key_tmp;
    *val_out = val_tmp;
    return e;
}

hipError_t launch_zstd_blocks(const uint8_t* d_text, uint64_t len, uint64_t b0, uint32_t nb, uint8_t* d_slots,
                              uint8_t* d_lz, uint32_t* d_size, uint32_t* d_type, uint64_t* d_len64,
                              hipStream_t s, Profiler* prof) {
    if (!nb) return hipSuccess;
    if (b0 * zstd::kBlockMax >= len) return hipErrorInvalidValue;
    static const bool timing = getenv("SYDELTA_PHASE_TIMING") != nullptr;
    ProfScope ps(prof, s, "k_zstd_block");
    hipLaunchKernelGGL(k_zstd_block, dim3(nb), dim3(kZT), 0, s, d_text, len, b0, d_slots, d_lz, (uint64_t)nb, d_size,
                       d_type, d_len64, timing ? 1u : 0u);
    return hipGetLastError();
}

// SYDELTA_PHASE_TIMING: k_zstd_block's phase ticks so far (8 entries, 100 MHz), then zeroed.
hipError_t zstd_phase_ticks(unsigned long long* out) {
    if (hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zstd_phase), sizeof(unsigned long long) * 16)) return e;
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_zstd_phase), z, sizeof z);
}

hipError_t launch_zstd_frame(const uint8_t* d_text, uint64_t len, uint64_t b0, uint32_t nb, uint64_t nblocks,
                             const uint8_t* d_slots, const uint32_t* d_size, const uint32_t* d_type, const uint64_t* d_off,
                             uint64_t base, uint8_t* d_out, hipStream_t s, Profiler* prof) {
    if (!nb) return hipSuccess;
    ProfScope ps(prof, s, "k_zstd_frame");
    hipLaunchKernelGGL(k_zstd_frame, dim3(nb), dim3(kZT), 0, s, d_text, len, b0, nblocks, d_slots, d_size, d_type,
                       d_off, base, d_out);
    return hipGetLastError();
}

// u32 exclusive sum of n items (d_in may equal d_out).
static hipError_t exclusive_sum_u32(const uint32_t* d_in, uint32_t* d_out, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    size_t tmp = 0;
    hipError_t e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d_in, d_out, (int)n, s))) return e;
    void* d_t = nullptr;
    if ((e = dev_malloc_async(&d_t, tmp ? tmp : 16, s))) return e;
    e = hipcub::DeviceScan::ExclusiveSum(d_t, tmp, d_in, d_out, (int)n, s);
    (void)hipFreeAsync(d_t, s);
    return e;
}

hipError_t launch_chain(const chain::ChainArgs& a, hipStream_t s, Profiler* prof) {
    // u32 node indices, int item counts for hipcub, grids of < 2^31 blocks
    if (a.M + 2 >= (1ull << 31) || a.nblk + 1 >= (1ull << 31) || a.K == 0 || a.K > 32) return hipErrorInvalidValue;
    if ((1ull << a.K) <= a.M + 1) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_chain");
    const uint64_t W = a.M + 2;
    hipError_t e;
    if ((e = hipMemsetAsync(a.res, 0, sizeof(chain::ChainResult), s))) return e;
    if (a.probed) {
        hipLaunchKernelGGL(k_chain_flag, dim3(grid_for(a.nblk + 1, 256)), dim3(256), 0, s, a);
        if ((e = exclusive_sum_u32(a.aflag, a.apfx, a.nblk + 1, s))) return e;
        if (a.nblk) hipLaunchKernelGGL(k_chain_place_aligned, dim3(grid_for(a.nblk, 256)), dim3(256), 0, s, a);
    }
    if (a.H) hipLaunchKernelGGL(k_chain_place_scan, dim3(grid_for(a.H, 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_chain_succ, dim3(grid_for(W, 256)), dim3(256), 0, s, a);
    for (uint32_t l = 0; l + 1 < a.K; ++l) hipLaunchKernelGGL(k_chain_lift, dim3(grid_for(W, 256)), dim3(256), 0, s, a, l);
    if ((e = hipMemsetAsync(a.on, 0, W, s))) return e;
    hipLaunchKernelGGL(k_chain_entry, dim3(1), dim3(64), 0, s, a);
    for (uint32_t l = a.K; l-- > 0;) hipLaunchKernelGGL(k_chain_mark, dim3(grid_for(W, 256)), dim3(256), 0, s, a, l);
    hipLaunchKernelGGL(k_chain_count, dim3(grid_for(a.M + 1, 256)), dim3(256), 0, s, a);
    if ((e = exclusive_sum_u32(a.cnt, a.off, a.M + 1, s))) return e;
    if (a.M) hipLaunchKernelGGL(k_chain_emit, dim3(grid_for(a.M, 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_chain_finish, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tail(const uint8_t* d_buf, const TailJob* d_jobs, uint32_t njobs, const uint32_t* d_weak,
                       const uint64_t* d_strong, int* d_flag, hipStream_t s) {
    if (!njobs) return hipSuccess;
    hipLaunchKernelGGL(k_tail, dim3(grid_for((uint64_t)njobs * 64, 256)), dim3(256), 0, s, d_buf, d_jobs, njobs, d_weak,
                       d_strong, d_flag);
    return hipGetLastError();
}

hipError_t launch_apply(const ApplyPiece* d_pieces, uint64_t npieces, const uint8_t* d_basis, const uint8_t* d_lit,
                        uint8_t* d_out, hipStream_t s, Profiler* prof) {
    if (!npieces) return hipSuccess;
    ProfScope ps(prof, s, "k_apply");
    for (uint64_t p0 = 0; p0 < npieces; p0 += 0x7FFFFFFFull) {
        const uint64_t cnt = std::min<uint64_t>(npieces - p0, 0x7FFFFFFFull);
        hipLaunchKernelGGL(k_apply, dim3((unsigned)cnt), dim3(256), 0, s, d_pieces + p0, d_basis, d_lit, d_out);
    }
    return hipGetLastError();
}

hipError_t launch_json_len(const JsonPiece* d_pieces, uint64_t npieces, const uint8_t* d_lit, uint64_t* d_len,
                           hipStream_t s, Profiler* prof) {
    if (!npieces) return hipSuccess;
    if (npieces > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_json_len");
    hipLaunchKernelGGL(k_json_len, dim3(grid_for(npieces * 64, 256)), dim3(256), 0, s, d_pieces, npieces, d_lit,
                       d_len);
    return hipGetLastError();
}

hipError_t launch_json_write(const JsonPiece* d_pieces, uint64_t npieces, const uint8_t* d_lit,
                             const uint64_t* d_off, uint64_t base, uint8_t* d_out, hipStream_t s, Profiler* prof) {
    if (!npieces) return hipSuccess;
    if (npieces > 0x7FFFFFFFull) return hipErrorInvalidValue;
    static std::once_flag once;
    static hipError_t attr = hipSuccess;
    std::call_once(once, [] {
        attr = hipFuncSetAttribute((const void*)k_json_write, hipFuncAttributeMaxDynamicSharedMemorySize, kJsonStage);
    });
    if (attr != hipSuccess) return attr;
    ProfScope ps(prof, s, "k_json_write");
    hipLaunchKernelGGL(k_json_write, dim3((unsigned)npieces), dim3(256), kJsonStage, s, d_pieces, d_lit, d_off, base,
                       d_out);
    return hipGetLastError();
}

hipError_t launch_sigjson_len(const sigjson::SigArgs& a, uint64_t* d_tile_len, hipStream_t s, Profiler* prof) {
    const uint64_t nt = (a.n + sigjson::kTile - 1) / sigjson::kTile;
    if (!nt) return hipSuccess;
    if (nt > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_sigjson_len");
    hipLaunchKernelGGL(k_sigjson_len, dim3((unsigned)nt), dim3(sigjson::kTile), 0, s, a, d_tile_len);
    return hipGetLastError();
}

hipError_t launch_sigjson_write(const sigjson::SigArgs& a, const uint64_t* d_tile_off, uint8_t* d_out, hipStream_t s,
                                Profiler* prof) {
    const uint64_t nt = (a.n + sigjson::kTile - 1) / sigjson::kTile;
    if (!nt) return hipSuccess;
    if (nt > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_sigjson_write");
    hipLaunchKernelGGL(k_sigjson_write, dim3((unsigned)nt), dim3(sigjson::kTile), 0, s, a, d_tile_off, d_out);
    return hipGetLastError();
}

hipError_t launch_sigparse_count(const uint8_t* d_text, uint64_t len, uint64_t* d_count, hipStream_t s, Profiler* prof) {
    const uint64_t nc = (len + sigjson::kParseChunk - 1) / sigjson::kParseChunk;
    if (!nc) return hipSuccess;
    if ((nc + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_sigparse_count");
    hipLaunchKernelGGL(k_sigparse_count, dim3(grid_for(nc, 256)), dim3(256), 0, s, d_text, len, d_count);
    return hipGetLastError();
}

hipError_t launch_sigparse(const uint8_t* d_text, uint64_t len, const uint64_t* d_rank, sydelta_block_checksum* d_out,
                           uint64_t cap, unsigned long long* d_bad, hipStream_t s, Profiler* prof) {
    const uint64_t nc = (len + sigjson::kParseChunk - 1) / sigjson::kParseChunk;
    if (!nc) return hipSuccess;
    if ((nc + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_sigparse");
    hipLaunchKernelGGL(k_sigparse, dim3(grid_for(nc, 256)), dim3(256), 0, s, d_text, len, d_rank, d_out, cap, d_bad);
    return hipGetLastError();
}

hipError_t launch_dparse_count(const dparse::DArgs& a, uint64_t* d_ocnt, uint64_t* d_lcnt, hipStream_t s,
                               Profiler* prof) {
    if (!a.nc) return hipSuccess;
    if ((a.nc + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_dparse_count");
    hipLaunchKernelGGL(k_dparse_count, dim3(grid_for(a.nc, 256)), dim3(256), 0, s, a, d_ocnt, d_lcnt);
    return hipGetLastError();
}

hipError_t launch_dparse_place(const dparse::DArgs& a, const uint64_t* d_orank, uint64_t* d_pos, hipStream_t s,
                               Profiler* prof) {
    if (!a.nc) return hipSuccess;
    if ((a.nc + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_dparse_place");
    hipLaunchKernelGGL(k_dparse_place, dim3(grid_for(a.nc, 256)), dim3(256), 0, s, a, d_orank, d_pos);
    return hipGetLastError();
}

hipError_t launch_dparse(const dparse::DArgs& a, const uint64_t* d_orank, const uint64_t* d_lrank, const uint64_t* d_pos,
                         uint64_t nops, sydelta_op* d_ops, uint8_t* d_lit, unsigned long long* d_bad, hipStream_t s,
                         Profiler* prof) {
    if (!a.nc) return hipSuccess;
    if ((a.nc + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_dparse");
    hipLaunchKernelGGL(k_dparse, dim3(grid_for(a.nc, 256)), dim3(256), 0, s, a, d_orank, d_lrank, d_pos, nops, d_ops,
                       d_lit, d_bad);
    return hipGetLastError();
}

// 64-bit exclusive sum (the text of a multi-GiB literal run overflows 32-bit offsets;
// hipcub accumulates in the input type, so the input is 64-bit too).
hipError_t launch_exclusive_sum_u64(const uint64_t* d_in, uint64_t* d_out, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    size_t tmp = 0;
    hipError_t e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d_in, d_out, (int)n, s))) return e;
    void* d_t = nullptr;
    if ((e = dev_malloc_async(&d_t, tmp ? tmp : 16, s))) return e;
    e = hipcub::DeviceScan::ExclusiveSum(d_t, tmp, d_in, d_out, (int)n, s);
    (void)hipFreeAsync(d_t, s);
    return e;
}

hipError_t launch_block_cmp(const uint8_t* d_src, uint64_t slen, const uint8_t* d_dst, uint64_t dlen, uint64_t bs,
                            uint8_t* d_changed, hipStream_t s, Profiler* prof) {
    const uint64_t nb = (slen + bs - 1) / bs;
    if (!nb) return hipSuccess;
    ProfScope ps(prof, s, "k_block_cmp");
    hipLaunchKernelGGL(k_block_cmp, dim3((unsigned)std::min<uint64_t>(nb, 1u << 20)), dim3(256), 0, s, d_src, slen,
                       d_dst, dlen, bs, nb, d_changed);
    return hipGetLastError();
}

hipError_t launch_hash_blocks(const uint8_t* d_buf, uint64_t len, uint64_t bs, const uint64_t* d_pos, uint32_t count,
                              uint64_t* d_out, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_hash_blocks, dim3(grid_for((uint64_t)count * 64, 256)), dim3(256), 0, s, d_buf, len, bs, d_pos,
                       count, d_out);
    return hipGetLastError();
}

hipError_t launch_xxh_files(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len, const uint64_t* d_pfx,
                            const uint64_t* d_aoff, const uint64_t* d_apfx, uint64_t nact, const uint32_t* d_order,
                            uint64_t nfiles, uint64_t npieces, uint64_t* d_C, uint64_t* d_out,
                            hipStream_t s, Profiler* prof) {
    if (!nfiles) return hipSuccess;
    const uint64_t cstride = xxh_chain_records(npieces);
    if (npieces) {
        ProfScope ps(prof, s, "k_xxh_pieces");
        hipLaunchKernelGGL(k_xxh_pieces, dim3(grid_for((npieces + kPieceRows - 1) / kPieceRows * 16, 256)), dim3(256),
                           0, s, d_buf, d_aoff, d_apfx, nact, npieces, cstride, d_C);
        if (hipError_t e = hipGetLastError()) return e;
    }
    ProfScope ps(prof, s, "k_xxh_chain");
    hipLaunchKernelGGL(k_xxh_chain, dim3((unsigned)((nfiles + 7) / 8)), dim3(64), 0, s, d_buf, d_off, d_len, d_pfx,
                       d_order, nfiles, cstride, d_C, d_out);
    return hipGetLastError();
}

hipError_t launch_synth_fill(uint8_t* d_buf, uint64_t len, uint64_t seed, hipStream_t s, uint64_t first) {
    if (!len) return hipSuccess;
    if (first % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_synth_fill, dim3(4096), dim3(256), 0, s, d_buf, len, seed, first / 8);
    return hipGetLastError();
}

hipError_t launch_synth_edit_blocks(uint8_t* d_dst, uint64_t len, uint64_t bs, uint64_t first, uint64_t seed,
                                    uint32_t rate_ppm, hipStream_t s) {
    if (!len) return hipSuccess;
    if (!bs || first % bs) return hipErrorInvalidValue;
    const uint64_t nb = (len + bs - 1) / bs;
    const uint64_t thresh = (uint64_t)(((unsigned __int128)rate_ppm << 32) / 1000000u);
    hipLaunchKernelGGL(k_synth_edit_blocks, dim3(grid_for(nb, 256)), dim3(256), 0, s, d_dst, len, bs, first / bs, nb,
                       seed, thresh);
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
