// sydelta_chain.hpp — K5b: the greedy walk of generator.rs:116-221 (:283-379) resolved on
// the device (SURVEY.md §2 K5 `resolve_chain`).
//
// After classification every full-window position of a source is known to hit (first
// block in index order with equal weak and strong) or not: the aligned hits of k_probe
// (one per block) and the scan hits (sorted positions).  The walk from x takes the first
// hit p >= x, emits Data[lit, p) and Copy(block of p), and continues at p + n
// (generator.rs:144).  So hit i has one successor, succ(i) = the first hit at or after
// pos_i + n: a forest whose edges point forward, and the walk is the path from the
// entry's first hit.  One source is resolved in four data-parallel steps:
//   1. merge: the aligned hits and the scan hits into one ascending list U (an aligned
//      hit's rank = its index among the aligned hits + the scan hits before it, a binary
//      search; a scan hit's = its index + the aligned hits before it, a prefix lookup);
//   2. succ: a binary search in U for pos + n; END past the source; UNK when pos + n lies
//      inside a probed block none of whose interior was scanned (the host walk then
//      scans that block on demand, so the device result is discarded: walk_src's
//      first_unknown);
//   3. path: pointer jumping, J_{k+1} = J_k o J_k, then for k = K-1 .. 0 every marked
//      hit marks J_k of itself, which marks f^t(first) for every t < 2^K;
//   4. ops: each marked hit emits Copy and, when its successor is a hit further than
//      pos + n, the literal run between them; an exclusive scan of the counts places them.
// The host adds the leading literal run (entry .. first hit) and the end of the walk
// (walk::finish_walk: the last literal run, or the tail rule of a final source).
//
// Every function below is the body of one thread of one kernel (sydelta_kernels.hip,
// launch_chain).  The host emulation of the device layer (tests/csrc/fake_device.cpp)
// runs the same bodies in loops, so the CPU suite checks them against the host walk.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sydelta.h"

namespace sydelta {
namespace chain {

constexpr uint32_t kNoHit = 0xFFFFFFFFu;  // k_probe: the aligned window did not hit

// Per-call outputs gathered by chain_finish (one D2H).
struct ChainResult {
    uint64_t nops;       // ops written to ChainArgs::ops
    uint64_t data_ops;   // of which Data
    uint64_t lit_bytes;  // their bytes
    uint64_t first_pos;  // position of the path's first hit (valid when first < M)
    uint64_t last_pos;   // position of its last hit
    uint64_t first, last;  // indices into U (M when the path is empty)
    uint32_t unk;        // the path reached an unclassified position: discard
    uint32_t bad;        // an index fell outside its array (inputs inconsistent): discard
};

struct ChainArgs {
    // the source (positions are those of walk::Src)
    uint64_t n;            // block size
    uint64_t p1;           // one past the last classified full-window position
    uint64_t kb, nblk;     // blocks kb .. kb+nblk-1 cover [p0, p1)
    uint64_t entry;        // where the walk starts (entry < p1)
    uint32_t probed;       // ahit/known/apfx valid
    uint32_t K;            // pointer-jumping levels: 2^K > M + 1
    const uint32_t* ahit;  // per local block: its aligned window's global block or kNoHit
    const uint8_t* known;  // per local block: every window start of it was scanned (walk::Src::scanned)
    uint32_t* aflag;       // nblk + 1: aligned-hit flags (scratch)
    uint32_t* apfx;        // nblk + 1: their exclusive prefix
    const uint64_t* hpos;  // scan hits, ascending, none at an aligned position that hit
    const uint32_t* hblk;
    uint64_t H;
    // U and the forest
    uint64_t M;            // |U| = aligned hits + H
    uint64_t* upos;
    uint32_t* ublk;
    uint32_t* jump;        // K levels of M + 2 entries; index M = END, M + 1 = UNK
    uint8_t* on;           // M + 2: on the path
    uint32_t* cnt;         // M + 1: ops per hit (cnt[M] = 0)
    uint32_t* off;         // M + 1: exclusive prefix of cnt
    // the basis file the Copies name
    uint64_t blk_base, nblocks, last_size;
    sydelta_op* ops;       // <= 2M ops
    ChainResult* res;
};

__host__ __device__ __forceinline__ bool known_block(const ChainArgs& a, uint64_t k) { return a.known[k] != 0; }

// A position x < p1 the walk may stand on without its class being known: inside a
// probed block (not its aligned start) none of whose window starts was scanned.  Such a
// block's aligned window hit (classify scans every block that missed), so a literal run
// that starts before the block reaches the aligned hit first; only a jump lands inside.
__host__ __device__ __forceinline__ bool unknown_at(const ChainArgs& a, uint64_t x) {
    return a.probed && x < a.p1 && x % a.n != 0 && !known_block(a, x / a.n - a.kb);
}

// First index of U with upos >= x (M if none).
__host__ __device__ __forceinline__ uint64_t lower_bound_u(const ChainArgs& a, uint64_t x) {
    uint64_t lo = 0, hi = a.M;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.upos[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// First index >= lo of U with upos >= x (M if none), for x > upos[lo - 1]: a galloping
// search from lo (a successor is usually the next hit or one close to it, so this reads a
// line or two where a binary search over U would make ~log2 M dependent reads).
__host__ __device__ __forceinline__ uint64_t lower_bound_from(const ChainArgs& a, uint64_t lo, uint64_t x) {
    uint64_t step = 1, hi = lo;
    while (hi < a.M && a.upos[hi] < x) {
        lo = hi + 1;
        hi = lo + step - 1 < a.M ? lo + step - 1 : a.M;
        step <<= 1;
    }
    // upos[lo - 1] < x (or lo is the start) and (hi == M or upos[hi] >= x): binary search [lo, hi)
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.upos[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Scan hits strictly before x.
__host__ __device__ __forceinline__ uint64_t scan_hits_before(const ChainArgs& a, uint64_t x) {
    uint64_t lo = 0, hi = a.H;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.hpos[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Step 1a (k < nblk + 1): the aligned-hit flags the exclusive scan turns into apfx.
__host__ __device__ __forceinline__ void chain_flag(const ChainArgs& a, uint64_t k) {
    a.aflag[k] = (k < a.nblk && a.ahit[k] != kNoHit) ? 1u : 0u;
}

// Step 1b (k < nblk): aligned hit of local block k into U.
__host__ __device__ __forceinline__ void chain_place_aligned(const ChainArgs& a, uint64_t k) {
    if (a.ahit[k] == kNoHit) return;
    const uint64_t p = (a.kb + k) * a.n;
    const uint64_t u = a.apfx[k] + scan_hits_before(a, p);
    if (u >= a.M) { a.res->bad = 1; return; }  // more aligned hits than the host counted
    a.upos[u] = p;
    a.ublk[u] = a.ahit[k];
}

// Step 1c (h < H): scan hit h into U.  The aligned hits before position p are those of
// blocks k*n < p, i.e. local blocks below ceil(p / n) - kb.
__host__ __device__ __forceinline__ void chain_place_scan(const ChainArgs& a, uint64_t h) {
    const uint64_t p = a.hpos[h];
    uint64_t before = 0;
    if (a.probed) {
        const uint64_t kc = (p + a.n - 1) / a.n;
        const uint64_t kl = kc > a.kb ? kc - a.kb : 0;
        before = a.apfx[kl < a.nblk ? kl : a.nblk];
    }
    if (h + before >= a.M) { a.res->bad = 1; return; }
    a.upos[h + before] = p;
    a.ublk[h + before] = a.hblk[h];
}

// Step 2 (i < M + 2): level 0 of the forest.
__host__ __device__ __forceinline__ void chain_succ(const ChainArgs& a, uint64_t i) {
    const uint32_t END = (uint32_t)a.M, UNK = (uint32_t)(a.M + 1);
    if (i >= a.M) {
        a.jump[i] = (uint32_t)i;  // END and UNK absorb
        return;
    }
    const uint64_t x = a.upos[i] + a.n;  // generator.rs:144 / :313
    uint32_t s;
    if (x >= a.p1) s = END;
    else if (unknown_at(a, x)) s = UNK;
    else s = (uint32_t)lower_bound_from(a, i + 1, x);  // upos[i] < x
    a.jump[i] = s;
}

// Step 3a (i < M + 2): level l + 1 from level l.
__host__ __device__ __forceinline__ void chain_lift(const ChainArgs& a, uint32_t l, uint64_t i) {
    const uint64_t W = a.M + 2;
    const uint32_t* J = a.jump + (uint64_t)l * W;
    a.jump[(uint64_t)(l + 1) * W + i] = J[J[i]];
}

// Step 3b (one thread, after `on` is cleared): the path's first hit (entry's class
// known), or UNK/END; the result record is reset here.
__host__ __device__ __forceinline__ void chain_entry(const ChainArgs& a) {
    const uint64_t i0 = unknown_at(a, a.entry) ? a.M + 1 : lower_bound_u(a, a.entry);
    a.on[i0] = 1;
    ChainResult& r = *a.res;
    r.nops = r.data_ops = r.lit_bytes = 0;
    r.first_pos = r.last_pos = 0;
    r.first = i0 < a.M ? i0 : a.M;
    r.last = a.M;
    r.unk = 0;  // r.bad: set by the merge, cleared before the launches
}

// Step 3c (i < M + 2): level l of the marking.  A mark set by another thread of the same
// launch may or may not be seen here; either way only hits of the path get marked.
__host__ __device__ __forceinline__ void chain_mark(const ChainArgs& a, uint32_t l, uint64_t i) {
    if (a.on[i]) a.on[a.jump[(uint64_t)l * (a.M + 2) + i]] = 1;
}

// Step 4a (i < M + 1): ops of hit i on the path (Copy, then the literal gap to its
// successor when that is a hit and the gap is not empty).
__host__ __device__ __forceinline__ void chain_count(const ChainArgs& a, uint64_t i) {
    uint32_t c = 0;
    if (i < a.M && a.on[i]) {
        const uint32_t s = a.jump[i];
        c = 1u + ((s < a.M && a.upos[s] > a.upos[i] + a.n) ? 1u : 0u);
    }
    a.cnt[i] = c;
}

// Step 4b (i < M): write hit i's ops at off[i]; returns its literal bytes (data op iff > 0)
// and records the path's last hit.
__host__ __device__ __forceinline__ uint64_t chain_emit(const ChainArgs& a, uint64_t i) {
    if (!a.on[i]) return 0;
    const uint64_t o = a.off[i];
    if (o + 1 >= 2 * a.M + 1) { a.res->bad = 1; return 0; }  // ops hold 2M entries
    const uint64_t b = a.ublk[i] - a.blk_base;  // generator.rs:135-140: Copy{offset, size}
    a.ops[o] = sydelta_op{SYDELTA_OP_COPY, 0, b * a.n, (b + 1 == a.nblocks) ? a.last_size : a.n};
    const uint32_t s = a.jump[i];
    if (s == (uint32_t)a.M) {
        a.res->last = i;
        a.res->last_pos = a.upos[i];
        return 0;
    }
    if (s < a.M && a.upos[s] > a.upos[i] + a.n) {
        const uint64_t lo = a.upos[i] + a.n, len = a.upos[s] - lo;
        a.ops[o + 1] = sydelta_op{SYDELTA_OP_DATA, 0, lo, len};
        return len;
    }
    return 0;
}

// Step 5 (one thread): totals and the first hit's position.
__host__ __device__ __forceinline__ void chain_finish(const ChainArgs& a) {
    ChainResult& r = *a.res;
    r.nops = a.off[a.M];
    r.unk = a.on[a.M + 1] ? 1u : 0u;
    if (r.first < a.M) r.first_pos = a.upos[r.first];
}

// Levels for M hits: 2^K > M + 1, so every path (at most M hits, then END) is marked.
__host__ __device__ __forceinline__ uint32_t chain_levels(uint64_t M) {
    uint32_t K = 1;
    while (K < 63 && (1ull << K) <= M + 1) ++K;
    return K;
}

}  // namespace chain
}  // namespace sydelta
