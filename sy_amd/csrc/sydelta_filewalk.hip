// sydelta_filewalk.hip — K10, the whole greedy walk of each file of a batch on the device
// (C4's batched small files).  Its own translation unit: the shared device code comes from
// sydelta_kcommon.hpp.
#include "sydelta_device.hpp"
#include "sydelta_internal.hpp"

namespace sydelta {

#include "sydelta_kcommon.hpp"

// ===========================================================================
// K10: the greedy walk of many small files, one wave per file (C4)
// ===========================================================================
// The batched match used to classify on the device in five host-synchronised phases
// (aligned probe, miss ranges, scans, phase probe, scans of the missed blocks) and walk on
// host threads.  Here one wave walks its file itself (generator.rs:116-221), classifying
// only the window starts the walk visits:
//   * the walk at x on the phase grid k*n + phi: the phase windows of the next blocks are
//     hashed four at a time, one 16-lane row each (row_hash, the signature kernel's layout),
//     and looked up one per lane (first candidate in index order with equal strong,
//     generator.rs:121-155); a hit copies and moves x by n, so the walk stays on the grid;
//   * a miss at x: the window starts (x, x + n) are rolled (rolling.rs:66-79), 64 per lane
//     from the closed form of their first window (wave scans of the lanes' 64-byte group
//     sums), tested against the file's Bloom filter in LDS; the passes are hashed four at
//     a time in position order and the first verified one is the walk's next hit (a Copy,
//     then a new phase grid); without one the walk continues at x + n, the next phase window.
// A copy-heavy file costs one window hash per block plus one roll of n starts per edited
// block, and a shift (an insertion or deletion) one new phase grid.  A wave per file keeps
// the walk's steps free of workgroup barriers, and a CU holds as many files as waves (the
// first form, a workgroup of four waves per file, spent half its time waiting at barriers:
// 5.28 ms for C4's 10 000 files, `profiles/r05d_*`).  The ops are written run-length coded
// (WalkRec) to the file's staging region, then moved to the compact output with one atomic
// per file.
constexpr uint32_t kWRun = 64;          // window starts per lane per roll pass
constexpr uint32_t kWSub = 64 * kWRun;  // window starts per roll pass (4096)
constexpr uint32_t kWMaxPass = 64;      // phase windows per pass at most (one lookup per lane)

// A self-indexed unit's Bloom filter and exact table: 2^k >= 2 nb words / slots each (at least
// 64): 64 bits per key, five of them set in one word (probe_hash / filt_mask, ~1e-5 false
// passes), and the table at load <= 1/2.
__host__ __device__ __forceinline__ uint32_t self_bits(uint32_t nb) {
    uint32_t k = 6;
    while ((1u << k) < 2 * nb) ++k;
    return k;
}
struct WalkLds {  // byte offsets of the dynamic LDS (one wave per workgroup)
    uint32_t filt, ntab, pw, pst, tab, lw, total;
};
__host__ __device__ __forceinline__ WalkLds walk_lds(uint32_t self_nb) {
    WalkLds L{};
    uint32_t o = 0;
    const uint32_t fw = self_nb ? 1u << self_bits(self_nb) : 0u;
    L.filt = o; o += 4 * fw;        // self-indexed: the file's Bloom filter
    L.ntab = o; o += 1024;
    L.pw = o; o += 4 * kWMaxPass;   // a pass's weak values
    L.pst = o; o += 8 * kWMaxPass;  // ... and strong hashes
    L.tab = o; o += 4 * fw;         // self-indexed: slot -> first block (in index order) of its weak value
    L.lw = o; o += 4 * ((self_nb + 3) & ~3u);  // ... and the file's weak values
    L.total = o;
    return L;
}
// SYDELTA_PHASE_TIMING (WalkArgs::ticks): wall-clock ticks of each wave, summed
constexpr int kWtSetup = 0, kWtHash = 1, kWtLookup = 2, kWtStage = 3, kWtRoll = 4, kWtVerify = 5, kWtOut = 6;
constexpr int kWtPasses = 8, kWtWindows = 9, kWtRolls = 10, kWtVerifies = 11;

// 64 bytes of the file at byte offset off (any alignment) as 16 dwords: four dword-aligned
// 16-byte loads and one dword, funnel-shifted; near the end (where those dwords could leave
// the readable granules, sydelta.h) byte by byte, bytes at or past len read as 0.
__device__ __forceinline__ void load64_any(const uint8_t* src, uint64_t len, uint64_t off, uint32_t (&x)[16]) {
    const uint64_t a4 = off & ~3ull;
    const uint32_t sh = (uint32_t)(off & 3);
    if (a4 + 68 <= ((len + 15) & ~15ull)) {
        const uint32_t* w = (const uint32_t*)(src + a4);
        uint32_t d[17];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u32x4 v;
            __builtin_memcpy(&v, w + 4 * i, 16);
            d[4 * i] = v.x;
            d[4 * i + 1] = v.y;
            d[4 * i + 2] = v.z;
            d[4 * i + 3] = v.w;
        }
        d[16] = sh ? w[16] : 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint32_t v = 0;
        for (int j = 0; j < 4; ++j) {
            const uint64_t p = off + 4 * i + j;
            if (p < len) v |= (uint32_t)src[p] << (8 * j);
        }
        x[i] = v;
    }
}

// First candidate in index order of file F with weak wk and strong st (generator.rs:127-133),
// or kNoBlock; one lane.
__device__ __forceinline__ uint32_t walk_lookup(const WalkArgs& a, const FileIx& F, uint32_t wk, uint64_t st) {
    const int64_t slot = table_find(a.keys + F.slot_off, F.bmask, wk);
    if (slot < 0) return kNoBlock;
    const uint64_t gs = F.slot_off + (uint64_t)slot;
    const uint32_t s0 = a.start[gs], c = a.cnt[gs];
    for (uint32_t j = 0; j < c; ++j)
        if (a.cstrong[s0 + j] == st) return a.order[s0 + j];
    return kNoBlock;
}

// The same from a self-indexed unit's LDS table (tab: linear probing by bucket_hash, each slot
// the lowest block of its weak value; lw: the file's weak values): the first block in index
// order with weak wk and strong st (sg: the file's strong hashes, global) -- the slot's block,
// or, when its strong differs (a weak collision), the next block with both (generator.rs:76-81,
// 127-133); one lane.
__device__ __forceinline__ uint32_t self_lookup(const uint32_t* tab, const uint32_t* lw, uint32_t tmask,
                                                const uint64_t* sg, uint32_t nbf, uint64_t gb0, uint32_t wk,
                                                uint64_t st) {
    uint32_t s = bucket_hash(wk) & tmask, e;
    for (;;) {
        e = tab[s];
        if (e == kNoBlock) return kNoBlock;
        if (lw[e] == wk) break;
        s = (s + 1) & tmask;
    }
    for (uint32_t j = e; j < nbf; ++j)
        if (lw[j] == wk && sg[j] == st) return (uint32_t)(gb0 + j);
    return kNoBlock;
}

// One window per row (row_hash's contract).  Issuing all four pieces' loads of a 4 KiB
// window at once (one round trip instead of four) took 64 more VGPRs: two waves per SIMD
// instead of four, and the walk 5.09 ms instead of 3.59 at C4 (`profiles/r05f_*`).
template <bool kAligned>
__device__ __forceinline__ void walk_hash(const uint8_t* p, uint32_t n, uint32_t& wk, uint64_t& st) {
    row_hash<kAligned>(p, n, wk, st);
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// The suffix p[0, ls) hashes to (weak, strong): the whole wave calls; every lane returns it.
__device__ __forceinline__ bool tail_matches(const uint8_t* p, uint64_t ls, uint32_t weak, uint64_t strong) {
    uint32_t wk = 0;
    uint64_t st = 0;
    if (ls > 240) {
        wave_hash_long(p, ls, wk, st);
    } else if ((threadIdx.x & 63) == 0) {
        wk = adler_scalar(p, ls);
        st = xxh3_short(p, ls);
    }
    return __builtin_amdgcn_readlane((int)(wk == weak && st == strong ? 1u : 0u), 0) != 0;
}

// The first verified hit among the window starts (x, yend), the window at x (weak wbase)
// missed: its position in q and block in qb (else q = yend, qb = kNoBlock); weak_hits counts
// the verified windows.  The whole wave calls (k_walk_files at a miss, k_preroll per miss).
template <bool kLdsFilt, class Look, class Tick, class Count>
__device__ __forceinline__ void walk_roll(const WalkArgs& a, const FileIx& F, const uint32_t* filt,
                                          const uint32_t* ntab, const uint8_t* src, uint64_t len, uint64_t x,
                                          uint64_t yend, uint32_t wbase, uint64_t& q, uint32_t& qb,
                                          uint32_t& weak_hits, Look&& look, Tick&& wtick, Count&& wcount) {
    const uint32_t lane = threadIdx.x & 63, row = lane >> 4, n = a.n;
    q = yend;
    qb = kNoBlock;
#pragma unroll 1
    for (uint64_t y0 = x + 1; y0 < yend && qb == kNoBlock; y0 += kWSub) {
        const uint64_t y1 = min(y0 + kWSub, yend);
        const uint64_t b = y0 - 1;
        wcount(kWtRolls, 1);
        uint32_t xo[16], xi[16];  // out [b + 64l, +64), in [b + n + 64l, +64)
        load64_any(src, len, b + 64ull * lane, xo);
        load64_any(src, len, b + n + 64ull * lane, xi);
        uint32_t so = 0, si = 0, vo = 0, vi = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            so = udot4(xo[i], 0x01010101u, so);
            si = udot4(xi[i], 0x01010101u, si);
            vo = udot4(xo[i], offw(i), vo);
            vi = udot4(xi[i], offw(i), vi);
        }
        const uint32_t gc = (si + 2 * kMod - so) % kMod;                                          // sum c
        const uint32_t gj = (uint32_t)(((uint64_t)(64 * lane) * gc + vi + 16 * kMod - vo) % kMod);  // sum j c
        uint32_t tt;
        const uint32_t sC = wave_scan_excl(gc, tt);
        const uint32_t sJ = wave_scan_excl(gj, tt);
        const uint32_t sO = wave_scan_excl(so, tt);
        const uint32_t o0 = xo[0] & 0xFF, i0 = xi[0] & 0xFF;  // byte j = 64 l: the last of the first window's c_j
        const uint32_t c0 = (i0 + kMod - o0) % kMod;
        const uint32_t C = (sC % kMod + c0) % kMod;
        const uint32_t J = (uint32_t)((sJ % kMod + (uint64_t)(64 * lane) * c0) % kMod);
        const uint32_t Out = (sO + o0) % kMod;
        const uint64_t d = 64ull * lane + 1;
        const uint32_t Ab = wbase & 0xFFFFu, Bb = wbase >> 16;
        uint32_t am = (Ab + C) % kMod;
        uint32_t bm = (uint32_t)(((uint64_t)Bb + d * ((Ab + kMod - 1) % kMod) % kMod + d * C % kMod + (kMod - J) +
                                  (kMod - (uint64_t)a.nm * Out % kMod)) % kMod);
        wtick(kWtStage);
        // roll the lane's 64 window starts; a start whose weak value passes the Bloom filter
        // is a candidate
        const uint64_t p0 = y0 + 64ull * lane;
        const uint32_t nvalid = p0 >= y1 ? 0u : (uint32_t)min((uint64_t)kWRun, y1 - p0);
        // the bytes the rolls take out / in: group offsets 1..64 (offset 64 is never used)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            xo[j] = __builtin_amdgcn_alignbyte(j < 15 ? xo[j + 1] : 0u, xo[j], 1);
            xi[j] = __builtin_amdgcn_alignbyte(j < 15 ? xi[j + 1] : 0u, xi[j], 1);
        }
        uint64_t pm = 0;
        uint32_t wlast = 0;
        // a global filter (a large index: 16 bits per key, ~0.8 % of starts pass) keeps the
        // weak values of a lane's first four passes, which are looked up in the exact table
        // below before anything is hashed (8 KiB per candidate otherwise)
        uint32_t wp[4] = {0, 0, 0, 0}, wpi[4] = {0, 0, 0, 0}, np = 0;
        // sixteen starts per round from the first four dwords (their filter words loaded
        // together: a global filter's reads are L2 round trips), then the dwords move down
        // four (a loop, not unrolled: the register arrays keep constant indices)
#pragma unroll 1
        for (uint32_t t = 0; t < kWRun / 16; ++t) {
            uint32_t hq[16], fwv[16], wv[16];
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                const ProbeHash h = probe_hash(am, bm);
                hq[b] = h.q;
                fwv[b] = filt[h.r >> F.fwshift];
                wv[b] = (bm << 16) | am;
                const uint32_t out = (xo[b >> 2] >> (8 * (b & 3))) & 0xFF;
                const uint32_t in = (xi[b >> 2] >> (8 * (b & 3))) & 0xFF;
                const uint32_t u = am + in + (kMod - out);  // [M-255, 2M+255)
                am = min(u, min(u - kMod, u - 2 * kMod));
                const uint32_t v = bm + am + ntab[out];  // [0, 3M)
                bm = min(v, min(v - kMod, v - 2 * kMod));
            }
            wlast = wv[15];
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                const uint32_t i = 16 * t + b;
                const uint32_t pass = i < nvalid ? filt_bit(fwv[b], hq[b]) : 0u;
                pm |= (uint64_t)pass << i;
                if (!kLdsFilt && pass) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (np == (uint32_t)j) {
                            wp[j] = wv[b];
                            wpi[j] = i;
                        }
                    ++np;
                }
            }
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                xo[j] = xo[j + 4];
                xi[j] = xi[j + 4];
            }
        }
        wbase = rl(wlast, 63);  // the next pass's base: lane 63's last start, b + 4096
        if (!kLdsFilt) {  // exact-table lookups of the first passes (generator.rs:121-124)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((uint32_t)j < np && table_find(a.keys + F.slot_off, F.bmask, wp[j]) < 0) pm &= ~(1ull << wpi[j]);
        }
        wtick(kWtRoll);
        // verify the candidates four at a time in position order (generator.rs:121-133);
        // weak_hits counts the verified windows
#pragma unroll 1
        for (;;) {
            uint32_t cand[4], nc = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint64_t lm = __ballot(pm != 0);
                cand[r] = 0;
                if (!lm) continue;
                const uint32_t fl = (uint32_t)__builtin_ctzll(lm);
                const uint32_t lo = rl((uint32_t)pm, fl), hi = rl((uint32_t)(pm >> 32), fl);
                const uint64_t m = ((uint64_t)hi << 32) | lo;
                const uint32_t bit = (uint32_t)__builtin_ctzll(m);
                cand[r] = 64 * fl + bit;
                if (lane == fl) pm &= pm - 1;
                ++nc;
            }
            if (!nc) break;
            uint32_t mine = row == 1 ? cand[1] : row == 2 ? cand[2] : row == 3 ? cand[3] : cand[0];
            if (row >= nc) mine = cand[0];
            uint32_t wk;
            uint64_t st;
            walk_hash<false>(src + y0 + mine, n, wk, st);
            uint32_t vb = kNoBlock;
            if ((lane & 15) == 0 && row < nc) vb = look(wk, st);
            weak_hits += nc;
            wcount(kWtVerifies, 1);
            for (uint32_t r = 0; r < nc; ++r) {
                const uint32_t bb = rl(vb, 16 * r);
                if (bb != kNoBlock) {
                    q = y0 + cand[r];
                    qb = bb;
                    break;
                }
            }
            if (qb != kNoBlock) break;
        }
        wtick(kWtVerify);
    }
}

// kLdsFilt: the unit is self-indexed -- its file's Bloom filter and exact candidate table are
// built in LDS from the file's signature (a batch's small files: no index build, no global
// lookups); else the index's filter and tables are read from global memory (L2-resident: a
// large single-file index, the segments of a chunk).
// kSlim: the walk of a pre-rolled part (launch_preroll), without the roll or the phase-window
// hashing: a unit that needs either (a phase change after a Copy at an unaligned position, a
// miss that was not pre-rolled) is left to the full kernel launched after it, which skips the
// units the slim one finished (marked in the unit table).  The full kernel's registers (the
// roll's) spill, and its spills cost a scratch round trip per block walked.
__device__ void expand_file(const ExpandArgs& a, uint32_t f, unsigned char* lds, uint32_t lds_bytes);
template <bool kLdsFilt, bool kSlim>
__global__ __launch_bounds__(64, 4) void k_walk_files(WalkArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const WalkUnit U = a.units[blockIdx.x];
    if (!kSlim && (U.final_ & kUnitDone)) return;  // walked by the slim kernel
    const uint32_t lane = threadIdx.x, row = lane >> 4;
    const uint32_t n = a.n;
    const uint64_t gb0 = a.fblk[U.file], nbf = a.fblk[U.file + 1] - gb0, ls = a.last_size[U.file];
    const uint32_t sbits = kLdsFilt ? self_bits((uint32_t)nbf) : 0u;
    const FileIx F = kLdsFilt ? FileIx{0, 0, gb0, 32 - sbits, 0} : a.files[U.file];
    const WalkLds L = walk_lds(a.self_nb);
    const uint32_t* filt = kLdsFilt ? (const uint32_t*)(smem + L.filt) : a.filt + F.filt_off;
    uint32_t* tab = (uint32_t*)(smem + L.tab);
    uint32_t* lw = (uint32_t*)(smem + L.lw);
    const uint32_t tmask = (1u << sbits) - 1;
    auto look = [&](uint32_t wk, uint64_t st) -> uint32_t {
        if constexpr (kLdsFilt)
            return self_lookup(tab, lw, tmask, a.strong + gb0, (uint32_t)nbf, gb0, wk, st);
        else
            return walk_lookup(a, F, wk, st);
    };
    uint32_t* ntab = (uint32_t*)(smem + L.ntab);
    uint32_t* pw = (uint32_t*)(smem + L.pw);
    uint64_t* pst = (uint64_t*)(smem + L.pst);
    uint64_t tlast = a.ticks ? wall_clock64() : 0;
    auto wtick = [&](int k) {  // SYDELTA_PHASE_TIMING: the wave's time since the last tick into ticks[k]
        if (a.ticks && lane == 0) {
            const uint64_t t = wall_clock64();
            atomicAdd(a.ticks + k, (unsigned long long)(t - tlast));
            tlast = t;
        }
    };
    auto wcount = [&](int k, uint64_t v) {
        if (a.ticks && lane == 0) atomicAdd(a.ticks + k, (unsigned long long)v);
    };
    const uint8_t* src = a.base + U.src;
    const uint64_t len = U.len, end = U.end;

    {  // self-indexed: the file's Bloom filter and candidate table; the roll table
        if constexpr (kLdsFilt) {
            uint32_t* fl = (uint32_t*)(smem + L.filt);
            const uint32_t fw = 1u << sbits;
            for (uint32_t i = lane; i < fw; i += 64) {
                fl[i] = 0;
                tab[i] = kNoBlock;
            }
            for (uint32_t i = lane; i < nbf; i += 64) lw[i] = a.weak[gb0 + i];
            __syncthreads();
            // each key: its filter bits, then its slot (linear probing; the lowest block of a weak
            // value keeps the slot, so candidates are found in index order)
            for (uint32_t i = lane; i < nbf; i += 64) {
                const uint32_t w = lw[i];
                const ProbeHash h = probe_hash(w);
                atomicOr(fl + (h.r >> F.fwshift), filt_mask(h.q));
                uint32_t sl = bucket_hash(w) & tmask;
                for (;;) {
                    uint32_t e = tab[sl];
                    if (e == kNoBlock) {
                        e = atomicCAS(tab + sl, kNoBlock, i);
                        if (e == kNoBlock) break;
                    }
                    if (lw[e] == w) {
                        atomicMin(tab + sl, i);
                        break;
                    }
                    sl = (sl + 1) & tmask;
                }
            }
        }
        for (uint32_t i = lane; i < 256; i += 64) ntab[i] = kMod - 1 - (a.nm * i) % kMod;
    }
    // the tail rule (generator.rs:156-184): the suffix of the basis's last block's size
    const bool tail_ok = U.final_ && nbf && ls < n && len >= ls &&
                         tail_matches(src + (len - ls), ls, a.weak[gb0 + nbf - 1], a.strong[gb0 + nbf - 1]);
    __syncthreads();  // the filter and ntab in LDS
    wtick(kWtSetup);

    // run-length coded output (lane 0 writes; the state is wave-uniform)
    WalkRec* stg = a.stage + U.rec_off;
    uint32_t nrec = 0, ck = 0, ca = 0;  // the open Copy run: ck Copies from block ca (ck 0: none)
    auto put = [&](uint32_t kind, uint32_t aa, uint64_t off) {
        if (lane == 0) stg[nrec] = WalkRec{kind, aa, off};
        ++nrec;
    };
    auto close_run = [&]() {
        if (ck) put(ck, ca, 0);
        ck = 0;
    };
    auto data = [&](uint64_t lo, uint64_t hi) {
        if (hi > lo) {
            close_run();
            put(0, (uint32_t)(hi - lo), lo);
        }
    };
    auto copy = [&](uint32_t g) {
        if (ck && g == ca + ck) {
            ++ck;
        } else {
            close_run();
            ck = 1;
            ca = g;
        }
    };
    uint32_t weak_hits = 0, hits = 0;

    uint64_t x = U.entry, lit = U.entry;
    uint32_t phi = 0xFFFFFFFFu;
    uint64_t rk0 = 0, rk1 = 0;  // lane w holds the result (rres) and weak (rwk) of block rk0 + w at phase phi
    uint64_t kph = 0;           // the block where the walk took phase phi
    uint32_t rres = kNoBlock, rwk = 0;
    // x = k n + ph: the slim kernel keeps it without a division per block (a 64-bit division by
    // a variable n is a long instruction sequence, and the walk steps a block at a time); the
    // full kernel divides at every step, which keeps its registers from spilling (LDS filter)
    // or spills fewer (global filter: 2 VGPRs against 5)
    uint64_t k = 0;
    uint32_t ph = 0;
    bool resync = true;  // k, ph from x by a division (after a move other than by n)
    auto move_to = [&](uint64_t nx) {
        if (nx == x + n)
            ++k;
        else
            resync = true;
        x = nx;
    };
#pragma unroll 1
    while (x < end) {
        if (resync || !kSlim) {
            k = x / n;
            ph = (uint32_t)(x - k * n);
            resync = false;
            if (kSlim && ph != 0) return;  // a new phase grid: the full kernel's
        }
        if (ph != phi || k >= rk1) {
            // ---- phase pass: windows (k + w) n + ph, w < cnt, four per row_hash round.  The
            // passes of one phase grow (4, then twice the blocks walked at this phase, up to
            // 64): a long run of Copies costs few passes, and a phase change soon after a pass
            // began wastes little of it.
            if (ph != phi) kph = k;
            const uint64_t left = (end - x + n - 1) / n;
            const uint32_t cnt = (uint32_t)min(left, min((uint64_t)kWMaxPass, max((uint64_t)4, 2 * (k - kph))));
            if (kSlim || (ph == 0 && a.ahit)) {  // phase 0 with the aligned probe's results: nothing to hash
                rres = kNoBlock;
                rwk = 0;
                if (lane < cnt) {
                    rres = a.ahit[k + lane - U.kb];
                    rwk = a.apw[k + lane - U.kb];
                }
                phi = ph;
                rk0 = k;
                rk1 = k + cnt;
                goto have_pass;
            }
#pragma unroll 1
            for (uint32_t j = 0; j < cnt; j += 4) {
                const uint32_t w = j + row;
                const uint64_t pos = (k + (w < cnt ? w : j)) * n + ph;
                uint32_t wk;
                uint64_t st;
                if ((ph & 15) == 0)
                    walk_hash<true>(src + pos, n, wk, st);
                else
                    walk_hash<false>(src + pos, n, wk, st);
                if ((lane & 15) == 0 && w < cnt) {
                    pw[w] = wk;
                    pst[w] = st;
                }
            }
            wtick(kWtHash);
            __syncthreads();  // the rows' results to the lanes
            rres = kNoBlock;
            rwk = 0;
            if (lane < cnt) {  // lookups (generator.rs:121-155), one window per lane
                rwk = pw[lane];
                const ProbeHash h = probe_hash(rwk);
                if (filt_pass(filt[h.r >> F.fwshift], h.q)) rres = look(rwk, pst[lane]);
            }
            __syncthreads();  // pw / pst are rewritten by the next pass
            wtick(kWtLookup);
            wcount(kWtPasses, 1);
            wcount(kWtWindows, cnt);
            phi = ph;
            rk0 = k;
            rk1 = k + cnt;
        }
    have_pass:
        const uint32_t blk = rl(rres, (uint32_t)(k - rk0));
        if (blk < kPreMark) {  // generator.rs:135-146
            ++hits;
            data(lit, x);
            copy(blk);
            move_to(x + n);
            lit = x;
            continue;
        }
        // ---- the window at x misses: roll (x, min(x + n, end)) for the first hit.  A pass
        // rolls 4096 window starts from the window at its base b = y0 - 1 (the phase window x,
        // then the previous pass's last start), whose (A, B) it knows: lane l's first start
        // p = b + d, d = 64 l + 1, follows in closed form (rolling.rs:66-79 applied d times):
        //   A(p) = A(b) + C(d),  B(p) = B(b) + d (A(b) - 1) + d C(d) - J(d) - n Out(d)  (mod M)
        // with c_j = in_j - out_j (out_j = byte b + j, in_j = byte b + n + j), C(d) = sum_{j<d} c_j,
        // J(d) = sum_{j<d} j c_j, Out(d) = sum_{j<d} out_j: exclusive wave scans of the lanes'
        // 64-byte group sums (as residues mod M), each lane's bytes in registers.
        const uint64_t yend = min(x + n, end);  // later starts are the next unit's
        uint64_t q = yend;
        uint32_t qb = kNoBlock;
        const uint32_t wb = rl(rwk, (uint32_t)(k - rk0));  // weak of the window at x (pre-rolled: the result)
        if (kLdsFilt || blk == kNoBlock) {  // (a batch's walks, kLdsFilt, are never pre-rolled)
            if (kSlim) return;  // not pre-rolled: the full kernel's
            walk_roll<kLdsFilt>(a, F, filt, ntab, src, len, x, yend, wb, q, qb, weak_hits, look, wtick, wcount);
        } else {  // pre-rolled (k_preroll): the first hit of (x, min(x + n, p1))
            weak_hits += wb >> 14;
            if (blk != kPreNone && x + (wb & 0x3FFFu) < yend) {
                q = x + (wb & 0x3FFFu);
                qb = blk & ~kPreMark;
            }
        }
        if (qb != kNoBlock) {
            ++hits;
            data(lit, q);
            copy(qb);
            move_to(q + n);
            lit = x;
        } else {
            move_to(yend);  // the next phase window (or the end of the full windows)
        }
    }
    // the walk's end.  A final unit: the tail rule at p* = len - last_size, then the last
    // literal run; another: the literal run up to end (the next unit continues it; the
    // host joins the two Data ops) and the exit (> end after a Copy that crosses it).
    uint64_t exit;
    if (U.final_) {
        if (tail_ok && ls <= len && len - ls >= lit) {
            data(lit, len - ls);
            copy((uint32_t)(gb0 + nbf - 1));
            lit = len;
            ++hits;
        }
        data(lit, len);
        exit = len;
    } else {
        data(lit, end);
        exit = max(x, end);
    }
    close_run();
    unsigned long long base = U.rec_off;  // no compact output: the records stay where they were staged
    if (a.out) {
        // move the records to the compact output (one atomic per file)
        __threadfence_block();
        base = 0;
        if (lane == 0 && nrec) base = atomicAdd(a.total, (unsigned long long)nrec);
        base = (uint32_t)rl((uint32_t)base, 0);
        for (uint32_t i = lane; i < nrec; i += 64) {
            const volatile WalkRec* r = stg + i;
            a.out[base + i] = WalkRec{r->kind, r->a, r->off};
        }
    }
    if (lane == 0) {
        a.fout[blockIdx.x] = WalkFileOut{(uint32_t)base, nrec, weak_hits, hits, exit, 0};
        if (a.fout_dev) a.fout_dev[blockIdx.x] = WalkFileOut{(uint32_t)base, nrec, weak_hits, hits, exit, 0};
    }
    if (kSlim && lane == 0) const_cast<WalkUnit*>(a.units)[blockIdx.x].final_ = U.final_ | kUnitDone;
    if constexpr (kLdsFilt) {
        if (a.x.ops) {  // the op lists on the device: the file's last unit to finish expands them
            __threadfence();  // this unit's records and results before its count
            uint32_t last = 0;
            if (lane == 0) last = atomicAdd(a.xdone + U.file, 1u) + 1 == a.x.fu[U.file + 1] - a.x.fu[U.file];
            if (rl(last, 0)) {
                __threadfence();  // the other units' records and results after their counts
                __syncthreads();  // (the walk's LDS is free)
                expand_file(a.x, U.file, smem, L.total);
            }
        }
    }
    wtick(kWtOut);
}

// ===========================================================================
// K10's pre-roll (a chunk's aligned misses, launch_preroll)
// ===========================================================================
// A chunk walk spends most of its time rolling the window starts after each missed aligned
// block, one wave per segment doing its misses in turn.  The pre-roll does those rolls
// beforehand, one wave per miss: the walk then reads each miss's result instead.
// The misses are listed first (one thread per block, a wave-aggregated atomic).
__global__ __launch_bounds__(1024) void k_miss_list(const uint32_t* ahit, uint64_t b0, uint64_t b1, uint32_t* list,
                                                    unsigned long long* count) {
    __shared__ uint32_t wc[64];  // per (wave, quarter): misses, then their list offset
    __shared__ uint32_t wbase;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t g = b0 + (uint64_t)blockIdx.x * 4096 + t;  // the workgroup's 4096 blocks, 4 per thread
    uint64_t m[4];
    bool miss[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t r = g + 1024 * i;
        miss[i] = r < b1 && ahit[r] == kNoBlock;
        m[i] = __ballot(miss[i]);
        if (lane == 0) wc[4 * w + i] = (uint32_t)__popcll(m[i]);
    }
    __syncthreads();
    if (t == 0) {  // one atomic per workgroup
        uint32_t s = 0;
        for (int j = 0; j < 64; ++j) {
            const uint32_t c = wc[j];
            wc[j] = s;
            s += c;
        }
        wbase = s ? (uint32_t)atomicAdd(count, (unsigned long long)s) : 0u;
    }
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (miss[i]) list[wbase + wc[4 * w + i] + __popcll(m[i] & below)] = (uint32_t)(g + 1024 * i);
}

__global__ __launch_bounds__(64, 4) void k_preroll(WalkArgs a, uint32_t* ahit, uint32_t* apw, uint64_t kb,
                                                   uint64_t pend, uint64_t len, const uint32_t* list,
                                                   const unsigned long long* count, uint64_t max_miss) {
    __shared__ uint32_t ntab[256];
    const uint32_t lane = threadIdx.x;
    const uint64_t m = *count;
    // more misses than max_miss (a shifted source: every aligned window misses, and the walk
    // visits few of them): none is pre-rolled, the walk rolls the ones it meets
    if (blockIdx.x >= m || m > max_miss) return;
    for (uint32_t i = lane; i < 256; i += 64) ntab[i] = kMod - 1 - (a.nm * i) % kMod;
    __syncthreads();
    const FileIx F = a.files[0];
    const uint32_t* filt = a.filt + F.filt_off;
    const uint64_t n = a.n;
#pragma unroll 1
    for (uint64_t i = blockIdx.x; i < m; i += gridDim.x) {
        const uint32_t r = list[i];
        const uint64_t x = (kb + r) * n;
        uint64_t q;
        uint32_t qb, wh = 0;
        walk_roll<false>(a, F, filt, ntab, a.base, len, x, min(x + n, pend), apw[r], q, qb, wh,
                         [&](uint32_t wk, uint64_t st) { return walk_lookup(a, F, wk, st); }, [](int) {},
                         [](int, uint64_t) {});
        if (lane == 0) {  // (the walk's miss at x, with the roll's result: launch_preroll)
            ahit[r] = qb == kNoBlock ? kPreNone : (qb | kPreMark);
            apw[r] = (qb == kNoBlock ? 0u : (uint32_t)(q - x)) | (min(wh, 0x3FFFFu) << 14);
        }
    }
}

// ===========================================================================
// K10's op lists expanded on the device (WalkArgs::x)
// ===========================================================================
// The last unit of a file to finish its walk (a per-file counter) expands the file's op list,
// so the expansion's writes to host memory overlap the other files' walks.  The file's units'
// records are gathered into the wave's LDS (free once its walk is done) in unit order; lane 0
// chains them (the walk from the previous unit's exit: a unit that started there, or earlier
// with a leading literal run reaching it, which is cut there) and merges a Data op ending at a
// unit's end with the next unit's first one; then every lane takes ops i = lane, lane + 64, ...:
// the record holding op i (a binary search of the records' op prefix) gives it -- a Data op, or
// Copy (g - gb0) n of block g of a copy run, sized n or the basis's last size.  The ops go to
// host-mapped memory as three 8-byte stores per lane (24-byte stride).  cap: records the LDS
// holds; a file with more (or more than 64 units, or units that do not chain) gets bad = 1.
__device__ void expand_file(const ExpandArgs& a, uint32_t f, unsigned char* lds, uint32_t lds_bytes) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* ustart = (uint32_t*)lds;  // 65 entries, then s_m, s_bad
    uint32_t* sv = ustart + 65;
    WalkRec* rec = (WalkRec*)(lds + 272);
    const uint32_t cap = (lds_bytes - 272) / (sizeof(WalkRec) + 4);
    uint32_t* pre = (uint32_t*)(rec + cap);  // inclusive op prefix over the merged records
    const uint32_t u0 = a.fu[f], u1 = a.fu[f + 1], nu = u1 - u0;
    ExpandOut* res = a.res + f;
    // gather the units' staged records
    uint32_t total = 0;
    bool over = nu > 64;
    for (uint32_t k = 0; k < nu && !over; ++k) {
        const uint32_t c = a.fout[u0 + k].count;
        if (total + c > cap) {
            over = true;
            break;
        }
        const WalkRec* src = a.stage + a.units[u0 + k].rec_off;
        for (uint32_t i = lane; i < c; i += 64) rec[total + i] = src[i];
        if (lane == 0) ustart[k] = total;
        total += c;
    }
    if (over) {
        if (lane == 0) *res = ExpandOut{0, 0, 0, 0, 0, 1, 0};
        return;
    }
    if (lane == 0) ustart[nu] = total;
    __syncthreads();
    uint32_t wh = 0, vh = 0;  // (every lane's partial sums of the units' counters)
    for (uint32_t k = lane; k < nu; k += 64) {
        wh += a.fout[u0 + k].weak_hits;
        vh += a.fout[u0 + k].hits;
    }
    if (lane == 0) {  // chain and merge in place (the output index never passes the input's)
        uint32_t m = 0, bad = 0;
        for (uint32_t k = 0; k < nu && !bad; ++k) {
            uint32_t r0 = ustart[k];
            const uint32_t r1 = ustart[k + 1];
            if (k > 0) {
                const uint64_t pe = a.fout[u0 + k - 1].exit, entry = a.units[u0 + k].entry;
                if (entry != pe) {
                    if (pe > entry && r0 < r1 && rec[r0].kind == 0 && rec[r0].off == entry &&
                        rec[r0].off + rec[r0].a >= pe) {
                        const uint64_t h = rec[r0].off + rec[r0].a;
                        if (h == pe) {
                            ++r0;
                        } else {
                            rec[r0].a = (uint32_t)(h - pe);
                            rec[r0].off = pe;
                        }
                    } else {
                        bad = 1;
                    }
                }
            }
            for (uint32_t r = r0; r < r1 && !bad; ++r) {
                const WalkRec x = rec[r];
                if (!x.kind && m && !rec[m - 1].kind && rec[m - 1].off + rec[m - 1].a == x.off)
                    rec[m - 1].a += x.a;
                else
                    rec[m++] = x;
            }
        }
        sv[0] = m;
        sv[1] = bad;
    }
    __syncthreads();
    const uint32_t m = sv[0];
    if (sv[1]) {
        if (lane == 0) *res = ExpandOut{0, 0, 0, 0, 0, 1, 0};
        return;
    }
    // op counts: an inclusive prefix over the records, 64 at a time
    uint32_t carry = 0, nd = 0;
    uint64_t lit = 0;
    for (uint32_t b = 0; b < m; b += 64) {
        const uint32_t i = b + lane;
        const WalkRec x = i < m ? rec[i] : WalkRec{1, 0, 0};
        const uint32_t c = i < m ? (x.kind ? x.kind : 1u) : 0u;
        if (i < m && !x.kind) {
            ++nd;
            lit += x.a;
        }
        uint32_t tot;
        const uint32_t ex = wave_scan_excl(c, tot);
        if (i < m) pre[i] = carry + ex + c;
        carry += tot;
    }
    __syncthreads();
    const uint64_t T = carry;
    const uint64_t gb0 = a.fblk[f], nbf = a.fblk[f + 1] - gb0, ls = a.last_size[f];
    if (T > a.op_off[f + 1] - a.op_off[f]) {  // (cannot happen: the host sizes by the units' bound)
        if (lane == 0) *res = ExpandOut{0, 0, 0, 0, 0, 1, 0};
        return;
    }
    uint64_t* w = (uint64_t*)(a.ops + a.op_off[f]);
    uint32_t r = 0;  // the record of this lane's op (ops ascend: search from the last one)
    for (uint32_t i = lane; i < (uint32_t)T; i += 64) {
        uint32_t lo = r, hi = m - 1;
        while (lo < hi) {  // the first record whose prefix passes i
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] > i) hi = mid; else lo = mid + 1;
        }
        r = lo;
        const WalkRec x = rec[r];
        uint64_t k, oa, ob;
        if (!x.kind) {
            k = SYDELTA_OP_DATA;
            oa = x.off;
            ob = x.a;
        } else {
            const uint64_t g = (uint64_t)x.a - gb0 + (i - (pre[r] - x.kind));
            k = SYDELTA_OP_COPY;
            oa = g * a.n;
            ob = g + 1 == nbf ? ls : (uint64_t)a.n;
        }
        w[3 * (uint64_t)i] = k;
        w[3 * (uint64_t)i + 1] = oa;
        w[3 * (uint64_t)i + 2] = ob;
    }
    // the file's counts
    uint32_t nd_t = nd;
    for (int o = 32; o; o >>= 1) {
        nd_t += __shfl_xor(nd_t, o);
        lit += __shfl_xor(lit, o);
        wh += __shfl_xor(wh, o);
        vh += __shfl_xor(vh, o);
    }
    if (lane == 0) *res = ExpandOut{T, nd_t, lit, wh, vh, 0, 0};
}

// ===========================================================================
// A chunk's ops written on the device (launch_chunk_write)
// ===========================================================================
// One wave per unit: its effective records 64 at a time (the plan's cut first record, the
// extension of its last one), an inclusive op prefix in LDS, then ops j = lane, lane + 64, ...
// of those records (the record holding op j by binary search), three 8-byte stores each.
__global__ __launch_bounds__(64) void k_chunk_write(const WalkUnit* __restrict__ units, const WalkRec* __restrict__ stage,
                                                    const CxPlan* __restrict__ plan, uint32_t n, uint64_t nbf, uint64_t ls,
                                                    uint64_t* __restrict__ ops) {
    __shared__ WalkRec rec[64];
    __shared__ uint32_t pre[64];
    const uint32_t lane = threadIdx.x;
    const CxPlan P = plan[blockIdx.x];
    const WalkRec* src = stage + units[blockIdx.x].rec_off;
    uint64_t o = P.first;
    for (uint32_t b = P.skip; b < P.cnt; b += 64) {
        const uint32_t i = b + lane;
        WalkRec x{1, 0, 0};
        uint32_t c = 0;
        if (i < P.cnt) {
            x = src[i];
            if (i == P.skip && (P.flags & 1)) {
                x.off = P.r0_off;
                x.a = P.r0_a;
            }
            c = x.kind ? x.kind : 1u;
        }
        uint32_t tot;
        const uint32_t ex = wave_scan_excl(c, tot);
        rec[lane] = x;
        pre[lane] = ex + c;  // (lanes past the records: the total)
        __syncthreads();
        for (uint32_t j = lane; j < tot; j += 64) {
            uint32_t lo = 0, hi = 63;
            while (lo < hi) {  // the first record whose prefix passes j
                const uint32_t mid = (lo + hi) >> 1;
                if (pre[mid] > j) hi = mid; else lo = mid + 1;
            }
            const WalkRec y = rec[lo];
            uint64_t kd, oa, ob;
            if (!y.kind) {
                kd = SYDELTA_OP_DATA;
                oa = y.off;
                ob = (uint64_t)y.a + (b + lo + 1 == P.cnt ? P.ext : 0ull);
            } else {
                const uint64_t g = (uint64_t)y.a + (j - (pre[lo] - y.kind));
                kd = SYDELTA_OP_COPY;
                oa = g * n;
                ob = g + 1 == nbf ? ls : (uint64_t)n;
            }
            uint64_t* w = ops + 3 * (o + j);
            w[0] = kd;
            w[1] = oa;
            w[2] = ob;
        }
        o += tot;
        __syncthreads();
    }
}

// ===========================================================================
// Launch wrappers
// ===========================================================================

hipError_t launch_walk_files(const WalkArgs& a, hipStream_t s, Profiler* prof, bool slim) {
    if (!a.nunits) return hipSuccess;
    if (a.n % 64 != 0 || a.n < 256 || a.n > kWalkMaxN || a.self_nb > kSelfIxMaxBlocks || (slim && (a.self_nb || !a.ahit)))
        return hipErrorInvalidValue;
    const WalkLds L = walk_lds(a.self_nb);
    ProfScope ps(prof, s, slim ? "k_walk_files_slim" : "k_walk_files");
    if (a.self_nb)
        hipLaunchKernelGGL((k_walk_files<true, false>), dim3(a.nunits), dim3(64), L.total, s, a);
    else if (slim)
        hipLaunchKernelGGL((k_walk_files<false, true>), dim3(a.nunits), dim3(64), L.total, s, a);
    else
        hipLaunchKernelGGL((k_walk_files<false, false>), dim3(a.nunits), dim3(64), L.total, s, a);
    return hipGetLastError();
}

hipError_t launch_chunk_write(const WalkUnit* units, const WalkRec* stage, const CxPlan* plan, uint32_t nunits,
                              uint32_t n, uint64_t nbf, uint64_t ls, sydelta_op* ops, hipStream_t s, Profiler* prof) {
    if (!nunits) return hipSuccess;
    if (!units || !stage || !plan || !ops || !n) return hipErrorInvalidValue;
    ProfScope ps(prof, s, "k_chunk_write");
    hipLaunchKernelGGL(k_chunk_write, dim3(nunits), dim3(64), 0, s, units, stage, plan, n, nbf, ls, (uint64_t*)ops);
    return hipGetLastError();
}

hipError_t launch_preroll(const WalkArgs& a, uint32_t* ahit, uint32_t* apw, uint64_t kb, uint64_t b0, uint64_t b1,
                          uint64_t pend, uint64_t len, uint32_t* list, unsigned long long* count, uint32_t waves,
                          uint64_t max_miss, hipStream_t s, Profiler* prof) {
    if (b1 <= b0) return hipSuccess;
    if (a.n % 64 != 0 || a.n < 256 || a.n > kWalkMaxN || !ahit || !apw || !waves || b1 - b0 >= (1ull << 31))
        return hipErrorInvalidValue;
    {
        ProfScope ps(prof, s, "k_miss_list");
        hipLaunchKernelGGL(k_miss_list, dim3((unsigned)((b1 - b0 + 4095) / 4096)), dim3(1024), 0, s, ahit, b0, b1, list,
                           count);
    }
    ProfScope ps(prof, s, "k_preroll");
    hipLaunchKernelGGL(k_preroll, dim3(waves), dim3(64), 0, s, a, ahit, apw, kb, pend, len, list, count, max_miss);
    return hipGetLastError();
}

}  // namespace sydelta
