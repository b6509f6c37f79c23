// sydelta_walk.hpp — the host side of the match after classification: per-source hit
// lists, the greedy walk over them (generator.rs:116-221 / 283-379) and its split,
// chained, joined parallel form.  Plain C++ (no HIP): sydelta_api.cpp drives it, and
// tests/csrc/host_fuzz.cpp runs it under AddressSanitizer/UBSan against a restated
// greedy walk on synthetic hit lists.
#pragma once
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/sydelta.h"

// Op arrays grow without zero-filling: resize() default-initialises the POD ops, so a
// parallel walk can size the joined array and fill it from several threads.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
// Op arrays of 1 MiB and more may come from a registered arena: sydelta_api.cpp installs
// pinned host memory when the device walk is on, so a device-resolved op list lands in
// the delta's own array by DMA.  Without an arena: the heap.
struct OpArena {
    void* (*alloc)(size_t bytes) = nullptr;  // nullptr result: use the heap
    bool (*release)(void* p) = nullptr;      // true if p came from alloc (and is released)
};
inline OpArena& op_arena() {
    static OpArena a;
    return a;
}
constexpr size_t kOpArenaMin = 1u << 20;
// Op slabs: a batch whose op lists the device expands (sydelta_api.cpp) reserves every file's
// op array from one pinned, host-mapped slab.  While the calling thread has a slab open,
// allocate() takes from it; deallocate() recognises slab memory and counts it off.
struct OpSlabHooks {
    void* (*take)(size_t bytes) = nullptr;  // from the calling thread's open slab, else nullptr
    bool (*give)(void* p) = nullptr;        // true if p lies in a slab (then counted off)
};
inline OpSlabHooks& op_slab() {
    static OpSlabHooks h;
    return h;
}

template <class T>
struct OpAlloc {
    using value_type = T;
    OpAlloc() = default;
    template <class U>
    OpAlloc(const OpAlloc<U>&) {}
    T* allocate(size_t n) {
        const OpSlabHooks& S = op_slab();
        if (S.take)
            if (void* p = S.take(n * sizeof(T))) return (T*)p;
        const OpArena& A = op_arena();
        if (n * sizeof(T) >= kOpArenaMin && A.alloc)
            if (void* p = A.alloc(n * sizeof(T))) return (T*)p;
        return std::allocator<T>().allocate(n);
    }
    void deallocate(T* p, size_t n) {
        const OpSlabHooks& S = op_slab();
        if (S.give && S.give(p)) return;
        const OpArena& A = op_arena();
        if (n * sizeof(T) >= kOpArenaMin && A.release && A.release(p)) return;
        std::allocator<T>().deallocate(p, n);
    }
    template <class U>
    void construct(U* p) noexcept {  // no zero fill (as NoInitAlloc)
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
    friend bool operator==(const OpAlloc&, const OpAlloc&) { return true; }
    friend bool operator!=(const OpAlloc&, const OpAlloc&) { return false; }
};
using OpVec = std::vector<sydelta_op, OpAlloc<sydelta_op>>;

namespace sydelta {
namespace walk {

constexpr uint32_t kNoBlk = 0xFFFFFFFFu;
constexpr uint64_t kUnknownNone = UINT64_MAX;

// One source being classified: a whole file of a batch, or a chunk of one file.
// Scan-hit lists: filled by index (Classifier::scan), so no zero fill on resize.
using HitPos = std::vector<uint64_t, NoInitAlloc<uint64_t>>;
using HitBlk = std::vector<uint32_t, NoInitAlloc<uint32_t>>;

struct Src {
    uint32_t file = 0;          // basis file in the index
    uint64_t off = 0;           // byte offset of source position 0 from the launch base
    uint64_t len = 0;           // bytes readable from position 0 (zeros beyond, see load_chunk)
    uint64_t flen = 0;          // source file length (Delta::source_size)
    uint64_t p0 = 0, p1 = 0;    // full-window positions to classify, [p0, p1); p0 % n == 0
    uint64_t kb = 0, nblk = 0;  // blocks kb .. kb+nblk-1 (position k*n) cover [p0, p1)
    bool probed = false;
    std::vector<uint32_t, NoInitAlloc<uint32_t>> ahit;  // probed: per block, its aligned window's hit or kNoBlk
    uint64_t nahit = 0;            // aligned windows that hit
    std::vector<uint8_t> scanned;  // probed: per block, all its window starts were scanned
    HitPos hpos;                   // hits found by scans, sorted, unique
    HitBlk hblk;                   // their global block indices
    std::vector<uint64_t> ppos;    // probed: per block, its phase-probed window start or kUnknownNone
    std::vector<uint32_t> phit;    // ... and that window's hit or kNoBlk
};

// Merge sorted (pos, blk) lists into c's hits (equal positions carry equal blocks).
template <class PV = HitPos, class BV = HitBlk>
inline void merge_hits(Src& c, const PV& pos, const BV& blk) {
    if (pos.empty()) return;
    if (c.hpos.empty() || pos.front() > c.hpos.back()) {  // later positions: append
        c.hpos.insert(c.hpos.end(), pos.begin(), pos.end());
        c.hblk.insert(c.hblk.end(), blk.begin(), blk.end());
        return;
    }
    HitPos np;
    HitBlk nb;
    np.reserve(c.hpos.size() + pos.size());
    nb.reserve(c.hpos.size() + pos.size());
    size_t i = 0, j = 0;
    while (i < c.hpos.size() || j < pos.size()) {
        if (j == pos.size() || (i < c.hpos.size() && c.hpos[i] < pos[j])) {
            np.push_back(c.hpos[i]); nb.push_back(c.hblk[i]); ++i;
        } else if (i == c.hpos.size() || pos[j] < c.hpos[i]) {
            np.push_back(pos[j]); nb.push_back(blk[j]); ++j;
        } else {
            np.push_back(pos[j]); nb.push_back(blk[j]); ++i; ++j;
        }
    }
    c.hpos.swap(np);
    c.hblk.swap(nb);
}

// First position of [x, p) whose class is unknown (window starts inside a probed
// block that was not scanned; its aligned start k*n is known), or kUnknownNone.
inline uint64_t first_unknown(const Src& c, uint64_t n, uint64_t x, uint64_t p) {
    if (!c.probed || x >= p) return kUnknownNone;
    const uint64_t kend = std::min(c.kb + c.nblk, (p - 1) / n + 1);
    for (uint64_t k = std::max(c.kb, x / n); k < kend; ++k) {
        if (c.scanned[k - c.kb]) continue;
        uint64_t lo = std::max(x, k * n + 1);
        const uint64_t hi = std::min(p, k * n + n);
        // a phase-probed window start inside the block is classified too
        if (lo < hi && !c.ppos.empty() && c.ppos[k - c.kb] == lo) ++lo;
        if (lo < hi) return lo;
    }
    return kUnknownNone;
}

// The basis file a walk copies from.
struct BasisInfo {
    uint64_t blk_base;   // its first global block
    uint64_t nblocks;
    uint64_t last_size;  // size of its last block
};

// The end of a walk that stopped at x (>= end, or no hit left before end) with its
// literal run open since lit: a non-final chunk ends with that run up to `end` and
// *exit = max(x, end); a final source applies the tail rule (generator.rs:156-184: only
// p* = len - last_size can match) and ends with the last literal run.
inline void finish_walk(const Src& c, uint64_t n, uint64_t lit, uint64_t x, uint64_t end, const BasisInfo& bi,
                        bool final_src, int tail_match, OpVec& ops, uint64_t* exit) {
    auto data = [&](uint64_t a, uint64_t b) {
        if (b > a) ops.push_back({SYDELTA_OP_DATA, 0, a, b - a});
    };
    if (!final_src) {
        data(lit, end);
        *exit = std::max(x, end);
        return;
    }
    if (tail_match && bi.nblocks) {
        const uint64_t pstar = c.flen - bi.last_size;
        if (pstar >= lit) {
            data(lit, pstar);
            const uint64_t b = bi.nblocks - 1;
            ops.push_back({SYDELTA_OP_COPY, 0, b * n, bi.last_size});
            lit = c.flen;
        }
    }
    data(lit, c.flen);
    *exit = c.flen;
}

// Greedy walk (generator.rs:116-221 / 283-379) over c's classified positions from
// `entry` up to `end` (c.p1, or a split point of a parallel walk).  ops get
// Data(source offset, len) and Copy(basis offset, size); consecutive Copies are never
// merged (generator.rs:135-140).  A non-final chunk ends with the literal run up to
// `end` (continued by the next chunk) and *exit = where the walk left [entry, end).  A
// final source (its file ends inside it) applies the tail rule (generator.rs:156-184:
// only p* = len - last_size can match) and the last literal run.  Returns 1 with
// *need = the first position whose class is unknown (ops rolled back).
inline int walk_src(const Src& c, uint64_t n, uint64_t entry, uint64_t end, const BasisInfo& bi, bool final_src,
                    int tail_match, OpVec& ops, uint64_t* exit, uint64_t* need) {
    const size_t ops0 = ops.size();  // appended to; rolled back on a need
    {
        const uint64_t span = c.p1 > c.p0 ? c.p1 - c.p0 : 1;
        const double frac = end > entry ? double(end - entry) / double(span) : 0.0;
        ops.reserve(ops0 + (size_t)(2.0 * double(c.hpos.size() + c.nahit) * std::min(1.0, frac)) + 16);
    }
    uint64_t x = entry, lit = entry;
    auto data = [&](uint64_t a, uint64_t b) {
        if (b > a) ops.push_back({SYDELTA_OP_DATA, 0, a, b - a});
    };
    auto copy = [&](uint64_t gblk) {
        const uint64_t b = gblk - bi.blk_base;
        ops.push_back({SYDELTA_OP_COPY, 0, b * n, (b + 1 == bi.nblocks) ? bi.last_size : n});
    };
    size_t i = std::lower_bound(c.hpos.begin(), c.hpos.end(), x) - c.hpos.begin();
    const size_t H = c.hpos.size();
    const uint64_t kend = c.kb + c.nblk;
    uint64_t ka = c.kb;  // next aligned window that may hit (probed sources)
    uint64_t kp = c.kb;  // next block whose phase-probed window may hit
    const bool has_phase = c.probed && !c.ppos.empty();
    while (x < end) {
        // aligned windows before x are behind the walk (after a Copy of block k found
        // below, x = (k+1)*n: ka catches up here, so the run fast path resumes)
        if (c.probed && ka * n < x) ka = (x + n - 1) / n;
        if (c.probed && x == lit && ka < kend && ka * n == x) {
            // a run of aligned Copies (the rsync case): at an aligned x whose aligned window
            // hit, that window is the earliest hit (a scan hit at x names the same block,
            // phase-probed windows lie inside blocks), so copy it and jump a block.  The run
            // is measured first and written through a pointer (locals: the op stores cannot
            // alias them).
            const uint32_t* ah = c.ahit.data() - c.kb;
            uint64_t k1 = ka;
            while (k1 < kend && k1 * n < end && ah[k1] != kNoBlk) ++k1;
            if (k1 > ka) {
                const uint64_t bb = bi.blk_base, nbb = bi.nblocks, ls = bi.last_size;
                const size_t o = ops.size();
                ops.resize(o + (k1 - ka));
                sydelta_op* w = ops.data() + o;
                for (uint64_t k = ka; k < k1; ++k) {
                    const uint64_t g = ah[k] - bb;
                    *w++ = {SYDELTA_OP_COPY, 0, g * n, g + 1 == nbb ? ls : n};
                }
                x = k1 * n;
                lit = x;
                ka = k1;
                if (x >= end) break;
            }
        }
        // next hit at or after x and before end: the next scan hit or the next aligned hit
        while (i < H && c.hpos[i] < x) ++i;
        if (x == lit && x < end && i < H && c.hpos[i] == x) {
            // a run of scan-hit Copies (a source shifted off the block grid: C3b, C4): a
            // hit at x itself is the earliest hit at or after x (an aligned or phase-probed
            // hit there names the same block), so copy it and jump a block, as below
            do {
                copy(c.hblk[i]);
                x += n;
                while (++i < H && c.hpos[i] < x) {
                }
            } while (x < end && i < H && c.hpos[i] == x);
            lit = x;
            continue;
        }
        if (has_phase && x == lit && x < end) {
            // a run of phase-probed Copies (the shifted blocks after an insertion, C4): the
            // window at x itself is the earliest hit at or after x (an aligned or scan hit
            // there names the same block), so copy it and jump a block
            uint64_t k = x / n;
            if (k >= c.kb && k < kend && c.ppos[k - c.kb] == x && c.phit[k - c.kb] != kNoBlk) {
                do {
                    copy(c.phit[k - c.kb]);
                    x += n;
                    ++k;
                } while (x < end && k < kend && c.ppos[k - c.kb] == x && c.phit[k - c.kb] != kNoBlk);
                lit = x;
                continue;
            }
        }
        uint64_t p = end;
        uint32_t pb = kNoBlk;
        if (i < H && c.hpos[i] < end) { p = c.hpos[i]; pb = c.hblk[i]; }
        if (c.probed) {
            while (ka < kend && ka * n < p && c.ahit[ka - c.kb] == kNoBlk) ++ka;
            if (ka < kend && ka * n < p) { p = ka * n; pb = c.ahit[ka - c.kb]; }
            if (has_phase) {  // phase-probed hits (one window per block, inside it)
                if (kp * n + n <= x) kp = x / n;
                while (kp < kend && kp * n < p &&
                       (c.ppos[kp - c.kb] < x || c.ppos[kp - c.kb] == kUnknownNone || c.phit[kp - c.kb] == kNoBlk))
                    ++kp;
                if (kp < kend && c.ppos[kp - c.kb] < p && c.ppos[kp - c.kb] >= x && c.phit[kp - c.kb] != kNoBlk) {
                    p = c.ppos[kp - c.kb];
                    pb = c.phit[kp - c.kb];
                }
            }
        }
        const uint64_t u = first_unknown(c, n, x, p);
        if (u != kUnknownNone) {
            *need = u;
            ops.resize(ops0);
            return 1;
        }
        if (pb == kNoBlk) {
            x = end;
            break;
        }
        data(lit, p);
        copy(pb);
        x = p + n;  // generator.rs:144 / :313
        lit = x;
    }
    finish_walk(c, n, lit, x, end, bi, final_src, tail_match, ops, exit);
    return 0;
}

// Process-wide worker pool shared by every caller's parallel host work (walk
// segments, probe-result fills): concurrent entry-point calls share its threads
// instead of each starting its own.  Size: SYDELTA_HOST_THREADS,
// else the hardware threads capped at 16.  Threads start on first use and are never
// joined (the pool outlives static destruction).
class HostPool {
  public:
    struct Batch {
        std::function<void(int)> f;
        int n = 0;
        std::atomic<int> next{0}, done{0};
        std::atomic<bool> ok{true};
        std::mutex mu;
        std::condition_variable cv;
        void work() {
            for (;;) {
                const int i = next.fetch_add(1);
                if (i >= n) return;
                try {
                    f(i);
                } catch (...) {
                    ok = false;
                }
                if (done.fetch_add(1) + 1 == n) {
                    std::lock_guard<std::mutex> lk(mu);
                    cv.notify_all();
                }
            }
        }
    };
    static HostPool& get() {
        static HostPool* p = new HostPool();  // never destroyed: workers may still wait on it at exit
        return *p;
    }
    int size() const { return nthreads_; }
    // Run f(0..n): the caller works on the batch too, so a call completes even when
    // every pool thread is busy with other callers' batches.  False if a task threw.
    bool run(int n, std::function<void(int)> f) {
        if (n <= 0) return true;
        auto b = std::make_shared<Batch>();
        b->f = std::move(f);
        b->n = n;
        const int helpers = std::min(n - 1, nthreads_);
        if (helpers > 0) {
            try {
                start();
                std::lock_guard<std::mutex> lk(mu_);
                for (int i = 0; i < helpers; ++i) q_.push_back(b);
            } catch (...) {  // no threads: the caller runs the whole batch
            }
            cv_.notify_all();
        }
        b->work();
        std::unique_lock<std::mutex> lk(b->mu);
        b->cv.wait(lk, [&] { return b->done.load() == b->n; });
        return b->ok;
    }

  private:
    HostPool() {
        const char* e = getenv("SYDELTA_HOST_THREADS");
        const unsigned hw = std::thread::hardware_concurrency();
        nthreads_ = (e && *e) ? std::max(0, atoi(e)) : (int)std::min(16u, std::max(1u, hw));
    }
    void start() {
        std::call_once(once_, [this] {
            for (int t = 0; t < nthreads_; ++t) std::thread([this] { loop(); }).detach();
        });
    }
    void loop() {
        for (;;) {
            std::shared_ptr<Batch> b;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                b = std::move(q_.front());
                q_.pop_front();
            }
            b->work();
        }
    }
    int nthreads_ = 0;
    std::once_flag once_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Batch>> q_;
};

// Run task(t) for t in [0, n) on the shared pool (and the calling thread).  No
// exception leaves: returns false when a task threw (out of memory), so the C entry
// points can report SYDELTA_E_OOM.
template <class F>
bool run_parallel(int n, F&& task) {
    if (n == 1) {
        try {
            task(0);
            return true;
        } catch (...) {
            return false;
        }
    }
    try {
        return HostPool::get().run(n, [&](int t) { task(t); });
    } catch (...) {
        return false;
    }
}

// No known hit starts in (x - n, x): no Copy can cover x, so every walk that starts
// before x lands exactly on x (a step is +1, or +n from a hit).  Scan hits, aligned hits
// of probed blocks and phase-probed hits are consulted; a position only an on-demand
// scan would classify counts as no hit here (the walk then reports it, and the caller
// walks sequentially).
inline bool no_hit_before(const Src& c, uint64_t n, uint64_t x) {
    const uint64_t lo = x >= n ? x - n + 1 : 0;  // (x - n, x) = [lo, x)
    if (lo >= x) return true;
    const auto it = std::lower_bound(c.hpos.begin(), c.hpos.end(), lo);
    if (it != c.hpos.end() && *it < x) return false;
    if (c.probed) {
        for (uint64_t k = lo / n; k * n < x; ++k) {  // the blocks [lo, x) touches (at most two)
            if (k < c.kb || k >= c.kb + c.nblk) continue;
            if (k * n >= lo && c.ahit[k - c.kb] != kNoBlk) return false;
            if (!c.ppos.empty() && c.ppos[k - c.kb] != kUnknownNone && c.ppos[k - c.kb] >= lo &&
                c.ppos[k - c.kb] < x && c.phit[k - c.kb] != kNoBlk)
                return false;
        }
    }
    return true;
}

// Split points of a parallel walk of c from `entry`, at most T0 segments, st.back() ==
// c.p1.  Each cut is a position the walk is known to land on (no_hit_before), so the
// segments chain without a re-walk: the ideal cut itself, else the first multiple of n
// or scan hit after it that qualifies (rsync-shaped sources shifted off the block grid
// put every Copy at a scan hit, C3b), else the multiple of n (then the chain re-walks
// the next segment when the walk does not land there).
inline std::vector<uint64_t> split_points(const Src& c, uint64_t n, uint64_t entry, int T0) {
    std::vector<uint64_t> st{entry};
    for (int t = 1; t < T0; ++t) {
        const uint64_t ideal = entry + (c.p1 - entry) / T0 * t;
        const uint64_t lim = std::min(c.p1, ideal + 64 * n);
        uint64_t q = ideal / n * n, pick = 0;
        if (no_hit_before(c, n, ideal)) pick = ideal;
        auto h = std::lower_bound(c.hpos.begin(), c.hpos.end(), ideal);
        uint64_t m = (ideal + n - 1) / n * n;
        for (int tries = 0; !pick && tries < 128; ++tries) {
            const uint64_t hp = h != c.hpos.end() ? *h : UINT64_MAX;
            const uint64_t x = std::min(hp, m);
            if (x >= lim) break;
            if (no_hit_before(c, n, x)) pick = x;
            if (x == hp) ++h;
            if (x == m) m += n;
        }
        if (pick) q = pick;
        if (q > st.back() && q < c.p1) st.push_back(q);
    }
    st.push_back(c.p1);
    return st;
}

struct SplitTiming {
    double walk_ms = 0, seg_max_ms = 0, seg_min_ms = 0, chain_ms = 0, join_ms = 0;
};

// Op counts of a joined list (Delta stats), counted by the join's copy tasks.
struct OpCounts {
    uint64_t copy_ops = 0, data_ops = 0, literal_bytes = 0;
};

// The walk of c from `entry` split at st[1..T) (split_points): every segment walked
// concurrently from its split point, then chained -- segment t's true entry is segment
// t-1's exit; a segment entered elsewhere is walked again from there -- and joined,
// merging a Data op that ends where the next segment's first Data op starts.  The
// result equals walk_src(c, n, entry, c.p1, ...).  pool.take(size) / pool.give(OpVec&&)
// recycle op arrays.  Returns 0 (done: ops, *exit), 1 (a segment reached an
// unclassified position: the caller walks sequentially) or -1 (out of host memory).
template <class Pool, class Clock>
int walk_split(const Src& c, uint64_t n, const std::vector<uint64_t>& st, const BasisInfo& bi, bool final_src,
               int tail_match, OpVec& ops, uint64_t* exit, Pool& pool, Clock clock, SplitTiming* tm,
               OpCounts* counts = nullptr) {
    const int T = (int)st.size() - 1;
    const uint64_t nh = c.nahit + c.hpos.size();
    std::vector<OpVec> part(T);
    std::vector<uint64_t> ex(T, 0), need(T, 0);
    std::vector<int> rc(T, 0);
    const double t0 = clock();
    OpVec joined = pool.take(nh);  // before the segments' arrays, so they do not take it
    for (int t = 0; t < T; ++t) part[t] = pool.take(2 * nh / T + 64);
    struct Give {
        std::vector<OpVec>& v;
        Pool& pool;
        ~Give() {
            for (auto& x : v) pool.give(std::move(x));
        }
    } give{part, pool};
    std::vector<double> tseg(T, 0.0);
    auto seg = [&](int t, uint64_t from) {
        const double ts = clock();
        // walk into a vector whose header lives on this thread's stack: the segments'
        // headers sit side by side in `part`, and every push_back writes its end pointer
        // (false sharing made 8 concurrent segments ~8x slower than one)
        OpVec local;
        local.swap(part[t]);
        local.clear();
        const bool fin = final_src && t == T - 1;
        uint64_t e = 0, nd = 0;
        const int r = walk_src(c, n, from, st[t + 1], bi, fin, tail_match, local, &e, &nd);
        local.swap(part[t]);
        rc[t] = r;
        ex[t] = e;
        need[t] = nd;
        tseg[t] = clock() - ts;
    };
    if (!run_parallel(T, [&](int t) { seg(t, st[t]); })) return -1;
    const double t_walk = clock();
    if (rc[0]) return 1;
    for (int t = 1; t < T; ++t) {
        if (ex[t - 1] != st[t]) seg(t, ex[t - 1]);
        if (rc[t]) return 1;
    }
    // join: the first op of segment t merges into the joined list's last when both are
    // Data and contiguous
    std::vector<size_t> at(T + 1, 0), skip(T, 0);
    bool last_data = false;  // the joined list so far ends with a Data op ending at last_end
    uint64_t last_end = 0;
    for (int t = 0; t < T; ++t) {
        const OpVec& v = part[t];
        if (!v.empty() && last_data && v[0].kind == SYDELTA_OP_DATA && last_end == v[0].a) {
            skip[t] = 1;
            last_end += v[0].b;
        }
        at[t + 1] = at[t] + v.size() - skip[t];
        if (v.size() > skip[t]) {
            last_data = v.back().kind == SYDELTA_OP_DATA;
            last_end = v.back().a + v.back().b;
        }
    }
    const double t_chain = clock();
    ops.swap(joined);
    pool.give(std::move(joined));
    ops.resize(at[T]);
    struct alignas(64) Cnt {
        uint64_t data = 0, lit = 0;
    };
    std::vector<Cnt> cnt(T);
    if (!run_parallel(T, [&](int t) {
            if (part[t].size() <= skip[t]) return;
            const sydelta_op* from = part[t].data() + skip[t];
            const size_t m = part[t].size() - skip[t];
            memcpy(ops.data() + at[t], from, m * sizeof(sydelta_op));
            if (!counts) return;
            uint64_t nd = 0, lit = 0;
            for (size_t i = 0; i < m; ++i) {
                const bool d = from[i].kind != SYDELTA_OP_COPY;
                nd += d;
                lit += d ? from[i].b : 0;
            }
            cnt[t].data = nd;
            cnt[t].lit = lit;
        }))
        return -1;
    // merged lengths: the op before each skipped one absorbs it (a run of skipped
    // segments adds up in the same op, in order)
    for (int t = 1; t < T; ++t)
        if (skip[t]) ops[at[t] - 1].b += part[t][0].b;
    if (counts) {  // a merged Data op's bytes stay in the total
        *counts = OpCounts{};
        for (int t = 0; t < T; ++t) {
            counts->data_ops += cnt[t].data;
            counts->literal_bytes += cnt[t].lit + (skip[t] ? part[t][0].b : 0);
        }
        counts->copy_ops = ops.size() - counts->data_ops;
    }
    *exit = ex[T - 1];
    if (tm) {
        tm->walk_ms = t_walk - t0;
        tm->seg_max_ms = *std::max_element(tseg.begin(), tseg.end());
        tm->seg_min_ms = *std::min_element(tseg.begin(), tseg.end());
        tm->chain_ms = t_chain - t_walk;
        tm->join_ms = clock() - t_chain;
    }
    return 0;
}

}  // namespace walk
}  // namespace sydelta
