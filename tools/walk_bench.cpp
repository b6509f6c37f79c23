// walk_bench.cpp — host timing of the greedy walk (sydelta_walk.hpp) on the C5 shape:
// one 8 GiB chunk at bs 8192 = 1 Mi blocks, aligned probe hits on 99 % of them, the 1 %
// edited blocks scanned (no hit inside).  Not product code; CPU only.
//   g++ -O3 -std=c++17 -I include -I sy_amd/csrc tools/walk_bench.cpp -o build/walk_bench -lpthread
#include <algorithm>
#include <chrono>
#include <random>
#include <stdio.h>
#include <vector>

#include "sydelta_walk.hpp"

using namespace sydelta::walk;

struct Pool {  // recycles arrays across repetitions, best fit like the library's take_ops
    std::vector<OpVec> v;
    OpVec take(size_t want) {
        size_t best = v.size();
        for (size_t i = 0; i < v.size(); ++i)
            if (v[i].capacity() >= want && (best == v.size() || v[i].capacity() < v[best].capacity())) best = i;
        OpVec o;
        if (best < v.size()) {
            o.swap(v[best]);
            v.erase(v.begin() + best);
        }
        o.clear();
        o.reserve(want);
        return o;
    }
    void give(OpVec&& o) { v.push_back(std::move(o)); }
};

int main(int argc, char** argv) {
    const uint64_t n = 8192, nblk = 1 << 20, flen = n * nblk;
    const int T = argc > 1 ? atoi(argv[1]) : 8;
    Src c;
    c.flen = c.len = flen;
    c.p0 = 0;
    c.p1 = flen - n + 1;
    c.kb = 0;
    c.nblk = nblk;
    c.probed = true;
    c.ahit.resize(nblk);
    c.scanned.assign(nblk, 0);
    std::mt19937_64 rng(1);
    for (uint64_t k = 0; k < nblk; ++k) {
        const bool edited = rng() % 100 == 0;
        c.ahit[k] = edited ? kNoBlk : (uint32_t)k;
        if (edited) c.scanned[k] = 1;
        else ++c.nahit;
    }
    const BasisInfo bi{0, nblk, n};
    Pool pool;
    OpVec ops, sops;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<double> tser, tsplit;
    for (int rep = 0; rep < reps; ++rep) {
        ops.clear();
        ops.reserve(2 * nblk);
        uint64_t exit = 0, need = 0;
        auto t0 = std::chrono::steady_clock::now();
        const int r = walk_src(c, n, 0, c.p1, bi, true, 0, ops, &exit, &need);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        pool.give(std::move(sops));
        sops = OpVec();
        uint64_t sexit = 0;
        auto t1 = std::chrono::steady_clock::now();
        SplitTiming tm;
        const auto tz = std::chrono::steady_clock::now();
        const int r2 = walk_split(c, n, split_points(c, n, 0, T), bi, true, 0, sops, &sexit, pool,
                                  [&] { return std::chrono::duration<double, std::milli>(
                                            std::chrono::steady_clock::now() - tz).count(); },
                                  &tm);
        const double ms2 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        bool same = sops.size() == ops.size();
        for (size_t i = 0; same && i < ops.size(); ++i)
            same = ops[i].kind == sops[i].kind && ops[i].a == sops[i].a && ops[i].b == sops[i].b;
        if (rep) { tser.push_back(ms); tsplit.push_back(ms2); }
        if (reps <= 5) printf("serial walk %.3f ms (%zu ops, rc %d)  split walk over %d segments %.3f ms (rc %d, %s): walk %.3f "
               "(segments %.3f-%.3f) chain %.3f join %.3f\n", ms, ops.size(), r, T, ms2, r2,
               same ? "same ops" : "DIFFERENT", tm.walk_ms, tm.seg_min_ms, tm.seg_max_ms, tm.chain_ms, tm.join_ms);
    }
    if (!tser.empty()) {
        std::sort(tser.begin(), tser.end());
        std::sort(tsplit.begin(), tsplit.end());
        printf("median of %zu: serial %.3f ms, split over %d segments %.3f ms\n", tser.size(), tser[tser.size() / 2],
               T, tsplit[tsplit.size() / 2]);
    }
    return 0;
}
