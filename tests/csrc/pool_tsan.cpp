// pool_tsan.cpp — the shared host pool (sydelta_walk.hpp HostPool / run_parallel)
// under ThreadSanitizer: 10 caller threads at once, each running split walks over 2, 3
// and 8 segments on its own synthetic source (the re-entrant shape of 10 concurrent
// file transfers), every result checked against the same walk run serially.  Built
// and run by tests/test_host_sanitizers.py; no GPU, no library link.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <thread>
#include <vector>

#include "sydelta_walk.hpp"

using namespace sydelta::walk;

struct Pool {
    OpVec take(size_t) { return OpVec(); }
    void give(OpVec&&) {}
};

static bool same(const OpVec& a, const OpVec& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i].kind != b[i].kind || a[i].a != b[i].a || a[i].b != b[i].b) return false;
    return true;
}

static int caller(int id, int iters) {
    std::mt19937_64 rng(1000 + id);
    int bad = 0;
    for (int it = 0; it < iters; ++it) {
        const uint64_t n = 1 + rng() % 32, flen = n + rng() % 20000;
        Src c;
        c.flen = c.len = flen;
        c.p1 = flen - n + 1;
        c.nblk = (c.p1 + n - 1) / n;
        for (uint64_t p = 0; p < c.p1; ++p)
            if (rng() % 23 == 0) {
                c.hpos.push_back(p);
                c.hblk.push_back((uint32_t)(rng() % 50));
            }
        const BasisInfo bi{0, 50, 1 + rng() % n};
        OpVec ref;
        uint64_t rexit = 0, need = 0;
        walk_src(c, n, 0, c.p1, bi, true, 0, ref, &rexit, &need);
        for (int T : {2, 3, 8}) {
            OpVec ops;
            uint64_t ex = 0;
            Pool pool;
            const int r = walk_split(c, n, split_points(c, n, 0, T), bi, true, 0, ops, &ex, pool, [] { return 0.0; },
                                     nullptr);
            if (r != 0 || ex != rexit || !same(ops, ref)) ++bad;
        }
        // a plain batch on the shared pool
        std::vector<uint64_t> acc(64, 0);
        run_parallel(64, [&](int t) { acc[t] = (uint64_t)t * t; });
        for (int t = 0; t < 64; ++t)
            if (acc[t] != (uint64_t)t * t) ++bad;
    }
    return bad;
}

int main() {
    std::vector<std::thread> th;
    std::vector<int> bad(10, 0);
    for (int i = 0; i < 10; ++i) th.emplace_back([&, i] { bad[i] = caller(i, 40); });
    for (auto& t : th) t.join();
    int tot = 0;
    for (int b : bad) tot += b;
    if (tot) {
        fprintf(stderr, "%d mismatches\n", tot);
        return 1;
    }
    printf("pool_tsan ok: %d pool threads\n", HostPool::get().size());
    return 0;
}
