// walk_bench_c4.cpp — host timing of the batched greedy walks (sydelta_walk.hpp walk_src)
// on the C4 shape: 10 000 sources of 1 MiB + 1 byte at bs 4096 (256 blocks), a 1-byte
// insertion at a random offset (aligned probe hits before it, one scan hit per block at
// the shifted phase after it, those blocks scanned) and 16 substituted bytes (their
// blocks miss and are scanned).  Per-file op vectors like sydelta_delta's.  CPU only.
//   clang++ -O3 -std=c++17 -I include -I sy_amd/csrc tools/walk_bench_c4.cpp -o build/walk_bench_c4 -lpthread
#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <stdio.h>
#include <thread>
#include <vector>

#include "sydelta_walk.hpp"

using namespace sydelta::walk;

int main(int argc, char** argv) {
    const uint64_t n = 4096, fsz = 1 << 20, nb = fsz / n;
    const int nf = argc > 1 ? atoi(argv[1]) : 10000;
    const int T = argc > 2 ? atoi(argv[2]) : 8;
    std::mt19937_64 rng(4);
    std::vector<Src> src(nf);
    for (int f = 0; f < nf; ++f) {
        Src& c = src[f];
        c.flen = c.len = fsz + 1;
        c.p0 = 0;
        c.p1 = fsz + 1 - n + 1;
        c.kb = 0;
        c.nblk = (c.p1 + n - 1) / n;
        c.probed = true;
        c.ahit.assign(c.nblk, kNoBlk);
        c.scanned.assign(c.nblk, 0);
        const uint64_t ins = rng() % (fsz + 1);
        std::vector<uint8_t> edited(nb + 1, 0);
        for (int j = 0; j < 16; ++j) edited[(rng() % (fsz + 1)) / n] = 1;
        for (uint64_t k = 0; k < c.nblk; ++k) {
            const uint64_t p = k * n;
            if (p + n <= ins && !edited[k]) { c.ahit[k] = (uint32_t)(f * nb + k); ++c.nahit; }
            else c.scanned[k] = 1;
        }
        for (uint64_t b = 0; b < nb; ++b) {  // shifted copies of basis block b at b*n + 1
            const uint64_t p = b * n + 1;
            if (b * n + n <= ins || p >= c.p1 || edited[b] || (p / n < c.nblk && !c.scanned[p / n])) continue;
            c.hpos.push_back(p);
            c.hblk.push_back((uint32_t)(f * nb + b));
        }
    }
    const bool keep = argc > 3 && atoi(argv[3]) == 1;  // 1: op vectors kept between repetitions (warm)
    std::vector<OpVec> kept(nf);
    for (int rep = 0; rep < 5; ++rep) {
        std::vector<OpVec> out(nf);
        if (keep) out.swap(kept);
        for (auto& o : out) o.clear();
        std::atomic<int> next{0};
        const auto t0 = std::chrono::steady_clock::now();
        auto worker = [&] {
            for (;;) {
                const int f0 = next.fetch_add(32);
                if (f0 >= nf) break;
                for (int f = f0; f < std::min(nf, f0 + 32); ++f) {
                    const BasisInfo bi{(uint64_t)f * nb, nb, n};
                    uint64_t exit = 0, need = 0;
                    walk_src(src[f], n, 0, src[f].p1, bi, true, 0, out[f], &exit, &need);
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(worker);
        worker();
        for (auto& t : th) t.join();
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        size_t ops = 0;
        for (auto& o : out) ops += o.size();
        const auto t1 = std::chrono::steady_clock::now();
        if (keep) out.swap(kept);
        out.clear();
        out.shrink_to_fit();
        const double fms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        printf("%d files, %d threads: walks %.3f ms (%zu ops, %.1f ns/op/thread), free %.3f ms\n", nf, T, ms, ops,
               ms * 1e6 * T / ops, fms);
    }
}
