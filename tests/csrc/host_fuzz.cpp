// host_fuzz.cpp — the library's host logic under AddressSanitizer + UBSan (VERDICT r01
// item 9; built and run by tests/test_host_sanitizers.py, CPU only, no GPU call):
//   walk   the greedy walk (sydelta_walk.hpp: walk_src with on-demand classification,
//          walk_split over 2/3/8 segments) on random synthetic hit lists against a
//          restated greedy walk (generator.rs:116-221 / 283-379)
//   join   sydelta_delta_append of random chunk deltas against a restated merge
//   json   the serde_json parsers on a corpus of malformed, mutated and huge inputs;
//          writer -> parser -> writer round trips (ssh.rs:967-1003, sy-remote.rs:146-175)
//   ops    sydelta_delta_from_ops validation
// Exit status 0 and "host_fuzz ok" on success; any sanitizer report aborts.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "sydelta.h"
#include "sydelta_walk.hpp"

using namespace sydelta::walk;

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            abort();                                                           \
        }                                                                      \
    } while (0)

static std::mt19937_64 rng(0x5E1D0F22);
static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

// ---------------------------------------------------------------------------
// walk
// ---------------------------------------------------------------------------
struct Case {
    uint64_t n, flen, entry;
    BasisInfo bi;
    bool final_src;
    int tail_match;
    std::vector<uint32_t> H;  // per full-window position: hit block or kNoBlk
};

// The greedy walk restated over the hit function (generator.rs:116-221).
static std::vector<sydelta_op> ref_walk(const Case& k, uint64_t p1, uint64_t* exit) {
    std::vector<sydelta_op> ops;
    auto data = [&](uint64_t a, uint64_t b) {
        if (b > a) ops.push_back({SYDELTA_OP_DATA, 0, a, b - a});
    };
    auto copy = [&](uint64_t g) {
        const uint64_t b = g - k.bi.blk_base;
        ops.push_back({SYDELTA_OP_COPY, 0, b * k.n, b + 1 == k.bi.nblocks ? k.bi.last_size : k.n});
    };
    uint64_t x = k.entry, lit = k.entry;
    for (;;) {
        uint64_t p = x;
        while (p < p1 && k.H[p] == kNoBlk) ++p;
        if (p >= p1) break;
        data(lit, p);
        copy(k.H[p]);
        x = p + k.n;
        lit = x;
    }
    if (!k.final_src) {
        data(lit, p1);
        *exit = std::max(x, p1);
        return ops;
    }
    if (k.tail_match && k.bi.nblocks && k.flen >= k.bi.last_size && k.flen - k.bi.last_size >= lit) {
        data(lit, k.flen - k.bi.last_size);
        copy(k.bi.blk_base + k.bi.nblocks - 1);
        lit = k.flen;
    }
    data(lit, k.flen);
    *exit = k.flen;
    return ops;
}

static bool same(const OpVec& a, const std::vector<sydelta_op>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i].kind != b[i].kind || a[i].a != b[i].a || a[i].b != b[i].b) return false;
    return true;
}

// Hits of block k's interior positions (k*n+1 .. k*n+n-1, below p1).
static void block_hits(const Case& k, uint64_t blk, uint64_t p1, std::vector<uint64_t>& pos,
                       std::vector<uint32_t>& b) {
    pos.clear();
    b.clear();
    for (uint64_t p = blk * k.n + 1; p < std::min(p1, blk * k.n + k.n); ++p)
        if (k.H[p] != kNoBlk) { pos.push_back(p); b.push_back(k.H[p]); }
}

struct Pool {
    std::vector<OpVec> v;
    OpVec take(size_t want) {
        OpVec o;
        if (!v.empty()) { o.swap(v.back()); v.pop_back(); }
        o.clear();
        o.reserve(std::min<size_t>(want, 1 << 16));
        return o;
    }
    void give(OpVec&& o) {
        if (v.size() < 4) v.push_back(std::move(o));
    }
};

static void walk_case(int it) {
    Case k;
    const uint64_t nsel[] = {1, 2, 3, 7, 16, 64};
    k.n = nsel[rnd(6)];
    k.flen = rnd(it % 7 == 0 ? 40 : 3000);
    const uint64_t p1 = k.flen >= k.n ? k.flen - k.n + 1 : 0;
    k.entry = p1 ? rnd(it % 3 == 0 ? p1 : 1) : 0;
    k.bi.blk_base = rnd(3) * 5;
    k.bi.nblocks = 1 + rnd(40);
    k.bi.last_size = 1 + rnd(k.n);
    k.final_src = rnd(4) != 0;
    // the device's tail check runs only when the file holds the last block (tail_flags)
    k.tail_match = k.flen >= k.bi.last_size ? (int)rnd(2) : 0;
    const double dens[] = {0.0, 0.003, 0.05, 0.3, 1.0};
    const double d = dens[rnd(5)];
    std::uniform_real_distribution<double> U(0, 1);
    k.H.assign(p1, kNoBlk);
    for (uint64_t p = 0; p < p1; ++p)
        if (U(rng) < d) k.H[p] = (uint32_t)(k.bi.blk_base + rnd(k.bi.nblocks));
    uint64_t rexit = 0;
    const std::vector<sydelta_op> expect = ref_walk(k, p1, &rexit);

    Src c;
    c.flen = k.flen;
    c.len = k.flen;
    c.p0 = 0;
    c.p1 = p1;
    c.kb = 0;
    c.nblk = (p1 + k.n - 1) / k.n;
    c.probed = rnd(2) != 0;
    std::vector<uint64_t> pos;
    std::vector<uint32_t> blk;
    if (c.probed) {
        c.ahit.assign(c.nblk, kNoBlk);
        c.scanned.assign(c.nblk, 0);
        const bool phase = rnd(2) != 0;
        if (phase) {
            c.ppos.assign(c.nblk, kUnknownNone);
            c.phit.assign(c.nblk, kNoBlk);
        }
        for (uint64_t b = 0; b < c.nblk; ++b) {
            c.ahit[b] = k.H[b * k.n];
            c.nahit += c.ahit[b] != kNoBlk;
            if (rnd(3) == 0) {  // scanned up front
                c.scanned[b] = 1;
                block_hits(k, b, p1, pos, blk);
                merge_hits(c, pos, blk);
            } else if (phase && k.n > 1 && rnd(2)) {  // one phase-probed window inside it
                const uint64_t q = b * k.n + 1 + rnd(k.n - 1);
                if (q < p1) {
                    c.ppos[b] = q;
                    c.phit[b] = k.H[q];
                    if (k.H[q] != kNoBlk) merge_hits(c, {q}, {k.H[q]});
                }
            }
        }
    } else {
        for (uint64_t p = 0; p < p1; ++p)
            if (k.H[p] != kNoBlk) { pos.push_back(p); blk.push_back(k.H[p]); }
        merge_hits(c, pos, blk);
    }
    // the sequential walk, classifying on demand (Classifier::walk)
    OpVec ops;
    uint64_t exit = 0;
    for (int round = 0;; ++round) {
        uint64_t need = 0;
        const int r = walk_src(c, k.n, k.entry, p1, k.bi, k.final_src, k.tail_match, ops, &exit, &need);
        if (!r) break;
        CHECK(round < 100000);
        CHECK(c.probed && need >= k.entry && need < p1);
        const uint64_t b = need / k.n;
        CHECK(!c.scanned[b]);
        c.scanned[b] = 1;
        block_hits(k, b, p1, pos, blk);
        merge_hits(c, pos, blk);
    }
    if (!same(ops, expect) || exit != rexit) {
        fprintf(stderr, "walk mismatch it=%d n=%llu flen=%llu entry=%llu: %zu vs %zu ops\n", it,
                (unsigned long long)k.n, (unsigned long long)k.flen, (unsigned long long)k.entry, ops.size(),
                expect.size());
        abort();
    }
    // the split walk over 2/3/8 segments on the fully classified source
    if (c.probed)
        for (uint64_t b = 0; b < c.nblk; ++b)
            if (!c.scanned[b]) {
                c.scanned[b] = 1;
                block_hits(k, b, p1, pos, blk);
                merge_hits(c, pos, blk);
            }
    Pool pool;
    for (int T : {2, 3, 8}) {
        if (p1 <= k.entry) continue;
        const std::vector<uint64_t> st = split_points(c, k.n, k.entry, T);
        OpVec sops;
        uint64_t sexit = 0;
        SplitTiming tm;
        OpCounts oc;
        const int r = walk_split(c, k.n, st, k.bi, k.final_src, k.tail_match, sops, &sexit, pool,
                                 [] { return 0.0; }, &tm, &oc);
        CHECK(r == 0);
        if (!same(sops, expect) || sexit != rexit) {
            fprintf(stderr, "split walk mismatch it=%d T=%d (%zu segments)\n", it, T, st.size() - 1);
            abort();
        }
        {  // the join's op counts equal a direct count of the joined list
            uint64_t nd = 0, lit = 0;
            for (auto& o : sops)
                if (o.kind != SYDELTA_OP_COPY) { ++nd; lit += o.b; }
            CHECK(oc.data_ops == nd && oc.literal_bytes == lit && oc.copy_ops == sops.size() - nd);
        }
    }
}

// ---------------------------------------------------------------------------
// join: sydelta_delta_append
// ---------------------------------------------------------------------------
static void join_case() {
    sydelta_delta* acc = sydelta_delta_new(1000, 16);
    CHECK(acc);
    std::vector<sydelta_op> expect;
    const int parts = 1 + (int)rnd(6);
    uint64_t at = 0;
    for (int t = 0; t < parts; ++t) {
        std::vector<sydelta_op> v;
        const int m = (int)rnd(5);
        for (int i = 0; i < m; ++i) {
            if (rnd(2)) {
                v.push_back({SYDELTA_OP_COPY, 0, rnd(100) * 16, 16});
                at += 16;
            } else {
                const uint64_t len = 1 + rnd(50);
                v.push_back({SYDELTA_OP_DATA, 0, at, len});
                at += len;
            }
        }
        // restated merge: a leading Data op contiguous with the trailing one joins it
        for (size_t i = 0; i < v.size(); ++i) {
            if (i == 0 && !expect.empty() && expect.back().kind == SYDELTA_OP_DATA && v[0].kind == SYDELTA_OP_DATA &&
                expect.back().a + expect.back().b == v[0].a)
                expect.back().b += v[0].b;
            else
                expect.push_back(v[i]);
        }
        sydelta_delta* part = sydelta_delta_from_ops(v.empty() ? nullptr : v.data(), v.size(), 1000, 16);
        CHECK(part);
        CHECK(sydelta_delta_append(acc, part) == SYDELTA_OK);
        sydelta_delta_free(part);
    }
    CHECK(sydelta_delta_num_ops(acc) == expect.size());
    const sydelta_op* o = sydelta_delta_ops(acc);
    for (size_t i = 0; i < expect.size(); ++i)
        CHECK(o[i].kind == expect[i].kind && o[i].a == expect[i].a && o[i].b == expect[i].b);
    sydelta_delta_free(acc);
}

// ---------------------------------------------------------------------------
// json
// ---------------------------------------------------------------------------
static std::string delta_text(const sydelta_delta* d, const uint8_t* lit, uint64_t lit_len) {
    uint64_t len = 0;
    CHECK(sydelta_delta_to_json(d, lit, lit_len, nullptr, 0, &len) == SYDELTA_OK);
    std::string s(len, '\0');
    uint64_t len2 = 0;
    CHECK(sydelta_delta_to_json(d, lit, lit_len, &s[0], len, &len2) == SYDELTA_OK && len2 == len);
    return s;
}

// Parse; on success the writer reproduces a text that parses to the same delta.
static void parse_delta(const std::string& t) {
    sydelta_delta* d = nullptr;
    if (sydelta_delta_from_json(t.data(), t.size(), &d) != SYDELTA_OK) {
        CHECK(d == nullptr);
        CHECK(sydelta_last_error() != nullptr);
        return;
    }
    CHECK(d);
    const std::string w = delta_text(d, nullptr, 0);
    sydelta_delta* d2 = nullptr;
    CHECK(sydelta_delta_from_json(w.data(), w.size(), &d2) == SYDELTA_OK);
    CHECK(delta_text(d2, nullptr, 0) == w);
    sydelta_delta_free(d2);
    sydelta_delta_free(d);
}

static void parse_sigs(const std::string& t) {
    sydelta_block_checksum* s = nullptr;
    uint64_t n = 0;
    if (sydelta_checksums_from_json(t.data(), t.size(), &s, &n) != SYDELTA_OK) return;
    const uint64_t len = sydelta_checksums_to_json(s, n, nullptr, 0);
    std::string w(len, '\0');
    CHECK(sydelta_checksums_to_json(s, n, &w[0], len) == len);
    sydelta_block_checksum* s2 = nullptr;
    uint64_t n2 = 0;
    CHECK(sydelta_checksums_from_json(w.data(), w.size(), &s2, &n2) == SYDELTA_OK && n2 == n);
    CHECK(n == 0 || memcmp(s, s2, n * sizeof(*s)) == 0);
    sydelta_checksums_free(s2);
    sydelta_checksums_free(s);
}

static std::string mutate(std::string t) {
    const int k = 1 + (int)rnd(4);
    for (int i = 0; i < k && !t.empty(); ++i) {
        const uint64_t p = rnd(t.size());
        switch (rnd(6)) {
            case 0: t[p] = (char)rnd(256); break;                                  // any byte
            case 1: t.erase(p, 1 + rnd(8)); break;                                 // delete
            case 2: t.insert(p, 1, "{}[]\",:-.0eE\\u"[rnd(15)]); break;            // structural
            case 3: t.resize(p); break;                                            // truncate
            case 4: t.insert(p, t.substr(rnd(t.size()), rnd(32))); break;          // duplicate a span
            default: t.insert(p, std::string(1 + rnd(4), ' ')); break;
        }
    }
    return t;
}

static void json_fuzz() {
    // hand-written malformed and edge inputs
    const char* corpus[] = {
        "", " ", "{", "}", "[]", "null", "{\"ops\":[]}", "{\"ops\":[],\"source_size\":0}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4096}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4096,\"ops\":[]}",
        "{\"ops\":[{\"Copy\":{\"offset\":1,\"size\":2}}],\"source_size\":3,\"block_size\":4}",
        "{\"ops\":[{\"Copy\":{\"offset\":1,\"offset\":1,\"size\":2}}],\"source_size\":3,\"block_size\":4}",
        "{\"ops\":[{\"Data\":[1,2,256]}],\"source_size\":3,\"block_size\":4}",
        "{\"ops\":[{\"Data\":[1,2,-1]}],\"source_size\":3,\"block_size\":4}",
        "{\"ops\":[{\"Data\":[1,2,3]}],\"source_size\":18446744073709551616,\"block_size\":4}",
        "{\"ops\":[{\"Data\":[1,2,3]}],\"source_size\":1e999999,\"block_size\":4}",
        "{\"ops\":[{\"Bogus\":[]}],\"source_size\":3,\"block_size\":4}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":\"\\ud800\"}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":\"\\u12\"}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":\"\\q\"}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":tru}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":01}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":1.}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":-}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":[1,2,]}",
        "{\"ops\":[],\"source_size\":0,\"block_size\":4} trailing",
        "[{\"index\":0,\"offset\":0,\"size\":1,\"weak\":4294967296,\"strong\":0}]",
        "[{\"index\":0,\"offset\":0,\"size\":1,\"weak\":1,\"strong\":18446744073709551615}]",
        "[{\"index\":0,\"index\":0,\"offset\":0,\"size\":1,\"weak\":1,\"strong\":0}]",
    };
    for (const char* c : corpus) {
        parse_delta(c);
        parse_sigs(c);
        std::string s(c);
        s.push_back('\0');  // an embedded NUL inside the length
        parse_delta(s);
    }
    // deep nesting in a skipped value, beyond and within the depth limit
    for (int depth : {100, 127, 129, 5000, 200000}) {
        std::string t = "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":";
        t += std::string(depth, '[') + std::string(depth, ']') + "}";
        parse_delta(t);
        std::string u = "{\"ops\":[],\"source_size\":0,\"block_size\":4,\"x\":" + std::string(depth, '[');
        parse_delta(u);
    }
    // writer -> mutations -> parser, for random deltas with literal bytes
    for (int it = 0; it < 300; ++it) {
        std::vector<uint8_t> lit(1 + rnd(3000));
        for (auto& b : lit) b = (uint8_t)rnd(256);
        std::vector<sydelta_op> ops;
        uint64_t at = 0;
        const int m = (int)rnd(12);
        for (int i = 0; i < m; ++i) {
            if (rnd(2)) {
                ops.push_back({SYDELTA_OP_COPY, 0, rng(), rng()});
            } else if (at < lit.size()) {
                const uint64_t len = std::min<uint64_t>(1 + rnd(400), lit.size() - at);
                ops.push_back({SYDELTA_OP_DATA, 0, at, len});
                at += len;
            }
        }
        sydelta_delta* d = sydelta_delta_from_ops(ops.empty() ? nullptr : ops.data(), ops.size(), rng(), 1 + rnd(1 << 20));
        CHECK(d);
        const std::string t = delta_text(d, lit.data(), lit.size());
        parse_delta(t);
        for (int k = 0; k < 20; ++k) parse_delta(mutate(t));
        sydelta_delta_free(d);
        // checksums
        std::vector<sydelta_block_checksum> sigs(rnd(20));
        for (size_t i = 0; i < sigs.size(); ++i)
            sigs[i] = {i, i * 4096, 4096, (uint32_t)rng(), 0, rng()};
        const uint64_t len = sydelta_checksums_to_json(sigs.data(), sigs.size(), nullptr, 0);
        std::string st(len, '\0');
        CHECK(sydelta_checksums_to_json(sigs.data(), sigs.size(), &st[0], len) == len);
        parse_sigs(st);
        for (int k = 0; k < 20; ++k) parse_sigs(mutate(st));
    }
    // a huge delta: 1 Mi Copy ops + a 16 MiB Data run
    {
        std::vector<sydelta_op> ops(1 << 20);
        for (size_t i = 0; i < ops.size(); ++i) ops[i] = {SYDELTA_OP_COPY, 0, i * 4096, 4096};
        std::vector<uint8_t> lit(16 << 20);
        for (size_t i = 0; i < lit.size(); ++i) lit[i] = (uint8_t)(i * 131);
        ops.push_back({SYDELTA_OP_DATA, 0, 0, lit.size()});
        sydelta_delta* d = sydelta_delta_from_ops(ops.data(), ops.size(), 1ull << 40, 4096);
        CHECK(d);
        const std::string t = delta_text(d, lit.data(), lit.size());
        sydelta_delta* d2 = nullptr;
        CHECK(sydelta_delta_from_json(t.data(), t.size(), &d2) == SYDELTA_OK);
        CHECK(sydelta_delta_num_ops(d2) == ops.size());
        CHECK(memcmp(sydelta_delta_literal(d2, ops.size() - 1), lit.data(), lit.size()) == 0);
        CHECK(delta_text(d2, nullptr, 0) == t);
        sydelta_delta_free(d2);
        sydelta_delta_free(d);
    }
}

static void ops_validation() {
    sydelta_op bad[2] = {{SYDELTA_OP_COPY, 0, 0, 4}, {7, 0, 0, 4}};
    CHECK(sydelta_delta_from_ops(bad, 2, 8, 4) == nullptr);
    CHECK(sydelta_last_error() != nullptr);
    CHECK(sydelta_delta_from_ops(nullptr, 3, 8, 4) == nullptr);
    sydelta_delta* d = sydelta_delta_from_ops(nullptr, 0, 0, 4);
    CHECK(d && sydelta_delta_num_ops(d) == 0);
    sydelta_delta_free(d);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 3000;
    for (int it = 0; it < iters; ++it) walk_case(it);
    for (int it = 0; it < 500; ++it) join_case();
    ops_validation();
    json_fuzz();
    printf("host_fuzz ok: %d walks\n", iters);
    return 0;
}
