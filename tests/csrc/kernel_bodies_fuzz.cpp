// kernel_bodies_fuzz.cpp — TEST INFRASTRUCTURE, built with -fsanitize=address,undefined by
// tests/test_host_sanitizers.py.  The per-thread bodies the gfx950 kernels run, driven on
// the CPU with every array allocated at exactly the size the kernels assume, so an index
// outside its array (a GPU fault on the device) is an AddressSanitizer report here:
//
//  * the device walk (sydelta_chain.hpp, K5b): random classified sources -- probed and
//    unprobed, scanned and unscanned blocks, dense and sparse hits, entries inside the
//    source, final and non-final -- resolved in launch_chain's order with the marking
//    levels' threads in a random order each, then assembled as walk_device does; the op
//    list and exit equal walk_src's (sydelta_walk.hpp), and a path that walk_src cannot
//    finish (an unclassified position) is exactly one that reaches UNK;
//  * the zstd block coder (sydelta_zstd.hpp, K7z): block_content_seq on random texts with
//    its scratch as separate exact-size arrays; and a thread-by-thread replica of
//    k_zstd_block's parallel bit scatter (runs of 144 aligned bytes per thread, suffix
//    sums, OR-ed words) whose streams must equal the sequential writer's bytes;
//  * the zstd repeat-offset coder (rep_code) against a restatement of the decoder's
//    history rules started from a history the coder does not know;
//  * the signature JSON writer (sydelta_sigjson.hpp, K7s): k_sigjson_write's tiles on
//    random signatures, each tile's text staged in an array of exactly its length and
//    stored chunk by chunk (chunks shuffled) into an output of exactly the text's length
//    at a random alignment; the text equals a printf-built one and the length bounds hold;
//  * its parse (K7p): texts in exact-size arrays parse back to their signature, and a
//    mutated text is refused or is the compact text of what it parses to;
//  * the Delta JSON parse (sydelta_dparse.hpp, K7d): the same two properties for the ops
//    region of random deltas' compact text.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "sydelta_chain.hpp"
#include "sydelta_sigjson.hpp"
#include "sydelta_dparse.hpp"
#include "sydelta_walk.hpp"
#include "sydelta_zstd.hpp"

using namespace sydelta;

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
            abort();                                                      \
        }                                                                 \
    } while (0)

template <class T>
struct Arr {  // exact-size heap array (ASan-visible bounds)
    std::unique_ptr<T[]> p;
    explicit Arr(size_t n) : p(new T[n ? n : 1]) {
        if (!n) p.reset(new T[0]);
    }
    T* get() { return p.get(); }
};

// ---------------------------------------------------------------------------
// device walk
// ---------------------------------------------------------------------------
static int chain_case(std::mt19937_64& rng, uint64_t* walked_on_device) {
    auto U = [&](uint64_t lo, uint64_t hi) { return std::uniform_int_distribution<uint64_t>(lo, hi)(rng); };
    const uint64_t n = std::vector<uint64_t>{1, 2, 4, 7, 16, 64}[U(0, 5)];
    const uint64_t kb = U(0, 5), nblk = U(0, 300);
    walk::Src c;
    c.p0 = kb * n;
    c.p1 = nblk ? c.p0 + (nblk - 1) * n + U(1, n) : c.p0;
    c.kb = kb;
    c.nblk = nblk;
    c.flen = c.p1 + n - 1 + U(0, 3);
    c.len = c.flen;
    const bool final_src = U(0, 1);
    walk::BasisInfo bi{U(0, 1000), 60, U(1, n)};
    const double dense = std::vector<double>{0.0, 0.02, 0.3, 1.0}[U(0, 3)];
    const bool probed = U(0, 1) && nblk;
    auto rnd_blk = [&]() { return (uint32_t)(bi.blk_base + U(0, bi.nblocks - 1)); };
    if (probed) {
        c.probed = true;
        c.ahit.resize(nblk);
        c.scanned.assign(nblk, 0);
        for (uint64_t k = 0; k < nblk; ++k) {
            c.ahit[k] = U(0, 99) < 60 ? rnd_blk() : walk::kNoBlk;
            if (c.ahit[k] != walk::kNoBlk) ++c.nahit;
            c.scanned[k] = c.ahit[k] == walk::kNoBlk || U(0, 99) < 20;
        }
    }
    for (uint64_t p = c.p0; p < c.p1; ++p) {
        const uint64_t k = p / n - kb;
        if (probed && !c.scanned[k]) continue;
        const bool aligned_hit = probed && p % n == 0 && c.ahit[k] != walk::kNoBlk;
        if (aligned_hit) {
            if (U(0, 1)) { c.hpos.push_back(p); c.hblk.push_back(c.ahit[k]); }  // same hit from the scan
        } else if (std::uniform_real_distribution<double>(0, 1)(rng) < dense) {
            c.hpos.push_back(p);
            c.hblk.push_back(rnd_blk());
        }
    }
    const uint64_t entry = c.p1 > c.p0 ? c.p0 + U(0, c.p1 - c.p0 - 1) : c.p0;
    if (entry >= c.p1) return 0;
    const int tail_match = (int)U(0, 1);
    // reference
    OpVec ref;
    uint64_t rexit = 0, need = 0;
    const int rrc = walk::walk_src(c, n, entry, c.p1, bi, final_src, tail_match, ref, &rexit, &need);
    // device form: scan hits minus aligned duplicates, exact-size arrays
    std::vector<uint64_t> hp;
    std::vector<uint32_t> hb;
    for (size_t h = 0; h < c.hpos.size(); ++h) {
        const uint64_t p = c.hpos[h];
        if (probed && p % n == 0 && c.ahit[p / n - kb] != walk::kNoBlk) continue;
        hp.push_back(p);
        hb.push_back(c.hblk[h]);
    }
    const uint64_t H = hp.size(), M = (probed ? c.nahit : 0) + H, W = M + 2, nb = probed ? nblk : 0;
    const uint32_t K = chain::chain_levels(M);
    Arr<uint32_t> ahit(nb), aflag(nb + 1), apfx(nb + 1), ublk(M), hblk(H), jump(K * W), cnt(M + 1), off(M + 1);
    Arr<uint8_t> known(nb);
    Arr<uint64_t> hpos(H), upos(M);
    Arr<uint8_t> on(W);
    Arr<sydelta_op> ops(2 * M);
    Arr<chain::ChainResult> res(1);
    for (uint64_t k = 0; k < nb; ++k) ahit.get()[k] = c.ahit[k];
    for (uint64_t k = 0; k < nb; ++k) known.get()[k] = c.scanned[k];
    std::copy(hp.begin(), hp.end(), hpos.get());
    std::copy(hb.begin(), hb.end(), hblk.get());
    chain::ChainArgs a{};
    a.n = n; a.p1 = c.p1; a.kb = kb; a.nblk = nb; a.entry = entry; a.probed = probed; a.K = K;
    a.ahit = ahit.get(); a.known = known.get(); a.aflag = aflag.get(); a.apfx = apfx.get();
    a.hpos = hpos.get(); a.hblk = hblk.get(); a.H = H; a.M = M; a.upos = upos.get(); a.ublk = ublk.get();
    a.jump = jump.get(); a.on = on.get(); a.cnt = cnt.get(); a.off = off.get();
    a.blk_base = bi.blk_base; a.nblocks = bi.nblocks; a.last_size = bi.last_size;
    a.ops = ops.get(); a.res = res.get();
    // launch_chain's order (sydelta_kernels.hip), threads of the racy levels shuffled
    memset(a.res, 0, sizeof(chain::ChainResult));
    auto excl = [](const uint32_t* in, uint32_t* out, uint64_t m) {
        uint32_t acc = 0;
        for (uint64_t i = 0; i < m; ++i) { const uint32_t v = in[i]; out[i] = acc; acc += v; }
    };
    if (probed) {
        for (uint64_t k = 0; k <= nb; ++k) chain::chain_flag(a, k);
        excl(a.aflag, a.apfx, nb + 1);
        for (uint64_t k = 0; k < nb; ++k) chain::chain_place_aligned(a, k);
    }
    for (uint64_t h = 0; h < H; ++h) chain::chain_place_scan(a, h);
    for (uint64_t i = 0; i < W; ++i) chain::chain_succ(a, i);
    for (uint32_t l = 0; l + 1 < K; ++l)
        for (uint64_t i = 0; i < W; ++i) chain::chain_lift(a, l, i);
    memset(a.on, 0, W);
    chain::chain_entry(a);
    std::vector<uint64_t> order(W);
    std::iota(order.begin(), order.end(), 0);
    for (uint32_t l = K; l-- > 0;) {
        std::shuffle(order.begin(), order.end(), rng);
        for (uint64_t i : order) chain::chain_mark(a, l, i);
    }
    for (uint64_t i = 0; i <= M; ++i) chain::chain_count(a, i);
    excl(a.cnt, a.off, M + 1);
    for (uint64_t i = 0; i < M; ++i) {
        const uint64_t lit = chain::chain_emit(a, i);
        if (lit) { a.res->data_ops++; a.res->lit_bytes += lit; }
    }
    chain::chain_finish(a);
    const chain::ChainResult r = *a.res;
    CHECK(!r.bad);
    CHECK((r.unk != 0) == (rrc == 1));
    if (r.unk) return 0;
    // walk_device's assembly
    OpVec got;
    const bool lead = r.first < M && r.first_pos > entry;
    if (lead) got.push_back({SYDELTA_OP_DATA, 0, entry, r.first_pos - entry});
    for (uint64_t i = 0; i < r.nops; ++i) got.push_back(a.ops[i]);
    const uint64_t x = r.first < M ? r.last_pos + n : c.p1;
    const uint64_t lit = r.first < M ? x : entry;
    uint64_t exit = 0;
    walk::finish_walk(c, n, lit, x, c.p1, bi, final_src, tail_match, got, &exit);
    CHECK(exit == rexit);
    CHECK(got.size() == ref.size());
    for (size_t i = 0; i < got.size(); ++i)
        CHECK(got[i].kind == ref[i].kind && got[i].a == ref[i].a && got[i].b == ref[i].b);
    uint64_t nd = 0, lb = 0;
    for (uint64_t i = 0; i < r.nops; ++i)
        if (a.ops[i].kind == SYDELTA_OP_DATA) { ++nd; lb += a.ops[i].b; }
    CHECK(nd == r.data_ops && lb == r.lit_bytes);
    ++*walked_on_device;
    return 1;
}

// ---------------------------------------------------------------------------
// zstd
// ---------------------------------------------------------------------------
// k_zstd_block's entropy-only streams, thread by thread (256 threads, 144-byte aligned
// runs, suffix sums of the runs' bits, OR-ed 32-bit words): must equal the sequential
// writer's stream bytes.
static void scatter_replica(const uint8_t* in, uint32_t n, const zstd::HufCode& code, bool four,
                            std::vector<std::vector<uint8_t>>& streams) {
    constexpr uint32_t T = 256, R = 144;
    for (uint32_t st = 0; st < (four ? 4u : 1u); ++st) {
        uint32_t first, count;
        zstd::stream_range(n, four, st, first, count);
        const uint32_t nw = (count * zstd::kMaxBits + 1 + 31) / 32 + 1;
        Arr<uint32_t> words(nw);
        memset(words.get(), 0, 4 * nw);
        const uint32_t A = first & ~15u, lim = first + count;
        std::vector<uint32_t> part(T);
        for (uint32_t t = 0; t < T; ++t) {
            uint32_t bits = 0;
            for (uint32_t k = 0; k < R; ++k) {
                const uint32_t p = A + R * t + k;
                if (p >= first && p < lim) bits += code.len[in[p]];
            }
            part[t] = bits;
        }
        uint32_t total = 0;
        for (uint32_t t = 0; t < T; ++t) total += part[t];
        for (uint32_t t = 0; t < T; ++t) {
            uint32_t off = 0;
            for (uint32_t u = t + 1; u < T; ++u) off += part[u];
            uint32_t word = off >> 5, fill = off & 31;
            uint64_t acc = 0;
            for (uint32_t kk = R; kk-- > 0;) {
                const uint32_t p = A + R * t + kk;
                if (p >= first && p < lim) {
                    acc |= (uint64_t)code.code[in[p]] << fill;
                    fill += code.len[in[p]];
                    if (fill >= 32) { words.get()[word] |= (uint32_t)acc; acc >>= 32; fill -= 32; ++word; }
                }
            }
            if (fill) words.get()[word] |= (uint32_t)acc;
        }
        words.get()[total >> 5] |= 1u << (total & 31);
        const uint32_t bytes = total / 8 + 1;
        streams.emplace_back((uint8_t*)words.get(), (uint8_t*)words.get() + bytes);
    }
}

static void seq_streams(const uint8_t* in, uint32_t n, const zstd::HufCode& c, bool four,
                        std::vector<std::vector<uint8_t>>& streams) {
    for (uint32_t st = 0; st < (four ? 4u : 1u); ++st) {
        uint32_t f, cnt;
        zstd::stream_range(n, four, st, f, cnt);
        std::vector<uint8_t> w;
        uint64_t acc = 0;
        uint32_t nb = 0;
        for (uint32_t i = cnt; i-- > 0;) {
            acc |= (uint64_t)c.code[in[f + i]] << nb;
            nb += c.len[in[f + i]];
            while (nb >= 8) { w.push_back((uint8_t)acc); acc >>= 8; nb -= 8; }
        }
        acc |= 1ull << nb;
        ++nb;
        while (nb > 0) { w.push_back((uint8_t)acc); acc >>= 8; nb = nb > 8 ? nb - 8 : 0; }
        streams.push_back(w);
    }
}

static std::vector<uint8_t> gen_text(std::mt19937_64& rng) {
    auto U = [&](uint64_t lo, uint64_t hi) { return std::uniform_int_distribution<uint64_t>(lo, hi)(rng); };
    const uint32_t n = (uint32_t)U(0, 3 * zstd::kBlockMax + 100);
    std::vector<uint8_t> t;
    t.reserve(n);
    const int kind = (int)U(0, 4);
    if (kind == 0) {  // Delta-JSON-like
        t.insert(t.end(), {'{', '"', 'o', 'p', 's', '"', ':', '['});
        uint64_t off = U(0, 1ull << 30) * 4096;
        while (t.size() < n) {
            char buf[96];
            int m;
            if (U(0, 9) < 8) {
                m = snprintf(buf, sizeof buf, "{\"Copy\":{\"offset\":%llu,\"size\":4096}},", (unsigned long long)off);
                off += U(0, 3) ? 4096 : U(0, 1ull << 40);
            } else {
                m = snprintf(buf, sizeof buf, "{\"Data\":[%d,%d,%d]},", (int)U(0, 255), (int)U(0, 255), (int)U(0, 255));
            }
            t.insert(t.end(), buf, buf + m);
        }
        t.resize(n);
    } else if (kind == 1) {  // small alphabet
        const uint32_t a = (uint32_t)U(1, 127);
        for (uint32_t i = 0; i < n; ++i) t.push_back((uint8_t)U(0, a - 1));
    } else if (kind == 2) {  // runs
        while (t.size() < n) t.insert(t.end(), U(1, 400), (uint8_t)U(0, 255));
        t.resize(n);
    } else if (kind == 3) {  // binary
        for (uint32_t i = 0; i < n; ++i) t.push_back((uint8_t)U(0, 255));
    } else {  // periodic with edits
        std::vector<uint8_t> per(U(1, 300));
        for (auto& x : per) x = (uint8_t)U(32, 126);
        for (uint32_t i = 0; i < n; ++i) t.push_back(per[i % per.size()]);
        for (uint32_t e = 0; e < n / 100; ++e) t[U(0, n - 1)] = (uint8_t)U(0, 127);
    }
    return t;
}

static void zstd_case(std::mt19937_64& rng, uint64_t* blocks, uint64_t* replica_checked) {
    const std::vector<uint8_t> text = gen_text(rng);
    const uint32_t len = (uint32_t)text.size();
    Arr<uint8_t> in(len);  // exact: a read past the text is a report
    memcpy(in.get(), text.data(), len);
    for (uint32_t p0 = 0; p0 < len; p0 += zstd::kBlockMax) {
        const uint32_t n = std::min<uint32_t>(zstd::kBlockMax, len - p0);
        const uint8_t* b = in.get() + p0;
        Arr<uint8_t> slot(zstd::kBlockMax), lit(zstd::kBlockMax), streams(4 * zstd::kStreamBytesMax),
            body(zstd::kBodyBytes);
        Arr<uint32_t> best(zstd::kBlockMax);
        Arr<zstd::Seq> seq(zstd::kMaxSeq);
        Arr<zstd::FseCT> fse(3);
        const zstd::SeqScratch sc{best.get(), seq.get(), lit.get(), streams.get(), body.get(), fse.get()};
        uint32_t type = 9;
        const uint32_t size = zstd::block_content_seq(b, n, slot.get(), sc, &type);
        CHECK(type <= 2);
        CHECK(type != 2 || size < n);
        CHECK(type != 0 || size == n);
        ++*blocks;
        // the kernel's parallel streams against the sequential ones
        uint32_t h[256] = {0}, distinct = 0, hi = 0;
        for (uint32_t i = 0; i < n; ++i) ++h[b[i]];
        for (uint32_t s = 0; s < 256; ++s)
            if (h[s]) { ++distinct; hi = s; }
        if (distinct >= 2 && hi < zstd::kSymbols) {
            std::unique_ptr<zstd::HufCode> code(new zstd::HufCode);
            std::unique_ptr<zstd::HufWork> work(new zstd::HufWork);
            zstd::huf_build(h, *code, *work);
            const bool four = n > zstd::kSingleStreamMax;
            std::vector<std::vector<uint8_t>> a, s;
            scatter_replica(b, n, *code, four, a);
            seq_streams(b, n, *code, four, s);
            CHECK(a == s);
            // the code is complete (Kraft sum 1) and limited to 11 bits
            uint64_t kraft = 0;
            for (uint32_t x = 0; x < zstd::kSymbols; ++x)
                if (code->len[x]) {
                    CHECK(code->len[x] <= zstd::kMaxBits);
                    kraft += 1ull << (zstd::kMaxBits - code->len[x]);
                }
            CHECK(kraft == (1ull << zstd::kMaxBits));
            ++*replica_checked;
        }
    }
}

static void sigjson_case(std::mt19937_64& rng, uint64_t* entries) {
    const uint64_t n = 1 + rng() % 1500;
    const uint64_t bss[] = {1, 512, 4096, 8192, 131072, 1ull << 32};
    const uint64_t bs = bss[rng() % 6];
    const uint64_t last = 1 + rng() % bs;
    std::unique_ptr<uint32_t[]> weak(new uint32_t[n]);
    std::unique_ptr<uint64_t[]> strong(new uint64_t[n]);
    for (uint64_t i = 0; i < n; ++i) {
        const int k = (int)(rng() % 3);
        weak[i] = k == 0 ? (uint32_t)rng() : k == 1 ? (uint32_t)(rng() % 100) : 0xFFFFFFFFu;
        strong[i] = k == 0 ? rng() : k == 1 ? rng() % 1000 : ~0ull;
    }
    const sigjson::SigArgs a{weak.get(), strong.get(), n, bs, last};
    std::string ref = "[";
    char tmp[256];
    for (uint64_t i = 0; i < n; ++i) {
        snprintf(tmp, sizeof tmp, "%s{\"index\":%llu,\"offset\":%llu,\"size\":%llu,\"weak\":%u,\"strong\":%llu}",
                 i ? "," : "", (unsigned long long)i, (unsigned long long)(i * bs),
                 (unsigned long long)(i + 1 == n ? last : bs), weak[i], (unsigned long long)strong[i]);
        ref += tmp;
    }
    ref += "]";
    uint64_t lo = 0, hi = 0;
    sigjson::text_bounds(n, bs, last, lo, hi);
    CHECK(ref.size() >= lo && ref.size() <= hi);
    // the output: exactly the text's length, at a random offset from a 16-byte boundary
    const size_t shift = rng() % 16;
    std::unique_ptr<uint8_t[]> raw(new uint8_t[ref.size() + shift]);
    uint8_t* out = raw.get() + shift;
    const uint64_t nt = (n + sigjson::kTile - 1) / sigjson::kTile;
    uint64_t toff = 0;
    for (uint64_t t = 0; t < nt; ++t) {
        const uint64_t i0 = t * sigjson::kTile, i1 = std::min<uint64_t>(n, i0 + sigjson::kTile);
        std::vector<uint32_t> off(i1 - i0 + 1, 0);
        for (uint64_t i = i0; i < i1; ++i) off[i - i0 + 1] = off[i - i0] + sigjson::entry_len(a, i);
        const uint32_t tot = off[i1 - i0];
        CHECK(tot <= sigjson::kStage);
        std::unique_ptr<uint8_t[]> stage(new uint8_t[tot]);
        for (uint64_t i = i0; i < i1; ++i) CHECK(sigjson::entry_write(a, i, stage.get() + off[i - i0]) == off[i - i0 + 1] - off[i - i0]);
        uint8_t* dst = out + toff;
        const uintptr_t c0 = (uintptr_t)dst & ~(uintptr_t)15, c1 = ((uintptr_t)dst + tot + 15) & ~(uintptr_t)15;
        std::vector<uintptr_t> cs;
        for (uintptr_t c = c0; c < c1; c += 16) cs.push_back(c);
        std::shuffle(cs.begin(), cs.end(), rng);
        for (uintptr_t c : cs) sigjson::store_chunk(stage.get(), tot, dst, c);
        toff += tot;
    }
    CHECK(toff == ref.size());
    CHECK(memcmp(out, ref.data(), ref.size()) == 0);
    *entries += n;
}

// zstd repeat offsets (sydelta_zstd.hpp rep_code): the Offset_Values the coder picks,
// read back by an independent restatement of the decoder's history rules (RFC 8878
// 3.1.1.5) that starts from a history the coder does not know, give every distance back.
static void repcode_case(std::mt19937_64& rng, uint64_t* reps_used) {
    uint32_t enc[3] = {0, 0, 0};
    uint32_t h[3] = {1 + (uint32_t)(rng() % 50), 1 + (uint32_t)(rng() % 50), 1 + (uint32_t)(rng() % 50)};
    const uint32_t pool[6] = {1 + (uint32_t)(rng() % 40), 1 + (uint32_t)(rng() % 40), 2 + (uint32_t)(rng() % 40),
                              41, 42, 43};
    for (int i = 0; i < 400; ++i) {
        const uint32_t ll = rng() % 3 == 0 ? 0 : (uint32_t)(rng() % 20);
        const uint32_t d = rng() % 4 == 0 ? 1 + (uint32_t)(rng() % 100000) : pool[rng() % 6];
        const uint32_t ov = zstd::rep_code(enc, ll, d);
        uint32_t off;
        if (ov > 3) {
            off = ov - 3;
            h[2] = h[1]; h[1] = h[0]; h[0] = off;
        } else {
            const uint32_t idx = ov - 1 + (ll == 0 ? 1 : 0);
            if (idx == 0) off = h[0];
            else if (idx == 1) { off = h[1]; h[1] = h[0]; h[0] = off; }
            else if (idx == 2) { off = h[2]; h[2] = h[1]; h[1] = h[0]; h[0] = off; }
            else { off = h[0] - 1; h[2] = h[1]; h[1] = h[0]; h[0] = off; }
            ++*reps_used;
        }
        CHECK(off == d);
        CHECK(ov >= 1);
    }
}

// K7p: the parse bodies on texts in arrays of exactly their length (a read past the text
// is an ASan report): serde's compact text of a random signature parses back to it; a
// mutated text is either refused or re-serializes to itself (the device accepts the
// compact form only).
static std::vector<uint8_t> sig_text(const std::vector<sydelta_block_checksum>& v) {
    std::string t = "[";
    char tmp[256];
    for (size_t i = 0; i < v.size(); ++i) {
        snprintf(tmp, sizeof tmp, "%s{\"index\":%llu,\"offset\":%llu,\"size\":%llu,\"weak\":%u,\"strong\":%llu}",
                 i ? "," : "", (unsigned long long)v[i].index, (unsigned long long)v[i].offset,
                 (unsigned long long)v[i].size, v[i].weak, (unsigned long long)v[i].strong);
        t += tmp;
    }
    t += "]";
    return std::vector<uint8_t>(t.begin(), t.end());
}
static bool parse_all(const std::vector<uint8_t>& text, std::vector<sydelta_block_checksum>& out) {
    const uint64_t len = text.size();
    std::unique_ptr<uint8_t[]> t(new uint8_t[len ? len : 1]);
    if (len) memcpy(t.get(), text.data(), len);
    const uint64_t nc = (len + sigjson::kParseChunk - 1) / sigjson::kParseChunk;
    if (len < 2 || !nc) return false;
    std::vector<uint64_t> rank(nc + 1, 0);
    for (uint64_t c = 0; c < nc; ++c) rank[c + 1] = rank[c] + sigjson::chunk_entries(t.get(), len, c);
    std::unique_ptr<sydelta_block_checksum[]> o(new sydelta_block_checksum[rank[nc] ? rank[nc] : 1]);
    for (uint64_t c = nc; c-- > 0;)
        if (sigjson::chunk_parse(t.get(), len, c, rank[c], o.get(), rank[nc]) != UINT64_MAX) return false;
    out.assign(o.get(), o.get() + rank[nc]);
    return true;
}
static void sigparse_case(std::mt19937_64& rng, uint64_t* accepted, uint64_t* refused) {
    const size_t n = rng() % 300;
    std::vector<sydelta_block_checksum> v(n);
    for (size_t i = 0; i < n; ++i) {
        const int k = (int)(rng() % 3);
        v[i] = sydelta_block_checksum{i, i * 4096, k ? 4096u : 1 + rng() % 4096, k == 2 ? 0xFFFFFFFFu : (uint32_t)rng(),
                                      0, k == 1 ? ~0ull : rng() % (k ? 1000 : ~0ull)};
    }
    const std::vector<uint8_t> text = sig_text(v);
    std::vector<sydelta_block_checksum> back;
    CHECK(parse_all(text, back));
    CHECK(back.size() == n);
    for (size_t i = 0; i < n; ++i)
        CHECK(back[i].index == v[i].index && back[i].offset == v[i].offset && back[i].size == v[i].size &&
              back[i].weak == v[i].weak && back[i].strong == v[i].strong);
    static const char alpha[] = "0123456789{}[],:\"az -";
    for (int m = 0; m < 20; ++m) {
        std::vector<uint8_t> t = text;
        const int k = 1 + (int)(rng() % 3);
        for (int j = 0; j < k; ++j) {
            const int op = (int)(rng() % 3);
            const size_t at = t.empty() ? 0 : rng() % t.size();
            if (op == 0 && !t.empty()) t[at] = (uint8_t)alpha[rng() % (sizeof alpha - 1)];
            else if (op == 1) t.insert(t.begin() + at, (uint8_t)alpha[rng() % (sizeof alpha - 1)]);
            else if (!t.empty()) t.erase(t.begin() + at);
        }
        std::vector<sydelta_block_checksum> got;
        if (parse_all(t, got)) {
            CHECK(sig_text(got) == t);
            ++*accepted;
        } else {
            ++*refused;
        }
    }
}

// K7d: the Delta JSON parse bodies on texts in arrays of exactly their length; the ops
// region of a random delta's compact text parses back to it; a mutated text is refused
// or its ops region is the compact text of what it parses to.
struct DOp {
    bool copy;
    uint64_t o, s;
    std::vector<uint8_t> lit;
};
static std::string dops_text(const std::vector<DOp>& v) {
    std::string t;
    char tmp[96];
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) t += ",";
        if (v[i].copy) {
            snprintf(tmp, sizeof tmp, "{\"Copy\":{\"offset\":%llu,\"size\":%llu}}", (unsigned long long)v[i].o,
                     (unsigned long long)v[i].s);
            t += tmp;
        } else {
            t += "{\"Data\":[";
            for (size_t k = 0; k < v[i].lit.size(); ++k) {
                if (k) t += ",";
                t += std::to_string((unsigned)v[i].lit[k]);
            }
            t += "]}";
        }
    }
    return t;
}
// Parse the ops region of text (head, region, tail) with the chunk bodies; false if refused.
static bool dparse_all(const std::string& text, std::vector<DOp>& out) {
    const std::string key = "],\"source_size\":";
    const size_t at = text.rfind(key);
    if (text.size() < 8 || at == std::string::npos || at < 8 || text.compare(0, 8, "{\"ops\":[") != 0) return false;
    const uint64_t len = text.size();
    std::unique_ptr<uint8_t[]> t(new uint8_t[len]);
    memcpy(t.get(), text.data(), len);
    const dparse::DArgs a{t.get(), at, (at - 8 + dparse::kChunk - 1) / dparse::kChunk};
    std::vector<uint64_t> orank(a.nc + 1, 0), lrank(a.nc + 1, 0);
    for (uint64_t c = 0; c < a.nc; ++c) {
        uint64_t no, nl;
        dparse::chunk_count(a, c, no, nl);
        orank[c + 1] = orank[c] + no;
        lrank[c + 1] = lrank[c] + nl;
    }
    const uint64_t nops = orank[a.nc], nlit = lrank[a.nc];
    if (a.nc && !nops) return false;
    std::unique_ptr<uint64_t[]> pos(new uint64_t[nops ? nops : 1]);
    std::unique_ptr<sydelta_op[]> ops(new sydelta_op[nops ? nops : 1]);
    std::unique_ptr<uint8_t[]> lit(new uint8_t[nlit ? nlit : 1]);
    for (uint64_t c = 0; c < a.nc; ++c) dparse::chunk_place(a, c, orank[c], pos.get());
    for (uint64_t c = a.nc; c-- > 0;)
        if (dparse::chunk_parse(a, c, orank.data(), lrank.data(), pos.get(), nops, ops.get(), lit.get()) != dparse::kNoBad)
            return false;
    out.clear();
    for (uint64_t i = 0; i < nops; ++i) {
        DOp d{ops[i].kind == SYDELTA_OP_COPY, ops[i].a, ops[i].b, {}};
        if (!d.copy) {
            CHECK(ops[i].a + ops[i].b <= nlit);
            d.lit.assign(lit.get() + ops[i].a, lit.get() + ops[i].a + ops[i].b);
        }
        out.push_back(d);
    }
    return true;
}
static void dparse_case(std::mt19937_64& rng, uint64_t* accepted, uint64_t* refused) {
    std::vector<DOp> v(rng() % 40);
    for (auto& d : v) {
        d.copy = rng() % 2;
        d.o = rng() % 3 ? rng() % 100000 : ~0ull;
        d.s = rng() % 5000;
        if (!d.copy) {
            d.lit.resize(rng() % 4 ? rng() % 40 : rng() % 3000);
            for (auto& b : d.lit) b = (uint8_t)rng();
        }
    }
    const std::string tail = "],\"source_size\":123,\"block_size\":4096}";
    const std::string text = "{\"ops\":[" + dops_text(v) + tail;
    std::vector<DOp> back;
    CHECK(dparse_all(text, back));
    CHECK(back.size() == v.size());
    for (size_t i = 0; i < v.size(); ++i)
        CHECK(back[i].copy == v[i].copy && (v[i].copy ? back[i].o == v[i].o && back[i].s == v[i].s : back[i].lit == v[i].lit));
    static const char alpha[] = "0123456789{}[],:\"aDC -";
    for (int m = 0; m < 24; ++m) {
        std::string t = text;
        if (m >= 20 && !v.empty()) {
            // junk before the first op, ending in "}," so an op start follows it
            std::string junk = "},";
            for (int j = (int)(rng() % 4); j > 0; --j) junk.insert(junk.begin(), alpha[rng() % (sizeof alpha - 1)]);
            t.insert(8, junk);
            std::vector<DOp> got;
            CHECK(!dparse_all(t, got));
            ++*refused;
            continue;
        }
        for (int j = 0, k = 1 + (int)(rng() % 3); j < k; ++j) {
            const int op = (int)(rng() % 3);
            const size_t at = rng() % t.size();
            if (op == 0) t[at] = alpha[rng() % (sizeof alpha - 1)];
            else if (op == 1) t.insert(t.begin() + at, alpha[rng() % (sizeof alpha - 1)]);
            else if (t.size() > 1) t.erase(t.begin() + at);
        }
        std::vector<DOp> got;
        if (dparse_all(t, got)) {
            const size_t at = t.rfind("],\"source_size\":");
            CHECK(t.substr(8, at - 8) == dops_text(got));
            ++*accepted;
        } else {
            ++*refused;
        }
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    std::mt19937_64 rng(20261017);
    uint64_t walked = 0, cases = 0;
    for (int it = 0; it < iters; ++it) cases += chain_case(rng, &walked) >= 0;
    uint64_t blocks = 0, replica = 0;
    for (int it = 0; it < std::max(1, iters / 25); ++it) zstd_case(rng, &blocks, &replica);
    uint64_t reps = 0;
    for (int it = 0; it < std::max(1, iters / 10); ++it) repcode_case(rng, &reps);
    CHECK(reps > 0);
    uint64_t acc = 0, ref = 0;
    for (int it = 0; it < std::max(1, iters / 10); ++it) sigparse_case(rng, &acc, &ref);
    CHECK(acc > 0 && ref > 0);
    uint64_t dacc = 0, dref = 0;
    for (int it = 0; it < std::max(1, iters / 10); ++it) dparse_case(rng, &dacc, &dref);
    CHECK(dacc > 0 && dref > 0);
    uint64_t sj = 0;
    for (int it = 0; it < std::max(1, iters / 10); ++it) sigjson_case(rng, &sj);
    CHECK(walked > (uint64_t)iters / 4);
    printf("kernel bodies ok: %llu chain cases (%llu resolved on the device path), %llu zstd blocks, %llu stream "
           "replicas, %llu repeat offsets, %llu signature JSON entries, %llu/%llu mutated texts accepted/refused, "
           "%llu/%llu mutated Delta texts accepted/refused\n",
           (unsigned long long)cases, (unsigned long long)walked, (unsigned long long)blocks,
           (unsigned long long)replica, (unsigned long long)reps, (unsigned long long)sj, (unsigned long long)acc,
           (unsigned long long)ref, (unsigned long long)dacc, (unsigned long long)dref);
    return 0;
}
