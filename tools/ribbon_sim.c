// ribbon_sim.c -- build-owned design tool (not product code, not the oracle): measures the
// false-pass rate of level-1 filters for the C3 scan on real Adler-32 values
// (1 Mi random 4 KiB blocks as keys, rolled windows of random bytes as queries):
// the one-hash Bloom of k_scan_r (150 KiB) against a sharded homogeneous ribbon
// (Dillinger & Walzer 2021) of the same size, with the probe hashes the kernel computes.
//   gcc -O2 -o /tmp/ribbon_sim tools/ribbon_sim.c && /tmp/ribbon_sim [shards] [w]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define M 65521u
static uint64_t sm = 0x5E1D0002;
static uint64_t rnd(void) {
    uint64_t z = (sm += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint32_t umul24(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)(a & 0xFFFFFF) * (b & 0xFFFFFF)); }
static void probe_hash(uint32_t A, uint32_t B, uint32_t* q, uint32_t* r) {
    *q = umul24(A, 0x9E3779u) + umul24(B, 0x85EBCBu);
    *r = umul24(A, 0xC2B2AFu) + umul24(B, 0x27D4EBu);
}
static uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
// ribbon coordinates of a weak value from (q, r): shard, start in [0, ms - w], coefficient
static int W = 64;
static uint32_t NS, MS;  // shards, slots (bits) per shard
static int MIX = 1;
static void coords(uint32_t q, uint32_t r, uint32_t* sh, uint32_t* st, uint64_t* c) {
    uint32_t h1 = q ^ rotl(r, 15), h2 = r ^ rotl(q, 9);
    if (!MIX) {  // the probe hashes as they are: shard and start from q and r, coefficient from both
        *sh = (uint32_t)(((uint64_t)(q >> 8) * (NS << 8)) >> 32);
        if (NS == 1024) *sh = q >> 22;
        *st = (uint32_t)(((uint64_t)(r >> 8) * ((MS - W + 1) << 8)) >> 32);
        *c = ((uint64_t)(q ^ rotl(r, 16)) | 1) & (W == 32 ? 0xFFFFFFFFull : ~0ull);
        if (W == 64) *c |= (uint64_t)(r ^ rotl(q, 11)) << 32;
        return;
    }
    *sh = (uint32_t)(((uint64_t)(h1 >> 8) * (NS << 8)) >> 32);
    *st = (uint32_t)(((uint64_t)(h2 >> 8) * ((MS - W + 1) << 8)) >> 32);
    uint64_t cc = ((uint64_t)(h1 ^ rotl(h2, 7)) << 32) | (h2 ^ rotl(h1, 21));
    if (W == 32) cc &= 0xFFFFFFFFull;
    *c = cc | 1;
}
int main(int argc, char** argv) {
    NS = argc > 1 ? atoi(argv[1]) : 512;
    W = argc > 2 ? atoi(argv[2]) : 64;
    MIX = argc > 3 ? atoi(argv[3]) : 1;
    const uint32_t total_bits = 38400u * 32;
    MS = total_bits / NS / 32 * 32;  // whole words per shard
    const int nk = 1 << 20, n = 4096;
    uint32_t* keys = malloc(4 * nk);
    uint8_t blk[4096];
    for (int k = 0; k < nk; ++k) {
        for (int i = 0; i < n; i += 8) { uint64_t v = rnd(); memcpy(blk + i, &v, 8); }
        uint64_t a = 1, b = 0;
        for (int i = 0; i < n; ++i) { a += blk[i]; b += a; }
        keys[k] = (uint32_t)(((b % M) << 16) | (a % M));
    }
    // Bloom, one hash, kL1WordsR words (l1r_word)
    uint32_t* bl = calloc(38400, 4);
    for (int k = 0; k < nk; ++k) {
        uint32_t q, r;
        probe_hash(keys[k] & 0xFFFF, keys[k] >> 16, &q, &r);
        uint32_t w = (uint32_t)(((uint64_t)(q >> 8) * (38400u << 8)) >> 32);
        bl[w] |= 1u << (q & 31);
    }
    // level-2 blocked Bloom (2^19 words, 3 bits from q, word from r: k_idx_insert)
    uint32_t* l2 = calloc(1u << 19, 4);
    for (int k = 0; k < nk; ++k) {
        uint32_t q, r;
        probe_hash(keys[k] & 0xFFFF, keys[k] >> 16, &q, &r);
        l2[r >> 13] |= (1u << (q & 31)) | (1u << ((q >> 5) & 31)) | (1u << ((q >> 10) & 31));
    }
    // homogeneous ribbon per shard
    uint64_t* rows = calloc((size_t)NS * MS, 8);
    uint8_t* z = calloc((size_t)NS * MS, 1);
    long redundant = 0;
    for (int k = 0; k < nk; ++k) {
        uint32_t q, r, sh, st;
        uint64_t c;
        probe_hash(keys[k] & 0xFFFF, keys[k] >> 16, &q, &r);
        coords(q, r, &sh, &st, &c);
        uint64_t* R = rows + (size_t)sh * MS;
        for (;;) {
            if (!R[st]) { R[st] = c; break; }
            c ^= R[st];
            if (!c) { ++redundant; break; }
            int t = __builtin_ctzll(c);
            st += t;
            c >>= t;
        }
    }
    long freev = 0;
    for (uint32_t s = 0; s < NS; ++s) {
        uint64_t* R = rows + (size_t)s * MS;
        uint8_t* Z = z + (size_t)s * MS;
        for (int i = (int)MS - 1; i >= 0; --i) {
            if (!R[i]) { Z[i] = rnd() & 1; ++freev; continue; }
            int p = 0;
            for (int j = 1; j < W && i + j < (int)MS; ++j) if ((R[i] >> j) & 1) p ^= Z[i + j];
            Z[i] = p;
        }
    }
    // check keys and measure false passes on rolled windows of fresh random bytes
    for (int k = 0; k < nk; ++k) {
        uint32_t q, r, sh, st;
        uint64_t c;
        probe_hash(keys[k] & 0xFFFF, keys[k] >> 16, &q, &r);
        coords(q, r, &sh, &st, &c);
        int p = 0;
        for (int j = 0; j < W; ++j) if ((c >> j) & 1) p ^= z[(size_t)sh * MS + st + j];
        if (p) { printf("FALSE NEGATIVE key %d\n", k); return 1; }
    }
    const long nq = 20000000;
    uint8_t* buf = malloc(nq + n);
    for (long i = 0; i < nq + n; i += 8) { uint64_t v = rnd(); memcpy(buf + i, &v, 8); }
    uint64_t a = 1, b = 0;
    for (int i = 0; i < n; ++i) { a += buf[i]; b += a; }
    a %= M; b %= M;
    long pb = 0, pr = 0, pb2 = 0, pr2 = 0, p2 = 0;
    for (long p = 0; p < nq; ++p) {
        uint32_t q, r, sh, st;
        uint64_t c;
        probe_hash((uint32_t)a, (uint32_t)b, &q, &r);
        uint32_t w = (uint32_t)(((uint64_t)(q >> 8) * (38400u << 8)) >> 32);
        pb += (bl[w] >> (q & 31)) & 1;
        coords(q, r, &sh, &st, &c);
        int par = 0;
        for (int j = 0; j < W; ++j) if ((c >> j) & 1) par ^= z[(size_t)sh * MS + st + j];
        pr += par == 0;
        const uint32_t m2 = (1u << (q & 31)) | (1u << ((q >> 5) & 31)) | (1u << ((q >> 10) & 31));
        const int l2p = (l2[r >> 13] & m2) == m2;
        p2 += l2p;
        pb2 += l2p && ((bl[w] >> (q & 31)) & 1);
        pr2 += l2p && par == 0;
        const uint32_t out = buf[p], in = buf[p + n];
        a = (a + M - out + in) % M;
        b = (b + 3 * (uint64_t)M - (uint64_t)n * out % M + a - 1) % M;
    }
    printf("shards %u x %u bits (w %d): %u bits/key %.3f; redundant keys %ld, free columns %ld\n", NS, MS, W,
           NS * MS, (double)NS * MS / nk, redundant, freev);
    printf("false pass: bloom %.4f  ribbon %.4f; level 2 alone %.5f, after bloom %.5f (x%.3f), after ribbon %.5f (x%.3f)\n",
           (double)pb / nq, (double)pr / nq, (double)p2 / nq, (double)pb2 / nq, (double)pb2 / pb / ((double)p2 / nq),
           (double)pr2 / nq, (double)pr2 / pr / ((double)p2 / nq));
    return 0;
}
