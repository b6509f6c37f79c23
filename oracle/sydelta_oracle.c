/*
 * sydelta_oracle.c — CPU restatement of nijaru/sy `src/delta` (v0.0.43).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the HIP
 * product path in sy_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's `cpu_baseline` leg may load it, and only as the checker or the
 * reported CPU baseline — never as the thing measured or shipped.
 *
 * The reference is Rust; no cargo/rustc exists in this image, so the
 * reference cannot be built.  What is restated here:
 *
 *   oracle_adler32            src/delta/rolling.rs:35-45   (Adler32::hash)
 *   oracle_rolling_*          src/delta/rolling.rs:26-91   (new/update_block/roll/digest)
 *   oracle_xxh3_64            third-party crate xxhash-rust 0.8.15 (Cargo.lock:4124-4127),
 *                             feature "xxh3": XXH3-64, seed 0, default 192-byte secret.
 *                             Not vendored in the reference; restated from the published
 *                             XXH3 algorithm (frozen since xxHash 0.8.0) and pinned in
 *                             tests against python-xxhash 3.8.1 (libxxhash 0.8.2).
 *   oracle_compute_checksums  src/delta/checksum.rs:31-80   (in-memory form of the file read)
 *   oracle_compute_checksums_file  same, with the per-block open/seek/read of checksum.rs:50-59
 *   oracle_generate_delta     src/delta/generator.rs:242-379 (in-memory scan)
 *   oracle_generate_delta_streaming  src/delta/generator.rs:67-228 (256 KiB refill window;
 *                             chunk size is a parameter so tests can exercise refills)
 *   oracle_apply_delta        src/delta/applier.rs:22-56 (in-memory)
 *   oracle_calculate_block_size  src/delta/mod.rs:20-23
 *
 * Ops are returned as descriptors: Copy{offset,size} -> (kind=0, a=offset, b=size);
 * Data(bytes) -> (kind=1, a=offset of the literal run in the new file, b=length).
 * Every literal run in the reference is a contiguous slice of the new file
 * (literal_buffer is flushed whenever a Copy is emitted), so the descriptor
 * names exactly the bytes of DeltaOp::Data.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <stdio.h>
#include <fcntl.h>
#include <unistd.h>
#include <pthread.h>

#define MOD_ADLER 65521u /* rolling.rs:22 */

/* ------------------------------------------------------------------ */
/* Adler-32 (rolling.rs)                                              */
/* ------------------------------------------------------------------ */

/* rolling.rs:35-45 — per byte a=(a+x)%M, b=(b+a)%M; digest (b<<16)|a. */
uint32_t oracle_adler32(const uint8_t *data, uint64_t len) {
    uint32_t a = 1, b = 0;
    for (uint64_t i = 0; i < len; i++) {
        a = (a + data[i]) % MOD_ADLER;
        b = (b + a) % MOD_ADLER;
    }
    return (b << 16) | a;
}

typedef struct { uint32_t a, b; uint64_t block_size; } oracle_rolling;

/* rolling.rs:26-32 */
void oracle_rolling_new(oracle_rolling *r, uint64_t block_size) { r->a = 1; r->b = 0; r->block_size = block_size; }
/* rolling.rs:48-56 */
void oracle_rolling_update_block(oracle_rolling *r, const uint8_t *blk, uint64_t len) {
    r->a = 1; r->b = 0;
    for (uint64_t i = 0; i < len; i++) {
        r->a = (r->a + blk[i]) % MOD_ADLER;
        r->b = (r->b + r->a) % MOD_ADLER;
    }
}
/* rolling.rs:66-79 — u32 arithmetic exactly as written (n = block_size as u32). */
void oracle_rolling_roll(oracle_rolling *r, uint8_t old_byte, uint8_t new_byte) {
    uint32_t old = old_byte, nw = new_byte, n = (uint32_t)r->block_size;
    r->a = (r->a + MOD_ADLER * 2u - old + nw) % MOD_ADLER;
    uint32_t n_old = (n * old) % MOD_ADLER;
    r->b = (r->b + MOD_ADLER * 3u - n_old + r->a - 1u) % MOD_ADLER;
}
/* rolling.rs:82-84 */
uint32_t oracle_rolling_digest(const oracle_rolling *r) { return (r->b << 16) | r->a; }

/* ------------------------------------------------------------------ */
/* XXH3-64 (xxhash-rust 0.8.15 `xxh3::Xxh3` digest == one-shot xxh3_64) */
/* ------------------------------------------------------------------ */

static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull
#define PMX1 0x165667919E3779F9ull
#define PMX2 0x9FB21C651E98DF25ull

static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; } /* little-endian host */
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t swap64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint64_t fold64(uint64_t a, uint64_t b) {
    unsigned __int128 p = (unsigned __int128)a * b;
    return (uint64_t)p ^ (uint64_t)(p >> 64);
}
static inline uint64_t xxh64_aval(uint64_t h) {
    h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32; return h;
}
static inline uint64_t xxh3_aval(uint64_t h) { h ^= h >> 37; h *= PMX1; h ^= h >> 32; return h; }
static inline uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24); h *= PMX2; h ^= (h >> 35) + len; h *= PMX2; return h ^ (h >> 28);
}
static inline uint64_t mix16(const uint8_t *in, const uint8_t *sec) {
    return fold64(rd64(in) ^ rd64(sec), rd64(in + 8) ^ rd64(sec + 8));
}

static uint64_t xxh3_len_0to16(const uint8_t *in, uint64_t len) {
    const uint8_t *s = kSecret;
    if (len > 8) {
        uint64_t bf1 = rd64(s + 24) ^ rd64(s + 32), bf2 = rd64(s + 40) ^ rd64(s + 48);
        uint64_t lo = rd64(in) ^ bf1, hi = rd64(in + len - 8) ^ bf2;
        uint64_t acc = len + swap64(lo) + hi + fold64(lo, hi);
        return xxh3_aval(acc);
    }
    if (len >= 4) {
        uint32_t i1 = rd32(in), i2 = rd32(in + len - 4);
        uint64_t bf = rd64(s + 8) ^ rd64(s + 16);
        uint64_t i64 = (uint64_t)i2 + ((uint64_t)i1 << 32);
        return rrmxmx(i64 ^ bf, len);
    }
    if (len) {
        uint8_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
        uint32_t comb = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) | (uint32_t)c3 | ((uint32_t)len << 8);
        uint64_t bf = (uint64_t)(rd32(s) ^ rd32(s + 4));
        return xxh64_aval((uint64_t)comb ^ bf);
    }
    return xxh64_aval(rd64(s + 56) ^ rd64(s + 64));
}

static uint64_t xxh3_len_17to128(const uint8_t *in, uint64_t len) {
    const uint8_t *s = kSecret;
    uint64_t acc = len * P64_1;
    if (len > 32) {
        if (len > 64) {
            if (len > 96) { acc += mix16(in + 48, s + 96); acc += mix16(in + len - 64, s + 112); }
            acc += mix16(in + 32, s + 64); acc += mix16(in + len - 48, s + 80);
        }
        acc += mix16(in + 16, s + 32); acc += mix16(in + len - 32, s + 48);
    }
    acc += mix16(in, s); acc += mix16(in + len - 16, s + 16);
    return xxh3_aval(acc);
}

static uint64_t xxh3_len_129to240(const uint8_t *in, uint64_t len) {
    const uint8_t *s = kSecret;
    uint64_t acc = len * P64_1, acc_end;
    unsigned nb = (unsigned)(len / 16), i;
    for (i = 0; i < 8; i++) acc += mix16(in + 16 * i, s + 16 * i);
    acc_end = mix16(in + len - 16, s + 136 - 17);
    acc = xxh3_aval(acc);
    for (i = 8; i < nb; i++) acc_end += mix16(in + 16 * i, s + 16 * (i - 8) + 3);
    return xxh3_aval(acc + acc_end);
}

static inline void acc512(uint64_t acc[8], const uint8_t *in, const uint8_t *sec) {
    for (int i = 0; i < 8; i++) {
        uint64_t dv = rd64(in + 8 * i), dk = dv ^ rd64(sec + 8 * i);
        acc[i ^ 1] += dv;
        acc[i] += (uint64_t)(uint32_t)dk * (dk >> 32);
    }
}
static inline void scramble(uint64_t acc[8], const uint8_t *sec) {
    for (int i = 0; i < 8; i++) {
        uint64_t a = acc[i];
        a ^= a >> 47; a ^= rd64(sec + 8 * i); a *= P32_1; acc[i] = a;
    }
}

static uint64_t xxh3_long(const uint8_t *in, uint64_t len) {
    uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    const uint64_t block_len = 1024;               /* 16 stripes x 64 B */
    uint64_t nb_blocks = (len - 1) / block_len;
    for (uint64_t n = 0; n < nb_blocks; n++) {
        for (unsigned s = 0; s < 16; s++) acc512(acc, in + n * block_len + 64 * s, kSecret + 8 * s);
        scramble(acc, kSecret + 192 - 64);
    }
    uint64_t nbs = ((len - 1) - block_len * nb_blocks) / 64;
    for (uint64_t s = 0; s < nbs; s++) acc512(acc, in + nb_blocks * block_len + 64 * s, kSecret + 8 * s);
    acc512(acc, in + len - 64, kSecret + 192 - 64 - 7);
    uint64_t r = len * P64_1;
    for (int i = 0; i < 4; i++) r += fold64(acc[2 * i] ^ rd64(kSecret + 11 + 16 * i), acc[2 * i + 1] ^ rd64(kSecret + 11 + 16 * i + 8));
    return xxh3_aval(r);
}

uint64_t oracle_xxh3_64(const uint8_t *in, uint64_t len) {
    if (len <= 16) return xxh3_len_0to16(in, len);
    if (len <= 128) return xxh3_len_17to128(in, len);
    if (len <= 240) return xxh3_len_129to240(in, len);
    return xxh3_long(in, len);
}

/* ------------------------------------------------------------------ */
/* mod.rs:20-23                                                        */
/* ------------------------------------------------------------------ */
uint64_t oracle_calculate_block_size(uint64_t file_size) {
    uint64_t s = (uint64_t)sqrt((double)file_size);   /* `as usize` truncates */
    if (s < 512) s = 512;
    if (s > 128 * 1024) s = 128 * 1024;
    return s;
}

/* ------------------------------------------------------------------ */
/* checksum.rs:31-80 — signature                                       */
/* ------------------------------------------------------------------ */

typedef struct {
    const uint8_t *buf; uint64_t len, bs, nblocks;
    uint32_t *weak; uint64_t *strong; uint64_t *size;
    uint64_t next; pthread_mutex_t mu;
} sig_job;

static void sig_block(const sig_job *j, uint64_t i) {
    uint64_t off = i * j->bs, sz = j->len - off < j->bs ? j->len - off : j->bs;
    j->weak[i] = oracle_adler32(j->buf + off, sz);
    j->strong[i] = oracle_xxh3_64(j->buf + off, sz);
    if (j->size) j->size[i] = sz;
}

static void *sig_worker(void *arg) {
    sig_job *j = (sig_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint64_t lo = j->next; j->next += 256;
        pthread_mutex_unlock(&j->mu);
        if (lo >= j->nblocks) break;
        uint64_t hi = lo + 256 < j->nblocks ? lo + 256 : j->nblocks;
        for (uint64_t i = lo; i < hi; i++) sig_block(j, i);
    }
    return NULL;
}

/* In-memory restatement of compute_checksums: ceil(len/bs) blocks (:41), block i at
 * offset i*bs with size = bytes available (:50-59), weak = Adler32::hash (:62),
 * strong = Xxh3 digest (:65-67); empty input -> 0 blocks (:36-38).  `threads` > 1
 * mirrors the rayon par_iter (:46-48); output is in index order either way.
 * Returns the number of blocks. */
uint64_t oracle_compute_checksums(const uint8_t *buf, uint64_t len, uint64_t bs,
                                  uint32_t *weak, uint64_t *strong, uint64_t *size, int threads) {
    if (len == 0 || bs == 0) return 0;
    sig_job j = {buf, len, bs, (len + bs - 1) / bs, weak, strong, size, 0};
    pthread_mutex_init(&j.mu, NULL);
    if (threads <= 1) {
        for (uint64_t i = 0; i < j.nblocks; i++) sig_block(&j, i);
    } else {
        pthread_t th[256];
        if (threads > 256) threads = 256;
        for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, sig_worker, &j);
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    }
    pthread_mutex_destroy(&j.mu);
    return j.nblocks;
}

/* File-based variant: per block File::open + seek + vec![0;bs] + read (checksum.rs:50-59). */
typedef struct { const char *path; uint64_t len, bs, nblocks; uint32_t *weak; uint64_t *strong;
                 uint64_t next; int err; pthread_mutex_t mu; } sigf_job;
static void *sigf_worker(void *arg) {
    sigf_job *j = (sigf_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint64_t i = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->nblocks) break;
        int fd = open(j->path, O_RDONLY);
        if (fd < 0) { j->err = 1; break; }
        uint8_t *b = (uint8_t *)malloc(j->bs);
        ssize_t got = pread(fd, b, j->bs, (off_t)(i * j->bs));
        close(fd);
        if (got < 0) { j->err = 1; free(b); break; }
        j->weak[i] = oracle_adler32(b, (uint64_t)got);
        j->strong[i] = oracle_xxh3_64(b, (uint64_t)got);
        free(b);
    }
    return NULL;
}
int64_t oracle_compute_checksums_file(const char *path, uint64_t bs, uint32_t *weak, uint64_t *strong,
                                      uint64_t cap, int threads) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    off_t len = lseek(fd, 0, SEEK_END);
    close(fd);
    if (len <= 0) return 0;
    uint64_t nb = ((uint64_t)len + bs - 1) / bs;
    if (nb > cap) return -2;
    sigf_job j = {path, (uint64_t)len, bs, nb, weak, strong, 0, 0};
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, sigf_worker, &j);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j.mu);
    return j.err ? -1 : (int64_t)nb;
}

/* ------------------------------------------------------------------ */
/* Candidate map: HashMap<u32, Vec<&BlockChecksum>> (generator.rs:75-81) */
/* Chained buckets; each chain keeps insertion (= index) order.          */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t mask;
    int64_t *head;   /* bucket -> first entry (block index) or -1 */
    int64_t *next;   /* block index -> next block index with the same bucket, in index order */
    int64_t *tail;
} cand_map;

static inline uint32_t bucket_of(uint32_t w, uint32_t mask) { return (w * 0x9E3779B1u) >> 7 & mask; }

static int map_build(cand_map *m, const uint32_t *weak, uint64_t n) {
    uint32_t cap = 1;
    while (cap < 2 * n + 2 && cap < (1u << 30)) cap <<= 1;
    m->mask = cap - 1;
    m->head = (int64_t *)malloc(sizeof(int64_t) * cap);
    m->tail = (int64_t *)malloc(sizeof(int64_t) * cap);
    m->next = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    if (!m->head || !m->tail || !m->next) return -1;
    for (uint32_t i = 0; i < cap; i++) m->head[i] = m->tail[i] = -1;
    for (uint64_t i = 0; i < n; i++) {
        uint32_t b = bucket_of(weak[i], m->mask);
        m->next[i] = -1;
        if (m->tail[b] < 0) m->head[b] = (int64_t)i; else m->next[m->tail[b]] = (int64_t)i;
        m->tail[b] = (int64_t)i;
    }
    return 0;
}
static void map_free(cand_map *m) { free(m->head); free(m->tail); free(m->next); }

/* Op sink */
typedef struct { uint8_t *kind; uint64_t *a; uint64_t *b; uint64_t n, cap; int overflow; } op_sink;
static inline void emit(op_sink *o, uint8_t k, uint64_t a, uint64_t b) {
    if (o->n < o->cap) { o->kind[o->n] = k; o->a[o->n] = a; o->b[o->n] = b; }
    else o->overflow = 1;
    o->n++;
}

typedef struct {
    const uint32_t *weak; const uint64_t *strong; const uint64_t *offset; const uint64_t *size; uint64_t n;
} sigs_t;

/* Full-window probe (generator.rs:289-323 / :121-155): weak -> candidates in index
 * order -> first with equal strong wins; its size is NOT checked (:299 / :133).
 * Returns block index or -1.  *strong_calls counts Xxh3 invocations. */
static int64_t probe_full(const cand_map *m, const sigs_t *S, uint32_t weak, const uint8_t *win,
                          uint64_t bs, uint64_t *stats) {
    uint32_t b = bucket_of(weak, m->mask);
    int64_t i = m->head[b];
    int any = 0; uint64_t strong = 0;
    for (; i >= 0; i = m->next[i]) {
        if (S->weak[i] != weak) continue;
        if (!any) { any = 1; strong = oracle_xxh3_64(win, bs); if (stats) { stats[0]++; } }
        if (S->strong[i] == strong) return i;
    }
    return -1;
}
/* Tail probe (generator.rs:325-353 / :156-184): Adler32::hash(partial); candidates need
 * size == partial.len() && strong equal. */
static int64_t probe_tail(const cand_map *m, const sigs_t *S, const uint8_t *part, uint64_t plen, uint64_t *stats) {
    uint32_t weak = oracle_adler32(part, plen);
    uint32_t b = bucket_of(weak, m->mask);
    int any = 0; uint64_t strong = 0;
    for (int64_t i = m->head[b]; i >= 0; i = m->next[i]) {
        if (S->weak[i] != weak) continue;
        if (!any) { any = 1; strong = oracle_xxh3_64(part, plen); if (stats) stats[1]++; }
        if (S->size[i] == plen && S->strong[i] == strong) return i;
    }
    return -1;
}

/* generator.rs:242-379 — generate_delta on a fully loaded buffer.
 * Returns op count (may exceed cap; then only cap ops were written) or -1 on OOM.
 * stats (optional, 2 x u64): [0] full-window strong hashes, [1] tail strong hashes. */
int64_t oracle_generate_delta(const uint8_t *src, uint64_t len,
                              const uint32_t *weak, const uint64_t *strong, const uint64_t *offset,
                              const uint64_t *size, uint64_t nsig, uint64_t bs,
                              uint8_t *kind, uint64_t *a, uint64_t *b, uint64_t cap, uint64_t *stats) {
    sigs_t S = {weak, strong, offset, size, nsig};
    op_sink o = {kind, a, b, 0, cap, 0};
    if (len == 0) return 0;                                  /* :262-268 */
    cand_map m;
    if (map_build(&m, weak, nsig)) return -1;
    uint64_t lit_start = 0, lit_len = 0, pos = 0;
    oracle_rolling r; oracle_rolling_new(&r, bs);
    if (len >= bs) oracle_rolling_update_block(&r, src, bs);  /* :275-278 */
    while (pos < len) {
        int found = 0;
        uint64_t remaining = len - pos;
        if (remaining >= bs) {                               /* :285-323 */
            int64_t c = probe_full(&m, &S, oracle_rolling_digest(&r), src + pos, bs, stats);
            if (c >= 0) {
                if (lit_len) { emit(&o, 1, lit_start, lit_len); lit_len = 0; }
                emit(&o, 0, offset[c], size[c]);
                pos += bs; found = 1;
                if (pos + bs <= len) oracle_rolling_update_block(&r, src + pos, bs);
            }
        } else {                                             /* :324-353 */
            int64_t c = probe_tail(&m, &S, src + pos, remaining, stats);
            if (c >= 0) {
                if (lit_len) { emit(&o, 1, lit_start, lit_len); lit_len = 0; }
                emit(&o, 0, offset[c], size[c]);
                pos += remaining; found = 1;
            }
        }
        if (!found) {                                        /* :355-366 */
            if (!lit_len) lit_start = pos;
            lit_len++;
            pos += 1;
            if (pos > 0 && pos + bs - 1 < len) oracle_rolling_roll(&r, src[pos - 1], src[pos + bs - 1]);
        }
    }
    if (lit_len) emit(&o, 1, lit_start, lit_len);            /* :370-372 */
    map_free(&m);
    return (int64_t)o.n;
}

/* generator.rs:67-228 — generate_delta_streaming.  The source "file" is the buffer
 * `src`; each File::read returns min(chunk, bytes left) like a regular file.
 * `chunk` is CHUNK_SIZE (256 KiB in the reference, :72); tests shrink it to
 * exercise window refills.  Literal descriptors carry absolute source offsets. */
int64_t oracle_generate_delta_streaming(const uint8_t *src, uint64_t len,
                                        const uint32_t *weak, const uint64_t *strong, const uint64_t *offset,
                                        const uint64_t *size, uint64_t nsig, uint64_t bs, uint64_t chunk,
                                        uint8_t *kind, uint64_t *a, uint64_t *b, uint64_t cap, uint64_t *stats) {
    sigs_t S = {weak, strong, offset, size, nsig};
    op_sink o = {kind, a, b, 0, cap, 0};
    if (len == 0) return 0;                                  /* :86-92 */
    cand_map m;
    if (map_build(&m, weak, nsig)) return -1;
    uint64_t fpos = 0;                 /* next byte of the "file" to read */
    uint64_t wbase = 0;                /* absolute offset of window[0] */
    uint64_t wlen = 0;                 /* window.len() */
    /* The window is always a contiguous slice src[wbase .. wbase+wlen). */
    uint64_t bytes_read = len - fpos < chunk ? len - fpos : chunk;   /* :102 */
    fpos += bytes_read; wlen = bytes_read;
    oracle_rolling r; oracle_rolling_new(&r, bs);
    if (wlen >= bs) oracle_rolling_update_block(&r, src + wbase, bs);
    uint64_t wpos = 0;
    uint64_t lit_start = 0, lit_len = 0;
    while (wpos < wlen) {                                    /* :116 */
        uint64_t remaining = wlen - wpos;
        int found = 0;
        const uint8_t *w = src + wbase;
        if (remaining >= bs) {                               /* :121-155 */
            int64_t c = probe_full(&m, &S, oracle_rolling_digest(&r), w + wpos, bs, stats);
            if (c >= 0) {
                if (lit_len) { emit(&o, 1, lit_start, lit_len); lit_len = 0; }
                emit(&o, 0, offset[c], size[c]);
                wpos += bs; found = 1;
                if (wpos + bs <= wlen) oracle_rolling_update_block(&r, w + wpos, bs);
            }
        } else if (remaining > 0) {                          /* :156-184 */
            int64_t c = probe_tail(&m, &S, w + wpos, remaining, stats);
            if (c >= 0) {
                if (lit_len) { emit(&o, 1, lit_start, lit_len); lit_len = 0; }
                emit(&o, 0, offset[c], size[c]);
                wpos += remaining; found = 1;
            }
        }
        if (!found && wpos < wlen) {                         /* :186-197 */
            if (!lit_len) lit_start = wbase + wpos;
            lit_len++;
            if (wpos + bs < wlen) oracle_rolling_roll(&r, w[wpos], w[wpos + bs]);
            wpos += 1;
        }
        if (wpos >= bs && bytes_read > 0 && wlen - wpos < bs) {   /* :199-215 */
            wbase += wpos; wlen -= wpos; wpos = 0;           /* window.drain(0..window_pos) */
            bytes_read = len - fpos < chunk ? len - fpos : chunk;
            if (bytes_read > 0) {
                fpos += bytes_read; wlen += bytes_read;
                if (wlen >= bs) oracle_rolling_update_block(&r, src + wbase, bs);
            }
        }
    }
    if (lit_len) emit(&o, 1, lit_start, lit_len);
    map_free(&m);
    return (int64_t)o.n;
}

/* applier.rs:22-56 restated on buffers.  Returns bytes written, or -1 if a Copy
 * reads past the basis (read_exact error, :37). */
int64_t oracle_apply_delta(const uint8_t *basis, uint64_t basis_len, const uint8_t *src,
                           const uint8_t *kind, const uint64_t *a, const uint64_t *b, uint64_t nops,
                           uint8_t *out, uint64_t out_cap) {
    uint64_t w = 0;
    for (uint64_t i = 0; i < nops; i++) {
        const uint8_t *from;
        if (kind[i] == 0) { if (a[i] + b[i] > basis_len) return -1; from = basis + a[i]; }
        else from = src + a[i];
        if (w + b[i] > out_cap) return -1;
        memcpy(out + w, from, b[i]);
        w += b[i];
    }
    return (int64_t)w;
}
