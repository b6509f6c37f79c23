// sydelta_zstd.hpp — zstd frames (RFC 8878) for the compressed Delta JSON that sy sends
// to the receiver (src/transport/ssh.rs:1009-1017: compress(delta_json, Compression::Zstd),
// src/compress/mod.rs:71-76: zstd::Encoder level 3; the receiver decompresses with any
// zstd decoder, sy-remote.rs:160-179).
//
// Each block of <= 128 KiB of text is one Compressed block, coded two ways and the smaller
// kept: literals only (Huffman-coded, 4 streams or 1 below 1 KiB, the weights in direct
// representation; no sequences), or literals + sequences (matches at a handful of
// candidate distances -- the JSON skeleton's '{' gaps, sampled repeat distances, runs --
// with block-local repeat offsets and FSE tables from the block's own code counts).  A
// block neither shrinks is stored Raw, a block of one repeated byte RLE.  The bytes differ
// from libzstd's level 3: the contract is decode(frame) == text, checked against
// libzstd's decoder; the ratios are in DESIGN.md section 11.
//
// The functions here are the pieces every block needs whoever runs them: the device
// kernel (sydelta_kernels.hip, k_zstd_block: one workgroup per block, parallel bit
// scatter) and the sequential host encoder of the tests (tests/csrc/zstd_ref.cpp) call
// the same code builder and header writers, so their outputs must be byte-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>

namespace sydelta {
namespace zstd {

constexpr uint32_t kBlockMax = 128 * 1024;  // Block_Maximum_Size (window 128 KiB)
constexpr uint32_t kMaxBits = 11;           // Max_Number_of_Bits of a literals Huffman code
constexpr uint32_t kSymbols = 128;          // direct weight representation: symbols 0..127
constexpr uint32_t kSingleStreamMax = 1023; // 10-bit sizes: one stream below this
constexpr uint32_t kFrameHeader = 14;       // magic, FHD, Window_Descriptor, 8-byte FCS
constexpr uint32_t kStreamBytesMax = (kBlockMax / 4) * kMaxBits / 8 + 8;  // one of 4 streams

// Frame header: magic 0xFD2FB528; FHD 0xC0 (8-byte Frame_Content_Size, not single
// segment, no checksum, no dictionary); Window_Descriptor 0x38 (2^17 = 128 KiB).
__host__ __device__ __forceinline__ void frame_header(uint8_t* p, uint64_t content_size) {
    p[0] = 0x28; p[1] = 0xB5; p[2] = 0x2F; p[3] = 0xFD;
    p[4] = 0xC0;
    p[5] = 0x38;
    for (int i = 0; i < 8; ++i) p[6 + i] = (uint8_t)(content_size >> (8 * i));
}

// Block_Header: Last_Block, Block_Type (0 Raw, 1 RLE, 2 Compressed), Block_Size.
__host__ __device__ __forceinline__ void block_header(uint8_t* p, bool last, uint32_t type, uint32_t size) {
    const uint32_t h = (last ? 1u : 0u) | (type << 1) | (size << 3);
    p[0] = (uint8_t)h; p[1] = (uint8_t)(h >> 8); p[2] = (uint8_t)(h >> 16);
}

// A literals Huffman code over symbols 0..127.
struct HufCode {
    uint8_t len[kSymbols];    // code length in bits, 0 = absent
    uint16_t code[kSymbols];  // canonical code (RFC 8878 4.2.1: by weight, then symbol)
    uint32_t max_bits;        // longest code (the table log the decoder derives)
    uint32_t last;            // highest present symbol (its weight is implied)
};

// Scratch of huf_build (the device keeps it in LDS: ~3.6 KiB of private arrays would
// otherwise live in scratch memory).
struct HufWork {
    uint64_t w[2 * kSymbols];
    uint32_t depth[2 * kSymbols];
    uint16_t parent[2 * kSymbols];
    uint32_t bl[64];
    uint8_t sym[kSymbols];
};

// Length-limited Huffman code for the histogram h (h[s] = count of symbol s, s < 128,
// at least two symbols present).  Optimal lengths from the two-queue merge over the
// symbols sorted by (count, symbol), then lengths above kMaxBits folded back with the
// JPEG Annex K.3 adjustment (Kraft sum stays 1) and handed out again in frequency order.
// Deterministic: host and device derive the same code.
__host__ __device__ inline void huf_build(const uint32_t* h, HufCode& c, HufWork& wk) {
    uint8_t* sym = wk.sym;
    uint64_t* w = wk.w;
    uint16_t* parent = wk.parent;
    uint32_t* depth = wk.depth;
    uint32_t* bl = wk.bl;
    uint32_t n = 0;
    for (uint32_t s = 0; s < kSymbols; ++s) {
        c.len[s] = 0;
        c.code[s] = 0;
        if (h[s]) sym[n++] = (uint8_t)s;
    }
    // insertion sort by (count, symbol) ascending
    for (uint32_t i = 1; i < n; ++i) {
        const uint8_t x = sym[i];
        uint32_t j = i;
        while (j > 0 && (h[sym[j - 1]] > h[x] || (h[sym[j - 1]] == h[x] && sym[j - 1] > x))) {
            sym[j] = sym[j - 1];
            --j;
        }
        sym[j] = x;
    }
    // two-queue Huffman: leaves 0..n-1 (sorted), internal nodes n..2n-2 in creation order
    for (uint32_t i = 0; i < n; ++i) w[i] = h[sym[i]];
    uint32_t li = 0, ni = n, nn = n;
    auto pick = [&]() -> uint32_t {
        if (li < n && (ni >= nn || w[li] <= w[ni])) return li++;
        return ni++;
    };
    while (nn < 2 * n - 1) {
        const uint32_t a = pick(), b = pick();
        w[nn] = w[a] + w[b];
        parent[a] = parent[b] = (uint16_t)nn;
        ++nn;
    }
    depth[2 * n - 2] = 0;
    for (uint32_t i = 2 * n - 2; i-- > 0;) depth[i] = depth[parent[i]] + 1;
    // counts per length; fold lengths > kMaxBits (JPEG Annex K.3)
    for (uint32_t i = 0; i < 64; ++i) bl[i] = 0;
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t d = depth[i] < 63 ? depth[i] : 63;
        ++bl[d];
        if (d > maxlen) maxlen = d;
    }
    for (uint32_t i = maxlen; i > kMaxBits; --i) {
        while (bl[i] > 0) {
            uint32_t j = i - 2;
            while (j > 1 && bl[j] == 0) --j;
            bl[i] -= 2;
            bl[i - 1] += 1;
            bl[j + 1] += 2;
            bl[j] -= 1;
        }
    }
    // lengths back to the symbols: the least frequent get the longest codes
    uint32_t k = 0;
    c.max_bits = 0;
    for (uint32_t L = (maxlen < kMaxBits ? maxlen : kMaxBits); L >= 1; --L)
        for (uint32_t m = 0; m < bl[L]; ++m, ++k) {
            c.len[sym[k]] = (uint8_t)L;
            if (L > c.max_bits) c.max_bits = L;
        }
    // canonical codes: longest first, ascending symbols within a length
    uint32_t next = 0;
    for (uint32_t L = c.max_bits; L >= 1; --L) {
        for (uint32_t s = 0; s < kSymbols; ++s)
            if (c.len[s] == L) c.code[s] = (uint16_t)next++;
        next >>= 1;
    }
    c.last = 0;
    for (uint32_t s = 0; s < kSymbols; ++s)
        if (c.len[s]) c.last = s;
}

// Huffman_Tree_Description, direct representation: headerByte = 127 + Number_of_Symbols
// (the symbols before the last present one), then their 4-bit weights, two per byte,
// the first in the high nibble; Weight = max_bits + 1 - length (0 = absent).  Returns
// its size.
__host__ __device__ inline uint32_t huf_tree_desc(const HufCode& c, uint8_t* p) {
    const uint32_t ns = c.last;  // weights stored for symbols 0 .. last-1
    p[0] = (uint8_t)(127 + ns);
    for (uint32_t i = 0; i < (ns + 1) / 2; ++i) p[1 + i] = 0;
    for (uint32_t s = 0; s < ns; ++s) {
        const uint32_t wt = c.len[s] ? c.max_bits + 1 - c.len[s] : 0;
        p[1 + s / 2] |= (uint8_t)((s & 1) ? wt : (wt << 4));
    }
    return 1 + (ns + 1) / 2;
}

// Literals_Section_Header of Compressed literals: one stream with 10-bit sizes (3 bytes)
// or four streams with 18-bit sizes (5 bytes).  Returns its size.
__host__ __device__ __forceinline__ uint32_t lit_header(uint8_t* p, bool four, uint32_t regen, uint32_t comp) {
    if (!four) {
        const uint32_t v = 2u | (0u << 2) | (regen << 4) | (comp << 14);
        p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16);
        return 3;
    }
    const uint64_t v = 2ull | (3ull << 2) | ((uint64_t)regen << 4) | ((uint64_t)comp << 22);
    for (int i = 0; i < 5; ++i) p[i] = (uint8_t)(v >> (8 * i));
    return 5;
}

// Stream s of a block of `regen` literals: [first, first + count).
__host__ __device__ __forceinline__ void stream_range(uint32_t regen, bool four, uint32_t s, uint32_t& first,
                                                      uint32_t& count) {
    if (!four) { first = 0; count = regen; return; }
    const uint32_t seg = (regen + 3) / 4;
    first = s * seg < regen ? s * seg : regen;
    const uint32_t end = s == 3 ? regen : ((s + 1) * seg < regen ? (s + 1) * seg : regen);
    count = end - first;
}

// ---------------------------------------------------------------------------
// Sequences (matches): RFC 8878 3.1.1.3.2, predefined FSE tables only
// ---------------------------------------------------------------------------
// A Delta's JSON repeats one skeleton per op ({"Copy":{"offset":...,"size":...}}), so the
// matches that pay are at the distance of the previous op's text.  Candidate distances
// are 1 (runs), the block's most common gaps between consecutive '{', and its most common
// short repeat distances (every kRepStep-th position's nearest earlier copy of its next 4
// bytes within 255: a Data op's repeated numbers, other periodic text); each position's
// best candidate is found independently (the device does all positions at once), a
// greedy parse takes a match of >= kMinMatch wherever one starts, and the sequences are
// FSE-coded with tables built from the block's own code counts (RLE for a code that
// never changes).
constexpr uint32_t kMinMatch = 6;
constexpr uint32_t kProbe = 32;     // bytes compared per candidate when ranking them
constexpr uint32_t kGapCands = 4;   // most common '{' gaps
constexpr uint32_t kRepCands = 3;   // most common sampled repeat distances
constexpr uint32_t kCands = 1 + kGapCands + kRepCands;
constexpr uint32_t kRepStep = 8;    // positions between repeat-distance samples
constexpr uint32_t kRepMin = 4;     // samples a repeat distance needs to become a candidate
constexpr uint32_t kMaxSeq = kBlockMax / kMinMatch;

// Literals_Length / Match_Length codes (RFC 8878 3.1.1.3.2.1.1): code, its extra bits.
// Lengths past the table's irregular start follow the highest set bit (zstd's
// ZSTD_LLcode / ZSTD_MLcode deltas 19 and 36); the tables are namespace-scope constants
// (a per-call array initialised in private memory made each code a scratch round trip
// on the device).
constexpr uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                                  20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
constexpr uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint32_t kMLBase[21] = {35,  37,  39,  41,   43,   47,   51,   59,    67,    83,    99,
                                  131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
constexpr uint8_t kMLBits[21] = {1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__host__ __device__ __forceinline__ uint32_t highbit32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
__host__ __device__ __forceinline__ void ll_code(uint32_t ll, uint32_t& code, uint32_t& bits) {
    if (ll < 16) { code = ll; bits = 0; return; }
    if (ll >= 64) {  // codes 25..35: [2^h, 2^(h+1)) with h extra bits
        const uint32_t h = highbit32(ll);
        code = h < 16 ? h + 19 : 35u;
        bits = kLLBits[code];
        return;
    }
    uint32_t c = 24;
    while (kLLBase[c] > ll) --c;
    code = c;
    bits = kLLBits[c];
}
__host__ __device__ __forceinline__ void ml_code(uint32_t ml, uint32_t& code, uint32_t& bits) {
    if (ml < 35) { code = ml - 3; bits = 0; return; }
    if (ml >= 131) {  // codes 43..52: ml - 3 in [2^h, 2^(h+1)) with h extra bits
        const uint32_t h = highbit32(ml - 3);
        const uint32_t c = h < 16 ? h + 4 : 20u;  // index into kMLBase (h = 7 -> 11)
        code = 32 + c;
        bits = kMLBits[c];
        return;
    }
    uint32_t c = 10;
    while (kMLBase[c] > ml) --c;
    code = 32 + c;
    bits = kMLBits[c];
}

// One FSE compression table built from a normalized distribution (zstd's
// FSE_buildCTable: symbols spread with step 5/8 table + 3, "less than 1" symbols in the
// top cells, state table sorted by symbol).
struct FseCT {
    uint16_t state[512];    // next-state table (tableSize entries, log <= 9)
    int32_t delta_nb[53];   // deltaNbBits per symbol
    int32_t delta_find[53]; // deltaFindState per symbol
    uint32_t log;
};
// The table builds' work arrays (the device keeps them in LDS: as a thread's private
// arrays they live in scratch memory, a round trip per access in the spreading loops).
struct FseWork {
    uint8_t sym[512];
    uint32_t cumul[54];
    int16_t norm[53];
};
__host__ __device__ inline void fse_build(FseCT& t, const int16_t* norm, uint32_t nsym, uint32_t log, FseWork& fw) {
    const uint32_t size = 1u << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint8_t* sym = fw.sym;
    uint32_t* cumul = fw.cumul;
    uint32_t high = size - 1;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= nsym; ++u) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            sym[high--] = (uint8_t)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
        }
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s < nsym; ++s)
        for (int k = 0; k < norm[s]; ++k) {
            sym[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < size; ++u) t.state[cumul[sym[u]]++] = (uint16_t)(size + u);
    int32_t total = 0;
    for (uint32_t s = 0; s < nsym; ++s) {
        const int n = norm[s];
        if (n == 0) {  // absent: never coded (zstd's case 0)
            t.delta_nb[s] = (int32_t)(((log + 1) << 16) - (1u << log));
            t.delta_find[s] = 0;
        } else if (n == -1 || n == 1) {
            t.delta_nb[s] = (int32_t)((log << 16) - (1u << log));
            t.delta_find[s] = total - 1;
            total += 1;
        } else {
            uint32_t hb = 0;
            while ((2u << hb) <= (uint32_t)(n - 1)) ++hb;  // highbit(n - 1), n >= 2
            const uint32_t max_out = log - hb;
            t.delta_nb[s] = (int32_t)((max_out << 16) - ((uint32_t)n << max_out));
            t.delta_find[s] = total - n;
            total += n;
        }
    }
    t.log = log;
}

// Backward bitstream writer (zstd's BIT_CStream): bits LSB-first, whole bytes out.
struct BitW {
    uint8_t* p;
    uint32_t bytes;
    uint64_t acc;
    uint32_t nb;
    __host__ __device__ void add(uint64_t v, uint32_t n) {
        if (!n) return;
        acc |= (v & ((1ull << n) - 1)) << nb;
        nb += n;
        while (nb >= 8) { p[bytes++] = (uint8_t)acc; acc >>= 8; nb -= 8; }
    }
    __host__ __device__ void close() {
        add(1, 1);
        if (nb) { p[bytes++] = (uint8_t)acc; acc = 0; nb = 0; }
    }
};
__host__ __device__ __forceinline__ uint32_t fse_init(const FseCT& t, uint32_t s) {
    const uint32_t nbo = (uint32_t)((t.delta_nb[s] + (1 << 15)) >> 16);
    const uint32_t v = (nbo << 16) - (uint32_t)t.delta_nb[s];
    return t.state[(v >> nbo) + t.delta_find[s]];
}
__host__ __device__ __forceinline__ void fse_encode(BitW& w, const FseCT& t, uint32_t& st, uint32_t s) {
    const uint32_t nbo = (uint32_t)((int32_t)st + t.delta_nb[s]) >> 16;
    w.add(st, nbo);
    st = t.state[(st >> nbo) + t.delta_find[s]];
}

struct Seq {
    uint32_t ll, ml, off;  // literal length, match length (>= kMinMatch), distance
    uint32_t ov;           // Offset_Value: 1-3 a repeat offset, else off + 3 (rep_code)
};

// Offset_Value of a match at distance d after ll literals, and the decoder's update of
// the repeat-offset history (RFC 8878 3.1.1.5; zstd's ZSTD_updateRep).  Blocks are coded
// independently, so the history a block enters with is unknown to its coder: rep[] holds
// only what this block's own sequences put there (0 = unknown), and a repeat code is used
// only for a known entry.  Index r of the repeated offset is Offset_Value - 1, plus 1
// when ll == 0 (then r = 3 means rep[0] - 1).
// The history as three scalars (no indexed array: on the device an indexed private array
// lives in scratch memory, a round trip per access in a loop over every sequence).
__host__ __device__ __forceinline__ uint32_t rep_code3(uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t ll,
                                                       uint32_t d) {
    const uint32_t ll0 = ll == 0 ? 1u : 0u;
    const uint32_t c3 = r0 > 1 ? r0 - 1 : 0u;  // candidate r = 3: rep[0] - 1
    // candidates r = ll0 .. ll0 + 2 in order: (r0, r1, r2) or (r1, r2, r0 - 1)
    const uint32_t va = ll0 ? r1 : r0, vb = ll0 ? r2 : r1, vc = ll0 ? c3 : r2;
    uint32_t ov = d + 3;
    if (va && va == d) ov = 1;
    else if (vb && vb == d) ov = 2;
    else if (vc && vc == d) ov = 3;
    if (ov > 3) {
        r2 = r1;
        r1 = r0;
        r0 = d;
    } else if (ov - 1 + ll0 > 0) {
        if (ov - 1 + ll0 >= 2) r2 = r1;
        r1 = r0;
        r0 = d;
    }
    return ov;
}
__host__ __device__ __forceinline__ uint32_t rep_code(uint32_t* rep, uint32_t ll, uint32_t d) {
    return rep_code3(rep[0], rep[1], rep[2], ll, d);
}

// Normalized counts of a block's codes (FSE_Compressed mode): table log L in [5, maxlog]
// with 2^L >= 2 x the distinct codes, every present code >= 1, the rounding error taken
// from / given to the most frequent codes.  Deterministic (host and device alike).
__host__ __device__ inline uint32_t fse_normalize(const uint32_t* cnt, uint32_t nsym, uint32_t total, uint32_t maxlog,
                                                  int16_t* norm) {
    uint32_t distinct = 0;
    for (uint32_t s = 0; s < nsym; ++s) distinct += cnt[s] != 0;
    uint32_t L = 5;
    while (L < maxlog && ((1u << L) < 2 * distinct || (1u << L) < total)) ++L;
    const uint32_t size = 1u << L;
    int32_t sum = 0;
    for (uint32_t s = 0; s < nsym; ++s) {
        int32_t v = 0;
        if (cnt[s]) {
            v = (int32_t)(((uint64_t)cnt[s] * size) / total);
            if (v < 1) v = 1;
        }
        norm[s] = (int16_t)v;
        sum += v;
    }
    // the difference goes to (or comes from) the largest entries, one step at a time
    while (sum != (int32_t)size) {
        uint32_t big = 0;
        for (uint32_t s = 1; s < nsym; ++s)
            if (norm[s] > norm[big]) big = s;
        if (sum < (int32_t)size) {
            norm[big] = (int16_t)(norm[big] + ((int32_t)size - sum));
            sum = (int32_t)size;
        } else {
            const int32_t take = sum - (int32_t)size < norm[big] - 1 ? sum - (int32_t)size : norm[big] - 1;
            norm[big] = (int16_t)(norm[big] - take);
            sum -= take;
            if (take == 0) break;  // cannot happen with 2^L >= 2 x distinct
        }
    }
    return L;
}

// FSE table description (RFC 8878 4.1.1; zstd's FSE_writeNCount): accuracy log - 5, then
// each count + 1 in a variable number of bits, a run of zero counts as 2-bit repeat
// flags.  Returns its size.
__host__ __device__ inline uint32_t fse_write_ncount(uint8_t* out, const int16_t* norm, uint32_t nsym, uint32_t L) {
    uint32_t o = 0;
    uint32_t bits = (L - 5), nbits = 4;
    int32_t remaining = (1 << L) + 1, threshold = 1 << L;
    uint32_t nb = L + 1;
    uint32_t s = 0;
    bool prev0 = false;
    uint32_t last = nsym;  // past the last nonzero count
    while (last > 0 && norm[last - 1] == 0) --last;
    auto flush16 = [&]() {
        if (nbits > 16) {
            out[o++] = (uint8_t)bits;
            out[o++] = (uint8_t)(bits >> 8);
            bits >>= 16;
            nbits -= 16;
        }
    };
    while (s < last && remaining > 1) {
        if (prev0) {
            uint32_t start = s;
            while (s < last && !norm[s]) ++s;
            while (s >= start + 24) {
                start += 24;
                bits += 0xFFFFu << nbits;
                out[o++] = (uint8_t)bits;
                out[o++] = (uint8_t)(bits >> 8);
                bits >>= 16;
            }
            while (s >= start + 3) {
                start += 3;
                bits += 3u << nbits;
                nbits += 2;
            }
            bits += (s - start) << nbits;
            nbits += 2;
            flush16();
        }
        int32_t count = norm[s++];
        const int32_t mx = (2 * threshold - 1) - remaining;
        remaining -= count < 0 ? -count : count;
        count++;
        if (count >= threshold) count += mx;
        bits += (uint32_t)count << nbits;
        nbits += nb;
        nbits -= count < mx ? 1u : 0u;
        prev0 = count == 1;
        while (remaining < threshold) {
            --nb;
            threshold >>= 1;
        }
        flush16();
    }
    out[o++] = (uint8_t)bits;
    out[o++] = (uint8_t)(bits >> 8);
    o -= 2;
    o += (nbits + 7) / 8;
    return o;
}

// One code's table for a block: RLE (one distinct code: mode 1, the table is that byte)
// or FSE_Compressed (mode 2) from the block's counts.  Writes the table description at
// out, returns its size; *mode, and t for the coder (log 0 for RLE: no state bits).
__host__ __device__ inline uint32_t seq_table(const uint32_t* cnt, uint32_t nsym, uint32_t total, uint32_t maxlog,
                                              FseCT& t, uint32_t* mode, uint8_t* out, FseWork& fw) {
    uint32_t distinct = 0, only = 0;
    for (uint32_t s = 0; s < nsym; ++s)
        if (cnt[s]) { ++distinct; only = s; }
    if (distinct == 1) {
        *mode = 1;
        out[0] = (uint8_t)only;
        for (uint32_t s = 0; s < nsym; ++s) { t.delta_nb[s] = 0; t.delta_find[s] = 0; }
        t.state[0] = 0;
        t.state[1] = 0;
        t.log = 0;
        return 1;
    }
    int16_t* norm = fw.norm;
    const uint32_t L = fse_normalize(cnt, nsym, total, maxlog, norm);
    fse_build(t, norm, nsym, L, fw);
    *mode = 2;
    return fse_write_ncount(out, norm, nsym, L);
}

// The codes of a sequence.
__host__ __device__ __forceinline__ void seq_codes(const Seq& q, uint32_t& lc, uint32_t& lb, uint32_t& mc,
                                                   uint32_t& mb, uint32_t& oc, uint32_t& ov) {
    ll_code(q.ll, lc, lb);
    ml_code(q.ml, mc, mb);
    ov = q.ov;
    oc = highbit32(ov);  // ov >= 1
}

// Sequences_Section of ns sequences into p; returns its size.  Tables per block (RLE or
// FSE_Compressed from the block's code counts; the FseCT arguments are scratch, sized for
// tables up to log 9).  Order of zstd's ZSTD_encodeSequences: the last sequence starts
// the states, then every earlier one from the end: OF, ML, LL state bits, then LL, ML, OF
// extra bits; states flushed ML, OF, LL (the decoder reads LL, OF, ML first).
// The code counts of ns sequences (zeroed first).  The device counts in parallel instead.
__host__ __device__ inline void seq_counts(const Seq* sq, uint32_t ns, uint32_t* cll, uint32_t* cml, uint32_t* cof) {
    for (uint32_t i = 0; i < 36; ++i) cll[i] = 0;
    for (uint32_t i = 0; i < 53; ++i) cml[i] = 0;
    for (uint32_t i = 0; i < 32; ++i) cof[i] = 0;
    uint32_t lc, lb, mc, mb, oc, ov;
    for (uint32_t i = 0; i < ns; ++i) {
        seq_codes(sq[i], lc, lb, mc, mb, oc, ov);
        ++cll[lc];
        ++cml[mc];
        ++cof[oc];
    }
}

// Sequences_Section from the code counts (seq_counts).  The sequences are read last to
// first, eight at a time (independent loads in flight: a one-thread loop over
// sequences in HBM otherwise waits a full round trip per sequence).
// The Sequences_Section header: Number_of_Sequences, the modes byte and the three tables
// (built into tll / tml / tof).  Returns its size.
__host__ __device__ inline uint32_t seq_section_head(uint32_t ns, uint8_t* p, const uint32_t* cll, const uint32_t* cml,
                                                     const uint32_t* cof, FseCT& tll, FseCT& tml, FseCT& tof,
                                                     FseWork& fw) {
    uint32_t o = 0;
    if (ns < 128) {
        p[o++] = (uint8_t)ns;
    } else if (ns < 0x7F00) {
        p[o++] = (uint8_t)((ns >> 8) + 0x80);
        p[o++] = (uint8_t)ns;
    } else {
        p[o++] = 0xFF;
        p[o++] = (uint8_t)(ns - 0x7F00);
        p[o++] = (uint8_t)((ns - 0x7F00) >> 8);
    }
    if (!ns) return o;
    const uint32_t modes_at = o++;
    uint32_t mll, mof, mml;
    o += seq_table(cll, 36, ns, 9, tll, &mll, p + o, fw);
    o += seq_table(cof, 32, ns, 8, tof, &mof, p + o, fw);
    o += seq_table(cml, 53, ns, 9, tml, &mml, p + o, fw);
    p[modes_at] = (uint8_t)((mll << 6) | (mof << 4) | (mml << 2));
    return o;
}

__host__ __device__ inline uint32_t seq_section_counted(const Seq* sq, uint32_t ns, uint8_t* p, const uint32_t* cll,
                                                        const uint32_t* cml, const uint32_t* cof, FseCT& tll,
                                                        FseCT& tml, FseCT& tof) {
    FseWork fw;
    const uint32_t o = seq_section_head(ns, p, cll, cml, cof, tll, tml, tof, fw);
    if (!ns) return o;
    uint32_t lc, lb, mc, mb, oc, ov;
    BitW w{p + o, 0, 0, 0};
    seq_codes(sq[ns - 1], lc, lb, mc, mb, oc, ov);
    uint32_t sml = tml.log ? fse_init(tml, mc) : 0, sof = tof.log ? fse_init(tof, oc) : 0;
    uint32_t sll = tll.log ? fse_init(tll, lc) : 0;
    w.add(sq[ns - 1].ll, lb);
    w.add(sq[ns - 1].ml - 3, mb);
    w.add(ov, oc);
    constexpr uint32_t kAhead = 8;
    for (uint32_t hi = ns - 1; hi > 0;) {  // sequences [lo, hi), last first
        const uint32_t lo = hi > kAhead ? hi - kAhead : 0;
        Seq q[kAhead];
#pragma unroll
        for (uint32_t k = 0; k < kAhead; ++k)
            if (lo + k < hi) q[k] = sq[lo + k];
#pragma unroll
        for (uint32_t k = kAhead; k-- > 0;) {
            if (lo + k >= hi) continue;
            seq_codes(q[k], lc, lb, mc, mb, oc, ov);
            if (tof.log) fse_encode(w, tof, sof, oc);
            if (tml.log) fse_encode(w, tml, sml, mc);
            if (tll.log) fse_encode(w, tll, sll, lc);
            w.add(q[k].ll, lb);
            w.add(q[k].ml - 3, mb);
            w.add(ov, oc);
        }
        hi = lo;
    }
    w.add(sml, tml.log);
    w.add(sof, tof.log);
    w.add(sll, tll.log);
    w.close();
    return o + w.bytes;
}

__host__ __device__ inline uint32_t seq_section(const Seq* sq, uint32_t ns, uint8_t* p, FseCT& tll, FseCT& tml,
                                                FseCT& tof) {
    uint32_t cll[36], cml[53], cof[32];
    seq_counts(sq, ns, cll, cml, cof);
    return seq_section_counted(sq, ns, p, cll, cml, cof, tll, tml, tof);
}

// Raw_Literals_Block header (1, 2 or 3 bytes by size); returns its size.
__host__ __device__ __forceinline__ uint32_t raw_lit_header(uint8_t* p, uint32_t n) {
    if (n < 32) { p[0] = (uint8_t)(n << 3); return 1; }
    if (n < 4096) { p[0] = (uint8_t)((1u << 2) | ((n & 15) << 4)); p[1] = (uint8_t)(n >> 4); return 2; }
    p[0] = (uint8_t)((3u << 2) | ((n & 15) << 4)); p[1] = (uint8_t)(n >> 4); p[2] = (uint8_t)(n >> 12);
    return 3;
}

// The '{' at p counts its distances (<= 255) to the three '{' before it: a Copy op's
// text holds two, so its distance to the previous op's is the second or third.
template <class T>
__host__ __device__ __forceinline__ void gap_count(const T& in, uint32_t p, uint32_t* gaps) {
    uint32_t seen = 0;
    for (uint32_t d = 1; d < 256 && d <= p && seen < 3; ++d)
        if (in[p - d] == '{') {
            ++gaps[d];
            ++seen;
        }
}

// Repeat distance of position p (sampled every kRepStep positions): the smallest d in
// [2, 255] with in[p, p+4) == in[p-d, p-d+4), 0 when there is none or the 4 bytes
// continue a run (distance 1 is always a candidate).
template <class T>
__host__ __device__ inline uint32_t repeat_dist(const T& in, uint32_t n, uint32_t p) {
    if (p < 2 || p + 4 > n) return 0;
    const uint8_t b0 = in[p], b1 = in[p + 1], b2 = in[p + 2], b3 = in[p + 3];
    if (in[p - 1] == b0 && b0 == b1 && b1 == b2 && b2 == b3) return 0;
    const uint32_t lim = p < 255 ? p : 255;
    // the 4 bytes at p - d as one word, slid back a byte per step (one read per distance)
    const uint32_t v = (uint32_t)b0 | ((uint32_t)b1 << 8) | ((uint32_t)b2 << 16) | ((uint32_t)b3 << 24);
    uint32_t w = (uint32_t)in[p - 2] | ((uint32_t)in[p - 1] << 8) | ((uint32_t)b0 << 16) | ((uint32_t)b1 << 24);
    for (uint32_t d = 2; d <= lim; ++d) {
        if (w == v) return d;
        if (d < lim) w = (w << 8) | (uint32_t)in[p - d - 1];
    }
    return 0;
}

// Candidate distances of a block: 1, then the most common '{' distances (gap_count), then
// the most common sampled repeat distances (repeat_dist) seen >= kRepMin times, each list
// without the distances already taken, ties to the smaller distance.  Returns the count
// (<= kCands).
__host__ __device__ inline uint32_t pick_cands(const uint32_t* gaps, const uint32_t* reps, uint32_t* cand) {
    uint32_t k = 0;
    cand[k++] = 1;
    for (uint32_t list = 0; list < 2; ++list) {
        const uint32_t* h = list == 0 ? gaps : reps;
        const uint32_t want = list == 0 ? kGapCands : kRepCands, floor = list == 0 ? 1u : kRepMin;
        for (uint32_t taken = 0; taken < want; ++taken) {
            uint32_t best = 0, bc = 0;
            for (uint32_t g = 2; g < 256; ++g) {
                bool dup = false;
                for (uint32_t j = 0; j < k; ++j) dup |= cand[j] == g;
                if (!dup && h[g] >= floor && h[g] > bc) { bc = h[g]; best = g; }
            }
            if (!bc) break;
            cand[k++] = best;
        }
    }
    return k;
}

// Best candidate at position p of in[0, n): the longest match (compared up to kProbe
// bytes) among the candidates, ties to the earlier candidate; 0 when < kMinMatch.
// Packed as (length << 24) | distance.
// Four bytes from any address, little-endian (one unaligned dword load on the device).
__host__ __device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
// How many bytes in[a, a + lim) and in[b, b + lim) share from their start: four at a time.
__host__ __device__ __forceinline__ uint32_t common_len(const uint8_t* in, uint32_t a, uint32_t b, uint32_t lim) {
    uint32_t l = 0;
    for (; l + 4 <= lim; l += 4)
        if (const uint32_t x = ld32u(in + a + l) ^ ld32u(in + b + l)) return l + ((uint32_t)__builtin_ctz(x) >> 3);
    while (l < lim && in[a + l] == in[b + l]) ++l;
    return l;
}
// common_len(in, p, q, kProbe) with the kProbe bytes at p already loaded (w): past a
// first word that matches, the seven other loads at q issued together.
__host__ __device__ __forceinline__ uint32_t probe_len(const uint32_t* w, const uint8_t* in, uint32_t q) {
    // the first four bytes alone decide most candidates (below kMinMatch either way)
    if (const uint32_t x = w[0] ^ ld32u(in + q)) return (uint32_t)__builtin_ctz(x) >> 3;
    uint32_t l = kProbe;
#pragma unroll
    for (uint32_t k = kProbe / 4; k-- > 1;)
        if (const uint32_t x = w[k] ^ ld32u(in + q + 4 * k)) l = 4 * k + ((uint32_t)__builtin_ctz(x) >> 3);
    return l;
}
__host__ __device__ __forceinline__ uint32_t best_at(const uint8_t* in, uint32_t n, uint32_t p, const uint32_t* cand,
                                                     uint32_t nc) {
    uint32_t bl = 0, bi = 0;
    if (p + kProbe <= n) {
        uint32_t w[kProbe / 4];
#pragma unroll
        for (uint32_t k = 0; k < kProbe / 4; ++k) w[k] = ld32u(in + p + 4 * k);
        for (uint32_t c = 0; c < nc; ++c) {
            const uint32_t d = cand[c];
            if (d > p) continue;
            const uint32_t l = probe_len(w, in, p - d);
            if (l > bl) { bl = l; bi = c; }
        }
    } else {
        for (uint32_t c = 0; c < nc; ++c) {
            const uint32_t d = cand[c];
            if (d > p) continue;
            const uint32_t l = common_len(in, p, p - d, n - p);
            if (l > bl) { bl = l; bi = c; }
        }
    }
    return bl >= kMinMatch ? (bl << 24) | cand[bi] : 0;
}

// Hash candidates, for matches at any distance inside the block (a Data op's numbers
// repeat hundreds of bytes apart): the block in rounds of kHashRound positions; a position
// looks up the last earlier-round position whose next 4 bytes hash alike (tab: position +
// 1, 0 empty) and takes that match when it is longer than its best candidate and at least
// kHashMinNear (distance < kHashNear) or kHashMinFar bytes long (a far offset costs more
// bits); after the round every position of it is put (the later position wins).  The
// device runs a round's lookups in parallel, then its puts (atomicMax): the same table.
constexpr uint32_t kHashBits = 13, kHashRound = 2048, kHashMinNear = 6, kHashMinFar = 8, kHashNear = 4096;
__host__ __device__ __forceinline__ uint32_t hash4(const uint8_t* in, uint32_t p) {
    return (ld32u(in + p) * 2654435761u) >> (32 - kHashBits);  // the 4 bytes little-endian
}
__host__ __device__ __forceinline__ void hash_look(const uint8_t* in, uint32_t n, uint32_t p, const uint32_t* tab,
                                                   uint32_t* best) {
    if (p + 4 > n) return;
    const uint32_t e = tab[hash4(in, p)];
    if (!e) return;
    const uint32_t q = e - 1, d = p - q;
    const uint32_t lim = (n - p) < kProbe ? (n - p) : kProbe;
    const uint32_t l = common_len(in, p, q, lim);
    if (l >= (d < kHashNear ? kHashMinNear : kHashMinFar) && l > (best[p] >> 24)) best[p] = (l << 24) | d;
}
__host__ __device__ __forceinline__ void hash_put(const uint8_t* in, uint32_t n, uint32_t p, uint32_t* tab) {
    if (p + 4 > n) return;
    uint32_t& e = tab[hash4(in, p)];
    if (p + 1 > e) e = p + 1;
}

// Greedy parse of a block from the per-position bests.  Its path is a function of the
// position alone (so the device resolves it in parallel, k_zstd_block): at p a match when
// parse_take (a best starts there and the next position's is not longer: a one-position
// lazy parse) of match_len bytes (the best, extended past kProbe at its own distance),
// else one literal.  The distance a sequence codes depends on the repeat history: the
// repeat distance rep[0] when it matches as far (matches of <= kProbe bytes; seq_dist).
__host__ __device__ __forceinline__ bool parse_take(const uint32_t* best, uint32_t n, uint32_t p) {
    const uint32_t b = best[p];
    return b && !(p + 1 < n && (best[p + 1] >> 24) > (b >> 24));
}
__host__ __device__ __forceinline__ uint32_t match_len(const uint8_t* in, uint32_t n, uint32_t p, uint32_t b) {
    uint32_t l = b >> 24;
    const uint32_t d = b & 0xFFFFFFu;
    if (l == kProbe) l += common_len(in, p + l, p + l - d, n - p - l);
    return l;
}
__host__ __device__ __forceinline__ uint32_t seq_dist(const uint8_t* in, uint32_t p, uint32_t l, uint32_t d0,
                                                      const uint32_t* rep) {
    if (rep[0] && rep[0] != d0 && rep[0] <= p) {  // an equally long match at the repeat distance is cheaper
        if (common_len(in, p, p - rep[0], l) >= l) return rep[0];
    }
    return d0;
}

// The parse, sequentially: literal bytes gathered into lit.  Returns the number of
// sequences; *nlit = literals (including the last ones, after the last sequence);
// *covered = matched bytes.
__host__ __device__ inline uint32_t greedy_parse(const uint8_t* in, uint32_t n, const uint32_t* best,
                                                 const uint32_t* cand, Seq* sq, uint8_t* lit, uint32_t* nlit,
                                                 uint32_t* covered) {
    uint32_t p = 0, ls = 0, ns = 0, nl = 0, cov = 0;
    uint32_t rep[3] = {0, 0, 0};
    while (p < n) {
        if (!parse_take(best, n, p)) { lit[nl++] = in[p++]; continue; }
        const uint32_t b = best[p];
        const uint32_t l = match_len(in, n, p, b);
        const uint32_t d = seq_dist(in, p, l, b & 0xFFFFFFu, rep);
        sq[ns] = Seq{p - ls, l, d, 0};
        sq[ns].ov = rep_code(rep, p - ls, d);
        ++ns;
        cov += l;
        p += l;
        ls = p;
    }
    *nlit = nl;
    *covered = cov;
    return ns;
}

// Literals section of lit[0, nl): Huffman-coded (4 streams above kSingleStreamMax
// literals, else 1) when that is possible and smaller than the raw section, else Raw.
// scratch holds 4 * kStreamBytesMax bytes.  Returns its size (<= nl + 3).
__host__ __device__ inline uint32_t lit_section_seq(const uint8_t* lit, uint32_t nl, uint8_t* out, uint8_t* scratch,
                                                    uint32_t* h, HufCode& c, HufWork& wk) {
    for (uint32_t s = 0; s < 256; ++s) h[s] = 0;
    for (uint32_t i = 0; i < nl; ++i) ++h[lit[i]];
    uint32_t distinct = 0, hi = 0;
    for (uint32_t s = 0; s < 256; ++s)
        if (h[s]) { ++distinct; hi = s; }
    auto raw = [&]() -> uint32_t {
        const uint32_t hs = raw_lit_header(out, nl);
        for (uint32_t i = 0; i < nl; ++i) out[hs + i] = lit[i];
        return hs + nl;
    };
    const uint32_t raw_size = nl + (nl < 32 ? 1 : nl < 4096 ? 2 : 3);
    if (distinct < 2 || hi >= kSymbols) return raw();
    huf_build(h, c, wk);
    const bool four = nl > kSingleStreamMax;
    const uint32_t hs = four ? 5 : 3;
    const uint32_t tsz = huf_tree_desc(c, out + hs);
    uint32_t o = hs + tsz + (four ? 6 : 0);
    uint32_t ssz[4] = {0, 0, 0, 0};
    for (uint32_t st = 0; st < (four ? 4u : 1u); ++st) {
        uint32_t f, cnt;
        stream_range(nl, four, st, f, cnt);
        // symbols last to first, LSB-first, then the closing 1 bit (BIT_closeCStream)
        uint8_t* w = scratch + st * kStreamBytesMax;
        uint32_t bytes = 0, nb = 0;
        uint64_t acc = 0;
        for (uint32_t i = cnt; i-- > 0;) {
            acc |= (uint64_t)c.code[lit[f + i]] << nb;
            nb += c.len[lit[f + i]];
            while (nb >= 8) { w[bytes++] = (uint8_t)acc; acc >>= 8; nb -= 8; }
        }
        acc |= 1ull << nb;
        ++nb;
        while (nb > 0) { w[bytes++] = (uint8_t)acc; acc >>= 8; nb = nb > 8 ? nb - 8 : 0; }
        if (o + bytes >= raw_size || (!four && o + bytes - hs > kSingleStreamMax)) return raw();
        for (uint32_t i = 0; i < bytes; ++i) out[o + i] = w[i];
        o += bytes;
        ssz[st] = bytes;
    }
    lit_header(out, four, nl, o - hs);
    if (four)
        for (uint32_t k = 0; k < 3; ++k) {
            out[hs + tsz + 2 * k] = (uint8_t)ssz[k];
            out[hs + tsz + 2 * k + 1] = (uint8_t)(ssz[k] >> 8);
        }
    return o;
}

// Scratch of the literals + sequences coding of one block (views of separate arrays, so
// a CPU build under AddressSanitizer sees each one's bounds): per position bests,
// sequences, literals, stream bytes, the content.  The device keeps one set per block of
// a batch in HBM (SeqArrays).
constexpr uint32_t kBodyBytes = 2 * kBlockMax + 64;  // see lz_content
struct SeqScratch {
    uint32_t* best;    // kBlockMax
    Seq* seq;          // kMaxSeq
    uint8_t* lit;      // kBlockMax
    uint8_t* streams;  // 4 * kStreamBytesMax
    uint8_t* body;     // kBodyBytes
    FseCT* fse;        // 3: the LL, ML, OF tables of the block
};
constexpr uint64_t kFseBytes = (3 * sizeof(FseCT) + 15) / 16 * 16;
// Bytes of the arrays of one block's SeqScratch.
constexpr uint64_t kSeqScratchBytes =
    4ull * kBlockMax + sizeof(Seq) * (uint64_t)kMaxSeq + kBlockMax + 4ull * kStreamBytesMax + kBodyBytes + kFseBytes;
// Block i's scratch inside one allocation of nb * kSeqScratchBytes (arrays grouped by
// kind, each 16-byte aligned).
__host__ __device__ __forceinline__ SeqScratch seq_scratch_at(uint8_t* base, uint64_t nb, uint64_t i) {
    SeqScratch sc;
    uint8_t* p = base;
    sc.best = (uint32_t*)p + i * kBlockMax;                      p += 4ull * kBlockMax * nb;
    sc.seq = (Seq*)p + i * kMaxSeq;                              p += sizeof(Seq) * (uint64_t)kMaxSeq * nb;
    sc.lit = p + i * kBlockMax;                                  p += (uint64_t)kBlockMax * nb;
    sc.streams = p + i * (4ull * kStreamBytesMax);               p += 4ull * kStreamBytesMax * nb;
    sc.body = p + i * (uint64_t)kBodyBytes;                       p += (uint64_t)kBodyBytes * nb;
    sc.fse = (FseCT*)(p + i * kFseBytes);
    return sc;
}

// The literals + sequences content of a block whose bests are in sc.best: greedy parse,
// literals section, sequences section into sc.body.  Returns its size, or 0 when the
// block has no match.  One thread (the device's thread 0) runs it.
// A sequence costs at most 57 bits (LL and ML codes + 16 extra bits each, OF code 8 + 8
// extra bits) and covers >= kMinMatch bytes, so the content is <= nl + 7 + 7.2 (n - nl) / 4
// < 2n + 64 = kBodyBytes.
__host__ __device__ inline uint32_t lz_content(const uint8_t* in, uint32_t n, const uint32_t* cand, const SeqScratch& sc,
                                               uint32_t* h, HufCode& c, HufWork& wk) {
    uint32_t nl = 0, cov = 0;
    const uint32_t ns = greedy_parse(in, n, sc.best, cand, sc.seq, sc.lit, &nl, &cov);
    if (!ns) return 0;
    uint32_t z = lit_section_seq(sc.lit, nl, sc.body, sc.streams, h, c, wk);
    z += seq_section(sc.seq, ns, sc.body + z, sc.fse[0], sc.fse[1], sc.fse[2]);
    return z;
}

// Whether a block tries literals + sequences: at least 1/32 of its positions have a
// candidate match (literal-heavy JSON has almost none and stays entropy-only).
__host__ __device__ __forceinline__ bool lz_worth(uint32_t nbest, uint32_t n) { return (uint64_t)nbest * 32 >= n; }

// The sequential form of one block (the host emulation of the device layer and the
// tests' reference encoder): writes the Compressed block content into slot (kBlockMax
// bytes) and returns its size with *type = 2, or returns n with *type = 0 (store Raw) /
// 1 with *type = 1 (RLE).  A block whose candidate matches cover >= 1/8 of it is coded
// as literals + sequences, any other as literals only.  k_zstd_block produces the same
// bytes with parallel histograms, candidate search and bit scatter.
__host__ inline uint32_t block_content_seq(const uint8_t* in, uint32_t n, uint8_t* slot, const SeqScratch& sc,
                                           uint32_t* type) {
    static thread_local uint32_t hh[256];
    static thread_local HufCode code;
    static thread_local HufWork work;
    uint32_t h[256] = {0};
    for (uint32_t i = 0; i < n; ++i) ++h[in[i]];
    uint32_t distinct = 0;
    for (uint32_t s = 0; s < 256; ++s) distinct += h[s] != 0;
    *type = 0;
    if (distinct == 1 && n > 1) { *type = 1; return 1; }
    if (n < 2) return n;
    // candidate distances and the greedy parse
    uint32_t gaps[256] = {0}, reps[256] = {0};
    for (uint32_t p = 0; p < n; ++p)
        if (in[p] == '{') gap_count(in, p, gaps);
    for (uint32_t p = 0; p < n; p += kRepStep)
        if (const uint32_t d = repeat_dist(in, n, p)) ++reps[d];
    uint32_t cand[kCands];
    const uint32_t nc = pick_cands(gaps, reps, cand);
    // entropy-only content (built in body: a Raw literals section is n + 3 bytes; only a
    // content smaller than the block goes to the slot)
    uint32_t size = lit_section_seq(in, n, sc.body, sc.streams, hh, code, work);
    sc.body[size++] = 0;  // Sequences_Section: Number_of_Sequences = 0
    if (size < n)
        for (uint32_t i = 0; i < size; ++i) slot[i] = sc.body[i];
    // literals + sequences when enough positions have a candidate match: the smaller
    // content wins (ties: entropy-only)
    uint32_t nbest = 0;
    for (uint32_t p = 0; p < n; ++p) sc.best[p] = best_at(in, n, p, cand, nc);
    {
        std::unique_ptr<uint32_t[]> tab(new uint32_t[1u << kHashBits]());
        for (uint32_t r0 = 0; r0 < n; r0 += kHashRound) {
            const uint32_t r1 = r0 + kHashRound < n ? r0 + kHashRound : n;
            for (uint32_t p = r0; p < r1; ++p) hash_look(in, n, p, tab.get(), sc.best);
            for (uint32_t p = r0; p < r1; ++p) hash_put(in, n, p, tab.get());
        }
    }
    for (uint32_t p = 0; p < n; ++p) nbest += sc.best[p] != 0;
    if (lz_worth(nbest, n)) {
        const uint32_t z = lz_content(in, n, cand, sc, hh, code, work);
        if (z && z < size) {
            if (z < n)
                for (uint32_t i = 0; i < z; ++i) slot[i] = sc.body[i];
            size = z;
        }
    }
    if (size >= n) return n;  // not smaller: Raw
    *type = 2;
    return size;
}

// Bytes of a frame for `len` bytes of content at worst (every block Raw).
__host__ __device__ __forceinline__ uint64_t frame_bound(uint64_t len) {
    const uint64_t nb = len ? (len + kBlockMax - 1) / kBlockMax : 1;
    return kFrameHeader + 3 * nb + len;
}

}  // namespace zstd
}  // namespace sydelta
