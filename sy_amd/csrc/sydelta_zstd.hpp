// sydelta_zstd.hpp — zstd frames (RFC 8878) for the compressed Delta JSON that sy sends
// to the receiver (src/transport/ssh.rs:1009-1017: compress(delta_json, Compression::Zstd),
// src/compress/mod.rs:71-76: zstd::Encoder level 3; the receiver decompresses with any
// zstd decoder, sy-remote.rs:160-179).
//
// The encoder is entropy-only: each block of <= 128 KiB of text is one Compressed block
// whose literals are Huffman-coded (4 streams, or 1 below 1 KiB, the weights in direct
// representation) and which has no sequences; a block Huffman does not shrink is stored
// Raw, a block of one repeated byte RLE.  The JSON of a Delta is decimal byte lists and
// keys over ~20 symbols (~3.4 bits per character), so this keeps the frame format and its
// decoders while the work per block is a histogram, a <= 128-symbol code and one bit
// scatter.  The bytes differ from libzstd's level 3 (matches, other entropy tables): the
// contract is decode(frame) == text, checked against libzstd's decoder.
//
// The functions here are the pieces every block needs whoever runs them: the device
// kernel (sydelta_kernels.hip, k_zstd_block: one workgroup per block, parallel bit
// scatter) and the sequential host encoder of the tests (tests/csrc/zstd_ref.cpp) call
// the same code builder and header writers, so their outputs must be byte-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// The sequential form of one block (the host emulation of the device layer and the
// tests' reference encoder): writes the Compressed block content into slot (kBlockMax
// bytes) and returns its size with *type = 2, or returns n with *type = 0 (store Raw) /
// 1 with *type = 1 (RLE).  scratch holds 4 * kStreamBytesMax bytes.  k_zstd_block
// produces the same bytes with a parallel bit scatter.
__host__ inline uint32_t block_content_seq(const uint8_t* in, uint32_t n, uint8_t* slot, uint8_t* scratch,
                                           uint32_t* type) {
    uint32_t h[256] = {0};
    for (uint32_t i = 0; i < n; ++i) ++h[in[i]];
    uint32_t distinct = 0, hi = 0;
    for (uint32_t s = 0; s < 256; ++s)
        if (h[s]) { ++distinct; hi = s; }
    *type = 0;
    if (distinct == 1 && n > 1) { *type = 1; return 1; }
    if (distinct < 2 || hi >= kSymbols) return n;
    HufCode c;
    HufWork wk;
    huf_build(h, c, wk);
    const bool four = n > kSingleStreamMax;
    const uint32_t hs = four ? 5 : 3;
    const uint32_t tsz = huf_tree_desc(c, slot + hs);
    uint32_t o = hs + tsz + (four ? 6 : 0);
    uint32_t ssz[4] = {0, 0, 0, 0};
    for (uint32_t st = 0; st < (four ? 4u : 1u); ++st) {
        uint32_t f, cnt;
        stream_range(n, four, st, f, cnt);
        // symbols last to first, LSB-first, then the closing 1 bit (BIT_closeCStream)
        uint8_t* w = scratch + st * kStreamBytesMax;
        uint32_t bytes = 0, nb = 0;
        uint64_t acc = 0;
        for (uint32_t i = cnt; i-- > 0;) {
            acc |= (uint64_t)c.code[in[f + i]] << nb;
            nb += c.len[in[f + i]];
            while (nb >= 8) { w[bytes++] = (uint8_t)acc; acc >>= 8; nb -= 8; }
        }
        acc |= 1ull << nb;
        ++nb;
        while (nb > 0) { w[bytes++] = (uint8_t)acc; acc >>= 8; nb = nb > 8 ? nb - 8 : 0; }
        if (o + bytes + 1 >= n || (!four && o + bytes - hs > kSingleStreamMax)) return n;  // not smaller: Raw
        for (uint32_t i = 0; i < bytes; ++i) slot[o + i] = w[i];
        o += bytes;
        ssz[st] = bytes;
    }
    lit_header(slot, four, n, o - hs);
    if (four)
        for (uint32_t k = 0; k < 3; ++k) {
            slot[hs + tsz + 2 * k] = (uint8_t)ssz[k];
            slot[hs + tsz + 2 * k + 1] = (uint8_t)(ssz[k] >> 8);
        }
    slot[o] = 0;  // Sequences_Section: Number_of_Sequences = 0
    *type = 2;
    return o + 1;
}

// Bytes of a frame for `len` bytes of content at worst (every block Raw).
__host__ __device__ __forceinline__ uint64_t frame_bound(uint64_t len) {
    const uint64_t nb = len ? (len + kBlockMax - 1) / kBlockMax : 1;
    return kFrameHeader + 3 * nb + len;
}

}  // namespace zstd
}  // namespace sydelta
