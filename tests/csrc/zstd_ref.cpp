// zstd_ref.cpp — TEST INFRASTRUCTURE: the sequential host form of the device zstd
// encoder (sy_amd/csrc/sydelta_zstd.hpp), built by tests/test_zstd.py.  Same block
// split, same code builder and header writers as k_zstd_block, streams written one bit
// after another; the device output must equal this byte for byte, and libzstd's decoder
// must give the input back.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "sydelta_zstd.hpp"

using namespace sydelta::zstd;

namespace {
// One literals stream: symbols in[first, first+count) written last to first, LSB-first,
// then the closing 1 bit (RFC 8878 4.2.2 / zstd's BIT_closeCStream).
void put_stream(const uint8_t* in, uint32_t count, const HufCode& c, std::vector<uint8_t>& out) {
    uint64_t acc = 0;
    uint32_t nb = 0;
    for (uint32_t i = count; i-- > 0;) {
        acc |= (uint64_t)c.code[in[i]] << nb;
        nb += c.len[in[i]];
        while (nb >= 8) {
            out.push_back((uint8_t)acc);
            acc >>= 8;
            nb -= 8;
        }
    }
    acc |= 1ull << nb;
    ++nb;
    while (nb > 0) {
        out.push_back((uint8_t)acc);
        acc >>= 8;
        nb = nb > 8 ? nb - 8 : 0;
    }
}

// Block content (type 2) or an empty vector when the block is stored Raw/RLE instead.
std::vector<uint8_t> compress_block(const uint8_t* in, uint32_t n, uint32_t* type) {
    uint32_t h[256] = {0};
    for (uint32_t i = 0; i < n; ++i) ++h[in[i]];
    uint32_t distinct = 0, hi = 0;
    for (uint32_t s = 0; s < 256; ++s)
        if (h[s]) { ++distinct; hi = s; }
    if (distinct == 1 && n > 1) { *type = 1; return {}; }
    if (distinct < 2 || hi >= kSymbols) { *type = 0; return {}; }
    HufCode c;
    HufWork wk;
    huf_build(h, c, wk);
    const bool four = n > kSingleStreamMax;
    uint8_t tree[1 + kSymbols / 2];
    const uint32_t tsz = huf_tree_desc(c, tree);
    std::vector<uint8_t> streams[4];
    const uint32_t ns = four ? 4 : 1;
    for (uint32_t s = 0; s < ns; ++s) {
        uint32_t f, cnt;
        stream_range(n, four, s, f, cnt);
        put_stream(in + f, cnt, c, streams[s]);
    }
    uint32_t comp = tsz + (four ? 6 : 0);
    for (uint32_t s = 0; s < ns; ++s) comp += (uint32_t)streams[s].size();
    const uint32_t total = (four ? 5 : 3) + comp + 1;
    if (total >= n || (!four && comp > kSingleStreamMax)) { *type = 0; return {}; }
    std::vector<uint8_t> out(8);
    out.resize(lit_header(out.data(), four, n, comp));
    out.insert(out.end(), tree, tree + tsz);
    if (four)
        for (uint32_t s = 0; s < 3; ++s) {
            out.push_back((uint8_t)streams[s].size());
            out.push_back((uint8_t)(streams[s].size() >> 8));
        }
    for (uint32_t s = 0; s < ns; ++s) out.insert(out.end(), streams[s].begin(), streams[s].end());
    out.push_back(0);  // Sequences_Section: Number_of_Sequences = 0
    *type = 2;
    return out;
}
}  // namespace

// The frame for in[0, len) into out (cap >= frame_bound(len)); returns its size or 0.
extern "C" size_t zstd_ref_compress(const uint8_t* in, size_t len, uint8_t* out, size_t cap) {
    if (cap < frame_bound(len)) return 0;
    frame_header(out, len);
    size_t o = kFrameHeader;
    const size_t nb = len ? (len + kBlockMax - 1) / kBlockMax : 1;
    for (size_t b = 0; b < nb; ++b) {
        const size_t p = b * kBlockMax;
        const uint32_t n = (uint32_t)(len - p < kBlockMax ? len - p : kBlockMax);
        const bool last = b + 1 == nb;
        uint32_t type = 0;
        std::vector<uint8_t> body = n ? compress_block(in + p, n, &type) : std::vector<uint8_t>();
        if (type == 2) {
            block_header(out + o, last, 2, (uint32_t)body.size());
            memcpy(out + o + 3, body.data(), body.size());
            o += 3 + body.size();
        } else if (type == 1) {
            block_header(out + o, last, 1, n);
            out[o + 3] = in[p];
            o += 4;
        } else {
            block_header(out + o, last, 0, n);
            if (n) memcpy(out + o + 3, in + p, n);
            o += 3 + n;
        }
    }
    return o;
}
