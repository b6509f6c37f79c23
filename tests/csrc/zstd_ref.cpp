// zstd_ref.cpp — TEST INFRASTRUCTURE: the sequential host form of the device zstd
// encoder (sy_amd/csrc/sydelta_zstd.hpp: block_content_seq, the block code builder and
// header writers that k_zstd_block shares), built by tests/test_zstd.py.  The device
// output must equal this byte for byte, and libzstd's decoder must give the input back.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "sydelta_zstd.hpp"

using namespace sydelta::zstd;

// The frame for in[0, len) into out (cap >= frame_bound(len)); returns its size or 0.
extern "C" size_t zstd_ref_compress(const uint8_t* in, size_t len, uint8_t* out, size_t cap) {
    if (cap < frame_bound(len)) return 0;
    std::vector<uint8_t> slot(kBlockMax), lz(kSeqScratchBytes);
    const SeqScratch scratch = seq_scratch_at(lz.data(), 1, 0);
    frame_header(out, len);
    size_t o = kFrameHeader;
    const size_t nb = len ? (len + kBlockMax - 1) / kBlockMax : 1;
    for (size_t b = 0; b < nb; ++b) {
        const size_t p = b * kBlockMax;
        const uint32_t n = (uint32_t)(len - p < kBlockMax ? len - p : kBlockMax);
        uint32_t type = 0;
        const uint32_t size = n ? block_content_seq(in + p, n, slot.data(), scratch, &type) : 0;
        block_header(out + o, b + 1 == nb, type, type == 2 ? size : n);
        const uint8_t* src = type == 2 ? slot.data() : in + p;
        if (size) memcpy(out + o + 3, src, size);
        o += 3 + size;
    }
    return o;
}
