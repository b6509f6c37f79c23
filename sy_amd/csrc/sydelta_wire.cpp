// sydelta_wire.cpp — the delta path's wire formats.
//
// sy moves both sides of the delta as JSON (serde_json, compact):
//   * `sy-remote checksums` prints serde_json::to_string(&Vec<BlockChecksum>)
//     (src/bin/sy-remote.rs:146-147); the sender parses it (src/transport/ssh.rs:967-973);
//   * the sender serialises the Delta (ssh.rs:1003-1008), zstd-compresses it and the
//     receiver parses it back before apply_delta (sy-remote.rs:153-175).
// serde's derive output for these types is fixed by their declarations:
//   BlockChecksum {index, offset, size, weak, strong}            checksum.rs:10-21
//   Delta {ops, source_size, block_size}                          generator.rs:19-25
//   DeltaOp::Copy{offset, size} -> {"Copy":{"offset":O,"size":S}}
//   DeltaOp::Data(Vec<u8>)      -> {"Data":[b0,b1,...]}           generator.rs:10-15
// integers in decimal, no whitespace.  Host writers and parsers for both, and the
// device writer of a Delta whose literal bytes are in HBM (sydelta_kernels.hip K7:
// literal runs dominate the text, ~3.6 characters per byte).
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <memory>

#include "sydelta_host.hpp"
#include "sydelta_internal.hpp"

using namespace sydelta;

namespace {
// decimal text of 0..255 followed by ','; length in kByteLen
struct ByteText {
    char s[256][4];
    uint8_t len[256];
    ByteText() {
        for (int b = 0; b < 256; ++b) {
            len[b] = (uint8_t)snprintf(s[b], 4, "%d", b);
        }
    }
};
const ByteText kBytes;

inline char* put_u64(char* p, uint64_t v) {
    char t[20];
    int n = 0;
    do {
        t[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *p++ = t[--n];
    return p;
}
inline void put(std::string& o, const char* lit) { o.append(lit); }
inline void put_num(std::string& o, uint64_t v) {
    char t[24];
    o.append(t, put_u64(t, v) - t);
}

// Minimal strict-enough JSON reader for the two schemas above (whitespace allowed,
// unknown object keys skipped like serde's default, integers only).
struct Reader {
    const char* p;
    const char* e;
    std::string err;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool eat(char c) {
        ws();
        if (p < e && *p == c) { ++p; return true; }
        return false;
    }
    bool expect(char c) {
        if (eat(c)) return true;
        err = std::string("expected '") + c + "' at byte " + std::to_string(pos());
        return false;
    }
    size_t pos() const { return (size_t)(p - b0); }
    const char* b0;
    bool key(std::string& k) {
        ws();
        if (p >= e || *p != '"') { err = "expected a key at byte " + std::to_string(pos()); return false; }
        ++p;
        const char* s = p;
        while (p < e && *p != '"') {
            if (*p == '\\') { err = "escaped keys are not used by these types"; return false; }
            ++p;
        }
        if (p >= e) { err = "unterminated key"; return false; }
        k.assign(s, p - s);
        ++p;
        return expect(':');
    }
    bool u64(uint64_t& v) {
        ws();
        if (p >= e || *p < '0' || *p > '9') { err = "expected an unsigned integer at byte " + std::to_string(pos()); return false; }
        const char* q = p;
        v = 0;
        while (p < e && *p >= '0' && *p <= '9') {
            const uint64_t d = (uint64_t)(*p - '0');
            if (v > (UINT64_MAX - d) / 10) { err = "integer overflow at byte " + std::to_string(pos()); return false; }
            v = v * 10 + d;
            ++p;
        }
        if (p - q > 1 && *q == '0') {  // serde_json: "invalid number" (no leading zeros)
            err = "invalid number at byte " + std::to_string((size_t)(q - b0));
            return false;
        }
        return true;
    }
    // skip one JSON value (an unknown key's), validating it as serde_json's parser would
    // (its default recursion limit is 128 levels)
    bool skip(int depth = 0) {
        ws();
        if (p >= e) { err = "unexpected end"; return false; }
        if (depth > 128) { err = "recursion limit exceeded"; return false; }
        if (*p == '{' || *p == '[') {
            const bool obj = *p == '{';
            ++p;
            if (eat(obj ? '}' : ']')) return true;
            do {
                if (obj) {
                    ws();
                    if (p >= e || *p != '"' || !string()) { err = "expected a key at byte " + std::to_string(pos()); return false; }
                    if (!expect(':')) return false;
                }
                if (!skip(depth + 1)) return false;
            } while (eat(','));
            return expect(obj ? '}' : ']');
        }
        if (*p == '"') return string();
        for (const char* lit : {"true", "false", "null"}) {
            const size_t l = strlen(lit);
            if ((size_t)(e - p) >= l && memcmp(p, lit, l) == 0) { p += l; return true; }
        }
        // number: -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
        const char* s = p;
        auto digits = [&]() { const char* q = p; while (p < e && *p >= '0' && *p <= '9') ++p; return p > q; };
        if (p < e && *p == '-') ++p;
        if (p < e && *p == '0') ++p;
        else if (!digits()) { p = s; err = "expected a value at byte " + std::to_string(pos()); return false; }
        if (p < e && *p == '.') { ++p; if (!digits()) { err = "bad number at byte " + std::to_string(pos()); return false; } }
        if (p < e && (*p == 'e' || *p == 'E')) {
            ++p;
            if (p < e && (*p == '+' || *p == '-')) ++p;
            if (!digits()) { err = "bad number at byte " + std::to_string(pos()); return false; }
        }
        return true;
    }
    // a string at p (escapes checked for shape, control characters rejected)
    bool string() {
        ++p;
        while (p < e) {
            const unsigned char c = (unsigned char)*p;
            if (c == '"') { ++p; return true; }
            if (c < 0x20) { err = "control character in string at byte " + std::to_string(pos()); return false; }
            if (c == '\\') {
                if (++p >= e) break;
                if (*p == 'u') {
                    for (int i = 0; i < 4; ++i)
                        if (++p >= e || !isxdigit((unsigned char)*p)) { err = "bad \\u escape"; return false; }
                } else if (!*p || !strchr("\"\\/bfnrt", *p)) {
                    err = "bad escape at byte " + std::to_string(pos());
                    return false;
                }
            }
            ++p;
        }
        err = "unterminated string";
        return false;
    }
    // serde's derived Deserialize rejects a repeated field ("duplicate field `x`")
    bool once(unsigned& seen, unsigned bit, const char* name) {
        if (seen & bit) { err = std::string("duplicate field `") + name + "`"; return false; }
        seen |= bit;
        return true;
    }
};
struct DevBuf_wire {
    void* p = nullptr;
    hipStream_t s = nullptr;
    ~DevBuf_wire() {
        if (p) (void)hipFreeAsync(p, s);
    }
};
}  // namespace

// serde_json::to_string(&Vec<BlockChecksum>)  (sy-remote.rs:147, without println's '\n')
extern "C" uint64_t sydelta_checksums_to_json(const sydelta_block_checksum* sigs, uint64_t n, char* buf,
                                              uint64_t cap) {
    // the exact length first (digit counts), then the text straight into buf: one pass
    // each, no intermediate string
    auto digits = [](uint64_t v) {
        uint64_t d = 1;
        while (v >= 10) {
            v /= 10;
            ++d;
        }
        return d;
    };
    uint64_t total = 2;  // [ ]
    for (uint64_t i = 0; i < n; ++i)
        total += (i ? 1 : 0) + 46 + digits(sigs[i].index) + digits(sigs[i].offset) + digits(sigs[i].size) +
                 digits(sigs[i].weak) + digits(sigs[i].strong);
    if (!buf || cap < total) return total;
    char* p = buf;
    *p++ = '[';
    for (uint64_t i = 0; i < n; ++i) {
        if (i) *p++ = ',';
        memcpy(p, "{\"index\":", 9);
        p = put_u64(p + 9, sigs[i].index);
        memcpy(p, ",\"offset\":", 10);
        p = put_u64(p + 10, sigs[i].offset);
        memcpy(p, ",\"size\":", 8);
        p = put_u64(p + 8, sigs[i].size);
        memcpy(p, ",\"weak\":", 8);
        p = put_u64(p + 8, sigs[i].weak);
        memcpy(p, ",\"strong\":", 10);
        p = put_u64(p + 10, sigs[i].strong);
        *p++ = '}';
    }
    *p++ = ']';
    return total;
}

// serde_json::from_str::<Vec<BlockChecksum>>  (ssh.rs:967-973)
extern "C" int sydelta_checksums_from_json(const char* json, uint64_t len, sydelta_block_checksum** out,
                                           uint64_t* n_out) try {
    if (!json || !out || !n_out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    *n_out = 0;
    Reader r{json, json + len, {}, json};
    std::vector<sydelta_block_checksum> v;
    auto bad = [&]() { return fail(SYDELTA_E_INVAL, "checksum JSON: %s", r.err.c_str()); };
    if (!r.expect('[')) return bad();
    if (!r.eat(']')) {
        do {
            if (!r.expect('{')) return bad();
            sydelta_block_checksum c{};
            unsigned seen = 0;
            if (!r.eat('}')) {
                do {
                    std::string k;
                    if (!r.key(k)) return bad();
                    uint64_t x = 0;
                    if (k == "index" || k == "offset" || k == "size" || k == "weak" || k == "strong") {
                        const unsigned bit = k == "index" ? 1 : k == "offset" ? 2 : k == "size" ? 4 : k == "weak" ? 8 : 16;
                        if (!r.once(seen, bit, k.c_str())) return bad();
                        if (!r.u64(x)) return bad();
                        if (k == "index") c.index = x;
                        else if (k == "offset") c.offset = x;
                        else if (k == "size") c.size = x;
                        else if (k == "weak") {
                            if (x > 0xFFFFFFFFull) { r.err = "weak out of u32 range"; return bad(); }
                            c.weak = (uint32_t)x;
                        } else c.strong = x;
                    } else if (!r.skip()) {
                        return bad();
                    }
                } while (r.eat(','));
                if (!r.expect('}')) return bad();
            }
            if (seen != 31) { r.err = "missing field in checksum " + std::to_string(v.size()); return bad(); }
            v.push_back(c);
        } while (r.eat(','));
        if (!r.expect(']')) return bad();
    }
    r.ws();
    if (r.p != r.e) { r.err = "trailing characters"; return bad(); }
    if (!v.empty()) {
        *out = (sydelta_block_checksum*)malloc(v.size() * sizeof(sydelta_block_checksum));
        if (!*out) return fail(SYDELTA_E_OOM, "out of memory");
        memcpy(*out, v.data(), v.size() * sizeof(sydelta_block_checksum));
    }
    *n_out = v.size();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// serde_json::to_string(&Delta)  (ssh.rs:1003).  Literal bytes: the delta's own (host
// entry points), or `lit` indexed by the Data ops' source offsets (device deltas).
extern "C" int sydelta_delta_to_json(const sydelta_delta* d, const uint8_t* lit, uint64_t lit_len, char* buf,
                                     uint64_t cap, uint64_t* out_len) try {
    if (!d || !out_len) return fail(SYDELTA_E_INVAL, "NULL argument");
    const bool own = !lit;
    if (own && d->lit_off.size() != d->ops.size())
        return fail(SYDELTA_E_INVAL, "device delta: pass the source bytes as lit");
    uint64_t total = 0;
    std::string o;
    // size first (cheap), then write straight into buf when it fits
    auto op_len = [&](const sydelta_op& x, const uint8_t* bytes) -> uint64_t {
        char t[24];
        if (x.kind == SYDELTA_OP_COPY)
            return 28 + (put_u64(t, x.a) - t) + (put_u64(t, x.b) - t);  // {"Copy":{"offset":,"size":}}
        uint64_t L = 11 + (x.b ? x.b - 1 : 0);                           // {"Data":[]} + commas
        for (uint64_t i = 0; i < x.b; ++i) L += kBytes.len[bytes[i]];
        return L;
    };
    std::vector<const uint8_t*> src(d->ops.size(), nullptr);
    for (size_t i = 0; i < d->ops.size(); ++i) {
        const sydelta_op& x = d->ops[i];
        if (x.kind == SYDELTA_OP_DATA) {
            if (own) {
                src[i] = d->lit.data() + d->lit_off[i];
            } else {
                if (x.a > lit_len || x.b > lit_len - x.a)
                    return fail(SYDELTA_E_INVAL, "op %zu: Data outside the literal buffer", i);
                src[i] = lit + x.a;
            }
        }
    }
    char t[24];
    total = 8;  // {"ops":[
    for (size_t i = 0; i < d->ops.size(); ++i) total += op_len(d->ops[i], src[i]) + (i ? 1 : 0);
    total += 16 + (put_u64(t, d->source_size) - t) + 14 + (put_u64(t, d->block_size) - t) + 1;
    *out_len = total;
    if (!buf || cap < total) return SYDELTA_OK;
    char* p = buf;
    auto lit_s = [&](const char* s) { const size_t l = strlen(s); memcpy(p, s, l); p += l; };
    lit_s("{\"ops\":[");
    for (size_t i = 0; i < d->ops.size(); ++i) {
        const sydelta_op& x = d->ops[i];
        if (i) *p++ = ',';
        if (x.kind == SYDELTA_OP_COPY) {
            lit_s("{\"Copy\":{\"offset\":");
            p = put_u64(p, x.a);
            lit_s(",\"size\":");
            p = put_u64(p, x.b);
            lit_s("}}");
        } else {
            lit_s("{\"Data\":[");
            const uint8_t* b = src[i];
            for (uint64_t k = 0; k < x.b; ++k) {
                if (k) *p++ = ',';
                memcpy(p, kBytes.s[b[k]], 4);  // 4 bytes available: the text is followed by more text or "]}"
                p += kBytes.len[b[k]];
            }
            lit_s("]}");
        }
    }
    lit_s("],\"source_size\":");
    p = put_u64(p, d->source_size);
    lit_s(",\"block_size\":");
    p = put_u64(p, d->block_size);
    *p++ = '}';
    return (uint64_t)(p - buf) == total ? SYDELTA_OK : fail(SYDELTA_E_KERNEL, "delta JSON length mismatch");
} catch (...) {
    return sydelta::host_exception();
}

// serde_json::from_str::<Delta>  (sy-remote.rs:175): a host delta with its literal bytes,
// ready for sydelta_apply_delta.
extern "C" int sydelta_delta_from_json(const char* json, uint64_t len, sydelta_delta** out) try {
    if (!json || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    Reader r{json, json + len, {}, json};
    std::unique_ptr<sydelta_delta> d(new sydelta_delta());
    auto bad = [&]() { return fail(SYDELTA_E_INVAL, "delta JSON: %s", r.err.c_str()); };
    unsigned seen = 0;
    if (!r.expect('{')) return bad();
    if (!r.eat('}')) {
        do {
            std::string k;
            if (!r.key(k)) return bad();
            if (k == "ops") {
                if (!r.once(seen, 1, "ops")) return bad();
                if (!r.expect('[')) return bad();
                if (!r.eat(']')) {
                    do {
                        if (!r.expect('{')) return bad();
                        std::string tag;
                        if (!r.key(tag)) return bad();
                        if (tag == "Copy") {
                            uint64_t off = 0, size = 0;
                            unsigned f = 0;
                            if (!r.expect('{')) return bad();
                            if (!r.eat('}')) {
                                do {
                                    std::string ck;
                                    if (!r.key(ck)) return bad();
                                    if (ck == "offset") { if (!r.once(f, 1, "offset") || !r.u64(off)) return bad(); }
                                    else if (ck == "size") { if (!r.once(f, 2, "size") || !r.u64(size)) return bad(); }
                                    else if (!r.skip()) return bad();
                                } while (r.eat(','));
                                if (!r.expect('}')) return bad();
                            }
                            if (f != 3) { r.err = "Copy needs offset and size"; return bad(); }
                            d->ops.push_back({SYDELTA_OP_COPY, 0, off, size});
                            d->lit_off.push_back(UINT64_MAX);
                        } else if (tag == "Data") {
                            const uint64_t start = d->lit.size();
                            if (!r.expect('[')) return bad();
                            if (!r.eat(']')) {
                                do {
                                    uint64_t b = 0;
                                    if (!r.u64(b)) return bad();
                                    if (b > 255) { r.err = "Data byte out of range"; return bad(); }
                                    d->lit.push_back((uint8_t)b);
                                } while (r.eat(','));
                                if (!r.expect(']')) return bad();
                            }
                            d->ops.push_back({SYDELTA_OP_DATA, 0, start, d->lit.size() - start});
                            d->lit_off.push_back(start);
                        } else {
                            r.err = "unknown DeltaOp variant " + tag;
                            return bad();
                        }
                        if (!r.expect('}')) return bad();
                    } while (r.eat(','));
                    if (!r.expect(']')) return bad();
                }
            } else if (k == "source_size") {
                if (!r.once(seen, 2, "source_size") || !r.u64(d->source_size)) return bad();
            } else if (k == "block_size") {
                if (!r.once(seen, 4, "block_size") || !r.u64(d->block_size)) return bad();
            } else if (!r.skip()) {
                return bad();
            }
        } while (r.eat(','));
        if (!r.expect('}')) return bad();
    }
    r.ws();
    if (r.p != r.e) { r.err = "trailing characters"; return bad(); }
    if (seen != 7) { r.err = "missing field (ops, source_size, block_size)"; return bad(); }
    finish_stats(d.get());
    *out = d.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// serde_json::to_string(&Delta) on the device (K7): the literal runs (3.6 characters per
// byte on average) are formatted in HBM; the op table goes up once, pinned.
extern "C" int sydelta_delta_to_json_device(const sydelta_delta* d, const uint8_t* d_lit, uint64_t lit_len,
                                            uint8_t* d_out, uint64_t out_cap, uint64_t* out_len, void* stream) try {
    if (!d || !out_len) return fail(SYDELTA_E_INVAL, "NULL argument");
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    struct Pinned {
        JsonPiece* p = nullptr;
        size_t cap = 0;
        ~Pinned() { if (p) (void)hipHostFree(p); }
    };
    static thread_local Pinned pin;
    size_t need = 0;
    for (const sydelta_op& o : d->ops) need += o.kind == SYDELTA_OP_COPY ? 1 : std::max<uint64_t>(1, (o.b + kJsonChunk - 1) / kJsonChunk);
    if (need > pin.cap) {
        if (pin.p) { (void)hipHostFree(pin.p); pin.p = nullptr; pin.cap = 0; }
        const size_t cap = std::max<size_t>(need, 1024) * 5 / 4;
        HIP_TRY(hipHostMalloc((void**)&pin.p, cap * sizeof(JsonPiece), hipHostMallocDefault));
        pin.cap = cap;
    }
    size_t np = 0;
    for (size_t i = 0; i < d->ops.size(); ++i) {
        const sydelta_op& o = d->ops[i];
        const uint32_t sep = i ? kJsonSep : 0u;
        if (o.kind == SYDELTA_OP_COPY) {
            pin.p[np++] = {0, o.a, o.b, 0, sep};
            continue;
        }
        if (o.a > lit_len || o.b > lit_len - o.a)
            return fail(SYDELTA_E_INVAL, "op %zu: Data outside the literal buffer", i);
        if (o.b && !d_lit) return fail(SYDELTA_E_INVAL, "NULL literal buffer");
        const uint64_t nch = std::max<uint64_t>(1, (o.b + kJsonChunk - 1) / kJsonChunk);
        for (uint64_t c = 0; c < nch; ++c) {
            uint32_t fl = kJsonData;
            if (c == 0) fl |= kJsonFirst | sep;
            if (c + 1 == nch) fl |= kJsonLast;
            const uint64_t off = c * kJsonChunk;
            pin.p[np++] = {o.a + off, 0, 0, (uint32_t)std::min<uint64_t>(kJsonChunk, o.b - off), fl};
        }
    }
    char tail[96];
    char* t = tail;
    t += sprintf(t, "],\"source_size\":%llu,\"block_size\":%llu}", (unsigned long long)d->source_size,
                 (unsigned long long)d->block_size);
    const uint64_t tail_len = (uint64_t)(t - tail);
    static const char kHead[] = "{\"ops\":[";
    uint64_t body = 0;
    CallProf cp;
    DevBuf_wire buf;
    if (np) {
        const size_t pb = (np * sizeof(JsonPiece) + 255) & ~(size_t)255;
        const size_t lb = (np * 8 + 255) & ~(size_t)255;
        HIP_TRY(dev_malloc_async(&buf.p, pb + lb + np * 8, s));
        buf.s = s;
        JsonPiece* d_pieces = (JsonPiece*)buf.p;
        uint64_t* d_len = (uint64_t*)((uint8_t*)buf.p + pb);
        uint64_t* d_off = (uint64_t*)((uint8_t*)buf.p + pb + lb);
        HIP_TRY(hipMemcpyAsync(d_pieces, pin.p, np * sizeof(JsonPiece), hipMemcpyHostToDevice, s));
        HIP_TRY(launch_json_len(d_pieces, np, d_lit, d_len, s, cp.get()));
        HIP_TRY(launch_exclusive_sum_u64(d_len, d_off, np, s));
        uint64_t last_off = 0, last_len = 0;
        HIP_TRY(hipMemcpyAsync(&last_off, d_off + np - 1, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&last_len, d_len + np - 1, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        body = last_off + last_len;
        // the text of every op is bounded from both sides by its byte count; a body
        // outside the bounds means a sizing fault: never write with it
        uint64_t lo = 0, hi = 0;
        for (size_t i = 0; i < d->ops.size(); ++i) {
            const sydelta_op& o = d->ops[i];
            const uint64_t sep = i ? 1 : 0;
            if (o.kind == SYDELTA_OP_COPY) { lo += sep + 30; hi += sep + 28 + 40; }
            else { lo += sep + 11 + (o.b ? 2 * o.b - 1 : 0); hi += sep + 11 + (o.b ? 4 * o.b - 1 : 0); }
        }
        if (body < lo || body > hi)
            return fail(SYDELTA_E_KERNEL, "delta JSON sizing out of bounds (%llu not in [%llu, %llu])",
                        (unsigned long long)body, (unsigned long long)lo, (unsigned long long)hi);
        *out_len = 8 + body + tail_len;
        if (d_out && out_cap >= *out_len)
            HIP_TRY(launch_json_write(d_pieces, np, d_lit, d_off, 8, d_out, s, cp.get()));
    }
    *out_len = 8 + body + tail_len;
    if (d_out && out_cap >= *out_len) {
        HIP_TRY(hipMemcpyAsync(d_out, kHead, 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_out + 8 + body, tail, tail_len, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipStreamSynchronize(s));  // pinned piece table and host strings are reused / go away
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// ---------------------------------------------------------------------------
// serde_json::to_string(&Vec<BlockChecksum>) of a signature in HBM (sy-remote.rs:146-147;
// sydelta_sigjson.hpp, K7s): tile lengths on the device, their exclusive scan, the total
// checked against the bounds the implied fields give, then the text.
// ---------------------------------------------------------------------------
extern "C" int sydelta_checksums_to_json_device(const uint32_t* d_weak, const uint64_t* d_strong, uint64_t n,
                                                uint64_t block_size, uint64_t last_size, uint8_t* d_out,
                                                uint64_t out_cap, uint64_t* out_len, void* stream) try {
    if (!out_len) return fail(SYDELTA_E_INVAL, "NULL argument");
    if (n && (!d_weak || !d_strong)) return fail(SYDELTA_E_INVAL, "NULL signature arrays");
    if (n && (block_size == 0 || block_size > (1ull << 32) || last_size == 0 || last_size > block_size))
        return fail(SYDELTA_E_INVAL, "block_size %llu / last_size %llu out of range", (unsigned long long)block_size,
                    (unsigned long long)last_size);
    if (n && n - 1 > (UINT64_MAX - last_size) / block_size)
        return fail(SYDELTA_E_INVAL, "offsets of %llu blocks overflow", (unsigned long long)n);
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    uint64_t lo = 0, hi = 0;
    sigjson::text_bounds(n, block_size, last_size, lo, hi);
    if (n == 0) {
        *out_len = 2;
        if (d_out && out_cap >= 2) {
            HIP_TRY(hipMemcpyAsync(d_out, "[]", 2, hipMemcpyHostToDevice, s));
            HIP_TRY(hipStreamSynchronize(s));
        }
        return SYDELTA_OK;
    }
    const sigjson::SigArgs a{d_weak, d_strong, n, block_size, last_size};
    const uint64_t nt = (n + sigjson::kTile - 1) / sigjson::kTile;
    CallProf cp;
    DevBuf_wire buf;
    HIP_TRY(dev_malloc_async(&buf.p, 2 * nt * 8, s));
    buf.s = s;
    uint64_t* d_tlen = (uint64_t*)buf.p;
    uint64_t* d_toff = d_tlen + nt;
    HIP_TRY(launch_sigjson_len(a, d_tlen, s, cp.get()));
    HIP_TRY(launch_exclusive_sum_u64(d_tlen, d_toff, nt, s));
    uint64_t last_off = 0, last_len = 0;
    HIP_TRY(hipMemcpyAsync(&last_off, d_toff + nt - 1, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&last_len, d_tlen + nt - 1, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t total = last_off + last_len;
    // a total outside the bounds means a sizing fault: never write with it
    if (total < lo || total > hi)
        return fail(SYDELTA_E_KERNEL, "signature JSON sizing out of bounds (%llu not in [%llu, %llu])",
                    (unsigned long long)total, (unsigned long long)lo, (unsigned long long)hi);
    *out_len = total;
    if (d_out && out_cap >= total) {
        HIP_TRY(launch_sigjson_write(a, d_toff, d_out, s, cp.get()));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// serde_json::from_str::<Vec<BlockChecksum>> (ssh.rs:967-973) of a text in HBM that is
// exactly the compact form sy-remote prints (sydelta_sigjson.hpp, K7p): '{' per 64-byte
// chunk, their exclusive scan (the ranks), then every entry parsed and its surroundings
// checked; the first position that breaks the form is reported and the caller parses
// the text with sydelta_checksums_from_json instead.
extern "C" int sydelta_checksums_from_json_device(const uint8_t* d_text, uint64_t len, sydelta_block_checksum* d_out,
                                                  uint64_t cap, uint64_t* n_out, void* stream) try {
    if (!n_out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *n_out = 0;
    if (len < 2 || !d_text) return fail(SYDELTA_E_INVAL, "checksum JSON: not serde's compact form at byte 0");
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    const uint64_t nc = (len + sigjson::kParseChunk - 1) / sigjson::kParseChunk;
    CallProf cp;
    DevBuf_wire buf;
    HIP_TRY(dev_malloc_async(&buf.p, 2 * nc * 8 + 8, s));
    buf.s = s;
    uint64_t* d_cnt = (uint64_t*)buf.p;
    uint64_t* d_rank = d_cnt + nc;
    unsigned long long* d_bad = (unsigned long long*)(d_rank + nc);
    HIP_TRY(hipMemsetAsync(d_bad, 0xFF, 8, s));
    HIP_TRY(launch_sigparse_count(d_text, len, d_cnt, s, cp.get()));
    HIP_TRY(launch_exclusive_sum_u64(d_cnt, d_rank, nc, s));
    HIP_TRY(launch_sigparse(d_text, len, d_rank, d_out, d_out ? cap : 0, d_bad, s, cp.get()));
    uint64_t tail[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyAsync(&tail[0], d_rank + nc - 1, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&tail[1], d_cnt + nc - 1, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&tail[2], d_bad, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (tail[2] != UINT64_MAX)
        return fail(SYDELTA_E_INVAL, "checksum JSON: not serde's compact form at byte %llu",
                    (unsigned long long)tail[2]);
    *n_out = tail[0] + tail[1];
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// serde_json::from_str::<Delta> (sy-remote.rs:175) of a text in HBM in the compact form
// the sender writes (sydelta_dparse.hpp, K7d).  The host checks the head and parses the
// tail (`],"source_size":N,"block_size":B}`) from two small copies; the device ranks and
// parses the ops and literal bytes between them.  Data ops of the result index d_lit
// (op.a = offset of its first literal byte), as sydelta_apply_delta_device reads them.
namespace {
// A u64 in serde's compact spelling at t[p, e): digits, no leading zero; returns the
// digits consumed or 0.
size_t host_dec(const char* t, size_t p, size_t e, uint64_t& v) {
    uint64_t x = 0;
    size_t k = 0;
    while (p + k < e && t[p + k] >= '0' && t[p + k] <= '9') {
        const uint64_t d = (uint64_t)(t[p + k] - '0');
        if (x > (UINT64_MAX - d) / 10) return 0;
        x = x * 10 + d;
        ++k;
    }
    if (!k || (k > 1 && t[p] == '0')) return 0;
    v = x;
    return k;
}
}  // namespace

extern "C" int sydelta_delta_from_json_device(const uint8_t* d_text, uint64_t len, uint8_t* d_lit, uint64_t lit_cap,
                                              uint64_t* lit_len, sydelta_delta** out, void* stream) try {
    if (!lit_len) return fail(SYDELTA_E_INVAL, "NULL argument");
    *lit_len = 0;
    if (out) *out = nullptr;
    auto bad_at = [](uint64_t p) {
        return fail(SYDELTA_E_INVAL, "Delta JSON: not serde's compact form at byte %llu", (unsigned long long)p);
    };
    static const char kTailKey[] = "],\"source_size\":";
    // the shortest text: {"ops":[],"source_size":0,"block_size":0}
    if (!d_text || len < dparse::kHead + (sizeof kTailKey - 1) + 17) return bad_at(0);
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    // head and tail (the tail is < 80 bytes: two u64 and the keys)
    char head[dparse::kHead], tail[96];
    const uint64_t tl = std::min<uint64_t>(len - dparse::kHead, sizeof tail);
    HIP_TRY(hipMemcpyAsync(head, d_text, dparse::kHead, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(tail, d_text + len - tl, tl, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (memcmp(head, "{\"ops\":[", dparse::kHead) != 0) return bad_at(0);
    size_t at = SIZE_MAX;  // the last "],\"source_size\":" in the tail
    for (size_t i = 0; i + sizeof kTailKey - 1 <= tl; ++i)
        if (memcmp(tail + i, kTailKey, sizeof kTailKey - 1) == 0) at = i;
    if (at == SIZE_MAX) return bad_at(len - tl);
    uint64_t src_size = 0, blk = 0;
    size_t q = at + sizeof kTailKey - 1, k;
    static const char kBs[] = ",\"block_size\":";
    if (!(k = host_dec(tail, q, tl, src_size))) return bad_at(len - tl + q);
    q += k;
    if (tl - q < sizeof kBs - 1 || memcmp(tail + q, kBs, sizeof kBs - 1) != 0) return bad_at(len - tl + q);
    q += sizeof kBs - 1;
    if (!(k = host_dec(tail, q, tl, blk))) return bad_at(len - tl + q);
    q += k;
    if (!(q + 1 == tl && tail[q] == '}')) return bad_at(len - tl + q);
    const uint64_t E = len - tl + at;  // the ops array's ']'
    if (E < dparse::kHead) return bad_at(E);
    dparse::DArgs a{d_text, E, (E - dparse::kHead + dparse::kChunk - 1) / dparse::kChunk};
    uint64_t nops = 0, nlit = 0;
    CallProf cp;
    DevBuf_wire buf;
    const uint64_t nc = a.nc;
    HIP_TRY(dev_malloc_async(&buf.p, (4 * (nc + 1) + 1) * 8, s));
    buf.s = s;
    uint64_t* d_ocnt = (uint64_t*)buf.p;
    uint64_t* d_lcnt = d_ocnt + nc + 1;
    uint64_t* d_orank = d_lcnt + nc + 1;
    uint64_t* d_lrank = d_orank + nc + 1;
    unsigned long long* d_bad = (unsigned long long*)(d_lrank + nc + 1);
    HIP_TRY(hipMemsetAsync(d_ocnt, 0, 2 * (nc + 1) * 8, s));
    HIP_TRY(hipMemsetAsync(d_bad, 0xFF, 8, s));
    if (nc) {
        HIP_TRY(launch_dparse_count(a, d_ocnt, d_lcnt, s, cp.get()));
        HIP_TRY(launch_exclusive_sum_u64(d_ocnt, d_orank, nc + 1, s));  // [nc]: the totals
        HIP_TRY(launch_exclusive_sum_u64(d_lcnt, d_lrank, nc + 1, s));
        HIP_TRY(hipMemcpyAsync(&nops, d_orank + nc, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&nlit, d_lrank + nc, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    if (nc && nops == 0) return bad_at(dparse::kHead);  // a non-empty ops region starts with an op
    *lit_len = nlit;
    if (d_lit && lit_cap < nlit)
        return fail(SYDELTA_E_INVAL, "literal buffer holds %llu bytes, the delta has %llu",
                    (unsigned long long)lit_cap, (unsigned long long)nlit);
    std::unique_ptr<sydelta_delta> d(new sydelta_delta());
    d->source_size = src_size;
    d->block_size = blk;
    if (nops) {
        DevBuf_wire ob;
        HIP_TRY(dev_malloc_async(&ob.p, nops * (8 + sizeof(sydelta_op)), s));
        ob.s = s;
        uint64_t* d_pos = (uint64_t*)ob.p;
        sydelta_op* d_ops = (sydelta_op*)(d_pos + nops);
        HIP_TRY(launch_dparse_place(a, d_orank, d_pos, s, cp.get()));
        HIP_TRY(launch_dparse(a, d_orank, d_lrank, d_pos, nops, d_ops, d_lit, d_bad, s, cp.get()));
        uint64_t b = 0;
        HIP_TRY(hipMemcpyAsync(&b, d_bad, 8, hipMemcpyDeviceToHost, s));
        if (out) {
            d->ops.resize(nops);
            HIP_TRY(hipMemcpyAsync(d->ops.data(), d_ops, nops * sizeof(sydelta_op), hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(hipStreamSynchronize(s));
        if (b != UINT64_MAX) return bad_at(b);
    }
    for (const sydelta_op& o : d->ops) {
        if (o.kind == SYDELTA_OP_COPY) ++d->stats.copy_ops;
        else { ++d->stats.data_ops; d->stats.literal_bytes += o.b; }
    }
    if (out) *out = d.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// ---------------------------------------------------------------------------
// zstd frame of a text in HBM (ssh.rs:1009-1017: compress(delta_json, Compression::Zstd);
// sydelta_zstd.hpp).  The text goes through in batches of 4096 blocks (512 MiB): block
// contents into per-block slots (k_zstd_block), their placement (an exclusive scan of
// 3 + content), then the frame (k_zstd_frame); scratch is one batch of slots.
// ---------------------------------------------------------------------------
extern "C" uint64_t sydelta_zstd_bound(uint64_t len) { return zstd::frame_bound(len); }

extern "C" int sydelta_zstd_compress_device(int device, const uint8_t* d_in, uint64_t len, uint8_t* d_out,
                                            uint64_t out_cap, uint64_t* out_len, void* stream) try {
    if (!out_len) return fail(SYDELTA_E_INVAL, "NULL argument");
    if (len && !d_in) return fail(SYDELTA_E_INVAL, "NULL input");
    if (len && ((uintptr_t)d_in & 15)) return fail(SYDELTA_E_INVAL, "input must be 16-byte aligned");
    if (!d_out || out_cap < zstd::frame_bound(len))
        return fail(SYDELTA_E_INVAL, "output holds %llu bytes, a frame of %llu bytes needs up to %llu",
                    (unsigned long long)out_cap, (unsigned long long)len,
                    (unsigned long long)zstd::frame_bound(len));
    SYDELTA_ENTER_DEVICE(device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    if (len == 0) {  // one empty Raw block, the last
        uint8_t f[zstd::kFrameHeader + 3];
        zstd::frame_header(f, 0);
        zstd::block_header(f + zstd::kFrameHeader, true, 0, 0);
        HIP_TRY(hipMemcpyAsync(d_out, f, sizeof f, hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));
        *out_len = sizeof f;
        return SYDELTA_OK;
    }
    const uint64_t nblocks = (len + zstd::kBlockMax - 1) / zstd::kBlockMax;
    // blocks per batch (512 MiB of text, ~6 GiB of scratch: 1.5 MiB a block): four rounds of the 1024 blocks
    // 256 CUs hold at once (four per CU), so the rounds' stragglers overlap; SYDELTA_ZSTD_BATCH overrides
    uint64_t kBatch = 4096;
    if (const char* e = getenv("SYDELTA_ZSTD_BATCH"))
        if (const uint64_t v = strtoull(e, nullptr, 10)) kBatch = std::min<uint64_t>(v, 1 << 20);
    auto al = [](uint64_t b) { return (b + 255) & ~(uint64_t)255; };
    uint64_t nb_max, o_lz, o_size, o_type, o_len, o_off, total;
    DevBuf_wire buf;
    for (;;) {  // a device short of memory gets smaller batches (down to 64 blocks)
        nb_max = std::min<uint64_t>(nblocks, kBatch);
        o_lz = al(nb_max * zstd::kBlockMax);
        o_size = o_lz + al(nb_max * zstd::kSeqScratchBytes);
        o_type = o_size + al(4 * nb_max);
        o_len = o_type + al(4 * nb_max);
        o_off = o_len + al(8 * nb_max);
        total = o_off + al(8 * nb_max);
        const hipError_t e = dev_malloc_async(&buf.p, total, s);
        if (e == hipSuccess) break;
        if (e != hipErrorOutOfMemory || kBatch <= 64) HIP_TRY(e);
        (void)hipGetLastError();
        kBatch /= 2;
    }
    buf.s = s;
    uint8_t* B = (uint8_t*)buf.p;
    uint8_t* d_lz = B + o_lz;
    uint32_t* d_size = (uint32_t*)(B + o_size);
    uint32_t* d_type = (uint32_t*)(B + o_type);
    uint64_t* d_len = (uint64_t*)(B + o_len);
    uint64_t* d_off = (uint64_t*)(B + o_off);
    CallProf cp;
    uint64_t pos = zstd::kFrameHeader;
    for (uint64_t b0 = 0; b0 < nblocks; b0 += kBatch) {
        const uint32_t nb = (uint32_t)std::min<uint64_t>(kBatch, nblocks - b0);
        HIP_TRY(launch_zstd_blocks(d_in, len, b0, nb, B, d_lz, d_size, d_type, d_len, s, cp.get()));
        HIP_TRY(launch_exclusive_sum_u64(d_len, d_off, nb, s));
        HIP_TRY(launch_zstd_frame(d_in, len, b0, nb, nblocks, B, d_size, d_type, d_off, pos, d_out, s, cp.get()));
        uint64_t last[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(&last[0], d_off + nb - 1, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&last[1], d_len + nb - 1, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        const uint64_t batch = last[0] + last[1];
        // every block is at most 3 + its own size (Raw), so the frame stays within the bound
        if (batch > 3ull * nb + std::min<uint64_t>(len - b0 * zstd::kBlockMax, (uint64_t)nb * zstd::kBlockMax))
            return fail(SYDELTA_E_KERNEL, "zstd: batch at block %llu larger than its bound",
                        (unsigned long long)b0);
        pos += batch;
    }
    *out_len = pos;
    if (getenv("SYDELTA_PHASE_TIMING")) {
        unsigned long long t[16];
        HIP_TRY(zstd_phase_ticks(t));
        fprintf(stderr, "zstd block phases (ms of block time, summed over blocks): histogram+code %.2f, entropy "
                "streams %.2f, candidate distances %.2f, candidate matches %.2f, hash rounds %.2f, lz content %.2f "
                "(walks %.2f, chain %.2f, gather %.2f, repeat flags %.2f, repeats %.2f, literals %.2f, sequences "
                "header %.2f, sequences bits %.2f), rest %.2f; %llu sequences\n",
                t[0] / 1e5, t[1] / 1e5, t[2] / 1e5, t[3] / 1e5, t[4] / 1e5, t[5] / 1e5, t[7] / 1e5, t[8] / 1e5,
                t[9] / 1e5, t[14] / 1e5, t[10] / 1e5, t[11] / 1e5, t[13] / 1e5, t[12] / 1e5, t[6] / 1e5, t[15]);
    }
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}
