/*
 * sydelta.h — C ABI of the MI355X-native delta hot path (libsydelta.so).
 *
 * Drop-in boundary for nijaru/sy v0.0.43 `src/delta` (the re-exports at
 * src/delta/mod.rs:9-16 plus calculate_block_size at mod.rs:20-23).  Every
 * entry point names the reference interface it replaces; INTEGRATION.md shows
 * the Rust `extern "C"` block and the safe wrappers a maintainer adds to sy.
 *
 * Conventions
 *  - Plain pointers and sizes only; no torch / HIP types in signatures.  A
 *    `void *stream` is a hipStream_t (NULL = the library's per-thread stream, created
 *    blocking so it is ordered against work on the legacy default stream).
 *  - Return value: SYDELTA_OK (0) or a negative SYDELTA_E_* code; the message
 *    of the last failure on the calling thread is sydelta_last_error().  This
 *    mirrors the reference's io::Result: I/O failures -> SYDELTA_E_IO
 *    (File::open/read errors propagated by `?`, checksum.rs:50-59,
 *    generator.rs:83-84); no panics on data.
 *  - Re-entrant: callers are tokio spawn_blocking threads (ssh.rs:913), up to
 *    --parallel (default 10) at once (sync/mod.rs:673).  Device init is
 *    call_once per device; every call uses its own stream and buffers.
 *  - Devices: every entry point leaves the calling thread's current HIP device
 *    as it found it (hipGetDevice before == after), whichever devices it worked
 *    on (`device` arguments, an index's device, the path-level binding below,
 *    sydelta_trim's and sydelta_delta_multi_device's device switches), on success
 *    and on every error return.
 *  - Scratch kept between calls (per thread and device: scan / probe / walk
 *    buffers and pinned host buffers) is released when the thread exits and by
 *    sydelta_trim, which frees it for every thread not inside a call.
 *  - Data layout in HBM: byte buffers as given; signatures as SoA
 *    (weak u32[n], strong u64[n]).  Device buffers passed in must be readable
 *    up to the end of the 16-byte granule holding their last byte (true for
 *    hipMalloc and the torch caching allocator).
 *  - Semantics are bit-exact with the reference for block_size in
 *    [1, 131072] (the production domain, mod.rs:22).  Above 128 KiB the
 *    reference's streaming generator diverges from its own in-memory one
 *    (SURVEY.md App. A R10); the streaming entry rejects such sizes with
 *    SYDELTA_E_INVAL, the in-memory entry follows generate_delta.
 */
#ifndef SYDELTA_H
#define SYDELTA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYDELTA_ABI_VERSION 1

enum {
    SYDELTA_OK = 0,
    SYDELTA_E_NODEV = -1,  /* no usable gfx950 device / HIP runtime error at init */
    SYDELTA_E_OOM = -2,    /* device or host allocation failed */
    SYDELTA_E_INVAL = -3,  /* bad argument (block_size 0, NULL pointer, ...) */
    SYDELTA_E_KERNEL = -4, /* kernel launch / execution error */
    SYDELTA_E_IO = -5      /* file open/read/write error (path-level API) */
};

/* checksum.rs:9-21 `struct BlockChecksum {index, offset, size, weak, strong}` */
typedef struct sydelta_block_checksum {
    uint64_t index;
    uint64_t offset;
    uint64_t size;
    uint32_t weak;
    uint32_t reserved; /* zero */
    uint64_t strong;
} sydelta_block_checksum;

/* generator.rs:10-15 `enum DeltaOp { Copy{offset,size}, Data(Vec<u8>) }`
 *   kind = SYDELTA_OP_COPY: a = basis offset, b = size (from the matched checksum)
 *   kind = SYDELTA_OP_DATA: a = offset of the literal run in the source, b = length;
 *          the bytes are source[a .. a+b) (every reference literal run is a
 *          contiguous source slice: literal_buffer is flushed at each Copy). */
enum { SYDELTA_OP_COPY = 0, SYDELTA_OP_DATA = 1 };
typedef struct sydelta_op {
    uint32_t kind;
    uint32_t reserved;
    uint64_t a;
    uint64_t b;
} sydelta_op;

/* Observability counters (SURVEY.md §5 Metrics): per match call. */
typedef struct sydelta_match_stats {
    uint64_t positions;      /* full-window positions scanned (len - bs + 1) */
    uint64_t weak_hits;      /* positions whose weak hash has candidates (strong hashed) */
    uint64_t verified_hits;  /* positions whose (weak, strong) matched a block */
    uint64_t copy_ops;
    uint64_t data_ops;
    uint64_t literal_bytes;
} sydelta_match_stats;

typedef struct sydelta_index sydelta_index; /* device-resident probe table built from a signature */
typedef struct sydelta_delta sydelta_delta; /* result of a match: op list (host memory) */
typedef struct sydelta_delta_batch sydelta_delta_batch; /* one delta per file of a batched match */

int sydelta_abi_version(void);
const char *sydelta_last_error(void);
/* Number of visible HIP devices (0 without a GPU; never initialises a device). */
int sydelta_device_count(int *count);

/* Devices of the path-level entry points (sydelta_compute_checksums,
 * sydelta_generate_delta(_streaming), sydelta_estimate_change_ratio).  sy calls them from
 * up to --parallel (default 10) spawn_blocking threads at once (sync/mod.rs:672-697,
 * cli.rs:178-180, ssh.rs:913), and Rust makes no device current: each calling thread is
 * bound on its first path-level call to the allowed device with the fewest bound threads
 * (ties round-robin) and keeps it (its stream and buffers live there); a thread's exit
 * unbinds it.  The device-pointer entry points take their device explicitly. */
/* Restrict automatic binding to devices[0..n) (n = 0: every visible device); threads
 * already bound keep their device. */
int sydelta_set_devices(const int *devices, int n);
/* Bind the calling thread's path-level calls to `device`, or (-1) let its next call bind
 * it automatically. */
int sydelta_set_thread_device(int device);
/* The device the calling thread's path-level calls use (bound now if it was not). */
int sydelta_thread_device(int *device);
/* Release memory the library keeps between calls for reuse: index allocations held per
 * device (made on library streams), the recycled op arrays, and the scan / probe / walk
 * buffers (device and pinned host memory) of the calling thread and of every other thread
 * that is not inside a call (a thread inside a call keeps its own until it exits or a
 * later trim). */
void sydelta_trim(void);

/* mod.rs:20-23 `calculate_block_size(file_size) -> usize`: sqrt clamped to 512..=131072. */
uint64_t sydelta_calculate_block_size(uint64_t file_size);

/* ---------------------------------------------------------------------------
 * Device-resident core.  Buffers live in HBM; results are bit-exact with the
 * reference on the same bytes.
 * ------------------------------------------------------------------------- */

/* Signature of a device buffer: compute_checksums' per-block loop
 * (checksum.rs:46-76): ceil(len/bs) blocks, block i = [i*bs, min(len,(i+1)*bs)),
 * weak = Adler32::hash (rolling.rs:35-45), strong = XXH3-64 seed 0
 * (checksum.rs:65-67).  d_weak / d_strong are device arrays of ceil(len/bs). */
int sydelta_signature_device(int device, const uint8_t *d_buf, uint64_t len, uint64_t block_size,
                             uint32_t *d_weak, uint64_t *d_strong, void *stream);

/* Build the probe table for a basis signature: the candidate map
 * `HashMap<u32, Vec<&BlockChecksum>>` of generator.rs:75-81 (candidates in index
 * order).  weak/strong hold nblocks entries (device pointers if
 * arrays_on_device, else host).  Block i has offset i*block_size and size
 * block_size except the last, whose size is last_size (1..block_size).
 * Host arrays: the index is built when the call returns.  Device arrays: they are
 * copied in `stream`'s order (the caller may overwrite them after that point of the
 * stream) and the call returns without waiting; the table is built on a library
 * stream (one file; a batch: on `stream`) and every call that uses the index orders
 * its own stream after the build, so work the caller queues meanwhile (the source's
 * upload, its aligned probe) overlaps it. */
int sydelta_index_create(int device, const uint32_t *weak, const uint64_t *strong, uint64_t nblocks,
                         uint64_t block_size, uint64_t last_size, int arrays_on_device, void *stream,
                         sydelta_index **out);
/* The index's device memory is released in the order of the stream it was created on
 * (a caller stream must outlive the index; NULL: the creating thread's library stream,
 * which lives as long as the process). */
void sydelta_index_free(sydelta_index *idx);

/* Rolling match of a device-resident source against the index: the greedy
 * scan of generate_delta (generator.rs:242-379; equal to
 * generate_delta_streaming, :67-228, for block_size <= 128 KiB).  The op list
 * is returned in host memory.  len may be 0 (no ops). */
int sydelta_match_device(sydelta_index *idx, const uint8_t *d_src, uint64_t len, void *stream,
                         sydelta_delta **out);

uint64_t sydelta_delta_num_ops(const sydelta_delta *d);
const sydelta_op *sydelta_delta_ops(const sydelta_delta *d);
uint64_t sydelta_delta_source_size(const sydelta_delta *d); /* Delta::source_size (generator.rs:22) */
uint64_t sydelta_delta_block_size(const sydelta_delta *d);  /* Delta::block_size (generator.rs:24) */
/* Literal bytes of op i when the delta was produced from host data (buffer or
 * path entry points); NULL for Copy ops or device-only sources. */
const uint8_t *sydelta_delta_literal(const sydelta_delta *d, uint64_t op_index);
int sydelta_delta_stats(const sydelta_delta *d, sydelta_match_stats *out);
/* Delta::compression_ratio (generator.rs:30-55). */
double sydelta_delta_compression_ratio(const sydelta_delta *d);
void sydelta_delta_free(sydelta_delta *d);

/* ---------------------------------------------------------------------------
 * Host-buffer entry points (pinned staging + H2D inside).
 * ------------------------------------------------------------------------- */

/* compute_checksums on an in-memory file image (checksum.rs:31-80).
 * out must hold ceil(len/bs) entries; *n_out receives the count. */
int sydelta_compute_checksums_buf(int device, const uint8_t *buf, uint64_t len, uint64_t block_size,
                                  sydelta_block_checksum *out, uint64_t cap, uint64_t *n_out);
/* generate_delta on an in-memory source (generator.rs:242-379).  sigs as
 * produced by compute_checksums (index order, offset = index*block_size). */
int sydelta_generate_delta_buf(int device, const uint8_t *src, uint64_t len, const sydelta_block_checksum *sigs,
                               uint64_t nsigs, uint64_t block_size, sydelta_delta **out);

/* ---------------------------------------------------------------------------
 * Path-level mirror of src/delta's public API (file I/O on the host).
 * ------------------------------------------------------------------------- */

/* checksum.rs:31 `compute_checksums(path: &Path, block_size: usize) -> io::Result<Vec<BlockChecksum>>`.
 * *out is allocated by the library (free with sydelta_checksums_free); empty
 * file -> *n = 0 (checksum.rs:36-38). */
int sydelta_compute_checksums(const char *path, uint64_t block_size, sydelta_block_checksum **out, uint64_t *n);
void sydelta_checksums_free(sydelta_block_checksum *p);

/* generator.rs:67 `generate_delta_streaming(source_path, dest_checksums, block_size) -> io::Result<Delta>`. */
int sydelta_generate_delta_streaming(const char *source_path, const sydelta_block_checksum *sigs, uint64_t nsigs,
                                     uint64_t block_size, sydelta_delta **out);
/* generator.rs:242 `generate_delta(source_path, dest_checksums, block_size) -> io::Result<Delta>`. */
int sydelta_generate_delta(const char *source_path, const sydelta_block_checksum *sigs, uint64_t nsigs,
                           uint64_t block_size, sydelta_delta **out);

/* applier.rs:22 `apply_delta(old_file, delta, new_file) -> io::Result<DeltaStats>`
 * (receiver side; host file I/O, no device work).  The delta must carry its
 * literal bytes (produced by a host-data entry point).  DeltaStats fields:
 * applier.rs:9-13. */
typedef struct sydelta_apply_stats {
    uint64_t operations_count;
    uint64_t literal_bytes;
    uint64_t bytes_written;
} sydelta_apply_stats;
int sydelta_apply_delta(const char *old_file, const sydelta_delta *d, const char *new_file, sydelta_apply_stats *out);

/* applier.rs:22-56 `apply_delta` on device-resident bytes: d_out
 * receives the reconstructed file.  Copy ops read d_basis[offset, +size) (past the end:
 * SYDELTA_E_IO, as read_exact fails); Data ops of a device delta (sydelta_match_device)
 * read d_lit[op source offset, +len) -- the source the delta was generated from, or any
 * buffer laid out the same way.  out_cap must hold the reconstructed size. */
int sydelta_apply_delta_device(int device, const uint8_t *d_basis, uint64_t basis_len, const sydelta_delta *d,
                               const uint8_t *d_lit, uint64_t lit_len, uint8_t *d_out, uint64_t out_cap,
                               void *stream, sydelta_apply_stats *out);

/* rolling.rs:35-45 `Adler32::hash` (host utility for the re-exported Adler32 type). */
uint32_t sydelta_adler32_hash(const uint8_t *data, uint64_t len);

/* ---------------------------------------------------------------------------
 * Batched (many independent files, BASELINE config 4).  Segment table:
 * file f occupies d_buf[off[f] .. off[f]+len[f]); all files share block_size.
 * Signature output for file f starts at entry sig_off[f] (= sum of
 * ceil(len/bs) over earlier files).
 * ------------------------------------------------------------------------- */
int sydelta_signature_batch_device(int device, const uint8_t *d_buf, const uint64_t *off, const uint64_t *len,
                                   uint64_t nfiles, uint64_t block_size, uint32_t *d_weak, uint64_t *d_strong,
                                   void *stream);

/* Batched index: nfiles basis signatures concatenated in file order (as
 * sydelta_signature_batch_device writes them); file f has nblocks[f] blocks, the
 * last of size last_size[f] (ignored when nblocks[f] == 0).  nblocks/last_size are
 * host arrays; weak/strong are device arrays if arrays_on_device.  Each file gets
 * its own candidate map (generator.rs:75-81), as if sy called generate_delta once
 * per file. */
int sydelta_index_create_batch(int device, const uint32_t *weak, const uint64_t *strong, const uint64_t *nblocks,
                               const uint64_t *last_size, uint64_t nfiles, uint64_t block_size, int arrays_on_device,
                               void *stream, sydelta_index **out);
/* Batched rolling match: source f = d_buf[src_off[f] .. +src_len[f]) (16-byte
 * aligned) against basis f of idx, all files in one launch.  Result f is the
 * delta sy's generate_delta would return for that pair. */
int sydelta_match_batch_device(sydelta_index *idx, const uint8_t *d_buf, const uint64_t *src_off,
                               const uint64_t *src_len, uint64_t nfiles, void *stream, sydelta_delta_batch **out);
/* Signature + match of many independent (basis, source) pairs in one call: for each pair,
 * compute_checksums of the basis (checksum.rs:31-80) then generate_delta of the source against
 * it (generator.rs:242-379), as the three calls above would do.  The files are taken in two
 * groups whose signatures and walks overlap, and no index is built (each walk builds its
 * file's candidate map in on-chip memory).  Needs block_size % 64 == 0 in [256, 8192], bases
 * of at most 1024 blocks and 16-byte aligned files (else SYDELTA_E_INVAL: use the three
 * calls). */
int sydelta_delta_pairs_device(int device, const uint8_t *d_basis, const uint64_t *basis_off,
                               const uint64_t *basis_len, const uint8_t *d_src, const uint64_t *src_off,
                               const uint64_t *src_len, uint64_t nfiles, uint64_t block_size, void *stream,
                               sydelta_delta_batch **out);
uint64_t sydelta_delta_batch_count(const sydelta_delta_batch *b);
/* Borrowed pointer, valid until sydelta_delta_batch_free. */
const sydelta_delta *sydelta_delta_batch_get(const sydelta_delta_batch *b, uint64_t i);
/* Totals over the batch (weak_hits is only counted per batch). */
int sydelta_delta_batch_stats(const sydelta_delta_batch *b, sydelta_match_stats *out);
void sydelta_delta_batch_free(sydelta_delta_batch *b);

/* ---------------------------------------------------------------------------
 * Chunk-sharded match of ONE large file over several devices (BASELINE config 5,
 * SURVEY.md §8e).  Not a reference entry point: it splits generate_delta
 * (generator.rs:242-379) of one (source, signature) pair at block-aligned chunk
 * boundaries so each rank classifies its own chunk against the all-gathered
 * signature (file 0 of idx, global block indices).  The walks are then chained:
 * chunk 0 is walked from 0; chunk g from the exit of chunk g-1 (which may lie up to
 * block_size-1 bytes inside chunk g after a Copy); the per-chunk deltas joined with
 * sydelta_delta_append equal generate_delta's op list for the whole file.
 *
 * d_buf holds source bytes [buf_pos, buf_pos + buf_len) in device memory (16-byte
 * aligned; buf_pos a multiple of 16 and <= pos_begin rounded down to 16).  The chunk
 * classifies full-window positions [pos_begin, min(pos_end, file_len-block_size+1));
 * pos_begin is a multiple of block_size.  The buffer must reach byte
 * min(file_len, pos_end + block_size - 1), or file_len for the chunk holding the
 * file's last full window (pos_end >= file_len - block_size + 1), which also
 * applies the tail rule (generator.rs:156-184).  The buffer must stay valid until
 * sydelta_chunk_free: a walk that jumps into a block classified only by its aligned
 * window scans that block on demand.
 * ------------------------------------------------------------------------- */
typedef struct sydelta_chunk sydelta_chunk;
int sydelta_chunk_classify(sydelta_index *idx, const uint8_t *d_buf, uint64_t buf_pos, uint64_t buf_len,
                           uint64_t file_len, uint64_t pos_begin, uint64_t pos_end, void *stream,
                           sydelta_chunk **out);
/* Greedy walk from entry (>= pos_begin).  *out: the ops for [entry, *exit_pos); a
 * non-final chunk ends with its literal run up to its last position (continued by
 * the next chunk's leading Data op), a final chunk ends at file_len.
 * With the device walk (bs % 64 == 0, 256..8192; SYDELTA_CHUNK_WALK) classify launches
 * the probe and the walk from the chunk's segment starts and returns; walk waits for
 * them and walks again only the segments whose true entry differs.  sydelta_chunk_free
 * waits for work still running on a chunk that was never walked. */
int sydelta_chunk_walk(sydelta_chunk *c, uint64_t entry, uint64_t *exit_pos, sydelta_delta **out);
void sydelta_chunk_free(sydelta_chunk *c);
/* A delta holding a copy of n ops (e.g. one received from the sender, to apply on the
 * device); NULL if ops is NULL with n > 0 or an op's kind is neither SYDELTA_OP_COPY nor
 * SYDELTA_OP_DATA (sydelta_last_error says which). */
sydelta_delta *sydelta_delta_from_ops(const sydelta_op *ops, uint64_t n, uint64_t source_size, uint64_t block_size);
/* Empty delta (Delta { ops: [], source_size, block_size }) to append chunk deltas to. */
sydelta_delta *sydelta_delta_new(uint64_t source_size, uint64_t block_size);
/* dst.ops += src.ops, merging dst's trailing Data op with src's leading Data op when
 * they are contiguous (literal runs stay maximal, generator.rs:186-197). */
int sydelta_delta_append(sydelta_delta *dst, const sydelta_delta *src);

/* The same split inside one process (no reference counterpart; the in-process form of
 * bench.py's one-process-per-GPU C5): one file chunk-sharded over ndev devices.  Basis
 * chunk g = d_basis[g][0, basis_len[g]) on devices[g], every chunk but the last a whole
 * number of blocks; it is signed there, and each device pulls the other chunks' slices of
 * the signature SoA with peer copies (hipMemcpyPeerAsync, xGMI between MI355X devices of
 * a node) and builds the whole file's index.  Source chunk g classifies full-window
 * positions [src_pos[g], src_pos[g+1]) (the last: to the end) on devices[g] from d_src[g],
 * which holds source bytes [src_pos[g], src_pos[g] + src_buf_len[g]) as
 * sydelta_chunk_classify requires (src_pos[0] = 0, block-aligned starts; a chunk's buffer
 * reaches block_size - 1 bytes past its end).  The walks are chained inside the library;
 * *out equals generate_delta's op list for the whole file (generator.rs:242-379).  A
 * device may be listed more than once. */
int sydelta_delta_multi_device(const int *devices, int ndev, const uint8_t *const *d_basis, const uint64_t *basis_len,
                               const uint8_t *const *d_src, const uint64_t *src_pos, const uint64_t *src_buf_len,
                               uint64_t src_len, uint64_t block_size, sydelta_delta **out);

/* ---------------------------------------------------------------------------
 * Wire formats: serde_json's compact text of the types sy
 * moves between sender and receiver.
 * ------------------------------------------------------------------------- */
/* serde_json::to_string(&Vec<BlockChecksum>) (sy-remote.rs:146-147, println without
 * the newline).  Returns the text length; writes it when buf holds that many bytes. */
uint64_t sydelta_checksums_to_json(const sydelta_block_checksum *sigs, uint64_t n, char *buf, uint64_t cap);
/* serde_json::from_str::<Vec<BlockChecksum>> (ssh.rs:967-973).  *out is malloc'ed
 * (free with sydelta_checksums_free). */
int sydelta_checksums_from_json(const char *json, uint64_t len, sydelta_block_checksum **out, uint64_t *n);
/* serde_json::to_string(&Delta) (ssh.rs:1003).  Literal bytes: the delta's own when
 * lit is NULL (host entry points), else lit[op source offset, +len) (device deltas).
 * *out_len = text length; the text is written when buf holds it. */
int sydelta_delta_to_json(const sydelta_delta *d, const uint8_t *lit, uint64_t lit_len, char *buf, uint64_t cap,
                          uint64_t *out_len);
/* The same text produced on the device from literal bytes in HBM (d_lit indexed by the
 * Data ops' source offsets) into d_out; *out_len as above (computed on the device). */
int sydelta_delta_to_json_device(const sydelta_delta *d, const uint8_t *d_lit, uint64_t lit_len, uint8_t *d_out,
                                 uint64_t out_cap, uint64_t *out_len, void *stream);
/* serde_json::to_string(&Vec<BlockChecksum>) of a signature in HBM, written on the device:
 * the line `sy-remote checksums` prints (sy-remote.rs:146-147) and ssh.rs:967-973 parses,
 * for the SoA sydelta_signature_device writes (n blocks in index order, block i at offset
 * i * block_size, size block_size except the last, last_size in (0, block_size]).  Same
 * text as sydelta_checksums_to_json.  *out_len = text length (computed on the device);
 * the text is written when d_out holds it (d_out NULL: length only). */
int sydelta_checksums_to_json_device(const uint32_t *d_weak, const uint64_t *d_strong, uint64_t n,
                                     uint64_t block_size, uint64_t last_size, uint8_t *d_out, uint64_t out_cap,
                                     uint64_t *out_len, void *stream);
/* serde_json::from_str::<Vec<BlockChecksum>> (ssh.rs:967-973) on the device, for text in
 * HBM that is exactly the compact form sy-remote prints (serde_json::to_string: fields in
 * checksum.rs's order, no whitespace); d_out (device, cap entries; NULL: validate and
 * count only) receives the entries in order (those past cap are not written), *n_out
 * their count.  Any other spelling --
 * including ones serde accepts, such as whitespace or other key orders -- returns
 * SYDELTA_E_INVAL naming the first byte that breaks the form: parse those with
 * sydelta_checksums_from_json. */
int sydelta_checksums_from_json_device(const uint8_t *d_text, uint64_t len, sydelta_block_checksum *d_out,
                                       uint64_t cap, uint64_t *n_out, void *stream);
/* serde_json::from_str::<Delta> (sy-remote.rs:175) on the device, for text in HBM in the
 * compact form the sender writes (serde_json::to_string, ssh.rs:1003).  *lit_len = the
 * delta's literal bytes; with d_lit (device, lit_cap >= *lit_len) they are written there
 * in op order, and *out (when not NULL) receives the ops, source_size and block_size,
 * its Data ops indexing d_lit (op.a = offset of the first byte) as
 * sydelta_apply_delta_device reads them.  Any other spelling returns SYDELTA_E_INVAL
 * naming the first byte that breaks the form: parse those with sydelta_delta_from_json. */
int sydelta_delta_from_json_device(const uint8_t *d_text, uint64_t len, uint8_t *d_lit, uint64_t lit_cap,
                                   uint64_t *lit_len, sydelta_delta **out, void *stream);
/* The zstd frame (RFC 8878) of d_in[0, len) into d_out, on the device: what ssh.rs:1009-1017
 * sends (compress(delta_json, Compression::Zstd), compress/mod.rs:71-76) and sy-remote
 * decompresses (sy-remote.rs:160-179) -- typically the text of sydelta_delta_to_json_device.
 * One 128 KiB block per workgroup: Huffman-coded literals alone, or literals + FSE-coded
 * sequences (matches at the JSON skeleton's distances), Raw / RLE where smaller; any zstd
 * decoder returns the input; the bytes differ from libzstd level 3's.  d_in 16-byte
 * aligned and readable to the end of its last 16-byte granule; out_cap >=
 * sydelta_zstd_bound(len); *out_len = frame size. */
uint64_t sydelta_zstd_bound(uint64_t len);
int sydelta_zstd_compress_device(int device, const uint8_t *d_in, uint64_t len, uint8_t *d_out, uint64_t out_cap,
                                 uint64_t *out_len, void *stream);
/* serde_json::from_str::<Delta> (sy-remote.rs:175): a host delta holding its literal
 * bytes, ready for sydelta_apply_delta. */
int sydelta_delta_from_json(const char *json, uint64_t len, sydelta_delta **out);

/* ---------------------------------------------------------------------------
 * Local transport, files already in device memory.
 * ------------------------------------------------------------------------- */
typedef struct sydelta_block_compare_stats {
    uint64_t blocks;          /* ceil(src_len / block_size) */
    uint64_t changed_blocks;  /* local.rs changed_blocks */
    uint64_t literal_bytes;   /* bytes of the changed blocks */
    uint64_t bytes_written;   /* src_len */
} sydelta_block_compare_stats;
/* The block-compare loop of src/transport/local.rs:541-619 (:682-760): d_changed[k] = 1
 * iff block k of the source (length min(bs, src_len - k*bs)) differs from block k of the
 * destination in length or bytes.  d_changed holds ceil(src_len / block_size) bytes. */
int sydelta_block_compare_device(int device, const uint8_t *d_src, uint64_t src_len, const uint8_t *d_dst,
                                 uint64_t dst_len, uint64_t block_size, uint8_t *d_changed, void *stream,
                                 sydelta_block_compare_stats *out);
/* ratio.rs:11-45 `ChangeRatioResult`. */
typedef struct sydelta_change_ratio {
    double change_ratio;
    uint64_t blocks_sampled;
    uint64_t blocks_changed;
    int32_t use_delta;
    int32_t reserved;
    double threshold;
} sydelta_change_ratio;
/* ratio.rs:78-192 `estimate_change_ratio` on device-resident bytes (sample_count < 0:
 * 20, threshold < 0: 0.75, the defaults of :85-86). */
int sydelta_estimate_change_ratio_device(int device, const uint8_t *d_src, uint64_t src_len, const uint8_t *d_dst,
                                         uint64_t dst_len, uint64_t block_size, int64_t sample_count,
                                         double threshold, void *stream, sydelta_change_ratio *out);
/* ratio.rs:78 `estimate_change_ratio(source: &Path, dest: &Path, block_size, sample_count:
 * Option<usize>, threshold: Option<f64>) -> io::Result<ChangeRatioResult>` on two paths:
 * the sampled blocks are read from the files and hashed on the current device
 * (sample_count < 0 / threshold < 0: the defaults).  Open/read failures -> SYDELTA_E_IO. */
int sydelta_estimate_change_ratio(const char *source_path, const char *dest_path, uint64_t block_size,
                                  int64_t sample_count, double threshold, sydelta_change_ratio *out);

/* ---------------------------------------------------------------------------
 * Whole-file XXH3-64, bytes already in device memory.
 * ------------------------------------------------------------------------- */
/* XxHash3Hasher::hash_file / hash_data (src/integrity/xxhash3.rs:17-40): *out =
 * xxh3_64(d_buf[0, len)) with seed 0 (the streaming digest equals the one-shot hash). */
int sydelta_xxh3_device(int device, const uint8_t *d_buf, uint64_t len, void *stream, uint64_t *out);
/* The same for nfiles files [offs[f], offs[f] + lens[f]) of d_buf (host arrays), as the
 * verify loop of integrity/mod.rs:104 hashes them one by one: out[f] (host) = hash.
 * Every range must lie inside [0, buf_len). */
int sydelta_xxh3_batch_device(int device, const uint8_t *d_buf, uint64_t buf_len, const uint64_t *offs, const uint64_t *lens,
                              uint64_t nfiles, void *stream, uint64_t *out);

/* ---------------------------------------------------------------------------
 * Measurement support (used by bench.py; not part of the reference API).
 * ------------------------------------------------------------------------- */
/* When on, the library records a HIP event pair around every kernel it
 * launches (on the stream it launches on) and accumulates per-kernel time. */
void sydelta_set_profiling(int on);
/* JSON object {"kernel": {"ms": total, "count": n}, ...}; returns bytes written
 * (excluding NUL) or the size needed if cap is too small. Clears with reset. */
size_t sydelta_profile_json(char *buf, size_t cap, int reset);
/* Walks resolved on the device (K5b, SYDELTA_DEVICE_WALK=1) and walks it handed back to
 * the host walk (the path reached a position only an on-demand scan classifies), since
 * the library was loaded. */
int sydelta_walk_counters(uint64_t *device_walks, uint64_t *device_fallbacks);
/* Files of batched matches whose op lists the device expanded (K10, each file's last walk
 * unit; the host had few threads for them or SYDELTA_DEVICE_EXPAND=1), and batches whose
 * expansion went back to the host (a file needed a re-walk), since the library was loaded. */
int sydelta_expand_counters(uint64_t *device_files, uint64_t *host_batches);
/* Deterministic synthetic bytes on the device: counter-based splitmix64 of
 * (seed, 8-byte word index), little endian (oracle.synth_bytes). */
int sydelta_synth_fill(uint8_t *d_buf, uint64_t len, uint64_t seed, void *stream);
/* d_dst = d_src with each byte independently replaced, with probability
 * rate_ppm / 1e6, by a different uniform byte (BASELINE config 3). */
int sydelta_synth_mutate(uint8_t *d_dst, const uint8_t *d_src, uint64_t len, uint64_t seed, uint32_t rate_ppm,
                         void *stream);

/* Ranged forms for sharded inputs: bytes [first, first + len) of the same streams
 * (first a multiple of 8 for fill). */
int sydelta_synth_fill_range(uint8_t *d_buf, uint64_t first, uint64_t len, uint64_t seed, void *stream);
/* BASELINE config 5 edit model: d_dst = d_src with, in each block_size-aligned block
 * k (global index) selected with probability rate_ppm / 1e6, one byte at a
 * pseudo-random offset replaced by a different byte.  d_src/d_dst hold bytes
 * [first, first + len), first a multiple of block_size. */
int sydelta_synth_mutate_blocks(uint8_t *d_dst, const uint8_t *d_src, uint64_t first, uint64_t len,
                                uint64_t block_size, uint64_t seed, uint32_t rate_ppm, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SYDELTA_H */
