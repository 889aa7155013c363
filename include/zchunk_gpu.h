/*
 * zchunk_gpu.h — C ABI of the MI355X (gfx950) Zarr chunk-codec path.
 *
 * This is the drop-in boundary for the reference's chunk codec path
 * (sci-rs/zarr v0.0.1).  Every entry point below replaces one piece of the
 * reference; the file:line it replaces is cited next to it.  All arguments
 * are plain pointers and sizes; no torch / HIP C++ types appear in the
 * signatures (`stream` is an opaque hipStream_t passed as void*).
 *
 * Reference interface being replaced (paths relative to the reference root):
 *   - trait Compression { decoder(R)->Box<dyn Read>; encoder(W)->Box<dyn Write> }
 *       src/compression/mod.rs:30-34, dispatch mod.rs:72-108
 *   - enum CompressionType {Raw, Bzip2, Gzip, Lz4, Xz}  src/compression/mod.rs:40-51
 *   - DefaultChunkReader::read_chunk / read_chunk_into   src/chunk.rs:270-301
 *   - DefaultChunkWriter::write_chunk                    src/chunk.rs:306-323
 *   - ReadableDataChunk::read_data (exact-N read, byte order, bool rule)
 *                                                        src/chunk.rs:103-116,163-222
 *   - WriteableDataChunk::write_data                     src/chunk.rs:118-140,169-237
 *
 * Semantics kept from the reference (see DESIGN.md "Parity contract"):
 *   - decode produces EXACTLY num_elements*elem_size bytes (read_exact,
 *     chunk.rs:112-113): a longer stream is truncated silently, a shorter one
 *     is ZCG_ERR_UNEXPECTED_EOF (tests.rs:191-219).
 *   - big-endian dtypes are byte-swapped per element (byteorder read_*_into);
 *     single-byte types and bool ignore endianness (data_type.rs:425-432).
 *   - bool: decoded byte != 0 -> 1 (chunk.rs:175-190).
 *   - encode requires the element count to equal product(chunk_shape)
 *     (chunk.rs:309-318) -> ZCG_ERR_INVALID_DATA otherwise.
 *   - only the first gzip member / LZ4 frame / xz stream / bzip2 stream is
 *     decoded (single-stream decoders of flate2/lz4-rs/xz2/bzip2).
 *
 * Threading: one zcg_ctx per device; a ctx is not shared across host threads
 * without external locking.  Work on distinct streams is independent.
 */
#ifndef ZCHUNK_GPU_H
#define ZCHUNK_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZCG_ABI_VERSION 1

/* CompressionType variants (src/compression/mod.rs:40-51).  Numbering is
 * this ABI's own; the JSON codec ids are mapped by the host layer. */
enum zcg_codec {
    ZCG_CODEC_RAW = 0,   /* raw.rs:13-24 */
    ZCG_CODEC_BZIP2 = 1, /* bzip.rs:16-46 */
    ZCG_CODEC_GZIP = 2,  /* gzip.rs:16-57 */
    ZCG_CODEC_LZ4 = 3,   /* lz.rs:45-93 */
    ZCG_CODEC_XZ = 4     /* xz.rs:15-43 */
};

/* Per-chunk status words; map 1:1 onto std::io::ErrorKind of the reference. */
enum zcg_status {
    ZCG_OK = 0,
    ZCG_ERR_UNEXPECTED_EOF = 1, /* io::ErrorKind::UnexpectedEof (short stream) */
    ZCG_ERR_INVALID_DATA = 2,   /* corrupt stream / wrong element count        */
    ZCG_ERR_INVALID_INPUT = 3,  /* dtype mismatch (chunk.rs:261-264), bad args */
    ZCG_ERR_UNSUPPORTED = 4,    /* e.g. LZ4 dictionary frames                  */
    ZCG_ERR_OUTPUT_TOO_SMALL = 5, /* encode: dst capacity below the stream size */
    ZCG_ABSENT = 6,             /* store: no chunk file (get() -> Ok(None), read_chunk -> None) */
    ZCG_ERR_IO = 7,             /* store: a filesystem error (open/lock/read/write)  */
    ZCG_ERR_NOT_FOUND = 8,      /* store: key outside the hierarchy (io::ErrorKind::NotFound,
                                   filesystem.rs:180-186)                        */
    ZCG_ERR_RUNTIME = 100       /* HIP runtime failure (see zcg_last_error)     */
};

/* Decode flags (zcg_compression.flags).  The reference's read_exact never
 * reaches the gzip CRC32/ISIZE trailer or the LZ4 content checksum on a
 * full-length read, so neither is verified.  LZ4
 * block checksums are verified as LZ4F does, unless this flag skips them
 * (the decoded bytes are the same; only a corrupt checksum word changes the
 * status).  Bits 0x1 and 0x2 are reserved. */
#define ZCG_FLAG_SKIP_LZ4_BLOCK_CHECKSUM 0x4u
/* Use the wave-serial inflate kernel instead of the parallel one (the two are
 * bit-identical; the serial one is kept as a differential reference). */
#define ZCG_FLAG_SERIAL_INFLATE 0x100u
/* Accumulate internal kernel statistics (development builds / profiling; the
 * default build compiles the inflate wave kernel's counters out, so there the
 * flag changes nothing). */
#define ZCG_FLAG_DEBUG_COUNTERS 0x200u
/* Xz decode keeps 32 KiB of history in LDS instead of 4 KiB: far matches
 * stop re-reading the output from L2/HBM, at 3 instead of 8 chunks per CU. */
#define ZCG_FLAG_XZ_RING_32K 0x400u
/* LZ4 block decoder choice (bit-identical): one wave per block (speculative
 * parse, byte-parallel resolve) or one lane per block; by default the batch
 * size picks: waves below 131 072 blocks, both side by side (on a second
 * stream) below 196 608, lanes from there. */
#define ZCG_FLAG_LZ4_WAVE_PER_BLOCK 0x800u
#define ZCG_FLAG_LZ4_LANE_PER_BLOCK 0x1000u
/* Gzip decode kernel choice (all bit-identical).  By default a batch of at
 * most 3 chunks per CU (one generation of the 256-lane kernel) runs the
 * 256-lane round kernel (fine 256-bit segments, one workgroup of 4 waves per
 * chunk: half the latency of a lone chunk), a larger one the one-wave-per-chunk
 * kernel (coarse segments, 16 chunks per CU).  These flags force one. */
#define ZCG_FLAG_INFLATE_BLOCK_PAR 0x2000u
#define ZCG_FLAG_INFLATE_WAVE 0x4000u
/* Gzip encode at levels 1-9 is byte-identical to zlib 1.2.11 / flate2
 * (gzip.rs:54-56) by default (deflate_fast for 1-3, deflate_slow for 4-9).
 * This flag selects the faster segmented coder instead (16 KiB blocks, each
 * ended by an empty stored block; the stream inflates to the same data, but
 * its bytes differ from zlib's).  Level 0 always uses the segmented coder. */
#define ZCG_FLAG_GZIP_SEGMENTED 0x8000u
/* Test hook: the one-wave-per-chunk inflate kernel sizes its first segments
 * at 116 % instead of 108 % of the estimated block bits, which makes the
 * first round of all-literal 16 383-symbol blocks cap a list and halve the
 * segment size (the round-6 regression test of that path).  Same output. */
#define ZCG_FLAG_DEBUG_INFLATE_LONG_SEG 0x10000u

/* CompressionType + its configuration (camelCase JSON keys in the reference). */
typedef struct zcg_compression {
    int32_t codec;            /* enum zcg_codec                                 */
    int32_t gzip_level;       /* gzip.rs:16-20, -1 / out of [0,9] -> 6 (28-34)  */
    int32_t lz4_block_size;   /* lz.rs:45-50, rounded to 64K/256K/1M/4M (55-65) */
    int32_t bzip2_block_size; /* bzip.rs:16-21, 1..9                            */
    int32_t xz_preset;        /* xz.rs:15-20                                    */
    uint32_t flags;           /* ZCG_FLAG_*                                     */
} zcg_compression;

/* Effective element type (data_type.rs:417-432). */
typedef struct zcg_dtype {
    uint8_t elem_size;  /* 1, 2, 4 or 8 */
    uint8_t big_endian; /* 1 for '>' types of size > 1 */
    uint8_t is_bool;    /* 1 for "bool" */
    uint8_t reserved;
} zcg_dtype;

/* What one batch shares: the array's codec, dtype and chunk element count
 * (ArrayMetadata, lib.rs:382-402; get_chunk_num_elements lib.rs:474-480). */
typedef struct zcg_array {
    zcg_compression compression;
    zcg_dtype dtype;
    uint64_t chunk_num_elements;
} zcg_array;

/* One chunk of a batch.  All pointers are DEVICE pointers, caller-owned.
 *  decode: src = compressed stream (src_len bytes), dst = N*elem_size bytes
 *  encode: src = N*elem_size bytes of native (little-endian) elements,
 *          dst = output buffer of capacity dst_cap bytes                  */
typedef struct zcg_chunk {
    const void* src;
    uint64_t src_len;
    void* dst;
    uint64_t dst_cap;
} zcg_chunk;

typedef struct zcg_ctx zcg_ctx;

/* ---- context -------------------------------------------------------- */
int zcg_abi_version(void);
/* The kernels' tuning constants this library was built with, as
 * "kernel:K=V,...;kernel:K=V,..." (A/B builds under tools/ change them; the
 * product build uses the defaults, which tests/test_abi.py checks). */
const char* zcg_build_config(void);
zcg_ctx* zcg_create(int device);
void zcg_destroy(zcg_ctx* ctx);
const char* zcg_last_error(const zcg_ctx* ctx);
/* Effective parameters the reference would use (gzip.rs:28-34, lz.rs:55-65). */
int32_t zcg_effective_gzip_level(int32_t level);
int32_t zcg_effective_lz4_block_size(int32_t block_size);
int zcg_codec_on_gpu(int32_t codec, int encode);

/* ---- device-resident batch API (the hot path) ------------------------
 * Replaces N calls of DefaultChunk::read_chunk_into (chunk.rs:288-301) with
 * one batched, stream-ordered launch sequence.  `d_chunks` and `d_status`
 * are device arrays of n entries.  Asynchronous on `stream`; returns a
 * zcg_status for argument/launch errors only — per-chunk results land in
 * d_status.  Workspace is grown on first use of a given batch shape
 * (hipMalloc), so steady-state calls do no allocation and are capturable.
 * The workspace is kept per stream (gzip decode: ~0.9 GB at full batch,
 * zcg_workspace_bytes gives the figure); a context keeps at most 4 streams'
 * workspaces and frees the least recently used one (after a device-wide
 * synchronize) when a fifth stream arrives. */
int zcg_decode_batch(zcg_ctx* ctx, const zcg_array* array, const zcg_chunk* d_chunks,
                     uint32_t n, int32_t* d_status, void* stream);

/* Replaces N calls of DefaultChunk::write_chunk (chunk.rs:306-323).
 * d_out_len[i] receives the encoded stream length of chunk i.  LZ4 encode
 * accepts at most 4096 LZ4 blocks per chunk (256 MiB at the 64 KiB default
 * block size); beyond that it returns ZCG_ERR_UNSUPPORTED (zcg_last_error
 * says why) and launches nothing. */
int zcg_encode_batch(zcg_ctx* ctx, const zcg_array* array, const zcg_chunk* d_chunks,
                     uint32_t n, uint64_t* d_out_len, int32_t* d_status, void* stream);

/* Upper bound of an encoded chunk of `src_len` bytes for this codec. */
uint64_t zcg_encode_bound(const zcg_compression* c, uint64_t src_len);

/* Bytes of device workspace a batch of this shape needs (informational). */
uint64_t zcg_workspace_bytes(const zcg_array* array, uint32_t n, int encode);

/* ---- host-memory conveniences (one read_chunk / write_chunk) ---------
 * zcg_read_chunk == DefaultChunkReader::read_chunk body (chunk.rs:270-286)
 * on host buffers: H2D of the stream, GPU decode, D2H of the elements.
 * `dst` receives N*elem_size bytes (host-native order). */
int zcg_read_chunk(zcg_ctx* ctx, const zcg_array* array, const void* src, uint64_t src_len,
                   void* dst);
/* zcg_write_chunk == DefaultChunkWriter::write_chunk (chunk.rs:306-323):
 * `n_elements` must equal array->chunk_num_elements (else INVALID_DATA). */
int zcg_write_chunk(zcg_ctx* ctx, const zcg_array* array, const void* elems,
                    uint64_t n_elements, void* out, uint64_t out_cap, uint64_t* out_len);

/* Host-resident batch (e2e path): pinned staging, H2D, decode, D2H.
 * srcs/src_lens/dsts/status are host arrays of n entries. */
int zcg_read_chunks_host(zcg_ctx* ctx, const zcg_array* array, uint32_t n,
                         const void* const* srcs, const uint64_t* src_lens, void* const* dsts,
                         int32_t* status);

/* ---- region assembly ----------------------------
 * Replaces ZarrNdarrayReader::read_ndarray / read_ndarray_into_with_buffer
 * (ndarray.rs:153-268): decoded chunks that already sit in HBM are
 * scattered into one bounding box on the device.  Chunk order is the
 * array's memory layout (ndarray.rs:453-462: ColumnMajor -> dim 0 fastest,
 * RowMajor -> last dim fastest); the output is any strided view of
 * bbox_shape (out_strides in elements, ndarray's ArrayViewMut).  Edge chunks
 * overhang the array and are read over their full nominal extent
 * (get_chunk_bounds, ndarray.rs:434-446); chunks are the ones
 * bounded_coord_iter visits (ndarray.rs:410-432). */
#define ZCG_MAX_DIMS 8
typedef struct zcg_region {
    uint32_t ndim;         /* 1..ZCG_MAX_DIMS                                   */
    uint32_t elem_size;    /* 1, 2, 4, 8 (decoded, host-native element bytes)    */
    uint32_t chunk_order;  /* 0 = RowMajor (C), 1 = ColumnMajor (F), lib.rs Order */
    uint32_t fill_missing; /* 1: read_ndarray — every element no chunk covers gets
                              fill_value (Array::from_elem, ndarray.rs:164-171);
                              0: read_ndarray_into — such elements are untouched */
    uint64_t array_shape[ZCG_MAX_DIMS];
    uint64_t chunk_shape[ZCG_MAX_DIMS];
    uint64_t bbox_offset[ZCG_MAX_DIMS];
    uint64_t bbox_shape[ZCG_MAX_DIMS];
    int64_t out_strides[ZCG_MAX_DIMS]; /* per array dim, in elements */
    uint64_t fill_value;   /* elem_size low bytes, host order (get_effective_fill_value) */
} zcg_region;

/* The chunk grid range a region reads: grid_lo[d] .. grid_lo[d]+grid_n[d]
 * (bounded_coord_iter, ndarray.rs:410-432).  Returns the number of chunks
 * (0 when the box misses the array). */
uint64_t zcg_region_grid(const zcg_region* r, uint64_t* grid_lo, uint64_t* grid_n);

/* d_chunk_table: device array of zcg_region_grid() DEVICE pointers to the
 * decoded chunks (N*elem_size bytes each), C order over the grid range
 * (dim 0 slowest); NULL = chunk absent (read_chunk -> Ok(None)).  d_out is
 * the base of the output view.  Asynchronous on `stream`. */
int zcg_read_region(zcg_ctx* ctx, const zcg_region* r, const void* const* d_chunk_table,
                    void* d_out, void* stream);

/* The inverse scatter of ZarrNdarrayWriter::write_ndarray (ndarray.rs:276-385):
 * the box (d_in, a strided view of bbox_shape) is written into the chunk
 * slots of d_chunk_table (same grid range and order as zcg_read_region; every
 * element of the box that falls in a non-NULL chunk is written, at its
 * chunk-local position in the chunk memory order).  The caller pre-fills
 * slots of partially covered chunks with the existing chunk (or fill value)
 * and encodes the slots afterwards (zcg_encode_batch).  fill_missing is
 * ignored.  Asynchronous on `stream`. */
int zcg_write_region(zcg_ctx* ctx, const zcg_region* r, void* const* d_chunk_table,
                     const void* d_in, void* stream);

/* ---- FilesystemHierarchy chunk files ---------------
 * The e2e path's two ends: chunk files read into pinned staging by a pool of
 * `io_threads` host threads (open + shared flock + read, as ReadableStore::get,
 * src/store/filesystem.rs:201-210), H2D, zcg_decode_batch, D2H into `dsts`
 * (N*elem_size bytes each), pipelined over two streams in sub-batches of
 * <= 256 MiB (1 GiB for xz/bzip2); status[i] = ZCG_ABSENT for a missing chunk (read_chunk -> None,
 * src/storage.rs:226-234), ZCG_ERR_IO for a filesystem error, else the decode
 * status.  The write direction encodes `elems` (N*elem_size host bytes each)
 * on the GPU and writes each file as WriteableStore::set (filesystem.rs:260-280):
 * create_dir_all(parent), open, exclusive flock, truncate, write.  Paths come
 * from the caller (get_chunk_key, storage.rs:109-127).  Blocking. */
int zcg_store_read_chunks(zcg_ctx* ctx, const zcg_array* array, uint32_t n, const char* const* paths,
                          void* const* dsts, int32_t* status, uint32_t io_threads);
int zcg_store_write_chunks(zcg_ctx* ctx, const zcg_array* array, uint32_t n, const char* const* paths,
                           const void* const* elems, int32_t* status, uint32_t io_threads);
/* Device-resident ends of the same two calls, for callers whose chunks live in
 * HBM (read_ndarray / write_ndarray, ndarray.rs:195-268,276-385, which call
 * read_chunk_into / write_chunk per chunk through the same store get()/set()):
 *  - zcg_store_read_chunks_device decodes each file straight into the caller's
 *    DEVICE slot d_dsts[i] (N*elem_size bytes); only the statuses come back.
 *    A slot whose chunk is absent or unreadable is left untouched.
 *  - zcg_store_write_chunks_device encodes the DEVICE element slots d_elems[i]
 *    and writes each file as set() does (exclusive flock, then truncate).
 * `status` is a host array; both calls block until the files are read/written.
 * Destinations of zcg_store_read_chunks that are page-locked host memory
 * (hipHostMalloc / hipHostRegister) receive the decoded chunk by a direct D2H. */
int zcg_store_read_chunks_device(zcg_ctx* ctx, const zcg_array* array, uint32_t n, const char* const* paths,
                                 void* const* d_dsts, int32_t* status, uint32_t io_threads);
int zcg_store_write_chunks_device(zcg_ctx* ctx, const zcg_array* array, uint32_t n, const char* const* paths,
                                  const void* const* d_elems, int32_t* status, uint32_t io_threads);

/* ---- several GPUs in one process -------------------------
 * Chunk i goes to devices[i mod n_devices]; one host thread and one context
 * per device, no collective (chunks are independent, chunk.rs:282,297); the
 * per-chunk status arrays are merged.  Same arguments as the single-context
 * calls; returns the first failing device's return code. */
typedef struct zcg_multi zcg_multi;
zcg_multi* zcg_multi_create(const int* devices, uint32_t n_devices);
void zcg_multi_destroy(zcg_multi* multi);
const char* zcg_multi_last_error(const zcg_multi* multi);
uint32_t zcg_multi_device_count(const zcg_multi* multi);
int zcg_multi_read_chunks_host(zcg_multi* multi, const zcg_array* array, uint32_t n, const void* const* srcs,
                               const uint64_t* src_lens, void* const* dsts, int32_t* status);
int zcg_multi_store_read_chunks(zcg_multi* multi, const zcg_array* array, uint32_t n,
                                const char* const* paths, void* const* dsts, int32_t* status,
                                uint32_t io_threads);
int zcg_multi_store_write_chunks(zcg_multi* multi, const zcg_array* array, uint32_t n,
                                 const char* const* paths, const void* const* elems, int32_t* status,
                                 uint32_t io_threads);

/* ---- array metadata JSON -------------------------
 * The Zarr v3.0-dev array document (ArrayMetadata's serde form, lib.rs:382-402;
 * DataType strings data_type.rs:165-240; ExtensibleDataType fallback
 * data_type.rs:282-310; CompressionType {"codec", "configuration"} with the
 * codecs' serde defaults, compression/mod.rs:36-51) parsed into the batch
 * API's descriptor, so a C or Rust caller can drive zcg_decode_batch from a
 * real hierarchy.  Returns ZCG_OK; ZCG_ERR_INVALID_DATA for a malformed
 * document (serde's io::ErrorKind::InvalidData); ZCG_ERR_UNSUPPORTED where the
 * reference panics (unknown endian/size character, an extended type without
 * fallback) or rejects the document (a must_understand extension,
 * storage.rs:172-176).  `err` (optional) receives a message. */
enum zcg_dtype_kind { ZCG_DT_BOOL = 0, ZCG_DT_INT = 1, ZCG_DT_UINT = 2, ZCG_DT_FLOAT = 3, ZCG_DT_RAW = 4 };
typedef struct zcg_array_meta {
    zcg_array array;            /* codec + configuration, effective dtype,
                                   chunk_num_elements = product(chunk_shape) (lib.rs:474-480) */
    uint32_t ndim;              /* len(shape) */
    uint32_t chunk_ndim;        /* len(chunk_shape) */
    uint32_t chunk_order;       /* chunk_memory_layout: 0 = "C" (RowMajor), 1 = "F" (ColumnMajor) */
    uint32_t dtype_kind;        /* enum zcg_dtype_kind of the effective type */
    uint32_t extended_type;     /* 1: data_type was an extension object (its fallback is used) */
    uint32_t has_fill_value;    /* fill_value present, not null, and convertible to the type */
    int32_t fill_value_status;  /* ZCG_OK, or why fill_value does not convert (get_effective_fill_value) */
    uint32_t reserved;
    uint64_t fill_value;        /* element bytes of the effective fill value, host order (0 = T::default()) */
    uint64_t shape[ZCG_MAX_DIMS];
    uint64_t chunk_shape[ZCG_MAX_DIMS];
    char separator[8];          /* chunk_grid.separator (get_chunk_key, storage.rs:109-127) */
} zcg_array_meta;

int zcg_array_meta_from_json(const char* json, uint64_t len, zcg_array_meta* out, char* err, uint64_t err_cap);

/* get_chunk_key (storage.rs:109-127): "/data/root/<path>/c<g0><sep><g1>...<sep><g(n-1)>",
 * with `path` canonicalised as canonicalize_path does (leading and trailing '/'
 * removed, lib.rs:187-189; an empty path gives "/data/root/c...") and `separator`
 * = chunk_grid.separator (zcg_array_meta.separator).  Writes at most cap-1 bytes
 * and a NUL (cap > 0); returns the key's full length, so a caller can size
 * `out`.  A FilesystemHierarchy file is the store root joined with the key
 * (filesystem.rs:142-190). */
uint64_t zcg_chunk_key(const char* path, const char* separator, const uint64_t* grid_position, uint32_t ndim,
                       char* out, uint64_t cap);

/* FilesystemHierarchy::get_path (src/store/filesystem.rs:151-190): the file a
 * key names under the store root `root`.  The key's leading '/'s are dropped
 * (it is taken relative to the root), empty and "." components vanish, ".."
 * stays in the path, and the key is refused with ZCG_ERR_NOT_FOUND when its
 * NET nesting (+1 per normal component, -1 per "..") is negative — the
 * reference's rule, so "a/../b" and even "../x" (net 0) are accepted, "../../x"
 * is not.  That rule lets "../x" resolve OUTSIDE the root: a reference flaw
 * restated on purpose (parity); callers writing untrusted keys should refuse
 * ".." components themselves.  The path is root + '/' + the normalised key
 * (just the key when root is empty, as PathBuf::join does).  *path_len (optional) receives its length;
 * `out` (cap bytes, NUL-terminated) may be NULL to query the length, and a cap
 * below path_len + 1 gives ZCG_ERR_OUTPUT_TOO_SMALL.  Returns ZCG_OK. */
int zcg_store_path(const char* root, const char* key, char* out, uint64_t cap, uint64_t* path_len);

#ifdef __cplusplus
}
#endif

#endif /* ZCHUNK_GPU_H */
