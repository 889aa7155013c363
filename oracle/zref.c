/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference chunk-codec path of sci-rs/zarr v0.0.1,
 * used as the parity checker by tests/, __graft_entry__.smoke() and as the
 * `cpu_baseline` leg of bench.py.  Nothing in the product path (zarr_amd/,
 * include/) links, loads or calls this file.
 *
 * What is restated here (reference file:line, relative to the reference root):
 *   - DefaultChunkReader::read_chunk   src/chunk.rs:270-286
 *   - ReadableDataChunk::read_data     src/chunk.rs:103-116 (+u8 163-167,
 *     bool 175-190, f16 208-222): exactly N*size bytes via read_exact, then a
 *     per-element byte swap for Big endian, bool = byte != 0.
 *   - DefaultChunkWriter::write_chunk  src/chunk.rs:306-323 and write_data
 *     chunk.rs:118-140 (+u8 169-173, bool 192-206, f16 224-237).
 *   - Codec construction: gzip.rs:28-57 (flate2 GzDecoder/GzEncoder),
 *     lz.rs:55-92 (lz4-rs Decoder / EncoderBuilder, Independent blocks),
 *     bzip.rs:35-46 (bzip2 BzDecoder/BzEncoder), xz.rs:34-43 (xz2).
 *
 * The codec arithmetic itself lives in third-party crates that are NOT
 * vendored in the reference (Cargo.toml:29-45, no Cargo.lock):
 *   flate2 ^1.0.22 feature "zlib" -> zlib      (here: zlib 1.2.11, zlib.h)
 *   lz4    ^1.23  -> lz4-sys bundled liblz4 1.9.x (here: liblz4.so.1 1.9.3)
 *   bzip2  ^0.4   -> bzip2-sys libbz2 1.0.x    (here: libbz2.so.1 1.0.8)
 *   xz2    ^0.1   -> lzma-sys liblzma 5.2.x    (here: liblzma.so.5 5.2.5)
 * Those same C libraries are linked here, so the codec arithmetic of the
 * oracle IS the reference's.  The Rust glue (header convention of flate2,
 * lz4-rs streaming preferences, exact-N reads, byte order) is restated in C.
 * liblz4/libbz2/liblzma ship without headers in this image, so the few
 * prototypes and structs used are declared below from their public APIs.
 *
 * Pinned against the reference's own golden vectors (tests/golden, see
 * tests/test_oracle.py): the doc-spec chunk of every codec (raw.rs:33-45,
 * gzip.rs:66-80, lz.rs:101-115, bzip.rs:55-72, xz.rs:52-75) decodes to
 * [1..6] as >i2, and encodes byte-exactly for raw/gzip(OS=255)/lz4/xz
 * (tests.rs:147-159); the 8 zarrita chunks decode to arange(120).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* Status words: identical numbering to include/zchunk_gpu.h. */
enum { ZR_OK = 0, ZR_EOF = 1, ZR_INVALID_DATA = 2, ZR_INVALID_INPUT = 3, ZR_UNSUPPORTED = 4,
       ZR_TOO_SMALL = 5 };
enum { ZR_RAW = 0, ZR_BZIP2 = 1, ZR_GZIP = 2, ZR_LZ4 = 3, ZR_XZ = 4 };

/* ---------------- liblz4 frame API (lz4frame.h of liblz4 1.9.x) -------- */
typedef struct LZ4F_cctx_s LZ4F_cctx;
typedef struct LZ4F_dctx_s LZ4F_dctx;
typedef struct {
    int blockSizeID;          /* LZ4F_blockSizeID_t: 4=64K 5=256K 6=1M 7=4M */
    int blockMode;            /* 0 linked, 1 independent */
    int contentChecksumFlag;  /* 0/1 */
    int frameType;            /* 0 frame */
    unsigned long long contentSize;
    unsigned dictID;
    int blockChecksumFlag;
} LZ4F_frameInfo_t;
typedef struct {
    LZ4F_frameInfo_t frameInfo;
    int compressionLevel;
    unsigned autoFlush;
    unsigned favorDecSpeed;
    unsigned reserved[3];
} LZ4F_preferences_t;
typedef struct { unsigned stableDst; unsigned reserved[3]; } LZ4F_decompressOptions_t;
extern unsigned LZ4F_isError(size_t code);
extern size_t LZ4F_createCompressionContext(LZ4F_cctx** c, unsigned version);
extern size_t LZ4F_freeCompressionContext(LZ4F_cctx* c);
extern size_t LZ4F_compressBegin(LZ4F_cctx* c, void* dst, size_t cap, const LZ4F_preferences_t* p);
extern size_t LZ4F_compressBound(size_t srcSize, const LZ4F_preferences_t* p);
extern size_t LZ4F_compressUpdate(LZ4F_cctx* c, void* dst, size_t cap, const void* src,
                                  size_t n, const void* opt);
extern size_t LZ4F_compressEnd(LZ4F_cctx* c, void* dst, size_t cap, const void* opt);
extern size_t LZ4F_createDecompressionContext(LZ4F_dctx** d, unsigned version);
extern size_t LZ4F_freeDecompressionContext(LZ4F_dctx* d);
extern size_t LZ4F_decompress(LZ4F_dctx* d, void* dst, size_t* dstSize, const void* src,
                              size_t* srcSize, const LZ4F_decompressOptions_t* opt);
#define LZ4F_VERSION 100

/* ---------------- libbz2 (bzlib.h of bzip2 1.0.x) ---------------------- */
typedef struct {
    char* next_in; unsigned int avail_in; unsigned int total_in_lo32; unsigned int total_in_hi32;
    char* next_out; unsigned int avail_out; unsigned int total_out_lo32; unsigned int total_out_hi32;
    void* state;
    void* (*bzalloc)(void*, int, int);
    void (*bzfree)(void*, void*);
    void* opaque;
} bz_stream;
extern int BZ2_bzCompressInit(bz_stream* s, int blockSize100k, int verbosity, int workFactor);
extern int BZ2_bzCompress(bz_stream* s, int action);
extern int BZ2_bzCompressEnd(bz_stream* s);
extern int BZ2_bzDecompressInit(bz_stream* s, int verbosity, int small);
extern int BZ2_bzDecompress(bz_stream* s);
extern int BZ2_bzDecompressEnd(bz_stream* s);
#define BZ_RUN 0
#define BZ_FINISH 2
#define BZ_OK 0
#define BZ_FINISH_OK 3
#define BZ_STREAM_END 4

/* ---------------- liblzma (lzma/base.h of xz 5.2.x) -------------------- */
typedef struct {
    const uint8_t* next_in; size_t avail_in; uint64_t total_in;
    uint8_t* next_out; size_t avail_out; uint64_t total_out;
    const void* allocator; void* internal;
    void *reserved_ptr1, *reserved_ptr2, *reserved_ptr3, *reserved_ptr4;
    uint64_t reserved_int1, reserved_int2;
    size_t reserved_int3, reserved_int4;
    int reserved_enum1, reserved_enum2;
} lzma_stream;
extern int lzma_easy_encoder(lzma_stream* s, uint32_t preset, int check);
extern int lzma_stream_decoder(lzma_stream* s, uint64_t memlimit, uint32_t flags);
extern int lzma_code(lzma_stream* s, int action);
extern void lzma_end(lzma_stream* s);
#define LZMA_OK 0
#define LZMA_STREAM_END 1
#define LZMA_RUN 0
#define LZMA_FINISH 3
#define LZMA_CHECK_CRC64 4

/* ----------------------------------------------------------------------
 * read_data post-processing (chunk.rs:103-116, 175-190): byteorder's
 * read_*_into::<BigEndian> swaps each element; bool maps byte != 0 -> 1.
 * Single-byte types and bool have NATIVE endianness (data_type.rs:429-430).
 */
static void zr_fix_elements(uint8_t* p, uint64_t nbytes, int elem_size, int big_endian,
                            int is_bool) {
    if (is_bool) {
        for (uint64_t i = 0; i < nbytes; i++) p[i] = p[i] != 0;
        return;
    }
    if (!big_endian || elem_size == 1) return;
    for (uint64_t e = 0; e + (uint64_t)elem_size <= nbytes; e += (uint64_t)elem_size)
        for (int a = 0, b = elem_size - 1; a < b; a++, b--) {
            uint8_t t = p[e + a]; p[e + a] = p[e + b]; p[e + b] = t;
        }
}

/* gzip.rs:28-34: level outside [0,9] (Java's -1 default) -> flate2 default 6. */
int zref_effective_gzip_level(int level) { return (level < 0 || level > 9) ? 6 : level; }

/* lz.rs:55-65: smallest lz4 BlockSize >= blockSize (64K, 256K, 1M, 4M). */
int zref_lz4_block_size_id(int block_size) {
    if (block_size <= 65536) return 4;
    if (block_size <= 262144) return 5;
    if (block_size <= 1048576) return 6;
    return 7;
}

/* ---------------- Gzip decode: flate2 read::GzDecoder ------------------
 * flate2 parses the member header itself (magic 1f 8b, CM 8, FLG with
 * FEXTRA/FNAME/FCOMMENT/FHCRC; FHCRC is verified against the CRC32 of the
 * header bytes), then runs zlib raw inflate (windowBits -15).  A read_exact
 * of N bytes stops as soon as N bytes are produced, so the CRC32/ISIZE
 * trailer is only consulted when the stream ends early (then: EOF). */
static int zr_gzip_header(const uint8_t* s, uint64_t n, uint64_t* hdr_len) {
    if (n < 10) return ZR_EOF;
    if (s[0] != 0x1f || s[1] != 0x8b || s[2] != 8) return ZR_INVALID_DATA;
    uint8_t flg = s[3];
    uint64_t p = 10;
    if (flg & 4) { /* FEXTRA */
        if (p + 2 > n) return ZR_EOF;
        uint64_t xlen = s[p] | ((uint64_t)s[p + 1] << 8);
        p += 2 + xlen;
        if (p > n) return ZR_EOF;
    }
    if (flg & 8) { /* FNAME */
        while (p < n && s[p]) p++;
        if (p >= n) return ZR_EOF;
        p++;
    }
    if (flg & 16) { /* FCOMMENT */
        while (p < n && s[p]) p++;
        if (p >= n) return ZR_EOF;
        p++;
    }
    if (flg & 2) { /* FHCRC: low 16 bits of CRC32 over the header so far */
        if (p + 2 > n) return ZR_EOF;
        uint32_t c = (uint32_t)crc32(0L, s, (uInt)p);
        if ((c & 0xffff) != (uint32_t)(s[p] | (s[p + 1] << 8))) return ZR_INVALID_DATA;
        p += 2;
    }
    *hdr_len = p;
    return ZR_OK;
}

/* flate2 read::GzDecoder = bufread::GzDecoder over BufReader::with_capacity
 * (32 KiB, r): the header is consumed from the buffered reader, then
 * zio::read hands zlib whatever fill_buf() returns (the rest of the current
 * 32 KiB window of the stream) with the remaining destination; read_exact
 * repeats until N bytes exist.  zlib keeps decoding the next symbol(s) after
 * the output is full as long as their bits are in the current window (LEN ->
 * LIT/MATCH leave only on `left == 0`), so a corrupt code right after byte N
 * is still an error in the reference: the windows are restated exactly. */
#define ZR_BUFREADER 32768u
static int zr_decode_gzip(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t dlen,
                          int verify_crc) {
    uint64_t h = 0;
    int st = zr_gzip_header(src, n, &h);
    if (st) return st;
    z_stream z;
    memset(&z, 0, sizeof z);
    if (inflateInit2(&z, -15) != Z_OK) return ZR_INVALID_DATA;
    uint64_t pos = h, got = 0;
    int r = Z_OK;
    while (got < dlen) {
        if (pos >= n) { r = Z_BUF_ERROR; break; }               /* eof: read() -> 0 */
        uint64_t wend = (pos / ZR_BUFREADER + 1) * ZR_BUFREADER;  /* fill_buf() */
        if (wend > n) wend = n;
        z.next_in = (Bytef*)(src + pos);
        z.avail_in = (uInt)(wend - pos);
        z.next_out = dst + got;
        z.avail_out = (uInt)(dlen - got);
        r = inflate(&z, Z_NO_FLUSH);
        uint64_t used = (wend - pos) - z.avail_in;
        pos += used;
        got = dlen - z.avail_out;
        if (r == Z_STREAM_END) break;
        if (r != Z_OK && r != Z_BUF_ERROR) break;
    }
    inflateEnd(&z);
    if (r != Z_OK && r != Z_BUF_ERROR && r != Z_STREAM_END) return ZR_INVALID_DATA;
    if (got < dlen) return ZR_EOF;
    if (verify_crc && r == Z_STREAM_END) {
        if (pos + 8 > n) return ZR_EOF;
        uint32_t c = (uint32_t)crc32(0L, dst, (uInt)dlen);
        uint32_t sc = src[pos] | (src[pos + 1] << 8) | (src[pos + 2] << 16) |
                      ((uint32_t)src[pos + 3] << 24);
        if (c != sc) return ZR_INVALID_DATA;
    }
    return ZR_OK;
}

/* ---------------- Lz4 decode: lz4-rs Decoder (LZ4F_decompress) -------- */
/* lz4-rs 1.23 Decoder: a 32 KiB buffer refilled with min(32 KiB, next)
 * bytes, where `next` starts at 11 and tracks LZ4F_decompress's size hint;
 * read() returns as soon as it produced output, read_exact loops.  So LZ4F
 * only ever sees the bytes its hint asked for: the content checksum after
 * the end mark is never fed on an exact-N read, while the next block header
 * usually is (it rides with the last piece of the block). */
static int zr_decode_lz4(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t dlen) {
    LZ4F_dctx* d = NULL;
    if (LZ4F_isError(LZ4F_createDecompressionContext(&d, LZ4F_VERSION))) return ZR_INVALID_DATA;
    uint64_t rpos = 0;                 /* reader position in src */
    uint64_t pos = 0, len = 0;         /* lz4-rs buf window [pos, len) */
    const uint8_t* buf = NULL;
    size_t next = 11;
    uint64_t out = 0;
    int st = ZR_OK;
    while (out < dlen && st == ZR_OK) {       /* read_exact -> read() */
        if (next == 0) { st = ZR_EOF; break; }  /* frame finished: read() -> 0 */
        uint64_t dst_off = 0;
        while (dst_off == 0) {
            if (pos >= len) {
                size_t need = next < 32768 ? next : 32768;
                uint64_t k = (n - rpos) < need ? (n - rpos) : need;
                if (k == 0) break;          /* reader eof: read() returns 0 */
                buf = src + rpos;
                rpos += k;
                pos = 0;
                len = k;
                next -= k;
            }
            while (out + dst_off < dlen && pos < len) {
                size_t ss = len - pos, ds = dlen - out - dst_off;
                size_t r = LZ4F_decompress(d, dst + out + dst_off, &ds, buf + pos, &ss, NULL);
                if (LZ4F_isError(r)) { st = ZR_INVALID_DATA; break; }
                pos += ss;
                dst_off += ds;
                if (r == 0) { next = 0; break; }
                if (next < r) next = r;
            }
            if (st != ZR_OK || next == 0) break;
        }
        if (st != ZR_OK) break;
        if (dst_off == 0) { st = ZR_EOF; break; }
        out += dst_off;
    }
    LZ4F_freeDecompressionContext(d);
    return st;
}

/* ---------------- Bzip2 decode: bzip2 read::BzDecoder -----------------
 * bufread::BzDecoder over BufReader::with_capacity(32 KiB): libbz2 is handed
 * the current 32 KiB window of the stream and the remaining destination.
 * (libbz2 verifies a block CRC and decodes the next block header/tables as
 * soon as a block's output completes, even with the output full — the
 * windowed feeding decides how much of that it can see.) */
static int zr_decode_bzip2(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t dlen) {
    bz_stream b;
    memset(&b, 0, sizeof b);
    if (BZ2_bzDecompressInit(&b, 0, 0) != BZ_OK) return ZR_INVALID_DATA;
    uint64_t pos = 0, got = 0;
    int st = ZR_OK;
    while (got < dlen) {
        if (pos >= n) { st = ZR_EOF; break; }
        uint64_t wend = (pos / ZR_BUFREADER + 1) * ZR_BUFREADER;
        if (wend > n) wend = n;
        b.next_in = (char*)(src + pos);
        b.avail_in = (unsigned)(wend - pos);
        b.next_out = (char*)(dst + got);
        b.avail_out = (unsigned)(dlen - got);
        int r = BZ2_bzDecompress(&b);
        pos += (wend - pos) - b.avail_in;
        got = dlen - b.avail_out;
        if (r == BZ_STREAM_END) { if (got < dlen) st = ZR_EOF; break; }
        if (r != BZ_OK) { st = ZR_INVALID_DATA; break; }
    }
    BZ2_bzDecompressEnd(&b);
    return st;
}

/* ---------------- Xz decode: xz2 read::XzDecoder (stream decoder) ------
 * bufread::XzDecoder over BufReader::with_capacity(32 KiB), stream decoder
 * with memlimit u64::MAX and no flags (single .xz stream, CRC64 checked by
 * liblzma as blocks complete); same windowed feeding as above. */
static int zr_decode_xz(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t dlen) {
    lzma_stream s;
    memset(&s, 0, sizeof s);
    if (lzma_stream_decoder(&s, UINT64_MAX, 0) != LZMA_OK) return ZR_INVALID_DATA;
    uint64_t pos = 0, got = 0;
    int st = ZR_OK;
    while (got < dlen) {
        int eof = pos >= n;
        uint64_t wend = eof ? n : (pos / ZR_BUFREADER + 1) * ZR_BUFREADER;
        if (wend > n) wend = n;
        s.next_in = src + pos;
        s.avail_in = wend - pos;
        s.next_out = dst + got;
        s.avail_out = dlen - got;
        int r = lzma_code(&s, eof ? LZMA_FINISH : LZMA_RUN);
        uint64_t used = (wend - pos) - s.avail_in;
        uint64_t made = (dlen - got) - s.avail_out;
        pos += used;
        got += made;
        if (r == LZMA_STREAM_END) { if (got < dlen) st = ZR_EOF; break; }
        if (r != LZMA_OK) { st = (r == 10 /*BUF_ERROR*/) ? ZR_EOF : ZR_INVALID_DATA; break; }
        if (eof && made == 0) { st = ZR_EOF; break; }
    }
    lzma_end(&s);
    return st;
}

/* DefaultChunkReader::read_chunk body (chunk.rs:270-286) on one stream:
 * dst receives exactly dlen = N*elem_size bytes in host-native order. */
int zref_decode(int codec, int elem_size, int big_endian, int is_bool, uint32_t flags,
                const uint8_t* src, uint64_t src_len, uint8_t* dst, uint64_t dlen) {
    if (dlen == 0) return ZR_OK; /* read_exact of an empty buffer never reads */
    int st;
    switch (codec) {
    case ZR_RAW:
        if (src_len < dlen) { /* read_exact copies what is there, then fails */
            memcpy(dst, src, src_len);
            return ZR_EOF;
        }
        memcpy(dst, src, dlen);
        st = ZR_OK;
        break;
    case ZR_GZIP: st = zr_decode_gzip(src, src_len, dst, dlen, flags & 1); break;
    case ZR_LZ4: st = zr_decode_lz4(src, src_len, dst, dlen); break;
    case ZR_BZIP2: st = zr_decode_bzip2(src, src_len, dst, dlen); break;
    case ZR_XZ: st = zr_decode_xz(src, src_len, dst, dlen); break;
    default: return ZR_INVALID_INPUT;
    }
    if (st == ZR_OK) zr_fix_elements(dst, dlen, elem_size, big_endian, is_bool);
    return st;
}

/* ---------------- encoders (write_chunk, chunk.rs:306-323) ------------ */
typedef struct { uint8_t* p; uint64_t n, cap; int overflow; } zr_sink;
static void sink_put(zr_sink* s, const void* d, uint64_t k) {
    if (s->n + k > s->cap) { s->overflow = 1; return; }
    memcpy(s->p + s->n, d, k);
    s->n += k;
}

/* flate2 write::GzEncoder with GzBuilder defaults: header
 * 1f 8b 08 00 | mtime 0 | XFL | OS 255, where XFL = 2 at level >= 9,
 * 4 at level <= 1, else 0 (pinned at level 6 by gzip.rs:66-80,95-96);
 * body = zlib raw deflate (windowBits -15, memLevel 8, default strategy);
 * trailer = CRC32 LE, ISIZE LE. */
static int zr_encode_gzip(int level, const uint8_t* b, uint64_t n, zr_sink* o) {
    int lvl = zref_effective_gzip_level(level);
    uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 255};
    hdr[8] = lvl >= 9 ? 2 : (lvl <= 1 ? 4 : 0);
    sink_put(o, hdr, 10);
    z_stream z;
    memset(&z, 0, sizeof z);
    if (deflateInit2(&z, lvl, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK)
        return ZR_INVALID_DATA;
    uint64_t bound = deflateBound(&z, (uLong)n) + 16;
    uint8_t* tmp = (uint8_t*)malloc(bound);
    z.next_in = (Bytef*)b;
    z.avail_in = (uInt)n;
    z.next_out = tmp;
    z.avail_out = (uInt)bound;
    int r = deflate(&z, Z_FINISH);
    uint64_t clen = bound - z.avail_out;
    deflateEnd(&z);
    if (r != Z_STREAM_END) { free(tmp); return ZR_INVALID_DATA; }
    sink_put(o, tmp, clen);
    free(tmp);
    uint32_t c = (uint32_t)crc32(0L, b, (uInt)n), sz = (uint32_t)n;
    uint8_t tr[8] = {c & 255, (c >> 8) & 255, (c >> 16) & 255, c >> 24,
                     sz & 255, (sz >> 8) & 255, (sz >> 16) & 255, sz >> 24};
    sink_put(o, tr, 8);
    return ZR_OK;
}

/* lz4-rs EncoderBuilder (lz.rs:85-92): level 0, Independent blocks, content
 * checksum on, no block checksum, no content size, autoFlush off; the
 * streaming API is fed `limit` = block-size bytes per LZ4F_compressUpdate. */
static int zr_encode_lz4(int block_size, const uint8_t* b, uint64_t n, zr_sink* o) {
    LZ4F_preferences_t p;
    memset(&p, 0, sizeof p);
    p.frameInfo.blockSizeID = zref_lz4_block_size_id(block_size);
    p.frameInfo.blockMode = 1;
    p.frameInfo.contentChecksumFlag = 1;
    static const size_t lim[8] = {0, 0, 0, 0, 65536, 262144, 1048576, 4194304};
    size_t limit = lim[p.frameInfo.blockSizeID];
    LZ4F_cctx* c = NULL;
    if (LZ4F_isError(LZ4F_createCompressionContext(&c, LZ4F_VERSION))) return ZR_INVALID_DATA;
    size_t cap = LZ4F_compressBound(limit, &p) + 64;
    uint8_t* buf = (uint8_t*)malloc(cap);
    int st = ZR_OK;
    size_t r = LZ4F_compressBegin(c, buf, cap, &p);
    if (LZ4F_isError(r)) st = ZR_INVALID_DATA; else sink_put(o, buf, r);
    for (uint64_t off = 0; st == ZR_OK && off < n; off += limit) {
        size_t k = (n - off) < limit ? (size_t)(n - off) : limit;
        r = LZ4F_compressUpdate(c, buf, cap, b + off, k, NULL);
        if (LZ4F_isError(r)) st = ZR_INVALID_DATA; else sink_put(o, buf, r);
    }
    if (st == ZR_OK) {
        r = LZ4F_compressEnd(c, buf, cap, NULL);
        if (LZ4F_isError(r)) st = ZR_INVALID_DATA; else sink_put(o, buf, r);
    }
    free(buf);
    LZ4F_freeCompressionContext(c);
    return st;
}

/* bzip2 write::BzEncoder::new(w, Compression::new(blockSize)) -> BZ2_bzCompressInit
 * (blockSize, verbosity 0, workFactor 30). */
static int zr_encode_bzip2(int block_size, const uint8_t* b, uint64_t n, zr_sink* o) {
    if (block_size < 1 || block_size > 9) return ZR_INVALID_INPUT;
    bz_stream s;
    memset(&s, 0, sizeof s);
    if (BZ2_bzCompressInit(&s, block_size, 0, 30) != BZ_OK) return ZR_INVALID_DATA;
    uint64_t cap = n + n / 50 + 1024;
    uint8_t* tmp = (uint8_t*)malloc(cap);
    s.next_in = (char*)b;
    s.avail_in = (unsigned)n;
    s.next_out = (char*)tmp;
    s.avail_out = (unsigned)cap;
    int r;
    do { r = BZ2_bzCompress(&s, BZ_FINISH); } while (r == BZ_FINISH_OK && s.avail_out);
    uint64_t clen = cap - s.avail_out;
    BZ2_bzCompressEnd(&s);
    if (r != BZ_STREAM_END) { free(tmp); return ZR_INVALID_DATA; }
    sink_put(o, tmp, clen);
    free(tmp);
    return ZR_OK;
}

/* xz2 write::XzEncoder::new(w, preset) -> lzma_easy_encoder(preset, CRC64). */
static int zr_encode_xz(int preset, const uint8_t* b, uint64_t n, zr_sink* o) {
    lzma_stream s;
    memset(&s, 0, sizeof s);
    if (lzma_easy_encoder(&s, (uint32_t)preset, LZMA_CHECK_CRC64) != LZMA_OK) return ZR_INVALID_INPUT;
    uint64_t cap = n + n / 16 + 4096;
    uint8_t* tmp = (uint8_t*)malloc(cap);
    s.next_in = b;
    s.avail_in = n;
    s.next_out = tmp;
    s.avail_out = cap;
    int r = lzma_code(&s, LZMA_FINISH);
    uint64_t clen = cap - s.avail_out;
    lzma_end(&s);
    if (r != LZMA_STREAM_END) { free(tmp); return ZR_INVALID_DATA; }
    sink_put(o, tmp, clen);
    free(tmp);
    return ZR_OK;
}

/* DefaultChunkWriter::write_chunk (chunk.rs:306-323).  `elems` holds the
 * chunk's elements in host-native order (n_elements of elem_size bytes);
 * write_data serialises them in the array's byte order (bool -> 0/1). */
int zref_encode(int codec, int param, int elem_size, int big_endian, int is_bool,
                const uint8_t* elems, uint64_t n_elements, uint64_t chunk_num_elements,
                uint8_t* out, uint64_t out_cap, uint64_t* out_len) {
    *out_len = 0;
    if (n_elements != chunk_num_elements) return ZR_INVALID_DATA; /* chunk.rs:309-318 */
    uint64_t nb = n_elements * (uint64_t)elem_size;
    uint8_t* ser = (uint8_t*)malloc(nb ? nb : 1);
    memcpy(ser, elems, nb);
    if (is_bool) {
        for (uint64_t i = 0; i < nb; i++) ser[i] = ser[i] != 0;
    } else {
        zr_fix_elements(ser, nb, elem_size, big_endian, 0);
    }
    zr_sink o = {out, 0, out_cap, 0};
    int st;
    switch (codec) {
    case ZR_RAW: sink_put(&o, ser, nb); st = ZR_OK; break;
    case ZR_GZIP: st = zr_encode_gzip(param, ser, nb, &o); break;
    case ZR_LZ4: st = zr_encode_lz4(param, ser, nb, &o); break;
    case ZR_BZIP2: st = zr_encode_bzip2(param, ser, nb, &o); break;
    case ZR_XZ: st = zr_encode_xz(param, ser, nb, &o); break;
    default: st = ZR_INVALID_INPUT;
    }
    free(ser);
    if (st == ZR_OK && o.overflow) st = ZR_TOO_SMALL;
    *out_len = o.n;
    return st;
}

/* ---------------- batch decode on a host thread pool (cpu_baseline) ---
 * One chunk per task, T worker threads (SURVEY §8(d) "CPU baseline").
 * srcs/dsts are host pointers; status receives one word per chunk. */
typedef struct {
    int codec, elem_size, big_endian, is_bool;
    uint32_t flags;
    const uint8_t* const* srcs;
    const uint64_t* src_lens;
    uint8_t* const* dsts;
    uint64_t dlen;
    int32_t* status;
    uint32_t n;
    volatile uint32_t next;
} zr_job;

static void* zr_worker(void* arg) {
    zr_job* j = (zr_job*)arg;
    for (;;) {
        uint32_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        j->status[i] = zref_decode(j->codec, j->elem_size, j->big_endian, j->is_bool, j->flags,
                                   j->srcs[i], j->src_lens[i], j->dsts[i], j->dlen);
    }
    return NULL;
}

int zref_decode_batch(int codec, int elem_size, int big_endian, int is_bool, uint32_t flags,
                      const uint8_t* const* srcs, const uint64_t* src_lens, uint8_t* const* dsts,
                      uint64_t dlen, uint32_t n, int32_t* status, int threads) {
    zr_job j = {codec, elem_size, big_endian, is_bool, flags, srcs, src_lens, dsts, dlen, status,
                n, 0};
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, zr_worker, &j);
    zr_worker(&j);
    for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* Batch encode on the same pool shape (C5's CPU baseline). */
typedef struct {
    int codec, param, elem_size, big_endian, is_bool;
    const uint8_t* const* srcs;
    uint64_t n_el;
    uint8_t* const* outs;
    uint64_t cap;
    uint64_t* out_lens;
    int32_t* status;
    uint32_t n;
    volatile uint32_t next;
} zr_ejob;

static void* zr_eworker(void* arg) {
    zr_ejob* j = (zr_ejob*)arg;
    for (;;) {
        uint32_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        j->status[i] = zref_encode(j->codec, j->param, j->elem_size, j->big_endian, j->is_bool,
                                   j->srcs[i], j->n_el, j->n_el, j->outs[i], j->cap,
                                   &j->out_lens[i]);
    }
    return NULL;
}

int zref_encode_batch(int codec, int param, int elem_size, int big_endian, int is_bool,
                      const uint8_t* const* srcs, uint64_t n_elements, uint8_t* const* outs,
                      uint64_t out_cap, uint64_t* out_lens, uint32_t n, int32_t* status,
                      int threads) {
    zr_ejob j = {codec, param, elem_size, big_endian, is_bool, srcs, n_elements, outs, out_cap,
                 out_lens, status, n, 0};
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, zr_eworker, &j);
    zr_eworker(&j);
    for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* ---------------- fixture helpers (test vectors only) -----------------
 * LZ4 frames with preferences the reference encoder never emits but the
 * reference decoder (LZ4F_decompress) accepts: linked blocks, block
 * checksums, content size, other block sizes, autoFlush (short blocks). */
int zref_lz4_frame_custom(int block_size_id, int linked, int content_checksum,
                          int block_checksum, int with_content_size, int auto_flush,
                          uint64_t feed, const uint8_t* b, uint64_t n, uint8_t* out,
                          uint64_t cap, uint64_t* out_len) {
    LZ4F_preferences_t p;
    memset(&p, 0, sizeof p);
    p.frameInfo.blockSizeID = block_size_id;
    p.frameInfo.blockMode = linked ? 0 : 1;
    p.frameInfo.contentChecksumFlag = content_checksum;
    p.frameInfo.blockChecksumFlag = block_checksum;
    p.frameInfo.contentSize = with_content_size ? n : 0;
    p.autoFlush = auto_flush;
    zr_sink o = {out, 0, cap, 0};
    LZ4F_cctx* c = NULL;
    if (LZ4F_isError(LZ4F_createCompressionContext(&c, LZ4F_VERSION))) return ZR_INVALID_DATA;
    if (feed == 0) feed = 65536;
    size_t bcap = LZ4F_compressBound(feed, &p) + 64;
    uint8_t* buf = (uint8_t*)malloc(bcap);
    int st = ZR_OK;
    size_t r = LZ4F_compressBegin(c, buf, bcap, &p);
    if (LZ4F_isError(r)) st = ZR_INVALID_DATA; else sink_put(&o, buf, r);
    for (uint64_t off = 0; st == ZR_OK && off < n; off += feed) {
        size_t k = (n - off) < feed ? (size_t)(n - off) : (size_t)feed;
        r = LZ4F_compressUpdate(c, buf, bcap, b + off, k, NULL);
        if (LZ4F_isError(r)) st = ZR_INVALID_DATA; else sink_put(&o, buf, r);
    }
    if (st == ZR_OK) {
        r = LZ4F_compressEnd(c, buf, bcap, NULL);
        if (LZ4F_isError(r)) st = ZR_INVALID_DATA; else sink_put(&o, buf, r);
    }
    free(buf);
    LZ4F_freeCompressionContext(c);
    *out_len = o.n;
    return (st == ZR_OK && o.overflow) ? ZR_TOO_SMALL : st;
}
