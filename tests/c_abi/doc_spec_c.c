/* A plain-C caller of the drop-in boundary (include/zchunk_gpu.h), no ctypes:
 * decodes the reference's doc-spec chunk of every CompressionType with
 * zcg_read_chunk and encodes it again with zcg_write_chunk.
 *
 * The vectors are the reference's own test data (src/compression/{raw,gzip,lz,
 * bzip,xz}.rs TEST_CHUNK_I16_*, driven by src/tests.rs:120-159): a ">i2" chunk
 * of shape 1x2x3 holding 1..6.  Encode must be byte-exact for raw, gzip (with
 * flate2's OS byte 255, gzip.rs:90-101), lz4 and xz; bzip2's reference vector is
 * not libbz2's output (bzip.rs:83-84), so its stream must decode back instead.
 * Exit status 0 and "doc_spec_c: ok" on success.  Built by tests/c_abi/Makefile. */
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include "zchunk_gpu.h"

static const uint8_t RAW[] = {0x00, 0x01, 0x00, 0x02, 0x00, 0x03, 0x00, 0x04, 0x00, 0x05, 0x00, 0x06};
static const uint8_t GZIP[] = {0x1f, 0x8b, 0x08, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x63, 0x60, 0x64, 0x60, 0x62,
                               0x60, 0x66, 0x60, 0x61, 0x60, 0x65, 0x60, 0x03, 0x00, 0xaa, 0xea, 0x6d, 0xbf, 0x0c, 0x00,
                               0x00, 0x00};
static const uint8_t LZ4[] = {0x04, 0x22, 0x4d, 0x18, 0x64, 0x40, 0xa7, 0x0c, 0x00, 0x00, 0x80, 0x00, 0x01, 0x00, 0x02, 0x00,
                              0x03, 0x00, 0x04, 0x00, 0x05, 0x00, 0x06, 0x00, 0x00, 0x00, 0x00, 0x41, 0x37, 0x33, 0x08};
static const uint8_t BZIP2[] = {0x42, 0x5a, 0x68, 0x39, 0x31, 0x41, 0x59, 0x26, 0x53, 0x59, 0x02, 0x3e, 0x0d, 0xd2, 0x00,
                                0x00, 0x00, 0x40, 0x00, 0x7f, 0x00, 0x20, 0x00, 0x31, 0x0c, 0x01, 0x0d, 0x31, 0xa8, 0x73,
                                0x94, 0x33, 0x7c, 0x5d, 0xc9, 0x14, 0xe1, 0x42, 0x40, 0x08, 0xf8, 0x37, 0x48};
static const uint8_t XZ[] = {0xfd, 0x37, 0x7a, 0x58, 0x5a, 0x00, 0x00, 0x04, 0xe6, 0xd6, 0xb4, 0x46, 0x02, 0x00, 0x21, 0x01,
                             0x16, 0x00, 0x00, 0x00, 0x74, 0x2f, 0xe5, 0xa3, 0x01, 0x00, 0x0b, 0x00, 0x01, 0x00, 0x02, 0x00,
                             0x03, 0x00, 0x04, 0x00, 0x05, 0x00, 0x06, 0x00, 0x0d, 0x03, 0x09, 0xca, 0x34, 0xec, 0x15, 0xa7,
                             0x00, 0x01, 0x24, 0x0c, 0xa6, 0x18, 0xd8, 0xd8, 0x1f, 0xb6, 0xf3, 0x7d, 0x01, 0x00, 0x00, 0x00,
                             0x00, 0x04, 0x59, 0x5a};

struct vec {
    const char* name;
    int32_t codec;
    const uint8_t* bytes;
    uint64_t len;
    int encode_exact;
};

int main(int argc, char** argv) {
    int device = argc > 1 ? atoi(argv[1]) : 0;
    if (zcg_abi_version() != ZCG_ABI_VERSION) { fprintf(stderr, "ABI version mismatch\n"); return 2; }
    zcg_ctx* ctx = zcg_create(device);
    if (!ctx) { fprintf(stderr, "zcg_create(%d) failed\n", device); return 2; }
    const struct vec vs[] = {{"raw", ZCG_CODEC_RAW, RAW, sizeof RAW, 1},
                             {"gzip", ZCG_CODEC_GZIP, GZIP, sizeof GZIP, 1},
                             {"lz4", ZCG_CODEC_LZ4, LZ4, sizeof LZ4, 1},
                             {"bzip2", ZCG_CODEC_BZIP2, BZIP2, sizeof BZIP2, 0},
                             {"xz", ZCG_CODEC_XZ, XZ, sizeof XZ, 1}};
    int bad = 0;
    for (size_t i = 0; i < sizeof vs / sizeof vs[0]; i++) {
        zcg_array a;
        memset(&a, 0, sizeof a);
        a.compression.codec = vs[i].codec;
        a.compression.gzip_level = -1;        /* GzipCompression::default (gzip.rs:37-47) */
        a.compression.lz4_block_size = 65536; /* lz.rs:68-70 */
        a.compression.bzip2_block_size = 9;   /* bzip.rs:23-25 */
        a.compression.xz_preset = 6;          /* xz.rs:22-24 */
        a.dtype.elem_size = 2;
        a.dtype.big_endian = 1; /* ">i2" (tests.rs:120-130) */
        a.chunk_num_elements = 6;
        int16_t out[6] = {0};
        int st = zcg_read_chunk(ctx, &a, vs[i].bytes, vs[i].len, out);
        for (int k = 0; k < 6 && st == ZCG_OK; k++)
            if (out[k] != k + 1) st = -1;
        if (st != ZCG_OK) { fprintf(stderr, "%s: decode status %d (%s)\n", vs[i].name, st, zcg_last_error(ctx)); bad++; continue; }
        const int16_t vals[6] = {1, 2, 3, 4, 5, 6};
        uint8_t enc[4096];
        uint64_t elen = 0;
        st = zcg_write_chunk(ctx, &a, vals, 6, enc, sizeof enc, &elen);
        if (st != ZCG_OK) { fprintf(stderr, "%s: encode status %d\n", vs[i].name, st); bad++; continue; }
        if (vs[i].codec == ZCG_CODEC_GZIP && elen > 9) enc[9] = 0; /* the reference test's OS-byte fudge (gzip.rs:90-101) */
        if (vs[i].encode_exact) {
            if (elen != vs[i].len || memcmp(enc, vs[i].bytes, elen) != 0) { fprintf(stderr, "%s: encode differs\n", vs[i].name); bad++; }
        } else {
            int16_t back[6] = {0};
            st = zcg_read_chunk(ctx, &a, enc, elen, back);
            if (st != ZCG_OK || memcmp(back, vals, sizeof vals) != 0) { fprintf(stderr, "%s: re-decode failed\n", vs[i].name); bad++; }
        }
        /* the write-side element-count check (chunk.rs:309-318) */
        if (zcg_write_chunk(ctx, &a, vals, 5, enc, sizeof enc, &elen) != ZCG_ERR_INVALID_DATA) { fprintf(stderr, "%s: count check\n", vs[i].name); bad++; }
        /* a short stream is UnexpectedEof (tests.rs:191-219) for raw */
        if (vs[i].codec == ZCG_CODEC_RAW && zcg_read_chunk(ctx, &a, RAW, 10, out) != ZCG_ERR_UNEXPECTED_EOF) { fprintf(stderr, "raw: short\n"); bad++; }
    }
    zcg_destroy(ctx);
    if (bad) return 1;
    printf("doc_spec_c: ok\n");
    return 0;
}
