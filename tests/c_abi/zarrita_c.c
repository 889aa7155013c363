/* A plain-C caller of the drop-in boundary reading a real hierarchy: the
 * reference's zarrita fixture (tests/data/zarrita.zr3, replayed by
 * tests/zarrita_compat.rs:30-46; a copy lives in tests/golden/zarrita), with no
 * Python and no hand-built descriptor:
 *   1. meta/root/seq/i2.array.json -> zcg_array_meta_from_json (ArrayMetadata's
 *      serde form, lib.rs:382-402)
 *   2. the chunk keys of the 2x2x2 grid -> zcg_chunk_key (get_chunk_key,
 *      storage.rs:109-127), joined to the store root (filesystem.rs:142-190)
 *   3. zcg_store_read_chunks: each file read under a shared flock (get(),
 *      filesystem.rs:201-210) and decoded on the GPU
 *   4. the 4x5x6 array assembled on the host from the C-order chunks (edge
 *      chunks overhang the array) and compared with arange(120), as
 *      zarrita_compat.rs:16-28 expects.
 * Usage: zarrita_c <store root> [device].  Prints "zarrita_c: ok". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zchunk_gpu.h"

static char* slurp(const char* path, uint64_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = (char*)malloc((size_t)n + 1);
    if (b && fread(b, 1, (size_t)n, f) != (size_t)n) { free(b); b = NULL; }
    fclose(f);
    if (b) { b[n] = 0; *len = (uint64_t)n; }
    return b;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: zarrita_c <store root> [device]\n"); return 2; }
    const char* root = argv[1];
    const int device = argc > 2 ? atoi(argv[2]) : 0;
    const char* array_path = "/seq/i2";
    char mpath[4096];
    snprintf(mpath, sizeof mpath, "%s/meta/root/seq/i2.array.json", root);
    uint64_t jlen = 0;
    char* json = slurp(mpath, &jlen);
    if (!json) { fprintf(stderr, "cannot read %s\n", mpath); return 2; }
    zcg_array_meta m;
    char err[256];
    int st = zcg_array_meta_from_json(json, jlen, &m, err, sizeof err);
    free(json);
    if (st != ZCG_OK) { fprintf(stderr, "array metadata: %d %s\n", st, err); return 1; }
    if (m.ndim != 3 || m.chunk_ndim != 3 || m.array.dtype.elem_size != 2 || m.array.compression.codec != ZCG_CODEC_GZIP) {
        fprintf(stderr, "unexpected metadata\n");
        return 1;
    }
    uint64_t grid[3], n = 1;
    for (int d = 0; d < 3; d++) {
        grid[d] = (m.shape[d] + m.chunk_shape[d] - 1) / m.chunk_shape[d];
        n *= grid[d];
    }
    const uint64_t N = m.array.chunk_num_elements;
    char** paths = (char**)calloc(n, sizeof(char*));
    void** dsts = (void**)calloc(n, sizeof(void*));
    int32_t* status = (int32_t*)calloc(n, sizeof(int32_t));
    uint64_t pos[3];
    for (uint64_t i = 0; i < n; i++) {
        pos[0] = i / (grid[1] * grid[2]);
        pos[1] = (i / grid[2]) % grid[1];
        pos[2] = i % grid[2];
        const uint64_t klen = zcg_chunk_key(array_path, m.separator, pos, 3, NULL, 0);
        char* key = (char*)malloc(klen + 1);
        zcg_chunk_key(array_path, m.separator, pos, 3, key, klen + 1);
        /* the store's get_path (filesystem.rs:151-190): root joined with the key */
        uint64_t plen = 0;
        if (zcg_store_path(root, key, NULL, 0, &plen) != ZCG_OK) { fprintf(stderr, "zcg_store_path(%s)\n", key); return 1; }
        paths[i] = (char*)malloc(plen + 1);
        if (zcg_store_path(root, key, paths[i], plen + 1, NULL) != ZCG_OK) return 1;
        free(key);
        dsts[i] = malloc(N * 2);
    }
    zcg_ctx* ctx = zcg_create(device);
    if (!ctx) { fprintf(stderr, "zcg_create(%d) failed\n", device); return 2; }
    st = zcg_store_read_chunks(ctx, &m.array, (uint32_t)n, (const char* const*)paths, dsts, status, 4);
    if (st != ZCG_OK) { fprintf(stderr, "zcg_store_read_chunks: %d %s\n", st, zcg_last_error(ctx)); return 1; }
    const uint64_t S0 = m.shape[0], S1 = m.shape[1], S2 = m.shape[2];
    const uint64_t C0 = m.chunk_shape[0], C1 = m.chunk_shape[1], C2 = m.chunk_shape[2];
    int16_t* out = (int16_t*)calloc(S0 * S1 * S2, sizeof(int16_t));
    int bad = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (status[i] != ZCG_OK) { fprintf(stderr, "%s: status %d\n", paths[i], status[i]); bad++; continue; }
        const uint64_t g0 = i / (grid[1] * grid[2]), g1 = (i / grid[2]) % grid[1], g2 = i % grid[2];
        const int16_t* c = (const int16_t*)dsts[i];
        for (uint64_t a = 0; a < C0; a++)
            for (uint64_t b = 0; b < C1; b++)
                for (uint64_t e = 0; e < C2; e++) {
                    const uint64_t x = g0 * C0 + a, y = g1 * C1 + b, z = g2 * C2 + e;
                    if (x < S0 && y < S1 && z < S2) out[(x * S1 + y) * S2 + z] = c[(a * C1 + b) * C2 + e];
                }
    }
    for (uint64_t i = 0; i < S0 * S1 * S2; i++)
        if (out[i] != (int16_t)i) { if (bad < 5) fprintf(stderr, "element %llu = %d\n", (unsigned long long)i, out[i]); bad++; }
    zcg_destroy(ctx);
    for (uint64_t i = 0; i < n; i++) { free(paths[i]); free(dsts[i]); }
    free(paths); free(dsts); free(status); free(out);
    if (bad) { printf("zarrita_c: %d mismatches\n", bad); return 1; }
    printf("zarrita_c: ok (%llu chunks, %s keys)\n", (unsigned long long)n, m.separator);
    return 0;
}
