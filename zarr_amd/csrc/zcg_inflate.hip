// zcg_inflate.hip — GzipCompression decode (src/compression/gzip.rs:49-52,
// flate2 read::GzDecoder over zlib raw inflate) on gfx950.
//
// Version 1 structure: one wave (64 lanes) per chunk.
//   * the gzip member header is parsed as flate2 does (magic, CM=8, FEXTRA,
//     FNAME, FCOMMENT, FHCRC verified), then RFC 1951 blocks are decoded;
//   * Huffman tables live in LDS: a 2^10-entry literal/length table and a
//     2^8-entry distance table, each entry one u32 (length, kind, extra bits,
//     value); codes longer than the table width take a canonical bit-serial
//     slow path (rare by construction: probability < 2^-10);
//   * the whole 32 KiB LZ77 window is an LDS ring, so every match source is
//     read from LDS; match bytes are copied by up to 64 lanes per round
//     (rounds of min(dist,64) bytes keep overlapping matches exact);
//   * decoded bytes leave the ring in 16 KiB element-aligned slabs with
//     16 B/lane coalesced stores, the '>'-type byte reversal / bool rule
//     fused into the store;
//   * decoding stops as soon as N*size bytes exist (read_exact, chunk.rs:
//     112-113): the CRC32/ISIZE trailer is not consulted on a full read,
//     exactly like flate2 (parity contract).
// The Huffman symbol decode is a wave-uniform serial chain; its throughput is
// bounded by scalar issue, not HBM.  DESIGN.md quantifies the bound.
#include "zcg_inflate_common.h"

namespace zcg {

__global__ __launch_bounds__(64) void inflate_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                     u64 D, DType t, u32 vflags,
                                                     i32* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) u8 ring[INF_RING];
    __shared__ u32 ltab[INF_LTAB];
    __shared__ u32 dtab[INF_DTAB];
    __shared__ HuffLds lh, dh;
    __shared__ u8 lens[320];
    __shared__ u32 bcache[BI_CACHE_WORDS];

    const u32 c = blockIdx.x;
    if (c >= n) return;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    int st = ZCG_OK;
    if (D == 0) { if (lane == 0) status[c] = ZCG_OK; return; }
    if (ch.dst_cap < D) { if (lane == 0) status[c] = ZCG_ERR_INVALID_INPUT; return; }

    const u8* s = (const u8*)ch.src;
    const u64 n_in = ch.src_len;
    u64 h = 0;
    st = gzip_header(s, n_in, &h);
    if (st != ZCG_OK) { if (lane == 0) status[c] = st; return; }

    BitIn b;
    bi_init(b, s + h, n_in - h, bcache);
    InfOut o{ring, 0, 0, (u8*)ch.dst, D, t};
    bool last = false;
    bool boundary = false;  // output filled exactly at a symbol boundary
    bool after_stored = false;
    int r = R_OK;
    while (r == R_OK && o.P < D) {
        if (last) { r = R_EXHAUSTED; break; }  // stream ended before N bytes
        u32 type = 0, slen = 0;
        r = read_block_header(b, &last, &type, &slen, lens, &lh, ltab, &dh, dtab);
        if (r != R_OK) break;
        if (type == 0) {  // stored: drain whole bytes of the bit buffer, then copy
            u32 done = 0;
            while (done < slen && b.cnt >= 8 && o.P < D) {
                if (!bi_has(b, 8)) { r = R_EXHAUSTED; break; }
                put_lit(o, bi_bits(b, 8));
                done++;
                inf_maybe_flush(o);
            }
            if (r != R_OK) break;
            if (done < slen && o.P < D) {
                u64 in0 = b.consumed >> 3;  // bit buffer is byte aligned and empty here
                while (done < slen && o.P < D) {
                    u32 k = slen - done;
                    const u64 room = INF_FLUSH - (o.P - o.F);
                    if (k > room) k = (u32)room;
                    if (k > 64 * 64) k = 64 * 64;
                    if ((u64)k > D - o.P) k = (u32)(D - o.P);
                    if (in0 + k > b.n) { r = R_EXHAUSTED; break; }
                    for (u32 i = lane; i < k; i += 64)
                        ring[(o.P + i) & (INF_RING - 1)] = b.src[in0 + i];
                    __builtin_amdgcn_wave_barrier();
                    o.P += k; in0 += k; done += k;
                    inf_maybe_flush(o);
                }
                bi_seek(b, in0 * 8);
            }
            boundary = (done == slen);
            after_stored = true;
            continue;
        }
        // ---- Huffman block body ---------------------------------------------
        after_stored = false;
        for (;;) {
            if (o.P >= D) { boundary = true; break; }
            u32 e;
            r = decode_sym(b, ltab, INF_LBITS, &e);
            if (r != R_OK) break;
            const u32 kind = (e >> 24) & 15;
            if (kind == K_LIT) {
                put_lit(o, e & 0xFF);
            } else if (kind == K_LEN) {
                const u32 ex = (e >> 16) & 0xFF;
                if (!bi_has(b, ex)) { r = R_EXHAUSTED; break; }
                u32 len = (e & 0xFFFF) + (ex ? bi_bits(b, ex) : 0);
                u32 de;
                r = decode_sym(b, dtab, INF_DBITS, &de);
                if (r != R_OK) break;
                if (((de >> 24) & 15) != K_DIST) { r = R_INVALID; break; }
                const u32 dex = (de >> 16) & 0xFF;
                if (!bi_has(b, dex)) { r = R_EXHAUSTED; break; }
                const u32 dist = (de & 0xFFFF) + (dex ? bi_bits(b, dex) : 0);
                if (dist > o.P) { r = R_INVALID; break; }  // "invalid distance too far back"
                if (o.P + len > D) {  // MATCH leaves with left == 0: no look-ahead
                    put_match(o, (u32)(D - o.P), dist);
                    boundary = false;
                    break;
                }
                put_match(o, len, dist);
            } else if (kind == K_EOB) {
                break;
            } else {
                r = R_INVALID;
                break;
            }
            inf_maybe_flush(o);
        }
    }
    if (r == R_OK && o.P >= D && boundary) {
        // look-ahead bounded by the 32 KiB window holding the last consumed bit
        const u64 last_byte = h + (b.consumed ? (b.consumed - 1) / 8 : 0);
        u64 wend = (last_byte / 32768 + 1) * 32768;
        if (wend > n_in) wend = n_in;
        b.limit = (wend - h) * 8;
        if (b.limit >= b.consumed) {
            int la = inf_lookahead(b, last, after_stored, lens, &lh, ltab, &dh, dtab);
            if (la == R_INVALID) r = R_INVALID;
        }
    }
    if (r == R_INVALID) st = ZCG_ERR_INVALID_DATA;
    else if (r == R_EXHAUSTED || o.P < D) st = ZCG_ERR_UNEXPECTED_EOF;
    if (st == ZCG_OK) {
        while (D - o.F > INF_FLUSH) inf_flush(o, o.F + INF_FLUSH);
        inf_flush(o, D);
    }
    if (lane == 0) status[c] = st;
}

hipError_t launch_inflate(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                          int32_t* d_status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    hipLaunchKernelGGL(inflate_kernel, dim3(n), dim3(64), 0, s, d_chunks, n, D, t,
                       a->compression.flags, d_status);
    return hipGetLastError();
}

}  // namespace zcg
