// zcg_lz4_dec.hip — Lz4Compression decode (src/compression/lz.rs:81-83,
// lz4-rs Decoder = LZ4F_decompress of liblz4 1.9.x) on gfx950.
//
// Layout / parallelism (one wave = one workgroup of 64 lanes):
//   * a wave owns G consecutive chunks (G = 64 / slots-per-chunk), lanes
//     0..G-1 parse the frame headers and walk the block headers of "their"
//     chunk into an LDS slot table (one slot per 64 KiB-or-larger block);
//   * every lane then decodes WHOLE BLOCKS, one block per lane (SIMT across
//     independent blocks): the LZ4 sequence parse is serial inside a block,
//     so the parallelism is across blocks, not inside one.  A 1 MiB chunk
//     written by the reference encoder (lz.rs:85-92: Independent 64 KiB
//     blocks) gives 16 blocks, so one wave decodes 4 chunks at a time;
//   * literal and match copies move 16 B per lane per access; matches with
//     offset < 16 expand their period in registers first;
//   * block k is placed at k*blockMax (LZ4F emits full blocks except the
//     last); a block that decodes short before the frame end, a linked-block
//     frame, or a frame needing more slots is re-decoded by one lane serially
//     with exact offsets (same code, exact placement) — correctness never
//     depends on the guess.
// Algorithmic bytes per chunk: C (compressed bytes read once) + D (decoded
// bytes written once).
//
// Error classification follows LZ4F_decodeHeader / LZ4_decompress_safe of
// lz4 1.9.3: bad magic/version/reserved bits/block size id/header checksum,
// block size > blockMax, block checksum mismatch, literal/match length
// overruns, offsets before the block (or frame, for linked blocks) start and
// matches ending in the last 5 bytes of the block capacity are INVALID_DATA;
// a frame whose data ends before N bytes is UNEXPECTED_EOF (after the
// content-size and content-checksum checks LZ4F's suffix stage makes).
// Offset 0 is accepted and yields zeros, as lz4 1.9.3 decodes it.
#include "zcg_common.h"

namespace zcg {

constexpr u32 LZ4_MAGIC = 0x184D2204u;
constexpr u32 LZ4_MIN_BMAX = 65536u;

enum : u32 { F_BLOCK_CKSUM = 1, F_LINKED = 2, F_FRAME_END = 4, F_TRUNC = 8, F_CONTENT_CKSUM = 16,
             F_CONTENT_SIZE = 32 };

struct Lz4Hdr {
    int st;       // header status
    u32 bmax;     // block max size
    u32 flags;    // F_*
    u32 hdr_len;  // bytes of the frame header
};

__device__ inline Lz4Hdr lz4_parse_header(const u8* s, u64 n) {
    Lz4Hdr h{ZCG_OK, 0, 0, 0};
    if (n < 4) { h.st = ZCG_ERR_UNEXPECTED_EOF; return h; }
    u32 magic = ld32(s);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame: LZ4F returns 0
        h.st = ZCG_ERR_UNEXPECTED_EOF;
        return h;
    }
    if (magic != LZ4_MAGIC) { h.st = ZCG_ERR_INVALID_DATA; return h; }
    if (n < 7) { h.st = ZCG_ERR_UNEXPECTED_EOF; return h; }
    u32 flg = s[4], bd = s[5];
    u32 hl = 7 + ((flg & 8) ? 8 : 0) + ((flg & 1) ? 4 : 0);
    if (n < hl) { h.st = ZCG_ERR_UNEXPECTED_EOF; return h; }
    if (((flg >> 6) & 3) != 1 || (flg & 2) || (bd & 0x8F)) { h.st = ZCG_ERR_INVALID_DATA; return h; }
    u32 id = (bd >> 4) & 7;
    if (id < 4) { h.st = ZCG_ERR_INVALID_DATA; return h; }
    u32 hc = (xxh32(s + 4, hl - 5, 0) >> 8) & 0xFF;
    if (hc != s[hl - 1]) { h.st = ZCG_ERR_INVALID_DATA; return h; }
    h.bmax = 1u << (8 + 2 * id);
    h.flags = ((flg & 0x10) ? F_BLOCK_CKSUM : 0) | ((flg & 0x20) ? 0 : F_LINKED) |
              ((flg & 0x04) ? F_CONTENT_CKSUM : 0) | ((flg & 0x08) ? F_CONTENT_SIZE : 0);
    h.hdr_len = hl;
    return h;
}

__device__ __forceinline__ u32 get_byte(const u32x4& w, u32 idx) {
    u32 d = idx < 4 ? w.x : (idx < 8 ? w.y : (idx < 12 ? w.z : w.w));
    return (d >> ((idx & 3) * 8)) & 0xFF;
}

// 16 bytes of the period-d pattern b[0..d) starting at phase `ph`.
__device__ __forceinline__ u32x4 pattern16(const u32x4& b, u32 d, u32 ph) {
    u32 r[4];
    u32 j = ph;  // ph < d
#pragma unroll
    for (int k = 0; k < 4; k++) {
        u32 v = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            v |= get_byte(b, j) << (8 * i);
            j = (j + 1 == d) ? 0 : j + 1;
        }
        r[k] = v;
    }
    return u32x4{r[0], r[1], r[2], r[3]};
}

// 16-byte register window over the compressed block: the token, length
// bytes and offset of a sequence come from registers, so a sequence costs one
// window load (prefetched before the previous match copy) instead of a chain
// of dependent byte loads.
__device__ __forceinline__ u32 win_byte(const u32x4& w, u32 d) {
    const u32 word = d < 8 ? (d < 4 ? w.x : w.y) : (d < 12 ? w.z : w.w);
    return (word >> ((d & 3) * 8)) & 0xFF;
}
// 16 bytes of the stream at q; bytes at or past `avail` read as 0
__device__ __forceinline__ u32x4 win_load(const u8* __restrict__ src, u64 q, u64 avail) {
    if (q + 16 <= avail) return ld16(src + q);
    u64 lo = 0, hi = 0;
    for (u32 k = 0; k < 16; k++) {
        const u64 b = (q + k < avail) ? (u64)src[q + k] : 0ull;
        if (k < 8) lo |= b << (8 * k);
        else hi |= b << (8 * (k - 8));
    }
    return u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
}
// w shifted down by d (< 16) bytes, zero fill
__device__ __forceinline__ u32x4 win_shift(const u32x4& w, u32 d) {
    u64 lo = ((u64)w.y << 32) | w.x, hi = ((u64)w.w << 32) | w.z;
    if (d >= 8) { lo = hi; hi = 0; d -= 8; }
    if (d) { lo = (lo >> (8 * d)) | (hi << (64 - 8 * d)); hi >>= 8 * d; }
    return u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
}
struct LzWin {  // 16 bytes of the stream at wb
    const u8* src;
    u64 avail;
    u32x4 w;
    u32 wb;
    __device__ __forceinline__ u32 byte(u32 q) {
        u32 d = q - wb;
        if (d >= 16) { w = win_load(src, q, avail); wb = q; d = 0; }
        return win_byte(w, d);
    }
    __device__ __forceinline__ void at(u32 q) { w = win_load(src, q, avail); wb = q; }
};

// Decode one LZ4 block (LZ4_decompress_safe semantics, capacity `cap`).
//   src/csize: compressed block;  src_avail: readable bytes from src
//   dst: chunk output base;  op0: output position of the block
//   lim: write limit (N*size); bytes at >= lim are parsed, never stored
//   low: lowest legal match source (block start, or frame start if linked)
__device__ int lz4_block(const u8* __restrict__ src, u32 csize, u64 src_avail, u8* dst, u64 op0,
                         u32 cap, u64 lim, u64 low, u32* out_n) {
    const u32 iend = csize;
    u32 ip = 0;
    u64 op = op0;
    const u64 oend = op0 + cap;
    const u64 wlim = oend < lim ? oend : lim;
    LzWin in{src, src_avail, u32x4{0, 0, 0, 0}, 0};
    in.at(0);
    for (;;) {
        if (ip >= iend) return ZCG_ERR_INVALID_DATA;
        const u32 token = in.byte(ip++);
        u32 lit = token >> 4;
        if (lit == 15) {
            if ((int64_t)ip >= (int64_t)iend - 15) return ZCG_ERR_INVALID_DATA;
            u32 s;
            do {
                s = in.byte(ip++);
                lit += s;
            } while (s == 255 && (int64_t)ip < (int64_t)iend - 15);
        }
        const u64 cpy = op + lit;
        if (cpy + 12 > oend || (int64_t)ip + lit > (int64_t)iend - 8) {
            // must be the last sequence: consume the input exactly
            if (ip + lit != iend || cpy > oend) return ZCG_ERR_INVALID_DATA;
            for (u32 i = 0; i < lit; i++)
                if (op + i < lim) dst[op + i] = src[ip + i];
            op = cpy;
            break;
        }
        // literals: from the window when they lie in it, else 16 B copies
        if (cpy + 16 <= wlim && (u64)ip + lit + 16 <= src_avail) {
            const u32 d = ip - in.wb;
            if (d < 16 && d + lit <= 16) {
                if (lit) st16(dst + op, win_shift(in.w, d));
            } else {
                for (u32 i = 0; i < lit; i += 16) st16(dst + op + i, ld16(src + ip + i));
            }
        } else {
            for (u32 i = 0; i < lit; i++)
                if (op + i < lim) dst[op + i] = src[ip + i];
        }
        ip += lit;
        op = cpy;
        // offset + match length
        const u32 off = in.byte(ip) | (in.byte(ip + 1) << 8);
        ip += 2;
        u32 ml = token & 15;
        if (ml == 15) {
            u32 s;
            do {
                s = in.byte(ip++);
                ml += s;
                if ((int64_t)ip >= (int64_t)iend - 4) return ZCG_ERR_INVALID_DATA;
            } while (s == 255);
        }
        ml += 4;
        if (op - low < off) return ZCG_ERR_INVALID_DATA;
        const u64 mend = op + ml;
        if (mend + 5 > oend) return ZCG_ERR_INVALID_DATA;
        // next sequence's window (token + offset + a few length bytes), in
        // flight during the match copy; kept when 8+ bytes of it remain
        if (ip - in.wb > 8) in.at(ip);
        u8* const d = dst + op;
        if (off == 0) {
            // lz4 1.9.3 accepts offset 0: LZ4_write32(op, 0) then copies the
            // match from itself, so the match bytes come out as zeros
            for (u32 i = 0; i < ml; i++)
                if (op + i < lim) dst[op + i] = 0;
        } else if (mend + 32 <= wlim) {
            if (off >= 16) {
                for (u32 i = 0; i < ml; i += 16) st16(d + i, ld16(d - off + i));
            } else {
                // period `off` pattern built in registers; then 16 B pieces at
                // distance D2 = smallest multiple of off >= 16 (<= 30 < 32).
                const u32x4 b = ld16(d - off);
                st16(d, pattern16(b, off, 0));
                st16(d + 16, pattern16(b, off, 16 % off));
                if (ml > 32) {
                    const u32 d2 = off * ((16 + off - 1) / off);
                    for (u32 i = 32; i < ml; i += 16) st16(d + i, ld16(d - d2 + i));
                }
            }
        } else {
            for (u32 i = 0; i < ml; i++)
                if (op + i < lim) dst[op + i] = dst[op + i - off];
        }
        op = mend;
    }
    *out_n = (u32)(op - op0);
    return ZCG_OK;
}

// LZ4F keeps going after the output is full when the block that filled it
// ended exactly at N: the next block header (fed to it together with the
// block's last bytes by lz4-rs) is read, and a size above blockMax is an
// error (LZ4F_ERROR_maxBlockSize_invalid).
__device__ __forceinline__ int lz4_next_header_check(const u8* s, u64 n, u64 pos, u32 bmax) {
    if (pos + 4 > n) return ZCG_OK;
    const u32 bs = ld32(s + pos);
    if (bs != 0 && (bs & 0x7FFFFFFFu) > bmax) return ZCG_ERR_INVALID_DATA;
    return ZCG_OK;
}

// Serial decode of a whole frame by one lane, exact output offsets.  Used for
// linked-block frames and whenever the per-block placement guess failed.
__device__ int lz4_frame_serial(const u8* s, u64 n, u8* dst, u64 D, u32 vflags) {
    Lz4Hdr h = lz4_parse_header(s, n);
    if (h.st != ZCG_OK) return h.st;
    u64 pos = h.hdr_len, out = 0;
    while (out < D) {
        if (pos + 4 > n) return ZCG_ERR_UNEXPECTED_EOF;
        const u32 bs = ld32(s + pos);
        pos += 4;
        if (bs == 0) {
            // end mark before N bytes: LZ4F's dstage_getSuffix still checks the
            // declared content size and the content checksum (lz4-rs feeds them)
            if (h.flags & F_CONTENT_SIZE) {
                const u64 declared = (u64)ld32(s + 6) | ((u64)ld32(s + 10) << 32);
                if (declared != out) return ZCG_ERR_INVALID_DATA;
            }
            if (h.flags & F_CONTENT_CKSUM) {
                if (pos + 4 > n) return ZCG_ERR_UNEXPECTED_EOF;
                if (xxh32(dst, out, 0) != ld32(s + pos)) return ZCG_ERR_INVALID_DATA;
            }
            return ZCG_ERR_UNEXPECTED_EOF;
        }
        const u32 cs = bs & 0x7FFFFFFFu;
        if (cs > h.bmax) return ZCG_ERR_INVALID_DATA;
        const u64 need = (u64)cs + ((h.flags & F_BLOCK_CKSUM) ? 4 : 0);
        if (pos + need > n) return ZCG_ERR_UNEXPECTED_EOF;
        if ((h.flags & F_BLOCK_CKSUM) && !(vflags & ZCG_FLAG_SKIP_LZ4_BLOCK_CHECKSUM)) {
            if (xxh32(s + pos, cs, 0) != ld32(s + pos + cs)) return ZCG_ERR_INVALID_DATA;
        }
        u32 got = 0;
        if (bs & 0x80000000u) {
            for (u32 i = 0; i < cs && out + i < D; i++) dst[out + i] = s[pos + i];
            got = cs;
        } else {
            const u64 low = (h.flags & F_LINKED) ? 0 : out;
            int st = lz4_block(s + pos, cs, n - pos, dst, out, h.bmax, D, low, &got);
            if (st != ZCG_OK) return st;
        }
        out += got;
        pos += need;
        if (out == D) return lz4_next_header_check(s, n, pos, h.bmax);
    }
    return ZCG_OK;
}

__global__ __launch_bounds__(64) void lz4_decode_kernel(const zcg_chunk* __restrict__ chunks,
                                                        u32 n, u64 D, DType t, u32 vflags, u32 G,
                                                        u32 S, i32* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) u8 smem[];
    // LDS carve: per slot 4 words, per chunk 4 words
    u32* slot_src = (u32*)smem;                  // [G*S] block data offset in src
    u32* slot_cs = slot_src + G * S;             // [G*S] raw block size word
    u32* slot_dec = slot_cs + G * S;             // [G*S] decoded size
    i32* slot_st = (i32*)(slot_dec + G * S);     // [G*S] block status
    u32* c_nslot = (u32*)(slot_st + G * S);      // [G]
    u32* c_bmax = c_nslot + G;                   // [G]
    u32* c_flags = c_bmax + G;                   // [G]
    i32* c_st = (i32*)(c_flags + G);             // [G] -1 = needs serial
    u32* c_jobbase = (u32*)(c_st + G);           // [G+1]

    const int lane = lane_id();
    const u32 c0 = blockIdx.x * G;

    // ---- phase 1: frame headers + block walk (lane j -> chunk c0+j) ------
    if ((u32)lane < G) {
        const u32 j = lane;
        const u32 c = c0 + j;
        u32 ns = 0, bmax = 0, fl = 0;
        int st = ZCG_OK;
        if (c < n && D > 0) {
            const zcg_chunk ch = chunks[c];
            const u8* s = (const u8*)ch.src;
            Lz4Hdr h = lz4_parse_header(s, ch.src_len);
            st = h.st;
            bmax = h.bmax;
            fl = h.flags;
            if (st == ZCG_OK && (fl & F_LINKED)) {
                st = -1;  // serial
            } else if (st == ZCG_OK) {
                u64 pos = h.hdr_len;
                while ((u64)ns * bmax < D) {
                    if (ns == S) { st = -1; break; }
                    if (pos + 4 > ch.src_len) { fl |= F_TRUNC; break; }
                    const u32 bs = ld32(s + pos);
                    if (bs == 0) { fl |= F_FRAME_END; break; }
                    const u32 cs = bs & 0x7FFFFFFFu;
                    if (cs > bmax) { st = ZCG_ERR_INVALID_DATA; break; }
                    const u64 need = (u64)cs + ((fl & F_BLOCK_CKSUM) ? 4 : 0);
                    if (pos + 4 + need > ch.src_len) { fl |= F_TRUNC; break; }
                    slot_src[j * S + ns] = (u32)(pos + 4);
                    slot_cs[j * S + ns] = bs;
                    ns++;
                    pos += 4 + need;
                }
                // peek at the header after the last walked block
                if (st == ZCG_OK && !(fl & (F_TRUNC | F_FRAME_END))) {
                    if (pos + 4 <= ch.src_len && ld32(s + pos) == 0) fl |= F_FRAME_END;
                }
            }
        } else if (c < n) {
            st = ZCG_OK;  // N == 0: read_exact of nothing
        }
        c_nslot[j] = (st == ZCG_OK) ? ns : 0;
        c_bmax[j] = bmax;
        c_flags[j] = fl;
        c_st[j] = st;
    }
    __syncthreads();
    if (lane == 0) {
        u32 acc = 0;
        for (u32 j = 0; j < G; j++) { c_jobbase[j] = acc; acc += c_nslot[j]; }
        c_jobbase[G] = acc;
    }
    __syncthreads();

    // ---- phase 2: one block per lane --------------------------------------
    const u32 njobs = c_jobbase[G];
    for (u32 job = lane; job < njobs; job += 64) {
        u32 j = 0;
        while (c_jobbase[j + 1] <= job) j++;
        const u32 k = job - c_jobbase[j];
        const zcg_chunk ch = chunks[c0 + j];
        const u8* s = (const u8*)ch.src;
        const u32 bmax = c_bmax[j];
        const u32 bs = slot_cs[j * S + k];
        const u32 cs = bs & 0x7FFFFFFFu;
        const u64 so = slot_src[j * S + k];
        const u64 op0 = (u64)k * bmax;
        u8* dst = (u8*)ch.dst;
        int st = ZCG_OK;
        u32 got = 0;
        if ((c_flags[j] & F_BLOCK_CKSUM) && !(vflags & ZCG_FLAG_SKIP_LZ4_BLOCK_CHECKSUM)) {
            if (xxh32(s + so, cs, 0) != ld32(s + so + cs)) st = ZCG_ERR_INVALID_DATA;
        }
        if (st == ZCG_OK) {
            if (bs & 0x80000000u) {
                const u64 lim = D - op0 < cs ? D - op0 : cs;
                for (u64 i = 0; i < lim; i += 16) {
                    if (i + 16 <= lim) st16(dst + op0 + i, ld16(s + so + i));
                    else for (u64 q = i; q < lim; q++) dst[op0 + q] = s[so + q];
                }
                got = cs;
            } else {
                st = lz4_block(s + so, cs, ch.src_len - so, dst, op0, bmax, D, op0, &got);
            }
        }
        slot_dec[j * S + k] = got;
        slot_st[j * S + k] = st;
    }
    __syncthreads();

    // ---- phase 3: per-chunk verdict; phase 4: serial fallback -------------
    if ((u32)lane < G && c0 + lane < n) {
        const u32 j = lane;
        int st = c_st[j];
        if (st == ZCG_OK && D > 0) {
            const u32 ns = c_nslot[j];
            const u32 bmax = c_bmax[j];
            u64 total = 0;
            for (u32 k = 0; k < ns; k++) {
                if (slot_st[j * S + k] != ZCG_OK) { st = slot_st[j * S + k]; break; }
                const u32 got = slot_dec[j * S + k];
                total = (u64)k * bmax + got;
                if (got != bmax && k + 1 < ns) { st = -1; break; }  // short block mid-frame
            }
            if (st == ZCG_OK && total == D && ns > 0) {  // last block ended exactly at N
                const zcg_chunk ch = chunks[c0 + j];
                const u32 k = ns - 1;
                const u64 pos = (u64)slot_src[j * S + k] + (slot_cs[j * S + k] & 0x7FFFFFFFu) +
                                ((c_flags[j] & F_BLOCK_CKSUM) ? 4 : 0);
                st = lz4_next_header_check((const u8*)ch.src, ch.src_len, pos, bmax);
            }
            if (st == ZCG_OK && total < D) {
                // frame ended / input ran out before N bytes; a short last
                // block followed by more blocks means the guess failed.
                if (c_flags[j] & F_TRUNC) st = ZCG_ERR_UNEXPECTED_EOF;
                else if (c_flags[j] & F_FRAME_END)  // suffix checks: exact serial path
                    st = (c_flags[j] & (F_CONTENT_CKSUM | F_CONTENT_SIZE)) ? -1 : ZCG_ERR_UNEXPECTED_EOF;
                else st = -1;
            }
        }
        if (st == -1) {
            const zcg_chunk ch = chunks[c0 + j];
            st = lz4_frame_serial((const u8*)ch.src, ch.src_len, (u8*)ch.dst, D, vflags);
        }
        c_st[j] = st;
        status[c0 + j] = st;
    }
    __syncthreads();

    // ---- phase 5: element transform ('>' types, bool) ---------------------
    if (t.swap || t.isbool) {
        __threadfence_block();
        for (u32 j = 0; j < G && c0 + j < n; j++)
            if (c_st[j] == ZCG_OK) wave_transform((u8*)chunks[c0 + j].dst, D, t);
    }
}

hipError_t launch_lz4_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                             int32_t* d_status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    u64 S = (D + LZ4_MIN_BMAX - 1) / LZ4_MIN_BMAX;
    if (S < 1) S = 1;
    if (S > 8192) return hipErrorInvalidValue;  // > 512 MiB chunks: not supported
    const u32 G = S >= 64 ? 1u : (u32)(64 / S);
    const size_t lds = (size_t)G * S * 16 + (size_t)G * 16 + (G + 1) * 4 + 16;
    const u32 grid = (n + G - 1) / G;
    hipLaunchKernelGGL(lz4_decode_kernel, dim3(grid), dim3(64), lds, s, d_chunks, n, D, t,
                       a->compression.flags, G, (u32)S, d_status);
    return hipGetLastError();
}

}  // namespace zcg
