// zcg_lz4_dec.hip — Lz4Compression decode (src/compression/lz.rs:81-83,
// lz4-rs Decoder = LZ4F_decompress of liblz4 1.9.x) on gfx950.
//
// Three launches per batch (workspace: a 16-byte record per chunk and per
// block slot):
//   1. lz4_frames_kernel — one lane per chunk parses the frame header and
//      walks the block headers into the slot table (block k of a frame is
//      placed at k*blockMax: LZ4F emits full blocks except the last);
//   2. lz4_blocks_kernel — ONE WAVE PER BLOCK (lz4-rs writes independent
//      blocks, lz.rs:88), four blocks per 256-thread workgroup.  The block is
//      decoded in steps over 64-byte windows of the compressed stream: every
//      lane parses a sequence speculatively at its own byte, pointer doubling
//      over the lanes' next-sequence offsets finds the true chain, a DPP
//      prefix sum places the sequences' output, the step's bytes are produced
//      byte-parallel into the wave's 4 KiB LDS ring (a byte, or a pointer to
//      an earlier byte), resolved, and stored with coalesced dword stores.
//      Long sequences go one at a time (section 2 below); stored blocks are
//      a coalesced 16 B/lane copy;
//   3. lz4_finish_kernel — one wave per chunk: per-chunk verdict from the
//      slots, LZ4F's look-ahead at the next block header, the exact serial
//      fallback (linked-block frames, a short block mid-frame, frames that
//      end before N), and the element transform ('>' types, bool).
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


// ---- slot table (workspace) -------------------------------------------
struct Lz4ChunkInfo {
    i32 st;      // header status; -1 = needs the serial path
    u32 nslot;   // blocks walked into the slot table
    u32 bmax;    // block maximum size
    u32 flags;   // F_*
};
struct Lz4Slot {
    u32 src_off;  // block data offset in the stream
    u32 bs;       // raw block size word (MSB = stored)
    u32 got;      // decoded bytes
    i32 st;       // block status
};

// 1. frame header + block walk, one lane per chunk
__global__ __launch_bounds__(256) void lz4_frames_kernel(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                         u32 S, Lz4ChunkInfo* __restrict__ info,
                                                         Lz4Slot* __restrict__ slots) {
    const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    u32 ns = 0, bmax = 0, fl = 0;
    int st = ZCG_OK;
    if (D > 0) {
        const zcg_chunk ch = chunks[c];
        const u8* s = (const u8*)ch.src;
        const Lz4Hdr h = lz4_parse_header(s, ch.src_len);
        st = h.st;
        bmax = h.bmax;
        fl = h.flags;
        if (st == ZCG_OK && (fl & F_LINKED)) {
            st = -1;  // serial
        } else if (st == ZCG_OK) {
            u64 pos = h.hdr_len;
            Lz4Slot* sl = slots + (u64)c * S;
            while ((u64)ns * bmax < D) {
                if (ns == S) { st = -1; break; }
                if (pos + 4 > ch.src_len) { fl |= F_TRUNC; break; }
                const u32 bs = ld32(s + pos);
                if (bs == 0) { fl |= F_FRAME_END; break; }
                const u32 cs = bs & 0x7FFFFFFFu;
                if (cs > bmax) { st = ZCG_ERR_INVALID_DATA; break; }
                const u64 need = (u64)cs + ((fl & F_BLOCK_CKSUM) ? 4 : 0);
                if (pos + 4 + need > ch.src_len) { fl |= F_TRUNC; break; }
                sl[ns].src_off = (u32)(pos + 4);
                sl[ns].bs = bs;
                ns++;
                pos += 4 + need;
            }
            // peek at the header after the last walked block
            if (st == ZCG_OK && !(fl & (F_TRUNC | F_FRAME_END))) {
                if (pos + 4 <= ch.src_len && ld32(s + pos) == 0) fl |= F_FRAME_END;
            }
        }
    }
    info[c] = Lz4ChunkInfo{st, st == ZCG_OK ? ns : 0u, bmax, fl};
}

// ---- 2. one wave per block ----------------------------------------------
// LZ4_decompress_safe of one independent block by one wave, in steps over
// 64-byte windows of the compressed stream:
//   * every lane parses a sequence speculatively at its own window byte
//     (token, length bytes and offset from one 16-byte load), giving the
//     offset of the next sequence;
//   * the true chain through the window (it starts at the window's first
//     byte) comes from pointer doubling over those offsets: lane k finds the
//     chain's k-th sequence with five ds_bpermute lookups, no serial walk;
//   * a wave prefix sum (DPP) places the sequences' output; LZ4's output-side
//     checks run per sequence;
//   * the step's output bytes are produced byte-parallel into a per-wave LDS
//     ring of 16-bit entries (a byte, or a pointer to an earlier byte of the
//     same step), the pointers are resolved (they point strictly backward),
//     and the bytes are stored to HBM with dword stores.  Match sources older
//     than the ring come from the block's HBM output behind a workgroup fence.
// Long sequences (> LZ_LIGHT bytes) go one at a time, LZ_ROUND bytes per round.
// Positions are block-relative.
enum : u32 { K_NORMAL = 0, K_LAST = 1, K_ERR = 2 };
constexpr u32 LZ_LIGHT = 32;
constexpr u32 LZ_RING = 2048;  // 16-bit entries per wave
constexpr u32 LZ_RMASK = LZ_RING - 1;
constexpr u32 LZ_ROUND = 1024;
constexpr u32 LZ_PTR = 0x8000u;

__device__ __forceinline__ u32x4 gwin_load(const gu8* __restrict__ src, u32 q, u64 avail) {
    if (q + 16 <= avail) return *(const gu32x4_ua*)(src + q);
    u64 lo = 0, hi = 0;
    for (u32 k = 0; k < 16; k++) {
        const u64 b = (q + k < avail) ? (u64)src[q + k] : 0ull;
        if (k < 8) lo |= b << (8 * k);
        else hi |= b << (8 * (k - 8));
    }
    return u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
}

// One LZ4 sequence parsed at block offset x (LZ4_decompress_safe's input-side
// rules; the output-side rules need the output position and are applied
// after the prefix sum).  Speculative: x need not be a true sequence start.
struct LzSeq {
    u32 kind;  // K_NORMAL, K_LAST (literals up to the block end), K_ERR
    u32 adv;   // bytes to the next sequence (K_NORMAL)
    u32 lit, lo, off, ml;  // literal count, literal start - x, offset, match length
};

// the 16 stream bytes at e + lane for every lane of the wave (wave-uniform bounds test)
__device__ __forceinline__ u32x4 gwin_wave(const gu8* __restrict__ src, u32 e, u64 avail) {
    const u32 lane = (u32)lane_id();
    if ((u64)e + 80 <= avail) return *(const gu32x4_ua*)(src + e + lane);
    return gwin_load(src, e + lane, avail);
}

// w: the 16 stream bytes at x
__device__ __forceinline__ LzSeq lz4_seq_at(const gu8* __restrict__ s, u32 iend, const u32x4& w, u32 x) {
    LzSeq q{K_ERR, 0, 0, 0, 0, 0};
    if (x >= iend) return q;  // no token left: LZ4_decompress_safe's `ip >= iend` error
    auto B = [&](u32 p) -> u32 {
        const u32 d = p - x;
        return d < 16 ? win_byte(w, d) : (u32)s[p];
    };
    const u32 tok = win_byte(w, 0);
    u32 lit = tok >> 4;
    u32 ip = x + 1;
    const int ie = (int)iend;
    if (lit == 15) {
        if ((int)ip >= ie - 15) return q;
        u32 b;
        do {
            b = B(ip++);
            lit += b;
        } while (b == 255 && (int)ip < ie - 15);
    }
    q.lit = lit;
    q.lo = ip - x;
    if ((i64)ip + lit > (i64)ie - 8) {  // must be the last sequence: consume the input exactly
        q.kind = ((u64)ip + lit == iend) ? K_LAST : K_ERR;
        return q;
    }
    ip += lit;
    q.off = B(ip) | (B(ip + 1) << 8);
    ip += 2;
    u32 ml = tok & 15;
    if (ml == 15) {
        u32 b;
        do {
            b = B(ip++);
            ml += b;
            if ((int)ip >= ie - 4) return q;
        } while (b == 255);
    }
    q.ml = ml + 4;
    q.kind = K_NORMAL;
    q.adv = ip - x;
    return q;
}

// inclusive prefix sum over the wave: DPP row shifts within each 16-lane row,
// then the row totals broadcast down (row_bcast:15 into rows 1 and 3,
// row_bcast:31 into rows 2 and 3)
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

struct LzRing {
    u16* r;           // this wave's ring (LDS)
    const gu8* s;     // compressed block
    gu8* dst;         // the block's output
    u32 lim;          // stored bytes of the block (N*size clips the last block)
    u32 fenced;       // HBM output below this position is visible to the wave's loads

    // entry of output byte j of a sequence at o (lit literals from the stream
    // at lsrc, then match bytes at distance off), in a round [rb, rb+rn)
    __device__ __forceinline__ u32 entry(u32 o, u32 lsrc, u32 lit, u32 off, u32 j, u32 rb, u32 rn) const {
        if (j < lit) return s[lsrc + j];
        if (off == 0) return 0;  // lz4 1.9.3 decodes offset 0 to zeros
        u32 m = j - lit;
        if (m >= off) m %= off;
        const u32 src = o + lit - off + m;  // < the byte itself
        if (src >= rb) return LZ_PTR | (src & LZ_RMASK);
        if (src + LZ_RING >= rb + rn) return r[src & LZ_RMASK];
        return dst[src];
    }
    // resolve [rb, rb+rn) (4 bytes per lane per pass) and store it to HBM
    __device__ __forceinline__ void finish(u32 rb, u32 rn) {
        const u32 lane = (u32)lane_id();
        for (u32 i0 = lane * 4; i0 < rn; i0 += 256) {
            u32 v[4];
#pragma unroll
            for (u32 t = 0; t < 4; t++) v[t] = i0 + t < rn ? r[(rb + i0 + t) & LZ_RMASK] : 0u;
            u32 wasp = 0;
#pragma unroll
            for (u32 t = 0; t < 4; t++) {
                if (v[t] & LZ_PTR) {
                    wasp |= 1u << t;
                    do { v[t] = r[v[t] & LZ_RMASK]; } while (v[t] & LZ_PTR);
                }
            }
            if (wasp) {
#pragma unroll
                for (u32 t = 0; t < 4; t++)
                    if (wasp & (1u << t)) r[(rb + i0 + t) & LZ_RMASK] = (u16)v[t];
            }
            const u32 wv = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
            const u32 p = rb + i0;
            if (i0 + 4 <= rn && p + 4 <= lim) {
                *(gu32*)(dst + p) = wv;  // unaligned dword store (gfx950 allows it)
            } else {
                for (u32 t = 0; t < 4 && i0 + t < rn; t++)
                    if (p + t < lim) dst[p + t] = (u8)(wv >> (8 * t));
            }
        }
    }
    // make HBM output below `need` visible before a round reads it
    __device__ __forceinline__ void need_visible(u32 need, u32 op) {
        if (need > fenced) {
            __threadfence_block();
            fenced = op;
        }
    }
};

#ifndef LZ_DBG
#define LZ_DBG 0  // 1: the wave decoder's debug counters compiled in (tools/lz4_stats.py)
#endif
// Debug counters (flag ZCG_FLAG_DEBUG_COUNTERS; LZ_DBG builds), summed over all blocks:
// steps, heavy steps, bytes, cycles of parse / chain / entries / finish / total.
__device__ unsigned long long g_lz_dbg[16];
extern "C" int zcg__debug_lz4_counters(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lz_dbg), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_lz_dbg), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

//   s/iend: the compressed block; avail: readable bytes from s
//   dst: the block's output; cap: blockMax; lim: bytes of the block below N*size
__device__ void lz4_block_wave(const gu8* __restrict__ s, u32 iend, u64 avail, gu8* dst, u32 cap, u32 lim,
                               u16* ring, bool dbg, u32* got_out, int* st_out) {
    const u32 lane = (u32)lane_id();
    u64 dc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // steps, heavy, -, parse, chain, entries, finish, total
    u64 tp = dbg ? __builtin_readcyclecounter() : 0;
    const u64 tstart = tp;
#define LZ_T(slot)                                              \
    if (dbg) {                                                  \
        const u64 _t = __builtin_readcyclecounter();            \
        dc[slot] += _t - tp;                                    \
        tp = _t;                                                \
    }
    LzRing R{ring, s, dst, lim, 0};
    u32 e = 0;   // block offset of the window's first (true) sequence
    u32 op = 0;  // output position
    int st = ZCG_OK;
    u32x4 w = gwin_wave(s, 0, avail);  // this window's stream bytes (lane l: e + l ..)
    for (;;) {
        const LzSeq q = lz4_seq_at(s, iend, w, e + lane);
        dc[0]++;
        LZ_T(3)
        // chain by pointer doubling: J^(2^b)(x) for x < 64; values >= 64 are
        // exits (a next sequence beyond the window), 255 a terminal sequence
        const u32 nx = q.kind == K_NORMAL ? lane + q.adv : 0xFFFFFFFFu;  // next sequence (window offset)
        const u32 j1 = nx < 64 ? nx : (nx == 0xFFFFFFFFu ? 255u : 64u);
        u32 jt[5];
        jt[0] = j1;
#pragma unroll
        for (int b = 1; b < 5; b++) {
            const u32 y = (u32)__shfl((int)jt[b - 1], (int)(jt[b - 1] & 63));
            jt[b] = jt[b - 1] < 64 ? y : jt[b - 1];
        }
        u32 pos = 0;  // lane k: the chain's k-th sequence (k < 32)
#pragma unroll
        for (int b = 0; b < 5; b++) {
            const u32 y = (u32)__shfl((int)jt[b], (int)(pos & 63));
            if (((lane >> b) & 1) && pos < 64) pos = y;
        }
        const bool valid = lane < 32 && pos < 64;
        const u32 nseq = (u32)__builtin_popcountll(__ballot(valid));
        // the sequence after the last one in the window: an exit offset, or 255
        const u32 last_next = (u32)__builtin_amdgcn_readlane((int)__shfl((int)nx, (int)(pos & 63)), (int)(nseq - 1));
        const bool term = last_next == 0xFFFFFFFFu;
        const u32x4 wn = gwin_wave(s, term ? e : e + last_next, avail);  // next window, in flight during the copies
        // gather the k-th sequence's fields
        const u32 sp = pos & 63;
        // (every shuffle runs on all lanes: a bpermute reads 0 from lanes outside EXEC)
        const u32 gkind = (u32)__shfl((int)q.kind, (int)sp);
        const u32 kkind = valid ? gkind : (u32)K_NORMAL;
        const u32 klit = (u32)__shfl((int)q.lit, (int)sp);
        const u32 kml = (u32)__shfl((int)q.ml, (int)sp);
        const u32 koff = (u32)__shfl((int)q.off, (int)sp);
        const u32 klo = (u32)__shfl((int)q.lo, (int)sp);
        const bool norm = valid && kkind == K_NORMAL;
        const u32 len = valid && kkind != K_ERR ? klit + (norm ? kml : 0u) : 0u;
        const u32 incl = wave_incl_scan(len);
        const u32 total = (u32)__builtin_amdgcn_readlane((int)incl, 63);
        const u32 excl = incl - len;
        const u32 o = op + excl;
        // the output-side rules of LZ4_decompress_safe (u64: lengths may be huge on corrupt input)
        bool err = false;
        if (valid) {
            const u64 cpy = (u64)o + klit;
            if (kkind == K_ERR) err = true;
            else if (kkind == K_LAST) err = cpy > cap;
            else err = (cpy + 12 > cap) || (cpy < koff) || (cpy + kml + 5 > cap);
        }
        if (__ballot(err)) { st = ZCG_ERR_INVALID_DATA; break; }
        const u32 koffn = norm ? koff : 0u;
        const u32 klsrc = e + sp + klo;
        const bool heavy = __ballot(valid && len > LZ_LIGHT) != 0;
        LZ_T(4)
        if (!heavy && total <= LZ_ROUND) {
            // one round, byte-parallel: byte i belongs to the last k with excl_k <= i
            const u32 pk = klit | ((klsrc - e) << 6) | (koffn << 16);  // lit <= 32, klsrc - e <= 66
            R.need_visible(op + total > LZ_RING ? op + total - LZ_RING : 0, op);
            for (u32 i0 = 0; i0 < total; i0 += 64) {  // wave-uniform: every lane takes part in the shuffles
                const u32 i = i0 + lane;
                u32 r = 0;
#pragma unroll
                for (u32 stp = 16; stp; stp >>= 1) {
                    const u32 c = r + stp;
                    const u32 oc = (u32)__shfl((int)excl, (int)(c & 63));
                    if (c < nseq && oc <= i) r = c;
                }
                const u32 ro = (u32)__shfl((int)excl, (int)r);
                const u32 rp = (u32)__shfl((int)pk, (int)r);
                const u32 rlit = rp & 63, rsrc = (rp >> 6) & 127;  // literal start, window-relative
                const u32 c = rsrc + (i - ro);                    // this byte's stream byte if a literal
                const u32 wlit = (u32)__shfl((int)w.x, (int)(c & 63)) & 0xFF;
                if (i < total) {
                    const u32 ix = (op + i) & LZ_RMASK;
                    u32 v;
                    if (i - ro < rlit) v = c < 64 ? wlit : (u32)s[e + c];
                    else v = R.entry(op + ro + rlit, 0, 0, rp >> 16, i - ro - rlit, op, total);  // the match part
                    ring[ix] = (u16)v;
                    // every byte of this pass is in the ring now (LDS operations of a
                    // wave complete in order): resolve, write back, store to HBM
                    if (v & LZ_PTR) {
                        do { v = ring[v & LZ_RMASK]; } while (v & LZ_PTR);
                        ring[ix] = (u16)v;
                    }
                    if (op + i < lim) dst[op + i] = (u8)v;
                }
            }
            LZ_T(5)
        } else {
            dc[1]++;
            // long sequences: one at a time, LZ_ROUND bytes per round, the
            // bytes spread over the lanes
            for (u32 k = 0; k < nseq; k++) {
                const u32 kl = (u32)__builtin_amdgcn_readlane((int)klit, (int)k);
                const u32 ks = (u32)__builtin_amdgcn_readlane((int)klsrc, (int)k);
                const u32 ko = (u32)__builtin_amdgcn_readlane((int)koffn, (int)k);
                const u32 kn = (u32)__builtin_amdgcn_readlane((int)len, (int)k);
                const u32 kpos = op + (u32)__builtin_amdgcn_readlane((int)excl, (int)k);
                for (u32 r0 = 0; r0 < kn; r0 += LZ_ROUND) {
                    const u32 rn = kn - r0 < LZ_ROUND ? kn - r0 : LZ_ROUND;
                    const u32 rb = kpos + r0;
                    R.need_visible(rb + rn > LZ_RING ? rb + rn - LZ_RING : 0, rb);
                    for (u32 j = lane; j < rn; j += 64)
                        ring[(rb + j) & LZ_RMASK] = (u16)R.entry(kpos, ks, kl, ko, r0 + j, rb, rn);
                    R.finish(rb, rn);
                }
            }
        }
        op += total;
        if (term) break;
        e += last_next;
        w = wn;
    }
    if (dbg) {
        dc[7] = __builtin_readcyclecounter() - tstart;
        dc[2] = op;
        if (lane < 8) {
            u64 v = 0;
#pragma unroll
            for (u32 k = 0; k < 8; k++) v = lane == k ? dc[k] : v;
            atomicAdd(&g_lz_dbg[lane], (unsigned long long)v);
        }
    }
#undef LZ_T
    *got_out = op;
    *st_out = st;
}

__global__ __launch_bounds__(256) void lz4_blocks_kernel(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                         u32 S, u32 vflags, const Lz4ChunkInfo* __restrict__ info,
                                                         Lz4Slot* __restrict__ slots) {
    __shared__ u16 rings[4][LZ_RING];
    // the wave index is wave-uniform: readfirstlane lets the compiler keep the
    // whole block walk in scalar registers and scalar branches
    const u32 wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u64 w = (u64)blockIdx.x * 4 + wv;
    u16* ring = rings[wv];
    const u32 c = (u32)(w / S);
    const u32 k = (u32)(w - (u64)c * S);
    if (c >= n) return;
    const Lz4ChunkInfo ci = info[c];
    if (ci.st != ZCG_OK || k >= ci.nslot) return;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    Lz4Slot* sl = slots + (u64)c * S + k;
    const u32 bs = sl->bs;
    const u32 cs = bs & 0x7FFFFFFFu;
    const u64 so = sl->src_off;
    const gu8* s = (const gu8*)ch.src + so;
    gu8* dst = (gu8*)ch.dst;
    const u64 op0 = (u64)k * ci.bmax;
    int st = ZCG_OK;
    u32 got = 0;
    if ((ci.flags & F_BLOCK_CKSUM) && !(vflags & ZCG_FLAG_SKIP_LZ4_BLOCK_CHECKSUM)) {
        u32 bad = 0;
        if (lane == 0) bad = xxh32((const u8*)s, cs, 0) != ld32((const u8*)s + cs);
        if (__builtin_amdgcn_readfirstlane(bad)) st = ZCG_ERR_INVALID_DATA;
    }
    if (st == ZCG_OK) {
        if (bs & 0x80000000u) {  // stored block: coalesced copy
            const u64 lim = D - op0 < cs ? D - op0 : cs;
            for (u64 i = (u64)lane * 16; i < lim; i += 1024) {
                if (i + 16 <= lim) *(gu32x4_ua*)(dst + op0 + i) = *(const gu32x4_ua*)(s + i);
                else for (u64 q = i; q < lim; q++) dst[op0 + q] = s[q];
            }
            got = cs;
        } else {
            const u64 lb = D - op0 < ci.bmax ? D - op0 : ci.bmax;
            lz4_block_wave(s, cs, ch.src_len - so, dst + op0, ci.bmax, (u32)lb, ring,
                           LZ_DBG && (vflags & ZCG_FLAG_DEBUG_COUNTERS) != 0, &got, &st);
        }
    }
    if (lane == 0) {
        sl->got = got;
        sl->st = st;
    }
}

// ---- 2b. one LANE per block (default) ---------------------------------------
// A C4 stream is ~14 000 sequences of ~4.7 output bytes per 64 KiB block, so
// per-sequence instruction count is what bounds the decoder.  Here every lane
// runs LZ4_decompress_safe on its own block (64 blocks per wave, no
// speculation, no cross-lane steps), and the output goes through a per-lane
// LDS ring of LZ_LRB bytes that is written to HBM in whole, aligned
// LZ_LRB/2-byte pieces (16-byte stores), so HBM sees full-sector writes even though
// the 64 lanes of a wave write 64 different blocks.  Match sources nearer
// than the ring come from LDS; older ones from the block's own HBM output,
// which this lane stored earlier (same-thread order).  Input comes through a
// 64-byte register buffer (LzBuf).
// Measured choices (A/B on one box): a 128-byte ring per lane,
// 64 lanes per workgroup, and the lane kernel from 131 072 blocks (8 192
// chunks of 16 blocks: lane 146 vs wave 140 GiB/s there, 77 vs 137 at 4 096).
constexpr u32 LZ_LRB = 128;         // ring bytes per lane (>= 2 * LZ_LPC)
constexpr u32 LZ_LPC = LZ_LRB / 2;  // flush granularity = longest piece written between flushes
constexpr u32 LZ_LRM = LZ_LRB - 1;
constexpr u32 LZ_LWG = 64;          // lanes per workgroup of the lane kernel
#ifndef LZ_LPW_SMALL
#define LZ_LPW_SMALL 64  // blocks per wave below LZ_LPW_THRESH blocks (fewer blocks per wave: more waves in flight)
#endif
#ifndef LZ_LPW_CORUN
#define LZ_LPW_CORUN 64  // blocks per wave of the lane kernel when it shares the GPU with the wave kernel
#endif
#ifndef LZ_LPW_THRESH
#define LZ_LPW_THRESH 262144
#endif
static_assert(LZ_LPW_SMALL >= 1 && LZ_LPW_SMALL <= LZ_LWG && LZ_LPW_CORUN >= 1 && LZ_LPW_CORUN <= LZ_LWG,
              "blocks per wave: the lane kernel launches LZ_LWG lanes per workgroup");
constexpr u64 LZ_LANE_MIN_BLOCKS = 131072;
// From 131 072 blocks (measured at 8 192 C4 chunks: lanes 50.6 ms, waves 54.3
// ms, 55 % lanes + 45 % waves side by side 45.0 ms) both kernels run at once on
// two streams; below it the waves alone are faster (4 096 chunks: waves 27.8,
// side by side 43.9; 6 144: 41.1 / 44.7), and from 262 144 blocks the lanes
// alone (16 384 chunks: 61.4 vs 79.2).
#ifndef LZ_CORUN_PCT
#define LZ_CORUN_PCT 55  // percent of the chunks decoded by lanes in a side-by-side batch
#endif
#ifndef LZ_CORUN_LO
#define LZ_CORUN_LO 131072
#endif
#ifndef LZ_CORUN_HI
#define LZ_CORUN_HI 196608
#endif

// The ring is written and read with byte-unaligned ds_write_b128 /
// ds_read_b128 (gfx950 LDS runs in the unaligned alignment mode;
// tools/probe/lds_unaligned checks it).  A lane's LDS block is
// [LZ_LRB ring | 32-byte mirror]; the mirror's first 16 bytes repeat the
// ring's first 16, so any 16 ring bytes are contiguous.  An append at ring
// offset w writes its vector at w (past the ring end it lands in the mirror,
// which is right), then a second time: at w + LZ_LRB when it touched the
// ring's first 16 bytes (the mirror), or, when it crossed the ring end, the
// wrapped part shifted down to the ring start as one aligned vector.  That
// vector's zero tail clobbers ring slots of bytes >= 98 back, so the ring
// serves sources nearer than LZ_NEAR = 96 (older ones come from HBM, where
// everything 64 bytes back is already flushed); the block stays 160 bytes,
// 64 lanes = 10 KiB, 16 workgroups per CU.
constexpr u32 LZ_LSTRIDE = LZ_LRB + 32;  // LDS bytes per lane
constexpr u32 LZ_NEAR = 96u;
typedef __attribute__((ext_vector_type(4))) u32 lz_v4;
__device__ __forceinline__ void lds_st16_ua(lu8* p, const u32x4& v) {
    const u32 a = (u32)(uintptr_t)p;
    const lz_v4 w = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(w) : "memory");
}
__device__ __forceinline__ u32x4 lds_ld16_ua(const lu8* p) {
    const u32 a = (u32)(uintptr_t)p;
    lz_v4 r;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return u32x4{r.x, r.y, r.z, r.w};
}

struct LaneRing {
    lu8* R;      // this lane's ring (16-byte aligned)
    gu8* dst;    // the block's output
    u32 lim;     // bytes of the block below N*size (never store at >= lim)
    u32 fl;      // output below fl is in HBM (a multiple of LZ_LPC)
    __device__ __forceinline__ void store_piece(u32 a) {
        if (a >= lim) return;
        const lu8* p = R + (a & LZ_LRM);
        if (a + LZ_LPC <= lim) {
#pragma unroll
            for (u32 i = 0; i < LZ_LPC / 16; i++) {
                const u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(p + 16 * i);
                *(gu32x4_ua*)(dst + a + 16 * i) = v;
            }
        } else {
            for (u32 i = 0; a + i < lim; i++) dst[a + i] = p[i];
        }
    }
    // store the whole pieces below op
    __device__ __forceinline__ void flush(u32 op) {
        while (op - fl >= LZ_LPC) { store_piece(fl); fl += LZ_LPC; }
    }
    __device__ __forceinline__ void finish(u32 op) {
        flush(op);
        for (u32 i = fl; i < op && i < lim; i++) dst[i] = R[i & LZ_LRM];
    }
    // append the first k (1..16) bytes of v at op: one unaligned 16-byte
    // write (bytes past op + k are stale and overwritten later), a second
    // one when it crosses the ring end or covers its first 16 bytes
    __device__ __forceinline__ void append16(u32& op, const u32x4& v, u32 k) {
        const u32 w = op & LZ_LRM;
        lds_st16_ua(R + w, v);
        if (w > LZ_LRB - 16) *(__attribute__((address_space(3))) u32x4*)R = win_shift(v, LZ_LRB - w);
        else if (w < 16) lds_st16_ua(R + w + LZ_LRB, v);
        op += k;
    }
    __device__ __forceinline__ u32x4 rd16(u32 p) const { return lds_ld16_ua(R + (p & LZ_LRM)); }
};

// v_perm_b32 selectors of the period-`off` pattern (off < 16): output dword d
// = perm(v.y, v.x, lo[d]) | perm(v.w, v.z, hi[d]); byte j takes source byte
// j mod off (0x0C selects a zero byte).  One table row per offset replaces
// a doubling loop (up to four 128-bit shift rounds).
__constant__ __attribute__((aligned(16))) u32 c_lz_pat[16][8] = {
    {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x01000100u, 0x01000100u, 0x01000100u, 0x01000100u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x00020100u, 0x01000201u, 0x02010002u, 0x00020100u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x03020100u, 0x03020100u, 0x03020100u, 0x03020100u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x03020100u, 0x02010004u, 0x01000403u, 0x00040302u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x03020100u, 0x01000504u, 0x05040302u, 0x03020100u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x03020100u, 0x00060504u, 0x04030201u, 0x01000605u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x03020100u, 0x07060504u, 0x03020100u, 0x07060504u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu},
    {0x03020100u, 0x07060504u, 0x0201000Cu, 0x06050403u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C00u, 0x0C0C0C0Cu},
    {0x03020100u, 0x07060504u, 0x01000C0Cu, 0x05040302u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0100u, 0x0C0C0C0Cu},
    {0x03020100u, 0x07060504u, 0x000C0C0Cu, 0x04030201u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x0C020100u, 0x0C0C0C0Cu},
    {0x03020100u, 0x07060504u, 0x0C0C0C0Cu, 0x03020100u, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x03020100u, 0x0C0C0C0Cu},
    {0x03020100u, 0x07060504u, 0x0C0C0C0Cu, 0x0201000Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x03020100u, 0x0C0C0C04u},
    {0x03020100u, 0x07060504u, 0x0C0C0C0Cu, 0x01000C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x03020100u, 0x0C0C0504u},
    {0x03020100u, 0x07060504u, 0x0C0C0C0Cu, 0x000C0C0Cu, 0x0C0C0C0Cu, 0x0C0C0C0Cu, 0x03020100u, 0x0C060504u}};
struct LzPat {
    u32x4 lo, hi;
};
__device__ __forceinline__ LzPat lz_pat_sel(u32 off) {  // any off: rows past 15 read row 0
    const u32 r = off < 16 ? off : 0u;
    const __attribute__((address_space(1))) u32x4* t = (const __attribute__((address_space(1))) u32x4*)&c_lz_pat[r][0];
    return LzPat{t[0], t[1]};
}
__device__ __forceinline__ u32x4 lz_pattern_perm(const u32x4& v, const LzPat& s) {
    return u32x4{__builtin_amdgcn_perm(v.y, v.x, s.lo.x) | __builtin_amdgcn_perm(v.w, v.z, s.hi.x),
                 __builtin_amdgcn_perm(v.y, v.x, s.lo.y) | __builtin_amdgcn_perm(v.w, v.z, s.hi.y),
                 __builtin_amdgcn_perm(v.y, v.x, s.lo.z) | __builtin_amdgcn_perm(v.w, v.z, s.hi.z),
                 __builtin_amdgcn_perm(v.y, v.x, s.lo.w) | __builtin_amdgcn_perm(v.w, v.z, s.hi.w)};
}

// the 16 output bytes at op - off (off >= 1; periodic when off < 16): from the
// ring when the source is near (its slots are not yet reused: off < LZ_LRB - 4,
// the 4 covering the stale tail of the last written dword), else from HBM
__device__ __forceinline__ u32x4 lz_src16(const LaneRing& O, u32 op, u32 off, const LzPat& ps) {
    const u32 p = op - off;
    if (off < LZ_NEAR) {
        const u32x4 v = O.rd16(p);
        return off < 16 ? lz_pattern_perm(v, ps) : v;
    }
    if (p + 16 <= O.lim) return *(const gu32x4_ua*)(O.dst + p);
    u64 lo = 0, hi = 0;  // the block's last bytes: nothing at >= lim is stored (or needed)
    for (u32 k = 0; k < 16; k++) {
        const u64 b = p + k < O.lim ? (u64)O.dst[p + k] : 0ull;
        if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
    }
    return u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
}

// A lane's input through a 64-byte register buffer (four 16-byte loads from a
// 16-byte aligned address, i.e. one or two whole lines per 48-64 bytes used)
// and a 16-byte working window cut from it with v_alignbyte.  With every lane
// streaming its own block, lines do not survive in L2 between the sparse
// 16-byte reloads of a plain window (each reload fetched a whole line).
__device__ __forceinline__ u32 sel4(u32 s, u32 a0, u32 a1, u32 a2, u32 a3) {
    return s == 0 ? a0 : s == 1 ? a1 : s == 2 ? a2 : a3;
}
struct LzBuf {
    const u8* src;
    u64 avail;
    u32x4 b0, b1, b2, b3;  // bytes [bb, bb + 64), bb 16-byte aligned
    u32 bb;
    u32x4 w;  // bytes [wb, wb + 16)
    u32 wb;
    __device__ __forceinline__ void load_buf(u32 q) {
        bb = q & ~15u;
        b0 = win_load(src, (u64)bb, avail);
        b1 = win_load(src, (u64)bb + 16, avail);
        b2 = win_load(src, (u64)bb + 32, avail);
        b3 = win_load(src, (u64)bb + 48, avail);
    }
    __device__ __forceinline__ void at(u32 q) {
        if (q - bb > 48) load_buf(q);
        const u32 d = q - bb;  // 0..48
        const u32 qd = d >> 4;
        // (the register barrier keeps the selects on values: folded into a
        // select of member addresses they would send the buffer to scratch)
        u32x4 c0 = b0, c1 = b1, c2 = b2, c3 = b3;
        asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
        const u32x4 lo = qd == 0 ? c0 : qd == 1 ? c1 : qd == 2 ? c2 : c3;
        const u32x4 hi = qd == 0 ? c1 : qd == 1 ? c2 : c3;  // (unused when d == 48)
        const u32 s4 = (d >> 2) & 3, sb = d & 3;
        // words s4 .. s4+4 of lo:hi
        const u32 y0 = sel4(s4, lo.x, lo.y, lo.z, lo.w), y1 = sel4(s4, lo.y, lo.z, lo.w, hi.x);
        const u32 y2 = sel4(s4, lo.z, lo.w, hi.x, hi.y), y3 = sel4(s4, lo.w, hi.x, hi.y, hi.z);
        const u32 y4 = sel4(s4, hi.x, hi.y, hi.z, hi.w);
        w = sb ? u32x4{__builtin_amdgcn_alignbyte(y1, y0, sb), __builtin_amdgcn_alignbyte(y2, y1, sb),
                       __builtin_amdgcn_alignbyte(y3, y2, sb), __builtin_amdgcn_alignbyte(y4, y3, sb)}
               : u32x4{y0, y1, y2, y3};
        wb = q;
    }
    __device__ __forceinline__ u32 byte(u32 q) {
        u32 d = q - wb;
        if (d >= 16) { at(q); d = 0; }
        return win_byte(w, d);
    }
};

// LZ4_decompress_safe of one block (the checks of lz4_block above, in its order),
// positions block-relative, low = 0 (independent blocks).  Every sequence takes
// the same short path on all lanes — literals as one 16-byte vector, the match
// as one 16-byte vector (ring, HBM or a periodic pattern), each appended with
// dword writes — so a wave's cost per step is one sequence, not the union of
// per-byte loops of its lanes; longer literals/matches loop in 16-byte pieces.
__device__ __forceinline__ int lz4_lane_block(const u8* __restrict__ src, u32 iend, u64 avail, LaneRing& O, u32 cap,
                              u32* out_n) {
    u32 ip = 0, op = 0;
    LzBuf in;
    in.src = src; in.avail = avail;
    in.load_buf(0);
    in.at(0);
    for (;;) {
        if (ip >= iend) return ZCG_ERR_INVALID_DATA;
        const u32 token = in.byte(ip++);
        u32 lit = token >> 4;
        if (lit == 15) {
            if ((i64)ip >= (i64)iend - 15) return ZCG_ERR_INVALID_DATA;
            u32 s;
            do {
                s = in.byte(ip++);
                lit += s;
            } while (s == 255 && (i64)ip < (i64)iend - 15);
        }
        const u64 cpy = (u64)op + lit;
        const bool last = cpy + 12 > cap || (i64)ip + lit > (i64)iend - 8;
        if (last && ((u64)ip + lit != iend || cpy > cap)) return ZCG_ERR_INVALID_DATA;
        // literals: 16 bytes at a time, from the window when they lie in it
        for (u32 j0 = 0; j0 < lit; j0 += 16) {
            const u32 d = ip - in.wb;
            const u32x4 v = (d + lit <= 16) ? win_shift(in.w, d) : win_load(src, ip, avail);
            const u32 k = lit - j0 < 16 ? lit - j0 : 16;
            O.append16(op, v, k);
            ip += k;
            O.flush(op);
        }
        if (last) break;
        const u32 off = in.byte(ip) | (in.byte(ip + 1) << 8);
        ip += 2;
        u32 ml = token & 15;
        if (ml == 15) {
            u32 s;
            do {
                s = in.byte(ip++);
                ml += s;
                if ((i64)ip >= (i64)iend - 4) return ZCG_ERR_INVALID_DATA;
            } while (s == 255);
        }
        ml += 4;
        if (op < off) return ZCG_ERR_INVALID_DATA;
        if ((u64)op + ml + 5 > cap) return ZCG_ERR_INVALID_DATA;
        if (ip - in.wb > 8) in.at(ip);  // the next sequence's window, in flight during the copy
        const LzPat ps = lz_pat_sel(off);  // (loaded for every sequence: counted by the waits)
        for (u32 r = ml; r > 0;) {
            const u32 k = r < 16 ? r : 16;
            // lz4 1.9.3 decodes offset 0 to zeros
            const u32x4 v = off ? lz_src16(O, op, off, ps) : u32x4{0u, 0u, 0u, 0u};
            O.append16(op, v, k);
            O.flush(op);
            r -= k;
        }
    }
    *out_n = op;
    return ZCG_OK;
}

__global__ __launch_bounds__(LZ_LWG, 1) void lz4_lanes_kernel(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                           u32 S, u32 vflags,
                                                           const Lz4ChunkInfo* __restrict__ info,
                                                           Lz4Slot* __restrict__ slots, u32 lpw) {
    __shared__ __attribute__((aligned(16))) u8 rings[LZ_LWG * LZ_LSTRIDE];
    if (threadIdx.x >= lpw) return;  // lpw blocks per wave
    const u64 g = (u64)blockIdx.x * lpw + threadIdx.x;
    const u32 c = (u32)(g / S);
    const u32 k = (u32)(g - (u64)c * S);
    if (c >= n) return;
    const Lz4ChunkInfo ci = info[c];
    if (ci.st != ZCG_OK || k >= ci.nslot) return;
    const zcg_chunk ch = chunks[c];
    Lz4Slot* sl = slots + (u64)c * S + k;
    const u32 bs = sl->bs;
    const u32 cs = bs & 0x7FFFFFFFu;
    const u64 so = sl->src_off;
    const u8* s = (const u8*)ch.src + so;
    gu8* dst = (gu8*)ch.dst + (u64)k * ci.bmax;
    const u64 op0 = (u64)k * ci.bmax;
    const u32 lb = (u32)(D - op0 < ci.bmax ? D - op0 : ci.bmax);
    int st = ZCG_OK;
    u32 got = 0;
    if ((ci.flags & F_BLOCK_CKSUM) && !(vflags & ZCG_FLAG_SKIP_LZ4_BLOCK_CHECKSUM))
        if (xxh32(s, cs, 0) != ld32(s + cs)) st = ZCG_ERR_INVALID_DATA;
    if (st == ZCG_OK) {
        if (bs & 0x80000000u) {  // stored block
            const u32 m = lb < cs ? lb : cs;
            u32 i = 0;
            for (; i + 16 <= m; i += 16) *(gu32x4_ua*)(dst + i) = ld16(s + i);
            for (; i < m; i++) dst[i] = s[i];
            got = cs;
        } else {
            LaneRing O{(lu8*)(rings + threadIdx.x * LZ_LSTRIDE), dst, lb, 0};
            const u64 avail = ch.src_len - so;
            st = lz4_lane_block(s, cs, avail, O, ci.bmax, &got);
            if (st == ZCG_OK) O.finish(got);
        }
    }
    sl->got = got;
    sl->st = st;
}

// ---- 3. per-chunk verdict, serial fallback, element transform -----------
__global__ __launch_bounds__(64) void lz4_finish_kernel(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                        DType t, u32 vflags, u32 S,
                                                        const Lz4ChunkInfo* __restrict__ info,
                                                        const Lz4Slot* __restrict__ slots,
                                                        i32* __restrict__ status) {
    const u32 c = blockIdx.x;
    if (c >= n) return;
    const int lane = lane_id();
    __shared__ int st_s;
    if (lane == 0) {
        const Lz4ChunkInfo ci = info[c];
        const Lz4Slot* sl = slots + (u64)c * S;
        int st = ci.st;
        if (st == ZCG_OK && D > 0) {
            const u32 ns = ci.nslot, bmax = ci.bmax;
            u64 total = 0;
            for (u32 k = 0; k < ns; k++) {
                if (sl[k].st != ZCG_OK) { st = sl[k].st; break; }
                const u32 got = sl[k].got;
                total = (u64)k * bmax + got;
                if (got != bmax && k + 1 < ns) { st = -1; break; }  // short block mid-frame
            }
            if (st == ZCG_OK && total == D && ns > 0) {  // last block ended exactly at N
                const zcg_chunk ch = chunks[c];
                const u64 pos = (u64)sl[ns - 1].src_off + (sl[ns - 1].bs & 0x7FFFFFFFu) +
                                ((ci.flags & F_BLOCK_CKSUM) ? 4 : 0);
                st = lz4_next_header_check((const u8*)ch.src, ch.src_len, pos, bmax);
            }
            if (st == ZCG_OK && total < D) {
                // frame ended / input ran out before N bytes; a short last
                // block followed by more blocks means the placement guess failed
                if (ci.flags & F_TRUNC) st = ZCG_ERR_UNEXPECTED_EOF;
                else if (ci.flags & F_FRAME_END)  // suffix checks: exact serial path
                    st = (ci.flags & (F_CONTENT_CKSUM | F_CONTENT_SIZE)) ? -1 : ZCG_ERR_UNEXPECTED_EOF;
                else st = -1;
            }
        }
        if (st == -1) {
            const zcg_chunk ch = chunks[c];
            st = lz4_frame_serial((const u8*)ch.src, ch.src_len, (u8*)ch.dst, D, vflags);
        }
        status[c] = st;
        st_s = st;
    }
    __syncthreads();
    if ((t.swap || t.isbool) && st_s == ZCG_OK) {
        __threadfence_block();
        wave_transform((u8*)chunks[c].dst, D, t);
    }
}

uint64_t lz4_decode_ws_bytes(const zcg_array* a, uint32_t n) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    u64 S = (D + LZ4_MIN_BMAX - 1) / LZ4_MIN_BMAX;
    if (S < 1) S = 1;
    return ((u64)n * sizeof(Lz4ChunkInfo) + 255) / 256 * 256 + (u64)n * S * sizeof(Lz4Slot);
}

hipError_t launch_lz4_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, int32_t* d_status,
                             void* ws, uint64_t ws_bytes, hipStream_t s, hipStream_t side, hipEvent_t fork,
                             hipEvent_t join) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    u64 S = (D + LZ4_MIN_BMAX - 1) / LZ4_MIN_BMAX;
    if (S < 1) S = 1;
    if (S > 65536 || ws_bytes < lz4_decode_ws_bytes(a, n)) return hipErrorInvalidValue;
    Lz4ChunkInfo* info = (Lz4ChunkInfo*)ws;
    Lz4Slot* slots = (Lz4Slot*)((u8*)ws + ((u64)n * sizeof(Lz4ChunkInfo) + 255) / 256 * 256);
    hipLaunchKernelGGL(lz4_frames_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d_chunks, n, D, (u32)S, info,
                       slots);
    const u64 waves = (u64)n * S;
    if ((waves + 3) / 4 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (D > 0) {
        // one lane per block needs ~16 waves per CU of blocks to hide its
        // latency; smaller batches run one wave per block
        const u32 fl = a->compression.flags;
        const bool forced = (fl & (ZCG_FLAG_LZ4_WAVE_PER_BLOCK | ZCG_FLAG_LZ4_LANE_PER_BLOCK)) != 0;
        const bool corun = !forced && waves >= LZ_CORUN_LO && waves < LZ_CORUN_HI;
        const bool wave = (fl & ZCG_FLAG_LZ4_WAVE_PER_BLOCK) ||
                          (!(fl & ZCG_FLAG_LZ4_LANE_PER_BLOCK) && !corun && waves < LZ_LANE_MIN_BLOCKS);
        hipStream_t s2 = corun && fork && join ? side : nullptr;
        if (wave) {
            hipLaunchKernelGGL(lz4_blocks_kernel, dim3((u32)((waves + 3) / 4)), dim3(256), 0, s, d_chunks, n, D,
                               (u32)S, a->compression.flags, (const Lz4ChunkInfo*)info, slots);
        } else if (s2) {
            // lanes for the first chunks on `s`, waves for the rest on the side
            // stream at the same time: the lane kernel is latency-bound and the
            // wave kernel VALU-bound, so they share the CUs
            const u32 n1 = (u32)((u64)n * LZ_CORUN_PCT / 100);
            hipError_t e = hipEventRecord(fork, s);
            if (e == hipSuccess) e = hipStreamWaitEvent(s2, fork, 0);
            if (e != hipSuccess) return e;
            const u64 w2 = (u64)(n - n1) * S;
            hipLaunchKernelGGL(lz4_blocks_kernel, dim3((u32)((w2 + 3) / 4)), dim3(256), 0, s2, d_chunks + n1, n - n1,
                               D, (u32)S, a->compression.flags, (const Lz4ChunkInfo*)info + n1, slots + (u64)n1 * S);
            const u64 w1 = (u64)n1 * S;
            if (w1)
                hipLaunchKernelGGL(lz4_lanes_kernel, dim3((u32)((w1 + LZ_LPW_CORUN - 1) / LZ_LPW_CORUN)), dim3(LZ_LWG),
                                   0, s, d_chunks, n1, D, (u32)S, a->compression.flags, (const Lz4ChunkInfo*)info,
                                   slots, (u32)LZ_LPW_CORUN);
            e = hipEventRecord(join, s2);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
            if (e != hipSuccess) return e;
        } else {
            const u32 lpw = waves < LZ_LPW_THRESH ? LZ_LPW_SMALL : LZ_LWG;
            hipLaunchKernelGGL(lz4_lanes_kernel, dim3((u32)((waves + lpw - 1) / lpw)), dim3(LZ_LWG), 0, s,
                               d_chunks, n, D, (u32)S, a->compression.flags, (const Lz4ChunkInfo*)info, slots, lpw);
        }
    }
    hipLaunchKernelGGL(lz4_finish_kernel, dim3(n), dim3(64), 0, s, d_chunks, n, D, t, a->compression.flags,
                       (u32)S, (const Lz4ChunkInfo*)info, (const Lz4Slot*)slots, d_status);
    return hipGetLastError();
}

const char* cfg_lz4_dec() {
    return "lz4_dec:CORUN=" ZCG_STR(LZ_CORUN_PCT) "/" ZCG_STR(LZ_CORUN_LO) "/" ZCG_STR(LZ_CORUN_HI) ",LPW="
        ZCG_STR(LZ_LPW_SMALL) "/" ZCG_STR(LZ_LPW_CORUN) "/" ZCG_STR(LZ_LPW_THRESH);
}

}  // namespace zcg
