// zcg_bz2_core.h — Bzip2Compression decode core (src/compression/bzip.rs:
// 35-46: bzip2 read::BzDecoder = libbz2 1.0.x BZ2_bzDecompress), the serial
// part of it, written once and instantiated twice:
//   * on gfx950 by zcg_bz2.hip (wave-uniform, Huffman tables in LDS, the
//     move-to-front list in one VGPR per lane, symbols streamed to HBM);
//   * on the host by tests/hostcore, fuzzed against libbz2 (the oracle).
//
// Serial part = everything libbz2's BZ2_decompress does for one block: the
// stream header ("BZh1".."BZh9"), the 48-bit block / end-of-stream magics,
// block CRC, randomised bit, origPtr, the symbol map, selectors (with the
// 1.0.8 rule that selectors beyond 18002 are read and ignored), delta-coded
// code lengths (1..20), libbz2's limit/base/perm decoding (so incomplete or
// over-subscribed codes decode exactly as libbz2 decodes them), RUNA/RUNB
// runs and the MTF stage, and the post-block sanity checks (origPtr < nblock).
// Its output is the BWT last column L[0..nblock) of the block.  The inverse
// BWT, RLE1 and the block CRC are data-parallel and live in the IO
// (parallel on the device, serial restatement on the host).
//
// Input model: libbz2 pulls whole bytes only when it needs bits, so after B
// bits the decoder has consumed ceil(B/8) bytes; the bit reader below peeks
// freely but charges consumption exactly that way, which keeps the 32 KiB
// BufReader-window semantics of the oracle (zr_decode_bzip2) intact.
#pragma once

#include <stdint.h>

#include "zcg_bz2_rnums.h"

#if defined(__HIP__)
#define ZB_INL __host__ __device__ __forceinline__
#else
#define ZB_INL inline __attribute__((always_inline))
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define ZB_U32(x) ((x) = __builtin_amdgcn_readfirstlane(x))
#define ZB_UB(c) (__builtin_amdgcn_readfirstlane((uint32_t)(c)) != 0)
// u64 `left` < small k on the scalar unit (it has no 64-bit ordered compare;
// the readfirstlane keeps the two halves from being re-fused into one)
#define ZB_LT(left, k) (__builtin_amdgcn_readfirstlane((uint32_t)((left) >> 32)) == 0 && (uint32_t)(left) < (uint32_t)(k))
#else
#define ZB_U32(x) ((void)0)
#define ZB_UB(c) (c)
#define ZB_LT(left, k) ((left) < (uint64_t)(k))
#endif

#ifndef ZB_TRACE
#define ZB_TRACE(bp, nb, v) ((void)0)
#endif

namespace zb {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

enum : int { ST_OK = 0, ST_EOF = 1, ST_INVALID = 2, ST_UNSUPPORTED = 4 };
// results of bz_block() besides the statuses above
enum : int { R_BLOCK = 10, R_END = 11, R_STOP = 12 };

constexpr u64 BUFREADER = 32768;    // bzip2-rs bufread window (oracle zr_decode_bzip2)
constexpr u32 MAX_SELECTORS = 18002;
constexpr u32 G_SIZE = 50;
constexpr u32 MAX_ALPHA = 258;
constexpr u32 LUT_BITS = 9;         // fast Huffman table width

// bzip2 CRC32: MSB-first, poly 0x04C11DB7, init/xorout ~0
ZB_INL u32 crc_byte(u32 c, u32 b) {
    c ^= b << 24;
    for (int k = 0; k < 8; k++) c = (c << 1) ^ (0x04C11DB7u & (0u - (c >> 31)));
    return c;
}

// Per-group decode tables (BZ2_hbCreateDecodeTables) + a LUT_BITS-wide fast
// table giving the same answer as libbz2's limit loop whenever that loop ends
// within LUT_BITS bits: entry = sym << 5 | len, or 0 = take the slow path.
struct Group {
    int32_t limit[24];
    int32_t base[24];
    u16 perm[MAX_ALPHA];
    u32 minlen;
};

// Persistent decoder state (one stream).
struct BzState {
    u64 n;          // input bytes
    u64 lim;        // visible input end (BufReader window once the output is full)
    u64 bitpos;     // bits consumed; bytes consumed = ceil(bitpos / 8)
    u32 level;      // blockSize100k
    u32 full;       // output already holds D bytes
    u32 header_done;
    u32 combined;   // computed combined CRC
    // current block
    u32 stored_crc, randomised, orig_ptr, nblock;
    u32 err_line;   // source line of the last INVALID verdict (diagnostics)
};

// IO concept (zcg_bz2.hip, tests/hostcore):
//   u32 peek(u64 bitpos, u32 nb)     next nb (<= 24) bits MSB-first (0 past n)
//   Group* group(u32 t)              6 decode-table slots (LDS on the device)
//   u16* lut(u32 t)                  6 fast tables of 2^LUT_BITS entries
//   u8* lens(u32 t)                  code lengths [6][258] scratch
//   void sel_put(u32 i, u32 g); u32 sel_get(u32 i)   selector store
//   void mtf_init(const u8* seq_to_unseq... ) -> via mtf_reset(map, nInUse)
//   u32 mtf_take(u32 nn)             byte at MTF index nn, moved to front
//   u32 mtf_front()                  byte at index 0
//   void l_put(u32 i, u32 byte); void l_run(u32 i, u32 byte, u32 count); void l_flush()

// Decode the next block (or the end-of-stream record).  Returns
//   R_BLOCK: L[0..s.nblock) written through io, s.orig_ptr/stored_crc set
//   R_END:   end of stream, combined CRC checked -> caller maps to OK/EOF
//   R_STOP:  visible input ran out (caller maps to OK if full, else EOF)
//   ST_INVALID / ST_UNSUPPORTED
template <class IO>
ZB_INL int bz_block(IO& io, BzState& s) {
#define ZB_ERR() do { s.err_line = __LINE__; return ST_INVALID; } while (0)
    u64 bp = s.bitpos;
    const u64 limbits = s.lim * 8;
// GET_BITS: consuming nb bits needs ceil((bp+nb)/8) <= lim visible bytes
#define ZB_BITS(nb, out)                                               \
    do {                                                               \
        if (ZB_LT(limbits - bp, nb)) { s.bitpos = bp; return R_STOP; } /* bp <= limbits */ \
        out = io.peek(bp, (nb));                                       \
        ZB_TRACE(bp, nb, out);                                         \
        bp += (nb);                                                    \
    } while (0)

    u32 uc = 0;
    if (!s.header_done) {
        ZB_BITS(8, uc);
        if (uc != 0x42) ZB_ERR();  // 'B'
        ZB_BITS(8, uc);
        if (uc != 0x5A) ZB_ERR();  // 'Z'
        ZB_BITS(8, uc);
        if (uc != 0x68) ZB_ERR();  // 'h'
        ZB_BITS(8, uc);
        if (uc < 0x31 || uc > 0x39) ZB_ERR();
        s.level = uc - 0x30;
        s.header_done = 1;
    }
    ZB_BITS(8, uc);
    if (uc == 0x17) {
        // end of stream: 72 45 38 50 90 + combined CRC
        for (int k = 0; k < 5; k++) {  // 72 45 38 50 90
            ZB_BITS(8, uc);
            if (uc != (u32)((0x7245385090ull >> (8 * (4 - k))) & 0xFF)) ZB_ERR();
        }
        u32 stored = 0;
        for (int k = 0; k < 4; k++) {
            ZB_BITS(8, uc);
            stored = (stored << 8) | uc;
        }
        s.bitpos = bp;
        if (stored != s.combined) ZB_ERR();
        return R_END;
    }
    if (uc != 0x31) ZB_ERR();
    {
        for (int k = 0; k < 5; k++) {  // 41 59 26 53 59
            ZB_BITS(8, uc);
            if (uc != (u32)((0x4159265359ull >> (8 * (4 - k))) & 0xFF)) ZB_ERR();
        }
    }
    u32 crc = 0;
    for (int k = 0; k < 4; k++) {
        ZB_BITS(8, uc);
        crc = (crc << 8) | uc;
    }
    s.stored_crc = crc;
    ZB_BITS(1, s.randomised);
    u32 orig = 0;
    for (int k = 0; k < 3; k++) {
        ZB_BITS(8, uc);
        orig = (orig << 8) | uc;
    }
    if (orig > 10 + 100000u * s.level) ZB_ERR();
    s.orig_ptr = orig;

    // ---- symbol map ----
    u32 used16;
    ZB_BITS(16, used16);
    u8* seq = io.seqbuf();
    u32 ninuse = 0;
    for (u32 i = 0; i < 16; i++) {
        if (used16 & (0x8000u >> i)) {
            u32 bits;
            ZB_BITS(16, bits);
            for (u32 j = 0; j < 16; j++)
                if (bits & (0x8000u >> j)) seq[ninuse++] = (u8)(i * 16 + j);
        }
    }
    if (ninuse == 0) ZB_ERR();
    const u32 alpha = ninuse + 2;

    // ---- selectors ----
    u32 ngroups, nsel;
    ZB_BITS(3, ngroups);
    if (ngroups < 2 || ngroups > 6) ZB_ERR();
    ZB_BITS(15, nsel);
    if (nsel < 1) ZB_ERR();
    {
        u32 pos = 0x543210u;  // MTF list of group ids, 4 bits each
        for (u32 i = 0; i < nsel; i++) {
            u32 j = 0;
            for (;;) {
                u32 b;
                ZB_BITS(1, b);
                if (b == 0) break;
                j++;
                if (j >= ngroups) ZB_ERR();
            }
            if (i < MAX_SELECTORS) {
                const u32 v = (pos >> (4 * j)) & 0xF;
                const u32 lowmask = (1u << (4 * j)) - 1;  // entries before j
                pos = (pos & ~((lowmask << 4) | 0xF)) | ((pos & lowmask) << 4) | v;
                // keep entries above j untouched
                io.sel_put(i, v);
            }
            ZB_U32(pos);
        }
        if (nsel > MAX_SELECTORS) nsel = MAX_SELECTORS;
    }

    // ---- coding tables ----
    for (u32 t = 0; t < ngroups; t++) {
        u32 curr;
        ZB_BITS(5, curr);
        u8* len = io.lens(t);
        for (u32 i = 0; i < alpha; i++) {
            for (;;) {
                if (curr < 1 || curr > 20) ZB_ERR();
                u32 b;
                ZB_BITS(1, b);
                if (b == 0) break;
                ZB_BITS(1, b);
                if (b == 0) curr++; else curr--;
            }
            len[i] = (u8)curr;
        }
    }
    for (u32 t = 0; t < ngroups; t++) {
        const u8* len = io.lens(t);
        Group* g = io.group(t);
        u32 minl = 32, maxl = 0;
        for (u32 i = 0; i < alpha; i++) {
            if (len[i] > maxl) maxl = len[i];
            if (len[i] < minl) minl = len[i];
        }
        // BZ2_hbCreateDecodeTables
        u32 pp = 0;
        for (u32 i = minl; i <= maxl; i++)
            for (u32 j = 0; j < alpha; j++)
                if (len[j] == i) g->perm[pp++] = (u16)j;
        for (u32 i = 0; i < 23; i++) g->base[i] = 0;
        for (u32 i = 0; i < alpha; i++) g->base[len[i] + 1]++;
        for (u32 i = 1; i < 23; i++) g->base[i] += g->base[i - 1];
        for (u32 i = 0; i < 23; i++) g->limit[i] = 0;
        int32_t vec = 0;
        for (u32 i = minl; i <= maxl; i++) {
            vec += (g->base[i + 1] - g->base[i]);
            g->limit[i] = vec - 1;
            vec <<= 1;
        }
        for (u32 i = minl + 1; i <= maxl; i++) g->base[i] = ((g->limit[i - 1] + 1) << 1) - g->base[i];
        g->minlen = minl;
        io.build_lut(t, g, alpha);
    }

    // ---- MTF values ----
    io.mtf_reset(seq, ninuse);
    const u32 eob = ninuse + 1;
    const u32 nmax = 100000u * s.level;
    u32 group_no = 0xFFFFFFFFu, group_pos = 0, gsel = 0;
    u32 nblock = 0;
    u32 es = 0, nrun = 0;  // pending RUNA/RUNB run: es+1 copies after the run ends
    bool in_run = false;
#ifndef ZB_GSAFE
#define ZB_GSAFE 1
#endif
    // a group's G_SIZE symbols take <= 20 bits each: when that many bits (plus
    // the table peek) are left at its start, no symbol of the group can reach
    // the input limit and the per-symbol check is skipped
    bool gsafe = false;
    for (;;) {
        // GET_MTF_VAL
        if (group_pos == 0) {
            group_no++;
            if (group_no >= nsel) ZB_ERR();
            group_pos = G_SIZE;
            gsel = io.sel_get(group_no);
            ZB_U32(gsel);
            gsafe = ZB_GSAFE && !ZB_LT(limbits - bp, G_SIZE * 20 + LUT_BITS);
        }
        group_pos--;
        u32 sym;
        {
            u32 hit = 0;
            if (gsafe || !ZB_LT(limbits - bp, LUT_BITS)) {
                const u32 e = io.lut_get(gsel, io.peek(bp, LUT_BITS));
                if (e) {
                    bp += e & 31;
                    sym = e >> 5;
                    hit = 1;
                }
            }
            if (!hit) {
                const Group* g = io.group(gsel);
                u32 zn = g->minlen;
                u32 zvec;
                ZB_BITS(zn, zvec);
                for (;;) {
                    if (zn > 20) ZB_ERR();
                    if ((int32_t)zvec <= g->limit[zn]) break;
                    zn++;
                    u32 zj;
                    ZB_BITS(1, zj);
                    zvec = (zvec << 1) | zj;
                }
                const int32_t k = (int32_t)zvec - g->base[zn];
                if (k < 0 || k >= (int32_t)MAX_ALPHA) ZB_ERR();
                sym = g->perm[k];
            }
        }
        ZB_U32(sym);
        if (sym <= 1) {  // RUNA / RUNB
            if (!in_run) {
                in_run = true;
                es = 0xFFFFFFFFu;  // -1
                nrun = 1;
            }
            if (nrun >= 2u * 1024 * 1024) ZB_ERR();
            es += (sym + 1) * nrun;
            nrun <<= 1;
            continue;
        }
        if (in_run) {
            in_run = false;
            es++;
            const u32 b = io.mtf_front();
            if ((u64)nblock + es > nmax) ZB_ERR();
            io.l_run(nblock, b, es);
            nblock += es;
        }
        if (sym == eob) break;
        if (nblock >= nmax) ZB_ERR();
        io.l_put(nblock, io.mtf_take(sym - 1));
        nblock++;
    }
    io.l_flush(nblock);
    if (s.orig_ptr >= nblock) ZB_ERR();
    s.nblock = nblock;
    s.bitpos = bp;
    return R_BLOCK;
#undef ZB_BITS
#undef ZB_ERR
}

// LUT for one group: the libbz2 limit loop run on every LUT_BITS-bit prefix.
ZB_INL u32 lut_entry(const Group* g, u32 x) {
    u32 zn = g->minlen;
    if (zn > LUT_BITS) return 0;
    for (;;) {
        const u32 zvec = x >> (LUT_BITS - zn);
        if ((int32_t)zvec <= g->limit[zn]) {
            const int32_t k = (int32_t)zvec - g->base[zn];
            if (k < 0 || k >= (int32_t)MAX_ALPHA) return 0;
            return ((u32)g->perm[k] << 5) | zn;
        }
        zn++;
        if (zn > LUT_BITS) return 0;
    }
}

// Whole-stream driver (read_exact of D bytes).  io.block_output(s) emits the
// current block: returns OUT_DONE (whole block emitted, block CRC verified,
// combined CRC updated), OUT_FULL (D reached inside the block), or a status.
enum : int { OUT_DONE = 20, OUT_FULL = 21 };

template <class IO>
ZB_INL int bz_stream(IO& io, BzState& s, u64 D) {
    if (D == 0) return ST_OK;
    for (;;) {
        const int r = bz_block(io, s);
        if (r == R_STOP || r == R_END) return s.full ? ST_OK : ST_EOF;
        if (r != R_BLOCK) return r;
        if (s.full) return ST_OK;  // next block decoded (validated) after N: nothing to emit
        const int o = io.block_output(s);
        if (o == OUT_FULL) return ST_OK;
        if (o != OUT_DONE) return o;
        if (io.out_pos() == D) {
            // output full exactly at a block end: libbz2 keeps parsing the
            // current 32 KiB input window
            s.full = 1;
            const u64 used = (s.bitpos + 7) >> 3;
            const u64 ve = ((used ? used - 1 : 0) / BUFREADER + 1) * BUFREADER;
            s.lim = ve < s.n ? ve : s.n;
        }
    }
}

}  // namespace zb
