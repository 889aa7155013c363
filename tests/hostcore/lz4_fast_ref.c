/* TEST INFRASTRUCTURE ONLY: a serial restatement of liblz4 1.9.3's block
 * compressor as LZ4F calls it for lz4-rs's frames (lz.rs:85-92: level 0,
 * independent blocks), i.e. LZ4_compress_fast_extState_fastReset with
 * acceleration 1 on a cleared table, no dictionary, limitedOutput with
 * dstCapacity = srcSize - 1 (LZ4F_makeBlock stores the block raw when this
 * returns 0).  A block below LZ4_64Klimit (65 547 bytes) uses the byU16
 * table: 2^13 u16 entries, hash4 of 4 bytes, every candidate in range; a
 * larger one (lz4 blockSize 256K/1M/4M) the byU32 table: 2^12 u32 entries,
 * hash5 of 5 bytes, candidates more than 65 535 back skipped.
 * tests/test_hostcore.py checks it byte for byte against liblz4's own
 * LZ4_compress_fast; the GPU encoder (zcg_lz4_enc.hip) restates the same
 * steps with a wave-parallel search.  Never linked into the product.
 *
 * It follows liblz4's LZ4_compress_generic closely (its search order and
 * hash-table updates decide the bytes), so it carries liblz4's notice:
 *   LZ4 - Fast LZ compression algorithm.  Copyright (C) 2011-present, Yann
 *   Collet.  BSD 2-Clause License: Redistribution and use in source and
 *   binary forms, with or without modification, are permitted provided that
 *   the following conditions are met: * Redistributions of source code must
 *   retain the above copyright notice, this list of conditions and the
 *   following disclaimer.  * Redistributions in binary form must reproduce the
 *   above copyright notice, this list of conditions and the following
 *   disclaimer in the documentation and/or other materials provided with the
 *   distribution.  THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND
 *   CONTRIBUTORS "AS IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT
 *   NOT LIMITED TO, THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR
 *   A PARTICULAR PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE COPYRIGHT
 *   OWNER OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL,
 *   SPECIAL, EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED
 *   TO, PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR
 *   PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY THEORY OF
 *   LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING
 *   NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS
 *   SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
 * (Altered: a restatement, not liblz4's source.) */
#include <stdint.h>
#include <string.h>

typedef uint8_t u8;
typedef uint32_t u32;

#define MINMATCH 4
#define MFLIMIT 12
#define LASTLITERALS 5
#define LZ4_minLength (MFLIMIT + 1)
#define ML_BITS 4
#define ML_MASK 15u
#define RUN_MASK 15u
#define SKIP_TRIGGER 6
#define LZ4_64Klimit (65536 + MFLIMIT - 1)
#define DISTANCE_MAX 65535u

static u32 rd32(const u8* p) { u32 v; memcpy(&v, p, 4); return v; }
static uint64_t rd64(const u8* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static int g_u32;  /* byU32 mode of the current block */
/* LZ4_hashPosition: hash4 (13 bits) for byU16, hash5 (12 bits) for byU32 */
static u32 hashp(const u8* p) {
    if (!g_u32) return (rd32(p) * 2654435761u) >> (32 - 13);
    return (u32)(((rd64(p) << 24) * 889523592379ull) >> (64 - 12));
}

/* LZ4_count: matching bytes of in and m, in < limit */
static u32 count(const u8* in, const u8* m, const u8* limit) {
    const u8* s = in;
    while (in < limit && *in == *m) { in++; m++; }
    return (u32)(in - s);
}

int zref_lz4_fast_block(const u8* src, int n, u8* dst, int cap) {
    static u32 table[1 << 13];
    memset(table, 0, sizeof(table));
    g_u32 = n >= LZ4_64Klimit;
    const u8* ip = src;
    const u8* anchor = src;
    const u8* const iend = src + n;
    const u8* const mflimitPlusOne = iend - MFLIMIT + 1;
    const u8* const matchlimit = iend - LASTLITERALS;
    u8* op = dst;
    u8* const olimit = dst + cap;
    if (n < LZ4_minLength) goto last_literals;
    table[hashp(ip)] = 0;  /* LZ4_putPosition(first byte) */
    ip++;
    u32 forwardH = hashp(ip);
    for (;;) {
        const u8* match;
        u8* token;
        {   /* find a match */
            const u8* forwardIp = ip;
            int step = 1;
            int searchMatchNb = 1 << SKIP_TRIGGER;
            for (;;) {
                const u32 h = forwardH;
                const u32 current = (u32)(forwardIp - src);
                const u32 matchIndex = table[h];
                ip = forwardIp;
                forwardIp += step;
                step = searchMatchNb++ >> SKIP_TRIGGER;
                if (forwardIp > mflimitPlusOne) goto last_literals;
                match = src + matchIndex;
                forwardH = hashp(forwardIp);
                table[h] = current;
                if (g_u32 && matchIndex + DISTANCE_MAX < current) continue;
                if (rd32(match) == rd32(ip)) break;
            }
        }
        /* catch up */
        while ((ip > anchor) & (match > src) && ip[-1] == match[-1]) { ip--; match--; }
        {   /* literals */
            const u32 lit = (u32)(ip - anchor);
            token = op++;
            if (op + lit + (2 + 1 + LASTLITERALS) + (lit / 255) > olimit) return 0;
            if (lit >= RUN_MASK) {
                u32 len = lit - RUN_MASK;
                *token = (u8)(RUN_MASK << ML_BITS);
                for (; len >= 255; len -= 255) *op++ = 255;
                *op++ = (u8)len;
            } else {
                *token = (u8)(lit << ML_BITS);
            }
            memcpy(op, anchor, lit);
            op += lit;
        }
    next_match:
        /* offset */
        op[0] = (u8)(ip - match);
        op[1] = (u8)((ip - match) >> 8);
        op += 2;
        {   /* match length */
            const u32 mc = count(ip + MINMATCH, match + MINMATCH, matchlimit);
            ip += mc + MINMATCH;
            if (op + (1 + LASTLITERALS) + (mc + 240) / 255 > olimit) return 0;
            if (mc >= ML_MASK) {
                u32 len = mc - ML_MASK;
                *token += ML_MASK;
                for (; len >= 510; len -= 510) { *op++ = 255; *op++ = 255; }
                if (len >= 255) { len -= 255; *op++ = 255; }
                *op++ = (u8)len;
            } else {
                *token += (u8)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimitPlusOne) break;
        /* fill table */
        table[hashp(ip - 2)] = (u32)(ip - 2 - src);
        {   /* test next position */
            const u32 h = hashp(ip);
            const u32 current = (u32)(ip - src);
            const u32 matchIndex = table[h];
            match = src + matchIndex;
            table[h] = current;
            if ((!g_u32 || matchIndex + DISTANCE_MAX >= current) && rd32(match) == rd32(ip)) {
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        forwardH = hashp(++ip);
    }
last_literals:
    {
        const u32 last = (u32)(iend - anchor);
        if (op + last + 1 + ((last + 255 - RUN_MASK) / 255) > olimit) return 0;
        if (last >= RUN_MASK) {
            u32 acc = last - RUN_MASK;
            *op++ = (u8)(RUN_MASK << ML_BITS);
            for (; acc >= 255; acc -= 255) *op++ = 255;
            *op++ = (u8)acc;
        } else {
            *op++ = (u8)(last << ML_BITS);
        }
        memcpy(op, anchor, last);
        op += last;
    }
    return (int)(op - dst);
}
