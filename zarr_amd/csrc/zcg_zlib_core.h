// zcg_zlib_core.h — the deflate_slow encoder of zlib 1.2.11 (levels 4-9),
// restated so that its output can be produced by data-parallel kernels and
// still be byte-identical to zlib's (GzipCompression::encoder, gzip.rs:54-56
// -> flate2 GzEncoder -> zlib deflate, windowBits -15, memLevel 8, default
// strategy).  Host and device (__host__ __device__), so tests/hostcore runs
// the same functions on the CPU against the system zlib.
//
// zlib's result decomposes into three deterministic pieces:
//
//  1. Per position p, the hash chain (15-bit rolling hash of p..p+2; every
//     position <= D-3 is inserted, in order, whatever the parse) and the
//     longest_match result for the two chain budgets deflate_slow can ask for
//     (max_chain, and max_chain >> 2 once prev_length >= good_match).  The
//     initial best_len (prev_length) only filters the result, so zz_search
//     computes both budgets in one walk, independently per position.
//  2. The lazy parse (zz_parse): a short sequential state machine over those
//     results, with zlib's TOO_FAR rule, its block flushes (16 383 symbols,
//     lit_bufsize - 1 for memLevel 8), and the window slides that decide
//     whether a block's bytes are still in the window (stored-block option).
//  3. Per block, _tr_flush_block (zz_plan_block): build_tree / gen_bitlen /
//     gen_codes / scan_tree / build_bl_tree with zlib's heap and its tie
//     order, the stored / static / dynamic decision on opt_len / static_len,
//     and the exact bits (send_all_trees, compress_block).
//
// The tree construction below is a statement-by-statement restatement of
// zlib's trees.c (build_tree, pqdownheap, gen_bitlen, gen_codes, scan_tree,
// send_tree, build_bl_tree), because the heap's tie order decides the code
// lengths and so the bytes.  zlib is (C) 1995-2017 Jean-loup Gailly and Mark
// Adler, under the zlib license:
//   This software is provided 'as-is', without any express or implied
//   warranty.  In no event will the authors be held liable for any damages
//   arising from the use of this software.  Permission is granted to anyone
//   to use this software for any purpose, including commercial applications,
//   and to alter it and redistribute it freely, subject to the following
//   restrictions: 1. The origin of this software must not be misrepresented;
//   you must not claim that you wrote the original software.  If you use this
//   software in a product, an acknowledgment in the product documentation
//   would be appreciated but is not required.  2. Altered source versions
//   must be plainly marked as such, and must not be misrepresented as being
//   the original software.  3. This notice may not be removed or altered from
//   any source distribution.
// (This file is an altered restatement, not zlib's source.)
#pragma once

#include <stdint.h>

#if defined(__HIP__)
#define ZZ_INL __host__ __device__ __forceinline__
#define ZZ_FN __host__ __device__
#else
#define ZZ_INL inline __attribute__((always_inline))
#define ZZ_FN inline
#endif

namespace zz {

constexpr uint32_t MIN_MATCH = 3, MAX_MATCH = 258;
constexpr uint32_t WSIZE = 32768;
constexpr uint32_t MIN_LOOKAHEAD = MAX_MATCH + MIN_MATCH + 1;  // 262
constexpr uint32_t MAX_DIST = WSIZE - MIN_LOOKAHEAD;            // 32506
constexpr uint32_t TOO_FAR = 4096;
constexpr uint32_t LIT_BUFSIZE = 1u << (8 + 6);  // memLevel 8
constexpr uint32_t BLOCK_SYMS = LIT_BUFSIZE - 1;  // symbols per flushed block
constexpr uint32_t NONE = 0xFFFFFFFFu;

constexpr int L_CODES = 286, D_CODES = 30, BL_CODES = 19, HEAP_SIZE = 2 * L_CODES + 1;
constexpr int MAX_BITS = 15, MAX_BL_BITS = 7, END_BLOCK = 256, LITERALS = 256;
constexpr int REP_3_6 = 16, REPZ_3_10 = 17, REPZ_11_138 = 18;

struct Config {
    uint32_t good, lazy, nice, chain;
};
// zlib's configuration_table: levels 1-3 run deflate_fast (`lazy` is then
// max_insert_length), 4-9 deflate_slow
ZZ_INL Config level_config(int level) {
    switch (level) {
        case 1: return {4, 4, 8, 4};
        case 2: return {4, 5, 16, 8};
        case 3: return {4, 6, 32, 32};
        case 4: return {4, 4, 16, 16};
        case 5: return {8, 16, 32, 32};
        case 7: return {8, 32, 128, 256};
        case 8: return {32, 128, 258, 1024};
        case 9: return {32, 258, 258, 4096};
        default: return {8, 16, 128, 128};
    }
}

ZZ_INL uint32_t hash3(uint32_t b0, uint32_t b1, uint32_t b2) { return ((b0 << 10) ^ (b1 << 5) ^ b2) & 0x7FFFu; }

// Window slides fill_window has done by the loop top at q (input fully
// available, as flate2 feeds it: 1 KiB-multiple writes fill the 64 KiB window
// the same way): slide k happens at the first loop top q with
// q - 32768 (k - 1) >= 65274, plus one more position while q <= D - 262
// (before the end, fill_window runs only once lookahead < 262).
ZZ_INL uint32_t slides_at(uint32_t q, uint32_t D) {
    const uint32_t thr = WSIZE + MAX_DIST + ((uint64_t)q + MIN_LOOKAHEAD <= D ? 1u : 0u);
    return q >= thr ? (q - thr) / WSIZE + 1 : 0u;
}

// longest_match at p for both chain budgets.  Result word: len | dist << 9
// (len 0 = no search; dist = p - the first candidate reaching len).  `full` walks cfg.chain candidates, `red` the first cfg.chain >> 2.
// BYTE(i) gives serialised byte i, PREV(i) the previous position with i's
// hash (NONE if none).
struct Match2 {
    uint32_t full, red;
};
template <class BYTE4, class BYTE, class PREV>
ZZ_FN Match2 search(uint32_t p, uint32_t D, const Config& cfg, const BYTE4& byte4, const BYTE& byte, const PREV& prev) {
    Match2 r{0u, 0u};
    if (p + MIN_MATCH > D) return r;
    uint32_t c = prev(p);
    // hash_head != NIL && strstart - hash_head <= MAX_DIST; hash_head is
    // window-relative, so the position at the window's base (absolute 0, or
    // k * 32768 after k slides) reads as NIL
    if (c == NONE || c == slides_at(p, D) * WSIZE || p - c > MAX_DIST) return r;
    const uint32_t look = D - p;
    const uint32_t mx = look < MAX_MATCH ? look : MAX_MATCH;
    const uint32_t nice = cfg.nice < look ? cfg.nice : look;
    const uint32_t lim = p > MAX_DIST ? p - MAX_DIST : 0u;  // later candidates must be > lim
    const uint32_t nred = cfg.chain >> 2;
    uint32_t best = 0, bstart = 0, pend = 0;  // pend: p's four bytes ending at best
    bool red_done = false;
    // the next link is read as soon as a candidate is known, so on the GPU
    // its load is in flight together with the candidate's byte loads
    uint32_t cn = prev(c);
    for (uint32_t k = 0; k < cfg.chain; k++) {
        if (k > 0) {
            c = cn;
            if (c == NONE || c <= lim) break;
            cn = prev(c);
        }
        // a candidate beats best only if bytes 0..best all match: the four
        // ending at best are checked first (zlib's scan_end test, widened)
        if (best >= MIN_MATCH && best < mx && pend != byte4(c + best - 3)) goto next;
        {
        // common prefix of p.. and c.. (c < p), capped at mx
        uint32_t len = 0;
        while (len + 4 <= mx) {
            const uint32_t x = byte4(p + len) ^ byte4(c + len);
            if (x) {
                len += (uint32_t)__builtin_ctz(x) >> 3;
                goto done;
            }
            len += 4;
        }
        while (len < mx && byte(p + len) == byte(c + len)) len++;
    done:
        if (len > best) {
            best = len;
            bstart = c;
            if (best >= nice) break;
            if (best >= MIN_MATCH && best < mx) pend = byte4(p + best - 3);
        }
        }
    next:
        if (k + 1 == nred) {
            r.red = best ? (best | ((p - bstart) << 9)) : 0u;
            red_done = true;
        }
    }
    r.full = best ? (best | ((p - bstart) << 9)) : 0u;
    if (!red_done) r.red = r.full;  // the walk ended (chain end / nice) within the reduced budget
    return r;
}

// ---- the lazy parse --------------------------------------------------------
// Symbols: literal = byte; match = 1 << 31 | (len - 3) << 16 | (dist - 1).
// A block flush is reported after the symbol that fills it, with its byte
// range [b0, b1) and whether its bytes are still in zlib's window.
struct BlockRec {
    uint32_t s0, s1;    // symbols
    uint32_t b0, b1;    // input bytes
    uint32_t in_win;    // _tr_flush_block's buf != NULL (stored block allowed)
    uint32_t last;
};

template <class GET, class BYTE, class EMIT, class FLUSH>
ZZ_FN void parse(uint32_t D, const Config& cfg, const GET& get, const BYTE& byte, EMIT& emit, FLUSH& flush) {
    uint32_t prev_len = MIN_MATCH - 1, prev_dist = 0, avail = 0, p = 0;
    uint32_t nsym = 0, s0 = 0, b0 = 0, slide = 0;
    auto top = [&](uint32_t q) {  // fill_window at a loop top: one slide when due
        const uint32_t wend = (D - slide) > 2 * WSIZE ? slide + 2 * WSIZE : D;
        if (wend - q < MIN_LOOKAHEAD && q - slide >= WSIZE + MAX_DIST) slide += WSIZE;
    };
    auto tally = [&](uint32_t sym, uint32_t end) {
        emit(nsym, sym);
        nsym++;
        if (nsym - s0 == BLOCK_SYMS) {
            BlockRec b{s0, nsym, b0, end, b0 >= slide ? 1u : 0u, 0u};
            flush(b);
            s0 = nsym;
            b0 = end;
        }
    };
    while (true) {
        top(p);
        if (p >= D) break;
        uint32_t ml = MIN_MATCH - 1, mdist = 0;
        if (p + MIN_MATCH <= D && prev_len < cfg.lazy) {
            const Match2 g = get(p);
            const uint32_t w = prev_len >= cfg.good ? g.red : g.full;
            const uint32_t len = w & 511u;
            if (len > prev_len) {  // longest_match found a longer one
                ml = len;
                mdist = w >> 9;
                if (ml == MIN_MATCH && mdist > TOO_FAR) ml = MIN_MATCH - 1;
            } else {
                ml = prev_len;  // (returns best_len = prev_length; only <= matters)
            }
        }
        if (prev_len >= MIN_MATCH && ml <= prev_len) {
            const uint32_t at = p - 1;
            tally(0x80000000u | ((prev_len - MIN_MATCH) << 16) | (prev_dist - 1), at + prev_len);
            p = at + prev_len;
            prev_len = MIN_MATCH - 1;
            avail = 0;
        } else if (avail) {
            tally(byte(p - 1), p);
            prev_len = ml;
            prev_dist = mdist;
            p++;
        } else {
            avail = 1;
            prev_len = ml;
            prev_dist = mdist;
            p++;
        }
    }
    if (avail) {  // the pending literal is tallied without a flush check
        emit(nsym, byte(p - 1));
        nsym++;
    }
    BlockRec b{s0, nsym, b0, D, b0 >= slide ? 1u : 0u, 1u};
    flush(b);
}

// ---- the same parse, one loop top at a time (segment-parallel form) ------------
// deflate_slow's state between loop tops.  A CANONICAL state (just after a
// match, or the start) is prev_len = 2, avail = 0: two parses that reach a
// canonical state at the same position agree from there on, which is what
// lets speculative per-segment parses be stitched.
struct PState {
    uint32_t p, prev_len, prev_dist, avail;
};
ZZ_INL PState fresh_state(uint32_t p) { return PState{p, MIN_MATCH - 1, 0u, 0u}; }
ZZ_INL bool canonical(const PState& s) { return s.prev_len == MIN_MATCH - 1 && s.avail == 0; }

// One loop top at s.p (< D).  emit(sym, start position) when a symbol leaves.
template <class GET, class BYTE, class EMIT>
ZZ_FN void step(PState& s, uint32_t D, const Config& cfg, const GET& get, const BYTE& byte, EMIT& emit) {
    const uint32_t p = s.p;
    uint32_t ml = MIN_MATCH - 1, mdist = 0;
    if (p + MIN_MATCH <= D && s.prev_len < cfg.lazy) {
        const Match2 g = get(p);
        const uint32_t w = s.prev_len >= cfg.good ? g.red : g.full;
        const uint32_t len = w & 511u;
        if (len > s.prev_len) {
            ml = len;
            mdist = w >> 9;
            if (ml == MIN_MATCH && mdist > TOO_FAR) ml = MIN_MATCH - 1;
        } else {
            ml = s.prev_len;
        }
    }
    if (s.prev_len >= MIN_MATCH && ml <= s.prev_len) {
        const uint32_t at = p - 1;
        emit(0x80000000u | ((s.prev_len - MIN_MATCH) << 16) | (s.prev_dist - 1), at);
        s.p = at + s.prev_len;
        s.prev_len = MIN_MATCH - 1;
        s.avail = 0;
    } else if (s.avail) {
        emit(byte(p - 1), p - 1);
        s.prev_len = ml;
        s.prev_dist = mdist;
        s.p = p + 1;
    } else {
        s.avail = 1;
        s.prev_len = ml;
        s.prev_dist = mdist;
        s.p = p + 1;
    }
}

ZZ_INL uint32_t sym_len(uint32_t sym) { return (sym & 0x80000000u) ? ((sym >> 16) & 0xFF) + MIN_MATCH : 1u; }


// Block k of a chunk whose parse emitted nsym symbols, nloop of them inside
// deflate_slow's loop (the last may be the pending literal tallied at
// Z_FINISH, which never flushes).  A block flushes when its 16 383rd loop
// symbol is tallied; the final block takes the rest (possibly none).
// pos(i) / sym(i): start position and word of symbol i.
ZZ_INL uint32_t num_blocks(uint32_t nloop) { return nloop / BLOCK_SYMS + 1; }
// (deflate_fast, `fast`: every symbol is tallied in the loop iteration that
// starts at it, so a block's flush comes at the top at its last symbol's
// start; deflate_slow tallies a symbol one iteration later)
template <class POS, class SYM>
ZZ_FN BlockRec block_rec(uint32_t k, uint32_t nsym, uint32_t nloop, uint32_t D, const POS& pos, const SYM& sym,
                         bool fast = false) {
    const uint32_t nfl = nloop / BLOCK_SYMS;  // in-loop flushes
    BlockRec b{};
    b.s0 = k * BLOCK_SYMS;
    b.last = k == nfl ? 1u : 0u;
    b.s1 = b.last ? nsym : b.s0 + BLOCK_SYMS;
    b.b0 = k == 0 ? 0u : pos(b.s0 - 1) + sym_len(sym(b.s0 - 1));
    uint32_t top;
    if (b.last) {
        b.b1 = D;
        top = D;
    } else {
        const uint32_t l = b.s1 - 1;
        b.b1 = pos(l) + sym_len(sym(l));
        top = fast ? pos(l) : pos(l) + 1;
    }
    b.in_win = b.b0 >= slides_at(top, D) * WSIZE ? 1u : 0u;
    return b;
}

// ---- deflate_fast (levels 1-3) ------------------------------------------------
// Greedy parse with the hash chains built as it goes: a position is inserted
// when it is a loop top, or inside a match no longer than max_insert_length
// (cfg.lazy), so unlike deflate_slow the chains depend on the parse and the
// parse runs serially.  TAB holds zlib's head[] and prev[] as window-relative
// Pos values (0 = NIL), slid like slide_hash:
//   u32 head(u32 h); void set_head(u32 h, u32 v); u32 prev(u32 i);
//   void set_prev(u32 i, u32 v); void slide();   (i = position & WMASK)
// emit(sym, start position) per symbol; returns the symbol count.  Every
// symbol is an in-loop tally (nloop = nsym; block_rec(..., fast = true)).
constexpr uint32_t WMASK = WSIZE - 1;
template <class TAB, class BYTE4, class BYTE, class EMIT>
ZZ_FN uint32_t parse_fast(uint32_t D, const Config& cfg, TAB& tab, const BYTE4& byte4, const BYTE& byte, EMIT& emit) {
    uint32_t p = 0, nsym = 0, base = 0;  // base: absolute position of window-relative 0
    auto insert = [&](uint32_t q) -> uint32_t {  // INSERT_STRING: the previous head (relative, 0 = NIL)
        const uint32_t h = hash3(byte(q), byte(q + 1), byte(q + 2));
        const uint32_t hh = tab.head(h);
        tab.set_prev((q - base) & WMASK, hh);
        tab.set_head(h, q - base);
        return hh;
    };
    while (p < D) {
        {  // fill_window at the loop top: one slide when due
            const uint32_t wend = (D - base) > 2 * WSIZE ? base + 2 * WSIZE : D;
            if (wend - p < MIN_LOOKAHEAD && p - base >= WSIZE + MAX_DIST) {
                tab.slide();
                base += WSIZE;
            }
        }
        uint32_t ml = 0, md = 0;
        if (D - p >= MIN_MATCH) {
            const uint32_t hh = insert(p);
            if (hh != 0 && (p - base) - hh <= MAX_DIST) {
                const uint32_t first = hh + base;
                auto pv = [&](uint32_t x) -> uint32_t {
                    if (x == p) return first;
                    const uint32_t r = tab.prev((x - base) & WMASK);
                    return r == 0 ? NONE : r + base;
                };
                const Match2 g = search(p, D, cfg, byte4, byte, pv);
                const uint32_t len = g.full & 511u;
                if (len >= MIN_MATCH) {
                    ml = len;
                    md = g.full >> 9;
                }
            }
        }
        if (ml) {
            emit(0x80000000u | ((ml - MIN_MATCH) << 16) | (md - 1), p);
            nsym++;
            if (ml <= cfg.lazy && D - (p + ml) >= MIN_MATCH)
                for (uint32_t q = p + 1; q < p + ml; q++) insert(q);
            p += ml;
        } else {
            emit(byte(p), p);
            nsym++;
            p++;
        }
    }
    return nsym;
}

// ---- trees (trees.c) ---------------------------------------------------------
ZZ_INL uint32_t len_code(uint32_t len) {  // 3..258 -> 0..28 (_length_code)
    if (len == 258) return 28;
    const uint32_t x = len - 3;
    if (x < 8) return x;
    const uint32_t k = 31 - __builtin_clz(x);
    return 4 * (k - 1) + ((x >> (k - 2)) & 3);
}
ZZ_INL uint32_t dist_code(uint32_t d) {  // 1..32768 -> 0..29 (d_code(d - 1))
    const uint32_t x = d - 1;
    if (x < 4) return x;
    const uint32_t k = 31 - __builtin_clz(x);
    return 2 * k + ((x >> (k - 1)) & 1);
}
ZZ_INL uint32_t extra_lbits(int c) { return c < 8 ? 0u : c == 28 ? 0u : (uint32_t)((c - 4) >> 2); }
ZZ_INL uint32_t extra_dbits(int c) { return c < 4 ? 0u : (uint32_t)((c - 2) >> 1); }
ZZ_INL uint32_t extra_blbits(int c) { return c == 16 ? 2u : c == 17 ? 3u : c == 18 ? 7u : 0u; }
ZZ_INL uint32_t base_length(int c) {
    if (c == 28) return 255;  // (258 - 3: code 285 has no extra bits)
    if (c < 8) return (uint32_t)c;
    const uint32_t k = (uint32_t)(c - 4) >> 2;  // extra bits
    return (4u + ((uint32_t)c & 3u)) << k;
}
ZZ_INL uint32_t base_dist(int c) {
    if (c < 4) return (uint32_t)c;
    const uint32_t k = (uint32_t)(c - 2) >> 1;
    return ((2u + ((uint32_t)c & 1u)) << k);
}
ZZ_INL uint32_t static_llen(int n) { return n < 144 ? 8u : n < 256 ? 9u : n < 280 ? 7u : 8u; }
ZZ_INL uint32_t bi_reverse(uint32_t code, int len) {
    uint32_t res = 0;
    do {
        res |= code & 1;
        code >>= 1, res <<= 1;
    } while (--len > 0);
    return res >> 1;
}
ZZ_INL int bl_order(int i) {
    const int o[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    return o[i];
}
// static code of litlen symbol n (bit-reversed, as zlib's static_ltree)
ZZ_INL uint32_t static_lcode(int n) {
    uint32_t c;
    if (n < 144) c = 0x30 + (uint32_t)n;
    else if (n < 256) c = 0x190 + (uint32_t)(n - 144);
    else if (n < 280) c = (uint32_t)(n - 256);
    else c = 0xC0 + (uint32_t)(n - 280);
    return bi_reverse(c, (int)static_llen(n));
}

template <int N>
struct TreeT {  // ct_data of one tree (dyn_ltree: HEAP_SIZE; dyn_dtree 2*D_CODES+1; bl_tree 2*BL_CODES+1)
    uint32_t freq[N];
    uint16_t len[N];
    uint16_t dad[N];
    uint16_t code[N];
    int max_code;
};
typedef TreeT<HEAP_SIZE> LTree;
typedef TreeT<2 * D_CODES + 1> DTree;
typedef TreeT<2 * BL_CODES + 1> BTree;
struct TreeWork {  // deflate_state's heap / depth / bl_count
    int heap[HEAP_SIZE];
    int heap_len, heap_max;
    uint8_t depth[HEAP_SIZE];
    uint16_t bl_count[MAX_BITS + 1];
};

template <class Tree>
ZZ_INL bool smaller(const Tree& t, int n, int m, const uint8_t* depth) {
    return t.freq[n] < t.freq[m] || (t.freq[n] == t.freq[m] && depth[n] <= depth[m]);
}

template <class Tree>
ZZ_FN void pqdownheap(TreeWork& w, const Tree& t, int k) {
    const int v = w.heap[k];
    int j = k << 1;
    while (j <= w.heap_len) {
        if (j < w.heap_len && smaller(t, w.heap[j + 1], w.heap[j], w.depth)) j++;
        if (smaller(t, v, w.heap[j], w.depth)) break;
        w.heap[k] = w.heap[j];
        k = j;
        j <<= 1;
    }
    w.heap[k] = v;
}

// kind: 0 litlen (static tree, extra base 257), 1 dist (static 5 bits), 2 bl
template <class Tree>
ZZ_FN void gen_bitlen(TreeWork& w, Tree& t, int kind, uint64_t& opt_len, uint64_t& static_len) {
    const int max_code = t.max_code;
    const int max_length = kind == 2 ? MAX_BL_BITS : MAX_BITS;
    int overflow = 0;
    for (int bits = 0; bits <= MAX_BITS; bits++) w.bl_count[bits] = 0;
    t.len[w.heap[w.heap_max]] = 0;  // root
    int h;
    for (h = w.heap_max + 1; h < HEAP_SIZE; h++) {
        const int n = w.heap[h];
        int bits = t.len[t.dad[n]] + 1;
        if (bits > max_length) bits = max_length, overflow++;
        t.len[n] = (uint16_t)bits;
        if (n > max_code) continue;  // not a leaf
        w.bl_count[bits]++;
        uint32_t xbits = 0;
        if (kind == 0 && n >= 257) xbits = extra_lbits(n - 257);
        if (kind == 1) xbits = extra_dbits(n);
        if (kind == 2) xbits = extra_blbits(n);
        const uint64_t f = t.freq[n];
        opt_len += f * (uint64_t)(bits + xbits);
        if (kind == 0) static_len += f * (uint64_t)(static_llen(n) + xbits);
        if (kind == 1) static_len += f * (uint64_t)(5 + xbits);
    }
    if (overflow == 0) return;
    do {
        int bits = max_length - 1;
        while (w.bl_count[bits] == 0) bits--;
        w.bl_count[bits]--;
        w.bl_count[bits + 1] += 2;
        w.bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    h = HEAP_SIZE;
    for (int bits = max_length; bits != 0; bits--) {
        int n = w.bl_count[bits];
        while (n != 0) {
            const int m = w.heap[--h];
            if (m > max_code) continue;
            if ((unsigned)t.len[m] != (unsigned)bits) {
                opt_len += ((uint64_t)bits - t.len[m]) * t.freq[m];  // (wraps like zlib's ulg when shorter)
                t.len[m] = (uint16_t)bits;
            }
            n--;
        }
    }
}

template <class Tree>
ZZ_FN void gen_codes(Tree& t, int max_code, const uint16_t* bl_count) {
    uint16_t next_code[MAX_BITS + 1];
    uint32_t code = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        const int len = t.len[n];
        if (len == 0) continue;
        t.code[n] = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

template <class Tree>
ZZ_FN void build_tree(TreeWork& w, Tree& t, int kind, int elems, uint64_t& opt_len, uint64_t& static_len) {
    int n, m, max_code = -1, node;
    w.heap_len = 0, w.heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (t.freq[n] != 0) {
            w.heap[++(w.heap_len)] = max_code = n;
            w.depth[n] = 0;
        } else {
            t.len[n] = 0;
        }
    }
    while (w.heap_len < 2) {
        node = w.heap[++(w.heap_len)] = (max_code < 2 ? ++max_code : 0);
        t.freq[node] = 1;
        w.depth[node] = 0;
        opt_len--;
        if (kind == 0) static_len -= static_llen(node);
        if (kind == 1) static_len -= 5;
    }
    t.max_code = max_code;
    for (n = w.heap_len / 2; n >= 1; n--) pqdownheap(w, t, n);
    node = elems;
    do {
        n = w.heap[1];  // pqremove
        w.heap[1] = w.heap[w.heap_len--];
        pqdownheap(w, t, 1);
        m = w.heap[1];
        w.heap[--(w.heap_max)] = n;
        w.heap[--(w.heap_max)] = m;
        t.freq[node] = t.freq[n] + t.freq[m];
        w.depth[node] = (uint8_t)((w.depth[n] >= w.depth[m] ? w.depth[n] : w.depth[m]) + 1);
        t.dad[n] = t.dad[m] = (uint16_t)node;
        w.heap[1] = node++;
        pqdownheap(w, t, 1);
    } while (w.heap_len >= 2);
    w.heap[--(w.heap_max)] = w.heap[1];
    gen_bitlen(w, t, kind, opt_len, static_len);
    gen_codes(t, max_code, w.bl_count);
}

// scan_tree / send_tree walk: calls f(kind, value) per emitted code-length
// symbol: kind 0 = a plain length (value), 1 = REP_3_6 (count), 2 = REPZ_3_10,
// 3 = REPZ_11_138.  scan_tree's frequency counting and send_tree's emission
// are the same walk.  `len(i)` must return the guard 0xffff at max_code + 1.
template <class LEN, class F>
ZZ_FN void rle_walk(const LEN& lenf, int max_code, F& f) {
    int prevlen = -1, curlen, nextlen = lenf(0), count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = lenf(n + 1);
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            do { f(0, curlen); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                f(0, curlen);
                count--;
            }
            f(1, count);
        } else if (count <= 10) {
            f(2, count);
        } else {
            f(3, count);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) {
            max_count = 138, min_count = 3;
        } else if (curlen == nextlen) {
            max_count = 6, min_count = 3;
        } else {
            max_count = 7, min_count = 4;
        }
    }
}

// ---- _tr_flush_block: the block's plan --------------------------------------
constexpr uint32_t BT_STORED = 0, BT_STATIC = 1, BT_DYN = 2;
struct BlockWork {
    LTree lt;
    DTree dt;
    BTree bt;
    TreeWork w;
};
struct BlockPlan {
    uint32_t type;
    uint32_t max_blindex;
    uint64_t opt_len, static_len;
};
// lt.freq / dt.freq must hold the block's symbol counts (END_BLOCK included).
ZZ_FN BlockPlan plan_block(BlockWork& bw, uint32_t stored_len, bool in_win) {
    BlockPlan pl{};
    uint64_t opt = 0, stat = 0;
    build_tree(bw.w, bw.lt, 0, L_CODES, opt, stat);
    build_tree(bw.w, bw.dt, 1, D_CODES, opt, stat);
    // build_bl_tree
    for (int i = 0; i < BL_CODES; i++) bw.bt.freq[i] = 0;
    {
        auto cnt = [&](int k, int v) {
            if (k == 0) bw.bt.freq[v]++;
            else bw.bt.freq[k == 1 ? REP_3_6 : k == 2 ? REPZ_3_10 : REPZ_11_138]++;
        };
        const int lm = bw.lt.max_code, dm = bw.dt.max_code;
        auto ll = [&](int i) -> int { return i == lm + 1 ? 0xffff : bw.lt.len[i]; };
        auto dl = [&](int i) -> int { return i == dm + 1 ? 0xffff : bw.dt.len[i]; };
        rle_walk(ll, lm, cnt);
        rle_walk(dl, dm, cnt);
    }
    uint64_t bl_opt = 0, bl_stat = 0;
    build_tree(bw.w, bw.bt, 2, BL_CODES, bl_opt, bl_stat);
    opt += bl_opt;
    int mb;
    for (mb = BL_CODES - 1; mb >= 3; mb--)
        if (bw.bt.len[bl_order(mb)] != 0) break;
    opt += 3 * ((uint64_t)mb + 1) + 5 + 5 + 4;
    pl.max_blindex = (uint32_t)mb;
    pl.opt_len = opt;
    pl.static_len = stat;
    uint64_t opt_lenb = (opt + 3 + 7) >> 3;
    const uint64_t static_lenb = (stat + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if ((uint64_t)stored_len + 4 <= opt_lenb && in_win) pl.type = BT_STORED;
    else if (static_lenb == opt_lenb) pl.type = BT_STATIC;
    else pl.type = BT_DYN;
    return pl;
}

// Bits of the block header + trees (dynamic: send_all_trees), fed to
// put(value, nbits) in stream order; the 3 block-type bits come first.
template <class PUT>
ZZ_FN void send_header(const BlockWork& bw, const BlockPlan& pl, bool last, PUT& put) {
    if (pl.type == BT_STATIC) {
        put((1u << 1) + (last ? 1u : 0u), 3);
        return;
    }
    if (pl.type == BT_STORED) {
        put(last ? 1u : 0u, 3);
        return;
    }
    put((2u << 1) + (last ? 1u : 0u), 3);
    const int lcodes = bw.lt.max_code + 1, dcodes = bw.dt.max_code + 1, blcodes = (int)pl.max_blindex + 1;
    put((uint32_t)(lcodes - 257), 5);
    put((uint32_t)(dcodes - 1), 5);
    put((uint32_t)(blcodes - 4), 4);
    for (int rank = 0; rank < blcodes; rank++) put(bw.bt.len[bl_order(rank)], 3);
    auto snd = [&](int k, int v) {
        if (k == 0) {
            put(bw.bt.code[v], bw.bt.len[v]);
        } else if (k == 1) {
            put(bw.bt.code[REP_3_6], bw.bt.len[REP_3_6]);
            put((uint32_t)(v - 3), 2);
        } else if (k == 2) {
            put(bw.bt.code[REPZ_3_10], bw.bt.len[REPZ_3_10]);
            put((uint32_t)(v - 3), 3);
        } else {
            put(bw.bt.code[REPZ_11_138], bw.bt.len[REPZ_11_138]);
            put((uint32_t)(v - 11), 7);
        }
    };
    const int lm = bw.lt.max_code, dm = bw.dt.max_code;
    auto ll = [&](int i) -> int { return i == lm + 1 ? 0xffff : bw.lt.len[i]; };
    auto dl = [&](int i) -> int { return i == dm + 1 ? 0xffff : bw.dt.len[i]; };
    rle_walk(ll, lm, snd);
    rle_walk(dl, dm, snd);
}

// code (bit-reversed) and bits of one symbol under the block's trees:
// out[0..3] = (code, nbits) pairs: litlen code, length extra, dist code, dist extra
struct SymBits {
    uint32_t v[4], n[4];
};
ZZ_INL SymBits sym_bits(uint32_t sym, bool stat, const uint16_t* lcode, const uint16_t* llen, const uint16_t* dcode,
                        const uint16_t* dlen) {
    SymBits s{{0, 0, 0, 0}, {0, 0, 0, 0}};
    if (!(sym & 0x80000000u)) {
        const int c = (int)(sym & 0xFF);
        s.v[0] = stat ? static_lcode(c) : lcode[c];
        s.n[0] = stat ? static_llen(c) : llen[c];
        return s;
    }
    const uint32_t lc = (sym >> 16) & 0xFF;  // len - 3
    const uint32_t dist = (sym & 0xFFFF) + 1;
    const int code = (int)len_code(lc + 3);
    const int ls = code + LITERALS + 1;
    s.v[0] = stat ? static_lcode(ls) : lcode[ls];
    s.n[0] = stat ? static_llen(ls) : llen[ls];
    s.n[1] = extra_lbits(code);
    s.v[1] = lc - base_length(code);
    const int dc = (int)dist_code(dist);
    s.v[2] = stat ? bi_reverse((uint32_t)dc, 5) : dcode[dc];
    s.n[2] = stat ? 5u : dlen[dc];
    s.n[3] = extra_dbits(dc);
    s.v[3] = (dist - 1) - base_dist(dc);
    return s;
}

}  // namespace zz
