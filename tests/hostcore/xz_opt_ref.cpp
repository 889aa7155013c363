// TEST INFRASTRUCTURE ONLY: a serial restatement of the GPU xz encoder's
// optimal-parse mode (zarr_amd/csrc/zcg_xz_opt.hip, presets 4-9), step for
// step, so tests/test_gpu_encode.py can compare the GPU's streams byte for
// byte (liblzma decoding them is the reference-side check).  Never linked
// into the product.
//
// The algorithm (the GPU kernels' contract):
//   * match candidates per position p of the serialised chunk s[0, n):
//     the nearest q in [p-64, p) with s[q..q+1] == s[p..p+1] (p + 3 <= n),
//     then a 4-byte hash chain (20-bit multiplicative hash, nearest first, 16
//     links, distances < the preset's dictionary and < 2^23) keeping strictly
//     longer matches (>= 4; stop at 64 bytes or the maximum); the three
//     longest candidates are kept (lengths ascending);
//   * the chunk is coded in 256 KiB segments, each an independent LZMA2 run:
//     a state reset (+ properties) at its first LZMA chunk, the dictionary
//     shared (segment 0's first chunk resets it); LZMA lc=0 lp=0 pb=2;
//   * the parse: windows of <= 256 positions (clipped to the segment end);
//     a shortest path over literal / short-rep / rep0-3 / match arcs whose
//     prices (1/16 bit) come from the probabilities at the window start;
//     lengths 2..8 and the last three of each rep / candidate range; ties go
//     to the earlier node, then to literal < short rep < rep0..3 < match,
//     shorter first;
//   * LZMA2 chunks end before 65 472 compressed bytes (then the window is
//     re-planned); a chunk that does not shrink is stored uncompressed and the
//     next LZMA chunk resets the state (liblzma's encoder rule).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

enum : u32 {
    E_IS_MATCH = 0, E_IS_REP = 192, E_IS_REP_G0 = 204, E_IS_REP_G1 = 216, E_IS_REP_G2 = 228,
    E_IS_REP0_LONG = 240, E_POS_SLOT = 432, E_SPEC_POS = 688, E_ALIGN = 802, E_LEN = 818, E_REP_LEN = 1332,
    E_LITERAL = 1846, XO_PROBS = 1846 + 0x300
};
enum : u32 { EL_CHOICE = 0, EL_CHOICE2 = 1, EL_LOW = 2, EL_MID = 130, EL_HIGH = 258 };
#ifndef XO_SEG_KB
#define XO_SEG_KB 256
#endif
constexpr u32 XO_SEG = XO_SEG_KB << 10, XO_WIN = 256, XO_K = 3, XO_DEPTH = 16, XO_NICE = 64, XO_W2 = 64, XO_LENS = 8;
constexpr u32 XO_CMAX = 65536 - 64, XO_MAXLEN = 273;
constexpr u32 XO_PROPS = (2 * 5 + 0) * 9 + 0;  // pb=2 lp=0 lc=0

// -log2((i*16+8)/2048) in 1/16 bit, rounded
const u8 kPrice[128] = {128, 103, 91, 83, 77, 73, 69, 65, 63, 60, 58, 56, 54, 52, 50, 49, 47, 46, 45, 43, 42, 41,
                        40, 39, 38, 37, 36, 35, 35, 34, 33, 32, 32, 31, 30, 30, 29, 28, 28, 27, 27, 26, 25, 25,
                        24, 24, 23, 23, 22, 22, 21, 21, 21, 20, 20, 19, 19, 18, 18, 18, 17, 17, 17, 16, 16, 15,
                        15, 15, 14, 14, 14, 13, 13, 13, 12, 12, 12, 12, 11, 11, 11, 10, 10, 10, 10, 9, 9, 9,
                        9, 8, 8, 8, 7, 7, 7, 7, 7, 6, 6, 6, 6, 5, 5, 5, 5, 4, 4, 4, 4, 4, 3, 3,
                        3, 3, 3, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 0, 0, 0};

u32 crc32_tab[256];
u64 crc64_tab[256];
void init_tabs() {
    static bool done = false;
    if (done) return;
    done = true;
    for (u32 i = 0; i < 256; i++) {
        u32 c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc32_tab[i] = c;
        u64 d = i;
        for (int k = 0; k < 8; k++) d = (d & 1) ? 0xC96C5795D7870F42ull ^ (d >> 1) : d >> 1;
        crc64_tab[i] = d;
    }
}

inline u32 st_lit(u32 s) { return s < 4 ? 0 : (s < 10 ? s - 3 : s - 6); }
inline u32 st_match(u32 s) { return s < 7 ? 7 : 10; }
inline u32 st_rep(u32 s) { return s < 7 ? 8 : 11; }
inline u32 st_short(u32 s) { return s < 7 ? 9 : 11; }
inline u32 slot_of(u32 d) {
    if (d < 4) return d;
    const u32 lg = 31 - __builtin_clz(d);
    return 2 * lg + ((d >> (lg - 1)) & 1);
}

struct Rc {  // LZMA range encoder + model
    std::vector<u8> out;
    u64 low = 0;
    u32 range = 0xFFFFFFFFu, cache = 0;
    u64 cache_size = 1;
    u16 pr[XO_PROBS];
    void reset_rc() { low = 0; range = 0xFFFFFFFFu; cache = 0; cache_size = 1; }
    void reset_probs() { for (u32 i = 0; i < XO_PROBS; i++) pr[i] = 1024; }
    void shift_low() {
        if ((u32)low < 0xFF000000u || (u32)(low >> 32) != 0) {
            const u32 carry = (u32)(low >> 32);
            u32 temp = cache;
            do {
                out.push_back((u8)((temp + carry) & 0xFF));
                temp = 0xFF;
            } while (--cache_size != 0);
            cache = (u32)(low >> 24) & 0xFF;
        }
        cache_size++;
        low = (low & 0x00FFFFFFull) << 8;
    }
    void bit(u32 i, u32 b) {
        const u32 p = pr[i], bound = (range >> 11) * p;
        if (!b) { range = bound; pr[i] = (u16)(p + ((2048 - p) >> 5)); }
        else { low += bound; range -= bound; pr[i] = (u16)(p - (p >> 5)); }
        while (range < (1u << 24)) { range <<= 8; shift_low(); }
    }
    void tree(u32 base, u32 nb, u32 v) {
        u32 m = 1;
        for (int i = (int)nb - 1; i >= 0; i--) { const u32 b = (v >> i) & 1; bit(base + m, b); m = (m << 1) | b; }
    }
    void rtree(u32 base, u32 nb, u32 v) {
        u32 m = 1;
        for (u32 i = 0; i < nb; i++) { const u32 b = (v >> i) & 1; bit(base + m, b); m = (m << 1) | b; }
    }
    void direct(u32 v, u32 nb) {
        for (int i = (int)nb - 1; i >= 0; i--) {
            range >>= 1;
            if ((v >> i) & 1) low += range;
            while (range < (1u << 24)) { range <<= 8; shift_low(); }
        }
    }
    void length(u32 lb, u32 l, u32 ps) {
        if (l < 8) { bit(lb + EL_CHOICE, 0); tree(lb + EL_LOW + (ps << 3), 3, l); }
        else if (l < 16) { bit(lb + EL_CHOICE, 1); bit(lb + EL_CHOICE2, 0); tree(lb + EL_MID + (ps << 3), 3, l - 8); }
        else { bit(lb + EL_CHOICE, 1); bit(lb + EL_CHOICE2, 1); tree(lb + EL_HIGH, 8, l - 16); }
    }
    void distance(u32 d, u32 len) {
        const u32 lps = len - 2 < 3 ? len - 2 : 3, slot = slot_of(d);
        tree(E_POS_SLOT + (lps << 6), 6, slot);
        if (slot >= 4) {
            const u32 nd = (slot >> 1) - 1, base = (2 | (slot & 1)) << nd, red = d - base;
            if (slot < 14) rtree(E_SPEC_POS + base - slot - 1, nd, red);
            else { direct(red >> 4, nd - 4); rtree(E_ALIGN, 4, red & 15); }
        }
    }
    // prices from the current probabilities
    u32 pb(u32 i, u32 b) const { const u32 p = pr[i]; return kPrice[(b ? 2048 - p : p) >> 4]; }
    u32 ptree(u32 base, u32 nb, u32 v) const {
        u32 m = 1, s = 0;
        for (int i = (int)nb - 1; i >= 0; i--) { const u32 b = (v >> i) & 1; s += pb(base + m, b); m = (m << 1) | b; }
        return s;
    }
    u32 prtree(u32 base, u32 nb, u32 v) const {
        u32 m = 1, s = 0;
        for (u32 i = 0; i < nb; i++) { const u32 b = (v >> i) & 1; s += pb(base + m, b); m = (m << 1) | b; }
        return s;
    }
    u32 plen(u32 lb, u32 l, u32 ps) const {
        if (l < 8) return pb(lb + EL_CHOICE, 0) + ptree(lb + EL_LOW + (ps << 3), 3, l);
        if (l < 16) return pb(lb + EL_CHOICE, 1) + pb(lb + EL_CHOICE2, 0) + ptree(lb + EL_MID + (ps << 3), 3, l - 8);
        return pb(lb + EL_CHOICE, 1) + pb(lb + EL_CHOICE2, 1) + ptree(lb + EL_HIGH, 8, l - 16);
    }
    u32 pdist(u32 d, u32 len) const {
        const u32 lps = len - 2 < 3 ? len - 2 : 3, slot = slot_of(d);
        u32 s = ptree(E_POS_SLOT + (lps << 6), 6, slot);
        if (slot >= 4) {
            const u32 nd = (slot >> 1) - 1, base = (2 | (slot & 1)) << nd, red = d - base;
            if (slot < 14) s += prtree(E_SPEC_POS + base - slot - 1, nd, red);
            else s += (nd - 4) * 16 + prtree(E_ALIGN, 4, red & 15);
        }
        return s;
    }
    u32 plit(u32 sym, u32 st, u32 mbyte) const {  // lc = lp = 0: one literal coder
        if (st < 7) return ptree(E_LITERAL, 8, sym);
        u32 s = 0, mb = mbyte, off = 0x100, m = 1;
        for (int k = 7; k >= 0; k--) {
            const u32 b = (sym >> k) & 1;
            mb <<= 1;
            const u32 mbit = mb & off;
            s += pb(E_LITERAL + off + mbit + m, b);
            m = (m << 1) | b;
            off &= b ? mbit : ~mbit;
        }
        return s;
    }
    void lit(u32 sym, u32 st, u32 mbyte) {
        if (st < 7) { tree(E_LITERAL, 8, sym); return; }
        u32 mb = mbyte, off = 0x100, m = 1;
        for (int k = 7; k >= 0; k--) {
            const u32 b = (sym >> k) & 1;
            mb <<= 1;
            const u32 mbit = mb & off;
            bit(E_LITERAL + off + mbit + m, b);
            m = (m << 1) | b;
            off &= b ? mbit : ~mbit;
        }
    }
};

// candidates of every position: XO_K (len, dist) pairs, lengths ascending, 0 = none
void find_candidates(const u8* s, u32 n, u64 dsize, std::vector<u32>& cl, std::vector<u32>& cd) {
    cl.assign((u64)n * XO_K, 0);
    cd.assign((u64)n * XO_K, 0);
    const u32 HB = 20;
    std::vector<int> head(1u << HB, -1), prev(n, -1);
    const u64 dmax = dsize < (1ull << 23) ? dsize : (1ull << 23);
    for (u32 p = 0; p < n; p++) {
        u32 L[24], Dd[24], c = 0, best = 1;
        const u32 mx = n - p < XO_MAXLEN ? n - p : XO_MAXLEN;
        if (p + 3 <= n) {  // nearest 2-byte repeat within XO_W2
            for (u32 q = p; q-- > (p > XO_W2 ? p - XO_W2 : 0);) {
                if (s[q] == s[p] && s[q + 1] == s[p + 1]) {
                    u32 l = 0;
                    while (l < mx && s[q + l] == s[p + l]) l++;
                    best = l;
                    L[c] = l; Dd[c] = p - q - 1; c++;
                    break;
                }
            }
        }
        if (p + 4 <= n) {
            u32 v;
            memcpy(&v, s + p, 4);
            const u32 h = (v * 2654435761u) >> (32 - HB);
            if (best < 3) best = 3;
            int q = head[h];
            for (u32 dep = 0; dep < XO_DEPTH && q >= 0; dep++) {
                if ((u64)(p - (u32)q) > dmax) break;
                u32 l = 0;
                while (l < mx && s[q + l] == s[p + l]) l++;
                if (l > best) {
                    best = l;
                    L[c] = l; Dd[c] = p - (u32)q - 1; c++;
                    if (l >= XO_NICE || l == mx) break;
                }
                q = prev[q];
            }
            prev[p] = head[h];
            head[h] = (int)p;
        }
        const u32 k0 = c > XO_K ? c - XO_K : 0;
        for (u32 k = k0; k < c; k++) { cl[(u64)p * XO_K + k - k0] = L[k]; cd[(u64)p * XO_K + k - k0] = Dd[k]; }
    }
}

struct Node {
    u64 key;  // price << 20 | source node << 11 | arc
    u32 state, reps[4];
};
constexpr u64 KEY_NONE = ~0ull;
inline u64 mkkey(u32 price, u32 src, u32 arc) { return ((u64)price << 20) | ((u64)src << 11) | arc; }
// arcs: 0 literal, 1 short rep, 2 + r*274 + len rep r, 1100 + len match
inline bool keep_len(u32 l, u32 L) { return l <= XO_LENS || L - l <= 2; }

}  // namespace

extern "C" uint64_t zref_xz_opt_bound(uint64_t n) { return n + n / 16 + 4096; }

// The .xz stream of s[0, n) (CRC64) into out (cap >= zref_xz_opt_bound(n)); returns its length.
extern "C" uint64_t zref_xz_opt_encode(const uint8_t* s, uint64_t n64, uint32_t dict_lg, uint8_t* out, uint64_t cap) {
    init_tabs();
    const u32 n = (u32)n64;
    std::vector<u8> O;
    const u8 hdr[12] = {0xFD, 0x37, 0x7A, 0x58, 0x5A, 0x00, 0x00, 0x04, 0xE6, 0xD6, 0xB4, 0x46};
    O.insert(O.end(), hdr, hdr + 12);
    u64 unpadded = 0;
    if (n > 0) {
        u32 hc = 0xFFFFFFFFu;
        const u8 bh[8] = {0x02, 0x00, 0x21, 0x01, (u8)(2 * (dict_lg - 12)), 0, 0, 0};
        for (u8 x : bh) { O.push_back(x); hc = crc32_tab[(hc ^ x) & 0xFF] ^ (hc >> 8); }
        hc = ~hc;
        for (int k = 0; k < 4; k++) O.push_back((hc >> (8 * k)) & 0xFF);
        const u64 cdata0 = O.size();
        std::vector<u32> cl, cd;
        find_candidates(s, n, 1ull << dict_lg, cl, cd);
        Rc C;
        std::vector<Node> nd(XO_WIN + 1);
        std::vector<Node> path;
        for (u32 s0 = 0; s0 < n; s0 += XO_SEG) {
            const u32 s1 = n - s0 < XO_SEG ? n : s0 + XO_SEG;
            bool need_dict = s0 == 0, need_props = true, need_state = true;
            u32 state = 0, reps[4] = {0, 0, 0, 0};
            u32 p = s0;
            while (p < s1) {
                // ---- one LZMA2 chunk ----
                if (need_state) { C.reset_probs(); state = 0; reps[0] = reps[1] = reps[2] = reps[3] = 0; }
                C.reset_rc();
                C.out.clear();
                const u32 u0 = p;
                size_t pi = 0;
                path.clear();
                while (p < s1 && C.out.size() + C.cache_size + 5 < XO_CMAX) {
                    if (pi == path.size()) {
                        // ---- plan a window [p, e) ----
                        const u32 e = s1 - p < XO_WIN ? s1 : p + XO_WIN, W = e - p;
                        for (u32 j = 0; j <= W; j++) nd[j].key = KEY_NONE;
                        nd[0].key = 0;
                        nd[0].state = state;
                        memcpy(nd[0].reps, reps, sizeof(reps));
                        for (u32 i = 0; i < W; i++) {
                            Node& a = nd[i];
                            if (i > 0) {  // this node's state and reps from its best arc
                                const u32 src = (u32)(a.key >> 11) & 511, arc = (u32)a.key & 2047;
                                const Node& b = nd[src];
                                if (arc == 0) { a.state = st_lit(b.state); memcpy(a.reps, b.reps, sizeof(reps)); }
                                else if (arc == 1) { a.state = st_short(b.state); memcpy(a.reps, b.reps, sizeof(reps)); }
                                else if (arc < 1100) {
                                    const u32 r = (arc - 2) / 274;
                                    a.state = st_rep(b.state);
                                    a.reps[0] = b.reps[r];
                                    for (u32 k = 0, t = 1; k < 4; k++) if (k != r) a.reps[t++] = b.reps[k];
                                } else {
                                    const u32 l = arc - 1100, at0 = p + src;
                                    u32 d = 0;
                                    for (u32 k = 0; k < XO_K; k++) {  // the candidate whose range holds l
                                        const u32 Lk = cl[(u64)at0 * XO_K + k];
                                        if (Lk && l <= (Lk < e - at0 ? Lk : e - at0)) { d = cd[(u64)at0 * XO_K + k]; break; }
                                    }
                                    a.state = st_match(b.state);
                                    a.reps[0] = d; a.reps[1] = b.reps[0]; a.reps[2] = b.reps[1]; a.reps[3] = b.reps[2];
                                }
                            }
                            const u32 P = (u32)(a.key >> 20), at = p + i, ps = at & 3, st = a.state;
                            const u32* rp = a.reps;
                            auto relax = [&](u32 j, u32 price, u32 arc) {
                                const u64 k = mkkey(price, i, arc);
                                if (k < nd[j].key) nd[j].key = k;
                            };
                            const u32 mbyte = at > rp[0] ? s[at - rp[0] - 1] : 0;
                            relax(i + 1, P + C.pb(E_IS_MATCH + (st << 4) + ps, 0) + C.plit(s[at], st, mbyte), 0);
                            const u32 mbase = P + C.pb(E_IS_MATCH + (st << 4) + ps, 1);
                            const u32 rbase = mbase + C.pb(E_IS_REP + st, 1);
                            if (at > rp[0] && s[at] == mbyte)
                                relax(i + 1, rbase + C.pb(E_IS_REP_G0 + st, 0) + C.pb(E_IS_REP0_LONG + (st << 4) + ps, 0), 1);
                            const u32 mx = e - at < XO_MAXLEN ? e - at : XO_MAXLEN;
                            for (u32 r = 0; r < 4; r++) {
                                if (at <= rp[r]) continue;
                                u32 rl = 0;
                                while (rl < mx && s[at + rl] == s[at - rp[r] - 1 + rl]) rl++;
                                if (rl < 2) continue;
                                u32 pr = rbase;
                                if (r == 0) pr += C.pb(E_IS_REP_G0 + st, 0) + C.pb(E_IS_REP0_LONG + (st << 4) + ps, 1);
                                else {
                                    pr += C.pb(E_IS_REP_G0 + st, 1);
                                    if (r == 1) pr += C.pb(E_IS_REP_G1 + st, 0);
                                    else pr += C.pb(E_IS_REP_G1 + st, 1) + C.pb(E_IS_REP_G2 + st, r - 2);
                                }
                                for (u32 l = 2; l <= rl; l++)
                                    if (keep_len(l, rl)) relax(i + l, pr + C.plen(E_REP_LEN, l - 2, ps), 2 + r * 274 + l);
                            }
                            const u32 mb0 = mbase + C.pb(E_IS_REP + st, 0);
                            u32 lprev = 1;
                            for (u32 k = 0; k < XO_K; k++) {
                                const u32 Lk = cl[(u64)at * XO_K + k];
                                if (!Lk) continue;
                                const u32 L = Lk < mx ? Lk : mx, d = cd[(u64)at * XO_K + k];
                                for (u32 l = lprev + 1 > 2 ? lprev + 1 : 2; l <= L; l++)
                                    if (keep_len(l, L)) relax(i + l, mb0 + C.plen(E_LEN, l - 2, ps) + C.pdist(d, l), 1100 + l);
                                if (L > lprev) lprev = L;
                            }
                        }
                        // the path to the window end
                        path.clear();
                        for (u32 j = W; j > 0;) {
                            const u32 src = (u32)(nd[j].key >> 11) & 511, arc = (u32)nd[j].key & 2047;
                            Node t;
                            t.key = arc;
                            t.state = j - src;  // length
                            if (arc >= 1100) {
                                const u32 at0 = p + src, l = arc - 1100;
                                t.reps[0] = 0;
                                for (u32 k = 0; k < XO_K; k++) {
                                    const u32 Lk = cl[(u64)at0 * XO_K + k];
                                    if (Lk && l <= (Lk < e - at0 ? Lk : e - at0)) { t.reps[0] = cd[(u64)at0 * XO_K + k]; break; }
                                }
                            }
                            path.push_back(t);
                            j = src;
                        }
                        std::reverse(path.begin(), path.end());
                        pi = 0;
                    }
                    // ---- code one symbol of the path ----
                    const Node& a = path[pi++];
                    const u32 arc = (u32)a.key, len = a.state, ps = p & 3;
                    if (arc == 0) {
                        C.bit(E_IS_MATCH + (state << 4) + ps, 0);
                        C.lit(s[p], state, p > reps[0] ? s[p - reps[0] - 1] : 0);
                        state = st_lit(state);
                    } else if (arc == 1) {
                        C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                        C.bit(E_IS_REP + state, 1);
                        C.bit(E_IS_REP_G0 + state, 0);
                        C.bit(E_IS_REP0_LONG + (state << 4) + ps, 0);
                        state = st_short(state);
                    } else if (arc < 1100) {
                        const u32 r = (arc - 2) / 274;
                        C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                        C.bit(E_IS_REP + state, 1);
                        if (r == 0) {
                            C.bit(E_IS_REP_G0 + state, 0);
                            C.bit(E_IS_REP0_LONG + (state << 4) + ps, 1);
                        } else {
                            C.bit(E_IS_REP_G0 + state, 1);
                            if (r == 1) C.bit(E_IS_REP_G1 + state, 0);
                            else { C.bit(E_IS_REP_G1 + state, 1); C.bit(E_IS_REP_G2 + state, r - 2); }
                            const u32 d = reps[r];
                            for (u32 k = r; k > 0; k--) reps[k] = reps[k - 1];
                            reps[0] = d;
                        }
                        C.length(E_REP_LEN, len - 2, ps);
                        state = st_rep(state);
                    } else {
                        const u32 d = a.reps[0];
                        C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                        C.bit(E_IS_REP + state, 0);
                        C.length(E_LEN, len - 2, ps);
                        C.distance(d, len);
                        reps[3] = reps[2]; reps[2] = reps[1]; reps[1] = reps[0]; reps[0] = d;
                        state = st_match(state);
                    }
                    p += len;
                }
                for (int k = 0; k < 5; k++) C.shift_low();
                const u32 usz = p - u0 - 1;
                if (C.out.size() >= p - u0) {  // stored: liblzma's rule, the state resets next
                    O.push_back(need_dict ? 0x01 : 0x02);
                    O.push_back((usz >> 8) & 0xFF);
                    O.push_back(usz & 0xFF);
                    O.insert(O.end(), s + u0, s + p);
                    need_dict = false;
                    need_state = true;
                    continue;
                }
                const u32 csz = (u32)C.out.size() - 1;
                const u32 ctl = need_props ? (need_dict ? 0xE0u : 0xC0u) : (need_state ? 0xA0u : 0x80u);
                O.push_back(ctl | (usz >> 16));
                O.push_back((usz >> 8) & 0xFF);
                O.push_back(usz & 0xFF);
                O.push_back((csz >> 8) & 0xFF);
                O.push_back(csz & 0xFF);
                if (need_props) O.push_back(XO_PROPS);
                O.insert(O.end(), C.out.begin(), C.out.end());
                need_dict = need_props = need_state = false;
            }
        }
        O.push_back(0x00);
        const u64 csize = O.size() - cdata0;
        while ((O.size() - cdata0) & 3) O.push_back(0);
        u64 crc = ~0ull;
        for (u32 k = 0; k < n; k++) crc = crc64_tab[(crc ^ s[k]) & 0xFF] ^ (crc >> 8);
        crc = ~crc;
        for (int k = 0; k < 8; k++) O.push_back((u8)(crc >> (8 * k)));
        unpadded = 12 + csize + 8;
    }
    const u64 idx0 = O.size();
    u32 ic = 0xFFFFFFFFu;
    auto iout = [&](u32 b) { O.push_back((u8)b); ic = crc32_tab[(ic ^ b) & 0xFF] ^ (ic >> 8); };
    auto ivli = [&](u64 v) { while (v >= 0x80) { iout((u32)(v & 0x7F) | 0x80); v >>= 7; } iout((u32)v); };
    iout(0x00);
    ivli(n > 0 ? 1 : 0);
    if (n > 0) { ivli(unpadded); ivli(n); }
    while ((O.size() - idx0) & 3) iout(0x00);
    ic = ~ic;
    for (int k = 0; k < 4; k++) O.push_back((ic >> (8 * k)) & 0xFF);
    const u64 isize = O.size() - idx0;
    const u64 fbw = (u64)(u32)(isize / 4 - 1) | (0x0400ull << 32);
    u32 fc = 0xFFFFFFFFu;
    for (int k = 0; k < 6; k++) fc = crc32_tab[(fc ^ (u32)(fbw >> (8 * k))) & 0xFF] ^ (fc >> 8);
    fc = ~fc;
    for (int k = 0; k < 4; k++) O.push_back((fc >> (8 * k)) & 0xFF);
    for (int k = 0; k < 6; k++) O.push_back((u8)(fbw >> (8 * k)));
    O.push_back(0x59);
    O.push_back(0x5A);
    if (O.size() > cap) return 0;
    memcpy(out, O.data(), O.size());
    return O.size();
}
