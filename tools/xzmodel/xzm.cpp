// tools/xzmodel/xzm.cpp — DEV TOOLING ONLY (never linked into the product).
// A CPU model of the GPU xz encoder (zarr_amd/csrc/zcg_xz_enc.hip) for trying
// parse strategies quickly: the same .xz container (stream header, one block,
// LZMA2 chunks, CRC64, index, footer), the same LZMA model and range coder.
//   mode 0: the GPU kernel's parse (rep0 only, greedy + one-step lazy)
//   mode 1: price-driven optimal parse over windows (reps 0-3, short rep,
//           matched literals, every match length), liblzma-style prices
// Build: g++ -O2 -shared -fPIC -o libxzm.so xzm.cpp ; driven by xzm.py.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

namespace {

enum : u32 {
    E_IS_MATCH = 0, E_IS_REP = 192, E_IS_REP_G0 = 204, E_IS_REP_G1 = 216, E_IS_REP_G2 = 228,
    E_IS_REP0_LONG = 240, E_POS_SLOT = 432, E_SPEC_POS = 688, E_ALIGN = 802, E_LEN = 818, E_REP_LEN = 1332,
    E_LITERAL = 1846
};
enum : u32 { EL_CHOICE = 0, EL_CHOICE2 = 1, EL_LOW = 2, EL_MID = 130, EL_HIGH = 258 };
constexpr u32 PROBS = 1846 + (0x300u << 4);
constexpr u32 CMAX = 65536 - 64, UMAX = (1u << 21) - 273;
constexpr u32 PB = 2, MATCH_MAX = 273;
u32 LC = 3, LP = 0;
inline u32 litctx(u32 at, u32 pv) { return ((at & ((1u << LP) - 1)) << LC) + (LC ? pv >> (8 - LC) : 0); }

u32 crc32_tab[256];
u64 crc64_tab[256];
u32 price_tab[128];  // -log2(p) in 1/16 bit, p = (i*16+8)/2048
bool tabs = false;
int g_short = 1;
int g_lens = 0;
u32 g_seg = 0;
int g_k3 = 0;
u32 g_w2 = 0;
u32 g_kmax = 0;
u32 g_group = 64;  // > 0: the nearest 2-byte repeat only within this distance  // 1: the chain key is the exact 3-byte prefix  // > 0: a state reset every g_seg input bytes (matches may cross)  // > 0: a match's lengths relaxed: 2..g_lens and the last three
struct Coder;
Coder* g_frz = nullptr;
u16 g_dump[1846 + (0x300u << 4)];
bool g_dumping = false;
void init_tabs() {
    if (tabs) return;
    tabs = true;
    for (u32 i = 0; i < 256; i++) {
        u32 c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc32_tab[i] = c;
        u64 d = i;
        for (int k = 0; k < 8; k++) d = (d & 1) ? 0xC96C5795D7870F42ull ^ (d >> 1) : d >> 1;
        crc64_tab[i] = d;
    }
    for (u32 i = 0; i < 128; i++) {
        const double p = (i * 16.0 + 8.0) / 2048.0;
        double b = -__builtin_log2(p) * 16.0;
        price_tab[i] = (u32)(b + 0.5);
    }
}

struct Coder {
    std::vector<u8>* out;
    u64 low = 0;
    u32 range = 0xFFFFFFFFu, cache = 0;
    u64 cache_size = 1;
    u16 probs[PROBS];
    void reset_rc() { low = 0; range = 0xFFFFFFFFu; cache = 0; cache_size = 1; }
    void reset_probs() { for (u32 i = 0; i < PROBS; i++) probs[i] = 1024; }
    void shift_low() {
        if ((u32)low < 0xFF000000u || (u32)(low >> 32) != 0) {
            const u32 carry = (u32)(low >> 32);
            u32 temp = cache;
            do {
                out->push_back((u8)((temp + carry) & 0xFF));
                temp = 0xFF;
            } while (--cache_size != 0);
            cache = (u32)(low >> 24) & 0xFF;
        }
        cache_size++;
        low = (low & 0x00FFFFFFull) << 8;
    }
    void bit(u32 pi, u32 b) {
        const u32 p = probs[pi];
        const u32 bound = (range >> 11) * p;
        if (b == 0) { range = bound; probs[pi] = (u16)(p + ((2048 - p) >> 5)); }
        else { low += bound; range -= bound; probs[pi] = (u16)(p - (p >> 5)); }
        while (range < (1u << 24)) { range <<= 8; shift_low(); }
    }
    void tree(u32 base, u32 nbits, u32 v) {
        u32 m = 1;
        for (int i = (int)nbits - 1; i >= 0; i--) { const u32 b = (v >> i) & 1; bit(base + m, b); m = (m << 1) | b; }
    }
    void rtree(u32 base, u32 nbits, u32 v) {
        u32 m = 1;
        for (u32 i = 0; i < nbits; i++) { const u32 b = (v >> i) & 1; bit(base + m, b); m = (m << 1) | b; }
    }
    void direct(u32 v, u32 nbits) {
        for (int i = (int)nbits - 1; i >= 0; i--) {
            range >>= 1;
            if ((v >> i) & 1) low += range;
            while (range < (1u << 24)) { range <<= 8; shift_low(); }
        }
    }
    void length(u32 lbase, u32 l, u32 ps) {  // l = len - 2
        if (l < 8) { bit(lbase + EL_CHOICE, 0); tree(lbase + EL_LOW + (ps << 3), 3, l); }
        else if (l < 16) { bit(lbase + EL_CHOICE, 1); bit(lbase + EL_CHOICE2, 0); tree(lbase + EL_MID + (ps << 3), 3, l - 8); }
        else { bit(lbase + EL_CHOICE, 1); bit(lbase + EL_CHOICE2, 1); tree(lbase + EL_HIGH, 8, l - 16); }
    }
    static u32 slot_of(u32 dist) {
        if (dist < 4) return dist;
        const u32 lg = 31 - __builtin_clz(dist);
        return 2 * lg + ((dist >> (lg - 1)) & 1);
    }
    void distance(u32 dist, u32 len) {
        const u32 lps = len - 2 < 3 ? len - 2 : 3;
        const u32 slot = slot_of(dist);
        tree(E_POS_SLOT + (lps << 6), 6, slot);
        if (slot >= 4) {
            const u32 nd = (slot >> 1) - 1;
            const u32 base = (2 | (slot & 1)) << nd;
            const u32 red = dist - base;
            if (slot < 14) rtree(E_SPEC_POS + base - slot - 1, nd, red);
            else { direct(red >> 4, nd - 4); rtree(E_ALIGN, 4, red & 15); }
        }
    }
    // ---- prices (1/16 bit) from the current probabilities ----
    u32 pb(u32 pi, u32 b) const { const u32 p = probs[pi]; return price_tab[(b ? 2048 - p : p) >> 4]; }
    u32 ptree(u32 base, u32 nbits, u32 v) const {
        u32 m = 1, s = 0;
        for (int i = (int)nbits - 1; i >= 0; i--) { const u32 b = (v >> i) & 1; s += pb(base + m, b); m = (m << 1) | b; }
        return s;
    }
    u32 prtree(u32 base, u32 nbits, u32 v) const {
        u32 m = 1, s = 0;
        for (u32 i = 0; i < nbits; i++) { const u32 b = (v >> i) & 1; s += pb(base + m, b); m = (m << 1) | b; }
        return s;
    }
    u32 plen(u32 lbase, u32 l, u32 ps) const {
        if (l < 8) return pb(lbase + EL_CHOICE, 0) + ptree(lbase + EL_LOW + (ps << 3), 3, l);
        if (l < 16) return pb(lbase + EL_CHOICE, 1) + pb(lbase + EL_CHOICE2, 0) + ptree(lbase + EL_MID + (ps << 3), 3, l - 8);
        return pb(lbase + EL_CHOICE, 1) + pb(lbase + EL_CHOICE2, 1) + ptree(lbase + EL_HIGH, 8, l - 16);
    }
    u32 pdist(u32 dist, u32 len) const {
        const u32 lps = len - 2 < 3 ? len - 2 : 3;
        const u32 slot = slot_of(dist);
        u32 s = ptree(E_POS_SLOT + (lps << 6), 6, slot);
        if (slot >= 4) {
            const u32 nd = (slot >> 1) - 1;
            const u32 base = (2 | (slot & 1)) << nd;
            const u32 red = dist - base;
            if (slot < 14) s += prtree(E_SPEC_POS + base - slot - 1, nd, red);
            else s += (nd - 4) * 16 + prtree(E_ALIGN, 4, red & 15);
        }
        return s;
    }
};

struct Out {
    std::vector<u8> v;
    void b(u32 x) { v.push_back((u8)x); }
};

inline u32 st_lit(u32 s) { return s < 4 ? 0 : (s < 10 ? s - 3 : s - 6); }
inline u32 st_match(u32 s) { return s < 7 ? 7 : 10; }
inline u32 st_rep(u32 s) { return s < 7 ? 8 : 11; }
inline u32 st_short(u32 s) { return s < 7 ? 9 : 11; }

struct Matches {  // per position: candidate matches (len ascending, dist)
    std::vector<u32> off;
    std::vector<u32> len, dist;
};

// hash-chain match finder over the whole input (dictionary >= input)
Matches find_matches(const u8* s, u32 n, u32 depth, u32 nice) {
    Matches M;
    M.off.assign(n + 1, 0);
    const u32 HB = g_k3 ? 24 : 20;
    std::vector<int> head(1u << HB, -1), prev(n, -1), h2(1u << 16, -1), h3(1u << 16, -1);
    for (u32 p = 0; p < n; p++) {
        M.off[p] = (u32)M.len.size();
        u32 best = 1;
        const u32 mx0 = std::min<u32>(MATCH_MAX, n - p);
        if (g_short && p + 3 <= n) {  // bt4's hash2 / hash3 heads: the nearest 2- and 3-byte repeats
            const u32 k2 = s[p] | (u32)s[p + 1] << 8;
            const u32 k3 = ((k2 | (u32)s[p + 2] << 16) * 2654435761u) >> 16;
            int q2 = g_short == 2 ? -1 : h2[k2];
            const int q3 = g_short == 3 ? -1 : h3[k3];
            if (g_w2 && q2 >= 0 && p - (u32)q2 > g_w2) q2 = -1;
            for (int q : {q2, q3}) {
                if (q < 0) continue;
                u32 l = 0;
                while (l < mx0 && s[q + l] == s[p + l]) l++;
                if (l > best && (l >= 3 || p - q <= 256)) { best = l; M.len.push_back(l); M.dist.push_back(p - (u32)q - 1); }
            }
            h2[k2] = (int)p;
            h3[k3] = (int)p;
        }
        if (p + (g_k3 ? 3 : 4) <= n) {
            u32 v = 0;
            memcpy(&v, s + p, g_k3 ? 3 : 4);
            const u32 h = g_k3 ? (v & 0xFFFFFF) : (v * 2654435761u) >> (32 - HB);
            int q = head[h];
            u32 cnt = 0;
            if (best < (g_k3 ? 2u : 3u)) best = g_k3 ? 2 : 3;
            const u32 mx = mx0;
            while (q >= 0 && cnt < depth) {
                cnt++;
                u32 l = 0;
                while (l < mx && s[q + l] == s[p + l]) l++;
                if (l > best) {
                    best = l;
                    M.len.push_back(l);
                    M.dist.push_back(p - (u32)q - 1);
                    if (l >= nice || l == mx) break;
                }
                q = prev[q];
            }
            prev[p] = head[h];
            head[h] = (int)p;
        }
        if (g_kmax && M.len.size() - M.off[p] > g_kmax) {  // keep the longest g_kmax candidates
            const u32 o = M.off[p], c = (u32)M.len.size() - o;
            for (u32 k = 0; k < g_kmax; k++) { M.len[o + k] = M.len[o + c - g_kmax + k]; M.dist[o + k] = M.dist[o + c - g_kmax + k]; }
            M.len.resize(o + g_kmax);
            M.dist.resize(o + g_kmax);
        }
    }
    M.off[n] = (u32)M.len.size();
    return M;
}

struct Node {
    u32 price;
    u32 prev;      // position the arc comes from
    u32 kind;      // 0 literal, 1 short rep, 2+i rep i (len), 6 match
    u32 len, dist; // (match) length, distance
    u32 state;
    u32 reps[4];
};

}  // namespace

// Encode `n` bytes into an .xz stream (CRC64); returns the stream length
// (out must hold n + n/8 + 4096 bytes).  mode 0: GPU parse, 1: optimal parse.
extern "C" void xzm_lclp(u32 lc, u32 lp, u32 kmax) { LC = lc; LP = lp; g_kmax = kmax; }
extern "C" void xzm_group(u32 g) { g_group = g; }
extern "C" void xzm_set(int shortm, int lens, u32 seg, int k3, u32 w2) { g_short = shortm; g_lens = lens; g_seg = seg; g_k3 = k3; g_w2 = w2; }
extern "C" u64 xzm_encode(const u8* s, u32 n, u8* outp, int mode, u32 depth, u32 nice, u32 window) {
    init_tabs();
    static Coder frz;
    if (mode == 3) {  // frozen prices: the probabilities a greedy pass ends with
        std::vector<u8> tmp(n + n / 8 + 4096);
        g_dumping = true;
        xzm_encode(s, n, tmp.data(), 2, depth, nice, window);
        g_dumping = false;
        memcpy(frz.probs, g_dump, sizeof(g_dump));
        g_frz = &frz;
    }
    Out O;
    const u8 hdr[12] = {0xFD, 0x37, 0x7A, 0x58, 0x5A, 0x00, 0x00, 0x04, 0xE6, 0xD6, 0xB4, 0x46};
    for (u8 x : hdr) O.b(x);
    u64 unpadded = 0;
    if (n > 0) {
        const u32 dprop = 2u * (23u - 12u);  // preset 6: 8 MiB
        u32 hc = 0xFFFFFFFFu;
        const u8 bh[8] = {0x02, 0x00, 0x21, 0x01, (u8)dprop, 0, 0, 0};
        for (u8 x : bh) { O.b(x); hc = crc32_tab[(hc ^ x) & 0xFF] ^ (hc >> 8); }
        hc = ~hc;
        for (int k = 0; k < 4; k++) O.b((hc >> (8 * k)) & 0xFF);
        const u64 cdata0 = O.v.size();
        Matches M = find_matches(s, n, depth, nice);
        Coder C;
        std::vector<u8> chunk;
        C.out = &chunk;
        u32 state = 0, reps[4] = {0, 0, 0, 0};
        bool need_dict = true, need_props = true, need_state = true;
        u32 p = 0;
        std::vector<Node> opt;
        // path of the current window, in order
        std::vector<Node> path;
        size_t path_i = 0;
        while (p < n) {
            chunk.clear();
            if (need_state) { C.reset_probs(); state = 0; reps[0] = reps[1] = reps[2] = reps[3] = 0; }
            C.reset_rc();
            const u32 u0 = p;
            path.clear();
            path_i = 0;
            // save model state to rewind an incompressible chunk
            const u32 umax = g_seg ? std::min<u32>(UMAX, g_seg - (u0 % g_seg)) : UMAX;
            while (p < n && (p - u0) < umax && chunk.size() + C.cache_size + 5 < CMAX) {
                const u32 ps = p & ((1u << PB) - 1);
                const u32 prevb = p ? s[p - 1] : 0;
                const u32 litbase = E_LITERAL + 0x300u * litctx(p, prevb);
                auto enc_lit = [&](u32 at) {
                    const u32 sym = s[at];
                    const u32 pps = at & ((1u << PB) - 1);
                    const u32 pv = at ? s[at - 1] : 0;
                    const u32 base = E_LITERAL + 0x300u * litctx(at, pv);
                    C.bit(E_IS_MATCH + (state << 4) + pps, 0);
                    if (state < 7) {
                        C.tree(base, 8, sym);
                    } else {
                        u32 mb = at > reps[0] ? s[at - reps[0] - 1] : 0, off = 0x100, m = 1;
                        for (int k = 7; k >= 0; k--) {
                            const u32 b = (sym >> k) & 1;
                            mb <<= 1;
                            const u32 mbit = mb & off;
                            C.bit(base + off + mbit + m, b);
                            m = (m << 1) | b;
                            off &= b ? mbit : ~mbit;
                        }
                    }
                    state = st_lit(state);
                };
                auto rep_len = [&](u32 at, u32 r) -> u32 {
                    if (at <= r) return 0;
                    const u32 mx = std::min<u32>(MATCH_MAX, n - at);
                    u32 l = 0;
                    while (l < mx && s[at + l] == s[at - r - 1 + l]) l++;
                    return l;
                };
                if (mode == 0) {
                    (void)litbase;
                    const u32 mx = std::min<u32>(MATCH_MAX, n - p);
                    u32 rl = (mx >= 2) ? rep_len(p, reps[0]) : 0;
                    u32 hl = 0, hd = 0;
                    if (mx >= 4 && M.off[p + 1] > M.off[p]) {
                        hl = std::min<u32>(M.len[M.off[p + 1] - 1], 64);
                        hd = M.dist[M.off[p + 1] - 1];
                        if (hl > mx) hl = mx;
                        if (p + 1 < n && hl < 64 && rl + 1 < hl && M.off[p + 2] > M.off[p + 1]) {
                            const u32 nl = std::min<u32>(M.len[M.off[p + 2] - 1], 64);
                            if (nl > hl + 1) { hl = 0; rl = 0; }
                        }
                    }
                    if (rl >= 2 && rl + 1 >= hl) {
                        C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                        C.bit(E_IS_REP + state, 1);
                        C.bit(E_IS_REP_G0 + state, 0);
                        C.bit(E_IS_REP0_LONG + (state << 4) + ps, 1);
                        C.length(E_REP_LEN, rl - 2, ps);
                        state = st_rep(state);
                        p += rl;
                    } else if (hl >= 4) {
                        C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                        C.bit(E_IS_REP + state, 0);
                        C.length(E_LEN, hl - 2, ps);
                        C.distance(hd, hl);
                        reps[3] = reps[2]; reps[2] = reps[1]; reps[1] = reps[0]; reps[0] = hd;
                        state = st_match(state);
                        p += hl;
                    } else {
                        enc_lit(p);
                        p += 1;
                    }
                    continue;
                }
                // ---- mode 2: liblzma's fast-mode decisions (reps 0-3, short matches, lazy) ----
                if (mode == 2) {
                    auto chp = [](u32 small, u32 big) { return (big >> 7) > small; };
                    const u32 avail = n - p;
                    Node a{};
                    a.kind = 0;
                    a.len = 1;
                    do {
                        if (avail < 2) break;
                        u32 rlb = 0, ri = 0;
                        bool done = false;
                        for (u32 r = 0; r < 4; r++) {
                            const u32 l = rep_len(p, reps[r]);
                            if (l >= nice) { a.kind = 2 + r; a.len = l; done = true; break; }
                            if (l > rlb) { rlb = l; ri = r; }
                        }
                        if (done) break;
                        u32 ml = 0, md = 0;
                        int k = (int)M.off[p + 1] - 1;
                        if (k >= (int)M.off[p]) { ml = M.len[k]; md = M.dist[k]; }
                        if (ml >= nice) { a.kind = 6; a.len = ml; a.dist = md; break; }
                        while (k > (int)M.off[p] && ml == M.len[k - 1] + 1 && chp(M.dist[k - 1], md)) {
                            k--;
                            ml = M.len[k];
                            md = M.dist[k];
                        }
                        if (ml == 2 && md >= 0x80) ml = 1;
                        if (rlb >= 2 && (rlb + 1 >= ml || (rlb + 2 >= ml && md >= (1u << 9)) ||
                                         (rlb + 3 >= ml && md >= (1u << 15)))) {
                            a.kind = 2 + ri; a.len = rlb; break;
                        }
                        if (ml < 2 || avail <= 2) break;
                        if (p + 1 < n && M.off[p + 2] > M.off[p + 1]) {
                            const u32 nl = M.len[M.off[p + 2] - 1], nd = M.dist[M.off[p + 2] - 1];
                            if (nl >= 2 && ((nl >= ml && nd < md) || (nl == ml + 1 && !chp(md, nd)) || nl > ml + 1 ||
                                            (nl + 1 >= ml && ml >= 3 && chp(nd, md))))
                                break;
                        }
                        const u32 lim = ml - 1 > 2 ? ml - 1 : 2;
                        bool rep_next = false;
                        for (u32 r = 0; r < 4 && !rep_next; r++) rep_next = p + 1 < n && rep_len(p + 1, reps[r]) >= lim;
                        if (rep_next) break;
                        a.kind = 6; a.len = ml; a.dist = md;
                    } while (false);
                    path.assign(1, a);
                    path_i = 0;
                }
                // ---- mode 1: optimal parse of a window starting at p ----
                auto plan = [&](u32 p0, u32 W, u32 st0, const u32* reps0, std::vector<Node>& outp) {
                    const Coder& PC = mode == 3 ? *g_frz : C;
                    opt.assign(W + 1, Node{0xFFFFFFFFu, 0, 0, 0, 0, 0, {0, 0, 0, 0}});
                    opt[0].price = 0;
                    opt[0].state = st0;
                    memcpy(opt[0].reps, reps0, sizeof(reps));
                    u32 lim = W;
                    for (u32 i = 0; i < lim && i < W; i++) {
                        const Node& nd = opt[i];
                        if (nd.price == 0xFFFFFFFFu) continue;
                        const u32 at = p0 + i;
                        const u32 aps = at & ((1u << PB) - 1);
                        const u32 st = nd.state;
                        const u32* rp = nd.reps;
                        auto relax = [&](u32 j, u32 price, u32 kind, u32 len, u32 dist, u32 nst, const u32* nrep) {
                            if (j > W) return;
                            if (price < opt[j].price) {
                                Node& t = opt[j];
                                t.price = price; t.prev = i; t.kind = kind; t.len = len; t.dist = dist; t.state = nst;
                                memcpy(t.reps, nrep, sizeof(t.reps));
                            }
                        };
                        // literal
                        {
                            const u32 sym = s[at];
                            const u32 pv = at ? s[at - 1] : 0;
                            const u32 base = E_LITERAL + 0x300u * litctx(at, pv);
                            u32 pr = nd.price + PC.pb(E_IS_MATCH + (st << 4) + aps, 0);
                            if (st < 7) {
                                pr += PC.ptree(base, 8, sym);
                            } else {
                                u32 mb = at > rp[0] ? s[at - rp[0] - 1] : 0, off = 0x100, m = 1;
                                for (int k = 7; k >= 0; k--) {
                                    const u32 b = (sym >> k) & 1;
                                    mb <<= 1;
                                    const u32 mbit = mb & off;
                                    pr += PC.pb(base + off + mbit + m, b);
                                    m = (m << 1) | b;
                                    off &= b ? mbit : ~mbit;
                                }
                            }
                            relax(i + 1, pr, 0, 1, 0, st_lit(st), rp);
                        }
                        const u32 mbase = nd.price + PC.pb(E_IS_MATCH + (st << 4) + aps, 1);
                        const u32 rbase = mbase + PC.pb(E_IS_REP + st, 1);
                        // short rep
                        if (at > rp[0] && s[at] == s[at - rp[0] - 1]) {
                            const u32 pr = rbase + PC.pb(E_IS_REP_G0 + st, 0) + PC.pb(E_IS_REP0_LONG + (st << 4) + aps, 0);
                            relax(i + 1, pr, 1, 1, rp[0], st_short(st), rp);
                        }
                        // rep matches
                        for (u32 r = 0; r < 4; r++) {
                            const u32 rl = rep_len(at, rp[r]);
                            if (rl < 2) continue;
                            u32 pr = rbase;
                            if (r == 0) pr += PC.pb(E_IS_REP_G0 + st, 0) + PC.pb(E_IS_REP0_LONG + (st << 4) + aps, 1);
                            else {
                                pr += PC.pb(E_IS_REP_G0 + st, 1);
                                if (r == 1) pr += PC.pb(E_IS_REP_G1 + st, 0);
                                else pr += PC.pb(E_IS_REP_G1 + st, 1) + PC.pb(E_IS_REP_G2 + st, r - 2);
                            }
                            u32 nrep[4];
                            nrep[0] = rp[r];
                            for (u32 k = 0, t = 1; k < 4; k++) if (k != r) nrep[t++] = rp[k];
                            for (u32 l = 2; l <= rl; l++) relax(i + l, pr + PC.plen(E_REP_LEN, l - 2, aps), 2 + r, l, rp[r], st_rep(st), nrep);
                            if (i + rl > lim && rl >= 32) lim = std::min<u32>(W, i + rl);
                        }
                        // normal matches
                        const u32 mb0 = mbase + PC.pb(E_IS_REP + st, 0);
                        u32 lprev = 1;
                        for (u32 k = M.off[at]; k < M.off[at + 1]; k++) {
                            const u32 L = std::min<u32>(M.len[k], n - at), d = M.dist[k];
                            u32 nrep[4] = {d, rp[0], rp[1], rp[2]};
                            for (u32 l = std::max<u32>(lprev + 1, 2); l <= L; l++) {
                                if (g_lens && l < L && l > g_lens && L - l > 2) continue;
                                relax(i + l, mb0 + PC.plen(E_LEN, l - 2, aps) + PC.pdist(d, l), 6, l, d, st_match(st), nrep);
                            }
                            lprev = L;
                        }
                    }
                    // backtrack the best path to W (or the last reached node)
                    u32 end = W;
                    while (end > 0 && opt[end].price == 0xFFFFFFFFu) end--;
                    std::vector<Node> rev;
                    for (u32 j = end; j > 0; j = opt[j].prev) rev.push_back(opt[j]);
                    outp.assign(rev.rbegin(), rev.rend());
                };
                if ((mode == 1 || mode == 3) && path_i >= path.size()) {
                    plan(p, std::min<u32>(window, n - p), state, reps, path);
                    path_i = 0;
                }
                if (mode == 5 && path_i >= path.size()) {
                    // G windows planned independently from the same start state / prices
                    path.clear();
                    const u32 se = g_seg ? std::min<u32>(n, (p / g_seg + 1) * g_seg) : n;
                    for (u32 k = 0; k < g_group; k++) {
                        const u32 p0 = p + k * window;
                        if (p0 >= se) break;
                        std::vector<Node> tmp;
                        plan(p0, std::min<u32>(window, se - p0), state, reps, tmp);
                        path.insert(path.end(), tmp.begin(), tmp.end());
                    }
                    path_i = 0;
                }
                Node a = path[path_i++];
                if (mode == 5) {  // the plan's distances against the actual reps
                    if (a.kind == 1 && !(p > reps[0] && reps[0] == a.dist)) a.kind = 0;
                    else if (a.kind >= 2 && a.kind < 6) {
                        u32 r = 4;
                        for (u32 k = 0; k < 4 && r == 4; k++) if (reps[k] == a.dist) r = k;
                        a.kind = r < 4 ? 2 + r : 6;
                    }
                }
                if (a.kind == 0) {
                    enc_lit(p);
                    p += 1;
                } else if (a.kind == 1) {
                    C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                    C.bit(E_IS_REP + state, 1);
                    C.bit(E_IS_REP_G0 + state, 0);
                    C.bit(E_IS_REP0_LONG + (state << 4) + ps, 0);
                    state = st_short(state);
                    p += 1;
                } else if (a.kind < 6) {
                    const u32 r = a.kind - 2;
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
                    C.length(E_REP_LEN, a.len - 2, ps);
                    state = st_rep(state);
                    p += a.len;
                } else {
                    C.bit(E_IS_MATCH + (state << 4) + ps, 1);
                    C.bit(E_IS_REP + state, 0);
                    C.length(E_LEN, a.len - 2, ps);
                    C.distance(a.dist, a.len);
                    reps[3] = reps[2]; reps[2] = reps[1]; reps[1] = reps[0]; reps[0] = a.dist;
                    state = st_match(state);
                    p += a.len;
                }
            }
            path.clear();  // a chunk boundary ends the window (the model may reset)
            path_i = 0;
            for (int k = 0; k < 5; k++) C.shift_low();
            const u32 usz = p - u0 - 1;
            if (chunk.size() >= p - u0) {  // uncompressed chunk
                O.b(need_dict ? 0x01u : 0x02u);
                O.b((usz >> 8) & 0xFF);
                O.b(usz & 0xFF);
                for (u32 k = u0; k < p; k++) O.b(s[k]);
                need_dict = false;
                need_state = true;
                continue;
            }
            const u32 csz = (u32)chunk.size() - 1;
            const u32 ctl = need_props ? (need_dict ? 0xE0u : 0xC0u) : (need_state ? 0xA0u : 0x80u);
            O.b(ctl | (usz >> 16));
            O.b((usz >> 8) & 0xFF);
            O.b(usz & 0xFF);
            O.b((csz >> 8) & 0xFF);
            O.b(csz & 0xFF);
            if (need_props) O.b((PB * 5 + LP) * 9 + LC);
            O.v.insert(O.v.end(), chunk.begin(), chunk.end());
            need_dict = need_props = need_state = false;
            if (g_seg && p % g_seg == 0) need_state = true;  // independent segments: a state reset
        }
        if (g_dumping) memcpy(g_dump, C.probs, sizeof(g_dump));
        O.b(0x00);
        const u64 csize = O.v.size() - cdata0;
        while ((O.v.size() - cdata0) & 3) O.b(0);
        u64 crc = ~0ull;
        for (u32 k = 0; k < n; k++) crc = crc64_tab[(crc ^ s[k]) & 0xFF] ^ (crc >> 8);
        crc = ~crc;
        for (int k = 0; k < 8; k++) O.b((u32)(crc >> (8 * k)) & 0xFF);
        unpadded = 12 + csize + 8;
    }
    const u64 idx0 = O.v.size();
    u32 ic = 0xFFFFFFFFu;
    auto iout = [&](u32 b) { O.b(b); ic = crc32_tab[(ic ^ b) & 0xFF] ^ (ic >> 8); };
    auto ivli = [&](u64 v) { while (v >= 0x80) { iout((u32)(v & 0x7F) | 0x80); v >>= 7; } iout((u32)v); };
    iout(0x00);
    ivli(n > 0 ? 1 : 0);
    if (n > 0) { ivli(unpadded); ivli(n); }
    while ((O.v.size() - idx0) & 3) iout(0x00);
    ic = ~ic;
    for (int k = 0; k < 4; k++) O.b((ic >> (8 * k)) & 0xFF);
    const u64 isize = O.v.size() - idx0;
    const u32 bsz = (u32)(isize / 4 - 1);
    const u64 fbw = (u64)bsz | (0x0400ull << 32);
    u32 fc = 0xFFFFFFFFu;
    for (int k = 0; k < 6; k++) fc = crc32_tab[(fc ^ (u32)(fbw >> (8 * k))) & 0xFF] ^ (fc >> 8);
    fc = ~fc;
    for (int k = 0; k < 4; k++) O.b((fc >> (8 * k)) & 0xFF);
    for (int k = 0; k < 6; k++) O.b((u32)(fbw >> (8 * k)) & 0xFF);
    O.b(0x59);
    O.b(0x5A);
    memcpy(outp, O.v.data(), O.v.size());
    return O.v.size();
}
