// zlib_ref.cpp — TEST INFRASTRUCTURE ONLY.
//
// A serial CPU driver of zarr_amd/csrc/zcg_zlib_core.h (the zlib 1.2.11
// deflate_slow restatement the GPU gzip encoder runs): hash chains by a
// head table, zz::search at every position, zz::parse, and per block
// zz::plan_block + the bits.  tests/test_hostcore.py compares its raw-deflate
// output with the system zlib (levels 4-9) byte for byte; the GPU kernels are
// compared with this and with zlib.  Never linked into the product.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../zarr_amd/csrc/zcg_zlib_core.h"

namespace {
struct BitOut {
    uint8_t* out;
    uint64_t cap, n = 0;
    uint64_t acc = 0;
    uint32_t nb = 0;
    bool over = false;
    void byte(uint32_t b) {
        if (n < cap) out[n] = (uint8_t)b; else over = true;
        n++;
    }
    void put(uint32_t v, uint32_t bits) {
        if (!bits) return;
        acc |= (uint64_t)(v & ((bits == 32) ? 0xFFFFFFFFu : ((1u << bits) - 1))) << nb;
        nb += bits;
        while (nb >= 8) { byte((uint32_t)acc & 0xFF); acc >>= 8; nb -= 8; }
    }
    void windup() {
        if (nb) { byte((uint32_t)acc & 0xFF); acc = 0; nb = 0; }
    }
};
}  // namespace

// zlib's head[] / prev[] (window-relative Pos, 0 = NIL) for zz::parse_fast
struct FastTab {
    std::vector<uint16_t> hd, pv;
    FastTab() : hd(1u << 15, 0), pv(zz::WSIZE, 0) {}
    uint32_t head(uint32_t h) const { return hd[h]; }
    void set_head(uint32_t h, uint32_t v) { hd[h] = (uint16_t)v; }
    uint32_t prev(uint32_t i) const { return pv[i]; }
    void set_prev(uint32_t i, uint32_t v) { pv[i] = (uint16_t)v; }
    void slide() {  // slide_hash
        for (auto& x : hd) x = x >= zz::WSIZE ? (uint16_t)(x - zz::WSIZE) : 0;
        for (auto& x : pv) x = x >= zz::WSIZE ? (uint16_t)(x - zz::WSIZE) : 0;
    }
};

static int64_t emit_blocks(const uint8_t* src, const std::vector<uint32_t>& syms,
                           const std::vector<zz::BlockRec>& blocks, uint8_t* out, uint64_t cap);

extern "C" int64_t zz_host_deflate(const uint8_t* src, uint32_t D, int level, uint8_t* out, uint64_t cap) {
    using namespace zz;
    const Config cfg = level_config(level);
    if (level >= 1 && level <= 3) {  // deflate_fast: the parse builds its chains
        auto byte = [&](uint32_t i) -> uint32_t { return src[i]; };
        auto byte4 = [&](uint32_t i) -> uint32_t {
            uint32_t v;
            memcpy(&v, src + i, 4);
            return v;
        };
        FastTab tab;
        std::vector<uint32_t> syms, pos;
        auto emit = [&](uint32_t s, uint32_t at) { syms.push_back(s); pos.push_back(at); };
        const uint32_t nsym = parse_fast(D, cfg, tab, byte4, byte, emit);
        std::vector<BlockRec> blocks;
        auto P = [&](uint32_t i) -> uint32_t { return pos[i]; };
        auto Y = [&](uint32_t i) -> uint32_t { return syms[i]; };
        for (uint32_t k = 0; k < num_blocks(nsym); k++) blocks.push_back(block_rec(k, nsym, nsym, D, P, Y, true));
        return emit_blocks(src, syms, blocks, out, cap);
    }
    std::vector<uint32_t> prev(D ? D : 1, NONE), head(1u << 15, NONE);
    for (uint32_t p = 0; p + MIN_MATCH <= D; p++) {
        const uint32_t h = hash3(src[p], src[p + 1], src[p + 2]);
        prev[p] = head[h];
        head[h] = p;
    }
    auto byte = [&](uint32_t i) -> uint32_t { return src[i]; };
    auto byte4 = [&](uint32_t i) -> uint32_t {
        uint32_t v;
        memcpy(&v, src + i, 4);
        return v;
    };
    auto pr = [&](uint32_t i) -> uint32_t { return prev[i]; };
    std::vector<Match2> g(D ? D : 1);
    for (uint32_t p = 0; p < D; p++) g[p] = search(p, D, cfg, byte4, byte, pr);
    std::vector<uint32_t> syms;
    std::vector<BlockRec> blocks;
    auto get = [&](uint32_t p) -> Match2 { return g[p]; };
    auto emit = [&](uint32_t, uint32_t s) { syms.push_back(s); };
    auto flush = [&](const BlockRec& b) { blocks.push_back(b); };
    parse(D, cfg, get, byte, emit, flush);
    return emit_blocks(src, syms, blocks, out, cap);
}

static int64_t emit_blocks(const uint8_t* src, const std::vector<uint32_t>& syms,
                           const std::vector<zz::BlockRec>& blocks, uint8_t* out, uint64_t cap) {
    using namespace zz;
    BitOut bo{out, cap};
    BlockWork* bw = new BlockWork;
    for (const BlockRec& b : blocks) {
        for (int i = 0; i < HEAP_SIZE; i++) bw->lt.freq[i] = 0;
        for (int i = 0; i < 2 * D_CODES + 1; i++) bw->dt.freq[i] = 0;
        for (uint32_t k = b.s0; k < b.s1; k++) {
            const uint32_t s = syms[k];
            if (!(s & 0x80000000u)) {
                bw->lt.freq[s & 0xFF]++;
            } else {
                bw->lt.freq[len_code(((s >> 16) & 0xFF) + 3) + LITERALS + 1]++;
                bw->dt.freq[dist_code((s & 0xFFFF) + 1)]++;
            }
        }
        bw->lt.freq[END_BLOCK] = 1;
        const BlockPlan pl = plan_block(*bw, b.b1 - b.b0, b.in_win != 0);
        auto put = [&](uint32_t v, uint32_t n) { bo.put(v, n); };
        send_header(*bw, pl, b.last != 0, put);
        if (pl.type == BT_STORED) {
            bo.windup();
            const uint32_t len = b.b1 - b.b0;
            bo.put(len & 0xFFFF, 16);
            bo.put(~len & 0xFFFF, 16);
            for (uint32_t i = b.b0; i < b.b1; i++) bo.put(src[i], 8);
        } else {
            const bool st = pl.type == BT_STATIC;
            for (uint32_t k = b.s0; k < b.s1; k++) {
                const SymBits sb = sym_bits(syms[k], st, bw->lt.code, bw->lt.len, bw->dt.code, bw->dt.len);
                for (int j = 0; j < 4; j++) bo.put(sb.v[j], sb.n[j]);
            }
            bo.put(st ? static_lcode(END_BLOCK) : bw->lt.code[END_BLOCK], st ? 7u : bw->lt.len[END_BLOCK]);
        }
        if (b.last) bo.windup();
    }
    delete bw;
    return bo.over ? -1 : (int64_t)bo.n;
}

// The GPU's segment-parallel parse, emulated serially: every segment of `seg`
// positions parsed speculatively from a canonical start (pass 1, canonical
// loop tops marked in a bitmap), each segment's parse continued past its end
// until it reaches a canonical loop top the next segments' parses marked
// (pass 2), the true path stitched through the sync points, blocks cut by
// zz::block_rec.  Must equal zlib byte for byte for any `seg`.
extern "C" int64_t zz_host_deflate_seg(const uint8_t* src, uint32_t D, int level, uint32_t seg, uint8_t* out,
                                       uint64_t cap) {
    using namespace zz;
    const Config cfg = level_config(level);
    std::vector<uint32_t> prev(D ? D : 1, NONE), head(1u << 15, NONE);
    for (uint32_t p = 0; p + MIN_MATCH <= D; p++) {
        const uint32_t h = hash3(src[p], src[p + 1], src[p + 2]);
        prev[p] = head[h];
        head[h] = p;
    }
    auto byte = [&](uint32_t i) -> uint32_t { return src[i]; };
    auto byte4 = [&](uint32_t i) -> uint32_t {
        uint32_t v;
        memcpy(&v, src + i, 4);
        return v;
    };
    auto pr = [&](uint32_t i) -> uint32_t { return prev[i]; };
    std::vector<Match2> g(D ? D : 1);
    for (uint32_t p = 0; p < D; p++) g[p] = search(p, D, cfg, byte4, byte, pr);
    auto get = [&](uint32_t p) -> Match2 { return g[p]; };
    const uint32_t nseg = D ? (D + seg - 1) / seg : 1;
    std::vector<std::vector<uint32_t>> sy(nseg), ps(nseg), ty(nseg), tp(nseg);
    std::vector<PState> end(nseg);
    std::vector<uint8_t> canon(D + 1, 0);
    std::vector<uint32_t> sync_q(nseg, NONE);
    std::vector<uint8_t> fin_lit(nseg, 0), tail_fin(nseg, 0);
    for (uint32_t k = 0; k < nseg; k++) {  // pass 1
        const uint32_t S0 = k * seg, S1 = (k + 1 == nseg) ? D : (k + 1) * seg;
        PState st = fresh_state(S0);
        auto em = [&](uint32_t s, uint32_t at) { sy[k].push_back(s); ps[k].push_back(at); };
        while (st.p < S1 && st.p < D) {
            if (canonical(st)) canon[st.p] = 1;
            step(st, D, cfg, get, byte, em);
        }
        if (k + 1 == nseg && st.avail) {  // Z_FINISH: the pending literal
            em(byte(st.p - 1), st.p - 1);
            st.avail = 0;
            fin_lit[k] = 1;
        }
        end[k] = st;
    }
    for (uint32_t k = 0; k + 1 < nseg; k++) {  // pass 2
        const uint32_t S1 = (k + 1) * seg;
        PState st = end[k];
        auto em = [&](uint32_t s, uint32_t at) { ty[k].push_back(s); tp[k].push_back(at); };
        while (true) {
            if (st.p >= D) {
                if (st.avail) {
                    em(byte(st.p - 1), st.p - 1);
                    tail_fin[k] = 1;
                }
                break;
            }
            if (st.p >= S1 && canonical(st) && canon[st.p]) {
                sync_q[k] = st.p;
                break;
            }
            step(st, D, cfg, get, byte, em);
        }
    }
    std::vector<uint32_t> syms, pos;
    bool finlit = false;
    uint32_t cur = 0, idx = 0;
    while (true) {
        for (uint32_t i = idx; i < sy[cur].size(); i++) { syms.push_back(sy[cur][i]); pos.push_back(ps[cur][i]); }
        if (cur + 1 == nseg) { finlit = fin_lit[cur]; break; }
        for (uint32_t i = 0; i < ty[cur].size(); i++) { syms.push_back(ty[cur][i]); pos.push_back(tp[cur][i]); }
        if (sync_q[cur] == NONE) { finlit = tail_fin[cur]; break; }
        const uint32_t q = sync_q[cur];
        const uint32_t nx = q / seg;
        uint32_t j = 0;
        while (j < ps[nx].size() && ps[nx][j] < q) j++;
        cur = nx;
        idx = j;
    }
    const uint32_t nsym = (uint32_t)syms.size(), nloop = nsym - (finlit ? 1u : 0u);
    auto P = [&](uint32_t i) { return pos[i]; };
    auto Y = [&](uint32_t i) { return syms[i]; };
    BitOut bo{out, cap};
    BlockWork* bw = new BlockWork;
    const uint32_t nb = num_blocks(nloop);
    for (uint32_t k = 0; k < nb; k++) {
        const BlockRec b = block_rec(k, nsym, nloop, D, P, Y);
        for (int i = 0; i < HEAP_SIZE; i++) bw->lt.freq[i] = 0;
        for (int i = 0; i < 2 * D_CODES + 1; i++) bw->dt.freq[i] = 0;
        for (uint32_t q = b.s0; q < b.s1; q++) {
            const uint32_t s = syms[q];
            if (!(s & 0x80000000u)) bw->lt.freq[s & 0xFF]++;
            else {
                bw->lt.freq[len_code(((s >> 16) & 0xFF) + 3) + LITERALS + 1]++;
                bw->dt.freq[dist_code((s & 0xFFFF) + 1)]++;
            }
        }
        bw->lt.freq[END_BLOCK] = 1;
        const BlockPlan pl = plan_block(*bw, b.b1 - b.b0, b.in_win != 0);
        auto put = [&](uint32_t v, uint32_t n) { bo.put(v, n); };
        send_header(*bw, pl, b.last != 0, put);
        if (pl.type == BT_STORED) {
            bo.windup();
            const uint32_t len = b.b1 - b.b0;
            bo.put(len & 0xFFFF, 16);
            bo.put(~len & 0xFFFF, 16);
            for (uint32_t i = b.b0; i < b.b1; i++) bo.put(src[i], 8);
        } else {
            const bool st = pl.type == BT_STATIC;
            for (uint32_t q = b.s0; q < b.s1; q++) {
                const SymBits sb = sym_bits(syms[q], st, bw->lt.code, bw->lt.len, bw->dt.code, bw->dt.len);
                for (int j = 0; j < 4; j++) bo.put(sb.v[j], sb.n[j]);
            }
            bo.put(st ? static_lcode(END_BLOCK) : bw->lt.code[END_BLOCK], st ? 7u : bw->lt.len[END_BLOCK]);
        }
        if (b.last) bo.windup();
    }
    delete bw;
    return bo.over ? -1 : (int64_t)bo.n;
}
