// host_cores.cpp — TEST INFRASTRUCTURE ONLY.
//
// Host instantiations of the device decode cores (zarr_amd/csrc/*_core.h),
// so the CPU test suite can fuzz the exact decoder logic the gfx950 kernels
// run against the oracle (oracle/libzref.so = the reference's C codec
// libraries) on thousands of corrupted streams.  Never used by the product
// path: zarr_amd loads only libzchunk_gpu.so.
#include <stdint.h>
#include <string.h>

#include "../../zarr_amd/csrc/zcg_xz_core.h"

namespace {

uint64_t crc64_byte(uint64_t c, uint32_t b) {
    c ^= b;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xC96C5795D7870F42ull & (0ull - (c & 1)));
    return c;
}

struct XzHostIO {
    uint64_t n, D, pos;
    const uint8_t* src;
    uint8_t* dst;
    uint16_t probs[1846 + (0x300 << 4)];
    uint8_t tail[64];  // output bytes from D on (a BCJ block's look-past, zx::xz_decode)
    uint8_t& at(uint64_t i) { return i < D ? dst[i] : tail[i - D]; }
    void make_uniform() {}
    uint32_t in(uint64_t i) const { return src[i]; }
    uint32_t pget(uint32_t i) const { return probs[i]; }
    void pset(uint32_t i, uint32_t v) { probs[i] = (uint16_t)v; }
    void init_probs(uint32_t count) { for (uint32_t i = 0; i < count; i++) probs[i] = 1024; }
    bool lclp_ok(uint32_t) const { return true; }
    void put(uint32_t b) { at(pos++) = (uint8_t)b; }
    uint32_t back(uint64_t dist) { return at(pos - 1 - dist); }
    void copy(uint64_t d, uint32_t len) {
        for (uint32_t k = 0; k < len; k++) at(pos + k) = at(pos + k - d);
        pos += len;
    }
    void copy_in(uint64_t ip, uint32_t len) {
        for (uint32_t k = 0; k < len; k++) at(pos + k) = src[ip + k];
        pos += len;
    }
    void finish() {}
    void reset() { pos = 0; }
    uint32_t tail_byte(uint64_t i) { return at(i); }
    void set_byte(uint64_t i, uint32_t v) { dst[i] = (uint8_t)v; }
    void apply_delta(uint64_t a, uint64_t b, uint32_t dist) {
        for (uint64_t i = a; i < b; i++)
            if (i >= a + dist) dst[i] = (uint8_t)(dst[i] + dst[i - dist]);
    }
    struct Buf {
        uint8_t* p;
        uint32_t get(uint64_t i) const { return p[i]; }
        void set(uint64_t i, uint32_t v) { p[i] = (uint8_t)v; }
    };
    uint32_t out_byte(uint64_t i) const { return dst[i]; }
    zx::BcjState apply_bcj(uint64_t a, uint64_t b, uint32_t id, uint32_t start) {
        Buf buf{dst + a};
        return zx::bcj_serial(buf, b - a, id, start);
    }
    void sha256(uint64_t a, uint64_t b, uint32_t* h) const {
        zx::sha256_init(h);
        uint64_t q = a;
        for (; q + 64 <= b; q += 64) {
            uint32_t m[16];
            for (int i = 0; i < 16; i++)
                m[i] = ((uint32_t)dst[q + 4 * i] << 24) | ((uint32_t)dst[q + 4 * i + 1] << 16) |
                       ((uint32_t)dst[q + 4 * i + 2] << 8) | dst[q + 4 * i + 3];
            zx::sha256_compress(h, m);
        }
        zx::sha256_tail(h, dst + q, (uint32_t)(b - q), b - a);
    }
    uint64_t check(uint32_t id, uint64_t a, uint64_t b) const {
        if (id == 4) {
            uint64_t c = ~0ull;
            for (uint64_t q = a; q < b; q++) c = crc64_byte(c, dst[q]);
            return ~c;
        }
        uint32_t c = 0xFFFFFFFFu;
        for (uint64_t q = a; q < b; q++) c = zx::crc32_byte(c, dst[q]);
        return ~c;
    }
};

}  // namespace

extern "C" int zh_xz_decode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t D) {
    static thread_local XzHostIO io;
    io.n = n;
    io.D = D;
    io.pos = 0;
    io.src = src;
    io.dst = dst;
    return zx::xz_decode(io);
}

// ---------------------------------------------------------------------------
// Bzip2: serial core (zcg_bz2_core.h) + a serial restatement of libbz2's
// output stage (T^-1 vector, tPos walk, unRLE_obuf_to_output_FAST, block CRC)
// standing in for the device's parallel stages.
#include <vector>

#include "../../zarr_amd/csrc/zcg_bz2_core.h"

namespace {

struct BzHostIO {
    const uint8_t* src;
    uint64_t n, D, pos;
    uint8_t* dst;
    zb::Group g[6];
    uint16_t lutt[6][1 << zb::LUT_BITS];
    uint8_t lenb[6][258];
    uint8_t selb[zb::MAX_SELECTORS];
    uint8_t mtf[256];
    uint8_t seqb[256];
    std::vector<uint8_t> L;
    std::vector<uint32_t> tt;
    // libbz2 output-stage state (carried between blocks only via CRCs)
    uint32_t peek(uint64_t bp, uint32_t nb) const {
        uint64_t byte = bp >> 3, w = 0;
        for (int k = 0; k < 5; k++) w = (w << 8) | (byte + k < n ? src[byte + k] : 0u);
        const uint32_t sh = 40 - (uint32_t)(bp & 7) - nb;
        return (uint32_t)((w >> sh) & ((1ull << nb) - 1));
    }
    zb::Group* group(uint32_t t) { return &g[t]; }
    uint8_t* lens(uint32_t t) { return lenb[t]; }
    uint8_t* seqbuf() { return seqb; }
    void build_lut(uint32_t t, const zb::Group* gg, uint32_t) {
        for (uint32_t x = 0; x < (1u << zb::LUT_BITS); x++) lutt[t][x] = (uint16_t)zb::lut_entry(gg, x);
    }
    uint32_t lut_get(uint32_t t, uint32_t x) const { return lutt[t][x]; }
    void sel_put(uint32_t i, uint32_t v) { selb[i] = (uint8_t)v; }
    uint32_t sel_get(uint32_t i) const { return selb[i]; }
    void mtf_reset(const uint8_t* seq, uint32_t k) { for (uint32_t i = 0; i < k; i++) mtf[i] = seq[i]; }
    uint32_t mtf_front() const { return mtf[0]; }
    uint32_t mtf_take(uint32_t nn) {
        const uint8_t v = mtf[nn];
        memmove(mtf + 1, mtf, nn);
        mtf[0] = v;
        return v;
    }
    void l_put(uint32_t i, uint32_t b) { L[i] = (uint8_t)b; }
    void l_run(uint32_t i, uint32_t b, uint32_t cnt) { memset(&L[i], (int)b, cnt); }
    void l_flush(uint32_t) {}
    uint64_t out_pos() const { return pos; }

    int block_output(zb::BzState& s) {
        const uint32_t nblock = s.nblock;
        uint32_t cftab[257];
        uint32_t unz[256] = {0};
        for (uint32_t i = 0; i < nblock; i++) unz[L[i]]++;
        cftab[0] = 0;
        for (int i = 1; i <= 256; i++) cftab[i] = cftab[i - 1] + unz[i - 1];
        for (uint32_t i = 0; i < nblock; i++) tt[i] = L[i];
        for (uint32_t i = 0; i < nblock; i++) tt[cftab[L[i]]++] |= (i << 8);
        const uint32_t bound = 100000u * s.level;
        uint32_t tpos = tt[s.orig_ptr] >> 8;
        uint32_t used = 0, crc = 0xFFFFFFFFu;
        int32_t out_len = 0;
        uint32_t out_ch = 0, k0, k1;
        const uint32_t savePP = nblock + 1;
        int32_t rntogo = 0, rtpos = 0;  // BZ_RAND_INIT_MASK
#define GETF(c) do { if (tpos >= bound) return zb::ST_INVALID; tpos = tt[tpos]; c = tpos & 0xff; tpos >>= 8; } while (0)
#define RUPD(c) do { if (s.randomised) { if (rntogo == 0) { rntogo = zb::kRNums[rtpos]; if (++rtpos == 512) rtpos = 0; } \
                     rntogo--; c ^= (rntogo == 1) ? 1u : 0u; } } while (0)
#define EMIT(c) do { dst[pos++] = (uint8_t)(c); crc = zb::crc_byte(crc, (c)); } while (0)
        GETF(k0);
        RUPD(k0);
        used++;
        if (s.randomised) {
            // unRLE_obuf_to_output_FAST, randomised branch
            for (;;) {
                for (;;) {
                    if (pos == D) return zb::OUT_FULL;
                    if (out_len == 0) break;
                    EMIT(out_ch);
                    out_len--;
                }
                if (used == savePP) break;
                if (used > savePP) return zb::ST_INVALID;
                out_len = 1;
                out_ch = k0;
                GETF(k1); RUPD(k1); used++;
                if (used == savePP) continue;
                if (k1 != k0) { k0 = k1; continue; }
                out_len = 2;
                GETF(k1); RUPD(k1); used++;
                if (used == savePP) continue;
                if (k1 != k0) { k0 = k1; continue; }
                out_len = 3;
                GETF(k1); RUPD(k1); used++;
                if (used == savePP) continue;
                if (k1 != k0) { k0 = k1; continue; }
                GETF(k1); RUPD(k1); used++;
                out_len = (int32_t)k1 + 4;
                GETF(k0); RUPD(k0); used++;
            }
        } else {
            for (;;) {
                if (out_len > 0) {
                    for (;;) {
                        if (pos == D) return zb::OUT_FULL;
                        if (out_len == 1) break;
                        EMIT(out_ch);
                        out_len--;
                    }
                eq_one:
                    if (pos == D) return zb::OUT_FULL;
                    EMIT(out_ch);
                }
                if (used > savePP) return zb::ST_INVALID;
                if (used == savePP) break;
                out_ch = k0;
                GETF(k1); used++;
                if (k1 != k0) { k0 = k1; goto eq_one; }
                if (used == savePP) goto eq_one;
                out_len = 2;
                GETF(k1); used++;
                if (used == savePP) continue;
                if (k1 != k0) { k0 = k1; continue; }
                out_len = 3;
                GETF(k1); used++;
                if (used == savePP) continue;
                if (k1 != k0) { k0 = k1; continue; }
                GETF(k1); used++;
                out_len = (int32_t)k1 + 4;
                GETF(k0); used++;
            }
        }
#undef GETF
#undef RUPD
#undef EMIT
        crc = ~crc;
        if (crc != s.stored_crc) return zb::ST_INVALID;
        s.combined = ((s.combined << 1) | (s.combined >> 31)) ^ crc;
        return zb::OUT_DONE;
    }
};

}  // namespace

extern "C" int zh_bz2_decode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t D) {
    static thread_local BzHostIO* io = nullptr;
    if (!io) {
        io = new BzHostIO();
        io->L.resize(900000);
        io->tt.resize(900000);
    }
    io->src = src;
    io->n = n;
    io->D = D;
    io->pos = 0;
    io->dst = dst;
    zb::BzState s;
    memset(&s, 0, sizeof s);
    s.n = n;
    s.lim = n;
    return zb::bz_stream(*io, s, D);
}
