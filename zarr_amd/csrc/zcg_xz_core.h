// zcg_xz_core.h — XzCompression decode core (src/compression/xz.rs:34-43:
// xz2 read::XzDecoder = liblzma 5.2 lzma_stream_decoder, memlimit u64::MAX,
// no flags), written once and instantiated twice:
//   * on gfx950 by zcg_xz.hip (IO = LDS probability model + LDS history ring
//     + wave-parallel match copies into the chunk's HBM output);
//   * on the host by tests/hostcore (IO = plain arrays), where the same code
//     is fuzzed against liblzma (the oracle) on corrupted streams.
// The product path only ever runs the device instantiation.
//
// What is restated (the .xz container of xz-file-format-1.0.4 and LZMA2 as
// liblzma 5.2 decodes them), including the acceptance rules that decide
// INVALID_DATA vs UNEXPECTED_EOF:
//   stream header (magic, flags CRC32, reserved bits) -> blocks (header CRC32,
//   reserved flag bits, compressed/uncompressed size VLIs, filter flags,
//   header padding; LZMA2 chunks with their dictionary/state/property reset
//   rules; lc+lp<=4; distances checked against the decoded dictionary; the
//   final range-coder normalisation and code==0 at every chunk end; exact
//   compressed chunk sizes; block padding; CRC32/CRC64 check) -> index
//   (record count, unpadded/uncompressed sizes against the decoded blocks,
//   padding, CRC32) -> stream footer (magic, CRC32, backward size, flags).
//
// read_exact semantics (chunk.rs:112-113): decoding stops once D = N*size
// bytes exist.  liblzma keeps going inside the lzma_code() call that filled
// the output, over the input window the BufReader handed it (32 KiB windows,
// see oracle/zref.c zr_decode_xz): after the output is full, this core keeps
// validating headers/sizes/checks up to that window's end and stops there
// with OK.  Truncation before D bytes is UNEXPECTED_EOF.
//
// Filters: LZMA2 with up to three delta / BCJ x86 / PowerPC / IA-64 / ARM /
// ARM-Thumb / SPARC filters before it.  An LZMA1 block is InvalidData, as in
// liblzma 5.2 (its .xz decoder rejects LZMA1 blocks with LZMA_DATA_ERROR).
// Checks: CRC32, CRC64 and SHA-256 are verified; the IDs liblzma does not
// know are skipped, as it does.  xz2's XzEncoder writes a single LZMA2 filter
// with CRC64.  A read that stops inside a BCJ block follows liblzma's simple
// coder, which decodes past the caller's end to release the bytes its filter
// loop held back (xz_decode below); only chains it does not model (two BCJ
// stages, or a delta under the BCJ) keep UNSUPPORTED for a stop whose last
// bytes could start a cut-off instruction.
#pragma once

#include <stdint.h>

#if defined(__HIP__)
#define ZX_INL __host__ __device__ __forceinline__
#else
#define ZX_INL inline __attribute__((always_inline))
#endif
#if defined(__HIP__)
#define ZX_HOT __host__ __device__ __attribute__((noinline))
#else
#define ZX_HOT inline
#endif

namespace zx {

// Wave-uniform hint: the device decoder's state is identical in every lane;
// readfirstlane tells the compiler so (SGPRs, scalar branches).
#if defined(__HIP_DEVICE_COMPILE__)
#define ZX_U32(x) ((x) = __builtin_amdgcn_readfirstlane(x))
#define ZX_UB(c) (__builtin_amdgcn_readfirstlane((uint32_t)(c)) != 0)
#define ZX_UPH(x) __builtin_amdgcn_readfirstlane(x)
#define ZX_U64(x) ((x) = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((x) >> 32)) << 32) | \
                          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x)))
#else
#define ZX_U32(x) ((void)0)
#define ZX_UB(c) (c)
#define ZX_UPH(x) (x)
#define ZX_U64(x) ((void)0)
#endif

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

// status codes (values of enum zcg_status; NEED_BIG = internal retry code)
enum : int { ST_OK = 0, ST_EOF = 1, ST_INVALID = 2, ST_UNSUPPORTED = 4, ST_NEED_BIG = 101 };

constexpr u64 BUFREADER = 32768;  // xz2 bufread window (oracle zr_decode_xz)
constexpr u64 VLI_MAX = 0x7FFFFFFFFFFFFFFFull;
constexpr u64 VLI_UNKNOWN = ~0ull;
constexpr u64 UNPADDED_MIN = 5;
constexpr u64 UNPADDED_MAX = VLI_MAX & ~3ull;

// LZMA probability model layout (u16 entries)
enum : u32 {
    P_IS_MATCH = 0,      // [12][16]
    P_IS_REP = 192,      // [12]
    P_IS_REP_G0 = 204,   // [12]
    P_IS_REP_G1 = 216,   // [12]
    P_IS_REP_G2 = 228,   // [12]
    P_IS_REP0_LONG = 240,  // [12][16]
    P_POS_SLOT = 432,    // [4][64]
    P_SPEC_POS = 688,    // [114]
    P_ALIGN = 802,       // [16]
    P_LEN = 818,         // length coder (514)
    P_REP_LEN = 1332,    // rep length coder (514)
    P_LITERAL = 1846     // [0x300 << (lc+lp)]
};
enum : u32 { L_CHOICE = 0, L_CHOICE2 = 1, L_LOW = 2, L_MID = 130, L_HIGH = 258 };

ZX_INL u32 probs_count(u32 lclp) { return P_LITERAL + (0x300u << lclp); }

ZX_INL u32 check_size(u32 id) {
    // lzma_check_size(): 0,4,4,4,8,8,8,16,16,16,32,32,32,64,64,64
    return id == 0 ? 0u : (4u << ((id - 1) / 3));
}

ZX_INL u32 vli_size(u64 v) {
    u32 k = 0;
    do { v >>= 7; ++k; } while (v != 0);
    return k;
}

// CRC32 (IEEE, reflected) bit-serial update, for headers/index (a few bytes).
ZX_INL u32 crc32_byte(u32 c, u32 b) {
    c ^= b;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    return c;
}

// SHA-256 (FIPS 180-4) for the block check with ID 10 (liblzma verifies
// it: a mismatch is LZMA_DATA_ERROR).  The IO streams the block's output
// through sha256_compress (16 big-endian words per 64-byte block);
// sha256_tail pads the last partial block.
ZX_INL u32 sha_rotr(u32 x, u32 n) { return (x >> n) | (x << (32 - n)); }
ZX_INL void sha256_init(u32* h) {
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}
ZX_INL void sha256_compress(u32* h, const u32* m) {
    const u32 K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    u32 w[16];
    for (int i = 0; i < 16; i++) w[i] = m[i];
    u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        u32 wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const u32 w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const u32 s0 = sha_rotr(w15, 7) ^ sha_rotr(w15, 18) ^ (w15 >> 3);
            const u32 s1 = sha_rotr(w2, 17) ^ sha_rotr(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
        }
        const u32 S1 = sha_rotr(e, 6) ^ sha_rotr(e, 11) ^ sha_rotr(e, 25);
        const u32 ch = (e & f) ^ (~e & g);
        const u32 t1 = hh + S1 + ch + K[i] + wi;
        const u32 S0 = sha_rotr(a, 2) ^ sha_rotr(a, 13) ^ sha_rotr(a, 22);
        const u32 mj = (a & b) ^ (a & c) ^ (b & c);
        const u32 t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
// last[0, r) = the message's final r < 64 bytes; total = message length
ZX_INL void sha256_tail(u32* h, const u8* last, u32 r, u64 total) {
    u8 blk[128];
    for (u32 i = 0; i < 128; i++) blk[i] = 0;
    for (u32 i = 0; i < r; i++) blk[i] = last[i];
    blk[r] = 0x80;
    const u32 nb = r + 9 <= 64 ? 1u : 2u;
    const u64 bits = total * 8;
    for (u32 k = 0; k < 8; k++) blk[64 * nb - 1 - k] = (u8)(bits >> (8 * k));
    for (u32 q = 0; q < nb; q++) {
        u32 m[16];
        for (u32 i = 0; i < 16; i++)
            m[i] = ((u32)blk[64 * q + 4 * i] << 24) | ((u32)blk[64 * q + 4 * i + 1] << 16) |
                   ((u32)blk[64 * q + 4 * i + 2] << 8) | blk[64 * q + 4 * i + 3];
        sha256_compress(h, m);
    }
}

// 64-bit mixing hash of the (unpadded, uncompressed) size pairs; stands in
// for liblzma's index hash (best available check over the same pairs, in
// order): equal lists <=> equal hashes up to collisions.
ZX_INL u64 pair_hash(u64 h, u64 a, u64 b) {
    u64 x = h ^ (a * 0x9E3779B97F4A7C15ull);
    x = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    x ^= b * 0x94D049BB133111EBull;
    x = (x ^ (x >> 32)) * 0xD6E8FEB86659FD93ull;
    return x ^ (x >> 31);
}

struct IndexSums {
    u64 count, blocks_size, uncompressed, list_size, hash;
};

ZX_INL void sums_add(IndexSums& s, u64 unpadded, u64 usize) {
    s.count++;
    s.blocks_size += (unpadded + 3) & ~3ull;
    s.uncompressed += usize;
    s.list_size += vli_size(unpadded) + vli_size(usize);
    s.hash = pair_hash(s.hash, unpadded, usize);
}

// One adaptive binary decision of the LZMA range decoder (liblzma
// rc_bit: bound = (range >> 11) * p; code < bound -> bit 0, p += (2048-p)>>5;
// else bit 1, range -= bound, code -= bound, p -= p>>5).  On the device the
// state is wave-uniform, and the sequence is written as 14 SALU instructions
// (one compare, four SCC selects) — the compiler's own lowering of the
// selects round-trips the compare through a lane mask three times.
ZX_INL u32 rc_bit(u32& range, u32& code, u32& p) {
#if defined(__HIP_DEVICE_COMPILE__)
    u32 b, rb, t, q0, q1, bit;
    ZX_U32(range); ZX_U32(code); ZX_U32(p);  // folded away when already scalar
    asm("s_lshr_b32 %[b], %[r], 11\n\t"
        "s_mul_i32 %[b], %[b], %[p]\n\t"
        "s_sub_u32 %[rb], %[r], %[b]\n\t"
        "s_sub_u32 %[t], %[c], %[b]\n\t"
        "s_sub_u32 %[q0], 0x800, %[p]\n\t"
        "s_lshr_b32 %[q0], %[q0], 5\n\t"
        "s_add_u32 %[q0], %[p], %[q0]\n\t"
        "s_lshr_b32 %[q1], %[p], 5\n\t"
        "s_sub_u32 %[q1], %[p], %[q1]\n\t"
        "s_cmp_lt_u32 %[c], %[b]\n\t"
        "s_cselect_b32 %[r], %[b], %[rb]\n\t"
        "s_cselect_b32 %[c], %[c], %[t]\n\t"
        "s_cselect_b32 %[p], %[q0], %[q1]\n\t"
        "s_cselect_b32 %[bit], 0, 1"
        : [r] "+s"(range), [c] "+s"(code), [p] "+s"(p), [b] "=&s"(b), [rb] "=&s"(rb),
          [t] "=&s"(t), [q0] "=&s"(q0), [q1] "=&s"(q1), [bit] "=&s"(bit)
        :
        : "scc");
    return bit;
#else
    const u32 bound = (range >> 11) * p;
    if (code < bound) {
        range = bound;
        p += (2048 - p) >> 5;
        return 0;
    }
    range -= bound;
    code -= bound;
    p -= p >> 5;
    return 1;
#endif
}

// The LZMA symbol loop of one LZMA2 chunk: a separate (non-inlined on the
// device) function so its ~50 live values get their own register allocation,
// all 32-bit (the kernel restricts streams and chunks to < 4 GiB).  Returns
// ST_CONT when the chunk ended cleanly, otherwise the final status.
struct LzJob {
    u32 ip, lim, rlim, n, D, Dfull, chunk_end, dict_start, dsz, u_end, kstart, csz, full;
    u32 rc_range, rc_code, lc, lp, pb, state, rep0, rep1, rep2, rep3;
};
constexpr int ST_CONT = -1;

template <class IO>
ZX_HOT int lzma_symbols(IO& io_r, LzJob& j) {
    IO io = io_r;
    io.make_uniform();  // device: function arguments arrive as per-lane values
    u32 ip = j.ip, lim = j.lim;
    u32 rlim = j.rlim, n = j.n, D = j.D, Dfull = j.Dfull, chunk_end = j.chunk_end, dict_start = j.dict_start;
    u32 dsz = j.dsz, u_end = j.u_end, kstart = j.kstart, csz = j.csz;
    u32 fullw = j.full;
    u32 rc_range = j.rc_range, rc_code = j.rc_code;
    u32 lc = j.lc, lp = j.lp, pb = j.pb;
    u32 state = j.state, rep0 = j.rep0, rep1 = j.rep1, rep2 = j.rep2, rep3 = j.rep3;
    ZX_U32(ip); ZX_U32(lim); ZX_U32(rlim); ZX_U32(n); ZX_U32(D); ZX_U32(Dfull); ZX_U32(chunk_end);
    ZX_U32(dict_start); ZX_U32(dsz); ZX_U32(u_end); ZX_U32(kstart); ZX_U32(csz); ZX_U32(fullw);
    ZX_U32(rc_range); ZX_U32(rc_code); ZX_U32(lc); ZX_U32(lp); ZX_U32(pb);
    ZX_U32(state); ZX_U32(rep0); ZX_U32(rep1); ZX_U32(rep2); ZX_U32(rep3);
    bool full = fullw != 0;
    const u32 pb_mask = (1u << pb) - 1, lp_mask = (1u << lp) - 1;
    int rv = ST_CONT;
    // An input overrun inside a symbol is recorded here and reported at the
    // next symbol boundary (or at any earlier return, which it overrides);
    // the rest of that symbol decodes zero bytes, so the bit loops have no
    // exits.  liblzma returns the same status at the same input position.
    int frv = ST_CONT;
#define ZX_RET(v) do { rv = frv != ST_CONT ? frv : (v); goto out; } while (0)
#define ZX_SET_FULL() do { full = true; u32 ve = (u32)((((u64)ip - 1) / BUFREADER + 1) * BUFREADER); \
                           lim = ve < n ? ve : n; } while (0)

#define ZX_NORM()                                                              \
    do {                                                                       \
        if (rc_range < (1u << 24)) {                                           \
            const bool ok_ = ip < lim && ip < rlim;                            \
            if (!ok_ && frv == ST_CONT) frv = ip >= lim ? (full ? ST_OK : ST_EOF) : ST_INVALID; \
            rc_range <<= 8;                                                    \
            rc_code = (rc_code << 8) | (ok_ ? io.in(ip) : 0u);                 \
            ip += ok_ ? 1u : 0u;                                               \
        }                                                                      \
    } while (0)
// branch-free binary decision (the hot instruction sequence); the state is
// scalar (wave-uniform) here, so the selects below are s_cselect / masks
#define ZX_BIT(pidx, bitvar)                                     \
    do {                                                         \
        ZX_NORM();                                               \
        const u32 pi_ = (pidx);                                  \
        u32 p_ = io.pget(pi_);                                   \
        bitvar = rc_bit(rc_range, rc_code, p_);                  \
        io.pset(pi_, p_);                                        \
    } while (0)

        // Structured symbol decoder: one loop iteration per LZMA symbol;
        // every binary decision is the branch-free ZX_BIT sequence on
        // wave-uniform (scalar) state.
#define ZX_TREE(base, nbits, out)                                    \
    do {                                                             \
        u32 m_ = 1;                                                  \
        for (u32 k_ = 0; k_ < (nbits); k_++) {                       \
            u32 b_;                                                  \
            ZX_BIT((base) + m_, b_);                                 \
            m_ = (m_ << 1) | b_;                                     \
        }                                                            \
        out = m_ - (1u << (nbits));                                  \
    } while (0)
        for (;;) {
            ZX_U32(rc_range); ZX_U32(rc_code); ZX_U32(state); ZX_U32(ip); ZX_U64(io.pos);
            ZX_U32(rep0); ZX_U32(rep1); ZX_U32(rep2); ZX_U32(rep3);
            if (frv != ST_CONT) ZX_RET(frv);
            if ((u32)io.pos > u_end) ZX_RET(ST_INVALID);  // more than the declared size
            if ((u32)io.pos >= Dfull && !full) ZX_SET_FULL();  // (a match may step over Dfull < D)
            const u32 dlim = chunk_end < D ? chunk_end : D;
            if ((u32)io.pos == dlim) {
                // the main loop ends at the dictionary limit; one more
                // normalisation, then (chunk end) code must be 0
                ZX_NORM();
                if ((u32)io.pos != chunk_end) ZX_RET(ST_OK);  // output full mid-chunk
                if (rc_code != 0) ZX_RET(ST_INVALID);
                if (ip - kstart != csz) ZX_RET(ST_INVALID);
                ZX_RET(ST_CONT);
            }
            const u32 dpos = (u32)io.pos - dict_start;
            const u32 pos_state = dpos & pb_mask;
            u32 bit;
            ZX_BIT(P_IS_MATCH + (state << 4) + pos_state, bit);
            if (bit == 0) {
                // ---- literal ----
                const u32 prev = dpos ? io.back(0) : 0u;
                const u32 tb = P_LITERAL + 0x300u * (((dpos & lp_mask) << lc) + (prev >> (8 - lc)));
                u32 m = 1;
                if (state < 7) {
                    do {
                        ZX_BIT(tb + m, bit);
                        m = (m << 1) | bit;
                    } while (m < 0x100);
                } else {
                    u32 mb = io.back(rep0);
                    u32 off = 0x100;
                    do {
                        mb <<= 1;
                        const u32 mbit = mb & off;
                        ZX_BIT(tb + off + mbit + m, bit);
                        m = (m << 1) | bit;
                        off &= mbit ^ (bit - 1u);  // leaves matched mode on mismatch
                    } while (m < 0x100);
                }
                io.put(m & 0xFF);
                state = state < 4 ? 0 : (state < 10 ? state - 3 : state - 6);
                continue;
            }
            u32 lbase;
            ZX_BIT(P_IS_REP + state, bit);
            if (bit == 0) {  // simple match
                rep3 = rep2;
                rep2 = rep1;
                rep1 = rep0;
                lbase = P_LEN;
                state = state < 7 ? 7 : 10;
            } else {  // repeated match
                if (dpos == 0) ZX_RET(ST_INVALID);  // dict_is_distance_valid(dict, 0)
                ZX_BIT(P_IS_REP_G0 + state, bit);
                if (bit == 0) {
                    ZX_BIT(P_IS_REP0_LONG + (state << 4) + pos_state, bit);
                    if (bit == 0) {  // short rep: one byte at rep0
                        state = state < 7 ? 9 : 11;
                        io.put(io.back(rep0));
                        continue;
                    }
                } else {
                    u32 dist;
                    ZX_BIT(P_IS_REP_G1 + state, bit);
                    if (bit == 0) {
                        dist = rep1;
                    } else {
                        ZX_BIT(P_IS_REP_G2 + state, bit);
                        if (bit == 0) {
                            dist = rep2;
                        } else {
                            dist = rep3;
                            rep3 = rep2;
                        }
                        rep2 = rep1;
                    }
                    rep1 = rep0;
                    rep0 = dist;
                }
                lbase = P_REP_LEN;
                state = state < 7 ? 8 : 11;
            }
            // ---- length ----
            u32 len;
            ZX_BIT(lbase + L_CHOICE, bit);
            if (bit == 0) {
                ZX_TREE(lbase + L_LOW + (pos_state << 3), 3, len);
            } else {
                ZX_BIT(lbase + L_CHOICE2, bit);
                if (bit == 0) {
                    ZX_TREE(lbase + L_MID + (pos_state << 3), 3, len);
                    len += 8;
                } else {
                    ZX_TREE(lbase + L_HIGH, 8, len);
                    len += 16;
                }
            }
            len += 2;
            if (lbase == P_LEN) {
                // ---- distance ----
                const u32 lps = len - 2 < 3 ? len - 2 : 3;
                u32 slot;
                ZX_TREE(P_POS_SLOT + (lps << 6), 6, slot);
                u32 dist;
                if (slot < 4) {
                    dist = slot;
                } else {
                    const u32 nd = (slot >> 1) - 1;
                    dist = (2 | (slot & 1)) << nd;
                    u32 rb, rn;
                    if (slot < 14) {
                        rb = P_SPEC_POS + dist - slot - 1;
                        rn = nd;
                    } else {
                        u32 direct = 0;
                        for (u32 k = 0; k < nd - 4; k++) {
                            ZX_NORM();
                            rc_range >>= 1;
                            rc_code -= rc_range;
                            const u32 t = 0u - (rc_code >> 31);
                            rc_code += rc_range & t;
                            direct = (direct << 1) + (t + 1);
                            ZX_U32(rc_range); ZX_U32(rc_code); ZX_U32(direct);
                        }
                        dist += direct << 4;
                        rb = P_ALIGN;
                        rn = 4;
                    }
                    u32 mm = 1;
                    for (u32 k = 0; k < rn; k++) {
                        ZX_BIT(rb + mm, bit);
                        mm = (mm << 1) | bit;
                        dist |= bit << k;
                    }
                }
                rep0 = dist;
                if (rep0 == 0xFFFFFFFFu) ZX_RET(ST_INVALID);  // EOPM with known size
                const u32 dfull = dpos < dsz ? dpos : dsz;
                if (rep0 >= dfull) ZX_RET(ST_INVALID);
            }
            // ---- copy, clipped at the dictionary limit ----
            {
                const u32 room = dlim - (u32)io.pos;
                const u32 k = len <= room ? len : room;
                io.copy((u64)rep0 + 1, k);
                if (k < len) {
                    if (dlim == chunk_end) ZX_RET(ST_INVALID);  // match crosses the chunk end
                    if ((u32)io.pos > u_end) ZX_RET(ST_INVALID);
                    ZX_SET_FULL();
                    ZX_RET(ST_OK);  // output full, rest of the match pending
                }
            }
        }
#undef ZX_TREE
#undef ZX_BIT
#undef ZX_NORM
out:
    io_r = io;
    j.ip = ip; j.lim = lim; j.full = full ? 1u : 0u;
    j.rc_range = rc_range; j.rc_code = rc_code;
    j.state = state; j.rep0 = rep0; j.rep1 = rep1; j.rep2 = rep2; j.rep3 = rep3;
    return rv;
#undef ZX_RET
#undef ZX_STOP
#undef ZX_SET_FULL
}

// IO concept (see zcg_xz.hip / tests/hostcore/host_cores.cpp):
//   u64 n, D, pos;                       input size, output size, output pos
//   u32 in(u64 i);                       input byte i (i < n)
//   u32 pget(u32 i); void pset(u32 i, u32 v);   probability model
//   void init_probs(u32 count);          all = 1024
//   bool lclp_ok(u32 lclp);              false -> ST_NEED_BIG (LDS too small)
//   void put(u32 b);                     append one byte
//   u32 back(u64 dist);                  byte at pos-1-dist
//   void copy(u64 d, u32 len);           append len bytes from d bytes back
//   void copy_in(u64 ip, u32 len);       append input bytes [ip, ip+len)
//   u64 check(u32 id, u64 a, u64 b);     CRC32 (id 1) / CRC64 (id 4) of out[a,b)
//   void sha256(u64 a, u64 b, u32* h);   SHA-256 state words of out[a,b)
//   void finish();                       make all output visible in dst
//   void apply_delta(u64 a, u64 b, u32 dist);  delta filter decode of out[a,b) in place
//   BcjState apply_bcj(u64 a, u64 b, u32 id, u32 start);  BCJ filter decode of out[a,b) (bcj_run below):
//                                        where its loop stopped, and the x86 state there
//   void reset();                        output position back to 0 (the stream is decoded again)
//   u32 tail_byte(u64 i);                output byte i >= D (decoded past the caller's end)
//   void set_byte(u64 i, u32 v);         output byte i < D (after finish())
//   u32 out_byte(u64 i);                 output byte i (after finish())
// A block whose chain is delta + LZMA2 (liblzma's delta decoder passes the
// LZMA2 output through, then adds the byte `dist` back: out[i] += out[i-dist],
// history zero at the block start) or BCJ + LZMA2 (liblzma simple/*.c: branch
// targets converted back from absolute to relative) is filter-decoded when
// it ends (before its check, which covers the filtered bytes) or, if
// decoding stops inside it, by xz_decode's wrapper.  LZMA2 matches read the
// unfiltered dictionary, which a block never shares with the next (its first
// chunk resets the dictionary).  A BCJ filter converts an instruction only
// when all its bytes are known; liblzma's simple coder decodes past the
// caller's output end to finish one.  For one BCJ stage fed by LZMA2 that
// look-past decode is modelled exactly (xz_decode); for other chains a stop
// whose last bytes could start an instruction (bcj_tail_open) is
// UNSUPPORTED rather than possibly different bytes.
// Chains of up to three such filters before LZMA2 (liblzma's limit) decode
// in reverse chain order, each over the previous one's output.
struct FilterPending {
    u64 start;
    u32 n;         // filters before LZMA2 (0: none)
    u32 kind[3];   // chain order: 3 delta, 4..9 BCJ x86 / PowerPC / IA-64 / ARM / ARM-Thumb / SPARC (the filter ids)
    u32 param[3];  // delta distance / BCJ start offset
};

// ---- BCJ decoders, serial (liblzma simple/{x86,powerpc,ia64,arm,armthumb,sparc}.c
// restated from the published algorithm): buf[0, len) is one block's output,
// `pos0` its start offset; the whole block in one call equals liblzma's
// incremental calls (each leaves the bytes of an unfinished instruction).
// one aligned word of the ARM (BL), PowerPC (b/bl with AA=0 LK=1) or SPARC (call) filters
template <class B>
ZX_INL void bcj_word(B& buf, u64 i, u32 id, u32 now) {
    const u32 b0 = buf.get(i), b1 = buf.get(i + 1), b2 = buf.get(i + 2), b3 = buf.get(i + 3);
    if (id == 7) {  // ARM
        if (b3 != 0xEB) return;
        const u32 dest = (((b2 << 16) | (b1 << 8) | b0) << 2) - (now + 8);
        const u32 d = dest >> 2;
        buf.set(i + 2, (d >> 16) & 0xFF);
        buf.set(i + 1, (d >> 8) & 0xFF);
        buf.set(i, d & 0xFF);
    } else if (id == 5) {  // PowerPC (big-endian)
        if ((b0 >> 2) != 0x12 || (b3 & 3) != 1) return;
        const u32 src = ((b0 & 3) << 24) | (b1 << 16) | (b2 << 8) | (b3 & ~3u);
        const u32 dest = src - now;
        buf.set(i, 0x48 | ((dest >> 24) & 3));
        buf.set(i + 1, (dest >> 16) & 0xFF);
        buf.set(i + 2, (dest >> 8) & 0xFF);
        buf.set(i + 3, ((b3 & 3) | dest) & 0xFF);
    } else if (id == 9) {  // SPARC
        if (!((b0 == 0x40 && (b1 & 0xC0) == 0) || (b0 == 0x7F && (b1 & 0xC0) == 0xC0))) return;
        u32 src = ((b0 << 24) | (b1 << 16) | (b2 << 8) | b3) << 2;
        u32 dest = (src - now) >> 2;
        dest = (((0u - ((dest >> 22) & 1)) << 22) & 0x3FFFFFFFu) | (dest & 0x3FFFFFu) | 0x40000000u;
        buf.set(i, dest >> 24);
        buf.set(i + 1, (dest >> 16) & 0xFF);
        buf.set(i + 2, (dest >> 8) & 0xFF);
        buf.set(i + 3, dest & 0xFF);
    }
}
// one 16-byte IA-64 bundle: the template's branch slots, 41-bit slots from bit 5
template <class B>
ZX_INL void bcj_ia64_bundle(B& buf, u64 i, u32 now) {
    const u32 branch[32] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                            4, 4, 6, 6, 0, 0, 7, 7, 4, 4, 0, 0, 4, 4, 0, 0};
    const u32 mask = branch[buf.get(i) & 0x1F];
    u32 bit_pos = 5;
    for (u32 slot = 0; slot < 3; slot++, bit_pos += 41) {
        if (((mask >> slot) & 1) == 0) continue;
        const u32 byte_pos = bit_pos >> 3, bit_res = bit_pos & 7;
        u64 instr = 0;
        for (u32 j = 0; j < 6; j++) instr |= (u64)buf.get(i + j + byte_pos) << (8 * j);
        u64 norm = instr >> bit_res;
        if (((norm >> 37) & 0xF) != 0x5 || ((norm >> 9) & 0x7) != 0) continue;
        u32 src = (u32)((norm >> 13) & 0xFFFFF);
        src |= (u32)((norm >> 36) & 1) << 20;
        src <<= 4;
        const u32 dest = (src - now) >> 4;
        norm &= ~((u64)0x8FFFFF << 13);
        norm |= (u64)(dest & 0xFFFFF) << 13;
        norm |= (u64)(dest & 0x100000) << (36 - 20);
        instr &= (1ull << bit_res) - 1;
        instr |= norm << bit_res;
        for (u32 j = 0; j < 6; j++) buf.set(i + j + byte_pos, (u32)(instr >> (8 * j)) & 0xFF);
    }
}
ZX_INL bool bcj_x86_ms(u32 b) { return b == 0 || b == 0xFF; }
// Scan state of a BCJ filter where its loop stopped: `stop` = the first
// position (relative to the block start) the loop did not process (liblzma's
// `filtered`), and for x86 the prev_mask / prev_pos carried to the next call.
struct BcjState {
    u64 stop;
    u32 prev_mask, prev_pos;
};
// bytes per loop step window: x86 5 (opcode + rel32), IA-64 16 (a bundle),
// the others 4 (a word or a Thumb BL pair)
ZX_INL u32 bcj_window(u32 id) { return id == 4 ? 5u : id == 6 ? 16u : 4u; }
// liblzma's simple coder keeps 2 x unfiltered_max bytes of buffer
// (simple_coder.c): x86 5, IA-64 16, the others 4
ZX_INL u32 bcj_allocated(u32 id) { return 2u * (id == 4 ? 5u : id == 6 ? 16u : 4u); }
// The filter loop over buf[i0, len) from state st (liblzma simple/*.c;
// whole-block equivalent to its incremental calls).  Returns the new state;
// *last = the last position < lim_last the loop processed (or ~0).
template <class B>
ZX_INL BcjState bcj_run(B& buf, u64 i0, u64 len, u32 id, u32 pos0, BcjState st, u64 lim_last = 0, u64* last = nullptr) {
    u64 i = i0;
    if (id == 4) {  // x86: E8 (call) / E9 (jmp) rel32, with the prev_mask heuristic
        const bool allowed[8] = {true, true, true, false, true, false, false, false};
        const u32 bitnum[8] = {0, 1, 2, 2, 3, 3, 3, 3};
        u32 prev_mask = st.prev_mask, prev_pos = st.prev_pos;
        while (i + 5 <= len) {
            if (last && i < lim_last) *last = i;
            const u32 b0 = buf.get(i);
            if (b0 != 0xE8 && b0 != 0xE9) { i++; continue; }
            const u32 now = pos0 + (u32)i;
            const u32 off = now - prev_pos;
            prev_pos = now;
            if (off > 5) prev_mask = 0;
            else
                for (u32 k = 0; k < off; k++) prev_mask = (prev_mask & 0x77) << 1;
            u32 b4 = buf.get(i + 4);
            if (bcj_x86_ms(b4) && allowed[(prev_mask >> 1) & 7] && (prev_mask >> 1) < 0x10) {
                u32 src = (b4 << 24) | (buf.get(i + 3) << 16) | (buf.get(i + 2) << 8) | buf.get(i + 1);
                u32 dest;
                for (;;) {
                    dest = src - (now + 5);
                    if (prev_mask == 0) break;
                    const u32 k = bitnum[prev_mask >> 1];
                    if (!bcj_x86_ms((dest >> (24 - k * 8)) & 0xFF)) break;
                    src = dest ^ ((1u << (32 - k * 8)) - 1);
                }
                buf.set(i + 4, (~(((dest >> 24) & 1) - 1)) & 0xFF);
                buf.set(i + 3, (dest >> 16) & 0xFF);
                buf.set(i + 2, (dest >> 8) & 0xFF);
                buf.set(i + 1, dest & 0xFF);
                i += 5;
                prev_mask = 0;
            } else {
                i++;
                prev_mask |= 1;
                if (bcj_x86_ms(b4)) prev_mask |= 0x10;
            }
        }
        return BcjState{i, prev_mask, prev_pos};
    }
    if (id == 8) {  // ARM-Thumb: BL pairs, 2-byte steps
        while (i + 4 <= len) {
            if (last && i < lim_last) *last = i;
            const u32 b1 = buf.get(i + 1), b3 = buf.get(i + 3);
            if ((b1 & 0xF8) != 0xF0 || (b3 & 0xF8) != 0xF8) { i += 2; continue; }
            u32 src = ((b1 & 7) << 19) | (buf.get(i) << 11) | ((b3 & 7) << 8) | buf.get(i + 2);
            src <<= 1;
            u32 dest = (src - (pos0 + (u32)i + 4)) >> 1;
            buf.set(i + 1, 0xF0 | ((dest >> 19) & 7));
            buf.set(i, (dest >> 11) & 0xFF);
            buf.set(i + 3, 0xF8 | ((dest >> 8) & 7));
            buf.set(i + 2, dest & 0xFF);
            i += 4;
        }
        return BcjState{i, 0u, 0u};
    }
    const u32 w = id == 6 ? 16u : 4u;  // IA-64 bundles / 4-byte words, each independent
    for (; i + w <= len; i += w) {
        if (last && i < lim_last) *last = i;
        if (id == 6) bcj_ia64_bundle(buf, i, pos0 + (u32)i);
        else bcj_word(buf, i, id, pos0 + (u32)i);
    }
    return BcjState{i, 0u, 0u};
}
template <class B>
ZX_INL BcjState bcj_serial(B& buf, u64 len, u32 id, u32 pos0) {
    return bcj_run(buf, 0, len, id, pos0, BcjState{0, 0u, pos0 - 5});
}
// After decoding stopped inside a BCJ block at io.pos: could its last bytes
// start an instruction whose conversion depends on bytes not decoded?
// (Kept for chains the tail decode below does not cover.)
template <class IO>
ZX_INL bool bcj_tail_open(IO& io, u64 a, u32 id) {
    const u64 len = io.pos - a;
    if (id == 4) {  // an E8/E9 in the last 4 bytes
        for (u64 k = 1; k <= 4 && k <= len; k++) {
            const u32 x = io.out_byte(io.pos - k);
            if (x == 0xE8 || x == 0xE9) return true;
        }
        return false;
    }
    if (id == 8) return (len & 1) || (len >= 1 && (io.out_byte(io.pos - 1) & 0xF8) == 0xF0);
    if (id == 6) return (len & 15) != 0;  // a partial last bundle
    return (len & 3) != 0;  // a partial last word
}

// Decode the pending filters over [fp.start, io.pos); `partial`: decoding
// stopped inside the block, so a BCJ stage whose input tail is open makes the
// result UNSUPPORTED (checked on that stage's input, after the stages before it)
template <class IO>
ZX_INL bool apply_filters(IO& io, const FilterPending& fp, bool partial) {
    io.finish();
    for (u32 k = fp.n; k-- > 0;) {
        if (fp.kind[k] == 3) {
            io.apply_delta(fp.start, io.pos, fp.param[k]);
        } else {
            if (partial && bcj_tail_open(io, fp.start, fp.kind[k])) return false;
            io.apply_bcj(fp.start, io.pos, fp.kind[k], fp.param[k]);
        }
        io.finish();
    }
    return true;
}
template <class IO>
ZX_INL int xz_decode_blocks(IO& io, FilterPending& fp, u64 Ddec, u64 Dfull, bool tail, u64* lzend);
// Block-relative view of one block's output for the BCJ tail loop: bytes
// below N from the output, bytes from N on (decoded past the caller's end)
// from the IO's tail store; writes land only below N.
template <class IO>
struct BcjTailBuf {
    IO* io;
    u64 a, D;
    bool write;
    ZX_INL u32 get(u64 i) { return a + i < D ? io->out_byte(a + i) : io->tail_byte(a + i); }
    ZX_INL void set(u64 i, u32 v) {
        if (write && a + i < D) io->set_byte(a + i, v);
    }
};
// A read that stops inside a block whose innermost filter (the one LZMA2
// feeds) is BCJ and the only BCJ of the chain.  liblzma's simple coder
// (simple_coder.c) holds back the bytes its loop has not processed and, to
// release them, decodes past the caller's end into its buffer of
// 2 x unfiltered_max bytes.  Modelled with two more decodes of the stream:
//   A: past N with no input window limit (read_exact keeps calling read(),
//      which refills the window), to find E, the least decoded extent at
//      which the filter loop passes N (or the LZMA2 data ends): input that
//      ends, or data that fail, before E give UnexpectedEof / InvalidData;
//   C: up to U + allocated (U = where the loop stopped at N), with the
//      window limit from E on (the call that releases byte N - 1 sees only
//      its window): a data error there is InvalidData, running out is not.
// The loop then runs over C's extent, and the outer (delta) filters over
// [start, N).  Chains with a second BCJ, or a delta under the BCJ, keep the
// open-tail rule (UNSUPPORTED).
template <class IO>
ZX_INL int xz_decode(IO& io) {
    const u64 D = io.D;
    FilterPending fp, keep;
    fp.start = 0;
    fp.n = 0;
    keep = fp;
    // pass 0: the read itself; 1: A; 2: C (one call site, so the stream
    // decoder is inlined once)
    u64 Ddec = D, Dfull = D, a = 0, U = 0, E = 0, lzend = ~0ull;
    u32 id = 0, so = 0, nf = 0;
    BcjState s0{0, 0u, 0u};
    int rA = ST_OK;
    for (u32 pass = 0;; pass++) {
        if (pass > 0) {
            io.reset();
            fp.n = 0;
        }
        lzend = ~0ull;
        const int r = xz_decode_blocks(io, fp, Ddec, Dfull, pass > 0, &lzend);
        if (pass == 0) {
            if (!fp.n) return r;
            nf = fp.n;
            id = fp.kind[nf - 1];
            bool one_bcj = id != 3;
            for (u32 k = 0; k + 1 < nf; k++)
                if (fp.kind[k] != 3) one_bcj = false;
            if (r != ST_OK || !one_bcj) {
                if (!apply_filters(io, fp, r == ST_OK)) return ST_UNSUPPORTED;
                return r;
            }
            a = fp.start;
            so = fp.param[nf - 1];
            keep = fp;
            io.finish();
            s0 = io.apply_bcj(a, D, id, so);  // [a, a + stop) converted
            U = a + s0.stop;
            if (U >= D) break;                // nothing held back
            Ddec = U + bcj_allocated(id);
            Dfull = ~0ull;                    // A: no window limit
            continue;
        }
        if (pass == 1) {
            rA = r;
            const u64 XA = io.pos;
            io.finish();
            BcjTailBuf<IO> tb{&io, a, D, false};
            u64 lastp = ~0ull;
            const BcjState sA = bcj_run(tb, s0.stop, XA - a, id, so, s0, D - a, &lastp);
            if (a + sA.stop >= D) {
                E = lastp == ~0ull ? D : a + lastp + bcj_window(id);
                if (E < D) E = D;
                if (lzend != ~0ull && lzend < E) E = lzend;
            } else if (lzend != ~0ull) {
                E = lzend;  // end_was_reached: everything counts as filtered
            } else {
                return rA == ST_OK ? ST_INVALID : rA;  // (rA is EOF or InvalidData here)
            }
            Dfull = E;  // C: the window limit from E on
            continue;
        }
        if (r != ST_OK) return r;
        const u64 XC = io.pos;
        fp = keep;
        io.finish();
        s0 = io.apply_bcj(a, D, id, so);
        BcjTailBuf<IO> tw{&io, a, D, true};
        bcj_run(tw, s0.stop, XC - a, id, so, s0);  // (at the LZMA2 end the unprocessed rest stays as decoded)
        io.finish();
        break;
    }
    for (u32 k = nf - 1; k-- > 0;) {  // outer delta stages over [start, N)
        io.apply_delta(a, D, keep.param[k]);
        io.finish();
    }
    return ST_OK;
}
template <class IO>
ZX_INL int xz_decode_blocks(IO& io, FilterPending& fp, u64 Ddec, u64 Dfull, bool tail, u64* lzend) {
    const u64 n = io.n;
    const u64 D = io.D;
    u64 ip = 0;       // input position
    u64 lim = n;      // visible input end (moves to the BufReader window end once full)
    bool full = false;

#define ZX_STOP() return full ? ST_OK : ST_EOF
#define ZX_NEED(k) do { if (ip + (u64)(k) > lim) ZX_STOP(); } while (0)
#define ZX_SET_FULL() do { full = true; u64 ve = ((ip - 1) / BUFREADER + 1) * BUFREADER; \
                           lim = ve < n ? ve : n; } while (0)

    if (D == 0) return ST_OK;  // read_exact of an empty buffer never reads
    if (n >= 0xFFFFFFFFull || D >= 0xFFFFFFFFull) return ST_UNSUPPORTED;  // 32-bit positions

    // ---- stream header (stream_flags_decoder.c: magic, CRC32, flags) ----
    ZX_NEED(12);
    {
        if (io.in(0) != 0xFD || io.in(1) != 0x37 || io.in(2) != 0x7A || io.in(3) != 0x58 ||
            io.in(4) != 0x5A || io.in(5) != 0x00)
            return ST_INVALID;
        u32 c = 0xFFFFFFFFu;
        c = crc32_byte(c, io.in(6));
        c = crc32_byte(c, io.in(7));
        c = ~c;
        const u32 stored = io.in(8) | (io.in(9) << 8) | (io.in(10) << 16) | (io.in(11) << 24);
        if (c != stored) return ST_INVALID;
        if (io.in(6) != 0 || (io.in(7) & 0xF0)) return ST_INVALID;
    }
    const u32 check_id = io.in(7) & 0x0F;
    const u32 csz_check = check_size(check_id);
    ip = 12;

    IndexSums blocks = {0, 0, 0, 0, 0};

    // ---- blocks ----------------------------------------------------------
    for (;;) {
        ZX_NEED(1);
        const u32 b0 = io.in(ip);
        if (b0 == 0) break;  // Index Indicator
        const u32 hsize = (b0 + 1) * 4;
        ZX_NEED(hsize);  // lzma_bufcpy of the whole header first
        const u64 h0 = ip, hend = ip + hsize - 4;
        {
            u32 c = 0xFFFFFFFFu;
            for (u64 q = h0; q < hend; q++) c = crc32_byte(c, io.in(q));
            c = ~c;
            const u32 stored = io.in(hend) | (io.in(hend + 1) << 8) | (io.in(hend + 2) << 16) |
                               (io.in(hend + 3) << 24);
            if (c != stored) return ST_INVALID;
        }
        const u32 bflags = io.in(h0 + 1);
        if (bflags & 0x3C) return ST_INVALID;
        u64 hp = h0 + 2;
        u64 dec_csize = VLI_UNKNOWN, dec_usize = VLI_UNKNOWN;
        // single-call lzma_vli_decode: running out of header is DATA_ERROR
        auto vli_hdr = [&](u64* out) -> bool {
            u64 v = 0;
            for (u32 k = 0;; k++) {
                if (hp >= hend) return false;
                const u32 b = io.in(hp++);
                v |= (u64)(b & 0x7F) << (7 * k);
                if (!(b & 0x80)) {
                    if (b == 0 && k > 0) return false;
                    *out = v;
                    return true;
                }
                if (k + 1 == 9) return false;
            }
        };
        if (bflags & 0x40) {
            if (!vli_hdr(&dec_csize)) return ST_INVALID;
            // lzma_block_unpadded_size() == 0 -> DATA_ERROR
            if (dec_csize == 0 || dec_csize > VLI_MAX) return ST_INVALID;
            const u64 unp = dec_csize + hsize + csz_check;
            if (unp > UNPADDED_MAX || unp < dec_csize) return ST_INVALID;
        }
        if (bflags & 0x80) {
            if (!vli_hdr(&dec_usize)) return ST_INVALID;
        }
        const u32 nfilt = (bflags & 3) + 1;
        u64 fid[4];
        u32 dict_prop = 0, nf = 0, fkind[3] = {0, 0, 0}, fparam[3] = {0, 0, 0};
        bool unsupported_chain = false;
        for (u32 f = 0; f < nfilt; f++) {
            u64 id = 0, psz = 0;
            if (!vli_hdr(&id)) return ST_INVALID;
            if (id >= (1ull << 62)) return ST_INVALID;
            if (!vli_hdr(&psz)) return ST_INVALID;
            if (psz > hend - hp) return ST_INVALID;
            fid[f] = id;
            // lzma_properties_decode of the filters liblzma 5.2 knows
            if (id == 0x21) {  // LZMA2
                if (psz != 1) return ST_INVALID;
                dict_prop = io.in(hp);
                if (dict_prop > 40) return ST_INVALID;
            } else if (id == 0x03) {  // delta: distance = property + 1
                if (psz != 1) return ST_INVALID;
                if (f < 3) { fkind[f] = 3; fparam[f] = io.in(hp) + 1; nf = f + 1; }
            } else if (id >= 0x04 && id <= 0x09) {  // BCJ filters: optional 4-byte start offset
                if (psz != 0 && psz != 4) return ST_INVALID;
                if (f < 3) {
                    fkind[f] = (u32)id;
                    fparam[f] = psz == 4 ? io.in(hp) | (io.in(hp + 1) << 8) | (io.in(hp + 2) << 16) | (io.in(hp + 3) << 24)
                                         : 0u;
                    nf = f + 1;
                }
            } else if (id == 0x4000000000000001ull) {  // LZMA1
                if (psz != 5) return ST_INVALID;
                unsupported_chain = true;
            } else {
                return ST_INVALID;  // unknown filter: OPTIONS_ERROR
            }
            hp += psz;
        }
        while (hp < hend)
            if (io.in(hp++) != 0) return ST_INVALID;  // header padding
        // validate_chain(): LZMA1/LZMA2 only as the last filter, last must be one
        for (u32 f = 0; f < nfilt; f++) {
            const bool lz = fid[f] == 0x21 || fid[f] == 0x4000000000000001ull;
            if (lz != (f + 1 == nfilt)) return ST_INVALID;
        }
        // liblzma 5.2's .xz decoder rejects an LZMA1 block with LZMA_DATA_ERROR
        // (measured with the oracle over lc/lp/pb, dictionary sizes, checks and
        // size fields), so it is InvalidData here too
        if (unsupported_chain) return ST_INVALID;

        ip = h0 + hsize;
        const u64 cstart = ip;             // block compressed data start
        const u64 ustart = io.pos;         // block uncompressed data start
        fp.start = ustart;
        fp.n = nf;
        for (u32 k = 0; k < 3; k++) { fp.kind[k] = fkind[k]; fp.param[k] = fparam[k]; }
        const u64 climit = (dec_csize != VLI_UNKNOWN) ? dec_csize
                                                       : (VLI_MAX & ~3ull) - hsize - csz_check;
        const u64 c_end = (climit > n) ? ~0ull : cstart + climit;  // compressed bytes < c_end
        const u64 u_end = (dec_usize != VLI_UNKNOWN) ? ustart + dec_usize : ~0ull;

        // LZMA2 dictionary: lz_decoder rounds up to >= 4096 and a multiple of 16
        u64 dsz = (dict_prop == 40) ? 0xFFFFFFFFull
                                    : ((u64)(2 | (dict_prop & 1)) << (dict_prop / 2 + 11));
        if (dsz < 4096) dsz = 4096;
        dsz = (dsz + 15) & ~15ull;

        // LZMA2 / LZMA state
        bool need_dict_reset = true, need_props = true;
        u64 dict_start = io.pos;
        u32 lc = 0, lp = 0, pb = 0;
        u32 state = 0, rep0 = 0, rep1 = 0, rep2 = 0, rep3 = 0;
        u32 rc_range = 0xFFFFFFFFu, rc_code = 0;

        for (;;) {  // LZMA2 chunks
            ZX_NEED(1);
            if (ip >= c_end) return ST_INVALID;
            const u32 ctl = io.in(ip++);
            if (ctl == 0) {  // end of LZMA2 data
                if (tail && io.pos >= D) {  // the simple coder's end_was_reached: nothing past it is read
                    *lzend = io.pos;
                    return ST_OK;
                }
                break;
            }
            if (ctl >= 0xE0 || ctl == 1) {
                need_props = true;
                need_dict_reset = true;
            } else if (need_dict_reset) {
                return ST_INVALID;
            }
            bool new_props = false, state_reset = false;
            if (ctl >= 0x80) {
                if (ctl >= 0xC0) {
                    need_props = false;
                    new_props = true;
                } else if (need_props) {
                    return ST_INVALID;
                } else if (ctl >= 0xA0) {
                    state_reset = true;
                }
            } else if (ctl > 2) {
                return ST_INVALID;
            }
            if (need_dict_reset) {
                need_dict_reset = false;
                dict_start = io.pos;  // dict_reset(): empty dictionary, prev byte 0
                if (io.pos >= Ddec) return ST_OK;  // decode_buffer returns after a reset when out is full
            }
            if (ctl >= 0x80) {
                // ---- LZMA chunk header ----
                ZX_NEED(4);
                if (ip + 4 > c_end) return ST_INVALID;
                const u32 usz = ((ctl & 0x1F) << 16) + (io.in(ip) << 8) + io.in(ip + 1) + 1;
                const u32 csz = (io.in(ip + 2) << 8) + io.in(ip + 3) + 1;
                ip += 4;
                if (new_props) {
                    ZX_NEED(1);
                    if (ip >= c_end) return ST_INVALID;
                    u32 pr = io.in(ip++);
                    if (pr > (4 * 5 + 4) * 9 + 8) return ST_INVALID;
                    pb = pr / (9 * 5);
                    pr -= pb * 9 * 5;
                    lp = pr / 9;
                    lc = pr - lp * 9;
                    if (lc + lp > 4) return ST_INVALID;
                    if (!io.lclp_ok(lc + lp)) return ST_NEED_BIG;
                    state_reset = true;
                }
                if (state_reset) {
                    io.init_probs(probs_count(lc + lp));
                    state = 0;
                    rep0 = rep1 = rep2 = rep3 = 0;
                }
                const u64 kstart = ip;  // chunk compressed data start
                const u64 rlim = (kstart + csz < c_end) ? kstart + csz : c_end;
                // range decoder init: 5 bytes, the first one must be 0
                rc_range = 0xFFFFFFFFu;
                rc_code = 0;
                for (int k = 0; k < 5; k++) {
                    ZX_NEED(1);
                    if (ip >= rlim) return ST_INVALID;
                    const u32 b = io.in(ip++);
                    if (k == 0 && b != 0) return ST_INVALID;
                    rc_code = (rc_code << 8) | b;
                    ZX_U32(rc_code);
                }
                LzJob j;
                j.ip = (u32)ip; j.lim = (u32)lim; j.rlim = (u32)rlim; j.n = (u32)n; j.D = (u32)Ddec;
                j.Dfull = Dfull > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)Dfull;
                j.chunk_end = (u32)(io.pos + usz); j.dict_start = (u32)dict_start;
                j.dsz = dsz > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)dsz;
                j.u_end = u_end > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)u_end;
                j.kstart = (u32)kstart; j.csz = csz; j.full = full ? 1u : 0u;
                j.rc_range = rc_range; j.rc_code = rc_code; j.lc = lc; j.lp = lp; j.pb = pb;
                j.state = state; j.rep0 = rep0; j.rep1 = rep1; j.rep2 = rep2; j.rep3 = rep3;
                const int r = lzma_symbols(io, j);
                ip = j.ip; lim = j.lim; full = j.full != 0;
                rc_range = j.rc_range; rc_code = j.rc_code;
                state = j.state; rep0 = j.rep0; rep1 = j.rep1; rep2 = j.rep2; rep3 = j.rep3;
                if (r != ST_CONT) return r;
            } else {
                // ---- uncompressed chunk ----
                ZX_NEED(2);
                if (ip + 2 > c_end) return ST_INVALID;
                u32 left = ((io.in(ip) << 8) | io.in(ip + 1)) + 1;
                ip += 2;
                while (left > 0) {
                    if (io.pos == Ddec) return ST_OK;  // dict full: dict_write copies nothing
                    ZX_NEED(1);
                    u64 k = left;
                    if (k > lim - ip) k = lim - ip;
                    if (k > Ddec - io.pos) k = Ddec - io.pos;
                    if (!full && io.pos < Dfull && k > Dfull - io.pos) k = Dfull - io.pos;
                    if (ip + k > c_end) return ST_INVALID;
                    io.copy_in(ip, (u32)k);
                    ip += k;
                    left -= (u32)k;
                    if (io.pos > u_end) return ST_INVALID;
                    if (io.pos == Dfull && !full) ZX_SET_FULL();
                }
            }
        }
        // ---- block end (block_decoder.c SEQ_CODE -> PADDING -> CHECK) ----
        if (fp.n) {  // the filters' output is what the check covers
            apply_filters(io, fp, false);
            fp.n = 0;
        }
        const u64 actual_c = ip - cstart;
        const u64 actual_u = io.pos - ustart;
        if (dec_csize != VLI_UNKNOWN && actual_c != dec_csize) return ST_INVALID;
        if (dec_usize != VLI_UNKNOWN && actual_u != dec_usize) return ST_INVALID;
        for (u64 padded = actual_c; padded & 3; padded++) {
            ZX_NEED(1);
            if (io.in(ip++) != 0) return ST_INVALID;
        }
        if (csz_check) {
            ZX_NEED(csz_check);  // lzma_bufcpy of the whole check first
            if (check_id == 1 || check_id == 4) {
                io.finish();
                const u64 c = io.check(check_id, ustart, io.pos);
                for (u32 k = 0; k < csz_check; k++)
                    if (io.in(ip + k) != (u32)((c >> (8 * k)) & 0xFF)) return ST_INVALID;
            } else if (check_id == 10) {  // SHA-256 (the digest's bytes in order)
                io.finish();
                u32 hsh[8];
                io.sha256(ustart, io.pos, hsh);
                for (u32 k = 0; k < 32; k++)
                    if (io.in(ip + k) != ((hsh[k >> 2] >> (24 - 8 * (k & 3))) & 0xFFu)) return ST_INVALID;
            }
            ip += csz_check;
        }
        sums_add(blocks, hsize + actual_c + csz_check, actual_u);
    }

    // ---- index (index_hash.c lzma_index_hash_decode) ----------------------
    const u64 istart = ip;
    u32 icrc = 0xFFFFFFFFu;
    auto ibyte = [&](u32* b) -> int {  // 0 = ok, 1 = no input
        if (ip >= lim) return 1;
        *b = io.in(ip++);
        icrc = crc32_byte(icrc, *b);
        return 0;
    };
    // streaming lzma_vli_decode: partial input waits, padding zeros invalid
    auto ivli = [&](u64* out) -> int {  // 0 ok, 1 no input, 2 invalid
        u64 v = 0;
        for (u32 k = 0;; k++) {
            u32 b;
            if (ibyte(&b)) return 1;
            v |= (u64)(b & 0x7F) << (7 * k);
            if (!(b & 0x80)) {
                if (b == 0 && k > 0) return 2;
                *out = v;
                return 0;
            }
            if (k + 1 == 9) return 2;
        }
    };
    {
        u32 ind;
        if (ibyte(&ind)) ZX_STOP();
        (void)ind;  // == 0, checked by the block loop
        u64 count = 0;
        int r = ivli(&count);
        if (r == 1) ZX_STOP();
        if (r == 2 || count != blocks.count) return ST_INVALID;
        IndexSums rec = {0, 0, 0, 0, 0};
        for (u64 i = 0; i < count; i++) {
            u64 unp = 0, usz = 0;
            r = ivli(&unp);
            if (r == 1) ZX_STOP();
            if (r == 2) return ST_INVALID;
            if (unp < UNPADDED_MIN || unp > UNPADDED_MAX) return ST_INVALID;
            r = ivli(&usz);
            if (r == 1) ZX_STOP();
            if (r == 2) return ST_INVALID;
            sums_add(rec, unp, usz);
            if (blocks.blocks_size < rec.blocks_size || blocks.uncompressed < rec.uncompressed ||
                blocks.list_size < rec.list_size)
                return ST_INVALID;
        }
        const u64 unpadded_index = 1 + vli_size(count) + rec.list_size + 4;
        for (u64 pad = (4 - (unpadded_index & 3)) & 3; pad > 0; pad--) {
            u32 b;
            if (ibyte(&b)) ZX_STOP();
            if (b != 0) return ST_INVALID;
        }
        if (blocks.blocks_size != rec.blocks_size || blocks.uncompressed != rec.uncompressed ||
            blocks.list_size != rec.list_size || blocks.hash != rec.hash)
            return ST_INVALID;
        const u32 crc = ~icrc;
        for (int k = 0; k < 4; k++) {
            if (ip >= lim) ZX_STOP();
            if (io.in(ip++) != ((crc >> (8 * k)) & 0xFF)) return ST_INVALID;
        }
        const u64 index_size = (unpadded_index + 3) & ~3ull;
        (void)istart;
        // ---- stream footer ----
        ZX_NEED(12);
        if (io.in(ip + 10) != 0x59 || io.in(ip + 11) != 0x5A) return ST_INVALID;
        u32 c = 0xFFFFFFFFu;
        for (int k = 4; k < 10; k++) c = crc32_byte(c, io.in(ip + k));
        c = ~c;
        const u32 stored = io.in(ip) | (io.in(ip + 1) << 8) | (io.in(ip + 2) << 16) | (io.in(ip + 3) << 24);
        if (c != stored) return ST_INVALID;
        if (io.in(ip + 8) != 0 || (io.in(ip + 9) & 0xF0)) return ST_INVALID;
        const u64 bsize = ((u64)(io.in(ip + 4) | (io.in(ip + 5) << 8) | (io.in(ip + 6) << 16) |
                                 ((u32)io.in(ip + 7) << 24)) + 1) * 4;
        if (bsize != index_size) return ST_INVALID;
        if ((io.in(ip + 9) & 0x0F) != check_id) return ST_INVALID;
        ip += 12;
    }
    // LZMA_STREAM_END: fewer than D bytes is UnexpectedEof
    return full ? ST_OK : ST_EOF;
#undef ZX_STOP
#undef ZX_NEED
#undef ZX_SET_FULL
}

}  // namespace zx
