// zcg_xz_enc.h — pieces shared by the xz encoders (zcg_xz_enc.hip: the
// greedy coder of presets 0-3; zcg_xz_opt.hip: the optimal-parse coder of
// presets 4-9): the LZMA model layout, the wave-uniform range encoder with
// its lane-distributed output staging, and the serialised-input readers.
#pragma once
#include "zcg_common.h"

namespace zcg {

constexpr u32 XE_DEPTH = 16;  // hash-chain candidates per position (liblzma fast mode: 4 + nice/4)
constexpr u32 XE_NICE = 64;   // stop walking at a match this long
constexpr u32 XE_PROBS = 1846 + (0x300u << 3);  // lc + lp = 3
constexpr u32 XE_CMAX = 65536 - 64;             // compressed bytes per LZMA2 chunk (+ margin)
constexpr u32 XE_UMAX = (1u << 21) - 273;       // uncompressed bytes per LZMA2 chunk
constexpr u32 XE_LC = 3, XE_PB = 2;

// model layout (same as the decoder's)
enum : u32 {
    E_IS_MATCH = 0, E_IS_REP = 192, E_IS_REP_G0 = 204, E_IS_REP_G1 = 216, E_IS_REP_G2 = 228, E_IS_REP0_LONG = 240,
    E_POS_SLOT = 432,
    E_SPEC_POS = 688, E_ALIGN = 802, E_LEN = 818, E_REP_LEN = 1332, E_LITERAL = 1846
};
enum : u32 { EL_CHOICE = 0, EL_CHOICE2 = 1, EL_LOW = 2, EL_MID = 130, EL_HIGH = 258 };

// log2 of the dictionary of lzma_easy presets 0..9: 256K, 1M, 2M, 4M, 4M, 8M,
// 8M, 16M, 32M, 64M (the LZMA2 property is 2*(lg-12))
__device__ __forceinline__ u32 xe_dict_lg(int preset) {
    const int p = (preset < 0 || preset > 9) ? 6 : preset;
    return p == 0 ? 18u : (p == 1 ? 20u : (p == 2 ? 21u : (p <= 4 ? 22u : (p <= 6 ? 23u : (u32)(p + 17)))));
}

struct XeEnc {
    // serialised input
    const gu8* src;
    u64 n;
    DType t;
    // output
    gu8* dst;
    u64 cap, pos;
    u32 lbuf;
    bool over;
    // range coder
    u64 low;
    u32 range, cache;
    u64 cache_size;
    lu16* probs;
    int lane;

    __device__ __forceinline__ u32 sb(u64 p) const {  // serialised byte p
        return (u32)norm_byte(src[swap_pos(p, t)], t);
    }
    __device__ __forceinline__ void out(u32 b) {
        if (pos < cap) {
            if ((u32)lane == (pos & 63)) lbuf = b;
            if ((pos & 63) == 63) dst[(pos & ~63ull) + lane] = (u8)lbuf;
        } else {
            over = true;
        }
        pos++;
    }
    __device__ __forceinline__ void out_flush() {
        const u64 g = pos & ~63ull;
        const u64 e = pos < cap ? pos : cap;
        if (g + lane < e) dst[g + lane] = (u8)lbuf;
    }
    // Move the output position back to `at` (<= pos): bytes before `at` stay.
    // If `at`'s 64-byte group was already stored, reload it into the staging
    // registers (each lane reads back the byte it stored, except header bytes
    // that patch() stored from lane 0 — hence the fence).
    __device__ __forceinline__ void rewind(u64 at) {
        if ((at >> 6) != (pos >> 6)) {
            __threadfence_block();
            const u64 g = at & ~63ull;
            if (g + lane < cap) lbuf = dst[g + lane];
        }
        pos = at;
    }
    // Append `len` serialised input bytes starting at q0, 64 per step: lane j
    // of the wave takes byte (j - pos) mod 64 of the step (one rotation).
    __device__ __forceinline__ void out_run(u64 q0, u64 len) {
        for (u64 k = 0; k < len; k += 64) {
            const u32 cnt = (len - k) < 64 ? (u32)(len - k) : 64u;
            const u32 o = (u32)(pos & 63);
            const u32 v = ((u32)lane < cnt) ? sb(q0 + k + lane) : 0u;
            const u32 rot = (u32)__shfl((int)v, (lane - (int)o) & 63);
            if ((u32)lane >= o && (u32)lane < o + cnt) lbuf = rot;
            if (o + cnt >= 64) {
                const u64 g = pos & ~63ull;
                if (g + lane < cap) dst[g + lane] = (u8)lbuf;
                if ((u32)lane < o + cnt - 64) lbuf = rot;
            }
            if (pos + cnt > cap) over = true;
            pos += cnt;
        }
    }
    // byte `at` < pos, possibly still in the staging group
    __device__ __forceinline__ void patch(u64 at, u32 b) {
        if (at >= cap) return;
        if ((at >> 6) == (pos >> 6)) {
            if ((u32)lane == (at & 63)) lbuf = b;
        } else if (lane == 0) {
            dst[at] = (u8)b;
        }
    }
    __device__ __forceinline__ void rc_reset() {
        low = 0; range = 0xFFFFFFFFu; cache = 0; cache_size = 1;
    }
    __device__ __forceinline__ void shift_low() {
        if ((u32)low < 0xFF000000u || (u32)(low >> 32) != 0) {
            const u32 carry = (u32)(low >> 32);
            u32 temp = cache;
            do {
                out((temp + carry) & 0xFF);
                temp = 0xFF;
            } while (--cache_size != 0);
            cache = (u32)(low >> 24) & 0xFF;
        }
        cache_size++;
        low = (low & 0x00FFFFFFull) << 8;
    }
    __device__ __forceinline__ void bit(u32 pi, u32 b) {
        const u32 p = probs[pi];
        const u32 bound = (range >> 11) * p;
        if (b == 0) {
            range = bound;
            probs[pi] = (u16)(p + ((2048 - p) >> 5));
        } else {
            low += bound;
            range -= bound;
            probs[pi] = (u16)(p - (p >> 5));
        }
        while (range < (1u << 24)) {
            range <<= 8;
            shift_low();
        }
    }
    __device__ __forceinline__ void tree(u32 base, u32 nbits, u32 v) {
        u32 m = 1;
        for (int i = (int)nbits - 1; i >= 0; i--) {
            const u32 b = (v >> i) & 1;
            bit(base + m, b);
            m = (m << 1) | b;
        }
    }
    __device__ __forceinline__ void rtree(u32 base, u32 nbits, u32 v) {
        u32 m = 1;
        for (u32 i = 0; i < nbits; i++) {
            const u32 b = (v >> i) & 1;
            bit(base + m, b);
            m = (m << 1) | b;
        }
    }
    __device__ __forceinline__ void direct(u32 v, u32 nbits) {
        for (int i = (int)nbits - 1; i >= 0; i--) {
            range >>= 1;
            if ((v >> i) & 1) low += range;
            while (range < (1u << 24)) {
                range <<= 8;
                shift_low();
            }
        }
    }
    __device__ __forceinline__ void length(u32 lbase, u32 l, u32 ps) {  // l = len - 2
        if (l < 8) {
            bit(lbase + EL_CHOICE, 0);
            tree(lbase + EL_LOW + (ps << 3), 3, l);
        } else if (l < 16) {
            bit(lbase + EL_CHOICE, 1);
            bit(lbase + EL_CHOICE2, 0);
            tree(lbase + EL_MID + (ps << 3), 3, l - 8);
        } else {
            bit(lbase + EL_CHOICE, 1);
            bit(lbase + EL_CHOICE2, 1);
            tree(lbase + EL_HIGH, 8, l - 16);
        }
    }
    __device__ __forceinline__ void distance(u32 dist, u32 len) {
        const u32 lps = len - 2 < 3 ? len - 2 : 3;
        u32 slot;
        if (dist < 4) {
            slot = dist;
        } else {
            const u32 lg = 31 - __builtin_clz(dist);
            slot = 2 * lg + ((dist >> (lg - 1)) & 1);
        }
        tree(E_POS_SLOT + (lps << 6), 6, slot);
        if (slot >= 4) {
            const u32 nd = (slot >> 1) - 1;
            const u32 base = (2 | (slot & 1)) << nd;
            const u32 red = dist - base;
            if (slot < 14) {
                rtree(E_SPEC_POS + base - slot - 1, nd, red);
            } else {
                direct(red >> 4, nd - 4);
                rtree(E_ALIGN, 4, red & 15);
            }
        }
    }
};

// serialised bytes x..x+3 of a chunk (little-endian in the result)
typedef __attribute__((address_space(1))) u32 xe_gu32_ua __attribute__((aligned(1)));
__device__ __forceinline__ u32 xe_ser4(const u8* src, u64 x, const DType& t) {
    if (!t.swap && !t.isbool) return *(const xe_gu32_ua*)((const __attribute__((address_space(1))) u8*)src + x);  // (global, not flat)
    return (u32)norm_byte(src[swap_pos(x, t)], t) | ((u32)norm_byte(src[swap_pos(x + 1, t)], t) << 8) |
           ((u32)norm_byte(src[swap_pos(x + 2, t)], t) << 16) | ((u32)norm_byte(src[swap_pos(x + 3, t)], t) << 24);
}

__device__ __forceinline__ u32 xe_ser1(const u8* src, u64 x, const DType& t) {
    return norm_byte(src[swap_pos(x, t)], t);
}

// ---- host side ----
// presets 4-9: the optimal-parse coder (zcg_xz_opt.hip), as liblzma's
// presets 4-9 use its normal (optimal) mode; 0-3: the greedy coder
inline bool xz_uses_opt(const zcg_array* a) {
    const int p = a->compression.xz_preset;
    return (p < 0 || p > 9 ? 6 : p) >= 4;
}
// radix-sort scratch bytes for `tot` (key, position) pairs
u64 xe_sort_scratch(u64 tot);
// keys, radix sort and chain links of one match-finder sub-batch (zcg_xz_enc.hip)
hipError_t launch_xe_chains(const zcg_chunk* d_chunks, u32 c0, u64 D, u64 tot, DType t, u32 cbits, u32* ka, u32* kb,
                            u32* va, u32* vb, u32* prev, void* cub, u64 cub_bytes, hipStream_t s);
uint64_t xz_opt_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_xz_opt(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, uint64_t* d_out_len,
                         int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s);

}  // namespace zcg
