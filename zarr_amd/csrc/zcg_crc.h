// zcg_crc.h — CRC32 (IEEE) / CRC64 (ECMA-182, xz) helpers shared by the xz
// decoder and encoder: table-driven per-lane segment CRCs over HBM combined
// with GF(2) x^(8n) shifts (zlib's crc32_combine generalised to 64 bits).
#pragma once

#include "zcg_common.h"

namespace zcg {

constexpr u64 CRC64_POLY = 0xC96C5795D7870F42ull;  // ECMA-182, reflected (xz CRC64)
constexpr u32 CRC32_POLY = 0xEDB88320u;

struct Crc64Table {
    u64 t[256];
    constexpr Crc64Table() : t() {
        for (u32 i = 0; i < 256; i++) {
            u64 c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (CRC64_POLY & (0ull - (c & 1)));
            t[i] = c;
        }
    }
};
static __constant__ Crc64Table g_crc64 = Crc64Table();

// a*b mod P in the reflected bit order (bit 63 = x^0), zlib's multmodp.
template <typename T, T POLY>
__device__ inline T gf2_mulmod(T a, T b) {
    const int W = sizeof(T) * 8;
    T m = (T)1 << (W - 1), p = 0;
    if (a == 0) return 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (T)((b >> 1) ^ POLY) : (T)(b >> 1);
    }
    return p;
}

// x^(8*nbytes) mod P
template <typename T, T POLY>
__device__ inline T gf2_xpow8n(u64 nbytes) {
    const int W = sizeof(T) * 8;
    T r = (T)1 << (W - 1);          // x^0
    T p = (T)1 << (W - 1 - 8);      // x^8
    while (nbytes) {
        if (nbytes & 1) r = gf2_mulmod<T, POLY>(p, r);
        p = gf2_mulmod<T, POLY>(p, p);
        nbytes >>= 1;
    }
    return r;
}

// CRC of dst[a, b) by the whole wave (all lanes return the same value).
template <typename T, T POLY>
__device__ __forceinline__ T wave_crc(const u8* dst, u64 a, u64 b) {
    const int lane = lane_id();
    const u64 len = b - a;
    const u64 seg = ((len + 63) / 64 + 15) & ~15ull;
    const u64 s0 = a + (u64)lane * seg;
    const u64 s1 = (s0 + seg < b) ? s0 + seg : b;
    T c = (T)~(T)0;
    for (u64 p = s0; p < s1; p += 16) {
        if (p + 16 <= s1) {
            u32x4 v = ld16(dst + p);
            u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const u32 byte = (w[q] >> (8 * k)) & 0xFF;
                    if (sizeof(T) == 8) c = (T)(g_crc64.t[(c ^ byte) & 0xFF] ^ ((u64)c >> 8));
                    else c = (T)(g_crc32_table[(c ^ byte) & 0xFF] ^ ((u32)c >> 8));
                }
            }
        } else {
            for (u64 q = p; q < s1; q++) {
                const u32 byte = dst[q];
                if (sizeof(T) == 8) c = (T)(g_crc64.t[(c ^ byte) & 0xFF] ^ ((u64)c >> 8));
                else c = (T)(g_crc32_table[(c ^ byte) & 0xFF] ^ ((u32)c >> 8));
            }
        }
    }
    c = ~c;
    const u64 my_len = s1 > s0 ? s1 - s0 : 0;
    // combine lane CRCs in order: crc(A||B) = crc(A)*x^(8|B|) ^ crc(B)
    const T xs = gf2_xpow8n<T, POLY>(seg);
    T total = 0;  // CRC of the empty message
    for (int l = 0; l < 64; l++) {
        const T cl = (T)__shfl((u64)c, l);
        const u64 ll = __shfl(my_len, l);
        if (ll == 0) continue;
        const T sh = (ll == seg) ? xs : gf2_xpow8n<T, POLY>(ll);
        total = gf2_mulmod<T, POLY>(sh, total) ^ cl;
    }
    return total;
}



// CRC of the bytes get(p), p in [a, b), by the whole wave (all lanes return
// the same value).  `get` may apply a transform (e.g. write_data byte order).
template <typename T, T POLY, class Get>
__device__ __forceinline__ T wave_crc_fn(const Get& get, u64 a, u64 b) {
    const int lane = lane_id();
    const u64 len = b - a;
    const u64 seg = ((len + 63) / 64 + 15) & ~15ull;
    const u64 s0 = a + (u64)lane * seg;
    const u64 s1 = (s0 + seg < b) ? s0 + seg : b;
    T c = (T)~(T)0;
    for (u64 q = s0; q < s1; q++) {
        const u32 byte = get(q);
        if (sizeof(T) == 8) c = (T)(g_crc64.t[(c ^ byte) & 0xFF] ^ ((u64)c >> 8));
        else c = (T)(g_crc32_table[(c ^ byte) & 0xFF] ^ ((u32)c >> 8));
    }
    c = ~c;
    const u64 my_len = s1 > s0 ? s1 - s0 : 0;
    const T xs = gf2_xpow8n<T, POLY>(seg);
    T total = 0;
    for (int l = 0; l < 64; l++) {
        const T cl = (T)__shfl((u64)c, l);
        const u64 ll = __shfl(my_len, l);
        if (ll == 0) continue;
        const T sh = (ll == seg) ? xs : gf2_xpow8n<T, POLY>(ll);
        total = gf2_mulmod<T, POLY>(sh, total) ^ cl;
    }
    return total;
}

}  // namespace zcg
