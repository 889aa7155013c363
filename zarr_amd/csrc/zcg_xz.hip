// zcg_xz.hip — XzCompression decode (src/compression/xz.rs:34-43, xz2
// read::XzDecoder = liblzma 5.2 stream decoder) on gfx950.
//
// LZMA is one serial range-coded bit stream per chunk, so the parallelism is
// across chunks: one wave (one 64-lane workgroup) per chunk.  The decoder
// itself (zcg_xz_core.h) runs wave-uniformly — every lane computes the same
// state, which keeps control flow convergent — and the lanes fan out where
// the work is data-parallel:
//   * the probability model (7 990 u16 for lc+lp<=3; 14 134 for lc+lp=4,
//     via a second launch with the larger LDS carve) lives in LDS; every
//     lane reads/writes the same entry (LDS broadcast, no bank conflicts);
//   * decoded bytes go to an LDS history ring (4 KiB; 32 KiB with
//     ZCG_FLAG_XZ_RING_32K); a match copies all its bytes in one wave-parallel
//     step (byte k of a match at distance d is byte k mod d of the d bytes
//     before it, all already decoded), reading the ring for the last
//     ring - 512 bytes and the chunk's HBM output for far distances (older,
//     already flushed and fenced);
//   * the ring drains to HBM in 16-B-per-lane coalesced stores;
//   * the block check (CRC32/CRC64) is 64 per-lane segment CRCs over HBM,
//     combined with GF(2) x^(8n) shifts (zlib's crc32_combine, 64-bit);
//   * '>'-types / bool are transformed in place at the end (the ring keeps
//     raw bytes because far matches re-read the output).
// Algorithmic bytes per chunk: C + D.  The kernel is latency-bound on the
// serial range decoder (one dependent LDS round trip per coded bit), not HBM.
#include "zcg_common.h"
#include "zcg_crc.h"
#include "zcg_xz_core.h"

namespace zcg {

constexpr u32 XZ_RING = 4096;         // default LDS history (8 chunks per CU)
constexpr u32 XZ_RING_BIG = 32768;    // ZCG_FLAG_XZ_RING_32K (3 chunks per CU)
constexpr u32 XZ_PROBS_SMALL = 1846 + (0x300u << 3);  // lc+lp <= 3
constexpr u32 XZ_PROBS_BIG = 1846 + (0x300u << 4);    // lc+lp == 4

// Device IO of zx::xz_decode: LDS model + LDS ring + HBM output.
template <u32 XZ_RING>
struct XzDevIO {
    u64 n, D, pos;
    const gu8* __restrict__ src;
    gu8* dst;
    lu16* probs;
    lu8* ring;
    u32 nprob_cap;
    u64 gfl;  // output bytes already stored to HBM (and fenced)
    int lane;

    __device__ __forceinline__ void make_uniform() {
        n = ru64(n); D = ru64(D); pos = ru64(pos); gfl = ru64(gfl);
        src = (const gu8*)ru64((u64)src); dst = (gu8*)ru64((u64)dst);
        probs = (lu16*)(uintptr_t)__builtin_amdgcn_readfirstlane((u32)(uintptr_t)probs);
        ring = (lu8*)(uintptr_t)__builtin_amdgcn_readfirstlane((u32)(uintptr_t)ring);
        nprob_cap = __builtin_amdgcn_readfirstlane(nprob_cap);
    }
    // one input byte through the scalar cache: the aligned dword holding it
    // is loaded with s_load (constant address space), so the read never
    // crosses the buffer's last aligned dword and needs no lane broadcast
    __device__ __forceinline__ u32 in(u64 i) {
        const u64 a = (u64)(uintptr_t)(src + i);
        const u32 w = *(const __attribute__((address_space(4))) u32*)(uintptr_t)(a & ~3ull);
        return (w >> ((u32)(a & 3) * 8)) & 0xFF;
    }
    // wave-uniform values are moved to SGPRs so the decoder runs on the SALU
    __device__ __forceinline__ u32 pget(u32 i) { return __builtin_amdgcn_readfirstlane(probs[i]); }
    __device__ __forceinline__ void pset(u32 i, u32 v) { probs[i] = (u16)v; }
    __device__ __forceinline__ void init_probs(u32 count) {
        for (u32 i = lane; i < count; i += 64) probs[i] = 1024;
    }
    __device__ __forceinline__ bool lclp_ok(u32 lclp) { return zx::probs_count(lclp) <= nprob_cap; }

    // store ring bytes [gfl, e) to HBM, then fence; bytes from D on (a BCJ
    // block decoded past the caller's end, zx::xz_decode) stay in the ring
    __device__ __forceinline__ void flush(u64 e) {
        if (e > D) e = D;
        const u64 a = gfl;
        u64 a16 = (a + 15) & ~15ull;
        if (a16 > e) a16 = e;
        if ((u64)lane < a16 - a) dst[a + lane] = ring[(a + lane) & (XZ_RING - 1)];
        const u64 e16 = e & ~15ull;
        if (e16 >= a16) {
            for (u64 p = a16 + (u64)lane * 16; p < e16; p += 64 * 16)
                *(gu32x4_ua*)(dst + p) = *(const __attribute__((address_space(3))) u32x4*)(ring + (p & (XZ_RING - 1)));
            if ((u64)lane < e - e16) dst[e16 + lane] = ring[(e16 + lane) & (XZ_RING - 1)];
        }
        gfl = e;
        __threadfence_block();
    }
    // The ring keeps the last XZ_RING bytes; flushes run every XZ_RING / 2
    // bytes, so a byte is read from the ring while it is at most
    // XZ_RING - 512 back (a copy overwrites <= 273 + 64 slots ahead of its
    // sources) and from the flushed HBM output beyond that.
    __device__ __forceinline__ bool in_ring(u64 s) const { return s + (XZ_RING - 512) >= pos; }
    __device__ __forceinline__ void put(u32 b) {
        ring[pos & (XZ_RING - 1)] = (u8)b;
        pos++;
        if (pos - gfl > XZ_RING / 2) flush(pos & ~15ull);
    }
    __device__ __forceinline__ u32 back(u64 dist) {
        const u64 s = pos - 1 - dist;
        return __builtin_amdgcn_readfirstlane(in_ring(s) ? (u32)ring[s & (XZ_RING - 1)] : (u32)dst[s]);
    }
    __device__ __forceinline__ void copy(u64 d, u32 len) {
        if (pos + len - gfl > XZ_RING / 2) flush(pos & ~15ull);
        for (u32 base = 0; base < len; base += 64) {
            const u32 k = base + lane;
            if (k < len) {
                const u64 s = pos - d + ((u64)k < d ? (u64)k : (u64)k % d);
                const u8 v = in_ring(s) ? ring[s & (XZ_RING - 1)] : dst[s];
                ring[(pos + k) & (XZ_RING - 1)] = v;
            }
        }
        pos += len;
    }
    __device__ __forceinline__ void copy_in(u64 ip, u32 len) {
        while (len > 0) {
            const u32 k = len < 256 ? len : 256;
            if (pos + k - gfl > XZ_RING / 2) flush(pos & ~15ull);
            for (u32 q = lane; q < k; q += 64) ring[(pos + q) & (XZ_RING - 1)] = src[ip + q];
            pos += k;
            ip += k;
            len -= k;
        }
    }
    __device__ __forceinline__ void finish() {
        if (gfl != pos) flush(pos);
    }
    __device__ __forceinline__ void reset() {
        pos = 0;
        gfl = 0;
    }
    // output byte i >= D: in the ring (at most 32 past D, XZ_RING back)
    __device__ __forceinline__ u32 tail_byte(u64 i) const {
        return __builtin_amdgcn_readfirstlane((u32)ring[i & (XZ_RING - 1)]);
    }
    // output byte i < D in HBM (wave-uniform value; read back after finish())
    __device__ __forceinline__ void set_byte(u64 i, u32 v) { dst[i] = (u8)v; }
    // delta filter decode of dst[a, b) in place (out[i] += out[i - dist]),
    // wave-parallel: rows of `dist` bytes, 64 rows per step, one wave scan
    // per column with the column's running sum carried in LDS (the model's
    // probabilities are free between blocks and after the last one)
    __device__ void apply_delta(u64 a, u64 b, u32 dist) {
        for (u32 c = lane; c < dist; c += 64) probs[c] = 0;
        __syncthreads();
        const u64 len = b > a ? b - a : 0;
        const u64 rows = (len + dist - 1) / dist;
        for (u64 r0 = 0; r0 < rows; r0 += 64) {
            const u64 r = r0 + (u64)lane;
            for (u32 c = 0; c < dist; c++) {
                const u64 i = a + r * dist + c;
                const bool in = r < rows && i < b;
                u32 x = in ? (u32)dst[i] : 0u;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const u32 y = (u32)__shfl_up((int)x, o, 64);
                    if (lane >= o) x += y;
                }
                x += (u32)probs[c];
                if (in) dst[i] = (u8)x;
                const u32 carry = (u32)__builtin_amdgcn_readlane((int)x, 63) & 0xFF;
                __syncthreads();
                if (lane == 0) probs[c] = (u16)carry;
                __syncthreads();
            }
        }
        __threadfence_block();
    }
    // BCJ decode of out[a, b) in HBM (zx::bcj_serial's result): the word
    // filters (ARM, PowerPC, SPARC; IA-64 bundles) convert every aligned word
    // independently, one per lane; x86 and ARM-Thumb walk their candidate positions in order
    // (a wave ballot per 64 positions, the candidates handled wave-uniformly:
    // a conversion skips the instruction's bytes, so the bytes a later
    // candidate reads are never ones an earlier conversion wrote)
    struct GBuf {
        gu8* p;
        __device__ __forceinline__ u32 get(u64 i) const { return __builtin_amdgcn_readfirstlane((u32)p[i]); }
        __device__ __forceinline__ void set(u64 i, u32 v) { p[i] = (u8)v; }
    };
    struct LaneBuf {
        gu8* p;
        __device__ __forceinline__ u32 get(u64 i) const { return (u32)p[i]; }
        __device__ __forceinline__ void set(u64 i, u32 v) { p[i] = (u8)v; }
    };
    // an output byte already in HBM (after finish()), wave-uniform
    __device__ __forceinline__ u32 out_byte(u64 i) const { return __builtin_amdgcn_readfirstlane((u32)dst[i]); }
    // returns where the serial loop would have stopped, and the x86 state there
    __device__ zx::BcjState apply_bcj(u64 a, u64 b, u32 id, u32 start) {
        const u64 len = b > a ? b - a : 0;
        gu8* d = dst + a;
        zx::BcjState st{0, 0u, start - 5};
        if (id == 7 || id == 5 || id == 9) {
            st.stop = len & ~3ull;
            LaneBuf lb{d};
            for (u64 i = 4 * (u64)lane; i + 4 <= len; i += 4 * 64) zx::bcj_word(lb, i, id, start + (u32)i);
        } else if (id == 6) {
            st.stop = len & ~15ull;
            LaneBuf lb{d};
            for (u64 i = 16 * (u64)lane; i + 16 <= len; i += 16 * 64) zx::bcj_ia64_bundle(lb, i, start + (u32)i);
        } else if (id == 4 && len >= 5) {
            GBuf g{d};
            const bool allowed[8] = {true, true, true, false, true, false, false, false};
            const u32 bitnum[8] = {0, 1, 2, 2, 3, 3, 3, 3};
            u32 prev_mask = 0, prev_pos = start - 5;
            u64 next = 0;
            const u64 limit = len - 5;
            for (u64 base = 0; base <= limit; base += 64) {
                const u64 p = base + (u64)lane;
                const u32 x = p <= limit ? (u32)d[p] : 0u;
                u64 m = __ballot(p <= limit && (x == 0xE8 || x == 0xE9));
                while (m) {
                    const u64 i = base + (u64)__builtin_ctzll(m);
                    m &= m - 1;
                    if (i < next) continue;
                    const u32 now = start + (u32)i;
                    const u32 off = now - prev_pos;
                    prev_pos = now;
                    if (off > 5) prev_mask = 0;
                    else
                        for (u32 k = 0; k < off; k++) prev_mask = (prev_mask & 0x77) << 1;
                    const u32 b4 = g.get(i + 4);
                    if (zx::bcj_x86_ms(b4) && allowed[(prev_mask >> 1) & 7] && (prev_mask >> 1) < 0x10) {
                        u32 src = (b4 << 24) | (g.get(i + 3) << 16) | (g.get(i + 2) << 8) | g.get(i + 1);
                        u32 dest;
                        for (;;) {
                            dest = src - (now + 5);
                            if (prev_mask == 0) break;
                            const u32 k = bitnum[prev_mask >> 1];
                            if (!zx::bcj_x86_ms((dest >> (24 - k * 8)) & 0xFF)) break;
                            src = dest ^ ((1u << (32 - k * 8)) - 1);
                        }
                        if (lane == 0) {
                            d[i + 4] = (u8)(~(((dest >> 24) & 1) - 1));
                            d[i + 3] = (u8)(dest >> 16);
                            d[i + 2] = (u8)(dest >> 8);
                            d[i + 1] = (u8)dest;
                        }
                        __threadfence_block();
                        next = i + 5;
                        prev_mask = 0;
                    } else {
                        prev_mask |= 1;
                        if (zx::bcj_x86_ms(b4)) prev_mask |= 0x10;
                    }
                }
            }
            st.stop = len - 4 > next ? len - 4 : next;
            st.prev_mask = prev_mask;
            st.prev_pos = prev_pos;
        } else if (id == 8) {
            GBuf g{d};
            u64 next = 0;
            for (u64 base = 0; base + 4 <= len; base += 128) {
                const u64 i = base + 2 * (u64)lane;
                const bool in = i + 4 <= len;
                const u32 b1 = in ? (u32)d[i + 1] : 0u, b3 = in ? (u32)d[i + 3] : 0u;
                u64 m = __ballot(in && (b1 & 0xF8) == 0xF0 && (b3 & 0xF8) == 0xF8);
                while (m) {
                    const u64 c = base + 2 * (u64)__builtin_ctzll(m);
                    m &= m - 1;
                    if (c < next) continue;
                    const u32 c1 = g.get(c + 1), c3 = g.get(c + 3);
                    u32 src = ((c1 & 7) << 19) | (g.get(c) << 11) | ((c3 & 7) << 8) | g.get(c + 2);
                    src <<= 1;
                    const u32 dest = (src - (start + (u32)c + 4)) >> 1;
                    if (lane == 0) {
                        d[c + 1] = (u8)(0xF0 | ((dest >> 19) & 7));
                        d[c] = (u8)(dest >> 11);
                        d[c + 3] = (u8)(0xF8 | ((dest >> 8) & 7));
                        d[c + 2] = (u8)dest;
                    }
                    __threadfence_block();
                    next = c + 4;
                }
            }
            if (len >= 4) {
                const u64 e = (len - 3 + 1) & ~1ull;  // the first even position the loop cannot process
                st.stop = e > next ? e : next;
            }
        }
        __threadfence_block();
        return st;
    }
    // SHA-256 of out[a, b) (check ID 10): 256 bytes per round come in as one
    // dword per lane (big-endian words), the four blocks are compressed on
    // the scalar path from v_readlane words
    __device__ __attribute__((noinline)) void sha256(u64 a, u64 b, u32* h) {
        zx::sha256_init(h);
        u64 q = a;
        while (q + 64 <= b) {
            const u64 rem = (b - q) / 64;
            const u32 nblk = rem < 4 ? (u32)rem : 4u;
            u32 wv = 0;
            if ((u32)lane < 16 * nblk) {
                const u64 o = q + 4ull * lane;
                wv = ((u32)dst[o] << 24) | ((u32)dst[o + 1] << 16) | ((u32)dst[o + 2] << 8) | (u32)dst[o + 3];
            }
            for (u32 k = 0; k < nblk; k++) {
                u32 m[16];
#pragma unroll
                for (u32 i = 0; i < 16; i++) m[i] = __builtin_amdgcn_readlane(wv, (int)(16 * k + i));
                zx::sha256_compress(h, m);
            }
            q += 64ull * nblk;
        }
        u8 last[64];
        const u32 r = (u32)(b - q);
        for (u32 i = 0; i < r; i++) last[i] = __builtin_amdgcn_readfirstlane((u32)dst[q + i]);
        zx::sha256_tail(h, last, r, b - a);
        for (u32 i = 0; i < 8; i++) h[i] = __builtin_amdgcn_readfirstlane(h[i]);
    }
    __device__ __forceinline__ u64 check(u32 id, u64 a, u64 b) {
        if (id == 4) return wave_crc<u64, CRC64_POLY>((const u8*)dst, a, b);
        return (u64)wave_crc<u32, CRC32_POLY>((const u8*)dst, a, b);
    }
};

template <u32 NPROB, u32 XZ_RING>
__global__ __launch_bounds__(64) void xz_decode_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                       u64 D, DType t, int retry,
                                                       i32* __restrict__ status) {
    __shared__ u16 probs[NPROB];
    __shared__ __attribute__((aligned(16))) u8 ring[XZ_RING];
    const u32 c = blockIdx.x;
    if (c >= n) return;
    const int lane = lane_id();
    if (retry && __builtin_amdgcn_readfirstlane(status[c]) != zx::ST_NEED_BIG) return;
    const zcg_chunk ch = chunks[c];
    if (D > 0 && ch.dst_cap < D) {
        if (lane == 0) status[c] = ZCG_ERR_INVALID_INPUT;
        return;
    }
    XzDevIO<XZ_RING> io;
    io.n = ch.src_len;
    io.D = D;
    io.pos = 0;
    io.src = (const gu8*)ch.src;
    io.dst = (gu8*)ch.dst;
    io.probs = (lu16*)probs;
    io.ring = (lu8*)ring;
    io.nprob_cap = NPROB;
    io.gfl = 0;
    io.lane = lane;
    int st = zx::xz_decode(io);
    io.finish();
    if (st == ZCG_OK && (t.swap || t.isbool)) wave_transform((u8*)ch.dst, D, t);
    if (lane == 0) status[c] = st;
}

hipError_t launch_xz_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                            int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    (void)ws; (void)ws_bytes;
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    if (a->compression.flags & ZCG_FLAG_XZ_RING_32K) {
        hipLaunchKernelGGL((xz_decode_kernel<XZ_PROBS_SMALL, XZ_RING_BIG>), dim3(n), dim3(64), 0, s, d_chunks, n,
                           D, t, 0, d_status);
        hipLaunchKernelGGL((xz_decode_kernel<XZ_PROBS_BIG, XZ_RING_BIG>), dim3(n), dim3(64), 0, s, d_chunks, n, D,
                           t, 1, d_status);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((xz_decode_kernel<XZ_PROBS_SMALL, XZ_RING>), dim3(n), dim3(64), 0, s, d_chunks, n, D, t,
                       0, d_status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // chunks that switched to lc+lp = 4 re-run with the larger model
    hipLaunchKernelGGL((xz_decode_kernel<XZ_PROBS_BIG, XZ_RING>), dim3(n), dim3(64), 0, s, d_chunks, n, D, t,
                       1, d_status);
    return hipGetLastError();
}

uint64_t xz_decode_ws_bytes(const zcg_array* a, uint32_t n) {
    (void)a; (void)n;
    return 0;
}

}  // namespace zcg
