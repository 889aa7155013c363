// zcg_inflate_par.hip — parallel inflate of gzip chunks on gfx950
// (GzipCompression decode, src/compression/gzip.rs:49-52 -> flate2 -> zlib).
//
// A deflate block is one serial Huffman stream, so a chunk gets lane
// parallelism by SPECULATIVE, SELF-SYNCHRONISING decoding (one wave/chunk):
//
//   round: the wave stages the next ~4 KiB of the stream in LDS; lane i
//     decodes from bit R0 + i*SEG as if a symbol started there, recording
//     every token (literal, match, EOB/invalid/exhausted marker) and its
//     start bit, until it is MARGIN bits past lane i+1's start.
//   sync:  Huffman decoders resynchronise quickly: lane i's path (true from
//     its own sync point on) meets lane i+1's recorded token starts within a
//     few symbols; from that common start bit both paths are identical, so
//     lane i owns the true tokens up to it and lane i+1 from it.  Lane 0 is
//     true by construction; the valid chain ends at the first lane that
//     broke it (no sync within MARGIN, token cap, or a marker on its valid
//     range) — one ballot, no serial walk.
//   place: a wave prefix sum over the lanes' output lengths positions every
//     token; the round is cut at STAGE bytes (and at N, with zlib's look-
//     ahead semantics when N falls on a token boundary).
//   LZ77:  literals land in an LDS stage; matches resolve in rounds (each
//     lane walks its own matches in order and copies one as soon as its
//     source bytes are resolved — the earliest unresolved match is always
//     resolvable, so this terminates); sources before the round come from a
//     32 KiB LDS window ring.  Copies read B[src + k mod dist] so the reads of
//     one match never depend on its own writes.
//   commit: the stage is flushed to HBM with 16 B/lane stores (byte order /
//     bool transform fused) and appended to the window ring.
// Block headers, stored blocks and the post-N look-ahead use the wave-uniform
// reader of zcg_inflate_common.h.  Results are bit-identical to the serial
// kernel (zcg_inflate.hip), which tests/ compare it against.
#include "zcg_inflate_common.h"

namespace zcg {

constexpr u32 PI_LANES = 64;
constexpr u32 PI_SEG = 512;     // bits per lane segment
constexpr u32 PI_MARGIN = 160;  // bits past the next lane's start searched for sync
constexpr u32 PI_TMAX = 48;     // tokens recorded per lane per round
constexpr u32 PI_STAGE = 8192;  // bytes of output per round (power of 2)
constexpr u32 PI_WIN = 32768;   // LZ77 window ring
constexpr u32 PI_IN_WORDS = (PI_LANES * PI_SEG + PI_MARGIN + 4 * 64) / 32 + 8;

// token word: literal = byte value; match = 1<<31 | (len-3)<<16 | (dist-1);
// markers (bit 30): EOB, invalid code, input exhausted.
constexpr u32 T_MATCH = 0x80000000u;
constexpr u32 T_EOB = 0x40000000u;
constexpr u32 T_BAD = 0x40000001u;
constexpr u32 T_EXH = 0x40000002u;

__device__ __forceinline__ bool tok_is_marker(u32 t) { return (t & 0xC0000000u) == 0x40000000u; }
__device__ __forceinline__ u32 tok_len(u32 t) { return (t & T_MATCH) ? ((t >> 16) & 0xFF) + 3 : 1; }
__device__ __forceinline__ u32 tok_dist(u32 t) { return (t & 0x7FFF) + 1; }

struct ParLds {
    u8 win[PI_WIN];                         // LZ77 window ring (absolute pos & 32767)
    u8 stage[PI_STAGE];                     // this round's output (absolute pos & 8191)
    u32 in[PI_IN_WORDS];                    // staged stream words
    u32 tok[PI_LANES * PI_TMAX];            // tokens, lane-major
    u16 tpos[PI_LANES * PI_TMAX];           // token start bit - lane start bit
    u32 resolved[PI_STAGE / 32];            // MRR bitmap over round offsets
    u32 ltab[1u << INF_LBITS];
    u32 dtab[1u << INF_DBITS];
    HuffLds lh, dh;
    u8 lens[320];
    u32 bcache[BI_CACHE_WORDS];
    u32 ntok[PI_LANES];
    u32 endp[PI_LANES];                     // bit after the last decoded token
    i32 nstart[PI_LANES + 1];               // first valid token of lane i (set by lane i-1)
    u32 ctl[8];                             // round broadcast words
};

// 64 stream bits starting at absolute bit q (staged window starts at bit0).
__device__ __forceinline__ u64 peek64(const u32* in, u32 q, u32 bit0) {
    const u32 rel = q - bit0;
    const u32 w = rel >> 5, sh = rel & 31;
    const u64 lo = ((u64)in[w + 1] << 32) | in[w];
    u64 v = lo >> sh;
    if (sh) v |= (u64)in[w + 2] << (64 - sh);
    return v;
}

// Canonical decode of a long code from the bits of v (LSB first).
__device__ __forceinline__ u32 slow_sym(u64 v, const HuffLds* h, bool dist, u32* used) {
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; len++) {
        code |= (int)((v >> (len - 1)) & 1);
        const int cnt = h->count[len];
        if (code - cnt < first) {
            *used = len;
            return sym_entry(h->sym[index + (code - first)], len, dist);
        }
        index += cnt;
        first += cnt;
        first <<= 1;
        code <<= 1;
    }
    *used = 0;
    return mk_entry(0, K_BAD, 0, 0);
}

// Decode one token at bit q.  Returns the token word; *adv = bits consumed.
__device__ __forceinline__ u32 decode_token(const ParLds& L, u32 q, u32 bit0, u32* adv) {
    const u64 v = peek64(L.in, q, bit0);
    u32 e = L.ltab[(u32)v & ((1u << INF_LBITS) - 1)];
    u32 l = e >> 28;
    if (l == 0) {
        if (((e >> 24) & 15) == K_BAD) { *adv = 1; return T_BAD; }
        e = slow_sym(v, &L.lh, false, &l);
        if (l == 0) { *adv = 1; return T_BAD; }
    }
    const u32 kind = (e >> 24) & 15;
    if (kind == K_LIT) { *adv = l; return e & 0xFF; }
    if (kind == K_EOB) { *adv = l; return T_EOB; }
    if (kind != K_LEN) { *adv = l; return T_BAD; }
    const u32 ex = (e >> 16) & 0xFF;
    const u32 len = (e & 0xFFFF) + ((u32)(v >> l) & ((1u << ex) - 1));
    const u32 t = l + ex;
    const u64 vd = v >> t;
    u32 de = L.dtab[(u32)vd & ((1u << INF_DBITS) - 1)];
    u32 dl = de >> 28;
    if (dl == 0) {
        if (((de >> 24) & 15) == K_BAD) { *adv = t + 1; return T_BAD; }
        de = slow_sym(vd, &L.dh, true, &dl);
        if (dl == 0) { *adv = t + 1; return T_BAD; }
    }
    if (((de >> 24) & 15) != K_DIST) { *adv = t + dl; return T_BAD; }
    const u32 dex = (de >> 16) & 0xFF;
    const u32 dist = (de & 0xFFFF) + ((u32)(vd >> dl) & ((1u << dex) - 1));
    *adv = t + dl + dex;
    return T_MATCH | ((len - 3) << 16) | (dist - 1);
}

// Read the byte at absolute output position q (window ring or stage).
__device__ __forceinline__ u8 out_byte(const ParLds& L, u64 q, u64 S) {
    return q < S ? L.win[q & (PI_WIN - 1)] : L.stage[q & (PI_STAGE - 1)];
}

// Flush [from, to) of the stage to dst (transform fused); append to window.
__device__ void par_commit(ParLds& L, u8* dst, u64 from, u64 to, const DType& t) {
    const int lane = lane_id();
    __syncthreads();
    const u64 a16 = (from + 15) & ~15ull, b16 = to & ~15ull;
    if (a16 < b16) {
        for (u64 p = a16 + (u64)lane * 16; p < b16; p += 64 * 16) {
            const u32x4 v = *(const u32x4*)(L.stage + (p & (PI_STAGE - 1)));
            st16(dst + p, transform16(v, t));
            *(u32x4*)(L.win + (p & (PI_WIN - 1))) = v;
        }
    }
    // edges (and everything when the range is shorter than one group)
    const u64 e0 = a16 < b16 ? a16 : to;
    for (u64 q = from + lane; q < e0; q += 64) {
        const u8 v = L.stage[q & (PI_STAGE - 1)];
        dst[swap_pos(q, t)] = norm_byte(v, t);
        L.win[q & (PI_WIN - 1)] = v;
    }
    if (a16 < b16)
        for (u64 q = b16 + lane; q < to; q += 64) {
            const u8 v = L.stage[q & (PI_STAGE - 1)];
            dst[swap_pos(q, t)] = norm_byte(v, t);
            L.win[q & (PI_WIN - 1)] = v;
        }
    __syncthreads();
}

__device__ __forceinline__ u32 wave_excl_scan(u32 v) {
    const int lane = lane_id();
    u32 x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x - v;
}

__global__ __launch_bounds__(64) void inflate_par_kernel(const zcg_chunk* __restrict__ chunks,
                                                         u32 n, u64 D, DType t, u32 vflags,
                                                         i32* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    ParLds& L = *(ParLds*)smem_raw;
    const u32 c = blockIdx.x;
    if (c >= n) return;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    if (D == 0) { if (lane == 0) status[c] = ZCG_OK; return; }
    if (ch.dst_cap < D) { if (lane == 0) status[c] = ZCG_ERR_INVALID_INPUT; return; }
    const u8* s = (const u8*)ch.src;
    const u64 n_in = ch.src_len;
    u64 h = 0;
    int st = gzip_header(s, n_in, &h);
    if (st == ZCG_OK && n_in - h >= (1ull << 28)) st = ZCG_ERR_UNSUPPORTED;  // u32 bit positions
    if (st != ZCG_OK) { if (lane == 0) status[c] = st; return; }

    u8* dst = (u8*)ch.dst;
    const u8* ds = s + h;                  // deflate stream
    const u64 n_ds = n_in - h;
    const u32 total_bits = (u32)(n_ds * 8);
    BitIn b;
    bi_init(b, ds, n_ds, L.bcache);
    u64 P = 0;                             // output bytes produced (and committed)
    bool last = false, boundary = false, after_stored = false;
    int r = R_OK;

    while (r == R_OK && P < D) {
        if (last) { r = R_EXHAUSTED; break; }
        u32 type = 0, slen = 0;
        r = read_block_header(b, &last, &type, &slen, L.lens, &L.lh, L.ltab, &L.dh, L.dtab);
        if (r != R_OK) break;
        if (type == 0) {
            // ---- stored block: byte copies through the stage ----------------
            u64 in0 = b.consumed >> 3;  // byte aligned after LEN/NLEN
            u32 done = 0;
            while (done < slen && P < D) {
                u32 k = slen - done;
                if (k > PI_STAGE) k = PI_STAGE;
                if ((u64)k > D - P) k = (u32)(D - P);
                if (in0 + k > n_ds) { r = R_EXHAUSTED; break; }
                for (u32 i = lane; i < k; i += 64) L.stage[(P + i) & (PI_STAGE - 1)] = ds[in0 + i];
                par_commit(L, dst, P, P + k, t);
                P += k; in0 += k; done += k;
            }
            if (r != R_OK) break;
            bi_seek(b, in0 * 8);
            boundary = (done == slen);
            after_stored = true;
            continue;
        }
        after_stored = false;
        // ---- Huffman block body: speculative parallel rounds -----------------
        u32 R0 = (u32)b.consumed;
        bool block_end = false;
        while (!block_end && r == R_OK && P < D) {
            // stage the stream words of this round
            const u32 bit0 = R0 & ~31u;
            const u64 byte0 = bit0 >> 3;
            for (u32 w = lane; w < PI_IN_WORDS; w += 64) {
                const u64 q = byte0 + 4ull * w;
                u32 v = 0;
                if (q + 4 <= n_ds) v = ld32(ds + q);
                else
                    for (u32 i = 0; i < 4; i++)
                        if (q + i < n_ds) v |= (u32)ds[q + i] << (8 * i);
                L.in[w] = v;
            }
            for (u32 i = lane; i <= PI_LANES; i += 64) L.nstart[i] = 0;
            __syncthreads();

            // ---- speculative decode --------------------------------------------
            const u32 p = R0 + (u32)lane * PI_SEG;
            const u32 limit = (lane == PI_LANES - 1) ? p + PI_SEG : p + PI_SEG + PI_MARGIN;
            u32 q = p, nt = 0;
            u32* mytok = L.tok + lane * PI_TMAX;
            u16* mypos = L.tpos + lane * PI_TMAX;
            while (q < limit && nt < PI_TMAX) {
                u32 adv;
                u32 tk = decode_token(L, q, bit0, &adv);
                if (q + adv > total_bits) tk = T_EXH;
                mytok[nt] = tk;
                mypos[nt] = (u16)(q - p);
                nt++;
                if (tok_is_marker(tk)) { q += (tk == T_EOB) ? adv : 0; break; }
                q += adv;
            }
            L.ntok[lane] = nt;
            L.endp[lane] = q;
            __syncthreads();

            // ---- sync with the next lane's path --------------------------------
            i32 cut = -1;  // index of my first token owned by lane+1
            if (lane < (int)PI_LANES - 1) {
                const u32 pn = p + PI_SEG;
                const u32 nn = L.ntok[lane + 1];
                const u16* npos = L.tpos + (lane + 1) * PI_TMAX;
                u32 j = 0;
                for (u32 a = 0; a < nt; a++) {
                    const u32 pa = p + mypos[a];
                    if (pa < pn) continue;
                    while (j < nn && pn + npos[j] < pa) j++;
                    if (j >= nn) break;
                    if (pn + npos[j] == pa) { cut = (i32)a; L.nstart[lane + 1] = (i32)j; break; }
                }
            }
            __syncthreads();
            const i32 a0 = L.nstart[lane];
            // valid range [a0, bnd) and whether this lane ends the chain
            const bool last_is_marker = nt > 0 && tok_is_marker(mytok[nt - 1]);
            u32 bnd = (cut >= 0) ? (u32)cut : nt;
            bool brk = (cut < 0);
            u32 marker = 0;
            if (last_is_marker && nt - 1 < bnd) {  // marker lies on my valid range
                bnd = nt - 1;
                brk = true;
                marker = mytok[nt - 1];
            }
            const unsigned long long bm = __ballot(brk);
            const int Lb = (int)__builtin_ctzll(bm);  // lane that ends the chain (lane 63 always breaks)
            const bool active = lane <= Lb;
            // ---- output placement -------------------------------------------------
            u32 olen = 0;
            if (active)
                for (u32 a = (u32)a0; a < bnd; a++) olen += tok_len(mytok[a]);
            const u32 base = wave_excl_scan(olen);
            const u32 total = __shfl(base + olen, Lb, 64);
            const u64 room = D - P;
            const u32 cap = room < PI_STAGE ? (u32)room : PI_STAGE;
            // round end (bit position of the first token not taken) and status
            u32 round_end = __shfl(L.endp[Lb] , Lb, 64);
            u32 mk = __shfl(marker, Lb, 64);
            u32 take_lane = Lb;  // last lane whose tokens are (partly) taken
            u32 take_end = bnd;  // per-lane: tokens [a0, take_end) are emitted
            bool final_round = false, fin_boundary = false;
            if (total > cap || (total == cap && cap == room)) {
                // cut at `cap` bytes: first lane whose prefix reaches cap
                const bool over = active && (base + olen >= cap) && olen > 0;
                const unsigned long long om = __ballot(over && base < cap);
                const int cl = om ? (int)__builtin_ctzll(om) : Lb;
                take_lane = cl;
                mk = 0;
                if (lane == cl) {
                    u32 acc = base, a = (u32)a0;
                    if (cap == room) {
                        // final round: take tokens until N bytes exist
                        while (a < bnd && acc < cap) { acc += tok_len(mytok[a]); a++; }
                        L.ctl[1] = (acc == cap) ? 1u : 0u;  // exact boundary -> look-ahead
                        L.ctl[2] = a < nt ? p + mypos[a] : L.endp[lane];
                    } else {
                        while (a < bnd && acc + tok_len(mytok[a]) <= cap) { acc += tok_len(mytok[a]); a++; }
                        L.ctl[1] = 0;
                        L.ctl[2] = a < nt ? p + mypos[a] : L.endp[lane];
                    }
                    L.ctl[0] = acc;  // bytes emitted this round
                    take_end = a;
                }
                final_round = (cap == room);
                __syncthreads();
                fin_boundary = L.ctl[1] != 0;
                round_end = L.ctl[2];
                if (lane > cl) take_end = (u32)a0;  // nothing taken
            }
            const bool take = lane <= (int)take_lane;
            if (!take) take_end = (u32)a0;
            const u32 emitted = (total > cap || (total == cap && cap == room)) ? L.ctl[0] : total;
            __syncthreads();
            // ---- errors on the taken range -----------------------------------------
            if (mk == T_BAD) { r = R_INVALID; break; }
            if (mk == T_EXH) { r = R_EXHAUSTED; break; }
            // "invalid distance too far back": dist > bytes before the match
            bool far = false;
            {
                u32 o = base;
                for (u32 a = (u32)a0; a < take_end; a++) {
                    const u32 tk = mytok[a];
                    if ((tk & T_MATCH) && tok_dist(tk) > P + o) far = true;
                    o += tok_len(tk);
                }
            }
            if (__any(far)) { r = R_INVALID; break; }
            // ---- literals --------------------------------------------------------------
            const u64 S = P;
            for (u32 w = lane; w < PI_STAGE / 32; w += 64) L.resolved[w] = 0;
            __syncthreads();
            {
                u32 o = base;
                for (u32 a = (u32)a0; a < take_end; a++) {
                    const u32 tk = mytok[a];
                    if (!(tk & T_MATCH)) {
                        L.stage[(S + o) & (PI_STAGE - 1)] = (u8)tk;
                        atomicOr(&L.resolved[o >> 5], 1u << (o & 31));
                    }
                    o += tok_len(tk);
                }
            }
            __syncthreads();
            // ---- matches: multi-round resolution ---------------------------------------
            {
                u32 a = (u32)a0, o = base;
                for (;;) {
                    while (a < take_end) {
                        const u32 tk = mytok[a];
                        if (!(tk & T_MATCH)) { a++; o++; continue; }
                        const u32 len0 = tok_len(tk), d = tok_dist(tk);
                        const u32 len = (o + len0 > emitted) ? emitted - o : len0;  // cut at N
                        const int64_t src = (int64_t)o - d;  // round-relative
                        const u32 span = d < len0 ? d : len0;
                        bool ready = true;
                        if (src + (int64_t)span > 0) {
                            const u32 lo = src < 0 ? 0u : (u32)src;
                            const u32 hi = (u32)(src + span);  // exclusive, <= o
                            for (u32 x = lo; x < hi && ready;) {
                                const u32 wv = L.resolved[x >> 5];
                                const u32 nb = (hi - x) < (32 - (x & 31)) ? (hi - x) : (32 - (x & 31));
                                const u32 m = (nb == 32) ? 0xFFFFFFFFu : (((1u << nb) - 1) << (x & 31));
                                if ((wv & m) != m) ready = false;
                                x += nb;
                            }
                        }
                        if (!ready) break;
                        // out[o+k] = B[src + k mod d], reads independent of this match's writes
                        u32 ph = 0;
                        for (u32 k = 0; k < len; k += 8) {
                            u8 v[8];
#pragma unroll
                            for (int z = 0; z < 8; z++) {
                                v[z] = out_byte(L, (u64)((int64_t)S + src + ph), S);
                                ph = (ph + 1 == d) ? 0 : ph + 1;
                            }
#pragma unroll
                            for (int z = 0; z < 8; z++)
                                if (k + z < len) L.stage[(S + o + k + z) & (PI_STAGE - 1)] = v[z];
                        }
                        // mark [o, o+len) resolved
                        for (u32 x = o; x < o + len;) {
                            const u32 nb = (o + len - x) < (32 - (x & 31)) ? (o + len - x) : (32 - (x & 31));
                            const u32 m = (nb == 32) ? 0xFFFFFFFFu : (((1u << nb) - 1) << (x & 31));
                            atomicOr(&L.resolved[x >> 5], m);
                            x += nb;
                        }
                        a++;
                        o += len0;
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    if (!__any(a < take_end)) break;
                }
            }
            // ---- commit ----------------------------------------------------------------------
            par_commit(L, dst, S, S + emitted, t);
            P = S + emitted;
            if (final_round) {
                boundary = fin_boundary;
                bi_seek(b, round_end);
                break;
            }
            if (mk == T_EOB) {
                block_end = true;
                bi_seek(b, round_end);  // endp of the EOB lane: bit after EOB
            }
            R0 = round_end;
            if (P >= D) { boundary = true; bi_seek(b, R0); }
        }
    }
    if (r == R_OK && P >= D && boundary) {
        const u64 last_byte = h + (b.consumed ? (b.consumed - 1) / 8 : 0);
        u64 wend = (last_byte / 32768 + 1) * 32768;
        if (wend > n_in) wend = n_in;
        b.limit = (wend - h) * 8;
        if (b.limit >= b.consumed) {
            const int la = inf_lookahead(b, last, after_stored, L.lens, &L.lh, L.ltab, &L.dh, L.dtab);
            if (la == R_INVALID) r = R_INVALID;
        }
    }
    if (r == R_INVALID) st = ZCG_ERR_INVALID_DATA;
    else if (r == R_EXHAUSTED || P < D) st = ZCG_ERR_UNEXPECTED_EOF;
    if (lane == 0) status[c] = st;
}

size_t inflate_par_lds_bytes() { return sizeof(ParLds); }

hipError_t launch_inflate_par(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                              int32_t* d_status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    static bool attr_set = false;
    const size_t lds = sizeof(ParLds);
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)inflate_par_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(inflate_par_kernel, dim3(n), dim3(64), lds, s, d_chunks, n, D, t,
                       a->compression.flags, d_status);
    return hipGetLastError();
}

}  // namespace zcg
