// zcg_api.cpp — C ABI of include/zchunk_gpu.h: context, dispatch by
// CompressionType (the reference's `match *self` in
// src/compression/mod.rs:72-108), workspace, and the host-memory
// conveniences that implement one DefaultChunk::read_chunk / write_chunk
// (src/chunk.rs:270-323) around the device batch kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "zcg_common.h"

using namespace zcg;

struct zcg_store_slots;

struct zcg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // internal stream of the host conveniences
    std::string err;
    // device workspace of the batch kernels, one per stream, so batches
    // enqueued on different streams of one ctx never share scratch
    // (at most WS_MAX of them: the least recently used one is freed when a
    // new stream needs one; a gzip workspace is ~100 MiB)
    struct Ws {
        void* stream;
        void* p;
        size_t bytes;
        uint64_t used;
        // the LZ4 decoder's side stream and its fork/join events, owned by
        // this (ctx, stream) pair: created on first use, never shared
        hipStream_t side = nullptr;
        hipEvent_t fork = nullptr, join = nullptr;
    };
    static constexpr size_t WS_MAX = 4;
    std::vector<Ws> ws;
    uint64_t ws_tick = 0;
    // host-convenience staging
    void* d_buf = nullptr;
    size_t d_buf_bytes = 0;
    void* h_pin = nullptr;
    size_t h_pin_bytes = 0;
    // store pipeline slots (zcg_store.cpp), created on first use
    zcg_store_slots* store = nullptr;
};

namespace zcg {
int ctx_device(zcg_ctx* ctx) { return ctx->device; }
void ctx_set_error(zcg_ctx* ctx, const std::string& e) { ctx->err = e; }
zcg_store_slots* store_slots_new(int device);
void store_slots_free(zcg_store_slots* p);
zcg_store_slots* ctx_store_slots(zcg_ctx* ctx) {
    if (!ctx->store) {
        ctx->store = store_slots_new(ctx->device);
        if (!ctx->store) ctx->err = "store: stream/event creation failed";
    }
    return ctx->store;
}
}  // namespace zcg

namespace {

int fail(zcg_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) {
        ctx->err = std::string(what) + ": " + hipGetErrorString(e);
    }
    return ZCG_ERR_RUNTIME;
}

bool dtype_ok(const zcg_dtype& d) {
    if (d.is_bool) return d.elem_size == 1;
    return d.elem_size == 1 || d.elem_size == 2 || d.elem_size == 4 || d.elem_size == 8;
}

int ensure_dev(zcg_ctx* ctx, void** p, size_t* have, size_t need) {
    if (*have >= need && *p) return ZCG_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    size_t sz = need < 4096 ? 4096 : need;
    hipError_t e = hipMalloc(p, sz);
    if (e != hipSuccess) return fail(ctx, e, "hipMalloc");
    *have = sz;
    return ZCG_OK;
}

int ensure_pin(zcg_ctx* ctx, size_t need) {
    if (ctx->h_pin_bytes >= need && ctx->h_pin) return ZCG_OK;
    if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
    ctx->h_pin = nullptr;
    ctx->h_pin_bytes = 0;
    size_t sz = need < 4096 ? 4096 : need;
    hipError_t e = hipHostMalloc(&ctx->h_pin, sz, hipHostMallocDefault);
    if (e != hipSuccess) return fail(ctx, e, "hipHostMalloc");
    ctx->h_pin_bytes = sz;
    return ZCG_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

void ws_release(zcg_ctx::Ws& w) {
    if (w.p) (void)hipFree(w.p);
    if (w.fork) (void)hipEventDestroy(w.fork);
    if (w.join) (void)hipEventDestroy(w.join);
    if (w.side) (void)hipStreamDestroy(w.side);
    w.p = nullptr;
    w.fork = w.join = nullptr;
    w.side = nullptr;
}

// the side stream + events of a workspace (nullptr side on failure: the
// caller then runs single-stream)
void ws_side(zcg_ctx::Ws* w) {
    if (w->side) return;
    hipStream_t st = nullptr;
    hipEvent_t f = nullptr, j = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
        hipEventCreateWithFlags(&f, hipEventDisableTiming) == hipSuccess &&
        hipEventCreateWithFlags(&j, hipEventDisableTiming) == hipSuccess) {
        w->side = st;
        w->fork = f;
        w->join = j;
        return;
    }
    if (j) (void)hipEventDestroy(j);
    if (f) (void)hipEventDestroy(f);
    if (st) (void)hipStreamDestroy(st);
}

// the workspace of batches enqueued on `stream`, grown to at least `need` bytes
int stream_ws(zcg_ctx* ctx, void* stream, size_t need, zcg_ctx::Ws** out) {
    zcg_ctx::Ws* w = nullptr;
    for (auto& x : ctx->ws)
        if (x.stream == stream) w = &x;
    if (!w) {
        if (ctx->ws.size() >= zcg_ctx::WS_MAX) {
            // evict the least recently used stream's workspace; that stream may
            // already be destroyed by the caller, so wait for the whole device
            size_t v = 0;
            for (size_t i = 1; i < ctx->ws.size(); i++)
                if (ctx->ws[i].used < ctx->ws[v].used) v = i;
            (void)hipDeviceSynchronize();
            ws_release(ctx->ws[v]);
            ctx->ws.erase(ctx->ws.begin() + (long)v);
        }
        ctx->ws.push_back({stream, nullptr, 0, 0});
        w = &ctx->ws.back();
    }
    w->used = ++ctx->ws_tick;
    if (w->bytes < need) (void)hipStreamSynchronize((hipStream_t)stream);  // old scratch may be in use
    const int r = ensure_dev(ctx, &w->p, &w->bytes, need);
    *out = w;
    return r;
}

}  // namespace

namespace zcg {
namespace {
std::mutex g_dev_mu;
std::map<int, uint32_t> g_dev_cus;
std::map<std::pair<const void*, int>, hipError_t> g_lds_attr;
}  // namespace

uint32_t device_cu_count() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_dev_mu);
    auto it = g_dev_cus.find(dev);
    if (it != g_dev_cus.end()) return it->second;
    int v = 0;
    const uint32_t cus =
        (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? (uint32_t)v
                                                                                                      : 256u;
    g_dev_cus[dev] = cus;
    return cus;
}

hipError_t lds_attr_once(const void* kernel, int bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_dev_mu);
    const auto key = std::make_pair(kernel, dev);
    auto it = g_lds_attr.find(key);
    if (it != g_lds_attr.end() && it->second == hipSuccess) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    g_lds_attr[key] = e;
    return e;
}
}  // namespace zcg

extern "C" {

int zcg_abi_version(void) { return ZCG_ABI_VERSION; }


const char* zcg_build_config(void) {
    static const std::string cfg = std::string(zcg::cfg_inflate_wave()) + ";" + zcg::cfg_inflate_par() + ";" +
                                   zcg::cfg_deflate() + ";" + zcg::cfg_raw() + ";" + zcg::cfg_region() + ";" +
                                   zcg::cfg_lz4_dec() + ";" + zcg::cfg_xz_opt() + ";" + zcg::cfg_bz2();
    return cfg.c_str();
}

zcg_ctx* zcg_create(int device) {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || device < 0 || device >= cnt) return nullptr;
    zcg_ctx* ctx = new zcg_ctx();
    ctx->device = device;
    (void)hipSetDevice(device);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return nullptr;
    }
    return ctx;
}

void zcg_destroy(zcg_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->store) store_slots_free(ctx->store);
    for (auto& w : ctx->ws) ws_release(w);
    if (ctx->d_buf) (void)hipFree(ctx->d_buf);
    if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* zcg_last_error(const zcg_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int32_t zcg_effective_gzip_level(int32_t level) { return (level < 0 || level > 9) ? 6 : level; }

int32_t zcg_effective_lz4_block_size(int32_t bs) {
    if (bs <= 65536) return 65536;
    if (bs <= 262144) return 262144;
    if (bs <= 1048576) return 1048576;
    return 4194304;
}

int zcg_codec_on_gpu(int32_t codec, int encode) {
    switch (codec) {
    case ZCG_CODEC_RAW: return 1;
    case ZCG_CODEC_LZ4: return 1;
    case ZCG_CODEC_GZIP: return 1;
    case ZCG_CODEC_XZ: return 1;
    case ZCG_CODEC_BZIP2: return 1;
    default: return 0;
    }
}

uint64_t zcg_encode_bound(const zcg_compression* c, uint64_t n) {
    switch (c->codec) {
    case ZCG_CODEC_RAW: return n;
    case ZCG_CODEC_GZIP:  // 16 KiB segment slots (stored worst case + sync) + header/trailer
        return 18 + ((n + 16383) / 16384) * (16384 + 128) + 64;
    case ZCG_CODEC_LZ4: {
        const uint64_t b = (uint64_t)zcg_effective_lz4_block_size(c->lz4_block_size);
        return 15 + (n / b + 1) * (b + 8) + 8;
    }
    case ZCG_CODEC_BZIP2:  // RLE1 can grow a block by 5/4; Huffman of that stays below 9/8
        return n + n / 4 + 65536;
    default: return n + n / 8 + 65536;
    }
}

// Gzip decode: the 256-lane kernel for a batch that fits one generation of
// it (3 workgroups per CU), the one-wave-per-chunk kernel above that
// (measured, 4 096 C2 chunks vs fewer: 128-512 chunks 9.2-9.8 ms vs 17-18 ms,
// 1 024 18.6 vs 18.2, 4 096 55.7 vs 31.5).
static bool inflate_par_pick(const zcg_array* a, uint32_t n) {
    const uint32_t f = a->compression.flags;
    if (f & ZCG_FLAG_INFLATE_BLOCK_PAR) return true;
    if (f & ZCG_FLAG_INFLATE_WAVE) return false;
    return n <= 3 * zcg::device_cu_count();
}

uint64_t zcg_workspace_bytes(const zcg_array* a, uint32_t n, int encode) {
    if (!a) return 0;
    if (a->compression.codec == ZCG_CODEC_BZIP2)
        return encode ? bzip2_encode_ws_bytes(a, n) : bzip2_decode_ws_bytes(a, n);
    if (a->compression.codec == ZCG_CODEC_XZ && encode) return xz_encode_ws_bytes(a, n);
    if (a->compression.codec == ZCG_CODEC_GZIP)
        return encode ? deflate_ws_bytes(a, n)
                      : ((a->compression.flags & ZCG_FLAG_SERIAL_INFLATE) ? 0
                         : inflate_par_pick(a, n) ? inflate_par_ws_bytes(a, n)
                                                                                : inflate_wave_ws_bytes(a, n));
    if (a->compression.codec == ZCG_CODEC_LZ4) return encode ? lz4_encode_ws_bytes(a, n) : lz4_decode_ws_bytes(a, n);
    return 0;
}

int zcg_decode_batch(zcg_ctx* ctx, const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                     int32_t* d_status, void* stream) {
    if (!ctx || !a || (n && (!d_chunks || !d_status))) return ZCG_ERR_INVALID_INPUT;
    if (!dtype_ok(a->dtype)) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    switch (a->compression.codec) {
    case ZCG_CODEC_RAW: e = launch_raw(a, d_chunks, n, d_status, nullptr, 0, s); break;
    case ZCG_CODEC_LZ4: {
        zcg_ctx::Ws* w = nullptr;
        const int r = stream_ws(ctx, stream, lz4_decode_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        ws_side(w);
        e = launch_lz4_decode(a, d_chunks, n, d_status, w->p, w->bytes, s, w->side, w->fork, w->join);
        break;
    }
    case ZCG_CODEC_GZIP: {
        if (a->compression.flags & ZCG_FLAG_SERIAL_INFLATE) {
            e = launch_inflate(a, d_chunks, n, d_status, s);
            break;
        }
        zcg_ctx::Ws* w = nullptr;
        if (inflate_par_pick(a, n)) {
            const int r = stream_ws(ctx, stream, inflate_par_ws_bytes(a, n), &w);
            if (r != ZCG_OK) return r;
            e = launch_inflate_par(a, d_chunks, n, d_status, w->p, w->bytes, s);
            break;
        }
        const int r = stream_ws(ctx, stream, inflate_wave_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        e = launch_inflate_wave(a, d_chunks, n, d_status, w->p, w->bytes, s);
        break;
    }
    case ZCG_CODEC_XZ: e = launch_xz_decode(a, d_chunks, n, d_status, nullptr, 0, s); break;
    case ZCG_CODEC_BZIP2: {
        zcg_ctx::Ws* w = nullptr;
        const int r = stream_ws(ctx, stream, bzip2_decode_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        e = launch_bzip2_decode(a, d_chunks, n, d_status, w->p, w->bytes, s);
        break;
    }
    default: return ZCG_ERR_INVALID_INPUT;
    }
    if (e != hipSuccess) return fail(ctx, e, "decode launch");
    return ZCG_OK;
}

int zcg_encode_batch(zcg_ctx* ctx, const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                     uint64_t* d_out_len, int32_t* d_status, void* stream) {
    if (!ctx || !a || (n && (!d_chunks || !d_status || !d_out_len))) return ZCG_ERR_INVALID_INPUT;
    if (!dtype_ok(a->dtype)) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    switch (a->compression.codec) {
    case ZCG_CODEC_RAW: e = launch_raw(a, d_chunks, n, d_status, d_out_len, 1, s); break;
    case ZCG_CODEC_LZ4: {
        // The match-finder sort key holds (chunk, block) in 12 bits: at most
        // 4096 LZ4 blocks per chunk (256 MiB chunks at the 64 KiB default).
        const uint64_t B = (uint64_t)zcg_effective_lz4_block_size(a->compression.lz4_block_size);
        const uint64_t D = a->chunk_num_elements * (uint64_t)a->dtype.elem_size;
        if ((D + B - 1) / B > 4096) {
            ctx->err = "LZ4 encode supports at most 4096 blocks per chunk (" + std::to_string((D + B - 1) / B) +
                       " requested); use a larger block size or smaller chunks";
            return ZCG_ERR_UNSUPPORTED;
        }
        zcg_ctx::Ws* w = nullptr;
        const int r = stream_ws(ctx, stream, lz4_encode_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        e = launch_lz4_encode(a, d_chunks, n, d_out_len, d_status, w->p, w->bytes, s);
        break;
    }
    case ZCG_CODEC_GZIP: {
        zcg_ctx::Ws* w = nullptr;
        const int r = stream_ws(ctx, stream, deflate_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        ws_side(w);
        e = launch_deflate(a, d_chunks, n, d_out_len, d_status, w->p, w->bytes, s, w->side, w->fork, w->join);
        break;
    }
    case ZCG_CODEC_XZ: {
        zcg_ctx::Ws* w = nullptr;
        const int r = stream_ws(ctx, stream, xz_encode_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        e = launch_xz_encode(a, d_chunks, n, d_out_len, d_status, w->p, w->bytes, s);
        break;
    }
    case ZCG_CODEC_BZIP2: {
        const int32_t lv = a->compression.bzip2_block_size;
        if (lv < 1 || lv > 9) {  // BZ2_bzCompressInit rejects it (bzip2-rs panics)
            ctx->err = "bzip2 block size must be 1..9";
            return ZCG_ERR_INVALID_INPUT;
        }
        zcg_ctx::Ws* w = nullptr;
        const int r = stream_ws(ctx, stream, bzip2_encode_ws_bytes(a, n), &w);
        if (r != ZCG_OK) return r;
        e = launch_bzip2_encode(a, d_chunks, n, d_out_len, d_status, w->p, w->bytes, s);
        break;
    }
    default:
        ctx->err = "codec has no GPU encoder in this build";
        return ZCG_ERR_UNSUPPORTED;
    }
    if (e != hipSuccess) return fail(ctx, e, "encode launch");
    return ZCG_OK;
}

int zcg_read_chunks_host(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const void* const* srcs,
                         const uint64_t* src_lens, void* const* dsts, int32_t* status) {
    if (!ctx || !a) return ZCG_ERR_INVALID_INPUT;
    if (!dtype_ok(a->dtype)) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    (void)hipSetDevice(ctx->device);
    const uint64_t D = a->chunk_num_elements * (uint64_t)a->dtype.elem_size;
    // device layout: [desc n][status n][src blobs (256-aligned)][dst n*D]
    size_t off_desc = 0;
    size_t off_stat = align_up(off_desc + sizeof(zcg_chunk) * n, 256);
    size_t off_src = align_up(off_stat + sizeof(int32_t) * n, 256);
    std::vector<size_t> so(n);
    size_t p = off_src;
    for (uint32_t i = 0; i < n; i++) { so[i] = p; p = align_up(p + src_lens[i], 256); }
    size_t off_dst = p;
    size_t total = align_up(off_dst + (size_t)D * n, 256);
    int r = ensure_dev(ctx, &ctx->d_buf, &ctx->d_buf_bytes, total);
    if (r) return r;
    r = ensure_pin(ctx, total);
    if (r) return r;
    uint8_t* hp = (uint8_t*)ctx->h_pin;
    uint8_t* dp = (uint8_t*)ctx->d_buf;
    zcg_chunk* hd = (zcg_chunk*)(hp + off_desc);
    for (uint32_t i = 0; i < n; i++) {
        memcpy(hp + so[i], srcs[i], src_lens[i]);
        hd[i].src = dp + so[i];
        hd[i].src_len = src_lens[i];
        hd[i].dst = dp + off_dst + (size_t)D * i;
        hd[i].dst_cap = D;
    }
    hipError_t e = hipMemcpyAsync(dp, hp, off_dst, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return fail(ctx, e, "H2D");
    r = zcg_decode_batch(ctx, a, (const zcg_chunk*)(dp + off_desc), n, (int32_t*)(dp + off_stat),
                         ctx->stream);
    if (r) return r;
    e = hipMemcpyAsync(hp + off_stat, dp + off_stat, sizeof(int32_t) * n, hipMemcpyDeviceToHost,
                       ctx->stream);
    if (e == hipSuccess && D)
        e = hipMemcpyAsync(hp + off_dst, dp + off_dst, (size_t)D * n, hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return fail(ctx, e, "D2H");
    const int32_t* hs = (const int32_t*)(hp + off_stat);
    for (uint32_t i = 0; i < n; i++) {
        status[i] = hs[i];
        if (hs[i] == ZCG_OK && D) memcpy(dsts[i], hp + off_dst + (size_t)D * i, D);
    }
    return ZCG_OK;
}

int zcg_read_chunk(zcg_ctx* ctx, const zcg_array* a, const void* src, uint64_t src_len,
                   void* dst) {
    int32_t st = ZCG_OK;
    void* const dsts[1] = {dst};
    const void* const srcs[1] = {src};
    int r = zcg_read_chunks_host(ctx, a, 1, srcs, &src_len, dsts, &st);
    return r ? r : st;
}

int zcg_write_chunk(zcg_ctx* ctx, const zcg_array* a, const void* elems, uint64_t n_elements,
                    void* out, uint64_t out_cap, uint64_t* out_len) {
    if (!ctx || !a || !out_len) return ZCG_ERR_INVALID_INPUT;
    *out_len = 0;
    if (!dtype_ok(a->dtype)) return ZCG_ERR_INVALID_INPUT;
    if (n_elements != a->chunk_num_elements) return ZCG_ERR_INVALID_DATA;  // chunk.rs:309-318
    if (!zcg_codec_on_gpu(a->compression.codec, 1)) {
        ctx->err = "codec has no GPU encoder in this build";
        return ZCG_ERR_UNSUPPORTED;
    }
    (void)hipSetDevice(ctx->device);
    const uint64_t nb = n_elements * (uint64_t)a->dtype.elem_size;
    const uint64_t cap = zcg_encode_bound(&a->compression, nb);
    // device layout: [desc][status][out_len][src nb][dst cap]
    size_t off_stat = 256, off_len = 512, off_src = 1024;
    size_t off_dst = align_up(off_src + nb, 256);
    size_t total = align_up(off_dst + cap, 256);
    int r = ensure_dev(ctx, &ctx->d_buf, &ctx->d_buf_bytes, total);
    if (r) return r;
    r = ensure_pin(ctx, total);
    if (r) return r;
    uint8_t* hp = (uint8_t*)ctx->h_pin;
    uint8_t* dp = (uint8_t*)ctx->d_buf;
    zcg_chunk* hd = (zcg_chunk*)hp;
    hd->src = dp + off_src;
    hd->src_len = nb;
    hd->dst = dp + off_dst;
    hd->dst_cap = cap;
    memcpy(hp + off_src, elems, nb);
    hipError_t e = hipMemcpyAsync(dp, hp, off_dst, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return fail(ctx, e, "H2D");
    r = zcg_encode_batch(ctx, a, (const zcg_chunk*)dp, 1, (uint64_t*)(dp + off_len),
                         (int32_t*)(dp + off_stat), ctx->stream);
    if (r) return r;
    e = hipMemcpyAsync(hp + off_stat, dp + off_stat, off_src - off_stat, hipMemcpyDeviceToHost,
                       ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return fail(ctx, e, "D2H");
    const int32_t st = *(int32_t*)(hp + off_stat);
    const uint64_t len = *(uint64_t*)(hp + off_len);
    if (st != ZCG_OK) return st;
    if (len > out_cap) return ZCG_ERR_OUTPUT_TOO_SMALL;
    e = hipMemcpy(out, dp + off_dst, len, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(ctx, e, "D2H");
    *out_len = len;
    return ZCG_OK;
}

uint64_t zcg_region_grid(const zcg_region* r, uint64_t* grid_lo, uint64_t* grid_n) {
    if (!r || r->ndim < 1 || r->ndim > ZCG_MAX_DIMS) return 0;
    uint64_t cnt = 1;
    for (uint32_t d = 0; d < r->ndim; d++) {
        const uint64_t cs = r->chunk_shape[d] ? r->chunk_shape[d] : 1;
        // bounded_coord_iter (ndarray.rs:410-432): bbox intersected with the
        // array bounds (BoundingBox::intersect, saturating), floor/ceil by chunk
        const uint64_t o = r->bbox_offset[d];
        const uint64_t e = std::min(r->bbox_offset[d] + r->bbox_shape[d], r->array_shape[d]);
        const uint64_t s = e > o ? e - o : 0;
        const uint64_t lo = o / cs, hi = (o + s + cs - 1) / cs;
        if (grid_lo) grid_lo[d] = lo;
        if (grid_n) grid_n[d] = hi - lo;
        cnt *= hi - lo;
    }
    return cnt;
}

static int region_call(zcg_ctx* ctx, const zcg_region* r, const void* const* d_chunk_table, void* d_box,
                       void* stream, uint32_t dir);

int zcg_read_region(zcg_ctx* ctx, const zcg_region* r, const void* const* d_chunk_table, void* d_out,
                    void* stream) {
    return region_call(ctx, r, d_chunk_table, d_out, stream, 0);
}

int zcg_write_region(zcg_ctx* ctx, const zcg_region* r, void* const* d_chunk_table, const void* d_in,
                     void* stream) {
    return region_call(ctx, r, (const void* const*)d_chunk_table, (void*)d_in, stream, 1);
}

static int region_call(zcg_ctx* ctx, const zcg_region* r, const void* const* d_chunk_table, void* d_out,
                       void* stream, uint32_t dir) {
    if (!ctx || !r || r->ndim < 1 || r->ndim > ZCG_MAX_DIMS) return ZCG_ERR_INVALID_INPUT;
    const uint32_t es = r->elem_size;
    if (es != 1 && es != 2 && es != 4 && es != 8) return ZCG_ERR_INVALID_INPUT;
    const uint32_t nd = r->ndim;
    uint64_t lo[ZCG_MAX_DIMS], gn[ZCG_MAX_DIMS];
    const uint64_t nchunks = zcg_region_grid(r, lo, gn);
    RegionArgs a{};
    a.nd = nd;
    a.es = es;
    a.fill = (r->fill_missing && !dir) ? 1u : 0u;
    a.dir = dir;
    a.V = 16 / es;
    a.fillv = r->fill_value;
    uint64_t tstr_arr[ZCG_MAX_DIMS];
    {
        uint64_t st = 1;
        for (int d = (int)nd - 1; d >= 0; d--) { tstr_arr[d] = st; st *= gn[d]; }
    }
    uint64_t total = 1, cst = 1;
    for (uint32_t k = 0; k < nd; k++) {
        const uint32_t d = r->chunk_order == 1 ? k : nd - 1 - k;  // fast-first
        const uint64_t cs = r->chunk_shape[d], bs = r->bbox_shape[d];
        if (cs == 0 || cs >= (1ull << 32)) return ZCG_ERR_INVALID_INPUT;
        const uint64_t orr = r->bbox_offset[d] % cs;
        if (bs + orr >= (1ull << 32)) {
            ctx->err = "region: box extent along a dimension must stay below 2^32 elements";
            return ZCG_ERR_UNSUPPORTED;
        }
        a.bs[k] = (uint32_t)bs;
        a.orr[k] = (uint32_t)orr;
        a.cs[k] = (uint32_t)cs;
        a.ob[k] = lo[d];
        a.gn[k] = gn[d];
        a.tstr[k] = tstr_arr[d];
        a.cstr[k] = cst;
        a.ostr[k] = r->out_strides[d];
        cst *= cs;
        total *= bs;
    }
    a.total = total;
    if (total == 0) return ZCG_OK;
    if (!d_out || (nchunks && !d_chunk_table)) return ZCG_ERR_INVALID_INPUT;
    (void)hipSetDevice(ctx->device);
    const hipError_t e = launch_region(a, d_chunk_table, d_out, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ctx, e, "region launch");
    return ZCG_OK;
}

}  // extern "C"
