// zcg_store.cpp — the FilesystemHierarchy end of the chunk path (SURVEY
// §8(f) rank 1): batched chunk-file reads into pinned staging, overlapped with
// H2D + GPU decode + D2H on two streams, and the write direction; plus the
// in-process multi-GPU entry (chunk i -> device i mod G).
//
// File semantics follow the reference store (paths relative to its root):
//   ReadableStore::get       src/store/filesystem.rs:201-210
//     open, flock(LOCK_SH) (fs2 lock_shared), read; a missing file is
//     Ok(None) -> ZCG_ABSENT (read_chunk returns None, storage.rs:226-234)
//   WriteableStore::set      src/store/filesystem.rs:260-280
//     create_dir_all(parent), open(read|write|create), flock(LOCK_EX)
//     (lock_exclusive), set_len(0) AFTER the lock, write; the lock ends
//     with the file handle.
// Chunk keys -> paths (get_chunk_key, storage.rs:109-127, and the sandboxing
// of filesystem.rs:142-190) are the caller's; this layer takes paths.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "zcg_common.h"

extern "C" {
int zcg_decode_batch(zcg_ctx* ctx, const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, int32_t* d_status,
                     void* stream);
int zcg_encode_batch(zcg_ctx* ctx, const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                     uint64_t* d_out_len, int32_t* d_status, void* stream);
uint64_t zcg_encode_bound(const zcg_compression* c, uint64_t src_len);
}
// zcg_api.cpp: the store's per-context resources
namespace zcg {
int ctx_device(zcg_ctx* ctx);
void ctx_set_error(zcg_ctx* ctx, const std::string& e);
}  // namespace zcg

namespace {

using namespace zcg;

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// run fn(i) for i in [0, count) on up to `threads` host threads
void pfor(uint32_t threads, size_t count, const std::function<void(size_t)>& fn) {
    if (count == 0) return;
    const uint32_t t = (uint32_t)std::min<size_t>(std::max<uint32_t>(threads, 1), count);
    if (t == 1) {
        for (size_t i = 0; i < count; i++) fn(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    pool.reserve(t);
    for (uint32_t k = 0; k < t; k++)
        pool.emplace_back([&] {
            for (size_t i; (i = next.fetch_add(1)) < count;) fn(i);
        });
    for (auto& th : pool) th.join();
}

// create_dir_all of the parent of `path`
bool mkdirs_parent(const std::string& path) {
    const size_t slash = path.find_last_of('/');
    if (slash == std::string::npos || slash == 0) return true;
    std::string dir = path.substr(0, slash);
    struct stat sb;
    if (stat(dir.c_str(), &sb) == 0) return S_ISDIR(sb.st_mode);
    for (size_t p = 1; p <= dir.size(); p++) {
        if (p == dir.size() || dir[p] == '/') {
            const std::string part = dir.substr(0, p);
            if (mkdir(part.c_str(), 0777) != 0 && errno != EEXIST) return false;
        }
    }
    return true;
}

// pinned host + device buffers of one pipeline slot, grown on demand
struct Slot {
    int device = 0;
    void* h_in = nullptr;
    size_t h_in_bytes = 0;
    void* h_out = nullptr;
    size_t h_out_bytes = 0;
    void* d_buf = nullptr;
    size_t d_bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool pending = false;
    ~Slot() {
        (void)hipSetDevice(device);
        if (pending && done) (void)hipEventSynchronize(done);
        if (h_in) (void)hipHostFree(h_in);
        if (h_out) (void)hipHostFree(h_out);
        if (d_buf) (void)hipFree(d_buf);
        if (done) (void)hipEventDestroy(done);
        if (stream) (void)hipStreamDestroy(stream);
    }
    hipError_t init(int dev) {
        device = dev;
        hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
        return e;
    }
    static hipError_t grow_pinned(void** p, size_t* have, size_t need) {
        if (*have >= need && *p) return hipSuccess;
        if (*p) (void)hipHostFree(*p);
        *p = nullptr;
        *have = 0;
        hipError_t e = hipHostMalloc(p, std::max<size_t>(need, 4096), hipHostMallocDefault);
        if (e == hipSuccess) *have = std::max<size_t>(need, 4096);
        return e;
    }
    hipError_t grow(size_t in, size_t out, size_t dev) {
        hipError_t e = grow_pinned(&h_in, &h_in_bytes, in);
        if (e == hipSuccess) e = grow_pinned(&h_out, &h_out_bytes, out);
        if (e == hipSuccess && (d_bytes < dev || !d_buf)) {
            if (d_buf) (void)hipFree(d_buf);
            d_buf = nullptr;
            d_bytes = 0;
            e = hipMalloc(&d_buf, std::max<size_t>(dev, 4096));
            if (e == hipSuccess) d_bytes = std::max<size_t>(dev, 4096);
        }
        return e;
    }
};

constexpr size_t STORE_BATCH_BYTES = 256ull << 20;  // decoded bytes per pipeline sub-batch
// The serial-stream codecs need many chunks in flight to fill the GPU (one
// wave per chunk): their sub-batches are 4x larger.
size_t store_batch_bytes(const zcg_array* a) {
    const int32_t c = a->compression.codec;
    return (c == ZCG_CODEC_XZ || c == ZCG_CODEC_BZIP2) ? 4 * STORE_BATCH_BYTES : STORE_BATCH_BYTES;
}

struct OpenFile {
    int fd = -1;
    uint64_t size = 0;
    int32_t st = ZCG_OK;
};

}  // namespace

struct zcg_store_slots {
    Slot s[2];
};

namespace zcg {
// per-context store slots (created on first use, owned by the context)
zcg_store_slots* ctx_store_slots(zcg_ctx* ctx);
void store_slots_free(zcg_store_slots* p) { delete p; }
zcg_store_slots* store_slots_new(int device) {
    auto* p = new zcg_store_slots();
    for (auto& s : p->s)
        if (s.init(device) != hipSuccess) {
            delete p;
            return nullptr;
        }
    return p;
}
}  // namespace zcg

extern "C" int zcg_store_read_chunks(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths,
                                     void* const* dsts, int32_t* status, uint32_t io_threads) {
    if (!ctx || !a || (n && (!paths || !dsts || !status))) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    const int dev = ctx_device(ctx);
    (void)hipSetDevice(dev);
    zcg_store_slots* S = ctx_store_slots(ctx);
    if (!S) return ZCG_ERR_RUNTIME;
    const uint64_t D = a->chunk_num_elements * (uint64_t)a->dtype.elem_size;
    const uint32_t per = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, D ? store_batch_bytes(a) / D : n));
    const uint32_t nb = (n + per - 1) / per;
    std::vector<std::vector<OpenFile>> files(2);
    std::vector<std::vector<size_t>> offs(2);
    int rc = ZCG_OK;
    auto fail = [&](hipError_t e, const char* what) {
        ctx_set_error(ctx, std::string(what) + ": " + hipGetErrorString(e));
        rc = ZCG_ERR_RUNTIME;
    };
    // copy-out of sub-batch b (after its D2H): decoded chunks -> caller buffers
    auto finish = [&](uint32_t b) {
        Slot& sl = S->s[b & 1];
        sl.pending = false;
        hipError_t e = hipEventSynchronize(sl.done);
        if (e != hipSuccess) { fail(e, "store decode"); return; }
        const uint32_t i0 = b * per, m = std::min(per, n - i0);
        const std::vector<OpenFile>& fs = files[b & 1];
        const int32_t* st = (const int32_t*)((uint8_t*)sl.h_out + (size_t)m * D);
        pfor(io_threads, m, [&](size_t k) {
            if (fs[k].st != ZCG_OK) { status[i0 + k] = fs[k].st; return; }
            status[i0 + k] = st[k];
            if (st[k] == ZCG_OK && D) memcpy(dsts[i0 + k], (uint8_t*)sl.h_out + k * D, D);
        });
    };
    for (uint32_t b = 0; b < nb && rc == ZCG_OK; b++) {
        Slot& sl = S->s[b & 1];
        if (sl.pending) finish(b - 2);  // the slot's previous sub-batch
        if (rc != ZCG_OK) break;
        const uint32_t i0 = b * per, m = std::min(per, n - i0);
        std::vector<OpenFile>& fs = files[b & 1];
        fs.assign(m, OpenFile{});
        // 1. open + shared lock + size (filesystem.rs:201-210)
        pfor(io_threads, m, [&](size_t k) {
            OpenFile& f = fs[k];
            f.fd = open(paths[i0 + k], O_RDONLY | O_CLOEXEC);
            if (f.fd < 0) { f.st = errno == ENOENT ? ZCG_ABSENT : ZCG_ERR_IO; return; }
            struct stat sb;
            if (fstat(f.fd, &sb) != 0) f.st = ZCG_ERR_IO;
            else if (!S_ISREG(sb.st_mode)) f.st = ZCG_ABSENT;  // not a file: get() -> Ok(None) (is_file())
            else if (flock(f.fd, LOCK_SH) != 0) f.st = ZCG_ERR_IO;
            if (f.st != ZCG_OK) {
                close(f.fd);
                f.fd = -1;
                return;
            }
            f.size = (uint64_t)sb.st_size;
        });
        // layout of the pinned staging: [desc m][status m][streams 256-aligned]
        std::vector<size_t>& of = offs[b & 1];
        of.assign(m, 0);
        size_t p = al256(sizeof(zcg_chunk) * m) + al256(sizeof(int32_t) * m);
        const size_t off_src = p;
        for (uint32_t k = 0; k < m; k++) {
            of[k] = p;
            p = al256(p + fs[k].size);
        }
        const size_t in_bytes = p, out_bytes = (size_t)m * D + al256(sizeof(int32_t) * m);
        hipError_t e = sl.grow(in_bytes, out_bytes, in_bytes + (size_t)m * D);
        if (e != hipSuccess) { fail(e, "store staging"); break; }
        // 2. read every file straight into pinned memory; the lock ends with close
        pfor(io_threads, m, [&](size_t k) {
            OpenFile& f = fs[k];
            if (f.fd < 0) return;
            uint8_t* d = (uint8_t*)sl.h_in + of[k];
            uint64_t got = 0;
            while (got < f.size) {
                const ssize_t r = pread(f.fd, d + got, f.size - got, (off_t)got);
                if (r <= 0) break;
                got += (uint64_t)r;
            }
            f.size = got;  // a file that shrank while read: the bytes that were there
            close(f.fd);
            f.fd = -1;
        });
        // 3. descriptors (device pointers), H2D, decode, D2H of elements + status
        uint8_t* dbase = (uint8_t*)sl.d_buf;
        zcg_chunk* hd = (zcg_chunk*)sl.h_in;
        const size_t d_out = al256(in_bytes);
        for (uint32_t k = 0; k < m; k++) {
            hd[k].src = dbase + of[k];
            hd[k].src_len = fs[k].st == ZCG_OK ? fs[k].size : 0;
            hd[k].dst = dbase + d_out + (size_t)k * D;
            hd[k].dst_cap = D;
        }
        (void)off_src;
        e = hipMemcpyAsync(dbase, sl.h_in, in_bytes, hipMemcpyHostToDevice, sl.stream);
        if (e != hipSuccess) { fail(e, "store H2D"); break; }
        int32_t* d_status = (int32_t*)(dbase + al256(sizeof(zcg_chunk) * m));
        const int r = zcg_decode_batch(ctx, a, (const zcg_chunk*)dbase, m, d_status, (void*)sl.stream);
        if (r != ZCG_OK) { rc = r; break; }
        if (D) e = hipMemcpyAsync(sl.h_out, dbase + d_out, (size_t)m * D, hipMemcpyDeviceToHost, sl.stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync((uint8_t*)sl.h_out + (size_t)m * D, d_status, sizeof(int32_t) * m,
                               hipMemcpyDeviceToHost, sl.stream);
        if (e == hipSuccess) e = hipEventRecord(sl.done, sl.stream);
        if (e != hipSuccess) { fail(e, "store D2H"); break; }
        sl.pending = true;
        // 4. copy out the previous sub-batch while this one runs on the GPU
        if (b >= 1 && S->s[(b - 1) & 1].pending) finish(b - 1);
    }
    for (uint32_t b = nb >= 2 ? nb - 2 : 0; b < nb; b++)
        if (S->s[b & 1].pending) {
            if (rc == ZCG_OK) finish(b);
            else { (void)hipEventSynchronize(S->s[b & 1].done); S->s[b & 1].pending = false; }
        }
    for (auto& fs : files)
        for (auto& f : fs)
            if (f.fd >= 0) close(f.fd);
    return rc;
}

extern "C" int zcg_store_write_chunks(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths,
                                      const void* const* elems, int32_t* status, uint32_t io_threads) {
    if (!ctx || !a || (n && (!paths || !elems || !status))) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    const int dev = ctx_device(ctx);
    (void)hipSetDevice(dev);
    zcg_store_slots* S = ctx_store_slots(ctx);
    if (!S) return ZCG_ERR_RUNTIME;
    const uint64_t D = a->chunk_num_elements * (uint64_t)a->dtype.elem_size;
    const uint64_t cap = al256(zcg_encode_bound(&a->compression, D));
    const uint32_t per = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(n, store_batch_bytes(a) / std::max<uint64_t>(D + cap, 1)));
    const uint32_t nb = (n + per - 1) / per;
    int rc = ZCG_OK;
    auto fail = [&](hipError_t e, const char* what) {
        ctx_set_error(ctx, std::string(what) + ": " + hipGetErrorString(e));
        rc = ZCG_ERR_RUNTIME;
    };
    // writes sub-batch b's encoded chunks to their files (after its D2H)
    auto finish = [&](uint32_t b) {
        Slot& sl = S->s[b & 1];
        sl.pending = false;
        hipError_t e = hipEventSynchronize(sl.done);
        if (e != hipSuccess) { fail(e, "store encode"); return; }
        const uint32_t i0 = b * per, m = std::min(per, n - i0);
        const uint8_t* ho = (const uint8_t*)sl.h_out;
        const uint64_t* lens = (const uint64_t*)(ho + (size_t)m * cap);
        const int32_t* st = (const int32_t*)(ho + (size_t)m * cap + al256(8 * m));
        pfor(io_threads, m, [&](size_t k) {
            if (st[k] != ZCG_OK) { status[i0 + k] = st[k]; return; }
            const std::string path = paths[i0 + k];
            if (!mkdirs_parent(path)) { status[i0 + k] = ZCG_ERR_IO; return; }
            const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
            if (fd < 0) { status[i0 + k] = ZCG_ERR_IO; return; }
            int32_t s2 = ZCG_OK;
            // lock, then truncate (filesystem.rs:273-276), then write
            if (flock(fd, LOCK_EX) != 0 || ftruncate(fd, 0) != 0) s2 = ZCG_ERR_IO;
            const uint8_t* d = ho + k * cap;
            uint64_t put = 0;
            while (s2 == ZCG_OK && put < lens[k]) {
                const ssize_t w = pwrite(fd, d + put, lens[k] - put, (off_t)put);
                if (w <= 0) s2 = ZCG_ERR_IO;
                else put += (uint64_t)w;
            }
            if (close(fd) != 0 && s2 == ZCG_OK) s2 = ZCG_ERR_IO;
            status[i0 + k] = s2;
        });
    };
    for (uint32_t b = 0; b < nb && rc == ZCG_OK; b++) {
        Slot& sl = S->s[b & 1];
        if (sl.pending) finish(b - 2);
        if (rc != ZCG_OK) break;
        const uint32_t i0 = b * per, m = std::min(per, n - i0);
        // device: [desc][status][out_len][elements m*D][encoded m*cap]
        const size_t o_st = al256(sizeof(zcg_chunk) * m), o_len = o_st + al256(4 * m);
        const size_t o_el = o_len + al256(8 * m), o_enc = al256(o_el + (size_t)m * D);
        const size_t out_bytes = (size_t)m * cap + al256(8 * m) + al256(4 * m);
        hipError_t e = sl.grow(o_el + (size_t)m * D, out_bytes, o_enc + (size_t)m * cap);
        if (e != hipSuccess) { fail(e, "store staging"); break; }
        uint8_t* hb = (uint8_t*)sl.h_in;
        uint8_t* db = (uint8_t*)sl.d_buf;
        zcg_chunk* hd = (zcg_chunk*)hb;
        pfor(io_threads, m, [&](size_t k) {
            if (D) memcpy(hb + o_el + k * D, elems[i0 + k], D);
            hd[k].src = db + o_el + k * D;
            hd[k].src_len = D;
            hd[k].dst = db + o_enc + k * cap;
            hd[k].dst_cap = cap;
        });
        e = hipMemcpyAsync(db, hb, o_el + (size_t)m * D, hipMemcpyHostToDevice, sl.stream);
        if (e != hipSuccess) { fail(e, "store H2D"); break; }
        const int r = zcg_encode_batch(ctx, a, (const zcg_chunk*)db, m, (uint64_t*)(db + o_len),
                                       (int32_t*)(db + o_st), (void*)sl.stream);
        if (r != ZCG_OK) { rc = r; break; }
        uint8_t* ho = (uint8_t*)sl.h_out;
        e = hipMemcpyAsync(ho, db + o_enc, (size_t)m * cap, hipMemcpyDeviceToHost, sl.stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ho + (size_t)m * cap, db + o_len, 8 * (size_t)m, hipMemcpyDeviceToHost, sl.stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ho + (size_t)m * cap + al256(8 * m), db + o_st, 4 * (size_t)m,
                               hipMemcpyDeviceToHost, sl.stream);
        if (e == hipSuccess) e = hipEventRecord(sl.done, sl.stream);
        if (e != hipSuccess) { fail(e, "store D2H"); break; }
        sl.pending = true;
        if (b >= 1 && S->s[(b - 1) & 1].pending) finish(b - 1);
    }
    for (uint32_t b = nb >= 2 ? nb - 2 : 0; b < nb; b++)
        if (S->s[b & 1].pending) {
            if (rc == ZCG_OK) finish(b);
            else { (void)hipEventSynchronize(S->s[b & 1].done); S->s[b & 1].pending = false; }
        }
    return rc;
}

// ---- multi-GPU: chunk i -> devices[i mod G], one host thread
// and one context per device, no collective, per-chunk status merged -------
extern "C" {
zcg_ctx* zcg_create(int device);
void zcg_destroy(zcg_ctx* ctx);
const char* zcg_last_error(const zcg_ctx* ctx);
int zcg_read_chunks_host(zcg_ctx* ctx, const zcg_array* array, uint32_t n, const void* const* srcs,
                         const uint64_t* src_lens, void* const* dsts, int32_t* status);
}

struct zcg_multi {
    std::vector<zcg_ctx*> ctx;
    std::string err;
};

namespace {
// run f(g, ids) on one thread per device with the ids i = g, g+G, ...
int multi_run(zcg_multi* mu, uint32_t n, const std::function<int(uint32_t, const std::vector<uint32_t>&)>& f) {
    const uint32_t G = (uint32_t)mu->ctx.size();
    std::vector<int> rcs(G, ZCG_OK);
    std::vector<std::thread> th;
    for (uint32_t g = 0; g < G; g++)
        th.emplace_back([&, g] {
            std::vector<uint32_t> ids;
            for (uint32_t i = g; i < n; i += G) ids.push_back(i);
            if (!ids.empty()) rcs[g] = f(g, ids);
        });
    for (auto& t : th) t.join();
    for (uint32_t g = 0; g < G; g++)
        if (rcs[g] != ZCG_OK) {
            mu->err = std::string("device ") + std::to_string(g) + ": " + zcg_last_error(mu->ctx[g]);
            return rcs[g];
        }
    return ZCG_OK;
}
}  // namespace

extern "C" zcg_multi* zcg_multi_create(const int* devices, uint32_t n_devices) {
    if (!devices || n_devices == 0) return nullptr;
    auto* mu = new zcg_multi();
    for (uint32_t g = 0; g < n_devices; g++) {
        zcg_ctx* c = zcg_create(devices[g]);
        if (!c) {
            for (auto* x : mu->ctx) zcg_destroy(x);
            delete mu;
            return nullptr;
        }
        mu->ctx.push_back(c);
    }
    return mu;
}

extern "C" void zcg_multi_destroy(zcg_multi* mu) {
    if (!mu) return;
    for (auto* c : mu->ctx) zcg_destroy(c);
    delete mu;
}

extern "C" const char* zcg_multi_last_error(const zcg_multi* mu) { return mu ? mu->err.c_str() : "no context"; }

extern "C" uint32_t zcg_multi_device_count(const zcg_multi* mu) { return mu ? (uint32_t)mu->ctx.size() : 0; }

extern "C" int zcg_multi_read_chunks_host(zcg_multi* mu, const zcg_array* a, uint32_t n, const void* const* srcs,
                                          const uint64_t* src_lens, void* const* dsts, int32_t* status) {
    if (!mu || !a || (n && (!srcs || !src_lens || !dsts || !status))) return ZCG_ERR_INVALID_INPUT;
    return multi_run(mu, n, [&](uint32_t g, const std::vector<uint32_t>& ids) {
        const size_t m = ids.size();
        std::vector<const void*> s(m);
        std::vector<uint64_t> l(m);
        std::vector<void*> d(m);
        std::vector<int32_t> st(m, ZCG_OK);
        for (size_t k = 0; k < m; k++) { s[k] = srcs[ids[k]]; l[k] = src_lens[ids[k]]; d[k] = dsts[ids[k]]; }
        const int r = zcg_read_chunks_host(mu->ctx[g], a, (uint32_t)m, s.data(), l.data(), d.data(), st.data());
        for (size_t k = 0; k < m; k++) status[ids[k]] = st[k];
        return r;
    });
}

extern "C" int zcg_multi_store_read_chunks(zcg_multi* mu, const zcg_array* a, uint32_t n, const char* const* paths,
                                           void* const* dsts, int32_t* status, uint32_t io_threads) {
    if (!mu || !a || (n && (!paths || !dsts || !status))) return ZCG_ERR_INVALID_INPUT;
    return multi_run(mu, n, [&](uint32_t g, const std::vector<uint32_t>& ids) {
        const size_t m = ids.size();
        std::vector<const char*> p(m);
        std::vector<void*> d(m);
        std::vector<int32_t> st(m, ZCG_OK);
        for (size_t k = 0; k < m; k++) { p[k] = paths[ids[k]]; d[k] = dsts[ids[k]]; }
        const int r = zcg_store_read_chunks(mu->ctx[g], a, (uint32_t)m, p.data(), d.data(), st.data(), io_threads);
        for (size_t k = 0; k < m; k++) status[ids[k]] = st[k];
        return r;
    });
}

extern "C" int zcg_multi_store_write_chunks(zcg_multi* mu, const zcg_array* a, uint32_t n, const char* const* paths,
                                            const void* const* elems, int32_t* status, uint32_t io_threads) {
    if (!mu || !a || (n && (!paths || !elems || !status))) return ZCG_ERR_INVALID_INPUT;
    return multi_run(mu, n, [&](uint32_t g, const std::vector<uint32_t>& ids) {
        const size_t m = ids.size();
        std::vector<const char*> p(m);
        std::vector<const void*> el(m);
        std::vector<int32_t> st(m, ZCG_OK);
        for (size_t k = 0; k < m; k++) { p[k] = paths[ids[k]]; el[k] = elems[ids[k]]; }
        const int r = zcg_store_write_chunks(mu->ctx[g], a, (uint32_t)m, p.data(), el.data(), st.data(), io_threads);
        for (size_t k = 0; k < m; k++) status[ids[k]] = st[k];
        return r;
    });
}
