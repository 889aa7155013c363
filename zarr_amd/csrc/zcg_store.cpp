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
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
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

// Persistent fork-join pool of host I/O threads (one per context's store):
// run(t, n, fn) calls fn(i) for i in [0, n) on the caller plus t-1 workers.
// Workers are created once and reused by every phase of every call.
class IoPool {
  public:
    ~IoPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        start_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void run(uint32_t threads, size_t count, const std::function<void(size_t)>& fn) {
        if (count == 0) return;
        const uint32_t t = (uint32_t)std::min<size_t>(std::max<uint32_t>(threads, 1), count);
        if (t == 1) {
            for (size_t i = 0; i < count; i++) fn(i);
            return;
        }
        std::unique_lock<std::mutex> lk(mu_);
        while (workers_.size() < t - 1) {
            const uint32_t id = (uint32_t)workers_.size();
            workers_.emplace_back([this, id] { worker(id); });
        }
        fn_ = &fn;
        count_ = count;
        next_.store(0);
        want_ = t - 1;
        finished_ = 0;
        gen_++;
        lk.unlock();
        start_.notify_all();
        for (size_t i; (i = next_.fetch_add(1)) < count;) fn(i);
        lk.lock();
        done_.wait(lk, [&] { return finished_ == want_; });
        fn_ = nullptr;
    }

  private:
    void worker(uint32_t id) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            start_.wait(lk, [&] { return quit_ || (gen_ != seen && id < want_); });
            if (quit_) return;
            seen = gen_;
            const std::function<void(size_t)>* fn = fn_;
            const size_t count = count_;
            lk.unlock();
            for (size_t i; (i = next_.fetch_add(1)) < count;) (*fn)(i);
            lk.lock();
            if (++finished_ == want_) done_.notify_one();
        }
    }
    std::mutex mu_;
    std::condition_variable start_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t count_ = 0;
    std::atomic<size_t> next_{0};
    uint32_t want_ = 0, finished_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

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
// Chunks per read sub-batch.  Gzip, xz and bzip2 decode one chunk per wave
// (or workgroup), and a wave's time does not depend on how many run beside
// it up to 16 per CU: a sub-batch needs >= 2 048 chunks (4 096 in flight over
// the two pipeline slots) to run at the device rate, whatever D is.
uint64_t store_read_batch_chunks(const zcg_array* a, uint64_t D) {
    const int32_t c = a->compression.codec;
    uint64_t per = D ? store_batch_bytes(a) / D : ~0ull;
    if (c == ZCG_CODEC_GZIP || c == ZCG_CODEC_XZ || c == ZCG_CODEC_BZIP2) {
        const uint64_t cap = D ? (4ull << 30) / D : ~0ull;  // <= 4 GiB of decoded bytes per slot
        per = std::max<uint64_t>(per, std::min<uint64_t>(2048, cap));
    }
    return std::max<uint64_t>(per, 1);
}

// true when every pointer is page-locked host memory the GPU can copy into
bool all_pinned(void* const* p, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, p[i]) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (at.type != hipMemoryTypeHost) return false;
    }
    return true;
}

}  // namespace

struct zcg_store_slots {
    Slot s[2];
    IoPool pool;
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

namespace {

// How one store read lands its decoded chunks.
enum class Dst {
    HostStaged,  // pageable host buffers: D2H into pinned staging, copied out by the pool
    HostPinned,  // page-locked host buffers: D2H straight into them
    Device,      // device buffers: decoded in place, nothing crosses back but statuses
};

// ReadableStore::get for a batch (filesystem.rs:201-210): is_file() (stat;
// anything but a regular file -> Ok(None) -> ZCG_ABSENT), then open + shared
// flock + read under the lock, close.  The reader pool holds at most one
// descriptor per thread.  Files are read into pinned staging sized from the
// stat pass; a file that grew between stat and its locked read makes the
// sub-batch re-stage (bounded retries).
int store_read_impl(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths, void* const* dsts,
                    int32_t* status, uint32_t io_threads, bool device_dsts) {
    if (!ctx || !a || (n && (!paths || !dsts || !status))) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    const int dev = ctx_device(ctx);
    (void)hipSetDevice(dev);
    zcg_store_slots* S = ctx_store_slots(ctx);
    if (!S) return ZCG_ERR_RUNTIME;
    IoPool& pool = S->pool;
    const uint64_t D = a->chunk_num_elements * (uint64_t)a->dtype.elem_size;
    const Dst mode = device_dsts ? Dst::Device : (all_pinned(dsts, n) ? Dst::HostPinned : Dst::HostStaged);
    const uint32_t per = (uint32_t)std::min<uint64_t>(n, store_read_batch_chunks(a, D));
    const uint32_t nb = (n + per - 1) / per;
    std::vector<int32_t> fst[2];  // per sub-batch slot: file status (OK / ABSENT / IO)
    int rc = ZCG_OK;
    auto fail = [&](hipError_t e, const char* what) {
        ctx_set_error(ctx, std::string(what) + ": " + hipGetErrorString(e));
        rc = ZCG_ERR_RUNTIME;
    };
    // sub-batch b is done on the GPU: statuses (and staged chunks) -> caller
    auto finish = [&](uint32_t b) {
        Slot& sl = S->s[b & 1];
        sl.pending = false;
        hipError_t e = hipEventSynchronize(sl.done);
        if (e != hipSuccess) { fail(e, "store decode"); return; }
        const uint32_t i0 = b * per, m = std::min(per, n - i0);
        const std::vector<int32_t>& fs = fst[b & 1];
        const size_t o_st = mode == Dst::HostStaged ? (size_t)m * D : 0;
        const int32_t* st = (const int32_t*)((uint8_t*)sl.h_out + o_st);
        pool.run(io_threads, m, [&](size_t k) {
            if (fs[k] != ZCG_OK) { status[i0 + k] = fs[k]; return; }
            status[i0 + k] = st[k];
            if (mode == Dst::HostStaged && st[k] == ZCG_OK && D)
                memcpy(dsts[i0 + k], (uint8_t*)sl.h_out + k * D, D);
        });
    };
    std::vector<uint64_t> size(per), off(per);
    std::vector<uint8_t> grew(per);
    for (uint32_t b = 0; b < nb && rc == ZCG_OK; b++) {
        Slot& sl = S->s[b & 1];
        if (sl.pending) finish(b - 2);  // the slot's previous sub-batch
        if (rc != ZCG_OK) break;
        const uint32_t i0 = b * per, m = std::min(per, n - i0);
        std::vector<int32_t>& fs = fst[b & 1];
        fs.assign(m, ZCG_OK);
        size_t in_bytes = 0;
        for (int attempt = 0;; attempt++) {
            // 1. is_file() + size of every chunk file
            pool.run(io_threads, m, [&](size_t k) {
                struct stat sb;
                grew[k] = 0;
                if (stat(paths[i0 + k], &sb) != 0 || !S_ISREG(sb.st_mode)) {
                    fs[k] = ZCG_ABSENT;  // get() -> Ok(None) -> read_chunk None (storage.rs:226-234)
                    size[k] = 0;
                } else {
                    fs[k] = ZCG_OK;
                    size[k] = (uint64_t)sb.st_size;
                }
            });
            // staging layout: [desc m][status m][streams, 256-B aligned]
            size_t p = al256(sizeof(zcg_chunk) * m) + al256(sizeof(int32_t) * m);
            for (uint32_t k = 0; k < m; k++) {
                off[k] = p;
                p = al256(p + size[k]);
            }
            in_bytes = p;
            const size_t out_bytes = (mode == Dst::HostStaged ? (size_t)m * D : 0) + al256(sizeof(int32_t) * m);
            const size_t dev_bytes = al256(in_bytes) + (mode == Dst::Device ? 0 : (size_t)m * D);
            hipError_t e = sl.grow(in_bytes, out_bytes, dev_bytes);
            if (e != hipSuccess) { fail(e, "store staging"); break; }
            // 2. open + shared lock + read under the lock + close, one file per task
            std::atomic<uint32_t> n_grew{0};
            pool.run(io_threads, m, [&](size_t k) {
                if (fs[k] != ZCG_OK) return;
                const int fd = open(paths[i0 + k], O_RDONLY | O_CLOEXEC);
                if (fd < 0) { fs[k] = ZCG_ERR_IO; return; }
                struct stat sb;
                if (flock(fd, LOCK_SH) != 0 || fstat(fd, &sb) != 0) {
                    fs[k] = ZCG_ERR_IO;
                } else if ((uint64_t)sb.st_size > size[k]) {
                    grew[k] = 1;  // changed since the stat pass: re-stage this sub-batch
                    n_grew++;
                } else {
                    const uint64_t want = (uint64_t)sb.st_size;
                    uint8_t* d = (uint8_t*)sl.h_in + off[k];
                    uint64_t got = 0;
                    while (got < want) {
                        const ssize_t r = pread(fd, d + got, want - got, (off_t)got);
                        if (r < 0 && errno == EINTR) continue;
                        if (r <= 0) break;
                        got += (uint64_t)r;
                    }
                    size[k] = got;
                }
                close(fd);  // releases the lock
            });
            if (n_grew.load() == 0) break;
            if (attempt >= 4) {  // a writer keeps growing the files: report them as I/O errors
                for (uint32_t k = 0; k < m; k++)
                    if (grew[k]) fs[k] = ZCG_ERR_IO;
                break;
            }
        }
        if (rc != ZCG_OK) break;
        // 3. descriptors (device pointers), H2D, decode, D2H of statuses (+ elements)
        uint8_t* dbase = (uint8_t*)sl.d_buf;
        zcg_chunk* hd = (zcg_chunk*)sl.h_in;
        const size_t d_out = al256(in_bytes);
        for (uint32_t k = 0; k < m; k++) {
            hd[k].src = dbase + off[k];
            hd[k].src_len = fs[k] == ZCG_OK ? size[k] : 0;
            hd[k].dst = mode == Dst::Device ? dsts[i0 + k] : (void*)(dbase + d_out + (size_t)k * D);
            hd[k].dst_cap = D;
        }
        hipError_t e = hipMemcpyAsync(dbase, sl.h_in, in_bytes, hipMemcpyHostToDevice, sl.stream);
        if (e != hipSuccess) { fail(e, "store H2D"); break; }
        int32_t* d_status = (int32_t*)(dbase + al256(sizeof(zcg_chunk) * m));
        const int r = zcg_decode_batch(ctx, a, (const zcg_chunk*)dbase, m, d_status, (void*)sl.stream);
        if (r != ZCG_OK) { rc = r; break; }
        uint8_t* ho = (uint8_t*)sl.h_out;
        if (mode == Dst::HostStaged && D) {
            e = hipMemcpyAsync(ho, dbase + d_out, (size_t)m * D, hipMemcpyDeviceToHost, sl.stream);
            ho += (size_t)m * D;
        } else if (mode == Dst::HostPinned && D) {
            for (uint32_t k = 0; k < m && e == hipSuccess; k++)  // absent / unreadable: left untouched
                if (fs[k] == ZCG_OK)
                    e = hipMemcpyAsync(dsts[i0 + k], dbase + d_out + (size_t)k * D, D, hipMemcpyDeviceToHost,
                                       sl.stream);
        }
        if (e == hipSuccess)
            e = hipMemcpyAsync(ho, d_status, sizeof(int32_t) * m, hipMemcpyDeviceToHost, sl.stream);
        if (e == hipSuccess) e = hipEventRecord(sl.done, sl.stream);
        if (e != hipSuccess) { fail(e, "store D2H"); break; }
        sl.pending = true;
        // 4. finish the previous sub-batch while this one runs on the GPU
        if (b >= 1 && S->s[(b - 1) & 1].pending) finish(b - 1);
    }
    for (uint32_t b = nb >= 2 ? nb - 2 : 0; b < nb; b++)
        if (S->s[b & 1].pending) {
            if (rc == ZCG_OK) finish(b);
            else { (void)hipEventSynchronize(S->s[b & 1].done); S->s[b & 1].pending = false; }
        }
    return rc;
}

// WriteableStore::set for a batch (filesystem.rs:260-280) after a GPU encode of
// host (device_src = false) or device-resident element slots.
int store_write_impl(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths,
                     const void* const* elems, int32_t* status, uint32_t io_threads, bool device_src) {
    if (!ctx || !a || (n && (!paths || !elems || !status))) return ZCG_ERR_INVALID_INPUT;
    if (n == 0) return ZCG_OK;
    const int dev = ctx_device(ctx);
    (void)hipSetDevice(dev);
    zcg_store_slots* S = ctx_store_slots(ctx);
    if (!S) return ZCG_ERR_RUNTIME;
    IoPool& pool = S->pool;
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
        pool.run(io_threads, m, [&](size_t k) {
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
                if (w < 0 && errno == EINTR) continue;
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
        // device: [desc][status][out_len][elements m*D (host source only)][encoded m*cap]
        const size_t o_st = al256(sizeof(zcg_chunk) * m), o_len = o_st + al256(4 * m);
        const size_t o_el = o_len + al256(8 * m);
        const size_t el_bytes = device_src ? 0 : (size_t)m * D;
        const size_t o_enc = al256(o_el + el_bytes);
        const size_t out_bytes = (size_t)m * cap + al256(8 * m) + al256(4 * m);
        hipError_t e = sl.grow(o_el + el_bytes, out_bytes, o_enc + (size_t)m * cap);
        if (e != hipSuccess) { fail(e, "store staging"); break; }
        uint8_t* hb = (uint8_t*)sl.h_in;
        uint8_t* db = (uint8_t*)sl.d_buf;
        zcg_chunk* hd = (zcg_chunk*)hb;
        pool.run(io_threads, m, [&](size_t k) {
            if (!device_src && D) memcpy(hb + o_el + k * D, elems[i0 + k], D);
            hd[k].src = device_src ? elems[i0 + k] : (const void*)(db + o_el + k * D);
            hd[k].src_len = D;
            hd[k].dst = db + o_enc + k * cap;
            hd[k].dst_cap = cap;
        });
        e = hipMemcpyAsync(db, hb, o_el + el_bytes, hipMemcpyHostToDevice, sl.stream);
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

}  // namespace

extern "C" int zcg_store_read_chunks(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths,
                                     void* const* dsts, int32_t* status, uint32_t io_threads) {
    return store_read_impl(ctx, a, n, paths, dsts, status, io_threads, false);
}

extern "C" int zcg_store_read_chunks_device(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths,
                                            void* const* d_dsts, int32_t* status, uint32_t io_threads) {
    return store_read_impl(ctx, a, n, paths, d_dsts, status, io_threads, true);
}

extern "C" int zcg_store_write_chunks(zcg_ctx* ctx, const zcg_array* a, uint32_t n, const char* const* paths,
                                      const void* const* elems, int32_t* status, uint32_t io_threads) {
    return store_write_impl(ctx, a, n, paths, elems, status, io_threads, false);
}

extern "C" int zcg_store_write_chunks_device(zcg_ctx* ctx, const zcg_array* a, uint32_t n,
                                             const char* const* paths, const void* const* d_elems,
                                             int32_t* status, uint32_t io_threads) {
    return store_write_impl(ctx, a, n, paths, d_elems, status, io_threads, true);
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
