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
    void make_uniform() {}
    uint32_t in(uint64_t i) const { return src[i]; }
    uint32_t pget(uint32_t i) const { return probs[i]; }
    void pset(uint32_t i, uint32_t v) { probs[i] = (uint16_t)v; }
    void init_probs(uint32_t count) { for (uint32_t i = 0; i < count; i++) probs[i] = 1024; }
    bool lclp_ok(uint32_t) const { return true; }
    void put(uint32_t b) { dst[pos++] = (uint8_t)b; }
    uint32_t back(uint64_t dist) const { return dst[pos - 1 - dist]; }
    void copy(uint64_t d, uint32_t len) {
        for (uint32_t k = 0; k < len; k++) dst[pos + k] = dst[pos + k - d];
        pos += len;
    }
    void copy_in(uint64_t ip, uint32_t len) {
        memcpy(dst + pos, src + ip, len);
        pos += len;
    }
    void finish() {}
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
