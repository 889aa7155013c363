// zcg_meta.cpp — Zarr v3.0-dev array metadata JSON -> zcg_array (C ABI
// zcg_array_meta_from_json), so a C or Rust caller can drive the batch API
// from a real hierarchy without building descriptors by hand.
//
// Restates the reference's serde rules (paths relative to the reference root):
//   ArrayMetadata fields                          src/lib.rs:382-402
//     shape, data_type, chunk_grid {type, chunk_shape, separator},
//     chunk_memory_layout ("C" | "F"), extensions, attributes are required;
//     fill_value is optional (null / absent -> None); compressor defaults to
//     Raw (#[serde(default)]).
//   must_understand extensions -> UnknownRequiredExtension  src/storage.rs:172-176
//   DataType strings "bool", "i1", "u1", "[<>][iuf][1248]", "rN"   src/data_type.rs:165-240
//   ExtensibleDataType {extension, type, fallback} + effective_type
//                                                  src/data_type.rs:282-310
//   CompressionType {"codec", "configuration"} with per-codec defaults
//     gzip level -1, lz4 blockSize 65536, bzip2 blockSize 9, xz preset 6
//                                                  src/compression/{mod,gzip,lz,bzip,xz}.rs
//   get_chunk_num_elements                         src/lib.rs:474-480
//   get_effective_fill_value (fill value as T, else T::default())  src/lib.rs:448-454
// A malformed document is ZCG_ERR_INVALID_DATA (serde -> io::ErrorKind::InvalidData);
// the reference's panics (an unknown endian or size character, an extended
// type without fallback: `todo!()`) and must-understand extensions are
// ZCG_ERR_UNSUPPORTED here.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/zchunk_gpu.h"

namespace {

struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0;
    bool is_int = false;   // the number token had no fraction/exponent
    bool neg = false;
    uint64_t mag = 0;      // |integer| when is_int (saturating)
    std::string s;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;
    const JVal* get(const char* k) const {
        for (auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct Parser {
    const char* p;
    const char* e;
    std::string err;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    bool fail(const char* m) {
        if (err.empty()) err = m;
        return false;
    }
    bool lit(const char* w) {
        const size_t n = strlen(w);
        if ((size_t)(e - p) < n || memcmp(p, w, n) != 0) return false;
        p += n;
        return true;
    }
    static void utf8(std::string& o, uint32_t c) {
        if (c < 0x80) o += (char)c;
        else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 63)); }
        else if (c < 0x10000) {
            o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63));
        } else {
            o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 63));
            o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63));
        }
    }
    bool hex4(uint32_t& v) {
        if (e - p < 4) return false;
        v = 0;
        for (int i = 0; i < 4; i++) {
            const char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return false;
        }
        return true;
    }
    bool str(std::string& o) {
        if (p >= e || *p != '"') return fail("expected a string");
        p++;
        while (p < e && *p != '"') {
            const unsigned char c = (unsigned char)*p++;
            if (c < 0x20) return fail("control character in a string");
            if (c != '\\') { o += (char)c; continue; }
            if (p >= e) return fail("truncated escape");
            const char x = *p++;
            switch (x) {
            case '"': o += '"'; break;
            case '\\': o += '\\'; break;
            case '/': o += '/'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'n': o += '\n'; break;
            case 'r': o += '\r'; break;
            case 't': o += '\t'; break;
            case 'u': {
                uint32_t c1;
                if (!hex4(c1)) return fail("bad \\u escape");
                if (c1 >= 0xD800 && c1 < 0xDC00) {
                    uint32_t c2;
                    if (!lit("\\u") || !hex4(c2) || c2 < 0xDC00 || c2 > 0xDFFF) return fail("bad surrogate pair");
                    c1 = 0x10000 + ((c1 - 0xD800) << 10) + (c2 - 0xDC00);
                } else if (c1 >= 0xDC00 && c1 <= 0xDFFF) {
                    return fail("lone surrogate");
                }
                utf8(o, c1);
                break;
            }
            default: return fail("bad escape");
            }
        }
        if (p >= e) return fail("unterminated string");
        p++;
        return true;
    }
    bool number(JVal& v) {
        const char* s0 = p;
        v.kind = JVal::NUM;
        if (p < e && *p == '-') { v.neg = true; p++; }
        if (p >= e || !(*p >= '0' && *p <= '9')) return fail("bad number");
        if (*p == '0' && p + 1 < e && p[1] >= '0' && p[1] <= '9') return fail("leading zero");
        v.is_int = true;
        uint64_t m = 0;
        bool sat = false;
        while (p < e && *p >= '0' && *p <= '9') {
            const uint64_t d = (uint64_t)(*p - '0');
            if (m > (UINT64_MAX - d) / 10) sat = true;
            else m = m * 10 + d;
            p++;
        }
        if (p < e && *p == '.') {
            v.is_int = false;
            p++;
            if (p >= e || !(*p >= '0' && *p <= '9')) return fail("bad fraction");
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            v.is_int = false;
            p++;
            if (p < e && (*p == '+' || *p == '-')) p++;
            if (p >= e || !(*p >= '0' && *p <= '9')) return fail("bad exponent");
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        v.mag = sat ? UINT64_MAX : m;
        if (sat) v.is_int = false;
        v.num = strtod(std::string(s0, p).c_str(), nullptr);
        return true;
    }
    bool value(JVal& v, int depth) {
        if (depth > 64) return fail("nesting too deep");
        ws();
        if (p >= e) return fail("unexpected end");
        const char c = *p;
        if (c == '{') {
            p++;
            v.kind = JVal::OBJ;
            ws();
            if (p < e && *p == '}') { p++; return true; }
            for (;;) {
                ws();
                std::string k;
                if (!str(k)) return false;
                ws();
                if (p >= e || *p != ':') return fail("expected ':'");
                p++;
                JVal x;
                if (!value(x, depth + 1)) return false;
                v.obj.emplace_back(std::move(k), std::move(x));
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == '}') { p++; return true; }
                return fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            p++;
            v.kind = JVal::ARR;
            ws();
            if (p < e && *p == ']') { p++; return true; }
            for (;;) {
                JVal x;
                if (!value(x, depth + 1)) return false;
                v.arr.push_back(std::move(x));
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == ']') { p++; return true; }
                return fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.kind = JVal::STR; return str(v.s); }
        if (lit("true")) { v.kind = JVal::BOOL; v.b = true; return true; }
        if (lit("false")) { v.kind = JVal::BOOL; v.b = false; return true; }
        if (lit("null")) { v.kind = JVal::NUL; return true; }
        return number(v);
    }
};

// DataType (data_type.rs:116-123) as (kind, size, big endian)
enum DtKind { DT_BOOL, DT_INT, DT_UINT, DT_FLOAT, DT_RAW };
struct Dt {
    DtKind kind;
    uint32_t size;  // bytes
    bool big;
};

// DataTypeVisitor::visit_str (data_type.rs:165-240); returns 0, or a status
int parse_dtype(const std::string& s, Dt& d, std::string& err) {
    if (s == "bool") { d = {DT_BOOL, 1, false}; return ZCG_OK; }
    if (s == "i1") { d = {DT_INT, 1, false}; return ZCG_OK; }
    if (s == "u1") { d = {DT_UINT, 1, false}; return ZCG_OK; }
    if (!s.empty() && s[0] == 'r') {
        const std::string n = s.substr(1);
        if (n.empty() || n.size() > 18 || n.find_first_not_of("0123456789") != std::string::npos) {
            err = "invalid data type " + s;
            return ZCG_ERR_INVALID_DATA;
        }
        const unsigned long long bits = strtoull(n.c_str(), nullptr, 10);
        if (bits % 8) { err = "invalid data type " + s; return ZCG_ERR_INVALID_DATA; }
        d = {DT_RAW, (uint32_t)(bits / 8), false};
        return ZCG_OK;
    }
    if (s.size() == 3) {
        // the reference panics (`expect("TODO")` / `unwrap()`) on an unknown
        // endian or size character
        bool big;
        if (s[0] == '>') big = true;
        else if (s[0] == '<') big = false;
        else { err = "unknown endianness in " + s + " (the reference panics)"; return ZCG_ERR_UNSUPPORTED; }
        const char k = s[1], z = s[2];
        const bool isz = z == '1' || z == '2' || z == '4' || z == '8';
        const bool fsz = z == '2' || z == '4' || z == '8';
        if (k == 'i' || k == 'u') {
            if (!isz) { err = "unknown size in " + s + " (the reference panics)"; return ZCG_ERR_UNSUPPORTED; }
            d = {k == 'i' ? DT_INT : DT_UINT, (uint32_t)(z - '0'), big};
            return ZCG_OK;
        }
        if (k == 'f') {
            if (!fsz) { err = "unknown size in " + s + " (the reference panics)"; return ZCG_ERR_UNSUPPORTED; }
            d = {DT_FLOAT, (uint32_t)(z - '0'), big};
            return ZCG_OK;
        }
    }
    err = "invalid data type " + s;
    return ZCG_ERR_INVALID_DATA;
}

uint16_t f32_to_f16(float f) {  // round to nearest even (half's from_f32)
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ex = (x >> 23) & 0xFF;
    uint32_t man = x & 0x7FFFFFu;
    if (ex == 0xFF) return (uint16_t)(sign | 0x7C00u | (man ? (0x200u | (man >> 13)) : 0));
    const int e = (int)ex - 127 + 15;
    if (e >= 0x1F) return (uint16_t)(sign | 0x7C00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) h++;
    return (uint16_t)(sign | h);
}

// get_effective_fill_value (lib.rs:448-454): serde_json::from_value::<T>
int fill_bits(const JVal& v, const Dt& d, uint64_t& out, std::string& err) {
    out = 0;
    if (d.kind == DT_BOOL) {
        if (v.kind != JVal::BOOL) { err = "fill_value is not a bool"; return ZCG_ERR_INVALID_DATA; }
        out = v.b ? 1 : 0;
        return ZCG_OK;
    }
    if (v.kind != JVal::NUM) { err = "fill_value is not a number"; return ZCG_ERR_INVALID_DATA; }
    if (d.kind == DT_FLOAT) {
        if (d.size == 8) { memcpy(&out, &v.num, 8); return ZCG_OK; }
        const float f = (float)v.num;
        if (d.size == 4) { uint32_t u; memcpy(&u, &f, 4); out = u; return ZCG_OK; }
        out = f32_to_f16(f);
        return ZCG_OK;
    }
    if (d.kind == DT_INT || d.kind == DT_UINT) {
        if (!v.is_int) { err = "fill_value is not an integer"; return ZCG_ERR_INVALID_DATA; }
        const unsigned bits = 8 * d.size;
        if (d.kind == DT_UINT) {
            if (v.neg && v.mag) { err = "fill_value out of range"; return ZCG_ERR_INVALID_DATA; }
            if (bits < 64 && v.mag >> bits) { err = "fill_value out of range"; return ZCG_ERR_INVALID_DATA; }
            out = v.mag;
        } else {
            const uint64_t lim = bits == 64 ? (uint64_t)1 << 63 : (uint64_t)1 << (bits - 1);
            if (v.neg ? v.mag > lim : v.mag >= lim) { err = "fill_value out of range"; return ZCG_ERR_INVALID_DATA; }
            out = v.neg ? (uint64_t)(-(int64_t)(v.mag - 1) - 1) : v.mag;
            if (bits < 64) out &= (((uint64_t)1 << bits) - 1);
        }
        return ZCG_OK;
    }
    err = "raw data types have no fill value";
    return ZCG_ERR_UNSUPPORTED;
}

int64_t cfg_int(const JVal* conf, const char* key, int64_t def, bool& bad) {
    if (!conf) return def;
    const JVal* x = conf->get(key);
    if (!x) return def;
    if (x->kind != JVal::NUM || !x->is_int) { bad = true; return def; }
    // the configuration fields are i32 in the reference (serde rejects a value
    // outside the type's range with InvalidData)
    if (x->neg ? x->mag > 0x80000000ull : x->mag > 0x7FFFFFFFull) { bad = true; return def; }
    return x->neg ? -(int64_t)x->mag : (int64_t)x->mag;
}

int parse_meta(const char* json, uint64_t len, zcg_array_meta* out, std::string& err) {
    Parser P{json, json + len, {}};
    JVal root;
    if (!P.value(root, 0)) { err = "JSON: " + P.err; return ZCG_ERR_INVALID_DATA; }
    P.ws();
    if (P.p != P.e) { err = "JSON: trailing characters"; return ZCG_ERR_INVALID_DATA; }
    if (root.kind != JVal::OBJ) { err = "array metadata is not an object"; return ZCG_ERR_INVALID_DATA; }
    memset(out, 0, sizeof *out);
    // required fields (no #[serde(default)] in lib.rs:382-402)
    const char* req[] = {"shape", "data_type", "chunk_grid", "chunk_memory_layout", "extensions", "attributes"};
    for (const char* k : req)
        if (!root.get(k)) { err = std::string("missing field `") + k + "`"; return ZCG_ERR_INVALID_DATA; }
    const JVal& shape = *root.get("shape");
    if (shape.kind != JVal::ARR) { err = "shape is not an array"; return ZCG_ERR_INVALID_DATA; }
    const JVal& grid = *root.get("chunk_grid");
    if (grid.kind != JVal::OBJ || !grid.get("type") || !grid.get("chunk_shape") || !grid.get("separator")) {
        err = "chunk_grid needs type, chunk_shape and separator";
        return ZCG_ERR_INVALID_DATA;
    }
    const JVal& gt = *grid.get("type");
    const JVal& cshape = *grid.get("chunk_shape");
    const JVal& sep = *grid.get("separator");
    if (gt.kind != JVal::STR || sep.kind != JVal::STR || cshape.kind != JVal::ARR) {
        err = "chunk_grid field types";
        return ZCG_ERR_INVALID_DATA;
    }
    if (shape.arr.size() > ZCG_MAX_DIMS || cshape.arr.size() > ZCG_MAX_DIMS) {
        err = "more dimensions than ZCG_MAX_DIMS";
        return ZCG_ERR_UNSUPPORTED;
    }
    out->ndim = (uint32_t)shape.arr.size();
    for (size_t i = 0; i < shape.arr.size(); i++) {
        const JVal& x = shape.arr[i];
        if (x.kind != JVal::NUM || !x.is_int || x.neg) { err = "shape entries must be u64"; return ZCG_ERR_INVALID_DATA; }
        out->shape[i] = x.mag;
    }
    uint64_t nel = 1;
    for (size_t i = 0; i < cshape.arr.size(); i++) {
        const JVal& x = cshape.arr[i];
        if (x.kind != JVal::NUM || !x.is_int || x.neg || x.mag > 0xFFFFFFFFull) {
            err = "chunk_shape entries must be u32";
            return ZCG_ERR_INVALID_DATA;
        }
        out->chunk_shape[i] = x.mag;
        if (x.mag && nel > UINT64_MAX / x.mag) { err = "chunk_shape product overflows u64"; return ZCG_ERR_INVALID_DATA; }
        nel *= x.mag;
    }
    out->chunk_ndim = (uint32_t)cshape.arr.size();
    if (sep.s.size() >= sizeof out->separator) { err = "separator too long"; return ZCG_ERR_UNSUPPORTED; }
    memcpy(out->separator, sep.s.c_str(), sep.s.size() + 1);
    const JVal& lay = *root.get("chunk_memory_layout");
    if (lay.kind != JVal::STR || (lay.s != "C" && lay.s != "F")) { err = "chunk_memory_layout must be C or F"; return ZCG_ERR_INVALID_DATA; }
    out->chunk_order = lay.s == "F" ? 1 : 0;
    // extensions: must_understand -> UnknownRequiredExtension (storage.rs:172-176)
    const JVal& ext = *root.get("extensions");
    if (ext.kind != JVal::ARR) { err = "extensions is not an array"; return ZCG_ERR_INVALID_DATA; }
    for (const JVal& x : ext.arr) {
        if (x.kind != JVal::OBJ || !x.get("extension") || x.get("extension")->kind != JVal::STR ||
            !x.get("must_understand") || x.get("must_understand")->kind != JVal::BOOL) {
            err = "extension metadata needs extension and must_understand";
            return ZCG_ERR_INVALID_DATA;
        }
        if (x.get("must_understand")->b) {
            err = "Encountered an unknown extension that must be understood: " + x.get("extension")->s;
            return ZCG_ERR_UNSUPPORTED;
        }
    }
    if (root.get("attributes")->kind != JVal::OBJ) { err = "attributes is not an object"; return ZCG_ERR_INVALID_DATA; }
    // data type, with ExtensibleDataType::effective_type (data_type.rs:282-310)
    const JVal& dtv = *root.get("data_type");
    Dt d{};
    int st;
    if (dtv.kind == JVal::STR) {
        st = parse_dtype(dtv.s, d, err);
        if (st) return st;
    } else if (dtv.kind == JVal::OBJ && dtv.get("extension") && dtv.get("type")) {
        const JVal* fb = dtv.get("fallback");
        if (!fb || fb->kind == JVal::NUL) { err = "extended data type without fallback (the reference: todo!())"; return ZCG_ERR_UNSUPPORTED; }
        if (fb->kind != JVal::STR) { err = "fallback is not a data type"; return ZCG_ERR_INVALID_DATA; }
        st = parse_dtype(fb->s, d, err);
        if (st) return st;
        out->extended_type = 1;
    } else {
        err = "invalid data_type";
        return ZCG_ERR_INVALID_DATA;
    }
    out->dtype_kind = (uint32_t)d.kind;
    out->array.dtype.elem_size = (uint8_t)(d.size > 255 ? 0 : d.size);
    out->array.dtype.big_endian = (d.big && d.size > 1 && d.kind != DT_BOOL) ? 1 : 0;
    out->array.dtype.is_bool = d.kind == DT_BOOL ? 1 : 0;
    out->array.chunk_num_elements = nel;
    // compressor (mod.rs:36-51), default Raw
    zcg_compression& c = out->array.compression;
    c.codec = ZCG_CODEC_RAW;
    c.gzip_level = -1;
    c.lz4_block_size = 65536;
    c.bzip2_block_size = 9;
    c.xz_preset = 6;
    if (const JVal* comp = root.get("compressor")) {
        if (comp->kind != JVal::OBJ || !comp->get("codec") || comp->get("codec")->kind != JVal::STR) {
            err = "compressor needs a codec";
            return ZCG_ERR_INVALID_DATA;
        }
        const std::string& id = comp->get("codec")->s;
        const JVal* conf = comp->get("configuration");
        if (conf && conf->kind != JVal::OBJ && conf->kind != JVal::NUL) { err = "configuration is not an object"; return ZCG_ERR_INVALID_DATA; }
        if (conf && conf->kind == JVal::NUL) conf = nullptr;
        bool bad = false;
        if (id == "raw") {
            c.codec = ZCG_CODEC_RAW;
        } else if (id == "https://purl.org/zarr/spec/codec/gzip/1.0") {
            c.codec = ZCG_CODEC_GZIP;
            c.gzip_level = (int32_t)cfg_int(conf, "level", -1, bad);
        } else if (id == "lz4") {
            c.codec = ZCG_CODEC_LZ4;
            c.lz4_block_size = (int32_t)cfg_int(conf, "blockSize", 65536, bad);
        } else if (id == "bzip2") {
            c.codec = ZCG_CODEC_BZIP2;
            const int64_t b = cfg_int(conf, "blockSize", 9, bad);
            if (b < 0 || b > 255) bad = true;  // u8 field (bzip.rs:18-21)
            c.bzip2_block_size = (int32_t)b;
        } else if (id == "xz") {
            c.codec = ZCG_CODEC_XZ;
            c.xz_preset = (int32_t)cfg_int(conf, "preset", 6, bad);
        } else {
            err = "unknown codec " + id;
            return ZCG_ERR_INVALID_DATA;
        }
        if (bad) { err = "bad codec configuration"; return ZCG_ERR_INVALID_DATA; }
    }
    // fill value (Option<Value>; get_effective_fill_value, lib.rs:448-454)
    if (const JVal* fv = root.get("fill_value")) {
        if (fv->kind != JVal::NUL) {
            out->has_fill_value = 1;
            st = fill_bits(*fv, d, out->fill_value, err);
            if (st) {
                out->has_fill_value = 0;
                out->fill_value_status = st;
            }
        }
    }
    // (serde does not compare the lengths of shape and chunk_shape; only
    // ArrayMetadata::new asserts it, lib.rs:411-415)
    return ZCG_OK;
}

}  // namespace

extern "C" int zcg_array_meta_from_json(const char* json, uint64_t len, zcg_array_meta* out, char* err,
                                        uint64_t err_cap) {
    if (!json || !out) return ZCG_ERR_INVALID_INPUT;
    std::string e;
    const int st = parse_meta(json, len, out, e);
    if (err && err_cap) {
        const size_t n = e.size() < err_cap - 1 ? e.size() : (size_t)err_cap - 1;
        memcpy(err, e.c_str(), n);
        err[n] = 0;
    }
    return st;
}

// FilesystemHierarchy::get_path (filesystem.rs:151-190) on Unix paths.  The
// key is split the way std::path::Path::components does: leading '/'s are the
// root (dropped: the key is taken relative to the store), empty components
// ("a//b", a trailing '/') and "." components vanish (a file the OS names
// the same with or without them), ".." stays literal (the
// OS resolves it against the joined path, as it does for the reference's
// PathBuf).  Only the NET nesting is checked: +1 per normal component, -1 per
// "..", NotFound when the total is negative (so "a/../b" and "../a/b" are
// accepted, "a/../../b" too, and "../../x" is not).
extern "C" int zcg_store_path(const char* root, const char* key, char* out, uint64_t cap, uint64_t* path_len) {
    if (!root || !key) return ZCG_ERR_INVALID_INPUT;
    std::string rel;
    long nest = 0;
    const char* p = key;
    while (*p == '/') p++;
    while (*p) {
        const char* e = p;
        while (*e && *e != '/') e++;
        const size_t n = (size_t)(e - p);
        const bool cur = n == 1 && p[0] == '.';
        const bool par = n == 2 && p[0] == '.' && p[1] == '.';
        if (n && !cur) {
            nest += par ? -1 : 1;
            if (!rel.empty()) rel += '/';
            rel.append(p, n);
        }
        p = *e ? e + 1 : e;
    }
    if (nest < 0) return ZCG_ERR_NOT_FOUND;
    // PathBuf::from(root).join(rel): an empty root joins to the relative path
    std::string path = root;
    if (!rel.empty()) {
        if (path.empty()) path = rel;
        else {
            if (path.back() != '/') path += '/';
            path += rel;
        }
    }
    if (path_len) *path_len = path.size();
    if (!out || cap < path.size() + 1) {
        if (out && cap) out[0] = 0;
        return out ? ZCG_ERR_OUTPUT_TOO_SMALL : ZCG_OK;
    }
    memcpy(out, path.c_str(), path.size() + 1);
    return ZCG_OK;
}

extern "C" uint64_t zcg_chunk_key(const char* path, const char* separator, const uint64_t* grid_position,
                                  uint32_t ndim, char* out, uint64_t cap) {
    std::string p = path ? path : "";
    size_t a = 0, b = p.size();
    while (a < b && p[a] == '/') a++;  // trim_start_matches('/')
    while (b > a && p[b - 1] == '/') b--;  // trim_end_matches('/')
    std::string key = "/data/root";
    if (b > a) key += "/" + p.substr(a, b - a);
    key += "/c";
    for (uint32_t i = 0; i < ndim; i++) {
        key += std::to_string(grid_position[i]);
        if (i + 1 < ndim && separator) key += separator;
    }
    if (out && cap) {
        const size_t k = key.size() < cap - 1 ? key.size() : (size_t)cap - 1;
        memcpy(out, key.data(), k);
        out[k] = 0;
    }
    return key.size();
}
