// ply.cpp -- PLY mesh reader for Shape "plymesh" (host side of the boundary).
//
// Behaviour of CreatePLYMesh (src/shapes/plymesh.cpp:107-235) on top of the
// rply library (src/ext/rply.cpp): ascii, binary_little_endian and
// binary_big_endian files; vertex x/y/z required; nx/ny/nz when all three are
// present; uv from the first complete pair of u/v, s/t, texture_u/texture_v,
// texture_s/texture_t; faces from "vertex_indices" lists -- triangles kept,
// quads split into (0,1,2) and (3,0,2), other polygons skipped with a warning;
// a vertex index out of range is an error.  Every property value is read in
// its stored type and converted to float as rply's double -> (float) does.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "host_common.h"

namespace pt {

namespace {

enum PlyType { kI8, kU8, kI16, kU16, kI32, kU32, kF32, kF64, kBad };

PlyType ply_type(const std::string& s) {
    if (s == "char" || s == "int8") return kI8;
    if (s == "uchar" || s == "uint8") return kU8;
    if (s == "short" || s == "int16") return kI16;
    if (s == "ushort" || s == "uint16") return kU16;
    if (s == "int" || s == "int32") return kI32;
    if (s == "uint" || s == "uint32") return kU32;
    if (s == "float" || s == "float32") return kF32;
    if (s == "double" || s == "float64") return kF64;
    return kBad;
}

int type_size(PlyType t) {
    switch (t) {
        case kI8: case kU8: return 1;
        case kI16: case kU16: return 2;
        case kI32: case kU32: case kF32: return 4;
        case kF64: return 8;
        default: return 0;
    }
}

struct Prop {
    std::string name;
    PlyType type = kBad;
    bool list = false;
    PlyType count_type = kBad;
};

struct Element {
    std::string name;
    long count = 0;
    std::vector<Prop> props;
};

// Sequential value source over the file body (ascii tokens or binary words).
class Reader {
  public:
    // `data` must outlive the reader; values start at byte `start`.
    Reader(const std::string& data, size_t start, int format) : b_(data), fmt_(format), pos_(start) {
        if (fmt_ == 0) ss_.str(data.substr(start));
    }
    double get(PlyType t) {
        if (fmt_ == 0) {
            std::string tok;
            if (!(ss_ >> tok)) throw PtError(PT_ERR_PARSE, "plymesh: unexpected end of ascii data");
            if (t == kF32 || t == kF64) return std::strtod(tok.c_str(), nullptr);
            return (double)std::strtoll(tok.c_str(), nullptr, 10);
        }
        const int n = type_size(t);
        if (pos_ + (size_t)n > b_.size()) throw PtError(PT_ERR_PARSE, "plymesh: unexpected end of binary data");
        unsigned char raw[8];
        std::memcpy(raw, b_.data() + pos_, (size_t)n);
        pos_ += (size_t)n;
        const bool big = fmt_ == 2;
        if (big) for (int i = 0; i < n / 2; ++i) std::swap(raw[i], raw[n - 1 - i]);  // host is little-endian
        switch (t) {
            case kI8: { int8_t v; std::memcpy(&v, raw, 1); return v; }
            case kU8: { uint8_t v; std::memcpy(&v, raw, 1); return v; }
            case kI16: { int16_t v; std::memcpy(&v, raw, 2); return v; }
            case kU16: { uint16_t v; std::memcpy(&v, raw, 2); return v; }
            case kI32: { int32_t v; std::memcpy(&v, raw, 4); return v; }
            case kU32: { uint32_t v; std::memcpy(&v, raw, 4); return v; }
            case kF32: { float v; std::memcpy(&v, raw, 4); return v; }
            case kF64: { double v; std::memcpy(&v, raw, 8); return v; }
            default: throw PtError(PT_ERR_PARSE, "plymesh: bad property type");
        }
    }

  private:
    const std::string& b_;
    int fmt_;
    size_t pos_;
    std::istringstream ss_;
};

}  // namespace

void read_ply(const std::string& path, PlyMesh* out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw PtError(PT_ERR_IO, "Couldn't open PLY file \"" + path + "\"");
    std::stringstream all;
    all << f.rdbuf();
    const std::string data = all.str();
    // header
    size_t p = 0;
    auto line = [&]() {
        size_t e = data.find('\n', p);
        if (e == std::string::npos) throw PtError(PT_ERR_PARSE, "Unable to read the header of PLY file \"" + path + "\"");
        std::string l = data.substr(p, e - p);
        p = e + 1;
        if (!l.empty() && l.back() == '\r') l.pop_back();
        return l;
    };
    if (line() != "ply") throw PtError(PT_ERR_PARSE, "Unable to read the header of PLY file \"" + path + "\"");
    int fmt = -1;
    std::vector<Element> els;
    for (;;) {
        std::istringstream ls(line());
        std::string kw;
        ls >> kw;
        if (kw == "end_header") break;
        if (kw == "format") {
            std::string f2;
            ls >> f2;
            fmt = f2 == "ascii" ? 0 : f2 == "binary_little_endian" ? 1 : f2 == "binary_big_endian" ? 2 : -1;
            if (fmt < 0) throw PtError(PT_ERR_PARSE, "plymesh: unknown format " + f2);
        } else if (kw == "element") {
            Element e;
            ls >> e.name >> e.count;
            els.push_back(e);
        } else if (kw == "property") {
            if (els.empty()) throw PtError(PT_ERR_PARSE, "plymesh: property before element");
            Prop pr;
            std::string t;
            ls >> t;
            if (t == "list") {
                std::string ct, it;
                ls >> ct >> it >> pr.name;
                pr.list = true;
                pr.count_type = ply_type(ct);
                pr.type = ply_type(it);
            } else {
                pr.type = ply_type(t);
                ls >> pr.name;
            }
            if (pr.type == kBad || (pr.list && pr.count_type == kBad))
                throw PtError(PT_ERR_PARSE, "plymesh: unknown property type in \"" + path + "\"");
            els.back().props.push_back(pr);
        }  // comment / obj_info: ignored
    }
    if (fmt < 0) throw PtError(PT_ERR_PARSE, "plymesh: missing format line");
    long nv = 0, nf = 0;
    const Element* ve = nullptr;
    for (const auto& e : els) {
        if (e.name == "vertex") { nv = e.count; ve = &e; }
        else if (e.name == "face") nf = e.count;
    }
    if (nv == 0 || nf == 0) throw PtError(PT_ERR_PARSE, path + ": PLY file is invalid! No face/vertex elements found!");
    auto has = [&](const char* n) {
        for (const auto& pr : ve->props)
            if (!pr.list && pr.name == n) return true;
        return false;
    };
    if (!(has("x") && has("y") && has("z"))) throw PtError(PT_ERR_PARSE, path + ": Vertex coordinate property not found!");
    out->hasN = has("nx") && has("ny") && has("nz");
    const char* uvNames[4][2] = {{"u", "v"}, {"s", "t"}, {"texture_u", "texture_v"}, {"texture_s", "texture_t"}};
    std::string un, vn;
    for (auto& pr : uvNames)
        if (has(pr[0]) && has(pr[1])) { un = pr[0]; vn = pr[1]; break; }
    out->hasUV = !un.empty();
    out->P.assign((size_t)3 * nv, 0.f);
    out->N.assign(out->hasN ? (size_t)3 * nv : 0, 0.f);
    out->UV.assign(out->hasUV ? (size_t)2 * nv : 0, 0.f);
    out->idx.clear();
    Reader rd(data, p, fmt);
    bool badIndex = false;
    for (const auto& e : els) {
        for (long i = 0; i < e.count; ++i) {
            for (const auto& pr : e.props) {
                if (pr.list) {
                    const long len = (long)rd.get(pr.count_type);
                    std::vector<int> face;
                    for (long k = 0; k < len; ++k) face.push_back((int)rd.get(pr.type));
                    if (e.name != "face" || pr.name != "vertex_indices") continue;
                    if (len != 3 && len != 4) {
                        std::fprintf(stderr, "plymesh: Ignoring face with %d vertices (only triangles and quads "
                                             "are supported!)\n", (int)len);
                        continue;
                    }
                    for (int v : face)
                        if (v < 0 || v >= nv) badIndex = true;
                    out->idx.insert(out->idx.end(), {face[0], face[1], face[2]});
                    if (len == 4) out->idx.insert(out->idx.end(), {face[3], face[0], face[2]});
                    continue;
                }
                const double v = rd.get(pr.type);
                if (e.name != "vertex") continue;
                const float fv = (float)v;
                if (pr.name == "x") out->P[3 * i] = fv;
                else if (pr.name == "y") out->P[3 * i + 1] = fv;
                else if (pr.name == "z") out->P[3 * i + 2] = fv;
                else if (out->hasN && pr.name == "nx") out->N[3 * i] = fv;
                else if (out->hasN && pr.name == "ny") out->N[3 * i + 1] = fv;
                else if (out->hasN && pr.name == "nz") out->N[3 * i + 2] = fv;
                else if (out->hasUV && pr.name == un) out->UV[2 * i] = fv;
                else if (out->hasUV && pr.name == vn) out->UV[2 * i + 1] = fv;
            }
        }
    }
    if (badIndex) throw PtError(PT_ERR_PARSE, "plymesh: Vertex reference out of bounds in \"" + path + "\"");
}

}  // namespace pt
