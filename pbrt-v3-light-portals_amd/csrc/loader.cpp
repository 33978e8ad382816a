// loader.cpp -- host .pbrt scene loader for the hot path's supported subset.
//
// Mirrors the reference's tokenizer (src/core/parser.cpp:252-366), parameter
// lists (parser.cpp:711-781), graphics state and directive semantics
// (src/core/api.cpp) closely enough that the flattened pt_scene_desc equals
// the reference's post-WorldEnd Scene: world-space triangles
// (triangle.cpp:75), aaplanes (plane.cpp:117-128), one DiffuseAreaLight per
// emitting triangle (api.cpp:1370-1378), PortalArealight + AAPortals parsed
// from portalData (portal_arealight.cpp:245-300), CameraToWorld = Inverse(CTM)
// at Camera, and Film/Sampler/Integrator parameters with reference defaults.
// Anything outside the subset fails loudly with PT_ERR_UNSUPPORTED.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pt.h"
#include "host_common.h"

namespace pt {

// ---------------------------------------------------------------------------
// Matrix4x4 / Transform (src/core/transform.{h,cpp}) -- host restatement
// ---------------------------------------------------------------------------
HM4 hm4_identity() {
    HM4 r;
    std::memset(&r, 0, sizeof r);
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1;
    return r;
}
HM4 hm4_mul(const HM4& a, const HM4& b) {  // transform.h:86-93
    HM4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j] +
                        a.m[i][3] * b.m[3][j];
    return r;
}
HM4 hm4_transpose(const HM4& a) {
    HM4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = a.m[j][i];
    return r;
}
bool hm4_inverse(const HM4& mm, HM4* out) {  // transform.cpp:85-137
    int indxc[4], indxr[4];
    int ipiv[4] = {0, 0, 0, 0};
    float minv[4][4];
    std::memcpy(minv, mm.m, sizeof minv);
    bool ok = true;
    for (int i = 0; i < 4; i++) {
        int irow = 0, icol = 0;
        float big = 0.f;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (std::abs(minv[j][k]) >= big) {
                            big = std::abs(minv[j][k]);
                            irow = j;
                            icol = k;
                        }
                    } else if (ipiv[k] > 1)
                        ok = false;
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(minv[irow][k], minv[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (minv[icol][icol] == 0.f) ok = false;
        float pivinv = (float)(1. / (double)minv[icol][icol]);
        minv[icol][icol] = 1.;
        for (int j = 0; j < 4; j++) minv[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                float save = minv[j][icol];
                minv[j][icol] = 0;
                for (int k = 0; k < 4; k++) minv[j][k] -= minv[icol][k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--) {
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(minv[k][indxr[j]], minv[k][indxc[j]]);
    }
    std::memcpy(out->m, minv, sizeof minv);
    return ok;
}

HXF hxf_identity() { return HXF{hm4_identity(), hm4_identity()}; }
HXF hxf_from_matrix(const HM4& m) {
    HXF t;
    t.m = m;
    hm4_inverse(m, &t.mi);
    return t;
}
HXF hxf_inverse(const HXF& t) { return HXF{t.mi, t.m}; }
HXF hxf_mul(const HXF& a, const HXF& b) { return HXF{hm4_mul(a.m, b.m), hm4_mul(b.mi, a.mi)}; }
HXF hxf_translate(float x, float y, float z) {  // transform.cpp:141-147
    HXF t = hxf_identity();
    t.m.m[0][3] = x; t.m.m[1][3] = y; t.m.m[2][3] = z;
    t.mi.m[0][3] = -x; t.mi.m[1][3] = -y; t.mi.m[2][3] = -z;
    return t;
}
HXF hxf_scale(float x, float y, float z) {  // transform.cpp:149-153
    HXF t = hxf_identity();
    t.m.m[0][0] = x; t.m.m[1][1] = y; t.m.m[2][2] = z;
    t.mi.m[0][0] = 1 / x; t.mi.m[1][1] = 1 / y; t.mi.m[2][2] = 1 / z;
    return t;
}
static float radians(float deg) { return (kPi / 180) * deg; }  // pbrt.h:336
HXF hxf_rotate(float theta, float ax, float ay, float az) {  // transform.cpp:179-203
    V3 a = normalize(v3(ax, ay, az));
    float s = std::sin(radians(theta));
    float c = std::cos(radians(theta));
    HM4 m = hm4_identity();
    m.m[0][0] = a.x * a.x + (1 - a.x * a.x) * c;
    m.m[0][1] = a.x * a.y * (1 - c) - a.z * s;
    m.m[0][2] = a.x * a.z * (1 - c) + a.y * s;
    m.m[0][3] = 0;
    m.m[1][0] = a.x * a.y * (1 - c) + a.z * s;
    m.m[1][1] = a.y * a.y + (1 - a.y * a.y) * c;
    m.m[1][2] = a.y * a.z * (1 - c) - a.x * s;
    m.m[1][3] = 0;
    m.m[2][0] = a.x * a.z * (1 - c) - a.y * s;
    m.m[2][1] = a.y * a.z * (1 - c) + a.x * s;
    m.m[2][2] = a.z * a.z + (1 - a.z * a.z) * c;
    m.m[2][3] = 0;
    return HXF{m, hm4_transpose(m)};
}
bool hxf_lookat(V3 pos, V3 look, V3 up, HXF* out) {  // transform.cpp:205-238
    HM4 c2w;
    std::memset(&c2w, 0, sizeof c2w);
    c2w.m[0][3] = pos.x; c2w.m[1][3] = pos.y; c2w.m[2][3] = pos.z; c2w.m[3][3] = 1;
    V3 dir = normalize(look - pos);
    if (len(cross(normalize(up), dir)) == 0) {
        *out = hxf_identity();
        return false;
    }
    V3 right = normalize(cross(normalize(up), dir));
    V3 newUp = cross(dir, right);
    c2w.m[0][0] = right.x; c2w.m[1][0] = right.y; c2w.m[2][0] = right.z; c2w.m[3][0] = 0.;
    c2w.m[0][1] = newUp.x; c2w.m[1][1] = newUp.y; c2w.m[2][1] = newUp.z; c2w.m[3][1] = 0.;
    c2w.m[0][2] = dir.x; c2w.m[1][2] = dir.y; c2w.m[2][2] = dir.z; c2w.m[3][2] = 0.;
    HM4 w2c;
    hm4_inverse(c2w, &w2c);
    *out = HXF{w2c, c2w};
    return true;
}
HXF hxf_perspective(float fov, float n, float f) {  // transform.cpp:303-311
    HM4 p;
    std::memset(&p, 0, sizeof p);
    p.m[0][0] = 1; p.m[1][1] = 1;
    p.m[2][2] = f / (f - n); p.m[2][3] = -f * n / (f - n);
    p.m[3][2] = 1;
    float invTanAng = 1 / std::tan(radians(fov) / 2);
    return hxf_mul(hxf_scale(invTanAng, invTanAng, 1), hxf_from_matrix(p));
}
bool hxf_swaps_handedness(const HXF& t) {  // transform.cpp:248-253
    const auto& m = t.m.m;
    float det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    return det < 0;
}
static void store_xf(const HXF& t, pt_transform* out) {
    std::memcpy(out->m, t.m.m, 64);
    std::memcpy(out->minv, t.mi.m, 64);
}
M4 to_m4(const HM4& h) {
    M4 r;
    std::memcpy(r.m, h.m, 64);
    return r;
}

// ---------------------------------------------------------------------------
// Tokenizer (parser.cpp:252-318) and number parsing (parser.cpp:322-366)
// ---------------------------------------------------------------------------
namespace {

struct Token {
    std::string s;
    bool quoted = false;
};

class Tokenizer {
  public:
    explicit Tokenizer(std::string text) : src_(std::move(text)) {}
    bool next(Token* t) {
        for (;;) {
            if (pos_ >= src_.size()) return false;
            char ch = src_[pos_++];
            if (ch == ' ' || ch == '\n' || ch == '\t' || ch == '\r') continue;
            if (ch == '"') {
                std::string s;
                for (;;) {
                    if (pos_ >= src_.size()) throw PtError(PT_ERR_PARSE, "premature EOF in string");
                    ch = src_[pos_++];
                    if (ch == '"') break;
                    if (ch == '\n') throw PtError(PT_ERR_PARSE, "unterminated string");
                    if (ch == '\\') {
                        if (pos_ >= src_.size()) throw PtError(PT_ERR_PARSE, "premature EOF");
                        char e = src_[pos_++];
                        switch (e) {
                            case 'b': s.push_back('\b'); break;
                            case 'f': s.push_back('\f'); break;
                            case 'n': s.push_back('\n'); break;
                            case 'r': s.push_back('\r'); break;
                            case 't': s.push_back('\t'); break;
                            default: s.push_back(e); break;
                        }
                    } else
                        s.push_back(ch);
                }
                t->s = s;
                t->quoted = true;
                return true;
            }
            if (ch == '[' || ch == ']') {
                t->s = std::string(1, ch);
                t->quoted = false;
                return true;
            }
            if (ch == '#') {
                while (pos_ < src_.size() && src_[pos_] != '\n' && src_[pos_] != '\r') ++pos_;
                continue;  // comments are skipped by the parser (parser.cpp:838-842)
            }
            size_t start = pos_ - 1;
            while (pos_ < src_.size()) {
                char c = src_[pos_];
                if (c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '"' || c == '[' || c == ']') break;
                ++pos_;
            }
            t->s = src_.substr(start, pos_ - start);
            t->quoted = false;
            return true;
        }
    }

  private:
    std::string src_;
    size_t pos_ = 0;
};

double parse_number(const std::string& str) {
    if (str.size() == 1) {
        if (!(str[0] >= '0' && str[0] <= '9')) throw PtError(PT_ERR_PARSE, "expected a number: " + str);
        return str[0] - '0';
    }
    bool isInt = !str.empty();
    for (char ch : str)
        if (!(ch >= '0' && ch <= '9')) isInt = false;
    char* end = nullptr;
    double val;
    if (isInt)
        val = double(std::strtol(str.c_str(), &end, 10));
    else
        val = std::strtof(str.c_str(), &end);
    if (val == 0 && end == str.c_str()) throw PtError(PT_ERR_PARSE, "expected a number: " + str);
    return val;
}

struct Param {
    std::string type, name;
    std::vector<double> nums;
    std::vector<std::string> strs;
    std::vector<float> s60;  // "spectrum"/"blackbody"/"xyz": the SampledSpectrum value (60 bins each)
};

struct ParamSet {
    std::vector<Param> params;
    const Param* find(const char* name, std::initializer_list<const char*> types) const {
        for (auto it = params.rbegin(); it != params.rend(); ++it) {
            if (it->name != name) continue;
            for (const char* ty : types)
                if (it->type == ty) return &*it;
        }
        return nullptr;
    }
    bool has(const char* name) const {
        for (const auto& p : params)
            if (p.name == name) return true;
        return false;
    }
    float float1(const char* n, float def) const {
        const Param* p = find(n, {"float"});
        return (p && !p->nums.empty()) ? (float)p->nums[0] : def;
    }
    const Param* floats(const char* n) const { return find(n, {"float"}); }
    int int1(const char* n, int def) const {
        const Param* p = find(n, {"integer"});
        return (p && !p->nums.empty()) ? int(p->nums[0]) : def;
    }
    bool bool1(const char* n, bool def) const {
        const Param* p = find(n, {"bool"});
        if (!p) return def;
        if (!p->strs.empty()) {
            if (p->strs[0] == "true") return true;
            if (p->strs[0] == "false") return false;
            throw PtError(PT_ERR_PARSE, "bad bool value for " + std::string(n));
        }
        return def;
    }
    std::string string1(const char* n, const std::string& def) const {
        const Param* p = find(n, {"string"});
        return (p && !p->strs.empty()) ? p->strs[0] : def;
    }
    bool point3(const char* n, V3* out) const {
        const Param* p = find(n, {"point", "point3"});
        if (!p || p->nums.size() < 3) return false;
        *out = v3((float)p->nums[0], (float)p->nums[1], (float)p->nums[2]);
        return true;
    }
    // FindOneSpectrum for the SampledSpectrum build: "rgb" parameters go
    // through FromRGB with the Illuminant default (paramset.cpp:110-120,
    // spectrum.h:420-421); spectral ones keep the 60-bin value computed
    // when the parameter list was parsed.
    bool spectrum60(const char* n, float out[60]) const {
        for (auto it = params.rbegin(); it != params.rend(); ++it) {
            if (it->name != n || it->type != "rgb") continue;
            if (!it->s60.empty()) {
                for (int i = 0; i < 60; ++i) out[i] = it->s60[i];
            } else {
                if (it->nums.size() < 3) throw PtError(PT_ERR_PARSE, "rgb needs 3 values");
                const float rgb[3] = {(float)it->nums[0], (float)it->nums[1], (float)it->nums[2]};
                s60_from_rgb(rgb, false, out);
            }
            return true;
        }
        return false;
    }
    // FindOneSpectrum for the RGB build: "rgb"/"color" are RGB triples
    // (RGBSpectrum::FromRGB); spectral types were reduced to "rgb" by
    // spectral_to_rgb when the parameter list was parsed.
    bool spectrum(const char* n, float out[3]) const {
        for (auto it = params.rbegin(); it != params.rend(); ++it) {
            if (it->name != n) continue;
            if (it->type == "rgb" || it->type == "color") {
                if (it->nums.size() < 3) throw PtError(PT_ERR_PARSE, "rgb needs 3 values");
                for (int i = 0; i < 3; ++i) out[i] = (float)it->nums[i];
                return true;
            }
        }
        return false;
    }
};

// TrowbridgeReitzDistribution::RoughnessToAlpha (microfacet.h:127-132), float
// arithmetic and the platform logf as the reference binary evaluates it.
float tr_roughness_to_alpha(float roughness) {
    roughness = std::max(roughness, (float)1e-3);
    const float x = std::log(roughness);
    return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
}

struct Directive {
    std::string name;
    ParamSet ps;
};

struct GraphicsState {
    std::string material = "matte";
    ParamSet materialParams;
    std::string areaLight;
    ParamSet areaLightParams;
    bool reverseOrientation = false;
};

}  // namespace

// ---------------------------------------------------------------------------
// Scene builder
// ---------------------------------------------------------------------------
struct pt_host_scene_impl {
    std::vector<float> P, N, S, UV;
    bool anyN = false, anyS = false, anyUV = false;
    std::vector<pt_triangle> tris;
    std::vector<pt_aaplane> planes;
    std::vector<pt_sphere> spheres;
    std::vector<pt_prim> prims;
    std::vector<pt_material> materials;
    std::vector<pt_light> lights;
    std::vector<pt_portal> portals;
    std::string film_filename = "pbrt.exr";
    bool spectral = false;
    std::vector<float> mat_s60, light_s60;  // 3 x 60 per material, 60 per light (spectral scenes)
    pt_scene_desc desc{};
};

namespace {

class Loader {
  public:
    explicit Loader(pt_host_scene_impl* out) : out_(out) {}

    void parse_file(const std::string& path) {
        std::ifstream f(path, std::ios::binary);
        if (!f) throw PtError(PT_ERR_IO, "cannot open " + path);
        std::stringstream ss;
        ss << f.rdbuf();
        std::string dir = path.substr(0, path.find_last_of('/') == std::string::npos ? 0 : path.find_last_of('/') + 1);
        dirs_.push_back(dir);
        if (dirs_.size() == 1) searchDir_ = dir;  // SetSearchDirectory (parser.cpp:1095)
        parse_text(ss.str());
        dirs_.pop_back();
    }

    void finish() {
        if (!worldEnded_) throw PtError(PT_ERR_PARSE, "missing WorldEnd");
    }

  private:
    pt_host_scene_impl* out_;
    std::vector<std::string> dirs_;
    std::string searchDir_;
    HXF ctm_ = hxf_identity();
    std::vector<HXF> xfStack_;
    GraphicsState gs_;
    std::vector<GraphicsState> gsStack_;
    std::map<std::string, HXF> namedCS_;
    std::map<std::string, std::pair<std::string, ParamSet>> namedMaterials_;
    Directive camera_{"perspective", {}}, film_{"image", {}}, sampler_{"halton", {}}, integrator_{"path", {}},
        filter_{"box", {}}, accel_{"bvh", {}};
    HXF cameraToWorld_ = hxf_identity();
    bool inWorld_ = false, worldEnded_ = false;

    // ---- parameter lists (parser.cpp:711-781) ----
    ParamSet parse_params(Tokenizer& tk, Token* pending, bool* havePending) {
        ParamSet ps;
        for (;;) {
            Token decl;
            if (!tk.next(&decl)) { *havePending = false; return ps; }
            if (!decl.quoted) { *pending = decl; *havePending = true; return ps; }
            Param p;
            {
                std::istringstream is(decl.s);
                is >> p.type >> p.name;
                if (p.name.empty()) throw PtError(PT_ERR_PARSE, "bad parameter declaration \"" + decl.s + "\"");
            }
            if (p.type == "point3") p.type = "point";
            if (p.type == "vector3") p.type = "vector";
            if (p.type == "normal3") p.type = "normal";
            if (p.type == "color") p.type = "rgb";
            Token v;
            if (!tk.next(&v)) throw PtError(PT_ERR_PARSE, "premature EOF in parameter list");
            auto add = [&](const Token& t) {
                if (t.quoted) {
                    if (!p.nums.empty()) throw PtError(PT_ERR_PARSE, "mixed string and numeric parameters");
                    p.strs.push_back(t.s);
                } else {
                    if (!p.strs.empty()) throw PtError(PT_ERR_PARSE, "mixed string and numeric parameters");
                    p.nums.push_back(parse_number(t.s));
                }
            };
            if (!v.quoted && v.s == "[") {
                for (;;) {
                    Token x;
                    if (!tk.next(&x)) throw PtError(PT_ERR_PARSE, "premature EOF in [");
                    if (!x.quoted && x.s == "]") break;
                    add(x);
                }
            } else
                add(v);
            spectral_to_rgb(&p);
            ps.params.push_back(std::move(p));
        }
    }

    // The RGB build stores every spectral parameter as RGBSpectrum at parse
    // time (paramset.cpp:122-208): "spectrum" wavelength/value pairs or SPD
    // file names (FromSampled), "blackbody" (temperature, scale) pairs,
    // "xyz" triples (FromXYZ).  Rewrite them as "rgb" parameters.
    void spectral_to_rgb(Param* p) const {
        std::vector<double> rgbs;
        std::vector<float> s60;
        auto push = [&](const float c[3]) { for (int k = 0; k < 3; ++k) rgbs.push_back(c[k]); };
        if (p->type == "spectrum") {
            if (!p->strs.empty()) {
                for (const std::string& name : p->strs) {
                    std::string fn = (!name.empty() && name[0] == '/') ? name : searchDir_ + name;
                    std::vector<float> vals;
                    float c[3] = {0, 0, 0}, c60[60] = {0};
                    if (!read_float_file(fn, &vals)) {
                        std::fprintf(stderr, "Warning: Unable to read SPD file \"%s\".  Using black distribution.\n",
                                     fn.c_str());
                    } else {
                        std::vector<float> wl, v;
                        for (size_t j = 0; j + 1 < vals.size(); j += 2) wl.push_back(vals[j]), v.push_back(vals[j + 1]);
                        rgb_from_sampled(wl.data(), v.data(), (int)wl.size(), c);
                        s60_from_sampled(wl.data(), v.data(), (int)wl.size(), c60);
                    }
                    push(c);
                    s60.insert(s60.end(), c60, c60 + 60);
                }
            } else {
                if (p->nums.size() % 2) throw PtError(PT_ERR_PARSE, "spectrum \"" + p->name + "\" needs wavelength/value pairs");
                std::vector<float> wl, v;
                for (size_t j = 0; j < p->nums.size(); j += 2) wl.push_back((float)p->nums[j]), v.push_back((float)p->nums[j + 1]);
                float c[3], c60[60];
                rgb_from_sampled(wl.data(), v.data(), (int)wl.size(), c);
                s60_from_sampled(wl.data(), v.data(), (int)wl.size(), c60);
                push(c);
                s60.insert(s60.end(), c60, c60 + 60);
            }
        } else if (p->type == "blackbody") {
            if (p->nums.size() % 2) throw PtError(PT_ERR_PARSE, "blackbody \"" + p->name + "\" needs (T, scale) pairs");
            for (size_t j = 0; j < p->nums.size(); j += 2) {
                float c[3], c60[60];
                rgb_from_blackbody((float)p->nums[j], (float)p->nums[j + 1], c);
                s60_blackbody((float)p->nums[j], (float)p->nums[j + 1], c60);
                push(c);
                s60.insert(s60.end(), c60, c60 + 60);
            }
        } else if (p->type == "xyz") {
            if (p->nums.size() % 3) throw PtError(PT_ERR_PARSE, "xyz \"" + p->name + "\" needs triples");
            for (size_t j = 0; j < p->nums.size(); j += 3) {
                const float xyz[3] = {(float)p->nums[j], (float)p->nums[j + 1], (float)p->nums[j + 2]};
                float c[3], c60[60];
                xyz_to_rgb(xyz, c);
                s60_from_rgb(c, true, c60);  // FromXYZ: Reflectance default (spectrum.h:422-427)
                push(c);
                s60.insert(s60.end(), c60, c60 + 60);
            }
        } else {
            return;
        }
        p->type = "rgb";
        p->nums = std::move(rgbs);
        p->s60 = std::move(s60);
        p->strs.clear();
    }

    std::vector<float> read_nums(Tokenizer& tk, int n) {
        std::vector<float> v;
        Token t;
        bool bracket = false;
        while ((int)v.size() < n) {
            if (!tk.next(&t)) throw PtError(PT_ERR_PARSE, "premature EOF");
            if (!t.quoted && t.s == "[") { bracket = true; continue; }
            v.push_back((float)parse_number(t.s));
        }
        if (bracket) {
            if (!tk.next(&t) || t.s != "]") throw PtError(PT_ERR_PARSE, "expected ]");
        }
        return v;
    }
    std::string read_string(Tokenizer& tk) {
        Token t;
        if (!tk.next(&t) || !t.quoted) throw PtError(PT_ERR_PARSE, "expected quoted string");
        return t.s;
    }

    void parse_text(const std::string& text) {
        Tokenizer tk(text);
        Token t;
        bool havePending = false;
        for (;;) {
            if (havePending) { havePending = false; }
            else if (!tk.next(&t)) break;
            const std::string& d = t.s;
            if (t.quoted) throw PtError(PT_ERR_PARSE, "unexpected string " + d);
            auto params = [&](Directive* dst, const std::string& name) {
                dst->name = name;
                dst->ps = parse_params(tk, &t, &havePending);
            };
            if (d == "AttributeBegin") {
                gsStack_.push_back(gs_);
                xfStack_.push_back(ctm_);
            } else if (d == "AttributeEnd") {
                if (gsStack_.empty()) throw PtError(PT_ERR_PARSE, "unmatched AttributeEnd");
                gs_ = gsStack_.back(); gsStack_.pop_back();
                ctm_ = xfStack_.back(); xfStack_.pop_back();
            } else if (d == "TransformBegin") {
                xfStack_.push_back(ctm_);
            } else if (d == "TransformEnd") {
                if (xfStack_.empty()) throw PtError(PT_ERR_PARSE, "unmatched TransformEnd");
                ctm_ = xfStack_.back(); xfStack_.pop_back();
            } else if (d == "Identity") {
                ctm_ = hxf_identity();
            } else if (d == "Translate") {
                auto v = read_nums(tk, 3);
                ctm_ = hxf_mul(ctm_, hxf_translate(v[0], v[1], v[2]));
            } else if (d == "Scale") {
                auto v = read_nums(tk, 3);
                ctm_ = hxf_mul(ctm_, hxf_scale(v[0], v[1], v[2]));
            } else if (d == "Rotate") {
                auto v = read_nums(tk, 4);
                ctm_ = hxf_mul(ctm_, hxf_rotate(v[0], v[1], v[2], v[3]));
            } else if (d == "LookAt") {
                auto v = read_nums(tk, 9);
                HXF la;
                hxf_lookat(v3(v[0], v[1], v[2]), v3(v[3], v[4], v[5]), v3(v[6], v[7], v[8]), &la);
                ctm_ = hxf_mul(ctm_, la);
            } else if (d == "Transform" || d == "ConcatTransform") {
                auto v = read_nums(tk, 16);
                HM4 m;
                for (int i = 0; i < 16; ++i) m.m[i / 4][i % 4] = v[i];
                HXF x = hxf_from_matrix(hm4_transpose(m));  // pbrtTransform (api.cpp)
                ctm_ = (d == "Transform") ? x : hxf_mul(ctm_, x);
            } else if (d == "CoordinateSystem") {
                namedCS_[read_string(tk)] = ctm_;
            } else if (d == "CoordSysTransform") {
                std::string n = read_string(tk);
                auto it = namedCS_.find(n);
                if (it != namedCS_.end()) ctm_ = it->second;
            } else if (d == "ReverseOrientation") {
                gs_.reverseOrientation = !gs_.reverseOrientation;
            } else if (d == "Camera") {
                std::string n = read_string(tk);
                params(&camera_, n);
                cameraToWorld_ = hxf_inverse(ctm_);  // pbrtCamera
                namedCS_["camera"] = cameraToWorld_;
            } else if (d == "Film") {
                std::string n = read_string(tk); params(&film_, n);
            } else if (d == "Sampler") {
                std::string n = read_string(tk); params(&sampler_, n);
            } else if (d == "Integrator") {
                std::string n = read_string(tk); params(&integrator_, n);
                // the hero integrators exist only in the SampledSpectrum build
                out_->spectral = (n == "hero_path" || n == "hero_path_mis");
            } else if (d == "PixelFilter") {
                std::string n = read_string(tk); params(&filter_, n);
            } else if (d == "Accelerator") {
                std::string n = read_string(tk); params(&accel_, n);
            } else if (d == "WorldBegin") {
                inWorld_ = true;
                ctm_ = hxf_identity();
                namedCS_["world"] = ctm_;
            } else if (d == "WorldEnd") {
                world_end();
            } else if (d == "Material") {
                std::string n = read_string(tk);
                Directive tmp;
                params(&tmp, n);
                gs_.material = n;
                gs_.materialParams = tmp.ps;
            } else if (d == "MakeNamedMaterial") {
                std::string n = read_string(tk);
                Directive tmp;
                params(&tmp, n);
                namedMaterials_[n] = {tmp.ps.string1("type", ""), tmp.ps};
            } else if (d == "NamedMaterial") {
                std::string n = read_string(tk);
                auto it = namedMaterials_.find(n);
                if (it == namedMaterials_.end()) throw PtError(PT_ERR_PARSE, "unknown named material " + n);
                gs_.material = it->second.first;
                gs_.materialParams = it->second.second;
            } else if (d == "AreaLightSource") {
                std::string n = read_string(tk);
                Directive tmp;
                params(&tmp, n);
                gs_.areaLight = n;
                gs_.areaLightParams = tmp.ps;
            } else if (d == "LightSource") {
                std::string n = read_string(tk);
                Directive tmp;
                params(&tmp, n);
                light_source(n, tmp.ps);
            } else if (d == "Shape") {
                std::string n = read_string(tk);
                Directive tmp;
                params(&tmp, n);
                shape(n, tmp.ps);
            } else if (d == "Include") {
                std::string f = read_string(tk);
                if (f.empty() || f[0] != '/') f = searchDir_ + f;  // ResolveFilename (fileutil.cpp:105-114)
                parse_file(f);
            } else if (d == "Texture" || d == "MakeNamedMedium" || d == "MediumInterface" || d == "ObjectBegin" ||
                       d == "ObjectEnd" || d == "ObjectInstance" || d == "TransformTimes" ||
                       d == "ActiveTransform") {
                throw PtError(PT_ERR_UNSUPPORTED, "directive " + d + " is outside the supported subset");
            } else {
                throw PtError(PT_ERR_PARSE, "unknown directive " + d);
            }
        }
    }

    // TextureParams lookup order: shape parameters, then material parameters
    float f1(const char* n, float def, bool* found, const ParamSet& shapeParams) const {
        const Param* p = shapeParams.floats(n);
        if (!p) p = gs_.materialParams.floats(n);
        if (found) *found = p && !p->nums.empty();
        return (p && !p->nums.empty()) ? (float)p->nums[0] : def;
    }
    void spectrum2(const char* n, float out[3], const ParamSet& shapeParams) const {
        gs_.materialParams.spectrum(n, out);
        shapeParams.spectrum(n, out);
    }
    void no_textures(std::initializer_list<const char*> names, const ParamSet& shapeParams) const {
        for (const char* tex : names)
            if (gs_.materialParams.find(tex, {"texture"}) || shapeParams.find(tex, {"texture"}))
                throw PtError(PT_ERR_UNSUPPORTED, std::string("textured \"") + tex + "\" is outside the supported subset");
    }

    int material_for(const ParamSet& shapeParams) {
        // GraphicsState::GetMaterialForShape: shape params may override the
        // current material's parameters (api.cpp, TextureParams lookup order).
        std::string name = gs_.material;
        pt_material m{};
        if (name == "" || name == "none") {
            m.kind = PT_MAT_NONE;
        } else if (name == "matte") {
            m.kind = PT_MAT_MATTE;
            float kd[3] = {0.5f, 0.5f, 0.5f};  // CreateMatteMaterial default (matte.cpp:64-71)
            if (gs_.materialParams.find("Kd", {"texture"}) || shapeParams.find("Kd", {"texture"}))
                throw PtError(PT_ERR_UNSUPPORTED, "textured Kd is outside the supported subset");
            gs_.materialParams.spectrum("Kd", kd);
            shapeParams.spectrum("Kd", kd);
            float sigma = gs_.materialParams.float1("sigma", 0.f);
            sigma = shapeParams.float1("sigma", sigma);
            if (sigma != 0.f) throw PtError(PT_ERR_UNSUPPORTED, "OrenNayar (sigma != 0) is outside the supported subset");
            m.kd[0] = kd[0]; m.kd[1] = kd[1]; m.kd[2] = kd[2];
            m.sigma = sigma;
        } else if (name == "metal") {
            // CreateMetalMaterial (metal.cpp:113-131).  The default eta/k are
            // the measured copper spectra reduced by FromSampled (metal.cpp:116-122).
            m.kind = PT_MAT_METAL;
            for (const char* tex : {"eta", "k", "roughness", "uroughness", "vroughness", "bumpmap"})
                if (gs_.materialParams.find(tex, {"texture"}) || shapeParams.find(tex, {"texture"}))
                    throw PtError(PT_ERR_UNSUPPORTED, "textured metal parameters are outside the supported subset");
            float eta[3], k[3];
            bool hasEta = gs_.materialParams.spectrum("eta", eta);
            hasEta = shapeParams.spectrum("eta", eta) || hasEta;
            bool hasK = gs_.materialParams.spectrum("k", k);
            hasK = shapeParams.spectrum("k", k) || hasK;
            if (!hasEta) copper_spectrum(false, eta);
            if (!hasK) copper_spectrum(true, k);
            const float rough = f1("roughness", .01f, nullptr, shapeParams);
            bool hu = false, hv = false;
            float ur = f1("uroughness", 0.f, &hu, shapeParams), vr = f1("vroughness", 0.f, &hv, shapeParams);
            if (!hu) ur = rough;
            if (!hv) vr = rough;
            bool remap = gs_.materialParams.bool1("remaproughness", true);
            remap = shapeParams.bool1("remaproughness", remap);
            if (remap) {
                ur = tr_roughness_to_alpha(ur);
                vr = tr_roughness_to_alpha(vr);
            }
            for (int i = 0; i < 3; ++i) { m.eta[i] = eta[i]; m.k[i] = k[i]; }
            m.alpha[0] = std::max(0.001f, ur);  // TrowbridgeReitzDistribution ctor (microfacet.h:109-113)
            m.alpha[1] = std::max(0.001f, vr);
        } else if (name == "glass" || name == "dispersive_glass") {
            // CreateGlassMaterial (glass.cpp:85-100) / CreateDispersiveGlassMaterial
            // (dispersive_glass.cpp:125-143)
            const bool disp = name == "dispersive_glass";
            m.kind = disp ? PT_MAT_DISPERSIVE_GLASS : PT_MAT_GLASS;
            no_textures({"Kr", "Kt", "eta", "index", "etaMin", "etaMax", "indexMin", "indexMax", "uroughness",
                         "vroughness", "bumpmap"}, shapeParams);
            float kr[3] = {1, 1, 1}, kt[3] = {1, 1, 1};
            spectrum2("Kr", kr, shapeParams);
            spectrum2("Kt", kt, shapeParams);
            bool found = false;
            if (disp) {
                m.ior_min = f1("etaMin", 0.f, &found, shapeParams);
                if (!found) m.ior_min = f1("indexMin", 1.5f, nullptr, shapeParams);
                m.ior_max = f1("etaMax", 0.f, &found, shapeParams);
                if (!found) m.ior_max = f1("indexMax", 1.5f, nullptr, shapeParams);
            } else {
                m.ior = f1("eta", 0.f, &found, shapeParams);
                if (!found) m.ior = f1("index", 1.5f, nullptr, shapeParams);
            }
            float ur = f1("uroughness", 0.f, nullptr, shapeParams), vr = f1("vroughness", 0.f, nullptr, shapeParams);
            bool remap = gs_.materialParams.bool1("remaproughness", false);
            remap = shapeParams.bool1("remaproughness", remap);
            m.specular = (ur == 0 && vr == 0) ? 1 : 0;
            // DispersiveGlassMaterial remaps the shared roughness once per
            // wavelength BSDF, cumulatively (dispersive_glass.cpp:91-95), so
            // its four lobes carry four different alphas: not represented.
            if (disp && remap && !m.specular)
                throw PtError(PT_ERR_UNSUPPORTED,
                              "rough dispersive_glass with remaproughness is outside the supported subset");
            if (remap) {
                ur = tr_roughness_to_alpha(ur);
                vr = tr_roughness_to_alpha(vr);
            }
            for (int i = 0; i < 3; ++i) { m.kr[i] = kr[i]; m.kt[i] = kt[i]; }
            m.alpha[0] = std::max(0.001f, ur);
            m.alpha[1] = std::max(0.001f, vr);
        } else if (name == "mirror") {
            // CreateMirrorMaterial (mirror.cpp:54-60)
            m.kind = PT_MAT_MIRROR;
            no_textures({"Kr", "bumpmap"}, shapeParams);
            float kr[3] = {0.9f, 0.9f, 0.9f};
            spectrum2("Kr", kr, shapeParams);
            for (int i = 0; i < 3; ++i) m.kr[i] = kr[i];
        } else if (name == "plastic") {
            // CreatePlasticMaterial (plastic.cpp:72-83)
            m.kind = PT_MAT_PLASTIC;
            no_textures({"Kd", "Ks", "roughness", "bumpmap"}, shapeParams);
            float kd[3] = {0.25f, 0.25f, 0.25f}, ks[3] = {0.25f, 0.25f, 0.25f};
            spectrum2("Kd", kd, shapeParams);
            spectrum2("Ks", ks, shapeParams);
            float rough = f1("roughness", .1f, nullptr, shapeParams);
            bool remap = gs_.materialParams.bool1("remaproughness", true);
            remap = shapeParams.bool1("remaproughness", remap);
            if (remap) rough = tr_roughness_to_alpha(rough);
            for (int i = 0; i < 3; ++i) { m.kd[i] = kd[i]; m.ks[i] = ks[i]; }
            m.alpha[0] = m.alpha[1] = std::max(0.001f, rough);
        } else {
            throw PtError(PT_ERR_UNSUPPORTED, "material \"" + name + "\" is outside the supported subset");
        }
        if (out_->spectral) material_s60(name, shapeParams);
        out_->materials.push_back(m);
        return (int)out_->materials.size() - 1;
    }

    // 60-bin reflectances of a material in a SampledSpectrum scene, with the
    // same parameter precedence and defaults as the RGB values above.
    void material_s60(const std::string& name, const ParamSet& shapeParams) {
        float v[3][60];
        auto fill = [&](int slot, const char* pname, float def) {
            for (int i = 0; i < 60; ++i) v[slot][i] = def;  // Spectrum(def)
            gs_.materialParams.spectrum60(pname, v[slot]);
            shapeParams.spectrum60(pname, v[slot]);
        };
        for (int k = 0; k < 3; ++k) for (int i = 0; i < 60; ++i) v[k][i] = 0.f;
        if (name == "matte") fill(0, "Kd", 0.5f);
        else if (name == "glass" || name == "dispersive_glass") { fill(1, "Kr", 1.f); fill(2, "Kt", 1.f); }
        else if (name == "mirror") fill(1, "Kr", 0.9f);
        else if (name != "" && name != "none")
            throw PtError(PT_ERR_UNSUPPORTED, "material \"" + name + "\" in a SampledSpectrum (hero) scene");
        for (int k = 0; k < 3; ++k) out_->mat_s60.insert(out_->mat_s60.end(), v[k], v[k] + 60);
    }
    void light_s60(const ParamSet& ps, const char* lname, pt_light* L) {
        float Lv[60], sc[60], out[60];
        for (int i = 0; i < 60; ++i) Lv[i] = sc[i] = 1.f;  // Spectrum(1.0) defaults
        ps.spectrum60(lname, Lv);
        ps.spectrum60("scale", sc);
        for (int i = 0; i < 60; ++i) out[i] = Lv[i] * sc[i];
        if (L->kind == PT_LIGHT_INFINITE) {
            // InfiniteAreaLight keeps an RGB map: texel = (L * scale).ToRGBSpectrum() (infinite.cpp:57-61)
            float xyz[3];
            s60_to_xyz(out, xyz);
            xyz_to_rgb(xyz, L->L);
            for (int i = 0; i < 60; ++i) out[i] = 0.f;
        }
        out_->light_s60.insert(out_->light_s60.end(), out, out + 60);
    }

    // CreateTriangleMesh + TriangleMesh ctor (triangle.cpp:55-120): vertices,
    // normals and tangents to world space, one Triangle (and one
    // DiffuseAreaLight, api.cpp MakeShapes) per index triple.
    void add_mesh(const ParamSet& ps, uint32_t oflags, const std::vector<float>& P, const std::vector<float>& Nv,
                  const std::vector<float>& Sv, const std::vector<float>& UVv, const std::vector<int>& idx) {
        const HXF o2w = ctm_;
        const int nv = (int)P.size() / 3;
        if (idx.size() % 3 != 0) throw PtError(PT_ERR_PARSE, "indices not a multiple of 3");
        for (int v : idx)
            if (v < 0 || v >= nv) throw PtError(PT_ERR_PARSE, "trianglemesh index out of range");
        const bool hasN = (int)Nv.size() == 3 * nv, hasS = (int)Sv.size() == 3 * nv, hasUV = (int)UVv.size() == 2 * nv;
        const int base = (int)out_->P.size() / 3;
        for (int i = 0; i < nv; ++i) {
            V3 w = xf_point(to_m4(o2w.m), v3(P[3 * i], P[3 * i + 1], P[3 * i + 2]));  // triangle.cpp:75
            out_->P.push_back(w.x); out_->P.push_back(w.y); out_->P.push_back(w.z);
            V3 n = v3(0, 0, 0), s = v3(0, 0, 0);
            if (hasN) n = xf_normal(to_m4(o2w.mi), v3(Nv[3 * i], Nv[3 * i + 1], Nv[3 * i + 2]));
            if (hasS) s = xf_vector(to_m4(o2w.m), v3(Sv[3 * i], Sv[3 * i + 1], Sv[3 * i + 2]));
            out_->N.push_back(n.x); out_->N.push_back(n.y); out_->N.push_back(n.z);
            out_->S.push_back(s.x); out_->S.push_back(s.y); out_->S.push_back(s.z);
            out_->UV.push_back(hasUV ? UVv[2 * i] : 0.f);
            out_->UV.push_back(hasUV ? UVv[2 * i + 1] : 0.f);
        }
        out_->anyN |= hasN; out_->anyS |= hasS; out_->anyUV |= hasUV;
        const int mat = material_for(ps);
        const uint32_t flags =
            oflags | (hasN ? PT_TRI_HAS_N : 0u) | (hasS ? PT_TRI_HAS_S : 0u) | (hasUV ? PT_TRI_HAS_UV : 0u);
        const int ntri = (int)idx.size() / 3;
        for (int t = 0; t < ntri; ++t) {
            pt_triangle tr{};
            tr.v[0] = base + idx[3 * t]; tr.v[1] = base + idx[3 * t + 1]; tr.v[2] = base + idx[3 * t + 2];
            tr.material = mat;
            tr.area_light = -1;
            tr.flags = flags;
            const int ti = (int)out_->tris.size();
            if (!gs_.areaLight.empty()) {
                if (gs_.areaLight != "diffuse" && gs_.areaLight != "area")
                    throw PtError(PT_ERR_UNSUPPORTED, "area light \"" + gs_.areaLight + "\" on a triangle mesh");
                pt_light L{};
                L.kind = PT_LIGHT_DIFFUSE_AREA;
                diffuse_params(gs_.areaLightParams, &L);
                if (out_->spectral) light_s60(gs_.areaLightParams, "L", &L);
                L.shape = ti;
                L.first_portal = 0; L.n_portals = 0;
                out_->lights.push_back(L);
                tr.area_light = (int)out_->lights.size() - 1;
            }
            out_->tris.push_back(tr);
            out_->prims.push_back(pt_prim{PT_PRIM_TRIANGLE, ti});
        }
    }

    // Error()/Warning() (error.cpp:89-102): print and continue
    static void warn(const std::string& msg) { std::fprintf(stderr, "Error: %s\n", msg.c_str()); }

    void shape(const std::string& name, const ParamSet& ps) {
        if (!inWorld_) throw PtError(PT_ERR_PARSE, "Shape outside WorldBegin");
        const HXF o2w = ctm_;
        const bool ro = gs_.reverseOrientation;
        const bool sh = hxf_swaps_handedness(o2w);
        uint32_t oflags = (ro ? PT_TRI_REVERSE_ORIENTATION : 0u) | (sh ? PT_TRI_SWAPS_HANDEDNESS : 0u);
        if (name == "trianglemesh" || name == "plymesh") {
            if (ps.find("alpha", {"texture", "float"}) || ps.find("shadowalpha", {"texture", "float"}))
                throw PtError(PT_ERR_UNSUPPORTED, "alpha textures are outside the supported subset");
            std::vector<float> P, N, S, UV;
            std::vector<int> idx;
            if (name == "trianglemesh") {
                // CreateTriangleMeshShape (triangle.cpp:911-971): missing indices or P, or an index past the
                // last vertex, is an Error() that yields no shapes (and so no area lights) while the scene
                // goes on; a uv / S / N array of the wrong length is discarded.  Empty arrays ("point P" [])
                // are present with zero values: a mesh of zero triangles.  Counts follow the parser
                // (parser.cpp:523-615): a point / normal / vector array keeps its whole triples, a uv array
                // its whole pairs, and only nvi / 3 triangles are made.
                const Param* pi = ps.find("indices", {"integer"});
                const Param* pp = ps.find("P", {"point"});
                // the reference's lookup order: point2 uv, point2 st, then float uv, float st
                const Param* puv = ps.find("uv", {"point2"});
                if (!puv) puv = ps.find("st", {"point2"});
                if (!puv) puv = ps.find("uv", {"float"});
                if (!puv) puv = ps.find("st", {"float"});
                const int nv = pp ? (int)(pp->nums.size() / 3) : 0;
                const int nuv = puv ? (int)(puv->nums.size() / 2) : 0;
                bool useUV = puv != nullptr && nuv > 0;
                if (useUV && nuv < nv) {
                    warn("Not enough of \"uv\"s for triangle mesh.  Expected " + std::to_string(nv) + ", found " +
                         std::to_string(nuv) + ".  Discarding.");
                    useUV = false;
                }
                if (!pi) { warn("Vertex indices \"indices\" not provided with triangle mesh shape"); return; }
                if (!pp) { warn("Vertex positions \"P\" not provided with triangle mesh shape"); return; }
                const Param* pS = ps.find("S", {"vector"});
                const Param* pn = ps.find("N", {"normal"});
                const bool useS = pS && (int)(pS->nums.size() / 3) == nv;
                const bool useN = pn && (int)(pn->nums.size() / 3) == nv;
                if (pS && !useS) warn("Number of \"S\"s for triangle mesh must match \"P\"s");
                if (pn && !useN) warn("Number of \"N\"s for triangle mesh must match \"P\"s");
                for (double v : pi->nums) {
                    if (int(v) >= nv) {
                        warn("trianglemesh has out of-bounds vertex index " + std::to_string(int(v)) + " (" +
                             std::to_string(nv) + " \"P\" values were given");
                        return;
                    }
                    idx.push_back(int(v));
                }
                idx.resize(idx.size() / 3 * 3);  // CreateTriangleMesh(..., nvi / 3, ...)
                if (idx.empty()) return;           // zero triangles: no shapes
                for (int k = 0; k < 3 * nv; ++k) P.push_back((float)pp->nums[k]);
                if (useN) for (int k = 0; k < 3 * nv; ++k) N.push_back((float)pn->nums[k]);
                if (useS) for (int k = 0; k < 3 * nv; ++k) S.push_back((float)pS->nums[k]);
                if (useUV) for (int k = 0; k < 2 * nv; ++k) UV.push_back((float)puv->nums[k]);
            } else {
                // CreatePLYMesh (plymesh.cpp:107-235); filename relative to the search directory
                std::string f = ps.string1("filename", "");
                if (!f.empty() && f[0] != '/') f = searchDir_ + f;
                PlyMesh m;
                read_ply(f, &m);
                P = std::move(m.P);
                N = std::move(m.N);
                UV = std::move(m.UV);
                idx = std::move(m.idx);
            }
            add_mesh(ps, oflags, P, N, S, UV, idx);
        } else if (name == "loopsubdiv") {
            // CreateLoopSubdiv (loopsubdiv.cpp:400-437): missing data is an
            // Error() that yields no shapes; the mesh carries P and N only
            const int levels = ps.int1("levels", ps.int1("nlevels", 3));
            const Param* pi = ps.find("indices", {"integer"});
            const Param* pp = ps.find("P", {"point"});
            if (!pi) { warn("Vertex indices \"indices\" not provided for LoopSubdiv shape."); return; }
            if (!pp) { warn("Vertex positions \"P\" not provided for LoopSubdiv shape."); return; }
            std::vector<int> idx;
            std::vector<float> P, sP, sN;
            std::vector<int> sIdx;
            for (double v : pi->nums) idx.push_back(int(v));
            for (double v : pp->nums) P.push_back((float)v);
            loop_subdivide(levels, idx, P, &sP, &sN, &sIdx);
            add_mesh(ps, oflags, sP, sN, {}, {}, sIdx);
        } else if (name == "sphere") {
            // CreateSphereShape (sphere.cpp:381-391); the renderer applies the
            // Sphere ctor's clamps (sphere.h:50-59)
            pt_sphere sp{};
            sp.radius = ps.float1("radius", 1.f);
            sp.zmin = ps.float1("zmin", -sp.radius);
            sp.zmax = ps.float1("zmax", sp.radius);
            sp.phimax = ps.float1("phimax", 360.f);
            if (!(sp.radius > 0)) throw PtError(PT_ERR_UNSUPPORTED, "sphere radius must be positive");
            sp.material = material_for(ps);
            sp.area_light = -1;
            sp.flags = oflags;
            store_xf(o2w, &sp.object_to_world);
            const int sidx = (int)out_->spheres.size();
            if (!gs_.areaLight.empty()) {
                if (gs_.areaLight != "diffuse" && gs_.areaLight != "area")
                    throw PtError(PT_ERR_UNSUPPORTED, "area light \"" + gs_.areaLight + "\" on a sphere");
                pt_light L{};
                L.kind = PT_LIGHT_DIFFUSE_SPHERE;
                diffuse_params(gs_.areaLightParams, &L);
                if (out_->spectral) light_s60(gs_.areaLightParams, "L", &L);
                L.shape = sidx;
                out_->lights.push_back(L);
                sp.area_light = (int)out_->lights.size() - 1;
            }
            out_->spheres.push_back(sp);
            out_->prims.push_back(pt_prim{PT_PRIM_SPHERE, sidx});
        } else if (name == "aaplane") {
            // CreateAAPlaneShape (plane.cpp:117-128)
            V3 lo = v3(0, 0, 0), hi = v3(0, 0, 0);
            ps.point3("lo", &lo);
            ps.point3("hi", &hi);
            pt_aaplane pl{};
            pl.lo[0] = lo.x; pl.lo[1] = lo.y; pl.lo[2] = lo.z;
            pl.hi[0] = hi.x; pl.hi[1] = hi.y; pl.hi[2] = hi.z;
            pl.axis = ps.int1("axis", 2);
            if (pl.axis < 0 || pl.axis > 2) throw PtError(PT_ERR_PARSE, "aaplane axis must be 0, 1 or 2");
            pl.material = material_for(ps);
            pl.area_light = -1;
            pl.flags = oflags;
            store_xf(o2w, &pl.object_to_world);
            int pidx = (int)out_->planes.size();
            if (!gs_.areaLight.empty()) {
                pt_light L{};
                if (gs_.areaLight == "portal") {
                    if (out_->spectral)
                        throw PtError(PT_ERR_UNSUPPORTED, "portal lights in a SampledSpectrum (hero) scene");
                    L.kind = PT_LIGHT_PORTAL_AREA;
                    portal_params(gs_.areaLightParams, &L);
                } else if (gs_.areaLight == "diffuse" || gs_.areaLight == "area") {
                    // MakeAreaLight "diffuse" on an AAPlaneShape (api.cpp:768-786, creeper.pbrt:38-49):
                    // a DiffuseAreaLight sampled through Shape::Sample(ref) / Shape::Pdf(ref, wi)
                    // (shape.cpp:56-91) over the plane's own Sample / Intersect (plane.cpp:15-72);
                    // parameters it does not read ("strategy", "portalData") are ignored as the
                    // reference's ParamSet does (unused-parameter warning only)
                    if (out_->spectral)
                        throw PtError(PT_ERR_UNSUPPORTED, "aaplane area lights in a SampledSpectrum (hero) scene");
                    L.kind = PT_LIGHT_DIFFUSE_PLANE;
                    diffuse_params(gs_.areaLightParams, &L);
                    L.first_portal = 0; L.n_portals = 0;
                } else
                    throw PtError(PT_ERR_UNSUPPORTED, "area light \"" + gs_.areaLight + "\"");
                L.shape = pidx;
                out_->lights.push_back(L);
                pl.area_light = (int)out_->lights.size() - 1;
            }
            out_->planes.push_back(pl);
            out_->prims.push_back(pt_prim{PT_PRIM_AAPLANE, pidx});
        } else {
            throw PtError(PT_ERR_UNSUPPORTED, "shape \"" + name + "\" is outside the supported subset");
        }
    }

    // MakeLight (api.cpp) with the CTM as LightToWorld; lights keep
    // declaration order (RenderOptions::lights).
    void light_source(const std::string& name, const ParamSet& ps) {
        if (!inWorld_) throw PtError(PT_ERR_PARSE, "LightSource outside WorldBegin");
        if (name == "infinite" || name == "exinfinite") {
            // CreateInfiniteLight (infinite.cpp:185-196)
            if (!ps.string1("mapname", "").empty())
                throw PtError(PT_ERR_UNSUPPORTED, "infinite light \"mapname\" (image maps) is outside the supported subset");
            pt_light L{};
            L.kind = PT_LIGHT_INFINITE;
            float Lv[3] = {1, 1, 1}, sc[3] = {1, 1, 1};
            ps.spectrum("L", Lv);
            ps.spectrum("scale", sc);
            for (int i = 0; i < 3; ++i) L.L[i] = Lv[i] * sc[i];
            L.n_samples = std::max(1, ps.int1("samples", ps.int1("nsamples", 1)));
            L.shape = -1;
            store_xf(ctm_, &L.light_to_world);
            if (out_->spectral) light_s60(ps, "L", &L);
            out_->lights.push_back(L);
            return;
        }
        if (out_->spectral)
            throw PtError(PT_ERR_UNSUPPORTED, "LightSource \"" + name + "\" in a SampledSpectrum (hero) scene");
        if (name == "point") {
            // CreatePointLight (point.cpp:80-88)
            pt_light L{};
            L.kind = PT_LIGHT_POINT;
            float I[3] = {1, 1, 1}, sc[3] = {1, 1, 1};
            ps.spectrum("I", I);
            ps.spectrum("scale", sc);
            for (int i = 0; i < 3; ++i) L.L[i] = I[i] * sc[i];
            V3 from = v3(0, 0, 0);
            ps.point3("from", &from);
            L.n_samples = std::max(1, ps.int1("samples", ps.int1("nsamples", 1)));
            L.shape = -1;
            store_xf(hxf_mul(hxf_translate(from.x, from.y, from.z), ctm_), &L.light_to_world);
            out_->lights.push_back(L);
            return;
        }
        throw PtError(PT_ERR_UNSUPPORTED, "LightSource \"" + name + "\" is outside the supported subset");
    }

    static void diffuse_params(const ParamSet& ps, pt_light* L) {  // CreateDiffuseAreaLight (diffuse.cpp)
        float Lv[3] = {1, 1, 1}, sc[3] = {1, 1, 1};
        ps.spectrum("L", Lv);
        ps.spectrum("scale", sc);
        for (int i = 0; i < 3; ++i) L->L[i] = Lv[i] * sc[i];
        L->two_sided = ps.bool1("twosided", false) ? 1 : 0;
        L->strategy = PT_PORTAL_LIGHT;
        L->n_samples = std::max(1, ps.int1("samples", ps.int1("nsamples", 1)));  // Light ctor (light.h)
        store_xf(hxf_identity(), &L->light_to_world);
    }

    void portal_params(const ParamSet& ps, pt_light* L) {  // CreateAAPortal (portal_arealight.cpp:245-300)
        diffuse_params(ps, L);
        std::string data = ps.string1("portalData", "");
        std::string st = ps.string1("strategy", "light");
        if (st == "light") L->strategy = PT_PORTAL_LIGHT;
        else if (st == "portal") L->strategy = PT_PORTAL_UNIFORM;
        else if (st == "projection") L->strategy = PT_PORTAL_PROJECTION;
        else throw PtError(PT_ERR_PARSE, "AAPortal strategy unknown: " + st);
        L->first_portal = (int)out_->portals.size();
        L->n_portals = 0;
        // sexpresso::parse(portalData).getChild(0): the first top-level list,
        // whose children are (AA lox loy loz hix hiy hiz axis +|-) entries.
        std::vector<std::vector<std::string>> entries;
        parse_portal_sexpr(data, &entries);
        for (const auto& e : entries) {
            if (e.empty() || e[0] != "AA") continue;
            if (e.size() < 9) throw PtError(PT_ERR_PARSE, "AA portal needs 8 arguments");
            pt_portal p{};
            for (int k = 0; k < 3; ++k) p.lo[k] = std::strtof(e[1 + k].c_str(), nullptr);
            for (int k = 0; k < 3; ++k) p.hi[k] = std::strtof(e[4 + k].c_str(), nullptr);
            p.axis = (int)std::strtol(e[7].c_str(), nullptr, 10);
            p.facing_fw = (e[8] == "+") ? 1 : 0;
            out_->portals.push_back(p);
            L->n_portals++;
        }
        if (L->n_portals > PT_MAX_PORTALS)
            throw PtError(PT_ERR_UNSUPPORTED, "more than PT_MAX_PORTALS (" + std::to_string(PT_MAX_PORTALS) +
                                                  ") portals on one light");
    }

    static void parse_portal_sexpr(const std::string& s, std::vector<std::vector<std::string>>* out) {
        // Minimal s-expression reader for the portalData grammar.
        size_t i = 0;
        auto skip = [&]() { while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i; };
        skip();
        if (i >= s.size()) return;
        if (s[i] != '(')
            throw PtError(PT_ERR_PARSE, "portalData must be a list of portal lists, e.g. \"((AA ...))\"");
        ++i;  // enter the first top-level list
        for (;;) {
            skip();
            if (i >= s.size()) throw PtError(PT_ERR_PARSE, "unterminated portalData");
            if (s[i] == ')') break;
            if (s[i] != '(') throw PtError(PT_ERR_PARSE, "portalData entries must be lists (the reference iterates child lists)");
            ++i;
            std::vector<std::string> e;
            for (;;) {
                skip();
                if (i >= s.size()) throw PtError(PT_ERR_PARSE, "unterminated portal entry");
                if (s[i] == ')') { ++i; break; }
                size_t st = i;
                while (i < s.size() && s[i] != ' ' && s[i] != ')' && s[i] != '(' && s[i] != '\t' && s[i] != '\n') ++i;
                e.push_back(s.substr(st, i - st));
            }
            out->push_back(e);
        }
    }

    void world_end() {
        if (!inWorld_) throw PtError(PT_ERR_PARSE, "WorldEnd without WorldBegin");
        worldEnded_ = true;
        inWorld_ = false;
        pt_scene_desc& d = out_->desc;
        std::memset(&d, 0, sizeof d);
        // Accelerator (bvh.cpp:740-760)
        if (accel_.name != "bvh") throw PtError(PT_ERR_UNSUPPORTED, "accelerator \"" + accel_.name + "\"");
        if (accel_.ps.string1("splitmethod", "sah") != "sah")
            throw PtError(PT_ERR_UNSUPPORTED, "only splitmethod \"sah\" is supported");
        d.bvh_max_prims = accel_.ps.int1("maxnodeprims", 4);
        // Film (film.cpp:213-252)
        if (film_.name != "image") throw PtError(PT_ERR_UNSUPPORTED, "film \"" + film_.name + "\"");
        out_->film_filename = film_.ps.string1("filename", "pbrt.exr");  // CreateFilm (film.cpp:213-225)
        d.film.xres = film_.ps.int1("xresolution", 1280);
        d.film.yres = film_.ps.int1("yresolution", 720);
        d.film.crop[0] = 0; d.film.crop[1] = 1; d.film.crop[2] = 0; d.film.crop[3] = 1;
        if (const Param* cr = film_.ps.floats("cropwindow")) {
            if (cr->nums.size() != 4) throw PtError(PT_ERR_PARSE, "cropwindow needs 4 values");
            float c[4];
            for (int i = 0; i < 4; ++i) c[i] = (float)cr->nums[i];
            auto clamp01 = [](float v) { return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); };
            d.film.crop[0] = clamp01(smin(c[0], c[1]));
            d.film.crop[1] = clamp01(smax(c[0], c[1]));
            d.film.crop[2] = clamp01(smin(c[2], c[3]));
            d.film.crop[3] = clamp01(smax(c[2], c[3]));
        }
        d.film.scale = film_.ps.float1("scale", 1.f);
        d.film.diagonal = film_.ps.float1("diagonal", 35.f);
        d.film.max_sample_luminance = film_.ps.float1("maxsampleluminance", kInf);
        // Filter (filters/box.cpp:43-47, filters/gaussian.cpp)
        if (filter_.name == "box") {
            d.film.filter = PT_FILTER_BOX;
            d.film.filter_radius[0] = filter_.ps.float1("xwidth", 0.5f);
            d.film.filter_radius[1] = filter_.ps.float1("ywidth", 0.5f);
        } else if (filter_.name == "gaussian") {
            d.film.filter = PT_FILTER_GAUSSIAN;
            d.film.filter_radius[0] = filter_.ps.float1("xwidth", 2.f);
            d.film.filter_radius[1] = filter_.ps.float1("ywidth", 2.f);
            d.film.gaussian_alpha = filter_.ps.float1("alpha", 2.f);
        } else
            throw PtError(PT_ERR_UNSUPPORTED, "pixel filter \"" + filter_.name + "\"");
        // Camera (perspective.cpp:236-283)
        if (camera_.name != "perspective") throw PtError(PT_ERR_UNSUPPORTED, "camera \"" + camera_.name + "\"");
        store_xf(cameraToWorld_, &d.camera.camera_to_world);
        d.camera.shutter_open = camera_.ps.float1("shutteropen", 0.f);
        d.camera.shutter_close = camera_.ps.float1("shutterclose", 1.f);
        d.camera.lens_radius = camera_.ps.float1("lensradius", 0.f);
        d.camera.focal_distance = camera_.ps.float1("focaldistance", 1e6f);
        float frame = camera_.ps.float1("frameaspectratio", float(d.film.xres) / float(d.film.yres));
        if (frame > 1.f) {
            d.camera.screen_window[0] = -frame; d.camera.screen_window[1] = frame;
            d.camera.screen_window[2] = -1.f; d.camera.screen_window[3] = 1.f;
        } else {
            d.camera.screen_window[0] = -1.f; d.camera.screen_window[1] = 1.f;
            d.camera.screen_window[2] = -1.f / frame; d.camera.screen_window[3] = 1.f / frame;
        }
        if (const Param* sw = camera_.ps.floats("screenwindow")) {
            if (sw->nums.size() != 4) throw PtError(PT_ERR_PARSE, "screenwindow needs 4 values");
            for (int i = 0; i < 4; ++i) d.camera.screen_window[i] = (float)sw->nums[i];
        }
        float fov = camera_.ps.float1("fov", 90.f);
        float halffov = camera_.ps.float1("halffov", -1.f);
        if (halffov > 0.f) fov = 2.f * halffov;
        d.camera.fov = fov;
        // Sampler (halton.cpp:133-139)
        if (sampler_.name != "halton") throw PtError(PT_ERR_UNSUPPORTED, "sampler \"" + sampler_.name + "\"");
        d.sampler.spp = sampler_.ps.int1("pixelsamples", 16);
        d.sampler.sample_pixel_center = sampler_.ps.bool1("samplepixelcenter", false) ? 1 : 0;
        // Integrator (path.cpp:191-214, directlighting.cpp:86-118)
        std::string lsDefault = "uniform";  // the fork's PathIntegrator default (path.cpp:210-211)
        bool noRR = false;
        if (integrator_.name == "path") {
            d.integrator.kind = PT_INTEGRATOR_PATH;
        } else if (integrator_.name == "mypath") {
            // MyPathIntegrator (mypath.cpp): PathIntegrator::Li without the
            // Russian-roulette block (path.cpp:177-185), default light
            // strategy "spatial" (mypath.cpp:169-170).
            d.integrator.kind = PT_INTEGRATOR_PATH;
            noRR = true;
            lsDefault = "spatial";
        } else if (integrator_.name == "hero_path") {
            d.integrator.kind = PT_INTEGRATOR_HERO_PATH;  // CreateHeroPathIntegrator (hero_path.cpp:192-212)
        } else if (integrator_.name == "hero_path_mis") {
            d.integrator.kind = PT_INTEGRATOR_HERO_PATH_MIS;  // CreateHeroPathMISIntegrator (hero_path_mis.cpp:330-354)
            lsDefault = "spatial";
        } else if (integrator_.name == "directlighting") {
            d.integrator.kind = PT_INTEGRATOR_DIRECT;
            const std::string st = integrator_.ps.string1("strategy", "all");
            if (st == "one") d.integrator.direct_strategy = PT_DIRECT_ONE;
            else {
                if (st != "all")
                    std::fprintf(stderr, "Warning: Strategy \"%s\" for direct lighting unknown. Using \"all\".\n",
                                 st.c_str());
                d.integrator.direct_strategy = PT_DIRECT_ALL;
            }
        } else
            throw PtError(PT_ERR_UNSUPPORTED, "integrator \"" + integrator_.name + "\"");
        d.integrator.max_depth = integrator_.ps.int1("maxdepth", 5);
        d.integrator.rr_threshold = integrator_.ps.float1("rrthreshold", 1.f);
        // no RR: `maxComp(beta * etaScale) < -inf` never holds, so the block never runs
        if (noRR) d.integrator.rr_threshold = -kInf;
        // CreateLightSampleDistribution (lightdistrib.cpp:46-66): one light is always uniform
        std::string ls = integrator_.ps.string1("lightsamplestrategy", lsDefault);
        if (ls == "uniform" || out_->lights.size() == 1) d.integrator.light_strategy = PT_LIGHTS_UNIFORM;
        else if (ls == "power") d.integrator.light_strategy = PT_LIGHTS_POWER;
        else if (d.integrator.kind == PT_INTEGRATOR_HERO_PATH_MIS) {
            if (ls != "spatial")  // unknown names fall back to spatial (lightdistrib.cpp:59-64)
                std::fprintf(stderr, "Error: Light sample distribution type \"%s\" unknown. Using \"spatial\".\n",
                             ls.c_str());
            d.integrator.light_strategy = PT_LIGHTS_SPATIAL;
        } else throw PtError(PT_ERR_UNSUPPORTED, "lightsamplestrategy \"" + ls + "\" with several lights");
        if (const Param* pb = integrator_.ps.find("pixelbounds", {"integer"})) {
            if (pb->nums.size() == 4) {
                d.integrator.has_pixel_bounds = 1;
                for (int i = 0; i < 4; ++i) d.integrator.pixel_bounds[i] = int(pb->nums[i]);
            }
        }
    }
};

}  // namespace

void host_scene_fill_desc(pt_host_scene_impl* hs) {
    pt_scene_desc& d = hs->desc;
    d.n_vertices = (int)hs->P.size() / 3;
    d.P = hs->P.empty() ? nullptr : hs->P.data();
    d.N = hs->anyN ? hs->N.data() : nullptr;
    d.S = hs->anyS ? hs->S.data() : nullptr;
    d.UV = hs->anyUV ? hs->UV.data() : nullptr;
    d.n_triangles = (int)hs->tris.size();
    d.triangles = hs->tris.data();
    d.n_planes = (int)hs->planes.size();
    d.planes = hs->planes.data();
    d.n_prims = (int)hs->prims.size();
    d.prims = hs->prims.data();
    d.n_materials = (int)hs->materials.size();
    d.materials = hs->materials.data();
    d.n_lights = (int)hs->lights.size();
    d.lights = hs->lights.data();
    d.n_portals = (int)hs->portals.size();
    d.portals = hs->portals.data();
    d.n_spheres = (int)hs->spheres.size();
    d.spheres = hs->spheres.data();
    d.spectral = hs->spectral ? 1 : 0;
    d.material_s60 = hs->spectral ? hs->mat_s60.data() : nullptr;
    d.light_s60 = hs->spectral ? hs->light_s60.data() : nullptr;
}

pt_host_scene_impl* load_pbrt_file(const char* path) {
    std::unique_ptr<pt_host_scene_impl> hs(new pt_host_scene_impl);
    Loader ld(hs.get());
    ld.parse_file(path);
    ld.finish();
    host_scene_fill_desc(hs.get());
    return hs.release();
}

const pt_scene_desc* host_scene_desc(const pt_host_scene_impl* hs) { return &hs->desc; }
const char* host_scene_film_filename(const pt_host_scene_impl* hs) { return hs->film_filename.c_str(); }
void host_scene_free(pt_host_scene_impl* hs) { delete hs; }

}  // namespace pt
