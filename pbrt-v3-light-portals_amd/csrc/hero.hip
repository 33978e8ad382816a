// hero.hip -- the hero-wavelength integrators on the device (included by
// render.hip after kernels.hip).
//
// The reference runs hero_path / hero_path_mis only in its SampledSpectrum
// build: every radiance quantity is 60 bins over 400-700 nm and four hero
// wavelengths per camera sample drive dispersion (integrators/hero.cpp,
// hero_path.cpp, hero_path_mis.cpp).  The paths run on the same wavefront as
// PathIntegrator: k_camera + k_hero_init start them, k_trace traces their
// continuation and shadow rays, k_shade_hero advances each by one vertex,
// with the 60-bin throughput / radiance / pending light-sample term in
// bin-major SoA (coalesced across the wave) and the light sample's term added
// by the next step when its shadow ray comes back unoccluded -- the order in
// which the reference adds it.  BSDF values are evaluated with the RGB lobe
// code three bins at a time (every lobe is f = R * scalar), the lobe set being
// chosen from the full 60-bin reflectances; the direction, pdf and lobe type
// are sampled once per vertex.  A finished sample's radiance is copied
// slot-major for k_film_s60, which filters it in the reference's FilmTile
// order.

#pragma once
#include "kernels.hip"

namespace pt {

constexpr int kNS = 60;

// The 60-bin loops over the bin-major state run in groups of kG bins: a
// group's loads are all issued before its stores (the arrays may alias, so
// the compiler cannot move a load above an earlier store itself).
#ifndef PT_HERO_G
#define PT_HERO_G 12
#endif
constexpr int kG = PT_HERO_G;  // 3, 6 or 12 (whole 3-bin chunks)
static_assert(kNS % kG == 0 && kG % 3 == 0, "bin groups hold whole chunks");
// Layout of the per-slot 60-bin state (DevHeroPaths): slot-major (AoS, 240 B
// per slot: a lane's bin group is one contiguous run of 16-byte loads, whatever
// the spread of the slots in the path queue) or bin-major (stride n).
#ifndef PT_HERO_AOS
#define PT_HERO_AOS 1
#endif
constexpr bool kAos = PT_HERO_AOS != 0;
// g: the slot's bin 0; N: the bin stride (1 slot-major, n bin-major)
__device__ __forceinline__ void gload(const float* g, uint32_t N, int i0, float* r) {
    if constexpr (kAos && kG % 4 == 0) {
        const float4* p = reinterpret_cast<const float4*>(g + i0);
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) {
            const float4 v = p[q];
            r[4 * q] = v.x; r[4 * q + 1] = v.y; r[4 * q + 2] = v.z; r[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kG; ++j) r[j] = g[(uint32_t)(i0 + j) * N];
    }
}
__device__ __forceinline__ void gstore(float* g, uint32_t N, int i0, const float* r) {
    if constexpr (kAos && kG % 4 == 0) {
        float4* p = reinterpret_cast<float4*>(g + i0);
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) p[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
    } else {
#pragma unroll
        for (int j = 0; j < kG; ++j) g[(uint32_t)(i0 + j) * N] = r[j];
    }
}

struct DevHero {
    const float* XYZ;        // 3 x 60 CIE matching functions (SampledSpectrum::Init)
    const float* illum;      // 7 x 60 RGB->illuminant basis (W C M Y R G B)
    const float* mat_s60;    // n_materials x 3 x 60
    const int* mat_nb;       // n_materials: bit j = spectrum j is not black (after Clamp)
    const float* light_s60;  // n_lights x 60
    const float* wcdf;       // SpectralDistribution CDF, 61 entries
    // light sample distribution: one (func, cdf, funcInt) per voxel (spatial)
    // or a single one (uniform / power); n_lights + (n_lights + 1) + 1 floats each
    const float* dist;
    int dist_stride;
    int spatial;             // SpatialLightDistribution lookups
    int nv0, nv1, nv2;
    V3 wb_min, wb_max;       // scene.WorldBound()
    int mis;                 // hero_path_mis (else hero_path)
    float* out60;            // per batch slot: the sample's 60-bin radiance
    float* out_y;            // per batch slot: its L.y(), -inf if a bin is NaN (k_film_s60's sanitiser input)
};

__device__ __forceinline__ float s60_y(const DevHero& h, const float* c) {  // spectrum.h:407-413
    float yy = 0.f;
    for (int i = 0; i < kNS; ++i) yy += h.XYZ[kNS + i] * c[i];
    return yy * (float)(700 - 400) / (float)(106.856895f * kNS);
}
// SampledSpectrum::FromRGB(rgb, Illuminant) (spectrum.cpp:136-172), one bin
// at a time: the reference's branch picks three basis spectra (W C M Y R G B)
// and weights; bin i is then its elementwise ops in the same order
struct RgbIllum {
    float a[3];
    int k[3];
};
__device__ __forceinline__ RgbIllum rgb_illum(S3 rgb) {
    const float c0 = rgb.c[0], c1 = rgb.c[1], c2 = rgb.c[2];
    auto mk = [](float a0, int k0, float a1, int k1, float a2, int k2) { return RgbIllum{{a0, a1, a2}, {k0, k1, k2}}; };
    if (c0 <= c1 && c0 <= c2)
        return c1 <= c2 ? mk(c0, 0, c1 - c0, 1, c2 - c1, 6) : mk(c0, 0, c2 - c0, 1, c1 - c2, 5);
    if (c1 <= c0 && c1 <= c2)
        return c0 <= c2 ? mk(c1, 0, c0 - c1, 2, c2 - c0, 6) : mk(c1, 0, c2 - c1, 2, c0 - c2, 4);
    return c0 <= c1 ? mk(c2, 0, c0 - c2, 3, c1 - c0, 5) : mk(c2, 0, c1 - c2, 3, c0 - c1, 4);
}
__device__ __forceinline__ float rgb_illum_bin(const DevHero& h, const RgbIllum& c, int i) {
    float r = 0.f;
    r += h.illum[c.k[0] * kNS + i] * c.a[0];
    r += h.illum[c.k[1] * kNS + i] * c.a[1];
    r += h.illum[c.k[2] * kNS + i] * c.a[2];
    const float v = r * .86445f;
    return v < 0 ? 0.f : (v > kInf ? kInf : v);  // Clamp(0, Infinity)
}
__device__ __forceinline__ void s60_from_rgb_illum(const DevHero& h, S3 rgb, float* r) {
    const RgbIllum c = rgb_illum(rgb);
    for (int i = 0; i < kNS; ++i) r[i] = rgb_illum_bin(h, c, i);
}
__device__ __forceinline__ float s60_y_zero() {  // Spectrum(0).y()
    return 0.f * (float)(700 - 400) / (float)(106.856895f * kNS);
}

// the 60-bin BSDF of a surface: the lobe set from a representative material,
// values per 3-bin chunk from a material copy holding that chunk's reflectances
struct HeroBsdf {
    Bsdf b;    // lobes from a representative material; b.rkd / rkr / rkt hold the current 3-bin chunk
    int mi;
    int kind;  // the representative's kind (dispersive glass -> glass with the hero eta)
};
template <int kFt>
__device__ __forceinline__ void hb_make(const DevScene& sc, const DevHero& h, int mi, const SurfHit& si, float eta,
                                        HeroBsdf* hb) {
    pt_material rep = sc.mats[PT_IDX(mi, sc.n_mats)];  // lobe-selection stand-in
    hb->mi = mi;
    const int nb = h.mat_nb[mi];
    const float one = (nb & 1) ? 1.f : 0.f, r = (nb & 2) ? 1.f : 0.f, t = (nb & 4) ? 1.f : 0.f;
    for (int c = 0; c < 3; ++c) { rep.kd[c] = one; rep.kr[c] = r; rep.kt[c] = t; }
    if (rep.kind == PT_MAT_DISPERSIVE_GLASS) { rep.kind = PT_MAT_GLASS; rep.ior = eta; }
    make_bsdf<kFt>(&rep, si, 550.f, &hb->b);
    hb->b.m = &sc.mats[PT_IDX(mi, sc.n_mats)];  // lobes read only kind / ks / eta / k / alpha through it
    hb->kind = rep.kind;
}
__device__ __forceinline__ void hb_chunk(const DevHero& h, HeroBsdf* hb, int k) {
    const float* ms = h.mat_s60 + (size_t)hb->mi * 3 * kNS;
    hb->b.rkd = s3(ms[3 * k], ms[3 * k + 1], ms[3 * k + 2]);
    hb->b.rkr = s3(ms[kNS + 3 * k], ms[kNS + 3 * k + 1], ms[kNS + 3 * k + 2]);
    hb->b.rkt = s3(ms[2 * kNS + 3 * k], ms[2 * kNS + 3 * k + 1], ms[2 * kNS + 3 * k + 2]);
}
// 12 bins of the spectra the material kind reads (Kd: matte; Kr, Kt: glass;
// Kr: mirror; all three otherwise), as 16-byte loads, and chunk c of them
// written into the material copy.
struct HbGroup {
    float v[3][kG];
};
__device__ __forceinline__ void hb_group(const DevHero& h, const HeroBsdf* hb, int i0, HbGroup* g) {
    const int kind = hb->kind;
    const int use = kind == PT_MAT_MATTE ? 1 : (kind == PT_MAT_GLASS ? 6 : (kind == PT_MAT_MIRROR ? 2 : 7));
    const float* ms = h.mat_s60 + (size_t)hb->mi * 3 * kNS + i0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < kG; ++q) g->v[j][q] = (use >> j & 1) ? ms[j * kNS + q] : 0.f;
}
__device__ __forceinline__ float g_at(const HbGroup& g, int j, int b) { return g.v[j][b]; }
__device__ __forceinline__ void hb_chunk_g(HeroBsdf* hb, const HbGroup& g, int c) {
    hb->b.rkd = s3(g_at(g, 0, 3 * c), g_at(g, 0, 3 * c + 1), g_at(g, 0, 3 * c + 2));
    hb->b.rkr = s3(g_at(g, 1, 3 * c), g_at(g, 1, 3 * c + 1), g_at(g, 1, 3 * c + 2));
    hb->b.rkt = s3(g_at(g, 2, 3 * c), g_at(g, 2, 3 * c + 1), g_at(g, 2, 3 * c + 2));
}
template <int kFt>
__device__ __forceinline__ float hb_f1(const DevHero& h, HeroBsdf* hb, V3 wo, V3 wi, int bin) {
    hb_chunk(h, hb, bin / 3);
    return bsdf_f<kFt>(hb->b, wo, wi, kBxAll).c[bin % 3];
}

// The lobe sum of BSDF::f (reflection.cpp:713-726) for local directions and
// a fixed reflect test, at the chunk the material copy currently holds.
template <int kFt>
__device__ __forceinline__ S3 hb_lobes_f(const Bsdf& b, V3 wo, V3 wi, bool reflect) {
    S3 f = s3(0.f);
    for (int i = 0; i < Ft<kFt>::max_lobes; ++i) {
        if (i >= b.n) break;
        const int k = lobe_at(b, i), t = lobe_type(k);
        if (lobe_matches(k, kBxAll) && ((reflect && (t & kBxR)) || (!reflect && (t & kBxT))))
            f = f + lobe_f<kFt>(b, k, wo, wi);
    }
    return f;
}
// A lobe's value at fixed local directions with the chunk's reflectance
// factored out: f_c = (((clamp0(X)_c * a) * b) * c) / d is the per-channel
// operation chain of lobe_f / lobe_sample (devfuncs.h) for every lobe of the
// hero materials (x * 1 and x / 1 are exact, so shorter chains pad with
// ones).  The direction-only part (D, G, Fresnel, cosines) is computed once
// per vertex instead of once per 3-bin chunk.  src: 0 Kd, 1 Kr, 2 Kt, -1 a
// lobe that returned black.
struct LobeTerm {
    int src;
    float a, b, c, d;
};
struct HbTerms {
    LobeTerm t[2];
    int n;
    bool generic;  // metal / plastic microfacet lobes: evaluate per chunk (hb_lobes_f)
};
__device__ __forceinline__ LobeTerm lobe_term(int src, float a, float b = 1.f, float c = 1.f, float d = 1.f) {
    return LobeTerm{src, a, b, c, d};
}
template <int kFt>
__device__ __forceinline__ LobeTerm lobe_f_term(const Bsdf& b, int k, V3 wo, V3 wi) {  // lobe_f
    const LobeTerm black = lobe_term(-1, 0.f);
    if (k == kLbLambert || !(Ft<kFt>::micro || Ft<kFt>::spec)) return lobe_term(0, kInvPi);
    if (!Ft<kFt>::micro) return black;  // specular lobes: f = 0
    const float ax = b.m->alpha[0], ay = b.m->alpha[1];
    if (k == kLbMfRefl) {  // mfrefl_f, dielectric Fresnel
        const float cosO = fabsf(wo.z), cosI = fabsf(wi.z);
        V3 wh = wi + wo;
        if (cosI == 0 || cosO == 0) return black;
        if (wh.x == 0 && wh.y == 0 && wh.z == 0) return black;
        wh = normalize(wh);
        const V3 whf = dot(wh, v3(0, 0, 1)) < 0.f ? -wh : wh;
        const float F = fr_dielectric(dot(wi, whf), 1.f, b.eta);
        return lobe_term(1, tr_D(ax, ay, wh), tr_G(ax, ay, wo, wi), F, 4 * cosI * cosO);
    }
    if (k == kLbMfTrans) {  // mftrans_f
        if (wo.z * wi.z > 0) return black;
        const float cosO = wo.z, cosI = wi.z;
        if (cosI == 0 || cosO == 0) return black;
        const float eta = wo.z > 0 ? (b.eta / 1.f) : (1.f / b.eta);
        V3 wh = normalize(wo + wi * eta);
        if (wh.z < 0) wh = -wh;
        if (dot(wo, wh) * dot(wi, wh) > 0) return black;
        const float F = fr_dielectric(dot(wo, wh), 1.f, b.eta);
        const float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
        const float factor = 1 / eta;
        const float v = fabsf(tr_D(ax, ay, wh) * tr_G(ax, ay, wo, wi) * eta * eta * absdot(wi, wh) * absdot(wo, wh) *
                              factor * factor / (cosI * cosO * sqrtDenom * sqrtDenom));
        return lobe_term(2, 1.f - F, v);
    }
    return black;
}
// hb_lobes_f's lobe selection, as terms
template <int kFt>
__device__ __forceinline__ HbTerms hb_terms_f(const Bsdf& b, V3 wo, V3 wi, bool reflect) {
    HbTerms T;
    T.n = 0;
    T.generic = Ft<kFt>::micro && (b.m->kind == PT_MAT_METAL || b.m->kind == PT_MAT_PLASTIC);
    auto sel = [&](int k) {
        const int t = lobe_type(k);
        return lobe_matches(k, kBxAll) && ((reflect && (t & kBxR)) || (!reflect && (t & kBxT)));
    };
    // at most two lobes; T.t[] is written at constant indices (no private array)
    const bool s0 = b.n > 0 && sel(b.lk0), s1 = Ft<kFt>::max_lobes > 1 && b.n > 1 && sel(b.lk1);
    if (s0) T.t[0] = lobe_f_term<kFt>(b, b.lk0, wo, wi);
    if (s1) {
        const LobeTerm t1 = lobe_f_term<kFt>(b, b.lk1, wo, wi);
        if (s0) T.t[1] = t1;
        else T.t[0] = t1;
    }
    T.n = (s0 ? 1 : 0) + (s1 ? 1 : 0);
    return T;
}
// the value lobe_sample returned for a sampled specular lobe (local wo, wi;
// `type` = the sampled BxDFType), as one term
template <int kFt>
__device__ __forceinline__ HbTerms hb_terms_spec(const Bsdf& b, int type, V3 wo, V3 wi) {
    HbTerms T;
    T.n = 1;
    T.generic = false;
    const int k = (lobe_type(b.lk0) & kBxSpecular) ? b.lk0 : b.lk1;
    const float az = fabsf(wi.z);
    const bool entering = wo.z > 0;
    const float etaI = entering ? 1.f : b.eta, etaT = entering ? b.eta : 1.f;
    const float ratio = (etaI * etaI) / (etaT * etaT);
    if (k == kLbSpecRefl) T.t[0] = lobe_term(1, 1.f, 1.f, 1.f, az);
    else if (k == kLbSpecReflD) T.t[0] = lobe_term(1, fr_dielectric(wi.z, 1.f, b.eta), 1.f, 1.f, az);
    else if (k == kLbSpecTrans) T.t[0] = lobe_term(2, 1.f - fr_dielectric(wi.z, 1.f, b.eta), ratio, 1.f, az);
    else {  // FresnelSpecular
        const float F = fr_dielectric(wo.z, 1.f, b.eta);
        T.t[0] = (type & kBxT) ? lobe_term(2, 1 - F, ratio, 1.f, az) : lobe_term(1, F, 1.f, 1.f, az);
    }
    return T;
}
// the terms at the chunk the BSDF currently holds, summed as BSDF::f does
__device__ __forceinline__ S3 hb_eval(const HbTerms& T, const Bsdf& b) {
    S3 f = s3(0.f);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (i >= T.n) break;
        const LobeTerm& t = T.t[i];
        if (t.src < 0) { f = f + s3(0.f); continue; }
        const S3 X = clamp0(t.src == 0 ? b.rkd : (t.src == 1 ? b.rkr : b.rkt));
        f = f + (((X * t.a) * t.b) * t.c) / t.d;
    }
    return f;
}

// BSDF::f over all 60 bins: the shading-frame change and the reflect test
// once, the lobe values per 3-bin chunk; out(k, f) receives chunk k.
// bsdf_f(b, woW, wiW, kBxAll) as terms: its frame change, wo.z == 0 test
// (black: no terms) and lobe selection
template <int kFt>
__device__ __forceinline__ HbTerms hb_terms_world(const Bsdf& b, V3 woW, V3 wiW) {
    const V3 wo = w2l(b, woW), wi = w2l(b, wiW);
    HbTerms T = hb_terms_f<kFt>(b, wo, wi, dot(wiW, b.ng) * dot(woW, b.ng) > 0);
    if (wo.z == 0) T.n = 0;
    return T;
}
// one bin of bsdf_f(b, woW, wiW) for the terms of those directions
template <int kFt>
__device__ __forceinline__ float hb_f1_t(const DevHero& h, HeroBsdf* hb, const HbTerms& T, V3 woW, V3 wiW, int bin) {
    hb_chunk(h, hb, bin / 3);
    return (T.generic ? bsdf_f<kFt>(hb->b, woW, wiW, kBxAll) : hb_eval(T, hb->b)).c[bin % 3];
}
template <int kFt, typename Out>
__device__ __forceinline__ void hb_f_all(const DevHero& h, HeroBsdf* hb, const HbTerms& T, V3 woW, V3 wiW, Out out) {
    const Bsdf& b = hb->b;
    #pragma unroll 1
    for (int i0 = 0; i0 < kNS; i0 += kG) {  // out(i0, f) receives bins i0 .. i0 + kG - 1
        float f[kG];
        HbGroup g;
        hb_group(h, hb, i0, &g);
#pragma unroll
        for (int c = 0; c < kG / 3; ++c) {
            hb_chunk_g(hb, g, c);
            const S3 v = T.generic ? bsdf_f<kFt>(b, woW, wiW, kBxAll) : hb_eval(T, b);
            f[3 * c] = v.c[0]; f[3 * c + 1] = v.c[1]; f[3 * c + 2] = v.c[2];
        }
        out(i0, f);
    }
}

// light distribution of a point (lightdistrib.cpp:68-78, 112-175)
__device__ __forceinline__ const float* hero_dist(const DevHero& h, V3 p) {
    if (!h.spatial) return h.dist;
    V3 o = p - h.wb_min;  // Bounds3::Offset
    if (h.wb_max.x > h.wb_min.x) o.x /= h.wb_max.x - h.wb_min.x;
    if (h.wb_max.y > h.wb_min.y) o.y /= h.wb_max.y - h.wb_min.y;
    if (h.wb_max.z > h.wb_min.z) o.z /= h.wb_max.z - h.wb_min.z;
    int a = (int)(o.x * h.nv0), b = (int)(o.y * h.nv1), c = (int)(o.z * h.nv2);
    a = a < 0 ? 0 : (a > h.nv0 - 1 ? h.nv0 - 1 : a);
    b = b < 0 ? 0 : (b > h.nv1 - 1 ? h.nv1 - 1 : b);
    c = c < 0 ? 0 : (c > h.nv2 - 1 ? h.nv2 - 1 : c);
    return h.dist + ((size_t)(a * h.nv1 + b) * h.nv2 + c) * (size_t)h.dist_stride;
}
// Distribution1D::SampleDiscrete (sampling.h:90-101) on (func, cdf, funcInt)
__device__ __forceinline__ int dist_sample(const float* d, int n, float u, float* pdf) {
    const float* cdf = d + n;
    const float funcInt = d[2 * n + 1];
    const int off = find_interval(cdf, n + 1, u);
    *pdf = (funcInt > 0) ? d[off] / (funcInt * n) : 0;
    return off;
}

// the 60-bin radiance of an area light seen from -wi (DiffuseAreaLight::L)
__device__ __forceinline__ void light_L60(const DevHero& h, const DevLight& l, int li, V3 n, V3 w, float* out) {
    const bool vis = l.two_sided || dot(n, w) > 0;
    const float* L = h.light_s60 + (size_t)li * kNS;
    for (int i = 0; i < kNS; ++i) out[i] = vis ? L[i] : 0.f;
}

// Per-slot state of a hero path on the wavefront (kAos: slot-major, else
// bin-major with stride n): the 60-bin throughput, radiance and pending
// light-sample contribution, and the scalars of hero_path*.cpp's loop.
struct DevHeroPaths {
    float* beta;  // 60 n
    float* L;     // 60 n; copied to DevHero::out60 (slot-major, k_film_s60's layout) when the path ends
    float* nee;   // 60 n: SampleEmitterHero's term, added if its shadow ray is unoccluded
    float* hs;    // kHsPad n
};
constexpr int kHsWvl = 0;       // 4: the hero wavelengths
constexpr int kHsPath = 4;      // 4: pathWvlPdf
constexpr int kHsPrev = 8;      // 4: prevPathWvlPdf
constexpr int kHsEtaScale = 12;
constexpr int kHsBsdfPdf = 13;
constexpr int kHsFlags = 14;    // kHf* (uint bits)
constexpr int kHs = 15;
constexpr int kHsPad = 16;  // scalars per slot when slot-major (64 B)
// index of bin / scalar i of a slot
__device__ __forceinline__ size_t hbin_at(uint32_t N, uint32_t slot, int i) {
    return kAos ? (size_t)slot * kNS + i : (size_t)i * N + slot;
}
__device__ __forceinline__ size_t hs_at(uint32_t N, uint32_t slot, int i) {
    return kAos ? (size_t)slot * kHsPad + i : (size_t)i * N + slot;
}
constexpr uint32_t kHfWvlDep = 1u, kHfLastSpec = 2u, kHfPend = 4u;


__device__ __forceinline__ int wvl_index(float w) {  // indexFromWavelength
    const int idx = (int)((w - (float)400) * ((float)kNS / (float)300));
    return idx < kNS - 1 ? idx : kNS - 1;
}
// wvlPdf[b]: 1, or the SpectralDistribution pdf of the bin for the hero bins
__device__ __forceinline__ float wvl_pdf(const DevHero& h, const int* wi, int b) {
    return (wi[0] == b || wi[1] == b || wi[2] == b || wi[3] == b) ? h.wcdf[b + 1] - h.wcdf[b] : 1.f;
}
// t of the closest hit found by the traversal (ray.tMax after BVHAccel::Intersect):
// the hit primitive's own test gives the same t whatever tMax was when it hit
__device__ __forceinline__ float hit_t(const DevScene& sc, int prim, const Ray& ray) {
    const float4 r0 = sc.prims[3 * PT_IDX(prim, sc.n_prims)];
    const float4 r1 = sc.prims[3 * PT_IDX(prim, sc.n_prims) + 1];
    const uint32_t fl = __float_as_uint(r0.w);
    float t = kInf;
    if (fl & kPrimAnalytic) {
        shape_test<true>(sc, fl, __float_as_int(r1.w), ray, &t);
    } else {
        const float4 r2 = sc.prims[3 * PT_IDX(prim, sc.n_prims) + 2];
        tri_hit(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, tri_shear(ray.d), &t);
    }
    return t;
}

// Camera-sample set-up after k_camera: the four hero wavelengths
// (hero.cpp:113-150) and the path state (hero_path.cpp:60-75).
__global__ __launch_bounds__(256) void k_hero_init(DevScene sc, DevHero h, DevPaths ps, DevHeroPaths hp,
                                                   uint32_t total)
#ifdef PT_TU_HERO
{
    const uint32_t N = (uint32_t)ps.n;
    for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < total; slot += gridDim.x * blockDim.x) {
        const float uw = halton_dim(sc, hidx_of(ps, slot), sc.wvl_dim);
        for (int i = 0; i < 4; ++i) {
            // rotateValue: fmod(sample + i / 4, 1.0) in double (hero.cpp:45-47)
            const float s = (float)fmod((double)(uw + (float)i / (float)4), 1.0);
            // SpectralDistribution::sampleWavelength (distr.h:91-101): lower_bound over the CDF
            int k = 0;
            while (k < kNS + 1 && h.wcdf[k] < s) ++k;
            int bin = k - 1;
            bin = bin < 0 ? 0 : (bin > kNS - 1 ? kNS - 1 : bin);
            const float minv = h.wcdf[bin], maxv = h.wcdf[bin + 1], diff = maxv - minv;
            const float alpha = (s - minv) / diff;
            hp.hs[hs_at(N, slot, kHsWvl + i)] = (float)400 + (float)300 * ((alpha + (float)bin) / (float)kNS);
            hp.hs[hs_at(N, slot, kHsPath + i)] = 1.f;
            hp.hs[hs_at(N, slot, kHsPrev + i)] = 1.f;
        }
        hp.hs[hs_at(N, slot, kHsEtaScale)] = 1.f;
        hp.hs[hs_at(N, slot, kHsBsdfPdf)] = 0.f;
        hp.hs[hs_at(N, slot, kHsFlags)] = __uint_as_float(0u);
        for (int b = 0; b < kNS; ++b) {
            hp.beta[hbin_at(N, slot, b)] = 1.f;
            hp.L[hbin_at(N, slot, b)] = 0.f;
        }
    }
}
#else
;
#endif

// One vertex of a hero path (hero_path.cpp:76-189, hero_path_mis.cpp:110-327):
// first the pending light sample of the previous vertex (added if its shadow
// ray came back unoccluded), then the hit of the continuation ray.  Emits the
// shadow ray of SampleEmitterHero and the next continuation ray.
template <int kFt>
__device__ __forceinline__ void hero_step(const DevScene& sc, const DevHero& h, const DevPaths& ps, const DevHeroPaths& hp,
                          uint32_t slot, RayList* rays, bool* overflow, uint32_t* ab) {
    const uint32_t N = (uint32_t)ps.n;
    uint32_t st = *st_word(ps, slot);
    float* Lg = hp.L + hbin_at(N, slot, 0);
    float* Bg = hp.beta + hbin_at(N, slot, 0);
    float* Ng = hp.nee + hbin_at(N, slot, 0);
    float* H = hp.hs + hs_at(N, slot, 0);
    const uint32_t BS = kAos ? 1u : N;  // bin / scalar stride
    uint32_t hf = __float_as_uint(H[kHsFlags * BS]);
    rays->n = 0;
    // algorithmic path-state bytes: each 60-bin array (L, nee, beta) counted
    // once per direction it is touched in this step (tch bits), plus the
    // scalar fields and queue entries
    uint32_t tch = 0, sb = 4 + 4 + 4 + 4 + 4;  // queue entry; st and H flags read and written
    auto count = [&]() { *ab += sb + 4 * kNS * (uint32_t)__builtin_popcount(tch); };
    if (st & kStNee) {
        if (hf & kHfPend) sb += 4;  // hitA
        if ((hf & kHfPend) && *hit_word(ps, slot, kHdHitA) == 0)
            #pragma unroll 1
            for (int i0 = 0; i0 < kNS; i0 += kG) {
                float l[kG], x[kG];
                tch |= 1u, gload(Lg, BS, i0, l);
                tch |= 2u, gload(Ng, BS, i0, x);
#pragma unroll
                for (int j = 0; j < kG; ++j) l[j] += x[j];
                tch |= 8u, gstore(Lg, BS, i0, l);
            }
        st &= ~kStNee;
        hf &= ~kHfPend;
    }
    // the finished sample's radiance, slot-major for the film gather
    auto finish = [&]() {
        // 240 B per slot as 15 float4 stores; y = spectrum.h:407-413 with the
        // bins summed in order, NaN test of hero.cpp:118-140 folded in
        float4* o = reinterpret_cast<float4*>(h.out60 + (size_t)slot * kNS);
        float yy = 0.f;
        bool nan = false;
        #pragma unroll 1
        for (int i0 = 0; i0 < kNS; i0 += kG) {
            float l[kG];
            tch |= 1u, gload(Lg, BS, i0, l);
#pragma unroll
            for (int j = 0; j < kG; ++j) {
                yy += h.XYZ[kNS + i0 + j] * l[j];
                nan |= __builtin_isnan(l[j]);
            }
            if constexpr (kG % 4 == 0) {
#pragma unroll
                for (int j = 0; j < kG; j += 4) o[(i0 + j) / 4] = make_float4(l[j], l[j + 1], l[j + 2], l[j + 3]);
            } else {
#pragma unroll
                for (int j = 0; j < kG; ++j) h.out60[(size_t)slot * kNS + i0 + j] = l[j];
            }
        }
        const float yv = yy * (float)(700 - 400) / (float)(106.856895f * kNS);
        h.out_y[slot] = nan ? -__builtin_inff() : yv;
        sb += 4 * kNS + 4;
    };
    if (!(st & kStCont)) {
        H[kHsFlags * BS] = __uint_as_float(hf);
        *st_word(ps, slot) = st;
        finish();
        count();
        return;
    }
    st &= ~kStCont;
    Dims dm{&sc, hidx_of(ps, slot), (int)(st & kStDimMask), false};
    int bounces = (int)((st >> kStBounceShift) & 0xffu);
    float wvls[4], pathWvlPdf[4], prev[4];
    int wvlIdx[4];
    for (int k = 0; k < 4; ++k) {
        wvls[k] = H[(kHsWvl + k) * BS];
        wvlIdx[k] = wvl_index(wvls[k]);
        pathWvlPdf[k] = H[(kHsPath + k) * BS];
        prev[k] = H[(kHsPrev + k) * BS];
    }
    float etaScale = H[kHsEtaScale * BS], bsdfPdf = H[kHsBsdfPdf * BS];
    bool isWvlDependent = (hf & kHfWvlDep) != 0;
    const bool isLastSpecular = (hf & kHfLastSpec) != 0;
    Ray ray = load_ray(ps.ray, slot, kInf);
    sb += 4 + 56 + 24 + 4;  // hidx, H wavelengths / pdfs / etaScale / bsdfPdf, ray, hit
    const V3 rayO = ray.o;
    const int hpr = *hit_word(ps, slot, kHdHit);
    SurfHit si;
    const bool found = hpr >= 0 && surface_at<Ft<kFt>::sph>(sc, hpr, ray, &si);
    // Lo += beta * Le, weighted (hero_path.cpp:84-104, hero_path_mis.cpp:120-166)
    auto add_emitted = [&](auto Le, float emPdf) {
        const float sw = pathWvlPdf[0] + pathWvlPdf[1] + pathWvlPdf[2] + pathWvlPdf[3];
        const float s = (pathWvlPdf[0] + prev[0] * emPdf) + (pathWvlPdf[1] + prev[1] * emPdf) +
                        (pathWvlPdf[2] + prev[2] * emPdf) + (pathWvlPdf[3] + prev[3] * emPdf);
        const float mwc = bsdfPdf / (bsdfPdf + emPdf);
        #pragma unroll 1
        for (int i0 = 0; i0 < kNS; i0 += kG) {
            float l[kG], bv[kG];
            tch |= 1u, gload(Lg, BS, i0, l);
            tch |= 4u, gload(Bg, BS, i0, bv);
#pragma unroll
            for (int j = 0; j < kG; ++j) {
                const int i = i0 + j;
                if (!h.mis)
                    l[j] += isWvlDependent ? (bv[j] * Le(i)) / (wvl_pdf(h, wvlIdx, i) * sw) : bv[j] * Le(i);
                else if (bounces == 0)
                    l[j] += bv[j] * Le(i);
                else
                    l[j] += (bv[j] * Le(i)) * (isWvlDependent ? 1.0f / (wvl_pdf(h, wvlIdx, i) * s) : mwc);
            }
            tch |= 8u, gstore(Lg, BS, i0, l);
        }
    };
    bool cont = false;
    if (!found) {
        for (int li = 0; Ft<kFt>::inf && li < sc.n_lights; ++li) {
            const DevLight& l = sc.lights[li];
            if (l.kind != PT_LIGHT_INFINITE) continue;
            const RgbIllum ri = rgb_illum(inf_Le(l, ray.d));  // Spectrum(Lmap->Lookup, Illuminant)
            bool black = true;
            for (int i = 0; i < kNS; ++i) black &= rgb_illum_bin(h, ri, i) == 0.f;
            if (black) continue;
            const float emPdf = (h.mis && bounces > 0 && !isLastSpecular) ? inf_pdf_li(l, ray.d) : 0.f;
            add_emitted([&](int i) { return rgb_illum_bin(h, ri, i); }, emPdf);
        }
    } else {
        int mat, light;
        prim_info<Ft<kFt>::sph>(sc, hpr, &mat, &light);
        if (light >= 0) {
            const DevLight& l = sc.lights[PT_IDX(light, sc.n_lights)];
            const bool vis = l.two_sided || dot(si.n, -ray.d) > 0;  // DiffuseAreaLight::L
            const float* Lrow = h.light_s60 + (size_t)light * kNS;
            bool black = true;
            for (int i = 0; i < kNS; ++i) black &= (vis ? Lrow[i] : 0.f) == 0.f;
            if (!black) {
                float emPdf = 0;
                if (h.mis && bounces > 0 && !isLastSpecular) {  // PdfEmitterHero (hero_path_mis.cpp:46-76)
                    const float tHit = hit_t(sc, hpr, ray);
                    emPdf = (tHit * tHit) / (absdot(si.n, si.wo) * l.area);  // it.shape->Area()
                    const float* d = hero_dist(h, rayO);
                    const int nl = sc.n_lights;
                    emPdf = emPdf * (d[light] / (d[2 * nl + 1] * nl));
                }
                add_emitted([&](int i) { return vis ? Lrow[i] : 0.f; }, emPdf);
            }
        }
        const pt_material& M = sc.mats[PT_IDX(mat, sc.n_mats)];
        if (bounces >= sc.max_depth) {
        } else if (M.kind == PT_MAT_NONE) {  // bounces-- ; continue
            store_ray(ps.ray, slot, Ray{offset_ray_origin(si.p, si.perr, si.n, ray.d), ray.d, kInf});
            sb += 24;
            rays->push(slot << 2 | kRayCont);
            cont = true;
        } else {
            const bool disp = M.kind == PT_MAT_DISPERSIVE_GLASS;
            float etas[4] = {M.ior, M.ior, M.ior, M.ior};
            if (disp) {  // one BSDF per wavelength (dispersive_glass.cpp:62-118)
                const float lminsq = (float)(400 * 400), lmaxsq = (float)(700 * 700);
                const float cauchyB = (lminsq * M.ior_max - lmaxsq * M.ior_min) / (lminsq - lmaxsq);
                const float cauchyC = lminsq * (M.ior_max - cauchyB);
                for (int i = 0; i < 4; ++i) etas[i] = cauchyB + cauchyC / (wvls[i] * wvls[i]);
            }
            HeroBsdf hb0;
            hb_make<kFt>(sc, h, mat, si, etas[0], &hb0);
            const bool isectWvlDep = disp && hb0.b.n > 0;
            // f and pdf of the i-th wavelength's BSDF at one bin
            // f and pdf of the i-th wavelength's BSDF at one bin; T0 / pdf0: hb0's
            // terms and pdf at (wo, wi)
            auto f1_pdf = [&](bool perWvl, int i, const HbTerms& T0, float pdf0, V3 wo, V3 wi, int bin, float* pdf) {
                if (!perWvl || i == 0) {
                    *pdf = pdf0;
                    return hb_f1_t<kFt>(h, &hb0, T0, wo, wi, bin);
                }
                HeroBsdf hbi;
                hb_make<kFt>(sc, h, mat, si, etas[i], &hbi);
                const float f = hb_f1<kFt>(h, &hbi, wo, wi, bin);
                *pdf = bsdf_pdf<kFt>(hbi.b, wo, wi, kBxAll);
                return f;
            };
            if (h.mis && bsdf_num<kFt>(hb0.b, kBxNonSpecular) > 0 && sc.n_lights > 0) {
                // SampleEmitterHero (hero_path_mis.cpp:78-108); the shadow ray is
                // traced by the next k_trace and the term added by the next step
                const float* d = hero_dist(h, si.p);
                const int nl = sc.n_lights;
                float lpdf;
                const int li = dist_sample(d, nl, dm.get1(), &lpdf);
                float emPdf = lpdf;
                if (lpdf != 0.f) {
                    const float u0 = dm.get1(), u1 = dm.get1();
                    float epdf = 0;
                    V3 wi = v3(0, 0, 0), sp, sn, spe;
                    const DevLight& l = sc.lights[PT_IDX(li, sc.n_lights)];
                    const S3 Lrgb = area_sample_li<kFt>(sc, l, si, u0, u1, &wi, &epdf, &sp, &sn, &spe);
                    if (epdf != 0.f) {
                        const V3 origin = offset_ray_origin(si.p, si.perr, si.n, sp - si.p);
                        const V3 target = offset_ray_origin(sp, spe, sn, origin - sp);
                        const V3 dd = target - origin;
                        store_ray(ps.rayA, slot, Ray{origin, dd, 1 - kShadowEps});
                        sb += 28;
                        rays->push(slot << 2 | kRayShadow);
                        st |= kStNee;
                        // the term as if unoccluded
                        emPdf = emPdf * epdf;
                        const bool inf = l.kind == PT_LIGHT_INFINITE;
                        const bool vis = inf || l.two_sided || dot(sn, -wi) > 0;
                        const RgbIllum ri = rgb_illum(Lrgb);
                        const float* Lrow = h.light_s60 + (size_t)li * kNS;
                        auto Li = [&](int i) { return (inf ? rgb_illum_bin(h, ri, i) : (vis ? Lrow[i] : 0.f)) / emPdf; };
                        bool haveLi = false;
                        for (int i = 0; i < kNS; ++i) haveLi |= Li(i) != 0.f;
                        if (haveLi && emPdf > 0.f) {
                            const V3 wo = si.wo;
                            const float cosv = absdot(wi, si.sn);
                            const bool depN = isWvlDependent || isectWvlDep;
                            const HbTerms Tn = hb_terms_world<kFt>(hb0.b, wo, wi);
                            const float pdfn = bsdf_pdf<kFt>(hb0.b, wo, wi, kBxAll);
                            const float mwn = depN ? 0.f : emPdf / (emPdf + pdfn);
                            bool fnb = false;  // !IsBlack(f); the term itself when no bin is wavelength-dependent
                            hb_f_all<kFt>(h, &hb0, Tn, wo, wi, [&](int i0, const float* f) {
#pragma unroll
                                for (int j = 0; j < kG; ++j) fnb |= f[j] != 0.f;
                                if (!depN) {
                                    float bv[kG], nv[kG];
                                    tch |= 4u, gload(Bg, BS, i0, bv);
#pragma unroll
                                    for (int j = 0; j < kG; ++j) nv[j] = ((bv[j] * Li(i0 + j)) * (f[j] * cosv)) * mwn;
                                    tch |= 16u, gstore(Ng, BS, i0, nv);
                                }
                            });
                            if (fnb) {
                                if (depN) {
                                    float fv[4], bp[4];
                                    for (int i = 0; i < 4; ++i) fv[i] = f1_pdf(isectWvlDep, i, Tn, pdfn, wo, wi, wvlIdx[i], &bp[i]);
                                    const float s = (pathWvlPdf[0] * emPdf + pathWvlPdf[0] * bp[0]) +
                                                    (pathWvlPdf[1] * emPdf + pathWvlPdf[1] * bp[1]) +
                                                    (pathWvlPdf[2] * emPdf + pathWvlPdf[2] * bp[2]) +
                                                    (pathWvlPdf[3] * emPdf + pathWvlPdf[3] * bp[3]);
                                    #pragma unroll 1
                                    for (int i0 = 0; i0 < kNS; i0 += kG) {
                                        float bv[kG], nv[kG];
                                        tch |= 4u, gload(Bg, BS, i0, bv);
#pragma unroll
                                        for (int j = 0; j < kG; ++j) {
                                            const int b = i0 + j;
                                            float f = 0.0f;  // f[wvlIdx[i]] += f_i, in order
                                            for (int i = 0; i < 4; ++i)
                                                if (wvlIdx[i] == b) f += fv[i];
                                            const float mw = emPdf / (wvl_pdf(h, wvlIdx, b) * s);
                                            nv[j] = ((bv[j] * Li(b)) * (f * cosv)) * mw;
                                        }
                                        tch |= 16u, gstore(Ng, BS, i0, nv);
                                    }
                                }
                                hf |= kHfPend;
                            }
                        }
                    }
                }
            }
            // BSDF sampling (hero_path.cpp:128-189, hero_path_mis.cpp:250-327)
            const V3 wo = -ray.d;
            V3 wi = v3(0, 0, 0);
            int flags = 0;
            const float u0 = dm.get1(), u1 = dm.get1();
            bsdfPdf = 0;
            bool fnb = false, curWvlDep = false, dep = false;
            float keep0 = 0.f;  // f[wvlIdx[0]]
            // the direction, pdf and lobe type do not depend on the reflectances:
            // sample at chunk 0, then only the values of the other chunks (the
            // sampled specular lobe's value, or BSDF::f's lobe sum at the sampled
            // local direction as in BSDF::Sample_f), from the factored terms
            V3 woL = v3(0, 0, 0), wiL = v3(0, 0, 0);
            bool reflectS = false, specS = false;
            {
                hb_chunk(h, &hb0, 0);
                const S3 v0 = bsdf_sample<kFt>(hb0.b, wo, &wi, u0, u1, &bsdfPdf, kBxAll, &flags, &wiL);
                curWvlDep = isectWvlDep && (flags & kBxT);
                dep = isWvlDependent || curWvlDep;
                specS = (flags & kBxSpecular) != 0;
                woL = w2l(hb0.b, wo);
                reflectS = dot(wi, hb0.b.ng) * dot(wo, hb0.b.ng) > 0;
                const HbTerms T = specS ? hb_terms_spec<kFt>(hb0.b, flags, woL, wiL)
                                        : hb_terms_f<kFt>(hb0.b, woL, wiL, reflectS);
                const float cosv = absdot(wi, si.sn);
                #pragma unroll 1
                for (int i0 = 0; bsdfPdf != 0.f && i0 < kNS; i0 += kG) {  // pdf 0: every chunk returns 0
                    float f[kG];
                    HbGroup g;
                    hb_group(h, &hb0, i0, &g);
#pragma unroll
                    for (int c = 0; c < kG / 3; ++c) {
                        const int k = i0 / 3 + c;
                        S3 v = v0;
                        if (k > 0) {
                            hb_chunk_g(&hb0, g, c);
                            v = T.generic ? hb_lobes_f<kFt>(hb0.b, woL, wiL, reflectS) : hb_eval(T, hb0.b);
                        }
                        f[3 * c] = v.c[0]; f[3 * c + 1] = v.c[1]; f[3 * c + 2] = v.c[2];
                    }
#pragma unroll
                    for (int j = 0; j < kG; ++j) {
                        fnb |= f[j] != 0.f;
                        if (i0 + j == wvlIdx[0]) keep0 = f[j];
                    }
                    if (!dep) {  // beta *= f |cos| / pdf (unused if f is black)
                        float bv[kG];
                        tch |= 4u, gload(Bg, BS, i0, bv);
#pragma unroll
                        for (int j = 0; j < kG; ++j) bv[j] *= (f[j] * cosv) / bsdfPdf;
                        tch |= 32u, gstore(Bg, BS, i0, bv);
                    }
                }
            }
            if (fnb && bsdfPdf != 0.f) {
                const float cosv = absdot(wi, si.sn);
                if (dep) {
                    for (int i = 0; i < 4; ++i) prev[i] = pathWvlPdf[i];
                    float fv[4];
                    fv[0] = keep0;  // zeroAllBinsBut(wvlIdx[0])
                    pathWvlPdf[0] *= bsdfPdf;
                    HbTerms Td;
                    Td.n = 0;
                    Td.generic = false;
                    float pdfd = 0.f;
                    if (!curWvlDep) {  // every wavelength takes hb0 at (wo, wi)
                        Td = hb_terms_world<kFt>(hb0.b, wo, wi);
                        pdfd = bsdf_pdf<kFt>(hb0.b, wo, wi, kBxAll);
                    }
                    for (int i = 1; i < 4; ++i) {
                        float p;
                        fv[i] = f1_pdf(curWvlDep, i, Td, pdfd, wo, wi, wvlIdx[i], &p);
                        pathWvlPdf[i] *= p;
                    }
                    #pragma unroll 1
                    for (int i0 = 0; i0 < kNS; i0 += kG) {
                        float bv[kG];
                        tch |= 4u, gload(Bg, BS, i0, bv);
#pragma unroll
                        for (int j = 0; j < kG; ++j) {
                            const int b = i0 + j;
                            float f = b == wvlIdx[0] ? fv[0] : 0.f;
                            for (int i = 1; i < 4; ++i)
                                if (wvlIdx[i] == b) f += fv[i];
                            bv[j] *= f * cosv;
                        }
                        tch |= 32u, gstore(Bg, BS, i0, bv);
                    }
                }
                bool bnb = false;
                for (int i = 0; i < kNS; ++i) bnb |= (tch |= 4u, Bg[i * BS]) != 0.f;
                if (bnb) {
                    ray = Ray{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf};
                    if ((flags & kBxSpecular) && (flags & kBxT)) {
                        const float eta = hb0.b.eta;
                        etaScale *= (dot(wo, si.n) > 0) ? (eta * eta) : 1 / (eta * eta);
                    }
                    float mc = Bg[0] * etaScale;  // beta read above
                    for (int i = 1; i < kNS; ++i) mc = smax(mc, (tch |= 4u, Bg[i * BS]) * etaScale);
                    bool alive = true;
                    if (mc < sc.rr_threshold && bounces > 3) {
                        const float q = smax(0.05f, 1 - mc);
                        if (dm.get1() < q) alive = false;
                        else
                            #pragma unroll 1
                            for (int i0 = 0; i0 < kNS; i0 += kG) {
                                float bv[kG];
                                tch |= 4u, gload(Bg, BS, i0, bv);
#pragma unroll
                                for (int j = 0; j < kG; ++j) bv[j] /= 1 - q;
                                tch |= 32u, gstore(Bg, BS, i0, bv);
                            }
                    }
                    if (alive) {
                        isWvlDependent |= curWvlDep;
                        hf = (hf & ~(kHfWvlDep | kHfLastSpec)) | (isWvlDependent ? kHfWvlDep : 0u) |
                             ((flags & kBxSpecular) ? kHfLastSpec : 0u);
                        store_ray(ps.ray, slot, ray);
                        sb += 24 + 40;  // ray; H pdfs / etaScale / bsdfPdf
                        rays->push(slot << 2 | kRayCont);
                        cont = true;
                        ++bounces;
                        for (int k = 0; k < 4; ++k) {
                            H[(kHsPath + k) * BS] = pathWvlPdf[k];
                            H[(kHsPrev + k) * BS] = prev[k];
                        }
                        H[kHsEtaScale * BS] = etaScale;
                        H[kHsBsdfPdf * BS] = bsdfPdf;
                    }
                }
            }
        }
    }
    if (cont) st |= kStCont;
    if (dm.overflow) { st |= kStDimOverflow; *overflow = true; }
    st = (st & ~(kStDimMask | (0xffu << kStBounceShift))) | (uint32_t)min(dm.dim, (int)kStDimMask) |
         ((uint32_t)(bounces & 0xff) << kStBounceShift);
    H[kHsFlags * BS] = __uint_as_float(hf);
    *st_word(ps, slot) = st;
    if (!(st & (kStCont | kStNee))) finish();
    sb += 4 * (rays->n + ((st & (kStCont | kStNee)) ? 1u : 0u));  // ray / path queue entries written
    count();
}

template <int kFt>
__device__ __forceinline__ void shade_hero_batch(const DevScene& sc, const DevHero& h, const DevPaths& ps,
                                                 const DevHeroPaths& hp, const uint32_t* __restrict__ pq,
                                                 const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
                                                 uint32_t* rq_out_count, uint32_t* pq_out, uint32_t* pq_out_count,
                                                 DevStats* stats) {
    const uint32_t n = *pq_count;
    bool overflow = false;
    PT_WAVEQ(wq);
    uint32_t ab = 0;  // this lane's algorithmic path-state bytes
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        RayList rays;
        bool keep = false;
        uint32_t slot = 0;
        if (i < n) {
            slot = pq[i];
            hero_step<kFt>(sc, h, ps, hp, slot, &rays, &overflow, &ab);
            keep = (*st_word(ps, slot) & (kStCont | kStNee)) != 0;
        }
        wq_push(wq, rays, keep, slot, rq_out_count, rq_out, pq_out);
    }
    wq_flush(wq, rq_out_count, rq_out, pq_out);
    if (overflow) atomicAdd(&stats->dim_overflow, 1ull);
    const unsigned long long abw = wave_sum_u64((unsigned long long)ab);
    if (lane_id() == 0 && abw) atomicAdd(&stats->shade_bytes, abw);
}

// register-budget variants (PT_HERO_WAVES): compiler default, 2 or 4 waves per SIMD
#define PT_HERO_SHADE(name, attr)                                                                                   \
    template <int kFt> __global__ __launch_bounds__(kShadeBlock) attr void name(                                                      \
        DevScene sc, DevHero h, DevPaths ps, DevHeroPaths hp, const uint32_t* __restrict__ pq,                     \
        const uint32_t* __restrict__ pq_count, uint32_t* rq_out, uint32_t* rq_out_count, uint32_t* pq_out,        \
        uint32_t* pq_out_count, DevStats* stats) PT_HERO_BODY
#ifdef PT_TU_HERO
#define PT_HERO_BODY { shade_hero_batch<kFt>(sc, h, ps, hp, pq, pq_count, rq_out, rq_out_count, pq_out, pq_out_count, stats); }
#else
#define PT_HERO_BODY ;
#endif
PT_HERO_SHADE(k_shade_hero, )
PT_HERO_SHADE(k_shade_hero_w2, __attribute__((amdgpu_waves_per_eu(2))))
PT_HERO_SHADE(k_shade_hero_w4, __attribute__((amdgpu_waves_per_eu(4))))
#undef PT_HERO_SHADE
#undef PT_HERO_BODY

// Film for SampledSpectrum samples: k_film's ordered per-pixel gather with a
// 60-bin FilmTile contribSum (lane = bin), converted by ToXYZ at the merge
// (film.h:121-161, film.cpp:117-130, spectrum.h:395-406).
__global__ __launch_bounds__(256) void k_film_s60(DevHero h, DevPaths ps, FilmConsts fc,
                                                  const int* __restrict__ pixslot, int p0, int np, int nsamp, int bx0,
                                                  int by0, int bw, int bh, float4* accum)
#ifdef PT_TU_HERO
{
    const int cw = fc.crop_x1 - fc.crop_x0;
    const int sbw = fc.sb_x1 - fc.sb_x0;
    const int total = bw * bh;
    const int lane = (int)lane_id();
    const int nwaves = (int)(gridDim.x * blockDim.x) >> 6;
    for (int t = (int)(blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < total; t += nwaves) {
        const int tx = bx0 + t % bw, ty = by0 + t / bw;
        const int wy0 = max(ty - fc.win, fc.sb_y0), wy1 = min(ty + fc.win, fc.sb_y1 - 1);
        const int wx0 = max(tx - fc.win, fc.sb_x0), wx1 = min(tx + fc.win, fc.sb_x1 - 1);
        if (wy0 > wy1 || wx0 > wx1) continue;
        const size_t o = (size_t)(ty - fc.crop_y0) * cw + (tx - fc.crop_x0);
        float4 acc = accum[o];
        bool touched = false;
        const int ty0 = (wy0 - fc.sb_y0) >> 4, ty1 = (wy1 - fc.sb_y0) >> 4;
        const int tx0 = (wx0 - fc.sb_x0) >> 4, tx1 = (wx1 - fc.sb_x0) >> 4;
        for (int tr = ty0; tr <= ty1; ++tr) {
            for (int tc = tx0; tc <= tx1; ++tc) {
                const int qy0 = max(wy0, fc.sb_y0 + 16 * tr), qy1 = min(wy1, fc.sb_y0 + 16 * tr + 15);
                const int qx0 = max(wx0, fc.sb_x0 + 16 * tc), qx1 = min(wx1, fc.sb_x0 + 16 * tc + 15);
                float binsum = 0.f, wsum = 0.f;  // lane b < 60 holds contribSum[b]
                bool any = false;
                for (int qy = qy0; qy <= qy1; ++qy) {
                    for (int qx = qx0; qx <= qx1; ++qx) {
                        const int p = pixslot[(qy - fc.sb_y0) * sbw + (qx - fc.sb_x0)] - p0;
                        if (p < 0 || p >= np) continue;
                        for (int c0 = 0; c0 < nsamp; c0 += 64) {
                            const int sl = c0 + lane;
                            bool touch = false;
                            float w = 0.f, k = 1.f;
                            uint32_t slot = 0;
                            if (sl < nsamp) {
                                slot = (uint32_t)p * (uint32_t)nsamp + (uint32_t)sl;
                                const float2 pf = ps.pfilm[slot];
                                const float dx = pf.x - 0.5f, dy = pf.y - 0.5f;
                                const int x0 = (int)ceilf(dx - fc.rx), x1 = (int)floorf(dx + fc.rx) + 1;
                                const int y0 = (int)ceilf(dy - fc.ry), y1 = (int)floorf(dy + fc.ry) + 1;
                                touch = !(tx < x0 || tx >= x1 || ty < y0 || ty >= y1);
                                if (touch) {
                                    // radiance sanitiser (hero.cpp:118-140) and maxSampleLuminance
                                    const float yv = h.out_y[slot];  // -inf: a NaN bin
                                    if ((double)yv < -1e-5 || __builtin_isinf(yv)) k = 0.f;
                                    else if (yv > fc.max_lum) k = fc.max_lum / yv;
                                    else k = 1.f;
                                    const float fxv = fabsf((tx - dx) * fc.inv_rx * 16);
                                    const float fyv = fabsf((ty - dy) * fc.inv_ry * 16);
                                    int ix = (int)floorf(fxv); ix = ix < 15 ? ix : 15;
                                    int iy = (int)floorf(fyv); iy = iy < 15 ? iy : 15;
                                    w = fc.table[iy * 16 + ix];
                                }
                            }
                            uint64_t m = __ballot(touch);
                            if (m) any = true;
                            // touching samples in order, four per round: their loads are
                            // issued together, the sums stay in sample order
                            while (m) {
                                int js[4];
                                float vs[4];
#pragma unroll
                                for (int q = 0; q < 4; ++q) {
                                    js[q] = m ? __ffsll((unsigned long long)m) - 1 : -1;
                                    m &= m - 1;
                                    const uint32_t sj = (uint32_t)__shfl((int)slot, js[q] < 0 ? 0 : js[q]);
                                    vs[q] = (js[q] >= 0 && lane < kNS) ? h.out60[(size_t)sj * kNS + lane] : 0.f;
                                }
#pragma unroll
                                for (int q = 0; q < 4; ++q) {
                                    if (js[q] < 0) break;
                                    const float kj = lane_val(k, js[q]), wj = lane_val(w, js[q]);
                                    if (lane < kNS) {
                                        float v = vs[q];
                                        if (kj == 0.f) v = 0.f;        // L = Spectrum(0.f)
                                        else if (kj != 1.f) v = v * kj;  // L *= maxSampleLuminance / L.y()
                                        binsum += (v * 1.f) * wj;
                                    }
                                    wsum += wj;
                                }
                            }
                        }
                    }
                }
                if (!any) continue;
                // ToXYZ of the tile pixel's contribSum, bins in order
                float x = 0.f, y = 0.f, z = 0.f;
                for (int i = 0; i < kNS; ++i) {
                    const float c = lane_val(binsum, i);
                    x += h.XYZ[i] * c;
                    y += h.XYZ[kNS + i] * c;
                    z += h.XYZ[2 * kNS + i] * c;
                }
                const float scale = (float)(700 - 400) / (float)(106.856895f * kNS);
                acc.x += x * scale;
                acc.y += y * scale;
                acc.z += z * scale;
                acc.w += wsum;
                touched = true;
            }
        }
        if (touched && lane == 0) accum[o] = acc;
    }
}
#else
;
#endif

// k_film_s60 with the source samples staged through LDS.  k_film_s60 reads a
// sample's 240-B radiance once for every film pixel its filter footprint
// reaches (~16 with the 2-pixel Gaussian) and at 128 spp those re-reads miss
// L2 (29 GB per launch against ~2 GB of samples).  Here a block owns an 8x8
// square of film pixels (16 waves, each wave 2x2 of them, lane = bin as in
// k_film_s60) and streams the source pixels its filter windows reach through
// LDS, 128 samples at a time, double-buffered (one barrier per chunk): each
// sample is read from HBM once per block, (8 + 2 win)^2 / 64 times in all.
// Every film pixel still consumes the stream in its own order -- FilmTile by
// FilmTile (tile row, tile column), source pixels in scan order, samples in
// order -- because the block's stream is that order over the union of the
// windows and a film pixel skips what lies outside its own; the per-bin sums,
// the ToXYZ per FilmTile and the merges are k_film_s60's operations in
// k_film_s60's order (bit-identical films).
constexpr int kF60Ch = 128;      // samples per staged chunk
constexpr int kF60MaxWin = 5;    // larger filter windows take k_film_s60
constexpr int kF60List = (8 + 2 * kF60MaxWin) * (8 + 2 * kF60MaxWin);
__global__ __launch_bounds__(1024) void k_film_s60_blk(DevHero h, DevPaths ps, FilmConsts fc,
                                                       const int* __restrict__ pixslot, int p0, int np, int nsamp,
                                                       int bx0, int by0, int bw, int bh, float4* accum)
#ifdef PT_TU_HERO
{
    __shared__ float4 s_v[2][kF60Ch * kNS / 4];  // the chunk's 60-bin radiances, slot-major
    __shared__ float4 s_m[2][kF60Ch];            // dx, dy, sanitiser factor k
    __shared__ int4 s_b[2][kF60Ch];              // the sample's pixel bounds x0, x1, y0, y1 (AddSample)
    __shared__ int s_lp[kF60List], s_lq[kF60List];  // stream: batch pixel, (qy - sb_y0) << 16 | (qx - sb_x0)
    __shared__ float s_tab[256];
    __shared__ int s_n;
    const int tid = (int)threadIdx.x, lane = (int)lane_id();
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nbx = (bw + 7) >> 3;
    const int gx0 = bx0 + ((int)blockIdx.x % nbx) * 8, gy0 = by0 + ((int)blockIdx.x / nbx) * 8;
    const int gx1 = min(gx0 + 7, bx0 + bw - 1), gy1 = min(gy0 + 7, by0 + bh - 1);
    const int rx0 = max(gx0 - fc.win, fc.sb_x0), rx1 = min(gx1 + fc.win, fc.sb_x1 - 1);
    const int ry0 = max(gy0 - fc.win, fc.sb_y0), ry1 = min(gy1 + fc.win, fc.sb_y1 - 1);
    const int sbw = fc.sb_x1 - fc.sb_x0;
    if (tid < 256) s_tab[tid] = fc.table[tid];
    // the stream: source pixels of this batch inside the region, FilmTile by
    // FilmTile, scan order within a tile (wave 0, ballot-compacted)
    if (wid == 0) {
        int n = 0;
        if (rx0 <= rx1 && ry0 <= ry1) {
            for (int tr = (ry0 - fc.sb_y0) >> 4; tr <= (ry1 - fc.sb_y0) >> 4; ++tr) {
                for (int tc = (rx0 - fc.sb_x0) >> 4; tc <= (rx1 - fc.sb_x0) >> 4; ++tc) {
                    const int qy0 = max(ry0, fc.sb_y0 + 16 * tr), qy1 = min(ry1, fc.sb_y0 + 16 * tr + 15);
                    const int qx0 = max(rx0, fc.sb_x0 + 16 * tc), qx1 = min(rx1, fc.sb_x0 + 16 * tc + 15);
                    const int rw = qx1 - qx0 + 1, cnt = rw * (qy1 - qy0 + 1);
                    for (int b = 0; b < cnt; b += 64) {
                        const int k = b + lane;
                        int p = -1, qy = 0, qx = 0;
                        if (k < cnt) {
                            qy = qy0 + k / rw;
                            qx = qx0 + k % rw;
                            p = pixslot[(qy - fc.sb_y0) * sbw + (qx - fc.sb_x0)] - p0;
                        }
                        const bool ok = p >= 0 && p < np;
                        const uint64_t m = __ballot(ok);
                        if (ok) {
                            const int at = n + (int)lanes_below(m);
                            s_lp[at] = p;
                            s_lq[at] = ((qy - fc.sb_y0) << 16) | (qx - fc.sb_x0);  // sb may start below 0
                        }
                        n += __popcll(m);
                    }
                }
            }
        }
        if (lane == 0) s_n = n;
    }
    // this wave's film pixels: 2x2, wave (w & 3, w >> 2) of the 4x4 grid of pairs
    int tx[4], ty[4], wx0[4], wx1[4], wy0[4], wy1[4];
    bool on[4], any[4] = {false, false, false, false}, touched[4] = {false, false, false, false};
    float binsum[4] = {0.f, 0.f, 0.f, 0.f}, wsum[4] = {0.f, 0.f, 0.f, 0.f};
    float4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        tx[j] = gx0 + 2 * (wid & 3) + (j & 1);
        ty[j] = gy0 + 2 * (wid >> 2) + (j >> 1);
        wy0[j] = max(ty[j] - fc.win, fc.sb_y0), wy1[j] = min(ty[j] + fc.win, fc.sb_y1 - 1);
        wx0[j] = max(tx[j] - fc.win, fc.sb_x0), wx1[j] = min(tx[j] + fc.win, fc.sb_x1 - 1);
        on[j] = tx[j] <= gx1 && ty[j] <= gy1 && wy0[j] <= wy1[j] && wx0[j] <= wx1[j];
        acc[j] = on[j] ? accum[(size_t)(ty[j] - fc.crop_y0) * (fc.crop_x1 - fc.crop_x0) + (tx[j] - fc.crop_x0)]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const int n = s_n;
    const int nch = (nsamp + kF60Ch - 1) / kF60Ch;
    const int total = n * nch;
    // staging registers: two float4 of radiance and (threads < 128) one sample's metadata
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, rm = r0;
    int4 rb = make_int4(0, 0, 0, 0);
    auto stage_load = [&](int e) {
        const int i = e / nch, c = e - i * nch;
        const int cnt = min(kF60Ch, nsamp - c * kF60Ch);
        const size_t s0 = (size_t)s_lp[i] * (size_t)nsamp + (size_t)c * kF60Ch;
        const float4* src = reinterpret_cast<const float4*>(h.out60 + s0 * kNS);
        const int nf = cnt * (kNS / 4);
        if (tid < nf) r0 = src[tid];
        if (tid + 1024 < nf) r1 = src[tid + 1024];
        if (tid < cnt) {
            const uint32_t slot = (uint32_t)(s0 + tid);
            const float2 pf = ps.pfilm[slot];
            const float dx = pf.x - 0.5f, dy = pf.y - 0.5f;
            rb = make_int4((int)ceilf(dx - fc.rx), (int)floorf(dx + fc.rx) + 1, (int)ceilf(dy - fc.ry),
                           (int)floorf(dy + fc.ry) + 1);
            // radiance sanitiser (hero.cpp:118-140) and maxSampleLuminance
            const float yv = h.out_y[slot];  // -inf: a NaN bin
            float k;
            if ((double)yv < -1e-5 || __builtin_isinf(yv)) k = 0.f;
            else if (yv > fc.max_lum) k = fc.max_lum / yv;
            else k = 1.f;
            rm = make_float4(dx, dy, k, 0.f);
        }
    };
    auto stage_store = [&](int e, int b) {
        const int i = e / nch, c = e - i * nch;
        const int cnt = min(kF60Ch, nsamp - c * kF60Ch);
        const int nf = cnt * (kNS / 4);
        if (tid < nf) s_v[b][tid] = r0;
        if (tid + 1024 < nf) s_v[b][tid + 1024] = r1;
        if (tid < cnt) {
            s_m[b][tid] = rm;
            s_b[b][tid] = rb;
        }
    };
    // ToXYZ of a film pixel's FilmTile contribSum, merged (k_film_s60's order)
    auto close_tile = [&](int j) {
        if (any[j]) {
            float x = 0.f, y = 0.f, z = 0.f;
            for (int i = 0; i < kNS; ++i) {
                const float c = lane_val(binsum[j], i);
                x += h.XYZ[i] * c;
                y += h.XYZ[kNS + i] * c;
                z += h.XYZ[2 * kNS + i] * c;
            }
            const float scale = (float)(700 - 400) / (float)(106.856895f * kNS);
            acc[j].x += x * scale;
            acc[j].y += y * scale;
            acc[j].z += z * scale;
            acc[j].w += wsum[j];
            touched[j] = true;
        }
        binsum[j] = 0.f;
        wsum[j] = 0.f;
        any[j] = false;
    };
    if (total > 0) {
        stage_load(0);
        stage_store(0, 0);
    }
    __syncthreads();
    int cur_tile = -1;
    for (int e = 0; e < total; ++e) {
        const int b = e & 1;
        if (e + 1 < total) stage_load(e + 1);
        const int i = e / nch, c = e - i * nch;
        const int cnt = min(kF60Ch, nsamp - c * kF60Ch);
        const int q = s_lq[i];
        const int qy = (q >> 16) + fc.sb_y0, qx = (q & 0xffff) + fc.sb_x0;
        const int tile = ((q >> 20) << 16) | ((q & 0xffff) >> 4);
        if (tile != cur_tile) {
#pragma unroll
            for (int j = 0; j < 4; ++j) close_tile(j);
            cur_tile = tile;
        }
        bool need = false;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            need |= on[j] && qx >= wx0[j] && qx <= wx1[j] && qy >= wy0[j] && qy <= wy1[j];
        if (need) {
            float4 mh[2];
            int4 bh2[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int sl = hh * 64 + lane;
                mh[hh] = sl < cnt ? s_m[b][sl] : make_float4(0.f, 0.f, 0.f, 0.f);
                bh2[hh] = sl < cnt ? s_b[b][sl] : make_int4(1, 0, 1, 0);  // empty bounds: no touch
            }
            const float* sv = reinterpret_cast<const float*>(&s_v[b][0]);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!(on[j] && qx >= wx0[j] && qx <= wx1[j] && qy >= wy0[j] && qy <= wy1[j])) continue;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    if (hh * 64 >= cnt) break;
                    const int4 bb = bh2[hh];
                    const bool touch = !(tx[j] < bb.x || tx[j] >= bb.y || ty[j] < bb.z || ty[j] >= bb.w);
                    float w = 0.f;
                    if (touch) {
                        const float dx = mh[hh].x, dy = mh[hh].y;
                        const float fxv = fabsf((tx[j] - dx) * fc.inv_rx * 16);
                        const float fyv = fabsf((ty[j] - dy) * fc.inv_ry * 16);
                        int ix = (int)floorf(fxv); ix = ix < 15 ? ix : 15;
                        int iy = (int)floorf(fyv); iy = iy < 15 ? iy : 15;
                        w = s_tab[iy * 16 + ix];
                    }
                    const float k = mh[hh].z;
                    uint64_t m = __ballot(touch);
                    if (m) any[j] = true;
                    while (m) {
                        int js[4];
                        float vs[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            js[u] = m ? __ffsll((unsigned long long)m) - 1 : -1;
                            m &= m - 1;
                            vs[u] = (js[u] >= 0 && lane < kNS) ? sv[(hh * 64 + js[u]) * kNS + lane] : 0.f;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (js[u] < 0) break;
                            const float kj = lane_val(k, js[u]), wj = lane_val(w, js[u]);
                            if (lane < kNS) {
                                float v = vs[u];
                                if (kj == 0.f) v = 0.f;        // L = Spectrum(0.f)
                                else if (kj != 1.f) v = v * kj;  // L *= maxSampleLuminance / L.y()
                                binsum[j] += (v * 1.f) * wj;
                            }
                            wsum[j] += wj;
                        }
                    }
                }
            }
        }
        if (e + 1 < total) stage_store(e + 1, b ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        close_tile(j);
        if (touched[j] && lane == 0)
            accum[(size_t)(ty[j] - fc.crop_y0) * (fc.crop_x1 - fc.crop_x0) + (tx[j] - fc.crop_x0)] = acc[j];
    }
}
#else
;
#endif

// k_film_s60_sq<F>: the 60-bin film with one wave per F x F square of film
// pixels, each source sample read once per square instead of once per film
// pixel it reaches (k_film_s60: ~16 re-reads with the 2-pixel Gaussian, 36.5 GB
// per C3h launch).  Lane = bin, as in k_film_s60; the square's K = F^2 FilmTile
// contribSums are K registers per lane.  The wave walks the union of the K
// filter windows FilmTile by FilmTile (tile row, tile column), source pixels in
// scan order, samples in order -- every film pixel's own samples are a
// subsequence of that walk, in its own order -- and at each FilmTile's end
// converts each touched contribSum with ToXYZ and merges it (film.cpp:117-130),
// as k_film_s60 does pixel by pixel.  No barrier: the wave loads each sample's
// 240 B itself (four in flight).  A sample adds w = +0 to the film pixels it
// does not reach (the weight is computed branch-free per film pixel): a sum that
// starts at +0 and only ever adds finite values is never -0, so x + (+-0) == x
// bit for bit (the sanitiser zeroes every sample with an infinite or NaN bin).
template <int FX, int FY, int G>  // FX x FY film pixels per wave, G sample loads in flight
__global__ __launch_bounds__(64) void k_film_s60_sq(DevHero h, DevPaths ps, FilmConsts fc,
                                                    const int* __restrict__ pixslot, int p0, int np, int nsamp,
                                                    int bx0, int by0, int bw, int bh, float4* accum)
#ifdef PT_TU_HERO
{
    constexpr int K = FX * FY;
    static_assert(K <= 32, "film pixels of a square fit the anyk bits and the wave");
    __shared__ float s_tab[256];
    const int lane = (int)lane_id();
    for (int i = lane; i < 256; i += 64) s_tab[i] = fc.table[i];
    __syncthreads();
    const int nbx = (bw + FX - 1) / FX;
    const int gx0 = bx0 + ((int)blockIdx.x % nbx) * FX, gy0 = by0 + ((int)blockIdx.x / nbx) * FY;
    const int gx1 = min(gx0 + FX - 1, bx0 + bw - 1), gy1 = min(gy0 + FY - 1, by0 + bh - 1);
    const int rx0 = max(gx0 - fc.win, fc.sb_x0), rx1 = min(gx1 + fc.win, fc.sb_x1 - 1);
    const int ry0 = max(gy0 - fc.win, fc.sb_y0), ry1 = min(gy1 + fc.win, fc.sb_y1 - 1);
    if (rx0 > rx1 || ry0 > ry1) return;
    const int sbw = fc.sb_x1 - fc.sb_x0, cw = fc.crop_x1 - fc.crop_x0;
    // film pixel k of the square is (gx0 + k % FX, gy0 + k / FX); lane k holds its accumulator
    const int myx = gx0 + lane % FX, myy = gy0 + lane / FX;
    const bool myon = lane < K && myx <= gx1 && myy <= gy1;
    float4 acc = myon ? accum[(size_t)(myy - fc.crop_y0) * cw + (myx - fc.crop_x0)] : make_float4(0.f, 0.f, 0.f, 0.f);
    bool touched = false;
    float binsum[K], wsum[K];
#pragma unroll
    for (int k = 0; k < K; ++k) binsum[k] = wsum[k] = 0.f;
    uint32_t anyk = 0;  // film pixels the current FilmTile reached
    for (int tr = (ry0 - fc.sb_y0) >> 4; tr <= (ry1 - fc.sb_y0) >> 4; ++tr) {
        for (int tc = (rx0 - fc.sb_x0) >> 4; tc <= (rx1 - fc.sb_x0) >> 4; ++tc) {
            const int qy0 = max(ry0, fc.sb_y0 + 16 * tr), qy1 = min(ry1, fc.sb_y0 + 16 * tr + 15);
            const int qx0 = max(rx0, fc.sb_x0 + 16 * tc), qx1 = min(rx1, fc.sb_x0 + 16 * tc + 15);
            for (int qy = qy0; qy <= qy1; ++qy) {
                for (int qx = qx0; qx <= qx1; ++qx) {
                    const int p = pixslot[(qy - fc.sb_y0) * sbw + (qx - fc.sb_x0)] - p0;
                    if (p < 0 || p >= np) continue;
                    // the square's film pixels whose window [t - win, t + win] holds q
                    uint32_t wm = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int tx = gx0 + k % FX, ty = gy0 + k / FX;
                        const bool in = tx <= gx1 && ty <= gy1 && qx >= tx - fc.win && qx <= tx + fc.win &&
                                        qy >= ty - fc.win && qy <= ty + fc.win;
                        wm |= in ? 1u << k : 0u;
                    }
                    if (!wm) continue;
                    for (int c0 = 0; c0 < nsamp; c0 += 64) {
                        const int sl = c0 + lane;
                        uint32_t slot = 0;
                        float ks = 1.f, dx = 0.f, dy = 0.f;
                        int x0 = 1, x1 = 0, y0 = 1, y1 = 0;  // empty bounds: no film pixel
                        if (sl < nsamp) {
                            slot = (uint32_t)p * (uint32_t)nsamp + (uint32_t)sl;
                            const float2 pf = ps.pfilm[slot];
                            dx = pf.x - 0.5f;
                            dy = pf.y - 0.5f;
                            x0 = (int)ceilf(dx - fc.rx);
                            x1 = (int)floorf(dx + fc.rx) + 1;
                            y0 = (int)ceilf(dy - fc.ry);
                            y1 = (int)floorf(dy + fc.ry) + 1;
                            // radiance sanitiser (hero.cpp:118-140) and maxSampleLuminance
                            const float yv = h.out_y[slot];  // -inf: a NaN bin
                            if ((double)yv < -1e-5 || __builtin_isinf(yv)) ks = 0.f;
                            else if (yv > fc.max_lum) ks = fc.max_lum / yv;
                        }
                        float wk[K];
                        uint64_t mall = 0;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int tx = gx0 + k % FX, ty = gy0 + k / FX;
                            const bool touch = ((wm >> k) & 1u) && !(tx < x0 || tx >= x1 || ty < y0 || ty >= y1);
                            float w = 0.f;
                            if (touch) {
                                const float fxv = fabsf((tx - dx) * fc.inv_rx * 16);
                                const float fyv = fabsf((ty - dy) * fc.inv_ry * 16);
                                int ix = (int)floorf(fxv); ix = ix < 15 ? ix : 15;
                                int iy = (int)floorf(fyv); iy = iy < 15 ? iy : 15;
                                w = s_tab[iy * 16 + ix];
                            }
                            wk[k] = w;
                            const uint64_t mk = __ballot(touch);
                            anyk |= mk ? 1u << k : 0u;
                            mall |= mk;
                        }
                        // the samples that reach any film pixel of the square, in order, G per round
                        while (mall) {
                            int js[G];
                            float vs[G];
#pragma unroll
                            for (int u = 0; u < G; ++u) {
                                js[u] = mall ? __ffsll((unsigned long long)mall) - 1 : -1;
                                mall &= mall - 1;
                                const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)slot, js[u] < 0 ? 0 : js[u]);
                                vs[u] = (js[u] >= 0 && lane < kNS) ? h.out60[(size_t)sj * kNS + lane] : 0.f;
                            }
#pragma unroll
                            for (int u = 0; u < G; ++u) {
                                if (js[u] < 0) break;
                                const float kj = lane_val(ks, js[u]);
                                float v = vs[u];
                                if (kj == 0.f) v = 0.f;        // L = Spectrum(0.f)
                                else if (kj != 1.f) v = v * kj;  // L *= maxSampleLuminance / L.y()
#pragma unroll
                                for (int k = 0; k < K; ++k) {
                                    const float wj = lane_val(wk[k], js[u]);  // +0 where the sample misses k
                                    binsum[k] += (v * 1.f) * wj;
                                    wsum[k] += wj;
                                }
                            }
                        }
                    }
                }
            }
            // the FilmTile's end: ToXYZ of each reached film pixel's contribSum, merged in tile order
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if ((anyk >> k) & 1u) {
                    float x = 0.f, y = 0.f, z = 0.f;
                    for (int i = 0; i < kNS; ++i) {
                        const float c = lane_val(binsum[k], i);
                        x += h.XYZ[i] * c;
                        y += h.XYZ[kNS + i] * c;
                        z += h.XYZ[2 * kNS + i] * c;
                    }
                    const float scale = (float)(700 - 400) / (float)(106.856895f * kNS);
                    if (lane == k) {
                        acc.x += x * scale;
                        acc.y += y * scale;
                        acc.z += z * scale;
                        acc.w += wsum[k];
                        touched = true;
                    }
                }
                binsum[k] = 0.f;
                wsum[k] = 0.f;
            }
            anyk = 0;
        }
    }
    if (touched && myon) accum[(size_t)(myy - fc.crop_y0) * cw + (myx - fc.crop_x0)] = acc;
}
#else
;
#endif

// SpatialLightDistribution::ComputeDistribution (lightdistrib.cpp:175-236)
// for every voxel: 128 radical-inverse points, each light's Li.y() / pdf,
// floored at 0.001 x the average, as a Distribution1D (sampling.h:65-88).
// `ri` holds RadicalInverse(0..4, i) for i < 128; `light_y` each area
// light's Lemit.y().
__global__ void k_hero_spatial(DevScene sc, DevHero h, const float* __restrict__ ri, const float* __restrict__ light_y,
                               float* dist)
#ifdef PT_TU_HERO
{
    const int nvox = h.nv0 * h.nv1 * h.nv2;
    const int nl = sc.n_lights;
    float tmp[kNS];
    for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nvox; v += gridDim.x * blockDim.x) {
        const int a = v / (h.nv1 * h.nv2), b = (v / h.nv2) % h.nv1, c = v % h.nv2;
        const V3 p0 = v3((float)a / (float)h.nv0, (float)b / (float)h.nv1, (float)c / (float)h.nv2);
        const V3 p1 = v3((float)(a + 1) / (float)h.nv0, (float)(b + 1) / (float)h.nv1, (float)(c + 1) / (float)h.nv2);
        auto lerp3 = [&](V3 t) {
            return v3((1 - t.x) * h.wb_min.x + t.x * h.wb_max.x, (1 - t.y) * h.wb_min.y + t.y * h.wb_max.y,
                      (1 - t.z) * h.wb_min.z + t.z * h.wb_max.z);
        };
        const V3 qa = lerp3(p0), qb = lerp3(p1);
        const V3 vmn = v3(smin(qa.x, qb.x), smin(qa.y, qb.y), smin(qa.z, qb.z));
        const V3 vmx = v3(smax(qa.x, qb.x), smax(qa.y, qb.y), smax(qa.z, qb.z));
        float* d = dist + (size_t)v * h.dist_stride;
        for (int j = 0; j < nl; ++j) d[j] = 0.f;
        for (int i = 0; i < 128; ++i) {
            const V3 t = v3(ri[5 * i], ri[5 * i + 1], ri[5 * i + 2]);
            SurfHit intr{};
            intr.p = v3((1 - t.x) * vmn.x + t.x * vmx.x, (1 - t.y) * vmn.y + t.y * vmx.y,
                        (1 - t.z) * vmn.z + t.z * vmx.z);
            intr.wo = v3(1, 0, 0);
            for (int j = 0; j < nl; ++j) {
                const DevLight& l = sc.lights[j];
                V3 wi, sp, sn, spe;
                float pdf = 0;
                const S3 Lrgb = area_sample_li<kFtAll>(sc, l, intr, ri[5 * i + 3], ri[5 * i + 4], &wi, &pdf, &sp, &sn, &spe);
                if (!(pdf > 0)) continue;
                float y;
                if (l.kind == PT_LIGHT_INFINITE) {
                    s60_from_rgb_illum(h, Lrgb, tmp);
                    y = s60_y(h, tmp);
                } else {
                    y = (l.two_sided || dot(sn, -wi) > 0) ? light_y[j] : s60_y_zero();
                }
                d[j] += y / pdf;
            }
        }
        float sum = 0;
        for (int j = 0; j < nl; ++j) sum += d[j];
        const float avg = sum / (float)(128 * (size_t)nl);
        const float minc = (avg > 0) ? (float)(.001 * (double)avg) : 1.f;
        for (int j = 0; j < nl; ++j) d[j] = d[j] < minc ? minc : d[j];
        float* cdf = d + nl;  // Distribution1D ctor
        cdf[0] = 0;
        for (int j = 1; j < nl + 1; ++j) cdf[j] = cdf[j - 1] + d[j - 1] / nl;
        const float funcInt = cdf[nl];
        if (funcInt == 0) for (int j = 1; j < nl + 1; ++j) cdf[j] = (float)j / (float)nl;
        else for (int j = 1; j < nl + 1; ++j) cdf[j] /= funcInt;
        d[2 * nl + 1] = funcInt;
    }
}
#else
;
#endif

}  // namespace pt
