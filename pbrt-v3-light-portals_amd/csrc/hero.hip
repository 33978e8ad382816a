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
constexpr int kG = 12;
__device__ __forceinline__ void gload(const float* g, uint32_t N, int i0, float* r) {
#pragma unroll
    for (int j = 0; j < kG; ++j) r[j] = g[(uint32_t)(i0 + j) * N];
}
__device__ __forceinline__ void gstore(float* g, uint32_t N, int i0, const float* r) {
#pragma unroll
    for (int j = 0; j < kG; ++j) g[(uint32_t)(i0 + j) * N] = r[j];
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
};

__device__ __forceinline__ float s60_y(const DevHero& h, const float* c) {  // spectrum.h:407-413
    float yy = 0.f;
    for (int i = 0; i < kNS; ++i) yy += h.XYZ[kNS + i] * c[i];
    return yy * (float)(700 - 400) / (float)(106.856895f * kNS);
}
// SampledSpectrum::FromRGB(rgb, Illuminant) (spectrum.cpp:136-172)
__device__ __forceinline__ void s60_from_rgb_illum(const DevHero& h, S3 rgb, float* r) {
    for (int i = 0; i < kNS; ++i) r[i] = 0.f;
    auto add = [&](float a, int k) {
        for (int i = 0; i < kNS; ++i) r[i] += h.illum[k * kNS + i] * a;
    };
    const float c0 = rgb.c[0], c1 = rgb.c[1], c2 = rgb.c[2];
    if (c0 <= c1 && c0 <= c2) {
        add(c0, 0);
        if (c1 <= c2) { add(c1 - c0, 1); add(c2 - c1, 6); }
        else { add(c2 - c0, 1); add(c1 - c2, 5); }
    } else if (c1 <= c0 && c1 <= c2) {
        add(c1, 0);
        if (c0 <= c2) { add(c0 - c1, 2); add(c2 - c0, 6); }
        else { add(c2 - c1, 2); add(c0 - c2, 4); }
    } else {
        add(c2, 0);
        if (c0 <= c1) { add(c0 - c2, 3); add(c1 - c0, 5); }
        else { add(c1 - c2, 3); add(c0 - c1, 4); }
    }
    for (int i = 0; i < kNS; ++i) {
        float v = r[i] * .86445f;
        r[i] = v < 0 ? 0.f : (v > kInf ? kInf : v);  // Clamp(0, Infinity)
    }
}
__device__ __forceinline__ float s60_y_zero() {  // Spectrum(0).y()
    return 0.f * (float)(700 - 400) / (float)(106.856895f * kNS);
}
__device__ __forceinline__ bool s60_black(const float* c) {
    for (int i = 0; i < kNS; ++i)
        if (c[i] != 0.f) return false;
    return true;
}

// the 60-bin BSDF of a surface: the lobe set from a representative material,
// values per 3-bin chunk from a material copy holding that chunk's reflectances
struct HeroBsdf {
    Bsdf b;
    pt_material rep;  // lobe-selection stand-in; chunk values are written into it
    int mi;
};
__device__ __forceinline__ void hb_make(const DevScene& sc, const DevHero& h, int mi, const SurfHit& si, float eta,
                                        HeroBsdf* hb) {
    hb->rep = sc.mats[PT_IDX(mi, sc.n_mats)];
    hb->mi = mi;
    const int nb = h.mat_nb[mi];
    const float one = (nb & 1) ? 1.f : 0.f, r = (nb & 2) ? 1.f : 0.f, t = (nb & 4) ? 1.f : 0.f;
    for (int c = 0; c < 3; ++c) { hb->rep.kd[c] = one; hb->rep.kr[c] = r; hb->rep.kt[c] = t; }
    if (hb->rep.kind == PT_MAT_DISPERSIVE_GLASS) { hb->rep.kind = PT_MAT_GLASS; hb->rep.ior = eta; }
    make_bsdf<kFtAll>(&hb->rep, si, 550.f, &hb->b);
    hb->b.m = &hb->rep;
}
__device__ __forceinline__ void hb_chunk(const DevHero& h, HeroBsdf* hb, int k) {
    const float* ms = h.mat_s60 + (size_t)hb->mi * 3 * kNS;
    for (int c = 0; c < 3; ++c) {
        hb->rep.kd[c] = ms[3 * k + c];
        hb->rep.kr[c] = ms[kNS + 3 * k + c];
        hb->rep.kt[c] = ms[2 * kNS + 3 * k + c];
    }
}
__device__ __forceinline__ void hb_f(const DevHero& h, HeroBsdf* hb, V3 wo, V3 wi, float* f) {
    for (int k = 0; k < kNS / 3; ++k) {
        hb_chunk(h, hb, k);
        const S3 v = bsdf_f<kFtAll>(hb->b, wo, wi, kBxAll);
        f[3 * k] = v.c[0]; f[3 * k + 1] = v.c[1]; f[3 * k + 2] = v.c[2];
    }
}
// 12 bins of the spectra the material kind reads (Kd: matte; Kr, Kt: glass;
// Kr: mirror; all three otherwise), as 16-byte loads, and chunk c of them
// written into the material copy.
struct HbGroup {
    float4 v[3][kG / 4];
};
__device__ __forceinline__ void hb_group(const DevHero& h, const HeroBsdf* hb, int i0, HbGroup* g) {
    const int kind = hb->rep.kind;
    const int use = kind == PT_MAT_MATTE ? 1 : (kind == PT_MAT_GLASS ? 6 : (kind == PT_MAT_MIRROR ? 2 : 7));
    const float4* ms = (const float4*)(h.mat_s60 + (size_t)hb->mi * 3 * kNS + i0);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) g->v[j][q] = (use >> j & 1) ? ms[j * kNS / 4 + q] : make_float4(0, 0, 0, 0);
}
__device__ __forceinline__ float g_at(const HbGroup& g, int j, int b) {
    const float4 v = g.v[j][b / 4];
    const int r = b % 4;
    return r == 0 ? v.x : (r == 1 ? v.y : (r == 2 ? v.z : v.w));
}
__device__ __forceinline__ void hb_chunk_g(HeroBsdf* hb, const HbGroup& g, int c) {
    for (int q = 0; q < 3; ++q) {
        hb->rep.kd[q] = g_at(g, 0, 3 * c + q);
        hb->rep.kr[q] = g_at(g, 1, 3 * c + q);
        hb->rep.kt[q] = g_at(g, 2, 3 * c + q);
    }
}
__device__ __forceinline__ float hb_f1(const DevHero& h, HeroBsdf* hb, V3 wo, V3 wi, int bin) {
    hb_chunk(h, hb, bin / 3);
    return bsdf_f<kFtAll>(hb->b, wo, wi, kBxAll).c[bin % 3];
}

// The lobe sum of BSDF::f (reflection.cpp:713-726) for local directions and
// a fixed reflect test, at the chunk the material copy currently holds.
__device__ __forceinline__ S3 hb_lobes_f(const Bsdf& b, V3 wo, V3 wi, bool reflect) {
    S3 f = s3(0.f);
    for (int i = 0; i < Ft<kFtAll>::max_lobes; ++i) {
        if (i >= b.n) break;
        const int k = lobe_at(b, i), t = lobe_type(k);
        if (lobe_matches(k, kBxAll) && ((reflect && (t & kBxR)) || (!reflect && (t & kBxT))))
            f = f + lobe_f<kFtAll>(b, k, wo, wi);
    }
    return f;
}
// BSDF::f over all 60 bins: the shading-frame change and the reflect test
// once, the lobe values per 3-bin chunk; out(k, f) receives chunk k.
template <typename Out>
__device__ __forceinline__ void hb_f_all(const DevHero& h, HeroBsdf* hb, V3 woW, V3 wiW, Out out) {
    const Bsdf& b = hb->b;
    const V3 wo = w2l(b, woW), wi = w2l(b, wiW);
    const bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    for (int i0 = 0; i0 < kNS; i0 += kG) {  // out(i0, f) receives bins i0 .. i0 + kG - 1
        float f[kG];
        HbGroup g;
        hb_group(h, hb, i0, &g);
#pragma unroll
        for (int c = 0; c < kG / 3; ++c) {
            hb_chunk_g(hb, g, c);
            const S3 v = wo.z == 0 ? s3(0.f) : hb_lobes_f(b, wo, wi, reflect);
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

// Per-slot state of a hero path on the wavefront (bin-major SoA, stride n):
// the 60-bin throughput, radiance and pending light-sample contribution, and
// the scalars of hero_path*.cpp's loop.
struct DevHeroPaths {
    float* beta;  // 60 n
    float* L;     // 60 n; copied to DevHero::out60 (slot-major, k_film_s60's layout) when the path ends
    float* nee;   // 60 n: SampleEmitterHero's term, added if its shadow ray is unoccluded
    float* hs;    // kHs n
};
constexpr int kHsWvl = 0;       // 4: the hero wavelengths
constexpr int kHsPath = 4;      // 4: pathWvlPdf
constexpr int kHsPrev = 8;      // 4: prevPathWvlPdf
constexpr int kHsEtaScale = 12;
constexpr int kHsBsdfPdf = 13;
constexpr int kHsFlags = 14;    // kHf* (uint bits)
constexpr int kHs = 15;
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
        const float uw = halton_dim(sc, ps.hidx[slot], sc.wvl_dim);
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
            hp.hs[(kHsWvl + i) * N + slot] = (float)400 + (float)300 * ((alpha + (float)bin) / (float)kNS);
            hp.hs[(kHsPath + i) * N + slot] = 1.f;
            hp.hs[(kHsPrev + i) * N + slot] = 1.f;
        }
        hp.hs[kHsEtaScale * N + slot] = 1.f;
        hp.hs[kHsBsdfPdf * N + slot] = 0.f;
        hp.hs[kHsFlags * N + slot] = __uint_as_float(0u);
        for (int b = 0; b < kNS; ++b) {
            hp.beta[b * N + slot] = 1.f;
            hp.L[b * N + slot] = 0.f;
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
__device__ __forceinline__ void hero_step(const DevScene& sc, const DevHero& h, const DevPaths& ps, const DevHeroPaths& hp,
                          uint32_t slot, uint32_t* rays, uint32_t* nrays, bool* overflow) {
    const uint32_t N = (uint32_t)ps.n;
    uint32_t st = ps.st[slot];
    float* Lg = hp.L + slot;
    float* Bg = hp.beta + slot;
    float* Ng = hp.nee + slot;
    float* H = hp.hs + slot;
    uint32_t hf = __float_as_uint(H[kHsFlags * N]);
    *nrays = 0;
    if (st & kStNee) {
        if ((hf & kHfPend) && ps.hitA[slot] == 0)
            for (int i0 = 0; i0 < kNS; i0 += kG) {
                float l[kG], x[kG];
                gload(Lg, N, i0, l);
                gload(Ng, N, i0, x);
#pragma unroll
                for (int j = 0; j < kG; ++j) l[j] += x[j];
                gstore(Lg, N, i0, l);
            }
        st &= ~kStNee;
        hf &= ~kHfPend;
    }
    // the finished sample's radiance, slot-major for the film gather
    auto finish = [&]() {
        float* o = h.out60 + (size_t)slot * kNS;
        for (int i0 = 0; i0 < kNS; i0 += kG) {
            float l[kG];
            gload(Lg, N, i0, l);
#pragma unroll
            for (int j = 0; j < kG; ++j) o[i0 + j] = l[j];
        }
    };
    if (!(st & kStCont)) {
        H[kHsFlags * N] = __uint_as_float(hf);
        ps.st[slot] = st;
        finish();
        return;
    }
    st &= ~kStCont;
    Dims dm{&sc, ps.hidx[slot], (int)(st & kStDimMask), false};
    int bounces = (int)((st >> kStBounceShift) & 0xffu);
    float wvls[4], pathWvlPdf[4], prev[4];
    int wvlIdx[4];
    for (int k = 0; k < 4; ++k) {
        wvls[k] = H[(kHsWvl + k) * N];
        wvlIdx[k] = wvl_index(wvls[k]);
        pathWvlPdf[k] = H[(kHsPath + k) * N];
        prev[k] = H[(kHsPrev + k) * N];
    }
    float etaScale = H[kHsEtaScale * N], bsdfPdf = H[kHsBsdfPdf * N];
    bool isWvlDependent = (hf & kHfWvlDep) != 0;
    const bool isLastSpecular = (hf & kHfLastSpec) != 0;
    Ray ray = load_ray6(ps.ray, N, slot, kInf);
    const V3 rayO = ray.o;
    const int hpr = ps.hit[slot];
    SurfHit si;
    const bool found = hpr >= 0 && surface_at<true>(sc, hpr, ray, &si);
    float tmp[kNS];  // infinite lights' FromRGB(Illuminant) radiance
    // Lo += beta * Le, weighted (hero_path.cpp:84-104, hero_path_mis.cpp:120-166)
    auto add_emitted = [&](auto Le, float emPdf) {
        const float sw = pathWvlPdf[0] + pathWvlPdf[1] + pathWvlPdf[2] + pathWvlPdf[3];
        const float s = (pathWvlPdf[0] + prev[0] * emPdf) + (pathWvlPdf[1] + prev[1] * emPdf) +
                        (pathWvlPdf[2] + prev[2] * emPdf) + (pathWvlPdf[3] + prev[3] * emPdf);
        const float mwc = bsdfPdf / (bsdfPdf + emPdf);
        for (int i0 = 0; i0 < kNS; i0 += kG) {
            float l[kG], bv[kG];
            gload(Lg, N, i0, l);
            gload(Bg, N, i0, bv);
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
            gstore(Lg, N, i0, l);
        }
    };
    bool cont = false;
    if (!found) {
        for (int li = 0; li < sc.n_lights; ++li) {
            const DevLight& l = sc.lights[li];
            if (l.kind != PT_LIGHT_INFINITE) continue;
            s60_from_rgb_illum(h, inf_Le(l, ray.d), tmp);  // Spectrum(Lmap->Lookup, Illuminant)
            if (s60_black(tmp)) continue;
            const float emPdf = (h.mis && bounces > 0 && !isLastSpecular) ? inf_pdf_li(l, ray.d) : 0.f;
            add_emitted([&](int i) { return tmp[i]; }, emPdf);
        }
    } else {
        int mat, light;
        prim_info<true>(sc, hpr, &mat, &light);
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
            store_ray6(ps.ray, N, slot, Ray{offset_ray_origin(si.p, si.perr, si.n, ray.d), ray.d, kInf});
            rays[(*nrays)++] = slot << 2 | kRayCont;
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
            hb_make(sc, h, mat, si, etas[0], &hb0);
            const bool isectWvlDep = disp && hb0.b.n > 0;
            // f and pdf of the i-th wavelength's BSDF at one bin
            auto f1_pdf = [&](bool perWvl, int i, V3 wo, V3 wi, int bin, float* pdf) {
                if (!perWvl || i == 0) {
                    const float f = hb_f1(h, &hb0, wo, wi, bin);
                    *pdf = bsdf_pdf<kFtAll>(hb0.b, wo, wi, kBxAll);
                    return f;
                }
                HeroBsdf hbi;
                hb_make(sc, h, mat, si, etas[i], &hbi);
                const float f = hb_f1(h, &hbi, wo, wi, bin);
                *pdf = bsdf_pdf<kFtAll>(hbi.b, wo, wi, kBxAll);
                return f;
            };
            if (h.mis && bsdf_num<kFtAll>(hb0.b, kBxNonSpecular) > 0 && sc.n_lights > 0) {
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
                    const S3 Lrgb = area_sample_li<kFtAll>(sc, l, si, u0, u1, &wi, &epdf, &sp, &sn, &spe);
                    if (epdf != 0.f) {
                        const V3 origin = offset_ray_origin(si.p, si.perr, si.n, sp - si.p);
                        const V3 target = offset_ray_origin(sp, spe, sn, origin - sp);
                        const V3 dd = target - origin;
                        float* a = ps.rayA;
                        a[slot] = origin.x; a[N + slot] = origin.y; a[2 * N + slot] = origin.z;
                        a[3 * N + slot] = dd.x; a[4 * N + slot] = dd.y; a[5 * N + slot] = dd.z;
                        a[6 * N + slot] = 1 - kShadowEps;
                        rays[(*nrays)++] = slot << 2 | kRayShadow;
                        st |= kStNee;
                        // the term as if unoccluded
                        emPdf = emPdf * epdf;
                        const bool inf = l.kind == PT_LIGHT_INFINITE;
                        const bool vis = inf || l.two_sided || dot(sn, -wi) > 0;
                        if (inf) s60_from_rgb_illum(h, Lrgb, tmp);
                        const float* Lrow = h.light_s60 + (size_t)li * kNS;
                        auto Li = [&](int i) { return (inf ? tmp[i] : (vis ? Lrow[i] : 0.f)) / emPdf; };
                        bool haveLi = false;
                        for (int i = 0; i < kNS; ++i) haveLi |= Li(i) != 0.f;
                        if (haveLi && emPdf > 0.f) {
                            const V3 wo = si.wo;
                            const float cosv = absdot(wi, si.sn);
                            const bool depN = isWvlDependent || isectWvlDep;
                            const float mwn = depN ? 0.f : emPdf / (emPdf + bsdf_pdf<kFtAll>(hb0.b, wo, wi, kBxAll));
                            bool fnb = false;  // !IsBlack(f); the term itself when no bin is wavelength-dependent
                            hb_f_all(h, &hb0, wo, wi, [&](int i0, const float* f) {
#pragma unroll
                                for (int j = 0; j < kG; ++j) fnb |= f[j] != 0.f;
                                if (!depN) {
                                    float bv[kG], nv[kG];
                                    gload(Bg, N, i0, bv);
#pragma unroll
                                    for (int j = 0; j < kG; ++j) nv[j] = ((bv[j] * Li(i0 + j)) * (f[j] * cosv)) * mwn;
                                    gstore(Ng, N, i0, nv);
                                }
                            });
                            if (fnb) {
                                if (depN) {
                                    float fv[4], bp[4];
                                    for (int i = 0; i < 4; ++i) fv[i] = f1_pdf(isectWvlDep, i, wo, wi, wvlIdx[i], &bp[i]);
                                    const float s = (pathWvlPdf[0] * emPdf + pathWvlPdf[0] * bp[0]) +
                                                    (pathWvlPdf[1] * emPdf + pathWvlPdf[1] * bp[1]) +
                                                    (pathWvlPdf[2] * emPdf + pathWvlPdf[2] * bp[2]) +
                                                    (pathWvlPdf[3] * emPdf + pathWvlPdf[3] * bp[3]);
                                    for (int i0 = 0; i0 < kNS; i0 += kG) {
                                        float bv[kG], nv[kG];
                                        gload(Bg, N, i0, bv);
#pragma unroll
                                        for (int j = 0; j < kG; ++j) {
                                            const int b = i0 + j;
                                            float f = 0.0f;  // f[wvlIdx[i]] += f_i, in order
                                            for (int i = 0; i < 4; ++i)
                                                if (wvlIdx[i] == b) f += fv[i];
                                            const float mw = emPdf / (wvl_pdf(h, wvlIdx, b) * s);
                                            nv[j] = ((bv[j] * Li(b)) * (f * cosv)) * mw;
                                        }
                                        gstore(Ng, N, i0, nv);
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
            // sample at chunk 0, then only the values of the other chunks (a
            // specular lobe is cheap to re-run; a non-specular one is BSDF::f's
            // lobe sum at the sampled local direction, as in BSDF::Sample_f)
            V3 woL = v3(0, 0, 0), wiL = v3(0, 0, 0);
            bool reflectS = false, specS = false;
            {
                hb_chunk(h, &hb0, 0);
                const S3 v0 = bsdf_sample<kFtAll>(hb0.b, wo, &wi, u0, u1, &bsdfPdf, kBxAll, &flags, &wiL);
                curWvlDep = isectWvlDep && (flags & kBxT);
                dep = isWvlDependent || curWvlDep;
                specS = (flags & kBxSpecular) != 0;
                woL = w2l(hb0.b, wo);
                reflectS = dot(wi, hb0.b.ng) * dot(wo, hb0.b.ng) > 0;
                const float cosv = absdot(wi, si.sn);
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
                            if (specS) {
                                int fl2 = 0;
                                float pdf2 = 0;
                                V3 wi2;
                                v = bsdf_sample<kFtAll>(hb0.b, wo, &wi2, u0, u1, &pdf2, kBxAll, &fl2);
                            } else {
                                v = hb_lobes_f(hb0.b, woL, wiL, reflectS);
                            }
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
                        gload(Bg, N, i0, bv);
#pragma unroll
                        for (int j = 0; j < kG; ++j) bv[j] *= (f[j] * cosv) / bsdfPdf;
                        gstore(Bg, N, i0, bv);
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
                    for (int i = 1; i < 4; ++i) {
                        float p;
                        fv[i] = f1_pdf(curWvlDep, i, wo, wi, wvlIdx[i], &p);
                        pathWvlPdf[i] *= p;
                    }
                    for (int i0 = 0; i0 < kNS; i0 += kG) {
                        float bv[kG];
                        gload(Bg, N, i0, bv);
#pragma unroll
                        for (int j = 0; j < kG; ++j) {
                            const int b = i0 + j;
                            float f = b == wvlIdx[0] ? fv[0] : 0.f;
                            for (int i = 1; i < 4; ++i)
                                if (wvlIdx[i] == b) f += fv[i];
                            bv[j] *= f * cosv;
                        }
                        gstore(Bg, N, i0, bv);
                    }
                }
                bool bnb = false;
                for (int i = 0; i < kNS; ++i) bnb |= Bg[i * N] != 0.f;
                if (bnb) {
                    ray = Ray{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf};
                    if ((flags & kBxSpecular) && (flags & kBxT)) {
                        const float eta = hb0.b.eta;
                        etaScale *= (dot(wo, si.n) > 0) ? (eta * eta) : 1 / (eta * eta);
                    }
                    float mc = Bg[0] * etaScale;
                    for (int i = 1; i < kNS; ++i) mc = smax(mc, Bg[i * N] * etaScale);
                    bool alive = true;
                    if (mc < sc.rr_threshold && bounces > 3) {
                        const float q = smax(0.05f, 1 - mc);
                        if (dm.get1() < q) alive = false;
                        else
                            for (int i0 = 0; i0 < kNS; i0 += kG) {
                                float bv[kG];
                                gload(Bg, N, i0, bv);
#pragma unroll
                                for (int j = 0; j < kG; ++j) bv[j] /= 1 - q;
                                gstore(Bg, N, i0, bv);
                            }
                    }
                    if (alive) {
                        isWvlDependent |= curWvlDep;
                        hf = (hf & ~(kHfWvlDep | kHfLastSpec)) | (isWvlDependent ? kHfWvlDep : 0u) |
                             ((flags & kBxSpecular) ? kHfLastSpec : 0u);
                        store_ray6(ps.ray, N, slot, ray);
                        rays[(*nrays)++] = slot << 2 | kRayCont;
                        cont = true;
                        ++bounces;
                        for (int k = 0; k < 4; ++k) {
                            H[(kHsPath + k) * N] = pathWvlPdf[k];
                            H[(kHsPrev + k) * N] = prev[k];
                        }
                        H[kHsEtaScale * N] = etaScale;
                        H[kHsBsdfPdf * N] = bsdfPdf;
                    }
                }
            }
        }
    }
    if (cont) st |= kStCont;
    if (dm.overflow) { st |= kStDimOverflow; *overflow = true; }
    st = (st & ~(kStDimMask | (0xffu << kStBounceShift))) | ((uint32_t)dm.dim & kStDimMask) |
         ((uint32_t)bounces << kStBounceShift);
    H[kHsFlags * N] = __uint_as_float(hf);
    ps.st[slot] = st;
    if (!(st & (kStCont | kStNee))) finish();
}

__device__ __forceinline__ void shade_hero_batch(const DevScene& sc, const DevHero& h, const DevPaths& ps,
                                                 const DevHeroPaths& hp, const uint32_t* __restrict__ pq,
                                                 const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
                                                 uint32_t* rq_out_count, uint32_t* pq_out, uint32_t* pq_out_count,
                                                 DevStats* stats) {
    const uint32_t n = *pq_count;
    bool overflow = false;
    PT_WAVEQ(wq);
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        uint32_t rays[3];
        uint32_t nrays = 0;
        bool keep = false;
        uint32_t slot = 0;
        if (i < n) {
            slot = pq[i];
            hero_step(sc, h, ps, hp, slot, rays, &nrays, &overflow);
            keep = (ps.st[slot] & (kStCont | kStNee)) != 0;
        }
        wq_push(wq, rays, nrays, keep, slot, rq_out_count, rq_out, pq_out);
    }
    wq_flush(wq, rq_out_count, rq_out, pq_out);
    if (overflow) atomicAdd(&stats->dim_overflow, 1ull);
}

// register-budget variants (PT_HERO_WAVES): compiler default, 2 or 4 waves per SIMD
#define PT_HERO_SHADE(name, attr)                                                                                   \
    __global__ __launch_bounds__(kShadeBlock) attr void name(                                                      \
        DevScene sc, DevHero h, DevPaths ps, DevHeroPaths hp, const uint32_t* __restrict__ pq,                     \
        const uint32_t* __restrict__ pq_count, uint32_t* rq_out, uint32_t* rq_out_count, uint32_t* pq_out,        \
        uint32_t* pq_out_count, DevStats* stats) PT_HERO_BODY
#ifdef PT_TU_HERO
#define PT_HERO_BODY { shade_hero_batch(sc, h, ps, hp, pq, pq_count, rq_out, rq_out_count, pq_out, pq_out_count, stats); }
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
                                    const float* L = h.out60 + (size_t)slot * kNS;
                                    bool nan = false;
                                    for (int i = 0; i < kNS; ++i) nan |= __builtin_isnan(L[i]);
                                    const float yv = s60_y(h, L);
                                    if (nan || (double)yv < -1e-5 || __builtin_isinf(yv)) k = 0.f;
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
