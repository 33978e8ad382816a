// hero.hip -- the hero-wavelength integrators on the device (included by
// render.hip after kernels.hip).
//
// The reference runs hero_path / hero_path_mis only in its SampledSpectrum
// build: every radiance quantity is 60 bins over 400-700 nm and four hero
// wavelengths per camera sample drive dispersion (integrators/hero.cpp,
// hero_path.cpp, hero_path_mis.cpp).  Carrying 2 x 240 B of spectral path
// state through the wavefront queues would double the HBM traffic of every
// bounce for a mode with no shared work between paths, so this path is a
// megakernel: one thread per camera sample, the bounce loop in registers /
// private memory, traversal inline (the LDS-stack `traverse` of kernels.hip),
// the 60-bin radiance of each sample written once to `out60` and filtered by
// k_film_s60 in the reference's FilmTile order.  BSDF values are evaluated
// with the RGB lobe code three bins at a time (every lobe is f = R * scalar),
// the lobe set being chosen from the full 60-bin reflectances; a lobe's
// scalar factors do not depend on the bin, so each chunk is bit-identical to
// the 60-bin evaluation.

namespace pt {

constexpr int kNS = 60;

struct DevHero {
    const float* XYZ;        // 3 x 60 CIE matching functions (SampledSpectrum::Init)
    const float* illum;      // 7 x 60 RGB->illuminant basis (W C M Y R G B)
    const float* mat_s60;    // n_materials x 3 x 60
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
__device__ __forceinline__ bool nonblack_clamped(const float* v) {
    for (int i = 0; i < kNS; ++i)
        if ((v[i] < 0 ? 0.f : v[i]) != 0.f) return true;
    return false;
}
__device__ __forceinline__ void hb_make(const DevScene& sc, const DevHero& h, int mi, const SurfHit& si, float eta,
                                        HeroBsdf* hb) {
    hb->rep = sc.mats[PT_IDX(mi, sc.n_mats)];
    hb->mi = mi;
    const float* ms = h.mat_s60 + (size_t)mi * 3 * kNS;
    const float one = nonblack_clamped(ms) ? 1.f : 0.f, r = nonblack_clamped(ms + kNS) ? 1.f : 0.f,
                t = nonblack_clamped(ms + 2 * kNS) ? 1.f : 0.f;
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
__device__ __forceinline__ float hb_f1(const DevHero& h, HeroBsdf* hb, V3 wo, V3 wi, int bin) {
    hb_chunk(h, hb, bin / 3);
    return bsdf_f<kFtAll>(hb->b, wo, wi, kBxAll).c[bin % 3];
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

struct HeroCounters {
    unsigned long long closest, shadow, nodes, prims;
};

// One hero path (hero_path.cpp:57-189, hero_path_mis.cpp:110-327).
__device__ void hero_li(const DevScene& sc, const DevHero& h, Ray ray, const float* wvls, Dims& dm,
                        int (*stk)[kTraceBlock], int* spill, HeroCounters& ctr, float* Lo) {
    float beta[kNS], wvlPdf[kNS], f[kNS], tmp[kNS];
    for (int i = 0; i < kNS; ++i) { Lo[i] = 0.f; beta[i] = 1.f; wvlPdf[i] = 1.f; }
    float etaScale = 1, bsdfPdf = 0;
    bool isWvlDependent = false, isLastSpecular = false;
    float pathWvlPdf[4] = {1, 1, 1, 1}, prev[4] = {1, 1, 1, 1};
    int wvlIdx[4];
    for (int i = 0; i < 4; ++i) {
        int idx = (int)((wvls[i] - (float)400) * ((float)kNS / (float)300));  // indexFromWavelength
        wvlIdx[i] = idx < kNS - 1 ? idx : kNS - 1;
        wvlPdf[wvlIdx[i]] = h.wcdf[wvlIdx[i] + 1] - h.wcdf[wvlIdx[i]];
    }
    for (int bounces = 0;; ++bounces) {
        const V3 rayO = ray.o;
        float tHit = kInf;
        ++ctr.closest;
        const int hp = traverse<false, true>(sc, sc.nodes, sc.prims, ray, stk, spill, &ctr.nodes, &ctr.prims, &tHit);
        SurfHit si;
        const bool found = hp >= 0 && surface_at<true>(sc, hp, ray, &si);
        if (!found) {
            for (int li = 0; li < sc.n_lights; ++li) {
                const DevLight& l = sc.lights[li];
                if (l.kind != PT_LIGHT_INFINITE) continue;
                s60_from_rgb_illum(h, inf_Le(l, ray.d), tmp);  // Spectrum(Lmap->Lookup, Illuminant)
                if (s60_black(tmp)) continue;
                if (!h.mis) {
                    const float sw = pathWvlPdf[0] + pathWvlPdf[1] + pathWvlPdf[2] + pathWvlPdf[3];
                    for (int i = 0; i < kNS; ++i)
                        Lo[i] += isWvlDependent ? (beta[i] * tmp[i]) / (wvlPdf[i] * sw) : beta[i] * tmp[i];
                } else if (bounces == 0) {
                    for (int i = 0; i < kNS; ++i) Lo[i] += beta[i] * tmp[i];
                } else {
                    const float emPdf = isLastSpecular ? 0.f : inf_pdf_li(l, ray.d);
                    const float s = (pathWvlPdf[0] + prev[0] * emPdf) + (pathWvlPdf[1] + prev[1] * emPdf) +
                                    (pathWvlPdf[2] + prev[2] * emPdf) + (pathWvlPdf[3] + prev[3] * emPdf);
                    const float mwc = bsdfPdf / (bsdfPdf + emPdf);
                    for (int i = 0; i < kNS; ++i)
                        Lo[i] += (beta[i] * tmp[i]) * (isWvlDependent ? 1.0f / (wvlPdf[i] * s) : mwc);
                }
            }
            break;
        }
        int mat, light;
        prim_info<true>(sc, hp, &mat, &light);
        if (light >= 0) {
            const DevLight& l = sc.lights[PT_IDX(light, sc.n_lights)];
            light_L60(h, l, light, si.n, -ray.d, tmp);
            if (!s60_black(tmp)) {
                if (!h.mis) {
                    const float sw = pathWvlPdf[0] + pathWvlPdf[1] + pathWvlPdf[2] + pathWvlPdf[3];
                    for (int i = 0; i < kNS; ++i)
                        Lo[i] += isWvlDependent ? (beta[i] * tmp[i]) / (wvlPdf[i] * sw) : beta[i] * tmp[i];
                } else if (bounces == 0) {
                    for (int i = 0; i < kNS; ++i) Lo[i] += beta[i] * tmp[i];
                } else {
                    float emPdf = 0;
                    if (!isLastSpecular) {  // PdfEmitterHero (hero_path_mis.cpp:46-76)
                        emPdf = (tHit * tHit) / (absdot(si.n, si.wo) * l.area);  // it.shape->Area()
                        const float* d = hero_dist(h, rayO);
                        const int nl = sc.n_lights;
                        emPdf = emPdf * (d[light] / (d[2 * nl + 1] * nl));
                    }
                    const float s = (pathWvlPdf[0] + prev[0] * emPdf) + (pathWvlPdf[1] + prev[1] * emPdf) +
                                    (pathWvlPdf[2] + prev[2] * emPdf) + (pathWvlPdf[3] + prev[3] * emPdf);
                    const float mwc = bsdfPdf / (bsdfPdf + emPdf);
                    for (int i = 0; i < kNS; ++i)
                        Lo[i] += (beta[i] * tmp[i]) * (isWvlDependent ? 1.0f / (wvlPdf[i] * s) : mwc);
                }
            }
        }
        if (bounces >= sc.max_depth) break;
        const pt_material& M = sc.mats[PT_IDX(mat, sc.n_mats)];
        if (M.kind == PT_MAT_NONE) {
            ray = Ray{offset_ray_origin(si.p, si.perr, si.n, ray.d), ray.d, kInf};
            bounces--;
            continue;
        }
        const bool disp = M.kind == PT_MAT_DISPERSIVE_GLASS;
        HeroBsdf hb[4];
        bool isectWvlDep = false;
        if (disp) {  // one BSDF per wavelength (dispersive_glass.cpp:62-118)
            const float lminsq = (float)(400 * 400), lmaxsq = (float)(700 * 700);
            const float cauchyB = (lminsq * M.ior_max - lmaxsq * M.ior_min) / (lminsq - lmaxsq);
            const float cauchyC = lminsq * (M.ior_max - cauchyB);
            for (int i = 0; i < 4; ++i) hb_make(sc, h, mat, si, cauchyB + cauchyC / (wvls[i] * wvls[i]), &hb[i]);
            isectWvlDep = hb[0].b.n > 0;
        } else {
            hb_make(sc, h, mat, si, M.ior, &hb[0]);
        }
        if (h.mis && bsdf_num<kFtAll>(hb[0].b, kBxNonSpecular) > 0 && sc.n_lights > 0) {
            // SampleEmitterHero (hero_path_mis.cpp:78-108)
            const float* d = hero_dist(h, si.p);
            const int nl = sc.n_lights;
            float emPdf = 0;
            V3 wi = v3(0, 0, 0);
            bool haveLi = false;
            float lpdf;
            const int li = dist_sample(d, nl, dm.get1(), &lpdf);
            emPdf = lpdf;
            if (lpdf != 0.f) {
                const float u0 = dm.get1(), u1 = dm.get1();
                float epdf = 0;
                V3 sp, sn, spe;
                const DevLight& l = sc.lights[PT_IDX(li, sc.n_lights)];
                const S3 Lrgb = area_sample_li<kFtAll>(sc, l, si, u0, u1, &wi, &epdf, &sp, &sn, &spe);
                bool occluded = true;
                if (epdf != 0.f) {
                    const V3 origin = offset_ray_origin(si.p, si.perr, si.n, sp - si.p);
                    const V3 target = offset_ray_origin(sp, spe, sn, origin - sp);
                    ++ctr.shadow;
                    occluded = traverse<true, true>(sc, sc.nodes, sc.prims, Ray{origin, target - origin, 1 - kShadowEps},
                                                    stk, spill, &ctr.nodes, &ctr.prims) >= 0;
                }
                if (epdf == 0.f || occluded) emPdf = 0.f;
                else {
                    emPdf = emPdf * epdf;
                    if (l.kind == PT_LIGHT_INFINITE) s60_from_rgb_illum(h, Lrgb, tmp);
                    else light_L60(h, l, li, sn, -wi, tmp);
                    for (int i = 0; i < kNS; ++i) tmp[i] = tmp[i] / emPdf;
                    haveLi = !s60_black(tmp);
                }
            }
            if (haveLi && emPdf > 0.f) {
                const V3 wo = si.wo;
                hb_f(h, &hb[0], wo, wi, f);
                if (!s60_black(f)) {
                    float mw[kNS];
                    if (isWvlDependent || isectWvlDep) {
                        for (int i = 0; i < kNS; ++i) f[i] = 0.0f;
                        float bp[4];
                        for (int i = 0; i < 4; ++i) {
                            HeroBsdf* b = &hb[isectWvlDep ? i : 0];
                            f[wvlIdx[i]] += hb_f1(h, b, wo, wi, wvlIdx[i]);
                            bp[i] = bsdf_pdf<kFtAll>(b->b, wo, wi, kBxAll);
                        }
                        const float s = (pathWvlPdf[0] * emPdf + pathWvlPdf[0] * bp[0]) +
                                        (pathWvlPdf[1] * emPdf + pathWvlPdf[1] * bp[1]) +
                                        (pathWvlPdf[2] * emPdf + pathWvlPdf[2] * bp[2]) +
                                        (pathWvlPdf[3] * emPdf + pathWvlPdf[3] * bp[3]);
                        for (int i = 0; i < kNS; ++i) mw[i] = emPdf / (wvlPdf[i] * s);
                    } else {
                        const float bp = bsdf_pdf<kFtAll>(hb[0].b, wo, wi, kBxAll);
                        const float m = emPdf / (emPdf + bp);
                        for (int i = 0; i < kNS; ++i) mw[i] = m;
                    }
                    const float cosv = absdot(wi, si.sn);
                    for (int i = 0; i < kNS; ++i) f[i] *= cosv;
                    for (int i = 0; i < kNS; ++i) Lo[i] += ((beta[i] * tmp[i]) * f[i]) * mw[i];
                }
            }
        }
        // BSDF sampling
        const V3 wo = -ray.d;
        V3 wi = v3(0, 0, 0);
        int flags = 0;
        const float u0 = dm.get1(), u1 = dm.get1();
        bsdfPdf = 0;
        for (int k = 0; k < kNS / 3; ++k) {
            hb_chunk(h, &hb[0], k);
            const S3 v = bsdf_sample<kFtAll>(hb[0].b, wo, &wi, u0, u1, &bsdfPdf, kBxAll, &flags);
            f[3 * k] = v.c[0]; f[3 * k + 1] = v.c[1]; f[3 * k + 2] = v.c[2];
        }
        if (s60_black(f) || bsdfPdf == 0.f) break;
        const bool curWvlDep = isectWvlDep && (flags & kBxT);
        const float cosv = absdot(wi, si.sn);
        if (isWvlDependent || curWvlDep) {
            for (int i = 0; i < 4; ++i) prev[i] = pathWvlPdf[i];
            const float keep = f[wvlIdx[0]];
            for (int i = 0; i < kNS; ++i) f[i] = 0.f;
            f[wvlIdx[0]] = keep;  // zeroAllBinsBut(wvlIdx[0])
            pathWvlPdf[0] *= bsdfPdf;
            for (int i = 1; i < 4; ++i) {
                HeroBsdf* b = &hb[curWvlDep ? i : 0];
                f[wvlIdx[i]] += hb_f1(h, b, wo, wi, wvlIdx[i]);
                pathWvlPdf[i] *= bsdf_pdf<kFtAll>(b->b, wo, wi, kBxAll);
            }
            for (int i = 0; i < kNS; ++i) beta[i] *= f[i] * cosv;
        } else {
            for (int i = 0; i < kNS; ++i) beta[i] *= (f[i] * cosv) / bsdfPdf;
        }
        if (s60_black(beta)) break;
        ray = Ray{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf};
        if ((flags & kBxSpecular) && (flags & kBxT)) {
            const float eta = hb[0].b.eta;
            etaScale *= (dot(wo, si.n) > 0) ? (eta * eta) : 1 / (eta * eta);
        }
        float mc = beta[0] * etaScale;
        for (int i = 1; i < kNS; ++i) mc = smax(mc, beta[i] * etaScale);
        if (mc < sc.rr_threshold && bounces > 3) {
            const float q = smax(0.05f, 1 - mc);
            if (dm.get1() < q) break;
            for (int i = 0; i < kNS; ++i) beta[i] /= 1 - q;
        }
        isWvlDependent |= curWvlDep;
        isLastSpecular = (flags & kBxSpecular) != 0;
    }
}

// One thread per (pixel, sample) slot of the batch: camera sample, the four
// hero wavelengths (hero.cpp:113-150) and the path; writes pfilm and out60.
__global__ __launch_bounds__(kTraceBlock) void k_hero(DevScene sc, DevHero h, DevPaths ps,
                                                      const int2* __restrict__ pix, int npix, int s0, int nsamp,
                                                      HaltonPixelConsts hp, int* spill, DevStats* stats) {
    __shared__ int stk[kStackLds][kTraceBlock];
    const uint32_t total = (uint32_t)npix * (uint32_t)nsamp;
    const size_t gtid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    int* myspill = spill + gtid * (64 - kStackLds);
    HeroCounters ctr{0, 0, 0, 0};
    bool overflow = false;
    float L[kNS];
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += gridDim.x * blockDim.x) {
        const uint32_t slot = base + threadIdx.x;
        if (slot >= total) continue;
        const uint32_t p = slot / (uint32_t)nsamp, sl = slot - p * (uint32_t)nsamp;
        const int2 px = pix[p];
        const uint32_t off = halton_pixel_offset(sc, px.x, px.y, hp.exp1, hp.scale0, hp.mi0, hp.mi1);
        const uint32_t idx = off + (uint32_t)(s0 + (int)sl) * sc.hal_stride;
        const float fx = (float)px.x + halton_dim(sc, idx, 0);
        const float fy = (float)px.y + halton_dim(sc, idx, 1);
        float lx = 0.5f, ly = 0.5f;
        if (sc.lens_radius > 0) { lx = halton_dim(sc, idx, 3); ly = halton_dim(sc, idx, 4); }
        const float uw = halton_dim(sc, idx, sc.wvl_dim);
        const Ray r = camera_ray(sc, fx, fy, lx, ly);
        float wvls[4];
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
            wvls[i] = (float)400 + (float)300 * ((alpha + (float)bin) / (float)kNS);
        }
        Dims dm{&sc, idx, sc.wvl_dim + 1, false};
        hero_li(sc, h, r, wvls, dm, stk, myspill, ctr, L);
        overflow |= dm.overflow;
        ps.pfilm[slot] = make_float2(fx, fy);
        float* o = h.out60 + (size_t)slot * kNS;
        for (int i = 0; i < kNS; ++i) o[i] = L[i];
    }
    flush_stats(stats, ctr.closest, ctr.shadow, ctr.nodes, ctr.prims);
    if (overflow) atomicAdd(&stats->dim_overflow, 1ull);
}

// Film for SampledSpectrum samples: k_film's ordered per-pixel gather with a
// 60-bin FilmTile contribSum (lane = bin), converted by ToXYZ at the merge
// (film.h:121-161, film.cpp:117-130, spectrum.h:395-406).
__global__ __launch_bounds__(256) void k_film_s60(DevHero h, DevPaths ps, FilmConsts fc,
                                                  const int* __restrict__ pixslot, int p0, int np, int nsamp, int bx0,
                                                  int by0, int bw, int bh, float4* accum) {
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
                            while (m) {
                                const int j = __ffsll((unsigned long long)m) - 1;
                                m &= m - 1;
                                const uint32_t sj = (uint32_t)__shfl((int)slot, j);
                                const float kj = lane_val(k, j), wj = lane_val(w, j);
                                if (lane < kNS) {
                                    float v = h.out60[(size_t)sj * kNS + lane];
                                    if (kj == 0.f) v = 0.f;        // L = Spectrum(0.f)
                                    else if (kj != 1.f) v = v * kj;  // L *= maxSampleLuminance / L.y()
                                    binsum += (v * 1.f) * wj;
                                }
                                wsum += wj;
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

// SpatialLightDistribution::ComputeDistribution (lightdistrib.cpp:175-236)
// for every voxel: 128 radical-inverse points, each light's Li.y() / pdf,
// floored at 0.001 x the average, as a Distribution1D (sampling.h:65-88).
// `ri` holds RadicalInverse(0..4, i) for i < 128; `light_y` each area
// light's Lemit.y().
__global__ void k_hero_spatial(DevScene sc, DevHero h, const float* __restrict__ ri, const float* __restrict__ light_y,
                               float* dist) {
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

}  // namespace pt
