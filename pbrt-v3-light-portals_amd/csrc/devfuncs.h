// devfuncs.h -- device functions of the hot path (gfx950).  Each restates a
// reference function (file:line cited) with the same float operation order.
#pragma once

#undef PT_FILE_ID
#define PT_FILE_ID 1  // PT_IDX source tag
#include "device.h"

namespace pt {

// ----------------------------------------------------------------------------
// Halton sampler: HaltonSampler::SampleDimension (samplers/halton.cpp:118-127)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float radical_inverse_base3(uint32_t a) {  // lowdiscrepancy.cpp:389-403
    const float invBase = 1.0f / 3.0f;
    uint64_t rev = 0;
    float invBaseN = 1;
    while (a) {
        uint32_t next = a / 3u;
        uint32_t digit = a - next * 3u;
        rev = rev * 3u + digit;
        invBaseN *= invBase;
        a = next;
    }
    return smin((float)rev * invBaseN, kOneMinusEps);
}

template <typename Rev>
__device__ __forceinline__ float scrambled_ri_digits(float c0, uint32_t a, const DivMagic& dm, const uint16_t* perm) {
    Rev rev = 0;
    float invBaseN = 1;
    // Digits four at a time: the digit chain is ALU only, so the four
    // permutation gathers are issued back to back and waited on once (a
    // digit past the end is 0, a valid index whose entry is not used).  The
    // accumulation keeps the reference's per-digit order.
    while (a) {
        uint32_t d[4], live = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t next = fast_div(a, dm);
            d[k] = a - next * dm.base;
            live += a != 0u ? 1u : 0u;
            a = next;
        }
        uint32_t pv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) pv[k] = perm[d[k]];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if ((uint32_t)k < live) {
                rev = rev * (Rev)dm.base + (Rev)pv[k];
                invBaseN *= dm.inv_base;
            }
        }
    }
    return smin(invBaseN * ((float)rev + c0), kOneMinusEps);
}

__device__ __forceinline__ float scrambled_radical_inverse(const DivMagic& dm, const uint16_t* perm, float c0,
                                                           uint32_t a) {  // :405-424
    // reversedDigits < base^nDigits <= base * a: with base * a < 2^32 the
    // reference's 64-bit accumulator never leaves 32 bits (same value, same float)
    if ((uint64_t)a * dm.base < (1ull << 32)) return scrambled_ri_digits<uint32_t>(c0, a, dm, perm);
    return scrambled_ri_digits<uint64_t>(c0, a, dm, perm);
}
__device__ __forceinline__ float scrambled_radical_inverse(const DevScene& sc, int dim, uint32_t a) {
    return scrambled_radical_inverse(sc.divs[dim], sc.perm + sc.prime_sums[dim], sc.perm_c0[dim], a);
}

// dim must be < sc.max_dim (checked by the caller).
__device__ __forceinline__ float halton_dim(const DevScene& sc, uint32_t idx, int dim) {
    if (sc.center && dim < 2) return 0.5f;
    if (dim == 0) return (float)reverse_bits32(idx >> sc.hal_exp0) * 0x1p-32f;  // RadicalInverse(0, .)
    if (dim == 1) return radical_inverse_base3(fast_div(idx, sc.div_scale1));
    return scrambled_radical_inverse(sc, dim, idx);
}

// The Halton tables of the leading DevScene::hal_lds_dims dimensions staged in
// LDS by the shading kernel (the digit loop's permutation gathers are its
// longest chain of dependent loads): per dimension {magic, base | first
// permutation entry << 16, shift | shift(base^2) << 8, magic(base^2)} and
// {c0, 1/base}, then those dimensions' permutation entries.
struct HalLds {
    const uint4* rec;
    const float2* cb;
    const uint16_t* perm;
    int dims;
};
__device__ __forceinline__ HalLds stage_halton(const DevScene& sc, uint4* lds) {
    const int D = sc.hal_lds_dims;
    uint4* rec = lds;
    float2* cb = (float2*)(lds + D);
    uint16_t* perm = (uint16_t*)(cb + D);
    for (int i = threadIdx.x; i < D; i += blockDim.x) {
        const DivMagic dm = sc.divs[i];
        const DivMagic d2 = sc.divs2[i];
        rec[i] = make_uint4(dm.magic, dm.base | ((uint32_t)sc.prime_sums[i] << 16), dm.shift | (d2.shift << 8), d2.magic);
        cb[i] = make_float2(sc.perm_c0[i], dm.inv_base);
    }
    for (int i = threadIdx.x; i < sc.hal_lds_perm; i += blockDim.x) perm[i] = sc.perm[i];
    __syncthreads();
    return HalLds{rec, cb, perm, D};
}
// ScrambledRadicalInverseSpecialized (lowdiscrepancy.cpp:405-424) two digits
// per step: one division by base^2 gives both (q = d0 + base * d1), and
// (rev * base + perm[d0]) * base + perm[d1] == rev * base^2 + (perm[d0] * base
// + perm[d1]) exactly in the integer accumulator; invBaseN keeps the
// reference's one float multiply per digit.  The loop runs exactly the
// number of digit pairs (no masked slots); an odd last digit is a itself.
template <typename Rev>
__device__ __forceinline__ float scrambled_ri_pairs(float c0, float invBase, uint32_t a, const DivMagic& dm,
                                                    const DivMagic& d2, const uint16_t* perm) {
    Rev rev = 0;
    float invBaseN = 1;
    while (a >= dm.base) {
        const uint32_t next = fast_div(a, d2);
        const uint32_t q = a - next * d2.base;
        const uint32_t d1 = fast_div(q, dm);
        const uint32_t d0 = q - d1 * dm.base;
        const uint32_t p0 = perm[d0], p1 = perm[d1];
        rev = rev * (Rev)d2.base + ((Rev)p0 * (Rev)dm.base + (Rev)p1);
        invBaseN *= invBase;
        invBaseN *= invBase;
        a = next;
    }
    if (a) {
        rev = rev * (Rev)dm.base + (Rev)perm[a];
        invBaseN *= invBase;
    }
    return smin(invBaseN * ((float)rev + c0), kOneMinusEps);
}
// halton_dim with the staged tables for dimensions below hl.dims.
__device__ __forceinline__ float halton_dim(const DevScene& sc, const HalLds& hl, uint32_t idx, int dim) {
    if (dim < 2 || dim >= hl.dims) return halton_dim(sc, idx, dim);
    const uint4 r = hl.rec[dim];
    const float2 cb = hl.cb[dim];
    const uint32_t b = r.y & 0xffffu;
    const DivMagic dm{b, r.x, r.z & 0xffu, cb.y};
    const DivMagic d2{b * b, r.w, r.z >> 8, 0.f};
    const uint16_t* perm = hl.perm + (r.y >> 16);
    // rev < base^nDigits <= base * a: below 2^32 the reference's 64-bit
    // accumulator never leaves 32 bits
    if ((uint64_t)idx * b < (1ull << 32)) return scrambled_ri_pairs<uint32_t>(cb.x, cb.y, idx, dm, d2, perm);
    return scrambled_ri_pairs<uint64_t>(cb.x, cb.y, idx, dm, d2, perm);
}

// Per-pixel Halton offset (halton.cpp:96-113); values stay far below 2^32.
__device__ __forceinline__ uint32_t halton_pixel_offset(const DevScene& sc, int px, int py, int exp1,
                                                        uint32_t scale0, uint32_t mi0, uint32_t mi1) {
    uint32_t stride = sc.hal_stride;
    if (stride <= 1) return 0;
    int pmx = px % 128; if (pmx < 0) pmx += 128;
    int pmy = py % 128; if (pmy < 0) pmy += 128;
    uint64_t off = 0;
    {   // InverseRadicalInverse<2>(pm.x, exp0)
        uint64_t inv = (uint64_t)pmx, index = 0;
        for (int i = 0; i < sc.hal_exp0; ++i) { uint64_t d = inv % 2u; inv /= 2u; index = index * 2u + d; }
        off += index * (uint64_t)(stride / scale0) * (uint64_t)mi0;
    }
    {   // InverseRadicalInverse<3>(pm.y, exp1)
        uint64_t inv = (uint64_t)pmy, index = 0;
        for (int i = 0; i < exp1; ++i) { uint64_t d = inv % 3u; inv /= 3u; index = index * 3u + d; }
        off += index * (uint64_t)(stride / sc.hal_scale1) * (uint64_t)mi1;
    }
    return (uint32_t)(off % stride);
}

// ----------------------------------------------------------------------------
// Triangle::Intersect / IntersectP ray-triangle test (triangle.cpp:189-292)
// ----------------------------------------------------------------------------
__device__ __forceinline__ bool tri_test(V3 p0, V3 p1, V3 p2, const Ray& ray, float* tHit, float* b0o,
                                         float* b1o, float* b2o) {
    V3 p0t = p0 - ray.o, p1t = p1 - ray.o, p2t = p2 - ray.o;
    int kz = maxdim(vabs(ray.d));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    V3 d = permute(ray.d, kx, ky, kz);
    p0t = permute(p0t, kx, ky, kz);
    p1t = permute(p1t, kx, ky, kz);
    p2t = permute(p2t, kx, ky, kz);
    float Sx = -d.x / d.z, Sy = -d.y / d.z, Sz = 1.f / d.z;
    p0t.x += Sx * p0t.z; p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z; p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z; p2t.y += Sy * p2t.z;
    float e0 = p1t.x * p2t.y - p1t.y * p2t.x;
    float e1 = p2t.x * p0t.y - p2t.y * p0t.x;
    float e2 = p0t.x * p1t.y - p0t.y * p1t.x;
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        double p2txp1ty = (double)p2t.x * (double)p1t.y;
        double p2typ1tx = (double)p2t.y * (double)p1t.x;
        e0 = (float)(p2typ1tx - p2txp1ty);
        double p0txp2ty = (double)p0t.x * (double)p2t.y;
        double p0typ2tx = (double)p0t.y * (double)p2t.x;
        e1 = (float)(p0typ2tx - p0txp2ty);
        double p1txp0ty = (double)p1t.x * (double)p0t.y;
        double p1typ0tx = (double)p1t.y * (double)p0t.x;
        e2 = (float)(p1typ0tx - p1txp0ty);
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz; p1t.z *= Sz; p2t.z *= Sz;
    float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < ray.tmax * det)) return false;
    else if (det > 0 && (tScaled <= 0 || tScaled > ray.tmax * det)) return false;
    float invDet = 1 / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    float t = tScaled * invDet;
    float maxZt = maxcomp(vabs(v3(p0t.z, p1t.z, p2t.z)));
    float deltaZ = gammaf(3) * maxZt;
    float maxXt = maxcomp(vabs(v3(p0t.x, p1t.x, p2t.x)));
    float maxYt = maxcomp(vabs(v3(p0t.y, p1t.y, p2t.y)));
    float deltaX = gammaf(5) * (maxXt + maxZt);
    float deltaY = gammaf(5) * (maxYt + maxZt);
    float deltaE = 2 * (gammaf(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = maxcomp(vabs(v3(e0, e1, e2)));
    float deltaT = 3 * (gammaf(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * fabsf(invDet);
    if (t <= deltaT) return false;
    *tHit = t;
    *b0o = b0; *b1o = b1; *b2o = b2;
    return true;
}

// The ray-only part of Triangle::Intersect's set-up (triangle.cpp:205-222):
// the permutation axis kz and the shear Sx, Sy, Sz, computed once per ray by
// the traversal kernels instead of once per primitive test (same operations,
// so the same values).
struct TriShear {
    float sx, sy, sz;
    int kz;
};
__device__ __forceinline__ TriShear tri_shear(const V3& rd) {
    const int kz = maxdim(vabs(rd));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    const V3 d = permute(rd, kx, ky, kz);
    return TriShear{-d.x / d.z, -d.y / d.z, 1.f / d.z, kz};
}

// Accept/reject + t of tri_test, written for SIMD execution: the same float
// operations in the same order, the early exits folded into one predicate
// (only the rare double-precision edge recomputation stays a branch).
__device__ __forceinline__ bool tri_hit(V3 p0, V3 p1, V3 p2, const Ray& ray, const TriShear& sh, float* tHit) {
    V3 p0t = p0 - ray.o, p1t = p1 - ray.o, p2t = p2 - ray.o;
    const int kz = sh.kz;
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    p0t = permute(p0t, kx, ky, kz);
    p1t = permute(p1t, kx, ky, kz);
    p2t = permute(p2t, kx, ky, kz);
    const float Sx = sh.sx, Sy = sh.sy, Sz = sh.sz;
    p0t.x += Sx * p0t.z; p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z; p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z; p2t.y += Sy * p2t.z;
    float e0 = p1t.x * p2t.y - p1t.y * p2t.x;
    float e1 = p2t.x * p0t.y - p2t.y * p0t.x;
    float e2 = p0t.x * p1t.y - p0t.y * p1t.x;
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        double p2txp1ty = (double)p2t.x * (double)p1t.y;
        double p2typ1tx = (double)p2t.y * (double)p1t.x;
        e0 = (float)(p2typ1tx - p2txp1ty);
        double p0txp2ty = (double)p0t.x * (double)p2t.y;
        double p0typ2tx = (double)p0t.y * (double)p2t.x;
        e1 = (float)(p0typ2tx - p0txp2ty);
        double p1txp0ty = (double)p1t.x * (double)p0t.y;
        double p1typ0tx = (double)p1t.y * (double)p0t.x;
        e2 = (float)(p1typ0tx - p1txp0ty);
    }
    bool ok = !((e0 < 0 || e1 < 0 || e2 < 0) & (e0 > 0 || e1 > 0 || e2 > 0));
    const float det = e0 + e1 + e2;
    ok &= det != 0;
    p0t.z *= Sz; p1t.z *= Sz; p2t.z *= Sz;
    const float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    const float tmd = ray.tmax * det;
    ok &= !((det < 0) & ((tScaled >= 0) | (tScaled < tmd)));
    ok &= !((det > 0) & ((tScaled <= 0) | (tScaled > tmd)));
    const float invDet = 1 / det;
    const float t = tScaled * invDet;
    const float maxZt = maxcomp(vabs(v3(p0t.z, p1t.z, p2t.z)));
    const float deltaZ = gammaf(3) * maxZt;
    const float maxXt = maxcomp(vabs(v3(p0t.x, p1t.x, p2t.x)));
    const float maxYt = maxcomp(vabs(v3(p0t.y, p1t.y, p2t.y)));
    const float deltaX = gammaf(5) * (maxXt + maxZt);
    const float deltaY = gammaf(5) * (maxYt + maxZt);
    const float deltaE = 2 * (gammaf(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    const float maxE = maxcomp(vabs(v3(e0, e1, e2)));
    const float deltaT = 3 * (gammaf(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * fabsf(invDet);
    ok &= !(t <= deltaT);
    *tHit = t;
    return ok;
}

// ----------------------------------------------------------------------------
// AAPlaneShape::Intersect (plane.cpp:15-55) -- test part
// ----------------------------------------------------------------------------
__device__ __forceinline__ bool plane_test(const DevPlane& pl, const Ray& ray, float* tHit, V3* pHitObj) {
    Ray rT = xf_ray_keep_tmax(pl.w2o, ray);
    float t = (pl.lo_a - rT.o[pl.ax]) / rT.d[pl.ax];
    V3 pHit = rT.o + t * rT.d;
    if (pHit[pl.ax0] > pl.lo_a0 && pHit[pl.ax0] < pl.hi_a0 && pHit[pl.ax1] > pl.lo_a1 &&
        pHit[pl.ax1] < pl.hi_a1 && t < rT.tmax) {
        *tHit = t;
        *pHitObj = pHit;
        return true;
    }
    return false;
}

struct SurfHit {
    V3 p, perr, n, wo;
    V3 sn, sdpdu;
    int prim;  // BVH-order primitive index
};

__device__ __forceinline__ V3 vload3(const float* a, int i) { return v3(a[3 * i], a[3 * i + 1], a[3 * i + 2]); }

// Full Triangle::Intersect for the winning primitive: SurfaceInteraction
// (triangle.cpp:297-420, interaction.cpp:44-89).  Returns false when the
// reference would reject (it never does for the primitive that won in the
// traversal, which already applied the same tests).
// trflags: the triangle's PT_TRI_* flags; its index record (uv / normal /
// tangent vertex indices) is read only when the mesh carries one of them.
__device__ __forceinline__ bool tri_surface(const DevScene& sc, int ti, uint32_t trflags, const Ray& ray, SurfHit* si,
                                            V3 p0, V3 p1, V3 p2) {
    pt_triangle tr;
    tr.flags = trflags;
    if (trflags & (PT_TRI_HAS_UV | PT_TRI_HAS_N | PT_TRI_HAS_S)) tr = sc.tris[PT_IDX(ti, sc.n_tris)];
    Ray r2 = ray;
    r2.tmax = kInf;
    float t, b0, b1, b2;
    if (!tri_test(p0, p1, p2, r2, &t, &b0, &b1, &b2)) return false;
    float uv[3][2];
    bool hasUV = (tr.flags & PT_TRI_HAS_UV) && sc.UV;
    if (hasUV) {
        for (int i = 0; i < 3; ++i) { uv[i][0] = sc.UV[2 * PT_IDX(tr.v[i], sc.n_verts)]; uv[i][1] = sc.UV[2 * PT_IDX(tr.v[i], sc.n_verts) + 1]; }
    } else {
        uv[0][0] = 0; uv[0][1] = 0; uv[1][0] = 1; uv[1][1] = 0; uv[2][0] = 1; uv[2][1] = 1;
    }
    float duv02[2] = {uv[0][0] - uv[2][0], uv[0][1] - uv[2][1]};
    float duv12[2] = {uv[1][0] - uv[2][0], uv[1][1] - uv[2][1]};
    V3 dp02 = p0 - p2, dp12 = p1 - p2;
    float determinant = duv02[0] * duv12[1] - duv02[1] * duv12[0];
    bool degenerateUV = fabs((double)determinant) < 1e-8;
    V3 dpdu = v3(0, 0, 0), dpdv = v3(0, 0, 0);
    if (!degenerateUV) {
        float invdet = 1 / determinant;
        dpdu = (duv12[1] * dp02 - duv02[1] * dp12) * invdet;
        dpdv = (-duv12[0] * dp02 + duv02[0] * dp12) * invdet;
    }
    if (degenerateUV || len2(cross(dpdu, dpdv)) == 0) {
        V3 ng = cross(p2 - p0, p1 - p0);
        if (len2(ng) == 0) return false;
        coordinate_system(normalize(ng), &dpdu, &dpdv);
    }
    float xs = fabsf(b0 * p0.x) + fabsf(b1 * p1.x) + fabsf(b2 * p2.x);
    float ys = fabsf(b0 * p0.y) + fabsf(b1 * p1.y) + fabsf(b2 * p2.y);
    float zs = fabsf(b0 * p0.z) + fabsf(b1 * p1.z) + fabsf(b2 * p2.z);
    si->perr = gammaf(7) * v3(xs, ys, zs);
    si->p = (b0 * p0 + b1 * p1) + b2 * p2;
    si->wo = normalize(-ray.d);
    V3 n = normalize(cross(dp02, dp12));
    bool ro = (tr.flags & PT_TRI_REVERSE_ORIENTATION) != 0;
    bool sh = (tr.flags & PT_TRI_SWAPS_HANDEDNESS) != 0;
    if (ro ^ sh) n = -n;
    si->n = n;
    si->sn = n;
    si->sdpdu = dpdu;
    bool hasN = (tr.flags & PT_TRI_HAS_N) && sc.N;
    bool hasS = (tr.flags & PT_TRI_HAS_S) && sc.S;
    if (hasN || hasS) {
        V3 ns;
        if (hasN) {
            ns = (b0 * vload3(sc.N, PT_IDX(tr.v[0], sc.n_verts)) + b1 * vload3(sc.N, PT_IDX(tr.v[1], sc.n_verts))) + b2 * vload3(sc.N, PT_IDX(tr.v[2], sc.n_verts));
            ns = (len2(ns) > 0) ? normalize(ns) : si->n;
        } else
            ns = si->n;
        V3 ss;
        if (hasS) {
            ss = (b0 * vload3(sc.S, PT_IDX(tr.v[0], sc.n_verts)) + b1 * vload3(sc.S, PT_IDX(tr.v[1], sc.n_verts))) + b2 * vload3(sc.S, PT_IDX(tr.v[2], sc.n_verts));
            ss = (len2(ss) > 0) ? normalize(ss) : normalize(dpdu);
        } else
            ss = normalize(dpdu);
        V3 ts = cross(ss, ns);
        if (len2(ts) > 0.f) { ts = normalize(ts); ss = cross(ts, ns); }
        else coordinate_system(ns, &ss, &ts);
        if (ro) ts = -ts;
        si->sn = normalize(cross(ss, ts));  // SetShadingGeometry(..., true)
        si->n = faceforward(si->n, si->sn);
        si->sdpdu = ss;
    }
    return true;
}

// Full AAPlaneShape::Intersect SurfaceInteraction, transformed to world space
// (plane.cpp:35-50, transform.cpp:262-297).
__device__ __forceinline__ bool plane_surface(const DevPlane& pl, const Ray& ray, SurfHit* si) {
    Ray r2 = ray;
    r2.tmax = kInf;
    float t;
    V3 pHit;
    if (!plane_test(pl, r2, &t, &pHit)) return false;
    V3 dpdu = v3(-1, 0, 0), dpdv = v3(0, 1, 0);
    V3 n = normalize(cross(dpdu, dpdv));
    V3 sn = n;
    if (pl.ro_xor_sh) { n = n * -1.f; sn = sn * -1.f; }
    V3 wo = normalize(-xf_vector(pl.w2o, ray.d));  // -ray.d of the object-space ray, normalised (Interaction ctor)
    si->p = xf_point_err_in(pl.o2w, pHit, v3(0.01f, 0.01f, 0.01f), &si->perr);
    si->n = normalize(xf_normal(pl.w2o, n));
    si->wo = normalize(xf_vector(pl.o2w, wo));
    si->sn = normalize(xf_normal(pl.w2o, sn));
    si->sdpdu = xf_vector(pl.o2w, dpdu);
    si->sn = faceforward(si->sn, si->n);
    return true;
}

// ----------------------------------------------------------------------------
// Sphere (shapes/sphere.cpp) with EFloat running error bounds (core/efloat.h)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float clamp11(float v) { return v < -1 ? -1.f : (v > 1 ? 1.f : v); }
struct EF {
    float v, lo, hi;
};
__device__ __forceinline__ EF ef(float v) { return EF{v, v, v}; }
__device__ __forceinline__ EF ef_err(float v, float err) {  // EFloat(v, err)
    if (err == 0.f) return EF{v, v, v};
    return EF{v, next_down(v - err), next_up(v + err)};
}
__device__ __forceinline__ EF operator+(EF a, EF b) { return EF{a.v + b.v, next_down(a.lo + b.lo), next_up(a.hi + b.hi)}; }
__device__ __forceinline__ EF operator-(EF a, EF b) { return EF{a.v - b.v, next_down(a.lo - b.hi), next_up(a.hi - b.lo)}; }
__device__ __forceinline__ EF operator*(EF a, EF b) {
    const float p0 = a.lo * b.lo, p1 = a.hi * b.lo, p2 = a.lo * b.hi, p3 = a.hi * b.hi;
    return EF{a.v * b.v, next_down(smin(smin(p0, p1), smin(p2, p3))), next_up(smax(smax(p0, p1), smax(p2, p3)))};
}
__device__ __forceinline__ EF operator/(EF a, EF b) {
    if (b.lo < 0 && b.hi > 0) return EF{a.v / b.v, -kInf, kInf};
    const float d0 = a.lo / b.lo, d1 = a.hi / b.lo, d2 = a.lo / b.hi, d3 = a.hi / b.hi;
    return EF{a.v / b.v, next_down(smin(smin(d0, d1), smin(d2, d3))), next_up(smax(smax(d0, d1), smax(d2, d3)))};
}
// Quadratic(EFloat...) (efloat.h:266-287)
__device__ __forceinline__ bool ef_quadratic(EF A, EF B, EF C, EF* t0, EF* t1) {
    const double discrim = (double)B.v * (double)B.v - 4. * (double)A.v * (double)C.v;
    if (discrim < 0.) return false;
    const double rootDiscrim = sqrt(discrim);
    const EF fr = ef_err((float)rootDiscrim, (float)((double)(kMachineEps) * rootDiscrim));
    const EF q = (B.v < 0) ? ef(-.5f) * (B - fr) : ef(-.5f) * (B + fr);
    *t0 = q / A;
    *t1 = C / q;
    if (t0->v > t1->v) { const EF t = *t0; *t0 = *t1; *t1 = t; }
    return true;
}

// Sphere::Intersect / IntersectP up to the accepted hit (sphere.cpp:50-112 /
// 148-200): object-space ray with error bounds, conservative roots, partial
// sphere clipping with the second root.  Returns the hit distance, the
// object-space point and phi.
__device__ __forceinline__ bool sphere_test(const DevSphere& s, const Ray& r, float* tHit, V3* pHitOut) {
    V3 oErr, dErr;
    V3 o = xf_point_err(s.w2o, r.o, &oErr);
    const V3 d = xf_vector_err(s.w2o, r.d, &dErr);
    const float l2 = len2(d);
    if (l2 > 0) {  // Transform::operator()(Ray, oError, dError) (transform.h:382-394)
        const float dt = dot(vabs(d), oErr) / l2;
        o = o + d * dt;
    }
    const EF ox = ef_err(o.x, oErr.x), oy = ef_err(o.y, oErr.y), oz = ef_err(o.z, oErr.z);
    const EF dx = ef_err(d.x, dErr.x), dy = ef_err(d.y, dErr.y), dz = ef_err(d.z, dErr.z);
    const EF a = dx * dx + dy * dy + dz * dz;
    const EF b = ef(2.f) * (dx * ox + dy * oy + dz * oz);
    const EF c = ox * ox + oy * oy + oz * oz - ef(s.radius) * ef(s.radius);
    EF t0, t1;
    if (!ef_quadratic(a, b, c, &t0, &t1)) return false;
    if (t0.hi > r.tmax || t1.lo <= 0) return false;
    EF ts = t0;
    if (ts.lo <= 0) {
        ts = t1;
        if (ts.hi > r.tmax) return false;
    }
    const float twoPi = 2 * kPi;
    V3 pHit = o + d * ts.v;
    pHit = pHit * (s.radius / len(pHit));
    if (pHit.x == 0 && pHit.y == 0) pHit.x = 1e-5f * s.radius;
    float phi = libm_atan2f(pHit.y, pHit.x);
    if (phi < 0) phi += twoPi;
    if ((s.zmin > -s.radius && pHit.z < s.zmin) || (s.zmax < s.radius && pHit.z > s.zmax) || phi > s.phi_max) {
        if (ts.v == t1.v) return false;
        if (t1.hi > r.tmax) return false;
        ts = t1;
        pHit = o + d * ts.v;
        pHit = pHit * (s.radius / len(pHit));
        if (pHit.x == 0 && pHit.y == 0) pHit.x = 1e-5f * s.radius;
        phi = libm_atan2f(pHit.y, pHit.x);
        if (phi < 0) phi += twoPi;
        if ((s.zmin > -s.radius && pHit.z < s.zmin) || (s.zmax < s.radius && pHit.z > s.zmax) || phi > s.phi_max)
            return false;
    }
    *tHit = ts.v;
    *pHitOut = pHit;
    return true;
}

// SurfaceInteraction of Sphere::Intersect (sphere.cpp:114-140), to world space
// (transform.cpp:262-297).  Only what shading reads: p, pError, n, shading
// n and dpdu.
__device__ __forceinline__ bool sphere_surface(const DevSphere& s, const Ray& ray, SurfHit* si) {
    Ray r2 = ray;
    r2.tmax = kInf;
    float t;
    V3 pHit;
    if (!sphere_test(s, r2, &t, &pHit)) return false;
    const float theta = libm_acosf(clamp11(pHit.z / s.radius));
    const float zRadius = sqrtf(pHit.x * pHit.x + pHit.y * pHit.y);
    const float invZRadius = 1 / zRadius;
    const float cosPhi = pHit.x * invZRadius, sinPhi = pHit.y * invZRadius;
    const V3 dpdu = v3(-s.phi_max * pHit.y, s.phi_max * pHit.x, 0);
    const V3 dpdv = (s.theta_max - s.theta_min) * v3(pHit.z * cosPhi, pHit.z * sinPhi, -s.radius * libm_sinf(theta));
    V3 n = normalize(cross(dpdu, dpdv));
    if (s.ro_xor_sh) n = n * -1.f;
    const V3 pError = gammaf(5) * vabs(pHit);
    si->p = xf_point_err_in(s.o2w, pHit, pError, &si->perr);
    si->n = normalize(xf_normal(s.w2o, n));
    si->wo = normalize(xf_vector(s.o2w, normalize(-xf_vector(s.w2o, ray.d))));  // Interaction ctor normalises wo
    si->sn = faceforward(si->n, si->n);
    si->sdpdu = xf_vector(s.o2w, dpdu);
    return true;
}

// Leaf test of a non-triangle primitive record (plane, or sphere when the
// kernel is compiled with kSph).
template <bool kSph = true>
__device__ __forceinline__ bool shape_test(const DevScene& sc, uint32_t flags, int idx, const Ray& ray, float* t) {
    V3 ph;
    if (kSph && (flags & kPrimSphere)) return sphere_test(sc.spheres[PT_IDX(idx, sc.n_spheres)], ray, t, &ph);
    return plane_test(sc.planes[PT_IDX(idx, sc.n_planes)], ray, t, &ph);
}

// surface_at / prim_info from the primitive's first two record words when the
// caller has them already (k_shade loads them one path ahead)
// A primitive's 48-byte record (BVH order): words 0-2 .xyz hold a
// triangle's world vertices -- the same floats as the vertex array
// (TriangleMesh, triangle.cpp:75) -- and the .w words its flags, shape index
// and packed material / area light (device.h kPrimTriShift, prim_info_word).
struct PrimRec {
    float4 r0, r1, r2;
};
__device__ __forceinline__ PrimRec prim_rec(const DevScene& sc, int prim) {
    const float4* p = sc.prims + 3 * PT_IDX(prim, sc.n_prims);
    return PrimRec{p[0], p[1], p[2]};
}

template <bool kSph = true>
__device__ __forceinline__ bool surface_at(const DevScene& sc, int prim, const PrimRec& rec, const Ray& ray,
                                           SurfHit* si) {
    uint32_t flags = __float_as_uint(rec.r0.w);
    int idx = __float_as_int(rec.r1.w);
    bool ok;
    if (kSph && (flags & kPrimSphere)) ok = sphere_surface(sc.spheres[PT_IDX(idx, sc.n_spheres)], ray, si);
    else if (flags & kPrimPlane) ok = plane_surface(sc.planes[PT_IDX(idx, sc.n_planes)], ray, si);
    else  // a triangle record: only here is idx a triangle index (analytic records hold a shape index)
        ok = tri_surface(sc, idx, (flags >> kPrimTriShift) & 31u, ray, si, v3(rec.r0.x, rec.r0.y, rec.r0.z),
                         v3(rec.r1.x, rec.r1.y, rec.r1.z), v3(rec.r2.x, rec.r2.y, rec.r2.z));
    si->prim = prim;
    return ok;
}
template <bool kSph = true>
__device__ __forceinline__ bool surface_at(const DevScene& sc, int prim, const Ray& ray, SurfHit* si) {
    return surface_at<kSph>(sc, prim, prim_rec(sc, prim), ray, si);
}

template <bool kSph = true>
__device__ __forceinline__ void prim_info(const DevScene& sc, const PrimRec& rec, int* material, int* light) {
    uint32_t flags = __float_as_uint(rec.r0.w);
    if (!(flags & kPrimInfoTable)) {  // GeometricPrimitive's material / area light from the record
        const uint32_t w = __float_as_uint(rec.r2.w);
        *material = (int)(w & 0xffffu);
        *light = (int)(w >> 16) - 1;
        return;
    }
    int idx = __float_as_int(rec.r1.w);
    if (kSph && (flags & kPrimSphere)) {
        *material = sc.spheres[PT_IDX(idx, sc.n_spheres)].material;
        *light = sc.spheres[PT_IDX(idx, sc.n_spheres)].area_light;
    } else if (flags & kPrimPlane) {
        *material = sc.planes[PT_IDX(idx, sc.n_planes)].material;
        *light = sc.planes[PT_IDX(idx, sc.n_planes)].area_light;
    } else {
        const pt_triangle& t = sc.tris[PT_IDX(idx, sc.n_tris)];
        *material = t.material;
        *light = t.area_light;
    }
}
template <bool kSph = true>
__device__ __forceinline__ void prim_info(const DevScene& sc, int prim, int* material, int* light) {
    prim_info<kSph>(sc, prim_rec(sc, prim), material, light);
}

// ----------------------------------------------------------------------------
// BSDF: MatteMaterial (matte.cpp:45-62) -> BSDF{LambertianReflection}
// (reflection.h:167-213, reflection.cpp:211-213, 416-427, 713-829)
// ----------------------------------------------------------------------------
// ----------------------------------------------------------------------------
// Shading-frame trigonometry (reflection.h:55-90) and the Trowbridge-Reitz
// microfacet distribution (microfacet.h:105-133, microfacet.cpp:155-345)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float cos2_theta(V3 w) { return w.z * w.z; }
__device__ __forceinline__ float sin2_theta(V3 w) { return smax(0.f, 1.f - cos2_theta(w)); }
__device__ __forceinline__ float sin_theta(V3 w) { return sqrtf(sin2_theta(w)); }
__device__ __forceinline__ float tan_theta(V3 w) { return sin_theta(w) / w.z; }
__device__ __forceinline__ float tan2_theta(V3 w) { return sin2_theta(w) / cos2_theta(w); }
__device__ __forceinline__ float cos_phi(V3 w) {
    const float st = sin_theta(w);
    return (st == 0) ? 1.f : clamp11(w.x / st);
}
__device__ __forceinline__ float sin_phi(V3 w) {
    const float st = sin_theta(w);
    return (st == 0) ? 0.f : clamp11(w.y / st);
}
__device__ __forceinline__ float cos2_phi(V3 w) { return cos_phi(w) * cos_phi(w); }
__device__ __forceinline__ float sin2_phi(V3 w) { return sin_phi(w) * sin_phi(w); }

__device__ __forceinline__ float tr_D(float ax, float ay, V3 wh) {
    const float t2 = tan2_theta(wh);
    if (__builtin_isinf(t2)) return 0.f;
    const float cos4 = cos2_theta(wh) * cos2_theta(wh);
    const float e = (cos2_phi(wh) / (ax * ax) + sin2_phi(wh) / (ay * ay)) * t2;
    return 1 / (kPi * ax * ay * cos4 * (1 + e) * (1 + e));
}
__device__ __forceinline__ float tr_lambda(float ax, float ay, V3 w) {
    const float at = fabsf(tan_theta(w));
    if (__builtin_isinf(at)) return 0.f;
    const float alpha = sqrtf(cos2_phi(w) * ax * ax + sin2_phi(w) * ay * ay);
    const float a2t2 = (alpha * at) * (alpha * at);
    return (-1 + sqrtf(1.f + a2t2)) / 2;
}
__device__ __forceinline__ float tr_G1(float ax, float ay, V3 w) { return 1 / (1 + tr_lambda(ax, ay, w)); }
__device__ __forceinline__ float tr_G(float ax, float ay, V3 wo, V3 wi) {
    return 1 / (1 + tr_lambda(ax, ay, wo) + tr_lambda(ax, ay, wi));
}
// TrowbridgeReitzSample11 (microfacet.cpp:238-282).  The normal-incidence
// branch calls the double-precision sqrt/cos/sin of <math.h> on float
// arguments, as the reference's unqualified calls resolve.
__device__ __forceinline__ void tr_sample11(float cosTheta, float U1, float U2, float* sx, float* sy) {
    if ((double)cosTheta > .9999) {
        const float r = (float)sqrt((double)(U1 / (1 - U1)));
        const float phi = (float)(6.28318530718 * (double)U2);
        *sx = (float)((double)r * dcos_mod((double)phi));
        *sy = (float)((double)r * dsin_mod((double)phi));
        return;
    }
    const float sinTheta = sqrtf(smax(0.f, 1.f - cosTheta * cosTheta));
    const float tanTheta = sinTheta / cosTheta;
    const float a = 1 / tanTheta;
    const float G1 = 2 / (1 + sqrtf(1.f + 1.f / (a * a)));
    const float A = 2 * U1 / G1 - 1;
    float tmp = 1.f / (A * A - 1.f);
    if ((double)tmp > 1e10) tmp = (float)1e10;
    const float B = tanTheta;
    const float D = sqrtf(smax(B * B * tmp * tmp - (A * A - B * B) * tmp, 0.f));
    const float sx1 = B * tmp - D;
    const float sx2 = B * tmp + D;
    *sx = (A < 0 || sx2 > 1.f / tanTheta) ? sx1 : sx2;
    float S;
    if (U2 > 0.5f) { S = 1.f; U2 = 2.f * (U2 - .5f); }
    else { S = -1.f; U2 = 2.f * (.5f - U2); }
    const float z = (U2 * (U2 * (U2 * 0.27385f - 0.73369f) + 0.46341f)) /
                    (U2 * (U2 * (U2 * 0.093073f + 0.309420f) - 1.000000f) + 0.597999f);
    *sy = S * z * sqrtf(1.f + *sx * *sx);
}
__device__ __forceinline__ V3 tr_sample_wh(float ax, float ay, V3 wo, float u0, float u1) {  // visible normals
    const bool flip = wo.z < 0;
    const V3 wi = flip ? -wo : wo;
    const V3 ws = normalize(v3(ax * wi.x, ay * wi.y, wi.z));
    float sx, sy;
    tr_sample11(ws.z, u0, u1, &sx, &sy);
    const float tmp = cos_phi(ws) * sx - sin_phi(ws) * sy;
    sy = sin_phi(ws) * sx + cos_phi(ws) * sy;
    sx = tmp;
    sx = ax * sx;
    sy = ay * sy;
    V3 wh = normalize(v3(-sx, -sy, 1.f));
    if (flip) wh = -wh;
    return wh;
}
__device__ __forceinline__ float tr_pdf(float ax, float ay, V3 wo, V3 wh) {  // MicrofacetDistribution::Pdf
    return tr_D(ax, ay, wh) * tr_G1(ax, ay, wo) * absdot(wo, wh) / fabsf(wo.z);
}
// FrConductor with etaI = 1 (reflection.cpp:71-96)
__device__ __forceinline__ S3 fr_conductor(float cosThetaI, S3 etat, S3 k) {
    cosThetaI = clamp11(cosThetaI);
    const S3 eta = etat / s3(1.f);
    const S3 etak = k / s3(1.f);
    const float c2 = cosThetaI * cosThetaI;
    const float s2 = 1.f - c2;
    const S3 eta2 = eta * eta, etak2 = etak * etak;
    const S3 t0 = eta2 - etak2 - s3(s2);
    const S3 a2b2 = ssqrt(t0 * t0 + (eta2 * 4.f) * etak2);
    const S3 t1 = a2b2 + s3(c2);
    const S3 a = ssqrt((a2b2 + t0) * 0.5f);
    const S3 t2 = a * ((float)2 * cosThetaI);
    const S3 Rs = (t1 - t2) / (t1 + t2);
    const S3 t3 = a2b2 * c2 + s3(s2 * s2);
    const S3 t4 = t2 * s2;
    const S3 Rp = Rs * (t3 - t4) / (t3 + t4);
    return (Rp + Rs) * 0.5f;
}

// ----------------------------------------------------------------------------
// BSDF (reflection.{h,cpp}) with up to two BxDFs ("lobes"), built by the
// materials matte.cpp, metal.cpp, glass.cpp, dispersive_glass.cpp (bsdf[0]),
// mirror.cpp, plastic.cpp.  Lobe parameters are read from the material record
// when evaluated.
// ----------------------------------------------------------------------------
constexpr int kBxR = 1, kBxT = 2, kBxDiffuse = 4, kBxGlossy = 8, kBxSpecular = 16, kBxAll = 31;  // BxDFType
constexpr int kBxNonSpecular = kBxAll & ~kBxSpecular;
// kLbSpecRefl: SpecularReflection with FresnelNoOp (mirror); kLbSpecReflD / kLbSpecTrans:
// SpecularReflection(FresnelDielectric) / SpecularTransmission, the smooth
// dielectric when allowMultipleLobes is false (DirectLightingIntegrator).
enum LobeKind { kLbLambert = 1, kLbMfRefl = 2, kLbMfTrans = 3, kLbFresnelSpec = 4, kLbSpecRefl = 5, kLbSpecReflD = 6,
                kLbSpecTrans = 7 };

// Scene features the shading code is compiled for (template argument kFt).
// The host picks the smallest instantiation covering the scene (render.hip,
// scene_features); code for absent materials / lights is compiled out, which
// cuts the shading kernel's register pressure for the all-matte scenes.
enum : int {
    kFtMicro = 1,       // metal, plastic, rough glass: microfacet lobes, two-lobe BSDFs
    kFtSpecular = 2,    // smooth glass, dispersive glass, mirror: specular lobes
    kFtInfinite = 4,    // an InfiniteAreaLight
    kFtSphere = 8,      // Sphere shapes (and sphere area lights)
    kFtAll = 15,
    // a reduction, outside kFtAll: every light is a PortalArealight, so the
    // path kernel leaves EstimateDirect's MIS branch out (fewer live registers)
    kFtPortalOnly = 16
};
template <int kFt>
struct Ft {
    static constexpr bool micro = (kFt & kFtMicro) != 0;
    static constexpr bool spec = (kFt & kFtSpecular) != 0;
    static constexpr bool inf = (kFt & kFtInfinite) != 0;
    static constexpr bool sph = (kFt & kFtSphere) != 0;
    static constexpr bool mis = (kFt & kFtPortalOnly) == 0;  // lights sampled by the MIS branch may occur
    static constexpr int max_lobes = (micro || spec) ? 2 : 1;
};

__device__ __forceinline__ int lobe_type(int k) {
    switch (k) {
        case kLbLambert: return kBxR | kBxDiffuse;
        case kLbMfRefl: return kBxR | kBxGlossy;
        case kLbMfTrans: return kBxT | kBxGlossy;
        case kLbFresnelSpec: return kBxR | kBxT | kBxSpecular;
        case kLbSpecTrans: return kBxT | kBxSpecular;
        default: return kBxR | kBxSpecular;
    }
}
__device__ __forceinline__ S3 clamp0(S3 r) {  // Spectrum::Clamp()
    for (int i = 0; i < 3; ++i) r.c[i] = r.c[i] < 0 ? 0 : r.c[i];
    return r;
}

struct Bsdf {
    int n;
    int lk0, lk1;          // lobe kinds in BSDF::Add order (distinct within a BSDF)
    float eta;             // BSDF::eta
    const pt_material* m;
    V3 ns, ng, ss, ts;
    // the material's constant Kd / Kr / Kt, held by value: the hero
    // integrators overwrite them per 3-bin chunk of the 60-bin reflectances
    // (a private material copy behind `m` would live in scratch)
    S3 rkd, rkr, rkt;
};

__device__ __forceinline__ V3 refl_z(V3 wo) { return v3(-wo.x, -wo.y, wo.z); }
// FrDielectric (reflection.cpp:47-69)
__device__ __forceinline__ float fr_dielectric(float cosThetaI, float etaI, float etaT) {
    cosThetaI = clamp11(cosThetaI);
    if (!(cosThetaI > 0.f)) {
        const float t = etaI; etaI = etaT; etaT = t;
        cosThetaI = fabsf(cosThetaI);
    }
    const float sinThetaI = sqrtf(smax(0.f, 1 - cosThetaI * cosThetaI));
    const float sinThetaT = etaI / etaT * sinThetaI;
    if (sinThetaT >= 1) return 1;
    const float cosThetaT = sqrtf(smax(0.f, 1 - sinThetaT * sinThetaT));
    const float Rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    const float Rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) / 2;
}
// Refract (reflection.h:97-108)
__device__ __forceinline__ bool refract(V3 wi, V3 n, float eta, V3* wt) {
    const float cosThetaI = dot(n, wi);
    const float sin2ThetaI = smax(0.f, 1 - cosThetaI * cosThetaI);
    const float sin2ThetaT = eta * eta * sin2ThetaI;
    if (sin2ThetaT >= 1) return false;
    const float cosThetaT = sqrtf(1 - sin2ThetaT);
    *wt = (-wi) * eta + n * (eta * cosThetaI - cosThetaT);
    return true;
}
// Scale (R or T) and Fresnel term of the MicrofacetReflection lobe
__device__ __forceinline__ S3 mfrefl_R(const Bsdf& b) {
    const pt_material* m = b.m;
    if (m->kind == PT_MAT_METAL) return s3(1.f);
    if (m->kind == PT_MAT_PLASTIC) return clamp0(s3(m->ks[0], m->ks[1], m->ks[2]));
    return clamp0(b.rkr);
}
__device__ __forceinline__ S3 mfrefl_F(const Bsdf& b, float cosThetaI) {
    const pt_material* m = b.m;
    if (m->kind == PT_MAT_METAL)  // FresnelConductor::Evaluate (reflection.cpp:118-120)
        return fr_conductor(fabsf(cosThetaI), s3(m->eta[0], m->eta[1], m->eta[2]), s3(m->k[0], m->k[1], m->k[2]));
    if (m->kind == PT_MAT_PLASTIC) return s3(fr_dielectric(cosThetaI, 1.5f, 1.f));
    return s3(fr_dielectric(cosThetaI, 1.f, b.eta));
}
// MicrofacetReflection::f (reflection.cpp:259-271)
__device__ __forceinline__ S3 mfrefl_f(const Bsdf& b, V3 wo, V3 wi) {
    const float cosO = fabsf(wo.z), cosI = fabsf(wi.z);
    V3 wh = wi + wo;
    if (cosI == 0 || cosO == 0) return s3(0.f);
    if (wh.x == 0 && wh.y == 0 && wh.z == 0) return s3(0.f);
    wh = normalize(wh);
    const V3 whf = dot(wh, v3(0, 0, 1)) < 0.f ? -wh : wh;  // Faceforward(wh, (0,0,1))
    const S3 F = mfrefl_F(b, dot(wi, whf));
    const float ax = b.m->alpha[0], ay = b.m->alpha[1];
    return mfrefl_R(b) * tr_D(ax, ay, wh) * tr_G(ax, ay, wo, wi) * F / (4 * cosI * cosO);
}
// MicrofacetTransmission::f / Pdf (reflection.cpp:279-303, 479-493); etaA = 1, etaB = eta
__device__ __forceinline__ S3 mftrans_f(const Bsdf& b, V3 wo, V3 wi) {
    if (wo.z * wi.z > 0) return s3(0.f);
    const float cosO = wo.z, cosI = wi.z;
    if (cosI == 0 || cosO == 0) return s3(0.f);
    const float eta = wo.z > 0 ? (b.eta / 1.f) : (1.f / b.eta);
    V3 wh = normalize(wo + wi * eta);
    if (wh.z < 0) wh = -wh;
    if (dot(wo, wh) * dot(wi, wh) > 0) return s3(0.f);
    const S3 F = s3(fr_dielectric(dot(wo, wh), 1.f, b.eta));
    const float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
    const float factor = 1 / eta;  // TransportMode::Radiance
    const float ax = b.m->alpha[0], ay = b.m->alpha[1];
    const float v = fabsf(tr_D(ax, ay, wh) * tr_G(ax, ay, wo, wi) * eta * eta * absdot(wi, wh) * absdot(wo, wh) *
                          factor * factor / (cosI * cosO * sqrtDenom * sqrtDenom));
    return ((s3(1.f) - F) * clamp0(b.rkt)) * v;
}
__device__ __forceinline__ float mftrans_pdf(const Bsdf& b, V3 wo, V3 wi) {
    if (wo.z * wi.z > 0) return 0;
    const float eta = wo.z > 0 ? (b.eta / 1.f) : (1.f / b.eta);
    const V3 wh = normalize(wo + wi * eta);
    if (dot(wo, wh) * dot(wi, wh) > 0) return 0;
    const float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
    const float dwh_dwi = fabsf((eta * eta * dot(wi, wh)) / (sqrtDenom * sqrtDenom));
    return tr_pdf(b.m->alpha[0], b.m->alpha[1], wo, wh) * dwh_dwi;
}
__device__ __forceinline__ S3 lambert_R(const Bsdf& b) { return clamp0(b.rkd); }

template <int kFt = kFtAll>
__device__ __forceinline__ S3 lobe_f(const Bsdf& b, int k, V3 wo, V3 wi) {  // BxDF::f
    if (k == kLbLambert || !(Ft<kFt>::micro || Ft<kFt>::spec)) return lambert_R(b) * kInvPi;
    if (!Ft<kFt>::micro) return s3(0.f);  // specular lobes: f = 0
    if (k == kLbMfRefl) return mfrefl_f(b, wo, wi);
    if (k == kLbMfTrans) return mftrans_f(b, wo, wi);
    return s3(0.f);
}
template <int kFt = kFtAll>
__device__ __forceinline__ float lobe_pdf(const Bsdf& b, int k, V3 wo, V3 wi) {  // BxDF::Pdf
    if (k == kLbLambert || !(Ft<kFt>::micro || Ft<kFt>::spec)) return (wo.z * wi.z > 0) ? fabsf(wi.z) * kInvPi : 0;
    if (!Ft<kFt>::micro) return 0.f;  // specular lobes: pdf = 0
    if (k == kLbMfRefl) {
        if (!(wo.z * wi.z > 0)) return 0.f;
        const V3 wh = normalize(wo + wi);
        return tr_pdf(b.m->alpha[0], b.m->alpha[1], wo, wh) / (4 * dot(wo, wh));
    }
    if (k == kLbMfTrans) return mftrans_pdf(b, wo, wi);
    return 0.f;
}
// BxDF::Sample_f; *type narrowed by FresnelSpecular.  Non-specular lobes only
// when the scene has no specular materials (kFt without kFtSpecular).
template <int kFt = kFtAll>
__device__ __forceinline__ S3 lobe_sample(const Bsdf& b, int k, V3 wo, V3* wi, float u0, float u1, float* pdf,
                                          int* type) {
    const pt_material* m = b.m;
    if (k == kLbLambert || !(Ft<kFt>::micro || Ft<kFt>::spec)) {
        *wi = cosine_sample_hemisphere(u0, u1);
        if (wo.z < 0) wi->z *= -1;
        *pdf = lobe_pdf<kFt>(b, kLbLambert, wo, *wi);
        return lobe_f<kFt>(b, kLbLambert, wo, *wi);
    }
    if (Ft<kFt>::micro && (k == kLbMfRefl || k == kLbMfTrans || !Ft<kFt>::spec)) {
        const float ax = m->alpha[0], ay = m->alpha[1];
        if (wo.z == 0) return s3(0.f);
        const V3 wh = tr_sample_wh(ax, ay, wo, u0, u1);
        if (dot(wo, wh) < 0) return s3(0.f);
        if (k == kLbMfRefl) {
            *wi = -wo + (2 * dot(wo, wh)) * wh;  // Reflect
            if (!(wo.z * wi->z > 0)) return s3(0.f);
            *pdf = tr_pdf(ax, ay, wo, wh) / (4 * dot(wo, wh));
            return mfrefl_f(b, wo, *wi);
        }
        const float eta = wo.z > 0 ? (1.f / b.eta) : (b.eta / 1.f);
        if (!refract(wo, wh, eta, wi)) return s3(0.f);
        *pdf = mftrans_pdf(b, wo, *wi);
        return mftrans_f(b, wo, *wi);
    }
    if (!Ft<kFt>::spec) return s3(0.f);
    if (k == kLbSpecRefl) {  // SpecularReflection::Sample_f, FresnelNoOp
        *wi = refl_z(wo);
        *pdf = 1;
        return (s3(1.f) * clamp0(b.rkr)) / fabsf(wi->z);
    }
    if (k == kLbSpecReflD) {  // SpecularReflection::Sample_f (reflection.h:400-410), FresnelDielectric(1, eta)
        *wi = refl_z(wo);
        *pdf = 1;
        return (s3(fr_dielectric(wi->z, 1.f, b.eta)) * clamp0(b.rkr)) / fabsf(wi->z);
    }
    if (k == kLbSpecTrans) {  // SpecularTransmission::Sample_f (reflection.cpp:183-199), etaA = 1, etaB = eta
        const bool entering = wo.z > 0;
        const float etaI = entering ? 1.f : b.eta;
        const float etaT = entering ? b.eta : 1.f;
        const V3 n = dot(v3(0, 0, 1), wo) < 0.f ? v3(0, 0, -1) : v3(0, 0, 1);  // Faceforward(n, wo)
        if (!refract(wo, n, etaI / etaT, wi)) return s3(0.f);
        *pdf = 1;
        S3 ft = clamp0(b.rkt) * (s3(1.f) - s3(fr_dielectric(wi->z, 1.f, b.eta)));
        ft = ft * ((etaI * etaI) / (etaT * etaT));  // TransportMode::Radiance
        return ft / fabsf(wi->z);
    }
    // FresnelSpecular::Sample_f (reflection.cpp:520-554), etaA = 1, etaB = eta
    const float F = fr_dielectric(wo.z, 1.f, b.eta);
    if (u0 < F) {
        *wi = refl_z(wo);
        *type = kBxSpecular | kBxR;
        *pdf = F;
        return (clamp0(b.rkr) * F) / fabsf(wi->z);
    }
    const bool entering = wo.z > 0;
    const float etaI = entering ? 1.f : b.eta;
    const float etaT = entering ? b.eta : 1.f;
    const V3 n = dot(v3(0, 0, 1), wo) < 0.f ? v3(0, 0, -1) : v3(0, 0, 1);  // Faceforward(n, wo)
    if (!refract(wo, n, etaI / etaT, wi)) return s3(0.f);
    S3 ft = clamp0(b.rkt) * (1 - F);
    ft = ft * ((etaI * etaI) / (etaT * etaT));  // TransportMode::Radiance
    *type = kBxSpecular | kBxT;
    *pdf = 1 - F;
    return ft / fabsf(wi->z);
}

__device__ __forceinline__ void add_lobe(Bsdf* b, int k) {
    if (b->n == 0) b->lk0 = k;
    else b->lk1 = k;
    ++b->n;
}
// Material::ComputeScatteringFunctions(..., Radiance, allowMultipleLobes = true)
// + BSDF ctor (reflection.h:167-172).  wvl0: the camera's hero wavelength.
template <int kFt = kFtAll>
__device__ __forceinline__ void make_bsdf(const pt_material* m, const SurfHit& si, float wvl0, Bsdf* b,
                                          bool multi = true) {
    b->ns = si.sn;
    b->ng = si.n;
    b->ss = normalize(si.sdpdu);
    b->ts = cross(b->ns, b->ss);
    b->m = m;
    b->rkd = s3(m->kd[0], m->kd[1], m->kd[2]);
    b->rkr = s3(m->kr[0], m->kr[1], m->kr[2]);
    b->rkt = s3(m->kt[0], m->kt[1], m->kt[2]);
    b->n = 0;
    b->lk0 = b->lk1 = 0;
    b->eta = 1;
    const int kind = m->kind;
    if (kind == PT_MAT_MATTE || !(Ft<kFt>::micro || Ft<kFt>::spec)) {
        if (!is_black(lambert_R(*b))) add_lobe(b, kLbLambert);
    } else if (Ft<kFt>::micro && kind == PT_MAT_METAL) {
        add_lobe(b, kLbMfRefl);
    } else if (Ft<kFt>::spec && kind == PT_MAT_MIRROR) {
        if (!is_black(clamp0(s3(m->kr[0], m->kr[1], m->kr[2])))) add_lobe(b, kLbSpecRefl);
    } else if (Ft<kFt>::micro && kind == PT_MAT_PLASTIC) {
        if (!is_black(lambert_R(*b))) add_lobe(b, kLbLambert);
        if (!is_black(clamp0(s3(m->ks[0], m->ks[1], m->ks[2])))) add_lobe(b, kLbMfRefl);
    } else if (kind == PT_MAT_GLASS || kind == PT_MAT_DISPERSIVE_GLASS) {
        float eta = m->ior;
        if (kind == PT_MAT_DISPERSIVE_GLASS) {  // Cauchy's equation (dispersive_glass.cpp:62-73)
            const float lminsq = (float)(400 * 400), lmaxsq = (float)(700 * 700);
            const float cauchyB = (lminsq * m->ior_max - lmaxsq * m->ior_min) / (lminsq - lmaxsq);
            const float cauchyC = lminsq * (m->ior_max - cauchyB);
            eta = cauchyB + cauchyC / (wvl0 * wvl0);
        }
        b->eta = eta;
        const bool hasR = !is_black(clamp0(s3(m->kr[0], m->kr[1], m->kr[2])));
        const bool hasT = !is_black(clamp0(s3(m->kt[0], m->kt[1], m->kt[2])));
        if (!hasR && !hasT) return;
        if (Ft<kFt>::spec && (m->specular || !Ft<kFt>::micro)) {
            if (multi) add_lobe(b, kLbFresnelSpec);
            else {  // glass.cpp:66-83 with isSpecular
                if (hasR) add_lobe(b, kLbSpecReflD);
                if (hasT) add_lobe(b, kLbSpecTrans);
            }
        } else if (Ft<kFt>::micro) {
            if (hasR) add_lobe(b, kLbMfRefl);
            if (hasT) add_lobe(b, kLbMfTrans);
        }
    }
}
__device__ __forceinline__ V3 w2l(const Bsdf& b, V3 v) { return v3(dot(v, b.ss), dot(v, b.ts), dot(v, b.ns)); }
__device__ __forceinline__ int lobe_at(const Bsdf& b, int i) { return i == 0 ? b.lk0 : b.lk1; }
__device__ __forceinline__ V3 l2w(const Bsdf& b, V3 v) {
    return v3(b.ss.x * v.x + b.ts.x * v.y + b.ns.x * v.z, b.ss.y * v.x + b.ts.y * v.y + b.ns.y * v.z,
              b.ss.z * v.x + b.ts.z * v.y + b.ns.z * v.z);
}
__device__ __forceinline__ bool lobe_matches(int k, int flags) { return (lobe_type(k) & flags) == lobe_type(k); }
template <int kFt = kFtAll>
__device__ __forceinline__ int bsdf_num(const Bsdf& b, int flags) {  // BSDF::NumComponents
    int n = 0;
    for (int i = 0; i < Ft<kFt>::max_lobes; ++i)
        if (i < b.n) n += lobe_matches(lobe_at(b, i), flags) ? 1 : 0;
    return n;
}
template <int kFt = kFtAll>
__device__ __forceinline__ S3 bsdf_f(const Bsdf& b, V3 woW, V3 wiW, int flags) {  // reflection.cpp:713-726
    const V3 wo = w2l(b, woW), wi = w2l(b, wiW);
    if (wo.z == 0) return s3(0.f);
    const bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    S3 f = s3(0.f);
    for (int i = 0; i < Ft<kFt>::max_lobes; ++i) {
        if (i >= b.n) break;
        const int k = lobe_at(b, i), t = lobe_type(k);
        if (lobe_matches(k, flags) && ((reflect && (t & kBxR)) || (!reflect && (t & kBxT))))
            f = f + lobe_f<kFt>(b, k, wo, wi);
    }
    return f;
}
template <int kFt = kFtAll>
__device__ __forceinline__ float bsdf_pdf(const Bsdf& b, V3 woW, V3 wiW, int flags) {  // reflection.cpp:814-829
    if (b.n == 0) return 0.f;
    const V3 wo = w2l(b, woW), wi = w2l(b, wiW);
    if (wo.z == 0) return 0.f;
    float pdf = 0.f;
    int matching = 0;
    for (int i = 0; i < Ft<kFt>::max_lobes; ++i) {
        if (i >= b.n) break;
        const int k = lobe_at(b, i);
        if (lobe_matches(k, flags)) { ++matching; pdf += lobe_pdf<kFt>(b, k, wo, wi); }
    }
    return matching > 0 ? pdf / matching : 0.f;
}
// BSDF::Sample_f (reflection.cpp:747-812); *pdf stays 0 wherever the reference
// returns black before writing it; *sampled is the sampled BxDFType.
template <int kFt = kFtAll>
__device__ __forceinline__ S3 bsdf_sample(const Bsdf& b, V3 woW, V3* wiW, float u0, float u1, float* pdf, int flags,
                                          int* sampled, V3* wiLocal = nullptr) {
    const int matchingComps = bsdf_num<kFt>(b, flags);
    if (matchingComps == 0) { *pdf = 0; *sampled = 0; return s3(0.f); }
    int comp = (int)floorf(u0 * matchingComps);
    comp = comp < matchingComps - 1 ? comp : matchingComps - 1;
    int bk = b.lk0, count = comp;
    for (int i = 0; i < Ft<kFt>::max_lobes; ++i) {
        if (i >= b.n) break;
        if (lobe_matches(lobe_at(b, i), flags) && count-- == 0) { bk = lobe_at(b, i); break; }
    }
    const float ur0 = smin(u0 * matchingComps - comp, kOneMinusEps);
    const V3 wo = w2l(b, woW);
    if (wo.z == 0) { *sampled = 0; return s3(0.f); }
    *pdf = 0;
    *sampled = lobe_type(bk);
    V3 wi = v3(0, 0, 0);
    S3 f = lobe_sample<kFt>(b, bk, wo, &wi, ur0, u1, pdf, sampled);
    if (*pdf == 0) { *sampled = 0; return s3(0.f); }
    *wiW = l2w(b, wi);
    if (wiLocal) *wiLocal = wi;
    const bool spec = (lobe_type(bk) & kBxSpecular) != 0;
    if (!spec && matchingComps > 1)
        for (int i = 0; i < Ft<kFt>::max_lobes; ++i) {
            if (i >= b.n) break;
            const int k = lobe_at(b, i);
            if (k != bk && lobe_matches(k, flags)) *pdf += lobe_pdf<kFt>(b, k, wo, wi);
        }
    if (matchingComps > 1) *pdf /= matchingComps;
    if (!spec) {
        const bool reflect = dot(*wiW, b.ng) * dot(woW, b.ng) > 0;
        f = s3(0.f);
        for (int i = 0; i < Ft<kFt>::max_lobes; ++i) {
            if (i >= b.n) break;
            const int k = lobe_at(b, i), t = lobe_type(k);
            if (lobe_matches(k, flags) && ((reflect && (t & kBxR)) || (!reflect && (t & kBxT))))
                f = f + lobe_f<kFt>(b, k, wo, wi);
        }
    }
    return f;
}

// ----------------------------------------------------------------------------
// Lights: DiffuseAreaLight (lights/diffuse.{h,cpp}), AAPlaneShape sampling
// ----------------------------------------------------------------------------
__device__ __forceinline__ S3 area_L(const DevLight& l, V3 n, V3 w) {  // diffuse.h:58-60
    return (l.two_sided || dot(n, w) > 0) ? l.L : s3(0.f);
}

__device__ __forceinline__ V3 plane_normal(const DevPlane& pl) {  // plane.cpp:74-83
    V3 r = v3(0, 0, 0);
    r.set(pl.ax, 1);
    if (!pl.facing_fw) r = r * -1.f;
    return r;
}
__device__ __forceinline__ bool plane_in_front(const DevPlane& pl, V3 p) {  // plane.cpp:109-115
    return pl.facing_fw ? (p[pl.ax] > pl.lo_a) : (p[pl.ax] < pl.lo_a);
}
__device__ __forceinline__ void plane_sample(const DevPlane& pl, float u0, float u1, V3* p, V3* n, V3* perr,
                                             float* pdf) {  // plane.cpp:57-72
    V3 loW = xf_point(pl.o2w, pl.lo), hiW = xf_point(pl.o2w, pl.hi);
    V3 q = v3(0, 0, 0);
    q.set(pl.ax, loW[pl.ax]);
    q.set(pl.ax0, loW[pl.ax0] + (hiW[pl.ax0] - loW[pl.ax0]) * u0);
    q.set(pl.ax1, loW[pl.ax1] + (hiW[pl.ax1] - loW[pl.ax1]) * u1);
    *p = q;
    *n = plane_normal(pl);
    *perr = v3(0.1f, 0.1f, 0.1f);
    *pdf = 1 / pl.area;
}
__device__ __forceinline__ void tri_sample(const DevScene& sc, int ti, float u0, float u1, V3* p, V3* n, V3* perr,
                                           float* pdf) {  // triangle.cpp:584-609
    const pt_triangle tr = sc.tris[PT_IDX(ti, sc.n_tris)];
    float su0 = sqrtf(u0);
    float b0 = 1 - su0, b1 = u1 * su0;
    V3 p0 = vload3(sc.P, PT_IDX(tr.v[0], sc.n_verts)), p1 = vload3(sc.P, PT_IDX(tr.v[1], sc.n_verts)), p2 = vload3(sc.P, PT_IDX(tr.v[2], sc.n_verts));
    float b2 = 1 - b0 - b1;
    *p = (b0 * p0 + b1 * p1) + b2 * p2;
    *n = normalize(cross(p1 - p0, p2 - p0));
    if ((tr.flags & PT_TRI_HAS_N) && sc.N) {
        V3 ns = (b0 * vload3(sc.N, PT_IDX(tr.v[0], sc.n_verts)) + b1 * vload3(sc.N, PT_IDX(tr.v[1], sc.n_verts))) + b2 * vload3(sc.N, PT_IDX(tr.v[2], sc.n_verts));
        *n = faceforward(*n, ns);
    } else if (((tr.flags & PT_TRI_REVERSE_ORIENTATION) != 0) ^ ((tr.flags & PT_TRI_SWAPS_HANDEDNESS) != 0)) {
        *n = *n * -1.f;
    }
    V3 pa = (vabs(b0 * p0) + vabs(b1 * p1)) + vabs(b2 * p2);
    *perr = gammaf(6) * pa;
    *pdf = 1 / sc.tri_area[PT_IDX(ti, sc.n_tris)];
}

// ----------------------------------------------------------------------------
// InfiniteAreaLight with a constant 1x1 Lmap (lights/infinite.cpp:43-132)
// ----------------------------------------------------------------------------
// MIPMap::triangle at level 0 of a 1x1 map, ImageWrap::Repeat (mipmap.h:264-274)
PTHD S3 lmap_triangle(S3 v, float st0, float st1) {
    const float s = st0 * 1 - 0.5f, t = st1 * 1 - 0.5f;
    const int s0 = (int)floorf(s), t0 = (int)floorf(t);
    const float ds = s - s0, dt = t - t0;
    S3 r = v * ((1 - ds) * (1 - dt));
    r = r + v * ((1 - ds) * dt);
    r = r + v * (ds * (1 - dt));
    r = r + v * (ds * dt);
    return r;
}
PTHD float spherical_theta(V3 v) { return libm_acosf(v.z < -1 ? -1.f : (v.z > 1 ? 1.f : v.z)); }  // geometry.h:1636
PTHD float spherical_phi(V3 v) {                                                                  // geometry.h:1640
    const float p = libm_atan2f(v.y, v.x);
    return (p < 0) ? (p + 2 * kPi) : p;
}
constexpr float kInv2Pi = 0.15915494309189533577f;
// Distribution1D::SampleContinuous (sampling.h:71-89) over n entries
PTHD float dist1d_sample_cont(const float* func, const float* cdf, float funcInt, int n, float u, float* pdf, int* off) {
    const int offset = find_interval(cdf, n + 1, u);
    if (off) *off = offset;
    float du = u - cdf[offset];
    if ((cdf[offset + 1] - cdf[offset]) > 0) du /= (cdf[offset + 1] - cdf[offset]);
    if (pdf) *pdf = (funcInt > 0) ? func[offset] / funcInt : 0;
    return (offset + du) / n;
}
// InfiniteAreaLight::Le (infinite.cpp:91-95)
__device__ __forceinline__ S3 inf_Le(const DevLight& l, V3 d) {
    const V3 w = normalize(xf_vector(l.w2l, d));
    return lmap_triangle(l.L, spherical_phi(w) * kInv2Pi, spherical_theta(w) * kInvPi);
}
// InfiniteAreaLight::Sample_Li (infinite.cpp:97-121); *sp is the visibility
// target ref.p + wi * 2 worldRadius (zero error bounds and normal)
__device__ __forceinline__ S3 inf_sample_li(const DevLight& l, V3 refp, float u0, float u1, V3* wi, float* pdf,
                                            V3* sp) {
    float pdf0, pdf1;
    int v;
    const float d1 = dist1d_sample_cont(l.mfunc, l.mcdf, l.mint, 2, u1, &pdf1, &v);
    const float d0 = dist1d_sample_cont(l.cfunc + 2 * v, l.ccdf + 3 * v, l.cint[v], 2, u0, &pdf0, nullptr);
    const float mapPdf = pdf0 * pdf1;
    if (mapPdf == 0) { *pdf = 0; return s3(0.f); }
    const float theta = d1 * kPi, phi = d0 * 2 * kPi;
    const float cosTheta = libm_cosf(theta), sinTheta = libm_sinf(theta);
    const float sinPhi = libm_sinf(phi), cosPhi = libm_cosf(phi);
    *wi = xf_vector(l.l2w, v3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta));
    *pdf = mapPdf / (2 * kPi * kPi * sinTheta);
    if (sinTheta == 0) *pdf = 0;
    *sp = refp + *wi * (2 * l.radius);
    return lmap_triangle(l.L, d0, d1);
}
// InfiniteAreaLight::Pdf_Li (infinite.cpp:123-131) + Distribution2D::Pdf (sampling.h:136-142)
__device__ __forceinline__ float inf_pdf_li(const DevLight& l, V3 w) {
    const V3 wi = xf_vector(l.w2l, w);
    const float theta = spherical_theta(wi), phi = spherical_phi(wi);
    const float sinTheta = libm_sinf(theta);
    if (sinTheta == 0) return 0;
    int iu = (int)(phi * kInv2Pi * 2), iv = (int)(theta * kInvPi * 2);
    iu = iu < 0 ? 0 : (iu > 1 ? 1 : iu);
    iv = iv < 0 ? 0 : (iv > 1 ? 1 : iv);
    return (l.cfunc[2 * iv + iu] / l.mint) / (2 * kPi * kPi * sinTheta);
}

// Sphere::Sample(u, pdf) (sphere.cpp:226-236): uniform area sample
__device__ __forceinline__ void sphere_sample_area(const DevSphere& s, float u0, float u1, V3* p, V3* n, V3* perr,
                                                   float* pdf) {
    // UniformSampleSphere (sampling.cpp:98-103)
    const float z = 1 - 2 * u0;
    const float r = sqrtf(smax(0.f, 1.f - z * z));
    const float phi = 2 * kPi * u1;
    const V3 w = v3(r * libm_cosf(phi), r * libm_sinf(phi), z);
    V3 pObj = v3(0, 0, 0) + w * s.radius;
    *n = normalize(xf_normal(s.w2o, pObj));
    if (s.ro) *n = *n * -1.f;
    pObj = pObj * (s.radius / len(pObj));
    const V3 pObjError = gammaf(5) * vabs(pObj);
    *p = xf_point_err_in(s.o2w, pObj, pObjError, perr);
    *pdf = 1 / s.area;
}

// Sphere::Sample(ref, u, pdf) (sphere.cpp:238-301): area sampling from inside,
// else uniform sampling of the subtended cone (with the small-angle branch).
__device__ __forceinline__ void sphere_sample_ref(const DevSphere& s, const SurfHit& ref, float u0, float u1, V3* p,
                                                  V3* n, V3* perr, float* pdf) {
    const V3 pCenter = s.center;
    const V3 pOrigin = offset_ray_origin(ref.p, ref.perr, ref.n, pCenter - ref.p);
    if (dist2(pOrigin, pCenter) <= s.radius * s.radius) {
        sphere_sample_area(s, u0, u1, p, n, perr, pdf);
        V3 wi = *p - ref.p;
        if (len2(wi) == 0) *pdf = 0;
        else {
            wi = normalize(wi);
            *pdf *= dist2(ref.p, *p) / absdot(*n, -wi);
        }
        if (__builtin_isinf(*pdf)) *pdf = 0.f;
        return;
    }
    const float dc = len(ref.p - pCenter);
    const float invDc = 1 / dc;
    const V3 wc = (pCenter - ref.p) * invDc;
    V3 wcX, wcY;
    coordinate_system(wc, &wcX, &wcY);
    const float sinThetaMax = s.radius * invDc;
    const float sinThetaMax2 = sinThetaMax * sinThetaMax;
    const float invSinThetaMax = 1 / sinThetaMax;
    const float cosThetaMax = sqrtf(smax(0.f, 1 - sinThetaMax2));
    float cosTheta = (cosThetaMax - 1) * u0 + 1;
    float sinTheta2 = 1 - cosTheta * cosTheta;
    if (sinThetaMax2 < 0.00068523f) {  // sin^2(1.5 deg): Taylor expansion branch
        sinTheta2 = sinThetaMax2 * u0;
        cosTheta = sqrtf(1 - sinTheta2);
    }
    const float cosAlpha = sinTheta2 * invSinThetaMax +
                           cosTheta * sqrtf(smax(0.f, 1.f - sinTheta2 * invSinThetaMax * invSinThetaMax));
    const float sinAlpha = sqrtf(smax(0.f, 1.f - cosAlpha * cosAlpha));
    const float phi = u1 * 2 * kPi;
    // SphericalDirection(sinAlpha, cosAlpha, phi, -wcX, -wcY, -wc) (geometry.h:1629-1634)
    const V3 nWorld = ((-wcX) * (sinAlpha * libm_cosf(phi)) + (-wcY) * (sinAlpha * libm_sinf(phi))) + (-wc) * cosAlpha;
    const V3 pWorld = pCenter + nWorld * s.radius;
    *p = pWorld;
    *perr = gammaf(5) * vabs(pWorld);
    *n = s.ro ? nWorld * -1.f : nWorld;
    *pdf = 1 / (2 * kPi * (1 - cosThetaMax));
}

// DiffuseAreaLight::Sample_Li + Shape::Sample(ref, u, pdf) (diffuse.cpp:69-84, shape.cpp:56-74)
template <int kFt = kFtAll>
__device__ __forceinline__ S3 area_sample_li(const DevScene& sc, const DevLight& l, const SurfHit& ref, float u0,
                                             float u1, V3* wi, float* pdf, V3* sp, V3* sn, V3* spe) {
    V3 p, n, pe;
    if (Ft<kFt>::inf && l.kind == PT_LIGHT_INFINITE) {
        *sn = v3(0, 0, 0);
        *spe = v3(0, 0, 0);
        return inf_sample_li(l, ref.p, u0, u1, wi, pdf, sp);
    }
    if (l.kind == PT_LIGHT_POINT) {  // PointLight::Sample_Li (point.cpp:41-49)
        *wi = normalize(l.center - ref.p);
        *pdf = 1.f;
        *sp = l.center; *sn = v3(0, 0, 0); *spe = v3(0, 0, 0);
        return l.L / dist2(l.center, ref.p);
    }
    if (Ft<kFt>::sph && l.kind == PT_LIGHT_DIFFUSE_SPHERE) {
        sphere_sample_ref(sc.spheres[PT_IDX(l.shape, sc.n_spheres)], ref, u0, u1, &p, &n, &pe, pdf);
        if (*pdf == 0 || len2(p - ref.p) == 0) { *pdf = 0; return s3(0.f); }
        *wi = normalize(p - ref.p);
        *sp = p; *sn = n; *spe = pe;
        return area_L(l, n, -*wi);
    }
    if (l.kind == PT_LIGHT_DIFFUSE_AREA) tri_sample(sc, l.shape, u0, u1, &p, &n, &pe, pdf);
    else plane_sample(sc.planes[PT_IDX(l.shape, sc.n_planes)], u0, u1, &p, &n, &pe, pdf);
    V3 w = p - ref.p;
    if (len2(w) == 0) *pdf = 0;
    else {
        w = normalize(w);
        *pdf *= dist2(ref.p, p) / absdot(n, -w);
        if (__builtin_isinf(*pdf)) *pdf = 0.f;
    }
    if (*pdf == 0 || len2(p - ref.p) == 0) { *pdf = 0; return s3(0.f); }
    *wi = normalize(p - ref.p);
    *sp = p; *sn = n; *spe = pe;
    return area_L(l, n, -*wi);
}

// Shape::Pdf(ref, wi) for the light's shape (shape.cpp:76-91)
template <int kFt = kFtAll>
__device__ __forceinline__ float area_pdf_li(const DevScene& sc, const DevLight& l, const SurfHit& ref, V3 wi) {
    if (Ft<kFt>::inf && l.kind == PT_LIGHT_INFINITE) return inf_pdf_li(l, wi);
    float area = l.area;
    Ray r{offset_ray_origin(ref.p, ref.perr, ref.n, wi), wi, kInf};
    SurfHit isl;
    bool ok;
    if (Ft<kFt>::sph && l.kind == PT_LIGHT_DIFFUSE_SPHERE) {  // Sphere::Pdf (sphere.cpp:303-315)
        const DevSphere& s = sc.spheres[PT_IDX(l.shape, sc.n_spheres)];
        const V3 pOrigin = offset_ray_origin(ref.p, ref.perr, ref.n, s.center - ref.p);
        if (!(dist2(pOrigin, s.center) <= s.radius * s.radius)) {
            const float sinThetaMax2 = s.radius * s.radius / dist2(ref.p, s.center);
            const float cosThetaMax = sqrtf(smax(0.f, 1 - sinThetaMax2));
            return 1 / (2 * kPi * (1 - cosThetaMax));  // UniformConePdf (sampling.cpp:132-134)
        }
        ok = sphere_surface(s, r, &isl);
        area = s.area;
    } else if (l.kind == PT_LIGHT_DIFFUSE_AREA) {
        // Triangle::Intersect on this one triangle (tMax = Infinity).
        const pt_triangle tr = sc.tris[PT_IDX(l.shape, sc.n_tris)];
        ok = tri_surface(sc, l.shape, tr.flags, r, &isl, vload3(sc.P, PT_IDX(tr.v[0], sc.n_verts)),
                         vload3(sc.P, PT_IDX(tr.v[1], sc.n_verts)), vload3(sc.P, PT_IDX(tr.v[2], sc.n_verts)));
    } else {
        ok = plane_surface(sc.planes[PT_IDX(l.shape, sc.n_planes)], r, &isl);
    }
    if (!ok) return 0;
    float pdf = dist2(ref.p, isl.p) / (absdot(isl.n, -wi) * area);
    if (__builtin_isinf(pdf)) pdf = 0.f;
    return pdf;
}

}  // namespace pt
