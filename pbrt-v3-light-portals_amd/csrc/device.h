// device.h -- device-resident scene and path-state layouts shared by the
// wavefront kernels (kernels.hip) and the host driver (render.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/pt.h"
#include "ptmath.h"

namespace pt {

// AAPlaneShape with everything the kernels need precomputed
// (src/shapes/plane.h:15-32): object-space lo/hi, axes, facingFw =
// !reverseOrientation, and the ObjectToWorld / WorldToObject matrices.
struct DevPlane {
    V3 lo, hi;
    int ax, ax0, ax1;
    // lo/hi along (ax, ax0, ax1), so no bound is read from memory at a
    // run-time component offset (plane.cpp:23-31, 109-115)
    float lo_a, lo_a0, lo_a1, hi_a0, hi_a1;
    int facing_fw;
    int ro_xor_sh;
    int material;
    int area_light;
    float area;
    M4 o2w, w2o;
};

// Sphere (src/shapes/sphere.h:50-59): the ctor's clamped members, the
// ObjectToWorld / WorldToObject matrices and ObjectToWorld(0, 0, 0).
struct DevSphere {
    float radius, zmin, zmax, theta_min, theta_max, phi_max;
    float area;        // Sphere::Area (sphere.cpp:224)
    int ro;            // reverseOrientation (Sphere::Sample normal flip)
    int ro_xor_sh;     // reverseOrientation ^ transformSwapsHandedness (SurfaceInteraction ctor)
    int material;
    int area_light;
    V3 center;
    M4 o2w, w2o;
};

struct DevLight {
    int kind;
    int n_samples;
    S3 L;
    int two_sided;
    int shape;
    int strategy;
    int first_portal;
    int n_portals;
    float area;
    // InfiniteAreaLight (lights/infinite.cpp) with a constant 1x1 Lmap
    M4 l2w, w2l;
    V3 center;
    float radius;
    float cfunc[4], ccdf[6], cint[2];  // Distribution2D conditionals (2 x 2)
    float mfunc[2], mcdf[3], mint;     // and marginal
};

// Prim record flags (word 0 .w of the 48-byte record)
constexpr uint32_t kPrimPlane = 1u;       // AAPlaneShape (else Triangle)
constexpr uint32_t kPrimDegenerate = 2u;  // Triangle::Intersect always rejects (triangle.cpp:309-315)
constexpr uint32_t kPrimSphere = 4u;      // Sphere
constexpr uint32_t kPrimAnalytic = kPrimPlane | kPrimSphere;  // record holds a shape index, not vertices
constexpr uint32_t kPrimInfoTable = 8u;   // material / area light too large for word 2 .w: read the shape table
// The shading step reads everything the reference's GeometricPrimitive /
// Triangle hands it for a C2-style mesh from the record itself: bits 8-12 of
// word 0 .w carry the triangle's PT_TRI_* flags, word 2 .w the material
// (bits 0-15) and area light + 1 (bits 16-31), so a hit needs no triangle
// table or vertex-array load unless the mesh has uv / normals / tangents.
constexpr uint32_t kPrimTriShift = 8u;
// Bits 16-17 of word 0 .w: the material's lobe class (k_shade_sort groups the path queue by it): 0 matte / none /
// no material (and misses), 1 specular lobes only (mirror, smooth glass), 2 microfacet lobes (metal, plastic, rough
// glass)
constexpr uint32_t kPrimClassShift = 16u;
__host__ __device__ constexpr uint32_t material_class(int kind, bool specular) {
    return (kind == PT_MAT_METAL || kind == PT_MAT_PLASTIC) ? 2u
           : kind == PT_MAT_MIRROR                          ? 1u
           : (kind == PT_MAT_GLASS || kind == PT_MAT_DISPERSIVE_GLASS) ? (specular ? 1u : 2u)
                                                                       : 0u;
}
__host__ __device__ constexpr uint32_t prim_info_word(int material, int light) {
    return (uint32_t)(material & 0xffff) | ((uint32_t)(light + 1) << 16);
}
__host__ __device__ constexpr bool prim_info_fits(int material, int light) {
    return material >= 0 && material < 0xffff && light >= -1 && light + 1 < 0xffff;
}

// PT_GUARDS (diagnostic build, `make guard`): scene-table indices on the
// shading path are range-checked; the first failing check records
// file_id * 100000 + line in g_pt_guard and index 0 is used instead of
// faulting.  Production builds compile PT_IDX(i, n) to i.
#ifdef PT_GUARDS
__device__ unsigned int g_pt_guard;
__device__ __forceinline__ int pt_idx(int i, int n, unsigned int where) {
    if ((unsigned)i < (unsigned)n) return i;
    atomicCAS(&g_pt_guard, 0u, where);
    return 0;
}
#define PT_IDX(i, n) pt_idx((i), (n), PT_FILE_ID * 100000u + __LINE__)
#else
#define PT_IDX(i, n) (i)
#endif

struct DevScene {
    // BVH: 2 x float4 per LinearBVHNode; 3 x float4 per primitive in BVH order
    const float4* nodes;
    const float4* prims;
    int n_nodes;
    int n_prims;
    // the same tree collapsed to 4-wide nodes (render.hip build_wide): 7 x float4 per node, k_trace_w
    const float4* wnodes;
    int n_wnodes;
    float wide_scale;  // largest |coordinate| of the root bounds (k_trace_w's absolute tie margin)
    const pt_triangle* tris;
    const float* P;
    const float* N;
    const float* S;
    const float* UV;
    const DevPlane* planes;
    const DevPlane* portal_planes;
    const DevSphere* spheres;
    const pt_material* mats;
    const DevLight* lights;
    int n_lights;
    int n_tris, n_planes, n_pplanes, n_spheres, n_mats, n_verts;  // table sizes (PT_GUARDS builds check against them)
    const float* ldist_func;
    const float* ldist_cdf;
    float ldist_int;
    const float* tri_area;
    // Halton sampler (samplers/halton.cpp)
    const uint16_t* perm;
    const int* prime_sums;
    const DivMagic* divs;   // per dimension: prime base, magic, shift, 1/base
    const DivMagic* divs2;  // per dimension: division by base^2 (two digits per step, staged tables)
    const float* perm_c0;   // per dimension: invBase * perm[0] / (1 - invBase)
    int max_dim;
    int hal_lds_dims;       // leading dimensions whose tables the shading kernel stages in LDS (0: none)
    int hal_lds_perm;       // their permutation entries (prime_sums[hal_lds_dims])
    int hal_lds_bytes;      // bytes of the staged Halton tables (16-byte aligned): the scene tables follow
    int hal_exp0;
    uint32_t hal_scale1;
    DivMagic div_scale1;
    uint32_t hal_stride;
    int center;
    // camera (cameras/perspective.cpp)
    M4 r2c;
    M4 c2w;
    float lens_radius, focal_distance;
    // integrator (integrators/path.cpp, directlighting.cpp)
    int max_depth;
    float rr_threshold;
    int integrator;         // pt_integrator_kind
    int dl_strategy;        // pt_direct_strategy
    int dl_arrays;          // 2D sample arrays requested (0 unless "all")
    int dl_frames;          // recursion stack frames allocated per sample
    int wvl_dim;            // Halton dimension of CameraSample::wvl (5, or arrayEndDim with arrays)
};

// Scene tables the shading kernel stages in LDS next to the Halton tables
// (k_shade_tab, small scenes): byte offsets from the start of the table
// region, each 16-byte aligned, in this order.  The host sizes the region with
// the same function.
struct TabLayout {
    uint32_t prims, mats, lights, planes, pplanes, lfunc, lcdf, end;
};
__host__ __device__ inline uint32_t tab_align16(uint32_t b) { return (b + 15u) & ~15u; }
__host__ __device__ inline TabLayout tab_layout(int n_prims, int n_mats, int n_lights, int n_planes, int n_pplanes) {
    TabLayout t;
    uint32_t o = 0;
    t.prims = o; o = tab_align16(o + 48u * (uint32_t)n_prims);
    t.mats = o; o = tab_align16(o + (uint32_t)sizeof(pt_material) * (uint32_t)n_mats);
    t.lights = o; o = tab_align16(o + (uint32_t)sizeof(DevLight) * (uint32_t)n_lights);
    t.planes = o; o = tab_align16(o + (uint32_t)sizeof(DevPlane) * (uint32_t)n_planes);
    t.pplanes = o; o = tab_align16(o + (uint32_t)sizeof(DevPlane) * (uint32_t)n_pplanes);
    t.lfunc = o; o = tab_align16(o + 4u * (uint32_t)(n_lights > 0 ? n_lights : 1));
    t.lcdf = o; o = tab_align16(o + 4u * (uint32_t)(n_lights + 2));
    t.end = o;
    return t;
}

// Per-path state for one batch of nslots camera samples, as per-slot records:
// a path step's fields share a sector instead of one 4-B field per sector
// (the path queue is compacted every bounce, so a wave's slots are spread).
//   head  4 words {st (kSt* bits, NEE flags at kStNfShift), hit, hitA, hitB}:
//               the step's first loads (what it reads next); the trace kernels
//               write the hit words.  Kept as four SoA arrays (word k of slot s at
//               k * n + s): a 4-B store that a record would share with 3 other
//               slots' words shares its sector with 7 (C2 measured faster, C3 equal)
//   body  32 B  {L.xyz, hidx} {beta.xyz, etaScale}
//   nee   64 B  the deferred EstimateDirect payload (kNee* offsets)
//   Lfin  12 B  the radiance of a finished sample
//   ray / rayA / rayB  32 B  {o.xyz, d.x} {d.yz, tMax, 0} (kernels.hip load_ray)
struct DevPaths {
    int n;
    uint4* head;        // n: the four head-word arrays of n words each (st_word / hit_word)
    float4* body;       // 2n
    float2* pfilm;      // CameraSample::pFilm
    float* ray;         // 8n continuation ray
    float* rayA;        // 8n NEE ray A (MIS shadow ray: its tMax), same record
    float* rayB;        // 8n NEE ray B, same record
    float* nee;         // kNee floats per slot
    float* Lfin;        // 3n: the finished sample's L (pixel-major, dense: what the film pass reads)
    // DirectLightingIntegrator only (null otherwise): see kDl* below
    int* dli;           // kDlInts * n
    float* dlf;         // kDlFloats * n
    float* dlframe;     // kDlFrame * frames * n: the specular recursion stack
};

// head / body words of a slot
constexpr int kHdSt = 0, kHdHit = 1, kHdHitA = 2, kHdHitB = 3;
constexpr int kBdL = 0, kBdHidx = 3, kBdBeta = 4, kBdEta = 7;
__device__ __forceinline__ uint32_t* st_word(const DevPaths& ps, uint32_t slot) {
    return reinterpret_cast<uint32_t*>(ps.head) + slot;
}
__device__ __forceinline__ int* hit_word(const DevPaths& ps, uint32_t slot, int k) {
    return reinterpret_cast<int*>(ps.head) + ((uint32_t)k * (uint32_t)ps.n + slot);
}
__device__ __forceinline__ float* body_word(const DevPaths& ps, uint32_t slot, int k) {
    return reinterpret_cast<float*>(ps.body) + (8u * slot + (uint32_t)k);
}
__device__ __forceinline__ uint32_t hidx_of(const DevPaths& ps, uint32_t slot) {
    return __float_as_uint(*body_word(ps, slot, kBdHidx));
}

// DirectLightingIntegrator per-sample state (kernels.hip shade_dl).
// Integer fields (dli[k * n + slot]):
constexpr int kDlD = 0;      // current recursion depth (frame index)
constexpr int kDlJ = 1;      // UniformSampleAllLights: current light
constexpr int kDlK = 2;      //   current array entry
constexpr int kDlN = 3;      //   entries in the current light's arrays
constexpr int kDlAoff = 4;   // Sampler::array2DOffset
constexpr int kDlAi = 5;     // index of the current uLight array (uScattering = +1)
constexpr int kDlMode = 6;   // kind of the pending EstimateDirect (kDlMode*)
constexpr int kDlS = 7;      // pixel sample number (sample-array indices s*n .. s*n+n-1)
constexpr int kDlPix = 8;    // the pixel's Halton offset (GetIndexForSample(0))
constexpr int kDlInts = 9;
constexpr int kDlModeArray = 0, kDlModeSingle = 1, kDlModeOne = 2;
// Float fields (dlf[k * n + slot]):
constexpr int kDlLnee = 0;   // 3: UniformSampleAllLights' running sum over lights
constexpr int kDlLd = 3;     // 3: current light's sum over array entries
constexpr int kDlLpdf = 6;   // "one": light selection pdf
constexpr int kDlFloats = 7;
// Frame f fields (dlframe[(f * kDlFrame + k) * n + slot]):
constexpr int kFrL = 0;      // 3: the vertex's L so far
constexpr int kFrRay = 3;    // 6: the ray that found the vertex (to rebuild its BSDF)
constexpr int kFrPrim = 9;   // hit primitive (int bits)
constexpr int kFrFac = 10;   // 3: f of the pending specular child
constexpr int kFrCos = 13;   // |wi . ns|
constexpr int kFrPdf = 14;   // pdf
constexpr int kFrPhase = 15; // 0: reflection child pending (transmission next), 1: transmission child
constexpr int kDlFrame = 16;

// st bits: sampler dimension (PrimeTableSize 1000 < 4096), bounces, flags,
// and the pending NEE payload's kNf* flags
constexpr uint32_t kStDimMask = 0xfffu;
constexpr uint32_t kStBounceShift = 12;      // 8 bits
constexpr uint32_t kStSpecular = 1u << 20;
constexpr uint32_t kStCont = 1u << 21;       // continuation ray pending
constexpr uint32_t kStNee = 1u << 22;        // NEE payload pending
constexpr uint32_t kStDimOverflow = 1u << 23;
constexpr uint32_t kStNfShift = 24;          // kNf* << 24
constexpr uint32_t kStNfMask = 0x7fu << kStNfShift;

// NEE payload: kNee floats per slot (ps.nee[kNee * slot + k]), four 16-B
// quarters read as the resolve needs them
constexpr int kNee = 16;
constexpr int kNeeBeta = 0;    // 3: beta at the vertex                              | quarter 0
constexpr int kNeeLpdf = 3;    // light selection pdf (UniformSampleOneLight)
constexpr int kNeeF = 4;       // 3: f*|cos| (portal kinds) or c1 (MIS light part)   | quarter 1
constexpr int kNeePdf = 7;     // portal-kind sampling pdf
constexpr int kNeeLi = 8;      // 3: Li fallback on miss (portal kinds) / f2 (MIS)   | quarter 2
constexpr int kNeeSw = 11;     // MIS scattering weight
constexpr int kNeeSpdf = 12;   // MIS scattering pdf                                 | quarter 3
constexpr int kNeePortalPdf = 13;
constexpr int kNeeLight = 14;  // light index (int bits)
// the shading step writes whole quarters ({beta, lpdf} {F, pdf} {Li, sw} {spdf, portal pdf, light, -})
static_assert(kNeeBeta == 0 && kNeeLpdf == 3 && kNeeF == 4 && kNeePdf == 7 && kNeeLi == 8 && kNeeSw == 11 &&
                  kNeeSpdf == 12 && kNeePortalPdf == 13 && kNeeLight == 14,
              "payload quarters");

constexpr uint32_t kNfPortal = 1u;     // portal-light estimator (ray A closest)
constexpr uint32_t kNfMis = 2u;        // standard MIS (ray A shadow, ray B closest)
constexpr uint32_t kNfA = 4u;          // ray A traced
constexpr uint32_t kNfB = 8u;          // ray B traced
constexpr uint32_t kNfDivPortal = 16u; // divide by portal pdf (projection strategy)
constexpr uint32_t kNfC1 = 32u;        // MIS light contribution present (needs unoccluded A)
constexpr uint32_t kNfLi0 = 64u;       // portal kinds: the Li fallback on a miss is zero (quarter 2 not written)

// Ray queue entry kinds (low 2 bits)
constexpr uint32_t kRayCont = 0, kRayA = 1, kRayShadow = 2, kRayB = 3;

struct DevStats {
    unsigned long long closest;
    unsigned long long shadow;
    unsigned long long nodes;
    unsigned long long prims;
    unsigned long long dim_overflow;
    unsigned long long lane_iters;  // k_trace_pt: lane-iterations executed (SIMD slots)
    unsigned long long lane_steps;  // k_trace_pt: node visits + primitive tests performed
    unsigned long long shade_bytes;  // k_shade (path integrator): algorithmic path-state bytes moved
    unsigned long long wnodes;       // k_trace_w: wide-node visits (7 x 16 B each)
    unsigned long long wprims;       // k_trace_w: primitive tests
    unsigned long long retraced;     // k_trace_w: rays handed to the binary traversal (near ties, infinite 1/d)
};

}  // namespace pt
