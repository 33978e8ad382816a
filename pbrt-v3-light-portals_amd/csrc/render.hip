// render.hip -- host driver of the wavefront path tracer and the C ABI
// (include/pt.h).  Replaces SamplerIntegrator::Render (integrator.cpp:
// 526-637) for the PathIntegrator: the scene is flattened once into device
// buffers, then the (pixel x sample) index space runs as batches of
// independent paths through camera -> {trace, shade}* -> film kernels.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "host_common.h"
// Kernel declarations (bodies compile in the tu_*.hip translation units, in
// parallel); the PT_GUARDS diagnostic build compiles everything here so its
// g_pt_guard symbol is the one every kernel writes.
#ifdef PT_GUARDS
#define PT_TU_TRACE 1
#define PT_TU_SHADE 1
#define PT_TU_MISC 1
#define PT_TU_HERO 1
#include "tu_trace.hip"
#include "tu_shade.hip"
#include "tu_misc.hip"
#include "tu_hero.hip"
#else
#include "hero.hip"
#endif

namespace pt {

static thread_local std::string g_last_error;

#define HIPCHK(x)                                                                                         \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess) throw PtError(PT_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        if (count <= n && p) return;
        release();
        size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, bytes);
        if (e != hipSuccess) throw PtError(PT_ERR_OOM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
        p = (T*)q;
        n = count;
    }
    void upload(const T* h, size_t count) {
        alloc(count);
        if (count) HIPCHK(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
    }
    void upload(const std::vector<T>& v) { upload(v.data(), v.size()); }
};

// ---------------------------------------------------------------------------
// Halton tables (lowdiscrepancy.cpp:40-124, 2490-2504; halton.cpp:45-93)
// ---------------------------------------------------------------------------
struct HaltonTables {
    std::vector<int> primes, prime_sums;
    std::vector<uint16_t> perms;
};
static const HaltonTables& halton_tables() {
    static HaltonTables t = [] {
        HaltonTables h;
        for (int c = 2; (int)h.primes.size() < 1000; ++c) {
            bool ok = true;
            for (int q : h.primes) {
                if (q * q > c) break;
                if (c % q == 0) { ok = false; break; }
            }
            if (ok) h.primes.push_back(c);
        }
        int s = 0;
        for (int p : h.primes) { h.prime_sums.push_back(s); s += p; }
        h.perms.resize((size_t)s);
        // RNG in its default state (rng.h:129) and Shuffle (sampling.h:152-158)
        uint64_t state = 0x853c49e6748fea9bULL, inc = 0xda3e39cb94b95bdbULL;
        auto next = [&]() {
            uint64_t old = state;
            state = old * 0x5851f42d4c957f2dULL + inc;
            uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
            uint32_t rot = (uint32_t)(old >> 59u);
            return (xs >> rot) | (xs << ((~rot + 1u) & 31));
        };
        auto bounded = [&](uint32_t b) {
            uint32_t threshold = (~b + 1u) % b;
            for (;;) { uint32_t r = next(); if (r >= threshold) return r % b; }
        };
        uint16_t* p = h.perms.data();
        for (int P : h.primes) {
            for (int j = 0; j < P; ++j) p[j] = (uint16_t)j;
            for (int j = 0; j < P; ++j) {
                int other = j + (int)bounded((uint32_t)(P - j));
                std::swap(p[j], p[other]);
            }
            p += P;
        }
        return h;
    }();
    return t;
}

static DivMagic make_div_magic(uint32_t d) {
    DivMagic m{};
    m.base = d;
    m.inv_base = (float)1 / (float)d;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;  // ceil(log2 d)
    m.magic = (uint32_t)((((unsigned __int128)1 << 32) * ((1ull << l) - d)) / d + 1);
    m.shift = l - 1;
    return m;
}

static void extended_gcd(uint64_t a, uint64_t b, int64_t* x, int64_t* y) {  // halton.cpp:51-61
    if (b == 0) { *x = 1; *y = 0; return; }
    int64_t d = (int64_t)(a / b), xp, yp;
    extended_gcd(b, a % b, &xp, &yp);
    *x = yp;
    *y = xp - (d * yp);
}
static uint64_t mult_inverse(int64_t a, int64_t n) {
    int64_t x, y;
    extended_gcd((uint64_t)a, (uint64_t)n, &x, &y);
    int64_t r = x - (x / n) * n;
    return (uint64_t)(r < 0 ? r + n : r);
}

// ---------------------------------------------------------------------------
// Device scene
// ---------------------------------------------------------------------------
struct Frame {
    int crop_x0, crop_y0, crop_x1, crop_y1;
    int sb_x0, sb_y0, sb_x1, sb_y1;
    int pb_x0, pb_y0, pb_x1, pb_y1;  // integrator pixelBounds
    int ntx, nty;
    int width() const { return crop_x1 - crop_x0; }
    int height() const { return crop_y1 - crop_y0; }
};

constexpr int kMaxPipes = 4;  // render_tiles pipelines (PT_PIPES)

struct Work {
    DBuf<uint32_t> rq0, rq1, pq0, pq1, counts;
    DBuf<uint32_t> rqr;  // k_trace_w: ray-queue entries handed to the binary traversal (counts[6])
    DBuf<uint32_t> pqs;  // k_shade_sort: the path queue grouped by material class per chunk
    DBuf<uint4> head;   // DevPaths records (device.h)
    DBuf<float4> body;
    DBuf<float2> pfilm;
    DBuf<float> ray, rayA, rayB, nee, Lfin;
    DBuf<int> spill;
    DBuf<DevStats> stats;
    DBuf<DevStats> stats_rt;  // the retrace launches after k_trace_w (their rays are the retraced_rays)
    DBuf<int> dli;                 // DirectLighting state (kDl*)
    DBuf<float> dlf, dlframe;
    DBuf<float> h_out60, h_outy, h_L60, h_beta60, h_nee60, h_hs;  // hero integrators: 60-bin state per slot
    size_t cap = 0, hero_cap = 0;
    int dl_frames = 0;             // > 0: DirectLighting buffers with this many frames per slot
    hipStream_t stream = nullptr;  // this pipeline's stream (render_tiles)
    uint32_t* host_counts = nullptr;  // pinned: queue sizes read back per bounce
    Work() = default;
    Work(const Work&) = delete;
    Work& operator=(const Work&) = delete;
    ~Work() {
        if (stream) (void)hipStreamDestroy(stream);
        if (host_counts) (void)hipHostFree(host_counts);
    }
    void ensure(size_t n, size_t spill_threads, int frames, int hero_slots) {
        if (!host_counts) {
            void* p = nullptr;
            // written by k_next_counts at the end of each bounce (system-coherent, no copy engine or blit)
            if (hipHostMalloc(&p, 8 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
                throw PtError(PT_ERR_OOM, "hipHostMalloc failed");
            host_counts = (uint32_t*)p;
        }
        if (hero_slots > 0 && (size_t)hero_slots > hero_cap) {
            h_out60.alloc((size_t)hero_slots * kNSpec);
            h_outy.alloc((size_t)hero_slots);
            h_L60.alloc((size_t)hero_slots * kNSpec);
            h_beta60.alloc((size_t)hero_slots * kNSpec);
            h_nee60.alloc((size_t)hero_slots * kNSpec);
            h_hs.alloc((size_t)hero_slots * kHsPad);
            hero_cap = (size_t)hero_slots;
        }
        if (frames > 0 && (n > cap || frames != dl_frames)) {
            dli.alloc((size_t)kDlInts * n);
            dlf.alloc((size_t)kDlFloats * n);
            dlframe.alloc((size_t)kDlFrame * (size_t)frames * n);
            dl_frames = frames;
        }
        if (n > cap) {
            rq0.alloc(3 * n); rq1.alloc(3 * n); rqr.alloc(3 * n); pq0.alloc(n); pq1.alloc(n); pqs.alloc(n);
            head.alloc(n); body.alloc(2 * n); pfilm.alloc(n); ray.alloc(8 * n); rayA.alloc(8 * n);
            rayB.alloc(8 * n); nee.alloc((size_t)kNee * n); Lfin.alloc(3 * n);
            cap = n;
        }
        spill.alloc(spill_threads * 64);  // k_trace_pt: 64 words per lane (entries past its LDS rows)
        counts.alloc(8);
        stats.alloc(1);
        stats_rt.alloc(1);
    }
    DevPaths paths(int n) {
        DevPaths p{};
        p.n = n;
        p.head = head.p; p.body = body.p; p.pfilm = pfilm.p;
        p.ray = ray.p; p.rayA = rayA.p; p.rayB = rayB.p;
        p.nee = nee.p;
        p.Lfin = Lfin.p;
        p.dli = dl_frames > 0 ? dli.p : nullptr;
        p.dlf = dl_frames > 0 ? dlf.p : nullptr;
        p.dlframe = dl_frames > 0 ? dlframe.p : nullptr;
        return p;
    }
};

// Restores a device as current when destroyed (dev < 0: nothing to restore).
struct DeviceRestore {
    int dev = -1;
    ~DeviceRestore() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

}  // namespace pt

struct pt_scene {
    // declared first, destroyed last: gives the caller back its current device after every buffer and
    // stream of the scene was freed with the scene's own device current
    pt::DeviceRestore restore_dev;
    pt::DBuf<float4> nodes, prims;
    pt::DBuf<float4> wnodes;  // the BVH collapsed to 4-wide nodes (build_wide; k_trace_w)
    pt::DBuf<pt_triangle> tris;
    pt::DBuf<float> P, N, S, UV, lfunc, lcdf, tri_area, perm_c0;
    pt::DBuf<pt::DevPlane> planes, pplanes;
    pt::DBuf<pt::DevSphere> spheres;
    pt::DBuf<pt_material> mats;
    pt::DBuf<pt::DevLight> lights;
    pt::DBuf<uint16_t> perm;
    pt::DBuf<int> psums;
    pt::DBuf<pt::DivMagic> divs, divs2;
    pt::DevScene dev{};
    // hero integrators (SampledSpectrum scenes): tables, light distributions, per-slot radiance
    bool hero = false;
    pt::DevHero hh{};
    pt::DBuf<float> h_xyz, h_illum, h_mat, h_light, h_wcdf, h_dist;
    pt::DBuf<int> h_matnb;
    pt::HaltonPixelConsts hpc{};
    pt::FilmConsts film{};
    pt::Frame fr{};
    pt_film_desc filmdesc{};
    int spp = 0;
    std::vector<pt::LinearNode> host_nodes;
    std::vector<int> host_prim_order;
    pt::Work work[pt::kMaxPipes];  // one set of path-state buffers per pipeline
    int pipes = 2;                 // pipelines render_tiles runs batches on (PT_PIPES)
    int device = 0;
    int num_cus = 256;
    size_t target_slots = 0;  // batch size in camera samples; 0: 96 M (32 M for the 60-bin hero state)
    int dl_max_samples = 1;      // DirectLighting: largest Light::nSamples
    size_t lds_scene_bytes = 0;  // > 0: k_trace stages the BVH in LDS
    size_t hal_lds_bytes = 0;    // dynamic LDS of k_shade: the staged Halton tables (DevScene::hal_lds_dims)
    bool shade_tab = false;      // k_shade_tab: the scene tables staged in LDS as well (small scenes)
    int hero_waves = 2;          // k_shade_hero register budget (PT_HERO_WAVES=1|2|4); C3h: 2 > 4 > 1
    bool count_bytes = false;    // pt_set_count_bytes: the shading build that counts algorithmic path-state bytes
    int shade_variant = 0;       // 0: compiler register budget, 3: k_shade_tab at 3 waves per SIMD (default when
                                 // that build has no scratch), 4: k_shade at 3 waves per SIMD (the same, tables
                                 // too large for LDS), 5: k_shade_tab
    int features = pt::kFtAll;   // scene features the shading kernel is compiled for (kFt*)
    bool has_spheres = true;     // trace kernels with the sphere test
    int trace_persist = 2;       // 0: k_trace, 1: k_trace_pt, 2: k_trace_nb (branch-reduced)
    bool trace_lean = true;      // LDS scenes under trace_persist 2: k_trace_lds (PT_TRACE_LEAN=0: k_trace_nb)
    size_t oct_lds_bytes = 0;    // > 0: k_trace_oct (octant images of an LDS-sized BVH; opt-in PT_TRACE_OCT=1)
    size_t wide_lds_bytes = 0;   // > 0: k_trace_w, its dynamic LDS (PT_TRACE_WIDE=0 disables): LDS-resident scenes the
                                 // 4-wide BVH image + primitive records + stack, HBM-resident ones the stack rows
    bool wide_hbm = false;       // k_trace_w<true>: the wide image and the primitives from HBM
    uint32_t mat_classes = 1;    // material classes among the primitives (bit c: kPrimClassShift class c present)
    bool shade_sort = false;     // PT_SHADE_SORT=1: k_shade_sort before the path integrator's shading when 2+ classes
                                 // (C3 @256: 424.8 vs 452.6 Msamples/s without -- the queue order from the pixel-major
                                 // batches keeps most waves one class already)
    int wide_rows = 0;           // k_trace_w stack rows per lane (dummy row + deepest stack + 3 push rows)
    int wide_lds_rows = 0;       // of them in LDS (k_trace_w<true>: the rest in the lane's spill column)
    int leaf_min_w = 48;         // k_trace_w: lanes parked at leaves that trigger a primitive-test step (PT_LEAF_MIN_W;
                                 // C2 16 / 32 / 48 / 64: 10.39 / 9.12 / 8.69 / 8.67 ms per launch)
    int trace_bpc = 16;          // persistent trace blocks per CU
    int shade_bpc = 48;          // shading blocks per CU (grid-stride; PT_SHADE_BPC): 12 rounds of the 2-wave kernels' 4 resident blocks (8: C4 k_shade 13.0 vs 10.0 ms, C3 362 vs 375 Msamples/s)
    int film_t = 0;              // RGB film, filter windows of 2-16 pixels: PT_FILM_T=1 takes k_film_t (lane = film pixel; faster at 256 spp, slower at 1024: DESIGN §10)
    int film_blk = 0;            // hero film: PT_FILM_BLK=1 takes the LDS-staged k_film_s60_blk (slower: DESIGN §10)
    int film_sq = 1;             // hero film: k_film_s60_sq over 2 x 2 film-pixel squares (PT_FILM_SQ=0: k_film_s60 per pixel)
    int film_sk = -1;            // RGB film: k_film_sk (skewed lane-per-pixel walks) for win 2 (-1, default: C3's 2-pixel
                                 // Gaussian 20.5 -> 5.1 ms per launch), PT_FILM_SK=1 also for win 1 (box: equal), 0 never
    int film_skew = 1;           // k_film_sk: PT_FILM_SKEW=0/1/2 -- the lanes' walks unskewed / skewed by column / by column and row
    int batch_equal = 0;         // renders of at most this many batches get equal batches (PT_BATCH_EQUAL)
    int refill_min = 16;         // idle lanes that trigger a refill from the wave's queue chunk
    int leaf_min = 40;           // k_trace_nb: lanes parked at leaves that trigger a primitive-test step
    int leaf_min_pt = 16;        // k_trace_pt (HBM-resident BVHs): the same threshold
    int trace_spill = 1;         // BVH deeper than the LDS stack: keep the global spill path
    int stack_rows = pt::kStackLds;  // LDS stack entries per lane in k_trace_pt
    // pt_init(n > 1, ids): one replica per further device of the process
    // (same scene, same host-built BVH), rendered by one host thread each
    std::vector<std::unique_ptr<pt_scene>> replicas;
    std::vector<int> devices;  // ids[0..n) the scene was created for (primary first)
    ~pt_scene() {
        // replicas first (each makes its own device current), then this scene's streams and buffers are
        // freed with its own device current; restore_dev then makes the caller's device current again
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess) restore_dev.dev = cur;
        replicas.clear();
        (void)hipSetDevice(device);
    }
};

// Multi-process communicator (pt_comm_create): RCCL over the GPUs of the job
struct pt_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the frame's reduce (pt_render_frame_dist), created once
    ~pt_comm() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (comm) (void)ncclCommDestroy(comm);
    }
};

namespace pt {

static int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Smallest shading-kernel feature set (devfuncs.h kFt*) covering the scene's
// materials and lights.  PT_SHADE_FEATURES overrides it (a superset renders the
// same image: the extra code is simply unreachable).
static int scene_features(const pt_scene_desc* d) {
    int f = 0;
    if (!d || (d->n_materials > 0 && !d->materials) || (d->n_lights > 0 && !d->lights)) return kFtAll;
    for (int i = 0; i < d->n_materials; ++i) {
        const pt_material& m = d->materials[i];
        if (m.kind == PT_MAT_METAL || m.kind == PT_MAT_PLASTIC) f |= kFtMicro;
        if (m.kind == PT_MAT_MIRROR) f |= kFtSpecular;
        if (m.kind == PT_MAT_GLASS || m.kind == PT_MAT_DISPERSIVE_GLASS) f |= m.specular ? kFtSpecular : kFtMicro;
    }
    for (int i = 0; i < d->n_lights; ++i)
        if (d->lights[i].kind == PT_LIGHT_INFINITE) f |= kFtInfinite;
    if (d->n_spheres > 0) f |= kFtSphere;
    bool portalOnly = d->n_lights > 0;
    for (int i = 0; i < d->n_lights; ++i) portalOnly &= d->lights[i].kind == PT_LIGHT_PORTAL_AREA;
    if (portalOnly) f |= kFtPortalOnly;
    return f;
}

using ShadeKernel = void (*)(DevScene, DevPaths, const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                             uint32_t*, DevStats*);
template <int kFt>
static ShadeKernel shade_kernel_ft(int variant, bool ab) {
    switch (variant) {
        case 3: return ab ? k_shade_w3<kFt, true> : k_shade_w3<kFt, false>;
        case 4: return ab ? k_shade_w3h<kFt, true> : k_shade_w3h<kFt, false>;
        case 5: return ab ? k_shade_tab<kFt, true> : k_shade_tab<kFt, false>;
        default: return ab ? k_shade<kFt, true> : k_shade<kFt, false>;
    }
}
// Instantiated feature sets: all-matte, + infinite light, + spheres, + both,
// both BSDF kinds + infinite light without spheres, everything.  Other combinations take the full kernel.
// ab: the build that counts the algorithmic path-state bytes (pt_set_count_bytes)
static ShadeKernel shade_kernel(int variant, int features, bool ab = false) {
    if (features == kFtPortalOnly) return shade_kernel_ft<kFtPortalOnly>(variant, ab);  // matte, portal lights only
    switch (features & kFtAll) {
        case 0: return shade_kernel_ft<0>(variant, ab);
        case kFtInfinite: return shade_kernel_ft<kFtInfinite>(variant, ab);
        case kFtSphere: return shade_kernel_ft<kFtSphere>(variant, ab);
        case kFtInfinite | kFtSphere: return shade_kernel_ft<kFtInfinite | kFtSphere>(variant, ab);
        case kFtMicro | kFtSpecular | kFtInfinite:  // the dielectric Cornell box (C3): no sphere code
            return shade_kernel_ft<kFtMicro | kFtSpecular | kFtInfinite>(variant, ab);
        default: return shade_kernel_ft<kFtAll>(variant, ab);
    }
}

using HeroKernel = void (*)(DevScene, DevHero, DevPaths, DevHeroPaths, const uint32_t*, const uint32_t*, uint32_t*,
                           uint32_t*, uint32_t*, uint32_t*, DevStats*);
template <int kFt>
static HeroKernel hero_kernel_ft(int waves) {
    return waves == 1 ? k_shade_hero<kFt> : (waves == 2 ? k_shade_hero_w2<kFt> : k_shade_hero_w4<kFt>);
}
// instantiated (tu_hero.hip): matte-only, smooth specular, + infinite light, no spheres, everything
static HeroKernel hero_kernel(int waves, int features) {
    switch (features & kFtAll) {
        case 0: return hero_kernel_ft<0>(waves);
        case kFtSpecular: return hero_kernel_ft<kFtSpecular>(waves);
        case kFtInfinite:
        case kFtSpecular | kFtInfinite: return hero_kernel_ft<kFtSpecular | kFtInfinite>(waves);
        case kFtMicro:
        case kFtMicro | kFtSpecular:
        case kFtMicro | kFtInfinite:
        case kFtMicro | kFtSpecular | kFtInfinite: return hero_kernel_ft<kFtMicro | kFtSpecular | kFtInfinite>(waves);
        default: return hero_kernel_ft<kFtAll>(waves);
    }
}

using TraceNbKernel = void (*)(DevScene, DevPaths, const uint32_t*, const uint32_t*, uint32_t*, int, int, DevStats*);
static TraceNbKernel trace_nb_kernel(bool lds, bool sph) {
    return lds ? (sph ? k_trace_nb<true, true> : k_trace_nb<true, false>)
               : (sph ? k_trace_nb<false, true> : k_trace_nb<false, false>);
}
static TraceNbKernel trace_lds_kernel(bool sph) { return sph ? k_trace_lds<true> : k_trace_lds<false>; }
static TraceNbKernel trace_oct_kernel(bool sph) { return sph ? k_trace_oct<true> : k_trace_oct<false>; }
using TracePtKernel = void (*)(DevScene, DevPaths, const uint32_t*, const uint32_t*, uint32_t*, int, int, int, int*,
                               DevStats*);
static TracePtKernel trace_pt_kernel(bool lds, bool spill, bool sph) {
    if (lds) {
        if (spill) return sph ? k_trace_pt<true, true, true> : k_trace_pt<true, true, false>;
        return sph ? k_trace_pt<true, false, true> : k_trace_pt<true, false, false>;
    }
    if (spill) return sph ? k_trace_pt<false, true, true> : k_trace_pt<false, true, false>;
    return sph ? k_trace_pt<false, false, true> : k_trace_pt<false, false, false>;
}
using TraceKernel = void (*)(DevScene, DevPaths, const uint32_t*, const uint32_t*, int*, DevStats*);
static TraceKernel trace_kernel(bool lds, bool sph) {
    return lds ? (sph ? k_trace<true, true> : k_trace<true, false>) : (sph ? k_trace<false, true> : k_trace<false, false>);
}

// InfiniteAreaLight ctor + Preprocess (infinite.cpp:43-83): LightToWorld,
// world bounding sphere of the BVH root, and the Distribution2D over the 2x2
// sin(theta)-weighted luminance image of the constant map.
static void init_infinite(const pt_light& l, const std::vector<LinearNode>& nodes, DevLight* dl) {
    std::memcpy(dl->l2w.m, l.light_to_world.m, 64);
    std::memcpy(dl->w2l.m, l.light_to_world.minv, 64);
    if (!nodes.empty()) {
        const V3 pmin = v3(nodes[0].bmin[0], nodes[0].bmin[1], nodes[0].bmin[2]);
        const V3 pmax = v3(nodes[0].bmax[0], nodes[0].bmax[1], nodes[0].bmax[2]);
        dl->center = (pmin + pmax) * 0.5f;  // Bounds3::BoundingSphere (geometry.h:959-962)
        const V3 c = dl->center;
        const bool inside = c.x >= pmin.x && c.x <= pmax.x && c.y >= pmin.y && c.y <= pmax.y && c.z >= pmin.z &&
                            c.z <= pmax.z;
        dl->radius = inside ? len(c - pmax) : 0.f;
    } else {
        dl->center = v3(0, 0, 0);
        dl->radius = 0.f;
    }
    const int width = 2, height = 2;
    float img[4];
    for (int v = 0; v < height; ++v) {
        const float vp = (v + .5f) / (float)height;
        const float sinTheta = std::sin(kPi * (v + .5f) / height);
        for (int u = 0; u < width; ++u) {
            const float up = (u + .5f) / (float)width;
            img[u + v * width] = lum_y(lmap_triangle(dl->L, up, vp));
            img[u + v * width] *= sinTheta;
        }
    }
    auto build1d = [](const float* f, int n, float* cdf, float* funcInt) {  // Distribution1D (sampling.h:57-69)
        cdf[0] = 0;
        for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + f[i - 1] / n;
        *funcInt = cdf[n];
        if (*funcInt == 0) { for (int i = 1; i < n + 1; ++i) cdf[i] = (float)i / (float)n; }
        else { for (int i = 1; i < n + 1; ++i) cdf[i] /= *funcInt; }
    };
    for (int v = 0; v < height; ++v) {
        for (int u = 0; u < width; ++u) dl->cfunc[2 * v + u] = img[v * width + u];
        build1d(dl->cfunc + 2 * v, width, dl->ccdf + 3 * v, &dl->cint[v]);
        dl->mfunc[v] = dl->cint[v];
    }
    build1d(dl->mfunc, height, dl->mcdf, &dl->mint);
}

// RadicalInverse(baseIndex, a) (lowdiscrepancy.cpp:427-...) for the
// SpatialLightDistribution sample points: base 2 through ReverseBits64 in
// double, bases 3..11 by RadicalInverseSpecialized (lowdiscrepancy.h:98-111).
static float radical_inverse_host(int baseIndex, uint64_t a) {
    if (baseIndex == 0) {
        uint64_t r = 0;
        for (int i = 0; i < 64; ++i) r |= ((a >> i) & 1ull) << (63 - i);
        return (float)(r * 0x1p-64);
    }
    static const int primes[5] = {2, 3, 5, 7, 11};
    const uint64_t base = (uint64_t)primes[baseIndex];
    const float invBase = (float)1 / (float)base;
    uint64_t reversed = 0;
    float invBaseN = 1;
    while (a) {
        uint64_t next = a / base, digit = a - next * base;
        reversed = reversed * base + digit;
        invBaseN *= invBase;
        a = next;
    }
    return std::min(reversed * invBaseN, 0x1.fffffep-1f);
}
// Distribution1D ctor (sampling.h:65-88) into [func | cdf | funcInt]
static void dist1d_host(const std::vector<float>& f, float* out) {
    const int n = (int)f.size();
    for (int i = 0; i < n; ++i) out[i] = f[i];
    float* cdf = out + n;
    cdf[0] = 0;
    for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + f[i - 1] / n;
    const float funcInt = cdf[n];
    if (funcInt == 0)
        for (int i = 1; i < n + 1; ++i) cdf[i] = (float)i / (float)n;
    else
        for (int i = 1; i < n + 1; ++i) cdf[i] /= funcInt;
    out[2 * n + 1] = funcInt;
}
// HeroSamplerIntegrator::Preprocess (hero.cpp:57-66), HeroPathMIS::Preprocess
// (hero_path_mis.cpp:104-108): spectral distribution of the summed light
// power (Light::Power, diffuse.cpp:65-67, infinite.cpp:86-90) and the light
// sample distribution (lightdistrib.cpp:46-66).
static void build_hero(pt_scene* s, const pt_scene_desc* d, const std::vector<DevLight>& lights,
                       const std::vector<float>& area, const std::vector<DevSphere>& spheres) {
    if (!d->material_s60 || !d->light_s60) throw PtError(PT_ERR_INVALID_ARG, "spectral scene without 60-bin tables");
    for (int i = 0; i < d->n_lights; ++i)
        if (d->lights[i].kind == PT_LIGHT_PORTAL_AREA || d->lights[i].kind == PT_LIGHT_POINT ||
            d->lights[i].kind == PT_LIGHT_DIFFUSE_PLANE)
            throw PtError(PT_ERR_UNSUPPORTED, "hero integrators support area and infinite lights");
    const SpecTables60& t = spectral_tables();
    std::vector<float> xyz(3 * kNSpec), illum(7 * kNSpec);
    for (int i = 0; i < kNSpec; ++i) { xyz[i] = t.X[i]; xyz[kNSpec + i] = t.Y[i]; xyz[2 * kNSpec + i] = t.Z[i]; }
    for (int k = 0; k < 7; ++k)
        for (int i = 0; i < kNSpec; ++i) illum[k * kNSpec + i] = t.illum[k][i];
    s->h_xyz.upload(xyz);
    s->h_illum.upload(illum);
    s->h_mat.upload(d->material_s60, (size_t)d->n_materials * 3 * kNSpec);
    {   // per material: bit j set when spectrum j is not black after Clamp() (the lobe set's IsBlack tests)
        std::vector<int> nb((size_t)std::max(1, d->n_materials), 0);
        for (int m = 0; m < d->n_materials; ++m)
            for (int j = 0; j < 3; ++j)
                for (int i = 0; i < kNSpec; ++i) {
                    const float v = d->material_s60[((size_t)m * 3 + j) * kNSpec + i];
                    if ((v < 0 ? 0.f : v) != 0.f) { nb[m] |= 1 << j; break; }
                }
        s->h_matnb.upload(nb);
    }
    s->h_light.upload(d->light_s60, (size_t)std::max(1, d->n_lights) * kNSpec);
    const int nl = d->n_lights;
    std::vector<std::vector<float>> power((size_t)nl, std::vector<float>(kNSpec));
    for (int li = 0; li < nl; ++li) {
        const pt_light& l = d->lights[li];
        if (l.kind == PT_LIGHT_INFINITE) {
            const S3 texel = lmap_triangle(lights[li].L, .5f, .5f);  // Lmap->Lookup((.5, .5), .5)
            float sp[60];
            s60_from_rgb(texel.c, false, sp);
            const float k = kPi * lights[li].radius * lights[li].radius;
            for (int i = 0; i < kNSpec; ++i) power[li][i] = sp[i] * k;
        } else {
            const float a = l.kind == PT_LIGHT_DIFFUSE_AREA ? area[l.shape] : spheres[l.shape].area;
            const float* L = d->light_s60 + (size_t)li * kNSpec;
            for (int i = 0; i < kNSpec; ++i) power[li][i] = ((L[i] * (float)(l.two_sided ? 2 : 1)) * a) * kPi;
        }
    }
    std::vector<float> sum(kNSpec, 0.f), wcdf(kNSpec + 1);
    for (int li = 0; li < nl; ++li)
        for (int i = 0; i < kNSpec; ++i) sum[i] += power[li][i];
    wcdf[0] = 0.f;  // DiscreteDistribution::Set (distr.h:30-39)
    for (int i = 0; i < kNSpec; ++i) wcdf[i + 1] = wcdf[i] + sum[i];
    const float invsum = 1.f / wcdf[kNSpec];
    for (int i = 1; i < kNSpec; ++i) wcdf[i] *= invsum;
    wcdf[kNSpec] = 1.0f;
    s->h_wcdf.upload(wcdf);
    DevHero& h = s->hh;
    h = DevHero{};
    h.XYZ = s->h_xyz.p;
    h.illum = s->h_illum.p;
    h.mat_s60 = s->h_mat.p;
    h.mat_nb = s->h_matnb.p;
    h.light_s60 = s->h_light.p;
    h.wcdf = s->h_wcdf.p;
    h.mis = d->integrator.kind == PT_INTEGRATOR_HERO_PATH_MIS;
    h.dist_stride = 2 * nl + 2;
    h.spatial = h.mis && nl > 1 && d->integrator.light_strategy == PT_LIGHTS_SPATIAL;
    if (!h.spatial) {
        std::vector<float> func((size_t)std::max(nl, 1), 1.f), dist((size_t)h.dist_stride, 0.f);
        if (d->integrator.light_strategy == PT_LIGHTS_POWER && nl > 1)
            for (int li = 0; li < nl; ++li) func[li] = s60_y(power[li].data());
        if (nl > 0) {
            func.resize((size_t)nl);
            dist1d_host(func, dist.data());
        }
        s->h_dist.upload(dist);
    } else {
        // SpatialLightDistribution ctor (lightdistrib.cpp:80-104): voxel grid over WorldBound()
        const LinearNode& root = s->host_nodes[0];
        const V3 mn = v3(root.bmin[0], root.bmin[1], root.bmin[2]), mx = v3(root.bmax[0], root.bmax[1], root.bmax[2]);
        const V3 diag = mx - mn;
        const int ax = (diag.x > diag.y && diag.x > diag.z) ? 0 : (diag.y > diag.z ? 1 : 2);
        const float bmax = diag[ax];
        int nv[3];
        for (int i = 0; i < 3; ++i) nv[i] = std::max(1, (int)std::round(diag[i] / bmax * 64));
        h.nv0 = nv[0]; h.nv1 = nv[1]; h.nv2 = nv[2];
        h.wb_min = mn; h.wb_max = mx;
        const size_t nvox = (size_t)nv[0] * nv[1] * nv[2];
        if (nvox * (size_t)h.dist_stride > ((size_t)1 << 30))
            throw PtError(PT_ERR_UNSUPPORTED, "spatial light distribution too large (voxels x lights)");
        s->h_dist.alloc(nvox * (size_t)h.dist_stride);
        std::vector<float> ri(5 * 128), ly((size_t)nl);
        for (int i = 0; i < 128; ++i)
            for (int b = 0; b < 5; ++b) ri[5 * i + b] = radical_inverse_host(b, (uint64_t)i);
        for (int li = 0; li < nl; ++li) ly[li] = s60_y(d->light_s60 + (size_t)li * kNSpec);
        DBuf<float> dri, dly;
        dri.upload(ri);
        dly.upload(ly);
        h.dist = s->h_dist.p;
        hipLaunchKernelGGL(k_hero_spatial, dim3(ceil_div((long)nvox, 128)), dim3(128), 0, 0, s->dev, h, dri.p, dly.p,
                           s->h_dist.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipDeviceSynchronize());
    }
    h.dist = s->h_dist.p;
    s->hero = true;
}

static void build_scene(pt_scene* s, const pt_scene_desc* d, const pt_scene* bvh_src) {
    if (!d) throw PtError(PT_ERR_INVALID_ARG, "null scene description");
    if (d->n_prims < 0 || d->n_triangles < 0 || d->n_planes < 0 || d->n_lights < 0 || d->n_materials < 0)
        throw PtError(PT_ERR_INVALID_ARG, "negative counts in scene description");
    if (d->n_triangles > 0 && !d->P) throw PtError(PT_ERR_INVALID_ARG, "triangles without vertices");
    for (int i = 0; i < d->n_prims; ++i) {
        const pt_prim& p = d->prims[i];
        if (p.kind == PT_PRIM_TRIANGLE) {
            if (p.index < 0 || p.index >= d->n_triangles) throw PtError(PT_ERR_INVALID_ARG, "bad triangle prim");
        } else if (p.kind == PT_PRIM_AAPLANE) {
            if (p.index < 0 || p.index >= d->n_planes) throw PtError(PT_ERR_INVALID_ARG, "bad plane prim");
        } else if (p.kind == PT_PRIM_SPHERE) {
            if (p.index < 0 || p.index >= d->n_spheres || !d->spheres)
                throw PtError(PT_ERR_INVALID_ARG, "bad sphere prim");
        } else
            throw PtError(PT_ERR_INVALID_ARG, "bad prim kind");
    }
    for (int i = 0; i < d->n_triangles; ++i) {
        const pt_triangle& t = d->triangles[i];
        for (int k = 0; k < 3; ++k)
            if (t.v[k] < 0 || t.v[k] >= d->n_vertices) throw PtError(PT_ERR_INVALID_ARG, "triangle vertex out of range");
        if (t.material < 0 || t.material >= d->n_materials) throw PtError(PT_ERR_INVALID_ARG, "bad material index");
        if (t.area_light >= d->n_lights) throw PtError(PT_ERR_INVALID_ARG, "bad light index");
    }
    for (int i = 0; i < d->n_planes; ++i) {
        const pt_aaplane& p = d->planes[i];
        if (p.axis < 0 || p.axis > 2) throw PtError(PT_ERR_INVALID_ARG, "bad plane axis");
        if (p.material < 0 || p.material >= d->n_materials) throw PtError(PT_ERR_INVALID_ARG, "bad material index");
    }
    for (int i = 0; i < d->n_spheres; ++i) {
        const pt_sphere& sp = d->spheres[i];
        if (!(sp.radius > 0)) throw PtError(PT_ERR_INVALID_ARG, "sphere radius must be positive");
        if (sp.material < 0 || sp.material >= d->n_materials) throw PtError(PT_ERR_INVALID_ARG, "bad material index");
        if (sp.area_light >= d->n_lights) throw PtError(PT_ERR_INVALID_ARG, "bad light index");
    }
    for (int i = 0; i < d->n_materials; ++i) {
        int k = d->materials[i].kind;
        if (k < PT_MAT_NONE || k > PT_MAT_PLASTIC) throw PtError(PT_ERR_UNSUPPORTED, "unsupported material kind");
        if (k == PT_MAT_MATTE && d->materials[i].sigma != 0.f)
            throw PtError(PT_ERR_UNSUPPORTED, "OrenNayar (sigma != 0) not supported");
        if ((k == PT_MAT_METAL || k == PT_MAT_PLASTIC ||
             ((k == PT_MAT_GLASS || k == PT_MAT_DISPERSIVE_GLASS) && !d->materials[i].specular)) &&
            !(d->materials[i].alpha[0] > 0 && d->materials[i].alpha[1] > 0))
            throw PtError(PT_ERR_INVALID_ARG, "microfacet alpha must be positive");
    }
    for (int i = 0; i < d->n_lights; ++i) {
        const pt_light& l = d->lights[i];
        if (l.kind == PT_LIGHT_DIFFUSE_AREA) {
            if (l.shape < 0 || l.shape >= d->n_triangles) throw PtError(PT_ERR_INVALID_ARG, "bad light shape");
        } else if (l.kind == PT_LIGHT_DIFFUSE_SPHERE) {
            if (l.shape < 0 || l.shape >= d->n_spheres) throw PtError(PT_ERR_INVALID_ARG, "bad sphere light shape");
        } else if (l.kind == PT_LIGHT_DIFFUSE_PLANE) {
            if (l.shape < 0 || l.shape >= d->n_planes) throw PtError(PT_ERR_INVALID_ARG, "bad plane light shape");
        } else if (l.kind == PT_LIGHT_PORTAL_AREA) {
            if (l.shape < 0 || l.shape >= d->n_planes) throw PtError(PT_ERR_INVALID_ARG, "bad portal light shape");
            if (l.n_portals > kMaxPortals)
                throw PtError(PT_ERR_UNSUPPORTED, "more than PT_MAX_PORTALS (" + std::to_string(kMaxPortals) +
                                                      ") portals on one light");
            if (l.n_portals < 0 || l.first_portal < 0 || l.first_portal + l.n_portals > d->n_portals)
                throw PtError(PT_ERR_INVALID_ARG, "bad portal range");
        } else if (l.kind != PT_LIGHT_INFINITE && l.kind != PT_LIGHT_POINT)
            throw PtError(PT_ERR_UNSUPPORTED, "unsupported light kind");
    }
    if (d->sampler.spp <= 0) throw PtError(PT_ERR_INVALID_ARG, "spp must be > 0");
    if (d->film.xres <= 0 || d->film.yres <= 0) throw PtError(PT_ERR_INVALID_ARG, "bad film resolution");
    if (d->integrator.max_depth < 0 || d->integrator.max_depth > 250)
        throw PtError(PT_ERR_UNSUPPORTED, "maxdepth must be in [0, 250]");

    // ---- BVH (host build, reference order; replicas reuse the primary's) ----
    if (bvh_src) {
        s->host_nodes = bvh_src->host_nodes;
        s->host_prim_order = bvh_src->host_prim_order;
    } else if (d->bvh_nodes) {  // the caller's (the reference's) flattened BVH, prims in its order
        if (d->n_bvh_nodes <= 0) throw PtError(PT_ERR_INVALID_ARG, "prebuilt BVH without nodes");
        const LinearNode* nn = (const LinearNode*)d->bvh_nodes;
        s->host_nodes.assign(nn, nn + d->n_bvh_nodes);
        for (int i = 0; i < d->n_bvh_nodes; ++i) {
            const LinearNode& n = s->host_nodes[i];
            const bool ok = n.nprims > 0 ? (n.offset >= 0 && (int64_t)n.offset + n.nprims <= d->n_prims)
                                         : (n.offset > i && n.offset < d->n_bvh_nodes && i + 1 < d->n_bvh_nodes &&
                                            n.axis < 3);
            if (!ok) throw PtError(PT_ERR_INVALID_ARG, "prebuilt BVH node " + std::to_string(i) + " out of range");
        }
        s->host_prim_order.resize((size_t)d->n_prims);
        for (int i = 0; i < d->n_prims; ++i) s->host_prim_order[i] = i;
    } else
        build_bvh(d, &s->host_nodes, &s->host_prim_order);
    std::vector<float4> nodes(2 * s->host_nodes.size());
    for (size_t i = 0; i < s->host_nodes.size(); ++i) {
        const LinearNode& n = s->host_nodes[i];
        nodes[2 * i] = make_float4(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0]);
        uint32_t npax = (uint32_t)n.nprims | ((uint32_t)n.axis << 16);
        nodes[2 * i + 1] = make_float4(n.bmax[1], n.bmax[2], __builtin_bit_cast(float, n.offset),
                                       __builtin_bit_cast(float, npax));
    }
    auto Pv = [&](int k) { return v3(d->P[3 * k], d->P[3 * k + 1], d->P[3 * k + 2]); };
    std::vector<float4> prims(3 * s->host_prim_order.size());
    uint32_t class_mask = 1u;  // material classes among the primitives (misses: class 0)
    for (size_t i = 0; i < s->host_prim_order.size(); ++i) {
        const pt_prim& p = d->prims[s->host_prim_order[i]];
        uint32_t flags = 0;
        V3 a = v3(0, 0, 0), b = a, c = a;
        int pmat = 0, plight = -1;
        if (p.kind == PT_PRIM_AAPLANE) {
            flags = kPrimPlane;
            pmat = d->planes[p.index].material; plight = d->planes[p.index].area_light;
        } else if (p.kind == PT_PRIM_SPHERE) {
            flags = kPrimSphere;
            pmat = d->spheres[p.index].material; plight = d->spheres[p.index].area_light;
        } else {
            const pt_triangle& t = d->triangles[p.index];
            pmat = t.material; plight = t.area_light;
            flags |= (t.flags & 31u) << kPrimTriShift;
            a = Pv(t.v[0]); b = Pv(t.v[1]); c = Pv(t.v[2]);
            // Would Triangle::Intersect reject every ray after the t test?
            // (triangle.cpp:297-318: degenerate dp/duv and zero geometric normal)
            float uv[3][2] = {{0, 0}, {1, 0}, {1, 1}};
            if ((t.flags & PT_TRI_HAS_UV) && d->UV)
                for (int k = 0; k < 3; ++k) { uv[k][0] = d->UV[2 * t.v[k]]; uv[k][1] = d->UV[2 * t.v[k] + 1]; }
            float duv02[2] = {uv[0][0] - uv[2][0], uv[0][1] - uv[2][1]};
            float duv12[2] = {uv[1][0] - uv[2][0], uv[1][1] - uv[2][1]};
            V3 dp02 = a - c, dp12 = b - c;
            float det = duv02[0] * duv12[1] - duv02[1] * duv12[0];
            bool degUV = std::fabs((double)det) < 1e-8;
            V3 dpdu = v3(0, 0, 0), dpdv = v3(0, 0, 0);
            if (!degUV) {
                float inv = 1 / det;
                dpdu = (duv12[1] * dp02 - duv02[1] * dp12) * inv;
                dpdv = (-duv12[0] * dp02 + duv02[0] * dp12) * inv;
            }
            if (degUV || len2(cross(dpdu, dpdv)) == 0) {
                if (len2(cross(c - a, b - a)) == 0) flags |= kPrimDegenerate;
            }
        }
        prims[3 * i + 1] = make_float4(b.x, b.y, b.z, __builtin_bit_cast(float, p.index));
        if (pmat >= 0 && pmat < d->n_materials) {
            const uint32_t mc = material_class(d->materials[pmat].kind, d->materials[pmat].specular != 0);
            flags |= mc << kPrimClassShift;
            class_mask |= 1u << mc;
        }
        uint32_t info = 0;
        if (prim_info_fits(pmat, plight)) info = prim_info_word(pmat, plight);
        else flags |= kPrimInfoTable;
        prims[3 * i] = make_float4(a.x, a.y, a.z, __builtin_bit_cast(float, flags));
        prims[3 * i + 2] = make_float4(c.x, c.y, c.z, __builtin_bit_cast(float, info));
    }
    s->nodes.upload(nodes);
    s->prims.upload(prims);
    s->mat_classes = class_mask;
    s->tris.upload(d->triangles, (size_t)d->n_triangles);
    s->P.upload(d->P, (size_t)3 * d->n_vertices);
    if (d->N) s->N.upload(d->N, (size_t)3 * d->n_vertices);
    if (d->S) s->S.upload(d->S, (size_t)3 * d->n_vertices);
    if (d->UV) s->UV.upload(d->UV, (size_t)2 * d->n_vertices);

    // ---- triangle areas (triangle.cpp:576-582) ----
    std::vector<float> area((size_t)d->n_triangles);
    for (int i = 0; i < d->n_triangles; ++i) {
        const pt_triangle& t = d->triangles[i];
        V3 p0 = Pv(t.v[0]), p1 = Pv(t.v[1]), p2 = Pv(t.v[2]);
        area[i] = (float)(0.5 * (double)len(cross(p1 - p0, p2 - p0)));
    }
    s->tri_area.upload(area);

    // ---- planes and portals (plane.h:15-32, aaportal.cpp:8-13) ----
    auto make_plane = [&](const float* lo, const float* hi, int axis, bool ro, bool sh, const pt_transform& o2w,
                          int material, int light) {
        DevPlane pl{};
        pl.lo = v3(lo[0], lo[1], lo[2]);
        pl.hi = v3(hi[0], hi[1], hi[2]);
        pl.ax = axis;
        pl.ax0 = axis == 2 ? 0 : (axis == 0 ? 1 : 2);
        pl.ax1 = axis == 2 ? 1 : (axis == 0 ? 2 : 0);
        pl.lo_a = pl.lo[pl.ax];
        pl.lo_a0 = pl.lo[pl.ax0];
        pl.lo_a1 = pl.lo[pl.ax1];
        pl.hi_a0 = pl.hi[pl.ax0];
        pl.hi_a1 = pl.hi[pl.ax1];
        pl.facing_fw = ro ? 0 : 1;
        pl.ro_xor_sh = (ro != sh) ? 1 : 0;
        pl.material = material;
        pl.area_light = light;
        std::memcpy(pl.o2w.m, o2w.m, 64);
        std::memcpy(pl.w2o.m, o2w.minv, 64);
        V3 loW = xf_point(pl.o2w, pl.lo), hiW = xf_point(pl.o2w, pl.hi);
        pl.area = (hiW[pl.ax0] - loW[pl.ax0]) * (hiW[pl.ax1] - loW[pl.ax1]);
        return pl;
    };
    std::vector<DevPlane> planes;
    for (int i = 0; i < d->n_planes; ++i) {
        const pt_aaplane& p = d->planes[i];
        planes.push_back(make_plane(p.lo, p.hi, p.axis, (p.flags & PT_TRI_REVERSE_ORIENTATION) != 0,
                                    (p.flags & PT_TRI_SWAPS_HANDEDNESS) != 0, p.object_to_world, p.material,
                                    p.area_light));
    }
    std::vector<DevSphere> spheres;
    for (int i = 0; i < d->n_spheres; ++i) {
        const pt_sphere& sp = d->spheres[i];
        const SphereMembers sm = sphere_members(sp);
        DevSphere ds{};
        ds.radius = sm.radius; ds.zmin = sm.zmin; ds.zmax = sm.zmax;
        ds.theta_min = sm.theta_min; ds.theta_max = sm.theta_max; ds.phi_max = sm.phi_max;
        ds.area = sm.area;
        const bool ro = (sp.flags & PT_TRI_REVERSE_ORIENTATION) != 0, sh = (sp.flags & PT_TRI_SWAPS_HANDEDNESS) != 0;
        ds.ro = ro ? 1 : 0;
        ds.ro_xor_sh = (ro != sh) ? 1 : 0;
        ds.material = sp.material;
        ds.area_light = sp.area_light;
        std::memcpy(ds.o2w.m, sp.object_to_world.m, 64);
        std::memcpy(ds.w2o.m, sp.object_to_world.minv, 64);
        ds.center = xf_point(ds.o2w, v3(0, 0, 0));
        spheres.push_back(ds);
    }
    std::vector<DevPlane> pplanes((size_t)d->n_portals);
    std::vector<DevLight> lights;
    for (int i = 0; i < d->n_lights; ++i) {
        const pt_light& l = d->lights[i];
        DevLight dl{};
        dl.kind = l.kind;
        dl.L = s3(l.L[0], l.L[1], l.L[2]);
        dl.two_sided = l.two_sided;
        dl.shape = l.shape;
        dl.strategy = l.strategy;
        dl.first_portal = l.first_portal;
        dl.n_portals = l.n_portals;
        dl.n_samples = std::max(1, l.n_samples);
        if (l.kind == PT_LIGHT_INFINITE) init_infinite(l, s->host_nodes, &dl);
        else if (l.kind == PT_LIGHT_DIFFUSE_AREA) dl.area = area[l.shape];
        else if (l.kind == PT_LIGHT_DIFFUSE_SPHERE) dl.area = spheres[l.shape].area;
        else if (l.kind == PT_LIGHT_POINT) {  // pLight = LightToWorld(Point3f(0, 0, 0)) (point.h:55)
            M4 m;
            std::memcpy(m.m, l.light_to_world.m, 64);
            dl.center = xf_point(m, v3(0, 0, 0));
        }
        else {
            dl.area = planes[l.shape].area;
            const pt_aaplane& lp = d->planes[l.shape];
            for (int k = 0; k < l.n_portals; ++k) {
                const pt_portal& po = d->portals[l.first_portal + k];
                pplanes[l.first_portal + k] = make_plane(po.lo, po.hi, po.axis, !po.facing_fw,
                                                         (lp.flags & PT_TRI_SWAPS_HANDEDNESS) != 0,
                                                         lp.object_to_world, -1, -1);
            }
        }
        lights.push_back(dl);
    }
    s->planes.upload(planes);
    s->spheres.upload(spheres);
    s->pplanes.upload(pplanes);
    s->lights.upload(lights);
    s->mats.upload(d->materials, (size_t)d->n_materials);

    // ---- light selection distribution (lightdistrib.cpp:68-75, integrator.cpp:515-522) ----
    int nl = d->n_lights;
    std::vector<float> func((size_t)std::max(nl, 1), 1.f), cdf((size_t)nl + 2, 0.f);
    float funcInt = 0;
    if (nl > 0) {
        if (d->integrator.light_strategy == PT_LIGHTS_POWER && nl > 1) {
            for (int i = 0; i < nl; ++i) {
                const DevLight& l = lights[i];
                if (l.kind == PT_LIGHT_INFINITE) {  // InfiniteAreaLight::Power (infinite.cpp:85-89)
                    func[i] = lum_y(lmap_triangle(l.L, .5f, .5f) * (kPi * l.radius * l.radius));
                    continue;
                }
                if (l.kind == PT_LIGHT_POINT) {  // PointLight::Power (point.cpp:51)
                    func[i] = lum_y(l.L * (4 * kPi));
                    continue;
                }
                S3 pw = ((l.L * (float)(l.two_sided ? 2 : 1)) * l.area) * kPi;  // DiffuseAreaLight::Power
                func[i] = lum_y(pw);
            }
        }
        cdf[0] = 0;
        for (int i = 1; i < nl + 1; ++i) cdf[i] = cdf[i - 1] + func[i - 1] / nl;
        funcInt = cdf[nl];
        if (funcInt == 0) { for (int i = 1; i < nl + 1; ++i) cdf[i] = (float)i / (float)nl; }
        else { for (int i = 1; i < nl + 1; ++i) cdf[i] /= funcInt; }
    }
    s->lfunc.upload(func);
    s->lcdf.upload(cdf);

    // ---- film (film.cpp:45-86) ----
    const pt_film_desc& f = d->film;
    Frame& fr = s->fr;
    fr.crop_x0 = (int)std::ceil((float)f.xres * f.crop[0]);
    fr.crop_y0 = (int)std::ceil((float)f.yres * f.crop[2]);
    fr.crop_x1 = (int)std::ceil((float)f.xres * f.crop[1]);
    fr.crop_y1 = (int)std::ceil((float)f.yres * f.crop[3]);
    if (fr.crop_x1 <= fr.crop_x0 || fr.crop_y1 <= fr.crop_y0) throw PtError(PT_ERR_INVALID_ARG, "empty crop window");
    float rx = f.filter_radius[0], ry = f.filter_radius[1];
    if (!(rx > 0) || !(ry > 0)) throw PtError(PT_ERR_INVALID_ARG, "filter radius must be > 0");
    fr.sb_x0 = (int)std::floor((float)fr.crop_x0 + 0.5f - rx);
    fr.sb_y0 = (int)std::floor((float)fr.crop_y0 + 0.5f - ry);
    fr.sb_x1 = (int)std::ceil((float)fr.crop_x1 - 0.5f + rx);
    fr.sb_y1 = (int)std::ceil((float)fr.crop_y1 - 0.5f + ry);
    fr.pb_x0 = fr.sb_x0; fr.pb_y0 = fr.sb_y0; fr.pb_x1 = fr.sb_x1; fr.pb_y1 = fr.sb_y1;
    if (d->integrator.has_pixel_bounds) {
        const int* pb = d->integrator.pixel_bounds;
        fr.pb_x0 = std::max(fr.pb_x0, std::min(pb[0], pb[1]));
        fr.pb_x1 = std::min(fr.pb_x1, std::max(pb[0], pb[1]));
        fr.pb_y0 = std::max(fr.pb_y0, std::min(pb[2], pb[3]));
        fr.pb_y1 = std::min(fr.pb_y1, std::max(pb[2], pb[3]));
    }
    fr.ntx = ceil_div(fr.sb_x1 - fr.sb_x0, 16);
    fr.nty = ceil_div(fr.sb_y1 - fr.sb_y0, 16);
    s->filmdesc = f;
    FilmConsts& fc = s->film;
    fc.crop_x0 = fr.crop_x0; fc.crop_y0 = fr.crop_y0; fc.crop_x1 = fr.crop_x1; fc.crop_y1 = fr.crop_y1;
    fc.sb_x0 = fr.sb_x0; fc.sb_y0 = fr.sb_y0; fc.sb_x1 = fr.sb_x1; fc.sb_y1 = fr.sb_y1;
    fc.rx = rx; fc.ry = ry;
    fc.inv_rx = 1 / rx; fc.inv_ry = 1 / ry;
    {   // source pixels whose samples can reach a film pixel t: a sample of pixel q has pFilm in [q, q + 1]
        // (the pixel plus a [0, 1) offset, rounded), so AddSample's bounds (film.h:121-161) give
        // ceil(q + f - 0.5 - r) <= t <= floor(q + f - 0.5 + r), i.e. |q - t| <= floor(0.5 + r) -- with a
        // margin of floor(0.5 + r) + 0.5 - r on both sides, which float rounding cannot cross unless it is
        // tiny (then one more pixel).  Round 2 used ceil(r + 0.5): 7 x 7 source pixels for the
        // 2-pixel Gaussian instead of 5 x 5.
        const float r = std::max(rx, ry);
        int w = (int)std::floor(0.5f + r);
        if ((float)w + 0.5f - r < 1e-3f) w += 1;
        fc.win = w;
    }
    fc.max_lum = f.max_sample_luminance;
    {
        float expX = 0, expY = 0, alpha = f.gaussian_alpha;
        if (f.filter == PT_FILTER_GAUSSIAN) {
            expX = std::exp(-alpha * rx * rx);
            expY = std::exp(-alpha * ry * ry);
        } else if (f.filter != PT_FILTER_BOX)
            throw PtError(PT_ERR_UNSUPPORTED, "unsupported filter");
        int off = 0;
        for (int y = 0; y < 16; ++y)
            for (int x = 0; x < 16; ++x, ++off) {
                float px = (x + 0.5f) * rx / 16, py = (y + 0.5f) * ry / 16;
                if (f.filter == PT_FILTER_GAUSSIAN) {
                    float gx = smax(0.f, (float)(std::exp(-alpha * px * px) - expX));
                    float gy = smax(0.f, (float)(std::exp(-alpha * py * py) - expY));
                    fc.table[off] = gx * gy;
                } else
                    fc.table[off] = 1.f;
            }
    }

    // ---- Halton (halton.cpp:65-93) ----
    const HaltonTables& ht = halton_tables();
    int res[2] = {fr.sb_x1 - fr.sb_x0, fr.sb_y1 - fr.sb_y0};
    int scales[2], exps[2];
    for (int i = 0; i < 2; ++i) {
        int base = i == 0 ? 2 : 3, scale = 1, e = 0;
        while (scale < std::min(res[i], 128)) { scale *= base; ++e; }
        scales[i] = scale;
        exps[i] = e;
    }
    uint32_t stride = (uint32_t)(scales[0] * scales[1]);
    if ((uint64_t)stride * (uint64_t)d->sampler.spp > 0xffffffffull)
        throw PtError(PT_ERR_UNSUPPORTED, "Halton sample index exceeds 32 bits (spp too large)");
    s->hpc.exp1 = exps[1];
    s->hpc.scale0 = (uint32_t)scales[0];
    s->hpc.mi0 = (uint32_t)mult_inverse(scales[1], scales[0]);
    s->hpc.mi1 = (uint32_t)mult_inverse(scales[0], scales[1]);
    // DirectLighting: the sample arrays occupy [5, 5 + 2 * arrays) and the
    // recursion's dimensions depend on the scene, so keep every prime.
    const bool direct = d->integrator.kind == PT_INTEGRATOR_DIRECT;
    int max_dim = direct ? 1000 : std::min(1000, 6 + 8 * (d->integrator.max_depth + 1));
    std::vector<DivMagic> divs((size_t)max_dim), divs2((size_t)max_dim);
    std::vector<float> c0((size_t)max_dim);
    for (int i = 0; i < max_dim; ++i) {
        divs[i] = make_div_magic((uint32_t)ht.primes[i]);
        divs2[i] = make_div_magic((uint32_t)ht.primes[i] * (uint32_t)ht.primes[i]);
        const float invBase = (float)1 / (float)ht.primes[i];
        c0[i] = invBase * (float)ht.perms[(size_t)ht.prime_sums[i]] / (1 - invBase);
    }
    size_t nperm = (size_t)(max_dim < 1000 ? ht.prime_sums[max_dim] : (int)ht.perms.size());
    s->perm.upload(ht.perms.data(), nperm);
    s->psums.upload(ht.prime_sums.data(), (size_t)max_dim);
    s->divs.upload(divs);
    s->divs2.upload(divs2);
    s->perm_c0.upload(c0);
    s->spp = d->sampler.spp;

    // ---- camera (camera.h ProjectiveCamera, perspective.cpp:45-66) ----
    const pt_camera_desc& cam = d->camera;
    HXF camToScreen = hxf_perspective(cam.fov, 1e-2f, 1000.f);
    const float* sw = cam.screen_window;
    HXF s2r = hxf_mul(hxf_mul(hxf_scale((float)f.xres, (float)f.yres, 1), hxf_scale(1 / (sw[1] - sw[0]), 1 / (sw[2] - sw[3]), 1)),
                      hxf_translate(-sw[0], -sw[3], 0));
    HXF r2c = hxf_mul(hxf_inverse(camToScreen), hxf_inverse(s2r));

    DevScene& ds = s->dev;
    ds.nodes = s->nodes.p;
    ds.prims = s->prims.p;
    ds.n_nodes = (int)s->host_nodes.size();
    ds.n_prims = (int)s->host_prim_order.size();
    ds.tris = s->tris.p;
    ds.P = s->P.p;
    ds.N = d->N ? s->N.p : nullptr;
    ds.S = d->S ? s->S.p : nullptr;
    ds.UV = d->UV ? s->UV.p : nullptr;
    ds.planes = s->planes.p;
    ds.portal_planes = s->pplanes.p;
    ds.spheres = s->spheres.p;
    ds.mats = s->mats.p;
    ds.lights = s->lights.p;
    ds.n_lights = nl;
    ds.n_tris = d->n_triangles;
    ds.n_planes = d->n_planes;
    ds.n_pplanes = d->n_portals;
    ds.n_spheres = d->n_spheres;
    ds.n_mats = d->n_materials;
    ds.n_verts = d->n_vertices;
    ds.ldist_func = s->lfunc.p;
    ds.ldist_cdf = s->lcdf.p;
    ds.ldist_int = funcInt;
    ds.tri_area = s->tri_area.p;
    ds.perm = s->perm.p;
    ds.prime_sums = s->psums.p;
    ds.divs = s->divs.p;
    ds.divs2 = s->divs2.p;
    ds.perm_c0 = s->perm_c0.p;
    ds.max_dim = max_dim;
    // the shading kernel stages the leading dimensions' tables in LDS: as many as fit kHalLdsMax
    // (16 + 4 bytes per dimension + 2 per permutation entry); PT_HAL_LDS=0 disables
    {
        int D = 0;
        const char* e = std::getenv("PT_HAL_LDS");
        if (!(e && e[0] == '0'))
            while (D < max_dim && D < (int)ht.prime_sums.size() - 1 &&
                   (size_t)24 * (D + 1) + 2 * (size_t)ht.prime_sums[D + 1] <= kHalLdsMax && ht.prime_sums[D + 1] < 65536)
                ++D;
        ds.hal_lds_dims = D;
        ds.hal_lds_perm = D > 0 ? ht.prime_sums[D] : 0;
        ds.hal_lds_bytes = (int)tab_align16(D > 0 ? (uint32_t)(24 * D + 2 * ds.hal_lds_perm) : 0u);
        s->hal_lds_bytes = (size_t)ds.hal_lds_bytes;
        // k_shade_tab: the scene tables after them, when they fit kTabLdsMax (PT_SHADE_TAB=0 disables)
        const TabLayout tl = tab_layout((int)s->host_prim_order.size(), d->n_materials, nl, d->n_planes, d->n_portals);
        const char* et = std::getenv("PT_SHADE_TAB");
        s->shade_tab = tl.end <= kTabLdsMax && !(et && et[0] == '0');
        if (s->shade_tab) s->hal_lds_bytes += tl.end;
    }
    ds.hal_exp0 = exps[0];
    ds.hal_scale1 = (uint32_t)scales[1];
    ds.div_scale1 = make_div_magic((uint32_t)scales[1]);
    if (scales[1] == 1) { ds.div_scale1.magic = 0; ds.div_scale1.shift = 0; }
    ds.hal_stride = stride;
    ds.center = d->sampler.sample_pixel_center;
    ds.r2c = to_m4(r2c.m);
    std::memcpy(ds.c2w.m, cam.camera_to_world.m, 64);
    ds.lens_radius = cam.lens_radius;
    ds.focal_distance = cam.focal_distance;
    ds.max_depth = d->integrator.max_depth;
    ds.rr_threshold = d->integrator.rr_threshold;
    ds.integrator = d->integrator.kind;
    ds.dl_strategy = d->integrator.direct_strategy;
    ds.dl_arrays = 0;
    ds.dl_frames = 0;
    if (direct) {
        // DirectLightingIntegrator::Preprocess (directlighting.cpp:43-56): "all"
        // requests two 2D arrays of nSamples per light per depth
        if (ds.dl_strategy == PT_DIRECT_ALL && d->n_lights > 0) ds.dl_arrays = 2 * d->n_lights * ds.max_depth;
        if (5 + 2 * ds.dl_arrays >= 1000)
            throw PtError(PT_ERR_UNSUPPORTED, "DirectLighting sample arrays exceed the Halton dimension table");
        // recursion frames: specular lobes are the only way below depth 0
        ds.dl_frames = (s->features & kFtSpecular) ? std::max(1, ds.max_depth) : 1;
        s->dl_max_samples = 1;
        for (int i = 0; i < d->n_lights; ++i) s->dl_max_samples = std::max(s->dl_max_samples, d->lights[i].n_samples);
    }
    ds.wvl_dim = ds.dl_arrays > 0 ? 5 + 2 * ds.dl_arrays : 5;
    if (d->spectral && (d->integrator.kind == PT_INTEGRATOR_HERO_PATH || d->integrator.kind == PT_INTEGRATOR_HERO_PATH_MIS))
        build_hero(s, d, lights, area, spheres);
    else if (d->integrator.kind == PT_INTEGRATOR_HERO_PATH || d->integrator.kind == PT_INTEGRATOR_HERO_PATH_MIS)
        throw PtError(PT_ERR_INVALID_ARG, "hero integrators need a spectral (SampledSpectrum) scene description");
}

// Largest batch the device indexing supports: path-state fields are
// addressed as field * N + slot in 32-bit arithmetic (kNee payload floats;
// the hero integrators' 60-bin SoA), so (fields + 1) * N must stay below 2^32.
static uint64_t slot_limit(const pt_scene* s) {
    const uint64_t fields = s->hero ? (uint64_t)kNSpec + 1 : (uint64_t)kNee + 1;
    return 0xffffffffull / fields;
}

// Pixels of tiles t with t % stride == offset, tile order then scan order
// (integrator.cpp:533-560), restricted to the integrator's pixelBounds.
// tiles receives, per selected non-empty tile, its first index into pix and
// its pixel rectangle.
struct TileSpan {
    int first;
    int x0, y0, x1, y1;
};
static void tile_pixels(const Frame& fr, int offset, int stride, std::vector<int2>* pix, std::vector<TileSpan>* tiles) {
    pix->clear();
    tiles->clear();
    int nt = fr.ntx * fr.nty;
    for (int t = 0; t < nt; ++t) {
        if (t % stride != offset) continue;
        int tx = t % fr.ntx, ty = t / fr.ntx;
        int x0 = fr.sb_x0 + tx * 16, y0 = fr.sb_y0 + ty * 16;
        int x1 = std::min(x0 + 16, fr.sb_x1), y1 = std::min(y0 + 16, fr.sb_y1);
        const int first = (int)pix->size();
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x)
                if (x >= fr.pb_x0 && x < fr.pb_x1 && y >= fr.pb_y0 && y < fr.pb_y1) pix->push_back(make_int2(x, y));
        if ((int)pix->size() > first) tiles->push_back({first, x0, y0, x1, y1});
    }
}

// Which traversal / shading kernel launch_trace / render_tiles run for this
// scene (pt_scene_query PT_Q_TRACE_KERNEL / PT_Q_SHADE_KERNEL; the bench names
// the kernel its roofline is for).
static int trace_kernel_id(const pt_scene* s) {
    if (s->wide_lds_bytes && !s->count_bytes) return s->wide_hbm ? 7 : 6;
    if (s->trace_persist == 2 && !s->trace_spill && s->lds_scene_bytes && s->trace_lean)
        return s->oct_lds_bytes ? 5 : 3;
    if (s->trace_persist == 2 && !s->trace_spill) return 2;
    return s->trace_persist ? 1 : 0;
}
static int shade_variant_of(const pt_scene* s) { return s->shade_tab && s->shade_variant == 0 ? 5 : s->shade_variant; }
static int shade_kernel_id(const pt_scene* s) {
    if (s->hero) return s->hero_waves == 1 ? 7 : (s->hero_waves == 2 ? 8 : 9);
    if (s->dev.integrator == PT_INTEGRATOR_DIRECT) return 6;
    return shade_variant_of(s);
}

// One traversal launch over the nrays entries of ray queue rq (counts[0] holds
// their number, counts[4] the persistent kernels' fetch cursor, zero): the
// kernel this scene renders with (see create_scene_on).
// One binary (reference-order) traversal launch over the nrays entries of ray queue rq (*cnt holds their
// number, *fetch the persistent kernels' fetch cursor, zero): the kernel this scene renders with when it does
// not take k_trace_w (see create_scene_on), and the retrace kernel behind k_trace_w.
static void launch_binary(pt_scene* s, Work& w, const DevPaths& ps, const uint32_t* rq, uint32_t* cnt,
                          uint32_t* fetch, uint32_t nrays, hipStream_t st, DevStats* stats) {
    const dim3 pg(std::max(1, std::min(ceil_div(nrays, kTraceBlock), s->num_cus * s->trace_bpc)));
    if (s->trace_persist == 2 && !s->trace_spill && s->lds_scene_bytes && s->trace_lean && s->oct_lds_bytes) {
        // k_trace_oct: eight octant images of the BVH + the primitive records + the stack, 4 blocks per CU
        const dim3 og(std::max(1, std::min(ceil_div(nrays, kOctBlock), s->num_cus * 4)));
        hipLaunchKernelGGL(trace_oct_kernel(s->has_spheres), og, dim3(kOctBlock), s->oct_lds_bytes, st, s->dev, ps, rq,
                           cnt, fetch, s->refill_min, s->leaf_min, stats);
    } else if (s->trace_persist == 2 && !s->trace_spill && s->lds_scene_bytes && s->trace_lean) {
        // k_trace_lds: LDS scene, stack of a dummy row + depth rows + the row a push writes above
        const size_t lds = s->lds_scene_bytes + (size_t)(s->stack_rows + 2) * kTraceBlock * sizeof(int);
        hipLaunchKernelGGL(trace_lds_kernel(s->has_spheres), pg, dim3(kTraceBlock), lds, st, s->dev, ps, rq, cnt,
                           fetch, s->refill_min, s->leaf_min, stats);
    } else if (s->trace_persist == 2 && !s->trace_spill) {
        // branch-reduced persistent traversal; LDS stack of depth+1 rows
        const size_t lds = s->lds_scene_bytes + (size_t)(s->stack_rows + 1) * kTraceBlock * sizeof(int);
        hipLaunchKernelGGL(trace_nb_kernel(s->lds_scene_bytes != 0, s->has_spheres), pg, dim3(kTraceBlock), lds, st,
                           s->dev, ps, rq, cnt, fetch, s->refill_min, s->leaf_min, stats);
    } else if (s->trace_persist) {
        // persistent: about one resident wave set; lanes refill from *fetch
        auto kt = trace_pt_kernel(s->lds_scene_bytes != 0, s->trace_spill != 0, s->has_spheres);
        const size_t lds = s->lds_scene_bytes + (size_t)s->stack_rows * kTraceBlock * sizeof(int);
        hipLaunchKernelGGL(kt, pg, dim3(kTraceBlock), lds, st, s->dev, ps, rq, cnt, fetch, s->refill_min,
                           s->leaf_min_pt, s->stack_rows, w.spill.p, stats);
    } else {
        const dim3 tg(std::max(1, std::min(ceil_div(nrays, kTraceBlock), s->num_cus * 16)));
        if (s->lds_scene_bytes)
            hipLaunchKernelGGL(trace_kernel(true, s->has_spheres), tg, dim3(kTraceBlock), s->lds_scene_bytes, st,
                               s->dev, ps, rq, cnt, w.spill.p, stats);
        else
            hipLaunchKernelGGL(trace_kernel(false, s->has_spheres), tg, dim3(kTraceBlock), 0, st, s->dev, ps, rq, cnt,
                               w.spill.p, stats);
    }
}

// One traversal of the nrays entries of ray queue rq (counts[0] holds their number, counts[4] the persistent
// kernels' fetch cursor, zero): k_trace_w over the queue and the binary kernel over the rays it hands back
// (near ties, infinite 1/d: counts[6] their number, counts[7] that launch's fetch cursor), or the binary
// kernel alone (no wide image, or the counting frame, pt_set_count_bytes).
static void launch_trace(pt_scene* s, Work& w, const DevPaths& ps, const uint32_t* rq, uint32_t* counts, uint32_t nrays,
                         hipStream_t st) {
    if (s->wide_lds_bytes && !s->count_bytes) {
        const dim3 pg(std::max(1, std::min(ceil_div(nrays, kTraceBlock), s->num_cus * s->trace_bpc)));
        hipLaunchKernelGGL(s->wide_hbm ? k_trace_w<true> : k_trace_w<false>, pg, dim3(kTraceBlock), s->wide_lds_bytes,
                           st, s->dev, ps, rq, counts + 0, counts + 4, s->refill_min, s->leaf_min_w, w.rqr.p,
                           counts + 6, s->wide_lds_rows, (uint32_t*)w.spill.p, w.stats.p);
        launch_binary(s, w, ps, w.rqr.p, counts + 6, counts + 7, std::min<uint32_t>(nrays, s->num_cus * 2 * kTraceBlock),
                      st, w.stats_rt.p);
        return;
    }
    launch_binary(s, w, ps, rq, counts + 0, counts + 4, nrays, st, w.stats.p);
}

// End of a bounce: the output queue sizes become the next bounce's input sizes,
// and go to the host's pinned words directly.  A hipMemcpyAsync here ran as a
// 1024-thread blit kernel that waited (up to 9 ms, C2 kernel trace) for a CU
// with room beside the other pipeline's persistent trace blocks; one lane
// fits anywhere.
__global__ void k_next_counts(uint32_t* c, volatile uint32_t* host) {
    const uint32_t rays = c[2], paths = c[3];
    host[0] = rays;
    host[1] = paths;
    c[0] = rays;
    c[1] = paths;
    c[2] = 0;
    c[3] = 0;
    c[4] = 0;
    c[5] = 0;
    c[6] = 0;
    c[7] = 0;
}

__global__ void k_set_counts(uint32_t* c, uint32_t rays, uint32_t paths) {
    c[0] = rays;
    c[1] = paths;
    c[2] = 0;
    c[3] = 0;
    c[4] = 0;
    c[5] = 0;
    c[6] = 0;
    c[7] = 0;
}

// A pipeline's counters: its kernels' and the retrace launches' (k_trace_w hands rays back to the binary
// traversal; those count their rays, node visits and primitive tests, and are the retraced rays)
static DevStats read_stats(const Work& w) {
    DevStats d{}, r{};
    HIPCHK(hipMemcpy(&d, w.stats.p, sizeof(DevStats), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&r, w.stats_rt.p, sizeof(DevStats), hipMemcpyDeviceToHost));
    d.closest += r.closest;
    d.shadow += r.shadow;
    d.nodes += r.nodes;
    d.prims += r.prims;
    d.lane_iters += r.lane_iters;
    d.retraced += r.closest + r.shadow;
    return d;
}

struct RenderResult {
    DevStats st{};
    double render_ms = 0, trace_ms = 0, shade_ms = 0;
    uint64_t launches = 0, samples = 0, shade_launches = 0;
    bool wide = false;  // traversed with k_trace_w (node / primitive counters: the retraced rays only)
};

// Render the given tiles into the device accumulation buffer d_accum
// (float4 per cropped pixel).  Synchronous on `stream` (reads queue sizes
// back once per bounce).
static RenderResult render_tiles(pt_scene* s, int offset, int stride, int s_begin, int s_end, float4* d_accum,
                                 hipStream_t stream) {
    if (stride <= 0 || offset < 0 || offset >= stride) throw PtError(PT_ERR_INVALID_ARG, "bad tile partition");
    if (s_begin < 0 || s_end < s_begin) throw PtError(PT_ERR_INVALID_ARG, "bad sample range");
    if ((uint64_t)s->dev.hal_stride * (uint64_t)s_end > 0xffffffffull)
        throw PtError(PT_ERR_UNSUPPORTED, "Halton sample index exceeds 32 bits");
    if (s->dev.dl_arrays > 0 &&  // sample-array entries use indices up to s_end * nSamples
        (uint64_t)s->dev.hal_stride * (uint64_t)s_end * (uint64_t)s->dl_max_samples > 0xffffffffull)
        throw PtError(PT_ERR_UNSUPPORTED, "Halton sample-array index exceeds 32 bits");
    const Frame& fr = s->fr;
    std::vector<int2> pix;
    std::vector<TileSpan> tiles;
    tile_pixels(fr, offset, stride, &pix, &tiles);
    RenderResult rr;
    rr.wide = s->wide_lds_bytes && !s->count_bytes;
    const int npix = (int)pix.size();
    const int spp = s_end - s_begin;
    if (npix == 0 || spp == 0) return rr;
    const int sbw = fr.sb_x1 - fr.sb_x0, sbh = fr.sb_y1 - fr.sb_y0;
    std::vector<int> pixslot((size_t)sbw * sbh, -1);
    for (int i = 0; i < npix; ++i) pixslot[(size_t)(pix[i].y - fr.sb_y0) * sbw + (pix[i].x - fr.sb_x0)] = i;
    // Batches are groups of whole tiles (in tile order) x runs of samples:
    // as many tiles as fit target_slots with all their samples, so each
    // batch carries complete FilmTiles; a single tile too large for that
    // runs its samples in chunks of S.
    struct Group {
        int p0, np, S;
        int bx0, by0, bx1, by1;
    };
    std::vector<Group> groups;
    // default batches: 96 M camera samples (C2: 64 M 877, 96 M 897, 128 M 896, 160 M 896 Msamples/s, same box),
    // 32 M for the hero integrators (1.2 KB of path state per slot: 38 GB per pipeline; C3h 8 / 16 / 32 / 64 M:
    // 107.0 / 109.1 / 110.1 / 110.3 Msamples/s)
    size_t target = s->target_slots ? s->target_slots : (s->hero ? (size_t)32 << 20 : (size_t)96 << 20);
    {   // a render of only a few batches (one rank's shard of a multi-GPU frame) is split into equal batches, a
        // multiple of the pipelines, so the pipelines finish together instead of one running a short remainder
        // batch alone (PT_BATCH_EQUAL=<max batches>, 0 = off)
        const size_t total = (size_t)npix * (size_t)spp;
        const size_t nb = (total + target - 1) / target;
        const int pipes = std::max(1, std::min(s->pipes, kMaxPipes));
        if (nb > 0 && (int)nb <= s->batch_equal) {
            const size_t nbe = (nb + (size_t)pipes - 1) / (size_t)pipes * (size_t)pipes;
            const size_t per_tile = (size_t)256 * (size_t)spp;  // whole 16x16 tiles
            target = std::max(per_tile, ((total + nbe - 1) / nbe + per_tile - 1) / per_tile * per_tile);
        }
    }
    size_t max_slots = 0;
    for (size_t i = 0; i < tiles.size();) {
        size_t j = i;
        size_t gp = 0;
        Group g{tiles[i].first, 0, 0, INT_MAX, INT_MAX, INT_MIN, INT_MIN};
        while (j < tiles.size()) {
            const size_t tp = (size_t)((j + 1 < tiles.size() ? tiles[j + 1].first : npix) - tiles[j].first);
            if (j > i && (gp + tp) * (size_t)spp > target) break;
            gp += tp;
            g.bx0 = std::min(g.bx0, tiles[j].x0);
            g.by0 = std::min(g.by0, tiles[j].y0);
            g.bx1 = std::max(g.bx1, tiles[j].x1);
            g.by1 = std::max(g.by1, tiles[j].y1);
            ++j;
        }
        g.np = (int)gp;
        g.S = (int)std::max<size_t>(1, std::min<size_t>((size_t)spp, target / gp));
        // film pixels the group's samples can reach: its rectangle grown by
        // the filter window, clipped to the cropped film
        g.bx0 = std::max(g.bx0 - s->film.win, s->film.crop_x0);
        g.by0 = std::max(g.by0 - s->film.win, s->film.crop_y0);
        g.bx1 = std::min(g.bx1 + s->film.win, s->film.crop_x1);
        g.by1 = std::min(g.by1 + s->film.win, s->film.crop_y1);
        max_slots = std::max(max_slots, gp * (size_t)g.S);
        groups.push_back(g);
        i = j;
    }
    if (max_slots > slot_limit(s)) throw PtError(PT_ERR_INVALID_ARG, "batch exceeds the path-state indexing limit");
    DBuf<int2> dpix;
    dpix.upload(pix);
    DBuf<int> dslot;
    dslot.upload(pixslot);
    const int maxBlocksTrace = s->num_cus * 16;
    const int maxBlocksShade = s->num_cus * s->shade_bpc;
    const bool direct = s->dev.integrator == PT_INTEGRATOR_DIRECT;
    // k_film_sk (RGB films with windows of 1-2 pixels) reads k_camera's footprint records instead of pFilm
    FilmMeta fmeta{0, s->film.rx, s->film.ry, s->film.inv_rx, s->film.inv_ry};
    const bool sk = s->film_sk > 0 || (s->film_sk < 0 && !s->film_t);  // an explicit PT_FILM_T=1 keeps k_film_t
    if (!s->hero && sk && s->film.win >= (s->film_sk > 0 ? 1 : 2) && s->film.win <= kFilmSkMaxWin) fmeta.win = s->film.win;
    // Batches run on `pipes` pipelines (host thread + stream + path-state
    // buffers each), dealt round-robin: while one batch traces, another
    // shades, so the latency-bound trace and shading kernels overlap on the
    // device.  Each batch's film pass waits for the previous batch's (event
    // chain): the FilmTiles are merged in the reference's tile order.
    struct Batch { int g, s0; };
    std::vector<Batch> batches;
    for (int gi = 0; gi < (int)groups.size(); ++gi)
        for (int s0 = s_begin; s0 < s_end; s0 += groups[gi].S) batches.push_back({gi, s0});
    const int pipes = std::max(1, std::min({s->pipes, kMaxPipes, (int)batches.size()}));
    for (int k = 0; k < pipes; ++k) {
        Work& w = s->work[k];
        HIPCHK(hipSetDevice(s->device));
        w.ensure(max_slots, (size_t)std::max(maxBlocksTrace, s->num_cus * s->trace_bpc) * kTraceBlock,
                 direct ? s->dev.dl_frames : 0, s->hero ? (int)max_slots : 0);
        if (!w.stream) HIPCHK(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
        HIPCHK(hipMemsetAsync(w.stats.p, 0, sizeof(DevStats), w.stream));
        HIPCHK(hipMemsetAsync(w.stats_rt.p, 0, sizeof(DevStats), w.stream));
    }
    // the caller's stream has everything before this call (e.g. the film clear)
    {
        hipEvent_t e0;
        HIPCHK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
        HIPCHK(hipEventRecord(e0, stream));
        for (int k = 0; k < pipes; ++k) HIPCHK(hipStreamWaitEvent(s->work[k].stream, e0, 0));
        HIPCHK(hipStreamSynchronize(stream));
        (void)hipEventDestroy(e0);
    }
    std::vector<hipEvent_t> film_done(batches.size());
    for (auto& e : film_done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::mutex mu;
    std::condition_variable cv;
    std::vector<char> film_recorded(batches.size(), 0);
    // PT_SYNC_CHECK=1 (diagnostics): synchronise after every launch so a
    // device fault is reported against the kernel and bounce that raised it.
    const bool syncCheck = std::getenv("PT_SYNC_CHECK") != nullptr;
    struct PipeTiming { double trace_ms = 0, shade_ms = 0; uint64_t launches = 0, shade_launches = 0, samples = 0; };
    std::vector<PipeTiming> pt(pipes);
    std::vector<std::exception_ptr> err(pipes);
    auto run_pipe = [&](int k) {
        Work& w = s->work[k];
        hipStream_t st = w.stream;
        HIPCHK(hipSetDevice(s->device));
        DevPaths ps = w.paths((int)max_slots);
        DevHeroPaths hps{};
        DevHero hh = s->hh;
        if (s->hero) {
            hh.out60 = w.h_out60.p;
            hh.out_y = w.h_outy.p;
            hps = DevHeroPaths{w.h_beta60.p, w.h_L60.p, w.h_nee60.p, w.h_hs.p};
        }
        std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
        std::vector<char> is_shade;
        auto tev_new = [&](bool shade) {
            hipEvent_t e0, e1;
            HIPCHK(hipEventCreate(&e0));
            HIPCHK(hipEventCreate(&e1));
            tev.push_back({e0, e1});
            is_shade.push_back(shade ? 1 : 0);
            return tev.back();
        };
        auto sync_check = [&](const char* what, int it) {
            if (!syncCheck) return;
            const hipError_t e = hipStreamSynchronize(st);
            if (e != hipSuccess)
                throw PtError(PT_ERR_DEVICE, std::string(what) + " (bounce iteration " + std::to_string(it) + "): " +
                                                 hipGetErrorString(e));
        };
        uint32_t* counts = w.counts.p;
        for (size_t bi = (size_t)k; bi < batches.size(); bi += (size_t)pipes) {
            const Group& g = groups[batches[bi].g];
            const int s0 = batches[bi].s0;
            const int ns = std::min(g.S, s_end - s0);
            const uint32_t nb = (uint32_t)g.np * (uint32_t)ns;
            hipLaunchKernelGGL(fmeta.win > 0 ? k_camera<true> : k_camera<false>, dim3(std::max(1, std::min(ceil_div(nb, 256), s->num_cus * 16))), dim3(256), 0,
                               st, s->dev, ps, dpix.p + g.p0, g.np, s0, ns, s->hpc, w.rq0.p, w.pq0.p, fmeta);
            if (s->hero)  // the hero wavelengths and 60-bin path state of every camera sample
                hipLaunchKernelGGL(k_hero_init, dim3(std::max(1, std::min(ceil_div(nb, 256), s->num_cus * 16))),
                                   dim3(256), 0, st, s->dev, hh, ps, hps, nb);
            hipLaunchKernelGGL(k_set_counts, dim3(1), dim3(1), 0, st, counts, nb, nb);
            HIPCHK(hipGetLastError());
            sync_check("k_camera", 0);
            uint32_t *rq_in = w.rq0.p, *rq_out = w.rq1.p, *pq_in = w.pq0.p, *pq_out = w.pq1.p;
            uint32_t nrays = nb, npaths = nb;
            int iter = 0;
            while (npaths > 0) {
                // counts[0]/[1] hold the input sizes, [2]/[3] the output sizes
                if (nrays > 0) {
                    auto e = tev_new(false);
                    HIPCHK(hipEventRecord(e.first, st));
                    launch_trace(s, w, ps, rq_in, counts, nrays, st);
                    HIPCHK(hipEventRecord(e.second, st));
                    pt[k].launches++;
                    sync_check("k_trace", iter);
                }
                const dim3 sg(std::max(1, std::min(ceil_div(npaths, kShadeBlock), maxBlocksShade)));
                auto es = tev_new(true);
                HIPCHK(hipEventRecord(es.first, st));
                if (s->hero) {
                    hipLaunchKernelGGL(hero_kernel(s->hero_waves, s->features),
                                       sg, dim3(kShadeBlock), 0, st, s->dev, hh, ps, hps, pq_in, counts + 1, rq_out,
                                       counts + 2, pq_out, counts + 3, w.stats.p);
                } else {
                    const ShadeKernel kshade =
                        direct ? k_shade_dl<kFtAll>
                               : shade_kernel(shade_variant_of(s), s->features, s->count_bytes);
                    // scenes with two or more material classes: the path queue grouped by class per 4096-entry
                    // chunk first, so a shading wave's paths mostly take one BSDF's code (k_shade_sort)
                    const bool sorted = !direct && s->shade_sort && __builtin_popcount(s->mat_classes) > 1;
                    if (sorted)
                        hipLaunchKernelGGL(k_shade_sort, dim3(std::max(1, ceil_div(npaths, kSortChunk))), dim3(256), 0,
                                           st, s->dev, ps, pq_in, counts + 1, w.pqs.p);
                    // dynamic LDS: the Halton tables, + the scene tables for the builds that stage them (variants 3
                    // and 5; k_shade and k_shade_w3h read the tables from HBM: ds.hal_lds_bytes alone)
                    const int sv = shade_variant_of(s);
                    const size_t shade_lds = direct ? 0 : ((sv == 3 || sv == 5) ? s->hal_lds_bytes
                                                                                   : (size_t)s->dev.hal_lds_bytes);
                    hipLaunchKernelGGL(kshade, sg, dim3(kShadeBlock), shade_lds, st, s->dev, ps,
                                       sorted ? w.pqs.p : pq_in, counts + 1, rq_out, counts + 2, pq_out, counts + 3,
                                       w.stats.p);
                }
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(es.second, st));
                pt[k].shade_launches++;
                sync_check("k_shade", iter);
                hipLaunchKernelGGL(k_next_counts, dim3(1), dim3(1), 0, st, counts, w.host_counts);
                HIPCHK(hipGetLastError());
                HIPCHK(hipStreamSynchronize(st));
                nrays = ((volatile uint32_t*)w.host_counts)[0];
                npaths = ((volatile uint32_t*)w.host_counts)[1];
                std::swap(rq_in, rq_out);
                std::swap(pq_in, pq_out);
                if (++iter > 100000) throw PtError(PT_ERR_STATE, "path loop did not terminate");
            }
            if (bi > 0) {  // FilmTiles merge in batch (tile) order
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return film_recorded[bi - 1] != 0; });
                lk.unlock();
                HIPCHK(hipStreamWaitEvent(st, film_done[bi - 1], 0));
            }
            const int bw = g.bx1 - g.bx0, bh = g.by1 - g.by0;
            if (bw > 0 && bh > 0) {
                const dim3 fg(std::max(1, std::min(ceil_div(bw * bh, 4), s->num_cus * 32)));
                if (s->hero && s->film_sq && !s->film_blk) {
                    // k_film_s60_sq: one wave per 2 x 2 film pixels, 16 sample loads in flight (C3h: 2 x 2 beat
                    // 3 x 2, 4 x 2 and 3 x 3 squares, and 16 loads beat 4 and 8)
                    hipLaunchKernelGGL((k_film_s60_sq<2, 2, 16>), dim3(ceil_div(bw, 2) * ceil_div(bh, 2)), dim3(64), 0, st,
                                       hh, ps, s->film, dslot.p, g.p0, g.np, ns, g.bx0, g.by0, bw, bh, d_accum);
                } else if (s->hero && s->film_blk && s->film.win <= kF60MaxWin)
                    hipLaunchKernelGGL(k_film_s60_blk, dim3(ceil_div(bw, 8) * ceil_div(bh, 8)), dim3(1024), 0, st, hh,
                                       ps, s->film, dslot.p, g.p0, g.np, ns, g.bx0, g.by0, bw, bh, d_accum);
                else if (s->hero)
                    hipLaunchKernelGGL(k_film_s60, fg, dim3(256), 0, st, hh, ps, s->film, dslot.p, g.p0, g.np,
                                       ns, g.bx0, g.by0, bw, bh, d_accum);
                else if (fmeta.win > 0) {
                    hipLaunchKernelGGL(k_film_prep, dim3(std::max(1, std::min(ceil_div(nb, 256), s->num_cus * 16))),
                                       dim3(256), 0, st, ps, s->film.max_lum, nb);
                    hipLaunchKernelGGL(k_film_sk, dim3(ceil_div(bw, 64 / (2 * fmeta.win + 1)) *
                                                       ceil_div(bh, 2 * fmeta.win + 1)),
                                       dim3(64), 0, st, ps, s->film, dslot.p, g.p0, g.np, ns, g.bx0, g.by0, bw, bh,
                                       d_accum, s->film_skew);
                }
                else if (s->film_t && s->film.win >= 2 && s->film.win <= 16)  // box (win 1): k_film is faster
                    hipLaunchKernelGGL(k_film_t, dim3(ceil_div(ceil_div(bw, 8) * ceil_div(bh, 8), 4)), dim3(256), 0, st, ps,
                                       s->film, dslot.p, g.p0, g.np, ns, g.bx0, g.by0, bw, bh, d_accum);
                else
                    hipLaunchKernelGGL(k_film, fg, dim3(256), 0, st, ps, s->film, dslot.p, g.p0, g.np, ns, g.bx0,
                                       g.by0, bw, bh, d_accum);
                HIPCHK(hipGetLastError());
                sync_check("k_film", 0);
            }
            HIPCHK(hipEventRecord(film_done[bi], st));
            {
                std::lock_guard<std::mutex> lk(mu);
                film_recorded[bi] = 1;
            }
            cv.notify_all();
            pt[k].samples += nb;
        }
        HIPCHK(hipStreamSynchronize(st));
        for (size_t i = 0; i < tev.size(); ++i) {
            float t = 0;
            HIPCHK(hipEventElapsedTime(&t, tev[i].first, tev[i].second));
            (is_shade[i] ? pt[k].shade_ms : pt[k].trace_ms) += t;
            (void)hipEventDestroy(tev[i].first);
            (void)hipEventDestroy(tev[i].second);
        }
    };
    const auto t0 = std::chrono::steady_clock::now();
    {
        std::vector<std::thread> th;
        for (int k = 1; k < pipes; ++k)
            th.emplace_back([&, k] {
                try {
                    run_pipe(k);
                } catch (...) {
                    err[k] = std::current_exception();
                    std::lock_guard<std::mutex> lk(mu);  // release waiters: mark this pipe's batches done
                    for (size_t bi = (size_t)k; bi < batches.size(); bi += (size_t)pipes) film_recorded[bi] = 1;
                    cv.notify_all();
                }
            });
        try {
            run_pipe(0);
        } catch (...) {
            err[0] = std::current_exception();
            std::lock_guard<std::mutex> lk(mu);
            for (size_t bi = 0; bi < batches.size(); bi += (size_t)pipes) film_recorded[bi] = 1;
            cv.notify_all();
        }
        for (auto& t : th) t.join();
    }
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    rr.render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto& e : film_done) (void)hipEventDestroy(e);
    for (int k = 0; k < pipes; ++k) {
        const DevStats d = read_stats(s->work[k]);
        rr.st.closest += d.closest; rr.st.shadow += d.shadow; rr.st.nodes += d.nodes; rr.st.prims += d.prims;
        rr.st.dim_overflow += d.dim_overflow; rr.st.lane_iters += d.lane_iters; rr.st.lane_steps += d.lane_steps;
        rr.st.shade_bytes += d.shade_bytes;
        rr.st.wnodes += d.wnodes; rr.st.wprims += d.wprims; rr.st.retraced += d.retraced;
        rr.trace_ms += pt[k].trace_ms;
        rr.shade_ms += pt[k].shade_ms;
        rr.launches += pt[k].launches;
        rr.shade_launches += pt[k].shade_launches;
        rr.samples += pt[k].samples;
    }
    if (rr.st.dim_overflow) throw PtError(PT_ERR_UNSUPPORTED, "Halton dimension table exhausted");
#ifdef PT_GUARDS
    unsigned int guard = 0;
    HIPCHK(hipMemcpyFromSymbol(&guard, HIP_SYMBOL(g_pt_guard), sizeof guard));
    if (guard)
        throw PtError(PT_ERR_STATE, "PT_GUARDS: index out of range at " +
                                        std::string(guard / 100000 == 1 ? "devfuncs.h" : "kernels.hip") + ":" +
                                        std::to_string(guard % 100000));
#endif
    if (std::getenv("PT_TRACE_DEBUG") && rr.st.lane_iters)
        std::fprintf(stderr, "[pt] trace SIMD utilisation %.3f (%llu steps / %llu lane-iterations)\n",
                     (double)(rr.st.nodes + rr.st.prims) / (double)rr.st.lane_iters,
                     (unsigned long long)(rr.st.nodes + rr.st.prims), (unsigned long long)rr.st.lane_iters);
    return rr;
}

// Film::WriteImage (film.cpp:169-211) for an accumulation buffer holding
// Film::Pixel's XYZ sum and filter weight sum.
static void resolve_film(size_t np, float scale, const float* accum, float* rgb) {
    for (size_t o = 0; o < np; ++o) {
        const float* c = &accum[4 * o];
        const float px[3] = {c[0], c[1], c[2]};
        float out[3];
        out[0] = 3.240479f * px[0] - 1.537150f * px[1] - 0.498535f * px[2];
        out[1] = -0.969256f * px[0] + 1.875991f * px[1] + 0.041556f * px[2];
        out[2] = 0.055648f * px[0] - 0.204043f * px[1] + 1.057311f * px[2];
        float ws = 0.f + c[3];
        if (ws != 0) {
            float invWt = (float)1 / ws;
            for (int k = 0; k < 3; ++k) out[k] = smax(0.f, out[k] * invWt);
        }
        float splat[3];
        splat[0] = 3.240479f * 0.f - 1.537150f * 0.f - 0.498535f * 0.f;
        splat[1] = -0.969256f * 0.f + 1.875991f * 0.f + 0.041556f * 0.f;
        splat[2] = 0.055648f * 0.f - 0.204043f * 0.f + 1.057311f * 0.f;
        for (int k = 0; k < 3; ++k) {
            out[k] += 1.f * splat[k];
            out[k] *= scale;
            rgb[3 * o + k] = out[k];
        }
    }
}

static void resolve(const pt_scene* s, const float* accum, float* rgb) {
    resolve_film((size_t)s->fr.width() * s->fr.height(), s->filmdesc.scale, accum, rgb);
}

// Cropped film size from the description alone (Film::Film, film.cpp:50-60).
static void crop_size(const pt_film_desc& f, int* w, int* h) {
    if (f.xres <= 0 || f.yres <= 0) throw PtError(PT_ERR_INVALID_ARG, "bad film resolution");
    const int x0 = (int)std::ceil((float)f.xres * f.crop[0]), x1 = (int)std::ceil((float)f.xres * f.crop[1]);
    const int y0 = (int)std::ceil((float)f.yres * f.crop[2]), y1 = (int)std::ceil((float)f.yres * f.crop[3]);
    if (x1 <= x0 || y1 <= y0) throw PtError(PT_ERR_INVALID_ARG, "empty crop window");
    *w = x1 - x0;
    *h = y1 - y0;
}

static void fill_stats(const RenderResult& r, pt_stats* st) {
    if (!st) return;
    st->camera_rays = r.samples;
    st->closest_rays = r.st.closest;
    st->shadow_rays = r.st.shadow;
    st->node_visits = r.st.nodes;
    st->prim_tests = r.st.prims;
    st->samples = r.samples;
    st->render_ms = r.render_ms;
    st->trace_ms = r.trace_ms;
    st->trace_launches = r.launches;
    st->shade_ms = r.shade_ms;
    st->shade_launches = r.shade_launches;
    st->shade_bytes = r.st.shade_bytes;
    st->reduce_ms = 0;
    st->retraced_rays = r.st.retraced;
    st->wide_node_visits = r.st.wnodes;
    st->wide_prim_tests = r.st.wprims;
    st->trace_wide = r.wide ? 1 : 0;
    st->reserved = 0;
}

template <class F>
static pt_status guarded(F&& f) {
    try {
        f();
        return PT_OK;
    } catch (const PtError& e) {
        g_last_error = e.what();
        return e.status;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of host memory";
        return PT_ERR_OOM;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return PT_ERR_STATE;
    }
}

static void require_device() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) throw PtError(PT_ERR_DEVICE, "no HIP device available (the product has no CPU fallback)");
}

#define NCCLCHK(x)                                                                                      \
    do {                                                                                                \
        ncclResult_t r_ = (x);                                                                          \
        if (r_ != ncclSuccess) throw PtError(PT_ERR_DEVICE, std::string(#x) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// The devices of this process (pt_init); empty: the calling thread's current device.
static std::vector<int> g_devices;
static std::mutex g_devices_mu;

// Deepest traversal stack the flattened BVH can need: interior nodes on the
// longest root-to-leaf path (each pushes one entry).
static int bvh_stack_bound(const std::vector<LinearNode>& nodes) {
    if (nodes.empty()) return 0;
    int best = 0;
    std::vector<std::pair<int, int>> todo{{0, 0}};
    while (!todo.empty()) {
        auto [i, d] = todo.back();
        todo.pop_back();
        if (i < 0 || i >= (int)nodes.size()) continue;
        if (nodes[i].nprims > 0) { best = std::max(best, d); continue; }
        todo.push_back({i + 1, d + 1});
        todo.push_back({nodes[i].offset, d + 1});
    }
    return best;
}

// The binary BVH collapsed to 4-wide nodes for k_trace_w (kernels.hip): a wide node takes its binary
// node's two children and opens the interior child of largest surface area until it holds four children
// (or only leaves are left); every child is a node of the reference's tree with its exact bounds -- an
// interior one becomes the next wide node, a leaf keeps its primitive range (bvh.cpp:640-658 layout).
// Image per wide node (`stride` bytes, 112 in LDS, 128 in HBM: one cache line): {lo.x of children 0-3} {hi.x}
// {lo.y} {hi.y} {lo.z} {hi.z} {child words} [pad];
// child word = 0x80000000 | byte offset of a wide node in the image (the kernel adds the LDS base), or
// first primitive | count << 24 for a leaf; unused slots: bounds +inf / -inf (never hit) and word 0.
// *rows: LDS stack rows per lane -- the dummy row, the deepest stack a node can be visited at, and the three
// rows the node step writes above its top.  Returns false when the tree does not fit the child-word encoding.
static bool build_wide(const std::vector<LinearNode>& bn, uint32_t stride, std::vector<float4>* img, int* n_wide,
                       int* rows) {
    const size_t q4 = stride / 16;  // float4s per wide node (7, or 8 with a pad for one 128-B line each)
    img->clear();
    *n_wide = 0;
    *rows = 0;
    if (bn.empty()) return true;
    for (const LinearNode& n : bn)
        if (n.nprims > 127 || (n.nprims > 0 && (uint64_t)n.offset + n.nprims > (1u << 24))) return false;
    auto area = [&](int i) {
        const LinearNode& n = bn[i];
        const double dx = (double)n.bmax[0] - n.bmin[0], dy = (double)n.bmax[1] - n.bmin[1],
                     dz = (double)n.bmax[2] - n.bmin[2];
        return dx * dy + dy * dz + dx * dz;
    };
    struct Wide { int bin[4], wid[4]; };  // children: binary node ids (-1 unused), wide ids of interior ones
    std::vector<Wide> wn(1);
    struct Todo { int bin, wide, depth; };
    std::vector<Todo> todo{{0, 0, 0}};
    int max_depth = 0;
    std::vector<int> ch;
    while (!todo.empty()) {
        const Todo t = todo.back();
        todo.pop_back();
        ch.clear();
        if (bn[t.bin].nprims > 0) ch.push_back(t.bin);  // a one-leaf tree
        else { ch.push_back(t.bin + 1); ch.push_back(bn[t.bin].offset); }
        while (ch.size() < 4) {
            int best = -1;
            for (int k = 0; k < (int)ch.size(); ++k)
                if (bn[ch[k]].nprims == 0 && (best < 0 || area(ch[k]) > area(ch[best]))) best = k;
            if (best < 0) break;
            const int c = ch[best];
            ch[best] = c + 1;
            ch.push_back(bn[c].offset);
        }
        max_depth = std::max(max_depth, t.depth);
        Wide w{{-1, -1, -1, -1}, {-1, -1, -1, -1}};
        for (int k = 0; k < (int)ch.size(); ++k) {
            w.bin[k] = ch[k];
            if (bn[ch[k]].nprims == 0) {
                w.wid[k] = (int)wn.size();
                wn.push_back(Wide{});
                // visited with up to (children - 1) entries pushed above the parent's stack
                todo.push_back({ch[k], w.wid[k], t.depth + (int)ch.size() - 1});
            }
        }
        wn[t.wide] = w;
    }
    const size_t nw = wn.size();
    if (nw * stride >= 0x80000000ull) return false;
    img->assign(nw * q4, make_float4(0, 0, 0, 0));
    for (size_t i = 0; i < nw; ++i) {
        float lo[3][4], hi[3][4];
        uint32_t word[4];
        for (int k = 0; k < 4; ++k) {
            const int c = wn[i].bin[k];
            if (c < 0) {
                for (int a = 0; a < 3; ++a) { lo[a][k] = INFINITY; hi[a][k] = -INFINITY; }
                word[k] = 0;
                continue;
            }
            const LinearNode& n = bn[c];
            for (int a = 0; a < 3; ++a) { lo[a][k] = n.bmin[a]; hi[a][k] = n.bmax[a]; }
            word[k] = n.nprims > 0 ? ((uint32_t)n.offset | ((uint32_t)n.nprims << 24))
                                   : (0x80000000u | (uint32_t)(stride * (uint32_t)wn[i].wid[k]));
        }
        float4* q = img->data() + q4 * i;
        for (int a = 0; a < 3; ++a) {
            q[2 * a] = make_float4(lo[a][0], lo[a][1], lo[a][2], lo[a][3]);
            q[2 * a + 1] = make_float4(hi[a][0], hi[a][1], hi[a][2], hi[a][3]);
        }
        q[6] = make_float4(__builtin_bit_cast(float, word[0]), __builtin_bit_cast(float, word[1]),
                           __builtin_bit_cast(float, word[2]), __builtin_bit_cast(float, word[3]));
    }
    *n_wide = (int)nw;
    *rows = max_depth + 4;
    return true;
}

// One device's copy of the scene: build (or copy the BVH of bvh_src),
// upload, and pick the kernel variants for it.
static std::unique_ptr<pt_scene> create_scene_on(int device, const pt_scene_desc* desc, const pt_scene* bvh_src) {
    HIPCHK(hipSetDevice(device));
    std::unique_ptr<pt_scene> s(new pt_scene);
    s->device = device;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, s->device));
    s->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    s->features = scene_features(desc);
    if (const char* t = std::getenv("PT_SHADE_FEATURES")) s->features |= std::atoi(t) & kFtAll;
    build_scene(s.get(), desc, bvh_src);
    const int sbound = bvh_stack_bound(s->host_nodes);
    s->trace_spill = sbound > kStackLds;
    s->stack_rows = s->trace_spill ? kStackLds : std::max(1, sbound);
    if (const char* t = std::getenv("PT_STACK_ROWS")) {  // test hook: force the spill path
        s->stack_rows = std::max(1, std::min(kStackLds, std::atoi(t)));
        s->trace_spill = sbound > s->stack_rows;
    }
    // kernel variants: LDS-resident BVH for small scenes (PT_TRACE_LDS=0 disables),
    // shading register budget (PT_SHADE_VARIANT=0|3|5, below)
    const size_t scene_bytes = (2 * (size_t)s->dev.n_nodes + 3 * (size_t)s->dev.n_prims) * sizeof(float4);
    const char* e = std::getenv("PT_TRACE_LDS");
    s->lds_scene_bytes = (scene_bytes > 0 && scene_bytes <= (size_t)kLdsSceneMax && !(e && e[0] == '0'))
                             ? scene_bytes : 0;
    if (const char* t = std::getenv("PT_HERO_WAVES")) s->hero_waves = std::atoi(t);
    const char* v = std::getenv("PT_SHADE_VARIANT");
    if (v) {
        s->shade_variant = std::atoi(v);
        if (s->shade_variant != 0 && s->shade_variant != 3 && s->shade_variant != 4 && s->shade_variant != 5)
            throw PtError(PT_ERR_INVALID_ARG, "PT_SHADE_VARIANT must be 0, 3, 4 or 5");
        // k_shade_w3 and k_shade_tab stage the scene tables in LDS: without room for them (tables larger
        // than kTabLdsMax, or PT_SHADE_TAB=0) the launch's dynamic LDS holds only the Halton tables, so
        // those builds would copy past their allocation -- take k_shade instead
        if (!s->shade_tab && s->shade_variant != 4) s->shade_variant = 0;
        if (s->shade_variant == 3 || s->shade_variant == 4) s->shade_bpc = kShadeBpcW3;
    } else if (s->shade_tab && !s->hero && s->features == kFtPortalOnly) {
        // the 3-waves-per-SIMD build of k_shade_tab when it needs no scratch (spills cost more than the
        // third wave gains), with the grid-stride loop sized for it (PT_SHADE_BPC overrides).  Only for
        // portal-only scenes: the MIS kernels' 3-wave build gives up the body prefetch (kLean), and with
        // two pipelines overlapping the 2-wave build, which leaves VGPRs for two trace waves per SIMD,
        // renders C4 faster (442 vs 431 Msamples/s) although its isolated launches are slower
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, (const void*)shade_kernel(3, s->features)) == hipSuccess && fa.localSizeBytes == 0) {
            s->shade_variant = 3;
            s->shade_bpc = kShadeBpcW3;
        }
    } else if (!s->shade_tab && !s->hero && s->features == kFtPortalOnly) {
        // the same 3-wave build with the scene tables read from HBM (C5's ten million primitive records)
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, (const void*)shade_kernel(4, s->features)) == hipSuccess && fa.localSizeBytes == 0) {
            s->shade_variant = 4;
            s->shade_bpc = kShadeBpcW3;
        }
    }
    s->has_spheres = (s->features & kFtSphere) != 0;
    if (const char* t = std::getenv("PT_TRACE_PERSIST")) s->trace_persist = std::atoi(t);
    if (const char* t = std::getenv("PT_TRACE_LEAN")) s->trace_lean = t[0] != '0';
    {   // k_trace_oct when four blocks of it fit a CU's LDS (160 KB): octant images + primitives + stack
        const size_t oct = 8 * 32 * (size_t)s->dev.n_nodes + 48 * (size_t)s->dev.n_prims +
                           (size_t)(s->stack_rows + 2) * kOctBlock * sizeof(int);
        const char* t = std::getenv("PT_TRACE_OCT");
        // the CU's LDS from the device (gfx950: 160 KB); without room for four blocks: k_trace_lds
        const size_t cu_lds = prop.maxSharedMemoryPerMultiProcessor > 0 ? (size_t)prop.maxSharedMemoryPerMultiProcessor
                                                                          : (size_t)prop.sharedMemPerMultiprocessor;
        s->oct_lds_bytes = (s->lds_scene_bytes && !s->trace_spill && 4 * oct <= cu_lds && t && t[0] == '1') ? oct : 0;
    }
    {   // k_trace_w (4-wide BVH) for scenes without spheres (the sphere test's EFloat acceptance is left to the
        // binary order); the binary kernel stays the retrace and counting traversal.  LDS-resident scenes (the
        // k_trace_lds ones): image + primitives staged in LDS; HBM-resident ones (the k_trace_pt / k_trace_nb ones):
        // image in HBM, LDS stack rows + spill
        const char* t = std::getenv("PT_TRACE_WIDE");
        const bool lds = s->trace_persist == 2 && !s->trace_spill && s->lds_scene_bytes && s->trace_lean &&
                         !s->oct_lds_bytes;
        const bool hbm = !s->lds_scene_bytes && s->trace_persist >= 1;
        std::vector<float4> img;
        int nw = 0, rows = 0;
        if ((lds || hbm) && !s->has_spheres && !(t && t[0] == '0') &&
            build_wide(s->host_nodes, lds ? kWideStrideLds : kWideStrideHbm, &img, &nw, &rows) && nw > 0) {
            const size_t scene = lds ? (size_t)nw * kWideStrideLds + (size_t)s->dev.n_prims * 48 : 0;
            // HBM: at most kWideLdsRowsMax rows per lane in LDS (12 blocks of 128 lanes at 6 waves per SIMD), the
            // rest in the spill column (kSpillWords entries)
            int lrows = lds ? rows : std::min(rows, kWideLdsRowsMax);
            if (const char* r = std::getenv("PT_WIDE_LDS_ROWS"))  // test hook: force the HBM kernel's spill path
                if (hbm) lrows = std::max(1, std::min(lrows, std::atoi(r)));
            if ((lds && scene <= (size_t)kLdsSceneMax + 4096 && rows <= 64) ||
                (hbm && rows - lrows <= kSpillWords)) {
                s->wnodes.upload(img);
                s->dev.wnodes = s->wnodes.p;
                s->dev.n_wnodes = nw;
                float sc_max = 0;
                for (int k = 0; k < 3; ++k)
                    sc_max = std::max({sc_max, std::fabs(s->host_nodes[0].bmin[k]), std::fabs(s->host_nodes[0].bmax[k])});
                s->dev.wide_scale = sc_max;
                s->wide_hbm = hbm;
                s->wide_rows = rows;
                s->wide_lds_rows = lrows;
                s->wide_lds_bytes = scene + (size_t)lrows * kTraceBlock * sizeof(uint32_t);
            }
        }
        if (const char* l = std::getenv("PT_LEAF_MIN_W")) s->leaf_min_w = std::max(1, std::atoi(l));
        else if (s->wide_hbm) s->leaf_min_w = s->leaf_min_pt;
    }
    // A BVH traversed from HBM by the binary walk (k_trace_pt / k_trace_nb: scenes with spheres) renders its
    // batches on one pipeline: that traversal is bound by the latency of its node fetches at 7 waves per SIMD,
    // and a shading launch beside it takes waves and memory bandwidth from it (round 5, C5: 168.4 / 167.9 vs
    // 163.4 / 163.7 Msamples/s). The wide traversal from HBM (k_trace_w<true>) and the
    // LDS-resident scenes keep two (round 6, C5 @16 spp: 236.7 / 236.2 vs 226.3 / 227.2; C2 / C3 / C4 2-12 %)
    if (!s->lds_scene_bytes && !s->wide_hbm) s->pipes = 1;
    if (std::getenv("PT_TRACE_DEBUG"))
        std::fprintf(stderr, "[pt] BVH stack rows %d (spill %d), LDS scene %zu B, wide %zu B (%d nodes, %d rows), "
                     "trace kernel %s\n", s->stack_rows, s->trace_spill, s->lds_scene_bytes, s->wide_lds_bytes,
                     s->dev.n_wnodes, s->wide_rows,
                     s->wide_lds_bytes                                                             ? "k_trace_w"
                     : s->trace_persist == 2 && !s->trace_spill && s->lds_scene_bytes && s->trace_lean ? "k_trace_lds"
                     : s->trace_persist == 2 && !s->trace_spill                                    ? "k_trace_nb"
                     : s->trace_persist                                                            ? "k_trace_pt"
                                                                                                   : "k_trace");
    if (const char* t = std::getenv("PT_FILM_BLK")) s->film_blk = std::atoi(t);
    if (const char* t = std::getenv("PT_FILM_SQ")) s->film_sq = std::atoi(t);
    if (const char* t = std::getenv("PT_FILM_T")) s->film_t = std::atoi(t);
    if (const char* t = std::getenv("PT_FILM_SK")) s->film_sk = std::atoi(t);
    if (const char* t = std::getenv("PT_FILM_SKEW")) s->film_skew = std::min(2, std::max(0, std::atoi(t)));
    if (const char* t = std::getenv("PT_SHADE_BPC")) s->shade_bpc = std::max(1, std::min(64, std::atoi(t)));
    if (const char* t = std::getenv("PT_TRACE_BPC")) s->trace_bpc = std::max(1, std::min(64, std::atoi(t)));
    if (const char* t = std::getenv("PT_REFILL")) s->refill_min = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("PT_LEAF_MIN")) s->leaf_min = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("PT_LEAF_MIN_PT")) s->leaf_min_pt = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("PT_BATCH_EQUAL")) s->batch_equal = std::max(0, std::atoi(t));
    if (const char* t = std::getenv("PT_SHADE_SORT")) s->shade_sort = t[0] != '0';
    if (const char* t = std::getenv("PT_PIPES")) s->pipes = std::max(1, std::min(kMaxPipes, std::atoi(t)));
    return s;
}

__global__ void k_film_add(float4* __restrict__ dst, const float4* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 a = dst[i], b = src[i];
        dst[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
}

static void add_stats(RenderResult* a, const RenderResult& b) {
    a->st.closest += b.st.closest; a->st.shadow += b.st.shadow; a->st.nodes += b.st.nodes; a->st.prims += b.st.prims;
    a->st.dim_overflow += b.st.dim_overflow; a->st.lane_iters += b.st.lane_iters; a->st.lane_steps += b.st.lane_steps;
    a->samples += b.samples;
    a->launches += b.launches;
    a->trace_ms += b.trace_ms;
    a->shade_ms += b.shade_ms;
    a->shade_launches += b.shade_launches;
    a->st.shade_bytes += b.st.shade_bytes;
    a->st.wnodes += b.st.wnodes; a->st.wprims += b.st.wprims; a->st.retraced += b.st.retraced;
    a->wide |= b.wide;
    a->render_ms = std::max(a->render_ms, b.render_ms);
}

// The whole frame on every device of the scene (SamplerIntegrator::Render
// with the tile loop dealt round-robin over the devices, t % n == k), one host
// thread per device, each into its own device film; the films are summed on
// the primary device in device order (peer copies over xGMI) -- a fixed order,
// so the result does not depend on thread timing.
static RenderResult render_all_devices(pt_scene* s, float4* d_accum0) {
    const int nd = 1 + (int)s->replicas.size();
    std::vector<pt_scene*> sc(nd);
    sc[0] = s;
    for (int k = 1; k < nd; ++k) sc[k] = s->replicas[k - 1].get();
    const size_t np = (size_t)s->fr.width() * s->fr.height();
    std::vector<std::unique_ptr<DBuf<float4>>> films(nd);
    std::vector<RenderResult> res(nd);
    std::vector<std::exception_ptr> err(nd);
    std::vector<std::thread> th;
    for (int k = 0; k < nd; ++k)
        th.emplace_back([&, k] {
            try {
                HIPCHK(hipSetDevice(sc[k]->device));
                float4* film = d_accum0;
                if (k > 0) {
                    films[k].reset(new DBuf<float4>);
                    films[k]->alloc(np);
                    film = films[k]->p;
                    HIPCHK(hipMemset(film, 0, np * sizeof(float4)));
                }
                res[k] = render_tiles(sc[k], k, nd, 0, sc[k]->spp, film, nullptr);
            } catch (...) {
                err[k] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    HIPCHK(hipSetDevice(s->device));
    RenderResult out = res[0];
    if (nd > 1) {
        DBuf<float4> tmp;
        tmp.alloc(np);
        for (int k = 1; k < nd; ++k) {
            HIPCHK(hipMemcpyPeer(tmp.p, s->device, films[k]->p, sc[k]->device, np * sizeof(float4)));
            hipLaunchKernelGGL(k_film_add, dim3(std::max(1, std::min(ceil_div((long)np, 256), 4096))), dim3(256), 0, 0,
                               d_accum0, tmp.p, np);
            HIPCHK(hipGetLastError());
            add_stats(&out, res[k]);
        }
        HIPCHK(hipDeviceSynchronize());
    }
    return out;
}

}  // namespace pt

using namespace pt;

extern "C" {

int pt_abi_version(void) { return PT_ABI_VERSION; }

pt_status pt_scene_query(const pt_scene* s, int32_t key, int64_t* value) {
    return guarded([&] {
        if (!s || !value) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        switch (key) {
            case PT_Q_PIPELINES:  // -1 when a replica (pt_init(n > 1)) differs from the primary
                *value = s->pipes;
                for (auto& r : s->replicas) if (r->pipes != s->pipes) *value = -1;
                break;
            case PT_Q_BATCH_SLOTS:
                *value = (int64_t)s->target_slots;
                for (auto& r : s->replicas) if (r->target_slots != s->target_slots) *value = -1;
                break;
            case PT_Q_TRACE_LDS_BYTES: *value = (int64_t)s->lds_scene_bytes; break;
            case PT_Q_TRACE_SPILL: *value = s->trace_spill; break;
            case PT_Q_FEATURES: *value = s->features; break;
            case PT_Q_TRACE_KERNEL: *value = trace_kernel_id(s); break;
            case PT_Q_SHADE_KERNEL: *value = shade_kernel_id(s); break;
            default: throw PtError(PT_ERR_INVALID_ARG, "unknown pt_scene_query key");
        }
    });
}
const char* pt_last_error(void) { return g_last_error.c_str(); }

pt_status pt_load_pbrt(const char* path, pt_host_scene** out) {
    return guarded([&] {
        if (!path || !out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        *out = (pt_host_scene*)load_pbrt_file(path);
    });
}
const pt_scene_desc* pt_host_scene_desc(const pt_host_scene* hs) {
    return hs ? host_scene_desc((const pt_host_scene_impl*)hs) : nullptr;
}
const char* pt_host_scene_film_filename(const pt_host_scene* hs) {
    return hs ? host_scene_film_filename((const pt_host_scene_impl*)hs) : nullptr;
}
void pt_host_scene_free(pt_host_scene* hs) {
    if (hs) host_scene_free((pt_host_scene_impl*)hs);
}

pt_status pt_init(int device_count, const int32_t* device_ids) {
    return guarded([&] {
        require_device();
        int n = 0;
        HIPCHK(hipGetDeviceCount(&n));
        if (device_count < 1) throw PtError(PT_ERR_INVALID_ARG, "device_count must be >= 1");
        std::vector<int> ids((size_t)device_count);
        for (int k = 0; k < device_count; ++k) {
            ids[k] = device_ids ? device_ids[k] : k;
            if (ids[k] < 0 || ids[k] >= n) throw PtError(PT_ERR_INVALID_ARG, "device id out of range");
        }
        HIPCHK(hipSetDevice(ids[0]));
        std::lock_guard<std::mutex> lk(g_devices_mu);
        g_devices = ids;
    });
}

pt_status pt_shutdown(void) {
    return guarded([&] {
        std::lock_guard<std::mutex> lk(g_devices_mu);
        g_devices.clear();
    });
}

pt_status pt_comm_unique_id(uint8_t* id_out) {
    return guarded([&] {
        if (!id_out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        static_assert(sizeof(ncclUniqueId) == PT_COMM_ID_BYTES, "ncclUniqueId size");
        ncclUniqueId id;
        NCCLCHK(ncclGetUniqueId(&id));
        std::memcpy(id_out, &id, sizeof id);
    });
}

pt_status pt_comm_create(int nranks, int rank, const uint8_t* id, pt_comm** out) {
    return guarded([&] {
        if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) throw PtError(PT_ERR_INVALID_ARG, "bad argument");
        require_device();
        std::unique_ptr<pt_comm> c(new pt_comm);
        HIPCHK(hipGetDevice(&c->device));
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        NCCLCHK(ncclCommInitRank(&c->comm, nranks, uid, rank));
        c->nranks = nranks;
        c->rank = rank;
        *out = c.release();
    });
}

void pt_comm_destroy(pt_comm* comm) { delete comm; }

pt_status pt_film_reduce(pt_comm* comm, const pt_scene* s, float* d_accum, int root, void* stream) {
    return guarded([&] {
        if (!comm || !s || !d_accum || root < 0 || root >= comm->nranks) throw PtError(PT_ERR_INVALID_ARG, "bad argument");
        const size_t n = 4 * (size_t)s->fr.width() * s->fr.height();
        NCCLCHK(ncclReduce(d_accum, d_accum, n, ncclFloat, ncclSum, root, comm->comm, (hipStream_t)stream));
    });
}

pt_status pt_render_frame_dist(pt_scene* s, pt_comm* comm, float* d_accum, void* stream, pt_stats* stats) {
    return guarded([&] {
        if (!s || !comm || !d_accum) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        const size_t np = (size_t)s->fr.width() * s->fr.height();
        HIPCHK(hipMemsetAsync(d_accum, 0, np * sizeof(float4), (hipStream_t)stream));
        RenderResult r = render_tiles(s, comm->rank, comm->nranks, 0, s->spp, (float4*)d_accum, (hipStream_t)stream);
        // the frame's one collective, bracketed by events on its stream: reduce_ms is this rank's wait for
        // the slowest rank plus the transfer, the figure that tells tail imbalance from reduce cost
        if (!comm->ev0) HIPCHK(hipEventCreate(&comm->ev0));
        if (!comm->ev1) HIPCHK(hipEventCreate(&comm->ev1));
        HIPCHK(hipEventRecord(comm->ev0, (hipStream_t)stream));
        NCCLCHK(ncclReduce(d_accum, d_accum, 4 * np, ncclFloat, ncclSum, 0, comm->comm, (hipStream_t)stream));
        HIPCHK(hipEventRecord(comm->ev1, (hipStream_t)stream));
        HIPCHK(hipEventSynchronize(comm->ev1));  // returns after the reduce (pt.h)
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, comm->ev0, comm->ev1));
        fill_stats(r, stats);
        if (stats) stats->reduce_ms = ms;
    });
}

pt_status pt_scene_create(const pt_scene_desc* desc, pt_scene** out) {
    return guarded([&] {
        if (!out) throw PtError(PT_ERR_INVALID_ARG, "null out");
        require_device();
        std::vector<int> ids;
        {
            std::lock_guard<std::mutex> lk(g_devices_mu);
            ids = g_devices;
        }
        if (ids.empty()) {
            int d = 0;
            HIPCHK(hipGetDevice(&d));
            ids.push_back(d);
        }
        std::unique_ptr<pt_scene> s = create_scene_on(ids[0], desc, nullptr);
        for (size_t k = 1; k < ids.size(); ++k) s->replicas.push_back(create_scene_on(ids[k], desc, s.get()));
        HIPCHK(hipSetDevice(ids[0]));
        s->devices = ids;
        *out = s.release();
    });
}

void pt_scene_destroy(pt_scene* scene) { delete scene; }

pt_status pt_scene_bvh(const pt_scene* s, int32_t* n_nodes, void* nodes32, int32_t* n_prims, int32_t* prim_order) {
    return guarded([&] {
        if (!s) throw PtError(PT_ERR_INVALID_ARG, "null scene");
        if (n_nodes) *n_nodes = (int32_t)s->host_nodes.size();
        if (n_prims) *n_prims = (int32_t)s->host_prim_order.size();
        if (nodes32) std::memcpy(nodes32, s->host_nodes.data(), s->host_nodes.size() * sizeof(LinearNode));
        if (prim_order)
            for (size_t i = 0; i < s->host_prim_order.size(); ++i) prim_order[i] = s->host_prim_order[i];
    });
}

pt_status pt_build_bvh_host(const pt_scene_desc* d, int32_t* n_nodes, void* nodes32, int32_t node_cap,
                            int32_t* n_prims, int32_t* prim_order, int32_t prim_cap) {
    return guarded([&] {
        if (!d || !n_nodes) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        std::vector<LinearNode> nodes;
        std::vector<int> order;
        build_bvh(d, &nodes, &order);
        *n_nodes = (int32_t)nodes.size();
        if (n_prims) *n_prims = (int32_t)order.size();
        if (nodes32) {
            if ((int64_t)nodes.size() > node_cap) throw PtError(PT_ERR_INVALID_ARG, "node buffer too small");
            std::memcpy(nodes32, nodes.data(), nodes.size() * sizeof(LinearNode));
        }
        if (prim_order) {
            if ((int64_t)order.size() > prim_cap) throw PtError(PT_ERR_INVALID_ARG, "prim order buffer too small");
            for (size_t i = 0; i < order.size(); ++i) prim_order[i] = order[i];
        }
    });
}

pt_status pt_film_size(const pt_scene* s, int32_t* w, int32_t* h) {
    return guarded([&] {
        if (!s) throw PtError(PT_ERR_INVALID_ARG, "null scene");
        if (w) *w = s->fr.width();
        if (h) *h = s->fr.height();
    });
}

pt_status pt_render_tiles(pt_scene* s, int tile_offset, int tile_stride, float* d_accum, void* stream,
                          pt_stats* stats) {
    return guarded([&] {
        if (!s || !d_accum) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        RenderResult r = render_tiles(s, tile_offset, tile_stride, 0, s->spp, (float4*)d_accum, (hipStream_t)stream);
        fill_stats(r, stats);
    });
}

pt_status pt_render_range(pt_scene* s, int tile_offset, int tile_stride, int sample_begin, int sample_end,
                          float* d_accum, void* stream, pt_stats* stats) {
    return guarded([&] {
        if (!s || !d_accum) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        RenderResult r = render_tiles(s, tile_offset, tile_stride, sample_begin, sample_end, (float4*)d_accum,
                                      (hipStream_t)stream);
        fill_stats(r, stats);
    });
}

static void render_to_host(pt_scene* s, int tile_offset, int tile_stride, int s_begin, int s_end, float* accum_out,
                           pt_stats* stats) {
    size_t np = (size_t)s->fr.width() * s->fr.height();
    DBuf<float4> acc;
    acc.alloc(np);
    HIPCHK(hipMemset(acc.p, 0, np * sizeof(float4)));
    RenderResult r = render_tiles(s, tile_offset, tile_stride, s_begin, s_end, acc.p, nullptr);
    HIPCHK(hipMemcpy(accum_out, acc.p, np * sizeof(float4), hipMemcpyDeviceToHost));
    fill_stats(r, stats);
}

pt_status pt_render_accum(pt_scene* s, int tile_offset, int tile_stride, float* accum_out, pt_stats* stats) {
    return guarded([&] {
        if (!s || !accum_out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        render_to_host(s, tile_offset, tile_stride, 0, s->spp, accum_out, stats);
    });
}

pt_status pt_render_range_accum(pt_scene* s, int tile_offset, int tile_stride, int sample_begin, int sample_end,
                                float* accum_out, pt_stats* stats) {
    return guarded([&] {
        if (!s || !accum_out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        render_to_host(s, tile_offset, tile_stride, sample_begin, sample_end, accum_out, stats);
    });
}

pt_status pt_resolve_film(const pt_scene* s, const float* accum, float* rgb_out) {
    return guarded([&] {
        if (!s || !accum || !rgb_out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        resolve(s, accum, rgb_out);
    });
}

pt_status pt_resolve_film_host(const pt_scene_desc* d, const float* accum, float* rgb_out) {
    return guarded([&] {
        if (!d || !accum || !rgb_out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        int w = 0, h = 0;
        crop_size(d->film, &w, &h);
        resolve_film((size_t)w * h, d->film.scale, accum, rgb_out);
    });
}

pt_status pt_film_size_host(const pt_scene_desc* d, int32_t* w, int32_t* h) {
    return guarded([&] {
        if (!d) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        int ww = 0, hh = 0;
        crop_size(d->film, &ww, &hh);
        if (w) *w = ww;
        if (h) *h = hh;
    });
}

pt_status pt_render(pt_scene* s, float* rgb_out, pt_stats* stats) {
    return guarded([&] {
        if (!s || !rgb_out) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        size_t np = (size_t)s->fr.width() * s->fr.height();
        HIPCHK(hipSetDevice(s->device));
        DBuf<float4> acc;
        acc.alloc(np);
        HIPCHK(hipMemset(acc.p, 0, np * sizeof(float4)));
        RenderResult r = s->replicas.empty() ? render_tiles(s, 0, 1, 0, s->spp, acc.p, nullptr)
                                             : render_all_devices(s, acc.p);
        std::vector<float> h(4 * np);
        HIPCHK(hipMemcpy(h.data(), acc.p, np * sizeof(float4), hipMemcpyDeviceToHost));
        resolve(s, h.data(), rgb_out);
        fill_stats(r, stats);
    });
}

pt_status pt_set_batch_slots(pt_scene* s, int64_t slots) {
    return guarded([&] {
        if (!s || slots <= 0) throw PtError(PT_ERR_INVALID_ARG, "bad argument");
        // every replica (pt_init(n > 1)) gets the same batch size, checked against its own limit
        if ((uint64_t)slots > slot_limit(s))
            throw PtError(PT_ERR_INVALID_ARG, "batch slots exceed the 32-bit path-state indexing limit (" +
                                                  std::to_string(slot_limit(s)) + ")");
        for (auto& r : s->replicas)
            if ((uint64_t)slots > slot_limit(r.get()))
                throw PtError(PT_ERR_INVALID_ARG, "batch slots exceed a replica's path-state indexing limit");
        s->target_slots = (size_t)slots;
        for (auto& r : s->replicas) r->target_slots = (size_t)slots;
    });
}

pt_status pt_set_count_bytes(pt_scene* s, int32_t on) {
    return guarded([&] {
        if (!s) throw PtError(PT_ERR_INVALID_ARG, "null scene");
        s->count_bytes = on != 0;
        for (auto& r : s->replicas) r->count_bytes = on != 0;
    });
}

pt_status pt_set_pipelines(pt_scene* s, int32_t pipelines) {
    return guarded([&] {
        if (!s || pipelines < 1 || pipelines > kMaxPipes) throw PtError(PT_ERR_INVALID_ARG, "pipelines must be in [1, 4]");
        s->pipes = pipelines;
        for (auto& r : s->replicas) r->pipes = pipelines;
    });
}

pt_status pt_write_pfm(const char* path, const float* rgb, int32_t width, int32_t height) {
    return guarded([&] {
        if (!path || !rgb || width <= 0 || height <= 0) throw PtError(PT_ERR_INVALID_ARG, "bad argument");
        write_pfm(path, rgb, width, height);
    });
}

pt_status pt_write_image(const char* path, const float* rgb, int32_t width, int32_t height, int32_t full_xres,
                         int32_t full_yres, int32_t x0, int32_t y0) {
    return guarded([&] {
        if (!path || !rgb || width <= 0 || height <= 0 || x0 < 0 || y0 < 0 || x0 + width > full_xres ||
            y0 + height > full_yres)
            throw PtError(PT_ERR_INVALID_ARG, "pt_write_image: bad bounds");
        write_image(path, rgb, width, height, full_xres, full_yres, x0, y0);
    });
}
pt_status pt_write_film_image(const pt_scene_desc* d, const char* path, const float* rgb) {
    return guarded([&] {
        if (!d || !path || !rgb) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        const pt_film_desc& f = d->film;
        const int x0 = (int)std::ceil((float)f.xres * f.crop[0]), x1 = (int)std::ceil((float)f.xres * f.crop[1]);
        const int y0 = (int)std::ceil((float)f.yres * f.crop[2]), y1 = (int)std::ceil((float)f.yres * f.crop[3]);
        if (x1 <= x0 || y1 <= y0) throw PtError(PT_ERR_INVALID_ARG, "empty film crop");
        write_image(path, rgb, x1 - x0, y1 - y0, f.xres, f.yres, x0, y0);
    });
}

// ---- test hooks ----
pt_status pt_debug_libm_trig(int n, const float* x, float* sin_out, float* cos_out) {
    return guarded([&] {
        for (int i = 0; i < n; ++i) {
            sin_out[i] = libm_sinf(x[i]);
            cos_out[i] = libm_cosf(x[i]);
        }
    });
}
pt_status pt_debug_spectrum(int kind, int n, const float* vals, float* out) {
    return guarded([&] {
        if (!vals || !out || n < 0) throw PtError(PT_ERR_INVALID_ARG, "pt_debug_spectrum: bad arguments");
        if (kind == 0) {
            std::vector<float> wl(n), v(n);
            for (int i = 0; i < n; ++i) wl[i] = vals[2 * i], v[i] = vals[2 * i + 1];
            rgb_from_sampled(wl.data(), v.data(), n, out);
        } else if (kind == 1) {
            rgb_from_blackbody(vals[0], vals[1], out);
        } else if (kind == 2) {
            xyz_to_rgb(vals, out);
        } else if (kind == 3) {
            for (int i = 0; i < n; ++i) blackbody_radiance(&vals[2 * i], 1, vals[2 * i + 1], &out[i]);
        } else {
            throw PtError(PT_ERR_INVALID_ARG, "pt_debug_spectrum: unknown kind");
        }
    });
}
pt_status pt_debug_halton(pt_scene* s, int n, const uint32_t* idx, const int32_t* dims, float* out) {
    return guarded([&] {
        DBuf<uint32_t> di; DBuf<int> dd; DBuf<float> o;
        di.upload(idx, (size_t)n); dd.upload(dims, (size_t)n); o.alloc((size_t)n);
        hipLaunchKernelGGL(k_debug_halton, dim3(ceil_div(n, 256)), dim3(256), (size_t)s->dev.hal_lds_bytes, 0, s->dev,
                           di.p, dd.p, n, o.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpy(out, o.p, sizeof(float) * n, hipMemcpyDeviceToHost));
    });
}
pt_status pt_debug_pixel_offsets(pt_scene* s, int n, const int32_t* pixxy, uint32_t* out) {
    return guarded([&] {
        DBuf<int2> dp; DBuf<uint32_t> o;
        dp.upload((const int2*)pixxy, (size_t)n); o.alloc((size_t)n);
        hipLaunchKernelGGL(k_debug_pixel_offset, dim3(ceil_div(n, 256)), dim3(256), 0, 0, s->dev, s->hpc, dp.p, n, o.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpy(out, o.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    });
}
pt_status pt_debug_camera_rays(pt_scene* s, int n, const float* film_xy, float* out6) {
    return guarded([&] {
        DBuf<float> df, o;
        df.upload(film_xy, (size_t)2 * n); o.alloc((size_t)6 * n);
        hipLaunchKernelGGL(k_debug_camera, dim3(ceil_div(n, 256)), dim3(256), 0, 0, s->dev, df.p, n, o.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpy(out6, o.p, sizeof(float) * 6 * n, hipMemcpyDeviceToHost));
    });
}
pt_status pt_debug_trace(pt_scene* s, int n, const float* rays7, int any, int32_t* out_prim) {
    return guarded([&] {
        DBuf<float> dr; DBuf<int> o, sp;
        dr.upload(rays7, (size_t)7 * n); o.alloc((size_t)n); sp.alloc((size_t)n * (64 - kStackLds));
        hipLaunchKernelGGL(k_debug_trace, dim3(ceil_div(n, kTraceBlock)), dim3(kTraceBlock), 0, 0, s->dev, dr.p, n,
                           any, sp.p, o.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpy(out_prim, o.p, sizeof(int) * n, hipMemcpyDeviceToHost));
    });
}

pt_status pt_debug_trace_frame(pt_scene* s, int n, const float* rays7, int any, int32_t* out_prim,
                               uint64_t* counters) {
    pt_stats st{};
    const pt_status r = pt_debug_trace_frame_ex(s, n, rays7, any, out_prim, &st);
    if (r == PT_OK && counters) {
        counters[0] = st.node_visits;
        counters[1] = st.prim_tests;
    }
    return r;
}

pt_status pt_debug_trace_frame_ex(pt_scene* s, int n, const float* rays7, int any, int32_t* out_prim,
                                  pt_stats* stats) {
    return guarded([&] {
        if (!s || n < 0 || (n && (!rays7 || !out_prim))) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        if (stats) *stats = pt_stats{};
        if (n == 0) return;
        HIPCHK(hipSetDevice(s->device));
        Work w;
        w.ensure((size_t)n, (size_t)s->num_cus * std::max(16, s->trace_bpc) * kTraceBlock, 0, 0);
        DevPaths ps = w.paths(n);
        // ray records (kernels.hip load_ray): {o.xyz, d.x} {d.yz, tMax, 0}
        std::vector<float> soa((size_t)8 * n, 0.f);
        std::vector<uint32_t> rq((size_t)n);
        for (int i = 0; i < n; ++i) {
            for (int c = 0; c < 7; ++c) soa[(size_t)8 * i + c] = rays7[7 * (size_t)i + c];
            rq[i] = ((uint32_t)i << 2) | (any ? kRayShadow : kRayCont);
        }
        HIPCHK(hipMemcpy(any ? w.rayA.p : w.ray.p, soa.data(), soa.size() * sizeof(float), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(w.rq0.p, rq.data(), rq.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemset(w.stats.p, 0, sizeof(DevStats)));
        HIPCHK(hipMemset(w.stats_rt.p, 0, sizeof(DevStats)));
        hipLaunchKernelGGL(k_set_counts, dim3(1), dim3(1), 0, 0, w.counts.p, (uint32_t)n, 0u);
        launch_trace(s, w, ps, w.rq0.p, w.counts.p, (uint32_t)n, 0);
        HIPCHK(hipGetLastError());
        HIPCHK(hipDeviceSynchronize());
        // the head's hit words (device.h): hit for closest-hit queries, hitA for any-hit ones
        HIPCHK(hipMemcpy(out_prim, (const int*)w.head.p + (size_t)(any ? kHdHitA : kHdHit) * n, sizeof(int32_t) * n,
                         hipMemcpyDeviceToHost));
        if (stats) {
            const DevStats d = read_stats(w);
            RenderResult rr;
            rr.st = d;
            rr.wide = s->wide_lds_bytes && !s->count_bytes;
            fill_stats(rr, stats);
        }
    });
}

pt_status pt_debug_bsdf(pt_scene* s, int material, int n, const float* in8, float* out8) {
    return guarded([&] {
        if (!s || n < 0 || (n && (!in8 || !out8))) throw PtError(PT_ERR_INVALID_ARG, "null argument");
        if (material < 0 || material >= (int)s->mats.n) throw PtError(PT_ERR_INVALID_ARG, "material out of range");
        if (n == 0) return;
        DBuf<float> di, dout;
        di.upload(in8, (size_t)8 * n);
        dout.alloc((size_t)8 * n);
        hipLaunchKernelGGL(k_debug_bsdf, dim3(ceil_div(n, 128)), dim3(128), 0, 0, s->dev, material, di.p, n, dout.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpy(out8, dout.p, sizeof(float) * 8 * n, hipMemcpyDeviceToHost));
    });
}

}  // extern "C"
