/*
 * pt.h -- C ABI of the MI355X-native wavefront path tracer.
 *
 * This is the drop-in boundary for the reference's SamplerIntegrator plugin
 * surface.  A pbrt-v3 build binds these symbols from a `GpuPathIntegrator`
 * registered in RenderOptions::MakeIntegrator:
 *
 *   reference interface                                     replaced by
 *   ------------------------------------------------------  -----------------------------
 *   Integrator::Render(const Scene&)                        pt_render / pt_render_tiles
 *     src/core/integrator.h:53-58, integrator.cpp:526-637
 *   PathIntegrator::Li(...)  src/integrators/path.cpp:64-189  (device wavefront, no host call)
 *   CreatePathIntegrator(ParamSet, Sampler, Camera)         pt_integrator_desc
 *     src/integrators/path.cpp:191-214
 *   CreateDirectLightingIntegrator                          pt_integrator_desc (kind DIRECT)
 *     src/integrators/directlighting.cpp:86-118
 *   CreateHaltonSampler  src/samplers/halton.cpp:133-139    pt_sampler_desc
 *   CreatePerspectiveCamera  src/cameras/perspective.cpp    pt_camera_desc
 *   CreateFilm / CreateBoxFilter / CreateGaussianFilter     pt_film_desc
 *     src/core/film.cpp:213-252, src/filters/{box,gaussian}.cpp
 *   Scene{aggregate, lights}  src/core/scene.h:50-80         pt_scene_desc + pt_scene_create
 *   CreateBVHAccelerator  src/accelerators/bvh.cpp:740-760   built inside pt_scene_create
 *   MakeShapes "trianglemesh"/"plymesh"/"loopsubdiv"/"sphere"/"aaplane"
 *     src/core/api.cpp:432-546                              pt_triangle / pt_sphere / pt_aaplane
 *   MakeAreaLight "diffuse"/"portal"  src/core/api.cpp:768-786      pt_light
 *   CreateAAPortal  src/lights/portal_arealight.cpp:245-300          pt_light + pt_portal
 *   pbrtParseFile  src/core/parser.cpp:1094                 pt_load_pbrt (host scene loader)
 *   Film::WriteImage  src/core/film.cpp:169-211              pt_write_pfm
 *
 * Conventions: plain pointers + sizes, no C++ types, no exceptions across the
 * boundary.  Every call returns pt_status; pt_last_error() gives a message.
 * All host arrays passed in are copied; the caller keeps ownership.  All
 * calls for one device come from one host thread.
 */
#ifndef PT_H
#define PT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 11

typedef enum pt_status {
    PT_OK = 0,
    PT_ERR_INVALID_ARG = 1,
    PT_ERR_PARSE = 2,
    PT_ERR_UNSUPPORTED = 3,
    PT_ERR_DEVICE = 4,
    PT_ERR_OOM = 5,
    PT_ERR_STATE = 6,
    PT_ERR_IO = 7
} pt_status;

/* ---- scene description (world space, the reference's post-parse Scene) ---- */

enum pt_prim_kind { PT_PRIM_TRIANGLE = 0, PT_PRIM_AAPLANE = 1, PT_PRIM_SPHERE = 2 };

enum pt_material_kind {
    PT_MAT_NONE = 0,   /* "" / "none": null BSDF, path passes through   */
    PT_MAT_MATTE = 1,  /* MatteMaterial  src/materials/matte.cpp:45-62 */
    PT_MAT_METAL = 2,  /* MetalMaterial  src/materials/metal.cpp:58-79 */
    PT_MAT_GLASS = 3,  /* GlassMaterial  src/materials/glass.cpp:45-83 */
    PT_MAT_DISPERSIVE_GLASS = 4, /* DispersiveGlassMaterial  src/materials/dispersive_glass.cpp:48-123 */
    PT_MAT_MIRROR = 5, /* MirrorMaterial  src/materials/mirror.cpp:44-52 */
    PT_MAT_PLASTIC = 6 /* PlasticMaterial  src/materials/plastic.cpp:45-70 */
};

enum pt_light_kind {
    PT_LIGHT_DIFFUSE_AREA = 0, /* DiffuseAreaLight on one triangle   src/lights/diffuse.cpp */
    PT_LIGHT_PORTAL_AREA = 1,  /* PortalArealight on one aaplane     src/lights/portal_arealight.cpp */
    PT_LIGHT_INFINITE = 2,     /* InfiniteAreaLight, constant L (no "mapname")  src/lights/infinite.cpp */
    PT_LIGHT_DIFFUSE_SPHERE = 3, /* DiffuseAreaLight on one sphere    src/lights/diffuse.cpp, shapes/sphere.cpp */
    PT_LIGHT_POINT = 4,         /* PointLight at LightToWorld(0,0,0), L = I * scale  src/lights/point.cpp */
    PT_LIGHT_DIFFUSE_PLANE = 5  /* DiffuseAreaLight on one aaplane (scenes/blender/creeper/out/creeper.pbrt:38-49):
                                   Shape::Sample(ref) / Shape::Pdf(ref, wi)  src/core/shape.cpp:56-91 over
                                   AAPlaneShape::Sample / Intersect  src/shapes/plane.cpp:15-72 */
};

/* Portals per PortalArealight.  The reference sizes its per-call portal
 * distribution as a VLA (portal_arealight.cpp:42); the loader and
 * pt_scene_create refuse more than this many with PT_ERR_UNSUPPORTED. */
#define PT_MAX_PORTALS 64

enum pt_portal_strategy {      /* PortalStrategy  src/lights/portal_arealight.h:12 */
    PT_PORTAL_LIGHT = 0,       /* "light"      SampleUniformLight */
    PT_PORTAL_UNIFORM = 1,     /* "portal"     SampleUniformPortal */
    PT_PORTAL_PROJECTION = 2   /* "projection" SampleProjection */
};

enum pt_filter_kind { PT_FILTER_BOX = 0, PT_FILTER_GAUSSIAN = 1 };

enum pt_light_sample_strategy { PT_LIGHTS_UNIFORM = 0, PT_LIGHTS_POWER = 1,
                                PT_LIGHTS_SPATIAL = 2 /* SpatialLightDistribution, lightdistrib.cpp:80-330 */ };

enum pt_integrator_kind {
    PT_INTEGRATOR_PATH = 0,    /* PathIntegrator            src/integrators/path.cpp */
    PT_INTEGRATOR_DIRECT = 1,  /* DirectLightingIntegrator  src/integrators/directlighting.cpp */
    PT_INTEGRATOR_HERO_PATH = 2,     /* HeroPathIntegrator (60-bin SampledSpectrum)  src/integrators/hero_path.cpp */
    PT_INTEGRATOR_HERO_PATH_MIS = 3  /* HeroPathMISIntegrator                        src/integrators/hero_path_mis.cpp */
};
enum pt_direct_strategy {      /* LightStrategy  src/integrators/directlighting.h */
    PT_DIRECT_ALL = 0,         /* "all": UniformSampleAllLights with per-light sample arrays */
    PT_DIRECT_ONE = 1          /* "one": UniformSampleOneLight (uniform choice) */
};

/* Transform (src/core/transform.h): m and its stored inverse mInv, row-major. */
typedef struct pt_transform {
    float m[16];
    float minv[16];
} pt_transform;

/* Flags on a triangle (bit set). */
#define PT_TRI_REVERSE_ORIENTATION 1u  /* Shape::reverseOrientation */
#define PT_TRI_SWAPS_HANDEDNESS 2u     /* Shape::transformSwapsHandedness */
#define PT_TRI_HAS_N 4u                /* TriangleMesh::n present */
#define PT_TRI_HAS_UV 8u               /* TriangleMesh::uv present */
#define PT_TRI_HAS_S 16u               /* TriangleMesh::s present */

/* One Triangle shape (src/shapes/triangle.h); vertices are already in world
 * space (TriangleMesh ctor, triangle.cpp:75). */
typedef struct pt_triangle {
    int32_t v[3];        /* indices into pt_scene_desc vertex arrays */
    int32_t material;    /* index into materials */
    int32_t area_light;  /* index into lights, or -1 */
    uint32_t flags;      /* PT_TRI_* */
} pt_triangle;

/* AAPlaneShape (src/shapes/plane.h:12-70). lo/hi are object space. */
typedef struct pt_aaplane {
    float lo[3];
    float hi[3];
    int32_t axis;
    int32_t material;
    int32_t area_light;
    uint32_t flags;                /* PT_TRI_REVERSE_ORIENTATION | PT_TRI_SWAPS_HANDEDNESS */
    pt_transform object_to_world;  /* m = ObjectToWorld, minv = WorldToObject */
} pt_aaplane;

/* Sphere (src/shapes/sphere.{h,cpp}); parameters as given to
 * CreateSphereShape (radius, zmin, zmax, phimax in degrees); the renderer
 * derives the clamped Sphere members (sphere.h:50-59). */
typedef struct pt_sphere {
    float radius;
    float zmin, zmax;
    float phimax;
    int32_t material;
    int32_t area_light;
    uint32_t flags;                /* PT_TRI_REVERSE_ORIENTATION | PT_TRI_SWAPS_HANDEDNESS */
    pt_transform object_to_world;  /* m = ObjectToWorld, minv = WorldToObject */
} pt_sphere;

/* Primitive in scene order (RenderOptions::primitives, api.cpp:1431-1433). */
typedef struct pt_prim {
    int32_t kind;   /* pt_prim_kind */
    int32_t index;  /* into triangles, planes or spheres */
} pt_prim;

typedef struct pt_material {
    int32_t kind;    /* pt_material_kind */
    float kd[3];     /* matte: constant Kd (Clamp() is applied by the renderer) */
    float sigma;     /* matte: OrenNayar sigma in degrees; only 0 supported */
    float eta[3];    /* metal: constant eta */
    float k[3];      /* metal: constant k */
    float alpha[2];  /* metal / plastic / rough glass: TrowbridgeReitz alphax, alphay
                        (after RoughnessToAlpha when remaproughness, and the 0.001
                        floor of the ctor) */
    float ks[3];     /* plastic: constant Ks */
    float kr[3];     /* glass / dispersive / mirror: constant Kr */
    float kt[3];     /* glass / dispersive: constant Kt */
    float ior;       /* glass: "eta" / "index" */
    float ior_min;   /* dispersive: "etaMin" / "indexMin" */
    float ior_max;   /* dispersive: "etaMax" / "indexMax" */
    int32_t specular;/* glass / dispersive: uroughness == 0 && vroughness == 0 */
} pt_material;

/* AAPortal (src/portals/aaportal.h) as parsed from portalData. */
typedef struct pt_portal {
    float lo[3];
    float hi[3];
    int32_t axis;
    int32_t facing_fw;
} pt_portal;

typedef struct pt_light {
    int32_t kind;         /* pt_light_kind */
    float L[3];           /* Lemit = L * scale */
    int32_t two_sided;
    int32_t shape;        /* triangle (diffuse), plane (portal) or sphere (diffuse sphere) index */
    int32_t strategy;     /* pt_portal_strategy (portal lights) */
    int32_t first_portal; /* into portals */
    int32_t n_portals;
    int32_t n_samples;    /* Light::nSamples ("nsamples"/"samples", >= 1) */
    pt_transform light_to_world; /* infinite: LightToWorld (CTM at the LightSource);
                                    point: Translate(from) * LightToWorld */
} pt_light;

typedef struct pt_camera_desc {
    pt_transform camera_to_world;  /* RenderOptions::CameraToWorld */
    float fov;
    float screen_window[4];        /* xmin, xmax, ymin, ymax */
    float lens_radius;
    float focal_distance;
    float shutter_open;
    float shutter_close;
} pt_camera_desc;

typedef struct pt_film_desc {
    int32_t xres, yres;
    float crop[4];                 /* xmin, xmax, ymin, ymax in [0,1] */
    int32_t filter;                /* pt_filter_kind */
    float filter_radius[2];
    float gaussian_alpha;
    float scale;
    float max_sample_luminance;
    float diagonal;
} pt_film_desc;

typedef struct pt_sampler_desc {
    int32_t spp;
    int32_t sample_pixel_center;
} pt_sampler_desc;

typedef struct pt_integrator_desc {
    int32_t max_depth;
    float rr_threshold;
    int32_t light_strategy;        /* pt_light_sample_strategy */
    int32_t has_pixel_bounds;
    int32_t pixel_bounds[4];       /* x0, x1, y0, y1 as in the "pixelbounds" param */
    int32_t kind;                  /* pt_integrator_kind */
    int32_t direct_strategy;       /* pt_direct_strategy (kind == PT_INTEGRATOR_DIRECT) */
} pt_integrator_desc;

typedef struct pt_scene_desc {
    int32_t n_vertices;
    const float* P;     /* 3*n_vertices, world space */
    const float* N;     /* 3*n_vertices or NULL */
    const float* S;     /* 3*n_vertices or NULL */
    const float* UV;    /* 2*n_vertices or NULL */
    int32_t n_triangles;
    const pt_triangle* triangles;
    int32_t n_planes;
    const pt_aaplane* planes;
    int32_t n_prims;
    const pt_prim* prims;
    int32_t n_materials;
    const pt_material* materials;
    int32_t n_lights;
    const pt_light* lights;
    int32_t n_portals;
    const pt_portal* portals;
    int32_t bvh_max_prims;          /* "maxnodeprims", default 4 */
    pt_camera_desc camera;
    pt_film_desc film;
    pt_sampler_desc sampler;
    pt_integrator_desc integrator;
    int32_t n_spheres;
    const pt_sphere* spheres;
    /* SampledSpectrum scenes (spectral = 1: the hero integrators, which the
     * reference runs in its PBRT_SAMPLED_SPECTRUM build; 60 bins over
     * 400-700 nm, spectrum.h:48-51).  NULL / 0 for RGB scenes. */
    int32_t spectral;
    const float* material_s60; /* n_materials x 3 x 60: matte Kd | -, glass / dispersive_glass -, Kr, Kt; mirror -, Kr */
    const float* light_s60;    /* n_lights x 60: area lights' Lemit = L * scale (infinite lights use their RGB L) */
    /* Optional prebuilt BVH: the reference's flattened BVHAccel::nodes
     * (32-byte LinearBVHNode records, bvh.cpp:95-104).  When bvh_nodes is
     * non-NULL, prims[] are in the BVH's primitive order
     * (BVHAccel::primitives) and pt_scene_create builds no BVH of its own;
     * NULL / 0: the SAH build of bvh.cpp:236-402 runs on prims[] in scene order. */
    int32_t n_bvh_nodes;
    const void* bvh_nodes;
} pt_scene_desc;

/* ---- statistics (reference counters, src/core/scene.cpp:40-42 etc.) ---- */
typedef struct pt_stats {
    uint64_t camera_rays;      /* "Integrator/Camera rays traced" */
    uint64_t closest_rays;     /* "Regular ray intersection tests" */
    uint64_t shadow_rays;      /* "Shadow ray intersection tests" */
    uint64_t node_visits;      /* BVH nodes whose bounds were tested */
    uint64_t prim_tests;       /* leaf primitive intersection tests */
    uint64_t samples;          /* camera samples rendered */
    double render_ms;          /* device wall time of the render (events) */
    double trace_ms;           /* summed duration of the trace kernel (HIP events on the launch stream) */
    uint64_t trace_launches;
    double shade_ms;           /* summed duration of the shading kernel */
    uint64_t shade_launches;
    uint64_t shade_bytes;      /* algorithmic path-state bytes the shading kernel moved: path / mypath
                                  integrators only with pt_set_count_bytes on (0 otherwise); the
                                  hero_path / hero_path_mis shading kernels always count (a 2-wave
                                  build either way: the counter register costs them no occupancy) */
    double reduce_ms;          /* pt_render_frame_dist: the ncclReduce of the film (HIP events on the stream) */
    /* ABI 11: the 4-wide traversal (k_trace_w, LDS-resident scenes without spheres).  It returns the
       reference's hits but not its visit order, so with trace_wide set node_visits / prim_tests count only
       the rays it handed back to the binary traversal (retraced_rays: near ties within 2^-15 of the closest
       t, hits at t <= 0, directions with a zero component); the reference's counters come from a render with
       pt_set_count_bytes on, which traverses in the reference's order throughout. */
    uint64_t retraced_rays;
    uint64_t wide_node_visits; /* 4-wide node visits (112 B each) */
    uint64_t wide_prim_tests;  /* primitive tests of the wide traversal */
    int32_t trace_wide;        /* 1: this render traversed with k_trace_w */
    int32_t reserved;
} pt_stats;

/* ---- host scene loader (.pbrt subset) ---- */
typedef struct pt_host_scene pt_host_scene;

pt_status pt_load_pbrt(const char* path, pt_host_scene** out);
const pt_scene_desc* pt_host_scene_desc(const pt_host_scene* hs);
void pt_host_scene_free(pt_host_scene* hs);

/* ---- device scene + render ---- */
typedef struct pt_scene pt_scene;

int pt_abi_version(void);
const char* pt_last_error(void);

/* The devices this process renders on: device_ids[0..count)
 * (NULL: 0..count-1).  Scenes created afterwards hold one replica per device
 * (the BVH is built once on the host) and pt_render deals the 16x16 tiles
 * round-robin over them, one host thread per device (the reference's
 * ParallelFor2D over tiles, integrator.cpp:533-538), summing the device films
 * on device_ids[0] in device order (Film::MergeFilmTile, film.cpp:117-130).
 * count 1 is the single-device path; without pt_init the calling thread's
 * current HIP device is used. */
pt_status pt_init(int device_count, const int32_t* device_ids);
/* Forget the device list (scenes keep their devices until destroyed). */
pt_status pt_shutdown(void);

/* Build the SAH BVH on the host (BVHAccel, bvh.cpp:236-402) and upload the
 * flattened scene to device memory. */
pt_status pt_scene_create(const pt_scene_desc* desc, pt_scene** out);
void pt_scene_destroy(pt_scene* scene);

/* Read back the flattened BVH (32-byte LinearBVHNode records, bvh.cpp:95-104)
 * and the primitive order, for parity tests.  Pass NULL to query counts. */
pt_status pt_scene_bvh(const pt_scene* scene, int32_t* n_nodes, void* nodes32,
                       int32_t* n_prims, int32_t* prim_order);

/* Host-only BVH build (no device needed): same nodes as pt_scene_bvh.
 * n_nodes / n_prims receive the counts (pass NULL buffers to query them);
 * a buffer smaller than its count (node_cap nodes, prim_cap entries) is
 * PT_ERR_INVALID_ARG. */
pt_status pt_build_bvh_host(const pt_scene_desc* desc, int32_t* n_nodes, void* nodes32, int32_t node_cap,
                            int32_t* n_prims, int32_t* prim_order, int32_t prim_cap);

/* Render the whole sample-bound region serially on this device and write the
 * final RGB image (croppedPixelBounds, 3 floats per pixel, WriteImage
 * semantics) to rgb_out.  stats may be NULL. */
pt_status pt_render(pt_scene* scene, float* rgb_out, pt_stats* stats);

/* Multi-GPU building block: render the 16x16 image tiles t with
 * t % tile_stride == tile_offset into a device-resident accumulation buffer
 * (4 floats per cropped pixel: Film::Pixel's xyz[3] + filterWeightSum
 * (film.h:98-105), zeroed by the caller), on `stream` (hipStream_t, may be
 * NULL).  Each tile's FilmTile partial sum is formed in the reference's
 * order and merged in tile order (film.cpp:117-130), so buffers from
 * disjoint tile sets or sample ranges combine by plain addition.  Returns
 * when the work is done (the call synchronises `stream`). */
pt_status pt_render_tiles(pt_scene* scene, int tile_offset, int tile_stride,
                          float* d_accum, void* stream, pt_stats* stats);

/* Same as pt_render_tiles for camera-sample indices [sample_begin,
 * sample_end) of every pixel (the Halton sequence continues past the scene's
 * spp), so N ranks can each render a disjoint sample range of one frame. */
pt_status pt_render_range(pt_scene* scene, int tile_offset, int tile_stride,
                          int sample_begin, int sample_end, float* d_accum,
                          void* stream, pt_stats* stats);

/* ---- multi-process (one process per GPU): RCCL over xGMI ----
 * Rank 0 calls pt_comm_unique_id and hands the PT_COMM_ID_BYTES to every rank
 * (any launcher channel); each rank selects its GPU (pt_init(1, &id)) and calls
 * pt_comm_create.  pt_render_frame_dist renders the tiles t % nranks == rank
 * into d_accum (zeroed by the call) on `stream` and sums the films onto rank 0
 * with one ncclReduce -- the frame's only collective.  It returns after that
 * reduce has completed on `stream` (the host waits for it: stats->reduce_ms is
 * read back from events around it). */
#define PT_COMM_ID_BYTES 128
typedef struct pt_comm pt_comm;
pt_status pt_comm_unique_id(uint8_t* id_out);
pt_status pt_comm_create(int nranks, int rank, const uint8_t* id, pt_comm** out);
void pt_comm_destroy(pt_comm* comm);
/* ncclReduce(sum) of a device film (4 floats per cropped pixel) to `root`. */
pt_status pt_film_reduce(pt_comm* comm, const pt_scene* scene, float* d_accum, int root, void* stream);
pt_status pt_render_frame_dist(pt_scene* scene, pt_comm* comm, float* d_accum, void* stream, pt_stats* stats);

/* Resolve an accumulation buffer (host memory, 4 floats per pixel: XYZ sum +
 * weight sum) into the final RGB image exactly as Film::WriteImage does
 * (film.cpp:169-211). */
pt_status pt_resolve_film(const pt_scene* scene, const float* accum, float* rgb_out);

/* Host-only variants (no device needed): resolve an accumulation buffer
 * with the film parameters of a scene description, and its cropped size.
 * Used by rank 0 after the cross-rank reduce and by CPU tests. */
pt_status pt_resolve_film_host(const pt_scene_desc* desc, const float* accum, float* rgb_out);
pt_status pt_film_size_host(const pt_scene_desc* desc, int32_t* width, int32_t* height);

/* Same as pt_render_tiles but synchronous, into a host buffer (4 floats per
 * cropped pixel, zero-initialised by the call). */
pt_status pt_render_accum(pt_scene* scene, int tile_offset, int tile_stride,
                          float* accum_out, pt_stats* stats);

/* Same as pt_render_range but synchronous, into a host buffer. */
pt_status pt_render_range_accum(pt_scene* scene, int tile_offset, int tile_stride,
                                int sample_begin, int sample_end, float* accum_out,
                                pt_stats* stats);

/* Number of in-flight paths per wavefront batch (default 96M; 32M for the
 * hero integrators).  Memory for path state is ~230 bytes per slot (~1.2 KB
 * for the hero integrators).  Batches beyond the 32-bit path-state indexing
 * limit (~252M slots; ~70M for hero scenes) are PT_ERR_INVALID_ARG. */
pt_status pt_set_batch_slots(pt_scene* scene, int64_t slots);

/* Batches in flight (default 2 for scenes whose BVH fits LDS, 1 for BVHs
 * traversed from HBM): each pipeline is a host thread, a stream and its own
 * path-state buffers; one batch's trace kernel overlaps another's shading.
 * 1 runs the batches one after the other (isolated kernel timings). */
pt_status pt_set_pipelines(pt_scene* scene, int32_t pipelines);
/* Count the shading kernel's algorithmic path-state bytes (pt_stats.shade_bytes)
 * in the renders that follow (default off: the count costs the 3-waves-per-SIMD
 * shading build a register, so it runs a separate instantiation).  Applies to
 * the path / mypath integrators; the hero integrators always count.  It is the
 * counting frame's switch as a whole: with it on, every traversal runs the
 * binary kernels in the reference's visit order (no k_trace_w), so the render's
 * node_visits / prim_tests are the reference's counters. */
pt_status pt_set_count_bytes(pt_scene* scene, int32_t on);

/* Read back a setting of a device scene (what the environment overrides and
 * the pt_set_* calls left in effect), so callers can restore or report it.
 * PIPELINES / BATCH_SLOTS read -1 when the scene's replicas (pt_init(n > 1))
 * do not all carry the primary's value. */
enum pt_scene_key {
    PT_Q_PIPELINES = 0,        /* pt_set_pipelines value (PT_PIPES) */
    PT_Q_BATCH_SLOTS = 1,      /* pt_set_batch_slots value (0 = the default) */
    PT_Q_TRACE_LDS_BYTES = 2,  /* bytes of BVH + primitives the trace kernel stages in LDS (0 = reads HBM) */
    PT_Q_TRACE_SPILL = 3,      /* 1 when traversal stacks spill past the LDS rows (deep BVHs) */
    PT_Q_FEATURES = 4,         /* scene-feature set the shading kernel is instantiated for */
    PT_Q_TRACE_KERNEL = 5,     /* traversal kernel of a render: 0 k_trace, 1 k_trace_pt, 2 k_trace_nb, 3 k_trace_lds,
                                  5 k_trace_oct, 6 k_trace_w (+ k_trace_lds over its retrace queue) */
    PT_Q_SHADE_KERNEL = 6      /* shading kernel: 0 k_shade, 3 k_shade_w3, 4 k_shade_w3h, 5 k_shade_tab, 6 k_shade_dl,
                                  7 / 8 / 9 k_shade_hero / _w2 / _w4 */
};
pt_status pt_scene_query(const pt_scene* scene, int32_t key, int64_t* value);

/* Number of cropped pixels (rgb_out holds 3x this many floats). */
pt_status pt_film_size(const pt_scene* scene, int32_t* width, int32_t* height);

/* Film::WriteImage to a PFM file (imageio.cpp WritePFM). */
pt_status pt_write_pfm(const char* path, const float* rgb, int32_t width, int32_t height);
/* WriteImage (imageio.cpp:81-122): format by suffix (.exr half RGB with
 * display window = full resolution and data window = [x0, x0+width) x
 * [y0, y0+height); .pfm; .png / .tga 8-bit gamma-corrected).  rgb is the
 * cropped image, width x height x 3, row-major from the top. */
pt_status pt_write_image(const char* path, const float* rgb, int32_t width, int32_t height, int32_t full_xres,
                         int32_t full_yres, int32_t x0, int32_t y0);
/* Film::WriteImage (film.cpp:169-211 + the write above) for a rendered scene:
 * rgb = pt_render output; the cropped pixel bounds come from desc->film. */
pt_status pt_write_film_image(const pt_scene_desc* desc, const char* path, const float* rgb);
/* Film "filename" of a loaded scene (film.cpp CreateFilm; default "pbrt.exr"). */
const char* pt_host_scene_film_filename(const pt_host_scene* hs);

/* ---- test hooks (used by the parity tests; not part of the render path) ---- */
/* The shared host/device sinf/cosf port used by ConcentricSampleDisk,
 * evaluated on the host (compare with the platform libm). */
pt_status pt_debug_libm_trig(int n, const float* x, float* sin_out, float* cos_out);
/* Spectral parameter reduction of the loader (RGBSpectrum build), on the host:
 * kind 0: vals = n (lambda, value) pairs -> RGBSpectrum::FromSampled
 *         (spectrum.h, paramset.cpp:152-169), out = rgb[3];
 * kind 1: vals = (T, scale) -> blackbody parameter (paramset.cpp:134-150), out = rgb[3];
 * kind 2: vals = xyz[3] -> FromXYZ (spectrum.h:58-62), out = rgb[3];
 * kind 3: vals = n (lambda, T) pairs -> Blackbody() radiance (spectrum.cpp:939-955), out = n values. */
pt_status pt_debug_spectrum(int kind, int n, const float* vals, float* out);
/* HaltonSampler::SampleDimension(idx[i], dims[i]) on the device. */
pt_status pt_debug_halton(pt_scene* scene, int n, const uint32_t* idx, const int32_t* dims, float* out);
/* HaltonSampler per-pixel offsets for (x, y) pairs. */
pt_status pt_debug_pixel_offsets(pt_scene* scene, int n, const int32_t* pixxy, uint32_t* out);
/* Camera rays (o, d) for film positions (pLens = (0.5, 0.5)). */
pt_status pt_debug_camera_rays(pt_scene* scene, int n, const float* film_xy, float* out6);
/* BVH traversal for rays (o, d, tMax): closest primitive index in BVH order
 * (any = 0) or occlusion flag (any = 1); -1 for a miss. */
pt_status pt_debug_trace(pt_scene* scene, int n, const float* rays7, int any, int32_t* out_prim);
/* The same queries through the traversal kernel pt_render runs for this scene
 * (persistent, ray-queue driven, LDS-staged BVH when it fits): closest-hit rays
 * take tMax = Infinity as the path tracer's do (rays7[6] is read for any = 1
 * only).  counters (may be NULL): [0] BVH node visits, [1] primitive tests of
 * the batch, the reference's BVHAccel counters (bvh.cpp:659-770). */
pt_status pt_debug_trace_frame(pt_scene* scene, int n, const float* rays7, int any, int32_t* out_prim,
                               uint64_t* counters);
/* The same batch with the traversal's full counters (closest / shadow rays, node visits, primitive tests,
 * and for k_trace_w its wide-node visits, primitive tests and retraced rays) in *stats. */
pt_status pt_debug_trace_frame_ex(pt_scene* scene, int n, const float* rays7, int any, int32_t* out_prim,
                                  pt_stats* stats);
/* BSDF::f / Pdf / Sample_f of scene material `material` in the local shading
 * frame (n = (0,0,1)): per record in8 = wo[3], wi[3], u0, u1 and
 * out8 = f[3], pdf, sampled wi[3], sampled pdf (f is the sampled f when wi
 * is all zero).  src/core/reflection.cpp:713-829. */
pt_status pt_debug_bsdf(pt_scene* scene, int material, int n, const float* in8, float* out8);

#ifdef __cplusplus
}
#endif

#endif /* PT_H */
