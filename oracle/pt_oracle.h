/*
 * pt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the reference's hot path
 * (Jorgeromeu/pbrt-v3-light-portals: SamplerIntegrator::Render +
 * PathIntegrator::Li + portal direct lighting).  It is the parity checker for
 * the HIP path and the CPU baseline leg of bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product never links or calls it.
 *
 * Parity pinning: the reference is NOT buildable here (its four git
 * submodules -- glog, openexr, ptex, zlib -- are empty, and a build would
 * need stand-in headers, which this project does not write).  The oracle is
 * pinned by the reference's own known-answer tests (src/tests/sampling.cpp
 * RadicalInverse / ScrambledRadicalInverse, src/tests/analytic_scenes.cpp
 * furnace radiance, src/tests/shapes.cpp triangle watertightness) -- see
 * tests/test_oracle_known_answers.py and DESIGN.md "Oracle".
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>
#include "../include/pt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_stats {
    uint64_t camera_rays;
    uint64_t closest_rays;
    uint64_t shadow_rays;
    uint64_t node_visits;
    uint64_t prim_tests;
    uint64_t samples;
    uint64_t closest_node_visits;  /* node_visits / prim_tests of the closest-hit rays only; */
    uint64_t closest_prim_tests;   /* the any-hit share is the difference */
} oracle_stats;

/* Render the scene exactly as SamplerIntegrator::Render with a PathIntegrator
 * would with --nthreads 1 (tiles merged in tile order).  nthreads > 1 renders
 * tiles concurrently but still merges in tile order, so the image is
 * bit-identical to the serial one.  rgb_out: 3 floats per cropped pixel.
 * max_tiles >= 0 restricts rendering to the first max_tiles tiles (for a
 * bounded CPU-baseline sample); -1 renders everything. */
int oracle_render(const pt_scene_desc* desc, float* rgb_out, int nthreads,
                  int max_tiles, oracle_stats* stats);

/* Like oracle_render, but returns the un-resolved film (4 floats per cropped
 * pixel: Film::Pixel xyz[3] + filterWeightSum after merging the selected
 * tiles in tile order) -- the quantity the GPU film accumulates. */
int oracle_render_accum(const pt_scene_desc* desc, float* accum_out,
                        int nthreads, int tile_offset, int tile_stride,
                        oracle_stats* stats);

/* Accumulation for camera-sample indices [s_begin, s_end) of every pixel of
 * tiles t % tile_stride == tile_offset (the Halton sequence continues past
 * the scene's spp). */
int oracle_render_range(const pt_scene_desc* desc, float* accum_out, int nthreads,
                        int tile_offset, int tile_stride, int s_begin, int s_end,
                        oracle_stats* stats);

/* 0: libm cosf/sinf as the reference binary calls them (default);
 * 1: correctly rounded trig, as the device computes it. */
void oracle_set_trig(int correctly_rounded);
int oracle_film_size(const pt_scene_desc* desc, int* w, int* h);
float oracle_scrambled_radical_inverse_perm(int base_index, uint64_t a, const uint16_t* perm);
int oracle_trace(const pt_scene_desc* desc, int n, const float* rays7, int any, int32_t* out);
int oracle_trace_counted(const pt_scene_desc* desc, int n, const float* rays7, int any, int32_t* out,
                         uint64_t* counts);

/* Flattened BVH for comparison with the product's host BVH builder.
 * nodes: 8 x uint32 per node (32-byte LinearBVHNode image). */
int oracle_build_bvh(const pt_scene_desc* desc, int32_t* n_nodes,
                     uint32_t* nodes, int32_t* prim_order, int32_t cap);

/* BSDF of scene material `mat` in the local shading frame (n = (0,0,1)),
 * batched like the product's pt_debug_bsdf: in8 = wo[3], wi[3], u0, u1 ->
 * out8 = f[3], pdf, sampled wi[3], sampled pdf (f = sampled f when wi = 0). */
int oracle_bsdf_batch(const pt_scene_desc* d, int mat, int n, const float* in8, float* out8);

/* Known-answer helpers (src/core/lowdiscrepancy.cpp). */
float oracle_radical_inverse(int base_index, uint64_t a);
float oracle_scrambled_radical_inverse(int base_index, uint64_t a);
int oracle_prime(int i);
/* Halton sampler value for (pixel, sample, dim) given the sample bounds
 * (src/samplers/halton.cpp:96-127). */
float oracle_halton_sample(int sb_x0, int sb_y0, int sb_x1, int sb_y1,
                           int px, int py, int64_t sample, int dim);
int64_t oracle_halton_index(int sb_x0, int sb_y0, int sb_x1, int sb_y1,
                            int px, int py, int64_t sample);
/* Halton permutation table entry (ComputeRadicalInversePermutations). */
int oracle_halton_perm(int64_t flat_index);

/* Watertight ray-triangle test (Triangle::Intersect, triangle.cpp:189-425);
 * returns 1 on hit and writes t, b0..b2. */
int oracle_ray_triangle(const float o[3], const float d[3], float tmax,
                        const float p0[3], const float p1[3], const float p2[3],
                        float* t, float b[3]);

/* Camera ray for a film position (GenerateRayDifferential + CameraToWorld). */
int oracle_camera_ray(const pt_scene_desc* desc, float film_x, float film_y,
                      float o[3], float d[3]);

/* The reference's unit tests for this path, restated (src/tests/shapes.cpp,
 * src/tests/sampling.cpp); see tests/test_reference_unit_tests.py. */
int oracle_test_reintersect(int i, int n_dirs, float* tri9, float* rays7, int* self_hits);
int oracle_test_triangle_sampling(int i, int count, double* unif, double* tri_est, float* tri9, float* pc3,
                                  int* bad_pdf);
/* FullSphere.Reintersect / PartialSphere.Normal / PartialSphere.Reintersect
 * (src/tests/shapes.cpp:428-498) for RNG seed i (see pt_oracle.c). */
int oracle_test_sphere(int i, int partial, int mode, int n_dirs, float* params4, float* rays7, int* self_hits,
                       float* out);
int oracle_triangle_intersect(const float tri9[9], const float ray7[7], int any, float* t);
int oracle_dist1d(const float* func, int n, int mode, float u, float* out);

#ifdef __cplusplus
}
#endif

#endif
