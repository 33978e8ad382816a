// host_common.h -- host-side declarations shared by the loader, the BVH
// builder and the render driver.
#pragma once

#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/pt.h"
#include "ptmath.h"

namespace pt {

// Error carried to the C ABI boundary (converted to pt_status there).
struct PtError : std::runtime_error {
    pt_status status;
    PtError(pt_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

// Host Matrix4x4 / Transform (src/core/transform.{h,cpp})
struct HM4 {
    float m[4][4];
};
struct HXF {
    HM4 m, mi;
};
HM4 hm4_identity();
HM4 hm4_mul(const HM4& a, const HM4& b);
bool hm4_inverse(const HM4& m, HM4* out);
HXF hxf_identity();
HXF hxf_from_matrix(const HM4& m);
HXF hxf_inverse(const HXF& t);
HXF hxf_mul(const HXF& a, const HXF& b);
HXF hxf_translate(float x, float y, float z);
HXF hxf_scale(float x, float y, float z);
HXF hxf_perspective(float fov, float n, float f);
bool hxf_swaps_handedness(const HXF& t);
M4 to_m4(const HM4& h);

// Sphere members after the ctor's clamps (shapes/sphere.h:50-59), from the
// CreateSphereShape parameters; Area() (sphere.cpp:224).
struct SphereMembers {
    float radius, zmin, zmax, theta_min, theta_max, phi_max, area;
};
inline float clamp_to(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }  // Clamp (pbrt.h:309)
inline SphereMembers sphere_members(const pt_sphere& s) {
    SphereMembers m;
    m.radius = s.radius;
    const float zlo = smin(s.zmin, s.zmax), zhi = smax(s.zmin, s.zmax);
    m.zmin = clamp_to(zlo, -s.radius, s.radius);
    m.zmax = clamp_to(zhi, -s.radius, s.radius);
    m.theta_min = std::acos(clamp_to(zlo / s.radius, -1, 1));
    m.theta_max = std::acos(clamp_to(zhi / s.radius, -1, 1));
    m.phi_max = (kPi / 180) * clamp_to(s.phimax, 0, 360);  // Radians (pbrt.h:329)
    m.area = m.phi_max * m.radius * (m.zmax - m.zmin);
    return m;
}

// Loader
struct pt_host_scene_impl;
pt_host_scene_impl* load_pbrt_file(const char* path);
const pt_scene_desc* host_scene_desc(const pt_host_scene_impl* hs);
void host_scene_free(pt_host_scene_impl* hs);
const char* host_scene_film_filename(const pt_host_scene_impl* hs);

// Axis-aligned box (Bounds3f)
struct BBox {
    V3 pmin, pmax;
};

// Flattened BVH (bvh.cpp:95-104 LinearBVHNode, 32 bytes)
struct LinearNode {
    float bmin[3];
    float bmax[3];
    int32_t offset;      // primitivesOffset (leaf) / secondChildOffset (interior)
    uint16_t nprims;
    uint8_t axis;
    uint8_t pad;
};
static_assert(sizeof(LinearNode) == 32, "LinearBVHNode must be 32 bytes");

// Shape "plymesh" file contents (ply.cpp).
struct PlyMesh {
    std::vector<float> P, N, UV;
    std::vector<int> idx;
    bool hasN = false, hasUV = false;
};
void read_ply(const std::string& path, PlyMesh* out);

// imageio.cpp: Film output (WriteImage by suffix)
void write_image(const std::string& name, const float* rgb, int xres, int yres, int totalX, int totalY, int x0,
                 int y0);
void write_pfm(const std::string& name, const float* rgb, int xres, int yres);
uint16_t float_to_half(float x);
uint8_t to_byte(float v);

// spectrum.cpp: spectral parameters reduced to RGB (RGBSpectrum build)
float interpolate_spectrum_samples(const float* lambda, const float* vals, int n, float l);
void xyz_to_rgb(const float xyz[3], float rgb[3]);
void rgb_from_sampled(const float* lambda, const float* v, int n, float rgb[3]);
void rgb_from_blackbody(float T, float scale, float rgb[3]);
void blackbody_radiance(const float* lambda, int n, float T, float* Le);
void copper_spectrum(bool k, float rgb[3]);
// 60-bin SampledSpectrum (hero integrators): bins over [400, 700] nm
constexpr int kNSpec = 60, kLambdaStart = 400, kLambdaEnd = 700;  // spectrum.h:48-51
struct SpecTables60 {
    float X[60], Y[60], Z[60];
    float refl[7][60], illum[7][60];  // White Cyan Magenta Yellow Red Green Blue
};
const SpecTables60& spectral_tables();
float average_spectrum_samples(const float* lambda, const float* vals, int n, float l0, float l1);
void s60_from_sampled(const float* lambda, const float* v, int n, float out[60]);
void s60_from_rgb(const float rgb[3], bool reflectance, float out[60]);
void s60_to_xyz(const float s[60], float xyz[3]);
float s60_y(const float s[60]);
void s60_blackbody(float T, float scale, float out[60]);  // metal's default eta (k=false) / k
bool read_float_file(const std::string& path, std::vector<float>* values);
// Shape "loopsubdiv" (shapes/loopsubdiv.cpp:137-398): refined limit-surface
// mesh in object space -- positions, shading normals, triangle indices.
void loop_subdivide(int levels, const std::vector<int>& indices, const std::vector<float>& P,
                    std::vector<float>* outP, std::vector<float>* outN, std::vector<int>* outIdx);

// SAH BVH build over the scene's primitives (bvh.cpp:190-402, 640-658).
// prim_order[i] = index into desc->prims of the i-th primitive in BVH order.
void build_bvh(const pt_scene_desc* d, std::vector<LinearNode>* nodes, std::vector<int>* prim_order);

// World bound of primitive i of desc->prims.
BBox prim_world_bound(const pt_scene_desc* d, int i);

}  // namespace pt
