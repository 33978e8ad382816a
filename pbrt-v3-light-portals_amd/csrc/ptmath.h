// ptmath.h -- scalar math shared by the host scene preparation and the gfx950
// kernels.  Operation order follows the reference (pbrt-v3, float build,
// no FMA contraction) so that device results match the reference bit for bit
// where the platform allows; everything is compiled with -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define PTHD __host__ __device__ __forceinline__

namespace pt {

constexpr float kPi = 3.14159265358979323846f;        // core/pbrt.h:210
constexpr float kInvPi = 0.31830988618379067154f;     // core/pbrt.h:211
constexpr float kPiOver2 = 1.57079632679489661923f;   // core/pbrt.h:214
constexpr float kPiOver4 = 0.78539816339744830961f;   // core/pbrt.h:215
constexpr float kShadowEps = 0.0001f;                 // core/pbrt.h:209
constexpr float kOneMinusEps = 0x1.fffffep-1f;        // core/rng.h:56-58
constexpr float kInf = __builtin_huge_valf();
constexpr float kMachineEps = 0x1p-24f;  // MachineEpsilon (pbrt.h:196): numeric_limits<float>::epsilon() * 0.5

// gamma(n) (core/pbrt.h:294-296) evaluated in float.
PTHD float gammaf(int n) {
    const float me = 0x1p-24f;
    return ((float)n * me) / (1.0f - (float)n * me);
}

PTHD float smax(float a, float b) { return (a < b) ? b : a; }  // std::max
PTHD float smin(float a, float b) { return (b < a) ? b : a; }  // std::min

PTHD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
PTHD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

PTHD float next_up(float v) {  // core/pbrt.h:246-258
    if (__builtin_isinf(v) && v > 0.f) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = f2u(v);
    if (v >= 0) ++ui; else --ui;
    return u2f(ui);
}
PTHD float next_down(float v) {  // core/pbrt.h:260-270
    if (__builtin_isinf(v) && v < 0.f) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = f2u(v);
    if (v > 0) --ui; else ++ui;
    return u2f(ui);
}

struct V3 {
    float x, y, z;
    PTHD float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    PTHD void set(int i, float f) { if (i == 0) x = f; else if (i == 1) y = f; else z = f; }
};
PTHD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
PTHD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PTHD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PTHD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
PTHD V3 operator*(V3 a, float f) { return v3(a.x * f, a.y * f, a.z * f); }   // v * f
PTHD V3 operator*(float f, V3 a) { return v3(f * a.x, f * a.y, f * a.z); }   // f * v
PTHD V3 vabs(V3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
PTHD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PTHD float absdot(V3 a, V3 b) { return fabsf(dot(a, b)); }
PTHD float len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
PTHD float len(V3 a) { return sqrtf(len2(a)); }
// Vector3::operator/(f): multiply by (1/f)  (geometry.h:244-248)
PTHD V3 vdiv(V3 a, float f) { float inv = 1.0f / f; return v3(a.x * inv, a.y * inv, a.z * inv); }
// Point3::operator/(f): inv * x  (geometry.h:650-654)
PTHD V3 pdiv(V3 a, float f) { float inv = 1.0f / f; return v3(inv * a.x, inv * a.y, inv * a.z); }
PTHD V3 normalize(V3 a) { return vdiv(a, len(a)); }
// Cross product evaluated in double (geometry.h:1110-1116)
PTHD V3 cross(V3 a, V3 b) {
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return v3((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)),
              (float)((ax * by) - (ay * bx)));
}
PTHD V3 faceforward(V3 n, V3 v) { return (dot(n, v) < 0.f) ? -n : n; }
PTHD float maxcomp(V3 v) { return smax(v.x, smax(v.y, v.z)); }
PTHD int maxdim(V3 v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
PTHD V3 vmin(V3 a, V3 b) { return v3(smin(a.x, b.x), smin(a.y, b.y), smin(a.z, b.z)); }
PTHD V3 vmax(V3 a, V3 b) { return v3(smax(a.x, b.x), smax(a.y, b.y), smax(a.z, b.z)); }
PTHD float dist2(V3 a, V3 b) { return len2(a - b); }
PTHD V3 permute(V3 v, int x, int y, int z) { return v3(v[x], v[y], v[z]); }

PTHD void coordinate_system(V3 v1, V3* v2, V3* v3o) {  // geometry.h:1173-1180
    if (fabsf(v1.x) > fabsf(v1.y))
        *v2 = vdiv(v3(-v1.z, 0, v1.x), sqrtf(v1.x * v1.x + v1.z * v1.z));
    else
        *v2 = vdiv(v3(0, v1.z, -v1.y), sqrtf(v1.y * v1.y + v1.z * v1.z));
    *v3o = cross(v1, *v2);
}

// RGBSpectrum (core/spectrum.h:102-300)
struct S3 {
    float c[3];
};
PTHD S3 s3(float v) { return S3{{v, v, v}}; }
PTHD S3 s3(float a, float b, float c) { return S3{{a, b, c}}; }
PTHD S3 operator*(S3 a, S3 b) { return s3(a.c[0] * b.c[0], a.c[1] * b.c[1], a.c[2] * b.c[2]); }
PTHD S3 operator*(S3 a, float f) { return s3(a.c[0] * f, a.c[1] * f, a.c[2] * f); }
PTHD S3 operator/(S3 a, float f) { return s3(a.c[0] / f, a.c[1] / f, a.c[2] / f); }
PTHD S3 operator/(S3 a, S3 b) { return s3(a.c[0] / b.c[0], a.c[1] / b.c[1], a.c[2] / b.c[2]); }
PTHD S3 operator-(S3 a, S3 b) { return s3(a.c[0] - b.c[0], a.c[1] - b.c[1], a.c[2] - b.c[2]); }
PTHD S3 ssqrt(S3 a) { return s3(sqrtf(a.c[0]), sqrtf(a.c[1]), sqrtf(a.c[2])); }  // Sqrt(Spectrum)
PTHD S3 operator+(S3 a, S3 b) { return s3(a.c[0] + b.c[0], a.c[1] + b.c[1], a.c[2] + b.c[2]); }
PTHD bool is_black(S3 a) { return a.c[0] == 0.f && a.c[1] == 0.f && a.c[2] == 0.f; }
PTHD float max_comp(S3 a) { float m = a.c[0]; m = smax(m, a.c[1]); m = smax(m, a.c[2]); return m; }
PTHD float lum_y(S3 a) { return 0.212671f * a.c[0] + 0.715160f * a.c[1] + 0.072169f * a.c[2]; }
PTHD bool has_nan(S3 a) { return __builtin_isnan(a.c[0]) || __builtin_isnan(a.c[1]) || __builtin_isnan(a.c[2]); }

// ---- 4x4 transforms (core/transform.h) --------------------------------------
struct M4 {
    float m[4][4];
};

// Point transform, no error (transform.h:222-233)
PTHD V3 xf_point(const M4& m, V3 p) {
    float x = p.x, y = p.y, z = p.z;
    float xp = m.m[0][0] * x + m.m[0][1] * y + m.m[0][2] * z + m.m[0][3];
    float yp = m.m[1][0] * x + m.m[1][1] * y + m.m[1][2] * z + m.m[1][3];
    float zp = m.m[2][0] * x + m.m[2][1] * y + m.m[2][2] * z + m.m[2][3];
    float wp = m.m[3][0] * x + m.m[3][1] * y + m.m[3][2] * z + m.m[3][3];
    if (wp == 1) return v3(xp, yp, zp);
    return pdiv(v3(xp, yp, zp), wp);
}
// Vector transform (transform.h:236-241)
PTHD V3 xf_vector(const M4& m, V3 v) {
    return v3(m.m[0][0] * v.x + m.m[0][1] * v.y + m.m[0][2] * v.z,
              m.m[1][0] * v.x + m.m[1][1] * v.y + m.m[1][2] * v.z,
              m.m[2][0] * v.x + m.m[2][1] * v.y + m.m[2][2] * v.z);
}
// Normal transform with the stored inverse, transposed (transform.h:244-249)
PTHD V3 xf_normal(const M4& mi, V3 n) {
    return v3(mi.m[0][0] * n.x + mi.m[1][0] * n.y + mi.m[2][0] * n.z,
              mi.m[0][1] * n.x + mi.m[1][1] * n.y + mi.m[2][1] * n.z,
              mi.m[0][2] * n.x + mi.m[1][2] * n.y + mi.m[2][2] * n.z);
}
// Point transform with absolute error output (transform.h:278-300)
PTHD V3 xf_point_err(const M4& m, V3 p, V3* err) {
    float x = p.x, y = p.y, z = p.z;
    float xp = (m.m[0][0] * x + m.m[0][1] * y) + (m.m[0][2] * z + m.m[0][3]);
    float yp = (m.m[1][0] * x + m.m[1][1] * y) + (m.m[1][2] * z + m.m[1][3]);
    float zp = (m.m[2][0] * x + m.m[2][1] * y) + (m.m[2][2] * z + m.m[2][3]);
    float wp = (m.m[3][0] * x + m.m[3][1] * y) + (m.m[3][2] * z + m.m[3][3]);
    float xs = fabsf(m.m[0][0] * x) + fabsf(m.m[0][1] * y) + fabsf(m.m[0][2] * z) + fabsf(m.m[0][3]);
    float ys = fabsf(m.m[1][0] * x) + fabsf(m.m[1][1] * y) + fabsf(m.m[1][2] * z) + fabsf(m.m[1][3]);
    float zs = fabsf(m.m[2][0] * x) + fabsf(m.m[2][1] * y) + fabsf(m.m[2][2] * z) + fabsf(m.m[2][3]);
    *err = gammaf(3) * v3(xs, ys, zs);
    if (wp == 1) return v3(xp, yp, zp);
    return pdiv(v3(xp, yp, zp), wp);
}
// Vector transform with absolute error output (transform.h:337-352)
PTHD V3 xf_vector_err(const M4& m, V3 v, V3* err) {
    const float g3 = gammaf(3);
    err->x = g3 * (fabsf(m.m[0][0] * v.x) + fabsf(m.m[0][1] * v.y) + fabsf(m.m[0][2] * v.z));
    err->y = g3 * (fabsf(m.m[1][0] * v.x) + fabsf(m.m[1][1] * v.y) + fabsf(m.m[1][2] * v.z));
    err->z = g3 * (fabsf(m.m[2][0] * v.x) + fabsf(m.m[2][1] * v.y) + fabsf(m.m[2][2] * v.z));
    return xf_vector(m, v);
}
// Point transform with incoming error (transform.h:303-334)
PTHD V3 xf_point_err_in(const M4& m, V3 p, V3 pe, V3* err) {
    float x = p.x, y = p.y, z = p.z;
    float xp = (m.m[0][0] * x + m.m[0][1] * y) + (m.m[0][2] * z + m.m[0][3]);
    float yp = (m.m[1][0] * x + m.m[1][1] * y) + (m.m[1][2] * z + m.m[1][3]);
    float zp = (m.m[2][0] * x + m.m[2][1] * y) + (m.m[2][2] * z + m.m[2][3]);
    float wp = (m.m[3][0] * x + m.m[3][1] * y) + (m.m[3][2] * z + m.m[3][3]);
    const float g3 = gammaf(3);
    float e[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
        e[r] = (g3 + 1.0f) * (fabsf(m.m[r][0]) * pe.x + fabsf(m.m[r][1]) * pe.y + fabsf(m.m[r][2]) * pe.z) +
               g3 * (fabsf(m.m[r][0] * x) + fabsf(m.m[r][1] * y) + fabsf(m.m[r][2] * z) + fabsf(m.m[r][3]));
    *err = v3(e[0], e[1], e[2]);
    if (wp == 1.f) return v3(xp, yp, zp);
    return pdiv(v3(xp, yp, zp), wp);
}

struct Ray {
    V3 o, d;
    float tmax;
};

// Transform::operator()(const Ray&): offset origin to the error bound and
// shorten tMax (transform.h:251-264).
PTHD Ray xf_ray(const M4& m, Ray r) {
    V3 oe;
    V3 o = xf_point_err(m, r.o, &oe);
    V3 d = xf_vector(m, r.d);
    float l2 = len2(d);
    float tmax = r.tmax;
    if (l2 > 0) {
        float dt = dot(vabs(d), oe) / l2;
        o = o + d * dt;
        tmax -= dt;
    }
    return Ray{o, d, tmax};
}
// Transform::operator()(const Ray&, oError*, dError*): same offset, tMax
// unchanged (transform.h:382-394) -- used by AAPlaneShape::Intersect.
PTHD Ray xf_ray_keep_tmax(const M4& m, Ray r) {
    V3 oe;
    V3 o = xf_point_err(m, r.o, &oe);
    V3 d = xf_vector(m, r.d);
    float l2 = len2(d);
    if (l2 > 0) {
        float dt = dot(vabs(d), oe) / l2;
        o = o + d * dt;
    }
    return Ray{o, d, r.tmax};
}

// OffsetRayOrigin (geometry.h:1608-1622)
PTHD V3 offset_ray_origin(V3 p, V3 perr, V3 n, V3 w) {
    float d = dot(vabs(n), perr);
    V3 off = d * n;
    if (dot(w, n) < 0) off = -off;
    V3 po = p + off;
    if (off.x > 0) po.x = next_up(po.x); else if (off.x < 0) po.x = next_down(po.x);
    if (off.y > 0) po.y = next_up(po.y); else if (off.y < 0) po.y = next_down(po.y);
    if (off.z > 0) po.z = next_up(po.z); else if (off.z < 0) po.z = next_down(po.z);
    return po;
}

// ---- sampling (core/sampling.{h,cpp}) ----------------------------------------
// sinf / cosf exactly as the reference binary gets them from the host libm
// (glibc 2.35 flt-32 sinf/cosf: fast pi/2 reduction + degree-5/6 double
// polynomials).  Verified bit-identical to the host libm for every float in
// [-3.5, 3.5] (tests/test_trig_port.py) -- ConcentricSampleDisk only needs
// [-pi/4, 3pi/4].  Evaluated without FMA; the FMA build of libm rounds to the
// same floats on that range.
constexpr double kScHpiInv = 0x1.45f306dc9c883p+23;  // 2/pi * 2^24
constexpr double kScHpi = 0x1.921fb54442d18p+0;
constexpr double kScC0 = 0x1p+0, kScC1 = -0x1.ffffffd0c621cp-2, kScC2 = 0x1.55553e1068f19p-5,
                 kScC3 = -0x1.6c087e89a359dp-10, kScC4 = 0x1.99343027bf8c3p-16;
constexpr double kScS1 = -0x1.555545995a603p-3, kScS2 = 0x1.1107605230bc4p-7, kScS3 = -0x1.994eb3774cf24p-13;
PTHD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }
// cneg: quadrants 2-3 use the second table, whose cosine coefficients are negated.
PTHD float sincos_poly(double x, double x2, bool cneg, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = kScS2 + x2 * kScS3;
        double x7 = x3 * x2;
        double s = x + x3 * kScS1;
        return (float)(s + x7 * s1);
    }
    const double c0 = cneg ? -kScC0 : kScC0, c1 = cneg ? -kScC1 : kScC1, c2v = cneg ? -kScC2 : kScC2,
                 c3 = cneg ? -kScC3 : kScC3, c4 = cneg ? -kScC4 : kScC4;
    double x4 = x2 * x2;
    double c2 = c3 + x2 * c4;
    double c1s = c0 + x2 * c1;
    double x6 = x4 * x2;
    double c = c1s + x4 * c2v;
    return (float)(c + x6 * c2);
}
// |x| < 120 (the reduce_large branch is not reachable from the hot path).
PTHD float libm_sinf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincos_poly(x, s, false, 0);
    }
    double r = x * kScHpiInv;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * kScHpi;
    double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sincos_poly(x * s, x * x, (n & 2) != 0, n);
}
PTHD float libm_cosf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x2, false, 1);
    }
    double r = x * kScHpiInv;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * kScHpi;
    double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sincos_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
}

PTHD void concentric_sample_disk(float u0, float u1, float* ox, float* oy) {  // sampling.cpp:113-130
    float x = 2.f * u0 - 1, y = 2.f * u1 - 1;
    if (x == 0 && y == 0) { *ox = 0; *oy = 0; return; }
    float theta, r;
    if (fabsf(x) > fabsf(y)) { r = x; theta = kPiOver4 * (y / x); }
    else { r = y; theta = kPiOver2 - kPiOver4 * (x / y); }
    *ox = r * libm_cosf(theta);
    *oy = r * libm_sinf(theta);
}
PTHD V3 cosine_sample_hemisphere(float u0, float u1) {  // sampling.h:160-164
    float dx, dy;
    concentric_sample_disk(u0, u1, &dx, &dy);
    float z = sqrtf(smax(0.f, 1 - dx * dx - dy * dy));
    return v3(dx, dy, z);
}
PTHD float power_heuristic(float f, float g) {  // sampling.h:172-175 (nf = ng = 1)
    float a = 1 * f, b = 1 * g;
    return (a * a) / (a * a + b * b);
}
// FindInterval over a CDF of `size` entries (core/pbrt.h:408-420)
PTHD int find_interval(const float* cdf, int size, float u) {
    int first = 0, n = size;
    while (n > 0) {
        int half = n >> 1, middle = first + half;
        if (cdf[middle] <= u) { first = middle + 1; n -= half + 1; }
        else n = half;
    }
    int r = first - 1;
    r = r < 0 ? 0 : r;
    return r > size - 2 ? size - 2 : r;
}

// ---- acosf / atanf / atan2f as the reference binary's libm computes them ------
// glibc's flt-32 e_acosf.c, s_atanf.c and e_atan2f.c (the fdlibm float
// algorithms): needed bit-exact for SphericalTheta / SphericalPhi
// (geometry.h) in the infinite light.  Validated against the host libm by
// tests/test_oracle_known_answers.py.
constexpr float kAcPi = 3.1415925026e+00f, kAcPio2Hi = 1.5707962513e+00f, kAcPio2Lo = 7.5497894159e-08f;
constexpr float kAcP0 = 1.6666667163e-01f, kAcP1 = -3.2556581497e-01f, kAcP2 = 2.0121252537e-01f,
                kAcP3 = -4.0055535734e-02f, kAcP4 = 7.9153501429e-04f, kAcP5 = 3.4793309169e-05f;
constexpr float kAcQ1 = -2.4033949375e+00f, kAcQ2 = 2.0209457874e+00f, kAcQ3 = -6.8828397989e-01f,
                kAcQ4 = 7.7038154006e-02f;
PTHD float libm_acosf(float x) {
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return hx > 0 ? 0.0f : kAcPi + 2.0f * kAcPio2Lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix <= 0x32800000) return kAcPio2Hi + kAcPio2Lo;
        const float z = x * x;
        const float p = z * (kAcP0 + z * (kAcP1 + z * (kAcP2 + z * (kAcP3 + z * (kAcP4 + z * kAcP5)))));
        const float q = 1.0f + z * (kAcQ1 + z * (kAcQ2 + z * (kAcQ3 + z * kAcQ4)));
        const float r = p / q;
        return kAcPio2Hi - (x - (kAcPio2Lo - x * r));
    } else if (hx < 0) {
        const float z = (1.0f + x) * 0.5f;
        const float p = z * (kAcP0 + z * (kAcP1 + z * (kAcP2 + z * (kAcP3 + z * (kAcP4 + z * kAcP5)))));
        const float q = 1.0f + z * (kAcQ1 + z * (kAcQ2 + z * (kAcQ3 + z * kAcQ4)));
        const float sq = sqrtf(z);
        const float r = p / q;
        const float w = r * sq - kAcPio2Lo;
        return kAcPi - 2.0f * (sq + w);
    } else {
        const float z = (1.0f - x) * 0.5f;
        const float sq = sqrtf(z);
        const float df = u2f(f2u(sq) & 0xfffff000u);
        const float c = (z - df * df) / (sq + df);
        const float p = z * (kAcP0 + z * (kAcP1 + z * (kAcP2 + z * (kAcP3 + z * (kAcP4 + z * kAcP5)))));
        const float q = 1.0f + z * (kAcQ1 + z * (kAcQ2 + z * (kAcQ3 + z * kAcQ4)));
        const float r = p / q;
        const float w = r * sq + c;
        return 2.0f * (df + w);
    }
}
PTHD float libm_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -zz : zz;
}
PTHD float libm_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)f2u(x), hy = (int32_t)f2u(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return libm_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 26) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -26) z = 0.0f;
    else z = libm_atanf(fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// ---- double-precision sin/cos for moderate arguments ---------------------------
// The reference calls <math.h>'s double cos/sin in TrowbridgeReitzSample11
// (phi in [0, 2pi)).  These follow the classic fdlibm kernels (k_sin.c,
// k_cos.c) after a two-constant pi/2 reduction: < 1 ulp in double, so the
// float results the reference derives from them agree with glibc except when
// a double lands within 1 ulp of a float rounding boundary (~2^-28 odds).
// Valid for |x| < 2^19 * pi/2.
constexpr double kDS1 = -1.66666666666666324348e-01, kDS2 = 8.33333333332248946124e-03,
                 kDS3 = -1.98412698298579493134e-04, kDS4 = 2.75573137070700676789e-06,
                 kDS5 = -2.50507602534068634195e-08, kDS6 = 1.58969099521155010221e-10;
constexpr double kDC1 = 4.16666666666666019037e-02, kDC2 = -1.38888888888741095749e-03,
                 kDC3 = 2.48015872894767294178e-05, kDC4 = -2.75573143513906633035e-07,
                 kDC5 = 2.08757232129817482790e-09, kDC6 = -1.13596475577881948265e-11;
constexpr double kPio2_1 = 1.57079632673412561417e+00, kPio2_1t = 6.07710050650619224932e-11;
constexpr double kInvPio2 = 6.36619772367581382433e-01;
PTHD double dk_sin(double x, double y) {
    const double z = x * x, v = z * x;
    const double r = kDS2 + z * (kDS3 + z * (kDS4 + z * (kDS5 + z * kDS6)));
    return x - ((z * (0.5 * y - v * r) - y) - v * kDS1);
}
PTHD double dk_cos(double x, double y) {
    const double z = x * x;
    const double r = z * (kDC1 + z * (kDC2 + z * (kDC3 + z * (kDC4 + z * (kDC5 + z * kDC6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}
PTHD void dsincos_reduce(double x, int* q, double* hi, double* lo) {
    const double n = __builtin_rint(x * kInvPio2);
    const double r = x - n * kPio2_1;
    const double w = n * kPio2_1t;
    *hi = r - w;
    *lo = (r - *hi) - w;
    *q = (int)n & 3;
}
PTHD double dsin_mod(double x) {
    int q; double a, b;
    dsincos_reduce(x, &q, &a, &b);
    switch (q) {
        case 0: return dk_sin(a, b);
        case 1: return dk_cos(a, b);
        case 2: return -dk_sin(a, b);
        default: return -dk_cos(a, b);
    }
}
PTHD double dcos_mod(double x) {
    int q; double a, b;
    dsincos_reduce(x, &q, &a, &b);
    switch (q) {
        case 0: return dk_cos(a, b);
        case 1: return -dk_sin(a, b);
        case 2: return -dk_cos(a, b);
        default: return dk_sin(a, b);
    }
}

// ---- low discrepancy (core/lowdiscrepancy.{h,cpp}) ----------------------------
PTHD uint32_t reverse_bits32(uint32_t n) {
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    return n;
}

// Division of a 32-bit index by a per-dimension prime with a precomputed
// multiplier (round-up method with the "add" step), exact for all uint32.
struct DivMagic {
    uint32_t base;
    uint32_t magic;
    uint32_t shift;
    float inv_base;  // (float)1 / (float)base, as the reference computes it
};
PTHD uint32_t fast_div(uint32_t n, const DivMagic& dm) {
    uint32_t q = (uint32_t)(((uint64_t)n * dm.magic) >> 32);
    uint32_t t = ((n - q) >> 1) + q;
    return t >> dm.shift;
}

}  // namespace pt
