/*
 * pt_oracle.c -- TEST INFRASTRUCTURE ONLY (see pt_oracle.h).
 *
 * Plain-C restatement of the reference hot path.  Every function cites the
 * reference file:line it restates (paths relative to the reference root).
 * Floating point follows the reference's operation order exactly; it must be
 * compiled with -O2 -ffp-contract=off and without -ffast-math so that, like
 * the reference's g++ -O2 x86-64 build, no FMA contraction happens.
 */
#include "pt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* core/pbrt.h constants and helpers                                        */
/* ------------------------------------------------------------------------ */

#define PI_F 3.14159265358979323846f          /* pbrt.h:210 */
#define INVPI_F 0.31830988618379067154f       /* pbrt.h:211 */
#define PIOVER2_F 1.57079632679489661923f     /* pbrt.h:214 */
#define PIOVER4_F 0.78539816339744830961f     /* pbrt.h:215 */
#define SHADOW_EPS 0.0001f                    /* pbrt.h:209 */
static const float ONE_MINUS_EPS = 0x1.fffffep-1f; /* rng.h:56-58 */

/* gamma(n) = (n*eps)/(1-n*eps), evaluated in float (pbrt.h:294-296). */
static float gammaf(int n) {
    const float me = FLT_EPSILON * 0.5f;
    float a = (float)n * me;
    return a / (1.0f - (float)n * me);
}
static float G2, G3, G5, G6, G7;

/* Trig used by ConcentricSampleDisk: 0 = the platform libm's cosf/sinf (what
 * the reference binary calls), 1 = correctly rounded (double evaluation,
 * one rounding) -- the device's choice.  See DESIGN.md "Parity". */
static int g_cr_trig = 0;
static float o_cosf(float x) { return g_cr_trig ? (float)cos((double)x) : cosf(x); }
static float o_sinf(float x) { return g_cr_trig ? (float)sin((double)x) : sinf(x); }

static float fmaxs(float a, float b) { return (a < b) ? b : a; } /* std::max */
static float fmins(float a, float b) { return (b < a) ? b : a; } /* std::min */

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static float next_float_up(float v) { /* pbrt.h:246-258 */
    if (isinf(v) && v > 0.) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = f2u(v);
    if (v >= 0) ++ui; else --ui;
    return u2f(ui);
}
static float next_float_down(float v) { /* pbrt.h:260-270 */
    if (isinf(v) && v < 0.) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = f2u(v);
    if (v > 0) --ui; else ++ui;
    return u2f(ui);
}

/* ------------------------------------------------------------------------ */
/* core/geometry.h vector algebra                                           */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y, z; } V3;
typedef struct { float c[3]; } RGB;  /* RGBSpectrum, spectrum.h:348 */

static V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static float vidx(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static void vset(V3* v, int i, float f) { if (i == 0) v->x = f; else if (i == 1) v->y = f; else v->z = f; }
static V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static V3 vmul(V3 a, float f) { return v3(a.x * f, a.y * f, a.z * f); }      /* v * f */
static V3 fmulv(float f, V3 a) { return v3(f * a.x, f * a.y, f * a.z); }     /* f * v */
static V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static V3 vabs(V3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* geometry.h:1098 */
static float vabsdot(V3 a, V3 b) { return fabsf(vdot(a, b)); }
static float vlen2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static float vlen(V3 a) { return sqrtf(vlen2(a)); }
/* operator/(f): inv = 1/f then multiply (geometry.h:244-248) */
static V3 vdiv(V3 a, float f) { float inv = (float)1 / f; return v3(a.x * inv, a.y * inv, a.z * inv); }
/* Point3 operator/(f): inv * x (geometry.h:650-654) */
static V3 pdiv(V3 a, float f) { float inv = (float)1 / f; return v3(inv * a.x, inv * a.y, inv * a.z); }
static V3 vnorm(V3 a) { return vdiv(a, vlen(a)); } /* geometry.h:1137-1139 */
/* Cross in double (geometry.h:1110-1116) */
static V3 vcross(V3 a, V3 b) {
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return v3((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)),
              (float)((ax * by) - (ay * bx)));
}
static V3 faceforward(V3 n, V3 v) { return (vdot(n, v) < 0.f) ? vneg(n) : n; }
static float maxcomp(V3 v) { return fmaxs(v.x, fmaxs(v.y, v.z)); }
static int maxdim(V3 v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
static V3 vmin(V3 a, V3 b) { return v3(fmins(a.x, b.x), fmins(a.y, b.y), fmins(a.z, b.z)); }
static V3 vmax(V3 a, V3 b) { return v3(fmaxs(a.x, b.x), fmaxs(a.y, b.y), fmaxs(a.z, b.z)); }
static float dist2(V3 a, V3 b) { return vlen2(vsub(a, b)); }

static void coordinate_system(V3 v1, V3* v2, V3* v3o) { /* geometry.h:1173-1180 */
    if (fabsf(v1.x) > fabsf(v1.y))
        *v2 = vdiv(v3(-v1.z, 0, v1.x), sqrtf(v1.x * v1.x + v1.z * v1.z));
    else
        *v2 = vdiv(v3(0, v1.z, -v1.y), sqrtf(v1.y * v1.y + v1.z * v1.z));
    *v3o = vcross(v1, *v2);
}

static RGB rgb1(float v) { RGB r = {{v, v, v}}; return r; }
static RGB rgbv(const float* c) { RGB r = {{c[0], c[1], c[2]}}; return r; }
static RGB smul(RGB a, RGB b) { RGB r = {{a.c[0] * b.c[0], a.c[1] * b.c[1], a.c[2] * b.c[2]}}; return r; }
static RGB smulf(RGB a, float f) { RGB r = {{a.c[0] * f, a.c[1] * f, a.c[2] * f}}; return r; }
static RGB sdivf(RGB a, float f) { RGB r = {{a.c[0] / f, a.c[1] / f, a.c[2] / f}}; return r; }
static RGB sadd(RGB a, RGB b) { RGB r = {{a.c[0] + b.c[0], a.c[1] + b.c[1], a.c[2] + b.c[2]}}; return r; }
static int sblack(RGB a) { return a.c[0] == 0. && a.c[1] == 0. && a.c[2] == 0.; }
static float smaxc(RGB a) { float m = a.c[0]; m = fmaxs(m, a.c[1]); m = fmaxs(m, a.c[2]); return m; }
static float sy(RGB a) { /* spectrum.h:408-411 */
    return 0.212671f * a.c[0] + 0.715160f * a.c[1] + 0.072169f * a.c[2];
}
static int snan(RGB a) { return isnan(a.c[0]) || isnan(a.c[1]) || isnan(a.c[2]); }

/* ------------------------------------------------------------------------ */
/* core/transform.{h,cpp}                                                   */
/* ------------------------------------------------------------------------ */
typedef struct { float m[4][4]; } M4;
typedef struct { M4 m, mi; } XF;

static M4 m4_from(const float* a) { M4 r; memcpy(r.m, a, 64); return r; }
static XF xf_from(const pt_transform* t) { XF x; x.m = m4_from(t->m); x.mi = m4_from(t->minv); return x; }
static XF xf_inv(XF t) { XF r; r.m = t.mi; r.mi = t.m; return r; }
static M4 m4_ident(void) { M4 r; memset(&r, 0, sizeof r); r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1; return r; }

static M4 m4_mul(M4 a, M4 b) { /* transform.h:86-93 */
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] +
                        a.m[i][2] * b.m[2][j] + a.m[i][3] * b.m[3][j];
    return r;
}
static XF xf_mul(XF a, XF b) { XF r; r.m = m4_mul(a.m, b.m); r.mi = m4_mul(b.mi, a.mi); return r; } /* transform.cpp:244-246 */

static M4 m4_inverse(M4 mm) { /* transform.cpp:85-137 (Gauss-Jordan, full pivoting) */
    int indxc[4], indxr[4];
    int ipiv[4] = {0, 0, 0, 0};
    float minv[4][4];
    memcpy(minv, mm.m, sizeof minv);
    for (int i = 0; i < 4; i++) {
        int irow = 0, icol = 0;
        float big = 0.f;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (fabsf(minv[j][k]) >= big) {
                            big = fabsf(minv[j][k]);
                            irow = j;
                            icol = k;
                        }
                    }
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) { float t = minv[irow][k]; minv[irow][k] = minv[icol][k]; minv[icol][k] = t; }
        indxr[i] = irow;
        indxc[i] = icol;
        float pivinv = (float)(1. / (double)minv[icol][icol]);
        minv[icol][icol] = 1.;
        for (int j = 0; j < 4; j++) minv[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                float save = minv[j][icol];
                minv[j][icol] = 0;
                for (int k = 0; k < 4; k++) minv[j][k] -= minv[icol][k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--) {
        if (indxr[j] != indxc[j]) {
            for (int k = 0; k < 4; k++) {
                float t = minv[k][indxr[j]];
                minv[k][indxr[j]] = minv[k][indxc[j]];
                minv[k][indxc[j]] = t;
            }
        }
    }
    M4 r; memcpy(r.m, minv, sizeof minv); return r;
}
static XF xf_matrix(M4 m) { XF r; r.m = m; r.mi = m4_inverse(m); return r; }
static XF xf_scale(float x, float y, float z) { /* transform.cpp:149-153 */
    XF r; r.m = m4_ident(); r.mi = m4_ident();
    r.m.m[0][0] = x; r.m.m[1][1] = y; r.m.m[2][2] = z;
    r.mi.m[0][0] = 1 / x; r.mi.m[1][1] = 1 / y; r.mi.m[2][2] = 1 / z;
    return r;
}
static XF xf_translate(float x, float y, float z) { /* transform.cpp:141-147 */
    XF r; r.m = m4_ident(); r.mi = m4_ident();
    r.m.m[0][3] = x; r.m.m[1][3] = y; r.m.m[2][3] = z;
    r.mi.m[0][3] = -x; r.mi.m[1][3] = -y; r.mi.m[2][3] = -z;
    return r;
}
static XF xf_perspective(float fov, float n, float f) { /* transform.cpp:303-311 */
    M4 p; memset(&p, 0, sizeof p);
    p.m[0][0] = 1; p.m[1][1] = 1; p.m[2][2] = f / (f - n); p.m[2][3] = -f * n / (f - n); p.m[3][2] = 1;
    float rad = (PI_F / 180) * fov; /* Radians(fov), pbrt.h:336 */
    float invTanAng = 1 / tanf(rad / 2);
    return xf_mul(xf_scale(invTanAng, invTanAng, 1), xf_matrix(p));
}

/* Point transform without error (transform.h:222-233) */
static V3 xf_pt(const M4* m, V3 p) {
    float x = p.x, y = p.y, z = p.z;
    float xp = m->m[0][0] * x + m->m[0][1] * y + m->m[0][2] * z + m->m[0][3];
    float yp = m->m[1][0] * x + m->m[1][1] * y + m->m[1][2] * z + m->m[1][3];
    float zp = m->m[2][0] * x + m->m[2][1] * y + m->m[2][2] * z + m->m[2][3];
    float wp = m->m[3][0] * x + m->m[3][1] * y + m->m[3][2] * z + m->m[3][3];
    if (wp == 1) return v3(xp, yp, zp);
    return pdiv(v3(xp, yp, zp), wp);
}
/* Vector transform (transform.h:236-241) */
static V3 xf_vec(const M4* m, V3 v) {
    float x = v.x, y = v.y, z = v.z;
    return v3(m->m[0][0] * x + m->m[0][1] * y + m->m[0][2] * z,
              m->m[1][0] * x + m->m[1][1] * y + m->m[1][2] * z,
              m->m[2][0] * x + m->m[2][1] * y + m->m[2][2] * z);
}
/* Normal transform uses mInv transposed (transform.h:244-249) */
static V3 xf_nrm(const XF* t, V3 n) {
    const M4* mi = &t->mi;
    float x = n.x, y = n.y, z = n.z;
    return v3(mi->m[0][0] * x + mi->m[1][0] * y + mi->m[2][0] * z,
              mi->m[0][1] * x + mi->m[1][1] * y + mi->m[2][1] * z,
              mi->m[0][2] * x + mi->m[1][2] * y + mi->m[2][2] * z);
}
/* Point transform with absolute error (transform.h:278-300) */
static V3 xf_pt_err(const M4* m, V3 p, V3* err) {
    float x = p.x, y = p.y, z = p.z;
    float xp = (m->m[0][0] * x + m->m[0][1] * y) + (m->m[0][2] * z + m->m[0][3]);
    float yp = (m->m[1][0] * x + m->m[1][1] * y) + (m->m[1][2] * z + m->m[1][3]);
    float zp = (m->m[2][0] * x + m->m[2][1] * y) + (m->m[2][2] * z + m->m[2][3]);
    float wp = (m->m[3][0] * x + m->m[3][1] * y) + (m->m[3][2] * z + m->m[3][3]);
    float xs = fabsf(m->m[0][0] * x) + fabsf(m->m[0][1] * y) + fabsf(m->m[0][2] * z) + fabsf(m->m[0][3]);
    float ys = fabsf(m->m[1][0] * x) + fabsf(m->m[1][1] * y) + fabsf(m->m[1][2] * z) + fabsf(m->m[1][3]);
    float zs = fabsf(m->m[2][0] * x) + fabsf(m->m[2][1] * y) + fabsf(m->m[2][2] * z) + fabsf(m->m[2][3]);
    *err = fmulv(G3, v3(xs, ys, zs));
    if (wp == 1) return v3(xp, yp, zp);
    return pdiv(v3(xp, yp, zp), wp);
}
/* Point transform with incoming error (transform.h:303-334) */
static V3 xf_pt_err_in(const M4* m, V3 p, V3 pe, V3* err) {
    float x = p.x, y = p.y, z = p.z;
    float xp = (m->m[0][0] * x + m->m[0][1] * y) + (m->m[0][2] * z + m->m[0][3]);
    float yp = (m->m[1][0] * x + m->m[1][1] * y) + (m->m[1][2] * z + m->m[1][3]);
    float zp = (m->m[2][0] * x + m->m[2][1] * y) + (m->m[2][2] * z + m->m[2][3]);
    float wp = (m->m[3][0] * x + m->m[3][1] * y) + (m->m[3][2] * z + m->m[3][3]);
    float e[3];
    for (int r = 0; r < 3; ++r) {
        e[r] = (G3 + (float)1) * (fabsf(m->m[r][0]) * pe.x + fabsf(m->m[r][1]) * pe.y + fabsf(m->m[r][2]) * pe.z) +
               G3 * (fabsf(m->m[r][0] * x) + fabsf(m->m[r][1] * y) + fabsf(m->m[r][2] * z) + fabsf(m->m[r][3]));
    }
    *err = v3(e[0], e[1], e[2]);
    if (wp == 1.) return v3(xp, yp, zp);
    return pdiv(v3(xp, yp, zp), wp);
}

typedef struct { V3 o, d; float tMax; } Ray;

/* Transform::operator()(const Ray&) -- origin error offset, tMax -= dt (transform.h:251-264) */
static Ray xf_ray(const M4* m, Ray r) {
    V3 oe;
    V3 o = xf_pt_err(m, r.o, &oe);
    V3 d = xf_vec(m, r.d);
    float l2 = vlen2(d);
    float tMax = r.tMax;
    if (l2 > 0) {
        float dt = vdot(vabs(d), oe) / l2;
        o = vadd(o, vmul(d, dt));
        tMax -= dt;
    }
    Ray out = {o, d, tMax};
    return out;
}
/* Transform::operator()(const Ray&, oError*, dError*) -- no tMax update (transform.h:382-394) */
static Ray xf_ray_err(const M4* m, Ray r) {
    V3 oe;
    V3 o = xf_pt_err(m, r.o, &oe);
    V3 d = xf_vec(m, r.d);
    float l2 = vlen2(d);
    if (l2 > 0) {
        float dt = vdot(vabs(d), oe) / l2;
        o = vadd(o, vmul(d, dt));
    }
    Ray out = {o, d, r.tMax};
    return out;
}

/* ------------------------------------------------------------------------ */
/* core/interaction.h                                                        */
/* ------------------------------------------------------------------------ */
static V3 offset_ray_origin(V3 p, V3 pErr, V3 n, V3 w) { /* geometry.h:1608-1622 */
    float d = vdot(vabs(n), pErr);
    V3 off = fmulv(d, n);
    if (vdot(w, n) < 0) off = vneg(off);
    V3 po = vadd(p, off);
    for (int i = 0; i < 3; ++i) {
        float oi = vidx(off, i);
        if (oi > 0) vset(&po, i, next_float_up(vidx(po, i)));
        else if (oi < 0) vset(&po, i, next_float_down(vidx(po, i)));
    }
    return po;
}
static Ray spawn_ray(V3 p, V3 pErr, V3 n, V3 d) { /* interaction.h:66-69 */
    Ray r = {offset_ray_origin(p, pErr, n, d), d, INFINITY};
    return r;
}

/* Surface interaction subset used on the hot path. */
typedef struct {
    V3 p, pError, n, wo;
    V3 dpdu;       /* geometric dpdu */
    V3 sn, sdpdu;  /* shading.n, shading.dpdu */
    int prim;      /* primitive index in BVH order */
} SI;

/* ------------------------------------------------------------------------ */
/* Scene (flattened from pt_scene_desc)                                     */
/* ------------------------------------------------------------------------ */
typedef struct { V3 pmin, pmax; } BB;
static BB bb_empty(void) { BB b; b.pmin = v3(FLT_MAX, FLT_MAX, FLT_MAX); b.pmax = v3(-FLT_MAX, -FLT_MAX, -FLT_MAX); return b; }
static BB bb_pp(V3 a, V3 b) { BB r; r.pmin = vmin(a, b); r.pmax = vmax(a, b); return r; }
static BB bb_union(BB a, BB b) { BB r; r.pmin = vmin(a.pmin, b.pmin); r.pmax = vmax(a.pmax, b.pmax); return r; }
static BB bb_unionp(BB a, V3 p) { BB r; r.pmin = vmin(a.pmin, p); r.pmax = vmax(a.pmax, p); return r; }
static float bb_sa(BB b) { V3 d = vsub(b.pmax, b.pmin); return 2 * (d.x * d.y + d.x * d.z + d.y * d.z); }
static int bb_maxext(BB b) { V3 d = vsub(b.pmax, b.pmin); if (d.x > d.y && d.x > d.z) return 0; else if (d.y > d.z) return 1; return 2; }
static V3 bb_offset(BB b, V3 p) {
    V3 o = vsub(p, b.pmin);
    if (b.pmax.x > b.pmin.x) o.x /= b.pmax.x - b.pmin.x;
    if (b.pmax.y > b.pmin.y) o.y /= b.pmax.y - b.pmin.y;
    if (b.pmax.z > b.pmin.z) o.z /= b.pmax.z - b.pmin.z;
    return o;
}

typedef struct {
    BB bounds;
    int offset;        /* primitivesOffset / secondChildOffset */
    uint16_t nprims;
    uint8_t axis;
} LNode;

typedef struct {
    V3 lo, hi;                 /* object space */
    int ax, ax0, ax1;
    int facingFw;              /* = !reverseOrientation (plane.h:24) */
    int ro_xor_sh;             /* reverseOrientation ^ transformSwapsHandedness */
    XF o2w, w2o;
    float area;                /* plane.h:29-31 */
} Plane;

/* Sphere (shapes/sphere.h:50-59): clamped members, transforms, center */
typedef struct {
    float radius, zMin, zMax, thetaMin, thetaMax, phiMax, area;
    int ro, ro_xor_sh;
    XF o2w, w2o;
    V3 center; /* ObjectToWorld(Point3f(0, 0, 0)) */
} Sphere;

typedef struct {
    const pt_scene_desc* d;
    int nprims;
    int* prim_kind;            /* BVH order */
    int* prim_index;
    LNode* nodes;
    int nnodes;
    Plane* planes;
    Sphere* spheres;
    XF* light_xf;              /* per light: light_to_world */
    float* tri_area;           /* per triangle (for triangle lights) */
    /* portal planes (AAPortal::portal), per desc portal */
    Plane* portal_planes;
    /* light distribution (Distribution1D) */
    float* ldist_func;
    float* ldist_cdf;
    float ldist_int;
    int nlights;
    struct Inf* inf;           /* per light: InfiniteAreaLight data (kind INFINITE) */
    /* camera */
    M4 raster_to_camera;
    M4 camera_to_world;
    float lens_radius, focal_distance;
    /* film */
    int crop_x0, crop_y0, crop_x1, crop_y1;
    int sb_x0, sb_y0, sb_x1, sb_y1;
    float filter_table[256];
    float fr_x, fr_y;
    /* halton */
    int base_scales[2], base_exps[2], sample_stride, mult_inverse[2];
    int spp;
    int s_begin, s_end;  /* camera-sample index range rendered per pixel */
    int max_depth;
    int integrator;            /* pt_integrator_kind */
    int dl_strategy;           /* pt_direct_strategy */
    int n2D;                   /* DirectLighting "all": requested 2D arrays */
    int* sizes2D;
    float rr_threshold;
    int pix_x0, pix_y0, pix_x1, pix_y1; /* integrator pixelBounds */
} Scene;

/* ------------------------------------------------------------------------ */
/* core/lowdiscrepancy + samplers/halton + core/rng                          */
/* ------------------------------------------------------------------------ */
#define PRIME_TABLE_SIZE 1000
static int g_primes[PRIME_TABLE_SIZE];
static int g_prime_sums[PRIME_TABLE_SIZE];
static uint16_t* g_perms = NULL;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

typedef struct { uint64_t state, inc; } RNG; /* rng.h:53-150 */
static uint32_t rng_u32(RNG* r) {
    uint64_t old = r->state;
    r->state = old * 0x5851f42d4c957f2dULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}
static uint32_t rng_u32b(RNG* r, uint32_t b) {
    uint32_t threshold = (~b + 1u) % b;
    for (;;) { uint32_t v = rng_u32(r); if (v >= threshold) return v % b; }
}

static void init_tables(void) {
    G2 = gammaf(2); G3 = gammaf(3); G5 = gammaf(5); G6 = gammaf(6); G7 = gammaf(7);
    /* Primes[1000] (lowdiscrepancy.cpp:40): the first 1000 primes. */
    int n = 0;
    for (int c = 2; n < PRIME_TABLE_SIZE; ++c) {
        int ok = 1;
        for (int k = 0; k < n && g_primes[k] * g_primes[k] <= c; ++k)
            if (c % g_primes[k] == 0) { ok = 0; break; }
        if (ok) g_primes[n++] = c;
    }
    int s = 0;
    for (int i = 0; i < PRIME_TABLE_SIZE; ++i) { g_prime_sums[i] = s; s += g_primes[i]; }
    /* ComputeRadicalInversePermutations (lowdiscrepancy.cpp:2490-2504) with a
     * default-state RNG (halton.cpp:69-72, rng.h:129) and Shuffle
     * (sampling.h:152-158). */
    g_perms = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)s);
    RNG rng = {0x853c49e6748fea9bULL, 0xda3e39cb94b95bdbULL};
    uint16_t* p = g_perms;
    for (int i = 0; i < PRIME_TABLE_SIZE; ++i) {
        int P = g_primes[i];
        for (int j = 0; j < P; ++j) p[j] = (uint16_t)j;
        for (int j = 0; j < P; ++j) {
            int other = j + (int)rng_u32b(&rng, (uint32_t)(P - j));
            uint16_t t = p[j]; p[j] = p[other]; p[other] = t;
        }
        p += P;
    }
}
static void ensure_init(void) { pthread_once(&g_once, init_tables); }

static uint32_t reverse_bits32(uint32_t n) { /* lowdiscrepancy.h:64-71 */
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    return n;
}
static uint64_t reverse_bits64(uint64_t n) {
    uint64_t n0 = reverse_bits32((uint32_t)n);
    uint64_t n1 = reverse_bits32((uint32_t)(n >> 32));
    return (n0 << 32) | n1;
}
/* RadicalInverseSpecialized<base> (lowdiscrepancy.cpp:388-403) */
static float radical_inverse_b(int base, uint64_t a) {
    const float invBase = (float)1 / (float)base;
    uint64_t rev = 0;
    float invBaseN = 1;
    while (a) {
        uint64_t next = a / (uint64_t)base;
        uint64_t digit = a - next * (uint64_t)base;
        rev = rev * (uint64_t)base + digit;
        invBaseN *= invBase;
        a = next;
    }
    return fmins((float)rev * invBaseN, ONE_MINUS_EPS);
}
/* RadicalInverse (lowdiscrepancy.cpp:427-...) */
static float radical_inverse(int baseIndex, uint64_t a) {
    if (baseIndex == 0) return (float)((double)reverse_bits64(a) * 0x1p-64);
    return radical_inverse_b(g_primes[baseIndex], a);
}
/* ScrambledRadicalInverseSpecialized<base> (lowdiscrepancy.cpp:405-424) */
static float scrambled_radical_inverse(int baseIndex, uint64_t a, const uint16_t* perm) {
    const int base = g_primes[baseIndex];
    const float invBase = (float)1 / (float)base;
    uint64_t rev = 0;
    float invBaseN = 1;
    while (a) {
        uint64_t next = a / (uint64_t)base;
        uint64_t digit = a - next * (uint64_t)base;
        rev = rev * (uint64_t)base + perm[digit];
        invBaseN *= invBase;
        a = next;
    }
    return fmins(invBaseN * ((float)rev + invBase * (float)perm[0] / (1 - invBase)), ONE_MINUS_EPS);
}

static int64_t mod64(int64_t a, int64_t b) { int64_t r = a - (a / b) * b; return (r < 0) ? r + b : r; }
static void extended_gcd(uint64_t a, uint64_t b, int64_t* x, int64_t* y) { /* halton.cpp:51-61 */
    if (b == 0) { *x = 1; *y = 0; return; }
    int64_t d = (int64_t)(a / b), xp, yp;
    extended_gcd(b, a % b, &xp, &yp);
    *x = yp;
    *y = xp - (d * yp);
}
static uint64_t mult_inverse(int64_t a, int64_t n) { /* halton.cpp:45-49 */
    int64_t x, y;
    extended_gcd((uint64_t)a, (uint64_t)n, &x, &y);
    return (uint64_t)mod64(x, n);
}

typedef struct { int base_scales[2], base_exps[2], stride, mult_inv[2]; int center; } Halton;

static void halton_init(Halton* h, int sbx0, int sby0, int sbx1, int sby1, int center) { /* halton.cpp:65-93 */
    int res[2] = {sbx1 - sbx0, sby1 - sby0};
    for (int i = 0; i < 2; ++i) {
        int base = (i == 0) ? 2 : 3;
        int scale = 1, ex = 0;
        int lim = res[i] < 128 ? res[i] : 128;
        while (scale < lim) { scale *= base; ++ex; }
        h->base_scales[i] = scale;
        h->base_exps[i] = ex;
    }
    h->stride = h->base_scales[0] * h->base_scales[1];
    h->mult_inv[0] = (int)mult_inverse(h->base_scales[1], h->base_scales[0]);
    h->mult_inv[1] = (int)mult_inverse(h->base_scales[0], h->base_scales[1]);
    h->center = center;
}
static uint64_t inverse_radical_inverse(int base, uint64_t inv, int nDigits) { /* lowdiscrepancy.h:83-91 */
    uint64_t index = 0;
    for (int i = 0; i < nDigits; ++i) {
        uint64_t digit = inv % (uint64_t)base;
        inv /= (uint64_t)base;
        index = index * (uint64_t)base + digit;
    }
    return index;
}
static int64_t halton_pixel_offset(const Halton* h, int px, int py) { /* halton.cpp:96-113 */
    int64_t off = 0;
    if (h->stride > 1) {
        int pm[2] = {(int)mod64(px, 128), (int)mod64(py, 128)};
        for (int i = 0; i < 2; ++i) {
            uint64_t dimOffset = inverse_radical_inverse(i == 0 ? 2 : 3, (uint64_t)pm[i], h->base_exps[i]);
            off = (int64_t)((uint64_t)off + dimOffset * (uint64_t)(h->stride / h->base_scales[i]) * (uint64_t)h->mult_inv[i]);
        }
        off %= h->stride;
    }
    return off;
}
static float halton_dim(const Halton* h, int64_t index, int dim) { /* halton.cpp:118-127 */
    if (h->center && (dim == 0 || dim == 1)) return 0.5f;
    if (dim == 0) return radical_inverse(dim, (uint64_t)(index >> h->base_exps[0]));
    if (dim == 1) return radical_inverse(dim, (uint64_t)(index / h->base_scales[1]));
    return scrambled_radical_inverse(dim, (uint64_t)index, g_perms + g_prime_sums[dim]);
}

/* GlobalSampler (sampler.cpp:137-196).  PathIntegrator requests no sample
 * arrays (arrayEndDim == arrayStartDim == 5: nothing is skipped); the
 * DirectLightingIntegrator's "all" strategy requests 2D arrays, which occupy
 * dimensions [5, arrayEndDim) and are drawn from the pixel's sample indices
 * s*n .. s*n+n-1 (StartPixel, sampler.cpp:137-162). */
#define ARRAY_START_DIM 5 /* sampler.h:122 */
typedef struct {
    const Halton* h;
    int64_t index;             /* GetIndexForSample(s) */
    int dim;
    int64_t pixOff;            /* GetIndexForSample(0) */
    int s;                     /* currentPixelSampleIndex */
    int arrayEndDim;
    int n2D, off2D;            /* requested 2D arrays / array2DOffset */
    const int* sizes2D;
    int overflow;              /* a dimension past the prime table was requested */
} Samp;
static float samp_dim(Samp* s, int64_t index, int dim) {
    if (dim >= PRIME_TABLE_SIZE) { s->overflow = 1; return 0.5f; } /* the reference CHECK-fails here */
    return halton_dim(s->h, index, dim);
}
static float get1d(Samp* s) {
    if (s->dim >= ARRAY_START_DIM && s->dim < s->arrayEndDim) s->dim = s->arrayEndDim;
    return samp_dim(s, s->index, s->dim++);
}
static void get2d(Samp* s, float* u) {
    if (s->dim + 1 >= ARRAY_START_DIM && s->dim < s->arrayEndDim) s->dim = s->arrayEndDim;
    u[0] = samp_dim(s, s->index, s->dim);
    u[1] = samp_dim(s, s->index, s->dim + 1);
    s->dim += 2;
}
/* Sampler::Get2DArray (sampler.cpp:89-94): the next requested array, or NULL */
static int get2d_array(Samp* s, int n, float* out) {
    if (s->off2D == s->n2D) return 0;
    int i = s->off2D++;
    int dim = ARRAY_START_DIM + 2 * i;
    for (int k = 0; k < n; ++k) {
        int64_t idx = s->pixOff + (int64_t)(s->s * n + k) * s->h->stride;
        out[2 * k] = samp_dim(s, idx, dim);
        out[2 * k + 1] = samp_dim(s, idx, dim + 1);
    }
    (void)s->sizes2D;
    return 1;
}

/* ------------------------------------------------------------------------ */
/* core/sampling                                                            */
/* ------------------------------------------------------------------------ */
static void concentric_sample_disk(const float* u, float* out) { /* sampling.cpp:113-130 */
    float ox = 2.f * u[0] - 1, oy = 2.f * u[1] - 1;
    if (ox == 0 && oy == 0) { out[0] = 0; out[1] = 0; return; }
    float theta, r;
    if (fabsf(ox) > fabsf(oy)) { r = ox; theta = PIOVER4_F * (oy / ox); }
    else { r = oy; theta = PIOVER2_F - PIOVER4_F * (ox / oy); }
    out[0] = r * o_cosf(theta);
    out[1] = r * o_sinf(theta);
}
static V3 cosine_sample_hemisphere(const float* u) { /* sampling.h:160-164 */
    float d[2];
    concentric_sample_disk(u, d);
    float z = sqrtf(fmaxs((float)0, 1 - d[0] * d[0] - d[1] * d[1]));
    return v3(d[0], d[1], z);
}
static float power_heuristic(float fPdf, float gPdf) { /* sampling.h:172-175, nf=ng=1 */
    float f = 1 * fPdf, g = 1 * gPdf;
    return (f * f) / (f * f + g * g);
}
static int find_interval_cdf(const float* cdf, int size, float u) { /* pbrt.h:408-420 */
    int first = 0, len = size;
    while (len > 0) {
        int half = len >> 1, middle = first + half;
        if (cdf[middle] <= u) { first = middle + 1; len -= half + 1; }
        else len = half;
    }
    int r = first - 1;
    if (r < 0) r = 0;
    if (r > size - 2) r = size - 2;
    return r;
}
/* Distribution1D (sampling.h:55-110) */
static void dist1d_build(const float* f, int n, float* cdf, float* funcInt) {
    cdf[0] = 0;
    for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + f[i - 1] / n;
    *funcInt = cdf[n];
    if (*funcInt == 0) { for (int i = 1; i < n + 1; ++i) cdf[i] = (float)i / (float)n; }
    else { for (int i = 1; i < n + 1; ++i) cdf[i] /= *funcInt; }
}
static int dist1d_sample_discrete(const float* func, const float* cdf, float funcInt, int n, float u, float* pdf) {
    int off = find_interval_cdf(cdf, n + 1, u);
    if (pdf) *pdf = (funcInt > 0) ? func[off] / (funcInt * n) : 0;
    return off;
}

/* ------------------------------------------------------------------------ */
/* shapes/triangle.cpp                                                      */
/* ------------------------------------------------------------------------ */
static V3 vtx(const pt_scene_desc* d, int i) { return v3(d->P[3 * i], d->P[3 * i + 1], d->P[3 * i + 2]); }
static V3 nrm_at(const pt_scene_desc* d, int i) { return v3(d->N[3 * i], d->N[3 * i + 1], d->N[3 * i + 2]); }
static V3 s_at(const pt_scene_desc* d, int i) { return v3(d->S[3 * i], d->S[3 * i + 1], d->S[3 * i + 2]); }
static V3 permute(V3 v, int x, int y, int z) { return v3(vidx(v, x), vidx(v, y), vidx(v, z)); }

static void tri_uvs(const pt_scene_desc* d, const pt_triangle* t, float uv[3][2]) { /* triangle.h:114-124 */
    if ((t->flags & PT_TRI_HAS_UV) && d->UV) {
        for (int i = 0; i < 3; ++i) { uv[i][0] = d->UV[2 * t->v[i]]; uv[i][1] = d->UV[2 * t->v[i] + 1]; }
    } else {
        uv[0][0] = 0; uv[0][1] = 0; uv[1][0] = 1; uv[1][1] = 0; uv[2][0] = 1; uv[2][1] = 1;
    }
}

/* Triangle::Intersect / IntersectP common test (triangle.cpp:189-292, 427-532).
 * full != 0: Intersect semantics (incl. the degenerate-triangle rejection and
 * the SurfaceInteraction); full == 0: IntersectP semantics. */
static int tri_intersect(const pt_scene_desc* d, int ti, const Ray* ray, float* tHit, SI* si, int full) {
    const pt_triangle* tr = &d->triangles[ti];
    V3 p0 = vtx(d, tr->v[0]), p1 = vtx(d, tr->v[1]), p2 = vtx(d, tr->v[2]);
    V3 p0t = vsub(p0, ray->o), p1t = vsub(p1, ray->o), p2t = vsub(p2, ray->o);
    int kz = maxdim(vabs(ray->d));
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    V3 dd = permute(ray->d, kx, ky, kz);
    p0t = permute(p0t, kx, ky, kz);
    p1t = permute(p1t, kx, ky, kz);
    p2t = permute(p2t, kx, ky, kz);
    float Sx = -dd.x / dd.z, Sy = -dd.y / dd.z, Sz = 1.f / dd.z;
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
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return 0;
    float det = e0 + e1 + e2;
    if (det == 0) return 0;
    p0t.z *= Sz; p1t.z *= Sz; p2t.z *= Sz;
    float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < ray->tMax * det)) return 0;
    else if (det > 0 && (tScaled <= 0 || tScaled > ray->tMax * det)) return 0;
    float invDet = 1 / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    float t = tScaled * invDet;
    float maxZt = maxcomp(vabs(v3(p0t.z, p1t.z, p2t.z)));
    float deltaZ = G3 * maxZt;
    float maxXt = maxcomp(vabs(v3(p0t.x, p1t.x, p2t.x)));
    float maxYt = maxcomp(vabs(v3(p0t.y, p1t.y, p2t.y)));
    float deltaX = G5 * (maxXt + maxZt);
    float deltaY = G5 * (maxYt + maxZt);
    float deltaE = 2 * (G2 * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = maxcomp(vabs(v3(e0, e1, e2)));
    float deltaT = 3 * (G3 * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * fabsf(invDet);
    if (t <= deltaT) return 0;
    if (!full) { if (tHit) *tHit = t; return 1; }

    /* partial derivatives (triangle.cpp:297-318) */
    V3 dpdu = v3(0, 0, 0), dpdv = v3(0, 0, 0);
    float uv[3][2];
    tri_uvs(d, tr, uv);
    float duv02[2] = {uv[0][0] - uv[2][0], uv[0][1] - uv[2][1]};
    float duv12[2] = {uv[1][0] - uv[2][0], uv[1][1] - uv[2][1]};
    V3 dp02 = vsub(p0, p2), dp12 = vsub(p1, p2);
    float determinant = duv02[0] * duv12[1] - duv02[1] * duv12[0];
    int degenerateUV = fabs((double)determinant) < 1e-8;
    if (!degenerateUV) {
        float invdet = 1 / determinant;
        dpdu = vmul(vsub(fmulv(duv12[1], dp02), fmulv(duv02[1], dp12)), invdet);
        dpdv = vmul(vadd(fmulv(-duv12[0], dp02), fmulv(duv02[0], dp12)), invdet);
    }
    if (degenerateUV || vlen2(vcross(dpdu, dpdv)) == 0) {
        V3 ng = vcross(vsub(p2, p0), vsub(p1, p0));
        if (vlen2(ng) == 0) return 0;
        coordinate_system(vnorm(ng), &dpdu, &dpdv);
    }
    if (tHit) *tHit = t;
    if (!si) return 1;
    float xs = fabsf(b0 * p0.x) + fabsf(b1 * p1.x) + fabsf(b2 * p2.x);
    float ys = fabsf(b0 * p0.y) + fabsf(b1 * p1.y) + fabsf(b2 * p2.y);
    float zs = fabsf(b0 * p0.z) + fabsf(b1 * p1.z) + fabsf(b2 * p2.z);
    si->pError = fmulv(G7, v3(xs, ys, zs));
    si->p = vadd(vadd(fmulv(b0, p0), fmulv(b1, p1)), fmulv(b2, p2));
    si->wo = vnorm(vneg(ray->d));
    si->dpdu = dpdu;
    si->sdpdu = dpdu;
    /* isect->n = isect->shading.n = Normalize(Cross(dp02, dp12)) (triangle.cpp:347-349) */
    V3 n = vnorm(vcross(dp02, dp12));
    int ro = (tr->flags & PT_TRI_REVERSE_ORIENTATION) != 0;
    int sh = (tr->flags & PT_TRI_SWAPS_HANDEDNESS) != 0;
    if (ro ^ sh) n = vneg(n);
    si->n = n;
    si->sn = n;
    if (((tr->flags & PT_TRI_HAS_N) && d->N) || ((tr->flags & PT_TRI_HAS_S) && d->S)) {
        /* shading geometry (triangle.cpp:351-420) */
        V3 ns;
        if ((tr->flags & PT_TRI_HAS_N) && d->N) {
            ns = vadd(vadd(fmulv(b0, nrm_at(d, tr->v[0])), fmulv(b1, nrm_at(d, tr->v[1]))), fmulv(b2, nrm_at(d, tr->v[2])));
            if (vlen2(ns) > 0) ns = vnorm(ns); else ns = si->n;
        } else ns = si->n;
        V3 ss;
        if ((tr->flags & PT_TRI_HAS_S) && d->S) {
            ss = vadd(vadd(fmulv(b0, s_at(d, tr->v[0])), fmulv(b1, s_at(d, tr->v[1]))), fmulv(b2, s_at(d, tr->v[2])));
            if (vlen2(ss) > 0) ss = vnorm(ss); else ss = vnorm(si->dpdu);
        } else ss = vnorm(si->dpdu);
        V3 ts = vcross(ss, ns);
        if (vlen2(ts) > 0.f) { ts = vnorm(ts); ss = vcross(ts, ns); }
        else coordinate_system(ns, &ss, &ts);
        if (ro) ts = vneg(ts);
        /* SetShadingGeometry(ss, ts, ..., true) (interaction.cpp:72-89) */
        si->sn = vnorm(vcross(ss, ts));
        si->n = faceforward(si->n, si->sn);
        si->sdpdu = ss;
    }
    return 1;
}

static float tri_area(const pt_scene_desc* d, int ti) { /* triangle.cpp:576-582 */
    const pt_triangle* tr = &d->triangles[ti];
    V3 p0 = vtx(d, tr->v[0]), p1 = vtx(d, tr->v[1]), p2 = vtx(d, tr->v[2]);
    return (float)(0.5 * (double)vlen(vcross(vsub(p1, p0), vsub(p2, p0))));
}

/* Triangle::Sample(u, pdf) (triangle.cpp:584-609) */
static void tri_sample(const Scene* sc, int ti, const float* u, V3* p, V3* n, V3* pErr, float* pdf) {
    const pt_scene_desc* d = sc->d;
    const pt_triangle* tr = &d->triangles[ti];
    float su0 = sqrtf(u[0]);
    float b0 = 1 - su0, b1 = u[1] * su0;
    V3 p0 = vtx(d, tr->v[0]), p1 = vtx(d, tr->v[1]), p2 = vtx(d, tr->v[2]);
    float b2 = 1 - b0 - b1;
    *p = vadd(vadd(fmulv(b0, p0), fmulv(b1, p1)), fmulv(b2, p2));
    *n = vnorm(vcross(vsub(p1, p0), vsub(p2, p0)));
    if ((tr->flags & PT_TRI_HAS_N) && d->N) {
        V3 ns = vadd(vadd(fmulv(b0, nrm_at(d, tr->v[0])), fmulv(b1, nrm_at(d, tr->v[1]))), fmulv(b2, nrm_at(d, tr->v[2])));
        *n = faceforward(*n, ns);
    } else if (((tr->flags & PT_TRI_REVERSE_ORIENTATION) != 0) ^ ((tr->flags & PT_TRI_SWAPS_HANDEDNESS) != 0)) {
        *n = vmul(*n, -1); /* it.n *= -1 */
    }
    V3 pa = vadd(vadd(vabs(fmulv(b0, p0)), vabs(fmulv(b1, p1))), vabs(fmulv(b2, p2)));
    *pErr = fmulv(G6, pa);
    *pdf = 1 / sc->tri_area[ti];
}

/* ------------------------------------------------------------------------ */
/* shapes/plane.cpp (AAPlaneShape)                                          */
/* ------------------------------------------------------------------------ */
static void plane_init(Plane* pl, V3 lo, V3 hi, int axis, int reverseOrientation, int swaps, XF o2w) {
    pl->lo = lo; pl->hi = hi; pl->ax = axis;
    pl->ax0 = axis == 2 ? 0 : (axis == 0 ? 1 : 2);
    pl->ax1 = axis == 2 ? 1 : (axis == 0 ? 2 : 0);
    pl->facingFw = !reverseOrientation;
    pl->ro_xor_sh = (reverseOrientation != 0) ^ (swaps != 0);
    pl->o2w = o2w; pl->w2o = xf_inv(o2w);
    V3 loW = xf_pt(&o2w.m, lo), hiW = xf_pt(&o2w.m, hi);
    pl->area = (vidx(hiW, pl->ax0) - vidx(loW, pl->ax0)) * (vidx(hiW, pl->ax1) - vidx(loW, pl->ax1));
}
static V3 plane_normal(const Plane* pl) { /* plane.cpp:74-83 */
    V3 r = v3(0, 0, 0);
    vset(&r, pl->ax, 1);
    if (!pl->facingFw) r = vmul(r, -1);
    return r;
}
static int plane_in_front(const Plane* pl, V3 p) { /* plane.cpp:109-115 */
    if (pl->facingFw) return vidx(p, pl->ax) > vidx(pl->lo, pl->ax);
    return vidx(p, pl->ax) < vidx(pl->lo, pl->ax);
}
/* AAPlaneShape::Intersect (plane.cpp:15-55) */
static int plane_intersect(const Plane* pl, const Ray* ray, float* tHit, SI* si) {
    Ray rT = xf_ray_err(&pl->w2o.m, *ray);
    float t = (vidx(pl->lo, pl->ax) - vidx(rT.o, pl->ax)) / vidx(rT.d, pl->ax);
    V3 pHit = vadd(rT.o, fmulv(t, rT.d));
    if (vidx(pHit, pl->ax0) > vidx(pl->lo, pl->ax0) && vidx(pHit, pl->ax0) < vidx(pl->hi, pl->ax0) &&
        vidx(pHit, pl->ax1) > vidx(pl->lo, pl->ax1) && vidx(pHit, pl->ax1) < vidx(pl->hi, pl->ax1) &&
        t < rT.tMax) {
        if (tHit) *tHit = t;
        if (si) {
            V3 err = v3(0.01f, 0.01f, 0.01f);
            V3 dpdu = v3(-1, 0, 0), dpdv = v3(0, 1, 0);
            /* object-space SurfaceInteraction (interaction.cpp:44-70) */
            V3 n = vnorm(vcross(dpdu, dpdv));
            V3 sn = n;
            if (pl->ro_xor_sh) { n = vmul(n, -1); sn = vmul(sn, -1); }
            V3 wo = vnorm(vneg(rT.d)); /* -ray.d of the object-space ray, normalised (Interaction ctor) */
            /* Transform::operator()(SurfaceInteraction) (transform.cpp:262-297) */
            const XF* t2 = &pl->o2w;
            si->p = xf_pt_err_in(&t2->m, pHit, err, &si->pError);
            si->n = vnorm(xf_nrm(t2, n));
            si->wo = vnorm(xf_vec(&t2->m, wo));
            si->dpdu = xf_vec(&t2->m, dpdu);
            si->sn = vnorm(xf_nrm(t2, sn));
            si->sdpdu = xf_vec(&t2->m, dpdu);
            si->sn = faceforward(si->sn, si->n);
        }
        return 1;
    }
    return 0;
}
/* AAPlaneShape::Sample(u, pdf) (plane.cpp:57-72) */
static void plane_sample(const Plane* pl, const float* u, V3* p, V3* n, V3* pErr, float* pdf) {
    V3 loW = xf_pt(&pl->o2w.m, pl->lo), hiW = xf_pt(&pl->o2w.m, pl->hi);
    V3 q = v3(0, 0, 0);
    vset(&q, pl->ax, vidx(loW, pl->ax));
    vset(&q, pl->ax0, vidx(loW, pl->ax0) + (vidx(hiW, pl->ax0) - vidx(loW, pl->ax0)) * u[0]);
    vset(&q, pl->ax1, vidx(loW, pl->ax1) + (vidx(hiW, pl->ax1) - vidx(loW, pl->ax1)) * u[1]);
    *p = q;
    *n = plane_normal(pl);
    *pErr = v3(0.1f, 0.1f, 0.1f);
    *pdf = 1 / pl->area;
}

/* ------------------------------------------------------------------------ */
/* shapes/sphere.cpp with core/efloat.h running error bounds                 */
/* ------------------------------------------------------------------------ */
static float clampf11(float v) { return v < -1 ? -1.f : (v > 1 ? 1.f : v); } /* Clamp (pbrt.h:309-316) */
static float clampf_to(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
static void sphere_init(Sphere* s, const pt_sphere* p) { /* Sphere ctor (sphere.h:50-59) */
    float r = p->radius;
    float zlo = fmins(p->zmin, p->zmax), zhi = fmaxs(p->zmin, p->zmax);
    s->radius = r;
    s->zMin = clampf_to(zlo, -r, r);
    s->zMax = clampf_to(zhi, -r, r);
    s->thetaMin = acosf(clampf_to(zlo / r, -1, 1));
    s->thetaMax = acosf(clampf_to(zhi / r, -1, 1));
    s->phiMax = (PI_F / 180) * clampf_to(p->phimax, 0, 360);
    s->area = s->phiMax * s->radius * (s->zMax - s->zMin); /* Sphere::Area (sphere.cpp:224) */
    s->ro = (p->flags & PT_TRI_REVERSE_ORIENTATION) != 0;
    s->ro_xor_sh = s->ro ^ ((p->flags & PT_TRI_SWAPS_HANDEDNESS) != 0);
    memcpy(s->o2w.m.m, p->object_to_world.m, 64);
    memcpy(s->o2w.mi.m, p->object_to_world.minv, 64);
    s->w2o.m = s->o2w.mi; s->w2o.mi = s->o2w.m;
    s->center = xf_pt(&s->o2w.m, v3(0, 0, 0));
}

typedef struct { float v, lo, hi; } EFl; /* EFloat without the debug-only precise value */
static EFl ef1(float v) { EFl r = {v, v, v}; return r; }
static EFl ef_e(float v, float err) { /* EFloat(v, err) */
    EFl r = {v, v, v};
    if (err != 0.f) { r.lo = next_float_down(v - err); r.hi = next_float_up(v + err); }
    return r;
}
static EFl ef_add(EFl a, EFl b) { EFl r = {a.v + b.v, next_float_down(a.lo + b.lo), next_float_up(a.hi + b.hi)}; return r; }
static EFl ef_sub(EFl a, EFl b) { EFl r = {a.v - b.v, next_float_down(a.lo - b.hi), next_float_up(a.hi - b.lo)}; return r; }
static EFl ef_mul(EFl a, EFl b) {
    float p0 = a.lo * b.lo, p1 = a.hi * b.lo, p2 = a.lo * b.hi, p3 = a.hi * b.hi;
    EFl r = {a.v * b.v, next_float_down(fmins(fmins(p0, p1), fmins(p2, p3))),
             next_float_up(fmaxs(fmaxs(p0, p1), fmaxs(p2, p3)))};
    return r;
}
static EFl ef_div(EFl a, EFl b) {
    EFl r;
    r.v = a.v / b.v;
    if (b.lo < 0 && b.hi > 0) { r.lo = -INFINITY; r.hi = INFINITY; return r; }
    float d0 = a.lo / b.lo, d1 = a.hi / b.lo, d2 = a.lo / b.hi, d3 = a.hi / b.hi;
    r.lo = next_float_down(fmins(fmins(d0, d1), fmins(d2, d3)));
    r.hi = next_float_up(fmaxs(fmaxs(d0, d1), fmaxs(d2, d3)));
    return r;
}
static int ef_quadratic(EFl A, EFl B, EFl C, EFl* t0, EFl* t1) { /* efloat.h:266-287 */
    double discrim = (double)B.v * (double)B.v - 4. * (double)A.v * (double)C.v;
    if (discrim < 0.) return 0;
    double rootDiscrim = sqrt(discrim);
    EFl fr = ef_e((float)rootDiscrim, (float)((double)(FLT_EPSILON * 0.5f) * rootDiscrim));
    EFl q = (B.v < 0) ? ef_mul(ef1(-.5f), ef_sub(B, fr)) : ef_mul(ef1(-.5f), ef_add(B, fr));
    *t0 = ef_div(q, A);
    *t1 = ef_div(C, q);
    if (t0->v > t1->v) { EFl t = *t0; *t0 = *t1; *t1 = t; }
    return 1;
}
/* Vector transform with absolute error (transform.h:337-352) */
static V3 xf_vec_err(const M4* m, V3 v, V3* err) {
    err->x = G3 * (fabsf(m->m[0][0] * v.x) + fabsf(m->m[0][1] * v.y) + fabsf(m->m[0][2] * v.z));
    err->y = G3 * (fabsf(m->m[1][0] * v.x) + fabsf(m->m[1][1] * v.y) + fabsf(m->m[1][2] * v.z));
    err->z = G3 * (fabsf(m->m[2][0] * v.x) + fabsf(m->m[2][1] * v.y) + fabsf(m->m[2][2] * v.z));
    return xf_vec(m, v);
}
/* the clipped-sphere test on a candidate hit point (sphere.cpp:73-81) */
static void sphere_point(const Sphere* s, V3 o, V3 d, float t, V3* pHit, float* phi) {
    V3 p = vadd(o, vmul(d, t));
    p = vmul(p, s->radius / vlen(p));
    if (p.x == 0 && p.y == 0) p.x = 1e-5f * s->radius;
    float ph = atan2f(p.y, p.x);
    if (ph < 0) ph += 2 * PI_F;
    *pHit = p; *phi = ph;
}
static int sphere_clipped(const Sphere* s, V3 p, float phi) {
    return (s->zMin > -s->radius && p.z < s->zMin) || (s->zMax < s->radius && p.z > s->zMax) || phi > s->phiMax;
}
/* Sphere::Intersect (sphere.cpp:50-146); IntersectP (148-200) is the same
 * test without the SurfaceInteraction (si == NULL). */
static int sphere_intersect(const Sphere* s, const Ray* r, float* tHit, SI* si) {
    V3 oErr, dErr;
    V3 o = xf_pt_err(&s->w2o.m, r->o, &oErr);
    V3 d = xf_vec_err(&s->w2o.m, r->d, &dErr);
    float l2 = vlen2(d);
    if (l2 > 0) { /* Transform::operator()(Ray, oError*, dError*) (transform.h:382-394) */
        float dt = vdot(vabs(d), oErr) / l2;
        o = vadd(o, vmul(d, dt));
    }
    EFl ox = ef_e(o.x, oErr.x), oy = ef_e(o.y, oErr.y), oz = ef_e(o.z, oErr.z);
    EFl dx = ef_e(d.x, dErr.x), dy = ef_e(d.y, dErr.y), dz = ef_e(d.z, dErr.z);
    EFl a = ef_add(ef_add(ef_mul(dx, dx), ef_mul(dy, dy)), ef_mul(dz, dz));
    EFl b = ef_mul(ef1(2.f), ef_add(ef_add(ef_mul(dx, ox), ef_mul(dy, oy)), ef_mul(dz, oz)));
    EFl c = ef_sub(ef_add(ef_add(ef_mul(ox, ox), ef_mul(oy, oy)), ef_mul(oz, oz)),
                   ef_mul(ef1(s->radius), ef1(s->radius)));
    EFl t0, t1;
    if (!ef_quadratic(a, b, c, &t0, &t1)) return 0;
    if (t0.hi > r->tMax || t1.lo <= 0) return 0;
    EFl ts = t0;
    if (ts.lo <= 0) {
        ts = t1;
        if (ts.hi > r->tMax) return 0;
    }
    V3 pHit;
    float phi;
    sphere_point(s, o, d, ts.v, &pHit, &phi);
    if (sphere_clipped(s, pHit, phi)) {
        if (ts.v == t1.v) return 0; /* EFloat::operator== compares v */
        if (t1.hi > r->tMax) return 0;
        ts = t1;
        sphere_point(s, o, d, ts.v, &pHit, &phi);
        if (sphere_clipped(s, pHit, phi)) return 0;
    }
    if (tHit) *tHit = ts.v;
    if (si) {
        float theta = acosf(clampf11(pHit.z / s->radius));
        float zRadius = sqrtf(pHit.x * pHit.x + pHit.y * pHit.y);
        float invZRadius = 1 / zRadius;
        float cosPhi = pHit.x * invZRadius, sinPhi = pHit.y * invZRadius;
        V3 dpdu = v3(-s->phiMax * pHit.y, s->phiMax * pHit.x, 0);
        V3 dpdv = fmulv(s->thetaMax - s->thetaMin, v3(pHit.z * cosPhi, pHit.z * sinPhi, -s->radius * sinf(theta)));
        V3 pError = fmulv(G5, vabs(pHit));
        /* SurfaceInteraction ctor (interaction.cpp:44-70) */
        V3 n = vnorm(vcross(dpdu, dpdv));
        if (s->ro_xor_sh) n = vmul(n, -1);
        V3 wo = vnorm(vneg(d));
        /* Transform::operator()(SurfaceInteraction) (transform.cpp:262-297) */
        si->p = xf_pt_err_in(&s->o2w.m, pHit, pError, &si->pError);
        si->n = vnorm(xf_nrm(&s->o2w, n));
        si->wo = vnorm(xf_vec(&s->o2w.m, wo));
        si->dpdu = xf_vec(&s->o2w.m, dpdu);
        si->sn = vnorm(xf_nrm(&s->o2w, n));
        si->sdpdu = xf_vec(&s->o2w.m, dpdu);
        si->sn = faceforward(si->sn, si->n);
    }
    return 1;
}
/* Sphere::Sample(u, pdf) (sphere.cpp:226-236) */
static void sphere_sample_area(const Sphere* s, const float* u, V3* p, V3* n, V3* pErr, float* pdf) {
    float z = 1 - 2 * u[0]; /* UniformSampleSphere (sampling.cpp:98-103) */
    float r = sqrtf(fmaxs(0.f, 1.f - z * z));
    float phi = 2 * PI_F * u[1];
    V3 w = v3(r * cosf(phi), r * sinf(phi), z);
    V3 pObj = vadd(v3(0, 0, 0), vmul(w, s->radius));
    *n = vnorm(xf_nrm(&s->o2w, pObj));
    if (s->ro) *n = vmul(*n, -1);
    pObj = vmul(pObj, s->radius / vlen(pObj));
    V3 pObjError = fmulv(G5, vabs(pObj));
    *p = xf_pt_err_in(&s->o2w.m, pObj, pObjError, pErr);
    *pdf = 1 / s->area;
}
/* Sphere::Sample(ref, u, pdf) (sphere.cpp:238-301) */
static void sphere_sample_ref(const Sphere* s, const SI* ref, const float* u, V3* p, V3* n, V3* pErr, float* pdf) {
    V3 pCenter = s->center;
    V3 pOrigin = offset_ray_origin(ref->p, ref->pError, ref->n, vsub(pCenter, ref->p));
    if (dist2(pOrigin, pCenter) <= s->radius * s->radius) {
        sphere_sample_area(s, u, p, n, pErr, pdf);
        V3 wi = vsub(*p, ref->p);
        if (vlen2(wi) == 0) *pdf = 0;
        else {
            wi = vnorm(wi);
            *pdf *= dist2(ref->p, *p) / vabsdot(*n, vneg(wi));
        }
        if (isinf(*pdf)) *pdf = 0.f;
        return;
    }
    float dc = vlen(vsub(ref->p, pCenter));
    float invDc = 1 / dc;
    V3 wc = vmul(vsub(pCenter, ref->p), invDc);
    V3 wcX, wcY;
    coordinate_system(wc, &wcX, &wcY);
    float sinThetaMax = s->radius * invDc;
    float sinThetaMax2 = sinThetaMax * sinThetaMax;
    float invSinThetaMax = 1 / sinThetaMax;
    float cosThetaMax = sqrtf(fmaxs(0.f, 1 - sinThetaMax2));
    float cosTheta = (cosThetaMax - 1) * u[0] + 1;
    float sinTheta2 = 1 - cosTheta * cosTheta;
    if (sinThetaMax2 < 0.00068523f) { /* sin^2(1.5 deg) */
        sinTheta2 = sinThetaMax2 * u[0];
        cosTheta = sqrtf(1 - sinTheta2);
    }
    float cosAlpha = sinTheta2 * invSinThetaMax +
                     cosTheta * sqrtf(fmaxs(0.f, 1.f - sinTheta2 * invSinThetaMax * invSinThetaMax));
    float sinAlpha = sqrtf(fmaxs(0.f, 1.f - cosAlpha * cosAlpha));
    float phi = u[1] * 2 * PI_F;
    /* SphericalDirection(sinAlpha, cosAlpha, phi, -wcX, -wcY, -wc) (geometry.h:1629-1634) */
    V3 nW = vadd(vadd(vmul(vneg(wcX), sinAlpha * cosf(phi)), vmul(vneg(wcY), sinAlpha * sinf(phi))),
                 vmul(vneg(wc), cosAlpha));
    V3 pW = vadd(pCenter, vmul(nW, s->radius));
    *p = pW;
    *pErr = fmulv(G5, vabs(pW));
    *n = s->ro ? vmul(nW, -1) : nW;
    *pdf = 1 / (2 * PI_F * (1 - cosThetaMax));
}

/* ------------------------------------------------------------------------ */
/* accelerators/bvh.cpp                                                     */
/* ------------------------------------------------------------------------ */
typedef struct { int primNum; BB bounds; V3 centroid; } PInfo;
typedef struct BNode { BB bounds; struct BNode* c[2]; int axis, first, n; } BNode;

typedef struct {
    PInfo* info;
    int* ordered; int nordered;
    BNode* pool; int npool;
    int maxPrims;
} BuildCtx;

static int bucket_of(BB cb, V3 c, int dim) {
    int b = (int)(12 * vidx(bb_offset(cb, c), dim));
    if (b == 12) b = 11;
    return b;
}
/* std::partition (libstdc++ bidirectional __partition) */
static PInfo* partition_buckets(PInfo* first, PInfo* last, BB cb, int dim, int split) {
    for (;;) {
        for (;;) {
            if (first == last) return first;
            else if (bucket_of(cb, first->centroid, dim) <= split) ++first;
            else break;
        }
        --last;
        for (;;) {
            if (first == last) return first;
            else if (!(bucket_of(cb, last->centroid, dim) <= split)) --last;
            else break;
        }
        PInfo t = *first; *first = *last; *last = t;
        ++first;
    }
}

static BNode* recursive_build(BuildCtx* b, int start, int end) { /* bvh.cpp:236-402 (SAH) */
    BNode* node = &b->pool[b->npool++];
    BB bounds = bb_empty();
    for (int i = start; i < end; ++i) bounds = bb_union(bounds, b->info[i].bounds);
    int nPrimitives = end - start;
    if (nPrimitives == 1) {
        node->first = b->nordered;
        for (int i = start; i < end; ++i) b->ordered[b->nordered++] = b->info[i].primNum;
        node->n = nPrimitives; node->bounds = bounds; node->c[0] = node->c[1] = NULL;
        return node;
    }
    BB cb = bb_empty();
    for (int i = start; i < end; ++i) cb = bb_unionp(cb, b->info[i].centroid);
    int dim = bb_maxext(cb);
    int mid = (start + end) / 2;
    if (vidx(cb.pmax, dim) == vidx(cb.pmin, dim)) {
        node->first = b->nordered;
        for (int i = start; i < end; ++i) b->ordered[b->nordered++] = b->info[i].primNum;
        node->n = nPrimitives; node->bounds = bounds; node->c[0] = node->c[1] = NULL;
        return node;
    }
    if (nPrimitives <= 2) {
        /* std::nth_element on two elements == insertion sort by centroid[dim] */
        mid = (start + end) / 2;
        if (vidx(b->info[start + 1].centroid, dim) < vidx(b->info[start].centroid, dim)) {
            PInfo t = b->info[start]; b->info[start] = b->info[start + 1]; b->info[start + 1] = t;
        }
    } else {
        int count[12] = {0};
        BB bb[12];
        for (int i = 0; i < 12; ++i) bb[i] = bb_empty();
        for (int i = start; i < end; ++i) {
            int k = bucket_of(cb, b->info[i].centroid, dim);
            count[k]++;
            bb[k] = bb_union(bb[k], b->info[i].bounds);
        }
        float cost[11];
        for (int i = 0; i < 11; ++i) {
            BB b0 = bb_empty(), b1 = bb_empty();
            int c0 = 0, c1 = 0;
            for (int j = 0; j <= i; ++j) { b0 = bb_union(b0, bb[j]); c0 += count[j]; }
            for (int j = i + 1; j < 12; ++j) { b1 = bb_union(b1, bb[j]); c1 += count[j]; }
            cost[i] = 1 + ((float)c0 * bb_sa(b0) + (float)c1 * bb_sa(b1)) / bb_sa(bounds);
        }
        float minCost = cost[0];
        int split = 0;
        for (int i = 1; i < 11; ++i) if (cost[i] < minCost) { minCost = cost[i]; split = i; }
        float leafCost = (float)nPrimitives;
        if (nPrimitives > b->maxPrims || minCost < leafCost) {
            PInfo* pm = partition_buckets(&b->info[start], &b->info[end - 1] + 1, cb, dim, split);
            mid = (int)(pm - &b->info[0]);
        } else {
            node->first = b->nordered;
            for (int i = start; i < end; ++i) b->ordered[b->nordered++] = b->info[i].primNum;
            node->n = nPrimitives; node->bounds = bounds; node->c[0] = node->c[1] = NULL;
            return node;
        }
    }
    BNode* c0 = recursive_build(b, start, mid);
    BNode* c1 = recursive_build(b, mid, end);
    node->c[0] = c0; node->c[1] = c1;
    node->bounds = bb_union(c0->bounds, c1->bounds);
    node->axis = dim; node->n = 0;
    return node;
}
static int flatten(Scene* sc, BNode* n, int* offset) { /* bvh.cpp:640-658 */
    LNode* ln = &sc->nodes[*offset];
    ln->bounds = n->bounds;
    int my = (*offset)++;
    if (n->n > 0) { ln->offset = n->first; ln->nprims = (uint16_t)n->n; ln->axis = 0; }
    else {
        ln->axis = (uint8_t)n->axis; ln->nprims = 0;
        flatten(sc, n->c[0], offset);
        ln->offset = flatten(sc, n->c[1], offset);
    }
    return my;
}

static BB prim_world_bound(const Scene* sc, int kind, int idx) {
    const pt_scene_desc* d = sc->d;
    if (kind == PT_PRIM_TRIANGLE) { /* triangle.cpp:180-187 */
        const pt_triangle* t = &d->triangles[idx];
        return bb_unionp(bb_pp(vtx(d, t->v[0]), vtx(d, t->v[1])), vtx(d, t->v[2]));
    }
    /* Shape::WorldBound = ObjectToWorld(ObjectBound()) (shape.cpp:52, transform.cpp:238-249) */
    BB b;
    const M4* m;
    if (kind == PT_PRIM_SPHERE) { /* Sphere::ObjectBound (sphere.cpp:44-47) */
        const Sphere* sp = &sc->spheres[idx];
        b = bb_pp(v3(-sp->radius, -sp->radius, sp->zMin), v3(sp->radius, sp->radius, sp->zMax));
        m = &sp->o2w.m;
    } else {
        const Plane* pl = &sc->planes[idx];
        b = bb_pp(pl->lo, pl->hi);
        m = &pl->o2w.m;
    }
    V3 mn = b.pmin, mx = b.pmax;
    BB r; V3 q = xf_pt(m, v3(mn.x, mn.y, mn.z)); r.pmin = q; r.pmax = q;
    r = bb_unionp(r, xf_pt(m, v3(mx.x, mn.y, mn.z)));
    r = bb_unionp(r, xf_pt(m, v3(mn.x, mx.y, mn.z)));
    r = bb_unionp(r, xf_pt(m, v3(mn.x, mn.y, mx.z)));
    r = bb_unionp(r, xf_pt(m, v3(mn.x, mx.y, mx.z)));
    r = bb_unionp(r, xf_pt(m, v3(mx.x, mx.y, mn.z)));
    r = bb_unionp(r, xf_pt(m, v3(mx.x, mn.y, mx.z)));
    r = bb_unionp(r, xf_pt(m, v3(mx.x, mx.y, mx.z)));
    return r;
}

static void build_bvh(Scene* sc) { /* bvh.cpp:190-228 */
    const pt_scene_desc* d = sc->d;
    int n = d->n_prims;
    sc->nprims = n;
    sc->prim_kind = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    sc->prim_index = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    sc->nnodes = 0;
    sc->nodes = NULL;
    if (n == 0) return;
    BuildCtx b;
    b.info = (PInfo*)malloc(sizeof(PInfo) * (size_t)n);
    b.ordered = (int*)malloc(sizeof(int) * (size_t)n);
    b.nordered = 0;
    b.pool = (BNode*)malloc(sizeof(BNode) * (size_t)(2 * n));
    b.npool = 0;
    b.maxPrims = d->bvh_max_prims > 0 ? (d->bvh_max_prims < 255 ? d->bvh_max_prims : 255) : 4;
    for (int i = 0; i < n; ++i) {
        b.info[i].primNum = i;
        b.info[i].bounds = prim_world_bound(sc, d->prims[i].kind, d->prims[i].index);
        b.info[i].centroid = vadd(fmulv(.5f, b.info[i].bounds.pmin), fmulv(.5f, b.info[i].bounds.pmax));
    }
    BNode* root = recursive_build(&b, 0, n);
    sc->nodes = (LNode*)calloc((size_t)b.npool, sizeof(LNode));
    int off = 0;
    flatten(sc, root, &off);
    sc->nnodes = off;
    for (int i = 0; i < n; ++i) {
        sc->prim_kind[i] = d->prims[b.ordered[i]].kind;
        sc->prim_index[i] = d->prims[b.ordered[i]].index;
    }
    free(b.info); free(b.ordered); free(b.pool);
}

/* Bounds3::IntersectP(ray, invDir, dirIsNeg) (geometry.h:1584-1606) */
static int bb_hit(const BB* b, const Ray* ray, V3 invDir, const int* neg) {
    const float k = 1 + 2 * G3;
    float tMin = ((neg[0] ? b->pmax : b->pmin).x - ray->o.x) * invDir.x;
    float tMax = ((neg[0] ? b->pmin : b->pmax).x - ray->o.x) * invDir.x;
    float tyMin = ((neg[1] ? b->pmax : b->pmin).y - ray->o.y) * invDir.y;
    float tyMax = ((neg[1] ? b->pmin : b->pmax).y - ray->o.y) * invDir.y;
    tMax *= k;
    tyMax *= k;
    if (tMin > tyMax || tyMin > tMax) return 0;
    if (tyMin > tMin) tMin = tyMin;
    if (tyMax < tMax) tMax = tyMax;
    float tzMin = ((neg[2] ? b->pmax : b->pmin).z - ray->o.z) * invDir.z;
    float tzMax = ((neg[2] ? b->pmin : b->pmax).z - ray->o.z) * invDir.z;
    tzMax *= k;
    if (tMin > tzMax || tzMin > tMax) return 0;
    if (tzMin > tMin) tMin = tzMin;
    if (tzMax < tMax) tMax = tzMax;
    return (tMin < ray->tMax) && (tMax > 0);
}

typedef struct { uint64_t closest, shadow, nodes, prims, camera, dim_overflow; } Counters;

/* Scene::Intersect -> BVHAccel::Intersect (scene.cpp:45-49, bvh.cpp:662-700) */
static int scene_intersect(const Scene* sc, Ray* ray, SI* si, Counters* ctr) {
    ctr->closest++;
    if (!sc->nnodes) return 0;
    int hit = 0, hitPrim = -1;
    V3 invDir = v3(1 / ray->d.x, 1 / ray->d.y, 1 / ray->d.z);
    int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    int toVisit = 0, cur = 0;
    int stack[64];
    for (;;) {
        const LNode* node = &sc->nodes[cur];
        ctr->nodes++;
        if (bb_hit(&node->bounds, ray, invDir, neg)) {
            if (node->nprims > 0) {
                for (int i = 0; i < node->nprims; ++i) {
                    int pi = node->offset + i;
                    float t;
                    int ok;
                    ctr->prims++;
                    if (sc->prim_kind[pi] == PT_PRIM_TRIANGLE)
                        ok = tri_intersect(sc->d, sc->prim_index[pi], ray, &t, NULL, 1);
                    else if (sc->prim_kind[pi] == PT_PRIM_SPHERE)
                        ok = sphere_intersect(&sc->spheres[sc->prim_index[pi]], ray, &t, NULL);
                    else
                        ok = plane_intersect(&sc->planes[sc->prim_index[pi]], ray, &t, NULL);
                    if (ok) { ray->tMax = t; hit = 1; hitPrim = pi; } /* GeometricPrimitive::Intersect */
                }
                if (toVisit == 0) break;
                cur = stack[--toVisit];
            } else {
                if (neg[node->axis]) { stack[toVisit++] = cur + 1; cur = node->offset; }
                else { stack[toVisit++] = node->offset; cur = cur + 1; }
            }
        } else {
            if (toVisit == 0) break;
            cur = stack[--toVisit];
        }
    }
    if (hit && si) {
        /* the winning primitive's SurfaceInteraction (same ray o,d) */
        Ray r2 = *ray; r2.tMax = INFINITY;
        float t;
        if (sc->prim_kind[hitPrim] == PT_PRIM_TRIANGLE) tri_intersect(sc->d, sc->prim_index[hitPrim], &r2, &t, si, 1);
        else if (sc->prim_kind[hitPrim] == PT_PRIM_SPHERE)
            sphere_intersect(&sc->spheres[sc->prim_index[hitPrim]], &r2, &t, si);
        else plane_intersect(&sc->planes[sc->prim_index[hitPrim]], &r2, &t, si);
        si->prim = hitPrim;
    }
    return hit;
}
/* Scene::IntersectP -> BVHAccel::IntersectP (scene.cpp:51-55, bvh.cpp:702-738) */
static int scene_intersect_p(const Scene* sc, const Ray* ray, Counters* ctr) {
    ctr->shadow++;
    if (!sc->nnodes) return 0;
    V3 invDir = v3(1.f / ray->d.x, 1.f / ray->d.y, 1.f / ray->d.z);
    int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    int stack[64];
    int toVisit = 0, cur = 0;
    for (;;) {
        const LNode* node = &sc->nodes[cur];
        ctr->nodes++;
        if (bb_hit(&node->bounds, ray, invDir, neg)) {
            if (node->nprims > 0) {
                for (int i = 0; i < node->nprims; ++i) {
                    int pi = node->offset + i;
                    ctr->prims++;
                    int ok;
                    /* GeometricPrimitive::IntersectP -> Shape::IntersectP; the
                     * AAPlaneShape has no override so Shape::IntersectP calls
                     * Intersect (shape.h:58-62) */
                    if (sc->prim_kind[pi] == PT_PRIM_TRIANGLE)
                        ok = tri_intersect(sc->d, sc->prim_index[pi], ray, NULL, NULL, 0);
                    else if (sc->prim_kind[pi] == PT_PRIM_SPHERE)
                        ok = sphere_intersect(&sc->spheres[sc->prim_index[pi]], ray, NULL, NULL);
                    else
                        ok = plane_intersect(&sc->planes[sc->prim_index[pi]], ray, NULL, NULL);
                    if (ok) return 1;
                }
                if (toVisit == 0) break;
                cur = stack[--toVisit];
            } else {
                if (neg[node->axis]) { stack[toVisit++] = cur + 1; cur = node->offset; }
                else { stack[toVisit++] = node->offset; cur = cur + 1; }
            }
        } else {
            if (toVisit == 0) break;
            cur = stack[--toVisit];
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Microfacet distribution and Fresnel (core/microfacet.{h,cpp},             */
/* core/reflection.{h,cpp})                                                  */
/* ------------------------------------------------------------------------ */
static float cos2t(V3 w) { return w.z * w.z; }                               /* reflection.h:57-90 */
static float sin2t(V3 w) { return fmaxs((float)0, (float)1 - cos2t(w)); }
static float sint(V3 w) { return sqrtf(sin2t(w)); }
static float tant(V3 w) { return sint(w) / w.z; }
static float tan2t(V3 w) { return sin2t(w) / cos2t(w); }
static float cosp(V3 w) { float st = sint(w); return (st == 0) ? 1 : clampf11(w.x / st); }
static float sinp(V3 w) { float st = sint(w); return (st == 0) ? 0 : clampf11(w.y / st); }
static float cos2p(V3 w) { return cosp(w) * cosp(w); }
static float sin2p(V3 w) { return sinp(w) * sinp(w); }

static float trD(float ax, float ay, V3 wh) { /* microfacet.cpp:155-163 */
    float tan2Theta = tan2t(wh);
    if (isinf(tan2Theta)) return 0.;
    const float cos4Theta = cos2t(wh) * cos2t(wh);
    float e = (cos2p(wh) / (ax * ax) + sin2p(wh) / (ay * ay)) * tan2Theta;
    return 1 / (PI_F * ax * ay * cos4Theta * (1 + e) * (1 + e));
}
static float trLambda(float ax, float ay, V3 w) { /* microfacet.cpp:176-184 */
    float absTanTheta = fabsf(tant(w));
    if (isinf(absTanTheta)) return 0.;
    float alpha = sqrtf(cos2p(w) * ax * ax + sin2p(w) * ay * ay);
    float alpha2Tan2Theta = (alpha * absTanTheta) * (alpha * absTanTheta);
    return (-1 + sqrtf(1.f + alpha2Tan2Theta)) / 2;
}
static float trG1(float ax, float ay, V3 w) { return 1 / (1 + trLambda(ax, ay, w)); } /* microfacet.h:54-57 */
static float trG(float ax, float ay, V3 wo, V3 wi) { return 1 / (1 + trLambda(ax, ay, wo) + trLambda(ax, ay, wi)); }

/* microfacet.cpp:238-282; the normal-incidence branch uses <math.h>'s double
 * sqrt/cos/sin, which the reference's unqualified calls resolve to. */
static void trSample11(float cosTheta, float U1, float U2, float* slope_x, float* slope_y) {
    if (cosTheta > .9999) {
        float r = (float)sqrt((double)(U1 / (1 - U1)));
        float phi = (float)(6.28318530718 * U2);
        *slope_x = (float)(r * cos((double)phi));
        *slope_y = (float)(r * sin((double)phi));
        return;
    }
    float sinTheta = sqrtf(fmaxs((float)0, (float)1 - cosTheta * cosTheta));
    float tanTheta = sinTheta / cosTheta;
    float a = 1 / tanTheta;
    float G1 = 2 / (1 + sqrtf(1.f + 1.f / (a * a)));
    float A = 2 * U1 / G1 - 1;
    float tmp = 1.f / (A * A - 1.f);
    if (tmp > 1e10) tmp = (float)1e10;
    float B = tanTheta;
    float D = sqrtf(fmaxs((float)(B * B * tmp * tmp - (A * A - B * B) * tmp), (float)0));
    float slope_x_1 = B * tmp - D;
    float slope_x_2 = B * tmp + D;
    *slope_x = (A < 0 || slope_x_2 > 1.f / tanTheta) ? slope_x_1 : slope_x_2;
    float S;
    if (U2 > 0.5f) { S = 1.f; U2 = 2.f * (U2 - .5f); }
    else { S = -1.f; U2 = 2.f * (.5f - U2); }
    float z = (U2 * (U2 * (U2 * 0.27385f - 0.73369f) + 0.46341f)) /
              (U2 * (U2 * (U2 * 0.093073f + 0.309420f) - 1.000000f) + 0.597999f);
    *slope_y = S * z * sqrtf(1.f + *slope_x * *slope_x);
}
static V3 trSample(V3 wi, float alpha_x, float alpha_y, float U1, float U2) { /* microfacet.cpp:284-305 */
    V3 wiStretched = vnorm(v3(alpha_x * wi.x, alpha_y * wi.y, wi.z));
    float slope_x, slope_y;
    trSample11(wiStretched.z, U1, U2, &slope_x, &slope_y);
    float tmp = cosp(wiStretched) * slope_x - sinp(wiStretched) * slope_y;
    slope_y = sinp(wiStretched) * slope_x + cosp(wiStretched) * slope_y;
    slope_x = tmp;
    slope_x = alpha_x * slope_x;
    slope_y = alpha_y * slope_y;
    return vnorm(v3(-slope_x, -slope_y, 1.));
}
static V3 trSampleWh(float ax, float ay, V3 wo, const float* u) { /* microfacet.cpp:307-336, visible area */
    int flip = wo.z < 0;
    V3 wh = trSample(flip ? vneg(wo) : wo, ax, ay, u[0], u[1]);
    if (flip) wh = vneg(wh);
    return wh;
}
static float trPdf(float ax, float ay, V3 wo, V3 wh) { /* microfacet.cpp:338-345 */
    return trD(ax, ay, wh) * trG1(ax, ay, wo) * vabsdot(wo, wh) / fabsf(wo.z);
}
static RGB sdiv(RGB a, RGB b) { RGB r = {{a.c[0] / b.c[0], a.c[1] / b.c[1], a.c[2] / b.c[2]}}; return r; }
static RGB ssub(RGB a, RGB b) { RGB r = {{a.c[0] - b.c[0], a.c[1] - b.c[1], a.c[2] - b.c[2]}}; return r; }
static RGB ssqrt(RGB a) { RGB r = {{sqrtf(a.c[0]), sqrtf(a.c[1]), sqrtf(a.c[2])}}; return r; }
/* FrConductor (reflection.cpp:71-96) */
static RGB frConductor(float cosThetaI, RGB etai, RGB etat, RGB k) {
    cosThetaI = clampf11(cosThetaI);
    RGB eta = sdiv(etat, etai);
    RGB etak = sdiv(k, etai);
    float cosThetaI2 = cosThetaI * cosThetaI;
    float sinThetaI2 = (float)(1. - cosThetaI2);
    RGB eta2 = smul(eta, eta);
    RGB etak2 = smul(etak, etak);
    RGB t0 = ssub(ssub(eta2, etak2), rgb1(sinThetaI2));
    RGB a2plusb2 = ssqrt(sadd(smul(t0, t0), smul(smulf(eta2, 4), etak2)));
    RGB t1 = sadd(a2plusb2, rgb1(cosThetaI2));
    RGB a = ssqrt(smulf(sadd(a2plusb2, t0), 0.5f));
    RGB t2 = smulf(a, (float)2 * cosThetaI);
    RGB Rs = sdiv(ssub(t1, t2), sadd(t1, t2));
    RGB t3 = sadd(smulf(a2plusb2, cosThetaI2), rgb1(sinThetaI2 * sinThetaI2));
    RGB t4 = smulf(t2, sinThetaI2);
    RGB Rp = sdiv(smul(Rs, ssub(t3, t4)), sadd(t3, t4));
    return smulf(sadd(Rp, Rs), 0.5f);
}

/* ------------------------------------------------------------------------ */
/* BSDF (core/reflection.{h,cpp}) and the materials that build it:           */
/* matte.cpp, metal.cpp, glass.cpp, dispersive_glass.cpp, mirror.cpp,         */
/* plastic.cpp.  A BSDF holds up to two BxDFs ("lobes").                      */
/* ------------------------------------------------------------------------ */
/* BxDFType (reflection.h:70-77) */
#define BX_REFLECTION 1
#define BX_TRANSMISSION 2
#define BX_DIFFUSE 4
#define BX_GLOSSY 8
#define BX_SPECULAR 16
#define BX_ALL 31
enum { LB_LAMBERT = 1, LB_MFREFL, LB_MFTRANS, LB_FRESNELSPEC, LB_SPECREFL, LB_SPECTRANS };
enum { FR_NOOP = 0, FR_CONDUCTOR, FR_DIELECTRIC };
typedef struct {
    int kind, type, fres;
    RGB R;               /* R (reflection) or T (transmission) scale */
    RGB T;               /* FresnelSpecular's T */
    RGB feta, fk;        /* FresnelConductor(1, eta, k) */
    float fetaI, fetaT;  /* FresnelDielectric(etaI, etaT) */
    float etaA, etaB;    /* transmission lobes */
    float ax, ay;        /* TrowbridgeReitz */
} Lobe;
typedef struct {
    int n;
    Lobe lb[2];
    float eta;           /* BSDF::eta */
    V3 ns, ng, ss, ts;
} BSDF;

/* FrDielectric (reflection.cpp:47-69) */
static float frDielectric(float cosThetaI, float etaI, float etaT) {
    cosThetaI = clampf11(cosThetaI);
    int entering = cosThetaI > 0.f;
    if (!entering) { float t = etaI; etaI = etaT; etaT = t; cosThetaI = fabsf(cosThetaI); }
    float sinThetaI = sqrtf(fmaxs((float)0, 1 - cosThetaI * cosThetaI));
    float sinThetaT = etaI / etaT * sinThetaI;
    if (sinThetaT >= 1) return 1;
    float cosThetaT = sqrtf(fmaxs((float)0, 1 - sinThetaT * sinThetaT));
    float Rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    float Rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) / 2;
}
static RGB fresnel_eval(const Lobe* l, float cosThetaI) {
    if (l->fres == FR_CONDUCTOR) return frConductor(fabsf(cosThetaI), rgb1(1.), l->feta, l->fk); /* reflection.cpp:118-120 */
    if (l->fres == FR_DIELECTRIC) return rgb1(frDielectric(cosThetaI, l->fetaI, l->fetaT));      /* :128-130 */
    return rgb1(1.);                                                                            /* FresnelNoOp */
}
/* Refract (reflection.h:97-108) */
static int refract(V3 wi, V3 n, float eta, V3* wt) {
    float cosThetaI = vdot(n, wi);
    float sin2ThetaI = fmaxs((float)0, (float)(1 - cosThetaI * cosThetaI));
    float sin2ThetaT = eta * eta * sin2ThetaI;
    if (sin2ThetaT >= 1) return 0;
    float cosThetaT = sqrtf(1 - sin2ThetaT);
    *wt = vadd(vmul(vneg(wi), eta), vmul(n, eta * cosThetaI - cosThetaT));
    return 1;
}
static int same_hemi(V3 w, V3 wp) { return w.z * wp.z > 0; }

/* MicrofacetReflection::f (reflection.cpp:259-271) */
static RGB mfrefl_f(const Lobe* l, V3 wo, V3 wi) {
    float cosThetaO = fabsf(wo.z), cosThetaI = fabsf(wi.z);
    V3 wh = vadd(wi, wo);
    if (cosThetaI == 0 || cosThetaO == 0) return rgb1(0.);
    if (wh.x == 0 && wh.y == 0 && wh.z == 0) return rgb1(0.);
    wh = vnorm(wh);
    V3 whf = vdot(wh, v3(0, 0, 1)) < 0.f ? vneg(wh) : wh; /* Faceforward */
    RGB F = fresnel_eval(l, vdot(wi, whf));
    return sdivf(smul(smulf(smulf(l->R, trD(l->ax, l->ay, wh)), trG(l->ax, l->ay, wo, wi)), F),
                 4 * cosThetaI * cosThetaO);
}
/* MicrofacetTransmission::f (reflection.cpp:279-303) */
static RGB mftrans_f(const Lobe* l, V3 wo, V3 wi) {
    if (same_hemi(wo, wi)) return rgb1(0);
    float cosThetaO = wo.z, cosThetaI = wi.z;
    if (cosThetaI == 0 || cosThetaO == 0) return rgb1(0);
    float eta = wo.z > 0 ? (l->etaB / l->etaA) : (l->etaA / l->etaB);
    V3 wh = vnorm(vadd(wo, vmul(wi, eta)));
    if (wh.z < 0) wh = vneg(wh);
    if (vdot(wo, wh) * vdot(wi, wh) > 0) return rgb1(0);
    RGB F = rgb1(frDielectric(vdot(wo, wh), l->etaA, l->etaB));
    float sqrtDenom = vdot(wo, wh) + eta * vdot(wi, wh);
    float factor = 1 / eta; /* TransportMode::Radiance */
    float v = fabsf(trD(l->ax, l->ay, wh) * trG(l->ax, l->ay, wo, wi) * eta * eta * vabsdot(wi, wh) *
                    vabsdot(wo, wh) * factor * factor / (cosThetaI * cosThetaO * sqrtDenom * sqrtDenom));
    return smulf(smul(ssub(rgb1(1.f), F), l->R), v);
}
static float mftrans_pdf(const Lobe* l, V3 wo, V3 wi) { /* reflection.cpp:479-493 */
    if (same_hemi(wo, wi)) return 0;
    float eta = wo.z > 0 ? (l->etaB / l->etaA) : (l->etaA / l->etaB);
    V3 wh = vnorm(vadd(wo, vmul(wi, eta)));
    if (vdot(wo, wh) * vdot(wi, wh) > 0) return 0;
    float sqrtDenom = vdot(wo, wh) + eta * vdot(wi, wh);
    float dwh_dwi = fabsf((eta * eta * vdot(wi, wh)) / (sqrtDenom * sqrtDenom));
    return trPdf(l->ax, l->ay, wo, wh) * dwh_dwi;
}
/* BxDF::f */
static RGB lobe_f(const Lobe* l, V3 wo, V3 wi) {
    switch (l->kind) {
        case LB_LAMBERT: return smulf(l->R, INVPI_F);
        case LB_MFREFL: return mfrefl_f(l, wo, wi);
        case LB_MFTRANS: return mftrans_f(l, wo, wi);
        default: return rgb1(0.f); /* specular lobes: delta distributions */
    }
}
/* BxDF::Pdf */
static float lobe_pdf(const Lobe* l, V3 wo, V3 wi) {
    switch (l->kind) {
        case LB_LAMBERT: return same_hemi(wo, wi) ? fabsf(wi.z) * INVPI_F : 0; /* reflection.cpp:425-427 */
        case LB_MFREFL: { /* reflection.cpp:458-462 */
            if (!same_hemi(wo, wi)) return 0;
            V3 wh = vnorm(vadd(wo, wi));
            return trPdf(l->ax, l->ay, wo, wh) / (4 * vdot(wo, wh));
        }
        case LB_MFTRANS: return mftrans_pdf(l, wo, wi);
        default: return 0;
    }
}
/* BxDF::Sample_f; *type may be narrowed (FresnelSpecular) */
static RGB lobe_sample(const Lobe* l, V3 wo, V3* wi, const float* u, float* pdf, int* type) {
    switch (l->kind) {
        case LB_LAMBERT: { /* reflection.cpp:416-423 */
            *wi = cosine_sample_hemisphere(u);
            if (wo.z < 0) wi->z *= -1;
            *pdf = lobe_pdf(l, wo, *wi);
            return lobe_f(l, wo, *wi);
        }
        case LB_MFREFL: { /* reflection.cpp:443-456 */
            if (wo.z == 0) return rgb1(0.);
            V3 wh = trSampleWh(l->ax, l->ay, wo, u);
            if (vdot(wo, wh) < 0) return rgb1(0.);
            *wi = vadd(vneg(wo), vmul(wh, 2 * vdot(wo, wh))); /* Reflect */
            if (!same_hemi(wo, *wi)) return rgb1(0.f);
            *pdf = trPdf(l->ax, l->ay, wo, wh) / (4 * vdot(wo, wh));
            return mfrefl_f(l, wo, *wi);
        }
        case LB_MFTRANS: { /* reflection.cpp:466-477 */
            if (wo.z == 0) return rgb1(0.);
            V3 wh = trSampleWh(l->ax, l->ay, wo, u);
            if (vdot(wo, wh) < 0) return rgb1(0.);
            float eta = wo.z > 0 ? (l->etaA / l->etaB) : (l->etaB / l->etaA);
            if (!refract(wo, wh, eta, wi)) return rgb1(0.);
            *pdf = mftrans_pdf(l, wo, *wi);
            return mftrans_f(l, wo, *wi);
        }
        case LB_SPECREFL: { /* SpecularReflection::Sample_f (reflection.h:400-410) */
            *wi = v3(-wo.x, -wo.y, wo.z);
            *pdf = 1;
            return sdivf(smul(fresnel_eval(l, wi->z), l->R), fabsf(wi->z));
        }
        case LB_SPECTRANS: { /* SpecularTransmission::Sample_f (reflection.cpp:183-199) */
            int entering = wo.z > 0;
            float etaI = entering ? l->etaA : l->etaB;
            float etaT = entering ? l->etaB : l->etaA;
            V3 n = vdot(v3(0, 0, 1), wo) < 0.f ? v3(0, 0, -1) : v3(0, 0, 1); /* Faceforward(n, wo) */
            if (!refract(wo, n, etaI / etaT, wi)) return rgb1(0);
            *pdf = 1;
            RGB ft = smul(l->R, ssub(rgb1(1.), rgb1(frDielectric(wi->z, l->etaA, l->etaB))));
            ft = smulf(ft, (etaI * etaI) / (etaT * etaT)); /* TransportMode::Radiance */
            return sdivf(ft, fabsf(wi->z));
        }
        case LB_FRESNELSPEC: { /* FresnelSpecular::Sample_f (reflection.cpp:520-554) */
            float F = frDielectric(wo.z, l->etaA, l->etaB);
            if (u[0] < F) {
                *wi = v3(-wo.x, -wo.y, wo.z);
                *type = BX_SPECULAR | BX_REFLECTION;
                *pdf = F;
                return sdivf(smulf(l->R, F), fabsf(wi->z));
            } else {
                int entering = wo.z > 0;
                float etaI = entering ? l->etaA : l->etaB;
                float etaT = entering ? l->etaB : l->etaA;
                V3 n = vdot(v3(0, 0, 1), wo) < 0.f ? v3(0, 0, -1) : v3(0, 0, 1); /* Faceforward(n, wo) */
                if (!refract(wo, n, etaI / etaT, wi)) return rgb1(0);
                RGB ft = smulf(l->T, 1 - F); /* T * (1 - F) */
                ft = smulf(ft, (etaI * etaI) / (etaT * etaT)); /* TransportMode::Radiance */
                *type = BX_SPECULAR | BX_TRANSMISSION;
                *pdf = 1 - F;
                return sdivf(ft, fabsf(wi->z));
            }
        }
    }
    return rgb1(0.f);
}

static void add_lobe(BSDF* b, int kind, int type, RGB R) {
    Lobe* l = &b->lb[b->n++];
    memset(l, 0, sizeof *l);
    l->kind = kind; l->type = type; l->R = R;
}
static RGB clamp0(RGB r) { /* Spectrum::Clamp() */
    for (int i = 0; i < 3; ++i) r.c[i] = r.c[i] < 0 ? 0 : (r.c[i] > INFINITY ? INFINITY : r.c[i]);
    return r;
}
/* Material::ComputeScatteringFunctions(si, arena, Radiance, allowMultipleLobes)
 * + BSDF ctor (reflection.h:167-172).  wvl0: the camera's hero wavelength.
 * PathIntegrator passes allowMultipleLobes = true (path.cpp:106), the
 * DirectLightingIntegrator the default false (directlighting.cpp:72): smooth
 * glass is then SpecularReflection + SpecularTransmission (glass.cpp:62-83). */
static void make_bsdf(const pt_material* m, const SI* si, float wvl0, int multi, BSDF* b) {
    b->ns = si->sn; b->ng = si->n;
    b->ss = vnorm(si->sdpdu);
    b->ts = vcross(b->ns, b->ss);
    b->n = 0;
    b->eta = 1;
    switch (m->kind) {
        case PT_MAT_MATTE: { /* matte.cpp:45-62, sigma = 0 */
            RGB r = clamp0(rgbv(m->kd));
            if (!sblack(r)) add_lobe(b, LB_LAMBERT, BX_REFLECTION | BX_DIFFUSE, r);
            break;
        }
        case PT_MAT_METAL: { /* metal.cpp:58-79 */
            add_lobe(b, LB_MFREFL, BX_REFLECTION | BX_GLOSSY, rgb1(1.));
            Lobe* l = &b->lb[0];
            l->fres = FR_CONDUCTOR; l->feta = rgbv(m->eta); l->fk = rgbv(m->k);
            l->ax = m->alpha[0]; l->ay = m->alpha[1];
            break;
        }
        case PT_MAT_MIRROR: { /* mirror.cpp:44-52 */
            RGB r = clamp0(rgbv(m->kr));
            if (!sblack(r)) { add_lobe(b, LB_SPECREFL, BX_REFLECTION | BX_SPECULAR, r); b->lb[0].fres = FR_NOOP; }
            break;
        }
        case PT_MAT_PLASTIC: { /* plastic.cpp:45-70 */
            RGB kd = clamp0(rgbv(m->kd));
            if (!sblack(kd)) add_lobe(b, LB_LAMBERT, BX_REFLECTION | BX_DIFFUSE, kd);
            RGB ks = clamp0(rgbv(m->ks));
            if (!sblack(ks)) {
                add_lobe(b, LB_MFREFL, BX_REFLECTION | BX_GLOSSY, ks);
                Lobe* l = &b->lb[b->n - 1];
                l->fres = FR_DIELECTRIC; l->fetaI = 1.5f; l->fetaT = 1.f;
                l->ax = m->alpha[0]; l->ay = m->alpha[1];
            }
            break;
        }
        case PT_MAT_GLASS:
        case PT_MAT_DISPERSIVE_GLASS: { /* glass.cpp:45-83, dispersive_glass.cpp:48-123 (bsdf[0]) */
            float eta = m->ior;
            if (m->kind == PT_MAT_DISPERSIVE_GLASS) {
                const float lminsq = (float)(400 * 400), lmaxsq = (float)(700 * 700);
                const float cauchyB = (lminsq * m->ior_max - lmaxsq * m->ior_min) / (lminsq - lmaxsq);
                const float cauchyC = lminsq * (m->ior_max - cauchyB);
                eta = cauchyB + cauchyC / (wvl0 * wvl0);
            }
            b->eta = eta;
            RGB R = clamp0(rgbv(m->kr)), T = clamp0(rgbv(m->kt));
            if (sblack(R) && sblack(T)) break;
            if (m->specular && multi) {
                add_lobe(b, LB_FRESNELSPEC, BX_REFLECTION | BX_TRANSMISSION | BX_SPECULAR, R);
                b->lb[0].etaA = 1.f; b->lb[0].etaB = eta;
                b->lb[0].T = T;
            } else if (m->specular) {
                if (!sblack(R)) {
                    add_lobe(b, LB_SPECREFL, BX_REFLECTION | BX_SPECULAR, R);
                    Lobe* l = &b->lb[b->n - 1];
                    l->fres = FR_DIELECTRIC; l->fetaI = 1.f; l->fetaT = eta;
                }
                if (!sblack(T)) {
                    add_lobe(b, LB_SPECTRANS, BX_TRANSMISSION | BX_SPECULAR, T);
                    Lobe* l = &b->lb[b->n - 1];
                    l->etaA = 1.f; l->etaB = eta;
                }
            } else {
                if (!sblack(R)) {
                    add_lobe(b, LB_MFREFL, BX_REFLECTION | BX_GLOSSY, R);
                    Lobe* l = &b->lb[b->n - 1];
                    l->fres = FR_DIELECTRIC; l->fetaI = 1.f; l->fetaT = eta;
                    l->ax = m->alpha[0]; l->ay = m->alpha[1];
                }
                if (!sblack(T)) {
                    add_lobe(b, LB_MFTRANS, BX_TRANSMISSION | BX_GLOSSY, T);
                    Lobe* l = &b->lb[b->n - 1];
                    l->etaA = 1.f; l->etaB = eta;
                    l->ax = m->alpha[0]; l->ay = m->alpha[1];
                }
            }
            break;
        }
        default: break;
    }
}
static V3 w2l(const BSDF* b, V3 v) { return v3(vdot(v, b->ss), vdot(v, b->ts), vdot(v, b->ns)); }
static V3 l2w(const BSDF* b, V3 v) {
    return v3(b->ss.x * v.x + b->ts.x * v.y + b->ns.x * v.z,
              b->ss.y * v.x + b->ts.y * v.y + b->ns.y * v.z,
              b->ss.z * v.x + b->ts.z * v.y + b->ns.z * v.z);
}
static int lobe_matches(const Lobe* l, int flags) { return (l->type & flags) == l->type; }
static int bsdf_num(const BSDF* b, int flags) { /* BSDF::NumComponents */
    int n = 0;
    for (int i = 0; i < b->n; ++i) n += lobe_matches(&b->lb[i], flags);
    return n;
}
static RGB bsdf_f(const BSDF* b, V3 woW, V3 wiW, int flags) { /* reflection.cpp:713-726 */
    V3 wi = w2l(b, wiW), wo = w2l(b, woW);
    if (wo.z == 0) return rgb1(0);
    int reflect = vdot(wiW, b->ng) * vdot(woW, b->ng) > 0;
    RGB f = rgb1(0);
    for (int i = 0; i < b->n; ++i) {
        const Lobe* l = &b->lb[i];
        if (lobe_matches(l, flags) && ((reflect && (l->type & BX_REFLECTION)) || (!reflect && (l->type & BX_TRANSMISSION))))
            f = sadd(f, lobe_f(l, wo, wi));
    }
    return f;
}
static float bsdf_pdf(const BSDF* b, V3 woW, V3 wiW, int flags) { /* reflection.cpp:814-829 */
    if (b->n == 0) return 0.f;
    V3 wo = w2l(b, woW), wi = w2l(b, wiW);
    if (wo.z == 0) return 0.;
    float pdf = 0.f;
    int matching = 0;
    for (int i = 0; i < b->n; ++i)
        if (lobe_matches(&b->lb[i], flags)) { ++matching; pdf += lobe_pdf(&b->lb[i], wo, wi); }
    return matching > 0 ? pdf / matching : 0.f;
}
/* BSDF::Sample_f (reflection.cpp:747-812); *sampled = the sampled BxDFType */
static RGB bsdf_sample_f(const BSDF* b, V3 woW, V3* wiW, const float* u, float* pdf, int flags, int* sampled) {
    int matchingComps = bsdf_num(b, flags);
    if (matchingComps == 0) { *pdf = 0; *sampled = 0; return rgb1(0); }
    int comp = (int)floorf(u[0] * matchingComps);
    if (comp > matchingComps - 1) comp = matchingComps - 1;
    const Lobe* bx = NULL;
    int count = comp;
    for (int i = 0; i < b->n; ++i)
        if (lobe_matches(&b->lb[i], flags) && count-- == 0) { bx = &b->lb[i]; break; }
    float ur[2] = {fmins(u[0] * matchingComps - comp, ONE_MINUS_EPS), u[1]};
    V3 wo = w2l(b, woW), wi = v3(0, 0, 0);
    if (wo.z == 0) { *sampled = 0; return rgb1(0); }
    *pdf = 0;
    *sampled = bx->type;
    RGB f = lobe_sample(bx, wo, &wi, ur, pdf, sampled);
    if (*pdf == 0) { *sampled = 0; return rgb1(0); }
    *wiW = l2w(b, wi);
    if (!(bx->type & BX_SPECULAR) && matchingComps > 1)
        for (int i = 0; i < b->n; ++i)
            if (&b->lb[i] != bx && lobe_matches(&b->lb[i], flags)) *pdf += lobe_pdf(&b->lb[i], wo, wi);
    if (matchingComps > 1) *pdf /= matchingComps;
    if (!(bx->type & BX_SPECULAR)) {
        int reflect = vdot(*wiW, b->ng) * vdot(woW, b->ng) > 0;
        f = rgb1(0.);
        for (int i = 0; i < b->n; ++i) {
            const Lobe* l = &b->lb[i];
            if (lobe_matches(l, flags) && ((reflect && (l->type & BX_REFLECTION)) || (!reflect && (l->type & BX_TRANSMISSION))))
                f = sadd(f, lobe_f(l, wo, wi));
        }
    }
    return f;
}

/* ------------------------------------------------------------------------ */
/* Lights                                                                    */
/* ------------------------------------------------------------------------ */
static RGB area_L(const pt_light* l, V3 n, V3 w) { /* diffuse.h:58-60 */
    return (l->two_sided || vdot(n, w) > 0) ? rgbv(l->L) : rgb1(0);
}
/* SurfaceInteraction::Le (interaction.cpp:148-151) */
static int si_light(const Scene* sc, const SI* si) {
    int kind = sc->prim_kind[si->prim], idx = sc->prim_index[si->prim];
    if (kind == PT_PRIM_TRIANGLE) return sc->d->triangles[idx].area_light;
    if (kind == PT_PRIM_SPHERE) return sc->d->spheres[idx].area_light;
    return sc->d->planes[idx].area_light;
}
static RGB si_Le(const Scene* sc, const SI* si, V3 w) {
    int li = si_light(sc, si);
    if (li < 0) return rgb1(0);
    return area_L(&sc->d->lights[li], si->n, w);
}
static int si_material(const Scene* sc, const SI* si) {
    int kind = sc->prim_kind[si->prim], idx = sc->prim_index[si->prim];
    if (kind == PT_PRIM_TRIANGLE) return sc->d->triangles[idx].material;
    if (kind == PT_PRIM_SPHERE) return sc->d->spheres[idx].material;
    return sc->d->planes[idx].material;
}

/* ------------------------------------------------------------------------ */
/* InfiniteAreaLight with a constant 1x1 Lmap (lights/infinite.cpp:43-132)    */
/* ------------------------------------------------------------------------ */
typedef struct Inf {
    RGB L;                      /* the Lmap texel: L * scale */
    XF l2w;                     /* LightToWorld (WorldToLight = its inverse) */
    V3 center;                  /* Preprocess: WorldBound().BoundingSphere */
    float radius;
    /* Distribution2D over the 2x2 sinTheta-weighted luminance image */
    float cfunc[2][2], ccdf[2][3], cint[2];
    float mfunc[2], mcdf[3], mint;
} Inf;

/* MIPMap::triangle at level 0 of a 1x1 map with ImageWrap::Repeat (mipmap.h:264-274) */
static RGB lmap_triangle(RGB v, float st0, float st1) {
    float s = st0 * 1 - 0.5f, t = st1 * 1 - 0.5f;
    int s0 = (int)floorf(s), t0 = (int)floorf(t);
    float ds = s - s0, dt = t - t0;
    RGB r = smulf(v, (1 - ds) * (1 - dt));
    r = sadd(r, smulf(v, (1 - ds) * dt));
    r = sadd(r, smulf(v, ds * (1 - dt)));
    r = sadd(r, smulf(v, ds * dt));
    return r;
}
/* MIPMap::Lookup(st, width) (mipmap.h:245-261): every width < 1 is level < 0 here */
static RGB lmap_lookup(const Inf* I, float st0, float st1) { return lmap_triangle(I->L, st0, st1); }

static float spherical_theta(V3 v) { return acosf(clampf11(v.z)); }          /* geometry.h:1636-1638 */
static float spherical_phi(V3 v) {                                           /* geometry.h:1640-1643 */
    float p = atan2f(v.y, v.x);
    return (p < 0) ? (p + 2 * PI_F) : p;
}
#define INV2PI_F 0.15915494309189533577f /* pbrt.h */

/* Distribution1D::SampleContinuous (sampling.h:71-89) */
static float dist1d_sample_cont(const float* func, const float* cdf, float funcInt, int n, float u, float* pdf,
                                int* off) {
    int offset = find_interval_cdf(cdf, n + 1, u);
    if (off) *off = offset;
    float du = u - cdf[offset];
    if ((cdf[offset + 1] - cdf[offset]) > 0) du /= (cdf[offset + 1] - cdf[offset]);
    if (pdf) *pdf = (funcInt > 0) ? func[offset] / funcInt : 0;
    return (offset + du) / n;
}

/* InfiniteAreaLight ctor (sampling image + Distribution2D) and Preprocess */
static void inf_init(Scene* sc, int li) {
    const pt_light* l = &sc->d->lights[li];
    Inf* I = &sc->inf[li];
    I->L = rgbv(l->L);
    I->l2w = xf_from(&l->light_to_world);
    /* Scene::WorldBound() = BVH root bounds; Bounds3::BoundingSphere (geometry.h:959-962) */
    if (sc->nnodes > 0) {
        V3 pmin = sc->nodes[0].bounds.pmin, pmax = sc->nodes[0].bounds.pmax;
        I->center = vmul(vadd(pmin, pmax), 0.5f);
        int inside = I->center.x >= pmin.x && I->center.x <= pmax.x && I->center.y >= pmin.y &&
                     I->center.y <= pmax.y && I->center.z >= pmin.z && I->center.z <= pmax.z;
        I->radius = inside ? vlen(vsub(I->center, pmax)) : 0;
    } else {
        /* empty Bounds3f: pMin = +max, pMax = -max: center 0, not inside */
        I->center = v3(0, 0, 0);
        I->radius = 0;
    }
    /* img[u + v*width] = Lmap->Lookup((up, vp), fwidth).y() * sin(Pi (v+.5)/height) */
    const int width = 2, height = 2;
    float img[4];
    for (int v = 0; v < height; ++v) {
        float vp = (v + .5f) / (float)height;
        float sinTheta = sinf(PI_F * (v + .5f) / height);
        for (int u = 0; u < width; ++u) {
            float up = (u + .5f) / (float)width;
            img[u + v * width] = sy(lmap_lookup(I, up, vp));
            img[u + v * width] *= sinTheta;
        }
    }
    for (int v = 0; v < height; ++v) {
        for (int u = 0; u < width; ++u) I->cfunc[v][u] = img[v * width + u];
        dist1d_build(I->cfunc[v], width, I->ccdf[v], &I->cint[v]);
        I->mfunc[v] = I->cint[v];
    }
    dist1d_build(I->mfunc, height, I->mcdf, &I->mint);
}
/* InfiniteAreaLight::Le (infinite.cpp:91-95) */
static RGB inf_Le(const Inf* I, V3 d) {
    V3 w = vnorm(xf_vec(&I->l2w.mi, d));
    return lmap_lookup(I, spherical_phi(w) * INV2PI_F, spherical_theta(w) * INVPI_F);
}
/* InfiniteAreaLight::Sample_Li (infinite.cpp:97-121); *sp is the visibility
 * target ref.p + wi * 2 worldRadius (zero error bounds and normal) */
static RGB inf_sample_li(const Inf* I, const SI* ref, const float* u, V3* wi, float* pdf, V3* sp) {
    float pdfs[2];
    int v;
    float d1 = dist1d_sample_cont(I->mfunc, I->mcdf, I->mint, 2, u[1], &pdfs[1], &v);
    float d0 = dist1d_sample_cont(I->cfunc[v], I->ccdf[v], I->cint[v], 2, u[0], &pdfs[0], NULL);
    float mapPdf = pdfs[0] * pdfs[1];
    if (mapPdf == 0) { *pdf = 0; return rgb1(0.f); }
    float theta = d1 * PI_F, phi = d0 * 2 * PI_F;
    float cosTheta = cosf(theta), sinTheta = sinf(theta);
    float sinPhi = sinf(phi), cosPhi = cosf(phi);
    *wi = xf_vec(&I->l2w.m, v3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta));
    *pdf = mapPdf / (2 * PI_F * PI_F * sinTheta);
    if (sinTheta == 0) *pdf = 0;
    *sp = vadd(ref->p, vmul(*wi, 2 * I->radius));
    return lmap_lookup(I, d0, d1);
}
/* InfiniteAreaLight::Pdf_Li (infinite.cpp:123-131) + Distribution2D::Pdf (sampling.h:136-142) */
static float inf_pdf_li(const Inf* I, V3 w) {
    V3 wi = xf_vec(&I->l2w.mi, w);
    float theta = spherical_theta(wi), phi = spherical_phi(wi);
    float sinTheta = sinf(theta);
    if (sinTheta == 0) return 0;
    float p0 = phi * INV2PI_F, p1 = theta * INVPI_F;
    int iu = (int)(p0 * 2), iv = (int)(p1 * 2);
    iu = iu < 0 ? 0 : (iu > 1 ? 1 : iu);
    iv = iv < 0 ? 0 : (iv > 1 ? 1 : iv);
    return (I->cfunc[iv][iu] / I->mint) / (2 * PI_F * PI_F * sinTheta);
}

/* DiffuseAreaLight::Sample_Li (diffuse.cpp:69-84) + Shape::Sample(ref,u,pdf) (shape.cpp:56-74) */
static RGB area_sample_li(const Scene* sc, const pt_light* l, const SI* ref, const float* u, V3* wi, float* pdf,
                          V3* sp, V3* sn, V3* spErr) {
    V3 p, n, pe;
    if (l->kind == PT_LIGHT_INFINITE) {
        *sn = v3(0, 0, 0);
        *spErr = v3(0, 0, 0);
        return inf_sample_li(&sc->inf[l - sc->d->lights], ref, u, wi, pdf, sp);
    }
    if (l->kind == PT_LIGHT_POINT) { /* PointLight::Sample_Li (point.cpp:41-49) */
        V3 pl = xf_pt(&sc->light_xf[l - sc->d->lights].m, v3(0, 0, 0));
        *wi = vnorm(vsub(pl, ref->p));
        *pdf = 1.f;
        *sp = pl; *sn = v3(0, 0, 0); *spErr = v3(0, 0, 0);
        return sdivf(rgbv(l->L), dist2(pl, ref->p));
    }
    if (l->kind == PT_LIGHT_DIFFUSE_SPHERE) { /* Sphere::Sample(ref, u, pdf) override */
        sphere_sample_ref(&sc->spheres[l->shape], ref, u, &p, &n, &pe, pdf);
        if (*pdf == 0 || vlen2(vsub(p, ref->p)) == 0) { *pdf = 0; return rgb1(0); }
        *wi = vnorm(vsub(p, ref->p));
        *sp = p; *sn = n; *spErr = pe;
        return area_L(l, n, vneg(*wi));
    }
    if (l->kind == PT_LIGHT_DIFFUSE_AREA) tri_sample(sc, l->shape, u, &p, &n, &pe, pdf);
    else plane_sample(&sc->planes[l->shape], u, &p, &n, &pe, pdf);
    V3 w = vsub(p, ref->p);
    if (vlen2(w) == 0) *pdf = 0;
    else {
        w = vnorm(w);
        *pdf *= dist2(ref->p, p) / vabsdot(n, vneg(w));
        if (isinf(*pdf)) *pdf = 0.f;
    }
    if (*pdf == 0 || vlen2(vsub(p, ref->p)) == 0) { *pdf = 0; return rgb1(0); }
    *wi = vnorm(vsub(p, ref->p));
    *sp = p; *sn = n; *spErr = pe;
    return area_L(l, n, vneg(*wi));
}

/* Shape::Pdf(ref, wi) (shape.cpp:76-91) for a triangle light */
static float area_pdf_li(const Scene* sc, const pt_light* l, const SI* ref, V3 wi) {
    if (l->kind == PT_LIGHT_INFINITE) return inf_pdf_li(&sc->inf[l - sc->d->lights], wi);
    Ray r = spawn_ray(ref->p, ref->pError, ref->n, wi);
    SI isl;
    float tHit;
    int ok;
    float area;
    if (l->kind == PT_LIGHT_DIFFUSE_SPHERE) { /* Sphere::Pdf (sphere.cpp:303-315) */
        const Sphere* s = &sc->spheres[l->shape];
        V3 pOrigin = offset_ray_origin(ref->p, ref->pError, ref->n, vsub(s->center, ref->p));
        if (!(dist2(pOrigin, s->center) <= s->radius * s->radius)) {
            float sinThetaMax2 = s->radius * s->radius / dist2(ref->p, s->center);
            float cosThetaMax = sqrtf(fmaxs(0, 1 - sinThetaMax2));
            return 1 / (2 * PI_F * (1 - cosThetaMax)); /* UniformConePdf (sampling.cpp:132-134) */
        }
        ok = sphere_intersect(s, &r, &tHit, &isl);
        area = s->area;
    } else if (l->kind == PT_LIGHT_DIFFUSE_AREA) {
        ok = tri_intersect(sc->d, l->shape, &r, &tHit, &isl, 1);
        area = sc->tri_area[l->shape];
    } else {
        ok = plane_intersect(&sc->planes[l->shape], &r, &tHit, &isl);
        area = sc->planes[l->shape].area;
    }
    if (!ok) return 0;
    float pdf = dist2(ref->p, isl.p) / (vabsdot(isl.n, vneg(wi)) * area);
    if (isinf(pdf)) pdf = 0.f;
    return pdf;
}

/* EstimateDirect, standard MIS branch (integrator.cpp:124-258), specular=false,
 * handleMedia=false, non-delta area light. */
static RGB estimate_direct_mis(const Scene* sc, const SI* it, const BSDF* bsdf, const float* uScattering,
                               int lightIdx, const float* uLight, Counters* ctr) {
    const pt_light* l = &sc->d->lights[lightIdx];
    RGB Ld = rgb1(0);
    float lightWeight = 0, scatteringWeight = 0;
    V3 wi;
    float lightPdf = 0, scatteringPdf = 0;
    V3 sp, sn, spe;
    RGB Li = area_sample_li(sc, l, it, uLight, &wi, &lightPdf, &sp, &sn, &spe);
    if (lightPdf > 0 && !sblack(Li)) {
        RGB f = smulf(bsdf_f(bsdf, it->wo, wi, BX_ALL & ~BX_SPECULAR), vabsdot(wi, it->sn));
        scatteringPdf = bsdf_pdf(bsdf, it->wo, wi, BX_ALL & ~BX_SPECULAR);
        if (!sblack(f)) {
            /* VisibilityTester::Unoccluded -> SpawnRayTo(Interaction) (light.cpp:59-61, interaction.h:75-80) */
            V3 origin = offset_ray_origin(it->p, it->pError, it->n, vsub(sp, it->p));
            V3 target = offset_ray_origin(sp, spe, sn, vsub(origin, sp));
            Ray sr = {origin, vsub(target, origin), 1 - SHADOW_EPS};
            if (scene_intersect_p(sc, &sr, ctr)) Li = rgb1(0);
            if (!sblack(Li)) {
                if (l->kind == PT_LIGHT_POINT) { /* IsDeltaLight (integrator.cpp:186-188) */
                    Ld = sadd(Ld, sdivf(smul(f, Li), lightPdf));
                } else {
                    lightWeight = power_heuristic(lightPdf, scatteringPdf);
                    Ld = sadd(Ld, sdivf(smulf(smul(f, Li), lightWeight), lightPdf));
                }
            }
        }
    }
    if (l->kind != PT_LIGHT_POINT) {
        int sampledType = 0;
        RGB f = bsdf_sample_f(bsdf, it->wo, &wi, uScattering, &scatteringPdf, BX_ALL & ~BX_SPECULAR, &sampledType);
        f = smulf(f, vabsdot(wi, it->sn));
        if (!sblack(f) && scatteringPdf > 0) {
            scatteringWeight = 1;
            lightPdf = area_pdf_li(sc, l, it, wi);
            if (lightPdf == 0) return Ld;
            scatteringWeight = power_heuristic(scatteringPdf, lightPdf);
            SI lis;
            Ray r = spawn_ray(it->p, it->pError, it->n, wi);
            int found = scene_intersect(sc, &r, &lis, ctr);
            RGB Li2 = rgb1(0);
            if (found) {
                if (si_light(sc, &lis) == lightIdx) Li2 = si_Le(sc, &lis, vneg(wi));
            } else if (l->kind == PT_LIGHT_INFINITE) {
                Li2 = inf_Le(&sc->inf[lightIdx], r.d); /* light.Le(ray) */
            }
            if (!sblack(Li2)) {
                Ld = sadd(Ld, sdivf(smulf(smul(smul(f, Li2), rgb1(1)), scatteringWeight), scatteringPdf));
            }
        }
    }
    return Ld;
}

/* PortalArealight::EstimateDirect (portal_arealight.cpp:29-239).  u1 is
 * uScattering and u2 (uLight) is unused, per the argument order at
 * integrator.cpp:132.  selectedPortal is call-local (the reference's shared
 * member is a data race; its serial behaviour is this one). */
static RGB estimate_direct_portal(const Scene* sc, const SI* it, const BSDF* bsdf, const float* u1,
                                  int lightIdx, Counters* ctr) {
    const pt_light* l = &sc->d->lights[lightIdx];
    const Plane* lp = &sc->planes[l->shape];
    RGB Ld = rgb1(0);
    if (l->strategy != PT_PORTAL_LIGHT) {
        int np = l->n_portals;
        float dist[64];
        float sum = 0;
        int behindAll = 1;
        V3 pObj = xf_pt(&lp->w2o.m, it->p);
        for (int i = 0; i < np; i++) {
            const Plane* pp = &sc->portal_planes[l->first_portal + i];
            if (!plane_in_front(pp, pObj)) { dist[i] = 0; continue; }
            behindAll = 0;
            /* InFrustum() returns true (aaportal.cpp:101-104) */
            dist[i] = 1;
            sum += dist[i];
        }
        if (!behindAll) {
            if (sum == 0) return rgb1(0);
            for (int i = 0; i < np; i++) dist[i] /= sum;
            float cdf[65], funcInt, portalPdf;
            dist1d_build(dist, np, cdf, &funcInt);
            int sel = dist1d_sample_discrete(dist, cdf, funcInt, np, u1[0], &portalPdf);
            const Plane* pp = &sc->portal_planes[l->first_portal + sel];
            if (plane_in_front(pp, pObj)) {
                V3 wi;
                float pdf = 0;
                if (l->strategy == PT_PORTAL_UNIFORM) {
                    /* EstimateDirectPortal (158-198) + AAPortal::SamplePortal (aaportal.cpp:73-83) */
                    V3 sp, sn, spe;
                    float areaPdf;
                    plane_sample(pp, u1, &sp, &sn, &spe, &areaPdf);
                    wi = vnorm(vsub(sp, it->p));
                    pdf = dist2(it->p, sp) / (vabsdot(plane_normal(pp), vneg(wi)) * pp->area);
                } else {
                    /* EstimateDirectProj (200-239) + AAPortal::SampleProj (aaportal.cpp:114-159) */
                    V3 dLo = vnorm(vsub(it->p, lp->lo));
                    V3 dHi = vnorm(vsub(it->p, lp->hi));
                    if (dLo.z == 0 || dHi.z == 0) pdf = 0;
                    else {
                        float tLo = (vidx(pp->lo, pp->ax) - vidx(lp->lo, lp->ax)) / vidx(dLo, lp->ax);
                        float tHi = (vidx(pp->lo, pp->ax) - vidx(lp->hi, lp->ax)) / vidx(dHi, lp->ax);
                        V3 projLo = vadd(lp->lo, vmul(dLo, tLo));
                        V3 projHi = vadd(lp->hi, vmul(dHi, tHi));
                        V3 isectHi = vmax(pp->lo, projLo);
                        V3 isectLo = vmin(pp->hi, projHi);
                        float len0 = vidx(isectHi, pp->ax0) - vidx(isectLo, pp->ax0);
                        float len1 = vidx(isectHi, pp->ax1) - vidx(isectLo, pp->ax1);
                        V3 sampled = v3(0, 0, 0);
                        vset(&sampled, pp->ax, vidx(pp->lo, pp->ax));
                        vset(&sampled, pp->ax0, vidx(isectLo, pp->ax0) + u1[0] * len0);
                        vset(&sampled, pp->ax1, vidx(isectLo, pp->ax1) + u1[0] * len1);
                        V3 sampledWorld = xf_pt(&pp->w2o.m, sampled);
                        wi = vsub(sampledWorld, it->p);
                        pdf = dist2(it->p, sampled) / (vabsdot(plane_normal(pp), vneg(wi)) * (len0 * len1));
                    }
                }
                if (pdf > 0) {
                    RGB Li = rgb1(0);
                    SI lis;
                    Ray r = spawn_ray(it->p, it->pError, it->n, wi);
                    if (scene_intersect(sc, &r, &lis, ctr)) Li = si_Le(sc, &lis, vneg(wi));
                    RGB f = smulf(bsdf_f(bsdf, it->wo, wi, BX_ALL & ~BX_SPECULAR), vabsdot(wi, it->sn));
                    if (!sblack(f) && !sblack(Li)) Ld = sadd(Ld, sdivf(smul(f, Li), pdf));
                }
                if (l->strategy == PT_PORTAL_PROJECTION) Ld = sdivf(Ld, portalPdf);
                return Ld;
            }
        }
    }
    /* EstimateDirectLight (115-156) */
    {
        V3 wi;
        float pdf = 0;
        V3 sp, sn, spe;
        RGB Li = area_sample_li(sc, l, it, u1, &wi, &pdf, &sp, &sn, &spe);
        if (!sblack(Li) && pdf > 0) {
            SI lis;
            Ray r = spawn_ray(it->p, it->pError, it->n, wi);
            if (scene_intersect(sc, &r, &lis, ctr)) Li = si_Le(sc, &lis, vneg(wi));
            RGB f = smulf(bsdf_f(bsdf, it->wo, wi, BX_ALL & ~BX_SPECULAR), vabsdot(wi, it->sn));
            if (!sblack(f) && !sblack(Li)) Ld = sadd(Ld, sdivf(smul(f, Li), pdf));
        }
    }
    return Ld;
}

/* ------------------------------------------------------------------------ */
/* PathIntegrator::Li (path.cpp:64-189)                                      */
/* ------------------------------------------------------------------------ */
static RGB path_li(const Scene* sc, Ray ray, float wvl0, Samp* smp, Counters* ctr) {
    RGB L = rgb1(0), beta = rgb1(1);
    int specularBounce = 0;
    int bounces;
    float etaScale = 1;
    const int nLights = sc->nlights;
    for (bounces = 0;; ++bounces) {
        SI isect;
        int found = scene_intersect(sc, &ray, &isect, ctr);
        if (bounces == 0 || specularBounce) {
            if (found) L = sadd(L, smul(beta, si_Le(sc, &isect, vneg(ray.d))));
            else
                for (int li = 0; li < sc->d->n_lights; ++li) /* scene.infiniteLights, in light order */
                    if (sc->d->lights[li].kind == PT_LIGHT_INFINITE)
                        L = sadd(L, smul(beta, inf_Le(&sc->inf[li], ray.d)));
        }
        if (!found || bounces >= sc->max_depth) break;
        int mi = si_material(sc, &isect);
        const pt_material* mat = (mi >= 0) ? &sc->d->materials[mi] : NULL;
        if (!mat || mat->kind == PT_MAT_NONE) {
            ray = spawn_ray(isect.p, isect.pError, isect.n, ray.d);
            bounces--;
            continue;
        }
        BSDF bsdf;
        make_bsdf(mat, &isect, wvl0, 1, &bsdf);
        if (bsdf_num(&bsdf, BX_ALL & ~BX_SPECULAR) > 0) {
            /* UniformSampleOneLight (integrator.cpp:100-122) */
            RGB Ld = rgb1(0);
            if (nLights > 0) {
                float lightPdf;
                float ul = get1d(smp);
                int lightNum = dist1d_sample_discrete(sc->ldist_func, sc->ldist_cdf, sc->ldist_int, nLights, ul, &lightPdf);
                if (lightPdf != 0) {
                    float uLight[2], uScattering[2];
                    get2d(smp, uLight);
                    get2d(smp, uScattering);
                    RGB e;
                    if (sc->d->lights[lightNum].kind == PT_LIGHT_PORTAL_AREA)
                        e = estimate_direct_portal(sc, &isect, &bsdf, uScattering, lightNum, ctr);
                    else
                        e = estimate_direct_mis(sc, &isect, &bsdf, uScattering, lightNum, uLight, ctr);
                    Ld = sdivf(e, lightPdf);
                }
            }
            L = sadd(L, smul(beta, Ld));
        }
        V3 wo = vneg(ray.d), wi = v3(0, 0, 0);
        float pdf = 0;
        int sampled = 0;
        float u[2];
        get2d(smp, u);
        RGB f = bsdf_sample_f(&bsdf, wo, &wi, u, &pdf, BX_ALL, &sampled);
        if (sblack(f) || pdf == 0.f) break;
        beta = smul(beta, sdivf(smulf(f, vabsdot(wi, isect.sn)), pdf));
        specularBounce = (sampled & BX_SPECULAR) != 0;
        if ((sampled & BX_SPECULAR) && (sampled & BX_TRANSMISSION)) {
            float eta = bsdf.eta;
            etaScale *= (vdot(wo, isect.n) > 0) ? (eta * eta) : 1 / (eta * eta);
        }
        ray = spawn_ray(isect.p, isect.pError, isect.n, wi);
        RGB rrBeta = smulf(beta, etaScale);
        if (smaxc(rrBeta) < sc->rr_threshold && bounces > 3) {
            float q = fmaxs((float).05, 1 - smaxc(rrBeta));
            if (get1d(smp) < q) break;
            beta = sdivf(beta, 1 - q);
        }
    }
    return L;
}

/* ------------------------------------------------------------------------ */
/* Camera (cameras/perspective.cpp:100-154, camera.h ProjectiveCamera)       */
/* ------------------------------------------------------------------------ */
static void camera_init(Scene* sc) {
    const pt_camera_desc* c = &sc->d->camera;
    const pt_film_desc* f = &sc->d->film;
    sc->camera_to_world = m4_from(c->camera_to_world.m);
    XF camToScreen = xf_perspective(c->fov, 1e-2f, 1000.f);
    const float* sw = c->screen_window;
    /* ScreenToRaster = Scale(res) * Scale(1/(x1-x0), 1/(y0-y1), 1) * Translate(-x0, -y1, 0) */
    XF s2r = xf_mul(xf_mul(xf_scale((float)f->xres, (float)f->yres, 1),
                           xf_scale(1 / (sw[1] - sw[0]), 1 / (sw[2] - sw[3]), 1)),
                    xf_translate(-sw[0], -sw[3], 0));
    XF r2s = xf_inv(s2r);
    XF r2c = xf_mul(xf_inv(camToScreen), r2s);
    sc->raster_to_camera = r2c.m;
    sc->lens_radius = c->lens_radius;
    sc->focal_distance = c->focal_distance;
}
static Ray camera_ray(const Scene* sc, float fx, float fy, const float* pLens) {
    V3 pCamera = xf_pt(&sc->raster_to_camera, v3(fx, fy, 0));
    Ray r;
    r.o = v3(0, 0, 0);
    r.d = vnorm(v3(pCamera.x, pCamera.y, pCamera.z));
    r.tMax = INFINITY;
    if (sc->lens_radius > 0) {
        float d2[2];
        concentric_sample_disk(pLens, d2);
        float lx = sc->lens_radius * d2[0], ly = sc->lens_radius * d2[1];
        float ft = sc->focal_distance / r.d.z;
        V3 pFocus = vadd(r.o, vmul(r.d, ft));
        r.o = v3(lx, ly, 0);
        r.d = vnorm(vsub(pFocus, r.o));
    }
    return xf_ray(&sc->camera_to_world, r);
}

/* ------------------------------------------------------------------------ */
/* Film (core/film.{h,cpp})                                                  */
/* ------------------------------------------------------------------------ */
static void film_init(Scene* sc) {
    const pt_film_desc* f = &sc->d->film;
    /* croppedPixelBounds (film.cpp:55-60) */
    sc->crop_x0 = (int)ceilf((float)f->xres * f->crop[0]);
    sc->crop_y0 = (int)ceilf((float)f->yres * f->crop[2]);
    sc->crop_x1 = (int)ceilf((float)f->xres * f->crop[1]);
    sc->crop_y1 = (int)ceilf((float)f->yres * f->crop[3]);
    sc->fr_x = f->filter_radius[0];
    sc->fr_y = f->filter_radius[1];
    /* GetSampleBounds (film.cpp:80-86) */
    sc->sb_x0 = (int)floorf((float)sc->crop_x0 + 0.5f - sc->fr_x);
    sc->sb_y0 = (int)floorf((float)sc->crop_y0 + 0.5f - sc->fr_y);
    sc->sb_x1 = (int)ceilf((float)sc->crop_x1 - 0.5f + sc->fr_x);
    sc->sb_y1 = (int)ceilf((float)sc->crop_y1 - 0.5f + sc->fr_y);
    /* filter table (film.cpp:68-77) */
    int off = 0;
    float expX = 0, expY = 0, alpha = f->gaussian_alpha;
    if (f->filter == PT_FILTER_GAUSSIAN) {
        expX = expf(-alpha * sc->fr_x * sc->fr_x);
        expY = expf(-alpha * sc->fr_y * sc->fr_y);
    }
    for (int y = 0; y < 16; ++y) {
        for (int x = 0; x < 16; ++x, ++off) {
            float px = (x + 0.5f) * sc->fr_x / 16;
            float py = (y + 0.5f) * sc->fr_y / 16;
            if (f->filter == PT_FILTER_GAUSSIAN) {
                float gx = fmaxs((float)0, (float)(expf(-alpha * px * px) - expX));
                float gy = fmaxs((float)0, (float)(expf(-alpha * py * py) - expY));
                sc->filter_table[off] = gx * gy;
            } else {
                sc->filter_table[off] = 1.f;
            }
        }
    }
}

typedef struct { float c[3]; float w; } TPix;
typedef struct {
    int x0, y0, x1, y1; /* tile pixel bounds */
    TPix* px;
} FilmTile;

static void tile_add_sample(const Scene* sc, FilmTile* t, float fx, float fy, RGB L, float sw) { /* film.h:121-161 */
    float maxLum = sc->d->film.max_sample_luminance;
    if (sy(L) > maxLum) L = smulf(L, maxLum / sy(L));
    float dx = fx - 0.5f, dy = fy - 0.5f;
    int p0x = (int)ceilf(dx - sc->fr_x), p0y = (int)ceilf(dy - sc->fr_y);
    int p1x = (int)floorf(dx + sc->fr_x) + 1, p1y = (int)floorf(dy + sc->fr_y) + 1;
    if (p0x < t->x0) p0x = t->x0;
    if (p0y < t->y0) p0y = t->y0;
    if (p1x > t->x1) p1x = t->x1;
    if (p1y > t->y1) p1y = t->y1;
    int ifx[64], ify[64];
    float invrx = 1 / sc->fr_x, invry = 1 / sc->fr_y;
    for (int x = p0x; x < p1x; ++x) {
        float v = fabsf((x - dx) * invrx * 16);
        int i = (int)floorf(v); ifx[x - p0x] = i < 15 ? i : 15;
    }
    for (int y = p0y; y < p1y; ++y) {
        float v = fabsf((y - dy) * invry * 16);
        int i = (int)floorf(v); ify[y - p0y] = i < 15 ? i : 15;
    }
    int w = t->x1 - t->x0;
    for (int y = p0y; y < p1y; ++y)
        for (int x = p0x; x < p1x; ++x) {
            float fw = sc->filter_table[ify[y - p0y] * 16 + ifx[x - p0x]];
            TPix* p = &t->px[(x - t->x0) + (y - t->y0) * w];
            RGB c = smulf(smulf(L, sw), fw);
            p->c[0] += c.c[0]; p->c[1] += c.c[1]; p->c[2] += c.c[2];
            p->w += fw;
        }
}

/* ------------------------------------------------------------------------ */
/* integrators/directlighting.cpp                                           */
/* ------------------------------------------------------------------------ */
static RGB dl_estimate(const Scene* sc, const SI* it, const BSDF* bsdf, const float* uScattering, int lightIdx,
                       const float* uLight, Counters* ctr) { /* EstimateDirect (integrator.cpp:124-135) dispatch */
    if (sc->d->lights[lightIdx].kind == PT_LIGHT_PORTAL_AREA)
        return estimate_direct_portal(sc, it, bsdf, uScattering, lightIdx, ctr);
    return estimate_direct_mis(sc, it, bsdf, uScattering, lightIdx, uLight, ctr);
}
/* UniformSampleAllLights (integrator.cpp:69-98) */
static RGB dl_sample_all(const Scene* sc, const SI* it, const BSDF* bsdf, Samp* smp, Counters* ctr) {
    RGB L = rgb1(0);
    for (int j = 0; j < sc->d->n_lights; ++j) {
        int n = sc->d->lights[j].n_samples;
        float* uLA = (float*)malloc(sizeof(float) * 2 * (size_t)n);
        float* uSA = (float*)malloc(sizeof(float) * 2 * (size_t)n);
        int okL = get2d_array(smp, n, uLA);
        int okS = get2d_array(smp, n, uSA);
        if (!okL || !okS) {
            float uLight[2], uScattering[2];
            get2d(smp, uLight);
            get2d(smp, uScattering);
            L = sadd(L, dl_estimate(sc, it, bsdf, uScattering, j, uLight, ctr));
        } else {
            RGB Ld = rgb1(0);
            for (int k = 0; k < n; ++k) Ld = sadd(Ld, dl_estimate(sc, it, bsdf, uSA + 2 * k, j, uLA + 2 * k, ctr));
            L = sadd(L, sdivf(Ld, (float)n));
        }
        free(uLA); free(uSA);
    }
    return L;
}
/* UniformSampleOneLight without a light distribution (integrator.cpp:100-122) */
static RGB dl_sample_one(const Scene* sc, const SI* it, const BSDF* bsdf, Samp* smp, Counters* ctr) {
    int nLights = sc->d->n_lights;
    if (nLights == 0) return rgb1(0);
    int lightNum = (int)(get1d(smp) * nLights);
    if (lightNum > nLights - 1) lightNum = nLights - 1;
    float lightPdf = (float)1 / nLights;
    float uLight[2], uScattering[2];
    get2d(smp, uLight);
    get2d(smp, uScattering);
    return sdivf(dl_estimate(sc, it, bsdf, uScattering, lightNum, uLight, ctr), lightPdf);
}
static RGB dl_li(const Scene* sc, Ray ray, float wvl0, Samp* smp, int depth, Counters* ctr);
/* SamplerIntegrator::SpecularReflect / SpecularTransmit (integrator.cpp:639-770), no differentials */
static RGB dl_specular(const Scene* sc, const SI* isect, const BSDF* bsdf, int type, float wvl0, Samp* smp, int depth,
                       Counters* ctr) {
    float u[2];
    get2d(smp, u);
    V3 wi = v3(0, 0, 0);
    float pdf = 0;
    int sampled = 0;
    RGB f = bsdf_sample_f(bsdf, isect->wo, &wi, u, &pdf, type | BX_SPECULAR, &sampled);
    if (pdf > 0.f && !sblack(f) && vabsdot(wi, isect->sn) != 0.f) {
        Ray rd = spawn_ray(isect->p, isect->pError, isect->n, wi);
        RGB Li = dl_li(sc, rd, wvl0, smp, depth + 1, ctr);
        return sdivf(smulf(smul(f, Li), vabsdot(wi, isect->sn)), pdf);
    }
    return rgb1(0);
}
/* DirectLightingIntegrator::Li (directlighting.cpp:58-84) */
static RGB dl_li(const Scene* sc, Ray ray, float wvl0, Samp* smp, int depth, Counters* ctr) {
    RGB L = rgb1(0);
    SI isect;
    if (!scene_intersect(sc, &ray, &isect, ctr)) {
        for (int li = 0; li < sc->d->n_lights; ++li) /* Light::Le: only the infinite light emits */
            if (sc->d->lights[li].kind == PT_LIGHT_INFINITE) L = sadd(L, inf_Le(&sc->inf[li], ray.d));
        return L;
    }
    int mi = si_material(sc, &isect);
    const pt_material* mat = (mi >= 0) ? &sc->d->materials[mi] : NULL;
    if (!mat || mat->kind == PT_MAT_NONE)
        return dl_li(sc, spawn_ray(isect.p, isect.pError, isect.n, ray.d), wvl0, smp, depth, ctr);
    BSDF bsdf;
    make_bsdf(mat, &isect, wvl0, 0, &bsdf);
    L = sadd(L, si_Le(sc, &isect, isect.wo));
    if (sc->d->n_lights > 0) {
        if (sc->dl_strategy == PT_DIRECT_ALL) L = sadd(L, dl_sample_all(sc, &isect, &bsdf, smp, ctr));
        else L = sadd(L, dl_sample_one(sc, &isect, &bsdf, smp, ctr));
    }
    if (depth + 1 < sc->max_depth) {
        L = sadd(L, dl_specular(sc, &isect, &bsdf, BX_REFLECTION, wvl0, smp, depth, ctr));
        L = sadd(L, dl_specular(sc, &isect, &bsdf, BX_TRANSMISSION, wvl0, smp, depth, ctr));
    }
    return L;
}

static void render_tile(const Scene* sc, const Halton* h, int tx, int ty, FilmTile* ft, Counters* ctr) {
    const int ts = 16;
    int x0 = sc->sb_x0 + tx * ts, y0 = sc->sb_y0 + ty * ts;
    int x1 = x0 + ts < sc->sb_x1 ? x0 + ts : sc->sb_x1;
    int y1 = y0 + ts < sc->sb_y1 ? y0 + ts : sc->sb_y1;
    /* Film::GetFilmTile (film.cpp:95-106) */
    int px0 = (int)ceilf((float)x0 - 0.5f - sc->fr_x), py0 = (int)ceilf((float)y0 - 0.5f - sc->fr_y);
    int px1 = (int)floorf((float)x1 - 0.5f + sc->fr_x) + 1, py1 = (int)floorf((float)y1 - 0.5f + sc->fr_y) + 1;
    if (px0 < sc->crop_x0) px0 = sc->crop_x0;
    if (py0 < sc->crop_y0) py0 = sc->crop_y0;
    if (px1 > sc->crop_x1) px1 = sc->crop_x1;
    if (py1 > sc->crop_y1) py1 = sc->crop_y1;
    if (px1 < px0) px1 = px0;
    if (py1 < py0) py1 = py0;
    ft->x0 = px0; ft->y0 = py0; ft->x1 = px1; ft->y1 = py1;
    ft->px = (TPix*)calloc((size_t)((px1 - px0) * (py1 - py0) + 1), sizeof(TPix));
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            if (!(x >= sc->pix_x0 && x < sc->pix_x1 && y >= sc->pix_y0 && y < sc->pix_y1)) continue;
            int64_t off = halton_pixel_offset(h, x, y);
            for (int s = sc->s_begin; s < sc->s_end; ++s) {
                Samp smp;
                memset(&smp, 0, sizeof smp);
                smp.h = h; smp.index = off + (int64_t)s * h->stride; smp.dim = 0;
                smp.pixOff = off; smp.s = s;
                smp.n2D = sc->n2D; smp.sizes2D = sc->sizes2D;
                smp.arrayEndDim = ARRAY_START_DIM + 2 * sc->n2D;
                float uf[2], ul[2];
                get2d(&smp, uf);                 /* pFilm */
                float fx = (float)x + uf[0], fy = (float)y + uf[1];
                (void)get1d(&smp);               /* time */
                get2d(&smp, ul);                 /* pLens */
                float uw = get1d(&smp);          /* wvl (fork, sampler.cpp:51) */
                /* Camera::GenerateWvls (camera.cpp:62-76): only wvls[0] is used on the RGB path */
                float wvl0 = (float)400 + (float)300 * uw;
                Ray r = camera_ray(sc, fx, fy, ul);
                ctr->camera++;
                RGB L = sc->integrator == PT_INTEGRATOR_DIRECT ? dl_li(sc, r, wvl0, &smp, 0, ctr)
                                                               : path_li(sc, r, wvl0, &smp, ctr);
                if (smp.overflow) ctr->dim_overflow++;
                /* radiance sanitiser (integrator.cpp:592-613) */
                if (snan(L)) L = rgb1(0);
                else if (sy(L) < -1e-5) L = rgb1(0);
                else if (isinf(sy(L))) L = rgb1(0);
                tile_add_sample(sc, ft, fx, fy, L, 1.f);
            }
        }
}

static void rgb_to_xyz(const float* rgb, float* xyz) { /* spectrum.h:64-68 */
    xyz[0] = 0.412453f * rgb[0] + 0.357580f * rgb[1] + 0.180423f * rgb[2];
    xyz[1] = 0.212671f * rgb[0] + 0.715160f * rgb[1] + 0.072169f * rgb[2];
    xyz[2] = 0.019334f * rgb[0] + 0.119193f * rgb[1] + 0.950227f * rgb[2];
}
static void xyz_to_rgb(const float* xyz, float* rgb) { /* spectrum.h:58-62 */
    rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
}

/* ------------------------------------------------------------------------ */
/* Scene setup / teardown                                                    */
/* ------------------------------------------------------------------------ */
static int scene_setup(Scene* sc, const pt_scene_desc* d) {
    ensure_init();
    memset(sc, 0, sizeof *sc);
    sc->d = d;
    sc->light_xf = (XF*)calloc((size_t)(d->n_lights + 1), sizeof(XF));
    for (int i = 0; i < d->n_lights; ++i) {
        memcpy(sc->light_xf[i].m.m, d->lights[i].light_to_world.m, 64);
        memcpy(sc->light_xf[i].mi.m, d->lights[i].light_to_world.minv, 64);
    }
    sc->spheres = (Sphere*)calloc((size_t)(d->n_spheres + 1), sizeof(Sphere));
    for (int i = 0; i < d->n_spheres; ++i) sphere_init(&sc->spheres[i], &d->spheres[i]);
    sc->planes = (Plane*)calloc((size_t)(d->n_planes + 1), sizeof(Plane));
    for (int i = 0; i < d->n_planes; ++i) {
        const pt_aaplane* p = &d->planes[i];
        plane_init(&sc->planes[i], v3(p->lo[0], p->lo[1], p->lo[2]), v3(p->hi[0], p->hi[1], p->hi[2]), p->axis,
                   (p->flags & PT_TRI_REVERSE_ORIENTATION) != 0, (p->flags & PT_TRI_SWAPS_HANDEDNESS) != 0,
                   xf_from(&p->object_to_world));
    }
    sc->tri_area = (float*)calloc((size_t)(d->n_triangles + 1), sizeof(float));
    for (int i = 0; i < d->n_triangles; ++i) sc->tri_area[i] = tri_area(d, i);
    /* AAPortal::portal = AAPlaneShape(light transforms, !facingFw, lo, hi, axis) (aaportal.cpp:8-13) */
    sc->portal_planes = (Plane*)calloc((size_t)(d->n_portals + 1), sizeof(Plane));
    for (int li = 0; li < d->n_lights; ++li) {
        const pt_light* l = &d->lights[li];
        if (l->kind != PT_LIGHT_PORTAL_AREA) continue;
        const pt_aaplane* lp = &d->planes[l->shape];
        for (int k = 0; k < l->n_portals; ++k) {
            const pt_portal* po = &d->portals[l->first_portal + k];
            plane_init(&sc->portal_planes[l->first_portal + k], v3(po->lo[0], po->lo[1], po->lo[2]),
                       v3(po->hi[0], po->hi[1], po->hi[2]), po->axis, !po->facing_fw,
                       (lp->flags & PT_TRI_SWAPS_HANDEDNESS) != 0, xf_from(&lp->object_to_world));
        }
    }
    build_bvh(sc);
    sc->inf = (struct Inf*)calloc((size_t)(d->n_lights + 1), sizeof(Inf));
    for (int i = 0; i < d->n_lights; ++i)
        if (d->lights[i].kind == PT_LIGHT_INFINITE) inf_init(sc, i);
    /* light distribution: "uniform" (lightdistrib.cpp:68-75) or "power" (integrator.cpp:515-522) */
    sc->nlights = d->n_lights;
    sc->ldist_func = (float*)calloc((size_t)(d->n_lights + 1), sizeof(float));
    sc->ldist_cdf = (float*)calloc((size_t)(d->n_lights + 2), sizeof(float));
    for (int i = 0; i < d->n_lights; ++i) {
        if (d->integrator.light_strategy == PT_LIGHTS_POWER && d->n_lights > 1) { /* lightdistrib.cpp:47-50 */
            const pt_light* l = &d->lights[i];
            if (l->kind == PT_LIGHT_INFINITE) {
                /* InfiniteAreaLight::Power() = Pi r^2 Lmap->Lookup((.5,.5), .5) (infinite.cpp:85-89) */
                const Inf* I = &sc->inf[i];
                sc->ldist_func[i] = sy(smulf(lmap_lookup(I, .5f, .5f), PI_F * I->radius * I->radius));
                continue;
            }
            if (l->kind == PT_LIGHT_POINT) { /* PointLight::Power = 4 Pi I (point.cpp:51) */
                sc->ldist_func[i] = sy(smulf(rgbv(l->L), 4 * PI_F));
                continue;
            }
            float area = l->kind == PT_LIGHT_DIFFUSE_AREA     ? sc->tri_area[l->shape]
                         : l->kind == PT_LIGHT_DIFFUSE_SPHERE ? sc->spheres[l->shape].area
                                                               : sc->planes[l->shape].area;
            /* DiffuseAreaLight::Power() = (twoSided ? 2 : 1) * Lemit * area * Pi (diffuse.cpp:62-64) */
            RGB pw = smulf(smulf(smulf(rgbv(l->L), (float)(l->two_sided ? 2 : 1)), area), PI_F);
            sc->ldist_func[i] = sy(pw);
        } else sc->ldist_func[i] = 1;
    }
    if (d->n_lights > 0) dist1d_build(sc->ldist_func, d->n_lights, sc->ldist_cdf, &sc->ldist_int);
    camera_init(sc);
    film_init(sc);
    sc->spp = d->sampler.spp;
    sc->s_begin = 0;
    sc->s_end = d->sampler.spp;
    sc->max_depth = d->integrator.max_depth;
    sc->integrator = d->integrator.kind;
    sc->dl_strategy = d->integrator.direct_strategy;
    sc->n2D = 0;
    sc->sizes2D = NULL;
    if (sc->integrator == PT_INTEGRATOR_DIRECT && sc->dl_strategy == PT_DIRECT_ALL && d->n_lights > 0) {
        /* DirectLightingIntegrator::Preprocess (directlighting.cpp:43-56): per depth, per
         * light, two arrays of RoundCount(nSamples) = nSamples (GlobalSampler) */
        sc->n2D = 2 * d->n_lights * sc->max_depth;
        sc->sizes2D = (int*)malloc(sizeof(int) * (size_t)(sc->n2D + 1));
        for (int i = 0; i < sc->n2D; ++i) sc->sizes2D[i] = d->lights[(i / 2) % d->n_lights].n_samples;
    }
    sc->rr_threshold = d->integrator.rr_threshold;
    sc->pix_x0 = sc->sb_x0; sc->pix_y0 = sc->sb_y0; sc->pix_x1 = sc->sb_x1; sc->pix_y1 = sc->sb_y1;
    if (d->integrator.has_pixel_bounds) {
        /* Intersect(pixelBounds, Bounds2i{{pb0,pb2},{pb1,pb3}}) (path.cpp:196-207) */
        const int* pb = d->integrator.pixel_bounds;
        int bx0 = pb[0] < pb[1] ? pb[0] : pb[1], bx1 = pb[0] < pb[1] ? pb[1] : pb[0];
        int by0 = pb[2] < pb[3] ? pb[2] : pb[3], by1 = pb[2] < pb[3] ? pb[3] : pb[2];
        if (bx0 > sc->pix_x0) sc->pix_x0 = bx0;
        if (by0 > sc->pix_y0) sc->pix_y0 = by0;
        if (bx1 < sc->pix_x1) sc->pix_x1 = bx1;
        if (by1 < sc->pix_y1) sc->pix_y1 = by1;
    }
    return 0;
}
static void scene_free(Scene* sc) {
    free(sc->planes); free(sc->spheres); free(sc->light_xf); free(sc->sizes2D); free(sc->tri_area); free(sc->portal_planes);
    free(sc->prim_kind); free(sc->prim_index); free(sc->nodes);
    free(sc->ldist_func); free(sc->ldist_cdf); free(sc->inf);
}

typedef struct {
    const Scene* sc;
    const Halton* h;
    FilmTile* tiles;
    int ntx, ntiles;
    int next;
    int toff, tstride;
    pthread_mutex_t mu;
    Counters total;
} Pool;

static void* worker(void* arg) {
    Pool* p = (Pool*)arg;
    Counters c = {0, 0, 0, 0, 0};
    for (;;) {
        pthread_mutex_lock(&p->mu);
        int t = p->next++;
        pthread_mutex_unlock(&p->mu);
        if (t >= p->ntiles) break;
        if (t % p->tstride != p->toff) { p->tiles[t].px = NULL; continue; }
        render_tile(p->sc, p->h, t % p->ntx, t / p->ntx, &p->tiles[t], &c);
    }
    pthread_mutex_lock(&p->mu);
    p->total.closest += c.closest; p->total.shadow += c.shadow; p->total.nodes += c.nodes;
    p->total.prims += c.prims; p->total.camera += c.camera; p->total.dim_overflow += c.dim_overflow;
    pthread_mutex_unlock(&p->mu);
    return NULL;
}

/* Renders tiles; forms the per-pixel film XYZ + weight by Film::MergeFilmTile
 * in tile order (film.cpp:117-130), optionally returned as accum_out, and
 * optionally the resolved RGB image. */
static int render_common(const pt_scene_desc* desc, float* rgb_out, float* accum_out, int nthreads, int max_tiles,
                         int tile_offset, int tile_stride, int s_begin, int s_end, oracle_stats* stats) {
    Scene sc;
    if (!desc) return 1;
    scene_setup(&sc, desc);
    if (s_end >= 0) { sc.s_begin = s_begin; sc.s_end = s_end; }
    Halton h;
    halton_init(&h, sc.sb_x0, sc.sb_y0, sc.sb_x1, sc.sb_y1, desc->sampler.sample_pixel_center);
    int ex = sc.sb_x1 - sc.sb_x0, ey = sc.sb_y1 - sc.sb_y0;
    int ntx = (ex + 15) / 16, nty = (ey + 15) / 16;
    int ntiles = ntx * nty;
    if (max_tiles >= 0 && max_tiles < ntiles) ntiles = max_tiles;
    Pool pool;
    memset(&pool, 0, sizeof pool);
    pool.sc = &sc; pool.h = &h; pool.ntx = ntx; pool.ntiles = ntiles; pool.next = 0;
    pool.toff = tile_offset; pool.tstride = tile_stride > 0 ? tile_stride : 1;
    pool.tiles = (FilmTile*)calloc((size_t)(ntiles + 1), sizeof(FilmTile));
    pthread_mutex_init(&pool.mu, NULL);
    if (nthreads <= 1) worker(&pool);
    else {
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
        for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, worker, &pool);
        for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
        free(th);
    }
    int cw = sc.crop_x1 - sc.crop_x0, ch = sc.crop_y1 - sc.crop_y0;
    size_t npix = (size_t)(cw > 0 ? cw : 0) * (size_t)(ch > 0 ? ch : 0);
    float* xyz = (float*)calloc(npix * 4 + 4, sizeof(float));
    if (accum_out) memset(accum_out, 0, sizeof(float) * 4 * npix);
    for (int t = 0; t < ntiles; ++t) {
        FilmTile* ft = &pool.tiles[t];
        if (!ft->px) continue;
        int w = ft->x1 - ft->x0;
        for (int y = ft->y0; y < ft->y1; ++y)
            for (int x = ft->x0; x < ft->x1; ++x) {
                TPix* tp = &ft->px[(x - ft->x0) + (y - ft->y0) * w];
                size_t o = (size_t)(x - sc.crop_x0) + (size_t)(y - sc.crop_y0) * (size_t)cw;
                float x3[3];
                rgb_to_xyz(tp->c, x3);
                for (int i = 0; i < 3; ++i) xyz[4 * o + i] += x3[i];
                xyz[4 * o + 3] += tp->w;
                if (accum_out) {
                    for (int i = 0; i < 3; ++i) accum_out[4 * o + i] += x3[i];
                    accum_out[4 * o + 3] += tp->w;
                }
            }
        free(ft->px);
    }
    if (rgb_out) {
        /* Film::WriteImage (film.cpp:169-211), splatScale = 1, no splats */
        float scale = desc->film.scale;
        for (size_t o = 0; o < npix; ++o) {
            float rgb[3];
            xyz_to_rgb(&xyz[4 * o], rgb);
            float ws = xyz[4 * o + 3];
            if (ws != 0) {
                float invWt = (float)1 / ws;
                rgb[0] = fmaxs((float)0, rgb[0] * invWt);
                rgb[1] = fmaxs((float)0, rgb[1] * invWt);
                rgb[2] = fmaxs((float)0, rgb[2] * invWt);
            }
            float splat[3] = {0, 0, 0}, srgb[3];
            xyz_to_rgb(splat, srgb);
            for (int i = 0; i < 3; ++i) { rgb[i] += 1.f * srgb[i]; rgb[i] *= scale; }
            rgb_out[3 * o] = rgb[0]; rgb_out[3 * o + 1] = rgb[1]; rgb_out[3 * o + 2] = rgb[2];
        }
    }
    if (stats) {
        stats->camera_rays = pool.total.camera;
        stats->closest_rays = pool.total.closest;
        stats->shadow_rays = pool.total.shadow;
        stats->node_visits = pool.total.nodes;
        stats->prim_tests = pool.total.prims;
        stats->samples = pool.total.camera;
    }
    free(xyz);
    free(pool.tiles);
    pthread_mutex_destroy(&pool.mu);
    scene_free(&sc);
    return pool.total.dim_overflow ? 3 : 0; /* 3: Halton dimension past the prime table */
}

int oracle_render(const pt_scene_desc* desc, float* rgb_out, int nthreads, int max_tiles, oracle_stats* stats) {
    return render_common(desc, rgb_out, NULL, nthreads, max_tiles, 0, 1, 0, -1, stats);
}
int oracle_render_accum(const pt_scene_desc* desc, float* accum_out, int nthreads, int tile_offset, int tile_stride,
                        oracle_stats* stats) {
    return render_common(desc, NULL, accum_out, nthreads, -1, tile_offset, tile_stride, 0, -1, stats);
}
int oracle_render_range(const pt_scene_desc* desc, float* accum_out, int nthreads, int tile_offset, int tile_stride,
                        int s_begin, int s_end, oracle_stats* stats) {
    return render_common(desc, NULL, accum_out, nthreads, -1, tile_offset, tile_stride, s_begin, s_end, stats);
}
void oracle_set_trig(int correctly_rounded) { g_cr_trig = correctly_rounded; }

/* BSDF of a material in the shading frame ns = ng = (0,0,1), ss = (1,0,0):
 * f and pdf for (wo, wi), and Sample_f for (wo, u).  Known-answer hook. */
static void local_bsdf(const pt_material* m, int multi, BSDF* b) {
    SI si;
    memset(&si, 0, sizeof si);
    si.n = v3(0, 0, 1); si.sn = v3(0, 0, 1); si.sdpdu = v3(1, 0, 0);
    make_bsdf(m, &si, 550.f, multi, b);
}
/* Batched BSDF hook with the layout of the product's pt_debug_bsdf: per record
 * in8 = wo[3], wi[3], u0, u1 -> out8 = f[3], pdf, sampled wi[3], sampled pdf
 * (f is the sampled f when wi is all zero). */
int oracle_bsdf_batch(const pt_scene_desc* d, int mat, int n, const float* in8, float* out8) {
    BSDF b;
    if (!d || mat < 0 || mat >= d->n_materials) return 1;
    local_bsdf(&d->materials[mat], d->integrator.kind != PT_INTEGRATOR_DIRECT, &b);
    for (int i = 0; i < n; ++i) {
        const float* a = in8 + 8 * i;
        float* o = out8 + 8 * i;
        V3 wo = v3(a[0], a[1], a[2]), wi = v3(a[3], a[4], a[5]);
        RGB f = rgb1(0);
        float pdf = 0;
        int zero = wi.x == 0 && wi.y == 0 && wi.z == 0;
        if (!zero) { f = bsdf_f(&b, wo, wi, BX_ALL); pdf = bsdf_pdf(&b, wo, wi, BX_ALL); }
        float u[2] = {a[6], a[7]};
        V3 ws = v3(0, 0, 0);
        float spdf = 0;
        int sampled = 0;
        RGB sf = bsdf_sample_f(&b, wo, &ws, u, &spdf, BX_ALL, &sampled);
        if (zero) f = sf;
        o[0] = f.c[0]; o[1] = f.c[1]; o[2] = f.c[2]; o[3] = pdf;
        o[4] = ws.x; o[5] = ws.y; o[6] = ws.z; o[7] = spdf;
    }
    return 0;
}
int oracle_film_size(const pt_scene_desc* desc, int* w, int* h) {
    Scene sc;
    memset(&sc, 0, sizeof sc);
    sc.d = desc;
    film_init(&sc);
    *w = sc.crop_x1 - sc.crop_x0;
    *h = sc.crop_y1 - sc.crop_y0;
    return 0;
}
/* ScrambledRadicalInverse with a caller-supplied permutation (for the
 * reference's own LowDiscrepancy.ScrambledRadicalInverse test). */
float oracle_scrambled_radical_inverse_perm(int base_index, uint64_t a, const uint16_t* perm) {
    ensure_init();
    return scrambled_radical_inverse(base_index, a, perm);
}
/* Closest-hit (any = 0) or any-hit (any = 1) BVH query: returns the index
 * into desc->prims of the hit primitive, -1 for none (any-hit: 1/0). */
int oracle_trace(const pt_scene_desc* desc, int n, const float* rays7, int any, int32_t* out) {
    Scene sc;
    scene_setup(&sc, desc);
    Counters c = {0, 0, 0, 0, 0};
    int* inv = (int*)malloc(sizeof(int) * (size_t)(sc.nprims + 1));
    for (int i = 0; i < sc.nprims; ++i) {
        inv[i] = -1;
        for (int j = 0; j < desc->n_prims; ++j)
            if (desc->prims[j].kind == sc.prim_kind[i] && desc->prims[j].index == sc.prim_index[i]) { inv[i] = j; break; }
    }
    for (int i = 0; i < n; ++i) {
        const float* r = rays7 + 7 * i;
        Ray ray = {v3(r[0], r[1], r[2]), v3(r[3], r[4], r[5]), r[6]};
        if (any) out[i] = scene_intersect_p(&sc, &ray, &c);
        else {
            SI si;
            memset(&si, 0, sizeof si);
            si.prim = -1;
            int h = scene_intersect(&sc, &ray, &si, &c);
            out[i] = h ? inv[si.prim] : -1;
        }
    }
    free(inv);
    scene_free(&sc);
    return 0;
}

int oracle_build_bvh(const pt_scene_desc* desc, int32_t* n_nodes, uint32_t* nodes, int32_t* prim_order, int32_t cap) {
    Scene sc;
    scene_setup(&sc, desc);
    *n_nodes = sc.nnodes;
    if (nodes && sc.nnodes <= cap) {
        for (int i = 0; i < sc.nnodes; ++i) {
            const LNode* n = &sc.nodes[i];
            float b[6] = {n->bounds.pmin.x, n->bounds.pmin.y, n->bounds.pmin.z,
                          n->bounds.pmax.x, n->bounds.pmax.y, n->bounds.pmax.z};
            memcpy(&nodes[8 * i], b, 24);
            nodes[8 * i + 6] = (uint32_t)n->offset;
            nodes[8 * i + 7] = (uint32_t)n->nprims | ((uint32_t)n->axis << 16);
        }
    }
    if (prim_order && sc.nprims <= cap) {
        /* report primitive order as indices into desc->prims */
        for (int i = 0; i < sc.nprims; ++i) {
            int found = -1;
            for (int j = 0; j < desc->n_prims; ++j)
                if (desc->prims[j].kind == sc.prim_kind[i] && desc->prims[j].index == sc.prim_index[i]) { found = j; break; }
            prim_order[i] = found;
        }
    }
    scene_free(&sc);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Known-answer exports                                                      */
/* ------------------------------------------------------------------------ */
float oracle_radical_inverse(int base_index, uint64_t a) { ensure_init(); return radical_inverse(base_index, a); }
float oracle_scrambled_radical_inverse(int base_index, uint64_t a) {
    ensure_init();
    return scrambled_radical_inverse(base_index, a, g_perms + g_prime_sums[base_index]);
}
int oracle_prime(int i) { ensure_init(); return g_primes[i]; }
int oracle_halton_perm(int64_t i) { ensure_init(); return g_perms[i]; }
float oracle_halton_sample(int x0, int y0, int x1, int y1, int px, int py, int64_t sample, int dim) {
    ensure_init();
    Halton h;
    halton_init(&h, x0, y0, x1, y1, 0);
    int64_t idx = halton_pixel_offset(&h, px, py) + sample * h.stride;
    return halton_dim(&h, idx, dim);
}
int64_t oracle_halton_index(int x0, int y0, int x1, int y1, int px, int py, int64_t sample) {
    ensure_init();
    Halton h;
    halton_init(&h, x0, y0, x1, y1, 0);
    return halton_pixel_offset(&h, px, py) + sample * h.stride;
}
int oracle_ray_triangle(const float o[3], const float d[3], float tmax, const float p0[3], const float p1[3],
                        const float p2[3], float* t, float b[3]) {
    ensure_init();
    float P[9] = {p0[0], p0[1], p0[2], p1[0], p1[1], p1[2], p2[0], p2[1], p2[2]};
    pt_triangle tri = {{0, 1, 2}, 0, -1, 0};
    pt_scene_desc dd;
    memset(&dd, 0, sizeof dd);
    dd.n_vertices = 3; dd.P = P; dd.n_triangles = 1; dd.triangles = &tri;
    Ray r = {v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), tmax};
    SI si;
    float th;
    int ok = tri_intersect(&dd, 0, &r, &th, &si, 1);
    if (ok) {
        *t = th;
        /* recover barycentrics from p = b0 p0 + b1 p1 + b2 p2 is not needed by
         * callers; report the hit point instead */
        b[0] = si.p.x; b[1] = si.p.y; b[2] = si.p.z;
    }
    return ok;
}
int oracle_camera_ray(const pt_scene_desc* desc, float fx, float fy, float o[3], float d[3]) {
    Scene sc;
    ensure_init();
    memset(&sc, 0, sizeof sc);
    sc.d = desc;
    camera_init(&sc);
    float pl[2] = {0.5f, 0.5f};
    Ray r = camera_ray(&sc, fx, fy, pl);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    d[0] = r.d.x; d[1] = r.d.y; d[2] = r.d.z;
    return 0;
}
