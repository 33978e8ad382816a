// stub_pbrt.h -- a minimal re-declaration of the pbrt-v3 classes the
// GpuPathIntegrator binding (integration/gpupath.cpp) reads, for compiling and
// exercising the binding without the reference's build (which needs its git
// submodules).  Not reference source: the names, members and signatures follow
// the reference headers cited below, plus the small accessor patch a
// maintainer adds next to the binding (marked "PATCH", listed in
// INTEGRATION.md).  Bodies exist only where the binding or its test driver
// call them.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace pbrt {

typedef float Float;  // CMakeLists.txt:12 (PBRT_FLOAT_AS_DOUBLE off)
static constexpr Float Infinity = std::numeric_limits<Float>::infinity();

// core/geometry.h
template <typename T>
struct Vector2 { T x = 0, y = 0; Vector2() = default; Vector2(T x, T y) : x(x), y(y) {} };
template <typename T>
struct Point2 { T x = 0, y = 0; Point2() = default; Point2(T x, T y) : x(x), y(y) {} };
template <typename T>
struct Point3 {
    T x = 0, y = 0, z = 0;
    Point3() = default;
    Point3(T x, T y, T z) : x(x), y(y), z(z) {}
    T operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
template <typename T>
struct Vector3 { T x = 0, y = 0, z = 0; Vector3() = default; Vector3(T x, T y, T z) : x(x), y(y), z(z) {} };
template <typename T>
struct Normal3 { T x = 0, y = 0, z = 0; Normal3() = default; Normal3(T x, T y, T z) : x(x), y(y), z(z) {} };
typedef Vector2<Float> Vector2f;
typedef Point2<Float> Point2f;
typedef Point2<int> Point2i;
typedef Point3<Float> Point3f;
typedef Vector3<Float> Vector3f;
typedef Normal3<Float> Normal3f;
template <typename T>
struct Bounds2 { Point2<T> pMin, pMax; };
typedef Bounds2<int> Bounds2i;

// core/transform.h: Matrix4x4 + Transform (m, mInv), GetMatrix / GetInverseMatrix
struct Matrix4x4 {
    Float m[4][4];
    Matrix4x4() { for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) m[i][j] = i == j; }
};
class Transform {
  public:
    Transform() = default;
    Transform(const Matrix4x4& m, const Matrix4x4& mInv) : m(m), mInv(mInv) {}
    const Matrix4x4& GetMatrix() const { return m; }
    const Matrix4x4& GetInverseMatrix() const { return mInv; }
    bool SwapsHandedness() const {  // transform.cpp: sign of the upper 3x3 determinant
        Float det = m.m[0][0] * (m.m[1][1] * m.m[2][2] - m.m[1][2] * m.m[2][1]) -
                    m.m[0][1] * (m.m[1][0] * m.m[2][2] - m.m[1][2] * m.m[2][0]) +
                    m.m[0][2] * (m.m[1][0] * m.m[2][1] - m.m[1][1] * m.m[2][0]);
        return det < 0;
    }
  private:
    Matrix4x4 m, mInv;
};

// core/spectrum.h (RGBSpectrum build)
class RGBSpectrum {
  public:
    RGBSpectrum(Float v = 0.f) { c[0] = c[1] = c[2] = v; }
    static RGBSpectrum FromRGB(const Float rgb[3]) { RGBSpectrum s; for (int i = 0; i < 3; ++i) s.c[i] = rgb[i]; return s; }
    void ToRGB(Float* rgb) const { for (int i = 0; i < 3; ++i) rgb[i] = c[i]; }
  private:
    Float c[3];
};
typedef RGBSpectrum Spectrum;

// core/error.h
inline void Error(const char* fmt, ...) {
    va_list a;
    va_start(a, fmt);
    std::fprintf(stderr, "Error: ");
    std::vfprintf(stderr, fmt, a);
    std::fprintf(stderr, "\n");
    va_end(a);
}

// core/paramset.h: the Find* queries (paramset.h:95-109)
class ParamSet {
  public:
    void AddFloat(const std::string& n, std::vector<Float> v) { floats[n] = std::move(v); }
    void AddInt(const std::string& n, std::vector<int> v) { ints[n] = std::move(v); }
    void AddBool(const std::string& n, bool v) { bools[n] = v; }
    void AddString(const std::string& n, const std::string& v) { strings[n] = v; }
    Float FindOneFloat(const std::string& n, Float d) const {
        auto it = floats.find(n);
        return it != floats.end() && it->second.size() == 1 ? it->second[0] : d;
    }
    int FindOneInt(const std::string& n, int d) const {
        auto it = ints.find(n);
        return it != ints.end() && it->second.size() == 1 ? it->second[0] : d;
    }
    bool FindOneBool(const std::string& n, bool d) const {
        auto it = bools.find(n);
        return it != bools.end() ? it->second : d;
    }
    std::string FindOneString(const std::string& n, const std::string& d) const {
        auto it = strings.find(n);
        return it != strings.end() ? it->second : d;
    }
    const Float* FindFloat(const std::string& n, int* cnt) const {
        auto it = floats.find(n);
        if (it == floats.end()) { *cnt = 0; return nullptr; }
        *cnt = (int)it->second.size();
        return it->second.data();
    }
    const int* FindInt(const std::string& n, int* cnt) const {
        auto it = ints.find(n);
        if (it == ints.end()) { *cnt = 0; return nullptr; }
        *cnt = (int)it->second.size();
        return it->second.data();
    }
  private:
    std::map<std::string, std::vector<Float>> floats;
    std::map<std::string, std::vector<int>> ints;
    std::map<std::string, bool> bools;
    std::map<std::string, std::string> strings;
};

struct SurfaceInteraction {};  // core/interaction.h (only default-constructed here)

// core/texture.h, textures/constant.h
template <typename T>
class Texture {
  public:
    virtual T Evaluate(const SurfaceInteraction&) const = 0;
    virtual ~Texture() {}
};
template <typename T>
class ConstantTexture : public Texture<T> {
  public:
    ConstantTexture(const T& value) : value(value) {}
    T Evaluate(const SurfaceInteraction&) const { return value; }
  private:
    T value;
};

// core/material.h, materials/matte.h
class Material {
  public:
    virtual ~Material() {}
};
class MatteMaterial : public Material {
  public:
    MatteMaterial(const std::shared_ptr<Texture<Spectrum>>& Kd, const std::shared_ptr<Texture<Float>>& sigma,
                  const std::shared_ptr<Texture<Float>>& bumpMap)
        : Kd(Kd), sigma(sigma), bumpMap(bumpMap) {}
    const std::shared_ptr<Texture<Spectrum>>& GetKd() const { return Kd; }        // PATCH
    const std::shared_ptr<Texture<Float>>& GetSigma() const { return sigma; }     // PATCH
  private:
    std::shared_ptr<Texture<Spectrum>> Kd;
    std::shared_ptr<Texture<Float>> sigma, bumpMap;
};

// core/microfacet.h:105-133: the static remap of roughness to alpha
class TrowbridgeReitzDistribution {
  public:
    static inline Float RoughnessToAlpha(Float roughness) {
        roughness = std::max(roughness, (Float)1e-3);
        Float x = std::log(roughness);
        return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
    }
};

// materials/metal.h:49-69
class MetalMaterial : public Material {
  public:
    MetalMaterial(const std::shared_ptr<Texture<Spectrum>>& eta, const std::shared_ptr<Texture<Spectrum>>& k,
                  const std::shared_ptr<Texture<Float>>& rough, const std::shared_ptr<Texture<Float>>& urough,
                  const std::shared_ptr<Texture<Float>>& vrough, const std::shared_ptr<Texture<Float>>& bump,
                  bool remapRoughness)
        : eta(eta), k(k), roughness(rough), uRoughness(urough), vRoughness(vrough), bumpMap(bump),
          remapRoughness(remapRoughness) {}
    // PATCH: read access to the members (metal.h:65-68)
    const std::shared_ptr<Texture<Spectrum>>& GetEta() const { return eta; }
    const std::shared_ptr<Texture<Spectrum>>& GetK() const { return k; }
    const std::shared_ptr<Texture<Float>>& GetRoughness() const { return roughness; }
    const std::shared_ptr<Texture<Float>>& GetURoughness() const { return uRoughness; }
    const std::shared_ptr<Texture<Float>>& GetVRoughness() const { return vRoughness; }
    bool RemapRoughness() const { return remapRoughness; }
  private:
    std::shared_ptr<Texture<Spectrum>> eta, k;
    std::shared_ptr<Texture<Float>> roughness, uRoughness, vRoughness;
    std::shared_ptr<Texture<Float>> bumpMap;
    bool remapRoughness;
};

// materials/glass.h:48-76
class GlassMaterial : public Material {
  public:
    GlassMaterial(const std::shared_ptr<Texture<Spectrum>>& Kr, const std::shared_ptr<Texture<Spectrum>>& Kt,
                  const std::shared_ptr<Texture<Float>>& uRoughness, const std::shared_ptr<Texture<Float>>& vRoughness,
                  const std::shared_ptr<Texture<Float>>& index, const std::shared_ptr<Texture<Float>>& bumpMap,
                  bool remapRoughness)
        : Kr(Kr), Kt(Kt), uRoughness(uRoughness), vRoughness(vRoughness), index(index), bumpMap(bumpMap),
          remapRoughness(remapRoughness) {}
    // PATCH: read access to the members (glass.h:71-75)
    const std::shared_ptr<Texture<Spectrum>>& GetKr() const { return Kr; }
    const std::shared_ptr<Texture<Spectrum>>& GetKt() const { return Kt; }
    const std::shared_ptr<Texture<Float>>& GetURoughness() const { return uRoughness; }
    const std::shared_ptr<Texture<Float>>& GetVRoughness() const { return vRoughness; }
    const std::shared_ptr<Texture<Float>>& GetIndex() const { return index; }
    bool RemapRoughness() const { return remapRoughness; }
  private:
    std::shared_ptr<Texture<Spectrum>> Kr, Kt;
    std::shared_ptr<Texture<Float>> uRoughness, vRoughness;
    std::shared_ptr<Texture<Float>> index;
    std::shared_ptr<Texture<Float>> bumpMap;
    bool remapRoughness;
};

// materials/dispersive_glass.h:47-78 (the fork's Cauchy-dispersion glass)
class DispersiveGlassMaterial : public Material {
  public:
    DispersiveGlassMaterial(const std::shared_ptr<Texture<Spectrum>>& Kr, const std::shared_ptr<Texture<Spectrum>>& Kt,
                            const std::shared_ptr<Texture<Float>>& uRoughness,
                            const std::shared_ptr<Texture<Float>>& vRoughness,
                            const std::shared_ptr<Texture<Float>>& indexMin,
                            const std::shared_ptr<Texture<Float>>& indexMax,
                            const std::shared_ptr<Texture<Float>>& bumpMap, bool remapRoughness)
        : Kr(Kr), Kt(Kt), uRoughness(uRoughness), vRoughness(vRoughness), indexMin(indexMin), indexMax(indexMax),
          bumpMap(bumpMap), remapRoughness(remapRoughness) {}
    // PATCH: read access to the members (dispersive_glass.h:70-76)
    const std::shared_ptr<Texture<Spectrum>>& GetKr() const { return Kr; }
    const std::shared_ptr<Texture<Spectrum>>& GetKt() const { return Kt; }
    const std::shared_ptr<Texture<Float>>& GetURoughness() const { return uRoughness; }
    const std::shared_ptr<Texture<Float>>& GetVRoughness() const { return vRoughness; }
    const std::shared_ptr<Texture<Float>>& GetIndexMin() const { return indexMin; }
    const std::shared_ptr<Texture<Float>>& GetIndexMax() const { return indexMax; }
    bool RemapRoughness() const { return remapRoughness; }
  private:
    std::shared_ptr<Texture<Spectrum>> Kr, Kt;
    std::shared_ptr<Texture<Float>> uRoughness, vRoughness;
    std::shared_ptr<Texture<Float>> indexMin;
    std::shared_ptr<Texture<Float>> indexMax;
    std::shared_ptr<Texture<Float>> bumpMap;
    bool remapRoughness;
};

// materials/mirror.h:48-64
class MirrorMaterial : public Material {
  public:
    MirrorMaterial(const std::shared_ptr<Texture<Spectrum>>& r, const std::shared_ptr<Texture<Float>>& bump)
        : Kr(r), bumpMap(bump) {}
    const std::shared_ptr<Texture<Spectrum>>& GetKr() const { return Kr; }  // PATCH
  private:
    std::shared_ptr<Texture<Spectrum>> Kr;
    std::shared_ptr<Texture<Float>> bumpMap;
};

// materials/plastic.h:48-70
class PlasticMaterial : public Material {
  public:
    PlasticMaterial(const std::shared_ptr<Texture<Spectrum>>& Kd, const std::shared_ptr<Texture<Spectrum>>& Ks,
                    const std::shared_ptr<Texture<Float>>& roughness, const std::shared_ptr<Texture<Float>>& bumpMap,
                    bool remapRoughness)
        : Kd(Kd), Ks(Ks), roughness(roughness), bumpMap(bumpMap), remapRoughness(remapRoughness) {}
    // PATCH: read access to the members (plastic.h:67-69)
    const std::shared_ptr<Texture<Spectrum>>& GetKd() const { return Kd; }
    const std::shared_ptr<Texture<Spectrum>>& GetKs() const { return Ks; }
    const std::shared_ptr<Texture<Float>>& GetRoughness() const { return roughness; }
    bool RemapRoughness() const { return remapRoughness; }
  private:
    std::shared_ptr<Texture<Spectrum>> Kd, Ks;
    std::shared_ptr<Texture<Float>> roughness, bumpMap;
    const bool remapRoughness;
};

// core/shape.h (shape.h:52-88)
class Shape {
  public:
    Shape(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation)
        : ObjectToWorld(ObjectToWorld), WorldToObject(WorldToObject), reverseOrientation(reverseOrientation),
          transformSwapsHandedness(ObjectToWorld->SwapsHandedness()) {}
    virtual ~Shape() {}
    const Transform *ObjectToWorld, *WorldToObject;
    const bool reverseOrientation;
    const bool transformSwapsHandedness;
};

// shapes/triangle.h:52-120
struct TriangleMesh {
    TriangleMesh(int nTriangles, const int* vertexIndices, int nVertices, const Point3f* P, const Vector3f* S,
                 const Normal3f* N, const Point2f* UV)
        : nTriangles(nTriangles), nVertices(nVertices), vertexIndices(vertexIndices, vertexIndices + 3 * nTriangles) {
        p.reset(new Point3f[nVertices]);
        for (int i = 0; i < nVertices; ++i) p[i] = P[i];  // (the reference transforms to world space here)
        if (N) { n.reset(new Normal3f[nVertices]); for (int i = 0; i < nVertices; ++i) n[i] = N[i]; }
        if (S) { s.reset(new Vector3f[nVertices]); for (int i = 0; i < nVertices; ++i) s[i] = S[i]; }
        if (UV) { uv.reset(new Point2f[nVertices]); for (int i = 0; i < nVertices; ++i) uv[i] = UV[i]; }
    }
    const int nTriangles, nVertices;
    std::vector<int> vertexIndices;
    std::unique_ptr<Point3f[]> p;
    std::unique_ptr<Normal3f[]> n;
    std::unique_ptr<Vector3f[]> s;
    std::unique_ptr<Point2f[]> uv;
};
class Triangle : public Shape {
  public:
    Triangle(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation,
             const std::shared_ptr<TriangleMesh>& mesh, int triNumber)
        : Shape(ObjectToWorld, WorldToObject, reverseOrientation), mesh(mesh) {
        v = &mesh->vertexIndices[3 * triNumber];
    }
    const TriangleMesh* GetMesh() const { return mesh.get(); }  // PATCH
    const int* GetVertexIndices() const { return v; }           // PATCH
  private:
    std::shared_ptr<TriangleMesh> mesh;
    const int* v;
};

// shapes/plane.h:12-70 (public members)
class AAPlaneShape : public Shape {
  public:
    AAPlaneShape(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation,
                 const Point3f& lo, const Point3f& hi, int axis, bool /*facingFw: ignored, plane.h:24*/)
        : Shape(ObjectToWorld, WorldToObject, reverseOrientation), facingFw(!reverseOrientation), lo(lo), hi(hi),
          ax(axis), ax0(axis == 2 ? 0 : (axis == 0 ? 1 : 2)), ax1(axis == 2 ? 1 : (axis == 0 ? 2 : 0)) {}
    bool facingFw;
    Point3f lo;
    Point3f hi;
    const int ax;
    const int ax0;
    const int ax1;
};

// shapes/sphere.h:47-76
class Sphere : public Shape {
  public:
    Sphere(const Transform* ObjectToWorld, const Transform* WorldToObject, bool reverseOrientation, Float radius,
           Float zMin, Float zMax, Float phiMax)
        : Shape(ObjectToWorld, WorldToObject, reverseOrientation), radius(radius),
          zMin(std::min(std::max(std::min(zMin, zMax), -radius), radius)),
          zMax(std::min(std::max(std::max(zMin, zMax), -radius), radius)), phiMaxDegrees(phiMax) {}
    // PATCH: the creation parameters (the members keep phiMax in radians,
    // Radians(Clamp(phiMax, 0, 360)), which does not round-trip exactly)
    Float Radius() const { return radius; }
    Float ZMin() const { return zMin; }
    Float ZMax() const { return zMax; }
    Float PhiMaxDegrees() const { return phiMaxDegrees; }
  private:
    const Float radius;
    const Float zMin, zMax;
    const Float phiMaxDegrees;
};

// portals/aaportal.h: the portal rectangle on the light's transforms (aaportal.cpp:8-12)
class AAPortal {
  public:
    AAPortal(const Point3f& lo, const Point3f& hi, int axis, bool facingFw, AAPlaneShape& light)
        : light(light), portal(light.ObjectToWorld, light.WorldToObject, !facingFw, lo, hi, axis, facingFw) {}
    const AAPlaneShape& light;
    const AAPlaneShape portal;
};

// core/light.h:63-101
class Light {
  public:
    Light(int flags, int nSamples) : flags(flags), nSamples(nSamples) {}
    virtual ~Light() {}
    const int flags;
    const int nSamples;
};
class AreaLight : public Light {
  public:
    AreaLight(int nSamples) : Light(/* LightFlags::Area */ 8, nSamples) {}
};

// lights/diffuse.h:49-80
class DiffuseAreaLight : public AreaLight {
  public:
    DiffuseAreaLight(const Spectrum& Lemit, int nSamples, const std::shared_ptr<Shape>& shape, bool twoSided = false)
        : AreaLight(nSamples), Lemit(Lemit), shape(shape), twoSided(twoSided) {}
    const Spectrum& GetLemit() const { return Lemit; }     // PATCH
    bool TwoSided() const { return twoSided; }             // PATCH
    const Shape* GetShape() const { return shape.get(); }  // PATCH
  protected:
    const Spectrum Lemit;
    std::shared_ptr<Shape> shape;
    const bool twoSided;
};

// lights/point.h:49-71: pLight = LightToWorld(Point3f(0, 0, 0)) (point.h:55)
class PointLight : public Light {
  public:
    PointLight(const Point3f& pLight, const Spectrum& I) : Light(/* DeltaPosition */ 1, 1), pLight(pLight), I(I) {}
    const Point3f& GetPosition() const { return pLight; }  // PATCH
    const Spectrum& GetIntensity() const { return I; }     // PATCH
  private:
    const Point3f pLight;
    const Spectrum I;
};

// core/mipmap.h: the queries the binding makes of an InfiniteAreaLight's Lmap
template <typename T>
class MIPMap {
  public:
    MIPMap(int w, int h, std::vector<T> texels) : w(w), h(h), texels(std::move(texels)) {}
    int Width() const { return w; }
    int Height() const { return h; }
    const T& Texel(int level, int s, int t) const { (void)level; return texels[(size_t)t * w + s]; }
  private:
    int w, h;
    std::vector<T> texels;
};

// lights/infinite.h:52-76; without "mapname" the constructor builds a 1x1 Lmap
// holding L (infinite.cpp:43-61), as this one does
class InfiniteAreaLight : public Light {
  public:
    InfiniteAreaLight(const Transform& LightToWorld, const Spectrum& L, int nSamples)
        : Light(/* Infinite */ 8, nSamples), LightToWorld(LightToWorld),
          Lmap(new MIPMap<RGBSpectrum>(1, 1, std::vector<RGBSpectrum>{L})) {}
    // PATCH: LightToWorld (light.h protected member) and Lmap
    const Transform& GetLightToWorld() const { return LightToWorld; }
    const MIPMap<RGBSpectrum>* GetLmap() const { return Lmap.get(); }
  private:
    const Transform LightToWorld;
    std::unique_ptr<MIPMap<RGBSpectrum>> Lmap;
};

// lights/portal_arealight.h
enum class PortalStrategy { SampleUniformPortal, SampleUniformLight, SampleProjection };
class PortalArealight : public DiffuseAreaLight {
  public:
    PortalArealight(const Spectrum& Le, int nSamples, const std::shared_ptr<AAPlaneShape>& light,
                    std::vector<AAPortal> portals, const PortalStrategy strategy, bool twoSided = false)
        : DiffuseAreaLight(Le, nSamples, light, twoSided), portals(std::move(portals)), shape(light), strat(strategy) {}
    const std::vector<AAPortal> portals;
    std::shared_ptr<AAPlaneShape> shape;
    const PortalStrategy strat;
};

// core/primitive.h
class Primitive {
  public:
    virtual ~Primitive() {}
};
class Aggregate : public Primitive {};
class GeometricPrimitive : public Primitive {
  public:
    GeometricPrimitive(const std::shared_ptr<Shape>& shape, const std::shared_ptr<Material>& material,
                       const std::shared_ptr<AreaLight>& areaLight)
        : shape(shape), material(material), areaLight(areaLight) {}
    const AreaLight* GetAreaLight() const { return areaLight.get(); }
    const Material* GetMaterial() const { return material.get(); }
    const Shape* GetShape() const { return shape.get(); }  // PATCH
  private:
    std::shared_ptr<Shape> shape;
    std::shared_ptr<Material> material;
    std::shared_ptr<AreaLight> areaLight;
};

// accelerators/bvh.{h,cpp}: LinearBVHNode (bvh.cpp:95-104; the stub's test
// driver fills records of it, the binding only sees the pointer) and the
// flattened tree
struct Bounds3f { Point3f pMin, pMax; };
struct LinearBVHNode {
    Bounds3f bounds;
    union {
        int primitivesOffset;   // leaf
        int secondChildOffset;  // interior
    };
    uint16_t nPrimitives;  // 0 -> interior node
    uint8_t axis;          // interior node: xyz
    uint8_t pad[1];        // ensure 32 byte total size
};
static_assert(sizeof(LinearBVHNode) == 32, "LinearBVHNode is 32 bytes");
class BVHAccel : public Aggregate {
  public:
    // stub constructor: the flattened result of the reference's build
    // (BVHAccel::BVHAccel, bvh.cpp:186-236) handed in by the test driver
    BVHAccel(std::vector<std::shared_ptr<Primitive>> orderedPrims, std::vector<LinearBVHNode> flat)
        : primitives(std::move(orderedPrims)), flat(std::move(flat)) {
        nodes = this->flat.empty() ? nullptr : this->flat.data();
    }
    const std::vector<std::shared_ptr<Primitive>>& GetPrimitives() const { return primitives; }  // PATCH
    const LinearBVHNode* GetNodes() const { return nodes; }                                       // PATCH
  private:
    std::vector<std::shared_ptr<Primitive>> primitives;
    std::vector<LinearBVHNode> flat;
    LinearBVHNode* nodes = nullptr;
};

// core/scene.h:50-80
class Scene {
  public:
    Scene(std::shared_ptr<Primitive> aggregate, const std::vector<std::shared_ptr<Light>>& lights)
        : lights(lights), aggregate(aggregate) {}
    const Primitive* GetAggregate() const { return aggregate.get(); }  // PATCH
    std::vector<std::shared_ptr<Light>> lights;
  private:
    std::shared_ptr<Primitive> aggregate;
};

// core/filter.h, core/film.h:59-95, core/camera.h:51-70
class Filter {
  public:
    Filter(const Vector2f& radius) : radius(radius), invRadius(1 / radius.x, 1 / radius.y) {}
    virtual ~Filter() {}
    const Vector2f radius, invRadius;
};
class Film {
  public:
    Film(const Point2i& resolution, std::unique_ptr<Filter> filt, Float diagonal, const std::string& filename)
        : fullResolution(resolution), diagonal(diagonal * .001f), filter(std::move(filt)), filename(filename) {}
    const Point2i fullResolution;
    const Float diagonal;
    std::unique_ptr<Filter> filter;
    const std::string filename;
};
class Camera {
  public:
    Camera(Film* film) : film(film) {}
    virtual ~Camera() { delete film; }
    Film* film;
};
class Sampler {
  public:
    virtual ~Sampler() {}
};

// core/integrator.h:53-58
class Integrator {
  public:
    virtual ~Integrator() {}
    virtual void Render(const Scene& scene) = 0;
};

}  // namespace pbrt
