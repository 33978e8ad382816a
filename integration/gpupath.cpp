// gpupath.cpp -- GpuPathIntegrator: pbrt-v3's Scene flattened into the C ABI
// of the MI355X path tracer (include/pt.h).  See gpupath.h.
#include "gpupath.h"

#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "accelerators/bvh.h"
#include "core/error.h"
#include "core/film.h"
#include "core/primitive.h"
#include "core/microfacet.h"
#include "lights/diffuse.h"
#include "lights/infinite.h"
#include "lights/point.h"
#include "lights/portal_arealight.h"
#include "materials/dispersive_glass.h"
#include "materials/glass.h"
#include "materials/matte.h"
#include "materials/metal.h"
#include "materials/mirror.h"
#include "materials/plastic.h"
#include "portals/aaportal.h"
#include "shapes/plane.h"
#include "shapes/sphere.h"
#include "shapes/triangle.h"
#include "textures/constant.h"

namespace pbrt {

static void to_pt(const Transform& t, pt_transform* out) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            out->m[4 * i + j] = t.GetMatrix().m[i][j];
            out->minv[4 * i + j] = t.GetInverseMatrix().m[i][j];
        }
}

// The value of a ConstantTexture (false for any other texture); a null
// texture keeps *out.
template <typename T>
static bool constant_value(const std::shared_ptr<Texture<T>>& t, T* out) {
    if (!t) return true;
    const auto* c = dynamic_cast<const ConstantTexture<T>*>(t.get());
    if (!c) return false;
    *out = c->Evaluate(SurfaceInteraction());
    return true;
}
// A microfacet material's alpha: RoughnessToAlpha when it remaps, then the
// TrowbridgeReitzDistribution ctor's floor (microfacet.h:109-132).
static Float tr_alpha(Float rough, bool remap) {
    if (remap) rough = TrowbridgeReitzDistribution::RoughnessToAlpha(rough);
    return std::max(Float(0.001), rough);
}

static uint32_t shape_flags(const Shape& s) {
    return (s.reverseOrientation ? PT_TRI_REVERSE_ORIENTATION : 0u) |
           (s.transformSwapsHandedness ? PT_TRI_SWAPS_HANDEDNESS : 0u);
}

bool FlattenScene(const Scene& scene, const GpuRenderSettings& settings, GpuFlatScene* f, std::string* err) {
    *f = GpuFlatScene{};
    auto fail = [&](const std::string& m) { *err = m; return false; };
    // Scene::aggregate must be the BVHAccel the reference built (api.cpp
    // MakeAccelerator): its flattened nodes and primitive order are handed to
    // the device as they are, so traversal visits the same nodes.
    const BVHAccel* bvh = dynamic_cast<const BVHAccel*>(scene.GetAggregate());
    if (!bvh) return fail("gpupath: the scene aggregate is not a BVHAccel");

    // lights in Scene::lights order (UniformLightDistribution indexes them so)
    std::unordered_map<const Light*, int> lightIndex;
    for (size_t i = 0; i < scene.lights.size(); ++i) lightIndex[scene.lights[i].get()] = (int)i;
    std::unordered_map<const Material*, int> materialIndex;
    std::unordered_map<const TriangleMesh*, int> meshBase;
    std::unordered_map<const Shape*, int> triIndex, planeIndex, sphereIndex;
    bool anyN = false, anyS = false, anyUV = false;
    for (const auto& p : bvh->GetPrimitives()) {
        const auto* gp = dynamic_cast<const GeometricPrimitive*>(p.get());
        const Triangle* t = gp ? dynamic_cast<const Triangle*>(gp->GetShape()) : nullptr;
        if (t) {
            anyN |= t->GetMesh()->n != nullptr;
            anyS |= t->GetMesh()->s != nullptr;
            anyUV |= t->GetMesh()->uv != nullptr;
        }
    }

    auto material = [&](const Material* m, int* out) -> bool {
        auto it = materialIndex.find(m);
        if (it != materialIndex.end()) { *out = it->second; return true; }
        pt_material pm;
        std::memset(&pm, 0, sizeof pm);
        if (!m) {
            pm.kind = PT_MAT_NONE;  // Material "none": null BSDF (path.cpp:108-113)
        } else if (const auto* mm = dynamic_cast<const MatteMaterial*>(m)) {
            const auto* kd = dynamic_cast<const ConstantTexture<Spectrum>*>(mm->GetKd().get());
            const auto* sg = dynamic_cast<const ConstantTexture<Float>*>(mm->GetSigma().get());
            if (!kd || !sg) { *err = "gpupath: matte with non-constant textures"; return false; }
            pm.kind = PT_MAT_MATTE;
            kd->Evaluate(SurfaceInteraction()).ToRGB(pm.kd);
            pm.sigma = sg->Evaluate(SurfaceInteraction());
        } else if (const auto* me = dynamic_cast<const MetalMaterial*>(m)) {
            // MetalMaterial::ComputeScatteringFunctions (metal.cpp:58-79)
            Spectrum eta, k;
            Float rough = 0, ur = 0, vr = 0;
            if (!constant_value(me->GetEta(), &eta) || !constant_value(me->GetK(), &k) ||
                !constant_value(me->GetRoughness(), &rough) || !constant_value(me->GetURoughness(), &ur) ||
                !constant_value(me->GetVRoughness(), &vr)) {
                *err = "gpupath: metal with non-constant textures";
                return false;
            }
            if (!me->GetURoughness()) ur = rough;
            if (!me->GetVRoughness()) vr = rough;
            pm.kind = PT_MAT_METAL;
            eta.ToRGB(pm.eta);
            k.ToRGB(pm.k);
            pm.alpha[0] = tr_alpha(ur, me->RemapRoughness());
            pm.alpha[1] = tr_alpha(vr, me->RemapRoughness());
        } else if (const auto* gm = dynamic_cast<const GlassMaterial*>(m)) {
            // GlassMaterial::ComputeScatteringFunctions (glass.cpp:45-83)
            Spectrum kr(1.f), kt(1.f);
            Float ur = 0, vr = 0, eta = 1.5f;
            if (!constant_value(gm->GetKr(), &kr) || !constant_value(gm->GetKt(), &kt) ||
                !constant_value(gm->GetURoughness(), &ur) || !constant_value(gm->GetVRoughness(), &vr) ||
                !constant_value(gm->GetIndex(), &eta)) {
                *err = "gpupath: glass with non-constant textures";
                return false;
            }
            pm.kind = PT_MAT_GLASS;
            kr.ToRGB(pm.kr);
            kt.ToRGB(pm.kt);
            pm.ior = eta;
            pm.specular = (ur == 0 && vr == 0) ? 1 : 0;  // isSpecular before the remap (glass.cpp:56)
            pm.alpha[0] = tr_alpha(ur, gm->RemapRoughness());
            pm.alpha[1] = tr_alpha(vr, gm->RemapRoughness());
        } else if (const auto* dg = dynamic_cast<const DispersiveGlassMaterial*>(m)) {
            // DispersiveGlassMaterial::ComputeScatteringFunctions (dispersive_glass.cpp:48-123):
            // eta by Cauchy from wvls[0] between indexMin and indexMax
            Spectrum kr(1.f), kt(1.f);
            Float ur = 0, vr = 0, etaMin = 1.5f, etaMax = 1.5f;
            if (!constant_value(dg->GetKr(), &kr) || !constant_value(dg->GetKt(), &kt) ||
                !constant_value(dg->GetURoughness(), &ur) || !constant_value(dg->GetVRoughness(), &vr) ||
                !constant_value(dg->GetIndexMin(), &etaMin) || !constant_value(dg->GetIndexMax(), &etaMax)) {
                *err = "gpupath: dispersive glass with non-constant textures";
                return false;
            }
            pm.kind = PT_MAT_DISPERSIVE_GLASS;
            kr.ToRGB(pm.kr);
            kt.ToRGB(pm.kt);
            pm.ior_min = etaMin;
            pm.ior_max = etaMax;
            pm.specular = (ur == 0 && vr == 0) ? 1 : 0;
            if (dg->RemapRoughness() && !pm.specular) {  // remapped once per wavelength BSDF, cumulatively (:91-95)
                *err = "gpupath: rough dispersive glass with remaproughness is not flattened";
                return false;
            }
            pm.alpha[0] = tr_alpha(ur, dg->RemapRoughness());
            pm.alpha[1] = tr_alpha(vr, dg->RemapRoughness());
        } else if (const auto* mr = dynamic_cast<const MirrorMaterial*>(m)) {
            Spectrum kr(0.9f);  // mirror.cpp:44-52
            if (!constant_value(mr->GetKr(), &kr)) {
                *err = "gpupath: mirror with a non-constant Kr";
                return false;
            }
            pm.kind = PT_MAT_MIRROR;
            kr.ToRGB(pm.kr);
        } else if (const auto* pl = dynamic_cast<const PlasticMaterial*>(m)) {
            Spectrum kd(0.25f), ks(0.25f);  // plastic.cpp:45-70
            Float rough = 0.1f;
            if (!constant_value(pl->GetKd(), &kd) || !constant_value(pl->GetKs(), &ks) ||
                !constant_value(pl->GetRoughness(), &rough)) {
                *err = "gpupath: plastic with non-constant textures";
                return false;
            }
            pm.kind = PT_MAT_PLASTIC;
            kd.ToRGB(pm.kd);
            ks.ToRGB(pm.ks);
            pm.alpha[0] = pm.alpha[1] = tr_alpha(rough, pl->RemapRoughness());
        } else {
            *err = "gpupath: unsupported material (matte, metal, glass, dispersive glass, mirror, plastic)";
            return false;
        }
        *out = (int)f->materials.size();
        materialIndex[m] = *out;
        f->materials.push_back(pm);
        return true;
    };
    auto area_light = [&](const AreaLight* l) { return l ? lightIndex.at(l) : -1; };

    // ---- primitives in the BVH's order ----
    for (const auto& p : bvh->GetPrimitives()) {
        const auto* gp = dynamic_cast<const GeometricPrimitive*>(p.get());
        if (!gp) return fail("gpupath: only GeometricPrimitives are supported (no instancing)");
        int mi;
        if (!material(gp->GetMaterial(), &mi)) return false;
        const Shape* sh = gp->GetShape();
        if (const auto* t = dynamic_cast<const Triangle*>(sh)) {
            const TriangleMesh* mesh = t->GetMesh();
            auto it = meshBase.find(mesh);
            if (it == meshBase.end()) {  // append the mesh's world-space vertices once
                const int base = (int)f->P.size() / 3;
                it = meshBase.emplace(mesh, base).first;
                for (int v = 0; v < mesh->nVertices; ++v) {
                    f->P.insert(f->P.end(), {mesh->p[v].x, mesh->p[v].y, mesh->p[v].z});
                    if (anyN) {
                        if (mesh->n) f->N.insert(f->N.end(), {mesh->n[v].x, mesh->n[v].y, mesh->n[v].z});
                        else f->N.insert(f->N.end(), {0.f, 0.f, 0.f});
                    }
                    if (anyS) {
                        if (mesh->s) f->S.insert(f->S.end(), {mesh->s[v].x, mesh->s[v].y, mesh->s[v].z});
                        else f->S.insert(f->S.end(), {0.f, 0.f, 0.f});
                    }
                    if (anyUV) {
                        if (mesh->uv) f->UV.insert(f->UV.end(), {mesh->uv[v].x, mesh->uv[v].y});
                        else f->UV.insert(f->UV.end(), {0.f, 0.f});
                    }
                }
            }
            pt_triangle pt;
            const int* v = t->GetVertexIndices();
            for (int k = 0; k < 3; ++k) pt.v[k] = it->second + v[k];
            pt.material = mi;
            pt.area_light = area_light(gp->GetAreaLight());
            pt.flags = shape_flags(*t) | (mesh->n ? PT_TRI_HAS_N : 0u) | (mesh->uv ? PT_TRI_HAS_UV : 0u) |
                       (mesh->s ? PT_TRI_HAS_S : 0u);
            triIndex[t] = (int)f->triangles.size();
            f->prims.push_back({PT_PRIM_TRIANGLE, (int32_t)f->triangles.size()});
            f->triangles.push_back(pt);
        } else if (const auto* a = dynamic_cast<const AAPlaneShape*>(sh)) {
            pt_aaplane pl;
            std::memset(&pl, 0, sizeof pl);
            const Float lo[3] = {a->lo.x, a->lo.y, a->lo.z}, hi[3] = {a->hi.x, a->hi.y, a->hi.z};
            std::memcpy(pl.lo, lo, sizeof lo);
            std::memcpy(pl.hi, hi, sizeof hi);
            pl.axis = a->ax;
            pl.material = mi;
            pl.area_light = area_light(gp->GetAreaLight());
            pl.flags = shape_flags(*a);
            to_pt(*a->ObjectToWorld, &pl.object_to_world);
            planeIndex[a] = (int)f->planes.size();
            f->prims.push_back({PT_PRIM_AAPLANE, (int32_t)f->planes.size()});
            f->planes.push_back(pl);
        } else if (const auto* sp = dynamic_cast<const Sphere*>(sh)) {
            pt_sphere ps;  // CreateSphereShape's parameters (sphere.cpp:381-391)
            std::memset(&ps, 0, sizeof ps);
            ps.radius = sp->Radius();
            ps.zmin = sp->ZMin();
            ps.zmax = sp->ZMax();
            ps.phimax = sp->PhiMaxDegrees();
            ps.material = mi;
            ps.area_light = area_light(gp->GetAreaLight());
            ps.flags = shape_flags(*sp);
            to_pt(*sp->ObjectToWorld, &ps.object_to_world);
            sphereIndex[sp] = (int)f->spheres.size();
            f->prims.push_back({PT_PRIM_SPHERE, (int32_t)f->spheres.size()});
            f->spheres.push_back(ps);
        } else
            return fail("gpupath: unsupported shape (triangles, aaplanes and spheres are flattened)");
    }

    // ---- lights ----
    for (const auto& lp : scene.lights) {
        pt_light l;
        std::memset(&l, 0, sizeof l);
        l.n_samples = lp->nSamples;
        if (const auto* pl = dynamic_cast<const PortalArealight*>(lp.get())) {
            l.kind = PT_LIGHT_PORTAL_AREA;
            auto it = planeIndex.find(pl->shape.get());
            if (it == planeIndex.end()) return fail("gpupath: portal light whose aaplane is not in the aggregate");
            l.shape = it->second;
            l.strategy = pl->strat == PortalStrategy::SampleUniformLight ? PT_PORTAL_LIGHT
                         : pl->strat == PortalStrategy::SampleUniformPortal ? PT_PORTAL_UNIFORM
                                                                            : PT_PORTAL_PROJECTION;
            l.first_portal = (int32_t)f->portals.size();
            l.n_portals = (int32_t)pl->portals.size();
            for (const AAPortal& po : pl->portals) {  // the portal rectangle in light space (aaportal.cpp:8-12)
                pt_portal q;
                const Float lo[3] = {po.portal.lo.x, po.portal.lo.y, po.portal.lo.z};
                const Float hi[3] = {po.portal.hi.x, po.portal.hi.y, po.portal.hi.z};
                std::memcpy(q.lo, lo, sizeof lo);
                std::memcpy(q.hi, hi, sizeof hi);
                q.axis = po.portal.ax;
                q.facing_fw = po.portal.facingFw ? 1 : 0;
                f->portals.push_back(q);
            }
            pl->GetLemit().ToRGB(l.L);
            l.two_sided = pl->TwoSided() ? 1 : 0;
        } else if (const auto* dl = dynamic_cast<const DiffuseAreaLight*>(lp.get())) {
            // on a triangle, a sphere or an aaplane (creeper.pbrt:38-49)
            const Shape* shp = dl->GetShape();
            if (triIndex.count(shp)) { l.kind = PT_LIGHT_DIFFUSE_AREA; l.shape = triIndex.at(shp); }
            else if (sphereIndex.count(shp)) { l.kind = PT_LIGHT_DIFFUSE_SPHERE; l.shape = sphereIndex.at(shp); }
            else if (planeIndex.count(shp)) { l.kind = PT_LIGHT_DIFFUSE_PLANE; l.shape = planeIndex.at(shp); }
            else return fail("gpupath: diffuse area light whose shape is not in the aggregate");
            dl->GetLemit().ToRGB(l.L);
            l.two_sided = dl->TwoSided() ? 1 : 0;
        } else if (const auto* pt = dynamic_cast<const PointLight*>(lp.get())) {
            // PointLight (point.cpp:41-49): pLight; the renderer takes it as
            // LightToWorld(0, 0, 0), so a translation to pLight reproduces it exactly
            l.kind = PT_LIGHT_POINT;
            l.shape = -1;
            pt->GetIntensity().ToRGB(l.L);
            Matrix4x4 m, mi;
            const Point3f& p = pt->GetPosition();
            m.m[0][3] = p.x; m.m[1][3] = p.y; m.m[2][3] = p.z;
            mi.m[0][3] = -p.x; mi.m[1][3] = -p.y; mi.m[2][3] = -p.z;
            to_pt(Transform(m, mi), &l.light_to_world);
        } else if (const auto* il = dynamic_cast<const InfiniteAreaLight*>(lp.get())) {
            // a constant radiance is the 1x1 Lmap infinite.cpp:43-61 builds without "mapname" (L itself); any
            // 1x1 map is constant, a larger image map is not flattened
            const MIPMap<RGBSpectrum>* lm = il->GetLmap();
            if (!lm || lm->Width() != 1 || lm->Height() != 1)
                return fail("gpupath: infinite light with an image map (only a constant radiance is flattened)");
            l.kind = PT_LIGHT_INFINITE;
            l.shape = -1;
            lm->Texel(0, 0, 0).ToRGB(l.L);
            to_pt(il->GetLightToWorld(), &l.light_to_world);
        } else
            return fail("gpupath: unsupported light (diffuse area, portal, point and constant infinite lights)");
        f->lights.push_back(l);
    }

    // ---- the reference's flattened BVH ----
    // BVHAccel::nodes points at LinearBVHNode records (bvh.cpp:95-104: Bounds3f, primitivesOffset /
    // secondChildOffset, nPrimitives, axis, pad -- 32 bytes, which bvh.h only forward-declares): the node count
    // (bvh.cpp:199, a local of the constructor) is 1 + the largest index the depth-first layout reaches from
    // node 0, found by walking it; no primitives: no nodes (bvh.cpp:190)
    const unsigned char* raw = reinterpret_cast<const unsigned char*>(bvh->GetNodes());
    int nn = 0;
    if (raw && !bvh->GetPrimitives().empty()) {
        auto field = [&](int i, int off, int bytes) {
            int32_t v = 0;
            std::memcpy(&v, raw + (size_t)i * 32 + off, (size_t)bytes);
            return v;
        };
        std::vector<int> todo{0};
        while (!todo.empty()) {
            const int i = todo.back();
            todo.pop_back();
            nn = std::max(nn, i + 1);
            if ((field(i, 28, 2) & 0xffff) == 0) {  // nPrimitives == 0: interior, children i + 1 and offset
                todo.push_back(i + 1);
                todo.push_back(field(i, 24, 4));
            }
        }
    }
    f->bvh.resize((size_t)nn * 32);
    if (nn) std::memcpy(f->bvh.data(), raw, f->bvh.size());

    pt_scene_desc& d = f->desc;
    std::memset(&d, 0, sizeof d);
    d.n_vertices = (int32_t)f->P.size() / 3;
    d.P = f->P.empty() ? nullptr : f->P.data();
    d.N = anyN ? f->N.data() : nullptr;
    d.S = anyS ? f->S.data() : nullptr;
    d.UV = anyUV ? f->UV.data() : nullptr;
    d.n_triangles = (int32_t)f->triangles.size();
    d.triangles = f->triangles.data();
    d.n_planes = (int32_t)f->planes.size();
    d.planes = f->planes.data();
    d.n_prims = (int32_t)f->prims.size();
    d.prims = f->prims.data();
    d.n_materials = (int32_t)f->materials.size();
    d.materials = f->materials.data();
    d.n_lights = (int32_t)f->lights.size();
    d.lights = f->lights.data();
    d.n_portals = (int32_t)f->portals.size();
    d.portals = f->portals.data();
    d.n_spheres = (int32_t)f->spheres.size();
    d.spheres = f->spheres.data();
    d.bvh_max_prims = 4;
    d.camera = settings.camera;
    d.film = settings.film;
    d.sampler = settings.sampler;
    d.integrator = settings.integrator;
    if (d.integrator.light_strategy != PT_LIGHTS_UNIFORM && d.n_lights == 1)
        d.integrator.light_strategy = PT_LIGHTS_UNIFORM;  // one light: always uniform (lightdistrib.cpp:50)
    d.n_bvh_nodes = nn;
    d.bvh_nodes = f->bvh.data();
    return true;
}

void GpuPathIntegrator::Render(const Scene& scene) {
    GpuFlatScene flat;
    std::string err;
    if (!FlattenScene(scene, settings, &flat, &err)) {
        Error("%s", err.c_str());  // pbrt's error style: report and return (error.cpp:89-102)
        return;
    }
    pt_scene* s = nullptr;
    if (pt_init((int)devices.size(), devices.data()) != PT_OK || pt_scene_create(&flat.desc, &s) != PT_OK) {
        Error("gpupath: %s", pt_last_error());
        return;
    }
    int32_t w = 0, h = 0;
    pt_film_size(s, &w, &h);
    rgb.assign((size_t)3 * w * h, 0.f);
    if (pt_render(s, rgb.data(), &stats) != PT_OK) Error("gpupath: %s", pt_last_error());
    else if (!settings.filename.empty() &&
             pt_write_film_image(&flat.desc, settings.filename.c_str(), rgb.data()) != PT_OK)
        Error("gpupath: %s", pt_last_error());
    pt_scene_destroy(s);
}

static GpuRenderSettings common_settings(const ParamSet& params, const ParamSet& cameraParams,
                                         const ParamSet& filmParams, const std::string& filterName,
                                         const ParamSet& filterParams, const ParamSet& samplerParams,
                                         const Transform& cameraToWorld, const Camera& camera);
static std::vector<int> gpu_list(const ParamSet& params) {
    std::vector<int> gpus{0};
    int ng = 0;
    if (const int* g = params.FindInt("gpus", &ng))
        if (ng > 0) gpus.assign(g, g + ng);
    return gpus;
}
static void pixel_bounds(const ParamSet& params, pt_integrator_desc* d) {
    int np = 0;
    if (const int* pb = params.FindInt("pixelbounds", &np))
        if (np == 4) {
            d->has_pixel_bounds = 1;
            for (int i = 0; i < 4; ++i) d->pixel_bounds[i] = pb[i];
        }
}

GpuPathIntegrator* CreateGpuPathIntegrator(const ParamSet& params, const ParamSet& cameraParams,
                                           const ParamSet& filmParams, const std::string& filterName,
                                           const ParamSet& filterParams, const ParamSet& samplerParams,
                                           const Transform& cameraToWorld, std::shared_ptr<const Camera> camera) {
    GpuRenderSettings s = common_settings(params, cameraParams, filmParams, filterName, filterParams, samplerParams,
                                          cameraToWorld, *camera);
    // PathIntegrator (path.cpp:191-214; the fork's default strategy "uniform", path.cpp:210-211)
    s.integrator.kind = PT_INTEGRATOR_PATH;
    s.integrator.max_depth = params.FindOneInt("maxdepth", 5);
    s.integrator.rr_threshold = params.FindOneFloat("rrthreshold", 1.f);
    const std::string ls = params.FindOneString("lightsamplestrategy", "uniform");
    s.integrator.light_strategy = ls == "power" ? PT_LIGHTS_POWER : PT_LIGHTS_UNIFORM;
    pixel_bounds(params, &s.integrator);
    return new GpuPathIntegrator(std::move(s), std::move(camera), gpu_list(params));
}

GpuPathIntegrator* CreateGpuDirectLightingIntegrator(const ParamSet& params, const ParamSet& cameraParams,
                                                     const ParamSet& filmParams, const std::string& filterName,
                                                     const ParamSet& filterParams, const ParamSet& samplerParams,
                                                     const Transform& cameraToWorld,
                                                     std::shared_ptr<const Camera> camera) {
    GpuRenderSettings s = common_settings(params, cameraParams, filmParams, filterName, filterParams, samplerParams,
                                          cameraToWorld, *camera);
    // DirectLightingIntegrator (directlighting.cpp:86-118): "strategy" all (default) | one
    s.integrator.kind = PT_INTEGRATOR_DIRECT;
    s.integrator.max_depth = params.FindOneInt("maxdepth", 5);
    s.integrator.rr_threshold = 1.f;
    s.integrator.light_strategy = PT_LIGHTS_UNIFORM;
    const std::string st = params.FindOneString("strategy", "all");
    s.integrator.direct_strategy = st == "one" ? PT_DIRECT_ONE : PT_DIRECT_ALL;
    pixel_bounds(params, &s.integrator);
    return new GpuPathIntegrator(std::move(s), std::move(camera), gpu_list(params));
}

static GpuRenderSettings common_settings(const ParamSet& params, const ParamSet& cameraParams,
                                         const ParamSet& filmParams, const std::string& filterName,
                                         const ParamSet& filterParams, const ParamSet& samplerParams,
                                         const Transform& cameraToWorld, const Camera& camera) {
    GpuRenderSettings s;
    std::memset(&s.camera, 0, sizeof s.camera);
    std::memset(&s.film, 0, sizeof s.film);
    std::memset(&s.sampler, 0, sizeof s.sampler);
    std::memset(&s.integrator, 0, sizeof s.integrator);
    const Film* film = camera.film;
    // Film (film.cpp:213-252): resolution, crop window, scale, luminance clamp
    s.film.xres = film->fullResolution.x;
    s.film.yres = film->fullResolution.y;
    s.film.crop[0] = 0; s.film.crop[1] = 1; s.film.crop[2] = 0; s.film.crop[3] = 1;
    int nc = 0;
    if (const Float* cr = filmParams.FindFloat("cropwindow", &nc)) {
        if (nc == 4) {
            auto clamp01 = [](Float v) { return v < 0 ? 0.f : (v > 1 ? 1.f : v); };
            s.film.crop[0] = clamp01(std::min(cr[0], cr[1]));
            s.film.crop[1] = clamp01(std::max(cr[0], cr[1]));
            s.film.crop[2] = clamp01(std::min(cr[2], cr[3]));
            s.film.crop[3] = clamp01(std::max(cr[2], cr[3]));
        }
    }
    s.film.scale = filmParams.FindOneFloat("scale", 1.f);
    s.film.diagonal = filmParams.FindOneFloat("diagonal", 35.f);
    s.film.max_sample_luminance = filmParams.FindOneFloat("maxsampleluminance", Infinity);
    s.film.filter = filterName == "gaussian" ? PT_FILTER_GAUSSIAN : PT_FILTER_BOX;
    s.film.filter_radius[0] = film->filter->radius.x;
    s.film.filter_radius[1] = film->filter->radius.y;
    s.film.gaussian_alpha = filterParams.FindOneFloat("alpha", 2.f);
    s.filename = film->filename;
    // PerspectiveCamera (perspective.cpp:236-283)
    {
        pt_transform t;
        std::memset(&t, 0, sizeof t);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                t.m[4 * i + j] = cameraToWorld.GetMatrix().m[i][j];
                t.minv[4 * i + j] = cameraToWorld.GetInverseMatrix().m[i][j];
            }
        s.camera.camera_to_world = t;
    }
    s.camera.shutter_open = cameraParams.FindOneFloat("shutteropen", 0.f);
    s.camera.shutter_close = cameraParams.FindOneFloat("shutterclose", 1.f);
    s.camera.lens_radius = cameraParams.FindOneFloat("lensradius", 0.f);
    s.camera.focal_distance = cameraParams.FindOneFloat("focaldistance", 1e6f);
    const Float frame = cameraParams.FindOneFloat("frameaspectratio", Float(s.film.xres) / Float(s.film.yres));
    if (frame > 1.f) {
        s.camera.screen_window[0] = -frame; s.camera.screen_window[1] = frame;
        s.camera.screen_window[2] = -1.f; s.camera.screen_window[3] = 1.f;
    } else {
        s.camera.screen_window[0] = -1.f; s.camera.screen_window[1] = 1.f;
        s.camera.screen_window[2] = -1.f / frame; s.camera.screen_window[3] = 1.f / frame;
    }
    int nsw = 0;
    if (const Float* sw = cameraParams.FindFloat("screenwindow", &nsw))
        if (nsw == 4)
            for (int i = 0; i < 4; ++i) s.camera.screen_window[i] = sw[i];
    Float fov = cameraParams.FindOneFloat("fov", 90.f);
    const Float halffov = cameraParams.FindOneFloat("halffov", -1.f);
    if (halffov > 0.f) fov = 2.f * halffov;
    s.camera.fov = fov;
    // HaltonSampler (halton.cpp:133-139)
    s.sampler.spp = samplerParams.FindOneInt("pixelsamples", 16);
    s.sampler.sample_pixel_center = samplerParams.FindOneBool("samplepixelcenter", false) ? 1 : 0;
    (void)params;
    return s;
}

}  // namespace pbrt
