// test_gpupath.cpp -- drives the GpuPathIntegrator binding the way pbrt-v3
// would: the scene is turned into reference-style objects (TriangleMesh /
// Triangle / AAPlaneShape / Sphere shapes, Matte / Metal / Glass / Mirror /
// Plastic materials with ConstantTextures, DiffuseAreaLight / PortalArealight
// with AAPortals / PointLight / InfiniteAreaLight, GeometricPrimitives in a
// BVHAccel holding the reference-order SAH build, Scene, Film, Camera and the
// RenderOptions ParamSets), the "gpupath" or "gpudirectlighting" integrator
// (by the scene's Integrator) renders it through Render(scene), and the image
// is compared with pt_render of the loader's own description.
//
//   test_gpupath scene.pbrt binding.pfm direct.pfm
//
// Exit 0: identical images and counters; 3: they differ; 1: error.
#include <cstdio>
#include <cstring>
#include <map>

#include "gpupath.h"
#include "accelerators/bvh.h"
#include "lights/infinite.h"
#include "lights/point.h"
#include "lights/portal_arealight.h"
#include "materials/dispersive_glass.h"
#include "materials/glass.h"
#include "materials/matte.h"
#include "materials/metal.h"
#include "materials/mirror.h"
#include "materials/plastic.h"
#include "shapes/plane.h"
#include "shapes/sphere.h"
#include "shapes/triangle.h"
#include "textures/constant.h"

using namespace pbrt;

static Transform xf(const pt_transform& t) {
    Matrix4x4 m, mi;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            m.m[i][j] = t.m[4 * i + j];
            mi.m[i][j] = t.minv[4 * i + j];
        }
    return Transform(m, mi);
}

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: test_gpupath scene.pbrt binding.pfm direct.pfm\n");
        return 1;
    }
    pt_host_scene* hs = nullptr;
    if (pt_load_pbrt(argv[1], &hs) != PT_OK) {
        std::fprintf(stderr, "load: %s\n", pt_last_error());
        return 1;
    }
    const pt_scene_desc& d = *pt_host_scene_desc(hs);

    // ---- reference-style scene objects ----
    // Meshes are already in world space; a shape's ObjectToWorld only decides
    // transformSwapsHandedness (identity, or a mirror for flagged triangles).
    Matrix4x4 mirror;
    mirror.m[0][0] = -1;
    auto identity = std::make_shared<Transform>();
    auto mirrored = std::make_shared<Transform>(mirror, mirror);
    std::vector<Point3f> P(d.n_vertices);
    std::vector<Normal3f> N(d.N ? d.n_vertices : 0);
    std::vector<Vector3f> S(d.S ? d.n_vertices : 0);
    std::vector<Point2f> UV(d.UV ? d.n_vertices : 0);
    for (int i = 0; i < d.n_vertices; ++i) {
        P[i] = Point3f(d.P[3 * i], d.P[3 * i + 1], d.P[3 * i + 2]);
        if (d.N) N[i] = Normal3f(d.N[3 * i], d.N[3 * i + 1], d.N[3 * i + 2]);
        if (d.S) S[i] = Vector3f(d.S[3 * i], d.S[3 * i + 1], d.S[3 * i + 2]);
        if (d.UV) UV[i] = Point2f(d.UV[2 * i], d.UV[2 * i + 1]);
    }
    // one TriangleMesh per combination of per-vertex attributes present
    const uint32_t attr = PT_TRI_HAS_N | PT_TRI_HAS_UV | PT_TRI_HAS_S;
    std::map<uint32_t, std::vector<int>> groups;
    for (int t = 0; t < d.n_triangles; ++t) groups[d.triangles[t].flags & attr].push_back(t);
    std::vector<std::shared_ptr<Shape>> triShape(d.n_triangles);
    for (auto& g : groups) {
        std::vector<int> idx;
        for (int t : g.second)
            for (int k = 0; k < 3; ++k) idx.push_back(d.triangles[t].v[k]);
        auto mesh = std::make_shared<TriangleMesh>((int)g.second.size(), idx.data(), d.n_vertices, P.data(),
                                                   (g.first & PT_TRI_HAS_S) ? S.data() : nullptr,
                                                   (g.first & PT_TRI_HAS_N) ? N.data() : nullptr,
                                                   (g.first & PT_TRI_HAS_UV) ? UV.data() : nullptr);
        for (size_t k = 0; k < g.second.size(); ++k) {
            const pt_triangle& tr = d.triangles[g.second[k]];
            const Transform* o2w = (tr.flags & PT_TRI_SWAPS_HANDEDNESS) ? mirrored.get() : identity.get();
            triShape[g.second[k]] = std::make_shared<Triangle>(o2w, o2w, (tr.flags & PT_TRI_REVERSE_ORIENTATION) != 0,
                                                               mesh, (int)k);
        }
    }
    std::vector<std::shared_ptr<Transform>> keep;
    std::vector<std::shared_ptr<AAPlaneShape>> planeShape(d.n_planes);
    for (int i = 0; i < d.n_planes; ++i) {
        const pt_aaplane& p = d.planes[i];
        auto o2w = std::make_shared<Transform>(xf(p.object_to_world));
        pt_transform inv;
        std::memcpy(inv.m, p.object_to_world.minv, 64);
        std::memcpy(inv.minv, p.object_to_world.m, 64);
        auto w2o = std::make_shared<Transform>(xf(inv));
        keep.push_back(o2w);
        keep.push_back(w2o);
        planeShape[i] = std::make_shared<AAPlaneShape>(o2w.get(), w2o.get(), (p.flags & PT_TRI_REVERSE_ORIENTATION) != 0,
                                                       Point3f(p.lo[0], p.lo[1], p.lo[2]),
                                                       Point3f(p.hi[0], p.hi[1], p.hi[2]), p.axis, true);
    }
    std::vector<std::shared_ptr<Sphere>> sphereShape(d.n_spheres);
    for (int i = 0; i < d.n_spheres; ++i) {
        const pt_sphere& p = d.spheres[i];
        auto o2w = std::make_shared<Transform>(xf(p.object_to_world));
        pt_transform inv;
        std::memcpy(inv.m, p.object_to_world.minv, 64);
        std::memcpy(inv.minv, p.object_to_world.m, 64);
        auto w2o = std::make_shared<Transform>(xf(inv));
        keep.push_back(o2w);
        keep.push_back(w2o);
        sphereShape[i] = std::make_shared<Sphere>(o2w.get(), w2o.get(), (p.flags & PT_TRI_REVERSE_ORIENTATION) != 0,
                                                  p.radius, p.zmin, p.zmax, p.phimax);
    }
    // materials: constant textures holding the loader's values; the microfacet
    // ones carry alpha already remapped, so remapRoughness = false
    auto cs = [](const float* v) { return std::make_shared<ConstantTexture<Spectrum>>(Spectrum::FromRGB(v)); };
    auto cf = [](float v) { return std::make_shared<ConstantTexture<Float>>(v); };
    std::vector<std::shared_ptr<Material>> mats(d.n_materials);
    for (int i = 0; i < d.n_materials; ++i) {
        const pt_material& m = d.materials[i];
        if (m.kind == PT_MAT_MATTE)
            mats[i] = std::make_shared<MatteMaterial>(cs(m.kd), cf(m.sigma), nullptr);
        else if (m.kind == PT_MAT_METAL)
            mats[i] = std::make_shared<MetalMaterial>(cs(m.eta), cs(m.k), cf(m.alpha[0]), cf(m.alpha[0]), cf(m.alpha[1]),
                                                      nullptr, false);
        else if (m.kind == PT_MAT_GLASS)
            mats[i] = std::make_shared<GlassMaterial>(cs(m.kr), cs(m.kt), cf(m.specular ? 0.f : m.alpha[0]),
                                                      cf(m.specular ? 0.f : m.alpha[1]), cf(m.ior), nullptr, false);
        else if (m.kind == PT_MAT_DISPERSIVE_GLASS)
            mats[i] = std::make_shared<DispersiveGlassMaterial>(cs(m.kr), cs(m.kt), cf(m.specular ? 0.f : m.alpha[0]),
                                                                cf(m.specular ? 0.f : m.alpha[1]), cf(m.ior_min),
                                                                cf(m.ior_max), nullptr, false);
        else if (m.kind == PT_MAT_MIRROR)
            mats[i] = std::make_shared<MirrorMaterial>(cs(m.kr), nullptr);
        else if (m.kind == PT_MAT_PLASTIC)
            mats[i] = std::make_shared<PlasticMaterial>(cs(m.kd), cs(m.ks), cf(m.alpha[0]), nullptr, false);
        else if (m.kind != PT_MAT_NONE) {
            std::fprintf(stderr, "test_gpupath: material kind %d is not built by this driver\n", m.kind);
            return 1;
        }
    }
    std::vector<std::shared_ptr<Light>> lights;
    std::vector<std::shared_ptr<AreaLight>> areaLights(d.n_lights);
    for (int i = 0; i < d.n_lights; ++i) {
        const pt_light& l = d.lights[i];
        const Spectrum L = Spectrum::FromRGB(l.L);
        if (l.kind == PT_LIGHT_PORTAL_AREA) {
            std::vector<AAPortal> portals;
            for (int k = 0; k < l.n_portals; ++k) {
                const pt_portal& po = d.portals[l.first_portal + k];
                portals.emplace_back(Point3f(po.lo[0], po.lo[1], po.lo[2]), Point3f(po.hi[0], po.hi[1], po.hi[2]),
                                     po.axis, po.facing_fw != 0, *planeShape[l.shape]);
            }
            const PortalStrategy st = l.strategy == PT_PORTAL_LIGHT ? PortalStrategy::SampleUniformLight
                                      : l.strategy == PT_PORTAL_UNIFORM ? PortalStrategy::SampleUniformPortal
                                                                        : PortalStrategy::SampleProjection;
            areaLights[i] = std::make_shared<PortalArealight>(L, l.n_samples, planeShape[l.shape], std::move(portals),
                                                              st, l.two_sided != 0);
        } else if (l.kind == PT_LIGHT_DIFFUSE_AREA) {
            areaLights[i] = std::make_shared<DiffuseAreaLight>(L, l.n_samples, triShape[l.shape], l.two_sided != 0);
        } else if (l.kind == PT_LIGHT_DIFFUSE_SPHERE) {
            areaLights[i] = std::make_shared<DiffuseAreaLight>(L, l.n_samples, sphereShape[l.shape], l.two_sided != 0);
        } else if (l.kind == PT_LIGHT_DIFFUSE_PLANE) {
            areaLights[i] = std::make_shared<DiffuseAreaLight>(L, l.n_samples, planeShape[l.shape], l.two_sided != 0);
        } else if (l.kind == PT_LIGHT_POINT) {
            // pLight = LightToWorld(Point3f(0, 0, 0)) (point.h:55; Transform::operator()(Point3f))
            const float* m = l.light_to_world.m;
            Point3f p(m[3], m[7], m[11]);
            if (m[15] != 1) p = Point3f(m[3] / m[15], m[7] / m[15], m[11] / m[15]);
            lights.push_back(std::make_shared<PointLight>(p, L));
            continue;
        } else if (l.kind == PT_LIGHT_INFINITE) {
            lights.push_back(std::make_shared<InfiniteAreaLight>(xf(l.light_to_world), L, l.n_samples));
            continue;
        } else {
            std::fprintf(stderr, "test_gpupath: light kind %d is not built by this driver\n", l.kind);
            return 1;
        }
        lights.push_back(areaLights[i]);
    }
    std::vector<std::shared_ptr<Primitive>> prims;  // RenderOptions::primitives, scene order
    for (int i = 0; i < d.n_prims; ++i) {
        const pt_prim& p = d.prims[i];
        if (p.kind == PT_PRIM_TRIANGLE) {
            const pt_triangle& t = d.triangles[p.index];
            prims.push_back(std::make_shared<GeometricPrimitive>(
                triShape[p.index], mats[t.material], t.area_light >= 0 ? areaLights[t.area_light] : nullptr));
        } else if (p.kind == PT_PRIM_AAPLANE) {
            const pt_aaplane& pl = d.planes[p.index];
            prims.push_back(std::make_shared<GeometricPrimitive>(
                planeShape[p.index], mats[pl.material], pl.area_light >= 0 ? areaLights[pl.area_light] : nullptr));
        } else if (p.kind == PT_PRIM_SPHERE) {
            const pt_sphere& sp = d.spheres[p.index];
            prims.push_back(std::make_shared<GeometricPrimitive>(
                sphereShape[p.index], mats[sp.material], sp.area_light >= 0 ? areaLights[sp.area_light] : nullptr));
        } else {
            std::fprintf(stderr, "test_gpupath: prim kind %d is not built by this driver\n", p.kind);
            return 1;
        }
    }
    // BVHAccel: the reference-order SAH build (bvh.cpp:236-402, restated by pt_build_bvh_host)
    int32_t nn = 0, np = 0;
    if (pt_build_bvh_host(&d, &nn, nullptr, 0, &np, nullptr, 0) != PT_OK) return 1;
    std::vector<LinearBVHNode> nodes(nn);
    std::vector<int32_t> order(np);
    if (pt_build_bvh_host(&d, &nn, nodes.data(), nn, &np, order.data(), np) != PT_OK) return 1;
    std::vector<std::shared_ptr<Primitive>> ordered;
    for (int32_t k : order) ordered.push_back(prims[k]);
    Scene scene(std::make_shared<BVHAccel>(std::move(ordered), std::move(nodes)), lights);

    // ---- RenderOptions ParamSets and the camera ----
    ParamSet cameraPs, filmPs, filterPs, samplerPs, integratorPs;
    cameraPs.AddFloat("fov", {d.camera.fov});
    cameraPs.AddFloat("screenwindow", {d.camera.screen_window[0], d.camera.screen_window[1], d.camera.screen_window[2],
                                       d.camera.screen_window[3]});
    cameraPs.AddFloat("lensradius", {d.camera.lens_radius});
    cameraPs.AddFloat("focaldistance", {d.camera.focal_distance});
    cameraPs.AddFloat("shutteropen", {d.camera.shutter_open});
    cameraPs.AddFloat("shutterclose", {d.camera.shutter_close});
    filmPs.AddFloat("cropwindow", {d.film.crop[0], d.film.crop[1], d.film.crop[2], d.film.crop[3]});
    filmPs.AddFloat("scale", {d.film.scale});
    filmPs.AddFloat("diagonal", {d.film.diagonal});
    filmPs.AddFloat("maxsampleluminance", {d.film.max_sample_luminance});
    filterPs.AddFloat("alpha", {d.film.gaussian_alpha});
    samplerPs.AddInt("pixelsamples", {d.sampler.spp});
    samplerPs.AddBool("samplepixelcenter", d.sampler.sample_pixel_center != 0);
    integratorPs.AddInt("maxdepth", {d.integrator.max_depth});
    integratorPs.AddString("strategy", d.integrator.direct_strategy == PT_DIRECT_ONE ? "one" : "all");
    integratorPs.AddFloat("rrthreshold", {d.integrator.rr_threshold});
    integratorPs.AddString("lightsamplestrategy", d.integrator.light_strategy == PT_LIGHTS_POWER ? "power" : "uniform");
    if (d.integrator.has_pixel_bounds)
        integratorPs.AddInt("pixelbounds", {d.integrator.pixel_bounds[0], d.integrator.pixel_bounds[1],
                                            d.integrator.pixel_bounds[2], d.integrator.pixel_bounds[3]});
    Film* film = new Film(Point2i(d.film.xres, d.film.yres),
                          std::unique_ptr<Filter>(new Filter(Vector2f(d.film.filter_radius[0], d.film.filter_radius[1]))),
                          d.film.diagonal, argv[2]);
    auto camera = std::make_shared<Camera>(film);
    // RenderOptions::MakeIntegrator: "gpudirectlighting" for a DirectLighting scene, else "gpupath"
    const std::string filterName = d.film.filter == PT_FILTER_GAUSSIAN ? "gaussian" : "box";
    std::unique_ptr<GpuPathIntegrator> integ(
        d.integrator.kind == PT_INTEGRATOR_DIRECT
            ? CreateGpuDirectLightingIntegrator(integratorPs, cameraPs, filmPs, filterName, filterPs, samplerPs,
                                                xf(d.camera.camera_to_world), camera)
            : CreateGpuPathIntegrator(integratorPs, cameraPs, filmPs, filterName, filterPs, samplerPs,
                                      xf(d.camera.camera_to_world), camera));
    if (d.integrator.kind != PT_INTEGRATOR_PATH && d.integrator.kind != PT_INTEGRATOR_DIRECT) {
        std::fprintf(stderr, "test_gpupath: integrator kind %d is not bound\n", d.integrator.kind);
        return 1;
    }
    integ->Render(scene);
    if (integ->Image().empty()) return 1;

    // ---- the loader's description through pt_render ----
    pt_scene* s = nullptr;
    const int32_t dev0 = 0;
    if (pt_init(1, &dev0) != PT_OK || pt_scene_create(&d, &s) != PT_OK) {
        std::fprintf(stderr, "direct: %s\n", pt_last_error());
        return 1;
    }
    int32_t w = 0, h = 0;
    pt_film_size(s, &w, &h);
    std::vector<float> rgb((size_t)3 * w * h);
    pt_stats st{};
    if (pt_render(s, rgb.data(), &st) != PT_OK || pt_write_film_image(&d, argv[3], rgb.data()) != PT_OK) {
        std::fprintf(stderr, "direct: %s\n", pt_last_error());
        return 1;
    }
    pt_scene_destroy(s);
    pt_host_scene_free(hs);
    const pt_stats& bs = integ->Stats();
    const bool same = rgb.size() == integ->Image().size() &&
                      std::memcmp(rgb.data(), integ->Image().data(), rgb.size() * sizeof(float)) == 0 &&
                      bs.closest_rays == st.closest_rays && bs.shadow_rays == st.shadow_rays &&
                      bs.node_visits == st.node_visits && bs.prim_tests == st.prim_tests;
    std::printf("%s: %dx%d rays %llu+%llu nodes %llu prims %llu\n", same ? "identical" : "DIFFERENT", w, h,
                (unsigned long long)bs.closest_rays, (unsigned long long)bs.shadow_rays,
                (unsigned long long)bs.node_visits, (unsigned long long)bs.prim_tests);
    return same ? 0 : 3;
}
