// gpupath.h -- the reference-side drop-in for the MI355X path tracer: a
// pbrt-v3 Integrator whose Render(const Scene&) flattens the reference's own
// scene objects into the C ABI's pt_scene_desc (include/pt.h) and renders on
// the GPU(s).  A maintainer adds integration/gpupath.{h,cpp} to
// pbrt-v3-light-portals, applies the accessor patch listed in INTEGRATION.md
// and registers the integrator in RenderOptions::MakeIntegrator
// (src/core/api.cpp:1788-1815):
//
//     else if (IntegratorName == "gpupath")
//         integrator = CreateGpuPathIntegrator(IntegratorParams, CameraParams, FilmParams, FilterName,
//                                              FilterParams, SamplerParams, CameraToWorld[0], camera);
//
//     else if (IntegratorName == "gpudirectlighting")
//         integrator = CreateGpuDirectLightingIntegrator(IntegratorParams, CameraParams, FilmParams, FilterName,
//                                                        FilterParams, SamplerParams, CameraToWorld[0], camera);
//
// "gpupath" replaces PathIntegrator (src/integrators/path.cpp:64-214): same
// "maxdepth" / "rrthreshold" / "lightsamplestrategy" / "pixelbounds"
// parameters; "gpudirectlighting" replaces DirectLightingIntegrator
// (src/integrators/directlighting.cpp:86-118): "strategy" / "maxdepth" /
// "pixelbounds".  Both use the scene's Halton sampler and perspective camera,
// the Film's filter, crop window and file name.
#ifndef PBRT_INTEGRATORS_GPUPATH_H
#define PBRT_INTEGRATORS_GPUPATH_H

#include <memory>
#include <string>
#include <vector>

#include "core/camera.h"
#include "core/integrator.h"
#include "core/paramset.h"
#include "core/scene.h"
#include "core/transform.h"

extern "C" {
#include "pt.h"  // this repo's include/
}

namespace pbrt {

// The flattened scene: owns every array pt_scene_desc points into.
struct GpuFlatScene {
    std::vector<float> P, N, S, UV;
    std::vector<pt_triangle> triangles;
    std::vector<pt_aaplane> planes;
    std::vector<pt_sphere> spheres;
    std::vector<pt_prim> prims;
    std::vector<pt_material> materials;
    std::vector<pt_light> lights;
    std::vector<pt_portal> portals;
    std::vector<unsigned char> bvh;  // LinearBVHNode records, 32 bytes each
    pt_scene_desc desc;
};

// Camera / film / sampler / integrator settings, read once from the same
// ParamSets the reference's Create* functions parse.
struct GpuRenderSettings {
    pt_camera_desc camera;
    pt_film_desc film;
    pt_sampler_desc sampler;
    pt_integrator_desc integrator;
    std::string filename;
};

// Flatten `scene` (Scene::aggregate = a BVHAccel of GeometricPrimitives over
// Triangle / AAPlaneShape / Sphere shapes; Matte, Metal, Glass, dispersive
// glass, Mirror and Plastic materials with constant textures; DiffuseAreaLight on a triangle,
// sphere or aaplane, PortalArealight, PointLight and a constant
// InfiniteAreaLight) into `out`.  Returns false and fills `err` for anything
// the device path does not implement.
bool FlattenScene(const Scene& scene, const GpuRenderSettings& settings, GpuFlatScene* out, std::string* err);

class GpuPathIntegrator : public Integrator {
  public:
    GpuPathIntegrator(GpuRenderSettings settings, std::shared_ptr<const Camera> camera,
                      std::vector<int> devices = {0})
        : settings(std::move(settings)), camera(std::move(camera)), devices(std::move(devices)) {}
    // Integrator::Render (integrator.h:53-58): flatten, render every tile on
    // the GPUs, write the Film's image (Film::WriteImage, film.cpp:169-211).
    void Render(const Scene& scene) override;
    // The rendered RGB image of the last Render (cropped pixel bounds, 3
    // floats per pixel) and its reference counters.
    const std::vector<float>& Image() const { return rgb; }
    const pt_stats& Stats() const { return stats; }

  private:
    GpuRenderSettings settings;
    std::shared_ptr<const Camera> camera;
    std::vector<int> devices;
    std::vector<float> rgb;
    pt_stats stats{};
};

// CreatePathIntegrator's parameters (path.cpp:191-214) plus the camera, film,
// filter and sampler ParamSets of RenderOptions (perspective.cpp:236-283,
// film.cpp:213-252, filters/{box,gaussian}.cpp, halton.cpp:133-139).
// Multiple GPUs of one process: "integer gpus" [ids...] (default [0]).
GpuPathIntegrator* CreateGpuPathIntegrator(const ParamSet& params, const ParamSet& cameraParams,
                                           const ParamSet& filmParams, const std::string& filterName,
                                           const ParamSet& filterParams, const ParamSet& samplerParams,
                                           const Transform& cameraToWorld, std::shared_ptr<const Camera> camera);

// CreateDirectLightingIntegrator's parameters (directlighting.cpp:86-118):
// "strategy" all | one, "maxdepth" (default 5), "pixelbounds"; the rest as above.
GpuPathIntegrator* CreateGpuDirectLightingIntegrator(const ParamSet& params, const ParamSet& cameraParams,
                                                     const ParamSet& filmParams, const std::string& filterName,
                                                     const ParamSet& filterParams, const ParamSet& samplerParams,
                                                     const Transform& cameraToWorld,
                                                     std::shared_ptr<const Camera> camera);

}  // namespace pbrt

#endif  // PBRT_INTEGRATORS_GPUPATH_H
