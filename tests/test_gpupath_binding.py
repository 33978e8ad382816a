"""The reference-side drop-in (integration/gpupath.{h,cpp}): a pbrt-v3
Integrator whose Render(const Scene&) flattens the reference's own scene
objects -- BVHAccel of GeometricPrimitives (Triangle / AAPlaneShape /
Sphere), Matte / Metal / Glass / Mirror / Plastic materials, DiffuseAreaLight
(triangle, sphere, aaplane) / PortalArealight + AAPortals / PointLight /
constant InfiniteAreaLight -- into pt_scene_desc (prebuilt BVH included) and
renders through the C ABI, as "gpupath" or "gpudirectlighting".

CPU: the binding compiles against stub pbrt headers that mirror the
reference's classes (integration/pbrt_stub) and the C header.  GPU: the
driver builds the reference-style objects for a scene, renders through
GpuPathIntegrator::Render and through pt_render of the loader's description:
bit-identical images and ray / node / primitive counters."""
import os
import subprocess

import pytest

from conftest import scene_variant

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTEG = os.path.join(REPO, "integration")
DRIVER = os.path.join(INTEG, "test_gpupath")


def test_binding_compiles_against_reference_api():
    subprocess.check_call(["g++", "-std=c++14", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                           "-fsyntax-only", "-I", os.path.join(INTEG, "pbrt_stub"), "-I",
                           os.path.join(REPO, "include"), os.path.join(INTEG, "gpupath.cpp")])


def test_driver_is_built():
    """build() links the driver against libptgpu.so (it travels to the GPU box)."""
    assert os.path.exists(DRIVER), "run `make -C integration` (build() does)"


AREA_LIGHT = ('AttributeBegin\n  AreaLightSource "diffuse" "rgb L" [30 30 30]\n'
              '  Material "matte" "rgb Kd" [0.725 0.71 0.68]\n'
              '  Shape "trianglemesh" "integer indices" [0 1 2 2 3 0]\n'
              '    "point P" [213 548 227  343 548 227  343 548 332  213 548 332]\nAttributeEnd\n')


def _variant(tmp_path, kind):
    if kind == "diffuse":  # the portal light replaced by a triangle area light under the ceiling hole
        txt = open(os.path.join(REPO, "scenes", "portal_cornell.pbrt")).read()
        a = txt.index("AttributeBegin\n  ReverseOrientation")
        b = txt.index("AttributeEnd", a) + len("AttributeEnd\n")
        return scene_variant(tmp_path, res=(48, 32), spp=4, extra=[(txt[a:b], AREA_LIGHT)])
    return scene_variant(tmp_path, res=(48, 32), spp=4, strategy=kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["light", "portal", "projection", "diffuse"])
def test_render_through_binding_matches_c_abi(tmp_path, kind):
    scene = _variant(tmp_path, kind)
    r = subprocess.run([DRIVER, scene, str(tmp_path / "binding.pfm"), str(tmp_path / "direct.pfm")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("identical")
    assert os.path.getsize(tmp_path / "binding.pfm") == os.path.getsize(tmp_path / "direct.pfm")


# The reference's own scenes through Render(const Scene&) (reference scene
# files imported verbatim): lamp (DirectLighting, MetalMaterial, plymesh with
# normals and uv, two portals), sandbox (DirectLighting, PointLight, a
# PortalArealight under a rotated Transform), creeper (PointLight, a
# DiffuseAreaLight on an aaplane, Scale -1 1 1 before LookAt),
# cornell_dielectric as path (glass, a constant infinite light) and
# killeroo-simple as path (plastic, a sphere area light).
REFERENCE_SCENES = {
    "lamp": dict(name="lamp/lamp.pbrt", res=(64, 64), spp=2),
    "lamp-path": dict(name="lamp/lamp.pbrt", res=(64, 64), spp=2,
                      extra=[('Integrator "directlighting"', 'Integrator "path" "integer maxdepth" [5]'),
                             ('"integer maxdepth" [100]', '')]),
    "sandbox": dict(name="creeper/sandbox.pbrt", res=(96, 96), spp=2),
    "creeper": dict(name="creeper/creeper.pbrt", res=(96, 96), spp=2),
    "cornell-dielectric-path": dict(name="cornell_dielectric.pbrt", res=(48, 48), spp=4),
    "killeroo-path": dict(name="killeroo-simple.pbrt", res=(48, 48), spp=2,
                          extra=[('Integrator "mypath"', 'Integrator "path"')]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("which", sorted(REFERENCE_SCENES))
def test_reference_scenes_through_binding(tmp_path, which):
    scene = scene_variant(tmp_path, **REFERENCE_SCENES[which])
    r = subprocess.run([DRIVER, scene, str(tmp_path / "binding.pfm"), str(tmp_path / "direct.pfm")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("identical"), r.stdout
