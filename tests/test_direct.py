"""DirectLightingIntegrator (src/integrators/directlighting.cpp) in the CPU
oracle: UniformSampleAllLights with the per-light 2D sample arrays the
Preprocess step requests (GlobalSampler arrays, sampler.cpp:137-196),
UniformSampleOneLight, and the SpecularReflect / SpecularTransmit recursion
(integrator.cpp:639-770) with the single-lobe dielectric of
allowMultipleLobes = false (glass.cpp:62-83).

The reference's tests hold no DirectLighting renders; the integrator is
pinned by analytic answers: direct light from a point light and from the
emitting interior of a sphere (Le + Kd Le), a mirror and a glass interface
reflecting / refracting a lit surface (Kr, Fresnel R and T (eta_i/eta_t)^2),
and "all" vs "one" agreeing in expectation."""
import math
import os

import numpy as np
import pytest

import ptgpu
import pyoracle


def write(tmp_path, name, txt):
    p = os.path.join(str(tmp_path), name)
    with open(p, "w") as f:
        f.write(txt)
    return p


def integ(strategy="all", maxdepth=5):
    return f'Integrator "directlighting" "string strategy" "{strategy}" "integer maxdepth" [{maxdepth}]'


def test_loader_reads_directlighting(tmp_path):
    p = write(tmp_path, "a.pbrt", 'Camera "perspective"\nFilm "image" "integer xresolution" [4] '
              '"integer yresolution" [4]\nIntegrator "directlighting" "string strategy" "one"\nWorldBegin\nWorldEnd\n')
    hs = ptgpu.HostScene(p)
    d = ptgpu.integrator_desc(hs)
    assert (d.kind, d.direct_strategy, d.max_depth) == (1, 1, 5)


def dl_sphere_furnace(tmp_path, strategy="all", nsamples=4, spp=64):
    """Camera inside a reverse-orientation sphere (Kd 0.5, emitting Le 0.5):
    direct lighting only, so L = Le + Kd * Le = 0.75."""
    return write(tmp_path, "dl_furnace.pbrt", f"""Camera "perspective" "float fov" [45]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [10] "integer yresolution" [10]
Sampler "halton" "integer pixelsamples" [{spp}]
{integ(strategy)}
WorldBegin
AttributeBegin
  ReverseOrientation
  AreaLightSource "diffuse" "rgb L" [0.5 0.5 0.5] "integer nsamples" [{nsamples}]
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  Shape "sphere" "float radius" [1]
AttributeEnd
WorldEnd
""")


@pytest.mark.parametrize("strategy,nsamples", [("all", 1), ("all", 4), ("one", 4)])
def test_dl_sphere_furnace(tmp_path, strategy, nsamples):
    hs = ptgpu.HostScene(dl_sphere_furnace(tmp_path, strategy, nsamples))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    assert abs(float(img.mean()) - 0.75) < 0.01, float(img.mean())
    # "all" with arrays: one shadow ray per light sample (EstimateDirect per array entry)
    if strategy == "all":
        assert st["shadow_rays"] == 10 * 10 * 64 * nsamples


def point_scene(tmp_path, strategy="all", mirror=None, spp=16, maxdepth=5, extra=""):
    """Camera at z = 1 looking down at the origin.  Without `mirror`: a matte
    floor at z = 0 under a point light at z = 2.  With `mirror` (a material
    line): that material is the z = 0 quad, a matte ceiling at z = 4 is lit by
    a point light at z = 3, and a matte floor at z = -2 by a point light at
    z = -1 (seen through a transmissive interface)."""
    cam = f"""LookAt 0 0 1  0 0 0  0 1 0
Camera "perspective" "float fov" [0.5]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [8] "integer yresolution" [8]
Sampler "halton" "integer pixelsamples" [{spp}]
{integ(strategy, maxdepth)}
WorldBegin
"""
    quad = 'Shape "trianglemesh" "point P" [-50 -50 {z}  50 -50 {z}  50 50 {z}  -50 50 {z}] "integer indices" [{i}]'
    up, down = "0 1 2 0 2 3", "0 2 1 0 3 2"
    if mirror is None:
        body = f"""LightSource "point" "rgb I" [5 5 5] "point from" [0 0 2]
AttributeBegin
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  {quad.format(z=0, i=up)}
AttributeEnd
"""
    else:
        body = f"""LightSource "point" "rgb I" [5 5 5] "point from" [0 0 3]
LightSource "point" "rgb I" [2 2 2] "point from" [0 0 -1]
AttributeBegin
  {mirror}
  {quad.format(z=0, i=up)}
AttributeEnd
AttributeBegin
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  {quad.format(z=4, i=down)}
  {quad.format(z=-2, i=up)}
AttributeEnd
"""
    return write(tmp_path, "dl_point.pbrt", cam + body + extra + "WorldEnd\n")


@pytest.mark.parametrize("strategy", ["all", "one"])
def test_dl_point_light(tmp_path, strategy):
    hs = ptgpu.HostScene(point_scene(tmp_path, strategy))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    expect = 0.5 / math.pi * 5 / 2 ** 2
    assert abs(float(img.mean()) - expect) < 1e-3 * expect, (float(img.mean()), expect)


def test_dl_mirror_reflects_lit_ceiling(tmp_path):
    """SpecularReflect: camera -> mirror (Kr 0.8, FresnelNoOp) -> ceiling at
    z = 4 lit straight on by I = 5 at distance 1: 0.8 * Kd/pi * 5."""
    hs = ptgpu.HostScene(point_scene(tmp_path, mirror='Material "mirror" "rgb Kr" [0.8 0.8 0.8]'))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    expect = 0.8 * 0.5 / math.pi * 5
    assert abs(float(img.mean()) - expect) < 1e-3 * expect, (float(img.mean()), expect)


def test_dl_glass_reflects_and_refracts(tmp_path):
    """Smooth glass under DirectLighting is SpecularReflection(FresnelDielectric)
    + SpecularTransmission: at normal incidence R = 0.04 of the lit ceiling
    plus T (1/1.5)^2 = 0.96 / 2.25 of the floor below (lit by I = 2 at 1)."""
    hs = ptgpu.HostScene(point_scene(tmp_path, mirror='Material "glass" "float index" [1.5]'))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    R = ((1.5 - 1) / (1.5 + 1)) ** 2
    ceiling = 0.5 / math.pi * 5
    floor = 0.5 / math.pi * 2
    expect = R * ceiling + (1 - R) / 1.5 ** 2 * floor
    assert abs(float(img.mean()) - expect) < 2e-3 * expect, (float(img.mean()), expect)


def test_dl_maxdepth_one_has_no_specular_recursion(tmp_path):
    hs = ptgpu.HostScene(point_scene(tmp_path, mirror='Material "mirror"', maxdepth=1))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    assert float(img.max()) == 0.0          # the mirror has no diffuse part; no recursion at depth 1
    assert st["closest_rays"] == 8 * 8 * 16


def test_dl_all_and_one_agree(tmp_path):
    """Two lights of different nsamples: "all" (arrays, 2 x 3 light samples)
    and "one" estimate the same direct lighting."""
    extra = 'AttributeBegin\n  Translate 0.5 0.5 2\n  AreaLightSource "area" "rgb L" [4 4 4] "integer nsamples" [3]\n' \
            '  Shape "sphere" "float radius" [0.3]\nAttributeEnd\n'
    res = {}
    for st in ("all", "one"):
        (tmp_path / st).mkdir()
        hs = ptgpu.HostScene(point_scene(tmp_path / st, st, spp=256, extra=extra))
        img, _ = pyoracle.render(hs.desc, nthreads=8)
        res[st] = float(img.mean())
    assert abs(res["all"] - res["one"]) < 0.02 * res["all"], res


def test_dl_array_dimensions_exhaust_gracefully(tmp_path):
    """More arrays than requested (a deep specular tree uses Get2DArray more
    than maxDepth times) falls back to Get2D pairs (integrator.cpp:80-86):
    the render completes and stays finite."""
    hs = ptgpu.HostScene(point_scene(tmp_path, mirror='Material "glass" "float index" [1.5]', maxdepth=4))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    assert np.isfinite(img).all()
