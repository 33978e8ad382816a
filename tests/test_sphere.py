"""Shape "sphere" (src/shapes/sphere.cpp) in the CPU oracle and the loader:
EFloat-bounded intersection of full and clipped spheres under transforms,
Sphere::Sample(ref) (area sampling from inside, cone sampling from outside)
and Sphere::Pdf behind a DiffuseAreaLight.

Pinned by the reference's own analytic test 'Sphere, Kd = 0.5, Le = 0.5'
(src/tests/analytic_scenes.cpp:135-165: reverse-orientation unit sphere,
camera at its centre, PathIntegrator depth 8, Halton 256, 10x10 box-filtered
film, expected radiance 1.0 +- 0.02), plus analytic irradiance from a sphere
light and analytic ray-sphere hits."""
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


def sphere_furnace(tmp_path, spp=256, maxdepth=8):
    """analytic_scenes.cpp:135-165 restated as a scene file: identity camera
    (fov 45, screen [-1,1]^2) inside a reverse-orientation unit sphere with
    Kd = 0.5 and a one-sided DiffuseAreaLight Le = 0.5."""
    return write(tmp_path, "sphere_furnace.pbrt", f"""Camera "perspective" "float fov" [45]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [10] "integer yresolution" [10]
Sampler "halton" "integer pixelsamples" [{spp}]
Integrator "path" "integer maxdepth" [{maxdepth}]
WorldBegin
AttributeBegin
  ReverseOrientation
  AreaLightSource "diffuse" "rgb L" [0.5 0.5 0.5]
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  Shape "sphere" "float radius" [1]
AttributeEnd
WorldEnd
""")


def test_sphere_furnace_known_answer(tmp_path):
    hs = ptgpu.HostScene(sphere_furnace(tmp_path))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    assert abs(float(img.mean()) - 1.0) < 0.02, float(img.mean())


def sphere_light_scene(tmp_path, r=0.5, d=4.0, L=10.0, maxdepth=1, spp=64, strategy="", extra=""):
    """Matte floor (Kd 0.5) lit by a sphere light of radius r centred at height
    d; narrow camera looking straight down at the origin."""
    return write(tmp_path, "sphere_light.pbrt", f"""LookAt 0 0 2  0 0 0  0 1 0
Camera "perspective" "float fov" [0.5]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [8] "integer yresolution" [8]
Sampler "halton" "integer pixelsamples" [{spp}]
Integrator "path" "integer maxdepth" [{maxdepth}] {strategy}
WorldBegin
AttributeBegin
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  Shape "trianglemesh" "point P" [-50 -50 0  50 -50 0  50 50 0  -50 50 0] "integer indices" [0 1 2 0 2 3]
AttributeEnd
AttributeBegin
  Translate 0 0 {d}
  AreaLightSource "area" "rgb L" [{L} {L} {L}]
  Material "matte" "rgb Kd" [0 0 0]
  Shape "sphere" "float radius" [{r}]
AttributeEnd
{extra}
WorldEnd
""")


def test_sphere_light_irradiance(tmp_path):
    """Lambertian floor under a sphere light: L_o = Kd L sin^2(theta_max)
    = Kd L (r/d)^2 straight below the centre (cone sampling + MIS)."""
    r, d, L = 0.5, 4.0, 10.0
    hs = ptgpu.HostScene(sphere_light_scene(tmp_path, r=r, d=d, L=L))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    expect = 0.5 * L * (r / d) ** 2
    assert abs(float(img.mean()) - expect) < 0.01 * expect, (float(img.mean()), expect)


def test_sphere_light_power_strategy(tmp_path):
    """Two sphere lights under "power" light selection: Power() uses
    Sphere::Area (diffuse.cpp:62-64); the estimate is unchanged."""
    r, d, L = 0.5, 4.0, 10.0
    extra = 'AttributeBegin\n  Translate 30 0 6\n  AreaLightSource "area" "rgb L" [3 3 3]\n' \
            '  Shape "sphere" "float radius" [2]\nAttributeEnd\n'
    hs = ptgpu.HostScene(sphere_light_scene(tmp_path, r=r, d=d, L=L, spp=128, extra=extra,
                                            strategy='"string lightsamplestrategy" "power"'))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    # the second light (d' = sqrt(30^2+6^2), r' = 2) adds Kd L' cos(theta) (r'/d')^2 approximately
    d2 = math.hypot(30, 6)
    expect = 0.5 * L * (r / d) ** 2 + 0.5 * 3 * (6 / d2) * (2 / d2) ** 2
    assert abs(float(img.mean()) - expect) < 0.02 * expect, (float(img.mean()), expect)


# ---- analytic ray-sphere hits ------------------------------------------------------------------

SPHERES = [  # (transform, params, centre, radius, clip) -- clip: object-space (zmin, zmax, phimax)
    ("Translate 0 0 0", '"float radius" [1]', (0, 0, 0), 1.0, None),
    ("Translate 3 0 0", '"float radius" [0.7] "float zmin" [-0.3] "float zmax" [0.5]', (3, 0, 0), 0.7,
     (-0.3, 0.5, 360)),
    ("Translate -3 0.5 0", '"float radius" [0.9] "float phimax" [250]', (-3, 0.5, 0), 0.9, (-0.9, 0.9, 250)),
    ("Translate 0 3 0  Scale 1 1 -1", '"float radius" [0.8] "float zmax" [0.2]', (0, 3, 0), 0.8,
     (-0.8, 0.2, 360)),
]


def spheres_scene(tmp_path):
    shapes = "".join(f'AttributeBegin\n  {xf}\n  Shape "sphere" {ps}\nAttributeEnd\n' for xf, ps, *_ in SPHERES)
    return write(tmp_path, "spheres.pbrt", f"""LookAt 0 0 -10  0 0 0  0 1 0
Camera "perspective" "float fov" [40]
Film "image" "integer xresolution" [32] "integer yresolution" [32]
Sampler "halton" "integer pixelsamples" [4]
Integrator "path"
WorldBegin
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [4 4 4]
  Shape "trianglemesh" "point P" [-1 6 -1  1 6 -1  0 6 1] "integer indices" [0 1 2]
AttributeEnd
{shapes}WorldEnd
""")


def _analytic_hits(o, d, spheres, margin):
    """Closest hit per ray in float64, or -2 where the answer is within
    `margin` of a decision boundary (grazing, clip edges, ties)."""
    best = np.full(len(o), np.inf)
    who = np.full(len(o), -1)
    unsure = np.zeros(len(o), bool)
    for k, (xf, ps, c, r, clip) in enumerate(spheres):
        oc = o - np.asarray(c, np.float64)
        if "Scale 1 1 -1" in xf:
            oc = oc * [1, 1, -1]
            dd = d * [1, 1, -1]
        else:
            dd = d
        b = np.einsum("ij,ij->i", oc, dd)
        cc = np.einsum("ij,ij->i", oc, oc) - r * r
        disc = b * b - cc
        ok = disc > 0
        unsure |= np.abs(disc) < margin
        sq = np.sqrt(np.maximum(disc, 0))
        for t in (-b - sq, -b + sq):
            p = oc + t[:, None] * dd
            inside = ok & (t > 0)
            if clip is not None:
                zmin, zmax, phimax = clip
                phi = np.mod(np.arctan2(p[:, 1], p[:, 0]), 2 * np.pi)
                edge = (np.abs(p[:, 2] - zmin) < margin) | (np.abs(p[:, 2] - zmax) < margin) | \
                       (np.abs(phi - math.radians(phimax)) < margin) | (phi < margin)
                unsure |= inside & edge
                inside &= (p[:, 2] >= zmin) & (p[:, 2] <= zmax) & (phi <= math.radians(phimax))
            closer = inside & (t < best)
            unsure |= inside & (np.abs(t - best) < margin)
            best = np.where(closer, t, best)
            who = np.where(closer, k, who)
    return np.where(unsure, -2, who)


def test_sphere_hits_match_analytic(tmp_path):
    hs = ptgpu.HostScene(spheres_scene(tmp_path))
    rng = np.random.default_rng(5)
    n = 20000
    o = np.stack([rng.uniform(-5, 5, n), rng.uniform(-2, 5, n), rng.uniform(-6, -3, n)], 1)
    tgt = np.stack([rng.uniform(-4.5, 4.5, n), rng.uniform(-1.5, 4.5, n), rng.uniform(-1, 1, n)], 1)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, np.full((n, 1), np.inf)], 1).astype(np.float32)
    got = pyoracle.trace(hs.desc, rays, False)
    exp = _analytic_hits(rays[:, :3].astype(np.float64), rays[:, 3:6].astype(np.float64), SPHERES, 1e-4)
    sure = exp != -2
    got_sphere = np.where(got >= 1, got - 1, -1)        # prim 0 is the light triangle
    assert sure.mean() > 0.98
    assert (got_sphere[sure] == exp[sure]).all(), np.nonzero(got_sphere[sure] != exp[sure])[0][:5]
    assert (exp[sure] >= 0).sum() > 2000 and (exp[sure] == 1).sum() > 100 and (exp[sure] == 2).sum() > 100
    # any-hit agrees with closest-hit existence
    anyh = pyoracle.trace(hs.desc, rays, True)
    assert ((anyh != 0) == (got >= 0)).all()


def test_sphere_parameters_and_bounds(tmp_path):
    """CreateSphereShape defaults and the Sphere ctor clamps feed the BVH
    bounds (ObjectToWorld(ObjectBound()), sphere.cpp:44-47)."""
    p = write(tmp_path, "s.pbrt", """Camera "perspective"
Film "image" "integer xresolution" [8] "integer yresolution" [8]
WorldBegin
Translate 1 2 3
Shape "sphere" "float radius" [2] "float zmin" [5] "float zmax" [-0.5]
WorldEnd
""")
    hs = ptgpu.HostScene(p)
    nodes, _ = hs.bvh()
    b = nodes[0, :6].view(np.float32)
    np.testing.assert_array_equal(b, np.float32([-1, 0, 2.5, 3, 4, 5]))   # z clamped to [-0.5, 2]


def test_sphere_scene_renders_in_oracle(tmp_path):
    hs = ptgpu.HostScene(spheres_scene(tmp_path))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    assert np.isfinite(img).all() and img.mean() > 0


# ---- PointLight (lights/point.cpp) -------------------------------------------------------------

def point_light_scene(tmp_path, h=2.0, I=5.0, maxdepth=1, spp=16, extra="", strategy=""):
    return write(tmp_path, "point.pbrt", f"""LookAt 0 0 1  0 0 0  0 1 0
Camera "perspective" "float fov" [0.5]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [8] "integer yresolution" [8]
Sampler "halton" "integer pixelsamples" [{spp}]
Integrator "path" "integer maxdepth" [{maxdepth}] {strategy}
WorldBegin
AttributeBegin
  Translate 0.5 0 0
  LightSource "point" "rgb I" [{I} {I} {I}] "point from" [-0.5 0 {h}]
AttributeEnd
AttributeBegin
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  Shape "trianglemesh" "point P" [-50 -50 0  50 -50 0  50 50 0  -50 50 0] "integer indices" [0 1 2 0 2 3]
AttributeEnd
{extra}
WorldEnd
""")


def test_point_light_known_answer(tmp_path):
    """Lambertian floor straight below a point light: L_o = Kd/pi * I / h^2
    (PointLight::Sample_Li, delta light: no MIS, no BSDF sample)."""
    h, I = 2.0, 5.0
    hs = ptgpu.HostScene(point_light_scene(tmp_path, h=h, I=I))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    expect = 0.5 / math.pi * I / h ** 2
    assert abs(float(img.mean()) - expect) < 1e-3 * expect, (float(img.mean()), expect)
    # one shadow ray per sample and no BSDF-sampled light ray; closest: camera + continuation
    assert st["shadow_rays"] == 8 * 8 * 16 and st["closest_rays"] == 2 * 8 * 8 * 16
