"""The reference's own unit tests for the hot path's triangle and
Distribution1D code, restated against the oracle (CPU) -- and, for the ray
queries, against the device through the C ABI (`-m gpu`).

  * Triangle.Reintersect   src/tests/shapes.cpp:155-206
  * Triangle.Sampling      src/tests/shapes.cpp:211-270
  * Triangle.BadCases      src/tests/shapes.cpp:545-560
  * Triangle.SolidAngle    src/tests/shapes.cpp:274-314
  * Sphere.SolidAngle      src/tests/shapes.cpp:316-349
  * FullSphere.Reintersect, PartialSphere.Normal, PartialSphere.Reintersect
                           src/tests/shapes.cpp:376-498
  * Distribution1D.Discrete / Continuous  src/tests/sampling.cpp:231-303
  * BSDFSampling.Lambertian src/tests/bsdfs.cpp:371-485 (tests/test_materials.py)

The RNG streams (RNG(i), pExp / pUnif, UniformSampleSphere) are the
reference test's own, regenerated inside the oracle (oracle_test_* hooks), so
the triangles and rays are the ones the reference's test binary checks.
"""
import os

import numpy as np
import pytest

import pyoracle

ONE_MINUS_EPS = float(np.float32(float.fromhex("0x1.fffffep-1")))


def test_triangle_reintersect():
    """1000 random triangles (log-uniform coordinates over 1e-8..1e8), 10000
    rays leaving each intersection point by SpawnRay and 10000 by SpawnRayTo:
    none may re-hit the triangle (Intersect or IntersectP)."""
    used = 0
    for i in range(1000):
        case = pyoracle.reintersect_case(i, 10000)
        if case is None:
            continue
        used += 1
        assert case[2] == 0, (i, case[2])
    assert used > 900      # the reference skips only degenerate / round-off-missed seeds


def test_triangle_sampling():
    """Triangle::Sample through Shape::Sample(ref) (solid-angle pdf) agrees
    with a uniform-spherical-sampling estimate of the subtended solid angle
    within 10 % (absolute below 1e-4), for 30 random triangles."""
    def error(a, b):
        if abs(a) < 1e-4 or abs(b) < 1e-4:
            return abs(a - b)
        return abs((a - b) / b)
    checked = 0
    for i in range(30):
        case = pyoracle.triangle_sampling_case(i)
        if case is None:
            continue
        unif, tri_est, _, _, bad = case
        assert bad == 0, i                      # EXPECT_GT(pdf, 0)
        if tri_est > 1e-3:
            checked += 1
            assert error(tri_est, unif) < 0.1, (i, unif, tri_est)
    assert checked >= 10


def girard_solid_angle(tri, p):
    """Triangle::SolidAngle (triangle.cpp:611-647): Girard's excess of the
    spherical triangle of the vertices projected about p (in double here)."""
    a = [np.asarray(v, np.float64) - np.asarray(p, np.float64) for v in tri]
    a = [v / np.linalg.norm(v) for v in a]
    c01, c12, c20 = np.cross(a[0], a[1]), np.cross(a[1], a[2]), np.cross(a[2], a[0])
    c01, c12, c20 = [c / np.linalg.norm(c) if np.dot(c, c) > 0 else c for c in (c01, c12, c20)]
    ang = lambda x, y: np.arccos(np.clip(np.dot(x, -y), -1, 1))
    return abs(ang(c01, c12) + ang(c12, c20) + ang(c20, c01) - np.pi)


def test_triangle_solid_angle():
    """Triangle.SolidAngle: for 50 random triangles (RNG(100 + i), pUnif over
    +-10) seen from a point pushed outside the box, the Triangle::Sample
    (Shape::Sample(ref), shape.cpp:56-74) estimate over 64 K radical-inverse
    samples agrees with the closed-form solid angle within 1.5 % (absolute
    when either is below 1e-4); every sample's pdf is positive."""
    def error(a, b):
        if abs(a) < 1e-4 or abs(b) < 1e-4:
            return abs(a - b)
        return abs((a - b) / b)
    checked = 0
    for i in range(50):
        case = pyoracle.triangle_sampling_case(100 + i, 64 * 1024)
        if case is None:
            continue
        _, tri_est, tri, pc, bad = case
        assert bad == 0, i
        sa = girard_solid_angle(tri, pc)
        assert error(sa, tri_est) < .015, (i, sa, tri_est)
        checked += 1
    assert checked >= 45


def sphere_scene(tmp_path, name, radius=1.0, zmin=-1.0, zmax=1.0, phimax=360.0, xf=""):
    """A one-sphere .pbrt (parameters written so they round-trip, %.9g)."""
    txt = f"""LookAt 0 0 -10 0 0 0 0 1 0
Camera "perspective"
Film "image" "integer xresolution" [4] "integer yresolution" [4]
Sampler "halton" "integer pixelsamples" [1]
WorldBegin
{xf}
Shape "sphere" "float radius" [{radius:.9g}] "float zmin" [{zmin:.9g}] "float zmax" [{zmax:.9g}] "float phimax" [{phimax:.9g}]
WorldEnd
"""
    p = os.path.join(str(tmp_path), name)
    with open(p, "w") as f:
        f.write(txt)
    return p


def mc_sphere_rays(p, n):
    """mcSolidAngle's rays (shapes.cpp:318-328): UniformSampleSphere of the
    (RadicalInverse(0, i), RadicalInverse(1, i)) points from p."""
    u0 = np.array([pyoracle.radical_inverse(0, k) for k in range(n)], np.float32)
    u1 = np.array([pyoracle.radical_inverse(1, k) for k in range(n)], np.float32)
    z = (np.float32(1) - np.float32(2) * u0).astype(np.float32)
    r = np.sqrt(np.maximum(np.float32(0), np.float32(1) - z * z)).astype(np.float32)
    phi = (np.float32(2 * np.pi) * u1).astype(np.float32)
    d = np.stack([r * np.cos(phi).astype(np.float32), r * np.sin(phi).astype(np.float32), z], 1).astype(np.float32)
    return np.ascontiguousarray(np.concatenate([np.broadcast_to(np.float32(p), (n, 3)), d,
                                                np.full((n, 1), np.inf, np.float32)], 1), np.float32)


SPHERE_XF = "Translate 1 .5 -.8\nRotate 30 1 0 0"   # Translate(1, .5, -.8) * RotateX(30)


def _sphere_cone_solid_angle(p, center=(1, .5, -.8), radius=1.0):
    """Sphere::SolidAngle (sphere.cpp:317-324) in float."""
    f = np.float32
    d2 = f(sum((f(a) - f(b)) * (f(a) - f(b)) for a, b in zip(p, center)))
    if d2 <= f(radius) * f(radius):
        return 4 * np.pi
    sin2 = f(f(radius) * f(radius) / d2)
    cos = np.sqrt(max(f(0), f(1) - sin2))
    return float(f(2 * np.pi) * (f(1) - f(cos)))


def test_sphere_solid_angle(tmp_path):
    """Sphere.SolidAngle: the unit sphere under Translate(1, .5, -.8) *
    RotateX(30); the quasi-Monte Carlo IntersectP estimate of its solid angle
    (128 K rays) is 4 pi within .01 from inside and matches the closed form
    within .001 from outside (the oracle's Sphere::IntersectP with its EFloat
    error bounds and transforms)."""
    import ptgpu
    hs = ptgpu.HostScene(sphere_scene(tmp_path, "sa.pbrt", xf=SPHERE_XF))
    n = 128 * 1024
    for p, tol in (((1, .9, -.8), .01), ((-.25, -1, .8), .001)):
        hits = pyoracle.trace(hs.desc, mc_sphere_rays(p, n), True)
        mc = float(np.count_nonzero(hits)) / (1 / (4 * np.pi) * n)
        assert abs(mc - _sphere_cone_solid_angle(p)) < tol, (p, mc, _sphere_cone_solid_angle(p))


@pytest.mark.parametrize("partial", [False, True])
def test_sphere_reintersect(partial):
    """FullSphere.Reintersect (100 seeds) and PartialSphere.Reintersect (100
    seeds: clipped z range and phiMax): 10000 SpawnRay(Faceforward(w, n)) and
    10000 SpawnRayTo rays leave each intersection point; none may re-hit the
    (convex) sphere under Intersect or IntersectP."""
    used = 0
    for i in range(100):
        case = pyoracle.sphere_case(i, partial, "reintersect")
        if case is None:
            continue
        assert case[2] == 0, (i, case[0], case[2])
        used += 1
    assert used >= 30


def test_partial_sphere_normal():
    """PartialSphere.Normal: the SurfaceInteraction normal of a partial sphere
    hit points along the hit point (identity transform): Dot(Normalize(n),
    Normalize(p)) == 1 within EXPECT_FLOAT_EQ's 4 ulps."""
    used = 0
    for i in range(100):
        case = pyoracle.sphere_case(i, True, "normal")
        if case is None:
            continue
        assert abs(case[1] - 1.0) <= 4 * np.finfo(np.float32).eps, (i, case)
        used += 1
    assert used >= 30


BAD_TRI = np.array([[-1113.45459, -79.049614, -56.2431908],
                    [-1113.45459, -87.0922699, -56.2431908],
                    [-1113.45459, -79.2090149, -56.2431908]], np.float32)
BAD_O = np.array([-1081.47925, 99.9999542, 87.7701111], np.float32)
BAD_D = np.array([-32.1072998, -183.355865, -144.607635], np.float32)


@pytest.mark.parametrize("tmax", [np.inf, 0.9999])
def test_triangle_bad_cases(tmax):
    """Triangle.BadCases: the degenerate triangle is never hit.  In the fork
    `Ray(o, d, 0.9999)` binds 0.9999 to the new `wvls` argument
    (geometry.h:1024-1027), so tMax is Infinity there; upstream's 0.9999 is
    checked as well.  The test asserts only Intersect; IntersectP has no
    degenerate-triangle rejection (triangle.cpp:427-574 returns after the
    deltaT test), so the shadow query reports the bogus hit -- the behaviour
    both oracle and device must reproduce."""
    ray = np.concatenate([BAD_O, BAD_D, [tmax]]).astype(np.float32)
    assert pyoracle.triangle_intersect(BAD_TRI, ray, any_hit=False)[0] is False
    assert pyoracle.triangle_intersect(BAD_TRI, ray, any_hit=True)[0] is True


def test_distribution1d_discrete():
    """Distribution1D.Discrete (src/tests/sampling.cpp:231-280), exact."""
    func = [0, 1., 0., 3.]
    assert [pyoracle.dist1d(func, "pdf", i) for i in range(4)] == [0, .25, 0, .75]
    off, pdf, _ = pyoracle.dist1d(func, "discrete", 0.)
    assert (off, pdf) == (1, 0.25)
    off, pdf, ur = pyoracle.dist1d(func, "discrete", 0.125)
    assert (off, pdf) == (1, 0.25) and abs(ur - 0.5) <= 4 * np.finfo(np.float32).eps
    assert pyoracle.dist1d(func, "discrete", .24999)[:2] == (1, 0.25)
    assert pyoracle.dist1d(func, "discrete", .250001)[:2] == (3, 0.75)
    off, pdf, ur = pyoracle.dist1d(func, "discrete", 0.625)
    assert (off, pdf) == (3, 0.75) and abs(ur - 0.5) <= 4 * np.finfo(np.float32).eps
    assert pyoracle.dist1d(func, "discrete", ONE_MINUS_EPS)[:2] == (3, 0.75)
    assert pyoracle.dist1d(func, "discrete", 1.)[:2] == (3, 0.75)
    # a stream of 1s up to the cross-over at 0.25 (+- 20 ulps), then only 3s
    u = np.float32(.25)
    umax = np.float32(.25)
    for _ in range(20):
        u = np.nextafter(u, np.float32(-1))
        umax = np.nextafter(umax, np.float32(2))
    while u < umax:
        k = pyoracle.dist1d(func, "discrete", float(u))[0]
        if k == 3:
            break
        assert k == 1
        u = np.nextafter(u, np.float32(2))
    assert u < umax
    while u <= umax:
        assert pyoracle.dist1d(func, "discrete", float(u))[0] == 3
        u = np.nextafter(u, np.float32(2))


def test_distribution1d_continuous():
    """Distribution1D.Continuous (src/tests/sampling.cpp:282-303)."""
    func = [1, 1, 2, 4, 8]
    feq = lambda a, b: abs(a - b) <= 4 * np.finfo(np.float32).eps * max(1.0, abs(b))   # EXPECT_FLOAT_EQ
    x, pdf, off = pyoracle.dist1d(func, "continuous", 0.)
    assert x == 0. and feq(pdf, 5 * 1. / 16.) and off == 0
    assert feq(pyoracle.dist1d(func, "continuous", 0.5)[0], .8)
    x, pdf, off = pyoracle.dist1d(func, "continuous", 0.75)
    assert feq(x, .9) and feq(pdf, 5 * 8. / 16.) and off == 4
    assert feq(pyoracle.dist1d(func, "continuous", 0.)[0], 0.)
    assert feq(pyoracle.dist1d(func, "continuous", 1.)[0], 1.)


# ---- device: the same ray queries through the C ABI ----

def one_triangle_scene(tmp_path, tri, name):
    """A one-triangle .pbrt whose vertices round-trip exactly (%.9g)."""
    pts = " ".join("%.9g" % float(c) for c in np.asarray(tri, np.float32).reshape(-1))
    txt = f"""LookAt 0 0 -10 0 0 0 0 1 0
Camera "perspective"
Film "image" "integer xresolution" [4] "integer yresolution" [4]
Sampler "halton" "integer pixelsamples" [1]
WorldBegin
Shape "trianglemesh" "integer indices" [0 1 2] "point P" [{pts}]
WorldEnd
"""
    p = os.path.join(str(tmp_path), name)
    with open(p, "w") as f:
        f.write(txt)
    return p


@pytest.mark.gpu
def test_reintersect_rays_device(tmp_path):
    """The spawned rays of 64 Triangle.Reintersect seeds through the device's
    closest-hit and any-hit traversal: no self-intersection, identical to the
    oracle ray for ray."""
    import ptgpu
    done = 0
    for i in range(200):
        case = pyoracle.reintersect_case(i, 2000)
        if case is None:
            continue
        tri, rays, bad = case
        assert bad == 0
        hs = ptgpu.HostScene(one_triangle_scene(tmp_path, tri, f"reint_{i}.pbrt"))
        assert np.array_equal(hs.mesh()["P"], tri)
        sc = ptgpu.Scene(hs)
        for any_hit in (False, True):
            # device: hit primitive (>= 0) or -1 for both queries; oracle: prim / -1
            # for Intersect, 1 / 0 for IntersectP
            hit = sc.debug_trace(rays, any_hit) >= 0
            ref = pyoracle.trace(hs.desc, rays, any_hit)
            assert not hit.any()
            assert np.array_equal(hit, (ref != 0) if any_hit else (ref >= 0))
        done += 1
        if done == 64:
            break
    assert done == 64


@pytest.mark.gpu
def test_triangle_sampling_rays_device(tmp_path):
    """The uniform-sphere rays of Triangle.Sampling (seeds 0-5, 64 K rays
    each) through the device's any-hit traversal: the same hit set as the
    oracle's IntersectP, so the same uniform solid-angle estimate."""
    import ptgpu
    for i in range(6):
        case = pyoracle.triangle_sampling_case(i, 64 * 1024)
        if case is None:
            continue
        unif, _, tri, pc, _ = case
        hs = ptgpu.HostScene(one_triangle_scene(tmp_path, tri, f"samp_{i}.pbrt"))
        sc = ptgpu.Scene(hs)
        j = np.arange(64 * 1024)
        u0 = np.array([pyoracle.radical_inverse(0, int(k)) for k in j], np.float32)
        u1 = np.array([pyoracle.radical_inverse(1, int(k)) for k in j], np.float32)
        z = (1 - 2 * u0).astype(np.float32)
        r = np.sqrt(np.maximum(np.float32(0), 1 - z * z)).astype(np.float32)
        phi = (np.float32(2 * np.pi) * u1).astype(np.float32)
        d = np.stack([r * np.cos(phi), r * np.sin(phi), z], 1).astype(np.float32)
        rays = np.concatenate([np.broadcast_to(pc, (len(j), 3)), d, np.full((len(j), 1), np.inf)], 1)
        rays = np.ascontiguousarray(rays, np.float32)
        got = sc.debug_trace(rays, True)
        ref = pyoracle.trace(hs.desc, rays, True)
        assert np.array_equal(got >= 0, ref != 0)


@pytest.mark.gpu
@pytest.mark.parametrize("tmax", [np.inf, 0.9999])
def test_triangle_bad_cases_device(tmp_path, tmax):
    import ptgpu
    hs = ptgpu.HostScene(one_triangle_scene(tmp_path, BAD_TRI, "bad.pbrt"))
    sc = ptgpu.Scene(hs)
    ray = np.concatenate([BAD_O, BAD_D, [tmax]]).astype(np.float32)[None, :]
    assert sc.debug_trace(ray, False)[0] < 0              # Intersect: degenerate, no hit
    assert sc.debug_trace(ray, True)[0] == 0              # IntersectP: the reference's bogus hit (prim 0)
    assert pyoracle.trace(hs.desc, ray, False)[0] < 0 and pyoracle.trace(hs.desc, ray, True)[0] == 1


@pytest.mark.gpu
def test_sphere_solid_angle_device(tmp_path):
    """Sphere.SolidAngle's 128 K rays through the device's any-hit traversal
    (sphere test with EFloat bounds and the rotated transform): the same hit
    set as the oracle, hence the same estimates."""
    import ptgpu
    hs = ptgpu.HostScene(sphere_scene(tmp_path, "sa.pbrt", xf=SPHERE_XF))
    sc = ptgpu.Scene(hs)
    for p in ((1, .9, -.8), (-.25, -1, .8)):
        rays = mc_sphere_rays(p, 128 * 1024)
        assert np.array_equal(sc.debug_trace(rays, True) >= 0, pyoracle.trace(hs.desc, rays, True) != 0)


@pytest.mark.gpu
@pytest.mark.parametrize("partial", [False, True])
def test_sphere_reintersect_device(tmp_path, partial):
    """The spawned rays of 16 {Full,Partial}Sphere.Reintersect seeds through the
    device's closest-hit and any-hit traversal: no self-intersection."""
    import ptgpu
    done = 0
    for i in range(100):
        case = pyoracle.sphere_case(i, partial, "reintersect", n_dirs=2000)
        if case is None:
            continue
        (radius, zmin, zmax, phimax), rays, bad = case
        assert bad == 0
        hs = ptgpu.HostScene(sphere_scene(tmp_path, f"sr_{int(partial)}_{i}.pbrt", radius, zmin, zmax, phimax))
        sc = ptgpu.Scene(hs)
        for any_hit in (False, True):
            hit = sc.debug_trace(rays, any_hit) >= 0
            ref = pyoracle.trace(hs.desc, rays, any_hit)
            assert not hit.any()
            assert np.array_equal(hit, (ref != 0) if any_hit else (ref >= 0))
        done += 1
        if done == 16:
            break
    assert done == 16
