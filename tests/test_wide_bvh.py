"""The 4-wide traversal (k_trace_w, kernels.hip; round 6) against the oracle's
binary BVHAccel walk (bvh.cpp:662-738).

k_trace_w visits the reference's leaves in another order, so its closest hit
is the reference's only where no second primitive is accepted within 2^-15 of
the winner's t: such rays (and hits at t <= 0, and directions with a zero
component) go back to the binary kernel.  These tests aim rays exactly at the
places where the order decides -- coplanar duplicate triangles (the reference
keeps the LAST accepted one, triangle.cpp:259-261 with `>`), shared edges and
vertices of a triangle fan (the watertight test accepts both triangles on an
edge), two crossing quads (equal t along their intersection line), an aaplane
lying on a triangle (plane.cpp has no t > 0 test) -- plus axis-aligned rays,
and require the hit primitive (closest) / occlusion (any hit) to equal the
oracle's for every ray, and the tie rays to have been retraced.  A scene with
a sphere touching a triangle must not take the wide kernel (the EFloat sphere
test is left to the reference's order).  The counting frame
(pt_set_count_bytes) traverses in the reference's order and reproduces the
reference's node / primitive counters."""
import numpy as np
import pytest

import ptgpu
import pyoracle
from conftest import assert_counters, scene_variant

pytestmark = pytest.mark.gpu


def _quad(p0, p1, p2, p3):
    return [p0, p1, p2, p3]


def _tie_scene(tmp_path, sphere=False):
    """Triangles (and an aaplane) arranged so that many rays meet two primitives
    at the same or nearly the same t."""
    meshes = []
    # a 4 x 4 fan of shared-edge triangles in the plane z = 3
    for i in range(4):
        for j in range(4):
            x0, y0 = -2 + i, -2 + j
            meshes.append(_quad((x0, y0, 3), (x0 + 1, y0, 3), (x0 + 1, y0 + 1, 3), (x0, y0 + 1, 3)))
    # the same quad twice (coplanar duplicates, same and opposite winding) in z = 1
    meshes.append(_quad((-1.5, -1.5, 1), (-0.5, -1.5, 1), (-0.5, -0.5, 1), (-1.5, -0.5, 1)))
    meshes.append(_quad((-1.5, -1.5, 1), (-0.5, -1.5, 1), (-0.5, -0.5, 1), (-1.5, -0.5, 1)))
    meshes.append(_quad((-1.5, -0.5, 1), (-0.5, -0.5, 1), (-0.5, -1.5, 1), (-1.5, -1.5, 1)))
    # two quads crossing along the line x = 1, z = 2 (equal t on it)
    meshes.append(_quad((0.5, -1, 1.5), (1.5, -1, 2.5), (1.5, 1, 2.5), (0.5, 1, 1.5)))
    meshes.append(_quad((0.5, -1, 2.5), (1.5, -1, 1.5), (1.5, 1, 1.5), (0.5, 1, 2.5)))
    shapes = []
    for q in meshes:
        pts = " ".join("%r %r %r" % p for p in q)
        shapes.append('Shape "trianglemesh" "integer indices" [0 1 2 2 3 0] "point P" [%s]' % pts)
    txt = """LookAt 0 0 -6  0 0 0  0 1 0
Camera "perspective" "float fov" [40]
Film "image" "integer xresolution" [24] "integer yresolution" [24] "string filename" ["tie.pfm"]
Sampler "halton" "integer pixelsamples" [4]
Integrator "path" "integer maxdepth" [3]
WorldBegin
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [4 4 4]
  Shape "trianglemesh" "integer indices" [0 1 2 2 3 0] "point P" [-1 3 -2  1 3 -2  1 3 0  -1 3 0]
AttributeEnd
Material "matte" "rgb Kd" [0.5 0.5 0.5]
%s
Shape "aaplane" "point lo" [0 -2 3] "point hi" [2 0 3] "integer axis" 2
""" % "\n".join(shapes)
    if sphere:
        txt += 'Translate -1 1 2.5\nShape "sphere" "float radius" [0.5]\n'
    txt += "WorldEnd\n"
    p = tmp_path / ("tie_sphere.pbrt" if sphere else "tie.pbrt")
    p.write_text(txt)
    return str(p)


def _tie_rays(n_rand, seed, any_hit):
    rng = np.random.default_rng(seed)
    targets = []
    for i in range(5):  # fan vertices, edge midpoints, diagonal points (z = 3)
        for j in range(5):
            targets.append((-2 + i, -2 + j, 3))
            targets.append((-1.5 + i, -2 + j, 3))
            targets.append((-2 + i, -1.5 + j, 3))
            targets.append((-1.75 + i, -1.75 + j, 3))
    for _ in range(200):  # the duplicates, their shared diagonal and edges (z = 1)
        u = rng.uniform(-1.5, -0.5)
        targets += [(u, u, 1), (u, -1.5, 1), (-0.5, u, 1), tuple(rng.uniform(-1.5, -0.5, 2)) + (1,)]
    for _ in range(300):  # the crossing line x = 1, z = 2
        targets.append((1.0, rng.uniform(-1, 1), 2.0))
    for _ in range(200):  # the aaplane on top of the fan (z = 3, x 0..2, y -2..0)
        targets.append((rng.uniform(0, 2), rng.uniform(-2, 0), 3.0))
    targets = np.array(targets, np.float64)
    t = np.repeat(targets, 4, axis=0)
    o = np.stack([rng.uniform(-3, 3, len(t)), rng.uniform(-3, 3, len(t)), rng.uniform(-5, -0.5, len(t))], 1)
    # some rays straight along z (zero x / y components: infinite 1/d)
    ax = rng.random(len(t)) < 0.1
    o[ax, :2] = t[ax, :2]
    d = t - o
    dist = np.linalg.norm(d, axis=1, keepdims=True)
    d /= dist
    o, d = o.astype(np.float32), d.astype(np.float32)
    d[ax, :2] = 0.0
    d[ax, 2] = 1.0
    tmax = np.full((len(t), 1), np.inf, np.float32)
    if any_hit:  # shadow rays ending exactly at / just before / just past the target
        f = rng.choice([1.0, 1 - 1e-4, 1 + 1e-4, 0.9999999], len(t))
        tmax = (dist[:, 0] * f).astype(np.float32)[:, None]
    rays = np.concatenate([o, d, tmax], 1).astype(np.float32)
    rnd = np.zeros((n_rand, 7), np.float32)
    rnd[:, :3] = np.stack([rng.uniform(-3, 3, n_rand), rng.uniform(-3, 3, n_rand), rng.uniform(-5, 5, n_rand)], 1)
    dd = rng.normal(size=(n_rand, 3))
    rnd[:, 3:6] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
    rnd[:, 6] = np.inf if not any_hit else rng.uniform(0.1, 8, n_rand)
    return np.concatenate([rays, rnd]).astype(np.float32)


@pytest.mark.parametrize("any_hit", [False, True])
@pytest.mark.parametrize("where", ["lds", "hbm"])
def test_wide_traversal_ties_match_oracle(tmp_path, monkeypatch, any_hit, where):
    """where: the wide image and primitives staged in LDS (k_trace_w<false>) or
    read from HBM (k_trace_w<true>, PT_TRACE_LDS=0; with a 2-row LDS stack so
    the spill column is exercised)."""
    if where == "hbm":
        monkeypatch.setenv("PT_TRACE_LDS", "0")
        monkeypatch.setenv("PT_WIDE_LDS_ROWS", "2")
    hs = ptgpu.HostScene(_tie_scene(tmp_path))
    sc = ptgpu.Scene(hs)
    assert sc.kernel_names()[0] == "k_trace_w"
    rays = _tie_rays(20000, 7, any_hit)
    _, order = sc.bvh()
    got, st = sc.debug_trace_frame_stats(rays, any_hit)
    ref, _, _ = pyoracle.trace_counted(hs.desc, rays, any_hit)
    if not any_hit:
        got = np.where(got >= 0, order[np.maximum(got, 0)], -1)
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, (len(bad), rays[bad[:4]], got[bad[:4]], ref[bad[:4]])
    assert st["trace_wide"] == 1
    assert st["closest_rays"] + st["shadow_rays"] == len(rays)
    # the duplicates, the crossing line and the axis-aligned rays must have gone back to the binary kernel
    assert st["retraced_rays"] > 0.05 * len(rays) if not any_hit else st["retraced_rays"] > 0
    print(f"rays {len(rays)} retraced {st['retraced_rays']} wide nodes {st['wide_node_visits']}")


def test_wide_traversal_not_taken_with_spheres(tmp_path):
    """A sphere touching a triangle: the scene keeps the binary traversal, and
    its hits equal the oracle's."""
    hs = ptgpu.HostScene(_tie_scene(tmp_path, sphere=True))
    sc = ptgpu.Scene(hs)
    assert sc.kernel_names()[0] == "k_trace_lds"
    rays = _tie_rays(4000, 8, False)
    rng = np.random.default_rng(9)
    tgt = np.array([-1, 1, 2.0]) + 0.5 * np.array([0, 0, 1]) + rng.normal(0, 1e-3, (2000, 3))
    o = np.stack([rng.uniform(-3, 3, 2000), rng.uniform(-3, 3, 2000), rng.uniform(-5, -1, 2000)], 1)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([rays, np.concatenate([o, d, np.full((2000, 1), np.inf)], 1)]).astype(np.float32)
    _, order = sc.bvh()
    got, nodes, prims = sc.debug_trace_frame(rays, False)
    ref, rnodes, rprims = pyoracle.trace_counted(hs.desc, rays, False)
    got = np.where(got >= 0, order[np.maximum(got, 0)], -1)
    assert np.array_equal(got, ref)
    assert (nodes, prims) == (rnodes, rprims)


def test_wide_tie_scene_render_matches_oracle(tmp_path):
    hs = ptgpu.HostScene(_tie_scene(tmp_path))
    sc = ptgpu.Scene(hs)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert gst["trace_wide"] == 1
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.parametrize("scene", ["portal_cornell.pbrt", "portal_room.pbrt", "cornell_dielectric.pbrt",
                                   "cornell_dielectric_hero.pbrt"])
@pytest.mark.parametrize("where", ["lds", "hbm"])
def test_counting_frame_reference_counters(tmp_path, monkeypatch, scene, where):
    """The default render (k_trace_w) and the counting frame (binary traversal in
    the reference's order) give the oracle's image bit for bit; the counting
    frame also the reference's node-visit / primitive-test counters."""
    if where == "hbm":
        monkeypatch.setenv("PT_TRACE_LDS", "0")
    path = scene_variant(tmp_path, name=scene, res=(48, 32), spp=8)
    hs = ptgpu.HostScene(path)
    sc = ptgpu.Scene(hs)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    keys = ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests")
    assert sc.kernel_names()[0] == "k_trace_w"
    got, gst = sc.render()
    assert gst["trace_wide"] == 1 and gst["wide_node_visits"] > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, keys)
    sc.set_count_bytes(True)
    assert sc.kernel_names()[0] == ("k_trace_lds" if where == "lds" else "k_trace_nb")
    got2, gst2 = sc.render()
    assert gst2["trace_wide"] == 0 and gst2["retraced_rays"] == 0
    assert np.array_equal(got2.view(np.uint32), ref.view(np.uint32))
    for k in keys:
        assert gst2[k] == rst[k], k
    print(f"{scene}: retraced {gst['retraced_rays']} of {gst['closest_rays'] + gst['shadow_rays']} rays; "
          f"wide nodes {gst['wide_node_visits']} vs binary {gst2['node_visits']}")
