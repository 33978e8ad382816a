"""The reference's remaining portal scenes (scenes/blender/creeper/out/, imported
verbatim by scripts/import_reference_scenes.py into scenes/creeper/):

* creeper.pbrt:38-49 -- a DiffuseAreaLight on an axis-1 aaplane (its
  "strategy"/"portalData" parameters are unused by "diffuse"), a point light,
  `Scale -1 1 1` before LookAt, DirectLighting.  The plane's lo/hi give an empty
  open interval on its ax0 axis (lo.z == hi.z == 0.24), so AAPlaneShape::
  Intersect (plane.cpp:23-31) never accepts a hit and Area() is 0
  (plane.h:29-31): Shape::Sample(ref)'s pdf is inf -> 0 (shape.cpp:70) and
  Shape::Pdf misses (shape.cpp:84) -- the light contributes nothing;
* sandbox.pbrt:45-56 -- a PortalArealight under a rotated Transform with five
  axis-2 '+' portals, strategy projection, DirectLighting: the only
  reference-held input that drives the rotated-CTM quirks:
  world lo/hi indexed by object axes (plane.h:29-31, plane.cpp:59-66), the
  portal pdf with the untransformed Normal() (aaportal.cpp:82), InFront in
  light object space (aaportal.cpp:98), WorldToObject applied to the sampled
  object-space point (aaportal.cpp:154);
* test00001.pbrt -- path, a trianglemesh emitter with normals and st;

and (round 4) the reference's other renderable blender scenes:

* lamp/test00001.pbrt -- DirectLighting over the lamp meshes, a DiffuseAreaLight
  on an aaplane given with the old loX/hiX parameters (CreateAAPlaneShape reads
  only "point lo"/"point hi", plane.cpp:117-128, so lo = hi = 0: the light is
  never hit nor sampled and the image is black, as the reference renders it);
* spotlight/test00001.pbrt -- DirectLighting "one" with two diffuse trianglemesh
  lights, one of them an empty mesh ("point P" [] ... "integer indices" []):
  CreateTriangleMeshShape makes zero triangles, so that AreaLightSource yields
  no light (triangle.cpp:911-971, api.cpp MakeShapes);
* spotlight/arealight.pbrt -- path maxdepth 10, the same old-parameter aaplane;
* window_portal_eq/test00001.pbrt -- DirectLighting "one", two diffuse lights.

GPU tests render each as written and as `path` (x strategies) through the C
ABI and compare with the oracle bit for bit, ray / node / prim counters
included.  CPU tests pin what the reference's own semantics imply
independently of the oracle."""
import ctypes
import os

import numpy as np
import pytest

import ptgpu
import pyoracle
from conftest import SCENES, assert_counters, scene_variant

COUNTERS = ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests")
AS_PATH = [('Integrator "directlighting"', 'Integrator "path"'), ('"integer maxdepth" [10]', '"integer maxdepth" [5]')]
# sandbox with its PortalArealight turned into a DiffuseAreaLight on the same rotated aaplane
SANDBOX_DIFFUSE = [('AreaLightSource "portal"', 'AreaLightSource "diffuse"')]


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _gpu_vs_oracle(path, nthreads=16):
    hs = ptgpu.HostScene(path)
    sc = ptgpu.Scene(hs)
    ref, rst = pyoracle.render(hs.desc, nthreads=nthreads)
    got, gst = sc.render()
    rmse = float(np.sqrt(np.mean((got.astype(np.float64) - ref.astype(np.float64)) ** 2)))
    print(f"{os.path.basename(path)}: mean={ref.mean():.6g} rmse={rmse:.3g} rays={gst['closest_rays']}+"
          f"{gst['shadow_rays']} nodes={gst['node_visits']}")
    assert np.isfinite(ref).all()
    assert np.array_equal(_bits(got), _bits(ref)), f"rmse {rmse}"
    assert_counters(gst, rst, COUNTERS)
    return ref, rst


# --------------------------------------------------------------------------- CPU

def test_reference_scenes_load():
    """Loader: the scenes as written (comma-separated points "-0.23," parse as
    strtof does, parser.cpp:322-368; unused area-light parameters ignored)."""
    hs = ptgpu.HostScene(os.path.join(SCENES, "creeper", "creeper.pbrt"))
    d = ptgpu.scene_desc(hs)
    assert (d.n_planes, d.n_lights, d.n_portals, d.integrator.kind, d.sampler.spp) == (1, 2, 0, 1, 1)
    kinds = [ctypes.cast(d.lights, ctypes.POINTER(ctypes.c_int32))[i * 42] for i in range(2)]  # 168-byte pt_light
    assert kinds == [4, 5]  # PT_LIGHT_POINT, PT_LIGHT_DIFFUSE_PLANE (declaration order)
    pl = np.ctypeslib.as_array(ctypes.cast(d.planes, ctypes.POINTER(ctypes.c_float)), shape=(6,))
    assert np.array_equal(pl, np.float32([-0.23, -0.23, 0.24, 0.23, 0.23, 0.24]))
    hs = ptgpu.HostScene(os.path.join(SCENES, "creeper", "sandbox.pbrt"))
    d = ptgpu.scene_desc(hs)
    assert (d.n_planes, d.n_lights, d.n_portals, d.integrator.kind, d.sampler.spp) == (1, 2, 5, 1, 5)
    hs = ptgpu.HostScene(os.path.join(SCENES, "creeper", "test00001.pbrt"))
    d = ptgpu.scene_desc(hs)
    assert (d.n_triangles, d.n_lights, d.integrator.kind) == (4, 2, 0)


ROUND4 = {  # scene: (tris, planes, lights, integrator kind, maxdepth, spp)
    "lamp/test00001.pbrt": (324, 1, 1, 1, 100, 20),
    "spotlight/test00001.pbrt": (3964, 0, 2, 1, 3, 25),
    "spotlight/arealight.pbrt": (3962, 1, 1, 0, 10, 10),
    "window_portal_eq/test00001.pbrt": (3962, 0, 2, 1, 5, 25),
}


@pytest.mark.parametrize("scene", sorted(ROUND4))
def test_round4_reference_scenes_load(scene):
    """The scenes load as the reference parses them: the empty trianglemesh
    under spotlight's first AreaLightSource gives no shape and no light (two
    lights, not three)."""
    d = ptgpu.scene_desc(ptgpu.HostScene(os.path.join(SCENES, scene)))
    got = (d.n_triangles, d.n_planes, d.n_lights, d.integrator.kind, d.integrator.max_depth, d.sampler.spp)
    assert got == ROUND4[scene]


def _mesh_scene(tmp_path, shape, light=True):
    """A one-emitter room (the furnace cube) plus `shape` under its own
    AreaLightSource: what CreateTriangleMeshShape's error paths leave."""
    from conftest import furnace_scene
    txt = open(furnace_scene(tmp_path, res=8, spp=4, maxdepth=3)).read()
    add = ("AttributeBegin\n" + ('  AreaLightSource "diffuse" "rgb L" [4 4 4]\n' if light else "") +
           "  " + shape + "\nAttributeEnd\n")
    txt = txt.replace("WorldEnd", add + "WorldEnd")
    p = os.path.join(str(tmp_path), "mesh_%d.pbrt" % (abs(hash(shape)) % 10 ** 8))
    open(p, "w").write(txt)
    return p


TRI = '"point P" [0 0 0.5  0.2 0 0.5  0 0.2 0.5]'


@pytest.mark.parametrize("shape,ntris", [
    ('Shape "trianglemesh" "point P" [] "normal N" [] "float st" [] "integer indices" []', 0),  # empty: no shapes
    ('Shape "trianglemesh" ' + TRI, 0),                                # no indices: Error, no shapes
    ('Shape "trianglemesh" "integer indices" [0 1 2]', 0),             # no P: Error, no shapes
    ('Shape "trianglemesh" ' + TRI + ' "integer indices" [0 1 3]', 0),  # index past the last vertex
    ('Shape "trianglemesh" ' + TRI + ' "integer indices" [0 1 2 1]', 1),  # nvi / 3 triangles
    ('Shape "trianglemesh" ' + TRI + ' "integer indices" [0 1 2] "float uv" [0 0 1 0]', 1),  # too few uv
    ('Shape "trianglemesh" ' + TRI + ' "integer indices" [0 1 2] "normal N" [0 0 1]', 1),    # N count mismatch
    ('Shape "trianglemesh" "point P" [0 0 0.5  0.2 0 0.5  0 0.2 0.5  9] "integer indices" [0 1 2]', 1),  # P excess
])
def test_trianglemesh_error_contract(tmp_path, shape, ntris):
    """CreateTriangleMeshShape (triangle.cpp:911-971): Error() and no shapes for
    missing P / indices or an out-of-range index, the scene renders on; a uv
    array with fewer entries than P, or an N / S array of another length, is
    discarded; excess point values and a trailing partial index triple are
    ignored (parser.cpp:603-615, CreateTriangleMesh(nvi / 3)).  An emitting
    mesh of zero triangles adds no light (MakeShapes makes one
    DiffuseAreaLight per shape)."""
    hs = ptgpu.HostScene(_mesh_scene(tmp_path, shape))
    d = ptgpu.scene_desc(hs)
    assert d.n_triangles == 12 + ntris
    assert d.n_lights == 12 + ntris
    if ntris:  # the discarded arrays: no uv / normals / tangents on the triangle (pt_triangle: 6 words)
        words = ctypes.cast(d.triangles, ctypes.POINTER(ctypes.c_uint32))
        assert words[12 * 6 + 5] & (4 | 8 | 16) == 0
    img, st = pyoracle.render(hs.desc, nthreads=4)
    assert np.isfinite(img).all() and st["samples"] == 8 * 8 * 4


@pytest.mark.parametrize("uvs,has_uv", [
    ('"float uv" [0 0 1 0] "point2 st" [0 0 1 0 0 1]', True),   # point2 st before float uv: st is used
    ('"point2 uv" [0 0 1 0] "float st" [0 0 1 0 0 1]', False),  # point2 uv (too few: discarded) wins
    ('"float st" [0 0 1 0 0 1] "float uv" [0 0 1 0]', False),   # float uv before float st
])
def test_trianglemesh_uv_lookup_order(tmp_path, uvs, has_uv):
    """CreateTriangleMeshShape looks the uv array up as point2 "uv", point2
    "st", float "uv", float "st" (triangle.cpp:918-923): the first found is
    used (and discarded when shorter than P), later ones are not consulted."""
    hs = ptgpu.HostScene(_mesh_scene(tmp_path, 'Shape "trianglemesh" ' + TRI + ' "integer indices" [0 1 2] ' + uvs))
    d = ptgpu.scene_desc(hs)
    words = ctypes.cast(d.triangles, ctypes.POINTER(ctypes.c_uint32))
    assert bool(words[12 * 6 + 5] & 8) == has_uv  # PT_TRI_HAS_UV


def test_empty_emitter_mesh_adds_no_light(tmp_path):
    """An empty trianglemesh under an AreaLightSource (spotlight/test00001.pbrt)
    leaves the scene exactly as if the attribute block were absent: same
    lights, same image, same ray counts (oracle)."""
    a = ptgpu.HostScene(_mesh_scene(tmp_path, 'Shape "trianglemesh" "point P" [] "integer indices" []'))
    from conftest import furnace_scene
    b = ptgpu.HostScene(furnace_scene(tmp_path, res=8, spp=4, maxdepth=3))
    assert ptgpu.scene_desc(a).n_lights == ptgpu.scene_desc(b).n_lights == 12
    ia, sa = pyoracle.render(a.desc, nthreads=4)
    ib, sb = pyoracle.render(b.desc, nthreads=4)
    assert np.array_equal(_bits(ia), _bits(ib))
    assert sa == sb


def test_creeper_degenerate_plane_light_contributes_nothing(tmp_path):
    """creeper.pbrt's aaplane emitter can neither be hit (empty open interval,
    plane.cpp:23-31) nor sampled (Area() == 0 -> pdf inf -> 0, shape.cpp:70;
    Pdf_Li misses, shape.cpp:84-91), and the point light's estimate does not
    read its sample values (delta light, integrator.cpp:148-200), so the image
    and the camera / closest / shadow ray counts equal those of the scene with
    the area light removed -- at the scene's full 500x500."""
    full = scene_variant(tmp_path, name="creeper/creeper.pbrt")
    txt = open(full).read()
    start = txt.index('AreaLightSource "diffuse"')
    end = txt.index('Shape "aaplane"')
    nolight = os.path.join(str(tmp_path), "creeper_nolight.pbrt")
    open(nolight, "w").write(txt[:start] + txt[end:])
    ha, hb = ptgpu.HostScene(full), ptgpu.HostScene(nolight)  # keep the descriptions alive while rendering
    a, sa = pyoracle.render(ha.desc, nthreads=8)
    b, sb = pyoracle.render(hb.desc, nthreads=8)
    assert a.mean() > 0
    assert np.array_equal(_bits(a), _bits(b))
    for k in ("camera_rays", "closest_rays", "shadow_rays"):
        assert sa[k] == sb[k], k


def _portal_scene(tmp_path, n_portals):
    ent = "".join("(AA %g 540 230 %g 540 300 1 -)" % (200 + 2 * i, 201 + 2 * i) for i in range(n_portals))
    txt = open(os.path.join(SCENES, "portal_cornell.pbrt")).read()
    import re
    txt = re.sub(r'"string portalData" "[^"]*"', '"string portalData" "(%s)"' % ent, txt)
    p = os.path.join(str(tmp_path), "portals_%d.pbrt" % n_portals)
    open(p, "w").write(txt)
    return p


def test_portal_count_cap(tmp_path):
    """PT_MAX_PORTALS (include/pt.h): the reference's per-call portal
    distribution is a VLA (portal_arealight.cpp:42); 64 portals load, 65 are
    PT_ERR_UNSUPPORTED from the loader, and the oracle refuses a description
    that claims more."""
    hs = ptgpu.HostScene(_portal_scene(tmp_path, 64))
    assert ptgpu.scene_desc(hs).n_portals == 64
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.HostScene(_portal_scene(tmp_path, 65))
    assert e.value.status == 3
    light = ctypes.cast(ptgpu.scene_desc(hs).lights, ctypes.POINTER(ctypes.c_int32))
    n_portals_field = 1 + 3 + 1 + 1 + 1 + 1  # pt_light: kind, L[3], two_sided, shape, strategy, first_portal
    assert light[n_portals_field] == 64
    light[n_portals_field] = 65
    with pytest.raises(RuntimeError, match="PT_MAX_PORTALS"):
        pyoracle.render(hs.desc, nthreads=1)


# --------------------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_creeper_as_written_matches_oracle(tmp_path):
    """creeper.pbrt as written: DirectLighting maxdepth 10, 500x500 @1 spp."""
    ref, _ = _gpu_vs_oracle(scene_variant(tmp_path, name="creeper/creeper.pbrt"))
    assert ref.mean() > 0


@pytest.mark.gpu
def test_creeper_as_path_matches_oracle(tmp_path):
    _gpu_vs_oracle(scene_variant(tmp_path, name="creeper/creeper.pbrt", spp=4, extra=AS_PATH))


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["projection", "light", "portal"])
def test_sandbox_directlighting_matches_oracle(tmp_path, strategy):
    """sandbox.pbrt as written (projection, 700x700 @5 spp) and with the other
    two strategies at 350x350."""
    res = None if strategy == "projection" else (350, 350)
    ref, _ = _gpu_vs_oracle(scene_variant(tmp_path, name="creeper/sandbox.pbrt", res=res, strategy=strategy))
    assert ref.mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["projection", "light", "portal"])
def test_sandbox_as_path_matches_oracle(tmp_path, strategy):
    """sandbox.pbrt with path maxdepth 5 x {light, portal, projection}."""
    ref, _ = _gpu_vs_oracle(scene_variant(tmp_path, name="creeper/sandbox.pbrt", res=(350, 350), spp=4,
                                          strategy=strategy, extra=AS_PATH))
    assert ref.mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["directlighting", "path"])
def test_rotated_diffuse_plane_light_matches_oracle(tmp_path, integrator):
    """A DiffuseAreaLight on the sandbox's rotated aaplane: MIS through
    Shape::Sample(ref) (world lo/hi indexed by object axes, Normal()
    untransformed, plane.cpp:57-72) and Shape::Pdf (object-space Intersect with
    no t > 0 test, plane.cpp:15-55)."""
    extra = SANDBOX_DIFFUSE + (AS_PATH if integrator == "path" else [])
    ref, rst = _gpu_vs_oracle(scene_variant(tmp_path, name="creeper/sandbox.pbrt", res=(350, 350), spp=4,
                                            extra=extra))
    assert ref.mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["path", "directlighting"])
def test_diffuse_plane_light_cornell_matches_oracle(tmp_path, integrator):
    """The portal Cornell's aaplane emitter as a plain DiffuseAreaLight
    (identity CTM, ReverseOrientation): the light is reached only through the
    ceiling hole, by MIS."""
    extra = [('AreaLightSource "portal"', 'AreaLightSource "diffuse"')]
    if integrator == "directlighting":
        extra.append(('Integrator "path"', 'Integrator "directlighting"'))
    ref, _ = _gpu_vs_oracle(scene_variant(tmp_path, res=(96, 54), spp=16, extra=extra))
    assert ref.mean() > 0


@pytest.mark.gpu
def test_test00001_matches_oracle(tmp_path):
    """test00001.pbrt as written: path maxdepth 10, trianglemesh emitter with
    shading normals and st, 500x500 @10 spp."""
    ref, _ = _gpu_vs_oracle(scene_variant(tmp_path, name="creeper/test00001.pbrt"))
    assert ref.mean() > 0


@pytest.mark.gpu
def test_portal_count_cap_device(tmp_path):
    """pt_scene_create refuses a light with more than PT_MAX_PORTALS portals."""
    hs = ptgpu.HostScene(_portal_scene(tmp_path, 64))
    light = ctypes.cast(ptgpu.scene_desc(hs).lights, ctypes.POINTER(ctypes.c_int32))
    light[8] = 65
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.Scene(hs)
    assert e.value.status == 3


@pytest.mark.gpu
@pytest.mark.parametrize("scene", sorted(ROUND4))
def test_round4_reference_scenes_as_written_match_oracle(tmp_path, scene):
    """The reference's lamp / spotlight / window_portal_eq scenes as written
    (DirectLighting "one" and path maxdepth 10, the scene's film and spp),
    bit-identical to the oracle with identical counters."""
    _gpu_vs_oracle(scene_variant(tmp_path, name=scene))


@pytest.mark.gpu
@pytest.mark.parametrize("scene", sorted(ROUND4))
def test_round4_reference_scenes_as_path_match_oracle(tmp_path, scene):
    """The same scenes as PathIntegrator maxdepth 5."""
    extra = [('Integrator "directlighting"', 'Integrator "path"'), ('"integer maxdepth" [10]', '"integer maxdepth" [5]'),
             ('"integer maxdepth" [100]', '"integer maxdepth" [5]'), ('"integer maxdepth" [3]', '"integer maxdepth" [5]')]
    _gpu_vs_oracle(scene_variant(tmp_path, name=scene, spp=8, extra=extra))
