"""Host loader and BVH builder (CPU): the flattened scene matches what the
reference's parser/api would build, and the product's SAH BVH equals the
oracle's restatement of BVHAccel::recursiveBuild node for node."""
import ctypes
import os

import numpy as np
import pytest

import ptgpu
import pyoracle
from conftest import SCENES, furnace_scene

REPO = os.path.dirname(SCENES)


class Desc(ctypes.Structure):
    """Prefix of pt_scene_desc (include/pt.h) for inspection."""
    _fields_ = [("n_vertices", ctypes.c_int32), ("P", ctypes.c_void_p), ("N", ctypes.c_void_p),
                ("S", ctypes.c_void_p), ("UV", ctypes.c_void_p), ("n_triangles", ctypes.c_int32),
                ("triangles", ctypes.c_void_p), ("n_planes", ctypes.c_int32), ("planes", ctypes.c_void_p),
                ("n_prims", ctypes.c_int32), ("prims", ctypes.c_void_p), ("n_materials", ctypes.c_int32),
                ("materials", ctypes.c_void_p), ("n_lights", ctypes.c_int32), ("lights", ctypes.c_void_p),
                ("n_portals", ctypes.c_int32), ("portals", ctypes.c_void_p), ("bvh_max_prims", ctypes.c_int32),
                ("cam_m", ctypes.c_float * 16), ("cam_minv", ctypes.c_float * 16), ("fov", ctypes.c_float),
                ("screen", ctypes.c_float * 4)]


def _desc(hs):
    return Desc.from_address(hs.desc)


def test_portal_cornell_counts():
    hs = ptgpu.HostScene(os.path.join(SCENES, "portal_cornell.pbrt"))
    d = _desc(hs)
    # 2 red + 2 green + 2 floor + 2 back + 2 front + 8 ceiling + 10 attic + 10 + 10 blocks
    assert d.n_triangles == 48
    assert d.n_planes == 1
    assert d.n_prims == 49
    assert d.n_lights == 1
    assert d.n_portals == 1
    assert d.bvh_max_prims == 4
    assert abs(d.fov - 37.5) < 1e-6
    # frame aspect 16:9 -> screen window [-16/9, 16/9] x [-1, 1] (perspective.cpp:251-263)
    assert np.allclose(list(d.screen), [-1920 / 1080, 1920 / 1080, -1, 1])


def test_camera_to_world_is_lookat_inverse():
    hs = ptgpu.HostScene(os.path.join(SCENES, "portal_cornell.pbrt"))
    d = _desc(hs)
    m = np.array(d.cam_m).reshape(4, 4)
    # LookAt 278 273 -800 -> 278 273 0, up y: camera-to-world maps origin to the eye
    assert np.allclose(m @ [0, 0, 0, 1], [278, 273, -800, 1])
    assert np.allclose(m @ [0, 0, 1, 0], [0, 0, 1, 0], atol=1e-6)
    mi = np.array(d.cam_minv).reshape(4, 4)
    assert np.allclose(m @ mi, np.eye(4), atol=1e-5)


@pytest.mark.parametrize("name", ["portal_cornell.pbrt"])
def test_bvh_matches_oracle(name):
    hs = ptgpu.HostScene(os.path.join(SCENES, name))
    n1, o1 = hs.bvh()
    n2, o2 = pyoracle.build_bvh(hs.desc)
    assert n1.shape == n2.shape
    assert np.array_equal(n1, n2)
    nprim = _desc(hs).n_prims
    assert np.array_equal(o1[:nprim], o2[:nprim])
    assert sorted(o1[:nprim]) == list(range(nprim))


def _soup_scene(tmp_path, n, seed, spread=100.0, maxprims=4):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (n, 1, 3))
    v = c + rng.normal(scale=spread / 20, size=(n, 3, 3))
    # a few degenerate / duplicated triangles on purpose
    if n >= 3:
        v[0, 2] = v[0, 1]
        v[1] = v[2]
    pts = " ".join("%r" % float(x) for x in v.astype(np.float32).reshape(-1))
    idx = " ".join(str(i) for i in range(3 * n))
    txt = f"""LookAt 0 0 -300 0 0 0 0 1 0
Camera "perspective" "float fov" [45]
Film "image" "integer xresolution" [16] "integer yresolution" [16]
Sampler "halton" "integer pixelsamples" [1]
Accelerator "bvh" "integer maxnodeprims" [{maxprims}]
WorldBegin
Shape "trianglemesh" "integer indices" [{idx}] "point P" [{pts}]
WorldEnd
"""
    p = tmp_path / f"soup_{n}_{seed}.pbrt"
    p.write_text(txt)
    return str(p)


@pytest.mark.parametrize("n,seed,maxprims", [(1, 0, 4), (2, 1, 4), (3, 2, 4), (17, 3, 4), (500, 4, 4),
                                             (2000, 5, 1), (2000, 6, 8),
                                             (150000, 7, 4)])  # > 2 x 32K: the threaded subtree build
def test_bvh_random_soups(tmp_path, n, seed, maxprims):
    hs = ptgpu.HostScene(_soup_scene(tmp_path, n, seed, maxprims=maxprims))
    n1, o1 = hs.bvh()
    n2, o2 = pyoracle.build_bvh(hs.desc)
    assert np.array_equal(n1, n2)
    assert np.array_equal(o1[:n], o2[:n])


def test_furnace_scene_loads(tmp_path):
    hs = ptgpu.HostScene(furnace_scene(tmp_path))
    d = _desc(hs)
    assert d.n_triangles == 12 and d.n_lights == 12  # one DiffuseAreaLight per triangle (api.cpp:1370-1378)


def test_portal_data_requires_outer_list(tmp_path):
    txt = open(os.path.join(SCENES, "portal_cornell.pbrt")).read()
    bad = txt.replace('"((AA 213 548.8 227 343 548.8 332 1 -))"', '"(AA 213 548.8 227 343 548.8 332 1 -)"')
    p = tmp_path / "bad_portal.pbrt"
    p.write_text(bad)
    with pytest.raises(ptgpu.PtError):
        ptgpu.HostScene(str(p))


def test_commas_in_numbers_are_tolerated(tmp_path):
    """parseNumber uses strtof and ignores trailing characters (parser.cpp:322-366)."""
    txt = open(os.path.join(SCENES, "portal_cornell.pbrt")).read()
    txt = txt.replace('"point lo" [193 650 207]', '"point lo" [193, 650, 207]')
    p = tmp_path / "commas.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    assert _desc(hs).n_planes == 1


def test_portal_room_scene(tmp_path):
    """Config 4 scene (scripts/make_portal_room.py): four portals on one
    PortalArealight, an infinite light, the committed file is what the
    generator writes."""
    import subprocess
    import sys
    out = tmp_path / "room.pbrt"
    subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "make_portal_room.py"), str(out)])
    assert out.read_text() == open(os.path.join(REPO, "scenes", "portal_room.pbrt")).read()
    hs = ptgpu.HostScene(str(out))
    d = ctypes.cast(ctypes.c_void_p(hs.desc), ctypes.POINTER(ptgpu.pt_scene_desc)).contents
    assert (d.n_lights, d.n_portals, d.n_planes) == (2, 4, 1)
    assert (d.film.xres, d.film.yres, d.sampler.spp, d.integrator.max_depth) == (3840, 2160, 1024, 8)
