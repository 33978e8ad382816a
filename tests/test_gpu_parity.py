"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on
the same inputs.  Integer / index results must be bit-exact; radiance must
match within the north_star tolerance (per-pixel RMSE < 1e-4 of the image,
relative to its mean for the unbounded 'projection' estimator) -- and the
renders are in fact required to be bit-identical, since the device performs
the oracle's float operations in the oracle's order."""
import os

import numpy as np
import pytest

import ptgpu
import pyoracle
from conftest import assert_counters, furnace_scene

pytestmark = pytest.mark.gpu

MINI = dict(res=(64, 36), spp=16)


def _scene(path, **kw):
    hs = ptgpu.HostScene(path)
    return hs, ptgpu.Scene(hs, **kw)


def _sample_bounds(hs):
    # box filter r = 0.5: sample bounds == crop window
    w, h = pyoracle.film_size(hs.desc)
    return (0, 0, w, h)


def test_halton_bit_exact(variant):
    hs, sc = _scene(variant(**MINI))
    sb = _sample_bounds(hs)
    rng = np.random.default_rng(1)
    n = 4000
    px = rng.integers(0, sb[2], n)
    py = rng.integers(0, sb[3], n)
    s = rng.integers(0, 16, n)
    dims = rng.integers(0, 40, n).astype(np.int32)
    idx = np.array([pyoracle.halton_index(sb, int(a), int(b), int(c)) for a, b, c in zip(px, py, s)], np.uint32)
    ref = np.array([pyoracle.halton_sample(sb, int(a), int(b), int(c), int(d)) for a, b, c, d in zip(px, py, s, dims)],
                   np.float32)
    got = sc.debug_halton(idx, dims)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_halton_division_extremes(variant):
    """Magic-number division by every per-dimension prime, at large indices."""
    hs, sc = _scene(variant(**MINI))
    dims = np.arange(2, 46, dtype=np.int32)
    vals = np.array([0, 1, 2, 3, 4294967295, 4294967294, 2147483648, 123456789, 31103, 31104 * 255 + 31103],
                    np.uint64)
    idx = np.repeat(vals, len(dims)).astype(np.uint32)
    dd = np.tile(dims, len(vals))
    got = sc.debug_halton(idx, dd)
    ref = np.array([pyoracle.scrambled_radical_inverse(int(d), int(i)) for i, d in zip(idx, dd)], np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_pixel_offsets(variant):
    hs, sc = _scene(variant(res=(300, 200), spp=4))
    sb = _sample_bounds(hs)
    pix = np.array([(x, y) for y in range(0, 200, 7) for x in range(0, 300, 5)], np.int32)
    got = sc.debug_pixel_offsets(pix)
    ref = np.array([pyoracle.halton_index(sb, int(x), int(y), 0) for x, y in pix], np.uint32)
    assert np.array_equal(got, ref)


def test_camera_rays_bit_exact(variant):
    hs, sc = _scene(variant(**MINI))
    rng = np.random.default_rng(2)
    film = np.stack([rng.uniform(0, 64, 2000), rng.uniform(0, 36, 2000)], 1).astype(np.float32)
    got = sc.debug_camera_rays(film)
    ref = np.array([np.concatenate(pyoracle.camera_ray(hs.desc, float(x), float(y))) for x, y in film], np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _random_rays(n, seed, tmax=np.inf):
    rng = np.random.default_rng(seed)
    o = np.stack([rng.uniform(1, 555, n), rng.uniform(1, 690, n), rng.uniform(-899, 558, n)], 1)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t = np.full((n, 1), tmax)
    return np.concatenate([o, d, t], 1).astype(np.float32)


@pytest.mark.parametrize("any_hit", [False, True])
def test_traversal_bit_exact(variant, any_hit):
    hs, sc = _scene(variant(**MINI))
    rays = _random_rays(20000, 3, tmax=np.inf if not any_hit else 300.0)
    _, order = sc.bvh()
    got = sc.debug_trace(rays, any_hit)
    ref = pyoracle.trace(hs.desc, rays, any_hit)
    if not any_hit:
        got = np.where(got >= 0, order[np.maximum(got, 0)], -1)
    else:
        got = (got >= 0).astype(np.int32)
    assert np.array_equal(got, ref)


def _edge_rays(sc, n_rand, n_edge, seed, tmax):
    """Random rays plus the slab test's edge cases (Bounds3::IntersectP,
    geometry.h:1584-1606): direction components +0 / -0 (inverse direction
    +inf / -inf) from origins lying exactly on BVH node bounds, where the
    reference's slab distances are 0 * inf = NaN."""
    nodes, _ = sc.bvh()
    b = np.ascontiguousarray(nodes[:, :6]).view(np.float32)  # bmin xyz, bmax xyz
    rng = np.random.default_rng(seed)
    axis_dirs = np.array([(1, 0, 0), (0, 1, 0), (0, 0, 1), (0.6, 0.8, 0), (0, 0.6, 0.8), (0.8, 0, 0.6)], np.float32)
    edge = np.zeros((n_edge, 7), np.float32)
    for k in range(n_edge):
        lo, hi = b[rng.integers(len(b))].reshape(2, 3)
        o = rng.uniform(lo - 5, hi + 5).astype(np.float32)
        on = rng.random(3) < 0.7  # coordinates put exactly on a bound of the node
        o = np.where(on, np.where(rng.random(3) < 0.5, lo, hi), o)
        d = axis_dirs[rng.integers(len(axis_dirs))] * np.where(rng.random(3) < 0.5, -1, 1).astype(np.float32)
        edge[k, :3], edge[k, 3:6], edge[k, 6] = o, d, tmax  # zero components keep their random sign
    return np.concatenate([_random_rays(n_rand, seed, tmax), edge]).astype(np.float32)


TRACE_KERNELS = {  # environment -> the traversal kernel the scene then renders with
    "k_trace_w": {},
    "k_trace_lds": {"PT_TRACE_WIDE": "0"},
    "k_trace_oct": {"PT_TRACE_OCT": "1"},
    "k_trace_nb_lds": {"PT_TRACE_LEAN": "0"},
    "k_trace_w_hbm": {"PT_TRACE_LDS": "0"},
    "k_trace_w_hbm_spill": {"PT_TRACE_LDS": "0", "PT_WIDE_LDS_ROWS": "2"},
    "k_trace_nb_hbm": {"PT_TRACE_LDS": "0", "PT_TRACE_WIDE": "0"},
    "k_trace_pt": {"PT_TRACE_PERSIST": "1"},
    "k_trace_pt_spill": {"PT_TRACE_PERSIST": "1", "PT_STACK_ROWS": "2", "PT_TRACE_LDS": "0", "PT_TRACE_WIDE": "0"},
    "k_trace": {"PT_TRACE_PERSIST": "0"},
}


@pytest.mark.parametrize("kernel", sorted(TRACE_KERNELS))
@pytest.mark.parametrize("any_hit", [False, True])
def test_frame_traversal_kernels_bit_exact(variant, monkeypatch, kernel, any_hit):
    """Every traversal kernel pt_render can run, on random and slab-edge-case
    rays: the hit primitive (closest) or occlusion flag (any-hit) and the
    reference's node-visit / primitive-test counters equal the oracle's."""
    for k, v in TRACE_KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    hs, sc = _scene(variant(**MINI))
    rays = _edge_rays(sc, 6000, 6000, 5, np.inf if not any_hit else 300.0)
    _, order = sc.bvh()
    assert sc.kernel_names()[0] == {"k_trace_nb_lds": "k_trace_nb", "k_trace_nb_hbm": "k_trace_nb",
                                    "k_trace_pt_spill": "k_trace_pt", "k_trace_w_hbm": "k_trace_w",
                                    "k_trace_w_hbm_spill": "k_trace_w"}.get(kernel, kernel)
    got, nodes, prims = sc.debug_trace_frame(rays, any_hit)
    ref, rnodes, rprims = pyoracle.trace_counted(hs.desc, rays, any_hit)
    if not any_hit:
        got = np.where(got >= 0, order[np.maximum(got, 0)], -1)
    assert np.array_equal(got, ref)
    if not kernel.startswith("k_trace_w"):  # k_trace_w's node / prim counters cover only the rays it retraced
        assert (nodes, prims) == (rnodes, rprims)


@pytest.mark.parametrize("kernel", ["k_trace_w", "k_trace_w_hbm", "k_trace_lds", "k_trace_pt", "k_trace_nb_hbm"])
def test_frame_traversal_tmax_edge_cases(variant, monkeypatch, kernel):
    """The box test's tMax comparison (tMin < ray.tMax) at the edge values:
    0, +-denormals, the denormal range, NaN, negative and random finite tMax
    around box distances.  Shadow rays (the rays whose tMax the trace
    kernels read from the record: closest-hit rays start at tMax = inf, as
    SpawnRay's, interaction.h:66-69) with such tMax values mixed into every
    wave, and tMax values around box distances: occlusion and node /
    primitive counters equal the oracle's (Bounds3::IntersectP,
    geometry.h:1584-1606, tMin < ray.tMax && tMax > 0)."""
    any_hit = True
    for k, v in TRACE_KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    hs, sc = _scene(variant(**MINI))
    rays = _edge_rays(sc, 4000, 4000, 11, np.inf)
    rng = np.random.default_rng(12)
    tiny = np.array([0.0, -0.0, 1e-45, 3e-45, 1e-40, 1.17549435e-38, 1e-30, np.nan, -1.0], np.float32)
    pick = rng.random(len(rays))
    tm = np.where(pick < 0.15, tiny[rng.integers(len(tiny), size=len(rays))],
                  np.where(pick < 0.6, rng.uniform(0, 20, len(rays)).astype(np.float32), np.float32(np.inf)))
    rays[:, 6] = tm.astype(np.float32)
    got, nodes, prims = sc.debug_trace_frame(rays, any_hit)
    ref, rnodes, rprims = pyoracle.trace_counted(hs.desc, rays, any_hit)
    assert np.array_equal(got, ref)
    if not kernel.startswith("k_trace_w"):
        assert (nodes, prims) == (rnodes, rprims)


def test_bvh_device_matches_oracle(variant):
    hs, sc = _scene(variant(**MINI))
    n1, o1 = sc.bvh()
    n2, o2 = pyoracle.build_bvh(hs.desc)
    assert np.array_equal(n1, n2)
    assert np.array_equal(o1, o2[:len(o1)])


def _rmse(a, b):
    # imgtool diff metric: MSE over 3*w*h channel values (src/tools/imgtool.cpp:333-441)
    return float(np.sqrt(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)))


@pytest.mark.parametrize("strategy", ["portal", "light", "projection"])
def test_render_matches_oracle(variant, strategy):
    path = variant(strategy=strategy, **MINI)
    hs, sc = _scene(path)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert got.shape == ref.shape
    assert np.isfinite(got).all()
    rmse = _rmse(got, ref)
    scale = max(1.0, float(np.mean(ref)))
    exact = float(np.mean(np.all(got.view(np.uint32) == ref.view(np.uint32), axis=2)))
    print(f"{strategy}: rmse={rmse:.3g} mean={ref.mean():.5g} bit-exact pixels={exact:.4f} "
          f"rays gpu={gst['closest_rays']}/{gst['shadow_rays']} oracle={rst['closest_rays']}/{rst['shadow_rays']}")
    assert rmse / scale < 1e-4          # north_star tolerance
    assert exact == 1.0                 # in fact bit-identical (same float ops, same order)
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_render_accum_tiles_partition(variant):
    hs, sc = _scene(variant(**MINI))
    full, _ = sc.render_accum(0, 1)
    a0, _ = sc.render_accum(0, 2)
    a1, _ = sc.render_accum(1, 2)
    np.testing.assert_allclose(a0 + a1, full, rtol=1e-6, atol=1e-6)


def test_furnace_known_answer(tmp_path):
    """src/tests/analytic_scenes.cpp:135-165 known answer (1.0 +- 0.02)."""
    hs, sc = _scene(furnace_scene(tmp_path, res=10, spp=256, maxdepth=8))
    img, _ = sc.render()
    assert abs(float(img.mean()) - 1.0) < 0.02


def test_small_batches_equal_large(variant):
    """Batching the sample range differently must not change the image."""
    path = variant(**MINI)
    hs = ptgpu.HostScene(path)
    a, _ = ptgpu.Scene(hs).render()
    b, _ = ptgpu.Scene(hs, batch_slots=64 * 36 * 3).render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_film_accumulation_matches_oracle(variant):
    """The device film (XYZ + weight per pixel, tile partials merged in tile
    order) against the oracle's Film::MergeFilmTile result."""
    hs, sc = _scene(variant(**MINI))
    got, _ = sc.render_accum(0, 1)
    ref, _ = pyoracle.render_accum(hs.desc, nthreads=8)
    exact = float(np.mean(np.all(got.view(np.uint32) == ref.view(np.uint32), axis=2)))
    print(f"film: bit-exact pixels={exact:.4f} max|d|={np.abs(got - ref).max():.3g}")
    assert exact == 1.0


def test_sample_range_matches_oracle(variant):
    """pt_render_range (the bench's sharding unit) for samples [16, 24) --
    past the scene's spp, as rank 1 of a weak-scaled run renders them."""
    hs, sc = _scene(variant(**MINI))
    got, gst = sc.render_range(16, 24)
    ref, rst = pyoracle.render_range(hs.desc, 16, 24, nthreads=8)
    assert gst["samples"] == rst["samples"] == 64 * 36 * 8
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_tile_groups_batching_equal(variant):
    """Batches of whole tiles (several groups) and of sample chunks inside a
    tile must reproduce the single-batch film bit for bit where the batch
    holds whole tiles, and within float rounding otherwise."""
    path = variant(res=(80, 40), spp=8)
    hs = ptgpu.HostScene(path)
    one, _ = ptgpu.Scene(hs).render_accum(0, 1)
    groups, _ = ptgpu.Scene(hs, batch_slots=16 * 16 * 8 * 3).render_accum(0, 1)   # 3 tiles per batch
    assert np.array_equal(one.view(np.uint32), groups.view(np.uint32))
    chunks, _ = ptgpu.Scene(hs, batch_slots=16 * 16 * 3).render_accum(0, 1)       # 3 samples per batch
    np.testing.assert_allclose(chunks, one, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("env", [{"PT_STACK_ROWS": "2"}, {"PT_TRACE_PERSIST": "0"}, {"PT_TRACE_PERSIST": "1"},
                                 {"PT_TRACE_PERSIST": "2"}, {"PT_TRACE_LDS": "0"},
                                 {"PT_TRACE_LDS": "0", "PT_TRACE_PERSIST": "2"}, {"PT_TRACE_OCT": "1"},
                                 {"PT_TRACE_WIDE": "0"}, {"PT_LEAF_MIN_W": "1"}, {"PT_LEAF_MIN_W": "64"},
                                 {"PT_TRACE_LDS": "0", "PT_WIDE_LDS_ROWS": "2"}])
def test_trace_variants_bit_exact(variant, monkeypatch, env):
    """Every traversal variant the driver can pick -- LDS stack with global
    spill (forced by a 2-entry LDS stack), the non-persistent kernel, the
    global-memory BVH -- renders the oracle's image bit for bit."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    hs, sc = _scene(variant(**MINI))
    got, gst = sc.render()
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("closest_rays", "shadow_rays", "node_visits", "prim_tests"))


SHADE_VARIANTS = [
    {"PT_SHADE_VARIANT": "0"},                          # k_shade (scene tables from HBM)
    {"PT_SHADE_VARIANT": "5"},                          # k_shade_tab, 2 waves per SIMD
    {"PT_SHADE_VARIANT": "3"},                          # k_shade_w3 (MIS scenes: the kLean 3-wave build)
    {"PT_SHADE_VARIANT": "3", "PT_SHADE_TAB": "0"},     # no table room: falls back to k_shade
    {"PT_SHADE_VARIANT": "5", "PT_SHADE_TAB": "0"},
    {"PT_SHADE_VARIANT": "4"},                          # k_shade_w3h: 3 waves, scene tables from HBM
    {"PT_SHADE_TAB": "0"},                              # default without table room (C5: k_shade_w3h if portal-only)
    {"PT_SHADE_SORT": "1"},                             # the path queue grouped by material class (k_shade_sort)
]


@pytest.mark.parametrize("scene", ["portal_cornell.pbrt", "portal_room.pbrt", "lamp/lamp.pbrt",
                                   "cornell_dielectric.pbrt"])
@pytest.mark.parametrize("env", SHADE_VARIANTS, ids=lambda e: "-".join("%s=%s" % kv for kv in e.items()))
def test_shade_variants_bit_exact(tmp_path, monkeypatch, scene, env):
    """Every shading build PT_SHADE_VARIANT can select, on a portal-only scene
    (C2), a portal + infinite-light MIS scene (C4), the reference's lamp
    scene (MIS over a diffuse aaplane + portal light) and the dielectric
    Cornell box (C3: smooth and rough dispersive glass + infinite light, the
    kFtMicro | kFtSpecular | kFtInfinite instantiation), renders the oracle's
    image bit for bit.  PT_SHADE_TAB=0 leaves no LDS room for the scene tables:
    variants 3 / 5 then fall back to k_shade instead of copying past the
    launch's LDS."""
    from conftest import scene_variant
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    path = scene_variant(tmp_path, name=scene, res=(48, 32), spp=8)
    hs, sc = _scene(path)
    if env == {"PT_SHADE_TAB": "0"}:
        assert sc.kernel_names()[1] == {"portal_cornell.pbrt": "k_shade_w3h", "portal_room.pbrt": "k_shade",
                                        "lamp/lamp.pbrt": "k_shade_dl", "cornell_dielectric.pbrt": "k_shade"}[scene]
    got, gst = sc.render()
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_shade_variant_rejects_unknown(variant, monkeypatch):
    monkeypatch.setenv("PT_SHADE_VARIANT", "7")
    hs = ptgpu.HostScene(variant(**MINI))
    with pytest.raises(ptgpu.PtError, match="PT_SHADE_VARIANT"):
        ptgpu.Scene(hs)


def _bsdf_records(n, seed):
    rng = np.random.default_rng(seed)
    wo = rng.normal(size=(n, 3))
    wo[: n // 8] = [1e-3, -2e-3, 1.0]               # normal incidence: TrowbridgeReitzSample11's double branch
    wo[n // 8: n // 4, 2] = np.abs(wo[n // 8: n // 4, 2]) * 50
    wo /= np.linalg.norm(wo, axis=1, keepdims=True)
    wi = rng.normal(size=(n, 3))
    wi /= np.linalg.norm(wi, axis=1, keepdims=True)
    wi[::5] = 0                                      # sample-only records
    u = rng.random((n, 2)) * 0.99999994
    return np.concatenate([wo, wi, u], 1).astype(np.float32)


@pytest.mark.parametrize("rough", ['"float roughness" [0.3]', '"float uroughness" [0.0] "float vroughness" [0.0]',
                                   '"float uroughness" [0.6] "float vroughness" [0.05]'])
def test_metal_bsdf_bit_exact(tmp_path, rough):
    """BSDF::f / Pdf / Sample_f of MetalMaterial (TrowbridgeReitz visible-normal
    sampling, FresnelConductor) and of the matte materials: device == oracle."""
    from test_materials import _metal_index, metal_scene
    hs, sc = _scene(metal_scene(tmp_path, rough=rough, **MINI))
    rec = _bsdf_records(20000, 11)
    for mat in range(len(hs.materials())):
        got = sc.debug_bsdf(mat, rec)
        ref = pyoracle.bsdf_batch(hs.desc, mat, rec)
        bad = np.nonzero(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=1))[0]
        assert len(bad) == 0, (mat, bad[:5], got[bad[:3]], ref[bad[:3]])
    assert _metal_index(hs) >= 0


@pytest.mark.parametrize("strategy", ["portal", "projection"])
def test_metal_render_matches_oracle(tmp_path, strategy):
    from test_materials import metal_scene
    hs, sc = _scene(metal_scene(tmp_path, rough='"float uroughness" [0.05] "float vroughness" [0.2]',
                                strategy=strategy, **MINI))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"]


def test_plymesh_metal_render_matches_oracle(tmp_path):
    from test_materials import ply_scene
    hs, sc = _scene(ply_scene(tmp_path, material='Material "metal" "rgb eta" [0.8 0.8 0.8] "rgb k" [0.8 0.8 0.8] '
                                                 '"float roughness" [0.1]', **MINI))
    ref, _ = pyoracle.render(hs.desc, nthreads=8)
    got, _ = sc.render()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


AREA_TRI = '''AttributeBegin
  AreaLightSource "diffuse" "rgb L" [8 6 4]
  Shape "trianglemesh" "point P" [-1 3 -1  1 3 -1  0 3 1] "integer indices" [0 1 2]
AttributeEnd
'''
METAL_BALL = '''AttributeBegin
  Material "metal" "rgb eta" [0.2 0.9 1.1] "rgb k" [3.9 2.4 2.2] "float roughness" [0.2]
  Shape "trianglemesh" "point P" [-2 0.01 -2  2 0.01 -2  0 2 0  2 0.01 2  -2 0.01 2]
        "integer indices" [0 1 2  1 3 2  3 4 2  4 0 2]
AttributeEnd
'''


@pytest.mark.parametrize("extra,strategy", [("plane", ""), ("plane+area", ""),
                                            ("plane+area+metal", '"string lightsamplestrategy" "power"')])
def test_infinite_light_render_matches_oracle(tmp_path, extra, strategy):
    """InfiniteAreaLight: escaped-ray Le, Sample_Li through the Distribution2D,
    Pdf_Li (acosf/atan2f ported from the reference's libm), MIS with area
    lights, power light distribution -- device == oracle bit for bit."""
    from test_infinite import FAR, PLANE, sky_scene
    parts = {"plane": PLANE, "area": AREA_TRI, "metal": METAL_BALL}
    ex = "".join(parts[k] for k in extra.split("+")) + FAR
    hs, sc = _scene(sky_scene(tmp_path, w=48, h=32, spp=16, rot=37, L="0.6 0.8 1.3", extra=ex, istrat=strategy))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"{extra}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"] and gst["shadow_rays"] == rst["shadow_rays"]


NEW_MATERIALS = [
    'Material "glass" "float index" [1.5]',
    'Material "glass" "float index" [1.33] "float uroughness" [0.4] "float vroughness" [0.15] "rgb Kr" [0.5 0.6 0.7]',
    'Material "glass" "float index" [1.6] "float roughness" [0.05] "bool remaproughness" "true"',
    'Material "dispersive_glass" "float etaMin" [1.3] "float etaMax" [1.6]',
    'Material "mirror" "rgb Kr" [0.8 0.7 0.9]',
    'Material "plastic" "rgb Kd" [0.4 0.3 0.2] "rgb Ks" [0.5 0.5 0.5] "float roughness" [0.1]',
    'Material "plastic" "rgb Kd" [0.1 0.6 0.2] "float roughness" [0.6] "bool remaproughness" "false"',
]


@pytest.mark.parametrize("material", NEW_MATERIALS)
def test_multilobe_bsdf_bit_exact(tmp_path, material):
    """BSDF::f / Pdf / Sample_f of the glass (FresnelSpecular, and
    MicrofacetReflection + MicrofacetTransmission), dispersive glass, mirror
    and plastic materials, from both sides of the surface: device == oracle."""
    from test_materials import material_scene
    hs, sc = _scene(material_scene(tmp_path, material, **MINI))
    rec = _bsdf_records(20000, 12)
    rec[1::3, 2] = -rec[1::3, 2]                    # wo below the surface: inside the dielectric
    for mat in range(len(hs.materials())):
        got = sc.debug_bsdf(mat, rec)
        ref = pyoracle.bsdf_batch(hs.desc, mat, rec)
        bad = np.nonzero(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=1))[0]
        assert len(bad) == 0, (mat, bad[:5], got[bad[:3]], ref[bad[:3]])


@pytest.mark.parametrize("material", NEW_MATERIALS)
@pytest.mark.parametrize("strategy", ["portal", "projection"])
def test_multilobe_render_matches_oracle(tmp_path, material, strategy):
    """Renders through the new materials: specular bounces (Le and NEE gating),
    etaScale / Russian roulette, dispersive wavelength from camera dimension 5."""
    from test_materials import material_scene
    hs, sc = _scene(material_scene(tmp_path, material, strategy=strategy, maxdepth=8, **MINI))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"{material[:40]}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"] and gst["shadow_rays"] == rst["shadow_rays"]


def test_loopsubdiv_render_matches_oracle(tmp_path):
    """A Loop-subdivided mesh (limit positions + shading normals, loopsubdiv.cpp)
    under glossy plastic: device == oracle bit for bit."""
    from test_loopsubdiv import _scene as loop_scene, icosa
    P, idx = icosa()
    hs, sc = _scene(loop_scene(tmp_path, P, idx, 2, xform="Rotate 20 0 1 0",
                           material='Material "plastic" "rgb Kd" [0.4 0.2 0.2] "float roughness" [0.05]'))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"]


@pytest.mark.parametrize("any_hit", [False, True])
def test_sphere_traversal_bit_exact(tmp_path, any_hit):
    """Sphere::Intersect / IntersectP (EFloat bounds, clipped and transformed
    spheres) in the device traversal == oracle, ray for ray."""
    from test_sphere import spheres_scene
    hs, sc = _scene(spheres_scene(tmp_path))
    rng = np.random.default_rng(9)
    n = 20000
    o = np.stack([rng.uniform(-5, 5, n), rng.uniform(-2, 5, n), rng.uniform(-6, 2, n)], 1)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, np.full((n, 1), np.inf if not any_hit else 4.0)], 1).astype(np.float32)
    _, order = sc.bvh()
    got = sc.debug_trace(rays, any_hit)
    ref = pyoracle.trace(hs.desc, rays, any_hit)
    if not any_hit:
        got = np.where(got >= 0, order[np.maximum(got, 0)], -1)
    else:
        got = (got >= 0).astype(np.int32)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("which", ["furnace", "light", "light_power", "spheres"])
def test_sphere_render_matches_oracle(tmp_path, which):
    """Sphere area lights (area sampling from inside, cone sampling from
    outside, Sphere::Pdf), clipped/transformed spheres: device == oracle."""
    import test_sphere as ts
    if which == "furnace":
        path = ts.sphere_furnace(tmp_path, spp=64)
    elif which == "light":
        path = ts.sphere_light_scene(tmp_path, maxdepth=4, spp=32)
    elif which == "light_power":
        extra = 'AttributeBegin\n  Translate 3 0 6\n  AreaLightSource "area" "rgb L" [3 3 3]\n' \
                '  Material "glass"\n  Shape "sphere" "float radius" [2]\nAttributeEnd\n'
        path = ts.sphere_light_scene(tmp_path, maxdepth=6, spp=32, extra=extra,
                                     strategy='"string lightsamplestrategy" "power"')
    else:
        path = ts.spheres_scene(tmp_path)
    hs, sc = _scene(path)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"{which}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"] and gst["shadow_rays"] == rst["shadow_rays"]


@pytest.mark.parametrize("extra", ["", "sphere", "power"])
def test_point_light_render_matches_oracle(tmp_path, extra):
    """PointLight (delta light: no MIS weight, no BSDF-sampled light ray),
    alone, next to a sphere light, and under "power" light selection."""
    import test_sphere as ts
    ex = ""
    if extra:
        ex = 'AttributeBegin\n  Translate 1 1 3\n  AreaLightSource "area" "rgb L" [2 2 2]\n' \
             '  Shape "sphere" "float radius" [0.5]\nAttributeEnd\n'
    hs, sc = _scene(ts.point_light_scene(tmp_path, maxdepth=5, spp=32, extra=ex,
                                         strategy='"string lightsamplestrategy" "power"' if extra == "power" else ""))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"] and gst["shadow_rays"] == rst["shadow_rays"]


def _dl_cases(tmp_path, which):
    import test_direct as td
    if which.startswith("furnace"):
        _, st, ns = which.split("-")
        return td.dl_sphere_furnace(tmp_path, st, int(ns), spp=16)
    if which == "point":
        return td.point_scene(tmp_path, "all")
    if which == "mirror":
        return td.point_scene(tmp_path, mirror='Material "mirror" "rgb Kr" [0.8 0.7 0.6]')
    if which == "glass":
        return td.point_scene(tmp_path, mirror='Material "glass" "float index" [1.5]', maxdepth=6)
    if which == "dispersive":
        return td.point_scene(tmp_path, "one", mirror='Material "dispersive_glass" "float etaMin" [1.3] '
                                                      '"float etaMax" [1.7]', maxdepth=4)
    if which == "mixed":
        extra = 'AttributeBegin\n  Translate 0.5 0.5 2\n  AreaLightSource "area" "rgb L" [4 4 4] ' \
                '"integer nsamples" [3]\n  Material "plastic"\n  Shape "sphere" "float radius" [0.3]\nAttributeEnd\n'
        return td.point_scene(tmp_path, "all", spp=16, extra=extra)
    # the portal Cornell scene under DirectLighting, both strategies
    return scene_variant_dl(tmp_path, which)


def scene_variant_dl(tmp_path, which):
    from conftest import scene_variant
    st = which.split("-")[1]
    return scene_variant(tmp_path, res=(48, 32), spp=8, strategy="portal",
                         extra=[('Integrator "path"', f'Integrator "directlighting" "string strategy" "{st}"')])


@pytest.mark.parametrize("which", ["furnace-all-1", "furnace-all-4", "furnace-one-4", "point", "mirror", "glass",
                                   "dispersive", "mixed", "cornell-all", "cornell-one"])
def test_directlighting_render_matches_oracle(tmp_path, which):
    """DirectLightingIntegrator on the device (sample arrays, UniformSampleAll/
    OneLight, the SpecularReflect / SpecularTransmit recursion with its stack
    of frames) == oracle, bit for bit, with identical ray counts."""
    hs, sc = _scene(_dl_cases(tmp_path, which))
    assert ptgpu.integrator_desc(hs).kind == 1
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"{which}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst["closest_rays"] == rst["closest_rays"] and gst["shadow_rays"] == rst["shadow_rays"]


def test_directlighting_single_lobe_glass_bsdf_bit_exact(tmp_path):
    """allowMultipleLobes = false: SpecularReflection(FresnelDielectric) +
    SpecularTransmission in place of FresnelSpecular."""
    import test_direct as td
    hs, sc = _scene(td.point_scene(tmp_path, mirror='Material "glass" "float index" [1.45] "rgb Kt" [0.9 0.8 0.7]'))
    rec = _bsdf_records(20000, 13)
    rec[1::3, 2] = -rec[1::3, 2]
    mat = [i for i, m in enumerate(hs.materials()) if m.kind == 3][0]
    got = sc.debug_bsdf(mat, rec)
    ref = pyoracle.bsdf_batch(hs.desc, mat, rec)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("strategy", ["portal", "light", "projection"])
def test_portal_room_matches_oracle(tmp_path, strategy):
    """Config 4 (four portals on one emitter + an infinite light, maxdepth 8)
    at a reduced film: device == oracle bit for bit."""
    from conftest import scene_variant
    hs, sc = _scene(scene_variant(tmp_path, name="portal_room.pbrt", res=(96, 54), spp=16, strategy=strategy))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"room/{strategy}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_cornell_dielectric_matches_oracle(tmp_path):
    """Config 3 (reference scenes/cornell_dielectric.pbrt: spectral walls and
    lights reduced to RGB, specular + rough dispersive glass, infinite light,
    gaussian filter; path maxdepth 5) at a reduced film: device == oracle bit
    for bit, identical ray / node / primitive counts."""
    from conftest import scene_variant
    hs, sc = _scene(scene_variant(tmp_path, name="cornell_dielectric.pbrt", res=(64, 64), spp=16))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"cornell_dielectric: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert ref.mean() > 0
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.parametrize("integrator", ["mypath", "directlighting"])
def test_killeroo_simple_matches_oracle(tmp_path, integrator):
    """Config 1 scene (reference scenes/killeroo-simple.pbrt: Loop-subdivided
    killeroos, plastic, sphere area light) as written ("mypath": no Russian
    roulette) and with the DirectLighting integrator config 1 names, at a
    reduced film: device == oracle bit for bit."""
    from conftest import scene_variant
    extra = [('Integrator "mypath" "integer maxdepth" 3', 'Integrator "directlighting"')] \
        if integrator == "directlighting" else None
    hs, sc = _scene(scene_variant(tmp_path, name="killeroo-simple.pbrt", res=(48, 48), spp=4, extra=extra))
    assert ptgpu.integrator_desc(hs).kind == (1 if integrator == "directlighting" else 0)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"killeroo/{integrator}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_killeroo_atrium_matches_oracle(tmp_path):
    """Config 5 scene family (scripts/make_atrium.py: Loop-subdivided
    killeroos in a skylight-portal atrium) with 12 copies (0.4 M triangles,
    same code path as the 300-copy / 10 M-triangle bench scene) at a reduced
    film: device == oracle bit for bit, identical traversal counters."""
    import re
    import subprocess
    import sys
    from conftest import REPO, SCENES
    src = tmp_path / "atrium12.pbrt"
    subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "make_atrium.py"), str(src),
                           "--copies", "12"])
    txt = src.read_text()
    txt = re.sub(r'Include "([^"]+)"', lambda m: 'Include "%s/%s"' % (SCENES, m.group(1)), txt)
    txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [64]', txt)
    txt = re.sub(r'"integer yresolution" \[\d+\]', '"integer yresolution" [36]', txt)
    txt = re.sub(r'"integer pixelsamples" \[\d+\]', '"integer pixelsamples" [4]', txt)
    src.write_text(txt)
    hs, sc = _scene(str(src))
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"atrium12: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_killeroo_atrium_full_scale_matches_oracle(tmp_path):
    """Config 5 as benchmarked: scenes/killeroo_atrium.pbrt, 300 Loop-
    subdivided killeroos, 9.98 M triangles, 17.95 M BVH nodes (prim indices far
    above 2^23, a stack deeper than the LDS rows: k_trace_pt's spill path), at
    a 64x36 @2 film: device == oracle bit for bit with identical traversal
    counters."""
    from conftest import scene_variant
    hs, sc = _scene(scene_variant(tmp_path, name="killeroo_atrium.pbrt", res=(64, 36), spp=2))
    assert hs.film_size() == (64, 36)
    ref, rst = pyoracle.render(hs.desc, nthreads=16)
    got, gst = sc.render()
    print(f"atrium300: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g} nodes={gst['node_visits']}")
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


LAMP_AS_PATH = [('Integrator "directlighting"', 'Integrator "path" "integer maxdepth" [5]'),
                ('"integer maxdepth" [100]', '')]


@pytest.mark.parametrize("integrator", ["directlighting", "path"])
@pytest.mark.parametrize("strategy", ["projection", "light", "portal"])
def test_lamp_matches_oracle(tmp_path, integrator, strategy):
    """The reference's own portal scene (scenes/lamp/lamp.pbrt, imported
    verbatim): two axis-2 portals, the second '+'-facing (AAPortal facingFw,
    aaportal.cpp:8-13; AAPlaneShape::InFront / Normal, plane.cpp:74-115),
    plymesh room / lampshade, metal leg and base.  As written
    (DirectLighting maxdepth 100, strategy projection, 5 spp) and as path
    maxdepth 5 with each strategy, at 100x100: device == oracle bit for bit,
    identical ray / node / primitive counters."""
    from conftest import scene_variant
    hs, sc = _scene(scene_variant(tmp_path, name="lamp/lamp.pbrt", res=(100, 100),
                                  spp=5 if integrator == "directlighting" else 8, strategy=strategy,
                                  extra=LAMP_AS_PATH if integrator == "path" else None))
    assert ptgpu.integrator_desc(hs).kind == (1 if integrator == "directlighting" else 0)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"lamp/{integrator}/{strategy}: mean={ref.mean():.5g} rmse={_rmse(got, ref):.3g}")
    assert ref.mean() > 0
    assert _rmse(got, ref) / max(1.0, float(ref.mean())) < 1e-4
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.parametrize("filt,spp", [("gaussian", 70), ("box", 9), ("gaussian3", 5)])
def test_film_pixel_lanes_match_oracle(tmp_path, monkeypatch, filt, spp):
    """k_film_t (opt-in PT_FILM_T=1: the RGB film with one lane per film
    pixel, 8x8 pixels per wave; filter windows of 2-16 pixels): the 2-pixel Gaussian of config 3 at
    70 spp (two 64-sample chunks per source pixel) and a 3-pixel Gaussian,
    plus the box filter (k_film), under a crop window with an odd film size
    and batches of two FilmTiles == the oracle's film bit for bit, and ==
    k_film (PT_FILM_T=0)."""
    import re
    from conftest import scene_variant
    path = scene_variant(tmp_path, name="cornell_dielectric.pbrt", res=(45, 38), spp=spp)
    txt = open(path).read().replace('Film "image"', 'Film "image" "float cropwindow" [0.07 0.95 0.12 0.9]')
    if filt == "box":
        txt = re.sub(r'PixelFilter "gaussian"\s*"float xwidth" \[2\]\s*"float ywidth" \[2\]', 'PixelFilter "box"', txt)
    elif filt == "gaussian3":
        txt = re.sub(r'"float ([xy])width" \[2\]', r'"float \1width" [3]', txt)
    p = tmp_path / f"film_{filt}.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    slots = 16 * 16 * spp * 2
    monkeypatch.setenv("PT_FILM_T", "1")
    got, _ = ptgpu.Scene(hs, batch_slots=slots).render_accum(0, 1)
    ref, _ = pyoracle.render_accum(hs.desc, nthreads=8)
    assert ref[..., 3].max() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    monkeypatch.setenv("PT_FILM_T", "0")
    old, _ = ptgpu.Scene(hs, batch_slots=slots).render_accum(0, 1)
    assert np.array_equal(old.view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("filt,spp,skew", [("gaussian", 68, "1"), ("gaussian", 70, "2"), ("gaussian", 68, "0"),
                                           ("gaussian", 68, "2"), ("box", 12, "1"), ("box", 9, "0"), ("box", 12, "2")])
def test_film_skewed_lanes_match_oracle(tmp_path, monkeypatch, filt, spp, skew):
    """k_film_sk (PT_FILM_SK=1: one lane per film pixel, the lanes' window
    walks unskewed (0), skewed by column (1) or so that every lane needing a
    source pixel reads it at the same step (2); the footprint from k_camera's
    FilmMeta records): the 2-pixel Gaussian
    of config 3 and the box filter, at sample counts that take the four-sample
    loads (68, 12) and the one-sample loop (70, 9), under a crop window with an
    odd film size and batches of two FilmTiles == the oracle's film bit for
    bit, and == k_film."""
    import re
    from conftest import scene_variant
    path = scene_variant(tmp_path, name="cornell_dielectric.pbrt", res=(45, 38), spp=spp)
    txt = open(path).read().replace('Film "image"', 'Film "image" "float cropwindow" [0.07 0.95 0.12 0.9]')
    if filt == "box":
        txt = re.sub(r'PixelFilter "gaussian"\s*"float xwidth" \[2\]\s*"float ywidth" \[2\]', 'PixelFilter "box"', txt)
    p = tmp_path / f"film_sk_{filt}.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    slots = 16 * 16 * spp * 2
    monkeypatch.setenv("PT_FILM_SK", "1")
    monkeypatch.setenv("PT_FILM_SKEW", skew)
    got, _ = ptgpu.Scene(hs, batch_slots=slots).render_accum(0, 1)
    ref, _ = pyoracle.render_accum(hs.desc, nthreads=8)
    assert ref[..., 3].max() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    monkeypatch.setenv("PT_FILM_SK", "0")
    old, _ = ptgpu.Scene(hs, batch_slots=slots).render_accum(0, 1)
    assert np.array_equal(old.view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("film_sk", ["1", "0"])
def test_film_max_sample_luminance_matches_oracle(tmp_path, monkeypatch, film_sk):
    """A finite Film "maxsampleluminance" (AddSample's clamp, film.h:121-161,
    after the radiance sanitiser, integrator.cpp:592-613) with the 2-pixel
    Gaussian: k_film_prep + k_film_sk (the default for this window) and k_film
    == the oracle's film bit for bit."""
    from conftest import scene_variant
    path = scene_variant(tmp_path, name="cornell_dielectric.pbrt", res=(40, 34), spp=16)
    txt = open(path).read().replace('Film "image"', 'Film "image" "float maxsampleluminance" [0.35]')
    p = tmp_path / "film_maxlum.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    monkeypatch.setenv("PT_FILM_SK", film_sk)
    got, _ = ptgpu.Scene(hs, batch_slots=16 * 16 * 16 * 2).render_accum(0, 1)
    ref, _ = pyoracle.render_accum(hs.desc, nthreads=8)
    assert ref[..., 3].max() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_full_config_sparse_tiles_bit_exact():
    """Parity at the benchmarked configuration: the C2 scene as benchmarked
    (1920x1080 @256 spp, path maxdepth 5, the default 96 M-slot batches and
    two pipelines) on the tiles t % 400 == 0 spread over the whole frame,
    against the oracle's film of the same tiles (SamplerIntegrator::Render,
    integrator.cpp:526-637) -- bit-identical film and identical counters."""
    hs = ptgpu.HostScene(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes",
                                      "portal_cornell.pbrt"))
    sc = ptgpu.Scene(hs)
    assert sc.film_size() == (1920, 1080)
    got, gst = sc.render_accum(0, 400)
    ref, rst = pyoracle.render_accum(hs.desc, nthreads=16, tile_offset=0, tile_stride=400)
    assert gst["samples"] == rst["samples"] == 21 * 256 * 256
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.parametrize("equal", ["1", "2"])
def test_batch_equal_two_pipelines_bit_exact(tmp_path, monkeypatch, equal):
    """PT_BATCH_EQUAL splits a render into equal batches (rounded to whole
    16x16 tiles: the FilmTile boundaries the ordered film merge depends on)
    run by two pipelines: a full render and a rank's tile shard
    (render_accum(rank, nranks)) give the oracle's film bit for bit."""
    from conftest import scene_variant
    monkeypatch.setenv("PT_BATCH_EQUAL", equal)
    monkeypatch.setenv("PT_PIPES", "2")
    path = scene_variant(tmp_path, name="portal_cornell.pbrt", res=(120, 72), spp=8)
    hs = ptgpu.HostScene(path)
    sc = ptgpu.Scene(hs, batch_slots=16 * 16 * 8 * 7)  # several batches per render
    assert sc.query("pipelines") == 2
    got, gst = sc.render_accum(0, 1)
    ref, rst = pyoracle.render_accum(hs.desc, nthreads=8)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    for r in range(3):
        got, gst = sc.render_accum(r, 3)
        ref, rst = pyoracle.render_accum(hs.desc, nthreads=8, tile_offset=r, tile_stride=3)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        assert_counters(gst, rst, ("samples", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_default_pipelines_follow_bvh_residency(tmp_path, monkeypatch):
    """Two pipelines by default for a BVH in LDS and for the wide traversal from
    HBM (PT_TRACE_LDS=0 forces it; C5's case), one for the binary traversal
    from HBM (PT_TRACE_WIDE=0 as well: scenes with spheres), and all render the
    oracle's film bit for bit."""
    from conftest import scene_variant
    monkeypatch.delenv("PT_PIPES", raising=False)
    path = scene_variant(tmp_path, name="portal_cornell.pbrt", res=(64, 48), spp=4)
    hs = ptgpu.HostScene(path)
    ref, rst = pyoracle.render_accum(hs.desc, nthreads=8)
    for lds, wide, pipes in (("1", "1", 2), ("0", "1", 2), ("0", "0", 1)):
        monkeypatch.setenv("PT_TRACE_LDS", lds)
        monkeypatch.setenv("PT_TRACE_WIDE", wide)
        sc = ptgpu.Scene(hs, batch_slots=16 * 16 * 4 * 3)
        assert sc.query("pipelines") == pipes
        got, gst = sc.render_accum(0, 1)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        assert_counters(gst, rst, ("samples", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


def test_count_bytes_build_renders_the_same(variant):
    """pt_set_count_bytes switches to the shading build that counts the
    algorithmic path-state bytes: the same image and counters, shade_bytes > 0
    only when it is on."""
    hs, sc = _scene(variant(**MINI))
    a, sa = sc.render()
    sc.set_count_bytes(True)
    b, sb = sc.render()
    sc.set_count_bytes(False)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa["shade_bytes"] == 0 and sb["shade_bytes"] > 0
    # the counting frame also traverses in the reference's order (binary kernel, reference counters)
    assert sb["trace_wide"] == 0
    assert_counters(sa, sb, ("closest_rays", "shadow_rays", "node_visits", "prim_tests", "shade_launches"))
