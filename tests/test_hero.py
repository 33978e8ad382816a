"""Hero-wavelength integrators (hero_path, hero_path_mis) in the reference's
SampledSpectrum build: 60-bin spectra, four hero wavelengths, dispersive
glass with one BSDF per wavelength, SpatialLightDistribution.

CPU: the loader's 60-bin parameters against an independent numpy restatement
of SampledSpectrum::FromSampled / FromRGB (spectrum.h:310-328,
spectrum.cpp:59-172), bit for bit; the oracle pinned by the reference's
furnace known answer (src/tests/analytic_scenes.cpp:135-165, Le/(1-Kd)) in
spectral form.  GPU: the device megakernel against the oracle, bit for bit,
on the reference's own scenes/cornell_dielectric.pbrt as written."""
import os
import re

import numpy as np
import pytest

import ptgpu
import pyoracle
from conftest import REPO, SCENES, assert_counters

F = np.float32
INC = os.path.join(REPO, "pbrt-v3-light-portals_amd", "csrc", "spectral_tables.inc")


def _tables():
    txt = open(INC).read()
    out = {}
    for name, body in re.findall(r"static const float k(\w+)\[\d+\] = \{(.*?)\};", txt, re.S):
        out[name] = np.array([float.fromhex(t.rstrip("f")) for t in re.findall(r"[-0-9a-fx.p+]+f", body)], F)
    return out


T = _tables()


def _lerp(t, a, b):
    return F(F(F(1) - t) * a) + F(t * b)


def _avg(lam, vals, l0, l1):
    """AverageSpectrumSamples (spectrum.cpp:59-90), float32 with double segment sums."""
    n = len(lam)
    if l1 <= lam[0]:
        return vals[0]
    if l0 >= lam[n - 1]:
        return vals[n - 1]
    if n == 1:
        return vals[0]
    s = F(0)
    if l0 < lam[0]:
        s = F(s + F(vals[0] * F(lam[0] - l0)))
    if l1 > lam[n - 1]:
        s = F(s + F(vals[n - 1] * F(l1 - lam[n - 1])))
    i = 0
    while l0 > lam[i + 1]:
        i += 1
    while i + 1 < n and l1 >= lam[i]:
        a = max(l0, lam[i]) if not (l0 < lam[i]) else lam[i]
        a = l0 if l0 > lam[i] else lam[i]
        b = l1 if l1 < lam[i + 1] else lam[i + 1]
        ia = _lerp(F(F(a - lam[i]) / F(lam[i + 1] - lam[i])), vals[i], vals[i + 1])
        ib = _lerp(F(F(b - lam[i]) / F(lam[i + 1] - lam[i])), vals[i], vals[i + 1])
        s = F(float(s) + 0.5 * float(F(ia + ib)) * float(F(b - a)))
        i += 1
    return F(s / F(l1 - l0))


def _bins():
    out = []
    for i in range(60):
        t0, t1 = F(F(i) / F(60)), F(F(i + 1) / F(60))
        out.append((_lerp(t0, F(400), F(700)), _lerp(t1, F(400), F(700))))
    return out


BINS = _bins()


def from_sampled60(lam, vals):
    lam, vals = np.asarray(lam, F), np.asarray(vals, F)
    return np.array([_avg(lam, vals, a, b) for a, b in BINS], F)


def from_rgb60(rgb, reflectance=False):
    names = ["White", "Cyan", "Magenta", "Yellow", "Red", "Green", "Blue"]
    kind = "Refl" if reflectance else "Illum"
    B = {n: from_sampled60(T["RGB2SpectLambda"], T[f"RGB{kind}2Spect{n}"]) for n in names}
    r = np.zeros(60, F)
    c0, c1, c2 = (F(v) for v in rgb)

    def add(a, n):
        nonlocal r
        r = (r + (B[n] * F(a)).astype(F)).astype(F)
    if c0 <= c1 and c0 <= c2:
        add(c0, "White")
        if c1 <= c2:
            add(F(c1 - c0), "Cyan"); add(F(c2 - c1), "Blue")
        else:
            add(F(c2 - c0), "Cyan"); add(F(c1 - c2), "Green")
    elif c1 <= c0 and c1 <= c2:
        add(c1, "White")
        if c0 <= c2:
            add(F(c0 - c1), "Magenta"); add(F(c2 - c0), "Blue")
        else:
            add(F(c2 - c1), "Magenta"); add(F(c0 - c2), "Red")
    else:
        add(c2, "White")
        if c0 <= c1:
            add(F(c0 - c2), "Yellow"); add(F(c1 - c0), "Green")
        else:
            add(F(c1 - c2), "Yellow"); add(F(c0 - c1), "Red")
    r = (r * (F(.94) if reflectance else F(.86445))).astype(F)
    return np.maximum(r, F(0))


def test_cornell_dielectric_as_written_is_spectral():
    """BASELINE config 3 as written: Integrator "hero_path_mis" (default
    lightsamplestrategy "spatial", three lights) in a SampledSpectrum scene."""
    path = "/tmp/_c3_hero.pbrt"
    txt = open(os.path.join(SCENES, "cornell_dielectric.pbrt")).read()
    txt = txt.replace('Integrator "path" "integer maxdepth" [5]', 'Integrator "hero_path_mis"')
    open(path, "w").write(txt)
    hs = ptgpu.HostScene(path)
    it = ptgpu.integrator_desc(hs)
    assert it.kind == 3 and it.light_strategy == 2 and it.max_depth == 5
    mats, lights = ptgpu.spectral_tables(hs)
    red = re.search(r"# Red wall.*?\"spectrum Kd\" \[(.*?)\]", txt, re.S).group(1).split()
    pairs = np.array(red, np.float64).reshape(-1, 2)
    ref = from_sampled60(pairs[:, 0], pairs[:, 1])
    assert any(np.array_equal(m[0].view(np.uint32), ref.view(np.uint32)) for m in mats)
    d = ptgpu.scene_desc(hs)
    assert d.n_lights == 3 and lights.shape == (3, 60)


def test_rgb_parameters_convert_as_illuminants(tmp_path):
    """ParamSet::AddRGBSpectrum uses FromRGB's Illuminant default in the
    SampledSpectrum build (paramset.cpp:110-120, spectrum.h:420-421)."""
    p = tmp_path / "s.pbrt"
    p.write_text('LookAt 0 0 -5 0 0 0 0 1 0\nCamera "perspective"\nFilm "image" "integer xresolution" [8] '
                 '"integer yresolution" [8]\nSampler "halton" "integer pixelsamples" [1]\n'
                 'Integrator "hero_path"\nWorldBegin\n'
                 'AttributeBegin\nAreaLightSource "diffuse" "rgb L" [3 2 1]\n'
                 'Material "matte" "rgb Kd" [0.2 0.5 0.3]\n'
                 'Shape "trianglemesh" "integer indices" [0 1 2] "point P" [-1 -1 0 1 -1 0 0 1 0]\n'
                 'AttributeEnd\nWorldEnd\n')
    hs = ptgpu.HostScene(str(p))
    mats, lights = ptgpu.spectral_tables(hs)
    assert np.array_equal(lights[0].view(np.uint32), from_rgb60([3, 2, 1]).view(np.uint32))
    assert np.array_equal(mats[0][0].view(np.uint32), from_rgb60([0.2, 0.5, 0.3]).view(np.uint32))


def spectral_furnace(tmp_path, integrator, res=8, spp=64, maxdepth=8):
    from conftest import assert_counters, furnace_scene
    txt = open(furnace_scene(tmp_path, res=res, spp=spp, maxdepth=maxdepth)).read()
    txt = txt.replace('Integrator "path" "integer maxdepth" [%d]' % maxdepth,
                      'Integrator "%s" "integer maxdepth" [%d]' % (integrator, maxdepth))
    txt = txt.replace('"rgb L" [0.5 0.5 0.5]', '"spectrum L" [400 0.5 700 0.5]')
    txt = txt.replace('"rgb Kd" [0.5 0.5 0.5]', '"spectrum Kd" [400 0.5 700 0.5]')
    p = tmp_path / f"sfurnace_{integrator}.pbrt"
    p.write_text(txt)
    return str(p)


def _flat_rgb():
    """sRGB of the flat SPD 1.0 through the 60-bin ToXYZ (spectrum.h:395-406)."""
    X, Y, Z = (from_sampled60(T["CIE_lambda"], T[k]).astype(np.float64) for k in ("CIE_X", "CIE_Y", "CIE_Z"))
    xyz = np.array([X.sum(), Y.sum(), Z.sum()]) * 300 / (106.856895 * 60)
    M = np.array([[3.240479, -1.537150, -0.498535], [-0.969256, 1.875991, 0.041556],
                  [0.055648, -0.204043, 1.057311]])
    return M @ xyz


@pytest.mark.parametrize("integrator", ["hero_path", "hero_path_mis"])
def test_spectral_furnace_known_answer(tmp_path, integrator):
    """Closed furnace, Kd = Le = 0.5 (flat SPDs): radiance Le / (1 - Kd) = 1
    in every bin (src/tests/analytic_scenes.cpp:135-165, tolerance 0.02),
    truncated at maxdepth 8: sum_k 0.5^(k+1), k <= 8.  The twelve emitting
    triangles exercise hero_path_mis's SpatialLightDistribution."""
    hs = ptgpu.HostScene(spectral_furnace(tmp_path, integrator))
    it = ptgpu.integrator_desc(hs)
    if integrator == "hero_path_mis":
        assert it.light_strategy == 2 and ptgpu.scene_desc(hs).n_lights == 12
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    expect = _flat_rgb() * sum(0.5 ** (k + 1) for k in range(9))
    assert np.allclose(img.reshape(-1, 3).mean(0), expect, rtol=0.02), (img.reshape(-1, 3).mean(0), expect)


def _c3_variant(tmp_path, integrator, res=40, spp=8, smooth=False, no_infinite=False):
    """smooth: the microfacet glass block made specular; no_infinite: the
    environment light dropped -- the hero kernel then runs its
    specular(+infinite) feature instantiation instead of the full one."""
    txt = open(os.path.join(SCENES, "cornell_dielectric.pbrt")).read()
    if smooth:
        txt = re.sub(r'"float [uv]roughness" \[ *[0-9.]+ *\]', "", txt)
    if no_infinite:
        txt = re.sub(r'LightSource "infinite"[^\n]*\n(\s*"spectrum [^\n]*\n)*', "", txt)
    txt = txt.replace('Integrator "path" "integer maxdepth" [5]', 'Integrator "%s"' % integrator)
    txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [%d]' % res, txt)
    txt = re.sub(r'"integer yresolution" \[\d+\]', '"integer yresolution" [%d]' % res, txt)
    txt = re.sub(r'"integer pixelsamples" \[\d+\]', '"integer pixelsamples" [%d]' % spp, txt)
    p = tmp_path / f"c3_{integrator}_{int(smooth)}{int(no_infinite)}.pbrt"
    p.write_text(txt)
    return str(p)


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["hero_path", "hero_path_mis"])
def test_hero_cornell_dielectric_matches_oracle(tmp_path, integrator):
    """Config 3 as written (hero_path_mis; also hero_path) on the device
    megakernel == the oracle, bit for bit, with identical ray / node /
    primitive counts."""
    hs = ptgpu.HostScene(_c3_variant(tmp_path, integrator))
    sc = ptgpu.Scene(hs)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    print(f"{integrator}: mean={ref.mean():.5g} max|d|={np.abs(got - ref).max():.3g}")
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["hero_path", "hero_path_mis"])
@pytest.mark.parametrize("no_infinite", [False, True])
def test_hero_cornell_dielectric_smooth_matches_oracle(tmp_path, integrator, no_infinite):
    """Both glass blocks specular (and optionally no environment light): the
    scene needs no microfacet lobes, so the device runs the smaller feature
    instantiations of the hero kernel (render.hip hero_kernel).  Bit-exact."""
    hs = ptgpu.HostScene(_c3_variant(tmp_path, integrator, smooth=True, no_infinite=no_infinite))
    MATTE, DISPERSIVE = 1, 4  # include/pt.h PT_MAT_*
    assert all(m.kind in (MATTE, DISPERSIVE) and (m.kind != DISPERSIVE or m.specular) for m in hs.materials())
    sc = ptgpu.Scene(hs)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("camera_rays", "closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.gpu
def test_hero_film_crop_and_batches_match_oracle(tmp_path):
    """The 60-bin film (k_film_s60) under a crop window, an odd-sized film and
    batches of a few FilmTiles (pixels on batch borders gather from several
    launches) == the oracle, bit for bit."""
    txt = open(_c3_variant(tmp_path, "hero_path_mis", res=40, spp=4)).read()
    txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [53]', txt)
    txt = txt.replace('Film "image"', 'Film "image" "float cropwindow" [0.13 0.91 0.08 0.77]')
    p = tmp_path / "c3_crop.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    ref, _ = pyoracle.render(hs.desc, nthreads=8)
    got, _ = ptgpu.Scene(hs, batch_slots=16 * 16 * 4 * 3).render()  # 3 FilmTiles per batch
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["hero_path", "hero_path_mis"])
def test_hero_furnace_matches_oracle(tmp_path, integrator):
    hs = ptgpu.HostScene(spectral_furnace(tmp_path, integrator, res=8, spp=16))
    sc = ptgpu.Scene(hs)
    ref, rst = pyoracle.render(hs.desc, nthreads=8)
    got, gst = sc.render()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert_counters(gst, rst, ("closest_rays", "shadow_rays", "node_visits", "prim_tests"))


@pytest.mark.gpu
@pytest.mark.parametrize("filt,spp", [("gaussian2", 136), ("box", 70), ("gaussian3", 20), ("gaussian6", 6)])
def test_hero_film_staged_matches_oracle(tmp_path, filt, spp):
    """The 60-bin film under a crop window and batches of two FilmTiles, with
    the box filter's 1-pixel window and Gaussian windows of 3, 4 and 7 pixels
    == the oracle, bit for bit; and the opt-in LDS-staged k_film_s60_blk
    (PT_FILM_BLK=1: several 128-sample chunks per source pixel at 136 spp, a
    partial chunk at 70 spp; a window above kF60MaxWin, gaussian radius 6,
    falls back to k_film_s60) give the identical film; the default film is
    k_film_s60_sq (2 x 2 squares, cut by the batch box and the crop window,
    windows reaching two or four FilmTiles) and PT_FILM_SQ=0 the per-pixel
    k_film_s60, bit-identical."""
    txt = open(_c3_variant(tmp_path, "hero_path_mis", res=24, spp=spp)).read()
    txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [37]', txt)
    txt = txt.replace('Film "image"', 'Film "image" "float cropwindow" [0.05 0.93 0.1 0.85]')
    if filt == "box":
        txt = re.sub(r'PixelFilter "gaussian"\s*"float xwidth" \[2\]\s*"float ywidth" \[2\]', 'PixelFilter "box"', txt)
    else:
        r = filt[len("gaussian"):]
        txt = re.sub(r'"float ([xy])width" \[2\]', r'"float \1width" [%s]' % r, txt)
    p = tmp_path / f"c3_film_{filt}.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    ref, _ = pyoracle.render(hs.desc, nthreads=8)
    slots = 16 * 16 * spp * 2  # two FilmTiles per batch
    got, _ = ptgpu.Scene(hs, batch_slots=slots).render()
    assert ref.mean() > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    os.environ["PT_FILM_BLK"] = "1"
    try:
        staged, _ = ptgpu.Scene(hs, batch_slots=slots).render()
    finally:
        del os.environ["PT_FILM_BLK"]
    assert np.array_equal(staged.view(np.uint32), got.view(np.uint32))
    # the default k_film_s60_sq (one wave per 2 x 2 film pixels walking the union of their windows) against the
    # per-pixel k_film_s60 (PT_FILM_SQ=0)
    os.environ["PT_FILM_SQ"] = "0"
    try:
        per_pixel, _ = ptgpu.Scene(hs, batch_slots=slots).render()
    finally:
        del os.environ["PT_FILM_SQ"]
    assert np.array_equal(per_pixel.view(np.uint32), got.view(np.uint32))
