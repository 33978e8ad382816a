"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu and call the
product only through the C ABI (libptgpu.so via ptgpu); the oracle
(oracle/libptoracle.so via pyoracle) is the checker."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pbrt-v3-light-portals_amd")
ORACLE = os.path.join(REPO, "oracle")
SCENES = os.path.join(REPO, "scenes")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _ensure_built():
    if not os.path.exists(os.path.join(ORACLE, "libptoracle.so")):
        subprocess.check_call(["make", "-s", "-C", ORACLE])
    if not os.path.exists(os.path.join(PKG, "libptgpu.so")):
        subprocess.check_call(["make", "-s", "-C", PKG, "-j8"])


_ensure_built()


def scene_variant(tmp_path, name="portal_cornell.pbrt", res=None, spp=None, strategy=None, maxdepth=None,
                  extra=None):
    """Write a variant of a committed scene (smaller film / spp / strategy)."""
    txt = open(os.path.join(SCENES, name)).read()
    if res is not None:
        import re
        txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [%d]' % res[0], txt)
        txt = re.sub(r'"integer yresolution" \[\d+\]', '"integer yresolution" [%d]' % res[1], txt)
    if spp is not None:
        import re
        txt = re.sub(r'"integer pixelsamples" \[\d+\]', '"integer pixelsamples" [%d]' % spp, txt)
    if strategy is not None:
        import re
        txt = re.sub(r'"string strategy" "\w+"', '"string strategy" "%s"' % strategy, txt)
    if maxdepth is not None:
        import re
        txt = re.sub(r'"integer maxdepth" \[\d+\]', '"integer maxdepth" [%d]' % maxdepth, txt)
    import re
    # the variant lives elsewhere: keep the scene's own relative PLY files and
    # Includes resolving against its directory under scenes/ (files named by
    # `extra` stay relative to the variant)
    sdir = os.path.dirname(os.path.join(SCENES, name))
    txt = re.sub(r'"string filename" \["(?!/)([^"]+\.ply)"\]',
                 lambda m: '"string filename" ["%s/%s"]' % (sdir, m.group(1)), txt)
    if extra:
        for a, b in extra:
            txt = txt.replace(a, b)
    txt = re.sub(r'Include "(?!/)([^"]+)"', lambda m: 'Include "%s/%s"' % (sdir, m.group(1)), txt)
    p = os.path.join(str(tmp_path), "v_%s_%s_%s_%s_%s" % (res, spp, strategy, maxdepth, name.replace("/", "_")))
    p = p.replace(" ", "").replace("(", "").replace(")", "").replace(",", "x")
    with open(p, "w") as f:
        f.write(txt)
    return p


@pytest.fixture
def variant(tmp_path):
    def make(**kw):
        return scene_variant(tmp_path, **kw)
    return make


def furnace_scene(tmp_path, res=10, spp=256, maxdepth=8):
    """Closed-box furnace: every face Kd = 0.5 and emitting Le = 0.5, camera
    inside.  Restates the reference's analytic test 'Sphere, Kd = 0.5,
    Le = 0.5' (src/tests/analytic_scenes.cpp:135-165, expected radiance 1.0,
    tolerance 0.02, CheckSceneAverage :54-66) with a triangulated cube: the
    answer Le/(1-Kd) does not depend on the enclosure's shape."""
    faces = [
        ([-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1]),
        ([-1, -1, 1], [-1, 1, 1], [1, 1, 1], [1, -1, 1]),
        ([-1, -1, -1], [-1, 1, -1], [-1, 1, 1], [-1, -1, 1]),
        ([1, -1, -1], [1, -1, 1], [1, 1, 1], [1, 1, -1]),
        ([-1, -1, -1], [-1, -1, 1], [1, -1, 1], [1, -1, -1]),
        ([-1, 1, -1], [1, 1, -1], [1, 1, 1], [-1, 1, 1]),
    ]
    pts = " ".join(" ".join(str(c) for c in v) for f in faces for v in f)
    idx = " ".join("%d %d %d %d %d %d" % (4 * i, 4 * i + 1, 4 * i + 2, 4 * i, 4 * i + 2, 4 * i + 3) for i in range(6))
    txt = f"""LookAt 0 0 0  0 0 1  0 1 0
Camera "perspective" "float fov" [45]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [{res}] "integer yresolution" [{res}]
Sampler "halton" "integer pixelsamples" [{spp}]
Integrator "path" "integer maxdepth" [{maxdepth}]
WorldBegin
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [0.5 0.5 0.5] "bool twosided" "true"
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  Shape "trianglemesh" "integer indices" [{idx}] "point P" [{pts}]
AttributeEnd
WorldEnd
"""
    p = os.path.join(str(tmp_path), "furnace_%d_%d.pbrt" % (res, spp))
    with open(p, "w") as f:
        f.write(txt)
    return p


# The reference's node-visit / primitive-test counters depend on its visit order.  The 4-wide traversal
# (k_trace_w, the default for LDS-resident scenes without spheres) returns the reference's hits in another
# order: its renders report trace_wide = 1, and node_visits / prim_tests then count only the rays it handed
# back to the binary traversal.  Renders with set_count_bytes(True) traverse in the reference's order
# throughout and report the reference's counters (test_gpu_parity.py::test_counting_frame_*).
ORDER_COUNTERS = ("node_visits", "prim_tests")


def assert_counters(gst, rst, keys):
    """GPU render counters against the oracle's: rays and samples always, the
    order-dependent node / primitive counters when the render traversed in the
    reference's order."""
    for k in keys:
        if k in ORDER_COUNTERS and gst.get("trace_wide"):
            continue
        assert gst[k] == rst[k], (k, gst[k], rst[k])
    if gst.get("trace_wide"):
        assert gst["retraced_rays"] <= gst["closest_rays"] + gst["shadow_rays"]
