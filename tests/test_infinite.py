"""InfiniteAreaLight (lights/infinite.cpp) with a constant map -- SURVEY.md
§8(a) row a21 -- on the oracle: escaped rays see Le, and a Lambertian plane
under a constant sky reflects Kd * L (energy of the MIS estimator with the
light's Distribution2D sampling and Pdf_Li)."""
import numpy as np
import pytest

import ptgpu
import pyoracle

SKY = '''LookAt 0 10 0  0 0 0  0 0 1
Camera "perspective" "float fov" [40]
Film "image" "integer xresolution" [{w}] "integer yresolution" [{h}]
Sampler "halton" "integer pixelsamples" [{spp}]
Integrator "path" "integer maxdepth" [{depth}] {istrat}
WorldBegin
AttributeBegin
  Rotate {rot} 1 0 0
  LightSource "infinite" "rgb L" [{L}]
AttributeEnd
{extra}
WorldEnd
'''

PLANE = '''AttributeBegin
  Material "matte" "rgb Kd" [0.5 0.5 0.5]
  Shape "trianglemesh" "point P" [-1000 0 -1000  1000 0 -1000  1000 0 1000  -1000 0 1000]
        "integer indices" [0 1 2 0 2 3]
AttributeEnd
'''
FAR = '''Shape "trianglemesh" "point P" [500 500 500  501 500 500  500 501 500] "integer indices" [0 1 2]
'''


def sky_scene(tmp_path, w=16, h=16, spp=64, depth=5, rot=30, L="1 1 1", extra=PLANE, istrat="", name="sky"):
    p = tmp_path / f"{name}.pbrt"
    p.write_text(SKY.format(w=w, h=h, spp=spp, depth=depth, rot=rot, L=L, extra=extra, istrat=istrat))
    return str(p)


def test_escaped_rays_see_L(tmp_path):
    hs = ptgpu.HostScene(sky_scene(tmp_path, extra=FAR, L="0.25 0.5 2", spp=4))
    img, st = pyoracle.render(hs.desc, nthreads=4)
    # Le = MIPMap::triangle of the constant texel: equal to L up to the
    # rounding of its four bilinear terms
    # (and of the film's RGB -> XYZ -> RGB round trip, ~1e-5)
    np.testing.assert_allclose(img.reshape(-1, 3).mean(0), [0.25, 0.5, 2.0], rtol=1e-4)
    assert st["closest_rays"] == st["camera_rays"]


@pytest.mark.parametrize("strategy", ['', '"string lightsamplestrategy" "power"'])
def test_plane_under_constant_sky(tmp_path, strategy):
    hs = ptgpu.HostScene(sky_scene(tmp_path, spp=256, istrat=strategy, extra=PLANE + FAR))
    img, _ = pyoracle.render(hs.desc, nthreads=8)
    assert abs(float(img.mean()) - 0.5) < 0.01


def test_infinite_light_params(tmp_path):
    p = tmp_path / "bad.pbrt"
    p.write_text(SKY.format(w=4, h=4, spp=1, depth=1, rot=0, L="1 1 1", extra="", istrat="").replace(
        '"rgb L" [1 1 1]', '"rgb L" [1 1 1] "string mapname" "sky.exr"'))
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.HostScene(str(p))
    assert e.value.status == 3
