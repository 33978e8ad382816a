"""pyoracle -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/libptoracle.so, the plain-C restatement of the
reference hot path (see oracle/pt_oracle.h).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product never does.
It consumes the same pt_scene_desc pointer the product's loader produces.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libptoracle.so")


class oracle_stats(ctypes.Structure):
    _fields_ = [("camera_rays", ctypes.c_uint64), ("closest_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("node_visits", ctypes.c_uint64),
                ("prim_tests", ctypes.c_uint64), ("samples", ctypes.c_uint64),
                ("closest_node_visits", ctypes.c_uint64), ("closest_prim_tests", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.oracle_render.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(oracle_stats)]
        L.oracle_render_accum.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(oracle_stats)]
        L.oracle_render_range.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(oracle_stats)]
        L.oracle_bsdf_batch.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp]
        L.oracle_set_trig.argtypes = [ctypes.c_int]
        L.oracle_set_trig.restype = None
        L.oracle_film_size.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_build_bvh.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), vp, vp, ctypes.c_int32]
        L.oracle_radical_inverse.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.oracle_radical_inverse.restype = ctypes.c_float
        L.oracle_scrambled_radical_inverse.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.oracle_scrambled_radical_inverse.restype = ctypes.c_float
        L.oracle_scrambled_radical_inverse_perm.argtypes = [ctypes.c_int, ctypes.c_uint64, vp]
        L.oracle_scrambled_radical_inverse_perm.restype = ctypes.c_float
        L.oracle_prime.argtypes = [ctypes.c_int]
        L.oracle_halton_perm.argtypes = [ctypes.c_int64]
        L.oracle_halton_sample.argtypes = [ctypes.c_int] * 6 + [ctypes.c_int64, ctypes.c_int]
        L.oracle_halton_sample.restype = ctypes.c_float
        L.oracle_halton_index.argtypes = [ctypes.c_int] * 6 + [ctypes.c_int64]
        L.oracle_halton_index.restype = ctypes.c_int64
        L.oracle_ray_triangle.argtypes = [vp, vp, ctypes.c_float, vp, vp, vp, vp, vp]
        L.oracle_camera_ray.argtypes = [vp, ctypes.c_float, ctypes.c_float, vp, vp]
        L.oracle_trace.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp]
        L.oracle_trace_counted.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, vp]
        L.oracle_test_reintersect.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.POINTER(ctypes.c_int)]
        L.oracle_test_triangle_sampling.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.POINTER(ctypes.c_double), vp, vp,
                                                    ctypes.POINTER(ctypes.c_int)]
        L.oracle_test_sphere.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
                                         ctypes.POINTER(ctypes.c_int), vp]
        L.oracle_triangle_intersect.argtypes = [vp, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.oracle_dist1d.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_float, vp]
        _lib = L
    return _lib


def set_trig(correctly_rounded: bool) -> None:
    """False: libm cosf/sinf (reference binary); True: correctly rounded (device)."""
    lib().oracle_set_trig(1 if correctly_rounded else 0)


def film_size(desc: int) -> Tuple[int, int]:
    w, h = ctypes.c_int(), ctypes.c_int()
    lib().oracle_film_size(ctypes.c_void_p(desc), ctypes.byref(w), ctypes.byref(h))
    return w.value, h.value


def _chk(rc: int) -> None:
    if rc == 3:
        raise RuntimeError("oracle: Halton dimension past the prime table (the reference CHECK-fails)")
    if rc == 4:
        raise RuntimeError("oracle: unsupported input (more than PT_MAX_PORTALS portals on one light)")
    if rc != 0:
        raise RuntimeError(f"oracle: error {rc}")


def render(desc: int, nthreads: int = 1, max_tiles: int = -1) -> Tuple[np.ndarray, dict]:
    w, h = film_size(desc)
    rgb = np.zeros((h, w, 3), np.float32)
    st = oracle_stats()
    _chk(lib().oracle_render(ctypes.c_void_p(desc), rgb.ctypes.data, nthreads, max_tiles, ctypes.byref(st)))
    return rgb, st.as_dict()


def render_accum(desc: int, nthreads: int = 1, tile_offset: int = 0, tile_stride: int = 1) -> Tuple[np.ndarray, dict]:
    w, h = film_size(desc)
    acc = np.zeros((h, w, 4), np.float32)
    st = oracle_stats()
    _chk(lib().oracle_render_accum(ctypes.c_void_p(desc), acc.ctypes.data, nthreads, tile_offset, tile_stride,
                                   ctypes.byref(st)))
    return acc, st.as_dict()


def render_range(desc: int, s_begin: int, s_end: int, nthreads: int = 1, tile_offset: int = 0,
                 tile_stride: int = 1) -> Tuple[np.ndarray, dict]:
    w, h = film_size(desc)
    acc = np.zeros((h, w, 4), np.float32)
    st = oracle_stats()
    _chk(lib().oracle_render_range(ctypes.c_void_p(desc), acc.ctypes.data, nthreads, tile_offset, tile_stride,
                                   s_begin, s_end, ctypes.byref(st)))
    return acc, st.as_dict()


def bsdf_batch(desc: int, mat: int, rec8: np.ndarray) -> np.ndarray:
    """BSDF::f / Pdf / Sample_f of material `mat` in the local frame n = (0,0,1):
    (n, 8) records wo, wi, u0, u1 -> (n, 8) f, pdf, sampled wi, sampled pdf."""
    rec8 = np.ascontiguousarray(rec8, np.float32)
    out = np.zeros_like(rec8)
    assert lib().oracle_bsdf_batch(ctypes.c_void_p(desc), mat, len(rec8), rec8.ctypes.data, out.ctypes.data) == 0
    return out


def build_bvh(desc: int) -> Tuple[np.ndarray, np.ndarray]:
    n = ctypes.c_int32()
    lib().oracle_build_bvh(ctypes.c_void_p(desc), ctypes.byref(n), None, None, 0)
    nodes = np.zeros((n.value, 8), np.uint32)
    order = np.zeros(max(1, 2 * n.value), np.int32)
    lib().oracle_build_bvh(ctypes.c_void_p(desc), ctypes.byref(n), nodes.ctypes.data, order.ctypes.data,
                           int(2 * n.value))
    return nodes, order


def trace(desc: int, rays7: np.ndarray, any_hit: bool) -> np.ndarray:
    rays7 = np.ascontiguousarray(rays7, np.float32)
    out = np.zeros(len(rays7), np.int32)
    lib().oracle_trace(ctypes.c_void_p(desc), len(rays7), rays7.ctypes.data, int(any_hit), out.ctypes.data)
    return out


def trace_counted(desc: int, rays7: np.ndarray, any_hit: bool) -> Tuple[np.ndarray, int, int]:
    """trace() plus the reference's BVH node-visit and primitive-test counts over the queries."""
    rays7 = np.ascontiguousarray(rays7, np.float32)
    out = np.zeros(len(rays7), np.int32)
    counts = np.zeros(2, np.uint64)
    _chk(lib().oracle_trace_counted(ctypes.c_void_p(desc), len(rays7), rays7.ctypes.data, int(any_hit),
                                    out.ctypes.data, counts.ctypes.data))
    return out, int(counts[0]), int(counts[1])


def camera_ray(desc: int, fx: float, fy: float) -> Tuple[np.ndarray, np.ndarray]:
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    lib().oracle_camera_ray(ctypes.c_void_p(desc), fx, fy, o.ctypes.data, d.ctypes.data)
    return o, d


def radical_inverse(base_index: int, a: int) -> float:
    return lib().oracle_radical_inverse(base_index, a)


def scrambled_radical_inverse(base_index: int, a: int, perm: np.ndarray = None) -> float:
    if perm is None:
        return lib().oracle_scrambled_radical_inverse(base_index, a)
    perm = np.ascontiguousarray(perm, np.uint16)
    return lib().oracle_scrambled_radical_inverse_perm(base_index, a, perm.ctypes.data)


def prime(i: int) -> int:
    return lib().oracle_prime(i)


def halton_sample(sb: Tuple[int, int, int, int], px: int, py: int, sample: int, dim: int) -> float:
    return lib().oracle_halton_sample(sb[0], sb[1], sb[2], sb[3], px, py, sample, dim)


def halton_index(sb: Tuple[int, int, int, int], px: int, py: int, sample: int) -> int:
    return lib().oracle_halton_index(sb[0], sb[1], sb[2], sb[3], px, py, sample)


def ray_triangle(o, d, tmax, p0, p1, p2):
    arrs = [np.ascontiguousarray(x, np.float32) for x in (o, d, p0, p1, p2)]
    t = np.zeros(1, np.float32)
    b = np.zeros(3, np.float32)
    hit = lib().oracle_ray_triangle(arrs[0].ctypes.data, arrs[1].ctypes.data, float(tmax), arrs[2].ctypes.data,
                                    arrs[3].ctypes.data, arrs[4].ctypes.data, t.ctypes.data, b.ctypes.data)
    return bool(hit), float(t[0])


# ---- the reference's unit tests for this path, restated in the oracle ----

def reintersect_case(i: int, n_dirs: int):
    """Triangle.Reintersect (src/tests/shapes.cpp:155-206) for RNG seed i:
    (triangle (3,3), spawned rays (2*n_dirs, 7), self-hit count) or None
    when the reference skips the seed."""
    tri = np.zeros(9, np.float32)
    rays = np.zeros((2 * n_dirs, 7), np.float32)
    bad = ctypes.c_int()
    ok = lib().oracle_test_reintersect(i, n_dirs, tri.ctypes.data, rays.ctypes.data, ctypes.byref(bad))
    return (tri.reshape(3, 3), rays, bad.value) if ok else None


def triangle_sampling_case(i: int, count: int = 512 * 1024):
    """Triangle.Sampling (src/tests/shapes.cpp:211-270) for RNG seed i:
    (uniform-sphere estimate, Triangle::Sample estimate, triangle, pc,
    non-positive pdf count) or None when skipped."""
    a, b = ctypes.c_double(), ctypes.c_double()
    tri = np.zeros(9, np.float32)
    pc = np.zeros(3, np.float32)
    bad = ctypes.c_int()
    ok = lib().oracle_test_triangle_sampling(i, count, ctypes.byref(a), ctypes.byref(b), tri.ctypes.data,
                                             pc.ctypes.data, ctypes.byref(bad))
    return (a.value, b.value, tri.reshape(3, 3), pc, bad.value) if ok else None


def sphere_case(i: int, partial: bool, mode: str, n_dirs: int = 10000):
    """The Sphere cases of src/tests/shapes.cpp (FullSphere.Reintersect,
    PartialSphere.Normal / Reintersect) for RNG seed i, or None when the
    reference skips the seed (its first ray misses).  mode 'reintersect' ->
    (params (radius, zmin, zmax, phimax), spawned rays (2*n_dirs, 7),
    self-hit count); mode 'normal' -> (params, dot(n, p) normalised)."""
    params = np.zeros(4, np.float32)
    out = np.zeros(1, np.float32)
    bad = ctypes.c_int()
    if mode == "reintersect":
        rays = np.zeros((2 * n_dirs, 7), np.float32)
        ok = lib().oracle_test_sphere(i, int(partial), 0, n_dirs, params.ctypes.data, rays.ctypes.data,
                                      ctypes.byref(bad), out.ctypes.data)
        return (params, rays, bad.value) if ok else None
    ok = lib().oracle_test_sphere(i, int(partial), 1, 0, params.ctypes.data, None, ctypes.byref(bad),
                                  out.ctypes.data)
    return (params, float(out[0])) if ok else None


def triangle_intersect(tri9, ray7, any_hit: bool = False):
    """Triangle::Intersect (any_hit False) / IntersectP of one triangle: (hit, t)."""
    tri9 = np.ascontiguousarray(tri9, np.float32).reshape(9)
    ray7 = np.ascontiguousarray(ray7, np.float32).reshape(7)
    t = ctypes.c_float()
    hit = lib().oracle_triangle_intersect(tri9.ctypes.data, ray7.ctypes.data, int(any_hit), ctypes.byref(t))
    return bool(hit), t.value


def dist1d(func, mode: str, u: float):
    """Distribution1D (sampling.h:55-110): mode 'discrete' -> (offset, pdf,
    uRemapped); 'continuous' -> (x, pdf, offset); 'pdf' -> DiscretePDF(int(u))."""
    f = np.ascontiguousarray(func, np.float32)
    out = np.zeros(3, np.float32)
    m = {"discrete": 0, "continuous": 1, "pdf": 2}[mode]
    assert lib().oracle_dist1d(f.ctypes.data, len(f), m, float(u), out.ctypes.data) == 0
    if mode == "discrete":
        return int(out[0]), float(out[1]), float(out[2])
    if mode == "continuous":
        return float(out[0]), float(out[1]), int(out[2])
    return float(out[0])
