"""ptgpu -- Python binding of the C ABI in include/pt.h (ctypes).

The product is the C-ABI library ``libptgpu.so`` (HIP kernels for gfx950 +
C++ host loader/BVH builder).  This module is plumbing for tests, bench.py and
__graft_entry__: it never computes anything itself and raises if the library
or a HIP device is missing -- there is no CPU fallback.

Reference interface mirrored: ``Scene`` ~ pbrt's Scene +
``SamplerIntegrator::Render`` for a ``PathIntegrator`` (src/core/integrator.cpp:
526-637, src/integrators/path.cpp:64-214).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PT_LIB selects a diagnostic build of the same library (e.g. libptgpu_guard.so)
LIB_PATH = os.path.join(HERE, os.environ.get("PT_LIB", "libptgpu.so"))

PT_OK = 0
STATUS_NAMES = {0: "PT_OK", 1: "PT_ERR_INVALID_ARG", 2: "PT_ERR_PARSE", 3: "PT_ERR_UNSUPPORTED",
                4: "PT_ERR_DEVICE", 5: "PT_ERR_OOM", 6: "PT_ERR_STATE", 7: "PT_ERR_IO"}


class PtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class pt_stats(ctypes.Structure):
    _fields_ = [("camera_rays", ctypes.c_uint64), ("closest_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("node_visits", ctypes.c_uint64),
                ("prim_tests", ctypes.c_uint64), ("samples", ctypes.c_uint64),
                ("render_ms", ctypes.c_double), ("trace_ms", ctypes.c_double),
                ("trace_launches", ctypes.c_uint64), ("shade_ms", ctypes.c_double),
                ("shade_launches", ctypes.c_uint64), ("shade_bytes", ctypes.c_uint64),
                ("reduce_ms", ctypes.c_double), ("retraced_rays", ctypes.c_uint64),
                ("wide_node_visits", ctypes.c_uint64), ("wide_prim_tests", ctypes.c_uint64),
                ("trace_wide", ctypes.c_int32), ("reserved", ctypes.c_int32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def lib() -> ctypes.CDLL:
    """Load libptgpu.so (built in-tree by ``make -C pbrt-v3-light-portals_amd``)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PtError(7, f"{LIB_PATH} is missing: build it with `make -C {HERE}` (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, f32p = ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_float)
    L.pt_last_error.restype = ctypes.c_char_p
    L.pt_abi_version.restype = ctypes.c_int
    L.pt_load_pbrt.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    L.pt_host_scene_desc.argtypes = [vp]
    L.pt_host_scene_desc.restype = vp
    L.pt_host_scene_free.argtypes = [vp]
    L.pt_host_scene_free.restype = None
    L.pt_init.argtypes = [ctypes.c_int, ctypes.POINTER(i32)]
    L.pt_shutdown.argtypes = []
    L.pt_comm_unique_id.argtypes = [vp]
    L.pt_comm_create.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.pt_comm_destroy.argtypes = [vp]
    L.pt_comm_destroy.restype = None
    L.pt_film_reduce.argtypes = [vp, vp, vp, ctypes.c_int, vp]
    L.pt_render_frame_dist.argtypes = [vp, vp, vp, vp, ctypes.POINTER(pt_stats)]
    L.pt_scene_create.argtypes = [vp, ctypes.POINTER(vp)]
    L.pt_scene_destroy.argtypes = [vp]
    L.pt_scene_destroy.restype = None
    L.pt_scene_bvh.argtypes = [vp, ctypes.POINTER(i32), vp, ctypes.POINTER(i32), vp]
    L.pt_build_bvh_host.argtypes = [vp, ctypes.POINTER(i32), vp, i32, ctypes.POINTER(i32), vp, i32]
    L.pt_film_size.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.pt_render.argtypes = [vp, f32p, ctypes.POINTER(pt_stats)]
    L.pt_render_accum.argtypes = [vp, ctypes.c_int, ctypes.c_int, f32p, ctypes.POINTER(pt_stats)]
    L.pt_render_range_accum.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p,
                                        ctypes.POINTER(pt_stats)]
    L.pt_render_tiles.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.POINTER(pt_stats)]
    L.pt_render_range.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
                                  ctypes.POINTER(pt_stats)]
    L.pt_resolve_film.argtypes = [vp, f32p, f32p]
    L.pt_resolve_film_host.argtypes = [vp, f32p, f32p]
    L.pt_film_size_host.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.pt_set_batch_slots.argtypes = [vp, ctypes.c_int64]
    L.pt_set_pipelines.argtypes = [vp, ctypes.c_int32]
    L.pt_scene_query.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
    L.pt_write_pfm.argtypes = [ctypes.c_char_p, f32p, i32, i32]
    L.pt_write_image.argtypes = [ctypes.c_char_p, f32p, i32, i32, i32, i32, i32, i32]
    L.pt_write_film_image.argtypes = [vp, ctypes.c_char_p, f32p]
    L.pt_host_scene_film_filename.argtypes = [vp]
    L.pt_host_scene_film_filename.restype = ctypes.c_char_p
    L.pt_debug_libm_trig.argtypes = [ctypes.c_int, vp, vp, vp]
    L.pt_debug_spectrum.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
    L.pt_debug_halton.argtypes = [vp, ctypes.c_int, vp, vp, vp]
    L.pt_debug_pixel_offsets.argtypes = [vp, ctypes.c_int, vp, vp]
    L.pt_debug_camera_rays.argtypes = [vp, ctypes.c_int, vp, vp]
    L.pt_debug_trace.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp]
    L.pt_debug_trace_frame.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, vp]
    L.pt_debug_trace_frame_ex.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, ctypes.POINTER(pt_stats)]
    L.pt_debug_bsdf.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp]
    _lib = L
    return L


def spectrum_rgb(kind: int, vals, n_out: int = 3) -> np.ndarray:
    """Host spectral reduction of the loader (pt_debug_spectrum): kind 0
    (lambda, value) pairs -> RGB, 1 (T, scale) blackbody -> RGB, 2 xyz -> RGB,
    3 (lambda, T) pairs -> Planck radiance."""
    v = np.ascontiguousarray(vals, dtype=np.float32).ravel()
    n = len(v) // 2 if kind in (0, 3) else len(v)
    out = np.zeros(n if kind == 3 else n_out, dtype=np.float32)
    _check(lib().pt_debug_spectrum(kind, n, v.ctypes.data, out.ctypes.data))
    return out


def _check(status: int) -> None:
    if status != PT_OK:
        raise PtError(status, lib().pt_last_error().decode())


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class pt_material(ctypes.Structure):
    """include/pt.h pt_material"""
    _fields_ = [("kind", ctypes.c_int32), ("kd", ctypes.c_float * 3), ("sigma", ctypes.c_float),
                ("eta", ctypes.c_float * 3), ("k", ctypes.c_float * 3), ("alpha", ctypes.c_float * 2),
                ("ks", ctypes.c_float * 3), ("kr", ctypes.c_float * 3), ("kt", ctypes.c_float * 3),
                ("ior", ctypes.c_float), ("ior_min", ctypes.c_float), ("ior_max", ctypes.c_float),
                ("specular", ctypes.c_int32)]


class _desc_prefix(ctypes.Structure):
    """Leading fields of include/pt.h pt_scene_desc (through the materials)."""
    _fields_ = [("n_vertices", ctypes.c_int32), ("P", ctypes.c_void_p), ("N", ctypes.c_void_p),
                ("S", ctypes.c_void_p), ("UV", ctypes.c_void_p), ("n_triangles", ctypes.c_int32),
                ("triangles", ctypes.c_void_p), ("n_planes", ctypes.c_int32), ("planes", ctypes.c_void_p),
                ("n_prims", ctypes.c_int32), ("prims", ctypes.c_void_p), ("n_materials", ctypes.c_int32),
                ("materials", ctypes.POINTER(pt_material))]


class pt_transform(ctypes.Structure):
    _fields_ = [("m", ctypes.c_float * 16), ("minv", ctypes.c_float * 16)]


class pt_camera_desc(ctypes.Structure):
    _fields_ = [("camera_to_world", pt_transform), ("fov", ctypes.c_float), ("screen_window", ctypes.c_float * 4),
                ("lens_radius", ctypes.c_float), ("focal_distance", ctypes.c_float),
                ("shutter_open", ctypes.c_float), ("shutter_close", ctypes.c_float)]


class pt_film_desc(ctypes.Structure):
    _fields_ = [("xres", ctypes.c_int32), ("yres", ctypes.c_int32), ("crop", ctypes.c_float * 4),
                ("filter", ctypes.c_int32), ("filter_radius", ctypes.c_float * 2), ("gaussian_alpha", ctypes.c_float),
                ("scale", ctypes.c_float), ("max_sample_luminance", ctypes.c_float), ("diagonal", ctypes.c_float)]


class pt_sampler_desc(ctypes.Structure):
    _fields_ = [("spp", ctypes.c_int32), ("sample_pixel_center", ctypes.c_int32)]


class pt_integrator_desc(ctypes.Structure):
    _fields_ = [("max_depth", ctypes.c_int32), ("rr_threshold", ctypes.c_float), ("light_strategy", ctypes.c_int32),
                ("has_pixel_bounds", ctypes.c_int32), ("pixel_bounds", ctypes.c_int32 * 4), ("kind", ctypes.c_int32),
                ("direct_strategy", ctypes.c_int32)]


class pt_scene_desc(ctypes.Structure):
    """include/pt.h pt_scene_desc (read-only view of the loader's output)."""
    _fields_ = _desc_prefix._fields_ + [
        ("n_lights", ctypes.c_int32), ("lights", ctypes.c_void_p), ("n_portals", ctypes.c_int32),
        ("portals", ctypes.c_void_p), ("bvh_max_prims", ctypes.c_int32), ("camera", pt_camera_desc),
        ("film", pt_film_desc), ("sampler", pt_sampler_desc), ("integrator", pt_integrator_desc),
        ("n_spheres", ctypes.c_int32), ("spheres", ctypes.c_void_p), ("spectral", ctypes.c_int32),
        ("material_s60", ctypes.POINTER(ctypes.c_float)), ("light_s60", ctypes.POINTER(ctypes.c_float)),
        ("n_bvh_nodes", ctypes.c_int32), ("bvh_nodes", ctypes.c_void_p)]


def scene_desc(hs: "HostScene") -> pt_scene_desc:
    """The scene's pt_scene_desc (a view into the loader's memory) -- host only."""
    return ctypes.cast(ctypes.c_void_p(hs.desc), ctypes.POINTER(pt_scene_desc)).contents


def spectral_tables(hs: "HostScene"):
    """(material_s60 (n_materials, 3, 60), light_s60 (n_lights, 60)) of a
    SampledSpectrum scene, or None for an RGB scene."""
    d = scene_desc(hs)
    if not d.spectral:
        return None
    m = np.ctypeslib.as_array(d.material_s60, shape=(d.n_materials, 3, 60)).copy()
    lt = np.ctypeslib.as_array(d.light_s60, shape=(max(1, d.n_lights), 60)).copy()[:d.n_lights]
    return m, lt


def integrator_desc(hs: "HostScene") -> pt_integrator_desc:
    """A copy of the scene's pt_integrator_desc -- host only."""
    d = ctypes.cast(ctypes.c_void_p(hs.desc), ctypes.POINTER(pt_scene_desc)).contents
    return pt_integrator_desc.from_buffer_copy(d.integrator)


class HostScene:
    """pbrtParseFile + pbrtWorldEnd (src/core/parser.cpp:1094, api.cpp:1702):
    the flattened world-space scene (pt_scene_desc) -- host only."""

    def __init__(self, path: str):
        self._h = ctypes.c_void_p()
        _check(lib().pt_load_pbrt(os.fsencode(path), ctypes.byref(self._h)))
        self.path = path

    @property
    def desc(self) -> int:
        return lib().pt_host_scene_desc(self._h)

    def bvh(self) -> Tuple[np.ndarray, np.ndarray]:
        """Host SAH BVH (bvh.cpp): (n, 8) uint32 LinearBVHNode images, prim order."""
        n, m = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().pt_build_bvh_host(self.desc, ctypes.byref(n), None, 0, ctypes.byref(m), None, 0))
        nodes = np.zeros((n.value, 8), np.uint32)
        order = np.zeros(max(1, m.value), np.int32)
        _check(lib().pt_build_bvh_host(self.desc, ctypes.byref(n), nodes.ctypes.data, n.value, ctypes.byref(m),
                                       order.ctypes.data, m.value))
        return nodes, order[:m.value]

    def materials(self) -> list:
        """The scene's pt_material records (copies) -- host only."""
        d = ctypes.cast(ctypes.c_void_p(self.desc), ctypes.POINTER(_desc_prefix)).contents
        return [pt_material.from_buffer_copy(d.materials[i]) for i in range(d.n_materials)]

    def mesh(self) -> dict:
        """World-space vertex arrays and triangles of the flattened scene
        (copies): P, N (None without shading normals), tri (m, 6) int32 =
        v0 v1 v2 material area_light flags -- host only."""
        d = ctypes.cast(ctypes.c_void_p(self.desc), ctypes.POINTER(_desc_prefix)).contents
        nv, nt = d.n_vertices, d.n_triangles

        def arr(ptr, n, dt):
            if not ptr or n == 0:
                return None
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(dt)), shape=(n,)).copy()
        P = arr(d.P, 3 * nv, ctypes.c_float)
        N = arr(d.N, 3 * nv, ctypes.c_float)
        T = arr(d.triangles, 6 * nt, ctypes.c_int32)
        return {"P": None if P is None else P.reshape(nv, 3), "N": None if N is None else N.reshape(nv, 3),
                "tri": np.zeros((0, 6), np.int32) if T is None else T.reshape(nt, 6)}

    def film_size(self) -> Tuple[int, int]:
        """Cropped film (width, height) -- host only."""
        w, h = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().pt_film_size_host(self.desc, ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    def spp(self) -> int:
        """Sampler "pixelsamples" of the scene -- host only."""
        return ctypes.cast(ctypes.c_void_p(self.desc), ctypes.POINTER(pt_scene_desc)).contents.sampler.spp

    @property
    def film_filename(self) -> str:
        return lib().pt_host_scene_film_filename(self._h).decode()

    def write_image(self, rgb: np.ndarray, path: Optional[str] = None) -> str:
        """Film::WriteImage of a rendered (h, w, 3) image to `path` (default:
        the scene's Film "filename"); returns the path written."""
        rgb = np.ascontiguousarray(rgb, np.float32)
        path = path or self.film_filename
        _check(lib().pt_write_film_image(self.desc, os.fsencode(path), _fptr(rgb)))
        return path

    def resolve(self, accum: np.ndarray) -> np.ndarray:
        """Film::WriteImage of an (h, w, 4) XYZ+weight accumulation -- host only."""
        w, h = self.film_size()
        accum = np.ascontiguousarray(accum, np.float32)
        if accum.size != 4 * w * h:
            raise PtError(1, f"accumulation buffer has {accum.size} floats, film needs {4 * w * h}")
        rgb = np.zeros((h, w, 3), np.float32)
        _check(lib().pt_resolve_film_host(self.desc, _fptr(accum), _fptr(rgb)))
        return rgb

    def close(self) -> None:
        if self._h:
            lib().pt_host_scene_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Scene:
    """Device scene (pt_scene_create): BVH + SoA buffers resident in HBM."""

    def __init__(self, host: HostScene, device: int = 0, batch_slots: Optional[int] = None,
                 devices: Optional[list] = None):
        """device: the GPU of this process; devices: several GPUs of this
        process (pt_init(n, ids): one scene replica per device, pt_render deals
        the tiles over them)."""
        self.host = host
        ids = list(devices) if devices else [device]
        arr = (ctypes.c_int32 * len(ids))(*ids)
        _check(lib().pt_init(len(ids), arr))
        self._s = ctypes.c_void_p()
        _check(lib().pt_scene_create(host.desc, ctypes.byref(self._s)))
        if batch_slots:
            _check(lib().pt_set_batch_slots(self._s, int(batch_slots)))

    def set_count_bytes(self, on: bool) -> None:
        """pt_set_count_bytes: stats['shade_bytes'] counted in the renders that follow."""
        _check(lib().pt_set_count_bytes(self._s, int(bool(on))))

    def set_pipelines(self, n: int) -> None:
        """pt_set_pipelines: batches in flight (1 = one after the other)."""
        _check(lib().pt_set_pipelines(self._s, int(n)))

    QUERY_KEYS = {"pipelines": 0, "batch_slots": 1, "trace_lds_bytes": 2, "trace_spill": 3, "features": 4,
                  "trace_kernel": 5, "shade_kernel": 6}
    TRACE_KERNELS = {0: "k_trace", 1: "k_trace_pt", 2: "k_trace_nb", 3: "k_trace_lds", 5: "k_trace_oct", 6: "k_trace_w",
                     7: "k_trace_w"}  # 7: k_trace_w<true>, the wide image and primitives from HBM
    SHADE_KERNELS = {0: "k_shade", 3: "k_shade_w3", 4: "k_shade_w3h", 5: "k_shade_tab", 6: "k_shade_dl", 7: "k_shade_hero",
                     8: "k_shade_hero_w2", 9: "k_shade_hero_w4"}

    def kernel_names(self) -> Tuple[str, str]:
        """(traversal kernel, shading kernel) a render of this scene launches."""
        return self.TRACE_KERNELS[self.query("trace_kernel")], self.SHADE_KERNELS[self.query("shade_kernel")]

    def query(self, key: str) -> int:
        """pt_scene_query: a setting in effect (pipelines, batch_slots,
        trace_lds_bytes, trace_spill, features, trace_kernel, shade_kernel)."""
        v = ctypes.c_int64()
        _check(lib().pt_scene_query(self._s, self.QUERY_KEYS[key], ctypes.byref(v)))
        return v.value

    @property
    def handle(self) -> int:
        return self._s.value

    def film_size(self) -> Tuple[int, int]:
        w, h = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().pt_film_size(self._s, ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    def render(self) -> Tuple[np.ndarray, dict]:
        """Integrator::Render for the whole frame; returns (H, W, 3) RGB."""
        w, h = self.film_size()
        rgb = np.zeros((h, w, 3), np.float32)
        st = pt_stats()
        _check(lib().pt_render(self._s, _fptr(rgb), ctypes.byref(st)))
        return rgb, st.as_dict()

    def render_accum(self, tile_offset: int = 0, tile_stride: int = 1) -> Tuple[np.ndarray, dict]:
        w, h = self.film_size()
        acc = np.zeros((h, w, 4), np.float32)
        st = pt_stats()
        _check(lib().pt_render_accum(self._s, tile_offset, tile_stride, _fptr(acc), ctypes.byref(st)))
        return acc, st.as_dict()

    def render_range(self, sample_begin: int, sample_end: int, tile_offset: int = 0,
                     tile_stride: int = 1) -> Tuple[np.ndarray, dict]:
        """Film (h, w, 4) for camera-sample indices [sample_begin, sample_end)."""
        w, h = self.film_size()
        acc = np.zeros((h, w, 4), np.float32)
        st = pt_stats()
        _check(lib().pt_render_range_accum(self._s, tile_offset, tile_stride, sample_begin, sample_end, _fptr(acc),
                                           ctypes.byref(st)))
        return acc, st.as_dict()

    def render_tiles_device(self, tile_offset: int, tile_stride: int, d_accum: int, stream: int = 0) -> dict:
        st = pt_stats()
        _check(lib().pt_render_tiles(self._s, tile_offset, tile_stride, ctypes.c_void_p(d_accum),
                                     ctypes.c_void_p(stream), ctypes.byref(st)))
        return st.as_dict()

    def render_range_device(self, tile_offset: int, tile_stride: int, s_begin: int, s_end: int, d_accum: int,
                            stream: int = 0) -> dict:
        st = pt_stats()
        _check(lib().pt_render_range(self._s, tile_offset, tile_stride, s_begin, s_end, ctypes.c_void_p(d_accum),
                                     ctypes.c_void_p(stream), ctypes.byref(st)))
        return st.as_dict()

    def resolve(self, accum: np.ndarray) -> np.ndarray:
        accum = np.ascontiguousarray(accum, np.float32)
        w, h = self.film_size()
        rgb = np.zeros((h, w, 3), np.float32)
        _check(lib().pt_resolve_film(self._s, _fptr(accum), _fptr(rgb)))
        return rgb

    def bvh(self) -> Tuple[np.ndarray, np.ndarray]:
        n, m = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().pt_scene_bvh(self._s, ctypes.byref(n), None, ctypes.byref(m), None))
        nodes = np.zeros((n.value, 8), np.uint32)
        order = np.zeros(m.value, np.int32)
        _check(lib().pt_scene_bvh(self._s, ctypes.byref(n), nodes.ctypes.data, ctypes.byref(m), order.ctypes.data))
        return nodes, order

    # ---- test hooks ----
    def debug_halton(self, idx: np.ndarray, dims: np.ndarray) -> np.ndarray:
        idx = np.ascontiguousarray(idx, np.uint32)
        dims = np.ascontiguousarray(dims, np.int32)
        out = np.zeros(len(idx), np.float32)
        _check(lib().pt_debug_halton(self._s, len(idx), idx.ctypes.data, dims.ctypes.data, out.ctypes.data))
        return out

    def debug_pixel_offsets(self, pix: np.ndarray) -> np.ndarray:
        pix = np.ascontiguousarray(pix, np.int32)
        out = np.zeros(len(pix), np.uint32)
        _check(lib().pt_debug_pixel_offsets(self._s, len(pix), pix.ctypes.data, out.ctypes.data))
        return out

    def debug_camera_rays(self, film_xy: np.ndarray) -> np.ndarray:
        film_xy = np.ascontiguousarray(film_xy, np.float32)
        out = np.zeros((len(film_xy), 6), np.float32)
        _check(lib().pt_debug_camera_rays(self._s, len(film_xy), film_xy.ctypes.data, out.ctypes.data))
        return out

    def debug_trace(self, rays7: np.ndarray, any_hit: bool) -> np.ndarray:
        rays7 = np.ascontiguousarray(rays7, np.float32)
        out = np.zeros(len(rays7), np.int32)
        _check(lib().pt_debug_trace(self._s, len(rays7), rays7.ctypes.data, int(any_hit), out.ctypes.data))
        return out

    def debug_trace_frame(self, rays7: np.ndarray, any_hit: bool) -> Tuple[np.ndarray, int, int]:
        """The queries through the frame's traversal kernel: (hits, node visits, primitive tests)."""
        rays7 = np.ascontiguousarray(rays7, np.float32)
        out = np.zeros(len(rays7), np.int32)
        cnt = np.zeros(2, np.uint64)
        _check(lib().pt_debug_trace_frame(self._s, len(rays7), rays7.ctypes.data, int(any_hit), out.ctypes.data,
                                          cnt.ctypes.data))
        return out, int(cnt[0]), int(cnt[1])

    def debug_trace_frame_stats(self, rays7: np.ndarray, any_hit: bool) -> Tuple[np.ndarray, dict]:
        """The queries through the frame's traversal kernel: (hits, the traversal's pt_stats)."""
        rays7 = np.ascontiguousarray(rays7, np.float32)
        out = np.zeros(len(rays7), np.int32)
        st = pt_stats()
        _check(lib().pt_debug_trace_frame_ex(self._s, len(rays7), rays7.ctypes.data, int(any_hit), out.ctypes.data,
                                             ctypes.byref(st)))
        return out, st.as_dict()

    def debug_bsdf(self, material: int, rec8: np.ndarray) -> np.ndarray:
        """(n, 8) records wo, wi, u0, u1 -> (n, 8) f, pdf, sampled wi, sampled pdf."""
        rec8 = np.ascontiguousarray(rec8, np.float32)
        out = np.zeros_like(rec8)
        _check(lib().pt_debug_bsdf(self._s, material, len(rec8), rec8.ctypes.data, out.ctypes.data))
        return out

    def close(self) -> None:
        if self._s:
            lib().pt_scene_destroy(self._s)
            self._s = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_pfm(path: str, rgb: np.ndarray) -> None:
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    _check(lib().pt_write_pfm(os.fsencode(path), _fptr(rgb), w, h))


def write_image(path: str, rgb: np.ndarray, full_res=None, offset=(0, 0)) -> None:
    """WriteImage by suffix (.exr/.pfm/.png/.tga) of a cropped (h, w, 3) image."""
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    fw, fh = full_res or (w, h)
    _check(lib().pt_write_image(os.fsencode(path), _fptr(rgb), w, h, fw, fh, offset[0], offset[1]))


def exported_symbols() -> list:
    """pt_* function names declared in include/pt.h."""
    import re
    hdr = os.path.join(os.path.dirname(HERE), "include", "pt.h")
    text = open(hdr).read()
    decl = re.compile(r"^(?:const\s+)?[a-z_]+\s*\*?\s*(pt_[a-z0-9_]+)\s*\(", re.M)
    return sorted(set(decl.findall(text)))


def comm_unique_id() -> bytes:
    """pt_comm_unique_id: the RCCL unique id rank 0 hands to every rank."""
    buf = ctypes.create_string_buffer(128)
    _check(lib().pt_comm_unique_id(buf))
    return buf.raw


class Comm:
    """pt_comm: RCCL communicator of a multi-process job on the current GPU."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        if len(uid) != 128:
            raise ValueError("unique id must be 128 bytes")
        self.nranks, self.rank = nranks, rank
        self._c = ctypes.c_void_p()
        _check(lib().pt_comm_create(nranks, rank, uid, ctypes.byref(self._c)))

    def render_frame(self, scene: "Scene", d_accum: int, stream: int = 0) -> dict:
        """pt_render_frame_dist: tiles t % nranks == rank, then the film reduce to rank 0."""
        st = pt_stats()
        _check(lib().pt_render_frame_dist(scene._s, self._c, ctypes.c_void_p(d_accum), ctypes.c_void_p(stream),
                                          ctypes.byref(st)))
        return st.as_dict()

    def reduce(self, scene: "Scene", d_accum: int, root: int = 0, stream: int = 0) -> None:
        _check(lib().pt_film_reduce(self._c, scene._s, ctypes.c_void_p(d_accum), root, ctypes.c_void_p(stream)))

    def close(self) -> None:
        if self._c:
            lib().pt_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
