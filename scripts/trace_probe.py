"""Trace-kernel probe: render a scene once per environment variant (set before
the scene is created) and print the trace counters, SIMD utilisation and time.

usage: PT_TRACE_DEBUG=1 python scripts/trace_probe.py scene.pbrt SPP "ENV=.. ENV=.." ...
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pbrt-v3-light-portals_amd"))
import ptgpu  # noqa: E402


def main():
    path, spp = sys.argv[1], int(sys.argv[2])
    hs = ptgpu.HostScene(path)
    import ctypes
    ctypes.cast(ctypes.c_void_p(hs.desc), ctypes.POINTER(ptgpu.pt_scene_desc)).contents.sampler.spp = spp
    for variant in sys.argv[3:]:
        saved = dict(os.environ)
        for kv in variant.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        sc = ptgpu.Scene(hs, device=0)
        sc.render()  # warm-up
        t0 = time.time()
        _, st = sc.render()
        dt = time.time() - t0
        rays = max(1, st["closest_rays"] + st["shadow_rays"])
        print(f"[{variant}] {dt * 1e3:.1f} ms trace {st['trace_ms']:.2f} ms ({st['trace_launches']} launches) shade "
              f"{st['shade_ms']:.2f} ms nodes/ray {st['node_visits'] / rays:.3f} "
              f"prims/ray {st['prim_tests'] / rays:.3f}", flush=True)
        del sc
        os.environ.clear()
        os.environ.update(saved)


if __name__ == "__main__":
    main()
