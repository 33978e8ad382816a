"""Diagnostic: dump rays where the device trace disagrees with the oracle on
the Triangle.Reintersect cases (writes gpurun_out/reint_diag.npz)."""
import os, sys, pathlib
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "oracle"), os.path.join(R, "pbrt-v3-light-portals_amd"), os.path.join(R, "tests")]
import numpy as np, pyoracle, ptgpu
from test_reference_unit_tests import one_triangle_scene
tmp = pathlib.Path("/tmp/ri"); tmp.mkdir(exist_ok=True)
out = {}
done = 0
for i in range(200):
    case = pyoracle.reintersect_case(i, 2000)
    if case is None:
        continue
    tri, rays, bad = case
    hs = ptgpu.HostScene(one_triangle_scene(tmp, tri, f"r{i}.pbrt"))
    sc = ptgpu.Scene(hs)
    for ah in (False, True):
        got = sc.debug_trace(rays, ah)
        ref = pyoracle.trace(hs.desc, rays, ah)
        g = (got >= 0) if not ah else got != 0
        r = (ref >= 0) if not ah else ref != 0
        bad_idx = np.nonzero(g != r)[0]
        if len(bad_idx):
            print(i, ah, len(bad_idx), "of", len(rays), flush=True)
            out[f"tri{i}"] = tri
            out[f"rays{i}_{int(ah)}"] = rays[bad_idx[:16]]
    done += 1
    if done == 64:
        break
os.makedirs(os.path.join(R, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(R, "gpurun_out", "reint_diag.npz"), **out)
print("cases", done)
