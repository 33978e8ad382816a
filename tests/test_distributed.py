"""N>1 path on CPU: world_size-2 gloo ranks run bench.py's frame logic
(shard.plan -> render_frame -> reduce to rank 0 -> host resolve), with the
oracle standing in for the per-rank device renderer (the device path is
covered by tests/test_gpu_parity.py).  The combined film must equal one
process rendering the whole frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import shard
from conftest import scene_variant


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scene, spp, mode, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest  # noqa: F401  (sys.path for the package and the oracle)
    import torch.distributed as dist
    import ptgpu
    import pyoracle
    import shard as sh
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        hs = ptgpu.HostScene(scene)
        w, h = hs.film_size()
        accum = torch.zeros((h, w, 4), dtype=torch.float32)
        my = sh.plan(rank, world, spp, mode)

        def render(s):
            acc, st = pyoracle.render_range(hs.desc, s.sample_begin, s.sample_end, nthreads=2,
                                            tile_offset=s.tile_offset, tile_stride=s.tile_stride)
            accum.add_(torch.from_numpy(acc))
            return st

        import time
        t0 = time.perf_counter()
        st = sh.render_frame(my, render, accum, None)
        t1 = time.perf_counter()
        sh.reduce_to_root(accum)
        t2 = time.perf_counter()
        # bench.py's per-rank diagnostics: every rank's render and reduce time, gathered
        times = sh.gather_rank_times((t1 - t0) * 1e3, (t2 - t1) * 1e3, world)
        n = torch.tensor([st["samples"]], dtype=torch.float64)
        dist.all_reduce(n)
        if rank == 0:
            import json
            json.dump(times, open(out + ".times.json", "w"))
            np.save(out, accum.numpy())
            np.save(out + ".rgb.npy", hs.resolve(accum.numpy()))
            np.save(out + ".n.npy", n.numpy())
    finally:
        dist.destroy_process_group()


def _run(tmp_path, mode, world=2):
    scene = scene_variant(tmp_path, res=(40, 24), spp=4)
    out = str(tmp_path / f"film_{mode}.npy")
    mp.start_processes(_worker, args=(world, _free_port(), scene, 4, mode, out), nprocs=world, join=True,
                       start_method="spawn")
    import json
    times = json.load(open(out + ".times.json"))
    assert times["ranks"] == world and len(times["per_rank_render_ms"]) == world
    for k in ("render_ms_per_step", "reduce_ms_per_step"):
        assert times[k]["max"] >= times[k]["min"] >= 0
    assert times["render_imbalance"] >= 1.0
    return scene, np.load(out), np.load(out + ".rgb.npy"), float(np.load(out + ".n.npy")[0])


def test_plan_partitions():
    for world in (1, 2, 3, 8):
        tiles = [shard.plan(r, world, 16, "tiles") for r in range(world)]
        assert sorted(t.tile_offset for t in tiles) == list(range(world))
        assert all(t.tile_stride == world and t.samples_per_pixel == 16 for t in tiles)
        split = [shard.plan(r, world, 16, "samples-split") for r in range(world)]
        assert split[0].sample_begin == 0 and split[-1].sample_end == 16
        assert all(a.sample_end == b.sample_begin for a, b in zip(split, split[1:]))
        weak = [shard.plan(r, world, 16, "samples") for r in range(world)]
        assert [(s.sample_begin, s.sample_end) for s in weak] == [(16 * r, 16 * r + 16) for r in range(world)]
    with pytest.raises(ValueError):
        shard.plan(2, 2, 4)
    with pytest.raises(ValueError):
        shard.plan(0, 1, 4, "pixels")


@pytest.mark.parametrize("mode", ["samples", "tiles"])
def test_two_rank_frame_matches_single_process(tmp_path, mode):
    import ptgpu
    import pyoracle
    scene, film, rgb, n = _run(tmp_path, mode)
    hs = ptgpu.HostScene(scene)
    w, h = hs.film_size()
    spp_total = shard.frame_samples(4, 2, mode)
    ref_film, st = pyoracle.render_range(hs.desc, 0, spp_total, nthreads=4)
    assert n == st["samples"] == w * h * spp_total
    # Films combine by addition; only the float summation order of pixels on
    # tile or rank boundaries differs from the single-process merge.
    np.testing.assert_allclose(film, ref_film, rtol=2e-6, atol=1e-7)
    ref_rgb = hs.resolve(ref_film)
    rmse = float(np.sqrt(np.mean((rgb.astype(np.float64) - ref_rgb) ** 2)))
    assert rmse < 1e-4 * max(1.0, float(ref_rgb.mean()))
    if mode == "tiles":
        # spp unchanged: the resolved frame is the reference render itself
        img, _ = pyoracle.render(hs.desc, nthreads=4)
        np.testing.assert_allclose(rgb, img, rtol=2e-6, atol=1e-7)


def test_rank_time_summary():
    """bench.py's multi-rank diagnostics (shard.summarize_rank_times): max / min
    render time, imbalance and reduce time of every rank."""
    t = shard.summarize_rank_times([(100.0, 5.0), (120.0, 1.0)])
    assert t["render_ms_per_step"] == {"max": 120.0, "min": 100.0, "mean": 110.0}
    assert t["reduce_ms_per_step"] == {"max": 5.0, "min": 1.0}
    assert abs(t["render_imbalance"] - 120 / 110) < 1e-3
    assert shard.gather_rank_times(7.0, 0.0, 1)["per_rank_render_ms"] == [7.0]


def test_host_resolve_matches_oracle_writeimage(tmp_path):
    import ptgpu
    import pyoracle
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=(24, 16), spp=2))
    film, _ = pyoracle.render_accum(hs.desc, nthreads=2)
    img, _ = pyoracle.render(hs.desc, nthreads=2)
    got = hs.resolve(film)
    assert np.array_equal(got.view(np.uint32), img.view(np.uint32))
