"""Multi-GPU paths on the device: the frame's 16x16 tiles dealt
round-robin over devices (t % N == k, integrator.cpp:533-538) and the films
summed (Film::MergeFilmTile is a sum, film.cpp:117-130).

  * in-process: pt_init(n, ids) + pt_render -- one scene replica and host
    thread per device, films summed on the first device in device order;
    on the one-GPU test box the replicas share device 0;
  * multi-process: ranks render their tile stride on the device and reduce
    over gloo (the CPU reduce of tests/test_distributed.py), and the
    library's RCCL communicator (pt_comm_create + pt_render_frame_dist) on a
    one-rank job.

Films from disjoint tile sets add; only pixels reached by three or more tiles
(filter spill at tile corners) can differ from the single-device merge order,
by rounding."""
import os
import socket

import numpy as np
import pytest

from conftest import scene_variant

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _same_counts(a, b):
    for k in ("samples", "closest_rays", "shadow_rays", "node_visits", "prim_tests"):
        assert a[k] == b[k], k


def _close(got, ref):
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-7)
    assert np.mean(got == ref) > 0.99


@pytest.mark.parametrize("ndev", [2, 3])
def test_replicas_match_single_device(tmp_path, ndev):
    import ptgpu
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=(72, 40), spp=8))
    one, st1 = ptgpu.Scene(hs, device=0).render()
    many, stn = ptgpu.Scene(hs, devices=[0] * ndev).render()
    _same_counts(st1, stn)
    _close(many, one)


def _gpus() -> int:
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_gpus() < 2, reason="needs two GPUs (the test box has one)")
def test_replicas_on_distinct_devices(tmp_path):
    """Replicas on two different devices: the films cross devices by
    hipMemcpyPeer and are summed on ids[0]; each replica's streams and
    buffers are freed with its own device current.  Same frame as one device."""
    import ptgpu
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=(72, 40), spp=8))
    one, st1 = ptgpu.Scene(hs, device=0).render()
    sc = ptgpu.Scene(hs, devices=[0, 1])
    many, stn = sc.render()
    del sc
    _same_counts(st1, stn)
    _close(many, one)


def test_replicas_take_batch_and_pipeline_settings(tmp_path):
    """pt_set_batch_slots / pt_set_pipelines reach every replica (the query
    reads -1 when a replica differs); a small batch on two replicas renders
    the single-device frame."""
    import ptgpu
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=(72, 40), spp=8))
    one, st1 = ptgpu.Scene(hs, device=0).render()
    sc = ptgpu.Scene(hs, devices=[0, 0], batch_slots=4096)
    sc.set_pipelines(3)
    assert sc.query("batch_slots") == 4096
    assert sc.query("pipelines") == 3
    many, stn = sc.render()
    _same_counts(st1, stn)
    _close(many, one)


def _worker(rank, world, port, scene, out, mode):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest  # noqa: F401  (sys.path for the package)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda:0")  # torch's HIP context first, then the library
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import ptgpu
    try:
        hs = ptgpu.HostScene(scene)
        sc = ptgpu.Scene(hs, device=0)
        w, h = sc.film_size()
        acc = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda:0")
        spp = hs.spp()
        if mode == "rccl":
            comm = ptgpu.Comm(world, rank, ptgpu.comm_unique_id())
            st = comm.render_frame(sc, acc.data_ptr(), 0)
            torch.cuda.synchronize()
            assert st["reduce_ms"] > 0 and st["render_ms"] > 0  # bench.py's per-rank diagnostics
            film = acc.cpu()
            comm.close()
        else:
            st = sc.render_range_device(rank, world, 0, spp, acc.data_ptr(), 0)
            torch.cuda.synchronize()
            film = acc.cpu()
            dist.reduce(film, dst=0)
        n = torch.tensor([st["samples"], st["closest_rays"], st["shadow_rays"]], dtype=torch.float64)
        dist.all_reduce(n)
        if rank == 0:
            np.save(out, film.numpy())
            np.save(out + ".n.npy", n.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,world", [("device-gloo", 2), ("rccl", 1)])
def test_rank_tile_split_matches_single_process(tmp_path, mode, world):
    import torch.multiprocessing as mp
    import ptgpu
    scene = scene_variant(tmp_path, res=(72, 40), spp=8)
    out = str(tmp_path / f"film_{mode}.npy")
    mp.start_processes(_worker, args=(world, _free_port(), scene, out, mode), nprocs=world, join=True,
                       start_method="spawn")
    film, n = np.load(out), np.load(out + ".n.npy")
    hs = ptgpu.HostScene(scene)
    ref, st = ptgpu.Scene(hs, device=0).render_accum()
    assert (n[0], n[1], n[2]) == (st["samples"], st["closest_rays"], st["shadow_rays"])
    _close(film, ref)
