"""shard -- how one frame is split over N ranks (one process per GPU).

The reference renders a frame with one process and a thread pool over 16x16
tiles (SamplerIntegrator::Render, src/core/integrator.cpp:526-637;
ParallelFor2D, src/core/parallel.cpp).  Every (pixel, sample) path is
independent, so the units shard with no data-path collective:

  * "tiles" (default, strong scaling): rank r renders tiles t with
    t % N == r at the full spp -- the reference's 16x16 tile loop
    (integrator.cpp:533-538) dealt round-robin; 1/2/4/8 ranks render the same
    frame.
  * "samples-split" (strong scaling): the scene's spp are divided among the
    ranks, rank r renders [spp*r//N, spp*(r+1)//N).
  * "samples" (opt-in WEAK scaling): rank r renders camera-sample indices
    [r*spp, (r+1)*spp) of every pixel -- the Halton sequence simply continues
    (HaltonSampler::GetIndexForSample, src/samplers/halton.cpp:96-110), so N
    ranks together produce a different, N*spp frame.

Each rank accumulates Film::Pixel (XYZ sum + filter-weight sum, film.h:98-105)
for its units; the films combine by addition (Film::MergeFilmTile is a sum,
film.cpp:117-130), done once per frame with a reduce to rank 0, which then
resolves the image (Film::WriteImage, film.cpp:169-211).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

MODES = ("tiles", "samples-split", "samples")


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    tile_offset: int
    tile_stride: int
    sample_begin: int
    sample_end: int

    @property
    def samples_per_pixel(self) -> int:
        return self.sample_end - self.sample_begin


def plan(rank: int, world: int, spp: int, mode: str = "tiles") -> Shard:
    """The units rank `rank` of `world` renders for a scene with `spp` samples
    per pixel."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    if spp < 1:
        raise ValueError("spp must be positive")
    if mode == "samples":
        return Shard(rank, world, 0, 1, rank * spp, (rank + 1) * spp)
    if mode == "samples-split":
        return Shard(rank, world, 0, 1, spp * rank // world, spp * (rank + 1) // world)
    if mode == "tiles":
        return Shard(rank, world, rank, world, 0, spp)
    raise ValueError(f"unknown shard mode {mode!r} (one of {MODES})")


def frame_samples(spp: int, world: int, mode: str) -> int:
    """Samples per pixel of the combined frame."""
    return spp * world if mode == "samples" else spp


def render_frame(shard: Shard, render: Callable[[Shard], dict], accum, reduce: Optional[Callable] = None) -> dict:
    """One frame on this rank: zero the film, render the shard into it, then
    sum the films onto rank 0.  `render(shard)` draws into `accum`;
    `reduce(accum)` is the cross-rank sum (torch.distributed.reduce to 0)."""
    accum.zero_()
    st = render(shard)
    if shard.world > 1 and reduce is not None:
        reduce(accum)
    return st


def device_renderer(scene, d_accum_ptr: int, stream: int) -> Callable[[Shard], dict]:
    """render() for render_frame on the GPU: pt_render_range into a device film."""
    def render(sh: Shard) -> dict:
        return scene.render_range_device(sh.tile_offset, sh.tile_stride, sh.sample_begin, sh.sample_end,
                                         d_accum_ptr, stream)
    return render


def reduce_to_root(accum) -> None:
    """torch.distributed reduce (the gloo CPU tests; the GPU bench reduces
    with the library's own RCCL communicator, ptgpu.Comm)."""
    import torch.distributed as dist
    dist.reduce(accum, dst=0)


def summarize_rank_times(per_rank) -> dict:
    """Per-step timing of every rank, so a scaling run can tell tail imbalance
    (one rank's tiles taking longer) from the cost of the frame's one
    collective.  per_rank: [(render_ms, reduce_ms), ...] in rank order --
    render_ms is the rank's own device render time of its shard, reduce_ms its
    ncclReduce of the film (HIP events around it: the wait for the slowest
    rank plus the transfer)."""
    rend = [float(r) for r, _ in per_rank]
    red = [float(x) for _, x in per_rank]
    mean = sum(rend) / len(rend)
    return {"ranks": len(per_rank),
            "render_ms_per_step": {"max": round(max(rend), 3), "min": round(min(rend), 3), "mean": round(mean, 3)},
            "render_imbalance": round(max(rend) / mean, 4) if mean > 0 else None,
            "reduce_ms_per_step": {"max": round(max(red), 3), "min": round(min(red), 3)},
            "per_rank_render_ms": [round(v, 3) for v in rend]}


def gather_rank_times(render_ms: float, reduce_ms: float, world: int, device="cpu") -> Optional[dict]:
    """All-gather (render_ms, reduce_ms) of every rank; the summary on every
    rank (world 1: this process alone, no collective)."""
    if world <= 1:
        return summarize_rank_times([(render_ms, reduce_ms)])
    import torch
    import torch.distributed as dist
    mine = torch.tensor([render_ms, reduce_ms], dtype=torch.float64, device=device)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    return summarize_rank_times([(float(t[0]), float(t[1])) for t in every])


def scaling(mode: str) -> str:
    return "weak" if mode == "samples" else "strong"
