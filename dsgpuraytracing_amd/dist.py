"""Multi-GPU tile sharding + framebuffer exchange (one process per GPU).

The reference has no multi-GPU path; pixels and samples are
independent and the scene is read-only, so the frame shards with no data-path
collective:
  * every rank holds the whole scene (replicated, <= a few hundred MB);
  * the reference's 32x32 tile FIFO (pathtracer.cpp:209-214) is dealt
    round-robin, tile_id mod world_size (interleaving balances the empty
    margins of the default Cornell-box framing);
  * each rank renders its tiles into a zero-initialised full frame on its GPU;
  * ONE exchange at the end: a sum-reduce of the frames onto rank 0 (RCCL over
    xGMI with the "nccl" backend; gloo on CPU for tests).  Non-owners add +0.0,
    so the assembled image is bit-identical to the 1-GPU image: the counter RNG
    keys every sample by (seed, pixel, sample), not by rank or schedule.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

Tile = Tuple[int, int, int, int]


def shard_tiles(tiles: Sequence[Tile], rank: int, world: int) -> List[Tile]:
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(tiles[rank::world])


def render_sharded(render_tiles: Callable[[List[Tile]], None], frame, tiles: Sequence[Tile], rank: int,
                   world: int, dst: int = 0, group=None):
    """Render this rank's share of `tiles` into `frame` (zeroed by the caller,
    a torch tensor on this rank's device) and sum-reduce the frames onto `dst`.
    `render_tiles(list_of_tiles)` writes those tiles' pixels into `frame`."""
    import torch.distributed as dist

    mine = shard_tiles(tiles, rank, world)
    render_tiles(mine)
    if world > 1:
        dist.reduce(frame, dst=dst, group=group)
    return frame


def init_from_env(backend: str):
    """torch.distributed init for `torchrun`-style env (RANK/WORLD_SIZE/MASTER_*)."""
    import os

    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend)
    return rank, world, local
