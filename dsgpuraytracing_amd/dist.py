"""Multi-GPU tile sharding + framebuffer exchange (one process per GPU).

The reference has no multi-GPU path; pixels and samples are
independent and the scene is read-only, so the frame shards with no data-path
collective:
  * every rank holds the whole scene (replicated, <= a few hundred MB);
  * the reference's 32x32 tile FIFO (pathtracer.cpp:209-214) is dealt
    diagonally, (column + row) mod world_size: interleaving balances the empty
    margins of the default Cornell-box framing, and unlike tile_id mod N it
    does not deal whole tile columns when the row length is a multiple of N
    (C3 on 8 GPUs: slowest rank 1.20x the mean with mod, 1.06x with diag,
    tools/shard_balance.py);
  * each rank renders its tiles into a PACKED buffer (PT_FLAG_PACKED: slot i
    = its i-th tile, 32x32 row-major), padded to ceil(n_tiles / world) slots;
  * ONE exchange at the end: a gather of the packed buffers onto rank 0 (RCCL
    over xGMI with the "nccl" backend, gloo on CPU for tests) -- each rank
    sends only its own tiles (1/world of the frame; 1.6 MB per rank at 1024^2
    on 8 GPUs, all seven links into the root in parallel), not a whole frame --
    then rank 0 scatters the tiles into the frame.  The counter RNG keys
    every sample by (seed, pixel, sample), not by rank or schedule, so the
    assembled image is bit-identical to the 1-GPU image.
  * back-to-back frames (PipelinedExchange): frame k's gather + scatter are
    queued behind its resolve on the current stream; the renders run on the
    library's render-slot streams, so they overlap frame k+1's render (a
    side-stream variant behind events is kept for A/Bs).
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np

Tile = Tuple[int, int, int, int]
TILE = 32


def tile_owner(tile: Tile, index: int, world: int, deal: str = "mod", tile_size: int = TILE) -> int:
    """Rank that renders `tile` (FIFO position `index`).  "mod": tile_id mod
    world; "diag": (column + row) mod world, so a rank's tiles also spread
    over every column when the row length is a multiple of world (plain mod
    then deals whole columns); "diagK": (column + K*row) mod world; "auto":
    diag3 at 8 or more ranks, diag below.  Columns
    and rows count tiles of `tile_size` pixels (the FIFO's tile edge)."""
    col, row = tile[0] // tile_size, tile[1] // tile_size
    if deal == "mod":
        return index % world
    if deal == "auto":
        # the measured best per world size (C3, slowest rank's share with the
        # RCCL exchange in the loop: profiles/r6/ab_split_deal.txt): diag3 at
        # 8 ranks (0.21 vs diag's 0.23 ms), diag below (N = 4: 0.317 vs
        # 0.322; N = 2 the two are the same checkerboard)
        deal = "diag3" if world >= 8 else "diag"
    if deal.startswith("diag") and (deal[4:] == "" or deal[4:].isdigit()):
        # "diagK": (column + K * row) mod world
        return (col + int(deal[4:] or 1) * row) % world
    raise ValueError(f"unknown tile deal {deal!r}")


def shard_tiles(tiles: Sequence[Tile], rank: int, world: int, deal: str = "mod", tile_size: int = TILE) -> List[Tile]:
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if deal == "mod":
        return list(tiles[rank::world])
    return [t for i, t in enumerate(tiles) if tile_owner(t, i, world, deal, tile_size) == rank]


def packed_index(tiles: Sequence[Tile], width: int, slot0: int = 0, slot: int = TILE):
    """(packed pixel index, frame pixel index) pairs of every pixel of `tiles`
    in the packed layout of `slot` x `slot` slots (PT_FLAG_PACKED: 32,
    PT_FLAG_PACKED16: 16; tile i -> [(slot0+i)*slot^2, +slot^2), pixel (x, y)
    at (y-ty)*slot + (x-tx)); frame index x + y*width."""
    src, dst = [], []
    for i, (tx, ty, tw, th) in enumerate(tiles):
        ly, lx = np.meshgrid(np.arange(th), np.arange(tw), indexing="ij")
        src.append(((slot0 + i) * slot * slot + ly * slot + lx).ravel())
        dst.append(((ty + ly) * width + tx + lx).ravel())
    if not src:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    return np.concatenate(src).astype(np.int64), np.concatenate(dst).astype(np.int64)


class TileExchange:
    """Packed-tile gather of a sharded frame onto `dst`.

    `render_packed(mine, packed)` renders this rank's tiles `mine` into
    `packed` (a (slots, 1024, 3) float32 tensor on this rank's device, slot i =
    mine[i]); `exchange(frame)` gathers every rank's packed tiles onto `dst`
    and writes them into `frame` ((H, W, 3) float32 on `dst`'s device).  The
    index maps are built once: a frame's tile deal does not change between
    steps.  The render must be queued on torch's current stream (a non-zero
    torch.cuda.Stream, see bench.py): the collective is ordered after the
    current stream's work, not after the pt_ctx's own stream."""

    def __init__(self, tiles: Sequence[Tile], width: int, height: int, rank: int, world: int, device,
                 dst: int = 0, group=None, deal: str = "diag", buffers: int = 1, tile_size: int = TILE,
                 deal_block: int = 0):
        import torch

        self.rank, self.world, self.dst, self.group = rank, world, dst, group
        self.width, self.height = width, height
        # the FIFO's edge tiles overhang the frame (raytrace_tile clamps them,
        # pathtracer.cpp:594-595); packed slots hold the clamped tiles
        tiles = [(x, y, min(w, width - x), min(h, height - y)) for (x, y, w, h) in tiles]
        self.deal = deal
        # the deal counts columns and rows of `deal_block` pixels (default: the
        # tile edge); 16x16 tiles dealt by 32x32 blocks keep a block's four
        # tiles on one rank
        db = deal_block or tile_size
        self.mine = shard_tiles(tiles, rank, world, deal, db)
        self.slots = max(len(shard_tiles(tiles, r, world, deal, db)) for r in range(world))
        # `buffers` packed buffers (PipelinedExchange: 2); `packed` is the current one
        # packed slots of the deal's tile edge (PT_FLAG_PACKED16 for 16x16 tiles)
        self.slot = 16 if tile_size <= 16 else TILE
        self.bufs = [torch.zeros((max(self.slots, 1), self.slot * self.slot, 3), dtype=torch.float32, device=device)
                     for _ in range(max(1, buffers))]
        self.packed = self.bufs[0]
        self.recv = None
        if rank == dst:
            self.recv = torch.zeros((world, max(self.slots, 1), self.slot * self.slot, 3), dtype=torch.float32,
                                    device=device)
            src, dstix = [], []
            for r in range(world):
                s, d = packed_index(shard_tiles(tiles, r, world, deal, db), width, slot0=r * max(self.slots, 1),
                                    slot=self.slot)
                src.append(s)
                dstix.append(d)
            src, dstix = np.concatenate(src), np.concatenate(dstix)
            self.src = torch.from_numpy(src).to(device)
            self.dstix = torch.from_numpy(dstix).to(device)
            # tiles covering the whole frame (every split of the FIFO): each
            # frame pixel reads its one packed pixel -- ONE gather kernel
            # straight into the frame, no temporary
            self.perm = None
            if len(dstix) == width * height:
                perm = np.full(width * height, -1, np.int64)
                perm[dstix] = src
                if (perm >= 0).all():
                    self.perm = torch.from_numpy(perm).to(device)

    def gather(self, packed=None):
        """Every rank's packed tiles (`packed`, default the current buffer)
        into `recv[rank]` on `dst` (one collective; with an initialised process
        group also at world size 1, so the RCCL path is the one a 1-GPU test
        exercises)."""
        import torch
        import torch.distributed as dist

        packed = self.packed if packed is None else packed
        coll = dist.is_available() and dist.is_initialized()
        if coll and packed.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo gathers host tensors only (tests / one-GPU rehearsals)
            src = packed.cpu()
            gl = [torch.empty_like(src) for _ in range(self.world)] if self.rank == self.dst else None
            dist.gather(src, gather_list=gl, dst=self.dst, group=self.group)
            if self.rank == self.dst:
                self.recv.copy_(torch.stack(gl))
        elif coll:
            gl = list(self.recv.unbind(0)) if self.rank == self.dst else None
            dist.gather(packed, gather_list=gl, dst=self.dst, group=self.group)
        else:
            self.recv[0].copy_(packed)

    def scatter(self, frame):
        """On `dst`: the gathered tiles into their frame pixels."""
        import torch

        if self.rank == self.dst:
            if self.perm is not None and frame.is_contiguous():
                torch.index_select(self.recv.view(-1, 3), 0, self.perm, out=frame.view(-1, 3))
            else:
                frame.view(-1, 3).index_copy_(0, self.dstix, self.recv.view(-1, 3).index_select(0, self.src))
        return frame

    def exchange(self, frame):
        self.gather()
        return self.scatter(frame)


class PipelinedExchange:
    """Back-to-back sharded frames with the exchange off the render's path.

    Frame k renders into packed buffer k % buffers (`packed_for(k)`, called BEFORE
    the render is queued); `exchange(k, frame)` gathers frame k's buffer onto
    `dst` and scatters it into `frame`.  The renders themselves run on the
    library's render-slot streams (pt_api.cpp), so frame k+1's render overlaps
    frame k's resolve and exchange whichever stream the exchange is queued on.
    Default: on the current stream, right behind frame k's resolve (ordered,
    no cross-stream hop; one packed buffer would do).  side=True: on a side
    stream behind an event (the current stream first waits, in
    `packed_for(k)`, until frame k-2's gather has read that buffer) -- kept
    for A/Bs.  `xev` collects (start, end) events around each exchange.
    Gathers, the shared receive buffer and scatters follow frame order.  On
    CPU tensors (tests) the same calls run synchronously.  The images are
    those of TileExchange, bit for bit."""

    def __init__(self, tiles: Sequence[Tile], width: int, height: int, rank: int, world: int, device,
                 dst: int = 0, group=None, deal: str = "diag", side: bool = False, buffers: int = 2,
                 tile_size: int = TILE, deal_block: int = 0):
        import torch

        # `buffers` packed buffers, frame k in buffer k % buffers: at least the
        # frames of one frame batch (bench.py --frames-per-launch), whose
        # resolves all run before the batch's exchanges
        self.ex = TileExchange(tiles, width, height, rank, world, device, dst=dst, group=group, deal=deal,
                               buffers=max(2, buffers), tile_size=tile_size, deal_block=deal_block)
        self.mine = self.ex.mine
        self.cuda = self.ex.bufs[0].is_cuda
        # side=False (default): the exchange is queued on the current stream
        # right behind the resolve -- no cross-stream hop between them: the
        # C4 split's N = 8 share 2.13 -> 1.86 ms per frame, the C3 shares
        # even (profiles/r6/ab_stream_queues.txt, sessions v and w)
        self.side = torch.cuda.Stream(device=self.ex.bufs[0].device) if self.cuda and side else None
        self.on_current = self.cuda and not side
        self.free = [None] * len(self.ex.bufs)  # per buffer: event after the gather that last read it
        self.xev = []

    def packed_for(self, k: int):
        import torch

        b = k % len(self.ex.bufs)
        if self.cuda and self.free[b] is not None:
            torch.cuda.current_stream().wait_event(self.free[b])
        self.ex.packed = self.ex.bufs[b]
        return self.ex.bufs[b]

    def exchange(self, k: int, frame, timed: bool = False):
        import torch

        buf = self.ex.bufs[k % len(self.ex.bufs)]
        if not self.cuda:
            self.ex.gather(buf)
            return self.ex.scatter(frame)
        if self.on_current:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self.ex.gather(buf)
            self.ex.scatter(frame)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            if timed:
                self.xev.append((e0, e1))
            return frame
        done = torch.cuda.Event()
        done.record()  # on the current (render) stream
        with torch.cuda.stream(self.side):
            self.side.wait_event(done)
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self.ex.gather(buf)
            self.ex.scatter(frame)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            free = torch.cuda.Event()
            free.record()
        self.free[k % len(self.ex.bufs)] = free
        if timed:
            self.xev.append((e0, e1))
        return frame

    def drain(self):
        """The current stream waits for every exchange issued so far."""
        import torch

        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)

    def exchange_ms(self) -> float:
        return float(np.mean([a.elapsed_time(b) for a, b in self.xev])) if self.xev else 0.0


def render_sharded(render_packed: Callable[[List[Tile], object], None], frame, tiles: Sequence[Tile], rank: int,
                   world: int, dst: int = 0, group=None, exchange: TileExchange | None = None):
    """Render this rank's share of `tiles` and assemble the frame on `dst`.
    `render_packed(mine, packed)` writes tile mine[i]'s pixels into packed[i]
    (PT_FLAG_PACKED layout).  Pass a TileExchange to reuse its buffers and
    index maps across frames.  A rank whose render raises still joins the
    exchange, then every rank raises RankFailure naming it (the status check
    comes after the gather, so no rank is left waiting in it)."""
    h, w = frame.shape[0], frame.shape[1]
    ex = exchange or TileExchange(tiles, w, h, rank, world, frame.device, dst=dst, group=group)
    guard = StepGuard(group)
    guard.run(render_packed, ex.mine, ex.packed)
    ex.exchange(frame)
    guard.check()
    return frame


# Environment knobs of libptgpu.so that change pixel VALUES (not only speed):
# the sample grouping (group size, the resident grid it is sized by) fixes
# each pixel's float summation order, the render tree (its tie-breaks between
# equidistant primitives) and the footprint cull decide values, and so does
# the library.  Ranks that disagree on them would assemble a frame that is not
# the 1-GPU frame bit for bit.
VALUE_KNOBS = ("PT_SAMPLE_GROUP", "PT_WAVES_PER_CU", "PT_NO_FOOTPRINT_CULL", "PT_BVH_BUILD",
               "PT_COLLAPSE", "PT_LBVH_PASSES", "PT_LBVH_CI", "PT_LBVH_MAXLEAF", "PT_SAH_BINS", "PT_SAH_CI",
               "PT_SAH_LEAF", "PT_LIB")
DEFAULT_TIMEOUT_S = 120


class RankFailure(RuntimeError):
    """Raised on EVERY rank when any rank failed (`failed` = [(rank, message)]).

    The reference exits the process on any device error
    (cuda_src/setup.cu:139-143, 173-177), which in a multi-process job would
    leave the other ranks blocked in the frame exchange until the process-group
    timeout.  Here a failing rank keeps taking part in the collectives of the
    frame it failed in, the ranks agree on a status at the next check point,
    and all of them raise this with the failing rank's pt_last_error."""

    def __init__(self, failed):
        self.failed = list(failed)
        super().__init__("; ".join(f"rank {r}: {m}" for r, m in self.failed))


def _flag_device(group=None):
    import torch
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"


def agree_status(err, group=None):
    """Collective: every rank passes its error message (None = fine).  Raises
    RankFailure on every rank if any rank failed; one int32 MAX all-reduce when
    all are fine."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        if err:
            raise RankFailure([(0, err)])
        return
    flag = torch.tensor([1 if err else 0], dtype=torch.int32, device=_flag_device(group))
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag.item()):
        msgs = [None] * dist.get_world_size(group)
        dist.all_gather_object(msgs, err, group=group)
        raise RankFailure([(r, m) for r, m in enumerate(msgs) if m])


class StepGuard:
    """Runs a rank's per-frame work without letting an exception leave the
    collective schedule: the first failure is recorded (and the work skipped
    from then on), the rank keeps joining the exchanges, and `check()` -- a
    collective, called at the caller's synchronisation points -- turns any
    rank's failure into RankFailure everywhere."""

    def __init__(self, group=None):
        self.group = group
        self.err = None

    def run(self, fn, *args, **kw):
        if self.err is not None:
            return None
        try:
            return fn(*args, **kw)
        except Exception as e:  # recorded, surfaced on every rank by check()
            self.err = f"{type(e).__name__}: {e}"
            return None

    def check(self):
        agree_status(self.err, self.group)


def check_value_knobs(extra=None, group=None):
    """Collective: refuse to render a split frame when the ranks' value knobs
    (VALUE_KNOBS, plus `extra`, e.g. the sample grouping a launch chose)
    differ.  Returns this rank's fingerprint."""
    import os

    import torch.distributed as dist

    mine = {k: os.environ.get(k) for k in VALUE_KNOBS}
    if extra:
        mine.update(extra)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return mine
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, mine, group=group)
    bad = [(r, f"value knobs {v} differ from rank 0's {allv[0]}") for r, v in enumerate(allv) if v != allv[0]]
    if bad:
        raise RankFailure(bad)
    return mine


def init_from_env(backend: str, timeout_s: float | None = None):
    """torch.distributed init for `torchrun`-style env (RANK/WORLD_SIZE/MASTER_*).
    A finite timeout (PT_DIST_TIMEOUT seconds, default 120) bounds how long a
    rank waits in a collective for a peer that died."""
    import datetime
    import os

    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if timeout_s is None:
        timeout_s = float(os.environ.get("PT_DIST_TIMEOUT", DEFAULT_TIMEOUT_S))
    timeout = datetime.timedelta(seconds=timeout_s)
    # PT_DIST_FORCE=1 (experiments): a one-rank group, so that a one-GPU run
    # (bench.py --emulate-shard) issues its exchange through RCCL and torch's
    # collective stream, as every rank of an N-GPU run does
    force = os.environ.get("PT_DIST_FORCE") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":  # RCCL: bind the group to this rank's GPU (eager communicator init)
            import torch
            dist.init_process_group(backend, timeout=timeout,
                                    device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group(backend, timeout=timeout)
    return rank, world, local
