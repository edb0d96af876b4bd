"""Multi-GPU execution of the per-scan path.

One process per GPU (torchrun; backend "nccl" = RCCL on the GPU box, "gloo" in CPU tests).
* Across scans the path is a pose chain — scan k's odometry and mapping need scan k-1's — so N GPUs
  run N independent replica sequences ("scaling": "weak"); torch.distributed carries only the start /
  stop barriers and the max-over-ranks elapsed time, no data-path collective.
* Within one search (C4: one sweep against a large local map) queries are independent given the map:
  shard_range splits them into contiguous (scan-ordered, hence spatially coherent) chunks, map
  replicated, again without a collective.
* Scan-to-map registration (Context.s2m_register, laserMapping.cpp:556-727) shards its query stacks
  the same way and has ONE exchange step per LM pass: an RCCL all-gather of fixed-size normal-equation
  records issued by the library on its own stream (k_s2m.hip). init_shard() creates that communicator
  from an initialised torch.distributed group (the 128-byte RCCL id travels over it).
"""
import time


def replica_start_frame(rank, stride=1000):
    """First frame of rank's replica sequence: a different stretch of the synthetic street."""
    return stride * int(rank)


def shard_range(n, rank, world):
    """Contiguous [lo, hi) share of n items for rank (sizes differ by at most one)."""
    base, extra = divmod(int(n), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def timed_region(fn, dist=None, sync=None, device=None):
    """Runs fn() between barrier + sync pairs and returns the max over ranks of the elapsed seconds
    (the contract of bench.py: every rank's time counts, the slowest one defines the job)."""
    if dist is not None:
        dist.barrier()
    if sync is not None:
        sync()
    t0 = time.perf_counter()
    out = fn()
    if sync is not None:
        sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def aggregate_rate(units_per_rank, world, elapsed):
    """Whole-job throughput: all ranks' units over the max-over-ranks time."""
    return units_per_rank * world / elapsed if elapsed > 0 else 0.0


def init_shard(ctx, dist=None, uid_fn=None):
    """Attach ctx (anything with shard_init(rank, world, uid)) to a communicator spanning the
    torch.distributed world: rank 0 makes the RCCL unique id (uid_fn, default lvo.shard_unique_id),
    broadcasts it over the existing process group, every rank then joins (collective)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        ctx.shard_init(0, 1, None)
        return 0, 1
    rank, world = dist.get_rank(), dist.get_world_size()
    if uid_fn is None:
        from . import shard_unique_id as uid_fn
    box = [uid_fn() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    ctx.shard_init(rank, world, box[0])
    return rank, world


def init_peer_exchange(ctx, dist=None):
    """Open the device-side record exchange (aloam_shard_peer_open) across the torch.distributed world:
    every rank publishes its 64-byte IPC handle (ctx.shard_peer_handle()), all-gathers the world's, opens
    them, then every rank learns every other's outcome (an all-gather that is also the barrier no Solve
    may start before: every rank has zeroed its counters). Collective; if any rank failed, every rank
    closes the exchange and RuntimeError is raised on all of them (fall back to init_shard / RCCL)."""
    if dist is None or not dist.is_initialized():
        ctx.shard_peer_open([ctx.shard_peer_handle()], 0)
        return 0, 1
    rank, world = dist.get_rank(), dist.get_world_size()
    err = None
    try:
        h = ctx.shard_peer_handle()
    except Exception as e:  # noqa: BLE001 - reported collectively below
        h, err = None, f"rank {rank}: {e}"
    handles = [None] * world
    dist.all_gather_object(handles, h)
    if err is None:
        if any(x is None for x in handles):
            err = f"rank {rank}: a peer has no handle"
        else:
            try:
                ctx.shard_peer_open(handles, rank)
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank}: {e}"
    errs = [None] * world
    dist.all_gather_object(errs, err)
    bad = [e for e in errs if e]
    if bad:
        try:
            ctx.shard_peer_close()
        except Exception:  # noqa: BLE001
            pass
        raise RuntimeError("device exchange unavailable: " + bad[0])
    return rank, world
