"""The N>1 harness of bench.py on CPU: world_size-2 gloo process group (127.0.0.1), barriers,
max-over-ranks timing, whole-job aggregation and query sharding."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lvo_amd_loader import lvo
    R = lvo.replicas
    import time
    # rank r works (r + 1) * 50 ms: the job time is the slowest rank's
    elapsed, out = R.timed_region(lambda: (time.sleep(0.05 * (rank + 1)), rank)[1], dist=dist)
    lo, hi = R.shard_range(233, rank, world)
    cover = torch.zeros(233, dtype=torch.int32)
    cover[lo:hi] += 1
    dist.all_reduce(cover)
    q.put((rank, elapsed, out, R.replica_start_frame(rank), int(cover.min()), int(cover.max()),
           R.aggregate_rate(10, world, elapsed)))
    dist.destroy_process_group()


def test_two_rank_gloo_harness():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    el = [r[1] for r in res]
    assert el[0] == el[1]                       # max over ranks, identical on every rank
    assert el[0] >= 0.1                          # the slow rank (2 x 50 ms) defines it
    assert [r[2] for r in res] == [0, 1]
    assert [r[3] for r in res] == [0, 1000]      # independent replica sequences
    assert all(r[4] == 1 and r[5] == 1 for r in res)   # every query on exactly one rank
    assert res[0][6] == pytest.approx(20 / el[0])


def test_shard_range_partitions():
    from lvo_amd_loader import lvo
    for n in (0, 1, 7, 232548):
        for w in (1, 2, 3, 8):
            rs = [lvo.replicas.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
