"""CPU checks of the sharded scan-to-map registration's host side: the library's slot
decomposition (aloam_shard_slot_range, a pure host function of libaloam_hip.so) and the RCCL-id
hand-off over a world_size-2 gloo group (127.0.0.1). The device exchange itself is in test_s2m.py."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from lvo_amd_loader import abi, lvo  # noqa: E402

NREC = abi.ALOAM_S2M_RECORDS


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 1000, 262_000])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8, 16])
def test_slot_ranges_partition_in_record_blocks(n, world):
    rs = [lvo.shard_slot_range(n, r, world) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))       # contiguous, rank order, no overlap
    per = max(1, -(-n // NREC))
    # every boundary is a record-block boundary: the global blocks (and so the reduction) do not depend
    # on the world size
    for lo, hi in rs:
        assert lo % per == 0 or lo == n
    # the blocks are spread evenly: no rank holds more than ceil(NREC / world) blocks
    rp = -(-NREC // world)
    assert max(hi - lo for lo, hi in rs) <= rp * per


def test_slot_range_rejects_bad_args():
    for args in ((-1, 0, 1), (10, 1, 1), (10, -1, 2), (10, 0, 0), (10, 0, NREC + 1)):
        with pytest.raises(lvo.ALOAMError):
            lvo.shard_slot_range(*args)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeCtx:
    """Stands in for lvo.Context (no GPU here): records what shard_init received."""
    def __init__(self):
        self.args = None

    def shard_init(self, rank, world, uid):
        self.args = (rank, world, uid)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lvo_amd_loader import lvo as L
    calls = []

    def uid_fn():
        calls.append(rank)
        return L.shard_unique_id()          # the real RCCL id (ncclGetUniqueId needs no GPU)

    c = _FakeCtx()
    L.replicas.init_shard(c, dist, uid_fn=uid_fn)
    q.put((rank, c.args[0], c.args[1], c.args[2], calls))
    dist.destroy_process_group()


def test_init_shard_broadcasts_one_id_over_gloo():
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
    assert [r[1] for r in res] == [0, 1] and all(r[2] == 2 for r in res)
    assert len(res[0][3]) == 128 and res[0][3] == res[1][3]     # one id, made on rank 0 only
    assert res[0][4] == [0] and res[1][4] == []


def test_init_shard_single_process_needs_no_id():
    c = _FakeCtx()
    assert lvo.replicas.init_shard(c, None) == (0, 1)
    assert c.args == (0, 1, None)


class _FakePeerCtx:
    """Stands in for lvo.Context's device-exchange calls: a rank-stamped 64-byte handle; `fail` makes
    shard_peer_open raise like a refused IPC mapping."""
    def __init__(self, rank, fail=False):
        self.rank, self.fail = rank, fail
        self.opened, self.closed = None, False

    def shard_peer_handle(self):
        return bytes([self.rank + 1]) * 64

    def shard_peer_open(self, handles, rank):
        if self.fail:
            raise lvo.ALOAMError("hipIpcOpenMemHandle: invalid argument")
        self.opened = (list(handles), rank)

    def shard_peer_close(self):
        self.closed = True


def _peer_worker(rank, world, port, fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lvo_amd_loader import lvo as L
    c = _FakePeerCtx(rank, fail=rank == fail_rank)
    try:
        L.replicas.init_peer_exchange(c, dist)
        err = None
    except RuntimeError as e:
        err = str(e)
    q.put((rank, c.opened, c.closed, err))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_init_peer_exchange_over_gloo(fail_rank):
    """replicas.init_peer_exchange: every rank opens the world's handles in rank order; one rank's failed
    open makes EVERY rank close the exchange and raise (the bench then falls back to RCCL together)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_peer_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    handles = [bytes([r + 1]) * 64 for r in range(world)]
    if fail_rank < 0:
        assert [r[1] for r in res] == [(handles, r) for r in range(world)]
        assert all(r[3] is None and not r[2] for r in res)
    else:
        assert all(r[3] and "rank 1" in r[3] and r[2] for r in res)


def test_init_peer_exchange_single_process_opens_own_handle():
    """Without a process group the device exchange is world 1: the context's own handle, rank 0."""
    c = _FakePeerCtx(0)
    assert lvo.replicas.init_peer_exchange(c, None) == (0, 1)
    assert c.opened == ([bytes([1]) * 64], 0)
