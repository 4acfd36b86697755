"""bench.settle_updates at world 2 and 8 (gloo, CPU): every rank runs the same number of untimed updates,
whatever its own clock says. Each fake update all-reduces like the data-parallel update does; ranks
that stopped on their own clocks drifted by one update and hung in mismatched collectives (the
round-5 2-rank rehearsal)."""
import os
import random
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, seconds, out):
    sys.path.insert(0, ROOT)
    import bench
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    rng = random.Random(rank)
    calls = [0]

    def one_update():  # uneven per-rank work, then the update's collective
        time.sleep(rng.uniform(0.0, 0.004) * (1 + rank))
        t = torch.ones(4)
        dist.all_reduce(t)
        assert float(t[0]) == world
        calls[0] += 1

    n = bench.settle_updates(one_update, seconds, world, dist)
    # a collective after the loop: hangs (timeout) if the ranks ran different counts
    c = torch.tensor([n], dtype=torch.int64)
    dist.all_reduce(c, op=dist.ReduceOp.MAX)
    out[rank] = (n, calls[0], int(c.item()))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize('world', [2, 8])  # 8: the driver's N-GPU run (one gloo rank per GPU)
def test_settle_updates_same_count_on_every_rank(world):
    port = 29000 + os.getpid() % 1000 + 7 * world
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, 0.3, out), nprocs=world, join=True)
    counts = [out[r] for r in range(world)]
    n0 = counts[0][0]
    assert n0 > 0
    for n, calls, mx in counts:
        assert n == calls == mx == n0


def test_settle_updates_single_process():
    sys.path.insert(0, ROOT)
    import bench
    calls = []
    n = bench.settle_updates(lambda: calls.append(time.sleep(0.001)), 0.05, 1, None)
    assert n == len(calls) > 0
    assert bench.settle_updates(lambda: calls.append(1), 0.0, 1, None) == 0
