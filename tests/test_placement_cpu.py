"""Host-thread placement of the data-parallel ranks (manette_amd/placement.py) and the bounded
communicator setup (manette_amd/comm.Deadline), on CPU. The reference starts `ew` emulator
processes per learner and leaves placement to the OS (runners.py:11-18); with one process per GPU,
eight ranks on one node start 8 x (ew + 1) busy threads, so each rank plans which cores its
threads take and caps ew when the node's cores cannot hold them."""
import os
import subprocess
import sys

import numpy as np
import pytest

from manette_amd import placement as pl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpulist_round_trip():
    for text, cpus in (('0-3,8,10-11', [0, 1, 2, 3, 8, 10, 11]), ('5', [5]), ('0-127', list(range(128)))):
        assert pl.parse_cpulist(text) == cpus
        assert pl.format_cpulist(cpus) == text


def _eight_gpu_node(allowed=range(128), quota=None):
    """8 GPUs, 4 per NUMA node, 64 cpus per node (a typical 2-socket MI355X host)."""
    return dict(allowed=list(allowed), quota=quota, node_of_rank=[0, 0, 0, 0, 1, 1, 1, 1],
                node_cpus={0: list(range(64)), 1: list(range(64, 128))})


def test_eight_ranks_get_disjoint_slices_on_their_gpus_node():
    topo = _eight_gpu_node()
    plans = [pl.plan(8, 32, r, 8, **topo) for r in range(8)]
    seen = set()
    for r, p in enumerate(plans):
        cpus = pl.parse_cpulist(p['cpus'])
        assert len(cpus) == 16 and p['cores_per_rank'] == 16
        node = topo['node_of_rank'][r]
        assert set(cpus) <= set(topo['node_cpus'][node])  # next to its GPU's PCIe root
        assert not (set(cpus) & seen)                     # no core shared with another rank
        seen |= set(cpus)
        assert p['sliced'] and not p['pinned'] and not p['oversubscribed'] and p['ew_used'] == 8
        assert p['spin_us'] == pl.SPIN_US and p['worker_cpus'] == [] and p['main_cpus'] == cpus
        q = pl.plan(8, 32, r, 8, mode='pin', **topo)  # one cpu per thread
        assert q['pinned'] and len(q['worker_cpus']) == 8 and len(set(q['worker_cpus'])) == 8
        assert set(q['worker_cpus']) <= set(cpus) and q['main_cpus'][0] not in q['worker_cpus']
        assert set(q['main_cpus']) | set(q['worker_cpus']) == set(cpus)
    assert len(seen) == 128


def test_oversubscribed_node_caps_ew_and_shortens_the_spin():
    # 32 allowed cpus for 8 ranks: 4 each, so ew 8 -> 3 (3 workers + the host thread)
    plans = [pl.plan(8, 32, r, 8, **_eight_gpu_node(allowed=list(range(16)) + list(range(64, 80)))) for r in range(8)]
    for p in plans:
        assert p['cores_per_rank'] == 4 and p['oversubscribed'] and p['sliced']
        assert p['ew_used'] == 3 and p['threads_per_rank'] == 4 and p['spin_us'] == pl.SPIN_US_OVERSUB
        assert len(p['main_cpus']) == 4
    # the container's quota binds before the slice: 16 cpus' worth for 8 ranks -> 2 each -> ew 1
    p = pl.plan(8, 32, 5, 8, **_eight_gpu_node(quota=16.0))
    assert p['cores_per_rank'] == 2 and p['ew_used'] == 1 and p['oversubscribed']


def test_single_rank_auto_leaves_the_scheduler_alone():
    p = pl.plan(8, 32, 0, 1, allowed=list(range(8)), quota=None)
    assert not p['pinned'] and not p['sliced'] and p['placement'] == 'off'
    assert p['ew_used'] == 8 and p['worker_cpus'] == [] and p['main_cpus'] == []
    assert p['oversubscribed'] and p['spin_us'] == pl.SPIN_US  # (reported, not acted on)
    p = pl.plan(8, 32, 0, 1, allowed=list(range(16)), quota=None, mode='on')  # ('on' = 'pin')
    assert p['pinned'] and p['ew_used'] == 8 and len(p['worker_cpus']) == 8
    p = pl.plan(8, 32, 0, 1, allowed=list(range(16)), quota=None, mode='slice')
    assert p['sliced'] and p['main_cpus'] == list(range(16)) and p['ew_used'] == 8
    p = pl.plan(8, 32, 3, 8, mode='off', **_eight_gpu_node())
    assert not p['pinned'] and not p['sliced'] and p['ew_used'] == 8


def test_unknown_topology_splits_the_allowed_cpus():
    plans = [pl.plan(2, 4, r, 4, allowed=list(range(12)), node_of_rank=[None] * 4) for r in range(4)]
    slices = [pl.parse_cpulist(p['cpus']) for p in plans]
    assert slices == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11]]
    assert all(p['ew_used'] == 2 and not p['oversubscribed'] for p in plans)
    # ew never exceeds the env count (the runner's W = min(ew, E))
    assert pl.plan(8, 3, 0, 2, allowed=list(range(16)))['ew_used'] == 3


def test_native_runner_pinned_workers_step_identically():
    """mh_runner_set_threads pins each worker (mh_runner_thread_cpus reads it back) and changes
    nothing the runner computes."""
    from manette_amd.environment import COL_LUT, ROW_LUT
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    from oracle import policy as opol
    tab = opol.tab_repetitions(10, 11)
    allowed = sorted(os.sched_getaffinity(0))
    bank = SyntheticBank(2, 6, episode_len=7)
    kw = dict(row_select=ROW_LUT, fixed_slots=True, resized=True, col_lut=COL_LUT)
    a, b = NativeRunners(bank, 3, tab, **kw), NativeRunners(bank, 3, tab, **kw)
    try:
        cpus = [allowed[i % len(allowed)] for i in (1, 2, 3)]
        b.set_threads(cpus, spin_us=50)
        assert b.thread_cpus() == cpus
        assert all(c == -1 or c in allowed for c in a.thread_cpus())
        na, nb = a.reset(), b.reset()
        rs = np.random.RandomState(1)
        for _ in range(10):
            assert na == nb
            np.testing.assert_array_equal(a.staging.numpy(), b.staging.numpy())
            np.testing.assert_array_equal(a.push_meta.numpy(), b.push_meta.numpy())
            act, rep = rs.randint(0, 6, 6).astype(np.int32), rs.randint(0, 11, 6).astype(np.int32)
            na, nb = a.step(act, rep), b.step(act, rep)
            np.testing.assert_array_equal(a.reward.numpy(), b.reward.numpy())
            np.testing.assert_array_equal(a.over.numpy(), b.over.numpy())
        with pytest.raises(RuntimeError):
            b.set_threads([-1])
    finally:
        a.stop()
        b.stop()


def _run(code):
    return subprocess.run([sys.executable, '-c', code], cwd=ROOT, capture_output=True, text=True, timeout=60)


def test_deadline_exits_nonzero_with_a_message():
    r = _run('import time\nfrom manette_amd.comm import Deadline\n'
             'with Deadline("the test collective", 2, 8, seconds=0.5):\n    time.sleep(20)\n')
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert 'the test collective did not complete within 0 s on rank 2 of 8' in r.stderr


def test_deadline_is_silent_when_the_block_finishes():
    r = _run('import time\nfrom manette_amd.comm import Deadline\n'
             'with Deadline("x", seconds=5.0) as d:\n    time.sleep(0.05)\nprint("done %.2f" % d.elapsed)\n')
    assert r.returncode == 0 and r.stdout.startswith('done') and r.stderr == ''
