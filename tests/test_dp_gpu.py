"""Stream ordering of the data-parallel update on one GPU.

paac._bucketed_update replays the backward as two graphs split at the launch that completes the
dense / head gradients (mt_net_backward_bucket_launches) and all-reduces the two gradient buckets
on a side stream between them, ordered by events e1 / e2 / e3; the apply graph waits for both.
At world 1 RCCL's in-place sum is the identity, so an ordering bug would leave the result
unchanged. Here the communicator is a stub that sleeps on the side stream (so a consumer that does
not wait runs first) and then doubles its bucket — a two-rank sum of identical replicas — with
the learner's 1/world fold set to 1/2. Every value of the run must then be bit-identical to the
same learner with the RCCL communicator (a bucket doubled too early or too late, or an apply that
does not wait, changes the gradient's direction, which the global-norm clip does not hide), and the
dense / head bucket must already hold its final gradient when its all-reduce starts.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

UPDATES = 5


class SlowDoublingComm(object):
    """Side-stream all-reduce stand-in: spin ~1 ms, snapshot the bucket, then sum it with an
    identical replica (x2)."""
    kind = 'stub'
    capturable = False

    def __init__(self):
        self.snaps = []

    def allreduce(self, t):
        torch.cuda._sleep(2_000_000)
        self.snaps.append((t.data_ptr(), t.clone()))
        t.mul_(2.0)

    def broadcast(self, t, root=0):
        pass

    def close(self):
        pass


def _run(config, tmp_path, stub):
    import bench
    L, _ = bench.make_learner(config, debugging_folder=str(tmp_path) + '/', episode_len=13, dp_force=True)
    L.start()
    try:
        assert L.dp and L.comm.kind == 'rccl'
        if stub is not None:
            L.comm.close()
            L.comm = stub
            L.grad_scale = 0.5
        for _ in range(UPDATES):
            L.book.new_update()
            L.rollout()
            L.update()
        torch.cuda.synchronize()
        native = getattr(L.comm, '_h', None) is not None
        one = native and os.environ.get('MT_DP_ONE_GRAPH', '1') != '0'
        # C-ABI communicators: the rollout's last step launches the whole update — one captured graph
        # (paac._dp_sequence) or the three graphs with the all-reduces between them
        # (mt_rollout_set_update_dp); a Python one: the first graph, the learner the rest
        assert L._buckets is not None and len(L._graphs) == (1 if one else 3) and L._update_in_rollout
        assert L._rollout_update == ('all' if native else 'first')
        c = lambda t: t.detach().cpu().numpy().copy()
        return dict(params=c(L.network.params), ms=c(L.network.ms), mom=c(L.network.mom), grad=c(L.network.grad),
                    states=c(L.states), values=c(L.values), y=c(L.y), idx=L.idx_h.numpy().copy(),
                    gs=L.global_step, split=L._buckets, grad_ptr=L.network.grad.data_ptr())
    finally:
        L.cleanup()


@pytest.mark.parametrize('config', ['pong-nips', 'seaquest-nature'])
def test_bucketed_update_stream_order(config, tmp_path):
    """The Python form of the bucketed update (the learner issues the all-reduces and graphs 2 and 3;
    a Python communicator), against the RCCL run (the native form)."""
    ref = _run(config, tmp_path / 'rccl', None)
    stub = SlowDoublingComm()
    got = _run(config, tmp_path / 'stub', stub)
    for k in ('params', 'ms', 'mom', 'states', 'values', 'y', 'idx'):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert got['gs'] == ref['gs']
    # the gradient itself: the all-reduced sum of two identical replicas
    np.testing.assert_array_equal(got['grad'], 2.0 * ref['grad'])
    # the last update's two all-reduces: the dense / head bucket first, then the conv bucket, each
    # already holding its final gradient (nothing wrote it after its all-reduce started)
    k = got['split']
    (p1, b1), (p2, b2) = stub.snaps[-2], stub.snaps[-1]
    assert p1 == got['grad_ptr'] + 4 * k and p2 == got['grad_ptr']
    np.testing.assert_array_equal(b1.cpu().numpy(), ref['grad'][k:])
    np.testing.assert_array_equal(b2.cpu().numpy(), ref['grad'][:k])


@pytest.mark.parametrize('config,one_graph', [('pong-nips', True), ('seaquest-nature', True), ('pong-nips', False)])
def test_native_bucketed_update_stream_order(config, one_graph, tmp_path, monkeypatch):
    """The native forms — one graph with the all-reduce stream forked and joined inside it
    (paac._dp_sequence), or the three graphs with the all-reduces enqueued between them by the
    rollout (mt_rollout_set_update_dp; MT_DP_ONE_GRAPH=0) — with the loopback communicator of the C
    ABI (mt_comm_init_loopback: the bucket doubled at once — a sum that started before its producer
    finished would be overwritten — then its stream held ~2 ms, so a consumer that does not wait
    runs first): every value bit-identical to the RCCL run, the gradient doubled."""
    from manette_amd.comm import LoopbackComm
    monkeypatch.setenv('MT_DP_ONE_GRAPH', '1' if one_graph else '0')
    ref = _run(config, tmp_path / 'rccl', None)
    got = _run(config, tmp_path / 'loopback', LoopbackComm(replicas=2, delay_us=2000))
    for k in ('params', 'ms', 'mom', 'states', 'values', 'y', 'idx'):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert got['gs'] == ref['gs']
    np.testing.assert_array_equal(got['grad'], 2.0 * ref['grad'])


def test_rollout_update_registration_order(tmp_path):
    """mt_rollout_set_update / _set_update_dp: registering either form replaces the
    other; unregistering with mt_rollout_set_update(NULL) clears both (a step must never launch a
    data-parallel update whose LR word was just unregistered); _set_update_dp(NULL) clears only the
    data-parallel form."""
    import ctypes as C
    import bench
    from manette_amd import _lib
    L, _ = bench.make_learner('pong-nips', debugging_folder=str(tmp_path) + '/', episode_len=13)
    L.start()
    lib = _lib.hip()
    form = C.c_int(-1)

    def current():
        _lib.check(lib.mt_rollout_update_form(L.native_step, C.byref(form)), 'mt_rollout_update_form')
        return form.value
    try:
        for _ in range(3):
            L.book.new_update()
            L.rollout()
            L.update()
        torch.cuda.synchronize()
        assert L._update_in_rollout and current() == 1
        g = L._graphs[0]
        g = g.value if isinstance(g, C.c_void_p) else g
        lr = C.c_void_p(L.network._lr_host.data_ptr())
        grad = L.network.grad
        from manette_amd.comm import LoopbackComm
        comm = LoopbackComm(replicas=1, delay_us=0)
        try:
            gs = (C.c_void_p * 3)(g, g, g)  # (registered only: nothing is launched here)
            _lib.check(lib.mt_rollout_set_update_dp(L.native_step, gs, comm._h, C.c_void_p(grad.data_ptr()),
                                                    grad.numel(), 16, lr, 0.0224, 8e7), 'set_update_dp')
            assert current() == 2
            _lib.check(lib.mt_rollout_set_update(L.native_step, None, None, 0.0, 0.0), 'set_update(NULL)')
            assert current() == 0  # both forms cleared
            _lib.check(lib.mt_rollout_set_update(L.native_step, g, lr, 0.0224, 8e7), 'set_update')
            assert current() == 1
            _lib.check(lib.mt_rollout_set_update_dp(L.native_step, None, None, None, 0, 0, None, 0.0, 0.0),
                       'set_update_dp(NULL)')
            assert current() == 1  # the single form stays
            _lib.check(lib.mt_rollout_set_update_dp(L.native_step, gs, comm._h, C.c_void_p(grad.data_ptr()),
                                                    grad.numel(), 16, lr, 0.0224, 8e7), 'set_update_dp')
            assert current() == 2  # replaces the single form
            _lib.check(lib.mt_rollout_set_update(L.native_step, g, lr, 0.0224, 8e7), 'set_update')
            assert current() == 1
        finally:
            comm.close()
        # the registered single-process update still runs the learner's rollout + update
        L.book.new_update()
        L.rollout()
        L.update()
        torch.cuda.synchronize()
    finally:
        L.cleanup()
