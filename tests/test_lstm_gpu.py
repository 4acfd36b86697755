"""LSTM arch (networks.py:227-258) on the device vs the float64 oracle, through the C ABI.

obs are memory windows [B][5][84][84][4*depth] (paac.py:79-83). Tolerances as the other
arches: forward 2e-5 relative, gradients 2e-4 relative L2 per variable (the cell kernel's
dot products run over K = 6432). With tens of frames the fp64 oracle finds a few max-pool
windows whose top two values differ by < 1e-6 relative; fp32 rounding may route such a
window's gradient to the other position (MaxPoolGrad is discontinuous there), which moves the
weight gradients of the pooled convs (conv1-3) by ~1e-3 relative L2 per flip. Those variables
are checked at 5e-3 when the oracle counts such near-ties (still far below any indexing or
layout error, which is O(1)); every other variable, and every variable when there is no
near-tie, at 2e-4.
The LSTM's TF1 kernel arithmetic is parity-unpinned (no LSTM checkpoint, TF absent): the
oracle restates BasicLSTMCell and is itself checked against torch's LSTM cell in
tests/test_oracle_torch.py.
"""
import numpy as np
import pytest
import torch

from oracle import nets

pytestmark = pytest.mark.gpu


def _net(depth, A, R, seed, act='relu'):
    from manette_amd.network import DeviceNetwork
    conf = dict(arch='LSTM', rgb=depth == 3, num_actions=A, nb_choices=R, softmax_temp=1.0,
                entropy_regularisation_strength=0.02, clip_norm=3.0, clip_norm_type='global',
                activation=act, alpha_leaky_relu=0.1)
    net = DeviceNetwork(conf)
    net.init_params(seed)
    # non-zero cell bias so every gate term is exercised (TF initialises it to zero)
    P = net.get_variables()
    P['rnn/basic_lstm_cell/bias'] = np.random.RandomState(seed).uniform(-0.5, 0.5, 128).astype(np.float32)
    net.set_variables(P)
    return net


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-12))


def _windows(rs, B, depth, zero_frac=0.3):
    obs = rs.randint(0, 256, size=(B, 5, 84, 84, 4 * depth)).astype(np.uint8)
    # zeroed leading frames, as after an episode end (paac.py:202-203)
    for b in range(B):
        k = rs.randint(0, 5) if rs.rand() < zero_frac else 0
        obs[b, :k] = 0
    return obs


@pytest.mark.parametrize('depth,A,R,act', [(1, 9, 11, 'relu'), (3, 4, 1, 'relu'), (1, 6, 3, 'leaky_relu')])
@pytest.mark.parametrize('B', [1, 6, 33])
def test_lstm_forward_parity(depth, A, R, act, B):
    net = _net(depth, A, R, seed=B, act=act)
    rs = np.random.RandomState(B)
    obs = _windows(rs, B, depth)
    v, pi, rep = net.forward(torch.from_numpy(obs).cuda())
    v2, pi2, rep2 = [t.clone() for t in net.forward(torch.from_numpy(obs).cuda(), infer=True, ws_key='i')]
    torch.cuda.synchronize()
    spec = nets.arch_spec('LSTM', depth, A, R)
    v0, pi0, rep0, _ = nets.forward(spec, net.get_variables(), obs, act=act, alpha=0.1)
    np.testing.assert_allclose(v.cpu().numpy(), v0, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy(), pi0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rep.cpu().numpy(), rep0, rtol=2e-5, atol=1e-6)
    np.testing.assert_array_equal(v2.cpu().numpy(), v.cpu().numpy())
    np.testing.assert_array_equal(pi2.cpu().numpy(), pi.cpu().numpy())


@pytest.mark.parametrize('depth,A,R,act', [(1, 9, 11, 'relu'), (3, 4, 1, 'relu'), (1, 6, 3, 'leaky_relu')])
@pytest.mark.parametrize('B', [4, 9, 32])
def test_lstm_loss_backward_parity(depth, A, R, act, B):
    net = _net(depth, A, R, seed=7 + B, act=act)
    rs = np.random.RandomState(100 + B)
    obs = _windows(rs, B, depth)
    a_idx = rs.randint(0, A, size=B).astype(np.int32)
    r_idx = rs.randint(0, R, size=B).astype(np.int32)
    y = rs.randn(B).astype(np.float32)
    adv = rs.randn(B).astype(np.float32)
    d = lambda x: torch.from_numpy(x).cuda()
    obs_d = d(obs)
    v, pi, rep = net.forward(obs_d)
    terms = torch.zeros(B, 4, device='cuda')
    net.loss_backward(obs_d, B, v, pi, rep, d(a_idx), d(r_idx), d(y), d(adv), loss_terms=terms)
    torch.cuda.synchronize()
    spec = nets.arch_spec('LSTM', depth, A, R)
    import parity_util  # the device's branches at the discontinuities (checked away from near-ties)
    P = net.get_variables()
    frames = obs.reshape((-1,) + obs.shape[2:])
    br = parity_util.device_branches(spec, P, frames, net.forward_branches(net.workspace(B), 2, B), act)
    loss, G, aux = nets.loss_and_grads(spec, P, obs, a_idx, r_idx, y, adv, 0.02, act=act, alpha=0.1,
                                       routes=br['routes'], branches=br['branches'], hbranch=br['hbranch'])
    got = net.get_variables('grad')
    parity_util.check_grads(spec, got, G, set())
    np.testing.assert_allclose(terms.cpu().numpy(), aux['terms'], rtol=1e-4, atol=1e-5)
    flat = net.grad.cpu().numpy()
    mask = np.ones(net.nparams, bool)
    for _, shape, off, _ in net.vars:
        mask[off:off + int(np.prod(shape))] = False
    assert not flat[mask].any()


def _np_memory_push(memory, fresh, masks):
    """paac.py:79-83 update_memory, then :202-203 memory[e] = 0 for ended episodes."""
    whole = memory.copy()
    memory[:, :-1] = memory[:, 1:]
    memory[:, -1] = fresh
    memory[masks == 0] = 0
    return whole


@pytest.mark.parametrize('E,depth', [(1, 1), (7, 1), (32, 3)])
def test_memory_push_bit_exact(E, depth):
    from manette_amd.network import memory_push
    rs = np.random.RandomState(E)
    mem = rs.randint(0, 256, size=(E, 5, 84, 84, 4 * depth)).astype(np.uint8)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    mem_d = d(mem)
    whole_d = torch.zeros_like(mem_d)
    for step in range(4):
        fresh = rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)
        masks = (rs.rand(E) > 0.3).astype(np.float32)
        memory_push(mem_d, whole_d, d(fresh), d(masks))
        whole = _np_memory_push(mem, fresh, masks)
        np.testing.assert_array_equal(whole_d.cpu().numpy(), whole)
        np.testing.assert_array_equal(mem_d.cpu().numpy(), mem)


def _window_rows_store(nz, t, E):
    """Frame-store rows [E][5] of the windows of step t: 0 (the zero frame) for the nz leading
    positions, else 1 + (t + k) * E + e (slot t + k of env e)."""
    w = np.zeros((E, 5), np.int64)
    for e in range(E):
        for k in range(5):
            w[e, k] = 0 if k < nz[e] else 1 + (t + k) * E + e
    return w


def _windows_from_store(slots, nz, t):
    """Explicit windows [E][5] of step t from the frame store (the reference's memory array)."""
    E = slots.shape[1]
    w = np.zeros((E, 5) + slots.shape[2:], np.uint8)
    for e in range(E):
        for k in range(5):
            if k >= nz[e]:
                w[e, k] = slots[t + k, e]
    return w


@pytest.mark.parametrize('E,T,depth', [(3, 2, 1), (4, 5, 1), (2, 3, 3)])
def test_lstm_frame_store_parity(E, T, depth):
    """mt_lstm_frames_forward / _windows_forward / _frames_backward on a frame store with random
    window zero-prefixes == the oracle on the explicit windows (paac.py:79-83 layout)."""
    A, R, act = 9, 11, 'relu'
    net = _net(depth, A, R, seed=E * 10 + T, act=act)
    rs = np.random.RandomState(E * 100 + T)
    C = 4 * depth
    fstore = rs.randint(0, 256, size=(1 + (T + 5) * E, 84, 84, C)).astype(np.uint8)
    fstore[0] = 0
    slots = fstore[1:].reshape(T + 5, E, 84, 84, C)
    nz = rs.choice([0, 0, 0, 1, 2, 4, 5], size=(T + 1, E)).astype(np.int32)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    fs_d, nz_d = d(fstore), d(nz)
    net.lstm_frames_forward(fs_d, 0, 1 + 5 * E, E, T)
    for t in range(1, T + 1):
        net.lstm_frames_forward(fs_d, 1 + (4 + t) * E, E, E, T)
    v = torch.zeros(T + 1, E, device='cuda')
    pi = torch.zeros(T + 1, E, A, device='cuda')
    rep = torch.zeros(T + 1, E, R, device='cuda')
    for t in range(T + 1):
        net.lstm_windows_forward(nz_d[t], t, E, T, out=(v[t], pi[t], rep[t]))
    torch.cuda.synchronize()
    spec = nets.arch_spec('LSTM', depth, A, R)
    P = net.get_variables()
    win = np.concatenate([_windows_from_store(slots, nz[t], t) for t in range(T + 1)])
    v0, pi0, rep0, _ = nets.forward(spec, P, win, act=act, alpha=0.1)
    np.testing.assert_allclose(v.cpu().numpy().reshape(-1), v0, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy().reshape(-1, A), pi0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rep.cpu().numpy().reshape(-1, R), rep0, rtol=2e-5, atol=1e-6)
    # train step over the T*E windows of steps 0..T-1
    N = T * E
    a_idx = rs.randint(0, A, size=N).astype(np.int32)
    r_idx = rs.randint(0, R, size=N).astype(np.int32)
    y = rs.randn(N).astype(np.float32)
    adv = rs.randn(N).astype(np.float32)
    terms = torch.zeros(N, 4, device='cuda')
    net.lstm_frames_backward(fs_d, nz_d[:T], E, T, pi[:T], rep[:T], v[:T], d(a_idx), d(r_idx), d(y), d(adv),
                             loss_terms=terms)
    torch.cuda.synchronize()
    wt = win[:N]
    import parity_util  # the distinct frames' branches, gathered per window position
    rows = np.concatenate([_window_rows_store(nz[t], t, E) for t in range(T)])
    br = parity_util.device_branches(spec, P, fstore, net.forward_branches(net.lstm_workspace(E, T), 1, E, T), act,
                                     win=rows)
    _, G, aux = nets.loss_and_grads(spec, P, wt, a_idx, r_idx, y, adv, 0.02, act=act, alpha=0.1,
                                    routes={k: v[rows.reshape(-1)] for k, v in br['routes'].items()},
                                    branches={k: v[rows.reshape(-1)] for k, v in br['branches'].items()},
                                    hbranch=br['hbranch'])
    got = net.get_variables('grad')
    parity_util.check_grads(spec, got, G, set())
    np.testing.assert_allclose(terms.cpu().numpy(), aux['terms'], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('E,T,depth', [(4, 5, 1), (3, 2, 3)])
def test_lstm_step_forward_xsum_cache_bit_exact(E, T, depth):
    """mt_lstm_step_forward's per-frame x-product sums (step 0 stores every frame's, steps t > 0 read
    the four older window positions from the cache, lstm.h XS) give exactly what the uncached
    mt_lstm_windows_forward computes from the slabs — over two rollouts with a parameter change
    between them (the cache is rebuilt at step 0), episode ends inside the rollout and leading
    zero frames."""
    A, R = 9, 11
    net = _net(depth, A, R, seed=7 * E + T)
    rs = np.random.RandomState(31 * E + T)
    C = 4 * depth
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    for rollout in range(2):
        fstore = rs.randint(0, 256, size=(1 + (T + 5) * E, 84, 84, C)).astype(np.uint8)
        fstore[0] = 0
        fs_d = d(fstore)
        nz = np.zeros((T + 1, E), np.int32)
        nz[0] = rs.choice([0, 0, 2, 5], size=E)
        over = rs.rand(T + 1, E) < 0.3  # step t-1's episode ends, read by step t
        nz_d = d(nz)
        over_d = d(over.astype(np.float32))
        got = [tuple(torch.zeros(*sh, device='cuda') for sh in ((E,), (E, A), (E, R))) for _ in range(T + 1)]
        for t in range(T + 1):
            net.lstm_step_forward(fs_d, t, E, T, nz_d, over_d[t - 1] if t > 0 else None, out=got[t])
        torch.cuda.synchronize()
        # the uncached windows over the same frame store (every row's x-product is in the workspace)
        # and the nz the steps derived on the device
        nz_dev = nz_d.clone()
        for t in range(T + 1):
            ref = tuple(torch.zeros(*sh, device='cuda') for sh in ((E,), (E, A), (E, R)))
            net.lstm_windows_forward(nz_dev[t].contiguous(), t, E, T, out=ref)
            torch.cuda.synchronize()
            for a, b in zip(got[t], ref):
                np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
        if rollout == 0:  # new parameters: the next rollout's step 0 must rebuild the cache
            with torch.no_grad():
                net.params.mul_(0.97).add_(0.001)


@pytest.mark.parametrize('pipeline', [True, False])
def test_lstm_learner_memory_windows(tmp_path, pipeline):
    """The learner's LSTM windows (frame store + nz, read at every step and by the train
    step) equal a numpy replay of the reference's memory bookkeeping (paac.py:107-112, :173-174,
    :202-203, :233-234) over the recorded states and episode-end masks, with resets inside the
    rollout and across updates; the LSTM update runs and changes the parameters. The learner runs
    the native macro-step (mt_rollout with the frame-store forward; nz derived on the device from
    the emulators' episode-end flags), pipelined (bootstrap in the rollout's last chain, update
    replayed as a hipGraph from the second update on) or not (bootstrap in the update)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import train as cli
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.paac import PAACLearner
    from manette_amd.synthetic import SyntheticBank
    a = cli.get_arg_parser().parse_args([])
    a.game, a.arch, a.emulator_counts, a.emulator_workers = 'ms_pacman', 'LSTM', 6, 2
    a.max_repetition, a.nb_choices = 10, 11
    a.runner, a.sampling, a.seed = 'native', 'device', 0
    a.pipeline = pipeline
    a.debugging_folder = str(tmp_path) + '/'
    a.max_global_steps = 1 << 40
    a.checkpoint_interval = 1 << 40
    np.random.seed(1234)
    explo = ExplorationPolicy(a)
    nc, ec = cli.get_network_and_environment_creator(a, explo)
    ec.create_bank = lambda first, n: SyntheticBank(first, n, episode_len=9)
    L = PAACLearner(nc, ec, explo, a)
    L.start()
    assert L.native_step is not None and L.boot_in_rollout == pipeline
    try:
        E, T = 6, L.max_local_steps
        mem = np.zeros((E, 5, 84, 84, 4), np.uint8)
        mem[:, -1] = L.states[0].cpu().numpy()
        p0 = L.network.params.cpu().numpy().copy()
        resets = 0
        for u in range(3):
            L.book.new_update()
            for t in range(T):
                L.step(t)
            torch.cuda.synchronize()
            slots = L.slots.cpu().numpy()
            masks = L.masks_h.numpy().copy()
            resets += int((masks == 0).sum())
            nz = L.nz_d.cpu().numpy()
            L.update()  # (unpipelined: the bootstrap forward derives nz[T] here; then nz[0] <- nz[T])
            torch.cuda.synchronize()
            nz_after = L.nz_d.cpu().numpy()
            if not pipeline:
                nz[T] = nz_after[T]
            np.testing.assert_array_equal(nz_after[T], nz[T])
            np.testing.assert_array_equal(nz_after[0], nz[T])  # carried into the next rollout
            for t in range(T):
                np.testing.assert_array_equal(_windows_from_store(slots, nz[t], t), mem, err_msg='u%d t%d' % (u, t))
                _np_memory_push(mem, slots[4 + t + 1], masks[t])
            np.testing.assert_array_equal(_windows_from_store(slots, nz[T], T), mem)  # bootstrap window
        assert resets > 0
        assert (L._graphs is not None) == pipeline
        p1 = L.network.params.cpu().numpy()
        assert np.isfinite(p1).all() and not np.array_equal(p0, p1)
    finally:
        L.cleanup()


@pytest.mark.parametrize('E,T', [(8, 5), (5, 3)])
def test_lstm_frames_backward_norm_partials(E, T):
    """mt_lstm_frames_backward with norm_partials (the single-GPU LSTM update, paac.py's
    partials_ready path): the same gradient bit for bit as without, and the partials its last
    launch leaves add up to the global norm of that gradient (actor_learner.py:59-63; oracle:
    float64) — the small K_h / fc6 / head / projection gradients ride in conv4's grouped launch,
    so a partial summed before they were complete would show here, whether or not a clip fires."""
    from oracle import optim
    A, R, act, depth = 9, 11, 'relu', 1
    net = _net(depth, A, R, seed=E * 7 + T, act=act)
    rs = np.random.RandomState(E * 31 + T)
    fstore = rs.randint(0, 256, size=(1 + (T + 5) * E, 84, 84, 4 * depth)).astype(np.uint8)
    fstore[0] = 0
    nz = rs.choice([0, 0, 0, 1, 2, 4, 5], size=(T + 1, E)).astype(np.int32)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    fs_d, nz_d = d(fstore), d(nz)
    net.lstm_frames_forward(fs_d, 0, 1 + 5 * E, E, T)
    for t in range(1, T + 1):
        net.lstm_frames_forward(fs_d, 1 + (4 + t) * E, E, E, T)
    v = torch.zeros(T + 1, E, device='cuda')
    pi = torch.zeros(T + 1, E, A, device='cuda')
    rep = torch.zeros(T + 1, E, R, device='cuda')
    for t in range(T + 1):
        net.lstm_windows_forward(nz_d[t], t, E, T, out=(v[t], pi[t], rep[t]))
    N = T * E
    args = (d(rs.randint(0, A, size=N).astype(np.int32)), d(rs.randint(0, R, size=N).astype(np.int32)),
            d(rs.randn(N).astype(np.float32)), d(rs.randn(N).astype(np.float32)))
    net.grad.zero_()
    net.lstm_frames_backward(fs_d, nz_d[:T], E, T, pi[:T], rep[:T], v[:T], *args)
    g0 = net.grad.clone()
    net.grad.zero_()
    net.partials.fill_(float('nan'))
    net.lstm_frames_backward(fs_d, nz_d[:T], E, T, pi[:T], rep[:T], v[:T], *args, norm_partials=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(net.grad.cpu().numpy(), g0.cpu().numpy())
    norm = float(np.sqrt(net.partials.double().sum().item()))
    ref = optim.global_norm([g0.cpu().numpy()])
    assert np.isfinite(norm) and abs(norm - ref) <= 1e-5 * ref, (norm, ref)


def test_lstm_frames_backward_launch_by_launch():
    """Every launch of mt_lstm_frames_backward is numbered by the launch window (bench.py times the
    LSTM train pass launch by launch): the backward issued as windows [0, k) then [k, ...) leaves
    the same gradient, bit for bit, as one call, and the windows count every launch."""
    import ctypes as C
    from manette_amd import _lib
    E, T, A, R, depth = 6, 5, 9, 11, 1
    net = _net(depth, A, R, seed=77, act='relu')
    rs = np.random.RandomState(78)
    fstore = rs.randint(0, 256, size=(1 + (T + 5) * E, 84, 84, 4 * depth)).astype(np.uint8)
    fstore[0] = 0
    nz = rs.choice([0, 0, 1, 3, 5], size=(T + 1, E)).astype(np.int32)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    fs_d, nz_d = d(fstore), d(nz)
    net.lstm_frames_forward(fs_d, 0, 1 + 5 * E, E, T)
    for t in range(1, T + 1):
        net.lstm_frames_forward(fs_d, 1 + (4 + t) * E, E, E, T)
    v = torch.zeros(T + 1, E, device='cuda')
    pi = torch.zeros(T + 1, E, A, device='cuda')
    rep = torch.zeros(T + 1, E, R, device='cuda')
    for t in range(T + 1):
        net.lstm_windows_forward(nz_d[t], t, E, T, out=(v[t], pi[t], rep[t]))
    N = T * E
    args = (d(rs.randint(0, A, size=N).astype(np.int32)), d(rs.randint(0, R, size=N).astype(np.int32)),
            d(rs.randn(N).astype(np.float32)), d(rs.randn(N).astype(np.float32)))
    bwd = lambda: net.lstm_frames_backward(fs_d, nz_d[:T], E, T, pi[:T], rep[:T], v[:T], *args)
    lib = _lib.hip()
    net.grad.zero_()
    lib.mt_launch_window(0, -1)
    bwd()
    total = lib.mt_launch_window(-1, -1)
    g0 = net.grad.clone()
    assert total >= 9  # loss, BPTT, zero-frame partials, gather, d flat, 4 conv launches, the last slab sum
    for k in (1, 3, 5, total - 1):
        net.grad.zero_()
        lib.mt_launch_window(0, k)
        bwd()
        assert lib.mt_launch_window(k, -1) == total
        bwd()
        lib.mt_launch_window(-1, -1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(net.grad.cpu().numpy(), g0.cpu().numpy(), err_msg='split at %d' % k)
