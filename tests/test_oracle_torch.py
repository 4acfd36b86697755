"""Cross-check the oracle's hand-derived network backward against torch autograd (CPU, fp64):
an independent implementation of the same graph (networks.py / policy_v_network.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from oracle import nets


def torch_loss(spec, P, obs, a_idx, r_idx, y, adv, beta, act='relu', alpha=0.1):
    T = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in P.items()}
    lstm = spec.get('lstm')
    if lstm:  # [B, 5, 84, 84, C] memory windows -> 5B frames
        obs = obs.reshape((-1,) + obs.shape[2:])
    x = torch.tensor(obs, dtype=torch.float64) / 255.0
    x = x.permute(0, 3, 1, 2)
    for (name, k, s, cin, cout, pad, pool) in spec['convs']:
        W = T['Network/%s/%s_weights' % (name, name)].permute(3, 2, 0, 1)
        b = T['Network/%s/%s_biases' % (name, name)]
        if pad == 'SAME':
            H = x.shape[2]
            O = -(-H // s)
            tot = max((O - 1) * s + k - H, 0)
            x = Fn.pad(x, (tot // 2, tot - tot // 2, tot // 2, tot - tot // 2))
        x = Fn.conv2d(x, W, b, stride=s)
        x = torch.relu(x) if act == 'relu' else torch.maximum(x, alpha * x)
        if pool:
            x = Fn.max_pool2d(x, 2, 2)
    flat = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten (networks.py:14-17)
    if lstm:
        # torch.nn.LSTMCell (gate order i, f, g, o) with the TF kernel (i, j, f, o) mapped onto it
        # and forget_bias folded into b_ih: an independent restatement of BasicLSTMCell.
        nh, S = lstm['hidden'], lstm['steps']
        K, kb = T['rnn/basic_lstm_cell/kernel'], T['rnn/basic_lstm_cell/bias']
        nin = K.shape[0] - nh
        perm = torch.cat([torch.arange(0, nh), torch.arange(2 * nh, 3 * nh), torch.arange(nh, 2 * nh),
                          torch.arange(3 * nh, 4 * nh)])
        fb = torch.zeros(4 * nh, dtype=torch.float64)
        fb[nh:2 * nh] = lstm['forget_bias']
        X = flat.reshape(-1, S, nin)
        Bw = X.shape[0]
        h5 = torch.zeros(Bw, nh, dtype=torch.float64)
        c5 = torch.zeros(Bw, nh, dtype=torch.float64)
        for t in range(S):
            h5, c5 = torch._VF.lstm_cell(X[:, t], (h5, c5), K[:nin, perm].T, K[nin:, perm].T, kb[perm] + fb,
                                         torch.zeros(4 * nh, dtype=torch.float64))
        flat = h5 @ T['Network/lstm/Variable'] + T['Network/lstm/Variable_1']
    fc = spec['fc'][0]
    h = flat @ T['Network/%s/%s_weights' % (fc, fc)] + T['Network/%s/%s_biases' % (fc, fc)]
    h = torch.relu(h) if act == 'relu' else torch.maximum(h, alpha * h)
    v = (h @ T['Training/Critic/critic_output/critic_output_weights'] +
         T['Training/Critic/critic_output/critic_output_biases']).reshape(-1)
    pi = torch.softmax(h @ T['Training/Actor/actor_output/actor_output_weights'] +
                       T['Training/Actor/actor_output/actor_output_biases'], 1)
    rep = torch.softmax(h @ T['Training/Repetition/repetition_output/repetition_output_weights'] +
                        T['Training/Repetition/repetition_output/repetition_output_biases'], 1)
    lpi = torch.log(pi + 1e-30)
    lrep = torch.log(rep + 1e-30)
    ent = -(pi * lpi).sum(1) - (rep * lrep).sum(1)
    B = len(v)
    sel = lpi[torch.arange(B), torch.tensor(a_idx)] + lrep[torch.arange(B), torch.tensor(r_idx)]
    advt = torch.tensor(adv, dtype=torch.float64)
    yt = torch.tensor(y, dtype=torch.float64)
    loss = 5.0 * (torch.mean(-(sel * advt + beta * ent)) + torch.mean(0.25 * (yt - v) ** 2))
    loss.backward()
    return float(loss), {k: t.grad.numpy() for k, t in T.items()}


@pytest.mark.parametrize('arch,depth,A,R,act', [('NIPS', 1, 6, 1, 'relu'), ('NATURE', 1, 4, 11, 'relu'),
                                                ('NIPS', 3, 5, 3, 'leaky_relu'), ('PWYX', 1, 4, 11, 'relu'),
                                                ('LSTM', 1, 9, 11, 'relu'), ('LSTM', 1, 4, 1, 'leaky_relu')])
def test_oracle_backward_vs_autograd(arch, depth, A, R, act):
    spec = nets.arch_spec(arch, depth, A, R)
    P = {k: v.astype(np.float64) for k, v in nets.init_params(spec, 1).items()}
    if arch == 'LSTM':  # non-zero cell bias so every gate term is exercised
        P['rnn/basic_lstm_cell/bias'] = np.random.RandomState(3).uniform(-0.5, 0.5, 128)
    rs = np.random.RandomState(2)
    B = 3
    shape = (B, 5, 84, 84, 4 * depth) if arch == 'LSTM' else (B, 84, 84, 4 * depth)
    obs = rs.randint(0, 256, size=shape).astype(np.uint8)
    a_idx = rs.randint(0, A, B)
    r_idx = rs.randint(0, R, B)
    y = rs.randn(B)
    adv = rs.randn(B)
    loss, G, _ = nets.loss_and_grads(spec, P, obs, a_idx, r_idx, y, adv, 0.05, act=act)
    tl, TG = torch_loss(spec, P, obs, a_idx, r_idx, y, adv, 0.05, act=act)
    assert abs(loss - tl) < 1e-10 * max(1, abs(tl))
    for k in TG:
        np.testing.assert_allclose(G[k].reshape(TG[k].shape), TG[k], rtol=1e-8, atol=1e-12, err_msg=k)


@pytest.mark.parametrize('arch,A,R', [('NIPS', 6, 1), ('NATURE', 4, 11), ('LSTM', 9, 11)])
def test_cpu_baseline_network_matches_oracle(arch, A, R):
    """The timed CPU baseline's torch network (oracle/torch_cpu.py) computes the oracle's graph."""
    from oracle.torch_cpu import TorchCPUNetwork
    net = TorchCPUNetwork(arch, 1, A, R, seed=4, threads=2)
    rs = np.random.RandomState(5)
    shape = (2, 5, 84, 84, 4) if arch == 'LSTM' else (2, 84, 84, 4)
    obs = rs.randint(0, 256, size=shape).astype(np.uint8)
    v, pi, rep = net.forward(obs)
    P = {k: t.detach().numpy() for k, t in net.P.items()}
    v0, pi0, rep0, _ = nets.forward(net.spec, P, obs)
    np.testing.assert_allclose(v, v0, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(pi, pi0, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(rep, rep0, rtol=1e-4, atol=1e-6)


def test_window_frames_oracle_equals_explicit_windows():
    """nets.window_frames_loss_and_grads (each distinct frame through the trunk once, windows as
    frame indices, the zero frame included) == nets.loss_and_grads on the explicit [B][5] windows
    the reference feeds (paac.py:79-83, :233-234)."""
    spec = nets.arch_spec('LSTM', 1, 5, 3)
    P = nets.init_params(spec, 3)
    P['rnn/basic_lstm_cell/bias'] = np.random.RandomState(1).uniform(-0.5, 0.5, 128).astype(np.float32)
    rs = np.random.RandomState(4)
    F, B = 6, 4
    frames = rs.randint(0, 256, size=(F, 84, 84, 4)).astype(np.uint8)
    frames[0] = 0
    win = np.array([[0, 0, 1, 2, 3], [1, 2, 3, 4, 5], [0, 0, 0, 0, 5], [2, 3, 4, 5, 1]])
    a, r = rs.randint(0, 5, B), rs.randint(0, 3, B)
    y, adv = rs.randn(B), rs.randn(B)
    l0, G0, aux0 = nets.loss_and_grads(spec, P, frames[win], a, r, y, adv, 0.02)
    l1, G1, aux1 = nets.window_frames_loss_and_grads(spec, P, frames, win, a, r, y, adv, 0.02, chunk=4)
    assert abs(l0 - l1) <= 1e-12 * abs(l0)
    np.testing.assert_allclose(aux1['terms'], aux0['terms'], rtol=1e-12)
    for k in G0:
        np.testing.assert_allclose(G1[k], G0[k], rtol=1e-9, atol=1e-14, err_msg=k)


@pytest.mark.parametrize('arch,depth', [('NIPS', 1), ('PWYX', 3)])
def test_chunked_frames_oracle_equals_loss_and_grads(arch, depth):
    """Non-recurrent archs: nets.window_frames_loss_and_grads with one frame per row (win = [[n]],
    the trunk in chunks — how tests/test_e2e_gpu.py bounds the oracle's memory at N = 160 RGB PWYX
    rows) == nets.loss_and_grads on the whole batch."""
    spec = nets.arch_spec(arch, depth, 4, 11)
    P = nets.init_params(spec, 5)
    rs = np.random.RandomState(6)
    B = 5
    obs = rs.randint(0, 256, size=(B, 84, 84, 4 * depth)).astype(np.uint8)
    a, r = rs.randint(0, 4, B), rs.randint(0, 11, B)
    y, adv = rs.randn(B), rs.randn(B)
    l0, G0, aux0 = nets.loss_and_grads(spec, P, obs, a, r, y, adv, 0.05)
    l1, G1, aux1 = nets.window_frames_loss_and_grads(spec, P, obs, np.arange(B)[:, None], a, r, y, adv, 0.05,
                                                     chunk=2)
    assert abs(l0 - l1) <= 1e-12 * abs(l0)
    np.testing.assert_allclose(aux1['terms'], aux0['terms'], rtol=1e-12)
    for k in G0:
        np.testing.assert_allclose(G1[k], G0[k], rtol=1e-9, atol=1e-14, err_msg=k)


@pytest.mark.parametrize('arch', ['PWYX', 'NIPS'])
def test_oracle_follows_supplied_branches(arch):
    """nets.loss_and_grads with routes / branches / hbranch equal to the oracle's own decisions (a
    'device' whose stored outputs are the oracle's, through tests/parity_util.device_branches) gives
    the default gradient exactly; flipping one ReLU branch of the last conv changes it."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import parity_util
    spec = nets.arch_spec(arch, 1, 4, 3)
    P = nets.init_params(spec, 2)
    rs = np.random.RandomState(3)
    B = 3
    obs = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
    a, r = rs.randint(0, 4, B), rs.randint(0, 3, B)
    y, adv = rs.randn(B), rs.randn(B)
    flat, layers = nets.trunk_forward(spec, P, obs)
    dev = {}
    for L in layers:
        if L['pool']:
            dev[L['name']] = (L['yp'].astype(np.float32), nets.pool_route(L['y'])[0])
        else:
            dev[L['name']] = (L['y'].astype(np.float32), None)
    _, _, _, cache = nets.heads_forward(spec, P, flat)
    dev['H'] = cache['h'].astype(np.float32)
    br = parity_util.device_branches(spec, P, obs, dev)
    _, G0, _ = nets.loss_and_grads(spec, P, obs, a, r, y, adv, 0.02)
    _, G1, _ = nets.loss_and_grads(spec, P, obs, a, r, y, adv, 0.02, routes=br['routes'], branches=br['branches'],
                                   hbranch=br['hbranch'])
    for k in G0:
        np.testing.assert_array_equal(G1[k], G0[k], err_msg=k)
    last = layers[-1]['name']
    flip = {k: v.copy() for k, v in br['branches'].items()}
    idx = np.argwhere(flip[last])[0]
    flip[last][tuple(idx)] = False
    _, G2, _ = nets.loss_and_grads(spec, P, obs, a, r, y, adv, 0.02, routes=br['routes'], branches=flip,
                                   hbranch=br['hbranch'])
    assert not np.array_equal(G2['Network/%s/%s_weights' % (last, last)], G0['Network/%s/%s_weights' % (last, last)])
