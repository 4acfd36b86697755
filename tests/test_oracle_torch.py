"""Cross-check the oracle's hand-derived network backward against torch autograd (CPU, fp64):
an independent implementation of the same graph (networks.py / policy_v_network.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from oracle import nets


def torch_loss(spec, P, obs, a_idx, r_idx, y, adv, beta, act='relu', alpha=0.1):
    T = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in P.items()}
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
                                                ('NIPS', 3, 5, 3, 'leaky_relu'), ('PWYX', 1, 4, 11, 'relu')])
def test_oracle_backward_vs_autograd(arch, depth, A, R, act):
    spec = nets.arch_spec(arch, depth, A, R)
    P = {k: v.astype(np.float64) for k, v in nets.init_params(spec, 1).items()}
    rs = np.random.RandomState(2)
    B = 3
    obs = rs.randint(0, 256, size=(B, 84, 84, 4 * depth)).astype(np.uint8)
    a_idx = rs.randint(0, A, B)
    r_idx = rs.randint(0, R, B)
    y = rs.randn(B)
    adv = rs.randn(B)
    loss, G, _ = nets.loss_and_grads(spec, P, obs, a_idx, r_idx, y, adv, 0.05, act=act)
    tl, TG = torch_loss(spec, P, obs, a_idx, r_idx, y, adv, 0.05, act=act)
    assert abs(loss - tl) < 1e-10 * max(1, abs(tl))
    for k in TG:
        np.testing.assert_allclose(G[k].reshape(TG[k].shape), TG[k], rtol=1e-8, atol=1e-12, err_msg=k)
