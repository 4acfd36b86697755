"""Parity of every libmanette_hip.so kernel against the oracle, through the C ABI (GPU box).

Tolerances: integer/byte work (preprocess, returns from identical inputs, sampling indices)
bit-exact; fp32 network math vs the float64 oracle within 2e-5 relative (forward) and
2e-4 relative L2 per variable (gradients) — the fp32 accumulation-order budget for K <= 3136.
"""
import numpy as np
import pytest
import torch

from oracle import nets, optim, preprocess, returns

pytestmark = pytest.mark.gpu

# (NATURE 18 x 11: the largest head region, 62 KB staged in LDS by the heads and loss kernels —
# 3,888 quads, past the 2,048 the kernels hold in registers)
CONFIGS = [('NIPS', 1, 6, 1), ('NIPS', 3, 4, 11), ('NATURE', 1, 4, 11), ('NATURE', 3, 18, 1),
           ('PWYX', 1, 4, 11), ('PWYX', 3, 6, 1), ('NATURE', 1, 18, 11)]


def _net(arch, depth, A, R, seed=0, act='relu'):
    from manette_amd.network import DeviceNetwork
    conf = dict(arch=arch, rgb=depth == 3, num_actions=A, nb_choices=R, softmax_temp=1.0,
                entropy_regularisation_strength=0.02, clip_norm=3.0, clip_norm_type='global',
                activation=act, alpha_leaky_relu=0.1)
    net = DeviceNetwork(conf)
    net.init_params(seed)
    return net


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-12))


@pytest.mark.parametrize('arch,depth,A,R', CONFIGS)
@pytest.mark.parametrize('B', [3, 37])
def test_forward_parity(arch, depth, A, R, B):
    net = _net(arch, depth, A, R, seed=B)
    rs = np.random.RandomState(B)
    obs = rs.randint(0, 256, size=(B, 84, 84, 4 * depth)).astype(np.uint8)
    v, pi, rep = net.forward(torch.from_numpy(obs).cuda())
    torch.cuda.synchronize()
    spec = nets.arch_spec(arch, depth, A, R)
    P = net.get_variables()
    v0, pi0, rep0, _ = nets.forward(spec, P, obs)
    np.testing.assert_allclose(v.cpu().numpy(), v0, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy(), pi0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rep.cpu().numpy(), rep0, rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize('arch,depth,A,R,act', [('NIPS', 1, 6, 1, 'relu'), ('NIPS', 3, 4, 11, 'relu'),
                                                 ('NIPS', 1, 9, 11, 'leaky_relu'), ('NATURE', 1, 4, 11, 'relu')])
@pytest.mark.parametrize('B', [1, 7, 32, 33])
def test_forward_infer_parity(arch, depth, A, R, act, B):
    """mt_forward_infer (NIPS: the fused trunk, trunk_fused.h) vs the oracle, and vs mt_forward
    (the layered GEMM path) on the same rows. B = 32 takes the XCD-aware block mapping, 7/33 not."""
    net = _net(arch, depth, A, R, seed=11 + B, act=act)
    rs = np.random.RandomState(1000 + B)
    obs = rs.randint(0, 256, size=(B, 84, 84, 4 * depth)).astype(np.uint8)
    obs_d = torch.from_numpy(obs).cuda()
    v, pi, rep = [t.clone() for t in net.forward(obs_d, infer=True, ws_key='infer')]
    v1, pi1, rep1 = net.forward(obs_d)
    torch.cuda.synchronize()
    spec = nets.arch_spec(arch, depth, A, R)
    v0, pi0, rep0, _ = nets.forward(spec, net.get_variables(), obs, act=act, alpha=0.1)
    np.testing.assert_allclose(v.cpu().numpy(), v0, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy(), pi0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rep.cpu().numpy(), rep0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(v.cpu().numpy(), v1.cpu().numpy(), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy(), pi1.cpu().numpy(), rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize('act', ['relu', 'leaky_relu'])
def test_forward_infer_large_batch(act):
    """B >= 256 gray NIPS takes the persistent throughput trunk (trunk_fused.h
    nips_conv_persist_kernel: no conv1 recompute, 256 blocks walking the envs): vs the oracle and
    vs the layered GEMM path on the same 300 rows."""
    B = 300
    net = _net('NIPS', 1, 6, 1, seed=5, act=act)
    rs = np.random.RandomState(77)
    obs = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
    obs_d = torch.from_numpy(obs).cuda()
    v, pi, rep = [t.clone() for t in net.forward(obs_d, infer=True, ws_key='infer_big')]
    v1, pi1, rep1 = net.forward(obs_d)
    torch.cuda.synchronize()
    spec = nets.arch_spec('NIPS', 1, 6, 1)
    v0, pi0, rep0, _ = nets.forward(spec, net.get_variables(), obs, act=act, alpha=0.1)
    np.testing.assert_allclose(v.cpu().numpy(), v0, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy(), pi0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rep.cpu().numpy(), rep0, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(v.cpu().numpy(), v1.cpu().numpy(), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy(), pi1.cpu().numpy(), rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize('arch,depth,A,R', CONFIGS)
@pytest.mark.parametrize('B', [5, 40])
def test_loss_backward_parity(arch, depth, A, R, B):
    net = _net(arch, depth, A, R, seed=7 + B)
    rs = np.random.RandomState(100 + B)
    obs = rs.randint(0, 256, size=(B, 84, 84, 4 * depth)).astype(np.uint8)
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
    spec = nets.arch_spec(arch, depth, A, R)
    P = net.get_variables()
    loss, G, aux = nets.loss_and_grads(spec, P, obs, a_idx, r_idx, y, adv, 0.02)
    got = net.get_variables('grad')
    import parity_util  # per variable AND per output channel (a one-channel corruption)
    parity_util.check_grads(spec, got, G, set())
    np.testing.assert_allclose(terms.cpu().numpy(), aux['terms'], rtol=1e-4, atol=1e-5)
    # alignment padding of the flat gradient is zero
    flat = net.grad.cpu().numpy()
    mask = np.ones(net.nparams, bool)
    for _, shape, off, _ in net.vars:
        mask[off:off + int(np.prod(shape))] = False
    assert not flat[mask].any()


@pytest.mark.parametrize('arch,depth,A,R', [('NIPS', 1, 6, 1), ('NIPS', 3, 4, 11), ('NATURE', 1, 4, 11),
                                            ('PWYX', 1, 4, 11)])
@pytest.mark.parametrize('E,T', [(7, 3), (32, 2)])
def test_forward_rows_then_backward_only(arch, depth, A, R, E, T):
    """mt_forward_rows of T batches of E rows into one train workspace (the rollout), then
    mt_loss_backward on the T*E rows with NO forward (the update) == the oracle's gradients of
    the flattened batch; the per-step outputs == the oracle forward (NIPS: the fused trunk also
    writes its conv activations)."""
    net = _net(arch, depth, A, R, seed=40 + E)
    rs = np.random.RandomState(E * 10 + T)
    N = T * E
    obs = rs.randint(0, 256, size=(T, E, 84, 84, 4 * depth)).astype(np.uint8)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    obs_d = d(obs)
    tws = net.workspace(N, 'train_rows')
    v = torch.zeros(T, E, device='cuda')
    pi = torch.zeros(T, E, A, device='cuda')
    rep = torch.zeros(T, E, R, device='cuda')
    for t in range(T):
        net.forward_rows(obs_d[t], E, tws, N, t * E, out=(v[t], pi[t], rep[t]), ws_key='rows')
    a_idx = rs.randint(0, A, size=N).astype(np.int32)
    r_idx = rs.randint(0, R, size=N).astype(np.int32)
    y = rs.randn(N).astype(np.float32)
    adv = rs.randn(N).astype(np.float32)
    flat = obs_d.view(N, 84, 84, 4 * depth)
    net.loss_backward(flat, N, v.view(N), pi.view(N, A), rep.view(N, R), d(a_idx), d(r_idx), d(y), d(adv),
                      ws_key='train_rows')
    torch.cuda.synchronize()
    spec = nets.arch_spec(arch, depth, A, R)
    P = net.get_variables()
    obs_n = obs.reshape(N, 84, 84, 4 * depth)
    v0, pi0, rep0, _ = nets.forward(spec, P, obs_n)
    np.testing.assert_allclose(v.cpu().numpy().reshape(-1), v0, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(pi.cpu().numpy().reshape(N, A), pi0, rtol=2e-5, atol=1e-6)
    _, G, _ = nets.loss_and_grads(spec, P, obs_n, a_idx, r_idx, y, adv, 0.02)
    import parity_util  # the device's branches at the discontinuities (checked away from near-ties)
    br = parity_util.device_branches(spec, P, obs_n, net.forward_branches(tws, 0, N))
    _, G, _ = nets.loss_and_grads(spec, P, obs_n, a_idx, r_idx, y, adv, 0.02, routes=br['routes'],
                                  branches=br['branches'], hbranch=br['hbranch'])
    parity_util.check_grads(spec, net.get_variables('grad'), G, set())


def test_leaky_relu_backward():
    net = _net('NIPS', 1, 6, 3, seed=3, act='leaky_relu')
    rs = np.random.RandomState(3)
    B = 9
    obs = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
    a_idx = rs.randint(0, 6, size=B).astype(np.int32)
    r_idx = rs.randint(0, 3, size=B).astype(np.int32)
    y = rs.randn(B).astype(np.float32)
    adv = rs.randn(B).astype(np.float32)
    d = lambda x: torch.from_numpy(x).cuda()
    v, pi, rep = net.forward(d(obs))
    net.loss_backward(d(obs), B, v, pi, rep, d(a_idx), d(r_idx), d(y), d(adv))
    spec = nets.arch_spec('NIPS', 1, 6, 3)
    _, G, _ = nets.loss_and_grads(spec, net.get_variables(), obs, a_idx, r_idx, y, adv, 0.02,
                                  act='leaky_relu', alpha=0.1)
    import parity_util
    parity_util.check_grads(spec, net.get_variables('grad'), G, set())


@pytest.mark.parametrize('T,E', [(5, 4), (5, 32), (20, 1000)])
def test_returns_bit_exact(T, E):
    from manette_amd.network import returns as dev_returns
    rs = np.random.RandomState(T * E)
    r = rs.choice([-1.0, 0.0, 1.0], size=(T, E)).astype(np.float32)
    m = (rs.rand(T, E) > 0.1).astype(np.float32)
    V = rs.randn(T, E).astype(np.float32)
    VT = rs.randn(E).astype(np.float32)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    y = torch.empty(T, E, device='cuda')
    adv = torch.empty(T, E, device='cuda')
    dev_returns(d(r), d(m), d(V), d(VT), 0.99, y, adv)
    y0, adv0 = returns.nstep_returns(r.astype(np.float64), m.astype(np.float64), V.astype(np.float64),
                                     VT, 0.99)
    np.testing.assert_array_equal(y.cpu().numpy(), y0.astype(np.float32))
    np.testing.assert_array_equal(adv.cpu().numpy(), adv0.astype(np.float32))


@pytest.mark.parametrize('arch,depth,A,R', [('NIPS', 1, 6, 1), ('NATURE', 1, 4, 11), ('PWYX', 1, 4, 11)])
@pytest.mark.parametrize('T,E', [(5, 8), (3, 5)])
def test_returns_loss_backward_fused(arch, depth, A, R, T, E):
    """mt_returns_loss_backward (the n-step scan inside the loss kernel) == mt_returns followed by
    mt_loss_backward: y, adv, loss terms and every gradient bit for bit; the scan reads rewards /
    masks from pinned host memory in place, as the learner does."""
    from manette_amd.network import returns as dev_returns, host_device_pointer
    net = _net(arch, depth, A, R, seed=T + E)
    rs = np.random.RandomState(100 * T + E)
    N = T * E
    obs = torch.from_numpy(rs.randint(0, 256, size=(N, 84, 84, 4 * depth)).astype(np.uint8)).cuda()
    v, pi, rep = [t.clone() for t in net.forward(obs)]
    a_idx = torch.from_numpy(rs.randint(0, A, N).astype(np.int32)).cuda()
    r_idx = torch.from_numpy(rs.randint(0, R, N).astype(np.int32)).cuda()
    rm = torch.zeros(2, T, E, dtype=torch.float32).pin_memory()
    rm[0] = torch.from_numpy(rs.choice([-1.0, 0.0, 1.0], size=(T, E)).astype(np.float32))
    rm[1] = torch.from_numpy((rs.rand(T, E) > 0.2).astype(np.float32))
    rm_dev = host_device_pointer(rm)
    VT = torch.from_numpy(rs.randn(E).astype(np.float32)).cuda()
    y0, adv0 = torch.empty(T, E, device='cuda'), torch.empty(T, E, device='cuda')
    lt0, lt1 = torch.empty(N, 4, device='cuda'), torch.empty(N, 4, device='cuda')
    dev_returns(rm_dev, rm_dev + 4 * N, v.view(T, E), VT, 0.99, y0, adv0)
    net.loss_backward(obs, N, v, pi, rep, a_idx, r_idx, y0.view(N), adv0.view(N), loss_terms=lt0)
    g0 = net.grad.clone()
    y1, adv1 = torch.empty(T, E, device='cuda'), torch.empty(T, E, device='cuda')
    net.grad.zero_()
    net.returns_loss_backward(obs, T, E, pi, rep, v, a_idx, r_idx, rm_dev, rm_dev + 4 * N, VT, 0.99, y1, adv1,
                              loss_terms=lt1, norm_partials=True)
    torch.cuda.synchronize()
    for a, b, k in ((y0, y1, 'y'), (adv0, adv1, 'adv'), (lt0, lt1, 'loss_terms'), (g0, net.grad, 'grad')):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=k)
    # the fused norm partials add up to the global norm of the gradient (oracle: float64)
    norm = float(np.sqrt(net.partials.double().sum().item()))
    ref = optim.global_norm([g0.cpu().numpy()])
    assert abs(norm - ref) <= 1e-5 * ref, (norm, ref)


@pytest.mark.parametrize('clip_type', ['global', 'ignore'])
@pytest.mark.parametrize('gscale', [1e-3, 10.0])
def test_clip_rmsprop(clip_type, gscale):
    net = _net('NIPS', 1, 6, 1)
    net.clip_type = 1 if clip_type == 'global' else 0
    rs = np.random.RandomState(1)
    n = net.nparams
    g = (rs.randn(n) * gscale).astype(np.float32)
    w0 = net.params.cpu().numpy().copy()
    ms0 = (1.0 + rs.rand(n)).astype(np.float32)
    mom0 = (rs.randn(n) * 1e-3).astype(np.float32)
    net.grad.copy_(torch.from_numpy(g))
    net.ms.copy_(torch.from_numpy(ms0))
    net.mom.copy_(torch.from_numpy(mom0))
    net.set_lr(0.0224)
    net.apply_gradients()
    torch.cuda.synchronize()
    norm = optim.global_norm([g])
    assert abs(float(net.norm_dev.item()) - norm) <= 1e-5 * norm
    s = optim.clip_scale(net.norm_dev.item(), 3.0) if clip_type == 'global' else np.float32(1.0)
    w, ms, mom = w0.copy(), ms0.copy(), np.zeros_like(mom0)
    mom[...] = mom0
    optim.rmsprop_apply(w, ms, mom, g * s, np.float32(0.0224), 0.99, 0.0, 0.1)
    np.testing.assert_array_equal(net.ms.cpu().numpy(), ms)
    np.testing.assert_array_equal(net.mom.cpu().numpy(), mom)
    np.testing.assert_array_equal(net.params.cpu().numpy(), w)


@pytest.mark.parametrize('rows_only', [False, True])
@pytest.mark.parametrize('depth', [1, 3])
def test_preprocess_bit_exact(depth, rows_only):
    from manette_amd.network import preprocess as dev_pre
    rs = np.random.RandomState(depth)
    E = 7
    counts = np.array([1, 4, 2, 3, 1, 4, 1], np.int32)
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
    raw = rs.randint(0, 256, size=(int(counts.sum()), 2, 210, 160, depth)).astype(np.uint8)
    prev = rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    out = torch.empty(E, 84, 84, 4 * depth, dtype=torch.uint8, device='cuda')
    if rows_only:  # runner-staged rows (the 84 the resize reads) + identity row LUT
        dev_pre(d(raw[:, :, preprocess.ROW_LUT]), d(offs), d(counts), E, depth, d(np.arange(84, dtype=np.int32)),
                d(preprocess.COL_LUT.astype(np.int32)), d(prev), out, src_rows=84)
    else:
        dev_pre(d(raw), d(offs), d(counts), E, depth, d(preprocess.ROW_LUT.astype(np.int32)),
                d(preprocess.COL_LUT.astype(np.int32)), d(prev), out)
    got = out.cpu().numpy()
    for e in range(E):
        pushes = [preprocess.pool_and_resize(raw[offs[e] + j, 0], raw[offs[e] + j, 1]) for j in range(counts[e])]
        np.testing.assert_array_equal(got[e], preprocess.stack_update(prev[e], pushes, depth))


@pytest.mark.parametrize('depth', [1, 3])
def test_preprocess_pooled_bit_exact(depth):
    """mt_preprocess_pooled: one staged screen per push, max(f0, f1) taken on the host."""
    from manette_amd.network import preprocess as dev_pre
    rs = np.random.RandomState(10 + depth)
    E = 6
    counts = np.array([4, 1, 3, 2, 4, 1], np.int32)
    offs = (4 * np.arange(E)).astype(np.int32)
    raw = rs.randint(0, 256, size=(4 * E, 2, 84, 160, depth)).astype(np.uint8)
    pooled = np.maximum(raw[:, 0], raw[:, 1])[:, None]
    prev = rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    out = torch.empty(E, 84, 84, 4 * depth, dtype=torch.uint8, device='cuda')
    dev_pre(d(pooled), d(offs), d(counts), E, depth, d(np.arange(84, dtype=np.int32)),
            d(preprocess.COL_LUT.astype(np.int32)), d(prev), out, src_rows=84, pooled=True)
    got = out.cpu().numpy()
    full = np.zeros((4 * E, 2, 210, 160, depth), np.uint8)
    full[:, :, preprocess.ROW_LUT] = raw
    for e in range(E):
        pushes = [preprocess.pool_and_resize(full[offs[e] + j, 0], full[offs[e] + j, 1]) for j in range(counts[e])]
        np.testing.assert_array_equal(got[e], preprocess.stack_update(prev[e], pushes, depth))


@pytest.mark.parametrize('depth', [1, 3])
def test_preprocess_resized_bit_exact(depth):
    """mt_preprocess_resized: each push's final 84x84 frame staged by the host, only stacked."""
    from manette_amd.network import preprocess as dev_pre
    rs = np.random.RandomState(20 + depth)
    E = 6
    counts = np.array([4, 1, 3, 2, 4, 1], np.int32)
    offs = (4 * np.arange(E)).astype(np.int32)
    final = rs.randint(0, 256, size=(4 * E, 84, 84, depth)).astype(np.uint8)
    prev = rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    out = torch.empty(E, 84, 84, 4 * depth, dtype=torch.uint8, device='cuda')
    dev_pre(d(final), d(offs), d(counts), E, depth, None, None, d(prev), out, resized=True)
    got = out.cpu().numpy()
    for e in range(E):
        pushes = [final[offs[e] + j] for j in range(counts[e])]
        np.testing.assert_array_equal(got[e], preprocess.stack_update(prev[e], pushes, depth))


EPSNEG = float(np.finfo(np.float32).epsneg)


def _draw_probs(p):
    """Distribution of the device draw (common.h draw_index): inverse CDF over (p_j - epsneg) for
    j < n-1, the last category taking the remainder. With every p_j >= epsneg it is numpy's
    multinomial(1, p - epsneg) of exploration_policy.py:108-116; a category below epsneg (where
    the reference's numpy raises 'pvals < 0') gets no mass and eats into the next one's interval."""
    p = np.asarray(p, np.float32)
    cum = np.cumsum([np.float64(np.float32(x) - np.float32(EPSNEG)) for x in p[:-1]])
    out = np.zeros(len(p))
    m = 0.0
    for j, c in enumerate(cum):
        out[j] = max(0.0, min(c, 1.0) - m)
        m = max(m, min(c, 1.0))
    out[-1] = max(0.0, 1.0 - m)
    return out


def _chi2_ok(counts, probs, alpha=1e-4):
    from scipy.stats import chi2
    nz = probs > 0
    assert counts[~nz].sum() == 0, 'a zero-probability category was drawn'
    n = counts.sum()
    exp = probs[nz] * n
    stat = float(((counts[nz] - exp) ** 2 / exp).sum())
    pval = chi2.sf(stat, max(int(nz.sum()) - 1, 1))
    assert pval > alpha, (stat, pval, counts, exp)


def _sample(pi, rep, seed, ctr, row0=0):
    from manette_amd.network import sample
    B = pi.shape[0]
    a = torch.empty(B, dtype=torch.int32, device='cuda')
    r = torch.empty(B, dtype=torch.int32, device='cuda')
    sample(pi, rep, seed, ctr, a, r, row0=row0)
    return a, r


@pytest.mark.parametrize('A,R', [(6, 1), (18, 11), (9, 11)])
def test_sample_chi_square_both_heads(A, R):
    """Chi-square goodness of fit of both heads (A = 18 Seaquest, R = 11 FiGAR10) against the
    reference's multinomial(1, p - epsneg) over 8 x 4096 draws; counters advance by one per call."""
    B, K = 4096, 8
    rs = np.random.RandomState(A * 100 + R)
    p = rs.dirichlet(np.ones(A)).astype(np.float32)
    q = rs.dirichlet(np.ones(R)).astype(np.float32)
    pi = torch.from_numpy(np.tile(p, (B, 1))).cuda()
    rep = torch.from_numpy(np.tile(q, (B, 1))).cuda()
    ctr = torch.zeros(B, dtype=torch.int64, device='cuda')
    ca, cr = np.zeros(A), np.zeros(R)
    for _ in range(K):
        a, r = _sample(pi, rep, 1234, ctr)
        ca += np.bincount(a.cpu().numpy(), minlength=A)
        cr += np.bincount(r.cpu().numpy(), minlength=R)
    assert (ctr.cpu().numpy() == K).all()
    _chi2_ok(ca, _draw_probs(p))
    if R > 1:
        _chi2_ok(cr, _draw_probs(q))
    else:
        assert cr[0] == B * K


def test_sample_epsneg_and_last_category_remainder():
    """Entries below float32 epsneg are never drawn (the reference's numpy raises on them); the
    last category takes the remainder 1 - sum_{j<n-1}(p_j - epsneg), including the epsneg mass
    the others give up; a near-one-hot row always draws its category."""
    B, K = 4096, 8
    p = np.array([0.5, 1e-9, 0.25, 0.0, 0.25 - 1e-9], np.float32)
    p = p / p.sum()
    q = np.array([1e-12, 1e-12, 1.0], np.float32)
    pi = torch.from_numpy(np.tile(p, (B, 1))).cuda()
    rep = torch.from_numpy(np.tile(q, (B, 1))).cuda()
    ctr = torch.zeros(B, dtype=torch.int64, device='cuda')
    ca = np.zeros(5)
    for _ in range(K):
        a, r = _sample(pi, rep, 77, ctr)
        ca += np.bincount(a.cpu().numpy(), minlength=5)
        assert (r.cpu().numpy() == 2).all()
    probs = _draw_probs(p)
    assert probs[1] == 0 and probs[3] == 0
    _chi2_ok(ca, probs)
    # a one-hot row: p = (1, 0, ..., 0) -> always category 0 (1 - epsneg > u for u < 1 - 2^-24)
    oh = np.zeros((B, 6), np.float32)
    oh[:, 0] = 1.0
    a, _ = _sample(torch.from_numpy(oh).cuda(), rep, 5, torch.zeros(B, dtype=torch.int64, device='cuda'))
    assert (a.cpu().numpy() == 0).mean() > 0.9999


def test_sample_rows_independent_and_global_row_ids():
    """Rows with the same pi draw independent streams (pairwise agreement = sum p^2); the draw is a
    pure function of (seed, global row, counter): rows [8, 16) of a 16-row call with row0 = 0 ==
    an 8-row call with row0 = 8 (a data-parallel rank's shard), and replaying the counters
    reproduces the draws."""
    A, R, B = 6, 11, 16
    rs = np.random.RandomState(3)
    p = rs.dirichlet(np.ones(A)).astype(np.float32)
    q = rs.dirichlet(np.ones(R)).astype(np.float32)
    pi = torch.from_numpy(np.tile(p, (B, 1))).cuda()
    rep = torch.from_numpy(np.tile(q, (B, 1))).cuda()
    ctr = torch.zeros(B, dtype=torch.int64, device='cuda')
    full = [tuple(t.cpu().numpy() for t in _sample(pi, rep, 9, ctr)) for _ in range(300)]
    ctr8 = torch.zeros(8, dtype=torch.int64, device='cuda')
    half = [tuple(t.cpu().numpy() for t in _sample(pi[8:].contiguous(), rep[8:].contiguous(), 9, ctr8, row0=8))
            for _ in range(300)]
    for (fa, fr), (ha, hr) in zip(full, half):
        np.testing.assert_array_equal(fa[8:], ha)
        np.testing.assert_array_equal(fr[8:], hr)
    ctr.zero_()
    again = [tuple(t.cpu().numpy() for t in _sample(pi, rep, 9, ctr)) for _ in range(300)]
    for (fa, fr), (ga, gr) in zip(full, again):
        np.testing.assert_array_equal(fa, ga)
        np.testing.assert_array_equal(fr, gr)
    acts = np.stack([f[0] for f in full])  # [300][16]
    agree = np.mean([np.mean(acts[:, i] == acts[:, j]) for i in range(B) for j in range(i + 1, B)])
    expect = float((_draw_probs(p) ** 2).sum())
    assert abs(agree - expect) < 0.02, (agree, expect)


def test_zero_copy_reads_see_host_rewrites_across_launches():
    """The zero-copy kernels read pinned (non-coherent) host memory with plain loads; a line a
    launch cached must not serve a later launch after the host rewrote it (each dispatch starts
    with a system-scope acquire — rollout.hip's pull kernel relies on it). 50 rounds: the host
    rewrites the staged frames in place, the same kernel reads them again."""
    from manette_amd.network import preprocess as dev_pre, host_device_pointer
    E, depth = 8, 1
    rs = np.random.RandomState(5)
    frames = torch.zeros(4 * E, 84, 84, depth, dtype=torch.uint8).pin_memory()
    fdev = host_device_pointer(frames)
    offs = torch.from_numpy((4 * np.arange(E)).astype(np.int32)).cuda()
    counts_h = rs.randint(1, 5, E).astype(np.int32)
    counts = torch.from_numpy(counts_h).cuda()
    prev = torch.from_numpy(rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)).cuda()
    out = torch.empty_like(prev)
    import ctypes as C
    from manette_amd import _lib
    for it in range(50):
        frames.numpy()[...] = rs.randint(0, 256, size=frames.shape).astype(np.uint8)
        _lib.check(_lib.hip().mt_preprocess_resized(C.c_void_p(fdev), C.c_void_p(offs.data_ptr()),
                                                    C.c_void_p(counts.data_ptr()), E, depth,
                                                    C.c_void_p(prev.data_ptr()), C.c_void_p(out.data_ptr()),
                                                    C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        f = frames.numpy()
        pv = prev.cpu().numpy()
        for e in range(E):
            pushes = [f[4 * e + j] for j in range(counts_h[e])]
            np.testing.assert_array_equal(got[e], preprocess.stack_update(pv[e], pushes, depth), err_msg='round %d' % it)


@pytest.mark.parametrize('arch,E,depth', [('NIPS', 7, 1), ('NIPS', 32, 1), ('NIPS', 5, 3), ('NATURE', 7, 1),
                                          ('NATURE', 64, 1), ('PWYX', 7, 1), ('PWYX', 5, 3), ('PWYX', 32, 3)])
def test_stacking_trunk_in_kernel_pull(arch, E, depth):
    """mt_forward_trunk_stacking — the rollout chain's conv kernel (NIPS: nips_conv_kernel<STACK>;
    gray NATURE: conv1 = the direct conv with DFwdStack's patch staging; PWYX gray / RGB:
    stack_conv1_kernel's env blocks, then its conv1 tiles per env) pulling each env's frames
    from pinned host staging behind its ready word (edge cache lines read with system-scope loads):
    the stacked state == the A2 oracle (bit-exact), and the trunk outputs (conv activations + dense
    partial slabs) == mt_forward_trunk on that state, bit for bit."""
    from manette_amd.network import host_device_pointer
    import ctypes as C
    net = _net(arch, depth, 6, 11, seed=E)
    rs = np.random.RandomState(30 + E + depth)
    counts = rs.randint(1, 5, E).astype(np.int32)
    counts[:2] = 4  # full slot groups: their last line borders the next env's first
    frames = torch.zeros(4 * E, 84, 84, depth, dtype=torch.uint8).pin_memory()
    frames.numpy()[...] = rs.randint(0, 256, size=frames.shape).astype(np.uint8)
    tag = 12345
    ready = torch.zeros(E, 32, dtype=torch.int32).pin_memory()  # MH_READY_STRIDE words per env
    ready.numpy()[:, 0] = (tag << 3) | counts
    prev_h = rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)
    prev = torch.from_numpy(prev_h).cuda()
    out = torch.zeros_like(prev)
    ws = net.workspace(E, 'stk')
    ws.zero_()
    net.forward_trunk_stacking(prev, C.c_void_p(host_device_pointer(frames)), C.c_void_p(host_device_pointer(ready)),
                               tag, out, E, ws_key='stk')
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    f = frames.numpy()
    for e in range(E):
        pushes = [f[4 * e + j] for j in range(counts[e])]
        np.testing.assert_array_equal(got[e], preprocess.stack_update(prev_h[e], pushes, depth), err_msg='env %d' % e)
    ws2 = net.workspace(E, 'plain')
    ws2.zero_()
    net.forward_trunk(out, E, ws_key='plain')
    torch.cuda.synchronize()
    assert torch.equal(ws[:ws2.numel()], ws2)


def _counter_words(net, ws, E):
    """The stacking chains' hand-off counters of a workspace of E rows (mt_net_workspace_region kind 4)."""
    import ctypes as C
    from manette_amd import _lib
    off, n = C.c_size_t(), C.c_size_t()
    _lib.check(_lib.hip().mt_net_workspace_region(net._h, 0, E, 0, 4, 0, C.byref(off), C.byref(n)), 'region')
    return ws[off.value:off.value + n.value].cpu().numpy().view(np.uint32)


@pytest.mark.parametrize('arch,depth', [('NIPS', 1), ('NATURE', 1), ('PWYX', 1), ('PWYX', 3)])
def test_stacking_trunk_unpublished_env_is_bounded(arch, depth):
    """An env whose ready word never carries the launch's tag (an emulator that died,
    emulator_runner.py:19-42's worker that never reports back): every wait of the stacking chain is
    bounded (~2 s of s_memrealtime), so the launch drains instead of hanging the GPU; the stalled
    env's new state is the previous one (no frame stacked, as wait_published's timeout rule says) and
    every other env is stacked bit-exactly. The timeout is RAISED in the status word and surfaced by
    the host as an MTError; the hand-off counters are all zero after the stalled launch (a producer
    whose consumer stopped waiting first still adds after the reset: the reset subtracts the full
    counts), and a second, fully published launch on the same workspace stacks and
    computes bit-exactly (its tiles do not pass their waits on a stale count)."""
    import time
    from manette_amd import _lib
    from manette_amd.network import WaitStatus, host_device_pointer
    import ctypes as C
    E, stalled = 7, 3
    net = _net(arch, depth, 6, 11, seed=3)
    rs = np.random.RandomState(40 + depth)
    counts = rs.randint(1, 5, E).astype(np.int32)
    frames = torch.zeros(4 * E, 84, 84, depth, dtype=torch.uint8).pin_memory()
    frames.numpy()[...] = rs.randint(0, 256, size=frames.shape).astype(np.uint8)
    tag = 4242
    ready = torch.zeros(E, 32, dtype=torch.int32).pin_memory()
    ready.numpy()[:, 0] = (tag << 3) | counts
    ready.numpy()[stalled, 0] = ((tag + 1) << 3) | counts[stalled]  # published for another launch
    prev_h = rs.randint(0, 256, size=(E, 84, 84, 4 * depth)).astype(np.uint8)
    prev = torch.from_numpy(prev_h).cuda()
    out = torch.zeros_like(prev)
    ws = net.workspace(E, 'stk_bounded')
    ws.zero_()
    status = WaitStatus()
    fdev, rdev = C.c_void_p(host_device_pointer(frames)), C.c_void_p(host_device_pointer(ready))
    torch.cuda.synchronize()
    t0 = time.time()
    net.forward_trunk_stacking(prev, fdev, rdev, tag, out, E, ws_key='stk_bounded', status=status)
    torch.cuda.synchronize()
    assert time.time() - t0 < 30.0
    with pytest.raises(_lib.MTError, match='timed out'):
        status.check('stacking trunk')
    got = out.cpu().numpy()
    f = frames.numpy()
    for e in range(E):
        pushes = [] if e == stalled else [f[4 * e + j] for j in range(counts[e])]
        want = prev_h[e] if e == stalled else preprocess.stack_update(prev_h[e], pushes, depth)
        np.testing.assert_array_equal(got[e], want, err_msg='env %d' % e)
    words = _counter_words(net, ws, E)
    assert (arch == 'NIPS') == (words.size == 0), words.size  # (NIPS: no in-launch hand-off)
    assert not words.any(), np.nonzero(words)

    # a second launch on the same workspace, every env published: no timeout, bit-exact
    tag2 = tag + 7
    counts2 = rs.randint(1, 5, E).astype(np.int32)
    frames.numpy()[...] = rs.randint(0, 256, size=frames.shape).astype(np.uint8)
    ready.numpy()[:, 0] = (tag2 << 3) | counts2
    prev2_h = got
    out2 = torch.zeros_like(prev)
    net.forward_trunk_stacking(out, fdev, rdev, tag2, out2, E, ws_key='stk_bounded', status=status)
    torch.cuda.synchronize()
    status.check('second stacking trunk')
    got2 = out2.cpu().numpy()
    for e in range(E):
        pushes = [f[4 * e + j] for j in range(counts2[e])]
        np.testing.assert_array_equal(got2[e], preprocess.stack_update(prev2_h[e], pushes, depth), err_msg='env %d' % e)
    assert not _counter_words(net, ws, E).any()
    ws2 = net.workspace(E, 'stk_bounded_plain')
    ws2.zero_()
    net.forward_trunk(out2, E, ws_key='stk_bounded_plain')
    torch.cuda.synchronize()
    assert torch.equal(ws[:ws2.numel()], ws2)  # (the counter words included: zero in both)


def test_nips_backward_above_fused_cap():
    """Above kNipsFusedBwdMaxRows (1,280 rows) the NIPS gray conv backward takes the layered
    trunk_backward (per-image slabs would grow without bound): the gradient of 1,281 rows
    (loss = 5/B sum of row terms) == the B-weighted sum of the fused path's gradients of rows
    [0, 1280) and of row 1280, within fp32 reduction order."""
    A, R = 6, 1
    net = _net('NIPS', 1, A, R, seed=21)
    rs = np.random.RandomState(21)
    B = 1281
    obs = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    a_idx = torch.from_numpy(rs.randint(0, A, B).astype(np.int32)).cuda()
    r_idx = torch.from_numpy(rs.randint(0, R, B).astype(np.int32)).cuda()
    y = torch.from_numpy(rs.randn(B).astype(np.float32)).cuda()
    adv = torch.from_numpy(rs.randn(B).astype(np.float32)).cuda()

    def grad(lo, hi):
        n = hi - lo
        v, pi, rep = net.forward(obs[lo:hi], ws_key=('cap', n))
        net.loss_backward(obs[lo:hi], n, v, pi, rep, a_idx[lo:hi], r_idx[lo:hi], y[lo:hi], adv[lo:hi],
                          ws_key=('cap', n))
        torch.cuda.synchronize()
        return net.grad.double().cpu().numpy() * n
    whole = grad(0, B)
    parts = grad(0, 1280) + grad(1280, B)
    assert np.linalg.norm(whole - parts) <= 2e-5 * np.linalg.norm(parts)
