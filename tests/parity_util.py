"""Shared parity helpers for the GPU tests (not a test module)."""
import numpy as np

from oracle import nets


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-12))


def channel_errs(got, ref):
    """L2 error of every output channel (last axis) of a weight gradient relative to the variable's
    RMS channel norm: a corruption of one channel (column 10 of the RGB conv1 weight
    gradient, ~1e-2 on this scale) is 1/C of the variable's error and can hide under a per-variable
    bound, while a channel whose own gradient is small after cancellation keeps an fp32 error that
    is large relative to itself but not to the scale of the variable."""
    g = np.asarray(got, np.float64).reshape(-1, np.shape(ref)[-1])
    r = np.asarray(ref, np.float64).reshape(g.shape)
    d = np.linalg.norm(g - r, axis=0)
    scale = np.linalg.norm(r) / np.sqrt(r.shape[1])
    return d / max(scale, 1e-30)


def check_grads(spec, got, G, loose, tight=2e-4, tie=5e-3):
    """Every variable's gradient within `tight` relative L2 of the oracle (`tie` for the variables in
    `loose`; the tests pass none since the oracle routes max-pool near-ties as the device did,
    device_branches), and — for every weight matrix / conv kernel — every output channel within the
    same bound (channel_errs)."""
    errs = {name: rel(got[name], G[name]) for name, _, _ in spec['vars']}
    bad = {n: e for n, e in errs.items() if e >= (tie if n in loose else tight)}
    assert not bad, (bad, sorted(loose))
    for name, _, _ in spec['vars']:
        if np.ndim(G[name]) < 2:
            continue
        ce = channel_errs(got[name], G[name])
        lim = tie if name in loose else tight
        assert (ce < lim).all(), (name, 'channels', np.nonzero(ce >= lim)[0].tolist(), float(ce.max()))


def device_branches(spec, P, frames, dev, act='relu', alpha=0.1, win=None, rows=None, chunk=32, tie=1e-5,
                    near=2e-5):
    """The device's decisions at the gradient's discontinuities, checked, for the oracle to follow.

    dev = DeviceNetwork.forward_branches(...): per conv layer the stored post-activation output and
    (pooled layers) the max-pool argmax, plus the dense output H. frames: the distinct frames the
    trunk ran on (dev's conv rows; `rows` selects the rows of dev that frames are, default all);
    win: the LSTM windows' frame indices [N, 5] (else row n = frame n), whose first N rows of H
    the train step used.
    - max pool: at every window whose top two fp64 values differ by >= `tie` x the layer's RMS,
      the device's position must equal MaxPoolGrad's first maximum (bit-exact index work);
    - ReLU / leaky ReLU: wherever the fp64 pre-activation is >= `near` x its RMS away from 0, the
      device's branch (its stored output > 0, resp. >= 0) must equal the oracle's;
    closer than that, fp32 rounding may take either side, and the oracle then takes the device's
    (nets.*_loss_and_grads routes= / branches= / hbranch=), so the gradients are compared at the
    tight bound. Returns dict(routes, branches, hbranch, ties, near)."""
    pos = (lambda x: x > 0) if act == 'relu' else (lambda x: x >= 0)
    sel = (lambda a: a) if rows is None else (lambda a: a[rows])
    routes, branches, ties, nears = {}, {}, 0, 0
    feats = []
    for c0 in range(0, len(frames), chunk):
        flat, layers = nets.trunk_forward(spec, P, frames[c0:c0 + chunk], act, alpha)
        feats.append(flat)
        for L in layers:
            y_dev, arg_dev = dev[L['name']]
            y_dev, arg_dev = sel(y_dev)[c0:c0 + chunk], None if arg_dev is None else sel(arg_dev)[c0:c0 + chunk]
            z = L['z']
            zs = np.sqrt(np.mean(z * z))
            if L['pool']:
                arg, gap = nets.pool_route(L['y'])
                ys = np.sqrt(np.mean(L['y'] ** 2))
                gap_abs = gap * np.maximum(np.abs(L['yp']), 1e-30)
                clear = gap_abs >= tie * ys
                bad = int(((arg_dev != arg) & clear).sum())
                assert bad == 0, (L['name'], c0, bad, 'device max-pool argmax differs from the oracle away from ties')
                ties += int((~clear).sum())
                routes.setdefault(L['name'], []).append(arg_dev)
                zq = nets.maxpool2(z)  # pre-activation of the window's maximum (act is monotonic)
            else:
                zq = z
            far = np.abs(zq) >= near * zs
            bad = int(((pos(y_dev) != pos(zq)) & far).sum())
            assert bad == 0, (L['name'], c0, bad, 'device activation branch differs from the oracle away from 0')
            nears += int((~far).sum())
            branches.setdefault(L['name'], []).append(np.where(far, pos(zq), pos(y_dev)))
    routes = {k: np.concatenate(v) for k, v in routes.items()}
    branches = {k: np.concatenate(v) for k, v in branches.items()}
    flat = np.concatenate(feats)
    flat = flat[np.asarray(win).reshape(-1)] if win is not None else flat
    _, _, _, cache = nets.heads_forward(spec, P, flat, act, alpha)
    hz = cache['hz']
    H_dev = dev['H'][:len(hz)]
    far = np.abs(hz) >= near * np.sqrt(np.mean(hz * hz))
    bad = int(((pos(H_dev) != pos(hz)) & far).sum())
    assert bad == 0, ('dense', bad, 'device activation branch differs from the oracle away from 0')
    nears += int((~far).sum())
    return dict(routes=routes, branches=branches, hbranch=np.where(far, pos(hz), pos(H_dev)), ties=ties, near=nears)
