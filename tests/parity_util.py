"""Shared parity helpers for the GPU tests (not a test module)."""
import numpy as np

from oracle import nets


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-12))


def channel_errs(got, ref):
    """Relative L2 error of every output channel (last axis) of a weight gradient: a corruption of
    one channel (column 10 of the RGB conv1 weight gradient) is 1/C of the variable's
    norm and can hide under a per-variable bound. Each channel's error is taken relative to its
    own norm, floored at a tenth of the variable's RMS channel norm (a dead-ReLU channel's
    gradient is ~0)."""
    g = np.asarray(got, np.float64).reshape(-1, np.shape(ref)[-1])
    r = np.asarray(ref, np.float64).reshape(g.shape)
    d = np.linalg.norm(g - r, axis=0)
    n = np.linalg.norm(r, axis=0)
    floor = 0.1 * np.linalg.norm(r) / np.sqrt(r.shape[1])
    return d / np.maximum(np.maximum(n, floor), 1e-30)


def check_grads(spec, got, G, loose, tight=2e-4, tie=5e-3):
    """Every variable's gradient within `tight` relative L2 of the oracle (`tie` for the variables in
    `loose`; the tests pass none since the oracle routes max-pool near-ties as the device did,
    device_routes), and — for every weight matrix / conv kernel — every output channel within the
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


def device_routes(spec, P, frames, dev, act='relu', alpha=0.1, chunk=32, tie=1e-5):
    """The device's max-pool routing as the oracle's, checked: dev = {conv name: [F, OH/2, OW/2, C]
    argmax bytes read from the device workspace (DeviceNetwork.pool_argmax)}. At every window whose
    top two fp64 values differ by >= `tie` relative, the device's position must equal MaxPoolGrad's
    first maximum (bit-exact index work); at the near-ties fp32 rounding may order the two either
    way, and the oracle then routes where the device did (nets.trunk_backward routes=), so the
    gradients are compared at the tight bound. Returns (routes, number of near-tie windows)."""
    ties = 0
    for c0 in range(0, len(frames), chunk):
        _, layers = nets.trunk_forward(spec, P, frames[c0:c0 + chunk], act, alpha)
        for L in layers:
            if not L['pool']:
                continue
            arg, gap = nets.pool_route(L['y'])
            d = dev[L['name']][c0:c0 + chunk]
            clear = gap >= tie
            bad = int(((d != arg) & clear).sum())
            assert bad == 0, (L['name'], c0, bad, 'device max-pool argmax differs from the oracle away from ties')
            ties += int((~clear).sum())
    return dev, ties
