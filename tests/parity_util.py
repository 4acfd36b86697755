"""Shared parity helpers for the GPU tests (not a test module)."""
import numpy as np

from oracle import nets


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-12))


def _tie_names(spec, layers):
    hit = []
    for L in layers:
        if not L['pool']:
            continue
        y = L['y']
        B, H, W, C = y.shape
        w = y[:, :H // 2 * 2, :W // 2 * 2].reshape(B, H // 2, 2, W // 2, 2, C).transpose(0, 1, 3, 5, 2, 4)
        s = np.sort(w.reshape(-1, 4), axis=1)
        gap = (s[:, 3] - s[:, 2]) / np.maximum(np.abs(s[:, 3]), 1e-30)
        if ((gap > 0) & (gap < 1e-5)).any():
            hit.append(L['name'])
    return hit


def near_tie_layers_frames(spec, P, frames, act='relu', alpha=0.1, chunk=32):
    """near_tie_layers over distinct frames [F,84,84,C] (the LSTM frame store), in chunks."""
    hit = set()
    for c0 in range(0, len(frames), chunk):
        _, layers = nets.trunk_forward(spec, P, frames[c0:c0 + chunk], act, alpha)
        hit.update(_tie_names(spec, layers))
    if not hit:
        return set()
    last = max(int(n[4:]) for n in hit)
    return {'Network/conv%d/conv%d_%s' % (i, i, k) for i in range(1, last + 1) for k in ('weights', 'biases')}


def near_tie_layers(spec, P, obs, act='relu', alpha=0.1):
    """Weight/bias names of the pooled convs at or below a 2x2 max-pool window whose top two values
    differ by < 1e-5 relative in the fp64 oracle: there fp32 rounding may route MaxPoolGrad to the
    other position (a discontinuity), moving those gradients by ~1e-3 relative L2 per flip."""
    _, _, _, cache = nets.forward(spec, P, obs, act=act, alpha=alpha)
    hit = _tie_names(spec, cache['layers'])
    if not hit:
        return set()
    last = max(int(n[4:]) for n in hit)
    return {'Network/conv%d/conv%d_%s' % (i, i, k) for i in range(1, last + 1) for k in ('weights', 'biases')}


def check_grads(spec, got, G, loose, tight=2e-4, tie=5e-3):
    errs = {name: rel(got[name], G[name]) for name, _, _ in spec['vars']}
    bad = {n: e for n, e in errs.items() if e >= (tie if n in loose else tight)}
    assert not bad, (bad, sorted(loose))
