"""SURVEY §8(d) cross-check of the CPU baseline's host loop (BUILD CONTAINER ONLY: imports the
reference from /root/reference, like tests/golden/make_golden.py; never runs on the GPU box).

Times the host plumbing of one PAAC update with a zero-cost network, on the same cheap
deterministic emulators (tests/golden/golden_env.GoldenEnv):
  reference  paac.PAACLearner.train() under make_golden's stub tensorflow (its Runners /
             EmulatorRunner worker processes, mp.Queue barrier, per-env Python loops);
  port       oracle/host_loop.HostLoop with ProcessRunners (the restatement bench.py's
             cpu_baseline leg times, there with the torch-CPU network and synthetic emulators).
env-steps/s from the difference of two run lengths (process start-up cancels out).
  python tools/plumbing_crosscheck.py [--ec 32 --ew 8 --ref /root/reference]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))


class ZeroNet(object):
    """host_loop network double: fixed-distribution outputs, no work."""

    def __init__(self, A, R):
        self.rng = np.random.RandomState(99)
        self.A, self.R = A, R

    def forward(self, states, bootstrap=False):
        import make_golden
        v, pi, rep = make_golden.fake_outputs(self.rng, len(states), self.A, self.R)
        return v if bootstrap else (v, pi, rep)

    def train(self, *a, **k):
        pass


def time_reference(ref, ec, ew, T, A, n):
    import make_golden
    t = time.perf_counter()
    make_golden.run_host_loop(ref, ec, ew, T, A, 0, 1, n, False)
    return time.perf_counter() - t


def time_port(ec, ew, T, A, n):
    from oracle import host_loop
    from golden_env import GoldenEnv
    emus = [GoldenEnv(i) for i in range(ec)]
    loop = host_loop.HostLoop(emus, ZeroNet(A, 1), [0], A, max_local_steps=T, workers=ew, record=False)
    t = time.perf_counter()
    loop.run(ec * T * n)
    return time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    ap.add_argument('--ec', type=int, default=32)
    ap.add_argument('--ew', type=int, default=8)
    ap.add_argument('--updates', type=int, default=200)
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    import make_golden
    make_golden._install_stubs()
    sys.path.insert(0, a.ref)
    T, A = 5, 6
    n1, n2 = 20, 20 + a.updates
    res = {}
    for name, fn in (('reference', lambda n: time_reference(a.ref, a.ec, a.ew, T, A, n)),
                     ('port', lambda n: time_port(a.ec, a.ew, T, A, n))):
        rates = []
        for _ in range(a.reps):
            t1, t2 = fn(n1), fn(n2)
            rates.append((n2 - n1) * a.ec * T / (t2 - t1))
        res[name] = rates
        print('%-9s ec=%d ew=%d: %s env-steps/s (median %.0f)' % (name, a.ec, a.ew, ' '.join('%.0f' % r for r in rates),
                                                                 float(np.median(rates))), flush=True)
    print('port / reference plumbing rate: %.2f' % (np.median(res['port']) / np.median(res['reference'])))


if __name__ == '__main__':
    main()
