"""Host timeline of the native rollout in the bench workload (mt_rollout_host_trace): runs
--updates bench updates, then prints the last --show macro-steps: per step the host phases
(launches, wait for indices, emulators, bookkeeping) and the gap since the previous step, so the
update's share and the steady-state period can be read off.
    python tools/host_trace.py [--config pong-nips --updates 30 --show 12]"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='pong-nips')
    ap.add_argument('--updates', type=int, default=30)
    ap.add_argument('--show', type=int, default=12)
    a = ap.parse_args()
    import tempfile
    import numpy as np
    import torch
    import bench
    from manette_amd import _lib
    L, _ = bench.make_learner(a.config, debugging_folder=tempfile.mkdtemp() + '/')
    L.start()
    try:
        for _ in range(a.updates):
            L.book.new_update()
            L.rollout()
            L.update()
        torch.cuda.synchronize()
        buf = np.zeros((256, 6))
        n = C.c_int()
        _lib.check(_lib.hip().mt_rollout_host_trace(L.native_step, C.c_void_p(buf.ctypes.data), a.show, C.byref(n)))
        tr = buf[:n.value]
        print('  t   since prev start   enqueue   wait-idx   emulators   book   (us)')
        for k in range(len(tr)):
            t, s0, s1, s2, s3, s4 = tr[k]
            gap = s0 - tr[k - 1][1] if k else float('nan')
            print('%3d   %8.1f          %7.1f   %8.1f   %9.1f   %5.1f' % (t, gap, s1 - s0, s2 - s1, s3 - s2, s4 - s3))
    finally:
        L.cleanup()


if __name__ == '__main__':
    main()
