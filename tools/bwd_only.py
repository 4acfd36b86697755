"""The update's train pass alone (for rocprofv3 PMC / kernel-trace passes): bench.make_learner's
learner after two real updates, then --reps train_backward() calls back to back (the backward of
the last rollout: forward reused, parameters unchanged).
  python tools/bwd_only.py [--config mspacman-lstm-figar --reps 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='mspacman-lstm-figar')
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    import tempfile
    import torch
    import bench
    L, _ = bench.make_learner(a.config, debugging_folder=tempfile.mkdtemp() + '/')
    L.start()
    try:
        for _ in range(2):
            L.book.new_update()
            L.rollout()
            L.update()
        torch.cuda.synchronize()
        for _ in range(a.reps):
            L.train_backward()
        torch.cuda.synchronize()
    finally:
        L.cleanup()
    print('done')


if __name__ == '__main__':
    main()
