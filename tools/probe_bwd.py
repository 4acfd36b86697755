"""Phase timeline of the fused NIPS conv backward (manette_amd/csrc/nips_bwd.h) from in-kernel
timestamps (probe build: s_memrealtime of lane 0 at each phase boundary of every block, slot 3).

    python -c "import os; from manette_amd import build as b; b.build_hip(out=os.path.abspath('manette_amd/libmanette_hip_probe.so'), defines=['MT_PROBE'])"
    MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so python tools/probe_bwd.py [--rows 160]

Runs the NIPS gray loss + backward on seeded rows a few times and prints, over the blocks of the
last run, the median / max of each phase and the spread of block start times.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=160)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    import torch
    from manette_amd import _lib
    from manette_amd.network import DeviceNetwork
    conf = dict(arch='NIPS', rgb=False, num_actions=6, nb_choices=1, softmax_temp=1.0,
                entropy_regularisation_strength=0.02, clip_norm=3.0, clip_norm_type='global',
                activation='relu', alpha_leaky_relu=0.1)
    net = DeviceNetwork(conf)
    net.init_params(3)
    B = a.rows
    rs = np.random.RandomState(1)
    d = lambda x: torch.from_numpy(x).cuda()
    obs = d(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8))
    a_idx = d(rs.randint(0, 6, size=B).astype(np.int32))
    r_idx = d(np.zeros(B, np.int32))
    y = d(rs.randn(B).astype(np.float32))
    adv = d(rs.randn(B).astype(np.float32))
    v, pi, rep = net.forward(obs)
    lib = _lib.hip()
    lib.mt_probe_read.restype = C.c_int
    lib.mt_probe_read.argtypes = [C.c_void_p, C.c_size_t]
    buf = np.zeros(5 * 1024 * 8, dtype=np.uint64)
    for _ in range(a.reps):
        net.loss_backward(obs, B, v, pi, rep, a_idx, r_idx, y, adv)
        torch.cuda.synchronize()
    _lib.check(lib.mt_probe_read(C.c_void_p(buf.ctypes.data), buf.size), 'mt_probe_read')
    pairs = (B + 1) // 2
    P = buf.reshape(5, 1024, 8)[3, :B + pairs, :5].astype(np.int64)
    us = lambda x: x * 0.01  # 100 MHz
    t0 = P[:, 0].min()
    img, par = P[:B], P[B:]
    print('image blocks %d: start spread %.2f us, end %+.2f .. %+.2f us' % (
        B, us(img[:, 0].max() - t0), us(img[:, 4].min() - t0), us(img[:, 4].max() - t0)))
    for name, i0, i1 in (('stage (loads -> LDS)', 0, 1), ('conv2 dX + mask', 1, 2), ('conv1 dW + db', 2, 4),
                         ('block total', 0, 4)):
        dt = us(img[:, i1] - img[:, i0])
        print('  %-22s median %6.2f us  max %6.2f us' % (name, np.median(dt), dt.max()))
    print('pair blocks %d: start %+.2f .. %+.2f us, end %+.2f .. %+.2f us' % (
        pairs, us(par[:, 0].min() - t0), us(par[:, 0].max() - t0), us(par[:, 4].min() - t0), us(par[:, 4].max() - t0)))
    for name, i0, i1 in (('stage (2 images)', 0, 1), ('conv2 dW + db', 1, 4), ('block total', 0, 4)):
        dt = us(par[:, i1] - par[:, i0])
        print('  %-22s median %6.2f us  max %6.2f us' % (name, np.median(dt), dt.max()))


if __name__ == '__main__':
    main()
