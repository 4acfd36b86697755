"""Phase timeline of one pipelined rollout step's GPU chain from in-kernel timestamps.

Needs the probe build of the HIP library (s_memrealtime at phase boundaries of every block of
nips_conv_kernel, nips_fc_kernel and heads_fwd_kernel):

    python -c "from manette_amd import build as b; b.build_hip(out='/root/repo/manette_amd/libmanette_hip_probe.so', defines=['MT_PROBE'])"
    MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so python tools/probe.py [--config pong-nips]

Runs a few warm updates of the bench workload, then one rollout step (whose pipelined chain
stacks + forwards the next step), and prints, per kernel, when its blocks started (relative to
the first conv block), the median / max duration of each phase and the gaps between kernels.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = {0: ('conv', ['stage (incl. wait)', 'conv1', 'conv2', 'act2']),
          1: ('fc', ['load+mfma', 'reduce+store']),
          2: ('heads', ['slab sum', 'heads gemv', 'softmax+draw+flag'])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='pong-nips')
    ap.add_argument('--updates', type=int, default=20)
    ap.add_argument('--isolated', action='store_true',
                    help='time the roofline launch alone (mt_forward_trunk_stacking, every env published, as '
                         'bench.py / tools/trunk_only.py) instead of a rollout step')
    a = ap.parse_args()
    import torch
    import bench
    import train as train_cli
    from manette_amd import _lib
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.paac import PAACLearner
    cfg = bench.CONFIGS[a.config]
    args = bench.build_args(cfg, 5, 'device', 0)
    explo = ExplorationPolicy(args)
    nc, ec_ = train_cli.get_network_and_environment_creator(args, explo)
    L = PAACLearner(nc, ec_, explo, args)
    L.is_chief = False
    L.start()
    lib = _lib.hip()
    lib.mt_probe_read.restype = C.c_int
    lib.mt_probe_read.argtypes = [C.c_void_p, C.c_size_t]
    buf = np.zeros(5 * 1024 * 8, dtype=np.uint64)
    for _ in range(a.updates):
        L.book.new_update()
        for t in range(L.max_local_steps):
            L.step(t)
        L.update()
    torch.cuda.synchronize()
    L.book.new_update()
    if os.environ.get('MT_ROLLOUT_AHEAD') == '1':
        # chains armed one step ahead (no replayed graph): stop after step T-2, so the last chain
        # that ran is step T-1's (a rollout step's chain, not the bootstrap's)
        for t in range(L.max_local_steps - 1):
            L.step(t)
    else:
        for t in range(L.max_local_steps):  # the last chain armed is the bootstrap forward's
            L.step(t)
    torch.cuda.synchronize()
    if a.isolated:
        E_ = cfg['ec']
        depth_ = 3 if cfg['rgb'] else 1
        g = torch.Generator(device='cuda').manual_seed(11)
        pushes = torch.randint(0, 256, (4 * E_, 84, 84, depth_), dtype=torch.uint8, device='cuda', generator=g)
        ready = torch.zeros(E_, 32, dtype=torch.int32)
        ready[:, 0] = (7 << 3) | 2
        ready = ready.cuda()
        out = torch.empty_like(L.states[0])
        for _ in range(10):
            L.network.forward_trunk_stacking(L.states[0], pushes, ready, 7, out, E_, ws_key='rollout')
        torch.cuda.synchronize()
    buf[:] = 0
    _lib.check(lib.mt_probe_read(C.c_void_p(buf.ctypes.data), buf.size), 'mt_probe_read')
    P = buf.reshape(5, 1024, 8).astype(np.int64)
    E = cfg['ec']
    ro = np.zeros(512 * 4, dtype=np.uint64)
    lib.mt_probe_read_rollout.restype = C.c_int
    lib.mt_probe_read_rollout.argtypes = [C.c_void_p, C.c_size_t]
    _lib.check(lib.mt_probe_read_rollout(C.c_void_p(ro.ctypes.data), ro.size), 'mt_probe_read_rollout')
    R = ro.reshape(512, 4)[:E].astype(np.int64)
    us = lambda x: x * 0.01  # 100 MHz ticks
    if cfg['arch'] == 'NATURE':  # the dataflow chain (nature_chain_kernel) + row fc + heads
        ch = np.zeros(512 * 4, dtype=np.uint64)
        lib.mt_probe_read_chain.restype = C.c_int
        lib.mt_probe_read_chain.argtypes = [C.c_void_p, C.c_size_t]
        _lib.check(lib.mt_probe_read_chain(C.c_void_p(ch.ctypes.data), ch.size), 'mt_probe_read_chain')
        X = ch.reshape(512, 4)[:E].astype(np.int64)
        t_last = X[:, 0].max()
        rel = lambda v: us(v - t_last)
        print('chain  per env (us): conv1 done - seen med %.2f max %.2f; conv2 done - conv1 med %.2f max %.2f; '
              'conv3 done - conv2 med %.2f max %.2f' % (
                  us(np.median(X[:, 1] - X[:, 0])), us((X[:, 1] - X[:, 0]).max()), us(np.median(X[:, 2] - X[:, 1])),
                  us((X[:, 2] - X[:, 1]).max()), us(np.median(X[:, 3] - X[:, 2])), us((X[:, 3] - X[:, 2]).max())))
        print('chain  publications seen over %.2f us (first..last); relative to the last: conv1 done max %+.2f, '
              'conv2 done max %+.2f, conv3 done max %+.2f us' % (us(t_last - X[:, 0].min()), rel(X[:, 1].max()),
                                                                  rel(X[:, 2].max()), rel(X[:, 3].max())))
        cb = np.zeros(2048 * 8, dtype=np.uint64)
        lib.mt_probe_read_chain_blocks.restype = C.c_int
        lib.mt_probe_read_chain_blocks.argtypes = [C.c_void_p, C.c_size_t]
        _lib.check(lib.mt_probe_read_chain_blocks(C.c_void_p(cb.ctypes.data), cb.size), 'mt_probe_read_chain_blocks')
        Bk = cb.reshape(2048, 8).astype(np.int64)
        n1, n2, n3 = 7 * E, 6 * E, 4 * E
        for name, lo, hi in (('conv1', 0, n1), ('conv2', n1, n1 + n2), ('conv3', n1 + n2, n1 + n2 + n3)):
            b = Bk[lo:hi]
            if name == 'conv1':
                print('%s  block phases med (us): seen->frames staged %.2f, frames->body done %.2f, stores drained '
                      '%.2f' % (name, us(np.median(b[:, 2] - b[:, 1])), us(np.median(b[:, 3] - b[:, 2])),
                                us(np.median(b[:, 4] - b[:, 3]))))
            else:
                w = b[:, 1] - b[:, 0]
                print('%s  block phases med (us): start->waited %.2f (max %.2f), waited->body done %.2f, stores '
                      'drained %.2f; starts %+.2f..%+.2f rel. last publish' % (
                          name, us(np.median(w)), us(w.max()), us(np.median(b[:, 3] - b[:, 1])),
                          us(np.median(b[:, 4] - b[:, 3])) if name == 'conv2' else 0.0, rel(b[:, 0].min()),
                          rel(b[:, 0].max())))
        e_last = int(np.argmax(X[:, 0]))
        for name, lo, bpi in (('conv2', n1, 6), ('conv3', n1 + n2, 4)):
            b = Bk[lo + bpi * e_last: lo + bpi * (e_last + 1)]
            print('%s  last env blocks: start %s waited %s done %s (rel. last publish)' % (
                name, ' '.join('%+.1f' % rel(x) for x in b[:, 0]), ' '.join('%+.1f' % rel(x) for x in b[:, 1]),
                ' '.join('%+.1f' % rel(x) for x in b[:, 3])))
        print('chain  last env %d: seen 0, conv1 %+.2f, conv2 %+.2f, conv3 %+.2f us' % (
            e_last, rel(X[e_last, 1]), rel(X[e_last, 2]), rel(X[e_last, 3])))
        nfc = 32 * 8 * ((E + 15) // 16 if E <= 32 else (E + 31) // 32)  # (row_fc: 8 K-splits, 16-env tiles up to E = 32)
        f = P[1, :nfc, :3]
        print('fc     blocks %d start %+.2f..%+.2f end %+.2f..%+.2f us (rel. last publish), block med %.2f' % (
            nfc, rel(f[:, 0].min()), rel(f[:, 0].max()), rel(f[:, 2].min()), rel(f[:, 2].max()),
            us(np.median(f[:, 2] - f[:, 0]))))
        h = P[2, :E, :4]
        print('heads  blocks %d start %+.2f..%+.2f end %+.2f..%+.2f us; phases med: slab sum %.2f, gemv %.2f, '
              'softmax+draw %.2f' % (E, rel(h[:, 0].min()), rel(h[:, 0].max()), rel(h[:, 3].min()), rel(h[:, 3].max()),
                                     us(np.median(h[:, 1] - h[:, 0])), us(np.median(h[:, 2] - h[:, 1])),
                                     us(np.median(h[:, 3] - h[:, 2]))))
        L.cleanup()
        return
    nblocks = {0: int((P[0, :, 0] != 0).sum()), 1: 16 * 8 * ((E + 15) // 16), 2: E}  # (conv: 9 per env; fc: 8 K-splits x 16-env tiles)
    t0 = P[0, :nblocks[0], 0].min()
    if R[:, 0].any():  # a pull kernel ran (non-stacking chains)
        seen, done = R[:, 0] - t0, R[:, 1] - t0
        pstart = R[::4, 2] - t0
        print('pull   per env: seen / done (us):', ' '.join('%d:%.1f/%.1f' % (e, us(seen[e]), us(done[e])) for e in range(E)))
        print('pull   start %+7.2f us (after the previous heads kernel), env words seen %+7.2f..%+7.2f us '
              '(median %+7.2f), copies done ..%+7.2f us, copy med %.2f us' % (
                  us(pstart.min()), us(seen.min()), us(seen.max()), us(np.median(seen)), us(done.max()),
                  us(np.median(done - seen))))
    c1 = P[0, :nblocks[0]]
    if c1[:, 6].any():  # conv1 sub-phases (wave 0): products issued, partials in LDS, reduced
        print('conv1  sub-phases med: mfma %.2f  partial write+barrier %.2f  reduce+act %.2f us' % (
            us(np.median(c1[:, 6] - c1[:, 1])), us(np.median(c1[:, 7] - c1[:, 6])), us(np.median(c1[:, 2] - c1[:, 7]))))
    pub = P[0, :nblocks[0], 5]
    if pub.any():  # in-kernel pull: when each conv block saw its env published (blockIdx order)
        pub = pub - t0
        print('conv   env published seen (us, per block): min %+7.2f median %+7.2f max %+7.2f; '
              'last block end - last seen %.2f us' % (us(pub.min()), us(np.median(pub)), us(pub.max()),
                                                     us(P[0, :nblocks[0], 4].max() - t0 - pub.max())))
    prev_end = None
    for k in (0, 1, 2):
        name, ph = PHASES[k]
        n = nblocks[k]
        p = P[k, :n, :len(ph) + 1]
        if a.isolated and k == 2:
            break
        start, end = p[:, 0], p[:, -1]
        line = '%-6s blocks %4d  start %+7.2f..%+7.2f us  end %+7.2f..%+7.2f us  block dur med %.2f max %.2f' % (
            name, n, us(start.min() - t0), us(start.max() - t0), us(end.min() - t0), us(end.max() - t0),
            us(np.median(end - start)), us((end - start).max()))
        if prev_end is not None:
            line += '  gap after previous kernel %.2f us' % us(start.min() - prev_end)
        print(line)
        for j, nm in enumerate(ph):
            d = p[:, j + 1] - p[:, j]
            print('    %-20s med %6.2f  p90 %6.2f  max %6.2f us' % (nm, us(np.median(d)), us(np.percentile(d, 90)),
                                                                     us(d.max())))
        prev_end = end.max()
    lb = P[4, :E * L.max_local_steps, :5]
    if lb[:, 0].any():  # the last update's loss kernel (slot 4) and the conv backward after it (slot 3)
        t4 = lb[:, 0].min()
        print('loss   blocks %4d  start %+7.2f..%+7.2f us  end %+7.2f..%+7.2f us  block dur med %.2f max %.2f' % (
            len(lb), 0.0, us(lb[:, 0].max() - t4), us(lb[:, 4].min() - t4), us(lb[:, 4].max() - t4),
            us(np.median(lb[:, 4] - lb[:, 0])), us((lb[:, 4] - lb[:, 0]).max())))
        for j, nm in enumerate(['loads + V(s_T)', 'n-step return', 'head grads', 'dz + dH stores']):
            d = lb[:, j + 1] - lb[:, j]
            print('    %-20s med %6.2f  p90 %6.2f  max %6.2f us' % (nm, us(np.median(d)), us(np.percentile(d, 90)),
                                                                     us(d.max())))
        cb = P[3, :, 0]
        cb = cb[cb > t4]
        if cb.size:
            print('conv bwd first block start %+7.2f us after the loss kernel start (loss end -> conv bwd start '
                  '%.2f us: the dense group and two boundaries)' % (us(cb.min() - t4), us(cb.min() - lb[:, 4].max())))
    L.cleanup()


if __name__ == '__main__':
    main()
