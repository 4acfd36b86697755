"""The roofline launch alone (for rocprofv3 PMC / kernel-trace passes): bench.py's stacking trunk
(mt_forward_trunk_stacking: nips_conv_kernel<C, true> in-kernel-pull form + nips_fc_kernel<C>, or
for gray NATURE nature_chain_kernel + row_fc_kernel; PWYX stack_conv1_kernel + conv2 .. conv4 +
row_fc_kernel; every env published, pushes in HBM; LSTM: mt_lstm_frames_forward of a step's E new frames) at the
workload's E, --reps launches back to back, random-init weights of the bench config.  python tools/trunk_only.py [--config pong-nips --reps 50]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='pong-nips')
    ap.add_argument('--reps', type=int, default=50)
    a = ap.parse_args()
    import torch
    import bench
    from manette_amd.network import DeviceNetwork
    from manette_amd.environment_creator import MINIMAL_ACTIONS
    cfg = bench.CONFIGS[a.config]
    assert cfg['arch'] in ('NIPS', 'PWYX', 'LSTM') or (cfg['arch'] == 'NATURE' and not cfg['rgb'])
    depth = 3 if cfg['rgb'] else 1
    E = cfg['ec']
    net = DeviceNetwork(dict(arch=cfg['arch'], rgb=cfg['rgb'], num_actions=MINIMAL_ACTIONS[cfg['game']],
                             nb_choices=cfg['nb_choices']))
    net.init_params(0)
    g = torch.Generator(device='cuda').manual_seed(3)
    if cfg['arch'] == 'LSTM':  # bench.py's LSTM roofline launch: a step's E new frames through the frame
        T = 5                  # trunk + the cell's x-product (mt_lstm_frames_forward, rows 1 + 5E ..)
        fstore = torch.randint(0, 256, (1 + (T + 5) * E, 84, 84, 4 * depth), dtype=torch.uint8, device='cuda',
                               generator=g)
        fstore[0].zero_()
        net.lstm_workspace(E, T)
        for _ in range(a.reps):
            net.lstm_frames_forward(fstore, 1 + 5 * E, E, E, T)
        torch.cuda.synchronize()
        print('ok', a.reps, 'launches')
        return
    prev = torch.randint(0, 256, (E, 84, 84, 4 * depth), dtype=torch.uint8, device='cuda', generator=g)
    pushes = torch.randint(0, 256, (4 * E, 84, 84, depth), dtype=torch.uint8, device='cuda', generator=g)
    counts = torch.ones(E, dtype=torch.int32) if cfg['max_repetition'] == 0 else \
        torch.from_numpy(np.random.RandomState(5).randint(1, 5, E).astype(np.int32))  # as bench.py
    ready = torch.zeros(E, 32, dtype=torch.int32)
    ready[:, 0] = (7 << 3) | counts
    ready = ready.cuda()
    out = torch.empty_like(prev)
    for _ in range(a.reps):
        net.forward_trunk_stacking(prev, pushes, ready, 7, out, E)
    torch.cuda.synchronize()
    print('ok', a.reps, 'launches')


if __name__ == '__main__':
    main()
