"""bench.py's trunk_batch_sweep launch alone (mt_forward_trunk at a large batch) for rocprofv3
passes: random-init NIPS weights of the bench config, --reps launches at --envs.
    python tools/sweep_only.py [--config pong-nips --envs 4096 --reps 10]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='pong-nips')
    ap.add_argument('--envs', type=int, default=4096)
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    import torch
    import bench
    from manette_amd.network import DeviceNetwork
    from manette_amd.environment_creator import MINIMAL_ACTIONS
    cfg = bench.CONFIGS[a.config]
    net = DeviceNetwork(dict(arch=cfg['arch'], rgb=cfg['rgb'], num_actions=MINIMAL_ACTIONS[cfg['game']],
                             nb_choices=cfg['nb_choices']))
    net.init_params(0)
    depth = 3 if cfg['rgb'] else 1
    g = torch.Generator(device='cuda').manual_seed(7)
    # (mt_forward_trunk reads a window of 5 frames per row for the LSTM arch: [B][5][84][84][C])
    shape = (a.envs, 5, 84, 84, 4 * depth) if cfg['arch'] == 'LSTM' else (a.envs, 84, 84, 4 * depth)
    obs = torch.randint(0, 256, shape, dtype=torch.uint8, device='cuda', generator=g)
    for _ in range(a.reps):
        net.forward_trunk(obs, a.envs, ws_key='sweep')
    torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()
