"""One rank of the data-parallel tests (launched by tests with WORLD_SIZE/RANK set).

gpu: PAACLearner on cuda:0 with torch.distributed (gloo), rank r owns global envs
     [r*ec, (r+1)*ec); after 3 updates the rank's flat parameters are saved.
cpu: the DP update protocol on the oracle (no GPU): each rank takes half of a fixed batch, the
     flat gradient is summed by all_reduce, scaled by 1/world, clipped by its global norm and
     applied with TF1 RMSProp (manette_amd.paac.PAACLearner.update's order).
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gpu_rank(out_dir):
    import train as cli
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.paac import PAACLearner
    rank = dist.get_rank()
    a = cli.get_arg_parser().parse_args([])
    a.game, a.arch, a.emulator_counts, a.emulator_workers = 'pong', 'NIPS', 8, 2
    a.runner, a.sampling, a.seed = 'native', 'device', 0
    a.debugging_folder = os.path.join(out_dir, 'r%d' % rank) + '/'
    a.max_global_steps = 1 << 40
    a.checkpoint_interval = 1 << 40
    a.env_id_offset = rank * a.emulator_counts
    explo = ExplorationPolicy(a)
    nc, ecr = cli.get_network_and_environment_creator(a, explo)
    L = PAACLearner(nc, ecr, explo, a)
    assert L.world == 2
    L.start()
    for _ in range(3):
        L.book.new_update()
        for t in range(L.max_local_steps):
            L.step(t)
        L.update()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, 'rank%d.npy' % rank), L.network.params.cpu().numpy())
    L.cleanup()


def cpu_batch():
    from oracle import nets
    spec = nets.arch_spec('NIPS', 1, 6, 3)
    P = nets.init_params(spec, 5)
    rs = np.random.RandomState(9)
    B = 8
    obs = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
    return spec, P, obs, rs.randint(0, 6, B), rs.randint(0, 3, B), rs.randn(B), rs.randn(B)


def dp_update(spec, P, obs, a, r, y, adv, world, rank, lr=0.0224):
    from oracle import nets, optim
    names = [n for (n, _, _) in spec['vars']]
    B = len(a)
    lo, hi = rank * B // world, (rank + 1) * B // world
    _, G, _ = nets.loss_and_grads(spec, P, obs[lo:hi], a[lo:hi], r[lo:hi], y[lo:hi], adv[lo:hi], 0.02)
    flat = torch.from_numpy(np.concatenate([G[n].reshape(-1) for n in names]).astype(np.float32))
    if world > 1:
        dist.all_reduce(flat)
    g = flat.numpy() * np.float32(1.0 / world)
    norm = optim.global_norm([g])
    s = optim.clip_scale(norm, 3.0)
    w = np.concatenate([P[n].reshape(-1) for n in names]).astype(np.float32)
    ms = np.ones_like(w)
    mom = np.zeros_like(w)
    optim.rmsprop_apply(w, ms, mom, g * s, np.float32(lr))
    return w


def cpu_rank(out_dir):
    spec, P, obs, a, r, y, adv = cpu_batch()
    w = dp_update(spec, P, obs, a, r, y, adv, dist.get_world_size(), dist.get_rank())
    np.save(os.path.join(out_dir, 'cpu_rank%d.npy' % dist.get_rank()), w)


if __name__ == '__main__':
    out_dir, mode = sys.argv[1], sys.argv[2]
    if mode == 'gpu':
        torch.cuda.set_device(0)
    dist.init_process_group('gloo')
    try:
        gpu_rank(out_dir) if mode == 'gpu' else cpu_rank(out_dir)
    finally:
        dist.destroy_process_group()
