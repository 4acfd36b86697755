"""One rank of the data-parallel tests (launched by tests with WORLD_SIZE/RANK set, or alone for
the single-process reference run).

gpu: PAACLearner on cuda:0 over the benchmarked path (native step, device sampling, resized
     staging, pipelined, update replayed as a hipGraph from the second update on). The job has
     ENVS global envs; rank r owns [r*ENVS/W, (r+1)*ENVS/W) (the runners.py:17-18 split over
     ranks), the gradient is summed by the learner's comm (torch.distributed on the gloo group:
     the ranks share one GPU, which RCCL does not allow) once per update. After every update
     the rank saves its parameters, its envs' states, global_step and episode records, so the
     test can compare a W-rank run with the single process that owns all ENVS envs.
resume: a W-rank run is stopped (rank 0 checkpoints) and resumed from rank 0's checkpoint.
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

ENVS = {'NIPS': 16, 'LSTM': 8}  # global envs of the job per arch
UPDATES = 4


def _learner(out_dir, rank, world, comm='torch', arch='NIPS'):
    import train as cli
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.paac import PAACLearner
    from manette_amd.synthetic import SyntheticBank
    a = cli.get_arg_parser().parse_args([])
    ec = ENVS[arch] // world
    a.game = 'breakout' if arch == 'NIPS' else 'ms_pacman'  # (configs[4]: MsPacman LSTM + FiGAR10)
    a.arch, a.emulator_counts, a.emulator_workers = arch, ec, 2
    a.max_repetition, a.nb_choices = 10, 11
    a.runner, a.sampling, a.seed, a.staging, a.pipeline = 'native', 'device', 0, 'resized', True
    a.comm = comm
    a.debugging_folder = os.path.join(out_dir, '%s_w%d_r%d' % (arch, world, rank)) + '/'
    a.max_global_steps = 1 << 40
    a.checkpoint_interval = 1 << 40
    a.env_id_offset = rank * ec
    explo = ExplorationPolicy(a)
    nc, ecr = cli.get_network_and_environment_creator(a, explo)
    # short episodes, so resets (and their global_step records) happen inside the run
    ecr.create_bank = lambda first, n: SyntheticBank(ecr.rank_offset + first, n, episode_len=23)
    L = PAACLearner(nc, ecr, explo, a)
    assert L.world == world
    L.start()
    return L


def gpu_rank(out_dir, rank, world, arch='NIPS'):
    L = _learner(out_dir, rank, world, arch=arch)
    rec = dict(params=[], states=[], gs=[], nz=[])
    params0 = L.network.params.cpu().numpy().copy()
    try:
        for _ in range(UPDATES):
            L.book.new_update()
            L.rollout()
            L.update()
            torch.cuda.synchronize()
            rec['params'].append(L.network.params.cpu().numpy().copy())
            rec['states'].append(L.states[1:].cpu().numpy().copy())
            rec['gs'].append(L.global_step)
            if L.lstm_bool:  # the memory windows' leading-zero counts (device-derived, paac.py:79-83)
                rec['nz'].append(L.nz_d.cpu().numpy().copy())
        L.book.drain()
        assert L._graphs is not None  # the graph path ran
        if world > 1 and arch != 'LSTM':  # the data-parallel update: two gradient buckets all-reduced on a side
            # stream, the first graph launched by the rollout's last step
            assert L._buckets is not None and len(L._graphs) == 3 and L._rollout_update == 'first' 
        elif world > 1:  # LSTM: backward | all-reduce of the whole gradient | apply (+ slot / nz carry)
            assert L._buckets is None and len(L._graphs) == 2 and not L._update_in_rollout
        np.savez(os.path.join(out_dir, '%s_w%d_r%d.npz' % (arch, world, rank)), params0=params0,
                 params=np.stack(rec['params']),
                 states=np.stack(rec['states']), gs=np.array(rec['gs']), nz=np.array(rec['nz']),
                 episodes=np.array(L.book.episodes, dtype=np.float64).reshape(-1, 3))
    finally:
        L.cleanup()


def resume_rank(out_dir, rank, world):
    """a W-rank run resumed from rank 0's checkpoint (the other ranks' folders have
    none, as train.py gives them rank<r>/ folders) continues from rank 0's step on every rank with
    rank 0's parameters, and the replicas stay identical."""
    L = _learner(out_dir, rank, world)
    try:
        for _ in range(2):
            L.book.new_update()
            L.rollout()
            L.update()
        saved = L.global_step
    finally:
        L.cleanup()  # rank 0 writes its checkpoint (save_vars(True))
    dist.barrier()
    L = _learner(out_dir, rank, world)
    try:
        start = L.global_step
        p_start = L.network.params.cpu().numpy().copy()
        for _ in range(2):
            L.book.new_update()
            L.rollout()
            L.update()
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, 'resume_r%d.npz' % rank), saved=saved, start=start, end=L.global_step,
                 p_start=p_start, params=L.network.params.cpu().numpy())
    finally:
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
    arch = sys.argv[3] if len(sys.argv) > 3 else 'NIPS'
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if mode in ('gpu', 'resume'):
        torch.cuda.set_device(0)
    if world == 1 and mode == 'gpu':  # the single process owning every env
        gpu_rank(out_dir, 0, 1, arch)
        sys.exit(0)
    dist.init_process_group('gloo')
    try:
        if mode == 'gpu':
            gpu_rank(out_dir, dist.get_rank(), world, arch)
        elif mode == 'resume':
            resume_rank(out_dir, dist.get_rank(), world)
        else:
            cpu_rank(out_dir)
    finally:
        dist.destroy_process_group()
