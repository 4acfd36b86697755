"""Benchmark of the PAAC+FiGAR rollout/update hot path on MI355X (BASELINE.json metric).

One "step" = one PAAC update: T rollout macro-steps over every env of the rank (device
forward, sampling, native emulator step, H2D of the pushed screens, device preprocess, host
bookkeeping) + bootstrap forward + n-step returns + fused loss backward + [RCCL all-reduce] +
clip/RMSProp. value = env-steps/s of the whole job = world * ec * T * K / max-over-ranks time.
Workload (N=1 default): BASELINE.json configs[1], Pong NIPS ec=32 ew=8 t_max=5, synthetic
84x84 frames (manette_amd/synthetic.py), random-init weights.

  python bench.py [--gpus N --steps K --warmup W --config pong-nips --sampling device]
  N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import re
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # BASELINE.json configs[1..4]; per-rank ec (weak scaling: ec per GPU fixed)
    'pong-nips': dict(game='pong', arch='NIPS', ec=32, ew=8, max_repetition=0, nb_choices=1, rgb=False),
    'breakout-nature-figar': dict(game='breakout', arch='NATURE', ec=64, ew=8, max_repetition=10,
                                  nb_choices=11, rgb=False),
    'seaquest-nature': dict(game='seaquest', arch='NATURE', ec=32, ew=8, max_repetition=0, nb_choices=1,
                            rgb=False),
    # the CLI's default arch and the arch of every FiGAR checkpoint
    'breakout-pwyx-figar-rgb': dict(game='breakout', arch='PWYX', ec=32, ew=8, max_repetition=10,
                                    nb_choices=11, rgb=True),
    # BASELINE.json configs[4]: MsPacman LSTM + FiGAR10, ec=256 over 8 GPUs = 32 per GPU
    'mspacman-lstm-figar': dict(game='ms_pacman', arch='LSTM', ec=32, ew=8, max_repetition=10, nb_choices=11,
                                rgb=False),
}
# BASELINE.json configs[0]: the reference's CPU-only case, timed only in the cpu_baseline leg
CPU_CONFIG0 = dict(game='pong', arch='NIPS', ec=4, ew=2, max_repetition=0, nb_choices=1, rgb=False)
MI355X_FP32_TFLOPS = 157.3   # dense fp32 (vector = MFMA), MI355X_MICROARCH.md
MI355X_HBM_GBS = 8000.0      # HBM3E peak, MI355X_MICROARCH.md


def load_pmc(config, kernels, name='pmc_trunk_%s.json'):
    """HBM bytes per roofline launch (the sum over its kernels of bytes per launch) from the
    committed PMC summary of this workload's roofline launch (profiles/pmc_trunk_<config>.json,
    written by tools/pmc_trunk.sh + tools/pmc_summary.py on tools/trunk_only.py: the same
    kernels, grid and inputs bench.py times), or None when a kernel is missing from it. A name
    matches itself and its template instantiations, all of them summed (PWYX: conv2 .. conv4 are
    three dconv_kernel<...> instantiations)."""
    if not kernels:
        return None
    path = os.path.join(ROOT, 'profiles', name % config)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if kernels == '*':  # every kernel of the roofline launch (the profiled program runs nothing else but
        # torch's allocation fills and copies)
        kernels = sorted({re.sub(r'^void ', '', k).split('<')[0] for k in d
                          if not k.startswith('__amd') and 'at::native' not in k})
    total = 0
    for kern in kernels:
        name_of = lambda k: k.replace('void ', '')
        hit = [v for k, v in d.items() if name_of(k) == kern or name_of(k).startswith(kern + '<')]
        if not hit:
            return None
        total += sum(v['hbm_bytes'] for v in hit)
    return dict(hbm_bytes=total, source='profiles/' + name % config)


def conv_out(h, k, s):
    return (h - k) // s + 1


def arch_flops(arch, depth, A, R):
    """Per layer: (kind, forward FLOPs = 2*MACs, weight floats, output floats) for NIPS / NATURE /
    PWYX / LSTM (networks.py:178-278), per frame for the trunk ('conv', LSTM 'lstm_x') and per
    sample for the rest. The LSTM build computes each distinct frame once (frame store), so its
    per-frame and per-window costs are counted separately (train_pass_flops)."""
    C = 4 * depth
    if arch == 'NIPS':
        convs = [(8, 4, C, 16, 'VALID', False), (4, 2, 16, 32, 'VALID', False)]
        F = 256
    elif arch == 'NATURE':
        convs = [(8, 4, C, 32, 'VALID', False), (4, 2, 32, 64, 'VALID', False), (3, 1, 64, 64, 'VALID', False)]
        F = 512
    else:
        convs = [(5, 1, C, 32, 'SAME', True), (5, 1, 32, 32, 'SAME', True), (4, 1, 32, 64, 'SAME', True),
                 (3, 1, 64, 64, 'SAME', False)]
        F = 128 if arch == 'LSTM' else 512
    h = 84
    layers = []
    for (k, s, cin, cout, pad, pool) in convs:
        h = conv_out(h, k, s) if pad == 'VALID' else -(-h // s)
        layers.append(('conv', 2.0 * h * h * cout * k * k * cin, k * k * cin * cout + cout, h * h * cout))
        if pool:
            h //= 2
    flat = h * h * convs[-1][3]
    if arch == 'LSTM':
        nh = 32
        layers.append(('lstm_x', 2.0 * flat * 4 * nh, flat * 4 * nh, 4 * nh))
        layers.append(('lstm_h', 5 * 2.0 * nh * 4 * nh, (nh + 1) * 4 * nh, 5 * 4 * nh))
        layers.append(('proj', 2.0 * nh * nh, nh * nh + nh, nh))
        flat = nh
    layers.append(('fc', 2.0 * flat * F, flat * F + F, F))
    layers.append(('heads', 2.0 * F * (1 + A + R), F * (1 + A + R) + 1 + A + R, 1 + A + R))
    return layers


FRAME_LAYERS = ('conv', 'lstm_x')


def train_pass_flops(layers, N, frame_rows=None):
    """FLOPs the update's train pass executes: the rollout already ran the forward of every row
    (mt_forward_rows / the LSTM frame store), so it is the backward only — dW of every layer and
    dX of every layer except the input conv (2x the forward minus conv1's forward), per row; LSTM:
    that of the frame_rows distinct frames + the N windows' cell / dense / heads."""
    if frame_rows is None:  # the forward is the rollout's: backward only (dW all, dX all but conv1)
        fwd = sum(l[1] for l in layers)
        return N * (2 * fwd - layers[0][1])
    per_frame = sum(l[1] for l in layers if l[0] in FRAME_LAYERS)
    per_win = sum(l[1] for l in layers if l[0] not in FRAME_LAYERS)
    return frame_rows * (2 * per_frame - layers[0][1]) + N * 2 * per_win


# CLOCK_BOOTTIME windows (ns) of each labelled graph_time measurement's timed replays: the clock of
# rocprofv3's dispatch timestamps, so tools/rocpd_summary.py can restrict a profile of this same
# command to the dispatches a bench number was computed from ("profile_windows" in the JSON line)
PROFILE_WINDOWS = {}


def graph_time(fn, inner, reps=5, label=None):
    """Device time per call of fn (which launches on torch's current stream): `inner` calls are
    captured as ONE hipGraph on a side stream, replayed once to warm up and then `reps` times, each
    replay between a HIP event pair on that stream. The kernels run back to back with no host
    launch gap (an eager loop of small launches measures the host's launch rate on a loaded box:
    BENCH_r02's 32 us vs 14 us). Returns the per-call microseconds of each replay."""
    import ctypes as C
    import torch
    from manette_amd import _lib
    lib = _lib.hip()
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    side.wait_stream(cur)
    torch.cuda.synchronize()
    out = []
    with torch.cuda.stream(side):
        sp = C.c_void_p(side.cuda_stream)
        _lib.check(lib.mt_graph_begin(sp), 'mt_graph_begin')
        g = C.c_void_p()
        try:
            for _ in range(inner):
                fn()
        finally:
            rc = lib.mt_graph_end(sp, C.byref(g))
        _lib.check(rc, 'mt_graph_end')
        try:
            _lib.check(lib.mt_graph_launch(g, sp), 'mt_graph_launch')
            side.synchronize()  # (the warm-up replay stays outside the labelled window)
            t0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
            evs = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(side)
                _lib.check(lib.mt_graph_launch(g, sp), 'mt_graph_launch')
                b.record(side)
                evs.append((a, b))
            side.synchronize()
            if label:
                PROFILE_WINDOWS[label] = [t0, time.clock_gettime_ns(time.CLOCK_BOOTTIME), inner * reps]
            out = [a.elapsed_time(b) * 1e3 / inner for a, b in evs]
        finally:
            lib.mt_graph_destroy(g)
    cur.wait_stream(side)
    return out


def stats_us(xs):
    xs = sorted(xs)
    return {'min_us': round(xs[0], 2), 'median_us': round(xs[len(xs) // 2], 2), 'max_us': round(xs[-1], 2),
            'n': len(xs)}


def launch_breakdown(fn, inner=20, reps=3):
    """Per-launch device time of a multi-launch call fn (the update's backward): the call is timed
    (graph_time) with only its first k launches issued (mt_launch_window(0, k)), k = 1..L; launch
    k's time = t(k) - t(k-1), each including its dependent kernel boundary."""
    from manette_amd import _lib
    lib = _lib.hip()
    lib.mt_launch_window(0, -1)
    try:
        fn()
    finally:
        L = lib.mt_launch_window(-1, -1)
    prev, out = 0.0, []
    for k in range(1, L + 1):
        try:
            t = float(np.median(graph_time(lambda: (lib.mt_launch_window(0, k), fn()), inner, reps, label=f'train_launches_{k}')))
        finally:
            lib.mt_launch_window(-1, -1)
        out.append(t - prev)
        prev = t
    return out, prev


def build_args(cfg, T, sampling, seed, debugging_folder=None):
    import train as train_cli
    a = train_cli.get_arg_parser().parse_args([])
    a.game = cfg['game']
    a.arch = cfg['arch']
    a.emulator_counts = cfg['ec']
    a.emulator_workers = cfg['ew']
    a.max_repetition = cfg['max_repetition']
    a.nb_choices = cfg['nb_choices']
    a.rgb = cfg['rgb']
    a.max_local_steps = T
    a.max_global_steps = 1 << 62
    a.checkpoint_interval = 1 << 62
    a.sampling = sampling
    a.runner = 'native'
    a.seed = seed
    a.debugging_folder = debugging_folder or tempfile.mkdtemp(prefix='manette_bench_')
    return a


def make_learner(config, T=5, sampling='device', seed=0, staging='resized', pipeline=True, update_graph=True,
                 rank=0, debugging_folder=None, episode_len=None, comm='rccl', dp_force=False, pin_threads='auto'):
    """The benchmarked learner of `config` (BASELINE.json configs[1..4]; tests/test_e2e_gpu.py
    checks exactly this path against the oracle). episode_len: a shorter synthetic episode (tests
    exercise resets); None = the synthetic default. dp_force: the data-parallel update (bucketed
    side-stream all-reduce between three update graphs) even at world 1 (paac.PAACLearner.dp)."""
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.paac import PAACLearner
    import train as train_cli
    cfg = CONFIGS[config]
    args = build_args(cfg, T, sampling, seed, debugging_folder)
    args.env_id_offset = rank * cfg['ec']
    args.staging = staging
    args.pipeline = pipeline
    args.update_graph = update_graph
    args.comm = comm
    args.dp_force = dp_force
    args.pin_threads = pin_threads
    np.random.seed(1234 + rank)
    explo = ExplorationPolicy(args)
    net_creator, env_creator = train_cli.get_network_and_environment_creator(args, explo)
    if episode_len is not None:
        from manette_amd.synthetic import SyntheticBank
        env_creator.create_bank = lambda first, n: SyntheticBank(env_creator.rank_offset + first, n, rgb=cfg['rgb'],
                                                                 episode_len=episode_len)
    learner = PAACLearner(net_creator, env_creator, explo, args)
    learner.is_chief = False  # no checkpoint writes from the benchmark
    return learner, args


def settle_updates(one_update, seconds, world, dist, cap=5000):
    """Untimed updates for `seconds` of rank 0's clock; returns their count. World > 1: rank 0
    decides before every update and broadcasts it over the control channel, so every rank runs the
    same updates — a rank one update ahead of rank 0 would wait in that update's all-reduce while
    rank 0 waits in the next control-channel collective (the 2-rank rehearsal hung that way when
    each rank read its own clock)."""
    import torch
    n = 0
    if seconds <= 0:
        return 0
    t_s = time.perf_counter()
    while n < cap:
        stop = time.perf_counter() - t_s >= seconds
        if world > 1:
            flag = torch.tensor([1 if stop else 0], dtype=torch.int64)
            dist.broadcast(flag, 0)
            stop = bool(flag.item())
        if stop:
            break
        one_update()
        n += 1
    return n


def cpu_baseline(cfg, T, seconds, rank):
    """The oracle ("port") restated reference loop on host cores: the reference's host loop and
    process runners (mp.Queue barrier) from oracle/host_loop.py, a torch-CPU fp32 network with the
    TF1 clip/RMSProp update (oracle/torch_cpu.py, standing in for TF1's CPU kernels), the same
    synthetic emulators with CPU preprocess. Bounded sample: as many updates as fit in ~seconds."""
    from oracle import host_loop, policy
    from manette_amd.environment_creator import MINIMAL_ACTIONS
    from manette_amd.synthetic import SyntheticEmulator
    A = MINIMAL_ACTIONS[cfg['game']]
    ec, ew = cfg['ec'], cfg['ew']
    tab = policy.tab_repetitions(cfg['max_repetition'], cfg['nb_choices'])
    cores = len(os.sched_getaffinity(0))
    omp = int(os.environ.get('OMP_NUM_THREADS', cores))
    cores = min(cores, omp)
    emus = [SyntheticEmulator(i, A, rgb=cfg['rgb']) for i in range(ec)]
    from oracle.torch_cpu import TorchCPUNetwork
    net = TorchCPUNetwork(cfg['arch'], 3 if cfg['rgb'] else 1, A, cfg['nb_choices'], seed=0, threads=cores)
    np.random.seed(1234)

    class Timed(host_loop.HostLoop):
        pass

    net_s = [0.0]
    orig_fwd = net.forward

    def fwd_hook(*a, **k):
        t = time.perf_counter()
        r = orig_fwd(*a, **k)
        if t_start[0] is not None:
            net_s[0] += time.perf_counter() - t
        return r
    net.forward = fwd_hook
    loop = Timed(emus, net, tab, A, max_local_steps=T, workers=ew, record=False, lstm=cfg['arch'] == 'LSTM')
    # warm up one update, then time whole updates until `seconds` elapse (at most 2000)
    steps_per_update = ec * T
    t_start = [None]
    n_upd = [0]
    orig_train = net.train

    def train_hook(*a, **k):
        t = time.perf_counter()
        orig_train(*a, **k)
        if t_start[0] is not None:
            net_s[0] += time.perf_counter() - t
        n_upd[0] += 1
        if n_upd[0] == 1:
            t_start[0] = time.perf_counter()
        elif time.perf_counter() - t_start[0] > seconds or n_upd[0] >= 2001:
            loop.global_step = 1 << 62  # stop after this update
    net.train = train_hook
    loop.run(1 << 61)
    elapsed = time.perf_counter() - t_start[0]
    timed = n_upd[0] - 1
    return dict(value=timed * steps_per_update / elapsed, unit='env-steps/s', cores=cores, kind='port',
                _net_ms_per_update=1e3 * net_s[0] / max(timed, 1),
                sample='%d PAAC updates (ec=%d, t_max=%d, %s) after 1 warm-up, %d emulator worker '
                       'processes, torch-CPU fp32 network on %d threads, %.1f s' % (timed, ec, T, cfg['arch'], ew, cores, elapsed))


def time_allreduce(learner, world, dist):
    """Per-rank device time of the RCCL all-reduce of each gradient bucket (paac._bucketed_update) and
    of the whole gradient, on a scratch copy: barrier, then HIP events around mt_allreduce on the
    rank's stream, 20 calls each; medians gathered to every rank. Never fails the bench line (a
    failure is reported in the object)."""
    import torch
    try:
        scratch = learner.network.grad.clone()
        k = getattr(learner, '_buckets', None)
        parts = {'whole': scratch}
        if k:
            parts['dense+heads (bucket 1)'] = scratch[k:]
            parts['conv (bucket 2)'] = scratch[:k]
        mine = {}
        for name, t in parts.items():
            for _ in range(3):
                learner.comm.allreduce(t)
            xs = []
            for _ in range(20):
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                learner.comm.allreduce(t)
                e1.record()
                e1.synchronize()
                xs.append(e0.elapsed_time(e1) * 1e3)
            mine[name] = {'bytes': 4 * t.numel(), 'median_us': round(float(np.median(xs)), 2),
                          'min_us': round(float(np.min(xs)), 2)}
        every = [None] * world
        dist.all_gather_object(every, mine)
        return {'per_rank': every, 'note': 'RCCL in-place sum of the bucket alone (barrier, then HIP events around '
                                           'mt_allreduce on the rank\'s stream; 20 calls); in the update the buckets '
                                           'run on a side stream beside the conv backward'}
    except Exception as e:  # (reported, not raised: the timed value above is already measured)
        return {'error': repr(e)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', default='pong-nips', choices=sorted(CONFIGS))
    ap.add_argument('--t_max', type=int, default=5)
    ap.add_argument('--sampling', default='device', choices=['device', 'host'])
    ap.add_argument('--cpu_seconds', type=float, default=15.0)
    ap.add_argument('--no_cpu_baseline', action='store_true')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--step_impl', default='native', choices=['native', 'python'],
                    help='macro-step orchestration: native (mt_rollout_step) or Python')
    ap.add_argument('--staging', default='resized', choices=['in_place', 'zero_copy', 'copy', 'pooled', 'resized'])
    ap.add_argument('--no_pipeline', dest='pipeline', action='store_false',
                    help='disable MT_ROLLOUT_PIPELINED (on by default)')
    ap.add_argument('--no_update_graph', dest='update_graph', action='store_false',
                    help='launch the update eagerly instead of replaying it as a hipGraph')
    ap.add_argument('--measure_updates', type=int, default=20,
                    help='updates after the timed region during which the rollout times its trunk kernels in place')
    ap.add_argument('--comm', default='rccl', choices=['rccl', 'torch'],
                    help='data-parallel gradient all-reduce (torch: torch.distributed on gloo — a rehearsal of the '
                         'N > 1 path on one GPU with MT_BENCH_SHARED_GPU=1, every rank on cuda:0)')
    ap.add_argument('--dp_force', action='store_true',
                    help='the data-parallel update at world 1 (RCCL communicator, bucketed side-stream all-reduce '
                         'between three update graphs, the learner launching the update): the per-GPU cost of the '
                         'N-GPU path (paac.PAACLearner.dp)')
    ap.add_argument('--pin_threads', default='auto', choices=['auto', 'slice', 'pin', 'on', 'off'],
                    help='host-thread placement (manette_amd/placement.py); auto: pinned when several ranks share '
                         'the node')
    ap.add_argument('--settle_s', type=float, default=1.0,
                    help='seconds of untimed updates before the warmup steps (host emulator threads, CPU clocks and '
                         'the graphs reach their steady state; the 5-update warmup of a 20-update run did not)')
    ap.add_argument('--trunk_sweep', default='256,1024,4096',
                    help='extra batch sizes the trunk kernel is timed at after the run ("" = none)')
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(0 if os.environ.get('MT_BENCH_SHARED_GPU') == '1' else local)
    if world > 1:  # control channel (barriers, max-over-ranks time, RCCL unique id); data: mt_allreduce
        dist.init_process_group('gloo')
    cfg = CONFIGS[a.config]
    T = a.t_max
    learner, args = make_learner(a.config, T, a.sampling, a.seed, a.staging, a.pipeline, a.update_graph, rank,
                                 comm=a.comm, dp_force=a.dp_force, pin_threads=a.pin_threads)
    learner.start()
    learner_dp = learner.dp
    if a.step_impl == 'python' and learner.native_step is not None:
        from manette_amd import _lib
        _lib.hip().mt_rollout_destroy(learner.native_step)
        learner.native_step = None

    def one_update():
        learner.book.new_update()
        learner.rollout()
        learner.update()

    # settle: untimed updates for --settle_s seconds (every rank the same count, rank 0's), so the
    # W warmup steps and the K timed ones start from the steady state; the graphs are captured and
    # registered within the first 3 updates, the rest is the host side (emulator threads' caches and
    # clocks) — a 5-update warmup left the r04 driver run ramping 603k -> 713k over its 20 updates
    if world > 1 or learner_dp:  # the first update's all-reduce, bounded like the communicator's setup
        from manette_amd import comm as comm_
        with comm_.Deadline('the first data-parallel update (all-reduce of the gradient)', rank, world):
            one_update()
            torch.cuda.synchronize()
    settle = settle_updates(one_update, a.settle_s, world, dist)
    for _ in range(a.warmup):
        one_update()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stats = None
    phase_names = ['launch_and_wait_us', 'emulators_us', 'bookkeeping_us', 'upload_enqueue_us']
    if learner.native_step is not None:
        import ctypes as C
        from manette_amd import _lib
        stats = (C.c_double * 7)()
        _lib.hip().mt_rollout_stats_ex(learner.native_step, stats, 7, 1)
    runner_stats = getattr(learner.runners, 'stats', None)  # (native runner) host-phase split
    if runner_stats:
        runner_stats(reset=True)
    w = max(1, a.steps // 4)  # sub-windows of the timed region
    win_stats = []  # per sub-window: the host phases of its macro-steps (read + reset at its end)
    t0 = time.perf_counter()
    marks = []  # host clock after each update: the value of sub-windows of the timed region
    for k in range(a.steps):
        one_update()
        marks.append(time.perf_counter())
        if stats is not None and (k + 1) % w == 0:
            _lib.hip().mt_rollout_stats_ex(learner.native_step, stats, 7, 1)
            win_stats.append(list(stats))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    emu_split = runner_stats() if runner_stats else None
    if stats is not None:
        _lib.hip().mt_rollout_stats_ex(learner.native_step, stats, 7, 0)
        tot = [sum(ws_[i] for ws_ in win_stats) + stats[i] for i in range(7)]
        n = max(tot[4], 1)
        step_phases = {k: round(tot[i] / n, 2) for i, k in enumerate(phase_names)}
        # launch_and_wait = host launches (this step's forward if not armed + the chains armed
        # ahead) + the spin for this step's sampled indices
        step_phases['of_which_enqueue_us'] = round(tot[5] / n, 2)
        step_phases['of_which_wait_us'] = round(tot[6] / n, 2)
        window_phases = [{k: round(ws_[i] / max(ws_[4], 1), 2) for i, k in enumerate(phase_names[:2])}
                         for ws_ in win_stats]
    else:
        step_phases = None
        window_phases = None
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    # host-thread placement of every rank (manette_amd/placement.py): cores, threads, pinning
    from manette_amd import placement as placement_
    threads = placement_.report(learner.placement) if learner.placement else None
    if world > 1:
        every_threads = [None] * world
        dist.all_gather_object(every_threads, threads)
    else:
        every_threads = [threads]
    # ---- measurements after the timed region (none of them is part of `value`) ----------------
    prof = {}
    # (1) roofline kernels where the timed loop runs them: the native rollout records an event
    #     pair around every step forward's trunk launches (NIPS: the stacking conv kernel + the
    #     dense kernel, between the pull and heads kernels of the pipelined chain) over
    #     --measure_updates more updates (mt_rollout_trunk_timing)
    inloop_us = None
    if learner.native_step is not None and a.measure_updates > 0:
        import ctypes as C
        from manette_amd import _lib
        lib = _lib.hip()
        tot, cnt = C.c_double(), C.c_int64()
        _lib.check(lib.mt_rollout_trunk_timing(learner.native_step, 1, C.byref(tot), C.byref(cnt)))
        for _ in range(a.measure_updates):
            one_update()
        torch.cuda.synchronize()
        _lib.check(lib.mt_rollout_trunk_timing(learner.native_step, 0, C.byref(tot), C.byref(cnt)))
        if cnt.value:
            inloop_us = tot.value / cnt.value
    # (2) data parallel: the replicas must hold identical parameters after the run (checked before
    #     the kernel timings below, which run clip + RMSProp again)
    replicas = None
    if world > 1:
        pf = learner.network.params.double()
        ck = torch.stack([pf.sum(), (pf * torch.arange(pf.numel(), device=pf.device, dtype=torch.float64)).sum()]).cpu()
        allck = [torch.zeros_like(ck) for _ in range(world)]
        dist.all_gather(allck, ck)
        replicas = all(torch.equal(x, allck[0]) for x in allck)
    # (2b) data parallel: the RCCL all-reduce of each gradient bucket (and of the whole gradient) on
    #      its own, every rank timing it with HIP events on its stream (in the update the buckets run
    #      on a side stream beside the conv backward: paac._bucketed_update); per-rank medians
    allreduce = None
    if world > 1 and getattr(learner.comm, 'kind', None) == 'rccl':
        allreduce = time_allreduce(learner, world, dist)
    # (3) kernels in isolation, each as a hipGraph of back-to-back calls replayed 5 times between
    #     HIP event pairs on its stream (graph_time: no host launch gaps); min / median per call
    E = cfg['ec']
    net = learner.network
    depth_ = 3 if cfg['rgb'] else 1
    stacking = getattr(learner, 'slot0_in_rollout', False)
    # PWYX: the rollout steps' conv1 launch pulls + stacks each env (stack_conv1_kernel), so the in-loop
    # trunk window includes the emulators: the roofline times the stacking trunk with every env published
    frame_stack = not learner.lstm_bool and getattr(learner, 'frame_stack_in_rollout', False)
    # the update's train pass (fused returns + loss + backward of the last rollout)
    bwd = learner.train_backward if learner.lstm_bool else learner._update_backward
    prof['train_pass'] = graph_time(bwd, 20, label='train_pass')
    # launch by launch (mt_launch_window numbers every launch of the backward, LSTM included)
    prof['train_launches'] = launch_breakdown(bwd)[0]
    # A11: clip + RMSProp alone (the norm partials the backward left; world > 1 adds mt_grad_sumsq)
    prof['clip_rmsprop'] = graph_time(lambda: net.apply_gradients(partials_ready=True), 40, label='clip_rmsprop')
    gen = torch.Generator(device='cuda').manual_seed(11)
    pushes = torch.randint(0, 256, (4 * E, 84, 84, depth_), dtype=torch.uint8, device='cuda', generator=gen)
    counts = torch.ones(E, dtype=torch.int32) if cfg['max_repetition'] == 0 else \
        torch.from_numpy(np.random.RandomState(5).randint(1, 5, E).astype(np.int32))
    stack_pushes = int(counts.sum())
    stk_out = torch.empty_like(learner.states[0])
    # A2: the stacking op on its own (mt_preprocess_resized: prev shifted by p channels + p frames)
    offs = torch.arange(0, 4 * E, 4, dtype=torch.int32, device='cuda')
    cnt_d = counts.to('cuda')
    from manette_amd import network as devnet_
    prof['stack'] = graph_time(lambda: devnet_.preprocess(pushes, offs, cnt_d, E, depth_, None, None, learner.states[0],
                                                          stk_out, resized=True), 40, label='stack')
    # A2 on the GPU in full (the north star's placement): each push's two raw screens -> frame-pool max
    # -> nearest 84x84 -> stack (mt_preprocess), reading (a) whole 210x160 screens in HBM, (b) the 84
    # screen rows the resize reads from pinned host memory over PCIe in place (the zero_copy staging)
    from manette_amd.environment import ROW_LUT as ROW_LUT_
    raw_hbm = torch.randint(0, 256, (4 * E, 2, 210, 160 * depth_), dtype=torch.uint8, device='cuda', generator=gen)
    rows_d = torch.from_numpy(ROW_LUT_.astype(np.int32)).cuda()
    ident_d = torch.arange(84, dtype=torch.int32, device='cuda')
    cols_d = learner.col_lut
    prof['preprocess_raw_hbm'] = graph_time(
        lambda: devnet_.preprocess(raw_hbm, offs, cnt_d, E, depth_, rows_d, cols_d, learner.states[0], stk_out,
                                   src_rows=210), 40, label='preprocess_raw_hbm')
    raw_pin = torch.empty((4 * E, 2, 84, 160 * depth_), dtype=torch.uint8, pin_memory=True)
    raw_pin.copy_(raw_hbm[:, :, :84].cpu())
    raw_pin_dev = devnet_.host_device_pointer(raw_pin)
    prof['preprocess_raw_pinned'] = graph_time(
        lambda: devnet_.preprocess(raw_pin_dev, offs, cnt_d, E, depth_, ident_d, cols_d, learner.states[0], stk_out,
                                   src_rows=84), 40, label='preprocess_raw_pinned')
    del raw_hbm
    if learner.lstm_bool:  # a step's new frames (trunk + cell x-product), + its E windows
        roll_fwd = lambda: learner._lstm_forward(1, learner.v_boot)
        roll_trunk = lambda: net.lstm_frames_forward(learner.fstore, 1 + 5 * E, E, E, T)
        plain_trunk = None
    else:
        roll_fwd = lambda: net.forward(learner.states[0], E, out=(learner.v_boot, learner.pi_roll, learner.rep_roll),
                                       ws_key='rollout', infer=True)
        plain_trunk = lambda: net.forward_trunk(learner.states[0], E, ws_key='rollout')
        if stacking or frame_stack:
            # the stacking rollout chain's kernels (the in-kernel-pull conv kernel + the dense
            # kernel) with every env's ready word already set and its pushes in HBM: nothing waits
            ready = torch.zeros(E, 32, dtype=torch.int32)  # MH_READY_STRIDE words per env
            ready[:, 0] = (7 << 3) | counts
            ready = ready.cuda()
            roll_trunk = lambda: net.forward_trunk_stacking(learner.states[0], pushes, ready, 7, stk_out, E,
                                                            ws_key='rollout')
        else:
            roll_trunk = plain_trunk
    prof['rollout_forward'] = graph_time(roll_fwd, 20, label='rollout_forward')
    prof['rollout_trunk'] = graph_time(roll_trunk, 40, label='roofline')
    if stacking or frame_stack:
        prof['plain_trunk'] = graph_time(plain_trunk, 40, label='plain_trunk')
    # the eager form (40 Python calls back to back between one event pair, BENCH_r02's method):
    # bounded by the host's launch rate when the box is loaded, kept to show the difference
    for _ in range(3):
        roll_trunk()
    s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_ev.record()
    for _ in range(40):
        roll_trunk()
    e_ev.record()
    torch.cuda.synchronize()
    prof['rollout_trunk_eager'] = s_ev.elapsed_time(e_ev) * 1e3 / 40.0
    # the same trunk launch at larger batches (supplementary: how far the kernel is from its
    # bounds once the grid fills the chip; the workload's own batch is E = ec above)
    sweep = []
    if not learner.lstm_bool and a.trunk_sweep:
        depth_ = 3 if cfg['rgb'] else 1
        g = torch.Generator(device='cuda').manual_seed(7)
        for Eb in [int(x) for x in a.trunk_sweep.split(',')]:
            obs_b = torch.randint(0, 256, (Eb, 84, 84, 4 * depth_), dtype=torch.uint8, device='cuda', generator=g)
            net.forward_trunk(obs_b, Eb, ws_key=('sweep', Eb))  # (workspace allocated outside the capture)
            sweep.append((Eb, float(np.median(graph_time(lambda: net.forward_trunk(obs_b, Eb, ws_key=('sweep', Eb)), 10,
                                                         3))) * 1e-3))
            del obs_b
            net._ws.pop(('sweep', Eb), None)
    ec = cfg['ec']
    value = world * ec * T * a.steps / elapsed

    if rank == 0:
        depth = 3 if cfg['rgb'] else 1
        A = args.num_actions
        layers = arch_flops(cfg['arch'], depth, A, cfg['nb_choices'])
        N = ec * T
        lstm = cfg['arch'] == 'LSTM'
        med = lambda xs: float(np.median(xs))
        tp_ms = med(prof['train_pass']) * 1e-3
        tp_flops = train_pass_flops(layers, N, 1 + (T + 4) * ec if lstm else None)
        rf_ms = med(prof['rollout_forward']) * 1e-3
        iso_ms = med(prof['rollout_trunk']) * 1e-3
        # one rollout step: E new frames (trunk) + E windows (LSTM) / E states
        fwd_flops = ec * sum(l[1] for l in layers)
        fwd_bytes = ec * 84 * 84 * 4 * depth + 4 * sum(l[2] for l in layers) + 4 * ec * sum(l[3] for l in layers)
        # trunk (roofline kernels): algorithmic bytes = the E states read once + the trunk weights
        # read once + the dense layer's pre-activation output written once; FLOP = E x (convs + dense)
        # 
        trunk = [l for l in layers if l[0] in ('conv', 'fc', 'lstm_x')]
        out_floats = trunk[-1][3]
        tk_bytes = ec * 84 * 84 * 4 * depth + 4 * sum(l[2] for l in trunk) + 4 * ec * out_floats
        tk_flops = ec * sum(l[1] for l in trunk)
        C_in = 4 * depth
        frame = 84 * 84 * depth
        # A2 stacking: the surviving channels of the previous state read, the p new frames read,
        # the new state written (mt_preprocess_resized, and the same work inside the conv kernel)
        stack_bytes = (4 * ec - stack_pushes) * frame + stack_pushes * frame + 4 * ec * frame
        graph_note = ('hipGraph of back-to-back calls replayed 5 times between HIP event pairs on its stream '
                      '(bench.graph_time); median per call, dispatch gaps included')
        if stacking or frame_stack:  # + the fused A2 stacking: the pushes read and the new state written
            tk_bytes += stack_pushes * frame + 4 * ec * frame
            # the rollout chain's own kernels; in the loop each conv block also waits for its env's
            # emulator (in-kernel pull), so the roofline times them with every env published
            tk_ms = iso_ms
            if cfg['arch'] == 'NIPS':
                kern = 'nips_conv_kernel<%d, true> (in-kernel pull) + nips_fc_kernel<%d>: the stacking rollout chain' % (
                    C_in, C_in)
                pmc_kernels = ['nips_conv_kernel<%d, true>' % C_in, 'nips_fc_kernel<%d>' % C_in]
            elif cfg['arch'] == 'NATURE':
                kern = ('nature_chain_kernel (stacking conv1 with in-kernel pull -> conv2 -> conv3, per-env hand-offs '
                        'in one launch) + row_fc_kernel (dense layer, one slab per conv row): the stacking rollout chain')
                pmc_kernels = ['nature_chain_kernel', 'row_fc_kernel']
            else:
                kern = ('stack_conv1_kernel (per-env pull + stack blocks, then conv1 tiles per env) + conv2 .. conv4 '
                        '(dconv_kernel, direct) + row_fc_kernel (dense): the stacking rollout chain')
                pmc_kernels = ['stack_conv1_kernel', 'dconv_kernel', 'row_fc_kernel']
            timing = ('mt_forward_trunk_stacking (every env published, its pushes in HBM: the kernels the timed loop '
                      'runs, with nothing to wait for), ' + graph_note)
        elif inloop_us is not None and not lstm:  # (LSTM: step 0's forward has 1 + 5E rows, the others E)
            tk_ms = inloop_us * 1e-3
            kern = 'trunk kernels of the rollout forward (implicit-GEMM convs + split-K dense)'
            timing = 'in the timed loop: HIP event pair around each macro-step forward\'s trunk launches ' \
                     '(mt_rollout_trunk_timing), %d updates after the timed region' % a.measure_updates
            pmc_kernels = None
        else:
            tk_ms = iso_ms
            kern = 'mt_forward_trunk (%s)' % ('LSTM frame trunk + cell x-product' if lstm else 'layered')
            timing = 'isolated mt_forward_trunk, ' + graph_note
            pmc_kernels = '*' if lstm else None  # (LSTM: tools/trunk_only.py runs exactly this launch)
        tk_gbs = tk_bytes / (tk_ms * 1e-3) / 1e9
        tk_tf = tk_flops / (tk_ms * 1e-3) / 1e12
        pmc = load_pmc(a.config, pmc_kernels)
        achieved = tp_flops / (tp_ms * 1e-3) / 1e12
        # per-kernel rows of SURVEY §8(d): A2, A9/A10 (the loss kernel with the fused n-step scan),
        # the backward's grouped launches, A11
        A_, R_ = A, cfg['nb_choices']
        O_ = 1 + A_ + R_
        F_ = layers[-2][3]
        P_ = net.nparams
        def row(name, ref, kernel, us, nbytes=None, flops=None, note=None):
            r = {'row': name, 'reference': ref, 'kernel': kernel, 'us': round(us, 2)}
            if nbytes is not None:
                gbs = nbytes / (us * 1e-6) / 1e9
                r.update(bound='hbm', algorithmic_bytes=int(nbytes), achieved_gbs=round(gbs, 1),
                         frac=round(gbs / MI355X_HBM_GBS, 4))
            if flops is not None:
                tf = flops / (us * 1e-6) / 1e12
                r.update(bound='mfma', algorithmic_flop=float(flops), achieved_tflops=round(tf, 3),
                         frac=round(tf / MI355X_FP32_TFLOPS, 4))
            if note:
                r['note'] = note
            return r
        kernels = [row('A2', 'atari_emulator.py:79-124, environment.py:58-80', 'preprocess_kernel (resized: stacking only)',
                       med(prof['stack']), stack_bytes,
                       note='standalone mt_preprocess_resized of the E envs (%d pushes); %s' % (stack_pushes, graph_note))]
        # the whole A2 on the GPU: per push the 84 screen rows the nearest resize reads, of both screens
        # (2 x 84 x 160 x depth B: whole lines, the kernel's 16-B loads), + the stack's bytes
        raw_bytes = stack_pushes * 2 * 84 * 160 * depth + stack_bytes - stack_pushes * frame
        kernels.append(row('A2 (GPU pool + resize + stack, HBM)', 'atari_emulator.py:79-124, environment.py:58-80',
                           'preprocess_kernel (mt_preprocess: 2 raw 210x160 screens per push -> max -> nearest '
                           '84x84 -> 4-frame stack)', med(prof['preprocess_raw_hbm']), raw_bytes,
                           note='raw screens resident in HBM; the same E envs and pushes as A2; ' + graph_note))
        pin_row = row('A2 (GPU pool + resize + stack, pinned host)', 'atari_emulator.py:79-124',
                      'preprocess_kernel (mt_preprocess on the zero_copy staging: the 84 resize rows of both screens '
                      'read over PCIe in place)', med(prof['preprocess_raw_pinned']), raw_bytes,
                      note='the bytes cross PCIe (achieved_gbs is the PCIe-inclusive rate; frac vs HBM is not its '
                           'bound); ' + graph_note)
        kernels.append(pin_row)
        if (stacking or frame_stack) and cfg['arch'] == 'NIPS':
            # (NIPS only: its plain trunk is the same kernel without the stack, nips_conv_kernel<C, false>;
            # NATURE's / PWYX's plain trunks are other kernels — the layered direct convs — so a difference
            # of the two would not be the stack's cost: round 5 printed -1.57 us for Seaquest)
            share = (med(prof['rollout_trunk']) - med(prof['plain_trunk']))
            kernels.append({'row': 'A2 (fused)', 'kernel': 'stacking share of nips_conv_kernel<%d, true>' % C_in,
                            'us': round(share, 2), 'note': 'stacking trunk minus the same kernel on a resident state '
                            '(nips_conv_kernel<%d, false> + the dense kernel): the cost of the in-kernel stack in '
                            'the benchmarked chain' % C_in})
        tl = prof['train_launches']
        if tl:
            boot = 4 * 9 * ec * F_ if stacking else 0
            loss_bytes = 4 * N * (2 * F_ + 2 * O_ + 4 + 6) + 4 * (F_ + 1) * O_ + boot
            loss_name = ('loss_bwd_kernel (loss + head dz / dH of the T*E windows; the LSTM update runs the n-step '
                         'scan in returns_kernel before its backward)' if lstm else
                         'loss_bwd_kernel (n-step scan' + (' + V(s_T) from the bootstrap slabs' if stacking else '')
                         + ' + loss + head dz / dH)')
            kernels.append(row('A10' if lstm else 'A9+A10', 'paac.py:219-231, policy_v_network.py:25-74', loss_name,
                               tl[0], loss_bytes, note='launch 1 of the update backward (bench.launch_breakdown)'))
            nconv = sum(1 for l in layers if l[0] == 'conv')
            if cfg['arch'] == 'NIPS' and not cfg['rgb']:  # the fused NIPS conv backward (nips_bwd.h)
                names = ['dense dX + head dW + dense dW',
                         'nips_conv_bwd_kernel (conv2 dX, conv1 dW + db per image; conv2 dW + db per image pair)',
                         'conv1 + conv2 slab sums + global-norm partials']
            else:
                if lstm:  # mt_lstm_frames_backward (lstm.h lstm_frames_bwd_impl), then the frame trunk's
                    names = ['lstm_bwd_kernel (BPTT of the T*E windows, dz of the gates)',
                             'lstm_zero_partials_kernel (the zero frame\'s gate-gradient partials)',
                             'lstm_gather_dxg_kernel (per-frame gate-gradient sums)',
                             'd flat = dxg K_x^T (conv4 act mask) + K_x dW']
                else:
                    names = ['dense dX + head dW + dense dW']
                for i in range(nconv - 1, -1, -1):
                    sfx = ' + conv%d slab sum' % (i + 2) if i < nconv - 1 else ''
                    if lstm and i == nconv - 1:
                        sfx += ' + K_h / fc6 / heads / projection dW (leading jobs)'
                    if i > 0 and cfg['arch'] in ('PWYX', 'LSTM') and i == 1:  # its own direct dX (dconv_bwd_solo)
                        names += ['conv2 dX (direct conv)', 'conv2 dW' + sfx]
                    else:
                        names.append(('conv%d dX + conv%d dW' % (i + 1, i + 1) if i > 0 else 'conv1 dW') + sfx)
                names.append('conv1 slab sum + global-norm partials')
            for k, us in enumerate(tl[1:]):
                nm = names[k] if k < len(names) else 'launch %d' % (k + 2)
                kernels.append(row('A10', 'actor_learner.py:49', nm if nm.startswith(('lstm_', 'nips_conv_bwd_kernel'))
                                   else 'group_kernel: ' + nm, us))
        kernels.append(row('A11', 'actor_learner.py:55-74', 'clip_rmsprop_kernel', med(prof['clip_rmsprop']),
                           28 * P_ + 4 * 512 + 4, note='%d params: w, ms, mom, g read (16 B) and w, ms, mom written '
                           '(12 B) per parameter; ' % P_ + graph_note))
        # the timed region in sub-windows (host clock after each update)
        edges = [t0] + marks
        wins = [world * ec * T * w / (edges[i + w] - edges[i]) for i in range(0, a.steps - w + 1, w)]
        line = {
            'metric': 'env-steps/sec (ec x t_max frames per update)',
            'value': round(value, 1),
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(elapsed / a.steps * 1e3, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'fp32',
            'data': 'synthetic emulators (seeded 210x160 screen rings, manette_amd/synthetic.py; no ALE): host '
                    'emulator threads pool + resize each push to 84x84, the GPU stacks the 4-frame states and runs '
                    'forward, sampling, returns, backward and RMSProp; random-init weights. The emulators are '
                    'near-free, so this is an upper bound for real ALE games (learner_only isolates the GPU side)',
            'config': {'workload': '%s ec=%d ew=%d t_max=%d per GPU, %s sampling, %s step, %s staging%s%s' % (
                a.config, ec, cfg['ew'], T, a.sampling, a.step_impl, a.staging, ', pipelined' if a.pipeline else '',
                ', data-parallel update forced at world 1 (RCCL)' if a.dp_force and world == 1 else ''),
                'arch': cfg['arch'], 'emulators_per_gpu': ec,
                'global_emulators': ec * world, 'parallelism': 'dp%d' % world,
                'dp_update': bool(learner_dp), 'settle_updates': settle},
            # bound = the resource the trunk's arithmetic intensity binds on the roofline (fp32 ridge
            # 157.3 TFLOP/s / 8 TB/s = 19.7 FLOP/B; NIPS E=32: 52 FLOP/B -> mfma); both fractions kept
            'roofline': dict(
                (('bound', 'mfma'), ('achieved', round(tk_tf, 3)), ('peak', MI355X_FP32_TFLOPS),
                 ('unit', 'TFLOP/s'), ('frac', round(tk_tf / MI355X_FP32_TFLOPS, 4)))
                if tk_flops / tk_bytes > MI355X_FP32_TFLOPS * 1e12 / (MI355X_HBM_GBS * 1e9) else
                (('bound', 'hbm'), ('achieved', round(tk_gbs, 1)), ('peak', MI355X_HBM_GBS), ('unit', 'GB/s'),
                 ('frac', round(tk_gbs / MI355X_HBM_GBS, 4))),
                kernel=kern, timing=timing,
                traffic=pmc['hbm_bytes'] if pmc else None,
                algorithmic_bytes_per_launch=tk_bytes, algorithmic_flop_per_launch=tk_flops,
                us_per_launch=round(tk_ms * 1e3, 2), hbm_gbs=round(tk_gbs, 1),
                hbm_frac=round(tk_gbs / MI355X_HBM_GBS, 4), flop_frac=round(tk_tf / MI355X_FP32_TFLOPS, 4),
                traffic_source=pmc['source'] if pmc else None),
            'trunk_in_loop': None if inloop_us is None else {
                'us_per_forward': round(inloop_us, 2),
                'note': 'event pair around each macro-step forward\'s trunk launches in the timed loop '
                        '(mt_rollout_trunk_timing, %d updates after the timed region)%s' % (
                            a.measure_updates, '; includes the conv blocks\' wait for their env\'s emulator '
                            '(in-kernel pull)' if stacking or frame_stack else
                            '; LSTM: frame trunk + cell x-product, averaged over step 0 (1 + 5E rows), steps '
                            '1..T-1 and the bootstrap (E rows each)' if lstm else '')},
            'train_pass': {'bound': 'mfma', 'kernels': ('backward of %d windows over %d distinct frames (forward reused from the rollout)' % (N, 1 + (T + 4) * ec)) if lstm else 'fused returns + loss + backward of %d rows (forward reused from the rollout)' % N,
                           'flop_count': 'executed backward: dW of every layer + dX of every layer but conv1',
                           'achieved': round(achieved, 3), 'peak': MI355X_FP32_TFLOPS, 'unit': 'TFLOP/s',
                           'frac': round(achieved / MI355X_FP32_TFLOPS, 4),
                           'ms_per_launch': round(tp_ms, 4), 'flop_per_launch': tp_flops,
                           'timing': graph_note, **stats_us(prof['train_pass'])},
            'kernels': kernels,
            'trunk_isolated': {'graph': stats_us(prof['rollout_trunk']),
                               'plain_trunk_graph': stats_us(prof['plain_trunk']) if 'plain_trunk' in prof else None,
                               'eager_us': round(prof['rollout_trunk_eager'], 2),
                               'note': 'graph = the roofline launch replayed as a hipGraph (5 replays of 40 calls); '
                                       'plain = mt_forward_trunk on a resident state (no stacking, no ready words); '
                                       'eager = 40 Python calls between one event pair (BENCH_r02\'s method: bounded '
                                       'by the host launch rate on a loaded box)'},
            'rollout_forward': {'ms': round(rf_ms, 4), 'tflops': round(fwd_flops / (rf_ms * 1e-3) / 1e12, 3),
                                'hbm_gbs': round(fwd_bytes / (rf_ms * 1e-3) / 1e9, 1),
                                'hbm_frac': round(fwd_bytes / (rf_ms * 1e-3) / 1e9 / MI355X_HBM_GBS, 4)},
            'value_windows': {'updates_per_window': w, 'values': [round(v, 1) for v in wins],
                              'spread': round((max(wins) - min(wins)) / float(np.median(wins)), 4),
                              'host_phases_us': window_phases,
                              'note': 'env-steps/s of consecutive sub-windows of the timed region (host clock after '
                                      'each update; the rollout waits on the device every macro-step), with each '
                                      'window\'s per-macro-step host phases (launch_and_wait = the GPU chain as the '
                                      'host sees it, emulators = the emulator threads)'},
        }
        line['host_threads'] = {'per_rank': every_threads,
                                'note': 'emulator worker threads + the host thread of each rank: its cpu slice '
                                        '(the allowed cpus on its GPU\'s NUMA node, split between the local ranks '
                                        'sharing it), the cores it may use (slice, container quota / local ranks), '
                                        'ew after the oversubscription cap, and whether they were pinned '
                                        '(--pin_threads auto: only with several ranks per node)'}
        if replicas is not None:
            line['replicas_identical'] = replicas
        if allreduce is not None:
            line['allreduce'] = allreduce
        if sweep:
            per_env_bytes = 84 * 84 * 4 * depth + 4 * out_floats
            w_bytes = 4 * sum(l[2] for l in trunk)
            per_env_flops = sum(l[1] for l in trunk)
            line['trunk_batch_sweep'] = [
                {'envs': Eb, 'us_per_launch': round(ms * 1e3, 2),
                 'hbm_gbs': round((Eb * per_env_bytes + w_bytes) / (ms * 1e-3) / 1e9, 1),
                 'hbm_frac': round((Eb * per_env_bytes + w_bytes) / (ms * 1e-3) / 1e9 / MI355X_HBM_GBS, 4),
                 'tflops': round(Eb * per_env_flops / (ms * 1e-3) / 1e12, 2),
                 'flop_frac': round(Eb * per_env_flops / (ms * 1e-3) / 1e12 / MI355X_FP32_TFLOPS, 4)}
                for Eb, ms in sweep]
        if step_phases:
            if emu_split:  # what the emulator threads spend per step (averaged over workers)
                step_phases['emulator_threads'] = {
                    'staging_us_per_worker': round(emu_split['stage_us'], 2),
                    'busy_us_per_worker': round(emu_split['busy_us'], 2),
                    'workers': learner.workers,
                    'note': 'per worker per macro-step: staging = %s; busy = the whole step phase (staging + '
                            'the synthetic emulation, FiGAR repeats and per-env publication); emulators_us = the '
                            'step\'s wall time to its last worker' % (
                                'frame pool + nearest resize + streaming copy of each push\'s 84x84 frame'
                                if a.staging == 'resized' else 'the copy of the staged screen rows')}
            line['macro_step_host_us'] = step_phases
        if world == 1 and not a.no_cpu_baseline:
            learner.cleanup()
            learner = None
            line['cpu_baseline'] = cpu_baseline(cfg, T, a.cpu_seconds, rank)
            # (vs_baseline stays null: BASELINE.md publishes no number for this metric; the ratio to
            # the CPU port timed here, on this box's host cores, is reported beside it)
            line['vs_cpu_baseline'] = round(value / line['cpu_baseline']['value'], 1)
            # BASELINE configs[0] (Pong NIPS ec=4 ew=2, the reference's CPU-only case), a shorter sample
            c0 = cpu_baseline(CPU_CONFIG0, T, a.cpu_seconds / 2, rank)
            c0.pop('_net_ms_per_update')
            c0['config'] = 'BASELINE.json configs[0]: pong NIPS ec=4 ew=2 t_max=%d' % T
            line['cpu_baseline_configs0'] = c0
            # learner-only: the network work of one update on each side (GPU: T + 1 rollout
            # forwards of E rows + the train pass; CPU port: its T + 1 forwards + train step)
            cpu_net = line['cpu_baseline'].pop('_net_ms_per_update')
            gpu_net = (T + 1) * rf_ms + tp_ms
            line['learner_only'] = {'gpu_ms_per_update': round(gpu_net, 4), 'cpu_ms_per_update': round(cpu_net, 3),
                                    'ratio': round(cpu_net / gpu_net, 1),
                                    'note': 'network work only (no emulators, no host loop): GPU = (T+1) isolated '
                                            'rollout forwards + the train pass; CPU = the port\'s torch-CPU forwards '
                                            '+ train step inside the cpu_baseline sample'}
        if PROFILE_WINDOWS:  # [boottime start ns, end ns, calls] of each labelled graph measurement
            line['profile_windows'] = dict(PROFILE_WINDOWS)
        print(json.dumps(line), flush=True)
    if learner is not None:
        learner.cleanup()
    shutil.rmtree(args.debugging_folder, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
