"""End-to-end learner parity on the GPU box: every path through PAACLearner that should produce
identical trajectories does, bit for bit, and the CLI trains / checkpoints / resumes."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _learner(tmp, runner, sampling, arch='NIPS', ec=8, game='pong', max_rep=0, nb=1, workers=2, seed=0,
             staging='in_place', pipeline=False):
    sys.path.insert(0, ROOT)
    import train as cli
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.paac import PAACLearner
    a = cli.get_arg_parser().parse_args([])
    a.game, a.arch, a.emulator_counts, a.emulator_workers = game, arch, ec, workers
    a.max_repetition, a.nb_choices = max_rep, nb
    a.runner, a.sampling, a.seed, a.staging, a.pipeline = runner, sampling, seed, staging, pipeline
    a.debugging_folder = str(tmp) + '/'
    a.max_global_steps = 1 << 40
    a.checkpoint_interval = 1 << 40
    a.lr_annealing_steps = 100000
    np.random.seed(1234)
    explo = ExplorationPolicy(a)
    nc, ec_ = cli.get_network_and_environment_creator(a, explo)
    L = PAACLearner(nc, ec_, explo, a)
    L.start()
    return L


def _run(L, updates):
    for _ in range(updates):
        L.book.new_update()
        for t in range(L.max_local_steps):
            L.step(t)
        L.update()
    torch.cuda.synchronize()


def _state(L):
    # slot 0 is excluded: the native stacking step carries slot T over into slot 0 inside the next
    # step 0's forward (mt_rollout_step), the Python path copies it at the end of update()
    return dict(params=L.network.params.cpu().numpy().copy(), ms=L.network.ms.cpu().numpy().copy(),
                states=L.states[1:].cpu().numpy().copy(), gs=L.global_step, episodes=list(L.book.episodes))


@pytest.mark.parametrize('max_rep,nb,staging,pipeline', [(0, 1, 'in_place', False), (10, 11, 'in_place', False),
                                                         (10, 11, 'zero_copy', False), (10, 11, 'copy', False),
                                                         (10, 11, 'pooled', False), (0, 1, 'in_place', True),
                                                         (10, 11, 'in_place', True), (10, 11, 'pooled', True),
                                                         (10, 11, 'resized', False), (0, 1, 'resized', True),
                                                         (10, 11, 'resized', True)])
def test_native_step_equals_python_step(tmp_path, max_rep, nb, staging, pipeline):
    """mt_rollout_step (C++ orchestration, sampling fused in the heads kernel; in-place, zero-copy,
    pooled or copied staging; optionally pipelined one step ahead behind a device wait) == the
    Python step() on the standalone kernels (mt_forward, mt_sample, hipMemcpy + mt_preprocess)."""
    A = _learner(tmp_path / 'a', 'native', 'device', max_rep=max_rep, nb=nb, staging=staging, pipeline=pipeline)
    assert A.native_step is not None
    _run(A, 6)
    sa = _state(A)
    A.cleanup()
    B = _learner(tmp_path / 'b', 'native', 'device', max_rep=max_rep, nb=nb, staging='copy')
    from manette_amd import _lib
    _lib.hip().mt_rollout_destroy(B.native_step)
    B.native_step = None
    _run(B, 6)
    sb = _state(B)
    B.cleanup()
    bad = {k: int(np.sum(sa[k] != sb[k])) for k in ('states', 'params', 'ms')}
    assert not any(bad.values()), bad
    assert sa['gs'] == sb['gs'] == 6 * 5 * 8


def test_native_runner_equals_reference_contract_runner(tmp_path):
    """Native emulator threads + GPU preprocess == reference-contract Python emulators with CPU
    preprocess (same seeds, host numpy sampling): identical trajectories and updates."""
    A = _learner(tmp_path / 'a', 'native', 'host', max_rep=10, nb=11)
    _run(A, 5)
    sa = _state(A)
    A.cleanup()
    B = _learner(tmp_path / 'b', 'python', 'host', max_rep=10, nb=11, workers=0)
    _run(B, 5)
    sb = _state(B)
    B.cleanup()
    for k in ('params', 'ms', 'states'):
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    assert sa['gs'] == sb['gs']


def test_python_runner_processes(tmp_path):
    A = _learner(tmp_path / 'a', 'python', 'host', workers=0)
    _run(A, 3)
    sa = _state(A)
    A.cleanup()
    B = _learner(tmp_path / 'b', 'python', 'host', workers=2)
    _run(B, 3)
    sb = _state(B)
    B.cleanup()
    np.testing.assert_array_equal(sa['params'], sb['params'])


def test_train_cli_checkpoint_resume(tmp_path):
    df = str(tmp_path / 'run') + '/'
    cmd = [sys.executable, os.path.join(ROOT, 'train.py'), '-g', 'breakout', '--arch', 'NATURE', '-ec', '8',
           '-ew', '2', '--max_repetition', '10', '--nb_choices', '11', '--max_global_steps', '200',
           '--checkpoint_interval', '80', '-df', df]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    args = json.load(open(df + 'args.json'))
    assert args['arch'] == 'NATURE' and args['nb_choices'] == 11
    from manette_amd import tf_bundle
    ck = sorted(os.listdir(df + 'checkpoints'))
    # TF tensor bundles + TF's `checkpoint` file, as tf.train.Saver writes them (max_to_keep 5)
    assert 'checkpoint' in ck and '-200.index' in ck and '-200.data-00000-of-00001' in ck
    assert sorted(os.listdir(df + 'optimizer_checkpoints')) == ['-200.data-00000-of-00001', '-200.index',
                                                                 'checkpoint']
    lines = open(df + 'checkpoints/checkpoint').read().splitlines()
    assert lines[0] == 'model_checkpoint_path: "-200"' and lines[-1] == 'all_model_checkpoint_paths: "-200"'
    z = tf_bundle.read_bundle(df + 'checkpoints/-200')
    assert z['Network/conv3/conv3_weights'].shape == (3, 3, 64, 64)
    assert z['Training/Repetition/repetition_output/repetition_output_weights'].shape == (512, 11)
    assert 'Network/fc4/fc4_weights/OptimizerVariables_1' in z
    o = tf_bundle.read_bundle(df + 'optimizer_checkpoints/-200')
    assert 'Network/fc4/fc4_weights/OptimizerVariables' in o and 'Network/fc4/fc4_weights' not in o
    np.testing.assert_array_equal(o['Network/fc4/fc4_weights/OptimizerVariables'],
                                  z['Network/fc4/fc4_weights/OptimizerVariables'])
    # TensorBoard event file of the run (actor_learner.py:82, paac.py:23-31): args text at step 0
    from manette_amd import summary
    evf = [f for f in os.listdir(df + 'tf') if f.startswith('events.out.tfevents.')]
    assert evf
    ev = summary.read_events(df + 'tf/' + evf[0])
    assert ev[0][2] == {'file_version': 'brain.Event:2'} and '"arch": "NATURE"' in ev[1][2]['text']
    # resume: starts from step 200 and continues to 280
    cmd[cmd.index('--max_global_steps') + 1] = '280'
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert 'Restoring network variables' in out.stdout + out.stderr
    assert '-280.index' in os.listdir(df + 'checkpoints')


@pytest.mark.parametrize('arch,extra', [('NATURE', ['--max_repetition', '10', '--nb_choices', '11']),
                                        ('LSTM', ['--max_repetition', '10', '--nb_choices', '11'])])
def test_eval_cli_restores_training_checkpoint(tmp_path, arch, extra):
    """train.py writes a TF-bundle checkpoint; test.py (test.py:29-116 flags) restores it and
    plays its episodes to the end, printing the reference's summary lines."""
    df = str(tmp_path / 'run') + '/'
    cmd = [sys.executable, os.path.join(ROOT, 'train.py'), '-g', 'ms_pacman', '--arch', arch, '-ec', '4',
           '-ew', '2', '--max_global_steps', '40', '--checkpoint_interval', '20', '-df', df] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    ev = subprocess.run([sys.executable, os.path.join(ROOT, 'test.py'), '-f', df, '-tc', '2', '-np', '3'],
                        capture_output=True, text=True, timeout=300)
    assert ev.returncode == 0, ev.stdout[-2000:] + ev.stderr[-2000:]
    assert 'Restoring network variables' in ev.stdout + ev.stderr
    lines = ev.stdout.splitlines()
    assert 'Performed 2 tests for ms_pacman.' in lines
    assert any(l.startswith('Mean: ') for l in lines) and any(l.startswith('Std: ') for l in lines)


def _dp_run(tmp_path, world, port, mode='gpu', arch='NIPS'):
    script = os.path.join(ROOT, 'tests', 'dp_worker.py')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK='0')
        procs.append(subprocess.Popen([sys.executable, script, str(tmp_path), mode, arch], env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, o[-2000:] + e[-3000:]
    if mode != 'gpu':
        return None
    return [np.load(os.path.join(str(tmp_path), '%s_w%d_r%d.npz' % (arch, world, r))) for r in range(world)]


@pytest.mark.parametrize('arch,envs,port', [('NIPS', 16, 29531), ('LSTM', 8, 29535)])
def test_dp_two_ranks_equal_single_process_union(tmp_path, arch, envs, port):
    """W=2 ranks (envs/2 each, gradient summed once per update, 1/W folded into the
    clip) == ONE process owning all the envs, through the product's update (graph-replayed from the
    second update on): the device draw hashes global env ids, so both runs take the same
    trajectory (states bit-identical per env), global_step advances by every env per macro-step
    on every rank (mh_book_set_shard), episodes carry the same global steps, and the parameters
    after every update agree within the fp32 reduction-order budget (the W=2 gradient is two
    half-batch sums added by the all-reduce instead of one sum). LSTM (configs[4]'s data-parallel
    leg): its update is backward | all-reduce of the whole gradient | apply, the
    apply also carrying the frame store's slots and windows; the device-derived windows (nz) are
    identical per env too (paac.py:79-83, :202-203)."""
    one = _dp_run(tmp_path, 1, port, arch=arch)[0]
    two = _dp_run(tmp_path, 2, port + 2, arch=arch)
    ec = envs // 2
    for r in range(2):
        np.testing.assert_array_equal(two[r]['gs'], one['gs'])
        np.testing.assert_array_equal(two[r]['states'], one['states'][:, :, r * ec:(r + 1) * ec],
                                      err_msg='rank %d trajectory' % r)
        if arch == 'LSTM':
            np.testing.assert_array_equal(two[r]['nz'], one['nz'][:, :, r * ec:(r + 1) * ec],
                                          err_msg='rank %d windows' % r)
    np.testing.assert_array_equal(two[0]['params'], two[1]['params'])  # replicas identical
    assert one['gs'][-1] == 4 * 5 * envs
    ep1 = sorted(map(tuple, one['episodes']))
    ep2 = sorted(map(tuple, np.concatenate([two[0]['episodes'], two[1]['episodes']])))
    assert len(ep1) > 0 and ep1 == ep2
    np.testing.assert_array_equal(two[0]['params0'], one['params0'])
    # parameter updates: relative L2 of (W2 - W1) against the update itself, per update
    prev = one['params0'].astype(np.float64)
    for u in range(one['params'].shape[0]):
        a, b = one['params'][u].astype(np.float64), two[0]['params'][u].astype(np.float64)
        step = np.linalg.norm(a - prev)
        assert step > 0 and np.linalg.norm(a - b) <= 1e-4 * step, (u, np.linalg.norm(a - b), step)
        prev = a


def test_dp_resume_from_rank0_checkpoint(tmp_path):
    """resuming a 2-rank run — rank 0 restores its checkpoint, rank 1's folder has
    none — continues from rank 0's global_step on both ranks with rank 0's parameters (broadcast at
    start), so both ranks follow one LR schedule and the replicas stay bit-identical."""
    _dp_run(tmp_path, 2, 29541, mode='resume')
    r0, r1 = [np.load(os.path.join(str(tmp_path), 'resume_r%d.npz' % r)) for r in range(2)]
    assert int(r0['saved']) == int(r1['saved']) == 2 * 5 * 16
    assert int(r0['start']) == int(r1['start']) == int(r0['saved'])
    assert int(r0['end']) == int(r1['end']) == int(r0['saved']) + 2 * 5 * 16
    np.testing.assert_array_equal(r0['p_start'], r1['p_start'])
    np.testing.assert_array_equal(r0['params'], r1['params'])


def test_rollout_refuses_a_second_stream(tmp_path):
    """The native rollout's chains spin in-kernel on host words; they must all run on one stream (two
    streams of waiting kernels sharing one of the GPU_MAX_HW_QUEUES hardware queues serialised into a
    timeout in round 2's env-group experiment), so a rollout handle refuses any stream but its first —
    before it launches anything — and then carries on on its own stream."""
    from manette_amd import _lib
    L = _learner(tmp_path, 'native', 'device', staging='resized', pipeline=True)
    try:
        L.book.new_update()
        L.rollout()
        L.update()
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            with pytest.raises(_lib.MTError, match='one stream'):
                L.rollout()
        L.book.new_update()
        L.rollout()  # the handle is still usable on its own stream
        L.update()
        torch.cuda.synchronize()
        assert np.isfinite(L.network.params.cpu().numpy()).all()
    finally:
        L.cleanup()
