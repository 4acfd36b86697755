"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own host code.

Test infrastructure only; runs in the build container, where the reference is mounted at
/root/reference (it does not exist on the GPU box, and nothing but this script reads it).
TensorFlow 1.x, ALE, cv2 are absent, so:
  * `tensorflow` is a permissive stub module: the reference's host modules only use it for
    graph/summary objects, which the fake session below replaces — no TF math is emulated;
  * `ale_python_interface.ALEInterface` is tests/golden/golden_env.FakeALE (seeded screens);
  * `scipy.misc.imresize` (removed from scipy) is a shim with the semantics it had:
    PIL Image.fromarray(uint8).resize((w, h), NEAREST) (scipy<=1.2 toimage/bytescale pass
    uint8 through unchanged); `cv2` is an empty stub (only imported, never called).
Outputs (numpy .npz without pickles, and JSON):
  G1 host_loop_*.npz   paac.PAACLearner.train() feeds (paac.py:86-297) + episode summaries
  G2 runner.json       EmulatorRunner._run bookkeeping (emulator_runner.py:19-42)
  G3 tab_rep.json      ExplorationPolicy.get_tab_repetitions (exploration_policy.py:56-62)
  G4 preprocess.npz    AtariEmulator frame pool / resize / stack (atari_emulator.py:79-124)
  G5 meta_graph.json   constants + op structure decoded from pretrained/*/checkpoints/*.meta
Usage: python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import glob
import hashlib
import json
import os
import struct
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from golden_env import GoldenEnv, FakeALE  # noqa: E402


# ---------------------------------------------------------------------------------------------
# stubs
# ---------------------------------------------------------------------------------------------
class _Any(object):
    """Accepts any attribute access / call / context use; records summary values."""
    log = []

    def __init__(self, *a, **k):
        self._a = a
        self._k = k

    def __getattr__(self, name):
        if name.startswith('__'):
            raise AttributeError(name)
        return _Any()

    def __call__(self, *a, **k):
        return _Any(*a, **k)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __iter__(self):
        return iter(())


def _install_stubs():
    tf = types.ModuleType('tensorflow')

    def _summary_value(tag=None, simple_value=None, histo=None, **k):
        return ('value', tag, simple_value)

    class _Summary(object):
        Value = staticmethod(_summary_value)

        def __init__(self, value=()):
            self.value = list(value)

    tf.Summary = _Summary
    tf.HistogramProto = _Any
    tf.summary = _Any()
    tf.InteractiveSession = _Any
    tf.Session = _Any
    tf.convert_to_tensor = lambda *a, **k: None
    tf.name_scope = _Any
    tf.device = _Any
    tf.placeholder = _Any
    tf.float32 = 'float32'
    tf.uint8 = 'uint8'
    tf.train = _Any()
    tf.contrib = _Any()
    sys.modules['tensorflow'] = tf
    contrib = types.ModuleType('tensorflow.contrib')
    contrib.rnn = _Any()
    sys.modules['tensorflow.contrib'] = contrib

    ale = types.ModuleType('ale_python_interface')
    ale.ALEInterface = FakeALE
    sys.modules['ale_python_interface'] = ale
    sys.modules['cv2'] = types.ModuleType('cv2')

    import scipy.misc
    from PIL import Image

    def imresize(arr, size, interp='nearest'):
        assert interp == 'nearest' and arr.dtype == np.uint8
        im = Image.fromarray(arr)
        return np.asarray(im.resize((size[1], size[0]), resample=Image.NEAREST))

    scipy.misc.imresize = imresize
    if not hasattr(scipy.misc, 'imsave'):
        scipy.misc.imsave = lambda *a, **k: None


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(np.asarray(a, dtype=np.uint8)).tobytes()).hexdigest()


# ---------------------------------------------------------------------------------------------
# G1: host loop
# ---------------------------------------------------------------------------------------------
class _Sentinel(object):
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return '<%s>' % self.name


class FakeNet(object):
    def __init__(self):
        for n in ['output_layer_v', 'output_layer_pi', 'output_layer_rep', 'input_ph', 'memory_ph',
                  'critic_target_ph', 'selected_action_ph', 'selected_repetition_ph',
                  'adv_actor_ph']:
            setattr(self, n, _Sentinel(n))


def fake_outputs(rng, B, A, R):
    v = rng.randn(B).astype(np.float32)
    la = rng.randn(B, A)
    pa = np.exp(la) / np.exp(la).sum(1, keepdims=True)
    pa = (0.9 * pa + 0.1 / A).astype(np.float32)
    lr_ = rng.randn(B, R)
    pr = np.exp(lr_) / np.exp(lr_).sum(1, keepdims=True)
    pr = (0.9 * pr + 0.1 / R).astype(np.float32)
    return v, pa, pr


class FakeSession(object):
    def __init__(self, net, learner, A, R, lstm):
        self.net = net
        self.learner = learner
        self.A, self.R, self.lstm = A, R, lstm
        self.rng = np.random.RandomState(99)
        self.rollout = []    # per forward: dict(state_sha, v, pi, rep)
        self.boot = []       # per update: dict(state_sha, v)
        self.train = []      # per update: feeds

    def run(self, fetches, feed_dict=None):
        n = self.net
        inp = feed_dict.get(n.memory_ph if self.lstm else n.input_ph)
        if isinstance(fetches, list) and len(fetches) == 3 and fetches[0] is n.output_layer_v:
            B = len(inp)
            v, pi, rep = fake_outputs(self.rng, B, self.A, self.R)
            self.rollout.append(dict(state_sha=sha(inp), v=v, pi=pi, rep=rep))
            return v, pi, rep
        if fetches is n.output_layer_v:
            B = len(inp)
            v = self.rng.randn(B).astype(np.float32)
            self.boot.append(dict(state_sha=sha(inp), v=v))
            return v
        if isinstance(fetches, list) and fetches[0] is self.learner.train_step:
            fd = feed_dict
            self.train.append(dict(
                state_sha=sha(inp),
                state_shape=np.asarray(np.shape(inp), dtype=np.int64),
                y=np.array(fd[n.critic_target_ph], dtype=np.float64, copy=True),
                adv=np.array(fd[n.adv_actor_ph], dtype=np.float64, copy=True),
                a_onehot=np.array(fd[n.selected_action_ph], dtype=np.float64, copy=True),
                r_onehot=np.array(fd[n.selected_repetition_ph], dtype=np.float64, copy=True),
                lr=np.float64(fd[self.learner.learning_rate]),
                global_step=np.int64(self.learner.global_step)))
            return None, None
        raise RuntimeError('unexpected fetches %r' % (fetches,))

    def close(self):
        pass


class SummaryCapture(object):
    def __init__(self):
        self.values = []  # (step, tag, value)

    def add_summary(self, summary, step=None):
        for v in getattr(summary, 'value', []):
            if isinstance(v, tuple) and v[0] == 'value':
                self.values.append((int(step), v[1], float(v[2])))

    def flush(self):
        pass


def run_host_loop(ref, ec, ew, T, A, max_rep, nb_choices, n_updates, lstm):
    import paac
    from exploration_policy import ExplorationPolicy
    args = argparse.Namespace(egreedy=False, epsilon=0.05, softmax_temp=1.0, keep_percentage=0.9,
                              annealed=False, max_repetition=max_rep, nb_choices=nb_choices)
    np.random.seed(1234)
    explo = ExplorationPolicy(args)
    L = paac.PAACLearner.__new__(paac.PAACLearner)
    L.checkpoint_interval = 10 ** 15
    L.debugging_folder = '/tmp/golden/'
    L.network_checkpoint_folder = '/tmp/golden/checkpoints/'
    L.optimizer_checkpoint_folder = '/tmp/golden/optimizer_checkpoints/'
    L.last_saving_step = 0
    L.device = '/cpu:0'
    L.game = 'golden'
    L.global_step = 0
    L.max_global_steps = ec * T * n_updates
    L.max_local_steps = T
    L.num_actions = A
    L.explo_policy = explo
    L.gamma = 0.99
    L.initial_lr = 0.0224
    L.lr_annealing_steps = 1000
    L.emulator_counts = ec
    L.emulators = np.asarray([GoldenEnv(i) for i in range(ec)])
    L.network = FakeNet()
    L.learning_rate = _Sentinel('lr')
    L.train_step = _Sentinel('train_step')
    L.summary_writer = SummaryCapture()
    L.network_saver = _Any()
    L.optimizer_saver = _Any()
    L.workers = ew
    L.total_repetitions = nb_choices
    L.lstm_bool = lstm
    L.tab_rep = explo.tab_rep
    L.init_network = lambda: 0
    hist = []
    L.log_histogram = lambda tag, values, step, bins=1000: hist.append((tag, np.asarray(values)))
    sess = FakeSession(L.network, L, A, nb_choices, lstm)
    L.session = sess
    try:
        L.train()
    except BaseException:
        # the reference's EmulatorRunner processes are non-daemon: stop them or exit hangs
        if getattr(L, 'runners', None) is not None:
            L.runners.stop()
        raise
    out = {}
    out['tab_rep'] = np.asarray(explo.tab_rep, dtype=np.int64)
    out['config'] = np.asarray([ec, ew, T, A, max_rep, nb_choices, n_updates, int(lstm)], np.int64)
    for i, r in enumerate(sess.rollout):
        out['roll_v_%d' % i] = r['v']
        out['roll_pi_%d' % i] = r['pi']
        out['roll_rep_%d' % i] = r['rep']
    out['roll_sha'] = np.asarray([r['state_sha'] for r in sess.rollout])
    for i, b in enumerate(sess.boot):
        out['boot_v_%d' % i] = b['v']
    out['boot_sha'] = np.asarray([b['state_sha'] for b in sess.boot])
    for i, t in enumerate(sess.train):
        for k, v in t.items():
            if k != 'state_sha':
                out['train_%s_%d' % (k, i)] = v
    out['train_sha'] = np.asarray([t['state_sha'] for t in sess.train])
    sv = L.summary_writer.values
    out['episode_step'] = np.asarray([s for s, tag, v in sv if tag == 'rl/reward'], np.int64)
    out['episode_reward'] = np.asarray([v for s, tag, v in sv if tag == 'rl/reward'], np.float64)
    out['episode_length'] = np.asarray([v for s, tag, v in sv if tag == 'rl/episode_length'], np.float64)
    for i, (tag, vals) in enumerate(hist):
        out["hist_%s_%d" % (tag, i // 2)] = np.array(vals, dtype=np.int64)
    out['final_global_step'] = np.int64(L.global_step)
    return out


# ---------------------------------------------------------------------------------------------
# G2: EmulatorRunner bookkeeping (in process)
# ---------------------------------------------------------------------------------------------
def run_runner(ref):
    from emulator_runner import EmulatorRunner
    from exploration_policy import ExplorationPolicy
    cases = []
    for (max_rep, nb) in [(10, 11), (0, 1), (10, 6)]:
        args = argparse.Namespace(egreedy=False, epsilon=0.05, softmax_temp=1.0, keep_percentage=0.9,
                                  annealed=False, max_repetition=max_rep, nb_choices=nb)
        tab = ExplorationPolicy(args).tab_rep
        ec, A = 4, 6
        emus = [GoldenEnv(i) for i in range(ec)]
        states = np.asarray([e.get_initial_state() for e in emus], np.uint8)
        variables = [states, np.zeros(ec, np.float32), np.zeros(ec, np.float32),
                     np.zeros((ec, A), np.float32), np.zeros((ec, nb), np.float32)]
        rs = np.random.RandomState(5 + nb)
        steps = []
        for step in range(6):
            a = rs.randint(0, A, size=ec)
            r = rs.randint(0, nb, size=ec)
            variables[3][:] = np.eye(A)[a]
            variables[4][:] = np.eye(nb)[r]

            class Q(object):
                def __init__(self):
                    self.items = [True, None]

                def get(self):
                    return self.items.pop(0)

            class Bar(object):
                def put(self, x):
                    pass

            EmulatorRunner(tab, 0, emus, variables, Q(), Bar())._run()
            steps.append(dict(a=a.tolist(), r=r.tolist(), reward=variables[1].tolist(),
                              over=variables[2].tolist(),
                              state_sha=[sha(variables[0][i]) for i in range(ec)],
                              env_k=[e.k for e in emus], env_steps=[e.steps for e in emus]))
        cases.append(dict(max_rep=max_rep, nb_choices=nb, tab_rep=list(tab), steps=steps))
    return cases


# ---------------------------------------------------------------------------------------------
# G3: tab_rep
# ---------------------------------------------------------------------------------------------
def run_tab_rep():
    from exploration_policy import ExplorationPolicy
    out = []
    for max_rep, nb in [(10, 11), (10, 6), (11, 10), (0, 1), (4, 2), (5, 3), (20, 4), (3, 5)]:
        args = argparse.Namespace(egreedy=False, epsilon=0.05, softmax_temp=1.0, keep_percentage=0.9,
                                  annealed=False, max_repetition=max_rep, nb_choices=nb)
        out.append(dict(max_repetition=max_rep, nb_choices=nb,
                        tab_rep=[int(x) for x in ExplorationPolicy(args).tab_rep]))
    return out


# ---------------------------------------------------------------------------------------------
# G4: preprocess (atari_emulator.py with FakeALE)
# ---------------------------------------------------------------------------------------------
def run_preprocess():
    import atari_emulator
    from scipy.misc import imresize
    out = {}
    rows = np.repeat(np.arange(210, dtype=np.uint8)[:, None], 160, axis=1)
    cols = np.repeat(np.arange(160, dtype=np.uint8)[None, :], 210, axis=0)
    out['row_lut'] = imresize(rows, (84, 84), interp='nearest')[:, 0].astype(np.int64)
    out['col_lut'] = imresize(cols, (84, 84), interp='nearest')[0, :].astype(np.int64)
    for rgb in (False, True):
        tag = 'rgb' if rgb else 'gray'
        args = argparse.Namespace(random_seed=3, rom_path='.', game='pong', random_start=False,
                                  single_life_episodes=False, visualize=0, rgb=rgb)
        emu = atari_emulator.AtariEmulator(0, args)
        emu.ale.over_after = 4 * 4 + 4 * 6  # initial 4 steps + 6 next() then game over
        obs = [emu.get_initial_state()]
        frames = [emu.ale.frame]
        terms = []
        for i in range(8):
            o, r, t = emu.next(i % 6)
            obs.append(o)
            frames.append(emu.ale.frame)
            terms.append(t)
            if t:
                obs.append(emu.get_initial_state())
                frames.append(emu.ale.frame)
                terms.append(-1)
        out['%s_obs' % tag] = np.asarray(obs, np.uint8)
        out['%s_frame_after' % tag] = np.asarray(frames, np.int64)
        out['%s_terms' % tag] = np.asarray(terms, np.int64)
    return out


# ---------------------------------------------------------------------------------------------
# G5: .meta decode (minimal protobuf wire-format reader; no TF needed)
# ---------------------------------------------------------------------------------------------
def _varint(b, i):
    r = 0
    s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7f) << s
        s += 7
        if c < 0x80:
            return r, i


def pb_fields(b):
    i = 0
    out = []
    while i < len(b):
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError('wire type %d' % wt)
        out.append((f, wt, v))
    return out


def _tensor_value(tb):
    dtype, fl, content, shape = None, [], None, []
    for f, wt, v in pb_fields(tb):
        if f == 1:
            dtype = v
        elif f == 2:
            for f2, _, v2 in pb_fields(v):
                if f2 == 2:
                    for f3, _, v3 in pb_fields(v2):
                        if f3 == 1:
                            shape.append(v3)
        elif f == 4:
            content = v
        elif f == 5:
            if wt == 2:
                fl.extend(struct.unpack('<%df' % (len(v) // 4), v))
            else:
                fl.append(struct.unpack('<f', v)[0])
    if dtype == 1:  # DT_FLOAT
        if content is not None:
            vals = list(struct.unpack('<%df' % (len(content) // 4), content))
        else:
            vals = fl
        return dict(dtype='float32', shape=shape, values=vals[:16])
    return dict(dtype=dtype, shape=shape)


def decode_meta(path):
    data = open(path, 'rb').read()
    graph = None
    for f, wt, v in pb_fields(data):
        if f == 2:
            graph = v
    nodes = []
    for f, wt, v in pb_fields(graph):
        if f != 1:
            continue
        nd = dict(name='', op='', inputs=[], attr={})
        for f2, _, v2 in pb_fields(v):
            if f2 == 1:
                nd['name'] = v2.decode()
            elif f2 == 2:
                nd['op'] = v2.decode()
            elif f2 == 3:
                nd['inputs'].append(v2.decode())
            elif f2 == 5:
                key, val = None, None
                for f3, _, v3 in pb_fields(v2):
                    if f3 == 1:
                        key = v3.decode()
                    elif f3 == 2:
                        val = v3
                if key == 'value':
                    for f4, _, v4 in pb_fields(val):
                        if f4 == 8:
                            nd['attr']['value'] = _tensor_value(v4)
                elif key in ('padding', 'data_format'):
                    for f4, _, v4 in pb_fields(val):
                        if f4 == 2:
                            nd['attr'][key] = v4.decode()
                elif key == 'strides' or key == 'ksize':
                    for f4, _, v4 in pb_fields(val):
                        if f4 == 1:
                            ints = []
                            for f5, wt5, v5 in pb_fields(v4):
                                if f5 == 3:
                                    if wt5 == 2:
                                        j = 0
                                        while j < len(v5):
                                            x, j = _varint(v5, j)
                                            ints.append(x)
                                    else:
                                        ints.append(v5)
                            nd['attr'][key] = ints
        nodes.append(nd)
    return nodes


def run_meta(ref):
    out = {}
    for path in sorted(glob.glob(os.path.join(ref, 'pretrained', '*', 'checkpoints', '*.meta'))):
        game = path.split(os.sep)[-3]
        nodes = decode_meta(path)
        byname = {n['name']: n for n in nodes}

        def scalar(name):
            n = byname.get(name)
            if n is None or 'value' not in n['attr']:
                return None
            v = n['attr']['value']
            return v['values'][0] if v.get('values') else None

        consts = {}
        for n in nodes:
            if n['op'] == 'Const' and 'value' in n['attr']:
                v = n['attr']['value']
                if v.get('dtype') == 'float32' and v.get('values') and len(v['values']) == 1 \
                        and (n['name'].startswith('Training') or n['name'].startswith('Optimizer')
                             or n['name'].startswith('Input') or 'random_uniform' in n['name']
                             or n['name'].startswith('Network')):
                    consts[n['name']] = v['values'][0]
        convs = [dict(name=n['name'], padding=n['attr'].get('padding'), strides=n['attr'].get('strides'))
                 for n in nodes if n['op'] == 'Conv2D' and n['name'].startswith('Network')]
        pools = [dict(name=n['name'], padding=n['attr'].get('padding'), ksize=n['attr'].get('ksize'),
                      strides=n['attr'].get('strides'))
                 for n in nodes if n['op'] == 'MaxPool' and n['name'].startswith('Network')]
        ops = sorted(set(n['op'] for n in nodes))
        rms = [dict(name=n['name'], inputs=n['inputs']) for n in nodes if n['op'] == 'ApplyRMSProp']
        # inputs of the RMSProp slot initialisers (ones vs zeros)
        slot_init = sorted(set(n['op'] + ':' + n['name'].split('/')[-1] for n in nodes
                               if 'OptimizerVariables' in n['name'] and n['name'].endswith('Initializer/ones')
                               or n['name'].endswith('Initializer/zeros') and 'OptimizerVariables' in n['name']))
        loss_nodes = [dict(name=n['name'], op=n['op'], inputs=n['inputs']) for n in nodes
                      if n['name'].startswith('Training/ComputeLoss') or n['name'].startswith('Training/Actor')
                      or n['name'].startswith('Training/Critic') or n['name'].startswith('Training/Repetition')
                      if n['op'] not in ('Const', 'Identity', 'VariableV2', 'Assign', 'RandomUniform',
                                         'Shape', 'Reshape', 'Placeholder')]
        clip_nodes = [dict(name=n['name'], op=n['op'], inputs=n['inputs']) for n in nodes
                      if 'clip_by_global_norm' in n['name'] and n['op'] not in ('Identity',)]
        out[game] = dict(n_nodes=len(nodes), consts=consts, convs=convs, pools=pools, ops=ops,
                         apply_rmsprop=rms, slot_init=slot_init, loss_nodes=loss_nodes,
                         clip_nodes=clip_nodes[:80])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    ap.add_argument('--out', default=HERE)
    a = ap.parse_args()
    _install_stubs()
    sys.path.insert(0, a.ref)
    os.makedirs('/tmp/golden', exist_ok=True)
    with open('/tmp/golden/args.json', 'w') as f:
        f.write('{}')

    for name, kw in [
        ('host_loop_nips_r1', dict(ec=4, ew=2, T=5, A=6, max_rep=0, nb_choices=1, n_updates=4, lstm=False)),
        ('host_loop_figar_r11', dict(ec=4, ew=2, T=5, A=4, max_rep=10, nb_choices=11, n_updates=4, lstm=False)),
        ('host_loop_lstm_r11', dict(ec=4, ew=2, T=5, A=9, max_rep=10, nb_choices=11, n_updates=3, lstm=True)),
    ]:
        out = run_host_loop(a.ref, **kw)
        np.savez_compressed(os.path.join(a.out, name + '.npz'), **out)
        print('wrote', name, len(out), 'arrays')

    with open(os.path.join(a.out, 'runner.json'), 'w') as f:
        json.dump(run_runner(a.ref), f)
    with open(os.path.join(a.out, 'tab_rep.json'), 'w') as f:
        json.dump(run_tab_rep(), f, indent=1)
    np.savez_compressed(os.path.join(a.out, 'preprocess.npz'), **run_preprocess())
    with open(os.path.join(a.out, 'meta_graph.json'), 'w') as f:
        json.dump(run_meta(a.ref), f, indent=0, sort_keys=True)
    print('done')


if __name__ == '__main__':
    main()
