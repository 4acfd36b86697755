"""Pin the oracle (CPU restatement) against vectors produced by the reference's own code
(tests/golden/make_golden.py). CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

from golden_env import GoldenEnv, fake_screen
from oracle import host_loop, nets, policy, preprocess, returns

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(np.asarray(a, dtype=np.uint8)).tobytes()).hexdigest()


def test_tab_rep_g3():
    for case in json.load(open(os.path.join(GOLDEN, 'tab_rep.json'))):
        assert policy.tab_repetitions(case['max_repetition'], case['nb_choices']) == case['tab_rep']


def test_runner_g2():
    for case in json.load(open(os.path.join(GOLDEN, 'runner.json'))):
        tab = case['tab_rep']
        assert tab == policy.tab_repetitions(case['max_rep'], case['nb_choices'])
        ec = 4
        emus = [GoldenEnv(i) for i in range(ec)]
        states = np.asarray([e.get_initial_state() for e in emus], np.uint8)
        rewards = np.zeros(ec, np.float32)
        over = np.zeros(ec, np.float32)
        for st in case['steps']:
            host_loop.emulator_runner_step(tab, emus, states, rewards, over, st['a'], st['r'])
            assert rewards.tolist() == st['reward']
            assert over.tolist() == st['over']
            assert [sha(states[i]) for i in range(ec)] == st['state_sha']
            assert [e.k for e in emus] == st['env_k']
            assert [e.steps for e in emus] == st['env_steps']


class ReplayNet(object):
    """Network double replaying the outputs the reference's fake session produced."""

    def __init__(self, g):
        self.g = g
        self.i = 0
        self.b = 0
        self.trains = []

    def forward(self, states, bootstrap=False):
        if bootstrap:
            assert sha(states) == self.g['boot_sha'][self.b]
            v = self.g['boot_v_%d' % self.b]
            self.b += 1
            return v
        assert sha(states) == self.g['roll_sha'][self.i], 'rollout forward %d sees other states' % self.i
        out = (self.g['roll_v_%d' % self.i], self.g['roll_pi_%d' % self.i], self.g['roll_rep_%d' % self.i])
        self.i += 1
        return out

    def train(self, flat_states, y, adv, a1, r1, lr):
        self.trains.append(sha(flat_states))


@pytest.mark.parametrize('name', ['host_loop_nips_r1', 'host_loop_figar_r11', 'host_loop_lstm_r11'])
def test_host_loop_g1(name):
    g = dict(np.load(os.path.join(GOLDEN, name + '.npz')))
    ec, ew, T, A, max_rep, nb, n_updates, lstm = [int(x) for x in g['config']]
    tab = policy.tab_repetitions(max_rep, nb)
    assert tab == g['tab_rep'].tolist()
    np.random.seed(1234)
    net = ReplayNet(g)
    loop = host_loop.HostLoop([GoldenEnv(i) for i in range(ec)], net, tab, A, max_local_steps=T,
                              gamma=0.99, initial_lr=0.0224, lr_annealing_steps=1000, lstm=bool(lstm))
    feeds = loop.run(ec * T * n_updates)
    assert len(feeds) == n_updates
    for u, f in enumerate(feeds):
        assert net.trains[u] == g['train_sha'][u]
        np.testing.assert_array_equal(f['y'], g['train_y_%d' % u])
        np.testing.assert_array_equal(f['adv'], g['train_adv_%d' % u])
        np.testing.assert_array_equal(f['a_onehot'], g['train_a_onehot_%d' % u])
        np.testing.assert_array_equal(f['r_onehot'], g['train_r_onehot_%d' % u])
        assert f['lr'] == g['train_lr_%d' % u]
        assert f['global_step'] == g['train_global_step_%d' % u]
        np.testing.assert_array_equal(loop.histograms[u][0], g['hist_actions_%d' % u])
        np.testing.assert_array_equal(loop.histograms[u][1], g['hist_repetitions_%d' % u])
    assert loop.global_step == int(g['final_global_step'])
    ep = np.asarray(loop.episodes)
    np.testing.assert_array_equal(ep[:, 0], g['episode_step'])
    np.testing.assert_array_equal(ep[:, 1], g['episode_reward'])
    np.testing.assert_array_equal(ep[:, 2], g['episode_length'])


def test_returns_matches_reference_dtypes():
    # y/adv of G1 recomputed from the replayed rewards/masks/values (bit-exact float64).
    g = dict(np.load(os.path.join(GOLDEN, 'host_loop_figar_r11.npz')))
    ec, ew, T, A, max_rep, nb, n_updates, lstm = [int(x) for x in g['config']]
    np.random.seed(1234)
    loop = host_loop.HostLoop([GoldenEnv(i) for i in range(ec)], ReplayNet(g),
                              policy.tab_repetitions(max_rep, nb), A, max_local_steps=T,
                              lr_annealing_steps=1000)
    for u, f in enumerate(loop.run(ec * T * n_updates)):
        y, adv = returns.nstep_returns(f['rewards'], f['masks'], f['values'], f['v_boot'], 0.99)
        np.testing.assert_array_equal(y.reshape(-1), g['train_y_%d' % u])
        np.testing.assert_array_equal(adv.reshape(-1), g['train_adv_%d' % u])


def test_preprocess_lut_g4():
    p = np.load(os.path.join(GOLDEN, 'preprocess.npz'))
    np.testing.assert_array_equal(preprocess.ROW_LUT, p['row_lut'])
    np.testing.assert_array_equal(preprocess.COL_LUT, p['col_lut'])


@pytest.mark.parametrize('rgb', [False, True])
def test_preprocess_stack_g4(rgb):
    p = np.load(os.path.join(GOLDEN, 'preprocess.npz'))
    tag = 'rgb' if rgb else 'gray'
    obs, frames, terms = p['%s_obs' % tag], p['%s_frame_after' % tag], p['%s_terms' % tag]
    depth = 3 if rgb else 1
    stack = preprocess.ObservationStack(depth)

    def push(f_before):
        # __action_repeat: 4 ALE acts, screens read after acts 3 and 4 (atari_emulator.py:90-100)
        stack.push(preprocess.pool_and_resize(fake_screen(f_before + 3, rgb), fake_screen(f_before + 4, rgb)))

    f = 0
    for _ in range(4):          # get_initial_state
        push(f)
        f += 4
    assert f == frames[0]
    np.testing.assert_array_equal(stack.stacked(), obs[0])
    i = 1
    for t in terms:
        if t == -1:             # reset after a terminal next()
            for _ in range(4):
                push(f)
                f += 4
        else:
            push(f)
            f += 4
        assert f == frames[i]
        np.testing.assert_array_equal(stack.stacked(), obs[i])
        i += 1


def test_stack_update_contract():
    # mt_preprocess contract == ObservationPool semantics for p = 1..4 pushes.
    rs = np.random.RandomState(0)
    st = preprocess.ObservationStack(1)
    for _ in range(4):
        st.push(rs.randint(0, 256, (84, 84, 1)).astype(np.uint8))
    for p in (1, 2, 3, 4):
        prev = st.stacked()
        pushes = [rs.randint(0, 256, (84, 84, 1)).astype(np.uint8) for _ in range(p)]
        for q in pushes:
            st.push(q)
        np.testing.assert_array_equal(preprocess.stack_update(prev, pushes), st.stacked())


def test_meta_graph_constants_g5():
    m = json.load(open(os.path.join(GOLDEN, 'meta_graph.json')))
    c = m['catcher']['consts']   # NIPS graph
    assert c['Training/ComputeLoss/scalar'] == 5.0             # loss_scaling
    assert c['Training/Critic/scalar'] == 0.25                 # critic factor
    assert np.float32(c['Training/Actor/Const']) == np.float32(1e-30)
    assert np.float32(c['Training/Repetition/Const']) == np.float32(1e-30)
    assert np.float32(c['Optimizer/OptimizerVariables/decay']) == np.float32(0.99)
    assert np.float32(c['Optimizer/OptimizerVariables/epsilon']) == np.float32(0.1)
    assert c['Optimizer/OptimizerVariables/momentum'] == 0.0
    assert c['Optimizer/clip_by_global_norm/mul/x'] == 3.0
    assert c['Optimizer/global_norm/Const_1'] == 2.0           # sqrt(sum 2*L2Loss)
    assert set(m['catcher']['slot_init']) == {'Const:ones', 'Const:zeros'}
    for n, v in c.items():  # rms slot = ones, momentum slot = zeros
        if n.endswith('OptimizerVariables/Initializer/ones'):
            assert v == 1.0
        if n.endswith('OptimizerVariables_1/Initializer/zeros'):
            assert v == 0.0
    # init bounds (weights use OUTPUT channels, biases input channels)
    spec = nets.arch_spec('NIPS', 1, 3, 1)
    bounds = {n: d for (n, _, d) in spec['vars']}
    for layer in ('conv1', 'conv2', 'fc3'):
        assert np.float32(c['Network/%s/random_uniform/max' % layer]) == \
            np.float32(bounds['Network/%s/%s_weights' % (layer, layer)])
        assert np.float32(c['Network/%s/random_uniform_1/max' % layer]) == \
            np.float32(bounds['Network/%s/%s_biases' % (layer, layer)])
    for scope, nm in (('Training/Critic', 'critic_output'), ('Training/Actor', 'actor_output'),
                      ('Training/Repetition', 'repetition_output')):
        assert np.float32(c['%s/%s/random_uniform/max' % (scope, nm)]) == \
            np.float32(bounds['%s/%s/%s_weights' % (scope, nm, nm)])
    # layer structure
    convs = m['catcher']['convs']
    assert [(x['padding'], x['strides']) for x in convs] == [('VALID', [1, 4, 4, 1]), ('VALID', [1, 2, 2, 1])]
    pw = m['seaquest']
    assert [x['padding'] for x in pw['convs']] == ['SAME'] * 4
    assert all(p['padding'] == 'VALID' and p['ksize'] == [1, 2, 2, 1] for p in pw['pools'])
    assert len(m['catcher']['apply_rmsprop']) == 12


def test_oracle_synthetic_emulator_equals_product_stream():
    """oracle/host_loop.SyntheticEmulator (the replay emulator of tests/test_e2e_gpu.py) restates
    the bench's synthetic stream (manette_amd/synthetic.py) on the oracle's preprocess:
    identical observations, rewards and terminals over resets, gray and RGB."""
    from oracle import host_loop
    from manette_amd.synthetic import SyntheticEmulator
    for gid, rgb in ((3, False), (17, True)):
        a = host_loop.SyntheticEmulator(gid, 3 if rgb else 1, episode_len=5)
        b = SyntheticEmulator(gid, 6, rgb=rgb, episode_len=5)
        np.testing.assert_array_equal(a.get_initial_state(), b.get_initial_state())
        for i in range(40):
            sa, ra, ta = a.next(0)
            sb, rb, tb = b.next(0)
            np.testing.assert_array_equal(sa, sb)
            assert ra == rb and ta == tb
            if ta:
                np.testing.assert_array_equal(a.get_initial_state(), b.get_initial_state())
