"""Host-side product components on CPU: native runner, bookkeeping, exploration policy and the
Python runner path, each against the oracle / the reference's golden vectors."""
import json
import os

import numpy as np
import pytest

from golden_env import GoldenEnv
from oracle import host_loop as ohl
from oracle import policy as opol
from oracle import preprocess as opre

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _args(max_rep, nb):
    import argparse
    return argparse.Namespace(egreedy=False, epsilon=0.05, softmax_temp=1.0, keep_percentage=0.9,
                              annealed=False, max_repetition=max_rep, nb_choices=nb)


def test_product_tab_rep_g3():
    from manette_amd.exploration_policy import ExplorationPolicy
    for case in json.load(open(os.path.join(GOLDEN, 'tab_rep.json'))):
        assert ExplorationPolicy(_args(case['max_repetition'], case['nb_choices'])).tab_rep == case['tab_rep']


def test_product_sampler_is_reference_stream():
    """Parity mode draws exactly the reference's numpy multinomial stream."""
    from manette_amd.exploration_policy import ExplorationPolicy
    g = dict(np.load(os.path.join(GOLDEN, 'host_loop_figar_r11.npz')))
    pol = ExplorationPolicy(_args(10, 11))
    np.random.seed(1234)
    ours = [pol.choose_indices(g['roll_pi_%d' % i], g['roll_rep_%d' % i]) for i in range(5)]
    np.random.seed(1234)
    ref = [(opol.multinomial_choose(g['roll_pi_%d' % i]), opol.multinomial_choose(g['roll_rep_%d' % i]))
           for i in range(5)]
    for (a, r), (a0, r0) in zip(ours, ref):
        assert a.tolist() == a0 and r.tolist() == r0
    # and they are the actions the reference fed to its first train_step
    a_first = np.argmax(g['train_a_onehot_0'], 1).reshape(5, 4)
    assert [a.tolist() for a, _ in ours] == a_first.tolist()


@pytest.mark.parametrize('name', ['host_loop_nips_r1', 'host_loop_figar_r11'])
def test_bookkeeper_and_python_runners_g1(name):
    """Product Runners(workers=0) + ExplorationPolicy + Bookkeeper reproduce the reference's
    episode summaries, histograms, global_step and train feeds' actions."""
    from manette_amd.bookkeeping import Bookkeeper
    from manette_amd.emulator_runner import EmulatorRunner
    from manette_amd.exploration_policy import ExplorationPolicy
    from manette_amd.runners import Runners
    g = dict(np.load(os.path.join(GOLDEN, name + '.npz')))
    ec, ew, T, A, max_rep, nb, n_updates, lstm = [int(x) for x in g['config']]
    pol = ExplorationPolicy(_args(max_rep, nb))
    emus = [GoldenEnv(i) for i in range(ec)]
    s0 = np.asarray([e.get_initial_state() for e in emus], np.uint8)
    variables = [s0, np.zeros(ec, np.float32), np.zeros(ec, np.float32), np.zeros(ec, np.int32),
                 np.zeros(ec, np.int32)]
    runners = Runners(pol.tab_rep, EmulatorRunner, emus, 0, variables)
    sh = runners.get_shared_variables()
    book = Bookkeeper(ec, A, pol.tab_rep)
    np.random.seed(1234)
    gs = 0
    i = 0
    rewards = np.zeros((T, ec), np.float32)
    masks = np.zeros((T, ec), np.float32)
    for u in range(n_updates):
        book.new_update()
        acts = []
        for t in range(T):
            a, r = pol.choose_indices(g['roll_pi_%d' % i], g['roll_rep_%d' % i])
            i += 1
            sh[3][...] = a
            sh[4][...] = r
            runners.update_environments()
            runners.wait_updated()
            gs = book.step(gs, a, r, sh[1], sh[2], rewards[t], masks[t])
            acts.append(a)
        assert gs == g['train_global_step_%d' % u]
        np.testing.assert_array_equal(np.concatenate(acts), np.argmax(g['train_a_onehot_%d' % u], 1))
        ha, hr = book.histograms()
        np.testing.assert_array_equal(ha, g['hist_actions_%d' % u])
        np.testing.assert_array_equal(hr, g['hist_repetitions_%d' % u])
    ep = np.asarray(book.episodes)
    np.testing.assert_array_equal(ep[:, 0], g['episode_step'])
    np.testing.assert_array_equal(ep[:, 1], g['episode_reward'])
    np.testing.assert_array_equal(ep[:, 2], g['episode_length'])


def test_python_runner_processes_g2():
    from manette_amd.emulator_runner import EmulatorRunner
    from manette_amd.runners import Runners
    case = json.load(open(os.path.join(GOLDEN, 'runner.json')))[0]
    ec = 4
    emus = [GoldenEnv(i) for i in range(ec)]
    s0 = np.asarray([e.get_initial_state() for e in emus], np.uint8)
    variables = [s0, np.zeros(ec, np.float32), np.zeros(ec, np.float32), np.zeros(ec, np.int32),
                 np.zeros(ec, np.int32)]
    runners = Runners(case['tab_rep'], EmulatorRunner, emus, 2, variables)
    runners.start()
    try:
        sh = runners.get_shared_variables()
        import hashlib
        for st in case['steps']:
            sh[3][...] = st['a']
            sh[4][...] = st['r']
            runners.update_environments()
            runners.wait_updated()
            assert sh[1].tolist() == st['reward']
            assert sh[2].tolist() == st['over']
            assert [hashlib.sha1(sh[0][e].tobytes()).hexdigest() for e in range(ec)] == st['state_sha']
    finally:
        runners.stop()


@pytest.mark.parametrize('max_rep,nb,workers', [(0, 1, 2), (10, 11, 3), (10, 6, 1)])
def test_native_runner_matches_python_emulator(max_rep, nb, workers):
    """libmanette_host's threads reproduce SyntheticEmulator (the reference contract) exactly:
    rewards, terminals, and the observation the device preprocess builds from the staged pushes."""
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank, SyntheticEmulator
    E, ep_len = 5, 7
    tab = opol.tab_repetitions(max_rep, nb)
    bank = SyntheticBank(0, E, episode_len=ep_len)
    nr = NativeRunners(bank, workers, tab)
    emus = [SyntheticEmulator(i, 6, episode_len=ep_len) for i in range(E)]
    try:
        tot = nr.reset()
        stacks = []
        for e in range(E):
            prev = np.zeros((84, 84, 4), np.uint8)
            st = _apply(nr, e, prev)
            np.testing.assert_array_equal(st, emus[e].get_initial_state())
            stacks.append(st)
        rs = np.random.RandomState(nb)
        states = np.asarray(stacks)
        rewards = np.zeros(E, np.float32)
        over = np.zeros(E, np.float32)
        for step in range(25):
            a = rs.randint(0, 6, E).astype(np.int32)
            r = rs.randint(0, nb, E).astype(np.int32)
            ohl.emulator_runner_step(tab, emus, states, rewards, over, a, r)
            nr.step(a, r)
            np.testing.assert_array_equal(nr.reward.numpy(), rewards)
            np.testing.assert_array_equal(nr.over.numpy(), over)
            for e in range(E):
                stacks[e] = _apply(nr, e, stacks[e])
                np.testing.assert_array_equal(stacks[e], states[e])
                assert nr.env_state(e) == (emus[e].k, emus[e].steps)
    finally:
        nr.stop()


def _apply(nr, e, prev):
    off = int(nr.push_offset[e])
    cnt = int(nr.push_count[e])
    assert 1 <= cnt <= 4
    fr = nr.staging.numpy()[off:off + cnt].reshape(cnt, 2, 210, 160, 1)
    pushes = [opre.pool_and_resize(fr[j, 0], fr[j, 1]) for j in range(cnt)]
    return opre.stack_update(prev, pushes)


def test_native_runner_rejects_bad_index():
    from manette_amd import _lib
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    nr = NativeRunners(SyntheticBank(0, 2), 1, [0, 3])
    try:
        with pytest.raises(_lib.MTError):
            nr.step(np.zeros(2, np.int32), np.array([0, 2], np.int32))
    finally:
        nr.stop()


def test_lut_product_matches_pil_fixture():
    from manette_amd.environment import COL_LUT, ROW_LUT
    p = np.load(os.path.join(GOLDEN, 'preprocess.npz'))
    np.testing.assert_array_equal(ROW_LUT, p['row_lut'])
    np.testing.assert_array_equal(COL_LUT, p['col_lut'])


def test_native_runner_row_selected_staging():
    """Staging only the resize's 84 rows carries exactly those rows of the whole screens."""
    from manette_amd.environment import ROW_LUT
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    tab = opol.tab_repetitions(10, 11)
    bank = SyntheticBank(3, 6, episode_len=9)
    full = NativeRunners(bank, 2, tab)
    rows = NativeRunners(bank, 3, tab, row_select=ROW_LUT)
    try:
        assert rows.src_rows == 84 and rows.frame_bytes == 84 * 160
        n1, n2 = full.reset(), rows.reset()
        rs = np.random.RandomState(0)
        for step in range(12):
            assert n1 == n2
            np.testing.assert_array_equal(full.push_meta.numpy(), rows.push_meta.numpy())
            a = full.staging.numpy()[:n1].reshape(n1, 2, 210, 160)[:, :, ROW_LUT]
            b = rows.staging.numpy()[:n2].reshape(n2, 2, 84, 160)
            np.testing.assert_array_equal(a, b)
            act = rs.randint(0, 6, 6).astype(np.int32)
            rep = rs.randint(0, 11, 6).astype(np.int32)
            n1, n2 = full.step(act, rep), rows.step(act, rep)
            np.testing.assert_array_equal(full.reward.numpy(), rows.reward.numpy())
    finally:
        full.stop()
        rows.stop()


def test_native_runner_fixed_slots_match_compact():
    """MH_RUNNER_FIXED_SLOTS stages env e's pushes at slots 4e.. with the same bytes, counts,
    rewards and terminals as the compact layout."""
    from manette_amd.environment import ROW_LUT
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    tab = opol.tab_repetitions(10, 11)
    bank = SyntheticBank(5, 7, episode_len=6)
    comp = NativeRunners(bank, 2, tab, row_select=ROW_LUT)
    fix = NativeRunners(bank, 3, tab, row_select=ROW_LUT, fixed_slots=True)
    try:
        n1, n2 = comp.reset(), fix.reset()
        rs = np.random.RandomState(1)
        for step in range(15):
            assert n2 == 4 * 7
            np.testing.assert_array_equal(fix.push_offset.numpy(), 4 * np.arange(7))
            np.testing.assert_array_equal(comp.push_count.numpy(), fix.push_count.numpy())
            for e in range(7):
                o1, o2, c = int(comp.push_offset[e]), 4 * e, int(comp.push_count[e])
                np.testing.assert_array_equal(comp.staging.numpy()[o1:o1 + c], fix.staging.numpy()[o2:o2 + c])
            act = rs.randint(0, 6, 7).astype(np.int32)
            rep = rs.randint(0, 11, 7).astype(np.int32)
            n1, n2 = comp.step(act, rep), fix.step(act, rep)
            np.testing.assert_array_equal(comp.reward.numpy(), fix.reward.numpy())
            np.testing.assert_array_equal(comp.over.numpy(), fix.over.numpy())
    finally:
        comp.stop()
        fix.stop()


def test_native_runner_in_place_frames_match_staging():
    """In-place frame mode (mh_runner_step_frames) names, per env and push, the bank screens whose
    bytes the staged mode copies: same counts, rewards and terminals, and bank[frame_idx] equals
    the staged screens byte for byte (oldest push first)."""
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    tab = opol.tab_repetitions(10, 11)
    E = 7
    bank = SyntheticBank(9, E, episode_len=5)
    comp = NativeRunners(bank, 2, tab)
    ip = NativeRunners(bank, 3, tab)
    flat = bank.screens.reshape(-1, 210 * 160)
    try:
        n1 = comp.reset()
        ip.reset_frames()
        rs = np.random.RandomState(2)
        for step in range(15):
            np.testing.assert_array_equal(comp.push_count.numpy(), ip.push_count.numpy())
            fr = ip.frames.numpy()
            for e in range(E):
                o, c = int(comp.push_offset[e]), int(comp.push_count[e])
                staged = comp.staging.numpy()[o:o + c].reshape(c, 2, 210 * 160)
                np.testing.assert_array_equal(flat[fr[e, :2 * c]].reshape(c, 2, -1), staged)
                assert (fr[e, :2 * c] // 64 == e).all()  # env e's own ring
            act = rs.randint(0, 6, E).astype(np.int32)
            rep = rs.randint(0, 11, E).astype(np.int32)
            n1 = comp.step(act, rep)
            ip.step_frames(act, rep)
            np.testing.assert_array_equal(comp.reward.numpy(), ip.reward.numpy())
            np.testing.assert_array_equal(comp.over.numpy(), ip.over.numpy())
    finally:
        comp.stop()
        ip.stop()


def test_native_runner_pooled_staging_is_frame_pool_max():
    """MH_RUNNER_POOLED stages one screen per push: the elementwise max of the two screens the
    unpooled layout stages (FramePool, atari_emulator.py:79-88), same slots, counts, rewards."""
    from manette_amd.environment import ROW_LUT
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    tab = opol.tab_repetitions(10, 11)
    E = 6
    bank = SyntheticBank(3, E, episode_len=7)
    two = NativeRunners(bank, 2, tab, row_select=ROW_LUT, fixed_slots=True)
    one = NativeRunners(bank, 3, tab, row_select=ROW_LUT, fixed_slots=True, pooled=True)
    assert one.staging.shape[1] == 1 and two.staging.shape[1] == 2
    try:
        two.reset(), one.reset()
        rs = np.random.RandomState(4)
        for step in range(12):
            np.testing.assert_array_equal(two.push_count.numpy(), one.push_count.numpy())
            for e in range(E):
                c = int(two.push_count[e])
                s2 = two.staging.numpy()[4 * e:4 * e + c]
                np.testing.assert_array_equal(one.staging.numpy()[4 * e:4 * e + c, 0], np.maximum(s2[:, 0], s2[:, 1]))
            act = rs.randint(0, 6, E).astype(np.int32)
            rep = rs.randint(0, 11, E).astype(np.int32)
            two.step(act, rep), one.step(act, rep)
            np.testing.assert_array_equal(two.reward.numpy(), one.reward.numpy())
            np.testing.assert_array_equal(two.over.numpy(), one.over.numpy())
    finally:
        two.stop()
        one.stop()


@pytest.mark.parametrize('rgb', [False, True])
def test_native_runner_resized_staging_is_pool_and_resize(rgb):
    """MH_RUNNER_RESIZED stages, per push, max(f0, f1) at the nearest-resize LUT rows and columns
    (atari_emulator.py:79-88, :113-124; SSE max + pshufb gather on the host) == the oracle's
    pool_and_resize of the two whole screens, byte for byte, with the same counts and rewards."""
    from manette_amd.environment import COL_LUT, ROW_LUT
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    tab = opol.tab_repetitions(10, 11)
    E = 5
    bank = SyntheticBank(11, E, rgb=rgb, episode_len=8)
    full = NativeRunners(bank, 2, tab, fixed_slots=True)
    rsz = NativeRunners(bank, 3, tab, row_select=ROW_LUT, fixed_slots=True, resized=True, col_lut=COL_LUT)
    depth = 3 if rgb else 1
    assert rsz.staging.shape == (4 * E, 1, 84 * 84 * depth)
    try:
        full.reset(), rsz.reset()
        rs = np.random.RandomState(7)
        for step in range(10):
            np.testing.assert_array_equal(full.push_count.numpy(), rsz.push_count.numpy())
            for e in range(E):
                for j in range(int(full.push_count[e])):
                    s = full.staging.numpy()[4 * e + j].reshape(2, 210, 160, depth)
                    want = opre.pool_and_resize(s[0], s[1])
                    np.testing.assert_array_equal(rsz.staging.numpy()[4 * e + j, 0].reshape(84, 84, depth), want)
            act = rs.randint(0, 6, E).astype(np.int32)
            rep = rs.randint(0, 11, E).astype(np.int32)
            full.step(act, rep), rsz.step(act, rep)
            np.testing.assert_array_equal(full.reward.numpy(), rsz.reward.numpy())
    finally:
        full.stop()
        rsz.stop()


def test_emulator_count_scope():
    """-ec per rank (the reference's per-agent count) or for the whole job (--ec_scope global):
    BASELINE's "ec=256 sharded 8x32" is -ec 256 --ec_scope global on 8 ranks."""
    import train
    assert train.shard_emulators(32, 'rank', 8, 3) == (32, 96)
    assert train.shard_emulators(256, 'global', 8, 3) == (32, 96)
    assert train.shard_emulators(256, 'global', 1, 0) == (256, 0)
    with pytest.raises(ValueError):
        train.shard_emulators(30, 'global', 8, 0)
    a = train.get_arg_parser().parse_args(['--ec_scope', 'global', '-ec', '256'])
    assert a.ec_scope == 'global' and a.emulator_counts == 256 and a.sampling == 'host'


@pytest.mark.parametrize('workers', [1, 3, 8])
def test_native_runner_per_env_publication_matches_blocks(workers):
    """With per-env ready words (the pipelined rollout's mode: each env staged and published as soon
    as it is stepped) every env's staging slots, push count, reward, episode flag and ready word
    equal the step without ready words (staging after the step), whatever the worker count."""
    import ctypes as C
    from manette_amd import _lib
    from manette_amd.environment import COL_LUT, ROW_LUT
    from manette_amd.runners import NativeRunners
    from manette_amd.synthetic import SyntheticBank
    E = 11
    tab = opol.tab_repetitions(10, 11)
    bank = SyntheticBank(4, E, episode_len=6)
    kw = dict(row_select=ROW_LUT, fixed_slots=True, resized=True, col_lut=COL_LUT)
    a, b = NativeRunners(bank, 2, tab, **kw), NativeRunners(bank, workers, tab, **kw)
    ready = np.zeros(E * 32, np.uint32)  # MH_READY_STRIDE words per env
    lib = _lib.host()
    try:
        na, nb = a.reset(), b.reset()
        rs = np.random.RandomState(workers)
        for step in range(12):
            act, rep = rs.randint(0, 6, E).astype(np.int32), rs.randint(0, 11, E).astype(np.int32)
            _lib.check_host(lib.mh_runner_set_ready(b._h, ready.ctypes.data_as(C.c_void_p), 100 + step),
                            'mh_runner_set_ready')
            na, nb = a.step(act, rep), b.step(act, rep)
            assert na == nb
            np.testing.assert_array_equal(a.push_meta.numpy(), b.push_meta.numpy())
            np.testing.assert_array_equal(a.staging.numpy(), b.staging.numpy())
            np.testing.assert_array_equal(a.reward.numpy(), b.reward.numpy())
            np.testing.assert_array_equal(a.over.numpy(), b.over.numpy())
            words = ready.reshape(E, 32)[:, 0]
            np.testing.assert_array_equal(words, ((100 + step) << 3) | a.push_count.numpy().astype(np.uint32))
        _lib.check_host(lib.mh_runner_set_ready(b._h, None, 0), 'mh_runner_set_ready')
    finally:
        a.stop()
        b.stop()
