"""End-to-end oracle parity of the BENCHMARKED path at every 1-GPU config size, the
PWYX + RGB + FiGAR10 config included.

The learner is bench.make_learner(config) — the exact object bench.py times: native emulator
threads, device sampling fused into the heads kernel, resized staging, the pipelined native
macro-step (NIPS: pull kernel + stacking conv kernel), the update replayed as a hipGraph from the
second update on; LSTM: the native frame-store macro-step. U updates run; the last one (a graph replay) is
checked against the oracle on everything it consumed and produced:

  trajectory  every state slot 0..T and the clipped rewards / masks == a replay of the oracle's
              synthetic emulators (oracle/host_loop.py: emulator_runner.py:24-41 + the
              atari_emulator.py preprocess) under the recorded action / repetition indices of
              every rollout so far (A1, A2, A4, A8)                              bit-exact
  forward     v / pi / rep of every rollout row and V(s_T) == oracle forward      2e-5 relative
  returns     y / adv == oracle.returns.nstep_returns (paac.py:219-231)          bit-exact
  gradient    every variable == oracle.nets.loss_and_grads of the T*E rows        2e-4 rel. L2
              (LSTM: of the T*E windows over the distinct frames), per variable and per
              output channel; max-pool windows and ReLU branches taken where the device
              took them, each decision equal to the oracle's away from fp64 near-ties  bit-exact
  loss terms  per row == oracle                                                   1e-4 relative
  optimizer   lr == get_lr(global_step); norm == ||grad|| (1e-5); params / ms / mom after the
              update == oracle.optim clip + TF1 RMSProp on the device gradient    bit-exact
Reference: paac.py:140-256, actor_learner.py:43-74, policy_v_network.py:25-74.
Synthetic episodes are shortened (episode_len) so episode ends and resets happen inside the run.
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import host_loop, nets, optim, policy, returns

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

UPDATES = 4
EPISODE_LEN = 13


def _replay(cfg, E, A, idx_all, T):
    """Oracle emulators stepped with the recorded indices: states [U][T+1][E], rewards / masks [U][T][E]."""
    depth = 3 if cfg['rgb'] else 1
    tab = policy.tab_repetitions(cfg['max_repetition'], cfg['nb_choices'])
    emus = [host_loop.SyntheticEmulator(e, depth, EPISODE_LEN) for e in range(E)]
    s = np.stack([em.get_initial_state() for em in emus])
    rew = np.zeros(E, np.float32)
    over = np.zeros(E, np.float32)
    out = []
    for idx in idx_all:
        states, rr, mm = [s.copy()], [], []
        for t in range(T):
            host_loop.emulator_runner_step(tab, emus, s, rew, over, idx[0, t], idx[1, t])
            states.append(s.copy())
            rr.append(np.clip(rew, -1.0, 1.0).astype(np.float32))
            mm.append((1.0 - over).astype(np.float32))
        out.append((np.stack(states), np.stack(rr), np.stack(mm)))
    return out


def _run(config, tmp_path, dp_force=False):
    import bench
    L, args = bench.make_learner(config, debugging_folder=str(tmp_path) + '/', episode_len=EPISODE_LEN,
                                 dp_force=dp_force)
    L.start()
    return L, args, bench.CONFIGS[config]


def _window_rows(nz, t, E):
    """Frame-store rows of the windows of step t: position k < nz reads the zero frame (row 0),
    else slot t + k (row 1 + (t + k) * E + e) — the reference's memory window (paac.py:79-83)."""
    w = np.zeros((E, 5), np.int64)
    for e in range(E):
        for k in range(5):
            w[e, k] = 0 if k < nz[e] else 1 + (t + k) * E + e
    return w


def _chunked_feats(spec, P, frames, chunk=32):
    """Trunk features of frames [F,84,84,C] in chunks (the fp64 im2col of 192 RGB PWYX frames at
    once would be 3 GB)."""
    return np.concatenate([nets.trunk_forward(spec, P, frames[c0:c0 + chunk])[0] for c0 in range(0, len(frames), chunk)])


CASES = [('pong-nips', False), ('breakout-nature-figar', False), ('seaquest-nature', False),
         ('mspacman-lstm-figar', False), ('breakout-pwyx-figar-rgb', False),
         # the data-parallel update at world 1: RCCL communicator, the backward captured
         # with both gradient buckets all-reduced by RCCL on their own stream beside the conv backward,
         # forked and joined inside ONE captured graph (paac._dp_sequence), norm partials after the
         # all-reduce, launched by the rollout's last step — everything the N-GPU run executes but the
         # cross-rank sum, which at world 1 is the identity
         ('pong-nips', True), ('seaquest-nature', True),
         # configs[4]'s data-parallel leg: the LSTM update as two graphs — backward |
         # eager RCCL all-reduce of the whole gradient | apply, whose second step also moves the frame
         # store's slots and nz behind the all-reduce (paac.py:79-83, :202-203)
         ('mspacman-lstm-figar', True)]


@pytest.mark.parametrize('config,dp', CASES, ids=['%s%s' % (c, '-dp-rccl' if d else '') for c, d in CASES])
def test_benchmarked_path_matches_oracle(config, dp, tmp_path):
    import parity_util
    L, args, cfg = _run(config, tmp_path, dp_force=dp)
    try:
        lstm = L.lstm_bool
        assert L.native_step is not None and L.boot_in_rollout and L._graph_ok()
        assert L.dp == dp
        if dp:
            assert L.comm is not None and L.comm.kind == 'rccl' and L.world == 1
        E, T, A, R = L.emulator_counts, L.max_local_steps, L.num_actions, L.total_repetitions
        N = E * T
        idx_all = []
        for u in range(UPDATES - 1):
            L.book.new_update()
            L.rollout()
            idx_all.append(L.idx_h.numpy().copy())
            L.update()
        assert L._graphs is not None  # the checked update is a graph replay
        if dp and not lstm:  # one graph: the backward, the two buckets' all-reduces forked onto their stream and
            # joined before the apply (paac._dp_sequence), launched by the rollout's last step
            assert L._buckets is not None and len(L._graphs) == 1 and L._update_in_rollout
            assert L._rollout_update == 'all' 
        elif dp:  # LSTM: backward | all-reduce of the whole gradient | apply (+ the slot / nz carry), one graph
            assert L._buckets is None and len(L._graphs) == 1 and not L._update_in_rollout
        # the parameters / slots the checked rollout runs with, read before it: from the third update
        # on, the rollout's last step launches the update itself (mt_rollout_set_update)
        torch.cuda.synchronize()
        c = lambda t: t.detach().cpu().numpy().copy()
        P = L.network.get_variables()
        flat_p, ms0, mom0 = c(L.network.params), c(L.network.ms), c(L.network.mom)
        slot0 = c(L.states[0])  # (copied from slot T by the previous update unless slot0_in_rollout)
        L.book.new_update()
        L.rollout()
        torch.cuda.synchronize()
        idx_all.append(L.idx_h.numpy().copy())
        states = c(L.states)
        # the rollout's last step launched this update (data parallel too: the one-graph form), so its
        # apply — and, without slot0_in_rollout, the slot T -> 0 copy — already ran: restore slot 0
        if L._update_in_rollout and not L.slot0_in_rollout:
            states[0] = slot0
        rm = L.rm_h.numpy().copy()
        values = c(L.values)
        gs = L.global_step
        if lstm:  # (the update's apply moves slots T.. to 0.. and nz[T] to nz[0])
            fstore, nz = c(L.fstore), c(L.nz_d)  # (nz derived on the device by the native step)
        L.update()
        torch.cuda.synchronize()
        # the forward values the rollout left that the backward branches on (ReLU outputs, max-pool
        # argmax, the dense output)
        dev = L.network.forward_branches(L.network.lstm_workspace(E, T), 1, E, T) if lstm else \
            L.network.forward_branches(L.train_ws, 0, N)
        # the benchmarked path: the rollout launched this update — the whole update, data parallel
        # included (one graph: backward, both buckets' all-reduces forked and joined, apply; 'all')
        assert L._update_in_rollout == (not lstm)
        # V(s_T): the rollout's last chain (pipelined native step) or the update's first forward (LSTM)
        v_boot, pi_all, rep_all = c(L.v_boot), c(L.pi_all), c(L.rep_all)
        grad, y, adv = L.network.get_variables('grad'), c(L.y), c(L.adv)
        grad_flat = c(L.network.grad)
        w1, ms1, mom1 = c(L.network.params), c(L.network.ms), c(L.network.mom)
        norm_dev = float(L.network.norm_dev.item())
        lr_dev = float(L.network._lr_host[0])
        terms = c(L.loss_terms)
    finally:
        L.cleanup()

    # ---- trajectory: states, rewards, masks (bit-exact) --------------------------------------
    rep_states, rep_r, rep_m = _replay(cfg, E, A, idx_all, T)[-1]
    for t in range(T + 1):
        np.testing.assert_array_equal(states[t], rep_states[t], err_msg='state slot %d' % t)
    np.testing.assert_array_equal(rm[0], rep_r)
    np.testing.assert_array_equal(rm[1], rep_m)
    assert gs == UPDATES * T * E
    assert (idx_all[-1][0] < A).all() and (idx_all[-1][1] < R).all() and (idx_all[-1] >= 0).all()

    # ---- forward of every rollout row + V(s_T) ----------------------------------------------
    spec = nets.arch_spec(cfg['arch'], 3 if cfg['rgb'] else 1, A, R)
    if lstm:
        feats = _chunked_feats(spec, P, fstore[:1 + (T + 5) * E])
        for t in range(T + 1):
            rows = _window_rows(nz[t], t, E)
            v0, pi0, rep0, _ = nets.heads_forward(spec, P, feats[rows.reshape(-1)])
            v_t = values[t] if t < T else v_boot
            np.testing.assert_allclose(v_t, v0, rtol=2e-5, atol=2e-5, err_msg='v step %d' % t)
            np.testing.assert_allclose(pi_all[t], pi0, rtol=2e-5, atol=1e-6, err_msg='pi step %d' % t)
            np.testing.assert_allclose(rep_all[t], rep0, rtol=2e-5, atol=1e-6, err_msg='rep step %d' % t)
    else:
        obs = states[:T + 1].reshape((T + 1) * E, 84, 84, -1)
        v0, pi0, rep0, _ = nets.heads_forward(spec, P, _chunked_feats(spec, P, obs))
        np.testing.assert_allclose(values.reshape(-1), v0[:N], rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(v_boot, v0[N:], rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(pi_all[:T].reshape(N, A), pi0[:N], rtol=2e-5, atol=1e-6)
        np.testing.assert_allclose(rep_all[:T].reshape(N, R), rep0[:N], rtol=2e-5, atol=1e-6)

    # ---- n-step returns (bit-exact with the reference's dtype trail) --------------------------
    y0, adv0 = returns.nstep_returns(rm[0].astype(np.float64), rm[1].astype(np.float64), values.astype(np.float64),
                                     v_boot, L.gamma)
    np.testing.assert_array_equal(y, y0.astype(np.float32))
    np.testing.assert_array_equal(adv, adv0.astype(np.float32))

    # ---- gradient of the T*E rows / windows ----------------------------------------------------
    a_idx, r_idx = idx_all[-1][0].reshape(N), idx_all[-1][1].reshape(N)
    beta = L.network.beta
    if lstm:
        win = np.concatenate([_window_rows(nz[t], t, E) for t in range(T)])
        Fb = 1 + (T + 4) * E
        br = parity_util.device_branches(spec, P, fstore[:Fb], dev, win=win, rows=slice(0, Fb))
        _, G, aux = nets.window_frames_loss_and_grads(spec, P, fstore[:Fb], win, a_idx, r_idx, y.reshape(N),
                                                      adv.reshape(N), beta, routes=br['routes'],
                                                      branches=br['branches'], hbranch=br['hbranch'])
    else:  # (row n = frame n: the chunked form of nets.loss_and_grads, pinned to it by a CPU test)
        obs_n = states[:T].reshape(N, 84, 84, -1)
        br = parity_util.device_branches(spec, P, obs_n, dev)
        _, G, aux = nets.window_frames_loss_and_grads(spec, P, obs_n, np.arange(N)[:, None], a_idx, r_idx,
                                                      y.reshape(N), adv.reshape(N), beta, routes=br['routes'],
                                                      branches=br['branches'], hbranch=br['hbranch'])
    # every max-pool window and ReLU branch as the device took it (each decision bit-exact vs the
    # oracle away from fp64 near-ties): every gradient at the tight bound (round 2 allowed 5e-3 for
    # the pooled convs of a batch with a max-pool near-tie)
    parity_util.check_grads(spec, grad, G, set())
    np.testing.assert_allclose(terms, aux['terms'], rtol=1e-4, atol=1e-5)

    # ---- global-norm clip + TF1 RMSProp (bit-exact given the device gradient and norm) --------
    assert np.float32(lr_dev) == np.float32(optim.get_lr(gs, L.initial_lr, L.lr_annealing_steps))
    ref_norm = optim.global_norm([grad_flat])
    assert abs(norm_dev - ref_norm) <= 1e-5 * ref_norm, (norm_dev, ref_norm)
    s = optim.clip_scale(norm_dev, L.network.clip_norm)
    w, ms, mom = flat_p.copy(), ms0.copy(), mom0.copy()
    optim.rmsprop_apply(w, ms, mom, grad_flat * s, np.float32(lr_dev), L.network.decay, 0.0, L.network.eps)
    np.testing.assert_array_equal(ms1, ms)
    np.testing.assert_array_equal(mom1, mom)
    np.testing.assert_array_equal(w1, w)
