"""PAAC host loop restatement (oracle and "port" CPU baseline).

paac.py:86-297 (train loop: rollout step :140-205, bootstrap + scan :219-231, flatten + feed
:233-256), runners.py:7-50 + emulator_runner.py:19-42 (env stepping), actor_learner.py:108-136
(reward clip, LR). The network is pluggable: `net.forward(states_uint8) -> (v, pi, rep)` and
`net.train(flat_states, y, adv, a_onehot, r_onehot, lr)` — a replay double for golden tests,
or OracleNetwork (numpy, float32) for the CPU baseline.
"""
import multiprocessing as mp
from multiprocessing.sharedctypes import RawArray
from ctypes import c_float, c_uint8

import numpy as np

from . import nets, optim, policy, preprocess, returns


class SyntheticEmulator(object):
    """The synthetic ALE stand-in of SURVEY §8(d) restated on the oracle's preprocess (test data
    for replays): per global env id, np.random.RandomState(1000 + id) draws a ring of 64 uniform
    210x160 screens, then 4096 rewards in {-1, 0, +1} with p = (0.05, 0.90, 0.05). Push k pools
    screens 2k, 2k+1 (mod 64) and resizes them (atari_emulator.py:79-100); next() returns reward k
    (mod 4096) and pushes; an episode ends after episode_len next() calls; get_initial_state()
    makes 4 pushes (environment.py / atari_emulator.py:102-124 contract)."""
    RING, REWARD_LEN = 64, 4096

    def __init__(self, global_env_id, depth=1, episode_len=997):
        rs = np.random.RandomState(1000 + int(global_env_id))
        self.screens = rs.randint(0, 256, size=(self.RING, 210, 160, depth), dtype=np.uint8)
        self.rewards = rs.choice(np.array([-1.0, 0.0, 1.0]), p=[0.05, 0.90, 0.05],
                                 size=self.REWARD_LEN).astype(np.float32)
        self.depth = depth
        self.episode_len = episode_len
        self.stack = preprocess.ObservationStack(depth)
        self.k = 0
        self.steps = 0

    def _push(self):
        f0 = self.screens[(2 * self.k) % self.RING]
        f1 = self.screens[(2 * self.k + 1) % self.RING]
        self.stack.push(preprocess.pool_and_resize(f0, f1))
        self.k += 1

    def get_initial_state(self):
        for _ in range(4):
            self._push()
        self.steps = 0
        return self.stack.stacked()

    def next(self, action):
        reward = float(self.rewards[self.k % self.REWARD_LEN])
        self._push()
        self.steps += 1
        return self.stack.stacked(), reward, self.steps >= self.episode_len


def emulator_runner_step(tab_rep, emulators, states, rewards, over, a_idx, r_idx):
    """emulator_runner.py:24-41 for a block of emulators (indices instead of one-hots)."""
    for i, emu in enumerate(emulators):
        act = policy.Action(tab_rep, a_idx[i], r_idx[i])
        new_s, reward, episode_over = emu.next(act.current_action)
        states[i] = emu.get_initial_state() if episode_over else new_s
        rewards[i] = reward
        over[i] = episode_over
        while act.is_repeated() and not episode_over:
            new_s, reward, episode_over = emu.next(act.repeat())
            states[i] = emu.get_initial_state() if episode_over else new_s
            rewards[i] += reward
            over[i] = episode_over


class InProcessRunners(object):
    """Runners with the workers' loop run inline (same arithmetic, no processes)."""

    def __init__(self, tab_rep, emulators, states, rewards, over, a_idx, r_idx):
        self.tab_rep = tab_rep
        self.emulators = emulators
        self.v = (states, rewards, over, a_idx, r_idx)

    def update_environments(self):
        s, r, o, a, rr = self.v
        emulator_runner_step(self.tab_rep, self.emulators, s, r, o, a, rr)

    def wait_updated(self):
        pass

    def stop(self):
        pass


def _worker(tab_rep, emulators, shm, lo, hi, shape, q, barrier):
    states = np.frombuffer(shm[0], np.uint8).reshape(shape)[lo:hi]
    rewards = np.frombuffer(shm[1], np.float32)[lo:hi]
    over = np.frombuffer(shm[2], np.float32)[lo:hi]
    a_idx = np.frombuffer(shm[3], np.float32)[lo:hi]
    r_idx = np.frombuffer(shm[4], np.float32)[lo:hi]
    while True:
        if q.get() is None:
            break
        emulator_runner_step(tab_rep, emulators, states, rewards, over,
                             a_idx.astype(np.int64), r_idx.astype(np.int64))
        barrier.put(True)


class ProcessRunners(object):
    """runners.py:7-50: ew forked worker processes, RawArray shared state, one go-Queue per
    worker and a barrier Queue (the reference's IPC pattern, kept for the CPU baseline)."""

    def __init__(self, tab_rep, emulators, workers, state_shape):
        E = len(emulators)
        self.shape = (E,) + tuple(state_shape)
        self.shm = [RawArray(c_uint8, int(np.prod(self.shape))), RawArray(c_float, E),
                    RawArray(c_float, E), RawArray(c_float, E), RawArray(c_float, E)]
        self.states = np.frombuffer(self.shm[0], np.uint8).reshape(self.shape)
        self.rewards = np.frombuffer(self.shm[1], np.float32)
        self.over = np.frombuffer(self.shm[2], np.float32)
        self.a_idx = np.frombuffer(self.shm[3], np.float32)
        self.r_idx = np.frombuffer(self.shm[4], np.float32)
        for i, e in enumerate(emulators):
            self.states[i] = e.get_initial_state()
        bounds = np.linspace(0, E, workers + 1).astype(int)
        self.queues = [mp.Queue() for _ in range(workers)]
        self.barrier = mp.Queue()
        self.procs = []
        for w in range(workers):
            p = mp.Process(target=_worker, args=(tab_rep, emulators[bounds[w]:bounds[w + 1]], self.shm,
                                                  bounds[w], bounds[w + 1], self.shape, self.queues[w],
                                                  self.barrier), daemon=True)
            p.start()
            self.procs.append(p)

    def update_environments(self):
        for q in self.queues:
            q.put(True)

    def wait_updated(self):
        for _ in self.queues:
            self.barrier.get()

    def stop(self):
        for q in self.queues:
            q.put(None)
        for p in self.procs:
            p.join(timeout=5)


class HostLoop(object):
    """paac.py:86-297 restated; returns the list of train feeds (for golden comparisons)."""

    def __init__(self, emulators, net, tab_rep, num_actions, max_local_steps=5, gamma=0.99,
                 initial_lr=0.0224, lr_annealing_steps=80000000, lstm=False, workers=0,
                 record=True):
        self.emulators = list(emulators)
        self.E = len(self.emulators)
        self.net = net
        self.tab_rep = list(tab_rep)
        self.A = num_actions
        self.R = len(self.tab_rep)
        self.T = max_local_steps
        self.gamma = gamma
        self.initial_lr = initial_lr
        self.lra = lr_annealing_steps
        self.lstm = lstm
        self.workers = workers
        self.record = record
        self.global_step = 0
        self.total_rewards = []
        self.total_steps = []
        self.episodes = []
        self.feeds = []
        self.histograms = []

    def run(self, max_global_steps):
        E, T, A, R = self.E, self.T, self.A, self.R
        s0 = np.asarray([e.get_initial_state() for e in self.emulators], dtype=np.uint8) \
            if self.workers == 0 else None
        if self.workers == 0:
            shared_states = s0
            shared_rewards = np.zeros(E, np.float32)
            shared_over = np.zeros(E, np.float32)
            a_sh = np.zeros(E, np.int64)
            r_sh = np.zeros(E, np.int64)
            runners = InProcessRunners(self.tab_rep, self.emulators, shared_states, shared_rewards,
                                       shared_over, a_sh, r_sh)
        else:
            runners = ProcessRunners(self.tab_rep, self.emulators, self.workers, (84, 84, 4 * self.emulators[0].depth))
            shared_states, shared_rewards, shared_over = runners.states, runners.rewards, runners.over
            a_sh, r_sh = runners.a_idx, runners.r_idx
        try:
            self._loop(runners, shared_states, shared_rewards, shared_over, a_sh, r_sh, max_global_steps)
        finally:
            runners.stop()
        return self.feeds

    def _loop(self, runners, shared_states, shared_rewards, shared_over, a_sh, r_sh, max_global_steps):
        E, T, A, R = self.E, self.T, self.A, self.R
        if self.lstm:  # paac.py:107-112
            memory = np.zeros((E, 5) + shared_states.shape[1:], dtype=np.uint8)
            whole_memory = np.zeros((T, E, 5) + shared_states.shape[1:], dtype=np.uint8)
            for e in range(E):
                memory[e, -1] = shared_states[e]
        emulator_steps = [0] * E
        total_episode_rewards = E * [0]
        y_batch = np.zeros((T, E))
        adv_batch = np.zeros((T, E))
        rewards = np.zeros((T, E))
        states = np.zeros((T,) + shared_states.shape, dtype=np.uint8)
        actions = np.zeros((T, E, A))
        repetitions = np.zeros((T, E, R))
        values = np.zeros((T, E))
        masks = np.zeros((T, E))
        while self.global_step < max_global_steps:
            total_action_rep = np.zeros((A, R))
            for t in range(T):
                v_t, pi_t, rep_t = self.net.forward(memory if self.lstm else shared_states)
                a_idx = policy.multinomial_choose(pi_t)
                r_idx = policy.multinomial_choose(rep_t)
                new_actions = np.eye(A)[a_idx]
                new_reps = np.eye(R)[r_idx]
                a_sh[:] = a_idx
                r_sh[:] = r_idx
                actions[t] = new_actions
                values[t] = v_t
                states[t] = shared_states
                repetitions[t] = new_reps
                runners.update_environments()
                runners.wait_updated()
                if self.lstm:  # paac.py:79-83
                    whole_memory[t] = memory
                    memory[:, :-1] = memory[:, 1:]
                    memory[:, -1] = shared_states
                masks[t] = 1.0 - shared_over.astype(np.float32)
                for e, (actual_reward, episode_over) in enumerate(zip(shared_rewards, shared_over)):
                    total_episode_rewards[e] += actual_reward
                    rewards[t, e] = optim.rescale_reward(actual_reward)
                    emulator_steps[e] += self.tab_rep[int(np.argmax(new_reps[e]))] + 1
                    self.global_step += 1
                    total_action_rep[int(np.argmax(new_actions[e]))][int(np.argmax(new_reps[e]))] += 1
                    if episode_over:
                        self.total_rewards.append(total_episode_rewards[e])
                        self.total_steps.append(emulator_steps[e])
                        self.episodes.append((self.global_step, float(total_episode_rewards[e]),
                                              float(emulator_steps[e])))
                        total_episode_rewards[e] = 0
                        emulator_steps[e] = 0
                        if self.lstm:
                            memory[e] = 0
            v_boot = self.net.forward(memory if self.lstm else shared_states, bootstrap=True)
            y_batch, adv_batch = returns.nstep_returns(rewards, masks, values, v_boot, self.gamma)
            flat_states = (whole_memory.reshape((T * E, 5) + shared_states.shape[1:]) if self.lstm
                           else states.reshape((T * E,) + shared_states.shape[1:]))
            lr = optim.get_lr(self.global_step, self.initial_lr, self.lra)
            feed = dict(states=flat_states, y=y_batch.reshape(-1), adv=adv_batch.reshape(-1),
                        a_onehot=actions.reshape(T * E, A).copy(), r_onehot=repetitions.reshape(T * E, R).copy(),
                        lr=lr, global_step=self.global_step, rewards=rewards.copy(), masks=masks.copy(),
                        values=values.copy(), v_boot=np.copy(v_boot))
            self.net.train(flat_states, feed['y'], feed['adv'], feed['a_onehot'], feed['r_onehot'], lr)
            nb_a = [sum(a) for a in total_action_rep]
            nb_r = [sum(r) for r in np.transpose(total_action_rep)]
            histo_a, histo_r = [], []
            for i in range(A):
                histo_a += [i] * int(nb_a[i])
            for i in range(R):
                histo_r += [self.tab_rep[i] + 1] * int(nb_r[i])
            self.histograms.append((np.array(histo_a), np.array(histo_r)))
            if self.record:
                self.feeds.append(feed)


class OracleNetwork(object):
    """numpy float32 network + TF1 clip/RMSProp: the "port" CPU baseline's learner."""

    def __init__(self, arch, depth, num_actions, num_reps, seed=0, beta=0.02, clip=3.0,
                 decay=0.99, eps=0.1, dtype=np.float32):
        self.spec = nets.arch_spec(arch, depth, num_actions, num_reps)
        self.P = nets.init_params(self.spec, seed)
        self.ms = {k: np.ones_like(v) for k, v in self.P.items()}
        self.mom = {k: np.zeros_like(v) for k, v in self.P.items()}
        self.beta, self.clip, self.decay, self.eps = beta, clip, decay, eps
        self.dtype = dtype

    def forward(self, states, bootstrap=False):
        v, pi, rep, _ = nets.forward(self.spec, self.P, states, dtype=self.dtype)
        v = v.astype(np.float32)
        if bootstrap:
            return v
        return v, pi.astype(np.float32), rep.astype(np.float32)

    def train(self, flat_states, y, adv, a_onehot, r_onehot, lr):
        _, G, _ = nets.loss_and_grads(self.spec, self.P, flat_states, np.argmax(a_onehot, 1),
                                      np.argmax(r_onehot, 1), y.astype(np.float32),
                                      adv.astype(np.float32), self.beta, dtype=self.dtype)
        names = [n for (n, _, _) in self.spec['vars']]
        norm = optim.global_norm([G[n] for n in names])
        s = optim.clip_scale(norm, self.clip)
        for n in names:
            optim.rmsprop_apply(self.P[n], self.ms[n], self.mom[n], G[n].astype(np.float32) * s, lr,
                                self.decay, 0.0, self.eps)
