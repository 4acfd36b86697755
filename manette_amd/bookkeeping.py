"""Per-step rollout bookkeeping (A8), vectorised over the env axis: paac.py:154-205.

Exact integer semantics of the reference loop:
  rewards[t] = clip(summed reward, +-1)                      (:180, actor_learner.py:108-114)
  masks[t] = 1 - over                                        (:176)
  emulator_steps[e] += tab_rep[r_e] + 1 (planned repeats)   (:183)
  global_step += 1 per env, in env order                    (:184)
  total_action_rep[a_e][r_e] += 1; nb_actions += r_e + 1     (:157, :187-189)
  on over: log (global_step at env e, total reward, emulator_steps), reset both   (:191-201)
Total episode rewards accumulate in float32 (the shared reward array is float32).
Data parallel (set_shard): a rank's envs are global envs [env_offset, env_offset + E) of a learner
stepping envs_total envs per macro-step; global_step then advances by envs_total (the same on
every rank) and episode records carry the global env's position, as one process would log them.
"""
import numpy as np


class Bookkeeper(object):
    def __init__(self, n_envs, num_actions, tab_rep):
        self.E = n_envs
        self.tab = np.asarray(tab_rep, dtype=np.int64)
        self.R = len(tab_rep)
        self.A = num_actions
        self.emulator_steps = np.zeros(n_envs, dtype=np.int64)
        self.total_episode_rewards = np.zeros(n_envs, dtype=np.float32)
        self.total_rewards = []
        self.total_steps = []
        self.episodes = []   # (global_step, reward, length)
        self.env_offset, self.envs_total = 0, n_envs
        self.new_update()

    def set_shard(self, env_offset, envs_total):
        assert 0 <= env_offset and env_offset + self.E <= envs_total
        self.env_offset, self.envs_total = int(env_offset), int(envs_total)

    def new_update(self):
        self.total_action_rep = np.zeros((self.A, self.R), dtype=np.int64)
        self.nb_actions = 0

    def step(self, global_step, a_idx, r_idx, reward, over, rewards_out, masks_out):
        """Returns the new global_step; fills rewards_out/masks_out (float32 views) in place."""
        a_idx = np.asarray(a_idx, dtype=np.int64)
        r_idx = np.asarray(r_idx, dtype=np.int64)
        reward = np.asarray(reward, dtype=np.float32)
        over = np.asarray(over)
        masks_out[...] = 1.0 - over.astype(np.float32)
        self.total_episode_rewards += reward
        rewards_out[...] = np.clip(reward, -1.0, 1.0)
        self.emulator_steps += self.tab[r_idx] + 1
        np.add.at(self.total_action_rep, (a_idx, r_idx), 1)
        self.nb_actions += int((r_idx + 1).sum())
        ended = np.nonzero(over)[0]
        for e in ended:
            self.total_rewards.append(float(self.total_episode_rewards[e]))
            self.total_steps.append(int(self.emulator_steps[e]))
            self.episodes.append((global_step + self.env_offset + int(e) + 1, float(self.total_episode_rewards[e]),
                                  int(self.emulator_steps[e])))
        self.total_episode_rewards[ended] = 0
        self.emulator_steps[ended] = 0
        return global_step + self.envs_total

    def histograms(self):
        """paac.py:269-275: the values log_histogram would receive."""
        nb_a = self.total_action_rep.sum(1)
        nb_r = self.total_action_rep.sum(0)
        histo_a = np.repeat(np.arange(self.A), nb_a)
        histo_r = np.repeat(self.tab + 1, nb_r)
        return histo_a, histo_r


class NativeBook(object):
    """The same bookkeeping in libmanette_host.so (mh_book_*), used by the learner so a native
    macro-step needs no Python; interface of Bookkeeper (tests pin one against the other)."""

    def __init__(self, n_envs, num_actions, tab_rep):
        import ctypes as C
        from . import _lib
        self._C = C
        self._lib = _lib
        self.E = n_envs
        self.A = num_actions
        self.tab = np.ascontiguousarray(np.asarray(tab_rep, dtype=np.int32))
        self.R = len(self.tab)
        h = C.c_void_p()
        _lib.check_host(_lib.host().mh_book_create(n_envs, num_actions, self.tab.ctypes.data_as(C.c_void_p),
                                                   self.R, C.byref(h)), 'mh_book_create')
        self._h = h
        self.total_rewards = []
        self.total_steps = []
        self.episodes = []

    def set_shard(self, env_offset, envs_total):
        self._lib.check_host(self._lib.host().mh_book_set_shard(self._h, int(env_offset), int(envs_total)),
                             'mh_book_set_shard')

    @property
    def handle(self):
        return self._h

    def step(self, global_step, a_idx, r_idx, reward, over, rewards_out, masks_out):
        C = self._C
        gs = C.c_int64(global_step)
        arrs = [np.ascontiguousarray(a_idx, np.int32), np.ascontiguousarray(r_idx, np.int32),
                np.ascontiguousarray(reward, np.float32), np.ascontiguousarray(over, np.float32)]
        assert rewards_out.flags.c_contiguous and masks_out.flags.c_contiguous
        self._lib.check_host(self._lib.host().mh_book_step(
            self._h, C.byref(gs), *[a.ctypes.data_as(C.c_void_p) for a in arrs],
            rewards_out.ctypes.data_as(C.c_void_p), masks_out.ctypes.data_as(C.c_void_p)), 'mh_book_step')
        self.drain()
        return gs.value

    def drain(self):
        C = self._C
        n = C.c_int(1)
        while n.value:
            st = np.zeros(256, np.int64)
            rw = np.zeros(256, np.float32)
            ln = np.zeros(256, np.int64)
            self._lib.check_host(self._lib.host().mh_book_pop_episodes(
                self._h, st.ctypes.data_as(C.c_void_p), rw.ctypes.data_as(C.c_void_p),
                ln.ctypes.data_as(C.c_void_p), 256, C.byref(n)))
            for i in range(n.value):
                self.total_rewards.append(float(rw[i]))
                self.total_steps.append(int(ln[i]))
                self.episodes.append((int(st[i]), float(rw[i]), int(ln[i])))

    def new_update(self):
        self._lib.check_host(self._lib.host().mh_book_new_update(self._h))

    def histograms(self):
        C = self._C
        hist = np.zeros((self.A, self.R), np.int64)
        nb = C.c_int64()
        self._lib.check_host(self._lib.host().mh_book_histogram(self._h, hist.ctypes.data_as(C.c_void_p),
                                                                C.byref(nb)))
        self.nb_actions = nb.value
        return np.repeat(np.arange(self.A), hist.sum(1)), np.repeat(self.tab.astype(np.int64) + 1, hist.sum(0))

    def __del__(self):
        h = getattr(self, '_h', None)
        if h:
            self._lib.host().mh_book_destroy(h)
            self._h = None
