"""Per-step rollout bookkeeping (A8), vectorised over the env axis: paac.py:154-205.

Exact integer semantics of the reference loop:
  rewards[t] = clip(summed reward, +-1)                      (:180, actor_learner.py:108-114)
  masks[t] = 1 - over                                        (:176)
  emulator_steps[e] += tab_rep[r_e] + 1 (planned repeats)   (:183)
  global_step += 1 per env, in env order                    (:184)
  total_action_rep[a_e][r_e] += 1; nb_actions += r_e + 1     (:157, :187-189)
  on over: log (global_step at env e, total reward, emulator_steps), reset both   (:191-201)
Total episode rewards accumulate in float32 (the shared reward array is float32).
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
        self.new_update()

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
            self.episodes.append((global_step + int(e) + 1, float(self.total_episode_rewards[e]),
                                  int(self.emulator_steps[e])))
        self.total_episode_rewards[ended] = 0
        self.emulator_steps[ended] = 0
        return global_step + self.E

    def histograms(self):
        """paac.py:269-275: the values log_histogram would receive."""
        nb_a = self.total_action_rep.sum(1)
        nb_r = self.total_action_rep.sum(0)
        histo_a = np.repeat(np.arange(self.A), nb_a)
        histo_r = np.repeat(self.tab + 1, nb_r)
        return histo_a, histo_r
