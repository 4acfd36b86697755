"""Synthetic ALE stand-in (ALE is not installed here or on the GPU box; no ROM can run).

Deterministic per-env streams from np.random.RandomState(1000 + global_env_id):
a ring of RING raw 210x160 screens (uniform uint8) and a reward table with
P(-1, 0, +1) = (0.05, 0.90, 0.05). Episodes end after EPISODE_LEN next() calls.
Each next() "plays" 4 ALE frames and exposes the last two screens (atari_emulator.py:90-100):
push k uses screens (ring[2k % RING], ring[(2k+1) % RING]); get_initial_state() makes 4 pushes.

Two faces of the same emulator:
  * SyntheticEmulator: the reference contract (BaseEnvironment.next -> 84x84x4 observation),
    preprocessed on the CPU — used by the Python runner path and the CPU baseline;
  * SyntheticBank: all envs' streams in two arrays for the native runner (libmanette_host),
    whose screens go to the GPU raw and are preprocessed by mt_preprocess.
"""
import numpy as np

from .environment import BaseEnvironment, FramePool, ObservationPool

RING = 64
REWARD_LEN = 4096
EPISODE_LEN = 997


def env_streams(global_env_id, depth=1, ring=RING, reward_len=REWARD_LEN):
    rs = np.random.RandomState(1000 + int(global_env_id))
    screens = rs.randint(0, 256, size=(ring, 210, 160, depth), dtype=np.uint8)
    rewards = rs.choice(np.array([-1.0, 0.0, 1.0]), p=[0.05, 0.90, 0.05], size=reward_len).astype(np.float32)
    return screens, rewards


class SyntheticEmulator(BaseEnvironment):
    def __init__(self, global_env_id, num_actions=6, rgb=False, episode_len=EPISODE_LEN):
        self.depth = 3 if rgb else 1
        self.screens, self.rewards = env_streams(global_env_id, self.depth)
        self.num_actions = num_actions
        self.episode_len = episode_len
        self.k = 0
        self.steps = 0
        self.frame_pool = FramePool(np.empty((2, 210, 160, self.depth), dtype=np.uint8))
        self.observation_pool = ObservationPool(np.zeros((84, 84, self.depth, 4), dtype=np.uint8), rgb)

    def _push(self):
        self.frame_pool.new_frame(self.screens[(2 * self.k) % RING])
        self.frame_pool.new_frame(self.screens[(2 * self.k + 1) % RING])
        self.observation_pool.new_observation(self.frame_pool.get_processed_frame())
        self.k += 1

    def get_initial_state(self):
        for _ in range(4):
            self._push()
        self.steps = 0
        return self.observation_pool.get_pooled_observations()

    def next(self, action):
        reward = float(self.rewards[self.k % REWARD_LEN])
        self._push()
        self.steps += 1
        return self.observation_pool.get_pooled_observations(), reward, self.steps >= self.episode_len

    def get_legal_actions(self):
        return np.arange(self.num_actions)

    def get_noop(self):
        return 0


class SyntheticBank(object):
    """Streams of envs [first, first+n) in the layout mh_runner_create takes. The screen ring
    lives in pinned (page-locked, device-mapped) host memory when a GPU is present, as an ALE
    worker's frame buffers would, so the GPU can read screens where the emulators left them
    (mh_runner_step_frames + mt_preprocess_frames)."""

    def __init__(self, first_env_id, n_envs, rgb=False, episode_len=EPISODE_LEN, pinned=None):
        import torch
        depth = 3 if rgb else 1
        self.depth = depth
        pinned = torch.cuda.is_available() if pinned is None else pinned
        self.screens_t = torch.empty((n_envs, RING, 210, 160, depth), dtype=torch.uint8, pin_memory=pinned)
        self.screens = self.screens_t.numpy()
        self.rewards = np.empty((n_envs, REWARD_LEN), dtype=np.float32)
        for i in range(n_envs):
            self.screens[i], self.rewards[i] = env_streams(first_env_id + i, depth)
        self.frame_bytes = 210 * 160 * depth
        self.episode_len = episode_len
