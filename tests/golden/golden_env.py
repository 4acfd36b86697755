"""Deterministic emulators used to generate and replay the host-loop golden fixtures.

Test infrastructure only. `GoldenEnv` honours the reference emulator contract
(environment.py:4-39: get_initial_state() / next(action) -> (obs uint8 84x84x(4*depth),
reward float, terminal bool)); its observations depend on the env id, a per-env call counter
and the action, so a replay that routes actions or resets wrongly produces different states.
`FakeALE` stands in for ale_python_interface.ALEInterface (un-vendored, not installed) with
seeded pseudo-random 210x160 screens, so atari_emulator.py's own preprocess can be recorded.
"""
import numpy as np


class GoldenEnv(object):
    def __init__(self, env_id, depth=1):
        self.id = int(env_id)
        self.depth = depth
        self.k = 0            # calls to next()/get_initial_state() so far
        self.steps = 0        # next() calls in the current episode
        self.episode_len = 4 + (self.id % 5)

    def _obs(self, action):
        base = (self.id * 37 + self.k * 11 + int(action) * 5) % 256
        obs = np.empty((84, 84, 4 * self.depth), dtype=np.uint8)
        for c in range(4 * self.depth):
            obs[:, :, c] = (base + 3 * c) % 256
        obs[0, 0, 0] = self.k % 256
        obs[1, 0, 0] = self.id % 256
        return obs

    def get_initial_state(self):
        self.k += 1
        self.steps = 0
        return self._obs(0)

    def next(self, action):
        self.k += 1
        self.steps += 1
        reward = float(((self.id + 3 * self.k + int(action)) % 7) - 3)  # [-3, 3]: exercises clipping
        terminal = self.steps >= self.episode_len
        return self._obs(action), reward, terminal


def fake_screen(frame_idx, rgb=False):
    """The screen FakeALE shows after its frame_idx-th act() call."""
    rs = np.random.RandomState(10007 + frame_idx)
    if rgb:
        return rs.randint(0, 256, size=(210, 160, 3)).astype(np.uint8)
    return rs.randint(0, 256, size=(210, 160, 1)).astype(np.uint8)


class FakeALE(object):
    """Minimal ALEInterface stand-in: 6 minimal actions, game over after `over_after` acts."""

    def __init__(self, over_after=10 ** 9):
        self.frame = 0
        self.over_after = over_after
        self.acts_in_game = 0

    def setInt(self, *a):
        pass

    def setFloat(self, *a):
        pass

    def setBool(self, *a):
        pass

    def loadROM(self, *a):
        pass

    def getMinimalActionSet(self):
        return np.arange(6, dtype=np.int32)

    def getScreenDims(self):
        return 160, 210

    def lives(self):
        return 3

    def act(self, a):
        self.frame += 1
        self.acts_in_game += 1
        return float((self.frame % 3) - 1)

    def getScreenGrayscale(self, out):
        out[...] = fake_screen(self.frame, rgb=False)

    def getScreenRGB(self, out):
        out[...] = fake_screen(self.frame, rgb=True)

    def game_over(self):
        return self.acts_in_game >= self.over_after

    def reset_game(self):
        self.acts_in_game = 0
