"""Emulator contract and the host-side frame pool / observation stack.

Interface of environment.py:4-80 (BaseEnvironment, FramePool, ObservationPool). The batched
device version of the same preprocess is mt_preprocess (A2); this CPU one serves emulators
that hand back finished observations (the reference contract) and the Python runner path.
"""
import numpy as np


class BaseEnvironment(object):
    def get_initial_state(self):
        """Reset; return the initial (84, 84, 4*depth) uint8 observation."""
        raise NotImplementedError()

    def next(self, action):
        """Apply action index; return (observation, reward, is_terminal)."""
        raise NotImplementedError()

    def get_legal_actions(self):
        raise NotImplementedError()

    def get_noop(self):
        raise NotImplementedError()

    def on_new_frame(self, frame):
        pass


def nearest_lut(n_in, n_out):
    """Source index of each output index for PIL NEAREST resize (what scipy.misc.imresize(...,
    interp='nearest') did, atari_emulator.py:85): x = 0.5*scale; idx = floor(x); x += scale."""
    scale = float(n_in) / float(n_out)
    out = np.empty(n_out, dtype=np.int32)
    x = 0.5 * scale
    for i in range(n_out):
        out[i] = min(int(np.floor(x)), n_in - 1)
        x += scale
    return out


ROW_LUT = nearest_lut(210, 84)
COL_LUT = nearest_lut(160, 84)


class FramePool(object):
    """environment.py:42-55: the last two screens; processed = max -> nearest 84x84."""

    def __init__(self, frame_pool, operation=None):
        self.frame_pool = frame_pool
        self.frame_pool_index = 0
        self.frames_in_pool = frame_pool.shape[0]
        self.operation = operation or process_frame_pool

    def new_frame(self, frame):
        self.frame_pool[self.frame_pool_index] = frame
        self.frame_pool_index = (self.frame_pool_index + 1) % self.frames_in_pool

    def get_processed_frame(self):
        return self.operation(self.frame_pool)


def process_frame_pool(frame_pool):
    """atari_emulator.py:79-88 (np.amax over the pool, nearest resize)."""
    img = np.amax(frame_pool, axis=0)
    return img[ROW_LUT][:, COL_LUT]


class ObservationPool(object):
    """environment.py:58-80: ring of 4 observations, stacked oldest -> newest."""

    def __init__(self, observation_pool, rgb=False):
        self.depth = 3 if rgb else 1
        self.observation_pool = observation_pool
        self.pool_size = observation_pool.shape[-1]
        self.current_observation_index = 0

    def new_observation(self, observation):
        self.observation_pool[:, :, :, self.current_observation_index] = observation.reshape(
            84, 84, self.depth)
        self.current_observation_index = (self.current_observation_index + 1) % self.pool_size

    def get_pooled_observations(self):
        perm = [(self.current_observation_index + i) % self.pool_size for i in range(self.pool_size)]
        return np.copy(self.observation_pool[:, :, :, perm]).reshape(84, 84, self.depth * self.pool_size)
