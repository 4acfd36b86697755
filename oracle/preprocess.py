"""Frame preprocess restatement (oracle): atari_emulator.py:79-124, environment.py:42-80.

Per emulator.next(): 4 ALE frames, the last 2 screens pooled by np.amax (FramePool of 2),
resized 210x160 -> 84x84 with scipy.misc.imresize(interp='nearest') (= PIL NEAREST), pushed
into a 4-deep ObservationPool whose stacked output is oldest -> newest, channel-last; RGB
stacks reshape (84,84,3,4) -> (84,84,12), i.e. [R_t0..R_t3, G_t0..G_t3, B_t0..B_t3].
"""
import numpy as np


def nearest_lut(n_in, n_out):
    """PIL NEAREST source index per output index: x = 0.5*scale; idx = floor(x); x += scale
    (incremental float64 accumulation; pinned against PIL by tests/golden/preprocess.npz)."""
    scale = float(n_in) / float(n_out)
    out = np.empty(n_out, dtype=np.int64)
    x = 0.5 * scale
    for i in range(n_out):
        out[i] = min(int(np.floor(x)), n_in - 1)
        x += scale
    return out


ROW_LUT = nearest_lut(210, 84)
COL_LUT = nearest_lut(160, 84)


def pool_and_resize(f0, f1):
    """f0, f1: (210, 160, depth) uint8 -> (84, 84, depth) uint8."""
    img = np.maximum(f0, f1)
    return img[ROW_LUT][:, COL_LUT]


class ObservationStack(object):
    """environment.py:58-80 ObservationPool (ring of 4, output oldest -> newest)."""

    def __init__(self, depth=1):
        self.depth = depth
        self.pool = np.zeros((84, 84, depth, 4), dtype=np.uint8)
        self.idx = 0

    def push(self, obs):
        self.pool[:, :, :, self.idx] = obs.reshape(84, 84, self.depth)
        self.idx = (self.idx + 1) % 4

    def stacked(self):
        perm = [(self.idx + i) % 4 for i in range(4)]
        return np.copy(self.pool[:, :, :, perm]).reshape(84, 84, self.depth * 4)


def stack_update(prev, pushes, depth=1):
    """Device-kernel contract (mt_preprocess): new stack from prev stack + p pooled pushes."""
    p = len(pushes)
    prev = prev.reshape(84, 84, depth, 4)
    out = np.empty_like(prev)
    for c in range(4):
        if c < 4 - p:
            out[:, :, :, c] = prev[:, :, :, c + p]
        else:
            out[:, :, :, c] = pushes[c - (4 - p)].reshape(84, 84, depth)
    return out.reshape(84, 84, 4 * depth)
