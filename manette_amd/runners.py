"""Host-side emulator runners (A1): runners.py:7-50 + emulator_runner.py:19-42.

NativeRunners  — the hot path: a libmanette_host.so thread pool steps a native emulator bank
                 and writes every env's pushed screens into ONE pinned staging buffer: compact
                 (copied to HBM on the learner's stream for mt_preprocess) or, with
                 fixed_slots, at slots [4e, 4e+n) for kernels that read it in place.
Runners        — the reference interface for Python emulators (BaseEnvironment objects,
                 e.g. an ALE wrapper): `ew` worker processes over shared memory, a go-queue per
                 worker and a barrier queue; workers=0 runs the same loop in process.
"""
import ctypes as C
import multiprocessing as mp
from multiprocessing.sharedctypes import RawArray

import numpy as np
import torch

from . import _lib
from .emulator_runner import EmulatorRunner, run_emulators


def _np(t):
    return t.numpy()


class NativeRunners(object):
    """row_select: screen rows to stage (None = whole 210-row screens). The learner passes the
    84 rows the nearest resize reads, so only those cross PCIe. fixed_slots: MH_RUNNER_FIXED_SLOTS
    (env e's pushes at staging slots 4e.., one worker phase per step). pooled: MH_RUNNER_POOLED
    (one staged screen per push, max of its two frames, atari_emulator.py:79-88). resized:
    MH_RUNNER_RESIZED (the final 84x84 frame of each push, pool + resize on the host threads;
    needs the 84-row row_select and the column LUT col_lut)."""

    def __init__(self, bank, n_workers, tab_rep, row_select=None, fixed_slots=False, pooled=False, resized=False,
                 col_lut=None):
        """in-place frame mode (reset_frames / step_frames) needs no row_select: the screens stay
        in the bank, only their indices are written (frames [E][8] + push_count)."""
        self.bank = bank
        self.E = bank.screens.shape[0]
        self.tab = np.ascontiguousarray(np.asarray(tab_rep, dtype=np.int32))
        self.rows = None if row_select is None else np.ascontiguousarray(np.asarray(row_select, np.int32))
        self.src_rows = 210 if self.rows is None else len(self.rows)
        self.frame_bytes = bank.frame_bytes // 210 * self.src_rows  # one staged screen
        if resized:
            self.frame_bytes = 84 * 84 * bank.depth
        h = C.c_void_p()
        lib = _lib.host()
        _lib.check_host(lib.mh_runner_create(
            self.E, int(n_workers), self.tab.ctypes.data_as(C.c_void_p), len(self.tab),
            bank.screens.ctypes.data_as(C.c_void_p), bank.screens.shape[1], bank.frame_bytes,
            bank.rewards.ctypes.data_as(C.c_void_p), bank.rewards.shape[1], bank.episode_len,
            None if self.rows is None else self.rows.ctypes.data_as(C.c_void_p),
            0 if self.rows is None else len(self.rows),
            (_lib.MH_RUNNER_FIXED_SLOTS if fixed_slots else 0) | (_lib.MH_RUNNER_POOLED if pooled else 0) |
            (_lib.MH_RUNNER_RESIZED if resized else 0), C.byref(h)), 'mh_runner_create')
        self.fixed_slots = bool(fixed_slots)
        self.pooled = bool(pooled)
        self.resized = bool(resized)
        if resized:
            self._cols = np.ascontiguousarray(np.asarray(col_lut, dtype=np.int32))
            _lib.check_host(lib.mh_runner_set_col_lut(h, self._cols.ctypes.data_as(C.c_void_p), len(self._cols)),
                            'mh_runner_set_col_lut')
        self._h = h
        pin = torch.cuda.is_available()
        mk = lambda *shape, dtype: torch.zeros(*shape, dtype=dtype, pin_memory=pin)
        self.staging = mk(4 * self.E, 1 if (pooled or resized) else 2, self.frame_bytes, dtype=torch.uint8)
        self.push_meta = mk(2, self.E, dtype=torch.int32)  # [offset; count]: one H2D copy
        self.push_offset = self.push_meta[0]
        self.push_count = self.push_meta[1]
        self.reward = mk(self.E, dtype=torch.float32)
        self.over = mk(self.E, dtype=torch.float32)
        self.frames = mk(self.E, 8, dtype=torch.int32)  # in-place mode: bank frame indices
        self.total = 0

    def _ptr(self, t):
        return C.c_void_p(t.data_ptr())

    def reset(self):
        """get_initial_state() of every env (paac.py:98): 4 pushes each."""
        tot = C.c_int()
        _lib.check_host(_lib.host().mh_runner_reset(self._h, self._ptr(self.staging), self._ptr(self.push_offset),
                                                    self._ptr(self.push_count), C.byref(tot)), 'mh_runner_reset')
        self.total = tot.value
        return self.total

    def step(self, a_idx, r_idx):
        """a_idx/r_idx: int32 host arrays/tensors [E]. Returns the number of staged pushes."""
        a = a_idx if isinstance(a_idx, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a_idx, np.int32))
        r = r_idx if isinstance(r_idx, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(r_idx, np.int32))
        tot = C.c_int()
        _lib.check_host(_lib.host().mh_runner_step(
            self._h, self._ptr(a), self._ptr(r), self._ptr(self.staging), self._ptr(self.push_offset),
            self._ptr(self.push_count), self._ptr(self.reward), self._ptr(self.over), C.byref(tot)),
            'mh_runner_step')
        self.total = tot.value
        return self.total

    def reset_frames(self):
        """get_initial_state() of every env, in-place mode: frames/push_count name the screens."""
        _lib.check_host(_lib.host().mh_runner_reset_frames(self._h, self._ptr(self.frames),
                                                           self._ptr(self.push_count)), 'mh_runner_reset_frames')

    def step_frames(self, a_idx, r_idx):
        """One macro-step, in-place mode (no screen copied): fills frames, push_count, reward, over."""
        a = a_idx if isinstance(a_idx, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a_idx, np.int32))
        r = r_idx if isinstance(r_idx, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(r_idx, np.int32))
        _lib.check_host(_lib.host().mh_runner_step_frames(
            self._h, self._ptr(a), self._ptr(r), self._ptr(self.frames), self._ptr(self.push_count),
            self._ptr(self.reward), self._ptr(self.over)), 'mh_runner_step_frames')

    def env_state(self, e):
        k = C.c_int64()
        s = C.c_int32()
        _lib.check_host(_lib.host().mh_runner_env_state(self._h, e, C.byref(k), C.byref(s)))
        return k.value, s.value

    def set_threads(self, cpus, spin_us=2000):
        """Pin worker w to cpus[w] and set the idle spin before the futex sleep
        (mh_runner_set_threads; manette_amd/placement.py plans both per rank)."""
        c = np.ascontiguousarray(np.asarray(list(cpus), dtype=np.int32))
        _lib.check_host(_lib.host().mh_runner_set_threads(self._h, c.ctypes.data_as(C.c_void_p), len(c), int(spin_us)),
                        'mh_runner_set_threads')

    def stats(self, reset=False):
        """(staging us, busy us) per worker per step and the step count since the last reset
        (mh_runner_stats): staging = frame pool + resize + copy into the pinned staging."""
        out = (C.c_double * 3)()
        _lib.check_host(_lib.host().mh_runner_stats(self._h, out, 3, int(bool(reset))), 'mh_runner_stats')
        return dict(stage_us=out[0], busy_us=out[1], steps=int(out[2]))

    def thread_cpus(self):
        """Per worker: the one cpu it may run on, or -1 (several allowed)."""
        out = np.zeros(256, np.int32)
        n = _lib.host().mh_runner_thread_cpus(self._h, out.ctypes.data_as(C.c_void_p), len(out))
        if n < 0:
            raise RuntimeError(_lib.host().mh_last_error().decode())
        return [int(x) for x in out[:n]]

    def stop(self):
        if getattr(self, '_h', None):
            _lib.host().mh_runner_destroy(self._h)
            self._h = None

    def __del__(self):
        self.stop()


class Runners(object):
    """runners.py:7-50 interface: Runners(tab_rep, EmulatorRunner, emulators, workers, variables)
    with variables = [states, rewards, over, action indices, repetition indices]."""

    def __init__(self, tab_rep, runner_cls, emulators, workers, variables):
        self.workers = workers
        if workers == 0:
            self.variables = variables
            self._inline = (tab_rep, list(emulators))
            return
        self.variables = [self._get_shared(v) for v in variables]
        self.queues = [mp.Queue() for _ in range(workers)]
        self.barrier = mp.Queue()
        blocks = np.array_split(np.arange(len(emulators)), workers)
        self.runners = [runner_cls(tab_rep, i, [emulators[j] for j in blk],
                                   [v[blk[0]:blk[-1] + 1] for v in self.variables], self.queues[i],
                                   self.barrier)
                        for i, blk in enumerate(blocks)]

    @staticmethod
    def _get_shared(array):
        ctype = {np.dtype(np.float32): C.c_float, np.dtype(np.float64): C.c_double,
                 np.dtype(np.uint8): C.c_uint8, np.dtype(np.int32): C.c_int32}[array.dtype]
        shared = RawArray(ctype, array.size)
        out = np.frombuffer(shared, array.dtype).reshape(array.shape)
        out[...] = array
        return out

    def start(self):
        if self.workers:
            for r in self.runners:
                r.daemon = True
                r.start()

    def stop(self):
        if self.workers:
            for q in self.queues:
                q.put(None)
            for r in self.runners:
                r.join(timeout=5)

    def get_shared_variables(self):
        return self.variables

    def update_environments(self):
        if self.workers == 0:
            tab_rep, emus = self._inline
            run_emulators(tab_rep, emus, self.variables)
            return
        for q in self.queues:
            q.put(True)

    def wait_updated(self):
        if self.workers == 0:
            return
        for _ in range(self.workers):
            self.barrier.get()
