"""Worker process stepping a block of Python emulators: emulator_runner.py:4-42 interface.

variables = [states, rewards, over, action indices, repetition indices] (indices instead of
the reference's one-hot rows: Action takes the argmax anyway)."""
from multiprocessing import Process

import numpy as np

from .exploration_policy import Action


def _onehot(i):
    v = np.zeros(int(i) + 1)
    v[int(i)] = 1.0
    return v


def run_emulators(tab_rep, emulators, variables):
    """emulator_runner.py:24-41 for one block."""
    states, rewards, over, a_idx, r_idx = variables[:5]
    for i, emulator in enumerate(emulators):
        act = Action(tab_rep, i, _onehot(a_idx[i]), _onehot(r_idx[i]))
        new_s, reward, episode_over = emulator.next(act.current_action)
        states[i] = emulator.get_initial_state() if episode_over else new_s
        rewards[i] = reward
        over[i] = episode_over
        while act.is_repeated() and not episode_over:
            new_s, reward, episode_over = emulator.next(act.repeat())
            states[i] = emulator.get_initial_state() if episode_over else new_s
            rewards[i] += reward
            over[i] = episode_over
        act.reset()


class EmulatorRunner(Process):
    def __init__(self, tab_rep, i, emulators, variables, queue, barrier):
        super(EmulatorRunner, self).__init__()
        self.id = i
        self.emulators = emulators
        self.variables = variables
        self.queue = queue
        self.barrier = barrier
        self.tab_rep = tab_rep

    def run(self):
        super(EmulatorRunner, self).run()
        self._run()

    def _run(self):
        while True:
            instruction = self.queue.get()
            if instruction is None:
                break
            run_emulators(self.tab_rep, self.emulators, self.variables)
            self.barrier.put(True)
