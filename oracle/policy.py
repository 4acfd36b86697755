"""Exploration / macro-action restatement (oracle): exploration_policy.py:5-116."""
import numpy as np


def tab_repetitions(max_repetition, nb_choices):
    """exploration_policy.py:56-62."""
    res = [0] * nb_choices
    res[-1] = max_repetition
    if nb_choices > 2:
        for i in range(1, nb_choices - 1):
            res[i] = int(max_repetition / (nb_choices - 1)) * i
    return res


class Action(object):
    """exploration_policy.py:5-36 (indices instead of one-hot rows)."""

    def __init__(self, tab_rep, a_idx, r_idx):
        self.current_action = int(a_idx)
        self.nb_repetitions_left = tab_rep[int(r_idx)]
        self.repeated = self.nb_repetitions_left > 0

    def repeat(self):
        self.nb_repetitions_left -= 1
        if self.nb_repetitions_left == 0:
            self.repeated = False
        return self.current_action

    def is_repeated(self):
        return self.repeated


def multinomial_choose(probs):
    """exploration_policy.py:108-116: one np.random.multinomial(1, p - epsneg) per row, from the
    GLOBAL numpy stream (the reference never seeds it; tests seed it)."""
    probs = probs - np.finfo(np.float32).epsneg
    return [int(np.nonzero(np.random.multinomial(1, p))[0]) for p in probs]


def e_greedy_choose(probs, epsilon):
    """exploration_policy.py:96-106."""
    out = []
    for p in probs:
        if np.random.rand(1)[0] < epsilon:
            out.append(np.random.randint(0, len(p)))
        else:
            out.append(np.argmax(p))
    return out


def argmax_choose(probs):
    """exploration_policy.py:89-94."""
    return [int(np.argmax(p)) for p in probs]
