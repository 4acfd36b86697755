"""Action selection and FiGAR macro-actions: the interface of exploration_policy.py:5-116.

Parity mode keeps the reference's numpy draws (global np.random stream, one multinomial per
row for the action and one for the repetition) so a seeded run samples exactly what the
reference samples; the device sampler (network.sample / mt_sample) is the perf-mode
alternative with the same distribution.
"""
import numpy as np

_EPSNEG = np.finfo(np.float32).epsneg


class Action(object):
    """exploration_policy.py:5-36."""

    def __init__(self, tab_rep, i, a, r):
        self.tab_rep = tab_rep
        self.id = i
        self.repeated = False
        self.current_action = 0
        self.nb_repetitions_left = 0
        self.init_from_list(a, r)

    def __str__(self):
        return 'id : %s, action %s repeated %s times.' % (self.id, self.current_action, self.nb_repetitions_left)

    def init_from_list(self, a, r):
        self.current_action = int(np.argmax(a))
        self.nb_repetitions_left = self.tab_rep[int(np.argmax(r))]
        if self.nb_repetitions_left > 0:
            self.repeated = True

    def repeat(self):
        self.nb_repetitions_left -= 1
        if self.nb_repetitions_left == 0:
            self.repeated = False
        return self.current_action

    def reset(self):
        self.repeated = False
        self.current_action = 0
        self.nb_repetitions_left = 0

    def is_repeated(self):
        return self.repeated


class ExplorationPolicy(object):
    """exploration_policy.py:39-116 (same constructor arguments and outputs)."""

    def __init__(self, args, test=False):
        self.test = test
        self.global_step = 0
        self.egreedy_policy = args.egreedy
        self.initial_epsilon = args.epsilon
        self.epsilon = args.epsilon
        self.softmax_temp = args.softmax_temp
        self.keep_percentage = args.keep_percentage
        self.annealed = args.annealed
        self.annealing_steps = getattr(args, 'annealed_steps', 80000000)
        self.max_repetition = args.max_repetition
        self.nb_choices = args.nb_choices
        self.tab_rep = self.get_tab_repetitions()

    def get_tab_repetitions(self):
        res = [0] * self.nb_choices
        res[-1] = self.max_repetition
        if self.nb_choices > 2:
            for i in range(1, self.nb_choices - 1):
                res[i] = int(self.max_repetition / (self.nb_choices - 1)) * i
        return res

    def get_epsilon(self):
        if self.global_step <= self.annealing_steps:
            return self.initial_epsilon - (self.global_step * self.initial_epsilon / self.annealing_steps)
        return 0.0

    def choose_indices(self, network_output_pi, network_output_rep):
        if self.test:
            a = self.argmax_choose(network_output_pi)
            r = self.argmax_choose(network_output_rep)
        elif self.egreedy_policy:
            a = self.e_greedy_choose(network_output_pi)
            r = self.e_greedy_choose(network_output_rep)
        else:
            a = self.multinomial_choose(network_output_pi)
            r = self.multinomial_choose(network_output_rep)
        self.global_step += len(network_output_pi)
        if self.annealed:
            # the reference calls a bare get_epsilon() here (NameError, exploration_policy.py:85)
            self.epsilon = self.get_epsilon()
        return np.asarray(a, dtype=np.int32), np.asarray(r, dtype=np.int32)

    def choose_next_actions(self, network_output_pi, network_output_rep, num_actions):
        a, r = self.choose_indices(network_output_pi, network_output_rep)
        return np.eye(num_actions)[a], np.eye(self.nb_choices)[r]

    def argmax_choose(self, probs):
        return [int(np.argmax(p)) for p in probs]

    def e_greedy_choose(self, probs):
        out = []
        for p in probs:
            if np.random.rand(1)[0] < self.epsilon:
                out.append(np.random.randint(0, len(p)))
            else:
                out.append(int(np.argmax(p)))
        return out

    def multinomial_choose(self, probs):
        # p - epsneg as the reference; entries below epsneg would make numpy >= 1.17 raise
        # "pvals < 0" (the reference crashes there) — they are clamped to 0, which changes
        # nothing whenever the reference itself can draw.
        probs = np.maximum(np.asarray(probs, dtype=np.float32) - _EPSNEG, 0)
        return [int(np.nonzero(np.random.multinomial(1, p))[0]) for p in probs]
