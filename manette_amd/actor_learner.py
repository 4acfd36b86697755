"""ActorLearner base: actor_learner.py:9-140 interface (folders, LR schedule, reward clip,
checkpoint save / restore, cleanup) over the HIP network.

Checkpoints: `<df>/checkpoints/-<global_step>.npz` (every variable under its TF name) and
`<df>/optimizer_checkpoints/-<global_step>.npz` (the RMSProp slots under their TF slot names
`<var>/OptimizerVariables` = ms and `<var>/OptimizerVariables_1` = mom), each directory with a
TF-style `checkpoint` index file; resume parses the step after the last '-' of the latest
checkpoint (networks.py:162-175). numpy archives are written and read without pickles.
"""
import logging
import os

import numpy as np


def _latest(folder):
    idx = os.path.join(folder, 'checkpoint')
    if not os.path.exists(idx):
        return None
    for line in open(idx):
        if line.startswith('model_checkpoint_path:'):
            name = line.split(':', 1)[1].strip().strip('"')
            path = name if os.path.isabs(name) else os.path.join(folder, name)
            return path if os.path.exists(path + '.npz') else None
    return None


def _write(folder, step, arrays, max_to_keep=None):
    os.makedirs(folder, exist_ok=True)
    base = os.path.join(folder, '-%d' % step)
    tmp = base + '.tmp.npz'
    np.savez(tmp, **arrays)
    os.replace(tmp, base + '.npz')
    with open(os.path.join(folder, 'checkpoint'), 'w') as f:
        f.write('model_checkpoint_path: "-%d"\n' % step)
    if max_to_keep:
        olds = sorted((int(n[1:-4]) for n in os.listdir(folder)
                       if n.startswith('-') and n.endswith('.npz') and not n.endswith('.tmp.npz')))
        for s in olds[:-max_to_keep]:
            os.remove(os.path.join(folder, '-%d.npz' % s))


class ActorLearner(object):
    def __init__(self, network_creator, environment_creator, explo_policy, args):
        self.checkpoint_interval = args.checkpoint_interval
        self.debugging_folder = args.debugging_folder
        self.network_checkpoint_folder = os.path.join(self.debugging_folder, 'checkpoints/')
        self.optimizer_checkpoint_folder = os.path.join(self.debugging_folder, 'optimizer_checkpoints/')
        self.last_saving_step = 0
        self.device = args.device
        self.game = args.game
        self.global_step = 0
        self.max_global_steps = args.max_global_steps
        self.max_local_steps = args.max_local_steps
        self.num_actions = args.num_actions
        self.explo_policy = explo_policy
        self.gamma = args.gamma
        self.initial_lr = args.initial_lr
        self.lr_annealing_steps = args.lr_annealing_steps
        self.emulator_counts = args.emulator_counts
        self.environment_creator = environment_creator
        self.network = network_creator()
        self.is_chief = True

    def save_vars(self, force=False):
        if force or self.global_step - self.last_saving_step >= self.checkpoint_interval:
            self.last_saving_step = self.global_step
            if not self.is_chief:
                return
            P = self.network.get_variables('params')
            ms = self.network.get_variables('ms')
            mom = self.network.get_variables('mom')
            _write(self.network_checkpoint_folder, self.last_saving_step, P)
            slots = {}
            for k in ms:
                slots[k + '/OptimizerVariables'] = ms[k]
                slots[k + '/OptimizerVariables_1'] = mom[k]
            _write(self.optimizer_checkpoint_folder, self.last_saving_step, slots, max_to_keep=1)

    def rescale_reward(self, reward):
        """Clip immediate reward (actor_learner.py:108-114)."""
        if reward > 1.0:
            reward = 1.0
        elif reward < -1.0:
            reward = -1.0
        return reward

    def init_network(self):
        os.makedirs(self.network_checkpoint_folder, exist_ok=True)
        os.makedirs(self.optimizer_checkpoint_folder, exist_ok=True)
        last_saving_step = 0
        path = _latest(self.network_checkpoint_folder)
        if path is None:
            logging.info('Initializing all variables')
            self.network.init_params(getattr(self, 'seed', 0))
        else:
            logging.info('Restoring network variables from previous run')
            with np.load(path + '.npz', allow_pickle=False) as z:
                self.network.set_variables({k: z[k] for k in z.files})
            last_saving_step = int(path[path.rindex('-') + 1:])
        opath = _latest(self.optimizer_checkpoint_folder)
        if opath is not None:
            logging.info('Restoring optimizer variables from previous run')
            with np.load(opath + '.npz', allow_pickle=False) as z:
                ms = {k[:-len('/OptimizerVariables')]: z[k] for k in z.files if k.endswith('/OptimizerVariables')}
                mom = {k[:-len('/OptimizerVariables_1')]: z[k] for k in z.files if k.endswith('/OptimizerVariables_1')}
            self.network.set_variables(ms, 'ms')
            self.network.set_variables(mom, 'mom')
        self.last_saving_step = last_saving_step
        return last_saving_step

    def get_lr(self):
        if self.global_step <= self.lr_annealing_steps:
            return self.initial_lr - (self.global_step * self.initial_lr / self.lr_annealing_steps)
        return 0.0

    def cleanup(self):
        self.save_vars(True)
