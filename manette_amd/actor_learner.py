"""ActorLearner base: actor_learner.py:9-140 interface (folders, LR schedule, reward clip,
checkpoint save / restore, cleanup) over the HIP network.

Checkpoints are TensorFlow tensor bundles (manette_amd/tf_bundle.py), as tf.train.Saver writes
them (actor_learner.py:84-87, :102-106): `<df>/checkpoints/-<global_step>.{index,data-00000-of-00001}`
holds every variable under its TF name plus its RMSProp slots `<var>/OptimizerVariables` (ms)
and `<var>/OptimizerVariables_1` (mom) (Saver() of all global variables, max_to_keep 5);
`<df>/optimizer_checkpoints/-<global_step>.*` holds the slots only (max_to_keep 1). Each folder
has TF's `checkpoint` text file (model_checkpoint_path + all_model_checkpoint_paths). Restore
(networks.py:162-175, actor_learner.py:116-130) reads the latest bundle of each folder and the
step after the last '-' of its name.
"""
import logging
import os

from . import tf_bundle

SLOT_MS, SLOT_MOM = '/OptimizerVariables', '/OptimizerVariables_1'


def _latest(folder):
    """tf.train.latest_checkpoint: the prefix named by `checkpoint`, if its index exists."""
    idx = os.path.join(folder, 'checkpoint')
    if not os.path.exists(idx):
        return None
    for line in open(idx):
        if line.startswith('model_checkpoint_path:'):
            name = line.split(':', 1)[1].strip().strip('"')
            path = name if os.path.isabs(name) else os.path.join(folder, name)
            return path if os.path.exists(path + '.index') else None
    return None


def _all_paths(folder):
    idx = os.path.join(folder, 'checkpoint')
    if not os.path.exists(idx):
        return []
    return [line.split(':', 1)[1].strip().strip('"') for line in open(idx)
            if line.startswith('all_model_checkpoint_paths:')]


def _write(folder, step, arrays, max_to_keep=5):
    os.makedirs(folder, exist_ok=True)
    name = '-%d' % step
    tf_bundle.write_bundle(os.path.join(folder, name), arrays)
    keep = [p for p in _all_paths(folder) if p != name] + [name]
    for old in keep[:-max_to_keep]:
        for f in os.listdir(folder):
            if f.startswith(old + '.'):
                os.remove(os.path.join(folder, f))
    keep = keep[-max_to_keep:]
    tmp = os.path.join(folder, 'checkpoint.tmp')
    with open(tmp, 'w') as f:
        f.write('model_checkpoint_path: "%s"\n' % name)
        for k in keep:
            f.write('all_model_checkpoint_paths: "%s"\n' % k)
    os.replace(tmp, os.path.join(folder, 'checkpoint'))


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
            slots = {}
            for k in ms:
                slots[k + SLOT_MS] = ms[k]
                slots[k + SLOT_MOM] = mom[k]
            _write(self.network_checkpoint_folder, self.last_saving_step, dict(P, **slots))
            _write(self.optimizer_checkpoint_folder, self.last_saving_step, slots, max_to_keep=1)

    def rescale_reward(self, reward):
        """Clip immediate reward (actor_learner.py:108-114)."""
        if reward > 1.0:
            reward = 1.0
        elif reward < -1.0:
            reward = -1.0
        return reward

    def _restore(self, tensors):
        """Variables and RMSProp slots of a bundle into the device buffers (names must match)."""
        names = {n for n, _, _, _ in self.network.vars}
        P, ms, mom = {}, {}, {}
        for k, v in tensors.items():
            if k.endswith(SLOT_MOM):
                mom[k[:-len(SLOT_MOM)]] = v
            elif k.endswith(SLOT_MS):
                ms[k[:-len(SLOT_MS)]] = v
            else:
                P[k] = v
        unknown = (set(P) | set(ms) | set(mom)) - names
        if unknown:
            raise ValueError('checkpoint variables not in this network: %s' % sorted(unknown)[:5])
        if P:
            self.network.set_variables(P)
        if ms:
            self.network.set_variables(ms, 'ms')
        if mom:
            self.network.set_variables(mom, 'mom')

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
            self._restore(tf_bundle.read_bundle(path))
            last_saving_step = int(path[path.rindex('-') + 1:])
        opath = _latest(self.optimizer_checkpoint_folder)
        if opath is not None:
            logging.info('Restoring optimizer variables from previous run')
            self._restore(tf_bundle.read_bundle(opath))
        self.last_saving_step = last_saving_step
        return last_saving_step

    def get_lr(self):
        if self.global_step <= self.lr_annealing_steps:
            return self.initial_lr - (self.global_step * self.initial_lr / self.lr_annealing_steps)
        return 0.0

    def cleanup(self):
        self.save_vars(True)
