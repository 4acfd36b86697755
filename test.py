"""Evaluation CLI, the reference's test.py (test.py:29-116): same flags, reads the run's
args.json, restores the latest TF checkpoint of `<folder>/checkpoints` (TF tensor bundle,
manette_amd/tf_bundle.py) into the device network and plays `test_count` episodes with the
ExplorationPolicy(args, test=False) draw and FiGAR action repetition (Action), then prints the
reference's summary lines.

Differences, each a fix or a missing dependency:
  * test.py:110 calls update_memory for every arch (NameError unless LSTM): done for LSTM only;
  * an emulator whose episode ended is not stepped again (ALE gives no reward after game over,
    the synthetic stand-in would keep streaming rewards);
  * Atari games run on the synthetic emulators (ALE absent, environment_creator.py); gif output
    needs imageio (absent): -gn is accepted and reported as unavailable.
"""
import argparse
import logging
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def update_memory(memory, states):
    """test.py:20-23."""
    memory[:, :-1] = memory[:, 1:]
    memory[:, -1] = states
    return memory


def get_arg_parser():
    parser = argparse.ArgumentParser()
    parser.add_argument('-f', '--folder', type=str, help="Folder where to save the debugging information.",
                        dest="folder", required=True)
    parser.add_argument('-tc', '--test_count', default='1', type=int,
                        help="The amount of tests to run on the given network", dest="test_count")
    parser.add_argument('-np', '--noops', default=30, type=int, help="Maximum amount of no-ops to use",
                        dest="noops")
    parser.add_argument('-gn', '--gif_name', default=None, type=str,
                        help="If provided, a gif will be produced and stored with this name", dest="gif_name")
    parser.add_argument('-gf', '--gif_folder', default='', type=str, help="The folder where to save gifs.",
                        dest="gif_folder")
    parser.add_argument('-d', '--device', default='/gpu:0', type=str,
                        help="Device to be used ('/cpu:0', '/gpu:0', '/gpu:1',...)", dest="device")
    return parser


def run(args, max_macro_steps=None):
    """Returns the per-emulator episode rewards."""
    import torch
    import train as train_cli
    from manette_amd import logger_utils, tf_bundle
    from manette_amd.actor_learner import _latest, SLOT_MS, SLOT_MOM
    from manette_amd.exploration_policy import Action, ExplorationPolicy

    device = args.device
    for k, v in logger_utils.load_args(os.path.join(args.folder, 'args.json')).items():
        setattr(args, k, v)
    args.max_global_steps = 0
    df = args.folder
    args.debugging_folder = '/tmp/logs'
    args.device = device
    args.random_start = False
    args.single_life_episodes = False
    if args.gif_name:
        logging.warning('gif output needs imageio, which is not installed: -gn ignored')
    args.actor_id = 0
    rng = np.random.RandomState(int(time.time()))
    args.random_seed = rng.randint(1000)

    explo_policy = ExplorationPolicy(args, test=False)
    network_creator, env_creator = train_cli.get_network_and_environment_creator(args, explo_policy)
    network = network_creator()
    path = _latest(os.path.join(df, 'checkpoints'))
    if path is None:
        logging.info('Initializing all variables')
        network.init_params(0)
    else:
        logging.info('Restoring network variables from previous run')
        t = tf_bundle.read_bundle(path)
        network.set_variables({k: v for k, v in t.items() if not k.endswith((SLOT_MS, SLOT_MOM))})

    n = args.test_count
    environments = [env_creator.create_environment(i) for i in range(n)]
    states = np.asarray([e.get_initial_state() for e in environments])
    if args.noops != 0:
        for i, environment in enumerate(environments):
            for _ in range(random.randint(0, args.noops)):
                state, _, _ = environment.next(0)
                states[i] = state
    lstm = args.arch == 'LSTM'
    if lstm:
        memory = np.zeros([n, 5] + list(states.shape[1:]), dtype=np.uint8)
        memory[:, -1] = states
    episodes_over = np.zeros(n, dtype=bool)
    rewards = np.zeros(n, dtype=np.float32)
    steps = 0
    while not all(episodes_over):
        x = torch.from_numpy(np.ascontiguousarray(memory if lstm else states)).cuda()
        _, pi, rep = network.forward(x, n, ws_key='test', infer=True)
        actions, repetitions = explo_policy.choose_next_actions(pi.cpu().numpy(), rep.cpu().numpy(),
                                                                env_creator.num_actions)
        for j, environment in enumerate(environments):
            if episodes_over[j]:
                continue
            macro_action = Action(explo_policy.tab_rep, j, actions[j], repetitions[j])
            state, r, episode_over = environment.next(macro_action.current_action)
            states[j] = state
            rewards[j] += r
            episodes_over[j] = episode_over
            while macro_action.is_repeated() and not episode_over:
                state, r, episode_over = environment.next(macro_action.repeat())
                states[j] = state
                rewards[j] += r
                episodes_over[j] = episode_over
            macro_action.reset()
        if lstm:
            memory = update_memory(memory, states)
        steps += 1
        if max_macro_steps is not None and steps >= max_macro_steps:
            break
    print('Performed {} tests for {}.'.format(n, args.game))
    print('Mean: {0:.2f}'.format(np.mean(rewards)))
    print('Min: {0:.2f}'.format(np.min(rewards)))
    print('Max: {0:.2f}'.format(np.max(rewards)))
    print('Std: {0:.2f}'.format(np.std(rewards)))
    return rewards


if __name__ == '__main__':
    logging.basicConfig(level=logging.INFO)
    run(get_arg_parser().parse_args())
