"""Environment factory: environment_creator.py:4-30 interface.

ALE (ale_python_interface) is not installed in this image, so Atari games are served by the
synthetic stand-in with the game's ALE minimal-action-set size (what environment_creator.py:28
reads from the ROM; sizes below are ALE's minimal action sets, cross-checked where the
reference's pretrained checkpoints pin a head width). If ale_python_interface becomes
importable, an ALE-backed emulator can be plugged in behind the same create_environment().
"""
from .synthetic import SyntheticBank, SyntheticEmulator

MINIMAL_ACTIONS = {
    'pong': 6, 'breakout': 4, 'seaquest': 18, 'ms_pacman': 9, 'space_invaders': 6, 'beam_rider': 9,
    'qbert': 6, 'enduro': 9, 'asterix': 9, 'alien': 18, 'amidar': 10, 'assault': 7, 'asteroids': 14,
    'atlantis': 4, 'bank_heist': 18, 'battle_zone': 18, 'boxing': 18, 'centipede': 18,
    'chopper_command': 18, 'crazy_climber': 9, 'demon_attack': 6, 'freeway': 3, 'frostbite': 18,
    'gopher': 8, 'gravitar': 18, 'hero': 18, 'kangaroo': 18, 'krull': 18, 'montezuma_revenge': 18,
    'private_eye': 18, 'riverraid': 18, 'road_runner': 18, 'robotank': 18, 'star_gunner': 18,
    'time_pilot': 10, 'tutankham': 8, 'up_n_down': 6, 'venture': 18, 'video_pinball': 9,
    'wizard_of_wor': 10, 'zaxxon': 18,
}


class EnvironmentCreator(object):
    def __init__(self, args):
        game = args.game.lower()
        if game == 'tetris' or game.endswith('-v0'):
            raise NotImplementedError('gym / tetris emulators are out of scope (SURVEY.md §2)')
        self.num_actions = MINIMAL_ACTIONS.get(game, 18)
        self.rgb = bool(getattr(args, 'rgb', False))
        self.rank_offset = int(getattr(args, 'env_id_offset', 0))
        self.create_environment = lambda i: SyntheticEmulator(self.rank_offset + i, self.num_actions,
                                                              rgb=self.rgb)

    def create_bank(self, first_local, n_envs):
        """Native bank of envs [first_local, first_local+n) (global ids offset by rank)."""
        return SyntheticBank(self.rank_offset + first_local, n_envs, rgb=self.rgb)
