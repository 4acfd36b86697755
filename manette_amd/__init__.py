"""manette_amd — MI355X-native PAAC+FiGAR rollout/update hot path.

Host side mirrors the reference's PAACLearner / runners / exploration-policy interfaces; the
device side is libmanette_hip.so (hand-written gfx950 HIP kernels behind a C ABI,
include/manette_hip.h) and the emulator runner is libmanette_host.so (include/manette_host.h).
"""
__version__ = '0.1.0'
