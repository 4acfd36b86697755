"""Optimizer restatement (oracle): clip_by_global_norm + TF1 ApplyRMSProp + LR schedule.

actor_learner.py:43-74 builds RMSPropOptimizer(lr, decay=--alpha, epsilon=--e) (momentum 0,
rms slot initialised to ONES — both pinned by tests/golden/meta_graph.json) and
clip_by_global_norm(grads, --clip_norm). TF1's ApplyRMSProp functor (training_ops):
    ms  += (grad^2 - ms) * (1 - rho)
    mom  = mom * momentum + (grad * lr) / sqrt(ms + epsilon)
    var -= mom
Everything here is float32 with TF's operation order so the elementwise update can be compared
bit-for-bit; only the global norm's summation order differs from any parallel reduction.
"""
import numpy as np


def global_norm(grads):
    """sqrt(sum_i 2 * L2Loss(g_i)) (clip_ops.global_norm), accumulated in float64."""
    return float(np.sqrt(sum(float(np.sum(np.asarray(g, np.float64) ** 2)) for g in grads)))


def clip_scale(norm, clip):
    """clip_by_global_norm: clip * min(1/norm, 1/clip), both factors float32."""
    norm = np.float32(norm)
    with np.errstate(divide='ignore'):
        inv = np.float32(1.0) / norm
    return np.float32(np.float32(clip) * np.minimum(inv, np.float32(1.0 / clip)))


def rmsprop_apply(w, ms, mom, g, lr, decay=0.99, momentum=0.0, eps=0.1):
    """In place, float32, TF1 ApplyRMSProp order of operations."""
    f = np.float32
    g = g.astype(f)
    ms += (g * g - ms) * (f(1.0) - f(decay))
    mom[...] = mom * f(momentum) + (g * f(lr)) / np.sqrt(ms + f(eps))
    w -= mom


def get_lr(global_step, initial_lr, lr_annealing_steps):
    """actor_learner.py:132-136."""
    if global_step <= lr_annealing_steps:
        return initial_lr - (global_step * initial_lr / lr_annealing_steps)
    return 0.0


def rescale_reward(reward):
    """actor_learner.py:108-114."""
    if reward > 1.0:
        reward = 1.0
    elif reward < -1.0:
        reward = -1.0
    return reward
