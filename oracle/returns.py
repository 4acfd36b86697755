"""n-step return / advantage scan (oracle), paac.py:219-231 + flatten :237-238.

Kept literally in the reference's numpy form so the dtype trail is the reference's own:
`estimated_return` starts as the float32 bootstrap V(s_T); `gamma * estimated_return` is a
python float times a float32 array (float32 product under numpy promotion); the reward,
mask and value arrays are float64, so everything after runs in float64. Not GAE (no lambda).
"""
import numpy as np


def nstep_returns(rewards, masks, values, v_boot, gamma):
    """rewards/masks/values: (T, E) float64; v_boot: (E,) float32. Returns y, adv (T, E) f64."""
    T = rewards.shape[0]
    y_batch = np.zeros_like(rewards, dtype=np.float64)
    adv_batch = np.zeros_like(rewards, dtype=np.float64)
    estimated_return = np.copy(v_boot)
    for t in reversed(range(T)):
        estimated_return = rewards[t] + gamma * estimated_return * masks[t]
        y_batch[t] = np.copy(estimated_return)
        adv_batch[t] = estimated_return - values[t]
    return y_batch, adv_batch
