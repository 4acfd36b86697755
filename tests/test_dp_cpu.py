"""World-size-2 gloo test of the data-parallel update protocol on CPU: sum-all-reduce of the flat
gradient, 1/world scale, global-norm clip on the averaged gradient, replicated RMSProp ==
the single-process update on the union batch (and both replicas identical)."""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def test_dp_protocol_two_ranks_gloo(tmp_path):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT='29541', WORLD_SIZE='2')
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, 'dp_worker.py'), str(tmp_path), 'cpu'],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, o[-2000:] + e[-3000:]
    w0 = np.load(os.path.join(str(tmp_path), 'cpu_rank0.npy'))
    w1 = np.load(os.path.join(str(tmp_path), 'cpu_rank1.npy'))
    np.testing.assert_array_equal(w0, w1)  # replicas stay identical
    import dp_worker
    spec, P, obs, a, r, y, adv = dp_worker.cpu_batch()
    ref = dp_worker.dp_update(spec, P, obs, a, r, y, adv, world=1, rank=0)
    # equal to the single-process update within fp32 rounding of the reduction order
    np.testing.assert_allclose(w0, ref, rtol=0, atol=2e-6)
