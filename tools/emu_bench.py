"""Host-only microbenchmark of the native emulator runner (no GPU): us per macro-step.
  python tools/emu_bench.py E W [ring] [gap_us]
ring < 64: a shorter synthetic screen ring (all in cache); gap_us: host idle time between steps
(the GPU forward in the real pipeline), excluded from the reported time."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from manette_amd.synthetic import SyntheticBank  # noqa: E402
from manette_amd.runners import NativeRunners  # noqa: E402
from manette_amd.environment import ROW_LUT, COL_LUT  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 32
W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ring = int(sys.argv[3]) if len(sys.argv) > 3 else 64
gap = float(sys.argv[4]) * 1e-6 if len(sys.argv) > 4 else 0.0
bank = SyntheticBank(0, E, pinned=bool(int(os.environ.get("PINNED", "0"))))  # PINNED=1: hipHostMalloc bank (GPU box)
if ring < bank.screens.shape[1]:
    bank.screens = np.ascontiguousarray(bank.screens[:, :ring])
r = NativeRunners(bank, W, [0], row_select=ROW_LUT, fixed_slots=True, resized=True, col_lut=COL_LUT)
r.reset()
a = np.zeros(E, np.int32)
rr = np.zeros(E, np.int32)
for _ in range(50):
    r.step(a, rr)
n = 2000
busy = 0.0
# READY=1: per-env ready words (the pipelined rollout's mode: per-env publication, dynamic env dealing)
ready = np.zeros(E * 32, np.uint32) if os.environ.get('READY') == '1' else None
if ready is not None:
    import ctypes as C
    from manette_amd import _lib
for k in range(n):
    if ready is not None:
        _lib.check_host(_lib.host().mh_runner_set_ready(r._h, ready.ctypes.data_as(C.c_void_p), k + 1), 'ready')
    t = time.perf_counter()
    r.step(a, rr)
    t1 = time.perf_counter()
    busy += t1 - t
    while time.perf_counter() - t1 < gap:
        pass
print('E=%d W=%d ring=%d gap=%.0fus: %.2f us per step' % (E, W, ring, gap * 1e6, busy / n * 1e6))
r.stop()
