"""The instrumentation build (libmanette_hip_probe.so, -DMT_PROBE: in-kernel phase timestamps) is
the one compile-time variant of the HIP library; it must build (manette_amd/build.py build_all) and
run the benchmarked rollout + update, so the probes tools/probe.py reads stay trustworthy."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_probe_build_runs_the_rollout_chain():
    lib = os.path.join(ROOT, 'manette_amd', 'libmanette_hip_probe.so')
    assert os.path.exists(lib), 'probe build missing: run __graft_entry__.build()'
    env = dict(os.environ, MANETTE_HIP_LIB=lib)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'probe.py'), '--updates', '3'], env=env,
                         cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = out.stdout.splitlines()
    # every kernel of the chain recorded its blocks' phases (conv: 9 blocks per env)
    for name, blocks in (('conv', 9 * 32), ('fc', 16 * 8 * 2), ('heads', 32)):  # (fc: 8 K-splits x 16-env tiles)
        hit = [ln for ln in lines if ln.startswith(name + ' ') and 'blocks' in ln]
        assert hit and int(hit[0].split()[2]) == blocks, (name, lines)
