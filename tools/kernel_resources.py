"""VGPR / SGPR / scratch / LDS of kernels in the built HIP library (CPU only): the code objects'
AMDGPU metadata notes, filtered by a kernel-name substring.

    python tools/kernel_resources.py nature_chain_kernel [--lib manette_amd/libmanette_hip.so]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_loads import code_objects, LLVM, ROOT  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('name')
    ap.add_argument('--lib', default=os.path.join(ROOT, 'manette_amd', 'libmanette_hip.so'))
    a = ap.parse_args()
    keys = ('.name:', '.vgpr_count', '.agpr_count', '.sgpr_count', '.private_segment_fixed_size',
            '.group_segment_fixed_size', '.vgpr_spill_count', '.sgpr_spill_count')
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(a.lib, tmp):
            txt = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '--notes', co], capture_output=True,
                                 text=True).stdout
            for blk in re.split(r'\n\s+- \.', txt):
                if a.name in blk:
                    vals = {k: re.search(re.escape(k.strip('.:')) + r':\s*(\S+)', blk) for k in keys}
                    print(' '.join('%s=%s' % (k.strip('.:'), v.group(1)) for k, v in vals.items() if v))


if __name__ == '__main__':
    main()
