"""Load / wait / barrier skeleton of a kernel in the built HIP library (CPU only, no GPU needed).

    python tools/isa_loads.py <kernel-name-substring> [--lib manette_amd/libmanette_hip.so] [--full]

Finds the gfx950 code objects inside the library's .hip_fatbin section (one offload bundle per
translation unit), disassembles the first kernel whose mangled name contains the substring and
prints its memory skeleton: runs of global loads / stores, s_waitcnt vmcnt, s_barrier and MFMA
issues, with their line numbers. What to look for (round 3, DESIGN.md "Next"): read-only operand
loads the source issues at kernel start but that the compiler sank to their first use — a global
load right after an s_barrier and followed by a vmcnt wait is one more memory round trip on the
block's critical path (fix: relaxed agent-scope atomic loads, or batch them in registers).
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = '/opt/rocm/lib/llvm/bin'
BUNDLER = '/opt/rocm/llvm/bin/clang-offload-bundler'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'
TARGET = 'hipv4-amdgcn-amd-amdhsa--gfx950'


def code_objects(lib, tmp):
    fat = os.path.join(tmp, 'fat.bin')
    subprocess.check_call([os.path.join(LLVM, 'llvm-objcopy'), '--dump-section=.hip_fatbin=' + fat, lib])
    data = open(fat, 'rb').read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for i, s in enumerate(starts):
        part = os.path.join(tmp, 'b%d.bin' % i)
        with open(part, 'wb') as f:
            f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(tmp, 'b%d.co' % i)
        r = subprocess.run([BUNDLER, '--unbundle', '--type=o', '--input=' + part, '--targets=' + TARGET,
                            '--output=' + co], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def kernels(co):
    txt = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '-s', '--wide', co], capture_output=True,
                         text=True).stdout
    names = []
    for line in txt.splitlines():
        p = line.split()
        if len(p) >= 8 and p[3] == 'FUNC' and not p[7].endswith('.kd'):
            names.append(p[7])
    return names


KEEP = re.compile(r'(global_load\w*|global_store\w*|global_atomic\w*|buffer_load\w*|flat_load\w*|s_waitcnt vmcnt\(\d+\)|'
                  r's_barrier|v_mfma\w*|s_endpgm|ds_read\w*|ds_write\w*)')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('name')
    ap.add_argument('--lib', default=os.path.join(ROOT, 'manette_amd', 'libmanette_hip.so'))
    ap.add_argument('--full', action='store_true', help='print every matching instruction, not runs')
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(a.lib, tmp):
            hit = [k for k in kernels(co) if a.name in k]
            if not hit:
                continue
            sym = hit[0]
            print('kernel:', sym[:200], '(%d matches)' % len(hit))
            dis = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--disassemble-symbols=' + sym, co],
                                 capture_output=True, text=True).stdout.splitlines()
            prev, count, first = None, 0, 0
            for n, line in enumerate(dis):
                m = KEEP.search(line.split('//')[0])
                if not m:
                    continue
                op = m.group(1) if a.full else m.group(1).split(' ')[0]
                if a.full:
                    print('%6d  %s' % (n, line.split('//')[0].strip()))
                    continue
                if op == prev:
                    count += 1
                    continue
                if prev is not None:
                    print('%6d  %3d x %s' % (first, count, prev))
                prev, count, first = op, 1, n
            if prev is not None:
                print('%6d  %3d x %s' % (first, count, prev))
            return 0
    print('no kernel matching %r in %s' % (a.name, a.lib))
    return 1


if __name__ == '__main__':
    sys.exit(main())
