"""Build the native libraries in-tree (no JIT cache, so the .so files travel with the repo).

  libmanette_hip.so        hipcc --offload-arch=gfx950: HIP kernels + C ABI (include/manette_hip.h)
  libmanette_hip_probe.so  the same with -DMT_PROBE: in-kernel phase timestamps (mt_probe_read,
                           tools/probe.py; tests/test_probe_gpu.py) — the one instrumentation build
  libmanette_host.so       g++: native emulator runner + bookkeeping (include/manette_host.h)
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
HIP_SOURCES = ['net.hip', 'misc.hip', 'rollout.hip', 'comm.hip']
HIP_HEADERS = ['common.h', 'gemm.h', 'jobs.h', 'nips_bwd.h', 'trunk_fused.h', 'lstm.h', 'dconv.h', 'nature_bwd.h']
HOST_SOURCES = ['runner.cpp', 'crc32c.cpp']
HIP_LIB = os.path.join(HERE, 'libmanette_hip.so')
PROBE_LIB = os.path.join(HERE, 'libmanette_hip_probe.so')
HOST_LIB = os.path.join(HERE, 'libmanette_host.so')
INCLUDE = os.path.join(os.path.dirname(HERE), 'include')


def _hipcc():
    for c in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', shutil.which('hipcc')):
        if c and os.path.exists(c):
            return c
    raise RuntimeError('hipcc not found')


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_hip(force=False, verbose=False, out=None, defines=()):
    """out / defines: a variant (the probe build: -DMT_PROBE) written next to the product library;
    select it at run time with MANETTE_HIP_LIB (manette_amd/_lib.py)."""
    target = out or HIP_LIB
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HIP_HEADERS] + [os.path.join(INCLUDE, 'manette_hip.h'),
                                                                  os.path.join(INCLUDE, 'manette_host.h'), HOST_LIB]
    if not force and not _stale(target, deps):
        return target
    # one hipcc per translation unit, in parallel (net.hip alone takes most of a serial build), then
    # one link; objects go to a private temporary directory (removed whatever happens), so a failed
    # compile leaves nothing stale and concurrent builds do not clobber each other's objects
    import concurrent.futures as cf
    import tempfile
    flags = ['--offload-arch=gfx950', '-O3', '-fPIC', '-std=c++17', '-Wno-unused-result'] + ['-D' + d for d in defines]
    jobs = int(os.environ.get('MT_BUILD_JOBS', '4'))
    tmpdir = tempfile.mkdtemp(prefix='manette_build_')
    try:
        objs = [os.path.join(tmpdir, os.path.basename(src) + '.o') for src in srcs]

        def compile_one(src, obj):
            cmd = [_hipcc()] + flags + ['-c', src, '-o', obj]
            if verbose:
                print(' '.join(cmd))
            subprocess.check_call(cmd, cwd=CSRC)

        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for f in [ex.submit(compile_one, src, obj) for src, obj in zip(srcs, objs)]:
                f.result()
        tmp = os.path.join(tmpdir, os.path.basename(target))
        cmd = [_hipcc(), '--offload-arch=gfx950', '-shared', '-fPIC', '-o', tmp] + objs + [
            '-L' + HERE, '-lmanette_host', '-Wl,-rpath,$ORIGIN', '-L/opt/rocm/lib', '-lrccl',
            '-Wl,-rpath,/opt/rocm/lib']
        if verbose:
            print(' '.join(cmd))
        subprocess.check_call(cmd, cwd=CSRC)
        shutil.move(tmp, target + '.tmp')
        os.replace(target + '.tmp', target)
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    return target


def build_host(force=False, verbose=False):
    srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES]
    deps = srcs + [os.path.join(INCLUDE, 'manette_host.h')]
    if not force and not _stale(HOST_LIB, deps):
        return HOST_LIB
    tmp = HOST_LIB + '.tmp'
    cmd = ['g++', '-O3', '-march=x86-64-v2', '-fPIC', '-shared', '-std=c++20', '-pthread', '-Wall',
           '-o', tmp] + srcs
    if verbose:
        print(' '.join(cmd))
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build_all(force=False, verbose=False):
    build_host(force, verbose)
    build_hip(force, verbose)
    build_hip(force, verbose, out=PROBE_LIB, defines=('MT_PROBE',))


if __name__ == '__main__':
    build_all(force='--force' in sys.argv, verbose=True)
