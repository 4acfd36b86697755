"""The C-ABI libraries load on a host without a GPU and export every declared symbol; the
network descriptor (layout, names, init bounds) matches the oracle's restatement. CPU only."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, 'include', header)).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = set(re.findall(r'\b(m[th]_[a-z0-9_]+)\s*\(', src))
    return names


def test_headers_match_bindings():
    from manette_amd import _lib
    assert _declared('manette_hip.h') == set(_lib.hip_symbols())
    assert _declared('manette_host.h') == set(_lib.host_symbols())


def test_libraries_export_every_symbol():
    from manette_amd import _lib
    hip = _lib.hip()
    host = _lib.host()
    for n in _declared('manette_hip.h'):
        assert hasattr(hip, n), n
    for n in _declared('manette_host.h'):
        assert hasattr(host, n), n
    assert hip.mt_version() >= 1


@pytest.mark.parametrize('arch,depth,A,R', [('NIPS', 1, 6, 1), ('NIPS', 3, 3, 11), ('NATURE', 1, 4, 11),
                                            ('NATURE', 3, 18, 1), ('PWYX', 1, 9, 11), ('PWYX', 3, 4, 11),
                                            ('LSTM', 1, 9, 11), ('LSTM', 3, 6, 1)])
def test_layout_matches_oracle(arch, depth, A, R):
    import ctypes as C
    from manette_amd import _lib
    from oracle import nets
    lib = _lib.hip()
    cfg = _lib.mt_net_config(_lib.MT_ARCH[arch], depth, A, R, 0, 0.1, 1.0)
    h = C.c_void_p()
    _lib.check(lib.mt_net_create(C.byref(cfg), C.byref(h)))
    try:
        nv = C.c_int()
        lib.mt_net_num_vars(h, C.byref(nv))
        spec = nets.arch_spec(arch, depth, A, R)
        assert nv.value == len(spec['vars'])
        prev_end = 0
        for i, (name, shape, bound) in enumerate(spec['vars']):
            buf = C.create_string_buffer(256)
            sh = (C.c_int64 * 4)()
            nd = C.c_int()
            off = C.c_size_t()
            b = C.c_float()
            _lib.check(lib.mt_net_var_info(h, i, buf, 256, sh, C.byref(nd), C.byref(off), C.byref(b)))
            assert buf.value.decode() == name
            assert tuple(sh[k] for k in range(nd.value)) == tuple(shape)
            assert np.float32(b.value) == np.float32(bound)
            assert off.value >= prev_end
            if i % 2 == 1:
                assert off.value == prev_end  # (weights, biases) contiguous
            else:
                assert off.value % 64 == 0
            prev_end = off.value + int(np.prod(shape))
        n = C.c_size_t()
        lib.mt_net_num_params(h, C.byref(n))
        assert n.value >= prev_end
        # SURVEY §8 parameter totals (checkpoint-consistent where a checkpoint exists)
        total = sum(int(np.prod(sh)) for _, sh, _ in spec['vars'])
        known = {('NIPS', 1, 6, 1): 678200, ('LSTM', 1, 9, 11): 930037}
        if (arch, depth, A, R) in known:
            assert total == known[(arch, depth, A, R)]
        ws = C.c_size_t()
        _lib.check(lib.mt_net_workspace_bytes(h, 160, C.byref(ws)))
        assert ws.value > 0
    finally:
        lib.mt_net_destroy(h)


def test_bad_config_reports_error():
    import ctypes as C
    from manette_amd import _lib
    lib = _lib.hip()
    cfg = _lib.mt_net_config(0, 2, 6, 1, 0, 0.1, 1.0)  # depth 2 is invalid
    h = C.c_void_p()
    rc = lib.mt_net_create(C.byref(cfg), C.byref(h))
    assert rc == 1 and b'depth' in lib.mt_last_error()
