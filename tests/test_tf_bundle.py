"""TF tensor-bundle checkpoints (manette_amd/tf_bundle.py) against the reference's own
pretrained checkpoint indices (tests/golden/pretrained/<game>/checkpoints/*.index, copied data
files of the reference; their .data shards and TF itself are absent). CPU only.

Pins: CRC32C known answers (incl. the masked CRC the reference index stores for an all-zero
4-byte tensor); every reference .index decodes with valid block checksums and re-encodes
BYTE-IDENTICALLY from its decoded entries (SSTable layout, restart interval, index separator,
footer, BundleHeader/EntryProto field encoding); the variable names and shapes each reference
checkpoint holds are exactly this build's parameter layout for that run's args.json plus the
two RMSProp slots per variable; write -> read round trip."""
import glob
import json
import os

import numpy as np
import pytest

from manette_amd import tf_bundle

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = sorted(glob.glob(os.path.join(HERE, 'golden', 'pretrained', '*', 'checkpoints', '*.index')))


def test_crc32c_known_answers():
    assert tf_bundle.crc32c(b'123456789') == 0xE3069283
    assert tf_bundle.crc32c(b'\x00' * 32) == 0x8A9136AA
    rs = np.random.RandomState(0)
    for n in (0, 1, 7, 8, 9, 1000, 4097):
        b = rs.bytes(n)
        assert tf_bundle.crc32c(b) == tf_bundle.crc32c_py(b)
    # Training/Repetition/.../repetition_output_biases/OptimizerVariables_1 of catcher (R = 1:
    # its momentum slot stays zero) stores the masked CRC of 4 zero bytes
    _, e = tf_bundle.read_index(os.path.join(HERE, 'golden', 'pretrained', 'catcher', 'checkpoints', '-5532928'))
    z = e['Training/Repetition/repetition_output/repetition_output_biases/OptimizerVariables_1']
    assert z['size'] == 4 and z['crc32c'] == tf_bundle.mask(tf_bundle.crc32c(b'\x00' * 4))


@pytest.mark.parametrize('path', FIX, ids=[p.split(os.sep)[-3] for p in FIX])
def test_reference_index_reencodes_byte_identical(path, tmp_path):
    assert len(FIX) == 8
    items = tf_bundle.read_table(path)  # checks every block's masked CRC32C
    assert items[0][0] == b'' and items[0][1] == tf_bundle.encode_header()
    _, entries = tf_bundle.read_index(path[:-len('.index')])
    out = str(tmp_path / 'x.index')
    tf_bundle.write_index_entries(out, entries)
    assert open(out, 'rb').read() == open(path, 'rb').read()
    # the data shard layout: tensors back to back in key order
    off = 0
    for name in sorted(entries):
        e = entries[name]
        assert e['offset'] == off and e['dtype'] == 1 and e['size'] == 4 * int(np.prod(e['shape']))
        off += e['size']


@pytest.mark.parametrize('path', FIX, ids=[p.split(os.sep)[-3] for p in FIX])
def test_reference_checkpoint_matches_layout(path):
    import ctypes as C
    from manette_amd import _lib
    from manette_amd.environment_creator import MINIMAL_ACTIONS
    run = os.path.dirname(os.path.dirname(path))
    args = json.load(open(os.path.join(run, 'args.json')))
    _, entries = tf_bundle.read_index(path[:-len('.index')])
    A = entries['Training/Actor/actor_output/actor_output_biases']['shape'][0]
    R = entries['Training/Repetition/repetition_output/repetition_output_biases']['shape'][0]
    assert R == args['nb_choices']
    if args['game'] in MINIMAL_ACTIONS:  # ALE games: the minimal action set of environment_creator
        assert A == MINIMAL_ACTIONS[args['game']]
    depth = 3 if args['rgb'] else 1
    cfg = _lib.mt_net_config(_lib.MT_ARCH[args['arch']], depth, A, R, 0, 0.1, 1.0)
    lib = _lib.hip()
    h = C.c_void_p()
    _lib.check(lib.mt_net_create(C.byref(cfg), C.byref(h)))
    try:
        nv = C.c_int()
        lib.mt_net_num_vars(h, C.byref(nv))
        want = {}
        for i in range(nv.value):
            buf = C.create_string_buffer(256)
            sh = (C.c_int64 * 4)()
            nd = C.c_int()
            _lib.check(lib.mt_net_var_info(h, i, buf, 256, sh, C.byref(nd), None, None))
            shape = tuple(sh[k] for k in range(nd.value))
            for suffix in ('', '/OptimizerVariables', '/OptimizerVariables_1'):
                want[buf.value.decode() + suffix] = shape
    finally:
        lib.mt_net_destroy(h)
    assert {k: v['shape'] for k, v in entries.items()} == want


def test_bundle_round_trip(tmp_path):
    rs = np.random.RandomState(1)
    t = {'Network/conv1/conv1_weights': rs.randn(8, 8, 4, 16).astype(np.float32),
         'Network/conv1/conv1_biases': rs.randn(16).astype(np.float32),
         'a/scalar_like': np.zeros((1,), np.float32),
         'big': rs.randn(300000).astype(np.float32)}
    pre = str(tmp_path / '-42')
    tf_bundle.write_bundle(pre, t)
    back = tf_bundle.read_bundle(pre)
    assert set(back) == set(t)
    for k in t:
        np.testing.assert_array_equal(back[k], t[k])
    # a corrupted tensor is detected
    data = bytearray(open(pre + '.data-00000-of-00001', 'rb').read())
    data[5] ^= 1
    open(pre + '.data-00000-of-00001', 'wb').write(bytes(data))
    with pytest.raises(ValueError):
        tf_bundle.read_bundle(pre)
