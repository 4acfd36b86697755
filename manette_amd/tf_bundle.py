"""TensorFlow tensor-bundle (V2) checkpoints, read and written without TensorFlow.

The reference saves with tf.train.Saver (networks.py:162-175, actor_learner.py save_vars):
`<folder>/checkpoints/-<global_step>.index` + `.data-00000-of-00001` and a `checkpoint` text
file naming the latest prefix. Format (TF 1.x, tensorflow/core/util/tensor_bundle and
core/lib/io/table):
  * .index is an SSTable (LevelDB table layout): data blocks of prefix-compressed entries with a
    restart array, each block followed by a 1-byte compression type (0 = none) and a masked
    CRC32C; a metaindex block (empty), an index block (one entry per data block: a separator
    key >= the block's last key -> BlockHandle), and a 48-byte footer (two BlockHandles padded
    to 40 bytes + magic 0xdb4775248b80fb57).
  * keys: "" -> BundleHeaderProto {num_shards=1, endianness=LITTLE, version{producer=1}};
    every tensor name -> BundleEntryProto {dtype, shape, shard_id, offset, size, crc32c}.
  * .data-00000-of-00001 holds the raw little-endian tensor bytes back to back; crc32c is the
    masked CRC32C of a tensor's bytes.
Pinned by tests/test_tf_bundle.py against the reference's own pretrained/*/checkpoints/*.index
files (committed as fixtures): decoding, and byte-identical re-encoding of the same entries.
"""
import os
import struct

import numpy as np

MAGIC = 0xdb4775248b80fb57
BLOCK_SIZE = 262144        # table::Options default (TF)
RESTART_INTERVAL = 16      # table::Options default (TF)
DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64}
DT_OF = {np.dtype(v): k for k, v in DT.items()}

# ---- CRC32C (Castagnoli), masked as LevelDB/TF do ---------------------------------------------
_T = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _T.append(_c)
_T = np.array(_T, dtype=np.uint32)


def crc32c(data):
    """CRC32C through libmanette_host.so (SSE4.2 crc32, include/manette_host.h mh_crc32c)."""
    import ctypes as C
    from . import _lib
    b = data if isinstance(data, (bytes, bytearray)) else bytes(data)
    buf = (C.c_char * len(b)).from_buffer_copy(b) if len(b) else None
    return int(_lib.host().mh_crc32c(buf, len(b), 0))


def crc32c_py(data, crc=0):
    """Table-driven restatement (tests pin the native one against it)."""
    c = (~crc) & 0xffffffff
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    for x in b.tolist():
        c = int(_T[(c ^ x) & 0xff]) ^ (c >> 8)
    return (~c) & 0xffffffff


def mask(crc):
    return ((((crc >> 15) | (crc << 17)) & 0xffffffff) + 0xa282ead8) & 0xffffffff


def unmask(m):
    r = (m - 0xa282ead8) & 0xffffffff
    return ((r >> 17) | (r << 15)) & 0xffffffff


# ---- varints / protobuf ------------------------------------------------------------------------
def _put_varint(n):
    out = bytearray()
    while True:
        b = n & 0x7f
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _get_varint(b, i):
    shift = n = 0
    while True:
        x = b[i]
        i += 1
        n |= (x & 0x7f) << shift
        if not x & 0x80:
            return n, i
        shift += 7


def _pb_fields(b):
    i, out = 0, []
    while i < len(b):
        key, i = _get_varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _get_varint(b, i)
        elif wt == 2:
            n, i = _get_varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = struct.unpack_from('<I', b, i)[0]
            i += 4
        elif wt == 1:
            v = struct.unpack_from('<Q', b, i)[0]
            i += 8
        else:
            raise ValueError('wire type %d' % wt)
        out.append((f, wt, v))
    return out


def _pb_varint_field(f, v):
    return _put_varint(f << 3) + _put_varint(v)


def _pb_bytes_field(f, v):
    return _put_varint((f << 3) | 2) + _put_varint(len(v)) + v


def _pb_fixed32_field(f, v):
    return _put_varint((f << 3) | 5) + struct.pack('<I', v)


def decode_entry(b):
    e = dict(dtype=1, shape=(), shard_id=0, offset=0, size=0, crc32c=0)
    for f, wt, v in _pb_fields(b):
        if f == 1:
            e['dtype'] = v
        elif f == 2:
            dims = []
            for g, _, dv in _pb_fields(v):
                if g == 2:
                    size = 0
                    for h, _, sv in _pb_fields(dv):
                        if h == 1:
                            size = sv
                    dims.append(size)
            e['shape'] = tuple(dims)
        elif f == 3:
            e['shard_id'] = v
        elif f == 4:
            e['offset'] = v
        elif f == 5:
            e['size'] = v
        elif f == 6:
            e['crc32c'] = v
    return e


def encode_entry(e):
    """BundleEntryProto in field order, default (zero) fields omitted as proto3 serialises."""
    out = b''
    if e['dtype']:
        out += _pb_varint_field(1, e['dtype'])
    shape = b''.join(_pb_bytes_field(2, _pb_varint_field(1, d) if d else b'') for d in e['shape'])
    out += _pb_bytes_field(2, shape)
    if e.get('shard_id', 0):
        out += _pb_varint_field(3, e['shard_id'])
    if e['offset']:
        out += _pb_varint_field(4, e['offset'])
    if e['size']:
        out += _pb_varint_field(5, e['size'])
    out += _pb_fixed32_field(6, e['crc32c'])
    return out


def encode_header(num_shards=1, producer=1):
    return _pb_varint_field(1, num_shards) + _pb_bytes_field(3, _pb_varint_field(1, producer))


# ---- SSTable -----------------------------------------------------------------------------------
def _read_block(buf, off, size, check=True):
    data = buf[off:off + size]
    ctype = buf[off + size]
    if ctype != 0:
        raise ValueError('compressed SSTable blocks are not supported')
    if check:
        want = unmask(struct.unpack_from('<I', buf, off + size + 1)[0])
        if crc32c(buf[off:off + size + 1]) != want:
            raise ValueError('SSTable block checksum mismatch at %d' % off)
    nrest = struct.unpack_from('<I', data, len(data) - 4)[0]
    end = len(data) - 4 - 4 * nrest
    items, i, key = [], 0, b''
    while i < end:
        shared, i = _get_varint(data, i)
        unshared, i = _get_varint(data, i)
        vlen, i = _get_varint(data, i)
        key = key[:shared] + data[i:i + unshared]
        i += unshared
        items.append((key, data[i:i + vlen]))
        i += vlen
    return items


def _handle(b, i=0):
    off, i = _get_varint(b, i)
    size, i = _get_varint(b, i)
    return off, size, i


def read_table(path, check=True):
    buf = open(path, 'rb').read()
    if struct.unpack_from('<Q', buf, len(buf) - 8)[0] != MAGIC:
        raise ValueError('%s: not an SSTable (bad magic)' % path)
    foot = buf[len(buf) - 48:]
    _, _, i = _handle(foot)
    ioff, isize, _ = _handle(foot, i)
    items = []
    for _, hv in _read_block(buf, ioff, isize, check):
        off, size, _ = _handle(hv)
        items.extend(_read_block(buf, off, size, check))
    return items


def _build_block(items):
    out, rest, prev = bytearray(), [], b''
    for n, (k, v) in enumerate(items):
        if n % RESTART_INTERVAL == 0:
            rest.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _put_varint(shared) + _put_varint(len(k) - shared) + _put_varint(len(v)) + k[shared:] + v
        prev = k
    if not rest:
        rest = [0]
    for r in rest:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(rest))
    return bytes(out)


def _short_successor(k):
    """BytewiseComparator::FindShortSuccessor."""
    for i, c in enumerate(k):
        if c != 0xff:
            return k[:i] + bytes([c + 1])
    return k


def _short_separator(a, b):
    """BytewiseComparator::FindShortestSeparator(a, limit=b)."""
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    if i < n:
        c = a[i]
        if c < 0xff and c + 1 < b[i]:
            return a[:i] + bytes([c + 1])
    return a


def write_table(path, items):
    """items: sorted (key bytes, value bytes)."""
    out = bytearray()
    index = []

    def emit(block):
        off = len(out)
        out.extend(block)
        trailer = b'\x00'
        out.extend(trailer + struct.pack('<I', mask(crc32c(block + trailer))))
        return off, len(block)

    cur, cur_bytes = [], 0
    pending = None  # (last key, handle) of the previous data block, its index key awaiting the next key
    for k, v in items:
        if pending is not None:
            index.append((_short_separator(pending[0], k), pending[1]))
            pending = None
        cur.append((k, v))
        cur_bytes += len(k) + len(v) + 8
        if cur_bytes >= BLOCK_SIZE:
            pending = (k, emit(_build_block(cur)))
            cur, cur_bytes = [], 0
    if cur:
        pending = (cur[-1][0], emit(_build_block(cur)))
    if pending is not None:
        index.append((_short_successor(pending[0]), pending[1]))
    meta = emit(_build_block([]))
    idx = emit(_build_block([(k, _put_varint(o) + _put_varint(s)) for k, (o, s) in index]))
    foot = _put_varint(meta[0]) + _put_varint(meta[1]) + _put_varint(idx[0]) + _put_varint(idx[1])
    foot += b'\x00' * (40 - len(foot)) + struct.pack('<Q', MAGIC)
    out.extend(foot)
    with open(path, 'wb') as f:
        f.write(out)


# ---- bundles -----------------------------------------------------------------------------------
def read_index(prefix):
    """-> (header fields, {name: entry})."""
    items = read_table(prefix + '.index')
    header, entries = None, {}
    for k, v in items:
        if k == b'':
            header = _pb_fields(v)
        else:
            entries[k.decode()] = decode_entry(v)
    return header, entries


def read_bundle(prefix):
    """{name: numpy array} (single shard)."""
    _, entries = read_index(prefix)
    data = open(prefix + '.data-00000-of-00001', 'rb').read()
    out = {}
    for name, e in entries.items():
        raw = data[e['offset']:e['offset'] + e['size']]
        if mask(crc32c(raw)) != e['crc32c']:
            raise ValueError('%s: tensor %s fails its crc32c' % (prefix, name))
        out[name] = np.frombuffer(raw, dtype=DT[e['dtype']]).reshape(e['shape']).copy()
    return out


def write_bundle(prefix, tensors):
    """tensors: {name: numpy array}; written in sorted-key order, as TF's BundleWriter does."""
    names = sorted(tensors)
    data = bytearray()
    items = [(b'', encode_header())]
    for name in names:
        a = np.ascontiguousarray(tensors[name])
        if a.dtype not in DT_OF:
            a = a.astype(np.float32)
        raw = a.tobytes()
        e = dict(dtype=DT_OF[a.dtype], shape=tuple(a.shape), offset=len(data), size=len(raw),
                 crc32c=mask(crc32c(raw)))
        data += raw
        items.append((name.encode(), encode_entry(e)))
    tmp = prefix + '.tmp'
    with open(tmp + '.data', 'wb') as f:
        f.write(data)
    write_table(tmp + '.index', items)
    os.replace(tmp + '.data', prefix + '.data-00000-of-00001')
    os.replace(tmp + '.index', prefix + '.index')


def write_index_entries(path, entries, header=None):
    """Re-encode a decoded index (tests: byte-identity with a TF-written .index)."""
    items = [(b'', header if header is not None else encode_header())]
    items += [(n.encode(), encode_entry(entries[n])) for n in sorted(entries)]
    write_table(path, items)
