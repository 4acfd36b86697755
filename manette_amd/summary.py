"""TensorBoard scalars of the reference learner as TF event files.

The reference opens tf.summary.FileWriter(<df>/tf) (actor_learner.py:82) and writes:
  * step 0: the args.json text (paac.py:23-31, tf.summary.text('text', ...));
  * per finished episode, at the global step the env's step took it to: rl/reward and
    rl/episode_length (paac.py:191-199);
  * after every update, when more than 50 episodes are done and global_step % 500 == 0:
    <tag>/{mean,min,max,std,std_over_mean} of the last 50 episodes, for rewards_per_episode and
    steps_per_episode (paac.py:65-77, :265-266).
(The histogram / stats / parameter summaries are built but never written by the reference.)

Written without TensorFlow: a TFRecord stream (uint64 length, masked CRC32C of the length,
payload, masked CRC32C of the payload — the CRC32C is libmanette_host's mh_crc32c) of Event
protos encoded by hand: Event{wall_time=1 double, step=2 int64, file_version=3 string,
summary=5}, Summary{value=1}, Summary.Value{tag=1, simple_value=2 float, tensor=8,
metadata=9}. read_events() parses the files back (tests).
"""
import os
import socket
import struct
import time

import numpy as np

from .tf_bundle import _pb_bytes_field, _pb_fields, _pb_varint_field, _put_varint, crc32c, mask


def _double_field(f, v):
    return _put_varint((f << 3) | 1) + struct.pack('<d', float(v))


def _float_field(f, v):
    return _put_varint((f << 3) | 5) + struct.pack('<f', float(v))


def _scalar_value(tag, value):
    return _pb_bytes_field(1, tag.encode()) + _float_field(2, value)


def _text_value(tag, text):
    # TensorProto{dtype=1: DT_STRING (7), tensor_shape=2: {}, string_val=8}; plugin "text"
    tensor = _pb_varint_field(1, 7) + _pb_bytes_field(2, b'') + _pb_bytes_field(8, text.encode())
    meta = _pb_bytes_field(1, _pb_bytes_field(1, b'text'))
    return _pb_bytes_field(1, tag.encode()) + _pb_bytes_field(9, meta) + _pb_bytes_field(8, tensor)


class EventWriter(object):
    """tf.summary.FileWriter's on-disk format: events.out.tfevents.<time>.<host> in `logdir`."""

    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, 'events.out.tfevents.%d.%s' % (int(time.time()), socket.gethostname()))
        self._f = open(self.path, 'wb')
        self._write(_double_field(1, time.time()) + _pb_bytes_field(3, b'brain.Event:2'))

    def _write(self, event):
        n = struct.pack('<Q', len(event))
        self._f.write(n + struct.pack('<I', mask(crc32c(n))) + event + struct.pack('<I', mask(crc32c(event))))

    def add_values(self, step, values):
        """values: serialized Summary.Value messages, written as one Event at `step`."""
        summ = b''.join(_pb_bytes_field(1, v) for v in values)
        self._write(_double_field(1, time.time()) + _pb_varint_field(2, int(step)) + _pb_bytes_field(5, summ))

    def add_scalars(self, step, pairs):
        self.add_values(step, [_scalar_value(t, v) for t, v in pairs])

    def add_text(self, step, tag, text):
        self.add_values(step, [_text_value(tag, text)])

    def flush(self):
        self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


class LearnerSummaries(object):
    """The reference's summary calls (paac.py:23-31, :65-77, :191-199, :265-266) on an EventWriter."""

    def __init__(self, debugging_folder):
        self.writer = EventWriter(os.path.join(debugging_folder, 'tf'))
        args = os.path.join(debugging_folder, 'args.json')
        if os.path.exists(args):
            self.writer.add_text(0, 'text', open(args).read())
        self.writer.flush()

    def episodes(self, records):
        """records: (global_step, total reward, emulator steps) per finished episode (book.episodes)."""
        for step, reward, length in records:
            self.writer.add_scalars(step, [('rl/reward', reward), ('rl/episode_length', length)])

    def log_values(self, values, tag, global_step, length=50, timestep=500):
        """paac.py:65-77."""
        if len(values) > length and global_step % timestep == 0:
            last = values[-50:]
            mean = np.mean(last)
            std = np.std(last)
            with np.errstate(divide='ignore', invalid='ignore'):
                ratio = min(2, np.absolute(std / mean))
            self.writer.add_scalars(global_step, [(tag + '/mean', mean), (tag + '/min', min(last)),
                                                  (tag + '/max', max(last)), (tag + '/std', std),
                                                  (tag + '/std_over_mean', ratio)])

    def flush(self):
        self.writer.flush()

    def close(self):
        self.writer.close()


def read_events(path):
    """Parse a TF event file: [(wall_time, step, {tag: value or text})], checking every CRC."""
    data = open(path, 'rb').read()
    out, i = [], 0
    while i < len(data):
        n = struct.unpack_from('<Q', data, i)[0]
        if struct.unpack_from('<I', data, i + 8)[0] != mask(crc32c(data[i:i + 8])):
            raise ValueError('length crc at %d' % i)
        ev = data[i + 12:i + 12 + n]
        if struct.unpack_from('<I', data, i + 12 + n)[0] != mask(crc32c(ev)):
            raise ValueError('data crc at %d' % i)
        i += 16 + n
        wall, step, vals = None, 0, {}
        for f, wt, v in _pb_fields(ev):
            if f == 1:
                wall = struct.unpack('<d', struct.pack('<Q', v))[0]
            elif f == 2:
                step = v
            elif f == 3:
                vals['file_version'] = bytes(v).decode()
            elif f == 5:
                for f2, _, val in _pb_fields(v):
                    if f2 != 1:
                        continue
                    tag, x = None, None
                    for f3, _, u in _pb_fields(val):
                        if f3 == 1:
                            tag = bytes(u).decode()
                        elif f3 == 2:
                            x = struct.unpack('<f', struct.pack('<I', u))[0]
                        elif f3 == 8:
                            x = b''.join(bytes(s) for g, _, s in _pb_fields(u) if g == 8).decode()
                    vals[tag] = x
        out.append((wall, step, vals))
    return out

