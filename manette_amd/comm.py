"""Data-parallel communicators of the learner.

The reference has no collective: its only shard unit is the contiguous env split of
runners.py:17-18. This build shards envs over ranks the same way and exchanges one thing per
update, the flat fp32 gradient (sum all-reduce), plus rank 0's parameters / RMSProp slots at start.

RcclComm   the product path: an RCCL communicator behind the C ABI (mt_comm_*, manette_amd/csrc/
           comm.hip), called on the learner's stream, capturable into the update's hipGraph.
           torch.distributed (gloo) is only the control channel that ships rank 0's unique id.
TorchComm  torch.distributed collectives on the existing process group: for topologies RCCL does
           not support, i.e. several ranks sharing one GPU (the world-2 tests on a 1-GPU box).
LoopbackComm  the C-ABI communicator without RCCL (tests: x replicas + a delay, exposing stream order).
The C-ABI communicators (RcclComm, LoopbackComm) carry `_h`, the mt_comm handle the native rollout
launches the data-parallel update with (mt_rollout_set_update_dp).
"""
import ctypes as C
import os
import sys
import threading
import time

import torch

from . import _lib
from ._lib import check

# Bound on the communicator's setup and on the first update's all-reduce (seconds): RCCL's init and
# collectives block until every rank arrives, so a rank that never starts (or died) would hang the
# whole job; past this bound the process prints what it waited for and exits with status 3.
DEFAULT_TIMEOUT_S = 300.0


class Deadline(object):
    """Context manager: if the block has not finished within `seconds` (MT_COMM_TIMEOUT_S, default
    DEFAULT_TIMEOUT_S), a watchdog thread writes '<what> did not complete ...' to stderr and ends
    the process with os._exit(exit_code) — a blocked RCCL call cannot be interrupted from Python,
    and a non-zero exit is what the launcher (torch.distributed.run) turns into a failed job."""

    def __init__(self, what, rank=0, world=1, seconds=None, exit_code=3):
        self.what, self.rank, self.world, self.exit_code = what, rank, world, exit_code
        self.seconds = float(os.environ.get('MT_COMM_TIMEOUT_S', DEFAULT_TIMEOUT_S)) if seconds is None else seconds
        self._done = threading.Event()
        self._t = None

    def _watch(self):
        if not self._done.wait(self.seconds):
            sys.stderr.write('manette: %s did not complete within %.0f s on rank %d of %d (a rank never arrived '
                             'or died): exiting\n' % (self.what, self.seconds, self.rank, self.world))
            sys.stderr.flush()
            os._exit(self.exit_code)

    def __enter__(self):
        self._t0 = time.perf_counter()
        self._t = threading.Thread(target=self._watch, name='manette-deadline', daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._done.set()
        self._t.join()
        self.elapsed = time.perf_counter() - self._t0
        return False


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class RcclComm(object):
    capturable = True
    kind = 'rccl'

    def __init__(self, rank, world, device_index):
        import torch.distributed as dist
        lib = _lib.hip()
        uid = C.create_string_buffer(_lib.MT_COMM_UID_BYTES)
        if rank == 0:
            check(lib.mt_comm_unique_id(uid), 'mt_comm_unique_id')
        h = C.c_void_p()
        with Deadline('RCCL communicator setup (unique id exchange + mt_comm_init)', rank, world):
            if world > 1:
                box = [uid.raw if rank == 0 else None]
                dist.broadcast_object_list(box, src=0)
                C.memmove(uid, box[0], _lib.MT_COMM_UID_BYTES)
            check(lib.mt_comm_init(uid, int(rank), int(world), int(device_index), C.byref(h)), 'mt_comm_init')
        self._h = h
        self.rank, self.world = rank, world

    def allreduce(self, t):
        """In-place sum of a contiguous fp32 device tensor over the ranks (mt_allreduce)."""
        assert t.dtype == torch.float32 and t.is_cuda and t.is_contiguous()
        check(_lib.hip().mt_allreduce(self._h, C.c_void_p(t.data_ptr()), t.numel(), _stream()), 'mt_allreduce')

    def broadcast(self, t, root=0):
        assert t.is_cuda and t.is_contiguous()
        check(_lib.hip().mt_broadcast(self._h, C.c_void_p(t.data_ptr()), t.numel() * t.element_size(), int(root),
                                      _stream()), 'mt_broadcast')

    def close(self):
        if getattr(self, '_h', None):
            _lib.hip().mt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class LoopbackComm(RcclComm):
    """A communicator behind the C ABI without RCCL (mt_comm_init_loopback): its all-reduce scales
    by `replicas` (the sum of identical replicas) and then holds the stream delay_us — the
    stream-order tests of the data-parallel update (tests/test_dp_gpu.py) on one GPU, where RCCL's
    one-rank sum is the identity and an ordering bug would not show."""
    kind = 'loopback'

    def __init__(self, replicas=2, delay_us=2000):
        h = C.c_void_p()
        check(_lib.hip().mt_comm_init_loopback(int(replicas), int(delay_us), C.byref(h)), 'mt_comm_init_loopback')
        self._h = h
        self.rank, self.world = 0, int(replicas)


class TorchComm(object):
    capturable = False
    kind = 'torch'

    def __init__(self, rank, world, device_index=None):
        self.rank, self.world = rank, world

    def allreduce(self, t):
        torch.distributed.all_reduce(t)

    def broadcast(self, t, root=0):
        torch.distributed.broadcast(t, root)

    def close(self):
        pass


def make(kind, rank, world, device_index):
    if kind == 'rccl':
        return RcclComm(rank, world, device_index)
    if kind == 'torch':
        return TorchComm(rank, world, device_index)
    raise ValueError('comm must be rccl or torch, not %r' % kind)


def broadcast_scalars(values, rank, src=0):
    """Host integers from rank `src` (control channel: torch.distributed, e.g. gloo)."""
    import torch.distributed as dist
    box = [list(values) if rank == src else None]
    dist.broadcast_object_list(box, src=src)
    return box[0]
