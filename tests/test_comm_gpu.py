"""RCCL behind the C ABI (mt_comm_*, manette_amd/csrc/comm.hip) on the GPU box.

One GPU per box: the communicator runs with world = 1 here (init, in-place sum all-reduce and
broadcast are identities, bit for bit), and the all-reduce is captured into a hipGraph and replayed
the way PAACLearner.update captures it. The multi-rank path is exercised by bench.py --gpus N on a
whole node (the driver's scaling runs); ranks sharing one GPU use the torch comm
(tests/test_learner_gpu.py::test_dp_two_ranks_equal_single_process_union)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rccl_world1_allreduce_broadcast_graph():
    from manette_amd import _lib
    from manette_amd.comm import RcclComm
    comm = RcclComm(0, 1, torch.cuda.current_device())
    try:
        r, w = C.c_int(), C.c_int()
        _lib.check(_lib.hip().mt_comm_info(comm._h, C.byref(r), C.byref(w)))
        assert (r.value, w.value) == (0, 1)
        g = torch.Generator(device='cuda').manual_seed(3)
        x = torch.randn(678464, device='cuda', generator=g)
        ref = x.clone()
        comm.allreduce(x)
        comm.broadcast(x, 0)
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
        # captured on a side stream (as the learner's update graph), replayed 3 times
        lib = _lib.hip()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            s = C.c_void_p(side.cuda_stream)
            _lib.check(lib.mt_graph_begin(s), 'mt_graph_begin')
            try:
                comm.allreduce(x)
            finally:
                h = C.c_void_p()
                rc = lib.mt_graph_end(s, C.byref(h))
            _lib.check(rc, 'mt_graph_end')
            for _ in range(3):
                _lib.check(lib.mt_graph_launch(h, s), 'mt_graph_launch')
        torch.cuda.synchronize()
        lib.mt_graph_destroy(h)
        assert torch.equal(x, ref)
        with pytest.raises(_lib.MTError):
            comm.broadcast(x, 1)  # root out of range -> status code, not a crash
    finally:
        comm.close()
