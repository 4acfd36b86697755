"""Diagnostic (tools only): the conv1 weight gradient of an RGB NIPS net at B=5 (the
test_loss_backward_parity[5-NIPS-3-4-11] case) with its fp64 oracle, saved to an npz, so two
library variants can be compared elementwise:
    python tools/dual_diag.py out.npz            (MANETTE_HIP_LIB selects the variant)
Used for the two-accumulator GEMM-core experiment."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '/root/repo'), 'tests'))
from manette_amd.network import DeviceNetwork
from oracle import nets
B, depth, A, R = 5, 3, 4, 11
conf = dict(arch='NIPS', num_actions=A, nb_choices=R, rgb=True, softmax_temp=1.0, entropy_regularisation_strength=0.02,
            clip_norm=3.0, clip_norm_type='global')
net = DeviceNetwork(conf, device='cuda:0'); net.init_params(7 + B)
rs = np.random.RandomState(100 + B)
obs = rs.randint(0, 256, size=(B, 84, 84, 4 * depth)).astype(np.uint8)
a_idx = rs.randint(0, A, size=B).astype(np.int32); r_idx = rs.randint(0, R, size=B).astype(np.int32)
y = rs.randn(B).astype(np.float32); adv = rs.randn(B).astype(np.float32)
d = lambda x: torch.from_numpy(x).cuda()
v, pi, rep = net.forward(d(obs))
net.loss_backward(d(obs), B, v, pi, rep, d(a_idx), d(r_idx), d(y), d(adv))
torch.cuda.synchronize()
got = net.get_variables('grad')['Network/conv1/conv1_weights']
spec = nets.arch_spec('NIPS', depth, A, R)
_, G, _ = nets.loss_and_grads(spec, net.get_variables(), obs, a_idx, r_idx, y, adv, 0.02)
ref = G['Network/conv1/conv1_weights']
# the product's inputs to the conv1 weight gradient, for tools/gemm_repro.hip (argv: <X.u8> <dY.f32>):
# obs [5][84][84][12] uint8 and the device's dY = conv1's output gradient [5][20][20][16] fp32
import ctypes as C
from manette_amd import _lib
off, n = C.c_size_t(), C.c_size_t()
ws = net.workspace(B)
_lib.check(_lib.hip().mt_net_workspace_region(net._h, 0, B, 0, 3, 0, C.byref(off), C.byref(n)))
dY = ws.cpu().numpy()[off.value:off.value + n.value].view(np.float32)
obs.tofile(sys.argv[1] + '.X.u8')
dY.tofile(sys.argv[1] + '.dY.f32')
# and the conv2 backward-data product's (tools/dgrad_repro.hip): dY2 = conv2's output gradient
# [5][9][9][32], W2 [4][4][16][32], act1 = conv1's output [5][20][20][16]
wsn = ws.cpu().numpy()
for kind, layer, name in ((3, 1, 'dY2'), (0, 0, 'act1')):
    _lib.check(_lib.hip().mt_net_workspace_region(net._h, 0, B, 0, kind, layer, C.byref(off), C.byref(n)))
    wsn[off.value:off.value + n.value].view(np.float32).tofile(sys.argv[1] + '.%s.f32' % name)
net.get_variables()['Network/conv2/conv2_weights'].astype(np.float32).tofile(sys.argv[1] + '.W2.f32')
print('dY: %d values, %d exact zeros, %d subnormal, channel 10: %d zeros %d subnormal, |max| %.3e' % (
    dY.size, (dY == 0).sum(), ((dY != 0) & (np.abs(dY) < np.finfo(np.float32).tiny)).sum(),
    (dY.reshape(-1, 16)[:, 10] == 0).sum(), ((dY.reshape(-1, 16)[:, 10] != 0) &
                                              (np.abs(dY.reshape(-1, 16)[:, 10]) < np.finfo(np.float32).tiny)).sum(),
    np.abs(dY).max()))
np.savez(sys.argv[1], got=got, ref=ref)
d = np.linalg.norm((got - ref).reshape(-1, 16), axis=0) / np.linalg.norm(ref.reshape(-1, 16), axis=0)
print(os.environ.get('MANETTE_HIP_LIB', 'product library'), 'per-channel rel L2:', ' '.join('%.1e' % x for x in d))
print('saved', sys.argv[1])
