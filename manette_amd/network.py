"""HIP-backed policy/value network: the device side of networks.py + policy_v_network.py +
the optimizer of actor_learner.py:43-74, driven through libmanette_hip.so.

torch tensors are used for device storage and the current stream only; every compute call is a
C-ABI launch. One flat fp32 buffer holds all variables (TF creation order and names); the
gradient and the RMSProp slots (`ms` initialised to ONES, `mom` to zeros — TF1
RMSPropOptimizer, pinned by tests/golden/meta_graph.json) share its layout.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import check


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class WaitStatus(object):
    """The word a bounded device wait sets when it times out (pinned, device-mapped: the kernels
    store 1 with system scope and carry on, so the launch drains). check() — after the stream has
    completed — surfaces a timeout as an MTError, as mt_rollout_step does for the rollout's own word,
    and re-arms the word."""

    def __init__(self):
        self.word = torch.zeros(1, dtype=torch.int32).pin_memory()
        self.dev = host_device_pointer(self.word)

    def check(self, what='device wait'):
        if int(self.word[0]) != 0:
            self.word[0] = 0
            raise _lib.MTError('%s: a bounded device wait timed out (a producer never published within ~2 s)'
                               % what)


class DeviceNetwork(object):
    """network_conf of train.py:52-63 -> device parameters + forward / backward / update."""

    def __init__(self, conf, device='cuda'):
        self.conf = dict(conf)
        self.device = torch.device(device)
        self.arch = conf.get('arch', 'NIPS')
        self.depth = 3 if conf.get('rgb', False) else 1
        self.num_actions = int(conf['num_actions'])
        self.num_reps = int(conf.get('nb_choices', 1))
        self.temp = float(conf.get('softmax_temp', 1.0))
        self.beta = float(conf.get('entropy_regularisation_strength', 0.02))
        self.clip_norm = float(conf.get('clip_norm', 3.0))
        clip_type = conf.get('clip_norm_type', 'global')
        if clip_type not in _lib.MT_CLIP:
            # actor_learner.py:65-67 ('local' iterates (g, v) tuples and cannot run)
            raise ValueError('clip_norm_type %r not supported' % clip_type)
        self.clip_type = _lib.MT_CLIP[clip_type]
        self.decay = float(conf.get('alpha', 0.99))
        self.eps = float(conf.get('e', 0.1))
        cfg = _lib.mt_net_config(_lib.MT_ARCH[self.arch], self.depth, self.num_actions,
                                 self.num_reps, _lib.MT_ACT[conf.get('activation', 'relu')],
                                 float(conf.get('alpha_leaky_relu', 0.1)), self.temp)
        lib = _lib.hip()
        h = C.c_void_p()
        check(lib.mt_net_create(C.byref(cfg), C.byref(h)), 'mt_net_create')
        self._h = h
        n = C.c_size_t()
        check(lib.mt_net_num_params(h, C.byref(n)))
        self.nparams = n.value
        nv = C.c_int()
        check(lib.mt_net_num_vars(h, C.byref(nv)))
        self.vars = []
        for i in range(nv.value):
            name = C.create_string_buffer(256)
            shape = (C.c_int64 * 4)()
            nd = C.c_int()
            off = C.c_size_t()
            bound = C.c_float()
            check(lib.mt_net_var_info(h, i, name, 256, shape, C.byref(nd), C.byref(off), C.byref(bound)))
            self.vars.append((name.value.decode(), tuple(shape[k] for k in range(nd.value)), off.value,
                              bound.value))
        f = C.c_int()
        check(lib.mt_net_feature_dim(h, C.byref(f)))
        self.feature_dim = f.value
        dev = self.device
        self.params = torch.zeros(self.nparams, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.params)
        self.ms = torch.ones_like(self.params)
        self.mom = torch.zeros_like(self.params)
        self.partials = torch.zeros(_lib.MT_NORM_PARTIALS, dtype=torch.float32, device=dev)
        self.norm_dev = torch.zeros(1, dtype=torch.float32, device=dev)
        # the LR lives in pinned, device-mapped host memory: mt_clip_rmsprop reads it in place
        self._lr_host = torch.zeros(1, dtype=torch.float32).pin_memory()
        self._lr_dev_addr = host_device_pointer(self._lr_host)
        self._ws = {}
        self._out = {}

    def __del__(self):
        h = getattr(self, '_h', None)
        if h:
            _lib.hip().mt_net_destroy(h)
            self._h = None

    # ---- parameters ------------------------------------------------------------------------
    def init_params(self, seed=0):
        """U(-d, d) per variable with the reference init bounds (networks.py:34-89); d < 0 is
        N(0, 1) (the LSTM projection, networks.py:124-125)."""
        rs = np.random.RandomState(seed)
        flat = np.zeros(self.nparams, dtype=np.float32)
        for name, shape, off, d in self.vars:
            n = int(np.prod(shape))
            flat[off:off + n] = (rs.uniform(-d, d, size=n) if d >= 0 else rs.standard_normal(size=n)).astype(np.float32)
        self.params.copy_(torch.from_numpy(flat))
        self.ms.fill_(1.0)
        self.mom.zero_()

    def get_variables(self, which='params'):
        flat = getattr(self, which).detach().cpu().numpy()
        return {name: flat[off:off + int(np.prod(shape))].reshape(shape).copy()
                for name, shape, off, _ in self.vars}

    def set_variables(self, values, which='params'):
        flat = getattr(self, which).detach().cpu().numpy().copy()
        for name, shape, off, _ in self.vars:
            if name in values:
                a = np.asarray(values[name], dtype=np.float32)
                assert a.shape == tuple(shape), (name, a.shape, shape)
                flat[off:off + a.size] = a.reshape(-1)
        getattr(self, which).copy_(torch.from_numpy(flat))

    # ---- buffers -----------------------------------------------------------------------------
    def workspace(self, batch, key=None):
        """Device workspace for `batch` rows, cached under `key` (default: the batch size)."""
        key = batch if key is None else key
        n = C.c_size_t()
        check(_lib.hip().mt_net_workspace_bytes(self._h, batch, C.byref(n)))
        ws = self._ws.get(key)
        if ws is None or ws.numel() < n.value:
            ws = torch.zeros(n.value, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def outputs(self, batch, key=None):
        k = (batch, key)
        o = self._out.get(k)
        if o is None:
            dev = self.device
            o = (torch.empty(batch, dtype=torch.float32, device=dev),
                 torch.empty(batch, self.num_actions, dtype=torch.float32, device=dev),
                 torch.empty(batch, self.num_reps, dtype=torch.float32, device=dev))
            self._out[k] = o
        return o

    def forward_branches(self, ws, layout, a, b=0):
        """Diagnostics / parity: the forward values a workspace keeps that the backward branches on
        (mt_net_workspace_region): {'convK': (output, argmax)} — the conv layer's post-activation
        output [rows, H', W', C] fp32 (a pooled layer's pooled map; its sign is the ReLU branch) and,
        for a pooled layer, the max-pool argmax [rows, H', W', C] uint8 (window position 0..3 =
        2 * row + col) else None — and 'H': the dense output [rows', F]. layout 0 = a forward of `a`
        rows; 1 = the LSTM frame store of E = a, T = b (conv rows = its 1 + (T + 5) E frames, H rows =
        its (T + 1) E windows); 2 = an LSTM forward of `a` windows (conv rows = 5 a frames)."""
        lib = _lib.hip()
        raw = ws.cpu().numpy()
        rows = {0: int(a), 1: 1 + (int(b) + 5) * int(a), 2: 5 * int(a)}[int(layout)]
        hrows = {0: int(a), 1: (int(b) + 1) * int(a), 2: int(a)}[int(layout)]
        convs = [v for v in self.vars if v[0].startswith('Network/conv') and v[0].endswith('_weights')]

        def region(kind, layer):
            off, n = C.c_size_t(), C.c_size_t()
            rc = lib.mt_net_workspace_region(self._h, int(layout), int(a), int(b), int(kind), int(layer),
                                             C.byref(off), C.byref(n))
            return (off.value, n.value) if rc == 0 else None

        out = {}
        for i, (name, shape, _, _) in enumerate(convs):
            cout = int(shape[3])
            off, n = region(0, i)
            side = int(round((n // 4 // (rows * cout)) ** 0.5))
            assert rows * side * side * cout * 4 == n, (name, n, rows, cout)
            y = raw[off:off + n].view(np.float32).reshape(rows, side, side, cout).copy()
            r = region(1, i)
            arg = raw[r[0]:r[0] + r[1]].reshape(rows, side, side, cout).copy() if r else None
            out[name.split('/')[1]] = (y, arg)
        off, n = region(2, 0)
        out['H'] = raw[off:off + n].view(np.float32).reshape(hrows, -1).copy()
        return out

    # ---- compute -----------------------------------------------------------------------------
    def forward(self, obs, batch=None, out=None, ws_key=None, infer=False):
        """obs: uint8 cuda tensor [B,84,84,4*depth]. Returns (v, pi, rep) device tensors.
        The activations stay in the workspace of `ws_key or batch` for loss_backward, unless
        infer=True (mt_forward_infer: fused trunk where built, nothing kept for a backward)."""
        B = int(batch if batch is not None else obs.shape[0])
        assert obs.dtype == torch.uint8 and obs.is_cuda and obs.is_contiguous()
        assert obs.numel() >= B * 84 * 84 * 4 * self.depth
        ws = self.workspace(B, ws_key)
        v, pi, rep = out if out is not None else self.outputs(B)
        fn = _lib.hip().mt_forward_infer if infer else _lib.hip().mt_forward
        check(fn(self._h, _ptr(self.params), _ptr(obs), B, _ptr(ws), ws.numel(), _ptr(v), _ptr(pi), _ptr(rep),
                 _stream()), 'mt_forward_infer' if infer else 'mt_forward')
        return v, pi, rep

    def forward_rows(self, obs, batch, train_ws, train_rows, row0, out, ws_key=None):
        """mt_forward_rows: inference forward of `batch` rows that also leaves their activations in
        rows [row0, row0 + batch) of train_ws (a workspace of train_rows rows), so the update's
        loss_backward on train_rows needs no forward. out = (v, pi, rep)."""
        B = int(batch)
        assert obs.dtype == torch.uint8 and obs.is_cuda and obs.is_contiguous()
        ws = self.workspace(B, ws_key)
        v, pi, rep = out
        check(_lib.hip().mt_forward_rows(self._h, _ptr(self.params), _ptr(obs), B, _ptr(ws), ws.numel(),
                                         _ptr(train_ws), train_ws.numel(), int(train_rows), int(row0), _ptr(v),
                                         _ptr(pi), _ptr(rep), _stream()), 'mt_forward_rows')
        return v, pi, rep

    def forward_trunk(self, obs, batch, ws_key=None):
        """mt_forward_trunk: the trunk half of the inference forward only (roofline timing)."""
        ws = self.workspace(batch, ws_key)
        check(_lib.hip().mt_forward_trunk(self._h, _ptr(self.params), _ptr(obs), int(batch), _ptr(ws), ws.numel(),
                                          _stream()), 'mt_forward_trunk')

    def forward_trunk_stacking(self, prev, frames, ready, tag, out, batch, ws_key=None, status=None):
        """mt_forward_trunk_stacking: the rollout chain's stacking trunk (in-kernel pull of each
        env's frames behind its ready word), diagnostics / parity / roofline timing. status: a
        WaitStatus whose word a timed-out device wait sets (check it once the stream completed)."""
        ws = self.workspace(batch, ws_key)
        addr = lambda x: x if isinstance(x, C.c_void_p) else _ptr(x)
        check(_lib.hip().mt_forward_trunk_stacking(self._h, _ptr(self.params), _ptr(prev), addr(frames), addr(ready),
                                                   C.c_uint32(tag), _ptr(out), int(batch), _ptr(ws), ws.numel(),
                                                   C.c_void_p(status.dev) if status is not None else None,
                                                   _stream()), 'mt_forward_trunk_stacking')
        return ws

    # ---- LSTM frame-store mode (include/manette_hip.h, mt_lstm_*) -------------------------------
    def lstm_workspace(self, E, T):
        n = C.c_size_t()
        check(_lib.hip().mt_lstm_frames_workspace_bytes(self._h, int(E), int(T), C.byref(n)))
        key = ('lstm_frames', E, T)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < n.value:
            ws = torch.empty(n.value, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def lstm_frames_forward(self, fstore, row0, nrows, E, T):
        """Trunk + cell x-product of frame rows [row0, row0 + nrows) of the frame store."""
        ws = self.lstm_workspace(E, T)
        check(_lib.hip().mt_lstm_frames_forward(self._h, _ptr(self.params), _ptr(fstore), int(row0), int(nrows),
                                                int(E), int(T), _ptr(ws), ws.numel(), _stream()),
              'mt_lstm_frames_forward')

    def lstm_windows_forward(self, nz_t, t, E, T, out):
        """The E windows of step t (T = bootstrap): out = (v [E], pi [E][A], rep [E][R])."""
        ws = self.lstm_workspace(E, T)
        v, pi, rep = out
        assert nz_t.dtype == torch.int32 and nz_t.is_cuda and nz_t.numel() == E
        check(_lib.hip().mt_lstm_windows_forward(self._h, _ptr(self.params), _ptr(nz_t), int(t), int(E), int(T),
                                                 _ptr(ws), ws.numel(), _ptr(v), _ptr(pi), _ptr(rep), _stream()),
              'mt_lstm_windows_forward')
        return v, pi, rep

    def lstm_step_forward(self, fstore, t, E, T, nz, over, out):
        """One rollout macro-step: step t's new frame rows + its E windows (mt_lstm_step_forward).
        nz: [T+1][E] int32 (device); t > 0 derives nz[t] from nz[t-1] and `over` (step t-1's
        episode-end flags: a device tensor, or the device address of pinned host memory)."""
        ws = self.lstm_workspace(E, T)
        v, pi, rep = out
        assert nz.dtype == torch.int32 and nz.is_cuda and nz.numel() == (T + 1) * E
        over_p = over if isinstance(over, (int, C.c_void_p)) or over is None else _ptr(over)
        check(_lib.hip().mt_lstm_step_forward(self._h, _ptr(self.params), _ptr(fstore), int(t), int(E), int(T),
                                              _ptr(nz), over_p, _ptr(ws), ws.numel(), _ptr(v), _ptr(pi), _ptr(rep),
                                              _stream()), 'mt_lstm_step_forward')
        return v, pi, rep

    def lstm_frames_backward(self, fstore, nz, E, T, pi, rep, v, a_idx, r_idx, y, adv, loss_terms=None,
                             norm_partials=False):
        """Gradient of the T*E windows of the last rollout into self.grad. norm_partials: as
        returns_loss_backward's (the global-norm partials left in self.partials; single process)."""
        ws = self.lstm_workspace(E, T)
        check(_lib.hip().mt_lstm_frames_backward(
            self._h, _ptr(self.params), _ptr(fstore), _ptr(nz), int(E), int(T), _ptr(ws), ws.numel(), _ptr(pi),
            _ptr(rep), _ptr(v), _ptr(a_idx), _ptr(r_idx), _ptr(y), _ptr(adv), self.beta, _ptr(self.grad),
            _ptr(loss_terms), _ptr(self.partials if norm_partials else None), _stream()), 'mt_lstm_frames_backward')
        return self.grad

    def loss_backward(self, obs, B, v, pi, rep, a_idx, r_idx, y, adv, loss_terms=None, ws_key=None):
        """Gradient of policy_v_network.py:25-74 into self.grad (needs forward() on obs first)."""
        ws = self.workspace(B, ws_key)
        for t in (a_idx, r_idx):
            assert t.dtype == torch.int32 and t.is_cuda
        check(_lib.hip().mt_loss_backward(
            self._h, _ptr(self.params), _ptr(obs), B, _ptr(ws), ws.numel(), _ptr(pi), _ptr(rep),
            _ptr(v), _ptr(a_idx), _ptr(r_idx), _ptr(y), _ptr(adv), self.beta, _ptr(self.grad),
            _ptr(loss_terms), _stream()), 'mt_loss_backward')
        return self.grad

    def returns_loss_backward(self, obs, T, E, pi, rep, values, a_idx, r_idx, rewards, masks, v_boot, gamma, y, adv,
                              loss_terms=None, ws_key=None, norm_partials=False, boot_ws=None):
        """mt_returns + mt_loss_backward in one call (rows t*E + e): the n-step scan of paac.py:219-231
        runs inside the loss kernel. rewards / masks: [T][E] device tensors or device addresses.
        norm_partials: the backward also leaves the global-norm partials in self.partials, so the
        following apply_gradients(partials_ready=True) skips mt_grad_sumsq (single process only).
        boot_ws: the rollout's E-row workspace holding the bootstrap's dense slabs (a rollout made
        with MT_ROLLOUT_BOOT_SLABS): V(s_T) is finished in the loss kernel and written to v_boot
        (mt_returns_loss_backward_boot)."""
        B = T * E
        ws = self.workspace(B, ws_key)
        addr = lambda x: C.c_void_p(x) if isinstance(x, int) else _ptr(x)
        if boot_ws is not None:
            check(_lib.hip().mt_returns_loss_backward_boot(
                self._h, _ptr(self.params), _ptr(obs), int(T), int(E), _ptr(ws), ws.numel(), _ptr(pi), _ptr(rep),
                _ptr(values), _ptr(a_idx), _ptr(r_idx), addr(rewards), addr(masks), _ptr(boot_ws), boot_ws.numel(),
                _ptr(v_boot), float(gamma), _ptr(y), _ptr(adv), self.beta, _ptr(self.grad), _ptr(loss_terms),
                _ptr(self.partials if norm_partials else None), _stream()), 'mt_returns_loss_backward_boot')
            return self.grad
        check(_lib.hip().mt_returns_loss_backward(
            self._h, _ptr(self.params), _ptr(obs), int(T), int(E), _ptr(ws), ws.numel(), _ptr(pi), _ptr(rep),
            _ptr(values), _ptr(a_idx), _ptr(r_idx), addr(rewards), addr(masks), _ptr(v_boot), float(gamma), _ptr(y),
            _ptr(adv), self.beta, _ptr(self.grad), _ptr(loss_terms), _ptr(self.partials if norm_partials else None),
            _stream()), 'mt_returns_loss_backward')
        return self.grad

    def set_lr(self, lr):
        """The LR of the next apply_gradients: written into pinned host memory that the RMSProp
        kernel reads in place (no copy; a captured graph also picks up the schedule)."""
        self._lr_host[0] = float(lr)

    def apply_gradients(self, inv_scale=1.0, partials_ready=False):
        """clip_by_global_norm + ApplyRMSProp on self.grad (actor_learner.py:47-74).
        inv_scale folds the 1/world of a data-parallel gradient sum. partials_ready: the backward
        already wrote the norm partials (returns_loss_backward(norm_partials=True), inv_scale 1)."""
        lib = _lib.hip()
        s = _stream()
        if not partials_ready:
            check(lib.mt_grad_sumsq(_ptr(self.grad), self.nparams, float(inv_scale), _ptr(self.partials), s),
                  'mt_grad_sumsq')
        check(lib.mt_clip_rmsprop(_ptr(self.params), _ptr(self.ms), _ptr(self.mom), _ptr(self.grad),
                                  self.nparams, _ptr(self.partials), C.c_void_p(self._lr_dev_addr), self.decay, 0.0,
                                  self.eps, self.clip_norm, self.clip_type, float(inv_scale),
                                  _ptr(self.norm_dev), s), 'mt_clip_rmsprop')


def sample(pi, rep, seed, counters, a_idx, r_idx, pair=None, row0=0):
    """Device multinomial draw (perf mode of exploration_policy.py:108-116); row0 = the global env
    id of row 0 (the uniforms hash the global env id, so a DP shard draws as the union would)."""
    B, A = pi.shape
    R = rep.shape[1]
    check(_lib.hip().mt_sample(_ptr(pi), _ptr(rep), B, A, R, C.c_uint64(seed), int(row0), _ptr(counters),
                               _ptr(a_idx), _ptr(r_idx), _ptr(pair), _stream()), 'mt_sample')


def host_device_pointer(t):
    """Device address of a pinned host tensor (hipHostGetDevicePointer)."""
    assert t.is_pinned()
    d = C.c_void_p()
    check(_lib.hip().mt_host_device_pointer(C.c_void_p(t.data_ptr()), C.byref(d)), 'mt_host_device_pointer')
    return d.value


def preprocess_frames(screens_dev, frame_idx, push_count, E, depth, row_lut, col_lut, prev, out):
    """atari_emulator.py:79-124 on device, reading each push's two screens where the emulators
    left them (screens_dev: device address of the bank, frame_idx [E][8], push_count [E])."""
    check(_lib.hip().mt_preprocess_frames(C.c_void_p(screens_dev), _ptr(frame_idx), _ptr(push_count), E, depth,
                                          _ptr(row_lut), _ptr(col_lut), _ptr(prev), _ptr(out), _stream()),
          'mt_preprocess_frames')


def memory_push(memory, whole_t, fresh, masks):
    """paac.py:79-83 + :202-203 on device: whole_t <- memory, shift + fresh, zero ended episodes."""
    E = memory.shape[0]
    frame = memory[0, 0].numel()
    check(_lib.hip().mt_memory_push(_ptr(memory), _ptr(whole_t), _ptr(fresh), _ptr(masks), E, frame, _stream()),
          'mt_memory_push')


def returns(rewards, masks, values, v_boot, gamma, y, adv):
    """paac.py:219-231 on device. rewards / masks: [T][E] device tensors, or device addresses
    (e.g. of pinned, device-mapped host memory the kernel reads in place)."""
    T, E = values.shape
    addr = lambda x: C.c_void_p(x) if isinstance(x, int) else _ptr(x)
    check(_lib.hip().mt_returns(addr(rewards), addr(masks), _ptr(values), _ptr(v_boot), float(gamma),
                                T, E, _ptr(y), _ptr(adv), _stream()), 'mt_returns')


def preprocess(raw, push_offset, push_count, E, depth, row_lut, col_lut, prev, out, src_rows=210, pooled=False,
               resized=False):
    """atari_emulator.py:79-124 frame pool + resize + stack on device (raw screens of src_rows
    rows: 210 = whole screens with the resize LUT, 84 = runner-selected rows, identity LUT).
    pooled: raw holds one screen per push, the frame-pool max already taken (mt_preprocess_pooled);
    resized: raw holds each push's final 84x84 frame (mt_preprocess_resized, stacking only)."""
    rp = C.c_void_p(raw) if isinstance(raw, int) else _ptr(raw)  # (int: a pinned buffer's device address)
    if resized:
        check(_lib.hip().mt_preprocess_resized(rp, _ptr(push_offset), _ptr(push_count), E, depth, _ptr(prev),
                                               _ptr(out), _stream()), 'mt_preprocess_resized')
        return
    name = 'mt_preprocess_pooled' if pooled else 'mt_preprocess'
    check(getattr(_lib.hip(), name)(rp, _ptr(push_offset), _ptr(push_count), E, depth, int(src_rows),
                                    _ptr(row_lut), _ptr(col_lut), _ptr(prev), _ptr(out), _stream()), name)
