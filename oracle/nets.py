"""numpy restatement of the policy/value networks, heads, loss and backward (oracle).

networks.py:14-127 (Operations), :152-155 (input scale), :178-192 (NIPS), :206-225 (PWYX),
:227-258 (LSTM), :261-278 (NATURE); policy_v_network.py:19-74 (heads + loss). NHWC activations, HWIO conv
weights, (in, out) dense weights, TF VALID/SAME padding, flatten in NHWC order.
Backward is the hand-derived gradient of the same graph (TF's ops: Conv2DBackprop*, MatMul
grads, ReluGrad on the activation output, Softmax/Log grads).
"""
import numpy as np
from numpy.lib.stride_tricks import as_strided


def arch_spec(arch, depth, num_actions, num_reps):
    """Layer list + TF variable names/shapes/init bounds (networks.py:34-89, :178-278)."""
    C = 4 * depth
    if arch == 'NIPS':
        convs = [('conv1', 8, 4, C, 16, 'VALID', False), ('conv2', 4, 2, 16, 32, 'VALID', False)]
        fc = ('fc3', 256)
    elif arch == 'NATURE':
        convs = [('conv1', 8, 4, C, 32, 'VALID', False), ('conv2', 4, 2, 32, 64, 'VALID', False),
                 ('conv3', 3, 1, 64, 64, 'VALID', False)]
        fc = ('fc4', 512)
    elif arch in ('PWYX', 'LSTM'):
        # LSTM (networks.py:227-258) runs the PWYX trunk on each of its 5 window frames
        convs = [('conv1', 5, 1, C, 32, 'SAME', True), ('conv2', 5, 1, 32, 32, 'SAME', True),
                 ('conv3', 4, 1, 32, 64, 'SAME', True), ('conv4', 3, 1, 64, 64, 'SAME', False)]
        fc = ('fc5', 512) if arch == 'PWYX' else ('fc6', 128)
    else:
        raise ValueError(arch)
    H = 84
    for (_, k, s, cin, cout, pad, pool) in convs:
        H = (H - k) // s + 1 if pad == 'VALID' else -(-H // s)
        if pool:
            H = H // 2
    flat = H * H * convs[-1][4]
    F = fc[1]
    vars_ = []
    for (name, k, s, cin, cout, pad, pool) in convs:
        vars_.append(('Network/%s/%s_weights' % (name, name), (k, k, cin, cout), 1.0 / np.sqrt(cout * k * k)))
        vars_.append(('Network/%s/%s_biases' % (name, name), (cout,), 1.0 / np.sqrt(cin * k * k)))
    lstm = None
    fc_in = flat
    if arch == 'LSTM':
        # Operations.rnn (networks.py:112-127): static_rnn of BasicLSTMCell(32, forget_bias=1) over
        # 5 steps of 6400 features, then matmul(h_5, w) + b. TF 1.3 names the cell variables
        # rnn/basic_lstm_cell/{kernel,bias} (get_variable ignores name_scope; kernel = [x, h] x 4
        # gates i, j, f, o; glorot-uniform kernel, zero bias); w, b are unnamed tf.Variables under
        # the Network/lstm name scope with N(0, 1) init (bound < 0 below means N(0, 1)). No LSTM
        # checkpoint exists: names and gate order follow TF 1.3 semantics, parity unpinned.
        n_hidden, n_steps = 32, 5
        lstm = dict(hidden=n_hidden, steps=n_steps, forget_bias=1.0)
        kin = flat + n_hidden
        vars_.append(('rnn/basic_lstm_cell/kernel', (kin, 4 * n_hidden), np.sqrt(6.0 / (kin + 4 * n_hidden))))
        vars_.append(('rnn/basic_lstm_cell/bias', (4 * n_hidden,), 0.0))
        vars_.append(('Network/lstm/Variable', (n_hidden, n_hidden), -1.0))
        vars_.append(('Network/lstm/Variable_1', (n_hidden,), -1.0))
        fc_in = n_hidden
    vars_.append(('Network/%s/%s_weights' % (fc[0], fc[0]), (fc_in, F), 1.0 / np.sqrt(fc_in)))
    vars_.append(('Network/%s/%s_biases' % (fc[0], fc[0]), (F,), 1.0 / np.sqrt(fc_in)))
    for scope, nm, n in [('Training/Critic', 'critic_output', 1), ('Training/Actor', 'actor_output', num_actions),
                         ('Training/Repetition', 'repetition_output', num_reps)]:
        vars_.append(('%s/%s/%s_weights' % (scope, nm, nm), (F, n), 1.0 / np.sqrt(F)))
        vars_.append(('%s/%s/%s_biases' % (scope, nm, nm), (n,), 1.0 / np.sqrt(F)))
    return dict(convs=convs, fc=fc, flat=flat, F=F, vars=vars_, A=num_actions, R=num_reps, lstm=lstm)


def _pads(H, k, s, padding):
    if padding == 'VALID':
        return (H - k) // s + 1, 0, 0
    O = -(-H // s)
    tot = max((O - 1) * s + k - H, 0)
    return O, tot // 2, tot - tot // 2  # TF SAME: extra padding after


def im2col(x, k, s, padding):
    """x [B,H,W,C] -> cols [B*OH*OW, k*k*C] (k order ky, kx, c)."""
    B, H, W, C = x.shape
    OH, pt, pb = _pads(H, k, s, padding)
    OW, pl, pr = _pads(W, k, s, padding)
    if pt or pb or pl or pr:
        x = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    x = np.ascontiguousarray(x)
    sb, sh, sw, sc = x.strides
    win = as_strided(x, shape=(B, OH, OW, k, k, C), strides=(sb, sh * s, sw * s, sh, sw, sc))
    return win.reshape(B * OH * OW, k * k * C), (OH, OW, pt, pl)


def col2im(dcols, xshape, k, s, padding):
    B, H, W, C = xshape
    OH, pt, pb = _pads(H, k, s, padding)
    OW, pl, pr = _pads(W, k, s, padding)
    d = dcols.reshape(B, OH, OW, k, k, C)
    dx = np.zeros((B, H + pt + pb, W + pl + pr, C), dtype=dcols.dtype)
    for ky in range(k):
        for kx in range(k):
            dx[:, ky:ky + s * (OH - 1) + 1:s, kx:kx + s * (OW - 1) + 1:s, :] += d[:, :, :, ky, kx, :]
    return dx[:, pt:pt + H, pl:pl + W, :]


def act_fwd(x, act, alpha):
    return np.maximum(x, 0) if act == 'relu' else np.maximum(x, alpha * x)


def act_bwd(y, act, alpha):
    # TF ReluGrad: grad * (y > 0); tf.maximum(x, a*x) grad: x >= a*x  <=>  y >= 0.
    if act == 'relu':
        return (y > 0).astype(y.dtype)
    return np.where(y >= 0, 1.0, alpha).astype(y.dtype)


def maxpool2(x):
    """2x2/2 VALID max pool (networks.py:108-110). Returns (y, argmax mask)."""
    B, H, W, C = x.shape
    OH, OW = H // 2, W // 2
    xc = x[:, :OH * 2, :OW * 2, :].reshape(B, OH, 2, OW, 2, C)
    y = xc.max(axis=(2, 4))
    return y


def maxpool2_bwd(x, y, dy, route=None):
    """TF MaxPoolGrad routes the gradient to the first max in the window (row-major scan).
    route (optional, [B, OH, OW, C] in 0..3 = 2 * row + col): the window position to route to
    instead — a device's own choice at near-ties, where fp32 rounding may order the top two
    values differently (tests/parity_util.py device_routes)."""
    B, H, W, C = x.shape
    OH, OW = H // 2, W // 2
    dx = np.zeros_like(x)
    if route is not None:
        for dy_ in range(2):
            for dx_ in range(2):
                dx[:, dy_:OH * 2:2, dx_:OW * 2:2, :] = np.where(route == 2 * dy_ + dx_, dy, 0)
        return dx
    taken = np.zeros((B, OH, OW, C), dtype=bool)
    for dy_ in range(2):
        for dx_ in range(2):
            xs = x[:, dy_:OH * 2:2, dx_:OW * 2:2, :]
            hit = (xs == y) & ~taken
            dx[:, dy_:OH * 2:2, dx_:OW * 2:2, :] += np.where(hit, dy, 0)
            taken |= hit
    return dx


def pool_route(x):
    """2x2/2 VALID max-pool windows of x [B,H,W,C]: the position of the first maximum (0..3,
    2 * row + col, MaxPoolGrad's choice) and the relative gap between the top two values."""
    B, H, W, C = x.shape
    OH, OW = H // 2, W // 2
    win = x[:, :OH * 2, :OW * 2, :].reshape(B, OH, 2, OW, 2, C).transpose(0, 1, 3, 5, 2, 4).reshape(B, OH, OW, C, 4)
    arg = np.argmax(win, axis=-1).astype(np.uint8)  # first maximum
    srt = np.sort(win, axis=-1)
    gap = (srt[..., 3] - srt[..., 2]) / np.maximum(np.abs(srt[..., 3]), 1e-30)
    return arg, gap


def softmax(z):
    m = z.max(axis=1, keepdims=True)
    e = np.exp(z - m)
    return e / e.sum(axis=1, keepdims=True)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_forward(spec, P, flat, dtype):
    """Operations.rnn (networks.py:112-127): flat [B*5, 6400] frame features (window-major) ->
    h = matmul(h_5, w) + b [B, 32]. BasicLSTMCell: z = [x_t, h_{t-1}] K + bias, gates (i, j, f, o),
    c_t = c_{t-1} sigmoid(f + 1) + sigmoid(i) tanh(j), h_t = tanh(c_t) sigmoid(o); zero state."""
    L = spec['lstm']
    nh, T = L['hidden'], L['steps']
    B = flat.shape[0] // T
    X = flat.reshape(B, T, -1)
    K = P['rnn/basic_lstm_cell/kernel'].astype(dtype)
    kb = P['rnn/basic_lstm_cell/bias'].astype(dtype)
    c = np.zeros((B, nh), dtype)
    h = np.zeros((B, nh), dtype)
    steps = []
    for t in range(T):
        xh = np.concatenate([X[:, t], h], axis=1)
        z = xh @ K + kb
        i, j, f, o = (z[:, g * nh:(g + 1) * nh] for g in range(4))
        si, tj, sf, so = sigmoid(i), np.tanh(j), sigmoid(f + L['forget_bias']), sigmoid(o)
        c_prev = c
        c = c_prev * sf + si * tj
        tc = np.tanh(c)
        h = tc * so
        steps.append(dict(xh=xh, si=si, tj=tj, sf=sf, so=so, c_prev=c_prev, tc=tc))
    w = P['Network/lstm/Variable'].astype(dtype)
    b = P['Network/lstm/Variable_1'].astype(dtype)
    return h @ w + b, dict(steps=steps, h5=h)


def lstm_backward(spec, P, lc, dout, dtype, G):
    """Gradient of lstm_forward: fills G for the cell and projection variables, returns dflat
    [B*5, 6400] (TF SigmoidGrad / TanhGrad: y(1-y), 1-y^2 on the forward outputs)."""
    L = spec['lstm']
    nh, T = L['hidden'], L['steps']
    w = P['Network/lstm/Variable'].astype(dtype)
    K = P['rnn/basic_lstm_cell/kernel'].astype(dtype)
    G['Network/lstm/Variable'] = lc['h5'].T @ dout
    G['Network/lstm/Variable_1'] = dout.sum(0)
    dh = dout @ w.T
    B = dh.shape[0]
    dc = np.zeros_like(dh)
    dK = np.zeros_like(K)
    dkb = np.zeros(K.shape[1], dtype)
    nin = K.shape[0] - nh
    dX = np.zeros((B, T, nin), dtype)
    for t in range(T - 1, -1, -1):
        st = lc['steps'][t]
        dzo = dh * st['tc'] * st['so'] * (1 - st['so'])
        dc = dc + dh * st['so'] * (1 - st['tc'] ** 2)
        dzi = dc * st['tj'] * st['si'] * (1 - st['si'])
        dzj = dc * st['si'] * (1 - st['tj'] ** 2)
        dzf = dc * st['c_prev'] * st['sf'] * (1 - st['sf'])
        dc = dc * st['sf']
        dz = np.concatenate([dzi, dzj, dzf, dzo], axis=1)
        dK += st['xh'].T @ dz
        dkb += dz.sum(0)
        dxh = dz @ K.T
        dX[:, t] = dxh[:, :nin]
        dh = dxh[:, nin:]
    G['rnn/basic_lstm_cell/kernel'] = dK
    G['rnn/basic_lstm_cell/bias'] = dkb
    return dX.reshape(B * T, nin)


def trunk_forward(spec, P, obs, act='relu', alpha=0.1, dtype=np.float64):
    """Input scale (networks.py:155) + the conv layers (+ pools) of one frame batch obs uint8
    [B,84,84,C]: returns (flat [B, spec['flat']] in NHWC order, layer caches)."""
    x = obs.astype(dtype) * dtype(1.0 / 255.0)  # networks.py:155
    layers = []
    for (name, k, s, cin, cout, pad, pool) in spec['convs']:
        W = P['Network/%s/%s_weights' % (name, name)].astype(dtype)
        b = P['Network/%s/%s_biases' % (name, name)].astype(dtype)
        cols, (OH, OW, _, _) = im2col(x, k, s, pad)
        z = (cols @ W.reshape(-1, cout) + b).reshape(x.shape[0], OH, OW, cout)  # pre-activation
        y = act_fwd(z, act, alpha)
        entry = dict(x=x, y=y, z=z, k=k, s=s, pad=pad, pool=pool, cout=cout, name=name)
        if pool:
            y2 = maxpool2(y)
            entry['yp'] = y2
            y = y2
        layers.append(entry)
        x = y
    return x.reshape(x.shape[0], -1), layers


def branch_factor(branch, act, alpha, dtype=np.float64):
    """act'(.) from the branch taken (True = the positive side: ReLU's x > 0, leaky's x >= 0)."""
    return np.where(branch, 1.0, 0.0 if act == 'relu' else alpha).astype(dtype)


def trunk_backward(spec, P, layers, dflat, G, act='relu', alpha=0.1, dtype=np.float64, routes=None,
                   branches=None):
    """Gradient of trunk_forward for dflat [B, flat]: conv weight / bias gradients ADDED into G
    (so chunks of frames accumulate), TF's Conv2DBackprop* / ReluGrad / MaxPoolGrad.
    routes (optional): {conv name: [B, OH/2, OW/2, C] pool positions} replacing MaxPoolGrad's own
    choice; branches (optional): {conv name: bool, the activation branch of every stored output
    (the pooled map of a pooled layer)} replacing ReluGrad's own — a device's decisions at the
    gradient's discontinuities (tests/parity_util.py device_branches)."""
    last = layers[-1]
    dx = dflat.reshape(last['yp'].shape if last['pool'] else last['y'].shape)
    for li in range(len(layers) - 1, -1, -1):
        L = layers[li]
        br = None if branches is None else branches.get(L['name'])
        if L['pool']:
            if br is not None:  # act' of the routed (max) position = act' of the pooled value
                dx = dx * branch_factor(br, act, alpha, dtype)
            dx = maxpool2_bwd(L['y'], L['yp'], dx, None if routes is None else routes.get(L['name']))
            dy = dx if br is not None else dx * act_bwd(L['y'], act, alpha)
        else:
            dy = dx * (branch_factor(br, act, alpha, dtype) if br is not None else act_bwd(L['y'], act, alpha))
        cols, _ = im2col(L['x'], L['k'], L['s'], L['pad'])
        dy2 = dy.reshape(-1, L['cout'])
        name = L['name']
        W = P['Network/%s/%s_weights' % (name, name)].astype(dtype)
        for key, val in (('Network/%s/%s_weights' % (name, name), (cols.T @ dy2).reshape(W.shape)),
                         ('Network/%s/%s_biases' % (name, name), dy2.sum(0))):
            G[key] = G[key] + val if key in G else val
        if li > 0:
            dcols = dy2 @ W.reshape(-1, L['cout']).T
            dx = col2im(dcols, L['x'].shape, L['k'], L['s'], L['pad'])


def heads_forward(spec, P, flat, act='relu', alpha=0.1, temp=1.0, dtype=np.float64):
    """[LSTM cell over the 5 window positions] + dense layer + the three heads, from the trunk
    features flat ([B, flat]; LSTM: [B*5, flat], window-major). Returns (v, pi, rep, cache)."""
    cache = dict(flat=flat)
    fc_in = flat
    if spec.get('lstm'):
        fc_in, cache['lstm'] = lstm_forward(spec, P, flat, dtype)
    fc = spec['fc'][0]
    Wf = P['Network/%s/%s_weights' % (fc, fc)].astype(dtype)
    bf = P['Network/%s/%s_biases' % (fc, fc)].astype(dtype)
    hz = fc_in @ Wf + bf
    h = act_fwd(hz, act, alpha)
    cache.update(fc_in=fc_in, h=h, hz=hz)
    Wc = P['Training/Critic/critic_output/critic_output_weights'].astype(dtype)
    bc = P['Training/Critic/critic_output/critic_output_biases'].astype(dtype)
    Wa = P['Training/Actor/actor_output/actor_output_weights'].astype(dtype)
    ba = P['Training/Actor/actor_output/actor_output_biases'].astype(dtype)
    Wr = P['Training/Repetition/repetition_output/repetition_output_weights'].astype(dtype)
    br = P['Training/Repetition/repetition_output/repetition_output_biases'].astype(dtype)
    v = (h @ Wc + bc).reshape(-1)                       # policy_v_network.py:22-23
    pi = softmax((h @ Wa + ba) / dtype(temp))           # :31, networks.py:97
    rep = softmax((h @ Wr + br) / dtype(temp))          # :47
    return v, pi, rep, cache


def forward(spec, P, obs, act='relu', alpha=0.1, temp=1.0, dtype=np.float64):
    """P: dict name -> array. obs uint8 [B,84,84,C] (LSTM: [B,5,84,84,C], the memory window of
    paac.py:79-83). Returns (v, pi, rep, cache)."""
    if spec.get('lstm'):
        obs = obs.reshape((-1,) + obs.shape[2:])
    flat, layers = trunk_forward(spec, P, obs, act, alpha, dtype)
    v, pi, rep, cache = heads_forward(spec, P, flat, act, alpha, temp, dtype)
    cache['layers'] = layers
    return v, pi, rep, cache


def heads_loss_and_grads(spec, P, v, pi, rep, c, a_idx, r_idx, y, adv, beta, act='relu', alpha=0.1, temp=1.0,
                         dtype=np.float64, hbranch=None):
    """Loss of policy_v_network.py:25-74 from heads_forward's outputs; gradients of the head,
    dense [and LSTM] variables into a new dict G. Returns (loss, G, dflat, aux)."""
    B = len(v)
    y = np.asarray(y, dtype)
    adv = np.asarray(adv, dtype)
    eps = dtype(1e-30)
    lpi = np.log(pi + eps)
    lrep = np.log(rep + eps)
    ent_pi = -(pi * lpi).sum(1)
    ent_rep = -(rep * lrep).sum(1)
    sel_pi = lpi[np.arange(B), a_idx]
    sel_rep = lrep[np.arange(B), r_idx]
    actor_obj = (sel_pi + sel_rep) * adv + beta * (ent_pi + ent_rep)
    critic = 0.25 * (y - v) ** 2
    loss = 5.0 * (np.mean(-actor_obj) + np.mean(critic))
    scale = 5.0 / B
    # critic
    dv = scale * 0.5 * (v - y)
    # softmax heads: dL/dp then the softmax Jacobian, then / temp
    def head_grad(p, lp, sel):
        oh = np.zeros_like(p)
        oh[np.arange(B), sel] = 1.0
        pe = p + eps
        dobj = oh * (adv[:, None] / pe) - beta * (lp + p / pe)
        g = -scale * dobj
        dz = p * (g - (p * g).sum(1, keepdims=True))
        return dz / temp
    dza = head_grad(pi, lpi, a_idx)
    dzr = head_grad(rep, lrep, r_idx)
    h = c['h']
    G = {}
    G['Training/Critic/critic_output/critic_output_weights'] = h.T @ dv[:, None]
    G['Training/Critic/critic_output/critic_output_biases'] = dv.sum(keepdims=True)
    G['Training/Actor/actor_output/actor_output_weights'] = h.T @ dza
    G['Training/Actor/actor_output/actor_output_biases'] = dza.sum(0)
    G['Training/Repetition/repetition_output/repetition_output_weights'] = h.T @ dzr
    G['Training/Repetition/repetition_output/repetition_output_biases'] = dzr.sum(0)
    Wc = P['Training/Critic/critic_output/critic_output_weights'].astype(dtype)
    Wa = P['Training/Actor/actor_output/actor_output_weights'].astype(dtype)
    Wr = P['Training/Repetition/repetition_output/repetition_output_weights'].astype(dtype)
    dh = (dv[:, None] @ Wc.T + dza @ Wa.T + dzr @ Wr.T) * (
        act_bwd(h, act, alpha) if hbranch is None else branch_factor(hbranch, act, alpha, dtype))
    fc = spec['fc'][0]
    Wf = P['Network/%s/%s_weights' % (fc, fc)].astype(dtype)
    G['Network/%s/%s_weights' % (fc, fc)] = c['fc_in'].T @ dh
    G['Network/%s/%s_biases' % (fc, fc)] = dh.sum(0)
    dflat = dh @ Wf.T
    if spec.get('lstm'):
        dflat = lstm_backward(spec, P, c['lstm'], dflat, dtype, G)
    terms = np.stack([critic, -((sel_pi + sel_rep) * adv), ent_pi, ent_rep], axis=1)
    return loss, G, dflat, dict(v=v, pi=pi, rep=rep, terms=terms)


def loss_and_grads(spec, P, obs, a_idx, r_idx, y, adv, beta, act='relu', alpha=0.1, temp=1.0,
                   dtype=np.float64, routes=None, branches=None, hbranch=None):
    """Loss of policy_v_network.py:25-74 and its gradient for every variable (dict)."""
    v, pi, rep, c = forward(spec, P, obs, act, alpha, temp, dtype)
    loss, G, dflat, aux = heads_loss_and_grads(spec, P, v, pi, rep, c, a_idx, r_idx, y, adv, beta, act, alpha,
                                               temp, dtype, hbranch)
    trunk_backward(spec, P, c['layers'], dflat, G, act, alpha, dtype, routes, branches)
    return loss, G, aux


def window_frames_loss_and_grads(spec, P, frames, win, a_idx, r_idx, y, adv, beta, act='relu', alpha=0.1,
                                 temp=1.0, dtype=np.float64, chunk=32, routes=None, branches=None, hbranch=None):
    """loss_and_grads of LSTM windows given as indices into distinct frames: window b's position k
    is frames[win[b, k]] (the reference builds each window as an explicit [5][84][84][C] slice of
    whole_memory, paac.py:79-83, :233-234; zeroed positions after an episode end are a zero frame).
    Every distinct frame goes through the trunk once (forward in chunks, features gathered per
    window position), and the trunk gradient is that of each frame's summed feature gradient —
    the same sums, by linearity, as the explicit windows' loss_and_grads (tests/test_oracle_torch.py
    pins the two against each other). frames: uint8 [F,84,84,C]; win: int [B,5]."""
    F = len(frames)
    flat = np.concatenate([trunk_forward(spec, P, frames[c0:c0 + chunk], act, alpha, dtype)[0]
                           for c0 in range(0, F, chunk)])
    v, pi, rep, c = heads_forward(spec, P, flat[np.asarray(win).reshape(-1)], act, alpha, temp, dtype)
    loss, G, dflat_w, aux = heads_loss_and_grads(spec, P, v, pi, rep, c, a_idx, r_idx, y, adv, beta, act, alpha,
                                                 temp, dtype, hbranch)
    dflat = np.zeros_like(flat)
    np.add.at(dflat, np.asarray(win).reshape(-1), dflat_w)
    for c0 in range(0, F, chunk):
        _, layers = trunk_forward(spec, P, frames[c0:c0 + chunk], act, alpha, dtype)
        rt = None if routes is None else {k: r[c0:c0 + chunk] for k, r in routes.items()}
        bt = None if branches is None else {k: r[c0:c0 + chunk] for k, r in branches.items()}
        trunk_backward(spec, P, layers, dflat[c0:c0 + chunk], G, act, alpha, dtype, rt, bt)
    return loss, G, aux


def init_params(spec, seed):
    """U(-d, d) with the TF init bounds of networks.py:34-89, N(0, 1) where d < 0
    (networks.py:124-125) (the TF RNG stream itself is not reproducible without TF; parity is
    on the bounds)."""
    rs = np.random.RandomState(seed)
    return {n: (rs.uniform(-d, d, size=shape) if d >= 0 else rs.standard_normal(size=shape)).astype(np.float32)
            for (n, shape, d) in spec['vars']}
