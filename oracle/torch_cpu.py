"""torch-CPU fp32 network for the timed "port" CPU baseline (bench.py cpu_baseline leg).

The reference runs its graph with TF1's multi-threaded CPU kernels (Eigen/MKL conv); the numpy
restatement in oracle/nets.py is the parity checker but is not a fair speed stand-in, so the
baseline's learner uses torch's CPU conv/GEMM kernels on the same graph (networks.py:178-278,
policy_v_network.py:19-74) with the TF1 clip_by_global_norm + ApplyRMSProp update
(actor_learner.py:43-74). Same forward/train API as host_loop.OracleNetwork.
"""
import numpy as np
import torch
import torch.nn.functional as Fn

from . import nets


class TorchCPUNetwork(object):
    def __init__(self, arch, depth, num_actions, num_reps, seed=0, beta=0.02, clip=3.0, decay=0.99,
                 eps=0.1, threads=None):
        if threads:
            torch.set_num_threads(int(threads))
        self.spec = nets.arch_spec(arch, depth, num_actions, num_reps)
        P = nets.init_params(self.spec, seed)
        self.names = [n for (n, _, _) in self.spec['vars']]
        self.P = {k: torch.from_numpy(P[k]).requires_grad_(True) for k in self.names}
        self.ms = {k: torch.ones_like(v) for k, v in self.P.items()}
        self.mom = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.beta, self.clip, self.decay, self.eps = beta, clip, decay, eps

    def _forward(self, states):
        P = self.P
        lstm = self.spec.get('lstm')
        if lstm:  # memory windows [B, 5, 84, 84, C] -> 5B frames (networks.py:239-241)
            states = np.ascontiguousarray(states).reshape((-1,) + states.shape[2:])
        x = torch.from_numpy(np.ascontiguousarray(states)).permute(0, 3, 1, 2).float() * (1.0 / 255.0)
        for (name, k, s, cin, cout, pad, pool) in self.spec['convs']:
            W = P['Network/%s/%s_weights' % (name, name)].permute(3, 2, 0, 1)
            if pad == 'SAME':
                H = x.shape[2]
                O = -(-H // s)
                tot = max((O - 1) * s + k - H, 0)
                x = Fn.pad(x, (tot // 2, tot - tot // 2, tot // 2, tot - tot // 2))
            x = torch.relu(Fn.conv2d(x, W, P['Network/%s/%s_biases' % (name, name)], stride=s))
            if pool:
                x = Fn.max_pool2d(x, 2, 2)
        flat = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
        if lstm:  # BasicLSTMCell(32, forget_bias=1) x 5 + linear projection (networks.py:112-127)
            nh, S = lstm['hidden'], lstm['steps']
            X = flat.reshape(-1, S, flat.shape[1])
            K, kb = P['rnn/basic_lstm_cell/kernel'], P['rnn/basic_lstm_cell/bias']
            h = torch.zeros(X.shape[0], nh)
            c = torch.zeros(X.shape[0], nh)
            for t in range(S):
                z = torch.cat([X[:, t], h], 1) @ K + kb
                i, j, f, o = z.split(nh, 1)
                c = c * torch.sigmoid(f + lstm['forget_bias']) + torch.sigmoid(i) * torch.tanh(j)
                h = torch.tanh(c) * torch.sigmoid(o)
            flat = h @ P['Network/lstm/Variable'] + P['Network/lstm/Variable_1']
        fc = self.spec['fc'][0]
        h = torch.relu(flat @ P['Network/%s/%s_weights' % (fc, fc)] + P['Network/%s/%s_biases' % (fc, fc)])
        v = (h @ P['Training/Critic/critic_output/critic_output_weights'] +
             P['Training/Critic/critic_output/critic_output_biases']).reshape(-1)
        pi = torch.softmax(h @ P['Training/Actor/actor_output/actor_output_weights'] +
                           P['Training/Actor/actor_output/actor_output_biases'], 1)
        rep = torch.softmax(h @ P['Training/Repetition/repetition_output/repetition_output_weights'] +
                            P['Training/Repetition/repetition_output/repetition_output_biases'], 1)
        return v, pi, rep

    def forward(self, states, bootstrap=False):
        with torch.no_grad():
            v, pi, rep = self._forward(states)
        if bootstrap:
            return v.numpy()
        return v.numpy(), pi.numpy(), rep.numpy()

    def train(self, flat_states, y, adv, a_onehot, r_onehot, lr):
        v, pi, rep = self._forward(flat_states)
        B = v.shape[0]
        lpi = torch.log(pi + 1e-30)
        lrep = torch.log(rep + 1e-30)
        ent = -(pi * lpi).sum(1) - (rep * lrep).sum(1)
        a = torch.from_numpy(np.argmax(a_onehot, 1))
        r = torch.from_numpy(np.argmax(r_onehot, 1))
        sel = lpi[torch.arange(B), a] + lrep[torch.arange(B), r]
        advt = torch.from_numpy(np.asarray(adv, np.float32))
        yt = torch.from_numpy(np.asarray(y, np.float32))
        loss = 5.0 * (torch.mean(-(sel * advt + self.beta * ent)) + torch.mean(0.25 * (yt - v) ** 2))
        grads = torch.autograd.grad(loss, [self.P[k] for k in self.names])
        with torch.no_grad():
            norm = float(torch.sqrt(sum((g.double() ** 2).sum() for g in grads)))
            scale = np.float32(self.clip) * min(np.float32(1.0) / np.float32(norm), np.float32(1.0 / self.clip))
            for k, g in zip(self.names, grads):
                g = g * float(scale)
                ms, mom, w = self.ms[k], self.mom[k], self.P[k]
                ms += (g * g - ms) * (1.0 - self.decay)
                mom.copy_((g * lr) / torch.sqrt(ms + self.eps))
                w -= mom
