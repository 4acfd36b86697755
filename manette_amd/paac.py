"""PAACLearner: the PAAC+FiGAR rollout/update loop (paac.py:15-301) on one MI355X per process.

train() = init_network; loop { rollout() (= step(t) for t in range(T)); update(); log; save_vars }; cleanup
(the reference has no step()/update(); these are the decomposition of paac.py:140-205 and
:219-256). Data stays in HBM: the (T+1, E, 84, 84, C) uint8 rollout state ring, values,
action/repetition indices, y/adv. Per macro-step only the sampled indices go device->host and
only the emulators' screens (or finished observations) + rewards go host->device.

Paths (args.runner):
  'native'  emulators stepped by libmanette_host threads (NativeRunners); their raw screens go
            H2D from one pinned staging buffer and mt_preprocess builds the stacks (A2).
  'python'  reference-contract Python emulators (Runners / EmulatorRunner processes); finished
            84x84xC observations go H2D.
Sampling (args.sampling): 'host' = the reference's numpy multinomial stream (parity mode),
'device' = mt_sample (perf mode, same distribution).
Data parallel: one process per GPU; env ids are offset by rank (rank r owns global envs
[r*ec, (r+1)*ec), the runners.py:17-18 split over ranks), each rank rolls out its own shard and
the flat gradient is summed by ONE all-reduce per update (RCCL behind the C ABI, mt_allreduce,
issued eagerly between the update's graph replays: _bucketed_update; manette_amd/comm.py); 1/world
is folded into mt_clip_rmsprop, so
clip + RMSProp see the global-batch mean gradient and the replicas stay identical. The device
draw hashes the global env id and global_step counts every env of the job (mh_book_set_shard),
so a W-rank run takes the same trajectory and LR schedule as one process owning all W*ec envs.
torch.distributed (gloo) is the control channel only: the RCCL unique id and, at start / resume,
rank 0's global_step.
"""
import logging
import os
import time

import numpy as np
import torch

from . import network as devnet
from .actor_learner import ActorLearner
from .bookkeeping import NativeBook
from .environment import COL_LUT, ROW_LUT
from .runners import NativeRunners, Runners
from .emulator_runner import EmulatorRunner


def merge_episode_records(parts):
    """Episode records (global_step, reward, length) of every rank, in the order one process owning
    every env would have finished them: by global step (each env's step is unique in a macro-step:
    global_step + env id + 1, paac.py:184), the rank order breaking no tie."""
    return sorted((int(g), float(r), int(n)) for part in parts for (g, r, n) in part)


class PAACLearner(ActorLearner):
    def __init__(self, network_creator, environment_creator, explo_policy, args):
        self.seed = int(getattr(args, 'seed', 0))
        super(PAACLearner, self).__init__(network_creator, environment_creator, explo_policy, args)
        self.workers = args.emulator_workers
        self.pin_threads = getattr(args, 'pin_threads', 'auto')
        self.total_repetitions = args.nb_choices
        self.lstm_bool = (args.arch == 'LSTM')
        self.tab_rep = explo_policy.tab_rep
        self.runner_kind = getattr(args, 'runner', 'native')
        self.sampling = getattr(args, 'sampling', 'host')
        # native runner screens: 'in_place' = the GPU reads them in the emulators' pinned bank (no
        # host copy); 'zero_copy' = staged rows read in place from pinned staging; 'copy' = staged
        # rows hipMemcpyAsync'd to HBM; 'pooled' = zero_copy with the frame-pool max taken by the
        # emulator threads (one staged screen per push); 'resized' = zero_copy of each push's final
        # 84x84 frame (pool + resize on the emulator threads, the GPU only stacks)
        self.staging = getattr(args, 'staging', 'resized')
        if self.staging not in ('in_place', 'zero_copy', 'copy', 'pooled', 'resized'):
            raise ValueError('staging must be in_place, zero_copy, copy, pooled or resized')
        # native step only: keep the GPU one macro-step ahead (MT_ROLLOUT_PIPELINED)
        self.pipeline = bool(getattr(args, 'pipeline', True))
        self.depth = 3 if getattr(args, 'rgb', False) else 1
        self.C = 4 * self.depth
        self.dist = torch.distributed.is_available() and torch.distributed.is_initialized()
        self.world = torch.distributed.get_world_size() if self.dist else 1
        self.rank = torch.distributed.get_rank() if self.dist else 0
        self.is_chief = self.rank == 0
        # global env id of env 0 (train.py: rank * ec); the device draw hashes global env ids
        self.env_offset = int(getattr(args, 'env_id_offset', self.rank * self.emulator_counts))
        self.comm_kind = getattr(args, 'comm', 'rccl')
        self.comm = None
        # the data-parallel update (bucketed all-reduce on a side stream between three update graphs,
        # norm partials after the all-reduce, the learner launching the update): world > 1, or forced
        # at world 1 (args.dp_force / MT_DP_FORCE=1), where the RCCL sum is the identity, so the
        # code the N-GPU run depends on runs, and is oracle-checked, on one GPU (tests/test_e2e_gpu.py)
        self.dp = self.world > 1 or bool(getattr(args, 'dp_force', False)) or os.environ.get('MT_DP_FORCE') == '1'
        self.grad_scale = 1.0 / self.world  # folded into clip + RMSProp: the all-reduced sum -> the mean
        if self.sampling == 'device' and getattr(args, 'egreedy', False):
            # the device draw is the multinomial of exploration_policy.py:108-116 only
            raise ValueError('--egreedy needs --sampling host (the device sampler draws multinomially)')
        self.dev = self.network.device
        E, T, C = self.emulator_counts, self.max_local_steps, self.C
        dev = self.dev
        if self.lstm_bool:
            # LSTM frame store (include/manette_hip.h, mt_lstm_*): row 0 = the zero frame, then
            # slots 0..T+4 of E states; slots 0..3 = the previous rollout's last 4 states, slot
            # 4 + t = self.states[t]. The reference's memory / whole_memory (paac.py:107-112,
            # :79-83, :202-203) become nz[t][e] = the window's leading zero frames.
            self.n_steps = 5
            self.fstore = torch.zeros(1 + (T + 5) * E, 84, 84, C, dtype=torch.uint8, device=dev)
            self.slots = self.fstore[1:].view(T + 5, E, 84, 84, C)
            self.states = self.slots[4:]
            self.nz_h = torch.zeros(T + 1, E, dtype=torch.int32, pin_memory=True)  # (Python step only)
            self.nz_d = torch.zeros(T + 1, E, dtype=torch.int32, device=dev)
            self._slots_tmp = torch.zeros(5, E, 84, 84, C, dtype=torch.uint8, device=dev) if T < 5 else None
        else:
            self.states = torch.zeros(T + 1, E, 84, 84, C, dtype=torch.uint8, device=dev)
        self.values = torch.zeros(T, E, dtype=torch.float32, device=dev)
        # [0] = action indices, [1] = repetition indices, each [T][E] (row t*E+e, paac.py:239)
        self.idx = torch.zeros(2, T, E, dtype=torch.int32, device=dev)
        self.a_idx = self.idx[0]
        self.r_idx = self.idx[1]
        self.y = torch.zeros(T, E, dtype=torch.float32, device=dev)
        self.adv = torch.zeros(T, E, dtype=torch.float32, device=dev)
        self.pi_roll = torch.zeros(E, self.num_actions, dtype=torch.float32, device=dev)
        self.rep_roll = torch.zeros(E, self.total_repetitions, dtype=torch.float32, device=dev)
        # per-step policy outputs: the train step reuses the rollout's forward (mt_forward_rows /
        # the LSTM frame store), the parameters being unchanged between a rollout and its update
        self.pi_all = torch.zeros(T + 1, E, self.num_actions, dtype=torch.float32, device=dev)
        self.rep_all = torch.zeros(T + 1, E, self.total_repetitions, dtype=torch.float32, device=dev)
        self.train_ws = None if self.lstm_bool else self.network.workspace(T * E, 'train')
        self.v_boot = torch.zeros(E, dtype=torch.float32, device=dev)
        self.loss_terms = torch.zeros(T * E, 4, dtype=torch.float32, device=dev)
        self.counters = torch.zeros(E, dtype=torch.int64, device=dev)
        pin = dict(pin_memory=True)
        self.rm_h = torch.zeros(2, T, E, dtype=torch.float32, **pin)
        # the returns kernel reads the rollout's clipped rewards / masks in place (no H2D copy)
        self.rm_h_dev = devnet.host_device_pointer(self.rm_h)
        self.rewards_h = self.rm_h[0]
        self.masks_h = self.rm_h[1]
        self.idx_h = torch.zeros(2, T, E, dtype=torch.int32, **pin)
        self.a_h = self.idx_h[0]
        self.r_h = self.idx_h[1]
        self.pi_h = torch.zeros(E, self.num_actions, dtype=torch.float32, **pin)
        self.rep_h = torch.zeros(E, self.total_repetitions, dtype=torch.float32, **pin)
        self.row_lut = torch.from_numpy(ROW_LUT.astype(np.int32)).to(dev)
        self.col_lut = torch.from_numpy(COL_LUT.astype(np.int32)).to(dev)
        self.event = torch.cuda.Event()
        self.book = NativeBook(E, self.num_actions, self.tab_rep)
        if self.world > 1:  # global_step counts every env of the job, as one process would
            self.book.set_shard(self.env_offset, E * self.world)
        self.native_step = None  # mt_rollout handle (native runner + device sampling)
        self.boot_in_rollout = False
        self.slot0_in_rollout = False
        self.runners = None
        self.placement = None    # host-thread plan of the native runner (_plan_threads)
        self.profile = None      # name -> [(start_event, end_event)] when profiling (bench.py)
        self.sample_seed = (self.seed * 1000003 + 1) & 0xffffffffffff  # rank-independent: rows are global
        # replay the update as hipGraph(s) from the second update on (native pipelined step)
        self.use_update_graph = bool(getattr(args, 'update_graph', True))
        self._graphs = None
        self._update_in_rollout = False  # mt_rollout_set_update(_dp) registered (_register_update)
        self._rollout_update = None  # 'all': the rollout launches the whole update; 'first': its first graph
        self._boot_ws = None  # the rollout's workspace whose bootstrap dense slabs the loss kernel finishes
        self._eager_updates = 0
        self._buckets = None  # data parallel: flat offset splitting the two all-reduce buckets
        self.summaries = None  # TensorBoard event files of the chief (manette_amd/summary.py)
        self._logged_episodes = 0

    # ------------------------------------------------------------------------------------------
    def _plan_threads(self):
        """This rank's host-thread placement (manette_amd/placement.py): the emulator worker count
        (capped when the node's cores are oversubscribed), their cpus and idle spin."""
        from . import placement
        lw = int(os.environ.get('LOCAL_WORLD_SIZE', '1'))
        lr = int(os.environ.get('LOCAL_RANK', '0'))
        mode = self.pin_threads
        if mode == 'off' or (mode == 'auto' and lw <= 1):  # (nothing placed: no topology reads)
            topo = dict(allowed=sorted(os.sched_getaffinity(0)), quota=placement.cgroup_cpu_limit())
        else:
            topo = placement.topology(lw)
        return placement.plan(self.workers, self.emulator_counts, min(lr, lw - 1), lw, mode=mode, **topo)

    def _start_runners(self):
        E, C = self.emulator_counts, self.C
        if self.runner_kind == 'native':
            from . import placement
            self.placement = self._plan_threads()
            self.workers = self.placement['ew_used']
            placement.apply_before_workers(self.placement)  # ('slice': the workers inherit the rank's cpus)
            bank = self.environment_creator.create_bank(0, E)
            self.bank = bank
            self.in_place = self.staging == 'in_place'
            self.pair_d = torch.zeros(2, E, dtype=torch.int32, device=self.dev)
            self.pair_h = torch.zeros(2, E, dtype=torch.int32, pin_memory=True)
            self.meta_d = torch.zeros(2, E, dtype=torch.int32, device=self.dev)
            self.off_d = self.meta_d[0]
            self.cnt_d = self.meta_d[1]
            if self.in_place:
                self.runners = NativeRunners(bank, self.workers, self.tab_rep)
                self.raw_d = None
                self.frames_d = torch.zeros(E, 8, dtype=torch.int32, device=self.dev)
                self.screens_dev = devnet.host_device_pointer(bank.screens_t)
                self.runners.reset_frames()
                self._upload_frames(self.states[0], self.states[0].clone())
            else:
                # only the 84 screen rows the nearest resize reads are staged (PCIe); zero_copy:
                # kernels read env e's pushes in place at staging slots 4e..
                fixed = self.sampling == 'device' and self.staging in ('zero_copy', 'pooled', 'resized')
                self.runners = NativeRunners(bank, self.workers, self.tab_rep, row_select=ROW_LUT,
                                             fixed_slots=fixed, pooled=self.staging == 'pooled',
                                             resized=self.staging == 'resized', col_lut=COL_LUT)
                self.stage_row_lut = torch.arange(84, dtype=torch.int32, device=self.dev)
                self.raw_d = torch.zeros(4 * E, self.runners.staging.shape[1], self.runners.frame_bytes,
                                         dtype=torch.uint8, device=self.dev)
                total = self.runners.reset()
                self._upload_pushes(total, self.states[0], self.states[0].clone())
            if self.placement['pinned'] or self.placement['sliced']:  # ('slice': no worker cpus, the spin only)
                self.runners.set_threads(self.placement['worker_cpus'], self.placement['spin_us'])
                placement.apply_main(self.placement)
            if self.sampling == 'device':
                self._make_native_step()
        else:
            emus = [self.environment_creator.create_environment(i) for i in range(E)]
            s0 = np.asarray([e.get_initial_state() for e in emus], dtype=np.uint8)
            variables = [s0, np.zeros(E, np.float32), np.zeros(E, np.float32), np.zeros(E, np.int32),
                         np.zeros(E, np.int32)]
            self.runners = Runners(self.tab_rep, EmulatorRunner, emus, self.workers, variables)
            self.runners.start()
            self.shared = self.runners.get_shared_variables()
            self.obs_h = torch.zeros(E, 84, 84, C, dtype=torch.uint8, pin_memory=True)
            self.obs_h.numpy()[...] = self.shared[0]
            self.states[0].copy_(self.obs_h, non_blocking=True)

    def _make_native_step(self):
        import ctypes as C
        from . import _lib
        net, r = self.network, self.runners
        E, T = self.emulator_counts, self.max_local_steps
        # LSTM: the frame store's workspace; each step's forward = its new frame rows + its E
        # windows (mt_lstm_step_forward), nz[t] derived on the device from the episode-end flags
        ws = net.lstm_workspace(E, T) if self.lstm_bool else net.workspace(E, 'rollout')
        p = lambda t: C.c_void_p(None if t is None else t.data_ptr())
        if self.in_place:
            flags, staging, frames, src_rows, rows = (_lib.MT_ROLLOUT_IN_PLACE, self.bank.screens_t, r.frames, 210,
                                                      self.row_lut)
        else:
            flags = _lib.MT_ROLLOUT_ZERO_COPY if self.staging in ('zero_copy', 'pooled', 'resized') else 0
            if self.staging == 'pooled':
                flags |= _lib.MT_ROLLOUT_POOLED
            if self.staging == 'resized':
                flags |= _lib.MT_ROLLOUT_RESIZED
            staging, frames, src_rows, rows = r.staging, None, r.src_rows, self.stage_row_lut
        self.sync_h = None
        # zero-copy modes: the heads kernel flags each env's pair as written (host polls, no event)
        self.ready_h = torch.zeros(self.emulator_counts, dtype=torch.int32, pin_memory=True) \
            if flags & (_lib.MT_ROLLOUT_ZERO_COPY | _lib.MT_ROLLOUT_IN_PLACE) else None
        if self.pipeline:
            if flags & (_lib.MT_ROLLOUT_ZERO_COPY | _lib.MT_ROLLOUT_IN_PLACE) == 0:
                raise ValueError('pipeline needs in_place, zero_copy or pooled staging')
            flags |= _lib.MT_ROLLOUT_PIPELINED
            self.sync_h = torch.zeros(2, dtype=torch.int32, pin_memory=True)
            # the bootstrap chain stops at the dense slabs; the update's loss kernel finishes V(s_T)
            # (mt_returns_loss_backward_boot). MT_BOOT_IN_LOSS=0: the chain runs its heads kernel.
            if not self.lstm_bool and os.environ.get('MT_BOOT_IN_LOSS', '1') != '0':
                flags |= _lib.MT_ROLLOUT_BOOT_SLABS
                self._boot_ws = ws
        self._bufs = _lib.mt_rollout_buffers(
            p(self.states), p(self.values), p(self.idx), p(self.pi_all), p(self.rep_all), p(ws), ws.numel(),
            p(self.counters), p(self.raw_d), src_rows, p(self.pair_d), p(self.pair_h), p(self.meta_d),
            p(rows), p(self.col_lut), p(self.idx_h), p(staging), p(r.push_meta), p(r.reward),
            p(r.over), p(self.rm_h), p(frames), p(self.sync_h), p(self.train_ws),
            0 if self.train_ws is None else self.train_ws.numel(),
            p(self.v_boot if self.pipeline else None), p(self.ready_h), flags, self.env_offset,
            p(self.nz_d if self.lstm_bool else None))
        h = C.c_void_p()
        _lib.check(_lib.hip().mt_rollout_create(net._h, self.emulator_counts, self.max_local_steps, r._h,
                                                self.book.handle, C.byref(self._bufs),
                                                C.c_uint64(self.sample_seed), C.byref(h)), 'mt_rollout_create')
        self.native_step = h
        self._over_dev = devnet.host_device_pointer(r.over) if self.lstm_bool else None
        self.boot_in_rollout = self.pipeline  # the last step's chain runs the bootstrap forward
        # the rollout's stacking forward (pipelined, resized staging; NIPS, gray NATURE) also carries
        # slot T over into slot 0 at the next step 0 (mt_rollout_step): the update does not copy it
        self.slot0_in_rollout = self.pipeline and self.staging == 'resized' and not self.lstm_bool and (
            self.network.arch == 'NIPS' or (self.network.arch == 'NATURE' and self.depth == 1))
        # the frame trunks' rollout steps stack in their conv1 launch (stack_conv1_kernel; slot 0 still
        # copied by the update)
        self.frame_stack_in_rollout = self.pipeline and self.staging == 'resized' and self.network.arch in ('PWYX', 'LSTM')
        self._gs = C.c_int64(0)

    def _upload_pushes(self, total, out, prev):
        """H2D of the compact staging (only the pushed screens), then mt_preprocess."""
        r = self.runners
        self.raw_d[:total].copy_(r.staging[:total], non_blocking=True)
        self.meta_d.copy_(r.push_meta, non_blocking=True)
        devnet.preprocess(self.raw_d, self.off_d, self.cnt_d, self.emulator_counts, self.depth,
                          self.stage_row_lut, self.col_lut, prev, out, src_rows=r.src_rows, pooled=r.pooled,
                          resized=r.resized)

    def _upload_frames(self, out, prev):
        """In-place mode: H2D of the frame indices + push counts (a few hundred bytes), then
        mt_preprocess_frames reads the screens in the pinned bank."""
        r = self.runners
        self.frames_d.copy_(r.frames, non_blocking=True)
        self.meta_d.copy_(r.push_meta, non_blocking=True)
        devnet.preprocess_frames(self.screens_dev, self.frames_d, self.cnt_d, self.emulator_counts, self.depth,
                                 self.row_lut, self.col_lut, prev, out)

    @staticmethod
    def _lib_ref(x):
        import ctypes as C
        return C.byref(x)

    def _mark(self, name):
        if self.profile is None:
            return None
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        self.profile.setdefault(name, []).append(ev)
        return ev[1]

    # ------------------------------------------------------------------------------------------
    def rollout(self):
        """The T macro-steps of one rollout (paac.py:140-205): one native call (mt_rollout_run)
        with the native step, else step(t) for t in 0..T-1."""
        if self.native_step is not None:
            from . import _lib
            self._gs.value = self.global_step
            _lib.check(_lib.hip().mt_rollout_run(self.native_step, devnet._ptr(self.network.params),
                                                 self._lib_ref(self._gs), devnet._stream()), 'mt_rollout_run')
            self.global_step = self._gs.value
            return
        for t in range(self.max_local_steps):
            self.step(t)

    def step(self, t):
        """One rollout macro-step (paac.py:140-205)."""
        net = self.network
        E = self.emulator_counts
        if self.native_step is not None:
            from . import _lib
            self._gs.value = self.global_step
            _lib.check(_lib.hip().mt_rollout_step(self.native_step, devnet._ptr(net.params), t,
                                                  self._lib_ref(self._gs), devnet._stream()), 'mt_rollout_step')
            self.global_step = self._gs.value
            return
        end = self._mark('rollout_forward')
        if self.lstm_bool:
            v, pi, rep = self._lstm_forward(t, self.values[t])
        else:
            v, pi, rep = net.forward_rows(self.states[t], E, self.train_ws, self.max_local_steps * E, t * E,
                                          out=(self.values[t], self.pi_all[t], self.rep_all[t]), ws_key='rollout')
        if end is not None:
            end.record()
        if self.sampling == 'device':
            devnet.sample(pi, rep, self.sample_seed, self.counters, self.a_idx[t], self.r_idx[t], row0=self.env_offset)
            self.a_h[t].copy_(self.a_idx[t], non_blocking=True)
            self.r_h[t].copy_(self.r_idx[t], non_blocking=True)
            self.event.record()
            self.event.synchronize()
            a = self.a_h[t].numpy()
            r = self.r_h[t].numpy()
        else:
            self.pi_h.copy_(pi, non_blocking=True)
            self.rep_h.copy_(rep, non_blocking=True)
            self.event.record()
            self.event.synchronize()
            a, r = self.explo_policy.choose_indices(self.pi_h.numpy(), self.rep_h.numpy())
            self.a_h[t].numpy()[...] = a
            self.r_h[t].numpy()[...] = r
            self.a_idx[t].copy_(self.a_h[t], non_blocking=True)
            self.r_idx[t].copy_(self.r_h[t], non_blocking=True)
        if self.runner_kind == 'native':
            if self.in_place:
                self.runners.step_frames(self.a_h[t], self.r_h[t])
                self._upload_frames(self.states[t + 1], self.states[t])
            else:
                total = self.runners.step(self.a_h[t], self.r_h[t])
                self._upload_pushes(total, self.states[t + 1], self.states[t])
            reward = self.runners.reward.numpy()
            over = self.runners.over.numpy()
        else:
            sh = self.shared
            sh[3][...] = a
            sh[4][...] = r
            self.runners.update_environments()
            self.runners.wait_updated()
            self.obs_h.numpy()[...] = sh[0]
            self.states[t + 1].copy_(self.obs_h, non_blocking=True)
            reward, over = sh[1], sh[2]
        self.global_step = self.book.step(self.global_step, a, r, reward, over,
                                          self.rewards_h[t].numpy(), self.masks_h[t].numpy())
        if self.lstm_bool:  # update_memory (shift in the new state) + episode-end reset (paac.py:173-174, :202-203)
            nz = self.nz_h.numpy()
            nz[t + 1] = np.where(self.masks_h[t].numpy() == 0, 5, np.maximum(nz[t] - 1, 0))

    def _lstm_forward(self, t, v_out):
        """Step t's new frames (step 0: the zero frame + slots 0..4 again, the parameters having
        changed) through trunk + cell x-product, then the recurrence of the E windows of step t."""
        E, T = self.emulator_counts, self.max_local_steps
        net = self.network
        if self.native_step is not None:  # nz lives on the device: nz[t] from nz[t-1] + step t-1's over flags
            return net.lstm_step_forward(self.fstore, t, E, T, self.nz_d, self._over_dev, out=(v_out, self.pi_all[t],
                                                                                              self.rep_all[t]))
        if t == 0:
            net.lstm_frames_forward(self.fstore, 0, 1 + 5 * E, E, T)
        else:
            net.lstm_frames_forward(self.fstore, 1 + (4 + t) * E, E, E, T)
        self.nz_d[t].copy_(self.nz_h[t], non_blocking=True)
        return net.lstm_windows_forward(self.nz_d[t], t, E, T, out=(v_out, self.pi_all[t], self.rep_all[t]))

    def update(self):
        """Bootstrap, n-step returns, fused loss backward, [all-reduce], clip + RMSProp
        (paac.py:219-256).

        Native pipelined step (non-LSTM): the device work of an update is a fixed sequence over
        fixed buffers (the LR is read from pinned host memory, the returns kernel reads the
        rollout's rewards / masks in place), so from the second update on it is replayed as one
        or two hipGraphs (mt_graph_*; split around the all_reduce when world > 1): one launch
        instead of a dozen, and no host launch gaps between the backward's kernels."""
        self.book.drain()
        lr = self.get_lr()
        if self._update_in_rollout:  # the rollout's last step stored lr and launched the update graph
            # the native step restates get_lr (actor_learner.py:132-136) in C++; the two must agree
            if np.float32(self._lr_word[0]) != np.float32(lr):
                raise RuntimeError('native LR schedule %r != get_lr() %r at global step %d'
                                   % (float(self._lr_word[0]), lr, self.global_step))
            if self._rollout_update == 'first':  # data parallel, Python communicator: the rollout
                self._bucketed_update(devnet._stream(), first_launched=True)  # launched graph 1 only
            return lr
        self.network.set_lr(lr)
        if self._graph_ok():
            if self._graphs is None and self._eager_updates >= 1:
                self._capture_update()
            if self._graphs is not None:
                s = devnet._stream()
                if self._buckets is not None and len(self._graphs) == 1:  # data parallel, one graph
                    self._launch_graph(self._graphs[0], s)
                    self._register_update()
                elif self._buckets is not None:  # data parallel, three graphs (see _capture_update)
                    self._bucketed_update(s)
                    self._register_update()
                elif len(self._graphs) > 1:  # backward | eager all-reduce | apply
                    self._launch_graph(self._graphs[0], s)
                    self.comm.allreduce(self.network.grad)
                    self._launch_graph(self._graphs[1], s)
                else:
                    self._launch_graph(self._graphs[0], s)
                    self._register_update()
                return lr
        self._eager_updates += 1
        self._update_backward()
        if self.dp:
            grad = self.network.grad
            if not self.lstm_bool and os.environ.get('MT_DP_BUCKETS', '1') != '0':
                # the captured update's two bucket sums, in its order: every size the graph will
                # replay has run (and connected its RCCL channels) before the capture
                off = self._dense_offset()
                self.comm.allreduce(grad[off:])
                self.comm.allreduce(grad[:off])
            else:
                self.comm.allreduce(grad)
        self._update_apply()
        return lr

    def _bucketed_update(self, s, first_launched=False):
        """Data-parallel update with the gradient all-reduced in two buckets on a side stream: the
        dense + head variables (the tail of the flat gradient, ~98 % of its bytes) as soon as the
        backward's second launch has written them, while the conv backward runs on the learner's
        stream, then the conv variables; clip + RMSProp wait for both. Every rollout kernel (the
        in-kernel waits) stays on the learner's stream; the side stream only ever runs the
        all-reduces, between the update's first launch and its apply. first_launched: the rollout's
        last macro-step already launched the first graph on this stream (mt_rollout_set_update), so
        the backward starts right behind the bootstrap chain, not after the return to Python."""
        cur = torch.cuda.current_stream()
        side, (e1, e2, e3) = self._ar_stream, self._ar_events
        g1, g2, g3 = self._graphs
        grad = self.network.grad
        if not first_launched:
            self._launch_graph(g1, s)         # loss + dense dX / dW + head dW (+ the first conv layer's)
        e1.record(cur)
        with torch.cuda.stream(side):
            side.wait_event(e1)
            self.comm.allreduce(grad[self._buckets:])
        self._launch_graph(g2, s)             # the rest of the conv backward (+ its slab sums)
        e2.record(cur)
        with torch.cuda.stream(side):
            side.wait_event(e2)
            self.comm.allreduce(grad[:self._buckets])
            e3.record(side)
        cur.wait_event(e3)
        self._launch_graph(g3, s)             # global-norm partials + clip + RMSProp

    def _graph_ok(self):
        return (self.use_update_graph and self.profile is None
                and self.native_step is not None and self.boot_in_rollout)

    def _update_backward(self):
        net = self.network
        E, T = self.emulator_counts, self.max_local_steps
        boot_done = self.boot_in_rollout and self.native_step is not None  # (queued behind the last step)
        if self.lstm_bool and not boot_done:
            self._lstm_forward(T, self.v_boot)
        elif not self.lstm_bool and not boot_done:
            net.forward(self.states[T], E, out=(self.v_boot, self.pi_roll, self.rep_roll), ws_key='rollout', infer=True)
        if self.lstm_bool:
            devnet.returns(self.rm_h_dev, self.rm_h_dev + 4 * T * E, self.values, self.v_boot, self.gamma, self.y,
                           self.adv)
            end = self._mark('train_pass')
            self.train_backward()
        else:
            # n-step scan (paac.py:219-231) inside the loss kernel: one launch fewer
            end = self._mark('train_pass')
            N = E * T
            net.returns_loss_backward(self.states[:T].reshape(N, 84, 84, self.C), T, E, self.pi_all[:T].reshape(N, -1),
                                      self.rep_all[:T].reshape(N, -1), self.values, self.idx[0].view(N),
                                      self.idx[1].view(N), self.rm_h_dev, self.rm_h_dev + 4 * T * E, self.v_boot,
                                      self.gamma, self.y, self.adv, loss_terms=self.loss_terms, ws_key='train',
                                      norm_partials=not self.dp, boot_ws=self._boot_ws if boot_done else None)
        if end is not None:
            end.record()

    def train_backward(self):
        """The train step of the last rollout (paac.py:233-256), backward only: its forward is the
        rollout's (same parameters, same rows / windows). Idempotent (bench.py times it alone)."""
        net = self.network
        E, T = self.emulator_counts, self.max_local_steps
        N = E * T
        if self.lstm_bool:
            # through each distinct frame once
            net.lstm_frames_backward(self.fstore, self.nz_d[:T], E, T, self.pi_all[:T], self.rep_all[:T],
                                     self.values, self.idx[0].view(N), self.idx[1].view(N), self.y.view(N),
                                     self.adv.view(N), loss_terms=self.loss_terms, norm_partials=not self.dp)
            return
        # the rollout's forwards already left every row's activations in the train workspace
        # (mt_forward_rows, row t*E + e as paac.py:236)
        obs = self.states[:T].reshape(N, 84, 84, self.C)
        self.network.loss_backward(obs, N, self.values.view(N), self.pi_all[:T].reshape(N, -1),
                                   self.rep_all[:T].reshape(N, -1), self.idx[0].view(N), self.idx[1].view(N),
                                   self.y.view(N), self.adv.view(N), loss_terms=self.loss_terms, ws_key='train')

    def _update_apply(self):
        T = self.max_local_steps
        self.network.apply_gradients(self.grad_scale, partials_ready=not self.dp)
        if self.lstm_bool:  # the next rollout's slots 0..4 = s_{T-4} .. s_T; windows carry over
            if T >= 5:
                self.slots[0:5].copy_(self.slots[T:T + 5])
            else:  # overlapping ranges: through a fixed buffer (graph-capturable, no allocation)
                self._slots_tmp.copy_(self.slots[T:T + 5])
                self.slots[0:5].copy_(self._slots_tmp)
            if self.native_step is not None:
                self.nz_d[0].copy_(self.nz_d[T])
            else:
                self.nz_h.numpy()[0] = self.nz_h.numpy()[T]
        elif not (self.native_step is not None and self.slot0_in_rollout):
            self.states[0].copy_(self.states[T])

    def _capture_update(self):
        """Record the update's device work on a side stream (nothing executes while capturing)."""
        import ctypes as C
        from . import _lib
        lib = _lib.hip()
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        torch.cuda.synchronize()
        def whole():
            self._update_backward()
            self._update_apply()

        def capture(parts):
            graphs = []
            with torch.cuda.stream(side):
                sp = devnet._stream()
                for fn in parts:
                    _lib.check(lib.mt_graph_begin(sp), 'mt_graph_begin')
                    try:
                        fn()
                    finally:
                        g = C.c_void_p()
                        rc = lib.mt_graph_end(sp, C.byref(g))
                    if rc != 0:
                        for h in graphs:
                            lib.mt_graph_destroy(h)
                    _lib.check(rc, 'mt_graph_end')
                    graphs.append(g)
            return graphs

        def window(first, count, fn):
            def run():
                lib.mt_launch_window(first, count)
                try:
                    fn()
                finally:
                    lib.mt_launch_window(-1, -1)
            return run

        self._buckets = None
        if not self.dp:  # one graph; the rollout's last step launches it (_register_update)
            graphs = capture([whole])
        elif not self.lstm_bool and os.environ.get('MT_DP_BUCKETS', '1') != '0':
            # data parallel: the backward's first launches, up to the one that completes the dense /
            # head gradients (mt_net_backward_bucket_launches), then the rest (the conv backward); the
            # all-reduce of each gradient bucket runs on the all-reduce stream as soon as its launches
            # are done, beside the conv backward, and the apply waits for both
            n_tail = C.c_int()
            _lib.check(lib.mt_net_backward_bucket_launches(self.network._h, C.byref(n_tail)),
                       'mt_net_backward_bucket_launches')
            k = n_tail.value
            self._buckets = self._dense_offset()
            self._ar_stream = torch.cuda.Stream()
            self._ar_events = tuple(torch.cuda.Event() for _ in range(3))
            graphs = None
            if getattr(self.comm, 'capturable', False) and os.environ.get('MT_DP_ONE_GRAPH', '1') != '0':
                # a C-ABI communicator: the whole sequence as ONE graph, the all-reduce stream forked and
                # joined by events inside the capture (no host enqueue between its parts: at world 1
                # the eager form's RCCL calls and event hops left ~18 + 28 us device gaps, profiles/r05f)
                try:
                    graphs = capture([lambda: self._dp_sequence(window(0, k, self._update_backward),
                                                                window(k, -1, self._update_backward))])
                except _lib.MTError as e:
                    logging.warning('data-parallel update not capturable as one graph (%s): three graphs', e)
                    graphs = None
            if graphs is None:  # three graphs, the all-reduces issued between their replays
                graphs = capture([window(0, k, self._update_backward), window(k, -1, self._update_backward),
                                  self._update_apply])
        else:  # backward | all-reduce of the whole gradient | apply (LSTM, or MT_DP_BUCKETS=0)
            graphs = None
            if getattr(self.comm, 'capturable', False) and os.environ.get('MT_DP_ONE_GRAPH', '1') != '0':
                def one():  # a C-ABI communicator: the sum captured between the two (one graph)
                    self._update_backward()
                    self.comm.allreduce(self.network.grad)
                    self._update_apply()
                try:
                    graphs = capture([one])
                except _lib.MTError as e:
                    logging.warning('data-parallel update not capturable as one graph (%s): two graphs', e)
                    graphs = None
            if graphs is None:
                graphs = capture([self._update_backward, self._update_apply])
        self._graphs = graphs
        self._graph_stream = side  # keep the capture stream alive with the graphs

    def _dp_sequence(self, first, rest):
        """The bucketed data-parallel update as stream work (captured into one graph): first() = the
        backward's launches up to the dense / head gradients, rest() = the conv backward. Each bucket's
        in-place sum runs on the all-reduce stream behind an event as soon as its gradients are
        complete; the apply (norm partials, clip + RMSProp) waits for both."""
        cap = torch.cuda.current_stream()
        ar, (e1, e2, e3) = self._ar_stream, self._ar_events
        grad = self.network.grad
        first()
        e1.record(cap)
        ar.wait_event(e1)
        with torch.cuda.stream(ar):
            self.comm.allreduce(grad[self._buckets:])  # dense + head bucket, beside the conv backward
        rest()
        e2.record(cap)
        ar.wait_event(e2)
        with torch.cuda.stream(ar):
            self.comm.allreduce(grad[:self._buckets])  # conv bucket
            e3.record(ar)
        cap.wait_event(e3)
        self._update_apply()

    def _dense_offset(self):
        """Flat-gradient offset of the first non-conv variable (the dense layer): variables are in
        TF creation order, the convs first (networks.py:178-278), so [0, off) is the conv bucket and
        [off, n) the dense + head bucket."""
        return min(off for name, _, off, _ in self.network.vars if '/conv' not in name)

    @staticmethod
    def _launch_graph(g, s):
        from . import _lib
        _lib.check(_lib.hip().mt_graph_launch(g, s), 'mt_graph_launch')

    def _register_update(self):
        """From the next rollout on, its last macro-step stores the LR and launches the update itself,
        right behind the bootstrap chain: no host round trip between the last emulator step and
        the update. Single process: the one update graph (mt_rollout_set_update). Data parallel
        (bucketed) with a C-ABI communicator (RCCL): the one graph of _dp_sequence (all-reduces
        forked / joined inside it), or if that could not be captured the three graphs with the
        buckets' all-reduces on the rollout's side stream between them (mt_rollout_set_update_dp);
        with a Python communicator (gloo rehearsals, test stubs) the rollout launches the first
        graph and the learner the rest (_bucketed_update). MT_UPDATE_IN_ROLLOUT=0: off."""
        if os.environ.get('MT_UPDATE_IN_ROLLOUT', '1') == '0' or self.native_step is None or self.lstm_bool \
                or (self.dp and self._buckets is None):
            # (LSTM: its update also moves the frame-store slots the next rollout starts from; the
            # unbucketed data-parallel update: backward | all-reduce | apply, launched by the learner)
            return
        import ctypes as C
        from . import _lib
        lib = _lib.hip()
        lr_ptr = self.network._lr_host.data_ptr()
        if len(self._graphs) == 1:  # the single-process update, or the data-parallel one as one graph
            self._rollout_update = 'all'
        elif getattr(self.comm, '_h', None) is not None:  # three graphs, a C-ABI communicator
            self._rollout_update = 'all'
            gs = (C.c_void_p * 3)(*[g.value if isinstance(g, C.c_void_p) else g for g in self._graphs])
            grad = self.network.grad
            _lib.check(lib.mt_rollout_set_update_dp(self.native_step, gs, self.comm._h, C.c_void_p(grad.data_ptr()),
                                                    grad.numel(), int(self._buckets), C.c_void_p(lr_ptr),
                                                    float(self.initial_lr), float(self.lr_annealing_steps)),
                       'mt_rollout_set_update_dp')
        else:  # three graphs, a Python communicator: the rollout launches the first
            self._rollout_update = 'first'
        if self._rollout_update == 'first' or len(self._graphs) == 1:
            _lib.check(lib.mt_rollout_set_update(self.native_step, self._graphs[0], lr_ptr,
                                                 float(self.initial_lr), float(self.lr_annealing_steps)),
                       'mt_rollout_set_update')
        self._lr_word = self.network._lr_host.numpy()  # (the pinned word the rollout writes)
        self._update_in_rollout = True

    def _destroy_graphs(self):
        if self._update_in_rollout and self.native_step is not None:
            from . import _lib
            _lib.hip().mt_rollout_set_update(self.native_step, None, None, 0.0, 1.0)
            _lib.hip().mt_rollout_set_update_dp(self.native_step, None, None, None, 0, 0, None, 0.0, 1.0)
        self._update_in_rollout = False
        if getattr(self, '_graphs', None):
            from . import _lib
            for g in self._graphs:
                _lib.hip().mt_graph_destroy(g)
        self._graphs = None

    def loss_value(self):
        """5*(mean(-(adv*logp + beta*H)) + mean(0.25(y-v)^2)) of the last update (host sync)."""
        t = self.loss_terms.double().mean(0).cpu().numpy()
        beta = self.network.beta
        return float(5.0 * (t[0] + t[1] - beta * (t[2] + t[3])))

    # ------------------------------------------------------------------------------------------
    def start(self):
        self.global_step = self.init_network()
        if self.dp:
            from . import comm
            self.comm = comm.make(self.comm_kind, self.rank, self.world, torch.cuda.current_device())
        if self.world > 1:
            # rank 0's run is the run: its checkpoint step (resume) and its parameters / slots
            # (bounded: the first collectives on the communicator, comm.Deadline)
            with comm.Deadline('start-of-run broadcast of rank 0\'s parameters', self.rank, self.world):
                self.global_step, self.last_saving_step = comm.broadcast_scalars(
                    [self.global_step, self.last_saving_step], self.rank)
                for t in (self.network.params, self.network.ms, self.network.mom):
                    self.comm.broadcast(t, 0)
                torch.cuda.current_stream().synchronize()
        self.global_step_start = self.global_step
        self._start_runners()
        if self.lstm_bool:  # memory = zeros except memory[:, -1] = initial state (paac.py:109-112)
            self.nz_h.numpy()[0] = 4
            self.nz_d[0].fill_(4)

    def write_summaries(self):
        """The reference's TensorBoard scalars of the last rollout + update (chief only):
        rl/reward and rl/episode_length per finished episode (paac.py:191-199), then
        rewards_per_episode/* and steps_per_episode/* (paac.py:65-77, :265-266).
        Data parallel: the episodes of every rank (the union's, as one process owning every env
        would log them) are gathered to the chief over the control channel at the reference's
        logging interval (2048 / ec updates, paac.py:277-285) — a per-update gather would cost more
        than the update — and the episode statistics are written when the gathered span crossed a
        multiple of 500 global steps (the reference tests global_step % 500 == 0 per update)."""
        if self.world > 1:
            return self._write_summaries_dp()
        if self.summaries is None:
            if not self.is_chief:
                return
            from .summary import LearnerSummaries
            self.summaries = LearnerSummaries(self.debugging_folder)
        self.book.drain()
        eps = self.book.episodes
        self.summaries.episodes(eps[self._logged_episodes:])
        self._logged_episodes = len(eps)
        self.summaries.log_values(self.book.total_rewards, 'rewards_per_episode', self.global_step)
        self.summaries.log_values(self.book.total_steps, 'steps_per_episode', self.global_step)
        self.summaries.flush()

    def _write_summaries_dp(self, interval=None, final=False):
        """final: the gather of the episodes finished since the last one (train()'s normal exit, every
        rank), so no episode of the run is left unlogged."""
        self._summary_calls = getattr(self, '_summary_calls', 0) + 1
        # the reference's interval counts updates of the whole job: 2048 / (global emulator count)
        interval = interval or max(1, 2048 // (self.emulator_counts * self.world))
        if not final and self._summary_calls % interval != 0:
            return
        self.book.drain()
        mine = [tuple(e) for e in self.book.episodes[self._logged_episodes:]]
        self._logged_episodes = len(self.book.episodes)
        parts = [None] * self.world
        torch.distributed.all_gather_object(parts, mine)
        if not self.is_chief:
            return
        if self.summaries is None:
            from .summary import LearnerSummaries
            self.summaries = LearnerSummaries(self.debugging_folder)
            self._union_rewards, self._union_steps, self._summary_step = [], [], self.global_step_start
        merged = merge_episode_records(parts)
        self.summaries.episodes(merged)
        self._union_rewards.extend(r for _, r, _ in merged)
        self._union_steps.extend(int(n) for _, _, n in merged)
        crossed = self.global_step // 500 > self._summary_step // 500
        self._summary_step = self.global_step
        if crossed:
            self.summaries.log_values(self._union_rewards, 'rewards_per_episode', self.global_step, timestep=1)
            self.summaries.log_values(self._union_steps, 'steps_per_episode', self.global_step, timestep=1)
        self.summaries.flush()

    def train(self):
        """Main actor learner loop (paac.py:86-297)."""
        self.start()
        counter = 0
        start_time = time.time()
        logging.debug('Starting training at Step %d', self.global_step)
        try:
            while self.global_step < self.max_global_steps:
                loop_start_time = time.time()
                self.book.new_update()
                if counter == 0 and self.world > 1:  # the first all-reduce, bounded (comm.Deadline)
                    from . import comm
                    with comm.Deadline('the first data-parallel update', self.rank, self.world):
                        self.rollout()
                        self.update()
                        torch.cuda.synchronize()
                else:
                    self.rollout()
                    self.update()
                self.write_summaries()
                counter += 1
                if counter % max(1, 2048 // self.emulator_counts) == 0:
                    torch.cuda.synchronize()
                    now = time.time()
                    tr = self.book.total_rewards
                    last_ten = 0.0 if len(tr) < 1 else float(np.mean(tr[-10:]))
                    steps_per_sec = self.max_local_steps * self.emulator_counts / (now - loop_start_time)
                    avg = (self.global_step - self.global_step_start) / (now - start_time)
                    logging.info('Ran %d steps, at %f steps/s (%f steps/s avg), last 10 rewards avg %f',
                                 self.global_step, steps_per_sec, avg, last_ten)
                self.save_vars()
            if self.world > 1:  # (every rank: a collective) the episodes since the last gather
                self._write_summaries_dp(final=True)
        finally:
            self.cleanup()

    def cleanup(self):
        try:
            torch.cuda.synchronize()
            self._destroy_graphs()
            super(PAACLearner, self).cleanup()
        finally:
            if self.native_step is not None:
                from . import _lib
                _lib.hip().mt_rollout_destroy(self.native_step)
                self.native_step = None
            if self.runners is not None:
                self.runners.stop()
                self.runners = None
            if self.comm is not None:
                self.comm.close()
                self.comm = None
            if self.summaries is not None:
                self.summaries.close()
                self.summaries = None
