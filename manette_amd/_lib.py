"""ctypes bindings of the two C-ABI libraries (include/manette_hip.h, include/manette_host.h).

The HIP library is the only compute path: if it is missing or fails to load, every device
call raises (there is no CPU fallback in the product).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
HIP_LIB = os.environ.get('MANETTE_HIP_LIB') or os.path.join(HERE, 'libmanette_hip.so')  # variant override
HOST_LIB = os.path.join(HERE, 'libmanette_host.so')

MT_ARCH = {'NIPS': 0, 'NATURE': 1, 'PWYX': 2, 'LSTM': 3}
MT_ACT = {'relu': 0, 'leaky_relu': 1}
MT_CLIP = {'ignore': 0, 'global': 1}
MT_NORM_PARTIALS = 512
MT_COMM_UID_BYTES = 128


class MTError(RuntimeError):
    pass


class mt_rollout_buffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ('states', 'values', 'idx', 'pi', 'rep', 'ws')] + \
               [('ws_bytes', C.c_size_t)] + \
               [(n, C.c_void_p) for n in ('counters', 'raw')] + [('src_rows', C.c_int32)] + \
               [(n, C.c_void_p) for n in ('pair', 'pair_host', 'meta', 'row_lut', 'col_lut', 'idx_host',
                                          'staging_host', 'meta_host', 'reward_host', 'over_host',
                                          'rm_host', 'frames_host', 'sync_host', 'train_ws')] + \
               [('train_ws_bytes', C.c_size_t), ('v_boot', C.c_void_p), ('ready_host', C.c_void_p), ('flags', C.c_int32),
                                                                       ('env_offset', C.c_int32), ('nz', C.c_void_p)]


MT_ROLLOUT_ZERO_COPY = 1
MT_ROLLOUT_IN_PLACE = 2
MT_ROLLOUT_POOLED = 4
MT_ROLLOUT_PIPELINED = 8
MT_ROLLOUT_RESIZED = 16
MT_ROLLOUT_BOOT_SLABS = 32
MH_RUNNER_RESIZED = 4
MH_RUNNER_FIXED_SLOTS = 1
MH_RUNNER_POOLED = 2


class mt_net_config(C.Structure):
    _fields_ = [('arch', C.c_int32), ('depth', C.c_int32), ('num_actions', C.c_int32),
                ('num_reps', C.c_int32), ('activation', C.c_int32), ('alpha_leaky', C.c_float),
                ('softmax_temp', C.c_float)]


_P = C.c_void_p
_I = C.c_int
_F = C.c_float
_SZ = C.c_size_t

_HIP_SIGS = {
    'mt_last_error': (C.c_char_p, []),
    'mt_version': (_I, []),
    'mt_launch_window': (_I, [_I, _I]),
    'mt_net_backward_bucket_launches': (_I, [_P, C.POINTER(_I)]),
    'mt_net_create': (_I, [C.POINTER(mt_net_config), C.POINTER(_P)]),
    'mt_net_destroy': (None, [_P]),
    'mt_net_num_params': (_I, [_P, C.POINTER(_SZ)]),
    'mt_net_num_vars': (_I, [_P, C.POINTER(_I)]),
    'mt_net_var_info': (_I, [_P, _I, C.c_char_p, _I, C.POINTER(C.c_int64), C.POINTER(_I),
                             C.POINTER(_SZ), C.POINTER(_F)]),
    'mt_net_feature_dim': (_I, [_P, C.POINTER(_I)]),
    'mt_net_workspace_bytes': (_I, [_P, _I, C.POINTER(_SZ)]),
    'mt_net_workspace_region': (_I, [_P, _I, _I, _I, _I, _I, C.POINTER(_SZ), C.POINTER(_SZ)]),
    'mt_forward': (_I, [_P, _P, _P, _I, _P, _SZ, _P, _P, _P, _P]),
    'mt_lstm_frames_workspace_bytes': (_I, [_P, _I, _I, C.POINTER(_SZ)]),
    'mt_lstm_frames_forward': (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _SZ, _P]),
    'mt_lstm_windows_forward': (_I, [_P, _P, _P, _I, _I, _I, _P, _SZ, _P, _P, _P, _P]),
    'mt_lstm_step_forward': (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P, _SZ, _P, _P, _P, _P]),
    'mt_lstm_frames_backward': (_I, [_P, _P, _P, _P, _I, _I, _P, _SZ, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P]),
    'mt_forward_rows': (_I, [_P, _P, _P, _I, _P, _SZ, _P, _SZ, _I, _I, _P, _P, _P, _P]),
    'mt_forward_trunk': (_I, [_P, _P, _P, _I, _P, _SZ, _P]),
    'mt_forward_trunk_stacking': (_I, [_P, _P, _P, _P, _P, C.c_uint32, _P, _I, _P, _SZ, _P, _P]),
    'mt_forward_infer': (_I, [_P, _P, _P, _I, _P, _SZ, _P, _P, _P, _P]),
    'mt_sample': (_I, [_P, _P, _I, _I, _I, C.c_uint64, _I, _P, _P, _P, _P, _P]),
    'mt_returns': (_I, [_P, _P, _P, _P, C.c_double, _I, _I, _P, _P, _P]),
    'mt_loss_backward': (_I, [_P, _P, _P, _I, _P, _SZ, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P]),
    'mt_returns_loss_backward': (_I, [_P, _P, _P, _I, _I, _P, _SZ, _P, _P, _P, _P, _P, _P, _P, _P, C.c_double, _P, _P,
                                      _F, _P, _P, _P, _P]),
    'mt_returns_loss_backward_boot': (_I, [_P, _P, _P, _I, _I, _P, _SZ, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P,
                                           C.c_double, _P, _P, _F, _P, _P, _P, _P]),
    'mt_grad_sumsq': (_I, [_P, _SZ, _F, _P, _P]),
    'mt_clip_rmsprop': (_I, [_P, _P, _P, _P, _SZ, _P, _P, _F, _F, _F, _F, _I, _F, _P, _P]),
    'mt_preprocess': (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P]),
    'mt_preprocess_pooled': (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P]),
    'mt_preprocess_resized': (_I, [_P, _P, _P, _I, _I, _P, _P, _P]),
    'mt_preprocess_frames': (_I, [_P, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    'mt_memory_push': (_I, [_P, _P, _P, _P, _I, _SZ, _P]),
    'mt_host_device_pointer': (_I, [_P, C.POINTER(_P)]),
    'mt_sum_slabs': (_I, [_P, _I, _SZ, _P, _P]),
    'mt_net_get_config': (_I, [_P, C.POINTER(mt_net_config)]),
    'mt_rollout_create': (_I, [_P, _I, _I, _P, _P, C.POINTER(mt_rollout_buffers), C.c_uint64, C.POINTER(_P)]),
    'mt_rollout_destroy': (None, [_P]),
    'mt_rollout_step': (_I, [_P, _P, _I, C.POINTER(C.c_int64), _P]),
    'mt_rollout_run': (_I, [_P, _P, C.POINTER(C.c_int64), _P]),
    'mt_rollout_stats': (_I, [_P, C.POINTER(C.c_double), _I]),
    'mt_rollout_stats_ex': (_I, [_P, _P, _I, _I]),
    'mt_rollout_host_trace': (_I, [_P, _P, _I, _P]),
    'mt_rollout_trunk_timing': (_I, [_P, _I, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    'mt_rollout_set_update': (_I, [_P, _P, _P, C.c_double, C.c_double]),
    'mt_rollout_update_form': (_I, [_P, C.POINTER(_I)]),
    'mt_rollout_set_update_dp': (_I, [_P, _P, _P, _P, _SZ, _SZ, _P, C.c_double, C.c_double]),
    'mt_comm_unique_id': (_I, [C.c_char_p]),
    'mt_comm_init': (_I, [C.c_char_p, _I, _I, _I, C.POINTER(_P)]),
    'mt_comm_init_loopback': (_I, [_I, _I, C.POINTER(_P)]),
    'mt_comm_destroy': (None, [_P]),
    'mt_comm_info': (_I, [_P, C.POINTER(_I), C.POINTER(_I)]),
    'mt_allreduce': (_I, [_P, _P, _SZ, _P]),
    'mt_broadcast': (_I, [_P, _P, _SZ, _I, _P]),
    'mt_graph_begin': (_I, [_P]),
    'mt_graph_end': (_I, [_P, C.POINTER(_P)]),
    'mt_graph_launch': (_I, [_P, _P]),
    'mt_graph_destroy': (_I, [_P]),
}

_HOST_SIGS = {
    'mh_last_error': (C.c_char_p, []),
    'mh_runner_create': (_I, [_I, _I, _P, _I, _P, _I, _SZ, _P, _I, _I, _P, _I, _I, C.POINTER(_P)]),
    'mh_runner_destroy': (None, [_P]),
    'mh_runner_reset': (_I, [_P, _P, _P, _P, C.POINTER(_I)]),
    'mh_runner_step': (_I, [_P, _P, _P, _P, _P, _P, _P, _P, C.POINTER(_I)]),
    'mh_runner_reset_frames': (_I, [_P, _P, _P]),
    'mh_runner_step_frames': (_I, [_P, _P, _P, _P, _P, _P, _P]),
    'mh_runner_env_state': (_I, [_P, _I, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    'mh_crc32c': (C.c_uint32, [_P, _SZ, C.c_uint32]),
    'mh_runner_set_col_lut': (_I, [_P, _P, _I]),
    'mh_runner_set_threads': (_I, [_P, _P, _I, _I]),
    'mh_runner_thread_cpus': (_I, [_P, _P, _I]),
    'mh_runner_stats': (_I, [_P, _P, _I, _I]),
    'mh_runner_set_ready': (_I, [_P, _P, C.c_uint32]),
    'mh_runner_step_begin': (_I, [_P, _P, _P, _P, _P, _P, _P, _P]),
    'mh_runner_step_end': (_I, [_P, C.POINTER(_I)]),
    'mh_book_create': (_I, [_I, _I, _P, _I, C.POINTER(_P)]),
    'mh_book_destroy': (None, [_P]),
    'mh_book_step': (_I, [_P, C.POINTER(C.c_int64), _P, _P, _P, _P, _P, _P]),
    'mh_book_new_update': (_I, [_P]),
    'mh_book_set_shard': (_I, [_P, C.c_int64, C.c_int64]),
    'mh_book_histogram': (_I, [_P, _P, C.POINTER(C.c_int64)]),
    'mh_book_pop_episodes': (_I, [_P, _P, _P, _P, _I, C.POINTER(_I)]),
}

_hip = None
_host = None


def _load(path, sigs):
    if not os.path.exists(path):
        raise MTError('%s is not built (run __graft_entry__.build() or python -m manette_amd.build)'
                      % path)
    lib = C.CDLL(path)
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def hip():
    global _hip
    if _hip is None:
        host()  # libmanette_hip.so links libmanette_host.so (rpath $ORIGIN)
        _hip = _load(HIP_LIB, _HIP_SIGS)
    return _hip


def host():
    global _host
    if _host is None:
        _host = _load(HOST_LIB, _HOST_SIGS)
    return _host


def check(rc, what='call'):
    if rc != 0:
        msg = hip().mt_last_error()
        raise MTError('%s failed (status %d): %s' % (what, rc, msg.decode() if msg else ''))


def check_host(rc, what='call'):
    if rc != 0:
        msg = host().mh_last_error()
        raise MTError('%s failed (status %d): %s' % (what, rc, msg.decode() if msg else ''))


def hip_symbols():
    return sorted(_HIP_SIGS)


def host_symbols():
    return sorted(_HOST_SIGS)
