// Native rollout macro-step: the per-step orchestration of paac.py:140-205 without Python.
// See include/manette_hip.h (mt_rollout_*). Host code + HIP runtime calls; the emulator threads
// and the bookkeeping live in libmanette_host.so (include/manette_host.h).
#include <chrono>

#include "common.h"
#include "../../include/manette_host.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct mt_rollout {
  const mt_net *net;
  int E, T, A, R, depth;
  size_t frame_bytes;
  mh_runner *runner;
  mh_book *book;
  mt_rollout_buffers b;
  uint64_t seed;
  hipEvent_t ev;
  bool zero_copy;
  uint8_t *staging_dev;  // device addresses of the host-mapped buffers (zero-copy mode)
  int32_t *meta_dev, *pair_dev;
  double acc[5];  // host wall us: launch+wait for indices, runner, book, upload+preprocess enqueue; steps
};

using namespace mt;

extern "C" int mt_rollout_create(const mt_net *net, int E, int T, void *runner, void *book,
                                 const mt_rollout_buffers *buffers, uint64_t seed,
                                 mt_rollout **out) {
  MT_CHECK_ARG(net && runner && book && buffers && out, "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  const mt_rollout_buffers &b = *buffers;
  const bool zc = (b.flags & MT_ROLLOUT_ZERO_COPY) != 0;
  MT_CHECK_ARG((b.flags & ~MT_ROLLOUT_ZERO_COPY) == 0, "unknown rollout flags %d", b.flags);
  MT_CHECK_ARG(b.states && b.values && b.idx && b.pi && b.rep && b.ws && b.counters &&
                   (zc || (b.raw && b.meta && b.pair)) && b.row_lut && b.col_lut && b.idx_host &&
                   b.staging_host && b.pair_host && b.src_rows >= 84 && b.src_rows <= 210 &&
                   b.meta_host && b.reward_host && b.over_host && b.rm_host,
               "null buffer");
  void *staging_dev = nullptr, *meta_dev = nullptr, *pair_dev = nullptr;
  if (zc) {  // the three buffers must be pinned + mapped (hipHostMalloc / torch pin_memory)
    MT_HIP(hipHostGetDevicePointer(&staging_dev, b.staging_host, 0));
    MT_HIP(hipHostGetDevicePointer(&meta_dev, b.meta_host, 0));
    MT_HIP(hipHostGetDevicePointer(&pair_dev, b.pair_host, 0));
  }
  mt_net_config cfg;
  MT_CHECK_ARG(mt_net_get_config(net, &cfg) == MT_OK, "bad net");
  size_t need = 0;
  if (mt_net_workspace_bytes(net, E, &need) != MT_OK) return MT_ERR_ARG;
  if (b.ws_bytes < need) {
    set_error("rollout workspace %zu < %zu bytes", b.ws_bytes, need);
    return MT_ERR_WORKSPACE;
  }
  mt_rollout *ro = new mt_rollout();
  ro->net = net;
  ro->E = E;
  ro->T = T;
  ro->A = cfg.num_actions;
  ro->R = cfg.num_reps;
  ro->depth = cfg.depth;
  ro->frame_bytes = (size_t)b.src_rows * 160 * cfg.depth;
  ro->runner = (mh_runner *)runner;
  ro->book = (mh_book *)book;
  ro->b = b;
  ro->seed = seed;
  ro->zero_copy = zc;
  ro->staging_dev = (uint8_t *)staging_dev;
  ro->meta_dev = (int32_t *)meta_dev;
  ro->pair_dev = (int32_t *)pair_dev;
  hipError_t e = hipEventCreateWithFlags(&ro->ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    delete ro;
    set_error("hipEventCreate: %s", hipGetErrorString(e));
    return MT_ERR_HIP;
  }
  *out = ro;
  return MT_OK;
}

extern "C" void mt_rollout_destroy(mt_rollout *ro) {
  if (!ro) return;
  (void)hipEventDestroy(ro->ev);
  delete ro;
}

#define MT_TRY_(x)                 \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != MT_OK) return rc_;  \
  } while (0)

extern "C" int mt_rollout_step(mt_rollout *ro, const float *params, int t, int64_t *global_step,
                               mt_stream_t stream) {
  MT_CHECK_ARG(ro && params && global_step, "null argument");
  MT_CHECK_ARG(t >= 0 && t < ro->T, "t=%d out of [0,%d)", t, ro->T);
  const mt_rollout_buffers &b = ro->b;
  hipStream_t s = (hipStream_t)stream;
  const int E = ro->E, T = ro->T;
  const double t0 = now_us();
  const size_t slot = (size_t)E * 84 * 84 * 4 * ro->depth;
  uint8_t *cur = b.states + (size_t)t * slot;
  uint8_t *nxt = cur + slot;
  int32_t *a_d = b.idx + (size_t)t * E, *r_d = b.idx + (size_t)T * E + (size_t)t * E;
  int32_t *a_h = b.idx_host + (size_t)t * E, *r_h = b.idx_host + (size_t)T * E + (size_t)t * E;
  // 1. policy/value forward + device sampling fused in its heads kernel (paac.py:144-147)
  const SampleArgs smp{ro->seed, b.counters, a_d, r_d, ro->zero_copy ? ro->pair_dev : b.pair};
  MT_TRY_(forward_sample(ro->net, params, cur, E, b.ws, b.ws_bytes, b.values + (size_t)t * E, b.pi,
                         b.rep, &smp, s));
  if (!ro->zero_copy)
    MT_HIP(hipMemcpyAsync(b.pair_host, b.pair, sizeof(int32_t) * 2 * E, hipMemcpyDeviceToHost, s));
  MT_HIP(hipEventRecord(ro->ev, s));
  // spin: a blocking wait sleeps past the ~50 us the chain takes and pays the wake-up latency
  hipError_t q;
  while ((q = hipEventQuery(ro->ev)) == hipErrorNotReady) __builtin_ia32_pause();
  MT_HIP(q);
  std::memcpy(a_h, b.pair_host, sizeof(int32_t) * E);
  std::memcpy(r_h, b.pair_host + E, sizeof(int32_t) * E);
  const double t1 = now_us();
  // 2. emulators (runners.py:44-50 / emulator_runner.py:24-41) + bookkeeping (paac.py:176-205)
  int total = 0;
  if (mh_runner_step(ro->runner, a_h, r_h, b.staging_host, b.meta_host, b.meta_host + E,
                     b.reward_host, b.over_host, &total) != 0) {
    set_error("mh_runner_step: %s", mh_last_error());
    return MT_ERR_ARG;
  }
  const double t2 = now_us();
  if (mh_book_step(ro->book, global_step, a_h, r_h, b.reward_host, b.over_host,
                   b.rm_host + (size_t)t * E, b.rm_host + (size_t)T * E + (size_t)t * E) != 0) {
    set_error("mh_book_step: %s", mh_last_error());
    return MT_ERR_ARG;
  }
  const double t3 = now_us();
  // 3. screens -> preprocess into slot t+1 (atari_emulator.py:79-124)
  const uint8_t *raw = ro->staging_dev;
  const int32_t *meta = ro->meta_dev;
  if (!ro->zero_copy) {
    MT_HIP(hipMemcpyAsync(b.raw, b.staging_host, (size_t)total * 2 * ro->frame_bytes,
                          hipMemcpyHostToDevice, s));
    MT_HIP(hipMemcpyAsync(b.meta, b.meta_host, sizeof(int32_t) * 2 * E, hipMemcpyHostToDevice, s));
    raw = b.raw;
    meta = b.meta;
  }
  const int rc = mt_preprocess(raw, meta, meta + E, E, ro->depth, b.src_rows, b.row_lut, b.col_lut,
                               cur, nxt, stream);
  const double t4 = now_us();
  ro->acc[0] += t1 - t0;
  ro->acc[1] += t2 - t1;
  ro->acc[2] += t3 - t2;
  ro->acc[3] += t4 - t3;
  ro->acc[4] += 1;
  return rc;
}

extern "C" int mt_rollout_stats(mt_rollout *ro, double *out5, int reset) {
  MT_CHECK_ARG(ro && out5, "null argument");
  for (int i = 0; i < 5; ++i) out5[i] = ro->acc[i];
  if (reset)
    for (int i = 0; i < 5; ++i) ro->acc[i] = 0;
  return MT_OK;
}
