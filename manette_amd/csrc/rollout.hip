// Native rollout macro-step: the per-step orchestration of paac.py:140-205 without Python.
// See include/manette_hip.h (mt_rollout_*). Host code + HIP runtime calls; the emulator threads
// and the bookkeeping live in libmanette_host.so (include/manette_host.h).
#include <algorithm>
#include <chrono>
#include <vector>

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
  std::vector<hipEvent_t> ev;  // [T] pair of step t ready (recorded once per rollout: chains are armed
                               // up to T steps ahead)
  bool zero_copy, in_place, pooled, resized, pipelined;
  bool pull;          // pipelined + resized: per-env ready words, pull kernel into HBM, tagged pairs
  bool stack_fwd;     // pull + NIPS / gray NATURE: the forward's conv(1) kernel stacks (no preprocess launch)
  bool lstm_stack = false;     // pull + LSTM: each step's conv1 launch pulls + stacks (launch_stack_conv1)
  bool frame_stack = false;    // pull + PWYX: the same in the forward's trunk (ws counters)
  uint32_t *lstm_sync = nullptr;  // its env queue (stack_conv1_sync_words(E), zero between launches)
  bool lstm;          // LSTM arch: frame-store forward per step (mt_lstm_step_forward), nz on the device
  bool boot_slabs;    // MT_ROLLOUT_BOOT_SLABS: the bootstrap chain ends at the dense slabs (no heads)
  const uint8_t *fstore = nullptr;  // LSTM: the frame store (states = its slot 4)
  const float *over_dev = nullptr;  // LSTM: device address of the pinned episode-end flags
  int armed_upto = -1;  // pipelined: last step whose chain (forward) is already enqueued
  int ahead = 1;        // pipelined: steps armed ahead (T: every chain of the rollout at its step 0)
  std::vector<uint32_t> fwd_of;  // [T] draw sequence number of step t's forward
  uint32_t seq = 0;   // host step sequence word value last stored
  uint8_t *staging_dev;  // device addresses of the host-mapped buffers (zero-copy mode)
  int32_t *meta_dev, *pair_dev, *frames_dev;
  uint32_t *seq_dev, *status_dev;
  uint32_t *ready_dev = nullptr;  // [E] pair-ready flags (device address of b.ready_host)
  uint32_t fwd_seq = 0;           // sequence number of the last enqueued forward + draw
  int64_t rollouts = 0;           // completed rollouts (calls with t = T-1)
  // pull: per-env ready words the emulator threads store (mh_runner_set_ready) and the
  // tagged (a, r) words the heads kernel stores (SampleArgs::packed); pinned, device-mapped
  uint32_t *env_ready_host = nullptr, *env_ready_dev = nullptr;
  uint64_t *packed_host = nullptr, *packed_dev = nullptr;
  uint8_t *frames_hbm = nullptr;   // [4E][84*84*depth] HBM copy of the pushes (pull kernel)
  int32_t *count_hbm = nullptr;    // [E] push counts
  double trace[256][6];  // host timestamps (us) of the last 256 steps: t, start, enqueued, indices, emulated, booked
  int64_t ntrace = 0;
  double acc[7];  // host wall us: launch+wait for indices, runner, book, upload+preprocess enqueue; steps;
                  // then the launch+wait split: enqueue (forward / armed chains), wait for the indices
  // mt_rollout_trunk_timing: event pairs recorded around each step forward's trunk launches
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> marks;
  size_t marks_used = 0;
  // Replayed rollout graph (NIPS stacking chains): step 0's forward + the chains of steps 1..T
  // (the bootstrap last) captured once and launched as one hipGraph per rollout — ~6 us of host
  // time where enqueueing the 6 chains took ~13 us each, on the step-0 critical path. The kernel
  // arguments are fixed, so the rollout's sequence bases live in device memory: gbase_dev[0] =
  // the host step word value at step 0 (ready-word tags), gbase_dev[1] = the draw sequence number
  // before step 0's forward; the bootstrap heads kernel adds T to both. Host mirror: gbase_next.
  hipGraphExec_t rgraph = nullptr;
  const float *rgraph_params = nullptr;
  hipStream_t cap_stream = nullptr;
  hipEvent_t gev = nullptr;       // recorded after each replay: device-error checks while waiting
  uint32_t *gbase_dev = nullptr;  // [2]
  uint32_t gbase_host[2] = {0, 0};  // staging of the (re)initialisation copy
  uint32_t gbase_next[2] = {0, 0};  // device values after the last replay
  bool gbase_valid = false;
  bool capturing = false;  // enqueue_forward / arm_step record offsets + bases
  bool graph_live = false; // this rollout runs from the replayed graph
  bool graph_off = false;  // MT_ROLLOUT_GRAPH=0
  // the one stream every macro-step runs on (the first call's): the chains' in-kernel waits spin on
  // host words, and two streams of waiting kernels that land on one hardware queue serialise into a
  // timeout (env groups), so a second stream is refused
  hipStream_t stream0 = nullptr;
  bool stream_set = false;
  // update launched at the end of the rollout (mt_rollout_set_update)
  hipGraphExec_t update_graph = nullptr;
  float *lr_host = nullptr;
  double initial_lr = 0.0, annealing_steps = 1.0;
  // ... or the data-parallel update (mt_rollout_set_update_dp): three graphs with the two gradient
  // buckets' all-reduces on a side stream between them, ordered by events
  hipGraphExec_t dp_graph[3] = {nullptr, nullptr, nullptr};
  mt_comm *dp_comm = nullptr;
  float *dp_grad = nullptr;
  size_t dp_n = 0, dp_split = 0;
  hipStream_t dp_side = nullptr;
  hipEvent_t dp_ev[3] = {nullptr, nullptr, nullptr};
};

using namespace mt;

extern "C" int mt_rollout_create(const mt_net *net, int E, int T, void *runner, void *book,
                                 const mt_rollout_buffers *buffers, uint64_t seed,
                                 mt_rollout **out) {
  MT_CHECK_ARG(net && runner && book && buffers && out, "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  const mt_rollout_buffers &b = *buffers;
  const bool ip = (b.flags & MT_ROLLOUT_IN_PLACE) != 0;
  const bool zc = ip || (b.flags & MT_ROLLOUT_ZERO_COPY) != 0;
  const bool pl = (b.flags & MT_ROLLOUT_PIPELINED) != 0;
  const bool po = (b.flags & MT_ROLLOUT_POOLED) != 0;
  const bool rz = (b.flags & MT_ROLLOUT_RESIZED) != 0;
  MT_CHECK_ARG((b.flags & ~(MT_ROLLOUT_ZERO_COPY | MT_ROLLOUT_IN_PLACE | MT_ROLLOUT_POOLED | MT_ROLLOUT_PIPELINED |
                            MT_ROLLOUT_RESIZED | MT_ROLLOUT_BOOT_SLABS)) == 0,
               "unknown rollout flags %d", b.flags);
  MT_CHECK_ARG(!(b.flags & MT_ROLLOUT_BOOT_SLABS) || (pl && b.v_boot && !b.nz),
               "MT_ROLLOUT_BOOT_SLABS needs a pipelined, non-LSTM rollout with v_boot");
  MT_CHECK_ARG(!ip || b.frames_host, "in-place rollout needs frames_host");
  MT_CHECK_ARG(b.env_offset >= 0, "env_offset must be >= 0");
  MT_CHECK_ARG((int)ip + (int)po + (int)rz <= 1, "in-place, pooled and resized staging are exclusive");
  MT_CHECK_ARG(!pl || (zc && b.sync_host), "pipelined rollout needs zero-copy or in-place screens and sync_host");
  MT_CHECK_ARG(b.states && b.values && b.idx && b.pi && b.rep && b.ws && b.counters &&
                   (zc || (b.raw && b.meta && b.pair)) && b.row_lut && b.col_lut && b.idx_host &&
                   b.staging_host && b.pair_host && b.src_rows >= 84 && b.src_rows <= 210 &&
                   b.meta_host && b.reward_host && b.over_host && b.rm_host,
               "null buffer");
  void *staging_dev = nullptr, *meta_dev = nullptr, *pair_dev = nullptr, *frames_dev = nullptr;
  if (zc) {  // these buffers must be pinned + mapped (hipHostMalloc / torch pin_memory)
    MT_HIP(hipHostGetDevicePointer(&staging_dev, b.staging_host, 0));
    MT_HIP(hipHostGetDevicePointer(&meta_dev, b.meta_host, 0));
    MT_HIP(hipHostGetDevicePointer(&pair_dev, b.pair_host, 0));
    if (ip) MT_HIP(hipHostGetDevicePointer(&frames_dev, b.frames_host, 0));
  }
  void *ready_dev = nullptr;
  if (zc && b.ready_host) {
    MT_HIP(hipHostGetDevicePointer(&ready_dev, b.ready_host, 0));
    for (int e = 0; e < E; ++e) b.ready_host[e] = 0;
  }
  void *sync_dev = nullptr;
  if (pl) {
    MT_HIP(hipHostGetDevicePointer(&sync_dev, b.sync_host, 0));
    b.sync_host[0] = 0;
    b.sync_host[1] = 0;
  }
  mt_net_config cfg;
  MT_CHECK_ARG(mt_net_get_config(net, &cfg) == MT_OK, "bad net");
  const bool lstm = cfg.arch == MT_ARCH_LSTM;
  MT_CHECK_ARG(lstm == (b.nz != nullptr), "nz is required for (and only for) the LSTM arch");
  MT_CHECK_ARG(!lstm || !b.train_ws, "the LSTM arch keeps its rows in the frame-store workspace (train_ws NULL)");
  void *over_dev = nullptr;
  if (lstm) MT_HIP(hipHostGetDevicePointer(&over_dev, b.over_host, 0));  // read by the windows kernel
  size_t need = 0;
  if ((lstm ? mt_lstm_frames_workspace_bytes(net, E, T, &need) : mt_net_workspace_bytes(net, E, &need)) != MT_OK)
    return MT_ERR_ARG;
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
  ro->in_place = ip;
  ro->pooled = po;
  ro->resized = rz;
  ro->pipelined = pl;
  ro->pull = pl && rz;
  // the stacking chains: NIPS (nips_conv_kernel<STACK>) and gray NATURE (conv1 = DFwdStack): each
  // env's conv1 waits for its own publication, no pull / preprocess kernel in front of the convs
  ro->stack_fwd = ro->pull && (cfg.arch == MT_ARCH_NIPS || (cfg.arch == MT_ARCH_NATURE && cfg.depth == 1));
  ro->lstm = lstm;
  ro->lstm_stack = ro->pull && lstm;
  ro->frame_stack = ro->pull && !lstm && cfg.arch == MT_ARCH_PWYX;
  ro->boot_slabs = (b.flags & MT_ROLLOUT_BOOT_SLABS) != 0;
  ro->over_dev = (const float *)over_dev;
  if (lstm) ro->fstore = b.states - (size_t)(1 + 4 * E) * 84 * 84 * 4 * cfg.depth;
  ro->frames_dev = (int32_t *)frames_dev;
  ro->ready_dev = (uint32_t *)ready_dev;
  ro->seq_dev = (uint32_t *)sync_dev;
  ro->status_dev = sync_dev ? (uint32_t *)sync_dev + 1 : nullptr;
  ro->staging_dev = (uint8_t *)staging_dev;
  ro->meta_dev = (int32_t *)meta_dev;
  ro->pair_dev = (int32_t *)pair_dev;
  if (ro->pull) {
    hipError_t e = hipHostMalloc((void **)&ro->env_ready_host, sizeof(uint32_t) * E * MH_READY_STRIDE,
                                 hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostMalloc((void **)&ro->packed_host, sizeof(uint64_t) * E, hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&ro->env_ready_dev, ro->env_ready_host, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&ro->packed_dev, ro->packed_host, 0);
    if (e == hipSuccess) e = hipMalloc((void **)&ro->frames_hbm, (size_t)4 * E * 84 * 84 * cfg.depth);
    if (e == hipSuccess) e = hipMalloc((void **)&ro->count_hbm, sizeof(int32_t) * 2 * E);  // counts; offsets 4e
    if (e == hipSuccess && ro->lstm_stack) {
      e = hipMalloc((void **)&ro->lstm_sync, sizeof(uint32_t) * stack_conv1_sync_words(E));
      if (e == hipSuccess) e = hipMemset(ro->lstm_sync, 0, sizeof(uint32_t) * stack_conv1_sync_words(E));
    }
    if (e == hipSuccess) {
      std::vector<int32_t> offs(E);
      for (int i = 0; i < E; ++i) offs[i] = 4 * i;
      e = hipMemcpy(ro->count_hbm + E, offs.data(), sizeof(int32_t) * E, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
      if (ro->env_ready_host) (void)hipHostFree(ro->env_ready_host);
      if (ro->packed_host) (void)hipHostFree(ro->packed_host);
      if (ro->frames_hbm) (void)hipFree(ro->frames_hbm);
      if (ro->count_hbm) (void)hipFree(ro->count_hbm);
      if (ro->lstm_sync) (void)hipFree(ro->lstm_sync);
      delete ro;
      set_error("pinned step words: %s", hipGetErrorString(e));
      return MT_ERR_HIP;
    }
    std::memset(ro->env_ready_host, 0, sizeof(uint32_t) * E * MH_READY_STRIDE);
    std::memset(ro->packed_host, 0, sizeof(uint64_t) * E);
  }
  // every chain of a rollout is armed by its step 0 call, right behind the step-0 forward: that
  // call waits for the update + the step-0 chain anyway (~80 us), so the ~11 us of launches per
  // chain land there instead of in front of the later steps' waits (step 1 was host-bound)
  ro->ahead = T;
  if (const char *v = std::getenv("MT_ROLLOUT_AHEAD")) ro->ahead = std::max(1, std::min(T, std::atoi(v)));
  if (const char *v = std::getenv("MT_ROLLOUT_GRAPH")) ro->graph_off = std::atoi(v) == 0;
  ro->fwd_of.assign(T, 0);
  ro->ev.assign(T, nullptr);
  for (int i = 0; i < T; ++i) {
    hipError_t e = hipEventCreateWithFlags(&ro->ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
      for (int j = 0; j < i; ++j) (void)hipEventDestroy(ro->ev[j]);
      delete ro;
      set_error("hipEventCreate: %s", hipGetErrorString(e));
      return MT_ERR_HIP;
    }
  }
  *out = ro;
  return MT_OK;
}

extern "C" void mt_rollout_destroy(mt_rollout *ro) {
  if (!ro) return;
  if (ro->rgraph) (void)hipGraphExecDestroy(ro->rgraph);
  if (ro->cap_stream) (void)hipStreamDestroy(ro->cap_stream);
  if (ro->gev) (void)hipEventDestroy(ro->gev);
  if (ro->gbase_dev) (void)hipFree(ro->gbase_dev);
  if (ro->dp_side) (void)hipStreamDestroy(ro->dp_side);
  for (hipEvent_t e : ro->dp_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ro->ev) (void)hipEventDestroy(e);
  for (auto &m : ro->marks) {
    (void)hipEventDestroy(m.first);
    (void)hipEventDestroy(m.second);
  }
  if (ro->pull) {
    (void)mh_runner_set_ready(ro->runner, nullptr, 0);
    (void)hipHostFree(ro->env_ready_host);
    (void)hipHostFree(ro->packed_host);
    (void)hipFree(ro->frames_hbm);
    (void)hipFree(ro->count_hbm);
    if (ro->lstm_sync) (void)hipFree(ro->lstm_sync);
  }
  delete ro;
}

#define MT_TRY_(x)                 \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != MT_OK) return rc_;  \
  } while (0)

// Device-side wait for the host's step sequence word (pipelined mode): one lane polls the
// host-mapped word with system-scope vector loads (never the scalar cache) until it equals seq.
// Bounded: after ~2 s (s_memrealtime, 100 MHz) it gives up, records the failure in status (the
// host turns it into an error at its next wait for the indices) and lets the stream drain.
__global__ void wait_seq_kernel(const uint32_t *seq_word, uint32_t seq, uint32_t *status) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(seq_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  // the preprocess that follows in the stream reads the staging in place: a new dispatch, whose
  // system-scope acquire drops any line cached before the host wrote it
}

// Pull kernel (pull mode: pipelined + resized): copies each env's pushes from the pinned staging into HBM as soon as
// its emulator thread has published it (ready[e] = (step << 3) | push count, mh_runner_set_ready),
// so the PCIe transfer of a step's frames overlaps the emulation of the other envs and the
// stacking conv kernel reads HBM only. Block = kPullEnvs consecutive envs (one runner worker's
// share at E = 32, ew = 8; a worker steps its envs in index order, so lane 0 polls only the next
// one: one PCIe read in flight per block, s_sleep between polls). Bounded like wait_seq_kernel:
// after ~2 s it records the failure in status and returns.
// Memory ordering. The host writes env e's frames, then `sfence` + a release store of ready[e]
// (runner.cpp). Lane 0 sees the word with a system-scope load (it bypasses the non-coherent
// caches); the block barrier orders every data load after it (a GPU issues no load ahead of a
// barrier). The staging is non-coherent pinned memory, so a data load may hit a cache line
// fetched EARLIER — within one launch that can only be a line another env's copy fetched: env
// slot groups are 4 x 7,056 B, so an env's first and last 128-B lines may hold bytes of its
// neighbours, which can be published later than the line was fetched. Those edge chunks are read
// with system-scope loads (never served from, nor trusted in, those caches); every other line of
// env e's range holds env e's bytes only and is first touched after ready[e]. (Lines fetched in an
// earlier launch do not survive: each dispatch starts with a system-scope acquire.) No cache
// invalidation is issued: a device-wide invalidate would also drop the trunk weights from L2.
constexpr int kPullEnvs = 4;
#ifdef MT_PROBE  // experiment builds: per env, when its word was seen and its copy done (tools/probe.py)
static __device__ unsigned long long mt_probe_ro[512 * 4];
extern "C" int mt_probe_read_rollout(unsigned long long *out, size_t n) {
  MT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mt_probe_ro), std::min(n, sizeof(mt_probe_ro) / 8) * 8));
  return MT_OK;
}
#define MT_PROBE_RO(e, p) \
  if ((e) < 512) mt_probe_ro[(e) * 4 + (p)] = __builtin_amdgcn_s_memrealtime()
#else
#define MT_PROBE_RO(e, p)
#endif
// a 16-B chunk whose 128-B line also holds bytes outside [lo, hi) (byte offsets): read it with
// two system-scope 8-byte loads
__device__ __forceinline__ uint4 pull_chunk(const uint4 *staging, size_t q, size_t lo, size_t hi) {
  const size_t a = q * 16, line = a & ~(size_t)127;
  if (line >= lo && line + 128 <= hi) return staging[q];
  const uint64_t *p = reinterpret_cast<const uint64_t *>(staging + q);
  const uint64_t x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
}

__global__ __launch_bounds__(256) void pull_frames_kernel(const uint4 *__restrict__ staging, const uint32_t *ready,
                                                          uint32_t want, uint32_t *status, int E, int frame16,
                                                          uint4 *__restrict__ frames, int32_t *__restrict__ count) {
  __shared__ int s_p;
  const int e0 = blockIdx.x * kPullEnvs, n = min(kPullEnvs, E - e0);
  const uint32_t tag = want & 0x1fffffffu;
  if (threadIdx.x == 0) MT_PROBE_RO(e0, 2);
  for (int k = 0; k < n; ++k) {
    const int e = e0 + k;
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t v;
      while (((v = __hip_atomic_load(ready + (size_t)e * MH_READY_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >>
              3) != tag) {
        __builtin_amdgcn_s_sleep(8);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
          __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          v = 0xffffffffu;  // timed out
          break;
        }
      }
      MT_PROBE_RO(e, 0);
      s_p = v == 0xffffffffu ? -1 : (int)(v & 7u);
    }
    __syncthreads();
    const int p0 = s_p;
    if (p0 < 0) return;  // timed out (uniform over the block)
    const int p = min(max(p0, 1), 4);
    const size_t base = (size_t)4 * e * frame16;  // slots 4e .. 4e + p - 1 are contiguous
    const size_t lo = base * 16, hi = (base + (size_t)4 * frame16) * 16;  // env e's slot group (bytes)
    for (int q = threadIdx.x; q < p * frame16; q += 256) frames[base + q] = pull_chunk(staging, base + q, lo, hi);
    if (threadIdx.x == 0) count[e] = p;
    __syncthreads();  // s_p is rewritten by the next round
    if (threadIdx.x == 0) MT_PROBE_RO(e, 1);
  }
}

namespace {
// the next event pair of the trunk timing (mt_rollout_trunk_timing), or null when it is off
int next_marks(mt_rollout *ro, const hipEvent_t **out) {
  *out = nullptr;
  if (!ro->timing) return MT_OK;
  if (ro->marks_used == ro->marks.size()) {
    hipEvent_t a, b;
    MT_HIP(hipEventCreate(&a));
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      set_error("hipEventCreate failed");
      return MT_ERR_HIP;
    }
    ro->marks.emplace_back(a, b);
  }
  *out = &ro->marks[ro->marks_used++].first;
  return MT_OK;
}

// forward of state slot t with the A3 draw fused into its heads kernel (paac.py:144-147); the
// indices land in idx[.][t] and the [2][E] pair; ev[t & 1] marks the pair ready.
// stacked: state slot t is built from slot t-1 + step t-1's pushes inside the forward's conv
// kernel (fused mt_preprocess_resized; ro->stack_fwd).
// t == 0 && stacked: slot 0 <- slot T of the previous rollout inside the forward (the copy of
// paac.py's states carrying over, otherwise a separate copy on the update's critical path).
int enqueue_forward(mt_rollout *ro, const float *params, int t, hipStream_t s, bool stacked = false,
                    uint32_t want = 0) {
  const mt_rollout_buffers &b = ro->b;
  const int E = ro->E, T = ro->T;
  const size_t slot = (size_t)E * 84 * 84 * 4 * ro->depth;
  // t > 0: the conv kernel pulls step t-1's pushes itself (ready words tagged `want`)
  StackSrc st = t > 0 ? StackSrc{b.states + (size_t)(t - 1) * slot, ro->staging_dev, nullptr, b.states + (size_t)t * slot}
                      : StackSrc{b.states + (size_t)T * slot, nullptr, nullptr, b.states};
  if (t > 0) {
    st.ready = ro->env_ready_dev;
    st.tag = want & 0x1fffffffu;  // (capturing: the offset k of gbase_dev[0])
    st.status = ro->status_dev;
    if (ro->capturing) st.tag_base = ro->gbase_dev;
  }
  int32_t *a_d = b.idx + (size_t)t * E, *r_d = b.idx + (size_t)T * E + (size_t)t * E;
  SampleArgs smp{ro->seed, b.counters, a_d, r_d, ro->zero_copy ? ro->pair_dev : b.pair};
  smp.ready = ro->ready_dev;
  if (ro->capturing) {  // draw sequence number gbase_dev[1] + t + 1 (mt_rollout_step sets fwd_of)
    smp.seq = (uint32_t)t + 1;
    smp.seq_base = ro->gbase_dev + 1;
  } else {
    smp.seq = ++ro->fwd_seq;
    ro->fwd_of[t] = smp.seq;
  }
  smp.packed = ro->packed_dev;
  smp.row0 = b.env_offset;
  // with a train workspace: activations into its rows t*E.., per-step pi / rep (mt_forward_rows)
  const TrainRows tr{(float *)b.train_ws, b.train_ws_bytes, T * E, t * E};
  const size_t po = b.train_ws ? (size_t)t * E : 0;
  const hipEvent_t *marks;
  MT_TRY_(next_marks(ro, &marks));
  if (ro->lstm) {  // step t's new frames + its E windows, pi / rep [T+1][E][.]
    // (pull mode, t > 0: the step's conv1 launch pulls + stacks env by env, arm_step launched no
    //  pull / preprocess kernel)
    const bool stk_lstm = ro->lstm_stack && t > 0;
    MT_TRY_(lstm_step_forward(ro->net, params, ro->fstore, t, E, T, b.nz, ro->over_dev, b.ws, b.ws_bytes,
                              b.values + (size_t)t * E, b.pi + (size_t)t * E * ro->A, b.rep + (size_t)t * E * ro->R,
                              &smp, s, marks, stk_lstm ? &st : nullptr, ro->lstm_sync));
  } else {
    MT_TRY_(forward_sample(ro->net, params, b.states + (size_t)t * slot, E, b.ws, b.ws_bytes,
                           b.values + (size_t)t * E, b.pi + po * ro->A, b.rep + po * ro->R, &smp, true, s,
                           b.train_ws ? &tr : nullptr, stacked ? &st : nullptr, marks));
  }
  if (!ro->zero_copy)
    MT_HIP(hipMemcpyAsync(b.pair_host, b.pair, sizeof(int32_t) * 2 * E, hipMemcpyDeviceToHost, s));
  if (!ro->capturing) MT_HIP(hipEventRecord(ro->ev[t], s));
  return MT_OK;
}

// preprocess of the pushes of macro-step t into state slot t+1 (atari_emulator.py:79-124)
int enqueue_preprocess(mt_rollout *ro, int t, int total, hipStream_t s) {
  const mt_rollout_buffers &b = ro->b;
  const int E = ro->E;
  const size_t slot = (size_t)E * 84 * 84 * 4 * ro->depth;
  const uint8_t *cur = b.states + (size_t)t * slot;
  uint8_t *nxt = b.states + (size_t)(t + 1) * slot;
  mt_stream_t st = (mt_stream_t)s;
  if (ro->in_place)
    return mt_preprocess_frames(ro->staging_dev, ro->frames_dev, ro->meta_dev + E, E, ro->depth, b.row_lut,
                                b.col_lut, cur, nxt, st);
  const uint8_t *raw = ro->staging_dev;
  const int32_t *meta = ro->meta_dev;
  if (!ro->zero_copy) {
    const size_t per_push = ro->resized ? (size_t)84 * 84 * ro->depth : (ro->pooled ? 1 : 2) * ro->frame_bytes;
    MT_HIP(hipMemcpyAsync(b.raw, b.staging_host, (size_t)total * per_push, hipMemcpyHostToDevice, s));
    MT_HIP(hipMemcpyAsync(b.meta, b.meta_host, sizeof(int32_t) * 2 * E, hipMemcpyHostToDevice, s));
    raw = b.raw;
    meta = b.meta;
  }
  if (ro->resized) return mt_preprocess_resized(raw, meta, meta + E, E, ro->depth, cur, nxt, st);
  return ro->pooled ? mt_preprocess_pooled(raw, meta, meta + E, E, ro->depth, b.src_rows, b.row_lut, b.col_lut,
                                           cur, nxt, st)
                    : mt_preprocess(raw, meta, meta + E, E, ro->depth, b.src_rows, b.row_lut, b.col_lut, cur,
                                    nxt, st);
}
// pipelined: arm step k's chain — it waits on the device for the host's step k-1, so it can be
// enqueued `ahead` = k - t >= 1 host steps early (t = the host's current step): the chain's
// wait (pull kernel per env, else wait_seq_kernel) is for the host step word value seq + ahead.
// Step T's chain is the bootstrap forward V(s_T) (paac.py:219-224).
int arm_step(mt_rollout *ro, const float *params, int k, int ahead, hipStream_t s) {
  const mt_rollout_buffers &b = ro->b;
  const int E = ro->E, T = ro->T;
  // (capturing: the offset k from the rollout's base gbase_dev[0] = the host step word at step 0)
  const uint32_t want = ro->capturing ? (uint32_t)k : ro->seq + (uint32_t)ahead;
  // pull: the pull kernel waits per env and copies the pushes into HBM; the preprocess of step
  // k-1 then reads them there — inside step k's forward conv kernel (stack_fwd, NIPS), else as
  // mt_preprocess_resized
  const bool stk = (ro->stack_fwd || ro->frame_stack) && (k < T || b.v_boot);
  if (ro->pull) {
    if (!stk && !ro->lstm_stack) {  // (the stacking conv kernel pulls each env itself)
      hipLaunchKernelGGL(pull_frames_kernel, dim3((E + kPullEnvs - 1) / kPullEnvs), dim3(256), 0, s,
                         reinterpret_cast<const uint4 *>(ro->staging_dev), ro->env_ready_dev, want, ro->status_dev, E,
                         (int)(84 * 84 * ro->depth / 16), reinterpret_cast<uint4 *>(ro->frames_hbm), ro->count_hbm);
      MT_LAUNCHED();
      const size_t slot = (size_t)E * 84 * 84 * 4 * ro->depth;
      MT_TRY_(mt_preprocess_resized(ro->frames_hbm, ro->count_hbm + E, ro->count_hbm, E, ro->depth,
                                    b.states + (size_t)(k - 1) * slot, b.states + (size_t)k * slot, (mt_stream_t)s));
    }
  } else {
    hipLaunchKernelGGL(wait_seq_kernel, dim3(1), dim3(64), 0, s, ro->seq_dev, want, ro->status_dev);
    MT_LAUNCHED();
    MT_TRY_(enqueue_preprocess(ro, k - 1, 4 * E, s));
  }
  if (k < T) {
    MT_TRY_(enqueue_forward(ro, params, k, s, stk, want));
  } else if (b.v_boot && ro->lstm) {  // bootstrap V(s_T): slot 4 + T's frames + the windows of step T
    const size_t slot = (size_t)E * 84 * 84 * 4 * ro->depth;
    StackSrc st{b.states + (size_t)(T - 1) * slot, ro->staging_dev, nullptr, b.states + (size_t)T * slot};
    st.ready = ro->env_ready_dev;
    st.tag = want & 0x1fffffffu;
    st.status = ro->status_dev;
    MT_TRY_(lstm_step_forward(ro->net, params, ro->fstore, T, E, T, b.nz, ro->over_dev, b.ws, b.ws_bytes, b.v_boot,
                              b.pi + (size_t)T * E * ro->A, b.rep + (size_t)T * E * ro->R, nullptr, s, nullptr,
                              ro->lstm_stack ? &st : nullptr, ro->lstm_sync));
  } else if (b.v_boot) {  // bootstrap V(s_T), no draw, no train rows
    const size_t slot = (size_t)E * 84 * 84 * 4 * ro->depth;
    const size_t po = b.train_ws ? (size_t)T * E : 0;
    StackSrc st{b.states + (size_t)(T - 1) * slot, ro->staging_dev, nullptr, b.states + (size_t)T * slot};
    st.ready = ro->env_ready_dev;
    st.tag = want & 0x1fffffffu;
    st.status = ro->status_dev;
    SampleArgs adv{};  // capturing: no draw; the heads (boot_slabs: dense) kernel advances the replay's bases by T
    if (ro->capturing) {
      st.tag_base = ro->gbase_dev;
      adv.advance = ro->gbase_dev;
      adv.advance_by = (uint32_t)T;
    }
    if (ro->boot_slabs)  // trunk + dense slabs only: the update's loss kernel finishes V(s_T)
      MT_TRY_(forward_boot(ro->net, params, b.states + (size_t)T * slot, E, b.ws, b.ws_bytes, s, stk ? &st : nullptr,
                           adv.advance, adv.advance_by));
    else
      MT_TRY_(forward_sample(ro->net, params, b.states + (size_t)T * slot, E, b.ws, b.ws_bytes, b.v_boot,
                             b.pi + po * ro->A, b.rep + po * ro->R, ro->capturing ? &adv : nullptr, true, s, nullptr,
                             stk ? &st : nullptr));
  }
  ro->armed_upto = k;
  return MT_OK;
}

// The replayed rollout graph applies to the stacking chains (NIPS, gray NATURE) with the bootstrap in the last
// chain, every chain armed at step 0, after a first eager rollout (step 0's forward then takes
// slot 0 from slot T), without trunk timing (its events are per launch).
bool graph_eligible(const mt_rollout *ro) {
  return !ro->graph_off && ro->pipelined && ro->stack_fwd && !ro->lstm && ro->packed_host && ro->b.v_boot &&
         ro->zero_copy && ro->ahead == ro->T && !ro->timing && ro->rollouts > 0;
}

// Step 0 of a rollout from the replayed graph: capture it on first use (or when the parameter
// buffer moved), bring the device bases in line with the host's counters when an eager rollout ran
// in between, launch, and set the host's expectations (draw tags, armed steps).
int replay_rollout_graph(mt_rollout *ro, const float *params, hipStream_t s) {
  const int T = ro->T;
  if (!ro->gbase_dev) {
    MT_HIP(hipMalloc((void **)&ro->gbase_dev, 2 * sizeof(uint32_t)));
    MT_HIP(hipEventCreateWithFlags(&ro->gev, hipEventDisableTiming));
    MT_HIP(hipStreamCreateWithFlags(&ro->cap_stream, hipStreamNonBlocking));
  }
  if (ro->rgraph && ro->rgraph_params != params) {
    MT_HIP(hipGraphExecDestroy(ro->rgraph));
    ro->rgraph = nullptr;
  }
  if (!ro->rgraph) {
    MT_HIP(hipStreamBeginCapture(ro->cap_stream, hipStreamCaptureModeThreadLocal));
    ro->capturing = true;
    int rc = enqueue_forward(ro, params, 0, ro->cap_stream, true);
    for (int k = 1; rc == MT_OK && k <= T; ++k) rc = arm_step(ro, params, k, k, ro->cap_stream);
    ro->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(ro->cap_stream, &g);
    if (rc != MT_OK) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    MT_HIP(ec);
    const hipError_t ei = hipGraphInstantiate(&ro->rgraph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) {
      ro->rgraph = nullptr;
      set_error("hipGraphInstantiate (rollout) failed: %s", hipGetErrorString(ei));
      return MT_ERR_HIP;
    }
    ro->rgraph_params = params;
  }
  if (!ro->gbase_valid || ro->gbase_next[0] != ro->seq || ro->gbase_next[1] != ro->fwd_seq) {
    // (stream-ordered after every earlier reader: the previous replay's bootstrap has advanced them)
    ro->gbase_host[0] = ro->seq;
    ro->gbase_host[1] = ro->fwd_seq;
    MT_HIP(hipMemcpyAsync(ro->gbase_dev, ro->gbase_host, sizeof(ro->gbase_host), hipMemcpyHostToDevice, s));
  }
  MT_HIP(hipGraphLaunch(ro->rgraph, s));
  MT_HIP(hipEventRecord(ro->gev, s));
  for (int t = 0; t < T; ++t) ro->fwd_of[t] = ro->fwd_seq + 1 + (uint32_t)t;
  ro->fwd_seq += (uint32_t)T;
  ro->gbase_next[0] = ro->seq + (uint32_t)T;  // (the host step word after this rollout's T steps)
  ro->gbase_next[1] = ro->fwd_seq;
  ro->gbase_valid = true;
  ro->armed_upto = T;
  ro->graph_live = true;
  return MT_OK;
}

// The registered update on stream s: the single graph (mt_rollout_set_update), or the data-parallel
// sequence (mt_rollout_set_update_dp: paac._bucketed_update's three graphs with the two gradient
// buckets' all-reduces on the side stream between them).
int launch_update(mt_rollout *ro, hipStream_t s) {
  if (ro->update_graph) {
    MT_HIP(hipGraphLaunch(ro->update_graph, s));
    return MT_OK;
  }
  float *g = ro->dp_grad;
  MT_HIP(hipGraphLaunch(ro->dp_graph[0], s));  // loss + dense / head gradients
  MT_HIP(hipEventRecord(ro->dp_ev[0], s));
  MT_HIP(hipStreamWaitEvent(ro->dp_side, ro->dp_ev[0], 0));
  MT_TRY_(mt_allreduce(ro->dp_comm, g + ro->dp_split, ro->dp_n - ro->dp_split, ro->dp_side));
  MT_HIP(hipGraphLaunch(ro->dp_graph[1], s));  // the rest of the conv backward
  MT_HIP(hipEventRecord(ro->dp_ev[1], s));
  MT_HIP(hipStreamWaitEvent(ro->dp_side, ro->dp_ev[1], 0));
  MT_TRY_(mt_allreduce(ro->dp_comm, g, ro->dp_split, ro->dp_side));
  MT_HIP(hipEventRecord(ro->dp_ev[2], ro->dp_side));
  MT_HIP(hipStreamWaitEvent(s, ro->dp_ev[2], 0));
  MT_HIP(hipGraphLaunch(ro->dp_graph[2], s));  // norm partials + clip + RMSProp
  return MT_OK;
}

}  // namespace

// One macro-step t (paac.py:140-205). Pipelined mode keeps the GPU ahead of the host's launch
// calls: step 0 enqueues the chains of steps 1..T (each behind device-side waits on the host's
// words: the ready word per env in pull mode, else wait_seq -> preprocess(t -> t+1)), from the
// second rollout on as one replayed graph, so when the emulators finish, the host only stores the
// words and the GPU runs the chain without a launch on the critical path. Stream order keeps every
// buffer hand-off safe: the staging of step t is read by chain t+1 only after the word, and
// rewritten by the emulators of step t+1 only after chain t+1's indices arrived.
extern "C" int mt_rollout_step(mt_rollout *ro, const float *params, int t, int64_t *global_step,
                               mt_stream_t stream) {
  MT_CHECK_ARG(ro && params && global_step, "null argument");
  MT_CHECK_ARG(t >= 0 && t < ro->T, "t=%d out of [0,%d)", t, ro->T);
  const mt_rollout_buffers &b = ro->b;
  hipStream_t s = (hipStream_t)stream;
  if (!ro->stream_set) {
    ro->stream0 = s;
    ro->stream_set = true;
  }
  MT_CHECK_ARG(s == ro->stream0, "every macro-step of a rollout handle runs on one stream (its in-kernel waits "
               "must not share a hardware queue with another stream's): got %p after %p", (void *)s,
               (void *)ro->stream0);
  const int E = ro->E, T = ro->T;
  const double t0 = now_us();
  int32_t *a_h = b.idx_host + (size_t)t * E, *r_h = b.idx_host + (size_t)T * E + (size_t)t * E;
  // 1. forward + draw of step t, unless a previous call already enqueued it
  if (t == 0 || !ro->pipelined) ro->armed_upto = -1;  // a new rollout (parameters changed)
  if (t == 0) {
    ro->graph_live = false;
    if (graph_eligible(ro)) MT_TRY_(replay_rollout_graph(ro, params, s));
  }
  if (ro->armed_upto < t) {
    // stack_fwd: after a completed rollout, slot 0 is taken from slot T inside this forward
    MT_TRY_(enqueue_forward(ro, params, t, s, t == 0 && ro->stack_fwd && ro->rollouts > 0));
    ro->armed_upto = t;
  }
  // 2. pipelined: arm steps up to t + depth (at most T) while the GPU works on step t, so the
  //    launches are off the critical path (every chain at step 0, see ahead — the GPU chain after the
  //    emulators is shorter than the launches of a chain)
  if (ro->pipelined)
    for (int k = ro->armed_upto + 1; k <= std::min(t + ro->ahead, T); ++k) MT_TRY_(arm_step(ro, params, k, k - t, s));
  const bool update_now = (ro->update_graph || ro->dp_graph[0]) && t == T - 1;
  const double t0w = now_us();
  // 3. wait for the indices of step t (spin: a blocking wait sleeps past the chain and pays the
  //    wake-up latency)
  // (with ready flags: poll the E flags the heads kernel stores after each pair — one cached host
  //  load each — and query the event only now and then, to surface a device error)
  const uint32_t want = ro->fwd_of[t];
  const hipEvent_t step_ev = ro->graph_live ? ro->gev : ro->ev[t];  // (device-error checks)
  if (ro->packed_host) {  // tagged (a, r) words: both halves carry the step's tag
    const uint32_t tag = want & 0xffffu;
    const volatile uint64_t *pw = ro->packed_host;
    for (int e = 0, spins = 0; e < E;) {
      const uint64_t v = __atomic_load_n(const_cast<const uint64_t *>(pw + e), __ATOMIC_ACQUIRE);
      if (((v >> 16) & 0xffffu) == tag && (v >> 48) == tag) {
        a_h[e] = (int32_t)(v & 0xffffu);
        r_h[e] = (int32_t)((v >> 32) & 0xffffu);
        ++e;
        continue;
      }
      __builtin_ia32_pause();
      if (++spins == 4096) {
        spins = 0;
        const hipError_t q = hipEventQuery(step_ev);
        if (q != hipSuccess && q != hipErrorNotReady) MT_HIP(q);
      }
    }
  } else if (ro->ready_dev) {
    const volatile uint32_t *rf = b.ready_host;
    for (int e = 0, spins = 0; e < E;) {
      if (__atomic_load_n(const_cast<const uint32_t *>(rf + e), __ATOMIC_ACQUIRE) == want) {
        ++e;
        continue;
      }
      __builtin_ia32_pause();
      if (++spins == 4096) {
        spins = 0;
        const hipError_t q = hipEventQuery(step_ev);
        if (q != hipSuccess && q != hipErrorNotReady) MT_HIP(q);
      }
    }
  } else {
    hipError_t q;
    while ((q = hipEventQuery(step_ev)) == hipErrorNotReady) __builtin_ia32_pause();
    MT_HIP(q);
  }
  if (ro->pipelined && __atomic_load_n(&b.sync_host[1], __ATOMIC_ACQUIRE) != 0) {
    set_error("device wait for the host step word timed out (host stalled > 2 s); rollout state is invalid");
    return MT_ERR_HIP;
  }
  if (!ro->packed_host) {
    std::memcpy(a_h, b.pair_host, sizeof(int32_t) * E);
    std::memcpy(r_h, b.pair_host + E, sizeof(int32_t) * E);
  }
  const double t1 = now_us();
  // 4. emulators (runners.py:44-50 / emulator_runner.py:24-41) + bookkeeping (paac.py:176-205)
  int total = 0;
  if (ro->pull && mh_runner_set_ready(ro->runner, ro->env_ready_host, ro->seq + 1) != 0) {
    set_error("mh_runner_set_ready: %s", mh_last_error());
    return MT_ERR_ARG;
  }
  const int rs = ro->in_place ? mh_runner_step_frames(ro->runner, a_h, r_h, b.frames_host, b.meta_host + E,
                                                    b.reward_host, b.over_host)
                              : mh_runner_step(ro->runner, a_h, r_h, b.staging_host, b.meta_host, b.meta_host + E,
                                               b.reward_host, b.over_host, &total);
  if (rs != 0) {
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
  // 5. the LR of the step reached, for a registered update (actor_learner.py:145-148; read by the
  //    RMSProp kernel when it runs, after this store), then release the armed chain (pipelined), or
  //    enqueue the preprocess now
  if (update_now) {
    const int64_t gs = *global_step;
    const double lr = (double)gs <= ro->annealing_steps
                          ? ro->initial_lr - ((double)gs * ro->initial_lr / ro->annealing_steps)
                          : 0.0;
    *ro->lr_host = (float)lr;
  }
  int rc = MT_OK;
  if (ro->pipelined) {
    ro->seq += 1;
    __atomic_store_n(&b.sync_host[0], ro->seq, __ATOMIC_RELEASE);
  } else {
    rc = enqueue_preprocess(ro, t, total, s);
  }
  // 6. the update right behind the bootstrap chain (mt_rollout_set_update / _dp). (Enqueued at this
  //    step's start instead, behind a device wait for the step word, it measured slower: the graph
  //    launch then delays the emulators of the last step, while here it overlaps the bootstrap
  //    chain; Pong 682-728k vs 731k, profiles/r05h.)
  if (rc == MT_OK && update_now) MT_TRY_(launch_update(ro, s));
  const double t4 = now_us();
  ro->acc[0] += t1 - t0;
  ro->acc[1] += t2 - t1;
  ro->acc[2] += t3 - t2;
  ro->acc[3] += t4 - t3;
  ro->acc[4] += 1;
  {
    double *tr = ro->trace[ro->ntrace++ & 255];
    tr[0] = t;
    tr[1] = t0;
    tr[2] = t0w;
    tr[3] = t1;
    tr[4] = t2;
    tr[5] = t3;
  }
  ro->acc[5] += t0w - t0;
  ro->acc[6] += t1 - t0w;
  if (rc == MT_OK && t == T - 1) ro->rollouts += 1;
  return rc;
}

extern "C" int mt_rollout_run(mt_rollout *ro, const float *params, int64_t *global_step, mt_stream_t stream) {
  MT_CHECK_ARG(ro && params && global_step, "null argument");
  for (int t = 0; t < ro->T; ++t) MT_TRY_(mt_rollout_step(ro, params, t, global_step, stream));
  return MT_OK;
}

extern "C" int mt_rollout_set_update(mt_rollout *ro, void *graph_exec, float *lr_host, double initial_lr,
                                     double annealing_steps) {
  MT_CHECK_ARG(ro, "null argument");
  MT_CHECK_ARG(!graph_exec || (lr_host && annealing_steps > 0.0), "a registered update needs lr_host and annealing_steps > 0");
  MT_CHECK_ARG(!graph_exec || ro->pipelined, "the rollout launches the update only in pipelined mode");
  ro->update_graph = (hipGraphExec_t)graph_exec;
  ro->lr_host = lr_host;
  ro->initial_lr = initial_lr;
  ro->annealing_steps = annealing_steps;
  // registering replaces a data-parallel update; unregistering (NULL) clears both forms, so no
  // registered update is left behind whose LR word was just set to NULL
  ro->dp_graph[0] = ro->dp_graph[1] = ro->dp_graph[2] = nullptr;
  return MT_OK;
}

extern "C" int mt_rollout_update_form(const mt_rollout *ro, int *form) {
  MT_CHECK_ARG(ro && form, "null argument");
  *form = ro->dp_graph[0] ? 2 : (ro->update_graph ? 1 : 0);
  return MT_OK;
}

extern "C" int mt_rollout_set_update_dp(mt_rollout *ro, void *const *graph_execs, mt_comm *comm, float *grad, size_t n,
                                        size_t split, float *lr_host, double initial_lr, double annealing_steps) {
  MT_CHECK_ARG(ro, "null argument");
  if (!graph_execs) {  // unregister
    ro->dp_graph[0] = ro->dp_graph[1] = ro->dp_graph[2] = nullptr;
    return MT_OK;
  }
  MT_CHECK_ARG(graph_execs[0] && graph_execs[1] && graph_execs[2] && comm && grad && lr_host,
               "a registered data-parallel update needs 3 graphs, a communicator, the gradient and lr_host");
  MT_CHECK_ARG(split <= n && annealing_steps > 0.0, "bucket split %zu of %zu, annealing steps %g", split, n,
               annealing_steps);
  MT_CHECK_ARG(ro->pipelined, "the rollout launches the update only in pipelined mode");
  if (!ro->dp_side) {
    MT_HIP(hipStreamCreateWithFlags(&ro->dp_side, hipStreamNonBlocking));
    for (hipEvent_t &e : ro->dp_ev) MT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  for (int i = 0; i < 3; ++i) ro->dp_graph[i] = (hipGraphExec_t)graph_execs[i];
  ro->dp_comm = comm;
  ro->dp_grad = grad;
  ro->dp_n = n;
  ro->dp_split = split;
  ro->update_graph = nullptr;
  ro->lr_host = lr_host;
  ro->initial_lr = initial_lr;
  ro->annealing_steps = annealing_steps;
  return MT_OK;
}

extern "C" int mt_rollout_stats(mt_rollout *ro, double *out5, int reset) {
  MT_CHECK_ARG(ro && out5, "null argument");
  for (int i = 0; i < 5; ++i) out5[i] = ro->acc[i];
  if (reset)
    for (int i = 0; i < 5; ++i) ro->acc[i] = 0;
  return MT_OK;
}

// Trunk timing of the macro-steps' forwards, in place (the kernels the rollout runs, as it runs
// them): enable != 0 starts recording an event pair around every step forward's trunk launches;
// enable == 0 stops, waits for the recorded events and returns their summed duration (us) and
// count, then forgets them. Each pair spans the trunk kernels of one forward (NIPS: the stacking
// conv kernel + the dense kernel) and the boundary between them.
extern "C" int mt_rollout_stats_ex(mt_rollout *ro, double *out, int n, int reset) {
  MT_CHECK_ARG(ro && out && n >= 0, "bad argument");
  for (int i = 0; i < n && i < 7; ++i) out[i] = ro->acc[i];
  if (reset)
    for (int i = 0; i < 7; ++i) ro->acc[i] = 0;
  return MT_OK;
}

extern "C" int mt_rollout_host_trace(mt_rollout *ro, double *out, int max_steps, int *n) {
  MT_CHECK_ARG(ro && out && n && max_steps >= 0, "bad argument");
  const int64_t have = std::min<int64_t>(std::min<int64_t>(ro->ntrace, 256), max_steps);
  for (int64_t k = 0; k < have; ++k) {
    const double *tr = ro->trace[(ro->ntrace - have + k) & 255];
    for (int j = 0; j < 6; ++j) out[k * 6 + j] = tr[j];
  }
  *n = (int)have;
  return MT_OK;
}

extern "C" int mt_rollout_trunk_timing(mt_rollout *ro, int enable, double *sum_us, int64_t *count) {
  MT_CHECK_ARG(ro, "null argument");
  double total = 0.0;
  for (size_t i = 0; i < ro->marks_used; ++i) {
    MT_HIP(hipEventSynchronize(ro->marks[i].second));
    float ms = 0.f;
    MT_HIP(hipEventElapsedTime(&ms, ro->marks[i].first, ro->marks[i].second));
    total += 1e3 * (double)ms;
  }
  if (sum_us) *sum_us = total;
  if (count) *count = (int64_t)ro->marks_used;
  ro->marks_used = 0;
  ro->timing = enable != 0;
  return MT_OK;
}
