// Shared helpers for the libmanette_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstring>

#include "../../include/manette_hip.h"
#include "../../include/manette_host.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace mt {

void set_error(const char *fmt, ...);

#define MT_CHECK_ARG(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::mt::set_error(__VA_ARGS__);      \
      return MT_ERR_ARG;                 \
    }                                    \
  } while (0)

#define MT_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ::mt::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                      \
      return MT_ERR_HIP;                                                              \
    }                                                                                 \
  } while (0)

// Check the launch that was just issued.
#define MT_LAUNCHED() MT_HIP(hipGetLastError())

// Launch window (mt_launch_window): off by default. When on, the grouped launches (launch_group) and
// the loss kernel are numbered from 0 in issue order and only those in [first, first + count) are
// issued — the rest return MT_OK without launching — so one backward call can be captured as
// several graphs (its data-parallel gradient buckets) or timed launch by launch (bench.py).
extern bool g_win_on;
extern int g_win_first, g_win_count, g_win_index;
__host__ inline bool launch_allowed() {
  if (!g_win_on) return true;
  const int i = g_win_index++;
  return i >= g_win_first && (g_win_count < 0 || i < g_win_first + g_win_count);
}

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// Wave-wide (64 lanes) reductions, every lane receiving the result, in a fixed order: DPP within
// each row of 16 lanes (quad swaps, then rotations by 4 and 8 — register-speed lane moves, where a
// ds_bpermute shuffle costs an LDS round trip per step), then the 4 row results read into scalar
// registers and combined as (r0 + r1) + (r2 + r3). All 64 lanes must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x124>(v);  // row_ror:4
  v += dpp_mov<0x128>(v);  // row_ror:8
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x124>(v));
  v = fmaxf(v, dpp_mov<0x128>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// A3 perf mode sampler: counter-based uniforms (splitmix64 of seed, GLOBAL row, per-row counter),
// inverse CDF over (p - epsneg(float32)) accumulated in double — the standalone sample kernel
// and the fused rollout heads kernel share it so both draw identical indices. The row is the
// global env id (local row + row0 = the rank's env offset), so a data-parallel rank draws exactly
// what a single process owning all envs would draw for the same env.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void row_uniforms(uint64_t seed, int b, uint64_t c, double *ua, double *ur) {
  const uint64_t h = mix64(seed ^ mix64(((uint64_t)b << 40) ^ c));
  const uint64_t h2 = mix64(h ^ 0x9e3779b97f4a7c15ULL);
  *ua = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  *ur = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ int draw_index(const float *p, int n, double u) {
  const double epsneg = 5.9604644775390625e-08;  // np.finfo(np.float32).epsneg
  double cum = 0.0;
  for (int j = 0; j < n - 1; ++j) {
    cum += (double)(p[j] - (float)epsneg);
    if (u < cum) return j;
  }
  return n - 1;
}

__device__ __forceinline__ void sample_row(const float *pa, int A, const float *pr, int R, uint64_t seed,
                                           int b, int row0, uint64_t *counters, int *a, int *r) {
  const uint64_t c = counters[b];
  counters[b] = c + 1;
  double ua, ur;
  row_uniforms(seed, b + row0, c, &ua, &ur);
  *a = draw_index(pa, A, ua);
  *r = draw_index(pr, R, ur);
}

// Rollout-path sampling fused into the heads kernel (mt_rollout_step): indices to device
// buffers and, when pair != null, to a host-mapped [2][B] pair.
struct SampleArgs {
  uint64_t seed;
  uint64_t *counters;
  int32_t *a_idx, *r_idx, *pair;
  // optional: ready[b] = seq is stored (system scope, after the pair) once row b's pair is written,
  // so a host polling pinned memory sees the pair without an event query (mt_rollout_step)
  uint32_t *ready = nullptr;
  uint32_t seq = 0;
  // optional, replaces pair + ready: one 8-byte store per row into host-mapped memory,
  // lo = (seq16 << 16) | a, hi = (seq16 << 16) | r (seq16 = seq & 0xffff): both halves carry the
  // tag, so a host that sees the tag in both has the pair, with no fence on the device side
  uint64_t *packed = nullptr;
  int32_t row0 = 0;  // global env id of row 0 (the rank's env offset): the uniforms hash row0 + b
  // replayed rollout graph (mt_rollout_step): the kernel arguments are fixed at capture, so the
  // per-rollout sequence numbers live in device memory: seq = *seq_base + seq (read at kernel
  // start); advance (bootstrap heads, no draw): block 0 adds advance_by to advance[0] and
  // advance[1] once every reader of this rollout has run (the next replay's bases)
  const uint32_t *seq_base = nullptr;
  uint32_t *advance = nullptr;
  uint32_t advance_by = 0;
};

}  // namespace mt

struct mt_net;
namespace mt {
// Rows [row0, row0 + batch) of a train workspace sized for `rows` rows: an inference forward
// given one leaves its activations there, so the update's mt_loss_backward needs no forward.
struct TrainRows {
  float *ws;
  size_t ws_bytes;
  int rows, row0;
};
// A2 stacking source of the NIPS conv kernel (trunk_fused.h): new state = prev shifted by p
// channels + the p newest final frames; push j of env e is the 84x84xD frame at
// frames + (4e + j) * 7056 D (the runner's fixed staging slots, or their HBM copy made by
// mt_rollout_step's pull kernel).
struct StackSrc {
  const uint8_t *prev;    // state slot t [B][84][84][C] (HBM)
  const uint8_t *frames;  // the pushes' final frames: HBM, or the device address of the pinned staging
  const int32_t *count;   // push_count [B]; NULL (and no ready words): no pushes (out = a copy of prev)
  uint8_t *out;           // state slot t + 1 (the forward's input)
  // in-kernel pull (mt_rollout_step's stacking chain): env e's frames are read from the pinned
  // staging itself once its emulator thread has published it, ready[e * MH_READY_STRIDE] =
  // (tag << 3) | push count
  // (device address of the host-mapped words, mh_runner_set_ready); bounded wait, status <- 1 on
  // timeout. count is then unused.
  const uint32_t *ready = nullptr;
  uint32_t tag = 0;
  uint32_t *status = nullptr;
  // replayed rollout graph: the tag waited for is (*tag_base + tag) & 0x1fffffff (device memory,
  // advanced by the graph's bootstrap heads kernel, SampleArgs::advance)
  const uint32_t *tag_base = nullptr;
};

// 16 bytes at byte offset `off` of a host-published buffer, where [lo, hi) is the byte range
// published together with them: a chunk whose 128-B cache line also holds bytes outside that
// range (published at another time, possibly after the line was fetched) is read with two
// system-scope 8-byte loads, never served from a non-coherent cached line; any other chunk with a
// plain 16-B load (its line is first touched after the publication; lines cached by an earlier
// launch are dropped by each dispatch's system-scope acquire).
__device__ __forceinline__ uint4 ld_published16(const uint8_t *base, size_t off, size_t lo, size_t hi) {
  const size_t line = off & ~(size_t)127;
  if (line >= lo && line + 128 <= hi) return *reinterpret_cast<const uint4 *>(base + off);
  const uint64_t *p = reinterpret_cast<const uint64_t *>(base + off);
  const uint64_t x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
}

// Lane 0: wait (bounded, ~2 s of s_memrealtime at 100 MHz) for ready[e * MH_READY_STRIDE] >> 3 == tag
// (one 128-B line per env, include/manette_host.h); returns the
// push count (ready & 7), or -1 after recording a timeout in *status. System-scope relaxed polls
// (they bypass the non-coherent caches) with s_sleep between them.
__device__ __forceinline__ int wait_published(const uint32_t *ready, int e, uint32_t tag, uint32_t *status) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t v;
  while (((v = __hip_atomic_load(ready + (size_t)e * MH_READY_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >> 3) !=
         tag) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      if (status) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return -1;
    }
  }
  return (int)(v & 7u);
}
// forward (mt_forward) with the A3 draw fused into the heads kernel; smp, tr and st may be null.
// st (inference only; NIPS, gray NATURE, PWYX): the conv1 launch first stacks the new state
// st->out (== obs) from st->prev and the pushed frames (mt_preprocess_resized's op, fused into the
// forward; PWYX: dconv.h launch_stack_conv1 with the workspace's counter region).
// marks (optional, two events): recorded around the trunk launches (convs + dense layer; not the
// heads), so a caller can time the trunk kernels where they really run (mt_rollout_trunk_timing).
int forward_sample(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                   size_t ws_bytes, float *v, float *pi, float *rep, const SampleArgs *smp, bool infer,
                   hipStream_t stream, const TrainRows *tr = nullptr, const StackSrc *st = nullptr,
                   const hipEvent_t *marks = nullptr);
// the bootstrap forward without heads (net.hip forward_boot_impl): trunk + dense slabs in ws
int forward_boot(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws, size_t ws_bytes,
                 hipStream_t stream, const StackSrc *st = nullptr, uint32_t *advance = nullptr,
                 uint32_t advance_by = 0);
// the native rollout's LSTM macro-step forward (lstm.h lstm_step_fwd_impl; mt_lstm_step_forward)
// st / sync: step t > 0 of the pipelined rollout stacks its new rows in its conv1 launch (lstm.h,
// dconv.h launch_stack_conv1), sync = stack_conv1_sync_words(E) zeroed device words
constexpr int stack_conv1_sync_words(int E) { return 32 + 32 * E; }  // 128-B lines: tiles done, env e stacked
int lstm_step_forward(const mt_net *net, const float *params, const uint8_t *fstore, int t, int E, int T,
                      int32_t *nz, const float *over, void *ws, size_t ws_bytes, float *v, float *pi, float *rep,
                      const SampleArgs *smp, hipStream_t stream, const hipEvent_t *marks = nullptr,
                      const StackSrc *st = nullptr, uint32_t *sync = nullptr);
}  // namespace mt
