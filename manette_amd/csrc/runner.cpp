// Native emulator runner (host cores) — see include/manette_host.h.
//
// Reference: runners.py:7-50 (np.split of the envs over `ew` workers, one go-Queue per
// worker, one barrier Queue) and emulator_runner.py:19-42 (per env: Action, next(), repeats
// while not terminal, reward sum, reset on terminal). Here the workers are persistent threads
// released by a generation counter and joined by an arrival counter (spin, then futex wait via
// std::atomic::wait), so a macro-step costs a few microseconds of synchronisation instead of
// 2*ew Queue round trips. Compact staging runs a step in two phases:
//   A: each worker steps its envs and records which screens each env pushed (last <= 4);
//   main: prefix sum of push counts -> compact staging offsets;
//   B: each worker copies its envs' screens into the staging buffer (pinned, H2D'd whole).
// Pooled staging (MH_RUNNER_POOLED) stages max(f0, f1) of a push's two screens — the emulator's
// frame pool — so one screen per push crosses PCIe. Resized staging (MH_RUNNER_RESIZED) also
// applies the nearest 84x84 resize on the host (SSE max + pshufb column gather), so only the
// final 7 KB frame of each push crosses PCIe (3.8x fewer bytes than the 84 staged rows of 2
// screens) and the GPU only stacks it.
// Fixed-slot staging (MH_RUNNER_FIXED_SLOTS) does A and B in one phase: env e's screens go to
// slots [4e, 4e+n), read in place by the GPU.
// In-place frames (mh_runner_step_frames) copies nothing: each worker writes, per env, the bank
// indices of the screens its pushes produced, and the GPU reads those screens where the
// emulators left them (a pinned, device-mapped bank).
#include <tmmintrin.h>
#include <xmmintrin.h>

#include <algorithm>
#include <climits>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

#include "../../include/manette_host.h"

namespace {

thread_local char g_err[512] = "";
void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

inline void cpu_relax() { __builtin_ia32_pause(); }

struct Env {
  const uint8_t *screens;  // [ring][frame_bytes]
  const float *rewards;    // [reward_len]
  int64_t k = 0;           // pushes so far (next() + reset pushes)
  int32_t steps = 0;       // next() calls in the current episode
  int64_t last[4];         // k of the last pushes, ring
  int npush = 0;           // pushes in the current macro-step (uncapped)
};

}  // namespace

struct mh_runner {
  int E = 0, W = 0;
  std::vector<int32_t> tab;
  int ring = 0;
  size_t fb = 0;        // bytes of one emulator screen (210 rows)
  size_t row_bytes = 0;
  std::vector<int32_t> rows;  // staged rows (empty = whole screen)
  size_t sfb = 0;       // bytes of one staged screen
  int reward_len = 0, episode_len = 0;
  std::vector<Env> env;
  std::vector<std::thread> threads;
  // job
  std::atomic<uint32_t> gen{0};
  std::atomic<int> arrived{0};
  std::atomic<bool> quit{false};
  bool fixed = false;
  bool pooled = false;  // stage max(f0, f1) of each push (one screen per slot)
  bool resized = false;  // stage the final 84x84 frame of each push (pool + nearest resize)
  int depth = 1;
  // resize: source rows whose lines are prefetched ahead of the row being gathered (MH_PREFETCH_ROWS,
  // default 1; the synthetic screens come from a 2 MB ring per env, so each push's rows miss the caches)
  int prefetch_rows = 1;
  std::vector<int32_t> cols;             // resize column LUT (84)
  // resize column gather, per 16-byte output chunk c of a row (84*depth bytes): the source bytes
  // lie in [chunk_base[c], chunk_base[c] + 48); shuf[c][v] picks them out of source vector v
  static constexpr int kMaxChunks = 16, kSrcVecs = 3;
  alignas(16) uint8_t shuf[kMaxChunks][kSrcVecs][16];
  int chunk_base[kMaxChunks];
  int nchunks = 0;

  // d (16-byte aligned, n a multiple of 16 — a final frame: 7056 * depth) <- s with streaming
  // stores; the caller fences (sfence) before publishing d
  static void stream_copy(uint8_t *d, const uint8_t *s, size_t n) {
    for (size_t x = 0; x < n; x += 16)
      _mm_stream_si128(reinterpret_cast<__m128i *>(d + x), _mm_load_si128(reinterpret_cast<const __m128i *>(s + x)));
  }

  // FramePool max + nearest resize of one push into its 84x84xdepth staging frame
  // (atari_emulator.py:79-88 + the imresize of :113-124): rows[q] / cols[x] are the LUTs. Per
  // output row: SSE max of the two source rows into a buffer, then each 16-byte output chunk is
  // OR-ed from pshufb of up to 3 source vectors (gray and RGB alike); the source lines of the row
  // PD rows ahead are prefetched while this one is gathered.
  void resize_push(uint8_t *d, const uint8_t *s0, const uint8_t *s1) const {
    const int rb = (int)row_bytes, ob = 84 * depth;
    alignas(16) uint8_t m[480 + 64];
    for (int x = rb; x < rb + 64; x += 16) _mm_store_si128(reinterpret_cast<__m128i *>(m + x), _mm_setzero_si128());
    const int PD = prefetch_rows;  // rows prefetched ahead
    auto prefetch_row = [&](int q) {
      const uint8_t *na = s0 + (size_t)rows[q] * row_bytes, *nb = s1 + (size_t)rows[q] * row_bytes;
      for (int x = 0; x < rb; x += 64) {
        _mm_prefetch(reinterpret_cast<const char *>(na + x), _MM_HINT_T0);
        _mm_prefetch(reinterpret_cast<const char *>(nb + x), _MM_HINT_T0);
      }
    };
    for (int q = 0; q < PD; ++q) prefetch_row(q);
    for (int q = 0; q < 84; ++q) {
      const uint8_t *a = s0 + (size_t)rows[q] * row_bytes, *b = s1 + (size_t)rows[q] * row_bytes;
      if (q + PD < 84) prefetch_row(q + PD);
      for (int x = 0; x < rb; x += 16)
        _mm_store_si128(reinterpret_cast<__m128i *>(m + x),
                        _mm_max_epu8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(a + x)),
                                     _mm_loadu_si128(reinterpret_cast<const __m128i *>(b + x))));
      uint8_t *o = d + (size_t)q * ob;
      for (int c = 0; c < nchunks; ++c) {
        const uint8_t *src = m + chunk_base[c];
        __m128i v = _mm_setzero_si128();
#pragma GCC unroll 3
        for (int k = 0; k < kSrcVecs; ++k)
          v = _mm_or_si128(v, _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 16 * k)),
                                               _mm_load_si128(reinterpret_cast<const __m128i *>(shuf[c][k]))));
        if (16 * c + 16 <= ob) {
          _mm_storeu_si128(reinterpret_cast<__m128i *>(o + 16 * c), v);
        } else {
          alignas(16) uint8_t t[16];
          _mm_store_si128(reinterpret_cast<__m128i *>(t), v);
          std::memcpy(o + 16 * c, t, ob - 16 * c);
        }
      }
    }
  }

  int phase = 0;  // 0 = reset, 1 = step A (+ B when fixed), 2 = copy B
  const int32_t *a_idx = nullptr, *r_idx = nullptr;
  uint8_t *staging = nullptr;
  int32_t *push_offset = nullptr, *push_count = nullptr;
  int32_t *frame_idx = nullptr;  // in-place mode: [E][8] bank frame indices (else null)
  float *reward = nullptr, *over = nullptr;
  // per-env ready words (fixed slots): env i's staging + push count are complete once
  // ready[i * MH_READY_STRIDE] == (ready_value << 3) | push count (mh_runner_set_ready); the GPU pulls env i while
  // the others are still being emulated
  uint32_t *ready = nullptr;
  uint32_t ready_value = 0;
  bool busy = false;  // mh_runner_step_begin dispatched, mh_runner_step_end not yet called
  // host-phase split of a step (mh_runner_stats): worker time in stage_env (frame pool + resize +
  // the streaming copy into the staging) and worker time in the whole phase, summed over workers
  // (own 128-B block: bumped by each worker at the end of its phase, while others still read the
  // per-step fields above)
  alignas(128) std::atomic<int64_t> stage_ns{0};
  std::atomic<int64_t> busy_ns{0}, stat_steps{0};
  char stats_pad[128 - 3 * sizeof(std::atomic<int64_t>)];
  bool nt_stores = true;  // resized frames: streaming stores (plain stores measured the same on the box)

  // Static env blocks: a worker keeps the same envs every step. (Round 6 dealt the envs of a
  // per-env-publication step dynamically, the next env to the first free worker, to balance FiGAR's
  // 1-4 pushes per env: the staging time per worker doubled on the box — Breakout 44 -> 80 us, Pong
  // 7.5 -> 9.5-12.7 us, profiles/r06h — each env's screens and state were then read by a different
  // core, often on another CCD, instead of from the L3 its worker had left them in.)
  int block_begin(int w) const { return (int)((int64_t)E * w / W); }
  int block_end(int w) const { return (int)((int64_t)E * (w + 1) / W); }

  void push(Env &e) {
    e.last[e.npush & 3] = e.k;
    e.npush++;
    e.k++;
  }
  // emulator.next(a): returns (reward, terminal); the screens are those of push k.
  float next(Env &e, bool *term) {
    const float r = e.rewards[e.k % reward_len];
    push(e);
    e.steps++;
    *term = e.steps >= episode_len;
    return r;
  }
  void initial(Env &e) {  // get_initial_state(): 4 noop action_repeats
    for (int i = 0; i < 4; ++i) push(e);
    e.steps = 0;
  }

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  void run_phase(int w) {
    const int64_t t0 = now_ns();
    int64_t st = 0;
    run_phase_(w, st);
    busy_ns.fetch_add(now_ns() - t0, std::memory_order_relaxed);
    stage_ns.fetch_add(st, std::memory_order_relaxed);
    if (w == 0 && phase == 1) stat_steps.fetch_add(1, std::memory_order_relaxed);
  }
  // a stage_env call, timed into st
  void stage_timed(int i, int64_t &st) {
    const int64_t t0 = now_ns();
    stage_env(i);
    st += now_ns() - t0;
  }
  void run_phase_(int w, int64_t &st) {
    const int b0 = block_begin(w), b1 = block_end(w);
    if (phase == 0) {
      for (int i = b0; i < b1; ++i) {
        env[i].npush = 0;
        initial(env[i]);
      }
    } else if (phase == 1) {
      const bool per_env = ready && fixed && !frame_idx;
      for (int i = b0; i < b1; ++i) {
        Env &e = env[i];
        e.npush = 0;
        int left = tab[r_idx[i]];  // Action.init_from_list (exploration_policy.py:13-17)
        bool term = false;
        float rs = next(e, &term);  // emulator_runner.py:27
        if (term) initial(e);       // :28-29
        while (left > 0 && !term) {  // :33-40 (float32 accumulation of the shared array)
          --left;
          rs += next(e, &term);
          if (term) initial(e);
        }
        reward[i] = rs;
        over[i] = term ? 1.f : 0.f;
        if (fixed) {
          push_offset[i] = 4 * i;
          push_count[i] = std::min(e.npush, 4);
        }
        if (per_env) {  // stage env i now and publish it (sfence: the streaming stores first)
          stage_timed(i, st);
          _mm_sfence();
          __atomic_store_n(ready + (size_t)i * MH_READY_STRIDE, (ready_value << 3) | (uint32_t)std::min(e.npush, 4),
                           __ATOMIC_RELEASE);
        }
      }
      if (per_env) return;
    }
    if (frame_idx) {  // in place: record where the pushed screens are, oldest first
      for (int i = b0; i < b1; ++i) {
        const Env &e = env[i];
        const int n = std::min(e.npush, 4);
        push_count[i] = n;
        for (int j = 0; j < n; ++j) {
          const int64_t kk = e.last[(e.npush - n + j) & 3];
          for (int f = 0; f < 2; ++f) frame_idx[i * 8 + 2 * j + f] = (int32_t)(i * ring + (2 * kk + f) % ring);
        }
      }
      return;
    }
    if (phase == 0 || phase == 2 || fixed) {
      for (int i = b0; i < b1; ++i) stage_timed(i, st);
      _mm_sfence();  // streaming stores visible before the phase is reported done
    }
  }

  // the pushes of env i into the staging (resized / pooled / raw rows)
  void stage_env(int i) {
    const Env &e = env[i];
    const int n = std::min(e.npush, 4);
    for (int j = 0; j < n; ++j) {
      const int64_t kk = e.last[(e.npush - n + j) & 3];
      if (resized) {
        // resized into an L1-resident buffer, then streamed to the staging with non-temporal
        // stores: the lines never sit modified in this core's cache, so the GPU reading them
        // over PCIe (while this thread works on the next env) does not snoop them out of it
        uint8_t *dst = staging + (size_t)(push_offset[i] + j) * sfb;
        if (!nt_stores) {
          resize_push(dst, e.screens + (size_t)((2 * kk) % ring) * fb, e.screens + (size_t)((2 * kk + 1) % ring) * fb);
          continue;
        }
        alignas(64) uint8_t buf[84 * 84 * 3 + 64];
        resize_push(buf, e.screens + (size_t)((2 * kk) % ring) * fb, e.screens + (size_t)((2 * kk + 1) % ring) * fb);
        stream_copy(dst, buf, sfb);
        continue;
      }
      if (pooled) {  // FramePool max (atari_emulator.py:79-88) of the staged rows, on the host
        uint8_t *d = staging + (size_t)(push_offset[i] + j) * sfb;
        const uint8_t *s0 = e.screens + (size_t)((2 * kk) % ring) * fb;
        const uint8_t *s1 = e.screens + (size_t)((2 * kk + 1) % ring) * fb;
        const size_t nr = rows.empty() ? 210 : rows.size();
        for (size_t q = 0; q < nr; ++q) {
          const size_t so = (rows.empty() ? q : (size_t)rows[q]) * row_bytes;
          uint8_t *dq = d + q * row_bytes;
          // SSE max, streamed to the staging (non-temporal: the GPU reads these lines over PCIe while
          // this thread works on, and must not snoop them out of its cache — as the resized frames)
          for (size_t x = 0; x < row_bytes; x += 16)
            _mm_stream_si128(reinterpret_cast<__m128i *>(dq + x),
                             _mm_max_epu8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(s0 + so + x)),
                                          _mm_loadu_si128(reinterpret_cast<const __m128i *>(s1 + so + x))));
        }
        continue;
      }
      uint8_t *dst = staging + (size_t)(push_offset[i] + j) * 2 * sfb;
      for (int f = 0; f < 2; ++f) {
        const uint8_t *src = e.screens + (size_t)((2 * kk + f) % ring) * fb;
        uint8_t *d = dst + f * sfb;
        if (rows.empty()) {
          std::memcpy(d, src, fb);
        } else {
          for (size_t q = 0; q < rows.size(); ++q)
            std::memcpy(d + q * row_bytes, src + (size_t)rows[q] * row_bytes, row_bytes);
        }
      }
    }
  }

  // Idle workers spin for kSpinUs of wall time before sleeping on the generation word: the longest
  // regular pause between two emulator steps is the update (the learner's backward + RMSProp and
  // the next rollout's first forward, ~0.1 ms), and a futex wake-up there cost ~10 us on the
  // critical path of every update (a fixed spin count measured ~85 us of pause on the box).
  // mh_runner_set_threads lowers it when the host's cores are oversubscribed (several ranks' worker
  // pools on one node), so an idle pool yields its cores to the other ranks' emulator threads.
  static constexpr int64_t kSpinUs = 2000;
  std::atomic<int64_t> spin_us{kSpinUs};
  void worker(int w) {
    uint32_t seen = 0;
    for (;;) {
      // spin, then sleep on the generation word
      int spins = 0;
      uint32_t g;
      auto t0 = std::chrono::steady_clock::now();
      const int64_t spin = spin_us.load(std::memory_order_relaxed);
      while ((g = gen.load(std::memory_order_acquire)) == seen) {
        cpu_relax();
        if ((++spins & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin))
          gen.wait(seen, std::memory_order_acquire);
      }
      seen = g;
      if (quit.load(std::memory_order_acquire)) return;
      run_phase(w);
      if (arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == W) arrived.notify_one();
    }
  }

  void dispatch(int ph) {
    dispatch_begin(ph);
    dispatch_wait();
  }
  void dispatch_begin(int ph) {
    phase = ph;
    arrived.store(0, std::memory_order_relaxed);
    gen.fetch_add(1, std::memory_order_acq_rel);
    gen.notify_all();
  }
  void dispatch_wait() {
    int spins = 0;
    int a;
    while ((a = arrived.load(std::memory_order_acquire)) != W) {
      if (++spins < 20000) cpu_relax();
      else arrived.wait(a, std::memory_order_acquire);
    }
  }

  int compact(int *total) {
    int off = 0;
    for (int i = 0; i < E; ++i) {
      const int n = std::min(env[i].npush, 4);
      push_offset[i] = off;
      push_count[i] = n;
      off += n;
    }
    *total = off;
    return 0;
  }
};

extern "C" const char *mh_last_error(void) { return g_err; }

extern "C" int mh_runner_create(int n_envs, int n_workers, const int32_t *tab_rep, int n_reps,
                                const uint8_t *screens, int ring, size_t frame_bytes,
                                const float *rewards, int reward_len, int episode_len,
                                const int32_t *row_select, int n_rows, int flags, mh_runner **out) {
  if (!out || !tab_rep || !screens || !rewards) {
    set_error("null argument");
    return 1;
  }
  if (n_envs < 1 || n_workers < 1 || n_reps < 1 || ring < 2 || frame_bytes == 0 ||
      reward_len < 1 || episode_len < 1 || frame_bytes % 210 != 0 || n_rows < 0 ||
      (flags & ~(MH_RUNNER_FIXED_SLOTS | MH_RUNNER_POOLED | MH_RUNNER_RESIZED)) != 0) {
    set_error("bad sizes");
    return 1;
  }
  if ((flags & MH_RUNNER_POOLED) && (frame_bytes / 210) % 16 != 0) {
    set_error("pooled staging needs screen rows of a multiple of 16 bytes (SSE max)");
    return 1;
  }
  if ((flags & MH_RUNNER_RESIZED) && (n_rows != 84 || (flags & MH_RUNNER_POOLED))) {
    set_error("resized staging needs the 84-row row_select (and excludes pooled)");
    return 1;
  }
  for (int q = 0; q < n_rows; ++q)
    if (!row_select || row_select[q] < 0 || row_select[q] >= 210) {
      set_error("row_select[%d] out of [0,210)", q);
      return 1;
    }
  for (int i = 0; i < n_reps; ++i)
    if (tab_rep[i] < 0) {
      set_error("negative repetition");
      return 1;
    }
  mh_runner *r = new mh_runner();
  r->E = n_envs;
  r->W = std::min(n_workers, n_envs);
  r->fixed = (flags & MH_RUNNER_FIXED_SLOTS) != 0;
  r->pooled = (flags & MH_RUNNER_POOLED) != 0;
  r->resized = (flags & MH_RUNNER_RESIZED) != 0;
  r->tab.assign(tab_rep, tab_rep + n_reps);
  r->ring = ring;
  r->fb = frame_bytes;
  r->row_bytes = frame_bytes / 210;
  r->depth = (int)(r->row_bytes / 160);
  if (n_rows > 0) r->rows.assign(row_select, row_select + n_rows);
  r->sfb = n_rows > 0 ? (size_t)n_rows * r->row_bytes : frame_bytes;
  if (r->resized) r->sfb = (size_t)84 * 84 * r->depth;
  r->reward_len = reward_len;
  r->episode_len = episode_len;
  if (const char *pd = std::getenv("MH_PREFETCH_ROWS")) r->prefetch_rows = std::max(0, std::min(84, std::atoi(pd)));
  r->env.resize(n_envs);
  for (int i = 0; i < n_envs; ++i) {
    r->env[i].screens = screens + (size_t)i * ring * frame_bytes;
    r->env[i].rewards = rewards + (size_t)i * reward_len;
  }
  for (int w = 0; w < r->W; ++w) r->threads.emplace_back([r, w] { r->worker(w); });
  *out = r;
  return 0;
}

extern "C" int mh_runner_set_threads(mh_runner *r, const int32_t *cpus, int n_cpus, int spin_us) {
  if (!r || (n_cpus > 0 && !cpus) || n_cpus < 0 || spin_us < 0) {
    set_error("null argument or negative count");
    return 1;
  }
  for (int i = 0; i < n_cpus; ++i)
    if (cpus[i] < 0 || cpus[i] >= CPU_SETSIZE) {
      set_error("cpu %d out of range", cpus[i]);
      return 1;
    }
  for (int w = 0; w < n_cpus && w < r->W; ++w) {  // (n_cpus < W: workers W.. keep their mask)
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpus[w], &set);
    const int rc = pthread_setaffinity_np(r->threads[w].native_handle(), sizeof(set), &set);
    if (rc != 0) {
      set_error("pthread_setaffinity_np(worker %d, cpu %d) failed: %d", w, cpus[w], rc);
      return 1;
    }
  }
  r->spin_us.store(spin_us, std::memory_order_relaxed);
  return 0;
}

extern "C" int mh_runner_stats(mh_runner *r, double *out, int n, int reset) {
  if (!r || (n > 0 && !out)) {
    set_error("null argument");
    return 1;
  }
  const double steps = (double)r->stat_steps.load(), w = (double)r->W;
  const double v[3] = {steps > 0 ? 1e-3 * (double)r->stage_ns.load() / (w * steps) : 0.0,
                       steps > 0 ? 1e-3 * (double)r->busy_ns.load() / (w * steps) : 0.0, steps};
  for (int i = 0; i < n && i < 3; ++i) out[i] = v[i];
  if (reset) {
    r->stage_ns.store(0);
    r->busy_ns.store(0);
    r->stat_steps.store(0);
  }
  return 0;
}

extern "C" int mh_runner_thread_cpus(mh_runner *r, int32_t *out, int n) {
  if (!r || (n > 0 && !out)) {
    set_error("null argument");
    return -1;
  }
  for (int w = 0; w < n && w < r->W; ++w) {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (pthread_getaffinity_np(r->threads[w].native_handle(), sizeof(set), &set) != 0) {
      set_error("pthread_getaffinity_np(worker %d) failed", w);
      return -1;
    }
    out[w] = CPU_COUNT(&set) == 1 ? -2 : -1;  // -1: several cpus allowed
    for (int c = 0; c < CPU_SETSIZE && out[w] == -2; ++c)
      if (CPU_ISSET(c, &set)) out[w] = c;
  }
  return r->W;
}

extern "C" int mh_runner_set_col_lut(mh_runner *r, const int32_t *col_lut, int n_cols) {
  if (!r || !col_lut) {
    set_error("null argument");
    return 1;
  }
  if (!r->resized || n_cols != 84 || r->row_bytes % 160 != 0 || (r->depth != 1 && r->depth != 3)) {
    set_error("col LUT needs a resized-staging runner and 84 columns");
    return 1;
  }
  for (int x = 0; x < 84; ++x)
    if (col_lut[x] < 0 || col_lut[x] >= 160 || (x && col_lut[x] < col_lut[x - 1])) {
      set_error("col_lut[%d] = %d out of [0,160) or not increasing", x, col_lut[x]);
      return 1;
    }
  r->cols.assign(col_lut, col_lut + 84);
  const int depth = r->depth, ob = 84 * depth;
  r->nchunks = (ob + 15) / 16;
  if (r->nchunks > mh_runner::kMaxChunks || (int)r->row_bytes + 64 > 480 + 64) {
    set_error("resize supports depth 1 or 3");
    return 1;
  }
  for (int c = 0; c < r->nchunks; ++c) {
    const int b0 = 16 * c;
    const int base = col_lut[b0 / depth] * depth + b0 % depth;  // source byte of the chunk's first byte
    r->chunk_base[c] = base;
    for (int k = 0; k < 16; ++k) {
      const int ob_k = b0 + k;
      const int off = ob_k < ob ? col_lut[ob_k / depth] * depth + ob_k % depth - base : -1;
      if (off >= 16 * mh_runner::kSrcVecs) {
        set_error("resize chunk %d spans more than %d source bytes", c, 16 * mh_runner::kSrcVecs);
        return 1;
      }
      for (int v = 0; v < mh_runner::kSrcVecs; ++v)
        r->shuf[c][v][k] = (off >= 16 * v && off < 16 * v + 16) ? (uint8_t)(off - 16 * v) : 0x80;
    }
  }
  return 0;
}

extern "C" void mh_runner_destroy(mh_runner *r) {
  if (!r) return;
  r->quit.store(true, std::memory_order_release);
  r->gen.fetch_add(1, std::memory_order_acq_rel);
  r->gen.notify_all();
  for (auto &t : r->threads) t.join();
  delete r;
}

extern "C" int mh_runner_reset(mh_runner *r, uint8_t *staging, int32_t *push_offset,
                               int32_t *push_count, int *total_pushes) {
  if (!r || !staging || !push_offset || !push_count || !total_pushes) {
    set_error("null argument");
    return 1;
  }
  if ((r->pooled || r->resized) && (reinterpret_cast<uintptr_t>(staging) & 15) != 0) {
    set_error("pooled / resized staging must be 16-byte aligned (streaming stores)");
    return 1;
  }
  r->staging = staging;
  r->push_offset = push_offset;
  r->push_count = push_count;
  for (int i = 0; i < r->E; ++i) {
    push_offset[i] = 4 * i;
    push_count[i] = 4;
  }
  *total_pushes = 4 * r->E;
  r->dispatch(0);
  return 0;
}

extern "C" int mh_runner_set_ready(mh_runner *r, uint32_t *ready, uint32_t value) {
  if (!r) {
    set_error("null argument");
    return 1;
  }
  if (ready && !(r->fixed && r->resized)) {
    set_error("per-env ready words need fixed, resized staging");
    return 1;
  }
  r->ready = ready;
  r->ready_value = value;
  return 0;
}

extern "C" int mh_runner_step_begin(mh_runner *r, const int32_t *a_idx, const int32_t *r_idx,
                                    uint8_t *staging, int32_t *push_offset, int32_t *push_count,
                                    float *reward, float *over) {
  if (!r || !a_idx || !r_idx || !staging || !push_offset || !push_count || !reward || !over) {
    set_error("null argument");
    return 1;
  }
  if (r->busy) {
    set_error("a step is already in flight");
    return 1;
  }
  if ((r->pooled || r->resized) && (reinterpret_cast<uintptr_t>(staging) & 15) != 0) {
    set_error("pooled / resized staging must be 16-byte aligned (streaming stores)");
    return 1;
  }
  const int nr = (int)r->tab.size();
  for (int i = 0; i < r->E; ++i)
    if (r_idx[i] < 0 || r_idx[i] >= nr) {
      set_error("r_idx[%d] = %d out of range [0,%d)", i, r_idx[i], nr);
      return 1;
    }
  if (r->resized && ((uintptr_t)staging & 15)) {
    set_error("resized staging must be 16-byte aligned");
    return 1;
  }
  r->a_idx = a_idx;
  r->r_idx = r_idx;
  r->staging = staging;
  r->push_offset = push_offset;
  r->push_count = push_count;
  r->reward = reward;
  r->over = over;
  r->busy = true;
  r->dispatch_begin(1);
  return 0;
}

extern "C" int mh_runner_step_end(mh_runner *r, int *total_pushes) {
  if (!r || !total_pushes) {
    set_error("null argument");
    return 1;
  }
  if (!r->busy) {
    set_error("no step in flight");
    return 1;
  }
  r->dispatch_wait();
  r->busy = false;
  if (r->fixed) {
    *total_pushes = 4 * r->E;
    return 0;
  }
  r->compact(total_pushes);
  r->dispatch(2);
  return 0;
}

extern "C" int mh_runner_step(mh_runner *r, const int32_t *a_idx, const int32_t *r_idx,
                              uint8_t *staging, int32_t *push_offset, int32_t *push_count,
                              float *reward, float *over, int *total_pushes) {
  if (!r || !a_idx || !r_idx || !staging || !push_offset || !push_count || !reward || !over ||
      !total_pushes) {
    set_error("null argument");
    return 1;
  }
  if (r->busy) {
    set_error("a step is already in flight");
    return 1;
  }
  if ((r->pooled || r->resized) && (reinterpret_cast<uintptr_t>(staging) & 15) != 0) {
    set_error("pooled / resized staging must be 16-byte aligned (streaming stores)");
    return 1;
  }
  const int nr = (int)r->tab.size();
  for (int i = 0; i < r->E; ++i)
    if (r_idx[i] < 0 || r_idx[i] >= nr) {
      set_error("r_idx[%d] = %d out of range [0,%d)", i, r_idx[i], nr);
      return 1;
    }
  if (r->resized && ((uintptr_t)staging & 15)) {
    set_error("resized staging must be 16-byte aligned");
    return 1;
  }
  r->a_idx = a_idx;
  r->r_idx = r_idx;
  r->staging = staging;
  r->push_offset = push_offset;
  r->push_count = push_count;
  r->reward = reward;
  r->over = over;
  r->dispatch(1);
  if (r->fixed) {
    *total_pushes = 4 * r->E;
    return 0;
  }
  r->compact(total_pushes);
  r->dispatch(2);
  return 0;
}

extern "C" int mh_runner_reset_frames(mh_runner *r, int32_t *frame_idx, int32_t *push_count) {
  if (!r || !frame_idx || !push_count) {
    set_error("null argument");
    return 1;
  }
  if ((int64_t)r->E * r->ring > INT32_MAX) {
    set_error("bank too large for int32 frame indices");
    return 1;
  }
  r->frame_idx = frame_idx;
  r->push_count = push_count;
  r->dispatch(0);
  r->frame_idx = nullptr;
  return 0;
}

extern "C" int mh_runner_step_frames(mh_runner *r, const int32_t *a_idx, const int32_t *r_idx,
                                     int32_t *frame_idx, int32_t *push_count, float *reward, float *over) {
  if (!r || !a_idx || !r_idx || !frame_idx || !push_count || !reward || !over) {
    set_error("null argument");
    return 1;
  }
  if ((int64_t)r->E * r->ring > INT32_MAX) {
    set_error("bank too large for int32 frame indices");
    return 1;
  }
  const int nr = (int)r->tab.size();
  for (int i = 0; i < r->E; ++i)
    if (r_idx[i] < 0 || r_idx[i] >= nr) {
      set_error("r_idx[%d] = %d out of range [0,%d)", i, r_idx[i], nr);
      return 1;
    }
  r->a_idx = a_idx;
  r->r_idx = r_idx;
  r->frame_idx = frame_idx;
  r->push_count = push_count;
  r->reward = reward;
  r->over = over;
  const bool fixed = r->fixed;
  r->fixed = false;  // no staging slots in this mode
  r->dispatch(1);
  r->fixed = fixed;
  r->frame_idx = nullptr;
  return 0;
}

extern "C" int mh_runner_env_state(const mh_runner *r, int e, int64_t *k, int32_t *steps) {
  if (!r || e < 0 || e >= r->E) {
    set_error("bad env index");
    return 1;
  }
  if (k) *k = r->env[e].k;
  if (steps) *steps = r->env[e].steps;
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Rollout bookkeeping (A8) — same semantics as manette_amd/bookkeeping.py (pinned to the
// reference's golden host-loop vectors), kept native so a macro-step needs no Python.
// ---------------------------------------------------------------------------------------------
struct mh_book {
  int E = 0, A = 0, R = 0;
  std::vector<int32_t> tab;
  std::vector<int64_t> emulator_steps;
  std::vector<float> total_reward;
  std::vector<int64_t> hist;  // [A][R]
  int64_t nb_actions = 0;
  int64_t env_offset = 0, envs_total = 0;  // data-parallel shard (mh_book_set_shard)
  struct Episode {
    int64_t step;
    float reward;
    int64_t length;
  };
  std::vector<Episode> episodes;  // FIFO
  size_t head = 0;
};

extern "C" int mh_book_create(int n_envs, int num_actions, const int32_t *tab_rep, int n_reps,
                              mh_book **out) {
  if (!out || !tab_rep || n_envs < 1 || num_actions < 1 || n_reps < 1) {
    set_error("bad argument");
    return 1;
  }
  mh_book *b = new mh_book();
  b->E = n_envs;
  b->A = num_actions;
  b->R = n_reps;
  b->tab.assign(tab_rep, tab_rep + n_reps);
  b->emulator_steps.assign(n_envs, 0);
  b->total_reward.assign(n_envs, 0.f);
  b->hist.assign((size_t)num_actions * n_reps, 0);
  b->envs_total = n_envs;
  *out = b;
  return 0;
}

extern "C" void mh_book_destroy(mh_book *b) { delete b; }

extern "C" int mh_book_step(mh_book *b, int64_t *global_step, const int32_t *a_idx,
                            const int32_t *r_idx, const float *reward, const float *over,
                            float *rewards_out, float *masks_out) {
  if (!b || !global_step || !a_idx || !r_idx || !reward || !over || !rewards_out || !masks_out) {
    set_error("null argument");
    return 1;
  }
  for (int e = 0; e < b->E; ++e) {
    const int a = a_idx[e], r = r_idx[e];
    if (a < 0 || a >= b->A || r < 0 || r >= b->R) {
      set_error("index out of range at env %d (a=%d, r=%d)", e, a, r);
      return 1;
    }
  }
  const int64_t gs0 = *global_step;
  for (int e = 0; e < b->E; ++e) {
    const float rw = reward[e];
    masks_out[e] = 1.0f - over[e];
    b->total_reward[e] += rw;
    rewards_out[e] = rw > 1.0f ? 1.0f : (rw < -1.0f ? -1.0f : rw);
    const int a = a_idx[e], r = r_idx[e];
    b->emulator_steps[e] += b->tab[r] + 1;
    b->hist[(size_t)a * b->R + r] += 1;
    b->nb_actions += r + 1;
    if (over[e] != 0.f) {
      b->episodes.push_back({gs0 + b->env_offset + e + 1, b->total_reward[e], b->emulator_steps[e]});
      b->total_reward[e] = 0.f;
      b->emulator_steps[e] = 0;
    }
  }
  *global_step = gs0 + b->envs_total;
  return 0;
}

extern "C" int mh_book_set_shard(mh_book *b, int64_t env_offset, int64_t envs_total) {
  if (!b || env_offset < 0 || envs_total < env_offset + b->E) {
    set_error("bad shard (offset %lld, total %lld)", (long long)env_offset, (long long)envs_total);
    return 1;
  }
  b->env_offset = env_offset;
  b->envs_total = envs_total;
  return 0;
}

extern "C" int mh_book_new_update(mh_book *b) {
  if (!b) {
    set_error("null argument");
    return 1;
  }
  std::fill(b->hist.begin(), b->hist.end(), 0);
  b->nb_actions = 0;
  return 0;
}

extern "C" int mh_book_histogram(const mh_book *b, int64_t *hist, int64_t *nb_actions) {
  if (!b) {
    set_error("null argument");
    return 1;
  }
  if (hist) std::copy(b->hist.begin(), b->hist.end(), hist);
  if (nb_actions) *nb_actions = b->nb_actions;
  return 0;
}

extern "C" int mh_book_pop_episodes(mh_book *b, int64_t *global_step, float *reward,
                                    int64_t *length, int max, int *n) {
  if (!b || !n) {
    set_error("null argument");
    return 1;
  }
  int k = 0;
  while (k < max && b->head < b->episodes.size()) {
    const auto &ep = b->episodes[b->head++];
    if (global_step) global_step[k] = ep.step;
    if (reward) reward[k] = ep.reward;
    if (length) length[k] = ep.length;
    ++k;
  }
  if (b->head == b->episodes.size()) {
    b->episodes.clear();
    b->head = 0;
  }
  *n = k;
  return 0;
}
