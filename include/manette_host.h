/*
 * manette_host.h — C ABI of libmanette_host.so: the native emulator runner of the PAAC hot
 * path (host cores). Replaces runners.py:7-50 + emulator_runner.py:19-42 for native emulator
 * banks: a pool of worker threads steps disjoint env blocks per macro-step (FiGAR repeats,
 * reward sums, terminal resets) and writes the screens each env pushed into ONE compact
 * pinned staging buffer that the caller hipMemcpyAsync's to HBM for mt_preprocess.
 *
 * The bank implemented here is the synthetic ALE stand-in (manette_amd/synthetic.py defines
 * it and precomputes its streams from seeded numpy RandomStates, so the Python and native
 * paths see identical screens and rewards):
 *   next(a):  push screens (ring[2k % ring], ring[(2k+1) % ring]); reward = rewards[k % L];
 *             k += 1; steps += 1; terminal = steps >= episode_len
 *   initial:  4 pushes as next(0) without reward; steps = 0   (atari_emulator.py:102-110)
 * Status codes as manette_hip.h (0 = ok); mh_last_error() describes the last failure.
 */
#ifndef MANETTE_HOST_H
#define MANETTE_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mh_runner mh_runner;

const char *mh_last_error(void);

/* screens: [n_envs][ring][frame_bytes] uint8 (frame_bytes = 210 rows x row_bytes), rewards:
 * [n_envs][reward_len] float32 (caller keeps both alive). tab_rep: FiGAR repetition table
 * (exploration_policy.py:56-62). row_select [n_rows] (or NULL / 0 for whole screens): stage only
 * these screen rows — the rows the 84x84 nearest resize reads (atari_emulator.py:85) — so a
 * push is n_rows*row_bytes per screen on PCIe instead of 210 rows.
 * flags & MH_RUNNER_FIXED_SLOTS: env e's pushes always go to staging slots [4e, 4e+count)
 * (push_offset[e] = 4e, *total_pushes = 4E) and each worker stages its envs while it steps them
 * (one worker release per macro-step) — for consumers that read the staging in place
 * (MT_ROLLOUT_ZERO_COPY). Otherwise the slots are compacted env-major (a prefix sum between
 * two worker phases) so a copy engine moves only the pushed screens. */
#define MH_RUNNER_FIXED_SLOTS 1
/* flags & MH_RUNNER_POOLED: each staging slot holds ONE screen per push, max(f0, f1) of its two
 * screens (the emulator's FramePool, atari_emulator.py:79-88), so half the bytes cross PCIe;
 * staging must hold 4*E slots of one staged screen. */
#define MH_RUNNER_POOLED 2
/* flags & MH_RUNNER_RESIZED (needs the 84-row row_select and mh_runner_set_col_lut before the
 * first reset/step): each staging slot holds the FINAL 84x84xdepth frame of a push — the frame
 * pool max and the nearest resize (atari_emulator.py:79-88, :113-124) done on the host — so
 * 7,056*depth bytes per push cross PCIe and the device only stacks it (mt_preprocess_resized). */
#define MH_RUNNER_RESIZED 4
int mh_runner_create(int n_envs, int n_workers, const int32_t *tab_rep, int n_reps,
                     const uint8_t *screens, int ring, size_t frame_bytes, const float *rewards,
                     int reward_len, int episode_len, const int32_t *row_select, int n_rows,
                     int flags, mh_runner **out);
/* Thread placement of the worker pool (one process per GPU sharing a node's cores; the reference's
 * runners.py:11-18 starts `ew` processes and leaves placement to the OS): worker w is pinned to
 * cpus[w] (w < n_cpus; the caller passes cores of its GPU's NUMA node not used by its own thread),
 * and idle workers spin spin_us microseconds of wall time before sleeping on the generation word
 * (2000 by default; the learner lowers it when the node's cores are oversubscribed). */
int mh_runner_set_threads(mh_runner *r, const int32_t *cpus, int n_cpus, int spin_us);
/* Diagnostics: out[w] = the one cpu worker w may run on, or -1 when several are allowed; returns
 * the worker count (or -1 on error). */
int mh_runner_thread_cpus(mh_runner *r, int32_t *out, int n);
/* Host-phase split of the steps since the last reset (diagnostics, bench.py): out[0] = worker time
 * in staging per worker per step (us: the frame pool + resize + the streaming copy of resized
 * staging, or the row copies of the other modes), out[1] = worker time in the whole step phase per
 * worker per step (us; the rest is the synthetic emulation and the per-env publication), out[2] =
 * steps counted. reset != 0 zeroes the counters after reading. */
int mh_runner_stats(mh_runner *r, double *out, int n, int reset);
/* The resize's column LUT (84 source columns, increasing) for MH_RUNNER_RESIZED. */
int mh_runner_set_col_lut(mh_runner *r, const int32_t *col_lut, int n_cols);
void mh_runner_destroy(mh_runner *r);

/* get_initial_state() of every env: 4 pushes each. Outputs as mh_runner_step. */
int mh_runner_reset(mh_runner *r, uint8_t *staging, int32_t *push_offset, int32_t *push_count,
                    int *total_pushes);

/* One macro-step (emulator_runner.py:24-41) of every env with action a_idx[e] repeated
 * tab_rep[r_idx[e]] more times unless the episode ends. Outputs:
 *   staging      [total_pushes][2][staged frame] ([total_pushes][staged frame] pooled): screens
 *                of the last <=4 pushes of each env,
 *                env-major, oldest first (a terminal's reset pushes included);
 *   push_offset  [E] first staging slot of env e; push_count [E] in 1..4;
 *   reward       [E] float32 sum over the repeats (shared float32 array semantics);
 *   over         [E] 1.0 if the episode ended (state is then the reset state).
 * staging must hold 4*E slots. */
int mh_runner_step(mh_runner *r, const int32_t *a_idx, const int32_t *r_idx, uint8_t *staging,
                   int32_t *push_offset, int32_t *push_count, float *reward, float *over,
                   int *total_pushes);

/* mh_runner_step split in two: _begin hands the step to the worker threads and returns at once
 * (the caller may enqueue GPU work meanwhile); _end waits for them and returns total_pushes.
 * No other runner call may come in between. */
int mh_runner_step_begin(mh_runner *r, const int32_t *a_idx, const int32_t *r_idx, uint8_t *staging,
                         int32_t *push_offset, int32_t *push_count, float *reward, float *over);
int mh_runner_step_end(mh_runner *r, int *total_pushes);

/* Per-env ready words (fixed + resized staging only; ready = NULL turns them off): during the
 * following mh_runner_step calls, the worker that steps env e stages e's pushes and its push count
 * and then stores ready[e * MH_READY_STRIDE] = (value << 3) | push_count[e] (release), so a
 * consumer polling that word (GPU kernels reading pinned, device-mapped memory: mt_rollout_step's
 * conv / pull kernels) can take env e while the other envs are still being emulated. Call before
 * every step with that step's value (compared modulo 2^29). Each env's word has a 128-B line of
 * its own (ready holds E * MH_READY_STRIDE words): a line the emulator threads keep writing while
 * hundreds of GPU pollers read it would bounce between the CPU caches and PCIe. */
#define MH_READY_STRIDE 32
int mh_runner_set_ready(mh_runner *r, uint32_t *ready, uint32_t value);

/* In-place frames: the same macro-step (and reset), but no screen is copied. Per env e,
 * push_count[e] in 1..4 and frame_idx[e*8 + 2j + f] (j < push_count[e], f = 0, 1) = index of the
 * f-th pooled screen of push j (oldest first) in the `screens` bank given to mh_runner_create,
 * i.e. the screen starts at screens + frame_idx * frame_bytes. A consumer that reads the bank in
 * place (mt_preprocess_frames on a pinned, device-mapped bank) must finish before the emulators
 * overwrite those ring slots; the synchronous PAAC step guarantees it for ring >= 16. */
int mh_runner_reset_frames(mh_runner *r, int32_t *frame_idx, int32_t *push_count);
int mh_runner_step_frames(mh_runner *r, const int32_t *a_idx, const int32_t *r_idx, int32_t *frame_idx,
                          int32_t *push_count, float *reward, float *over);

/* Per-env counters (for tests): k (next() calls incl. reset pushes) and steps in episode. */
int mh_runner_env_state(const mh_runner *r, int e, int64_t *k, int32_t *steps);

/* ---- rollout bookkeeping (A8): paac.py:154-205, vectorised over envs -----------------------
 * Per macro-step: masks = 1 - over; rewards = clip(reward, +-1) (actor_learner.py:108-114);
 * per env, in env order: total episode reward += reward (float32, the shared array's type),
 * emulator_steps += tab_rep[r] + 1 (planned repeats, :183), global_step += 1 (:184),
 * histogram[a][r] += 1 and nb_actions += r + 1 (:157, :187-189); on `over` an episode record
 * (global_step at that env, total reward, emulator_steps) is queued and both counters reset. */
typedef struct mh_book mh_book;
int mh_book_create(int n_envs, int num_actions, const int32_t *tab_rep, int n_reps, mh_book **out);
void mh_book_destroy(mh_book *b);
int mh_book_step(mh_book *b, int64_t *global_step, const int32_t *a_idx, const int32_t *r_idx,
                 const float *reward, const float *over, float *rewards_out, float *masks_out);
/* Data-parallel shard (runners.py:17-18 split over ranks): this book's envs are global envs
 * [env_offset, env_offset + n_envs) of a learner stepping envs_total envs per macro-step. Then
 * global_step advances by envs_total per macro-step (paac.py:184 counts every env the learner
 * trains on, identical on every rank) and env e's episode record carries
 * global_step_before + env_offset + e + 1, as a single process owning all envs would log it.
 * Default: env_offset 0, envs_total n_envs. */
int mh_book_set_shard(mh_book *b, int64_t env_offset, int64_t envs_total);
/* Start a new update: clears the action/repetition histogram and nb_actions (paac.py:135-136). */
int mh_book_new_update(mh_book *b);
/* hist [A][R] int64 of the current update, nb_actions (may be NULL). */
int mh_book_histogram(const mh_book *b, int64_t *hist, int64_t *nb_actions);
/* Pop up to max queued episodes (oldest first); *n receives the count popped. */
int mh_book_pop_episodes(mh_book *b, int64_t *global_step, float *reward, int64_t *length, int max,
                         int *n);

/* CRC32C (Castagnoli) of n bytes continuing from crc (0 to start), for the TF tensor-bundle
 * checkpoints of manette_amd/tf_bundle.py (tensorflow/core/util/tensor_bundle: masked CRC32C of
 * every tensor and SSTable block). */
uint32_t mh_crc32c(const void *data, size_t n, uint32_t crc);

#ifdef __cplusplus
}
#endif
#endif /* MANETTE_HOST_H */
