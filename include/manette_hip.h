/*
 * manette_hip.h — C ABI of libmanette_hip.so, the MI355X (gfx950) device side of the
 * PAAC+FiGAR rollout/update hot path.
 *
 * Conventions (every entry point):
 *   - returns int status, MT_OK (0) on success; mt_last_error() gives the message of the
 *     last failure on the calling thread;
 *   - every buffer is a caller-owned DEVICE pointer unless the name says _host; the library
 *     never allocates or synchronises inside a launch function, so each call can be captured
 *     into a hipGraph (mt_graph_*);
 *   - `stream` is a hipStream_t (NULL = the legacy default stream);
 *   - tensors are dense, row-major, NHWC for images, TF variable layouts for parameters
 *     (conv HWIO, dense (in, out)), fp32 arithmetic.
 *
 * Which reference interface each entry point replaces is cited per function
 * (paths relative to the reference repo andres-quintela/manette).
 */
#ifndef MANETTE_HIP_H
#define MANETTE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *mt_stream_t; /* hipStream_t */

enum {
  MT_OK = 0,
  MT_ERR_ARG = 1,         /* bad argument (shape, null pointer, out of range) */
  MT_ERR_HIP = 2,         /* a HIP runtime call failed */
  MT_ERR_UNSUPPORTED = 3, /* configuration not built into this library */
  MT_ERR_WORKSPACE = 4    /* workspace smaller than mt_net_workspace_bytes() */
};

/* --arch values of train.py:100 (networks.py:178-278). */
enum { MT_ARCH_NIPS = 0, MT_ARCH_NATURE = 1, MT_ARCH_PWYX = 2, MT_ARCH_LSTM = 3 };
/* --activation values of train.py:117 (networks.py:27-31). */
enum { MT_ACT_RELU = 0, MT_ACT_LEAKY = 1 };
/* --clip_norm_type values of train.py:96 (actor_learner.py:55-72). */
enum { MT_CLIP_IGNORE = 0, MT_CLIP_GLOBAL = 1 };

/* Number of fp32 partial sums mt_grad_sumsq writes (and mt_clip_rmsprop reads). */
#define MT_NORM_PARTIALS 512

/* Network configuration: the `network_conf` dict of train.py:52-63. */
typedef struct mt_net_config {
  int32_t arch;          /* MT_ARCH_* */
  int32_t depth;         /* 1 = gray, 3 = --rgb; input channels = 4*depth (networks.py:152) */
  int32_t num_actions;   /* A: ALE minimal action set size (environment_creator.py:28) */
  int32_t num_reps;      /* R = --nb_choices (exploration_policy.py:48) */
  int32_t activation;    /* MT_ACT_* */
  float alpha_leaky;     /* --alpha_leaky_relu */
  float softmax_temp;    /* --softmax_temp (networks.py:91-98) */
} mt_net_config;

typedef struct mt_net mt_net;

const char *mt_last_error(void);
int mt_version(void);

/* ---- network description / parameter layout -------------------------------------------
 * Replaces the TF graph construction of networks.py:130-278 + policy_v_network.py:19-57.
 * Parameters live in ONE flat fp32 buffer, variables in TF creation order (trunk, critic,
 * actor, repetition), each (weights, biases) pair contiguous, each pair 64-float aligned.
 * The gradient, RMSProp `ms` and `mom` slot buffers share that layout. */
int mt_net_create(const mt_net_config *cfg, mt_net **out);
void mt_net_destroy(mt_net *net);
int mt_net_num_params(const mt_net *net, size_t *n_floats);
int mt_net_num_vars(const mt_net *net, int *n);
/* TF variable name (e.g. "Network/conv1/conv1_weights"), shape, offset into the flat buffer,
 * and the uniform init bound d (networks.py:34-89: U(-d, d)); d < 0 means N(0,1) init. */
int mt_net_var_info(const mt_net *net, int i, char *name, int name_len, int64_t *shape4,
                    int *ndim, size_t *offset, float *init_bound);
int mt_net_feature_dim(const mt_net *net, int *f); /* width of the trunk output (256/512/...) */
int mt_net_get_config(const mt_net *net, mt_net_config *cfg);
/* Bytes of device workspace a forward/backward on `batch` rows needs. Zero-fill a workspace once
 * when it is allocated: the stacking chains keep per-env hand-off counters in it — the gray NATURE
 * chain (nature_chain_kernel) and the PWYX stacking conv1 launch, gray or RGB (stack_conv1_kernel) —
 * which every launch leaves at zero again, a launch whose bounded waits timed out included. */
int mt_net_workspace_bytes(const mt_net *net, int batch, size_t *bytes);
/* Diagnostics / parity: where a workspace keeps a forward value the backward branches on — kind 0:
 * conv layer `layer`'s stored output, post-activation ([rows][OH][OW][COUT] fp32; a pooled layer's
 * pooled map [rows][OH/2][OW/2][COUT]), whose sign is the ReLU branch; kind 1: a pooled layer's 2x2
 * max-pool argmax bytes ([rows][OH/2][OW/2][COUT] uint8, the window position 0..3 of the first
 * maximum in (row, col) order that the backward routes the gradient to, TF MaxPoolGrad); kind 2:
 * the dense layer's output H ([rows][F] fp32); kind 3: the gradient of conv layer `layer`'s output
 * after a backward ([rows][OH][OW][COUT] fp32, full resolution); kind 4: the stacking chains' hand-off
 * counters (uint32 words, zero between launches; empty for an arch without them). Byte offset and size. layout 0 = the workspace of
 * mt_forward / mt_forward_rows on a = batch rows; layout 1 = the LSTM frame-store workspace of
 * (E = a, T = b), conv rows = fstore rows, H rows = the (T+1)E windows; layout 2 = the LSTM
 * mt_forward workspace of a windows, conv rows = window frames (window-major, 5 per window). */
int mt_net_workspace_region(const mt_net *net, int layout, int a, int b, int kind, int layer, size_t *offset,
                            size_t *bytes);

/* ---- forward (A5-A7) ----------------------------------------------------------------------
 * Replaces session.run([output_layer_v, output_layer_pi, output_layer_rep], {input_ph: s})
 * (paac.py:144-146, :219-224) and the forward half of train_step (paac.py:254-256).
 * obs: [batch][84][84][4*depth] uint8 (for LSTM: [batch][5][84][84][4*depth]).
 * Outputs v [batch], pi [batch][A], rep [batch][R] (softmax probabilities).
 * Activations are kept in `ws` for a following mt_loss_backward on the same rows. */
int mt_forward(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
               size_t ws_bytes, float *v, float *pi, float *rep, mt_stream_t stream);

/* ---- inference forward (rollout steps, bootstrap V(s_T)) -----------------------------------
 * Same outputs as mt_forward (paac.py:144-146, :219-224) but keeps no activations for a backward
 * pass, so the NIPS arch runs its rollout trunk (manette_amd/csrc/trunk_fused.h: one conv kernel,
 * conv1 -> conv2 per (env, conv2 row) block, then the dense layer as its own MFMA GEMM kernel
 * writing 9 split-K slabs) followed by the heads kernel; other arches take mt_forward's layered
 * path. Same workspace size as mt_forward. (A one-launch variant whose last block per env
 * finished the heads measured 25 us vs 12.7 + 6.1 us: the release/acquire fences and the serial
 * tail cost more than the second launch.) */
int mt_forward_infer(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                     size_t ws_bytes, float *v, float *pi, float *rep, mt_stream_t stream);

/* Inference forward of `batch` rows that ALSO leaves their activations (and dense outputs H) in
 * rows [row0, row0 + batch) of a train workspace sized for train_rows rows
 * (mt_net_workspace_bytes(net, train_rows)). A rollout that forwards state slot t with
 * row0 = t*E fills the whole batch the update trains on (paac.py:236: row t*E + e), with the
 * parameters unchanged in between, so mt_loss_backward(train_rows) then needs no mt_forward: pass
 * it the rollout's v / pi / rep of every row. `ws` (batch rows) holds the split-K partials.
 * Not for the LSTM arch (its frame store does the same, mt_lstm_*). */
int mt_forward_rows(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                    size_t ws_bytes, void *train_ws, size_t train_ws_bytes, int train_rows, int row0, float *v,
                    float *pi, float *rep, mt_stream_t stream);

/* Trunk half of mt_forward_infer alone (roofline timing / diagnostics): the convs and the dense
 * layer's partial products, left in `ws` (NIPS: the conv kernel + the dense kernel). */
int mt_forward_trunk(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                     size_t ws_bytes, mt_stream_t stream);

/* The rollout chain's stacking trunk alone (roofline timing, parity tests): the conv kernel in its
 * in-kernel-pull form — per env, wait until ready[e * MH_READY_STRIDE] >> 3 == tag (one 128-B line
 * per env, manette_host.h), stack out = prev shifted by the push count (its low 3 bits) + that
 * many final frames (frames = [4*batch][84][84][depth], env e's pushes at slots 4e..; host-mapped
 * pinned staging or device memory) — then the dense layer's split-K partials, left in ws. NIPS:
 * nips_conv_kernel<STACK> + nips_fc_kernel; gray NATURE: nature_chain_kernel (stacking conv1 ->
 * conv2 -> conv3, per-env hand-offs in one launch) + the split-K dense GEMM; PWYX (gray or RGB):
 * stack_conv1_kernel (per-env pull + stack blocks, then conv1 tiles per env) + conv2 .. + the dense
 * GEMM. With every ready word already set nothing waits: the kernels' own duration.
 * Every device wait is bounded (~2 s): a wait that times out stores 1 into *status (a device-visible
 * word, e.g. mapped pinned memory; may be NULL) and the launch drains (an env never published keeps
 * its previous state); the caller reads *status after the stream has completed.
 * MT_ERR_UNSUPPORTED for the other archs (the LSTM steps stack in mt_rollout_step). */
int mt_forward_trunk_stacking(const mt_net *net, const float *params, const uint8_t *prev, const uint8_t *frames,
                              const uint32_t *ready, uint32_t tag, uint8_t *out, int batch, void *ws, size_t ws_bytes,
                              uint32_t *status, mt_stream_t stream);

/* ---- LSTM frame-store mode (the learner's LSTM path; manette_amd/csrc/lstm.h) -------------
 * The reference feeds each step's memory window [E][5][84][84][C] (paac.py:79-83) and the train
 * step the T*E windows of whole_memory (paac.py:233-234); consecutive windows share 4 frames.
 * Here the caller keeps ONE frame store fstore [1 + (T+5)*E][84][84][C] uint8: row 0 = zeros,
 * row 1 + slot*E + e = env e's state in slot `slot` (slots 0..3 = the previous rollout's last 4
 * states, slot 4 + t = the state before step t), and per window only nz = its number of leading
 * zero frames (reference memory[e] = 0 at an episode end, then shifted). Window (t, e) reads
 * zero frames at positions k < nz[t][e] and slot t + k otherwise.
 *  - mt_lstm_frames_forward: trunk + the cell's x-product of frame rows [row0, row0+nrows),
 *    kept in ws (step 0: rows [0, 1+5E) — zero frame + slots 0..4; step t: slot 4+t's E rows);
 *  - mt_lstm_windows_forward: the E windows of step t (t == T: the bootstrap windows) ->
 *    v [E], pi [E][A], rep [E][R] (paac.py:144-152, :219-224), nz_t = nz[t][0..E);
 *  - mt_lstm_step_forward: one macro-step of the rollout = frames_forward of step t's new rows
 *    + windows_forward of step t, with nz[t] derived on the device for t > 0 (nz [T+1][E]:
 *    nz[t][e] = over[e] != 0 ? 5 : max(nz[t-1][e] - 1, 0), `over` = step t-1's episode-end
 *    flags, device-readable — paac.py:173-174 update_memory, :202-203 the reset); the native
 *    rollout (mt_rollout_*) runs the same forward with the draw fused into its heads kernel.
 *    Steps run in order within a rollout (t > 0 after steps 0 .. t-1 on the same ws and
 *    parameters): step 0 stores each frame's x-product sum in ws, steps t > 0 read the 4 older
 *    frames' sums from there (mt_lstm_windows_forward always sums every frame from its slabs);
 *  - mt_lstm_frames_backward: loss + gradient of the T*E windows of steps 0..T-1 (the train
 *    step of paac.py:254-256) from the rollout's activations (unchanged parameters), with pi,
 *    rep, v [T*E] the rollout outputs; back-propagates through each distinct frame once.
 *    norm_partials (optional, [MT_NORM_PARTIALS]): as mt_returns_loss_backward's — the global-norm
 *    partials of the whole gradient from the backward's last launch (no mt_grad_sumsq needed). */
int mt_lstm_frames_workspace_bytes(const mt_net *net, int E, int T, size_t *bytes);
int mt_lstm_frames_forward(const mt_net *net, const float *params, const uint8_t *fstore, int row0, int nrows,
                           int E, int T, void *ws, size_t ws_bytes, mt_stream_t stream);
int mt_lstm_windows_forward(const mt_net *net, const float *params, const int32_t *nz_t, int t, int E, int T,
                            void *ws, size_t ws_bytes, float *v, float *pi, float *rep, mt_stream_t stream);
int mt_lstm_step_forward(const mt_net *net, const float *params, const uint8_t *fstore, int t, int E, int T,
                         int32_t *nz, const float *over, void *ws, size_t ws_bytes, float *v, float *pi,
                         float *rep, mt_stream_t stream);
int mt_lstm_frames_backward(const mt_net *net, const float *params, const uint8_t *fstore, const int32_t *nz,
                            int E, int T, void *ws, size_t ws_bytes, const float *pi, const float *rep,
                            const float *v, const int32_t *a_idx, const int32_t *r_idx, const float *y,
                            const float *adv, float entropy_beta, float *grad, float *loss_terms,
                            float *norm_partials, mt_stream_t stream);

/* ---- device multinomial sampling (perf mode of A3) -----------------------------------------
 * Replaces ExplorationPolicy.multinomial_choose (exploration_policy.py:108-116) with an
 * inverse-CDF draw on (p - float32 epsneg), the last category taking the remainder — the
 * distribution numpy's multinomial(1, p - epsneg) draws from. Uniforms come from a
 * counter-based hash of (seed, row0 + row, counters[row]); row0 = the global env id of row 0
 * (a data-parallel rank's env offset, runners.py:17-18 shard), so every env draws the same
 * stream whichever rank owns it. counters (device, one uint64 per row) are incremented by the
 * call, so a captured graph draws fresh numbers on every replay.
 * Writes int32 indices a_idx [batch], r_idx [batch], and (if pair != NULL) both again into
 * pair [2][batch] so one copy moves them to the host. */
int mt_sample(const float *pi, const float *rep, int batch, int num_actions, int num_reps,
              uint64_t seed, int row0, uint64_t *counters, int32_t *a_idx, int32_t *r_idx, int32_t *pair,
              mt_stream_t stream);

/* ---- n-step return / advantage scan (A9) ---------------------------------------------------
 * Replaces paac.py:219-231 (+ flatten :237-238). rewards/masks/values: [T][E] fp32,
 * v_boot: [E] (V(s_T)). Writes y, adv: [T][E] fp32 (row t*E+e). Arithmetic follows the
 * reference's numpy dtypes exactly (gamma is the python float: the first product gamma*V_T in
 * fp32, the rest fp64, fp32 output). */
/* rewards / masks may be device addresses of pinned host memory (the learner's [2][T][E]
 * bookkeeping output, read in place). */
int mt_returns(const float *rewards, const float *masks, const float *values, const float *v_boot,
               double gamma, int T, int E, float *y, float *adv, mt_stream_t stream);

/* ---- fused loss + backward (A10) ------------------------------------------------------------
 * Replaces optimizer.compute_gradients(network.loss) (actor_learner.py:49) with the loss of
 * policy_v_network.py:25-74. Requires the activations of mt_forward(obs, batch) in `ws`
 * (pi, rep, v as that call returned them). a_idx/r_idx: selected action / repetition index
 * (argmax of the one-hot feeds, paac.py:239-240). Overwrites every variable's gradient in the
 * flat `grad` and never touches its alignment padding, which the caller zeroes once when it
 * allocates grad (the clip's global norm sums the whole buffer). Also writes per-row loss terms
 * loss_terms [batch][4] = (critic 0.25(y-v)^2, -adv*(logpi_a+logrep_r), entropy_pi, entropy_rep). */
int mt_loss_backward(const mt_net *net, const float *params, const uint8_t *obs, int batch,
                     void *ws, size_t ws_bytes, const float *pi, const float *rep, const float *v,
                     const int32_t *a_idx, const int32_t *r_idx, const float *y, const float *adv,
                     float entropy_beta, float *grad, float *loss_terms, mt_stream_t stream);

/* mt_returns + mt_loss_backward in one call (the update of a rollout, batch = T*E rows t*E+e):
 * the loss kernel block of row (t, e) runs the n-step scan of env e from T-1 down to t itself
 * (the same arithmetic as mt_returns, bit for bit) — one launch fewer on the update's critical
 * path. y and adv ([T][E]) are still written. values: [T][E] = the v the rollout returned.
 * norm_partials (may be NULL): also write the MT_NORM_PARTIALS global-norm partials of the
 * gradient, as mt_grad_sumsq(grad, n, 1.0f) would for mt_clip_rmsprop (no data-parallel
 * all-reduce in between); the sum of squares is taken in the backward's last launch. */
int mt_returns_loss_backward(const mt_net *net, const float *params, const uint8_t *obs, int T, int E, void *ws,
                             size_t ws_bytes, const float *pi, const float *rep, const float *values,
                             const int32_t *a_idx, const int32_t *r_idx, const float *rewards,
                             const float *masks, const float *v_boot, double gamma, float *y, float *adv,
                             float entropy_beta, float *grad, float *loss_terms, float *norm_partials,
                             mt_stream_t stream);
/* mt_returns_loss_backward with the bootstrap finished here: boot_ws is the rollout's E-row
 * inference workspace whose dense-layer slabs the last chain left (MT_ROLLOUT_BOOT_SLABS); each
 * loss block sums env e's slabs in slab order, adds the bias, applies the activation and takes the
 * critic's dot product (the heads kernel's arithmetic) for V(s_T)[e] = v_boot[e] (written out),
 * then scans. Same outputs as mt_returns_loss_backward given that v_boot. */
int mt_returns_loss_backward_boot(const mt_net *net, const float *params, const uint8_t *obs, int T, int E, void *ws,
                                  size_t ws_bytes, const float *pi, const float *rep, const float *values,
                                  const int32_t *a_idx, const int32_t *r_idx, const float *rewards,
                                  const float *masks, const void *boot_ws, size_t boot_ws_bytes, float *v_boot,
                                  double gamma, float *y, float *adv, float entropy_beta, float *grad,
                                  float *loss_terms, float *norm_partials, mt_stream_t stream);

/* ---- global-norm clip + TF1 ApplyRMSProp (A11) ----------------------------------------------
 * Replaces clip_by_global_norm (actor_learner.py:59-63) + ApplyRMSProp (actor_learner.py:47-48,74).
 * mt_grad_sumsq writes MT_NORM_PARTIALS fp32 partial sums of (inv_scale*g)^2.
 * mt_clip_rmsprop: g' = inv_scale*g; norm = sqrt(sum partials);
 *   clip_type GLOBAL: g' *= clip * min(1/norm, 1/clip);
 *   ms += (g'^2 - ms)*(1 - decay); mom = momentum*mom + g'*lr/sqrt(ms + eps); w -= mom.
 * lr is read by the kernel from *lr_dev (device memory, or — as the learner does — the device
 * address of pinned host memory the host writes the schedule into, actor_learner.py:132-136), so
 * no copy is needed and a captured graph picks up the schedule. norm_out (device, may be NULL)
 * receives the pre-clip norm.
 * inv_scale folds the 1/world of a data-parallel all-reduce (sum) into the update. */
int mt_grad_sumsq(const float *g, size_t n, float inv_scale, float *partials, mt_stream_t stream);
int mt_clip_rmsprop(float *w, float *ms, float *mom, const float *g, size_t n,
                    const float *partials, const float *lr_dev, float decay, float momentum,
                    float eps, float clip, int clip_type, float inv_scale, float *norm_out,
                    mt_stream_t stream);

/* ---- frame preprocess + 4-frame stack (A2) --------------------------------------------------
 * Replaces AtariEmulator.__process_frame_pool / ObservationPool (atari_emulator.py:79-88,
 * environment.py:58-80): per env, each "push" is the pair of the last two ALE screens of one
 * emulator.next() (atari_emulator.py:90-100): pooled = max(f0, f1) (np.amax), resized to 84x84
 * with the nearest LUT (row_lut[84], col_lut[84] = source row/col), appended to the 4-deep
 * observation stack. Per env e: push_offset[e], push_count[e] (1..4) index the pushes (oldest
 * first) in `raw` = [total_pushes][2][src_rows][160][depth] uint8: whole screens (src_rows 210,
 * row_lut = the resize LUT) or the 84 rows the resize reads, staged by the runner (src_rows 84,
 * row_lut = identity). prev/out: [E][84][84][4*depth];
 * out[c] = prev[c+p] for c < 4-p, else the (c-(4-p))-th new push; RGB interleaves channels as
 * [R_t0..R_t3, G_t0..G_t3, B_t0..B_t3] (environment.py:75). out may not alias prev. */
int mt_preprocess(const uint8_t *raw, const int32_t *push_offset, const int32_t *push_count,
                  int E, int depth, int src_rows, const int32_t *row_lut, const int32_t *col_lut,
                  const uint8_t *prev, uint8_t *out, mt_stream_t stream);

/* Pooled variant: each staging slot holds ONE screen per push, max(f0, f1) already taken on the
 * host by the emulator's frame pool (mh_runner MH_RUNNER_POOLED): raw = [slots][src_rows][160][depth]. */
int mt_preprocess_pooled(const uint8_t *raw, const int32_t *push_offset, const int32_t *push_count,
                         int E, int depth, int src_rows, const int32_t *row_lut, const int32_t *col_lut,
                         const uint8_t *prev, uint8_t *out, mt_stream_t stream);

/* Resized variant (MT_ROLLOUT_RESIZED): staging slot push_offset[e] + j holds push j's FINAL
 * 84x84xdepth frame, pooled and resized by the host threads (mh_runner MH_RUNNER_RESIZED):
 * frames = [slots][84][84][depth]; the kernel only stacks it onto prev. */
int mt_preprocess_resized(const uint8_t *frames, const int32_t *push_offset, const int32_t *push_count, int E,
                          int depth, const uint8_t *prev, uint8_t *out, mt_stream_t stream);

/* In-place variant (MT_ROLLOUT_IN_PLACE): the pushes' screens are read where the emulators left
 * them. screens = a bank of whole 210-row screens [..][210][160][depth] (pinned + device-mapped
 * host memory, or device memory); push j's frame f of env e is screen frame_idx[e*8 + 2j + f]
 * (j < push_count[e]), as mh_runner_step_frames writes them (include/manette_host.h). Only the
 * 84 rows row_lut names are read. */
int mt_preprocess_frames(const uint8_t *screens, const int32_t *frame_idx, const int32_t *push_count,
                         int E, int depth, const int32_t *row_lut, const int32_t *col_lut,
                         const uint8_t *prev, uint8_t *out, mt_stream_t stream);

/* Device address of pinned (page-locked, mapped) host memory, e.g. an emulator screen bank. */
int mt_host_device_pointer(void *host, void **dev);

/* ---- LSTM memory window (paac.py:79-83 update_memory + :202-203 episode-end reset) --------
 * memory [E][5][frame] (the window each env's forward reads), whole_t [E][5][frame] = row t of
 * whole_memory, fresh [E][frame] = the new states, masks [E] = 1 - episode_over (float32).
 * whole_t <- memory; memory <- shift left + fresh; memory[e] <- 0 where masks[e] == 0.
 * frame = 84*84*4*depth bytes. */
int mt_memory_push(uint8_t *memory, uint8_t *whole_t, const uint8_t *fresh, const float *masks, int E,
                   size_t frame_bytes, mt_stream_t stream);

/* ---- native rollout macro-step (orchestrates A1-A3, A8; paac.py:140-205) -------------------
 * One call = one macro-step t of every env: mt_forward on state slot t with the A3 draw fused
 * into its heads kernel (indices into idx[0][t], idx[1][t] and the [2][E] pair) -> wait for the
 * pair (spin on the stream's event) -> mh_runner_step (native emulator threads,
 * libmanette_host.so) -> mh_book_step (bookkeeping into rm_host[.][t]) -> mt_preprocess of the
 * pushed screens into state slot t+1.
 * flags = 0: the pair is copied D2H and the screens + push metadata H2D (hipMemcpyAsync).
 * flags & MT_ROLLOUT_IN_PLACE (implies ZERO_COPY): no screen is staged at all — the emulators run
 * mh_runner_step_frames and mt_preprocess_frames reads their screens in place: staging_host is
 * then the emulators' screen bank (pinned, device-mapped), frames_host [E][8] the frame indices
 * and meta_host[E..2E) the push counts.
 * flags & MT_ROLLOUT_ZERO_COPY: the heads kernel writes the pair into pair_host and the
 * preprocess kernel reads staging_host / meta_host in place (host-mapped pinned memory): no
 * copy engine and no cross-engine wait on the per-step critical path; raw / meta / pair may then
 * be null. All buffers are caller-owned; `runner` / `book` are mh_runner* / mh_book* handles. */
#define MT_ROLLOUT_ZERO_COPY 1
#define MT_ROLLOUT_IN_PLACE 2
/* flags & MT_ROLLOUT_POOLED: the runner stages ONE pooled screen per push (MH_RUNNER_POOLED) and the
 * preprocess is mt_preprocess_pooled. */
#define MT_ROLLOUT_POOLED 4
/* flags & MT_ROLLOUT_PIPELINED (needs ZERO_COPY or IN_PLACE): each call enqueues step t+1's chain
 * (a bounded device wait on sync_host[0], preprocess, forward + draw) before it waits for step t's
 * indices, and after the emulators only stores the step word — no launch on the critical path.
 * sync_host = [2] uint32 pinned + mapped: [0] host step word, [1] device wait timeout status.
 * PIPELINED + RESIZED + the NIPS arch ("stacking" rollout): the chain of step t+1 is the conv
 * kernel — each (env, row) block waits for the word the emulator thread stores once its env is
 * staged (mh_runner_set_ready), reads that env's frames from the pinned staging and stacks state
 * slot t+1 from slot t itself (no pull or preprocess launch) — the dense kernel and the heads
 * kernel, which writes each env's (a, r) as one tagged 8-byte word into host memory (no fence).
 * Every chain of a rollout is armed at its step 0 (from the second rollout on as one replayed
 * hipGraph whose sequence tags live in device memory), and step 0's forward takes slot 0 from
 * slot T of the previous rollout (the update then needs no copy). Other pipelined modes: a pull
 * kernel per env copies the frames into HBM, then the preprocess kernel, then the forward. */
#define MT_ROLLOUT_PIPELINED 8
/* flags & MT_ROLLOUT_RESIZED: the runner stages each push's final 84x84 frame (MH_RUNNER_RESIZED,
 * staging [4E][84*84*depth]) and the preprocess is mt_preprocess_resized (row/col LUTs unused). */
#define MT_ROLLOUT_RESIZED 16
/* flags & MT_ROLLOUT_BOOT_SLABS (pipelined, v_boot set, not LSTM): the last chain's bootstrap
 * forward stops after the dense layer — its split-K slabs stay in ws — and the update's loss kernel
 * finishes V(s_T) itself (mt_returns_loss_backward_boot, which writes v_boot): one heads kernel and
 * one kernel boundary fewer between the last emulator step and the backward. */
#define MT_ROLLOUT_BOOT_SLABS 32
typedef struct mt_rollout mt_rollout;
typedef struct mt_rollout_buffers {
  /* device */
  uint8_t *states;             /* [T+1][E][84][84][4*depth] */
  float *values;               /* [T][E] */
  int32_t *idx;                /* [2][T][E]: action indices, then repetition indices */
  float *pi, *rep;             /* [E][A], [E][R] */
  void *ws;                    /* forward workspace for E rows */
  size_t ws_bytes;
  uint64_t *counters;          /* [E] sampling counters */
  uint8_t *raw;                /* [4E][2][src_rows*160*depth] screen staging */
  int32_t src_rows;            /* staged screen rows: 210, or 84 when the runner selects rows */
  int32_t *pair;               /* [2][E] device scratch: this step's indices for one D2H copy */
  int32_t *pair_host;          /* [2][E] pinned */
  int32_t *meta;               /* [2][E] push offsets; push counts */
  const int32_t *row_lut, *col_lut;
  /* pinned host */
  int32_t *idx_host;           /* [2][T][E] */
  uint8_t *staging_host;       /* [4E][2][src_rows*160*depth] */
  int32_t *meta_host;          /* [2][E] */
  float *reward_host, *over_host; /* [E] */
  float *rm_host;              /* [2][T][E]: clipped rewards; masks */
  int32_t *frames_host;        /* [E][8] in-place frame indices (MT_ROLLOUT_IN_PLACE), else NULL */
  uint32_t *sync_host;         /* [2] pipelined step word + wait status (MT_ROLLOUT_PIPELINED), else NULL */
  void *train_ws;              /* optional: train workspace of T*E rows; the forward of step t then also
                                  writes rows [t*E, (t+1)*E) (mt_forward_rows) and pi / rep are
                                  [T][E][.] per-step outputs; NULL: pi / rep are [E][.] */
  size_t train_ws_bytes;
  float *v_boot;               /* optional [E] (MT_ROLLOUT_PIPELINED): the last step's chain also runs the
                                  bootstrap forward of slot T (paac.py:219-224) into it, in the shadow
                                  of the host's last emulator step */
  uint32_t *ready_host;        /* [E] zero-copy modes: the heads kernel stores a step sequence number per
                                  env after writing its pair; the host polls these instead of an event
                                  (NULL: hipEventQuery) */
  int32_t flags;               /* MT_ROLLOUT_* */
  int32_t env_offset;          /* global env id of env 0 (data-parallel shard offset): the draw's row0 */
  int32_t *nz;                 /* LSTM arch only (else NULL): [T+1][E] device window zero counts; nz[0]
                                  is the caller's, step t > 0 derives nz[t] (mt_lstm_step_forward).
                                  With the LSTM arch `states` is slot 4 of a frame store
                                  [1 + (T+5)E][84][84][C] (mt_lstm_*), ws is its workspace
                                  (mt_lstm_frames_workspace_bytes), train_ws is NULL and pi / rep are
                                  [T+1][E][.] per-step outputs (row T: the bootstrap's) */
} mt_rollout_buffers;
int mt_rollout_create(const mt_net *net, int E, int T, void *runner, void *book,
                      const mt_rollout_buffers *buffers, uint64_t seed, mt_rollout **out);
void mt_rollout_destroy(mt_rollout *ro);
int mt_rollout_step(mt_rollout *ro, const float *params, int t, int64_t *global_step,
                    mt_stream_t stream);
/* The whole rollout: mt_rollout_step for t = 0 .. T-1 in one call (paac.py:140-205 without a
 * return to the caller between macro-steps). */
int mt_rollout_run(mt_rollout *ro, const float *params, int64_t *global_step, mt_stream_t stream);
/* Host wall-clock microseconds accumulated by mt_rollout_step, per phase: [0] launch + wait
 * for the sampled indices, [1] emulator step, [2] bookkeeping, [3] upload + preprocess
 * enqueue, [4] number of steps. reset != 0 zeroes the counters. */
int mt_rollout_stats(mt_rollout *ro, double *out5, int reset);
/* mt_rollout_stats plus the split of [0]: out[5] = host enqueue (the step's forward and the armed
 * chains' launches), out[6] = wait for the sampled indices; n = how many of the 7 values to copy. */
int mt_rollout_stats_ex(mt_rollout *ro, double *out, int n, int reset);
/* Host timeline of the last min(max_steps, 256) macro-steps, oldest first, 6 doubles each:
 * t, then host wall microseconds at the call's start, after its launches, when the sampled
 * indices were seen, after the emulator step, after the bookkeeping (diagnostics). */
int mt_rollout_host_trace(mt_rollout *ro, double *out, int max_steps, int *n);
/* Live timing of the trunk kernels the rollout runs (roofline measurement, bench.py): enable != 0
 * records an event pair around each step forward's trunk launches (NIPS: the stacking conv kernel
 * + the dense kernel); a call with enable == 0 waits for them and returns their summed duration
 * in microseconds and their count, then stops. Any call returns (and forgets) what was recorded. */
int mt_rollout_trunk_timing(mt_rollout *ro, int enable, double *sum_us, int64_t *count);

/* Update launched by the rollout itself (native pipelined step, replayed update graph): once
 * registered, the last macro-step of every rollout (after its bookkeeping) stores
 * lr = get_lr(global_step) — actor_learner.py:145-148: initial_lr - global_step * initial_lr /
 * annealing_steps while global_step <= annealing_steps, else 0, in double, then rounded to float —
 * into *lr_host (the pinned LR word the RMSProp kernel reads) and launches graph_exec (the update:
 * loss backward [, all-reduce], clip + RMSProp) on the rollout's stream, right behind the bootstrap
 * chain: the update then starts with no host round trip after the last emulator step (the caller
 * must not launch it again). graph_exec NULL unregisters every registered update, this form's and a
 * data-parallel one (mt_rollout_set_update_dp), before the graphs are destroyed. */
int mt_rollout_set_update(mt_rollout *ro, void *graph_exec, float *lr_host, double initial_lr,
                          double annealing_steps);
/* Diagnostics: the update the rollout launches — *form = 0 none, 1 mt_rollout_set_update's graph,
 * 2 mt_rollout_set_update_dp's three graphs. */
int mt_rollout_update_form(const mt_rollout *ro, int *form);

/* ---- data-parallel communicator (RCCL over xGMI; manette_amd/csrc/comm.hip) ----------------
 * The reference has no collective: its only shard unit is the contiguous env split of
 * runners.py:17-18 (np.split over workers). This build splits envs over ranks the same way (rank r
 * owns global envs [r*ec, (r+1)*ec)) and exchanges exactly one thing per update: the flat fp32
 * gradient, summed in place (mt_allreduce) between mt_returns_loss_backward and mt_clip_rmsprop
 * (inv_scale = 1/world), i.e. the union batch's mean gradient of actor_learner.py:49 before the
 * global-norm clip of :59-63. mt_broadcast copies rank 0's parameters / RMSProp slots at start
 * (and on resume). Both are stream-ordered and capturable into a hipGraph.
 * Bootstrap: rank 0 calls mt_comm_unique_id, ships the MT_COMM_UID_BYTES bytes to every rank over
 * any control channel (the learner uses torch.distributed's gloo store), then every rank calls
 * mt_comm_init(uid, rank, world, device) collectively. */
#define MT_COMM_UID_BYTES 128
typedef struct mt_comm mt_comm;
int mt_comm_unique_id(char *uid /* [MT_COMM_UID_BYTES] */);
int mt_comm_init(const char *uid, int rank, int world, int device, mt_comm **out);
void mt_comm_destroy(mt_comm *comm);
int mt_comm_info(const mt_comm *comm, int *rank, int *world);
/* In-place sum over ranks of n fp32 values (ncclAllReduce, ncclSum). */
int mt_allreduce(mt_comm *comm, float *buf, size_t n, mt_stream_t stream);
/* In-place broadcast of `bytes` bytes from rank `root`. */
int mt_broadcast(mt_comm *comm, void *buf, size_t bytes, int root, mt_stream_t stream);
/* Diagnostics / tests: a communicator without RCCL standing for `replicas` identical ranks. Its
 * mt_allreduce multiplies the buffer by `replicas` at once (the in-place sum of identical replicas)
 * and then holds the stream for delay_us microseconds; mt_broadcast is a no-op. A sum that started
 * before its producer finished, or a consumer that did not wait for it, changes the result (the
 * stream-order tests of the data-parallel update, tests/test_dp_gpu.py). */
int mt_comm_init_loopback(int replicas, int delay_us, mt_comm **out);

/* The data-parallel update launched by the rollout itself (the counterpart of mt_rollout_set_update
 * for world > 1, or forced at world 1): once registered, the last macro-step of every rollout stores
 * the LR as mt_rollout_set_update does and enqueues, with no return to the caller,
 *   graph_execs[0] (loss + dense / head gradients: the backward's first
 *   mt_net_backward_bucket_launches launches) on the rollout's stream;
 *   the in-place sum of grad[split, n) (mt_allreduce) on a side stream the rollout owns, behind it;
 *   graph_execs[1] (the rest of the conv backward) on the rollout's stream;
 *   the sum of grad[0, split) on the side stream, behind that;
 *   graph_execs[2] (norm partials + clip + RMSProp with inv_scale = 1/world) behind both sums.
 * The all-reduces run beside the conv backward, as PAACLearner._bucketed_update issues them from
 * Python (which the learner keeps for communicators outside the C ABI). graph_execs NULL
 * unregisters; registering either form replaces the other. */
int mt_rollout_set_update_dp(mt_rollout *ro, void *const *graph_execs, mt_comm *comm, float *grad, size_t n,
                             size_t split, float *lr_host, double initial_lr, double annealing_steps);

/* ---- small helpers ----------------------------------------------------------------------- */
/* out[i] = sum_z parts[z*n + i] (deterministic order); used for split reductions. */
int mt_sum_slabs(const float *parts, int nslabs, size_t n, float *out, mt_stream_t stream);

/* Launch window: after mt_launch_window(first, count), first >= 0, the library numbers its grouped
 * launches, loss-kernel launches and every launch of mt_lstm_frames_backward from 0 in issue order and issues only those with index in
 * [first, first + count) (count < 0: no upper end); the others return MT_OK without launching.
 * mt_launch_window(-1, -1), the default, turns it off. Used while CAPTURING: one
 * mt_returns_loss_backward* call recorded as two graphs, [0, 2) = the loss + the dense / head
 * gradient launch and [2, ...) = the conv backward, so a data-parallel learner all-reduces the
 * dense / head bucket while the conv backward runs (paac.py); and by bench.py to time a backward
 * launch by launch. Library-global: set it around calls of one thread only. Returns how many
 * launches were numbered since the previous call. */
int mt_launch_window(int first, int count);
/* How many leading launches of mt_returns_loss_backward* (non-LSTM) complete the gradient of every
 * variable from the dense layer on (the tail of the flat gradient, ~98 % of its bytes): a
 * data-parallel learner captures launches [0, n) and [n, ...) as two graphs and all-reduces the
 * tail between them while the rest of the conv backward runs. */
int mt_net_backward_bucket_launches(const mt_net *net, int *launches);

/* hipGraph capture of everything launched on `stream` between begin and end. */
int mt_graph_begin(mt_stream_t stream);
int mt_graph_end(mt_stream_t stream, void **graph_exec);
int mt_graph_launch(void *graph_exec, mt_stream_t stream);
int mt_graph_destroy(void *graph_exec);

#ifdef __cplusplus
}
#endif
#endif /* MANETTE_HIP_H */
