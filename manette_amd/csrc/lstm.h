// LSTM arch (networks.py:227-258, Operations.rnn :112-127) on gfx950. Included by net.hip only
// (uses its workspace/trunk helpers).
//
// The memory window [B][5][84][84][C] is 5B frames, window-major (row b*5+t), that go through the
// PWYX trunk (SAME convs + 2x2 pools, trunk_forward / trunk_backward of net.hip) to 6400
// features each. BasicLSTMCell(32, forget_bias=1) over the 5 frames:
//   z_t = [x_t, h_{t-1}] K + bias  (K = [6400 + 32][128], gates i, j, f, o),
//   c_t = c_{t-1} sigmoid(f + 1) + sigmoid(i) tanh(j),  h_t = tanh(c_t) sigmoid(o),
// then out = h_5 w + b (linear, N(0,1)-initialised), then fc6 (32 -> 128) + act, then the heads.
//
// Kernels:
//  * x_t K_x for all 5B frames is one split-K GEMM (M = 5B, N = 128, K = 6400) on the MFMA core;
//  * the recurrence, the projection and fc6's product run in lstm_fwd_kernel, one workgroup per
//    window (2 waves, thread g owns gate column g and keeps K_h[:, g] in registers);
//  * lstm_bwd_kernel runs BPTT per window and writes dz (pre-activation gate gradients, rows
//    b*5+t) — the operand of the K weight gradient (MFMA GEMMs) and of dX = dz K_x^T, which
//    is masked by conv4's activation and continues into the trunk backward.
#pragma once

namespace mt {

template <int C>
struct LstmArch : PwyxArch<C> {
  static constexpr bool LSTM = true;
  static constexpr int NH = 32;     // n_hidden
  static constexpr int STEPS = 5;   // n_steps (paac.py:108)
  static constexpr int G4 = 4 * NH; // gate columns
  static constexpr int F = 128;     // fc6 n_outputs
  static constexpr const char *FC = "fc6";
  static constexpr int FUSED_SLABS = 0;
  static constexpr int FC_ROWS = 0;
};

struct LstmWs {
  size_t xg, slab6, gates, cst, hprev, h5, out32, dout32, dgates;
  int xg_splits;
};

template <class Ar>
static int lstm_xg_splits(int B) {
  const int M = B * Ar::STEPS;
  const int s = pick_splits(cdiv(M, TileFc::BM) * cdiv(Ar::G4, TileFc::BN), Ar::FLAT, TileFc::BK, 128);
  return gemm_splits<TileFc>(Ar::FLAT, s);
}

// Workspace: trunk layers for the 5B frames, then the LSTM buffers (floats).
template <class Ar>
static WsLayout lstm_ws_layout(const mt_net *n, int B, LstmWs *X) {
  WsLayout L{};
  LstmWs W{};
  size_t off = 0;
  auto take = [&](size_t nf) {
    size_t o = off;
    off = align64(off + nf);
    return o;
  };
  const int rows = B * Ar::STEPS;
  size_t wslab = 0;
  ws_layers<Ar>(L, off, rows, wslab);
  W.xg_splits = lstm_xg_splits<Ar>(B);
  W.xg = take((size_t)W.xg_splits * rows * Ar::G4);
  W.slab6 = take((size_t)B * Ar::F);
  W.gates = take((size_t)rows * Ar::G4);
  W.cst = take((size_t)rows * Ar::NH);
  W.hprev = take((size_t)rows * Ar::NH);
  W.h5 = take((size_t)B * Ar::NH);
  W.out32 = take((size_t)B * Ar::NH);
  W.dout32 = take((size_t)B * Ar::NH);
  W.dgates = take((size_t)rows * Ar::G4);
  L.fc_splits = 1;
  L.fcslab = W.slab6;
  L.H = take((size_t)B * Ar::F);
  L.dz = take((size_t)B * n->O);
  L.dH = take((size_t)B * Ar::F);
  L.wslab = take(wslab);
  L.wslab2 = take(wslab);
  L.total = off;
  if (X) *X = W;
  return L;
}

template <class Ar>
static void build_layout_lstm(mt_net *n) {
  size_t off = 0;
  add_convs<Ar>(n, off);
  const int kin = Ar::FLAT + Ar::NH;
  // rnn/basic_lstm_cell/{kernel, bias}: glorot-uniform kernel, zero bias (TF 1.3 get_variable
  // defaults); Network/lstm/Variable{,_1}: N(0, 1) (networks.py:124-125; bound < 0 = normal).
  add_named_pair(n, off, "rnn/basic_lstm_cell/kernel", "rnn/basic_lstm_cell/bias", {kin, Ar::G4}, Ar::G4,
                 (float)std::sqrt(6.0 / (double)(kin + Ar::G4)), 0.f, &n->off_lstm);
  add_named_pair(n, off, "Network/lstm/Variable", "Network/lstm/Variable_1", {Ar::NH, Ar::NH}, Ar::NH, -1.f,
                 -1.f, &n->off_proj);
  const float bf = (float)(1.0 / std::sqrt((double)Ar::NH));
  add_pair(n, off, "Network", Ar::FC, {Ar::NH, Ar::F}, Ar::F, bf, bf, &n->off_fc);
  add_heads<Ar>(n, off);
  n->nparams = align64(off);
  n->F = Ar::F;
  n->flat = Ar::FLAT;
  n->nconv = Ar::NCONV;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// Row of the x-product slabs that position k of window b reads.
//  window layout (nz == null): the caller's [B][5] frames, row b*5 + k;
//  frame-store layout: row 0 is the zero frame, row 1 + slot*E + e is env e's state of frame
//  slot `slot`; window b = (step t0 + b / E, env b % E) holds nz[b] leading zero frames, then
//  slots t..t+4 (paac.py:79-83: the window of step t is s_{t-4} .. s_t).
//  nz_prev != null (the native rollout, one step's E windows): nz[b] is derived here from the
//  previous step's count and that step's episode-end flag over[b] (host-mapped, written by the
//  emulator threads before the step's chain runs) — update_memory shifts one frame in, an
//  episode end zeroes the whole window (paac.py:173-174, :202-203) — and stored to nz[b].
struct XgRows {
  int32_t *nz;
  int t0, E;
  const int32_t *nz_prev = nullptr;
  const float *over = nullptr;
  // leading zero frames of window b (thread 0 of the block stores the derived count)
  __device__ __forceinline__ int zeros(int b) const {
    if (!nz) return 0;
    if (!nz_prev) return nz[b];
    const int z = over[b] != 0.f ? 5 : max(nz_prev[b] - 1, 0);
    if (threadIdx.x == 0) nz[b] = z;
    return z;
  }
  __device__ __forceinline__ int row(int b, int k, int z) const {
    if (!nz) return b * 5 + k;
    if (k < z) return 0;
    return 1 + (t0 + b / E + k) * E + b % E;
  }
};

// One workgroup (128 threads) per window b. xg: split-K slabs of x_t K_x, [S][rows][128].
// XS (the native rollout's macro-steps, lstm_step_fwd_impl): a per-frame cache xsum[rows][128] of
// the slab sums. Step 0 (XS 1) sums every position from its slabs, as XS 0 does, and stores each
// window's frame rows, block 0 also the zero frame's (row 0); steps t > 0 (XS 2) sum only position
// 4 — the frame the step's frames forward just computed — and read positions 0..3 from the cache:
// those frames were summed earlier in the same rollout under the same parameters, in the same
// slab order, so the values are the ones XS 0 would compute (50 loads per thread instead of 250).
template <int NH, int STEPS, int XS = 0>
__global__ __launch_bounds__(128) void lstm_fwd_kernel(const float *__restrict__ xg, int S, int rows, XgRows map,
                                                       const float *__restrict__ Kh, const float *__restrict__ kb,
                                                       const float *__restrict__ Wp, const float *__restrict__ bp,
                                                       const float *__restrict__ W6, int F, float forget_bias,
                                                       float *__restrict__ gates, float *__restrict__ cst,
                                                       float *__restrict__ hprev, float *__restrict__ h5,
                                                       float *__restrict__ out32, float *__restrict__ slab6,
                                                       float *__restrict__ xsum = nullptr) {
  constexpr int G4 = 4 * NH;
  __shared__ float hs[NH], as[G4], os[NH];
  const int b = blockIdx.x, g = threadIdx.x;
  const int q = g / NH;  // 0 i, 1 j, 2 f, 3 o
  float c = 0.f;
  if (g < NH) hs[g] = 0.f;
  // Loads in the order they are consumed (a wave's loads return in issue order): the x-product
  // slab sums of all STEPS positions first (they do not depend on h; XB slabs x STEPS loads in
  // flight per batch, adds in slab order — the frame store's x-product has 50 split-K slabs), and
  // behind the first batch every parameter of the recurrence and the epilogue (relaxed atomics:
  // plain read-only loads are sunk to their use, behind the recurrence barriers — the projection
  // bias was a load round trip of its own at the end); same products, same order below
  float zx[STEPS];
  size_t xoff[STEPS];
  const int z = map.zeros(b);
#pragma unroll
  for (int t = 0; t < STEPS; ++t) {
    zx[t] = 0.f;
    xoff[t] = (size_t)map.row(b, t, z) * G4 + g;
  }
  constexpr int T0 = XS == 2 ? STEPS - 1 : 0;  // first position summed from the slabs
  float xc[STEPS];                             // (XS 2: the cached sums of positions 0 .. T0 - 1)
#pragma unroll
  for (int t = 0; t < T0; ++t) xc[t] = xsum[xoff[t]];
  constexpr int XB = 25;
  float v[STEPS][XB];
  auto load_batch = [&](int s0) {
#pragma unroll
    for (int t = T0; t < STEPS; ++t)
#pragma unroll
      for (int u = 0; u < XB; ++u) v[t][u] = xg[(size_t)min(s0 + u, S - 1) * rows * G4 + xoff[t]];
  };
  load_batch(0);
  auto ld = [](const float *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  float wcol[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) wcol[k] = ld(Kh + (size_t)k * G4 + g);
  const float bias = ld(kb + g);
  constexpr int NN = 1;  // fc6 columns per thread: F <= NN * G4 (the launch sites assert it)
  float wpc[NH], w6c[NN][NH];
  const int gp = min(g, NH - 1);
#pragma unroll
  for (int m = 0; m < NH; ++m) wpc[m] = ld(Wp + m * NH + gp);
  const float bpg = ld(bp + gp);
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    const int nn = min(g + G4 * j, F - 1);
#pragma unroll
    for (int k = 0; k < NH; ++k) w6c[j][k] = ld(W6 + (size_t)k * F + nn);
  }
  for (int s0 = 0;;) {
#pragma unroll
    for (int t = T0; t < STEPS; ++t)
#pragma unroll
      for (int u = 0; u < XB; ++u)
        if (s0 + u < S) zx[t] += v[t][u];
    s0 += XB;
    if (s0 >= S) break;
    load_batch(s0);
  }
#pragma unroll
  for (int t = 0; t < T0; ++t) zx[t] = xc[t];
  if constexpr (XS != 0) {  // (rows of one step are distinct per window, but for the zero frame: same value)
#pragma unroll
    for (int t = T0; t < STEPS; ++t) xsum[xoff[t]] = zx[t];
  }
  if constexpr (XS == 1) {
    if (b == 0) {  // the zero frame, whether or not window 0 reads it (later steps' leading zeros do)
      float z0 = 0.f;
      for (int s0 = 0; s0 < S; s0 += XB) {
        float w0[XB];
#pragma unroll
        for (int u = 0; u < XB; ++u) w0[u] = xg[(size_t)min(s0 + u, S - 1) * rows * G4 + g];
#pragma unroll
        for (int u = 0; u < XB; ++u)
          if (s0 + u < S) z0 += w0[u];
      }
      xsum[g] = z0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < STEPS; ++t) {
    const int row = b * STEPS + t;
    float z = zx[t];
    float hz = 0.f;
#pragma unroll
    for (int k = 0; k < NH; ++k) hz += hs[k] * wcol[k];
    z = (z + hz) + bias;
    const float a = q == 1 ? tanhf(z) : sigmoidf_(q == 2 ? z + forget_bias : z);
    as[g] = a;
    gates[(size_t)row * G4 + g] = a;
    if (g < NH) hprev[(size_t)row * NH + g] = hs[g];
    __syncthreads();
    if (g < NH) {
      c = c * as[2 * NH + g] + as[g] * as[NH + g];
      const float h = tanhf(c) * as[3 * NH + g];
      cst[(size_t)row * NH + g] = c;
      hs[g] = h;
    }
    __syncthreads();
  }
  if (g < NH) {
    h5[(size_t)b * NH + g] = hs[g];
    float o = 0.f;
#pragma unroll
    for (int m = 0; m < NH; ++m) o += hs[m] * wpc[m];
    o += bpg;
    os[g] = o;
    out32[(size_t)b * NH + g] = o;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    const int nn = g + G4 * j;
    if (nn < F) {
      float z6 = 0.f;
#pragma unroll
      for (int k = 0; k < NH; ++k) z6 += os[k] * w6c[j][k];
      slab6[(size_t)b * F + nn] = z6;
    }
  }
}

// BPTT of one window (128 threads): dH [B][F] (already masked by fc6's activation derivative).
template <int NH, int STEPS>
__global__ __launch_bounds__(128) void lstm_bwd_kernel(const float *__restrict__ dH, int F,
                                                       const float *__restrict__ W6, const float *__restrict__ Wp,
                                                       const float *__restrict__ Kh, const float *__restrict__ gates,
                                                       const float *__restrict__ cst, float *__restrict__ dout32,
                                                       float *__restrict__ dgates) {
  constexpr int G4 = 4 * NH, KS = G4 + 1;  // K_h rows padded by one float: thread g's row read below
  __shared__ float khs[NH * KS];              // is on bank (g + j) % 32, not all 32 threads on one
  __shared__ float dos[NH], dzs[G4];
  const int b = blockIdx.x, g = threadIdx.x;
  // every operand of the window requested up front, K_h first (relaxed atomics: plain read-only
  // loads are sunk to their use — one load latency per step and per 8 products otherwise; K_h's
  // LDS copy was two round trips of its own before the rest were requested): K_h column g, the
  // projection row, every step's gates and cell states; the same products as the round-4 kernel,
  // but the two long dot products below are summed in four quarters added ((p0 + p1) + p2) + p3
  // (round 5), not in one sequential walk: an fp32 reduction order of its own (the oracle checks it
  // at the gradient tolerance; nothing is pinned to the old order)
  float khv[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) khv[k] = __hip_atomic_load(Kh + (size_t)k * G4 + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int gc = min(g, NH - 1);
  float wpr[NH], gt[STEPS][4], cs[STEPS];
#pragma unroll
  for (int k = 0; k < NH; ++k) wpr[k] = __hip_atomic_load(Wp + gc * NH + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int t = 0; t < STEPS; ++t) {
    const float *ga = gates + (size_t)(b * STEPS + t) * G4;
#pragma unroll
    for (int q = 0; q < 4; ++q) gt[t][q] = __hip_atomic_load(ga + q * NH + gc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cs[t] = __hip_atomic_load(cst + (size_t)(b * STEPS + t) * NH + gc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // d out = dH W6^T (fc6 input gradient) and each step's d h_{t-1} = dz K_h^T: NH outputs of long
  // dot products, so all G4 = 4 NH threads take part — thread (q, o) sums quarter q of output o's
  // terms (its loads in one trip), the quarters added in order by thread o through LDS
  static_assert(G4 == 4 * NH && NH <= 64, "four quarter-threads per output");
  __shared__ float part[4][NH];
  const int q = g / NH, o = g - q * NH;
  {
    const int FQ = (F + 3) / 4, n0 = q * FQ, n1 = min(F, n0 + FQ);
    const float *w = W6 + (size_t)o * F;
    const float *d = dH + (size_t)b * F;
    float a = 0.f;
    for (int c0 = n0; c0 < n1; c0 += 32) {
      float dv[32], wv[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        dv[u] = d[min(c0 + u, F - 1)];
        wv[u] = w[min(c0 + u, F - 1)];
      }
#pragma unroll
      for (int u = 0; u < 32; ++u)
        if (c0 + u < n1) a += dv[u] * wv[u];
    }
    part[q][o] = a;
  }
#pragma unroll
  for (int k = 0; k < NH; ++k) khs[k * KS + g] = khv[k];  // (after the dot's loads: one round trip)
  __syncthreads();
  if (g < NH) {
    const float a = ((part[0][g] + part[1][g]) + part[2][g]) + part[3][g];
    dos[g] = a;
    dout32[(size_t)b * NH + g] = a;
  }
  __syncthreads();
  float dh = 0.f, dc = 0.f;
  if (g < NH) {  // d h_5 = d out w^T
#pragma unroll
    for (int k = 0; k < NH; ++k) dh += dos[k] * wpr[k];
  }
#pragma unroll
  for (int t = STEPS - 1; t >= 0; --t) {
    const int row = b * STEPS + t;
    if (g < NH) {
      if (t < STEPS - 1) dh = ((part[0][g] + part[1][g]) + part[2][g]) + part[3][g];
      const float si = gt[t][0], tj = gt[t][1], sf = gt[t][2], so = gt[t][3];
      const float c = cs[t];
      const float cp = t > 0 ? cs[t > 0 ? t - 1 : 0] : 0.f;
      const float tc = tanhf(c);
      const float dzo = dh * tc * (so * (1.f - so));
      dc = dc + dh * so * (1.f - tc * tc);
      const float dzi = dc * tj * (si * (1.f - si));
      const float dzj = dc * si * (1.f - tj * tj);
      const float dzf = dc * cp * (sf * (1.f - sf));
      dc = dc * sf;
      dzs[g] = dzi;
      dzs[NH + g] = dzj;
      dzs[2 * NH + g] = dzf;
      dzs[3 * NH + g] = dzo;
    }
    __syncthreads();
    dgates[(size_t)row * G4 + g] = dzs[g];
    if (t > 0) {  // d h_{t-1} = dz K_h^T: quarter q of output o's terms
      float a = 0.f;
#pragma unroll 8
      for (int j = q * NH; j < (q + 1) * NH; ++j) a += dzs[j] * khs[o * KS + j];
      part[q][o] = a;
    }
    __syncthreads();
  }
}

template <class Ar>
static int lstm_forward_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                             float *v, float *pi, float *rep, const SampleArgs *smp, hipStream_t s) {
  LstmWs X;
  const WsLayout L = lstm_ws_layout<Ar>(n, B, &X);
  const int rows = B * Ar::STEPS;
  MT_TRY((trunk_forward<Ar>(n, P, obs, rows, ws, L, s)));
  const float *flat = layer_out<Ar, Ar::NCONV - 1>(ws, L);
  const float *Kx = P + n->off_lstm;
  const float *Kh = Kx + (size_t)Ar::FLAT * Ar::G4;
  const float *kb = Kh + (size_t)Ar::NH * Ar::G4;
  MT_TRY((launch_gemm<TileFc>(LdRowMajor{flat, Ar::FLAT}, LdColMajor{Kx, Ar::G4, -1},
                              EpSlab{ws + X.xg, rows, Ar::G4}, rows, Ar::G4, Ar::FLAT, X.xg_splits, s)));
  const float *Wp = P + n->off_proj;
  const float *W6 = P + n->off_fc;
  static_assert(Ar::F <= Ar::G4, "lstm_fwd_kernel: one fc6 column per thread");
  hipLaunchKernelGGL((lstm_fwd_kernel<Ar::NH, Ar::STEPS>), dim3(B), dim3(Ar::G4), 0, s, ws + X.xg, X.xg_splits,
                     rows, XgRows{nullptr, 0, 0}, Kh, kb, Wp, Wp + Ar::NH * Ar::NH, W6, Ar::F, 1.0f, ws + X.gates, ws + X.cst,
                     ws + X.hprev, ws + X.h5, ws + X.out32, ws + X.slab6);
  MT_LAUNCHED();
  HeadParams hp = head_params(n, P);
  return launch_heads(B, s, ws + X.slab6, 1, B, W6 + (size_t)Ar::NH * Ar::F, n->cfg.activation, n->cfg.alpha_leaky,
                      hp, n->cfg.softmax_temp, ws + L.H, v, pi, rep, smp ? *smp : SampleArgs{});
}

template <class Ar>
static int lstm_backward_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                              const float *pi, const float *rep, const float *v, const int32_t *a_idx,
                              const int32_t *r_idx, const float *y, const float *adv, float beta, float *grad,
                              float *loss_terms, hipStream_t s) {
  LstmWs X;
  const WsLayout L = lstm_ws_layout<Ar>(n, B, &X);
  const int rows = B * Ar::STEPS;
  const int act = n->cfg.activation;
  const float al = n->cfg.alpha_leaky;
  MT_TRY(heads_backward<Ar>(n, P, B, ws, L, pi, rep, v, a_idx, r_idx, y, adv, beta, grad, loss_terms, s));
  const float *Kx = P + n->off_lstm;
  const float *Kh = Kx + (size_t)Ar::FLAT * Ar::G4;
  const float *Wp = P + n->off_proj;
  const float *W6 = P + n->off_fc;
  // fc6 dW, db: [out, 1]^T dH
  MT_TRY((launch_gemm<TileDenseW>(LdColMajor{ws + X.out32, Ar::NH, Ar::NH}, LdColMajor{ws + L.dH, Ar::F, -1},
                                  EpStore{grad + n->off_fc, Ar::F}, Ar::NH + 1, Ar::F, B, 1, s)));
  hipLaunchKernelGGL((lstm_bwd_kernel<Ar::NH, Ar::STEPS>), dim3(B), dim3(Ar::G4), 0, s, ws + L.dH, Ar::F, W6, Wp,
                     Kh, ws + X.gates, ws + X.cst, ws + X.dout32, ws + X.dgates);
  MT_LAUNCHED();
  // projection dW, db: [h_5, 1]^T d out
  MT_TRY((launch_gemm<TileDenseW>(LdColMajor{ws + X.h5, Ar::NH, Ar::NH}, LdColMajor{ws + X.dout32, Ar::NH, -1},
                                  EpStore{grad + n->off_proj, Ar::NH}, Ar::NH + 1, Ar::NH, B, 1, s)));
  // cell kernel: x rows [X]^T dz, then h rows + bias [h_{t-1}, 1]^T dz (bias follows K_h)
  MT_TRY((launch_gemm<TileDenseW>(LdColMajor{layer_out<Ar, Ar::NCONV - 1>(ws, L), Ar::FLAT, -1},
                                  LdColMajor{ws + X.dgates, Ar::G4, -1}, EpStore{grad + n->off_lstm, Ar::G4},
                                  Ar::FLAT, Ar::G4, rows, 1, s)));
  MT_TRY((launch_gemm<TileDenseW>(LdColMajor{ws + X.hprev, Ar::NH, Ar::NH}, LdColMajor{ws + X.dgates, Ar::G4, -1},
                                  EpStore{grad + n->off_lstm + (size_t)Ar::FLAT * Ar::G4, Ar::G4}, Ar::NH + 1,
                                  Ar::G4, rows, 1, s)));
  // d flat = dz K_x^T, masked by conv4's activation (conv4 is not pooled), then the trunk
  constexpr int K = Ar::NCONV - 1;
  static_assert(!pooled<Ar, K>(), "LSTM trunk ends in an unpooled conv");
  MT_TRY((launch_gemm<TileDenseX>(LdRowMajor{ws + X.dgates, Ar::G4}, LdRowMajor{Kx, Ar::G4},
                                  EpMasked{ws + L.dact[K], layer_out<Ar, K>(ws, L), Ar::FLAT, act, al}, rows,
                                  Ar::FLAT, Ar::G4, 1, s)));
  return trunk_backward<Ar, K>(n, P, obs, rows, ws, L, grad, s);
}

// ---------------------------------------------------------------------------------------------
// Frame-store mode (the learner's path). A window of step t is frames s_{t-4} .. s_t of one env
// with nz leading zero frames (paac.py:79-83, :202-203), so consecutive windows share 4 of their
// 5 frames and the trunk + x-product of every distinct frame is computed ONCE per parameter
// version: the frame store holds row 0 = the zero frame and rows 1 + slot*E + e (slot 0..3 = the
// previous rollout's last 4 states, slot 4 + t = s_t), and the workspace keeps every row's
// trunk activations and x-product slabs. The rollout computes the new rows of each step and the
// recurrence of its E windows (window t*E + e); the train pass reuses all of it (the parameters
// have not changed since the rollout) and back-propagates through each distinct frame once,
// with the gate gradients of the windows that read it summed per frame first (exact by
// linearity; fixed summation order).
// ---------------------------------------------------------------------------------------------
struct LstmFrameWs {
  WsLayout L;
  size_t xg, xsum, dxg, zpart, slab6, gates, cst, hprev, h5, out32, dout32, dgates;
  int S, R_max, R_bwd, W;
};

constexpr int kZeroParts = 64;  // partial sums of the zero frame's gate gradients

template <class Ar, int I = 0>
static size_t max_wgrad_slab(int B) {
  if constexpr (I < Ar::NCONV) return std::max(conv_wgrad_slab<LayerG<Ar, I>>(B), max_wgrad_slab<Ar, I + 1>(B));
  return 0;
}

template <class Ar>
static LstmFrameWs lstm_frame_layout(const mt_net *n, int E, int T) {
  LstmFrameWs X{};
  X.R_max = 1 + (T + 5) * E;
  X.R_bwd = 1 + (T + 4) * E;  // slot 4 + T (s_T) is read by the bootstrap only
  X.W = (T + 1) * E;          // windows of steps 0..T (T = bootstrap)
  size_t off = 0;
  auto take = [&](size_t nf) {
    size_t o = off;
    off = align64(off + nf);
    return o;
  };
  size_t wslab = 0;
  ws_layers<Ar>(X.L, off, X.R_max, wslab);
  wslab = std::max(wslab, max_wgrad_slab<Ar>(X.R_bwd));
  const int s = pick_splits(cdiv(E, TileFc::BM) * cdiv(Ar::G4, TileFc::BN), Ar::FLAT, TileFc::BK, 128);
  X.S = gemm_splits<TileFc>(Ar::FLAT, s);
  const size_t W = X.W, WT = (size_t)T * E;
  X.xg = take((size_t)X.S * X.R_max * Ar::G4);
  X.xsum = take((size_t)X.R_max * Ar::G4);
  X.dxg = take((size_t)X.R_max * Ar::G4);
  X.zpart = take((size_t)kZeroParts * Ar::G4);
  X.slab6 = take(W * Ar::F);
  X.gates = take(W * Ar::STEPS * Ar::G4);
  X.cst = take(W * Ar::STEPS * Ar::NH);
  X.hprev = take(W * Ar::STEPS * Ar::NH);
  X.h5 = take(W * Ar::NH);
  X.out32 = take(W * Ar::NH);
  X.dout32 = take(WT * Ar::NH);
  X.dgates = take(WT * Ar::STEPS * Ar::G4);
  X.L.fc_splits = 1;
  X.L.fcslab = X.slab6;
  X.L.H = take(W * Ar::F);
  X.L.dz = take(WT * n->O);
  X.L.dH = take(WT * Ar::F);
  X.L.wslab = take(wslab);
  X.L.wslab2 = take(wslab);
  X.L.total = off;
  return X;
}

// Zero frame (row 0): partial sums over window chunks of the gate gradients of the positions
// that read it (k < nz), 128 threads = gate columns; summed in chunk order by the gather kernel.
__global__ __launch_bounds__(128) void lstm_zero_partials_kernel(const float *__restrict__ dgates,
                                                                 const int32_t *__restrict__ nz, int W,
                                                                 float *__restrict__ part) {
  const int g = threadIdx.x, c = blockIdx.x;
  const int per = cdiv(W, gridDim.x);
  float acc = 0.f;
  for (int w = c * per; w < min(W, (c + 1) * per); ++w) {  // (a window's loads in one round trip)
    const int z = nz[w];
    float v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) v[k] = dgates[((size_t)w * 5 + k) * 128 + g];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (k < z) acc += v[k];
  }
  part[(size_t)c * 128 + g] = acc;
}

// dxg[r] = sum of the gate gradients of every (window, position) that reads frame row r:
// row 1 + j*E + e is position k of window (t = j - k, e) when 0 <= t < T and k >= nz[t][e].
__global__ __launch_bounds__(128) void lstm_gather_dxg_kernel(const float *__restrict__ dgates,
                                                              const int32_t *__restrict__ nz, int T, int E,
                                                              const float *__restrict__ zpart, int nparts,
                                                              float *__restrict__ dxg) {
  const int r = blockIdx.x, g = threadIdx.x;
  float acc = 0.f;
  if (r == 0) {  // the zero frame: the partials in batches of 16 loads in flight, added in order
    for (int c0 = 0; c0 < nparts; c0 += 16) {
      float p[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) p[u] = zpart[(size_t)min(c0 + u, nparts - 1) * 128 + g];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (c0 + u < nparts) acc += p[u];
    }
  } else {
    const int j = (r - 1) / E, e = (r - 1) % E;
    // every load first, from clamped addresses (a guarded load ends its block with a wait for it);
    // the terms that do not apply are skipped as before
    int zk[5];
    float v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int tc = min(max(j - k, 0), T - 1);
      zk[k] = nz[tc * E + e];
      v[k] = dgates[(((size_t)tc * E + e) * 5 + k) * 128 + g];
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int t = j - k;
      if (t >= 0 && t < T && k >= zk[k]) acc += v[k];
    }
  }
  dxg[(size_t)r * 128 + g] = acc;
}

// st (the native rollout's pipelined steps): rows [row0, row0 + nrows) are the step's E new
// states, stacked from st->prev and env e's pushes by the conv1 launch itself (dconv.h
// launch_stack_conv1: pull + stack + conv1 per env as each env is published; sync = its
// stack_conv1_sync_words(E) zeroed words), then conv2 .. conv4 layered (net.hip trunk_forward).
template <class Ar>
static int lstm_frames_fwd_impl(const mt_net *n, const float *P, const uint8_t *fstore, int row0, int nrows,
                                int E, int T, float *ws, hipStream_t s, const StackSrc *st = nullptr,
                                uint32_t *sync = nullptr) {
  const LstmFrameWs X = lstm_frame_layout<Ar>(n, E, T);
  MT_CHECK_ARG(row0 >= 0 && nrows >= 1 && row0 + nrows <= X.R_max, "rows [%d, %d) outside the frame store [0, %d)",
               row0, row0 + nrows, X.R_max);
  constexpr size_t FB = (size_t)84 * 84 * LayerG<Ar, 0>::CIN;
  WsLayout Ls = X.L;
  shift_rows<Ar>(Ls, (size_t)row0);
  MT_CHECK_ARG(!st || (sync && nrows == E && st->out == fstore + (size_t)row0 * FB),
               "stacking conv1: the step's E new rows, a counter region");
  FwdExtras ex;
  ex.st = st;
  ex.sync = sync;
  MT_TRY((trunk_forward<Ar>(n, P, fstore + (size_t)row0 * FB, nrows, ws, Ls, s, ex)));
  return launch_gemm<TileFc>(LdRowMajor{layer_out<Ar, Ar::NCONV - 1>(ws, Ls), Ar::FLAT},
                             LdColMajor{P + n->off_lstm, Ar::G4, -1},
                             EpSlab{ws + X.xg + (size_t)row0 * Ar::G4, X.R_max, Ar::G4}, nrows, Ar::G4, Ar::FLAT,
                             X.S, s);
}

// xs: the per-frame x-product sum cache (lstm_fwd_kernel XS; the native rollout's macro-steps only,
// whose step t > 0 follows steps 0 .. t - 1 of the same rollout under the same parameters)
template <class Ar>
static int lstm_windows_fwd_impl(const mt_net *n, const float *P, int32_t *nz_t, int t, int E, int T,
                                 float *ws, float *v, float *pi, float *rep, hipStream_t s,
                                 const SampleArgs *smp = nullptr, const int32_t *nz_prev = nullptr,
                                 const float *over = nullptr, bool xs = false) {
  MT_CHECK_ARG(t >= 0 && t <= T, "step %d outside [0, %d]", t, T);
  const LstmFrameWs X = lstm_frame_layout<Ar>(n, E, T);
  const size_t w0 = (size_t)t * E;
  const float *Kh = P + n->off_lstm + (size_t)Ar::FLAT * Ar::G4;
  const float *Wp = P + n->off_proj;
  const float *W6 = P + n->off_fc;
  static_assert(Ar::F <= Ar::G4, "lstm_fwd_kernel: one fc6 column per thread");
  auto kern = !xs ? &lstm_fwd_kernel<Ar::NH, Ar::STEPS, 0>
                  : (t == 0 ? &lstm_fwd_kernel<Ar::NH, Ar::STEPS, 1> : &lstm_fwd_kernel<Ar::NH, Ar::STEPS, 2>);
  hipLaunchKernelGGL(kern, dim3(E), dim3(Ar::G4), 0, s, ws + X.xg, X.S, X.R_max, XgRows{nz_t, t, E, nz_prev, over}, Kh,
                     Kh + Ar::NH * Ar::G4, Wp, Wp + Ar::NH * Ar::NH, W6, Ar::F, 1.0f,
                     ws + X.gates + w0 * Ar::STEPS * Ar::G4, ws + X.cst + w0 * Ar::STEPS * Ar::NH,
                     ws + X.hprev + w0 * Ar::STEPS * Ar::NH, ws + X.h5 + w0 * Ar::NH, ws + X.out32 + w0 * Ar::NH,
                     ws + X.slab6 + w0 * Ar::F, xs ? ws + X.xsum : nullptr);
  MT_LAUNCHED();
  HeadParams hp = head_params(n, P);
  return launch_heads(E, s, ws + X.slab6 + w0 * Ar::F, 1, E, W6 + (size_t)Ar::NH * Ar::F, n->cfg.activation,
                      n->cfg.alpha_leaky, hp, n->cfg.softmax_temp, ws + X.L.H + w0 * Ar::F, v, pi, rep,
                      smp ? *smp : SampleArgs{});
}

// One macro-step forward of the frame-store LSTM inside the native rollout (rollout.hip): the
// trunk + x-product of the step's new frame rows (step 0: the zero frame and slots 0..4 again,
// the parameters having changed; step t > 0: slot 4 + t), then the recurrence of its E windows
// with the draw fused into the heads kernel (smp; null for the bootstrap, t == T). t > 0: nz[t]
// is derived on the device from nz[t-1] and step t-1's episode-end flags `over` (XgRows).
// marks: optional event pair around the trunk launches (mt_rollout_trunk_timing).
template <class Ar>
static int lstm_step_fwd_impl(const mt_net *n, const float *P, const uint8_t *fstore, int t, int E, int T,
                              int32_t *nz, const float *over, float *ws, float *v, float *pi, float *rep,
                              const SampleArgs *smp, hipStream_t s, const hipEvent_t *marks,
                              const StackSrc *st = nullptr, uint32_t *sync = nullptr) {
  MT_CHECK_ARG(t >= 0 && t <= T, "step %d outside [0, %d]", t, T);
  MT_CHECK_ARG(t == 0 || over, "steps t > 0 need the episode-end flags");
  const int row0 = t == 0 ? 0 : 1 + (4 + t) * E, nrows = t == 0 ? 1 + 5 * E : E;
  if (marks) MT_HIP(hipEventRecord(marks[0], s));
  MT_CHECK_ARG(!st || t > 0, "step 0 has no pushes to stack");
  MT_TRY((lstm_frames_fwd_impl<Ar>(n, P, fstore, row0, nrows, E, T, ws, s, st, sync)));
  if (marks) MT_HIP(hipEventRecord(marks[1], s));
  return lstm_windows_fwd_impl<Ar>(n, P, nz + (size_t)t * E, t, E, T, ws, v, pi, rep, s, smp,
                                   t > 0 ? nz + (size_t)(t - 1) * E : nullptr, t > 0 ? over : nullptr, true);
}

template <class Ar>
static int lstm_frames_bwd_impl(const mt_net *n, const float *P, const uint8_t *fstore, const int32_t *nz, int E,
                                int T, float *ws, const float *pi, const float *rep, const float *v,
                                const int32_t *a_idx, const int32_t *r_idx, const float *y, const float *adv,
                                float beta, float *grad, float *loss_terms, hipStream_t s,
                                const NormOut &no = NormOut{}) {
  const LstmFrameWs X = lstm_frame_layout<Ar>(n, E, T);
  const WsLayout &L = X.L;
  const int W = T * E, rows = W * Ar::STEPS;
  const int act = n->cfg.activation;
  const float al = n->cfg.alpha_leaky;
  if (sizeof(float) * ((size_t)W + 4 * 64) > 160 * 1024) {
    set_error("batch %d exceeds the head-gradient LDS stage", W);
    return MT_ERR_ARG;
  }
  MT_TRY(loss_bwd_launch<Ar>(n, P, W, ws, L, pi, rep, v, a_idx, r_idx, y, adv, beta, loss_terms, s));
  const float *Kx = P + n->off_lstm;
  const float *Kh = Kx + (size_t)Ar::FLAT * Ar::G4;
  const float *Wp = P + n->off_proj;
  const float *W6 = P + n->off_fc;
  // (every launch of the frames backward is numbered by the launch window, so bench.py times it
  // launch by launch: bench.launch_breakdown)
  if (launch_allowed()) {
    hipLaunchKernelGGL((lstm_bwd_kernel<Ar::NH, Ar::STEPS>), dim3(W), dim3(Ar::G4), 0, s, ws + L.dH, Ar::F, W6, Wp,
                       Kh, ws + X.gates, ws + X.cst, ws + X.dout32, ws + X.dgates);
    MT_LAUNCHED();
  }
  // the small weight gradients — K_h rows + bias [h_{t-1}, 1]^T dz, fc6 [out, 1]^T dH, the heads,
  // the projection [h_5, 1]^T d out: a few blocks each, a serial walk of up to 10 K chunks — are off
  // the critical path: they run beside conv4's backward (trunk_backward's extra jobs, longest walk
  // first) instead of as four launches of their own (same products, same chunks)
  const JobPack small{
      gemm_job<TileDenseW>(LdColMajor{ws + X.hprev, Ar::NH, Ar::NH}, LdColMajor{ws + X.dgates, Ar::G4, -1},
                           EpStore{grad + n->off_lstm + (size_t)Ar::FLAT * Ar::G4, Ar::G4}, Ar::NH + 1, Ar::G4, rows,
                           1),
      gemm_job<TileDenseW>(LdColMajor{ws + X.out32, Ar::NH, Ar::NH}, LdColMajor{ws + L.dH, Ar::F, -1},
                           EpStore{grad + n->off_fc, Ar::F}, Ar::NH + 1, Ar::F, W, 1),
      head_wgrad_job<Ar>(n, W, ws, L, grad),
      gemm_job<TileDenseW>(LdColMajor{ws + X.h5, Ar::NH, Ar::NH}, LdColMajor{ws + X.dout32, Ar::NH, -1},
                           EpStore{grad + n->off_proj, Ar::NH}, Ar::NH + 1, Ar::NH, W, 1)};
  // per-frame gate gradients (the zero frame: chunk partials first)
  if (launch_allowed()) {
    hipLaunchKernelGGL(lstm_zero_partials_kernel, dim3(kZeroParts), dim3(Ar::G4), 0, s, ws + X.dgates, nz, W,
                       ws + X.zpart);
    MT_LAUNCHED();
  }
  if (launch_allowed()) {
    hipLaunchKernelGGL(lstm_gather_dxg_kernel, dim3(X.R_bwd), dim3(Ar::G4), 0, s, ws + X.dgates, nz, T, E,
                       ws + X.zpart, kZeroParts, ws + X.dxg);
    MT_LAUNCHED();
  }
  constexpr int K = Ar::NCONV - 1;
  const float *flat = layer_out<Ar, K>(ws, L);
  // d flat = dxg K_x^T (masked by conv4's activation; the trunk's critical path, first) and the
  // cell kernel's x rows [flat]^T dxg, one grouped launch
  const auto dx = gemm_job<TileDenseX>(LdRowMajor{ws + X.dxg, Ar::G4}, LdRowMajor{Kx, Ar::G4},
                                       EpMasked{ws + L.dact[K], flat, Ar::FLAT, act, al}, X.R_bwd, Ar::FLAT, Ar::G4, 1);
  const auto kxw = gemm_job<TileDenseW>(LdColMajor{flat, Ar::FLAT, -1}, LdColMajor{ws + X.dxg, Ar::G4, -1},
                                        EpStore{grad + n->off_lstm, Ar::G4}, Ar::FLAT, Ar::G4, X.R_bwd, 1);
  MT_TRY(launch_group(s, dx, kxw));
  return trunk_backward<Ar, K>(n, P, fstore, X.R_bwd, ws, L, grad, s, SlabJob{}, no, small);
}

}  // namespace mt
