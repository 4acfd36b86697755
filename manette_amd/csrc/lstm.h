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

// One workgroup (128 threads) per window b. xg: split-K slabs of x_t K_x, [S][5B][128].
template <int NH, int STEPS>
__global__ __launch_bounds__(128) void lstm_fwd_kernel(const float *__restrict__ xg, int S, int rows,
                                                       const float *__restrict__ Kh, const float *__restrict__ kb,
                                                       const float *__restrict__ Wp, const float *__restrict__ bp,
                                                       const float *__restrict__ W6, int F, float forget_bias,
                                                       float *__restrict__ gates, float *__restrict__ cst,
                                                       float *__restrict__ hprev, float *__restrict__ h5,
                                                       float *__restrict__ out32, float *__restrict__ slab6) {
  constexpr int G4 = 4 * NH;
  __shared__ float hs[NH], as[G4], os[NH];
  const int b = blockIdx.x, g = threadIdx.x;
  float wcol[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) wcol[k] = Kh[(size_t)k * G4 + g];
  const float bias = kb[g];
  const int q = g / NH;  // 0 i, 1 j, 2 f, 3 o
  float c = 0.f;
  if (g < NH) hs[g] = 0.f;
  __syncthreads();
  for (int t = 0; t < STEPS; ++t) {
    const int row = b * STEPS + t;
    float z = 0.f;
    for (int s = 0; s < S; ++s) z += xg[((size_t)s * rows + row) * G4 + g];
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
#pragma unroll 8
    for (int m = 0; m < NH; ++m) o += hs[m] * Wp[m * NH + g];
    o += bp[g];
    os[g] = o;
    out32[(size_t)b * NH + g] = o;
  }
  __syncthreads();
  for (int nn = g; nn < F; nn += G4) {
    float z6 = 0.f;
#pragma unroll 8
    for (int k = 0; k < NH; ++k) z6 += os[k] * W6[(size_t)k * F + nn];
    slab6[(size_t)b * F + nn] = z6;
  }
}

// BPTT of one window (128 threads): dH [B][F] (already masked by fc6's activation derivative).
template <int NH, int STEPS>
__global__ __launch_bounds__(128) void lstm_bwd_kernel(const float *__restrict__ dH, int F,
                                                       const float *__restrict__ W6, const float *__restrict__ Wp,
                                                       const float *__restrict__ Kh, const float *__restrict__ gates,
                                                       const float *__restrict__ cst, float *__restrict__ dout32,
                                                       float *__restrict__ dgates) {
  constexpr int G4 = 4 * NH;
  __shared__ float khs[NH * G4];
  __shared__ float dos[NH], dzs[G4];
  const int b = blockIdx.x, g = threadIdx.x;
  for (int i = g; i < NH * G4; i += G4) khs[i] = Kh[i];
  if (g < NH) {  // d out = dH W6^T  (fc6 input gradient)
    float a = 0.f;
    const float *w = W6 + (size_t)g * F;
    const float *d = dH + (size_t)b * F;
    for (int nn = 0; nn < F; ++nn) a += d[nn] * w[nn];
    dos[g] = a;
    dout32[(size_t)b * NH + g] = a;
  }
  __syncthreads();
  float dh = 0.f, dc = 0.f;
  if (g < NH) {  // d h_5 = d out w^T
#pragma unroll 8
    for (int k = 0; k < NH; ++k) dh += dos[k] * Wp[g * NH + k];
  }
  for (int t = STEPS - 1; t >= 0; --t) {
    const int row = b * STEPS + t;
    if (g < NH) {
      const float *ga = gates + (size_t)row * G4;
      const float si = ga[g], tj = ga[NH + g], sf = ga[2 * NH + g], so = ga[3 * NH + g];
      const float c = cst[(size_t)row * NH + g];
      const float cp = t > 0 ? cst[(size_t)(row - 1) * NH + g] : 0.f;
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
    if (g < NH) {  // d h_{t-1} = dz K_h^T
      float a = 0.f;
#pragma unroll 8
      for (int j = 0; j < G4; ++j) a += dzs[j] * khs[g * G4 + j];
      dh = a;
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
  hipLaunchKernelGGL((lstm_fwd_kernel<Ar::NH, Ar::STEPS>), dim3(B), dim3(Ar::G4), 0, s, ws + X.xg, X.xg_splits,
                     rows, Kh, kb, Wp, Wp + Ar::NH * Ar::NH, W6, Ar::F, 1.0f, ws + X.gates, ws + X.cst,
                     ws + X.hprev, ws + X.h5, ws + X.out32, ws + X.slab6);
  MT_LAUNCHED();
  HeadParams hp = head_params(n, P);
  hipLaunchKernelGGL(heads_fwd_kernel, dim3(B), dim3(256), 0, s, ws + X.slab6, 1, B, W6 + (size_t)Ar::NH * Ar::F,
                     n->cfg.activation, n->cfg.alpha_leaky, hp, n->cfg.softmax_temp, ws + L.H, v, pi, rep,
                     smp ? *smp : SampleArgs{});
  MT_LAUNCHED();
  return MT_OK;
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

}  // namespace mt
