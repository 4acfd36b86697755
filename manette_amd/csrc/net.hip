// Policy/value network of the PAAC hot path on gfx950: parameter layout, forward (A5-A7) and
// fused loss + backward (A10).
//
// Reference: networks.py:130-278 (trunks), policy_v_network.py:19-74 (heads + loss).
// Trunk products run on the fp32 MFMA GEMM core (gemm.h) with implicit im2col loaders; the
// small heads (critic 1, actor A, repetition R outputs) and the loss are one workgroup per row.
#include <string>
#include <vector>
#include <cmath>
#include <algorithm>
#include <tuple>

#include "gemm.h"
#include "jobs.h"
#include "trunk_fused.h"
#include "nips_bwd.h"
#include "dconv.h"
#include "nature_bwd.h"

namespace mt {

// ---------------------------------------------------------------------------------------------
// Architectures (compile-time geometry). C = 4*depth input channels. Layers = tuple of conv
// geometries; POOL bitmask = layers followed by a 2x2/2 VALID max pool (networks.py:108-110).
// ---------------------------------------------------------------------------------------------
template <int C>
struct NipsArch {  // networks.py:178-192
  using Layers = std::tuple<ConvGeom<C, 16, 8, 4, 84, 84, false>, ConvGeom<16, 32, 4, 2, 20, 20, false>>;
  static constexpr int NCONV = 2;
  static constexpr unsigned POOL = 0;
  static constexpr int FLAT = 9 * 9 * 32;  // 2592
  static constexpr int F = 256;
  static constexpr const char *FC = "fc3";
  static constexpr int FUSED_SLABS = FusedNips<C>::FC_SPLITS;  // inference forward: trunk_fused.h
  static constexpr int FC_ROWS = 0;                         // (the fused trunk has its own dense kernel)
  static constexpr bool LSTM = false;
};
template <int C>
struct NatureArch {  // networks.py:261-278
  using Layers = std::tuple<ConvGeom<C, 32, 8, 4, 84, 84, false>, ConvGeom<32, 64, 4, 2, 20, 20, false>,
                            ConvGeom<64, 64, 3, 1, 9, 9, false>>;
  static constexpr int NCONV = 3;
  static constexpr unsigned POOL = 0;
  static constexpr int FLAT = 7 * 7 * 64;  // 3136
  static constexpr int F = 512;
  static constexpr const char *FC = "fc4";
  static constexpr int FUSED_SLABS = 0;  // no fused inference trunk: layered path
  static constexpr int FC_ROWS = 7;      // dense layer by conv3 rows (row_fc_kernel)
  // its K-splits (= slabs): 8, 512 blocks at E = 32 / 64 (two per CU) instead of 7 rows' 448
  // (Breakout isolated step forward 39.5 -> 38.5 us; 4 splits, 256 blocks: slower; profiles/r06fcs)
  static constexpr int FC_SPLITS = 8;
  static constexpr bool LSTM = false;
};
template <int C>
struct PwyxArch {  // networks.py:206-225: SAME convs, 2x2 pools after conv1-3
  using Layers = std::tuple<ConvGeom<C, 32, 5, 1, 84, 84, true>, ConvGeom<32, 32, 5, 1, 42, 42, true>,
                            ConvGeom<32, 64, 4, 1, 21, 21, true>, ConvGeom<64, 64, 3, 1, 10, 10, true>>;
  static constexpr int NCONV = 4;
  static constexpr unsigned POOL = 0x7;
  static constexpr int FLAT = 10 * 10 * 64;  // 6400
  static constexpr int F = 512;
  static constexpr const char *FC = "fc5";
  static constexpr int FUSED_SLABS = 0;
  static constexpr int FC_ROWS = 10;  // dense layer by conv4 rows (row_fc_kernel)
  static constexpr int FC_SPLITS = 8;  // its K-splits: 512 blocks at E = 32 (10: 640), as NATURE's
  static constexpr bool LSTM = false;
};

template <class Ar, int I>
using LayerG = std::tuple_element_t<I, typename Ar::Layers>;

// gray NATURE: the rollout chain stacks in conv1 and runs its convs as one dataflow launch
// (dconv.h nature_chain_kernel)
template <class Ar>
constexpr bool nature_stacking() {
  if constexpr (Ar::LSTM || Ar::NCONV != 3) return false;
  else return LayerG<Ar, 0>::CIN == 4 && !LayerG<Ar, 0>::SAME;
}

// The NIPS gray trunk's conv backward as one launch of per-image workgroups (nips_bwd.h) instead of
// the layered trunk_backward.
// Its slabs are per image (257 x 16 floats each, summed serially per column), so above this batch
// the layered trunk_backward (split-K slabs capped at kSlabFloats) takes over: at the benchmarked
// batches (N = E * T <= 1,280) the fused form's two slab regions stay <= 21 MB each.
constexpr int kNipsFusedBwdMaxRows = 1280;
template <class Ar>
constexpr bool nips_fused_bwd() {
  if constexpr (Ar::LSTM || Ar::NCONV != 2 || Ar::FUSED_SLABS == 0) return false;
  else return LayerG<Ar, 0>::CIN == 4;
}
template <class Ar, int I>
constexpr bool pooled() {
  return (Ar::POOL >> I) & 1u;
}
// the frame trunks (PWYX, LSTM; gray or RGB): the rollout step's conv1 launch pulls + stacks each
// env as it is published (dconv.h stack_conv1_kernel), conv2 .. layered
template <class Ar>
constexpr bool frame_stacking() {
  using G = LayerG<Ar, 0>;
  return G::S == 1 && G::SAME && pooled<Ar, 0>() && (G::CIN == 4 || G::CIN == 12) && G::H == 84 && G::W == 84;
}
// spatial size of layer I's output after its (optional) pool
template <class Ar, int I>
constexpr int out_hw() {
  using G = LayerG<Ar, I>;
  return pooled<Ar, I>() ? G::OH / 2 : G::OH;
}

}  // namespace mt

struct VarInfo {
  std::string name;
  int ndim;
  int64_t shape[4];
  size_t offset;
  float bound;
};

struct mt_net {
  mt_net_config cfg;
  int C;       // input channels (4*depth)
  int F;       // trunk feature width
  int O;       // 1 + A + R head outputs
  int nconv;
  int flat;
  std::vector<VarInfo> vars;
  size_t nparams;
  size_t off_conv[4];  // weights offset of each conv (biases follow)
  size_t off_fc, off_critic, off_actor, off_rep;
  size_t off_lstm = 0, off_proj = 0;  // LSTM arch: cell kernel (+bias), projection w (+b)
};

namespace mt {

static size_t align64(size_t x) { return (x + 63) & ~size_t(63); }

static void add_named_pair(mt_net *n, size_t &off, const std::string &wname, const std::string &bname,
                           std::vector<int64_t> wshape, int64_t nb, float bw, float bb, size_t *woff) {
  off = align64(off);
  VarInfo w{};
  w.name = wname;
  w.ndim = (int)wshape.size();
  size_t ws = 1;
  for (int i = 0; i < w.ndim; ++i) {
    w.shape[i] = wshape[i];
    ws *= (size_t)wshape[i];
  }
  w.offset = off;
  w.bound = bw;
  VarInfo b{};
  b.name = bname;
  b.ndim = 1;
  b.shape[0] = nb;
  b.offset = off + ws;
  b.bound = bb;
  *woff = off;
  n->vars.push_back(w);
  n->vars.push_back(b);
  off = off + ws + (size_t)nb;
}

static void add_pair(mt_net *n, size_t &off, const std::string &scope, const std::string &nm,
                     std::vector<int64_t> wshape, int64_t nb, float bw, float bb, size_t *woff) {
  add_named_pair(n, off, scope + "/" + nm + "/" + nm + "_weights", scope + "/" + nm + "/" + nm + "_biases",
                 std::move(wshape), nb, bw, bb, woff);
}

template <class G>
static void add_conv(mt_net *n, size_t &off, int idx) {
  // networks.py:34-55: weights U(+-1/sqrt(filters*k*k)) (shape[3] is the OUTPUT channel count),
  // biases U(+-1/sqrt(in_channels*k*k)).
  const float bw = (float)(1.0 / std::sqrt((double)(G::COUT * G::KH * G::KW)));
  const float bb = (float)(1.0 / std::sqrt((double)(G::CIN * G::KH * G::KW)));
  std::string nm = "conv" + std::to_string(idx + 1);
  add_pair(n, off, "Network", nm, {G::KH, G::KW, G::CIN, G::COUT}, G::COUT, bw, bb,
           &n->off_conv[idx]);
}

template <class Ar, int I = 0>
static void add_convs(mt_net *n, size_t &off) {
  if constexpr (I < Ar::NCONV) {
    add_conv<LayerG<Ar, I>>(n, off, I);
    add_convs<Ar, I + 1>(n, off);
  }
}

template <class Ar>
static void add_heads(mt_net *n, size_t &off) {
  const float bh = (float)(1.0 / std::sqrt((double)Ar::F));
  const int A = n->cfg.num_actions, R = n->cfg.num_reps;
  // policy_v_network.py:22 (critic), :31 (actor), :47 (repetition) — TF creation order.
  add_pair(n, off, "Training/Critic", "critic_output", {Ar::F, 1}, 1, bh, bh, &n->off_critic);
  add_pair(n, off, "Training/Actor", "actor_output", {Ar::F, A}, A, bh, bh, &n->off_actor);
  add_pair(n, off, "Training/Repetition", "repetition_output", {Ar::F, R}, R, bh, bh, &n->off_rep);
}

template <class Ar>
static void build_layout(mt_net *n) {
  static_assert(out_hw<Ar, Ar::NCONV - 1>() * out_hw<Ar, Ar::NCONV - 1>() *
                    LayerG<Ar, Ar::NCONV - 1>::COUT == Ar::FLAT, "flatten width");
  size_t off = 0;
  add_convs<Ar>(n, off);
  const float bf = (float)(1.0 / std::sqrt((double)Ar::FLAT));  // networks.py:72-89
  add_pair(n, off, "Network", Ar::FC, {Ar::FLAT, Ar::F}, Ar::F, bf, bf, &n->off_fc);
  add_heads<Ar>(n, off);
  n->nparams = align64(off);
  n->F = Ar::F;
  n->flat = Ar::FLAT;
  n->nconv = Ar::NCONV;
}

// ---------------------------------------------------------------------------------------------
// Workspace layout (floats), a pure function of (net, batch).
// ---------------------------------------------------------------------------------------------
struct WsLayout {
  // per conv layer: act = post-activation conv output (unpooled layers), pool = pooled output and
  // parg = its window argmax bytes (pooled layers: the conv epilogue pools, EpBiasActPool), dact =
  // the gradient of the conv output (pre-activation after masking; full resolution)
  size_t act[4], pool[4], parg[4], dact[4], fcslab, H, dz, dH, wslab, wslab2, total;
  size_t sync;  // the stacking chains' counters (nature_chain_kernel, stack_conv1_kernel; u32, zero between launches)
  int fc_splits;
};

template <int N, int BK>
struct TileFor {
  using T = Tile<64, 64, 2, 2, BK>;
};
// Thin-N conv tiles (COUT or CIN of 16 / 32): the 4 waves split M, one 16-row fragment each
// (128 / 256-row thin tiles measured slower). BK is capped so the A stage stays <= 96 KB.
constexpr int kThinBM = 64;
constexpr int thin_bk(int bk) { return kThinBM * (bk + 4) * 4 > 98304 && bk % 32 == 0 ? thin_bk(bk / 2) : bk; }
template <int BK>
struct TileFor<16, BK> {
  using T = Tile<kThinBM, 16, 4, 1, thin_bk(BK)>;
};
template <int BK>
struct TileFor<32, BK> {
  using T = Tile<kThinBM, 32, 4, 1, thin_bk(BK)>;
};

// K-chunk of a forward conv: the whole K when it fits 256, else the largest of 256/192/128
// dividing it (one fill per chunk, all loads of a chunk in flight together).
template <int K>
constexpr int conv_bk() {
  return K <= 256 ? ((K + 15) / 16) * 16 : (K % 256 == 0 ? 256 : (K % 192 == 0 ? 192 : 128));
}

template <class G>
using TileConvFwd = typename TileFor<G::COUT, conv_bk<G::KK>()>::T;
template <class G>
using TileConvWgrad = typename TileFor<G::COUT, 64>::T;
// dX: BK 64 = half the LDS of 128, twice the resident workgroups (LSTM conv2 dX -5 %, Pong conv2 dX -7 %);
// 32 for the 64-channel inputs (LSTM conv4 group 59.6 -> 56.1 us, NATURE conv3 39.6 -> 38.7; the thin
// CIN-32 tile is slower at 32: LSTM conv3 181.6 -> 190.8, profiles/r06dg)
template <class G>
using TileConvDgrad = typename TileFor<G::CIN, G::CIN >= 64 ? 32 : 64>::T;

using TileFc = Tile<32, 64, 2, 2, 64>;       // dense forward, M = batch (small), split-K
// dense dW (GEMM-K = batch: 160 = 2 chunks at ec=32) and dX (GEMM-K = F, M = batch): latency-bound
// at rollout batches, so small tiles — more workgroups, fewer MFMAs per wave (Pong: dense group
// 12.1 -> 10.6 us; LSTM dense dW 17.1 -> 13.1 us)
using TileDenseW = Tile<32, 64, 2, 2, 80>;
using TileDenseX = Tile<32, 32, 2, 2, 128>;

static int pick_splits(int grid_mn, int K, int bk, int target = 512) {
  int s = target / (grid_mn > 0 ? grid_mn : 1);
  if (s < 1) s = 1;
  const int chunks = cdiv(K, bk);
  if (s > chunks) s = chunks;
  return s;
}

// K splits of a conv weight gradient (GEMM-K = B*OH*OW, tiny M x N): enough that a block walks
// at most kWgradChunks BK-chunks (each chunk is one load latency: with only M x N / 1024 MFMA
// tiles per wave the chunk chain, not the MFMA, sets a block's time), capped so the partial slabs
// stay <= kSlabFloats.
// (4 K-chunks of 64 per block: re-checked against 1, 2, 8, 16 — DESIGN §8)
constexpr int kWgradChunks = 4;
constexpr size_t kSlabFloats = (size_t)4 << 20;
template <class G>
static int conv_wgrad_splits(int B) {
  using T = TileConvWgrad<G>;
  const int M = G::KK + 1;
  const int K = B * G::OH * G::OW;
  int s = std::max(pick_splits(cdiv(M, T::BM) * cdiv(G::COUT, T::BN), K, T::BK), cdiv(cdiv(K, T::BK), kWgradChunks));
  s = std::min<int>(s, (int)std::max<size_t>(kSlabFloats / ((size_t)M * G::COUT), 1));
  return gemm_splits<T>(K, s);
}

template <class G>
static size_t conv_wgrad_slab(int B) {
  const int s = conv_wgrad_splits<G>(B);
  const size_t generic = s > 1 ? (size_t)s * (G::KK + 1) * G::COUT : 0;
  if constexpr (dconv_wgrad<G>())  // direct weight gradient (dconv.h)
    return std::max(generic, dwgrad_slab_floats<G, false>(B));
  return generic;
}

template <class Ar>
static int fc_splits(int B, int F) {
  if constexpr (Ar::FC_ROWS > 0) return Ar::FC_SPLITS;  // row_fc_kernel's K-splits
  const int s = pick_splits(cdiv(B, TileFc::BM) * cdiv(F, TileFc::BN), Ar::FLAT, TileFc::BK, 128);
  return gemm_splits<TileFc>(Ar::FLAT, s);
}

// The dense layer's partial slabs [splits][B][F] of the inference forwards: the row-split kernel
// (trunk_fused.h row_fc_kernel: one slab per conv output row, one memory round trip per block)
// where the arch has FC_ROWS, else the split-K GEMM. advance: the replayed rollout graph's
// sequence bases (row_fc_kernel's block 0).
template <class Ar>
static int launch_fc(const float *flat, int B, const float *Wfc, float *slabs, int splits, hipStream_t s,
                     uint32_t *advance = nullptr, uint32_t advance_by = 0) {
  if constexpr (Ar::FC_ROWS > 0)
    return launch_row_fc<Ar::FLAT / Ar::FC_ROWS, Ar::FC_ROWS, Ar::F, Ar::FC_SPLITS>(flat, B, Wfc, slabs, s, advance,
                                                                                  advance_by);
  else
    return launch_gemm<TileFc>(LdRowMajor{flat, Ar::FLAT}, LdColMajor{Wfc, Ar::F, -1}, EpSlab{slabs, B, Ar::F}, B,
                               Ar::F, Ar::FLAT, splits, s);
}

template <class Ar, int I = 0>
static void ws_layers(WsLayout &L, size_t &off, int B, size_t &wslab) {
  if constexpr (I < Ar::NCONV) {
    using G = LayerG<Ar, I>;
    auto take = [&](size_t nf) {
      size_t o = off;
      off = align64(off + nf);
      return o;
    };
    const size_t a = (size_t)B * G::OH * G::OW * G::COUT;
    const size_t p = pooled<Ar, I>() ? (size_t)B * (G::OH / 2) * (G::OW / 2) * G::COUT : 0;
    L.act[I] = take(pooled<Ar, I>() ? 0 : a);
    L.dact[I] = take(a);
    L.pool[I] = take(p);
    L.parg[I] = take(p / 4);  // bytes (COUT % 4 == 0)
    wslab = std::max(wslab, conv_wgrad_slab<G>(B));
    ws_layers<Ar, I + 1>(L, off, B, wslab);
  }
}

struct LstmWs;
template <class Ar>
static WsLayout lstm_ws_layout(const mt_net *n, int B, LstmWs *X);  // lstm.h

template <class Ar>
static WsLayout ws_layout(const mt_net *n, int B) {
  if constexpr (Ar::LSTM) return lstm_ws_layout<Ar>(n, B, nullptr);
  WsLayout L{};
  size_t off = 0;
  auto take = [&](size_t nf) {
    size_t o = off;
    off = align64(off + nf);
    return o;
  };
  size_t wslab = 0;
  ws_layers<Ar>(L, off, B, wslab);
  if constexpr (nips_fused_bwd<Ar>())  // per-image conv1 slabs (wslab), per-pair conv2 slabs (wslab2)
    if (B <= kNipsFusedBwdMaxRows)
      wslab = std::max(wslab, std::max((size_t)B * NipsConvBwdJob::SLAB1, (size_t)((B + 1) / 2) * NipsConvBwdJob::SLAB2));
  L.fc_splits = fc_splits<Ar>(B, Ar::F);
  L.fcslab = take((size_t)std::max(L.fc_splits, Ar::FUSED_SLABS) * B * Ar::F);
  L.H = take((size_t)B * Ar::F);
  L.dz = take((size_t)B * n->O);
  L.dH = take((size_t)B * Ar::F);
  L.wslab = take(wslab);
  L.wslab2 = take(wslab);  // ping-pong slab regions of consecutive conv layers (trunk_backward)
  // the rollout chains' counters (nature_chain_kernel; stack_conv1_kernel), zero between launches
  L.sync = take(nature_stacking<Ar>() ? (size_t)kChainSyncWords * B
                                      : frame_stacking<Ar>() && !Ar::LSTM ? (size_t)stack_conv1_sync_words(B) : 0);
  L.total = off;
  return L;
}

// ---------------------------------------------------------------------------------------------
// Kernels: slab sum, heads forward, loss + heads backward, heads weight gradient.
// ---------------------------------------------------------------------------------------------
static int sum_slabs(const float *P, int S, size_t n, float *out, hipStream_t s) {
  return launch_group(s, SlabJob{P, S, n, out});
}

struct HeadParams {
  const float *Wc, *bc, *Wa, *ba, *Wr, *br;
  int A, R, F;
  int nq;  // f32x4 quads of the head region [Wc, end of the parameters): critic | actor | repetition
};

// The three head (weights, biases) pairs are the last variables of every layout (add_heads), each
// 64-float aligned, so [Wc, P + nparams) is one contiguous 256-B-aligned region.
static HeadParams head_params(const mt_net *n, const float *P) {
  HeadParams h;
  h.F = n->F;
  h.A = n->cfg.num_actions;
  h.R = n->cfg.num_reps;
  h.Wc = P + n->off_critic;
  h.bc = h.Wc + h.F;
  h.Wa = P + n->off_actor;
  h.ba = h.Wa + (size_t)h.F * h.A;
  h.Wr = P + n->off_rep;
  h.br = h.Wr + (size_t)h.F * h.R;
  h.nq = (int)((n->nparams - n->off_critic) / 4);
  return h;
}

// Head output o (0 = critic, 1..A = actor, 1+A.. = repetition) inside the head region staged in
// LDS (heads_row): offset of its weight for feature 0, the feature stride, and its bias.
__device__ __forceinline__ void head_col_lds(const HeadParams &hp, int o, int &base, int &stride, int &bias) {
  // selects only (no branches): o is wave-uniform, so these are a few scalar instructions
  const int oa = (int)(hp.Wa - hp.Wc), orr = (int)(hp.Wr - hp.Wc);
  const bool c = o == 0, a = o <= hp.A;
  const int k = a ? o - 1 : o - 1 - hp.A;  // column within the actor / repetition block
  const int w0 = a ? oa : orr, st = a ? hp.A : hp.R;
  base = c ? 0 : w0 + k;
  stride = c ? 1 : st;
  bias = c ? hp.F : w0 + hp.F * st + k;
}

// Softmax over n logits held in lanes [0, n) of one wave (x/temp, TF: exp(x-max)/sum).
__device__ __forceinline__ float wave_softmax(float x, int lane, int n) {
  const float xm = lane < n ? x : -INFINITY;
  const float mx = wave_max(xm);
  const float e = lane < n ? expf(x - mx) : 0.f;
  const float s = wave_sum(e);
  return e / s;
}

constexpr int kMaxHeads = 64;  // 1 + A + R <= 64
constexpr int kMaxScan = 1024;  // max t_max of the fused n-step scan (mt_returns_loss_backward)

// draw_index (common.h) over probabilities held in lanes [0, n): same order and rounding.
__device__ __forceinline__ int wave_draw(float p, int n, double u) {
  const double epsneg = 5.9604644775390625e-08;
  double cum = 0.0;
  int res = n - 1;
  for (int j = 0; j < n - 1; ++j) {
    const float pj = lane_f(p, j);  // (j is wave-uniform: a readlane, not an LDS-routed shuffle)
    cum += (double)(pj - (float)epsneg);
    if (res == n - 1 && u < cum) res = j;
  }
  return res;
}

// One workgroup per row b (NT / 64 waves: 4 for F <= 256, 8 for F <= 512):
//  1. h = act(sum_z slabs[z][b] + b_fc) — the split-K dense layer finished here
//     (networks.py:57-70); every thread owns F/NT features;
//  2. logits_o = [h, 1] . W_o for the 1+A+R head outputs (policy_v_network.py:22, :31, :47):
//     wave w takes outputs o = w, w + NW, ...; lanes split F and reduce with DPP;
//  3. wave 0: v = logit_0, pi = softmax(logits_A / temp), rep = softmax(logits_R / temp);
//  4. rollout path (smp.counters != null): wave 0 draws (a, r) for the row (A3, common.h).
// Latency is everything here (32 blocks at E = 32, on the macro-step's critical chain), so every
// global load is issued at the start, in the order it is needed — vmcnt retires loads in issue
// order, so a wait for the first ones never waits for the later: the draw counter, then the slab
// partials, then the dense bias, then the whole head region (every output's weights and bias) as
// coalesced 16-B loads, staged into LDS beside h — and the row's uniforms are hashed from the
// counter while the slabs are in flight. (Round 4: each wave used to load its outputs' weight
// columns straight from HBM, lane f reading W[f][o] at a stride of A or R floats: one wave
// instruction touched 16-40 cache lines, ~5,600 line requests per block for NATURE's 15 outputs
// against ~500 for the region; the GEMV phase of the NATURE heads took 1.9 us.)
constexpr int kHeadQ = 8;  // region quads per thread held in registers from the kernel start
__device__ uint64_t g_zero_u64 = 0;  // read in place of an absent draw counter / sequence base

template <int FT, int SB, int NT>
__device__ __forceinline__ void heads_row(int b, const float *__restrict__ slabs, int S, int B,
                                          const float *__restrict__ fc_b, int act, float alpha, const HeadParams &hp,
                                          float temp, float *__restrict__ H, float *__restrict__ v,
                                          float *__restrict__ pi, float *__restrict__ rep, const SampleArgs &smp,
                                          float *Ws) {
  __shared__ float hs[NT * FT];
  __shared__ float zs[64];
  const int F = hp.F, O = 1 + hp.A + hp.R;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int FMAX = NT * FT / 64;  // feature terms per lane of a column walk
  constexpr int NW = NT / 64;
  // every load below is unconditional (clamped addresses, zeros by select): a guarded load would
  // end its basic block with a wait for it
  // (1) the draw counter and the sequence base (the uniforms need them first)
  const uint64_t cnt = *(smp.counters ? smp.counters + b : &g_zero_u64);
  const uint32_t seq_base = *(smp.seq_base ? smp.seq_base : reinterpret_cast<const uint32_t *>(&g_zero_u64));
  // (2) the slab partials of the thread's features (S = 9 for the NIPS trunk: one batch)
  const size_t zs_stride = (size_t)B * F;
  float t[FT][SB];
#pragma unroll
  for (int fi = 0; fi < FT; ++fi) {
    const float *p = slabs + (size_t)b * F + min((int)threadIdx.x + NT * fi, F - 1);
#pragma unroll
    for (int u = 0; u < SB; ++u) t[fi][u] = p[(size_t)min(u, S - 1) * zs_stride];
  }
  // (3) dense bias, then the head region's first KQ * NT quads (F > 256 on 512 threads: 6, so the
  // whole region of an A = 18, R = 1 head set (Seaquest, 2,593 quads) is requested here — the
  // remainder loop below was a second global round trip, ~0.5 us)
  constexpr int KQ = NT == 512 ? 6 : kHeadQ;
  float fb[FT];
#pragma unroll
  for (int fi = 0; fi < FT; ++fi) fb[fi] = fc_b[min((int)threadIdx.x + NT * fi, F - 1)];
  const f32x4 *hsrc = reinterpret_cast<const f32x4 *>(hp.Wc);
  f32x4 wq[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) wq[q] = hsrc[min((int)threadIdx.x + NT * q, hp.nq - 1)];
  if (smp.advance && b == 0 && threadIdx.x == 0) {  // the replayed rollout's last reader has run
    smp.advance[0] += smp.advance_by;
    smp.advance[1] += smp.advance_by;
  }
  double ua = 0.0, ur = 0.0;
  if (w == 0) row_uniforms(smp.seed, b + smp.row0, cnt, &ua, &ur);
  // slab sum in slab order + bias + activation
#pragma unroll
  for (int fi = 0; fi < FT; ++fi) {
    const int f = threadIdx.x + NT * fi;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < SB; ++u)
      if (u < S) acc += t[fi][u];
    for (int z = SB; z < S; ++z) acc += slabs[(size_t)b * F + min(f, F - 1) + (size_t)z * zs_stride];  // (S > SB)
    const float h = act_fwd(acc + fb[fi], act, alpha);
    if (f < F) {
      hs[f] = h;
      H[(size_t)b * F + f] = h;
    }
  }
  // the head region into LDS (the rest of a region larger than KQ * NT quads loaded here)
  f32x4 *wdst = reinterpret_cast<f32x4 *>(Ws);
#pragma unroll
  for (int q = 0; q < KQ; ++q)
    if ((int)threadIdx.x + NT * q < hp.nq) wdst[threadIdx.x + NT * q] = wq[q];
  for (int i = threadIdx.x + NT * KQ; i < hp.nq; i += NT) wdst[i] = hsrc[i];
  __syncthreads();
  MT_PROBE_AT(2, b, 1);
  // logits: the same products and order as a column walk f = lane, lane + 64, ... then the bias.
  // (The wave index through readfirstlane and, for F a multiple of 64, a wave-uniform term count:
  // a per-lane guard made each term an exec-masked block with its own LDS round trip, and the
  // column loop a divergent one — ~0.45 us per column of a wave, probe build.)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int jn = F >> 6;
  if ((F & 63) == 0) {
    // The wave's features read once; outputs o and o + NW per pass, every operand of both columns
    // (and their biases) requested at once. Lane offsets by 24-bit multiplies and wave-uniform term
    // offsets (j clamped to the last real term): the per-term 32-bit multiplies were quarter-rate,
    // and the bias a dependent LDS round trip after the reduction (round 6: 1.8 us for Seaquest's
    // 20 outputs, probe build).
    float hv[FMAX];
#pragma unroll
    for (int j = 0; j < FMAX; ++j) hv[j] = hs[min(lane + 64 * j, NT * FT - 1)];
    for (int o0 = wu; o0 < O; o0 += 2 * NW) {
      const int o1 = o0 + NW < O ? o0 + NW : o0;
      int b0, s0, c0, b1, s1, c1;
      head_col_lds(hp, o0, b0, s0, c0);
      head_col_lds(hp, o1, b1, s1, c1);
      const int l0 = b0 + __mul24(lane, s0), l1 = b1 + __mul24(lane, s1);
      float w0[FMAX], w1[FMAX];
#pragma unroll
      for (int j = 0; j < FMAX; ++j) {
        const int jj = min(j, jn - 1);
        w0[j] = Ws[l0 + jj * 64 * s0];
        w1[j] = Ws[l1 + jj * 64 * s1];
      }
      const float bias0 = Ws[c0], bias1 = Ws[c1];
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int j = 0; j < FMAX; ++j)
        if (j < jn) {
          a0 += hv[j] * w0[j];
          a1 += hv[j] * w1[j];
        }
      a0 = wave_sum(a0);
      a1 = wave_sum(a1);
      if (lane == 0) {
        zs[o0] = a0 + bias0;
        if (o1 != o0) zs[o1] = a1 + bias1;
      }
    }
  } else {
    for (int o = wu; o < O; o += NW) {
      int base, stride, bias;
      head_col_lds(hp, o, base, stride, bias);
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < FMAX; ++j)
        if (lane + 64 * j < F) acc += hs[lane + 64 * j] * Ws[base + (lane + 64 * j) * stride];
      acc = wave_sum(acc);
      if (lane == 0) zs[o] = acc + Ws[bias];
    }
  }
  __syncthreads();
  MT_PROBE_AT(2, b, 2);
  if (w != 0) return;
  const float z = lane < O ? zs[lane] : 0.f;
  if (lane == 0) v[b] = z;
  // actor logits sit in lanes 1..A, repetition logits in lanes 1+A..A+R: shift them to 0..
  // (wave-uniform shortcuts with identical results for finite logits: x / 1 = x, and a one-way
  // softmax is exp(0) / 1 = 1 — the two IEEE divisions and the whole repetition softmax were a
  // third of this single wave's instructions for the non-FiGAR heads)
  float za = __shfl(z, (lane + 1) & 63, 64);
  float zr = __shfl(z, (lane + 1 + hp.A) & 63, 64);
  if (temp != 1.f) {
    za = za / temp;
    zr = zr / temp;
  }
  const float pa = wave_softmax(za, lane, hp.A);
  const float pr = hp.R == 1 ? (lane == 0 ? 1.f : 0.f) : wave_softmax(zr, lane, hp.R);
  if (lane < hp.A) pi[(size_t)b * hp.A + lane] = pa;
  if (lane < hp.R) rep[(size_t)b * hp.R + lane] = pr;
  if (smp.counters) {
    const int a = wave_draw(pa, hp.A, ua), r = wave_draw(pr, hp.R, ur);
    if (lane == 0) {
      const uint32_t seq = seq_base + smp.seq;  // (graph replay: device base)
      if (smp.packed) {  // tagged pair, one 8-byte store, no fence (SampleArgs::packed)
        const uint64_t tag = (uint64_t)(seq & 0xffffu) << 16;
        const uint64_t word = ((tag | (uint32_t)r) << 32) | tag | (uint32_t)a;
        __hip_atomic_store(smp.packed + b, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else if (smp.pair) {
        smp.pair[b] = a;
        smp.pair[B + b] = r;
      }
      smp.counters[b] = cnt + 1;
      smp.a_idx[b] = a;
      smp.r_idx[b] = r;
      if (smp.ready && !smp.packed) {  // release: the pair stores are visible to the host before the flag
        __threadfence_system();
        __hip_atomic_store(smp.ready + b, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

template <int FT, int SB, int NT>
__global__ __launch_bounds__(NT) void heads_fwd_kernel(const float *__restrict__ slabs, int S, int B,
                                                        const float *__restrict__ fc_b, int act,
                                                        float alpha, HeadParams hp, float temp,
                                                        float *__restrict__ H, float *__restrict__ v,
                                                        float *__restrict__ pi,
                                                        float *__restrict__ rep, SampleArgs smp) {
  extern __shared__ __attribute__((aligned(16))) float head_region[];
  MT_PROBE_AT(2, blockIdx.x, 0);
  heads_row<FT, SB, NT>(blockIdx.x, slabs, S, B, fc_b, act, alpha, hp, temp, H, v, pi, rep, smp, head_region);
  MT_PROBE_AT(2, blockIdx.x, 3);
}

// heads_fwd_kernel for F features (<= 512) and S slabs: one feature per thread (256 threads for
// F <= 256, 512 above: the GEMV is instruction-issue bound with one wave per SIMD, so 8 waves take
// fewer output passes each — round 6) and SB >= S slabs in registers (else one batch of 16).
static int launch_heads(int rows, hipStream_t s, const float *slabs, int S, int B, const float *fc_b, int act,
                        float alpha, const HeadParams &hp, float temp, float *H, float *v, float *pi, float *rep,
                        const SampleArgs &smp) {
  if (hp.F > 512 || 1 + hp.A + hp.R > kMaxHeads) {
    set_error("heads: F = %d > 512 or %d outputs > %d", hp.F, 1 + hp.A + hp.R, kMaxHeads);
    return MT_ERR_ARG;
  }
  // dynamic LDS: the head region (<= 64 outputs x 513 rows: 132 KB at most)
  const size_t lds = (size_t)hp.nq * 16;
  if (lds > 150 * 1024) {
    set_error("heads: head region of %zu bytes exceeds the LDS", lds);
    return MT_ERR_ARG;
  }
#define MT_HEADS(FT_, SB_, NT_)                                                                              \
  do {                                                                                                       \
    static bool attr_set = false;                                                                            \
    if (!attr_set && lds > 64 * 1024) {                                                                      \
      MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&heads_fwd_kernel<FT_, SB_, NT_>),           \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));                   \
      attr_set = true;                                                                                       \
    }                                                                                                        \
    hipLaunchKernelGGL((heads_fwd_kernel<FT_, SB_, NT_>), dim3(rows), dim3(NT_), lds, s, slabs, S, B, fc_b,    \
                       act, alpha, hp, temp, H, v, pi, rep, smp);                                            \
  } while (0)
  if (hp.F <= 256) {
    if (S <= 1) MT_HEADS(1, 1, 256);
    else if (S <= 9) MT_HEADS(1, 9, 256);
    else MT_HEADS(1, 16, 256);
  } else {
    if (S <= 1) MT_HEADS(1, 1, 512);
    else if (S <= 9) MT_HEADS(1, 9, 512);
    else MT_HEADS(1, 16, 512);
  }
#undef MT_HEADS
  MT_LAUNCHED();
  return MT_OK;
}

#ifdef MT_PROBE
extern "C" int mt_probe_read(unsigned long long *out, size_t n) {
  MT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mt_probe_buf), std::min(n, sizeof(mt_probe_buf) / 8) * 8));
  return MT_OK;
}
extern "C" int mt_probe_read_chain(unsigned long long *out, size_t n) {
  MT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mt_probe_chain), std::min(n, sizeof(mt_probe_chain) / 8) * 8));
  return MT_OK;
}
extern "C" int mt_probe_read_chain_blocks(unsigned long long *out, size_t n) {
  MT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mt_probe_chainblk), std::min(n, sizeof(mt_probe_chainblk) / 8) * 8));
  return MT_OK;
}
#endif


// dL/dlogit for one softmax head (policy_v_network.py:29-57, :59-74), one wave, lanes [0, n):
// objective = adv*log(p_sel + 1e-30) + beta*H,  H = -sum p*log(p + 1e-30),  L = -scale*objective.
// Chain rule exactly as TF differentiates it: g_k = dL/dp_k, dz_k = p_k (g_k - sum_j p_j g_j),
// dlogit_k = dz_k / temp. Returns lane's dlogit; *ent, *lsel receive H and log(p_sel+eps).
__device__ __forceinline__ float head_softmax_grad(float p, int lane, int n, int sel, float adv,
                                                   float beta, float scale, float temp, float *ent,
                                                   float *lsel) {
  const float eps = 1e-30f;
  const bool on = lane < n;
  const float pe = p + eps;
  const float lp = on ? logf(pe) : 0.f;
  const float e = wave_sum(on ? -(p * lp) : 0.f);
  *ent = e;
  *lsel = __shfl(lp, sel, 64);
  // d objective / dp_k = adv*[k==sel]/(p+eps) + beta * d(-sum p log(p+eps))/dp_k
  //                    = adv*[k==sel]/(p+eps) - beta*(log(p+eps) + p/(p+eps))
  float dobj = on ? ((lane == sel ? adv / pe : 0.f) - beta * (lp + p / pe)) : 0.f;
  const float g = -scale * dobj;
  const float sg = wave_sum(on ? p * g : 0.f);
  return on ? p * (g - sg) / temp : 0.f;
}

// One workgroup per row b: head gradients dz[b][0..O) and dH[b][f] = act'(H) * sum_o dz_o W[f][o].
// Optional n-step scan inside the loss kernel (mt_returns_loss_backward): row b = t*E + e.
struct ReturnsSrc {
  const float *r = nullptr, *mask = nullptr, *VT = nullptr;  // r / mask [T][E] (host-mapped ok)
  double gamma = 0.0;
  int T = 0, E = 0;
  float *y_out = nullptr, *adv_out = nullptr;
  // bootstrap from the rollout's last chain without its heads kernel (mt_returns_loss_backward_boot):
  // V(s_T)[e] = [act(sum_z boot_slabs[z][e] + fc_b), 1] . [Wc, bc] computed by the loss block
  // itself (VT unused), written to vt_out[e] by the blocks of step 0
  const float *boot_slabs = nullptr, *fc_b = nullptr;
  int boot_S = 0;
  float *vt_out = nullptr;
};

// V(s_T)[e] of the bootstrap (ReturnsSrc::boot_slabs): the dense layer's split-K slabs summed in
// slab order + bias + act (heads_row's phase 1), then the critic's dot product as heads_row forms
// it (lanes over features in 64-strides, DPP wave sum, + bias) from the head region in LDS (Ws).
// Called by the whole block; the result is in *vt (LDS) after the call. stage(): the caller's LDS
// stores of the head region, run after this block's slab loads are issued and before the barrier.
template <class Pre, class Stage>
__device__ __forceinline__ void boot_value(const ReturnsSrc &rs, const HeadParams &hp, int e, int act, float alpha,
                                           const float *Ws, float *hsb, float *vt, const Pre &pre, const Stage &stage) {
  const int F = hp.F;
  const size_t zs_stride = (size_t)rs.E * F;
  if (F <= 512 && rs.boot_S <= 16) {
    // every slab partial and dense bias of the thread's features requested first, THEN pre() (the
    // caller's pinned-memory reward loads): vector loads retire in issue order, so a PCIe load
    // issued ahead of these made the slab sum wait for it (round 5)
    float t[2][16], fb[2];
#pragma unroll
    for (int fi = 0; fi < 2; ++fi) {
      const int fc = min((int)threadIdx.x + 256 * fi, F - 1);
      const float *p = rs.boot_slabs + (size_t)e * F + fc;
#pragma unroll
      for (int u = 0; u < 16; ++u) t[fi][u] = p[(size_t)min(u, rs.boot_S - 1) * zs_stride];
      fb[fi] = rs.fc_b[fc];
    }
    pre();
#pragma unroll
    for (int fi = 0; fi < 2; ++fi) {
      const int f = threadIdx.x + 256 * fi;
      if (f < F) {
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (u < rs.boot_S) acc += t[fi][u];
        hsb[f] = act_fwd(acc + fb[fi], act, alpha);
      }
    }
  } else {
    pre();
    for (int f = threadIdx.x; f < F; f += 256) {
      const float *p = rs.boot_slabs + (size_t)e * F + f;
      float acc = 0.f;
      for (int z = 0; z < rs.boot_S; z += 16) {
        float t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) t[u] = p[(size_t)min(z + u, rs.boot_S - 1) * zs_stride];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (z + u < rs.boot_S) acc += t[u];
      }
      hsb[f] = act_fwd(acc + rs.fc_b[f], act, alpha);
    }
  }
  stage();
  __syncthreads();
  if (threadIdx.x < 64) {  // heads_row's critic column: same products, same order
    const int lane = threadIdx.x;
    float acc = 0.f;
    if ((F & 63) == 0) {
      const int jn = F >> 6;
      float hv[8], wv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        hv[j] = hsb[min(lane + 64 * j, 511)];
        wv[j] = Ws[min(lane + 64 * j, F - 1)];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < jn) acc += hv[j] * wv[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (lane + 64 * j < F) acc += hsb[lane + 64 * j] * Ws[lane + 64 * j];
    }
    acc = wave_sum(acc);
    if (lane == 0) *vt = acc + Ws[F];
  }
  __syncthreads();
}

// returns_kernel's arithmetic for row b = (t, e): R from T-1 down to t, bit-identical to
// mt_returns. Thread k < 256 brings step t + k's reward / mask in (rk, mk: requested by the caller
// before its other work, one round trip), the rest load here; thread 0 scans (vb = V[b], which it
// loaded with the head inputs). Called by the whole block.
__device__ __forceinline__ void row_return(const ReturnsSrc &rs, float vb, int b, float vt,
                                           float rk, float mk, float *ya, float *buf) {
#pragma clang fp contract(off)
  const int T = rs.T, E = rs.E;
  const int t = b / E, e = b - t * E, n = T - t;  // steps t .. T-1
  if ((int)threadIdx.x < n) {
    buf[2 * threadIdx.x] = rk;
    buf[2 * threadIdx.x + 1] = mk;
  }
  for (int k = threadIdx.x + 256; k < n; k += 256) {
    buf[2 * k] = rs.r[(size_t)(t + k) * E + e];
    buf[2 * k + 1] = rs.mask[(size_t)(t + k) * E + e];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float g32 = __fmul_rn((float)rs.gamma, vt);
    double R = (double)buf[2 * (n - 1)] + (double)g32 * (double)buf[2 * (n - 1) + 1];
    const double gd = rs.gamma;
    for (int k = n - 2; k >= 0; --k) R = (double)buf[2 * k] + (gd * R) * (double)buf[2 * k + 1];
    ya[0] = (float)R;
    ya[1] = (float)(R - (double)vb);
    rs.y_out[b] = ya[0];
    rs.adv_out[b] = ya[1];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void loss_bwd_kernel(
    HeadParams hp, const float *__restrict__ H, const float *__restrict__ pi,
    const float *__restrict__ rep, const float *__restrict__ v, const int32_t *__restrict__ a_idx,
    const int32_t *__restrict__ r_idx, const float *__restrict__ y, const float *__restrict__ adv,
    float beta, float scale, float temp, int act, float alpha, float *__restrict__ dz,
    float *__restrict__ dH, float *__restrict__ loss_terms, ReturnsSrc rs) {
  __shared__ float dzs[kMaxHeads];
  __shared__ float ya[2];
  __shared__ float buf[2 * kMaxScan];
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // the head region (HeadParams::nq quads)
  const int b = blockIdx.x;
  MT_PROBE_AT(4, b, 0);
  const int A = hp.A, R = hp.R, O = 1 + A + R, F = hp.F;
  // Every load that does not depend on the return is issued first, so its latency overlaps the
  // scan's (the rewards / masks are read over PCIe from pinned memory): the row's head inputs
  // (threads < 64), H[b][f] of the thread's features and the head region as coalesced 16-B loads
  // (staged into LDS for the critic's dot product and dH; round 4: per-thread loads of W[f][.] at a
  // stride of A or R floats made ~2,800 cache-line requests per block for NATURE's heads, queued
  // ahead of the bootstrap slab loads).
  const int lane = threadIdx.x;
  float pa = 0.f, pr = 0.f, vb = 0.f, adv_in = 0.f, y_in = 0.f;
  int ai = 0, ri = 0;
  if (threadIdx.x < 64) {
    pa = lane < A ? pi[(size_t)b * A + lane] : 0.f;
    pr = lane < R ? rep[(size_t)b * R + lane] : 0.f;
    vb = v[b];
    ai = a_idx[b];
    ri = r_idx[b];
    if (!rs.r) {
      adv_in = adv[b];
      y_in = y[b];
    }
  }
  constexpr int FT = 2;  // F <= 512 in registers (more: read at the end)
  float hv[FT];
#pragma unroll
  for (int fi = 0; fi < FT; ++fi) hv[fi] = H[(size_t)b * F + min((int)threadIdx.x + 256 * fi, F - 1)];
  const f32x4 *hsrc = reinterpret_cast<const f32x4 *>(hp.Wc);
  f32x4 wq[kHeadQ];
#pragma unroll
  for (int q = 0; q < kHeadQ; ++q) wq[q] = hsrc[min((int)threadIdx.x + 256 * q, hp.nq - 1)];
  auto stage = [&]() {
    f32x4 *wdst = reinterpret_cast<f32x4 *>(Ws);
#pragma unroll
    for (int q = 0; q < kHeadQ; ++q)
      if ((int)threadIdx.x + 256 * q < hp.nq) wdst[threadIdx.x + 256 * q] = wq[q];
    for (int i = threadIdx.x + 256 * kHeadQ; i < hp.nq; i += 256) wdst[i] = hsrc[i];
  };
  bool staged = false;
  if (rs.r) {
    // this row's rewards / masks (pinned host memory, a PCIe round trip): requested right behind the
    // bootstrap slab loads (boot_value's pre), whose sum would otherwise wait for them
    float rk = 0.f, mk = 0.f;
    auto rewards = [&]() {
      const int t = b / rs.E, e = b - t * rs.E;
      if ((int)threadIdx.x < rs.T - t) {
        rk = rs.r[(size_t)(t + threadIdx.x) * rs.E + e];
        mk = rs.mask[(size_t)(t + threadIdx.x) * rs.E + e];
      }
    };
    float vt;
    if (rs.boot_slabs) {
      __shared__ float hsb[512];
      __shared__ float vts;
      const int e = b % rs.E;
      boot_value(rs, hp, e, act, alpha, Ws, hsb, &vts, rewards, stage);
      staged = true;
      vt = vts;
      if (rs.vt_out && b < rs.E && threadIdx.x == 0) rs.vt_out[e] = vt;
    } else {
      rewards();
      vt = rs.VT[b % rs.E];
    }
    MT_PROBE_AT(4, b, 1);
    row_return(rs, vb, b, vt, rk, mk, ya, buf);
  }
  MT_PROBE_AT(4, b, 2);
  if (!staged) stage();  // (visible to every thread after the barrier below)
  if (threadIdx.x < 64) {
    const float ad = rs.r ? ya[1] : adv_in;
    const float yb = rs.r ? ya[0] : y_in;
    float ent_a, ls_a, ent_r, ls_r;
    const float ga = head_softmax_grad(pa, lane, A, ai, ad, beta, scale, temp, &ent_a, &ls_a);
    const float gr = head_softmax_grad(pr, lane, R, ri, ad, beta, scale, temp, &ent_r, &ls_r);
    const float diff = yb - vb;
    // d/dv of scale * 0.25 * (y - v)^2  (policy_v_network.py:25-26)
    const float gv = scale * 0.25f * 2.0f * (vb - yb);
    if (lane == 0) dzs[0] = gv;
    if (lane < A) dzs[1 + lane] = ga;
    if (lane < R) dzs[1 + A + lane] = gr;
    if (lane == 0 && loss_terms) {
      loss_terms[(size_t)b * 4 + 0] = 0.25f * diff * diff;
      loss_terms[(size_t)b * 4 + 1] = -((ls_a + ls_r) * ad);
      loss_terms[(size_t)b * 4 + 2] = ent_a;
      loss_terms[(size_t)b * 4 + 3] = ent_r;
    }
  }
  __syncthreads();
  MT_PROBE_AT(4, b, 3);
  for (int o = threadIdx.x; o < O; o += 256) dz[(size_t)b * O + o] = dzs[o];
  // dH[b][f] = act'(H) * (dz_c Wc[f] + actor terms + repetition terms), in that order
  const int oa = (int)(hp.Wa - hp.Wc), orr = (int)(hp.Wr - hp.Wc);
  auto dh = [&](int f, float h) {
    float acc = dzs[0] * Ws[f];
    for (int k = 0; k < A; ++k) acc += dzs[1 + k] * Ws[oa + f * A + k];
    for (int k = 0; k < R; ++k) acc += dzs[1 + A + k] * Ws[orr + f * R + k];
    dH[(size_t)b * F + f] = acc * act_bwd(h, act, alpha);
  };
#pragma unroll
  for (int fi = 0; fi < FT; ++fi)
    if ((int)threadIdx.x + 256 * fi < F) dh(threadIdx.x + 256 * fi, hv[fi]);
  for (int f = threadIdx.x + 256 * FT; f < F; f += 256) dh(f, H[(size_t)b * F + f]);  // (F > 512: not built today)
  MT_PROBE_AT(4, b, 4);
}

// Head weight/bias gradient: G[f][o] = sum_b [H,1][b][f] * dz[b][o], scattered into the three
// (w, b) variable pairs of the flat gradient. Block = (64 features, output o): column o of dz is
// staged in LDS, the 4 waves take contiguous quarters of the rows (H read coalesced: consecutive
// lanes = consecutive features, 4 independent accumulators per lane), and the 4 wave partials are
// added in wave order through LDS (deterministic).
__device__ __forceinline__ void head_wgrad_body(const float *__restrict__ H, const float *__restrict__ dz, int B,
                                                int F, int A, int R, float *__restrict__ gc, float *__restrict__ ga,
                                                float *__restrict__ gr, int bx, int o, float *dzs) {
  // dzs: [B] column o, then [4][64] partials
  const int O = 1 + A + R;
  for (int i = threadIdx.x; i < B; i += 256) dzs[i] = dz[(size_t)i * O + o];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = bx * 64 + lane;  // f == F is the bias row
  const int q = (B + 3) / 4, b0 = w * q, b1 = min(B, b0 + q);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (f <= F) {
    int b = b0;
    if (f < F) {
      // 16 rows' loads in flight per trip (a 4-row trip waited out one load latency per 4 rows);
      // accumulator u still takes rows b0 + u, b0 + 4 + u, ... in order
      for (; b + 15 < b1; b += 16) {
        float h[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) h[u] = H[(size_t)(b + u) * F + f];
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u & 3] += h[u] * dzs[b + u];
      }
      for (; b + 3 < b1; b += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] += H[(size_t)(b + u) * F + f] * dzs[b + u];
      }
      for (; b < b1; ++b) a[0] += H[(size_t)b * F + f] * dzs[b];
    } else {
      for (; b < b1; ++b) a[0] += dzs[b];
    }
  }
  float *part = dzs + B;
  part[w * 64 + lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w != 0 || f > F) return;
  const float acc = ((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane];
  if (o == 0)
    gc[f] = acc;  // [F][1] weights then the bias at index F
  else if (o <= A)
    ga[(size_t)f * A + (o - 1)] = acc;
  else
    gr[(size_t)f * R + (o - 1 - A)] = acc;
}

// The head weight gradient as a job of a grouped launch: block (f chunk of 64, output o).
struct HeadWgradJob {
  const float *H, *dz;
  int B, F, A, R;
  float *gc, *ga, *gr;
  __host__ __device__ int gx() const { return (F + 1 + 63) / 64; }
  __host__ __device__ int blocks() const { return gx() * (1 + A + R); }
  size_t lds() const { return sizeof(float) * ((size_t)B + 4 * 64); }
  __device__ __forceinline__ void run(int id, float *smem) const {
    head_wgrad_body(H, dz, B, F, A, R, gc, ga, gr, id % gx(), id / gx(), smem);
  }
};

// ---------------------------------------------------------------------------------------------
// Layer drivers
// ---------------------------------------------------------------------------------------------
template <class G, bool U8>
static int conv_forward(const void *X, const float *Wt, const float *bias, float *Y, int B, int act,
                        float alpha, hipStream_t s) {
  using T = TileConvFwd<G>;
  LdIm2col<G, U8> la{reinterpret_cast<const typename InElem<U8>::T *>(X)};
  LdColMajor lb{Wt, G::COUT, -1};
  EpBiasAct ep{Y, bias, G::COUT, act, alpha};
  const int M = B * G::OH * G::OW;
  if constexpr (G::COUT % 32 == 0) {
    // small batches (a rollout step): a grid of under two workgroups per CU leaves most CUs idle
    // and each wave a long MFMA chain — 32 x 32 tiles, one 16 x 16 accumulator per wave
    using TS = Tile<32, 32, 2, 2, conv_bk<G::KK>()>;
    if (cdiv(M, T::BM) * cdiv(G::COUT, T::BN) < 512) return launch_gemm<TS>(la, lb, ep, M, G::COUT, G::KK, 1, s);
  }
  return launch_gemm<T>(la, lb, ep, M, G::COUT, G::KK, 1, s);
}

// Conv + bias + activation + 2x2/2 max pool in one product (pool-ordered rows, EpBiasActPool):
// Y = the pooled output, arg = the window position of each maximum.
template <class G, bool U8>
static int conv_forward_pool(const void *X, const float *Wt, const float *bias, float *Y, uint8_t *arg, int B,
                             int act, float alpha, hipStream_t s) {
  using T = TileConvFwd<G>;
  LdIm2col<G, U8, true> la{reinterpret_cast<const typename InElem<U8>::T *>(X)};
  LdColMajor lb{Wt, G::COUT, -1};
  EpBiasActPool<G> ep{Y, arg, bias, act, alpha};
  const int M = B * (G::OH / 2) * (G::OW / 2) * 4;
  if constexpr (G::COUT % 32 == 0) {
    using TS = Tile<32, 32, 2, 2, conv_bk<G::KK>()>;
    if (cdiv(M, T::BM) * cdiv(G::COUT, T::BN) < 512) return launch_gemm<TS>(la, lb, ep, M, G::COUT, G::KK, 1, s);
  }
  return launch_gemm<T>(la, lb, ep, M, G::COUT, G::KK, 1, s);
}

// dW (+db) of a conv -> grad[(KK+1) x COUT] (weights then biases): dW = im2col(X)^T . dY as a GEMM
// job into K-split slabs [S][KK+1][COUT] (one split: straight into gwb) and the slab-sum job that
// finishes it (no job when unsplit). db: when KK fills whole M-tiles (NIPS / NATURE, PWYX conv3),
// the column sums of dY per split go to slab row KK (BiasRowJob) — a 64-row MFMA tile for the one
// bias row would add a fifth of the product's work; otherwise the bias is a ones-row of the same
// GEMM (LdIm2colT), free in the last tile's spare rows.
template <class G, bool U8>
struct WgradJobs {
  PairJob<GemmJob<TileConvWgrad<G>, LdIm2colT<G, U8>, LdColMajor, EpSlab>, BiasRowJob<G::COUT>> gemm;
  SlabJob sum;
};
template <class G, bool U8>
static WgradJobs<G, U8> conv_wgrad_jobs(const void *X, const float *dY, float *slab, float *gwb, int B) {
  using T = TileConvWgrad<G>;
  const int M = G::KK + 1, K = B * G::OH * G::OW;
  const int S = conv_wgrad_splits<G>(B);
  LdIm2colT<G, U8> la{reinterpret_cast<const typename InElem<U8>::T *>(X)};
  LdColMajor lb{dY, G::COUT, -1};
  float *dst = S == 1 ? gwb : slab;
  constexpr bool sep = G::KK % T::BM == 0;
  const auto g = gemm_job<T>(la, lb, EpSlab{dst, M, G::COUT}, sep ? G::KK : M, G::COUT, K, S);
  const BiasRowJob<G::COUT> bias{dY, dst + (size_t)G::KK * G::COUT, (size_t)M * G::COUT, K, g.kchunk,
                                 sep ? g.gz : 0};
  WgradJobs<G, U8> j{{g, bias}, SlabJob{}};
  if (g.gz > 1) j.sum = SlabJob{slab, g.gz, (size_t)M * G::COUT, gwb};
  return j;
}

// The weight-gradient jobs of conv layer G: the direct kernel for the stride-1 SAME layers
// (DWgradJob, dconv.h), the generic GEMM otherwise; same slab layout and SlabJob either way.
template <class G, bool U8>
struct DWgradJobs {
  DWJobFor<G, U8> gemm;
  SlabJob sum;
};
template <class G, bool U8>
static auto conv_wgrad_jobs_sel(const void *X, const float *dY, float *slab, float *gwb, int B) {
  if constexpr (dconv_wgrad<G>()) {
    using J = DWJobFor<G, U8>;
    const int S = dwgrad_splits<G, U8>(B);
    return DWgradJobs<G, U8>{J{reinterpret_cast<const typename J::InT *>(X), dY, slab, B, S},
                             SlabJob{slab, B > 0 ? S : 0, J::D::SLAB, gwb}};
  } else {
    return conv_wgrad_jobs<G, U8>(X, dY, slab, gwb, B);
  }
}

// dX of a conv (transposed-conv gather), masked by the activation derivative of X, as a GEMM job.
template <class G>
static auto conv_dgrad_job(const float *dY, const float *Wt, const float *Xact, float *dX, int B, int act,
                           float alpha) {
  using T = TileConvDgrad<G>;
  if constexpr (PhaseGeom<G>::OK) {  // stride phases: K / (S*S), no multiplications by holes
    constexpr int S2 = G::S * G::S;
    const int mp = cdiv(B * PhaseGeom<G>::HQ * PhaseGeom<G>::WQ, T::BM) * T::BM;
    return gemm_job<T>(LdConvBwdAPhase<G>{dY, mp, B}, LdConvBwdBPhase<G>{Wt, mp / T::BM},
                       EpMaskedPhase<G>{dX, Xact, mp, B, act, alpha}, S2 * mp, G::CIN, PhaseGeom<G>::KP, 1);
  } else {
    return gemm_job<T>(LdConvBwdA<G>{dY}, LdConvBwdB<G>{Wt}, EpMasked{dX, Xact, G::CIN, act, alpha},
                       B * G::H * G::W, G::CIN, G::KH * G::KW * G::COUT, 1);
  }
}

// dX of a stride-1 conv whose input is the pooled output of conv GJ: the MaxPoolGrad routing and
// the activation mask run in the epilogue (EpMaskedUnpool), straight into GJ's full-res gradient.
template <class G, class GJ>
static auto conv_dgrad_unpool_job(const float *dY, const float *Wt, const float *Pj, const uint8_t *argj,
                                  float *dactj, int B, int act, float alpha) {
  using T = TileConvDgrad<G>;
  static_assert(!PhaseGeom<G>::OK, "pooled inputs feed stride-1 convs (networks.py:206-225)");
  return gemm_job<T>(LdConvBwdA<G>{dY}, LdConvBwdB<G>{Wt}, EpMaskedUnpool<GJ>{dactj, Pj, argj, act, alpha},
                     B * G::H * G::W, G::CIN, G::KH * G::KW * G::COUT, 1);
}

#define MT_TRY(x)              \
  do {                         \
    int rc_ = (x);             \
    if (rc_ != MT_OK) return rc_; \
  } while (0)

template <class Ar, int I>
static const float *layer_out(float *ws, const WsLayout &L) {
  return ws + (pooled<Ar, I>() ? L.pool[I] : L.act[I]);
}

// The layered trunk with the rollout chain's extras: st = the stacking source of conv1 (x = st->out;
// the NATURE gray chain: nature_chain_kernel; the frame trunks: stack_conv1_kernel, then conv2 ..
// layered), sync = the counters it uses (zero between launches).
struct FwdExtras {
  const StackSrc *st = nullptr;
  uint32_t *sync = nullptr;
};

template <class Ar, int I = 0>
static int trunk_forward(const mt_net *n, const float *P, const void *x, int B, float *ws,
                         const WsLayout &L, hipStream_t s, const FwdExtras &ex = FwdExtras{}) {
  if constexpr (I < Ar::NCONV) {
    using G = LayerG<Ar, I>;
    const float *W = P + n->off_conv[I];
    if (I == 0 && ex.st && !nature_stacking<Ar>() && !frame_stacking<Ar>()) {
      set_error("the stacking conv1 is built for the NIPS, the gray NATURE and the frame (PWYX / LSTM) trunks");
      return MT_ERR_UNSUPPORTED;
    }
    if constexpr (I == 0 && frame_stacking<Ar>()) {
      if (ex.st) {  // the rollout step: pull + stack + conv1 as one dataflow launch, then conv2 ..
        if (!ex.sync || x != ex.st->out) {
          set_error("stacking conv1: the input must be the new state rows, with a counter region");
          return MT_ERR_ARG;
        }
        MT_TRY((launch_stack_conv1<G>(*ex.st, W, ws + L.pool[0], (uint8_t *)(ws + L.parg[0]), B, n->cfg.activation,
                                      n->cfg.alpha_leaky, ex.sync, s)));
        return trunk_forward<Ar, 1>(n, P, layer_out<Ar, 0>(ws, L), B, ws, L, s);
      }
    }
    if constexpr (I == 0 && nature_stacking<Ar>()) {
      if (ex.st) {  // the rollout chain: stacking conv1 -> conv2 -> conv3 as one dataflow launch
        if (!ex.sync) {
          set_error("nature chain: no counter region");
          return MT_ERR_ARG;
        }
        return launch_nature_chain<LayerG<Ar, 0>, LayerG<Ar, 1>, LayerG<Ar, 2>>(
            *ex.st, W, P + n->off_conv[1], P + n->off_conv[2], ws + L.act[0], ws + L.act[1], ws + L.act[2], B,
            n->cfg.activation, n->cfg.alpha_leaky, ex.sync, s);
      }
    }
    // PWYX / LSTM frame trunk (stride-1 SAME) and NATURE (strided VALID): direct conv, patch in LDS (dconv.h)
    // (the RGB NATURE conv1's 768-deep K with its 24-row patch exceeds the LDS: generic)
    if constexpr ((G::S == 1 && G::SAME) || (Ar::NCONV == 3 && !G::SAME && G::CIN != 12))
      MT_TRY((conv_forward_direct<G, I == 0, pooled<Ar, I>()>(
          x, W, W + G::KK * G::COUT, ws + (pooled<Ar, I>() ? L.pool[I] : L.act[I]),
          pooled<Ar, I>() ? (uint8_t *)(ws + L.parg[I]) : nullptr, B, n->cfg.activation, n->cfg.alpha_leaky, s)));
    else if constexpr (pooled<Ar, I>())
      MT_TRY((conv_forward_pool<G, I == 0>(x, W, W + G::KK * G::COUT, ws + L.pool[I], (uint8_t *)(ws + L.parg[I]), B,
                                           n->cfg.activation, n->cfg.alpha_leaky, s)));
    else
      MT_TRY((conv_forward<G, I == 0>(x, W, W + G::KK * G::COUT, ws + L.act[I], B, n->cfg.activation,
                                      n->cfg.alpha_leaky, s)));
    return trunk_forward<Ar, I + 1>(n, P, layer_out<Ar, I>(ws, L), B, ws, L, s, ex);
  }
  return MT_OK;
}

// Conv layers I .. 0 of the backward, top down: one grouped launch per layer — its dX (the
// critical path, first), its dW GEMM and `pending` (the slab sum of layer I+1's dW) — then
// conv1's slab sum. Layer I's slabs live in region I % 2 (wslab / wslab2), so the slab sum of
// layer I+1 reads the other region while layer I's dW GEMM writes its own. `extra` (the LSTM's
// small cell / fc6 weight gradients: a few blocks, each a serial K walk) leads the top layer's
// grid, so its blocks start before the wide products fill the CUs instead of trailing them.
// Optional global-norm partials of the whole gradient written by the backward's last launch
// (world == 1: no all-reduce between the backward and the clip, so mt_grad_sumsq is not needed).
struct NormOut {
  float *partials = nullptr;  // [MT_NORM_PARTIALS]
  size_t n = 0;               // gradient floats
};

template <class Ar, int I, class X = NoJob>
static int trunk_backward(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                          const WsLayout &L, float *grad, hipStream_t s, SlabJob pending = SlabJob{},
                          const NormOut &no = NormOut{}, const X &extra = X{}) {
  using G = LayerG<Ar, I>;
  const int act = n->cfg.activation;
  const float al = n->cfg.alpha_leaky;
  const void *x = I == 0 ? (const void *)obs : (const void *)layer_out<Ar, (I > 0 ? I - 1 : 0)>(ws, L);
  if ((size_t)B * G::H * G::W * G::CIN >= ((size_t)1 << 31)) {  // LdIm2colT's 32-bit pixel offsets
    set_error("batch %d too large for the conv %d weight gradient", B, I);
    return MT_ERR_ARG;
  }
  if ((size_t)B * G::OH * G::OW * G::COUT * 4 >= ((size_t)1 << 31) - 16) {  // LdConvBwdA's 32-bit byte offsets
    set_error("batch %d too large for the conv %d input gradient", B, I);
    return MT_ERR_ARG;
  }
  const auto wg = conv_wgrad_jobs_sel<G, I == 0>(x, ws + L.dact[I], ws + (I % 2 ? L.wslab2 : L.wslab),
                                             grad + n->off_conv[I], B);
  if constexpr (I > 0) {
    constexpr int J = I - 1;
    using GJ = LayerG<Ar, J>;
    if constexpr (pooled<Ar, J>() && G::S == 1 && G::SAME && dconv_bwd_solo<G>()) {  // direct dX launch, then dW
      MT_TRY((conv_dgrad_unpool_solo<G, GJ>(ws + L.dact[I], P + n->off_conv[I], ws + L.pool[J],
                                           (const uint8_t *)(ws + L.parg[J]), ws + L.dact[J], B, act, al, s)));
      MT_TRY(launch_group(s, extra, wg.gemm, pending));
    } else if constexpr (stream_dx<G>()) {  // NATURE conv2: the weight-stationary streaming dX (nature_bwd.h)
      MT_TRY(launch_group(s, extra, DxStreamJob<G>{ws + L.dact[I], P + n->off_conv[I], ws + L.act[J], ws + L.dact[J], B,
                                            dx_stream_groups<G>(B), act, al},
                          wg.gemm, pending));
    } else if constexpr (pooled<Ar, J>()) {
      MT_TRY(launch_group(s, extra, conv_dgrad_unpool_job<G, GJ>(ws + L.dact[I], P + n->off_conv[I], ws + L.pool[J],
                                                           (const uint8_t *)(ws + L.parg[J]), ws + L.dact[J], B, act,
                                                           al),
                          wg.gemm, pending));
    } else {
      MT_TRY(launch_group(s, extra, conv_dgrad_job<G>(ws + L.dact[I], P + n->off_conv[I], ws + L.act[J], ws + L.dact[J], B,
                                               act, al),
                          wg.gemm, pending));
    }
    return trunk_backward<Ar, J>(n, P, obs, B, ws, L, grad, s, wg.sum, no);
  } else {
    MT_TRY(launch_group(s, extra, wg.gemm, pending));
    SlabJob last = wg.sum;
    if (no.partials && last.blocks() <= MT_NORM_PARTIALS / 2) {
      // conv1's slab sum writes the norm partials of its region, the rest of the gradient (complete
      // since the previous launches) is summed beside it: partials [0, slab blocks) + the rest
      last.sq = no.partials;
      const size_t b0 = n->off_conv[0], b1 = b0 + last.n;
      SumsqJob rest{grad, no.n, last.blocks() ? b0 : 0, last.blocks() ? b1 : 0, no.partials + last.blocks(),
                    MT_NORM_PARTIALS - last.blocks()};
      return launch_group(s, last, rest);
    }
    MT_TRY(launch_group(s, last));
    if (no.partials)  // (no room for the fused form: all partials from the complete gradient)
      return launch_group(s, SumsqJob{grad, no.n, 0, 0, no.partials, MT_NORM_PARTIALS});
    return MT_OK;
  }
}

// NIPS gray conv backward (nips_bwd.h): the per-image job, then the image-order slab sums of both
// layers (conv1's in region wslab, conv2's in wslab2) with the global-norm partials of the whole
// gradient when asked (the rest of the gradient, complete since the dense launch, beside them).
template <class Ar>
static int nips_conv_backward(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                              const WsLayout &L, float *grad, hipStream_t s, const NormOut &no) {
  using J = NipsConvBwdJob;
  static_assert(LayerG<Ar, 0>::KK + 1 == 257 && LayerG<Ar, 1>::KK + 1 == 257, "slab rows");
  float *slab1 = ws + L.wslab, *slab2 = ws + L.wslab2;
  MT_TRY(launch_nips_conv_bwd(s, J{obs, ws + L.act[0], ws + L.dact[1], P + n->off_conv[1], ws + L.dact[0], slab1,
                                   slab2, B, n->cfg.activation, n->cfg.alpha_leaky}));
  SlabJob s1{slab1, B, (size_t)J::SLAB1, grad + n->off_conv[0]};
  SlabJob s2{slab2, (B + 1) / 2, (size_t)J::SLAB2, grad + n->off_conv[1]};  // (per image pair)
  if (!no.partials) return launch_group(s, s1, s2);
  s1.sq = no.partials;
  s2.sq = no.partials + s1.blocks();
  const int used = s1.blocks() + s2.blocks();
  static_assert(MT_NORM_PARTIALS >= 2 * ((257 * 16 / 4 + kSlabCols - 1) / kSlabCols + (257 * 32 / 4 + kSlabCols - 1) / kSlabCols),
                "norm partials");
  // (the alignment padding between the two regions is zero in both the gradient and the skip)
  return launch_group(s, s1, s2,
                      SumsqJob{grad, no.n, n->off_conv[0], n->off_conv[1] + s2.n, no.partials + used,
                               MT_NORM_PARTIALS - used});
}

// Per-row conv buffers of a layout moved to start at row `row0` (the dense/head buffers stay).
template <class Ar, int I = 0>
static void shift_rows(WsLayout &L, size_t row0) {
  if constexpr (I < Ar::NCONV) {
    using G = LayerG<Ar, I>;
    const size_t a = row0 * G::OH * G::OW * G::COUT;
    L.act[I] += a;
    L.dact[I] += a;
    if constexpr (pooled<Ar, I>()) {
      const size_t p = row0 * (G::OH / 2) * (G::OW / 2) * G::COUT;
      L.pool[I] += p;
      L.parg[I] += p / 4;
    }
    shift_rows<Ar, I + 1>(L, row0);
  }
}

// Where a forward of B rows leaves its activations: its own workspace, or rows [row0, row0+B)
// of a train workspace (tr): conv buffers through a shifted layout, H at row0.
struct ActRows {
  float *base;
  WsLayout L;
  size_t h_off;  // float offset of row 0's H from base
};
template <class Ar>
static ActRows act_rows(const mt_net *n, float *ws, const WsLayout &L, const TrainRows *tr) {
  if (!tr) return ActRows{ws, L, L.H};
  ActRows a{tr->ws, ws_layout<Ar>(n, tr->rows), 0};
  a.h_off = a.L.H + (size_t)tr->row0 * Ar::F;
  shift_rows<Ar>(a.L, (size_t)tr->row0);
  return a;
}

template <class Ar>
static int forward_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                        float *v, float *pi, float *rep, const SampleArgs *smp, hipStream_t s,
                        const TrainRows *tr = nullptr, const hipEvent_t *marks = nullptr,
                        const StackSrc *st = nullptr) {
  const WsLayout L = ws_layout<Ar>(n, B);
  const ActRows A = act_rows<Ar>(n, ws, L, tr);
  if (marks) MT_HIP(hipEventRecord(marks[0], s));
  FwdExtras ex;
  ex.st = st;
  ex.sync = reinterpret_cast<uint32_t *>(ws + L.sync);
  MT_TRY((trunk_forward<Ar>(n, P, obs, B, A.base, A.L, s, ex)));
  const float *flat = layer_out<Ar, Ar::NCONV - 1>(A.base, A.L);
  // dense layer (networks.py:57-70), split-K partial slabs; heads kernel finishes bias + act.
  const float *Wfc = P + n->off_fc;
  MT_TRY((launch_fc<Ar>(flat, B, Wfc, ws + L.fcslab, L.fc_splits, s)));
  if (marks) MT_HIP(hipEventRecord(marks[1], s));
  HeadParams hp = head_params(n, P);
  return launch_heads(B, s, ws + L.fcslab, L.fc_splits, B, Wfc + (size_t)Ar::FLAT * Ar::F, n->cfg.activation,
                      n->cfg.alpha_leaky, hp, n->cfg.softmax_temp, A.base + A.h_off, v, pi, rep,
                      smp ? *smp : SampleArgs{});
}

// Inference forward (rollout steps, bootstrap): the NIPS trunk kernels where the arch has them
// (trunk_fused.h: conv -> act2, fc -> 9 slabs), whose slabs heads_fwd_kernel finishes; else the
// layered forward. st (NIPS only): stack the new state in the conv kernel (mt_rollout_step).
template <class Ar>
static int forward_infer_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                              float *v, float *pi, float *rep, const SampleArgs *smp, hipStream_t s,
                              const TrainRows *tr = nullptr, const StackSrc *st = nullptr,
                              const hipEvent_t *marks = nullptr) {
  if constexpr (Ar::FUSED_SLABS > 0) {
    constexpr int C = LayerG<Ar, 0>::CIN;
    using Fz = FusedNips<C>;
    const WsLayout L = ws_layout<Ar>(n, B);
    const ActRows A = act_rows<Ar>(n, ws, L, tr);
    const float *Wfc = P + n->off_fc;
    if (marks) MT_HIP(hipEventRecord(marks[0], s));
    MT_TRY((launch_nips_trunk<C>(obs, st, B, P + n->off_conv[0], P + n->off_conv[1], Wfc, n->cfg.activation,
                                 n->cfg.alpha_leaky, A.base + A.L.act[1], tr ? A.base + A.L.act[0] : nullptr,
                                 ws + L.fcslab, s)));
    MT_LAUNCHED();
    if (marks) MT_HIP(hipEventRecord(marks[1], s));
    HeadParams hp = head_params(n, P);
    return launch_heads(B, s, ws + L.fcslab, Fz::FC_SPLITS, B, Wfc + (size_t)Ar::FLAT * Ar::F, n->cfg.activation,
                        n->cfg.alpha_leaky, hp, n->cfg.softmax_temp, A.base + A.h_off, v, pi, rep,
                        smp ? *smp : SampleArgs{});
  } else {
    // (NATURE gray: conv1 stacks, trunk_forward refuses st for the other archs)
    return forward_impl<Ar>(n, P, obs, B, ws, v, pi, rep, smp, s, tr, marks, st);
  }
}

// Bootstrap forward without its heads (mt_rollout's last chain with MT_ROLLOUT_BOOT_SLABS): the
// trunk + the dense layer's split-K slabs left in ws (ws_layout(B).fcslab; NIPS: the fused trunk's
// FC_SPLITS slabs, else fc_splits), whose sum, bias, act and critic the update's loss kernel takes
// (mt_returns_loss_backward_boot). st: the NIPS stacking source; advance: the replayed rollout's
// sequence bases (the fused dense kernel advances them).
template <class Ar>
static int forward_boot_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws, hipStream_t s,
                             const StackSrc *st, uint32_t *advance, uint32_t advance_by) {
  const WsLayout L = ws_layout<Ar>(n, B);
  const float *Wfc = P + n->off_fc;
  if constexpr (Ar::FUSED_SLABS > 0) {
    constexpr int C = LayerG<Ar, 0>::CIN;
    return launch_nips_trunk<C>(obs, st, B, P + n->off_conv[0], P + n->off_conv[1], Wfc, n->cfg.activation,
                                n->cfg.alpha_leaky, ws + L.act[1], nullptr, ws + L.fcslab, s, advance, advance_by);
  } else {
    if (advance && Ar::FC_ROWS == 0) {  // (refused before anything is enqueued)
      set_error("sequence-base advance: row-split dense layers only");
      return MT_ERR_UNSUPPORTED;
    }
    FwdExtras ex;
    ex.st = st;
    ex.sync = reinterpret_cast<uint32_t *>(ws + L.sync);
    MT_TRY((trunk_forward<Ar>(n, P, obs, B, ws, L, s, ex)));
    return launch_fc<Ar>(layer_out<Ar, Ar::NCONV - 1>(ws, L), B, Wfc, ws + L.fcslab, L.fc_splits, s, advance,
                         advance_by);
  }
}

// Loss + head gradients (policy_v_network.py:25-74): writes dz, dH (masked by the trunk output's
// activation derivative) and the three head (w, b) gradients. Every variable's gradient is
// overwritten by the backward (no accumulation), so grad is not cleared: its alignment padding
// must be zero once (include/manette_hip.h, mt_loss_backward).
template <class Ar>
static int loss_bwd_launch(const mt_net *n, const float *P, int B, float *ws, const WsLayout &L, const float *pi,
                           const float *rep, const float *v, const int32_t *a_idx, const int32_t *r_idx,
                           const float *y, const float *adv, float beta, float *loss_terms, hipStream_t s,
                           const ReturnsSrc &rs = ReturnsSrc{}) {
  // loss scaling 5.0 and the batch mean (policy_v_network.py:70-74): scale = 5/B.
  const float scale = 5.0f / (float)B;
  HeadParams hp = head_params(n, P);
  if (!launch_allowed()) return MT_OK;
  const size_t lds = (size_t)hp.nq * 16;  // the head region (heads kernel: same bound)
  if (lds > 150 * 1024) {
    set_error("loss: head region of %zu bytes exceeds the LDS", lds);
    return MT_ERR_ARG;
  }
  static bool attr_set = false;
  if (!attr_set && lds > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&loss_bwd_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    attr_set = true;
  }
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(B), dim3(256), lds, s, hp, ws + L.H, pi, rep, v, a_idx, r_idx, y, adv,
                     beta, scale, n->cfg.softmax_temp, n->cfg.activation, n->cfg.alpha_leaky, ws + L.dz, ws + L.dH,
                     loss_terms, rs);
  MT_LAUNCHED();
  return MT_OK;
}

template <class Ar>
static HeadWgradJob head_wgrad_job(const mt_net *n, int B, float *ws, const WsLayout &L, float *grad) {
  return HeadWgradJob{ws + L.H, ws + L.dz, B, Ar::F, n->cfg.num_actions, n->cfg.num_reps,
                      grad + n->off_critic, grad + n->off_actor, grad + n->off_rep};
}

template <class Ar>
static int heads_backward(const mt_net *n, const float *P, int B, float *ws, const WsLayout &L, const float *pi,
                          const float *rep, const float *v, const int32_t *a_idx, const int32_t *r_idx,
                          const float *y, const float *adv, float beta, float *grad, float *loss_terms,
                          hipStream_t s) {
  if (sizeof(float) * ((size_t)B + 4 * 64) > 160 * 1024) {
    set_error("batch %d exceeds the head-gradient LDS stage", B);
    return MT_ERR_ARG;
  }
  MT_TRY(loss_bwd_launch<Ar>(n, P, B, ws, L, pi, rep, v, a_idx, r_idx, y, adv, beta, loss_terms, s));
  return launch_group(s, head_wgrad_job<Ar>(n, B, ws, L, grad));
}

// Launches of backward_impl up to the one that completes every dense / head gradient: the loss
// kernel, then [dense dX + dense dW + head dW] — the data-parallel split of the update
// (mt_net_backward_bucket_launches; checked at run time by backward_impl under a launch window).
constexpr int kDenseBucketLaunches = 2;

// Backward of the non-LSTM archs as grouped launches (gemm.h, launch_group): each launch runs
// every product whose inputs the previous one completed — loss | dense dX + dense dW + head dW |
// per conv layer I (top down): conv dX + conv dW + the slab sum of layer I+1's dW | conv1's slab
// sum — 2 + NCONV launches (the max pools are fused into the conv products) instead of two or three per layer.
template <class Ar>
static int backward_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws,
                         const float *pi, const float *rep, const float *v, const int32_t *a_idx,
                         const int32_t *r_idx, const float *y, const float *adv, float beta,
                         float *grad, float *loss_terms, hipStream_t s, const ReturnsSrc &rs = ReturnsSrc{},
                         const NormOut &no = NormOut{}) {
  const WsLayout L = ws_layout<Ar>(n, B);
  const int act = n->cfg.activation;
  const float al = n->cfg.alpha_leaky;
  if (sizeof(float) * ((size_t)B + 4 * 64) > 160 * 1024) {
    set_error("batch %d exceeds the head-gradient LDS stage", B);
    return MT_ERR_ARG;
  }
  MT_TRY(loss_bwd_launch<Ar>(n, P, B, ws, L, pi, rep, v, a_idx, r_idx, y, adv, beta, loss_terms, s, rs));
  constexpr int K = Ar::NCONV - 1;
  const float *flat = layer_out<Ar, K>(ws, L);
  const float *Wfc = P + n->off_fc;
  // dense dW, db: [flat, 1]^T . dH -> grad[(FLAT+1) x F]
  const auto dw = gemm_job<TileDenseW>(LdColMajor{flat, Ar::FLAT, Ar::FLAT}, LdColMajor{ws + L.dH, Ar::F, -1},
                                       EpStore{grad + n->off_fc, Ar::F}, Ar::FLAT + 1, Ar::F, B, 1);
  const HeadWgradJob hw = head_wgrad_job<Ar>(n, B, ws, L, grad);
  // dense dX: dH . W^T, masked by the last conv's activation (every trunk ends in an unpooled conv)
  static_assert(!pooled<Ar, K>(), "the trunk ends in an unpooled conv (networks.py:178-278)");
  const auto dx = gemm_job<TileDenseX>(LdRowMajor{ws + L.dH, Ar::F}, LdRowMajor{Wfc, Ar::F},
                                       EpMasked{ws + L.dact[K], flat, Ar::FLAT, act, al}, B, Ar::FLAT, Ar::F, 1);
  MT_TRY(launch_group(s, dx, dw, hw));
  // the data-parallel split point: every dense / head gradient is complete after this launch
  // (mt_net_backward_bucket_launches; paac._bucketed_update all-reduces that bucket next)
  if (g_win_on && g_win_index != kDenseBucketLaunches) {
    set_error("backward: the dense / head gradients completed after launch %d, not %d", g_win_index,
              kDenseBucketLaunches);
    return MT_ERR_UNSUPPORTED;
  }
  if constexpr (nips_fused_bwd<Ar>())
    if (B <= kNipsFusedBwdMaxRows) return nips_conv_backward<Ar>(n, P, obs, B, ws, L, grad, s, no);
  return trunk_backward<Ar, K>(n, P, obs, B, ws, L, grad, s, SlabJob{}, no);
}

}  // namespace mt

#include "lstm.h"

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
using namespace mt;

#define MT_ARCH_SWITCH(net, ...)                                                   \
  do {                                                                              \
    const int arch_ = (net)->cfg.arch, d_ = (net)->cfg.depth;                       \
    if (arch_ == MT_ARCH_NIPS && d_ == 1) { using Ar = NipsArch<4>; __VA_ARGS__; }         \
    else if (arch_ == MT_ARCH_NIPS && d_ == 3) { using Ar = NipsArch<12>; __VA_ARGS__; }   \
    else if (arch_ == MT_ARCH_NATURE && d_ == 1) { using Ar = NatureArch<4>; __VA_ARGS__; } \
    else if (arch_ == MT_ARCH_NATURE && d_ == 3) { using Ar = NatureArch<12>; __VA_ARGS__; } \
    else if (arch_ == MT_ARCH_PWYX && d_ == 1) { using Ar = PwyxArch<4>; __VA_ARGS__; }     \
    else if (arch_ == MT_ARCH_PWYX && d_ == 3) { using Ar = PwyxArch<12>; __VA_ARGS__; }    \
    else if (arch_ == MT_ARCH_LSTM && d_ == 1) { using Ar = LstmArch<4>; __VA_ARGS__; }     \
    else if (arch_ == MT_ARCH_LSTM && d_ == 3) { using Ar = LstmArch<12>; __VA_ARGS__; }    \
    else { set_error("arch %d depth %d not built", arch_, d_); return MT_ERR_UNSUPPORTED; } \
  } while (0)

extern "C" int mt_net_create(const mt_net_config *cfg, mt_net **out) {
  MT_CHECK_ARG(cfg && out, "null argument");
  MT_CHECK_ARG(cfg->depth == 1 || cfg->depth == 3, "depth must be 1 or 3");
  MT_CHECK_ARG(cfg->num_actions >= 1 && cfg->num_actions <= 32, "num_actions out of range [1,32]");
  MT_CHECK_ARG(cfg->num_reps >= 1 && cfg->num_reps <= 31, "num_reps out of range [1,31]");
  MT_CHECK_ARG(cfg->activation == MT_ACT_RELU || cfg->activation == MT_ACT_LEAKY, "bad activation");
  MT_CHECK_ARG(cfg->softmax_temp > 0.f, "softmax_temp must be > 0");
  mt_net *n = new mt_net();
  n->cfg = *cfg;
  n->C = 4 * cfg->depth;
  n->O = 1 + cfg->num_actions + cfg->num_reps;
  const int arch = cfg->arch, d = cfg->depth;
  if (arch == MT_ARCH_NIPS && d == 1) build_layout<NipsArch<4>>(n);
  else if (arch == MT_ARCH_NIPS && d == 3) build_layout<NipsArch<12>>(n);
  else if (arch == MT_ARCH_NATURE && d == 1) build_layout<NatureArch<4>>(n);
  else if (arch == MT_ARCH_NATURE && d == 3) build_layout<NatureArch<12>>(n);
  else if (arch == MT_ARCH_PWYX && d == 1) build_layout<PwyxArch<4>>(n);
  else if (arch == MT_ARCH_PWYX && d == 3) build_layout<PwyxArch<12>>(n);
  else if (arch == MT_ARCH_LSTM && d == 1) build_layout_lstm<LstmArch<4>>(n);
  else if (arch == MT_ARCH_LSTM && d == 3) build_layout_lstm<LstmArch<12>>(n);
  else {
    delete n;
    set_error("arch %d not built into this library", arch);
    return MT_ERR_UNSUPPORTED;
  }
  *out = n;
  return MT_OK;
}

extern "C" void mt_net_destroy(mt_net *net) { delete net; }

extern "C" int mt_net_num_params(const mt_net *net, size_t *n) {
  MT_CHECK_ARG(net && n, "null argument");
  *n = net->nparams;
  return MT_OK;
}

extern "C" int mt_net_num_vars(const mt_net *net, int *n) {
  MT_CHECK_ARG(net && n, "null argument");
  *n = (int)net->vars.size();
  return MT_OK;
}

extern "C" int mt_net_var_info(const mt_net *net, int i, char *name, int name_len, int64_t *shape4,
                               int *ndim, size_t *offset, float *init_bound) {
  MT_CHECK_ARG(net, "null net");
  MT_CHECK_ARG(i >= 0 && i < (int)net->vars.size(), "var index %d out of range", i);
  const VarInfo &v = net->vars[i];
  if (name && name_len > 0) {
    std::strncpy(name, v.name.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (shape4)
    for (int k = 0; k < 4; ++k) shape4[k] = k < v.ndim ? v.shape[k] : 0;
  if (ndim) *ndim = v.ndim;
  if (offset) *offset = v.offset;
  if (init_bound) *init_bound = v.bound;
  return MT_OK;
}

extern "C" int mt_net_get_config(const mt_net *net, mt_net_config *cfg) {
  MT_CHECK_ARG(net && cfg, "null argument");
  *cfg = net->cfg;
  return MT_OK;
}

extern "C" int mt_net_feature_dim(const mt_net *net, int *f) {
  MT_CHECK_ARG(net && f, "null argument");
  *f = net->F;
  return MT_OK;
}

extern "C" int mt_net_workspace_bytes(const mt_net *net, int batch, size_t *bytes) {
  MT_CHECK_ARG(net && bytes, "null argument");
  MT_CHECK_ARG(batch >= 1, "batch must be >= 1");
  MT_ARCH_SWITCH(net, { *bytes = ws_layout<Ar>(net, batch).total * sizeof(float); });
  return MT_OK;
}

extern "C" int mt_net_backward_bucket_launches(const mt_net *net, int *launches) {
  MT_CHECK_ARG(net && launches, "null argument");
  MT_ARCH_SWITCH(net, {
    if constexpr (Ar::LSTM) {
      set_error("the LSTM backward is not bucketed");
      return MT_ERR_UNSUPPORTED;
    } else {
      *launches = kDenseBucketLaunches;  // backward_impl: loss | dense dX + dense dW + head dW | convs
    }
  });
  return MT_OK;
}

// Byte range of a stored forward value in a workspace (diagnostics / parity; mt_net_workspace_region):
// kind 0 = conv layer `layer`'s stored output (post-activation; the pooled map of a pooled layer),
// kind 1 = a pooled layer's argmax bytes, kind 2 = the dense layer's post-activation output H,
// kind 3 = the conv output's gradient (the backward's dY of the layer's weight gradient),
// kind 4 = the stacking chains' hand-off counters (uint32 words, zero between launches; 0 bytes when
// the arch keeps none).
template <class Ar, int I = 0>
static int ws_region(const WsLayout &L, int kind, int layer, size_t rows, size_t *offset, size_t *bytes) {
  if (kind == 4) {
    *offset = L.sync * sizeof(float);
    *bytes = (L.total - L.sync) * sizeof(float);
    return MT_OK;
  }
  if (kind == 2) {
    *offset = L.H * sizeof(float);
    *bytes = rows * Ar::F * sizeof(float);
    return MT_OK;
  }
  if constexpr (I < Ar::NCONV) {
    if (layer != I) return ws_region<Ar, I + 1>(L, kind, layer, rows, offset, bytes);
    using G = LayerG<Ar, I>;
    constexpr bool P = pooled<Ar, I>();
    const size_t px = P ? (size_t)(G::OH / 2) * (G::OW / 2) : (size_t)G::OH * G::OW;
    if (kind == 0) {
      *offset = (P ? L.pool[I] : L.act[I]) * sizeof(float);
      *bytes = rows * px * G::COUT * sizeof(float);
      return MT_OK;
    }
    if (kind == 1 && P) {
      *offset = L.parg[I] * sizeof(float);
      *bytes = rows * px * G::COUT;
      return MT_OK;
    }
    if (kind == 3) {  // the gradient of the conv output (full resolution; written by the backward)
      *offset = L.dact[I] * sizeof(float);
      *bytes = rows * G::OH * G::OW * G::COUT * sizeof(float);
      return MT_OK;
    }
    set_error("conv layer %d has no region of kind %d", layer, kind);
    return MT_ERR_ARG;
  }
  set_error("no conv layer %d", layer);
  return MT_ERR_ARG;
}

template <class Ar>
static int ws_region_windows(const mt_net *net, int a, int kind, int layer, size_t *offset, size_t *bytes) {
  const WsLayout L = lstm_ws_layout<Ar>(net, a, nullptr);
  return ws_region<Ar>(L, kind, layer, kind == 2 ? (size_t)a : (size_t)a * Ar::STEPS, offset, bytes);
}

template <class Ar>
static int ws_region_frames(const mt_net *net, int E, int T, int kind, int layer, size_t *offset, size_t *bytes) {
  const LstmFrameWs X = lstm_frame_layout<Ar>(net, E, T);
  return ws_region<Ar>(X.L, kind, layer, kind == 2 ? (size_t)X.W : (size_t)X.R_max, offset, bytes);
}

extern "C" int mt_net_workspace_region(const mt_net *net, int layout, int a, int b, int kind, int layer,
                                       size_t *offset, size_t *bytes) {
  MT_CHECK_ARG(net && offset && bytes, "null argument");
  MT_CHECK_ARG(a >= 1 && (layout != 1 || b >= 1) && kind >= 0 && kind <= 4, "bad sizes or kind");
  MT_CHECK_ARG(kind != 4 || layout == 0, "the counter region (kind 4) is in the layout-0 workspace");
  MT_ARCH_SWITCH(net, {
    if (layout == 0) {
      if constexpr (Ar::LSTM) {
        set_error("layout 0 is the non-LSTM workspace");
        return MT_ERR_ARG;
      } else {
        return ws_region<Ar>(ws_layout<Ar>(net, a), kind, layer, (size_t)a, offset, bytes);
      }
    } else if (layout == 1 || layout == 2) {
      if constexpr (!Ar::LSTM) {
        set_error("layouts 1 and 2 are LSTM workspaces");
        return MT_ERR_ARG;
      } else {
        return layout == 1 ? ws_region_frames<Ar>(net, a, b, kind, layer, offset, bytes)
                           : ws_region_windows<Ar>(net, a, kind, layer, offset, bytes);
      }
    }
    set_error("layout %d", layout);
    return MT_ERR_ARG;
  });
  return MT_OK;
}

extern "C" int mt_forward(const mt_net *net, const float *params, const uint8_t *obs, int batch,
                          void *ws, size_t ws_bytes, float *v, float *pi, float *rep,
                          mt_stream_t stream) {
  return mt::forward_sample(net, params, obs, batch, ws, ws_bytes, v, pi, rep, nullptr, false,
                            (hipStream_t)stream);
}

// Trunk half of the inference forward (diagnostics / roofline timing): everything up to the
// dense layer's partial slabs that heads_fwd_kernel finishes — the fused NIPS trunk, else the
// layered convs + split-K fc (LSTM: the 5B-frame trunk + the cell's x-product slabs).
template <class Ar>
static int trunk_infer_impl(const mt_net *n, const float *P, const uint8_t *obs, int B, float *ws, hipStream_t s,
                            const StackSrc *st = nullptr) {
  if constexpr (Ar::LSTM) {
    LstmWs X;
    const WsLayout L = lstm_ws_layout<Ar>(n, B, &X);
    const int rows = B * Ar::STEPS;
    MT_TRY((trunk_forward<Ar>(n, P, obs, rows, ws, L, s)));
    return launch_gemm<TileFc>(LdRowMajor{layer_out<Ar, Ar::NCONV - 1>(ws, L), Ar::FLAT},
                               LdColMajor{P + n->off_lstm, Ar::G4, -1}, EpSlab{ws + X.xg, rows, Ar::G4}, rows,
                               Ar::G4, Ar::FLAT, X.xg_splits, s);
  } else {
    const WsLayout L = ws_layout<Ar>(n, B);
    const float *Wfc = P + n->off_fc;
    if constexpr (Ar::FUSED_SLABS > 0) {
      constexpr int C = LayerG<Ar, 0>::CIN;
      MT_TRY((launch_nips_trunk<C>(obs, st, B, P + n->off_conv[0], P + n->off_conv[1], Wfc,
                                   n->cfg.activation, n->cfg.alpha_leaky, ws + L.act[1], nullptr, ws + L.fcslab, s)));
      MT_LAUNCHED();
      return MT_OK;
    } else {
      FwdExtras ex;
      ex.st = st;
      ex.sync = reinterpret_cast<uint32_t *>(ws + L.sync);
      MT_TRY((trunk_forward<Ar>(n, P, obs, B, ws, L, s, ex)));
      return launch_fc<Ar>(layer_out<Ar, Ar::NCONV - 1>(ws, L), B, Wfc, ws + L.fcslab, L.fc_splits, s);
    }
  }
}

extern "C" int mt_forward_trunk(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                                size_t ws_bytes, mt_stream_t stream) {
  MT_CHECK_ARG(net && params && obs && ws, "null argument");
  MT_CHECK_ARG(batch >= 1, "batch must be >= 1");
  MT_ARCH_SWITCH(net, {
    const WsLayout L = ws_layout<Ar>(net, batch);
    if (ws_bytes < L.total * sizeof(float)) {
      set_error("workspace %zu < %zu bytes", ws_bytes, L.total * sizeof(float));
      return MT_ERR_WORKSPACE;
    }
    return trunk_infer_impl<Ar>(net, params, obs, batch, (float *)ws, (hipStream_t)stream);
  });
  return MT_OK;
}

extern "C" int mt_forward_trunk_stacking(const mt_net *net, const float *params, const uint8_t *prev,
                                         const uint8_t *frames, const uint32_t *ready, uint32_t tag, uint8_t *out,
                                         int batch, void *ws, size_t ws_bytes, uint32_t *status,
                                         mt_stream_t stream) {
  MT_CHECK_ARG(net && params && prev && frames && ready && out && ws, "null argument");
  MT_CHECK_ARG(batch >= 1, "batch must be >= 1");
  StackSrc st{prev, frames, nullptr, out};
  st.ready = ready;
  st.tag = tag & 0x1fffffffu;
  st.status = status;
  MT_ARCH_SWITCH(net, {
    const WsLayout L = ws_layout<Ar>(net, batch);
    if (ws_bytes < L.total * sizeof(float)) {
      set_error("workspace %zu < %zu bytes", ws_bytes, L.total * sizeof(float));
      return MT_ERR_WORKSPACE;
    }
    if constexpr (Ar::LSTM) {
      set_error("stacking trunk: the NIPS, gray NATURE and PWYX archs (the LSTM steps: mt_lstm_step_forward)");
      return MT_ERR_UNSUPPORTED;
    } else {
      return trunk_infer_impl<Ar>(net, params, out, batch, (float *)ws, (hipStream_t)stream, &st);
    }
  });
  return MT_OK;
}

extern "C" int mt_forward_rows(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                               size_t ws_bytes, void *train_ws, size_t train_ws_bytes, int train_rows, int row0,
                               float *v, float *pi, float *rep, mt_stream_t stream) {
  MT_CHECK_ARG(train_ws, "null train workspace");
  const TrainRows tr{(float *)train_ws, train_ws_bytes, train_rows, row0};
  return mt::forward_sample(net, params, obs, batch, ws, ws_bytes, v, pi, rep, nullptr, true, (hipStream_t)stream,
                            &tr);
}

extern "C" int mt_forward_infer(const mt_net *net, const float *params, const uint8_t *obs, int batch,
                                void *ws, size_t ws_bytes, float *v, float *pi, float *rep,
                                mt_stream_t stream) {
  return mt::forward_sample(net, params, obs, batch, ws, ws_bytes, v, pi, rep, nullptr, true,
                            (hipStream_t)stream);
}

int mt::forward_sample(const mt_net *net, const float *params, const uint8_t *obs, int batch,
                       void *ws, size_t ws_bytes, float *v, float *pi, float *rep, const SampleArgs *smp,
                       bool infer, hipStream_t stream, const TrainRows *tr, const StackSrc *st,
                       const hipEvent_t *marks) {
  MT_CHECK_ARG(net && params && obs && ws && v && pi && rep, "null argument");
  // (smp without counters: no draw — the replayed rollout graph's bootstrap carries only `advance`)
  MT_CHECK_ARG(!smp || !smp->counters || (smp->a_idx && smp->r_idx), "null sample buffer");
  MT_CHECK_ARG(batch >= 1, "batch must be >= 1");
  MT_ARCH_SWITCH(net, {
    const WsLayout L = ws_layout<Ar>(net, batch);
    if (ws_bytes < L.total * sizeof(float)) {
      set_error("workspace %zu < %zu bytes", ws_bytes, L.total * sizeof(float));
      return MT_ERR_WORKSPACE;
    }
    if (tr) {
      MT_CHECK_ARG(!Ar::LSTM, "train-row forwards are not built for the LSTM arch (frame store: mt_lstm_*)");
      MT_CHECK_ARG(tr->ws && tr->rows >= 1 && tr->row0 >= 0 && tr->row0 + batch <= tr->rows,
                   "train rows [%d, %d) outside [0, %d)", tr->row0, tr->row0 + batch, tr->rows);
      const size_t need = ws_layout<Ar>(net, tr->rows).total * sizeof(float);
      if (tr->ws_bytes < need) {
        set_error("train workspace %zu < %zu bytes", tr->ws_bytes, need);
        return MT_ERR_WORKSPACE;
      }
    }
    if constexpr (Ar::LSTM)
      return lstm_forward_impl<Ar>(net, params, obs, batch, (float *)ws, v, pi, rep, smp, stream);
    else
      MT_CHECK_ARG(!st || infer, "stacking forward is an inference forward");
      return infer ? forward_infer_impl<Ar>(net, params, obs, batch, (float *)ws, v, pi, rep, smp, stream, tr, st,
                                            marks)
                   : forward_impl<Ar>(net, params, obs, batch, (float *)ws, v, pi, rep, smp, stream, tr, marks);
  });
  return MT_OK;
}

int mt::forward_boot(const mt_net *net, const float *params, const uint8_t *obs, int batch, void *ws,
                     size_t ws_bytes, hipStream_t stream, const StackSrc *st, uint32_t *advance, uint32_t advance_by) {
  MT_CHECK_ARG(net && params && obs && ws && batch >= 1, "bad argument");
  MT_ARCH_SWITCH(net, {
    if constexpr (Ar::LSTM) {
      set_error("the LSTM bootstrap runs through mt_lstm_step_forward");
      return MT_ERR_UNSUPPORTED;
    } else {
      const WsLayout L = ws_layout<Ar>(net, batch);
      if (ws_bytes < L.total * sizeof(float)) {
        set_error("workspace %zu < %zu bytes", ws_bytes, L.total * sizeof(float));
        return MT_ERR_WORKSPACE;
      }
      return forward_boot_impl<Ar>(net, params, obs, batch, (float *)ws, stream, st, advance, advance_by);
    }
  });
  return MT_OK;
}

extern "C" int mt_loss_backward(const mt_net *net, const float *params, const uint8_t *obs,
                                int batch, void *ws, size_t ws_bytes, const float *pi,
                                const float *rep, const float *v, const int32_t *a_idx,
                                const int32_t *r_idx, const float *y, const float *adv,
                                float entropy_beta, float *grad, float *loss_terms,
                                mt_stream_t stream) {
  MT_CHECK_ARG(net && params && obs && ws && pi && rep && v && a_idx && r_idx && y && adv && grad,
               "null argument");
  MT_CHECK_ARG(batch >= 1, "batch must be >= 1");
  MT_ARCH_SWITCH(net, {
    const WsLayout L = ws_layout<Ar>(net, batch);
    if (ws_bytes < L.total * sizeof(float)) {
      set_error("workspace %zu < %zu bytes", ws_bytes, L.total * sizeof(float));
      return MT_ERR_WORKSPACE;
    }
    if constexpr (Ar::LSTM)
      return lstm_backward_impl<Ar>(net, params, obs, batch, (float *)ws, pi, rep, v, a_idx, r_idx, y, adv,
                                    entropy_beta, grad, loss_terms, (hipStream_t)stream);
    else
      return backward_impl<Ar>(net, params, obs, batch, (float *)ws, pi, rep, v, a_idx, r_idx, y, adv,
                               entropy_beta, grad, loss_terms, (hipStream_t)stream);
  });
  return MT_OK;
}

extern "C" int mt_returns_loss_backward(const mt_net *net, const float *params, const uint8_t *obs, int T, int E,
                                        void *ws, size_t ws_bytes, const float *pi, const float *rep,
                                        const float *values, const int32_t *a_idx, const int32_t *r_idx,
                                        const float *rewards, const float *masks, const float *v_boot, double gamma,
                                        float *y, float *adv, float entropy_beta, float *grad, float *loss_terms,
                                        float *norm_partials, mt_stream_t stream) {
  MT_CHECK_ARG(net && params && obs && ws && pi && rep && values && a_idx && r_idx && rewards && masks && v_boot &&
                   y && adv && grad,
               "null argument");
  MT_CHECK_ARG(T >= 1 && E >= 1 && T <= kMaxScan, "T=%d (<= %d) and E=%d must be >= 1", T, kMaxScan, E);
  const int batch = T * E;
  MT_ARCH_SWITCH(net, {
    if constexpr (Ar::LSTM) {
      set_error("mt_returns_loss_backward: the LSTM arch trains through mt_lstm_frames_backward");
      return MT_ERR_UNSUPPORTED;
    } else {
      const WsLayout L = ws_layout<Ar>(net, batch);
      if (ws_bytes < L.total * sizeof(float)) {
        set_error("workspace %zu < %zu bytes", ws_bytes, L.total * sizeof(float));
        return MT_ERR_WORKSPACE;
      }
      ReturnsSrc rs;
      rs.r = rewards;
      rs.mask = masks;
      rs.VT = v_boot;
      rs.gamma = gamma;
      rs.T = T;
      rs.E = E;
      rs.y_out = y;
      rs.adv_out = adv;
      NormOut no;
      no.partials = norm_partials;
      no.n = net->nparams;
      return backward_impl<Ar>(net, params, obs, batch, (float *)ws, pi, rep, values, a_idx, r_idx, y, adv,
                               entropy_beta, grad, loss_terms, (hipStream_t)stream, rs, no);
    }
  });
  return MT_OK;
}

extern "C" int mt_returns_loss_backward_boot(const mt_net *net, const float *params, const uint8_t *obs, int T, int E,
                                             void *ws, size_t ws_bytes, const float *pi, const float *rep,
                                             const float *values, const int32_t *a_idx, const int32_t *r_idx,
                                             const float *rewards, const float *masks, const void *boot_ws,
                                             size_t boot_ws_bytes, float *v_boot, double gamma, float *y, float *adv,
                                             float entropy_beta, float *grad, float *loss_terms, float *norm_partials,
                                             mt_stream_t stream) {
  MT_CHECK_ARG(net && params && obs && ws && pi && rep && values && a_idx && r_idx && rewards && masks && boot_ws &&
                   v_boot && y && adv && grad,
               "null argument");
  MT_CHECK_ARG(T >= 1 && E >= 1 && T <= kMaxScan, "T=%d (<= %d) and E=%d must be >= 1", T, kMaxScan, E);
  const int batch = T * E;
  MT_ARCH_SWITCH(net, {
    if constexpr (Ar::LSTM) {
      set_error("mt_returns_loss_backward_boot: the LSTM arch trains through mt_lstm_frames_backward");
      return MT_ERR_UNSUPPORTED;
    } else {
      const WsLayout L = ws_layout<Ar>(net, batch);
      const WsLayout LB = ws_layout<Ar>(net, E);
      if (ws_bytes < L.total * sizeof(float) || boot_ws_bytes < LB.total * sizeof(float)) {
        set_error("workspace %zu / bootstrap workspace %zu < %zu / %zu bytes", ws_bytes, boot_ws_bytes,
                  L.total * sizeof(float), LB.total * sizeof(float));
        return MT_ERR_WORKSPACE;
      }
      MT_CHECK_ARG(Ar::F <= 512, "F > 512");
      ReturnsSrc rs;
      rs.r = rewards;
      rs.mask = masks;
      rs.gamma = gamma;
      rs.T = T;
      rs.E = E;
      rs.y_out = y;
      rs.adv_out = adv;
      rs.boot_slabs = (const float *)boot_ws + LB.fcslab;
      rs.boot_S = Ar::FUSED_SLABS > 0 ? Ar::FUSED_SLABS : LB.fc_splits;
      rs.fc_b = params + net->off_fc + (size_t)Ar::FLAT * Ar::F;
      rs.vt_out = v_boot;
      NormOut no;
      no.partials = norm_partials;
      no.n = net->nparams;
      return backward_impl<Ar>(net, params, obs, batch, (float *)ws, pi, rep, values, a_idx, r_idx, y, adv,
                               entropy_beta, grad, loss_terms, (hipStream_t)stream, rs, no);
    }
  });
  return MT_OK;
}

// ---- LSTM frame-store mode (lstm.h) ----------------------------------------------------------
#define MT_LSTM_ONLY(net, ...)                                                  \
  MT_ARCH_SWITCH(net, {                                                         \
    if constexpr (Ar::LSTM) {                                                   \
      __VA_ARGS__;                                                              \
    } else {                                                                    \
      set_error("frame-store calls need the LSTM arch");                        \
      return MT_ERR_ARG;                                                        \
    }                                                                           \
  })

#define MT_LSTM_WS(E, T)                                                        \
  const LstmFrameWs X_ = lstm_frame_layout<Ar>(net, E, T);                      \
  if (ws_bytes < X_.L.total * sizeof(float)) {                                  \
    set_error("workspace %zu < %zu bytes", ws_bytes, X_.L.total * sizeof(float)); \
    return MT_ERR_WORKSPACE;                                                    \
  }

extern "C" int mt_lstm_frames_workspace_bytes(const mt_net *net, int E, int T, size_t *bytes) {
  MT_CHECK_ARG(net && bytes, "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  MT_LSTM_ONLY(net, { *bytes = lstm_frame_layout<Ar>(net, E, T).L.total * sizeof(float); });
  return MT_OK;
}

extern "C" int mt_lstm_frames_forward(const mt_net *net, const float *params, const uint8_t *fstore, int row0,
                                      int nrows, int E, int T, void *ws, size_t ws_bytes, mt_stream_t stream) {
  MT_CHECK_ARG(net && params && fstore && ws, "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  MT_LSTM_ONLY(net, {
    MT_LSTM_WS(E, T);
    return lstm_frames_fwd_impl<Ar>(net, params, fstore, row0, nrows, E, T, (float *)ws, (hipStream_t)stream);
  });
  return MT_OK;
}

extern "C" int mt_lstm_windows_forward(const mt_net *net, const float *params, const int32_t *nz_t, int t, int E,
                                       int T, void *ws, size_t ws_bytes, float *v, float *pi, float *rep,
                                       mt_stream_t stream) {
  MT_CHECK_ARG(net && params && nz_t && ws && v && pi && rep, "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  MT_LSTM_ONLY(net, {
    MT_LSTM_WS(E, T);
    // (nz_t is only read: no nz_prev)
    return lstm_windows_fwd_impl<Ar>(net, params, const_cast<int32_t *>(nz_t), t, E, T, (float *)ws, v, pi, rep,
                                     (hipStream_t)stream);
  });
  return MT_OK;
}

extern "C" int mt_lstm_step_forward(const mt_net *net, const float *params, const uint8_t *fstore, int t, int E,
                                    int T, int32_t *nz, const float *over, void *ws, size_t ws_bytes, float *v,
                                    float *pi, float *rep, mt_stream_t stream) {
  MT_CHECK_ARG(net && params && fstore && nz && ws && v && pi && rep, "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  return mt::lstm_step_forward(net, params, fstore, t, E, T, nz, over, ws, ws_bytes, v, pi, rep, nullptr,
                               (hipStream_t)stream);
}

int mt::lstm_step_forward(const mt_net *net, const float *params, const uint8_t *fstore, int t, int E, int T,
                          int32_t *nz, const float *over, void *ws, size_t ws_bytes, float *v, float *pi, float *rep,
                          const SampleArgs *smp, hipStream_t stream, const hipEvent_t *marks, const StackSrc *st,
                          uint32_t *sync) {
  MT_CHECK_ARG(!smp || (smp->counters && smp->a_idx && smp->r_idx), "null sample buffer");
  MT_LSTM_ONLY(net, {
    MT_LSTM_WS(E, T);
    return lstm_step_fwd_impl<Ar>(net, params, fstore, t, E, T, nz, over, (float *)ws, v, pi, rep, smp, stream,
                                  marks, st, sync);
  });
  return MT_OK;
}

extern "C" int mt_lstm_frames_backward(const mt_net *net, const float *params, const uint8_t *fstore,
                                       const int32_t *nz, int E, int T, void *ws, size_t ws_bytes, const float *pi,
                                       const float *rep, const float *v, const int32_t *a_idx, const int32_t *r_idx,
                                       const float *y, const float *adv, float entropy_beta, float *grad,
                                       float *loss_terms, float *norm_partials, mt_stream_t stream) {
  MT_CHECK_ARG(net && params && fstore && nz && ws && pi && rep && v && a_idx && r_idx && y && adv && grad,
               "null argument");
  MT_CHECK_ARG(E >= 1 && T >= 1, "E and T must be >= 1");
  MT_LSTM_ONLY(net, {
    MT_LSTM_WS(E, T);
    NormOut no;
    no.partials = norm_partials;
    no.n = net->nparams;
    return lstm_frames_bwd_impl<Ar>(net, params, fstore, nz, E, T, (float *)ws, pi, rep, v, a_idx, r_idx, y, adv,
                                    entropy_beta, grad, loss_terms, (hipStream_t)stream, no);
  });
  return MT_OK;
}

extern "C" int mt_sum_slabs(const float *parts, int nslabs, size_t n, float *out,
                            mt_stream_t stream) {
  MT_CHECK_ARG(parts && out && nslabs >= 1, "bad argument");
  return sum_slabs(parts, nslabs, n, out, (hipStream_t)stream);
}
