// Direct convolution for the stride-1 SAME convs of the PWYX trunk (networks.py:206-225; the LSTM
// arch runs it per window frame, networks.py:227-258) and the strided VALID convs of the NATURE
// trunk (networks.py:261-278): the forward (conv + bias + activation, + the 2x2/2 max pool and its
// argmax bytes), the backward-data product of the 5x5 layer (dX of a conv whose input is a pooled
// layer: MaxPoolGrad routing and the activation mask in the epilogue) and the weight gradients of
// the 5x5 layers (DWgradJob, at the end of the file). Which layers take which product, and the
// alternatives that were measured and not adopted, are documented where each choice is made.
//
// Why not the generic implicit-im2col GEMM (gemm.h, LdIm2col / LdConvBwdA): there every A element
// of every K chunk is re-derived from (row, k) — tap / channel divisions, SAME-padding clamps and
// selects — and fetched from L2: 5-8 VALU instructions per MFMA (rocprof PMC,
// profiles/r03c_pmc_generic_*), which sets the pace instead of the MFMA. Here a block stages its
// input PATCH once in LDS (zero-padded; u8 -> f32 for conv1), and the K walk reads each A fragment
// as ONE ds_read_b128 at (the lane's pixel) + (the tap's offset): no per-element address math.
//
// Block = NW = WM x WN waves, UPB "units" of one image x all output channels. A unit is one 2x2
// pool window (forward of a pooled layer: its 4 pixels are the 4 rows a lane's accumulator holds,
// so the pool is a register max) or a quad of consecutive pixels. A wave owns TMW 16-row M-tiles
// (4 units each) and TNW 16-column N-tiles: TMW x TNW accumulators of v_mfma_f32_16x16x4_f32.
//
// K order: k = tap * CI + c. A fragment element s of lane (r, g) of k-chunk kc is k = 16 kc + 4 g
// + s, i.e. channel quad q = 4 kc + g of tap q / (CI/4): 4 consecutive channels of one pixel = one
// 16-byte LDS read. The weights are staged chunk by chunk (CK k-values) into LDS in that fragment
// order — [kc][n-tile][lane][4], so a B fragment is one conflict-free ds_read_b128 —
// double-buffered: chunk c+1's global loads are in flight while chunk c is multiplied, one barrier
// per chunk. The backward-data product is the same direct conv on dY with the kernel flipped and
// its channel axes swapped (W'[ky'][kx'][co][ci] = W[KH-1-ky'][KW-1-kx'][ci][co], pad KH-1-PT):
// its staging reads 4 consecutive co of one (tap, ci) — one 16-byte load.
#pragma once
#include "gemm.h"

namespace mt {

// Probe builds (-DMT_PROBE): per env, when its publication was seen by a conv1 block (0) and when
// its last conv1 / conv2 / conv3 block finished (1, 2, 3); s_memrealtime, read by mt_probe_read_chain
// and per block (blockIdx < 2048) of nature_chain_kernel, slots: 0 start, 1 waited (consumers) /
// publication seen (conv1), 2 frames staged (conv1), 3 body done, 4 signal stores drained
#ifdef MT_PROBE
static __device__ unsigned long long mt_probe_chain[512 * 4];
static __device__ unsigned long long mt_probe_chainblk[2048 * 8];
#define MT_PROBE_CHAIN(e, p) \
  if ((e) < 512) mt_probe_chain[(e) * 4 + (p)] = __builtin_amdgcn_s_memrealtime()
#define MT_PROBE_BLK(p) \
  if (threadIdx.x == 0 && blockIdx.x < 2048) mt_probe_chainblk[blockIdx.x * 8 + (p)] = __builtin_amdgcn_s_memrealtime()
#else
#define MT_PROBE_CHAIN(e, p)
#define MT_PROBE_BLK(p)
#endif

// ---- problems ------------------------------------------------------------------------------
// Forward of conv G: X = its input [B][H][W][CIN] (u8 frames for conv1), Y = the pooled output
// [B][OH/2][OW/2][COUT] + argmax bytes (POOL, EpBiasActPool's layout and first-max rule) or the
// activation [B][OH][OW][COUT].
// COH_IN / COH_OUT (the in-launch hand-offs of nature_chain_kernel): X read / Y written with
// agent-scope relaxed atomics (sc1: coherent across the XCDs' L2s) instead of plain accesses.
template <class G, bool U8, bool POOL_, bool COH_IN = false, bool COH_OUT = false>
struct DFwd {
  static constexpr int CI = G::CIN, CO = G::COUT, KH = G::KH, KW = G::KW, PT = G::PT, PL = G::PL, S = G::S;
  static constexpr int H = G::H, W = G::W, OH = G::OH, OW = G::OW, KK = G::KK;
  static constexpr bool POOL = POOL_;
  using InT = typename InElem<U8>::T;
  const InT *X;
  const float *Wt, *bias;
  float *Y;
  uint8_t *arg;
  int act;
  float alpha;
  __device__ __forceinline__ f32x4 wquad(int k, int n) const {  // W(k .. k+3, n), zero past KK
    f32x4 v;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float x = Wt[(size_t)min(k + s, KK - 1) * CO + n];
      v[s] = k + s < KK ? x : 0.f;
    }
    return v;
  }
  struct Pre {
    float b;
  };
  __device__ __forceinline__ Pre pre(int, int, int n) const { return {bias[n]}; }
  __device__ __forceinline__ f32x4 load4(const InT *q) const {
    if constexpr (COH_IN && U8) {  // (a frame trunk's stacked state, stack_conv1_kernel)
      const uint32_t u = __hip_atomic_load(reinterpret_cast<const uint32_t *>(q), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      const float sc = 1.0f / 255.0f;  // InElem<true>::load4's arithmetic
      return f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc, (float)((u >> 16) & 0xff) * sc,
                   (float)(u >> 24) * sc};
    } else if constexpr (COH_IN) {
      const uint64_t *w = reinterpret_cast<const uint64_t *>(q);
      const uint64_t x = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t y = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return f32x4{__uint_as_float((uint32_t)x), __uint_as_float((uint32_t)(x >> 32)), __uint_as_float((uint32_t)y),
                   __uint_as_float((uint32_t)(y >> 32))};
    } else {
      return InElem<U8>::load4(q);
    }
  }
  __device__ __forceinline__ void put(size_t o, float v) const {
    if constexpr (COH_OUT)
      __hip_atomic_store(Y + o, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      Y[o] = v;
  }
  __device__ __forceinline__ void store(const Pre &p, int b, int u, int n, f32x4 v) const {
    if constexpr (POOL) {
      static_assert(!COH_OUT, "coherent stores of unpooled outputs only");
      constexpr int U = (G::OH / 2) * (G::OW / 2);
      float mx = act_fwd(v[0] + p.b, act, alpha);
      int am = 0;
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float y = act_fwd(v[q] + p.b, act, alpha);
        if (y > mx) {
          mx = y;
          am = q;
        }
      }
      const size_t o = ((size_t)b * U + u) * CO + n;
      Y[o] = mx;
      arg[o] = (uint8_t)am;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int px = 4 * u + q;
        if (px < OH * OW) put(((size_t)b * OH * OW + px) * CO + n, act_fwd(v[q] + p.b, act, alpha));
      }
    }
  }
};

// The NATURE rollout chain's conv1 with the A2 stacking and the in-kernel pull fused in (the NIPS
// chain's nips_stage_rows, trunk_fused.h): each block builds its patch rows from the previous
// state and env b's p new final frames — read from the pinned staging once env b's emulator thread
// has published it (StackSrc::ready; edge lines of its slot group with system-scope loads), or
// from HBM (count), or none (count == NULL: a copy of prev, slot 0 <- slot T) — converts them into
// the f32 patch (networks.py:155's u8 * (1/255), bit for bit the unstacked loader's) and writes
// the rows it owns to the new state slot. So env b's conv1 runs as soon as env b is emulated, not
// after the last env. Gray frames (one u32 = 4 channels per pixel), VALID.
template <class G, bool COH_OUT = false>
struct DFwdStack : DFwd<G, true, false, false, COH_OUT> {
  static_assert(G::CIN == 4 && !G::SAME && G::PT == 0 && G::PL == 0 && G::W % 4 == 0, "gray VALID conv1");
  static constexpr bool STAGES_PATCH = true;
  StackSrc st;
  // rows [r0, r0 + D::RIN) of image b into the patch As; rows [r0, own_end) are the block's to
  // write to st.out; fr: >= 4 * RIN * W bytes of LDS scratch (free until the caller's weight store)
  template <class D>
  __device__ __forceinline__ void stage_patch(int b, int r0, int own_end, float *As, uint8_t *fr) const {
    constexpr int H = G::H, W = G::W, RIN = D::RIN, NT = D::NT;
    static_assert(D::WP == W && D::WPX == W && D::CS == 4, "full-width patch rows, 4 floats per pixel");
    static_assert(RIN % 4 == 0 && H % 4 == 0 && G::S % 4 == 0, "16-B frame chunks");
    constexpr int PQ = RIN * W / 4;  // 4-pixel items of the patch
    constexpr int PIT = (PQ + NT - 1) / NT;
    const int tid = threadIdx.x;
    const int rows = min(RIN, H - r0);  // patch rows inside the image
    const int nq = rows * W / 4;
    __shared__ int s_p;
    // the previous state's rows, requested before the wait (their latency hides under it)
    const uint4 *prev = reinterpret_cast<const uint4 *>(st.prev + ((size_t)b * H + r0) * W * 4);
    uint4 pv[PIT];
#pragma unroll
    for (int it = 0; it < PIT; ++it) pv[it] = prev[min(tid + it * NT, nq - 1)];
    if (tid == 0) {
      int np = 0;
      if (st.ready) {
        const uint32_t tag = st.tag_base ? ((*st.tag_base + st.tag) & 0x1fffffffu) : st.tag;
        np = min(max(wait_published(st.ready, b, tag, st.status), 0), 4);  // (a timeout stacks no frame)
        MT_PROBE_CHAIN(b, 0);
        MT_PROBE_BLK(1);
      } else if (st.count) {
        np = min(max(st.count[b], 1), 4);
      }
      s_p = np;
    }
    __syncthreads();
    const int p = s_p;
    // the p pushes' rows (push j of env b = frame slot 4b + j), one round trip
    constexpr size_t F = (size_t)H * W;
    const size_t lo = 4 * (size_t)b * F, hi = lo + 4 * F;
    const int fq = rows * W / 16;
    for (int q = tid; q < p * fq; q += NT) {
      const int j = q / fq, qq = q - j * fq;
      const size_t off = ((size_t)4 * b + j) * F + (size_t)r0 * W + 16 * (size_t)qq;
      reinterpret_cast<uint4 *>(fr + j * RIN * W)[qq] =
          st.ready ? ld_published16(st.frames, off, lo, hi) : *reinterpret_cast<const uint4 *>(st.frames + off);
    }
    __syncthreads();
    MT_PROBE_BLK(2);
    // stack (preprocess_kernel's op: prev shifted by p channels, the p frames in the top ones),
    // the owned rows to the new state, every row into the patch
    uint4 *out = reinterpret_cast<uint4 *>(st.out + ((size_t)b * H + r0) * W * 4);
    const int own_q = (own_end - r0) * W / 4;
    const float sc = 1.0f / 255.0f;
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int q = tid + it * NT;
      if (PQ % NT != 0 && q >= PQ) break;
      uint32_t wv[4] = {pv[it].x, pv[it].y, pv[it].z, pv[it].w};
      if (q < nq) {
        uint32_t fw[4];
        for (int j = 0; j < p; ++j) fw[j] = reinterpret_cast<const uint32_t *>(fr + j * RIN * W)[q];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t v = p < 4 ? wv[k] >> (8 * p) : 0u;
          for (int j = 0; j < p; ++j) v |= ((fw[j] >> (8 * k)) & 0xffu) << (8 * (4 - p + j));
          wv[k] = v;
        }
        if (q < own_q) out[q] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      } else {
        wv[0] = wv[1] = wv[2] = wv[3] = 0u;  // (rows past the image: zero patch)
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t u = wv[k];
        *reinterpret_cast<f32x4 *>(As + 16 * q + 4 * k) =
            f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc, (float)((u >> 16) & 0xff) * sc,
                  (float)(u >> 24) * sc};
      }
    }
    __syncthreads();  // (fr aliases the weight buffer the caller fills next)
  }
};

// problems with their own patch staging (DFwdStack)
template <class P, class = void>
struct HasStagePatch : std::false_type {};
template <class P>
struct HasStagePatch<P, std::void_t<decltype(P::STAGES_PATCH)>> : std::bool_constant<P::STAGES_PATCH> {};

// dX of the stride-1 SAME conv G (input = the pooled output of conv GJ): X = dY of G
// [B][OH][OW][COUT], output = GJ's full-resolution conv-output gradient dact [B][GJ::OH][GJ::OW]
// [GJ::COUT]: g = dX * act'(pooled value) routed to the window's argmax position, zeros elsewhere
// (and in the row / column a VALID pool drops) — EpMaskedUnpool.
template <class G, class GJ>
struct DBwdUnpool {
  static_assert(G::S == 1 && G::SAME && G::H == G::OH && GJ::COUT == G::CIN, "pooled input of a stride-1 conv");
  static constexpr int CI = G::COUT, CO = G::CIN, KH = G::KH, KW = G::KW;
  static constexpr int PT = G::KH - 1 - G::PT, PL = G::KW - 1 - G::PL;
  static constexpr int H = G::H, W = G::W, OH = G::H, OW = G::W, S = 1, KK = G::KH * G::KW * G::COUT;
  static constexpr bool POOL = false;
  using InT = float;
  const float *X;     // dY
  const float *Wt;    // W of G (HWIO)
  const float *P;     // GJ's pooled output [B][H][W][CO]
  const uint8_t *arg;
  float *dact;        // GJ's conv-output gradient
  int act;
  float alpha;
  __device__ __forceinline__ f32x4 wquad(int k, int n) const {  // W'(k .. k+3, n): 4 co of one tap
    const int t = k / CI, c = k - t * CI;
    const int tf = (KH - 1 - t / KW) * KW + (KW - 1 - t % KW);
    return *reinterpret_cast<const f32x4 *>(Wt + ((size_t)tf * G::CIN + n) * G::COUT + c);
  }
  struct Pre {
    float p[4];
    uint8_t a[4];
  };
  __device__ __forceinline__ f32x4 load4(const float *q) const { return *reinterpret_cast<const f32x4 *>(q); }
  __device__ __forceinline__ Pre pre(int b, int u, int n) const {
    Pre r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const size_t i = ((size_t)b * H * W + min(4 * u + q, H * W - 1)) * CO + n;
      r.p[q] = P[i];
      r.a[q] = arg[i];
    }
    return r;
  }
  __device__ __forceinline__ void store(const Pre &pr, int b, int u, int n, f32x4 v) const {
    constexpr int C = GJ::COUT;
    constexpr size_t RW = (size_t)GJ::OW * C;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int px = 4 * u + q;
      if (px >= H * W) break;
      const int py = px / W, pxx = px - py * W;
      const float g = v[q] * act_bwd(pr.p[q], act, alpha);
      const int a = pr.a[q];
      float *d = dact + (((size_t)b * GJ::OH + 2 * py) * GJ::OW + 2 * pxx) * C + n;
      d[0] = a == 0 ? g : 0.f;
      d[C] = a == 1 ? g : 0.f;
      d[RW] = a == 2 ? g : 0.f;
      d[RW + C] = a == 3 ? g : 0.f;
      if constexpr (GJ::OW & 1) {
        if (pxx == W - 1) {
          d[2 * C] = 0.f;
          d[RW + 2 * C] = 0.f;
        }
      }
      if constexpr (GJ::OH & 1) {
        if (py == H - 1) {
          d[2 * RW] = 0.f;
          d[2 * RW + C] = 0.f;
          if constexpr (GJ::OW & 1) {
            if (pxx == W - 1) d[2 * RW + 2 * C] = 0.f;
          }
        }
      }
    }
  }
};

// ---- tiling ------------------------------------------------------------------------------------
// Patch pixel stride CS (floats): CI + 4 for 16-channel multiples (the A-fragment reads of a lane
// group then spread over the banks). Per-layer strides / row pads from a model of the LDS banks
// (tools/lds_banks.py: conflict cycles 8 -> 4-5 per read) measured no faster — the reads are
// latency, not LDS throughput — and cost the 5x5 dX an occupancy level (round 3). Persistent
// conv1 blocks staging the weights once also measured no faster (round 3, profiles/r03g).
constexpr int dconv_cs(int ci) { return ci % 16 == 0 ? ci + 4 : ci; }

template <class Pr, int WM_, int WN_, int TMW_, int CK_>
struct DConvCfg {
  static constexpr int WM = WM_, WN = WN_, TMW = TMW_, NW = WM * WN, NT = 64 * NW;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static constexpr int CI = Pr::CI, CO = Pr::CO, KH = Pr::KH, KW = Pr::KW, H = Pr::H, W = Pr::W, S = Pr::S;
  static constexpr int OH = Pr::OH, OW = Pr::OW;  // (input H x W, output OH x OW, stride S)
  static constexpr int QT = CI / 4;  // channel quads per tap
  static_assert(CI % 4 == 0, "channel quads");
  static constexpr int TAPS = KH * KW;
  static constexpr int KP = (Pr::KK + 15) / 16 * 16;  // K padded to whole 16-chunks (zero weights)
  static constexpr int KC = KP / 16;
  static constexpr int TN = CO / 16;
  static_assert(CO % 16 == 0 && TN % WN == 0, "N tiles");
  static constexpr int TNW = TN / WN;
  static constexpr int UPB = WM * TMW * 4;  // units per block
  static constexpr int PW = OW / 2;
  static constexpr int NPIX = OH * OW;
  static constexpr int U = Pr::POOL ? (OH / 2) * PW : (NPIX + 3) / 4;  // units per image
  static constexpr int BPI = (U + UPB - 1) / UPB;                       // blocks per image
  // output rows a block's units can touch, and the input rows / columns of its patch
  static constexpr int RSPAN0 = Pr::POOL ? 2 * ((UPB - 1) / PW + 2) : (4 * UPB - 1) / OW + 2;
  static constexpr int RSPAN = RSPAN0 < OH ? RSPAN0 : OH;
  static constexpr int RIN = (RSPAN - 1) * S + KH;
  static constexpr int WP = (OW - 1) * S + KW;                          // patch columns staged
  static constexpr int CS = dconv_cs(CI);                             // floats per patch pixel
  static constexpr int WPX = WP;                                        // patch row stride (pixels)
  static constexpr int ASZ = (RIN * WPX * CS + 3) / 4 * 4;
  static constexpr int CK = CK_ > 0 ? CK_ : KP;  // k per weight chunk
  static_assert(CK % 16 == 0, "chunk of whole 16-k steps");
  static constexpr bool TAPALIGNED = QT % 4 == 0 && CK % CI == 0;
  static_assert(TAPALIGNED || CK == KP, "a chunk that is not tap-aligned must hold the whole K");
  static constexpr int TPC = TAPALIGNED ? CK / CI : 0;  // taps per chunk
  static constexpr int CKC = CK / 16;
  static constexpr int NCH = KC / CKC;
  static_assert(NCH * CKC == KC, "whole chunks");
  static constexpr int BSZ = CKC * TN * 256;  // floats per staged weight chunk
  static constexpr int NBUF = NCH > 1 ? 2 : 1;
  static constexpr size_t LDS = (size_t)(ASZ + NBUF * BSZ) * 4;
  static constexpr int BITEMS = (CK / 4) * CO;  // (k quad, column) items of one chunk
  static constexpr int BIT = (BITEMS + NT - 1) / NT;
  static constexpr int AQ = RIN * WP * QT;  // patch channel quads
  static constexpr int AIT = (AQ + NT - 1) / NT;
};

// Tiles [t0, t1) of problem p, one after the other (a tile = UPB units of one image); smem =
// D::LDS bytes of dynamic LDS. With the whole K in one chunk (NCH = 1) the weights are staged once
// for all of them (the persistent launch, dconv_kernel); otherwise t1 = t0 + 1.
template <class Pr, int WM, int WN, int TMW, int CK>
__device__ __forceinline__ void dconv_body(const Pr &p, int t0, int t1, float *smem) {
  using D = DConvCfg<Pr, WM, WN, TMW, CK>;
  float *As = smem;
  float *Bs = smem + D::ASZ;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int r = lane & 15, g = lane >> 4;

  // weight chunk c -> registers, and into LDS in fragment order [kc][n-tile][lane = 16 g + r][s]
  // (chunked weights: two chunks in flight in registers — chunk c + 2's loads are issued before
  // chunk c is multiplied, so a chunk's L2 round trip spans two chunks' MFMAs, not one)
  f32x4 wr[D::BIT], wr2[D::NCH > 1 ? D::BIT : 1];
  // (no branches: a thread past the chunk's items loads and stores the last item again — the same
  // value to the same address — so the waits before these loads and stores count outstanding
  // loads instead of draining them at an exec-mask join)
  auto wload_to = [&](int c, f32x4 *dstr) {
#pragma unroll
    for (int it = 0; it < D::BIT; ++it) {
      const int item = min(tid + it * D::NT, D::BITEMS - 1);
      const int kq = item / D::CO, n = item - kq * D::CO;
      dstr[it] = p.wquad(c * D::CK + 4 * kq, n);
    }
  };
  auto wload = [&](int c) { wload_to(c, wr); };
  auto wstore_from = [&](float *dst, const f32x4 *srcr) {
#pragma unroll
    for (int it = 0; it < D::BIT; ++it) {
      const int item = min(tid + it * D::NT, D::BITEMS - 1);
      const int kq = item / D::CO, n = item - kq * D::CO;
      const int kcl = kq >> 2, gg = kq & 3, j = n >> 4, rr = n & 15;
      *reinterpret_cast<f32x4 *>(dst + ((kcl * D::TN + j) * 64 + gg * 16 + rr) * 4) = srcr[it];
    }
  };
  auto wstore = [&](float *dst) { wstore_from(dst, wr); };
  // A offsets of the k-chunks (one chunk: K not tap-aligned, small CI): tap and channel quad of
  // quad index 4 kc + g (past the last tap: any tap, its weights are zero)
  int aoffs[D::TAPALIGNED ? 1 : D::KC];
  if constexpr (!D::TAPALIGNED) {
#pragma unroll
    for (int kc = 0; kc < D::KC; ++kc) {
      const int q4 = 4 * kc + g, t0q = q4 / D::QT, cq = q4 - t0q * D::QT;
      const int t = min(t0q, D::TAPS - 1), ky = t / D::KW, kx = t - ky * D::KW;
      aoffs[kc] = (ky * D::WPX + kx) * D::CS + 4 * cq;
    }
  }
  wload(0);
  if constexpr (D::NCH > 1) {
    wload_to(1, wr2);
    t1 = t0 + 1;  // (chunked weights: one tile per block, no loop)
  }
  for (int bid = t0; bid < t1; ++bid) {
  const int b = bid / D::BPI;
  const int u0 = (bid - b * D::BPI) * D::UPB;
  const int oy0 = Pr::POOL ? 2 * (u0 / D::PW) : (4 * u0) / D::OW;  // output row of patch row 0
  if (bid > t0) __syncthreads();  // the previous tile's LDS reads are done
  // epilogue operands (bias; or the pooled values + argmax of the unpool) issued up front
  typename Pr::Pre pre[TMW][D::TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < D::TNW; ++j)
      pre[i][j] = p.pre(b, min(u0 + (wm * TMW + i) * 4 + g, D::U - 1), (wn * D::TNW + j) * 16 + r);

  if constexpr (HasStagePatch<Pr>::value) {
    // (the problem stages its own patch: DFwdStack; rows [oy0 S, own_end) of the new state are the
    // block's to write — up to the next block's first row)
    const int bi = bid - b * D::BPI;
    const int own_end = bi + 1 < D::BPI ? min(D::H, ((4 * (u0 + D::UPB)) / D::OW) * D::S) : D::H;
    p.template stage_patch<D>(b, oy0 * D::S, own_end, As, reinterpret_cast<uint8_t *>(Bs));
  } else {
  // the patch: input rows oy0 - PT .. oy0 - PT + RIN - 1, columns -PL .. -PL + WP - 1 (zeros
  // outside the image), in batches of 8 quads per thread (all loads of a batch in flight)
  const auto *img = p.X + (size_t)b * D::H * D::W * D::CI;
  constexpr int ABATCH = 8;
#pragma unroll
  for (int it0 = 0; it0 < D::AIT; it0 += ABATCH) {
    f32x4 v[ABATCH];
    int dst[ABATCH];
#pragma unroll
    for (int t = 0; t < ABATCH; ++t) {
      const int it = it0 + t;
      if (it < D::AIT) {
        const int item = min(tid + it * D::NT, D::AQ - 1);
        const int pix = item / D::QT, cq = item - pix * D::QT;
        const int pr = pix / D::WP, pc = pix - pr * D::WP;
        const int iy = oy0 * D::S - Pr::PT + pr, ix = pc - Pr::PL;
        const bool ok = (unsigned)iy < (unsigned)D::H && (unsigned)ix < (unsigned)D::W;
        const f32x4 x = p.load4(img + (size_t)(ok ? iy * D::W + ix : 0) * D::CI + 4 * cq);
        v[t] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
        dst[t] = (D::AQ % D::NT == 0 || tid + it * D::NT < D::AQ) ? (pr * D::WPX + pc) * D::CS + 4 * cq : -1;
      }
    }
#pragma unroll
    for (int t = 0; t < ABATCH; ++t)
      if (it0 + t < D::AIT && dst[t] >= 0) *reinterpret_cast<f32x4 *>(As + dst[t]) = v[t];
  }
  }

  // lane A bases: row r of M-tile i = unit (wave's tile i, r / 4), window / quad position r % 4
  int abase[TMW];
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    const int u = min(u0 + (wm * TMW + i) * 4 + (r >> 2), D::U - 1);  // (tail units: clamped, not stored)
    const int q = r & 3;
    int oy, ox;
    if constexpr (Pr::POOL) {
      const int py = u / D::PW;
      oy = 2 * py + (q >> 1);
      ox = 2 * (u - py * D::PW) + (q & 1);
    } else {
      const int px = min(4 * u + q, D::NPIX - 1);
      oy = px / D::OW;
      ox = px - oy * D::OW;
    }
    abase[i] = ((oy - oy0) * D::S * D::WPX + ox * D::S) * D::CS;
  }
  f32x4 acc[TMW][D::TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < D::TNW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const float *Bc, int c) {
#pragma unroll
    for (int kcl = 0; kcl < D::CKC; ++kcl) {
      int ao;
      if constexpr (D::TAPALIGNED) {  // tap t (wave-uniform) and channel quad (4 kcl) % QT + g
        const int t = c * D::TPC + (4 * kcl) / D::QT;
        ao = ((t / D::KW) * D::WPX + t % D::KW) * D::CS + 4 * ((4 * kcl) % D::QT) + 4 * g;
      } else {
        ao = aoffs[kcl];
      }
      f32x4 a[TMW], bb[D::TNW];
#pragma unroll
      for (int i = 0; i < TMW; ++i) a[i] = *reinterpret_cast<const f32x4 *>(As + abase[i] + ao);
#pragma unroll
      for (int j = 0; j < D::TNW; ++j)
        bb[j] = *reinterpret_cast<const f32x4 *>(Bc + ((kcl * D::TN + wn * D::TNW + j) * 64 + lane) * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
          for (int j = 0; j < D::TNW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], bb[j][s], acc[i][j], 0, 0, 0);
    }
  };

  if (D::NCH > 1 || bid == t0) wstore(Bs);
  __syncthreads();
  if constexpr (D::NCH == 1) {
    compute(Bs, 0);
  } else {
    // LDS buffer c & 1 holds chunk c; registers: wr = chunk c + 2 (even c), wr2 = chunk c + 1 / c + 3.
    // One barrier per chunk: buffer (c + 1) & 1 was last read by chunk c - 1, before the last barrier.
    // (sched_barrier: keeps each chunk's loads at the top of its iteration; the scheduler otherwise
    // sinks them below the MFMAs, to just before the barrier, and the next store waits them out)
    for (int c = 0; c < D::NCH; c += 2) {
      if (c + 2 < D::NCH) wload_to(c + 2, wr);
      __builtin_amdgcn_sched_barrier(0);
      compute(Bs, c);
      if (c + 1 >= D::NCH) break;
      wstore_from(Bs + D::BSZ, wr2);
      __syncthreads();
      if (c + 3 < D::NCH) wload_to(c + 3, wr2);
      __builtin_amdgcn_sched_barrier(0);
      compute(Bs + D::BSZ, c + 1);
      if (c + 2 >= D::NCH) break;
      wstore_from(Bs, wr);
      __syncthreads();
    }
  }

  // epilogue: lane (r, g) holds rows 4 g .. 4 g + 3 (unit g of the tile) of column r
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    const int u = u0 + (wm * TMW + i) * 4 + g;
    if (u >= D::U) continue;
#pragma unroll
    for (int j = 0; j < D::TNW; ++j) p.store(pre[i][j], b, u, (wn * D::TNW + j) * 16 + r, acc[i][j]);
  }
  }
}

// ntiles > gridDim.x (persistent, NCH = 1): block k runs the contiguous tiles [k T / G, (k+1) T / G)
// — an image's neighbouring tiles share their patch rows in the CU's caches. Otherwise one tile
// per block, XCD-aware (an XCD takes a contiguous run of blocks, so the overlapping patches of
// one image's blocks are fetched into one L2).
template <class Pr, int WM, int WN, int TMW, int CK>
__global__ __launch_bounds__(64 * WM * WN) void dconv_kernel(Pr p, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int G = gridDim.x;
  if (ntiles > G) {
    const int t0 = (int)((long)blockIdx.x * ntiles / G), t1 = (int)((long)(blockIdx.x + 1) * ntiles / G);
    dconv_body<Pr, WM, WN, TMW, CK>(p, t0, t1, smem);
  } else {
    const int t = xcd_tile(blockIdx.x, G);
    dconv_body<Pr, WM, WN, TMW, CK>(p, t, t + 1, smem);
  }
}

template <class Pr, int WM, int WN, int TMW, int CK>
static int launch_dconv(const Pr &p, int B, hipStream_t s) {
  using D = DConvCfg<Pr, WM, WN, TMW, CK>;
  static_assert(D::LDS <= 160 * 1024, "LDS budget");
  if (B <= 0 || !launch_allowed()) return MT_OK;
  auto kern = &dconv_kernel<Pr, WM, WN, TMW, CK>;
  static bool attr_set = false;
  if (!attr_set && D::LDS > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)D::LDS));
    attr_set = true;
  }
  const int ntiles = B * D::BPI;
  hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(D::NT), D::LDS, s, p, ntiles);
  MT_LAUNCHED();
  return MT_OK;
}

// ---- tile choice per layer shape (PWYX E = 32 frames: conv1 1,792 blocks, conv2 448, conv3 224,
// conv4 128) ----------------------------------------------------------------------------------
//  conv1 (CIN 4 / 12, the whole K in one chunk): 4 waves, 2 M-tiles per wave (8-wave blocks measured
//    no faster); the strided NATURE conv1 1 M-tile;
//  conv2 (32 -> 32): 8-wave blocks, two blocks per CU: four waves per SIMD hide the per-chunk
//    barrier (PWYX-RGB E=32 33.4 vs 36.7 us, LSTM 161 frames 143.6 vs 157.5 us, profiles/r03i); one
//    M-tile x both N-tiles per wave (round 6: the A fragment read once for two accumulators; LSTM
//    trunk 72.5 -> 71.1 us against 4 x 2 waves of 2 M-tiles x 1 N-tile, profiles/r06fwd — the same
//    8 x 1 layout on the 64-channel layers measured 4-17 % slower); one tap (CIN k) per weight chunk
//    (5-tap chunks: no faster);
//  64 output channels (conv3, conv4, NATURE conv2 / conv3): 8-wave blocks for the pooled conv3
//    (18.2 -> 15.3 us), 1 M-tile per wave; the unpooled conv4 (10 x 10 outputs) on 4 waves of one
//    M-tile x one N-tile, 4 units a block — twice the blocks of the 8-wave form, which round 3
//    preferred over the 4-wave 2 x 2 one (11.0 -> 10.1 us): LSTM trunk 71.0 -> 69.4 us, PWYX-RGB
//    113.4 -> 111.9 us (profiles/r06fwd64; smaller conv3 tiles measured 5-14 % slower).
template <class G, bool POOL>
struct DConvFor {
  static constexpr bool SMALLC = G::CIN % 16 != 0;  // conv1: the whole K in one chunk
  static constexpr bool C64 = G::COUT >= 64;
  static constexpr int WN = C64 ? (POOL ? 2 : 4) : 1;
  static constexpr int WM = C64 ? (POOL ? 4 : 1) : (SMALLC ? 4 : 8);
  static constexpr int TMW = SMALLC ? (G::S > 1 ? 1 : 2) : 1;
  // weight chunk: one tap for the 5x5 layers; 4 / 3 taps for the 4x4 / 3x3 ones (one tap left their
  // blocks 16 / 9 chunk steps of 16-32 MFMAs per wave, each behind a barrier)
  static constexpr int CK = SMALLC ? 0 : G::CIN * (G::KH == 4 ? 4 : G::KH == 3 ? 3 : 1);
};

template <class G, bool U8, bool POOL>
static int conv_forward_direct(const void *X, const float *W, const float *bias, float *Y, uint8_t *arg, int B,
                               int act, float alpha, hipStream_t s) {
  using F = DConvFor<G, POOL>;
  using Pr = DFwd<G, U8, POOL>;
  const Pr p{reinterpret_cast<const typename Pr::InT *>(X), W, bias, Y, arg, act, alpha};
  return launch_dconv<Pr, F::WM, F::WN, F::TMW, F::CK>(p, B, s);
}

// ---- the NATURE rollout chain's trunk as one dataflow launch ----------------------------------
// conv1 (DFwdStack: each env's blocks wait for its publication), conv2 and conv3 of every env in ONE
// grid: blocks [0, n1) are conv1 tiles, [n1, n1 + n2) conv2 tiles, then conv3, each role env-major.
// A conv2 block of env e starts once env e's conv1 blocks have stored their activations (a per-env
// counter), a conv3 block once env e's conv2 blocks have: env e's whole trunk runs while the
// emulators still step the later envs, instead of conv2 / conv3 waiting behind the LAST env's
// conv1 at two kernel boundaries. Deadlock-free: a block waits only for lower-indexed blocks (or
// the host), and each XCD dispatches its workgroups in index order, so the lowest unfinished block
// is always resident. The hand-off is tools/handoff_probe.hip's (0 stale of 200 launches):
// activations stored and loaded with agent-scope (sc1) accesses (DFwd COH_OUT / COH_IN), every
// wave's stores retired (vmcnt(0)) before the block barrier, then one relaxed agent-scope
// increment; a consumer's lane 0 polls the counter (s_sleep; bounded ~2 s -> status, then it
// proceeds: the host reports the error). The last conv3 block of env e resets env e's counters for
// the next launch.
// Tiles: 4 waves for every role (conv2 / conv3: 4 N-tiles of one 16-row M-tile, 4 units a block,
// so one env's conv2 spreads over 6 blocks and its conv3 over 4).
// conv2 / conv3 tiles of the chain: 1 M-tile x 4 N-tiles on 4 waves (chain_conv_tile)
template <class Pr>
using ChainCfg = DConvCfg<Pr, 1, 4, 1, Pr::CI>;

constexpr int kChainSyncWords = 96;  // nature_chain_kernel's counter words per env

template <class G1_, class G2_, class G3_>
struct NatureChain {
  using G1 = G1_;
  using G2 = G2_;
  using G3 = G3_;
  using P1 = DFwdStack<G1, true>;
  using P2 = DFwd<G2, false, false, true, true>;
  using P3 = DFwd<G3, false, false, true, false>;
  using D1 = DConvCfg<P1, 4, 1, 1, 0>;
  using D2 = ChainCfg<P2>;
  using D3 = ChainCfg<P3>;
  // (every role keeps its weights in registers: only the patches in LDS, + conv1's stacked frames)
  static constexpr size_t LDS =
      std::max((size_t)D1::ASZ * 4 + 4 * D1::RIN * G1::W, (size_t)std::max(D2::ASZ, D3::ASZ) * 4);
  static_assert(D1::NT == 256 && D2::NT == 256 && D3::NT == 256, "one block size for every role");
  static constexpr int BPE = D1::BPI + D2::BPI + D3::BPI;  // blocks per env
  // per env: conv1 / conv2 / conv3 done, each counter on its own 128-B line (words 0 / 32 / 64) —
  // polled lines shared by several envs delay the producers' increments (stack_conv1_kernel)
  static constexpr int SYNC_WORDS = kChainSyncWords, C2 = 32, C3 = 64;
};

__device__ __forceinline__ void chain_signal(uint32_t *c, uint32_t last, int e, int phase) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's (sc1) stores have completed
  __syncthreads();
  MT_PROBE_BLK(4);
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == last) MT_PROBE_CHAIN(e, phase);
    (void)old;
  }
}
__device__ __forceinline__ void chain_wait(const uint32_t *c, uint32_t want, uint32_t *status) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
        if (status) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
}

// A conv2 / conv3 tile of the chain kernel with its weights in registers: 4 waves, wave w owns
// N-tile w (16 output channels) over the WHOLE K, its KC B fragments loaded by the caller before
// the hand-off wait (so their latency hides under it), one M-tile (4 units) per block. The generic
// body stages the weights in LDS tap by tap, one barrier and one global round trip per tap: 16
// (conv2) / 9 (conv3) of them on the per-env critical path, 4-5 us of the 5-6 us a block took.
template <class Pr>
__device__ __forceinline__ void chain_load_b(const Pr &p, f32x4 (&bf)[ChainCfg<Pr>::KC]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kc = 0; kc < ChainCfg<Pr>::KC; ++kc) bf[kc] = p.wquad(16 * kc + 4 * g, 16 * w + r);
}
template <class Pr>
__device__ __forceinline__ void chain_conv_tile(const Pr &p, int t, float *As, const f32x4 (&bf)[ChainCfg<Pr>::KC]) {
  using D = ChainCfg<Pr>;
  static_assert(D::TN == 4 && D::UPB == 4, "one M-tile x 4 N-tiles per block");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, g = lane >> 4;
  const int b = t / D::BPI;
  const int u0 = (t - b * D::BPI) * D::UPB;
  const int oy0 = (4 * u0) / D::OW;  // output row of patch row 0
  const typename Pr::Pre pre = p.pre(b, min(u0 + g, D::U - 1), 16 * w + r);
  // the patch (rows oy0 - PT .., zeros outside the image), as dconv_body stages it
  const auto *img = p.X + (size_t)b * D::H * D::W * D::CI;
  constexpr int ABATCH = 8;
#pragma unroll
  for (int it0 = 0; it0 < D::AIT; it0 += ABATCH) {
    f32x4 v[ABATCH];
    int dst[ABATCH];
#pragma unroll
    for (int q = 0; q < ABATCH; ++q) {
      const int it = it0 + q;
      if (it < D::AIT) {
        const int item = min(tid + it * D::NT, D::AQ - 1);
        const int pix = item / D::QT, cq = item - pix * D::QT;
        const int pr = pix / D::WP, pc = pix - pr * D::WP;
        const int iy = oy0 * D::S - Pr::PT + pr, ix = pc - Pr::PL;
        const bool ok = (unsigned)iy < (unsigned)D::H && (unsigned)ix < (unsigned)D::W;
        const f32x4 x = p.load4(img + (size_t)(ok ? iy * D::W + ix : 0) * D::CI + 4 * cq);
        v[q] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
        dst[q] = (D::AQ % D::NT == 0 || tid + it * D::NT < D::AQ) ? (pr * D::WPX + pc) * D::CS + 4 * cq : -1;
      }
    }
#pragma unroll
    for (int q = 0; q < ABATCH; ++q)
      if (it0 + q < D::AIT && dst[q] >= 0) *reinterpret_cast<f32x4 *>(As + dst[q]) = v[q];
  }
  // lane A base: row r of the M-tile = unit r / 4, quad position r % 4
  int abase;
  {
    const int u = min(u0 + (r >> 2), D::U - 1);
    const int px = min(4 * u + (r & 3), D::NPIX - 1);
    const int oy = px / D::OW, ox = px - oy * D::OW;
    abase = ((oy - oy0) * D::S * D::WPX + ox * D::S) * D::CS;
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < D::KC; ++kc) {
    const int q4 = 4 * kc + g, tap = q4 / D::QT, cq = q4 - tap * D::QT;  // channel quad cq of tap `tap`
    const int tp = min(tap, D::TAPS - 1);
    const f32x4 a = *reinterpret_cast<const f32x4 *>(As + abase + ((tp / D::KW) * D::WPX + tp % D::KW) * D::CS + 4 * cq);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s4], bf[kc][s4], acc, 0, 0, 0);
  }
  if (u0 + g < D::U) p.store(pre, b, u0 + g, 16 * w + r, acc);
}

// The chain's conv1 tile (DFwdStack's staging) with its weights in registers too: 4 waves, wave w
// owns M-tile w (4 units) and both 16-channel N-tiles over the whole K (KC x 2 B fragments, loaded
// before the publication wait): no weight staging in LDS, no barrier behind the patch. fr: the
// stacked frames' scratch, after the patch.
template <class NC>
__device__ __forceinline__ void chain_conv1_tile(const typename NC::P1 &p, int t, float *As,
                                                 const f32x4 (&bf)[2][NC::D1::KC]) {
  using D = typename NC::D1;
  using Pr = typename NC::P1;
  static_assert(D::WM == 4 && D::WN == 1 && D::TN == 2 && D::UPB == 16 && !D::TAPALIGNED, "conv1 tiling");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, g = lane >> 4;
  const int b = t / D::BPI, bi = t - b * D::BPI;
  const int u0 = bi * D::UPB;
  const int oy0 = (4 * u0) / D::OW;
  typename Pr::Pre pre[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) pre[j] = p.pre(b, min(u0 + 4 * w + g, D::U - 1), 16 * j + r);
  const int own_end = bi + 1 < D::BPI ? min(D::H, ((4 * (u0 + D::UPB)) / D::OW) * D::S) : D::H;
  p.template stage_patch<D>(b, oy0 * D::S, own_end, As, reinterpret_cast<uint8_t *>(As + D::ASZ));
  int abase;
  {
    const int u = min(u0 + 4 * w + (r >> 2), D::U - 1);
    const int px = min(4 * u + (r & 3), D::NPIX - 1);
    const int oy = px / D::OW, ox = px - oy * D::OW;
    abase = ((oy - oy0) * D::S * D::WPX + ox * D::S) * D::CS;
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int kc = 0; kc < D::KC; ++kc) {
    const int q4 = 4 * kc + g, tap = min(q4 / D::QT, D::TAPS - 1), cq = q4 - (q4 / D::QT) * D::QT;
    const f32x4 a = *reinterpret_cast<const f32x4 *>(As + abase + ((tap / D::KW) * D::WPX + tap % D::KW) * D::CS + 4 * cq);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s4], bf[j][kc][s4], acc[j], 0, 0, 0);
  }
  if (u0 + 4 * w + g < D::U) {
#pragma unroll
    for (int j = 0; j < 2; ++j) p.store(pre[j], b, u0 + 4 * w + g, 16 * j + r, acc[j]);
  }
}

// The conv roles of block bid < E * NC::BPE.
template <class NC>
__device__ __forceinline__ void nature_conv_roles(const typename NC::P1 &p1, const typename NC::P2 &p2,
                                                  const typename NC::P3 &p3, uint32_t *sync, int E, uint32_t *status,
                                                  int bid, float *smem) {
  using D1 = typename NC::D1;
  using D2 = typename NC::D2;
  using D3 = typename NC::D3;
  const int n1 = E * D1::BPI, n2 = E * D2::BPI;
  MT_PROBE_BLK(0);
  if (bid < n1) {
    const int t = xcd_tile(bid, n1);  // (an env's conv1 tiles on one XCD: their patch rows overlap)
    f32x4 bf[2][D1::KC];
    {
      const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kc = 0; kc < D1::KC; ++kc) bf[j][kc] = p1.wquad(16 * kc + 4 * g, 16 * j + r);
    }
    chain_conv1_tile<NC>(p1, t, smem, bf);
    MT_PROBE_BLK(3);
    chain_signal(sync + NC::SYNC_WORDS * (t / D1::BPI), D1::BPI - 1, t / D1::BPI, 1);
  } else if (bid < n1 + n2) {
    const int t = bid - n1, e = t / D2::BPI;
    f32x4 bf[D2::KC];
    chain_load_b(p2, bf);
    chain_wait(sync + NC::SYNC_WORDS * e, D1::BPI, status);
    MT_PROBE_BLK(1);
    chain_conv_tile(p2, t, smem, bf);
    MT_PROBE_BLK(3);
    chain_signal(sync + NC::SYNC_WORDS * e + NC::C2, D2::BPI - 1, e, 2);
  } else {
    const int t = bid - n1 - n2, e = t / D3::BPI;
    uint32_t *c = sync + NC::SYNC_WORDS * e;
    f32x4 bf[D3::KC];
    chain_load_b(p3, bf);
    chain_wait(c + NC::C2, D2::BPI, status);
    MT_PROBE_BLK(1);
    chain_conv_tile(p3, t, smem, bf);
    MT_PROBE_BLK(3);
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(c + NC::C3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)D3::BPI - 1) {
      // env e's last conv3 block: reset env e's counters for the next launch. Every block adds to its
      // counter exactly once, timed out or not, so the conv1 / conv2 counters are reset by subtracting
      // their full counts rather than stored to zero: after a bounded wait timed out, a producer may
      // still add AFTER this point (its consumer stopped waiting first), and the word must still read
      // zero once the launch has drained. (C3's adds are all in: this block is the last.)
      MT_PROBE_CHAIN(e, 3);
      __hip_atomic_fetch_sub(c, (uint32_t)D1::BPI, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_sub(c + NC::C2, (uint32_t)D2::BPI, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c + NC::C3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


template <class NC>
__global__ __launch_bounds__(256) void nature_chain_kernel(typename NC::P1 p1, typename NC::P2 p2,
                                                           typename NC::P3 p3, uint32_t *sync, int E,
                                                           uint32_t *status) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  nature_conv_roles<NC>(p1, p2, p3, sync, E, status, blockIdx.x, smem);
}

template <class NC, class G1 = typename NC::G1, class G2 = typename NC::G2, class G3 = typename NC::G3>
static void nature_chain_params(const StackSrc &st, const float *W1, const float *W2, const float *W3, float *a1,
                                float *a2, float *a3, int act, float alpha, typename NC::P1 &p1, typename NC::P2 &p2,
                                typename NC::P3 &p3) {
  p1 = typename NC::P1{};
  p1.X = st.out;
  p1.Wt = W1;
  p1.bias = W1 + G1::KK * G1::COUT;
  p1.Y = a1;
  p1.act = act;
  p1.alpha = alpha;
  p1.st = st;
  p2 = typename NC::P2{a1, W2, W2 + G2::KK * G2::COUT, a2, nullptr, act, alpha};
  p3 = typename NC::P3{a2, W3, W3 + G3::KK * G3::COUT, a3, nullptr, act, alpha};
}

// The NATURE chain's trunk convs (stacking conv1 -> conv2 -> conv3) as one nature_chain_kernel
// launch. sync: NC::SYNC_WORDS * B zero-initialised words (left zero by every launch).
template <class G1, class G2, class G3>
static int launch_nature_chain(const StackSrc &st, const float *W1, const float *W2, const float *W3, float *a1,
                               float *a2, float *a3, int B, int act, float alpha, uint32_t *sync, hipStream_t s) {
  using NC = NatureChain<G1, G2, G3>;
  static_assert(NC::LDS <= 160 * 1024, "LDS budget");
  if (B <= 0 || !launch_allowed()) return MT_OK;
  typename NC::P1 p1;
  typename NC::P2 p2;
  typename NC::P3 p3;
  nature_chain_params<NC>(st, W1, W2, W3, a1, a2, a3, act, alpha, p1, p2, p3);
  auto kern = &nature_chain_kernel<NC>;
  static bool attr_set = false;
  if (!attr_set && NC::LDS > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)NC::LDS));
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(B * NC::BPE)), dim3(256), NC::LDS, s, p1, p2, p3, sync, B, st.status);
  MT_LAUNCHED();
  return MT_OK;
}

// ---- a frame trunk's rollout step: pull + stack + conv1 as one dataflow launch ----------------
// (round 4; the LSTM and PWYX rollouts, gray or RGB) Blocks [0, E * SPL): SPL per env (one 16-word
// item per thread: 2 gray, 6 RGB) — wait for env e's publication (StackSrc::ready), read its p
// pushes from the pinned staging (the edge lines of its slot group system-scope, ld_published16),
// stack them onto the previous state (preprocess_kernel's op: every state word = one colour
// channel's 4 frames, shifted by p bytes, the p new frame bytes on top), store the new state with
// agent-scope stores, drain, count one part of env e stacked. Blocks [E * SPL, .. + E * BPI): the
// trunk's conv1 tiles (DFwd, the same tiling and arithmetic as conv_forward_direct), env-major and
// XCD-aware; a tile of env e polls env e's word until its SPL parts are in, reads the state with
// agent-scope loads (COH_IN) and runs the conv1 body: the step's conv1 runs while the emulators
// still step later envs, instead of behind pull_frames_kernel -> preprocess_kernel -> conv1 after
// the LAST env. Every env's word has its own 128-B line: with the words packed (16 envs a line) the
// ~1,300 polling tiles delayed the env blocks' increments and the launch ended ~25 us after the
// last publication, no earlier than the layered conv1 (profiles/r04_ab). One block per env made
// the last env's stack a serial ~20 us (RGB) after its publication: SPL blocks share it.
// Deadlock-free as nature_chain_kernel (a tile waits only for stack blocks, all lower-indexed;
// bounded). sync = [tiles done][env e: line 1 + e] (32-word lines); the last tile resets every word
// for the next launch.
template <class G>
struct StackConv1 {
  using F = DConvFor<G, true>;
  using P1 = DFwd<G, true, true, true, false>;
  using D = DConvCfg<P1, F::WM, F::WN, F::TMW, F::CK>;
  static constexpr int DEPTH = G::CIN / 4;  // colour channels (1 gray, 3 RGB)
  static_assert(D::NT == 256 && (G::CIN == 4 || G::CIN == 12) && G::H == 84 && G::W == 84 && G::S == 1,
                "84x84 conv1 of 4 stacked frames, 4 waves");
  static constexpr int NI = 84 * 84 * DEPTH / 16;  // 16-word items per env: 441 gray, 1,323 RGB
  static constexpr int SPL = (NI + 255) / 256;     // stack blocks per env
  static constexpr size_t LDS = D::LDS;
  static_assert(LDS >= 256 * 17 * 4, "the stack blocks' word exchange fits the tiles' LDS");
};

// part `part` of env e's new state (84 x 84 x DEPTH words of 4 frames each): items part * 256 + tid,
// a 16-word item = one 16-B chunk of each push. The words go out through LDS (xs: 256 x 17 words)
// so that each store instruction writes 256 consecutive words: a thread's own 16 words, stored
// directly, put 4 B of every 64 B in each agent-scope store and wrote ~8x the state's bytes to HBM
// (PMC WRITE_SIZE 30 MB per PWYX-RGB launch for a 2.7 MB state + 9 MB of conv1 output).
template <int DEPTH>
__device__ __forceinline__ void frame_pull_stack(const StackSrc &st, int e, int part, uint32_t *sync, uint32_t *xs) {
  constexpr int NW = 84 * 84 * DEPTH, NI = NW / 16;
  static_assert(NW % 16 == 0, "whole 16-B frame chunks");
  const int tid = threadIdx.x;
  const int i = part * 256 + tid;
  const int ic = min(i, NI - 1);
  __shared__ int s_p;
  // the previous state's item requested before the wait (its latency hides under it)
  const uint4 *prev = reinterpret_cast<const uint4 *>(st.prev + (size_t)e * NW * 4);
  uint4 pv[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pv[c] = prev[4 * ic + c];
  if (tid == 0) {
    const uint32_t tag = st.tag_base ? ((*st.tag_base + st.tag) & 0x1fffffffu) : st.tag;
    s_p = min(max(wait_published(st.ready, e, tag, st.status), 0), 4);  // (a timeout stacks no frame)
    if (part == 0) MT_PROBE_CHAIN(e, 0);
  }
  __syncthreads();
  const int p = s_p;
  // push j of env e = frame slot 4e + j (NW bytes), its 16-B chunk i = state words 16 i .. 16 i + 15
  const size_t F = (size_t)NW, lo = 4 * (size_t)e * F, hi = lo + 4 * F;
  uint4 fv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    fv[j] = j < p ? ld_published16(st.frames, ((size_t)4 * e + j) * F + 16 * (size_t)ic, lo, hi)
                  : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int c = 0; c < 4; ++c) {  // words 16 i + 4 c .. + 3 -> xs[tid * 17 + 4 c + k] (stride 17: no bank conflicts)
    const uint32_t wv[4] = {pv[c].x, pv[c].y, pv[c].z, pv[c].w};
    uint32_t fw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[j] = c == 0 ? fv[j].x : c == 1 ? fv[j].y : c == 2 ? fv[j].z : fv[j].w;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t v = p < 4 ? wv[k] >> (8 * p) : 0u;
      for (int j = 0; j < p; ++j) v |= ((fw[j] >> (8 * k)) & 0xffu) << (8 * (4 - p + j));
      xs[tid * 17 + 4 * c + k] = v;
    }
  }
  __syncthreads();
  // word w = 256 q + tid of the part (item w / 16, word w % 16): one coalesced agent-scope store per q
  uint32_t *out = reinterpret_cast<uint32_t *>(st.out + (size_t)e * NW * 4) + 16 * (size_t)(part * 256);
  const int nw = 16 * min(256, NI - part * 256);  // the part's words
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int w = 256 * q + tid;
    if (w < nw) __hip_atomic_store(out + w, xs[(w >> 4) * 17 + (w & 15)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's (sc1) state stores have completed
  __syncthreads();
  if (tid == 0) {  // one part of env e stacked (its own 128-B line: see above)
    __hip_atomic_fetch_add(sync + 32 + 32 * e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    MT_PROBE_CHAIN(e, 1);
  }
}

template <class G>
__global__ __launch_bounds__(256) void stack_conv1_kernel(StackSrc st, typename StackConv1<G>::P1 p1, uint32_t *sync,
                                                          int E) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using C = StackConv1<G>;
  using D = typename C::D;
  const int nstk = E * C::SPL;
  if ((int)blockIdx.x < nstk) {
    frame_pull_stack<C::DEPTH>(st, (int)blockIdx.x / C::SPL, (int)blockIdx.x % C::SPL, sync,
                               reinterpret_cast<uint32_t *>(smem));
    return;
  }
  const int t = xcd_tile((int)blockIdx.x - nstk, E * D::BPI), b = t / D::BPI;  // (an env's tiles on one XCD)
  if (threadIdx.x == 0) {  // env b's SPL parts stacked (bounded wait, as chain_wait)
    const uint32_t *w = sync + 32 + 32 * b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)C::SPL) {
      __builtin_amdgcn_s_sleep(8);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
        if (st.status) __hip_atomic_store(st.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;  // (proceed; the host reports the error)
      }
    }
  }
  __syncthreads();
  dconv_body<typename C::P1, C::F::WM, C::F::WN, C::F::TMW, C::F::CK>(p1, t, t + 1, smem);
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(E * D::BPI) - 1) {
    // the last tile: reset the words for the next launch. The env words by subtracting SPL (each
    // stack block adds once): a stack block whose publication wait timed out may add after its tiles
    // stopped waiting, i.e. after this point, and the word must still read zero once the launch has
    // drained
    __hip_atomic_store(sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < E; ++k)
      __hip_atomic_fetch_sub(sync + 32 + 32 * k, (uint32_t)C::SPL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// pull + stack + conv1 of the E new frames of a rollout step: st->out = the new state rows, Y / arg =
// conv1's pooled output and argmax rows. sync: stack_conv1_sync_words(E) zeroed words.
template <class G>
static int launch_stack_conv1(const StackSrc &st, const float *W, float *Y, uint8_t *arg, int E, int act, float alpha,
                              uint32_t *sync, hipStream_t s) {
  using C = StackConv1<G>;
  static_assert(C::LDS <= 160 * 1024, "LDS budget");
  if (!st.ready || !st.prev || !st.frames || !st.out || !sync) {
    set_error("stacking conv1: ready words, previous / new state, staging and a counter region");
    return MT_ERR_ARG;
  }
  if (E <= 0 || !launch_allowed()) return MT_OK;
  auto kern = &stack_conv1_kernel<G>;
  static bool attr_set = false;
  if (!attr_set && C::LDS > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)C::LDS));
    attr_set = true;
  }
  const typename C::P1 p1{st.out, W, W + G::KK * G::COUT, Y, arg, act, alpha};
  hipLaunchKernelGGL(kern, dim3((unsigned)(E * C::SPL + E * C::D::BPI)), dim3(256), C::LDS, s, st, p1, sync, E);
  MT_LAUNCHED();
  return MT_OK;
}

// dX of stride-1 conv G unpooled into GJ's conv-output gradient: its own 8-wave launch ahead of the
// (weight-gradient) group, for the 5x5 32 -> 32 layer only (conv2: PWYX-RGB dX 147 + dW group 193 us
// vs 370 for the generic GEMM dX in the group, LSTM 257 + 367 vs 679, profiles/r03d/c5_*). Measured
// and not adopted: the direct dX as a 4-wave job of the grouped launch (its 54-88 KB patch sets the
// LDS of every block of the group, so the weight-gradient blocks beside it lose occupancy: 417 vs
// 370 us), and conv3's dX in its own launch (83 + 62 vs 123 us).
template <class G>
constexpr bool dconv_bwd_solo() {
  return G::KH == 5 && G::CIN == 32 && G::COUT == 32;
}

template <class G, class GJ>
static int conv_dgrad_unpool_solo(const float *dY, const float *Wt, const float *Pj, const uint8_t *argj, float *dactj,
                                  int B, int act, float alpha, hipStream_t s) {
  // 8 waves of one M-tile x both N-tiles (two accumulators per wave, the A fragment read once for
  // both): LSTM conv2 dX 257.1 -> 248.0 us against 4 x 2 waves of two M-tiles x one N-tile; 4 waves
  // of 2 x 2 tiles 256.6, 5-tap weight chunks 292.2 (profiles/r06dxc)
  return launch_dconv<DBwdUnpool<G, GJ>, 8, 1, 1, G::COUT>(DBwdUnpool<G, GJ>{dY, Wt, Pj, argj, dactj, act, alpha}, B,
                                                           s);
}

// ---- weight gradient ---------------------------------------------------------------------------
// dW (+ db) of a stride-1 SAME conv G as K-split slabs [S][KK + 1][COUT] (weight rows in HWIO
// order, then the bias row), summed by the caller's SlabJob exactly as the generic path's
// (conv_wgrad_jobs). GEMM view: M = KK rows (tap, ci), N = COUT, K = pixels.
// Block = (split sp, tap group tg): M-tiles [tg MPB, (tg + 1) MPB) over the split's pixel chunks.
// A chunk is 4 output rows of one image (x padded to a multiple of 4, zeros): its input patch
// (4 + KH - 1 rows, NHWC, u8 -> f32) and dY rows are staged in LDS; the next chunk's global loads
// are in flight (registers) while this one is multiplied. K order inside a 16-step kc = (row g of
// the chunk, x = 4 kc + s): lane (r, g) of M-tile m reads X[row g + ky][x + s + kx][ci] and
// dY[row g][x + s][co] — two LDS reads per MFMA-operand pair, each a ds_read_b32 at an immediate
// offset from a per-lane base (the (tap, ci) of row 16 m + r is decomposed once).
constexpr size_t kDwSlabCap = (size_t)8 << 20;  // slab floats (2x the generic path's kSlabFloats)

// Small-channel patches (conv1: 4 / 12 u8 channels): no channel pad (16-B pixel quads, one LDS store
// each) and the patch row stride padded instead, to the first whose offset puts lane group g = 1 on
// the other 16 banks — an A read of these M-tiles spans several taps of one row, so a channel pad
// cannot separate the groups (bank model of the A reads: 3.7 -> 2.9 LDS cycles per read gray, 3.9
// -> 2.3 RGB)
constexpr int dw_row_stride(int cs, int wp) {
  int w = wp;
  while ((w * cs) % 32 != 16) ++w;
  return w;
}

constexpr int dw_pad(int c, int wd) {  // channel stride whose row stride wd * cs puts lane group g = 1
  int best = c, bd = 99;               // on the other 16 banks (|(wd cs) % 32 - 16| smallest)
  for (int p = 0; p < 16; ++p) {
    const int d = (wd * (c + p)) % 32, e = d > 16 ? d - 16 : 16 - d;
    if (e < bd) {
      bd = e;
      best = c + p;
    }
  }
  return best;
}

template <class G, bool U8, int TMW_>
struct DWCfg {
  static_assert((G::S == 1 && G::SAME) || !G::SAME, "stride-1 SAME or VALID conv");
  using Geom = G;
  static constexpr int CIN = G::CIN, COUT = G::COUT, KH = G::KH, KW = G::KW, H = G::H, W = G::W, S = G::S;
  static constexpr int OH = G::OH, OW = G::OW;  // (input H x W, output OH x OW)
  static constexpr int KK = G::KK, TMW = TMW_;
  static constexpr int TN = COUT / 16;
  static_assert(COUT % 16 == 0 && 4 % TN == 0, "N tiles per 4 waves");
  static constexpr int WROWS = 4 / TN;  // wave rows (M sets) per block
  static constexpr int MPB = TMW * WROWS;
  static constexpr int MT = (KK + 15) / 16;
  static constexpr int TG = (MT + MPB - 1) / MPB;  // tap groups
  static constexpr int R = 4;                      // output rows per chunk (= lane groups g)
  static constexpr int RG = (OH + R - 1) / R;      // chunks per image
  static constexpr int WPAD = (OW + 3) / 4 * 4;    // output columns, padded
  static constexpr int KQ = WPAD / 4;              // 16-k steps per chunk
  static constexpr int WP = (WPAD - 1) * S + KW;   // patch columns
  static constexpr int RIN = (R - 1) * S + KH;     // patch rows
  static constexpr bool SMALLC = CIN < 16 && CIN % 4 == 0 && S == 1;
  static constexpr int CS = SMALLC ? CIN : dw_pad(CIN, S * WP), COS = dw_pad(COUT, WPAD);
  static constexpr int WPX = SMALLC ? dw_row_stride(CS, WP) : WP;  // patch row stride (pixels)
  static constexpr int XSZ = (RIN * WPX * CS + 3) / 4 * 4, YSZ = R * WPAD * COS;
  static constexpr size_t LDS = (size_t)(XSZ + YSZ) * 4;
  static constexpr int XQ = RIN * WP * (CIN / 4), YQ = R * WPAD * (COUT / 4);  // quads per chunk
  static constexpr int XIT = (XQ + 255) / 256, YIT = (YQ + 255) / 256;
  static constexpr size_t SLAB = (size_t)(KK + 1) * COUT;
  // Row-mapped staging (ROWMAP): wave w stages patch rows w, w + 4, ... and dY row w of a chunk; lane
  // l takes the row's quads l + 64 k, so its pixel (l / CQ + k PXK) and channel quad (l % CQ) are
  // fixed for the whole job: the global offsets are computed once, row validity is wave-uniform (a
  // zero-length buffer descriptor) and out-of-image columns read zero through the descriptor's range
  // check (offset 0x80000000). Per chunk a quad costs its load and its LDS store, nothing else.
  // (LUX lanes of a wave take patch quads: 63 for the RGB conv1's 3 quads per pixel, lane 63 idle)
  static constexpr int CQ = CIN / 4, CQO = COUT / 4;
  static constexpr bool ROWMAP = S == 1 && G::SAME && RIN % 4 == 0 && CQ <= 16 && 64 % CQO == 0;
  static constexpr int LUX = 64 - 64 % CQ;
  static constexpr int XROWS = RIN / 4, QRX = WP * CQ, KX = (QRX + LUX - 1) / LUX, PXK = LUX / CQ;
  static constexpr int QRY = WPAD * CQO, KY = (QRY + 63) / 64, PYK = 64 / CQO;
  // k steps whose every lane is inside the image and the row (one shared offset + k stride)
  static constexpr bool x_inner(int k) { return k * PXK >= G::PL && (k + 1) * PXK <= G::PL + W && (k + 1) * LUX <= QRX; }
  static constexpr bool y_inner(int k) { return (k + 1) * PYK <= OW && (k + 1) * 64 <= QRY; }
};

// Item-mapped chunk staging of DWgradJob (any layer): thread t stages items t, t + 256, ... of the
// chunk's flat (pixel, channel quad) lists, each decomposed per chunk.
template <class D, bool U8>
struct DwItemStage {
  using G = typename D::Geom;
  using InT = typename InElem<U8>::T;
  const InT *X;
  const float *dY;
  float *Xs, *Ys;
  f32x4 xr[D::XIT], yr[D::YIT];
  __device__ DwItemStage(const InT *X_, const float *dY_, float *Xs_, float *Ys_) : X(X_), dY(dY_), Xs(Xs_), Ys(Ys_) {}
  __device__ __forceinline__ void load(int c) {
    const int tid = threadIdx.x;
    const int b = c / D::RG, y0 = (c - b * D::RG) * D::R;
    const InT *xi = X + (size_t)b * D::H * D::W * D::CIN;
    const float *yi = dY + (size_t)b * D::OH * D::OW * D::COUT;
#pragma unroll
    for (int it = 0; it < D::XIT; ++it) {
      const int item = min(tid + 256 * it, D::XQ - 1);
      const int pix = item / (D::CIN / 4), cq = item - pix * (D::CIN / 4);
      const int pr = pix / D::WP, pc = pix - pr * D::WP;
      const int iy = y0 * D::S - G::PT + pr, ix = pc - G::PL;
      const bool ok = (unsigned)iy < (unsigned)D::H && (unsigned)ix < (unsigned)D::W;
      const f32x4 v = InElem<U8>::load4(xi + (size_t)(ok ? iy * D::W + ix : 0) * D::CIN + 4 * cq);
      xr[it] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int it = 0; it < D::YIT; ++it) {
      const int item = min(tid + 256 * it, D::YQ - 1);
      const int pix = item / (D::COUT / 4), cq = item - pix * (D::COUT / 4);
      const int pr = pix / D::WPAD, pc = pix - pr * D::WPAD;
      const int oy = y0 + pr;
      const bool ok = oy < D::OH && pc < D::OW;
      const f32x4 v = *reinterpret_cast<const f32x4 *>(yi + (size_t)(ok ? oy * D::OW + pc : 0) * D::COUT + 4 * cq);
      yr[it] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void store() {
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < D::XIT; ++it) {
      const int item = tid + 256 * it;
      if (D::XQ % 256 == 0 || item < D::XQ) {
        const int pix = item / (D::CIN / 4), cq = item - pix * (D::CIN / 4);
        const int pr = pix / D::WP, pc = pix - pr * D::WP;
        float *d = Xs + (pr * D::WPX + pc) * D::CS + 4 * cq;
        if constexpr (D::CS % 4 == 0) {
          *reinterpret_cast<f32x4 *>(d) = xr[it];
        } else {  // (four dword stores)
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = xr[it][e];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < D::YIT; ++it) {
      const int item = tid + 256 * it;
      if (D::YQ % 256 == 0 || item < D::YQ) {
        const int pix = item / (D::COUT / 4), cq = item - pix * (D::COUT / 4);
        float *d = Ys + pix * D::COS + 4 * cq;
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = yr[it][e];
      }
    }
  }
};

// Row-mapped chunk staging (DWCfg::ROWMAP): wave w stages patch rows w + 4 h and dY row w; every
// per-lane offset is computed once in the constructor.
template <class D, bool U8>
struct DwRowStage {
  using G = typename D::Geom;
  using InT = typename InElem<U8>::T;
  using XV = typename std::conditional<U8, uint32_t, f32x4>::type;  // (u8: the raw 4 bytes until the store)
  static constexpr uint32_t kOut = 0x80000000u;                     // an offset past any range: reads zero
  static constexpr int kRsrc3 = 0x00020000;                         // gfx9 raw buffer: 32-bit data format
  // the first inner k step of the patch / dY rows (-1: none); inner k = its offset + (k - K0) strides
  static constexpr int XK0 = [] { for (int k = 0; k < D::KX; ++k) if (D::x_inner(k)) return k; return -1; }();
  static constexpr int YK0 = [] { for (int k = 0; k < D::KY; ++k) if (D::y_inner(k)) return k; return -1; }();
  const InT *X;
  const float *dY;
  float *Xs, *Ys;
  int w, lane;
  uint32_t xo_in, xo[D::KX], yo_in, yo[D::KY];  // (xo / yo: the edge k steps; *_in: the inner ones' base)
  int xl, yl;                                   // LDS bases of the lane's first quad (row w)
  XV xr[D::XROWS * D::KX];
  f32x4 yr[D::KY];
  __device__ DwRowStage(const InT *X_, const float *dY_, float *Xs_, float *Ys_) : X(X_), dY(dY_), Xs(Xs_), Ys(Ys_) {
    w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    lane = threadIdx.x & 63;
    constexpr int EB = (int)sizeof(InT);
    const int px = lane / D::CQ, cq = lane - px * D::CQ;  // patch column (at k = 0) and channel quad
    xo_in = (uint32_t)(((px + (XK0 < 0 ? 0 : XK0) * D::PXK - G::PL) * D::CIN + 4 * cq) * EB);
#pragma unroll
    for (int k = 0; k < D::KX; ++k) {
      const int pc = px + k * D::PXK, ix = pc - G::PL;
      const bool ok = lane < D::LUX && lane + D::LUX * k < D::QRX && ix >= 0 && ix < D::W;
      xo[k] = ok ? (uint32_t)((ix * D::CIN + 4 * cq) * EB) : kOut;
    }
    const int py = lane / D::CQO, co = lane - py * D::CQO;
    yo_in = (uint32_t)(((py + (YK0 < 0 ? 0 : YK0) * D::PYK) * D::COUT + 4 * co) * 4);
#pragma unroll
    for (int k = 0; k < D::KY; ++k) {
      const int pc = py + k * D::PYK;
      const bool ok = lane + 64 * k < D::QRY && pc < D::OW;
      yo[k] = ok ? (uint32_t)((pc * D::COUT + 4 * co) * 4) : kOut;
    }
    xl = (w * D::WPX + px) * D::CS + 4 * cq;
    yl = (w * D::WPAD + py) * D::COS + 4 * co;
  }
  __device__ __forceinline__ void load(int c) {
    const int b = c / D::RG, y0 = (c - b * D::RG) * D::R;
    const InT *xi = X + (size_t)b * D::H * D::W * D::CIN;
#pragma unroll
    for (int h = 0; h < D::XROWS; ++h) {
      const int iy = y0 - G::PT + w + 4 * h;
      const bool rok = (unsigned)iy < (unsigned)D::H;  // (wave-uniform)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(xi + (size_t)(rok ? iy : 0) * D::W * D::CIN), (short)0, rok ? D::W * D::CIN * (int)sizeof(InT) : 0,
          kRsrc3);
#pragma unroll
      for (int k = 0; k < D::KX; ++k) {
        const bool inner = D::x_inner(k);
        const uint32_t vo = inner ? xo_in : xo[k];
        const int so = inner ? (k - XK0) * D::PXK * D::CIN * (int)sizeof(InT) : 0;
        if constexpr (U8)
          xr[h * D::KX + k] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0);
        else
          xr[h * D::KX + k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
      }
    }
    const int oy = y0 + w;
    const bool rok = oy < D::OH;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(dY + ((size_t)b * D::OH + (rok ? oy : 0)) * D::OW * D::COUT), (short)0, rok ? D::OW * D::COUT * 4 : 0,
        kRsrc3);
#pragma unroll
    for (int k = 0; k < D::KY; ++k) {
      const bool inner = D::y_inner(k);
      const uint32_t vo = inner ? yo_in : yo[k];
      const int so = inner ? (k - YK0) * D::PYK * D::COUT * 4 : 0;
      yr[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
    }
  }
  __device__ __forceinline__ void store() {
#pragma unroll
    for (int h = 0; h < D::XROWS; ++h)
#pragma unroll
      for (int k = 0; k < D::KX; ++k) {
        if (((k + 1) * D::LUX > D::QRX || D::LUX < 64) && (lane >= D::LUX || lane + D::LUX * k >= D::QRX))
          continue;  // (the row's last, partial k step; the idle lane)
        float *d = Xs + xl + (4 * h * D::WPX + k * D::PXK) * D::CS;
        f32x4 v;
        if constexpr (U8) {
          const uint32_t u = xr[h * D::KX + k];
          const float sc = 1.0f / 255.0f;  // InElem<true>::load4's arithmetic
          v = f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc, (float)((u >> 16) & 0xff) * sc,
                    (float)(u >> 24) * sc};
        } else {
          v = xr[h * D::KX + k];
        }
        if constexpr (D::CS % 4 == 0) {
          *reinterpret_cast<f32x4 *>(d) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = v[e];
        }
      }
#pragma unroll
    for (int k = 0; k < D::KY; ++k) {
      if ((k + 1) * 64 > D::QRY && lane + 64 * k >= D::QRY) continue;
      float *d = Ys + yl + k * D::PYK * D::COS;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = yr[k][e];
    }
  }
};

template <class G, bool U8, int TMW>
struct DWgradJob {
  using D = DWCfg<G, U8, TMW>;
  using InT = typename InElem<U8>::T;
  const InT *X;     // layer input [B][H][W][CIN]
  const float *dY;  // conv-output gradient [B][H][W][COUT]
  float *slab;      // [S][KK + 1][COUT]
  int B, S;
  __host__ __device__ int blocks() const { return B > 0 ? S * D::TG : 0; }
  size_t lds() const { return D::LDS; }

  __device__ __forceinline__ void run(int id, float *smem) const {
    id = xcd_tile(id, blocks());  // (the tap groups of a split: one XCD's L2)
    const int sp = id / D::TG, tg = id - sp * D::TG;
    const int NC = B * D::RG;
    const int c0 = (int)((long)sp * NC / S), c1 = (int)((long)(sp + 1) * NC / S);
    float *Xs = smem, *Ys = smem + D::XSZ;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int j = w % D::TN, wm = w / D::TN;  // the wave's N-tile and M set

    // per-lane operand bases: row 16 m + r = (tap, ci) of M-tile m = tg MPB + wm + WROWS i
    int abase[TMW];
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int row = min(16 * (tg * D::MPB + wm + D::WROWS * i) + r, D::KK - 1);  // (rows >= KK: not stored)
      const int t = row / D::CIN, ci = row - t * D::CIN, ky = t / D::KW, kx = t - ky * D::KW;
      abase[i] = ((g * D::S + ky) * D::WPX + kx) * D::CS + ci;
    }
    const int bbase = g * D::WPAD * D::COS + 16 * j + r;

    typename std::conditional<D::ROWMAP, DwRowStage<D, U8>, DwItemStage<D, U8>>::type st(X, dY, Xs, Ys);
    auto load = [&](int c) { st.load(c); };
    auto store = [&]() { st.store(); };

    f32x4 acc[TMW];
#pragma unroll
    for (int i = 0; i < TMW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dbs = 0.f;  // lane (r, g): dY[rows g][.][16 j + r] (the bias row, wave row 0)
    if (c0 < c1) load(c0);
    for (int c = c0; c < c1; ++c) {
      __syncthreads();  // the previous chunk's reads are done
      store();
      __syncthreads();
      if (c + 1 < c1) load(c + 1);  // in flight under this chunk's MFMAs
#pragma unroll
      for (int kq = 0; kq < D::KQ; ++kq) {
        float bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[s] = Ys[bbase + (4 * kq + s) * D::COS];
        float av[TMW][4];
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
          for (int s = 0; s < 4; ++s) av[i][s] = Xs[abase[i] + (4 * kq + s) * D::S * D::CS];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TMW; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][s], bv[s], acc[i], 0, 0, 0);
        dbs += (bv[0] + bv[1]) + (bv[2] + bv[3]);
      }
    }
    // slab rows of the wave's tiles: lane (r, g) holds rows 4 g .. 4 g + 3 of column 16 j + r
    float *o = slab + (size_t)sp * D::SLAB;
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int m = tg * D::MPB + wm + D::WROWS * i;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * m + 4 * g + q;
        if (row < D::KK) o[(size_t)row * D::COUT + 16 * j + r] = acc[i][q];
      }
    }
    if (tg == 0 && wm == 0) {
      dbs += __shfl_xor(dbs, 16, 64);
      dbs += __shfl_xor(dbs, 32, 64);
      if (g == 0) o[(size_t)D::KK * D::COUT + 16 * j + r] = dbs;
    }
  }
};

// Which layers take the direct weight gradient: the 5x5 stride-1 SAME layers (PWYX / LSTM conv1,
// conv2: PWYX-RGB conv1 272 vs 345 us, conv2 161 vs 196 us; LSTM conv2 281 vs 373, conv1 186 vs 267;
// profiles/r03e_*). Measured slower direct and left on the generic GEMM: the 4x4 / 3x3 layers (PWYX
// conv3 group 151 vs 125 us, LSTM 262 vs 210, conv4 79 vs 60) and the strided VALID layers (NATURE
// E=64 conv2 dX + dW group 94 vs 60 us, conv3 53 vs 46; profiles/r03k, r03n).
template <class G>
constexpr bool dconv_wgrad() {
  return G::S == 1 && G::SAME && G::KH == 5;
}
// M-tiles per wave: every M-tile of the layer in one tap group when that takes at most 10 per wave
// (the gray conv1's 7 M-tiles of (tap, ci) rows: 4; the RGB conv1's 19: 10, 232 VGPRs — each staged
// chunk then feeds all of them: RGB conv1 dW 225.3 -> 195.0 us, profiles/r06rgb); the 32 -> 32
// layer (50 M-tiles): 13 per wave, two tap groups of 26 tiles (236 VGPRs; with kDwSlabCap at 8M
// floats, 256 splits): conv2 dW 238.7 -> 232.6 us (LSTM), 137.1 -> 133.7 us (PWYX-RGB),
// profiles/r06dw13; otherwise 5 (4 for 64 output channels)
template <class G>
constexpr int dw_tmw() {
  constexpr int mt = (G::KK + 15) / 16, wrows = 4 / (G::COUT / 16);
  if (G::COUT >= 64) return 4;
  if ((mt + wrows - 1) / wrows <= 10) return (mt + wrows - 1) / wrows;
  if (G::CIN == 32 && mt == 50) return 13;
  constexpr int w5 = (mt + 5 * wrows - 1) / (5 * wrows) * 5 * wrows - mt;  // empty tile slots at 5
  constexpr int w4 = (mt + 4 * wrows - 1) / (4 * wrows) * 4 * wrows - mt;  // and at 4
  return w4 < w5 ? 4 : 5;
}
template <class G, bool U8>
using DWJobFor = DWgradJob<G, U8, dw_tmw<G>()>;

// splits: ~512 blocks (two per CU), at most one chunk each, slabs within kDwSlabCap
template <class G, bool U8>
inline int dwgrad_splits(int B) {
  using D = typename DWJobFor<G, U8>::D;
  int s = std::max(1, 512 / D::TG);
  s = std::min<long>(s, (long)B * D::RG);
  s = (int)std::min<size_t>((size_t)s, std::max<size_t>(kDwSlabCap / D::SLAB, 1));
  return std::max(s, 1);
}

template <class G, bool U8>
inline size_t dwgrad_slab_floats(int B) {
  return (size_t)dwgrad_splits<G, U8>(B) * DWJobFor<G, U8>::D::SLAB;
}

}  // namespace mt
