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

// ---- problems ------------------------------------------------------------------------------
// Forward of conv G: X = its input [B][H][W][CIN] (u8 frames for conv1), Y = the pooled output
// [B][OH/2][OW/2][COUT] + argmax bytes (POOL, EpBiasActPool's layout and first-max rule) or the
// activation [B][OH][OW][COUT].
template <class G, bool U8, bool POOL_>
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
  __device__ __forceinline__ void store(const Pre &p, int b, int u, int n, f32x4 v) const {
    if constexpr (POOL) {
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
        if (px < OH * OW) Y[((size_t)b * OH * OW + px) * CO + n] = act_fwd(v[q] + p.b, act, alpha);
      }
    }
  }
};

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
  f32x4 wr[D::BIT];
  auto wload = [&](int c) {
#pragma unroll
    for (int it = 0; it < D::BIT; ++it) {
      const int item = tid + it * D::NT;
      if (D::BITEMS % D::NT == 0 || item < D::BITEMS) {
        const int kq = item / D::CO, n = item - kq * D::CO;
        wr[it] = p.wquad(c * D::CK + 4 * kq, n);
      }
    }
  };
  auto wstore = [&](float *dst) {
#pragma unroll
    for (int it = 0; it < D::BIT; ++it) {
      const int item = tid + it * D::NT;
      if (D::BITEMS % D::NT == 0 || item < D::BITEMS) {
        const int kq = item / D::CO, n = item - kq * D::CO;
        const int kcl = kq >> 2, gg = kq & 3, j = n >> 4, rr = n & 15;
        *reinterpret_cast<f32x4 *>(dst + ((kcl * D::TN + j) * 64 + gg * 16 + rr) * 4) = wr[it];
      }
    }
  };
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
  if constexpr (D::NCH > 1) t1 = t0 + 1;  // (chunked weights: one tile per block, no loop)
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
        const f32x4 x = InElem<std::is_same<typename Pr::InT, uint8_t>::value>::load4(
            img + (size_t)(ok ? iy * D::W + ix : 0) * D::CI + 4 * cq);
        v[t] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
        dst[t] = (D::AQ % D::NT == 0 || tid + it * D::NT < D::AQ) ? (pr * D::WPX + pc) * D::CS + 4 * cq : -1;
      }
    }
#pragma unroll
    for (int t = 0; t < ABATCH; ++t)
      if (it0 + t < D::AIT && dst[t] >= 0) *reinterpret_cast<f32x4 *>(As + dst[t]) = v[t];
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
    for (int c = 0; c < D::NCH; ++c) {
      const bool more = c + 1 < D::NCH;
      if (more) wload(c + 1);
      compute(Bs + (c & 1) * D::BSZ, c);
      if (more) {
        wstore(Bs + ((c + 1) & 1) * D::BSZ);
        __syncthreads();
      }
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
//  conv2 (32 -> 32): 8-wave blocks (two N halves), two blocks per CU: four waves per SIMD hide the
//    per-chunk barrier (PWYX-RGB E=32 33.4 vs 36.7 us, LSTM 161 frames 143.6 vs 157.5 us,
//    profiles/r03i); 2 M-tiles per wave; one tap (CIN k) per weight chunk (5-tap chunks: no faster);
//  64 output channels (conv3, conv4, NATURE conv2 / conv3): 8-wave blocks for the small grids
//    (18.2 -> 15.3 us and 11.0 -> 10.1 us), 1 M-tile per wave.
template <class G, bool POOL>
struct DConvFor {
  static constexpr bool SMALLC = G::CIN % 16 != 0;  // conv1: the whole K in one chunk
  static constexpr bool C64 = G::COUT >= 64;
  static constexpr int WN = C64 ? (POOL ? 2 : 4) : (SMALLC ? 1 : 2);
  static constexpr int WM = C64 ? (POOL ? 4 : 2) : 4;
  static constexpr int TMW = SMALLC ? (G::S > 1 ? 1 : 2) : (C64 ? 1 : 2);
  static constexpr int CK = SMALLC ? 0 : G::CIN;
};

template <class G, bool U8, bool POOL>
static int conv_forward_direct(const void *X, const float *W, const float *bias, float *Y, uint8_t *arg, int B,
                               int act, float alpha, hipStream_t s) {
  using F = DConvFor<G, POOL>;
  using Pr = DFwd<G, U8, POOL>;
  const Pr p{reinterpret_cast<const typename Pr::InT *>(X), W, bias, Y, arg, act, alpha};
  return launch_dconv<Pr, F::WM, F::WN, F::TMW, F::CK>(p, B, s);
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
  return launch_dconv<DBwdUnpool<G, GJ>, 4, 2, (G::COUT >= 64 ? 1 : 2), G::COUT>(
      DBwdUnpool<G, GJ>{dY, Wt, Pj, argj, dactj, act, alpha}, B, s);
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
constexpr size_t kDwSlabCap = (size_t)4 << 20;  // slab floats (the generic path's kSlabFloats)

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
  static constexpr int CS = dw_pad(CIN, S * WP), COS = dw_pad(COUT, WPAD);
  static constexpr int XSZ = (RIN * WP * CS + 3) / 4 * 4, YSZ = R * WPAD * COS;
  static constexpr size_t LDS = (size_t)(XSZ + YSZ) * 4;
  static constexpr int XQ = RIN * WP * (CIN / 4), YQ = R * WPAD * (COUT / 4);  // quads per chunk
  static constexpr int XIT = (XQ + 255) / 256, YIT = (YQ + 255) / 256;
  static constexpr size_t SLAB = (size_t)(KK + 1) * COUT;
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
      abase[i] = ((g * D::S + ky) * D::WP + kx) * D::CS + ci;
    }
    const int bbase = g * D::WPAD * D::COS + 16 * j + r;

    f32x4 xr[D::XIT], yr[D::YIT];
    auto load = [&](int c) {
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
    };
    auto store = [&]() {
#pragma unroll
      for (int it = 0; it < D::XIT; ++it) {
        const int item = tid + 256 * it;
        if (D::XQ % 256 == 0 || item < D::XQ) {
          const int pix = item / (D::CIN / 4), cq = item - pix * (D::CIN / 4);
          float *d = Xs + pix * D::CS + 4 * cq;  // (CS % 4 may be != 0: four dword stores)
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = xr[it][e];
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
    };

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
// M-tiles per wave: 5 (4 for 64 output channels), or for a short K (the gray conv1: 7 M-tiles of
// (tap, ci) rows) just enough for one tap group — 5 would leave 3 of its 10 tile slots empty
template <class G>
constexpr int dw_tmw() {
  constexpr int mt = (G::KK + 15) / 16, wrows = 4 / (G::COUT / 16);
  if (G::COUT >= 64) return 4;
  if (mt <= 5 * wrows) return (mt + wrows - 1) / wrows;
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
