// Direct convolution for the stride-1 SAME convs of the PWYX trunk (networks.py:206-225; the LSTM
// arch runs it per window frame, networks.py:227-258): conv + bias + activation (+ the 2x2/2 max
// pool and its argmax bytes), forward.
//
// Why not the generic implicit-im2col GEMM (gemm.h, LdIm2col): there every A element of every
// K chunk is re-derived from (row, k) — tap / channel divisions, SAME-padding clamps and selects —
// and fetched from L2, 5-8 VALU instructions per MFMA (rocprof PMC, profiles/r03c_*), which at 4
// waves per CU sets the pace instead of the MFMA. Here a block stages its input PATCH once in LDS
// (zero-padded, u8 -> f32 for conv1), and the K walk reads each A fragment as ONE ds_read_b128 at
// (the lane's pixel) + (the tap's offset): no per-element address math at all.
//
// Block = 256 threads (4 waves, WM x WN), UPB "units" of one image x all COUT channels. A unit is
// one 2x2 pool window (POOL: its 4 pixels are the 4 rows a lane's accumulator holds, so the pool
// is a register max) or a quad of consecutive pixels (no pool). A wave owns TMW 16-row M-tiles
// (4 units each) and TNW 16-column N-tiles: TMW x TNW accumulators of v_mfma_f32_16x16x4_f32.
//
// K order: k = tap * CIN + c (HWIO flatten). A fragment element s of lane (r, g) of k-chunk kc is
// k = 16 kc + 4 g + s, i.e. channel quad q = 4 kc + g of tap q / (CIN/4): 4 consecutive channels
// of one pixel = one 16-byte LDS read. The weights are staged chunk by chunk (CK k-values) into
// LDS in that fragment order — [kc][n-tile][lane][4], so a B fragment is one conflict-free
// ds_read_b128 — double-buffered: chunk c+1's global loads are in flight while chunk c is
// multiplied, one barrier per chunk.
#pragma once
#include "gemm.h"

namespace mt {

template <class G, bool POOL, int WM, int WN, int TMW, int CK_>
struct DConvCfg {
  static_assert(G::S == 1 && G::SAME, "direct conv: stride-1 SAME convs");
  static_assert(WM * WN == 4, "4 waves");
  static constexpr int CIN = G::CIN, COUT = G::COUT, KH = G::KH, KW = G::KW;
  static constexpr int QT = CIN / 4;  // channel quads per tap
  static constexpr int TAPS = KH * KW;
  static constexpr int KP = (G::KK + 15) / 16 * 16;  // K padded to whole 16-chunks (zero weights)
  static constexpr int KC = KP / 16;
  static constexpr int TN = COUT / 16;
  static_assert(COUT % 16 == 0 && TN % WN == 0, "N tiles");
  static constexpr int TNW = TN / WN;
  static constexpr int UPB = WM * TMW * 4;  // units per block
  static constexpr int PH = G::OH / 2, PW = G::OW / 2;
  static constexpr int NPIX = G::OH * G::OW;
  static constexpr int U = POOL ? PH * PW : (NPIX + 3) / 4;  // units per image
  static constexpr int BPI = (U + UPB - 1) / UPB;             // blocks per image
  // output rows a block's units can touch, and the input rows / columns of its patch
  static constexpr int RSPAN0 = POOL ? 2 * ((UPB - 1) / PW + 2) : (4 * UPB - 1) / G::OW + 2;
  static constexpr int RSPAN = RSPAN0 < G::OH ? RSPAN0 : G::OH;
  static constexpr int RIN = RSPAN + KH - 1;
  static constexpr int WP = G::OW + KW - 1;
  static constexpr int CS = CIN % 16 == 0 ? CIN + 4 : CIN;  // floats per patch pixel (bank spread)
  static constexpr int ASZ = (RIN * WP * CS + 3) / 4 * 4;
  static constexpr int CK = CK_ > 0 ? CK_ : KP;  // k per weight chunk
  static_assert(CK % 16 == 0, "chunk of whole 16-k steps");
  static constexpr bool TAPALIGNED = QT % 4 == 0 && CK % CIN == 0;
  static_assert(TAPALIGNED || CK == KP, "a chunk that is not tap-aligned must hold the whole K");
  static constexpr int TPC = TAPALIGNED ? CK / CIN : 0;  // taps per chunk
  static constexpr int CKC = CK / 16;
  static constexpr int NCH = KC / CKC;
  static_assert(NCH * CKC == KC, "whole chunks");
  static constexpr int BSZ = CKC * TN * 256;  // floats per staged weight chunk
  static constexpr int NBUF = NCH > 1 ? 2 : 1;
  static constexpr size_t LDS = (size_t)(ASZ + NBUF * BSZ) * 4;
  static constexpr int BITEMS = (CK / 4) * COUT;  // (k quad, column) items of one chunk
  static constexpr int BIT = (BITEMS + 255) / 256;
  static constexpr int AQ = RIN * WP * QT;  // patch channel quads
  static constexpr int AIT = (AQ + 255) / 256;
};

template <class G, bool U8, bool POOL, int WM, int WN, int TMW, int CK>
__global__ __launch_bounds__(256) void dconv_fwd_kernel(const typename InElem<U8>::T *__restrict__ X,
                                                        const float *__restrict__ Wt, const float *__restrict__ bias,
                                                        float *__restrict__ Y, uint8_t *__restrict__ arg, int act,
                                                        float alpha) {
  using D = DConvCfg<G, POOL, WM, WN, TMW, CK>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *As = smem;
  float *Bs = smem + D::ASZ;
  // XCD-aware: an XCD takes a contiguous run of blocks, so the overlapping patches of one image's
  // blocks are fetched into one L2
  const int bid = xcd_tile(blockIdx.x, gridDim.x);
  const int b = bid / D::BPI;
  const int u0 = (bid - b * D::BPI) * D::UPB;
  const int oy0 = POOL ? 2 * (u0 / D::PW) : (4 * u0) / G::OW;  // output row of patch row 0
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int r = lane & 15, g = lane >> 4;

  // weight chunk c -> registers (k >= KK: zero, from a clamped address)
  f32x4 wr[D::BIT];
  auto wload = [&](int c) {
#pragma unroll
    for (int it = 0; it < D::BIT; ++it) {
      const int item = tid + it * 256;
      if (D::BITEMS % 256 == 0 || item < D::BITEMS) {
        const int kq = item / D::COUT, n = item - kq * D::COUT;
        const int k = c * D::CK + 4 * kq;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float x = Wt[(size_t)min(k + s, G::KK - 1) * D::COUT + n];
          wr[it][s] = k + s < G::KK ? x : 0.f;
        }
      }
    }
  };
  // ... and into LDS in fragment order [kc][n-tile][lane = 16 g + r][s]
  auto wstore = [&](float *dst) {
#pragma unroll
    for (int it = 0; it < D::BIT; ++it) {
      const int item = tid + it * 256;
      if (D::BITEMS % 256 == 0 || item < D::BITEMS) {
        const int kq = item / D::COUT, n = item - kq * D::COUT;
        const int kcl = kq >> 2, gg = kq & 3, j = n >> 4, rr = n & 15;
        *reinterpret_cast<f32x4 *>(dst + ((kcl * D::TN + j) * 64 + gg * 16 + rr) * 4) = wr[it];
      }
    }
  };
  wload(0);
  float bj[D::TNW];
#pragma unroll
  for (int j = 0; j < D::TNW; ++j) bj[j] = bias[(wn * D::TNW + j) * 16 + r];

  // the patch: input rows oy0 - PT .. oy0 - PT + RIN - 1, columns -PL .. -PL + WP - 1 (zeros
  // outside the image), in batches of 8 quads per thread (all loads of a batch in flight)
  const auto *img = X + (size_t)b * G::H * G::W * G::CIN;
  constexpr int ABATCH = 8;
#pragma unroll
  for (int it0 = 0; it0 < D::AIT; it0 += ABATCH) {
    f32x4 v[ABATCH];
    int dst[ABATCH];
#pragma unroll
    for (int t = 0; t < ABATCH; ++t) {
      const int it = it0 + t;
      if (it < D::AIT) {
        const int item = min(tid + it * 256, D::AQ - 1);
        const int pix = item / D::QT, cq = item - pix * D::QT;
        const int pr = pix / D::WP, pc = pix - pr * D::WP;
        const int iy = oy0 - G::PT + pr, ix = pc - G::PL;
        const bool ok = (unsigned)iy < (unsigned)G::H && (unsigned)ix < (unsigned)G::W;
        const f32x4 x = InElem<U8>::load4(img + (size_t)(ok ? iy * G::W + ix : 0) * G::CIN + 4 * cq);
        v[t] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
        dst[t] = (D::AQ % 256 == 0 || tid + it * 256 < D::AQ) ? (pr * D::WP + pc) * D::CS + 4 * cq : -1;
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
    if constexpr (POOL) {
      const int py = u / D::PW;
      oy = 2 * py + (q >> 1);
      ox = 2 * (u - py * D::PW) + (q & 1);
    } else {
      const int p = min(4 * u + q, D::NPIX - 1);
      oy = p / G::OW;
      ox = p - oy * G::OW;
    }
    abase[i] = ((oy - oy0) * D::WP + ox) * D::CS;
  }
  // A offsets of the k-chunks (one chunk: K not tap-aligned, small CIN): tap and channel quad of
  // quad index 4 kc + g (past the last tap: any tap, its weights are zero)
  int aoffs[D::TAPALIGNED ? 1 : D::KC];
  if constexpr (!D::TAPALIGNED) {
#pragma unroll
    for (int kc = 0; kc < D::KC; ++kc) {
      const int q4 = 4 * kc + g, t0 = q4 / D::QT, cq = q4 - t0 * D::QT;
      const int t = min(t0, D::TAPS - 1), ky = t / D::KW, kx = t - ky * D::KW;
      aoffs[kc] = (ky * D::WP + kx) * D::CS + 4 * cq;
    }
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
        ao = ((t / D::KW) * D::WP + t % D::KW) * D::CS + 4 * ((4 * kcl) % D::QT) + 4 * g;
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

  wstore(Bs);
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
    for (int j = 0; j < D::TNW; ++j) {
      const int n = (wn * D::TNW + j) * 16 + r;
      if constexpr (POOL) {  // EpBiasActPool: first maximum in window order
        float mx = act_fwd(acc[i][j][0] + bj[j], act, alpha);
        int am = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const float y = act_fwd(acc[i][j][q] + bj[j], act, alpha);
          if (y > mx) {
            mx = y;
            am = q;
          }
        }
        const size_t o = ((size_t)b * D::U + u) * D::COUT + n;
        Y[o] = mx;
        arg[o] = (uint8_t)am;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int p = 4 * u + q;
          if (p < D::NPIX) Y[((size_t)b * D::NPIX + p) * D::COUT + n] = act_fwd(acc[i][j][q] + bj[j], act, alpha);
        }
      }
    }
  }
}

template <class G, bool U8, bool POOL, int WM, int WN, int TMW, int CK>
static int launch_dconv(const void *X, const float *W, const float *bias, float *Y, uint8_t *arg, int B, int act,
                        float alpha, hipStream_t s) {
  using D = DConvCfg<G, POOL, WM, WN, TMW, CK>;
  static_assert(D::LDS <= 160 * 1024, "LDS budget");
  if (B <= 0 || !launch_allowed()) return MT_OK;
  auto kern = &dconv_fwd_kernel<G, U8, POOL, WM, WN, TMW, CK>;
  static bool attr_set = false;
  if (!attr_set && D::LDS > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)D::LDS));
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)B * D::BPI), dim3(256), D::LDS, s,
                     reinterpret_cast<const typename InElem<U8>::T *>(X), W, bias, Y, arg, act, alpha);
  MT_LAUNCHED();
  return MT_OK;
}

// Tile choice per PWYX layer shape (E = 32 frames: conv1 1,792 blocks, conv2 448 or 896, conv3
// 224, conv4 128).
#ifndef MT_DCONV_TMW2  // conv2 (CIN = COUT = 32): 2 M-tiles per wave (32 units per block) or 1
#define MT_DCONV_TMW2 2
#endif
template <class G, bool POOL>
struct DConvFor {
  static constexpr bool SMALLC = G::CIN % 16 != 0;  // conv1: the whole K in one chunk
  static constexpr int WN = (!POOL && G::COUT >= 64) ? 2 : 1;
  static constexpr int WM = 4 / WN;
  static constexpr int TMW = SMALLC ? 2 : (G::COUT >= 64 ? 1 : MT_DCONV_TMW2);
  static constexpr int CK = SMALLC ? 0 : G::CIN;
};

template <class G, bool U8, bool POOL>
static int conv_forward_direct(const void *X, const float *W, const float *bias, float *Y, uint8_t *arg, int B,
                               int act, float alpha, hipStream_t s) {
  using F = DConvFor<G, POOL>;
  return launch_dconv<G, U8, POOL, F::WM, F::WN, F::TMW, F::CK>(X, W, bias, Y, arg, B, act, alpha, s);
}

}  // namespace mt
