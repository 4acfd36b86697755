// Backward-data product of the NATURE trunk's strided conv2 (networks.py:261-278: 4x4 s2, 32 -> 64
// on 20x20) as an image-streaming, weight-stationary job of the layer's grouped launch, in place of
// the generic phase GEMM (gemm.h: LdConvBwdAPhase), whose blocks re-gather every dY element from L2
// per 64-deep K chunk and feed it to two MFMA tiles (N = 32 channels): ~130 MB of gathered dY per
// launch at N = 320 (DESIGN round 4).
//
// DxStreamJob: block = (stride phase, 16 input channels) x an image group. The block's B operand —
// W[py + S a][px + S b][ci-tile][all co] for its phase, the whole K — is staged ONCE into LDS in MFMA
// fragment order; then the block streams its images: each image's dY is staged once into a
// zero-bordered LDS patch (the next image's loads in flight in registers meanwhile), the phase's MT
// output M-tiles are dealt to the 4 waves, every A fragment is one ds_read_b128 at (the lane's phase
// pixel + the tap) x 4 consecutive co and every B fragment one conflict-free ds_read_b128. The
// epilogue applies the activation mask of the layer's input and scatters phase pixel (qy, qx) of
// channel ci to dX[S qy + py][S qx + px][ci]. The image groups are contiguous and XCD-aware (one
// group's blocks — every phase / channel tile of the same images — on one XCD's L2).
//
// Measured (round 5, profiles/r05c, tools/ab_bwd.sh: rocprof of the train pass, the conv2 group =
// dX + the generic dW + conv3's slab sum): Seaquest E=32 34.8 -> 30.4 us, Breakout E=64 59.3 ->
// 54.2 us. Not adopted, measured slower than the generic products on the same groups: the same job
// for conv3's stride-1 dX (27.2 -> 30.3 / 46.3 -> 51.1 us: the 9x9 output's zero-bordered 3x3 taps
// leave 51 % of its MFMA work useful, against the gather GEMM's full M tiles) and an output-
// stationary weight gradient accumulating a block's images in registers (conv2 group 38.0 / 68.3
// us, conv3 27.4 / 58.2 with it beside the generic dX: its 256 blocks' per-image chains were longer
// than the generic 500-block K split's).
#pragma once
#include "gemm.h"

namespace mt {

// Which conv layers take the streaming dX: the NATURE trunk's conv2 (strided VALID, phase-separable,
// 64 output channels; gray or RGB input of conv1 does not change it).
template <class G>
constexpr bool stream_dx() {
  return G::S > 1 && !G::SAME && G::COUT == 64 && G::CIN % 16 == 0 && G::KH % G::S == 0 && G::KW % G::S == 0 &&
         G::H % G::S == 0 && G::W % G::S == 0 && G::H / G::S == G::OH + G::KH / G::S - 1 &&
         G::W / G::S == G::OW + G::KW / G::S - 1;
}

// ---- dX ------------------------------------------------------------------------------------
// dX[S qy + py][S qx + px][ci] = sum_{a < KA, b < KB, co} P[qy + a][qx + b][co] W[py + S (KA-1-a)]
// [px + S (KB-1-b)][ci][co], P = dY zero-bordered by KA - 1 rows / KB - 1 columns (the full
// correlation of each stride phase; S = 1: one phase).
template <class G>
struct DxGeom {
  static constexpr int S = G::S, PH = S * S, KA = G::KH / S, KB = G::KW / S;
  static constexpr int HQ = G::H / S, WQ = G::W / S;                          // phase grid
  static constexpr int PR = G::OH + 2 * (KA - 1), PC = G::OW + 2 * (KB - 1);  // zero-bordered dY
  static constexpr int CS = G::COUT + 4;  // LDS floats per dY pixel (lanes r of a ds_read_b128 on distinct banks)
  static constexpr int IMG = PR * PC * CS;                 // LDS floats of the patch
  static constexpr int MQ = HQ * WQ, MT = (MQ + 15) / 16;  // phase pixels, M-tiles per (image, phase)
  static constexpr int NT = G::CIN / 16, CQ = G::COUT / 16;
  static constexpr int KC = KA * KB * CQ;  // 16-deep K chunks: (tap, co quarter)
  static constexpr int COMBOS = PH * NT;   // (phase, ci tile) per image group
  static constexpr int TPW = (MT + 3) / 4;  // M-tiles of wave 0 (wave w: tiles w, w + 4, ..)
  static constexpr int PQ = G::COUT / 4;    // dY quads per pixel
  static constexpr int YQ = G::OH * G::OW * PQ;  // dY quads per image
  static constexpr int PFQ = (YQ + 255) / 256;
  static constexpr int BSZ = KC * 256;  // the block's B operand in fragment order [kc][lane][4]
  static constexpr size_t LDS = (size_t)(IMG + BSZ) * sizeof(float);
};

template <class G>
struct DxStreamJob {
  using D = DxGeom<G>;
  const float *dY;    // [B][OH][OW][COUT]
  const float *Wt;    // HWIO
  const float *Xact;  // G's input [B][H][W][CIN] (post-activation: the mask)
  float *dX;          // [B][H][W][CIN]
  int B, GR, act;
  float alpha;
  __host__ __device__ int blocks() const { return B > 0 ? D::COMBOS * GR : 0; }
  size_t lds() const { return D::LDS; }

  __device__ __forceinline__ void run(int id, float *smem) const {
    id = xcd_tile(id, blocks());  // (one group's COMBOS blocks on one XCD)
    const int gi = id / D::COMBOS, c = id - gi * D::COMBOS;
    const int ph = c / D::NT, j = c - ph * D::NT;
    const int py = ph / D::S, px = ph - py * D::S;
    const int i0 = (int)((long)B * gi / GR), i1 = (int)((long)B * (gi + 1) / GR);
    const int tid = threadIdx.x, w = tid >> 6;
    float *Ps = smem, *Bs = smem + D::IMG;

    // the block's whole B operand, once, in fragment order: chunk kc = (tap t = (a, b), co quarter),
    // lane (r, g) -> W[ky][kx][16 j + r][16 (kc % CQ) + 4 g .. + 3]
    for (int i = tid; i < D::KC * 64; i += 256) {
      const int kc = i >> 6, l = i & 63, r = l & 15, g = l >> 4;
      const int t = kc / D::CQ, a = t / D::KB, b = t - a * D::KB;
      const int ky = py + D::S * (D::KA - 1 - a), kx = px + D::S * (D::KB - 1 - b);
      *reinterpret_cast<f32x4 *>(Bs + 4 * i) = *reinterpret_cast<const f32x4 *>(
          Wt + ((size_t)(ky * G::KW + kx) * G::CIN + 16 * j + r) * G::COUT + 16 * (kc % D::CQ) + 4 * g);
    }
    // zero the patch once: the border stays zero, each image rewrites the interior
    for (int i = tid; i < D::IMG / 4; i += 256) reinterpret_cast<f32x4 *>(Ps)[i] = f32x4{0.f, 0.f, 0.f, 0.f};

    f32x4 pf[D::PFQ];
    auto fetch = [&](int b) {  // image b's dY into registers
      const f32x4 *src = reinterpret_cast<const f32x4 *>(dY + (size_t)b * G::OH * G::OW * G::COUT);
#pragma unroll
      for (int q = 0; q < D::PFQ; ++q) pf[q] = src[min(tid + 256 * q, D::YQ - 1)];
    };
    auto put = [&]() {
#pragma unroll
      for (int q = 0; q < D::PFQ; ++q) {
        const int qi = tid + 256 * q;
        if (D::YQ % 256 == 0 || qi < D::YQ) {
          const int pix = qi / D::PQ, cq = qi - pix * D::PQ;
          const int oy = pix / G::OW, ox = pix - oy * G::OW;
          *reinterpret_cast<f32x4 *>(Ps + ((oy + D::KA - 1) * D::PC + ox + D::KB - 1) * D::CS + 4 * cq) = pf[q];
        }
      }
    };
    if (i0 < i1) fetch(i0);
    __syncthreads();  // (the zero fill before any interior store)
    for (int b = i0; b < i1; ++b) {
      if (b > i0) __syncthreads();  // the previous image's LDS reads are done
      put();
      if (b + 1 < i1) fetch(b + 1);  // in flight under this image's MFMAs
      __syncthreads();               // the patch is in LDS
      // wave w: M-tiles w, w + 4 (wave-uniform count: no per-tile branch inside the MFMA loop)
      if (w + 4 * (D::TPW - 1) < D::MT)
        image_pass<D::TPW>(Ps, Bs, b, py, px, j);
      else
        image_pass<D::TPW - 1>(Ps, Bs, b, py, px, j);
    }
  }

  template <int NU>
  __device__ __forceinline__ void image_pass(const float *Ps, const float *Bs, int b, int py, int px, int j) const {
    if constexpr (NU > 0) {
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
      float mk[NU][4];
      int abase[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int mt = w + 4 * u;
        const int m = min(16 * mt + r, D::MQ - 1), qy = m / D::WQ, qx = m - qy * D::WQ;
        abase[u] = (qy * D::PC + qx) * D::CS + 4 * g;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int mq = min(16 * mt + 4 * g + q, D::MQ - 1), y = mq / D::WQ, x = mq - y * D::WQ;
          mk[u][q] = Xact[(((size_t)b * G::H + D::S * y + py) * G::W + D::S * x + px) * G::CIN + 16 * j + r];
        }
      }
      f32x4 acc[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto load = [&](int kc, f32x4 &bf, f32x4 (&af)[NU]) {
        const int t = kc / D::CQ, a = t / D::KB, bb = t - a * D::KB;
        const int off = (a * D::PC + bb) * D::CS + 16 * (kc % D::CQ);
        bf = *reinterpret_cast<const f32x4 *>(Bs + 4 * (64 * kc + lane));
#pragma unroll
        for (int u = 0; u < NU; ++u) af[u] = *reinterpret_cast<const f32x4 *>(Ps + abase[u] + off);
      };
      f32x4 bf, af[NU];
      load(0, bf, af);
#pragma unroll 4
      for (int kc = 0; kc < D::KC; ++kc) {
        f32x4 bn, an[NU];
        load(min(kc + 1, D::KC - 1), bn, an);  // next chunk's operands in flight under these MFMAs
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int u = 0; u < NU; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[u][s], bf[s], acc[u], 0, 0, 0);
        bf = bn;
#pragma unroll
        for (int u = 0; u < NU; ++u) af[u] = an[u];
      }
      // lane (r, g) holds rows 16 mt + 4 g + q of column ci = 16 j + r
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int mt = w + 4 * u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int mq = 16 * mt + 4 * g + q;
          if (mq < D::MQ) {
            const int y = mq / D::WQ, x = mq - y * D::WQ;
            dX[(((size_t)b * G::H + D::S * y + py) * G::W + D::S * x + px) * G::CIN + 16 * j + r] =
                acc[u][q] * act_bwd(mk[u][q], act, alpha);
          }
        }
      }
    }
  }
};

// Image groups: ~256 blocks (one per CU).
template <class G>
inline int dx_stream_groups(int B) {
  return std::max(1, std::min(B, 256 / DxGeom<G>::COMBOS));
}

}  // namespace mt
