// Conv backward of the NIPS trunk (networks.py:178-192, gray frames: C = 4) in one launch of two
// kinds of workgroups, one per CU (each holds up to 138 KB of LDS):
//  * image blocks b < B: conv2 dX (stride phases) masked by conv1's activation derivative into LDS,
//    then conv1 dW and db of the image from LDS-resident operands -> slab1[b] = [257][16] (weight
//    rows in HWIO order, then the bias row);
//  * pair blocks q < ceil(B/2): conv2 dW and db of images 2q, 2q+1 -> slab2[q] = [257][32]
//    (on the CUs the image blocks leave idle: 240 blocks at B = 160);
// the next launch sums the slabs in index order (SlabJob). Replaces the layered path's two conv
// launches (trunk_backward: conv2 dX + conv2 dW, then conv1 dW + the conv2 slab sum), whose
// products re-read dact1, act1 and the frames from HBM and whose boundary costs a launch; here the
// HBM traffic is each image's frame (28 KB), act1 (25.6 KB, read twice), dact2 (10.4 KB, twice),
// W2 (32 KB from L2), dact1 (25.6 KB written: the workspace keeps the layered path's contents)
// and the slabs.
//
// All products on v_mfma_f32_16x16x4_f32 (fp32). 8 waves (2 per SIMD: one block per CU holds 138 KB
// of LDS, and the second wave's MFMAs issue while the first waits on LDS). Lane (r, g) = (lane & 15,
// lane >> 4); an MFMA takes A[r][k_g], B[k_g][r] and accumulates C[4g + i][r] in acc[i].
//   conv2 dX: wave w = stride phase (py, px) = ((w & 3) >> 1, w & 1) of the 20x20 input, half w >> 2
//     of its rows = the 100 phase pixels (qy, qx) (tiles 0-3 / 4-6 of 16), K = (a, b, co) = 2x2x32:
//     dX[2qy+py][2qx+px][ci] = sum dY2[qy-a][qx-b][co] W2[py+2a][px+2b][ci][co] (dY2 zero-bordered).
//   conv1 dW: rows kr = (ky, kx, ci) (16 tiles: ky = w, kx half = tile), K = the 400 output pixels:
//     dW1[kr][co] = (sum_p X[4oy+ky][4ox+kx][ci] dact1[p][co]) / 255 (the integer-valued frame bytes
//     are exact in fp32; the scale is applied once to the sum); the frame is stored split by the
//     stride phase (ky & 3, kx & 3) so 4 consecutive pixels are 4 consecutive bytes.
//   conv2 dW (pair blocks): rows kr = (ky, kx, ci) (16 tiles x 2 channel halves, 4 per wave), K =
//     the 81 output pixels (+3 zero) of each image: dW2[kr][co] = sum_p act1[2oy+ky][2ox+kx][ci] dY2[p][co].
//   bias rows: the column sums of the B operands the waves already hold (dact1 in conv1 dW, dY2 in
//     conv2 dW), reduced over the 4 lane groups by shuffles.
#pragma once
#include "gemm.h"
#include "trunk_fused.h"  // (MT_PROBE_AT: probe builds time the phases of block b in slot 3)

namespace mt {

struct NipsConvBwdJob {
  // frames [B][84][84][4] u8; act1 [B][20][20][16] (post-activation); dY2 = dact2 [B][9][9][32];
  // W2 [4][4][16][32]; dact1 (out, may be NULL) [B][20][20][16]; slab1 [B][257][16];
  // slab2 [pairs()][257][32]
  const uint8_t *X = nullptr;
  const float *act1 = nullptr, *dY2 = nullptr, *W2 = nullptr;
  float *dact1 = nullptr, *slab1 = nullptr, *slab2 = nullptr;
  int B = 0, act = 0;
  float alpha = 0.f;

  static constexpr int NT = 512;
  static constexpr int XROW = 24;                // bytes per row of a phase plane (21 used)
  static constexpr int XPLANE = 21 * XROW;       // (ky & 3, kx & 3, ci) plane: 21 x 24 bytes
  static constexpr int X_BYTES = 64 * XPLANE;    // 32256
  static constexpr int DS = 36;                  // floats per zero-bordered dY2 pixel (11 x 11)
  static constexpr int DY_FLOATS = 11 * 11 * DS;
  static constexpr int WS = 36;                  // floats per (tap, ci) row of W2
  static constexpr int W2_FLOATS = 16 * 16 * WS;
  static constexpr int PS = 404;                 // floats per channel of the transposed 20x20 maps
  static constexpr int MAP_FLOATS = 16 * PS;
  static constexpr int SLAB1 = 257 * 16, SLAB2 = 257 * 32;
  static constexpr size_t LDS = X_BYTES + sizeof(float) * (DY_FLOATS + W2_FLOATS + 2 * MAP_FLOATS);
  static_assert(2 * sizeof(float) * (DY_FLOATS + MAP_FLOATS) <= LDS, "pair block stage");

  __host__ __device__ int pairs() const { return (B + 1) / 2; }
  __host__ __device__ int blocks() const { return B + pairs(); }

  // dY2 of image b into the zero-bordered [11][11][DS] map and act1 into the transposed [16][PS]
  // map: load() issues the global loads, store() writes LDS (callers issue every load first)
  struct DyAct {
    f32x4 yv[2], av[4];
  };
  __device__ __forceinline__ DyAct load_dy_act(int b) const {
    const int tid = threadIdx.x;
    const f32x4 *ys = reinterpret_cast<const f32x4 *>(dY2 + (size_t)b * 81 * 32);
    const f32x4 *as = reinterpret_cast<const f32x4 *>(act1 + (size_t)b * 400 * 16);
    DyAct d;
#pragma unroll
    for (int u = 0; u < 2; ++u) d.yv[u] = ys[min(tid + NT * u, 647)];
#pragma unroll
    for (int u = 0; u < 4; ++u) d.av[u] = as[min(tid + NT * u, 1599)];
    return d;
  }
  __device__ __forceinline__ void store_dy_act(const DyAct &d, float *dyp, float *a1t) const {
    const int tid = threadIdx.x;
    for (int i = tid; i < 121 * 8; i += NT) {  // the zero border (40 pixels x 8 quads)
      const int p = i >> 3, Y = p / 11, Xc = p - 11 * Y;
      if (Y == 0 || Y == 10 || Xc == 0 || Xc == 10)
        *reinterpret_cast<f32x4 *>(dyp + p * DS + 4 * (i & 7)) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + NT * u;
      if (i < 648) {
        const int p = i >> 3, oy = p / 9, ox = p - 9 * oy;
        *reinterpret_cast<f32x4 *>(dyp + ((oy + 1) * 11 + ox + 1) * DS + 4 * (i & 7)) = d.yv[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + NT * u;
      if (i < 1600) {
        const int p = i >> 2, c = 4 * (i & 3);
#pragma unroll
        for (int e = 0; e < 4; ++e) a1t[(c + e) * PS + p] = d.av[u][e];
      }
    }
  }

  __device__ __forceinline__ void run(int bid, float *smem) const {
    if (bid < B)
      image_block(bid, smem);
    else
      pair_block(bid - B, smem);
  }

  __device__ __forceinline__ void image_block(int b, float *smem) const {
    float *dyp = smem;                    // [11][11][DS]: dY2[oy][ox] at (oy + 1, ox + 1), zero border
    float *w2s = dyp + DY_FLOATS;         // [16 taps][16 ci][WS]
    float *a1t = w2s + W2_FLOATS;         // [16 ci][PS]: act1 transposed
    float *dat = a1t + MAP_FLOATS;        // [16 co][PS]: dact1 transposed
    uint8_t *xq = reinterpret_cast<uint8_t *>(dat + MAP_FLOATS);  // [4][4][4 ci][21][XROW]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    MT_PROBE_AT(3, b, 0);

    // ---- stage: every global load of the image (frame, W2, dY2, act1) issued before the LDS stores ----
    // frame item = (row y, quad jq): pixels 4qx .. 4qx+3 for qx = 4jq .. 4jq+3 (clamped to 20)
    const uint4 *xs = reinterpret_cast<const uint4 *>(X + (size_t)b * 84 * 84 * 4);  // 21 uint4 per row
    uint4 xv[4];
    {
      const int it = min(tid, 84 * 6 - 1), y = it / 6, jq = it - 6 * (it / 6);
#pragma unroll
      for (int v = 0; v < 4; ++v) xv[v] = xs[y * 21 + min(4 * jq + v, 20)];
    }
    const f32x4 *wsrc = reinterpret_cast<const f32x4 *>(W2);
    f32x4 wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = wsrc[tid + NT * u];
    const DyAct da = load_dy_act(b);
    store_dy_act(da, dyp, a1t);
    if (tid < 84 * 6) {
      const int y = tid / 6, jq = tid - 6 * (tid / 6);
      uint8_t *row = xq + (y & 3) * 16 * XPLANE + (y >> 2) * XROW + 4 * jq;
#pragma unroll
      for (int p = 0; p < 4; ++p) {  // pixel phase x & 3
        const uint32_t c0 = (&xv[0].x)[p], c1 = (&xv[1].x)[p], c2 = (&xv[2].x)[p], c3 = (&xv[3].x)[p];
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
          const uint32_t d = ((c0 >> (8 * ci)) & 255u) | (((c1 >> (8 * ci)) & 255u) << 8) |
                             (((c2 >> (8 * ci)) & 255u) << 16) | ((c3 >> (8 * ci)) << 24);
          *reinterpret_cast<uint32_t *>(row + (p * 4 + ci) * XPLANE) = d;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + NT * u;
      *reinterpret_cast<f32x4 *>(w2s + (i >> 3) * WS + 4 * (i & 7)) = wv[u];
    }
    __syncthreads();
    MT_PROBE_AT(3, b, 1);

    // ---- conv2 dX of stride phase w & 3, row tiles 4h .. 4h+3 (h = w >> 2; tile 7 is empty) ----
    {
      const int ph = w & 3, py = ph >> 1, px = ph & 1, t0 = 4 * (w >> 2);
      const int nt = w >> 2 ? 3 : 4;  // (wave-uniform)
      int off[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = min(16 * (t0 + t) + r, 99), qy = q / 10, qx = q - 10 * qy;
        off[t] = ((qy + 1) * 11 + qx + 1) * DS + 4 * g;
      }
      // chunk kc = (a, b, co half): B = W2[py+2a][px+2b][ci = r][co0 + 4g ..], A = dY2 rows
      auto frags = [&](int kc, f32x4 &bf, f32x4 (&af)[4]) {
        const int ab = kc >> 1, a = ab >> 1, bb = ab & 1, co0 = (kc & 1) * 16;
        bf = *reinterpret_cast<const f32x4 *>(w2s + (((py + 2 * a) * 4 + px + 2 * bb) * 16 + r) * WS + co0 + 4 * g);
#pragma unroll
        for (int t = 0; t < 4; ++t) af[t] = *reinterpret_cast<const f32x4 *>(dyp + off[t] - (a * 11 + bb) * DS + co0);
      };
      f32x4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 bf, af[4];
      frags(0, bf, af);
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        f32x4 bn, an[4];
        if (kc + 1 < 8) frags(kc + 1, bn, an);  // next chunk's operands in flight under these MFMAs
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < nt) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[t][s], bf[s], acc[t], 0, 0, 0);
        if (kc + 1 < 8) {
          bf = bn;
#pragma unroll
          for (int t = 0; t < 4; ++t) af[t] = an[t];
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 16 * (t0 + t) + 4 * g + i;
          if (q < 100) {
            const int qy = q / 10, qx = q - 10 * qy;
            const int p = (2 * qy + py) * 20 + 2 * qx + px;
            const float v = acc[t][i] * act_bwd(a1t[r * PS + p], act, alpha);
            dat[r * PS + p] = v;
            if (dact1) dact1[((size_t)b * 400 + p) * 16 + r] = v;
          }
        }
    }
    __syncthreads();
    MT_PROBE_AT(3, b, 2);

    // ---- conv1 dW: tiles m = 2w + mt (ky = w, kx = 4 mt + (r >> 2), ci = r & 3); db1 from the
    //      B fragments every wave reads (wave 0 writes it) ----
    {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      float db = 0.f;  // lane (r, g): dact1[co = r] over pixels 16 kc + 4 g .. + 3
      // the lane's plane row base: plane (ky & 3, kx & 3 = r >> 2, ci = r & 3), row offset ky >> 2
      const uint8_t *pl = xq + ((w & 3) * 16 + r) * XPLANE + (w >> 2) * XROW;
      // fragments of chunk kc: pixels p0 .. p0+3 = 16 kc + 4 g .. (one row: 20 % 4 == 0)
      auto frag = [&](int kc, f32x4 &bf, uint32_t &u0, uint32_t &u1) {
        const int p0 = 16 * kc + 4 * g, oy = p0 / 20, ox0 = p0 - 20 * oy;
        bf = *reinterpret_cast<const f32x4 *>(dat + r * PS + p0);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(pl + oy * XROW + ox0);
        u0 = src[0];                                           // kx >> 2 = 0
        u1 = __builtin_amdgcn_alignbyte(src[1], src[0], 1);  // kx >> 2 = 1: one byte further
      };
      f32x4 bf;
      uint32_t u0, u1;
      frag(0, bf, u0, u1);
#pragma unroll 5
      for (int kc = 0; kc < 25; ++kc) {
        f32x4 bn;
        uint32_t n0, n1;
        frag(min(kc + 1, 24), bn, n0, n1);  // next chunk's operands in flight under this chunk's MFMAs
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)((u0 >> (8 * s)) & 255u), bf[s], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)((u1 >> (8 * s)) & 255u), bf[s], acc[1], 0, 0, 0);
        }
        db += (bf[0] + bf[1]) + (bf[2] + bf[3]);
        bf = bn;
        u0 = n0;
        u1 = n1;
      }
      const float sc = 1.0f / 255.0f;  // networks.py:155
      float *o = slab1 + (size_t)b * SLAB1;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[(16 * (2 * w + mt) + 4 * g + i) * 16 + r] = acc[mt][i] * sc;
      db += __shfl_xor(db, 16, 64);
      db += __shfl_xor(db, 32, 64);
      if (w == 0 && lane < 16) o[256 * 16 + r] = db;
    }
    MT_PROBE_AT(3, b, 4);
  }

  // conv2 dW + db of images 2q, 2q+1 (one when B is odd and q is the last pair)
  __device__ __forceinline__ void pair_block(int q, float *smem) const {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int nimg = 2 * q + 1 < B ? 2 : 1;
    float *dyp[2] = {smem, smem + DY_FLOATS + MAP_FLOATS};
    float *a1t[2] = {smem + DY_FLOATS, smem + 2 * DY_FLOATS + MAP_FLOATS};
    MT_PROBE_AT(3, B + q, 0);
    const DyAct d0 = load_dy_act(2 * q), d1 = load_dy_act(min(2 * q + 1, B - 1));
    store_dy_act(d0, dyp[0], a1t[0]);
    if (nimg == 2) store_dy_act(d1, dyp[1], a1t[1]);
    __syncthreads();
    MT_PROBE_AT(3, B + q, 1);
    f32x4 acc[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) acc[mt][0] = acc[mt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db0 = 0.f, db1 = 0.f;  // lane (r, g): dY2[co = r / 16 + r] over the pixels 4 j + g
    const int ky = w >> 1, kx0 = 2 * (w & 1);
    for (int im = 0; im < nimg; ++im) {
      const float *dy = dyp[im], *at = a1t[im];
#pragma unroll 3
      for (int j = 0; j < 21; ++j) {
        const int p = 4 * j + g, pc = min(p, 80), oy = pc / 9, ox = pc - 9 * oy;
        const int yo = p < 81 ? ((oy + 1) * 11 + ox + 1) * DS : 0;  // pixel (0, 0) of the border: zeros
        const float b0 = dy[yo + r], b1 = dy[yo + 16 + r];
        const float *ap = at + r * PS + (2 * oy + ky) * 20 + 2 * ox + kx0;
        const float a0 = ap[0], a1 = ap[1];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        db0 += b0;
        db1 += b1;
      }
    }
    float *o = slab2 + (size_t)q * SLAB2;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[(16 * (2 * w + mt) + 4 * g + i) * 32 + 16 * n + r] = acc[mt][n][i];
    db0 += __shfl_xor(db0, 16, 64);
    db0 += __shfl_xor(db0, 32, 64);
    db1 += __shfl_xor(db1, 16, 64);
    db1 += __shfl_xor(db1, 32, 64);
    if (w == 0 && lane < 16) {
      o[256 * 32 + r] = db0;
      o[256 * 32 + 16 + r] = db1;
    }
    MT_PROBE_AT(3, B + q, 4);
  }
};

__global__ __launch_bounds__(NipsConvBwdJob::NT) void nips_conv_bwd_kernel(NipsConvBwdJob j) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  j.run(blockIdx.x, smem);
}

// Image blocks then pair blocks, one launch (512 threads: not a grouped-launch job).
inline int launch_nips_conv_bwd(hipStream_t s, const NipsConvBwdJob &j) {
  static_assert(NipsConvBwdJob::LDS <= 160 * 1024, "LDS budget");
  if (j.B <= 0 || !launch_allowed()) return MT_OK;
  static bool attr_set = false;
  if (!attr_set) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&nips_conv_bwd_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)NipsConvBwdJob::LDS));
    attr_set = true;
  }
  hipLaunchKernelGGL(nips_conv_bwd_kernel, dim3(j.blocks()), dim3(NipsConvBwdJob::NT), NipsConvBwdJob::LDS, s, j);
  MT_LAUNCHED();
  return MT_OK;
}

}  // namespace mt
