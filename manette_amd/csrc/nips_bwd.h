// Conv backward of the NIPS trunk (networks.py:178-192, gray frames: C = 4) with one workgroup per
// image: conv2 dX (stride phases) masked by conv1's activation derivative into LDS, then conv1 dW and
// conv2 dW of the image from LDS-resident operands, written as per-image slabs [257][16] and
// [257][32] (weights rows in HWIO order, then the bias row) that the next launch sums in image order
// (SlabJob). Replaces the layered path's two conv launches (trunk_backward: conv2 dX + conv2 dW,
// then conv1 dW + the conv2 slab sum), whose products re-read dact1, act1 and the frames from HBM
// and whose boundary costs a launch; here the only HBM traffic is each image's frame (28 KB), act1
// (25.6 KB), dact2 (10.4 KB), W2 (32 KB, L2) and the slabs.
//
// All products on v_mfma_f32_16x16x4_f32 (fp32). Lane (r, g) = (lane & 15, lane >> 4); an MFMA
// takes A[r][k_g], B[k_g][r] and accumulates C[4g + i][r] in acc[i].
//   conv2 dX: wave w = stride phase (py, px) = (w >> 1, w & 1) of the 20x20 input; rows = the 100
//     phase pixels (qy, qx) (7 tiles of 16, the last partial), K = (a, b, co) = 2 x 2 x 32:
//     dX[2qy+py][2qx+px][ci] = sum dY2[qy-a][qx-b][co] W2[py+2a][px+2b][ci][co] (dY2 zero-bordered).
//   conv1 dW: rows kr = (ky, kx, ci) (16 tiles, 4 per wave), K = the 400 output pixels:
//     dW1[kr][co] = sum_p X[4oy+ky][4ox+kx][ci] / 255 * dact1[p][co]; the frame is stored split by
//     the stride phase (ky & 3, kx & 3) so 4 consecutive pixels are 4 consecutive bytes.
//   conv2 dW: rows kr = (ky, kx, ci) (16 tiles x 2 channel halves, 8 per wave), K = the 81 output
//     pixels (+3 zero): dW2[kr][co] = sum_p act1[2oy+ky][2ox+kx][ci] dY2[p][co].
#pragma once
#include "gemm.h"

namespace mt {

struct NipsConvBwdJob {
  // frames [B][84][84][4] u8; act1 [B][20][20][16] (post-activation); dY2 = dact2 [B][9][9][32];
  // W2 [4][4][16][32]; dact1 (out, may be NULL) [B][20][20][16]; slab1 [B][257][16]; slab2 [B][257][32]
  const uint8_t *X = nullptr;
  const float *act1 = nullptr, *dY2 = nullptr, *W2 = nullptr;
  float *dact1 = nullptr, *slab1 = nullptr, *slab2 = nullptr;
  int B = 0, act = 0;
  float alpha = 0.f;

  static constexpr int XROW = 24;                // bytes per row of a phase plane (21 used)
  static constexpr int XPLANE = 21 * XROW;       // (ky & 3, kx & 3, ci) plane: 21 x 24 bytes
  static constexpr int X_BYTES = 64 * XPLANE;    // 32256
  static constexpr int DS = 36;                  // floats per zero-bordered dY2 pixel (11 x 11)
  static constexpr int DY_FLOATS = 11 * 11 * DS;
  static constexpr int WS = 36;                  // floats per (tap, ci) row of W2
  static constexpr int W2_FLOATS = 16 * 16 * WS;
  static constexpr int PS = 404;                 // floats per channel of the transposed 20x20 maps
  static constexpr int MAP_FLOATS = 16 * PS;
  static constexpr int RED_FLOATS = 512;
  static constexpr int SLAB1 = 257 * 16, SLAB2 = 257 * 32;

  __host__ __device__ int blocks() const { return B; }
  size_t lds() const { return X_BYTES + sizeof(float) * (DY_FLOATS + W2_FLOATS + 2 * MAP_FLOATS + RED_FLOATS); }

  __device__ __forceinline__ void run(int b, float *smem) const {
    float *dyp = smem;                    // [11][11][DS]: dY2[oy][ox] at (oy + 1, ox + 1), zero border
    float *w2s = dyp + DY_FLOATS;         // [16 taps][16 ci][WS]
    float *a1t = w2s + W2_FLOATS;         // [16 ci][PS]: act1 transposed
    float *dat = a1t + MAP_FLOATS;        // [16 co][PS]: dact1 transposed
    float *red = dat + MAP_FLOATS;        // bias partials
    uint8_t *xq = reinterpret_cast<uint8_t *>(red + RED_FLOATS);  // [4][4][4 ci][21][XROW]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, g = lane >> 4;

    // ---- stage: every global load of the image issued before the first LDS write ----
    const uint4 *xs = reinterpret_cast<const uint4 *>(X + (size_t)b * 84 * 84 * 4);  // 21 uint4 per row
    uint4 xv[2][4];  // item = (row y, quad jq): pixels 4qx .. 4qx+3 for qx = 4jq .. 4jq+3 (clamped to 20)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = min(tid + 256 * u, 84 * 6 - 1), y = it / 6, jq = it - 6 * (it / 6);
#pragma unroll
      for (int v = 0; v < 4; ++v) xv[u][v] = xs[y * 21 + min(4 * jq + v, 20)];
    }
    const f32x4 *ys = reinterpret_cast<const f32x4 *>(dY2 + (size_t)b * 81 * 32);
    f32x4 yv[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) yv[u] = ys[min(tid + 256 * u, 647)];
    const f32x4 *wsrc = reinterpret_cast<const f32x4 *>(W2);
    f32x4 wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) wv[u] = wsrc[tid + 256 * u];
    const f32x4 *as = reinterpret_cast<const f32x4 *>(act1 + (size_t)b * 400 * 16);
    f32x4 av[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) av[u] = as[min(tid + 256 * u, 1599)];

    // dY2's zero border (40 pixels x 8 quads)
    for (int i = tid; i < 121 * 8; i += 256) {
      const int p = i >> 3, Y = p / 11, Xc = p - 11 * Y;
      if (Y == 0 || Y == 10 || Xc == 0 || Xc == 10)
        *reinterpret_cast<f32x4 *>(dyp + p * DS + 4 * (i & 7)) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = tid + 256 * u;
      if (it < 84 * 6) {
        const int y = it / 6, jq = it - 6 * (it / 6);
        uint8_t *row = xq + (y & 3) * 16 * XPLANE + (y >> 2) * XROW + 4 * jq;
#pragma unroll
        for (int p = 0; p < 4; ++p) {  // pixel phase x & 3
          const uint32_t c0 = (&xv[u][0].x)[p], c1 = (&xv[u][1].x)[p], c2 = (&xv[u][2].x)[p], c3 = (&xv[u][3].x)[p];
#pragma unroll
          for (int ci = 0; ci < 4; ++ci) {
            const uint32_t d = ((c0 >> (8 * ci)) & 255u) | (((c1 >> (8 * ci)) & 255u) << 8) |
                               (((c2 >> (8 * ci)) & 255u) << 16) | ((c3 >> (8 * ci)) << 24);
            *reinterpret_cast<uint32_t *>(row + (p * 4 + ci) * XPLANE) = d;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int i = tid + 256 * u;
      if (i < 648) {
        const int p = i >> 3, oy = p / 9, ox = p - 9 * oy;
        *reinterpret_cast<f32x4 *>(dyp + ((oy + 1) * 11 + ox + 1) * DS + 4 * (i & 7)) = yv[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = tid + 256 * u;
      *reinterpret_cast<f32x4 *>(w2s + (i >> 3) * WS + 4 * (i & 7)) = wv[u];
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int i = tid + 256 * u;
      if (i < 1600) {
        const int p = i >> 2, c = 4 * (i & 3);
#pragma unroll
        for (int e = 0; e < 4; ++e) a1t[(c + e) * PS + p] = av[u][e];
      }
    }
    __syncthreads();

    // ---- conv2 dX of stride phase w, masked by act1's derivative -> dat (and dact1) ----
    {
      const int py = w >> 1, px = w & 1;
      int off[7];
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        const int q = min(16 * t + r, 99), qy = q / 10, qx = q - 10 * qy;
        off[t] = ((qy + 1) * 11 + qx + 1) * DS + 4 * g;
      }
      f32x4 acc[7];
#pragma unroll
      for (int t = 0; t < 7; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        const int ab = kc >> 1, a = ab >> 1, bb = ab & 1, co0 = (kc & 1) * 16;
        const f32x4 bf = *reinterpret_cast<const f32x4 *>(w2s + (((py + 2 * a) * 4 + px + 2 * bb) * 16 + r) * WS + co0 + 4 * g);
        f32x4 af[7];
#pragma unroll
        for (int t = 0; t < 7; ++t) af[t] = *reinterpret_cast<const f32x4 *>(dyp + off[t] - (a * 11 + bb) * DS + co0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < 7; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[t][s], bf[s], acc[t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 7; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 16 * t + 4 * g + i;
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

    // ---- bias rows: db1[co] = sum of dact1 over the 400 pixels, db2[co] = sum of dY2 over 81 ----
    {
      const int c1 = tid & 15, s1 = tid >> 4;  // 16 pixel ranges of 25
      float t1 = 0.f;
      for (int p = 25 * s1; p < 25 * s1 + 25; ++p) t1 += dat[c1 * PS + p];
      red[tid] = t1;
      const int c2 = tid & 31, s2 = tid >> 5;  // 8 pixel subsets p = s2 + 8j
      float t2 = 0.f;
      for (int p = s2; p < 81; p += 8) t2 += dyp[((p / 9 + 1) * 11 + p % 9 + 1) * DS + c2];
      red[256 + tid] = t2;
    }
    __syncthreads();
    if (tid < 16) {
      float t = red[tid];
#pragma unroll
      for (int u = 1; u < 16; ++u) t += red[16 * u + tid];
      slab1[(size_t)b * SLAB1 + 256 * 16 + tid] = t;
    } else if (tid >= 64 && tid < 96) {
      const int c = tid - 64;
      float t = red[256 + c];
#pragma unroll
      for (int u = 1; u < 8; ++u) t += red[256 + 32 * u + c];
      slab2[(size_t)b * SLAB2 + 256 * 32 + c] = t;
    }

    // ---- conv1 dW: tiles m = 4w .. 4w+3 (ky = m >> 1, kx = 4 (m & 1) + (r >> 2), ci = r & 3) ----
    {
      f32x4 acc[4];
      int pl[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int ky = 2 * w + (mt >> 1);
        pl[mt] = ((ky & 3) * 16 + r) * XPLANE + (ky >> 2) * XROW;
      }
      const float sc = 1.0f / 255.0f;  // networks.py:155
#pragma unroll 5
      for (int kc = 0; kc < 25; ++kc) {
        const int p0 = 16 * kc + 4 * g, oy = p0 / 20, ox0 = p0 - 20 * oy;
        const f32x4 bf = *reinterpret_cast<const f32x4 *>(dat + r * PS + p0);
        const int ro = oy * XROW + ox0;
        f32x4 af[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const uint32_t *src = reinterpret_cast<const uint32_t *>(xq + pl[mt] + ro);
          const uint32_t u = (mt & 1) ? __builtin_amdgcn_alignbyte(src[1], src[0], 1) : src[0];
#pragma unroll
          for (int s = 0; s < 4; ++s) af[mt][s] = (float)((u >> (8 * s)) & 255u) * sc;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt][s], bf[s], acc[mt], 0, 0, 0);
      }
      float *o = slab1 + (size_t)b * SLAB1;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[(16 * (4 * w + mt) + 4 * g + i) * 16 + r] = acc[mt][i];
    }

    // ---- conv2 dW: tiles m = 4w + mt (ky = w, kx = mt, ci = r) x channel halves n ----
    {
      f32x4 acc[4][2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt][0] = acc[mt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
      for (int j = 0; j < 21; ++j) {
        const int p = 4 * j + g, pc = min(p, 80), oy = pc / 9, ox = pc - 9 * oy;
        const int yo = p < 81 ? ((oy + 1) * 11 + ox + 1) * DS : 0;  // pixel (0, 0) of the border: zeros
        const float b0 = dyp[yo + r], b1 = dyp[yo + 16 + r];
        const float *ap = a1t + r * PS + (2 * oy + w) * 20 + 2 * ox;
        float a[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) a[mt] = ap[mt];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt], b0, acc[mt][0], 0, 0, 0);
          acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt], b1, acc[mt][1], 0, 0, 0);
        }
      }
      float *o = slab2 + (size_t)b * SLAB2;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[(16 * (4 * w + mt) + 4 * g + i) * 32 + 16 * n + r] = acc[mt][n][i];
    }
  }
};

}  // namespace mt
