// Conv backward of the NIPS trunk (networks.py:178-192, gray frames: C = 4) with one workgroup per
// image: conv2 dX (stride phases) masked by conv1's activation derivative into LDS, then conv1 dW and
// conv2 dW of the image from LDS-resident operands, written as per-image slabs [257][16] and
// [257][32] (weights rows in HWIO order, then the bias row) that the next launch sums in image order
// (SlabJob). Replaces the layered path's two conv launches (trunk_backward: conv2 dX + conv2 dW,
// then conv1 dW + the conv2 slab sum), whose products re-read dact1, act1 and the frames from HBM
// and whose boundary costs a launch; here the only HBM traffic is each image's frame (28 KB), act1
// (25.6 KB), dact2 (10.4 KB), W2 (32 KB, L2) and the slabs.
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
//   conv2 dW: rows kr = (ky, kx, ci) (16 tiles x 2 channel halves, 4 per wave), K = the 81 output
//     pixels (+3 zero): dW2[kr][co] = sum_p act1[2oy+ky][2ox+kx][ci] dY2[p][co].
#pragma once
#include "gemm.h"
#include "trunk_fused.h"  // (MT_PROBE_AT: probe builds time the phases of block b in slot 3)

namespace mt {

struct NipsConvBwdJob {
  // frames [B][84][84][4] u8; act1 [B][20][20][16] (post-activation); dY2 = dact2 [B][9][9][32];
  // W2 [4][4][16][32]; dact1 (out, may be NULL) [B][20][20][16]; slab1 [B][257][16]; slab2 [B][257][32]
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
  static constexpr int RED_FLOATS = 2 * NT;
  static constexpr int SLAB1 = 257 * 16, SLAB2 = 257 * 32;
  static constexpr size_t LDS = X_BYTES + sizeof(float) * (DY_FLOATS + W2_FLOATS + 2 * MAP_FLOATS + RED_FLOATS);

  __device__ __forceinline__ void run(int b, float *smem) const {
    float *dyp = smem;                    // [11][11][DS]: dY2[oy][ox] at (oy + 1, ox + 1), zero border
    float *w2s = dyp + DY_FLOATS;         // [16 taps][16 ci][WS]
    float *a1t = w2s + W2_FLOATS;         // [16 ci][PS]: act1 transposed
    float *dat = a1t + MAP_FLOATS;        // [16 co][PS]: dact1 transposed
    float *red = dat + MAP_FLOATS;        // bias partials
    uint8_t *xq = reinterpret_cast<uint8_t *>(red + RED_FLOATS);  // [4][4][4 ci][21][XROW]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    MT_PROBE_AT(3, b, 0);

    // ---- stage: every global load of the image issued before the first LDS write ----
    // frame item = (row y, quad jq): pixels 4qx .. 4qx+3 for qx = 4jq .. 4jq+3 (clamped to 20)
    const uint4 *xs = reinterpret_cast<const uint4 *>(X + (size_t)b * 84 * 84 * 4);  // 21 uint4 per row
    uint4 xv[4];
    {
      const int it = min(tid, 84 * 6 - 1), y = it / 6, jq = it - 6 * (it / 6);
#pragma unroll
      for (int v = 0; v < 4; ++v) xv[v] = xs[y * 21 + min(4 * jq + v, 20)];
    }
    const f32x4 *ys = reinterpret_cast<const f32x4 *>(dY2 + (size_t)b * 81 * 32);
    f32x4 yv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) yv[u] = ys[min(tid + NT * u, 647)];
    const f32x4 *wsrc = reinterpret_cast<const f32x4 *>(W2);
    f32x4 wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = wsrc[tid + NT * u];
    const f32x4 *as = reinterpret_cast<const f32x4 *>(act1 + (size_t)b * 400 * 16);
    f32x4 av[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) av[u] = as[min(tid + NT * u, 1599)];

    // dY2's zero border (40 pixels x 8 quads)
    for (int i = tid; i < 121 * 8; i += NT) {
      const int p = i >> 3, Y = p / 11, Xc = p - 11 * Y;
      if (Y == 0 || Y == 10 || Xc == 0 || Xc == 10)
        *reinterpret_cast<f32x4 *>(dyp + p * DS + 4 * (i & 7)) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
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
    for (int u = 0; u < 2; ++u) {
      const int i = tid + NT * u;
      if (i < 648) {
        const int p = i >> 3, oy = p / 9, ox = p - 9 * oy;
        *reinterpret_cast<f32x4 *>(dyp + ((oy + 1) * 11 + ox + 1) * DS + 4 * (i & 7)) = yv[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + NT * u;
      *reinterpret_cast<f32x4 *>(w2s + (i >> 3) * WS + 4 * (i & 7)) = wv[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + NT * u;
      if (i < 1600) {
        const int p = i >> 2, c = 4 * (i & 3);
#pragma unroll
        for (int e = 0; e < 4; ++e) a1t[(c + e) * PS + p] = av[u][e];
      }
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
      f32x4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        const int ab = kc >> 1, a = ab >> 1, bb = ab & 1, co0 = (kc & 1) * 16;
        const f32x4 bf = *reinterpret_cast<const f32x4 *>(w2s + (((py + 2 * a) * 4 + px + 2 * bb) * 16 + r) * WS + co0 + 4 * g);
        f32x4 af[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) af[t] = *reinterpret_cast<const f32x4 *>(dyp + off[t] - (a * 11 + bb) * DS + co0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < nt) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[t][s], bf[s], acc[t], 0, 0, 0);
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

    // ---- bias rows: db1[co] = sum of dact1 over the 400 pixels, db2[co] = sum of dY2 over 81 ----
    {
      const int c1 = tid & 15, s1 = tid >> 4;  // 32 pixel ranges of 13 (the last one 3)
      float t1 = 0.f;
      for (int p = 13 * s1; p < min(400, 13 * s1 + 13); ++p) t1 += dat[c1 * PS + p];
      red[tid] = t1;
      const int c2 = tid & 31, s2 = tid >> 5;  // 16 pixel subsets p = s2 + 16j
      float t2 = 0.f;
      for (int p = s2; p < 81; p += 16) t2 += dyp[((p / 9 + 1) * 11 + p % 9 + 1) * DS + c2];
      red[NT + tid] = t2;
    }
    __syncthreads();
    if (tid < 16) {
      float t = red[tid];
#pragma unroll
      for (int u = 1; u < 32; ++u) t += red[16 * u + tid];
      slab1[(size_t)b * SLAB1 + 256 * 16 + tid] = t;
    } else if (tid >= 64 && tid < 96) {
      const int c = tid - 64;
      float t = red[NT + c];
#pragma unroll
      for (int u = 1; u < 16; ++u) t += red[NT + 32 * u + c];
      slab2[(size_t)b * SLAB2 + 256 * 32 + c] = t;
    }
    MT_PROBE_AT(3, b, 3);

    // ---- conv1 dW: tiles m = 2w + mt (ky = w, kx = 4 mt + (r >> 2), ci = r & 3) ----
    {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
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
    }
    MT_PROBE_AT(3, b, 4);

    // ---- conv2 dW: tiles m = 2w + mt (ky = w >> 1, kx = 2 (w & 1) + mt, ci = r) x channel halves ----
    {
      f32x4 acc[2][2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) acc[mt][0] = acc[mt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int ky = w >> 1, kx0 = 2 * (w & 1);
#pragma unroll 3
      for (int j = 0; j < 21; ++j) {
        const int p = 4 * j + g, pc = min(p, 80), oy = pc / 9, ox = pc - 9 * oy;
        const int yo = p < 81 ? ((oy + 1) * 11 + ox + 1) * DS : 0;  // pixel (0, 0) of the border: zeros
        const float b0 = dyp[yo + r], b1 = dyp[yo + 16 + r];
        const float *ap = a1t + r * PS + (2 * oy + ky) * 20 + 2 * ox + kx0;
        const float a0 = ap[0], a1 = ap[1];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      }
      float *o = slab2 + (size_t)b * SLAB2;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[(16 * (2 * w + mt) + 4 * g + i) * 32 + 16 * n + r] = acc[mt][n][i];
    }
    MT_PROBE_AT(3, b, 5);
  }
};

__global__ __launch_bounds__(NipsConvBwdJob::NT) void nips_conv_bwd_kernel(NipsConvBwdJob j) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  j.run(blockIdx.x, smem);
}

// One workgroup per image (its own launch: 512 threads, not a grouped-launch job).
inline int launch_nips_conv_bwd(hipStream_t s, const NipsConvBwdJob &j) {
  static_assert(NipsConvBwdJob::LDS <= 160 * 1024, "LDS budget");
  if (j.B <= 0 || !launch_allowed()) return MT_OK;
  static bool attr_set = false;
  if (!attr_set) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&nips_conv_bwd_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)NipsConvBwdJob::LDS));
    attr_set = true;
  }
  hipLaunchKernelGGL(nips_conv_bwd_kernel, dim3(j.B), dim3(NipsConvBwdJob::NT), NipsConvBwdJob::LDS, s, j);
  MT_LAUNCHED();
  return MT_OK;
}

}  // namespace mt
