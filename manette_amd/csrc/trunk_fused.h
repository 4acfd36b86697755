// Fused NIPS trunk for the rollout-batch forward (E small, latency-bound): one launch computes
// conv1 -> conv2 -> the dense layer's partial products (networks.py:178-192, :57-70), replacing
// three GEMM launches (conv1, conv2, split-K fc). Only the inference forward uses it (rollout
// steps and the bootstrap V(s_T)): no activations are kept for a backward pass.
//
// Workgroup = (env e, conv2 output row i), 9 per env. Its conv2 row reads conv1 rows 2i..2i+3,
// which read input rows 8i..8i+19: the block stages those 20 uint8 rows (contiguous in NHWC) in
// LDS, recomputes its 4 conv1 rows (1.8x the conv1 FLOPs over the 9 blocks of an env, in exchange
// for no inter-block hand-off), computes its conv2 row, and multiplies that row's 288 features by
// the matching 288 rows of the fc weight: the slab z = i of the split-K layout heads_fwd_kernel
// finishes (sum of the 9 slabs in fixed order + bias + act, heads, softmax, A3 draw).
//
// Convs run on v_mfma_f32_16x16x4_f32 (exact fp32) with the 4 waves splitting K; the 4 partial
// accumulators are added in wave order through LDS (deterministic). Input scaling x = u8 * (1/255)
// in fp32 as networks.py:155 (same expression as LdIm2col's loader).
//
// blockIdx -> (i, e) is XCD-aware: blocks are dealt round-robin over the 8 XCDs, so the linear
// index L = (bid % 8) * (grid / 8) + bid / 8 gives each XCD a contiguous run of L, i.e. 1-2 conv2
// rows, and the 295 KB fc weight chunk of a row is read from HBM by one or two XCDs' L2s instead
// of all eight (speed only; any placement computes the same values).
#pragma once
#include "gemm.h"

namespace mt {

template <int C>
struct FusedNips {
  static constexpr int ROWS2 = 9;         // conv2 output rows = blocks per env
  static constexpr int ROWS1 = 4;         // conv1 rows a block computes
  static constexpr int RIN = 20;          // input rows a block stages
  static constexpr int OW1 = 20, CO1 = 16, KK1 = 64 * C;
  static constexpr int OW2 = 9, CO2 = 32, KK2 = 256;
  static constexpr int A1S = 20;          // padded float stride of one conv1 pixel in LDS
  static constexpr int FEAT = OW2 * CO2;  // 288 features per conv2 row
  static constexpr int F = 256;
  static constexpr int M1 = ROWS1 * OW1;  // 80 conv1 pixels
  static constexpr int MT1 = (M1 + 15) / 16;  // 5 m-tiles
  static constexpr int KC1 = KK1 / 16, KC2 = KK2 / 16;
  static_assert(KC1 % 4 == 0 && KC2 % 4 == 0, "K chunks split over 4 waves");
  static constexpr int IN_BYTES = RIN * 84 * C;
  // LDS (floats unless noted)
  static constexpr int RED_FLOATS = 4 * MT1 * 16 * CO1;  // >= 4*16*32 (conv2) and 4*256 (fc)
  static constexpr size_t LDS_BYTES = IN_BYTES + sizeof(float) * (RED_FLOATS + M1 * A1S + FEAT);
};

// One block's work: conv2 row i of env e -> its fc partial slab. Returns e (the env).
// act1 / act2 (optional): [B][20][20][16] conv1 and [B][9][9][32] conv2 activations of this
// batch (rows of a train workspace, mt_forward_rows); block (e, i) writes conv1 rows 2i, 2i+1
// (the last block also 18, 19) and conv2 row i, so every value is written once.
template <int C>
__device__ __forceinline__ int nips_trunk_block(const uint8_t *__restrict__ obs, int B, const float *__restrict__ W1,
                                                const float *__restrict__ W2, const float *__restrict__ Wfc, int act,
                                                float alpha, float *__restrict__ slabs, float *smem,
                                                float *__restrict__ act1, float *__restrict__ act2) {
  using Fz = FusedNips<C>;
  float *red = smem;                              // [4 waves][..] partial accumulators
  float *a1 = red + Fz::RED_FLOATS;               // [80 pixels][A1S] conv1 rows 2i..2i+3
  float *a2 = a1 + Fz::M1 * Fz::A1S;              // [288] conv2 row i (NHWC flatten order)
  uint8_t *xin = reinterpret_cast<uint8_t *>(a2 + Fz::FEAT);  // [20][84][C] input rows 8i..

  const int nb = gridDim.x;
  const int bid = blockIdx.x;
  const int L = (nb % 8 == 0) ? (bid % 8) * (nb / 8) + bid / 8 : bid;
  const int i = L / B, e = L - i * B;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;

  // ---- stage input rows 8i..8i+19 (one contiguous run of 20*84*C bytes) ----
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(obs + ((size_t)e * 84 + 8 * i) * 84 * C);
    uint4 *dst = reinterpret_cast<uint4 *>(xin);
    for (int q = threadIdx.x; q < Fz::IN_BYTES / 16; q += 256) dst[q] = src[q];
  }
  // conv1 weight fragments of this wave's K chunks (c = w + 4j): B[k][n] = W1[k*16 + n]
  constexpr int J1 = Fz::KC1 / 4;
  float b1f[J1][4];
#pragma unroll
  for (int j = 0; j < J1; ++j) {
    const int k0 = 16 * (w + 4 * j) + 4 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) b1f[j][s] = W1[(size_t)(k0 + s) * Fz::CO1 + r];
  }
  __syncthreads();

  // ---- conv1 (VALID 8x8 stride 4): M = 80 pixels (4 rows x 20), N = 16, K = 64*C ----
  {
    f32x4 acc[Fz::MT1];
#pragma unroll
    for (int t = 0; t < Fz::MT1; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float sc = 1.0f / 255.0f;
#pragma unroll
    for (int j = 0; j < J1; ++j) {
      const int k0 = 16 * (w + 4 * j) + 4 * g;
      const int kpos = k0 / C, ci = k0 - kpos * C;
      const int ky = kpos >> 3, kx = kpos & 7;
      f32x4 a[Fz::MT1];
#pragma unroll
      for (int t = 0; t < Fz::MT1; ++t) {
        const int m = min(t * 16 + r, Fz::M1 - 1);
        const int orow = m / Fz::OW1, ox = m - orow * Fz::OW1;
        const uint32_t u = *reinterpret_cast<const uint32_t *>(xin + ((4 * orow + ky) * 84 + 4 * ox + kx) * C + ci);
        a[t] = f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc, (float)((u >> 16) & 0xff) * sc,
                     (float)(u >> 24) * sc};
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < Fz::MT1; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][s], b1f[j][s], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < Fz::MT1; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(w * Fz::MT1 * 16 + t * 16 + g * 4 + q) * Fz::CO1 + r] = acc[t][q];
  }
  // conv2 weight fragments (issued before the barrier so their latency overlaps the reduction)
  constexpr int J2 = Fz::KC2 / 4;
  float b2f[J2][2][4];
#pragma unroll
  for (int j = 0; j < J2; ++j) {
    const int k0 = 16 * (w + 4 * j) + 4 * g;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s = 0; s < 4; ++s) b2f[j][nt][s] = W2[(size_t)(k0 + s) * Fz::CO2 + nt * 16 + r];
  }
  __syncthreads();
  {
    const float *b1 = W1 + (size_t)Fz::KK1 * Fz::CO1;
    constexpr int P = Fz::MT1 * 16 * Fz::CO1;  // stride of one wave's partials
    for (int idx = threadIdx.x; idx < Fz::M1 * Fz::CO1; idx += 256) {
      const int m = idx / Fz::CO1, n = idx - m * Fz::CO1;
      const float s = ((red[idx] + red[P + idx]) + red[2 * P + idx]) + red[3 * P + idx];
      const float y = act_fwd(s + b1[n], act, alpha);
      a1[m * Fz::A1S + n] = y;
      if (act1 && (m < 2 * Fz::OW1 || i == Fz::ROWS2 - 1))  // conv1 rows 2i, 2i+1 (+ 18, 19)
        act1[(((size_t)e * Fz::OW1 + 2 * i) * Fz::OW1 + m) * Fz::CO1 + n] = y;
    }
  }
  __syncthreads();

  // ---- conv2 row i (VALID 4x4 stride 2): M = 9 pixels (padded to 16), N = 32, K = 256 ----
  {
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int ox = min(r, Fz::OW2 - 1);
#pragma unroll
    for (int j = 0; j < J2; ++j) {
      const int c = w + 4 * j;  // (ky, kx) = (c / 4, c % 4), channels 4g..4g+3
      const int ky = c >> 2, kx = c & 3;
      const f32x4 a = *reinterpret_cast<const f32x4 *>(a1 + (ky * Fz::OW1 + 2 * ox + kx) * Fz::A1S + 4 * g);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b2f[j][nt][s], acc[nt], 0, 0, 0);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(w * 16 + g * 4 + q) * Fz::CO2 + nt * 16 + r] = acc[nt][q];
  }
  __syncthreads();
  {
    const float *b2 = W2 + (size_t)Fz::KK2 * Fz::CO2;
    constexpr int P = 16 * Fz::CO2;
    for (int idx = threadIdx.x; idx < Fz::FEAT; idx += 256) {
      const int n = idx & (Fz::CO2 - 1);
      const float s = ((red[idx] + red[P + idx]) + red[2 * P + idx]) + red[3 * P + idx];
      const float y = act_fwd(s + b2[n], act, alpha);
      a2[idx] = y;
      if (act2) act2[((size_t)e * Fz::ROWS2 + i) * Fz::FEAT + idx] = y;
    }
  }
  __syncthreads();

  // ---- fc partial: slab[i][e][n] = sum_{f < 288} a2[f] * Wfc[i*288 + f][n] ----
  {
    const int c4 = threadIdx.x & 63, fg = threadIdx.x >> 6;  // 4 output columns x 72 features
    constexpr int FPG = Fz::FEAT / 4;
    const f32x4 *wp = reinterpret_cast<const f32x4 *>(Wfc + ((size_t)i * Fz::FEAT + fg * FPG) * Fz::F) + c4;
    const float *xp = a2 + fg * FPG;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int f = 0; f < FPG; ++f) acc += xp[f] * wp[(size_t)f * (Fz::F / 4)];
    reinterpret_cast<f32x4 *>(red)[fg * 64 + c4] = acc;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const f32x4 *rp = reinterpret_cast<const f32x4 *>(red);
    const f32x4 s = ((rp[threadIdx.x] + rp[64 + threadIdx.x]) + rp[128 + threadIdx.x]) + rp[192 + threadIdx.x];
    reinterpret_cast<f32x4 *>(slabs + ((size_t)i * B + e) * Fz::F)[threadIdx.x] = s;
  }
  return e;
}

template <int C>
__global__ __launch_bounds__(256) void nips_fused_trunk_kernel(const uint8_t *__restrict__ obs, int B,
                                                               const float *__restrict__ W1,
                                                               const float *__restrict__ W2,
                                                               const float *__restrict__ Wfc, int act,
                                                               float alpha, float *__restrict__ slabs,
                                                               float *__restrict__ act1, float *__restrict__ act2) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  (void)nips_trunk_block<C>(obs, B, W1, W2, Wfc, act, alpha, slabs, smem, act1, act2);
}

}  // namespace mt
