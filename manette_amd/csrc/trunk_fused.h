// NIPS trunk of the inference forward (rollout steps, bootstrap V(s_T)), E small and
// latency-bound: networks.py:178-192 (conv1 -> conv2) and :57-70 (the dense layer's products) as
// two launches, whose 9 split-K slabs heads_fwd_kernel finishes (sum in fixed order + bias + act,
// heads, softmax, A3 draw).
//
// 1. nips_conv_kernel — workgroup = (env e, conv2 output row i), 9 per env. Its conv2 row reads
//    conv1 rows 2i..2i+3, which read input rows 8i..8i+19: the block stages those 20 uint8 rows
//    (contiguous in NHWC) in LDS, recomputes its 4 conv1 rows (1.8x the conv1 FLOPs over the 9
//    blocks of an env, in exchange for no inter-block hand-off), computes its conv2 row and
//    writes those 288 activations to act2 [B][2592] (NHWC flatten order).
//    STACK variant (the pipelined rollout, resized staging): the block also does the A2 stacking
//    of mt_preprocess_resized (atari_emulator.py:79-124, environment.py:42-80) for its rows — the
//    previous state's rows from HBM and the env's p new final frames, stacked in LDS, the block's
//    own rows (8i..8i+7; the last block 64..83) written to the new state slot — so no separate
//    preprocess launch sits on the step's critical path. With ready words (in-kernel pull, the
//    rollout chain) each block waits for ITS env's publication by the emulator thread and reads
//    the frames from the pinned staging itself: an env's convs run while the later envs are still
//    being emulated, with no pull kernel and no kernel boundary in front of them.
// 2. nips_fc_kernel — the dense layer as a real GEMM: block = (16 output columns, K-split i of 8,
//    16 envs); slab[i][e][n] = sum over split i's features f of act2[e][f] Wfc[f][n] on MFMA. Each
//    fc weight is read once per 16 envs (the former one-launch trunk streamed the row's 295 KB
//    weight chunk through every (env, row) block: 85 MB of L2 -> CU traffic at E = 32).
//
// Convs and fc run on v_mfma_f32_16x16x4_f32 (exact fp32) with the 4 waves splitting K; the 4
// partial accumulators are added in wave order through LDS (deterministic). Input scaling
// x = u8 * (1/255) in fp32 as networks.py:155 (same expression as LdIm2col's loader).
//
// blockIdx -> (e, i) of the conv kernel is XCD-aware: blocks are dealt round-robin over the 8
// XCDs, so the linear index L = (bid % 8) * (grid / 8) + bid / 8 gives each XCD a contiguous run
// of L, env-major (L = 9 e + i): the 9 blocks of an env, whose 20-row input windows overlap by
// 12 rows, share one XCD's L2, so each frame crosses the fabric once, not 2.5 times. The fc
// kernel deals its (16-column, row i) blocks the same way, i-major: an XCD holds the 16 column
// blocks of 1-2 rows, so each 128-byte weight line (two 16-column halves) and each act2 row
// chunk is fetched by one XCD (speed only; any placement computes the same values).
#pragma once
#include "gemm.h"

// Phase timestamps (experiment builds only, -DMT_PROBE: build_hip(out=..., defines=['MT_PROBE'])):
// s_memrealtime (100 MHz, one clock for the whole device) of lane 0 at phase boundaries of every
// block of the rollout-forward kernels, read back with mt_probe_read (tools/probe.py).
#ifdef MT_PROBE
static __device__ unsigned long long mt_probe_buf[5 * 1024 * 8];  // kernels 0-2 rollout, 3 conv bwd, 4 loss
#define MT_PROBE_AT(k, b, p)                                                                     \
  do {                                                                                           \
    if (threadIdx.x == 0 && (b) < 1024) mt_probe_buf[((k) * 1024 + (b)) * 8 + (p)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define MT_PROBE_AT(k, b, p) \
  do {                       \
  } while (0)
#endif

namespace mt {

template <int C>
struct FusedNips {
  static constexpr int D = C / 4;         // 1 gray, 3 RGB
  static constexpr int ROWS2 = 9;         // conv2 output rows = blocks per env
  static constexpr int ROWS1 = 4;         // conv1 rows a block computes
  static constexpr int RIN = 20;          // input rows a block stages
  static constexpr int OW1 = 20, CO1 = 16, KK1 = 64 * C;
  static constexpr int OW2 = 9, CO2 = 32, KK2 = 256;
  static constexpr int A1S = 20;          // padded float stride of one conv1 pixel in LDS
  static constexpr int FEAT = OW2 * CO2;  // 288 features per conv2 row
  static constexpr int FLAT = ROWS2 * FEAT;
  static constexpr int F = 256;
  // (Half-row blocks — an env's chain over 18 blocks, half the conv1 MFMAs each — measured in
  // round 3: conv1 phase 2.60 vs 2.84 us, but the tail after the last publish unchanged and the
  // isolated trunk slower, 14.3 vs 13.6 us; profiles/r03p/.)
  static constexpr int BPE = ROWS2;       // blocks per env
  static constexpr int M1 = ROWS1 * OW1;  // conv1 pixels of a block (80)
  static constexpr int MT1 = (M1 + 15) / 16;  // m-tiles (5)
  static constexpr int KC1 = KK1 / 16, KC2 = KK2 / 16;
  // conv kernel waves. Gray frames: 8 waves, 2 per SIMD (waves w and w + 4 share SIMD w & 3).
  // conv1 "units": M-tiles 0-3 x 2 K-halves on waves 0-7 (32 MFMAs each), M-tile 4 x 4 K-quarters
  // on waves 0-3 (16 more each), so every SIMD issues 80 of the block's 320 conv1 MFMAs (round 5 ran
  // 10 waves, tiles 0-4 x 2 K-halves: SIMDs 0 and 1 held three units, 96 MFMAs, beside 64 — the
  // probe put the conv1 phase at 3.1 us, 1.7 of them MFMA issue); conv2 = 2 N-tiles x 4 K-quarters,
  // 4 partials. (The former 8-wave K-split — every wave all 5 tiles over 1/8 of K — spent ~1.1 us per
  // block writing and reducing 8 partials per output.) RGB: 4 waves splitting K (its 3x input rows
  // would not fit 64 KB of LDS beside more waves' partials).
  static constexpr int NW = C == 4 ? 8 : 4, NT = 64 * NW;
  static constexpr bool UNITS = C == 4;
  static constexpr int U1 = UNITS ? 2 * (MT1 - 1) + 4 : 0;  // conv1 partial slots: 8 half units + 4 quarters
  static_assert(UNITS ? (C == 4 && KC1 == 16 && KC2 == 16 && MT1 == 5 && NW == 8)
                      : (KC1 % NW == 0 && KC2 % NW == 0), "K chunks split over the waves");
  static constexpr int IN_BYTES = RIN * 84 * C;
  static constexpr int FR_BYTES = RIN * 84 * D;  // the block's rows of one new frame
  // LDS (floats unless noted)
  static constexpr int RED_UNITS = (U1 > 8 ? U1 : 8) * 16 * CO1;  // conv1's (12 slots) or conv2's partials
  static constexpr int RED_FLOATS = UNITS ? (RED_UNITS > FR_BYTES ? RED_UNITS : FR_BYTES)
                                          : NW * MT1 * 16 * CO1;  // >= conv2's partials
  static_assert(4 * FR_BYTES <= RED_FLOATS * 4, "staged frames alias the reduction buffer");
  // units (gray): W1 staged transposed in LDS ([16][W1P] floats) once per block with coalesced 16-B
  // loads, so each lane's B fragment is one ds_read_b128 — per-wave 4-byte fragment loads fetched
  // every W1 element 5 times (once per M-tile sharing a K-half)
  static constexpr int W1P = KK1 + 4;
  static constexpr int W1T_FLOATS = UNITS ? CO1 * W1P : 0;
  static constexpr size_t LDS_BYTES = IN_BYTES + sizeof(float) * (RED_FLOATS + M1 * A1S + W1T_FLOATS);
  // fc kernel
  // fc tile: 16 columns x 16 envs (round 5: 32 envs; the block's 54 KB of operands at ~70 GB/s per CU
  // from L2 / MALL and its 40 dependent MFMAs per wave were the 2.3 us block — half the envs per block
  // halves both, the column block's weights are read by two adjacent blocks of one XCD)
  static constexpr int FC_BN = 16, FC_BM = 16, FC_KC = FEAT / 16;  // 18 K chunks of 16
  // K-splits of the dense layer = the slabs the heads kernel sums: 8 (20-21 chunks of 16 each), so
  // E = 32 takes 16 x 8 x 2 = 256 blocks — one per CU — where 9 (one per conv2 row) put two of its
  // 288 blocks on 32 CUs (block 1.7 us, 2.5 us on those)
  static constexpr int FC_SPLITS = 8;
};

// Stage input rows 8i..8i+19 of env e into xin. STACK: build them from the previous state and
// the new frames, writing the block's own rows of the new state.
template <int C, bool STACK>
__device__ __forceinline__ void nips_stage_rows(const uint8_t *__restrict__ obs, const StackSrc &st, int e, int i,
                                                uint8_t *xin, uint8_t *fr) {
  using Fz = FusedNips<C>;
  const size_t row0 = ((size_t)e * 84 + 8 * i) * 84 * C;  // byte offset of row 8i of env e
  if constexpr (!STACK) {
    const uint4 *src = reinterpret_cast<const uint4 *>(obs + row0);
    uint4 *dst = reinterpret_cast<uint4 *>(xin);
    for (int q = threadIdx.x; q < Fz::IN_BYTES / 16; q += Fz::NT) dst[q] = src[q];
    return;
  } else {
    __shared__ int s_p;
    // (graph replay: the tag's base is requested first; its latency hides under the row copy)
    const uint32_t tag = st.tag_base ? ((*st.tag_base + st.tag) & 0x1fffffffu) : st.tag;
    {  // the previous state's rows
      const uint4 *src = reinterpret_cast<const uint4 *>(st.prev + row0);
      uint4 *dst = reinterpret_cast<uint4 *>(xin);
      for (int q = threadIdx.x; q < Fz::IN_BYTES / 16; q += Fz::NT) dst[q] = src[q];
    }
    int p;
    if (st.ready) {
      // in-kernel pull: wait for env e's publication, then read its p pushes' rows 8i..8i+19
      // from the pinned staging (slots 4e + j) in one round trip; the edge lines of env e's slot
      // group are read with system-scope loads (ld_published16)
      if (threadIdx.x == 0) s_p = wait_published(st.ready, e, tag, st.status);
      MT_PROBE_AT(0, blockIdx.x, 5);  // env e seen published
      __syncthreads();
      p = min(max(s_p, 0), 4);  // (a timeout stacks no frame; the host reports the error)
      const size_t F = (size_t)84 * 84 * Fz::D, lo = 4 * e * F, hi = lo + 4 * F;
      for (int q = threadIdx.x; q < p * (Fz::FR_BYTES / 16); q += Fz::NT) {
        const int j = q / (Fz::FR_BYTES / 16), qq = q - j * (Fz::FR_BYTES / 16);
        const size_t off = (((size_t)4 * e + j) * 84 + 8 * i) * 84 * Fz::D + 16 * (size_t)qq;
        reinterpret_cast<uint4 *>(fr + j * Fz::FR_BYTES)[qq] = ld_published16(st.frames, off, lo, hi);
      }
      __syncthreads();
    } else {
      // one round trip for the common case: the push count and push 0's rows with the prev rows
      // (count == NULL: no pushes, the new state is a copy of prev — slot 0 <- slot T of the
      // previous rollout, mt_rollout_step)
      if (threadIdx.x == 0) s_p = st.count ? st.count[e] : 0;
      if (st.count) {
        const size_t f0 = ((size_t)4 * e * 84 + 8 * i) * 84 * Fz::D;  // push 0 = slot 4e
        const uint4 *fs = reinterpret_cast<const uint4 *>(st.frames + f0);
        for (int q = threadIdx.x; q < Fz::FR_BYTES / 16; q += Fz::NT) reinterpret_cast<uint4 *>(fr)[q] = fs[q];
      }
      __syncthreads();
      p = st.count ? min(max(s_p, 1), 4) : 0;
      if (p > 1) {  // FiGAR repeats: pushes 1..p-1 (slots 4e+1..)
        for (int q = threadIdx.x; q < (p - 1) * (Fz::FR_BYTES / 16); q += Fz::NT) {
          const int j = 1 + q / (Fz::FR_BYTES / 16), qq = q - (j - 1) * (Fz::FR_BYTES / 16);
          const size_t fj = (((size_t)4 * e + j) * 84 + 8 * i) * 84 * Fz::D;
          reinterpret_cast<uint4 *>(fr + j * Fz::FR_BYTES)[qq] = reinterpret_cast<const uint4 *>(st.frames + fj)[qq];
        }
        __syncthreads();
      }
    }
    // word w of the rows = channels 4c..4c+3 of pixel (r, x), c < D: byte offset 4w in the state
    // rows and byte w in each frame's rows (C = 4D). Same op as preprocess_kernel<D, kSrcFinal>.
    uint32_t *xw = reinterpret_cast<uint32_t *>(xin);
    uint32_t *ow = reinterpret_cast<uint32_t *>(st.out + row0);
    // the block's own words (rows 8i .. 8i+7; the last block 64..83)
    const int own = (i == Fz::ROWS2 - 1 ? Fz::RIN : 8) * 84 * Fz::D;
    for (int w = threadIdx.x; w < Fz::RIN * 84 * Fz::D; w += Fz::NT) {
      uint32_t v = p < 4 ? xw[w] >> (8 * p) : 0u;
      for (int j = 0; j < p; ++j) v |= (uint32_t)fr[j * Fz::FR_BYTES + w] << (8 * (4 - p + j));
      xw[w] = v;
      if (w < own) ow[w] = v;
    }
  }
}

// One conv1 unit of the gray kernel: M-tile t (16 of the block's 80 conv1 pixels) over the NCH K
// chunks c0 .. c0 + NCH - 1 (chunk c = (ky, kx) pairs 4c .. 4c + 3, the 4 channels of each), every
// LDS operand read first (NCH words + NCH weight fragments in flight), then the converts and the
// MFMAs on two accumulators (even / odd chunks: independent chains), added at the end.
template <int C, int NCH>
__device__ __forceinline__ f32x4 nips_conv1_unit(const uint8_t *xin, const float *w1t, int t, int c0, int r, int g) {
  using Fz = FusedNips<C>;
  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const float sc = 1.0f / 255.0f;
  const int m = min(t * 16 + r, Fz::M1 - 1);
  const int orow = m / Fz::OW1, ox = m - orow * Fz::OW1;
  const uint8_t *xb = xin + ((4 * orow) * 84 + 4 * ox) * C;
  uint32_t au[NCH];
  f32x4 bw[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int kpos = 4 * (c0 + j) + g;  // (ky, kx) of k0 = 16 c + 4 g (C = 4: the 4 channels)
    au[j] = *reinterpret_cast<const uint32_t *>(xb + ((kpos >> 3) * 84 + (kpos & 7)) * C);
    bw[j] = *reinterpret_cast<const f32x4 *>(w1t + r * Fz::W1P + 16 * (c0 + j) + 4 * g);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them to save VGPRs)
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const uint32_t u = au[j];
    const f32x4 a = f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc, (float)((u >> 16) & 0xff) * sc,
                          (float)(u >> 24) * sc};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (j & 1)
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bw[j][s], acc1, 0, 0, 0);
      else
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bw[j][s], acc0, 0, 0, 0);
    }
  }
  return acc0 + acc1;
}

// conv1 -> conv2 of conv2 row i of env e; writes act2 [B][2592] row e's 288 features of row i.
// act1 (optional): [B][20][20][16] conv1 activations (rows of a train workspace, mt_forward_rows);
// block (e, i) writes conv1 rows 2i, 2i+1 (the last block also 18, 19), so each value is written
// once.
template <int C, bool STACK>
__global__ __launch_bounds__(FusedNips<C>::NT) void nips_conv_kernel(const uint8_t *__restrict__ obs, StackSrc st, int B,
                                                        const float *__restrict__ W1, const float *__restrict__ W2,
                                                        int act, float alpha, float *__restrict__ act2,
                                                        float *__restrict__ act1) {
  using Fz = FusedNips<C>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *red = smem;                              // [4 waves][..] partial accumulators
  float *a1 = red + Fz::RED_FLOATS;               // [80 pixels][A1S] conv1 rows 2i..2i+3
  float *w1t = a1 + Fz::M1 * Fz::A1S;              // units: [16][W1P] W1 transposed
  uint8_t *xin = reinterpret_cast<uint8_t *>(w1t + Fz::W1T_FLOATS);  // [20][84][C] input rows 8i..
  uint8_t *fr = reinterpret_cast<uint8_t *>(red);  // STACK: [4][20][84][D] new frames (before conv1)

  const int nb = gridDim.x;
  const int bid = blockIdx.x;
  MT_PROBE_AT(0, bid, 0);
  const int L = (nb % 8 == 0) ? (bid % 8) * (nb / 8) + bid / 8 : bid;
  // env-major: an env's blocks share an XCD
  const int e = L / Fz::BPE, i = L - e * Fz::BPE;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;

  // conv1 weight fragments of this wave's K chunks: B[k][n] = W1[k*16 + n]. K-split: chunks
  // c = w + NW j; units: chunks 8h .. 8h+7 of the wave's K-half h = w & 1
  constexpr int NW = Fz::NW;
  constexpr int J1 = Fz::UNITS ? 1 : Fz::KC1 / NW;  // (units: fragments read from the staged w1t)
  float b1f[J1][4];
  if constexpr (Fz::UNITS) {
    // W1 [KK1][16] as float4 (4 output channels of one k), written transposed into w1t
    constexpr int NQ = Fz::KK1 * Fz::CO1 / 4;
    f32x4 wv[(NQ + Fz::NT - 1) / Fz::NT];
#pragma unroll
    for (int u = 0; u < (NQ + Fz::NT - 1) / Fz::NT; ++u)
      wv[u] = reinterpret_cast<const f32x4 *>(W1)[min((int)threadIdx.x + Fz::NT * u, NQ - 1)];
#pragma unroll
    for (int u = 0; u < (NQ + Fz::NT - 1) / Fz::NT; ++u) {
      const int q = threadIdx.x + Fz::NT * u;
      if (q < NQ) {
        const int k = q >> 2, c4 = (q & 3) * 4;
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) w1t[(c4 + e2) * Fz::W1P + k] = wv[u][e2];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < J1; ++j) {
      const int k0 = 16 * (w + NW * j) + 4 * g;
#pragma unroll
      for (int s = 0; s < 4; ++s) b1f[j][s] = W1[(size_t)(k0 + s) * Fz::CO1 + r];
    }
  }
  nips_stage_rows<C, STACK>(obs, st, e, i, xin, fr);
  __syncthreads();
  MT_PROBE_AT(0, bid, 1);

  // ---- conv1 (VALID 8x8 stride 4): M = 4 rows x 20 columns, N = 16, K = 64*C ----
  if constexpr (Fz::UNITS) {
    // wave w: M-tile w >> 1, K-half w & 1 (K chunks 8 kh .. 8 kh + 7) -> slot w; waves 0..3 also
    // M-tile 4, K-quarter w (chunks 4w .. 4w + 3) -> slot 8 + w
    const int wu = __builtin_amdgcn_readfirstlane(w);  // (wave-uniform: scalar branches)
    const f32x4 acc = nips_conv1_unit<C, 8>(xin, w1t, wu >> 1, 8 * (wu & 1), r, g);
    f32x4 acc4 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wu < 4) acc4 = nips_conv1_unit<C, 4>(xin, w1t, 4, 4 * wu, r, g);
    MT_PROBE_AT(0, bid, 6);
#pragma unroll
    for (int q = 0; q < 4; ++q) red[(w * 16 + g * 4 + q) * Fz::CO1 + r] = acc[q];
    if (wu < 4)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[((8 + w) * 16 + g * 4 + q) * Fz::CO1 + r] = acc4[q];
  } else   {
    f32x4 acc[Fz::MT1];
#pragma unroll
    for (int t = 0; t < Fz::MT1; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float sc = 1.0f / 255.0f;
#pragma unroll
    for (int j = 0; j < J1; ++j) {
      const int k0 = 16 * (w + NW * j) + 4 * g;
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
    MT_PROBE_AT(0, bid, 6);  // (wave 0) conv1 products issued
#pragma unroll
    for (int t = 0; t < Fz::MT1; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(w * Fz::MT1 * 16 + t * 16 + g * 4 + q) * Fz::CO1 + r] = acc[t][q];
  }
  // conv2 weight fragments (issued before the barrier so their latency overlaps the reduction).
  // K-split: chunks w + NW j, both N-tiles; units (w < 8): N-tile w & 1, chunks 4 (w >> 1) + j
  constexpr int J2 = Fz::UNITS ? 4 : Fz::KC2 / NW;
  constexpr int NT2 = Fz::UNITS ? 1 : 2;
  float b2f[J2][NT2][4];
#pragma unroll
  for (int j = 0; j < J2; ++j) {
    const int k0 = 16 * (Fz::UNITS ? 4 * ((w >> 1) & 3) + j : w + NW * j) + 4 * g;
#pragma unroll
    for (int nt = 0; nt < NT2; ++nt)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        b2f[j][nt][s] = W2[(size_t)(k0 + s) * Fz::CO2 + (Fz::UNITS ? (w & 1) : nt) * 16 + r];
  }
  __syncthreads();
  MT_PROBE_AT(0, bid, 7);  // every wave's conv1 partials in LDS
  {
    const float *b1 = W1 + (size_t)Fz::KK1 * Fz::CO1;
    constexpr int P = Fz::MT1 * 16 * Fz::CO1;  // stride of one wave's partials (K-split)
    for (int idx = threadIdx.x; idx < Fz::M1 * Fz::CO1; idx += Fz::NT) {
      const int m = idx / Fz::CO1, n = idx - m * Fz::CO1;
      float s;
      if constexpr (Fz::UNITS) {  // tiles 0-3: K-halves 2t + 2t+1; tile 4: K-quarters 8..11 in order
        const int t = m >> 4, rr = m & 15;
        if (t < 4)
          s = red[((2 * t) * 16 + rr) * Fz::CO1 + n] + red[((2 * t + 1) * 16 + rr) * Fz::CO1 + n];
        else
          s = ((red[(8 * 16 + rr) * Fz::CO1 + n] + red[(9 * 16 + rr) * Fz::CO1 + n]) + red[(10 * 16 + rr) * Fz::CO1 + n]) +
              red[(11 * 16 + rr) * Fz::CO1 + n];
      } else {
        s = red[idx];
#pragma unroll
        for (int v = 1; v < NW; ++v) s += red[v * P + idx];  // wave order
      }
      const float y = act_fwd(s + b1[n], act, alpha);
      a1[m * Fz::A1S + n] = y;
      // conv1 rows 2i, 2i+1 (+ 18, 19), each by one block
      const int orow = m / Fz::OW1, cx = m - orow * Fz::OW1;
      if (act1 && (orow < 2 || i == Fz::ROWS2 - 1))
        act1[(((size_t)e * Fz::OW1 + 2 * i + orow) * Fz::OW1 + cx) * Fz::CO1 + n] = y;
    }
  }
  __syncthreads();
  MT_PROBE_AT(0, bid, 2);

  // ---- conv2 row i (VALID 4x4 stride 2): M = its 9 pixels (padded to 16), N = 32, K = 256 ----
  if constexpr (Fz::UNITS) {
    if (w < 8) {  // unit w: N-tile w & 1, K-quarter kq = w >> 1 (chunks 4kq .. 4kq+3: ky = kq, kx = j)
      const int kq = w >> 1;
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      const int ox = min(r, Fz::OW2 - 1);
#pragma unroll
      for (int j = 0; j < J2; ++j) {
        const f32x4 a = *reinterpret_cast<const f32x4 *>(a1 + (kq * Fz::OW1 + 2 * ox + j) * Fz::A1S + 4 * g);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if (j & 1)
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b2f[j][0][s], acc1, 0, 0, 0);
          else
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b2f[j][0][s], acc0, 0, 0, 0);
        }
      }
      const f32x4 acc = acc0 + acc1;
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(w * 16 + g * 4 + q) * 16 + r] = acc[q];
    }
  } else   {
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int ox = min(r, Fz::OW2 - 1);
#pragma unroll
    for (int j = 0; j < J2; ++j) {
      const int c = w + NW * j;  // (ky, kx) = (c / 4, c % 4), channels 4g..4g+3
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
  MT_PROBE_AT(0, bid, 3);
  {
    const float *b2 = W2 + (size_t)Fz::KK2 * Fz::CO2;
    constexpr int P = 16 * Fz::CO2;
    for (int idx = threadIdx.x; idx < Fz::OW2 * Fz::CO2; idx += Fz::NT) {
      const int n = idx & (Fz::CO2 - 1);
      float s;
      if constexpr (Fz::UNITS) {  // K-quarters 0..3 (in order) of N-tile n / 16: units 2 kq + n / 16
        const int m = idx >> 5, nt = n >> 4, c = n & 15;
        s = red[(nt * 16 + m) * 16 + c];
#pragma unroll
        for (int kq = 1; kq < 4; ++kq) s += red[((kq * 2 + nt) * 16 + m) * 16 + c];
      } else {
        s = red[idx];
#pragma unroll
        for (int v = 1; v < NW; ++v) s += red[v * P + idx];  // wave order
      }
      act2[((size_t)e * Fz::ROWS2 + i) * Fz::FEAT + idx] = act_fwd(s + b2[n], act, alpha);
    }
  }
  MT_PROBE_AT(0, bid, 4);
}

// Dense layer partial products by trunk rows: slabs[i][e][n] = sum_{f < FEAT} x[e][FEAT i + f]
// W[FEAT i + f][n] (x = the flattened last conv output [B][ROWS * FEAT], NHWC: row i of the conv
// output = features [FEAT i, FEAT (i + 1))). Grid (F / 16, ROWS, ceil(B / 32)); 4 waves split the
// FEAT / 16 K chunks of 16 (c = w + 4j), every operand load of a wave issued before its first MFMA
// (one memory round trip, where a generic split-K GEMM block walks its K chunks one load latency
// each: NATURE's dense layer 10 us as a TileFc GEMM at E = 64); partials added in wave order
// through LDS. advance (replayed rollout graph whose bootstrap has no heads kernel,
// SampleArgs::advance): block 0 adds advance_by to advance[0] and advance[1] — every reader of
// those bases in the replay has run.
constexpr int kRowFcBN = 16, kRowFcBM = 32;
// Block pb of a (gx, gy, gz) = (F / 16, ROWS, env chunks of BM) grid.
// SPLITS: K-splits (slabs) of the FLAT = FEAT x ROWS inputs, split i = 16-wide chunks
// [TC i / SPLITS, TC (i + 1) / SPLITS) — one conv output row each when SPLITS = ROWS
template <int FEAT, int ROWS, int F, int BM = kRowFcBM, int SPLITS = ROWS>
__device__ __forceinline__ void row_fc_body(const float *__restrict__ x, int B, const float *__restrict__ Wfc,
                                            float *__restrict__ slabs, uint32_t *advance, uint32_t advance_by, int pb,
                                            int gx, int gy, int gz) {
  constexpr int FLAT = FEAT * ROWS, TC = FLAT / 16, MT = BM / 16;
  constexpr int KC = (TC + SPLITS - 1) / SPLITS;  // chunks of the longest split
  static_assert(FEAT % 16 == 0 && F % kRowFcBN == 0 && BM % 16 == 0, "whole chunks, column blocks, M-tiles");
  __shared__ __attribute__((aligned(16))) float red[4][BM][kRowFcBN];
  if (advance && pb == 0 && threadIdx.x == 0) {
    advance[0] += advance_by;
    advance[1] += advance_by;
  }
  const int nbk = gx * gy * gz;
  const int L = (nbk % 8 == 0) ? (pb % 8) * (nbk / 8) + pb / 8 : pb;  // XCD-aware (see the top)
  // tile L = (env chunk fastest, then column block, then conv row): the env chunks of one (column
  // block, row) read the same 16 x FEAT weights and sit in one XCD's run of tiles, so at E = 64 the
  // weights come from HBM once, not once per 32 envs (PMC: Breakout NATURE row_fc 15.0 MB per call)
  const int zc = L % gz, xy = L / gz;
  const int xb = xy % gx, i = xy / gx;
  const int n0 = xb * kRowFcBN, e0 = zc * BM;
  const int c0 = (TC * i) / SPLITS, c1 = (TC * (i + 1)) / SPLITS;  // the split's chunks
  MT_PROBE_AT(1, pb, 0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  constexpr int JN = (KC + 3) / 4;
  f32x4 a[JN][MT];
  float b[JN][4];
  int rowt[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) rowt[t] = min(e0 + 16 * t + r, B - 1);
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int c = min(c0 + w + 4 * j, c1 - 1);  // (chunks past the split's last are loaded but not used)
    const int k0 = 16 * c + 4 * g;
#pragma unroll
    for (int t = 0; t < MT; ++t) a[j][t] = *reinterpret_cast<const f32x4 *>(x + (size_t)rowt[t] * FLAT + k0);
#pragma unroll
    for (int s = 0; s < 4; ++s) b[j][s] = Wfc[(size_t)(k0 + s) * F + n0 + r];
  }
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    if (c0 + w + 4 * j < c1) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][t][s], b[j][s], acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[w][t * 16 + g * 4 + q][r] = acc[t][q];
  __syncthreads();
  MT_PROBE_AT(1, pb, 1);
  for (int idx = threadIdx.x; idx < BM * kRowFcBN; idx += 256) {
    const int m = idx / kRowFcBN, n = idx - m * kRowFcBN;
    const float s = ((red[0][m][n] + red[1][m][n]) + red[2][m][n]) + red[3][m][n];
    if (e0 + m < B) slabs[((size_t)i * B + e0 + m) * F + n0 + n] = s;
  }
  MT_PROBE_AT(1, pb, 2);
}

// the NIPS trunk's dense kernel (FEAT = 288 features of each of its 9 conv2 rows)
template <int C>
__global__ __launch_bounds__(256) void nips_fc_kernel(const float *__restrict__ act2, int B,
                                                      const float *__restrict__ Wfc, float *__restrict__ slabs,
                                                      uint32_t *advance, uint32_t advance_by) {
  using Fz = FusedNips<C>;
  static_assert(Fz::FC_BN == kRowFcBN, "tile");
  row_fc_body<Fz::FEAT, Fz::ROWS2, Fz::F, Fz::FC_BM, Fz::FC_SPLITS>(act2, B, Wfc, slabs, advance, advance_by,
                                         (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, gridDim.x,
                                         gridDim.y, gridDim.z);
}

// the same for the layered trunks (NATURE: 7 rows of 448 features, PWYX: 10 rows of 640), in tiles
// of BM env rows: 16 up to 32 envs (the 16-env tiles of the NIPS dense kernel: Seaquest E = 32 5.24
// -> 4.95 us, PWYX-RGB 8.86 -> 8.04 us per launch), 32 beyond (Breakout E = 64: 6.95 vs 7.28 us with
// 16: its column block's weights would be read by four blocks instead of two; profiles/r06rf)
template <int FEAT, int ROWS, int F, int BM, int SPLITS = ROWS>
__global__ __launch_bounds__(256) void row_fc_kernel(const float *__restrict__ x, int B, const float *__restrict__ Wfc,
                                                     float *__restrict__ slabs, uint32_t *advance, uint32_t advance_by) {
  row_fc_body<FEAT, ROWS, F, BM, SPLITS>(x, B, Wfc, slabs, advance, advance_by,
                                 (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, gridDim.x, gridDim.y,
                                 gridDim.z);
}
template <int FEAT, int ROWS, int F, int SPLITS = ROWS>
static inline int launch_row_fc(const float *x, int B, const float *Wfc, float *slabs, hipStream_t s,
                                uint32_t *advance = nullptr, uint32_t advance_by = 0) {
  if (B <= 0 || !launch_allowed()) return MT_OK;
  if (B <= 32)
    hipLaunchKernelGGL((row_fc_kernel<FEAT, ROWS, F, 16, SPLITS>), dim3(F / kRowFcBN, SPLITS, (B + 15) / 16), dim3(256),
                       0, s, x, B, Wfc, slabs, advance, advance_by);
  else
    hipLaunchKernelGGL((row_fc_kernel<FEAT, ROWS, F, kRowFcBM, SPLITS>),
                       dim3(F / kRowFcBN, SPLITS, (B + kRowFcBM - 1) / kRowFcBM), dim3(256), 0, s, x, B, Wfc, slabs,
                       advance, advance_by);
  MT_LAUNCHED();
  return MT_OK;
}

// Throughput form of the NIPS conv trunk for large batches (gray frames, E >= kPersistMinEnvs):
// the latency form above recomputes 1.8x of conv1 so that 9 blocks can work on one env; once the
// grid fills the chip that recompute is pure cost. Here a persistent block (16 waves, one block
// per CU) stages W1 / W2 transposed in LDS once and walks envs e = blockIdx.x, += gridDim.x: the
// env's 84x84x4 frame in LDS; conv1 as 25 M-tiles of 16 pixels — tiles 0..23 two or one per wave
// (6 per SIMD: waves w, w+4, w+8, w+12 share one), tile 24 split into 4 K-quarters on waves 8..11
// (one per SIMD, 4 partials added in order) so every SIMD issues 400 MFMAs per env; A fragment =
// one u32 of 4 channels, B fragment = one ds_read_b128 of the transposed weights; bias + act into
// an LDS act1 [400][16]; then conv2 as 6 M-tiles x 2 N-tiles on waves 0..11 (3 per SIMD), act2 to
// HBM in the same NHWC flatten order. The next env's frame is loaded into registers during conv2.
// Same fp32 products (k-ordered MFMA chains) as the latency form, up to the summation split.
constexpr int kPersistMinEnvs = 256;
struct PersistNips {
  static constexpr int NT = 1024;                        // 16 waves
  static constexpr int XIN = 84 * 84 * 4;                // 28,224 B
  static constexpr int A1P = 20, A1 = 400 * A1P;         // act1 [400][20] floats
  static constexpr int WP = 260;                         // transposed weight row (floats)
  static constexpr int T24 = 4 * 256;                    // tile 24's 4 K-quarter partials
  static constexpr size_t LDS = XIN + sizeof(float) * (A1 + 16 * WP + 32 * WP + T24);
  static constexpr int NQ = (XIN / 16 + NT - 1) / NT;    // 16-B chunks of a frame per thread
};

// (one 16-wave block per CU by its LDS: 4 waves per SIMD, up to 128 VGPRs each)
__global__ __launch_bounds__(PersistNips::NT) void nips_conv_persist_kernel(
    const uint8_t *__restrict__ obs, int B, const float *__restrict__ W1, const float *__restrict__ W2, int act,
    float alpha, float *__restrict__ act2, float *__restrict__ act1_out) {
  using Pz = PersistNips;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint8_t *xin = reinterpret_cast<uint8_t *>(smem);
  float *a1 = reinterpret_cast<float *>(xin + Pz::XIN);
  float *w1t = a1 + Pz::A1;
  float *w2t = w1t + 16 * Pz::WP;
  float *p24 = w2t + 32 * Pz::WP;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < 256 * 16; i += Pz::NT) w1t[(i & 15) * Pz::WP + (i >> 4)] = W1[i];
  for (int i = threadIdx.x; i < 256 * 32; i += Pz::NT) w2t[(i & 31) * Pz::WP + (i >> 5)] = W2[i];
  const float *b1 = W1 + 256 * 16, *b2 = W2 + 256 * 32;
  const float bias1 = b1[r], bias2a = b2[r], bias2b = b2[16 + r];
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 nx[Pz::NQ];
  {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(obs + (size_t)min((int)blockIdx.x, B - 1) * Pz::XIN);
#pragma unroll
    for (int u = 0; u < Pz::NQ; ++u) nx[u] = src[min((int)threadIdx.x + Pz::NT * u, Pz::XIN / 16 - 1)];
  }
  const float sc = 1.0f / 255.0f;
  // conv1 work of wave w: tiles w and (w < 8) w + 16; waves 8..11 also K-quarter w - 8 of tile 24
  const bool two = w < 8, quarter = w >= 8 && w < 12;
  int base[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int m = min(16 * (w + 16 * t) + r, 399), oy = m / 20, ox = m - oy * 20;
    base[t] = (4 * oy * 84 + 4 * ox) * 4;
  }
  int base24;
  {
    const int m = 16 * 24 + r, oy = m / 20, ox = m - oy * 20;
    base24 = (4 * oy * 84 + 4 * ox) * 4;
  }
  for (int e = blockIdx.x; e < B; e += gridDim.x) {
#pragma unroll
    for (int u = 0; u < Pz::NQ; ++u) {
      const int q = threadIdx.x + Pz::NT * u;
      if (q < Pz::XIN / 16) reinterpret_cast<u32x4 *>(xin)[q] = nx[u];
    }
    __syncthreads();
    // ---- conv1 ----
    {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      f32x4 acc24 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int kc = 0; kc < 16; ++kc) {
        const int kpos = 4 * kc + g, off = ((kpos >> 3) * 84 + (kpos & 7)) * 4;
        const f32x4 bv = *reinterpret_cast<const f32x4 *>(w1t + r * Pz::WP + 16 * kc + 4 * g);
        f32x4 av[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint32_t u = *reinterpret_cast<const uint32_t *>(xin + base[t] + off);
          av[t] = f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc, (float)((u >> 16) & 0xff) * sc,
                        (float)(u >> 24) * sc};
        }
        // s outer, tiles inner: consecutive MFMAs on independent accumulators
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0][s], bv[s], acc[0], 0, 0, 0);
          if (two) acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1][s], bv[s], acc[1], 0, 0, 0);
        }
        if (quarter && (kc >> 2) == w - 8) {  // (wave-uniform)
          const uint32_t u = *reinterpret_cast<const uint32_t *>(xin + base24 + off);
          const f32x4 a24 = f32x4{(float)(u & 0xff) * sc, (float)((u >> 8) & 0xff) * sc,
                                  (float)((u >> 16) & 0xff) * sc, (float)(u >> 24) * sc};
#pragma unroll
          for (int s = 0; s < 4; ++s) acc24 = __builtin_amdgcn_mfma_f32_16x16x4f32(a24[s], bv[s], acc24, 0, 0, 0);
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (t == 0 || two)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = 16 * (w + 16 * t) + 4 * g + q;
            const float y = act_fwd(acc[t][q] + bias1, act, alpha);
            a1[m * Pz::A1P + r] = y;
            if (act1_out) act1_out[((size_t)e * 400 + m) * 16 + r] = y;
          }
      if (quarter)
#pragma unroll
        for (int q = 0; q < 4; ++q) p24[(w - 8) * 256 + (4 * g + q) * 16 + r] = acc24[q];
    }
    __syncthreads();
    if (threadIdx.x < 256) {  // tile 24: its 4 K-quarters in order, bias + act
      const int row = threadIdx.x >> 4, c = threadIdx.x & 15, m = 384 + row;
      const float s = ((p24[row * 16 + c] + p24[256 + row * 16 + c]) + p24[512 + row * 16 + c]) + p24[768 + row * 16 + c];
      const float y = act_fwd(s + b1[c], act, alpha);
      a1[m * Pz::A1P + c] = y;
      if (act1_out) act1_out[((size_t)e * 400 + m) * 16 + c] = y;
    }
    __syncthreads();
    {  // the next env's frame: loaded now, stored after this env's conv2 (xin is free)
      const u32x4 *src = reinterpret_cast<const u32x4 *>(obs + (size_t)min(e + (int)gridDim.x, B - 1) * Pz::XIN);
#pragma unroll
      for (int u = 0; u < Pz::NQ; ++u) nx[u] = src[min((int)threadIdx.x + Pz::NT * u, Pz::XIN / 16 - 1)];
    }
    // ---- conv2: waves 0..11, unit w: m-tile w / 2, n-tile w % 2 ----
    if (w < 12) {
      const int mt = w >> 1, ntile = w & 1;
      const int mr = min(16 * mt + r, 80), oy = mr / 9, ox = mr - oy * 9;
      const float *abase = a1 + (2 * oy * 20 + 2 * ox) * Pz::A1P + 4 * g;
      const float *bbase = w2t + (16 * ntile + r) * Pz::WP + 4 * g;
      // two accumulators (even / odd K chunks, added at the end): no dependent MFMA back to back
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int kc = 0; kc < 16; kc += 2) {
        const f32x4 av0 = *reinterpret_cast<const f32x4 *>(abase + ((kc >> 2) * 20 + (kc & 3)) * Pz::A1P);
        const f32x4 bv0 = *reinterpret_cast<const f32x4 *>(bbase + 16 * kc);
        const f32x4 av1 = *reinterpret_cast<const f32x4 *>(abase + (((kc + 1) >> 2) * 20 + ((kc + 1) & 3)) * Pz::A1P);
        const f32x4 bv1 = *reinterpret_cast<const f32x4 *>(bbase + 16 * (kc + 1));
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0[s], bv0[s], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av1[s], bv1[s], acc1, 0, 0, 0);
        }
      }
      const f32x4 acc = acc0 + acc1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = 16 * mt + 4 * g + q;
        if (m < 81)
          act2[(size_t)e * 2592 + m * 32 + 16 * ntile + r] = act_fwd(acc[q] + (ntile ? bias2b : bias2a), act, alpha);
      }
    }
    __syncthreads();
  }
}

// Launch the two trunk kernels: conv (optionally stacking) -> act2, fc -> slabs.
template <int C>
static inline int launch_nips_trunk(const uint8_t *obs, const StackSrc *st, int B, const float *W1, const float *W2,
                                    const float *Wfc, int act, float alpha, float *act2, float *act1, float *slabs,
                                    hipStream_t s, uint32_t *advance = nullptr, uint32_t advance_by = 0) {
  using Fz = FusedNips<C>;
  static_assert(Fz::LDS_BYTES <= 64 * 1024, "conv kernel LDS fits the default limit");
  if (st) {
    hipLaunchKernelGGL((nips_conv_kernel<C, true>), dim3(Fz::BPE * B), dim3(Fz::NT), Fz::LDS_BYTES, s, st->out, *st,
                       B, W1, W2, act, alpha, act2, act1);
  } else if (C == 4 && B >= kPersistMinEnvs) {
    if (advance) {
      set_error("sequence-base advance: stacking trunk launches only");
      return MT_ERR_ARG;
    }
    static int cus = 0;
    static bool attr = false;
    if (!cus) {
      int dev = 0;
      MT_HIP(hipGetDevice(&dev));
      MT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (!attr) {
      MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&nips_conv_persist_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)PersistNips::LDS));
      attr = true;
    }
    hipLaunchKernelGGL(nips_conv_persist_kernel, dim3(std::min(B, cus)), dim3(PersistNips::NT), PersistNips::LDS, s,
                       obs, B, W1, W2, act, alpha, act2, act1);
    MT_LAUNCHED();
    // the dense layer as a 64 x 64-tile GEMM in FC_SPLITS K-splits (the slab count the heads kernel
    // sums: 8 of 352 / 128 with 32-deep chunks): nips_fc_kernel's 16-column blocks would re-read act2
    // 16 times at this batch
    using TP = Tile<64, 64, 2, 2, 32>;
    static_assert(Fz::FLAT % TP::BK == 0, "whole chunks");
    if (gemm_splits<TP>(Fz::FLAT, Fz::FC_SPLITS) != Fz::FC_SPLITS) {
      set_error("persistent NIPS trunk: %d dense K-splits, the heads sum %d", gemm_splits<TP>(Fz::FLAT, Fz::FC_SPLITS),
                Fz::FC_SPLITS);
      return MT_ERR_ARG;
    }
    return launch_gemm<TP>(LdRowMajor{act2, Fz::FLAT}, LdColMajor{Wfc, Fz::F, -1}, EpSlab{slabs, B, Fz::F}, B, Fz::F,
                           Fz::FLAT, Fz::FC_SPLITS, s);
  } else {
    hipLaunchKernelGGL((nips_conv_kernel<C, false>), dim3(Fz::BPE * B), dim3(Fz::NT), Fz::LDS_BYTES, s, obs,
                       StackSrc{}, B, W1, W2, act, alpha, act2, act1);
  }
  hipLaunchKernelGGL(nips_fc_kernel<C>, dim3(Fz::F / Fz::FC_BN, Fz::FC_SPLITS, (B + Fz::FC_BM - 1) / Fz::FC_BM),
                     dim3(256), 0, s, act2, B, Wfc, slabs, advance, advance_by);
  return MT_OK;
}

}  // namespace mt
