// Weight gradient of the 8x8 stride-4 VALID input conv of the NIPS / NATURE trunks
// (networks.py:178-192, :261-278: conv1 84x84xC -> 20x20xCOUT), as a grouped-launch job.
//
//   dW[ky][kx][ci][co] = (1/255) * sum_{b, oy, ox} u8 X[b][4oy+ky][4ox+kx][ci] * dY[b][oy][ox][co]
//
// The generic product (LdIm2colT) spends ~11 VALU instructions per MFMA gathering single im2col
// bytes. Here the stride-4 taps are split into phases: ky = 4a + py, kx = 4c + px, so
// X[4oy+ky][4ox+kx] = Xp[py][px][oy+a][ox+c] with Xp the 21x21 phase planes; staged in LDS
// phase-major ([py][px][ci][qy][qx], u8), the 4 consecutive output pixels of one MFMA lane's
// fragment are 4 consecutive bytes — one (or, for c = 1, two aligned + v_alignbyte) ds_read_b32
// and four byte converts per 4 MFMAs. dY is staged transposed ([co][pixel]) so its fragment is one
// ds_read_b128. The 1/255 input scale is applied once to the accumulator (networks.py:155; the
// reference scales each input, the sum is the same up to rounding).
//
// Block = (image b, tap quarter q): quarter q holds the rows ky in {2q, 2q+1} (16*C of the 64*C
// weight rows), i.e. phases py in {2q%4, 2q%4+1} with a = q/2; its 4 waves split those C M-tiles.
// Each block writes its rows of image b's partial gradient into slab b (rows (ky,kx,ci) of
// [KK+1][COUT]); quarter 0 also writes the bias row (sum of dY over the image). The slab sum over
// the B images finishes the gradient (fixed order: deterministic).
#pragma once
#include "gemm.h"

namespace mt {

template <class G>
constexpr bool is_conv1_s4() {
  return G::KH == 8 && G::KW == 8 && G::S == 4 && G::H == 84 && G::W == 84 && !G::SAME && G::OH == 20 &&
         G::OW == 20 && G::COUT % 16 == 0 && G::CIN % 4 == 0;
}

template <int C, int COUT>
struct Conv1S4WgradJob {
  static constexpr int NT = COUT / 16;     // N tiles
  static constexpr int TPW = C / 4;        // M tiles per wave (a quarter = 16C rows = C tiles)
  static constexpr int QXP = 24;           // bytes per staged phase row (21 used)
  // one (py, px, ci) plane: qy = oy in [0, 20); +4 bytes so the 16 planes a fragment's lanes
  // read start on distinct LDS banks (a plane of 120 dwords put lanes r, r+4, ... on one bank)
  static constexpr int PLANE = 20 * QXP + 4;
  static constexpr int XS_BYTES = 2 * 4 * C * PLANE;
  static constexpr int PIXP = 404;         // padded pixel stride of dY^T (floats)
  static constexpr int KK = 64 * C;
  static constexpr int XS_ALLOC = (XS_BYTES + 15) / 16 * 16;
  static_assert(XS_ALLOC % 16 == 0, "dY^T stays 16-byte aligned");
  const uint8_t *X = nullptr;  // [B][84][84][C]
  const float *dY = nullptr;   // [B][20][20][COUT]
  float *slab = nullptr;       // [B][KK + 1][COUT]
  int B = 0;
  __host__ __device__ int blocks() const { return 4 * B; }
  size_t lds() const { return XS_ALLOC + sizeof(float) * COUT * PIXP; }
  __device__ __forceinline__ void run(int id, float *smem) const {
    const int b = id >> 2, q = id & 3, a = q >> 1, py0 = (2 * q) & 3;
    uint8_t *xs = reinterpret_cast<uint8_t *>(smem);
    float *dyt = reinterpret_cast<float *>(xs + XS_ALLOC);
    // ---- stage: input rows y = 4(qy + a) + py0 + pyl (qy < 20, pyl < 2), phase-major bytes, and
    //      dY^T. Every global load of the thread is issued before the first LDS write (a load /
    //      write loop would wait out one load latency per iteration). ----
    {
      constexpr int QPR = 84 * C / 16;                 // 16-byte chunks per input row
      constexpr int NX = (40 * QPR + 255) / 256;       // chunks per thread
      constexpr int ND = (400 * COUT / 4 + 255) / 256;  // dY float4 per thread
      const uint8_t *img = X + (size_t)b * 84 * 84 * C;
      const f32x4 *src = reinterpret_cast<const f32x4 *>(dY + (size_t)b * 400 * COUT);
      uint4 xv[NX];
      f32x4 dv[ND];
#pragma unroll
      for (int u = 0; u < NX; ++u) {
        const int w = min((int)threadIdx.x + 256 * u, 40 * QPR - 1);
        const int rr = w / QPR, k = w - rr * QPR;
        const int y = 4 * ((rr >> 1) + a) + py0 + (rr & 1);
        xv[u] = *reinterpret_cast<const uint4 *>(img + (size_t)y * 84 * C + 16 * k);
      }
#pragma unroll
      for (int u = 0; u < ND; ++u) dv[u] = src[min((int)threadIdx.x + 256 * u, 400 * COUT / 4 - 1)];
#pragma unroll
      for (int u = 0; u < NX; ++u) {
        const int w = threadIdx.x + 256 * u;
        if (w < 40 * QPR) {
          const int rr = w / QPR, k = w - rr * QPR;
          const int qy = rr >> 1, pyl = rr & 1;
          const uint32_t words[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
          for (int jb = 0; jb < 16; ++jb) {
            const int j = 16 * k + jb, x = j / C, ci = j - x * C;
            xs[((pyl * 4 + (x & 3)) * C + ci) * PLANE + qy * QXP + (x >> 2)] = (uint8_t)(words[jb >> 2] >> (8 * (jb & 3)));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < ND; ++u) {
        const int i = threadIdx.x + 256 * u;
        if (i < 400 * COUT / 4) {
          const int pix = i / (COUT / 4), c4 = (i - pix * (COUT / 4)) * 4;
#pragma unroll
          for (int e = 0; e < 4; ++e) dyt[(c4 + e) * PIXP + pix] = dv[u][e];
        }
      }
    }
    __syncthreads();
    // ---- products: wave w owns local tiles w*TPW .. ; lane (r, g) ----
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    int abase[TPW], ashift[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int lr = (w * TPW + t) * 16 + r;  // local weight row: (kyl, kx, ci)
      const int kyl = lr / (8 * C), rem = lr - kyl * (8 * C), kx = rem / C, ci = rem - kx * C;
      abase[t] = ((kyl * 4 + (kx & 3)) * C + ci) * PLANE;
      ashift[t] = kx >> 2;  // c: byte offset of the pixel run
    }
    f32x4 acc[TPW][NT];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
    for (int kc = 0; kc < 25; ++kc) {
      const int G4 = 4 * kc + g, oy = G4 / 5, oxg = G4 - 5 * oy;  // pixels (oy, 4oxg .. 4oxg+3)
      f32x4 bv[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        bv[nt] = *reinterpret_cast<const f32x4 *>(dyt + (nt * 16 + r) * PIXP + oy * 20 + 4 * oxg);
      const int off = oy * QXP + 4 * oxg;
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const uint32_t lo = *reinterpret_cast<const uint32_t *>(xs + abase[t] + off);
        const uint32_t hi = *reinterpret_cast<const uint32_t *>(xs + abase[t] + off + 4);
        const uint32_t u = __builtin_amdgcn_alignbyte(hi, lo, ashift[t]);
        const f32x4 av = f32x4{(float)(u & 0xff), (float)((u >> 8) & 0xff), (float)((u >> 16) & 0xff),
                               (float)(u >> 24)};
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[nt][s], acc[t][nt], 0, 0, 0);
      }
    }
    // ---- epilogue: rows (ky, kx, ci) of slab b, scaled by 1/255 ----
    float *out = slab + (size_t)b * (KK + 1) * COUT;
    const float sc = 1.0f / 255.0f;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int lr = (w * TPW + t) * 16 + 4 * g + qq;
        const int k = 2 * q * 8 * C + lr;  // rows of quarter q are contiguous: ky = 2q + lr / (8C)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) out[(size_t)k * COUT + nt * 16 + r] = acc[t][nt][qq] * sc;
      }
    if (q == 0) {  // bias row: sum of dY over the image's 400 pixels, 16 subsets per channel
      float *part = reinterpret_cast<float *>(smem);  // (xs is no longer read after the barrier)
      __syncthreads();
      for (int n0 = 0; n0 < COUT; n0 += 16) {
        const int co = n0 + (threadIdx.x & 15), sub = threadIdx.x >> 4;
        float s = 0.f;
        for (int p = sub; p < 400; p += 16) s += dyt[co * PIXP + p];
        part[threadIdx.x] = s;
        __syncthreads();
        if (threadIdx.x < 16) {
          float t = part[threadIdx.x];
#pragma unroll
          for (int u = 1; u < 16; ++u) t += part[u * 16 + threadIdx.x];
          out[(size_t)KK * COUT + n0 + threadIdx.x] = t;
        }
        __syncthreads();
      }
    }
  }
};

}  // namespace mt
