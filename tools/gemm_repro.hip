// Standalone reproducer for the GEMM core's conv weight-gradient product: the RGB
// NIPS conv1 dW of tests/test_kernels_gpu.py::test_loss_backward_parity[5-NIPS-3-4-11] —
// A = the transposed im2col of uint8 frames [5][84][84][12] (LdIm2colT), B = dY [2000][16]
// (column-major loader), M = 768 weight rows, N = 16 channels, K = 2000 pixels in 8 splits of 256
// (the last split 208 = 3 full BK chunks + one 16-deep partial chunk) — run with two B loaders:
//   old: the round-2 guarded fetch (a k < ke branch around the f32x4 load, zeros merged into the
//        register quad when it is not taken)
//   new: gemm.h's LdColMajor (clamped k, one load, zero by select)
// and compared per output channel against a double-precision host product. Build once per
// accumulator mode and run both:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMT_GEMM_DUAL=1 tools/gemm_repro.hip -o /tmp/repro1
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMT_GEMM_DUAL=0 tools/gemm_repro.hip -o /tmp/repro0
// Prints the max relative error of every (loader, channel) and exits 1 if any exceeds 1e-5.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../manette_amd/csrc/gemm.h"

namespace mt {
void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}
}  // namespace mt

using namespace mt;

// The round-2 form of LdColMajor::fetch (the rest of the loader is gemm.h's).
struct LdColMajorOld : LdColMajor {
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int row = row0 + rr, k = k0 + kk;
    const int nx = ones_row >= 0 ? ones_row : nrows;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (k < ke) {
      const float *p = X + (size_t)k * ld + row;
      if (row + 3 < nx && (ld & 3) == 0) {
        v = *reinterpret_cast<const f32x4 *>(p);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rw = row + e;
          if (rw < nx) v[e] = p[e];
          else if (rw == ones_row) v[e] = 1.f;
        }
      }
    }
    return v;
  }
};

using G = ConvGeom<12, 16, 8, 4, 84, 84, false>;
using T = Tile<64, 16, 4, 1, 64>;
constexpr int B = 5, M = G::KK, N = G::COUT, K = B * G::OH * G::OW, SPLITS = 8;

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
      exit(2);                                                            \
    }                                                                     \
  } while (0)

template <class LB>
static std::vector<float> run(const uint8_t *dX, const float *dY, float *dP) {
  CK(hipMemset(dP, 0, sizeof(float) * SPLITS * M * N));
  LdIm2colT<G, true> la{dX};
  LB lb;
  lb.X = dY;
  lb.ld = N;
  lb.ones_row = -1;
  if (launch_gemm<T>(la, lb, EpSlab{dP, M, N}, M, N, K, SPLITS, nullptr) != MT_OK) exit(3);
  CK(hipDeviceSynchronize());
  std::vector<float> P((size_t)SPLITS * M * N);
  CK(hipMemcpy(P.data(), dP, sizeof(float) * P.size(), hipMemcpyDeviceToHost));
  return P;
}

int main() {
  static_assert(K == 2000, "the failing test's shape");
  std::vector<uint8_t> X((size_t)B * G::H * G::W * G::CIN);
  std::vector<float> dY((size_t)K * N);
  uint64_t s = 12345;
  auto rnd = [&] {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return (uint32_t)(s >> 33);
  };
  for (auto &x : X) x = (uint8_t)rnd();
  for (auto &y : dY) y = ((int)(rnd() % 2001) - 1000) * 1e-3f;
  // reference: slab z, row kr = (ky, kx, ci), channel n = sum over pixels m of split z
  const int kchunk = cdiv(cdiv(K, T::BK), SPLITS) * T::BK;
  std::vector<double> ref((size_t)SPLITS * M * N, 0.0);
  for (int m = 0; m < K; ++m) {
    const int z = m / kchunk, b = m / (G::OH * G::OW), rem = m % (G::OH * G::OW);
    const int oy = rem / G::OW, ox = rem % G::OW;
    for (int kr = 0; kr < M; ++kr) {
      const int ky = kr / (G::KW * G::CIN), kx = (kr / G::CIN) % G::KW, ci = kr % G::CIN;
      const double a = X[(((size_t)b * G::H + oy * G::S + ky) * G::W + ox * G::S + kx) * G::CIN + ci] / 255.0;
      for (int n = 0; n < N; ++n) ref[((size_t)z * M + kr) * N + n] += a * dY[(size_t)m * N + n];
    }
  }
  uint8_t *dX;
  float *ddY, *dP;
  CK(hipMalloc(&dX, X.size()));
  CK(hipMalloc(&ddY, sizeof(float) * dY.size()));
  CK(hipMalloc(&dP, sizeof(float) * SPLITS * M * N));
  CK(hipMemcpy(dX, X.data(), X.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(ddY, dY.data(), sizeof(float) * dY.size(), hipMemcpyHostToDevice));
  int bad = 0;
  const char *names[2] = {"old", "new"};
  for (int v = 0; v < 2; ++v) {
    const std::vector<float> P = v == 0 ? run<LdColMajorOld>(dX, ddY, dP) : run<LdColMajor>(dX, ddY, dP);
    printf("MT_GEMM_DUAL=%d loader=%s:", MT_GEMM_DUAL, names[v]);
    for (int n = 0; n < N; ++n) {
      double num = 0, den = 0, last = 0;  // whole channel; and the last split alone
      for (int z = 0; z < SPLITS; ++z)
        for (int kr = 0; kr < M; ++kr) {
          const size_t i = ((size_t)z * M + kr) * N + n;
          const double d = P[i] - ref[i];
          num += d * d;
          den += ref[i] * ref[i];
          if (z == SPLITS - 1) last = std::fmax(last, std::fabs(d));
        }
      const double rel = std::sqrt(num / den);
      printf(" c%d=%.1e", n, rel);
      if (rel > 1e-5) {
        ++bad;
        printf("(!last-split max abs %.2e)", last);
      }
    }
    printf("\n");
  }
  printf("%s\n", bad ? "MISMATCH" : "all channels within 1e-5");
  return bad ? 1 : 0;
}
