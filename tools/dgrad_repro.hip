// Standalone reproducer for the NIPS conv2 backward-data product (the dual-accumulator
// finding): dact1 = (dY2 * W2^T gathered over the stride phases) * relu'(act1) with the GEMM core's
// phase loaders (LdConvBwdAPhase / LdConvBwdBPhase / EpMaskedPhase, net.hip conv_dgrad_job), B = 5,
// launched alone (variant 0) and as the product's grouped launch beside conv2's weight-gradient
// product and bias rows (variant 1), compared per output channel against a double-precision host
// product. Inputs: seeded random, or (argv[1] = a prefix written by tools/dual_diag.py) the
// product's own dY2, W2 and act1. Build once per accumulator mode:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMT_GEMM_DUAL=1 tools/dgrad_repro.hip -o tools/bin/dgrad_repro1
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMT_GEMM_DUAL=0 tools/dgrad_repro.hip -o tools/bin/dgrad_repro0
// Prints every channel whose relative L2 error exceeds 1e-5 and exits 1 if any does.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../manette_amd/csrc/gemm.h"
#include "../manette_amd/csrc/jobs.h"

namespace mt {
bool g_win_on = false;
int g_win_first = 0, g_win_count = -1, g_win_index = 0;
void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}
}  // namespace mt

using namespace mt;

using G = ConvGeom<16, 32, 4, 2, 20, 20, false>;  // NIPS conv2
using TD = Tile<64, 16, 4, 1, 64>;                // TileConvDgrad<G> (CIN = 16)
using TW = Tile<64, 32, 4, 1, 64>;                // TileConvWgrad<G> (COUT = 32)
constexpr int B = 5;

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
      exit(2);                                                            \
    }                                                                     \
  } while (0)

static bool read_all(const std::string &path, void *dst, size_t bytes) {
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) return false;
  const bool ok = fread(dst, 1, bytes, f) == bytes;
  fclose(f);
  return ok;
}

int main(int argc, char **argv) {
  using P = PhaseGeom<G>;
  std::vector<float> dY((size_t)B * G::OH * G::OW * G::COUT), W((size_t)G::KK * G::COUT),
      A1((size_t)B * G::H * G::W * G::CIN);
  uint64_t s = 777;
  auto rnd = [&] {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return (uint32_t)(s >> 33);
  };
  for (auto &x : dY) x = ((int)(rnd() % 2001) - 1000) * 1e-5f;
  for (auto &x : W) x = ((int)(rnd() % 2001) - 1000) * 1e-4f;
  for (auto &x : A1) x = (rnd() % 3 == 0) ? 0.f : (rnd() % 1000) * 1e-3f;
  if (argc > 1) {
    const std::string p = argv[1];
    if (!read_all(p + ".dY2.f32", dY.data(), 4 * dY.size()) || !read_all(p + ".W2.f32", W.data(), 4 * W.size()) ||
        !read_all(p + ".act1.f32", A1.data(), 4 * A1.size())) {
      fprintf(stderr, "cannot read %s.{dY2,W2,act1}.f32\n", argv[1]);
      return 4;
    }
    printf("inputs: %s\n", argv[1]);
  }
  // reference dX[b][iy][ix][ci] (relu mask from act1)
  std::vector<double> ref(A1.size(), 0.0);
  for (int b = 0; b < B; ++b)
    for (int oy = 0; oy < G::OH; ++oy)
      for (int ox = 0; ox < G::OW; ++ox)
        for (int ky = 0; ky < G::KH; ++ky)
          for (int kx = 0; kx < G::KW; ++kx)
            for (int ci = 0; ci < G::CIN; ++ci) {
              double t = 0;
              for (int co = 0; co < G::COUT; ++co)
                t += (double)dY[(((size_t)b * G::OH + oy) * G::OW + ox) * G::COUT + co] *
                     W[((size_t)(ky * G::KW + kx) * G::CIN + ci) * G::COUT + co];
              ref[(((size_t)b * G::H + G::S * oy + ky) * G::W + G::S * ox + kx) * G::CIN + ci] += t;
            }
  for (size_t i = 0; i < ref.size(); ++i)
    if (!(A1[i] > 0.f)) ref[i] = 0.0;

  float *ddY, *dW, *dA1, *dX, *dSlab, *dG;
  const int Kw = B * G::OH * G::OW;
  CK(hipMalloc(&ddY, 4 * dY.size()));
  CK(hipMalloc(&dW, 4 * W.size()));
  CK(hipMalloc(&dA1, 4 * A1.size()));
  CK(hipMalloc(&dX, 4 * A1.size()));
  CK(hipMalloc(&dSlab, sizeof(float) * 64 * (G::KK + 1) * G::COUT));
  CK(hipMalloc(&dG, sizeof(float) * (G::KK + 1) * G::COUT));
  CK(hipMemcpy(ddY, dY.data(), 4 * dY.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, W.data(), 4 * W.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dA1, A1.data(), 4 * A1.size(), hipMemcpyHostToDevice));
  const int mp = cdiv(B * P::HQ * P::WQ, TD::BM) * TD::BM;
  const auto dx = gemm_job<TD>(LdConvBwdAPhase<G>{ddY, mp, B}, LdConvBwdBPhase<G>{dW, mp / TD::BM},
                               EpMaskedPhase<G>{dX, dA1, mp, B, MT_ACT_RELU, 0.f}, G::S * G::S * mp, G::CIN, P::KP, 1);
  // conv2's weight-gradient pair of the same launch (net.hip conv_wgrad_jobs, 8 splits)
  const auto wg = gemm_job<TW>(LdIm2colT<G, false>{dA1}, LdColMajor{ddY, G::COUT, -1},
                               EpSlab{dSlab, G::KK + 1, G::COUT}, G::KK, G::COUT, Kw, 8);
  const BiasRowJob<G::COUT> bias{ddY, dSlab + (size_t)G::KK * G::COUT, (size_t)(G::KK + 1) * G::COUT, Kw, wg.kchunk,
                                 wg.gz};
  int bad = 0;
  for (int v = 0; v <= 1; ++v) {
    CK(hipMemset(dX, 0, 4 * A1.size()));
    const int rc = v == 0 ? launch_group(nullptr, dx)
                          : launch_group(nullptr, dx, PairJob<decltype(wg), BiasRowJob<G::COUT>>{wg, bias}, SlabJob{},
                                         NoJob{});
    if (rc != MT_OK) return 3;
    CK(hipDeviceSynchronize());
    std::vector<float> got(A1.size());
    CK(hipMemcpy(got.data(), dX, 4 * got.size(), hipMemcpyDeviceToHost));
    printf("MT_GEMM_DUAL=%d variant %d:", MT_GEMM_DUAL, v);
    int vbad = 0;
    for (int c = 0; c < G::CIN; ++c) {
      double num = 0, den = 0, mx = 0;
      for (size_t i = c; i < got.size(); i += G::CIN) {
        const double d = got[i] - ref[i];
        num += d * d;
        den += ref[i] * ref[i];
        mx = std::fmax(mx, std::fabs(d));
      }
      const double rel = std::sqrt(num / (den > 0 ? den : 1));
      if (rel > 1e-5) {
        ++vbad;
        printf(" c%d=%.1e(max abs %.1e)", c, rel, mx);
      }
    }
    printf(vbad ? "\n" : " all 16 channels within 1e-5\n");
    bad += vbad;
  }
  printf("%s\n", bad ? "MISMATCH" : "all variants match");
  return bad ? 1 : 0;
}
