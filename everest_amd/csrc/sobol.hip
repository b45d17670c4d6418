// Scrambled-Sobol normal base samples on the device.
//
// BoTorch draws qNEHVI's quasi-MC base samples with draw_sobol_normal_samples
// ([upstream] NormalQMCEngine(inv_transform=True) over torch.quasirandom.SobolEngine,
// scramble=True, seed drawn from the strategy's torch RNG, bofire/strategies/predictives/
// botorch.py:86): a 30-bit digital sequence with Owen/LMS scrambling, then
// z = sqrt(2) erfinv(2 (0.5 + (1 - eps)(u - 0.5)) - 1).  On the host that costs ~0.15 s per
// ask() at 2560 dimensions (scramble + serial draw + erfinv).  Here:
//   * evr_sobol_scramble (host): the scrambling matrices are the LSBs of the mt19937 stream
//     of torch.Generator().manual_seed(seed) (shift bits dim x 30, then dim x 30 x 30 lower-
//     triangular bits, upper triangle consumed and discarded, diagonal forced to 1), applied
//     to the direction numbers as GF(2) matrix-vector products — bit-identical to
//     SobolEngine.sobolstate / .shift;
//   * evr_sobol_normal (device): point k = shift XOR (XOR of direction numbers over the set
//     bits of gray(k)) — the closed form of the engine's sequential rightmost-zero walk —
//     scaled by 2^-30 (point 0 goes through float32 as SobolEngine._first_point does), then
//     the inverse-normal transform with torch's calc_erfinv (rational seed + 2 Newton steps).
#include <algorithm>
#include <cstdint>
#include <random>
#include <thread>
#include <vector>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int SOBOL_MAXBIT = 30;

// torch calc_erfinv restated (c10/util/math_compat / ATen Math.h): Pavlis' rational
// approximation followed by two Newton-Raphson steps.
__device__ __forceinline__ double erfinv_torch(double y) {
#pragma clang fp contract(off)
  const double a0 = 0.886226899, a1 = -1.645349621, a2 = 0.914624893, a3 = -0.140543331;
  const double b0 = -2.118377725, b1 = 1.442710462, b2 = -0.329097515, b3 = 0.012229801;
  const double c0 = -1.970840454, c1 = -1.624906493, c2 = 3.429567803, c3 = 1.641345311;
  const double d0 = 3.543889200, d1 = 1.637067800;
  const double ya = fabs(y);
  if (ya > 1.0) return nan("");
  if (ya == 1.0) return copysign(INFINITY, y);
  double x;
  if (ya <= 0.7) {
    const double z = y * y;
    const double num = (((a3 * z + a2) * z + a1) * z + a0);
    const double dem = ((((b3 * z + b2) * z + b1) * z + b0) * z + 1.0);
    x = y * num / dem;
  } else {
    const double z = sqrt(-log((1.0 - ya) / 2.0));
    const double num = ((c3 * z + c2) * z + c1) * z + c0;
    const double dem = (d1 * z + d0) * z + 1.0;
    x = copysign(num, y) / dem;
  }
  const double two_over_sqrt_pi = 2.0 / 1.7724538509055159;  // (T)2 / (T)sqrt(pi)
  x = x - (erf(x) - y) / (two_over_sqrt_pi * exp(-x * x));
  x = x - (erf(x) - y) / (two_over_sqrt_pi * exp(-x * x));
  return x;
}

// layout 0: out[k * nd + t];  layout 1: out[(o * np + p) * n + k] with t = p * m + o.
__global__ __launch_bounds__(256) void sobol_normal_kernel(int n, int nd, int d0, const long long* __restrict__ V,
                                                           const long long* __restrict__ shift, int layout, int m,
                                                           double* __restrict__ out) {
#pragma clang fp contract(off)
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)n * nd) return;
  int k, t;
  if (layout == 0) {
    t = (int)(e % nd);
    k = (int)(e / nd);
  } else {
    k = (int)(e % n);
    t = (int)(e / n);
  }
  const int dim = d0 + t;
  double u;
  if (k == 0) {
    u = (double)(float)shift[dim] / 1073741824.0;  // _first_point: int64 / 2**30 in float32
  } else {
    long long x = shift[dim];
    unsigned g = (unsigned)k ^ ((unsigned)k >> 1);
    const long long* row = V + (size_t)dim * SOBOL_MAXBIT;
    while (g) {
      const int bit = __builtin_ctz(g);
      x ^= row[bit];
      g &= g - 1;
    }
    u = (double)x * (1.0 / 1073741824.0);
  }
  const double eps = 2.220446049250313e-16;
  const double v = 0.5 + (1.0 - eps) * (u - 0.5);
  const double z = erfinv_torch(2.0 * v - 1.0) * 1.4142135623730951;
  size_t idx;
  if (layout == 0) {
    idx = (size_t)k * nd + t;
  } else {
    const int p = t / m, o = t - p * m;
    const int np = nd / m;
    idx = ((size_t)o * np + p) * n + k;
  }
  out[idx] = z;
}

}  // namespace evr

using namespace evr;

extern "C" {

int evr_sobol_scramble(int dim, unsigned long long seed, long long* V, long long* shift) {
  EVR_CHECK(dim >= 1 && V && shift, "evr_sobol_scramble: bad arguments");
  std::mt19937 mt((uint32_t)(seed & 0xffffffffull));
  for (int d = 0; d < dim; ++d) {
    long long s = 0;
    for (int b = 0; b < SOBOL_MAXBIT; ++b) s |= (long long)(mt() & 1u) << b;
    shift[d] = s;
  }
  // lower-triangular scrambling matrices, one row per bit: ltm_dots[d][p] = sum_{k<=p}
  // bit(d,p,k) 2^(29-k) with the diagonal forced to 1.
  std::vector<uint32_t> dots((size_t)dim * SOBOL_MAXBIT);
  for (int d = 0; d < dim; ++d)
    for (int p = 0; p < SOBOL_MAXBIT; ++p) {
      uint32_t r = 0;
      for (int k = 0; k < SOBOL_MAXBIT; ++k) {
        const uint32_t bit = mt() & 1u;
        if (k < p && bit) r |= 1u << (SOBOL_MAXBIT - 1 - k);
      }
      r |= 1u << (SOBOL_MAXBIT - 1 - p);
      dots[(size_t)d * SOBOL_MAXBIT + p] = r;
    }
  auto work = [&](int dbeg, int dend) {
    for (int d = dbeg; d < dend; ++d) {
      const uint32_t* ld = &dots[(size_t)d * SOBOL_MAXBIT];
      for (int j = 0; j < SOBOL_MAXBIT; ++j) {
        const uint32_t v = (uint32_t)V[(size_t)d * SOBOL_MAXBIT + j];
        long long t2 = 0;
        for (int p = SOBOL_MAXBIT - 1, l = 0; p >= 0; --p, ++l)
          t2 |= (long long)(__builtin_popcount(ld[p] & v) & 1) << l;
        V[(size_t)d * SOBOL_MAXBIT + j] = t2;
      }
    }
  };
  const int nth = dim >= 512 ? 8 : 1;
  if (nth == 1) {
    work(0, dim);
  } else {
    std::vector<std::thread> th;
    const int per = (dim + nth - 1) / nth;
    for (int i = 0; i < nth; ++i) {
      const int a = i * per, b = std::min(dim, a + per);
      if (a < b) th.emplace_back(work, a, b);
    }
    for (auto& t : th) t.join();
  }
  return 0;
}

int evr_sobol_normal(void* stream, int n, int nd, int d0, const long long* V, const long long* shift, int layout,
                     int m, double* out) {
  EVR_CHECK(n >= 0 && nd >= 0 && d0 >= 0 && V && shift && out, "evr_sobol_normal: bad arguments");
  EVR_CHECK(layout == 0 || (layout == 1 && m >= 1 && nd % m == 0), "evr_sobol_normal: bad layout");
  EVR_CHECK(n <= (1 << 30), "evr_sobol_normal: n exceeds the 2^30 points of a 30-bit sequence");
  const long long tot = (long long)n * nd;
  if (tot == 0) return 0;
  sobol_normal_kernel<<<cdiv(tot, 256), 256, 0, (hipStream_t)stream>>>(n, nd, d0, V, shift, layout, m, out);
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
