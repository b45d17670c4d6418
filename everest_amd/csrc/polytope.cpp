// Hit-and-run sampler over a polytope {x : A x <= b} (optionally restricted to the affine
// subspace x0 + span(N) of linear equalities) — the raw-candidate generator of optimize_acqf
// under linear constraints ([upstream] botorch HitAndRunPolytopeSampler through
// sample_q_batches_from_polytope, called by optimize_acqf at
// bofire/strategies/predictives/botorch.py:384-405; the same sampler draws RandomStrategy's
// constrained candidates, bofire/strategies/random.py:300-326).
//
// The chain is sequential by construction (every step starts from the previous point), so it
// runs on the host; what made the Python loop slow was ~40 numpy calls per step.  Step i draws
// its 2k + 1 variates from a counter-based stream (SplitMix64 of seed + counter), so any step
// can be restated alone: k standard normals by Box-Muller (cos branch) for the direction,
// one uniform for the position on the chord.  Every sum runs in index order, so
// tests/test_native_cpu.py restates the chain in plain Python and compares it step for step.
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/everest_amd.h"

namespace evr {
void set_error(const char* fmt, ...);
}

namespace {

inline uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// The c-th variate of the stream: SplitMix64's output at state seed + (c + 1) * golden gamma,
// as a double in [0, 1) from its top 53 bits.
inline double uniform_at(uint64_t seed, uint64_t c) {
  return static_cast<double>(splitmix64(seed + (c + 1) * 0x9E3779B97F4A7C15ull) >> 11) * 0x1.0p-53;
}

}  // namespace

extern "C" int evr_hit_and_run(int d, int rows, const double* A, const double* b, int k, const double* N,
                               const double* x0, long long n, unsigned long long seed, long long n_burnin,
                               long long n_thinning, double* out) {
  if (d < 1 || rows < 1 || k < 1 || k > d || n < 0 || n_burnin < 0 || n_thinning < 1 || !A || !b || !N || !x0 ||
      (n > 0 && !out)) {
    evr::set_error("evr_hit_and_run: bad arguments (d=%d rows=%d k=%d n=%lld burnin=%lld thinning=%lld)", d, rows,
                   k, n, n_burnin, n_thinning);
    return 1;
  }
  const double two_pi = 6.283185307179586;
  std::vector<double> x(x0, x0 + d), z(k), r(d);
  const long long total = n_burnin + n * n_thinning;
  const uint64_t per = 2ull * static_cast<uint64_t>(k) + 1ull;
  long long kept = 0;
  for (long long it = 0; it < total; ++it) {
    const uint64_t c0 = static_cast<uint64_t>(it) * per;
    for (int j = 0; j < k; ++j) {
      const double u1 = 1.0 - uniform_at(seed, c0 + 2ull * j);       // (0, 1]
      const double u2 = uniform_at(seed, c0 + 2ull * j + 1ull);
      z[j] = std::sqrt(-2.0 * std::log(u1)) * std::cos(two_pi * u2);
    }
    double nr2 = 0.0;
    for (int i = 0; i < d; ++i) {
      double s = 0.0;
      for (int j = 0; j < k; ++j) s += N[i * k + j] * z[j];
      r[i] = s;
      nr2 += s * s;
    }
    const double nr = std::sqrt(nr2);
    if (nr > 0.0) {
      for (int i = 0; i < d; ++i) r[i] /= nr;
      double tmax = 0.0, tmin = 0.0;
      bool has_max = false, has_min = false;
      for (int q = 0; q < rows; ++q) {
        double ar = 0.0, ax = 0.0;
        for (int i = 0; i < d; ++i) {
          ar += A[q * d + i] * r[i];
          ax += A[q * d + i] * x[i];
        }
        const double t = (b[q] - ax) / ar;
        if (ar > 1e-14) {
          if (!has_max || t < tmax) tmax = t;
          has_max = true;
        } else if (ar < -1e-14) {
          if (!has_min || t > tmin) tmin = t;
          has_min = true;
        }
      }
      const double u = uniform_at(seed, c0 + 2ull * k);
      const double step = tmin + (tmax - tmin) * u;
      for (int i = 0; i < d; ++i) x[i] += step * r[i];
    }
    if (it >= n_burnin && (it - n_burnin) % n_thinning == n_thinning - 1) {
      for (int i = 0; i < d; ++i) out[kept * d + i] = x[i];
      ++kept;
    }
  }
  return 0;
}
