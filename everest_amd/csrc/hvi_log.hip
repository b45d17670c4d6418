// Log-space hypervolume improvement (q = 1) on gfx950: [upstream] BoTorch
// qLogNoisyExpectedHypervolumeImprovement / qLogExpectedHypervolumeImprovement
// ._compute_log_qehvi with fat = True — the default acquisition of BoFire's MoboStrategy
// (bofire/data_models/strategies/predictives/mobo.py:27-29, built through
// get_acquisition_function at bofire/strategies/predictives/mobo.py:68-90).
//
// Per MC sample s, candidate c and box cell k of the sample's partition:
//   psi_kj = log fatplus(y_j - l_kj; tau_relu),  fatplus(z; t) = t (softplus(z/t) + 0.1/(1 + (z/t)^2))
//   lam_kj = log(min(u_kj, 1e10) - l_kj)
//   a_k    = sum_j fatmin(psi_kj, lam_kj; tau_max),
//            fatmin(a, b; t) = min(a, b) - t log(1 + pareto(|a - b| / t)),  pareto(x) = 2 / (2 + 2x + x^2)
//   LSE_sc = logsumexp_k a_k,   acq_c = logsumexp_s LSE_sc - log S.
// Every cell contributes (the fat tails never vanish), so the scan is dense: a 256-thread
// workgroup owns (sample s, CT candidates, range of cells); the cells are staged through LDS
// in chunks of 256 with their log lengths (one log per cell and objective, shared by the CT
// candidates); each thread walks every G-th cell of the chunk for its candidate keeping an
// online log-sum-exp state (running max m, s0 = sum exp(a - m), s_j = sum exp(a - m) da/dy_j)
// that is merged over the G thread groups and the cell-range splits in a fixed order
// (bitwise reproducible).  hvi_log_reduce then forms LSE_sc, the logmeanexp over samples and
// dG = gout * softmax_s(LSE_sc) * s_j / s0.
#include <algorithm>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int HL_THREADS = 256;
constexpr int HL_CHUNK = 256;

// log_fatplus, fatmin2 and LseState: common.hpp (shared with the general log scan)

// out: [s][split][2 + M][b]  (m, s0, s_j)
template <int M, bool BWD>
__global__ __launch_bounds__(HL_THREADS) void hvi_log_kernel(int b, int nsplit, int CT, int CB,
                                                             const double* __restrict__ G,
                                                             const int* __restrict__ off,
                                                             const double* __restrict__ lo,
                                                             const double* __restrict__ hi, double tr, double tm,
                                                             double* __restrict__ out) {
  constexpr int NO = 2 + (BWD ? M : 0);
  __shared__ double Ls[HL_CHUNK][M];
  __shared__ double Ws[HL_CHUNK][M];
  __shared__ double red[HL_THREADS][NO];
  const int s = blockIdx.y, split = blockIdx.z, tid = threadIdx.x;
  const int GR = HL_THREADS / CT;
  const int cl = tid % CT, g = tid / CT;
  const int c = blockIdx.x * CT + cl;
  double y[M];
#pragma unroll
  for (int j = 0; j < M; ++j) y[j] = (c < b) ? G[((size_t)s * M + j) * b + c] : 0.0;
  LseState<M, BWD> st;
  st.init();
  const int k0 = off[s] + split * CB;
  const int k1 = min(off[s + 1], k0 + CB);
  for (int ks = k0; ks < k1; ks += HL_CHUNK) {
    const int nc = min(HL_CHUNK, k1 - ks);
    __syncthreads();   // previous chunk consumed
    for (int e = tid; e < nc * M; e += HL_THREADS) {
      const int cell = e / M, j = e - cell * M;
      const double l = lo[(size_t)ks * M + e];
      const double u = fmin(hi[(size_t)ks * M + e], HL_UMAX);
      Ls[cell][j] = l;
      Ws[cell][j] = log(u - l);
    }
    __syncthreads();
    if (c < b) {
      for (int k = g; k < nc; k += GR) {
        double a = 0.0, da[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          double dpsi = 0.0, dfm = 0.0;
          const double psi = log_fatplus(y[j] - Ls[k][j], tr, BWD ? &dpsi : nullptr);
          a += fatmin2(psi, Ws[k][j], tm, BWD ? &dfm : nullptr);
          da[j] = dfm * dpsi;
        }
        st.add(a, da);
      }
    }
  }
  red[tid][0] = st.m;
  red[tid][1] = st.s0;
  if (BWD) {
#pragma unroll
    for (int j = 0; j < M; ++j) red[tid][2 + j] = st.g[j];
  }
  __syncthreads();
  if (g == 0 && c < b) {
    for (int q = 1; q < GR; ++q) {
      const double* r = red[q * CT + cl];
      st.merge(r[0], r[1], r + 2);
    }
    double* o = out + ((size_t)s * nsplit + split) * NO * b;
    o[c] = st.m;
    o[(size_t)b + c] = st.s0;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) o[(size_t)(2 + j) * b + c] = st.g[j];
    }
  }
}

// thread per candidate: merge the splits per sample (fixed order) -> LSE_sc (kept in the
// m slot of split 0), acq_c = logsumexp_s LSE_sc - log S; dG = gout softmax_s s_j / s0
template <int M, bool BWD>
__global__ void hvi_log_reduce(int b, int S, int nsplit, double* __restrict__ ws, const int* __restrict__ flags,
                               const double* __restrict__ gout, double* __restrict__ acq,
                               double* __restrict__ dG) {
  constexpr int NO = 2 + (BWD ? M : 0);
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= b) return;
  double mx = -INFINITY;
  for (int s = 0; s < S; ++s) {
    double* o = ws + (size_t)s * nsplit * NO * b;
    LseState<M, BWD> st;
    st.m = o[c];
    st.s0 = o[(size_t)b + c];
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) st.g[j] = o[(size_t)(2 + j) * b + c];
    }
    for (int q = 1; q < nsplit; ++q) {
      const double* r = o + (size_t)q * NO * b;
      double g2[BWD ? M : 1];
      if (BWD) {
#pragma unroll
        for (int j = 0; j < M; ++j) g2[j] = r[(size_t)(2 + j) * b + c];
      }
      st.merge(r[c], r[(size_t)b + c], g2);
    }
    const double lse = (st.s0 > 0.0) ? st.m + log(st.s0) : -INFINITY;
    o[c] = lse;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) o[(size_t)(2 + j) * b + c] = (st.s0 > 0.0) ? st.g[j] / st.s0 : 0.0;
    }
    mx = fmax(mx, lse);
  }
  double sum = 0.0;
  if (mx > -INFINITY) {
    for (int s = 0; s < S; ++s) sum += exp(ws[(size_t)s * nsplit * NO * b + c] - mx);
  }
  const double lme = (mx > -INFINITY) ? mx + log(sum) - log((double)S) : -INFINITY;
  bool bad = false;
  if (flags) {
#pragma unroll
    for (int j = 0; j < M; ++j) bad |= flags[(size_t)j * b + c] != 0;
  }
  if (acq) acq[c] = bad ? nan("") : lme;
  if (BWD) {
    const double go = gout ? gout[c] : 1.0;
    for (int s = 0; s < S; ++s) {
      const double* o = ws + (size_t)s * nsplit * NO * b;
      const double w = (lme > -INFINITY) ? go * exp(o[c] - lme) / (double)S : 0.0;
#pragma unroll
      for (int j = 0; j < M; ++j) dG[((size_t)s * M + j) * b + c] = w * o[(size_t)(2 + j) * b + c];
    }
  }
}

struct HlPlan {
  int CT, nsplit, CB;
};

static HlPlan hl_plan(const evr_qnehvi_state* st, int b) {
  HlPlan p;
  p.CT = b >= 48 ? 64 : (b > 16 ? 32 : 16);
  const int ctiles = cdiv(b, p.CT);
  const int maxc = std::max(st->max_cells, 1);
  const int want = std::max(1, cdiv(2048, (long long)ctiles * st->S));
  p.nsplit = std::min(want, cdiv(maxc, HL_CHUNK));
  p.CB = cdiv(cdiv(maxc, p.nsplit), HL_CHUNK) * HL_CHUNK;
  p.nsplit = cdiv(maxc, p.CB);
  return p;
}

long long hvi_log_workspace(const evr_qnehvi_state* st, int b, int backward) {
  const HlPlan p = hl_plan(st, b);
  return (long long)st->S * p.nsplit * (2 + (backward ? st->m : 0)) * b;
}

template <int M, bool BWD>
static int hvi_log_launch_m(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                            const double* gout, double* work, double* acq, double* dG) {
  const HlPlan p = hl_plan(st, b);
  dim3 grid(cdiv(b, p.CT), st->S, p.nsplit);
  hvi_log_kernel<M, BWD><<<grid, HL_THREADS, 0, s>>>(b, p.nsplit, p.CT, p.CB, G, st->cell_off, st->cell_lo,
                                                     st->cell_hi, st->tau_relu, st->tau_max, work);
  EVR_LAUNCH_CHECK();
  hvi_log_reduce<M, BWD><<<cdiv(b, 64), 64, 0, s>>>(b, st->S, p.nsplit, work, flags, gout, acq, dG);
  EVR_LAUNCH_CHECK();
  return 0;
}

int hvi_log_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                   const double* gout, double* work, double* acq, double* dG, bool backward) {
  EVR_CHECK(st->cell_lo && st->cell_hi && st->cell_off, "hvi (log): the log-space scan needs explicit cells");
  EVR_CHECK(st->tau_relu > 0.0 && st->tau_max > 0.0, "hvi (log): tau_relu / tau_max must be positive");
#define HL(MM)                                                                                         \
  case MM:                                                                                             \
    return backward ? hvi_log_launch_m<MM, true>(s, st, b, G, flags, gout, work, acq, dG)              \
                    : hvi_log_launch_m<MM, false>(s, st, b, G, flags, gout, work, acq, dG);
  switch (st->m) {
    HL(1) HL(2) HL(3) HL(4) HL(5) HL(6) HL(7) HL(8)
    default:
      EVR_CHECK(false, "hvi (log): number of objectives m=%d not supported (1..8)", st->m);
  }
#undef HL
}

}  // namespace evr
