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
//
// Compressed cells (device box decomposition: one u64 key per cell of point indices, the
// sample's point table) take hvi_logk_kernel instead.  Every lower bound l_kj is the
// coordinate -pt[P_j][j] of one of the sample's stride points, so psi_kj = log fatplus(y_j -
// l_kj) takes at most stride distinct values per (candidate, objective): the workgroup
// tabulates (psi, dpsi) over the point table once for its CT candidates in LDS, and the
// per-(cell, candidate) work drops to the M fatmins and the log-sum-exp step.  A thread owns
// cells (lam_kj = log(min(u, 1e10) - l) once per cell, shared by the CT candidates) and keeps
// CT online log-sum-exp states, merged over the workgroup by a fixed-order tree.  The output
// layout is hvi_log_kernel's, so hvi_log_reduce finishes both.  EVR_LOG=dense keeps the
// dense kernel (A/B).
#include <algorithm>
#include <cstdlib>
#include <cstring>

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

// workgroup per candidate, thread per sample: merge the splits per sample (fixed order) ->
// LSE_sc (kept in the m slot of split 0), then acq_c = logsumexp_s LSE_sc - log S by two
// fixed-order tree reductions (max, then sum of exp), and dG = gout softmax_s s_j / s0.
// (The earlier thread-per-candidate loop walked the S samples three times serially: ~320 us
// of load latency per launch at any b.)
constexpr int HLR_THREADS = 256;

template <int M, bool BWD>
__global__ __launch_bounds__(HLR_THREADS) void hvi_log_reduce(int b, int S, int nsplit, double* __restrict__ ws,
                                                              const int* __restrict__ flags,
                                                              const double* __restrict__ gout,
                                                              double* __restrict__ acq, double* __restrict__ dG) {
  constexpr int NO = 2 + (BWD ? M : 0);
  __shared__ double rd[HLR_THREADS];
  const int c = blockIdx.x, tid = threadIdx.x;
  double mloc = -INFINITY;
  for (int s = tid; s < S; s += HLR_THREADS) {
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
    mloc = fmax(mloc, lse);
  }
  rd[tid] = mloc;
  for (int h = HLR_THREADS / 2; h > 0; h >>= 1) {
    __syncthreads();
    if (tid < h) rd[tid] = fmax(rd[tid], rd[tid + h]);
  }
  __syncthreads();
  const double mx = rd[0];
  __syncthreads();
  double sl = 0.0;
  if (mx > -INFINITY)
    for (int s = tid; s < S; s += HLR_THREADS) sl += exp(ws[(size_t)s * nsplit * NO * b + c] - mx);
  rd[tid] = sl;
  for (int h = HLR_THREADS / 2; h > 0; h >>= 1) {
    __syncthreads();
    if (tid < h) rd[tid] += rd[tid + h];
  }
  __syncthreads();
  const double lme = (mx > -INFINITY) ? mx + log(rd[0]) - log((double)S) : -INFINITY;
  if (tid == 0) {
    bool bad = false;
    if (flags) {
#pragma unroll
      for (int j = 0; j < M; ++j) bad |= flags[(size_t)j * b + c] != 0;
    }
    if (acq) acq[c] = bad ? nan("") : lme;
  }
  if (BWD) {
    const double go = gout ? gout[c] : 1.0;
    for (int s = tid; s < S; s += HLR_THREADS) {
      const double* o = ws + (size_t)s * nsplit * NO * b;
      const double w = (lme > -INFINITY) ? go * exp(o[c] - lme) / (double)S : 0.0;
#pragma unroll
      for (int j = 0; j < M; ++j) dG[((size_t)s * M + j) * b + c] = w * o[(size_t)(2 + j) * b + c];
    }
  }
}

// keyed scan: LDS = point table (stride x M f64) | rank -> index (stride int) | table
// [CT][M][stride] of psi (forward) or (psi, dpsi) pairs (backward)
// candidates per workgroup: the per-cell work (key decode, M - 1 logs of the cell widths) is
// shared by CT candidates.  Backward: CT = 2, 512 threads (2 workgroups = 4 waves per SIMD);
// EVR_LOGK=4 selects CT = 4 / 1024 threads (A/B: 11.7 vs 9.7 ms at b = 512, it spills)
constexpr int HLK_CT_FWD = 4;
constexpr int HLK_MAXT = 1024;

__host__ __device__ inline size_t hlk_flt_off(int stride, int M) {
  return (((size_t)stride * M * 8 + (size_t)stride * 4) + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t hlk_tab_off(int stride, int M) {
  return (hlk_flt_off(stride, M) + sizeof(FastLogTabs) + 15) & ~(size_t)15;
}
// the table region is reused by the final merge (HL_THREADS x (2 [+ M]) doubles)
__host__ __device__ inline size_t hlk_lds_bytes(int stride, int M, int CT, bool bwd) {
  const size_t tab = (size_t)CT * M * stride * (bwd ? 16 : 8);
  const size_t red = (size_t)HLK_MAXT * (2 + (bwd ? M : 0)) * 8;
  return hlk_tab_off(stride, M) + (tab > red ? tab : red);
}

// online log-sum-exp step (LseState::add with the table exp)
template <int M, bool BWD>
__device__ __forceinline__ void lse_add_tab(LseState<M, BWD>& st, double a, const double* da, const FastLogTabs& T) {
  if (a == -INFINITY) return;
  const double e = exp_tab_neg(-fabs(a - st.m), T);
  if (a > st.m) {
    st.s0 = fma(st.s0, e, 1.0);
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) st.g[j] = fma(st.g[j], e, da[j]);
    }
    st.m = a;
  } else {
    st.s0 += e;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) st.g[j] = fma(e, da[j], st.g[j]);
    }
  }
}

template <int M, bool BWD, int CT, int HLK_THREADS>
__device__ __forceinline__ void hlk_merge_out(LseState<M, BWD>* st, int nc, double* tab, double* out, int s,
                                              int nsplit, int split, int b, int c0) {
  constexpr int NO = 2 + (BWD ? M : 0);
  const int tid = threadIdx.x;
  // fixed-order tree merge over the workgroup, one candidate at a time (in the table's LDS)
  double(*red)[NO] = reinterpret_cast<double(*)[NO]>(tab);
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if (c >= nc) break;
    __syncthreads();
    red[tid][0] = st[c].m;
    red[tid][1] = st[c].s0;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) red[tid][2 + j] = st[c].g[j];
    }
    for (int h = HLK_THREADS / 2; h > 0; h >>= 1) {
      __syncthreads();
      if (tid < h) {
        LseState<M, BWD> a;
        a.m = red[tid][0];
        a.s0 = red[tid][1];
        if (BWD) {
#pragma unroll
          for (int j = 0; j < M; ++j) a.g[j] = red[tid][2 + j];
        }
        a.merge(red[tid + h][0], red[tid + h][1], &red[tid + h][2]);
        red[tid][0] = a.m;
        red[tid][1] = a.s0;
        if (BWD) {
#pragma unroll
          for (int j = 0; j < M; ++j) red[tid][2 + j] = a.g[j];
        }
      }
    }
    if (tid == 0) {
      double* o = out + ((size_t)s * nsplit + split) * NO * b;
      const int gc = c0 + c;
      o[gc] = red[0][0];
      o[(size_t)b + gc] = red[0][1];
      if (BWD) {
#pragma unroll
        for (int j = 0; j < M; ++j) o[(size_t)(2 + j) * b + gc] = red[0][2 + j];
      }
    }
  }
}

template <int M, bool BWD, int CT, int HLK_THREADS>
__global__ __launch_bounds__(HLK_THREADS) void hvi_logk_kernel(int b, int nsplit, int CB, int stride,
                                                              const double* __restrict__ G,
                                                              const int* __restrict__ off,
                                                              const unsigned long long* __restrict__ keys,
                                                              const double* __restrict__ pts,
                                                              const int* __restrict__ rank0, double tr, double tm,
                                                              double* __restrict__ out) {
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char hl_dyn[];
  double* pt = (double*)hl_dyn;
  int* rk = (int*)(pt + (size_t)stride * M);
  FastLogTabs& T = *reinterpret_cast<FastLogTabs*>(hl_dyn + hlk_flt_off(stride, M));
  double* tab = (double*)(hl_dyn + hlk_tab_off(stride, M));
  T.fill(threadIdx.x, HLK_THREADS);
  __syncthreads();   // the psi table's objective-0 fatmins use T
  const int s = blockIdx.y, split = blockIdx.z, tid = threadIdx.x;
  const int c0 = blockIdx.x * CT;
  const double* gp = pts + (size_t)s * stride * M;
  for (int e = tid; e < stride * M; e += HLK_THREADS) pt[e] = gp[e];
  for (int e = tid; e < stride; e += HLK_THREADS) rk[e] = rank0[(size_t)s * stride + e];
  const double itm = 1.0 / tm;
  // table [c][j][p]: y_j - l = y_j + pt[p][j] (l = -pt[p][j], the dense kernel's operands
  // exactly).  Objective 0's upper bound is always the clamp (hi_0 = +inf), so its whole
  // fatmin term depends on (c, p) alone and is tabulated instead of psi: (value, derivative)
  for (int e = tid; e < CT * M * stride; e += HLK_THREADS) {
    const int c = e / (M * stride), r = e - c * (M * stride), j = r / stride, p = r - j * stride;
    const int gc = min(c0 + c, b - 1);
    const double lo = -gp[(size_t)p * M + j];
    const double z = G[((size_t)s * M + j) * b + gc] - lo;
    double dpsi = 0.0;
    double v = log_fatplus(z, tr, BWD ? &dpsi : nullptr);
    if (j == 0) {
      double dfm;
      v = fatmin_fast(v, log(HL_UMAX - lo), tm, itm, &dfm, T);
      dpsi *= dfm;
    }
    if (BWD) {
      tab[2 * (size_t)e] = v;
      tab[2 * (size_t)e + 1] = dpsi;
    } else {
      tab[e] = v;
    }
  }
  __syncthreads();
  const int nc = min(CT, b - c0);
  LseState<M, BWD> st[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) st[c].init();
  const int k0 = off[s] + split * CB;
  const int k1 = min(off[s + 1], k0 + CB);
  for (int k = k0 + tid; k < k1; k += HLK_THREADS) {
    const unsigned long long key = keys[k];
    int P[M];
    P[0] = rk[K::field(key, 0)];
#pragma unroll
    for (int j = 1; j < M; ++j) P[j] = K::field(key, j);
    double lam[M];
#pragma unroll
    for (int j = 1; j < M; ++j) {
      double bl = -INFINITY;
#pragma unroll
      for (int i = 0; i < j; ++i) bl = fmax(bl, pt[P[i] * M + j]);
      const double lo = -pt[P[j] * M + j];
      lam[j] = log_tab(fmin(-bl, HL_UMAX) - lo, T);
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      if (c < nc) {
        double a, da[M] = {};
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const size_t ti = ((size_t)c * M + j) * stride + P[j];
          double v, dv = 0.0;
          if (BWD) {
            const double2 pd = *reinterpret_cast<const double2*>(tab + 2 * ti);
            v = pd.x;
            dv = pd.y;
          } else {
            v = tab[ti];
          }
          if (j == 0) {
            a = v;
            da[0] = dv;
          } else {
            double dfm;
            a += fatmin_fast(v, lam[j], tm, itm, &dfm, T);
            da[j] = dfm * dv;
          }
        }
        lse_add_tab(st[c], a, da, T);
      }
    }
  }
  hlk_merge_out<M, BWD, CT, HLK_THREADS>(st, nc, tab, out, s, nsplit, split, b, c0);
}

// (A kd-bounded variant that skipped kd groups bounded below 2^-60 of the sample's sum was
// measured slower at the bench state — 10.3 vs 9.4 ms at b = 512, profiles/r05/m: with
// tau_relu = 1e-6 few groups fall below the bound — and removed in round 6.)

struct HlPlan {
  int CT, nsplit, CB;
  bool keyed;
};

// candidates per workgroup of the keyed backward (CT = 4 with 1024 threads measured slower:
// 11.7 vs 9.7 ms, the 128-VGPR cap spills)
constexpr int HLK_CT_BWD = 2;

static bool hl_keyed(const evr_qnehvi_state* st, bool bwd) {
  // EVR_LOG=dense: the dense kernel over the explicit rows even when keys exist (the parity
  // test's reference; read per plan)
  const char* e = std::getenv("EVR_LOG");
  const bool dense = e && !std::strcmp(e, "dense");
  return !dense && st->cell_keys && st->cell_pts && st->cell_rank0 && st->pts_stride > 0 &&
         hlk_lds_bytes(st->pts_stride, st->m, bwd ? HLK_CT_BWD : HLK_CT_FWD, bwd) <= 150 * 1024;
}

static HlPlan hl_plan(const evr_qnehvi_state* st, int b, bool bwd) {
  HlPlan p;
  p.keyed = hl_keyed(st, bwd);
  if (p.keyed)
    p.CT = bwd ? HLK_CT_BWD : HLK_CT_FWD;
  else
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
  const HlPlan p = hl_plan(st, b, backward != 0);
  return (long long)st->S * p.nsplit * (2 + (backward ? st->m : 0)) * b;
}

template <int M, bool BWD>
static int hvi_log_launch_m(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                            const double* gout, double* work, double* acq, double* dG) {
  const HlPlan p = hl_plan(st, b, BWD);
  dim3 grid(cdiv(b, p.CT), st->S, p.nsplit);
  if (p.keyed) {
    const size_t lds = hlk_lds_bytes(st->pts_stride, M, p.CT, BWD);
#define HLK_GO(CT_, NT_)                                                                                     \
  do {                                                                                                       \
    EVR_HIP(hipFuncSetAttribute((const void*)hvi_logk_kernel<M, BWD, CT_, NT_>,                              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                      \
    hvi_logk_kernel<M, BWD, CT_, NT_><<<grid, NT_, lds, s>>>(b, p.nsplit, p.CB, st->pts_stride, G,            \
                                                             st->cell_off, st->cell_keys, st->cell_pts,      \
                                                             st->cell_rank0, st->tau_relu, st->tau_max, work); \
  } while (0)
    if (!BWD)
      HLK_GO(HLK_CT_FWD, 1024);
    else
      HLK_GO(HLK_CT_BWD, 512);
#undef HLK_GO
  } else {
    EVR_CHECK(st->cell_lo && st->cell_hi, "hvi (log): the dense log-space scan needs explicit cells");
    hvi_log_kernel<M, BWD><<<grid, HL_THREADS, 0, s>>>(b, p.nsplit, p.CT, p.CB, G, st->cell_off, st->cell_lo,
                                                       st->cell_hi, st->tau_relu, st->tau_max, work);
  }
  EVR_LAUNCH_CHECK();
  hvi_log_reduce<M, BWD><<<b, HLR_THREADS, 0, s>>>(b, st->S, p.nsplit, work, flags, gout, acq, dG);
  EVR_LAUNCH_CHECK();
  return 0;
}

int hvi_log_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                   const double* gout, double* work, double* acq, double* dG, bool backward) {
  EVR_CHECK(st->cell_off && ((st->cell_lo && st->cell_hi) || st->cell_keys),
            "hvi (log): the log-space scan needs explicit or compressed cells");
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
