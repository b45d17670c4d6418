#include <algorithm>
#include <cstdlib>
#include <string>
// qNEHVI (q = 1) device kernels on gfx950: cached-Cholesky sampling, box-cell hypervolume
// improvement scan (forward + backward), Pareto / prune masks.
//
// Restates [upstream] BoTorch qNoisyExpectedHypervolumeImprovement as BoFire builds it
// (bofire/strategies/predictives/qnehvi.py:39-52): samples y_s = mu + L21 z_base + L22 z_q
// (sample_cached_cholesky, psd_safe_cholesky(max_tries=6) on the 1x1 new block), objective
// g = a*y + b (bofire/utils/torch_tools.py:389-398), HVI_s = sum_cells prod_j
// clamp_min(min(g_j, u_j) - l_j, 0), acquisition = mean_s HVI_s.
#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

// -------------------------------------------------------------------------------------
// samples: block = BX candidates x RY row groups (256 threads); the row sums of squares
// are split over the RY groups and reduced through LDS in a fixed order, then every
// group writes its share of the S samples.  Grid (candidate tiles, m).
// -------------------------------------------------------------------------------------
template <int BX>
__global__ __launch_bounds__(256) void qn_samples_kernel(int n, int nb, int S, int nh, int m, int b,
                                                         const double* __restrict__ R,
                                                         const double* __restrict__ cc,
                                                         const double* __restrict__ ym,
                                                         const double* __restrict__ ys,
                                                         const double* __restrict__ kxx,
                                                         const double* __restrict__ zq,
                                                         const double* __restrict__ oa,
                                                         const double* __restrict__ ob, double* __restrict__ G,
                                                         double* __restrict__ L22, int* __restrict__ flags) {
  constexpr int RY = 256 / BX;
  __shared__ double red[2][RY][BX];
  const int j = blockIdx.y;
  const int cx = threadIdx.x % BX, ry = threadIdx.x / BX;
  const int c = blockIdx.x * BX + cx;
  const bool live = c < b;
  const long long Rr = (long long)n + nb + nh + 1;
  const double* Rj = R + (size_t)j * Rr * b;
  double ssv = 0.0, ssw = 0.0;
  if (live) {
    for (int i = ry; i < n; i += RY) {
      const double v = Rj[(size_t)i * b + c];
      ssv = fma(v, v, ssv);
    }
    for (int i = n + ry; i < n + nb; i += RY) {
      const double v = Rj[(size_t)i * b + c];
      ssw = fma(v, v, ssw);
    }
  }
  red[0][ry][cx] = ssv;
  red[1][ry][cx] = ssw;
  __syncthreads();
  ssv = 0.0;
  ssw = 0.0;
#pragma unroll
  for (int g = 0; g < RY; ++g) {
    ssv += red[0][g][cx];
    ssw += red[1][g][cx];
  }
  if (!live) return;
  const double a = Rj[(size_t)(n + nb + nh) * b + c];
  const double s = ys[j];
  const double mu = ym[j] + s * (cc[j] + a);
  const double var = s * s * (kxx[j] - ssv);
  const double br = var - ssw;
  // psd_safe_cholesky on the 1x1 block: plain, then total jitter 1e-8*10^(t-1), t=1..6
  double l22 = nan("");
  int flag = 1;
  if (!isnan(br)) {
    for (int t = 0; t <= 6; ++t) {
      const double jit = (t == 0) ? 0.0 : 1e-8 * pow(10.0, (double)(t - 1));
      if (br + jit > 0.0) {
        l22 = sqrt(br + jit);
        flag = 0;
        break;
      }
    }
  }
  if (ry == 0) {
    L22[(size_t)j * b + c] = l22;
    flags[(size_t)j * b + c] = flag;
  }
  const double A = oa[j], B0 = ob[j];
  const double* h = Rj + (size_t)(n + nb) * b + c;
  for (int si = ry; si < S; si += RY) {
    const double y = (nh ? mu + h[(size_t)si * b] : mu) + l22 * zq[(size_t)si * m + j];
    G[((size_t)si * m + j) * b + c] = fma(A, y, B0);
  }
}

__global__ void mean_over_samples_kernel(int S, int b, const double* __restrict__ partial, double* __restrict__ acq) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= b) return;
  double s = 0.0;
  for (int i = 0; i < S; ++i) s += partial[(size_t)i * b + c];
  acq[c] = s / (double)S;
}

// samples backward: same (BX x RY) blocking; writes gR_j (Rr x b)
template <int BX>
__global__ __launch_bounds__(256) void qn_samples_bwd_kernel(int n, int nb, int S, int nh, int m, int b,
                                                             const double* __restrict__ R,
                                                             const double* __restrict__ ys,
                                                             const double* __restrict__ zq,
                                                             const double* __restrict__ oa,
                                                             const double* __restrict__ L22,
                                                             const double* __restrict__ dG, double* __restrict__ gR) {
  constexpr int RY = 256 / BX;
  __shared__ double red[2][RY][BX];
  const int j = blockIdx.y;
  const int cx = threadIdx.x % BX, ry = threadIdx.x / BX;
  const int c = blockIdx.x * BX + cx;
  const bool live = c < b;
  const long long Rr = (long long)n + nb + nh + 1;
  const double* Rj = R + (size_t)j * Rr * b;
  double* gj = gR + (size_t)j * Rr * b;
  const double A = oa[j];
  double dmu = 0.0, dl = 0.0;
  if (live) {
    for (int si = ry; si < S; si += RY) {
      const double dy = A * dG[((size_t)si * m + j) * b + c];
      dmu += dy;
      dl = fma(dy, zq[(size_t)si * m + j], dl);
      if (nh) gj[(size_t)(n + nb + si) * b + c] = dy;
    }
  }
  red[0][ry][cx] = dmu;
  red[1][ry][cx] = dl;
  __syncthreads();
  dmu = 0.0;
  dl = 0.0;
#pragma unroll
  for (int g = 0; g < RY; ++g) {
    dmu += red[0][g][cx];
    dl += red[1][g][cx];
  }
  if (!live) return;
  const double s = ys[j];
  if (ry == 0) gj[(size_t)(n + nb + nh) * b + c] = s * dmu;
  const double l22 = L22[(size_t)j * b + c];
  const double dbr = dl / (2.0 * l22);
  const double dssv = -s * s * dbr;  // var = s^2 (kxx - ssv); br = var - ssw
  const double dssw = -dbr;
  for (int i = ry; i < n; i += RY) gj[(size_t)i * b + c] = 2.0 * Rj[(size_t)i * b + c] * dssv;
  for (int i = n + ry; i < n + nb; i += RY) gj[(size_t)i * b + c] = 2.0 * Rj[(size_t)i * b + c] * dssw;
}

// -------------------------------------------------------------------------------------
// Pareto mask: thread per (sample s [fast], point i); O layout [j][i][s]
// -------------------------------------------------------------------------------------
template <int M>
__global__ void pareto_kernel(int S, int n, const double* __restrict__ O, const double* __restrict__ ref,
                              int dedup, unsigned char* __restrict__ mask, int* __restrict__ counts) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (s >= S) return;
  double yi[M];
  bool better = true;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    yi[j] = O[((size_t)j * n + i) * S + s];
    better &= yi[j] > ref[j];
  }
  bool nd = better;
  for (int k = 0; k < n && nd; ++k) {
    if (k == i) continue;
    bool ge = true, gt = false, eq = true;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const double v = O[((size_t)j * n + k) * S + s];
      ge &= v >= yi[j];
      gt |= v > yi[j];
      eq &= v == yi[j];
    }
    if (ge && gt) nd = false;
    if (dedup && eq && k < i) nd = false;
  }
  if (mask) mask[(size_t)s * n + i] = nd ? 1 : 0;
  if (counts && nd) atomicAdd(&counts[i], 1);
}

// The same test with the points of SB samples staged in LDS (loads of SB contiguous samples
// per (objective, point)); a thread walks point i's dominance scan over LDS broadcasts
// instead of n dependent L2 loads per (sample, point).
template <int M>
__global__ __launch_bounds__(256) void pareto_lds_kernel(int S, int n, int SB, const double* __restrict__ O,
                                                         const double* __restrict__ ref, int dedup,
                                                         unsigned char* __restrict__ mask, int* __restrict__ counts) {
  extern __shared__ double pts[];   // [SB][n][M]
  const int s0 = blockIdx.x * SB, sb = min(SB, S - s0);
  const int tot = M * n * sb;
  for (int e = threadIdx.x; e < tot; e += 256) {
    const int j = e / (n * sb), rem = e - j * n * sb, k = rem / sb, ss = rem - k * sb;
    pts[((size_t)ss * n + k) * M + j] = O[((size_t)j * n + k) * S + s0 + ss];
  }
  double rj[M];
#pragma unroll
  for (int j = 0; j < M; ++j) rj[j] = ref[j];
  __syncthreads();
  for (int p = threadIdx.x; p < sb * n; p += 256) {
    const int ss = p / n, i = p - ss * n;
    const double* P = pts + (size_t)ss * n * M;
    double yi[M];
    bool better = true;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      yi[j] = P[i * M + j];
      better &= yi[j] > rj[j];
    }
    bool nd = better;
    // 8 points per step: their 8 x M LDS loads are in flight together (the early exit is
    // taken per step; the outcome equals the point-by-point scan's)
    constexpr int U = 8;
    for (int k0 = 0; k0 < n && nd; k0 += U) {
      double v[U][M];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < M; ++j) v[u][j] = (k0 + u < n) ? P[(k0 + u) * M + j] : 0.0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u;
        if (k >= n || k == i) continue;
        bool ge = true, gt = false, eq = true;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          ge &= v[u][j] >= yi[j];
          gt |= v[u][j] > yi[j];
          eq &= v[u][j] == yi[j];
        }
        if (ge && gt) nd = false;
        if (dedup && eq && k < i) nd = false;
      }
    }
    if (mask) mask[(size_t)(s0 + ss) * n + i] = nd ? 1 : 0;
    if (counts && nd) atomicAdd(&counts[i], 1);
  }
}

// The same test with an exact f32 pre-filter: rounding to f32 is monotone, so
// f32(v) < f32(y) in some objective proves v < y there and k can neither dominate nor
// duplicate i.  Only the (k, i) pairs that pass every objective in f32 (a dominator, a
// duplicate or a near-tie) are decided in f64 — f64 compares issue at a quarter of the f32
// rate and were the bound of pareto_lds_kernel.  LDS: the points as f64 [SB][n][M] for the
// exact test and as f32 [SB][M][npad] (objective-major, 8-aligned runs of k) for the filter.
template <int M>
__global__ __launch_bounds__(256) void pareto_f32_kernel(int S, int n, int npad, int SB, const double* __restrict__ O,
                                                         const double* __restrict__ ref, int dedup,
                                                         unsigned char* __restrict__ mask, int* __restrict__ counts) {
  extern __shared__ double pts[];   // [SB][n][M] f64, then [SB][M][npad] f32
  // the f32 copy starts on a 16-byte boundary (float4 loads): round the f64 region up to
  // an even number of doubles
  float* ptf = reinterpret_cast<float*>(pts + (((size_t)SB * n * M + 1) & ~(size_t)1));
  const int s0 = blockIdx.x * SB, sb = min(SB, S - s0);
  const int tot = M * n * sb;
  for (int e = threadIdx.x; e < tot; e += 256) {
    const int j = e / (n * sb), rem = e - j * n * sb, k = rem / sb, ss = rem - k * sb;
    const double v = O[((size_t)j * n + k) * S + s0 + ss];
    pts[((size_t)ss * n + k) * M + j] = v;
    ptf[((size_t)ss * M + j) * npad + k] = (float)v;
  }
  for (int e = threadIdx.x; e < sb * M * (npad - n); e += 256) {   // padding: never passes
    const int r = e / (npad - n), k = n + (e - r * (npad - n));
    ptf[(size_t)r * npad + k] = -INFINITY;
  }
  double rj[M];
#pragma unroll
  for (int j = 0; j < M; ++j) rj[j] = ref[j];
  __syncthreads();
  for (int p = threadIdx.x; p < sb * n; p += 256) {
    const int ss = p / n, i = p - ss * n;
    const double* P = pts + (size_t)ss * n * M;
    const float* F = ptf + (size_t)ss * M * npad;
    double yi[M];
    float yf[M];
    bool better = true;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      yi[j] = P[i * M + j];
      yf[j] = (float)yi[j];
      better &= yi[j] > rj[j];
    }
    bool nd = better;
    for (int k0 = 0; k0 < n && nd; k0 += 8) {
      float4 va[M], vb[M];
#pragma unroll
      for (int j = 0; j < M; ++j) {
        va[j] = *reinterpret_cast<const float4*>(F + (size_t)j * npad + k0);
        vb[j] = *reinterpret_cast<const float4*>(F + (size_t)j * npad + k0 + 4);
      }
      // candidate bits: every objective >= in f32.  Direct compares (not the sign of a
      // difference): f32 rounding is monotone, so v >= y in f64 implies f32(v) >= f32(y),
      // infinities included; a NaN fails the compare here and in the exact test alike.
      bool ge8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) ge8[u] = k0 + u != i && k0 + u < n;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        ge8[0] &= va[j].x >= yf[j]; ge8[1] &= va[j].y >= yf[j];
        ge8[2] &= va[j].z >= yf[j]; ge8[3] &= va[j].w >= yf[j];
        ge8[4] &= vb[j].x >= yf[j]; ge8[5] &= vb[j].y >= yf[j];
        ge8[6] &= vb[j].z >= yf[j]; ge8[7] &= vb[j].w >= yf[j];
      }
      unsigned int cand = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) cand |= (unsigned int)ge8[u] << u;
      while (cand) {
        const int u = __builtin_ctz(cand);
        cand &= cand - 1;
        const int k = k0 + u;
        bool ge = true, gt = false, eq = true;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const double v = P[k * M + j];
          ge &= v >= yi[j];
          gt |= v > yi[j];
          eq &= v == yi[j];
        }
        if ((ge && gt) || (dedup && eq && k < i)) {
          nd = false;
          cand = 0;
        }
      }
    }
    if (mask) mask[(size_t)(s0 + ss) * n + i] = nd ? 1 : 0;
    if (counts && nd) atomicAdd(&counts[i], 1);
  }
}

// -------------------------------------------------------------------------------------
// qEI (q = 1, one output): plain MC sampling f_s = mu + sigma z_s with psd_safe_cholesky
// (3 jitter tries) on the 1x1 posterior covariance; acq = mean_s (a f_s + b - best_f)_+.
// R = [Linv; alpha^T] K_x ((n+1) x b).  Also writes gR = d acq / d R for the backward.
// [upstream] qExpectedImprovement as built at bofire/strategies/predictives/sobo.py:51-90.
// -------------------------------------------------------------------------------------
__global__ void qei_kernel(int n, int b, int S, const double* __restrict__ R, double cc, double ym, double ys,
                           double kxx, const double* __restrict__ z, double oa, double ob, double best_f,
                           double* __restrict__ acq, double* __restrict__ gR, int* __restrict__ flags) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= b) return;
  double ss = 0.0;
  for (int i = 0; i < n; ++i) {
    const double v = R[(size_t)i * b + c];
    ss = fma(v, v, ss);
  }
  const double mu = ym + ys * (cc + R[(size_t)n * b + c]);
  const double var = ys * ys * (kxx - ss);
  double sd = nan("");
  int flag = 1;
  if (!isnan(var)) {
    for (int t = 0; t <= 3; ++t) {
      const double jit = (t == 0) ? 0.0 : 1e-8 * pow(10.0, (double)(t - 1));
      if (var + jit > 0.0) {
        sd = sqrt(var + jit);
        flag = 0;
        break;
      }
    }
  }
  double tot = 0.0, dmu = 0.0, dsd = 0.0;
  for (int s = 0; s < S; ++s) {
    const double imp = oa * (mu + sd * z[s]) + ob - best_f;
    if (imp > 0.0) {
      tot += imp;
      dmu += oa;
      dsd += oa * z[s];
    }
  }
  acq[c] = tot / S;
  flags[c] = flag;
  if (gR) {
    dmu /= S;
    dsd /= S;
    const double dvar = dsd / (2.0 * sd);
    const double dss = -ys * ys * dvar;
    for (int i = 0; i < n; ++i) gR[(size_t)i * b + c] = 2.0 * R[(size_t)i * b + c] * dss;
    gR[(size_t)n * b + c] = ys * dmu;
  }
}

__global__ void scale_batched_kernel(long long per, const double* __restrict__ alpha, double* __restrict__ X) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= per) return;
  X[(size_t)blockIdx.y * per + e] *= alpha[blockIdx.y];
}

// E[b][r][idx[r]] += val[b]  (adds the row-selection matrix P, scaled, to E: nb x n)
__global__ void add_selection_kernel(int nb, int n, const int* __restrict__ idx, const double* __restrict__ val,
                                     double* __restrict__ E) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nb) return;
  const int b = blockIdx.y;
  E[((size_t)b * nb + r) * n + idx[r]] += val ? val[b] : 1.0;
}

__global__ void objective_affine_kernel(int m, int n, int S, const double* __restrict__ Y, const double* __restrict__ mu,
                                        const double* __restrict__ a, const double* __restrict__ bb,
                                        double* __restrict__ O) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long tot = (long long)m * n * S;
  if (e >= tot) return;
  const int j = (int)(e / ((long long)n * S));
  const int i = (int)((e / S) % n);
  const double mv = mu ? mu[(size_t)j * n + i] : 0.0;
  O[e] = fma(a[j], Y[e] + mv, bb[j]);
}

}  // namespace evr

using namespace evr;

#define EVR_DISPATCH_M(m, MACRO)                                                      \
  switch (m) {                                                                        \
    case 1: MACRO(1); break;                                                          \
    case 2: MACRO(2); break;                                                          \
    case 3: MACRO(3); break;                                                          \
    case 4: MACRO(4); break;                                                          \
    case 5: MACRO(5); break;                                                          \
    case 6: MACRO(6); break;                                                          \
    case 7: MACRO(7); break;                                                          \
    case 8: MACRO(8); break;                                                          \
    default: EVR_CHECK(false, "number of objectives m=%d not supported (1..8)", m);   \
  }

extern "C" {

int evr_qnehvi_samples(void* stream, const evr_qnehvi_state* st, int b, const double* R, double* G, double* L22,
                       int* flags) {
  EVR_CHECK(st && st->m >= 1 && st->S >= 1 && st->n >= 1 && st->nb >= 0, "evr_qnehvi_samples: bad state");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (b <= 256) {  // small batches: 16 candidates x 16 row groups per block
    dim3 grid(cdiv(b, 16), st->m);
    qn_samples_kernel<16><<<grid, 256, 0, s>>>(st->n, st->nb, st->S, qn_nh(st), st->m, b, R, st->c, st->ym, st->ys, st->kxx,
                                               st->zq, st->obj_a, st->obj_b, G, L22, flags);
  } else {
    dim3 grid(cdiv(b, 64), st->m);
    qn_samples_kernel<64><<<grid, 256, 0, s>>>(st->n, st->nb, st->S, qn_nh(st), st->m, b, R, st->c, st->ym, st->ys, st->kxx,
                                               st->zq, st->obj_a, st->obj_b, G, L22, flags);
  }
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_mean_over_samples(void* stream, int S, int b, const double* partial, double* acq) {
  if (b == 0) return 0;
  mean_over_samples_kernel<<<cdiv(b, 256), 256, 0, (hipStream_t)stream>>>(S, b, partial, acq);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_qnehvi_samples_backward(void* stream, const evr_qnehvi_state* st, int b, const double* R, const double* L22,
                                const double* dG, double* gR) {
  EVR_CHECK(st && st->m >= 1, "evr_qnehvi_samples_backward: bad state");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (b <= 256) {
    dim3 grid(cdiv(b, 16), st->m);
    qn_samples_bwd_kernel<16><<<grid, 256, 0, s>>>(st->n, st->nb, st->S, qn_nh(st), st->m, b, R, st->ys, st->zq, st->obj_a,
                                                   L22, dG, gR);
  } else {
    dim3 grid(cdiv(b, 64), st->m);
    qn_samples_bwd_kernel<64><<<grid, 256, 0, s>>>(st->n, st->nb, st->S, qn_nh(st), st->m, b, R, st->ys, st->zq, st->obj_a,
                                                   L22, dG, gR);
  }
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_pareto_mask(void* stream, int S, int n, int m, const double* O, const double* ref, int dedup,
                    unsigned char* mask, int* counts) {
  EVR_CHECK(S >= 1 && n >= 0, "evr_pareto_mask: bad sizes");
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  constexpr size_t kLds = 96 * 1024;
  const size_t per = (size_t)n * m * sizeof(double);
  // f32 pre-filter variant: f64 + f32 copies of SB samples per block, SB chosen so that two
  // blocks fit a CU's LDS (the f64-only scan when they do not)
  constexpr int f32_filter = 1;
  const int npad = (n + 7) & ~7;
  const size_t per2 = (size_t)n * m * sizeof(double) + (size_t)npad * m * sizeof(float);
  constexpr size_t kLds2 = 78 * 1024;
  if (f32_filter && per2 <= kLds2) {
    const int SB = (int)std::min<size_t>(4, kLds2 / per2);
    const size_t bytes = (((size_t)SB * n * m + 1) & ~(size_t)1) * sizeof(double) + (size_t)SB * npad * m * sizeof(float);
#define L(MM)                                                                                            \
  do {                                                                                                   \
    EVR_HIP(hipFuncSetAttribute((const void*)pareto_f32_kernel<MM>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));                \
    pareto_f32_kernel<MM><<<cdiv(S, SB), 256, bytes, s>>>(S, n, npad, SB, O, ref, dedup, mask, counts);  \
  } while (0)
    EVR_DISPATCH_M(m, L);
#undef L
  } else if (per <= kLds) {   // samples staged in LDS, as many per block as fit (at most 4)
    const int SB = (int)std::min<size_t>(4, kLds / per);
    const size_t bytes = per * SB;
#define L(MM)                                                                                            \
  do {                                                                                                   \
    EVR_HIP(hipFuncSetAttribute((const void*)pareto_lds_kernel<MM>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));                \
    pareto_lds_kernel<MM><<<cdiv(S, SB), 256, bytes, s>>>(S, n, SB, O, ref, dedup, mask, counts);       \
  } while (0)
    EVR_DISPATCH_M(m, L);
#undef L
  } else {
    dim3 grid(cdiv(S, 64), n);
#define L(MM) pareto_kernel<MM><<<grid, 64, 0, s>>>(S, n, O, ref, dedup, mask, counts)
    EVR_DISPATCH_M(m, L);
#undef L
  }
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_qei(void* stream, int n, int b, int S, const double* R, double c, double ym, double ys, double kxx,
            const double* z, double obj_a, double obj_b, double best_f, double* acq, double* gR, int* flags) {
  EVR_CHECK(n >= 1 && S >= 1, "evr_qei: bad sizes");
  if (b == 0) return 0;
  qei_kernel<<<cdiv(b, 256), 256, 0, (hipStream_t)stream>>>(n, b, S, R, c, ym, ys, kxx, z, obj_a, obj_b, best_f,
                                                            acq, gR, flags);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_scale_batched(void* stream, int B, long long per, const double* alpha, double* X) {
  if (per == 0) return 0;
  dim3 grid(cdiv(per, 256), B);
  scale_batched_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(per, alpha, X);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_add_selection(void* stream, int B, int nb, int n, const int* idx, const double* val, double* E) {
  if (nb == 0) return 0;
  dim3 grid(cdiv(nb, 256), B);
  add_selection_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(nb, n, idx, val, E);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_objective_affine(void* stream, int m, int n, int S, const double* Y, const double* mu, const double* a,
                         const double* b, double* O) {
  const long long tot = (long long)m * n * S;
  if (tot == 0) return 0;
  objective_affine_kernel<<<cdiv(tot, 256), 256, 0, (hipStream_t)stream>>>(m, n, S, Y, mu, a, b, O);
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
