// General qNEHVI / qEHVI evaluation on gfx950: q >= 1 joint candidate batches, objectives
// over selected model outputs (affine Maximize / Minimize, or CloseToTarget) and
// sigmoid-weighted output constraints.
//
// Restates [upstream] BoTorch qExpectedHypervolumeImprovement._compute_qehvi (shared by
// qNoisyExpectedHypervolumeImprovement) for the calls BoFire makes with
//   q = candidate_count            (bofire/strategies/predictives/botorch.py:385),
//   objective = get_multiobjective_objective  (bofire/utils/torch_tools.py:699-727; the
//               per-output callables :384-402),
//   constraints / eta = get_output_constraints (torch_tools.py:258-381, passed at
//               bofire/strategies/predictives/qnehvi.py:28-48 and mobo.py:50-86):
//   acq = mean_s sum_{T subset of the q points, T != {}} (-1)^(|T|+1) prod_{i in T} w_si
//             * sum_cells prod_k clamp(min(u_k, min_{i in T} g_k(y_si)) - l_k, 0)
//   w_si = exp(sum_c logsigmoid(-c(y_si) / eta_c))   (compute_smoothed_feasibility_indicator)
// with the joint samples of the q points y_s = mu + L21 z_base,s + L22 z_new,s
// (sample_cached_cholesky; L22 = psd_safe_cholesky(Sigma_new - L21 L21^T), 6 jitter tries).
//
// MI355X layout: the q-subset minimum of the objectives is a "virtual candidate" of the q = 1
// scan, so the 2^q - 1 subsets of every candidate run through the same sparse kd / tiled HVI
// scan as q = 1 (hvi.hip, per-sample partials kept), and two small kernels apply the signed
// feasibility weights and route the gradient back to the arg-min point.  The q x q new-block
// Gram, jittered Cholesky and sampling run per (output, candidate) workgroup over the rows of
// R = M K_x that the q = 1 path already produces (qnehvi_proj.hip); the backward is the
// analytic Cholesky adjoint (Murray 2016: A_bar = sym(L^-T Phi(L^T L_bar) L^-1)) mixed back
// into the generated gR of the transposed projection GEMM.
#include <algorithm>
#include <cstring>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

size_t proj_forward_ws_doubles(const evr_qnehvi_state* st, int b);
int proj_forward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* Kx, double* R,
                 double* norms, double* W);
size_t kcross_grad_ws_doubles(int n1, int n2, int d);
int kcross_grad_launch(hipStream_t s, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                       const double* scale1, const double* X2, const double* shift2, const double* scale2,
                       const double* lengthscales, const double* outputscale, const double* G, double* dX2,
                       double* work);
int dg_gemm(hipStream_t s, bool tA, int M, int N, int K, double alpha, const double* A, int lda, long long sA,
            const double* B, int ldb, long long sB, double beta, double* Cm, int ldc, long long sC, int batch,
            double* W);
size_t dg_gemm_ws_doubles(bool tA, int M, int N, int K, int batch);
long long hvi_raw_workspace(const evr_qnehvi_state* st, int b, bool backward);
int hvi_raw(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, bool backward, double* work,
            double* dG, int* nsplit);

constexpr int QG_MAXM = 8, QG_MAXC = 16;

// objectives / constraints by value (kernel argument)
struct QgObj {
  int m, mo, nc;
  int oo[QG_MAXM], ok[QG_MAXM];
  double p0[QG_MAXM], p1[QG_MAXM];
  int co[QG_MAXC];
  double cs[QG_MAXC], ct[QG_MAXC], ce[QG_MAXC];
};

struct QgDims {
  int n, nb, nh, S, m, b;
};

__device__ __forceinline__ double qg_obj(const QgObj& o, int k, double y) {
  if (o.ok[k] == EVR_OBJ_AFFINE) return fma(o.p0[k], y, o.p1[k]);
  return -pow(fabs(y - o.p0[k]), o.p1[k]);   // CloseToTarget: -|y - t|^e
}

__device__ __forceinline__ double qg_dobj(const QgObj& o, int k, double y) {
  if (o.ok[k] == EVR_OBJ_AFFINE) return o.p0[k];
  const double u = y - o.p0[k], e = o.p1[k];
  if (u == 0.0) return 0.0;                  // torch: sign(0) = 0 in abs' backward
  return -e * pow(fabs(u), e - 1.0) * (u > 0.0 ? 1.0 : -1.0);
}

// log-sigmoid, stable: min(x, 0) - log1p(exp(-|x|))
__device__ __forceinline__ double qg_logsig(double x) { return fmin(x, 0.0) - log1p(exp(-fabs(x))); }
__device__ __forceinline__ double qg_sig(double x) {
  return x >= 0.0 ? 1.0 / (1.0 + exp(-x)) : exp(x) / (1.0 + exp(x));
}

// [upstream] botorch.utils.safe_math.log_fatmoid — the fat-tailed (Cauchy, O(1/x^2) for
// x -> -inf) smooth Heaviside that compute_smoothed_feasibility_indicator(log=True, fat=True)
// uses in qLogNEHVI / qLogEHVI:  fatmoid(x) = 2/3 cauchy(x - m) for x < 0,
// 1 - 2/3 cauchy(x + m) otherwise, cauchy(x) = 1 / (1 + x^2), m = sqrt(1/3) (continuous, = 1/2
// at 0).  Log evaluated without cancellation on both branches; qg_dlog_fatmoid is its slope.
constexpr double QG_FATMOID_M = 0.57735026918962576;
__device__ __forceinline__ double qg_log_fatmoid(double x) {
  if (x < 0.0) {
    const double u = x - QG_FATMOID_M;
    return -0.40546510810816438 - log1p(u * u);   // log(2/3) - log(1 + u^2)
  }
  const double u = x + QG_FATMOID_M;
  return log1p(-(2.0 / 3.0) / (1.0 + u * u));
}
__device__ __forceinline__ double qg_dlog_fatmoid(double x) {
  if (x < 0.0) {
    const double u = x - QG_FATMOID_M;
    return -2.0 * u / (1.0 + u * u);
  }
  const double u = x + QG_FATMOID_M, w = 1.0 + u * u, c = (2.0 / 3.0) / w;
  return 2.0 * u * c / (w * (1.0 - c));
}

// fixed-order block sum over 256 threads (4 waves): xor-butterfly in the wave, then waves 0..3
__device__ __forceinline__ double qg_block_sum(double v, double* red4) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red4[wave] = v;
  __syncthreads();
  return ((red4[0] + red4[1]) + red4[2]) + red4[3];
}

// ---------------------------------------------------------------------------------------
// Gram of the q new points, jittered Cholesky of Sigma_new - L21 L21^T, joint samples.
// Workgroup (candidate c, output j), 256 threads over the R rows, then over the samples.
//   Sigma22[i][i'] = s^2 (k(x_i, x_i') - sum_{r<n} R_ri R_ri') - sum_{n<=r<n+nb} R_ri R_ri'
// (rows < n: L^-1 k or the fused root C k; rows [n, n+nb): L21 = G k of the split layout).
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(256) void qg_gram_samples(QgDims dm, int kind, int d, const double* __restrict__ R,
                                                       const double* __restrict__ X, const double* __restrict__ ls,
                                                       const double* __restrict__ shift,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ cc, const double* __restrict__ ym,
                                                       const double* __restrict__ ys, const double* __restrict__ kxx,
                                                       const double* __restrict__ zq, double* __restrict__ Y,
                                                       double* __restrict__ Lq, int* __restrict__ flags) {
  constexpr int NP = Q * (Q + 1) / 2;
  __shared__ double red4[4];
  __shared__ double Ls[Q * Q];
  __shared__ double mus[Q];
  const int c = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
  const int n = dm.n, nb = dm.nb, nh = dm.nh, m = dm.m;
  const int bq = dm.b * Q;
  const long long Rr = (long long)n + nb + nh + 1;
  const double* Rj = R + (size_t)j * Rr * bq + (size_t)c * Q;
  const double s = ys[j], s2 = s * s;
  double acc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = 0.0;
  for (int r = tid; r < n + nb; r += 256) {
    const double w = r < n ? s2 : 1.0;
    double v[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) v[i] = Rj[(size_t)r * bq + i];
    int p = 0;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 <= i; ++i2) acc[p++] += w * v[i] * v[i2];
  }
  double gram[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) gram[p] = qg_block_sum(acc[p], red4);
  if (tid == 0) {
    const double* lsj = ls + (size_t)j * d;
    double A[Q][Q];
    int p = 0;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 <= i; ++i2) {
        double kq = kxx[j];
        if (i2 != i) {
          double d2 = 0.0;
          const double* xa = X + ((size_t)c * Q + i) * d;
          const double* xb = X + ((size_t)c * Q + i2) * d;
          for (int t = 0; t < d; ++t) {
            const double sc = scale ? scale[t] : 1.0, sh = shift ? shift[t] : 0.0;
            const double u = ((xa[t] - sh) * sc - (xb[t] - sh) * sc) / lsj[t];
            d2 = fma(u, u, d2);
          }
          kq = kxx[j] * kernel_value(kind_of(kind, j), d2);
        }
        A[i][i2] = s2 * kq - gram[p++];
      }
    // psd_safe_cholesky: plain, then total diagonal jitter 1e-8 * 10^(t-1), t = 1..6
    double L[Q][Q];
    int flag = 1;
    bool nan_in = false;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 <= i; ++i2) nan_in |= isnan(A[i][i2]);
    for (int t = 0; t <= 6 && flag && !nan_in; ++t) {
      const double jit = (t == 0) ? 0.0 : 1e-8 * pow(10.0, (double)(t - 1));
      bool ok = true;
#pragma unroll
      for (int i = 0; i < Q; ++i) {
#pragma unroll
        for (int i2 = 0; i2 <= i; ++i2) {
          double v = A[i][i2] + (i == i2 ? jit : 0.0);
#pragma unroll
          for (int k = 0; k < i2; ++k) v -= L[i][k] * L[i2][k];
          if (i == i2) {
            if (!(v > 0.0)) ok = false;
            L[i][i] = ok ? sqrt(v) : 1.0;
          } else {
            L[i][i2] = v / L[i2][i2];
          }
        }
      }
      if (ok) flag = 0;
    }
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 < Q; ++i2) {
        const double v = flag ? nan("") : (i2 <= i ? L[i][i2] : 0.0);
        Ls[i * Q + i2] = v;
        Lq[((size_t)j * dm.b + c) * Q * Q + i * Q + i2] = v;
      }
    flags[(size_t)j * dm.b + c] = flag;
#pragma unroll
    for (int i = 0; i < Q; ++i) mus[i] = ym[j] + s * (cc[j] + Rj[(size_t)(Rr - 1) * bq + i]);
  }
  __syncthreads();
  for (int si = tid; si < dm.S; si += 256) {
    double z[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) z[i] = zq[((size_t)si * Q + i) * m + j];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      double y = mus[i] + (nh ? Rj[(size_t)(n + nb + si) * bq + i] : 0.0);
#pragma unroll
      for (int i2 = 0; i2 <= i; ++i2) y = fma(Ls[i * Q + i2], z[i2], y);
      Y[((size_t)si * m + j) * bq + (size_t)c * Q + i] = y;
    }
  }
}

// per point: objectives g_k and the feasibility weight w (sum of log-sigmoids, exp)
__device__ __forceinline__ void qg_point(const QgObj& o, const double* __restrict__ Ys, size_t stride, double* g,
                                         double& w) {
  for (int k = 0; k < o.mo; ++k) g[k] = qg_obj(o, k, Ys[(size_t)o.oo[k] * stride]);
  double lw = 0.0;
  for (int t = 0; t < o.nc; ++t) {
    const double cval = o.cs[t] * (Ys[(size_t)o.co[t] * stride] - o.ct[t]);
    lw += qg_logsig(-cval / o.ce[t]);
  }
  w = o.nc ? exp(lw) : 1.0;
}

// ---------------------------------------------------------------------------------------
// virtual candidates: thread per (candidate c, sample s); subset T (bit mask 1 .. 2^q - 1)
// -> Gv[s][k][c*nsub + T-1] = min_{i in T} g_k(y_si), Wv[s][c*nsub + T-1] = (-1)^(|T|+1) prod w_si
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(64) void qg_subsets(int S, int b, QgObj o, const double* __restrict__ Y,
                                                 double* __restrict__ Gv, double* __restrict__ Wv) {
  constexpr int NSUB = (1 << Q) - 1;
  const int c = blockIdx.x * 64 + threadIdx.x, s = blockIdx.y;
  if (c >= b) return;
  const size_t bq = (size_t)b * Q, bv = (size_t)b * NSUB;
  double g[Q][QG_MAXM], w[Q];
#pragma unroll
  for (int i = 0; i < Q; ++i) qg_point(o, Y + (size_t)s * o.m * bq + (size_t)c * Q + i, bq, g[i], w[i]);
  for (int T = 1; T <= NSUB; ++T) {
    const size_t col = (size_t)c * NSUB + (T - 1);
    double W = (__builtin_popcount(T) & 1) ? 1.0 : -1.0;
#pragma unroll
    for (int i = 0; i < Q; ++i)
      if (T >> i & 1) W *= w[i];
    Wv[(size_t)s * bv + col] = W;
    for (int k = 0; k < o.mo; ++k) {
      double z = INFINITY;
#pragma unroll
      for (int i = 0; i < Q; ++i)
        if (T >> i & 1) z = fmin(z, g[i][k]);
      Gv[((size_t)s * o.mo + k) * bv + col] = z;
    }
  }
}

// acq[c] = (1/S) sum_s sum_T Wv * HVI_T,s (per-split partials summed in order); NaN on flags
__global__ __launch_bounds__(256) void qg_combine_fwd(int S, int ns, int nsub, int b, int m,
                                                      const double* __restrict__ part, const double* __restrict__ Wv,
                                                      const int* __restrict__ flags, double* __restrict__ acq) {
  __shared__ double red4[4];
  const int c = blockIdx.x;
  const size_t bv = (size_t)b * nsub;
  double acc = 0.0;
  for (int e = threadIdx.x; e < S * nsub; e += 256) {
    const int s = e / nsub, T = e - s * nsub;
    const size_t col = (size_t)c * nsub + T;
    double h = 0.0;
    for (int k = 0; k < ns; ++k) h += part[((size_t)s * ns + k) * bv + col];
    acc = fma(Wv[(size_t)s * bv + col], h, acc);
  }
  const double tot = qg_block_sum(acc, red4);
  if (threadIdx.x == 0) {
    bool bad = false;
    for (int j = 0; j < m; ++j) bad |= flags[(size_t)j * b + c] != 0;
    acq[c] = bad ? nan("") : tot / (double)S;
  }
}

// ---------------------------------------------------------------------------------------
// backward of the subset / weight step: thread per (candidate c, sample s) ->
// dY[s][j][c*q + i] = d(gout_c * acq_c)/dy_sij.  dGv = d(sum_s HVI_s)/dGv / S (gout 1).
// The min's gradient goes to the first arg-min point of the subset (torch.min).
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(64) void qg_subsets_bwd(int S, int b, int ns, QgObj o, const double* __restrict__ Y,
                                                     const double* __restrict__ Wv, const double* __restrict__ dGv,
                                                     const double* __restrict__ part,
                                                     const double* __restrict__ gout, double* __restrict__ dY) {
  constexpr int NSUB = (1 << Q) - 1;
  const int c = blockIdx.x * 64 + threadIdx.x, s = blockIdx.y;
  if (c >= b) return;
  const size_t bq = (size_t)b * Q, bv = (size_t)b * NSUB;
  const double* Ys = Y + (size_t)s * o.m * bq + (size_t)c * Q;
  double g[Q][QG_MAXM], w[Q], dg[Q][QG_MAXM], dw[Q];
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    qg_point(o, Ys + i, bq, g[i], w[i]);
    dw[i] = 0.0;
    for (int k = 0; k < QG_MAXM; ++k) dg[i][k] = 0.0;
  }
  const double gc = gout ? gout[c] : 1.0;
  for (int T = 1; T <= NSUB; ++T) {
    const size_t col = (size_t)c * NSUB + (T - 1);
    const double W = Wv[(size_t)s * bv + col] * gc;
    for (int k = 0; k < o.mo; ++k) {
      const double dz = dGv[((size_t)s * o.mo + k) * bv + col];
      if (dz == 0.0) continue;
      int am = -1;
      double z = INFINITY;
#pragma unroll
      for (int i = 0; i < Q; ++i)
        if ((T >> i & 1) && (am < 0 || g[i][k] < z)) {
          am = i;
          z = g[i][k];
        }
#pragma unroll
      for (int i = 0; i < Q; ++i)
        if (i == am) dg[i][k] += W * dz;
    }
    if (o.nc) {
      double h = 0.0;
      for (int k = 0; k < ns; ++k) h += part[((size_t)s * ns + k) * bv + col];
      const double dWT = ((__builtin_popcount(T) & 1) ? 1.0 : -1.0) * gc * h / (double)S;
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        if (!(T >> i & 1)) continue;
        double pr = dWT;
#pragma unroll
        for (int i2 = 0; i2 < Q; ++i2)
          if (i2 != i && (T >> i2 & 1)) pr *= w[i2];
        dw[i] += pr;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    double dy[QG_MAXM];
    for (int jj = 0; jj < QG_MAXM; ++jj) dy[jj] = 0.0;
    for (int k = 0; k < o.mo; ++k) {
      const int jj = o.oo[k];
      dy[jj] += dg[i][k] * qg_dobj(o, k, Ys[(size_t)jj * bq + i]);
    }
    for (int t = 0; t < o.nc; ++t) {
      const int jj = o.co[t];
      const double cval = o.cs[t] * (Ys[(size_t)jj * bq + i] - o.ct[t]);
      // d w / d c_t = w * sigmoid(c_t / eta_t) * (-1 / eta_t)
      dy[jj] += dw[i] * w[i] * qg_sig(cval / o.ce[t]) * (-1.0 / o.ce[t]) * o.cs[t];
    }
    for (int jj = 0; jj < o.m; ++jj) dY[((size_t)s * o.m + jj) * bq + (size_t)c * Q + i] = dy[jj];
  }
}

// ---------------------------------------------------------------------------------------
// backward of the joint sampling: workgroup (candidate c, output j).
//   dmu_i = sum_s dY_si, dL_ii' = sum_s dY_si z_si' (i' <= i), A_bar = sym(L^-T Phi(L^T dL) L^-1)
//   cf[j][c] = -2 A_bar (gR rows < n scale it by s^2), dKqq[j][c] = s^2 A_bar, cm = s dmu.
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(256) void qg_samples_bwd(QgDims dm, const double* __restrict__ dY,
                                                      const double* __restrict__ zq, const double* __restrict__ Lq,
                                                      const double* __restrict__ ys, double* __restrict__ cf,
                                                      double* __restrict__ dKqq, double* __restrict__ cm) {
  constexpr int NP = Q * (Q + 1) / 2;
  __shared__ double red4[4];
  const int c = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
  const int m = dm.m, bq = dm.b * Q;
  double amu[Q], adl[NP];
#pragma unroll
  for (int i = 0; i < Q; ++i) amu[i] = 0.0;
#pragma unroll
  for (int p = 0; p < NP; ++p) adl[p] = 0.0;
  for (int si = tid; si < dm.S; si += 256) {
    double dy[Q], z[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      dy[i] = dY[((size_t)si * m + j) * bq + (size_t)c * Q + i];
      z[i] = zq[((size_t)si * Q + i) * m + j];
      amu[i] += dy[i];
    }
    int p = 0;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 <= i; ++i2, ++p) adl[p] = fma(dy[i], z[i2], adl[p]);
  }
  double dmu[Q], dl[NP];
#pragma unroll
  for (int i = 0; i < Q; ++i) dmu[i] = qg_block_sum(amu[i], red4);
#pragma unroll
  for (int p = 0; p < NP; ++p) dl[p] = qg_block_sum(adl[p], red4);
  if (tid != 0) return;
  const double s = ys[j];
  const double* L = Lq + ((size_t)j * dm.b + c) * Q * Q;
  double Lb[Q][Q], P[Q][Q], X[Q][Q], Ab[Q][Q];
  {
    int p = 0;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 < Q; ++i2) Lb[i][i2] = 0.0;
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int i2 = 0; i2 <= i; ++i2) Lb[i][i2] = dl[p++];
  }
  // P = Phi(L^T Lb): lower triangle, halved diagonal
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int i2 = 0; i2 < Q; ++i2) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < Q; ++k) v = fma(L[k * Q + i], Lb[k][i2], v);
      P[i][i2] = i2 < i ? v : (i2 == i ? 0.5 * v : 0.0);
    }
  // X = L^-T P  (solve L^T X = P, L^T upper: back substitution over rows)
#pragma unroll
  for (int col = 0; col < Q; ++col)
#pragma unroll
    for (int i = Q - 1; i >= 0; --i) {
      double v = P[i][col];
#pragma unroll
      for (int k = i + 1; k < Q; ++k) v -= L[k * Q + i] * X[k][col];
      X[i][col] = v / L[i * Q + i];
    }
  // Ab = X L^-1  (solve Ab L = X: columns from the right)
#pragma unroll
  for (int row = 0; row < Q; ++row)
#pragma unroll
    for (int i = Q - 1; i >= 0; --i) {
      double v = X[row][i];
#pragma unroll
      for (int k = i + 1; k < Q; ++k) v -= Ab[row][k] * L[k * Q + i];
      Ab[row][i] = v / L[i * Q + i];
    }
  double* cfj = cf + ((size_t)j * dm.b + c) * Q * Q;
  double* dkj = dKqq + ((size_t)j * dm.b + c) * Q * Q;
#pragma unroll
  for (int i = 0; i < Q; ++i)
#pragma unroll
    for (int i2 = 0; i2 < Q; ++i2) {
      const double a = 0.5 * (Ab[i][i2] + Ab[i2][i]);
      cfj[i * Q + i2] = -2.0 * a;
      dkj[i * Q + i2] = s * s * a;
    }
#pragma unroll
  for (int i = 0; i < Q; ++i) cm[(size_t)j * bq + (size_t)c * Q + i] = s * dmu[i];
}

// gR_j (Rr x bq): rows < n: s^2 sum_i' cf[i][i'] R[row][c q + i'], rows [n, n+nb): without s^2,
// sample rows: dY, mean row: cm
template <int Q>
__global__ __launch_bounds__(256) void qg_gen_gr(QgDims dm, const double* __restrict__ R, const double* __restrict__ dY,
                                                 const double* __restrict__ cf, const double* __restrict__ cm,
                                                 const double* __restrict__ ys, double* __restrict__ gR) {
  const int bq = dm.b * Q;
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col >= bq) return;
  const int Rr = dm.n + dm.nb + dm.nh + 1;
  const int rj = blockIdx.x;
  const int j = rj / Rr, row = rj - j * Rr;
  const int c = col / Q, i = col - c * Q;
  const size_t base = (size_t)rj * bq;
  double v;
  if (row < dm.n + dm.nb) {
    const double* cfr = cf + ((size_t)j * dm.b + c) * Q * Q + i * Q;
    const double* Rr0 = R + base + (size_t)c * Q;
    v = 0.0;
#pragma unroll
    for (int i2 = 0; i2 < Q; ++i2) v = fma(cfr[i2], Rr0[i2], v);
    if (row < dm.n) v *= ys[j] * ys[j];
  } else if (row < dm.n + dm.nb + dm.nh) {
    v = dY[((size_t)(row - dm.n - dm.nb) * dm.m + j) * bq + col];
  } else {
    v = cm[(size_t)j * bq + col];
  }
  gR[base + col] = v;
}

// dX[c q + i] += sum_j sum_{i' != i} 2 dKqq[j][c][i][i'] dk_j(x_i, x_i')/dx_i (raw coordinates)
template <int Q>
__global__ __launch_bounds__(64) void qg_kqq_grad(int b, int m, int d, int kind, const double* __restrict__ X,
                                                  const double* __restrict__ ls, const double* __restrict__ shift,
                                                  const double* __restrict__ scale, const double* __restrict__ kxx,
                                                  const double* __restrict__ dKqq, double* __restrict__ dX) {
  const int col = blockIdx.x * 64 + threadIdx.x;
  if (col >= b * Q) return;
  const int c = col / Q, i = col - c * Q;
  const double* xa = X + (size_t)col * d;
  double* out = dX + (size_t)col * d;
  for (int j = 0; j < m; ++j) {
    const double* lsj = ls + (size_t)j * d;
    for (int i2 = 0; i2 < Q; ++i2) {
      if (i2 == i) continue;
      const double coef = 2.0 * dKqq[((size_t)j * b + c) * Q * Q + i * Q + i2];
      if (coef == 0.0) continue;
      const double* xb = X + ((size_t)c * Q + i2) * d;
      double d2 = 0.0;
      for (int t = 0; t < d; ++t) {
        const double sc = scale ? scale[t] : 1.0;
        const double u = (xa[t] - xb[t]) * sc / lsj[t];
        d2 = fma(u, u, d2);
      }
      const double ks = coef * kxx[j] * kernel_dscale(kind_of(kind, j), d2);
      for (int t = 0; t < d; ++t) {
        const double sc = scale ? scale[t] : 1.0;
        out[t] += ks * (xa[t] - xb[t]) * sc * sc / (lsj[t] * lsj[t]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// objectives of baseline / prune samples with hard feasibility:
//   O[k][i][s] = g_k(Y[.][i][s] + mu[.][i]), and = ref_k where any constraint c > 0
// ([upstream] prune_inferior_points_multi_objective / _set_cell_bounds: infeasible samples
// are excluded from the Pareto sets by setting them to the reference point)
// ---------------------------------------------------------------------------------------
__global__ void qg_objective_kernel(int n, int S, QgObj o, const double* __restrict__ Y, const double* __restrict__ mu,
                                    const double* __restrict__ ref, double* __restrict__ O) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)n * S) return;
  const int i = (int)(e / S), s = (int)(e % S);
  auto y = [&](int j) { return Y[((size_t)j * n + i) * S + s] + (mu ? mu[(size_t)j * n + i] : 0.0); };
  bool feas = true;
  for (int t = 0; t < o.nc; ++t) feas &= !(o.cs[t] * (y(o.co[t]) - o.ct[t]) > 0.0);
  for (int k = 0; k < o.mo; ++k) O[((size_t)k * n + i) * S + s] = feas ? qg_obj(o, k, y(o.oo[k])) : ref[k];
}

// ---------------------------------------------------------------------------------------
// objective values and smoothed feasibility weights of model-output rows, through the same
// per-point function (qg_point) the general scan applies to every sample: G[k][i] = g_k(y_i),
// W[i] = exp(sum_c logsigmoid(-c(y_i) / eta_c)).  Y: m_model x n (output-major).
// ---------------------------------------------------------------------------------------
__global__ void qg_weights_kernel(int n, QgObj o, const double* __restrict__ Y, double* __restrict__ G,
                                  double* __restrict__ W) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double g[QG_MAXM], w;
  qg_point(o, Y + i, (size_t)n, g, w);
  for (int k = 0; k < o.mo; ++k) G[(size_t)k * n + i] = g[k];
  W[i] = w;
}

static int qg_params(const evr_qn_general* g, int m_model, QgObj* o) {
  EVR_CHECK(g && g->m_obj >= 1 && g->m_obj <= QG_MAXM && g->n_con >= 0 && g->n_con <= QG_MAXC && m_model >= 1 &&
                m_model <= QG_MAXM && g->obj_out && g->obj_kind && g->obj_p0 && g->obj_p1 &&
                (g->n_con == 0 || (g->con_out && g->con_sign && g->con_thr && g->con_eta)),
            "qnehvi_general: bad objective / constraint description (m_obj 1..%d, n_con 0..%d, outputs 1..%d)",
            QG_MAXM, QG_MAXC, QG_MAXM);
  std::memset(o, 0, sizeof(*o));
  o->m = m_model;
  o->mo = g->m_obj;
  o->nc = g->n_con;
  for (int k = 0; k < g->m_obj; ++k) {
    EVR_CHECK(g->obj_out[k] >= 0 && g->obj_out[k] < m_model, "qnehvi_general: objective %d reads output %d of %d", k,
              g->obj_out[k], m_model);
    EVR_CHECK(g->obj_kind[k] == EVR_OBJ_AFFINE || g->obj_kind[k] == EVR_OBJ_CLOSE_TO_TARGET,
              "qnehvi_general: objective kind %d", g->obj_kind[k]);
    o->oo[k] = g->obj_out[k];
    o->ok[k] = g->obj_kind[k];
    o->p0[k] = g->obj_p0[k];
    o->p1[k] = g->obj_p1[k];
  }
  for (int t = 0; t < g->n_con; ++t) {
    EVR_CHECK(g->con_out[t] >= 0 && g->con_out[t] < m_model && g->con_eta[t] > 0.0,
              "qnehvi_general: constraint %d (output %d, eta %g)", t, g->con_out[t], g->con_eta[t]);
    o->co[t] = g->con_out[t];
    o->cs[t] = g->con_sign[t];
    o->ct[t] = g->con_thr[t];
    o->ce[t] = g->con_eta[t];
  }
  return 0;
}

struct QgLayout {
  size_t Kx, R, P, Wf, Y, Lq, flags, Gv, Wv, hvi, dGv, dY, cf, dKqq, cm, gR, dKx, Wb, kg, total;
};

static QgLayout qg_layout(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, int q, int d, int b,
                          bool backward) {
  QgLayout L{};
  const size_t m = stm->m, n = stm->n, S = stm->S, bq = (size_t)b * q, nsub = ((size_t)1 << q) - 1;
  const size_t bv = (size_t)b * nsub, Rr = (size_t)qn_rows(stm), mo = sth->m;
  size_t o = 0;
  auto take = [&](size_t doubles) {
    const size_t r = o;
    o += (doubles + 31) & ~(size_t)31;
    return r;
  };
  L.Kx = take(m * n * bq);
  L.R = take(m * Rr * bq);
  L.P = take(m * (size_t)evr_qnehvi_norms_rows(stm) * 2 * bq);
  L.Wf = take(proj_forward_ws_doubles(stm, (int)bq));
  L.Y = take(S * m * bq);
  L.Lq = take(m * b * q * q);
  L.flags = take((m * b + 1) / 2);
  L.Gv = take(S * mo * bv);
  L.Wv = take(S * bv);
  L.hvi = take((size_t)hvi_raw_workspace(sth, (int)bv, backward));
  if (backward) {
    L.dGv = take(S * mo * bv);
    L.dY = take(S * m * bq);
    L.cf = take(m * b * q * q);
    L.dKqq = take(m * b * q * q);
    L.cm = take(m * bq);
    L.gR = take(m * Rr * bq);
    L.dKx = take(m * n * bq);
    L.Wb = take(dg_gemm_ws_doubles(true, (int)n, (int)bq, (int)Rr, (int)m));   // split-K partials of M^T gR
    L.kg = take(kcross_grad_ws_doubles((int)n, (int)bq, d));
  }
  L.total = o;
  return L;
}

static int qg_check(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                    const evr_qnehvi_model* md) {
  EVR_CHECK(stm && sth && g && md, "qnehvi_general: null argument");
  EVR_CHECK(g->q >= 1 && g->q <= EVR_QNG_MAX_Q, "qnehvi_general: q = %d outside 1..%d", g->q, EVR_QNG_MAX_Q);
  EVR_CHECK(sth->m == g->m_obj && sth->S == stm->S && !sth->log_hvi,
            "qnehvi_general: scan state must carry m = m_obj objectives, the same S, and log_hvi = 0");
  EVR_CHECK(md->n == stm->n && md->d >= 1 && md->M && md->Xn && md->lengthscales && g->zq && stm->c && stm->ym &&
                stm->ys && stm->kxx,
            "qnehvi_general: inconsistent model / state");
  return 0;
}

// ---------------------------------------------------------------------------------------
// Log-space general scan: [upstream] qLogExpectedHypervolumeImprovement._compute_log_qehvi
// (fat = True; shared by qLogNoisyExpectedHypervolumeImprovement) for q-point candidates,
// objectives over selected outputs and output constraints — MoboStrategy's default
// acquisition (bofire/strategies/predictives/mobo.py:47-90).  Per MC sample s, candidate c,
// explicit cell [l, u] of the sample's partition and q-subset T:
//   a_ik   = log fatplus(g_k(y_i) - l_k; tau_relu)
//   z_k(T) = fatmin_{i in T} a_ik                       (tau_max)
//   A(T)   = sum_k fatmin(z_k(T), log(min(u_k, 1e10) - l_k)) + sum_{i in T} lf_i
//   cell   = logdiffexp(logsumexp_{|T| odd} A(T), logsumexp_{|T| even} A(T))
//   LSE_sc = logsumexp_cells cell,   acq_c = logmeanexp_s LSE_sc
// lf_i = sum_t log_fatmoid(-c_t(y_i) / eta_t) (log feasibility, fat = True).  A workgroup owns (sample,
// CT candidates, range of cells); the cells are staged through LDS with their log lengths;
// each thread keeps an online log-sum-exp over its cells with Q (m_obj + 1) gradient slots
// (d / d g_ik and d / d lf_i), merged over the thread groups and splits in a fixed order.
// The backward walks the subsets a second time with the cell's final odd / even sums:
// d cell / d A(T) = +-exp(A(T) - cell).
// ---------------------------------------------------------------------------------------
constexpr int QL_THREADS = 256, QL_CHUNK = 128;

// fat-min over the members of subset T of x[0..Q) and its partials (members only)
template <int Q>
__device__ __forceinline__ double ql_fatmin_set(unsigned T, const double* x, double t, double* dz) {
  double xmin = INFINITY;
  int am = 0;
#pragma unroll
  for (int i = 0; i < Q; ++i)
    if ((T >> i & 1) && x[i] < xmin) {
      xmin = x[i];
      am = i;
    }
  if (!(T & (T - 1))) {   // a single point: exactly x
    if (dz)
#pragma unroll
      for (int i = 0; i < Q; ++i) dz[i] = (int)i == am ? 1.0 : 0.0;
    return xmin;
  }
  double S = 0.0, sp = 0.0;
  double pp[Q];
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    pp[i] = 0.0;
    if (T >> i & 1) {
      const double u = (x[i] - xmin) / t;
      const double p = 2.0 / (2.0 + u * (2.0 + u));
      S += p;
      pp[i] = (1.0 + u) * p * p;   // -pareto'(u)
      if (i != am) sp += pp[i];
    }
  }
  if (dz) {
#pragma unroll
    for (int i = 0; i < Q; ++i) dz[i] = (T >> i & 1) ? (i == am ? 1.0 - sp / S : pp[i] / S) : 0.0;
  }
  return xmin - t * log(S);
}

template <int MM, int Q, bool BWD>
__global__ __launch_bounds__(QL_THREADS) void qlog_scan(int b, int nsplit, int CT, int CB, QgObj o,
                                                        const double* __restrict__ Y,
                                                        const int* __restrict__ off, const double* __restrict__ lo,
                                                        const double* __restrict__ hi, double tr, double tm,
                                                        double* __restrict__ out) {
  constexpr int NG = Q * (MM + 1);
  constexpr int NO = 2 + (BWD ? NG : 0);
  constexpr unsigned NSUB = (1u << Q) - 1u;
  __shared__ double Ls[QL_CHUNK][MM];
  __shared__ double Ws[QL_CHUNK][MM];
  __shared__ double red[QL_THREADS / 2][NO];   // tree merge of the thread groups (GR a power of two)
  const int s = blockIdx.y, split = blockIdx.z, tid = threadIdx.x;
  const int mo = o.mo, bq = b * Q;
  const int GR = QL_THREADS / CT;
  const int cl = tid % CT, g = tid / CT;
  const int c = blockIdx.x * CT + cl;
  // this thread's candidate: objectives and log feasibility of its Q points
  double gv[Q][MM], lf[Q];
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    lf[i] = 0.0;
#pragma unroll
    for (int k = 0; k < MM; ++k) gv[i][k] = 0.0;
    if (c < b) {
      double gg[QG_MAXM], w;
      qg_point(o, Y + (size_t)s * o.m * bq + (size_t)c * Q + i, (size_t)bq, gg, w);
      double l = 0.0;
      for (int t = 0; t < o.nc; ++t) {
        const double cval = o.cs[t] * (Y[((size_t)s * o.m + o.co[t]) * bq + (size_t)c * Q + i] - o.ct[t]);
        l += qg_log_fatmoid(-cval / o.ce[t]);   // fat = True (qLog*)
      }
      lf[i] = l;
#pragma unroll
      for (int k = 0; k < MM; ++k) gv[i][k] = k < mo ? gg[k] : 0.0;
    }
  }
  LseState<NG, BWD> st;
  st.init();
  const int k0 = off[s] + split * CB;
  const int k1 = min(off[s + 1], k0 + CB);
  for (int ks = k0; ks < k1; ks += QL_CHUNK) {
    const int nc = min(QL_CHUNK, k1 - ks);
    __syncthreads();
    for (int e = tid; e < nc * mo; e += QL_THREADS) {
      const int cell = e / mo, j = e - cell * mo;
      const double l = lo[(size_t)ks * mo + e];
      const double u = fmin(hi[(size_t)ks * mo + e], HL_UMAX);
      Ls[cell][j] = l;
      Ws[cell][j] = log(u - l);
    }
    __syncthreads();
    if (c >= b) continue;
    for (int kc = g; kc < nc; kc += GR) {
      double a[Q][MM], da[Q][MM];
#pragma unroll
      for (int i = 0; i < Q; ++i)
#pragma unroll
        for (int k = 0; k < MM; ++k) {
          a[i][k] = 0.0;
          da[i][k] = 0.0;
          if (k < mo) a[i][k] = log_fatplus(gv[i][k] - Ls[kc][k], tr, BWD ? &da[i][k] : nullptr);
        }
      // forward: online log-sum-exp of the odd / even subsets
      double mp = -INFINITY, sp = 0.0, mn = -INFINITY, sn = 0.0;
      for (unsigned T = 1; T <= NSUB; ++T) {
        double A = 0.0;
#pragma unroll
        for (int k = 0; k < MM; ++k) {
          if (k >= mo) continue;
          double xk[Q];
#pragma unroll
          for (int i = 0; i < Q; ++i) xk[i] = a[i][k];
          const double z = ql_fatmin_set<Q>(T, xk, tm, nullptr);
          A += fatmin2(z, Ws[kc][k], tm, nullptr);
        }
#pragma unroll
        for (int i = 0; i < Q; ++i)
          if (T >> i & 1) A += lf[i];
        if (A == -INFINITY) continue;
        double& m_ = (__builtin_popcount(T) & 1) ? mp : mn;
        double& s_ = (__builtin_popcount(T) & 1) ? sp : sn;
        if (A > m_) {
          s_ = fma(s_, exp(m_ - A), 1.0);
          m_ = A;
        } else {
          s_ += exp(A - m_);
        }
      }
      if (sp == 0.0) continue;
      const double la = mp + log(sp), lb = sn > 0.0 ? mn + log(sn) : -INFINITY;
      if (!(la > lb)) continue;
      const double d = lb - la;
      const double cell = la + (d > -0.6931471805599453 ? log(-expm1(d)) : log1p(-exp(d)));
      double gcell[BWD ? NG : 1];
      if (BWD) {
        double ga[Q][MM], glf[Q];
#pragma unroll
        for (int i = 0; i < Q; ++i) {
          glf[i] = 0.0;
#pragma unroll
          for (int k = 0; k < MM; ++k) ga[i][k] = 0.0;
        }
        for (unsigned T = 1; T <= NSUB; ++T) {
          double A = 0.0, dl[MM], dzk[MM][Q];
#pragma unroll
          for (int k = 0; k < MM; ++k) {
            dl[k] = 0.0;
            if (k >= mo) continue;
            double xk[Q];
#pragma unroll
            for (int i = 0; i < Q; ++i) xk[i] = a[i][k];
            const double z = ql_fatmin_set<Q>(T, xk, tm, dzk[k]);
            A += fatmin2(z, Ws[kc][k], tm, &dl[k]);
          }
#pragma unroll
          for (int i = 0; i < Q; ++i)
            if (T >> i & 1) A += lf[i];
          if (A == -INFINITY) continue;
          const double cT = ((__builtin_popcount(T) & 1) ? 1.0 : -1.0) * exp(A - cell);
#pragma unroll
          for (int i = 0; i < Q; ++i) {
            if (!(T >> i & 1)) continue;
            glf[i] += cT;
#pragma unroll
            for (int k = 0; k < MM; ++k)
              if (k < mo) ga[i][k] = fma(cT * dl[k], dzk[k][i], ga[i][k]);
          }
        }
#pragma unroll
        for (int i = 0; i < Q; ++i) {
#pragma unroll
          for (int k = 0; k < MM; ++k) gcell[i * (MM + 1) + k] = ga[i][k] * da[i][k];
          gcell[i * (MM + 1) + MM] = glf[i];
        }
      }
      st.add(cell, gcell);
    }
  }
  for (int h = GR / 2; h >= 1; h /= 2) {   // fixed pairing: deterministic
    __syncthreads();
    if (g >= h && g < 2 * h) {
      double* r = red[(g - h) * CT + cl];
      r[0] = st.m;
      r[1] = st.s0;
      if (BWD) {
#pragma unroll
        for (int j = 0; j < NG; ++j) r[2 + j] = st.g[j];
      }
    }
    __syncthreads();
    if (g < h) {
      const double* r = red[g * CT + cl];
      st.merge(r[0], r[1], r + 2);
    }
  }
  if (g == 0 && c < b) {
    double* ob = out + ((size_t)s * nsplit + split) * NO * b;
    ob[c] = st.m;
    ob[(size_t)b + c] = st.s0;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < NG; ++j) ob[(size_t)(2 + j) * b + c] = st.g[j];
    }
  }
}

// workgroup per candidate, thread per sample: merge the splits per sample -> LSE_sc (split
// 0's m slot), the normalised gradient slots (g / s0) in split 0; acq_c = logmeanexp_s by
// fixed-order tree reductions (max, sum of exp); w_s (slot s0 of split 0) = gout softmax_s
// weight for the backward; NaN where the new-point Cholesky failed.  (A thread per
// candidate walking the S samples serially paid the load latency S times over.)
constexpr int QLR_THREADS = 256;

template <int MM, int Q, bool BWD>
__global__ __launch_bounds__(QLR_THREADS) void qlog_reduce(int b, int S, int nsplit, int m, double* __restrict__ ws,
                                                           const int* __restrict__ flags,
                                                           const double* __restrict__ gout, double* __restrict__ acq) {
  constexpr int NG = Q * (MM + 1);
  constexpr int NO = 2 + (BWD ? NG : 0);
  __shared__ double rd[QLR_THREADS];
  const int c = blockIdx.x, tid = threadIdx.x;
  double mloc = -INFINITY;
  for (int s = tid; s < S; s += QLR_THREADS) {
    double* o = ws + (size_t)s * nsplit * NO * b;
    LseState<NG, BWD> st;
    st.m = o[c];
    st.s0 = o[(size_t)b + c];
    if (BWD)
      for (int j = 0; j < NG; ++j) st.g[j] = o[(size_t)(2 + j) * b + c];
    for (int q = 1; q < nsplit; ++q) {
      const double* r = o + (size_t)q * NO * b;
      double g2[BWD ? NG : 1];
      if (BWD)
        for (int j = 0; j < NG; ++j) g2[j] = r[(size_t)(2 + j) * b + c];
      st.merge(r[c], r[(size_t)b + c], g2);
    }
    const double lse = (st.s0 > 0.0) ? st.m + log(st.s0) : -INFINITY;
    o[c] = lse;
    if (BWD)
      for (int j = 0; j < NG; ++j) o[(size_t)(2 + j) * b + c] = (st.s0 > 0.0) ? st.g[j] / st.s0 : 0.0;
    mloc = fmax(mloc, lse);
  }
  rd[tid] = mloc;
  for (int h = QLR_THREADS / 2; h > 0; h >>= 1) {
    __syncthreads();
    if (tid < h) rd[tid] = fmax(rd[tid], rd[tid + h]);
  }
  __syncthreads();
  const double mx = rd[0];
  __syncthreads();
  double sl = 0.0;
  if (mx > -INFINITY)
    for (int s = tid; s < S; s += QLR_THREADS) sl += exp(ws[(size_t)s * nsplit * NO * b + c] - mx);
  rd[tid] = sl;
  for (int h = QLR_THREADS / 2; h > 0; h >>= 1) {
    __syncthreads();
    if (tid < h) rd[tid] += rd[tid + h];
  }
  __syncthreads();
  const double lme = (mx > -INFINITY) ? mx + log(rd[0]) - log((double)S) : -INFINITY;
  if (tid == 0) {
    bool bad = false;
    for (int j = 0; j < m; ++j) bad |= flags[(size_t)j * b + c] != 0;
    acq[c] = bad ? nan("") : lme;
  }
  if (BWD) {
    const double go = gout ? gout[c] : 1.0;
    for (int s = tid; s < S; s += QLR_THREADS) {
      double* o = ws + (size_t)s * nsplit * NO * b;
      o[(size_t)b + c] = (lme > -INFINITY) ? go * exp(o[c] - lme) / (double)S : 0.0;
    }
  }
}

// thread per (sample, point): dY[s][j][p] from the weighted gradient slots through the
// objectives and the log feasibility (qg_dlog_fatmoid)
template <int MM, int Q>
__global__ void qlog_dy(int b, int S, int nsplit, QgObj o, const double* __restrict__ Y,
                        const double* __restrict__ ws, double* __restrict__ dY) {
  constexpr int NG = Q * (MM + 1);
  constexpr int NO = 2 + NG;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int bq = b * Q;
  if (e >= (long long)S * bq) return;
  const int s = (int)(e / bq), p = (int)(e % bq), c = p / Q, i = p % Q;
  const double* ob = ws + (size_t)s * nsplit * NO * b;
  const double w = ob[(size_t)b + c];
  const double* Ys = Y + (size_t)s * o.m * bq + p;
  double dy[QG_MAXM];
  for (int j = 0; j < QG_MAXM; ++j) dy[j] = 0.0;
  for (int k = 0; k < o.mo; ++k) {
    const int jj = o.oo[k];
    dy[jj] += w * ob[(size_t)(2 + i * (MM + 1) + k) * b + c] * qg_dobj(o, k, Ys[(size_t)jj * bq]);
  }
  const double glf = w * ob[(size_t)(2 + i * (MM + 1) + MM) * b + c];
  for (int t = 0; t < o.nc; ++t) {
    const int jj = o.co[t];
    const double cval = o.cs[t] * (Ys[(size_t)jj * bq] - o.ct[t]);
    dy[jj] += glf * qg_dlog_fatmoid(-cval / o.ce[t]) * (-o.cs[t] / o.ce[t]);
  }
  for (int j = 0; j < o.m; ++j) dY[((size_t)s * o.m + j) * bq + p] = dy[j];
}

struct QlPlan {
  int CT, nsplit, CB;
};

static QlPlan ql_plan(const evr_qnehvi_state* sth, int b) {
  QlPlan p;
  p.CT = b >= 48 ? 64 : (b > 16 ? 32 : 16);
  const int ctiles = cdiv(b, p.CT);
  const int maxc = std::max(sth->max_cells, 1);
  const int want = std::max(1, cdiv(2048, (long long)ctiles * sth->S));
  p.nsplit = std::min(want, cdiv(maxc, QL_CHUNK));
  p.CB = cdiv(cdiv(maxc, p.nsplit), QL_CHUNK) * QL_CHUNK;
  p.nsplit = cdiv(maxc, p.CB);
  return p;
}

#define QG_SWITCH(q, MACRO)                                                             \
  switch (q) {                                                                          \
    case 1: MACRO(1); break;                                                            \
    case 2: MACRO(2); break;                                                            \
    case 3: MACRO(3); break;                                                            \
    case 4: MACRO(4); break;                                                            \
    case 5: MACRO(5); break;                                                            \
    case 6: MACRO(6); break;                                                            \
    case 7: MACRO(7); break;                                                            \
    case 8: MACRO(8); break;                                                            \
    case 9: MACRO(9); break;                                                            \
    case 10: MACRO(10); break;                                                          \
    case 11: MACRO(11); break;                                                          \
    case 12: MACRO(12); break;                                                          \
    default: EVR_CHECK(false, "qnehvi_general: q = %d not supported", q);               \
  }

struct QlLayout {
  size_t Kx, R, P, Wf, Y, Lq, flags, LW, dY, cf, dKqq, cm, gR, dKx, Wb, kg, total;
  QlPlan plan;
  int MM;
};

static QlLayout ql_layout(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, int q, int d, int b,
                          bool backward) {
  QlLayout L{};
  const size_t m = stm->m, n = stm->n, S = stm->S, bq = (size_t)b * q;
  const size_t Rr = (size_t)qn_rows(stm);
  L.MM = sth->m <= 4 ? 4 : 8;
  L.plan = ql_plan(sth, b);
  const size_t NO = 2 + (backward ? (size_t)q * (L.MM + 1) : 0);
  size_t o = 0;
  auto take = [&](size_t doubles) {
    const size_t r = o;
    o += (doubles + 31) & ~(size_t)31;
    return r;
  };
  L.Kx = take(m * n * bq);
  L.R = take(m * Rr * bq);
  L.P = take(m * (size_t)evr_qnehvi_norms_rows(stm) * 2 * bq);
  L.Wf = take(proj_forward_ws_doubles(stm, (int)bq));
  L.Y = take(S * m * bq);
  L.Lq = take(m * b * q * q);
  L.flags = take((m * b + 1) / 2);
  L.LW = take(S * (size_t)L.plan.nsplit * NO * b);
  if (backward) {
    L.dY = take(S * m * bq);
    L.cf = take(m * b * q * q);
    L.dKqq = take(m * b * q * q);
    L.cm = take(m * bq);
    L.gR = take(m * Rr * bq);
    L.dKx = take(m * n * bq);
    L.Wb = take(dg_gemm_ws_doubles(true, (int)n, (int)bq, (int)Rr, (int)m));   // split-K partials of M^T gR
    L.kg = take(kcross_grad_ws_doubles((int)n, (int)bq, d));
  }
  L.total = o;
  return L;
}

}  // namespace evr

using namespace evr;

extern "C" {

long long evr_qng_workspace_doubles(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                                    const evr_qnehvi_model* md, int b, int backward) {
  if (!stm || !sth || !g || !md || b <= 0 || g->q < 1 || g->q > EVR_QNG_MAX_Q) return 0;
  return (long long)qg_layout(stm, sth, g->q, md->d, b, backward != 0).total;
}

int evr_qng_eval(void* stream, const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                 const evr_qnehvi_model* md, int b, const double* X, const double* gout, double* work, double* acq,
                 double* dX) {
  if (int rc = qg_check(stm, sth, g, md)) return rc;
  EVR_CHECK(X && work && acq && b >= 0, "evr_qng_eval: bad arguments");
  if (b == 0) return 0;
  QgObj o;
  if (int rc = qg_params(g, stm->m, &o)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int q = g->q, m = stm->m, n = stm->n, d = md->d, S = stm->S, nsub = (1 << q) - 1;
  const int bq = b * q, bv = b * nsub;
  const bool backward = dX != nullptr;
  const QgLayout L = qg_layout(stm, sth, q, d, b, backward);
  double* w = work;
  double* Kx = w + L.Kx;
  double* R = w + L.R;
  double* Y = w + L.Y;
  double* Lq = w + L.Lq;
  int* flags = (int*)(w + L.flags);
  double* Gv = w + L.Gv;
  double* Wv = w + L.Wv;
  double* hw = w + L.hvi;
  const QgDims dm{n, stm->nb, qn_nh(stm), S, m, b};

  if (int rc = evr_kernel_matrix(s, md->kind, m, n, bq, d, md->Xn, nullptr, nullptr, X, md->shift, md->scale,
                                 md->lengthscales, nullptr, nullptr, Kx))
    return rc;
  if (int rc = proj_forward(s, stm, bq, md->M, Kx, R, w + L.P, L.Wf != L.Y ? w + L.Wf : nullptr)) return rc;
#define GO(QQ)                                                                                                   \
  qg_gram_samples<QQ><<<dim3(b, m), 256, 0, s>>>(dm, md->kind, d, R, X, md->lengthscales, md->shift, md->scale,   \
                                                 stm->c, stm->ym, stm->ys, stm->kxx, g->zq, Y, Lq, flags);       \
  EVR_LAUNCH_CHECK();                                                                                            \
  qg_subsets<QQ><<<dim3(cdiv(b, 64), S), 64, 0, s>>>(S, b, o, Y, Gv, Wv);                                         \
  EVR_LAUNCH_CHECK()
  QG_SWITCH(q, GO);
#undef GO
  int ns = 1;
  double* dGv = backward ? w + L.dGv : nullptr;
  if (int rc = hvi_raw(s, sth, bv, Gv, backward, hw, dGv, &ns)) return rc;
  qg_combine_fwd<<<b, 256, 0, s>>>(S, ns, nsub, b, m, hw, Wv, flags, acq);
  EVR_LAUNCH_CHECK();
  if (!backward) return 0;
  double* dY = w + L.dY;
  double* cf = w + L.cf;
  double* dKqq = w + L.dKqq;
  double* cm = w + L.cm;
  double* gR = w + L.gR;
  double* dKx = w + L.dKx;
  const int Rr = qn_rows(stm);
#define GO(QQ)                                                                                                   \
  qg_subsets_bwd<QQ><<<dim3(cdiv(b, 64), S), 64, 0, s>>>(S, b, ns, o, Y, Wv, dGv, hw, gout, dY);                  \
  EVR_LAUNCH_CHECK();                                                                                            \
  qg_samples_bwd<QQ><<<dim3(b, m), 256, 0, s>>>(dm, dY, g->zq, Lq, stm->ys, cf, dKqq, cm);                        \
  EVR_LAUNCH_CHECK();                                                                                            \
  qg_gen_gr<QQ><<<dim3(m * Rr, cdiv(bq, 256)), 256, 0, s>>>(dm, R, dY, cf, cm, stm->ys, gR);                      \
  EVR_LAUNCH_CHECK()
  QG_SWITCH(q, GO);
#undef GO
  if (int rc = dg_gemm(s, true, n, bq, Rr, 1.0, md->M, n, (long long)Rr * n, gR, bq, (long long)Rr * bq, 0.0, dKx, bq,
                       (long long)n * bq, m, w + L.Wb))
    return rc;
  if (int rc = kcross_grad_launch(s, md->kind, m, n, bq, d, md->Xn, nullptr, nullptr, X, md->shift, md->scale,
                                  md->lengthscales, nullptr, dKx, dX, w + L.kg))
    return rc;
  if (q > 1) {
#define GO(QQ)                                                                                                   \
  qg_kqq_grad<QQ><<<cdiv(bq, 64), 64, 0, s>>>(b, m, d, md->kind, X, md->lengthscales, md->shift, md->scale,       \
                                              stm->kxx, dKqq, dX);                                               \
  EVR_LAUNCH_CHECK()
    QG_SWITCH(q, GO);
#undef GO
  }
  return 0;
}

int evr_objective_general(void* stream, int m_model, int n, int S, const evr_qn_general* g, const double* Y,
                          const double* mu, const double* ref, double* O) {
  QgObj o;
  if (int rc = qg_params(g, m_model, &o)) return rc;
  EVR_CHECK(Y && ref && O && n >= 0 && S >= 0, "evr_objective_general: bad arguments");
  const long long tot = (long long)n * S;
  if (tot == 0) return 0;
  qg_objective_kernel<<<cdiv(tot, 256), 256, 0, (hipStream_t)stream>>>(n, S, o, Y, mu, ref, O);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_objective_weights(void* stream, int m_model, int n, const evr_qn_general* g, const double* Y, double* G,
                          double* W) {
  QgObj o;
  if (int rc = qg_params(g, m_model, &o)) return rc;
  EVR_CHECK(Y && G && W && n >= 0, "evr_objective_weights: bad arguments");
  if (n == 0) return 0;
  qg_weights_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(n, o, Y, G, W);
  EVR_LAUNCH_CHECK();
  return 0;
}

long long evr_qlog_workspace_doubles(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                                     const evr_qnehvi_model* md, int b, int backward) {
  if (!stm || !sth || !g || !md || b <= 0 || g->q < 1 || g->q > EVR_QNG_MAX_Q) return 0;
  return (long long)ql_layout(stm, sth, g->q, md->d, b, backward != 0).total;
}

int evr_qlog_eval(void* stream, const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                  const evr_qnehvi_model* md, int b, const double* X, const double* gout, double* work, double* acq,
                  double* dX) {
  EVR_CHECK(stm && sth && g && md, "evr_qlog_eval: null argument");
  EVR_CHECK(g->q >= 1 && g->q <= EVR_QNG_MAX_Q, "evr_qlog_eval: q = %d outside 1..%d", g->q, EVR_QNG_MAX_Q);
  EVR_CHECK(sth->m == g->m_obj && sth->S == stm->S && sth->cell_lo && sth->cell_hi && sth->cell_off,
            "evr_qlog_eval: the scan state must carry m = m_obj objectives, the same S and explicit cells");
  EVR_CHECK(sth->tau_relu > 0.0 && sth->tau_max > 0.0, "evr_qlog_eval: tau_relu / tau_max must be positive");
  EVR_CHECK(md->n == stm->n && md->d >= 1 && md->M && md->Xn && md->lengthscales && g->zq && stm->c && stm->ym &&
                stm->ys && stm->kxx,
            "evr_qlog_eval: inconsistent model / state");
  EVR_CHECK(X && work && acq && b >= 0, "evr_qlog_eval: bad arguments");
  if (b == 0) return 0;
  QgObj o;
  if (int rc = qg_params(g, stm->m, &o)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int q = g->q, m = stm->m, n = stm->n, d = md->d, S = stm->S;
  const int bq = b * q;
  const bool backward = dX != nullptr;
  const QlLayout L = ql_layout(stm, sth, q, d, b, backward);
  double* w = work;
  double* Kx = w + L.Kx;
  double* R = w + L.R;
  double* Y = w + L.Y;
  double* Lq = w + L.Lq;
  int* flags = (int*)(w + L.flags);
  double* LW = w + L.LW;
  const QgDims dm{n, stm->nb, qn_nh(stm), S, m, b};
  if (int rc = evr_kernel_matrix(s, md->kind, m, n, bq, d, md->Xn, nullptr, nullptr, X, md->shift, md->scale,
                                 md->lengthscales, nullptr, nullptr, Kx))
    return rc;
  if (int rc = proj_forward(s, stm, bq, md->M, Kx, R, w + L.P, L.Wf != L.Y ? w + L.Wf : nullptr)) return rc;
  const QlPlan& P = L.plan;
  const dim3 grid(cdiv(b, P.CT), S, P.nsplit);
#define GO(QQ)                                                                                                    \
  qg_gram_samples<QQ><<<dim3(b, m), 256, 0, s>>>(dm, md->kind, d, R, X, md->lengthscales, md->shift, md->scale,    \
                                                 stm->c, stm->ym, stm->ys, stm->kxx, g->zq, Y, Lq, flags);        \
  EVR_LAUNCH_CHECK();                                                                                             \
  if (L.MM == 4) {                                                                                                \
    if (backward) qlog_scan<4, QQ, true><<<grid, QL_THREADS, 0, s>>>(b, P.nsplit, P.CT, P.CB, o, Y, sth->cell_off,  \
                                                                 sth->cell_lo, sth->cell_hi, sth->tau_relu,       \
                                                                 sth->tau_max, LW);                               \
    else qlog_scan<4, QQ, false><<<grid, QL_THREADS, 0, s>>>(b, P.nsplit, P.CT, P.CB, o, Y, sth->cell_off,          \
                                                          sth->cell_lo, sth->cell_hi, sth->tau_relu, sth->tau_max, \
                                                          LW);                                                    \
    EVR_LAUNCH_CHECK();                                                                                           \
    if (backward) qlog_reduce<4, QQ, true><<<b, QLR_THREADS, 0, s>>>(b, S, P.nsplit, m, LW, flags, gout, acq);    \
    else qlog_reduce<4, QQ, false><<<b, QLR_THREADS, 0, s>>>(b, S, P.nsplit, m, LW, flags, gout, acq);           \
    EVR_LAUNCH_CHECK();                                                                                           \
    if (backward) qlog_dy<4, QQ><<<cdiv((long long)S * bq, 256), 256, 0, s>>>(b, S, P.nsplit, o, Y, LW, w + L.dY); \
  } else {                                                                                                        \
    if (backward) qlog_scan<8, QQ, true><<<grid, QL_THREADS, 0, s>>>(b, P.nsplit, P.CT, P.CB, o, Y, sth->cell_off,  \
                                                                 sth->cell_lo, sth->cell_hi, sth->tau_relu,       \
                                                                 sth->tau_max, LW);                               \
    else qlog_scan<8, QQ, false><<<grid, QL_THREADS, 0, s>>>(b, P.nsplit, P.CT, P.CB, o, Y, sth->cell_off,          \
                                                          sth->cell_lo, sth->cell_hi, sth->tau_relu, sth->tau_max, \
                                                          LW);                                                    \
    EVR_LAUNCH_CHECK();                                                                                           \
    if (backward) qlog_reduce<8, QQ, true><<<b, QLR_THREADS, 0, s>>>(b, S, P.nsplit, m, LW, flags, gout, acq);    \
    else qlog_reduce<8, QQ, false><<<b, QLR_THREADS, 0, s>>>(b, S, P.nsplit, m, LW, flags, gout, acq);           \
    EVR_LAUNCH_CHECK();                                                                                           \
    if (backward) qlog_dy<8, QQ><<<cdiv((long long)S * bq, 256), 256, 0, s>>>(b, S, P.nsplit, o, Y, LW, w + L.dY); \
  }                                                                                                               \
  EVR_LAUNCH_CHECK()
  QG_SWITCH(q, GO);
#undef GO
  if (!backward) return 0;
  double* dY = w + L.dY;
  double* cf = w + L.cf;
  double* dKqq = w + L.dKqq;
  double* cm = w + L.cm;
  double* gR = w + L.gR;
  double* dKx = w + L.dKx;
  const int Rr = qn_rows(stm);
#define GO(QQ)                                                                                                   \
  qg_samples_bwd<QQ><<<dim3(b, m), 256, 0, s>>>(dm, dY, g->zq, Lq, stm->ys, cf, dKqq, cm);                        \
  EVR_LAUNCH_CHECK();                                                                                            \
  qg_gen_gr<QQ><<<dim3(m * Rr, cdiv(bq, 256)), 256, 0, s>>>(dm, R, dY, cf, cm, stm->ys, gR);                      \
  EVR_LAUNCH_CHECK()
  QG_SWITCH(q, GO);
#undef GO
  if (int rc = dg_gemm(s, true, n, bq, Rr, 1.0, md->M, n, (long long)Rr * n, gR, bq, (long long)Rr * bq, 0.0, dKx, bq,
                       (long long)n * bq, m, w + L.Wb))
    return rc;
  if (int rc = kcross_grad_launch(s, md->kind, m, n, bq, d, md->Xn, nullptr, nullptr, X, md->shift, md->scale,
                                  md->lengthscales, nullptr, dKx, dX, w + L.kg))
    return rc;
  if (q > 1) {
#define GO(QQ)                                                                                                   \
  qg_kqq_grad<QQ><<<cdiv(bq, 64), 64, 0, s>>>(b, m, d, md->kind, X, md->lengthscales, md->shift, md->scale,       \
                                              stm->kxx, dKqq, dX);                                               \
  EVR_LAUNCH_CHECK()
    QG_SWITCH(q, GO);
#undef GO
  }
  return 0;
}

}  // extern "C"

