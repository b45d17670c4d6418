// The training-row class of the restart-batch backward projection (qnehvi_small.hip qs_bwd),
// apart from the sample rows: it needs only the forward's R.  Its workgroups are the backward
// launch's z >= 1 slices, beside the sample-row workgroups (which hold one workgroup on 160 of
// the 256 CUs at the bench shape; in the tail of the restart scan they measured slower — the
// scan holds every slot — and that placement was removed).  For 16 training rows i of output
// j and a split of the rows r < n + nb of M_j
// (nb = 0: the fused root C; nb > 0: the split root's L^-1 and G blocks):
//   D[i][c]  = sum_r w_r M_j[r][i] R_j[r][c]                   (f64 MFMA, per-wave k-quarters)
// with w_r = s_j^2 on the L^-1 rows of the split root and 1 elsewhere: the two blocks' gR
// coefficients are -2 s_j^2 dbr and -2 dbr (L22^2 = s^2 (kxx - |L^-1 k|^2) - |G k|^2), so one
// class coefficient cf0 = -2 dbr (split) or -2 s^2 dbr (fused) covers both.
//   Q[c][k]  = sum_i D[i][c] dk(x_i, x_c)/dx_c[k]               (the cross-covariance gradient)
// The gR coefficient of this class (cf0[c], a reduction of the scan's dG over the samples) is a
// per-candidate scalar, so it is applied to Q in the dX reduction (qs_dx_reduce) instead of to
// D: the backward after the scan keeps only the sample rows and the coefficients.
#pragma once
#include "common.hpp"

namespace evr {

struct QsTail {
  const double* M;      // m x Rr x n
  const double* R;      // m x Rr x b
  const double* Xn;     // n x d (normalised training inputs)
  const double* X;      // b x d candidates (raw; may be the plan's pinned host buffer)
  const double* shift;  // d or null
  const double* scale;  // d or null
  const double* ls;     // m x d lengthscales
  double* part;         // dX partials, element-major: part[(c d + k) np + p]
  const double* ys;     // m output scales s_j (split root: rows < n of R are weighted by s_j^2)
  int n, nb, Rr, b, d, kind, nt, za, rows_per, poff, np;
  int nwg;              // workgroups (m za nt); a launch may carry padding ones past it
};

constexpr int QT_BI = 16;     // training rows per tail workgroup
constexpr int QT_MAXD = 8;    // input dims
constexpr int QT_B = 32;      // candidates
#ifndef EVR_QT_KB
#define EVR_QT_KB 8
#endif
constexpr int QT_KB = EVR_QT_KB;   // MFMA k-steps (4 rows each) per load batch (compile-time A/B knob)
// LDS (doubles): the waves' D tiles, then (aliased) the row groups' gradient partials; after
// them the candidates (normalised, b x d) and the inverse lengthscales (d)
constexpr int QT_RED = (4 * QT_BI * (QT_B + 1) > 8 * QT_B * QT_MAXD) ? 4 * QT_BI * (QT_B + 1) : 8 * QT_B * QT_MAXD;
constexpr int QT_LDS_DOUBLES = QT_RED + QT_B * QT_MAXD + QT_MAXD;

using qt_double4 = __attribute__((ext_vector_type(4))) double;

// one 256-thread workgroup: (tile, output j, row split z) = wg; partial index
// poff + (j za + z) nt + tile.  Registers stay low (it also runs inside hvi_kdw under that
// kernel's 96-VGPR bound): one candidate coordinate and one lengthscale per thread are loaded
// first (X may sit across PCIe: its latency hides behind the MFMA batches) and parked in LDS.
__device__ __forceinline__ void qs_tail_tile(const QsTail& t, int wg, double* lds) {
  if (wg >= t.nwg) return;   // whole workgroups: before any barrier
  const int per = t.nt * t.za;
  const int j = wg / per, rem = wg - j * per, z = rem / t.nt, tile = rem - z * t.nt;
  const int i0 = tile * QT_BI;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, kq = lane >> 4;
  const int n = t.n, b = t.b, d = t.d;
  const double* Mj = t.M + (size_t)j * t.Rr * n;
  const double* Rj = t.R + (size_t)j * t.Rr * b;
  double* xs = lds + QT_RED;                 // xs[c d + k]: (x - shift) scale / ls
  double* ils = xs + QT_B * QT_MAXD;         // 1 / ls_k
  const int bd = b * d;
  double xv = 0.0, lv = 1.0;   // candidate coordinate tid = (c, k) and ls_k
  if (tid < bd) {
    xv = t.X[tid];
    lv = t.ls[(size_t)j * d + tid % d];
  }
  // this wave's rows of the split: a quarter, whole k-steps.  Split root: the L^-1 block is
  // lower triangular, so its rows r < i0 are exact zeros in this tile's columns — the split's
  // rows start at i0 there and the waves share what remains
  const int zb0 = z * t.rows_per, ze = min(n + t.nb, zb0 + t.rows_per);
  const int zb = t.nb > 0 ? min(ze, max(zb0, i0)) : zb0;
  const double w0 = t.nb > 0 ? t.ys[j] * t.ys[j] : 1.0;
  const int rw = (((ze - zb + 3) / 4) + 3) & ~3;
  const int r0 = zb + wave * rw, r1 = min(ze, r0 + rw);
  const bool colok = i0 + i < n;
  qt_double4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
  for (int rb = r0; rb < r1; rb += 4 * QT_KB) {
    double av[QT_KB], b0[QT_KB], b1[QT_KB];
#pragma unroll
    for (int u = 0; u < QT_KB; ++u) {
      const int r = rb + 4 * u + kq;
      const bool rin = r < r1;
      const double w = r < n ? w0 : 1.0;
      av[u] = (rin && colok) ? Mj[(size_t)r * n + i0 + i] : 0.0;
      b0[u] = (rin && i < b) ? Rj[(size_t)r * b + i] * w : 0.0;
      b1[u] = (rin && 16 + i < b) ? Rj[(size_t)r * b + 16 + i] * w : 0.0;
    }
#pragma unroll
    for (int u = 0; u < QT_KB; ++u) {
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], b0[u], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], b1[u], a1, 0, 0, 0);
    }
  }
  if (tid < d) ils[tid] = 1.0 / lv;   // threads k < d hold ls_k (c = 0)
  if (tid < bd) {
    const int k = tid % d;
    xs[tid] = (xv - (t.shift ? t.shift[k] : 0.0)) * (t.scale ? t.scale[k] : 1.0) / lv;
  }
  // D map of v_mfma_f64_16x16x4: register q of lane l holds D[4q + (l >> 4)][l & 15]
  auto dk = reinterpret_cast<double(*)[QT_BI][QT_B + 1]>(lds);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    dk[wave][4 * q + kq][i] = a0[q];
    dk[wave][4 * q + kq][16 + i] = a1[q];
  }
  // thread (candidate c, row group g): rows i0 + g and i0 + g + 8 (their inputs load meanwhile)
  const int c = tid & (QT_B - 1), g = tid >> 5;
  double xr[2][QT_MAXD];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int irow = i0 + g + 8 * h;
#pragma unroll
    for (int k = 0; k < QT_MAXD; ++k) xr[h][k] = (irow < n && k < d) ? t.Xn[(size_t)irow * d + k] : 0.0;
  }
  __syncthreads();
  double acc[QT_MAXD];
#pragma unroll
  for (int k = 0; k < QT_MAXD; ++k) acc[k] = 0.0;
  double gk[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ii = g + 8 * h;
    gk[h] = ((dk[0][ii][c] + dk[1][ii][c]) + dk[2][ii][c]) + dk[3][ii][c];
  }
  if (c < b) {
    const int kj = kind_of(t.kind, j);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (i0 + g + 8 * h >= n) continue;
      double diff[QT_MAXD], d2 = 0.0;
#pragma unroll
      for (int k = 0; k < QT_MAXD; ++k) {
        // (x_c - x_i) / ls, with x_c / ls precomputed: the same value as qs_bwd's
        // ((x_c - shift) scale - x_i) / ls only up to rounding
        const double il = k < d ? ils[k] : 0.0;
        const double df = k < d ? xs[c * d + k] - xr[h][k] * il : 0.0;
        diff[k] = df * il;
        d2 = fma(df, df, d2);
      }
      const double sgl = gk[h] * kernel_dscale(kj, d2);
#pragma unroll
      for (int k = 0; k < QT_MAXD; ++k) acc[k] = fma(sgl, diff[k], acc[k]);
    }
  }
  __syncthreads();   // every thread has read dk (gx aliases it)
  auto gx = reinterpret_cast<double(*)[QT_B][QT_MAXD]>(lds);
#pragma unroll
  for (int k = 0; k < QT_MAXD; ++k) gx[g][c][k] = acc[k];
  __syncthreads();
  if (tid < QT_B * QT_MAXD) {
    const int cc = tid / QT_MAXD, k = tid - cc * QT_MAXD;
    double v = gx[0][cc][k];
#pragma unroll
    for (int q = 1; q < 8; ++q) v += gx[q][cc][k];
    if (cc < b && k < d) t.part[((size_t)cc * d + k) * t.np + t.poff + ((size_t)j * t.za + z) * t.nt + tile] = v;
  }
}

}  // namespace evr
