// qNEHVI projection GEMMs with fused prologue / epilogue (gfx950 f64 MFMA).
//
// Forward:  R_j = M_j K_x  (M_j = [L^-1; G; H^T; alpha^T], Rr x n; K_x: n x b), as in
// acquisition.py.  The epilogue also emits, per 64-row tile and candidate, the partial sums
// of squares of the L^-1 k rows (rows < n) and of the L21 rows (n <= row < n + nb), so the
// sampling step reads (rows-tiles x 2) partials and the S + 1 sample / mean rows instead of
// the whole 21 MB R (the old samples kernel re-read all of R with 40 workgroups).
//
// Backward: dK_x,j = M_j^T gR_j with gR_j never materialised.  gR_j is, per candidate c,
//   rows < n:            2 R[i][c] dssv(c)      (var = s^2 (kxx - |L^-1 k|^2))
//   n <= rows < n + nb:  2 R[i][c] dssw(c)      (L22^2 = var - |L21|^2)
//   sample rows s:       a_j dG[s][j][c]
//   mean row:            s_j dmu(c),  dmu = sum_s a_j dG, dl = sum_s a_j dG zq[s][j],
//                        dbr = dl / (2 L22), dssv = -s^2 dbr, dssw = -dbr.
// A small kernel reduces dmu, dl over the samples into per-candidate coefficients; the GEMM
// fetch then generates gR from R, dG and those coefficients — one pass over R and dG, no
// 21 MB gR write + re-read (the unfused qn_samples_bwd_kernel + gemm^T).  Both GEMMs split K
// (fixed-order reduction) when their tile grid cannot fill the 256 CUs (small candidate
// batches: the L-BFGS restarts).
//
// Tile: 64 x 64 outputs per 256-thread workgroup, 4 waves x (2 x 2) v_mfma_f64_16x16x4f64,
// K step 16 staged through LDS, global loads of step t+1 issued before the MFMAs of step t.
#include <algorithm>
#include <cstdlib>

#include <rocblas/rocblas.h>

#include "common.hpp"
#include "../../include/everest_amd.h"

using double4_t = __attribute__((ext_vector_type(4))) double;

#ifndef EVR_PK
#define EVR_PK 16
#endif
namespace evr {

constexpr int PT = 64, PK = EVR_PK, PPAD = 16;
constexpr int PU = PT * PK / 256;   // staged elements of A and of B per thread and k-step

// 64 x 64 f64 MFMA tile over k in [kbeg, kend): fa(row, k) / fb(k, col) fetch one element
// (tile-local row / col); the fetch of step t+1 is issued before the MFMAs of step t.
// TA: A element (row, k) is contiguous along row (coalesce the A fetch along rows).
template <bool TA, class FA, class FB>
__device__ __forceinline__ void proj_tile(int kbeg, int kend, FA fa, FB fb, double4_t (&acc)[4]) {
  __shared__ double As[PK][PT + PPAD];
  __shared__ double Bs[PK][PT + PPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  int am[PU], ak[PU], bn[PU], bk[PU];
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int e = u * 256 + tid;
    if (TA) { am[u] = e % PT; ak[u] = e / PT; } else { ak[u] = e % PK; am[u] = e / PK; }
    bn[u] = e % PT;
    bk[u] = e / PT;
  }
  double ra[PU], rb[PU];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int k = k0 + ak[u], kb = k0 + bk[u];
      ra[u] = (k < kend) ? fa(am[u], k) : 0.0;
      rb[u] = (kb < kend) ? fb(kb, bn[u]) : 0.0;
    }
  };
  if (kbeg < kend) fetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += PK) {
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      As[ak[u]][am[u]] = ra[u];
      Bs[bk[u]][bn[u]] = rb[u];
    }
    __syncthreads();
    if (k0 + PK < kend) fetch(k0 + PK);
    const int i = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < PK; kk += 4) {
      const double a0 = As[kk + kq][wm + i], a1 = As[kk + kq][wm + 16 + i];
      const double b0 = Bs[kk + kq][wn + i], b1 = Bs[kk + kq][wn + 16 + i];
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
    }
    __syncthreads();
  }
}

// visit the tile's outputs: f(local_row, local_col, value) — D map of v_mfma_f64_16x16x4:
// register r of lane l holds D[(l >> 4) + 4 r][l & 15]
template <class F>
__device__ __forceinline__ void proj_for_each(const double4_t (&acc)[4], F f) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int col = lane & 15, rq = lane >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) f(wm + (q >> 1) * 16 + rq + 4 * r, wn + (q & 1) * 16 + col, acc[q][r]);
}

// partial sums of squares of a 64 x 64 tile of R, by row class (cls 0: rows < n, 1: rows in
// [n, n + nb)), reduced over the tile's rows in a fixed order -> P[j][rt][cls][c]
__device__ __forceinline__ void proj_norms(const double (&sq)[2][2], int n0, int b, double* __restrict__ Pout) {
  __shared__ double red[4][32][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, rq = lane >> 4;
  double v4[2][2];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int cls = 0; cls < 2; ++cls) {
      double v = sq[ni][cls];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      v4[ni][cls] = v;
    }
  if (rq == 0) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      red[wave][ni * 16 + col][0] = v4[ni][0];
      red[wave][ni * 16 + col][1] = v4[ni][1];
    }
  }
  __syncthreads();
  if (tid < 128) {
    const int cls = tid >> 6, t = tid & 63;
    const int h = t >> 5, cw = t & 31;   // waves h (rows 0-31) and h + 2 (rows 32-63) share columns
    const double v = red[h][cw][cls] + red[h + 2][cw][cls];
    if (n0 + t < b) Pout[(size_t)cls * b + n0 + t] = v;
  }
}

// ---------------------------------------------------------------------------------------
// forward: R_j = M_j K_x,j (+ partial norms), optional split-K into W
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void qn_proj_fwd(int n, int nb, int Rr, int b, int m, const double* __restrict__ Mm,
                                                   const double* __restrict__ Kx, double* __restrict__ R,
                                                   double* __restrict__ P, int nrt, int ksplit, int kchunk,
                                                   double* __restrict__ W) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int t = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int bx = t % gx, by = (t / gx) % gy, bz = t / (gx * gy);
  const int j = bz / ksplit, kz = bz - j * ksplit;
  const int m0 = by * PT, n0 = bx * PT;
  const double* A = Mm + (size_t)j * Rr * n;
  const double* B = Kx + (size_t)j * n * b;
  double4_t acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  const int kbeg = kz * kchunk, kend = min(n, kbeg + kchunk);
  proj_tile<false>(
      kbeg, kend, [&](int r, int k) { return (m0 + r < Rr) ? A[(size_t)(m0 + r) * n + k] : 0.0; },
      [&](int k, int c) { return (n0 + c < b) ? B[(size_t)k * b + n0 + c] : 0.0; }, acc);
  if (ksplit > 1) {
    double* Wz = W + ((size_t)kz * m + j) * Rr * b;
    proj_for_each(acc, [&](int r, int c, double v) {
      if (m0 + r < Rr && n0 + c < b) Wz[(size_t)(m0 + r) * b + n0 + c] = v;
    });
    return;
  }
  double* Rj = R + (size_t)j * Rr * b;
  double sq[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  proj_for_each(acc, [&](int r, int c, double v) {
    const int row = m0 + r;
    if (row < Rr && n0 + c < b) Rj[(size_t)row * b + n0 + c] = v;
    const int ni = (c & 31) >> 4;
    if (row < n) sq[ni][0] += v * v;
    else if (row < n + nb) sq[ni][1] += v * v;
  });
  proj_norms(sq, n0, b, P + ((size_t)j * nrt + by) * 2 * b);
}

// split-K reduction of the forward: R = sum_kz W[kz] (fixed order) + the partial norms
__global__ __launch_bounds__(256) void qn_proj_fwd_reduce(int n, int nb, int Rr, int b, int m, int ksplit,
                                                          const double* __restrict__ W, double* __restrict__ R,
                                                          double* __restrict__ P, int nrt) {
  const int j = blockIdx.z;
  const int m0 = blockIdx.y * PT, n0 = blockIdx.x * PT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // reuse the MFMA D layout so proj_norms' reduction order applies unchanged
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int col = lane & 15, rq = lane >> 4;
  double sq[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  double* Rj = R + (size_t)j * Rr * b;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm + (q >> 1) * 16 + rq + 4 * r, c = n0 + wn + (q & 1) * 16 + col;
      double v = 0.0;
      if (row < Rr && c < b) {
#pragma unroll 4
        for (int kz = 0; kz < ksplit; ++kz) v += W[(((size_t)kz * m + j) * Rr + row) * b + c];
        Rj[(size_t)row * b + c] = v;
      }
      if (row < n) sq[q & 1][0] += v * v;
      else if (row < n + nb) sq[q & 1][1] += v * v;
    }
  proj_norms(sq, n0, b, P + ((size_t)j * nrt + blockIdx.y) * 2 * b);
}

// ---------------------------------------------------------------------------------------
// samples from the partial norms: thread per (candidate, output, chunk of SCH samples)
// ---------------------------------------------------------------------------------------
constexpr int SCH = 8;   // 16-sample chunks left 640 one-wave blocks at the bench shape

__global__ __launch_bounds__(64) void qn_samples_norms(int n, int nb, int S, int nh, int m, int b, int nrt_used,
                                                       int nrt,
                                                       const double* __restrict__ P, const double* __restrict__ R,
                                                       const double* __restrict__ cc, const double* __restrict__ ym,
                                                       const double* __restrict__ ys, const double* __restrict__ kxx,
                                                       const double* __restrict__ zq, const double* __restrict__ oa,
                                                       const double* __restrict__ ob, double* __restrict__ G,
                                                       double* __restrict__ L22, int* __restrict__ flags) {
  const int c = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y, chunk = blockIdx.z;
  if (c >= b) return;
  const long long Rr = (long long)n + nb + nh + 1;
  const double* Rj = R + (size_t)j * Rr * b;
  // the chunk's sample rows and z values do not depend on the norms: issue their loads
  // first so that they overlap the partial-norm sum
  const int s0 = chunk * SCH, ns = min(S - s0, SCH);
  const double* h = Rj + (size_t)(n + nb) * b + c;
  double hv[SCH], zv[SCH];
#pragma unroll
  for (int q = 0; q < SCH; ++q) {
    hv[q] = (nh && q < ns) ? h[(size_t)(s0 + q) * b] : 0.0;
    zv[q] = (q < ns) ? zq[(size_t)(s0 + q) * m + j] : 0.0;
  }
  const double* Pj = P + (size_t)j * nrt * 2 * b;
  double mu, l22;
  int flag;
  qn_mu_l22(Pj, nrt_used, b, c, Rj[(size_t)(Rr - 1) * b + c], ys[j], cc[j], ym[j], kxx[j], mu, l22, flag);
  if (chunk == 0) {
    L22[(size_t)j * b + c] = l22;
    flags[(size_t)j * b + c] = flag;
  }
  const double A = oa[j], B0 = ob[j];
#pragma unroll
  for (int q = 0; q < SCH; ++q) {
    if (q < ns) {
      G[((size_t)(s0 + q) * m + j) * b + c] = qn_sample_obj(mu, hv[q], nh != 0, l22, zv[q], A, B0);
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward coefficients of gR per (output, candidate): coef[j][0..2][c] =
// (2 dssv, 2 dssw, s dmu); fixed-order sums
// ---------------------------------------------------------------------------------------
constexpr int BC_C = 16, BC_G = 64;   // 16 candidates x 64 sample groups: 160 workgroups at b = 512, m = 5
__global__ __launch_bounds__(BC_C * BC_G) void qn_bwd_coef(int S, int m, int b, const double* __restrict__ dG,
                                                          const double* __restrict__ L22,
                                                          const double* __restrict__ ys,
                                                          const double* __restrict__ zq,
                                                          const double* __restrict__ oa,
                                                          double* __restrict__ coef) {
  __shared__ double red[BC_G][BC_C][2];
  const int j = blockIdx.y, cx = threadIdx.x % BC_C, g = threadIdx.x / BC_C;
  const int c = blockIdx.x * BC_C + cx;
  const double aj = oa[j];
  double dmu = 0.0, dl = 0.0;
  if (c < b) {
#pragma unroll 4
    for (int s = g; s < S; s += BC_G) {
      const double dy = aj * dG[((size_t)s * m + j) * b + c];
      dmu += dy;
      dl = fma(dy, zq[(size_t)s * m + j], dl);
    }
  }
  red[g][cx][0] = dmu;
  red[g][cx][1] = dl;
  __syncthreads();
  if (g < 8) {   // fixed order: 8 groups of 8, then the 8 partials
    dmu = red[g * 8][cx][0];
    dl = red[g * 8][cx][1];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      dmu += red[g * 8 + q][cx][0];
      dl += red[g * 8 + q][cx][1];
    }
  }
  __syncthreads();
  if (g < 8) {
    red[g][cx][0] = dmu;
    red[g][cx][1] = dl;
  }
  __syncthreads();
  if (g == 0 && c < b) {
    dmu = red[0][cx][0];
    dl = red[0][cx][1];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      dmu += red[q][cx][0];
      dl += red[q][cx][1];
    }
    const double sj = ys[j];
    const double dbr = dl / (2.0 * L22[(size_t)j * b + c]);
    coef[((size_t)j * 3 + 0) * b + c] = -2.0 * sj * sj * dbr;
    coef[((size_t)j * 3 + 1) * b + c] = -2.0 * dbr;
    coef[((size_t)j * 3 + 2) * b + c] = sj * dmu;
  }
}

// ---------------------------------------------------------------------------------------
// backward: dKx_j = M_j^T gR_j with gR generated in the fetch, optional split-K into W
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void qn_proj_bwd(int n, int nb, int S, int nh, int m, int b,
                                                   const double* __restrict__ Mm, const double* __restrict__ R,
                                                   const double* __restrict__ dG, const double* __restrict__ oa,
                                                   const double* __restrict__ coef, double* __restrict__ dK,
                                                   int ksplit, int kchunk, double* __restrict__ W) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int t = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int bx = t % gx, by = (t / gx) % gy, bz = t / (gx * gy);
  const int j = bz / ksplit, kz = bz - j * ksplit;
  const int m0 = by * PT, n0 = bx * PT;
  const int Rr = n + nb + nh + 1;
  const double* A = Mm + (size_t)j * Rr * n;   // A(row, k) = M_j[k][row]
  const double* Rj = R + (size_t)j * Rr * b;
  const double* cj = coef + (size_t)j * 3 * b;
  const double aj = oa[j];
  __shared__ double cf[3][PT];
  if (threadIdx.x < 3 * PT) {
    const int q = threadIdx.x / PT, c = threadIdx.x - q * PT;
    cf[q][c] = (n0 + c < b) ? cj[(size_t)q * b + n0 + c] : 0.0;
  }
  __syncthreads();
  double4_t acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  const int kbeg = kz * kchunk, kend = min(Rr, kbeg + kchunk);
  proj_tile<true>(
      kbeg, kend, [&](int r, int k) { return (m0 + r < n) ? A[(size_t)k * n + m0 + r] : 0.0; },
      [&](int k, int c) {
        if (n0 + c >= b) return 0.0;
        if (k < n) return Rj[(size_t)k * b + n0 + c] * cf[0][c];
        if (k < n + nb) return Rj[(size_t)k * b + n0 + c] * cf[1][c];
        if (k < n + nb + nh) return aj * dG[((size_t)(k - n - nb) * m + j) * b + n0 + c];
        return cf[2][c];
      },
      acc);
  double* out = (ksplit > 1) ? W + ((size_t)kz * m + j) * n * b : dK + (size_t)j * n * b;
  proj_for_each(acc, [&](int r, int c, double v) {
    if (m0 + r < n && n0 + c < b) out[(size_t)(m0 + r) * b + n0 + c] = v;
  });
}

__global__ __launch_bounds__(256) void qn_splitk_sum(long long per, int ksplit, const double* __restrict__ W,
                                                     double* __restrict__ out) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= per) return;
  double v = 0.0;
#pragma unroll 4
  for (int kz = 0; kz < ksplit; ++kz) v += W[(size_t)kz * per + e];
  out[e] = v;
}

// split K when the tile grid cannot fill the chip (aim at >= 512 workgroups, i.e. two per
// CU); each slice keeps >= 8 k-steps.  More slices than that only add partial-sum traffic.
static int proj_ksplit(int tiles, int K, int* kchunk) {
  int ks = 1;
  if (tiles < 512) ks = std::max(1, std::min(std::min(cdiv(512, tiles), K / (8 * PK)), 32));
  *kchunk = ks > 1 ? cdiv(cdiv(K, ks), PK) * PK : std::max(K, 1);
  return ks > 1 ? cdiv(K, *kchunk) : 1;
}

// ---------------------------------------------------------------------------------------
// Library-GEMM variant (rocBLAS dgemm for the plain contractions, hand-written fused
// epilogue / prologue kernels around them).  rocBLAS' f64 MFMA kernels reach ~48 TF/s at
// this shape vs ~26 TF/s for the 64x64 tile above; EVR_GEMM=mfma selects the fully fused
// kernels instead.
// ---------------------------------------------------------------------------------------
// partial norms of R rows [0, n + nb) per 64-row tile: block = 64 candidates x 4 row groups
__global__ __launch_bounds__(256) void qn_norms_rows(int n, int nb, int Rr, int b, int nrt,
                                                     const double* __restrict__ R, double* __restrict__ P) {
  const int j = blockIdx.z, rt = blockIdx.y;
  const int cx = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cx;
  __shared__ double red[4][64][2];
  double s0 = 0.0, s1 = 0.0;
  if (c < b) {
    const double* Rj = R + (size_t)j * Rr * b;
#pragma unroll 4
    for (int r = 0; r < 16; ++r) {
      const int row = rt * 64 + rg * 16 + r;
      if (row < n + nb) {
        const double v = Rj[(size_t)row * b + c];
        if (row < n) s0 = fma(v, v, s0);
        else s1 = fma(v, v, s1);
      }
    }
  }
  red[rg][cx][0] = s0;
  red[rg][cx][1] = s1;
  __syncthreads();
  if (rg < 2 && c < b) {
    const double v = ((red[0][cx][rg] + red[1][cx][rg]) + red[2][cx][rg]) + red[3][cx][rg];
    P[(((size_t)j * nrt + rt) * 2 + rg) * b + c] = v;
  }
}

// gR_j (Rr x b) from R, dG and the per-candidate coefficients (see the header).  Grid =
// (m * Rr rows, candidate tiles): no 64-bit division per element (the flat-index form spent
// 8.5 us on 31 MB at m = 5, Rr = 769, b = 512 on MI355X)
__global__ __launch_bounds__(256) void qn_gen_gr(int n, int nb, int nh, int m, int b, const double* __restrict__ R,
                                                 const double* __restrict__ dG, const double* __restrict__ oa,
                                                 const double* __restrict__ coef, double* __restrict__ gR) {
  const int Rr = n + nb + nh + 1;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= b) return;
  const int rj = blockIdx.x;
  const int j = rj / Rr, row = rj - j * Rr;
  const size_t e = (size_t)rj * b + c;
  const double* cj = coef + (size_t)j * 3 * b;
  double v;
  if (row < n) v = R[e] * cj[c];
  else if (row < n + nb) v = R[e] * cj[(size_t)b + c];
  else if (row < n + nb + nh) v = oa[j] * dG[((size_t)(row - n - nb) * m + j) * b + c];
  else v = cj[(size_t)2 * b + c];
  gR[e] = v;
}

static bool use_rocblas() {
  static const bool v = [] {
    const char* e = std::getenv("EVR_GEMM");
    return !(e && std::string(e) == "mfma");
  }();
  return v;
}

static rocblas_handle rb_handle() {
  thread_local rocblas_handle h = nullptr;
  if (!h && rocblas_create_handle(&h) != rocblas_status_success) h = nullptr;
  // bitwise-reproducible results: no atomics-based split-K in the Tensile kernels
  if (h) (void)rocblas_set_atomics_mode(h, rocblas_atomics_not_allowed);
  return h;
}

// row-major C = op(A) op(B) batched (alpha 1, beta 0) through rocBLAS' column-major dgemm
int rb_gemm(hipStream_t s, bool tA, int M, int N, int K, const double* A, int lda, long long sA,
                   const double* B, int ldb, long long sB, double* C, int ldc, long long sC, int batch) {
  rocblas_handle h = rb_handle();
  EVR_CHECK(h, "rocBLAS handle creation failed");
  EVR_CHECK(rocblas_set_stream(h, s) == rocblas_status_success, "rocblas_set_stream failed");
  const double one = 1.0, zero = 0.0;
  const rocblas_status st = rocblas_dgemm_strided_batched(h, rocblas_operation_none,
                                                           tA ? rocblas_operation_transpose : rocblas_operation_none,
                                                           N, M, K, &one, B, ldb, sB, A, lda, sA, &zero, C, ldc, sC,
                                                           batch);
  EVR_CHECK(st == rocblas_status_success, "rocblas_dgemm_strided_batched failed (%d)", (int)st);
  return 0;
}

// mean row of R (the operator's last row, alpha^T K_x): 16 candidates x 64 row groups per
// block, so a b = 512, m = 5 pass spreads over 160 workgroups (64-candidate blocks used only
// 40 CUs: 9.1 us for 10.5 MB on MI355X).  Each wave reads 4 rows x 128 B (one cache line per
// row); fixed-order sums: 8 strided rows per thread, then 8 groups of 8, then 8 partials
// (see proj_forward for why it is not a GEMM row)
constexpr int MR_C = 16, MR_G = 64;
__global__ __launch_bounds__(MR_C * MR_G) void qn_mean_row(int n, int Rr, int b, const double* __restrict__ Mm,
                                                          const double* __restrict__ Kx, double* __restrict__ R) {
  __shared__ double red[MR_G][MR_C];
  const int j = blockIdx.y, cx = threadIdx.x % MR_C, rg = threadIdx.x / MR_C;
  const int c = blockIdx.x * MR_C + cx;
  const double* a = Mm + ((size_t)j * Rr + (Rr - 1)) * n;
  const double* K = Kx + (size_t)j * n * b;
  double acc = 0.0;
  if (c < b) {
#pragma unroll 8
    for (int i = rg; i < n; i += MR_G) acc = fma(a[i], K[(size_t)i * b + c], acc);
  }
  red[rg][cx] = acc;
  __syncthreads();
  if (rg < 8) {
    double v = red[rg * 8][cx];
#pragma unroll
    for (int g = 1; g < 8; ++g) v += red[rg * 8 + g][cx];
    acc = v;
  }
  __syncthreads();
  if (rg < 8) red[rg][cx] = acc;
  __syncthreads();
  if (rg == 0 && c < b) {
    double v = red[0][cx];
#pragma unroll
    for (int g = 1; g < 8; ++g) v += red[g][cx];
    R[((size_t)j * Rr + (Rr - 1)) * b + c] = v;
  }
}

int gemm_backend_init() {
  if (use_rocblas()) EVR_CHECK(rb_handle(), "rocBLAS handle creation failed");
  return 0;
}

// ---- internal launchers (workspace supplied by the caller; qnehvi_plan.hip) ----------
size_t proj_forward_ws_doubles(const evr_qnehvi_state* st, int b) {
  const int Rr = qn_rows(st);
  if (use_rocblas()) return 0;
  int kchunk = 0;
  const int ks = proj_ksplit(cdiv(b, PT) * cdiv(Rr, PT) * st->m, st->n, &kchunk);
  return ks > 1 ? (size_t)ks * st->m * Rr * b : 0;
}

int proj_forward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* Kx, double* R,
                 double* norms, double* W) {
  if (b == 0) return 0;
  const int Rr = qn_rows(st);
  const int nrt = cdiv(Rr, PT);
  if (use_rocblas()) {
    // The mean row alpha^T k is the operator's last row; kept in the GEMM it adds a 13th
    // 64-row tile at Rr = 769 and unbalances the tile grid over the 256 CUs (MI355X,
    // 5 x {769, 768} x 512 x 512: 54 vs 40 us).  GEMM over the first Rr - 1 rows, the mean
    // row by qn_mean_row over the same K_x (rocBLAS' batched gemv took ~20 us there).
    if (int rc = rb_gemm(s, false, Rr - 1, b, st->n, Mm, st->n, (long long)Rr * st->n, Kx, b, (long long)st->n * b, R,
                         b, (long long)Rr * b, st->m))
      return rc;
    qn_mean_row<<<dim3(cdiv(b, MR_C), st->m), MR_C * MR_G, 0, s>>>(st->n, Rr, b, Mm, Kx, R);
    EVR_LAUNCH_CHECK();
    qn_norms_rows<<<dim3(cdiv(b, 64), cdiv(st->n + st->nb, 64), st->m), 256, 0, s>>>(st->n, st->nb, Rr, b, nrt, R,
                                                                                     norms);
    EVR_LAUNCH_CHECK();
    return 0;
  }
  int kchunk = 0;
  const int ks = proj_ksplit(cdiv(b, PT) * nrt * st->m, st->n, &kchunk);
  EVR_CHECK(ks == 1 || W, "proj_forward: split-K workspace missing");
  dim3 grid(cdiv(b, PT), nrt, st->m * ks);
  qn_proj_fwd<<<grid, 256, 0, s>>>(st->n, st->nb, Rr, b, st->m, Mm, Kx, R, norms, nrt, ks, kchunk, W);
  EVR_LAUNCH_CHECK();
  if (ks > 1) {
    qn_proj_fwd_reduce<<<dim3(cdiv(b, PT), nrt, st->m), 256, 0, s>>>(st->n, st->nb, Rr, b, st->m, ks, W, R, norms,
                                                                       nrt);
    EVR_LAUNCH_CHECK();
  }
  return 0;
}

// backward: the generated-gR MFMA kernel wins at small candidate batches (the L-BFGS
// restarts), gR materialisation + rocBLAS from b = 64 on (measured on MI355X)
static bool bwd_rocblas(int b) { return use_rocblas() && b >= 64; }

size_t proj_backward_ws_doubles(const evr_qnehvi_state* st, int b) {
  const int Rr = qn_rows(st);
  if (bwd_rocblas(b)) return (size_t)st->m * 3 * b + (size_t)st->m * Rr * b;   // coefficients + gR
  int kchunk = 0;
  const int ks = proj_ksplit(cdiv(b, PT) * cdiv(st->n, PT) * st->m, Rr, &kchunk);
  return (size_t)st->m * 3 * b + (ks > 1 ? (size_t)ks * st->m * st->n * b : 0);
}

int proj_backward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* R,
                  const double* L22, const double* dG, double* dKx, double* ws) {
  if (b == 0) return 0;
  const int Rr = qn_rows(st);
  double* coef = ws;
  qn_bwd_coef<<<dim3(cdiv(b, BC_C), st->m), BC_C * BC_G, 0, s>>>(st->S, st->m, b, dG, L22, st->ys, st->zq, st->obj_a, coef);
  EVR_LAUNCH_CHECK();
  if (bwd_rocblas(b)) {
    double* gR = ws + (size_t)st->m * 3 * b;
    qn_gen_gr<<<dim3(st->m * Rr, cdiv(b, 256)), 256, 0, s>>>(st->n, st->nb, qn_nh(st), st->m, b, R, dG, st->obj_a, coef, gR);
    EVR_LAUNCH_CHECK();
    return rb_gemm(s, true, st->n, b, Rr, Mm, st->n, (long long)Rr * st->n, gR, b, (long long)Rr * b, dKx, b,
                   (long long)st->n * b, st->m);
  }
  int kchunk = 0;
  const int ks = proj_ksplit(cdiv(b, PT) * cdiv(st->n, PT) * st->m, Rr, &kchunk);
  double* W = ws + (size_t)st->m * 3 * b;
  dim3 grid(cdiv(b, PT), cdiv(st->n, PT), st->m * ks);
  qn_proj_bwd<<<grid, 256, 0, s>>>(st->n, st->nb, st->S, qn_nh(st), st->m, b, Mm, R, dG, st->obj_a, coef, dKx, ks, kchunk, W);
  EVR_LAUNCH_CHECK();
  if (ks > 1) {
    const long long per = (long long)st->m * st->n * b;
    qn_splitk_sum<<<cdiv(per, 256), 256, 0, s>>>(per, ks, W, dKx);
    EVR_LAUNCH_CHECK();
  }
  return 0;
}

int samples_norms(hipStream_t s, const evr_qnehvi_state* st, int b, const double* R, const double* norms, double* G,
                  double* L22, int* flags, int tile_rows) {
  if (b == 0) return 0;
  const int Rr = qn_rows(st);
  const int nrt = cdiv(Rr, tile_rows);   // partial-norm tiles (64 rows here, 16 in qnehvi_small.hip)
  const int nrt_used = cdiv(st->n + st->nb, tile_rows);
  dim3 grid(cdiv(b, 64), st->m, cdiv(st->S, SCH));
  qn_samples_norms<<<grid, 64, 0, s>>>(st->n, st->nb, st->S, qn_nh(st), st->m, b, nrt_used, nrt, norms, R, st->c, st->ym, st->ys,
                                        st->kxx, st->zq, st->obj_a, st->obj_b, G, L22, flags);
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // namespace evr

using namespace evr;

extern "C" {

int evr_qnehvi_norms_rows(const evr_qnehvi_state* st) {
  if (!st) return 0;
  return cdiv((long long)qn_rows(st), PT);
}

long long evr_qnehvi_project_workspace_doubles(const evr_qnehvi_state* st, int b) {
  return (st && b > 0) ? (long long)proj_forward_ws_doubles(st, b) : 0;
}

int evr_qnehvi_project(void* stream, const evr_qnehvi_state* st, int b, const double* Mm, const double* Kx,
                       double* R, double* norms, double* work) {
  EVR_CHECK(st && Mm && Kx && R && norms && b >= 0, "evr_qnehvi_project: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const size_t wn = proj_forward_ws_doubles(st, b);
  const bool own = wn && !work;
  if (own) EVR_HIP(hipMallocAsync((void**)&work, sizeof(double) * wn, s));
  const int rc = proj_forward(s, st, b, Mm, Kx, R, norms, work);
  if (own) EVR_HIP(hipFreeAsync(work, s));
  return rc;
}

int evr_qnehvi_samples_norms(void* stream, const evr_qnehvi_state* st, int b, const double* R, const double* norms,
                             double* G, double* L22, int* flags) {
  EVR_CHECK(st && R && norms && G && L22 && flags && b >= 0, "evr_qnehvi_samples_norms: bad arguments");
  return samples_norms((hipStream_t)stream, st, b, R, norms, G, L22, flags, PT);
}

long long evr_qnehvi_project_backward_workspace_doubles(const evr_qnehvi_state* st, int b) {
  return (st && b > 0) ? (long long)proj_backward_ws_doubles(st, b) : 0;
}

int evr_qnehvi_project_backward(void* stream, const evr_qnehvi_state* st, int b, const double* Mm, const double* R,
                                const double* L22, const double* dG, double* dKx, double* work) {
  EVR_CHECK(st && Mm && R && L22 && dG && dKx && b >= 0, "evr_qnehvi_project_backward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool own = !work;
  if (own) EVR_HIP(hipMallocAsync((void**)&work, sizeof(double) * proj_backward_ws_doubles(st, b), s));
  const int rc = proj_backward(s, st, b, Mm, R, L22, dG, dKx, work);
  if (own) EVR_HIP(hipFreeAsync(work, s));
  return rc;
}

}  // extern "C"
