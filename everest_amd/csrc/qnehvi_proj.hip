// qNEHVI projection GEMMs with fused prologue / epilogue (gfx950 f64 MFMA, the
// gemm_core.hpp tile engine), the candidate-batch path (b > 32: raw screening, evaluation
// passes, joint batches; b <= 32 is qnehvi_small.hip).
//
// Forward:  R_j = M_j K_x  (M_j = [C_j; H_j^T; alpha_j^T] or [L^-1; G; H^T; alpha^T], Rr x n;
// K_x: n x b), as in acquisition.py.  All Rr rows, the mean row included, in one launch of
// 32 x 64 tiles.  The epilogue also emits, per 32-row tile and candidate, the partial sums of
// squares of the L^-1 k rows (rows < n) and of the L21 rows (n <= row < n + nb), so the
// sampling step reads (row tiles x 2) partials and the S + 1 sample / mean rows instead of
// the whole R.
//
// Backward: dK_x,j = M_j^T gR_j with gR_j never materialised.  gR_j is, per candidate c,
//   rows < n:            2 R[i][c] dssv(c)      (var = s^2 (kxx - |L^-1 k|^2))
//   n <= rows < n + nb:  2 R[i][c] dssw(c)      (L22^2 = var - |L21|^2)
//   sample rows s:       a_j dG[s][j][c]
//   mean row:            s_j dmu(c),  dmu = sum_s a_j dG, dl = sum_s a_j dG zq[s][j],
//                        dbr = dl / (2 L22), dssv = -s^2 dbr, dssw = -dbr.
// A small kernel reduces dmu, dl over the samples into per-candidate coefficients; the GEMM's
// B fetch then generates gR from R, dG and those coefficients — one pass over R and dG.
// Both GEMMs split K (fixed-order reduction) when their tile grid cannot fill the chip.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "gemm_core.hpp"
#include "../../include/everest_amd.h"

namespace evr {

using ProjF = DgCfg<32, 64, 16, false>;   // R = M K_x          (A = M: k-contiguous rows)
using ProjB = DgCfg<32, 32, 16, true>;    // dK_x = M^T gR      (A = M^T: m-contiguous)
constexpr int QN_NT = ProjF::BM;          // rows per partial-norm tile

int dg_ksplit(long long tiles, int K, int bk, int* kchunk);

// partial sums of squares of a BM x BN tile of R by row class (cls 0: rows < n, 1: rows in
// [n, n + nb)), reduced over the tile's rows in a fixed order -> Pout[cls][c] (b columns)
template <class C>
__device__ __forceinline__ void proj_tile_norms(const dg_double4 (&acc)[C::FM][C::FN], double* lds, int m0, int n0,
                                                int n, int nb, int b, double* __restrict__ Pout) {
  static_assert(C::FM == 1, "one 16-row block per wave");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, i = lane & 15, q = lane >> 4;
  double sq[C::FN][2];
#pragma unroll
  for (int bb = 0; bb < C::FN; ++bb) {
    sq[bb][0] = sq[bb][1] = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * C::WM + q + 4 * r;
      const double v = acc[0][bb][r];
      if (row < n) sq[bb][0] = fma(v, v, sq[bb][0]);
      else if (row < n + nb) sq[bb][1] = fma(v, v, sq[bb][1]);
    }
#pragma unroll
    for (int cls = 0; cls < 2; ++cls) {
      double v = sq[bb][cls];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      sq[bb][cls] = v;
    }
  }
  // the mainloop ended on a barrier: its LDS is free
  double (*red)[C::BN][2] = reinterpret_cast<double (*)[C::BN][2]>(lds);
  if (q == 0) {
#pragma unroll
    for (int bb = 0; bb < C::FN; ++bb) {
      red[wr][wc * C::WN + bb * 16 + i][0] = sq[bb][0];
      red[wr][wc * C::WN + bb * 16 + i][1] = sq[bb][1];
    }
  }
  __syncthreads();
  if (tid < 2 * C::BN) {
    const int cls = tid / C::BN, c = tid - cls * C::BN;
    const double v = red[0][c][cls] + red[1][c][cls];
    if (n0 + c < b) Pout[(size_t)cls * b + n0 + c] = v;
  }
}

// ---------------------------------------------------------------------------------------
// forward: R_j = M_j K_x,j (+ partial norms), optional split-K into W
// ---------------------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256, 4) void qn_proj_fwd(int n, int nb, int Rr, int b, int m, const double* __restrict__ Mm,
                                                      const double* __restrict__ Kx, double* __restrict__ R,
                                                      double* __restrict__ P, int nrt, int ksplit, int kchunk,
                                                      double* __restrict__ W) {
  using C = ProjF;
  __shared__ double lds[C::LDS_DOUBLES];
  const int gx = gridDim.x, gy = gridDim.y;
  const int t = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int bx = t % gx, by = (t / gx) % gy, bz = t / (gx * gy);
  const int j = bz / ksplit, kz = bz - j * ksplit;
  const int m0 = by * C::BM, n0 = bx * C::BN;
  const double* A = Mm + (size_t)j * Rr * n;
  const double* B = Kx + (size_t)j * n * b;
  // split root (nb > 0): rows r < n of M are L^-1's, lower triangular, so a row tile below n
  // contracts over k < m0 + BM only (the skipped k-steps are exact zeros, whole 16-steps at
  // the same chain positions: bitwise unchanged)
  const int kend = min(nb > 0 && m0 + C::BM <= n ? m0 + C::BM : n, kz * kchunk + kchunk), kbeg = kz * kchunk;
  dg_double4 acc[C::FM][C::FN];
  dg_mainloop<C>(
      lds, kbeg, kend,
      [&](int r, int k) -> dg_double2 {
        const bool ok = m0 + r < Rr;
        return dg_pair<VEC>(A + (size_t)(m0 + r) * n + k, ok && k < kend, ok && k + 1 < kend);
      },
      [&](int k, int c) -> dg_double2 {
        const bool ok = k < kend;
        return dg_pair<VEC>(B + (size_t)k * b + n0 + c, ok && n0 + c < b, ok && n0 + c + 1 < b);
      },
      acc);
  if (ksplit > 1) {
    double* Wz = W + ((size_t)kz * m + j) * Rr * b;
    dg_for_each<C>(acc, [&](int r, int c, double val) {
      if (m0 + r < Rr && n0 + c < b) Wz[(size_t)(m0 + r) * b + n0 + c] = val;
    });
    return;
  }
  double* Rj = R + (size_t)j * Rr * b;
  dg_for_each<C>(acc, [&](int r, int c, double val) {
    if (m0 + r < Rr && n0 + c < b) Rj[(size_t)(m0 + r) * b + n0 + c] = val;
  });
  proj_tile_norms<C>(acc, lds, m0, n0, n, nb, b, P + ((size_t)j * nrt + by) * 2 * b);
}

// split-K reduction of the forward: R = sum_kz W[kz] (fixed order), then the partial norms of
// each 32-row tile (thread per candidate column, rows in order)
__global__ __launch_bounds__(256) void qn_proj_fwd_reduce(int n, int nb, int Rr, int b, int m, int ksplit,
                                                          const double* __restrict__ W, double* __restrict__ R,
                                                          double* __restrict__ P, int nrt) {
  const int j = blockIdx.z, rt = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= b) return;
  double s0 = 0.0, s1 = 0.0;
  double* Rj = R + (size_t)j * Rr * b;
  for (int rr = 0; rr < QN_NT; ++rr) {
    const int row = rt * QN_NT + rr;
    if (row >= Rr) break;
    double v = 0.0;
    for (int kz = 0; kz < ksplit; ++kz) v += W[(((size_t)kz * m + j) * Rr + row) * b + c];
    Rj[(size_t)row * b + c] = v;
    if (row < n) s0 = fma(v, v, s0);
    else if (row < n + nb) s1 = fma(v, v, s1);
  }
  P[(((size_t)j * nrt + rt) * 2 + 0) * b + c] = s0;
  P[(((size_t)j * nrt + rt) * 2 + 1) * b + c] = s1;
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
// backward: dKx_j = M_j^T gR_j, gR never formed.  Its row classes scale whole columns
// (rows < n by 2 dssv(c), rows [n, n + nb) by 2 dssw(c), sample rows by a_j, the mean row is
// s_j dmu(c) itself), and a column scale commutes with the sum over rows: each class's rows
// are one plain GEMM segment over R / dG (the tile engine's main loop, no per-element work
// in the fetch), scaled in the epilogue, where the mean row's rank-1 term is added.
// Optional split-K into W (the classes intersected with the slice's k range).
// ---------------------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256, 4) void qn_proj_bwd(int n, int nb, int nh, int m, int b, const double* __restrict__ Mm,
                                                      const double* __restrict__ R, const double* __restrict__ dG,
                                                      const double* __restrict__ oa, const double* __restrict__ coef,
                                                      double* __restrict__ dK, int ksplit, int kchunk,
                                                      double* __restrict__ W) {
  using C = ProjB;
  __shared__ double lds[C::LDS_DOUBLES];
  const int gx = gridDim.x, gy = gridDim.y;
  const int t = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int bx = t % gx, by = (t / gx) % gy, bz = t / (gx * gy);
  const int j = bz / ksplit, kz = bz - j * ksplit;
  const int m0 = by * C::BM, n0 = bx * C::BN;
  const int Rr = n + nb + nh + 1;
  const double* A = Mm + (size_t)j * Rr * n;   // A(row, k) = M_j[k][row]
  const double* Rj = R + (size_t)j * Rr * b;
  const double* dGj = dG + (size_t)j * b;
  const double* cj = coef + (size_t)j * 3 * b;
  const double aj = oa[j];
  const int kbeg = kz * kchunk, kend = min(Rr, kbeg + kchunk);
  auto fa = [&](int k, int c) -> dg_double2 {
    return dg_pair<VEC>(A + (size_t)k * n + m0 + c, m0 + c < n, m0 + c + 1 < n);
  };
  // class segments of this slice: [lo, hi) of rows < n, [n, n + nb), the sample rows
  dg_double4 a0[C::FM][C::FN], a1[C::FM][C::FN], a2[C::FM][C::FN];
  {
    // split root: M[k][i] = L^-1[k][i] = 0 for k < i, so output rows i >= m0 start at k = m0
    // (m0 a multiple of the 16-deep k-step: the same chain positions, bitwise unchanged)
    const int lo = nb > 0 ? max(kbeg, m0) : kbeg, hi = min(kend, n);
    dg_mainloop<C>(lds, lo, hi, fa, [&](int k, int c) -> dg_double2 {
      return dg_pair<VEC>(Rj + (size_t)k * b + n0 + c, k < hi && n0 + c < b, k < hi && n0 + c + 1 < b);
    }, a0);
  }
  {
    const int lo = max(kbeg, n), hi = min(kend, n + nb);
    dg_mainloop<C>(lds, lo, hi, fa, [&](int k, int c) -> dg_double2 {
      return dg_pair<VEC>(Rj + (size_t)k * b + n0 + c, k < hi && n0 + c < b, k < hi && n0 + c + 1 < b);
    }, a1);
  }
  {
    const int lo = max(kbeg, n + nb), hi = min(kend, n + nb + nh);
    dg_mainloop<C>(lds, lo, hi, fa, [&](int k, int c) -> dg_double2 {
      return dg_pair<VEC>(dGj + (size_t)(k - n - nb) * m * b + n0 + c, k < hi && n0 + c < b, k < hi && n0 + c + 1 < b);
    }, a2);
  }
  const bool mean_in = Rr - 1 >= kbeg && Rr - 1 < kend;
  const double* Mmean = A + (size_t)(Rr - 1) * n;
  double* out = (ksplit > 1) ? W + ((size_t)kz * m + j) * n * b : dK + (size_t)j * n * b;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * C::WM, wn = (wave & 1) * C::WN, i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int x = 0; x < C::FM; ++x)
#pragma unroll
    for (int y = 0; y < C::FN; ++y) {
      const int col = n0 + wn + y * 16 + i;
      const bool cok = col < b;
      const double k0c = cok ? cj[col] : 0.0, k1c = cok ? cj[(size_t)b + col] : 0.0;
      const double k2c = cok ? cj[(size_t)2 * b + col] : 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + x * 16 + q + 4 * r;
        if (row < n && cok) {
          double v = fma(k0c, a0[x][y][r], fma(k1c, a1[x][y][r], aj * a2[x][y][r]));
          if (mean_in) v = fma(Mmean[row], k2c, v);
          out[(size_t)row * b + col] = v;
        }
      }
    }
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

static bool proj_vec(const evr_qnehvi_state* st, int b) { return st->n % 2 == 0 && b % 2 == 0; }

// ---- internal launchers (workspace supplied by the caller; qnehvi_plan.hip) ----------
size_t proj_forward_ws_doubles(const evr_qnehvi_state* st, int b) {
  const int Rr = qn_rows(st);
  int kchunk = 0;
  const int ks = dg_ksplit((long long)cdiv(b, ProjF::BN) * cdiv(Rr, ProjF::BM) * st->m, st->n, ProjF::BK, &kchunk);
  return ks > 1 ? (size_t)ks * st->m * Rr * b : 0;
}

int proj_forward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* Kx, double* R,
                 double* norms, double* W) {
  if (b == 0) return 0;
  const int Rr = qn_rows(st);
  const int nrt = cdiv(Rr, QN_NT);
  int kchunk = 0;
  const int ks = dg_ksplit((long long)cdiv(b, ProjF::BN) * nrt * st->m, st->n, ProjF::BK, &kchunk);
  EVR_CHECK(ks == 1 || W, "proj_forward: split-K workspace missing");
  dim3 grid(cdiv(b, ProjF::BN), nrt, st->m * ks);
  if (proj_vec(st, b))
    qn_proj_fwd<true><<<grid, 256, 0, s>>>(st->n, st->nb, Rr, b, st->m, Mm, Kx, R, norms, nrt, ks, kchunk, W);
  else
    qn_proj_fwd<false><<<grid, 256, 0, s>>>(st->n, st->nb, Rr, b, st->m, Mm, Kx, R, norms, nrt, ks, kchunk, W);
  EVR_LAUNCH_CHECK();
  if (ks > 1) {
    qn_proj_fwd_reduce<<<dim3(cdiv(b, 256), nrt, st->m), 256, 0, s>>>(st->n, st->nb, Rr, b, st->m, ks, W, R, norms,
                                                                        nrt);
    EVR_LAUNCH_CHECK();
  }
  return 0;
}

size_t proj_backward_ws_doubles(const evr_qnehvi_state* st, int b) {
  const int Rr = qn_rows(st);
  int kchunk = 0;
  const int ks = dg_ksplit((long long)cdiv(b, ProjB::BN) * cdiv(st->n, ProjB::BM) * st->m, Rr, ProjB::BK, &kchunk);
  return (size_t)st->m * 3 * b + (ks > 1 ? (size_t)ks * st->m * st->n * b : 0);
}

int proj_backward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* R,
                  const double* L22, const double* dG, double* dKx, double* ws) {
  if (b == 0) return 0;
  const int Rr = qn_rows(st);
  double* coef = ws;
  qn_bwd_coef<<<dim3(cdiv(b, BC_C), st->m), BC_C * BC_G, 0, s>>>(st->S, st->m, b, dG, L22, st->ys, st->zq, st->obj_a, coef);
  EVR_LAUNCH_CHECK();
  int kchunk = 0;
  const int ks = dg_ksplit((long long)cdiv(b, ProjB::BN) * cdiv(st->n, ProjB::BM) * st->m, Rr, ProjB::BK, &kchunk);
  double* W = ws + (size_t)st->m * 3 * b;
  dim3 grid(cdiv(b, ProjB::BN), cdiv(st->n, ProjB::BM), st->m * ks);
  if (proj_vec(st, b))
    qn_proj_bwd<true><<<grid, 256, 0, s>>>(st->n, st->nb, qn_nh(st), st->m, b, Mm, R, dG, st->obj_a, coef, dKx, ks,
                                           kchunk, W);
  else
    qn_proj_bwd<false><<<grid, 256, 0, s>>>(st->n, st->nb, qn_nh(st), st->m, b, Mm, R, dG, st->obj_a, coef, dKx, ks,
                                            kchunk, W);
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
  return cdiv((long long)qn_rows(st), QN_NT);
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
  return samples_norms((hipStream_t)stream, st, b, R, norms, G, L22, flags, QN_NT);
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
