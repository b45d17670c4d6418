// Small-batch (b <= 32) projections of the qNEHVI evaluation chain — the L-BFGS-B restart
// batch of ask() (BoFire: num_restarts candidates per optimiser evaluation,
// bofire/strategies/predictives/botorch.py:384-405; 20 in BASELINE configs[3]).
//
// At b = 20 the operator M (m x Rr x n, 15.7 MB at the bench shape) is the only large
// operand: both GEMMs are HBM streams over M with a 20-column right-hand side, not
// MFMA-bound contractions.  The 64 x 64-tile paths (rocBLAS forward, split-K MFMA backward)
// spent 19 + 25 us there plus five helper launches (mean row, norms, gR coefficients,
// split-K sum, cross-gradient reduction).  Here:
//   qs_fwd:  one workgroup per (16 rows of M_j, output j): K_x (kmat_kernel, once per
//            output: computing it inside every row tile costs 49x the f64 exp) staged in LDS
//            in 128-row chunks (two workgroups per CU: the m x 66 row tiles of the bench shape
//            are resident at once), v_mfma_f64_16x16x4 with a per-lane contiguous 128 B slice of each M row
//            (the contraction index is permuted per lane, identically in A and B), the four
//            waves' k-quarters reduced in a fixed order; epilogue writes R and the per-tile
//            partial sums of squares the sampling kernel reads.
//   qs_bwd:  one workgroup per (16 columns of M_j, output j): the gR coefficients (reduced
//            over the S samples in a fixed order), gR generated in the B fetch from R, dG and
//            the coefficients, dK_x = M_j^T gR by MFMA, and in the epilogue the cross-
//            covariance gradient of the tile's 16 training rows (dK_x never reaches HBM).
//   qs_dx_reduce: dX = sum over the (output, tile) partials in a fixed order.
// Every reduction order is fixed: results are bitwise reproducible.
#include <algorithm>

#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "qs_tail.hpp"
#include "../../include/everest_amd.h"

using double4_t = __attribute__((ext_vector_type(4))) double;

namespace evr {

constexpr int QS_B = 32;     // max candidates
constexpr int QS_FR = 16;    // rows of M per forward workgroup
constexpr int QS_KC = 128;   // K_x rows staged per chunk (~67 KB of LDS: two workgroups per CU)
constexpr int QS_BI = 16;    // columns of M (training rows) per backward workgroup
constexpr int QS_MAXD = 8;   // input dims handled in registers by the backward epilogue

__device__ __forceinline__ double4_t mfma4(double a, double b, double4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

#ifdef EVR_QS_PROF
// tools/qs_prof.hip: per-workgroup wall-clock stamps of qs_fwd / qs_bwd (s_memrealtime, 10 ns)
__device__ unsigned long long qs_prof[4096 * 8];
#define QS_STAMP(k) do { if (threadIdx.x == 0) qs_prof[(size_t)qs_bid * 8 + (k)] = wall_clock64(); } while (0)
#else
#define QS_STAMP(k) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------
// forward: R_j[r0 .. r0+15][c] = sum_k M_j[r][k] Kx_j[k][c]; P[j][tile][cls][c] partial norms.
// QS_FT = 512 threads (8 waves) per workgroup: at the bench shape the grid is m x Rr / 16 =
// 245 workgroups, fewer than the 256 CUs, so the waves of one workgroup are all the latency
// hiding a CU gets (4 waves: 10.4 us; each wave's chunk work halves with 8).
// ---------------------------------------------------------------------------------------
constexpr int QS_FT = 512;
constexpr int QS_FW = QS_FT / 64;                 // waves
constexpr int QS_RPP = QS_FT / QS_KC;             // M rows per staging pass (a thread per chunk column)
constexpr int QS_ML = QS_FR / QS_RPP;             // M values per thread and chunk
constexpr int QS_KL = (QS_KC * QS_B + QS_FT - 1) / QS_FT;   // K_x values per thread and chunk
// Two workgroups per CU (50 KB of LDS; four waves per SIMD: <= 128 VGPRs): the split root's m x 66 row tiles
// (330 workgroups) are resident in one round like the fused root's m x 49.
__global__ __launch_bounds__(QS_FT, 4) void qs_fwd(int n, int nb, int Rr, int b, const double* __restrict__ M,
                                                   const double* __restrict__ Kx, double* __restrict__ R,
                                                   double* __restrict__ P, int ntile) {
  // padded row of the staged M tile: 2 MP = 4 (mod 64 dwords) puts the 16 rows x 2
  // k-quarters of a ds_read_b64 lane half on 32 distinct bank pairs (conflict-free)
  constexpr int MP = QS_KC + 2;
  constexpr int MS_SZ = QS_FR * MP, KS_SZ = QS_KC * (QS_B + 1), RED_SZ = QS_FW * QS_FR * (QS_B + 1);
  static_assert(RED_SZ <= MS_SZ + KS_SZ, "the k-partials alias the chunk tiles");
  __shared__ double lds[MS_SZ + KS_SZ];
  auto Ms = reinterpret_cast<double(*)[MP]>(lds);                      // 16 x 128 slice of M_j (16.6 KB)
  auto Ks = reinterpret_cast<double(*)[QS_B + 1]>(lds + MS_SZ);        // 128 x b slice of K_x,j (33.8 KB)
  auto red = reinterpret_cast<double(*)[QS_FR][QS_B + 1]>(lds);       // the waves' k-partials (after the loop)
  const int tile = blockIdx.x, j = blockIdx.y, r0 = tile * QS_FR;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, kq = lane >> 4;
  const double* Mj = M + (size_t)j * Rr * n;
  const double* Kj = Kx + (size_t)j * n * b;
#ifdef EVR_QS_PROF
  const int qs_bid = 2048 + blockIdx.y * gridDim.x + blockIdx.x;   // after qs_bwd's records
#endif
  QS_STAMP(0);
  double4_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  // coalesced chunk loads into registers (a wave reads 512 contiguous bytes of one M row per
  // instruction; the chunk's K_x rows are one contiguous run of kn x b doubles), staged in
  // LDS afterwards; two register buffers, so the loads of chunks k + 1 and k + 2 are in flight
  // while chunk k is staged and multiplied (the K_x values past b x kn are never loaded).
  // K_x rows past the end of a partial chunk are zero (M's are too, but 0 x garbage is not 0).
  double mvA[QS_ML], kvA[QS_KL], mvB[QS_ML], kvB[QS_KL];
  const int kk = tid % QS_KC, rh = tid / QS_KC;   // staging: chunk column kk of rows rh, rh + RPP, ...
  auto load = [&](double (&mv)[QS_ML], double (&kv)[QS_KL], int kc) {
    const int kn = min(QS_KC, n - kc);
#pragma unroll
    for (int u = 0; u < QS_ML; ++u) {
      const int r = r0 + QS_RPP * u + rh;
      mv[u] = (r < Rr && kk < kn) ? Mj[(size_t)r * n + kc + kk] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < QS_KL; ++u) {
      const int e = u * QS_FT + tid;
      kv[u] = (e < kn * b) ? Kj[(size_t)kc * b + e] : 0.0;
    }
  };
  auto stage = [&](const double (&mv)[QS_ML], const double (&kv)[QS_KL]) {
#pragma unroll
    for (int u = 0; u < QS_ML; ++u) Ms[QS_RPP * u + rh][kk] = mv[u];
    // element e = u QS_FT + tid of the chunk's row-major run -> (e / b, e % b), stepped per u
    // (no per-element division: it kept 2 QS_KL index registers alive)
    int kr = tid / b, kc_ = tid - kr * b;
    const int dq = QS_FT / b, dr = QS_FT - dq * b;
#pragma unroll
    for (int u = 0; u < QS_KL; ++u) {
      if (u * QS_FT + tid < QS_KC * b) Ks[kr][kc_] = kv[u];   // every row of the chunk, columns < b
      kr += dq;
      kc_ += dr;
      if (kc_ >= b) {
        kc_ -= b;
        ++kr;
      }
    }
  };
  constexpr int KW = QS_KC / QS_FW;   // k per wave and chunk
  auto mult = [&]() {
#pragma unroll
    for (int t = 0; t < KW / 4; ++t) {
      const int k = wave * KW + 4 * t + kq;
      const double a = Ms[i][k];
      // columns >= b of Ks are never written: they only reach D's columns >= b (not stored)
      acc0 = mfma4(a, Ks[k][i], acc0);
      acc1 = mfma4(a, Ks[k][i + 16], acc1);
    }
  };
  // split root (nb > 0): rows r < n are L^-1's, lower triangular — the tile's rows reach
  // column r0 + 15 at most, so the chunks past it are exact zeros and are skipped
  const int kend = (nb > 0 && r0 < n) ? min(n, r0 + QS_FR) : n;
  load(mvA, kvA, 0);
  if (QS_KC < kend) load(mvB, kvB, QS_KC);
  for (int kc = 0; kc < kend; kc += 2 * QS_KC) {
    __syncthreads();   // the previous chunk's MFMAs are done with Ms, Ks
    stage(mvA, kvA);
    __syncthreads();
    if (kc == 0) QS_STAMP(1);
    if (kc + 2 * QS_KC < kend) load(mvA, kvA, kc + 2 * QS_KC);
    mult();
    if (kc + QS_KC >= kend) break;
    __syncthreads();
    stage(mvB, kvB);
    __syncthreads();
    if (kc + 3 * QS_KC < kend) load(mvB, kvB, kc + 3 * QS_KC);
    mult();
  }
  QS_STAMP(2);
  __syncthreads();   // every wave is done with Ms, Ks (red aliases them)
  // D map of v_mfma_f64_16x16x4: register q of lane l holds D[4q + (l >> 4)][l & 15]
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[wave][4 * q + kq][i] = acc0[q];
    red[wave][4 * q + kq][16 + i] = acc1[q];
  }
  __syncthreads();
  {
    const int rr = tid >> 5, c = tid & 31;   // one (row, column) per thread
    double v = red[0][rr][c];
#pragma unroll
    for (int w = 1; w < QS_FW; ++w) v += red[w][rr][c];
    if (r0 + rr < Rr && c < b) R[((size_t)j * Rr + r0 + rr) * b + c] = v;
    __syncthreads();
    red[0][rr][c] = v;
  }
  __syncthreads();
  if (tid < 2 * QS_B) {
    const int cls = tid / QS_B, c = tid - cls * QS_B;
    double s = 0.0;
#pragma unroll
    for (int rr = 0; rr < QS_FR; ++rr) {
      const int r = r0 + rr;
      const bool in = cls == 0 ? r < n : (r >= n && r < n + nb);
      if (in) s = fma(red[0][rr][c], red[0][rr][c], s);
    }
    if (c < b) P[(((size_t)j * ntile + tile) * 2 + cls) * b + c] = s;
  }
  QS_STAMP(3);
}

// ---------------------------------------------------------------------------------------
// backward: per (16 training rows i0.., output j): coefficients, dK_x tile = M_j^T gR (MFMA),
// cross-covariance gradient partial dXp[c][k][(j, z, tile)].  gR rows come from R (rows
// < n + nb, times the per-candidate coefficients), a_j dG (sample rows) or the coefficient
// itself (mean row); the chunk of 128 rows of M (16 columns) and of the gR sources is loaded
// with coalesced row segments.  The per-candidate coefficients scale whole row classes, so
// each class is summed apart and scaled in the epilogue, and the coefficients' own reduction
// over the samples overlaps the chunk loop.
// ---------------------------------------------------------------------------------------
constexpr int QS_RC = 128;   // rows of M per backward chunk

// (256, 2): two waves per SIMD, i.e. two workgroups per CU — without the bound the compiler
// took 244 VGPRs + 16 AGPRs (one workgroup per CU: the 480 workgroups of the bench shape ran
// in two rounds); bounded it fits 248 registers without scratch
constexpr int QS_SMAX = 1024;   // samples whose z values the backward stages in LDS
// The training-row classes (rows < n + nb) are the launch's z >= zsb workgroups (qs_tail.hpp):
// the sample-row workgroups (z < zsb) cover the S sample rows only, and the classes'
// coefficient goes to cfo[j][c] for the dX reduction (written by the (tile 0, split 0)
// workgroup of each output)
__global__ __launch_bounds__(256, 2) void qs_bwd(int n, int nb, int nh, int S, int m, int b, int d, int kind,
                                              const double* __restrict__ M, const double* __restrict__ R,
                                              const double* __restrict__ dG, const double* __restrict__ L22,
                                              const double* __restrict__ ys, const double* __restrict__ zq,
                                              const double* __restrict__ oa, const double* __restrict__ Xn,
                                              const double* __restrict__ X, const double* __restrict__ shift,
                                              const double* __restrict__ scale, const double* __restrict__ ls,
                                              double* __restrict__ dXp, int ntile, int rows_per, int np_all,
                                              double* __restrict__ cfo, int zsb, QsTail qtl) {
  __shared__ double cf[3][QS_B];   // [2]: the mean row's coefficient (0, 1 unused)
  __shared__ double red[8][QS_B][2];
  __shared__ double zl[QS_SMAX];   // z_j of the samples (the coefficient rounds read them here)
  // the chunk tiles and the epilogue's reduction buffers share one LDS region (~53 KB per
  // workgroup, two resident per CU)
  constexpr int MS_SZ = QS_RC * (QS_BI + 1), BS_SZ = QS_RC * (QS_B + 1);
  constexpr int DK_SZ = 4 * QS_BI * (QS_B + 1), GX_SZ = 8 * QS_B * QS_MAXD;
  static_assert(DK_SZ + GX_SZ <= MS_SZ + BS_SZ, "epilogue buffers alias the chunk tiles");
  __shared__ double lds[MS_SZ + BS_SZ];
  auto Ms = reinterpret_cast<double(*)[QS_BI + 1]>(lds);
  auto Bs = reinterpret_cast<double(*)[QS_B + 1]>(lds + MS_SZ);
  auto dk = reinterpret_cast<double(*)[QS_BI][QS_B + 1]>(lds);
  auto gx = reinterpret_cast<double(*)[QS_B][QS_MAXD]>(lds + DK_SZ);
  if ((int)blockIdx.z >= zsb) {   // the training-row classes: their own workgroups
    qs_tail_tile(qtl, ((int)blockIdx.y * qtl.za + ((int)blockIdx.z - zsb)) * qtl.nt + blockIdx.x, lds);
    return;
  }
  const int tile = blockIdx.x, j = blockIdx.y, z = blockIdx.z, i0 = tile * QS_BI;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Rr = n + nb + nh + 1;
#ifdef EVR_QS_PROF
  const int qs_bid = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
#endif
  QS_STAMP(0);
  // this split's rows of M; the mean row (Rr - 1, a rank-1 term) is added in the epilogue
  const int rbeg = n + nb + z * rows_per, rend = min(Rr - 1, rbeg + rows_per);
  const double aj = oa[j], sj = ys[j];
  const double* Mj = M + (size_t)j * Rr * n;
  // the epilogue's candidate coordinates (normalised) and inverse lengthscales, loaded first:
  // X may be the plan's pinned host buffer (PCIe latency, hidden behind the main loop)
  double xc[QS_MAXD];
  {
    const int c = tid & (QS_B - 1);
#pragma unroll
    for (int k = 0; k < QS_MAXD; ++k)
      xc[k] = (c < b && k < d) ? (X[(size_t)c * d + k] - (shift ? shift[k] : 0.0)) * (scale ? scale[k] : 1.0) : 0.0;
  }
  // chunk loads: M[r][i0 + col] (a wave covers 4 rows x 128 B), gR source (row, candidate)
  constexpr int ML = QS_RC * QS_BI / 256, BL = QS_RC * QS_B / 256;
  double mv[ML], bv[BL];
  auto load = [&](int rc) {
#pragma unroll
    for (int u = 0; u < ML; ++u) {
      const int e = u * 256 + tid, rr = e / QS_BI, cc = e % QS_BI, r = rc + rr;
      mv[u] = (r < rend && i0 + cc < n) ? Mj[(size_t)r * n + i0 + cc] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < BL; ++u) {
      const int e = u * 256 + tid, rr = e / QS_B, c = e % QS_B, r = rc + rr;
      bv[u] = (c < b && r < rend) ? dG[((size_t)(r - n - nb) * m + j) * b + c] : 0.0;
    }
  };
  // z_j of the samples, loaded first (the LDS store below then waits for these loads only:
  // vmcnt retires in issue order, and the chunk / coefficient loads are issued after them)
  double zr[QS_SMAX / 256];
#pragma unroll
  for (int u = 0; u < QS_SMAX / 256; ++u) {
    const int e = tid + 256 * u;
    zr[u] = e < S ? zq[(size_t)e * m + j] : 0.0;
  }
  load(rbeg);
  // 1. gR coefficients of this output (qn_bwd_coef's algebra): dmu = sum_s a dG, dl = sum_s a dG z,
  //    thread (candidate c, sample group g of 8), rounds of 16 samples summed in sample order.
  //    They scale only whole row classes of gR, so they are applied to the class sums in the
  //    epilogue: the rounds' loads ride along with the chunk loads below (round k is consumed
  //    after chunk k's MFMAs) instead of standing before the first chunk.
  const int cc_ = tid & (QS_B - 1), g_ = tid >> 5;
  constexpr int CU = 12;   // samples per thread and round: the most that stay in registers
  double dmu = 0.0, dl = 0.0;
  double dv[CU];
  int s0 = g_;
  auto coef_load = [&]() {
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const int s = s0 + 8 * u;
      dv[u] = (cc_ < b && s < S) ? dG[((size_t)s * m + j) * b + cc_] : 0.0;
    }
  };
  auto coef_acc = [&]() {
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const int s = s0 + 8 * u;
      const double dy = aj * dv[u];
      dmu += dy;
      dl = fma(dy, s < S ? zl[s] : 0.0, dl);
    }
    s0 += 8 * CU;
  };
  // with the sample rows in M (nh = S, one split over all of them) the coefficients are summed
  // from the staged chunks in LDS (Bs holds a_j dG of the chunk's samples) in the same
  // per-thread sample order — no separate dG loads or their dependent rounds
  const bool coef_lds = nh == S && zsb == 1;
  bool pend = !coef_lds && s0 < S;
  if (pend) coef_load();
#pragma unroll
  for (int u = 0; u < QS_SMAX / 256; ++u) {   // visible after the first chunk's barrier
    const int e = tid + 256 * u;
    if (e < S) zl[e] = zr[u];
  }
  QS_STAMP(1);
  // 2. dK tile over the sample rows (a_j applied while staging): D[i][c] = sum_r M[r][i0 + i] a_j dG[r][c]
  const int i = lane & 15, kq = lane >> 4;
  double4_t aB0 = {0, 0, 0, 0}, aB1 = {0, 0, 0, 0};
  for (int rc = rbeg; rc < rend; rc += QS_RC) {
    __syncthreads();   // the previous chunk's MFMAs are done with Ms, Bs
#pragma unroll
    for (int u = 0; u < ML; ++u) {
      const int e = u * 256 + tid;
      Ms[e / QS_BI][e % QS_BI] = mv[u];
    }
#pragma unroll
    for (int u = 0; u < BL; ++u) {
      const int e = u * 256 + tid, rr = e / QS_B, c = e % QS_B;
      Bs[rr][c] = bv[u] * aj;
    }
    __syncthreads();
    if (rc + QS_RC < rend) load(rc + QS_RC);
#pragma unroll
    for (int t = 0; t < QS_RC / 16; ++t) {
      const int rr = wave * (QS_RC / 4) + 4 * t + kq;
      const double a = Ms[rr][i];
      aB0 = mfma4(a, Bs[rr][i], aB0);
      aB1 = mfma4(a, Bs[rr][i + 16], aB1);
    }
    if (coef_lds) {
#pragma unroll
      for (int v = 0; v < QS_RC / 8; ++v) {
        const int rr = g_ + 8 * v, sidx = rc + rr - n - nb;
        if (sidx < S) {
          const double dy = Bs[rr][cc_];
          dmu += dy;
          dl = fma(dy, zl[sidx], dl);
        }
      }
    }
    if (pend) {   // the coefficient round issued with this chunk's loads
      coef_acc();
      pend = s0 < S;
      if (pend) coef_load();
    }
  }
  while (pend) {
    coef_acc();
    pend = s0 < S;
    if (pend) coef_load();
  }
  red[g_][cc_][0] = dmu;
  red[g_][cc_][1] = dl;
  __syncthreads();
  if (tid < QS_B) {
    double u = red[0][tid][0], v = red[0][tid][1];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      u += red[q][tid][0];
      v += red[q][tid][1];
    }
    const double dbr = tid < b ? v / (2.0 * L22[(size_t)j * b + tid]) : 0.0;
    cf[2][tid] = sj * u;
    // the training-row classes' coefficient: -2 dbr with the split root (its L^-1 rows carry
    // s^2 in the tail's weights), -2 s^2 dbr with the fused one
    if (tile == 0 && z == 0 && tid < b) cfo[(size_t)j * b + tid] = nb > 0 ? -2.0 * dbr : -2.0 * sj * sj * dbr;
  }
  QS_STAMP(2);
  // the epilogue's training rows and mean-row entries, loaded before the dk exchange so their
  // latency overlaps it: thread (candidate c, row group g) uses rows i0 + g and i0 + g + 8
  double xr[2][QS_MAXD], mrow[2];
  {
    const int g = tid >> 5;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int irow = i0 + g + 8 * h;
      const bool in = irow < n;
#pragma unroll
      for (int k = 0; k < QS_MAXD; ++k) xr[h][k] = (in && k < d) ? Xn[(size_t)irow * d + k] : 0.0;
      mrow[h] = (in && z == 0) ? Mj[(size_t)(Rr - 1) * n + irow] : 0.0;
    }
  }
  __syncthreads();   // all waves are done with Ms, Bs (dk aliases them); cf is ready
  {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      dk[wave][4 * q + kq][i] = aB0[q];
      dk[wave][4 * q + kq][16 + i] = aB1[q];
    }
  }
  __syncthreads();
  QS_STAMP(3);
  // 3. cross-covariance gradient of the tile's rows: thread (candidate c, row group g of 8),
  //    rows i0 + g and i0 + g + 8; dX_c += dK[i][c] dk(x_i, x_c)/dx_c (normalized units)
  {
    const int c = tid & (QS_B - 1), g = tid >> 5;
    double acc[QS_MAXD];
#pragma unroll
    for (int k = 0; k < QS_MAXD; ++k) acc[k] = 0.0;
    if (c < b) {
      double il[QS_MAXD];
#pragma unroll
      for (int k = 0; k < QS_MAXD; ++k) il[k] = k < d ? 1.0 / ls[(size_t)j * d + k] : 0.0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ii = g + 8 * h, irow = i0 + ii;
        if (irow >= n) continue;
        double gk = ((dk[0][ii][c] + dk[1][ii][c]) + dk[2][ii][c]) + dk[3][ii][c];
        if (z == 0) gk = fma(mrow[h], cf[2][c], gk);   // mean row
        double diff[QS_MAXD], d2 = 0.0;
#pragma unroll
        for (int k = 0; k < QS_MAXD; ++k) {
          const double df = k < d ? (xc[k] - xr[h][k]) * il[k] : 0.0;
          diff[k] = df * il[k];
          d2 = fma(df, df, d2);
        }
        const double sgl = gk * kernel_dscale(kind_of(kind, j), d2);
#pragma unroll
        for (int k = 0; k < QS_MAXD; ++k) acc[k] = fma(sgl, diff[k], acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < QS_MAXD; ++k) gx[g][c][k] = acc[k];
    __syncthreads();
    if (tid < QS_B * QS_MAXD) {
      const int cc = tid / QS_MAXD, k = tid - cc * QS_MAXD;
      double v = gx[0][cc][k];
#pragma unroll
      for (int q = 1; q < 8; ++q) v += gx[q][cc][k];
      // element-major partials (dXp[c][k][p], p = (j, z, tile)): the reduction reads each
      // element's partials contiguously
      if (cc < b && k < d) dXp[((size_t)cc * d + k) * np_all + ((size_t)j * zsb + z) * ntile + tile] = v;
    }
  }
  QS_STAMP(4);
}

// one wave per dX element (4 per workgroup): lane-strided partial sums over the element's
// contiguous partials, then a fixed xor-butterfly.  Host mode (hout != nullptr, the plan's host
// graph): every wave also writes its dX element (and the first b acq) to the pinned host
// buffer and fences it at system scope; after a workgroup barrier thread 0 writes the
// evaluation's sequence number into the workgroup's own completion word (hout[b + b d + w]);
// the host waits for all of them (no inter-workgroup counter, no second fence round, no
// separate copy-out kernel).  The sequence number (written by the host before the graph
// launch) is read at kernel entry, so its PCIe round trip overlaps the sums.
//
// With sval (the fused restart scan, hvi_kd3, leaves per-sample values sval[s][c]) the waves of
// the first b elements also form acq[c] = mean over the S samples (lane-strided, then the
// butterfly; NaN for a candidate whose new-point Cholesky failed) and write it to acq.
__global__ __launch_bounds__(256) void qs_dx_reduce(int np, int b, int d, const double* __restrict__ dXp,
                                                    const double* __restrict__ scale, double* __restrict__ dX,
                                                    double* __restrict__ acq, double* hout,
                                                    const double* seqp,
                                                    const double* __restrict__ sval, int S, int m,
                                                    const int* __restrict__ flags,
                                                    int npB, int ntA, const double* __restrict__ cfo) {
  const int lane = threadIdx.x & 63, e = blockIdx.x * 4 + (threadIdx.x >> 6);
  const bool ein = e < b * d;
  const int k = e % d;
  unsigned long long seq = 0;
  // every first-round load of the kernel (the element's partials, the per-sample values and the
  // Cholesky flags of an acquisition element) is issued before the first wait: one memory round
  // trip instead of three dependent ones.  The sequence number (pinned host memory: a PCIe read)
  // is issued after them — the memory counter retires in order, so a wait for the partials
  // would otherwise wait for the PCIe read too
  // (unconditional loads at clamped indices, selected afterwards: a guarded load let the
  // compiler fold the first partial's add into the guard's branch with a wait right after it,
  // one extra memory round trip per load group)
  const double* src = dXp + (size_t)(ein ? e : 0) * np;
  const double sck = scale ? scale[k] : 1.0;   // issued with the first loads, used at the end
  // partials p >= npB (the training-row class from the scan's tail, qs_tail.hpp) carry their
  // output's coefficient cf0[j][c], j = (p - npB) / ntA; the others weigh 1 (fma(1, x, v) is
  // v + x exactly)
  const int ce = ein ? e / d : 0;
  auto wsrc = [&](int p) { return cfo + (size_t)min(max(p - npB, 0) / max(ntA, 1), m - 1) * b + ce; };
  constexpr int NU = 10;
  double x[NU], wv[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    x[u] = src[min(lane + 64 * u, np - 1)];
    wv[u] = cfo ? *wsrc(lane + 64 * u) : 1.0;
  }
  const bool acq_e = ein && sval && e < b;
  double sv[4] = {0.0, 0.0, 0.0, 0.0};
  int fl = 0;
  if (sval) {
    const int ec = min(e, b - 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) sv[u] = sval[(size_t)min(lane + 64 * u, S - 1) * b + ec];
  }
  if (flags) {   // m <= 8 outputs: one flag per lane
    const int fv = flags[(size_t)min(lane, m - 1) * b + min(e, b - 1)];
    fl = (acq_e && lane < m) ? fv : 0;
  }
  // a relaxed system-scope atomic load, not a volatile one: the backend follows a volatile
  // load with a wait for every outstanding load
  if (hout && threadIdx.x == 0)
    seq = __hip_atomic_load(const_cast<unsigned long long*>(reinterpret_cast<const unsigned long long*>(seqp)),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  double av = 0.0;
  if (acq_e) {
    double a = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (lane + 64 * u < S) a += sv[u];
    for (int s = lane + 256; s < S; s += 64) a += sval[(size_t)s * b + e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    const bool bad = __any(fl != 0) != 0;
    av = bad ? nan("") : a / (double)S;
    if (lane == 0) acq[e] = av;
  }
  double v = 0.0;
#pragma unroll
  for (int u = 0; u < NU; ++u)
    if (ein && lane + 64 * u < np) v = fma(lane + 64 * u >= npB ? wv[u] : 1.0, x[u], v);
  if (ein)
    for (int p = lane + 64 * NU; p < np; p += 64) v = fma(cfo && p >= npB ? *wsrc(p) : 1.0, src[p], v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0 && ein) {
    const double r = v * sck;
    dX[e] = r;
    if (hout) {
      const double a = (e < b) ? (sval ? av : acq[e]) : 0.0;
      hout[b + e] = r;
      if (e < b) hout[e] = a;
      __threadfence_system();
    }
  }
  if (hout) {
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long* w = (unsigned long long*)(hout + b + (size_t)b * d + blockIdx.x);
      *(volatile unsigned long long*)w = seq;
    }
  }
}

// ---- launchers (qnehvi_plan.hip) ------------------------------------------------------
bool qs_applies(const evr_qnehvi_state* st, int b, int d) {
  return b >= 1 && b <= QS_B && d <= QS_MAXD && st->m >= 1 && st->S <= QS_SMAX;
}

int qs_ntile_fwd(const evr_qnehvi_state* st) { return cdiv(qn_rows(st), QS_FR); }

size_t qs_norms_doubles(const evr_qnehvi_state* st, int b) { return (size_t)st->m * qs_ntile_fwd(st) * 2 * b; }

// The training-row classes apart from the sample rows (qs_tail.hpp): the fused root's C rows, or
// the split root's L^-1 and G rows (nb > 0) weighted into one class.  Their workgroups ride in
// the backward's launch beside the sample-row workgroups (those hold one workgroup on 160 of the
// 256 CUs at the bench shape).  Measured and removed (round 5): the tail in the restart scan's
// launch (the scan holds every workgroup slot, so the tail stretched it by ~4 us) and inside
// qs_bwd's own workgroups.  A function of the state only, so a plan's layout (qs_dxp_doubles)
// and its launches always agree.
// training rows per tail workgroup's split: 256 (64 per wave, two load batches), or half the
// class (rounded to 16) when that is longer, so the class is two splits and the launch's
// m (2 + 1) 32 workgroups stay resident in one round at two per CU
static int qs_tail_rows(const evr_qnehvi_state* st) {
  const int half = ((st->n + st->nb + 1) / 2 + 15) & ~15;
  return half > 256 ? half : 256;
}
static int qs_tail_za(const evr_qnehvi_state* st) { return cdiv(st->n + st->nb, qs_tail_rows(st)); }

// one backward split over the S sample rows (the coefficients come from its chunks)
static int qs_zsplit(const evr_qnehvi_state*) { return 1; }
static int qs_rows_per(const evr_qnehvi_state* st) { return cdiv(std::max(1, qn_rows(st) - 1 - st->n - st->nb), QS_RC) * QS_RC; }

// workgroups of qs_dx_reduce = completion words it writes in host mode (<= 64 at b <= 32, d <= 8)
int qs_done_words(int b, int d) { return cdiv(b * d, 4); }

// dX partials per element: the sample rows' (output, tile) and the training-row classes' (output, split, tile)
static size_t qs_np_bwd(const evr_qnehvi_state* st) { return (size_t)st->m * qs_zsplit(st) * cdiv(st->n, QS_BI); }
static size_t qs_np_all(const evr_qnehvi_state* st) {
  return qs_np_bwd(st) + (size_t)st->m * qs_tail_za(st) * cdiv(st->n, QS_BI);
}

size_t qs_dxp_doubles(const evr_qnehvi_state* st, int b, int d) {
  return qs_np_all(st) * b * d + (size_t)st->m * b;   // + the classes' coefficients (m x b)
}

int qs_forward(hipStream_t s, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b, const double* Kx,
               double* R, double* P) {
  const int Rr = qn_rows(st), nt = qs_ntile_fwd(st);
  qs_fwd<<<dim3(nt, st->m), QS_FT, 0, s>>>(st->n, st->nb, Rr, b, md->M, Kx, R, P, nt);
  EVR_LAUNCH_CHECK();
  return 0;
}

static void qs_tail_fill(const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b, const double* X,
                         const double* R, double* dXp, QsTail* t) {
  const int nt = cdiv(st->n, QS_BI);
  *t = QsTail{md->M, R, md->Xn, X, md->shift, md->scale, md->lengthscales, dXp, st->ys, st->n, st->nb, qn_rows(st),
              b, md->d, md->kind, nt, qs_tail_za(st), qs_tail_rows(st), (int)qs_np_bwd(st), (int)qs_np_all(st),
              st->m * qs_tail_za(st) * nt};
}

int qs_backward(hipStream_t s, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b, const double* X,
                const double* R, const double* L22, const double* dG, double* dXp, double* dX, double* acq,
                double* hout, const double* seqp, const double* sval, const int* flags) {
  const int nt = cdiv(st->n, QS_BI), d = md->d, zs = qs_zsplit(st);
  const int rows_per = qs_rows_per(st);
  const int npB = (int)qs_np_bwd(st), np = (int)qs_np_all(st);
  double* cfo = dXp + (size_t)np * b * d;
  EVR_CHECK(st->S <= QS_SMAX && st->n > 0, "qs_backward: %d samples exceed the staged %d", st->S, QS_SMAX);
  QsTail t{};
  qs_tail_fill(st, md, b, X, R, dXp, &t);
  // the training-row classes' workgroups are the launch's z >= zs slices
  qs_bwd<<<dim3(nt, st->m, zs + t.za), 256, 0, s>>>(st->n, st->nb, qn_nh(st), st->S, st->m, b, d, md->kind, md->M, R,
                                                     dG, L22, st->ys, st->zq, st->obj_a, md->Xn, X, md->shift,
                                                     md->scale, md->lengthscales, dXp, nt, rows_per, np, cfo, zs, t);
  EVR_LAUNCH_CHECK();
  qs_dx_reduce<<<qs_done_words(b, d), 256, 0, s>>>(np, b, d, dXp, md->scale, dX, acq, hout, seqp, sval, st->S, st->m,
                                                   flags, npB, qs_tail_za(st) * nt, cfo);
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // namespace evr

using namespace evr;

namespace evr {
int samples_norms(hipStream_t s, const evr_qnehvi_state* st, int b, const double* R, const double* norms, double* G,
                  double* L22, int* flags, int tile_rows);
}

extern "C" {

int evr_qnehvi_small_applies(const evr_qnehvi_state* st, int b, int d) { return st && qs_applies(st, b, d) ? 1 : 0; }

long long evr_qnehvi_small_workspace_doubles(const evr_qnehvi_state* st, int b, int d, int which) {
  if (!st || !qs_applies(st, b, d)) return 0;
  return which == 0 ? (long long)qs_norms_doubles(st, b) : (long long)qs_dxp_doubles(st, b, d);
}

int evr_qnehvi_small_forward(void* stream, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                             const double* Kx, double* R, double* P) {
  EVR_CHECK(st && md && Kx && R && P && qs_applies(st, b, md->d), "evr_qnehvi_small_forward: bad arguments");
  return qs_forward((hipStream_t)stream, st, md, b, Kx, R, P);
}

int evr_qnehvi_small_samples(void* stream, const evr_qnehvi_state* st, int b, const double* R, const double* P,
                             double* G, double* L22, int* flags) {
  EVR_CHECK(st && R && P && G && L22 && flags && b >= 1 && b <= QS_B, "evr_qnehvi_small_samples: bad arguments");
  return samples_norms((hipStream_t)stream, st, b, R, P, G, L22, flags, QS_FR);
}

int evr_qnehvi_small_backward(void* stream, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                              const double* X, const double* R, const double* L22, const double* dG, double* dXp,
                              double* dX) {
  EVR_CHECK(st && md && X && R && L22 && dG && dXp && dX && qs_applies(st, b, md->d),
            "evr_qnehvi_small_backward: bad arguments");
  return qs_backward((hipStream_t)stream, st, md, b, X, R, L22, dG, dXp, dX, nullptr, nullptr, nullptr, nullptr,
                     nullptr);
}

}  // extern "C"
