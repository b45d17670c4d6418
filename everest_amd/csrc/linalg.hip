// Dense float64 linear algebra for the GP hot path on gfx950:
//   * batched GEMM on the f64 matrix cores (v_mfma_f64_16x16x4_f64),
//   * batched blocked Cholesky (NB = 64, right-looking: LDS diagonal-block kernel + MFMA
//     panel and lower-triangular trailing-update GEMMs) with the psd_safe_cholesky jitter
//     ladder, optionally fused with the blocked triangular inverse L^-1,
//   * batched triangular solve (L^-1 B / L^-T B) blocked by 64 rows through LDS.
// Replaces the [upstream] torch/LAPACK calls behind GPyTorch's Cholesky / solves
// (Appendix A.4).
#include <cmath>
#include <map>
#include <mutex>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "common.hpp"
#include "../../include/everest_amd.h"

using double4_t = __attribute__((ext_vector_type(4))) double;

namespace evr {

// ---------------------------------------------------------------------------------------
// GEMM: C = alpha * op(A) * op(B) + beta * C   (row-major, batched by blockIdx.z)
// Tile 64x64 per 256-thread workgroup, 4 waves each owning a 32x32 quadrant built from
// 2x2 MFMA 16x16 blocks, K-step 16 staged in LDS.  f64 MFMA fragment maps (gfx950):
//   A: lane l holds A[i = l&15][k = l>>4];  B: B[k = l>>4][j = l&15]
//   D: register r of lane l holds D[row = (l>>4) + 4r][col = l&15]
// ---------------------------------------------------------------------------------------
constexpr int GT = 64, GK = 16, GPAD = 16;

// Split-K: blockIdx.z = batch member * ksplit + k-slice.  With ksplit > 1 the raw partial
// products go to W[(slice * batch + member) * M * N] and gemm_splitk_reduce applies
// alpha / beta in a fixed slice order (deterministic).  Global loads of k-step t+1 are
// issued into registers before the MFMAs of step t (latency hiding for the narrow-N,
// long-K shapes of the posterior / qNEHVI operator products).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f64_kernel(int M, int N, int K, double alpha,
                                                       const double* __restrict__ A, int lda, long long sA,
                                                       const double* __restrict__ B, int ldb, long long sB,
                                                       double beta, double* __restrict__ C, int ldc, long long sC,
                                                       int lower_only, const int* __restrict__ skip, int ksplit,
                                                       int kchunk, double* __restrict__ W) {
  const int bz = blockIdx.z / ksplit, kz = blockIdx.z - bz * ksplit;
  if (skip && skip[bz]) return;  // batch member already failed (Cholesky ladder)
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  if (lower_only && n0 > m0 + GT - 1) return;  // tile strictly above the diagonal
  A += bz * sA;
  B += bz * sB;
  const int kbeg = kz * kchunk, kend = min(K, kbeg + kchunk);
  __shared__ double As[GK][GT + GPAD];
  __shared__ double Bs[GK][GT + GPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  double4_t acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  // per-thread staging coordinates (4 elements of A and of B per k-step)
  int am[4], ak[4], bn[4], bk[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = u * 256 + tid;
    if (!TA) { ak[u] = e & 15; am[u] = e >> 4; } else { am[u] = e & 63; ak[u] = e >> 6; }
    if (!TB) { bn[u] = e & 63; bk[u] = e >> 6; } else { bk[u] = e & 15; bn[u] = e >> 4; }
  }
  double ra[4], rb[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gm = m0 + am[u], gk = k0 + ak[u];
      ra[u] = (gm < M && gk < kend) ? (TA ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.0;
      const int gn = n0 + bn[u], gk2 = k0 + bk[u];
      rb[u] = (gn < N && gk2 < kend) ? (TB ? B[(size_t)gn * ldb + gk2] : B[(size_t)gk2 * ldb + gn]) : 0.0;
    }
  };
  if (kbeg < kend) fetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += GK) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      As[ak[u]][am[u]] = ra[u];
      Bs[bk[u]][bn[u]] = rb[u];
    }
    __syncthreads();
    if (k0 + GK < kend) fetch(k0 + GK);
    const int i = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const double a0 = As[kk + kq][wm + i], a1 = As[kk + kq][wm + 16 + i];
      const double b0 = Bs[kk + kq][wn + i], b1 = Bs[kk + kq][wn + 16 + i];
      acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc11, 0, 0, 0);
    }
    __syncthreads();
  }
  const int col = lane & 15, rq = lane >> 4;
  double* Cb = C + bz * sC;
  double* Wb = W ? W + ((size_t)kz * (gridDim.z / ksplit) + bz) * (size_t)M * N : nullptr;
  auto store = [&](const double4_t& acc, int mi, int ni) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm + mi * 16 + rq + 4 * r;
      const int cc = n0 + wn + ni * 16 + col;
      if (row < M && cc < N && (!lower_only || cc <= row)) {
        if (Wb) {
          Wb[(size_t)row * N + cc] = acc[r];
        } else {
          double* p = Cb + (size_t)row * ldc + cc;
          *p = alpha * acc[r] + (beta == 0.0 ? 0.0 : beta * (*p));
        }
      }
    }
  };
  store(acc00, 0, 0);
  store(acc01, 0, 1);
  store(acc10, 1, 0);
  store(acc11, 1, 1);
}

__global__ __launch_bounds__(256) void gemm_splitk_reduce(int M, int N, int batch, int ksplit, double alpha,
                                                          const double* __restrict__ W, double beta,
                                                          double* __restrict__ C, int ldc, long long sC) {
  const long long mn = (long long)M * N;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= mn) return;
  const int bz = blockIdx.y;
  double acc = 0.0;
  for (int kz = 0; kz < ksplit; ++kz) acc += W[((size_t)kz * batch + bz) * mn + e];
  const int row = (int)(e / N), cc = (int)(e - (long long)row * N);
  double* p = C + bz * sC + (size_t)row * ldc + cc;
  *p = alpha * acc + (beta == 0.0 ? 0.0 : beta * (*p));
}

// ---------------------------------------------------------------------------------------
// Triangular solve, in place on B (n x nrhs, row-major): X = L^-1 B or L^-T B.
// One workgroup per (64-column tile, batch); 64-row blocks; update GEMM through LDS.
// ---------------------------------------------------------------------------------------
constexpr int TT = 64;

// a 64 x 64 tile of op(L) into LDS, T[rr][cc] = op(L)[r0 + rr][c0 + cc] (zero outside n x n):
// all 16 loads of a thread are issued before the first LDS store — the load -> store loop
// kept one load in flight (the compiler cannot move a global load above an LDS store it may
// alias), 16 dependent memory round trips per tile
template <bool TRANS>
__device__ __forceinline__ void stage_tile_tt(double (*T)[TT + 1], const double* L, int ldl, int n, int r0, int c0) {
  double v[16];
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = tid + 256 * u, rr = e >> 6, cc = e & 63;
    const int gr = TRANS ? c0 + cc : r0 + rr, gc = TRANS ? r0 + rr : c0 + cc;
    v[u] = (gr < n && gc < n) ? L[(size_t)gr * ldl + gc] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = tid + 256 * u;
    T[e >> 6][e & 63] = v[u];
  }
}

template <bool TRANS>
__global__ __launch_bounds__(256) void trsm_kernel(int n, int nrhs, const double* __restrict__ Lm, long long sL,
                                                   int ldl, double* __restrict__ Bm, long long sB, int ldb) {
  const double* L = Lm + blockIdx.y * sL;
  double* B = Bm + blockIdx.y * sB;
  const int c0 = blockIdx.x * TT;
  __shared__ double Lt[TT][TT + 1];
  __shared__ double Xt[TT][TT + 1];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;  // 4x4 micro-tile: rows ty+16*a, cols tx+16*c
  const int nblk = (n + TT - 1) / TT;
  for (int it = 0; it < nblk; ++it) {
    const int bi = TRANS ? nblk - 1 - it : it;
    const int r0 = bi * TT;
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = r0 + ty + 16 * a, col = c0 + tx + 16 * c;
        acc[a][c] = (r < n && col < nrhs) ? B[(size_t)r * ldb + col] : 0.0;
      }
    const int jb0 = TRANS ? bi + 1 : 0, jb1 = TRANS ? nblk : bi;
    for (int bj = jb0; bj < jb1; ++bj) {
      const int s0 = bj * TT;
      {
        double xv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = tid + 256 * u, xr = s0 + (e >> 6), xc = c0 + (e & 63);
          xv[u] = (xr < n && xc < nrhs) ? B[(size_t)xr * ldb + xc] : 0.0;
        }
        stage_tile_tt<TRANS>(Lt, L, ldl, n, r0, s0);   // Lt[rr][cc] = op(L)[r0 + rr][s0 + cc]
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = tid + 256 * u;
          Xt[e >> 6][e & 63] = xv[u];
        }
      }
      __syncthreads();
#pragma unroll 4
      for (int q = 0; q < TT; ++q) {
        double lq[4], xq[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) lq[a] = Lt[ty + 16 * a][q];
#pragma unroll
        for (int c = 0; c < 4; ++c) xq[c] = Xt[q][tx + 16 * c];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[a][c] -= lq[a] * xq[c];
      }
      __syncthreads();
    }
    // stage RHS block and the diagonal block of op(L)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) Xt[ty + 16 * a][tx + 16 * c] = acc[a][c];
    stage_tile_tt<false>(Lt, L, ldl, n, r0, r0);   // L itself (lower)
    __syncthreads();
    const int rb = min(TT, n - r0);
    if (tid < TT) {
      const int col = tid;
      if (!TRANS) {
        for (int r = 0; r < rb; ++r) {
          double s = Xt[r][col];
          for (int q = 0; q < r; ++q) s -= Lt[r][q] * Xt[q][col];
          Xt[r][col] = s / Lt[r][r];
        }
      } else {
        for (int r = rb - 1; r >= 0; --r) {
          double s = Xt[r][col];
          for (int q = r + 1; q < rb; ++q) s -= Lt[q][r] * Xt[q][col];
          Xt[r][col] = s / Lt[r][r];
        }
      }
    }
    __syncthreads();
    for (int e = tid; e < TT * TT; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      const int gr = r0 + rr, gc = c0 + cc;
      if (gr < n && gc < nrhs) B[(size_t)gr * ldb + gc] = Xt[rr][cc];
    }
    __syncthreads();
  }
}

// Forward substitution L X = B (lower, no transpose) for n <= TS_MAXN, 16 right-hand-side
// columns per workgroup: 5 x 512 columns give 160 workgroups (trsm_kernel's 64-column tiles
// gave 40, each walking its blocks alone: 0.47 ms at n = 280).  Wave w solves columns
// 4w .. 4w + 3; within a wave, 16 lanes share a column, lane rg owning rows rg + 16a of the
// current 64-row block.  Solved rows stay in LDS for the later blocks' updates.  Per row the
// subtractions run in trsm_kernel's order (earlier blocks' q ascending, then the diagonal
// block's q ascending) with the same contractions, and the division last: bitwise its result.
constexpr int TS_C = 16, TS_MAXN = 512;
__global__ __launch_bounds__(256) void trsm16_kernel(int n, int nrhs, const double* __restrict__ Lm, long long sL,
                                                     int ldl, double* __restrict__ Bm, long long sB, int ldb) {
  const double* L = Lm + blockIdx.y * sL;
  double* B = Bm + blockIdx.y * sB;
  const int c0 = blockIdx.x * TS_C;
  __shared__ double Lt[TT][TT + 1];
  extern __shared__ double Xs[];   // (nblk * 64) x 16: solved rows
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rg = lane & 15, cl = wave * 4 + (lane >> 4), col = c0 + cl;
  const bool cin = col < nrhs;
  const int nblk = (n + TT - 1) / TT;
  for (int bi = 0; bi < nblk; ++bi) {
    const int r0 = bi * TT;
    double acc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int r = r0 + rg + 16 * a;
      acc[a] = (r < n && cin) ? B[(size_t)r * ldb + col] : 0.0;
    }
    for (int bj = 0; bj < bi; ++bj) {
      const int s0 = bj * TT;
      __syncthreads();   // Lt reuse
      stage_tile_tt<false>(Lt, L, ldl, n, r0, s0);
      __syncthreads();
#pragma unroll 4
      for (int q = 0; q < TT; ++q) {
        const double xq = Xs[(size_t)(s0 + q) * TS_C + cl];
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a] -= Lt[rg + 16 * a][q] * xq;
      }
    }
    __syncthreads();
    stage_tile_tt<false>(Lt, L, ldl, n, r0, r0);
    __syncthreads();
    const int rb = min(TT, n - r0);
    const int gl = lane & ~15;
#pragma unroll
    for (int ao = 0; ao < 4; ++ao) {
      for (int k = 0; k < 16; ++k) {
        const int q = 16 * ao + k;
        if (q >= rb) break;
        double xq = rg == k ? acc[ao] / Lt[q][q] : 0.0;
        xq = __shfl(xq, gl | k, 64);
        if (rg == k) acc[ao] = xq;
#pragma unroll
        for (int a = 0; a < 4; ++a)
          if (rg + 16 * a > q) acc[a] -= Lt[rg + 16 * a][q] * xq;
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rl = rg + 16 * a, r = r0 + rl;
      Xs[(size_t)r * TS_C + cl] = acc[a];
      if (r < n && cin) B[(size_t)r * ldb + col] = acc[a];
    }
  }
}

__global__ void set_identity_kernel(int n, double* M, long long sM, int ldm) {
  double* P = M + blockIdx.y * sM;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < (long long)n * n) {
    const int i = (int)(e / n), j = (int)(e % n);
    P[(size_t)i * ldm + j] = (i == j) ? 1.0 : 0.0;
  }
}

// ---------------------------------------------------------------------------------------
// Blocked right-looking Cholesky (NB = 64) with the diagonal-block inverses:
//   diag:   one workgroup factors L_kk and forms inv(L_kk) by elimination on [A_kk | I]
//           (64 barrier steps), flags a non-positive pivot in info[b];
//   panel:  L[k+nb:, k] <- L[k+nb:, k] inv(L_kk)^T       (MFMA GEMM, in place)
//   update: L[k+nb:, k+nb:] -= P P^T, lower triangle only  (MFMA GEMM)
// ---------------------------------------------------------------------------------------
constexpr int BNB = 64;

// (also clears the member's info word: no separate memset node per attempt)
__global__ void chol_init_kernel(int n, const double* __restrict__ A, long long sA, int lda, double* __restrict__ L,
                                 long long sL, int ldl, const double* __restrict__ jit, int* __restrict__ info) {
  const int b = blockIdx.y;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) info[b] = 0;
  if (e >= (long long)n * n) return;
  const int i = (int)(e / n), j = (int)(e % n);
  double v = (j <= i) ? A[b * sA + (size_t)i * lda + j] : 0.0;
  if (i == j) v += jit[b];
  L[b * sL + (size_t)i * ldl + j] = v;
}

// Factor the diagonal block at k0 (already updated), write L_kk into L and inv(L_kk) to
// Dinv (ld BNB).  Blocked inside the 64x64 block with 16-wide panels:
//   (1) wave 0 factors the 16x16 diagonal sub-block in registers (lane = row x column
//       quad; the pivot column / inverse row are exchanged through LDS with wave-level
//       ordering only) keeping unnormalised pivots d_j: L = L_unit d^1/2 and
//       inv(L) = d^-1/2 inv(L_unit), inv(L_unit) accumulated alongside;
//   (2) all waves: panel L21 = A21 L11^-T;   (3) trailing A22 -= L21 L21^T;
// then inv(L_kk) is assembled from the four diagonal inverses by block forward
// substitution (X_ij = -X_ii sum_k L_ik X_kj, by distance i - j).  12 workgroup barriers
// and 64 wave-synchronous pivot steps instead of 64 workgroup-wide steps.
constexpr int CP = 16;   // panel width
#ifdef EVR_CHOL_PROF
__device__ unsigned long long chol_prof[16];
#define CHOL_T(k) if (threadIdx.x == 0) chol_prof[k] += __builtin_readcyclecounter();
#define CHOL_T0(k) if (threadIdx.x == 0) chol_prof[k] -= __builtin_readcyclecounter();
#else
#define CHOL_T(k)
#define CHOL_T0(k)
#endif

__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// cross-lane helpers (f64 as two dwords): readlane (uniform result) and a DPP quad broadcast
// of lane s of every 4-lane group
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l), hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double bperm_f64(double v, int src_lane) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)x);
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ int quad_bcast32(int v, int s) {
  switch (s) {   // quad_perm [s, s, s, s]
    case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xf, 0xf, false);
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xf, 0xf, false);
    case 2: return __builtin_amdgcn_mov_dpp(v, 0xAA, 0xf, 0xf, false);
    default: return __builtin_amdgcn_mov_dpp(v, 0xFF, 0xf, 0xf, false);
  }
}

__device__ __forceinline__ double quad_bcast_f64(double v, int s) {
  const long long x = __double_as_longlong(v);
  const int lo = quad_bcast32((int)x, s), hi = quad_bcast32((int)(x >> 32), s);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}


// one wave: factor A[c0.., c0..] (16x16, lower) in place; inverse into X[c0.., c0..].
// Lane (row r, quad q) holds A[r][q + 4k].  Per pivot step the pivot comes by readlane (a
// uniform scalar: its reciprocal starts at once and the failure test is a scalar branch),
// the lane's own row entry A[r][j] by a DPP quad broadcast, and the column entries of the
// other rows (A[c][j]) and the finished inverse row by ds_bpermute (an LDS store / fence /
// load exchange measured 636 vs 532 cycles per pivot; a row-per-lane DPP leaf, a symmetric
// permlane leaf, a single-pivot bpermute leaf and an 8-column leaf measured slower too — rounds
// 3 to 6, DESIGN.md §4.3 — and were removed).
// Returns the first failing local pivot index or -1 (uniform over the wave).
__device__ __forceinline__ int panel_factor16(double (*A)[BNB + 1], double (*X)[BNB + 1], int c0, double* colj,
                                              double* erow, double* piv) {
  const int lane = threadIdx.x & 63, r = lane >> 2, q = lane & 3;
  double a[4], e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = q + 4 * k;
    a[k] = (c <= r) ? A[c0 + r][c0 + c] : 0.0;
    e[k] = (c == r) ? 1.0 : 0.0;
  }
  int bad = -1;
  // two pivots per exchange round: columns j, j1 = j + 1 and inverse rows j, j1 as they are
  // before step j arrive in one round of ds_bpermute; what step j1 reads after step j (its
  // pivot, its column entries A'[c][j1], the lane's own A'[r][j1], the inverse row E'[j1]) is
  // formed locally with step j's own operations — m = a * ip, fma(-m, x, y) on the same
  // operands — so every value is bitwise the one-pivot loop's, with half the exchange rounds
#pragma unroll
  for (int j = 0; j < CP; j += 2) {
    const int j1 = j + 1;
    const double p0 = readlane_f64(a[j >> 2], 4 * j + (j & 3));      // A[j][j]
    const double a10 = readlane_f64(a[j >> 2], 4 * j1 + (j & 3));    // A[j1][j]
    const double a11 = readlane_f64(a[j1 >> 2], 4 * j1 + (j1 & 3));  // A[j1][j1]
    const double arj = quad_bcast_f64(a[j >> 2], j & 3);             // A[r][j]
    double arj1 = quad_bcast_f64(a[j1 >> 2], j1 & 3);                // A[r][j1]
    double c0[4], c1[4], e0[4], e1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c0[k] = bperm_f64(a[j >> 2], 4 * q + 16 * k + (j & 3));
      c1[k] = bperm_f64(a[j1 >> 2], 4 * q + 16 * k + (j1 & 3));
      e0[k] = bperm_f64(e[k], 4 * j + q);
      e1[k] = bperm_f64(e[k], 4 * j1 + q);
    }
    if (!(p0 > 0.0)) {
      bad = j;
      break;
    }
    if (lane == 0) piv[j] = p0;
    double ip = __builtin_amdgcn_rcp(p0);
    ip = fma(ip, fma(-p0, ip, 1.0), ip);
    ip = fma(ip, fma(-p0, ip, 1.0), ip);
    {  // step j
      const double m = arj * ip;
      const bool below = r > j;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = q + 4 * k;
        const double dn = fma(-m, c0[k], a[k]);
        const double en = fma(-m, e0[k], e[k]);
        a[k] = (below && c > j && c <= r) ? dn : a[k];
        e[k] = (below && c <= j) ? en : e[k];
      }
    }
    // step j's updates of the values step j1 exchanges
    const double m10 = a10 * ip;                                      // row j1's multiplier
    const double p1 = fma(-m10, a10, a11);                            // A'[j1][j1]
    if (r >= j1) arj1 = fma(-(arj * ip), a10, arj1);                  // A'[r][j1]
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = q + 4 * k;
      if (c >= j1) c1[k] = fma(-(c0[k] * ip), a10, c1[k]);            // A'[c][j1]
      if (c <= j) e1[k] = fma(-m10, e0[k], e1[k]);                    // E'[j1][c]
    }
    if (!(p1 > 0.0)) {
      bad = j1;
      break;
    }
    if (lane == 0) piv[j1] = p1;
    double ip1 = __builtin_amdgcn_rcp(p1);
    ip1 = fma(ip1, fma(-p1, ip1, 1.0), ip1);
    ip1 = fma(ip1, fma(-p1, ip1, 1.0), ip1);
    {  // step j1
      const double m = arj1 * ip1;
      const bool below = r > j1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = q + 4 * k;
        const double dn = fma(-m, c1[k], a[k]);
        const double en = fma(-m, e1[k], e[k]);
        a[k] = (below && c > j1 && c <= r) ? dn : a[k];
        e[k] = (below && c <= j1) ? en : e[k];
      }
    }
  }
  (void)colj;
  (void)erow;
  if (bad >= 0) return bad;
  lds_wave_sync();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = q + 4 * k;
    A[c0 + r][c0 + c] = (c <= r) ? a[k] / sqrt(piv[c]) : 0.0;
    X[c0 + r][c0 + c] = (c <= r) ? e[k] / sqrt(piv[r]) : 0.0;
  }
  return -1;
}

// acc += P Q over one 16x16x16 block product on the f64 matrix cores (fragment maps as in
// gemm_f64_kernel); P = M1[pr.., pc..] (or its transpose), Q = M2[qr.., qc..] (or transpose).
template <bool PT, bool QT>
__device__ __forceinline__ double4_t mm16(const double (*M1)[BNB + 1], int pr, int pc, const double (*M2)[BNB + 1],
                                          int qr, int qc, double4_t acc) {
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < CP; kk += 4) {
    const double a = PT ? M1[pr + kk + kq][pc + i] : M1[pr + i][pc + kk + kq];
    const double b = QT ? M2[qr + i][qc + kk + kq] : M2[qr + kk + kq][qc + i];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  return acc;
}

// Factor the 64x64 block A (LDS, lower triangle, padding rows/cols as the identity) in
// place into L_kk and its inverse into X (zeroed by the caller).  All 256 threads; returns
// the first failing local pivot index or -1 (uniform over the workgroup).
__device__ __forceinline__ int factor_diag64(double (*A)[BNB + 1], double (*X)[BNB + 1], double* colj, double* erow, double* piv,
                             int* fail) {
  const int tid = threadIdx.x, wave = tid >> 6;
  if (tid == 0) *fail = -1;
  __syncthreads();
  CHOL_T0(0)
  for (int p = 0; p < BNB / CP; ++p) {
    const int c0 = p * CP;
    CHOL_T0(1)
    if (wave == 0) {
      const int bad = panel_factor16(A, X, c0, colj, erow, piv);
      if (bad >= 0 && (tid & 63) == 0) *fail = c0 + bad;
    }
    __syncthreads();
    CHOL_T(1)
    if (*fail >= 0) break;
    const int r0 = c0 + CP, R = BNB - r0;
    if (R == 0) break;
    CHOL_T0(2)
    // (2) panel L21 = A21 X11^T (X11 = inv(L11), lower): wave w < R/16 owns row tile w
    const int lane = tid & 63, fc = lane & 15, fr = lane >> 4;
    double4_t acc = {0, 0, 0, 0};
    if (wave < R / CP) acc = mm16<false, true>(A, r0 + CP * wave, c0, X, c0, c0, acc);
    __syncthreads();
    if (wave < R / CP)
#pragma unroll
      for (int q = 0; q < 4; ++q) A[r0 + CP * wave + fr + 4 * q][c0 + fc] = acc[q];
    __syncthreads();
    CHOL_T(2)
    CHOL_T0(3)
    // (3) trailing update of the lower tile triangle: A_ij -= L21_i L21_j^T
    {
      const int nt = R / CP;
      for (int tt = wave; tt < nt * (nt + 1) / 2; tt += 4) {
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= tt) ++ti;
        const int tj = tt - ti * (ti + 1) / 2;
        double4_t u = {0, 0, 0, 0};
        u = mm16<false, true>(A, r0 + CP * ti, c0, A, r0 + CP * tj, c0, u);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = fr + 4 * q;
          if (ti != tj || fc <= rr) A[r0 + CP * ti + rr][r0 + CP * tj + fc] -= u[q];
        }
      }
    }
    __syncthreads();
    CHOL_T(3)
  }
  CHOL_T(0)
  const int f = *fail;
  if (f >= 0) return f;
  CHOL_T0(4)
  // inv(L) off-diagonal blocks by distance dd = i - j: wave pr owns the pair (pr + dd, pr);
  // T = sum_k L_ik X_kj stays in the accumulator, which is already the B fragment of X_ii T
  for (int dd = 1; dd < BNB / CP; ++dd) {
    const int np = BNB / CP - dd;
    if (wave < np) {
      const int i = wave + dd, j = wave;
      const int lane = tid & 63, fc = lane & 15, fr = lane >> 4;
      double4_t tacc = {0, 0, 0, 0};
      for (int k = j; k < i; ++k) tacc = mm16<false, false>(A, CP * i, CP * k, X, CP * k, CP * j, tacc);
      double4_t y = {0, 0, 0, 0};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double a = X[CP * i + fc][CP * i + 4 * q + fr];
        y = __builtin_amdgcn_mfma_f64_16x16x4f64(a, tacc[q], y, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) X[CP * i + fr + 4 * q][CP * j + fc] = -y[q];
    }
    __syncthreads();
  }
  CHOL_T(4)
  return -1;
}

// store a factored diagonal block: L_kk (rows/cols < nb, lower) and inv(L_kk) (identity
// padding beyond nb, ld BNB)
__device__ __forceinline__ void store_diag64(const double (*A)[BNB + 1], const double (*X)[BNB + 1], int nb, double* L, int ldl,
                             int k0, double* Di) {
  for (int e = threadIdx.x; e < BNB * BNB; e += 256) {
    const int i = e >> 6, c = e & 63;
    if (i < nb && c < nb) {
      L[(size_t)(k0 + i) * ldl + k0 + c] = (c <= i) ? A[i][c] : 0.0;
      Di[(size_t)i * BNB + c] = (c <= i) ? X[i][c] : 0.0;
    } else {
      Di[(size_t)i * BNB + c] = (i == c) ? 1.0 : 0.0;
    }
  }
}

__global__ __launch_bounds__(256) void chol_diag_kernel(int n, int k0, double* __restrict__ Lm, long long sL, int ldl,
                                                        double* __restrict__ Dinv, long long sD,
                                                        int* __restrict__ info) {
  const int b = blockIdx.x;
  if (info[b]) return;
  double* L = Lm + b * sL;
  double* Di = Dinv + b * sD;
  const int nb = min(BNB, n - k0);
  __shared__ double A[BNB][BNB + 1];
  __shared__ double X[BNB][BNB + 1];
  __shared__ double colj[CP], erow[CP], piv[CP];
  __shared__ int fail;
  const int tid = threadIdx.x;
  {
    double v[16];   // all loads in flight before the LDS stores
    const int c = tid & 63, i0 = tid >> 6;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = 4 * u + i0;
      // padding rows / columns beyond nb factor as the identity
      v[u] = (i < nb && c <= i) ? L[(size_t)(k0 + i) * ldl + k0 + c] : (i == c ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      A[4 * u + i0][c] = v[u];
      X[4 * u + i0][c] = 0.0;
    }
  }
  const int f = factor_diag64(A, X, colj, erow, piv, &fail);
  if (f >= 0) {
    if (f < nb && tid == 0) info[b] = k0 + f + 1;
    if (f < nb) return;
  }
  store_diag64(A, X, nb, L, ldl, k0, Di);
}

// ---------------------------------------------------------------------------------------
// Fused right-looking steps (one launch per 64-column block instead of three):
//   chol_step_kernel(k): one workgroup per trailing lower tile (I, J) of step k.  Each
//     recomputes the two panel tiles it needs, P_I = A_Ik inv(L_kk)^T and P_J, from the
//     un-normalised panel (still in L) and Dinv_k, applies C_IJ -= P_I P_J^T, and the
//     workgroup of the next diagonal tile (k+1, k+1) — whose update is then complete —
//     factors it at once (L_k+1,k+1 and its inverse).  k = -1 factors block 0 only.
//   chol_panel_kernel: after the last step, every off-diagonal tile L_IK = A_IK Dinv_K^T in
//     place (the panels stay un-normalised while later steps still read them).
// Workgroups of one launch never read what another writes, so no inter-workgroup sync.
// ---------------------------------------------------------------------------------------
// quadrant of the 64x64 product P Q^T (P, Q row-major LDS tiles): wave (wr, wc) owns rows
// wr*32.., cols wc*32..; acc[bi][bj] in the MFMA D layout.
__device__ __forceinline__ void mm64_nt(const double (*P)[BNB + 1], const double (*Q)[BNB + 1], int wr, int wc,
                                        double4_t (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
#pragma unroll 4
  for (int kk = 0; kk < BNB; kk += 4) {
    const double a0 = P[wr + i][kk + kq], a1 = P[wr + 16 + i][kk + kq];
    const double b0 = Q[wc + i][kk + kq], b1 = Q[wc + 16 + i][kk + kq];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
}

// tile (row block r0, col block c0) of the matrix into LDS (rows >= n zero).  All 16 loads
// of a thread are issued before the first LDS store (a load -> store loop would wait on
// every load in turn); a wave reads 512 contiguous bytes of one row per instruction.
__device__ __forceinline__ void load_tile64(double (*T)[BNB + 1], const double* L, int ldl, int n, int r0, int c0) {
  double v[16];
  const int c = threadIdx.x & 63, i0 = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int i = 4 * u + i0;
    v[u] = (r0 + i < n && c0 + c < n) ? L[(size_t)(r0 + i) * ldl + c0 + c] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) T[4 * u + i0][c] = v[u];
}

__device__ __forceinline__ void load_dinv64(double (*T)[BNB + 1], const double* Di) {
  double v[16];
  const int c = threadIdx.x & 63, i0 = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = Di[(4 * u + i0) * BNB + c];
#pragma unroll
  for (int u = 0; u < 16; ++u) T[4 * u + i0][c] = v[u];
}

// write a wave's quadrant accumulators into an LDS tile (row-major)
__device__ __forceinline__ void put_quadrant(double (*T)[BNB + 1], int wr, int wc, const double4_t (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, col = lane & 15, rq = lane >> 4;
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[wr + bi * 16 + rq + 4 * r][wc + bj * 16 + col] = acc[bi][bj][r];
}

// quadrant of the 64x64 product P Q (both row-major LDS tiles)
__device__ __forceinline__ void mm64_nn(const double (*P)[BNB + 1], const double (*Q)[BNB + 1], int wr, int wc,
                                        double4_t (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
#pragma unroll 4
  for (int kk = 0; kk < BNB; kk += 4) {
    const double a0 = P[wr + i][kk + kq], a1 = P[wr + 16 + i][kk + kq];
    const double b0 = Q[kk + kq][wc + i], b1 = Q[kk + kq][wc + 16 + i];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
}

// Inverse tile of the fused sweep (chol_step_kernel, blockIdx beyond the trailing tiles):
// X = L^-1 is formed right-looking on the identity alongside the factorisation.  With
// B_ij = delta_ij I - sum_{s<i} L_is X_sj, the block row X_k = Dinv_k B_k is complete once
// step k - 1 has run, so step k applies B_ij -= L_ik (Dinv_k B_kj) to every i > k, j <= k
// (B_kk = I: the product is L_ik Dinv_k, the tile's first write).  L_ik = A_ik Dinv_k^T is
// recomputed from the un-normalised panel like the trailing tiles do; B lives in X and
// chol_final_kernel turns it into X_kj = Dinv_k B_kj.  The step's critical path is the next
// diagonal block's factor, which these tiles run beside.
__device__ __forceinline__ void chol_inv_tile(int n, int k, int i, int j, const double* L, int ldl, const double* Dk,
                                              double* X, int ldx, double (*TI)[BNB + 1], double (*TJ)[BNB + 1],
                                              double (*TD)[BNB + 1]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32, col = lane & 15, rq = lane >> 4;
  const int r0 = i * BNB, c0 = j * BNB, p0 = k * BNB;
  load_tile64(TI, L, ldl, n, r0, p0);                 // A_ik
  if (j < k) load_tile64(TJ, X, ldx, n, p0, c0);      // B_kj
  load_dinv64(TD, Dk);
  __syncthreads();
  double4_t pi[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  double4_t xk[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  mm64_nt(TI, TD, wr, wc, pi);                        // L_ik
  if (j < k) mm64_nn(TD, TJ, wr, wc, xk);             // X_kj = Dinv_k B_kj
  __syncthreads();
  put_quadrant(TI, wr, wc, pi);
  if (j < k) put_quadrant(TJ, wr, wc, xk);
  __syncthreads();
  double4_t u[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  mm64_nn(TI, j < k ? TJ : TD, wr, wc, u);
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + wr + bi * 16 + rq + 4 * r, cc = c0 + wc + bj * 16 + col;
        if (row < n && cc < n) {
          double* o = X + (size_t)row * ldx + cc;
          *o = (j < k) ? *o + (-1.0) * u[bi][bj][r] : -u[bi][bj][r];
        }
      }
}

__global__ __launch_bounds__(256) void chol_step_kernel(int n, int k, double* __restrict__ Lm, long long sL, int ldl,
                                                        double* __restrict__ Dinv, long long sD,
                                                        int* __restrict__ info, int ntrail, double* __restrict__ Xm,
                                                        long long sX, int ldx) {
  const int b = blockIdx.y;
  if (info[b]) return;
  double* L = Lm + b * sL;
  __shared__ double TI[BNB][BNB + 1];
  __shared__ double TJ[BNB][BNB + 1];
  __shared__ double TD[BNB][BNB + 1];
  __shared__ double colj[CP], erow[CP], piv[CP];
  __shared__ int fail;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32, col = lane & 15, rq = lane >> 4;
  if ((int)blockIdx.x >= ntrail) {   // inverse tile (i > k, j <= k) of the fused sweep
    const int t = blockIdx.x - ntrail;
    chol_inv_tile(n, k, k + 1 + t / (k + 1), t % (k + 1), L, ldl, Dinv + b * sD + (size_t)k * BNB * BNB,
                  Xm + b * sX, ldx, TI, TJ, TD);
    return;
  }
  int I = 0, J = 0;   // trailing tile (lower, row-major enumeration)
  {
    const int t = blockIdx.x;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    J = t - I * (I + 1) / 2;
  }
  const int r0 = (k + 1 + I) * BNB, c0 = (k + 1 + J) * BNB;
  double4_t acc[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  // C quadrant straight into the accumulator layout
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + wr + bi * 16 + rq + 4 * r, cc = c0 + wc + bj * 16 + col;
        acc[bi][bj][r] = (row < n && cc < n) ? L[(size_t)row * ldl + cc] : 0.0;
      }
  if (k >= 0) {
    const int p0 = k * BNB;
    const double* Dk = Dinv + b * sD + (size_t)k * BNB * BNB;
    load_tile64(TI, L, ldl, n, r0, p0);
    if (I != J) load_tile64(TJ, L, ldl, n, c0, p0);
    load_dinv64(TD, Dk);
    __syncthreads();
    // panel tiles P = A_panel Dinv_k^T, written back over their LDS source
    double4_t pi[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
    double4_t pj[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
    mm64_nt(TI, TD, wr, wc, pi);
    if (I != J) mm64_nt(TJ, TD, wr, wc, pj);
    __syncthreads();
    put_quadrant(TI, wr, wc, pi);
    if (I != J) put_quadrant(TJ, wr, wc, pj);
    __syncthreads();
    double4_t u[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
    mm64_nt(TI, I != J ? TJ : TI, wr, wc, u);
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[bi][bj][r] = acc[bi][bj][r] + (-1.0) * u[bi][bj][r];
  }
  if (I != 0 || J != 0) {   // plain trailing tile: store (lower triangle of a diagonal tile)
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + wr + bi * 16 + rq + 4 * r, cc = c0 + wc + bj * 16 + col;
          if (row < n && cc < n && (I != J || cc <= row)) L[(size_t)row * ldl + cc] = acc[bi][bj][r];
        }
    return;
  }
  // the next diagonal block: factor it now (padding rows / columns beyond nb as the identity)
  const int nb = min(BNB, n - r0);
  __syncthreads();   // TI / TJ free
  put_quadrant(TI, wr, wc, acc);
  __syncthreads();
  for (int e = tid; e < BNB * BNB; e += 256) {
    const int i = e >> 6, c = e & 63;
    TI[i][c] = (i < nb && c < nb) ? (c <= i ? TI[i][c] : 0.0) : (i == c ? 1.0 : 0.0);
    TJ[i][c] = 0.0;
  }
  const int f = factor_diag64(TI, TJ, colj, erow, piv, &fail);
  if (f >= 0) {
    if (f < nb && tid == 0) info[b] = r0 + f + 1;
    if (f < nb) return;
  }
  store_diag64(TI, TJ, nb, L, ldl, r0, Dinv + b * sD + (size_t)(k + 1) * BNB * BNB);
}

// off-diagonal tiles (I > K): L_IK = A_IK Dinv_K^T in place; with X (the fused inverse),
// workgroups beyond the panel tiles finish X: tile (k, j) = Dinv_k B_kj below the diagonal
// block, Dinv_k on it, zero above (a failed member: Dinv_k on the diagonal, zeros elsewhere)
__global__ __launch_bounds__(256) void chol_panel_kernel(int n, double* __restrict__ Lm, long long sL, int ldl,
                                                         const double* __restrict__ Dinv, long long sD,
                                                         const int* __restrict__ info, int npanel,
                                                         double* __restrict__ Xm, long long sX, int ldx) {
  const int b = blockIdx.y;
  __shared__ double TA[BNB][BNB + 1];
  __shared__ double TD[BNB][BNB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32, col = lane & 15, rq = lane >> 4;
  if ((int)blockIdx.x >= npanel) {
    const int nblk = (n + BNB - 1) / BNB, t = blockIdx.x - npanel, K = t / nblk, J = t % nblk;
    double* X = Xm + b * sX;
    const double* Dk = Dinv + b * sD + (size_t)K * BNB * BNB;
    if (J > K || (J < K && info[b])) {
      for (int e = tid; e < BNB * BNB; e += 256) {
        const int row = K * BNB + (e >> 6), cc = J * BNB + (e & 63);
        if (row < n && cc < n) X[(size_t)row * ldx + cc] = 0.0;
      }
      return;
    }
    if (J == K) {
      for (int e = tid; e < BNB * BNB; e += 256) {
        const int row = K * BNB + (e >> 6), cc = K * BNB + (e & 63);
        if (row < n && cc < n) X[(size_t)row * ldx + cc] = Dk[e];
      }
      return;
    }
    load_tile64(TA, X, ldx, n, K * BNB, J * BNB);   // B_KJ
    load_dinv64(TD, Dk);
    __syncthreads();
    double4_t p[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
    mm64_nn(TD, TA, wr, wc, p);
    __syncthreads();   // every wave has read TA before the stores overwrite its source rows
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = K * BNB + wr + bi * 16 + rq + 4 * r, cc = J * BNB + wc + bj * 16 + col;
          if (row < n && cc < n) X[(size_t)row * ldx + cc] = p[bi][bj][r];
        }
    return;
  }
  if (info[b]) return;
  double* L = Lm + b * sL;
  int I = 1, K = 0;
  {
    const int t = blockIdx.x;   // strictly lower tiles, row-major: row I has I tiles
    while (I * (I + 1) / 2 <= t) ++I;
    K = t - I * (I - 1) / 2;
  }
  load_tile64(TA, L, ldl, n, I * BNB, K * BNB);
  load_dinv64(TD, Dinv + b * sD + (size_t)K * BNB * BNB);
  __syncthreads();
  double4_t p[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  mm64_nt(TA, TD, wr, wc, p);
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = I * BNB + wr + bi * 16 + rq + 4 * r, cc = K * BNB + wc + bj * 16 + col;
        if (row < n && cc < n) L[(size_t)row * ldl + cc] = p[bi][bj][r];
      }
}

// ---------------------------------------------------------------------------------------
// Triangular inverse by block rows, one launch per row i (instead of two GEMMs):
//   X_ij = -Dinv_i sum_{k=j}^{i-1} L_ik X_kj   for every j < i (one workgroup each),
// X_ii = Dinv_i and zeros above the diagonal placed beforehand (place_diag_blocks_kernel).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tri_inv_row_kernel(int n, int i, const double* __restrict__ Lm, long long sL,
                                                          int ldl, const double* __restrict__ Dinv, long long sD,
                                                          double* __restrict__ Xm, long long sX, int ldx,
                                                          const int* __restrict__ skip) {
  const int b = blockIdx.y, j = blockIdx.x;
  if (skip && skip[b]) return;
  const double* L = Lm + b * sL;
  double* X = Xm + b * sX;
  __shared__ double TA[BNB][BNB + 1];
  __shared__ double TB[BNB][BNB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32, col = lane & 15, rq = lane >> 4, li = lane & 15,
            kq = lane >> 4;
  double4_t t[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  // the next step's tiles are loaded into registers while the current step's MFMAs run
  double ra[16], rb[16];
  const int tc = tid & 63, ti0 = tid >> 6;
  auto fetch = [&](int k) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = 4 * u + ti0;
      const int ra_row = i * BNB + r, ra_col = k * BNB + tc, rb_row = k * BNB + r, rb_col = j * BNB + tc;
      ra[u] = (ra_row < n && ra_col < n) ? L[(size_t)ra_row * ldl + ra_col] : 0.0;
      rb[u] = (rb_row < n && rb_col < n) ? X[(size_t)rb_row * ldx + rb_col] : 0.0;
    }
  };
  fetch(j);
  for (int k = j; k < i; ++k) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      TA[4 * u + ti0][tc] = ra[u];                    // L_ik
      TB[4 * u + ti0][tc] = rb[u];                    // X_kj
    }
    __syncthreads();
    if (k + 1 < i) fetch(k + 1);
    // T += L_ik X_kj  (B operand X[kk][c])
#pragma unroll 4
    for (int kk = 0; kk < BNB; kk += 4) {
      const double a0 = TA[wr + li][kk + kq], a1 = TA[wr + 16 + li][kk + kq];
      const double b0 = TB[kk + kq][wc + li], b1 = TB[kk + kq][wc + 16 + li];
      t[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, t[0][0], 0, 0, 0);
      t[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, t[0][1], 0, 0, 0);
      t[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, t[1][0], 0, 0, 0);
      t[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, t[1][1], 0, 0, 0);
    }
  }
  __syncthreads();
  put_quadrant(TB, wr, wc, t);                          // T
  load_dinv64(TA, Dinv + b * sD + (size_t)i * BNB * BNB);
  __syncthreads();
  double4_t y[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
#pragma unroll 4
  for (int kk = 0; kk < BNB; kk += 4) {
    const double a0 = TA[wr + li][kk + kq], a1 = TA[wr + 16 + li][kk + kq];
    const double b0 = TB[kk + kq][wc + li], b1 = TB[kk + kq][wc + 16 + li];
    y[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, y[0][0], 0, 0, 0);
    y[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, y[0][1], 0, 0, 0);
    y[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, y[1][0], 0, 0, 0);
    y[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, y[1][1], 0, 0, 0);
  }
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * BNB + wr + bi * 16 + rq + 4 * r, cc = j * BNB + wc + bj * 16 + col;
        if (row < n && cc < n) X[(size_t)row * ldx + cc] = -y[bi][bj][r];
      }
}

// ---------------------------------------------------------------------------------------
// Triangular inverse by 16-column panels, one launch (n <= NMAX): workgroup (c, b) owns
// columns [16c, 16c + 16) of X = L^-1, which lie in block column cb = 16c / 64.  Rows above
// block cb are zero, block cb is its slice of Dinv_cb, and every later block row i is
//   X_i = -Dinv_i sum_{k=cb}^{i-1} L_ik X_k
// with the solved rows X_k of its 16 columns resident in LDS.  The block rows of one column
// panel are serial, but each step is a 64 x 16 x 64 product (16 MFMAs per wave) instead of
// tri_inv_row_kernel's 64 x 64 x 64, and all column panels run at once: at n = 512 the
// critical path is 36 such steps in one launch instead of 7 launches of up to 8 full-tile
// steps.  Wave w owns rows 16w .. 16w + 15 of each block row; the A operands (L_ik, Dinv_i)
// come straight from global memory (L2-resident, shared by the panels of a member), the next
// step's issued before the current step's MFMAs.  Per element the accumulation sequence
// (k ascending, then kk in steps of 4, the same lane / register positions in the MFMA tile,
// out-of-range rows and columns loaded as zero) is tri_inv_row_kernel's: bitwise its result.
// ---------------------------------------------------------------------------------------
template <int NMAX>
__global__ __launch_bounds__(256) void tri_inv_col_kernel(int n, const double* __restrict__ Lm, long long sL,
                                                          int ldl, const double* __restrict__ Dinv, long long sD,
                                                          double* __restrict__ Xm, long long sX, int ldx,
                                                          const int* __restrict__ skip) {
  constexpr int TW = 16;
  __shared__ double Xs[NMAX][TW];    // solved rows of this panel (a half-wave reads 2 rows: conflict-free)
  __shared__ double Ts[BNB][TW];     // sum_k L_ik X_k of the current block row (B operand of Dinv_i)
  const int b = blockIdx.y, c0 = blockIdx.x * TW, cb = c0 / BNB, cl = c0 - cb * BNB;
  const double* L = Lm + b * sL;
  const double* Db = Dinv + b * sD;
  double* X = Xm + b * sX;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, kq = lane >> 4;
  const int nblk = (n + BNB - 1) / BNB;
  const bool skp = skip && skip[b];
  const int ncol = min(TW, n - c0);
  for (int e = tid; e < cb * BNB * TW; e += 256) {   // zeros above the diagonal block
    const int r = e / TW, c = e % TW;
    if (c < ncol) X[(size_t)r * ldx + c0 + c] = 0.0;
  }
  {
    const double* Dc = Db + (size_t)cb * BNB * BNB;
    for (int e = tid; e < BNB * TW; e += 256) {
      const int r = e / TW, c = e % TW, row = cb * BNB + r;
      const bool in = row < n && c < ncol;
      const double v = in ? Dc[(size_t)r * BNB + cl + c] : 0.0;
      Xs[row][c] = v;
      if (in) X[(size_t)row * ldx + c0 + c] = v;
    }
  }
  if (skp) {   // a failed member: zeros below the diagonal block, as the row kernels leave it
    for (int e = tid; e < (n - min(n, (cb + 1) * BNB)) * TW; e += 256) {
      const int r = (cb + 1) * BNB + e / TW, c = e % TW;
      if (c < ncol) X[(size_t)r * ldx + c0 + c] = 0.0;
    }
    return;
  }
  __syncthreads();
  double a[16], an[16];
  auto load_l = [&](double (&dst)[16], int i, int k) {
    const int row = i * BNB + 16 * w + li;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int col = k * BNB + 4 * s + kq;
      dst[s] = (row < n && col < n) ? L[(size_t)row * ldl + col] : 0.0;
    }
  };
  auto load_d = [&](double (&dst)[16], int i) {
    const double* Di = Db + (size_t)i * BNB * BNB + (size_t)(16 * w + li) * BNB;
#pragma unroll
    for (int s = 0; s < 16; ++s) dst[s] = Di[4 * s + kq];
  };
  if (cb + 1 < nblk) load_l(a, cb + 1, cb);
  for (int i = cb + 1; i < nblk; ++i) {
    double4_t t = {0, 0, 0, 0};
    for (int k = cb; k < i; ++k) {
      if (k + 1 < i) load_l(an, i, k + 1);
      else load_d(an, i);
#pragma unroll
      for (int s = 0; s < 16; ++s) t = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], Xs[k * BNB + 4 * s + kq][li], t, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = an[s];
    }
    // D map: register r of lane l holds T[16w + (l >> 4) + 4r][l & 15]
#pragma unroll
    for (int r = 0; r < 4; ++r) Ts[16 * w + kq + 4 * r][li] = t[r];
    __syncthreads();
    if (i + 1 < nblk) load_l(an, i + 1, cb);
    double4_t y = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 16; ++s) y = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], Ts[4 * s + kq][li], y, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i * BNB + 16 * w + kq + 4 * r;
      const bool in = row < n && li < ncol;
      const double v = -y[r];
      Xs[row][li] = in ? v : 0.0;
      if (in) X[(size_t)row * ldx + c0 + li] = v;
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) a[s] = an[s];
    __syncthreads();   // block row i in Xs, Ts free for the next block row
  }
}

// Inverse of every 64x64 diagonal block of a given lower-triangular L (grid (blocks, batch)):
// column-parallel forward substitution, row steps separated by barriers.
__global__ __launch_bounds__(256) void diag_block_inverse_kernel(int n, const double* __restrict__ Lm, long long sL,
                                                                 int ldl, double* __restrict__ Dinv, long long sD) {
  const int blk = blockIdx.x, b = blockIdx.y;
  const double* L = Lm + b * sL;
  double* Di = Dinv + b * sD + (size_t)blk * BNB * BNB;
  const int r0 = blk * BNB, nb = min(BNB, n - r0);
  __shared__ double T[BNB][BNB + 1];
  __shared__ double X[BNB][BNB + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < BNB * BNB; e += 256) {
    const int i = e / BNB, c = e % BNB;
    T[i][c] = (i < nb && c <= i) ? L[(size_t)(r0 + i) * ldl + r0 + c] : (i == c ? 1.0 : 0.0);
    X[i][c] = 0.0;
  }
  __syncthreads();
  // row r: X[r][c] = (delta_rc - sum_{c<=t<r} T[r][t] X[t][c]) / T[r][r], c <= r; 4 threads/column
  const int c = tid & 63, part = tid >> 6;
  for (int r = 0; r < BNB; ++r) {
    double s = 0.0;
    if (c <= r)
      for (int t = c + part; t < r; t += 4) s = fma(T[r][t], X[t][c], s);
    __shared__ double red[4][BNB];
    red[part][c] = s;
    __syncthreads();
    if (part == 0 && c <= r) {
      const double tot = red[0][c] + red[1][c] + red[2][c] + red[3][c];
      X[r][c] = ((r == c ? 1.0 : 0.0) - tot) / T[r][r];
    }
    __syncthreads();
  }
  for (int e = tid; e < BNB * BNB; e += 256) {
    const int i = e / BNB, cc = e % BNB;
    Di[(size_t)i * BNB + cc] = (i < nb && cc < nb) ? X[i][cc] : (i == cc ? 1.0 : 0.0);
  }
}

// X = 0 except the diagonal blocks, which receive Dinv (batch x nblk x 64 x 64)
__global__ void place_diag_blocks_kernel(int n, const double* __restrict__ Dinv, long long sD, double* __restrict__ X,
                                         long long sX, int ldx) {
  const int b = blockIdx.y;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)n * n) return;
  const int i = (int)(e / n), j = (int)(e % n);
  const int bi = i / BNB, bj = j / BNB;
  double v = 0.0;
  if (bi == bj) v = Dinv[b * sD + ((size_t)bi * BNB + (i - bi * BNB)) * BNB + (j - bj * BNB)];
  X[b * sX + (size_t)i * ldx + j] = v;
}

// the gemm_core.hpp engine (gemm.hip)
size_t dg_gemm_ws_doubles(bool tA, int M, int N, int K, int batch);
int dg_gemm(hipStream_t s, bool tA, int M, int N, int K, double alpha, const double* A, int lda, long long sA,
            const double* B, int ldb, long long sB, double beta, double* Cm, int ldc, long long sC, int batch,
            double* W);

}  // namespace evr

namespace {
using namespace evr;

// Per-stream scratch of the jitter ladder (diagonal-block inverses, the inverse's row
// products, jitter and info vectors), grown on demand and reused: the ladder synchronises
// its stream before returning, so the next call on that stream may overwrite it.  A
// hipMallocAsync / hipFreeAsync pair per call cost up to ~1.4 ms at 5 x 512 once the pool
// had released its memory.
struct LadderScratch {
  void* p = nullptr;
  size_t bytes = 0;
};

static int stream_scratch(int slot, hipStream_t s, size_t bytes, void** out) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, LadderScratch> pool;   // one entry per (use, stream), never freed
  std::lock_guard<std::mutex> lock(mu);
  LadderScratch& e = pool[{slot, s}];
  if (e.bytes < bytes) {
    if (e.p) EVR_HIP(hipFree(e.p));
    e.p = nullptr;
    e.bytes = 0;
    EVR_HIP(hipMalloc(&e.p, bytes));
    e.bytes = bytes;
  }
  *out = e.p;
  return 0;
}

static int ladder_scratch(hipStream_t s, size_t bytes, void** out) { return stream_scratch(0, s, bytes, out); }
static int gemm_scratch(hipStream_t s, size_t bytes, void** out) { return stream_scratch(1, s, bytes, out); }

// split-K partials: the stream's reusable scratch (stream order protects it), or a
// stream-ordered allocation while the stream is being captured into a graph (*pooled false:
// the caller frees it after the reduction)
static int splitk_scratch(hipStream_t s, size_t bytes, double** W, bool* pooled) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  EVR_HIP(hipStreamIsCapturing(s, &cap));
  if (cap == hipStreamCaptureStatusNone) {
    *pooled = true;
    return gemm_scratch(s, bytes, (void**)W);
  }
  *pooled = false;
  EVR_HIP(hipMallocAsync((void**)W, bytes, s));
  return 0;
}

int launch_gemm(hipStream_t s, bool tA, bool tB, int M, int N, int K, double alpha, const double* A, int lda,
                long long sA, const double* B, int ldb, long long sB, double beta, double* C, int ldc, long long sC,
                int batch, int lower_only = 0, const int* skip = nullptr, bool allow_split = false) {
  if (M == 0 || N == 0) return 0;
  if (!tB && !lower_only && !skip) {
    // the gemm_core.hpp engine (gemm.hip): every non-triangular product with B untransposed
    double* W = nullptr;
    bool pooled = true;
    const size_t wn = allow_split ? dg_gemm_ws_doubles(tA, M, N, K, batch) : 0;
    if (wn)
      if (int rc = splitk_scratch(s, sizeof(double) * wn, &W, &pooled)) return rc;
    if (int rc = dg_gemm(s, tA, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, W)) return rc;
    if (!pooled) EVR_HIP(hipFreeAsync(W, s));
    return 0;
  }
  const int tiles = cdiv(N, GT) * cdiv(M, GT) * batch;
  // Split K when the tile grid cannot fill the 256 CUs and each slice keeps >= 8 k-steps
  // (only for non-aliased outputs: the Cholesky panel update runs in place).
  int ksplit = 1;
  if (allow_split && !lower_only && !skip && tiles < 512) {
    ksplit = std::min(cdiv(1024, tiles), K / (8 * GK));
    ksplit = std::max(1, std::min(ksplit, 32));
  }
  const int kchunk = ksplit > 1 ? cdiv(cdiv(K, ksplit), GK) * GK : std::max(K, 1);
  if (ksplit > 1) ksplit = cdiv(K, kchunk);
  double* W = nullptr;
  bool pooled = false;
  if (ksplit > 1)
    if (int rc = splitk_scratch(s, sizeof(double) * (size_t)ksplit * batch * M * N, &W, &pooled)) return rc;
  dim3 grid(cdiv(N, GT), cdiv(M, GT), batch * ksplit);
#define G_(TA_, TB_)                                                                                       \
  gemm_f64_kernel<TA_, TB_><<<grid, 256, 0, s>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, \
                                                 lower_only, skip, ksplit, kchunk, W)
  if (!tA && !tB) G_(false, false);
  else if (!tA && tB) G_(false, true);
  else if (tA && !tB) G_(true, false);
  else G_(true, true);
#undef G_
  EVR_LAUNCH_CHECK();
  if (ksplit > 1) {
    dim3 g2(cdiv((long long)M * N, 256), batch);
    gemm_splitk_reduce<<<g2, 256, 0, s>>>(M, N, batch, ksplit, alpha, W, beta, C, ldc, sC);
    EVR_LAUNCH_CHECK();
    if (!pooled) EVR_HIP(hipFreeAsync(W, s));
  }
  return 0;
}

// One blocked factorisation attempt of every batch member (jitter already in L's diagonal).
// Default: the fused right-looking steps that recompute the panel per consumer (nblk + 1
// launches); EVR_CHOL=v1 the diag / panel GEMM / trailing GEMM sequence (3 launches per block,
// the parity tests' reference).  (A look-ahead form, nblk launches, measured slower — 1.43 vs
// 1.29 ms at n = 2048, profiles/r03/b — and was removed in round 6.)
static int chol_variant() {   // 1 fused right-looking, 2 v1 (read per call: tests switch it)
  const char* e = std::getenv("EVR_CHOL");
  return (e && !std::strcmp(e, "v1")) ? 2 : 1;
}
static bool chol_v1() { return chol_variant() == 2; }

// flags of the look-ahead steps: one int per (member, block) after the diagonal-block inverses
static size_t chol_dinv_doubles(int batch, int n) {
  const size_t nblk = (size_t)cdiv(n, BNB);
  return (size_t)batch * nblk * BNB * BNB + ((size_t)batch * nblk + 1) / 2;
}

// EVR_TRIINV (read per call; the parity tests' references): unset — the fused right-looking
// variant forms X = L^-1 in the same launches (n <= 1024); "col" — the separate one-launch
// column-panel inverse after the factorisation; "row" — the per-block-row launches
static int triinv_mode() {
  const char* tv = std::getenv("EVR_TRIINV");
  return !(tv && tv[0]) ? 0 : (!std::strcmp(tv, "row") ? 2 : 1);
}
static bool chol_inv_fused(int n) { return chol_variant() == 1 && n <= 1024 && triinv_mode() == 0; }

int chol_blocked(hipStream_t s, int batch, int n, double* L, int ldl, long long sL, double* Dinv, int* info,
                 double* X = nullptr, int ldx = 0, long long sX = 0) {
  const int nblk = (n + BNB - 1) / BNB;
  const long long sD = (long long)nblk * BNB * BNB;
  if (!chol_v1()) {
    for (int k = -1; k < nblk - 1; ++k) {
      const int T = nblk - 1 - k;   // trailing tile rows (block 0 alone for k = -1)
      const int tiles = k < 0 ? 1 : T * (T + 1) / 2;
      const int itiles = (X && k >= 0) ? (nblk - 1 - k) * (k + 1) : 0;
      chol_step_kernel<<<dim3(tiles + itiles, batch), 256, 0, s>>>(n, k, L, sL, ldl, Dinv, sD, info, tiles, X, sX,
                                                                   ldx);
      EVR_LAUNCH_CHECK();
    }
    const int npanel = nblk * (nblk - 1) / 2, nx = X ? nblk * nblk : 0;
    if (npanel + nx > 0) {
      chol_panel_kernel<<<dim3(npanel + nx, batch), 256, 0, s>>>(n, L, sL, ldl, Dinv, sD, info, npanel, X, sX, ldx);
      EVR_LAUNCH_CHECK();
    }
    return 0;
  }
  for (int kb = 0; kb < nblk; ++kb) {
    const int k0 = kb * BNB, nb = std::min(BNB, n - k0), r0 = k0 + nb, t = n - r0;
    double* Dk = Dinv + (size_t)kb * BNB * BNB;
    chol_diag_kernel<<<batch, 256, 0, s>>>(n, k0, L, sL, ldl, Dk, sD, info);
    EVR_LAUNCH_CHECK();
    if (t <= 0) break;
    double* P = L + (size_t)r0 * ldl + k0;
    // panel: P <- P Dk^T (in place; one 64-column tile, K loop completes before the store)
    if (launch_gemm(s, false, true, t, nb, nb, 1.0, P, ldl, sL, Dk, BNB, sD, 0.0, P, ldl, sL, batch, 0, info))
      return 1;
    // trailing update, lower triangle
    double* C = L + (size_t)r0 * ldl + r0;
    if (launch_gemm(s, false, true, t, t, nb, -1.0, P, ldl, sL, P, ldl, sL, 1.0, C, ldl, sL, batch, 1, info))
      return 1;
  }
  return 0;
}

// X = L^-1 from L and the diagonal-block inverses (block forward substitution).
int tri_inv_blocked(hipStream_t s, int batch, int n, const double* L, int ldl, long long sL, const double* Dinv,
                    double* X, int ldx, long long sX, double* T, const int* skip) {
  const int nblk = (n + BNB - 1) / BNB;
  const long long sD = (long long)nblk * BNB * BNB;
  if (!chol_v1() && n <= 1024 && triinv_mode() != 2) {
    dim3 g(cdiv(n, 16), batch);
    if (n <= 512) tri_inv_col_kernel<512><<<g, 256, 0, s>>>(n, L, sL, ldl, Dinv, sD, X, sX, ldx, skip);
    else tri_inv_col_kernel<1024><<<g, 256, 0, s>>>(n, L, sL, ldl, Dinv, sD, X, sX, ldx, skip);
    EVR_LAUNCH_CHECK();
    return 0;
  }
  dim3 g1(cdiv((long long)n * n, 256), batch);
  place_diag_blocks_kernel<<<g1, 256, 0, s>>>(n, Dinv, sD, X, sX, ldx);
  EVR_LAUNCH_CHECK();
  if (!chol_v1()) {
    for (int i = 1; i < nblk; ++i) {
      tri_inv_row_kernel<<<dim3(i, batch), 256, 0, s>>>(n, i, L, sL, ldl, Dinv, sD, X, sX, ldx, skip);
      EVR_LAUNCH_CHECK();
    }
    return 0;
  }
  const long long sT = (long long)BNB * n;
  for (int i = 1; i < nblk; ++i) {
    const int r0 = i * BNB, rb = std::min(BNB, n - r0);
    // T = L[r0:r0+rb, 0:r0] X[0:r0, 0:r0]
    if (launch_gemm(s, false, false, rb, r0, r0, 1.0, L + (size_t)r0 * ldl, ldl, sL, X, ldx, sX, 0.0, T, n, sT,
                    batch, 0, skip))
      return 1;
    // X[r0:r0+rb, 0:r0] = -inv(L_ii) T
    if (launch_gemm(s, false, false, rb, r0, rb, -1.0, Dinv + (size_t)i * BNB * BNB, BNB, sD, T, n, sT, 0.0,
                    X + (size_t)r0 * ldx, ldx, sX, batch, 0, skip))
      return 1;
  }
  return 0;
}

// Jitter ladder around chol_blocked: members that fail get jitter0*10^(t-1) added to A's
// diagonal and the batch is refactored (members that already succeeded recompute
// identically), as psd_safe_cholesky does per failing batch member.
int chol_ladder(hipStream_t s, int batch, int n, const double* A, int lda, long long sA, double* L, int ldl,
                long long sL, double jitter0, int max_tries, double* jitter_used, int* info_out, double* Linv,
                int ldi, long long sI) {
  const size_t dbytes = sizeof(double) * chol_dinv_doubles(batch, n);
  const size_t tbytes = Linv ? sizeof(double) * (size_t)batch * BNB * n : 0;
  double *Dinv = nullptr, *T = nullptr, *jit_d = nullptr;
  int* info_d = nullptr;
  {
    const size_t a = (dbytes + 255) & ~(size_t)255, t = (tbytes + 255) & ~(size_t)255;
    const size_t j = (sizeof(double) * batch + 255) & ~(size_t)255;
    unsigned char* base = nullptr;
    if (int rc = ladder_scratch(s, a + t + j + sizeof(int) * batch, (void**)&base)) return rc;
    Dinv = (double*)base;
    T = tbytes ? (double*)(base + a) : nullptr;
    jit_d = (double*)(base + a + t);
    info_d = (int*)(base + a + t + j);
  }
  std::vector<double> jit(batch, 0.0);
  std::vector<int> info(batch, 0);
  int rc = 0;
  const bool fused = Linv && chol_inv_fused(n);
  for (int t = 0; t <= max_tries; ++t) {
    EVR_HIP(hipMemcpyAsync(jit_d, jit.data(), sizeof(double) * batch, hipMemcpyHostToDevice, s));
    dim3 g1(cdiv((long long)n * n, 256), batch);
    chol_init_kernel<<<g1, 256, 0, s>>>(n, A, sA, lda, L, sL, ldl, jit_d, info_d);
    EVR_LAUNCH_CHECK();
    if ((rc = chol_blocked(s, batch, n, L, ldl, sL, Dinv, info_d, fused ? Linv : nullptr, ldi, sI))) break;
    EVR_HIP(hipMemcpyAsync(info.data(), info_d, sizeof(int) * batch, hipMemcpyDeviceToHost, s));
    EVR_HIP(hipStreamSynchronize(s));
    bool anyfail = false;
    for (int b = 0; b < batch; ++b)
      if (info[b]) {
        anyfail = true;
        if (t < max_tries) jit[b] = jitter0 * std::pow(10.0, (double)t);
      }
    if (!anyfail || t == max_tries) break;
  }
  if (!rc && Linv && !fused) rc = tri_inv_blocked(s, batch, n, L, ldl, sL, Dinv, Linv, ldi, sI, T, info_d);
  if (!rc) {
    if (jitter_used) EVR_HIP(hipMemcpyAsync(jitter_used, jit.data(), sizeof(double) * batch, hipMemcpyHostToDevice, s));
    if (info_out) EVR_HIP(hipMemcpyAsync(info_out, info_d, sizeof(int) * batch, hipMemcpyDeviceToDevice, s));
  }
  EVR_HIP(hipStreamSynchronize(s));  // host vectors and the stream's scratch must outlive the work
  return rc;
}
}  // namespace

namespace evr {
// Graph-capturable pieces for the MLL plan (mll_plan.hip): one psd_safe_cholesky attempt
// with the jitter vector already on the device (no host sync, no allocation) followed by the
// triangular inverse, and the GEMM without the split-K workspace allocation.
int chol_inverse_attempt(hipStream_t s, int batch, int n, const double* A, double* L, double* Linv, double* Dinv,
                         double* T, const double* jit_d, int* info_d) {
  dim3 g1(cdiv((long long)n * n, 256), batch);
  chol_init_kernel<<<g1, 256, 0, s>>>(n, A, (long long)n * n, n, L, (long long)n * n, n, jit_d, info_d);
  EVR_LAUNCH_CHECK();
  const long long nn = (long long)n * n;
  if (chol_inv_fused(n)) return chol_blocked(s, batch, n, L, n, nn, Dinv, info_d, Linv, n, nn);
  if (int rc = chol_blocked(s, batch, n, L, n, nn, Dinv, info_d)) return rc;
  return tri_inv_blocked(s, batch, n, L, n, nn, Dinv, Linv, n, nn, T, info_d);
}

size_t chol_inverse_dinv_doubles(int batch, int n) { return chol_dinv_doubles(batch, n); }

int gemm_plain(hipStream_t s, bool tA, bool tB, int M, int N, int K, double alpha, const double* A, int lda,
               long long sA, const double* B, int ldb, long long sB, double beta, double* C, int ldc, long long sC,
               int batch) {
  return launch_gemm(s, tA, tB, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, 0, nullptr, false);
}
}  // namespace evr

using namespace evr;

extern "C" {

int evr_gemm_f64(void* stream, int transA, int transB, int M, int N, int K, double alpha, const double* A,
                 int lda, long long strideA, const double* B, int ldb, long long strideB, double beta, double* C,
                 int ldc, long long strideC, int batch) {
  EVR_CHECK(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "evr_gemm_f64: bad sizes M=%d N=%d K=%d batch=%d", M, N,
            K, batch);
  const bool alias = C == A || C == B;
  return launch_gemm((hipStream_t)stream, transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C,
                     ldc, strideC, batch, 0, nullptr, !alias);
}

int evr_cholesky(void* stream, int batch, int n, const double* A, int lda, long long strideA, double* L, int ldl,
                 long long strideL, double jitter0, int max_tries, double* jitter_used, int* info) {
  EVR_CHECK(n >= 1 && batch >= 1 && max_tries >= 0, "evr_cholesky: bad sizes n=%d batch=%d", n, batch);
  EVR_CHECK(A != L, "evr_cholesky: A and L must not alias (the jitter ladder restarts from A)");
  return chol_ladder((hipStream_t)stream, batch, n, A, lda, strideA, L, ldl, strideL, jitter0, max_tries,
                     jitter_used, info, nullptr, 0, 0);
}

int evr_cholesky_inverse(void* stream, int batch, int n, const double* A, int lda, long long strideA, double* L,
                         int ldl, long long strideL, double* Linv, int ldi, long long strideI, double jitter0,
                         int max_tries, double* jitter_used, int* info) {
  EVR_CHECK(n >= 1 && batch >= 1 && max_tries >= 0, "evr_cholesky_inverse: bad sizes n=%d batch=%d", n, batch);
  EVR_CHECK(A != L && Linv != L && Linv != A, "evr_cholesky_inverse: A, L and Linv must not alias");
  return chol_ladder((hipStream_t)stream, batch, n, A, lda, strideA, L, ldl, strideL, jitter0, max_tries,
                     jitter_used, info, Linv, ldi, strideI);
}

int evr_trsm_lower(void* stream, int batch, int n, int nrhs, const double* L, int ldl, long long strideL,
                   int transpose, double* B, int ldb, long long strideB) {
  EVR_CHECK(n >= 1 && nrhs >= 0 && batch >= 1, "evr_trsm_lower: bad sizes");
  if (nrhs == 0) return 0;
  if (!transpose && n <= TS_MAXN) {
    const size_t xs = sizeof(double) * (size_t)cdiv(n, TT) * TT * TS_C;
    trsm16_kernel<<<dim3(cdiv(nrhs, TS_C), batch), 256, xs, (hipStream_t)stream>>>(n, nrhs, L, strideL, ldl, B,
                                                                                   strideB, ldb);
    EVR_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid(cdiv(nrhs, TT), batch);
  if (transpose)
    trsm_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(n, nrhs, L, strideL, ldl, B, strideB, ldb);
  else
    trsm_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(n, nrhs, L, strideL, ldl, B, strideB, ldb);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_tri_inv_lower(void* stream, int batch, int n, const double* L, int ldl, long long strideL, double* Linv,
                      int ldi, long long strideI) {
  EVR_CHECK(n >= 1 && batch >= 1, "evr_tri_inv_lower: bad sizes");
  EVR_CHECK(L != Linv, "evr_tri_inv_lower: L and Linv must not alias");
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (n + BNB - 1) / BNB;
  double *Dinv = nullptr, *T = nullptr;
  EVR_HIP(hipMallocAsync((void**)&Dinv, sizeof(double) * (size_t)batch * nblk * BNB * BNB, s));
  EVR_HIP(hipMallocAsync((void**)&T, sizeof(double) * (size_t)batch * BNB * n, s));
  dim3 g(nblk, batch);
  diag_block_inverse_kernel<<<g, 256, 0, s>>>(n, L, strideL, ldl, Dinv, (long long)nblk * BNB * BNB);
  int rc = 0;
  if (hipGetLastError() != hipSuccess) {
    set_error("evr_tri_inv_lower: launch failed");
    rc = 1;
  }
  if (!rc) rc = tri_inv_blocked(s, batch, n, L, ldl, strideL, Dinv, Linv, ldi, strideI, T, nullptr);
  (void)hipFreeAsync(Dinv, s);
  (void)hipFreeAsync(T, s);
  return rc;
}

}  // extern "C"
