// Kernel-matrix assembly and its gradients (RBF / Matérn-ν ARD) on gfx950.
//
// 64x64 output tile per 256-thread workgroup; both point tiles are normalised
// (Normalize input transform, bofire/surrogates/utils.py:144-154), divided by the
// lengthscales and staged in LDS with a +1 row pad; every thread owns a 4x4 micro-tile
// (rows ty+16a, cols tx+16c) so that each store instruction writes 16 consecutive
// doubles of a row.  Distances are formed from explicit differences (no x^2+x'^2-2xx'
// cancellation).  HBM-bound for small d: 8 bytes written per entry.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "gemm_core.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int KT = 64;
constexpr int KMAXD = 64;

template <int RA, int KIND>
__global__ __launch_bounds__(256) void kmat_kernel(int kind, int n1, int n2, int d, const double* __restrict__ X1,
                                                   const double* __restrict__ sh1, const double* __restrict__ sc1,
                                                   const double* __restrict__ X2, const double* __restrict__ sh2,
                                                   const double* __restrict__ sc2, const double* __restrict__ ls,
                                                   const double* __restrict__ os, const double* __restrict__ dg,
                                                   double* __restrict__ K,
                                                   const unsigned long long* seq_src, unsigned long long* seq_dst,
                                                   double* __restrict__ x_dst, int* __restrict__ zero_dst, int nzero) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // the posterior's arrival counters (post_proj_kernel) zeroed by the first workgroup: the
  // projection launches after this kernel has completed
  if (zero_dst && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
    for (int t = threadIdx.x; t < nzero; t += 256) zero_dst[t] = 0;
  // host-driven chains: the evaluation's sequence number (pinned host memory, posted with the
  // candidates) copied to device memory, so the chain's last kernel reads it from L2 instead of
  // across PCIe (this kernel's candidate loads pay that latency anyway)
  if (seq_dst && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
    *seq_dst = __hip_atomic_load(const_cast<unsigned long long*>(seq_src), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int b = blockIdx.z;
  const int i0 = blockIdx.y * (16 * RA), j0 = blockIdx.x * KT;
  const int ld = d + 1;
  double* A = smem;            // KT x ld
  double* Bt = smem + 16 * RA * ld;  // KT x ld
  const double* lsb = ls + (size_t)b * d;
  const int tid = threadIdx.x;
  // d < 16: at most 4 staging elements per thread; all loads issued before the first wait
  double xv[4], xw[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = tid + 256 * t;
    const int r = e / d;
    xv[t] = 0.0;
    xw[t] = 0.0;
    if (e < KT * d) {
      if (r < 16 * RA && i0 + r < n1) xv[t] = X1[(size_t)(i0 + r) * d + (e - r * d)];
      if (j0 + r < n2) xw[t] = X2[(size_t)(j0 + r) * d + (e - r * d)];
    }
  }
  // host-driven chains: the candidates (n2 <= KT: one column tile) copied to device memory by
  // the first workgroup, so that the chain's later kernels read them from L2, not across PCIe
  if (x_dst && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int e = tid + 256 * t;
      if (e < KT * d && e / d < n2) x_dst[e] = xw[t];
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = tid + 256 * t;
    if (e < KT * d) {
      const int r = e / d, k = e - r * d;
      const double il = 1.0 / lsb[k];
      double v = 0.0, w = 0.0;
      if (r < 16 * RA && i0 + r < n1) {
        v = xv[t];
        if (sh1) v -= sh1[k];
        if (sc1) v *= sc1[k];
      }
      if (j0 + r < n2) {
        w = xw[t];
        if (sh2) w -= sh2[k];
        if (sc2) w *= sc2[k];
      }
      if (r < 16 * RA) A[r * ld + k] = v * il;
      Bt[r * ld + k] = w * il;
    }
  }
  __shared__ double kexp[64];
  kexp_stage(kexp, tid, 256);
  __syncthreads();
  const int tx = tid & 15, ty = tid >> 4;
  double acc[RA][4];
#pragma unroll
  for (int a = 0; a < RA; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = 0.0;
  for (int k = 0; k < d; ++k) {
    double av[RA], bv[4];
#pragma unroll
    for (int a = 0; a < RA; ++a) av[a] = A[(ty + 16 * a) * ld + k];
#pragma unroll
    for (int c = 0; c < 4; ++c) bv[c] = Bt[(tx + 16 * c) * ld + k];
#pragma unroll
    for (int a = 0; a < RA; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double df = av[a] - bv[c];
        acc[a][c] = fma(df, df, acc[a][c]);
      }
  }
  const double scale = os ? os[b] : 1.0;
  const double dadd = dg ? dg[b] : 0.0;
  double* Kb = K + (size_t)b * n1 * n2;
#pragma unroll
  for (int a = 0; a < RA; ++a) {
    const int i = i0 + ty + 16 * a;
    if (i >= n1) continue;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = j0 + tx + 16 * c;
      if (j < n2) {
        double v = scale * kernel_value_t(KIND, acc[a][c], kexp);
        if (i == j) v += dadd;
        Kb[(size_t)i * n2 + j] = v;
      }
    }
  }
}

// Kernel-matrix assembly on the matrix cores for wide inputs (d >= 16): the 64x64 tile of
// dot products u1_i . u2_j (u = normalised x / ls) runs on v_mfma_f64_16x16x4f64 over the
// d axis, the epilogue forms d2 = |u1|^2 + |u2|^2 - 2 u1.u2 (clamped at 0; exactly 0 where a
// diagonal entry pairs bitwise-identical points, as GPyTorch's sq_dist does for x1_eq_x2),
// applies the kernel, outputscale and diagonal add, and streams the tile out: the f64 VALU
// distance loop of kmat_kernel (2 flop per coordinate per entry) was the bound at d = 32.
using kd4_t = __attribute__((ext_vector_type(4))) double;
using kd2_t = __attribute__((ext_vector_type(2))) double;

// The tile's kernel values (wave quadrant rows wm.., cols wn..; acc[q] in the MFMA D layout:
// register r of lane l is entry (wm + (q >> 1) 16 + (l >> 4) + 4 r, wn + (q & 1) 16 + (l & 15))).
// d2 = |u1|^2 + |u2|^2 - 2 u1.u2 clamped at 0, exactly 0 on a diagonal entry pairing bitwise-
// identical points (dtile: i0 == j0, the only tiles holding diagonal entries).
template <int KIND>
__device__ __forceinline__ void kmat_epilogue(const kd4_t (&acc)[4], const double* na, const double* nb2,
                                              const int* eqr, const double* kexp, int wm, int wn, bool dtile,
                                              double scale, double dadd, double (&vals)[4][4]) {
#pragma clang fp contract(off)   // explicit fma only: the same rounding in both kernels
  const int lane = threadIdx.x & 63, col = lane & 15, rq = lane >> 4;
  const double nbv[2] = {nb2[wn + col], nb2[wn + 16 + col]};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double d2 = fmax(fma(-2.0, acc[q][r], na[wm + (q >> 1) * 16 + rq + 4 * r] + nbv[q & 1]), 0.0);
#if defined(EVR_KMAT_PROF) && (EVR_KMAT_PROF & 1)   // profiling builds only: no kernel evaluation
      vals[q][r] = scale * d2;
#else
      vals[q][r] = scale * kernel_value_r(KIND, d2, kexp);
#endif
    }
  // the diagonal entries, apart (a per-entry test in the loop above became a branch around
  // each entry's LDS read): identical points take d2 = 0, every diagonal entry gets dadd
  if (dtile) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int li = wm + (q >> 1) * 16 + rq + 4 * r, lj = wn + (q & 1) * 16 + col;
        if (li == lj) vals[q][r] = (eqr[li] ? scale * kernel_value_r(KIND, 0.0, kexp) : vals[q][r]) + dadd;
      }
  }
}

// the tile's values to K (n1 x n2, row-major): interior tiles without per-entry guards
__device__ __forceinline__ void kmat_store(double* Kb, int n1, int n2, int i0, int j0, int wm, int wn,
                                           const double (&vals)[4][4]) {
  const int lane = threadIdx.x & 63, col = lane & 15, rq = lane >> 4;
  const int gi0 = i0 + wm + rq, gj0 = j0 + wn + col;
#if defined(EVR_KMAT_PROF) && (EVR_KMAT_PROF & 2)   // profiling builds only: no output stream
  if (vals[0][0] != -1.25) return;
#endif
  if (i0 + KT <= n1 && j0 + KT <= n2) {
    double* p = Kb + (size_t)gi0 * n2 + gj0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) p[(size_t)((q >> 1) * 16 + 4 * r) * n2 + (q & 1) * 16] = vals[q][r];
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = gi0 + (q >> 1) * 16 + 4 * r, gj = gj0 + (q & 1) * 16;
      if (gi < n1 && gj < n2) Kb[(size_t)gi * n2 + gj] = vals[q][r];
    }
}

// Operand staging of the MFMA kernels: rows i0.. of X1 and j0.. of X2 (zero beyond n1 / n2),
// the d columns normalised ((x - shift) scale) and divided by the lengthscales, transposed
// into As[k][r] / Bs[k][r] (zero for k >= d).  Every load is issued before the first wait.
// DP | 256 (16, 32, 64): thread tid owns column k = tid % DP of rows tid / DP + (256 / DP) t,
// one reciprocal of its lengthscale and branch-free clamped loads; DP = 48 the generic map.
template <int DP>
__device__ __forceinline__ void kmat_stage(double (*As)[KT + 2], double (*Bs)[KT + 2], const double* X1,
                                           const double* sh1, const double* sc1, const double* X2,
                                           const double* sh2, const double* sc2, const double* lsb, int n1,
                                           int n2, int d, int i0, int j0) {
  const int tid = threadIdx.x;
  if constexpr (256 % DP == 0) {
    constexpr int RS = 256 / DP, NE = KT / RS;
    const int k = tid % DP, rr = tid / DP;
    const bool kin = k < d;
    const int kc = kin ? k : 0;
    const double il = 1.0 / lsb[kc];
    const double s1 = sh1 ? sh1[kc] : 0.0, c1 = sc1 ? sc1[kc] : 1.0;
    const double s2 = sh2 ? sh2[kc] : 0.0, c2 = sc2 ? sc2[kc] : 1.0;
    double v[NE], w[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int r = rr + RS * t;
      v[t] = X1[(size_t)min(i0 + r, n1 - 1) * d + kc];
      w[t] = X2[(size_t)min(j0 + r, n2 - 1) * d + kc];
    }
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int r = rr + RS * t;
      // (v - 0) and v * 1 are exact: the same values as the optional shift / scale steps
      As[k][r] = (kin && i0 + r < n1) ? (v[t] - s1) * c1 * il : 0.0;
      Bs[k][r] = (kin && j0 + r < n2) ? (w[t] - s2) * c2 * il : 0.0;
    }
  } else {
    constexpr int NE = (KT * DP + 255) / 256;
    double v[NE], w[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int e = tid + 256 * t;
      const int r = e / DP, k = e - r * DP;
      v[t] = 0.0;
      w[t] = 0.0;
      if (e < KT * DP && k < d) {
        if (i0 + r < n1) v[t] = X1[(size_t)(i0 + r) * d + k];
        if (j0 + r < n2) w[t] = X2[(size_t)(j0 + r) * d + k];
      }
    }
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int e = tid + 256 * t;
      const int r = e / DP, k = e - r * DP;
      if (e < KT * DP) {
        double a = 0.0, c = 0.0;
        if (k < d) {
          const double il = 1.0 / lsb[k];
          if (i0 + r < n1) a = (v[t] - (sh1 ? sh1[k] : 0.0)) * (sc1 ? sc1[k] : 1.0) * il;
          if (j0 + r < n2) c = (w[t] - (sh2 ? sh2[k] : 0.0)) * (sc2 ? sc2[k] : 1.0) * il;
        }
        As[k][r] = a;
        Bs[k][r] = c;
      }
    }
  }
}

// squared row norms of the staged operands (one wave each, k in order) and, on a diagonal
// tile, which rows of the two operands are bitwise identical (a third wave)
template <int DP>
__device__ __forceinline__ void kmat_norms(const double (*As)[KT + 2], const double (*Bs)[KT + 2], double* na,
                                           double* nb2, int* eqr, bool dtile) {
  const int wave = threadIdx.x >> 6, r = threadIdx.x & 63;
  if (wave < 2) {
    const double (*S)[KT + 2] = wave == 0 ? As : Bs;
    double sq = 0.0;
#pragma unroll
    for (int k = 0; k < DP; ++k) sq = fma(S[k][r], S[k][r], sq);
    (wave == 0 ? na : nb2)[r] = sq;
  } else if (wave == 2 && dtile) {
    int eq = 1;
#pragma unroll
    for (int k = 0; k < DP; ++k) eq &= As[k][r] == Bs[k][r];
    eqr[r] = eq;
  }
}

template <int DP, int KIND>
__global__ __launch_bounds__(256) void kmat_mfma_kernel(int kind, int n1, int n2, int d,
                                                        const double* __restrict__ X1, const double* __restrict__ sh1,
                                                        const double* __restrict__ sc1, const double* __restrict__ X2,
                                                        const double* __restrict__ sh2, const double* __restrict__ sc2,
                                                        const double* __restrict__ ls, const double* __restrict__ os,
                                                        const double* __restrict__ dg, double* __restrict__ K) {
  // operand tiles As / Bs
  constexpr int OPS = 2 * DP * (KT + 2);
  __shared__ double smem[OPS];
  double (*As)[KT + 2] = reinterpret_cast<double (*)[KT + 2]>(smem);
  double (*Bs)[KT + 2] = reinterpret_cast<double (*)[KT + 2]>(smem + DP * (KT + 2));
  __shared__ double na[KT], nb2[KT];
  __shared__ int eqr[KT];   // diagonal tiles: row r of both operands bitwise identical
  __shared__ double kexp[64];
  const int gx = gridDim.x, gy = gridDim.y;
  const int t = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int bx = t % gx, by = (t / gx) % gy, b = t / (gx * gy);
  const int i0 = by * KT, j0 = bx * KT;
  const double* lsb = ls + (size_t)b * d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if defined(EVR_KMAT_PROF) && (EVR_KMAT_PROF & 16)   // profiling builds only: the grid's dispatch alone
  if (lsb[tid & 31] == -1.25) K[0] = 0.0;
  return;
#endif
  kmat_stage<DP>(As, Bs, X1, sh1, sc1, X2, sh2, sc2, lsb, n1, n2, d, i0, j0);
  kexp_stage(kexp, tid, 256);
  __syncthreads();
#if defined(EVR_KMAT_PROF) && (EVR_KMAT_PROF & 4)   // profiling builds only: staging alone
  if (As[tid & 31][tid >> 5] == -1.25) K[0] = Bs[0][0];
  return;
#endif
  kmat_norms<DP>(As, Bs, na, nb2, eqr, i0 == j0);
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int i = lane & 15, kq = lane >> 4;
  kd4_t acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
  for (int kk = 0; kk < DP; kk += 4) {
    const double a0 = As[kk + kq][wm + i], a1 = As[kk + kq][wm + 16 + i];
    const double b0 = Bs[kk + kq][wn + i], b1 = Bs[kk + kq][wn + 16 + i];
    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
  }
  __syncthreads();   // na / nb2
#if defined(EVR_KMAT_PROF) && (EVR_KMAT_PROF & 8)   // profiling builds only: staging, norms, MFMA
  if (acc[0][0] + acc[3][3] + na[lane] == -1.25) K[0] = acc[1][1] + acc[2][2];
  return;
#endif
  const double scale = os ? os[b] : 1.0;
  const double dadd = dg ? dg[b] : 0.0;
  double* Kb = K + (size_t)b * n1 * n2;
  // every value is formed first and the stores follow: a per-entry bounds branch around the
  // kernel evaluation serialised the 16 entries' dependent chains (SQ: ~90 VALU + 39 SALU per
  // entry, round 5); out-of-range entries compute on the zero padding and are not stored
  double vals[4][4];
  kmat_epilogue<KIND>(acc, na, nb2, eqr, kexp, wm, wn, i0 == j0, scale, dadd, vals);
  kmat_store(Kb, n1, n2, i0, j0, wm, wn, vals);
  // (LDS-staged row-segment epilogues, with and without non-temporal or 16-byte stores, were
  // measured slower at config 5 and removed in round 6: profiles/r05/p/kmat_epi*.json)
}

// Symmetric train matrix K(X, X) (the GP fit's case: both operands the same rows with the same
// normalisation): one workgroup per lower tile (I >= J) computes it exactly as
// kmat_mfma_kernel does (same staging, MFMA order and epilogue — u_i . u_j and u_j . u_i are
// the same products in the same k order, |u_i|^2 + |u_j|^2 commutes) and writes it twice: the
// tile in place and, for I > J, its transpose through LDS as 512-byte row segments.  Half the
// MFMA and epilogue work (the kernel is compute-heavy at d = 32: 17.7 us without the kernel
// evaluation vs 24.5 us, profiles/r04/u), the same output stream.
template <int DP, int KIND>
__global__ __launch_bounds__(256) void kmat_mfma_sym(int n, int d, int B, const double* __restrict__ X,
                                                     const double* __restrict__ sh, const double* __restrict__ sc,
                                                     const double* __restrict__ ls, const double* __restrict__ os,
                                                     const double* __restrict__ dg, double* __restrict__ K) {
  constexpr int OPS = 2 * DP * (KT + 2), OUT = KT * (KT + 1);
  __shared__ double smem[OPS > OUT ? OPS : OUT];
  double (*As)[KT + 2] = reinterpret_cast<double (*)[KT + 2]>(smem);
  double (*Bs)[KT + 2] = reinterpret_cast<double (*)[KT + 2]>(smem + DP * (KT + 2));
  __shared__ double na[KT], nb2[KT];
  __shared__ int eqr[KT];
  __shared__ double kexp[64];
  const int nt = (n + KT - 1) / KT, tpb = nt * (nt + 1) / 2;
  const int t = xcd_swizzle(blockIdx.x, gridDim.x);
  const int b = t / tpb, tl = t - b * tpb;
  int I = (int)((sqrt(8.0 * tl + 1.0) - 1.0) * 0.5);   // lower tiles row-major: row I holds I + 1 tiles
  while ((I + 1) * (I + 2) / 2 <= tl) ++I;
  while (I * (I + 1) / 2 > tl) --I;
  const int J = tl - I * (I + 1) / 2;
  const int i0 = I * KT, j0 = J * KT;
  const double* lsb = ls + (size_t)b * d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  kmat_stage<DP>(As, Bs, X, sh, sc, X, sh, sc, lsb, n, n, d, i0, j0);
  kexp_stage(kexp, tid, 256);
  __syncthreads();
  kmat_norms<DP>(As, Bs, na, nb2, eqr, I == J);
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int i = lane & 15, kq = lane >> 4;
  kd4_t acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
  for (int kk = 0; kk < DP; kk += 4) {
    const double a0 = As[kk + kq][wm + i], a1 = As[kk + kq][wm + 16 + i];
    const double b0 = Bs[kk + kq][wn + i], b1 = Bs[kk + kq][wn + 16 + i];
    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
  }
  __syncthreads();   // na / nb2 / eqr; every wave's As / Bs reads are done
  const double scale = os ? os[b] : 1.0;
  const double dadd = dg ? dg[b] : 0.0;
  double* Kb = K + (size_t)b * n * n;
  const int col = lane & 15, rq = lane >> 4;
  double vals[4][4];
  kmat_epilogue<KIND>(acc, na, nb2, eqr, kexp, wm, wn, I == J, scale, dadd, vals);
  kmat_store(Kb, n, n, i0, j0, wm, wn, vals);
  if (I == J) return;
  double (*T)[KT + 1] = reinterpret_cast<double (*)[KT + 1]>(smem);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) T[wm + (q >> 1) * 16 + rq + 4 * r][wn + (q & 1) * 16 + col] = vals[q][r];
  __syncthreads();
  const int gc = i0 + lane;   // column of the transposed tile
#pragma unroll 4
  for (int rr = wave; rr < KT; rr += 4) {
    const int gr = j0 + rr;
    if (gr < n && gc < n) Kb[(size_t)gr * n + gc] = T[lane][rr];
  }
}

// loads of up to KG_B outputs of one row are issued together (the b-outer loop serialised
// one global round trip per output: 22 us at m = 5, n = b = 512 on MI355X), 1/ls and the
// output scales of the chunk sit in LDS.
constexpr int KG_B = 8;
// outputs per LDS chunk / G loads in flight per row: 4 up to 8 dims (the compiler keeps the
// chunk's 1/ls table in registers across the row loop: 8 outputs x 8 dims did not fit two
// waves per SIMD), 8 up to 16 dims; at 32 / 64 dims the
// fully unrolled (output x dim) body of 8 outputs did not stay in registers (1.7 / 5.2 KB of
// scratch per lane), so those instantiations take 2 outputs per round and form the scaled
// differences twice instead of keeping a diff[] row
template <int MAXD>
__host__ __device__ constexpr int kg_outputs() { return MAXD <= 8 ? 4 : MAXD <= 16 ? KG_B : 2; }
// (256, 2) at MAXD = 8: unbounded, the unrolled (output x dim) body took 292 VGPRs + 36 AGPRs —
// one wave per SIMD, so the b = 512 pass's 2048 waves ran in two rounds (20.6 us)
template <int MAXD>
__global__ __launch_bounds__(256, MAXD <= 8 ? 2 : 1) void kcross_grad_kernel(int kind, int B, int n1, int n2, int d, int rows_per,
                                                          const double* __restrict__ X1,
                                                          const double* __restrict__ sh1,
                                                          const double* __restrict__ sc1,
                                                          const double* __restrict__ X2,
                                                          const double* __restrict__ sh2,
                                                          const double* __restrict__ sc2,
                                                          const double* __restrict__ ls,
                                                          const double* __restrict__ os,
                                                          const double* __restrict__ G, double* __restrict__ part) {
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cx;
  const int split = blockIdx.y;
  const int i0 = split * rows_per, i1 = min(n1, i0 + rows_per);
  __shared__ double red[4][64][MAXD];
  constexpr int KGO = kg_outputs<MAXD>();
  __shared__ double il_s[KGO][MAXD];
  __shared__ double os_s[KGO];
  double x2[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    double w = 0.0;
    if (k < d && c < n2) {
      w = X2[(size_t)c * d + k];
      if (sh2) w -= sh2[k];
      if (sc2) w *= sc2[k];
    }
    x2[k] = w;
  }
  double acc[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k) acc[k] = 0.0;
  const size_t bstride = (size_t)n1 * n2;
  for (int b0 = 0; b0 < B; b0 += KGO) {
    const int nb = min(KGO, B - b0);
    __syncthreads();
    for (int t = threadIdx.x; t < nb * MAXD; t += blockDim.x) {
      const int bb = t / MAXD, k = t % MAXD;
      il_s[bb][k] = (k < d) ? 1.0 / ls[(size_t)(b0 + bb) * d + k] : 0.0;
    }
    if ((int)threadIdx.x < nb) os_s[threadIdx.x] = os ? os[b0 + threadIdx.x] : 1.0;
    __syncthreads();
    if (c >= n2) continue;
    const double* Gc = G + (size_t)b0 * bstride + c;
#pragma unroll 1
    for (int i = i0 + ry; i < i1; i += 4) {
      double g[KGO];
#pragma unroll
      for (int bb = 0; bb < KGO; ++bb) g[bb] = (bb < nb) ? Gc[bb * bstride + (size_t)i * n2] : 0.0;
      double x1[MAXD];
#pragma unroll
      for (int k = 0; k < MAXD; ++k) {
        double v = 0.0;
        if (k < d) {
          v = X1[(size_t)i * d + k];
          if (sh1) v -= sh1[k];
          if (sc1) v *= sc1[k];
        }
        x1[k] = v;
      }
#pragma unroll
      for (int bb = 0; bb < KGO; ++bb) {
        if (bb < nb) {
          double d2 = 0.0;
#pragma unroll
          for (int k = 0; k < MAXD; ++k) {
            if (k < d) {
              const double df = (x2[k] - x1[k]) * il_s[bb][k];
              d2 = fma(df, df, d2);
            }
          }
          const double sgl = g[bb] * os_s[bb] * kernel_dscale(kind_of(kind, b0 + bb), d2);
#pragma unroll
          for (int k = 0; k < MAXD; ++k)
            if (k < d) {
              const double il = il_s[bb][k];
              acc[k] = fma(sgl, ((x2[k] - x1[k]) * il) * il, acc[k]);   // (x2 - x1)/ls^2
            }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXD; ++k) red[ry][cx][k] = acc[k];
  __syncthreads();
  if (ry == 0 && c < n2) {
    for (int k = 0; k < d; ++k) {
      const double v = ((red[0][cx][k] + red[1][cx][k]) + red[2][cx][k]) + red[3][cx][k];
      part[((size_t)split * n2 + c) * d + k] = v;
    }
  }
}

__global__ void kcross_grad_reduce(int nsplit, int n2, int d, const double* __restrict__ part,
                                   const double* __restrict__ sc2, double* __restrict__ dX2) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)n2 * d) return;
  const int k = (int)(e % d);
  const double sck = sc2 ? sc2[k] : 1.0;
  double v = 0.0;
  // 32 unconditional loads (clamped indices) in flight per round, summed in split order
  // afterwards: one memory round trip per 32 splits (the guarded unroll-8 loop waited per 8)
  for (int s0 = 0; s0 < nsplit; s0 += 32) {
    double t[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) t[u] = part[(size_t)min(s0 + u, nsplit - 1) * n2 * d + e];
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (s0 + u < nsplit) v += t[u];
  }
  dX2[e] = v * sck;
}

// row split of kcross_grad: up to 2048 blocks, >= 8 rows per block (two per row group).  At
// the b = 512 evaluation pass (n1 = 512, 8 column tiles) that is 512 blocks: two waves per
// SIMD instead of one (the 16-row floor left 256 blocks, one wave per SIMD and nothing to
// hide the G loads behind: 18.8 us for a 10.5 MB read)
static int kcross_nsplit(int n1, int n2) {
  const int ct = cdiv(n2, 64);
  int ns = cdiv(2048, ct);
  ns = std::max(1, std::min(ns, cdiv(n1, 8)));
  return ns;
}

size_t kcross_grad_ws_doubles(int n1, int n2, int d) { return (size_t)kcross_nsplit(n1, n2) * n2 * d; }

int kcross_grad_launch(hipStream_t s, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                       const double* scale1, const double* X2, const double* shift2, const double* scale2,
                       const double* lengthscales, const double* outputscale, const double* G, double* dX2,
                       double* work) {
  const int ns = kcross_nsplit(n1, n2);
  const int rows_per = cdiv(n1, ns);
  dim3 grid(cdiv(n2, 64), ns);
#define LAUNCH(MD)                                                                                         \
  kcross_grad_kernel<MD><<<grid, 256, 0, s>>>(kind, B, n1, n2, d, rows_per, X1, shift1, scale1, X2, shift2, \
                                              scale2, lengthscales, outputscale, G, work)
  if (d <= 8) LAUNCH(8);
  else if (d <= 16) LAUNCH(16);
  else if (d <= 32) LAUNCH(32);
  else LAUNCH(64);
#undef LAUNCH
  EVR_LAUNCH_CHECK();
  kcross_grad_reduce<<<cdiv((long long)n2 * d, 256), 256, 0, s>>>(ns, n2, d, work, scale2, dX2);
  EVR_LAUNCH_CHECK();
  return 0;
}

// part[b][i][k] = sum_j W[b][i][j] * dK_b[i][j]/dls_k, dK/dls_k = -dscale * diff_k^2 / ls_k^3
// (diff in normalized units).  One wave per (row i, output b), four rows per block: lane l sums
// j = l, l + 64, ... (its W loads and the row's inputs all issued before the arithmetic), then
// one fixed xor butterfly per dimension — no LDS, no barrier.  (The former block per row, 256
// threads over j, gave 2560 blocks at n = 512, B = 5: two residency rounds, 20.4 us.)  Rows are
// summed afterwards in a fixed order by colsum_kernel, so the MLL gradient is bitwise
// reproducible.
constexpr int KLS_ROWS = 4;
template <int MAXD>
__global__ __launch_bounds__(256) void kls_grad_kernel(int kind, int n, int d, const double* __restrict__ X,
                                                       const double* __restrict__ ls,
                                                       const double* __restrict__ W, double* __restrict__ part) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * KLS_ROWS + (threadIdx.x >> 6);
  if (i >= n) return;   // whole waves (no barrier below)
  const double* lsb = ls + (size_t)b * d;
  const double* Wr = W + ((size_t)b * n + i) * n;
  const int kb = kind_of(kind, b);
  double xi[MAXD], il[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    xi[k] = k < d ? X[(size_t)i * d + k] : 0.0;
    il[k] = k < d ? 1.0 / lsb[k] : 0.0;
  }
  double acc[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k) acc[k] = 0.0;
  // UJ columns per lane and round, their W entries (coalesced rows) in flight together; one
  // above 8 dims (the unrolled body would not stay in registers).  (Preloading the columns'
  // inputs as well: 147 VGPRs, 16.8 vs 15.5 us.)
  constexpr int UJ = MAXD <= 8 ? 4 : 1;
  for (int j0 = 0; j0 < n; j0 += 64 * UJ) {
    double w[UJ];
#pragma unroll
    for (int u = 0; u < UJ; ++u) w[u] = Wr[min(j0 + lane + 64 * u, n - 1)];
#pragma unroll
    for (int u = 0; u < UJ; ++u) {
      const int j = j0 + lane + 64 * u;
      if (j >= n) break;
      double sq[MAXD];
      double d2 = 0.0;
#pragma unroll
      for (int k = 0; k < MAXD; ++k)
        if (k < d) {
          const double df = (xi[k] - X[(size_t)j * d + k]) * il[k];
          sq[k] = df * df;
          d2 += sq[k];
        }
      const double s = -w[u] * kernel_dscale(kb, d2);
#pragma unroll
      for (int k = 0; k < MAXD; ++k)
        if (k < d) acc[k] = fma(s, sq[k] * il[k], acc[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    if (k < d) {
      double v = acc[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) part[((size_t)b * n + i) * d + k] = v;
    }
  }
}

// Above 16 dims: one block per (row i, output b), 256 threads over j (the wave-per-row form's
// per-lane (dimension x column) arrays do not stay in registers there).
template <int MAXD>
__global__ __launch_bounds__(256) void kls_grad_block_kernel(int kind, int n, int d, const double* __restrict__ X,
                                                       const double* __restrict__ ls,
                                                       const double* __restrict__ W, double* __restrict__ part) {
  const int b = blockIdx.y;
  const int i = blockIdx.x;
  const int tid = threadIdx.x;
  const double* lsb = ls + (size_t)b * d;
  const double* Wb = W + (size_t)b * n * n;
  __shared__ double red[256];
  double xi[MAXD], il[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k)
    if (k < d) {
      xi[k] = X[(size_t)i * d + k];
      il[k] = 1.0 / lsb[k];
    }
  double acc[MAXD];
#pragma unroll
  for (int k = 0; k < MAXD; ++k) acc[k] = 0.0;
  for (int j = tid; j < n; j += 256) {
    const double w = Wb[(size_t)i * n + j];
    double sq[MAXD];
    double d2 = 0.0;
#pragma unroll
    for (int k = 0; k < MAXD; ++k)
      if (k < d) {
        const double df = (xi[k] - X[(size_t)j * d + k]) * il[k];
        sq[k] = df * df;
        d2 += sq[k];
      }
    const double s = -w * kernel_dscale(kind_of(kind, b), d2);
#pragma unroll
    for (int k = 0; k < MAXD; ++k)
      if (k < d) acc[k] = fma(s, sq[k] * il[k], acc[k]);
  }
  // all d sums at once: a fixed xor butterfly per wave, then the four waves' partials in wave
  // order (one barrier; the former per-dimension LDS tree took 9 barriers per dimension)
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    if (k < d) {
      double v = acc[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) red[wave * MAXD + k] = v;
    }
  }
  __syncthreads();
  if (tid < d) {
    const double v = ((red[tid] + red[MAXD + tid]) + red[2 * MAXD + tid]) + red[3 * MAXD + tid];
    part[((size_t)b * n + i) * d + tid] = v;
  }
}

// out[b][k] = sum_i part[b][i][k]: one block per (b, k), strided partials + fixed LDS tree
__global__ __launch_bounds__(256) void colsum_kernel(int B, int n, int d, const double* __restrict__ part,
                                                     double* __restrict__ out) {
  const int b = blockIdx.x / d, k = blockIdx.x % d;
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += part[((size_t)b * n + i) * d + k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[(size_t)b * d + k] = red[0];
}

// Scalars of the exact MLL per output b:
// out[b] = {logdet = 2 sum log L_ii, quad = r.alpha, trKinv = ||Linv||_F^2, sum alpha, sum alpha^2}
// Pass 1: grid (B, MT_CHUNKS): rows i = chunk, chunk + MT_CHUNKS, ... of Linv read coalesced
// (threads over columns); per-chunk partials.  Pass 2 sums the chunks in a fixed order.
constexpr int MT_CHUNKS = 32;

__global__ __launch_bounds__(256) void mll_terms_kernel(int n, const double* __restrict__ L,
                                                        const double* __restrict__ Linv,
                                                        const double* __restrict__ r,
                                                        const double* __restrict__ alpha,
                                                        double* __restrict__ part) {
  // chunk ch: ||Linv||_F^2 over a contiguous 1/MT_CHUNKS of the n x n elements (the upper
  // triangle is exactly zero), 8 loads in flight per thread; the O(n) terms of rows
  // [ch*rc, ch*rc + rc) one row per thread
  const int b = blockIdx.x, ch = blockIdx.y;
  const int tid = threadIdx.x;
  const double* Lb = L + (size_t)b * n * n;
  const double* Ib = Linv + (size_t)b * n * n;
  const double* rb = r + (size_t)b * n;
  const double* ab = alpha + (size_t)b * n;
  double t[5] = {0, 0, 0, 0, 0};
  const size_t nn = (size_t)n * n, per = (nn + MT_CHUNKS - 1) / MT_CHUNKS;
  const size_t beg = ch * per, end = min(nn, beg + per);
  for (size_t e0 = beg + tid; e0 < end; e0 += 8 * 256) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t e = e0 + (size_t)u * 256;
      v[u] = e < end ? Ib[e] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) t[2] = fma(v[u], v[u], t[2]);
  }
  const int rc = (n + MT_CHUNKS - 1) / MT_CHUNKS;
  for (int i = ch * rc + tid; i < min(n, ch * rc + rc); i += 256) {
    t[0] += log(Lb[(size_t)i * n + i]);
    t[1] = fma(rb[i], ab[i], t[1]);
    t[3] += ab[i];
    t[4] = fma(ab[i], ab[i], t[4]);
  }
  __shared__ double red[5][256];
#pragma unroll
  for (int q = 0; q < 5; ++q) red[q][tid] = t[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o)
#pragma unroll
      for (int q = 0; q < 5; ++q) red[q][tid] += red[q][tid + o];
    __syncthreads();
  }
  if (tid < 5) part[((size_t)b * MT_CHUNKS + ch) * 5 + tid] = red[tid][0];
}

__global__ void mll_terms_finalize(int B, const double* __restrict__ part, double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * 5) return;
  const int b = e / 5, q = e % 5;
  double s = 0.0;
#pragma unroll 8
  for (int ch = 0; ch < MT_CHUNKS; ++ch) s += part[((size_t)b * MT_CHUNKS + ch) * 5 + q];
  out[e] = (q == 0) ? 2.0 * s : s;
}

// Column reduction of R = [Linv; alpha^T] K_x: block = 64 test points (lanes, coalesced
// rows) x 16 row groups (waves of 64 threads... 1024 threads); every thread sums its rows
// with 4 independent accumulators, the 16 group partials are combined in a fixed order.
__global__ __launch_bounds__(1024) void posterior_finalize_kernel(int B, int n, int nt, const double* __restrict__ R,
                                                                  const double* __restrict__ cc,
                                                                  const double* __restrict__ ym,
                                                                  const double* __restrict__ ys,
                                                                  const double* __restrict__ kxx,
                                                                  const double* __restrict__ noise,
                                                                  double* __restrict__ mean, double* __restrict__ var) {
  const int b = blockIdx.y;
  const int tx = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int t = blockIdx.x * 64 + tx;
  __shared__ double part[16][64];
  const double* Rb = R + (size_t)b * (n + 1) * nt;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (t < nt) {
    int i = g;
    for (; i + 48 < n; i += 64) {
      const double v0 = Rb[(size_t)i * nt + t], v1 = Rb[(size_t)(i + 16) * nt + t];
      const double v2 = Rb[(size_t)(i + 32) * nt + t], v3 = Rb[(size_t)(i + 48) * nt + t];
      s0 = fma(v0, v0, s0);
      s1 = fma(v1, v1, s1);
      s2 = fma(v2, v2, s2);
      s3 = fma(v3, v3, s3);
    }
    for (; i < n; i += 16) {
      const double v = Rb[(size_t)i * nt + t];
      s0 = fma(v, v, s0);
    }
  }
  part[g][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && t < nt) {
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) ss += part[k][tx];
    const double a = Rb[(size_t)n * nt + t];
    const double s = ys[b];
    mean[(size_t)b * nt + t] = ym[b] + s * (cc[b] + a);
    double v = kxx[b] - ss;
    if (noise) v += noise[b];
    var[(size_t)b * nt + t] = s * s * v;
  }
}

// ---------------------------------------------------------------------------------------
// Posterior projection (gemm_core.hpp engine): per output j, V = L^-1 K_* (n x nt) is never
// stored — each 32-row tile writes the partial sums of squares of its rows per test point,
// and the tiles of the last row block (the only ones whose k range is the whole of [0, n))
// also form the mean row alpha^T K_* from the staged K_* tiles.  L^-1 is lower triangular:
// row tile [m0, m0 + 32) contracts over k < m0 + 32 only (half the flops of the dense
// product; the skipped entries are exact zeros).  Longer row tiles are dispatched first.
// ---------------------------------------------------------------------------------------
// 32 x 64 tiles where they still give >= 4 workgroups per CU (the metric's 5 x 512 x 1024:
// 1280; B operand traffic per flop halved, 60.0 vs 64.2 us for the whole posterior), else
// 32 x 32 (the single-output config 2: 256 workgroups).  Wider (32 x 128) measured slower
// (67 us), and an XCD-owned column-tile order no different (tools/bench_post.py, profiles/r06/py)
using PostCfg = DgCfg<32, 32, 16, false>;
using PostCfgW = DgCfg<32, 64, 16, false>;
constexpr int POST_NT = PostCfg::BM;

// alpha^T B over the staged k-steps: the step's 16 alpha entries ride in the B image's first
// padding column (thread t < 16 loads alpha[k0 + t] with the operand fetch and stages it);
// thread (column c = tid % BN, row group g = tid / BN) accumulates rows g, g + NG, ... of every step
template <class C>
struct PostMeanHook {
  static constexpr int NG = 256 / C::BN, RPG = C::BK / NG;
  const double* alpha;   // nullptr: not the last row block
  int n;
  double av;
  double acc;
  __device__ __forceinline__ void prefetch(int k0) {
    if (!alpha) return;
    const int k = k0 + (int)threadIdx.x;
    if (threadIdx.x < C::BK) av = k < n ? alpha[k] : 0.0;
  }
  __device__ __forceinline__ void stage(double* Bs) {
    if (alpha && threadIdx.x < C::BK) Bs[threadIdx.x * C::BST + C::BN] = av;
  }
  __device__ __forceinline__ void step(const double* Bs, int, int) {
    if (!alpha) return;
    const int g = threadIdx.x / C::BN, c = threadIdx.x % C::BN;
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      const int r = g + NG * t;
      acc = fma(Bs[r * C::BST + C::BN], Bs[r * C::BST + c], acc);
    }
  }
};

// Posterior moments, fused into the projection: the last workgroup to finish a column tile
// (per output; an arrival counter zeroed by the K_* launch) sums the tile's row partials in the
// fixed order of the former post_finalize_kernel and writes mean and variance — one launch
// boundary less (the separate kernel took 4.9 us at the metric's shape)
struct PostMoments {
  int* cnt;             // B x gx arrival counters, 0 on entry
  const double* cc;     // constant means (B)
  const double* ym;
  const double* ys;
  const double* kxx;
  const double* noise;  // nullptr: latent posterior
  double* mean;
  double* var;
};

template <class C, bool VEC>
__global__ __launch_bounds__(256, 4) void post_proj_kernel(int n, int nt, const double* __restrict__ Mm,
                                                           const double* __restrict__ Kx, double* __restrict__ Pn,
                                                           double* __restrict__ mrow, PostMoments pm) {
  __shared__ double lds[C::LDS_DOUBLES];
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  // dispatch order = descending k range (the longest row blocks start first), then output,
  // then column tile; consecutive workgroups go round-robin over the XCDs, so every XCD gets
  // the same mix of long and short tiles (an XCD-contiguous tile order would hand whole
  // ranges of long tiles to some XCDs and short ones to others)
  const int f = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int bx = f % gx, j = (f / gx) % gz, by = gy - 1 - f / (gx * gz);
  const int m0 = by * C::BM, n0 = bx * C::BN;
  const double* A = Mm + (size_t)j * (n + 1) * n;
  const double* B = Kx + (size_t)j * n * nt;
  const int kend = min(n, m0 + C::BM);
  PostMeanHook<C> hook{by == gy - 1 ? A + (size_t)n * n : nullptr, n, 0.0, 0.0};
  dg_double4 acc[C::FM][C::FN];
  dg_mainloop<C>(
      lds, 0, kend,
      [&](int r, int k) -> dg_double2 {
        const bool ok = m0 + r < n;
        return dg_pair<VEC>(A + (size_t)(m0 + r) * n + k, ok && k < kend, ok && k + 1 < kend);
      },
      [&](int k, int c) -> dg_double2 {
        const bool ok = k < kend;
        return dg_pair<VEC>(B + (size_t)k * nt + n0 + c, ok && n0 + c < nt, ok && n0 + c + 1 < nt);
      },
      acc, hook);
  // the mainloop ended on a barrier: its LDS is free.  Column sums of squares over the
  // tile's rows (fixed order: the 16 rows of a wave by xor-shuffles, then the two waves)
  constexpr int BN = C::BN, NG = PostMeanHook<C>::NG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, i = lane & 15, q = lane >> 4;
  double* red = lds;              // [2][BN]
  double* redm = lds + 2 * BN;    // [NG][BN]
#pragma unroll
  for (int bb = 0; bb < C::FN; ++bb) {
    double sq = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double val = acc[0][bb][r];
      if (m0 + wr * C::WM + q + 4 * r < n) sq = fma(val, val, sq);
    }
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    if (q == 0) red[wr * BN + wc * C::WN + bb * 16 + i] = sq;
  }
  if (hook.alpha) redm[tid] = hook.acc;
  __syncthreads();
  // the partials go out as device-coherent stores (past the per-XCD L2s, which a __threadfence
  // would have to write back whole: 3x slower with K_* dirty in them), each writer waits for
  // its stores to complete, then one thread counts the tile's arrival; the last arrival reads
  // the partials with device-coherent loads and finalises the column tile
  if (tid < BN && n0 + tid < nt) {
    __hip_atomic_store(Pn + ((size_t)j * gy + by) * nt + n0 + tid, red[tid] + red[BN + tid], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (hook.alpha) {
      double a = 0.0;
#pragma unroll
      for (int g = 0; g < NG; ++g) a += redm[g * BN + tid];
      __hip_atomic_store(mrow + (size_t)j * nt + n0 + tid, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this thread's stores have completed
  }
  __syncthreads();
  __shared__ int last;
  if (tid == 0) last = atomicAdd(pm.cnt + (size_t)j * gx + bx, 1) == gy - 1;
  __syncthreads();
  if (!last) return;
  const int c = n0 + tid;
  if (tid < BN && c < nt) {
    const double* P = Pn + (size_t)j * gy * nt + c;
    // row tile rt's partial goes to s0 (rt even) or s1 (rt odd) in increasing rt; loads in
    // batches of 8 so their latencies overlap
    const double mr = __hip_atomic_load(mrow + (size_t)j * nt + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    double s0 = 0.0, s1 = 0.0;
    for (int r0 = 0; r0 < gy; r0 += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = r0 + u < gy ? __hip_atomic_load(P + (size_t)(r0 + u) * nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0;
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        if (r0 + u < gy) s0 += v[u];
        if (r0 + u + 1 < gy) s1 += v[u + 1];
      }
    }
    const double ss = s0 + s1;
    const double sj = pm.ys[j];
    pm.mean[(size_t)j * nt + c] = pm.ym[j] + sj * (pm.cc[j] + mr);
    double v = pm.kxx[j] - ss;
    if (pm.noise) v += pm.noise[j];
    pm.var[(size_t)j * nt + c] = sj * sj * v;
  }
}


}  // namespace evr

using namespace evr;

namespace evr {
// graph-capturable MLL terms (mll_plan.hip): chunk partials only, reduced by the caller
size_t mll_terms_part_doubles(int B) { return (size_t)B * MT_CHUNKS * 5; }
int mll_terms_chunks() { return MT_CHUNKS; }
int mll_terms_partials(hipStream_t s, int B, int n, const double* L, const double* Linv, const double* r,
                       const double* alpha, double* part) {
  mll_terms_kernel<<<dim3(B, MT_CHUNKS), 256, 0, s>>>(n, L, Linv, r, alpha, part);
  EVR_LAUNCH_CHECK();
  return 0;
}
int kernel_matrix_launch(void* stream, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                         const double* scale1, const double* X2, const double* shift2, const double* scale2,
                         const double* lengthscales, const double* outputscale, const double* diag_add, double* K,
                         const unsigned long long* seq_src = nullptr, unsigned long long* seq_dst = nullptr,
                         double* x_dst = nullptr, int* zero_dst = nullptr, int nzero = 0);
}  // namespace evr

extern "C" {

int evr_kernel_matrix(void* stream, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                      const double* scale1, const double* X2, const double* shift2, const double* scale2,
                      const double* lengthscales, const double* outputscale, const double* diag_add, double* K) {
  return kernel_matrix_launch(stream, kind, B, n1, n2, d, X1, shift1, scale1, X2, shift2, scale2, lengthscales,
                              outputscale, diag_add, K);
}

}  // extern "C"

namespace evr {
// evr_kernel_matrix with the host-driven chain's copies (the evaluation's sequence number and
// the candidates to device memory): the VALU kernel (d < 16, one output family) only
int kernel_matrix_launch(void* stream, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                         const double* scale1, const double* X2, const double* shift2, const double* scale2,
                         const double* lengthscales, const double* outputscale, const double* diag_add, double* K,
                         const unsigned long long* seq_src, unsigned long long* seq_dst, double* x_dst,
                         int* zero_dst, int nzero) {
  EVR_CHECK(!seq_dst || (seq_src && d < 16 && kind < KIND_MIXED && n1 > 0 && n2 > 0),
            "kernel_matrix_launch: the sequence copy needs the VALU kernel (d < 16, one family)");
  EVR_CHECK(!x_dst || (d < 16 && kind < KIND_MIXED && n1 > 0 && n2 > 0 && n2 <= KT),
            "kernel_matrix_launch: the candidate copy needs the VALU kernel (d < 16, one family, n2 <= %d)", KT);
  EVR_CHECK(kind_code_ok(kind, B), "evr_kernel_matrix: bad kernel kind %d for %d outputs", kind, B);
  EVR_CHECK(B >= 1 && n1 >= 0 && n2 >= 0 && d >= 1 && d <= KMAXD, "evr_kernel_matrix: bad sizes B=%d n1=%d n2=%d d=%d",
            B, n1, n2, d);
  if (n1 == 0 || n2 == 0) return 0;
  // counters to zero (evr_gp_posterior): by kmat_kernel's first workgroup on the VALU path,
  // by a memset before the launches otherwise
  if (zero_dst && nzero > 0 && (kind >= KIND_MIXED || d >= 16)) {
    EVR_HIP(hipMemsetAsync(zero_dst, 0, sizeof(int) * (size_t)nzero, (hipStream_t)stream));
    zero_dst = nullptr;
  }
  if (kind >= KIND_MIXED) {
    // one family per output: one launch per run of consecutive outputs of the same family
    for (int b0 = 0; b0 < B;) {
      const int k = kind_of(kind, b0);
      int b1 = b0 + 1;
      while (b1 < B && kind_of(kind, b1) == k) ++b1;
      if (int rc = evr_kernel_matrix(stream, k, b1 - b0, n1, n2, d, X1, shift1, scale1, X2, shift2, scale2,
                                     lengthscales + (size_t)b0 * d, outputscale ? outputscale + b0 : nullptr,
                                     diag_add ? diag_add + b0 : nullptr, K + (size_t)b0 * n1 * n2))
        return rc;
      b0 = b1;
    }
    return 0;
  }
  dim3 grid(cdiv(n2, KT), cdiv(n1, KT), B);
  if (d >= 16) {   // matrix-core distance expansion (see kmat_mfma_kernel)
    hipStream_t s = (hipStream_t)stream;
    // the symmetric train matrix (the same operand pointer): lower tiles only (kmat_mfma_sym)
    if (X1 == X2 && n1 == n2 && shift1 == shift2 && scale1 == scale2 && d <= 64 && d != 48) {
      const int nt = cdiv(n1, KT);
      const long long tiles = (long long)nt * (nt + 1) / 2 * B;
#define KS(DP_, K_) kmat_mfma_sym<DP_, K_><<<(unsigned)tiles, 256, 0, s>>>(n1, d, B, X1, shift1, scale1, lengthscales, \
                                                                          outputscale, diag_add, K)
#define KSD(DP_)                                \
  if (kind == RBF) KS(DP_, RBF);                \
  else if (kind == MATERN05) KS(DP_, MATERN05); \
  else if (kind == MATERN15) KS(DP_, MATERN15); \
  else KS(DP_, MATERN25)
      if (d <= 16) { KSD(16); }
      else if (d <= 32) { KSD(32); }
      else { KSD(64); }
#undef KSD
#undef KS
      EVR_LAUNCH_CHECK();
      return 0;
    }
    // (persistent forms — a few workgroups per CU walking the tiles; in round 6 with the next
    // tile's operand loads issued ahead of this tile's stores and out-of-range entries dropped
    // by a buffer descriptor — measured slower at config 5: 20.1 / 21.1 / 24.3 us at 4 / 2 / 1
    // workgroups per CU vs 19.0 us one-shot, profiles/r06/o; removed)
#define KMK(DP_, K_)                                                                                      \
  kmat_mfma_kernel<DP_, K_><<<grid, 256, 0, s>>>(kind, n1, n2, d, X1, shift1, scale1, X2, shift2, scale2, \
                                                 lengthscales, outputscale, diag_add, K)
#define KM(DP_)                         \
  if (kind == RBF) KMK(DP_, RBF);           \
  else if (kind == MATERN05) KMK(DP_, MATERN05); \
  else if (kind == MATERN15) KMK(DP_, MATERN15); \
  else KMK(DP_, MATERN25)
    if (d <= 16) { KM(16); }
    else if (d <= 32) { KM(32); }
    else if (d <= 48) { KM(48); }
    else { KM(64); }
#undef KMK
#undef KM
    EVR_LAUNCH_CHECK();
    return 0;
  }
  constexpr int ra = 2;   // 32 rows per workgroup (16 and 64 measured slower)
  const size_t lds = (size_t)(KT + 16 * ra) * (d + 1) * sizeof(double);
  dim3 g(cdiv(n2, KT), cdiv(n1, 16 * ra), B);
#define KTK(RA_, K_)                                                                              \
  kmat_kernel<RA_, K_><<<g, 256, lds, (hipStream_t)stream>>>(kind, n1, n2, d, X1, shift1, scale1, X2, shift2, \
                                                             scale2, lengthscales, outputscale, diag_add, K,         \
                                                             seq_src, seq_dst, x_dst, zero_dst, nzero)
#define KT_(RA_)                         \
  if (kind == RBF) KTK(RA_, RBF);           \
  else if (kind == MATERN05) KTK(RA_, MATERN05); \
  else if (kind == MATERN15) KTK(RA_, MATERN15); \
  else KTK(RA_, MATERN25)
  KT_(2);
#undef KTK
#undef KT_
  EVR_LAUNCH_CHECK();
  return 0;
}
}  // namespace evr

extern "C" {

int evr_kernel_cross_grad(void* stream, int kind, int B, int n1, int n2, int d, const double* X1,
                          const double* shift1, const double* scale1, const double* X2, const double* shift2,
                          const double* scale2, const double* lengthscales, const double* outputscale,
                          const double* G, double* dX2, double* work) {
  EVR_CHECK(kind_code_ok(kind, B) && B >= 1 && d >= 1 && d <= KMAXD, "evr_kernel_cross_grad: bad args");
  if (n2 == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool own = work == nullptr;
  if (own) EVR_HIP(hipMallocAsync((void**)&work, sizeof(double) * kcross_grad_ws_doubles(n1, n2, d), s));
  const int rc = kcross_grad_launch(s, kind, B, n1, n2, d, X1, shift1, scale1, X2, shift2, scale2, lengthscales,
                                    outputscale, G, dX2, work);
  if (own) EVR_HIP(hipFreeAsync(work, s));
  return rc;
}

long long evr_kernel_cross_grad_workspace_doubles(int n1, int n2, int d) {
  return (n1 > 0 && n2 > 0 && d > 0) ? (long long)kcross_grad_ws_doubles(n1, n2, d) : 0;
}

int evr_kernel_lengthscale_grad(void* stream, int kind, int B, int n, int d, const double* X,
                                const double* lengthscales, const double* W, double* gls, double* work) {
  EVR_CHECK(kind_code_ok(kind, B) && B >= 1 && n >= 1 && d >= 1 && d <= KMAXD,
            "evr_kernel_lengthscale_grad: bad args");
  EVR_CHECK(work != nullptr, "evr_kernel_lengthscale_grad: work (B*n*d doubles) required");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(cdiv(n, KLS_ROWS), B), gridb(n, B);
#define LAUNCH(MD) kls_grad_kernel<MD><<<grid, 256, 0, s>>>(kind, n, d, X, lengthscales, W, work)
#define LAUNCHB(MD) kls_grad_block_kernel<MD><<<gridb, 256, 0, s>>>(kind, n, d, X, lengthscales, W, work)
  if (d <= 8) LAUNCH(8);
  else if (d <= 16) LAUNCH(16);
  else if (d <= 32) LAUNCHB(32);
  else LAUNCHB(64);
#undef LAUNCHB
#undef LAUNCH
  EVR_LAUNCH_CHECK();
  colsum_kernel<<<B * d, 256, 0, s>>>(B, n, d, work, gls);
  EVR_LAUNCH_CHECK();
  return 0;
}


int evr_gp_mll_terms(void* stream, int B, int n, const double* L, const double* Linv, const double* r,
                     const double* alpha, double* out) {
  EVR_CHECK(B >= 1 && n >= 1, "evr_gp_mll_terms: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  double* part = nullptr;
  EVR_HIP(hipMallocAsync((void**)&part, sizeof(double) * (size_t)B * MT_CHUNKS * 5, s));
  mll_terms_kernel<<<dim3(B, MT_CHUNKS), 256, 0, s>>>(n, L, Linv, r, alpha, part);
  EVR_LAUNCH_CHECK();
  mll_terms_finalize<<<cdiv(B * 5, 64), 64, 0, s>>>(B, part, out);
  EVR_LAUNCH_CHECK();
  EVR_HIP(hipFreeAsync(part, s));
  return 0;
}

int evr_gp_posterior_finalize(void* stream, int B, int n, int nt, const double* R, const double* c,
                              const double* ym, const double* ys, const double* kxx, const double* noise_add,
                              double* mean, double* var) {
  EVR_CHECK(B >= 1 && n >= 1 && nt >= 0, "evr_gp_posterior_finalize: bad sizes");
  if (nt == 0) return 0;
  dim3 grid(cdiv(nt, 64), B);
  posterior_finalize_kernel<<<grid, 1024, 0, (hipStream_t)stream>>>(B, n, nt, R, c, ym, ys, kxx, noise_add, mean,
                                                                    var);
  EVR_LAUNCH_CHECK();
  return 0;
}

long long evr_gp_posterior_workspace_doubles(int B, int n, int nt) {
  // K_* (B x n x nt), the row-tile partials (B x ceil(n / 32) x nt), the mean row (B x nt) and
  // the column tiles' arrival counters (B x ceil(nt / 32) ints)
  return (B > 0 && n > 0 && nt > 0)
             ? (long long)B * nt * ((long long)n + cdiv(n, POST_NT) + 1) + cdiv(B * cdiv(nt, PostCfg::BN), 2)
             : 0;
}

int evr_gp_posterior(void* stream, int B, int n, int nt, int d, int kind, const double* Xn, const double* X,
                     const double* shift, const double* scale, const double* lengthscales, const double* M,
                     const double* c, const double* ym, const double* ys, const double* kxx,
                     const double* noise_add, double* mean, double* var, double* work) {
  EVR_CHECK(B >= 1 && n >= 1 && nt >= 0 && d >= 1 && Xn && M && work, "evr_gp_posterior: bad arguments");
  if (nt == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int nrt = cdiv(n, POST_NT);
  double* Kx = work;                                   // B x n x nt
  double* Pn = Kx + (size_t)B * n * nt;                // B x nrt x nt
  double* mrow = Pn + (size_t)B * nrt * nt;            // B x nt
  int* cnt = (int*)(mrow + (size_t)B * nt);            // B x ceil(nt / 32)
  const int ncnt = B * cdiv(nt, PostCfg::BN);
  if (int rc = kernel_matrix_launch(stream, kind, B, n, nt, d, Xn, nullptr, nullptr, X, shift, scale, lengthscales,
                                    nullptr, nullptr, Kx, nullptr, nullptr, nullptr, cnt, ncnt))
    return rc;
  const PostMoments pm{cnt, c, ym, ys, kxx, noise_add, mean, var};
  const bool vec = n % 2 == 0 && nt % 2 == 0 && (uintptr_t)M % 16 == 0 && (uintptr_t)Kx % 16 == 0;
  if ((long long)cdiv(nt, PostCfgW::BN) * nrt * B >= 1024) {
    const dim3 grid(cdiv(nt, PostCfgW::BN), nrt, B);
    if (vec) post_proj_kernel<PostCfgW, true><<<grid, 256, 0, s>>>(n, nt, M, Kx, Pn, mrow, pm);
    else post_proj_kernel<PostCfgW, false><<<grid, 256, 0, s>>>(n, nt, M, Kx, Pn, mrow, pm);
  } else {
    const dim3 grid(cdiv(nt, PostCfg::BN), nrt, B);
    if (vec) post_proj_kernel<PostCfg, true><<<grid, 256, 0, s>>>(n, nt, M, Kx, Pn, mrow, pm);
    else post_proj_kernel<PostCfg, false><<<grid, 256, 0, s>>>(n, nt, M, Kx, Pn, mrow, pm);
  }
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
