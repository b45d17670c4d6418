// Dense float64 linear algebra for the GP hot path on gfx950:
//   * batched GEMM on the f64 matrix cores (v_mfma_f64_16x16x4_f64),
//   * batched Cholesky with the psd_safe_cholesky jitter ladder (one workgroup per
//     matrix, right-looking, NB=32 LDS diagonal block),
//   * batched triangular solve (L^-1 B / L^-T B) blocked by 64 rows through LDS.
// Replaces the [upstream] torch/LAPACK calls behind GPyTorch's Cholesky / solves
// (Appendix A.4).
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

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f64_kernel(int M, int N, int K, double alpha,
                                                       const double* __restrict__ A, int lda, long long sA,
                                                       const double* __restrict__ B, int ldb, long long sB,
                                                       double beta, double* __restrict__ C, int ldc, long long sC) {
  A += blockIdx.z * sA;
  B += blockIdx.z * sB;
  C += blockIdx.z * sC;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  __shared__ double As[GK][GT + GPAD];
  __shared__ double Bs[GK][GT + GPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  double4_t acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += GK) {
#pragma unroll
    for (int e0 = 0; e0 < GT * GK; e0 += 256) {
      const int e = e0 + tid;
      int mm, kk;
      if (!TA) { kk = e & 15; mm = e >> 4; } else { mm = e & 63; kk = e >> 6; }
      const int gm = m0 + mm, gk = k0 + kk;
      double v = 0.0;
      if (gm < M && gk < K) v = TA ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk];
      As[kk][mm] = v;
      int nn;
      if (!TB) { nn = e & 63; kk = e >> 6; } else { kk = e & 15; nn = e >> 4; }
      const int gn = n0 + nn, gk2 = k0 + kk;
      double w = 0.0;
      if (gn < N && gk2 < K) w = TB ? B[(size_t)gn * ldb + gk2] : B[(size_t)gk2 * ldb + gn];
      Bs[kk][nn] = w;
    }
    __syncthreads();
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
  auto store = [&](const double4_t& acc, int mi, int ni) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm + mi * 16 + rq + 4 * r;
      const int cc = n0 + wn + ni * 16 + col;
      if (row < M && cc < N) {
        double* p = C + (size_t)row * ldc + cc;
        *p = alpha * acc[r] + (beta == 0.0 ? 0.0 : beta * (*p));
      }
    }
  };
  store(acc00, 0, 0);
  store(acc01, 0, 1);
  store(acc10, 1, 0);
  store(acc11, 1, 1);
}

// ---------------------------------------------------------------------------------------
// Cholesky with psd_safe_cholesky semantics: try plain; on a non-positive (or NaN) pivot
// restart from A with total diagonal jitter jitter0 * 10^(t-1), t = 1..max_tries.
// ---------------------------------------------------------------------------------------
constexpr int CNB = 32;
constexpr int CT = 64;  // trailing-update tile

__global__ __launch_bounds__(1024) void chol_kernel(int n, const double* __restrict__ A, long long sA, int lda,
                                                    double* __restrict__ Lout, long long sL, int ldl, double jitter0,
                                                    int max_tries, double* __restrict__ jitter_used,
                                                    int* __restrict__ info) {
  const int b = blockIdx.x;
  A += b * sA;
  double* L = Lout + b * sL;
  __shared__ double D[CNB][CNB + 1];
  __shared__ double Pi[CT][CNB + 1];
  __shared__ double Pj[CT][CNB + 1];
  __shared__ int fail;
  const int tid = threadIdx.x, nt = blockDim.x;
  double jit = 0.0;
  for (int t = 0; t <= max_tries; ++t) {
    jit = (t == 0) ? 0.0 : jitter0 * pow(10.0, (double)(t - 1));
    for (long long e = tid; e < (long long)n * n; e += nt) {
      const int i = (int)(e / n), j = (int)(e % n);
      double v = (j <= i) ? A[(size_t)i * lda + j] : 0.0;
      if (i == j) v += jit;
      L[(size_t)i * ldl + j] = v;
    }
    if (tid == 0) fail = 0;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += CNB) {
      const int nb = min(CNB, n - k0);
      // (1) diagonal block: unnormalised right-looking elimination, one barrier per column
      for (int e = tid; e < nb * nb; e += nt) {
        const int i = e / nb, j = e % nb;
        D[i][j] = (j <= i) ? L[(size_t)(k0 + i) * ldl + k0 + j] : 0.0;
      }
      __syncthreads();
      for (int j = 0; j < nb; ++j) {
        const double p = D[j][j];
        if (!(p > 0.0)) break;  // uniform across the workgroup
        const double ip = 1.0 / p;
        const int rem = nb - j - 1;
        for (int e = tid; e < rem * rem; e += nt) {
          const int i = j + 1 + e / rem, c = j + 1 + e % rem;
          if (c <= i) D[i][c] -= D[i][j] * D[c][j] * ip;
        }
        __syncthreads();
      }
      // pivots of the eliminated block are its diagonal; check them all
      bool bad = false;
      for (int j = 0; j < nb; ++j) bad |= !(D[j][j] > 0.0);
      if (bad) {
        if (tid == 0) fail = 1;
        __syncthreads();
        break;
      }
      // scale: L_ij = D_ij / sqrt(D_jj)
      double vals[2];
      int idx[2];
      int cnt = 0;
      for (int e = tid; e < nb * nb && cnt < 2; e += nt, ++cnt) {
        const int i = e / nb, j = e % nb;
        idx[cnt] = e;
        vals[cnt] = (j <= i) ? D[i][j] / sqrt(D[j][j]) : 0.0;
      }
      __syncthreads();
      for (int c = 0; c < cnt; ++c) {
        const int i = idx[c] / nb, j = idx[c] % nb;
        D[i][j] = vals[c];
        L[(size_t)(k0 + i) * ldl + k0 + j] = vals[c];
      }
      __syncthreads();
      // (2) panel: rows r >= k0+nb solve x D^T = a
      const int r0 = k0 + nb;
      for (int r = r0 + tid; r < n; r += nt) {
        double* row = L + (size_t)r * ldl + k0;
        double x[CNB];
#pragma unroll
        for (int c = 0; c < CNB; ++c) {
          if (c < nb) {
            double s = row[c];
#pragma unroll
            for (int q = 0; q < c; ++q) s -= x[q] * D[c][q];
            x[c] = s / D[c][c];
          }
        }
#pragma unroll
        for (int c = 0; c < CNB; ++c)
          if (c < nb) row[c] = x[c];
      }
      __syncthreads();
      // (3) trailing update of the lower triangle: C -= P P^T
      const int tr = n - r0;
      if (tr > 0) {
        const int T = (tr + CT - 1) / CT;
        for (int ti = 0; ti < T; ++ti) {
          for (int tj = 0; tj <= ti; ++tj) {
            for (int e = tid; e < CT * CNB; e += nt) {
              const int rr = e / CNB, cc = e % CNB;
              const int gi = r0 + ti * CT + rr, gj = r0 + tj * CT + rr;
              Pi[rr][cc] = (gi < n && cc < nb) ? L[(size_t)gi * ldl + k0 + cc] : 0.0;
              Pj[rr][cc] = (gj < n && cc < nb) ? L[(size_t)gj * ldl + k0 + cc] : 0.0;
            }
            __syncthreads();
            // 1024 threads x 4 outputs = 64x64 tile
            const int tx = tid & 31, ty = tid >> 5;  // cols tx, tx+32 ; rows ty, ty+32
#pragma unroll
            for (int a = 0; a < 2; ++a) {
#pragma unroll
              for (int c2 = 0; c2 < 2; ++c2) {
                const int rr = ty + 32 * a, cc = tx + 32 * c2;
                const int gi = r0 + ti * CT + rr, gj = r0 + tj * CT + cc;
                if (gi < n && gj <= gi) {
                  double s = 0.0;
#pragma unroll 8
                  for (int q = 0; q < CNB; ++q) s += Pi[rr][q] * Pj[cc][q];
                  L[(size_t)gi * ldl + gj] -= s;
                }
              }
            }
            __syncthreads();
          }
        }
      }
    }
    __syncthreads();
    if (!fail) break;
  }
  if (tid == 0) {
    if (jitter_used) jitter_used[b] = jit;
    if (info) info[b] = fail ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------------------
// Triangular solve, in place on B (n x nrhs, row-major): X = L^-1 B or L^-T B.
// One workgroup per (64-column tile, batch); 64-row blocks; update GEMM through LDS.
// ---------------------------------------------------------------------------------------
constexpr int TT = 64;

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
      for (int e = tid; e < TT * TT; e += 256) {
        const int rr = e >> 6, cc = e & 63;
        // Lt[rr][cc] = op(L)[r0+rr][s0+cc]
        double lv = 0.0;
        if (!TRANS) {
          const int gr = r0 + rr, gc = s0 + cc;
          if (gr < n && gc < n) lv = L[(size_t)gr * ldl + gc];
        } else {
          const int gr = s0 + cc, gc = r0 + rr;  // (L^T)[r][s] = L[s][r]
          if (gr < n && gc < n) lv = L[(size_t)gr * ldl + gc];
        }
        Lt[rr][cc] = lv;
        const int xr = s0 + rr, xc = c0 + cc;
        Xt[rr][cc] = (xr < n && xc < nrhs) ? B[(size_t)xr * ldb + xc] : 0.0;
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
    for (int e = tid; e < TT * TT; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      const int gr = r0 + rr, gc = r0 + cc;
      Lt[rr][cc] = (gr < n && gc < n) ? L[(size_t)gr * ldl + gc] : 0.0;  // L itself (lower)
    }
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

__global__ void set_identity_kernel(int n, double* M, long long sM, int ldm) {
  double* P = M + blockIdx.y * sM;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < (long long)n * n) {
    const int i = (int)(e / n), j = (int)(e % n);
    P[(size_t)i * ldm + j] = (i == j) ? 1.0 : 0.0;
  }
}

}  // namespace evr

using namespace evr;

extern "C" {

int evr_gemm_f64(void* stream, int transA, int transB, int M, int N, int K, double alpha, const double* A,
                 int lda, long long strideA, const double* B, int ldb, long long strideB, double beta, double* C,
                 int ldc, long long strideC, int batch) {
  EVR_CHECK(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "evr_gemm_f64: bad sizes M=%d N=%d K=%d batch=%d", M, N,
            K, batch);
  if (M == 0 || N == 0) return 0;
  dim3 grid(cdiv(N, GT), cdiv(M, GT), batch);
  hipStream_t s = (hipStream_t)stream;
  if (!transA && !transB)
    gemm_f64_kernel<false, false><<<grid, 256, 0, s>>>(M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C,
                                                        ldc, strideC);
  else if (!transA && transB)
    gemm_f64_kernel<false, true><<<grid, 256, 0, s>>>(M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C,
                                                       ldc, strideC);
  else if (transA && !transB)
    gemm_f64_kernel<true, false><<<grid, 256, 0, s>>>(M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C,
                                                       ldc, strideC);
  else
    gemm_f64_kernel<true, true><<<grid, 256, 0, s>>>(M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C,
                                                      ldc, strideC);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_cholesky(void* stream, int batch, int n, const double* A, int lda, long long strideA, double* L, int ldl,
                 long long strideL, double jitter0, int max_tries, double* jitter_used, int* info) {
  EVR_CHECK(n >= 1 && batch >= 1 && max_tries >= 0, "evr_cholesky: bad sizes n=%d batch=%d", n, batch);
  EVR_CHECK(A != L, "evr_cholesky: A and L must not alias (the jitter ladder restarts from A)");
  chol_kernel<<<batch, 1024, 0, (hipStream_t)stream>>>(n, A, strideA, lda, L, strideL, ldl, jitter0, max_tries,
                                                       jitter_used, info);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_trsm_lower(void* stream, int batch, int n, int nrhs, const double* L, int ldl, long long strideL,
                   int transpose, double* B, int ldb, long long strideB) {
  EVR_CHECK(n >= 1 && nrhs >= 0 && batch >= 1, "evr_trsm_lower: bad sizes");
  if (nrhs == 0) return 0;
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
  dim3 g1(cdiv((long long)n * n, 256), batch);
  set_identity_kernel<<<g1, 256, 0, (hipStream_t)stream>>>(n, Linv, strideI, ldi);
  EVR_LAUNCH_CHECK();
  return evr_trsm_lower(stream, batch, n, n, L, ldl, strideL, 0, Linv, ldi, strideI);
}

}  // extern "C"
