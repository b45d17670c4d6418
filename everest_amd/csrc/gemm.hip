// Batched f64 GEMM on the gfx950 matrix cores through the gemm_core.hpp tile engine:
//   C = alpha * op(A) * B + beta * C   (row-major, op(A) = A or A^T, batched by strides)
// The entry point of the posterior / operator GEMMs of the GP and qNEHVI paths and of
// evr_gemm_f64 for the shapes the engine serves (B not transposed, no triangular output).
// Split-K (fixed-order reduction, bitwise reproducible) when the tile grid cannot fill the
// chip.  Tile shape measured on MI355X (tools/micro/dgemm_probe.hip, profiles/r05/a, /b).
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "gemm_core.hpp"

namespace evr {

template <class C, bool VEC>
__global__ __launch_bounds__(256, 4) void dg_gemm_kernel(int M, int N, int K, double alpha,
                                                         const double* __restrict__ A, int lda, long long sA,
                                                         const double* __restrict__ B, int ldb, long long sB,
                                                         double beta, double* __restrict__ Cm, int ldc, long long sC,
                                                         int ksplit, int kchunk, double* __restrict__ W) {
  extern __shared__ double lds[];
  const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
  const int t = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), nwg);
  const int bx = t % gx, by = (t / gx) % gy, bzk = t / (gx * gy);
  const int bz = bzk / ksplit, kz = bzk - bz * ksplit;
  const int m0 = by * C::BM, n0 = bx * C::BN;
  const double* Az = A + bz * sA;
  const double* Bz = B + bz * sB;
  const int kbeg = kz * kchunk, kend = min(K, kbeg + kchunk);
  dg_double4 acc[C::FM][C::FN];
  dg_mainloop<C>(
      lds, kbeg, kend,
      [&](int x, int y) -> dg_double2 {
        if (C::TA) {   // x = k, y = tile column pair of A^T (= rows of C)
          const int k = x, mm = m0 + y;
          const bool ok = k < kend;
          return dg_pair<VEC>(Az + (size_t)k * lda + mm, ok && mm < M, ok && mm + 1 < M);
        }
        const int mm = m0 + x, k = y;
        const bool ok = mm < M;
        return dg_pair<VEC>(Az + (size_t)mm * lda + k, ok && k < kend, ok && k + 1 < kend);
      },
      [&](int k, int c) -> dg_double2 {
        const int nn = n0 + c;
        const bool ok = k < kend;
        return dg_pair<VEC>(Bz + (size_t)k * ldb + nn, ok && nn < N, ok && nn + 1 < N);
      },
      acc);
  if (ksplit > 1) {
    double* Wz = W + ((size_t)kz * (gridDim.z / ksplit) + bz) * (size_t)M * N;
    dg_for_each<C>(acc, [&](int r, int c, double val) {
      if (m0 + r < M && n0 + c < N) Wz[(size_t)(m0 + r) * N + n0 + c] = val;
    });
    return;
  }
  double* Cz = Cm + bz * sC;
  dg_for_each<C>(acc, [&](int r, int c, double val) {
    if (m0 + r < M && n0 + c < N) {
      double* p = Cz + (size_t)(m0 + r) * ldc + n0 + c;
      *p = beta == 0.0 ? alpha * val : alpha * val + beta * *p;
    }
  });
}

__global__ __launch_bounds__(256) void dg_splitk_reduce(int M, int N, int batch, int ksplit, double alpha,
                                                        const double* __restrict__ W, double beta,
                                                        double* __restrict__ Cm, int ldc, long long sC) {
  const long long mn = (long long)M * N;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= mn) return;
  const int bz = blockIdx.y;
  double acc = 0.0;
  // 8 unconditional loads (clamped slice indices) in flight per round, summed in slice order
  for (int k0 = 0; k0 < ksplit; k0 += 8) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = W[((size_t)min(k0 + u, ksplit - 1) * batch + bz) * mn + e];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u < ksplit) acc += t[u];
  }
  const int row = (int)(e / N), cc = (int)(e - (long long)row * N);
  double* p = Cm + bz * sC + (size_t)row * ldc + cc;
  *p = beta == 0.0 ? alpha * acc : alpha * acc + beta * *p;
}

// Tiles (tools/micro/dgemm_probe.hip, profiles/r05/a, /b): at the hot-path shapes the chip
// needs ~4 waves per SIMD to keep the f64 matrix pipe busy (the bare v_mfma_f64_16x16x4 loop
// reaches 33 / 45 / 47.5 TF/s at 1 / 2 / 4 waves per SIMD), so the tiles are small enough to
// give ~1000 workgroups: 32 x 64 for A k-contiguous (5 x 769 x 512 x 512: 51.1 us, 64 x 64
// tiles 64.6 us), 32 x 32 for A m-contiguous (5 x 512 x 512 x 770: 50.1 us vs 61.3 us).
using DgN = DgCfg<32, 64, 16, false>;
using DgT = DgCfg<32, 32, 16, true>;

template <class C>
static int dg_launch(hipStream_t s, int M, int N, int K, double alpha, const double* A, int lda, long long sA,
                     const double* B, int ldb, long long sB, double beta, double* Cm, int ldc, long long sC,
                     int batch, int ksplit, int kchunk, double* W, int vec) {
  const size_t lds = sizeof(double) * C::LDS_DOUBLES;
  dim3 grid(cdiv(N, C::BN), cdiv(M, C::BM), batch * ksplit);
  if (vec)
    dg_gemm_kernel<C, true><<<grid, 256, lds, s>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, Cm, ldc, sC, ksplit,
                                                   kchunk, W);
  else
    dg_gemm_kernel<C, false><<<grid, 256, lds, s>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, Cm, ldc, sC, ksplit,
                                                    kchunk, W);
  EVR_LAUNCH_CHECK();
  return 0;
}

// split K when the tile grid cannot fill the chip (aim at ~4 workgroups per CU); each slice
// keeps >= 8 k-steps
int dg_ksplit(long long tiles, int K, int bk, int* kchunk) {
  int ks = 1;
  if (tiles < 768)
    ks = (int)std::max<long long>(1, std::min<long long>(std::min<long long>(cdiv(1024, tiles), K / (8 * bk)), 32));
  *kchunk = ks > 1 ? cdiv(cdiv(K, ks), bk) * bk : std::max(K, 1);
  return ks > 1 ? cdiv(K, *kchunk) : 1;
}

static long long dg_tiles(bool tA, int M, int N, int batch) {
  return tA ? (long long)cdiv(N, DgT::BN) * cdiv(M, DgT::BM) * batch
            : (long long)cdiv(N, DgN::BN) * cdiv(M, DgN::BM) * batch;
}

size_t dg_gemm_ws_doubles(bool tA, int M, int N, int K, int batch) {
  int kchunk = 0;
  const int ks = dg_ksplit(dg_tiles(tA, M, N, batch), K, DgN::BK, &kchunk);
  return ks > 1 ? (size_t)ks * batch * M * N : 0;
}

// C = alpha op(A) B + beta C through the tile engine.  W: split-K workspace of
// dg_gemm_ws_doubles doubles (nullptr: no split).  16-byte operand fetches when every row
// start is 16-byte aligned.
int dg_gemm(hipStream_t s, bool tA, int M, int N, int K, double alpha, const double* A, int lda, long long sA,
            const double* B, int ldb, long long sB, double beta, double* Cm, int ldc, long long sC, int batch,
            double* W) {
  if (M == 0 || N == 0) return 0;
  auto al = [](const void* p, long long ld, long long st) {
    return ((uintptr_t)p % 16 == 0) && ld % 2 == 0 && st % 2 == 0;
  };
  // pairs run along k for a k-contiguous A (K even: no pair straddles the end), along M / N
  // otherwise (M, N even)
  const int vec = (al(A, lda, sA) && al(B, ldb, sB) && N % 2 == 0 && (tA ? M % 2 == 0 : K % 2 == 0)) ? 1 : 0;
  int kchunk = std::max(K, 1), ks = 1;
  if (W) ks = dg_ksplit(dg_tiles(tA, M, N, batch), K, DgN::BK, &kchunk);
  const int rc = tA ? dg_launch<DgT>(s, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, Cm, ldc, sC, batch, ks, kchunk,
                                     W, vec)
                    : dg_launch<DgN>(s, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, Cm, ldc, sC, batch, ks, kchunk,
                                     W, vec);
  if (rc) return rc;
  if (ks > 1) {
    dg_splitk_reduce<<<dim3(cdiv((long long)M * N, 256), batch), 256, 0, s>>>(M, N, batch, ks, alpha, W, beta, Cm, ldc,
                                                                             sC);
    EVR_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace evr
