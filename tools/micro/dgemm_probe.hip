// f64 MFMA GEMM probe (gfx950): the raw v_mfma_f64_16x16x4 issue rate, then tile variants
// of a register-staged, LDS double-buffered GEMM at the hot-path shapes (projection forward /
// backward, GP posterior), checked against a plain FMA kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/dgemm_probe.hip -o tools/_dgemm_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using double4_t = __attribute__((ext_vector_type(4))) double;
using double2_t = __attribute__((ext_vector_type(2))) double;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// ---- raw rate: NACC independent accumulators, ITERS rounds ----------------------------
template <int NACC>
__global__ __launch_bounds__(256) void mfma_rate(int iters, double* out, long long* cyc) {
  double4_t acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = {0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

// ---- reference ---------------------------------------------------------------------
// C[z][i][j] = sum_k A(i,k) B(k,j); A(i,k) = TA ? A[k*lda+i] : A[i*lda+k]; B row-major k x n
__global__ void ref_gemm(int M, int N, int K, bool TA, const double* A, int lda, long long sA, const double* B,
                         int ldb, long long sB, double* C, int ldc, long long sC) {
  const int j = blockIdx.x * 64 + threadIdx.x % 64, i = blockIdx.y * 4 + threadIdx.x / 64, z = blockIdx.z;
  if (i >= M || j >= N) return;
  const double* Az = A + z * sA;
  const double* Bz = B + z * sB;
  double acc = 0;
  for (int k = 0; k < K; ++k) acc = fma(TA ? Az[(size_t)k * lda + i] : Az[(size_t)i * lda + k], Bz[(size_t)k * ldb + j], acc);
  C[z * sC + (size_t)i * ldc + j] = acc;
}

// ---- tiled GEMM: BM x BN per 256-thread WG, 4 waves 2 x 2, BK k-step ------------------
// LDS: A k-contiguous (TA false): As[BM][BK + 2]; m-contiguous (TA): As[BK][BM + 16];
//      B n-contiguous: Bs[BK][BN + 16].  One barrier per k-step (double-buffered LDS),
//      the next step's global loads in registers across the MFMAs.
template <int BM, int BN, int BK, bool TA, int OCC, int WR = 2, int WC = 2, bool P128 = false>
__global__ __launch_bounds__(64 * WR * WC, OCC) void dg_kernel(int M, int N, int K, const double* __restrict__ A, int lda,
                                                      long long sA, const double* __restrict__ B, int ldb,
                                                      long long sB, double* __restrict__ C, int ldc, long long sC,
                                                      int swz) {
  constexpr int AST = TA ? (BM + 16) : (BK + 2);   // row stride of the A image
  constexpr int AROWS = TA ? BK : BM;
  constexpr int BST = BN + 16;
  constexpr int ASZ = AROWS * AST, BSZ = BK * BST;
  extern __shared__ double lds[];
  double* As0 = lds;
  double* Bs0 = lds + 2 * ASZ;
  // pairs per thread
  constexpr int NT = 64 * WR * WC;
  constexpr int AP = BM * BK / 2 / NT, BP = BK * BN / 2 / NT;
  static_assert(AP * 2 * NT == BM * BK && BP * 2 * NT == BK * BN, "tile/threads");
  const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
  const int flat = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int t = swz ? xcd_swizzle(flat, nwg) : flat;
  const int bx = t % gx, by = (t / gx) % gy, bz = t / (gx * gy);
  const int m0 = by * BM, n0 = bx * BN;
  A += bz * sA;
  B += bz * sB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int WM = BM / WR, WN = BN / WC, FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave tile");
  const int wm = (wave / WC) * WM, wn = (wave % WC) * WN;
  double4_t acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = {0, 0, 0, 0};
  // staging coordinates
  int ar[AP], ac[AP], br[BP], bc[BP];
#pragma unroll
  for (int u = 0; u < AP; ++u) {
    const int e = u * NT + tid;
    if (TA) { constexpr int PR = BM / 2; ar[u] = e / PR; ac[u] = (e % PR) * 2; }   // k row, m pair
    else { constexpr int PR = BK / 2; ar[u] = e / PR; ac[u] = (e % PR) * 2; }      // m row, k pair
  }
#pragma unroll
  for (int u = 0; u < BP; ++u) {
    const int e = u * NT + tid;
    constexpr int PR = BN / 2;
    br[u] = e / PR;
    bc[u] = (e % PR) * 2;
  }
  double2_t ra[AP], rb[BP];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < AP; ++u) {
      if (TA) {
        const int k = k0 + ar[u], m = m0 + ac[u];
        ra[u] = (k < K && m < M) ? *(const double2_t*)(A + (size_t)k * lda + m) : double2_t{0, 0};
      } else {
        const int m = m0 + ar[u], k = k0 + ac[u];
        ra[u] = (m < M && k < K) ? *(const double2_t*)(A + (size_t)m * lda + k) : double2_t{0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < BP; ++u) {
      const int k = k0 + br[u], n = n0 + bc[u];
      rb[u] = (k < K && n < N) ? *(const double2_t*)(B + (size_t)k * ldb + n) : double2_t{0, 0};
    }
  };
  auto stage = [&](int buf) {
    double* As = As0 + buf * ASZ;
    double* Bs = Bs0 + buf * BSZ;
#pragma unroll
    for (int u = 0; u < AP; ++u) *(double2_t*)(As + ar[u] * AST + ac[u]) = ra[u];
#pragma unroll
    for (int u = 0; u < BP; ++u) *(double2_t*)(Bs + br[u] * BST + bc[u]) = rb[u];
  };
  const int nk = (K + BK - 1) / BK;
  fetch(0);
  stage(0);
  __syncthreads();
  const int i = lane & 15, q = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) fetch((kt + 1) * BK);
    const double* As = As0 + (kt & 1) * ASZ;
    const double* Bs = Bs0 + (kt & 1) * BSZ;
    if (P128 && !TA) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 8) {
        double2_t af[FM];
        double bf0[FN], bf1[FN];
#pragma unroll
        for (int a = 0; a < FM; ++a) af[a] = *(const double2_t*)(As + (wm + a * 16 + i) * AST + kk + 2 * q);
#pragma unroll
        for (int b = 0; b < FN; ++b) {
          bf0[b] = Bs[(kk + 2 * q) * BST + wn + b * 16 + i];
          bf1[b] = Bs[(kk + 2 * q + 1) * BST + wn + b * 16 + i];
        }
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a][0], bf0[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a][1], bf1[b], acc[a][b], 0, 0, 0);
          }
      }
    } else
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double af[FM], bf[FN];
#pragma unroll
      for (int a = 0; a < FM; ++a)
        af[a] = TA ? As[(kk + q) * AST + wm + a * 16 + i] : As[(wm + a * 16 + i) * AST + kk + q];
#pragma unroll
      for (int b = 0; b < FN; ++b) bf[b] = Bs[(kk + q) * BST + wn + b * 16 + i];
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) stage((kt + 1) & 1);
    __syncthreads();
  }
  double* Cz = C + bz * sC;
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + a * 16 + q + 4 * r, col = n0 + wn + b * 16 + i;
        if (row < M && col < N) Cz[(size_t)row * ldc + col] = acc[a][b][r];
      }
}

struct Shape {
  const char* name;
  int batch, M, N, K;
  bool TA;
};

static double max_rel(const std::vector<double>& x, const std::vector<double>& y) {
  double m = 0, s = 0;
  for (size_t i = 0; i < x.size(); ++i) s = fmax(s, fabs(y[i]));
  for (size_t i = 0; i < x.size(); ++i) m = fmax(m, fabs(x[i] - y[i]));
  return m / (s > 0 ? s : 1);
}

template <int BM, int BN, int BK, int OCC, int WR = 2, int WC = 2, bool P128 = false>
static void run_variant(const Shape& sh, const double* A, const double* B, double* C, const std::vector<double>& ref,
                        int swz) {
  constexpr int NT = 64 * WR * WC;
  const int lda = sh.TA ? sh.M : sh.K;
  const long long sA = (long long)sh.M * sh.K, sB = (long long)sh.K * sh.N, sC = (long long)sh.M * sh.N;
  const int AROWS = sh.TA ? BK : BM, AST = sh.TA ? (BM + 16) : (BK + 2);
  const size_t lds = sizeof(double) * 2 * ((size_t)AROWS * AST + (size_t)BK * (BN + 16));
  dim3 grid((sh.N + BN - 1) / BN, (sh.M + BM - 1) / BM, sh.batch);
  auto launch = [&]() {
    if (sh.TA)
      hipLaunchKernelGGL((dg_kernel<BM, BN, BK, true, OCC, WR, WC, P128>), grid, dim3(NT), lds, 0, sh.M, sh.N, sh.K, A, lda, sA, B,
                         sh.N, sB, C, sh.N, sC, swz);
    else
      hipLaunchKernelGGL((dg_kernel<BM, BN, BK, false, OCC, WR, WC, P128>), grid, dim3(NT), lds, 0, sh.M, sh.N, sh.K, A, lda, sA,
                         B, sh.N, sB, C, sh.N, sC, swz);
  };
  if (lds > 160 * 1024) {
    printf("  %3dx%3dx%2d occ%d: lds %zu too big\n", BM, BN, BK, OCC, lds);
    return;
  }
  CK(hipFuncSetAttribute((const void*)dg_kernel<BM, BN, BK, true, OCC, WR, WC, P128>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)dg_kernel<BM, BN, BK, false, OCC, WR, WC, P128>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipMemset(C, 0, sizeof(double) * sC * sh.batch));
  launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<double> out(ref.size());
  CK(hipMemcpy(out.data(), C, sizeof(double) * out.size(), hipMemcpyDeviceToHost));
  const double err = max_rel(out, ref);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  const int reps = 20;
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double fl = 2.0 * sh.batch * sh.M * sh.N * (double)sh.K;
  printf("  %3dx%3dx%2d occ%d w%dx%d p%d swz%d: %8.2f us  %6.2f TF/s  wgs %5d  lds %6zu  err %.2e\n", BM, BN, BK,
         OCC, WR, WC, (int)P128, swz,
         ms * 1e3, fl / (ms * 1e-3) / 1e12, grid.x * grid.y * grid.z, lds, err);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  // raw MFMA rate
  {
    double* out;
    long long* cyc;
    CK(hipMalloc(&out, sizeof(double) * 256 * 4096));
    CK(hipMalloc(&cyc, sizeof(long long)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 2000;
    for (int nwg : {256, 512, 1024}) {
      hipLaunchKernelGGL((mfma_rate<8>), dim3(nwg), dim3(256), 0, 0, iters, out, cyc);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((mfma_rate<8>), dim3(nwg), dim3(256), 0, 0, iters, out, cyc);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      long long c;
      CK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
      const double fl = 2.0 * 16 * 16 * 4 * 8.0 * iters * nwg * 4;
      printf("mfma_f64_16x16x4 x8 acc: wgs %d  %.3f ms  %.2f TF/s  wave0 %.1f cyc/mfma\n", nwg, ms,
             fl / (ms * 1e-3) / 1e12, (double)c / (8.0 * iters));
    }
    CK(hipFree(out));
    CK(hipFree(cyc));
  }
  const Shape shapes[] = {
      {"proj_fwd 5x768x512x512", 5, 768, 512, 512, false},
      {"proj_fwd 5x769x512x512", 5, 769, 512, 512, false},
      {"proj_bwd 5x512x512x770 (TA)", 5, 512, 512, 770, true},
      {"posterior 5x513x1024x512", 5, 513, 1024, 512, false},
      {"fit W 5x512x512x512 (TA)", 5, 512, 512, 512, true},
  };
  for (const Shape& sh : shapes) {
    printf("%s\n", sh.name);
    const size_t na = (size_t)sh.batch * sh.M * sh.K, nb = (size_t)sh.batch * sh.K * sh.N,
                 nc = (size_t)sh.batch * sh.M * sh.N;
    std::vector<double> ha(na), hb(nb);
    srand(1);
    for (auto& v : ha) v = rand() / (double)RAND_MAX - 0.5;
    for (auto& v : hb) v = rand() / (double)RAND_MAX - 0.5;
    double *A, *B, *C, *R;
    CK(hipMalloc(&A, sizeof(double) * na));
    CK(hipMalloc(&B, sizeof(double) * nb));
    CK(hipMalloc(&C, sizeof(double) * nc));
    CK(hipMalloc(&R, sizeof(double) * nc));
    CK(hipMemcpy(A, ha.data(), sizeof(double) * na, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hb.data(), sizeof(double) * nb, hipMemcpyHostToDevice));
    const int lda = sh.TA ? sh.M : sh.K;
    hipLaunchKernelGGL(ref_gemm, dim3((sh.N + 63) / 64, (sh.M + 3) / 4, sh.batch), dim3(256), 0, 0, sh.M, sh.N, sh.K,
                       sh.TA, A, lda, (long long)sh.M * sh.K, B, sh.N, (long long)sh.K * sh.N, R, sh.N,
                       (long long)sh.M * sh.N);
    CK(hipDeviceSynchronize());
    std::vector<double> ref(nc);
    CK(hipMemcpy(ref.data(), R, sizeof(double) * nc, hipMemcpyDeviceToHost));
    run_variant<32, 64, 16, 4>(sh, A, B, C, ref, 1);
    run_variant<32, 64, 16, 4, 2, 2, true>(sh, A, B, C, ref, 1);
    run_variant<32, 32, 16, 8>(sh, A, B, C, ref, 1);
    run_variant<64, 64, 16, 2, 2, 4>(sh, A, B, C, ref, 1);    // 512 threads, wave 32x16
    run_variant<64, 64, 16, 2, 4, 2>(sh, A, B, C, ref, 1);    // 512 threads, wave 16x32
    run_variant<64, 64, 16, 2, 4, 2, true>(sh, A, B, C, ref, 1);
    run_variant<64, 64, 16, 4, 4, 1>(sh, A, B, C, ref, 1);    // 256 threads, wave 16x64
    run_variant<64, 32, 16, 4, 4, 1>(sh, A, B, C, ref, 1);    // 256 threads, wave 16x32
    run_variant<32, 64, 16, 4, 2, 2>(sh, A, B, C, ref, 0);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(R));
  }
  return 0;
}
