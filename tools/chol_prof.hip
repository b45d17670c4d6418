// Phase profile of the 64x64 diagonal-block factor (factor_diag64) with the EVR_CHOL_PROF
// cycle counters of linalg.hip: one workgroup per launch, many launches; prints average
// core-clock cycles per phase.  Build: hipcc --offload-arch=gfx950 -O3 -DEVR_CHOL_PROF
//   tools/chol_prof.hip everest_amd/csrc/gemm.hip -o tools/_chol_prof
#include <cstdio>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>
#include "../everest_amd/csrc/linalg.hip"

namespace evr {
void set_error(const char*, ...) {}
}

int main(int argc, char** argv) {
  const int n = 64, reps = 200;
  std::vector<double> A(n * n);
  const bool rbf = argc > 1 && std::string(argv[1]) == "rbf";
  if (rbf) {
    // a GP-shaped block: RBF kernel of 64 random points in [0, 1]^6 (lengthscale 0.7) + 1e-4 I
    std::vector<double> P(n * 6);
    unsigned x = 12345u;
    for (auto& v : P) {
      x = x * 1664525u + 1013904223u;
      v = (x >> 8) / double(1u << 24);
    }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double d2 = 0.0;
        for (int k = 0; k < 6; ++k) d2 += (P[i * 6 + k] - P[j * 6 + k]) * (P[i * 6 + k] - P[j * 6 + k]) / 0.49;
        A[i * n + j] = std::exp(-0.5 * d2) + (i == j ? 1e-4 : 0.0);
      }
  } else {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) A[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1 + i + j);
  }
  double *dA, *dD;
  int* info;
  hipMalloc(&dA, sizeof(double) * n * n);
  hipMalloc(&dD, sizeof(double) * n * n);
  hipMalloc(&info, sizeof(int));
  hipMemset(info, 0, sizeof(int));
  unsigned long long z[16] = {0};
  for (int r = 0; r < reps + 10; ++r) {
    if (r == 10) hipMemcpyToSymbol(HIP_SYMBOL(evr::chol_prof), z, sizeof(z));
    hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
    evr::chol_diag_kernel<<<1, 256>>>(n, 0, dA, 0, n, dD, 0, info);
  }
  hipDeviceSynchronize();
  unsigned long long p[16];
  hipMemcpyFromSymbol(p, HIP_SYMBOL(evr::chol_prof), sizeof(p));
  const char* names[5] = {"factor total", "leaves", "panel solves", "trailing updates", "inverse assembly"};
  for (int k = 0; k < 5; ++k) printf("{\"phase\": \"%s\", \"cycles\": %.0f}\n", names[k], (double)p[k] / reps);
  int h;
  hipMemcpy(&h, info, sizeof(int), hipMemcpyDeviceToHost);
  printf("{\"info\": %d}\n", h);
  // bit-pattern digest of the factor and its inverse (compare leaf variants for equality)
  std::vector<double> L(n * n), D(n * n);
  hipMemcpy(L.data(), dA, sizeof(double) * n * n, hipMemcpyDeviceToHost);
  hipMemcpy(D.data(), dD, sizeof(double) * n * n, hipMemcpyDeviceToHost);
  unsigned long long dg = 1469598103934665603ull;
  for (int i = 0; i < n * n; ++i) {
    unsigned long long u, v;
    memcpy(&u, &L[i], 8);
    memcpy(&v, &D[i], 8);
    dg = (dg ^ u) * 1099511628211ull;
    dg = (dg ^ v) * 1099511628211ull;
  }
  printf("{\"digest\": \"%016llx\"}\n", dg);
  // accuracy against a long-double Cholesky and triangular inverse of the same block
  std::vector<long double> Lr(n * n, 0.0L), Xr(n * n, 0.0L);
  for (int j = 0; j < n; ++j) {
    long double dsum = A[j * n + j];
    for (int k = 0; k < j; ++k) dsum -= Lr[j * n + k] * Lr[j * n + k];
    Lr[j * n + j] = std::sqrt(dsum);
    for (int i = j + 1; i < n; ++i) {
      long double v = A[i * n + j];
      for (int k = 0; k < j; ++k) v -= Lr[i * n + k] * Lr[j * n + k];
      Lr[i * n + j] = v / Lr[j * n + j];
    }
  }
  for (int j = 0; j < n; ++j) {
    Xr[j * n + j] = 1.0L / Lr[j * n + j];
    for (int i = j + 1; i < n; ++i) {
      long double v = 0.0L;
      for (int k = j; k < i; ++k) v += Lr[i * n + k] * Xr[k * n + j];
      Xr[i * n + j] = -v / Lr[i * n + i];
    }
  }
  long double el = 0, ex = 0, ml = 0, mx = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      el = std::fmax(el, std::fabs((long double)L[i * n + j] - Lr[i * n + j]));
      ex = std::fmax(ex, std::fabs((long double)D[i * n + j] - Xr[i * n + j]));
      ml = std::fmax(ml, std::fabs(Lr[i * n + j]));
      mx = std::fmax(mx, std::fabs(Xr[i * n + j]));
    }
  printf("{\"L_err_rel_max\": %.3e, \"Linv_err_rel_max\": %.3e, \"Linv_max\": %.3e}\n", (double)(el / ml),
         (double)(ex / mx), (double)mx);
  return 0;
}
