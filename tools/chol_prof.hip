// Phase profile of the 64x64 diagonal-block factor (factor_diag64) with the EVR_CHOL_PROF
// cycle counters of linalg.hip: one workgroup per launch, many launches; prints average
// core-clock cycles per phase.  Build: hipcc --offload-arch=gfx950 -O3 -DEVR_CHOL_PROF
//   tools/chol_prof.hip everest_amd/csrc/gemm.hip -o tools/_chol_prof
#include <cstdio>
#include <cstring>
#include <vector>
#include "../everest_amd/csrc/linalg.hip"

namespace evr {
void set_error(const char*, ...) {}
}

int main() {
  const int n = 64, reps = 200;
  std::vector<double> A(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1 + i + j);
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
  const char* names[5] = {"factor total", "panel16 (4x)", "panel solve (3x)", "trailing (3x)", "inverse assembly"};
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
  return 0;
}
