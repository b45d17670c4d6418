// Phase cycle counts of the Cholesky diagonal-block kernel (built with EVR_CHOL_PROF).
#include "../../everest_amd/csrc/linalg.hip"
#include <cstdio>
#include <vector>
#include <cmath>
int main() {
  const int n = 64, reps = 50;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = (i == j ? n : 0.0) + 1.0 / (1 + std::abs(i - j));
  double *A, *D;
  int* info;
  (void)hipMalloc(&A, n * n * 8);
  (void)hipMalloc(&D, n * n * 8);
  (void)hipMalloc(&info, 4);
  (void)hipMemset(info, 0, 4);
  unsigned long long z[16] = {0};
  for (int r = 0; r < reps + 1; ++r) {
    if (r == 1) (void)hipMemcpyToSymbol(HIP_SYMBOL(evr::chol_prof), z, sizeof(z));
    (void)hipMemcpy(A, h.data(), n * n * 8, hipMemcpyHostToDevice);
    evr::chol_diag_kernel<<<1, 256>>>(n, 0, A, 0, n, D, 0, info);
  }
  (void)hipDeviceSynchronize();
  unsigned long long t[16];
  (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(evr::chol_prof), sizeof(t));
  const char* names[5] = {"factor loop total", "panel factor16 (x4)", "panel solve (x3)", "trailing (x3)", "inverse assembly"};
  for (int k = 0; k < 5; ++k) printf("%-22s %10.0f cycles/call\n", names[k], (double)t[k] / reps);
  return 0;
}
