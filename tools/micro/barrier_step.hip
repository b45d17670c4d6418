// Micro-benchmark: cost of a 64-step LDS-publish / barrier chain in one 256-thread
// workgroup (the shape of the Cholesky diagonal-block kernel).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void chain(double* out, int steps) {
  __shared__ double buf[2][64];
  const int tid = threadIdx.x;
  double acc = tid * 1e-3 + 1.0;
  if (tid < 64) buf[0][tid] = acc;
  __syncthreads();
  for (int j = 0; j < steps; ++j) {
    const double p = buf[j & 1][j & 63];
    double ip = p;
    if (MODE >= 1) ip = 1.0 / p;
    if (MODE >= 2) ip = ip + sqrt(p);
    acc = fma(acc, 0.999, ip * 1e-9);
    if (tid < 64) buf[(j + 1) & 1][tid] = acc;
    __syncthreads();
  }
  out[blockIdx.x * 256 + tid] = acc;
}

__global__ void empty_k(double* out) { if (threadIdx.x == 0 && out == nullptr) out[0] = 1; }

int main() {
  double* d;
  hipMalloc(&d, 256 * 256 * sizeof(double));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto time = [&](auto fn, const char* name) {
    for (int w = 0; w < 3; ++w) fn();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 50; ++r) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.2f us\n", name, ms * 1000 / 50);
  };
  time([&] { empty_k<<<1, 256>>>(d); }, "empty");
  time([&] { chain<0><<<1, 256>>>(d, 64); }, "barrier x64");
  time([&] { chain<0><<<1, 256>>>(d, 640); }, "barrier x640");
  time([&] { chain<1><<<1, 256>>>(d, 640); }, "barrier+div x640");
  time([&] { chain<2><<<1, 256>>>(d, 640); }, "barrier+div+sqrt x640");
  time([&] { chain<1><<<256, 256>>>(d, 640); }, "256 WGs barrier+div x640");
  return 0;
}
