// Write-bandwidth ceiling of the config-5 kernel-matrix output (2048 x 2048 f64 = 33.5 MB):
// plain fills with 8, 16 and 32 bytes per lane per store instruction, cached and
// non-temporal, one-shot (a thread per 8 / 16 / 32 bytes) and grid-stride (2048 workgroups),
// timed with HIP events over 50 launches each.  Prints one JSON object (GB/s per variant).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/fill_probe.hip -o tools/_fill_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

using d2_t = __attribute__((ext_vector_type(2))) double;
using d4_t = __attribute__((ext_vector_type(4))) double;

template <int W, bool NT>   // W doubles per lane per store
__global__ __launch_bounds__(256) void fill_oneshot(double* __restrict__ p, long long n, double v) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * W;
  if (i + W > n) return;
  if (W == 1) {
    if (NT) __builtin_nontemporal_store(v, p + i);
    else p[i] = v;
  } else if (W == 2) {
    const d2_t x = {v, v};
    if (NT) __builtin_nontemporal_store(x, (d2_t*)(p + i));
    else *(d2_t*)(p + i) = x;
  } else {
    const d4_t x = {v, v, v, v};
    if (NT) __builtin_nontemporal_store(x, (d4_t*)(p + i));
    else *(d4_t*)(p + i) = x;
  }
}

template <int W, bool NT>
__global__ __launch_bounds__(256) void fill_stride(double* __restrict__ p, long long n, double v) {
  const long long step = (long long)gridDim.x * 256 * W;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * W; i + W <= n; i += step) {
    if (W == 2) {
      const d2_t x = {v, v};
      if (NT) __builtin_nontemporal_store(x, (d2_t*)(p + i));
      else *(d2_t*)(p + i) = x;
    } else {
      const d4_t x = {v, v, v, v};
      if (NT) __builtin_nontemporal_store(x, (d4_t*)(p + i));
      else *(d4_t*)(p + i) = x;
    }
  }
}

template <typename F>
static float timed(F f) {
  for (int r = 0; r < 5; ++r) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < 50; ++r) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / 50;
}

int main() {
  const long long n = 2048LL * 2048;
  const double bytes = 8.0 * n;
  double* p;
  CK(hipMalloc(&p, n * 8));
  printf("{\"bytes\": %.0f", bytes);
#define ONE(W, NT, name)                                                                          \
  {                                                                                               \
    const unsigned g = (unsigned)((n / W + 255) / 256);                                           \
    const float ms = timed([&] { fill_oneshot<W, NT><<<g, 256>>>(p, n, 1.0); });                   \
    printf(", \"%s_us\": %.2f, \"%s_GBs\": %.0f", name, ms * 1e3, name, bytes / (ms * 1e-3) / 1e9); \
  }
#define STR(W, NT, name)                                                                          \
  {                                                                                               \
    const float ms = timed([&] { fill_stride<W, NT><<<2048, 256>>>(p, n, 1.0); });                 \
    printf(", \"%s_us\": %.2f, \"%s_GBs\": %.0f", name, ms * 1e3, name, bytes / (ms * 1e-3) / 1e9); \
  }
  ONE(1, false, "b8");
  ONE(1, true, "b8_nt");
  ONE(2, false, "b16");
  ONE(2, true, "b16_nt");
  ONE(4, false, "b32");
  ONE(4, true, "b32_nt");
  STR(2, false, "b16_stride");
  STR(2, true, "b16_stride_nt");
  STR(4, false, "b32_stride");
  STR(4, true, "b32_stride_nt");
  CK(hipDeviceSynchronize());
  printf("}\n");
  return 0;
}
