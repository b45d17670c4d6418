// Shared helpers for the everest_amd HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

namespace evr {

// Thread-local last-error message, surfaced through evr_last_error().
void set_error(const char* fmt, ...);
const char* last_error();

#define EVR_HIP(call)                                                             \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::evr::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,               \
                       hipGetErrorString(e_));                                    \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

#define EVR_CHECK(cond, ...)                                                      \
  do {                                                                            \
    if (!(cond)) {                                                                \
      ::evr::set_error(__VA_ARGS__);                                              \
      return 2;                                                                   \
    }                                                                             \
  } while (0)

#define EVR_LAUNCH_CHECK()                                                        \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      ::evr::set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__,           \
                       hipGetErrorString(e_));                                    \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Kernel families (same numbering as include/everest_amd.h EVR_KERNEL_*).
enum KernelKind { RBF = 0, MATERN05 = 1, MATERN15 = 2, MATERN25 = 3 };

// k(r^2) for the stationary kernels GPyTorch exposes through BoFire
// (bofire/kernels/mapper.py:31-69).  Matérn uses dist = sqrt(max(d2, 1e-30)).
__device__ __forceinline__ double kernel_value(int kind, double d2) {
  if (kind == RBF) return exp(-0.5 * d2);
  const double d = sqrt(fmax(d2, 1e-30));
  if (kind == MATERN05) return exp(-d);
  if (kind == MATERN15) {
    const double s = 1.7320508075688772 * d;
    return (1.0 + s) * exp(-s);
  }
  const double s = 2.23606797749979 * d;
  return (1.0 + s + (5.0 / 3.0) * d2) * exp(-s);
}

// dk/d(x_d) = kernel_dscale(kind, d2) * (x_d - x'_d) / ls_d^2   (x in lengthscale units
// already divided out: caller multiplies by (x_d - x'_d)/ls_d^2 of normalized coords).
__device__ __forceinline__ double kernel_dscale(int kind, double d2) {
  if (kind == RBF) return -exp(-0.5 * d2);
  if (d2 < 1e-30) return 0.0;  // clamp_min(1e-30) kills the gradient there
  const double d = sqrt(d2);
  if (kind == MATERN05) return -exp(-d) / d;
  if (kind == MATERN15) return -3.0 * exp(-1.7320508075688772 * d);
  const double s = 2.23606797749979 * d;
  return -(5.0 / 3.0) * (1.0 + s) * exp(-s);
}

}  // namespace evr
