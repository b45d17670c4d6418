// Shared helpers for the everest_amd HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
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

// XCD-aware workgroup order (bijective for any nwg): consecutive blocks are dealt
// round-robin over the 8 XCDs, so give every XCD a contiguous chunk of the tile grid
// (neighbouring tiles share operand panels -> L2 hits).  Returns the tile index.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

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

// Compressed box cell (box_device.hip -> hvi.hip): one 64-bit key of the m defining-point
// indices of a local upper bound, field 0 (most significant) holding the rank of Z^0 in
// descending first coordinate.  bd_field_bits(m) bits per field.
__host__ __device__ constexpr int bd_field_bits(int m) { return m <= 4 ? 16 : (m == 5 ? 12 : 64 / m); }

template <int M>
struct CellKey {
  static constexpr int FB = bd_field_bits(M);
  static constexpr unsigned long long FMASK = (1ull << FB) - 1;
  __device__ static int field(unsigned long long k, int j) { return (int)((k >> (FB * (M - 1 - j))) & FMASK); }
  __device__ static unsigned long long set(unsigned long long k, int j, int v) {
    const int sh = FB * (M - 1 - j);
    return (k & ~(FMASK << sh)) | ((unsigned long long)v << sh);
  }
  // maximisation-space cell of the key: lo_j = -u_j, hi_j = -max_{k<j} Z^k_j (hi_0 = +inf).
  // pt: the sample's (points + dummies) x M table (minimisation space), rank0: rank -> index.
  __device__ static void decode(unsigned long long key, const double* pt, const int* rank0, double* lo,
                                double* hi) {
    int P[M];
    P[0] = rank0[field(key, 0)];
#pragma unroll
    for (int j = 1; j < M; ++j) P[j] = field(key, j);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double bl = -INFINITY;
#pragma unroll
      for (int k = 0; k < j; ++k) bl = fmax(bl, pt[P[k] * M + j]);
      lo[j] = -pt[P[j] * M + j];
      hi[j] = -bl;
    }
  }
};

}  // namespace evr
