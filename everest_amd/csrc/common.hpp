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

// exp(x) for the kernel arguments (x <= 0; valid up to x ~ 709): x = (64 k + j) ln2/64 + r
// with |r| <= ln2/128 (FMA Cody-Waite reduction), exp = 2^k * T[j] * (1 + p(r)), p a
// degree-6 Taylor polynomial (truncation < 1e-19 relative), T[j] = 2^(j/64) correctly
// rounded.  ~12 VALU ops against ~45 for the libm-style f64 exp (whose polynomial
// constants are rematerialised per call); error <= ~1 ulp.  The Matern epilogues of the
// kernel-matrix kernels are VALU-bound on exactly this.  NaN propagates; x < -760
// returns +0 like exp.
__device__ __constant__ static const double kExp2J64[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951,
};

// exp_k with the 2^(j/64) table read from T (an LDS copy, kexp_stage): a per-lane indexed
// __constant__ read is a vector memory load, and on gfx9 vmcnt retires loads and stores in
// issue order, so in a store-heavy epilogue every table load also waited for the stores
// issued before it.  Same arithmetic as exp_k: bitwise equal.
__device__ __forceinline__ double exp_k_t(double x, const double* __restrict__ T) {
  x = x < -760.0 ? -760.0 : x;
  const double kd = __builtin_rint(x * 92.33248261689366);
  const int k = (int)kd;
  double r = fma(kd, -0.010830424696249145, x);
  r = fma(kd, -3.623510646634843e-19, r);
  double q = fma(r, 1.0 / 720.0, 1.0 / 120.0);
  q = fma(q, r, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  const double p = fma(q, r * r, r);
  const double t = T[k & 63];
  return __builtin_ldexp(fma(t, p, t), k >> 6);
}
// copy of kExp2J64 into a workgroup's LDS (callers __syncthreads before use)
__device__ __forceinline__ void kexp_stage(double* T, int tid, int nthreads) {
  for (int i = tid; i < 64; i += nthreads) T[i] = kExp2J64[i];
}

__device__ __forceinline__ double exp_k(double x) {
  x = x < -760.0 ? -760.0 : x;
  const double kd = __builtin_rint(x * 92.33248261689366);
  const int k = (int)kd;
  double r = fma(kd, -0.010830424696249145, x);
  r = fma(kd, -3.623510646634843e-19, r);
  double q = fma(r, 1.0 / 720.0, 1.0 / 120.0);
  q = fma(q, r, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  const double p = fma(q, r * r, r);
  const double t = kExp2J64[k & 63];
  return __builtin_ldexp(fma(t, p, t), k >> 6);
}

// qNEHVI operator layout: H^T rows in M (S, or 0 for qEHVI) and total rows Rr.
template <class State>
inline int qn_nh(const State* st) { return st->no_h ? 0 : st->S; }
template <class State>
inline int qn_rows(const State* st) { return st->n + st->nb + qn_nh(st) + 1; }

// Kernel families (same numbering as include/everest_amd.h EVR_KERNEL_*).
enum KernelKind { RBF = 0, MATERN05 = 1, MATERN15 = 2, MATERN25 = 3 };
// A kind code is one family for every output (0..3) or KIND_MIXED with a 2-bit family per
// output j at bits 5 + 2 j (EVR_KERNEL_MIXED; at most KIND_MAX_MIXED outputs).
constexpr int KIND_MIXED = 16, KIND_MAX_MIXED = 13;
__host__ __device__ __forceinline__ int kind_of(int code, int j) {
  return code < KIND_MIXED ? code : (code >> (5 + 2 * j)) & 3;
}
inline bool kind_code_ok(int code, int B) {
  if (code >= 0 && code <= 3) return true;
  if (!(code & KIND_MIXED) || (code & 15) || B < 1 || B > KIND_MAX_MIXED) return false;
  return (code >> (5 + 2 * B)) == 0;
}

// k(r^2) for the stationary kernels GPyTorch exposes through BoFire
// (bofire/kernels/mapper.py:31-69).  Matérn uses dist = sqrt(max(d2, 1e-30)).
__device__ __forceinline__ double kernel_value(int kind, double d2) {
  if (kind == RBF) return exp_k(-0.5 * d2);
  const double d = sqrt(fmax(d2, 1e-30));
  if (kind == MATERN05) return exp_k(-d);
  if (kind == MATERN15) {
    const double s = 1.7320508075688772 * d;
    return (1.0 + s) * exp_k(-s);
  }
  const double s = 2.23606797749979 * d;
  return (1.0 + s + (5.0 / 3.0) * d2) * exp_k(-s);
}
// sqrt of a normal x > 0 (the Matérn distance after the 1e-30 clamp): v_rsq_f64, one
// Goldschmidt step and one Newton correction — 8 VALU ops against the ~20 of the libm-style
// f64 sqrt (denormal scaling, two corrections, class tests); within ~1 ulp of sqrt.
__device__ __forceinline__ double sqrt_pos(double x) {
#pragma clang fp contract(off)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  return fma(fma(-g, g, x), h, g);
}
// kernel_value_t with sqrt_pos (the MFMA kernel-matrix epilogues).  Every product and sum is
// spelled out (contraction off, explicit fma): the cross and the symmetric kernels inline it
// into different code, and the backend's free fusion of (1 + s) + (5/3) d2 differed between
// them by an ulp — K(X, X) must be bitwise the same through either.
__device__ __forceinline__ double kernel_value_r(int kind, double d2, const double* __restrict__ T) {
#pragma clang fp contract(off)
  if (kind == RBF) return exp_k_t(-0.5 * d2, T);
  const double d = sqrt_pos(fmax(d2, 1e-30));
  if (kind == MATERN05) return exp_k_t(-d, T);
  if (kind == MATERN15) {
    const double s = 1.7320508075688772 * d;
    return (1.0 + s) * exp_k_t(-s, T);
  }
  const double s = 2.23606797749979 * d;
  return fma(5.0 / 3.0, d2, 1.0 + s) * exp_k_t(-s, T);
}
// kernel_value with the exp table in LDS (bitwise equal)
__device__ __forceinline__ double kernel_value_t(int kind, double d2, const double* __restrict__ T) {
  if (kind == RBF) return exp_k_t(-0.5 * d2, T);
  const double d = sqrt(fmax(d2, 1e-30));
  if (kind == MATERN05) return exp_k_t(-d, T);
  if (kind == MATERN15) {
    const double s = 1.7320508075688772 * d;
    return (1.0 + s) * exp_k_t(-s, T);
  }
  const double s = 2.23606797749979 * d;
  return (1.0 + s + (5.0 / 3.0) * d2) * exp_k_t(-s, T);
}
__device__ __forceinline__ double kernel_dscale_t(int kind, double d2, const double* __restrict__ T) {
  if (kind == RBF) return -exp_k_t(-0.5 * d2, T);
  if (d2 < 1e-30) return 0.0;
  const double d = sqrt(d2);
  if (kind == MATERN05) return -exp_k_t(-d, T) / d;
  if (kind == MATERN15) return -3.0 * exp_k_t(-1.7320508075688772 * d, T);
  const double s = 2.23606797749979 * d;
  return -(5.0 / 3.0) * (1.0 + s) * exp_k_t(-s, T);
}

// dk/d(x_d) = kernel_dscale(kind, d2) * (x_d - x'_d) / ls_d^2   (x in lengthscale units
// already divided out: caller multiplies by (x_d - x'_d)/ls_d^2 of normalized coords).
__device__ __forceinline__ double kernel_dscale(int kind, double d2) {
  if (kind == RBF) return -exp_k(-0.5 * d2);
  if (d2 < 1e-30) return 0.0;  // clamp_min(1e-30) kills the gradient there
  const double d = sqrt(d2);
  if (kind == MATERN05) return -exp_k(-d) / d;
  if (kind == MATERN15) return -3.0 * exp_k(-1.7320508075688772 * d);
  const double s = 2.23606797749979 * d;
  return -(5.0 / 3.0) * (1.0 + s) * exp_k(-s);
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
  // as decode, for keys whose field 0 holds the point index itself (the kd-ordered group
  // keys written by cells_kd.hip) rather than the rank in descending first coordinate
  __device__ static void decode_direct(unsigned long long key, const double* pt, double* lo, double* hi) {
    int P[M];
#pragma unroll
    for (int j = 0; j < M; ++j) P[j] = field(key, j);
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

// ---- log-space hypervolume helpers (hvi_log.hip, qnehvi_general.hip) -------------------
constexpr double HL_UMAX = 1e10;   // clamp_max of the cell upper bounds (float64)

// log fatplus(z; tr) and d/dz
__device__ __forceinline__ double log_fatplus(double z, double tr, double* dpsi) {
  const double x = z / tr;
  double sp, dsp;
  if (x > 20.0) {   // torch softplus threshold
    sp = x;
    dsp = 1.0;
  } else if (x < -60.0) {
    // exp(x) < 1e-26 lies below half an ulp of 0.1 c = 0.1 / (1 + x^2) and of the 0.2 x c^2
    // term of the derivative for every x < -60 (checked exhaustively on a dense grid to
    // -1e8; below -745 exp underflows to 0 anyway), so F and dpsi round to the same doubles
    // with sp = dsp = 0: bitwise the full formula, minus an exp and a log1p.  With
    // tau_relu = 1e-6 this is every cell lying more than 6e-5 above y_j in objective j.
    sp = 0.0;
    dsp = 0.0;
  } else {
    const double e = exp(x);
    sp = log1p(e);
    dsp = e / (1.0 + e);
  }
  const double c = 1.0 / (1.0 + x * x);
  const double F = sp + 0.1 * c;
  if (dpsi) *dpsi = (dsp - 0.2 * x * c * c) / (tr * F);
  return log(tr * F);
}

// fatmin(a, b; t) and d/da
__device__ __forceinline__ double fatmin2(double a, double b, double t, double* da) {
  if (b == -INFINITY) {   // zero-width side: -inf log area, no gradient
    if (da) *da = 0.0;
    return -INFINITY;
  }
  const double x = fabs(a - b) / t;
  const double p = 2.0 / (2.0 + x * (2.0 + x));
  const double dq = p * p * (1.0 + x) / (1.0 + p);   // -pareto'(x) / (1 + pareto(x))
  if (da) *da = (a < b) ? 1.0 - dq : dq;
  return fmin(a, b) - t * log(1.0 + p);
}

// ---- table-driven f64 log1p / log / exp for the keyed log scan (hvi_logk_kernel): the
// OCML routines cost ~100 instructions each and there are ~7 per (cell, candidate).  The
// tables live in the caller's LDS (FastLogTabs::fill once per workgroup); results stay
// within ~2 ulps of the libm values.
struct FastLogTabs {
  double2 li[65];  // (log1p(i / 64), 1 / (1 + i / 64)): one 16-byte LDS read per log1p
  double et[64];   // 2^(j / 64)
  __device__ void fill(int tid, int nthreads) {
    for (int i = tid; i < 65; i += nthreads) {
      li[i] = make_double2(log1p(i / 64.0), 1.0 / (1.0 + i / 64.0));
      if (i < 64) et[i] = exp2(i / 64.0);
    }
  }
};

// 1 / d for d in [1, 2^1000]: hardware reciprocal seed + two Newton steps (<= 1 ulp, no
// scaling / fixup sequence: d is never denormal, infinite or zero here)
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// log1p(p) for p in [0, 1]: log1p(i / 64) + log1p(r), r = (p - i / 64) / (1 + i / 64) in
// [0, 1/64) by its Taylor series to r^8 (truncation < 3e-18)
__device__ __forceinline__ double log1p_tab(double p, const FastLogTabs& T) {
  const int i = min(64, (int)(p * 64.0));
  const double2 L = T.li[i];
  const double r = (p - i * (1.0 / 64.0)) * L.y;
  double q = -1.0 / 8.0;
  q = fma(q, r, 1.0 / 7.0);
  q = fma(q, r, -1.0 / 6.0);
  q = fma(q, r, 1.0 / 5.0);
  q = fma(q, r, -1.0 / 4.0);
  q = fma(q, r, 1.0 / 3.0);
  q = fma(q, r, -1.0 / 2.0);
  q = fma(q, r, 1.0);
  return fma(q, r, L.x);
}

// log(w), w > 0 finite (w <= 0: -inf): w = m 2^e with m in [1, 2)
__device__ __forceinline__ double log_tab(double w, const FastLogTabs& T) {
  if (!(w > 0.0)) return -INFINITY;
  int e;
  const double m = 2.0 * frexp(w, &e);   // frexp: [0.5, 1)
  constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
  const double e1 = (double)(e - 1);
  return fma(e1, LN2_HI, fma(e1, LN2_LO, log1p_tab(m - 1.0, T)));
}

// exp(x) for x <= 0 (x < -745.2: 0): x = k ln2 / 64 + r, |r| <= ln2 / 128, 2^(k/64) from
// the table, expm1(r) by its Taylor series to r^6
__device__ __forceinline__ double exp_tab_neg(double x, const FastLogTabs& T) {
  if (x < -745.2) return 0.0;
  constexpr double K64 = 92.33248261689365951;   // 64 / ln 2
  constexpr double C_HI = 1.08304246962070465088e-02, C_LO = 2.98155597433513719e-12;   // ln2 / 64
  const double kd = rint(x * K64);
  const int k = (int)kd;
  const double r = fma(-kd, C_LO, fma(-kd, C_HI, x));
  double q = 1.0 / 720.0;
  q = fma(q, r, 1.0 / 120.0);
  q = fma(q, r, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  const double t = T.et[k & 63];
  return ldexp(fma(t * r, q, t), k >> 6);
}

// fatmin for the tabulated keyed scan: x scaled by 1 / t, one division for 2 / q and the
// derivative's 1 / (1 + p) (q = 2 + 2x + x^2: p = 2 / q, 1 / (1 + p) = q / (q + 2)), log1p —
// within a few ulps of fatmin2
__device__ __forceinline__ double fatmin_fast(double a, double b, double t, double it, double* da,
                                              const FastLogTabs& T) {
  if (b == -INFINITY) {
    *da = 0.0;
    return -INFINITY;
  }
  const double x = fabs(a - b) * it;
  const double q = fma(x, 2.0 + x, 2.0);
  const double qq = q * (q + 2.0);
  // x = inf (a or b infinite): q(q+2) = inf, p = dq = 0 as the divided form gives
  const bool big = isinf(qq);
  const double w = big ? 0.0 : rcp_nr(qq);
  const double p = big ? 0.0 : 2.0 * (q + 2.0) * w;
  const double dq = big ? 0.0 : 4.0 * (1.0 + x) * w;   // -pareto'(x) / (1 + pareto(x))
  *da = (a < b) ? 1.0 - dq : dq;
  return fmin(a, b) - t * log1p_tab(p, T);
}

// online log-sum-exp with M gradient slots (running max m, s0 = sum exp(a - m),
// g_j = sum exp(a - m) da/dtheta_j)
template <int M, bool BWD>
struct LseState {
  double m, s0, g[BWD ? M : 1];
  __device__ void init() {
    m = -INFINITY;
    s0 = 0.0;
#pragma unroll
    for (int j = 0; j < (BWD ? M : 1); ++j) g[j] = 0.0;
  }
  // one exp on either branch (exp(-|a - m|) is exp(m - a) for a new maximum, exp(a - m)
  // otherwise, bitwise), so lanes that disagree on the branch do not pay two
  __device__ void add(double a, const double* da) {
    if (a == -INFINITY) return;
    const double e = exp(-fabs(a - m));   // 0 when m = -inf
    if (a > m) {
      s0 = fma(s0, e, 1.0);
      if (BWD) {
#pragma unroll
        for (int j = 0; j < M; ++j) g[j] = fma(g[j], e, da[j]);
      }
      m = a;
    } else {
      s0 += e;
      if (BWD) {
#pragma unroll
        for (int j = 0; j < M; ++j) g[j] = fma(e, da[j], g[j]);
      }
    }
  }
  __device__ void merge(double m2, double s2, const double* g2) {
    if (s2 == 0.0) return;
    const double M_ = fmax(m, m2);
    const double r1 = (s0 == 0.0) ? 0.0 : exp(m - M_), r2 = exp(m2 - M_);
    s0 = s0 * r1 + s2 * r2;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) g[j] = g[j] * r1 + g2[j] * r2;
    }
    m = M_;
  }
};

// The sampling step's per-(output, candidate) part (qn_samples_norms; fused into the restart
// scan hvi_kdb): mu = ym + s (c + a) with a the mean row of R, and the new-point root
// L22 = sqrt(s^2 (kxx - |C k|^2) - |L21|^2) from the per-tile partial sums of squares Pj
// (P[tile][class][c], class 0: kernel rows, 1: baseline rows), with psd_safe_cholesky's 1x1
// ladder (plain, then total jitter 1e-8 10^(t-1), t = 1..6); flag = 1 when every rung fails.
// One definition so that both kernels produce bitwise the same samples.
// The partial-norm sums of one (output, candidate): ssv over the class-0 tile sums (rows < n),
// ssw over class 1 (baseline rows).  Canonical order, shared by every kernel that forms them:
// four interleaved chains s_k = sum_{i} P[4 i + k] (i ascending), then (s_0 + s_1) + (s_2 + s_3)
// — so that one thread (qn_mu_l22) and four lanes (hvi_kdw) produce the same bits.
__device__ __forceinline__ double qn_norm_chain(const double* __restrict__ Pj, int nrt_used, int b, int c, int cls,
                                                int k) {
  double a = 0.0;
  int rt = k;
  for (; rt + 12 < nrt_used; rt += 16) {   // four loads of the chain in flight
    const double x0 = Pj[((size_t)rt * 2 + cls) * b + c], x1 = Pj[((size_t)(rt + 4) * 2 + cls) * b + c];
    const double x2 = Pj[((size_t)(rt + 8) * 2 + cls) * b + c], x3 = Pj[((size_t)(rt + 12) * 2 + cls) * b + c];
    a += x0;
    a += x1;
    a += x2;
    a += x3;
  }
  for (; rt < nrt_used; rt += 4) a += Pj[((size_t)rt * 2 + cls) * b + c];
  return a;
}

// mu, L22 (psd_safe ladder of 6) and the failure flag from the two norm sums
__device__ __forceinline__ void qn_mu_l22_from(double ssv, double ssw, double a, double s, double cc, double ym,
                                               double kxx, double& mu, double& l22, int& flag) {
  mu = ym + s * (cc + a);
  const double var = s * s * (kxx - ssv);
  const double br = var - ssw;
  l22 = nan("");
  flag = 1;
  if (!isnan(br)) {
    for (int t = 0; t <= 6; ++t) {
      const double jit = (t == 0) ? 0.0 : 1e-8 * pow(10.0, (double)(t - 1));
      if (br + jit > 0.0) {
        l22 = sqrt(br + jit);
        flag = 0;
        break;
      }
    }
  }
}

__device__ __forceinline__ void qn_mu_l22(const double* __restrict__ Pj, int nrt_used, int b, int c, double a,
                                          double s, double cc, double ym, double kxx, double& mu, double& l22,
                                          int& flag) {
  double ch[2][4];
#pragma unroll
  for (int cls = 0; cls < 2; ++cls)
#pragma unroll
    for (int k = 0; k < 4; ++k) ch[cls][k] = qn_norm_chain(Pj, nrt_used, b, c, cls, k);
  const double ssv = (ch[0][0] + ch[0][1]) + (ch[0][2] + ch[0][3]);
  const double ssw = (ch[1][0] + ch[1][1]) + (ch[1][2] + ch[1][3]);
  qn_mu_l22_from(ssv, ssw, a, s, cc, ym, kxx, mu, l22, flag);
}

// objective value of one sample: g = a (mu + h + L22 z) + b (h absent without sample rows)
__device__ __forceinline__ double qn_sample_obj(double mu, double hv, bool has_h, double l22, double zv, double A,
                                               double B) {
  const double y = (has_h ? mu + hv : mu) + l22 * zv;
  return fma(A, y, B);
}

// Where the restart scan takes its samples from: G (S x m x b, written by qn_samples_norms),
// or, with R set, formed in its staging from R's rows and the partial norms (the sampling
// launch fused away); sample s's workgroup 0 also writes L22 and the flags the backward and
// the dX reduction read.
struct KbSamples {
  const double* R;        // m x Rr x b projection, nullptr: read G
  const double* P;        // m x nrt x 2 x b partial norms
  const double *cc, *ym, *ys, *kxx, *zq, *oa, *ob;
  double* L22;
  int* flags;
  int n, nb, nh, nrt, nrt_used;
};

// Workgroup bitonic sort of P2 (power of two) unique integer keys in LDS (cells_kd.hip, box_device.hip).
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const int lo = __shfl_xor((int)(unsigned)v, m, 64), hi = __shfl_xor((int)(unsigned)(v >> 32), m, 64);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// Bitonic sort of P2 (a power of two) unique keys in LDS.  Stages whose partner distance j is
// at least 64 exchange through LDS (one barrier each); the stages with j < 64 pair lanes of one
// wave (index i = tid + NT t, so a wave holds 64 consecutive keys) and run in registers by
// xor-shuffles, min / max per pair, with one barrier per merge size: 41 instead of 91 barriers
// per sort at P2 = 8192 and NT = 1024.  Same result as the compare-and-swap network (keys are unique).
__device__ __forceinline__ unsigned int shfl_xor_key(unsigned int v, int m) {
  return (unsigned int)__shfl_xor((int)v, m, 64);
}
__device__ __forceinline__ unsigned long long shfl_xor_key(unsigned long long v, int m) { return shfl_xor_u64(v, m); }

template <typename KT, int NT>
__device__ __forceinline__ void wg_bitonic(KT* a, int P2) {
  for (int k = 2; k <= P2; k <<= 1) {
    int j = k >> 1;
    for (; j >= 64; j >>= 1) {
      for (int i = threadIdx.x; i < P2; i += NT) {
        const int l = i ^ j;
        if (l > i) {
          const KT x = a[i], y = a[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < P2; i += NT) {
      KT x = a[i];
      const bool up = (i & k) == 0;
      for (int jj = j; jj > 0; jj >>= 1) {
        const KT y = shfl_xor_key(x, jj);
        // the lower index of a pair keeps the minimum in an ascending run, the maximum otherwise
        x = (((i & jj) == 0) == up) ? (x < y ? x : y) : (x < y ? y : x);
      }
      a[i] = x;
    }
    __syncthreads();
  }
}

}  // namespace evr
