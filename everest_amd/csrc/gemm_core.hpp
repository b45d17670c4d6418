// f64 matrix-core GEMM tile engine for gfx950 (v_mfma_f64_16x16x4f64), shared by the
// posterior, the qNEHVI projections and the general GEMM entry point.
//
// One BM x BN output tile per 256-thread workgroup (4 waves in a 2 x 2 grid, each wave
// (BM/2) x (BN/2) = FM x FN MFMA blocks of 16 x 16).  K advances in steps of BK:
//   * the next step's operands are fetched into registers as 16-byte pairs (double2) while
//     the current step's MFMAs run;
//   * they are written to the other half of a double-buffered LDS image after the MFMAs, so
//     one workgroup barrier per k-step suffices;
//   * LDS images keep the global orientation (no transpose on the write), padded so that
//     both the 16-byte writes and the 8-byte fragment reads are bank-conflict free:
//       A k-contiguous  As[BM][BK + 2]      fragment lane l: As[m0 + (l & 15)][k + (l >> 4)]
//       A m-contiguous  As[BK][BM + 16]     fragment lane l: As[k + (l >> 4)][m0 + (l & 15)]
//       B n-contiguous  Bs[BK][BN + 16]     fragment lane l: Bs[k + (l >> 4)][n0 + (l & 15)]
// The operand fetchers are functors, so the B operand can be generated on the fly (the
// backward projection's gR from R, dG and per-candidate coefficients) and the epilogue is a
// functor over the MFMA D layout: register r of lane l of block (a, b) holds
//   D[row = wm + 16 a + (l >> 4) + 4 r][col = wn + 16 b + (l & 15)].
#pragma once
#include <hip/hip_runtime.h>

namespace evr {

using dg_double2 = __attribute__((ext_vector_type(2))) double;
using dg_double4 = __attribute__((ext_vector_type(4))) double;

template <int BM_, int BN_, int BK_, bool TA_>
struct DgCfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_;
  static constexpr bool TA = TA_;                        // A stored m-contiguous (A(i,k) = A[k][i])
  static constexpr int AST = TA ? (BM + 16) : (BK + 2);  // A image row stride (doubles)
  static constexpr int AROWS = TA ? BK : BM;
  static constexpr int BST = BN + 16;
  static constexpr int ASZ = AROWS * AST, BSZ = BK * BST;
  static constexpr int LDS_DOUBLES = 2 * (ASZ + BSZ);
  static constexpr int AP = BM * BK / 512, BP = BK * BN / 512;   // double2 pairs per thread and k-step
  static constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  static_assert(AP * 512 == BM * BK && BP * 512 == BK * BN, "tile does not split over 256 threads in pairs");
  static_assert(FM >= 1 && FN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole 16 x 16 blocks");
  static_assert(BK % 4 == 0, "k-step must be a multiple of the MFMA depth");
  // k-contiguous A: one 16-byte fragment read feeds two MFMAs.  Over each 8-deep k block the
  // first MFMA takes k = 2 (l >> 4), the second k = 2 (l >> 4) + 1 — the contraction order is
  // permuted identically in A and B (rows of 144 B keep the 16-byte reads aligned)
  static constexpr bool P128 = !TA && BK % 8 == 0;
  // independent accumulation chains per output: the k-step's four 4-deep MFMA slices go to
  // four accumulators, summed (c0 + c1) + (c2 + c3) at the end.  The operators these GEMMs
  // apply (the fused root C = Lv^T L^-1, L^-1) have entries far larger than their products
  // with a kernel column, so the rounding of the long running sums sets the error of R and,
  // through the L22^2 = var - |C k|^2 cancellation, of the samples: four chains cut the
  // rounding steps each product goes through by 4x (measured on the config-3 state,
  // tools/diag_split.py)
  static constexpr int NCH = BK / 4;
  static_assert(NCH == 4, "four chains: one per 4-deep slice of the 16-deep k-step");
};

// The workgroup's accumulators over k in [kbeg, kend) (kbeg a multiple of BK).  The
// fetchers receive tile-local coordinates and the absolute k of the pair's first element:
//   TA false: fa(r, k) = {A(r, k), A(r, k + 1)}        r in [0, BM), k - kbeg even
//   TA true:  fa(k, c) = {A(c, k), A(c + 1, k)}        c in [0, BM) even
//   fb(k, c)          = {B(k, c), B(k, c + 1)}        c in [0, BN) even
// and return zeros outside the operands (k >= kend included).
// no-op per-k-step hook (see dg_mainloop's fx)
struct DgNoHook {
  __device__ __forceinline__ void prefetch(int) {}
  __device__ __forceinline__ void stage(double*) {}
  __device__ __forceinline__ void step(const double*, int, int) {}
};

// fx: per-k-step hook for work over the staged B tile besides the MFMAs (the mean row
// alpha^T B of the posterior): fx.prefetch(k0) is called with each step's operand fetch,
// fx.stage(Bs) when that step's B image is written (the image's padding columns BN .. BST - 1
// are free for the hook), fx.step(Bs, k0, kn) once the step's B image (BK x BST doubles, rows
// k0 .. k0 + kn - 1 valid) is visible to every wave, before the MFMAs.
template <class C, class FA, class FB, class FX>
__device__ __forceinline__ void dg_mainloop(double* __restrict__ lds, int kbeg, int kend, FA fa, FB fb,
                                            dg_double4 (&acc)[C::FM][C::FN], FX& fx) {
  double* As0 = lds;
  double* Bs0 = lds + 2 * C::ASZ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * C::WM, wn = (wave & 1) * C::WN;
  dg_double4 ch[C::NCH][C::FM][C::FN];
#pragma unroll
  for (int h = 0; h < C::NCH; ++h)
#pragma unroll
    for (int a = 0; a < C::FM; ++a)
#pragma unroll
      for (int b = 0; b < C::FN; ++b) ch[h][a][b] = dg_double4{0.0, 0.0, 0.0, 0.0};
  int ar[C::AP], ac[C::AP], br[C::BP], bc[C::BP];
#pragma unroll
  for (int u = 0; u < C::AP; ++u) {
    const int e = u * 256 + tid;
    constexpr int PR = C::TA ? C::BM / 2 : C::BK / 2;   // pairs per image row
    ar[u] = e / PR;
    ac[u] = (e % PR) * 2;
  }
#pragma unroll
  for (int u = 0; u < C::BP; ++u) {
    const int e = u * 256 + tid;
    constexpr int PR = C::BN / 2;
    br[u] = e / PR;
    bc[u] = (e % PR) * 2;
  }
  dg_double2 ra[C::AP], rb[C::BP];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < C::AP; ++u) ra[u] = C::TA ? fa(k0 + ar[u], ac[u]) : fa(ar[u], k0 + ac[u]);
#pragma unroll
    for (int u = 0; u < C::BP; ++u) rb[u] = fb(k0 + br[u], bc[u]);
    fx.prefetch(k0);
  };
  auto stage = [&](int buf) {
    double* As = As0 + buf * C::ASZ;
    double* Bs = Bs0 + buf * C::BSZ;
#pragma unroll
    for (int u = 0; u < C::AP; ++u) *(dg_double2*)(As + ar[u] * C::AST + ac[u]) = ra[u];
#pragma unroll
    for (int u = 0; u < C::BP; ++u) *(dg_double2*)(Bs + br[u] * C::BST + bc[u]) = rb[u];
    fx.stage(Bs);
  };
  auto combine = [&]() {
#pragma unroll
    for (int a = 0; a < C::FM; ++a)
#pragma unroll
      for (int b = 0; b < C::FN; ++b) acc[a][b] = (ch[0][a][b] + ch[1][a][b]) + (ch[2][a][b] + ch[3][a][b]);
  };
  if (kbeg >= kend) {
    combine();
    return;
  }
  const int nk = (kend - kbeg + C::BK - 1) / C::BK;
  fetch(kbeg);
  stage(0);
  __syncthreads();
  const int i = lane & 15, q = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) fetch(kbeg + (kt + 1) * C::BK);
    const double* As = As0 + (kt & 1) * C::ASZ;
    const double* Bs = Bs0 + (kt & 1) * C::BSZ;
    fx.step(Bs, kbeg + kt * C::BK, min(C::BK, kend - kbeg - kt * C::BK));
    if constexpr (C::P128) {
#pragma unroll
      for (int kk = 0; kk < C::BK; kk += 8) {
        dg_double2 af[C::FM];
        double bf0[C::FN], bf1[C::FN];
#pragma unroll
        for (int a = 0; a < C::FM; ++a) af[a] = *(const dg_double2*)(As + (wm + a * 16 + i) * C::AST + kk + 2 * q);
#pragma unroll
        for (int b = 0; b < C::FN; ++b) {
          bf0[b] = Bs[(kk + 2 * q) * C::BST + wn + b * 16 + i];
          bf1[b] = Bs[(kk + 2 * q + 1) * C::BST + wn + b * 16 + i];
        }
#pragma unroll
        for (int a = 0; a < C::FM; ++a)
#pragma unroll
          for (int b = 0; b < C::FN; ++b) {
            const int h = kk / 4;   // chains (kk / 8) * 2 + {0, 1}
            ch[h][a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a][0], bf0[b], ch[h][a][b], 0, 0, 0);
            ch[h + 1][a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a][1], bf1[b], ch[h + 1][a][b], 0, 0, 0);
          }
      }
    } else {
#pragma unroll
    for (int kk = 0; kk < C::BK; kk += 4) {
      double af[C::FM], bf[C::FN];
#pragma unroll
      for (int a = 0; a < C::FM; ++a)
        af[a] = C::TA ? As[(kk + q) * C::AST + wm + a * 16 + i] : As[(wm + a * 16 + i) * C::AST + kk + q];
#pragma unroll
      for (int b = 0; b < C::FN; ++b) bf[b] = Bs[(kk + q) * C::BST + wn + b * 16 + i];
#pragma unroll
      for (int a = 0; a < C::FM; ++a)
#pragma unroll
        for (int b = 0; b < C::FN; ++b)
          ch[kk / 4][a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], ch[kk / 4][a][b], 0, 0, 0);
    }
    }
    if (kt + 1 < nk) stage((kt + 1) & 1);
    __syncthreads();
  }
  combine();
}

template <class C, class FA, class FB>
__device__ __forceinline__ void dg_mainloop(double* __restrict__ lds, int kbeg, int kend, FA fa, FB fb,
                                            dg_double4 (&acc)[C::FM][C::FN]) {
  DgNoHook h;
  dg_mainloop<C>(lds, kbeg, kend, fa, fb, acc, h);
}

// visit the accumulators: f(tile_row, tile_col, value)
template <class C, class F>
__device__ __forceinline__ void dg_for_each(const dg_double4 (&acc)[C::FM][C::FN], F f) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * C::WM, wn = (wave & 1) * C::WN;
  const int i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int a = 0; a < C::FM; ++a)
#pragma unroll
    for (int b = 0; b < C::FN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) f(wm + a * 16 + q + 4 * r, wn + b * 16 + i, acc[a][b][r]);
}

// 16-byte pair fetch {p[0], p[1]} with validity flags.  VEC: 16-byte aligned rows and even
// extents, so a pair is valid or invalid as a whole (v1 == v0): one predicated 16-byte load.
// Otherwise two 8-byte loads (odd leading dimensions, unaligned bases, odd extents).
template <bool VEC>
__device__ __forceinline__ dg_double2 dg_pair(const double* p, bool v0, bool v1) {
  if (VEC) return v0 ? *(const dg_double2*)p : dg_double2{0.0, 0.0};
  return dg_double2{v0 ? p[0] : 0.0, v1 ? p[1] : 0.0};
}

}  // namespace evr
