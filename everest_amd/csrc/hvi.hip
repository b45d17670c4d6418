// Box-cell hypervolume-improvement scan (q = 1), forward and backward, on gfx950.
//
// HVI_s(c) = sum_{cells k of sample s} prod_j max(0, min(g_scj, u_kj) - l_kj)
// ([upstream] qExpectedHypervolumeImprovement._compute_qehvi, the hot loop of BoFire's
// qNEHVI, bofire/strategies/predictives/qnehvi.py:39-52).
//
// "Tropical GEMM" tiling: a 256-thread block owns (candidate tile, sample s, chunk of the
// sample's cells).  Threads form TGC cell groups x TGB candidate groups; every thread keeps
// TB = 4 candidates' objective vectors in registers and walks TC = 4 cells per LDS
// sub-chunk, so each cell bound read from LDS feeds 4 candidates and each candidate 4
// cells.  The sample's cells are sorted by their first lower bound on the host, so a
// thread's 4 cells are neighbours and the per-tile test "some objective j has every cell
// lower bound >= every candidate value" skips whole 4x4 tiles that cannot contribute.
// Cell chunks are split across blocks (grid z) to fill the chip at small candidate
// batches (the L-BFGS restarts); per-(sample, chunk) partial sums are reduced in a fixed
// order by a second kernel — results are bitwise reproducible.
#include <algorithm>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int HV_THREADS = 256;
constexpr int HV_TB = 4;
constexpr int HV_TC = 4;

template <int M, int TGB>
__global__ __launch_bounds__(HV_THREADS) void hvi_fwd_tiled(int b, int nchunk, int CB, const double* __restrict__ G,
                                                            const double* __restrict__ lo,
                                                            const double* __restrict__ hi,
                                                            const int* __restrict__ off, double* __restrict__ work) {
  constexpr int TGC = HV_THREADS / TGB;
  constexpr int SUB = TGC * HV_TC;
  constexpr int BB = TGB * HV_TB;
  __shared__ double Ls[M][SUB];
  __shared__ double Us[M][SUB];
  __shared__ double red[TGC][BB + 1];
  const int s = blockIdx.y, chunk = blockIdx.z;
  const int tid = threadIdx.x, tgb = tid % TGB, tgc = tid / TGB;
  const int cbase = blockIdx.x * BB;
  double y[HV_TB][M];
  double ymax[M];
#pragma unroll
  for (int j = 0; j < M; ++j) ymax[j] = -INFINITY;
#pragma unroll
  for (int p = 0; p < HV_TB; ++p) {
    const int c = cbase + tgb + TGB * p;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      y[p][j] = (c < b) ? G[((size_t)s * M + j) * b + c] : -INFINITY;
      ymax[j] = fmax(ymax[j], y[p][j]);
    }
  }
  double acc[HV_TB];
#pragma unroll
  for (int p = 0; p < HV_TB; ++p) acc[p] = 0.0;
  const int k0 = off[s] + chunk * CB;
  const int k1 = min(off[s + 1], k0 + CB);
  for (int ks = k0; ks < k1; ks += SUB) {
    const int nc = min(SUB, k1 - ks);
    for (int e = tid; e < SUB * M; e += HV_THREADS) {
      const int cell = e / M, j = e % M;
      double l = INFINITY, u = INFINITY;
      if (cell < nc) {
        l = lo[(size_t)ks * M + e];
        u = hi[(size_t)ks * M + e];
      }
      Ls[j][cell] = l;
      Us[j][cell] = u;
    }
    __syncthreads();
    bool skip = false;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double lm = Ls[j][tgc * HV_TC];
#pragma unroll
      for (int i = 1; i < HV_TC; ++i) lm = fmin(lm, Ls[j][tgc * HV_TC + i]);
      skip |= lm >= ymax[j];
    }
    if (!skip) {
#pragma unroll
      for (int i = 0; i < HV_TC; ++i) {
        double l[M], u[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          l[j] = Ls[j][tgc * HV_TC + i];
          u[j] = Us[j][tgc * HV_TC + i];
        }
#pragma unroll
        for (int p = 0; p < HV_TB; ++p) {
          double prod = fmax(fmin(y[p][0], u[0]) - l[0], 0.0);
#pragma unroll
          for (int j = 1; j < M; ++j) prod *= fmax(fmin(y[p][j], u[j]) - l[j], 0.0);
          acc[p] += prod;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int p = 0; p < HV_TB; ++p) red[tgc][tgb + TGB * p] = acc[p];
  __syncthreads();
  for (int e = tid; e < BB; e += HV_THREADS) {
    double sum = 0.0;
    for (int g = 0; g < TGC; ++g) sum += red[g][e];
    const int c = cbase + e;
    if (c < b) work[((size_t)s * nchunk + chunk) * b + c] = sum;
  }
}

// d/dg_j of the same sum: pass_j * prod_{k != j} len_k with torch subgradients
// (clamp_min: raw >= 0; minimum: 1 if g < u, 1/2 if g == u, 0 if g > u).
template <int M, int TGB>
__global__ __launch_bounds__(HV_THREADS) void hvi_bwd_tiled(int b, int nchunk, int CB, const double* __restrict__ G,
                                                            const double* __restrict__ lo,
                                                            const double* __restrict__ hi,
                                                            const int* __restrict__ off, double* __restrict__ work) {
  constexpr int TGC = HV_THREADS / TGB;
  constexpr int SUB = TGC * HV_TC;
  constexpr int BB = TGB * HV_TB;
  __shared__ double Ls[M][SUB];
  __shared__ double Us[M][SUB];
  __shared__ double red[TGC][BB + 1];
  const int s = blockIdx.y, chunk = blockIdx.z;
  const int tid = threadIdx.x, tgb = tid % TGB, tgc = tid / TGB;
  const int cbase = blockIdx.x * BB;
  double y[HV_TB][M];
  double ymax[M];
#pragma unroll
  for (int j = 0; j < M; ++j) ymax[j] = -INFINITY;
#pragma unroll
  for (int p = 0; p < HV_TB; ++p) {
    const int c = cbase + tgb + TGB * p;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      y[p][j] = (c < b) ? G[((size_t)s * M + j) * b + c] : -INFINITY;
      ymax[j] = fmax(ymax[j], y[p][j]);
    }
  }
  double g[HV_TB][M];
#pragma unroll
  for (int p = 0; p < HV_TB; ++p)
#pragma unroll
    for (int j = 0; j < M; ++j) g[p][j] = 0.0;
  const int k0 = off[s] + chunk * CB;
  const int k1 = min(off[s + 1], k0 + CB);
  for (int ks = k0; ks < k1; ks += SUB) {
    const int nc = min(SUB, k1 - ks);
    for (int e = tid; e < SUB * M; e += HV_THREADS) {
      const int cell = e / M, j = e % M;
      double l = INFINITY, u = INFINITY;
      if (cell < nc) {
        l = lo[(size_t)ks * M + e];
        u = hi[(size_t)ks * M + e];
      }
      Ls[j][cell] = l;
      Us[j][cell] = u;
    }
    __syncthreads();
    bool skip = false;  // strict: a tie g == l still carries a subgradient
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double lm = Ls[j][tgc * HV_TC];
#pragma unroll
      for (int i = 1; i < HV_TC; ++i) lm = fmin(lm, Ls[j][tgc * HV_TC + i]);
      skip |= lm > ymax[j];
    }
    if (!skip) {
#pragma unroll
      for (int i = 0; i < HV_TC; ++i) {
        double l[M], u[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          l[j] = Ls[j][tgc * HV_TC + i];
          u[j] = Us[j][tgc * HV_TC + i];
        }
#pragma unroll
        for (int p = 0; p < HV_TB; ++p) {
          double len[M], pass[M];
#pragma unroll
          for (int j = 0; j < M; ++j) {
            const double raw = fmin(y[p][j], u[j]) - l[j];
            len[j] = fmax(raw, 0.0);
            const double dmin = (y[p][j] < u[j]) ? 1.0 : ((y[p][j] == u[j]) ? 0.5 : 0.0);
            pass[j] = (raw >= 0.0) ? dmin : 0.0;
          }
          double pre[M];
          pre[0] = 1.0;
#pragma unroll
          for (int j = 1; j < M; ++j) pre[j] = pre[j - 1] * len[j - 1];
          double suf = 1.0;
#pragma unroll
          for (int j = M - 1; j >= 0; --j) {
            g[p][j] = fma(pass[j], pre[j] * suf, g[p][j]);
            suf *= len[j];
          }
        }
      }
    }
    __syncthreads();
  }
  for (int j = 0; j < M; ++j) {
#pragma unroll
    for (int p = 0; p < HV_TB; ++p) {
      double v = 0.0;
#pragma unroll
      for (int jj = 0; jj < M; ++jj)
        if (jj == j) v = g[p][jj];
      red[tgc][tgb + TGB * p] = v;
    }
    __syncthreads();
    for (int e = tid; e < BB; e += HV_THREADS) {
      double sum = 0.0;
      for (int q = 0; q < TGC; ++q) sum += red[q][e];
      const int c = cbase + e;
      if (c < b) work[(((size_t)s * nchunk + chunk) * M + j) * b + c] = sum;
    }
    __syncthreads();
  }
}

// acq[c] = (1/S) sum_{s, chunk} work[s][chunk][c] — block of 16 candidates x 16 partial
// groups, fixed-order tree over the groups (bitwise reproducible).  A candidate whose
// new-point Cholesky block failed (flags[j][c] != 0 for some j) gets NaN.
__global__ __launch_bounds__(256) void hvi_reduce_fwd(int S, int nchunk, int b, int m, const double* __restrict__ work,
                                                      const int* __restrict__ flags, double* __restrict__ acq) {
  __shared__ double red[16][17];
  const int cx = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cx;
  const int tot = S * nchunk;
  double sum = 0.0;
  if (c < b)
    for (int k = g; k < tot; k += 16) sum += work[(size_t)k * b + c];
  red[g][cx] = sum;
  __syncthreads();
  for (int o = 8; o > 0; o >>= 1) {
    if (g < o) red[g][cx] += red[g + o][cx];
    __syncthreads();
  }
  if (g == 0 && c < b) {
    bool bad = false;
    if (flags)
      for (int j = 0; j < m; ++j) bad |= flags[(size_t)j * b + c] != 0;
    acq[c] = bad ? nan("") : red[0][cx] / (double)S;
  }
}

// dG[s][j][c] = gout[c]/S * sum_chunk work[s][chunk][j][c]
__global__ void hvi_reduce_bwd(int S, int nchunk, int M, int b, const double* __restrict__ work,
                               const double* __restrict__ gout, double* __restrict__ dG) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)S * M * b) return;
  const int c = (int)(e % b);
  const int j = (int)((e / b) % M);
  const int s = (int)(e / ((long long)b * M));
  double sum = 0.0;
  for (int k = 0; k < nchunk; ++k) sum += work[(((size_t)s * nchunk + k) * M + j) * b + c];
  dG[e] = (gout ? gout[c] : 1.0) / (double)S * sum;
}

struct HviPlan {
  int tgb, bb, ctiles, nchunk, cb;
};

static HviPlan hvi_plan(const evr_qnehvi_state* st, int b) {
  HviPlan p;
  p.tgb = (b <= 32) ? 4 : 16;
  p.bb = p.tgb * HV_TB;
  p.ctiles = (b + p.bb - 1) / p.bb;
  const int sub = (HV_THREADS / p.tgb) * HV_TC;
  const int maxc = st->max_cells > 0 ? st->max_cells : 1;
  // enough blocks to fill 256 CUs several times over, chunks a multiple of the sub-chunk
  const long long base = (long long)p.ctiles * st->S;
  int want = (int)((4096 + base - 1) / base);
  const int maxchunks = (maxc + sub - 1) / sub;
  p.nchunk = std::max(1, std::min(want, maxchunks));
  int cb = (maxc + p.nchunk - 1) / p.nchunk;
  cb = ((cb + sub - 1) / sub) * sub;
  p.cb = cb;
  p.nchunk = (maxc + cb - 1) / cb;
  return p;
}

}  // namespace evr

using namespace evr;

#define EVR_M_SWITCH(m, MACRO)                                                        \
  switch (m) {                                                                        \
    case 1: MACRO(1); break;                                                          \
    case 2: MACRO(2); break;                                                          \
    case 3: MACRO(3); break;                                                          \
    case 4: MACRO(4); break;                                                          \
    case 5: MACRO(5); break;                                                          \
    case 6: MACRO(6); break;                                                          \
    case 7: MACRO(7); break;                                                          \
    case 8: MACRO(8); break;                                                          \
    default: EVR_CHECK(false, "number of objectives m=%d not supported (1..8)", m);   \
  }

extern "C" {

long long evr_hvi_workspace_doubles(const evr_qnehvi_state* st, int b, int backward) {
  if (!st || b <= 0) return 0;
  HviPlan p = hvi_plan(st, b);
  return (long long)st->S * p.nchunk * b * (backward ? st->m : 1);
}

int evr_hvi_forward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                    double* work, double* acq) {
  EVR_CHECK(st && st->S >= 1 && work && acq, "evr_hvi_forward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  HviPlan p = hvi_plan(st, b);
  dim3 grid(p.ctiles, st->S, p.nchunk);
#define L(MM)                                                                                                   \
  if (p.tgb == 4)                                                                                               \
    hvi_fwd_tiled<MM, 4><<<grid, HV_THREADS, 0, s>>>(b, p.nchunk, p.cb, G, st->cell_lo, st->cell_hi,            \
                                                     st->cell_off, work);                                       \
  else                                                                                                          \
    hvi_fwd_tiled<MM, 16><<<grid, HV_THREADS, 0, s>>>(b, p.nchunk, p.cb, G, st->cell_lo, st->cell_hi,           \
                                                      st->cell_off, work)
  EVR_M_SWITCH(st->m, L);
#undef L
  EVR_LAUNCH_CHECK();
  hvi_reduce_fwd<<<cdiv(b, 16), 256, 0, s>>>(st->S, p.nchunk, b, st->m, work, flags, acq);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_hvi_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const double* gout,
                     double* work, double* dG) {
  EVR_CHECK(st && st->S >= 1 && work && dG, "evr_hvi_backward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  HviPlan p = hvi_plan(st, b);
  dim3 grid(p.ctiles, st->S, p.nchunk);
#define L(MM)                                                                                                   \
  if (p.tgb == 4)                                                                                               \
    hvi_bwd_tiled<MM, 4><<<grid, HV_THREADS, 0, s>>>(b, p.nchunk, p.cb, G, st->cell_lo, st->cell_hi,            \
                                                     st->cell_off, work);                                       \
  else                                                                                                          \
    hvi_bwd_tiled<MM, 16><<<grid, HV_THREADS, 0, s>>>(b, p.nchunk, p.cb, G, st->cell_lo, st->cell_hi,           \
                                                      st->cell_off, work)
  EVR_M_SWITCH(st->m, L);
#undef L
  EVR_LAUNCH_CHECK();
  const long long tot = (long long)st->S * st->m * b;
  hvi_reduce_bwd<<<cdiv(tot, 256), 256, 0, s>>>(st->S, p.nchunk, st->m, b, work, gout, dG);
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
