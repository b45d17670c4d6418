// Box-cell hypervolume-improvement scan (q = 1): forward, and fused forward + backward.
//
// HVI_s(c) = sum_{cells k of sample s} prod_j max(0, min(g_scj, u_kj) - l_kj)
// ([upstream] qExpectedHypervolumeImprovement._compute_qehvi, the hot loop of BoFire's
// qNEHVI, bofire/strategies/predictives/qnehvi.py:39-52).
//
// "Tropical GEMM" tiling: a 256-thread block owns (candidate tile, sample s, chunk of the
// sample's cells).  Threads form TGC cell groups x TGB candidate groups; every thread keeps
// TB = 4 candidates' objective vectors in registers and walks TC = 4 cells per LDS
// sub-chunk, so each cell bound read from LDS feeds 4 candidates and each candidate 4
// cells.  Cells are sorted by their first lower bound, so a thread's 4 cells are
// neighbours and the per-tile test "some objective j has every cell lower bound >= every
// candidate value" skips whole 4x4 tiles that cannot contribute.
//
// Cells arrive either as explicit [lo, hi] rows (host partition) or compressed: one 64-bit
// key of defining-point indices per cell plus the sample's point table in LDS
// (box_device.hip) — 8 bytes of HBM traffic per cell instead of 16 m, decoded while the
// sub-chunk is staged into LDS.
//
// The backward kernel computes the forward value in the same pass (the product of the
// clamped lengths is its prefix product), so forward_backward is one scan.  Cell chunks
// are split across blocks (grid z) to fill the chip at small candidate batches (the L-BFGS
// restarts); per-(sample, chunk) partials are reduced in a fixed order by a second kernel
// — results are bitwise reproducible.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int HV_THREADS = 256;
constexpr int HV_TB = 4;
constexpr int HV_TC = 4;

struct HviCells {
  const double* lo;
  const double* hi;
  const int* off;
  const unsigned long long* keys;
  const double* pts;
  const int* rank0;
  int stride;
};

template <int M, int TGB, bool KEYED, bool BWD>
__global__ __launch_bounds__(HV_THREADS) void hvi_tiled(int b, int nchunk, int CB, const double* __restrict__ G,
                                                        HviCells cells, double* __restrict__ work_f,
                                                        double* __restrict__ work_b) {
  constexpr int TGC = HV_THREADS / TGB;
  constexpr int SUB = TGC * HV_TC;
  constexpr int BB = TGB * HV_TB;
  __shared__ double Ls[M][SUB];
  __shared__ double Us[M][SUB];
  __shared__ double red[TGC][BB + 1];
  extern __shared__ __align__(16) unsigned char hv_dyn[];  // KEYED: point table + rank table
  const int s = blockIdx.y, chunk = blockIdx.z;
  const int tid = threadIdx.x, tgb = tid % TGB, tgc = tid / TGB;
  const int cbase = blockIdx.x * BB;
  double* spt = (double*)hv_dyn;
  int* srk = (int*)(spt + (KEYED ? (size_t)cells.stride * M : 0));
  if (KEYED) {
    const double* gp = cells.pts + (size_t)s * cells.stride * M;
    const int* gr = cells.rank0 + (size_t)s * cells.stride;
    for (int e = tid; e < cells.stride * M; e += HV_THREADS) spt[e] = gp[e];
    for (int e = tid; e < cells.stride; e += HV_THREADS) srk[e] = gr[e];
  }
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
  double g[BWD ? HV_TB : 1][M];
#pragma unroll
  for (int p = 0; p < HV_TB; ++p) {
    acc[p] = 0.0;
    if (BWD) {
#pragma unroll
      for (int j = 0; j < M; ++j) g[BWD ? p : 0][j] = 0.0;
    }
  }
  const int k0 = cells.off[s] + chunk * CB;
  const int k1 = min(cells.off[s + 1], k0 + CB);
  for (int ks = k0; ks < k1; ks += SUB) {
    const int nc = min(SUB, k1 - ks);
    if (KEYED) {
      __syncthreads();  // point table staged (first pass) / previous sub-chunk consumed
      for (int e = tid; e < SUB; e += HV_THREADS) {
        double l[M], u[M];
        if (e < nc) {
          CellKey<M>::decode(cells.keys[ks + e], spt, srk, l, u);
        } else {
#pragma unroll
          for (int j = 0; j < M; ++j) l[j] = u[j] = INFINITY;
        }
#pragma unroll
        for (int j = 0; j < M; ++j) {
          Ls[j][e] = l[j];
          Us[j][e] = u[j];
        }
      }
    } else {
      for (int e = tid; e < SUB * M; e += HV_THREADS) {
        const int cell = e / M, j = e % M;
        double l = INFINITY, u = INFINITY;
        if (cell < nc) {
          l = cells.lo[(size_t)ks * M + e];
          u = cells.hi[(size_t)ks * M + e];
        }
        Ls[j][cell] = l;
        Us[j][cell] = u;
      }
    }
    __syncthreads();
    // Tile skip: forward needs g > l somewhere per objective; the backward also carries a
    // subgradient at a tie g == l (clamp_min passes at 0), so it skips only on l > g.
    bool skip = false;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double lm = Ls[j][tgc * HV_TC];
#pragma unroll
      for (int i = 1; i < HV_TC; ++i) lm = fmin(lm, Ls[j][tgc * HV_TC + i]);
      skip |= BWD ? (lm > ymax[j]) : (lm >= ymax[j]);
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
          if (!BWD) {
            double prod = fmax(fmin(y[p][0], u[0]) - l[0], 0.0);
#pragma unroll
            for (int j = 1; j < M; ++j) prod *= fmax(fmin(y[p][j], u[j]) - l[j], 0.0);
            acc[p] += prod;
          } else {
            // d/dg_j: pass_j * prod_{k != j} len_k with torch subgradients
            // (clamp_min: raw >= 0; minimum: 1 if g < u, 1/2 if g == u, 0 if g > u).
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
            acc[p] += pre[M - 1] * len[M - 1];
            double suf = 1.0;
#pragma unroll
            for (int j = M - 1; j >= 0; --j) {
              g[BWD ? p : 0][j] = fma(pass[j], pre[j] * suf, g[BWD ? p : 0][j]);
              suf *= len[j];
            }
          }
        }
      }
    }
    if (!KEYED) __syncthreads();
  }
  // block reduction over the cell groups (fixed order)
  auto reduce_out = [&](auto value_of, double* dst_base, size_t dst_stride_c) {
    __syncthreads();
#pragma unroll
    for (int p = 0; p < HV_TB; ++p) red[tgc][tgb + TGB * p] = value_of(p);
    __syncthreads();
    for (int e = tid; e < BB; e += HV_THREADS) {
      double sum = 0.0;
      for (int q = 0; q < TGC; ++q) sum += red[q][e];
      const int c = cbase + e;
      if (c < b) dst_base[c * dst_stride_c] = sum;
    }
  };
  reduce_out([&](int p) { return acc[p]; }, work_f + ((size_t)s * nchunk + chunk) * b, 1);
  if (BWD) {
    for (int j = 0; j < M; ++j) {
      reduce_out(
          [&](int p) {
            double v = 0.0;
#pragma unroll
            for (int jj = 0; jj < M; ++jj)
              if (jj == j) v = g[BWD ? p : 0][jj];
            return v;
          },
          work_b + (((size_t)s * nchunk + chunk) * M + j) * b, 1);
    }
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

// Candidate-group width: fewest (padded candidate slots + per-tile cell staging) per cell.
static int hvi_target_blocks() {
  static int t = [] {
    const char* e = std::getenv("EVR_HVI_TARGET_BLOCKS");  // tuning knob, default 2048
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 2048;
  }();
  return t;
}

static HviPlan hvi_plan(const evr_qnehvi_state* st, int b) {
  HviPlan p;
  int best = 0;
  long long best_cost = 0;
  for (int tgb : {4, 8, 16}) {
    const int bb = tgb * HV_TB;
    const long long cost = (long long)((b + bb - 1) / bb) * (bb + 8);
    if (!best || cost < best_cost) {
      best = tgb;
      best_cost = cost;
    }
  }
  p.tgb = best;
  p.bb = p.tgb * HV_TB;
  p.ctiles = (b + p.bb - 1) / p.bb;
  const int sub = (HV_THREADS / p.tgb) * HV_TC;
  const int maxc = st->max_cells > 0 ? st->max_cells : 1;
  const long long base = (long long)p.ctiles * st->S;
  const int want = (int)((hvi_target_blocks() + base - 1) / base);
  const int maxchunks = (maxc + sub - 1) / sub;
  p.nchunk = std::max(1, std::min(want, maxchunks));
  int cb = (maxc + p.nchunk - 1) / p.nchunk;
  cb = ((cb + sub - 1) / sub) * sub;
  p.cb = cb;
  p.nchunk = (maxc + cb - 1) / cb;
  return p;
}

static HviCells hvi_cells(const evr_qnehvi_state* st) {
  return HviCells{st->cell_lo, st->cell_hi, st->cell_off, st->cell_keys, st->cell_pts, st->cell_rank0,
                  st->pts_stride};
}

template <int M, bool BWD>
static int hvi_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const HviPlan& p, const double* G,
                      double* wf, double* wb) {
  const HviCells cells = hvi_cells(st);
  dim3 grid(p.ctiles, st->S, p.nchunk);
  const bool keyed = st->cell_keys != nullptr;
  const size_t dyn = keyed ? (size_t)st->pts_stride * (M * sizeof(double) + sizeof(int)) : 0;
#define HV_GO(TGB_)                                                                                     \
  if (keyed)                                                                                            \
    hvi_tiled<M, TGB_, true, BWD><<<grid, HV_THREADS, dyn, s>>>(b, p.nchunk, p.cb, G, cells, wf, wb);  \
  else                                                                                                  \
    hvi_tiled<M, TGB_, false, BWD><<<grid, HV_THREADS, 0, s>>>(b, p.nchunk, p.cb, G, cells, wf, wb)
  if (p.tgb == 4) HV_GO(4);
  else if (p.tgb == 8) HV_GO(8);
  else HV_GO(16);
#undef HV_GO
  EVR_LAUNCH_CHECK();
  return 0;
}

static int hvi_check_state(const evr_qnehvi_state* st) {
  EVR_CHECK(st && st->S >= 1 && st->m >= 1 && st->cell_off, "hvi: bad state");
  EVR_CHECK(st->cell_keys ? (st->cell_pts && st->cell_rank0 && st->pts_stride > 0) : (st->cell_lo && st->cell_hi),
            "hvi: state has neither explicit nor compressed cells");
  EVR_CHECK(!st->cell_keys || (size_t)st->pts_stride * (st->m * 8 + 4) <= 64 * 1024,
            "hvi: point table of %d rows exceeds the LDS budget", st->pts_stride);
  return 0;
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
  return (long long)st->S * p.nchunk * b * (backward ? st->m + 1 : 1);
}

int evr_hvi_forward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                    double* work, double* acq) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(work && acq && G, "evr_hvi_forward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  HviPlan p = hvi_plan(st, b);
  int rc = 0;
#define L(MM) rc = hvi_launch<MM, false>(s, st, b, p, G, work, nullptr)
  EVR_M_SWITCH(st->m, L);
#undef L
  if (rc) return rc;
  hvi_reduce_fwd<<<cdiv(b, 16), 256, 0, s>>>(st->S, p.nchunk, b, st->m, work, flags, acq);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_hvi_forward_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                             const double* gout, double* work, double* acq, double* dG) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(work && dG && G, "evr_hvi_forward_backward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  HviPlan p = hvi_plan(st, b);
  double* wf = work;
  double* wb = work + (size_t)st->S * p.nchunk * b;
  int rc = 0;
#define L(MM) rc = hvi_launch<MM, true>(s, st, b, p, G, wf, wb)
  EVR_M_SWITCH(st->m, L);
#undef L
  if (rc) return rc;
  if (acq) {
    hvi_reduce_fwd<<<cdiv(b, 16), 256, 0, s>>>(st->S, p.nchunk, b, st->m, wf, flags, acq);
    EVR_LAUNCH_CHECK();
  }
  const long long tot = (long long)st->S * st->m * b;
  hvi_reduce_bwd<<<cdiv(tot, 256), 256, 0, s>>>(st->S, p.nchunk, st->m, b, wb, gout, dG);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_hvi_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const double* gout,
                     double* work, double* dG) {
  return evr_hvi_forward_backward(stream, st, b, G, nullptr, gout, work, nullptr, dG);
}

}  // extern "C"
