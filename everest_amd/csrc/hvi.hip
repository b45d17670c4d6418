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
#include "qs_tail.hpp"

#ifndef EVR_KD_EXP
#define EVR_KD_EXP 0   // experiment switches of the instrumented builds (0 = production)
#endif
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

// acq[c] = (1/S) sum_{s, chunk} work[s][chunk][c] — block of CX candidates x 256/CX partial
// groups, fixed-order tree over the groups (bitwise reproducible for a given CX; CX = 4 for
// the b <= 32 restart batches, whose wave-split scans leave S x 8 partials per candidate).
// A candidate whose new-point Cholesky block failed (flags[j][c] != 0 for some j) gets NaN.
template <int CX>
__device__ __forceinline__ void reduce_fwd_body(int blk, int S, int nchunk, int b, int m,
                                                const double* __restrict__ work, const int* __restrict__ flags,
                                                double* __restrict__ acq) {
  constexpr int G = 256 / CX;
  __shared__ double red[G][CX + 1];
  const int cx = threadIdx.x % CX, g = threadIdx.x / CX;
  const int c = blk * CX + cx;
  const int tot = S * nchunk;
  double sum = 0.0;
  if (c < b) {
    // 32 partials per thread in flight at once (the restart batch: S x 8 partials over 64
    // groups), summed in the same sequential order as the plain loop
    int k = g;
    for (; k + 31 * G < tot; k += 32 * G) {
      double x[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) x[u] = work[(size_t)(k + u * G) * b + c];
#pragma unroll
      for (int u = 0; u < 32; ++u) sum += x[u];
    }
#pragma unroll 8
    for (; k < tot; k += G) sum += work[(size_t)k * b + c];
  }
  red[g][cx] = sum;
  __syncthreads();
  for (int o = G / 2; o > 0; o >>= 1) {
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

template <int CX>
__global__ __launch_bounds__(256) void hvi_reduce_fwd(int S, int nchunk, int b, int m, const double* __restrict__ work,
                                                      const int* __restrict__ flags, double* __restrict__ acq) {
  reduce_fwd_body<CX>(blockIdx.x, S, nchunk, b, m, work, flags, acq);
}

// dG[s][j][c] = gout[c]/S * sum_chunk work[s][chunk][j][c] (elementwise; nchunk loads in flight)
__device__ __forceinline__ void reduce_bwd_body(int blk, int S, int nchunk, int M, int b,
                                                const double* __restrict__ work, const double* __restrict__ gout,
                                                double* __restrict__ dG) {
  const long long e = (long long)blk * 256 + threadIdx.x;
  if (e >= (long long)S * M * b) return;
  const int c = (int)(e % b);
  const int j = (int)((e / b) % M);
  const int s = (int)(e / ((long long)b * M));
  double sum = 0.0;
#pragma unroll 8
  for (int k = 0; k < nchunk; ++k) sum += work[(((size_t)s * nchunk + k) * M + j) * b + c];
  dG[e] = (gout ? gout[c] : 1.0) / (double)S * sum;
}

// both reductions of a forward + backward scan in one launch: blocks [0, nf) reduce the
// values (CX candidates each), the rest the sample gradients
template <int CX>
__global__ __launch_bounds__(256) void hvi_reduce_fb(int S, int nchunk, int b, int m, int nf,
                                                     const double* __restrict__ work, const int* __restrict__ flags,
                                                     double* __restrict__ acq, const double* __restrict__ dwork,
                                                     const double* __restrict__ gout, double* __restrict__ dG) {
  if ((int)blockIdx.x < nf) reduce_fwd_body<CX>(blockIdx.x, S, nchunk, b, m, work, flags, acq);
  else reduce_bwd_body(blockIdx.x - nf, S, nchunk, m, b, dwork, gout, dG);
}

static void hvi_reduce_fwd_launch(hipStream_t s, int S, int nchunk, int b, int m, const double* work,
                                  const int* flags, double* acq) {
  if (b <= 32)
    hvi_reduce_fwd<4><<<cdiv(b, 4), 256, 0, s>>>(S, nchunk, b, m, work, flags, acq);
  else
    hvi_reduce_fwd<16><<<cdiv(b, 16), 256, 0, s>>>(S, nchunk, b, m, work, flags, acq);
}

__global__ void hvi_reduce_bwd(int S, int nchunk, int M, int b, const double* __restrict__ work,
                               const double* __restrict__ gout, double* __restrict__ dG) {
  reduce_bwd_body(blockIdx.x, S, nchunk, M, b, work, gout, dG);
}

// ---------------------------------------------------------------------------------------
// Sparse scan over kd-ordered cell groups (cells_kd.hip).  A 256-thread workgroup owns
// (sample s, tile of 64 candidates) and ALL of the sample's cells:
//   A. group filter — lane = candidate, each wave walks a quarter of the 16-group chunks;
//      group g passes candidate c iff min-rank_j(g) < t_j(y_c) for every objective (t_j =
//      #{point rows with lower-bound value <= y_j}, binary search in sorted_lo);
//   B. cell filter — the passing (candidate, group) pairs, in candidate-major order, are
//      walked in windows of 256, one pair per thread: 16-bit mask of the group's cells with
//      rank_j < t_j for all j (exact: l <= y, the condition for a non-zero term or, at a tie,
//      a non-zero subgradient);
//   C. evaluation — the exact (cell, candidate) pairs of the window, one per thread: key
//      decoded against the point table in LDS, HVI term (+ its gradient), then an ordered
//      per-candidate sum (pairs of a candidate are contiguous) into the workgroup's
//      accumulators.  Every order is a function of the data only: bitwise reproducible.
// At the bench state ~0.7 % of the dense (cell, candidate) pairs reach C (vs ~32 % of the
// pairs the tiled kernel evaluates).
// ---------------------------------------------------------------------------------------
constexpr int KD_CT = 64;

struct HviKd {
  const int* goff;
  const unsigned long long* gkeys;
  const unsigned short* grk;
  const unsigned short* gbox;
  const double* sv;
  const double* pts;
  const int* rank0;
  int stride;
  int max_groups;
  unsigned long long* counters;
};

struct KdLds {
  size_t pt, r0, gb, mA, pA, bytes;
};

__host__ __device__ inline KdLds kd_lds(int stride, int M, int max_groups) {
  KdLds L;
  const size_t nq = (size_t)(max_groups + 15) / 16;
  size_t o = 0;
  L.pt = o;
  o += (size_t)stride * M * 8;
  L.r0 = o;
  o += (size_t)stride * 4;
  o = (o + 15) & ~(size_t)15;
  L.gb = o;
  o += (size_t)max_groups * 16;
  L.mA = o;
  o += nq * KD_CT * 2;
  o = (o + 15) & ~(size_t)15;
  L.pA = o;
  o += (KD_CT * nq + 4) * 4;   // 4 waves x (16 candidates x nq + 1)
  L.bytes = o;
  return L;
}

// k-th (0-based) set bit of a 16-bit mask
__device__ __forceinline__ int kth_bit16(unsigned int mask, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1) {
    const unsigned int lowbits = mask & ((1u << w) - 1u);
    const int c = __popc(lowbits);
    if (k >= c) {
      k -= c;
      mask >>= w;
      pos += w;
    } else {
      mask = lowbits;
    }
  }
  return pos;
}

// exclusive scan of v over the 256 threads (4 waves): wave shuffle scan + wave totals in
// LDS; returns the prefix, *total gets the sum.  wsum: 4 ints of LDS.
__device__ __forceinline__ int block_scan256(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(incl, o, 64);
    if (lane >= o) incl += x;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int off = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) off += (w < wave) ? wsum[w] : 0;
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return off + incl - v;
}

// DPP cross-lane moves (gfx9 encodings): row_shr:n = 0x110 + n, row_bcast:15 = 0x142,
// row_bcast:31 = 0x143.  Lanes without a valid source keep `old`.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i32(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xF, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = dpp_i32<CTRL, ROWMASK>(0, (int)x);
  const int hi = dpp_i32<CTRL, ROWMASK>(0, (int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// one Hillis-Steele step of the segmented scan: add the source lane's partial if it lies in
// the same segment (segments are contiguous runs of equal key)
template <int CTRL, int ROWMASK, int NV>
__device__ __forceinline__ void seg_step(int key, double (&val)[NV]) {
  const int k2 = dpp_i32<CTRL, ROWMASK>(-2, key);
  double x[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) x[v] = dpp_f64<CTRL, ROWMASK>(val[v]);
  if (k2 == key) {
#pragma unroll
    for (int v = 0; v < NV; ++v) val[v] += x[v];
  }
}
// wave-wide segmented inclusive scan (fixed tree: deterministic)
template <int NV>
__device__ __forceinline__ void seg_scan_wave(int key, double (&val)[NV]) {
  seg_step<0x111, 0xF>(key, val);
  seg_step<0x112, 0xF>(key, val);
  seg_step<0x114, 0xF>(key, val);
  seg_step<0x118, 0xF>(key, val);
  seg_step<0x142, 0xA>(key, val);
  seg_step<0x143, 0xC>(key, val);
}

// packed 16-bit "rank < threshold" test: for every u16 half of w, bit 15 of the half is set
// iff rank < t (ranks and thresholds < 2^15, so the signed 16-bit difference is negative)
typedef short kd_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned int kd_lt16(unsigned int w, unsigned int t) {
  const kd_s16x2 a = __builtin_bit_cast(kd_s16x2, w), b = __builtin_bit_cast(kd_s16x2, t);
  return __builtin_bit_cast(unsigned int, (kd_s16x2)(a - b));
}

// t[s][j][c] = #{point rows p of sample s : lower-bound value_j(p) <= G[s][j][c]} (binary
// search in the sample's ascending values, staged in LDS); one workgroup per (j, s).
__global__ __launch_bounds__(256) void hvi_thresholds(int b, int M, int stride, const double* __restrict__ G,
                                                      const double* __restrict__ sorted_lo, int* __restrict__ th) {
  extern __shared__ double thv[];
  const int j = blockIdx.x, s = blockIdx.y;
  const double* src = sorted_lo + ((size_t)s * M + j) * stride;
  for (int e = threadIdx.x; e < stride; e += 256) thv[e] = src[e];
  __syncthreads();
  const size_t row = ((size_t)s * M + j) * b;
  for (int c = threadIdx.x; c < b; c += 256) {
    const double y = G[row + c];
    int lo = 0, hi = stride;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (thv[mid] <= y) lo = mid + 1;
      else hi = mid;
    }
    th[row + c] = lo;
  }
}

// LDS staging with the loads of 4 elements issued before their stores
template <typename T>
__device__ __forceinline__ void kd_stage(T* __restrict__ dst, const T* __restrict__ src, int n) {
  int e = threadIdx.x;
  for (; e + 3 * 256 < n; e += 4 * 256) {
    const T a = src[e], b = src[e + 256], c = src[e + 512], d = src[e + 768];
    dst[e] = a;
    dst[e + 256] = b;
    dst[e + 512] = c;
    dst[e + 768] = d;
  }
  for (; e < n; e += 256) dst[e] = src[e];
}

// LDS-coherent wave-level sync: this wave's LDS writes are visible to its other lanes
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wave-wide exclusive scan of ints on DPP moves; *total = sum over the wave
__device__ __forceinline__ int wave_scan_excl(int v, int* total) {
  int x = v;
  x += dpp_i32<0x111, 0xF>(0, x);
  x += dpp_i32<0x112, 0xF>(0, x);
  x += dpp_i32<0x114, 0xF>(0, x);
  x += dpp_i32<0x118, 0xF>(0, x);
  x += dpp_i32<0x142, 0xA>(0, x);
  x += dpp_i32<0x143, 0xC>(0, x);
  *total = __builtin_amdgcn_readlane(x, 63);
  return x - v;
}

// Wave-independent sparse scan: the workgroup (sample s, tile of 64 candidates) stages the
// sample's point table, group minima, candidate values and thresholds once; after that
// barrier each wave owns 16 candidates and runs the group filter, the cell filter windows,
// the term evaluation and the accumulation alone (wave-level DPP scans, no workgroup
// barriers) — candidates are wave-exclusive, so the accumulators need no inter-wave order.
#ifndef EVR_KD_PROF
#define EVR_KD_PROF 0
#endif
// phase timers of the instrumented build (EVR_KD_PROF=1): per-wave clock deltas summed into
// counters[4 + phase] (0 stage, 1 group filter + prefix, 2 cell filter, 3 term evaluation,
// 4 segmented scan + accumulate)
#define KD_T0() long long kd_t = EVR_KD_PROF ? clock64() : 0; const long long kd_ts = kd_t; \
  const unsigned long long kd_w0 = EVR_KD_PROF ? wall_clock64() : 0; \
  unsigned long long kd_wst = 0, kd_wpf = 0; long long kd_np = 0, kd_nt = 0
#define KD_WSTAMP(v) do { if (EVR_KD_PROF == 2) v = wall_clock64(); } while (0)
// longest wave (counters[9]) and waves timed (counters[10]) of the instrumented build
#define KD_TEND()                                                                     \
  do {                                                                                \
    if (EVR_KD_PROF && kd.counters && (threadIdx.x & 63) == 0) {                     \
      if (EVR_KD_PROF == 1) {                                                         \
        atomicMax(kd.counters + 9, (unsigned long long)(clock64() - kd_ts));          \
        atomicAdd(kd.counters + 10, 1ull);                                            \
      }                                                                               \
      /* per-wave record (counters[16 + 8 w ...]): wall-clock start, staged, prefixed, */ \
      /* end, sample, split, group pairs, terms (EVR_KD_PROF=2)                        */ \
      const size_t kd_gw = ((size_t)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6); \
      unsigned long long* kd_r = kd.counters + 16 + 8 * kd_gw;                         \
      kd_r[0] = kd_w0;                                                                \
      kd_r[1] = kd_wst;                                                               \
      kd_r[2] = kd_wpf;                                                               \
      kd_r[3] = wall_clock64();                                                       \
      kd_r[4] = (unsigned long long)s;                                                \
      kd_r[5] = (unsigned long long)blockIdx.z;                                       \
      kd_r[6] = (unsigned long long)kd_np;                                            \
      kd_r[7] = (unsigned long long)kd_nt;                                            \
    }                                                                                 \
  } while (0)
#define KD_T(ph)                                                                      \
  do {                                                                                \
    if (EVR_KD_PROF == 1 && kd.counters) {                                            \
      const long long kd_n = clock64();                                               \
      if ((threadIdx.x & 63) == 0) atomicAdd(kd.counters + 4 + (ph), (unsigned long long)(kd_n - kd_t)); \
      kd_t = kd_n;                                                                    \
    }                                                                                 \
  } while (0)

// ---------------------------------------------------------------------------------------
// hvi_kd2 — the sparse scan over the kd-ordered groups (round 1's hvi_kd, whose bitwise twin it
// was, is gone since round 6) with a short instruction stream:
//   * chunk pre-filter: the minimum corner of every 16-group chunk (formed while staging)
//     rejects a (candidate, chunk) entry with one packed test; the surviving entries are
//     compacted by ballot and their 16 group tests run lane-dense, instead of every lane
//     walking the 16 groups of every chunk;
//   * owner lookups by marks: the pair -> entry map of the cell filter and the term -> pair
//     map of the evaluation are built by writing each source's first slot into a 64-entry
//     LDS row and taking a DPP max-scan (one LDS round trip + 6 DPP steps) instead of a
//     binary search of 6-9 dependent LDS reads per lane; the owner's fields then come over
//     ds_bpermute from its registers.
// ---------------------------------------------------------------------------------------
constexpr int KD_MAX_NQ = 32;   // 16-group chunks per sample (cells_kd keeps <= 512 groups)

__device__ __forceinline__ unsigned int pk_min_u16(unsigned int a, unsigned int b) {
  return min(a & 0xFFFFu, b & 0xFFFFu) | (min(a >> 16, b >> 16) << 16);
}

// group / chunk test: every objective's minimum rank below the candidate's threshold
__device__ __forceinline__ bool kd_pass4(const uint4 v, const uint4 t) {
  const unsigned int x = kd_lt16(v.x, t.x) & kd_lt16(v.y, t.y) & kd_lt16(v.z, t.z) & kd_lt16(v.w, t.w);
  return (x & 0x80008000u) == 0x80008000u;
}

// wave-wide inclusive max-scan on DPP moves (lanes without a source see -1)
__device__ __forceinline__ int wave_max_incl(int x) {
  x = max(x, dpp_i32<0x111, 0xF>(-1, x));
  x = max(x, dpp_i32<0x112, 0xF>(-1, x));
  x = max(x, dpp_i32<0x114, 0xF>(-1, x));
  x = max(x, dpp_i32<0x118, 0xF>(-1, x));
  x = max(x, dpp_i32<0x142, 0xA>(-1, x));
  x = max(x, dpp_i32<0x143, 0xC>(-1, x));
  return x;
}

// LDS of hvi_kd2 beyond its static arrays: the sample's point table, the (chunk, candidate)
// group masks and the per-wave u16 prefixes (which first hold the chunk-entry lists).  The
// group minima stay in L2 and the kd keys carry point indices, so neither the rank table nor
// the group table is staged: ~26 KB per workgroup instead of ~37 KB (6 instead of 4
// workgroups per CU on the LDS budget).
struct Kd2Lds {
  size_t pt, gb, mA, pA, bytes;
};
__host__ __device__ inline Kd2Lds kd2_lds(int stride, int M, int max_groups) {
  Kd2Lds L;
  const size_t nq = (size_t)(max_groups + 15) / 16;
  size_t o = 0;
  L.pt = o;
  o += (size_t)stride * M * 8;
  o = (o + 15) & ~(size_t)15;
  L.gb = o;
  o += (size_t)max_groups * 16;
  L.mA = o;
  o += nq * KD_CT * 2;
  o = (o + 15) & ~(size_t)15;
  L.pA = o;
  o += (KD_CT * nq + 4) * 2;
  L.bytes = o;
  return L;
}

// DPP move with an undefined old value (no zero-initialised destination): only read by lanes
// whose source lane exists — there the key move below carries the source's key, elsewhere the
// old -2, which matches no key
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64_u(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)x, CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), CTRL, ROWMASK, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// one segmented-scan step; returns whether any lane's source shared its key
template <int CTRL, int ROWMASK, int NV>
__device__ __forceinline__ bool seg_step_x(int key, double (&val)[NV]) {
  const int k2 = dpp_i32<CTRL, ROWMASK>(-2, key);
  const bool same = k2 == key;
  if (__ballot(same) == 0ull) return false;
  double x[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) x[v] = dpp_f64_u<CTRL, ROWMASK>(val[v]);
  if (same) {
#pragma unroll
    for (int v = 0; v < NV; ++v) val[v] += x[v];
  }
  return true;
}
// seg_scan_wave without the steps that would add nothing: segments are contiguous runs, so
// once a row-local shift finds no lane whose source shares its key, no longer shift can; the
// two row-broadcast steps are tested on their own.  The sums equal seg_scan_wave's when the
// keys outside the segments are unique (idle lanes pass -3 - lane).
template <int NV>
__device__ __forceinline__ void seg_scan_wave_x(int key, double (&val)[NV]) {
  if (seg_step_x<0x111, 0xF>(key, val) && seg_step_x<0x112, 0xF>(key, val) && seg_step_x<0x114, 0xF>(key, val))
    seg_step_x<0x118, 0xF>(key, val);
  seg_step_x<0x142, 0xA>(key, val);
  seg_step_x<0x143, 0xC>(key, val);
}

template <int M, bool BWD>
__global__ __launch_bounds__(256) void hvi_kd2(int b, int S, int ntiles, int nsplit, const double* __restrict__ G,
                                               const int* __restrict__ thg, HviKd kd,
                                               const double* __restrict__ gout, double* __restrict__ part,
                                               double* __restrict__ dG, int W, int balance, int ilv) {
  constexpr int NV = BWD ? M + 1 : 1;
  constexpr int CW = KD_CT / 4;            // candidate slots per wave
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kd_dyn[];
  __shared__ double yv[KD_CT][M];
  __shared__ uint4 thp[KD_CT];             // packed 16-bit thresholds (objectives >= M: 1)
  __shared__ double acc[KD_CT][NV];
  __shared__ uint4 cmin[KD_MAX_NQ];        // chunk minimum corners
  __shared__ int mk[4][64];                // per-wave owner marks (cell filter, then evaluation)
  int s, tile;
  {
    const int L = blockIdx.x + ntiles * blockIdx.y;
    if ((S & 7) == 0) {
      const int xcd = L & 7, k = L >> 3;
      s = xcd + 8 * (k / ntiles);
      tile = k % ntiles;
    } else {
      s = blockIdx.y;
      tile = blockIdx.x;
    }
  }
  // W waves share one 16-candidate group and split its chunks (small candidate batches:
  // the L-BFGS restarts), so a tile holds 64 / W candidates
  const int c0 = tile * (KD_CT / W), tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // slot -> candidate: the tile's 4 / W groups of 16 slots each take gsz = ceil(candidates of
  // the tile / groups) candidates, so a split tile (small batches) is balanced across its
  // wave groups (at b = 20: 10 + 10 instead of 16 + 4); full tiles map slot = candidate
  const int ngr = 4 / W;
  const int gsz = (W > 1 && balance) ? min(CW, (min(KD_CT / W, b - c0) + ngr - 1) / ngr) : CW;
  auto cand = [&](int c) { return c0 + (c >> 4) * gsz + (c & 15); };
  auto valid = [&](int c) { return (c & 15) < gsz && cand(c) < b; };
  const int stride = kd.stride;
  KD_T0();
  // The sample's 16-group chunks are dealt to the nsplit workgroups (and within one to its W
  // waves) round-robin when ilv is set: the kd order keeps a candidate's dominated cells in
  // neighbouring chunks, so contiguous ranges would leave most of a sample's terms to one or
  // two of its splits.  Workgroup-local chunk ql is the sample's chunk q0 + ql * qstep.
  const int split = blockIdx.z;
  const int Gsamp = kd.goff[s + 1] - kd.goff[s];
  const int NQall = (Gsamp + 15) >> 4;
  int q0, NQ, qstep;
  if (ilv) {
    q0 = split;
    qstep = nsplit;
    NQ = split < NQall ? (NQall - split + nsplit - 1) / nsplit : 0;
  } else {
    const int qper = (NQall + nsplit - 1) / nsplit;
    q0 = min(NQall, split * qper);
    qstep = 1;
    NQ = min(NQall, q0 + qper) - q0;                         // this workgroup's 16-group chunks
  }
  auto qgl = [&](int ql) { return q0 + ql * qstep; };       // workgroup-local -> sample chunk
  auto gend_of = [&](int ql) { return min(16, Gsamp - 16 * qgl(ql)); };
  int qw0 = 0, NQw = NQ, qwst = 1;                           // this wave's share (set below)
  const int gbase = kd.goff[s];
  // groups of this workgroup's chunks (the sample's last chunk may be short)
  const int Gs = 16 * NQ - ((NQ > 0 && qgl(NQ - 1) == NQall - 1) ? 16 * NQall - Gsamp : 0);
  const Kd2Lds Lo = kd2_lds(stride, M, kd.max_groups);
  double* pt = (double*)(kd_dyn + Lo.pt);
  unsigned short* mA = (unsigned short*)(kd_dyn + Lo.mA);
  unsigned short* pA = (unsigned short*)(kd_dyn + Lo.pA) + wave * (CW * NQ + 1);   // this wave's prefixes
  const uint4* gmin = (const uint4*)kd.gbox + gbase;   // group minimum corners
  uint4* gb = (uint4*)(kd_dyn + Lo.gb);                 // ... and their LDS copy

  kd_stage(pt, kd.pts + (size_t)s * stride * M, stride * M);
  // group minima into LDS and, from the same registers, each chunk's minimum corner by a
  // 16-lane xor-shuffle reduction (a chunk's 16 groups sit in 16 consecutive lanes): one
  // round of independent loads instead of a 16-step dependent loop per chunk
  for (int e = tid; e < 16 * NQ; e += 256) {
    const int q = e >> 4, g = 16 * qgl(q) + (e & 15);
    uint4 v = make_uint4(~0u, ~0u, ~0u, ~0u);   // identity of the packed u16 minimum
    if (g < Gsamp) {
      v = gmin[g];
      gb[e] = v;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      v.x = pk_min_u16(v.x, (unsigned int)__shfl_xor((int)v.x, o, 64));
      v.y = pk_min_u16(v.y, (unsigned int)__shfl_xor((int)v.y, o, 64));
      v.z = pk_min_u16(v.z, (unsigned int)__shfl_xor((int)v.z, o, 64));
      v.w = pk_min_u16(v.w, (unsigned int)__shfl_xor((int)v.w, o, 64));
    }
    if ((e & 15) == 0) cmin[q] = v;
  }
  for (int e = tid; e < KD_CT * M; e += 256) {
    const int j = e / KD_CT, c = e - j * KD_CT;
    yv[c][j] = valid(c) ? G[((size_t)s * M + j) * b + cand(c)] : -INFINITY;
  }
  if (tid < KD_CT) {
    const bool in = valid(tid);
    unsigned int w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      unsigned int v = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * q + h;
        const unsigned int t = (j < M) ? (in ? (unsigned int)thg[((size_t)s * M + j) * b + cand(tid)] : 0u) : 1u;
        v |= t << (16 * h);
      }
      w[q] = v;
    }
    thp[tid] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (int e = tid; e < KD_CT * NV; e += 256) (&acc[0][0])[e] = 0.0;
  __syncthreads();
  KD_T(0);
  KD_WSTAMP(kd_wst);
  const int wsub = wave % W;
  const int cbase = (wave / W) * CW;   // this wave's candidates: cbase .. cbase + 15 (tile-local)
  const int aslot = wave * CW;         // ... and its accumulator rows
  if (!valid(cbase)) return;
  if (ilv) {   // this wave's share of the workgroup's chunks: local chunk qw0 + k * qwst
    qw0 = wsub;
    qwst = W;
    NQw = wsub < NQ ? (NQ - wsub + W - 1) / W : 0;
  } else {
    const int qpw = (NQ + W - 1) / W;
    const int qa = min(NQ, wsub * qpw);
    qw0 = qa;
    NQw = min(NQ, qa + qpw) - qa;
  }
  const int NE = CW * NQw;

  // ---- A: chunk pre-filter (lane = (chunk, candidate) entry), ballot compaction of the
  //      surviving entries, then their 16 group tests lane-dense ----
  {
    unsigned short* ent = pA;   // entry list (pA is rewritten by the prefix)
    int nent = 0;
    for (int eb = 0; eb < NE; eb += 64) {
      const int e = eb + lane, q = qw0 + (e >> 4) * qwst, cl = e & 15;
      bool pass = false;
      if (e < NE) {
        mA[q * KD_CT + cbase + cl] = 0;
        pass = kd_pass4(cmin[q], thp[cbase + cl]);
      }
      const unsigned long long bal = __ballot(pass);
      if (pass) ent[nent + __popcll(bal & ((1ull << lane) - 1ull))] = (unsigned short)e;
      nent += __popcll(bal);
    }
    wave_sync();
    for (int i = lane; i < nent; i += 64) {
      const int e = ent[i], q = qw0 + (e >> 4) * qwst, cl = e & 15;
      const uint4 t = thp[cbase + cl];
      const int gend = gend_of(q);
      unsigned int mask = 0;
      for (int k = 0; k < gend; ++k) mask |= (unsigned int)kd_pass4(gb[q * 16 + k], t) << k;
      mA[q * KD_CT + cbase + cl] = (unsigned short)mask;
    }
    if (EVR_KD_PROF != 2 && kd.counters && lane == 0) atomicAdd(kd.counters + 3, (unsigned long long)nent);
  }
  wave_sync();
  // candidate-major prefix over the entries e = cl * NQw + q (a candidate's pairs contiguous);
  // each lane keeps the prefixes of its <= 8 entries in registers for the window marks
  const int per = (NE + 63) >> 6;                             // <= 8 (NQ <= KD_MAX_NQ)
  const int e0 = min(NE, lane * per), e1 = min(NE, e0 + per);
  // e / NQ = (e * magic) >> 16, exact for e <= 16 * KD_MAX_NQ
  const unsigned int nq_magic = NQw > 0 ? (65536u + (unsigned int)NQw - 1u) / (unsigned int)NQw : 0u;
  int PA;
  int preE[9];
  {
    int cl = (int)(((unsigned int)e0 * nq_magic) >> 16), q = e0 - cl * NQw;
    int cnt[8];
    int loc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cnt[k] = 0;
      if (e0 + k < e1) {
        cnt[k] = __popc(mA[(qw0 + q * qwst) * KD_CT + cbase + cl]);
        if (++q == NQw) q = 0, ++cl;
      }
      loc += cnt[k];
    }
    int run = wave_scan_excl(loc, &PA);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      preE[k] = run;
      if (e0 + k < e1) pA[e0 + k] = (unsigned short)run;
      run += cnt[k];
    }
    preE[8] = run;
    if (lane == 0) {
      pA[NE] = (unsigned short)PA;
      if (EVR_KD_PROF != 2 && kd.counters) {
        atomicAdd(kd.counters + 0, (unsigned long long)PA);
        atomicAdd(kd.counters + 2, (unsigned long long)max(0, min(b - cand(cbase), gsz)) * Gs);
      }
    }
  }
  wave_sync();
  KD_T(1);
  KD_WSTAMP(kd_wpf);
  if (EVR_KD_PROF == 2) kd_np = PA;

  int* mb = mk[wave];
  int* mc = mb;   // the evaluation reuses the row once the cell filter has read it
  int carryB = -1;
  for (int wb = 0; wb < PA; wb += 64) {
    // ---- B: pair -> entry by marks, then the cell filter (lane = passing pair) ----
    mb[lane] = -1;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (preE[k + 1] > preE[k] && preE[k] >= wb && preE[k] < wb + 64) mb[preE[k] - wb] = e0 + k;
    wave_sync();
    const int ownB = max(wave_max_incl(mb[lane]), carryB);
    carryB = __builtin_amdgcn_readlane(ownB, 63);
    const int p = wb + lane;
    unsigned int mB = 0;
    int cg = 0;
    if (p < PA) {
      const int cl = (int)(((unsigned int)ownB * nq_magic) >> 16), q = qw0 + (ownB - cl * NQw) * qwst;
      const int c = cbase + cl;
      const int g = 16 * qgl(q) + kth_bit16(mA[q * KD_CT + c], p - pA[ownB]);   // the sample's group
      const uint4* rp = (const uint4*)(kd.grk + (size_t)(gbase + g) * M * 16);
      const uint4 tq = thp[c];
      const unsigned int tw[4] = {tq.x, tq.y, tq.z, tq.w};
      unsigned int a[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = 0xFFFFFFFFu;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const unsigned int th16 = (tw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
        const unsigned int tt = th16 | (th16 << 16);
        const uint4 r1 = rp[2 * j], r2 = rp[2 * j + 1];
        a[0] &= kd_lt16(r1.x, tt);
        a[1] &= kd_lt16(r1.y, tt);
        a[2] &= kd_lt16(r1.z, tt);
        a[3] &= kd_lt16(r1.w, tt);
        a[4] &= kd_lt16(r2.x, tt);
        a[5] &= kd_lt16(r2.y, tt);
        a[6] &= kd_lt16(r2.z, tt);
        a[7] &= kd_lt16(r2.w, tt);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) mB |= (((a[i] >> 15) & 1u) | ((a[i] >> 30) & 2u)) << (2 * i);
      cg = (c << 16) | g;
    }
    const int cntB = __popc(mB);
    int EW;
    const int pre = wave_scan_excl(cntB, &EW);
    KD_T(2);
    if (EVR_KD_PROF == 2) kd_nt += EW;
    if (EVR_KD_PROF != 2 && kd.counters && lane == 0) atomicAdd(kd.counters + 1, (unsigned long long)EW);
    // ---- C: term -> pair by marks (software-pipelined: the next round's owner and key
    //      load are issued before the current round is evaluated) ----
    int carryC = -1;
    auto locate = [&](int cb, int& c, unsigned long long& key) {
      mc[lane] = -1;
      if (cntB > 0 && pre >= cb && pre < cb + 64) mc[pre - cb] = lane;
      wave_sync();
      const int o = max(wave_max_incl(mc[lane]), carryC);
      carryC = __builtin_amdgcn_readlane(o, 63);
      const int cgo = __shfl(cg, o, 64);
      const int mo = __shfl((int)mB, o, 64);
      const int po = __shfl(pre, o, 64);
      wave_sync();
      // the key load is issued by every lane (past the end: the sample's first key), so each
      // locate issues exactly one load and the compiler can count them across rounds
      const bool in = cb + lane < EW;
      c = in ? (cgo >> 16) : -1;
      const size_t kidx = in ? (size_t)(gbase + (cgo & 0xFFFF)) * 16 + kth_bit16((unsigned int)mo, cb + lane - po)
                             : (size_t)gbase * 16;
      key = kd.gkeys[kidx];
    };
    // Rounds alternate between two (owner, key) buffers: round r + 2's owner and key load are
    // issued into the buffer round r has just consumed, so the load is in flight while round
    // r + 1 is evaluated.  (A buffer copied from a register with a load in flight would make
    // the compiler wait for that load at the loop head.)
    auto term_round = [&](const int c, const unsigned long long key) {
      int rcv = -1;
      double val[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) val[v] = 0.0;
      if (c >= 0) {
        double l[M], u[M];
        K::decode_direct(key, pt, l, u);
        double y[M];
#pragma unroll
        for (int j = 0; j < M; ++j) y[j] = yv[c][j];
        if (!BWD) {
          double prod = fmax(fmin(y[0], u[0]) - l[0], 0.0);
#pragma unroll
          for (int j = 1; j < M; ++j) prod *= fmax(fmin(y[j], u[j]) - l[j], 0.0);
          val[0] = prod;
        } else {
          double len[M], pass[M];
#pragma unroll
          for (int j = 0; j < M; ++j) {
            const double raw = fmin(y[j], u[j]) - l[j];
            len[j] = fmax(raw, 0.0);
            const double dmin = (y[j] < u[j]) ? 1.0 : ((y[j] == u[j]) ? 0.5 : 0.0);
            pass[j] = (raw >= 0.0) ? dmin : 0.0;
          }
          double pre_[M];
          pre_[0] = 1.0;
#pragma unroll
          for (int j = 1; j < M; ++j) pre_[j] = pre_[j - 1] * len[j - 1];
          val[0] = pre_[M - 1] * len[M - 1];
          double suf = 1.0;
#pragma unroll
          for (int j = M - 1; j >= 0; --j) {
            val[NV > 1 ? 1 + j : 0] = pass[j] * pre_[j] * suf;
            suf *= len[j];
          }
        }
        rcv = c;
      }
      KD_T(3);
      seg_scan_wave_x<NV>(rcv >= 0 ? rcv : -3 - lane, val);
      const int rnext = __shfl_down(rcv, 1, 64);
      if (rcv >= 0 && (lane == 63 || rnext != rcv)) {
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[rcv - cbase + aslot][v] += val[v];
      }
      KD_T(4);
    };
    // Every path through the loop issues the same loads in the same order (locates past the
    // end are dummies), so the wait before a round's first key use counts only its own load.
    if (EW > 0) {
      int cA = -1, cB = -1;
      unsigned long long kA = 0, kB = 0;
      locate(0, cA, kA);
      locate(64, cB, kB);
      for (int cb = 0; cb < EW; cb += 128) {
        term_round(cA, kA);
        locate(cb + 128, cA, kA);
        if (cb + 64 < EW) term_round(cB, kB);
        locate(cb + 192, cB, kB);
      }
    }
    wave_sync();   // mb / mc are rewritten by the next window
  }
  wave_sync();
  KD_TEND();
  const int nst = nsplit * W;   // partial splits: workgroup splits x wave splits
  const size_t ss = ((size_t)s * nsplit + split) * W + wsub;
  if (lane < CW && valid(cbase + lane)) part[ss * b + cand(cbase + lane)] = acc[aslot + lane][0];
  if (BWD) {
    for (int e = lane; e < CW * M; e += 64) {
      const int j = e / CW, cl = e - j * CW, c = cbase + cl;
      if (!valid(c)) continue;
      const int gc = cand(c);
      const double v = acc[aslot + cl][NV > 1 ? 1 + j : 0];
      if (nst == 1) dG[((size_t)s * M + j) * b + gc] = (gout ? gout[gc] : 1.0) / (double)S * v;
      else dG[(ss * M + j) * b + gc] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// hvi_kdw — the restart-batch scan with one wave per (sample, candidate) and nothing shared
// between the waves but the sample's point table (staged in LDS once per workgroup of
// KW_WAVES candidates).  Per wave:
//   y_j of the candidate (G, or the sampling step fused in: KbSamples);
//   thresholds t_j = #{rows with lower-bound value <= y_j} by two wave-wide probes of the
//     sample's ascending values (64 bucket ends, then the 64 entries of the straddling
//     bucket) instead of a 9-step binary search;
//   the sample's groups, 64 per chunk and 8 chunks in flight: group tests; the passing groups
//     compacted in group order; their 16 cell tests (the group's rank rows), one group per
//     lane -> cell masks; the passing cells' key indices appended to the wave's term list in
//     (group, cell) order by a wave scan;
//   terms in rounds of 64, term t of the candidate on lane t % 64: key decoded against the
//     LDS point table, the term and its subgradients (hvi_kdb's arithmetic) summed per lane
//     in t order; then one fixed xor-butterfly per value.
// No workgroup barrier after the staging and no inter-wave order: a candidate's value and
// gradient depend on its own term sequence only, so they are bitwise the same in any batch
// (a restart batch sharded over ranks evaluates each candidate exactly as one rank does) and
// bitwise reproducible.  Equal to hvi_kdb to rounding (different summation order).
// Workgroup w runs on XCD w % 8: the candidate groups of a sample share one XCD's L2.
// ---------------------------------------------------------------------------------------
constexpr int KW_WAVES = 4;
constexpr int KW_NCH = 8;               // 64-group chunks whose group / cell tests are in flight together
constexpr int KW_TCAP = 64 * 16 + 64;   // one 64-group chunk's terms + a partial round
constexpr int KW_MAXG = 4096;           // groups per sample: term entries (16 g + cell) fit u16

__host__ __device__ inline size_t kw_pt_bytes(int stride, int M) { return ((size_t)stride * M * 8 + 15) & ~(size_t)15; }
// point table | per-wave term lists (u16 cell index within the sample) | per-wave passing-group
// lists (u16): ~24 KB at the bench state, so LDS admits 6 workgroups per CU
__host__ __device__ inline size_t kw_lds_bytes(int stride, int M) {
  return kw_pt_bytes(stride, M) + (size_t)KW_WAVES * KW_TCAP * 2 + (size_t)KW_WAVES * 64 * KW_NCH * 2;
}

// (256, 5): 5 waves per SIMD — at b = 20 the grid (S x 5 candidate groups = 1280 workgroups at
// S = 256) is resident in one round; unbounded the compiler took 100 VGPRs (4 per SIMD).
// M = 8 would spill at that bound and keeps 4.
template <int M>
__global__ __launch_bounds__(256, M <= 7 ? 5 : 4) void hvi_kdw(int b, int S, int ncg, const double* __restrict__ G, HviKd kd,
                                               KbSamples smp, double* __restrict__ sval, double* __restrict__ dG) {
  constexpr int NV = M + 1;
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kw_dyn[];
  const int wid = blockIdx.x, xcd = wid & 7, slot = wid >> 3;
  const int s = (slot / ncg) * 8 + xcd, cg = slot - (slot / ncg) * ncg;
  if (s >= S) return;   // the grid covers S rounded up to 8 samples: whole workgroups leave
  // the wave index (hence the candidate c) is wave-uniform: scalar registers, not a VGPR
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int stride = kd.stride;
  double* pt = (double*)kw_dyn;
  unsigned short* tl = (unsigned short*)(kw_dyn + kw_pt_bytes(stride, M)) + (size_t)wave * KW_TCAP;
  unsigned short* pl = (unsigned short*)(kw_dyn + kw_pt_bytes(stride, M) + (size_t)KW_WAVES * KW_TCAP * 2) +
                       (size_t)wave * 64 * KW_NCH;
  const int c = cg * KW_WAVES + wave;
  const bool cin = c < b;
  // EVR_KD_PROF=2 build: per (sample, candidate) wall-clock stamps (s_memrealtime, 10 ns):
  // start, after staging, after the thresholds, time in the group / cell phases, time in the
  // term rounds, end; term and passing-group counts (tools/kdw_waves.py)
  unsigned long long pf_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (EVR_KD_PROF == 2) pf_[0] = wall_clock64();
  // Every load that depends only on (sample, candidate) is issued before the staging barrier,
  // so the dependent chain after it starts at the threshold probes: the sampling step's inputs
  // (partial norms split over lanes: lane 8 j + 4 cls + k sums chain k of class cls of output
  // j, qn_norm_chain's order).  (Holding the thresholds' first probe or the first block's group
  // minima across the barrier as well spilled registers at the 5-waves bound.)
  const int gbase = kd.goff[s], Gs = kd.goff[s + 1] - gbase;
  const uint4* gmin = (const uint4*)kd.gbox + gbase;
  const double* tv = kd.sv + (size_t)s * M * stride;
  const int B1 = (stride + 63) >> 6;
  double yl = 0.0, part = 0.0;
  double hv = 0.0, zv = 0.0, am = 0.0;
  if (cin && smp.R) {
    const long long Rr = (long long)smp.n + smp.nb + smp.nh + 1;
    if (lane < 8 * M) {
      const int j = lane >> 3, cls = (lane >> 2) & 1, k = lane & 3;
      part = qn_norm_chain(smp.P + (size_t)j * smp.nrt * 2 * b, smp.nrt_used, b, c, cls, k);
    }
    if (lane < M) {
      const double* Rj = smp.R + (size_t)lane * Rr * b;
      hv = smp.nh ? Rj[(size_t)(smp.n + smp.nb + s) * b + c] : 0.0;
      zv = smp.zq[(size_t)s * M + lane];
      am = Rj[(size_t)(Rr - 1) * b + c];
    }
  } else if (cin && lane < M) {
    yl = G[((size_t)s * M + lane) * b + c];
  }
  {
    // the point table: a thread's loads all in flight before its LDS stores (a load -> store
    // loop waits on every load in turn)
    const double* src = kd.pts + (size_t)s * stride * M;
    const int ne = stride * M;
    for (int e0 = 0; e0 < ne; e0 += 8 * 256) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 256 + tid;
        v[u] = e < ne ? src[e] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 256 + tid;
        if (e < ne) pt[e] = v[u];
      }
    }
  }
  __syncthreads();
  if (!cin) return;
  if (EVR_KD_PROF == 2) pf_[1] = wall_clock64();
  // the thresholds' first probe (bucket ends) overlaps the sampling step below
  double v1[M];
  {
    const int i1 = min((lane + 1) * B1, stride) - 1;
#pragma unroll
    for (int j = 0; j < M; ++j) v1[j] = tv[(size_t)j * stride + i1];
  }

  // ---- y_j (lane j < M), then to every lane ----
  if (smp.R) {
    const int q = lane & ~3;   // the four chains of this lane's (output, class), fixed order
    const double tot = (__shfl(part, q, 64) + __shfl(part, q + 1, 64)) + (__shfl(part, q + 2, 64) + __shfl(part, q + 3, 64));
    const double ssv = __shfl(tot, 8 * (lane & 7), 64), ssw = __shfl(tot, 8 * (lane & 7) + 4, 64);
    if (lane < M) {
      const int j = lane;
      double mu, l22;
      int flag;
      qn_mu_l22_from(ssv, ssw, am, smp.ys[j], smp.cc[j], smp.ym[j], smp.kxx[j], mu, l22, flag);
      if (s == 0) {
        smp.L22[(size_t)j * b + c] = l22;
        smp.flags[(size_t)j * b + c] = flag;
      }
      yl = qn_sample_obj(mu, hv, smp.nh != 0, l22, zv, smp.oa[j], smp.ob[j]);
    }
  }
  double y[M];
#pragma unroll
  for (int j = 0; j < M; ++j) y[j] = __shfl(yl, j, 64);

  // ---- thresholds: two wave-wide probes per objective ----
  unsigned int tw[4] = {0x00010001u, 0x00010001u, 0x00010001u, 0x00010001u};   // t = 1 beyond M (as kdb)
  {
    int base[M];
#pragma unroll
    for (int j = 0; j < M; ++j) base[j] = min(__popcll(__ballot(v1[j] <= y[j])) * B1, stride);
    double v2[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int i2 = base[j] + lane;
      v2[j] = (lane < B1 && i2 < stride) ? tv[(size_t)j * stride + i2] : INFINITY;
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const unsigned int t = (unsigned int)(base[j] + __popcll(__ballot(lane < B1 && v2[j] <= y[j])));
      const int sh = 16 * (j & 1);
      tw[j >> 1] = (tw[j >> 1] & ~(0xFFFFu << sh)) | (t << sh);
    }
  }
  const uint4 tt = make_uint4(tw[0], tw[1], tw[2], tw[3]);
  if (EVR_KD_PROF == 2) pf_[2] = wall_clock64();

  // ---- the sample's groups in blocks of KW_NCH chunks of 64 (lane = group of a chunk):
  //      A. every chunk's group test, all minima loads in flight together; B. the passing
  //      groups compacted in group order; C. rounds of 64 passing groups, one per lane (rank
  //      rows loaded together): cell masks, the passing cells' key indices appended to the
  //      term list in (group, cell) order, full rounds of 64 terms evaluated as they fill ----
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
  auto term_add = [&](const unsigned long long key) {
    double l[M], u[M];
    K::decode_direct(key, pt, l, u);
    double len[M], pass[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const double raw = fmin(y[j], u[j]) - l[j];
      len[j] = fmax(raw, 0.0);
      const double dmin = (y[j] < u[j]) ? 1.0 : ((y[j] == u[j]) ? 0.5 : 0.0);
      pass[j] = (raw >= 0.0) ? dmin : 0.0;
    }
    double pre_[M];
    pre_[0] = 1.0;
#pragma unroll
    for (int j = 1; j < M; ++j) pre_[j] = pre_[j - 1] * len[j - 1];
    acc[0] += pre_[M - 1] * len[M - 1];
    double suf = 1.0;
#pragma unroll
    for (int j = M - 1; j >= 0; --j) {
      acc[1 + j] += pass[j] * pre_[j] * suf;
      suf *= len[j];
    }
  };
  // evaluate terms [0, nr * 64) of the list (nr full rounds) or, with part, one partial round
  auto rounds = [&](const int nr, const int part) {
    const int last = part > 0 ? nr : nr - 1;   // index of the final round
    if (last < 0) return;
    // every round issues exactly one, unconditional key load (lanes past the list read the
    // sample's first key; the last round reloads its own), so the wait before a round's terms
    // counts only that round's load (vmcnt(1)) and the next round's load stays in flight —
    // a conditional load merges at the loop head and forces vmcnt(0)
    auto ld = [&](const int r) -> unsigned long long {
      const int t = r * 64 + lane;
      const bool in = r < nr || lane < part;
      const unsigned int ix = in ? (unsigned int)tl[t] : 0u;
      return kd.gkeys[(size_t)gbase * 16 + ix];
    };
    unsigned long long kc = ld(0);
    for (int r = 0; r <= last; ++r) {
      const unsigned long long kn = ld(min(r + 1, last));
      __asm__ volatile("" ::: "memory");   // keep the next key's load issued before this round's terms
      if (r < nr || lane < part) term_add(kc);
      kc = kn;
    }
  };
  // the cell mask (16 bits) of group g for this candidate: rank_j < t_j in every objective
  auto cell_mask = [&](const int g) -> unsigned int {
    const uint4* rp = (const uint4*)(kd.grk + (size_t)(gbase + g) * M * 16);
    unsigned int a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const unsigned int th16 = (tw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      const unsigned int t2 = th16 | (th16 << 16);
      const uint4 r1 = rp[2 * j], r2 = rp[2 * j + 1];
      a[0] &= kd_lt16(r1.x, t2);
      a[1] &= kd_lt16(r1.y, t2);
      a[2] &= kd_lt16(r1.z, t2);
      a[3] &= kd_lt16(r1.w, t2);
      a[4] &= kd_lt16(r2.x, t2);
      a[5] &= kd_lt16(r2.y, t2);
      a[6] &= kd_lt16(r2.z, t2);
      a[7] &= kd_lt16(r2.w, t2);
    }
    unsigned int mB = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) mB |= (((a[k] >> 15) & 1u) | ((a[k] >> 30) & 2u)) << (2 * k);
    return mB;
  };
  int tn = 0;   // terms in the list (wave-uniform)
  unsigned long long pf_mark = EVR_KD_PROF == 2 ? wall_clock64() : 0;
  for (int G0 = 0; G0 < Gs; G0 += 64 * KW_NCH) {
    const int nch = min(KW_NCH, (Gs - G0 + 63) >> 6);
    // A. group tests of up to KW_NCH chunks: one minima load per chunk and lane, all in flight
    uint4 gm[KW_NCH];
#pragma unroll
    for (int k = 0; k < KW_NCH; ++k) {
      const int g = G0 + 64 * k + lane;
      // past the sample's groups: 0x7FFF ranks (cells_kd's padding), which fail the packed
      // signed compare (0xFFFF would read as -1 and pass)
      gm[k] = (k < nch && g < Gs) ? gmin[g] : make_uint4(0x7FFF7FFFu, 0x7FFF7FFFu, 0x7FFF7FFFu, 0x7FFF7FFFu);
    }
    // B. the passing groups, compacted in group order (chunk-major, lane order within a chunk)
    int np_ = 0;
#pragma unroll
    for (int k = 0; k < KW_NCH; ++k) {
      const unsigned long long bal = __ballot(kd_pass4(gm[k], tt));
      if (bal >> lane & 1ull) pl[np_ + __popcll(bal & ((1ull << lane) - 1ull))] = (unsigned short)(64 * k + lane);
      np_ += __popcll(bal);
    }
    if (EVR_KD_PROF == 2) pf_[7] += np_;
    wave_sync();
    // C. pair rounds of 64, one passing group per lane (its rank rows loaded together): cell
    //    masks -> the cells' key indices appended in (group, cell) order, term rounds as they fill
    for (int p0 = 0; p0 < np_; p0 += 64) {
      const int i = p0 + lane;
      const int g = i < np_ ? G0 + (int)pl[i] : -1;
      const unsigned int mB = g >= 0 ? cell_mask(g) : 0u;
      int tot;
      int p = tn + wave_scan_excl(__popc(mB), &tot);
      if (tot == 0) continue;
      const unsigned int kb = (unsigned int)g * 16u;   // within the sample (< KW_MAXG x 16)
      unsigned int mk = mB;
      while (mk) {
        const int c16 = __ffs(mk) - 1;
        mk &= mk - 1;
        tl[p++] = (unsigned short)(kb + (unsigned int)c16);
      }
      tn += tot;
      wave_sync();
      const int nr = tn >> 6;
      if (nr > 0) {
        if (EVR_KD_PROF == 2) {
          const unsigned long long t = wall_clock64();
          pf_[3] += t - pf_mark;
          pf_mark = t;
          pf_[6] += 64ull * nr;
        }
        rounds(nr, 0);
        if (EVR_KD_PROF == 2) {
          const unsigned long long t = wall_clock64();
          pf_[4] += t - pf_mark;
          pf_mark = t;
        }
        const int rem = tn - nr * 64;
        const unsigned short keep = lane < rem ? tl[nr * 64 + lane] : (unsigned short)0;
        wave_sync();
        if (lane < rem) tl[lane] = keep;
        wave_sync();
        tn = rem;
      }
    }
    wave_sync();   // pl is rewritten by the next block of chunks
  }
  if (EVR_KD_PROF == 2) {
    const unsigned long long t = wall_clock64();
    pf_[3] += t - pf_mark;
    pf_mark = t;
    pf_[6] += tn;
  }
  rounds(0, tn);
  if (EVR_KD_PROF == 2) pf_[4] += wall_clock64() - pf_mark;
  // ---- per value the lanes' sums, fixed butterfly ----
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double x = acc[v];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    acc[v] = x;
  }
  if (lane == 0) {
    sval[(size_t)s * b + c] = acc[0];
#pragma unroll
    for (int j = 0; j < M; ++j) dG[((size_t)s * M + j) * b + c] = 1.0 / (double)S * acc[1 + j];
  }
  if (EVR_KD_PROF == 2 && kd.counters && lane == 0) {
    pf_[5] = wall_clock64();
    unsigned long long* r = kd.counters + 16 + 8 * ((size_t)s * b + c);
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = pf_[q];
  }
}

struct HviPlan {
  int tgb, bb, ctiles, nchunk, cb;
};

// Candidate-group width: fewest (padded candidate slots + per-tile cell staging) per cell;
// chunks so that ~2048 workgroups fill the chip.
constexpr int HVI_TARGET_BLOCKS = 2048;

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
  const int want = (int)((HVI_TARGET_BLOCKS + base - 1) / base);
  const int maxchunks = (maxc + sub - 1) / sub;
  p.nchunk = std::max(1, std::min(want, maxchunks));
  int cb = (maxc + p.nchunk - 1) / p.nchunk;
  cb = ((cb + sub - 1) / sub) * sub;
  p.cb = cb;
  p.nchunk = (maxc + cb - 1) / cb;
  return p;
}

static HviKd hvi_kd_of(const evr_qnehvi_state* st) {
  return HviKd{st->grp_off, st->grp_keys, st->grp_rank, st->grp_box, st->sorted_lo, st->cell_pts, st->cell_rank0,
               st->pts_stride, st->max_groups, st->scan_counters};
}

// waves sharing one 16-candidate group in hvi_kd2 (chunks split between them): the
// restart batches (b <= 32) would leave 2-3 of the 4 waves idle otherwise
static int hvi_kd_wsplit(int b) {
  return b <= 16 ? 4 : (b <= 32 ? 2 : 1);
}

// group-range splits per sample: fill ~1024 workgroups at small candidate batches
static int hvi_kd_nsplit(const evr_qnehvi_state* st, int b) {
  const int tiles = cdiv(b, KD_CT / hvi_kd_wsplit(b)) * st->S;
  const int nq = (st->max_groups + 15) / 16;
  // ~1024 workgroups (more, smaller splits measured slower: profiles/r02/g/kd_wgs_*.json)
  constexpr int wgs = 1024;
  return std::max(1, std::min(std::min(cdiv(wgs, tiles), 16), std::max(nq, 1)));
}

// workspace (doubles): S x ns x b partials | S x M x b int thresholds | (ns > 1) S x ns x M x b dG
// partials, ns counting workgroup x wave splits
static long long hvi_kd_workspace(const evr_qnehvi_state* st, int b) {
  const long long ns = (long long)hvi_kd_nsplit(st, b) * hvi_kd_wsplit(b);
  return (long long)st->S * ns * b + ((long long)st->S * st->m * b + 1) / 2 +
         (ns > 1 ? (long long)st->S * ns * st->m * b : 0);
}

template <int M, bool BWD>
static int hvi_kd_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, const double* gout,
                         double* part, double* dG, const int* flags, double* acq) {
  const int W = hvi_kd_wsplit(b);
  const int ntiles = cdiv(b, KD_CT / W);
  const int nsb = hvi_kd_nsplit(st, b);   // workgroup splits
  const int ns = nsb * W;                 // partial splits (workgroup x wave)
  int* th = (int*)(part + (size_t)st->S * ns * b);   // workspace: thresholds, then dG partials
  double* dgp = (double*)(th + (((size_t)st->S * M * b + 1) & ~(size_t)1));
  hvi_thresholds<<<dim3(M, st->S), 256, (size_t)st->pts_stride * sizeof(double), s>>>(b, M, st->pts_stride, G,
                                                                                     st->sorted_lo, th);
  EVR_LAUNCH_CHECK();
  dim3 grid(ntiles, st->S, nsb);
  EVR_CHECK((st->max_groups + 15) / 16 <= KD_MAX_NQ, "hvi: %d kd groups per sample exceed the scan's %d",
            st->max_groups, 16 * KD_MAX_NQ);
  const Kd2Lds L2 = kd2_lds(st->pts_stride, M, st->max_groups);
  EVR_HIP(hipFuncSetAttribute((const void*)hvi_kd2<M, BWD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)L2.bytes));
  // balanced 16-slot groups; round-robin chunks for the wave-split restart batches (b <= 32),
  // contiguous ranges for larger batches
  hvi_kd2<M, BWD><<<grid, 256, L2.bytes, s>>>(b, st->S, ntiles, nsb, G, th, hvi_kd_of(st), gout, part,
                                                ns > 1 ? dgp : dG, W, 1, W > 1);
  EVR_LAUNCH_CHECK();
  if (acq && BWD && ns > 1) {   // one launch for both reductions
    const long long tot = (long long)st->S * M * b;
    const int nb = (int)cdiv(tot, 256);
    if (b <= 32) {
      const int nf = cdiv(b, 4);
      hvi_reduce_fb<4><<<nf + nb, 256, 0, s>>>(st->S, ns, b, M, nf, part, flags, acq, dgp, gout, dG);
    } else {
      const int nf = cdiv(b, 16);
      hvi_reduce_fb<16><<<nf + nb, 256, 0, s>>>(st->S, ns, b, M, nf, part, flags, acq, dgp, gout, dG);
    }
    EVR_LAUNCH_CHECK();
    return 0;
  }
  if (acq) {
    hvi_reduce_fwd_launch(s, st->S, ns, b, M, part, flags, acq);
    EVR_LAUNCH_CHECK();
  }
  if (BWD && ns > 1) {
    const long long tot = (long long)st->S * M * b;
    hvi_reduce_bwd<<<cdiv(tot, 256), 256, 0, s>>>(st->S, ns, M, b, dgp, gout, dG);
    EVR_LAUNCH_CHECK();
  }
  return 0;
}

static bool hvi_kdw_applies(const evr_qnehvi_state* st, int b) {
  if (!st || st->log_hvi || !st->grp_off || b < 1 || b > 32 || st->m < 1 || st->m > 8 || st->max_groups > KW_MAXG)
    return false;
  // the threshold probe reads 64 bucket ends, then the 64 entries of the straddling bucket:
  // exact for strides up to 64 x 64 rows only
  if (st->pts_stride > 64 * 64) return false;
  return kw_lds_bytes(st->pts_stride, st->m) <= 64 * 1024;
}

template <int M>
static int hvi_kdw_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                          double* dG, const KbSamples& smp) {
  const size_t lds = kw_lds_bytes(st->pts_stride, M);
  const int ncg = cdiv(b, KW_WAVES);
  const int wgs = cdiv(st->S, 8) * 8 * ncg;
  EVR_HIP(hipFuncSetAttribute((const void*)hvi_kdw<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hvi_kdw<M><<<wgs, 256, lds, s>>>(b, st->S, ncg, G, hvi_kd_of(st), smp, sval, dG);
  EVR_LAUNCH_CHECK();
  return 0;
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

long long hvi_log_workspace(const evr_qnehvi_state* st, int b, int backward);
int hvi_log_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                   const double* gout, double* work, double* acq, double* dG, bool backward);

static int hvi_check_state(const evr_qnehvi_state* st) {
  EVR_CHECK(st && st->S >= 1 && st->m >= 1 && st->cell_off, "hvi: bad state");
  if (st->log_hvi) return 0;   // hvi_log_launch checks its own inputs
  EVR_CHECK(st->cell_keys ? (st->cell_pts && st->cell_rank0 && st->pts_stride > 0) : (st->cell_lo && st->cell_hi),
            "hvi: state has neither explicit nor compressed cells");
  EVR_CHECK(!st->cell_keys || (size_t)st->pts_stride * (st->m * 8 + 4) <= 64 * 1024,
            "hvi: point table of %d rows exceeds the LDS budget", st->pts_stride);
  EVR_CHECK(!st->grp_off || (st->cell_keys && st->grp_keys && st->grp_rank && st->grp_box && st->sorted_lo &&
                             st->max_groups >= 0 &&
                             kd_lds(st->pts_stride, st->m, st->max_groups).bytes <= 96 * 1024),
            "hvi: inconsistent kd cell groups (stride %d, %d groups)", st->pts_stride, st->max_groups);
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
  if (st->log_hvi) return hvi_log_workspace(st, b, backward);
  if (st->grp_off) return hvi_kd_workspace(st, b);
  HviPlan p = hvi_plan(st, b);
  return (long long)st->S * p.nchunk * b * (backward ? st->m + 1 : 1);
}

int evr_hvi_forward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                    double* work, double* acq) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(work && acq && G, "evr_hvi_forward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (st->log_hvi) return hvi_log_launch(s, st, b, G, flags, nullptr, work, acq, nullptr, false);
  int rc = 0;
  if (st->grp_off) {
#define L(MM) rc = hvi_kd_launch<MM, false>(s, st, b, G, nullptr, work, nullptr, flags, acq)
    EVR_M_SWITCH(st->m, L);
#undef L
    return rc;
  }
  HviPlan p = hvi_plan(st, b);
#define L(MM) rc = hvi_launch<MM, false>(s, st, b, p, G, work, nullptr)
  EVR_M_SWITCH(st->m, L);
#undef L
  if (rc) return rc;
  hvi_reduce_fwd_launch(s, st->S, p.nchunk, b, st->m, work, flags, acq);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_hvi_forward_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const int* flags,
                             const double* gout, double* work, double* acq, double* dG) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(work && dG && G, "evr_hvi_forward_backward: bad arguments");
  if (b == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (st->log_hvi) return hvi_log_launch(s, st, b, G, flags, gout, work, acq, dG, true);
  if (st->grp_off) {
    int rc = 0;
#define L(MM) rc = hvi_kd_launch<MM, true>(s, st, b, G, gout, work, dG, flags, acq)
    EVR_M_SWITCH(st->m, L);
#undef L
    return rc;
  }
  HviPlan p = hvi_plan(st, b);
  double* wf = work;
  double* wb = work + (size_t)st->S * p.nchunk * b;
  int rc = 0;
#define L(MM) rc = hvi_launch<MM, true>(s, st, b, p, G, wf, wb)
  EVR_M_SWITCH(st->m, L);
#undef L
  if (rc) return rc;
  if (acq) {
    hvi_reduce_fwd_launch(s, st->S, p.nchunk, b, st->m, wf, flags, acq);
    EVR_LAUNCH_CHECK();
  }
  const long long tot = (long long)st->S * st->m * b;
  hvi_reduce_bwd<<<cdiv(tot, 256), 256, 0, s>>>(st->S, p.nchunk, st->m, b, wb, gout, dG);
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_hvi_restart_fb_applies(const evr_qnehvi_state* st, int b) { return hvi_kdw_applies(st, b) ? 1 : 0; }

int evr_hvi_restart_fb(void* stream, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                       double* dG) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(G && sval && dG && hvi_kdw_applies(st, b),
            "evr_hvi_restart_fb: bad arguments or the state / batch is not a kd restart batch (b <= 32)");
  int rc = 0;
  const KbSamples smp{};
#define L(MM) rc = hvi_kdw_launch<MM>((hipStream_t)stream, st, b, G, sval, dG, smp)
  EVR_M_SWITCH(st->m, L);
#undef L
  return rc;
}

}  // extern "C"

namespace evr {
// the restart scan with the sampling step fused into its staging (native plan, b <= 32): R / P
// from the projection, L22 / flags written by sample 0's workgroup
bool hvi_kdb_fused_applies(const evr_qnehvi_state* st, int b) {
  return hvi_kdw_applies(st, b) && st->obj_a && st->obj_b && st->zq;
}

int hvi_kdb_fused(hipStream_t s, const evr_qnehvi_state* st, int b, const double* R, const double* P, int nrt,
                  int nrt_used, double* L22, int* flags, double* sval, double* dG) {
  EVR_CHECK(R && P && L22 && flags && sval && dG && hvi_kdb_fused_applies(st, b), "hvi_kdb_fused: bad arguments");
  KbSamples smp{R, P, st->c, st->ym, st->ys, st->kxx, st->zq, st->obj_a, st->obj_b, L22, flags,
                st->n, st->nb, qn_nh(st), nrt, nrt_used};
  int rc = 0;
#define L(MM) rc = hvi_kdw_launch<MM>(s, st, b, nullptr, sval, dG, smp)
  EVR_M_SWITCH(st->m, L);
#undef L
  return rc;
}
}  // namespace evr

extern "C" {

int evr_hvi_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const double* gout,
                     double* work, double* dG) {
  return evr_hvi_forward_backward(stream, st, b, G, nullptr, gout, work, nullptr, dG);
}

}  // extern "C"

namespace evr {

// Per-sample HVI partials for the general evaluation (qnehvi_general.hip): part = work
// (S x nsplit x b, summed over the splits in order gives HVI_s(c)) and, with backward,
// dG = d(sum_s HVI_s)/dG / S (gout = 1).  Linear scans only (log_hvi = 0).
long long hvi_raw_workspace(const evr_qnehvi_state* st, int b, bool backward) {
  if (!st || b <= 0) return 0;
  if (st->grp_off) return hvi_kd_workspace(st, b);
  HviPlan p = hvi_plan(st, b);
  return (long long)st->S * p.nchunk * b * (backward ? st->m + 1 : 1);
}

int hvi_raw(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, bool backward, double* work,
            double* dG, int* nsplit) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(!st->log_hvi && work && G && nsplit && (!backward || dG), "hvi_raw: bad arguments");
  if (b == 0) return 0;
  int rc = 0;
  if (st->grp_off) {
    *nsplit = hvi_kd_nsplit(st, b) * hvi_kd_wsplit(b);
    if (backward) {
#define L(MM) rc = hvi_kd_launch<MM, true>(s, st, b, G, nullptr, work, dG, nullptr, nullptr)
      EVR_M_SWITCH(st->m, L);
#undef L
    } else {
#define L(MM) rc = hvi_kd_launch<MM, false>(s, st, b, G, nullptr, work, nullptr, nullptr, nullptr)
      EVR_M_SWITCH(st->m, L);
#undef L
    }
    return rc;
  }
  HviPlan p = hvi_plan(st, b);
  *nsplit = p.nchunk;
  double* wb = work + (size_t)st->S * p.nchunk * b;
  if (backward) {
#define L(MM) rc = hvi_launch<MM, true>(s, st, b, p, G, work, wb)
    EVR_M_SWITCH(st->m, L);
#undef L
    if (rc) return rc;
    const long long tot = (long long)st->S * st->m * b;
    hvi_reduce_bwd<<<cdiv(tot, 256), 256, 0, s>>>(st->S, p.nchunk, st->m, b, wb, nullptr, dG);
    EVR_LAUNCH_CHECK();
  } else {
#define L(MM) rc = hvi_launch<MM, false>(s, st, b, p, G, work, nullptr)
    EVR_M_SWITCH(st->m, L);
#undef L
  }
  return rc;
}

}  // namespace evr
