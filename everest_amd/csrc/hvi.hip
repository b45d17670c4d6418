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

template <int M, bool BWD>
__global__ __launch_bounds__(256) void hvi_kd(int b, int S, int ntiles, int nsplit, const double* __restrict__ G,
                                              const int* __restrict__ thg, HviKd kd,
                                              const double* __restrict__ gout, double* __restrict__ part,
                                              double* __restrict__ dG) {
  // nsplit > 1 (small candidate batches): the sample's 16-group chunks are split over
  // gridDim.z workgroups; part / dG then receive raw per-split partials
  // [s][split][c] / [s][split][j][c] for hvi_reduce_fwd / hvi_reduce_bwd (fixed order).
  constexpr int NV = BWD ? M + 1 : 1;
  constexpr int CW = KD_CT / 4;            // candidates per wave
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kd_dyn[];
  __shared__ double yv[KD_CT][M];
  __shared__ uint4 thp[KD_CT];             // packed 16-bit thresholds (objectives >= M: 1)
  __shared__ double acc[KD_CT][NV];
  __shared__ int wmask[4][64], wcg[4][64], wpre[4][64];
  // XCD-aware placement: the candidate tiles of one sample share one XCD's L2
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
  const int c0 = tile * KD_CT, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int stride = kd.stride;
  KD_T0();
  const int split = blockIdx.z;
  const int NQall = (kd.goff[s + 1] - kd.goff[s] + 15) >> 4;
  const int qper = (NQall + nsplit - 1) / nsplit;
  const int q0 = min(NQall, split * qper);
  const int NQ = min(NQall, q0 + qper) - q0;                 // this workgroup's 16-group chunks
  const int gbase = kd.goff[s] + 16 * q0;
  const int Gs = min(kd.goff[s + 1] - gbase, 16 * NQ);
  const KdLds Lo = kd_lds(stride, M, kd.max_groups);
  double* pt = (double*)(kd_dyn + Lo.pt);
  int* r0 = (int*)(kd_dyn + Lo.r0);
  uint4* gb = (uint4*)(kd_dyn + Lo.gb);
  unsigned short* mA = (unsigned short*)(kd_dyn + Lo.mA);
  int* pA = (int*)(kd_dyn + Lo.pA) + wave * (CW * NQ + 1);   // this wave's prefix array

  kd_stage(pt, kd.pts + (size_t)s * stride * M, stride * M);
  kd_stage(r0, kd.rank0 + (size_t)s * stride, stride);
  if (Gs > 0) kd_stage(gb, (const uint4*)kd.gbox + gbase, Gs);
  for (int e = tid; e < KD_CT * M; e += 256) {
    const int j = e / KD_CT, c = e - j * KD_CT;
    yv[c][j] = (c0 + c < b) ? G[((size_t)s * M + j) * b + c0 + c] : -INFINITY;
  }
  if (tid < KD_CT) {
    const bool in = c0 + tid < b;
    unsigned int w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      unsigned int v = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * q + h;
        const unsigned int t = (j < M) ? (in ? (unsigned int)thg[((size_t)s * M + j) * b + c0 + tid] : 0u) : 1u;
        v |= t << (16 * h);
      }
      w[q] = v;
    }
    thp[tid] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (int e = tid; e < KD_CT * NV; e += 256) (&acc[0][0])[e] = 0.0;
  __syncthreads();
  KD_T(0);
  const int cbase = wave * CW;   // this wave's candidates: cbase .. cbase + 15 (tile-local)
  if (c0 + cbase >= b) return;

  // ---- A: group filter; lane = (candidate, quarter of the 16-group chunks) ----
  {
    const int cl = lane & (CW - 1), qq = lane >> 4;
    const uint4 t = thp[cbase + cl];
    for (int q = qq; q < NQ; q += 4) {
      unsigned int mask = 0;
      const int gend = min(16, Gs - q * 16);
      for (int k = 0; k < gend; ++k) {
        const uint4 v = gb[q * 16 + k];
        const unsigned int x = kd_lt16(v.x, t.x) & kd_lt16(v.y, t.y) & kd_lt16(v.z, t.z) & kd_lt16(v.w, t.w);
        mask |= (unsigned int)((x & 0x80008000u) == 0x80008000u) << k;
      }
      mA[q * KD_CT + cbase + cl] = (unsigned short)mask;
    }
  }
  wave_sync();
  // candidate-major prefix over this wave's entries e = cl * NQ + q
  const int NE = CW * NQ;
  int PA;
  {
    const int per = (NE + 63) / 64;
    const int e0 = min(NE, lane * per), e1 = min(NE, e0 + per);
    int loc = 0;
    for (int e = e0; e < e1; ++e) loc += __popc(mA[(e % NQ) * KD_CT + cbase + e / NQ]);
    int run = wave_scan_excl(loc, &PA);
    for (int e = e0; e < e1; ++e) {
      pA[e] = run;
      run += __popc(mA[(e % NQ) * KD_CT + cbase + e / NQ]);
    }
    if (lane == 0) {
      pA[NE] = PA;
      if (kd.counters) {
        atomicAdd(kd.counters + 0, (unsigned long long)PA);
        atomicAdd(kd.counters + 2, (unsigned long long)max(0, min(b - c0 - cbase, CW)) * Gs);
      }
    }
  }
  wave_sync();
  KD_T(1);

  int* wm = wmask[wave];
  int* wc = wcg[wave];
  int* wp = wpre[wave];
  for (int wb = 0; wb < PA; wb += 64) {
    // ---- B: cell filter (lane = passing (candidate, group) pair), packed compares ----
    const int p = wb + lane;
    unsigned int mB = 0;
    int cg = 0;
    if (p < PA) {
      int lo = 0, hi = NE - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pA[mid] <= p) lo = mid;
        else hi = mid - 1;
      }
      const int cl = lo / NQ, q = lo - cl * NQ;
      const int c = cbase + cl;
      const int g = q * 16 + kth_bit16(mA[q * KD_CT + c], p - pA[lo]);
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
    int EW;
    const int pre = wave_scan_excl(__popc(mB), &EW);
    KD_T(2);
    wm[lane] = (int)mB;
    wc[lane] = cg;
    wp[lane] = pre;
    if (kd.counters && lane == 0) atomicAdd(kd.counters + 1, (unsigned long long)EW);
    wave_sync();
    // ---- C: evaluation (lane = exact (cell, candidate) term) ----
    // software-pipelined: the next round's term is located and its key load issued before
    // the current round is decoded and evaluated (hides the L2 latency of the key fetch)
    auto locate = [&](int q, int& c, unsigned long long& key) {
      int lo = 0, hi = 63;
      if (EVR_KD_EXP == 2) lo = hi = q & 63;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (wp[mid] <= q) lo = mid;
        else hi = mid - 1;
      }
      c = wc[lo] >> 16;
      const int g = wc[lo] & 0xFFFF;
      const int bit = kth_bit16((unsigned int)wm[lo], q - wp[lo]);
      key = kd.gkeys[(size_t)(gbase + g) * 16 + bit];
    };
    int cnext = -1;
    unsigned long long knext = 0;
    if (lane < EW) locate(lane, cnext, knext);
    for (int cb = 0; cb < EW; cb += 64) {
      const int q = cb + lane;
      const int c = cnext;
      const unsigned long long key = knext;
      cnext = -1;
      if (cb + 64 + lane < EW) locate(cb + 64 + lane, cnext, knext);
      int rcv = -1;
      double val[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) val[v] = 0.0;
      if (q < EW) {
        double l[M], u[M];
        if (EVR_KD_EXP == 1) {
#pragma unroll
          for (int j = 0; j < M; ++j) {
            l[j] = -1.0 + 1e-3 * (double)((key >> (8 * j)) & 0xFF);
            u[j] = l[j] + 0.5;
          }
        } else {
          K::decode_direct(key, pt, l, u);   // grp_keys carry point indices (cells_kd)
        }
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
      // segmented scan over the round (terms of a candidate are contiguous); segment ends
      // add into the candidate's accumulator (owned by this wave)
      seg_scan_wave<NV>(rcv, val);
      const int rnext = __shfl_down(rcv, 1, 64);
      if (rcv >= 0 && (lane == 63 || rnext != rcv)) {
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[rcv][v] += val[v];
      }
      KD_T(4);
    }
    wave_sync();   // wm / wc / wp are rewritten by the next window
  }
  wave_sync();
  // outputs of this wave's candidates
  const size_t ss = (size_t)s * nsplit + split;
  if (lane < CW && c0 + cbase + lane < b) part[ss * b + c0 + cbase + lane] = acc[cbase + lane][0];
  if (BWD) {
    for (int e = lane; e < CW * M; e += 64) {
      const int j = e / CW, cl = e - j * CW, c = cbase + cl;
      if (c0 + c >= b) continue;
      const double v = acc[c][NV > 1 ? 1 + j : 0];
      if (nsplit == 1) dG[((size_t)s * M + j) * b + c0 + c] = (gout ? gout[c0 + c] : 1.0) / (double)S * v;
      else dG[(ss * M + j) * b + c0 + c] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// hvi_kd2 — the same sparse scan as hvi_kd (same groups, cells and terms, same pair and term
// order, same segmented sums: bitwise identical results) with a shorter instruction stream:
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
// hvi_kd3 — the restart-batch (b <= 32) forward + backward scan in ONE launch: one workgroup
// per sample holds the sample's nz <= 4 group-range splits (hvi_kd2's count: 4 at S = 256, 2
// at S = 512) as 256-thread sub-workgroups, each running hvi_kd2's filter / window / term loop on its
// round-robin share of the 16-group chunks.  What the three-launch chain spread over kernels
// is done in LDS:
//   * the thresholds t_j(y_c) (hvi_thresholds) by binary search in the sample's ascending
//     lower bounds, staged once for all splits together with the point table;
//   * the split partials (hvi_reduce_fb's backward half): after one barrier every (candidate,
//     value) sums its splits x wave-split partials in hvi_kd2's partial order, so dG is
//     bitwise the kd2 + reduce_fb result; the per-sample values (sval[s][c]) are left for the
//     dX reduction kernel, which forms acq = mean over samples (qs_dx_reduce).
// ---------------------------------------------------------------------------------------
constexpr int KD3_NZ = 4;   // splits (sub-workgroups) per sample

struct Kd3Lds {
  size_t pt, th, zb, gb, mA, pA, per_z, bytes;
  int nqz;
};
__host__ __device__ inline Kd3Lds kd3_lds(int stride, int M, int max_groups, int nz) {
  Kd3Lds L;
  const int nq = (max_groups + 15) / 16;
  L.nqz = (nq + nz - 1) / nz;   // chunks of one split (round-robin share)
  size_t o = 0;
  L.pt = o;
  o += (size_t)stride * M * 8;
  L.th = o;
  o += (size_t)stride * M * 8;
  o = (o + 15) & ~(size_t)15;
  L.zb = o;
  // per split: group minima (16 per chunk), (chunk, candidate) masks, per-wave u16 prefixes
  L.gb = 0;
  size_t p = (size_t)L.nqz * 16 * 16;
  L.mA = p;
  p += (size_t)L.nqz * KD_CT * 2;
  p = (p + 15) & ~(size_t)15;
  L.pA = p;
  p += ((size_t)KD_CT * L.nqz + 4) * 2;
  L.per_z = (p + 15) & ~(size_t)15;
  L.bytes = o + L.per_z * nz;
  return L;
}

template <int M>
__global__ __launch_bounds__(1024) void hvi_kd3(int b, int S, int nz, const double* __restrict__ G, HviKd kd,
                                                double* __restrict__ sval, double* __restrict__ dG, int W,
                                                int balance) {
  constexpr int NV = M + 1;
  constexpr int CW = KD_CT / 4;   // candidate slots per wave
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kd_dyn[];
  __shared__ double yv[KD_CT][M];
  __shared__ __align__(16) unsigned short ths[KD_CT][8];   // packed thresholds (objectives >= M: 1)
  __shared__ double acc[KD3_NZ][KD_CT][NV];
  __shared__ uint4 cmin[KD3_NZ][KD_MAX_NQ];
  __shared__ int mk[KD3_NZ][4][64];
  const int s = blockIdx.x, tid = threadIdx.x, nth = blockDim.x;   // nth = 256 nz
  const int z = tid >> 8, t = tid & 255, lane = t & 63, wave = t >> 6;
  const int ngr = 4 / W;
  const int gsz = (W > 1 && balance) ? min(CW, (min(KD_CT / W, b) + ngr - 1) / ngr) : CW;
  auto cand = [&](int c) { return (c >> 4) * gsz + (c & 15); };
  auto valid = [&](int c) { return (c & 15) < gsz && cand(c) < b; };
  const int stride = kd.stride;
  const Kd3Lds Lo = kd3_lds(stride, M, kd.max_groups, nz);
  double* pt = (double*)(kd_dyn + Lo.pt);
  double* thv = (double*)(kd_dyn + Lo.th);
  unsigned char* zbase = kd_dyn + Lo.zb + Lo.per_z * z;
  uint4* gb = (uint4*)(zbase + Lo.gb);
  unsigned short* mA = (unsigned short*)(zbase + Lo.mA);
  const int Gsamp = kd.goff[s + 1] - kd.goff[s];
  const int NQall = (Gsamp + 15) >> 4;
  // this split's chunks: the sample's chunk z + ql * nz (round-robin, as hvi_kd2's ilv)
  const bool zin = z < nz;
  const int NQ = (zin && z < NQall) ? (NQall - z + nz - 1) / nz : 0;
  auto qgl = [&](int ql) { return z + ql * nz; };
  auto gend_of = [&](int ql) { return min(16, Gsamp - 16 * qgl(ql)); };
  const int gbase = kd.goff[s];
  const int Gs = 16 * NQ - ((NQ > 0 && qgl(NQ - 1) == NQall - 1) ? 16 * NQall - Gsamp : 0);
  unsigned short* pA = (unsigned short*)(zbase + Lo.pA) + wave * (CW * NQ + 1);
  const uint4* gmin = (const uint4*)kd.gbox + gbase;
  // EVR_KD_PROF=2 build: per-wave wall-clock stamps (s_memrealtime, 100 MHz) — entry, staged,
  // thresholds, filtered + prefixed, terms done, reduced — and the wave's pair / term counts
  unsigned long long st_[6] = {0, 0, 0, 0, 0, 0};
  long long np_ = 0, nt_ = 0;
  if (EVR_KD_PROF == 2) st_[0] = wall_clock64();

  // ---- staging (all splits): point table, ascending lower bounds, candidate values ----
  {
    const double* src = kd.pts + (size_t)s * stride * M;
    const double* srt = kd.sv + (size_t)s * M * stride;
    const int n = stride * M;
    for (int e = tid; e < n; e += nth) {
      const double a = src[e], c = srt[e];
      pt[e] = a;
      thv[e] = c;
    }
  }
  for (int e = t; e < 16 * NQ; e += 256) {
    const int q = e >> 4, g = 16 * qgl(q) + (e & 15);
    uint4 v = make_uint4(~0u, ~0u, ~0u, ~0u);
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
    if ((e & 15) == 0) cmin[z][q] = v;
  }
  for (int e = tid; e < KD_CT * M; e += nth) {
    const int j = e / KD_CT, c = e - j * KD_CT;
    yv[c][j] = valid(c) ? G[((size_t)s * M + j) * b + cand(c)] : -INFINITY;
  }
  for (int e = tid; e < KD3_NZ * KD_CT * NV; e += nth) (&acc[0][0][0])[e] = 0.0;
  __syncthreads();
  if (EVR_KD_PROF == 2) st_[1] = wall_clock64();
  // thresholds: t_j = #{rows with lower-bound value <= y_j} (hvi_thresholds' search)
  if (tid < KD_CT * 8) {
    const int c = tid >> 3, j = tid & 7;
    unsigned short v = 1;
    if (j < M) {
      v = 0;
      if (valid(c)) {
        const double y = yv[c][j];
        const double* tv = thv + (size_t)j * stride;
        int lo = 0, hi = stride;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (tv[mid] <= y) lo = mid + 1;
          else hi = mid;
        }
        v = (unsigned short)lo;
      }
    }
    ths[c][j] = v;
  }
  __syncthreads();
  if (EVR_KD_PROF == 2) st_[2] = st_[3] = st_[4] = wall_clock64();
  const uint4* thp = reinterpret_cast<const uint4*>(&ths[0][0]);
  const int wsub = wave % W;
  const int cbase = (wave / W) * CW;
  const int aslot = wave * CW;
  double (*accz)[NV] = acc[z];
  if (zin && valid(cbase)) {
    const int qw0 = wsub, qwst = W;
    const int NQw = wsub < NQ ? (NQ - wsub + W - 1) / W : 0;
    const int NE = CW * NQw;
    // ---- A: chunk pre-filter, ballot compaction, lane-dense group tests ----
    {
      unsigned short* ent = pA;
      int nent = 0;
      for (int eb = 0; eb < NE; eb += 64) {
        const int e = eb + lane, q = qw0 + (e >> 4) * qwst, cl = e & 15;
        bool pass = false;
        if (e < NE) {
          mA[q * KD_CT + cbase + cl] = 0;
          pass = kd_pass4(cmin[z][q], thp[cbase + cl]);
        }
        const unsigned long long bal = __ballot(pass);
        if (pass) ent[nent + __popcll(bal & ((1ull << lane) - 1ull))] = (unsigned short)e;
        nent += __popcll(bal);
      }
      wave_sync();
      for (int i = lane; i < nent; i += 64) {
        const int e = ent[i], q = qw0 + (e >> 4) * qwst, cl = e & 15;
        const uint4 tt = thp[cbase + cl];
        const int gend = gend_of(q);
        unsigned int mask = 0;
        for (int k = 0; k < gend; ++k) mask |= (unsigned int)kd_pass4(gb[q * 16 + k], tt) << k;
        mA[q * KD_CT + cbase + cl] = (unsigned short)mask;
      }
      if (EVR_KD_PROF != 2 && kd.counters && lane == 0) atomicAdd(kd.counters + 3, (unsigned long long)nent);
    }
    wave_sync();
    const int per = (NE + 63) >> 6;
    const int e0 = min(NE, lane * per), e1 = min(NE, e0 + per);
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
    if (EVR_KD_PROF == 2) {
      st_[3] = wall_clock64();
      np_ = PA;
    }
    int* mb = mk[z][wave];
    int* mc = mb;
    int carryB = -1;
    for (int wb = 0; wb < PA; wb += 64) {
      // ---- B: pair -> entry by marks, cell filter ----
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
        const int g = 16 * qgl(q) + kth_bit16(mA[q * KD_CT + c], p - pA[ownB]);
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
      if (EVR_KD_PROF == 2) nt_ += EW;
      if (EVR_KD_PROF != 2 && kd.counters && lane == 0) atomicAdd(kd.counters + 1, (unsigned long long)EW);
      // ---- C: term -> pair by marks, pipelined key loads, terms, segmented sums ----
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
        const bool in = cb + lane < EW;
        c = in ? (cgo >> 16) : -1;
        const size_t kidx = in ? (size_t)(gbase + (cgo & 0xFFFF)) * 16 + kth_bit16((unsigned int)mo, cb + lane - po)
                               : (size_t)gbase * 16;
        key = kd.gkeys[kidx];
      };
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
            val[1 + j] = pass[j] * pre_[j] * suf;
            suf *= len[j];
          }
          rcv = c;
        }
        seg_scan_wave_x<NV>(rcv >= 0 ? rcv : -3 - lane, val);
        const int rnext = __shfl_down(rcv, 1, 64);
        if (rcv >= 0 && (lane == 63 || rnext != rcv)) {
#pragma unroll
          for (int v = 0; v < NV; ++v) accz[rcv - cbase + aslot][v] += val[v];
        }
      };
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
      wave_sync();
    }
    if (EVR_KD_PROF == 2) st_[4] = wall_clock64();
  }
  __syncthreads();
  // ---- split partials, summed in hvi_kd2's partial order (split-major, wave-split minor) ----
  for (int e = tid; e < b * NV; e += nth) {
    const int v = e / b, gc = e - v * b;
    const int gi = gc / gsz, i = gc - gi * gsz;   // slot group and slot of candidate gc
    double sum = 0.0;
    for (int zz = 0; zz < nz; ++zz)
      for (int ws = 0; ws < W; ++ws) sum += acc[zz][(gi * W + ws) * CW + i][v];
    if (v == 0) sval[(size_t)s * b + gc] = sum;
    else dG[((size_t)s * M + (v - 1)) * b + gc] = 1.0 / (double)S * sum;
  }
  if (EVR_KD_PROF == 2 && kd.counters && lane == 0) {
    st_[5] = wall_clock64();
    unsigned long long* r = kd.counters + 16 + 8 * ((size_t)s * 16 + (tid >> 6));
#pragma unroll
    for (int k = 0; k < 6; ++k) r[k] = st_[k];
    r[6] = (unsigned long long)np_;
    r[7] = (unsigned long long)nt_ | ((unsigned long long)z << 40) | ((unsigned long long)(zin && valid(cbase)) << 48);
  }
}

// ---------------------------------------------------------------------------------------
// hvi_kdb — the restart-batch scan (b <= 32) with the work of a sample balanced over all 16
// waves of its workgroup.  hvi_kd3 keeps hvi_kd2's per-wave ownership (a wave's candidates x
// its round-robin chunks), and at optimised restart candidates a sample's terms concentrate in
// a few chunks: the heaviest wave of a workgroup carried ~3x the mean wave's terms while the
// other waves waited at the final barrier (tools/kd3_waves.py).  Here every phase is spread
// over the workgroup in candidate-major order:
//   A. (candidate, chunk) entries, one per thread: chunk test, then the chunk's 16 group tests
//      -> 16-bit group masks; a block scan of their popcounts numbers the passing (candidate,
//      group) pairs candidate-major, and each entry writes its pairs;
//   B. pairs, one per thread (layers of KB_THREADS): the group's 16 cell tests -> 16-bit cell
//      masks; a block scan numbers the terms and each pair writes its terms' (key index,
//      candidate);
//   C. terms split evenly over the 16 waves in rounds of 64: key decode, term and subgradients;
//      a wave share spanning few candidates (the usual case: a candidate's terms are one
//      contiguous run) sums per lane in registers and reduces once per candidate, otherwise
//      segmented sums keyed by candidate per round — into the wave's own accumulators;
//   then per (candidate, value) the 16 waves' partials summed in wave order.
// Pairs and terms go through LDS in slices of KB_PCAP / KB_TCAP, so any count is handled.
// Every order is a function of the data only: bitwise reproducible.  Not bitwise equal to
// hvi_kd2 (different summation order; equal to rounding).
// ---------------------------------------------------------------------------------------
constexpr int KB_THREADS = 1024, KB_WAVES = 16, KB_B = 32, KB_PCAP = 4096, KB_TCAP = 8192;
// candidate slots of the register accumulation (a wave share spanning more candidates takes
// the segmented-scan rounds)
constexpr int KB_SLOTS = 3;

struct KbLds {
  size_t pt, th, gbl, pinfo, tkey, tcand, acc, bytes;
};
__host__ __device__ inline KbLds kb_lds(int stride, int M, int max_groups) {
  KbLds L;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t r = o;
    o = (o + bytes + 15) & ~(size_t)15;
    return r;
  };
  L.pt = take((size_t)stride * M * 8);
  L.th = take((size_t)stride * M * 8);
  L.gbl = take((size_t)(max_groups + 15) / 16 * 16 * 16);
  L.pinfo = take((size_t)KB_PCAP * 4);   // (candidate << 16 | group) per pair of a slice
  L.tkey = take((size_t)KB_TCAP * 4);    // key index per term of a sub-slice
  L.tcand = take((size_t)KB_TCAP);       // candidate per term
  L.acc = take((size_t)KB_WAVES * KB_B * (M + 1) * 8);
  L.bytes = o;
  return L;
}

// block-wide exclusive scan of one int per thread (sum, or max with -1 as identity) in thread
// order; *total = the block's sum / max.  sh: KB_WAVES ints.
template <bool MAX>
__device__ __forceinline__ int kb_scan_excl(int v, int* sh, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc;
  if (MAX) {
    inc = wave_max_incl(v);
  } else {
    int t;
    inc = wave_scan_excl(v, &t) + v;
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  int pre = MAX ? -1 : 0, tot = MAX ? -1 : 0;
#pragma unroll
  for (int k = 0; k < KB_WAVES; ++k) {
    const int x = sh[k];
    if (k < w) pre = MAX ? max(pre, x) : pre + x;
    tot = MAX ? max(tot, x) : tot + x;
  }
  __syncthreads();
  int exw = __shfl_up(inc, 1, 64);
  if (lane == 0) exw = MAX ? -1 : 0;
  *total = tot;
  return MAX ? max(pre, exw) : pre + exw;
}

template <int M>
__global__ __launch_bounds__(KB_THREADS) void hvi_kdb(int b, int S, const double* __restrict__ G, HviKd kd,
                                                      KbSamples smp, double* __restrict__ sval,
                                                      double* __restrict__ dG) {
  constexpr int NV = M + 1;
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kd_dyn[];
  __shared__ double yv[KB_B][M];
  __shared__ __align__(16) unsigned short ths[KB_B][8];
  __shared__ uint4 cminq[KD_MAX_NQ];
  __shared__ int sh[KB_WAVES];
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int stride = kd.stride;
  const KbLds Lo = kb_lds(stride, M, kd.max_groups);
  double* pt = (double*)(kd_dyn + Lo.pt);
  double* thv = (double*)(kd_dyn + Lo.th);
  uint4* gbl = (uint4*)(kd_dyn + Lo.gbl);
  unsigned int* pinfo = (unsigned int*)(kd_dyn + Lo.pinfo);
  unsigned int* tkey = (unsigned int*)(kd_dyn + Lo.tkey);
  unsigned char* tcand = (unsigned char*)(kd_dyn + Lo.tcand);
  double* acc = (double*)(kd_dyn + Lo.acc);   // [wave][candidate][value]
  const int gbase = kd.goff[s];
  const int Gsamp = kd.goff[s + 1] - gbase;
  const int NQall = (Gsamp + 15) >> 4;
  const uint4* gmin = (const uint4*)kd.gbox + gbase;
  unsigned long long st_[7] = {0, 0, 0, 0, 0, 0, 0};
  long long nt_ = 0;
  if (EVR_KD_PROF == 2) st_[0] = wall_clock64();

  // ---- staging: point table, ascending lower bounds, group minima (+ chunk minima), values
  {
    const double* src = kd.pts + (size_t)s * stride * M;
    const double* srt = kd.sv + (size_t)s * M * stride;
    for (int e = tid; e < stride * M; e += KB_THREADS) {
      const double a = src[e], c = srt[e];
      pt[e] = a;
      thv[e] = c;
    }
  }
  for (int e = tid; e < 16 * NQall; e += KB_THREADS) {
    uint4 v = make_uint4(~0u, ~0u, ~0u, ~0u);
    if (e < Gsamp) {
      v = gmin[e];
      gbl[e] = v;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      v.x = pk_min_u16(v.x, (unsigned int)__shfl_xor((int)v.x, o, 64));
      v.y = pk_min_u16(v.y, (unsigned int)__shfl_xor((int)v.y, o, 64));
      v.z = pk_min_u16(v.z, (unsigned int)__shfl_xor((int)v.z, o, 64));
      v.w = pk_min_u16(v.w, (unsigned int)__shfl_xor((int)v.w, o, 64));
    }
    if ((e & 15) == 0) cminq[e >> 4] = v;
  }
  for (int e = tid; e < KB_B * M; e += KB_THREADS) {
    const int j = e / KB_B, c = e - j * KB_B;
    double y = -INFINITY;
    if (c < b) {
      if (smp.R) {
        // the sampling step (qn_samples_norms' arithmetic for this sample)
        const long long Rr = (long long)smp.n + smp.nb + smp.nh + 1;
        const double* Rj = smp.R + (size_t)j * Rr * b;
        const double hv = smp.nh ? Rj[(size_t)(smp.n + smp.nb + s) * b + c] : 0.0;
        const double zv = smp.zq[(size_t)s * M + j];
        double mu, l22;
        int flag;
        qn_mu_l22(smp.P + (size_t)j * smp.nrt * 2 * b, smp.nrt_used, b, c, Rj[(size_t)(Rr - 1) * b + c], smp.ys[j],
                  smp.cc[j], smp.ym[j], smp.kxx[j], mu, l22, flag);
        if (s == 0) {
          smp.L22[(size_t)j * b + c] = l22;
          smp.flags[(size_t)j * b + c] = flag;
        }
        y = qn_sample_obj(mu, hv, smp.nh != 0, l22, zv, smp.oa[j], smp.ob[j]);
      } else {
        y = G[((size_t)s * M + j) * b + c];
      }
    }
    yv[c][j] = y;
  }
  for (int e = tid; e < KB_WAVES * KB_B * NV; e += KB_THREADS) acc[e] = 0.0;
  __syncthreads();
  if (EVR_KD_PROF == 2) st_[1] = wall_clock64();
  // thresholds t_j = #{rows with lower-bound value <= y_j} (hvi_thresholds' search)
  if (tid < KB_B * 8) {
    const int c = tid >> 3, j = tid & 7;
    unsigned short v = 1;
    if (j < M) {
      v = 0;
      if (c < b) {
        const double y = yv[c][j];
        const double* tv = thv + (size_t)j * stride;
        int lo = 0, hi = stride;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (tv[mid] <= y) lo = mid + 1;
          else hi = mid;
        }
        v = (unsigned short)lo;
      }
    }
    ths[c][j] = v;
  }
  __syncthreads();
  const uint4* thp = reinterpret_cast<const uint4*>(&ths[0][0]);
  if (EVR_KD_PROF == 2) st_[2] = wall_clock64();

  // ---- A: entries e = c * NQall + q, one per thread ----
  const int NE = b * NQall;   // <= KB_B * KD_MAX_NQ = KB_THREADS
  unsigned int emk = 0;       // the entry's passing groups
  int ec = 0, eq = 0;
  if (tid < NE) {
    ec = tid / NQall;
    eq = tid - ec * NQall;
    const uint4 tt = thp[ec];
    if (kd_pass4(cminq[eq], tt)) {
      const int gend = min(16, Gsamp - 16 * eq);
      for (int k = 0; k < gend; ++k) emk |= (unsigned int)kd_pass4(gbl[eq * 16 + k], tt) << k;
    }
  }
  int PT;
  const int ep0 = kb_scan_excl<false>(__popc(emk), sh, &PT);   // the entry's first pair
  if (kd.counters && EVR_KD_PROF != 2 && tid == 0) {
    atomicAdd(kd.counters + 0, (unsigned long long)PT);
    atomicAdd(kd.counters + 2, (unsigned long long)b * Gsamp);
  }
  if (EVR_KD_PROF == 2) st_[3] = wall_clock64();

  constexpr int PPT = KB_PCAP / KB_THREADS;   // pairs per thread in a slice
  for (int P0 = 0; P0 < PT; P0 += KB_PCAP) {
    const int Pn = min(KB_PCAP, PT - P0);
    // ---- the slice's pairs (candidate, group), written by their entries ----
    {
      unsigned int mk = emk;
      int p = ep0;
      while (mk) {
        const int k = __ffs(mk) - 1;
        mk &= mk - 1;
        if (p >= P0 && p < P0 + Pn) pinfo[p - P0] = ((unsigned int)ec << 16) | (unsigned int)(16 * eq + k);
        ++p;
      }
    }
    __syncthreads();
    // ---- B: the group's cell tests; pair i = u * KB_THREADS + tid (layers of one pair per
    //      thread, so a thread writes at most 16 terms per layer) ----
    unsigned int pmk[PPT], pin[PPT];
    int tcnt[PPT], tpu[PPT];
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int i = u * KB_THREADS + tid;
      tcnt[u] = 0;
      pmk[u] = 0;
      pin[u] = 0;
      if (i < Pn) {
        const unsigned int info = pinfo[i];
        const int c = (int)(info >> 16), g = (int)(info & 0xFFFFu);
        const uint4* rp = (const uint4*)(kd.grk + (size_t)(gbase + g) * M * 16);
        const uint4 tq = thp[c];
        const unsigned int tw[4] = {tq.x, tq.y, tq.z, tq.w};
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
        pmk[u] = mB;
        pin[u] = info;
        tcnt[u] = __popc(mB);
      }
    }
    // term numbering in pair order: one block scan per populated layer
    int TT_ = 0;
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      tpu[u] = 0;
      if (u * KB_THREADS < Pn) {
        int tot;
        tpu[u] = TT_ + kb_scan_excl<false>(tcnt[u], sh, &tot);
        TT_ += tot;
      }
    }
    if (kd.counters && EVR_KD_PROF != 2 && tid == 0) atomicAdd(kd.counters + 1, (unsigned long long)TT_);
    if (EVR_KD_PROF == 2 && P0 == 0) st_[4] = wall_clock64();
    // ---- C: terms in sub-slices of KB_TCAP: (key index, candidate) written by their pairs,
    //      then split evenly over the waves ----
    for (int T0 = 0; T0 < TT_; T0 += KB_TCAP) {
      const int Tn = min(KB_TCAP, TT_ - T0);
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        if (pmk[u] == 0 || tpu[u] >= T0 + Tn || tpu[u] + tcnt[u] <= T0) continue;
        unsigned int mk = pmk[u];
        int t = tpu[u];
        const unsigned int kb = (unsigned int)(gbase + (int)(pin[u] & 0xFFFFu)) * 16u;
        const unsigned char cc = (unsigned char)(pin[u] >> 16);
        while (mk) {
          const int k = __ffs(mk) - 1;
          mk &= mk - 1;
          if (t >= T0 && t < T0 + Tn) {
            tkey[t - T0] = kb + (unsigned int)k;
            tcand[t - T0] = cc;
          }
          ++t;
        }
      }
      __syncthreads();
      // wave's share [tb, te) of the sub-slice
      const int tb = (int)(((long long)Tn * wave) / KB_WAVES), te = (int)(((long long)Tn * (wave + 1)) / KB_WAVES);
      double* accw = acc + (size_t)wave * KB_B * NV;
      auto locate = [&](int t, int& c, unsigned long long& key) {
        const bool in = t < te;
        const int tt = in ? t : tb;   // past the end: a valid dummy (the share's first term)
        key = kd.gkeys[tkey[tt]];
        c = in ? (int)tcand[tt] : -1;
      };
      // the term of key x candidate c and its subgradients (torch's min / clamp rules)
      auto term_value = [&](const unsigned long long key, const int c, double (&val)[NV]) {
        double l[M], u[M];
        K::decode_direct(key, pt, l, u);
        double len[M], pass[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const double y = yv[c][j];
          const double raw = fmin(y, u[j]) - l[j];
          len[j] = fmax(raw, 0.0);
          const double dmin = (y < u[j]) ? 1.0 : ((y == u[j]) ? 0.5 : 0.0);
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
          val[1 + j] = pass[j] * pre_[j] * suf;
          suf *= len[j];
        }
      };
      auto term_round = [&](const int c, const unsigned long long key) {
        int rcv = -1;
        double val[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) val[v] = 0.0;
        if (c >= 0) {
          term_value(key, c, val);
          rcv = c;
        }
        seg_scan_wave_x<NV>(rcv >= 0 ? rcv : -3 - lane, val);
        const int rnext = __shfl_down(rcv, 1, 64);
        if (rcv >= 0 && (lane == 63 || rnext != rcv)) {
#pragma unroll
          for (int v = 0; v < NV; ++v) accw[rcv * NV + v] += val[v];
        }
      };
      // the share's candidates: a contiguous range [cf, cl] (candidate-major terms)
      const int cf = te > tb ? (int)tcand[tb] : 0;
      const int cl = te > tb ? (int)tcand[te - 1] : -1;
      if (te > tb && cl - cf < KB_SLOTS) {
        // few candidates (long runs, the usual case): every lane sums its terms per candidate
        // slot in registers across the rounds, then one butterfly per (slot, value) — instead
        // of a segmented scan per round
        if (EVR_KD_PROF == 2) nt_ += te - tb;
        // three named slot rows, each added to with the term masked in (a + 0.0 = a: the
        // values are >= 0) — an indexed slot array (or a select on the slot) is lowered to
        // scratch memory by the compiler: 112 B / lane of spills, ~58 MB written per launch
        static_assert(KB_SLOTS == 3, "slot rows are spelled out");
        double as0[NV], as1[NV], as2[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) as0[v] = as1[v] = as2[v] = 0.0;
        auto term_acc = [&](const int c, const unsigned long long key) {
          if (c < 0) return;
          double val[NV];
          term_value(key, c, val);
          const int k = c - cf;
          const double w0 = k == 0 ? 1.0 : 0.0, w1 = k == 1 ? 1.0 : 0.0, w2 = k == 2 ? 1.0 : 0.0;
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            as0[v] = fma(w0, val[v], as0[v]);
            as1[v] = fma(w1, val[v], as1[v]);
            as2[v] = fma(w2, val[v], as2[v]);
          }
        };
        int cA, cB;
        unsigned long long kA, kB;
        locate(tb + lane, cA, kA);
        locate(tb + 64 + lane, cB, kB);
        for (int r = tb; r < te; r += 128) {
          term_acc(cA, kA);
          locate(r + 128 + lane, cA, kA);
          if (r + 64 < te) term_acc(cB, kB);
          locate(r + 192 + lane, cB, kB);
        }
        // per (slot, value) the wave sum by a DPP inclusive scan (VALU only, fixed order):
        // lane 63 holds the total
        auto slot_out = [&](const int kk, double (&a)[NV]) {
          if (cf + kk > cl) return;
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            double x = a[v];
            x += dpp_f64<0x111, 0xF>(x);
            x += dpp_f64<0x112, 0xF>(x);
            x += dpp_f64<0x114, 0xF>(x);
            x += dpp_f64<0x118, 0xF>(x);
            x += dpp_f64<0x142, 0xA>(x);
            x += dpp_f64<0x143, 0xC>(x);
            if (lane == 63) accw[(cf + kk) * NV + v] += x;
          }
        };
        slot_out(0, as0);
        slot_out(1, as1);
        slot_out(2, as2);
      } else if (te > tb) {
        if (EVR_KD_PROF == 2) nt_ += te - tb;
        int cA, cB;
        unsigned long long kA, kB;
        locate(tb + lane, cA, kA);
        locate(tb + 64 + lane, cB, kB);
        for (int r = tb; r < te; r += 128) {
          term_round(cA, kA);
          locate(r + 128 + lane, cA, kA);
          if (r + 64 < te) term_round(cB, kB);
          locate(r + 192 + lane, cB, kB);
        }
      }
      __syncthreads();   // tkey / tcand / acc rows reused
    }
  }
  if (EVR_KD_PROF == 2) st_[5] = wall_clock64();
  // ---- the waves' partials per (candidate, value), summed in wave order ----
  for (int e = tid; e < b * NV; e += KB_THREADS) {
    const int v = e / b, c = e - v * b;
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < KB_WAVES; ++w) sum += acc[((size_t)w * KB_B + c) * NV + v];
    if (v == 0) sval[(size_t)s * b + c] = sum;
    else dG[((size_t)s * M + (v - 1)) * b + c] = 1.0 / (double)S * sum;
  }
  if (EVR_KD_PROF == 2 && kd.counters && lane == 0) {
    st_[6] = wall_clock64();
    unsigned long long* r = kd.counters + 16 + 8 * ((size_t)s * 16 + wave);
#pragma unroll
    for (int k = 0; k < 7; ++k) r[k] = st_[k];
    r[7] = (unsigned long long)nt_;
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
// qtl.M != null: workgroups from nkdw on run the restart backward's training-row class
// (qs_tail.hpp) — dispatched last, into the slots the light (sample, candidate) waves free.
template <int M>
__global__ __launch_bounds__(256, M <= 7 ? 5 : 4) void hvi_kdw(int b, int S, int ncg, const double* __restrict__ G, HviKd kd,
                                               KbSamples smp, double* __restrict__ sval, double* __restrict__ dG,
                                               QsTail qtl, int nkdw, int ntail_first) {
  constexpr int NV = M + 1;
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kw_dyn[];
  // ntail_first > 0: the tail's workgroups come first instead (a multiple of 8: the scan's
  // workgroup -> XCD map is unchanged)
  if (qtl.M && ((int)blockIdx.x >= nkdw + ntail_first || (int)blockIdx.x < ntail_first)) {
    qs_tail_tile(qtl, ntail_first ? blockIdx.x : blockIdx.x - nkdw, (double*)kw_dyn);
    return;
  }
  const int wid = blockIdx.x - ntail_first, xcd = wid & 7, slot = wid >> 3;
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

// scan variant: 2 = hvi_kd2 (default), 1 = hvi_kd (EVR_KD=1 or evr_hvi_set_kd_variant)
static int g_kd_variant = 0;
static int kd_variant() {
  if (g_kd_variant == 0) {
    const char* e = std::getenv("EVR_KD");
    g_kd_variant = (e && std::atoi(e) == 1) ? 1 : 2;
  }
  return g_kd_variant;
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

static HviKd hvi_kd_of(const evr_qnehvi_state* st) {
  return HviKd{st->grp_off, st->grp_keys, st->grp_rank, st->grp_box, st->sorted_lo, st->cell_pts, st->cell_rank0,
               st->pts_stride, st->max_groups, st->scan_counters};
}

// waves sharing one 16-candidate group in hvi_kd2 (chunks split between them): the
// restart batches (b <= 32) would leave 2-3 of the 4 waves idle otherwise
static int hvi_kd_wsplit(int b) {
  if (kd_variant() != 2) return 1;
  return b <= 16 ? 4 : (b <= 32 ? 2 : 1);
}

// group-range splits per sample: fill ~1024 workgroups at small candidate batches
static int hvi_kd_nsplit(const evr_qnehvi_state* st, int b) {
  const int tiles = cdiv(b, KD_CT / hvi_kd_wsplit(b)) * st->S;
  const int nq = (st->max_groups + 15) / 16;
  static const int wgs = [] {   // EVR_KD_WGS: workgroups to fill (tuning knob, default 1024)
    const char* e = std::getenv("EVR_KD_WGS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 1024;
  }();
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
  const KdLds Lo = kd_lds(st->pts_stride, M, st->max_groups);
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
  if (kd_variant() == 1) {
    EVR_HIP(hipFuncSetAttribute((const void*)hvi_kd<M, BWD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)Lo.bytes));
    hvi_kd<M, BWD><<<grid, 256, Lo.bytes, s>>>(b, st->S, ntiles, ns, G, th, hvi_kd_of(st), gout, part,
                                                 ns > 1 ? dgp : dG);
  } else {
    EVR_CHECK((st->max_groups + 15) / 16 <= KD_MAX_NQ, "hvi: %d kd groups per sample exceed the scan's %d",
              st->max_groups, 16 * KD_MAX_NQ);
    const Kd2Lds L2 = kd2_lds(st->pts_stride, M, st->max_groups);
    EVR_HIP(hipFuncSetAttribute((const void*)hvi_kd2<M, BWD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)L2.bytes));
    static const int balance = [] {   // EVR_KD_BALANCE=0: 16-slot groups filled in order (A/B)
      const char* e = std::getenv("EVR_KD_BALANCE");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    // round-robin chunks for the wave-split restart batches (b <= 32); larger batches keep
    // contiguous ranges (bitwise equal to hvi_kd).  EVR_KD_ILV=0: contiguous everywhere (A/B)
    static const int ilv = [] {
      const char* e = std::getenv("EVR_KD_ILV");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    hvi_kd2<M, BWD><<<grid, 256, L2.bytes, s>>>(b, st->S, ntiles, nsb, G, th, hvi_kd_of(st), gout, part,
                                                  ns > 1 ? dgp : dG, W, balance, ilv && W > 1);
  }
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

// restart-scan kernel: 3 = hvi_kdw (default), 2 = hvi_kdb (balanced), 1 = hvi_kd3 (EVR_KDB=0 or
// evr_hvi_set_restart_variant)
static int g_restart_variant = 0;
static int restart_variant() {
  if (g_restart_variant == 0) {
    // EVR_RESTART_SCAN=kdw (default) | kdb | kd3; the older EVR_KDB=0 still selects kd3
    const char* e = std::getenv("EVR_RESTART_SCAN");
    const char* k = std::getenv("EVR_KDB");
    if (e && std::string(e) == "kdb") g_restart_variant = 2;
    else if ((e && std::string(e) == "kd3") || (k && k[0] == '0')) g_restart_variant = 1;
    else g_restart_variant = 3;
  }
  return g_restart_variant;
}

static bool hvi_kdw_applies(const evr_qnehvi_state* st, int b) {
  if (restart_variant() != 3 || !st || st->log_hvi || !st->grp_off || b < 1 || b > 32 || kd_variant() != 2 ||
      st->m < 1 || st->m > 8 || st->max_groups > KW_MAXG)
    return false;
  // the threshold probe reads 64 bucket ends, then the 64 entries of the straddling bucket:
  // exact for strides up to 64 x 64 rows only
  if (st->pts_stride > 64 * 64) return false;
  return kw_lds_bytes(st->pts_stride, st->m) <= 64 * 1024;
}

template <int M>
static int hvi_kdw_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                          double* dG, const KbSamples& smp, const QsTail* tail = nullptr) {
  size_t lds = kw_lds_bytes(st->pts_stride, M);
  const int ncg = cdiv(b, KW_WAVES);
  const int wgs = cdiv(st->S, 8) * 8 * ncg;
  QsTail tl{};
  int twgs = 0;
  if (tail) {
    tl = *tail;
    twgs = st->m * tl.za * tl.nt;
    lds = std::max(lds, (size_t)QT_LDS_DOUBLES * 8);
  }
  EVR_HIP(hipFuncSetAttribute((const void*)hvi_kdw<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // EVR_QS_TAIL_FIRST=1: the tail's workgroups dispatched before the scan's (A/B)
  const char* tfe = std::getenv("EVR_QS_TAIL_FIRST");
  const bool tfirst = tfe && tfe[0] == '1';
  const int nfirst = (tfirst && twgs) ? cdiv(twgs, 8) * 8 : 0;
  hvi_kdw<M><<<wgs + (nfirst ? nfirst : twgs), 256, lds, s>>>(b, st->S, ncg, G, hvi_kd_of(st), smp, sval, dG, tl, wgs,
                                                               nfirst);
  EVR_LAUNCH_CHECK();
  return 0;
}

static bool hvi_kdb_applies(const evr_qnehvi_state* st, int b) {
  if (restart_variant() != 2 || !st || st->log_hvi || !st->grp_off || b < 1 || b > KB_B || kd_variant() != 2 ||
      st->m < 1 || st->m > 8)
    return false;
  if ((st->max_groups + 15) / 16 > KD_MAX_NQ) return false;
  return kb_lds(st->pts_stride, st->m, st->max_groups).bytes <= 148 * 1024;
}

template <int M>
static int hvi_kdb_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                          double* dG, const KbSamples& smp) {
  const KbLds L = kb_lds(st->pts_stride, M, st->max_groups);
  EVR_HIP(hipFuncSetAttribute((const void*)hvi_kdb<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.bytes));
  hvi_kdb<M><<<st->S, KB_THREADS, L.bytes, s>>>(b, st->S, G, hvi_kd_of(st), smp, sval, dG);
  EVR_LAUNCH_CHECK();
  return 0;
}

// hvi_kd3 (one launch: thresholds, scan, split reduction) for the restart batches: kd cells,
// b <= 32, the kd2 variant, and its LDS within budget.  EVR_KD3=0 keeps the three-launch
// chain (A/B).
static bool hvi_kd3_applies(const evr_qnehvi_state* st, int b) {
  static const bool on = [] {
    const char* e = std::getenv("EVR_KD3");
    return !(e && e[0] == '0');
  }();
  if (!on || !st || st->log_hvi || !st->grp_off || b < 1 || b > 32 || kd_variant() != 2 || st->m < 1 || st->m > 8)
    return false;
  if ((st->max_groups + 15) / 16 > KD_MAX_NQ) return false;
  // the splits of hvi_kd2's launch (at most 4 sub-workgroups; S >= 256 at these batches)
  const int nz = hvi_kd_nsplit(st, b);
  return nz <= KD3_NZ && kd3_lds(st->pts_stride, st->m, st->max_groups, nz).bytes <= 128 * 1024;
}

template <int M>
static int hvi_kd3_launch(hipStream_t s, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                          double* dG) {
  const int W = hvi_kd_wsplit(b);
  // the same split count as hvi_kd2's launch (bitwise equal dG); one 256-thread
  // sub-workgroup per split
  const int nz = hvi_kd_nsplit(st, b);
  EVR_CHECK(nz >= 1 && nz <= KD3_NZ, "hvi_kd3: %d splits exceed %d sub-workgroups", nz, KD3_NZ);
  EVR_CHECK(cdiv(b, KD_CT / W) == 1, "hvi_kd3: %d candidates exceed one tile", b);
  const Kd3Lds L = kd3_lds(st->pts_stride, M, st->max_groups, nz);
  static const int balance = [] {
    const char* e = std::getenv("EVR_KD_BALANCE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  EVR_HIP(hipFuncSetAttribute((const void*)hvi_kd3<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.bytes));
  hvi_kd3<M><<<st->S, 256 * nz, L.bytes, s>>>(b, st->S, nz, G, hvi_kd_of(st), sval, dG, W, balance);
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

int evr_hvi_restart_fb_applies(const evr_qnehvi_state* st, int b) {
  return (hvi_kdw_applies(st, b) || hvi_kdb_applies(st, b) || hvi_kd3_applies(st, b)) ? 1 : 0;
}

int evr_hvi_restart_fb(void* stream, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                       double* dG) {
  if (int rc = hvi_check_state(st)) return rc;
  EVR_CHECK(G && sval && dG && (hvi_kdw_applies(st, b) || hvi_kdb_applies(st, b) || hvi_kd3_applies(st, b)),
            "evr_hvi_restart_fb: bad arguments or the state / batch is not a kd restart batch (b <= 32)");
  int rc = 0;
  if (hvi_kdw_applies(st, b)) {
    const KbSamples smp{};
#define L(MM) rc = hvi_kdw_launch<MM>((hipStream_t)stream, st, b, G, sval, dG, smp)
    EVR_M_SWITCH(st->m, L);
#undef L
    return rc;
  }
  if (hvi_kdb_applies(st, b)) {
    const KbSamples smp{};
#define L(MM) rc = hvi_kdb_launch<MM>((hipStream_t)stream, st, b, G, sval, dG, smp)
    EVR_M_SWITCH(st->m, L);
#undef L
    return rc;
  }
#define L(MM) rc = hvi_kd3_launch<MM>((hipStream_t)stream, st, b, G, sval, dG)
  EVR_M_SWITCH(st->m, L);
#undef L
  return rc;
}

}  // extern "C"

namespace evr {
// the restart scan with the sampling step fused into its staging (native plan, b <= 32 with
// the kdb variant): R / P from the projection, L22 / flags written by sample 0's workgroup
bool hvi_kdb_fused_applies(const evr_qnehvi_state* st, int b) {
  static const bool on = [] {
    const char* e = std::getenv("EVR_FUSED_SAMPLES");
    return !(e && e[0] == '0');
  }();
  return on && (hvi_kdw_applies(st, b) || hvi_kdb_applies(st, b)) && st->obj_a && st->obj_b && st->zq;
}

// tail (optional): the restart backward's training-row class, run in hvi_kdw's tail; *tail_ran
// says whether it was (hvi_kdb has no tail: the caller launches it itself)
int hvi_kdb_fused(hipStream_t s, const evr_qnehvi_state* st, int b, const double* R, const double* P, int nrt,
                  int nrt_used, double* L22, int* flags, double* sval, double* dG, const QsTail* tail,
                  bool* tail_ran) {
  if (tail_ran) *tail_ran = false;
  EVR_CHECK(R && P && L22 && flags && sval && dG && hvi_kdb_fused_applies(st, b), "hvi_kdb_fused: bad arguments");
  KbSamples smp{R, P, st->c, st->ym, st->ys, st->kxx, st->zq, st->obj_a, st->obj_b, L22, flags,
                st->n, st->nb, qn_nh(st), nrt, nrt_used};
  int rc = 0;
  if (hvi_kdw_applies(st, b)) {
#define L(MM) rc = hvi_kdw_launch<MM>(s, st, b, nullptr, sval, dG, smp, tail)
    EVR_M_SWITCH(st->m, L);
#undef L
    if (tail_ran) *tail_ran = tail != nullptr && rc == 0;
    return rc;
  }
#define L(MM) rc = hvi_kdb_launch<MM>(s, st, b, nullptr, sval, dG, smp)
  EVR_M_SWITCH(st->m, L);
#undef L
  return rc;
}
}  // namespace evr

extern "C" {

int evr_hvi_set_restart_variant(int variant) {
  EVR_CHECK(variant >= 1 && variant <= 3, "evr_hvi_set_restart_variant: variant must be 1 (kd3), 2 (kdb) or 3 (kdw), got %d",
            variant);
  g_restart_variant = variant;
  return 0;
}

int evr_hvi_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G, const double* gout,
                     double* work, double* dG) {
  return evr_hvi_forward_backward(stream, st, b, G, nullptr, gout, work, nullptr, dG);
}

int evr_hvi_set_kd_variant(int variant) {
  EVR_CHECK(variant == 1 || variant == 2, "evr_hvi_set_kd_variant: variant must be 1 or 2, got %d", variant);
  g_kd_variant = variant;
  return 0;
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
