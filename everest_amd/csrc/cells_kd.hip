// kd ordering of the box-decomposition cells for the sparse HVI scan (hvi.hip, hvi_kd).
//
// At the bench state (DTLZ2, m = 5, ~5.8k cells per MC sample) only ~0.7 % of the
// (cell, candidate) pairs have a non-zero HVI term: a cell contributes to candidate y only
// if its lower corner l <= y in every objective.  Ordering the cells of a sample so that 16
// consecutive cells form a tight group in lower-corner space lets the scan reject a whole
// group with one 5-way test on the group's minimum corner; a kd split order (median split
// on the objective of largest rank spread) takes the per-candidate group pass rate from
// ~17 % (cells ordered by first lower bound only) to ~4 %.
//
// Every lower bound l_j of a cell is the coordinate of one row of the sample's point table
// (l_j = -pts[P_j][j], box_device.hip), so the scan works in RANK space: rank_j(p) = position
// of row p in ascending -pts[.][j] (ties by row index).  A cell passes objective j iff
// rank_j(P_j) < t_j(y) with t_j(y) = #{rows p : -pts[p][j] <= y_j} — exact, ties included,
// and 16-bit integer compares instead of f64.
//
// One 1024-thread workgroup per sample:
//   1. rank tables rank_j(p) and the ascending value lists (sorted_lo, for the thresholds);
//   2. kd levels: per splittable segment (> 16 cells) the objective of largest rank spread
//      (LDS integer atomics), then ONE bitonic sort of (segment, rank, cell) keys orders
//      every segment by its objective; segments split at 16*ceil(len/32) so every group of
//      16 lies in one leaf;
//   3. outputs per group of 16: keys in kd order (field 0 rewritten from the rank to the point
//      index, so the scan decodes without the rank table), per-cell rank coordinates ([j][16]
//      u16, 0x7FFF padding) and the group's minimum rank per objective.
// Deterministic: keys are unique (cell index in the low bits), so the order never depends
// on thread timing.
#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int KD_THREADS = 1024;
constexpr int KD_MAX_CELLS = 8192;          // LDS sort buffer (64 KB)
constexpr int KD_MAX_GROUPS = KD_MAX_CELLS / 16;
constexpr unsigned short KD_PAD = 0x7FFF;   // > every threshold (ranks < 2^15: packed signed compares)

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const int lo = __shfl_xor((int)(unsigned)v, m, 64), hi = __shfl_xor((int)(unsigned)(v >> 32), m, 64);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// Bitonic sort of P2 (a power of two) unique keys in LDS.  Stages whose partner distance j is
// at least 64 exchange through LDS (one barrier each); the stages with j < 64 pair lanes of one
// wave (index i = tid + 1024 t, so a wave holds 64 consecutive keys) and run in registers by
// xor-shuffles, min / max per pair, with one barrier per merge size: 41 instead of 91 barriers
// per sort at P2 = 8192.  Same result as the compare-and-swap network (keys are unique).
__device__ __forceinline__ void kd_bitonic(unsigned long long* a, int P2) {
  for (int k = 2; k <= P2; k <<= 1) {
    int j = k >> 1;
    for (; j >= 64; j >>= 1) {
      for (int i = threadIdx.x; i < P2; i += KD_THREADS) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long x = a[i], y = a[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < P2; i += KD_THREADS) {
      unsigned long long x = a[i];
      const bool up = (i & k) == 0;
      for (int jj = j; jj > 0; jj >>= 1) {
        const unsigned long long y = shfl_xor_u64(x, jj);
        // the lower index of a pair keeps the minimum in an ascending run, the maximum otherwise
        x = (((i & jj) == 0) == up) ? (x < y ? x : y) : (x < y ? y : x);
      }
      a[i] = x;
    }
    __syncthreads();
  }
}

template <int M>
__global__ __launch_bounds__(KD_THREADS) void cells_kd_kernel(int stride, const int* __restrict__ off,
                                                             const int* __restrict__ goff,
                                                             const unsigned long long* __restrict__ keys,
                                                             const double* __restrict__ pts,
                                                             const int* __restrict__ rank0,
                                                             unsigned long long* __restrict__ okeys,
                                                             unsigned short* __restrict__ ork,
                                                             unsigned short* __restrict__ ogb,
                                                             double* __restrict__ osv) {
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kd_dyn[];
  __shared__ int segS[KD_MAX_GROUPS], segE[KD_MAX_GROUPS];
  __shared__ unsigned int mn[KD_MAX_GROUPS][M], mx[KD_MAX_GROUPS][M];
  __shared__ int sh_any;
  const int s = blockIdx.x, tid = threadIdx.x;
  const int c0 = off[s], C = off[s + 1] - c0;
  const int g0 = goff[s], G = goff[s + 1] - g0;
  unsigned long long* sb = (unsigned long long*)kd_dyn;               // P2 sort keys
  int P2 = 16;
  while (P2 < C) P2 <<= 1;
  double* pt = (double*)(sb + P2);                                     // stride x M
  unsigned short* rk = (unsigned short*)(pt + (size_t)stride * M);     // M x stride
  const double* gp = pts + (size_t)s * stride * M;
  const int* gr0 = rank0 + (size_t)s * stride;
  for (int e = tid; e < stride * M; e += KD_THREADS) pt[e] = gp[e];
  __syncthreads();
  // 1. rank tables and ascending lower-bound values per objective
  for (int e = tid; e < stride * M; e += KD_THREADS) {
    const int j = e / stride, p = e - j * stride;
    const double v = -pt[p * M + j];
    int r = 0;
    for (int q = 0; q < stride; ++q) {
      const double w = -pt[q * M + j];
      r += (w < v) || (w == v && q < p);
    }
    rk[j * stride + p] = (unsigned short)r;
    osv[((size_t)s * M + j) * stride + r] = v;
  }
  auto rank_of = [&](int cell, int j) -> unsigned int {
    const unsigned long long key = keys[c0 + cell];
    const int p = (j == 0) ? gr0[K::field(key, 0)] : K::field(key, j);
    return rk[j * stride + p];
  };
  for (int g = tid; g < G; g += KD_THREADS) {
    segS[g] = 0;
    segE[g] = G;
  }
  for (int i = tid; i < P2; i += KD_THREADS) sb[i] = (i < C) ? (unsigned long long)i : ~0ull;
  __syncthreads();
  // 2. kd levels
  for (int level = 0; level < 32; ++level) {
    if (tid == 0) sh_any = 0;
    for (int g = tid; g < G; g += KD_THREADS) {
      if (segS[g] == g) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
          mn[g][j] = 0xFFFFFFFFu;
          mx[g][j] = 0u;
        }
      }
    }
    __syncthreads();
    // segment rank spans: a segment is a run of whole groups of 16 cells, so the 16 lanes of
    // one group (uniform control flow) reduce by xor-shuffles first and one lane per group
    // updates the segment's LDS minimum / maximum (16x fewer same-address atomics)
    for (int i = tid; i < G * 16; i += KD_THREADS) {
      const int g = i >> 4, a = segS[g], e = segE[g];
      const int ncell = min(16 * e, C) - 16 * a;
      if (ncell <= 16) continue;
      sh_any = 1;
      const bool in = i < C;
      const int cell = in ? (int)(sb[i] & 0xFFFFu) : 0;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        unsigned int lo = in ? rank_of(cell, j) : 0xFFFFFFFFu, hi = in ? lo : 0u;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
          lo = min(lo, (unsigned int)__shfl_xor((int)lo, o, 16));
          hi = max(hi, (unsigned int)__shfl_xor((int)hi, o, 16));
        }
        if ((i & 15) == 0) {
          atomicMin(&mn[a][j], lo);
          atomicMax(&mx[a][j], hi);
        }
      }
    }
    __syncthreads();
    if (!sh_any) break;
    for (int i = tid; i < C; i += KD_THREADS) {
      const int g = i >> 4, a = segS[g], e = segE[g];
      const int ncell = min(16 * e, C) - 16 * a;
      const int cell = (int)(sb[i] & 0xFFFFu);
      unsigned long long v;
      if (ncell > 16) {
        int jb = 0;
        unsigned int best = mx[a][0] - mn[a][0];
#pragma unroll
        for (int j = 1; j < M; ++j) {
          const unsigned int sp = mx[a][j] - mn[a][j];
          if (sp > best) {
            best = sp;
            jb = j;
          }
        }
        v = rank_of(cell, jb);
      } else {
        v = (unsigned long long)i;  // finished segment: keep its order
      }
      sb[i] = ((unsigned long long)a << 40) | (v << 16) | (unsigned long long)cell;
    }
    __syncthreads();
    kd_bitonic(sb, P2);
    // split: [a, e) -> [a, a + h), [a + h, e), h = ceil(ncell / 32) groups
    int na[KD_MAX_GROUPS / KD_THREADS + 1], ne[KD_MAX_GROUPS / KD_THREADS + 1];
    int t = 0;
    for (int g = tid; g < G; g += KD_THREADS, ++t) {
      const int a = segS[g], e = segE[g];
      const int ncell = min(16 * e, C) - 16 * a;
      na[t] = a;
      ne[t] = e;
      if (ncell > 16) {
        const int h = (ncell + 31) / 32;
        if (g < a + h) ne[t] = a + h;
        else na[t] = a + h;
      }
    }
    __syncthreads();
    t = 0;
    for (int g = tid; g < G; g += KD_THREADS, ++t) {
      segS[g] = na[t];
      segE[g] = ne[t];
    }
    __syncthreads();
  }
  // 3. outputs: keys, rank coordinates and group minimum corners
  for (int i = tid; i < G * 16; i += KD_THREADS) {
    const int g = i >> 4, w = i & 15;
    const size_t gg = (size_t)(g0 + g);
    if (i < C) {
      const int cell = (int)(sb[i] & 0xFFFFu);
      const unsigned long long key = keys[c0 + cell];
      okeys[gg * 16 + w] = K::set(key, 0, gr0[K::field(key, 0)]);   // field 0: rank -> point index
#pragma unroll
      for (int j = 0; j < M; ++j) ork[(gg * M + j) * 16 + w] = (unsigned short)rank_of(cell, j);
    } else {
      okeys[gg * 16 + w] = 0ull;
#pragma unroll
      for (int j = 0; j < M; ++j) ork[(gg * M + j) * 16 + w] = KD_PAD;
    }
  }
  __syncthreads();
  for (int e = tid; e < G * 8; e += KD_THREADS) {
    const int g = e >> 3, j = e & 7;
    unsigned short v = 0;  // objectives beyond M always pass
    if (j < M) {
      v = KD_PAD;
      const size_t gg = (size_t)(g0 + g);
      for (int w = 0; w < 16; ++w) v = min(v, ork[(gg * M + j) * 16 + w]);
    }
    ogb[(size_t)(g0 + g) * 8 + j] = v;
  }
}

}  // namespace evr

using namespace evr;

extern "C" {

int evr_cells_kd_limits(int stride, int m, int max_cells, long long* lds_bytes) {
  EVR_CHECK(stride > 0 && m >= 1 && m <= 8, "evr_cells_kd_limits: bad arguments");
  int P2 = 16;
  while (P2 < max_cells) P2 <<= 1;
  const long long lds = (long long)P2 * 8 + (long long)stride * m * 10 + 16;
  if (lds_bytes) *lds_bytes = lds;
  return (max_cells <= KD_MAX_CELLS && stride < 0x7FFF && lds <= 96 * 1024) ? 0 : 3;
}

int evr_cells_kd_order_device(void* stream, int S, int m, int stride, const int* off, const int* goff,
                              int max_cells, const unsigned long long* keys, const double* pts,
                              const int* rank0, unsigned long long* okeys, unsigned short* ork,
                              unsigned short* ogb, double* osv) {
  EVR_CHECK(S >= 1 && m >= 1 && m <= 8 && off && goff && keys && pts && rank0 && okeys && ork && ogb && osv,
            "evr_cells_kd_order_device: bad arguments");
  long long lds = 0;
  EVR_CHECK(evr_cells_kd_limits(stride, m, max_cells, &lds) == 0,
            "evr_cells_kd_order_device: %d cells / %d point rows exceed the kd kernel limits", max_cells, stride);
  hipStream_t s = (hipStream_t)stream;
#define L(MM)                                                                                            \
  do {                                                                                                   \
    EVR_HIP(hipFuncSetAttribute((const void*)cells_kd_kernel<MM>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                  \
    cells_kd_kernel<MM><<<S, KD_THREADS, lds, s>>>(stride, off, goff, keys, pts, rank0, okeys, ork, ogb, \
                                                   osv);                                                 \
  } while (0)
  switch (m) {
    case 1: L(1); break;
    case 2: L(2); break;
    case 3: L(3); break;
    case 4: L(4); break;
    case 5: L(5); break;
    case 6: L(6); break;
    case 7: L(7); break;
    case 8: L(8); break;
  }
#undef L
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
