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
#include <cstdlib>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int KD_THREADS = 1024;
constexpr int KD_MAX_CELLS = 8192;          // LDS sort buffer (64 KB)
constexpr int KD_MAX_GROUPS = KD_MAX_CELLS / 16;
constexpr unsigned short KD_PAD = 0x7FFF;   // > every threshold (ranks < 2^15: packed signed compares)

// EVR_CKD_PROF builds (profiling only): per-sample phase clocks (s_memrealtime, 100 MHz), slot k of sample s at
// ckd_prof[16 s + k] (0 start, 1 rank tables, 2 spans, 3 keys, 4 sorts, 5 splits, 6 end, 7 levels)
#ifdef EVR_CKD_PROF
__device__ unsigned long long ckd_prof[16 * 4096];
#define CKD_T(k) if (threadIdx.x == 0 && blockIdx.x < 4096) ckd_prof[16 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();
#define CKD_ACC(k, t0) if (threadIdx.x == 0 && blockIdx.x < 4096) ckd_prof[16 * blockIdx.x + (k)] += __builtin_amdgcn_s_memrealtime() - (t0);
#define CKD_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define CKD_T(k)
#define CKD_ACC(k, t0)
#define CKD_NOW() 0ull
#endif

// the workgroup bitonic sort and the key shuffles: common.hpp (wg_bitonic, shared with box_device.hip)

// Segmented sort of the kd levels whose unfinished segments all hold at most KD_WS_MAX cells:
// one wave per segment (a compact list of segment start groups, dealt round-robin to the
// waves), the segment's keys padded with ~0 to the next power of two P and bitonic-sorted in
// registers — lane l holds elements l + 64 t, t < P / 64 — with no workgroup barrier: the
// partner of a stage j >= 64 is a register of the same lane, of a stage j < 64 the same
// register of lane l ^ j.  The keys of one segment share the segment field, so the order is
// the full sort's (wg_bitonic over all P2 keys: 91 stages and 41 barriers at P2 = 8192 for
// every level, even when the segments hold a few dozen cells).
constexpr int KD_WS_T = 16, KD_WS_MAX = 64 * KD_WS_T;
// branch-free compare-exchange: keep = all ones selects the minimum (u32 / u64 min, max and
// bit selects only: no per-pair lane masks, which held the unrolled stages' SGPRs)
__device__ __forceinline__ unsigned int kd_pick(unsigned int x, unsigned int y, unsigned int keep) {
  const unsigned int mn = x < y ? x : y, mx = x < y ? y : x;
  return (mn & keep) | (mx & ~keep);
}
__device__ __forceinline__ unsigned long long kd_pick(unsigned long long x, unsigned long long y,
                                                      unsigned int keep) {
  const unsigned long long mn = x < y ? x : y, mx = x < y ? y : x;
  const unsigned long long k = (unsigned long long)(int)keep;   // sign-extend: all ones or zero
  return (mn & k) | (mx & ~k);
}
template <typename KT>
__device__ __forceinline__ void kd_cswap(KT& x, KT& y, unsigned int up) {
  const KT a = x, b = y;
  x = kd_pick(a, b, up);
  y = kd_pick(a, b, ~up);
}

// one segment of n <= 64 T keys at sb[lo..], padded to P = 64 T (or 32 when T = 1); T is a
// compile-time register count, so every stage's partner register is static
template <typename KT, int T>
__device__ __forceinline__ void kd_wave_sort_seg(KT* sb, int lo, int n) {
  const int lane = threadIdx.x & 63;
  const int P = T == 1 ? (n <= 32 ? 32 : 64) : 64 * T;
  KT x[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int i = lane + 64 * t;
    x[t] = i < n ? sb[lo + i] : ~(KT)0;
  }
  for (int k = 2, lk = 1; k <= P; k <<= 1, ++lk) {
#pragma unroll
    for (int lj = 4; lj >= 0; --lj) {   // in-lane stages j = 64 tj, descending
      const int tj = 1 << lj;
      if (tj < T && 64 * tj < k) {
#pragma unroll
        for (int t = 0; t < T; ++t)
          if ((t & tj) == 0) kd_cswap(x[t], x[t | tj], ((unsigned int)((lane + 64 * t) & k) >> lk) - 1u);
      }
    }
    for (int j = min(k >> 1, 32), lj2 = min(lk - 1, 5); j > 0; j >>= 1, --lj2) {   // cross-lane stages
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int i = lane + 64 * t;
        const KT y = shfl_xor_key(x[t], j);
        // minimum where bit j of i equals bit k of i (ascending run, lower partner or descending
        // run, upper partner): keep = ((i >> lj) ^ (i >> lk)) & 1 ? 0 : all ones
        const unsigned int keep = (((unsigned int)(i >> lj2) ^ (unsigned int)(i >> lk)) & 1u) - 1u;
        x[t] = kd_pick(x[t], y, keep);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int i = lane + 64 * t;
    if (i < n) sb[lo + i] = x[t];
  }
}

template <typename KT>
__device__ void kd_wave_sort(KT* sb, const int* segl, int nseg, const int* segE, int C) {
  const int wave = threadIdx.x >> 6;
  for (int q = wave; q < nseg; q += KD_THREADS / 64) {
    const int a = segl[q], lo = 16 * a, n = min(16 * segE[a], C) - lo;
    // three register counts (P = 32 / 64, 256, 1024): a fourth and fifth instantiation pushed
    // the kernel past its SGPR budget (spills)
    if (n <= 64) kd_wave_sort_seg<KT, 1>(sb, lo, n);
    else if (n <= 256) kd_wave_sort_seg<KT, 4>(sb, lo, n);
    else kd_wave_sort_seg<KT, KD_WS_T>(sb, lo, n);
  }
}

// Sort-key layouts (segment start group a | order value v | cell), compared as integers: u64
// (a << 40 | v << 16 | cell) in general; u32 (a << 23 | v << 13 | cell) when every field fits —
// cells < 8192, groups < 512, rank values < 1023 — half the LDS and shuffle traffic per sort
// stage and the same order (every field is order-preserving in both layouts).
template <typename KT>
struct KdKey;
template <>
struct KdKey<unsigned long long> {
  static constexpr int CB = 16, AS = 40;
};
template <>
struct KdKey<unsigned int> {
  static constexpr int CB = 13, AS = 23;
};

template <int M, typename KT>
__global__ __launch_bounds__(KD_THREADS) void cells_kd_kernel(int stride, const int* __restrict__ off,
                                                             const int* __restrict__ goff,
                                                             const unsigned long long* __restrict__ keys,
                                                             const double* __restrict__ pts,
                                                             const int* __restrict__ rank0,
                                                             unsigned long long* __restrict__ okeys,
                                                             unsigned short* __restrict__ ork,
                                                             unsigned short* __restrict__ ogb,
                                                             double* __restrict__ osv, int ws_max) {
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char kd_dyn[];
  __shared__ int segS[KD_MAX_GROUPS], segE[KD_MAX_GROUPS];
  __shared__ unsigned int mn[KD_MAX_GROUPS][M], mx[KD_MAX_GROUPS][M];
  __shared__ int segl[KD_MAX_GROUPS];
  __shared__ int sh_any, sh_maxlen, sh_nseg;
  const int s = blockIdx.x, tid = threadIdx.x;
  const int c0 = off[s], C = off[s + 1] - c0;
  const int g0 = goff[s], G = goff[s + 1] - g0;
  constexpr int CB = KdKey<KT>::CB, AS = KdKey<KT>::AS;
  constexpr KT CMASK = ((KT)1 << CB) - 1;
  KT* sb = (KT*)kd_dyn;                                                // P2 sort keys
  int P2 = 16;
  while (P2 < C) P2 <<= 1;
  double* pt = (double*)(kd_dyn + (size_t)P2 * 8);                     // stride x M
  unsigned short* rk = (unsigned short*)(pt + (size_t)stride * M);     // M x stride
  const double* gp = pts + (size_t)s * stride * M;
  const int* gr0 = rank0 + (size_t)s * stride;
  CKD_T(0);
#ifdef EVR_CKD_PROF
  if (tid == 0 && s < 4096)
    for (int k = 2; k < 8; ++k) ckd_prof[16 * s + k] = 0;
#endif
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
  // (an LDS cache of every cell's M ranks instead of this key -> rank0 -> rank-table chain
  // measured the same: 129 vs 130 us of span passes per sample, profiles/r04/w)
  auto rank_of = [&](int cell, int j) -> unsigned int {
    const unsigned long long key = keys[c0 + cell];
    const int p = (j == 0) ? gr0[K::field(key, 0)] : K::field(key, j);
    return rk[j * stride + p];
  };
  for (int g = tid; g < G; g += KD_THREADS) {
    segS[g] = 0;
    segE[g] = G;
  }
  for (int i = tid; i < P2; i += KD_THREADS) sb[i] = (i < C) ? (KT)i : ~(KT)0;
  __syncthreads();
  CKD_T(1);
  // 2. kd levels
  for (int level = 0; level < 32; ++level) {
    unsigned long long ck = CKD_NOW();
    (void)ck;
    if (tid == 0) {
      sh_any = 0;
      sh_maxlen = 0;
      sh_nseg = 0;
    }
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
      if (g == a && (i & 15) == 0) {   // one lane per unfinished segment
        atomicMax(&sh_maxlen, ncell);
        segl[atomicAdd(&sh_nseg, 1)] = a;
      }
      const bool in = i < C;
      const int cell = in ? (int)(sb[i] & CMASK) : 0;
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
    CKD_ACC(2, ck);
    if (!sh_any) break;
    ck = CKD_NOW();
    for (int i = tid; i < C; i += KD_THREADS) {
      const int g = i >> 4, a = segS[g], e = segE[g];
      const int ncell = min(16 * e, C) - 16 * a;
      const int cell = (int)(sb[i] & CMASK);
      KT v;
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
        v = (KT)(i - 16 * a);  // finished segment: keep its order
      }
      sb[i] = ((KT)a << AS) | (v << CB) | (KT)cell;
    }
    __syncthreads();
    CKD_ACC(3, ck);
    ck = CKD_NOW();
    // the levels whose segments fit a wave sort them apart; the first levels sort the whole
    // buffer
    if (sh_maxlen <= ws_max) {
      kd_wave_sort(sb, segl, sh_nseg, segE, C);
      __syncthreads();
    } else {
      wg_bitonic<KT, KD_THREADS>(sb, P2);
    }
    CKD_ACC(4, ck);
    ck = CKD_NOW();
#ifdef EVR_CKD_PROF
    if (tid == 0 && s < 4096) ckd_prof[16 * s + 7] += 1;
#endif
    // split: [a, e) -> [a, a + h), [a + h, e), h = ceil(ncell / 32) groups
    static_assert(KD_MAX_GROUPS <= KD_THREADS, "one group per thread in the split");
    int na = 0, ne = 0;
    if (tid < G) {
      const int g = tid, a = segS[g], e = segE[g];
      const int ncell = min(16 * e, C) - 16 * a;
      na = a;
      ne = e;
      if (ncell > 16) {
        const int h = (ncell + 31) / 32;
        if (g < a + h) ne = a + h;
        else na = a + h;
      }
    }
    __syncthreads();
    if (tid < G) {
      segS[tid] = na;
      segE[tid] = ne;
    }
    __syncthreads();
    CKD_ACC(5, ck);
  }
  // 3. outputs: keys, rank coordinates and group minimum corners
  for (int i = tid; i < G * 16; i += KD_THREADS) {
    const int g = i >> 4, w = i & 15;
    const size_t gg = (size_t)(g0 + g);
    if (i < C) {
      const int cell = (int)(sb[i] & CMASK);
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
  CKD_T(6);
}

}  // namespace evr

using namespace evr;

extern "C" {

#ifdef EVR_CKD_PROF
// profiling builds only: copy the per-sample phase clocks (16 per sample) to the host
int evr_ckd_prof_read(unsigned long long* host, int nsamples) {
  EVR_HIP(hipDeviceSynchronize());
  EVR_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(ckd_prof), sizeof(unsigned long long) * 16 * (size_t)nsamples));
  return 0;
}
#endif

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
  // u32 sort keys when every field fits (KdKey), the u64 layout otherwise (the same order)
  const bool k32 = max_cells < 8192 && stride < 1023;
  const int ws_max = KD_WS_MAX;
#define LK(MM, KT_)                                                                                        \
  do {                                                                                                     \
    EVR_HIP(hipFuncSetAttribute((const void*)cells_kd_kernel<MM, KT_>,                                    \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                    \
    cells_kd_kernel<MM, KT_><<<S, KD_THREADS, lds, s>>>(stride, off, goff, keys, pts, rank0, okeys, ork, ogb, \
                                                        osv, ws_max);                                              \
  } while (0)
#define L(MM)                             \
  do {                                    \
    if (k32) LK(MM, unsigned int);        \
    else LK(MM, unsigned long long);      \
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
#undef LK
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
