// Exact box decomposition of the non-dominated region on the device, one workgroup per
// Monte-Carlo sample (S = 256..512 samples fill the 256 CUs).
//
// Same mathematics as box_decomposition.cpp (the host restatement of [upstream] BoTorch
// FastNondominatedPartitioning, alpha = 0, used by BoFire's qNEHVI at
// bofire/strategies/predictives/qnehvi.py:50): local upper bounds (LUBs) of the
// minimisation problem on z = -g, incremental update of Lacour, Klamroth & Fonseca (2017)
// over the sample's Pareto points in index order, one disjoint box per LUB.
//
// MI355X-first representation.  A LUB u is fully determined by its defining points
// Z^k(u), k = 0..m-1 (u_k = Z^k_k(u)), so the whole LUB is ONE 64-bit key of m point
// indices (12 bits each for m <= 5).  The sample's points live in LDS; the LUB keys in
// HBM (per-sample slab).  Field 0 holds the rank of Z^0 in descending z_0 order instead of
// the index, so sorting the keys sorts the cells by their first lower bound — the order
// the HVI tile-skip test wants — and, keys being unique, the final cell order is
// deterministic even though the LUB slab is updated with LDS atomics.
//
// Per Pareto point z:  (a) scan the slab, collect A = {u : u > z strictly};  (b) for every
// (u in A, j) test z_j >= max_{k != j} Z^k_j(u) and emit u^j = (z_j, u_-j) with Z^j = z;
// (c) new keys overwrite A's slots, the rest append (holes are tombstoned and compacted
// when they pile up).  Then every live LUB's box is tested non-empty and its key emitted;
// keys are bitonic-sorted (LDS when they fit, else in the HBM slab) and packed per sample;
// the HVI scan decodes them against the sample's point table (hvi.hip).
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int BD_THREADS = 1024;
constexpr unsigned long long BD_DEAD = ~0ull;
constexpr int BD_LDS_BYTES = 160 * 1024 - 2048;  // dynamic LDS budget (static counters aside)
constexpr int BD_STG = 256;                       // LDS staging of A's indices and the new keys

struct BdLayout {
  // per-sample slabs (elements): lub, buf: cap u64; aidx: cap int; pts: (n+m)*m double; inv0: n+m int
  long long cap;
  int n, m;
  size_t off_lub, off_buf, off_aidx, off_pts, off_inv0, off_nf, bytes;
};

static BdLayout bd_layout(int S, int n, int m, int cap) {
  BdLayout L;
  L.cap = cap;
  L.n = n;
  L.m = m;
  size_t o = 0;
  auto take = [&](size_t b) {
    size_t r = o;
    o += (b + 255) & ~(size_t)255;
    return r;
  };
  L.off_lub = take(sizeof(unsigned long long) * (size_t)S * cap);
  L.off_buf = take(sizeof(unsigned long long) * (size_t)S * cap);
  L.off_aidx = take(sizeof(int) * (size_t)S * cap);
  L.off_pts = take(sizeof(double) * (size_t)S * (n + m) * m);
  L.off_inv0 = take(sizeof(int) * (size_t)S * (n + m));
  L.off_nf = take(sizeof(int) * (size_t)S);
  L.bytes = o;
  return L;
}

// LDS bytes for the points (raw + filtered), flags, inverse rank table.
static size_t bd_lds_fixed(int n, int m) {
  return sizeof(double) * ((size_t)n * m + (size_t)(n + m) * m) + sizeof(int) * (size_t)(4 * n + 2 * m + 8);
}

// Bitonic sort (ascending) of P2 keys in `a` (LDS or global), all threads of the block.
template <typename Ptr>
__device__ void bd_bitonic(Ptr a, int P2) {
  for (int k = 2; k <= P2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P2; i += BD_THREADS) {
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
  }
}

// LS: the whole LUB slab (cap keys) lives in LDS, in the final sort buffer, and the first
// BD_STG entries of A's index list and of the new keys of a step in an LDS staging area, so a
// Pareto point's update makes no global round trip until BD_STG is exceeded (the slab in HBM
// cost three dependent L2 round trips per point: ~1.15 ms for 256 samples at the bench shape).
template <int M, bool LS>
__global__ __launch_bounds__(BD_THREADS) void bd_build_kernel(int S, int n, const double* __restrict__ obj,
                                                              const double* __restrict__ ref, int cap, int sortcap,
                                                              unsigned char* __restrict__ ws, BdLayout Lo,
                                                              int* __restrict__ counts, int* __restrict__ status,
                                                              int* hmap) {
  using K = CellKey<M>;
  extern __shared__ __align__(16) unsigned char smem[];
  const int s = blockIdx.x, tid = threadIdx.x;
  double* raw = (double*)smem;                  // n x M   (min-space, all points)
  double* pt = raw + (size_t)n * M;             // (n+M) x M filtered points then dummies
  int* flag = (int*)(pt + (size_t)(n + M) * M); // n
  int* pos = flag + n;                          // n
  int* inv0 = pos + n;                          // n + M: point index of rank r
  int* rank = inv0 + n + M;                     // n + M: rank of point index i
  unsigned long long* sbuf = (unsigned long long*)(((uintptr_t)(rank + n + M) + 15) & ~(uintptr_t)15);
  unsigned long long* stg = sbuf + sortcap;     // LS: BD_STG new keys
  int* astg = (int*)(stg + BD_STG);             // LS: BD_STG indices of A
  __shared__ int sh_nf, sh_nA, sh_nNew, sh_cnt, sh_err;

  unsigned long long* lub = LS ? sbuf : (unsigned long long*)(ws + Lo.off_lub) + (size_t)s * cap;
  unsigned long long* buf = (unsigned long long*)(ws + Lo.off_buf) + (size_t)s * cap;
  int* aidx = (int*)(ws + Lo.off_aidx) + (size_t)s * cap;
  double* gpts = (double*)(ws + Lo.off_pts) + (size_t)s * (n + M) * M;
  int* ginv0 = (int*)(ws + Lo.off_inv0) + (size_t)s * (n + M);

  // ---- 1. load, better-than-ref + Pareto filter with dedup (first occurrence kept) --------
  for (int e = tid; e < n * M; e += BD_THREADS) {
    const int i = e / M, j = e - i * M;
    raw[e] = -obj[((size_t)j * n + i) * S + s];
  }
  if (tid == 0) sh_err = 0;
  __syncthreads();
  for (int i = tid; i < n; i += BD_THREADS) {
    bool keep = true;
#pragma unroll
    for (int j = 0; j < M; ++j) keep &= raw[i * M + j] < -ref[j];  // g > ref  <=>  z < -ref
    for (int k = 0; k < n && keep; ++k) {
      if (k == i) continue;
      bool cand = true, le = true, lt = false, eq = true;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const double v = raw[k * M + j], w = raw[i * M + j];
        cand &= v < -ref[j];
        le &= v <= w;
        lt |= v < w;
        eq &= v == w;
      }
      if (cand && ((le && lt) || (eq && k < i))) keep = false;
    }
    flag[i] = keep ? 1 : 0;
  }
  __syncthreads();
  if (tid == 0) {  // ordered compaction (n is small; one thread keeps index order)
    int c = 0;
    for (int i = 0; i < n; ++i) {
      pos[i] = c;
      c += flag[i];
    }
    sh_nf = c;
  }
  __syncthreads();
  const int nf = sh_nf;
  for (int e = tid; e < n * M; e += BD_THREADS) {
    const int i = e / M;
    if (flag[i]) pt[pos[i] * M + (e - i * M)] = raw[e];
  }
  for (int e = tid; e < M * M; e += BD_THREADS) {  // dummies D_k: R_k at k, -inf elsewhere
    const int k = e / M, j = e - k * M;
    pt[(nf + k) * M + j] = (j == k) ? -ref[k] : -INFINITY;
  }
  __syncthreads();
  // rank of every point (and D_0) in descending z_0 (ties: index order); inv0[rank] = index
  for (int i = tid; i <= nf; i += BD_THREADS) {
    const double v = pt[i * M];
    int r = 0;
    for (int k = 0; k <= nf; ++k) {
      const double w = pt[k * M];
      r += (w > v) || (w == v && k < i);
    }
    inv0[r] = i;
    rank[i] = r;
  }
  __syncthreads();

  // ---- 2. incremental LUB update ------------------------------------------------------
  int Kend = 1, holes = 0;
  if (tid == 0) {
    unsigned long long k0 = 0;
    k0 = K::set(k0, 0, rank[nf]);  // rank of D_0
    for (int j = 1; j < M; ++j) k0 = K::set(k0, j, nf + j);
    lub[0] = k0;
  }
  __syncthreads();
  for (int p = 0; p < nf; ++p) {
    double z[M];
#pragma unroll
    for (int j = 0; j < M; ++j) z[j] = pt[p * M + j];
    if (tid == 0) {
      sh_nA = 0;
      sh_nNew = 0;
    }
    __syncthreads();
    // (a) LUBs strictly above z
    for (int u = tid; u < Kend; u += BD_THREADS) {
      const unsigned long long key = lub[u];
      if (key == BD_DEAD) continue;
      bool dom = pt[inv0[K::field(key, 0)] * M] > z[0];
#pragma unroll
      for (int j = 1; j < M; ++j) dom &= pt[K::field(key, j) * M + j] > z[j];
      if (dom) {
        const int k = atomicAdd(&sh_nA, 1);
        if (LS && k < BD_STG) astg[k] = u;
        else aidx[k] = u;
      }
    }
    __syncthreads();
    const int nA = sh_nA;
    // (b) admissible projections u^j
    for (int t = tid; t < nA * M; t += BD_THREADS) {
      const int a = t / M, j = t - a * M;
      const unsigned long long key = lub[(LS && a < BD_STG) ? astg[a] : aidx[a]];
      double zmax = -INFINITY;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        if (k == j) continue;
        const int pk = (k == 0) ? inv0[K::field(key, 0)] : K::field(key, k);
        zmax = fmax(zmax, pt[pk * M + j]);
      }
      if (z[j] >= zmax) {
        const int slot = atomicAdd(&sh_nNew, 1);
        if (slot < cap) {
          const unsigned long long nk = K::set(key, j, j == 0 ? rank[p] : p);
          if (LS && slot < BD_STG) stg[slot] = nk;
          else buf[slot] = nk;
        }
      }
    }
    __syncthreads();
    const int nNew = sh_nNew;
    if (Kend + (nNew > nA ? nNew - nA : 0) > cap || nNew > cap) {
      if (tid == 0) sh_err = 1;
      break;
    }
    // (c) overwrite A's slots, append the rest, tombstone the leftovers
    const int top = nNew > nA ? nNew : nA;
    for (int i = tid; i < top; i += BD_THREADS) {
      const bool st = LS && i < BD_STG;
      if (i < nNew) {
        const int dst = (i < nA) ? (st ? astg[i] : aidx[i]) : Kend + (i - nA);
        lub[dst] = st ? stg[i] : buf[i];
      } else {
        lub[st ? astg[i] : aidx[i]] = BD_DEAD;
      }
    }
    if (nNew > nA) Kend += nNew - nA;
    else holes += nA - nNew;
    __syncthreads();
    if (holes > 256 && holes * 4 > Kend) {  // compact (order is irrelevant: keys are sorted at the end)
      if (tid == 0) sh_cnt = 0;
      __syncthreads();
      for (int u = tid; u < Kend; u += BD_THREADS) {
        const unsigned long long key = lub[u];
        if (key != BD_DEAD) buf[atomicAdd(&sh_cnt, 1)] = key;
      }
      __syncthreads();
      const int cnt = sh_cnt;
      for (int u = tid; u < cnt; u += BD_THREADS) lub[u] = buf[u];
      Kend = cnt;
      holes = 0;
      __syncthreads();
    }
  }
  __syncthreads();
  if (sh_err) {
    if (tid == 0) {
      status[s] = 1;
      counts[s] = 0;
      if (hmap) {   // the host's mapped copy (evr_box_kd_pipeline): visible at the kernel's end
        hmap[s] = 0;
        hmap[S + s] = 1;
      }
    }
    return;
  }

  // ---- 3. non-empty boxes -> keys, sorted ---------------------------------------------
  if (tid == 0) sh_cnt = 0;
  __syncthreads();
  for (int u = tid; u < Kend; u += BD_THREADS) {
    const unsigned long long key = lub[u];
    if (key == BD_DEAD) continue;
    int P[M];
    P[0] = inv0[K::field(key, 0)];
#pragma unroll
    for (int j = 1; j < M; ++j) P[j] = K::field(key, j);
    bool ok = true;
#pragma unroll
    for (int j = 1; j < M; ++j) {  // box in min-space: [max_{k<j} Z^k_j, u_j); dim 0 unbounded below
      double lo = -INFINITY;
#pragma unroll
      for (int k = 0; k < j; ++k) lo = fmax(lo, pt[P[k] * M + j]);
      ok &= pt[P[j] * M + j] > lo;
    }
    if (ok) buf[atomicAdd(&sh_cnt, 1)] = key;
  }
  __syncthreads();
  const int C = sh_cnt;
  int P2 = 1;
  while (P2 < C) P2 <<= 1;
  if (P2 <= sortcap) {
    for (int i = tid; i < P2; i += BD_THREADS) sbuf[i] = (i < C) ? buf[i] : BD_DEAD;
    __syncthreads();
    wg_bitonic<unsigned long long, BD_THREADS>(sbuf, P2);   // in-wave stages by shuffles (41 barriers, not 91)
    for (int i = tid; i < C; i += BD_THREADS) buf[i] = sbuf[i];
  } else {
    for (int i = C + tid; i < P2; i += BD_THREADS) buf[i] = BD_DEAD;  // P2 <= cap (cap is a power of 2)
    __syncthreads();
    bd_bitonic(buf, P2);
  }
  // points + decode table for the pack kernel
  for (int e = tid; e < (nf + M) * M; e += BD_THREADS) gpts[e] = pt[e];
  for (int r = tid; r <= nf; r += BD_THREADS) ginv0[r] = inv0[r];
  if (tid == 0) {
    counts[s] = C;
    status[s] = 0;
    ((int*)(ws + Lo.off_nf))[s] = nf;
    if (hmap) {
      hmap[s] = C;
      hmap[S + s] = 0;
    }
  }
}

// explicit cells from compressed ones: cell off[s] + i of sample s -> lo / hi rows
template <int M>
__global__ __launch_bounds__(256) void cells_from_keys_kernel(int stride, const int* __restrict__ off,
                                                              const unsigned long long* __restrict__ keys,
                                                              const double* __restrict__ pts,
                                                              const int* __restrict__ rank0, double* __restrict__ lo,
                                                              double* __restrict__ hi) {
  using K = CellKey<M>;
  const int s = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int c0 = off[s], C = off[s + 1] - c0;
  if (i >= C) return;
  double l[M], h[M];
  K::decode(keys[c0 + i], pts + (size_t)s * stride * M, rank0 + (size_t)s * stride, l, h);
  const size_t o = (size_t)(c0 + i) * M;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    lo[o + j] = l[j];
    hi[o + j] = h[j];
  }
}

// compressed cells for the HVI scan: sorted keys packed at off[s], plus the point tables
template <int M>
__global__ __launch_bounds__(256) void bd_pack_keys_kernel(int S, int n, int cap, const unsigned char* __restrict__ ws,
                                                           BdLayout Lo, const int* __restrict__ off,
                                                           unsigned long long* __restrict__ keys,
                                                           double* __restrict__ pts, int* __restrict__ rank0) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int c0 = off[s], C = off[s + 1] - c0;
  if (i < C) keys[c0 + i] = ((const unsigned long long*)(ws + Lo.off_buf))[(size_t)s * cap + i];
  if (blockIdx.x == 0) {
    const size_t np = (size_t)(n + M);
    const double* gp = (const double*)(ws + Lo.off_pts) + s * np * M;
    const int* gi = (const int*)(ws + Lo.off_inv0) + s * np;
    // rows past the nf Pareto points + M dummies are unused: +inf (never a lower bound, and a
    // well-defined rank for the kd ordering of cells_kd.hip)
    const size_t nv = (size_t)((const int*)(ws + Lo.off_nf))[s] + M;
    for (size_t e = threadIdx.x; e < np * M; e += 256) pts[s * np * M + e] = e < nv * M ? gp[e] : INFINITY;
    for (size_t e = threadIdx.x; e < np; e += 256) rank0[s * np + e] = e + M <= nv ? gi[e] : 0;  // ranks 0..nf
  }
}

}  // namespace evr

using namespace evr;

#define EVR_BD_SWITCH(m, MACRO)                                                       \
  switch (m) {                                                                        \
    case 1: MACRO(1); break;                                                          \
    case 2: MACRO(2); break;                                                          \
    case 3: MACRO(3); break;                                                          \
    case 4: MACRO(4); break;                                                          \
    case 5: MACRO(5); break;                                                          \
    case 6: MACRO(6); break;                                                          \
    case 7: MACRO(7); break;                                                          \
    case 8: MACRO(8); break;                                                          \
    default: EVR_CHECK(false, "box decomposition: m=%d not supported (1..8)", m);     \
  }

extern "C" {

int evr_box_device_limits(int n, int m, int* max_points_out, long long* lds_bytes_out) {
  EVR_CHECK(m >= 1 && m <= 8 && n >= 0, "evr_box_device_limits: bad arguments");
  const long long idx_limit = (1ll << bd_field_bits(m)) - 2 - m;   // field values < 2^FB - 1
  const size_t fixed = bd_lds_fixed(n, m);
  if (max_points_out) *max_points_out = (int)std::min<long long>(idx_limit, 1 << 20);
  if (lds_bytes_out) *lds_bytes_out = (long long)fixed;
  return (n <= idx_limit && fixed + 16 + 8 * 64 <= (size_t)BD_LDS_BYTES) ? 0 : 3;
}

long long evr_box_device_workspace_bytes(int S, int n, int m, int cap) {
  if (S < 1 || n < 0 || m < 1 || cap < 1) return 0;
  return (long long)bd_layout(S, n, m, cap).bytes;
}

static int box_decompose_launch(void* stream, int S, int n, int m, const double* obj, const double* ref, int cap,
                                void* work, int* counts, int* status, int* hmap);

int evr_box_decompose_device(void* stream, int S, int n, int m, const double* obj, const double* ref, int cap,
                             void* work, int* counts, int* status) {
  return box_decompose_launch(stream, S, n, m, obj, ref, cap, work, counts, status, nullptr);
}

// hmap: optional device pointer of mapped host memory receiving [counts S | status S]
static int box_decompose_launch(void* stream, int S, int n, int m, const double* obj, const double* ref, int cap,
                                void* work, int* counts, int* status, int* hmap) {
  EVR_CHECK(S >= 1 && n >= 1 && m >= 1 && m <= 8 && obj && ref && work && counts && status,
            "evr_box_decompose_device: bad arguments");
  EVR_CHECK(cap >= 2 && (cap & (cap - 1)) == 0, "evr_box_decompose_device: cap must be a power of two");
  EVR_CHECK(evr_box_device_limits(n, m, nullptr, nullptr) == 0,
            "evr_box_decompose_device: n=%d points x m=%d exceed the device limits", n, m);
  const BdLayout Lo = bd_layout(S, n, m, cap);
  const size_t fixed = bd_lds_fixed(n, m) + 16;
  auto sort_cap = [&](size_t fx) {
    int c = 1;
    while ((size_t)(c * 2) * 8 + fx <= (size_t)BD_LDS_BYTES && c * 2 <= cap) c *= 2;
    return c;
  };
  // the LDS slab variant when the whole capacity fits beside the staging area (EVR_BD_LDS=0: HBM slab)
  const size_t fixed_ls = fixed + (size_t)BD_STG * (8 + 4);
  const char* ev = std::getenv("EVR_BD_LDS");
  const bool ls = sort_cap(fixed_ls) >= cap && !(ev && ev[0] == '0');
  const int sortcap = ls ? cap : sort_cap(fixed);
  const size_t lds = (ls ? fixed_ls : fixed) + (size_t)sortcap * 8;
  hipStream_t s = (hipStream_t)stream;
#define L2(MM, LS_)                                                                                          \
  do {                                                                                                       \
    EVR_HIP(hipFuncSetAttribute((const void*)bd_build_kernel<MM, LS_>,                                      \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                      \
    bd_build_kernel<MM, LS_><<<S, BD_THREADS, lds, s>>>(S, n, obj, ref, cap, sortcap, (unsigned char*)work, \
                                                        Lo, counts, status, hmap);                           \
  } while (0)
#define L(MM)            \
  if (ls) L2(MM, true);  \
  else L2(MM, false)
  EVR_BD_SWITCH(m, L);
#undef L
#undef L2
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_cells_from_keys(void* stream, int S, int m, int stride, const int* off, int max_cells,
                        const unsigned long long* keys, const double* pts, const int* rank0, double* lo,
                        double* hi) {
  EVR_CHECK(S >= 1 && m >= 1 && m <= 8 && stride > m && off && keys && pts && rank0 && lo && hi,
            "evr_cells_from_keys: bad arguments");
  if (max_cells <= 0) return 0;
  dim3 grid(cdiv(max_cells, 256), S);
  hipStream_t s = (hipStream_t)stream;
#define L(MM) cells_from_keys_kernel<MM><<<grid, 256, 0, s>>>(stride, off, keys, pts, rank0, lo, hi)
  EVR_BD_SWITCH(m, L);
#undef L
  EVR_LAUNCH_CHECK();
  return 0;
}

int evr_box_pack_keys_device(void* stream, int S, int n, int m, int cap, const void* work, const int* off,
                             int max_cells, unsigned long long* keys, double* pts, int* rank0) {
  EVR_CHECK(S >= 1 && n >= 1 && m >= 1 && m <= 8 && work && off && keys && pts && rank0,
            "evr_box_pack_keys_device: bad arguments");
  const BdLayout Lo = bd_layout(S, n, m, cap);
  dim3 grid(std::max(1, cdiv(max_cells, 256)), S);
  hipStream_t s = (hipStream_t)stream;
#define L(MM) \
  bd_pack_keys_kernel<MM><<<grid, 256, 0, s>>>(S, n, cap, (const unsigned char*)work, Lo, off, keys, pts, rank0)
  EVR_BD_SWITCH(m, L);
#undef L
  EVR_LAUNCH_CHECK();
  return 0;
}


// The device box decomposition, its packing and the kd ordering in one host call (the box
// worker thread of acquisition._decompose_async): bd_build, the per-sample counts to pinned
// host memory (the one synchronisation), the cell / group offsets formed on the host and sent
// back from the same pinned staging, then the pack and kd launches — no Python, hence no GIL
// hand-over, between the kernels (the Python sequence left ≈ 0.25 ms between bd_build and the
// pack launch, profiles/r04/z).  Outputs are sized by the caller for the capacity: keys S cap,
// okeys 16 (S cap / 16 + S), ork 16 m (S cap / 16 + S), ogb 8 (S cap / 16 + S).  want_kd: 0
// no kd, 1 kd when evr_cells_kd_limits accepts the counts.  info[0] = 1 when a sample overflowed
// cap (nothing packed: rerun with a larger cap), info[1] = 1 when the kd order was built,
// info[2] = the largest per-sample cell count; counts_host[s] = cells of sample s.
int evr_box_kd_pipeline(void* stream, int S, int n, int m, const double* obj, const double* ref, int cap,
                        void* work, int* counts_dev, int* status_dev, int* off_dev, int* goff_dev,
                        unsigned long long* keys, double* pts, int* rank0, int want_kd, unsigned long long* okeys,
                        unsigned short* ork, unsigned short* ogb, double* osv, int* counts_host, int* info) {
  EVR_CHECK(S >= 1 && counts_dev && status_dev && off_dev && goff_dev && keys && pts && rank0 && counts_host &&
                info && (!want_kd || (okeys && ork && ogb && osv)),
            "evr_box_kd_pipeline: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  // staging per thread in mapped, coherent host memory: bd_build writes [counts S | status S]
  // there itself (no read-back copy); [off S+1 | goff S+1] are read from it by the pack and kd
  // kernels and copied to the device arrays after them
  thread_local int* stage = nullptr;
  thread_local int* stage_d = nullptr;
  thread_local size_t stage_n = 0;
  thread_local int stage_dev = -1;
  // the previous call's kernels and copies read the staging on their own stream: an event
  // recorded after them is waited on before the staging is reused, reallocated or freed
  thread_local hipEvent_t copied = nullptr;
  if (copied) EVR_HIP(hipEventSynchronize(copied));
  int dev = 0;
  EVR_HIP(hipGetDevice(&dev));
  const size_t need = (size_t)4 * S + 2;
  if (stage_n < need || stage_dev != dev) {
    // the staging, its device pointer and the event belong to the device current when they
    // were made (one worker thread serves every device)
    if (copied) {
      (void)hipEventDestroy(copied);
      copied = nullptr;
    }
    if (stage) (void)hipHostFree(stage);
    stage = stage_d = nullptr;
    stage_n = 0;
    stage_dev = -1;
    EVR_HIP(hipHostMalloc((void**)&stage, sizeof(int) * need, hipHostMallocMapped | hipHostMallocCoherent));
    EVR_HIP(hipHostGetDevicePointer((void**)&stage_d, stage, 0));
    stage_n = need;
    stage_dev = dev;
  }
  if (!copied) EVR_HIP(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  int* hc = stage;
  int* hs = stage + S;
  int* hoff = stage + 2 * S;
  int* hgoff = hoff + S + 1;
  if (int rc = box_decompose_launch(stream, S, n, m, obj, ref, cap, work, counts_dev, status_dev, stage_d)) return rc;
  EVR_HIP(hipStreamSynchronize(s));
  info[0] = info[1] = info[2] = 0;
  int maxc = 0;
  for (int i = 0; i < S; ++i) {
    counts_host[i] = hc[i];
    if (hs[i]) info[0] = 1;
    maxc = std::max(maxc, hc[i]);
  }
  info[2] = maxc;
  if (info[0]) return 0;
  long long c = 0, g = 0;
  for (int i = 0; i < S; ++i) {
    hoff[i] = (int)c;
    hgoff[i] = (int)g;
    c += hc[i];
    g += (hc[i] + 15) / 16;
  }
  hoff[S] = (int)c;
  hgoff[S] = (int)g;
  EVR_CHECK(c <= (long long)S * cap && c < 0x7FFFFFFFLL, "evr_box_kd_pipeline: %lld cells exceed the capacity", c);
  // the pack and kd kernels read the offsets straight from the mapped staging (a few reads
  // per workgroup); the device copies the acquisition keeps follow them on the stream (blit
  // copies ahead of the kernels queued behind the other stream's work: ≈ 0.13 ms, r04ze)
  const int* moff = stage_d + 2 * S;
  const int* mgoff = moff + S + 1;
  if (int rc = evr_box_pack_keys_device(stream, S, n, m, cap, work, moff, maxc, keys, pts, rank0)) return rc;
  const int stride = n + m;
  if (want_kd && evr_cells_kd_limits(stride, m, maxc, nullptr) == 0) {
    if (int rc = evr_cells_kd_order_device(stream, S, m, stride, moff, mgoff, maxc, keys, pts, rank0, okeys, ork,
                                           ogb, osv))
      return rc;
    info[1] = 1;
  }
  EVR_HIP(hipMemcpyAsync(off_dev, hoff, sizeof(int) * (S + 1), hipMemcpyHostToDevice, s));
  EVR_HIP(hipMemcpyAsync(goff_dev, hgoff, sizeof(int) * (S + 1), hipMemcpyHostToDevice, s));
  EVR_HIP(hipEventRecord(copied, s));
  return 0;
}

}  // extern "C"
