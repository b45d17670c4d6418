// Host-side box decomposition of the non-dominated region (exact, or BoTorch's approximate
// partition for alpha > 0), one MC sample per task, parallel over samples with std::thread.
//
// Restates [upstream] BoTorch FastNondominatedPartitioning (alpha = 0, used by BoFire's
// qNEHVI, bofire/strategies/predictives/qnehvi.py:50): local upper bounds U(N) of the
// minimisation problem on z = -g with the incremental update of Lacour, Klamroth & Fonseca
// (2017), Alg. 3, then one disjoint box per local upper bound u:
//     dim 0: (-inf, u_0),  dim j >= 1: [max_{k<j} Z^k_j(u), u_j)
// mapped back to maximisation space (lower = -u, upper = -(box lower)).  Per-sample Pareto
// filtering (is_non_dominated + better-than-ref, _pad_batch_pareto_frontier) is done here too.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <limits>
#include <thread>
#include <vector>

#include "../../include/everest_amd.h"

namespace evr {
void set_error(const char* fmt, ...);
}

struct evr_cells {
  int S = 0, m = 0;
  std::vector<std::vector<double>> lo, hi;  // per sample, C_s x m
};

namespace {

struct LUB {
  int m;
  std::vector<double> U;  // K x m
  std::vector<double> Z;  // K x m x m  (Z[u][k][j]: coordinate j of defining point k)
  size_t K() const { return U.size() / (size_t)m; }
};

void init_lub(LUB& L, const std::vector<double>& R) {
  const int m = L.m;
  L.U.assign(R.begin(), R.end());
  L.Z.assign((size_t)m * m, -std::numeric_limits<double>::infinity());
  for (int j = 0; j < m; ++j) L.Z[(size_t)j * m + j] = R[j];
}

// One incremental update: the bounds strictly dominated by z (u > z in every coordinate)
// are replaced by their admissible projections u^j = (z_j, u_-j).  Removal is
// swap-with-last (the LUB set is unordered), so the cost is O(K m + |A| m^2).
void update_lub(LUB& L, const double* z, std::vector<size_t>& A, std::vector<double>& newU,
                std::vector<double>& newZ) {
  const int m = L.m;
  const size_t mm = (size_t)m * m;
  const size_t K = L.K();
  A.clear();
  for (size_t u = 0; u < K; ++u) {
    const double* uu = &L.U[u * m];
    bool dom = true;
    for (int j = 0; j < m && dom; ++j) dom = uu[j] > z[j];
    if (dom) A.push_back(u);
  }
  if (A.empty()) return;
  newU.clear();
  newZ.clear();
  for (size_t u : A) {
    const double* uu = &L.U[u * m];
    const double* zz = &L.Z[u * mm];
    for (int j = 0; j < m; ++j) {
      double zmax = -std::numeric_limits<double>::infinity();
      for (int k = 0; k < m; ++k)
        if (k != j) zmax = std::max(zmax, zz[(size_t)k * m + j]);
      if (z[j] >= zmax) {
        const size_t base = newU.size();
        newU.insert(newU.end(), uu, uu + m);
        newU[base + j] = z[j];
        const size_t zb = newZ.size();
        newZ.insert(newZ.end(), zz, zz + mm);
        for (int k = 0; k < m; ++k) newZ[zb + (size_t)j * m + k] = z[k];
      }
    }
  }
  // remove A (indices ascending) by swap-with-last, from the back
  size_t Kc = K;
  for (size_t t = A.size(); t-- > 0;) {
    const size_t u = A[t];
    const size_t last = Kc - 1;
    if (u != last) {
      std::copy(&L.U[last * m], &L.U[last * m] + m, &L.U[u * m]);
      std::copy(&L.Z[last * mm], &L.Z[last * mm] + mm, &L.Z[u * mm]);
    }
    --Kc;
  }
  L.U.resize(Kc * m);
  L.Z.resize(Kc * mm);
  L.U.insert(L.U.end(), newU.begin(), newU.end());
  L.Z.insert(L.Z.end(), newZ.begin(), newZ.end());
}

// Approximate partition (alpha > 0, m > 2): [upstream] BoTorch NondominatedPartitioning.
// _partition_space, the binary partitioning of Couckuyt, Deschrijver & Dhaene (2014), in the
// minimisation space z = -g.  Coordinates are indices into the augmented front sorted per
// objective: 0 = the ideal point (per-objective minimum of the front), 1..P = the front in
// ascending (stable) order, P+1 = the reference point.  A cell [l, u] (index pairs) is
//   accepted  if its upper corner is not dominated: every front point p has some j with
//             value(u)_j <= p_j;
//   split     if only its lower corner passes that test (the cell straddles the front), it is
//             wider than one index step in some objective and its volume exceeds alpha times
//             the volume between the ideal and reference points: along the objective of the
//             largest index span, the upper half loses round-half-even(span / 2) steps and the
//             lower half gains the rest;
//   dropped   otherwise (dominated, or straddling but too small: the approximation).
// Accepted cells are reported with index 0 mapped to -inf (upstream get_hypercell_bounds), so
// in maximisation space a cell touching the ideal side is unbounded above.
void approx_cells(int m, const std::vector<double>& Zf, int P, const double* Rn, double alpha,
                  std::vector<double>& lo_tmp, std::vector<double>& hi_tmp) {
  const double inf = std::numeric_limits<double>::infinity();
  // aug[j][k]: k-th smallest augmented value of objective j (k = 0..P+1)
  std::vector<std::vector<double>> aug(m, std::vector<double>(P + 2));
  std::vector<int> ord(P);
  double total = 1.0;
  for (int j = 0; j < m; ++j) {
    for (int i = 0; i < P; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return Zf[a * m + j] < Zf[b * m + j]; });
    for (int k = 0; k < P; ++k) aug[j][k + 1] = Zf[ord[k] * m + j];
    aug[j][0] = P ? aug[j][1] : Rn[j];
    aug[j][P + 1] = Rn[j];
    total *= Rn[j] - aug[j][0];
  }
  auto undominated = [&](const std::vector<int>& c) {   // c: m indices
    for (int i = 0; i < P; ++i) {
      bool some = false;
      for (int j = 0; j < m && !some; ++j) some = aug[j][c[j]] <= Zf[i * m + j];
      if (!some) return false;
    }
    return true;
  };
  auto emit = [&](const std::vector<int>& l, const std::vector<int>& u) {
    bool ok = true;
    const size_t b = lo_tmp.size();
    for (int j = 0; j < m; ++j) {
      const double zl = l[j] == 0 ? -inf : aug[j][l[j]], zu = aug[j][u[j]];
      lo_tmp.push_back(-zu);
      hi_tmp.push_back(-zl);
      ok &= zu > zl;
    }
    if (!ok) {   // empty cell (tied front values): no volume
      lo_tmp.resize(b);
      hi_tmp.resize(b);
    }
  };
  std::vector<std::vector<int>> stack;   // each: 2m indices (lower, upper)
  std::vector<int> cell(2 * m);
  for (int j = 0; j < m; ++j) {
    cell[j] = 0;
    cell[m + j] = P + 1;
  }
  stack.push_back(cell);
  std::vector<int> l(m), u(m);
  while (!stack.empty()) {
    cell = stack.back();
    stack.pop_back();
    for (int j = 0; j < m; ++j) {
      l[j] = cell[j];
      u[j] = cell[m + j];
    }
    if (P == 0 || undominated(u)) {
      emit(l, u);
      continue;
    }
    if (!undominated(l)) continue;
    int longest = 0, span = -1;
    double vol = 1.0;
    for (int j = 0; j < m; ++j) {
      const int dj = u[j] - l[j];
      if (dj > span) {   // first maximum, as torch.max
        span = dj;
        longest = j;
      }
      vol *= aug[j][u[j]] - aug[j][l[j]];
    }
    if (span <= 1 || !(vol / total > alpha)) continue;
    const int h1 = (int)std::nearbyint(span / 2.0), h2 = span - h1;
    std::vector<int> c1 = cell, c2 = cell;
    c1[m + longest] -= h1;
    c2[longest] += h2;
    stack.push_back(std::move(c1));
    stack.push_back(std::move(c2));
  }
}

void decompose_one(int n, int m, const double* obj, long long si, long long sj, const unsigned char* mask,
                   const double* ref, double alpha, std::vector<double>& lo_out, std::vector<double>& hi_out) {
  // candidate points: masked & better than ref
  std::vector<int> cand;
  cand.reserve(n);
  for (int i = 0; i < n; ++i) {
    if (mask && !mask[i]) continue;
    bool better = true;
    for (int j = 0; j < m; ++j) better &= obj[i * si + j * sj] > ref[j];
    if (better) cand.push_back(i);
  }
  // Pareto filter with dedup (first occurrence kept)
  std::vector<int> pts;
  for (size_t a = 0; a < cand.size(); ++a) {
    const int i = cand[a];
    bool nd = true;
    for (size_t bq = 0; bq < cand.size() && nd; ++bq) {
      if (bq == a) continue;
      const int k = cand[bq];
      bool ge = true, gt = false, eq = true;
      for (int j = 0; j < m; ++j) {
        const double v = obj[k * si + j * sj], w = obj[i * si + j * sj];
        ge &= v >= w;
        gt |= v > w;
        eq &= v == w;
      }
      if (ge && gt) nd = false;
      if (eq && bq < a) nd = false;
    }
    if (nd) pts.push_back(i);
  }
  std::vector<double> R(m);
  for (int j = 0; j < m; ++j) R[j] = -ref[j];
  std::vector<double> lo_tmp, hi_tmp;
  if (alpha > 0.0 && m > 2) {
    std::vector<double> Zf(pts.size() * m);
    for (size_t a = 0; a < pts.size(); ++a)
      for (int j = 0; j < m; ++j) Zf[a * m + j] = -obj[pts[a] * si + j * sj];
    approx_cells(m, Zf, (int)pts.size(), R.data(), alpha, lo_tmp, hi_tmp);
  } else {
  LUB L;
  L.m = m;
  init_lub(L, R);
  std::vector<double> nU, nZ, z(m);
  std::vector<size_t> A;
  for (int i : pts) {
    for (int j = 0; j < m; ++j) z[j] = -obj[i * si + j * sj];
    update_lub(L, z.data(), A, nU, nZ);
  }
  const size_t K = L.K();
  lo_tmp.reserve(K * m);
  hi_tmp.reserve(K * m);
  std::vector<double> lw(m), up(m);
  for (size_t u = 0; u < K; ++u) {
    const double* uu = &L.U[u * m];
    const double* zz = &L.Z[u * m * m];
    bool ok = true;
    for (int j = 0; j < m; ++j) {
      double boxlo = -std::numeric_limits<double>::infinity();
      for (int k = 0; k < j; ++k) boxlo = std::max(boxlo, zz[(size_t)k * m + j]);
      lw[j] = -uu[j];
      up[j] = -boxlo;
      ok &= up[j] > lw[j];
    }
    if (!ok) continue;
    lo_tmp.insert(lo_tmp.end(), lw.begin(), lw.end());
    hi_tmp.insert(hi_tmp.end(), up.begin(), up.end());
  }
  }
  // Cells sorted by their first lower bound (ties: remaining coordinates) so that a device
  // thread's neighbouring cells share a tight lower envelope (tile skip test in hvi.hip).
  const size_t C = lo_tmp.size() / m;
  std::vector<size_t> order(C);
  for (size_t i = 0; i < C; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    for (int j = 0; j < m; ++j) {
      const double x = lo_tmp[a * m + j], y = lo_tmp[b * m + j];
      if (x != y) return x < y;
    }
    return a < b;
  });
  lo_out.resize(C * m);
  hi_out.resize(C * m);
  for (size_t i = 0; i < C; ++i) {
    std::copy(&lo_tmp[order[i] * m], &lo_tmp[order[i] * m] + m, &lo_out[i * m]);
    std::copy(&hi_tmp[order[i] * m], &hi_tmp[order[i] * m] + m, &hi_out[i * m]);
  }
}

}  // namespace

extern "C" {

int evr_box_decompose(int S, int n, int m, const double* obj, long long ss, long long si, long long sj,
                      const unsigned char* mask, const double* ref, int num_threads, evr_cells** out) {
  return evr_box_decompose_approx(S, n, m, obj, ss, si, sj, mask, ref, 0.0, num_threads, out);
}

int evr_box_decompose_approx(int S, int n, int m, const double* obj, long long ss, long long si, long long sj,
                             const unsigned char* mask, const double* ref, double alpha, int num_threads,
                             evr_cells** out) {
  if (!out || !obj || !ref || S < 1 || n < 0 || m < 1 || !(alpha >= 0.0 && alpha < std::numeric_limits<double>::infinity())) {
    evr::set_error("evr_box_decompose: bad arguments");
    return 2;
  }
  evr_cells* c = new evr_cells();
  c->S = S;
  c->m = m;
  c->lo.resize(S);
  c->hi.resize(S);
  int T = num_threads > 0 ? num_threads : (int)std::thread::hardware_concurrency();
  T = std::max(1, std::min(T, S));
  std::atomic<int> next(0);
  auto work = [&]() {
    for (;;) {
      const int s = next.fetch_add(1);
      if (s >= S) break;
      decompose_one(n, m, obj + (size_t)s * ss, si, sj, mask ? mask + (size_t)s * n : nullptr, ref, alpha, c->lo[s],
                    c->hi[s]);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  *out = c;
  return 0;
}

long long evr_cells_total(const evr_cells* c) {
  long long t = 0;
  for (int s = 0; s < c->S; ++s) t += (long long)(c->lo[s].size() / c->m);
  return t;
}

int evr_cells_copy(const evr_cells* c, double* lo, double* hi, int* off) {
  long long pos = 0;
  for (int s = 0; s < c->S; ++s) {
    off[s] = (int)pos;
    const size_t cnt = c->lo[s].size();
    std::copy(c->lo[s].begin(), c->lo[s].end(), lo + pos * c->m);
    std::copy(c->hi[s].begin(), c->hi[s].end(), hi + pos * c->m);
    pos += (long long)(cnt / c->m);
  }
  off[c->S] = (int)pos;
  return 0;
}

void evr_cells_free(evr_cells* c) { delete c; }

}  // extern "C"
