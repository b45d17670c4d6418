// Native L-BFGS-B — see lbfgsb.hpp for what is restated and from where.
#include "lbfgsb.hpp"

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <new>
#include <utility>

#include "../../include/everest_amd.h"

namespace evr {

void set_error(const char* fmt, ...);

#define LB_CHECK(cond, msg)      \
  do {                           \
    if (!(cond)) {               \
      ::evr::set_error("%s", msg); \
      return 2;                  \
    }                            \
  } while (0)

namespace {

// Dense LU with partial pivoting of a k x k row-major matrix (k <= 2m = 20).
bool lu_factor(std::vector<double>& a, std::vector<int>& piv, int k) {
  piv.resize(k);
  for (int c = 0; c < k; ++c) {
    int p = c;
    double best = std::fabs(a[c * k + c]);
    for (int r = c + 1; r < k; ++r) {
      const double v = std::fabs(a[r * k + c]);
      if (v > best) best = v, p = r;
    }
    if (!(best > 0.0) || !std::isfinite(best)) return false;
    piv[c] = p;
    if (p != c)
      for (int j = 0; j < k; ++j) std::swap(a[c * k + j], a[p * k + j]);
    const double inv = 1.0 / a[c * k + c];
    for (int r = c + 1; r < k; ++r) {
      const double f = a[r * k + c] * inv;
      a[r * k + c] = f;
      if (f != 0.0)
        for (int j = c + 1; j < k; ++j) a[r * k + j] -= f * a[c * k + j];
    }
  }
  return true;
}

void lu_solve(const std::vector<double>& a, const std::vector<int>& piv, int k, double* b) {
  for (int c = 0; c < k; ++c)
    if (piv[c] != c) std::swap(b[c], b[piv[c]]);
  for (int r = 1; r < k; ++r) {
    double s = b[r];
    for (int j = 0; j < r; ++j) s -= a[r * k + j] * b[j];
    b[r] = s;
  }
  for (int r = k - 1; r >= 0; --r) {
    double s = b[r];
    for (int j = r + 1; j < k; ++j) s -= a[r * k + j] * b[j];
    b[r] = s / a[r * k + r];
  }
}

double dot(const double* a, const double* b, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

// four interleaved partial sums (vectorisable), combined in a fixed order
double dot4(const double* a, const double* b, int n) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int i = 0;
  for (; i + 3 < n; i += 4) {
    s0 += a[i] * b[i];
    s1 += a[i + 1] * b[i + 1];
    s2 += a[i + 2] * b[i + 2];
    s3 += a[i + 3] * b[i + 3];
  }
  for (; i < n; ++i) s0 += a[i] * b[i];
  return (s0 + s1) + (s2 + s3);
}

// The subspace step's W_F^T r and symmetric W_F^T W_F (k x k, rows of W_F contiguous, length
// n): every entry is dot4's arithmetic exactly (the four interleaved partial sums, the scalar
// tail into the first, (s0 + s1) + (s2 + s3)), so results do not depend on the path taken.
// gram[i * k + j] for j >= i only.
void gram_base(const double* W, int k, int n, const double* r, double* wv, double* gram) {
  for (int i = 0; i < k; ++i) {
    const double* wi = W + (size_t)i * n;
    wv[i] = dot4(wi, r, n);
    for (int j = i; j < k; ++j) gram[(size_t)i * k + j] = dot4(wi, W + (size_t)j * n, n);
  }
}

// AVX2 clone (no FMA, so no contraction: the same roundings as dot4): one 4-lane register per
// dot holds (s0, s1, s2, s3); row i is loaded once per block of four columns.
__attribute__((target("avx2"))) inline double gram_finish(__m256d acc, const double* a, const double* b, int n4,
                                                          int n) {
  alignas(32) double l[4];
  _mm256_store_pd(l, acc);
  for (int t = n4; t < n; ++t) l[0] += a[t] * b[t];
  return (l[0] + l[1]) + (l[2] + l[3]);
}

__attribute__((target("avx2"))) void gram_avx2(const double* W, int k, int n, const double* r, double* wv,
                                               double* gram) {
  const int n4 = n & ~3;
  auto finish = [n4, n](__m256d acc, const double* a, const double* b) __attribute__((target("avx2"))) {
    return gram_finish(acc, a, b, n4, n);
  };
  for (int i = 0; i < k; ++i) {
    const double* wi = W + (size_t)i * n;
    {
      __m256d acc = _mm256_setzero_pd();
      for (int t = 0; t < n4; t += 4) acc = _mm256_add_pd(acc, _mm256_mul_pd(_mm256_loadu_pd(wi + t), _mm256_loadu_pd(r + t)));
      wv[i] = finish(acc, wi, r);
    }
    int j = i;
    for (; j + 3 < k; j += 4) {
      const double* b0 = W + (size_t)j * n;
      const double* b1 = b0 + n;
      const double* b2 = b1 + n;
      const double* b3 = b2 + n;
      __m256d a0 = _mm256_setzero_pd(), a1 = a0, a2 = a0, a3 = a0;
      for (int t = 0; t < n4; t += 4) {
        const __m256d x = _mm256_loadu_pd(wi + t);
        a0 = _mm256_add_pd(a0, _mm256_mul_pd(x, _mm256_loadu_pd(b0 + t)));
        a1 = _mm256_add_pd(a1, _mm256_mul_pd(x, _mm256_loadu_pd(b1 + t)));
        a2 = _mm256_add_pd(a2, _mm256_mul_pd(x, _mm256_loadu_pd(b2 + t)));
        a3 = _mm256_add_pd(a3, _mm256_mul_pd(x, _mm256_loadu_pd(b3 + t)));
      }
      gram[(size_t)i * k + j] = finish(a0, wi, b0);
      gram[(size_t)i * k + j + 1] = finish(a1, wi, b1);
      gram[(size_t)i * k + j + 2] = finish(a2, wi, b2);
      gram[(size_t)i * k + j + 3] = finish(a3, wi, b3);
    }
    for (; j < k; ++j) {
      const double* bj = W + (size_t)j * n;
      __m256d acc = _mm256_setzero_pd();
      for (int t = 0; t < n4; t += 4) acc = _mm256_add_pd(acc, _mm256_mul_pd(_mm256_loadu_pd(wi + t), _mm256_loadu_pd(bj + t)));
      gram[(size_t)i * k + j] = finish(acc, wi, bj);
    }
  }
}

void gram(const double* W, int k, int n, const double* r, double* wv, double* g) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) gram_avx2(W, k, n, r, wv, g);
  else gram_base(W, k, n, r, wv, g);
}

}  // namespace

Lbfgsb::Lbfgsb(int n, int m, const double* lb, const double* ub, double factr, double pgtol, int maxls)
    : n_(n), m_(m), maxls_(maxls), factr_(factr), pgtol_(pgtol), epsmch_(std::numeric_limits<double>::epsilon()) {
  l_.assign(lb, lb + n);
  u_.assign(ub, ub + n);
  nbd_.resize(n);
  for (int i = 0; i < n; ++i) {
    const bool hl = std::isfinite(l_[i]), hu = std::isfinite(u_[i]);
    nbd_[i] = hl && hu ? 2 : hl ? 1 : hu ? 3 : 0;
  }
  iwhere_.assign(n, 0);
  x_.assign(n, 0.0);
  g_.assign(n, 0.0);
  z_.assign(n, 0.0);
  d_.assign(n, 0.0);
  t_.assign(n, 0.0);
  r_.assign(n, 0.0);
  ws_.assign((size_t)n * m, 0.0);
  wy_.assign((size_t)n * m, 0.0);
  sy_.assign((size_t)m * m, 0.0);
  ss_.assign((size_t)m * m, 0.0);
  pcol_.assign(m, 0);
  refresh_pcol();
}

void Lbfgsb::reset_memory() {
  col_ = 0;
  head_ = 0;
  theta_ = 1.0;
  iupdat_ = 0;
  minv_ok_ = false;
  refresh_pcol();
}

// [active] project the initial point, classify the variables.
int Lbfgsb::start(const double* x0) {
  cnstnd_ = false;
  boxed_ = true;
  for (int i = 0; i < n_; ++i) {
    double xi = x0[i];
    if (nbd_[i] > 0) {
      if (nbd_[i] <= 2 && xi <= l_[i]) xi = std::max(xi, l_[i]);
      else if (nbd_[i] >= 2 && xi >= u_[i]) xi = std::min(xi, u_[i]);
    }
    x_[i] = xi;
    if (nbd_[i] != 2) boxed_ = false;
    if (nbd_[i] == 0) {
      iwhere_[i] = -1;
    } else {
      cnstnd_ = true;
      iwhere_[i] = (nbd_[i] == 2 && u_[i] - l_[i] <= 0.0) ? 3 : 0;
    }
  }
  reset_memory();
  iter_ = 0;
  nfgv_ = 0;
  state_ = S_FG0;
  return LBFGSB_FG;
}

// [projgr] infinity norm of the projected gradient.
double Lbfgsb::projgr() const {
  double s = 0.0;
  for (int i = 0; i < n_; ++i) {
    double gi = g_[i];
    if (nbd_[i] != 0) {
      if (gi < 0.0) {
        if (nbd_[i] >= 2) gi = std::max(x_[i] - u_[i], gi);
      } else {
        if (nbd_[i] <= 2) gi = std::min(x_[i] - l_[i], gi);
      }
    }
    s = std::max(s, std::fabs(gi));
  }
  return s;
}

// M^-1 = [[-D, L^T], [L, theta S^T S]] over the col stored pairs (oldest first), LU-factored
// ([formt] factors the equivalent Schur complement theta S^T S + L D^-1 L^T).
bool Lbfgsb::form_minv() {
  const int c = col_, k = 2 * c;
  minv_lu_.assign((size_t)k * k, 0.0);
  auto A = [&](int i, int j) -> double& { return minv_lu_[(size_t)i * k + j]; };
  for (int i = 0; i < c; ++i) {
    A(i, i) = -sy_[(size_t)i * m_ + i];
    for (int j = 0; j < c; ++j) {
      if (i > j) {
        A(c + i, j) = sy_[(size_t)i * m_ + j];   // L
        A(j, c + i) = sy_[(size_t)i * m_ + j];   // L^T
      }
      const double s = i <= j ? ss_[(size_t)i * m_ + j] : ss_[(size_t)j * m_ + i];
      A(c + i, c + j) = theta_ * s;
    }
  }
  minv_ok_ = lu_factor(minv_lu_, minv_piv_, k);
  return minv_ok_;
}

bool Lbfgsb::bmv(const double* v, double* out) const {
  const int k = 2 * col_;
  if (!minv_ok_) return false;
  for (int i = 0; i < k; ++i) out[i] = v[i];
  lu_solve(minv_lu_, minv_piv_, k, out);
  return true;
}

// [cauchy] generalized Cauchy point along the projected steepest-descent path; on return
// z_ holds x^cp, c = W^T (x^cp - x) and iwhere_ marks the variables fixed at a bound.
int Lbfgsb::cauchy(std::vector<double>& xcp, std::vector<double>& c) {
  const int col = col_, col2 = 2 * col;
  xcp = x_;
  c.assign(col2, 0.0);
  std::vector<double>& p = sc_p_;
  std::vector<double>& v = sc_v_;
  std::vector<double>& wbp = sc_wbp_;
  p.assign(col2, 0.0);
  v.assign(col2, 0.0);
  wbp.assign(col2, 0.0);
  std::vector<double>& d = d_;
  bool bnded = true;
  int nfree = n_ + 1, nbreak = 0;
  std::vector<std::pair<double, int>>& bp = sc_bp_;
  bp.clear();
  double f1 = 0.0;
  for (int i = 0; i < n_; ++i) {
    const double neggi = -g_[i];
    double tl = 0.0, tu = 0.0;
    if (iwhere_[i] != 3 && iwhere_[i] != -1) {
      if (nbd_[i] <= 2) tl = x_[i] - l_[i];
      if (nbd_[i] >= 2) tu = u_[i] - x_[i];
      const bool xlower = nbd_[i] <= 2 && tl <= 0.0;
      const bool xupper = nbd_[i] >= 2 && tu <= 0.0;
      iwhere_[i] = 0;
      if (xlower) {
        if (neggi <= 0.0) iwhere_[i] = 1;
      } else if (xupper) {
        if (neggi >= 0.0) iwhere_[i] = 2;
      } else if (std::fabs(neggi) <= 0.0) {
        iwhere_[i] = -3;
      }
    }
    if (iwhere_[i] != 0 && iwhere_[i] != -1) {
      d[i] = 0.0;
    } else {
      d[i] = neggi;
      f1 -= neggi * neggi;
      for (int j = 0; j < col; ++j) {
        const int pj = col_index(j);
        p[j] += wy_[(size_t)pj * n_ + i] * neggi;
        p[col + j] += ws_[(size_t)pj * n_ + i] * neggi;
      }
      if (nbd_[i] <= 2 && nbd_[i] != 0 && neggi < 0.0) {
        bp.emplace_back(tl / (-neggi), i);
        ++nbreak;
      } else if (nbd_[i] >= 2 && neggi > 0.0) {
        bp.emplace_back(tu / neggi, i);
        ++nbreak;
      } else {
        --nfree;
        if (std::fabs(neggi) > 0.0) bnded = false;
      }
    }
  }
  for (int j = 0; j < col; ++j) p[col + j] *= theta_;
  if (nbreak == 0 && nfree == n_ + 1) return 0;   // d = 0: x is the GCP
  double f2 = -theta_ * f1;
  const double f2_org = f2;
  if (col > 0) {
    if (!bmv(p.data(), v.data())) return -1;
    f2 -= dot(v.data(), p.data(), col2);
  }
  double dtm = -f1 / f2, tsum = 0.0;
  // breakpoints in ascending (t, index) order — the order of a stable sort by t — popped
  // lazily from a heap (as [cauchy]'s hpsolb): the search usually stops after a few
  const auto later = [](const std::pair<double, int>& a, const std::pair<double, int>& b) {
    return a.first > b.first || (a.first == b.first && a.second > b.second);
  };
  std::make_heap(bp.begin(), bp.end(), later);
  int nleft = nbreak;
  double tj = 0.0;
  bool all_fixed = false;
  for (int k = 0; k < nbreak; ++k) {
    std::pop_heap(bp.begin(), bp.end() - k, later);
    const std::pair<double, int> next = bp[nbreak - 1 - k];
    const double tj0 = tj;
    tj = next.first;
    const int ibp = next.second;
    const double dt = tj - tj0;
    if (dtm < dt) break;
    tsum += dt;
    --nleft;
    const double dibp = d[ibp];
    d[ibp] = 0.0;
    double zibp;
    if (dibp > 0.0) {
      zibp = u_[ibp] - x_[ibp];
      xcp[ibp] = u_[ibp];
      iwhere_[ibp] = 2;
    } else {
      zibp = l_[ibp] - x_[ibp];
      xcp[ibp] = l_[ibp];
      iwhere_[ibp] = 1;
    }
    if (nleft == 0 && nbreak == n_) {
      dtm = dt;
      all_fixed = true;
      break;
    }
    const double dibp2 = dibp * dibp;
    f1 = f1 + dt * f2 + dibp2 - theta_ * dibp * zibp;
    f2 -= theta_ * dibp2;
    if (col > 0) {
      for (int j = 0; j < col2; ++j) c[j] += dt * p[j];
      for (int j = 0; j < col; ++j) {
        const int pj = col_index(j);
        wbp[j] = wy_[(size_t)pj * n_ + ibp];
        wbp[col + j] = theta_ * ws_[(size_t)pj * n_ + ibp];
      }
      if (!bmv(wbp.data(), v.data())) return -1;
      const double wmc = dot(c.data(), v.data(), col2);
      const double wmp = dot(p.data(), v.data(), col2);
      const double wmw = dot(wbp.data(), v.data(), col2);
      for (int j = 0; j < col2; ++j) p[j] -= dibp * wbp[j];
      f1 += dibp * wmc;
      f2 += 2.0 * dibp * wmp - dibp2 * wmw;
    }
    f2 = std::max(epsmch_ * f2_org, f2);
    if (nleft > 0) {
      dtm = -f1 / f2;
    } else if (bnded) {
      f1 = f2 = dtm = 0.0;
    } else {
      dtm = -f1 / f2;
    }
  }
  if (!all_fixed) {
    if (dtm <= 0.0) dtm = 0.0;
    tsum += dtm;
    for (int i = 0; i < n_; ++i) xcp[i] += tsum * d[i];
  }
  if (col > 0)
    for (int j = 0; j < col2; ++j) c[j] += dtm * p[j];
  return 0;
}

// [cmprlb + subsm, v3.0] direct primal subspace minimisation over the free variables at
// the GCP, then projection onto the box (kept if it is a descent direction) or the
// backtracking step along the subspace direction.  z holds x^cp on entry.
void Lbfgsb::subspace(std::vector<double>& z, const std::vector<double>& c) {
  const int col = col_, col2 = 2 * col;
  std::vector<int>& ind = sc_ind_;
  ind.clear();
  for (int i = 0; i < n_; ++i)
    if (iwhere_[i] <= 0) ind.push_back(i);
  const int nsub = (int)ind.size();
  if (nsub == 0 || col == 0) return;
  // r = -Z^T (theta (z - x) + g - W M c)
  std::vector<double>& mc = sc_mc_;
  std::vector<double>& r = sc_r_;
  mc.assign(col2, 0.0);
  r.assign(nsub, 0.0);
  bmv(c.data(), mc.data());
  for (int a = 0; a < nsub; ++a) {
    const int k = ind[a];
    double s = -theta_ * (z[k] - x_[k]) - g_[k];
    for (int j = 0; j < col; ++j) {
      const int pj = col_index(j);
      s += wy_[(size_t)pj * n_ + k] * mc[j] + ws_[(size_t)pj * n_ + k] * theta_ * mc[col + j];
    }
    r[a] = s;
  }
  // d = (Z^T B Z)^-1 r = r / theta + W_F (M^-1 - W_F^T W_F / theta)^-1 W_F^T r / theta^2
  std::vector<double>& N = sc_N_;
  std::vector<double>& wv = sc_wv_;
  N.assign(minv_lu_.size(), 0.0);
  wv.assign(col2, 0.0);
  {
    // rebuild M^-1 (the LU holds its factors) and subtract W_F^T W_F / theta
    const int k2 = col2;
    std::fill(N.begin(), N.end(), 0.0);
    for (int i = 0; i < col; ++i) {
      N[(size_t)i * k2 + i] = -sy_[(size_t)i * m_ + i];
      for (int j = 0; j < col; ++j) {
        if (i > j) {
          N[(size_t)(col + i) * k2 + j] = sy_[(size_t)i * m_ + j];
          N[(size_t)j * k2 + col + i] = sy_[(size_t)i * m_ + j];
        }
        const double s = i <= j ? ss_[(size_t)i * m_ + j] : ss_[(size_t)j * m_ + i];
        N[(size_t)(col + i) * k2 + col + j] = theta_ * s;
      }
    }
    // W_F (col2 x nsub, rows contiguous) gathered once; then W_F^T r and the symmetric
    // W_F^T W_F / theta as row dot products (vectorisable) instead of nsub rank-1 updates
    std::vector<double>& WF = wf_;
    WF.resize((size_t)k2 * nsub);
    for (int j = 0; j < col; ++j) {
      const int pj = col_index(j);
      const double* wyr = &wy_[(size_t)pj * n_];
      const double* wsr = &ws_[(size_t)pj * n_];
      double* a1 = &WF[(size_t)j * nsub];
      double* a2 = &WF[(size_t)(col + j) * nsub];
      if (nsub == n_) {
        for (int a = 0; a < nsub; ++a) {
          a1[a] = wyr[a];
          a2[a] = theta_ * wsr[a];
        }
      } else {
        for (int a = 0; a < nsub; ++a) {
          a1[a] = wyr[ind[a]];
          a2[a] = theta_ * wsr[ind[a]];
        }
      }
    }
    std::vector<double>& GG = sc_gram_;
    GG.resize((size_t)k2 * k2);
    gram(WF.data(), k2, nsub, r.data(), wv.data(), GG.data());
    for (int i = 0; i < k2; ++i)
      for (int j = i; j < k2; ++j) {
        const double gij = GG[(size_t)i * k2 + j] / theta_;
        N[(size_t)i * k2 + j] -= gij;
        if (j != i) N[(size_t)j * k2 + i] -= gij;
      }
  }
  std::vector<int>& piv = sc_piv_;
  std::vector<double>& dsub = sc_dsub_;
  dsub.assign(nsub, 0.0);
  if (lu_factor(N, piv, col2)) {
    lu_solve(N, piv, col2, wv.data());
    for (int a = 0; a < nsub; ++a) {
      const int k = ind[a];
      double s = 0.0;
      for (int j = 0; j < col; ++j) {
        const int pj = col_index(j);
        s += wy_[(size_t)pj * n_ + k] * wv[j] + theta_ * ws_[(size_t)pj * n_ + k] * wv[col + j];
      }
      dsub[a] = r[a] / theta_ + s / (theta_ * theta_);
    }
  } else {
    for (int a = 0; a < nsub; ++a) dsub[a] = r[a] / theta_;   // B = theta I on the subspace
  }
  // projection of x^cp + d onto the box
  std::vector<double>& xp = sc_xp_;
  xp = z;
  bool hit = false;
  for (int a = 0; a < nsub; ++a) {
    const int k = ind[a];
    const double xk = z[k], dk = dsub[a];
    if (nbd_[k] == 0) {
      z[k] = xk + dk;
    } else if (nbd_[k] == 1) {
      z[k] = std::max(l_[k], xk + dk);
      if (z[k] == l_[k]) hit = true;
    } else if (nbd_[k] == 2) {
      z[k] = std::min(u_[k], std::max(l_[k], xk + dk));
      if (z[k] == l_[k] || z[k] == u_[k]) hit = true;
    } else {
      z[k] = std::min(u_[k], xk + dk);
      if (z[k] == u_[k]) hit = true;
    }
  }
  if (!hit) return;
  double dd_p = 0.0;
  for (int i = 0; i < n_; ++i) dd_p += (z[i] - x_[i]) * g_[i];
  if (!(dd_p > 0.0)) return;
  // not a descent direction: backtrack along the subspace direction from x^cp
  z = xp;
  double alpha = 1.0, temp1 = alpha;
  int ibd = -1;
  for (int a = 0; a < nsub; ++a) {
    const int k = ind[a];
    const double dk = dsub[a];
    if (nbd_[k] != 0) {
      if (dk < 0.0 && nbd_[k] <= 2) {
        const double temp2 = l_[k] - z[k];
        if (temp2 >= 0.0) temp1 = 0.0;
        else if (dk * alpha < temp2) temp1 = temp2 / dk;
      } else if (dk > 0.0 && nbd_[k] >= 2) {
        const double temp2 = u_[k] - z[k];
        if (temp2 <= 0.0) temp1 = 0.0;
        else if (dk * alpha > temp2) temp1 = temp2 / dk;
      }
      if (temp1 < alpha) {
        alpha = temp1;
        ibd = a;
      }
    }
  }
  if (alpha < 1.0 && ibd >= 0) {
    const int k = ind[ibd];
    if (dsub[ibd] > 0.0) z[k] = u_[k], dsub[ibd] = 0.0;
    else if (dsub[ibd] < 0.0) z[k] = l_[k], dsub[ibd] = 0.0;
  }
  for (int a = 0; a < nsub; ++a) z[ind[a]] += alpha * dsub[a];
}

// [mainlb, label 222] Cauchy point, subspace step, search direction, line-search start.
int Lbfgsb::begin_iteration() {
  for (int attempt = 0; attempt < 3; ++attempt) {
    std::vector<double>& xcp = xcp_tmp_;   // kept between iterations: no allocation per iteration
    std::vector<double>& c = sc_c_;
    if (!cnstnd_ && col_ > 0) {
      z_ = x_;
      for (int i = 0; i < n_; ++i) iwhere_[i] = -1;
      // unconstrained: the subspace step is the full quasi-Newton step from x
      c.assign(2 * col_, 0.0);
      subspace(z_, c);
    } else {
      if (cauchy(xcp, c) != 0) {   // singular middle matrix: refresh the memory
        reset_memory();
        continue;
      }
      z_ = xcp;
      subspace(z_, c);
    }
    for (int i = 0; i < n_; ++i) d_[i] = z_[i] - x_[i];
    // [lnsrlb] maximum step and first trial step
    dtd_ = dot(d_.data(), d_.data(), n_);
    dnorm_ = std::sqrt(dtd_);
    stpmx_ = 1e10;
    if (cnstnd_) {
      if (iter_ == 0) {
        stpmx_ = 1.0;
      } else {
        for (int i = 0; i < n_; ++i) {
          const double a1 = d_[i];
          if (nbd_[i] == 0) continue;
          if (a1 < 0.0 && nbd_[i] <= 2) {
            const double a2 = l_[i] - x_[i];
            if (a2 >= 0.0) stpmx_ = 0.0;
            else if (a1 * stpmx_ < a2) stpmx_ = a2 / a1;
          } else if (a1 > 0.0 && nbd_[i] >= 2) {
            const double a2 = u_[i] - x_[i];
            if (a2 <= 0.0) stpmx_ = 0.0;
            else if (a1 * stpmx_ > a2) stpmx_ = a2 / a1;
          }
        }
      }
    }
    stp_ = (iter_ == 0 && !boxed_) ? std::min(1.0 / dnorm_, stpmx_) : 1.0;
    // a rounding-level stpmx < 1 would make the first trial exceed it (dcsrch's STP > STPMAX)
    if (stp_ > stpmx_) stp_ = stpmx_;
    t_ = x_;
    r_ = g_;
    fold_ = f_;
    ifun_ = 0;
    iback_ = 0;
    ls_task_ = 0;
    return ls_continue();
  }
  state_ = S_DONE;
  return LBFGSB_ABNORMAL;
}

// [lnsrlb from label 556] one More-Thuente step; returns FG (trial point in x_) or NEW_X,
// or handles a failed search (restore, refresh the memory, restart the iteration).
int Lbfgsb::ls_continue() {
  gd_ = dot(g_.data(), d_.data(), n_);
  bool fail = false;
  if (ifun_ == 0) {
    gdold_ = gd_;
    if (gd_ >= 0.0) fail = true;   // not a descent direction
  }
  if (!fail) {
    dcsrch(f_, gd_, stp_, 1e-3, 0.9, 0.1, 0.0, stpmx_);
    if (ls_task_ == 1) {
      ++ifun_;
      ++nfgv_;
      iback_ = ifun_ - 1;
      if (iback_ < maxls_) {
        if (stp_ == 1.0) x_ = z_;
        else
          for (int i = 0; i < n_; ++i) x_[i] = stp_ * d_[i] + t_[i];
        state_ = S_LNSRCH;
        return LBFGSB_FG;
      }
      --nfgv_;
      fail = true;
    } else if (ls_task_ == 4) {
      fail = true;
    }
  }
  if (fail) {
    x_ = t_;
    g_ = r_;
    f_ = fold_;
    if (col_ == 0) {
      ++iter_;
      state_ = S_DONE;
      return LBFGSB_ABNORMAL;
    }
    reset_memory();
    return begin_iteration();
  }
  // accepted: a new iterate
  ++iter_;
  sbgnrm_ = projgr();
  state_ = S_NEWX;
  return LBFGSB_NEW_X;
}

// [matupd] append the pair (s, y) = (d_, r_), theta = y'y / s'y, update S'Y and S'S.
void Lbfgsb::update_memory(double rr, double dr, double stp) {
  (void)stp;
  ++iupdat_;
  int itail;
  if (iupdat_ <= m_) {
    col_ = iupdat_;
    itail = (head_ + iupdat_ - 1) % m_;
  } else {
    itail = (head_ + m_) % m_;   // overwrite the oldest column, advance the head
    head_ = (head_ + 1) % m_;
    refresh_pcol();
  }
  std::copy(d_.begin(), d_.end(), ws_.begin() + (size_t)itail * n_);
  std::copy(r_.begin(), r_.end(), wy_.begin() + (size_t)itail * n_);
  theta_ = rr / dr;
  const int c = col_;
  if (iupdat_ > m_) {
    for (int i = 0; i < c - 1; ++i)
      for (int j = 0; j < c - 1; ++j) {
        if (i <= j) ss_[(size_t)i * m_ + j] = ss_[(size_t)(i + 1) * m_ + j + 1];
        if (i >= j) sy_[(size_t)i * m_ + j] = sy_[(size_t)(i + 1) * m_ + j + 1];
      }
  }
  for (int j = 0; j < c - 1; ++j) {
    const int pj = col_index(j);
    sy_[(size_t)(c - 1) * m_ + j] = dot(d_.data(), wy_.data() + (size_t)pj * n_, n_);
    ss_[(size_t)j * m_ + c - 1] = dot(ws_.data() + (size_t)pj * n_, d_.data(), n_);
  }
  ss_[(size_t)(c - 1) * m_ + c - 1] = dot(d_.data(), d_.data(), n_);
  sy_[(size_t)(c - 1) * m_ + c - 1] = dr;
}

int Lbfgsb::step(double f, const double* g) {
  switch (state_) {
    case S_FG0: {
      f_ = f;
      std::copy(g, g + n_, g_.begin());
      nfgv_ = 1;
      sbgnrm_ = projgr();
      if (sbgnrm_ <= pgtol_) {
        state_ = S_DONE;
        return LBFGSB_CONV_PGTOL;
      }
      return begin_iteration();
    }
    case S_LNSRCH: {
      bool finite = std::isfinite(f);
      for (int i = 0; i < n_ && finite; ++i) finite = std::isfinite(g[i]);
      if (!finite) {
        // a trial point with a non-finite value or gradient (an overflowing kernel gradient,
        // a NaN from the objective) is rejected: the More-Thuente search restarts from the
        // iterate with a 10x shorter step (counted against maxls like any other trial), so no
        // NaN ever enters the iterate, the curvature pairs or the bracket
        f_ = fold_;
        g_ = r_;
        stp_ *= 0.1;
        ls_task_ = 0;
        return ls_continue();
      }
      f_ = f;
      std::copy(g, g + n_, g_.begin());
      return ls_continue();
    }
    case S_NEWX: {
      if (sbgnrm_ <= pgtol_) {
        state_ = S_DONE;
        return LBFGSB_CONV_PGTOL;
      }
      const double ddum0 = std::max(std::max(std::fabs(fold_), std::fabs(f_)), 1.0);
      if (fold_ - f_ <= factr_ * epsmch_ * ddum0) {
        state_ = S_DONE;
        return LBFGSB_CONV_FACTR;
      }
      for (int i = 0; i < n_; ++i) r_[i] = g_[i] - r_[i];
      const double rr = dot(r_.data(), r_.data(), n_);
      double dr, ddum;
      if (stp_ == 1.0) {
        dr = gd_ - gdold_;
        ddum = -gdold_;
      } else {
        dr = (gd_ - gdold_) * stp_;
        for (int i = 0; i < n_; ++i) d_[i] *= stp_;
        ddum = -gdold_ * stp_;
      }
      if (dr > epsmch_ * ddum) {
        update_memory(rr, dr, stp_);
        if (!form_minv()) reset_memory();
      }
      return begin_iteration();
    }
    default:
      return LBFGSB_ERROR;
  }
}

// [dcsrch] More-Thuente line search (MINPACK-2), reverse communication through ls_task_:
// 0 start, 1 evaluate at stp, 2 converged, 3 warning (accept), 4 error.
static void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy, double& dy, double& stp, double fp,
                   double dp, bool& brackt, double stpmin, double stpmax) {
  const double sgnd = dp * (dx / std::fabs(dx));
  double stpf;
  if (fp > fx) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = std::max(std::max(std::fabs(theta), std::fabs(dx)), std::fabs(dp));
    double gamma = s * std::sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp < stx) gamma = -gamma;
    const double p = (gamma - dx) + theta;
    const double q = ((gamma - dx) + gamma) + dp;
    const double r = p / q;
    const double stpc = stx + r * (stp - stx);
    const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
    if (std::fabs(stpc - stx) < std::fabs(stpq - stx)) stpf = stpc;
    else stpf = stpc + (stpq - stpc) / 2.0;
    brackt = true;
  } else if (sgnd < 0.0) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = std::max(std::max(std::fabs(theta), std::fabs(dx)), std::fabs(dp));
    double gamma = s * std::sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp > stx) gamma = -gamma;
    const double p = (gamma - dp) + theta;
    const double q = ((gamma - dp) + gamma) + dx;
    const double r = p / q;
    const double stpc = stp + r * (stx - stp);
    const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    stpf = std::fabs(stpc - stp) > std::fabs(stpq - stp) ? stpc : stpq;
    brackt = true;
  } else if (std::fabs(dp) < std::fabs(dx)) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = std::max(std::max(std::fabs(theta), std::fabs(dx)), std::fabs(dp));
    double gamma = s * std::sqrt(std::max(0.0, (theta / s) * (theta / s) - (dx / s) * (dp / s)));
    if (stp > stx) gamma = -gamma;
    const double p = (gamma - dp) + theta;
    const double q = (gamma + (dx - dp)) + gamma;
    const double r = p / q;
    double stpc;
    if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
    else if (stp > stx) stpc = stpmax;
    else stpc = stpmin;
    const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (brackt) {
      stpf = std::fabs(stpc - stp) < std::fabs(stpq - stp) ? stpc : stpq;
      if (stp > stx) stpf = std::min(stp + 0.66 * (sty - stp), stpf);
      else stpf = std::max(stp + 0.66 * (sty - stp), stpf);
    } else {
      stpf = std::fabs(stpc - stp) > std::fabs(stpq - stp) ? stpc : stpq;
      stpf = std::min(stpmax, stpf);
      stpf = std::max(stpmin, stpf);
    }
  } else {
    if (brackt) {
      const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
      const double s = std::max(std::max(std::fabs(theta), std::fabs(dy)), std::fabs(dp));
      double gamma = s * std::sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
      if (stp > sty) gamma = -gamma;
      const double p = (gamma - dp) + theta;
      const double q = ((gamma - dp) + gamma) + dy;
      const double r = p / q;
      stpf = stp + r * (sty - stp);
    } else if (stp > stx) {
      stpf = stpmax;
    } else {
      stpf = stpmin;
    }
  }
  if (fp > fx) {
    sty = stp;
    fy = fp;
    dy = dp;
  } else {
    if (sgnd < 0.0) {
      sty = stx;
      fy = fx;
      dy = dx;
    }
    stx = stp;
    fx = fp;
    dx = dp;
  }
  stp = stpf;
}

void Lbfgsb::dcsrch(double f, double g, double& stp, double ftol, double gtol, double xtol, double stpmin,
                    double stpmax) {
  const double xtrapl = 1.1, xtrapu = 4.0;
  if (ls_task_ == 0) {
    if (stp < stpmin || stp > stpmax || g >= 0.0 || ftol < 0.0 || gtol < 0.0 || xtol < 0.0 || stpmin < 0.0 ||
        stpmax < stpmin) {
      ls_task_ = 4;
      return;
    }
    brackt_ = false;
    stage_ = 1;
    finit_ = f;
    ginit_ = g;
    gtest_ = ftol * ginit_;
    width_ = stpmax - stpmin;
    width1_ = width_ / 0.5;
    stx_ = 0.0;
    fx_ = finit_;
    gx_ = ginit_;
    sty_ = 0.0;
    fy_ = finit_;
    gy_ = ginit_;
    stmin_ = 0.0;
    stmax_ = stp + xtrapu * stp;
    ls_task_ = 1;
    return;
  }
  const double ftest = finit_ + stp * gtest_;
  if (stage_ == 1 && f <= ftest && g >= 0.0) stage_ = 2;
  int task = 1;
  if (brackt_ && (stp <= stmin_ || stp >= stmax_)) task = 3;
  if (brackt_ && stmax_ - stmin_ <= xtol * stmax_) task = 3;
  if (stp == stpmax && f <= ftest && g <= gtest_) task = 3;
  if (stp == stpmin && (f > ftest || g >= gtest_)) task = 3;
  if (f <= ftest && std::fabs(g) <= gtol * (-ginit_)) task = 2;
  if (task != 1) {
    ls_task_ = task;
    return;
  }
  if (stage_ == 1 && f <= fx_ && f > ftest) {
    const double fm = f - stp * gtest_;
    double fxm = fx_ - stx_ * gtest_, fym = fy_ - sty_ * gtest_;
    const double gm = g - gtest_;
    double gxm = gx_ - gtest_, gym = gy_ - gtest_;
    dcstep(stx_, fxm, gxm, sty_, fym, gym, stp, fm, gm, brackt_, stmin_, stmax_);
    fx_ = fxm + stx_ * gtest_;
    fy_ = fym + sty_ * gtest_;
    gx_ = gxm + gtest_;
    gy_ = gym + gtest_;
  } else {
    dcstep(stx_, fx_, gx_, sty_, fy_, gy_, stp, f, g, brackt_, stmin_, stmax_);
  }
  if (brackt_) {
    if (std::fabs(sty_ - stx_) >= 0.66 * width1_) stp = stx_ + 0.5 * (sty_ - stx_);
    width1_ = width_;
    width_ = std::fabs(sty_ - stx_);
  }
  if (brackt_) {
    stmin_ = std::min(stx_, sty_);
    stmax_ = std::max(stx_, sty_);
  } else {
    stmin_ = stp + xtrapl * (stp - stx_);
    stmax_ = stp + xtrapu * (stp - stx_);
  }
  stp = std::max(stp, stpmin);
  stp = std::min(stp, stpmax);
  if ((brackt_ && (stp <= stmin_ || stp >= stmax_)) || (brackt_ && stmax_ - stmin_ <= xtol * stmax_)) stp = stx_;
  ls_task_ = 1;
}

}  // namespace evr

using evr::Lbfgsb;

struct evr_lbfgsb {
  Lbfgsb* opt;
  int n;
};

extern "C" {

int evr_lbfgsb_create(int n, int m, const double* lb, const double* ub, double factr, double pgtol, int maxls,
                      evr_lbfgsb** out) {
  LB_CHECK(out && n >= 1 && m >= 1 && lb && ub && factr >= 0.0 && pgtol >= 0.0 && maxls >= 1,
           "evr_lbfgsb_create: bad arguments");
  for (int i = 0; i < n; ++i) LB_CHECK(!(lb[i] > ub[i]), "evr_lbfgsb_create: lower bound above upper bound");
  evr_lbfgsb* h = new (std::nothrow) evr_lbfgsb();
  LB_CHECK(h, "evr_lbfgsb_create: out of host memory");
  h->opt = new (std::nothrow) Lbfgsb(n, m, lb, ub, factr, pgtol, maxls);
  h->n = n;
  if (!h->opt) {
    delete h;
    LB_CHECK(false, "evr_lbfgsb_create: out of host memory");
  }
  *out = h;
  return 0;
}

int evr_lbfgsb_start(evr_lbfgsb* h, const double* x0, double* x) {
  if (!h || !x0 || !x) return evr::LBFGSB_ERROR;
  const int t = h->opt->start(x0);
  std::copy(h->opt->x(), h->opt->x() + h->n, x);
  return t;
}

int evr_lbfgsb_step(evr_lbfgsb* h, double f, const double* g, double* x) {
  if (!h || !g || !x) return evr::LBFGSB_ERROR;
  const int t = h->opt->step(f, g);
  std::copy(h->opt->x(), h->opt->x() + h->n, x);
  return t;
}

void evr_lbfgsb_stats(const evr_lbfgsb* h, int* nit, int* nfev, double* f, double* pgnorm) {
  if (!h) return;
  if (nit) *nit = h->opt->iterations();
  if (nfev) *nfev = h->opt->evaluations();
  if (f) *f = h->opt->f();
  if (pgnorm) *pgnorm = h->opt->projected_gradient_norm();
}

void evr_lbfgsb_destroy(evr_lbfgsb* h) {
  if (!h) return;
  delete h->opt;
  delete h;
}

}  // extern "C"
