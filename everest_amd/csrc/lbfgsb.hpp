// Native L-BFGS-B (bound-constrained limited-memory BFGS) for the acquisition restarts of
// ask(): restates the algorithm scipy.optimize.minimize(method="L-BFGS-B") runs inside
// [upstream] botorch gen_candidates_scipy (called from bofire/strategies/predictives/
// botorch.py:384-405): Byrd, Lu, Nocedal & Zhu (1995) with the v3.0 subspace step
// (Morales & Nocedal 2011) — generalized Cauchy point over the box breakpoints, direct
// primal subspace minimisation on the free variables (compact form B = theta I - W M W^T
// inverted by Sherman-Morrison-Woodbury), projection with the descent check and
// backtracking fallback, and the More-Thuente line search (ftol 1e-3, gtol 0.9, xtol 0.1).
// Defaults are scipy's: m = 10 corrections, factr = 1e7 (ftol 2.22e-9), pgtol = 1e-5,
// maxls = 20.
//
// Reverse communication: step(f, g) consumes f, g at x() and returns what the caller must
// do next (evaluate f, g at the new x(), or accept a new iterate, or stop).
#pragma once

#include <string>
#include <vector>

namespace evr {

enum LbfgsbTask : int {
  LBFGSB_FG = 1,          // evaluate f, g at x() and call step again
  LBFGSB_NEW_X = 2,       // an iteration finished; the caller may stop (maxiter/maxfun) or call step again
  LBFGSB_CONV_PGTOL = 3,  // projected gradient inf-norm <= pgtol
  LBFGSB_CONV_FACTR = 4,  // relative reduction of f <= factr * eps
  LBFGSB_ABNORMAL = 5,    // line search failed without any correction pairs
  LBFGSB_ERROR = 6,       // invalid input
};

class Lbfgsb {
 public:
  Lbfgsb(int n, int m, const double* lb, const double* ub, double factr, double pgtol, int maxls);
  // Initial point (projected onto the box); returns LBFGSB_FG.
  int start(const double* x0);
  // f, g at x(); returns the next task.
  int step(double f, const double* g);
  const double* x() const { return x_.data(); }
  double f() const { return f_; }
  const double* g() const { return g_.data(); }
  int iterations() const { return iter_; }
  int evaluations() const { return nfgv_; }
  double projected_gradient_norm() const { return sbgnrm_; }

 private:
  enum State { S_START, S_FG0, S_LNSRCH, S_NEWX, S_DONE };
  int n_, m_, maxls_;
  double factr_, pgtol_, epsmch_;
  std::vector<double> l_, u_;
  std::vector<int> nbd_, iwhere_;
  bool cnstnd_ = false, boxed_ = true;
  // iterate
  std::vector<double> x_, g_, z_, d_, t_, r_, xcp_tmp_;
  double f_ = 0, fold_ = 0, sbgnrm_ = 0;
  int iter_ = 0, nfgv_ = 0;
  State state_ = S_START;
  // limited memory: columns stored oldest .. newest (circular by head_)
  std::vector<double> ws_, wy_;            // n x m, column k at [k * n]
  std::vector<double> sy_, ss_;            // m x m (sy lower, ss upper, logical order)
  int col_ = 0, head_ = 0, iupdat_ = 0;
  double theta_ = 1.0;
  std::vector<double> minv_lu_;            // LU of the 2col x 2col M^-1
  std::vector<double> wf_;                 // subspace scratch: W over the free variables
  // per-iteration scratch kept between iterations (no allocation in the loop)
  std::vector<double> sc_p_, sc_v_, sc_wbp_, sc_mc_, sc_r_, sc_N_, sc_wv_, sc_dsub_, sc_xp_, sc_gram_, sc_c_;
  std::vector<std::pair<double, int>> sc_bp_;
  std::vector<int> sc_ind_, sc_piv_;
  std::vector<int> minv_piv_;
  bool minv_ok_ = false;
  // line search
  double stp_ = 0, stpmx_ = 0, gd_ = 0, gdold_ = 0, dnorm_ = 0, dtd_ = 0;
  int ifun_ = 0, iback_ = 0;
  // dcsrch state
  bool brackt_ = false;
  int stage_ = 0;
  double ginit_ = 0, gtest_ = 0, gx_ = 0, gy_ = 0, finit_ = 0, fx_ = 0, fy_ = 0, stx_ = 0, sty_ = 0, stmin_ = 0,
         stmax_ = 0, width_ = 0, width1_ = 0;
  int ls_task_ = 0;  // 0 start, 1 fg, 2 conv, 3 warning, 4 error

  double projgr() const;
  void reset_memory();
  bool form_minv();
  bool bmv(const double* v, double* out) const;  // out = M v  (length 2col)
  int cauchy(std::vector<double>& xcp, std::vector<double>& c);
  void subspace(std::vector<double>& z, const std::vector<double>& c);
  int begin_iteration();
  int ls_continue();
  void dcsrch(double f, double g, double& stp, double ftol, double gtol, double xtol, double stpmin, double stpmax);
  void update_memory(double rr, double dr, double stp);
  // storage slot of the k-th stored pair (oldest first); a table refreshed when head_ moves
  // (the modulo in every inner loop of the Cauchy / subspace steps was a division per term)
  std::vector<int> pcol_;
  void refresh_pcol() {
    for (int k = 0; k < m_; ++k) pcol_[k] = (head_ + k) % m_;
  }
  int col_index(int k) const { return pcol_[k]; }
};

}  // namespace evr
