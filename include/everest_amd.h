/*
 * everest_amd — MI355X-native (gfx950) GP-surrogate + qNEHVI hot path of BoFire.
 *
 * C-ABI drop-in boundary.  Plain pointers and sizes only; every device pointer is an
 * HBM allocation owned by the caller (torch tensors in the Python host layer); every
 * entry point enqueues on the given HIP stream (hipStream_t passed as void*) and returns
 * 0 on success, non-zero on error with the message in evr_last_error().  Layouts are
 * row-major float64 unless stated.
 *
 * The reference (experimental-design/everest = BoFire) has no FFI: its hot path hands
 * control to BoTorch/GPyTorch from Python.  Each entry point below names the reference
 * call site whose [upstream] arithmetic it replaces (paths relative to the reference root).
 */
#ifndef EVEREST_AMD_H
#define EVEREST_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define EVR_VERSION 1

/* kernel families: bofire/kernels/mapper.py:31-69 (RBFKernel, MaternKernel nu) */
#define EVR_KERNEL_RBF 0
#define EVR_KERNEL_MATERN05 1
#define EVR_KERNEL_MATERN15 2
#define EVR_KERNEL_MATERN25 3
/* one family per output (heterogeneous ModelListGP members, bofire/surrogates/
 * botorch_surrogates.py:79-128): EVR_KERNEL_MIXED | kind_j << (5 + 2 j), j < 13, wherever an
 * entry point takes `kind` together with a batch of outputs */
#define EVR_KERNEL_MIXED 16

int evr_version(void);
const char* evr_last_error(void);
int evr_device_arch(int device, char* buf, int buflen);
int evr_stream_sync(void* stream);

/* ---- kernel-matrix assembly ---------------------------------------------------------
 * K[b][i][j] = outputscale[b] * k( ||(x1n_i - x2n_j) / ls[b]|| ) (+ diag_add[b] if i==j)
 * x1n = (X1 - shift1) * scale1, x2n = (X2 - shift2) * scale2 per column (NULL = identity),
 * X1: n1 x d, X2: n2 x d, ls: B x d, K: B x n1 x n2 (ld n2).
 * Replaces gpytorch RBFKernel/MaternKernel forward under the Normalize input transform
 * called from bofire/surrogates/single_task_gp.py:48-66 and every posterior() call
 * (bofire/strategies/predictives/botorch.py:180; bofire/surrogates/botorch.py:27,33). */
int evr_kernel_matrix(void* stream, int kind, int B, int n1, int n2, int d,
                      const double* X1, const double* shift1, const double* scale1,
                      const double* X2, const double* shift2, const double* scale2,
                      const double* lengthscales, const double* outputscale,
                      const double* diag_add, double* K);

/* dX2[c][k] = sum_b sum_i G[b][i][c] * dK_b(x1_i, x2_c)/dX2[c][k]  (chain through shift2/scale2)
 * G: B x n1 x n2.  Backward of the cross-covariance for the acquisition gradient
 * (autograd inside gen_candidates_scipy, bofire/strategies/predictives/botorch.py:384-405). */
int evr_kernel_cross_grad(void* stream, int kind, int B, int n1, int n2, int d,
                          const double* X1, const double* shift1, const double* scale1,
                          const double* X2, const double* shift2, const double* scale2,
                          const double* lengthscales, const double* outputscale,
                          const double* G, double* dX2, double* work);
/* doubles of `work` evr_kernel_cross_grad needs (row-split partials); work NULL = allocate */
long long evr_kernel_cross_grad_workspace_doubles(int n1, int n2, int d);

/* MLL gradient pieces for the exact GP fit (fit_gpytorch_mll,
 * bofire/surrogates/single_task_gp.py:70-71):
 * gls[b][k] = sum_{i,j} W[b][i][j] * dK_b[i][j]/d ls[b][k]   (W symmetric, X normalized);
 * work: B*n*d doubles (per-row partials, summed in fixed order -> bitwise reproducible). */
int evr_kernel_lengthscale_grad(void* stream, int kind, int B, int n, int d, const double* X,
                                const double* lengthscales, const double* W, double* gls,
                                double* work);
/* out[b][0..4] = {2 sum log L_ii, r.alpha, ||Linv||_F^2 (= tr K^-1), sum alpha, sum alpha^2}
 * — the scalar terms of the exact MLL and of its noise/constant gradients. */
int evr_gp_mll_terms(void* stream, int B, int n, const double* L, const double* Linv,
                     const double* r, const double* alpha, double* out);

/* Native MLL plan for the GP fit: B exact GPs sharing the normalised inputs Xn (n x d,
 * device, must outlive the plan) with standardised targets Y (B x n, device, copied).  One
 * evr_mll_plan_eval is one hipGraph launch computing, per member b, with params (host) =
 * [lengthscales (B x d) | noise (B) | constant (B)]:
 *   out (host) = [terms (B x 5) as evr_gp_mll_terms | gls (B x d) as
 *                 evr_kernel_lengthscale_grad with W = alpha alpha^T - K^-1 | info (B)]
 * for K = k(Xn, Xn; ls_b) + noise_b I (psd_safe_cholesky attempt 0: a member with
 * info != 0 needs the jitter ladder, i.e. the unfused path).  Replaces the per-evaluation
 * op chain of the ExactMarginalLogLikelihood closure inside [upstream] fit_gpytorch_mll
 * (bofire/surrogates/single_task_gp.py:70-71). */
typedef struct evr_mll_plan evr_mll_plan;
int evr_mll_plan_create(void* stream, int kind, int B, int n, int d, const double* Xn, const double* Y,
                        evr_mll_plan** out);
int evr_mll_plan_eval(void* stream, evr_mll_plan* plan, const double* params, double* out);
void evr_mll_plan_destroy(evr_mll_plan* plan);

/* The lock-step fit of the plan's B members in native code (gp.fit_batch: one L-BFGS-B per
 * output over -MLL / n with the gpytorch priors, [upstream] fit_gpytorch_mll ->
 * scipy L-BFGS-B, bofire/surrogates/single_task_gp.py:70-71).  Member b: runs[b] an
 * evr_lbfgsb of dimension d + 2 over x = [noise, constant, raw lengthscales (softplus)],
 * task[b] its current task (EVR_LBFGSB_FG: x[b] is to be evaluated; 0: finished), f / g the
 * last evaluation it was given, nit / nfev / status as scipy's driver loop counts them
 * (status 0 converged, 1 iteration / evaluation limit, 2 abnormal line search, 3 error).
 * params (B x (d + 2), the plan's layout) carries the members' last evaluated parameters
 * across calls.  prior: ls (fam, a, b), noise (fam, a, b) with fam 0 none, 1 LogNormal,
 * 2 Gamma, 3 Normal.  Runs rounds (one plan evaluation of every member with task FG, then
 * each one's L-BFGS-B steps) until every member has finished (*pending = 0), or a round in
 * which an evaluated member's attempt-0 factor failed or its terms are not finite: then
 * nothing of that round is consumed and *pending = 1 (the caller evaluates that round
 * through the jitter ladder and hands the results to evr_lbfgsb_advance). */
int evr_mll_fit_rounds(void* stream, evr_mll_plan* plan, void** runs, int* task, double* x, double* f, double* g,
                       int* nit, int* nfev, int* status, int maxiter, int maxfun, const double* prior, double* params,
                       int* pending);
/* Host-only.  ll / n and its gradient in x = [noise, constant, raw lengthscales] per member
 * (B x (d + 2)), the ExactMarginalLogLikelihood with the hyperparameter priors (prior as in
 * evr_mll_fit_rounds) divided by n, from the plan's terms (B x 5) and lengthscale-gradient
 * pieces gls (B x d): the closure of fit_gpytorch_mll (bofire/surrogates/single_task_gp.py:70-71)
 * after the device work; evr_mll_fit_rounds applies the same code. */
int evr_mll_assemble(int B, int n, int d, const double* prior, const double* x, const double* terms,
                     const double* gls, double* ll, double* g);
/* One member's L-BFGS-B after its evaluation at x (f, g): scipy's driver loop up to the next
 * evaluation request or the end (the state machine evr_mll_fit_rounds applies). */
int evr_lbfgsb_advance(void* run, double f, const double* g, double* x, int* task, int* nit, int* nfev,
                       int* status, int maxiter, int maxfun);

/* ---- dense float64 linear algebra --------------------------------------------------- */
int evr_gemm_f64(void* stream, int transA, int transB, int M, int N, int K, double alpha,
                 const double* A, int lda, long long strideA, const double* B, int ldb,
                 long long strideB, double beta, double* C, int ldc, long long strideC, int batch);

/* Batched Cholesky with [upstream] linear_operator psd_safe_cholesky semantics: plain
 * attempt, then total diagonal jitter jitter0*10^(t-1) for t = 1..max_tries; info[b] = 0
 * on success, 1 if still not p.d. (NotPSDError).  A and L must not alias.
 * Replaces the Cholesky behind GPyTorch exact inference (K + sigma^2 I), the qNEHVI
 * baseline root (bofire/strategies/predictives/qnehvi.py:46, cache_root=True) and the
 * prune-sampling root (qnehvi.py:44, prune_baseline=True). */
int evr_cholesky(void* stream, int batch, int n, const double* A, int lda, long long strideA,
                 double* L, int ldl, long long strideL, double jitter0, int max_tries,
                 double* jitter_used, int* info);

/* evr_cholesky plus L^-1 (Linv) from the same blocked pass (diagonal-block inverses are
 * by-products of the factorisation).  A, L and Linv must not alias. */
int evr_cholesky_inverse(void* stream, int batch, int n, const double* A, int lda, long long strideA,
                         double* L, int ldl, long long strideL, double* Linv, int ldi,
                         long long strideI, double jitter0, int max_tries, double* jitter_used,
                         int* info);

/* In-place B <- L^-1 B (transpose=0) or L^-T B (transpose=1); L lower, n x n; B n x nrhs. */
int evr_trsm_lower(void* stream, int batch, int n, int nrhs, const double* L, int ldl,
                   long long strideL, int transpose, double* B, int ldb, long long strideB);
int evr_tri_inv_lower(void* stream, int batch, int n, const double* L, int ldl, long long strideL,
                      double* Linv, int ldi, long long strideI);

/* ---- GP posterior --------------------------------------------------------------------
 * Given R[b] = [Linv_b; alpha_b^T] * K(Xtr, Xtest)  ((n+1) x nt per output, ld nt):
 * mean[b][t] = ym[b] + ys[b]*(c[b] + R[b][n][t]);
 * var[b][t]  = ys[b]^2 * (kxx[b] - sum_{i<n} R[b][i][t]^2 + noise_add[b]).
 * Replaces [upstream] GPyTorch exact prediction (fast_pred_var covar cache) + Standardize
 * untransform, called at bofire/strategies/predictives/botorch.py:180 and
 * bofire/surrogates/botorch.py:27-33. */
int evr_gp_posterior_finalize(void* stream, int B, int n, int nt, const double* R,
                              const double* c, const double* ym, const double* ys,
                              const double* kxx, const double* noise_add,
                              double* mean, double* var);

/* Whole posterior in one call: K_x = k(Xn, normalize(X)) (kernel_matrix), then the moments
 * of R = M K_x (M = [Linv; alpha^T], B x (n+1) x n) without storing R: per 32-row tile sums
 * of squares, finalised as above by each column tile's last-arriving workgroup.  work:
 * evr_gp_posterior_workspace_doubles(B, n, nt) doubles (K_x, the row-tile partials, the mean
 * row and the arrival counters), 16-byte aligned, contents irrelevant on entry. */
long long evr_gp_posterior_workspace_doubles(int B, int n, int nt);
int evr_gp_posterior(void* stream, int B, int n, int nt, int d, int kind, const double* Xn, const double* X,
                     const double* shift, const double* scale, const double* lengthscales, const double* M,
                     const double* c, const double* ym, const double* ys, const double* kxx,
                     const double* noise_add, double* mean, double* var, double* work);

/* ---- qNEHVI (q = 1) -----------------------------------------------------------------
 * Replaces [upstream] qNoisyExpectedHypervolumeImprovement.forward/backward as built at
 * bofire/strategies/predictives/qnehvi.py:39-52 (cached-Cholesky sampling + box-cell HVI).
 * Per output j the precomputed operator M_j = [Linv; G; H^T; alpha^T] (rows Rr =
 * n + nb + S + 1; n + nb + 1 with no_h) has been applied to k(Xtr, x): R_j = M_j K_x
 * (Rr x b, ld b). */
typedef struct {
  int n, nb, S, m;          /* train points, pruned baseline, MC samples, objectives */
  const double* c;          /* m: constant mean (standardized space) */
  const double* ym;         /* m: Standardize mean */
  const double* ys;         /* m: Standardize std */
  const double* kxx;        /* m: prior variance k(x,x) */
  const double* zq;         /* S x m: base samples of the new point */
  const double* obj_a;      /* m: objective g_j = a_j*y_j + b_j */
  const double* obj_b;      /* m */
  /* box-decomposition cells (maximisation space), AoS per cell, ragged per sample */
  const double* cell_lo;    /* total_cells x m */
  const double* cell_hi;    /* total_cells x m (may be +inf) */
  const int* cell_off;      /* S + 1 */
  int max_cells;            /* max_s (cell_off[s+1] - cell_off[s]) — host-known, sizes the launch */
  /* compressed cells (device box decomposition, evr_box_pack_keys_device): when cell_keys is
   * not NULL the scan rebuilds every cell from its 64-bit key of defining-point indices and
   * the sample's point table, and cell_lo / cell_hi are not read. */
  const unsigned long long* cell_keys; /* total_cells */
  const double* cell_pts;   /* S x pts_stride x m: minimisation-space points, then m dummies */
  const int* cell_rank0;    /* S x pts_stride: point index of rank r (key field 0) */
  int pts_stride;           /* rows per sample of cell_pts / cell_rank0 */
  /* kd-ordered cell groups (evr_cells_kd_order_device, needs the compressed cells above):
   * when grp_off is not NULL the scan runs the sparse group -> cell -> term filter */
  const int* grp_off;                  /* S + 1: group offsets, 16 cells per group */
  const unsigned long long* grp_keys;  /* grp_off[S]*16 cell keys in kd order (field 0: point index) */
  const unsigned short* grp_rank;      /* grp_off[S] x m x 16 per-cell lower-bound ranks (0x7FFF pad) */
  const unsigned short* grp_box;       /* grp_off[S] x 8: per-group minimum rank per objective */
  const double* sorted_lo;             /* S x m x pts_stride ascending lower-bound values */
  int max_groups;                      /* max_s (grp_off[s+1] - grp_off[s]) */
  /* optional scan statistics (nullable, device): [0] += passing (candidate, group) pairs,
   * [1] += exact (cell, candidate) terms evaluated, [2] += (candidate, group) tests,
   * [3] += (candidate, 16-group chunk) entries passing the chunk pre-filter (hvi_kd2) */
  unsigned long long* scan_counters;
  /* 0: M = [Linv; G; H^T; alpha^T] (qNEHVI).  1: M carries no H^T rows (Rr = n + nb + 1) and
   * the samples have no baseline term, y_s = mu + L22 zq_s — qEHVI, where the cells come
   * from the observed Pareto front instead of per-sample baseline draws (nb = 0). */
  int no_h;
  /* 1: log-space scan (qLogNEHVI / qLogEHVI, fat = True): acq = logmeanexp_s logsumexp_cells
   * sum_j fatmin(log fatplus(y_j - l_j; tau_relu), log(min(u_j, 1e10) - l_j); tau_max), dense
   * over every cell; needs the explicit cells cell_lo / cell_hi (keys and kd groups unused). */
  int log_hvi;
  double tau_relu, tau_max;
} evr_qnehvi_state;

/* samples: G[s][j][c] = g_j(mu_j + h_js + L22_j zq[s][j]); aux L22: m x b; flags: m x b
 * (0 ok, 1 new-block Cholesky failed after 6 jitter tries). */
int evr_qnehvi_samples(void* stream, const evr_qnehvi_state* st, int b, const double* R,
                       double* G, double* L22, int* flags);
/* Workspace (doubles) the HVI scan needs for b candidates (per-(sample, cell-chunk)
 * partials); backward != 0 sizes it for evr_hvi_backward / evr_hvi_forward_backward. */
long long evr_hvi_workspace_doubles(const evr_qnehvi_state* st, int b, int backward);
/* acq[c] = mean_s HVI_s(G[s][:, c]) over the cells of sample s (register-tiled cell x
 * candidate scan, deterministic two-stage reduction); acq[c] = NaN where flags (m x b,
 * from evr_qnehvi_samples, nullable) report a failed new-point Cholesky block. */
int evr_hvi_forward(void* stream, const evr_qnehvi_state* st, int b, const double* G,
                    const int* flags, double* work, double* acq);
/* acq[c] = mean_s partial[s][c] */
int evr_mean_over_samples(void* stream, int S, int b, const double* partial, double* acq);
/* dG[s][j][c] = gout[c]/S * dHVI_s/dg_j (torch min/clamp_min/prod subgradients; gout NULL = 1) */
int evr_hvi_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G,
                     const double* gout, double* work, double* dG);
/* One fused scan: acq (as evr_hvi_forward, NaN on flags) and dG (as evr_hvi_backward). */
int evr_hvi_forward_backward(void* stream, const evr_qnehvi_state* st, int b, const double* G,
                             const int* flags, const double* gout, double* work, double* acq,
                             double* dG);
/* Restart-batch scan (kd cells, b <= 32) in one launch (hvi_kdw: one wave per sample and
 * candidate): what evr_hvi_forward_backward (gout = NULL) computes, in the wave's own
 * summation order.  sval (S x b) holds the per-sample HVI values, acq = their mean
 * (evr_mean_over_samples; the plan folds it into the dX reduction).  _applies: 1 when the
 * state / batch qualifies. */
int evr_hvi_restart_fb_applies(const evr_qnehvi_state* st, int b);
int evr_hvi_restart_fb(void* stream, const evr_qnehvi_state* st, int b, const double* G, double* sval,
                       double* dG);
/* gR_j (Rr x b): gradient w.r.t. R_j given dG (chains objective, sampling, L22 ladder) */
int evr_qnehvi_samples_backward(void* stream, const evr_qnehvi_state* st, int b, const double* R,
                                const double* L22, const double* dG, double* gR);

/* Fused projection path (qnehvi_proj.hip), replacing gemm + evr_qnehvi_samples +
 * evr_qnehvi_samples_backward + gemm^T:
 * evr_qnehvi_project: R_j = M_j Kx_j (M: m x Rr x n, Kx: m x n x b, R: m x Rr x b) and the
 *   per-64-row-tile partial sums of squares norms (m x evr_qnehvi_norms_rows(st) x 2 x b).
 * evr_qnehvi_samples_norms: G, L22, flags as evr_qnehvi_samples, from R's sample / mean rows
 *   and the partial norms.
 * evr_qnehvi_project_backward: dKx_j = M_j^T gR_j (n x b per output) with gR generated in
 *   the K loop from R, L22 and dG (never written to memory).
 * `work` (split-K partials, gR coefficients): the *_workspace_doubles size, NULL = allocate. */
int evr_qnehvi_norms_rows(const evr_qnehvi_state* st);
int evr_qnehvi_project(void* stream, const evr_qnehvi_state* st, int b, const double* M, const double* Kx,
                       double* R, double* norms, double* work);
long long evr_qnehvi_project_workspace_doubles(const evr_qnehvi_state* st, int b);
int evr_qnehvi_samples_norms(void* stream, const evr_qnehvi_state* st, int b, const double* R,
                             const double* norms, double* G, double* L22, int* flags);
int evr_qnehvi_project_backward(void* stream, const evr_qnehvi_state* st, int b, const double* M,
                                const double* R, const double* L22, const double* dG, double* dKx,
                                double* work);
long long evr_qnehvi_project_backward_workspace_doubles(const evr_qnehvi_state* st, int b);

/* Native evaluation plan of the whole qNEHVI chain (qnehvi_plan.hip): K_x, fused projection,
 * samples, HVI scan (+ backward: projection^T with generated gR, cross-covariance gradient)
 * in one call, every intermediate carved from `work`, optionally captured into a hipGraph
 * (use_graph) and replayed by evr_qnehvi_plan_run.  X: b x d raw (transformed) candidates;
 * acq: b; dX: b x d (backward).  The plan copies *st / *md; the buffers they and X / work /
 * acq / dX point to must outlive the plan.
 * Replaces one [upstream] qNoisyExpectedHypervolumeImprovement forward (+ autograd backward)
 * call of gen_candidates_scipy (bofire/strategies/predictives/botorch.py:384-405). */
typedef struct {
  int n, d, kind;              /* training points, input dims, EVR_KERNEL_* */
  const double* Xn;            /* n x d normalized training inputs */
  const double* lengthscales;  /* m x d */
  const double* shift;         /* d: Normalize lower bounds (candidates arrive raw) */
  const double* scale;         /* d: 1 / (upper - lower) */
  const double* M;             /* m x (n + nb + S + 1) x n forward operator [Linv; G; H^T; alpha^T] */
} evr_qnehvi_model;
typedef struct evr_qnehvi_plan evr_qnehvi_plan;
long long evr_qnehvi_plan_workspace_bytes(const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                                          int backward);
int evr_qnehvi_plan_create(void* stream, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                           int backward, const double* X, void* work, double* acq, double* dX, int use_graph,
                           evr_qnehvi_plan** out);
/* The b <= 32 (restart-batch) pieces of the plan chain, exposed op by op for measurement and
 * parity tests (qnehvi_small.hip): small_forward R, P (16-row norm tiles) from Kx; small_samples
 * G, L22, flags from them; small_backward dX (b x d, the cross-covariance gradient fused) from
 * R, L22, dG and the candidates X.  workspace_doubles(which = 0: P, 1: dXp). */
int evr_qnehvi_small_applies(const evr_qnehvi_state* st, int b, int d);
long long evr_qnehvi_small_workspace_doubles(const evr_qnehvi_state* st, int b, int d, int which);
int evr_qnehvi_small_forward(void* stream, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                             const double* Kx, double* R, double* P);
int evr_qnehvi_small_samples(void* stream, const evr_qnehvi_state* st, int b, const double* R, const double* P,
                             double* G, double* L22, int* flags);
int evr_qnehvi_small_backward(void* stream, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                              const double* X, const double* R, const double* L22, const double* dG, double* dXp,
                              double* dX);
int evr_qnehvi_plan_run(void* stream, evr_qnehvi_plan* plan);
/* One evaluation at host x (b x d): out (host) = [acq (b) | dX (b x d, backward plans)].
 * Runs a second graph [copy-in from fine-grained pinned memory, the chain, copy-out + a
 * completion word] and spins on that word: no blit copies and no stream synchronise per
 * evaluation (the hot loop of evr_qnehvi_plan_minimize; botorch's per-evaluation
 * forward+backward of gen_candidates_scipy's objective). */
int evr_qnehvi_plan_eval_host(void* stream, evr_qnehvi_plan* plan, const double* x, double* out);
void evr_qnehvi_plan_destroy(evr_qnehvi_plan* plan);

/* ---- acquisition restarts: native L-BFGS-B ------------------------------------------
 * Restatement of the bound-constrained L-BFGS-B (v3.0: Cauchy point, direct primal
 * subspace step with projection / backtracking, More-Thuente line search) that
 * scipy.optimize.minimize(method="L-BFGS-B") runs inside [upstream] botorch
 * gen_candidates_scipy, called by optimize_acqf from
 * bofire/strategies/predictives/botorch.py:384-405 (box bounds, no linear constraints).
 * Host-only.  Reverse communication: evr_lbfgsb_start returns EVR_LBFGSB_FG with the
 * (projected) x to evaluate; evr_lbfgsb_step(f, g at x) returns the next task and x.
 * m: corrections (scipy maxcor 10), factr = ftol / eps (1e7), pgtol (1e-5), maxls (20). */
#define EVR_LBFGSB_FG 1
#define EVR_LBFGSB_NEW_X 2
#define EVR_LBFGSB_CONV_PGTOL 3
#define EVR_LBFGSB_CONV_FACTR 4
#define EVR_LBFGSB_ABNORMAL 5
#define EVR_LBFGSB_ERROR 6
typedef struct evr_lbfgsb evr_lbfgsb;
int evr_lbfgsb_create(int n, int m, const double* lb, const double* ub, double factr, double pgtol, int maxls,
                      evr_lbfgsb** out);
int evr_lbfgsb_start(evr_lbfgsb* h, const double* x0, double* x);
int evr_lbfgsb_step(evr_lbfgsb* h, double f, const double* g, double* x);
void evr_lbfgsb_stats(const evr_lbfgsb* h, int* nit, int* nfev, double* f, double* pgnorm);
void evr_lbfgsb_destroy(evr_lbfgsb* h);

/* Hit-and-run sampler over {x : A x <= b} (rows x d, row-major), moving in x0 + span(N)
 * (N: d x k, row-major; k = d and N = I without equality constraints).  x0 must be
 * interior.  n_burnin + n * n_thinning steps from x0; every n_thinning-th step after the
 * burn-in is written to out (n x d).  Step i draws its variates 2k + 1 from a counter-based
 * SplitMix64 stream at counters i (2k + 1) + j: k Box-Muller normals (cos branch) for the
 * direction, one uniform for the point on the chord.  Host-only.
 * Replaces [upstream] HitAndRunPolytopeSampler / sample_q_batches_from_polytope, called by
 * optimize_acqf under linear constraints (bofire/strategies/predictives/botorch.py:384-405)
 * and by RandomStrategy (bofire/strategies/random.py:300-326). */
int evr_hit_and_run(int d, int rows, const double* A, const double* b, int k, const double* N,
                    const double* x0, long long n, unsigned long long seed, long long n_burnin,
                    long long n_thinning, double* out);

/* One joint restart problem driven natively on a backward plan: minimise
 * -sum_r acq(x_r) over the b restarts of `plan` in the box [lb, ub] (b*d host arrays each)
 * from x0 (b*d host), with scipy's wrapper rules (stop after maxiter iterations or more
 * than maxfun evaluations).  Each evaluation is one evr_qnehvi_plan_eval_host on `stream`,
 * with no Python in the loop.  Outputs (host): x (b*d,
 * clipped to the box), acq (b) at x, info[4] = {iterations, evaluations, status (0
 * converged, 1 iteration/evaluation limit, 2 abnormal line search), last task}.
 * Returns EVR_ERR_NOTPSD when an evaluation yields NaN (a new-point posterior block not
 * p.d. after the jitter ladder: [upstream] NotPSDError). */
#define EVR_ERR_NOTPSD 7
int evr_qnehvi_plan_minimize(void* stream, evr_qnehvi_plan* plan, const double* x0, const double* lb,
                             const double* ub, int maxiter, int maxfun, double factr, double pgtol, int m,
                             int maxls, double* x, double* acq, int* info);

/* ---- general qNEHVI / qEHVI evaluation (qnehvi_general.hip) ---------------------------
 * q >= 1 joint candidate batches (inclusion-exclusion over the 2^q - 1 subsets of the q
 * points), objectives over selected model outputs (Maximize / Minimize: a*y + b;
 * CloseToTarget: -|y - t|^e) and output constraints c(y) = sign*(y_out - thr) <= 0 weighted
 * by exp(sum logsigmoid(-c/eta)).  Replaces [upstream] qNoisyExpectedHypervolumeImprovement /
 * qExpectedHypervolumeImprovement forward + backward with q = candidate_count
 * (bofire/strategies/predictives/botorch.py:385), objective = get_multiobjective_objective
 * (bofire/utils/torch_tools.py:699-727, callables :384-402) and constraints / eta from
 * get_output_constraints (torch_tools.py:258-381, passed at
 * bofire/strategies/predictives/qnehvi.py:28-48 and mobo.py:50-86).
 * Model side: `stm` (m = model outputs; operator M / R layout as for q = 1, zq unused) and
 * `md`; scan side: `sth` (m = m_obj objectives, the cells, log_hvi = 0).  X: (b*q) x d raw
 * candidates, point i of candidate c at row c*q + i; acq: b; dX (NULL = forward only):
 * (b*q) x d; gout (nullable, b) weights the backward.  The objective / constraint arrays are
 * HOST arrays (copied into the launch); zq (S x q x m_model) is on the device. */
#define EVR_OBJ_AFFINE 0
#define EVR_OBJ_CLOSE_TO_TARGET 1
#define EVR_QNG_MAX_Q 12
typedef struct {
  int q;                    /* points per candidate, 1..8 */
  int m_obj;                /* objectives, 1..8 */
  const int* obj_out;       /* m_obj: model output index */
  const int* obj_kind;      /* m_obj: EVR_OBJ_* */
  const double* obj_p0;     /* m_obj: a (affine) / target (close-to-target) */
  const double* obj_p1;     /* m_obj: b (affine) / exponent (close-to-target) */
  int n_con;                /* output constraints, 0..16 */
  const int* con_out;       /* n_con: model output index */
  const double* con_sign;   /* n_con: c = sign*(y - thr) */
  const double* con_thr;
  const double* con_eta;    /* n_con: sigmoid temperature (BoFire: 1/steepness) */
  const double* zq;         /* device, S x q x m_model: base samples of the q new points */
} evr_qn_general;
long long evr_qng_workspace_doubles(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth,
                                    const evr_qn_general* g, const evr_qnehvi_model* md, int b, int backward);
int evr_qng_eval(void* stream, const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                 const evr_qnehvi_model* md, int b, const double* X, const double* gout, double* work,
                 double* acq, double* dX);
/* Log-space general evaluation ([upstream] qLogExpectedHypervolumeImprovement._compute_log_qehvi,
 * fat = True; qLogNEHVI / qLogEHVI, MoboStrategy's default, bofire/strategies/predictives/
 * mobo.py:47-90): as evr_qng_eval, with `sth` carrying EXPLICIT cells (cell_lo / cell_hi /
 * cell_off) and tau_relu / tau_max; per cell the q-subset areas are combined in log space
 * (log fatplus improvements, fat-min over the subset's points and with the log cell lengths,
 * log feasibilities summed over the subset, odd minus even sizes by logdiffexp), logsumexp
 * over the cells, logmeanexp over the samples. */
long long evr_qlog_workspace_doubles(const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                                     const evr_qnehvi_model* md, int b, int backward);
int evr_qlog_eval(void* stream, const evr_qnehvi_state* stm, const evr_qnehvi_state* sth, const evr_qn_general* g,
                  const evr_qnehvi_model* md, int b, const double* X, const double* gout, double* work,
                  double* acq, double* dX);
/* Objectives of baseline / prune samples (Y: m_model x n x S plus mu: m_model x n, nullable)
 * with hard feasibility: O[k][i][s] = g_k(y), or ref[k] where any constraint c > 0
 * ([upstream] prune_inferior_points_multi_objective and the qNEHVI baseline partitions drop
 * infeasible samples).  g->q / g->zq unused. */
int evr_objective_general(void* stream, int m_model, int n, int S, const evr_qn_general* g, const double* Y,
                          const double* mu, const double* ref, double* O);
/* Objective values and smoothed feasibility weights of model-output rows (Y: m_model x n,
 * output-major) through the per-point function the general scan applies to every MC sample:
 * G[k][i] = g_k(y_i) (get_objective_callable, bofire/utils/torch_tools.py:384-402) and
 * W[i] = exp(sum_c logsigmoid(-c(y_i) / eta_c)) ([upstream] compute_smoothed_feasibility_indicator
 * over the constrained_objective2botorch callables, torch_tools.py:258-337; W = 1 without
 * constraints).  g->q / g->zq unused. */
int evr_objective_weights(void* stream, int m_model, int n, const evr_qn_general* g, const double* Y, double* G,
                          double* W);

/* The PyTorch-ROCm operators torch.ops.everest_amd.qnehvi_* (everest_amd/csrc/torch_ops.cpp)
 * take a torch.classes.everest_amd.QnehviAcq: it copies the evr_qnehvi_state /
 * evr_qnehvi_model / evr_qn_general structs, holds references to the device tensors they
 * point into, and caches one plan per batch size (no raw addresses cross the boundary). */

/* ---- qEI (q = 1, single output) -----------------------------------------------------
 * R = [Linv; alpha^T] K(Xtr, x) ((n+1) x b).  acq[c] = mean_s (a*(mu + sd*z_s) + b - best_f)_+
 * with sd from psd_safe_cholesky (3 tries) of the posterior variance; gR (nullable) =
 * d acq / d R for the analytic backward; flags[c] = 1 if the jitter ladder failed.
 * Replaces [upstream] qExpectedImprovement (bofire/strategies/predictives/sobo.py:51-90). */
int evr_qei(void* stream, int n, int b, int S, const double* R, double c, double ym, double ys,
            double kxx, const double* z, double obj_a, double obj_b, double best_f, double* acq,
            double* gR, int* flags);

/* ---- Pareto / pruning ---------------------------------------------------------------
 * O: m x n x S (objective samples, layout [j][i][s]).  For every sample s and point i:
 * nd = not dominated (maximisation) & (O > ref all) [& first of duplicates if dedup].
 * mask (S x n bytes, may be NULL); counts (n ints, may be NULL) += nd.
 * Replaces prune_inferior_points_multi_objective (qnehvi.py:44) and the per-sample
 * Pareto filter of _pad_batch_pareto_frontier. */
int evr_pareto_mask(void* stream, int S, int n, int m, const double* O, const double* ref,
                    int dedup, unsigned char* mask, int* counts);

/* Elementwise objective on a sample tensor: O[j][i][s] = a_j*(Y[j][i][s] + mu[j][i]) + b_j */
int evr_objective_affine(void* stream, int m, int n, int S, const double* Y, const double* mu,
                         const double* a, const double* b, double* O);
/* X[b][e] *= alpha[b] for e < per (per-output variance scaling s_y^2 of covariances) */
int evr_scale_batched(void* stream, int B, long long per, const double* alpha, double* X);
/* E[b][r][idx[r]] += val[b] (adds the baseline row selection P to E, nb x n per output) */
int evr_add_selection(void* stream, int B, int nb, int n, const int* idx, const double* val, double* E);

/* ---- host box decomposition ----------------------------------------------------------
 * Exact partition of the non-dominated region above ref into disjoint boxes, per MC sample
 * (FastNondominatedPartitioning, alpha = 0, qnehvi.py:50; Lacour et al. 2017 local upper
 * bounds).  Host memory.  obj: element (s, i, j) at obj[s*ss + i*si + j*sj]; mask (S x n,
 * nullable) selects the candidate points (Pareto filter is re-applied on the host). */
typedef struct evr_cells evr_cells;
int evr_box_decompose(int S, int n, int m, const double* obj, long long ss, long long si,
                      long long sj, const unsigned char* mask, const double* ref, int num_threads,
                      evr_cells** out);
/* alpha > 0 (finite) with m > 2: the approximate partition of [upstream] BoTorch
 * NondominatedPartitioning(alpha) (bofire/strategies/predictives/qnehvi.py:50 passes the data
 * model's alpha, bofire/data_models/strategies/predictives/qnehvi.py:19); alpha = 0 or m <= 2
 * is the exact partition above. */
int evr_box_decompose_approx(int S, int n, int m, const double* obj, long long ss, long long si,
                             long long sj, const unsigned char* mask, const double* ref, double alpha,
                             int num_threads, evr_cells** out);
long long evr_cells_total(const evr_cells* c);
int evr_cells_copy(const evr_cells* c, double* lo, double* hi, int* off);
void evr_cells_free(evr_cells* c);

/* ---- device box decomposition (same partition as evr_box_decompose) --------------------
 * One workgroup per sample; obj is m x n x S on the device (objective values, maximisation),
 * ref (m) on the device.  Every LUB is a 64-bit key of defining-point indices, cap keys per
 * sample (power of two).  status[s] = 1 if sample s overflowed cap (retry with a larger
 * cap).  counts[s] = number of non-empty cells.  evr_box_pack_keys_device then packs the
 * sorted keys at off[s] (cells ordered by first lower bound) with the per-sample point tables
 * pts (S x (n+m) x m) and rank0 (S x (n+m)) -> evr_qnehvi_state.cell_keys / cell_pts /
 * cell_rank0, pts_stride n+m.  evr_cells_from_keys expands them into explicit lo / hi rows.
 * evr_box_device_limits returns 0 if (n, m) fits the kernel (LDS, key width), else 3. */
int evr_box_device_limits(int n, int m, int* max_points, long long* lds_bytes);
long long evr_box_device_workspace_bytes(int S, int n, int m, int cap);
int evr_box_decompose_device(void* stream, int S, int n, int m, const double* obj, const double* ref,
                             int cap, void* work, int* counts, int* status);
int evr_box_pack_keys_device(void* stream, int S, int n, int m, int cap, const void* work,
                             const int* off, int max_cells, unsigned long long* keys, double* pts,
                             int* rank0);
int evr_cells_from_keys(void* stream, int S, int m, int stride, const int* off, int max_cells,
                        const unsigned long long* keys, const double* pts, const int* rank0,
                        double* lo, double* hi);

/* ---- kd ordering of compressed cells for the sparse HVI scan -------------------------
 * Per sample (one workgroup each): rank tables of the point rows per objective, a kd split
 * order of the cells (median split on the objective of largest rank spread, leaves of 16),
 * then per group of 16 cells: the keys (okeys, goff[S]*16), the cells' lower-bound ranks
 * (ork, goff[S] x m x 16 u16, 0x7FFF padding), the group's minimum rank per objective (ogb,
 * goff[S] x 8 u16) and per sample the ascending lower-bound values (osv, S x m x stride).
 * goff[s] = sum_{s'<s} ceil(counts[s'] / 16).  evr_cells_kd_limits returns 0 if max_cells /
 * stride fit the kernel (LDS sort buffer), else 3 (the tiled scan is used then).
 * Replaces nothing in the reference: an MI355X-side index over the [upstream]
 * FastNondominatedPartitioning cells (bofire/strategies/predictives/qnehvi.py:50). */
/* evr_box_decompose_device + evr_box_pack_keys_device + evr_cells_kd_order_device in one host
 * call with one synchronisation (the per-sample counts): outputs sized by the caller for the
 * capacity (keys S*cap; okeys 16*G, ork 16*m*G, ogb 8*G with G = S*cap/16 + S; off / goff S+1);
 * info[0] = 1: a sample overflowed cap (rerun with a larger cap), info[1] = 1: kd order built,
 * info[2] = largest per-sample count; counts_host[s] = cells of sample s.  Replaces the
 * reference's host-side partition + cell list (bofire/strategies/predictives/qnehvi.py:39-52
 * -> [upstream] FastNondominatedPartitioning) for the sparse scan in one step. */
int evr_box_kd_pipeline(void* stream, int S, int n, int m, const double* obj, const double* ref, int cap,
                        void* work, int* counts_dev, int* status_dev, int* off_dev, int* goff_dev,
                        unsigned long long* keys, double* pts, int* rank0, int want_kd, unsigned long long* okeys,
                        unsigned short* ork, unsigned short* ogb, double* osv, int* counts_host, int* info);
int evr_cells_kd_limits(int stride, int m, int max_cells, long long* lds_bytes);
int evr_cells_kd_order_device(void* stream, int S, int m, int stride, const int* off, const int* goff,
                              int max_cells, const unsigned long long* keys, const double* pts,
                              const int* rank0, unsigned long long* okeys, unsigned short* ork,
                              unsigned short* ogb, double* osv);

/* ---- quasi-MC base samples -------------------------------------------------------------
 * Replaces [upstream] draw_sobol_normal_samples / torch.quasirandom.SobolEngine(scramble=True)
 * as called by the qNEHVI samplers (bofire/strategies/predictives/qnehvi.py:39-52, seed from
 * the strategy RNG bofire/strategies/predictives/botorch.py:86).
 * evr_sobol_scramble (host): V (dim x 30 int64, in/out) holds the unscrambled direction
 * numbers and receives SobolEngine(dim, scramble=True, seed).sobolstate; shift (dim) receives
 * .shift.  evr_sobol_normal (device): normal samples of points 0..n-1, dims [d0, d0+nd):
 * layout 0 -> out[k*nd + t]; layout 1 -> out[(o*np + p)*n + k] with t = p*m + o, np = nd/m. */
int evr_sobol_scramble(int dim, unsigned long long seed, long long* V, long long* shift);
/* The same for dimensions [d0, d0 + nd) of the dim-dimensional engine only: V (nd x 30) and
 * shift (nd) hold those dimensions (the stream is still drawn through dimension d0 + nd - 1;
 * the per-dimension work is skipped for the others). */
int evr_sobol_scramble_range(int dim, unsigned long long seed, int d0, int nd, long long* V, long long* shift);
/* The same in two steps: generate a seed's raw stream once (evr_sobol_stream_words(dim)
 * words cover every draw of up to dim dimensions; the draws of one seed at different
 * dimension counts are prefixes of the same stream), then scramble dimension ranges of any
 * dim it covers.  Lets the host start the stream before the dimension count is known. */
typedef struct evr_sobol_stream evr_sobol_stream;
long long evr_sobol_stream_words(int dim);
int evr_sobol_stream_create(unsigned long long seed, long long nwords, evr_sobol_stream** out);
int evr_sobol_scramble_stream(const evr_sobol_stream* st, int dim, int d0, int nd, long long* V, long long* shift);
void evr_sobol_stream_destroy(evr_sobol_stream* st);
int evr_sobol_normal(void* stream, int n, int nd, int d0, const long long* V, const long long* shift,
                     int layout, int m, double* out);

#ifdef __cplusplus
}
#endif
#endif /* EVEREST_AMD_H */
