// Native evaluation plan of the exact-GP marginal log likelihood and its gradient for the
// GP fit (tell(): [upstream] fit_gpytorch_mll -> scipy L-BFGS-B over ExactMarginalLogLikelihood,
// bofire/surrogates/single_task_gp.py:70-71).  One evaluation of B GPs that share the
// normalised inputs is one hipGraph launch:
//   [hyperparameters from pinned host memory] -> K + noise I -> psd_safe_cholesky attempt 0
//   (fused blocked factor + triangular inverse) -> r = y - c -> alpha = K^-1 r ->
//   W = alpha alpha^T - K^-1 -> dMLL/dlengthscale -> the scalar terms -> [terms, gradient
//   pieces and the Cholesky info to pinned host memory, completion word].
// The host spins on the completion word (no blit copies, no stream synchronise, no per-op
// launch cost): at n = 512 the per-evaluation cost of the unfused op chain was ~1.4 ms,
// mostly launch and synchronisation latency.  A member whose attempt-0 factor fails is
// reported through info; the caller reruns that evaluation through the jitter ladder.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "common.hpp"
#include "gemm_core.hpp"
#include "../../include/everest_amd.h"

namespace evr {
int chol_inverse_attempt(hipStream_t s, int batch, int n, const double* A, double* L, double* Linv, double* Dinv,
                         double* T, const double* jit_d, int* info_d);
size_t chol_inverse_dinv_doubles(int batch, int n);
int gemm_plain(hipStream_t s, bool tA, bool tB, int M, int N, int K, double alpha, const double* A, int lda,
               long long sA, const double* B, int ldb, long long sB, double beta, double* C, int ldc, long long sC,
               int batch);
size_t mll_terms_part_doubles(int B);
int mll_terms_chunks();
int mll_terms_partials(hipStream_t s, int B, int n, const double* L, const double* Linv, const double* r,
                       const double* alpha, double* part);

// W = alpha alpha^T - K^-1 = alpha alpha^T - L^-T L^-1 in one launch of the gemm_core.hpp
// engine (A = L^-T: L^-1 read m-contiguous).  L^-1 is lower triangular, so W[i][j] sums over
// k >= max(i, j) only: tile (by, bx) contracts over k >= 32 max(by, bx), the skipped terms
// exact zeros.  W is symmetric: only the lower tiles (by >= bx) are formed — ascending by,
// i.e. longest k range first, outputs interleaved — and each off-diagonal tile is also written
// transposed, through LDS as 256-byte row segments (W exactly symmetric; half the MFMA work of
// forming every tile).  The rank-1 alpha alpha^T term is the epilogue.
using MllW = DgCfg<32, 32, 16, true>;

template <bool VEC>
__global__ __launch_bounds__(256, 4) void mll_w_kernel(int n, int B, const double* __restrict__ Linv,
                                                       const double* __restrict__ alpha, double* __restrict__ W) {
  using C = MllW;
  static_assert(C::BM == C::BN, "square tiles");
  __shared__ double lds[C::LDS_DOUBLES > C::BM * (C::BN + 1) ? C::LDS_DOUBLES : C::BM * (C::BN + 1)];
  const int f = blockIdx.x, j = f % B, t = f / B;
  int by = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);   // lower tiles, row-major: row by holds by + 1
  while ((by + 1) * (by + 2) / 2 <= t) ++by;
  while (by * (by + 1) / 2 > t) --by;
  const int bx = t - by * (by + 1) / 2;
  const int m0 = by * C::BM, n0 = bx * C::BN;
  const size_t nn = (size_t)n * n;
  const double* Lj = Linv + j * nn;
  const int kbeg = m0;   // max(m0, n0): bx <= by
  dg_double4 acc[C::FM][C::FN];
  dg_mainloop<C>(
      lds, kbeg, n,
      [&](int k, int c) -> dg_double2 {
        return dg_pair<VEC>(Lj + (size_t)k * n + m0 + c, k < n && m0 + c < n, k < n && m0 + c + 1 < n);
      },
      [&](int k, int c) -> dg_double2 {
        return dg_pair<VEC>(Lj + (size_t)k * n + n0 + c, k < n && n0 + c < n, k < n && n0 + c + 1 < n);
      },
      acc);
  const double* aj = alpha + (size_t)j * n;
  double* Wj = W + j * nn;
  if (by == bx) {
    dg_for_each<C>(acc, [&](int r, int c, double v) {
      const int row = m0 + r, col = n0 + c;
      if (row < n && col < n) Wj[(size_t)row * n + col] = aj[row] * aj[col] - v;
    });
    return;
  }
  __syncthreads();   // every wave's main-loop LDS reads are done
  double(*T)[C::BN + 1] = reinterpret_cast<double(*)[C::BN + 1]>(lds);
  dg_for_each<C>(acc, [&](int r, int c, double v) {
    const int row = m0 + r, col = n0 + c;
    const double w = (row < n && col < n) ? aj[row] * aj[col] - v : 0.0;
    T[r][c] = w;
    if (row < n && col < n) Wj[(size_t)row * n + col] = w;
  });
  __syncthreads();
  // the transposed tile: row n0 + c of W holds T[.][c]; a thread per (row, 8-byte column)
  for (int e = threadIdx.x; e < C::BM * C::BN; e += 256) {
    const int c = e / C::BM, r = e - c * C::BM;
    const int row = n0 + c, col = m0 + r;
    if (row < n && col < n) Wj[(size_t)row * n + col] = T[r][c];
  }
}

// v = L^-1 r (TRANS false) and alpha = L^-T v (TRANS true) for the B members: one workgroup
// per 16 outputs of a member, L^-1's triangle only (k <= i, resp. k >= i).  Thread (output o,
// k-group g) sums k = g, g + 16, ... (non-transposed: the 16 lanes of a k-group row read 128
// contiguous bytes of row i; transposed: of row k), the 16 partials summed in g order: no
// split-K workspace and no second (reduction) launch — the split-K GEMM pair took 14 us per
// product at n = 512, almost all of it launch and reduction latency.
template <bool TRANS>
__global__ __launch_bounds__(256) void mll_matvec(int n, const double* __restrict__ L, const double* __restrict__ x,
                                                  double* __restrict__ out) {
  __shared__ double red[16][17];
  const int j = blockIdx.y, i0 = blockIdx.x * 16, t = threadIdx.x;
  const int o = TRANS ? (t & 15) : (t >> 4), g = TRANS ? (t >> 4) : (t & 15);
  const int i = i0 + o;
  const double* Lj = L + (size_t)j * n * n;
  const double* xj = x + (size_t)j * n;
  double s = 0.0;
  if (i < n) {
    const int kb = TRANS ? i0 : 0, ke = TRANS ? n : min(n, i0 + 16);
    // rounds of 8 loads in flight (k = kb + g + 16 u), the triangle's other entries skipped
    for (int k0 = kb; k0 < ke; k0 += 128) {
      double a[8], xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = min(k0 + g + 16 * u, n - 1);
        a[u] = TRANS ? Lj[(size_t)k * n + i] : Lj[(size_t)i * n + k];
        xv[u] = xj[k];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + g + 16 * u;
        if (k < ke && (TRANS ? k >= i : k <= i)) s = fma(a[u], xv[u], s);
      }
    }
  }
  red[o][g] = s;
  __syncthreads();
  if (t < 16 && i0 + t < n) {
    double v = red[t][0];
#pragma unroll
    for (int q = 1; q < 16; ++q) v += red[t][q];
    out[(size_t)j * n + i0 + t] = v;
  }
}

// hx: [ls (B x d) | noise (B) | constant (B) | sequence number]; also the residuals
// r = Y - constant (one launch: the constant comes straight from the host buffer, one read
// per wave since a wave's rows share a member when n >= 64)
__global__ void mll_copy_in(int B, int n, int d, const double* hx, const double* __restrict__ Y, double* ls,
                            double* noise, double* cst, double* __restrict__ r) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * d) ls[i] = hx[i];
  if (i < B) {
    noise[i] = hx[B * d + i];
    cst[i] = hx[B * d + B + i];
  }
  if (i < B * n) r[i] = Y[i] - hx[B * d + B + i / n];
}

// hout: [terms (B x 5: logdet, r.alpha, tr K^-1, sum alpha, sum alpha^2) | gls (B x d) |
//        info (B, as doubles) | completion word]; the terms' chunk partials summed in order
__global__ void mll_copy_out(int B, int d, int nch, const double* __restrict__ part, const double* __restrict__ gls,
                             const int* __restrict__ info, const double* hx, double* hout) {
  const int t = threadIdx.x;
  if (t < B * 5) {
    const int b = t / 5, q = t - b * 5;
    double s = 0.0;
    // the chunk partials' loads in flight together (clamped indices), summed in chunk order
    for (int c0 = 0; c0 < nch; c0 += 32) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = part[((size_t)b * nch + min(c0 + u, nch - 1)) * 5 + q];
#pragma unroll
      for (int u = 0; u < 32; ++u)
        if (c0 + u < nch) s += v[u];
    }
    hout[t] = q == 0 ? 2.0 * s : s;
  }
  for (int i = t; i < B * d; i += blockDim.x) hout[B * 5 + i] = gls[i];
  if (t < B) hout[B * 5 + B * d + t] = (double)info[t];
  __threadfence_system();
  __syncthreads();
  if (t == 0) {
    const unsigned long long seq = *(volatile const unsigned long long*)(hx + B * d + 2 * B);
    __threadfence_system();
    *(volatile unsigned long long*)(hout + B * 5 + B * d + B) = seq;
  }
}

}  // namespace evr

using namespace evr;

struct evr_mll_plan {
  int kind, B, n, d;
  const double* Xn;
  double *Y, *ls, *noise, *cst, *K, *L, *Linv, *Dinv, *T, *r, *v, *alpha, *gls, *gw, *part, *jit0;
  int* info;
  double *hx, *hout;
  hipGraph_t graph;
  hipGraphExec_t exec;
  unsigned long long seq;
};

static int mll_chain(hipStream_t s, evr_mll_plan* p, const double* dhx, double* dhout) {
  const int B = p->B, n = p->n, d = p->d;
  mll_copy_in<<<cdiv(std::max(B * d + B, B * n), 256), 256, 0, s>>>(B, n, d, dhx, p->Y, p->ls, p->noise, p->cst,
                                                                       p->r);
  EVR_LAUNCH_CHECK();
  if (int rc = evr_kernel_matrix(s, p->kind, B, n, n, d, p->Xn, nullptr, nullptr, p->Xn, nullptr, nullptr, p->ls,
                                 nullptr, p->noise, p->K))
    return rc;
  if (int rc = chol_inverse_attempt(s, B, n, p->K, p->L, p->Linv, p->Dinv, p->T, p->jit0, p->info)) return rc;
  double* W = p->K;   // K was consumed by the factorisation
  // v = L^-1 r, alpha = L^-T v: one-launch triangular matrix-vector products (mll_matvec)
  mll_matvec<false><<<dim3(cdiv(n, 16), B), 256, 0, s>>>(n, p->Linv, p->r, p->v);
  EVR_LAUNCH_CHECK();
  mll_matvec<true><<<dim3(cdiv(n, 16), B), 256, 0, s>>>(n, p->Linv, p->v, p->alpha);
  EVR_LAUNCH_CHECK();
  {
    const int T = cdiv(n, MllW::BM), lower = T * (T + 1) / 2;
    if (n % 2 == 0) mll_w_kernel<true><<<lower * B, 256, 0, s>>>(n, B, p->Linv, p->alpha, W);
    else mll_w_kernel<false><<<lower * B, 256, 0, s>>>(n, B, p->Linv, p->alpha, W);
    EVR_LAUNCH_CHECK();
  }
  if (int rc = evr_kernel_lengthscale_grad(s, p->kind, B, n, d, p->Xn, p->ls, W, p->gls, p->gw)) return rc;
  if (int rc = mll_terms_partials(s, B, n, p->L, p->Linv, p->r, p->alpha, p->part)) return rc;
  mll_copy_out<<<1, 256, 0, s>>>(B, d, mll_terms_chunks(), p->part, p->gls, p->info, dhx, dhout);
  EVR_LAUNCH_CHECK();
  return 0;
}

static void mll_free(evr_mll_plan* p) {
  if (!p) return;
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  double* bufs[] = {p->Y, p->ls, p->noise, p->cst, p->K, p->L, p->Linv, p->Dinv, p->T, p->r, p->v, p->alpha,
                    p->gls, p->gw, p->part, p->jit0};
  for (double* b : bufs)
    if (b) (void)hipFree(b);
  if (p->info) (void)hipFree(p->info);
  if (p->hx) (void)hipHostFree(p->hx);
  if (p->hout) (void)hipHostFree(p->hout);
  delete p;
}

extern "C" {

int evr_mll_plan_create(void* stream, int kind, int B, int n, int d, const double* Xn, const double* Y,
                        evr_mll_plan** out) {
  EVR_CHECK(out && Xn && Y && B >= 1 && n >= 1 && d >= 1 && kind >= 0 && kind <= 3,
            "evr_mll_plan_create: bad arguments");
  evr_mll_plan* p = new (std::nothrow) evr_mll_plan();
  EVR_CHECK(p, "evr_mll_plan_create: out of host memory");
  std::memset((void*)p, 0, sizeof(*p));
  p->kind = kind;
  p->B = B;
  p->n = n;
  p->d = d;
  p->Xn = Xn;
  const size_t nn = (size_t)n * n;
  struct {
    double** ptr;
    size_t count;
  } need[] = {{&p->Y, (size_t)B * n},   {&p->ls, (size_t)B * d},  {&p->noise, (size_t)B},
              {&p->cst, (size_t)B},     {&p->K, B * nn},          {&p->L, B * nn},
              {&p->Linv, B * nn},       {&p->Dinv, chol_inverse_dinv_doubles(B, n)},
              {&p->T, (size_t)B * 64 * n}, {&p->r, (size_t)B * n}, {&p->v, (size_t)B * n},
              {&p->alpha, (size_t)B * n}, {&p->gls, (size_t)B * d}, {&p->gw, (size_t)B * n * d},
              {&p->part, mll_terms_part_doubles(B)}, {&p->jit0, (size_t)B}};
  for (auto& q : need) {
    if (hipMalloc((void**)q.ptr, sizeof(double) * std::max<size_t>(q.count, 1)) != hipSuccess) {
      mll_free(p);
      EVR_CHECK(false, "evr_mll_plan_create: device allocation failed");
    }
  }
  if (hipMalloc((void**)&p->info, sizeof(int) * B) != hipSuccess ||
      hipHostMalloc((void**)&p->hx, sizeof(double) * ((size_t)B * (d + 2) + 1),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostMalloc((void**)&p->hout, sizeof(double) * ((size_t)B * (5 + d + 1) + 1),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    mll_free(p);
    EVR_CHECK(false, "evr_mll_plan_create: allocation failed");
  }
  std::memset(p->hx, 0, sizeof(double) * ((size_t)B * (d + 2) + 1));
  std::memset(p->hout, 0, sizeof(double) * ((size_t)B * (5 + d + 1) + 1));
  hipStream_t s = (hipStream_t)stream;
  int rc = 0;
  if (hipMemcpyAsync(p->Y, Y, sizeof(double) * B * n, hipMemcpyDeviceToDevice, s) != hipSuccess ||
      hipMemsetAsync(p->jit0, 0, sizeof(double) * B, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    rc = 1;
  double *dhx = nullptr, *dhout = nullptr;
  if (!rc && (hipHostGetDevicePointer((void**)&dhx, p->hx, 0) != hipSuccess ||
              hipHostGetDevicePointer((void**)&dhout, p->hout, 0) != hipSuccess))
    rc = 1;
  hipStream_t cs = nullptr;
  if (!rc && hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) rc = 1;
  if (!rc) {
    if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) rc = 1;
    if (!rc) rc = mll_chain(cs, p, dhx, dhout);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(cs, &g);
    if (!rc && e == hipSuccess && g && hipGraphInstantiate(&p->exec, g, nullptr, nullptr, 0) == hipSuccess)
      p->graph = g;
    else {
      if (g) (void)hipGraphDestroy(g);
      p->exec = nullptr;
      rc = rc ? rc : 1;
    }
  }
  if (cs) (void)hipStreamDestroy(cs);
  if (rc) {
    const std::string why = last_error();
    mll_free(p);
    EVR_CHECK(false, "evr_mll_plan_create: setup / graph capture failed (%s)", why.c_str());
  }
  *out = p;
  return 0;
}

int evr_mll_plan_eval(void* stream, evr_mll_plan* p, const double* params, double* out) {
  EVR_CHECK(p && params && out, "evr_mll_plan_eval: bad arguments");
  const int B = p->B, d = p->d;
  const size_t nin = (size_t)B * (d + 2), nout = (size_t)B * (5 + d + 1);
  hipStream_t s = (hipStream_t)stream;
  std::memcpy(p->hx, params, sizeof(double) * nin);
  const unsigned long long seq = ++p->seq;
  std::memcpy(p->hx + nin, &seq, sizeof(seq));
  std::atomic_thread_fence(std::memory_order_seq_cst);
  EVR_HIP(hipGraphLaunch(p->exec, s));
  volatile const unsigned long long* done = (volatile const unsigned long long*)(p->hout + nout);
  for (unsigned k = 1; *done != seq; ++k) {
    if ((k & 255) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipErrorNotReady) continue;
      EVR_HIP(q);
      if (*done != seq) EVR_CHECK(false, "evr_mll_plan_eval: evaluation finished without its completion word");
    }
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  std::memcpy(out, p->hout, sizeof(double) * nout);
  return 0;
}

void evr_mll_plan_destroy(evr_mll_plan* p) { mll_free(p); }

int evr_lbfgsb_advance(void* run, double f, const double* g, double* x, int* task, int* nit, int* nfev, int* status,
                       int maxiter, int maxfun) {
  EVR_CHECK(run && g && x && task && nit && nfev && status, "evr_lbfgsb_advance: bad arguments");
  evr_lbfgsb* h = (evr_lbfgsb*)run;
  ++*nfev;
  int t = evr_lbfgsb_step(h, f, g, x);
  while (t == EVR_LBFGSB_NEW_X) {
    ++*nit;
    if (*nit >= maxiter || *nfev > maxfun) {
      *status = 1;
      *task = 0;
      return 0;
    }
    t = evr_lbfgsb_step(h, f, g, x);
  }
  if (t == EVR_LBFGSB_FG) {
    *task = EVR_LBFGSB_FG;
    return 0;
  }
  *status = t == EVR_LBFGSB_ABNORMAL ? 2 : (t == EVR_LBFGSB_ERROR ? 3 : 0);
  *task = 0;
  return 0;
}

}  // extern "C"

namespace {
// gpytorch LogNormalPrior / GammaPrior / NormalPrior log densities and their derivatives
// (gp.prior_logpdf_np / prior_dlogpdf_np)
double prior_logpdf(int fam, double a, double b, double x) {
  if (fam == 1) {
    const double lx = std::log(x), z = (lx - a) / b;
    return -lx - std::log(b) - 0.5 * std::log(2.0 * M_PI) - 0.5 * (z * z);
  }
  if (fam == 2) return a * std::log(b) - std::lgamma(a) + (a - 1.0) * std::log(x) - b * x;
  const double z = (x - a) / b;
  return -0.5 * std::log(2.0 * M_PI * b * b) - 0.5 * (z * z);
}
double prior_dlogpdf(int fam, double a, double b, double x) {
  if (fam == 1) return (-1.0 - (std::log(x) - a) / (b * b)) / x;
  if (fam == 2) return (a - 1.0) / x - b;
  return -(x - a) / (b * b);
}
double softplus(double v) {   // numpy logaddexp(0, v)
  if (v == 0.0) return M_LN2;
  return v > 0.0 ? v + std::log1p(std::exp(-v)) : std::log1p(std::exp(v));
}


// -MLL / n's pieces for one member: ll / n and its gradient in x = [noise, constant, raw
// lengthscales] (ExactMarginalLogLikelihood with the hyperparameter priors, divided by n as
// fit_gpytorch_mll's closure does) from the plan's terms (logdet, r.alpha, tr K^-1, sum alpha,
// sum alpha^2) and lengthscale-gradient pieces gls; ls = softplus(raw).  Shared by the native
// round driver and gp.MLLBatch (evr_mll_assemble), so both drivers see the same bits.
void mll_assemble_one(int n, int d, const double* prior, const double* xb, const double* t, const double* gls,
                      double* llo, double* gout) {
  const int lf = (int)prior[0], nzf = (int)prior[3];
  const double logdet = t[0], quad = t[1], trKinv = t[2], sum_a = t[3], sum_a2 = t[4];
  double ll = -0.5 * quad - 0.5 * logdet - 0.5 * n * std::log(2.0 * M_PI);
  double d_noise = 0.5 * (sum_a2 - trKinv);
  const double d_const = sum_a;
  const double noise = xb[0];
  if (lf) {
    double s = 0.0;
    for (int j = 0; j < d; ++j) s += prior_logpdf(lf, prior[1], prior[2], softplus(xb[2 + j]));
    ll += s;
  }
  if (nzf) {
    ll += prior_logpdf(nzf, prior[4], prior[5], noise);
    d_noise += prior_dlogpdf(nzf, prior[4], prior[5], noise);
  }
  gout[0] = d_noise / n;
  gout[1] = d_const / n;
  for (int j = 0; j < d; ++j) {
    const double lsj = softplus(xb[2 + j]);
    double dl = 0.5 * gls[j];
    if (lf) dl += prior_dlogpdf(lf, prior[1], prior[2], lsj);
    gout[2 + j] = dl * (1.0 / (1.0 + std::exp(-xb[2 + j]))) / n;
  }
  *llo = ll / n;
}
}  // namespace

extern "C" {

int evr_mll_assemble(int B, int n, int d, const double* prior, const double* x, const double* terms,
                     const double* gls, double* ll, double* g) {
  EVR_CHECK(B >= 0 && n >= 1 && d >= 1 && prior && x && terms && gls && ll && g, "evr_mll_assemble: bad arguments");
  for (int b = 0; b < B; ++b)
    mll_assemble_one(n, d, prior, x + (size_t)b * (d + 2), terms + (size_t)b * 5, gls + (size_t)b * d, ll + b,
                     g + (size_t)b * (d + 2));
  return 0;
}

int evr_mll_fit_rounds(void* stream, evr_mll_plan* p, void** runs, int* task, double* x, double* f, double* g,
                       int* nit, int* nfev, int* status, int maxiter, int maxfun, const double* prior, double* params,
                       int* pending) {
  EVR_CHECK(p && runs && task && x && f && g && nit && nfev && status && prior && params && pending,
            "evr_mll_fit_rounds: bad arguments");
  const int B = p->B, d = p->d, n = p->n, nx = d + 2;
  std::vector<double> out((size_t)B * (5 + d + 1)), gb(nx);
  *pending = 0;
  for (;;) {
    bool any = false;
    for (int b = 0; b < B; ++b) {
      if (task[b] != EVR_LBFGSB_FG) continue;
      any = true;
      const double* xb = x + (size_t)b * nx;
      for (int j = 0; j < d; ++j) params[(size_t)b * d + j] = softplus(xb[2 + j]);
      params[(size_t)B * d + b] = xb[0];
      params[(size_t)B * d + B + b] = xb[1];
    }
    if (!any) return 0;
    if (int rc = evr_mll_plan_eval(stream, p, params, out.data())) return rc;
    const double* terms = out.data();
    const double* gls = terms + (size_t)5 * B;
    const double* info = gls + (size_t)B * d;
    for (int b = 0; b < B; ++b) {
      if (task[b] != EVR_LBFGSB_FG) continue;
      bool ok = info[b] == 0.0;
      for (int q = 0; q < 5; ++q) ok = ok && std::isfinite(terms[(size_t)b * 5 + q]);
      if (!ok) {
        *pending = 1;   // this round goes through the jitter ladder (the caller)
        return 0;
      }
    }
    for (int b = 0; b < B; ++b) {
      if (task[b] != EVR_LBFGSB_FG) continue;
      double* xb = x + (size_t)b * nx;
      double llb;
      mll_assemble_one(n, d, prior, xb, terms + (size_t)b * 5, gls + (size_t)b * d, &llb, gb.data());
      // minimise -MLL / n
      f[b] = -llb;
      for (int j = 0; j < nx; ++j) g[(size_t)b * nx + j] = -gb[j];
      if (int rc = evr_lbfgsb_advance(runs[b], f[b], g + (size_t)b * nx, xb, task + b, nit + b, nfev + b, status + b,
                                      maxiter, maxfun))
        return rc;
    }
  }
}

}  // extern "C"
