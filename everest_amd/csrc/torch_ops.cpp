// PyTorch-ROCm custom operators over the everest_amd C-ABI (TORCH_LIBRARY(everest_amd, m)).
//
// the numeric op boundary of the BoTorch Model.posterior / acquisition
// forward protocols (bofire/strategies/predictives/botorch.py:180,223,384) as registered torch
// operators, so that a torch-side caller can compose them (autograd.Function wrappers in
// everest_amd/torch_ops.py).  Every op runs on torch's current HIP stream, allocates its
// outputs and scratch with the torch caching allocator, checks device / dtype with
// TORCH_CHECK (-> RuntimeError) and raises the C-ABI's evr_last_error() on failure.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "../../include/everest_amd.h"

namespace {

// torch's current stream of the current device (ROCm torch exposes HIP devices as "cuda")
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "everest_amd ", what, " failed (status ", rc, "): ", evr_last_error());
}

at::Tensor dev64(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "everest_amd: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kDouble, "everest_amd: ", name, " must be float64");
  return t.contiguous();
}

at::Tensor scratch(int64_t doubles, const at::Tensor& like) {
  return at::empty({std::max<int64_t>(doubles, 1)}, like.options().dtype(at::kDouble));
}

const double* ptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr<double>() : nullptr; }

// K[b] = k(X1, X2; ls[b]) — evr_kernel_matrix
at::Tensor kernel_matrix(const at::Tensor& X1_, const at::Tensor& X2_, const at::Tensor& ls_, int64_t kind) {
  auto X1 = dev64(X1_, "X1"), X2 = dev64(X2_, "X2"), ls = dev64(ls_, "lengthscales");
  if (ls.dim() == 1) ls = ls.unsqueeze(0);
  TORCH_CHECK(X1.dim() == 2 && X2.dim() == 2 && ls.dim() == 2 && X1.size(1) == ls.size(1) && X2.size(1) == ls.size(1),
              "kernel_matrix: X1 (n1 x d), X2 (n2 x d), lengthscales (B x d)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(X1.device());
  const int64_t B = ls.size(0), n1 = X1.size(0), n2 = X2.size(0), d = ls.size(1);
  auto K = at::empty({B, n1, n2}, X1.options());
  check(evr_kernel_matrix(cur_stream(), (int)kind, (int)B, (int)n1, (int)n2, (int)d, X1.data_ptr<double>(), nullptr,
                          nullptr, X2.data_ptr<double>(), nullptr, nullptr, ls.data_ptr<double>(), nullptr, nullptr,
                          K.data_ptr<double>()),
        "kernel_matrix");
  return K;
}

// psd_safe_cholesky batch: (L, jitter used, info) — evr_cholesky
std::tuple<at::Tensor, at::Tensor, at::Tensor> cholesky(const at::Tensor& A_, double jitter0, int64_t max_tries) {
  auto A = dev64(A_, "A");
  const bool flat = A.dim() == 2;
  if (flat) A = A.unsqueeze(0);
  TORCH_CHECK(A.dim() == 3 && A.size(1) == A.size(2), "cholesky: A must be (B x) n x n");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const int64_t B = A.size(0), n = A.size(1);
  auto L = at::empty_like(A);
  auto jit = at::empty({B}, A.options());
  auto info = at::empty({B}, A.options().dtype(at::kInt));
  check(evr_cholesky(cur_stream(), (int)B, (int)n, A.data_ptr<double>(), (int)n, n * n, L.data_ptr<double>(), (int)n,
                     n * n, jitter0, (int)max_tries, jit.data_ptr<double>(), info.data_ptr<int>()),
        "cholesky");
  if (flat) return {L.squeeze(0), jit, info};
  return {L, jit, info};
}

// L^-1 of lower-triangular L (B x n x n) — evr_tri_inv_lower
at::Tensor tri_inv(const at::Tensor& L_) {
  auto L = dev64(L_, "L");
  const bool flat = L.dim() == 2;
  if (flat) L = L.unsqueeze(0);
  TORCH_CHECK(L.dim() == 3 && L.size(1) == L.size(2), "tri_inv: L must be (B x) n x n");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(L.device());
  const int64_t B = L.size(0), n = L.size(1);
  auto Li = at::empty_like(L);
  check(evr_tri_inv_lower(cur_stream(), (int)B, (int)n, L.data_ptr<double>(), (int)n, n * n, Li.data_ptr<double>(),
                          (int)n, n * n),
        "tri_inv");
  return flat ? Li.squeeze(0) : Li;
}

// exact GP posterior mean / variance per output — evr_gp_posterior
std::tuple<at::Tensor, at::Tensor> gp_posterior(const at::Tensor& Xn_, const at::Tensor& X_, const at::Tensor& shift_,
                                                const at::Tensor& scale_, const at::Tensor& ls_, const at::Tensor& M_,
                                                int64_t kind, const at::Tensor& c_, const at::Tensor& ym_,
                                                const at::Tensor& ys_, const at::Tensor& kxx_,
                                                const c10::optional<at::Tensor>& noise_) {
  auto Xn = dev64(Xn_, "Xn"), X = dev64(X_, "X"), shift = dev64(shift_, "shift"), scale = dev64(scale_, "scale");
  auto ls = dev64(ls_, "lengthscales"), M = dev64(M_, "M"), c = dev64(c_, "c"), ym = dev64(ym_, "ym");
  auto ys = dev64(ys_, "ys"), kxx = dev64(kxx_, "kxx");
  c10::optional<at::Tensor> noise;
  if (noise_.has_value()) noise = dev64(*noise_, "noise");
  TORCH_CHECK(M.dim() == 3 && ls.dim() == 2 && Xn.dim() == 2 && X.dim() == 2, "gp_posterior: bad ranks");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  const int64_t B = M.size(0), n = Xn.size(0), nt = X.size(0), d = Xn.size(1);
  TORCH_CHECK(M.size(1) == n + 1 && M.size(2) == n && X.size(1) == d && ls.size(0) == B && ls.size(1) == d,
              "gp_posterior: M must be B x (n+1) x n, X nt x d");
  auto mean = at::empty({B, nt}, X.options()), var = at::empty({B, nt}, X.options());
  auto work = scratch(evr_gp_posterior_workspace_doubles((int)B, (int)n, (int)nt), X);
  check(evr_gp_posterior(cur_stream(), (int)B, (int)n, (int)nt, (int)d, (int)kind, Xn.data_ptr<double>(),
                         X.data_ptr<double>(), shift.data_ptr<double>(), scale.data_ptr<double>(), ls.data_ptr<double>(),
                         M.data_ptr<double>(), c.data_ptr<double>(), ym.data_ptr<double>(), ys.data_ptr<double>(),
                         kxx.data_ptr<double>(), ptr(noise), mean.data_ptr<double>(), var.data_ptr<double>(),
                         work.data_ptr<double>()),
        "gp_posterior");
  return {mean, var};
}

// ---------------------------------------------------------------------------------------
// The acquisition behind torch.ops.everest_amd.qnehvi_*: a registered torch class that OWNS
// what the device chain reads — private copies of the state / model / objective structs and
// references to every device tensor they point into (so the tensors live as long as the
// object) — and caches one native plan per (batch size, backward) across calls.
// ---------------------------------------------------------------------------------------
struct QnehviAcq : torch::CustomClassHolder {
  evr_qnehvi_state stm{}, sth{};
  evr_qnehvi_model md{};
  bool fast = false;
  std::vector<at::Tensor> keep;
  struct General {
    evr_qn_general g{};
    std::vector<int> oo, ok, co;
    std::vector<double> p0, p1, cs, ct, ce;
    at::Tensor zq;
  };
  std::map<int64_t, std::unique_ptr<General>> gens;
  struct Plan {
    evr_qnehvi_plan* p = nullptr;
    at::Tensor work, X, acq, dX;
  };
  std::map<std::pair<int64_t, bool>, Plan> plans;
  int64_t n_evals = 0;

  template <class T>
  static T from_bytes(const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.device().is_cpu() && t.scalar_type() == at::kByte && t.numel() == (int64_t)sizeof(T),
                "QnehviAcq: ", what, " must be a CPU uint8 tensor of ", sizeof(T), " bytes");
    T v;
    std::memcpy(&v, t.contiguous().data_ptr(), sizeof(T));
    return v;
  }

  bool log_scan = false;   // general path through evr_qlog_eval (qLogNEHVI / qLogEHVI)

  QnehviAcq(const at::Tensor& stm_b, const at::Tensor& sth_b, const at::Tensor& md_b, bool fast_, bool log_,
            std::vector<at::Tensor> keep_)
      : fast(fast_), keep(std::move(keep_)), log_scan(log_) {
    stm = from_bytes<evr_qnehvi_state>(stm_b, "model-side state");
    sth = from_bytes<evr_qnehvi_state>(sth_b, "scan-side state");
    md = from_bytes<evr_qnehvi_model>(md_b, "model");
    TORCH_CHECK(md.M && md.Xn && md.lengthscales && md.n == stm.n && md.d >= 1, "QnehviAcq: inconsistent model");
  }

  ~QnehviAcq() override {
    for (auto& kv : plans) evr_qnehvi_plan_destroy(kv.second.p);
  }

  // objective / constraint description and base samples of q-point candidates (general path)
  void set_general(int64_t q, const at::Tensor& oo, const at::Tensor& ok, const at::Tensor& p0, const at::Tensor& p1,
                   const at::Tensor& co, const at::Tensor& cs, const at::Tensor& ct, const at::Tensor& ce,
                   const at::Tensor& zq) {
    TORCH_CHECK(q >= 1 && q <= EVR_QNG_MAX_Q, "QnehviAcq.set_general: q = ", q, " outside 1..", EVR_QNG_MAX_Q);
    auto ints = [](const at::Tensor& t) {
      auto c = t.to(at::kCPU, at::kInt).contiguous();
      return std::vector<int>(c.data_ptr<int>(), c.data_ptr<int>() + c.numel());
    };
    auto dbls = [](const at::Tensor& t) {
      auto c = t.to(at::kCPU, at::kDouble).contiguous();
      return std::vector<double>(c.data_ptr<double>(), c.data_ptr<double>() + c.numel());
    };
    auto G = std::make_unique<General>();
    G->oo = ints(oo);
    G->ok = ints(ok);
    G->co = ints(co);
    G->p0 = dbls(p0);
    G->p1 = dbls(p1);
    G->cs = dbls(cs);
    G->ct = dbls(ct);
    G->ce = dbls(ce);
    TORCH_CHECK(G->ok.size() == G->oo.size() && G->p0.size() == G->oo.size() && G->p1.size() == G->oo.size() &&
                    G->cs.size() == G->co.size() && G->ct.size() == G->co.size() && G->ce.size() == G->co.size(),
                "QnehviAcq.set_general: inconsistent objective / constraint arrays");
    G->zq = dev64(zq, "zq");
    G->g.q = (int)q;
    G->g.m_obj = (int)G->oo.size();
    G->g.obj_out = G->oo.data();
    G->g.obj_kind = G->ok.data();
    G->g.obj_p0 = G->p0.data();
    G->g.obj_p1 = G->p1.data();
    G->g.n_con = (int)G->co.size();
    G->g.con_out = G->co.empty() ? nullptr : G->co.data();
    G->g.con_sign = G->cs.empty() ? nullptr : G->cs.data();
    G->g.con_thr = G->ct.empty() ? nullptr : G->ct.data();
    G->g.con_eta = G->ce.empty() ? nullptr : G->ce.data();
    G->g.zq = G->zq.data_ptr<double>();
    gens[q] = std::move(G);
  }

  Plan& plan(int64_t b, bool backward, const at::Tensor& like, hipStream_t s) {
    auto key = std::make_pair(b, backward);
    auto it = plans.find(key);
    if (it != plans.end()) return it->second;
    Plan P;
    P.X = at::empty({b, (int64_t)md.d}, like.options());
    P.acq = at::empty({b}, like.options());
    P.dX = backward ? at::empty({b, (int64_t)md.d}, like.options()) : at::Tensor();
    P.work = at::empty({std::max<long long>(evr_qnehvi_plan_workspace_bytes(&stm, &md, (int)b, backward), 1)},
                       like.options().dtype(at::kByte));
    check(evr_qnehvi_plan_create(s, &stm, &md, (int)b, backward, P.X.data_ptr<double>(), P.work.data_ptr(),
                                 P.acq.data_ptr<double>(), backward ? P.dX.data_ptr<double>() : nullptr, 1, &P.p),
          "qnehvi_plan_create");
    return plans.emplace(key, std::move(P)).first->second;
  }

  // (acq, dX | undefined) at X: q = 1 on the fused chain through a cached plan (one graph
  // launch from its second use), q-point candidates through evr_qng_eval
  std::tuple<at::Tensor, at::Tensor> eval(const at::Tensor& X_, bool backward) {
    auto X = dev64(X_, "X");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
    hipStream_t s = cur_stream();
    if (fast) {
      TORCH_CHECK(X.dim() == 2 && X.size(1) == md.d, "qnehvi (q = 1 fast path): X must be b x d");
      const int64_t b = X.size(0);
      if (b == 0) return {at::empty({0}, X.options()), backward ? at::empty_like(X) : at::Tensor()};
      Plan& P = plan(b, backward, X, s);
      P.X.copy_(X);
      check(evr_qnehvi_plan_run(s, P.p), "qnehvi_plan_run");
      ++n_evals;
      return {P.acq.clone(), backward ? P.dX.clone() : at::Tensor()};
    }
    TORCH_CHECK(X.dim() == 3 && X.size(2) == md.d, "qnehvi (general path): X must be b x q x d");
    const int64_t b = X.size(0), q = X.size(1);
    auto it = gens.find(q);
    TORCH_CHECK(it != gens.end(), "qnehvi: no objective description / base samples set for q = ", q);
    const evr_qn_general* g = &it->second->g;
    auto acq = at::empty({b}, X.options());
    at::Tensor dX = backward ? at::empty_like(X) : at::Tensor();
    if (b == 0) return {acq, dX};
    if (log_scan) {
      auto work = scratch(evr_qlog_workspace_doubles(&stm, &sth, g, &md, (int)b, backward), X);
      check(evr_qlog_eval(s, &stm, &sth, g, &md, (int)b, X.data_ptr<double>(), nullptr, work.data_ptr<double>(),
                          acq.data_ptr<double>(), backward ? dX.data_ptr<double>() : nullptr),
            "qlog_eval");
    } else {
      auto work = scratch(evr_qng_workspace_doubles(&stm, &sth, g, &md, (int)b, backward), X);
      check(evr_qng_eval(s, &stm, &sth, g, &md, (int)b, X.data_ptr<double>(), nullptr, work.data_ptr<double>(),
                         acq.data_ptr<double>(), backward ? dX.data_ptr<double>() : nullptr),
            "qng_eval");
    }
    ++n_evals;
    return {acq, dX};
  }

  int64_t evals() const { return n_evals; }
  int64_t cached_plans() const { return (int64_t)plans.size(); }
};

using AcqPtr = c10::intrusive_ptr<QnehviAcq>;

at::Tensor qnehvi_forward(const AcqPtr& acq, const at::Tensor& X) { return std::get<0>(acq->eval(X, false)); }

// (acq, d acq_c / dX_c): one chain for the value and the analytic gradient
std::tuple<at::Tensor, at::Tensor> qnehvi_forward_backward(const AcqPtr& acq, const at::Tensor& X) {
  return acq->eval(X, true);
}

// d(sum_c grad_out_c acq_c)/dX: candidates are independent, so the per-candidate gradient
// of the device backward is scaled by grad_out (re-runs the chain; the autograd wrapper uses
// qnehvi_forward_backward's saved gradient instead)
at::Tensor qnehvi_backward(const AcqPtr& acq, const at::Tensor& X, const at::Tensor& grad_out_) {
  auto g = dev64(grad_out_, "grad_out");
  auto dX = std::get<1>(acq->eval(X, true));
  TORCH_CHECK(g.numel() == dX.size(0), "qnehvi_backward: grad_out must have one entry per candidate");
  std::vector<int64_t> shape(dX.dim(), 1);
  shape[0] = dX.size(0);
  return dX * g.view(shape);
}

}  // namespace

TORCH_LIBRARY(everest_amd, m) {
  m.class_<QnehviAcq>("QnehviAcq")
      .def(torch::init<at::Tensor, at::Tensor, at::Tensor, bool, bool, std::vector<at::Tensor>>())
      .def("set_general", &QnehviAcq::set_general)
      .def("evals", &QnehviAcq::evals)
      .def("cached_plans", &QnehviAcq::cached_plans);
  m.def("kernel_matrix(Tensor X1, Tensor X2, Tensor lengthscales, int kind) -> Tensor");
  m.def("cholesky(Tensor A, float jitter0, int max_tries) -> (Tensor, Tensor, Tensor)");
  m.def("tri_inv(Tensor L) -> Tensor");
  m.def("gp_posterior(Tensor Xn, Tensor X, Tensor shift, Tensor scale, Tensor lengthscales, Tensor M, int kind, "
        "Tensor c, Tensor ym, Tensor ys, Tensor kxx, Tensor? noise) -> (Tensor, Tensor)");
  m.def("qnehvi_forward(__torch__.torch.classes.everest_amd.QnehviAcq acq, Tensor X) -> Tensor");
  m.def("qnehvi_forward_backward(__torch__.torch.classes.everest_amd.QnehviAcq acq, Tensor X) -> (Tensor, Tensor)");
  m.def("qnehvi_backward(__torch__.torch.classes.everest_amd.QnehviAcq acq, Tensor X, Tensor grad_out) -> Tensor");
}

TORCH_LIBRARY_IMPL(everest_amd, CUDA, m) {
  m.impl("kernel_matrix", &kernel_matrix);
  m.impl("cholesky", &cholesky);
  m.impl("tri_inv", &tri_inv);
  m.impl("gp_posterior", &gp_posterior);
  m.impl("qnehvi_forward", &qnehvi_forward);
  m.impl("qnehvi_forward_backward", &qnehvi_forward_backward);
  m.impl("qnehvi_backward", &qnehvi_backward);
}
