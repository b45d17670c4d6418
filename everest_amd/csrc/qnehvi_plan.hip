// Native evaluation plan of the qNEHVI acquisition (q = 1): one C-ABI call runs the whole
// device chain of QNEHVI.forward / forward_backward (everest_amd/acquisition.py),
//   K_x = k(X_train, normalize(X))            kernel_matrix.hip
//   R, norms = M K_x                          qnehvi_proj.hip (fused epilogue)
//   G, L22, flags                             qnehvi_proj.hip (samples from the norms)
//   acq (, dG)                                hvi.hip (sparse kd scan or tiled scan)
//   dK_x = M^T gR (generated)                 qnehvi_proj.hip
//   dX = sum_j dK_x,j . dk/dx                 kernel_matrix.hip
// with every intermediate carved from one caller-owned workspace, optionally captured once
// into a hipGraph and replayed — the L-BFGS restarts of ask() (b = 20) issue one graph
// launch per iteration instead of a dozen kernel launches through the Python binding.
// The plan copies the state / model structs; the device buffers they point to, the
// workspace and the X / output buffers must outlive it (the Python QNEHVI object owns them).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <string>
#include <mutex>
#include <new>
#include <vector>

#include "common.hpp"
#include "qs_tail.hpp"
#include "lbfgsb.hpp"
#include "../../include/everest_amd.h"

namespace evr {
size_t proj_forward_ws_doubles(const evr_qnehvi_state* st, int b);
int proj_forward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* Kx, double* R,
                 double* norms, double* W);
size_t proj_backward_ws_doubles(const evr_qnehvi_state* st, int b);
int proj_backward(hipStream_t s, const evr_qnehvi_state* st, int b, const double* Mm, const double* R,
                  const double* L22, const double* dG, double* dKx, double* ws);
int samples_norms(hipStream_t s, const evr_qnehvi_state* st, int b, const double* R, const double* norms, double* G,
                  double* L22, int* flags, int tile_rows);
bool qs_applies(const evr_qnehvi_state* st, int b, int d);
size_t qs_norms_doubles(const evr_qnehvi_state* st, int b);
size_t qs_dxp_doubles(const evr_qnehvi_state* st, int b, int d);
int qs_forward(hipStream_t s, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b, const double* Kx,
               double* R, double* P);
int qs_done_words(int b, int d);
int qs_backward(hipStream_t s, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b, const double* X,
                const double* R, const double* L22, const double* dG, double* dXp, double* dX, double* acq,
                double* hout, const double* seqp, const double* sval, const int* flags);
int kernel_matrix_launch(void* stream, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                         const double* scale1, const double* X2, const double* shift2, const double* scale2,
                         const double* lengthscales, const double* outputscale, const double* diag_add, double* K,
                         const unsigned long long* seq_src = nullptr, unsigned long long* seq_dst = nullptr,
                         double* x_dst = nullptr, int* zero_dst = nullptr, int nzero = 0);
constexpr int QS_TILE_ROWS = 16;
constexpr int QN_NORM_TILE = 32;   // qnehvi_proj.hip QN_NT (the b > 32 projection tiles)
bool hvi_kdb_fused_applies(const evr_qnehvi_state* st, int b);
int hvi_kdb_fused(hipStream_t s, const evr_qnehvi_state* st, int b, const double* R, const double* P, int nrt,
                  int nrt_used, double* L22, int* flags, double* sval, double* dG);

// b <= 32 restart batches take the M-streaming small-batch kernels (qnehvi_small.hip);
// EVR_SMALL=0 keeps the 64 x 64-tile path for A/B timing and the parity test
static bool small_path(const evr_qnehvi_state* st, int b, int d) {
  const char* e = std::getenv("EVR_SMALL");   // read per plan (plans are built once per batch size)
  return !(e && std::string(e) == "0") && qs_applies(st, b, d);
}
size_t kcross_grad_ws_doubles(int n1, int n2, int d);
int kcross_grad_launch(hipStream_t s, int kind, int B, int n1, int n2, int d, const double* X1, const double* shift1,
                       const double* scale1, const double* X2, const double* shift2, const double* scale2,
                       const double* lengthscales, const double* outputscale, const double* G, double* dX2,
                       double* work);

struct PlanLayout {
  size_t Kx, R, P, Wf, G, L22, flags, hvi, dG, bws, dKx, kg, dxp, seqd, xd, bytes;
  bool small, fused_scan;
};

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static PlanLayout plan_layout(const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b, int backward) {
  PlanLayout L{};
  const size_t m = st->m, n = st->n, Rr = (size_t)qn_rows(st);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t r = o;
    o += al256(bytes);
    return r;
  };
  L.small = small_path(st, b, md->d);
  L.fused_scan = L.small && backward && evr_hvi_restart_fb_applies(st, b);
  L.Kx = take(8 * m * n * b);
  L.R = take(8 * m * Rr * b);
  L.P = take(8 * (L.small ? qs_norms_doubles(st, b) : m * (size_t)evr_qnehvi_norms_rows(st) * 2 * b));
  L.Wf = take(8 * (L.small ? 0 : proj_forward_ws_doubles(st, b)));
  L.G = take(8 * (size_t)st->S * m * b);
  L.L22 = take(8 * m * b);
  L.flags = take(4 * m * b);
  L.hvi = take(8 * (size_t)evr_hvi_workspace_doubles(st, b, backward));
  if (backward) {
    L.dG = take(8 * (size_t)st->S * m * b);
    if (L.small) {
      L.dxp = take(8 * qs_dxp_doubles(st, b, md->d));
    } else {
      L.bws = take(8 * proj_backward_ws_doubles(st, b));
      L.dKx = take(8 * m * n * b);
      L.kg = take(8 * kcross_grad_ws_doubles(st->n, b, md->d));
    }
  }
  L.seqd = take(8);   // the host-driven chain's sequence number, copied to device memory by kmat
  L.xd = take(8 * (size_t)b * md->d);   // the host-driven chain's candidates, copied likewise
  L.bytes = o;
  return L;
}

}  // namespace evr

using namespace evr;

struct evr_qnehvi_plan {
  evr_qnehvi_state st;
  evr_qnehvi_model md;
  int b, backward;
  const double* X;
  unsigned char* work;
  double* acq;
  double* dX;
  PlanLayout L;
  hipGraph_t graph;
  hipGraphExec_t exec;
  // host-driven evaluations (evr_qnehvi_plan_minimize): fine-grained pinned buffers read and
  // written by kernels of a second graph [copy-in, chain, copy-out], so one evaluation is one
  // graph launch and a spin on a completion word (no blit copies, no stream synchronise)
  double* hx;                    // x (b x d), then the evaluation's sequence number (u64)
  double* hout;                  // acq (b), dX (b x d), then the completion word (u64)
  hipGraph_t hgraph;
  hipGraphExec_t hexec;
  unsigned long long seq;
  unsigned int* counter;         // (kept for the recycled-resource layout; unused since round 4)
  int nwords;                    // completion words the host graph's last kernel writes
  int use_graph, nrun;           // device-mode graph wanted / runs so far (captured on the 2nd)
};

namespace evr {

// acq and dX to the host buffer, then (after every thread's system-scope fence) the
// evaluation's sequence number into the completion word the host spins on
__global__ __launch_bounds__(256) void plan_copy_out(int b, int n, const double* __restrict__ acq,
                                                     const double* __restrict__ dX, const double* hx,
                                                     double* hout) {
  for (int i = threadIdx.x; i < b; i += 256) hout[i] = acq[i];
  if (dX)
    for (int i = threadIdx.x; i < n; i += 256) hout[b + i] = dX[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long seq = *(volatile const unsigned long long*)(hx + n);
    __threadfence_system();
    *(volatile unsigned long long*)(hout + b + n) = seq;
  }
}

}  // namespace evr

// The chain on candidates X (device buffer, or in the host graph the pinned host buffer
// itself).  Host mode (hout): the b <= 32 backward's dX reduction also writes [acq | dX] and
// one completion word per reduction workgroup to hout (*done = their number); otherwise
// (*done = 0) the caller appends a copy-out kernel (one word).
static int plan_chain(hipStream_t s, const evr_qnehvi_plan* p, const double* X, double* hout = nullptr,
                      const double* seqp = nullptr, int* done = nullptr) {
  const evr_qnehvi_state* st = &p->st;
  const evr_qnehvi_model* md = &p->md;
  const int b = p->b, m = st->m, n = st->n, d = md->d;
  unsigned char* w = p->work;
  double* Kx = (double*)(w + p->L.Kx);
  double* R = (double*)(w + p->L.R);
  double* P = (double*)(w + p->L.P);
  double* G = (double*)(w + p->L.G);
  double* L22 = (double*)(w + p->L.L22);
  int* flags = (int*)(w + p->L.flags);
  double* hw = (double*)(w + p->L.hvi);
  const bool small = p->L.small;
  // (K_x generated inside the projection instead was measured slower at b = 20 twice — 29 vs
  // 17.6 us in round 3, chain 83.9 vs 73.7 us in round 4 — and removed)
  // host mode through the b <= 32 kernels: qs_dx_reduce reads the sequence number from the
  // device copy kmat makes (an L2 read instead of a PCIe read at the end of the chain)
  // (the copies ride in kmat_kernel, the VALU assembly: d < 16 and one kernel family)
  unsigned long long* seqd = (hout && seqp && small && d < 16 && md->kind < KIND_MIXED)
                                 ? (unsigned long long*)(w + p->L.seqd)
                                 : nullptr;
  // and the candidates: the later kernels of the chain read the device copy
  double* xd = seqd ? (double*)(w + p->L.xd) : nullptr;
  if (int rc = kernel_matrix_launch(s, md->kind, m, n, b, d, md->Xn, nullptr, nullptr, X, md->shift, md->scale,
                                    md->lengthscales, nullptr, nullptr, Kx,
                                    seqd ? (const unsigned long long*)seqp : nullptr, seqd, xd)) {
    return rc;
  } else if (small) {
    if (int rc = qs_forward(s, st, md, b, Kx, R, P)) return rc;
  } else if (int rc = proj_forward(s, st, b, md->M, Kx, R, P,
                                   p->L.Wf != p->L.G ? (double*)(w + p->L.Wf) : nullptr)) {
    return rc;
  }
  double* dG = (double*)(w + p->L.dG);
  if (xd) X = xd;
  if (small && p->backward && p->L.fused_scan && hvi_kdb_fused_applies(st, b)) {
    // the sampling step inside the restart scan's staging (one launch less); G is not formed
    if (int rc = hvi_kdb_fused(s, st, b, R, P, cdiv(qn_rows(st), QS_TILE_ROWS), cdiv(st->n + st->nb, QS_TILE_ROWS),
                               L22, flags, hw, dG))
      return rc;
    if (done) *done = hout ? qs_done_words(b, d) : 0;
    return qs_backward(s, st, md, b, X, R, L22, dG, (double*)(w + p->L.dxp), p->dX, p->acq, hout,
                       seqd ? (const double*)seqd : seqp, hw, flags);
  }
  if (int rc = samples_norms(s, st, b, R, P, G, L22, flags, small ? QS_TILE_ROWS : QN_NORM_TILE)) return rc;
  if (!p->backward) return evr_hvi_forward(s, st, b, G, flags, hw, p->acq);
  if (small && p->L.fused_scan) {
    // the restart scan in one launch (hvi_kdw); the per-sample values in the scan workspace
    // become acq inside the dX reduction
    if (int rc = evr_hvi_restart_fb(s, st, b, G, hw, dG)) return rc;
    if (done) *done = hout ? qs_done_words(b, d) : 0;
    return qs_backward(s, st, md, b, X, R, L22, dG, (double*)(w + p->L.dxp), p->dX, p->acq, hout,
                       seqd ? (const double*)seqd : seqp, hw, flags);
  }
  if (int rc = evr_hvi_forward_backward(s, st, b, G, flags, nullptr, hw, p->acq, dG)) return rc;
  if (small) {
    if (done) *done = hout ? qs_done_words(b, d) : 0;
    return qs_backward(s, st, md, b, X, R, L22, dG, (double*)(w + p->L.dxp), p->dX, p->acq, hout,
                       seqd ? (const double*)seqd : seqp, nullptr, nullptr);
  }
  double* dKx = (double*)(w + p->L.dKx);
  if (int rc = proj_backward(s, st, b, md->M, R, L22, dG, dKx, (double*)(w + p->L.bws))) return rc;
  return kcross_grad_launch(s, md->kind, m, n, b, d, md->Xn, nullptr, nullptr, X, md->shift, md->scale,
                            md->lengthscales, nullptr, dKx, p->dX, (double*)(w + p->L.kg));
}

// Host-evaluation resources of destroyed plans, recycled by the next plan of the same batch
// shape (every ask builds a new acquisition, hence new restart plans): the pinned buffers and
// the completion counter are reused, and the new chain's graph updates the old executable
// (hipGraphExecUpdate: same kernels, new arguments) instead of a fresh instantiation — 0.42 ms
// of first-evaluation setup plus the frees per plan (tools/plan_setup_probe.py).  A failed
// update (another kernel sequence) falls back to instantiating.  EVR_GRAPH_REUSE=0 disables.
struct PlanHostRes {
  int dev, b, n, backward;
  double* hx;
  double* hout;
  unsigned int* counter;
  hipGraphExec_t exec;
  hipGraph_t graph;
};
static std::mutex g_hres_mu;
static std::vector<PlanHostRes> g_hres;
static bool graph_reuse() {
  static const bool on = [] {
    const char* e = std::getenv("EVR_GRAPH_REUSE");
    return !(e && e[0] == '0');
  }();
  return on;
}

extern "C" {

long long evr_qnehvi_plan_workspace_bytes(const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                                          int backward) {
  if (!st || !md || b <= 0) return 0;
  return (long long)plan_layout(st, md, b, backward).bytes;
}

int evr_qnehvi_plan_create(void* stream, const evr_qnehvi_state* st, const evr_qnehvi_model* md, int b,
                           int backward, const double* X, void* work, double* acq, double* dX, int use_graph,
                           evr_qnehvi_plan** out) {
  EVR_CHECK(st && md && out && X && work && acq && b >= 1 && (!backward || dX) && md->M && md->Xn &&
                md->lengthscales && md->n == st->n && md->d >= 1 && kind_code_ok(md->kind, st->m),
            "evr_qnehvi_plan_create: bad arguments");
  evr_qnehvi_plan* p = new (std::nothrow) evr_qnehvi_plan();
  EVR_CHECK(p, "evr_qnehvi_plan_create: out of host memory");
  p->st = *st;
  p->md = *md;
  p->b = b;
  p->backward = backward ? 1 : 0;
  p->X = X;
  p->work = (unsigned char*)work;
  p->acq = acq;
  p->dX = dX;
  p->L = plan_layout(st, md, b, p->backward);
  p->graph = nullptr;
  p->exec = nullptr;
  p->hx = nullptr;
  p->hout = nullptr;
  p->hgraph = nullptr;
  p->hexec = nullptr;
  p->seq = 0;
  p->nwords = 1;
  p->counter = nullptr;
  // the device-mode graph is captured on the second run (a plan evaluated once — the raw
  // screening chunks — or only host-driven — the restarts, which use the host graph — never
  // pays for a capture and an instantiation)
  p->use_graph = use_graph ? 1 : 0;
  p->nrun = 0;
  (void)stream;
  *out = p;
  return 0;
}

// One non-blocking capture stream per device for the plans' graph captures (created once:
// a stream creation / destruction per plan cost host time at every ask's first restart
// evaluation); the returned lock serialises captures across threads.
static std::mutex g_cap_mu;
static hipStream_t capture_stream(std::unique_lock<std::mutex>* lk) {
  static hipStream_t streams[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  *lk = std::unique_lock<std::mutex>(g_cap_mu);
  if (!streams[dev] && hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking) != hipSuccess) {
    streams[dev] = nullptr;
    lk->unlock();
  }
  return streams[dev];
}

// Capture the device-mode chain into p->exec (private stream: the caller's stream, torch's,
// never enters capture mode).  On failure the plan keeps running the chain eagerly.
static void plan_capture(evr_qnehvi_plan* p) {
  p->use_graph = 0;
  std::unique_lock<std::mutex> cap_lk;
  hipStream_t cs = capture_stream(&cap_lk);
  if (!cs) return;
  int rc = hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) == hipSuccess ? 0 : 1;
  if (!rc) rc = plan_chain(cs, p, p->X);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(cs, &g);
  cap_lk.unlock();
  if (!rc && e == hipSuccess && g && hipGraphInstantiate(&p->exec, g, nullptr, nullptr, 0) == hipSuccess) {
    p->graph = g;
  } else {
    if (g) (void)hipGraphDestroy(g);
    p->exec = nullptr;
    (void)hipGetLastError();
  }
}

int evr_qnehvi_plan_run(void* stream, evr_qnehvi_plan* p) {
  EVR_CHECK(p, "evr_qnehvi_plan_run: null plan");
  hipStream_t s = (hipStream_t)stream;
  if (!p->exec && p->use_graph && p->nrun++ >= 1) plan_capture(p);
  if (p->exec) {
    EVR_HIP(hipGraphLaunch(p->exec, s));
    return 0;
  }
  return plan_chain(s, p, p->X);
}


void evr_qnehvi_plan_destroy(evr_qnehvi_plan* p) {
  if (!p) return;
  int dev = -1;
  if (graph_reuse() && p->hexec && p->hx && p->hout && hipGetDevice(&dev) == hipSuccess) {
    // the plan's evaluations have completed (plan_eval_raw waits for each), so the buffers and
    // the executable are idle; the counter is back at 0 (the last workgroup resets it)
    std::lock_guard<std::mutex> lk(g_hres_mu);
    if (g_hres.size() < 4) {
      g_hres.push_back({dev, p->b, p->b * p->md.d, p->backward, p->hx, p->hout, p->counter, p->hexec, p->hgraph});
      p->hx = nullptr;
      p->hout = nullptr;
      p->counter = nullptr;
      p->hexec = nullptr;
      p->hgraph = nullptr;
    }
  }
  if (p->hexec) (void)hipGraphExecDestroy(p->hexec);
  if (p->hgraph) (void)hipGraphDestroy(p->hgraph);
  if (p->hx) (void)hipHostFree(p->hx);
  if (p->hout) (void)hipHostFree(p->hout);
  if (p->counter) (void)hipFree(p->counter);
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  delete p;
}

// The host-evaluation buffers and graph, built on first use.
static int plan_host_setup(hipStream_t s, evr_qnehvi_plan* p) {
  if (p->hexec) return 0;
  const int b = p->b, n = b * p->md.d;
  hipGraphExec_t old_exec = nullptr;
  hipGraph_t old_graph = nullptr;
  int dev = -1;
  if (graph_reuse() && !p->hx && !p->hout && hipGetDevice(&dev) == hipSuccess) {
    std::lock_guard<std::mutex> lk(g_hres_mu);
    for (size_t i = 0; i < g_hres.size(); ++i) {
      const PlanHostRes& r = g_hres[i];
      if (r.dev == dev && r.b == b && r.n == n && r.backward == p->backward) {
        p->hx = r.hx;
        p->hout = r.hout;
        p->counter = r.counter;
        old_exec = r.exec;
        old_graph = r.graph;
        g_hres.erase(g_hres.begin() + (long)i);
        break;
      }
    }
  }
  if (!p->hx)
    EVR_HIP(hipHostMalloc((void**)&p->hx, sizeof(double) * (n + 1), hipHostMallocMapped | hipHostMallocCoherent));
  if (!p->hout)
    EVR_HIP(hipHostMalloc((void**)&p->hout, sizeof(double) * ((size_t)b * (1 + p->md.d) + 64),
                          hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(p->hx, 0, sizeof(double) * (n + 1));
  std::memset(p->hout, 0, sizeof(double) * ((size_t)b * (1 + p->md.d) + 64));
  double *dhx = nullptr, *dhout = nullptr;
  EVR_HIP(hipHostGetDevicePointer((void**)&dhx, p->hx, 0));
  EVR_HIP(hipHostGetDevicePointer((void**)&dhout, p->hout, 0));
  // (no completion counter since round 4: its hipMalloc and the synchronous hipMemset — which
  // waited for the device to drain — were the setup's largest host stalls, with the stream
  // creation / destruction now replaced by one capture stream per device)
  std::unique_lock<std::mutex> cap_lk;
  hipStream_t cs = capture_stream(&cap_lk);
  EVR_CHECK(cs, "qnehvi plan: no capture stream");
  int rc = hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) == hipSuccess ? 0 : 1;
  if (!rc) {
    // the kernels read x straight from the pinned buffer; the restart batch's dX reduction
    // writes the results and the completion word itself, other chains end in plan_copy_out
    int done = 0;
    rc = plan_chain(cs, p, dhx, dhout, dhx + n, &done);
    if (!rc && !done) plan_copy_out<<<1, 256, 0, cs>>>(b, n, p->acq, p->backward ? p->dX : nullptr, dhx, dhout);
    p->nwords = done > 0 ? done : 1;
  }
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(cs, &g);
  cap_lk.unlock();
  if (old_exec) {
    hipGraphNode_t err_node = nullptr;
    hipGraphExecUpdateResult ur = hipGraphExecUpdateError;
    const bool ok = !rc && e == hipSuccess && g && hipGraphExecUpdate(old_exec, g, &err_node, &ur) == hipSuccess &&
                    ur == hipGraphExecUpdateSuccess;
    if (old_graph) (void)hipGraphDestroy(old_graph);
    if (ok) {
      p->hexec = old_exec;
      p->hgraph = g;
      return 0;
    }
    (void)hipGraphExecDestroy(old_exec);
    (void)hipGetLastError();
  }
  if (!rc && e == hipSuccess && g && hipGraphInstantiate(&p->hexec, g, nullptr, nullptr, 0) == hipSuccess) {
    p->hgraph = g;
    return 0;
  }
  if (g) (void)hipGraphDestroy(g);
  p->hexec = nullptr;
  const std::string why = last_error();
  EVR_CHECK(false, "qnehvi plan: host-evaluation graph capture failed (%s)", why.c_str());
}

// One evaluation at host x (b x d); [acq | dX] left in p->hout.  (Queuing the next evaluation's
// graph behind a request-word wait was measured in rounds 3-5 and removed in round 6: the
// extra kernel boundary and the PCIe poll cost more than the hidden launch, profiles/r05/j.)
static int plan_eval_raw(hipStream_t s, evr_qnehvi_plan* p, const double* x) {
  const int b = p->b, n = b * p->md.d;
  if (int rc = plan_host_setup(s, p)) return rc;
  std::memcpy(p->hx, x, sizeof(double) * n);
  const unsigned long long seq = ++p->seq;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  __atomic_store_n((unsigned long long*)(p->hx + n), seq, __ATOMIC_RELEASE);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  EVR_HIP(hipGraphLaunch(p->hexec, s));
  // spin on the completion words; every 256 polls ask the stream whether it has drained (a
  // faulted or failed launch ends the wait with its error instead of spinning forever; a 30 s
  // limit backs the wait up)
  volatile const unsigned long long* done = (volatile const unsigned long long*)(p->hout + b + n);
  const int nw = p->nwords;
  auto finished = [&]() {
    for (int w = 0; w < nw; ++w)
      if (done[w] != seq) return false;
    return true;
  };
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned k = 1; !finished(); ++k) {
    if ((k & 255) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipErrorNotReady) {
        if ((k & 0xFFFFF) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
          EVR_CHECK(false, "qnehvi plan: evaluation %llu did not complete within 30 s", seq);
        continue;
      }
      EVR_HIP(q);
      if (!finished()) EVR_CHECK(false, "qnehvi plan: evaluation finished without its completion words");
    }
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  return 0;
}

// One evaluation of the restart batch at host x: f = -sum_r acq_r, g = -dX.
static int plan_eval_host(hipStream_t s, evr_qnehvi_plan* p, const double* x, double* f, double* g) {
  const int b = p->b, n = b * p->md.d;
  if (int rc = plan_eval_raw(s, p, x)) return rc;
  double acc = 0.0;
  for (int r = 0; r < b; ++r) {
    if (std::isnan(p->hout[r])) {
      ::evr::set_error("acquisition: posterior covariance block not p.d. after the jitter ladder (NotPSDError)");
      return EVR_ERR_NOTPSD;
    }
    acc += p->hout[r];
  }
  *f = -acc;
  for (int i = 0; i < n; ++i) g[i] = -p->hout[b + i];
  return 0;
}

int evr_qnehvi_plan_eval_host(void* stream, evr_qnehvi_plan* p, const double* x, double* out) {
  EVR_CHECK(p && x && out, "evr_qnehvi_plan_eval_host: bad arguments");
  if (int rc = plan_eval_raw((hipStream_t)stream, p, x)) return rc;
  std::memcpy(out, p->hout, sizeof(double) * (size_t)p->b * (p->backward ? 1 + p->md.d : 1));
  return 0;
}

int evr_qnehvi_plan_minimize(void* stream, evr_qnehvi_plan* p, const double* x0, const double* lb, const double* ub,
                             int maxiter, int maxfun, double factr, double pgtol, int mcor, int maxls, double* x,
                             double* acq, int* info) {
  EVR_CHECK(p && p->backward && p->dX && x0 && lb && ub && x && acq && info && maxiter >= 1 && maxfun >= 1 &&
                mcor >= 1 && maxls >= 1 && factr >= 0.0 && pgtol >= 0.0,
            "evr_qnehvi_plan_minimize: bad arguments (needs a backward plan)");
  const int b = p->b, n = b * p->md.d;
  for (int i = 0; i < n; ++i) EVR_CHECK(!(lb[i] > ub[i]), "evr_qnehvi_plan_minimize: lower bound above upper bound");
  hipStream_t s = (hipStream_t)stream;
  Lbfgsb opt(n, mcor, lb, ub, factr, pgtol, maxls);
  std::vector<double> g(n);
  double f = 0.0;
  int task = opt.start(x0), nit = 0, nfev = 0, status = 0;
  // scipy's _minimize_lbfgsb driver loop
  for (;;) {
    if (task == LBFGSB_FG) {
      if (int rc = plan_eval_host(s, p, opt.x(), &f, g.data())) return rc;
      ++nfev;
      task = opt.step(f, g.data());
    } else if (task == LBFGSB_NEW_X) {
      ++nit;
      if (nit >= maxiter || nfev > maxfun) {
        status = 1;
        break;
      }
      task = opt.step(f, g.data());
    } else {
      status = task == LBFGSB_ABNORMAL ? 2 : task == LBFGSB_ERROR ? 3 : 0;
      break;
    }
  }
  for (int i = 0; i < n; ++i) x[i] = std::min(ub[i], std::max(lb[i], opt.x()[i]));
  // re-evaluate at the clipped candidates ([upstream] gen_candidates_scipy's final no-grad call)
  if (int rc = plan_eval_host(s, p, x, &f, g.data())) return rc;
  std::memcpy(acq, p->hout, sizeof(double) * b);
  info[0] = nit;
  info[1] = nfev;
  info[2] = status;
  info[3] = task;
  return 0;
}

}  // extern "C"
