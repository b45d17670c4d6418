// Phase profile of the restart-batch backward projection qs_bwd at the bench shape (n = 512,
// fused root: Rr = n + S + 1 = 769, S = 256, m = 5, b = 20, d = 6, RBF) on synthetic operands:
// per-workgroup wall-clock stamps (EVR_QS_PROF build of qnehvi_small.hip, s_memrealtime 10 ns):
// start -> coefficient loads issued -> M^T gR chunk loop + coefficient rounds -> epilogue
// loads / dk exchange -> gradient + store;
// means / max over workgroups, start spread, launch span, and the HIP-event time per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DEVR_QS_PROF tools/qs_prof.hip -o tools/_qs_prof
#include <cstdio>
#include <vector>
#include <algorithm>
#include <string>
#include "../everest_amd/csrc/qnehvi_small.hip"

namespace evr {
void set_error(const char*, ...) {}
int samples_norms(hipStream_t, const evr_qnehvi_state*, int, const double*, const double*, double*, double*, int*,
                  int) {
  return 0;
}
}  // namespace evr

static double* dev_fill(size_t n, double lo, double hi, unsigned seed) {
  std::vector<double> h(n);
  unsigned x = seed * 2654435761u + 1u;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = lo + (hi - lo) * (x >> 8) / double(1u << 24);
  }
  double* d = nullptr;
  if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  return d;
}

int main(int argc, char** argv) {
  // "tail": the backward over the sample rows only (TAIL build of qs_bwd), and the tail kernel
  // (qs_tail.hpp, standalone launch) timed on its own
  const bool tail = argc > 1 && std::string(argv[1]) == "tail";
  const int n = 512, nb = 0, S = 256, nh = S, m = 5, b = 20, d = 6, kind = 0;
  const int Rr = n + nb + nh + 1, nt = (n + 15) / 16;
  const int tiles = nt * m, nch = ((tail ? nh : Rr - 1) + 127) / 128;
  int zs = std::max(1, std::min(nch, 512 / std::max(1, tiles)));
  zs = (nch + (nch + zs - 1) / zs - 1) / ((nch + zs - 1) / zs);
  if (tail) zs = 1;   // qnehvi_small.hip qs_zsplit: one split over the sample rows
  const int rows_per = ((nch + zs - 1) / zs) * 128;
  const int za = (n + 255) / 256;
  const int npB = m * zs * nt, np = npB + (tail ? m * za * nt : 0);
  double* M = dev_fill((size_t)m * Rr * n, -1, 1, 1);
  double* R = dev_fill((size_t)m * Rr * b, -1, 1, 2);
  double* dG = dev_fill((size_t)S * m * b, -1e-3, 1e-3, 3);
  double* L22 = dev_fill((size_t)m * b, 0.1, 0.2, 4);
  double* ys = dev_fill(m, 0.5, 1.5, 5);
  double* zq = dev_fill((size_t)S * m, -2, 2, 6);
  double* oa = dev_fill(m, -1, -1, 7);
  double* Xn = dev_fill((size_t)n * d, 0, 1, 8);
  double* X = dev_fill((size_t)b * d, 0, 1, 9);
  double* ls = dev_fill((size_t)m * d, 0.3, 1.3, 10);
  double* dXp = dev_fill((size_t)b * d * np + m * b, 0, 0, 11);
  double* cfo = dXp + (size_t)b * d * np;
  if (!M || !R || !dG || !L22 || !ys || !zq || !oa || !Xn || !X || !ls || !dXp) {
    printf("{\"error\": \"alloc\"}\n");
    return 1;
  }
  const dim3 grid(nt, m, zs);
#define QSB(G_, T_)                                                                                               \
  evr::qs_bwd<<<G_, T_>>>(n, nb, nh, S, m, b, d, kind, M, R, dG, L22, ys, zq, oa, Xn, X, nullptr, nullptr, ls, dXp, nt, \
                          rows_per, np, cfo, zs, evr::QsTail{})
  const int nwg = nt * m * zs;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 5; ++r)
    QSB(grid, 256);
  (void)hipEventRecord(e0);
  const int reps = 20;
  for (int r = 0; r < reps; ++r)
    QSB(grid, 256);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st((size_t)4096 * 8);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(evr::qs_prof), st.size() * sizeof(unsigned long long));
  unsigned long long t0 = ~0ull, t1 = 0, smax = 0;
  double ph[4] = {0, 0, 0, 0}, pm[4] = {0, 0, 0, 0};
  for (int w = 0; w < nwg; ++w) {
    const unsigned long long* s = &st[(size_t)w * 8];
    t0 = std::min(t0, s[0]);
    t1 = std::max(t1, s[4]);
    smax = std::max(smax, s[0]);
    for (int k = 0; k < 4; ++k) {
      const double v = (double)(s[k + 1] - s[k]) / 100.0;
      ph[k] += v / nwg;
      pm[k] = std::max(pm[k], v);
    }
  }
  // the forward projection at the same shape (records from 2048 on)
  const int ntf = (Rr + 15) / 16;
  double* Kx = dev_fill((size_t)m * n * b, 0, 1, 12);
  double* Rf = dev_fill((size_t)m * Rr * b, 0, 0, 13);
  double* Pf = dev_fill((size_t)m * ntf * 2 * b, 0, 0, 14);
  for (int r = 0; r < 5; ++r) evr::qs_fwd<<<dim3(ntf, m), evr::QS_FT>>>(n, nb, Rr, b, M, Kx, Rf, Pf, ntf);
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) evr::qs_fwd<<<dim3(ntf, m), evr::QS_FT>>>(n, nb, Rr, b, M, Kx, Rf, Pf, ntf);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float msf = 0;
  (void)hipEventElapsedTime(&msf, e0, e1);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(evr::qs_prof), st.size() * sizeof(unsigned long long));
  unsigned long long f0 = ~0ull, f1 = 0;
  double fp[3] = {0, 0, 0}, fm[3] = {0, 0, 0};
  const int nwf = ntf * m;
  for (int w = 0; w < nwf; ++w) {
    const unsigned long long* s = &st[(size_t)(2048 + w) * 8];
    f0 = std::min(f0, s[0]);
    f1 = std::max(f1, s[3]);
    for (int k = 0; k < 3; ++k) {
      const double v = (double)(s[k + 1] - s[k]) / 100.0;
      fp[k] += v / nwf;
      fm[k] = std::max(fm[k], v);
    }
  }
  float mst = 0;
  if (tail) {
    evr::QsTail tl{M, Rf, Xn, X, nullptr, nullptr, ls, dXp, ys, n, nb, Rr, b, d, kind, nt, za, 256, npB, np,
                   m * za * nt};
    // the default mode: the tail's workgroups as the backward launch's z >= 1 slices
    const dim3 gc(nt, m, zs + za);
    auto comb = [&]() {
      evr::qs_bwd<<<gc, 256>>>(n, nb, nh, S, m, b, d, kind, M, R, dG, L22, ys, zq, oa, Xn, X, nullptr, nullptr, ls,
                               dXp, nt, rows_per, np, cfo, zs, tl);
    };
    for (int r = 0; r < 5; ++r) comb();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) comb();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float msc = 0;
    (void)hipEventElapsedTime(&msc, e0, e1);
    printf("{\"qs_bwd_with_tail\": {\"grid\": [%d, %d, %d], \"launch_us\": %.2f}}\n", nt, m, zs + za, msc * 1e3 / reps);
  }
  printf("{\"qs_fwd\": {\"grid\": [%d, %d], \"launch_us\": %.2f, \"span_us\": %.2f, \"first_chunk_us\": [%.2f, %.2f], "
         "\"other_chunks_us\": [%.2f, %.2f], \"epilogue_us\": [%.2f, %.2f]}}\n",
         ntf, m, msf * 1e3 / reps, (double)(f1 - f0) / 100.0, fp[0], fm[0], fp[1], fm[1], fp[2], fm[2]);
  printf("{\"grid\": [%d, %d, %d], \"rows_per\": %d, \"launch_us\": %.2f, \"span_us\": %.2f, \"start_spread_us\": %.2f, "
         "\"coef_us\": [%.2f, %.2f], \"chunks_us\": [%.2f, %.2f], \"epi_loads_exchange_us\": [%.2f, %.2f], "
         "\"gradient_store_us\": [%.2f, %.2f]}\n",
         nt, m, zs, rows_per, ms * 1e3 / reps, (double)(t1 - t0) / 100.0, (double)(smax - t0) / 100.0, ph[0], pm[0],
         ph[1], pm[1], ph[2], pm[2], ph[3], pm[3]);
  return 0;
}
