// Scrambled-Sobol normal base samples on the device.
//
// BoTorch draws qNEHVI's quasi-MC base samples with draw_sobol_normal_samples
// ([upstream] NormalQMCEngine(inv_transform=True) over torch.quasirandom.SobolEngine,
// scramble=True, seed drawn from the strategy's torch RNG, bofire/strategies/predictives/
// botorch.py:86): a 30-bit digital sequence with Owen/LMS scrambling, then
// z = sqrt(2) erfinv(2 (0.5 + (1 - eps)(u - 0.5)) - 1).  On the host that costs ~0.15 s per
// ask() at 2560 dimensions (scramble + serial draw + erfinv).  Here:
//   * evr_sobol_scramble (host): the scrambling matrices are the LSBs of the mt19937 stream
//     of torch.Generator().manual_seed(seed) (shift bits dim x 30, then dim x 30 x 30 lower-
//     triangular bits, upper triangle consumed and discarded, diagonal forced to 1), applied
//     to the direction numbers as GF(2) matrix-vector products — bit-identical to
//     SobolEngine.sobolstate / .shift;
//   * evr_sobol_normal (device): point k = shift XOR (XOR of direction numbers over the set
//     bits of gray(k)) — the closed form of the engine's sequential rightmost-zero walk —
//     scaled by 2^-30 (point 0 goes through float32 as SobolEngine._first_point does), then
//     the inverse-normal transform with torch's calc_erfinv (rational seed + 2 Newton steps).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <functional>
#include <new>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {

constexpr int SOBOL_MAXBIT = 30;

// torch calc_erfinv restated (c10/util/math_compat / ATen Math.h): Pavlis' rational
// approximation followed by two Newton-Raphson steps.
__device__ __forceinline__ double erfinv_torch(double y) {
#pragma clang fp contract(off)
  const double a0 = 0.886226899, a1 = -1.645349621, a2 = 0.914624893, a3 = -0.140543331;
  const double b0 = -2.118377725, b1 = 1.442710462, b2 = -0.329097515, b3 = 0.012229801;
  const double c0 = -1.970840454, c1 = -1.624906493, c2 = 3.429567803, c3 = 1.641345311;
  const double d0 = 3.543889200, d1 = 1.637067800;
  const double ya = fabs(y);
  if (ya > 1.0) return nan("");
  if (ya == 1.0) return copysign(INFINITY, y);
  double x;
  if (ya <= 0.7) {
    const double z = y * y;
    const double num = (((a3 * z + a2) * z + a1) * z + a0);
    const double dem = ((((b3 * z + b2) * z + b1) * z + b0) * z + 1.0);
    x = y * num / dem;
  } else {
    const double z = sqrt(-log((1.0 - ya) / 2.0));
    const double num = ((c3 * z + c2) * z + c1) * z + c0;
    const double dem = (d1 * z + d0) * z + 1.0;
    x = copysign(num, y) / dem;
  }
  const double two_over_sqrt_pi = 2.0 / 1.7724538509055159;  // (T)2 / (T)sqrt(pi)
  x = x - (erf(x) - y) / (two_over_sqrt_pi * exp(-x * x));
  x = x - (erf(x) - y) / (two_over_sqrt_pi * exp(-x * x));
  return x;
}

// layout 0: out[k * nd + t];  layout 1: out[(o * np + p) * n + k] with t = p * m + o.
__global__ __launch_bounds__(256) void sobol_normal_kernel(int n, int nd, int d0, const long long* __restrict__ V,
                                                           const long long* __restrict__ shift, int layout, int m,
                                                           double* __restrict__ out) {
#pragma clang fp contract(off)
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)n * nd) return;
  int k, t;
  if (layout == 0) {
    t = (int)(e % nd);
    k = (int)(e / nd);
  } else {
    k = (int)(e % n);
    t = (int)(e / n);
  }
  const int dim = d0 + t;
  double u;
  if (k == 0) {
    u = (double)(float)shift[dim] / 1073741824.0;  // _first_point: int64 / 2**30 in float32
  } else {
    long long x = shift[dim];
    unsigned g = (unsigned)k ^ ((unsigned)k >> 1);
    const long long* row = V + (size_t)dim * SOBOL_MAXBIT;
    while (g) {
      const int bit = __builtin_ctz(g);
      x ^= row[bit];
      g &= g - 1;
    }
    u = (double)x * (1.0 / 1073741824.0);
  }
  const double eps = 2.220446049250313e-16;
  const double v = 0.5 + (1.0 - eps) * (u - 0.5);
  const double z = erfinv_torch(2.0 * v - 1.0) * 1.4142135623730951;
  size_t idx;
  if (layout == 0) {
    idx = (size_t)k * nd + t;
  } else {
    const int p = t / m, o = t - p * m;
    const int np = nd / m;
    idx = ((size_t)o * np + p) * n + k;
  }
  out[idx] = z;
}

// The mt19937 stream of torch.Generator().manual_seed(seed) (std::mt19937 seeding) as raw
// (untempered) state words, block after block of 624, each block twisted straight from the
// previous one into the output (three vectorisable segments).  Only the lowest bit of each
// tempered draw is used; tempering is linear over GF(2), so that bit is parity(word & mask),
// evaluated by the consumers in parallel.  Same bits as std::mt19937 (tests compare the
// scrambled engine state with torch.quasirandom.SobolEngine's).
struct MtWords {
  static constexpr int N = 624, Mo = 397;
  static uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  static uint32_t lsb_mask() {
    uint32_t mask = 0;
    for (int k = 0; k < 32; ++k) mask |= (temper(1u << k) & 1u) << k;
    return mask;
  }
  static uint32_t step(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  // out: ceil(n / 624) * 624 words; *done (if given) publishes the words written so far.
  // The twist loops vectorise; an AVX2 clone is picked at run time where the host has it.
#define EVR_MT_GENERATE_BODY                                                                            \
  uint32_t init[N];                                                                                     \
  init[0] = seed;                                                                                       \
  for (int i = 1; i < N; ++i) init[i] = 1812433253u * (init[i - 1] ^ (init[i - 1] >> 30)) + (uint32_t)i; \
  const uint32_t* o = init;                                                                             \
  for (size_t blk = 0; blk * N < n; ++blk) {                                                            \
    uint32_t* w = out + blk * N;                                                                        \
    for (int i = 0; i < N - Mo; ++i) w[i] = step(o[i], o[i + 1], o[i + Mo]);                           \
    for (int i = N - Mo; i < N - 1; ++i) w[i] = step(o[i], o[i + 1], w[i + Mo - N]);                   \
    w[N - 1] = step(o[N - 1], w[0], w[Mo - 1]);                                                         \
    o = w;                                                                                              \
    if (done && (blk & 15) == 15) done->store((blk + 1) * N, std::memory_order_release);               \
  }                                                                                                     \
  if (done) done->store((n + N - 1) / N * N, std::memory_order_release);
  __attribute__((target("avx2"))) static void generate_avx2(uint32_t seed, size_t n, uint32_t* out,
                                                            std::atomic<size_t>* done) {
    EVR_MT_GENERATE_BODY
  }
  static void generate_base(uint32_t seed, size_t n, uint32_t* out, std::atomic<size_t>* done) {
    EVR_MT_GENERATE_BODY
  }
#undef EVR_MT_GENERATE_BODY
  static void generate(uint32_t seed, size_t n, uint32_t* out, std::atomic<size_t>* done = nullptr) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) generate_avx2(seed, n, out, done);
    else generate_base(seed, n, out, done);
  }
};

}  // namespace evr

using namespace evr;

extern "C" {

int evr_sobol_scramble(int dim, unsigned long long seed, long long* V, long long* shift) {
  return evr_sobol_scramble_range(dim, seed, 0, dim, V, shift);
}

}  // extern "C"

namespace evr {
// A persistent pool of scrambling workers: run(k, f) hands f(0..k-1) to k workers, wait()
// returns when all are done.  One job at a time (a mutex serialises concurrent draws from the
// acquisition's scrambling threads).
class SobolPool {
 public:
  void run(int k, std::function<void(int)> f) {
    job_mu_.lock();
    std::unique_lock<std::mutex> lk(mu_);
    while ((int)th_.size() < k) th_.emplace_back([this, i = (int)th_.size()] { loop(i); });
    f_ = std::move(f);
    k_ = k;
    left_ = k;
    ++gen_;
    cv_.notify_all();
  }
  void wait() {
    {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [this] { return left_ == 0; });
    }
    job_mu_.unlock();
  }

 private:
  void loop(int i) {
    unsigned long long seen = 0;
    for (;;) {
      std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (i >= k_) continue;
        f = &f_;
      }
      (*f)(i);
      std::unique_lock<std::mutex> lk(mu_);
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex mu_, job_mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> th_;
  std::function<void(int)> f_;
  int k_ = 0, left_ = 0;
  unsigned long long gen_ = 0;
};

static SobolPool& sobol_pool() {
  static SobolPool* p = new SobolPool();   // never destroyed: the workers live for the process
  return *p;
}

// Dimensions [d0, d0 + nd) of a dim-dimensional engine from the raw words wp of its seed's
// stream: shift bits (dim x 30), then the scrambling-matrix bits (dim x 30 x 30).  With
// `done`, the words are still being generated: each worker waits until its range is in.
static void scramble_apply(const uint32_t* wp, int dim, int d0, int nd, long long* V, long long* shift,
                           const std::function<void()>& producer, std::atomic<size_t>* done) {
  const size_t nshift = (size_t)dim * SOBOL_MAXBIT, per_dim = (size_t)SOBOL_MAXBIT * SOBOL_MAXBIT;
  const uint32_t mask = MtWords::lsb_mask();
  auto bit = [wp, mask](size_t i) { return (uint32_t)__builtin_parity(wp[i] & mask); };
  // V / shift hold the requested dimensions (row d - d0)
  auto work = [&](int dbeg, int dend) {
    uint32_t col[SOBOL_MAXBIT];
    for (int d = dbeg; d < dend; ++d) {
      long long sh = 0;
      for (int b = 0; b < SOBOL_MAXBIT; ++b) sh |= (long long)bit((size_t)d * SOBOL_MAXBIT + b) << b;
      shift[d - d0] = sh;
      // lower-triangular scrambling matrix L (row p: bits k < p drawn, diagonal 1, upper
      // triangle consumed and discarded); the scrambled direction number has bit 29 - p =
      // parity(row_p & v) with row_p's bit 29 - k = L[p][k].  Stored by columns: col[b] is
      // the output pattern of input bit b = 29 - k, so the product is an XOR over v's set bits.
      const size_t bd = nshift + (size_t)d * per_dim;
      for (int k = 0; k < SOBOL_MAXBIT; ++k) col[SOBOL_MAXBIT - 1 - k] = 1u << (SOBOL_MAXBIT - 1 - k);
      for (int p = 1; p < SOBOL_MAXBIT; ++p)
        for (int k = 0; k < p; ++k)
          col[SOBOL_MAXBIT - 1 - k] |= bit(bd + p * SOBOL_MAXBIT + k) << (SOBOL_MAXBIT - 1 - p);
      for (int j = 0; j < SOBOL_MAXBIT; ++j) {
        uint32_t v = (uint32_t)V[(size_t)(d - d0) * SOBOL_MAXBIT + j] & ((1u << SOBOL_MAXBIT) - 1u), t2 = 0;
        while (v) {
          t2 ^= col[__builtin_ctz(v)];
          v &= v - 1;
        }
        V[(size_t)(d - d0) * SOBOL_MAXBIT + j] = t2;
      }
    }
  };
  // worker threads: the job's host-thread share (EVR_HOST_THREADS / OMP_NUM_THREADS, default
  // 16 — the GPU box's share), at least 128 dimensions each (the baseline draw of the bench
  // ask, ~1.4 k dimensions, waited ~0.54 ms on 8 threads with the device idle)
  static const int nmax = [] {
    const char* e = std::getenv("EVR_HOST_THREADS");
    if (!e) e = std::getenv("OMP_NUM_THREADS");
    const int v = e ? std::atoi(e) : 16;
    return std::max(1, std::min(v > 0 ? v : 16, 32));
  }();
  const int nth = std::max(1, std::min(nmax, nd / 128));
  if (nth == 1) {
    if (producer) producer();
    work(d0, d0 + nd);
    return;
  }
  const int per = (nd + nth - 1) / nth;
  auto part = [&](int i) {
    const int a = d0 + i * per, b = std::min(d0 + nd, a + per);
    if (a >= b) return;
    if (done) {
      const size_t need = nshift + (size_t)b * per_dim;
      while (done->load(std::memory_order_acquire) < need) std::this_thread::yield();
    }
    work(a, b);
  };
  // the parts on the persistent pool (spawning 16 threads per draw cost ~0.2 ms); the calling
  // thread generates the words meanwhile, or takes part 0 itself
  if (producer) {
    sobol_pool().run(nth, part);
    producer();
    sobol_pool().wait();
  } else {
    sobol_pool().run(nth - 1, [&](int i) { part(i + 1); });
    part(0);
    sobol_pool().wait();
  }
}
}  // namespace evr

struct evr_sobol_stream {
  std::vector<uint32_t> words;
  size_t n;
};

extern "C" {

int evr_sobol_scramble_range(int dim, unsigned long long seed, int d0, int nd, long long* V, long long* shift) {
  EVR_CHECK(dim >= 1 && V && shift && d0 >= 0 && nd >= 1 && d0 + nd <= dim,
            "evr_sobol_scramble_range: bad arguments");
  // the raw words are generated serially by this thread while the workers, one dimension
  // range each, start as soon as the words of their range are published; the stream is
  // needed through the last requested dimension's matrix bits
  const size_t nshift = (size_t)dim * SOBOL_MAXBIT, per_dim = (size_t)SOBOL_MAXBIT * SOBOL_MAXBIT;
  const size_t nneed = nshift + (size_t)(d0 + nd) * per_dim;
  // per-thread buffer, kept between calls (an ask() scrambles ~10 MB of draws three times)
  thread_local std::vector<uint32_t> words;
  const size_t nw = (nneed + MtWords::N - 1) / MtWords::N * MtWords::N;
  if (words.size() < nw) words.resize(nw);
  uint32_t* wp = words.data();   // the caller's buffer (a thread_local name would resolve to
                                 // each worker's own, empty instance)
  const uint32_t seed32 = (uint32_t)(seed & 0xffffffffull);
  std::atomic<size_t> done{0};
  scramble_apply(wp, dim, d0, nd, V, shift, [&] { MtWords::generate(seed32, nneed, wp, &done); }, &done);
  return 0;
}

long long evr_sobol_stream_words(int dim) {
  return dim >= 1 ? (long long)dim * SOBOL_MAXBIT * (1 + SOBOL_MAXBIT) : 0;
}

int evr_sobol_stream_create(unsigned long long seed, long long nwords, evr_sobol_stream** out) {
  EVR_CHECK(out && nwords >= 1, "evr_sobol_stream_create: bad arguments");
  evr_sobol_stream* st = new (std::nothrow) evr_sobol_stream();
  EVR_CHECK(st, "evr_sobol_stream_create: out of host memory");
  st->n = (size_t)nwords;
  st->words.resize((st->n + MtWords::N - 1) / MtWords::N * MtWords::N);
  MtWords::generate((uint32_t)(seed & 0xffffffffull), st->n, st->words.data());
  *out = st;
  return 0;
}

int evr_sobol_scramble_stream(const evr_sobol_stream* st, int dim, int d0, int nd, long long* V, long long* shift) {
  EVR_CHECK(st && dim >= 1 && V && shift && d0 >= 0 && nd >= 1 && d0 + nd <= dim,
            "evr_sobol_scramble_stream: bad arguments");
  const size_t nshift = (size_t)dim * SOBOL_MAXBIT, per_dim = (size_t)SOBOL_MAXBIT * SOBOL_MAXBIT;
  EVR_CHECK(nshift + (size_t)(d0 + nd) * per_dim <= st->n,
            "evr_sobol_scramble_stream: stream of %zu words too short for %d dims", st->n, dim);
  scramble_apply(st->words.data(), dim, d0, nd, V, shift, nullptr, nullptr);
  return 0;
}

void evr_sobol_stream_destroy(evr_sobol_stream* st) { delete st; }

int evr_sobol_normal(void* stream, int n, int nd, int d0, const long long* V, const long long* shift, int layout,
                     int m, double* out) {
  EVR_CHECK(n >= 0 && nd >= 0 && d0 >= 0 && V && shift && out, "evr_sobol_normal: bad arguments");
  EVR_CHECK(layout == 0 || (layout == 1 && m >= 1 && nd % m == 0), "evr_sobol_normal: bad layout");
  EVR_CHECK(n <= (1 << 30), "evr_sobol_normal: n exceeds the 2^30 points of a 30-bit sequence");
  const long long tot = (long long)n * nd;
  if (tot == 0) return 0;
  sobol_normal_kernel<<<cdiv(tot, 256), 256, 0, (hipStream_t)stream>>>(n, nd, d0, V, shift, layout, m, out);
  EVR_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
