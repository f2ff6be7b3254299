// Host-side AddressSanitizer driver for the C ABI (race detection /
// sanitizers row) -- TEST INFRASTRUCTURE.
//
// Linked against csrc/*.hip built with -Xarch_host -fsanitize=address (host code only; the
// GPU code objects are not instrumented: GPU ASan is not available on this pool). It drives
// every reference-name host-pointer wrapper (the ones that hipMalloc / hipMemcpy / hipFree
// with early-exit cleanup) and the device entry points' argument checks:
//   1. invalid arguments (bad sizes, null pointers, out-of-range ranks): each must fail
//      with a message and no memory error;
//   2. with a GPU present: a small valid problem through every wrapper, checked against a
//      naive computation here, with every device buffer the library hipMallocs counted
//      (linker-wrapped hipMalloc / hipFree) and required to be freed again.
// Without a GPU (the CPU container), part 2 is replaced by the same calls failing at their
// first hipMalloc, which walks every wrapper's error-cleanup path under ASan.
// Exit status 0 = all checks passed (ASan aborts with its own report on a memory error).
#include <hip/hip_runtime.h>
#include <sanitizer/lsan_interface.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/minitorch_hip.h"

// Every hipMalloc / hipFree the library makes goes through these (linked with
// -Wl,--wrap=hipMalloc,--wrap=hipFree): the count of live device buffers must return to
// zero after each wrapper call. (hipMemGetInfo is no leak detector here: the runtime's
// sub-allocator keeps freed small blocks, so free device memory drifts down either way.)
static long g_live = 0, g_mallocs = 0;
extern "C" hipError_t __real_hipMalloc(void** p, size_t n);
extern "C" hipError_t __real_hipFree(void* p);
extern "C" hipError_t __wrap_hipMalloc(void** p, size_t n) {
  const hipError_t e = __real_hipMalloc(p, n);
  if (e == hipSuccess && *p) { ++g_live; ++g_mallocs; }
  return e;
}
extern "C" hipError_t __wrap_hipFree(void* p) {
  if (p) --g_live;
  return __real_hipFree(p);
}

static int g_fail = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);              \
      fprintf(stderr, "\n");                     \
      ++g_fail;                                  \
    }                                            \
  } while (0)

static std::vector<float> randv(size_t n, unsigned seed) {
  std::vector<float> v(n);
  unsigned s = seed * 2654435761u + 1;
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
  }
  return v;
}

static double maxdiff(const std::vector<float>& a, const std::vector<double>& b) {
  double m = 0;
  for (size_t i = 0; i < a.size(); ++i) m = std::fmax(m, std::fabs((double)a[i] - b[i]));
  return m;
}

// naive attention for one [BH, N, d] problem: O and dQ/dK/dV for upstream dO
static void naive_attn(const std::vector<float>& q, const std::vector<float>& k,
                       const std::vector<float>& v, const std::vector<float>& dO, int BH, int N,
                       int d, bool causal, std::vector<double>& o, std::vector<double>& dq,
                       std::vector<double>& dk, std::vector<double>& dv) {
  const double sc = 1.0 / std::sqrt((double)d);
  o.assign((size_t)BH * N * d, 0); dq = o; dk = o; dv = o;
  std::vector<double> p(N), dp(N);
  for (int h = 0; h < BH; ++h) {
    const size_t b = (size_t)h * N * d;
    for (int i = 0; i < N; ++i) {
      const int kn = causal ? i + 1 : N;
      double mx = -1e300, sum = 0;
      for (int j = 0; j < kn; ++j) {
        double s = 0;
        for (int x = 0; x < d; ++x) s += (double)q[b + i * d + x] * k[b + j * d + x];
        p[j] = s * sc;
        mx = std::fmax(mx, p[j]);
      }
      for (int j = 0; j < kn; ++j) { p[j] = std::exp(p[j] - mx); sum += p[j]; }
      for (int j = 0; j < kn; ++j) p[j] /= sum;
      double delta = 0;
      for (int j = 0; j < kn; ++j) {
        dp[j] = 0;
        for (int x = 0; x < d; ++x) {
          o[b + i * d + x] += p[j] * v[b + j * d + x];
          dp[j] += (double)dO[b + i * d + x] * v[b + j * d + x];
        }
        delta += p[j] * dp[j];
      }
      for (int j = 0; j < kn; ++j) {
        const double ds = p[j] * (dp[j] - delta) * sc;
        for (int x = 0; x < d; ++x) {
          dq[b + i * d + x] += ds * k[b + j * d + x];
          dk[b + j * d + x] += ds * q[b + i * d + x];
          dv[b + j * d + x] += p[j] * dO[b + i * d + x];
        }
      }
    }
  }
}

static void invalid_args() {
  float one = 0.f;
  float* f = &one;
  // device entry points: argument checks before any launch
  CHECK(mt_flash_attn_fwd(MT_F32, 0, f, f, f, f, f, f, 0, 1, 1, 1, 0, 0, 0, 0, 0) != 0, "B=0 accepted");
  CHECK(mt_flash_attn_fwd(7, 0, f, f, f, f, f, f, 1, 1, 1, 1, 0, 0, 0, 0, 0) != 0, "dtype 7 accepted");
  CHECK(mt_flash_attn_fwd(MT_F32, 0, nullptr, f, f, f, f, f, 1, 1, 1, 1, 0, 0, 0, 0, 0) != 0,
        "null q accepted");
  CHECK(strlen(mt_last_error()) > 0, "no error message");
  CHECK(mt_flash_attn_fwd(MT_F32, 0, f, f, f, f, f, f, 1, 1, 1, 5000, 0, 0, 0, 0, 0) != 0, "d=5000 accepted");
  CHECK(mt_flash_attn_bwd(MT_F32, 0, f, f, f, f, f, f, f, f, f, f, 1, -1, 1, 1, 0, 0, 0) != 0,
        "H=-1 accepted");
  int64_t shp[9] = {1, 1, 1, 1, 1, 1, 1, 1, 1}, st[9] = {1, 1, 1, 1, 1, 1, 1, 1, 1};
  CHECK(mt_tensor_map(1, f, shp, st, 9, f, shp, st, 9, 0) != 0, "rank 9 accepted");
  CHECK(mt_tensor_reduce(1, f, shp, st, f, shp, st, 2, 5, 0.f, 0) != 0, "reduce dim 5 accepted");
  CHECK(mt_flash_set_kernel_policy(-12345) != 0, "unknown policy accepted");
  // host wrappers: rejected before allocating (they print and return)
  launch_flashattention_forward(f, f, f, f, f, f, -1, 2, 3, 4);
  launch_flashattention_forward_causal(nullptr, f, f, f, f, f, 1, 1, 1, 1);
  launch_flashattention_backward(f, f, f, f, f, f, f, f, f, f, 1, 1, 0, 4);
  launch_flashattention_backward_causal(f, f, f, f, f, f, f, f, nullptr, f, 1, 1, 1, 1);
  int ishp[9] = {1, 1, 1, 1, 1, 1, 1, 1, 1}, ist[9] = {1, 1, 1, 1, 1, 1, 1, 1, 1};
  tensorMap(f, ishp, ist, 1, f, ishp, ist, 1, 9, 1);  // rank 9: refused, no overflow
  tensorMap(f, ishp, ist, 1, f, ishp, ist, 1, 0, 1);
  tensorReduce(f, ishp, ist, 1, f, ishp, ist, 3, 0.f, 9, 1);
}

// --bisect: run one wrapper group at a time (1 flash, 2 softmax, 3 layernorm, 4 combine)
static int g_only = 0;
static bool want(int g) { return g_only == 0 || g_only == g; }

static void valid_problems(bool gpu) {
  const int B = 1, H = 2, N = 37, d = 24, BH = B * H;
  const size_t n = (size_t)BH * N * d, r = (size_t)BH * N;
  auto q = randv(n, 1), k = randv(n, 2), v = randv(n, 3), dO = randv(n, 4);
  std::vector<double> ro, rdq, rdk, rdv;
  for (int causal = 0; causal < 2 && want(1); ++causal) {
    naive_attn(q, k, v, dO, BH, N, d, causal, ro, rdq, rdk, rdv);
    std::vector<float> o(n, 7.f), m(r), l(r), dq(n), dk(n), dv(n);
    auto fwd = causal ? launch_flashattention_forward_causal : launch_flashattention_forward;
    auto bwd = causal ? launch_flashattention_backward_causal : launch_flashattention_backward;
    fwd(q.data(), k.data(), v.data(), o.data(), l.data(), m.data(), B, H, N, d);
    bwd(q.data(), k.data(), v.data(), o.data(), dq.data(), dk.data(), dv.data(), dO.data(),
        l.data(), m.data(), B, H, N, d);
    if (gpu) {
      CHECK(maxdiff(o, ro) < 1e-5, "O (causal=%d) off by %g", causal, maxdiff(o, ro));
      CHECK(maxdiff(dq, rdq) < 1e-5, "dQ off by %g", maxdiff(dq, rdq));
      CHECK(maxdiff(dk, rdk) < 1e-5, "dK off by %g", maxdiff(dk, rdk));
      CHECK(maxdiff(dv, rdv) < 1e-5, "dV off by %g", maxdiff(dv, rdv));
    }
  }
  // companion wrappers
  const int rows = 2 * 4 * 5, to = 9;
  auto s = randv((size_t)rows * to, 5), mask = randv(2 * to, 6), g = randv((size_t)rows * to, 7);
  std::vector<float> s0 = s;
  if (want(2)) launch_attn_softmax(s.data(), mask.data(), 2, 4, 5, to, false, nullptr);
  if (gpu && want(2)) {
    double worst = 0;
    for (int i = 0; i < rows; ++i) {
      const float* x = &s0[(size_t)i * to];
      const float* mk = &mask[(size_t)(i / 20) * to];
      double mx = -1e300, sum = 0;
      for (int j = 0; j < to; ++j) mx = std::fmax(mx, (double)x[j] + mk[j]);
      for (int j = 0; j < to; ++j) sum += std::exp(x[j] + mk[j] - mx);
      for (int j = 0; j < to; ++j)
        worst = std::fmax(worst, std::fabs(s[(size_t)i * to + j] - std::exp(x[j] + mk[j] - mx) / (sum + 1e-8)));
    }
    CHECK(worst < 1e-6, "softmax off by %g", worst);
  }
  if (want(2)) launch_attn_softmax_bw(g.data(), s.data(), rows, to, nullptr);
  const int R = 13, Hd = 32;
  auto x = randv((size_t)R * Hd, 8), gm = randv(Hd, 9), bt = randv(Hd, 10), dy = randv((size_t)R * Hd, 11);
  std::vector<float> ln((size_t)R * Hd), var(R), mean(R), dg(Hd), db(Hd), dx((size_t)R * Hd);
  if (want(3)) launch_layernorm(ln.data(), var.data(), mean.data(), x.data(), gm.data(), bt.data(), R, Hd, nullptr);
  if (want(3)) launch_layernorm_bw(dg.data(), db.data(), dx.data(), dy.data(), x.data(), gm.data(), bt.data(),
                      var.data(), mean.data(), R, Hd, nullptr, nullptr);
  if (gpu && want(3)) {
    double worst = 0;
    for (int i = 0; i < R; ++i) {
      double mu = 0, sq = 0;
      for (int j = 0; j < Hd; ++j) { mu += x[i * Hd + j]; sq += (double)x[i * Hd + j] * x[i * Hd + j]; }
      mu /= Hd;
      const double vr = sq / Hd - mu * mu + 1e-8;
      for (int j = 0; j < Hd; ++j)
        worst = std::fmax(worst, std::fabs(ln[i * Hd + j] - (gm[j] * (x[i * Hd + j] - mu) / std::sqrt(vr) + bt[j])));
    }
    CHECK(worst < 1e-4, "layernorm off by %g", worst);
  }
  // combine wrappers: c = a @ b, out = a + b, reduce sum over dim 1
  int sa[3] = {1, 3, 4}, sta[3] = {12, 4, 1}, sb[3] = {1, 4, 5}, stb[3] = {20, 5, 1},
      sc[3] = {1, 3, 5}, stc[3] = {15, 5, 1};
  auto a = randv(12, 12), bm = randv(20, 13);
  std::vector<float> c(15), z(12), red(3);
  if (!want(4)) return;
  MatrixMultiply(c.data(), sc, stc, a.data(), sa, sta, bm.data(), sb, stb, 1, 3, 5);
  tensorZip(z.data(), sa, sta, 12, 3, a.data(), sa, sta, 12, 3, a.data(), sa, sta, 12, 3, 1);
  int sr[3] = {1, 3, 1}, str_[3] = {3, 1, 1};
  tensorReduce(red.data(), sr, str_, 3, a.data(), sa, sta, 2, 0.f, 3, 1);
  tensorMap(z.data(), sa, sta, 12, a.data(), sa, sta, 12, 3, 4);
  if (gpu) {
    double wc = 0, wr = 0, wz = 0;
    for (int i = 0; i < 3; ++i) {
      double rs = 0;
      for (int j = 0; j < 4; ++j) rs += a[i * 4 + j];
      wr = std::fmax(wr, std::fabs(red[i] - rs));
      for (int j = 0; j < 5; ++j) {
        double acc = 0;
        for (int t = 0; t < 4; ++t) acc += (double)a[i * 4 + t] * bm[t * 5 + j];
        wc = std::fmax(wc, std::fabs(c[i * 5 + j] - acc));
      }
    }
    for (int i = 0; i < 12; ++i) wz = std::fmax(wz, std::fabs(z[i] + a[i]));
    CHECK(wc < 1e-5 && wr < 1e-5 && wz == 0, "combine off: mm %g reduce %g map %g", wc, wr, wz);
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);  // a sanitizer exit must not lose the progress lines
  int ndev = 0;
  const bool gpu = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
  printf("capi_asan: %s\n", gpu ? "GPU present: full wrapper paths" : "no GPU: error-cleanup paths");
  invalid_args();
  for (g_only = 1; g_only <= 4; ++g_only) {  // each wrapper group alone, then all together
    valid_problems(gpu);
    CHECK(g_live == 0, "group %d left %ld device buffers allocated", g_only, g_live);
  }
  g_only = 0;
  for (int it = 0; it < (gpu ? 5 : 1); ++it) valid_problems(gpu);
  CHECK(g_live == 0, "%ld device buffers left allocated", g_live);
  printf("capi_asan: %ld device allocations, %ld still live\n", g_mallocs, g_live);
  if (gpu) CHECK(g_mallocs > 100, "the wrappers' hipMalloc calls were not intercepted");
  // Leak check now, then leave without running the ROCm runtime's static destructors:
  // with a GPU present, libamdhip64's __cxa_finalize tears the HSA runtime down and then
  // frees host objects that ASan's device-aware allocator can no longer release
  // ("CHECK failed: sanitizer_allocator_device.h:125 dev_runtime_unloaded_", exit 1,
  // GPUTEST_r05) -- a teardown-order fault of the sanitizer runtime, after every check here.
  const int leaks = __lsan_do_recoverable_leak_check();
  CHECK(leaks == 0, "LeakSanitizer reported leaks (see its report above)");
  printf("capi_asan: %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
  fflush(stdout);
  fflush(stderr);
  _exit(g_fail ? 1 : 0);
}
