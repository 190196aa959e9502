// Host-AddressSanitizer driver for libpdd's C ABI (sanitizer
// build of the host code).  Built by scripts/asan_check.sh with the host
// side instrumented (-Xarch_host -fsanitize=address; device code untouched)
// and run on the GPU box.  It drives the host logic behind include/pdd.h --
// argument checks, sweep-plan table/chunk building, grouped plans, timing
// pools, create/destroy cycles -- on small random grids, and checks every
// sweep against a plain host sum:
//     plane[d][t] = sum_c X(c, t + table[d][c])   (pad 0 outside [0, N))
// Exit status 0 = all checks passed and no ASan report.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pdd.h"

static int failures = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      ++failures;                                          \
    }                                                      \
  } while (0)

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    std::exit(2);
  }
}

// one sweep of a random [C][N] 8-bit block over a random table, f32 or u8
static int factorised_cases = 0;
static void sweep_case(std::mt19937& rng, int64_t C, int64_t N, int64_t D, int span, int dtype,
                       bool timing, int flags = PDD_SWEEP_FACTOR) {
  std::vector<int32_t> tab((size_t)(D * C));
  std::uniform_int_distribution<int> sh(0, span);
  for (int64_t d = 0; d < D; ++d)
    for (int64_t c = 0; c < C; ++c)  // grows with d like a DM grid, jittered
      tab[(size_t)(d * C + c)] = (int32_t)((d * span) / std::max<int64_t>(1, D) * (C - c) / C + sh(rng) % 2);
  int mx = 0;
  for (int v : tab) mx = std::max(mx, v);
  const int64_t n_out = std::max<int64_t>(0, N - mx);
  std::vector<uint8_t> x8((size_t)(C * N));
  for (auto& v : x8) v = (uint8_t)(rng() & 255);
  std::vector<float> xf(x8.begin(), x8.end());

  pdd_sweep_plan* plan = nullptr;
  int rc = pdd_sweep_plan_create_ex(tab.data(), D, C, dtype, flags, &plan);
  CHECK(rc == 0 && plan, "plan_create C=%lld D=%lld span=%d dtype=%d: rc=%d %s", (long long)C,
        (long long)D, span, dtype, rc, pdd_last_error());
  if (rc != 0) return;
  int64_t n_pat = -1;
  const int fx = pdd_sweep_plan_factor(plan, &n_pat);
  CHECK(fx == 0 || ((fx == 2 || fx == 4) && C % fx == 0 && n_pat > 0),
        "factor %d (%lld patterns) for C=%lld dtype=%d", fx, (long long)n_pat, (long long)C, dtype);
  if (fx) ++factorised_cases;
  // unwritten pattern-image elements would show as NaNs / overflowed lanes
  CHECK(pdd_sweep_plan_set_poison(plan, 1) == 0, "set_poison");
  int64_t info[8] = {0};
  CHECK(pdd_sweep_plan_info(plan, info) == 0 && info[0] == D && info[1] == C, "plan_info");
  if (timing) CHECK(pdd_sweep_set_timing(plan, 1) == 0, "set_timing");

  const size_t in_bytes = (size_t)(C * N) * (dtype == PDD_F32 ? 4 : 1);
  void* dx = nullptr;
  float *dout = nullptr, *dpad = nullptr;
  const int64_t ld_out = std::max<int64_t>(1, n_out);
  hip_ok(hipMalloc(&dx, std::max<size_t>(in_bytes, 16)), "hipMalloc x");
  hip_ok(hipMalloc(&dout, (size_t)(D * ld_out) * 4), "hipMalloc out");
  hip_ok(hipMalloc(&dpad, (size_t)C * 4), "hipMalloc pads");
  hip_ok(hipMemcpy(dx, dtype == PDD_F32 ? (const void*)xf.data() : (const void*)x8.data(), in_bytes,
                   hipMemcpyHostToDevice), "H2D x");
  hip_ok(hipMemset(dpad, 0, (size_t)C * 4), "pads");
  rc = pdd_sweep_execute(plan, dx, N, N, PDD_PAD_VALUE, dpad, dout, ld_out, n_out, nullptr);
  CHECK(rc == 0, "execute: %s", pdd_last_error());
  hip_ok(hipDeviceSynchronize(), "sync");
  std::vector<float> got((size_t)(D * ld_out));
  hip_ok(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost), "D2H");
  int bad = 0;
  for (int64_t d = 0; d < D && bad < 5; ++d)
    for (int64_t t = 0; t < n_out && bad < 5; ++t) {
      double s = 0;
      for (int64_t c = 0; c < C; ++c) {
        const int64_t k = t + tab[(size_t)(d * C + c)];
        if (k >= 0 && k < N) s += x8[(size_t)(c * N + k)];
      }
      if ((double)got[(size_t)(d * ld_out + t)] != s) {
        ++bad;
        CHECK(false, "C=%lld N=%lld D=%lld span=%d dtype=%d variant=%lld max=%d: plane[%lld][%lld] = %g, want %g",
              (long long)C, (long long)N, (long long)D, span, dtype, (long long)info[7], mx, (long long)d, (long long)t,
              (double)got[(size_t)(d * ld_out + t)], s);
      }
    }
  if (timing) {
    float ms = -1;
    int64_t launches = -1;
    // a plan whose launches were not bracketed (generic kernel, empty plane)
    // reports "no timed launch"
    const int rt = pdd_sweep_timing_read(plan, &ms, &launches);
    CHECK((rt == 0 && launches >= 1 && ms >= 0) ||
              (rt != 0 && std::strstr(pdd_last_error(), "no timed launch")),
          "timing_read: rc %d, %lld launches: %s", rt, (long long)launches, pdd_last_error());
  }
  if (std::getenv("ABI_VERBOSE"))
    std::printf("case C=%lld N=%lld D=%lld span=%d dtype=%d timing=%d variant=%lld lds=%lld "
                "n_out=%lld bad=%d\n", (long long)C, (long long)N, (long long)D, span, dtype,
                (int)timing, (long long)info[7], (long long)info[4], (long long)n_out, bad);
  CHECK(pdd_sweep_plan_destroy(plan) == 0, "destroy");
  hip_ok(hipFree(dx), "free");
  hip_ok(hipFree(dout), "free");
  hip_ok(hipFree(dpad), "free");
}

// single-DM ops of include/pdd.h on small random blocks, against host loops;
// they share the library's per-stream scratch with the sweeps (partial sums,
// spectrum means, global statistics)
template <typename T>
static T* dev_copy(const std::vector<T>& h) {
  T* d = nullptr;
  hip_ok(hipMalloc(&d, std::max<size_t>(h.size() * sizeof(T), 16)), "hipMalloc");
  if (!h.empty()) hip_ok(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice), "H2D");
  return d;
}
template <typename T>
static std::vector<T> host_copy(const T* d, size_t n) {
  std::vector<T> h(n);
  hip_ok(hipDeviceSynchronize(), "sync");
  if (n) hip_ok(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost), "D2H");
  return h;
}

static void ops_case(std::mt19937& rng, int64_t C, int64_t N) {
  std::vector<uint8_t> x8((size_t)(C * N));  // time-major [N][C] for the prologues
  for (auto& v : x8) v = (uint8_t)(rng() & 255);
  // corner turn u8 [N][C] -> f32 [C][N]
  uint8_t* dx8 = dev_copy(x8);
  float* dcm = nullptr;
  hip_ok(hipMalloc(&dcm, (size_t)(C * N) * 4), "hipMalloc");
  CHECK(pdd_corner_turn(dx8, PDD_U8, N, C, C, dcm, PDD_F32, N, nullptr) == 0, "corner_turn: %s",
        pdd_last_error());
  std::vector<float> cm = host_copy(dcm, (size_t)(C * N));
  int bad = 0;
  for (int64_t c = 0; c < C; ++c)
    for (int64_t t = 0; t < N; ++t)
      bad += cm[(size_t)(c * N + t)] != (float)x8[(size_t)(t * C + c)];
  CHECK(bad == 0, "corner_turn C=%lld N=%lld: %d mismatches", (long long)C, (long long)N, bad);
  // shift + group sum (nsub 1 and C/4), value pads 7, shifts in [-40, 200]
  std::vector<int32_t> bins((size_t)C);
  for (auto& b : bins) b = (int32_t)(rng() % 241) - 40;
  int32_t* dbins = dev_copy(bins);
  std::vector<float> pads((size_t)C, 7.f);
  float* dpads = dev_copy(pads);
  for (int64_t nsub : {(int64_t)1, C / 4}) {
    if (nsub < 1 || C % nsub) continue;
    const int64_t n_out = std::max<int64_t>(1, N - 200);
    float* dout = nullptr;
    hip_ok(hipMalloc(&dout, (size_t)(nsub * n_out) * 4), "hipMalloc");
    CHECK(pdd_shift_group_sum(dcm, C, N, N, dbins, PDD_PAD_VALUE, dpads, nsub, dout, n_out, n_out,
                              nullptr) == 0, "shift_group_sum: %s", pdd_last_error());
    std::vector<float> got = host_copy(dout, (size_t)(nsub * n_out));
    const int64_t cps = C / nsub;
    int badg = 0;
    for (int64_t k = 0; k < nsub; ++k)
      for (int64_t t = 0; t < n_out; ++t) {
        double sum = 0;
        for (int64_t c = k * cps; c < (k + 1) * cps; ++c) {
          const int64_t u = t + bins[(size_t)c];
          sum += (u >= 0 && u < N) ? (double)x8[(size_t)(u * C + c)] : 7.0;
        }
        badg += (double)got[(size_t)(k * n_out + t)] != sum;
      }
    CHECK(badg == 0, "shift_group_sum C=%lld N=%lld nsub=%lld: %d mismatches", (long long)C,
          (long long)N, (long long)nsub, badg);
    hip_ok(hipFree(dout), "free");
  }
  // exact integer zero-DM + downsample by 2 (offset 510) of the time-major block
  if (C % 16 == 0 && N >= 2) {
    const int64_t f = 2, nout = N / f;
    uint16_t* dz = nullptr;
    hip_ok(hipMalloc(&dz, (size_t)(C * nout) * 2), "hipMalloc");
    CHECK(pdd_zdm_int_downsample(dx8, PDD_U8, N, C, C, f, PDD_ZDM_INT, 510, dz, nout, nullptr) == 0,
          "zdm_int_downsample: %s", pdd_last_error());
    std::vector<uint16_t> z = host_copy(dz, (size_t)(C * nout));
    std::vector<double> m((size_t)N);
    for (int64_t t = 0; t < N; ++t) {
      double sum = 0;
      for (int64_t c = 0; c < C; ++c) sum += x8[(size_t)(t * C + c)];
      m[(size_t)t] = std::nearbyint(sum / (double)C);  // round half to even
    }
    int badz = 0;
    for (int64_t c = 0; c < C; ++c)
      for (int64_t j = 0; j < nout; ++j) {
        double v = 510;
        for (int64_t k = 0; k < f; ++k) v += (double)x8[(size_t)((j * f + k) * C + c)] - m[(size_t)(j * f + k)];
        badz += (double)z[(size_t)(c * nout + j)] != v;
      }
    CHECK(badz == 0, "zdm_int_downsample C=%lld N=%lld: %d mismatches", (long long)C,
          (long long)N, badz);
    hip_ok(hipFree(dz), "free");
  }
  // whole-array statistics (float64 accumulation)
  float* d4 = nullptr;
  hip_ok(hipMalloc(&d4, 16), "hipMalloc");
  CHECK(pdd_global_stats(dcm, C, N, N, d4, nullptr) == 0, "global_stats: %s", pdd_last_error());
  std::vector<float> st = host_copy(d4, 4);
  double s1 = 0, s2 = 0, mn = 1e30, mx = -1e30;
  for (float v : cm) {
    s1 += v;
    mn = std::min(mn, (double)v);
    mx = std::max(mx, (double)v);
  }
  const double mean = s1 / (double)cm.size();
  for (float v : cm) s2 += (v - mean) * (v - mean);
  const double sd = std::sqrt(s2 / (double)cm.size());
  CHECK(std::fabs(st[0] - mean) <= 1e-4 * std::max(1.0, std::fabs(mean)) &&
            std::fabs(st[1] - sd) <= 1e-4 * std::max(1.0, sd) && st[2] == mn && st[3] == mx,
        "global_stats C=%lld N=%lld: {%g %g %g %g} want {%g %g %g %g}", (long long)C,
        (long long)N, st[0], st[1], st[2], st[3], mean, sd, mn, mx);
  hip_ok(hipFree(d4), "free");
  hip_ok(hipFree(dbins), "free");
  hip_ok(hipFree(dpads), "free");
  hip_ok(hipFree(dcm), "free");
  hip_ok(hipFree(dx8), "free");
}

int main() {
  int ndev = 0;
  hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  CHECK(pdd_version() >= 1, "version");
  CHECK(std::strlen(pdd_source_digest()) == 16, "source digest '%s'", pdd_source_digest());

  // argument checks: errors come back as status codes with a message
  pdd_sweep_plan* p = nullptr;
  int32_t t1[4] = {0, 1, 2, 3};
  CHECK(pdd_sweep_plan_create(nullptr, 1, 4, PDD_F32, &p) != 0 && std::strlen(pdd_last_error()),
        "null table accepted");
  CHECK(pdd_sweep_plan_create(t1, 0, 4, PDD_F32, &p) != 0, "D = 0 accepted");
  CHECK(pdd_sweep_plan_create(t1, 1, 4, 7, &p) != 0, "bad dtype accepted");
  CHECK(pdd_sweep_plan_create_grouped(t1, 0, 1, 4, PDD_F32, &p) != 0, "0 groups accepted");
  CHECK(pdd_sweep_execute(nullptr, nullptr, 1, 1, 0, nullptr, nullptr, 1, 1, nullptr) != 0,
        "null plan executed");
  CHECK(pdd_sweep_plan_destroy(nullptr) == 0 || std::strlen(pdd_last_error()), "destroy(null)");

  // random grids through every tiling rung the plan can pick
  std::mt19937 rng(1234);
  const int64_t Cs[] = {1, 7, 64, 96};
  const int64_t Ns[] = {1, 300, 5000};
  const int64_t Ds[] = {1, 5, 57, 130};
  const int spans[] = {0, 40, 900, 5000};
  int cases = 0;
  if (const char* one = std::getenv("ABI_ONE_CASE")) {  // "C,N,D,span,dtype,repeats"
    long long C, N, D;
    int span, dtype, reps;
    if (std::sscanf(one, "%lld,%lld,%lld,%d,%d,%d", &C, &N, &D, &span, &dtype, &reps) == 6) {
      for (int r = 0; r < reps; ++r) sweep_case(rng, C, N, D, span, dtype, (r & 1) != 0);
      std::printf("abi_asan: one case x %d, %d failures\n", reps, failures);
      return failures ? 1 : 0;
    }
  }
  for (int64_t C : Cs)
    for (int64_t N : Ns)
      for (int64_t D : Ds)
        for (int span : spans)
          for (int dtype : {PDD_F32, PDD_U8}) {
            if ((rng() & 3) != 0) continue;  // a quarter of the cross product
            sweep_case(rng, C, N, D, span, dtype, (cases & 1) != 0);
            ++cases;
          }

  // forced exact factorisation (groups of 4 / of 2 channels) on random
  // grids: the plan takes it wherever the windows fit, planes vs host sums
  const int before = factorised_cases;
  for (int64_t C : {8, 12, 64, 96})
    for (int64_t D : {5, 57, 130})
      for (int span : {0, 40, 300})
        for (int fl : {PDD_SWEEP_FACTOR | PDD_SWEEP_FACTOR_FORCE,
                       PDD_SWEEP_FACTOR | PDD_SWEEP_FACTOR_FORCE | PDD_SWEEP_FACTOR_G2}) {
          sweep_case(rng, C, 3000, D, span, PDD_U8, (D & 1) != 0, fl);
          ++cases;
        }
  CHECK(factorised_cases - before >= 24, "only %d forced grids factorised",
        factorised_cases - before);

  // single-DM ops interleaved with more sweeps (shared per-stream scratch)
  int ops = 0;
  for (int64_t C : {16, 64, 2048})
    for (int64_t N : {300, 4099}) {
      ops_case(rng, C, N);
      sweep_case(rng, 64, 3000, 40, 40, (ops & 1) ? PDD_U8 : PDD_F32, false);
      ++ops;
    }

  // grouped plans: create / info / destroy
  for (int rep = 0; rep < 20; ++rep) {
    const int64_t G = 1 + rep % 4, D = 3 + rep, C = 8 + 8 * (rep % 3);
    std::vector<int32_t> tab((size_t)(G * D * C));
    for (size_t i = 0; i < tab.size(); ++i) tab[i] = (int32_t)(i % 97);
    pdd_sweep_plan* q = nullptr;
    const int rc = pdd_sweep_plan_create_grouped(tab.data(), G, D, C, rep % 2 ? PDD_U8 : PDD_F32, &q);
    CHECK(rc == 0 && q, "grouped create rep %d: %s", rep, pdd_last_error());
    if (q) CHECK(pdd_sweep_plan_destroy(q) == 0, "grouped destroy");
  }
  // factorised plans do not chain: pdd_subband_chain says so (PDD_ENOCHAIN)
  // with nothing launched, instead of failing inside the stages
  {
    const int64_t C = 64, D = 48;
    std::vector<int32_t> tab((size_t)(D * C));
    for (int64_t d = 0; d < D; ++d)
      for (int64_t c = 0; c < C; ++c) tab[(size_t)(d * C + c)] = (int32_t)((d * (C - c)) / 16);
    pdd_sweep_plan *p1 = nullptr, *p2 = nullptr;
    const int r1 = pdd_sweep_plan_create_ex(tab.data(), D, C, PDD_U8,
                                            PDD_SWEEP_FACTOR | PDD_SWEEP_FACTOR_FORCE, &p1);
    std::vector<int32_t> tab2((size_t)(4 * D), 0);
    for (int64_t d = 0; d < 4; ++d)
      for (int64_t c = 0; c < D; ++c) tab2[(size_t)(d * D + c)] = (int32_t)(d * (D - c) / 8);
    const int r2 = pdd_sweep_plan_create_ex(tab2.data(), 4, D, PDD_F32, 0, &p2);
    CHECK(r1 == 0 && r2 == 0 && pdd_sweep_plan_factor(p1, nullptr) > 0,
          "chain plans: %d %d %s", r1, r2, pdd_last_error());
    if (r1 == 0 && r2 == 0) {
      const int64_t N = 4096;
      uint8_t* dx = nullptr;
      float *dpad = nullptr, *dout = nullptr;
      hip_ok(hipMalloc(&dx, (size_t)(C * N)), "hipMalloc x");
      hip_ok(hipMalloc(&dpad, (size_t)(D * 4) * 4), "hipMalloc pads");
      hip_ok(hipMalloc(&dout, (size_t)(4 * N) * 4), "hipMalloc out");
      hip_ok(hipMemset(dpad, 0, (size_t)(D * 4) * 4), "pads");
      const int rc = pdd_subband_chain(p1, dx, N, N, 1, PDD_PAD_VALUE, dpad, p2, dpad, dout, N,
                                       N - 64, 0, 1, nullptr);
      CHECK(rc == PDD_ENOCHAIN, "factorised stage-1 plan chained: rc %d %s", rc, pdd_last_error());
      hip_ok(hipDeviceSynchronize(), "sync");
      hip_ok(hipFree(dx), "free");
      hip_ok(hipFree(dpad), "free");
      hip_ok(hipFree(dout), "free");
    }
    if (p1) pdd_sweep_plan_destroy(p1);
    if (p2) pdd_sweep_plan_destroy(p2);
  }
  std::printf("abi_asan: %d sweep cases (%d factorised), %d op cases, %d failures\n", cases,
              factorised_cases, ops, failures);
  return failures ? 1 : 0;
}
