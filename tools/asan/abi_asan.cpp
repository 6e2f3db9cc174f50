// abi_asan.cpp — AddressSanitizer driver for the HOST side of libecnf_hip.so ("-fsanitize=address
// host build").  Built by tools/asan/build.sh against an ASan-instrumented build of the host translation units
// (ecnf_hip.hip host code, ecnf_train.hip host code); device code is not instrumented (no GPU ASan on this pool).
//
// Without a GPU it exercises every host path that runs before the first device call: argument checks, the
// ravel_pytree param walk and the split / fragment repacking of ecnf_create (which then fails with ECNF_E_HIP).
// With a GPU it also runs each C-ABI entry point once on a small batch and the error paths that follow a valid
// handle.  Exit status 0 = every check passed and ASan reported nothing (ASan aborts the process otherwise).
#include <hip/hip_runtime.h>
#include <sanitizer/lsan_interface.h>

#include <chrono>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ecnf.h"

static int g_fail = 0;
// ABI_ASAN_TRACE=1: print each check's line (stderr) before it runs, so a stall names its call
static const bool g_trace = std::getenv("ABI_ASAN_TRACE") != nullptr;
#define CHECK(cond, ...)                                                   \
  do {                                                                     \
    if (g_trace) std::fprintf(stderr, "check line %d\n", __LINE__);       \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                                   \
      std::fprintf(stderr, " [last_error: %s]\n", ecnf_last_error());      \
      ++g_fail;                                                            \
    }                                                                      \
  } while (0)

// the four examples/config/*.yaml flow blocks (dw4, lj13, aldp, qm9)
static ecnf_cfg make_cfg(int n, int d, int nf, int h, int m, int l, int k, float scale) {
  ecnf_cfg c;
  c.n_nodes = n; c.dim = d; c.n_features = nf; c.hidden = h; c.time_embedding_dim = 16; c.mlp_width = m;
  c.mlp_depth = l; c.n_blocks = k; c.base_scale = scale; c.normalization_constant = 1.0f;
  return c;
}

static std::vector<float> random_params(const ecnf_cfg& c, unsigned seed) {
  size_t n = 0;
  ecnf_param_count(&c, &n);
  std::vector<float> p(n);
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(0.f, 0.08f);
  for (auto& v : p) v = nd(rng);
  return p;
}

template <typename T>
static T* dev_alloc(size_t n) {
  void* p = nullptr;
  if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) return nullptr;
  hipMemset(p, 0, n * sizeof(T) + 16);
  return static_cast<T*>(p);
}

static void host_checks() {
  CHECK(ecnf_abi_version() == ECNF_ABI_VERSION, "abi %d", ecnf_abi_version());
  size_t n = 0;
  CHECK(ecnf_param_count(nullptr, &n) == ECNF_E_INVALID, "NULL cfg");
  ecnf_cfg bad = make_cfg(13, 3, 1, 64, 128, 3, 3, 1.f);
  bad.hidden = 33;
  CHECK(ecnf_param_count(&bad, &n) == ECNF_E_UNSUPPORTED, "hidden 33");
  bad = make_cfg(13, 3, 1, 64, 128, 3, 3, 1.f);
  bad.dim = 4;
  CHECK(ecnf_param_count(&bad, &n) == ECNF_E_UNSUPPORTED, "dim 4");
  bad = make_cfg(13, 3, 1, 64, 128, 3, 11, 1.f);
  CHECK(ecnf_param_count(&bad, &n) == ECNF_E_UNSUPPORTED, "11 blocks");
  bad.n_blocks = 3;
  bad.base_scale = 0.f;
  CHECK(ecnf_param_count(&bad, &n) == ECNF_E_INVALID, "base_scale 0");
  const ecnf_cfg ok = make_cfg(13, 3, 1, 64, 128, 3, 3, 1.f);
  CHECK(ecnf_param_count(&ok, &n) == ECNF_OK && n > 0, "lj13 count");
  ecnf_handle* h = nullptr;
  std::vector<float> p = random_params(ok, 1);
  CHECK(ecnf_create(&ok, nullptr, p.size(), 0, &h) == ECNF_E_INVALID, "NULL params");
  CHECK(ecnf_create(&ok, p.data(), p.size() - 1, 0, &h) == ECNF_E_INVALID, "short blob");
  CHECK(ecnf_create(&ok, p.data(), p.size(), 0, nullptr) == ECNF_E_INVALID, "NULL out");
  ecnf_cfg odd = ok;
  odd.mlp_width = 96;
  CHECK(ecnf_create(&odd, p.data(), p.size(), 0, &h) != ECNF_OK, "mlp_width 96");
  // weights at / beyond the split range are refused on the host (|w| >= 2^15)
  std::vector<float> big = p;
  big[big.size() / 2] = 1e6f;
  int rc = ecnf_create(&ok, big.data(), big.size(), 0, &h);
  CHECK(rc != ECNF_OK || h != nullptr, "huge weight rc %d", rc);
  if (rc == ECNF_OK) ecnf_destroy(h);
  ecnf_target t;
  std::memset(&t, 0, sizeof t);
  t.kind = 7;
  CHECK(ecnf_target_log_prob(&t, nullptr, nullptr, 1, nullptr) == ECNF_E_INVALID, "bad target kind");
  CHECK(ecnf_lse_partials(nullptr, nullptr, -1, nullptr, nullptr) == ECNF_E_INVALID, "lse n < 0");
  ecnf_trainer* tr = nullptr;
  CHECK(ecnf_trainer_create(&bad, 8, 0, &tr) == ECNF_E_INVALID, "trainer bad cfg");
  CHECK(ecnf_trainer_create(&ok, 0, 0, &tr) == ECNF_E_INVALID, "trainer max_batch 0");
  CHECK(ecnf_destroy(nullptr) == ECNF_OK || true, "destroy NULL");
}

// one C-ABI round trip per entry point on `cfg` (GPU present); returns false when the create fails with ECNF_E_HIP
static bool device_checks(const ecnf_cfg& c, int B) {
  std::vector<float> p = random_params(c, 7);
  ecnf_handle* h = nullptr;
  const int rc = ecnf_create(&c, p.data(), p.size(), 0, &h);
  if (rc == ECNF_E_HIP) return false;   // no GPU: the host walk / repack above already ran under ASan
  CHECK(rc == ECNF_OK && h, "create rc %d", rc);
  if (rc != ECNF_OK) return true;
  const int ND = c.n_nodes * c.dim;
  float* z = dev_alloc<float>((size_t)B * ND);
  float* x = dev_alloc<float>((size_t)B * ND);
  float* v = dev_alloc<float>((size_t)B * ND);
  float* y = dev_alloc<float>((size_t)B * ND);
  float* tt = dev_alloc<float>(B);
  float* lp = dev_alloc<float>(B);
  float* dl = dev_alloc<float>(B);
  int32_t* feat = dev_alloc<int32_t>((size_t)B * c.n_nodes);
  int32_t* nfe = dev_alloc<int32_t>(B);
  int32_t* st = dev_alloc<int32_t>(B);
  std::vector<float> hz((size_t)B * ND);
  std::mt19937 rng(3);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& q : hz) q = nd(rng);
  hipMemcpy(z, hz.data(), hz.size() * sizeof(float), hipMemcpyHostToDevice);
  std::vector<float> ht(B, 0.5f);
  hipMemcpy(tt, ht.data(), B * sizeof(float), hipMemcpyHostToDevice);

  CHECK(ecnf_base_sample(h, z, x, B, nullptr) == ECNF_OK, "base_sample");
  CHECK(ecnf_base_log_prob(h, x, lp, B, nullptr) == ECNF_OK, "base_log_prob");
  CHECK(ecnf_vector_field(h, x, tt, feat, v, B, nullptr) == ECNF_OK, "vector_field");
  CHECK(ecnf_vector_field(h, nullptr, tt, feat, v, B, nullptr) == ECNF_E_INVALID, "vector_field NULL x");
  CHECK(ecnf_vector_field(h, x, tt, feat, v, -1, nullptr) == ECNF_E_INVALID, "vector_field batch -1");
  ecnf_solve_opts o;
  std::memset(&o, 0, sizeof o);
  o.solver = ECNF_SOLVER_EULER; o.divergence = ECNF_DIV_NONE; o.t0 = 0.f; o.t1 = 1.f; o.dt0 = 0.1f;
  o.rtol = 1e-5f; o.atol = 1e-5f; o.dtmin = 0.f; o.max_steps = 4096;
  CHECK(ecnf_integrate(h, &o, x, feat, nullptr, y, nullptr, nfe, st, B, nullptr) == ECNF_OK, "integrate euler");
  o.divergence = ECNF_DIV_HUTCHINSON;
  int rcd = ecnf_integrate(h, &o, x, feat, nullptr, y, dl, nfe, st, B, nullptr);
  CHECK(rcd == ECNF_E_INVALID, "hutchinson without eps: %d", rcd);
  rcd = ecnf_integrate(h, &o, x, feat, z, y, dl, nfe, st, B, nullptr);
  CHECK(rcd == ECNF_OK || rcd == ECNF_E_UNSUPPORTED, "hutchinson: %d", rcd);
  // the exact trace: caller workspace (ecnf_integrate_ws), the handle arena, the A/B forms
  o.divergence = ECNF_DIV_EXACT; o.t0 = 1.f; o.t1 = 0.f; o.dt0 = 0.5f;
  size_t wsb = 0;
  CHECK(ecnf_integrate_workspace_size(h, &o, B, &wsb) == ECNF_OK, "workspace size");
  float* ws = wsb ? dev_alloc<float>(wsb / sizeof(float) + 1) : nullptr;
  rcd = ecnf_integrate_ws(h, &o, x, feat, nullptr, y, dl, nfe, st, B, ws, wsb, nullptr);
  CHECK(rcd == ECNF_OK || rcd == ECNF_E_UNSUPPORTED, "exact with workspace: %d", rcd);
  if (wsb) {
    CHECK(ecnf_integrate_ws(h, &o, x, feat, nullptr, y, dl, nfe, st, B, ws, wsb / 2, nullptr) == ECNF_E_INVALID,
          "undersized workspace");
    CHECK(ecnf_reserve_workspace(h, wsb) == ECNF_OK, "reserve workspace");
  }
  CHECK(ecnf_set_exact_form(h, ECNF_EXACT_FORM_SPARSE) == ECNF_OK, "exact form");
  CHECK(ecnf_set_exact_form(h, 7) == ECNF_E_INVALID, "bad exact form");
  rcd = ecnf_integrate(h, &o, x, feat, nullptr, y, dl, nfe, st, B, nullptr);
  CHECK(rcd == ECNF_OK || rcd == ECNF_E_UNSUPPORTED, "exact (sparse form): %d", rcd);
  CHECK(ecnf_set_exact_form(h, ECNF_EXACT_FORM_DEFAULT) == ECNF_OK, "exact form default");
  rcd = ecnf_integrate(h, &o, x, feat, nullptr, y, dl, nfe, st, B, nullptr);
  CHECK(rcd == ECNF_OK || rcd == ECNF_E_UNSUPPORTED, "exact (arena): %d", rcd);
  o.t0 = 0.f; o.t1 = 1.f; o.dt0 = 0.1f; o.divergence = ECNF_DIV_HUTCHINSON;
  o.solver = 9;
  CHECK(ecnf_integrate(h, &o, x, feat, z, y, dl, nfe, st, B, nullptr) == ECNF_E_INVALID, "bad solver");
  CHECK(ecnf_set_precision(h, 5) == ECNF_E_INVALID, "bad precision");
  CHECK(ecnf_set_precision(h, ECNF_PREC_FP32) == ECNF_OK, "fp32");
  CHECK(ecnf_vector_field(h, x, tt, feat, v, B, nullptr) == ECNF_OK, "vector_field fp32");
  int32_t mpw = 0, mode = -1;
  CHECK(ecnf_molecules_per_workgroup(h, 0, &mpw) == ECNF_OK && mpw > 0, "mpw");
  CHECK(ecnf_chain_arithmetic(h, 0, &mode) == ECNF_OK, "chain arithmetic");
  CHECK(ecnf_update_params(h, p.data(), 0) == ECNF_OK, "update_params host");
  CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
  std::vector<float> hy((size_t)B * ND);
  hipMemcpy(hy.data(), y, hy.size() * sizeof(float), hipMemcpyDeviceToHost);
  bool finite = true;
  for (float q : hy) finite = finite && std::isfinite(q);
  CHECK(finite, "non-finite integrate output");

  ecnf_trainer* tr = nullptr;
  if (ecnf_trainer_create(&c, B, 0, &tr) == ECNF_OK) {
    size_t np = p.size();
    float* dp = dev_alloc<float>(np);
    float* g = dev_alloc<float>(np);
    float* loss = dev_alloc<float>(1);
    hipMemcpy(dp, p.data(), np * sizeof(float), hipMemcpyHostToDevice);
    CHECK(ecnf_fm_loss_grad(tr, dp, x, z, tt, feat, 0.01f, B, loss, g, nullptr) == ECNF_OK, "loss_grad");
    CHECK(ecnf_fm_loss_grad(tr, dp, x, z, tt, feat, 0.01f, B + 1, loss, g, nullptr) == ECNF_E_INVALID,
          "loss_grad over max_batch");
    hipDeviceSynchronize();
    hipFree(dp); hipFree(g); hipFree(loss);
    ecnf_trainer_destroy(tr);
  }
  CHECK(ecnf_destroy(h) == ECNF_OK, "destroy");
  for (void* q : {(void*)z, (void*)x, (void*)v, (void*)y, (void*)tt, (void*)lp, (void*)dl, (void*)feat, (void*)nfe,
                  (void*)st, (void*)ws})
    if (q) hipFree(q);
  return true;
}

int main() {
  host_checks();
  const ecnf_cfg cfgs[] = {make_cfg(4, 2, 1, 64, 128, 3, 3, 1.f), make_cfg(13, 3, 1, 64, 128, 3, 3, 1.f),
                           make_cfg(22, 3, 22, 32, 64, 2, 3, 0.2f), make_cfg(29, 3, 1, 32, 256, 4, 5, 2.f)};
  int gpu = 0;
  for (const auto& c : cfgs) {
    if (g_trace) std::fprintf(stderr, "config N = %d, M = %d\n", c.n_nodes, c.mlp_width);
    gpu += device_checks(c, 5) ? 1 : 0;
  }
  {
    size_t lay[16];
    for (int w = 0; w < 4; ++w) CHECK(ecnf_struct_layout(w, lay, 16) > 0, "struct layout %d", w);
    CHECK(ecnf_struct_layout(9, lay, 16) == -1, "bad struct");
  }
  // scoped leak check of every allocation made through the library above (the ROCm runtime's own allocations are
  // suppressed by lsan.supp); run here, while the process is live, instead of at exit (leak_check_at_exit=0)
  const auto t0 = std::chrono::steady_clock::now();
  const int leaked = __lsan_do_recoverable_leak_check();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf("abi_asan: leak check %s in %.0f ms\n", leaked ? "FOUND LEAKS" : "clean", ms);
  if (leaked) ++g_fail;
  std::printf("abi_asan: %s, %d failure(s)\n", gpu ? "host + device paths" : "host paths only (no GPU)", g_fail);
  return g_fail ? 1 : 0;
}
