// Host-side AddressSanitizer driver of the C ABI (include/sw.h), SURVEY §5
// "race detection / sanitizers": libsw's host runtime (sw_api.cpp) is built
// with -Xarch_host -fsanitize=address (tools/asan_build.sh) and driven through
// every entry point.  Without a GPU it covers the paths that need none
// (defaults, geometry, argument validation, error text, destroy of a failed
// context); with one (`--gpu`) the whole lifecycle: create, state, clock,
// steps, calcN, physical fields, diagnostics, energy records, history, fp32
// buffers, profiling, destroy.  Exit status 0 = clean; ASan aborts otherwise.
#include <sw.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static int fails = 0;
#define EXPECT(cond)                                                      \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #cond); \
      ++fails;                                                            \
    }                                                                     \
  } while (0)

static void no_gpu_paths() {
  sw_config c;
  sw_config_default(&c);
  EXPECT(c.abi_version == SW_ABI_VERSION && c.precision == SW_PREC_F64);
  int32_t geo[8];
  c.nx = c.ny = 2048;
  c.nranks = 4;
  for (int s = 0; s < 4; ++s) EXPECT(sw_slab_geometry(&c, s, geo) == SW_OK && geo[4] == 512);
  EXPECT(sw_slab_geometry(&c, 4, geo) == SW_E_INVALID);
  EXPECT(sw_slab_geometry(nullptr, 0, geo) == SW_E_INVALID);
  c.nranks = 1;
  // invalid configurations fail before any device work, with an error text
  const int bad_nx[] = {16, 96, 16384};
  for (int nx : bad_nx) {
    sw_config b = c;
    b.nx = nx;
    sw_ctx* ctx = nullptr;
    EXPECT(sw_create(&ctx, &b) == SW_E_INVALID);
    EXPECT(ctx != nullptr && std::strlen(sw_last_error(ctx)) > 0);
    sw_destroy(ctx);
  }
  sw_config b = c;
  b.precision = 7;
  sw_ctx* ctx = nullptr;
  EXPECT(sw_create(&ctx, &b) == SW_E_INVALID);
  sw_destroy(ctx);
  b = c;
  b.abi_version = SW_ABI_VERSION - 1;
  EXPECT(sw_create(&ctx, &b) == SW_E_INVALID);
  EXPECT(sw_create(nullptr, &c) == SW_E_INVALID);
  EXPECT(std::strcmp(sw_last_error(nullptr), "null context") == 0);
  int32_t a, d, e;
  EXPECT(sw_get_dims(nullptr, &a, &d, &e) == SW_E_STATE);
  EXPECT(sw_step(nullptr, 1) == SW_E_STATE);
  sw_destroy(nullptr);
}

template <typename T>
static void lifecycle(int model, int stepper, int precision) {
  sw_config c;
  sw_config_default(&c);
  c.model = model;
  c.stepper = stepper;
  c.nx = c.ny = 64;
  c.dt = 1e-3;
  c.precision = precision;
  sw_ctx* ctx = nullptr;
  int rc = sw_create(&ctx, &c);
  if (rc != SW_OK) {
    std::fprintf(stderr, "sw_create: %s (%d)\n", sw_last_error(ctx), rc);
    ++fails;
    sw_destroy(ctx);
    return;
  }
  int32_t nkr, nl, nf;
  EXPECT(sw_get_dims(ctx, &nkr, &nl, &nf) == SW_OK);
  const size_t n = (size_t)nkr * nl * nf;
  std::vector<T> sol(2 * n), out(2 * n), N(2 * n);
  for (size_t i = 0; i < 2 * n; ++i) sol[i] = (T)(std::sin(0.37 * (double)i));  // small: a white-noise state at 1e3 blows up nonlinearly
  EXPECT(sw_set_state(ctx, sol.data(), sol.size() * sizeof(T)) == SW_OK);
  EXPECT(sw_set_state(ctx, sol.data(), sol.size() * sizeof(T) - 1) == SW_E_INVALID);
  EXPECT(sw_set_clock(ctx, 0.0, 0) == SW_OK);
  EXPECT(sw_set_energy_diagnostics(ctx, 2, 4) == SW_OK);
  EXPECT(sw_step(ctx, 10) == SW_OK);
  std::vector<sw_energy_record> rec(8);
  int64_t nrec = 0;
  EXPECT(sw_get_energy_diagnostics(ctx, rec.data(), 8, &nrec) == SW_OK && nrec == 4);
  EXPECT(sw_get_state(ctx, out.data(), out.size() * sizeof(T)) == SW_OK);
  EXPECT(sw_calcN(ctx, out.data(), N.data(), N.size() * sizeof(T)) == SW_OK);
  std::vector<T> phys((size_t)c.nx * c.ny);
  EXPECT(sw_get_physical(ctx, model == SW_MODEL_RSW ? SW_PHYS_ETA : SW_PHYS_PSI, phys.data(),
                         phys.size() * sizeof(T)) == SW_OK);
  double v = 0;
  rc = sw_diag(ctx, SW_DIAG_KE, &v);
  if (rc != SW_OK || !std::isfinite(v))
    std::fprintf(stderr, "sw_diag(KE) = %d (%s), value %g\n", rc, sw_last_error(ctx), v);
  EXPECT(rc == SW_OK && std::isfinite(v));
  EXPECT(sw_diag(ctx, SW_DIAG_CFL, &v) == SW_OK);
  EXPECT(sw_diag(ctx, 99, &v) == SW_E_INVALID);
  int32_t slots = -1;
  EXPECT(sw_history_slots(ctx, &slots) == SW_OK);
  for (int k = 1; k <= slots; ++k) {
    EXPECT(sw_get_history(ctx, k, N.data(), N.size() * sizeof(T)) == SW_OK);
    EXPECT(sw_set_history(ctx, k, N.data(), N.size() * sizeof(T)) == SW_OK);
  }
  EXPECT(sw_get_history(ctx, 3, N.data(), N.size() * sizeof(T)) == SW_E_INVALID);
  EXPECT(sw_reset_history(ctx) == SW_OK);
  sw_kernel_stat st[16];
  int32_t ns = 0;
  EXPECT(sw_profile_steps(ctx, 3, st, 16, &ns) == SW_OK && ns > 0);
  EXPECT(sw_step_alg_bytes(ctx) > 0);
  double t;
  int64_t step;
  EXPECT(sw_get_clock(ctx, &t, &step) == SW_OK && step == 13);
  sw_destroy(ctx);
}

int main(int argc, char** argv) {
  no_gpu_paths();
  if (argc > 1 && std::strcmp(argv[1], "--gpu") == 0) {
    lifecycle<double>(SW_MODEL_RSW, SW_STEP_FILTERED_AB3, SW_PREC_F64);
    lifecycle<float>(SW_MODEL_RSW, SW_STEP_IFMAB3, SW_PREC_F32);
    lifecycle<double>(SW_MODEL_QG2, SW_STEP_IFMRK4, SW_PREC_F64);
  }
  std::printf("abi_asan: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
