// Experiment (configs[3] one-batch latency): does a ray's early progress single out
// the batch's longest rays? tools/cpu_same.cpp's loop with probes: at attempts 32..4096 the
// ray's ln t and r, and its first step size and r at the start. Built and run by tools/exp_gr_predict.py; never part of the product.
#include <cmath>
#include <cstdint>

static constexpr int NPROBE = 9;  // attempts 32, 64, ..., 4096; then [dt, r] at attempt 0
static thread_local float* g_probe = nullptr;
static float* g_probe_base = nullptr;

static inline void probe_ray(int64_t i) { g_probe = g_probe_base + i * 2 * NPROBE; }
static inline void probe_hook(int a, double tau, const double* u, double dt) {
  if (a == 0 && std::isnan(g_probe[2 * 8])) {
    g_probe[2 * 8] = (float)dt;
    g_probe[2 * 8 + 1] = (float)u[0];
    return;
  }
  if (a < 32 || (a & (a - 1)) != 0) return;
  const int k = __builtin_ctz((unsigned)a) - 5;
  if (k >= 8 || !std::isnan(g_probe[2 * k])) return;
  g_probe[2 * k] = (float)tau;
  g_probe[2 * k + 1] = (float)u[0];
}
#define CPU_SAME_ATTEMPT_HOOK(attempts, tau, u, dt) probe_hook((attempts), (tau), (u), (dt))
#define CPU_SAME_RAY_HOOK(ray) probe_ray(ray)
#include "cpu_same.cpp"

extern "C" void exp_set_probe(float* base) { g_probe_base = base; }
