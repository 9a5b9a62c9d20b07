// count_flops.cpp -- the "instrumented restatement" that fixes the algorithmic FLOPs of the
// hot path: the product's own templated physics (art_core.h) instantiated with
// an op-counting scalar on the host. Convention: +, -, *, / and sqrt count 1 FLOP each, exp
// 1, sincos 2 (sin and cos), pow 1; comparisons, abs, sign and selects count 0. A fused
// multiply-add emitted by the compiler is 2 FLOPs under this convention, matching the
// MI355X FP64 peak's own accounting (78.6 TFLOP/s counts FMA = 2).
// Usage: count_flops > tools/flops.json
#include <cstdio>

#include "../adiabatic_raytracer_amd/csrc/art_core.h"

namespace art {
struct OC {
  double v;
  static long long n;
  OC() : v(0) {}
  OC(double x) : v(x) {}  // NOLINT
};
long long OC::n = 0;
inline OC operator+(OC a, OC b) { ++OC::n; return OC(a.v + b.v); }
inline OC operator-(OC a, OC b) { ++OC::n; return OC(a.v - b.v); }
inline OC operator*(OC a, OC b) { ++OC::n; return OC(a.v * b.v); }
inline OC operator/(OC a, OC b) { ++OC::n; return OC(a.v / b.v); }
inline OC operator-(OC a) { return OC(-a.v); }
inline OC& operator+=(OC& a, OC b) { return a = a + b; }
inline OC operator+(OC a, double b) { return a + OC(b); }
inline OC operator+(double a, OC b) { return OC(a) + b; }
inline OC operator-(OC a, double b) { return a - OC(b); }
inline OC operator-(double a, OC b) { return OC(a) - b; }
inline OC operator*(OC a, double b) { return a * OC(b); }
inline OC operator*(double a, OC b) { return OC(a) * b; }
inline OC operator/(OC a, double b) { return a / OC(b); }
inline OC operator/(double a, OC b) { return OC(a) / b; }
inline bool operator<(OC a, double b) { return a.v < b; }
inline bool operator<=(OC a, double b) { return a.v <= b; }
inline bool operator>(OC a, double b) { return a.v > b; }
inline bool operator>=(OC a, double b) { return a.v >= b; }
inline bool operator>(OC a, OC b) { return a.v > b.v; }
inline bool operator<(OC a, OC b) { return a.v < b.v; }
inline OC msqrt(OC x) { ++OC::n; return OC(sqrt(x.v)); }
inline OC frcp(OC x) { ++OC::n; return OC(1.0 / x.v); }
inline OC mexp(OC x) { ++OC::n; return OC(exp(x.v)); }
inline OC fexp(OC x) { ++OC::n; return OC(exp(x.v)); }
inline OC mabs(OC x) { return OC(fabs(x.v)); }
inline OC msign(OC x) { return OC(copysign(1.0, x.v)); }
inline void msincos(OC x, OC& s, OC& c) { OC::n += 2; s = OC(sin(x.v)); c = OC(cos(x.v)); }
inline OC msin(OC x) { ++OC::n; return OC(sin(x.v)); }
inline OC mcos(OC x) { ++OC::n; return OC(cos(x.v)); }
inline OC macos(OC x) { ++OC::n; return OC(acos(x.v)); }
inline OC matan2(OC y, OC x) { ++OC::n; return OC(atan2(y.v, x.v)); }
}  // namespace art

using namespace art;

template <class F>
long long count(F f) {
  OC::n = 0;
  f();
  return OC::n;
}

static void emit(bool flat, bool last) {
  art_params p{};
  p.theta_m = 0.2; p.omega_pul = 1.0; p.B0 = 1e14; p.rNS = 10.0; p.mass_ns = 1.0; p.mass_a = 1e-5; p.g_agg = 1e-12;
  p.bndry_lyr = -1.0; p.ln_t_end = 0.0; p.abstol = 1e-6; p.reltol = 1e-7; p.dtmin = 1e-13; p.maxiters = 100000;
  p.flat = flat ? 1 : 0; p.isotropic = 0; p.melrose = 1; p.integrator = 0; p.n_fixed = 1000; p.interp_points = 50;
  KParams K = make_kparams(p);
  // a typical exterior photon state (r > 1.01 rNS: all seven components computed)
  OC u[7] = {OC(20.0), OC(1.1), OC(0.3), OC(0.8), OC(5.0), OC(3.0), OC(-1.00000027e-5)};
  OC du[7], tau(-12.0);
  // the photon RHS the kernels run for this parameter set (rhs dispatches: GJ plasma without a
  // boundary layer -> rhs_photon_gj)
  const long long f_rhs = count([&] { rhs(K, true, u, tau, 1.00000027e-5, du); });
  const long long f_rhs_ax = count([&] { rhs_axion(K, u, tau, 1.00000027e-5, du); });
  const long long f_cond = count([&] { (void)condition(K, u, tau); });
  // a grid point of the scan: condition at t from the geometric recurrence (t *= q: 1 FLOP)
  const long long f_cond_scan = count([&] { (void)condition_t(K, u, OC(2e-5)); }) + 1;
  // cubic Hermite point (art_kernels.hip hermite7): 4 setup + 7 x 10
  OC u1[7], f0[7], f1[7], out[7], h(0.01), th(0.3);
  for (int i = 0; i < 7; ++i) { u1[i] = u[i]; f0[i] = du[i]; f1[i] = du[i]; }
  const long long f_herm = count([&] {
    const OC a = 1.0 - th, b = th * (th - 1.0), c1 = 1.0 - 2.0 * th, c2 = (th - 1.0) * h, c3 = th * h;
    for (int i = 0; i < 7; ++i) out[i] = a * u[i] + th * u1[i] + b * (c1 * (u1[i] - u[i]) + c2 * f0[i] + c3 * f1[i]);
  });
  // Vern6 stage inputs y = u + h Σ a_ij k_j: nonzeros per row 1,2,2,3,4,5,6,6 -> per component 2·nnz + 1
  const int nnz[8] = {1, 2, 2, 3, 4, 5, 6, 6};
  long long f_glue_v6 = 0;
  for (int s = 0; s < 8; ++s) f_glue_v6 += 7LL * (2 * nnz[s] + 1) + 1;  // + stage time tau + c h
  // error norm: 7 terms (7 mul, 6 add) + h* + abstol + max*reltol + /sc + square + acc, then /7 and sqrt
  const long long f_err = 7LL * (7 + 6 + 1 + 2 + 1 + 1 + 1) + 2;
  const long long f_ctrl = 8;  // two pow, /, /gamma, /q, fmax/fmin free, qold
  // RK4: inputs 3 x (7 x 2 + 1) + final 7 x 8 + 1
  const long long f_glue_rk4 = 3LL * (7 * 2 + 1) + 7LL * 8 + 1;
  // per-ray setup: initial_state (k_norm + celerity + transforms) and back transform
  OC x0[3] = {OC(12.0), OC(-5.0), OC(3.0)}, k0[3] = {OC(0.3), OC(0.2), OC(-0.5)}, uu[7], xe[3], ke[3];
  const long long f_init = count([&] { initial_state(K, x0, k0, 1.00000027e-5, -1.0, uu); });
  const long long f_back = count([&] { back_transform(K, u, 1.00000027e-5, xe, ke); });
  OC pos[3] = {OC(15.0), OC(3.0), OC(4.0)}, kp[3] = {OC(1e-6), OC(2e-6), OC(-1e-6)};
  const long long f_prob = count([&] { (void)prob_nonad_single(K, pos, kp, OC(1.00000027e-5)); });
  // scan_certified_code (double only, hand count): 4 Bernstein hulls x 11, the u7 bounds 4,
  // t0 and t1 3, two sincos 4 + ψ 2, b(end) 8, Δθ 2, Δψ 6, |b|max 5, the final test 5, and
  // the two-sided bound on b (two control-polygon variations 2 x 9, ℓ 7, lo/hi 5)
  const long long f_cert = 4 * 11 + 4 + 3 + 6 + 8 + 2 + 6 + 5 + 5 + 18 + 7 + 5;
  std::printf(
      "  \"%s\": {\n    \"rhs_photon\": %lld,\n    \"rhs_axion\": %lld,\n    \"condition\": %lld,\n"
      "    \"condition_scan_point\": %lld,\n    \"hermite_point\": %lld,\n"
      "    \"vern6_stage_glue\": %lld,\n    \"vern6_error_norm\": %lld,\n    \"controller\": %lld,\n"
      "    \"rk4_stage_glue\": %lld,\n    \"initial_state\": %lld,\n    \"back_transform\": %lld,\n"
      "    \"prob_nonad\": %lld,\n    \"scan_certificate\": %lld,\n    \"vern6_attempt\": %lld,\n"
      "    \"rk4_attempt\": %lld\n  }%s\n",
      flat ? "flat" : "gr", f_rhs, f_rhs_ax, f_cond, f_cond_scan, f_herm, f_glue_v6, f_err, f_ctrl, f_glue_rk4,
      f_init, f_back, f_prob, f_cert, 8 * f_rhs + f_glue_v6 + f_err + f_ctrl, 4 * f_rhs + f_glue_rk4, last ? "" : ",");
}

int main() {
  std::printf("{\n  \"convention\": \"+,-,*,/,sqrt,exp,pow = 1 FLOP; sincos = 2; FMA = 2; "
              "abs/sign/compare/select = 0\",\n");
  emit(true, false);
  emit(false, true);
  std::printf("}\n");
  return 0;
}
