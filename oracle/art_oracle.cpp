// ============================================================================
// art_oracle.cpp -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
//
// A CPU restatement of the hot path of SamWitte/Adiabatic_RayTracer (Julia),
// function by function, with every gradient taken by forward-mode dual numbers
// exactly where the reference calls ForwardDiff (RayTracer.jl:21,24,84-88,1427-1432).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
//
// PARITY STATUS: "parity unpinned" in the strict sense -- the reference is Julia
// (not installed here, no network), its integrator/AD live in unvendored, unpinned
// packages (OrdinaryDiffEq, DiffEqBase, ForwardDiff; no Project/Manifest.toml) and
// the reference ships no golden vectors or fixtures. This oracle
// is instead pinned by: the Vern6 tableau's order conditions (tests/test_tableau.py),
// Philox known-answer vectors, finite-difference / complex-step checks of every dual
// gradient, convergence against scipy DOP853 at rtol 1e-13, and closed-form physics
// invariants (tests/test_oracle_*.py).
//
// Integrator semantics restated from the OrdinaryDiffEq/DiffEqBase documentation
// (solve(prob, Vern6(), reltol=1e-7, abstol=1e-6, dtmin=1e-13, force_dtmin=true,
// maxiters=1e5), RayTracer.jl:383-384): Verner 6(5) tableau, RMS error norm over
// abstol + max(|uprev|,|u|)*reltol, PI step-size controller (beta1 = 7/60,
// beta2 = 1/15, gamma = 0.9, qmin = 0.2, qmax = 10, qoldinit = 1e-4), Hairer's
// initial-dt heuristic (ode_determine_initdt), ContinuousCallback sign scan at
// interp_points equally spaced points per step (RayTracer.jl:357-358). Documented
// deviation (unknowable without the package source): the dense output used for the
// sign scan is the cubic Hermite interpolant, and the root is then located on the
// TRUE trajectory by re-stepping from the step start (Illinois iteration).
// ============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/art.h"
#include "dual.h"

namespace oracle {

// Constants.jl:3-5
constexpr double c_km = 2.99792e5;
constexpr double hbar = 6.582119e-16;
constexpr double GNew = 132712000000.0;
constexpr double PI = 3.141592653589793;

using D1 = Dual<1>;
using D3 = Dual<3>;

// ---------------------------------------------------------------------------
// g_schwartz -- RayTracer.jl:455-501. Upper metric g^μν, signature (-,+,+,+).
// The interior switch uses the keyword default rNS = 10.0 (:455), which the hot-path
// callers never override.
template <class T>
struct Metric { T gtt, grr, gthth, gpp; };

template <class T>
Metric<T> g_schwartz(const T& r, const T& theta, double Mass_NS) {
  const double rNS_kw = 10.0;
  T rs = T(2 * GNew * Mass_NS / (c_km * c_km));
  const bool inside = val(r) <= rNS_kw;
  if (inside) rs = rs * cube(r / rNS_kw);  // :463
  T st = sin(theta);
  Metric<T> g;
  g.gtt = -1.0 / (1.0 - rs / r);
  g.grr = 1.0 - rs / r;
  g.gthth = 1.0 / sq(r);
  g.gpp = 1.0 / (sq(r) * sq(st));
  if (inside) {  // :496-497
    g.gtt = -4.0 / sq(3.0 * sqrt(1.0 - rs / rNS_kw) - sqrt(1.0 - sq(r) * rs / cube(rNS_kw)));
    g.grr = 1.0 - sq(r) * rs / cube(rNS_kw);
  }
  return g;
}

// ---------------------------------------------------------------------------
// Rotating oblique dipole, RayTracer.jl:1142-1151 / 1287-1292.
template <class T>
struct Dipole { T Br, Bth, Bph; };

template <class T>
Dipole<T> dipole(const T& r, const T& th, const T& ph, const T& t, const art_params& P) {
  T psi = ph - P.omega_pul * t;
  T Bnorm = P.B0 * cube(P.rNS / r) / 2.0;
  Dipole<T> B;
  B.Br = 2.0 * Bnorm * (std::cos(P.theta_m) * cos(th) + std::sin(P.theta_m) * sin(th) * cos(psi));
  B.Bth = Bnorm * (std::cos(P.theta_m) * sin(th) - std::sin(P.theta_m) * cos(th) * cos(psi));
  B.Bph = Bnorm * std::sin(P.theta_m) * sin(psi);
  return B;
}

inline double pole_omega_p(const art_params& P) {  // :1156-1157
  double nelec_pole = std::abs((2.0 * P.omega_pul * P.B0) / std::sqrt(4 * PI / 137) * (1.95e-2) * hbar);
  return std::sqrt(4 * PI * nelec_pole / 137 / 5.0e5);
}

// GJ plasma frequency from the dipole's Bz (shared by the vecSPH/vec/scalar forms).
template <class T>
T gj_omega_p_core(const T& r, const T& th, const T& ph, const T& t, const art_params& P) {
  Dipole<T> B = dipole(r, th, ph, t, P);
  T Bz = B.Br * cos(th) - B.Bth * sin(th);
  T nelec = abs((2.0 * P.omega_pul * Bz) / std::sqrt(4 * PI / 137) * 1.95e-2 * hbar);  // eV^3
  return sqrt(4 * PI * nelec / 137 / 5.0e5);
}

template <class T>
T add_boundary_layer(T wp, const T& r, const art_params& P, double bndry_lyr, double Mass_a) {
  // RayTracer.jl:1155-1162 (applied where r >= rNS)
  if (bndry_lyr > 0 && val(r) >= P.rNS) {
    double pole_val = pole_omega_p(P);
    double rmax = P.rNS * std::pow(pole_val / Mass_a, 2.0 / 3.0);
    wp = wp + pole_val * pow(P.rNS / r, 3.0 / 2.0) * exp(-(r - rmax * bndry_lyr) / (0.1 * rmax));
  }
  return wp;
}

// GJ_Model_ωp_vecSPH -- RayTracer.jl:1120-1170 (spherical input)
template <class T>
T GJ_wp_vecSPH(const T& r, const T& th, const T& ph, const T& t, const art_params& P,
               bool zeroIn, double bndry_lyr, double Mass_a) {
  T wp = gj_omega_p_core(r, th, ph, t, P);
  wp = add_boundary_layer(wp, r, P, bndry_lyr, Mass_a);
  if (zeroIn && val(r) <= P.rNS) wp = T(0.0);  // :1165-1167
  return wp;
}

// GJ_Model_ωp_vec -- RayTracer.jl:1066-1103 (Cartesian input, no zeroIn)
inline double GJ_wp_vec(const double x[3], double t, const art_params& P, double bndry_lyr, double Mass_a) {
  double r = std::sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
  double ph = std::atan2(x[1], x[0]);
  double th = std::acos(x[2] / r);
  double wp = gj_omega_p_core(r, th, ph, t, P);
  return add_boundary_layer(wp, r, P, bndry_lyr, Mass_a);
}

// GJ_Model_ωp_scalar -- RayTracer.jl:1172-1209, as called by Find_Conversion_Surface
inline double GJ_wp_scalar(const double x[3], double t, const art_params& P) {
  double r = std::sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
  double ph = std::atan2(x[1], x[0]);
  double th = std::acos(x[2] / r);
  return gj_omega_p_core(r, th, ph, t, P);
}

// GJ_Model_Sphereical -- RayTracer.jl:1268-1309, sphericalX=true, return_comp=-1:
// covariant (Br/sqrt(g^rr), Bθ/sqrt(g^θθ), Bφ/sqrt(g^φφ)).
template <class T>
void GJ_Sphereical(const T& r, const T& th, const T& ph, const T& t, const art_params& P,
                   double Mass_NS, bool flat, T out[3]) {
  if (flat) Mass_NS = 0.0;
  Dipole<T> B = dipole(r, th, ph, t, P);
  Metric<T> g = g_schwartz(r, th, Mass_NS);
  out[0] = B.Br / sqrt(g.grr);
  out[1] = B.Bth / sqrt(g.gthth);
  out[2] = B.Bph / sqrt(g.gpp);
}

// return_comp = 0..3 (RayTracer.jl:1300-1307)
template <class T>
T GJ_Sphereical_comp(const T& r, const T& th, const T& ph, const T& t, const art_params& P,
                     double Mass_NS, bool flat, int comp) {
  if (flat) Mass_NS = 0.0;
  Dipole<T> B = dipole(r, th, ph, t, P);
  Metric<T> g = g_schwartz(r, th, Mass_NS);
  if (comp == 0) return sqrt(sq(B.Br) + sq(B.Bth) + sq(B.Bph)) * 1.95e-2;
  if (comp == 1) return B.Br / sqrt(g.grr) * g.grr * 1.95e-2;
  if (comp == 2) return B.Bth / sqrt(g.gthth) * g.gthth * 1.95e-2;
  return B.Bph / sqrt(g.gpp) * g.gpp * 1.95e-2;
}

// K_par -- RayTracer.jl:1044-1058 (flat keyword default false)
template <class T>
T K_par(const T& r, const T& th, const T& ph, const T& k1, const T& k2, const T& k3,
        const T& t_start, const art_params& P, double Mass_NS) {
  T Bs[3];
  GJ_Sphereical(r, th, ph, t_start, P, Mass_NS, false, Bs);
  Metric<T> g = g_schwartz(r, th, Mass_NS);
  T Bmag = sqrt(g.grr * sq(Bs[0]) + g.gthth * sq(Bs[1]) + g.gpp * sq(Bs[2]));
  return (g.grr * k1 * Bs[0] + g.gthth * k2 * Bs[1] + g.gpp * k3 * Bs[2]) / Bmag;
}

// hamiltonian -- RayTracer.jl:530-556 (melrose = true branch). The in-place clamp
// x[:,1] < rNS -> rNS (:531) replaces r by a CONSTANT (zero partials), as ForwardDiff does.
template <class T>
T hamiltonian(T r, const T& th, const T& ph, const T& k1, const T& k2, const T& k3,
              const T& time0, const T& erg, const art_params& P, double Mass_NS,
              bool iso, double bndry_lyr) {
  if (val(r) < P.rNS) r = T(P.rNS);
  T omP = GJ_wp_vecSPH(r, th, ph, time0, P, false, bndry_lyr, P.mass_a);
  Metric<T> g = g_schwartz(r, th, Mass_NS);
  T ksqr = g.gtt * sq(erg) + g.grr * sq(k1) + g.gthth * sq(k2) + g.gpp * sq(k3);
  if (iso) return 0.5 * (ksqr + sq(omP));
  T kpar = K_par(r, th, ph, k1, k2, k3, time0, P, Mass_NS);
  return 0.5 * (ksqr + sq(omP) * (sq(erg) / g.grr - sq(kpar)) / (sq(erg) / g.grr));
}

// hamiltonian_axion -- RayTracer.jl:632-640 (no clamp)
template <class T>
T hamiltonian_axion(const T& r, const T& th, const T& k1, const T& k2, const T& k3, const T& erg,
                    double Mass_NS) {
  Metric<T> g = g_schwartz(r, th, Mass_NS);
  T ksqr = g.gtt * sq(erg) + g.grr * sq(k1) + g.gthth * sq(k2) + g.gpp * sq(k3);
  return 0.5 * ksqr;
}

// ---------------------------------------------------------------------------
// func! -- RayTracer.jl:71-91. Returns du; `u` is mutated like the reference's view:
// the ∂k call's hamiltonian(view(u,:,1:3), ...) clamps u[1] in place (:85, :531).
void rhs_photon(const art_params& P, double u[7], double lnt, double erg, double du[7]) {
  const double t = std::exp(lnt);
  const double Mass_NS = P.flat ? 0.0 : P.mass_ns;
  const double time = 0.0 + t;  // time0 = zeros(batchsize) (MainRunner.jl:177)
  Metric<double> gu = g_schwartz(u[0], u[1], Mass_NS);
  const double E = -u[6];
  const bool iso = P.isotropic != 0;
  {  // :84  -grad_x H . c t g_rr / E / erg   (bndry_lyr not passed -> -1)
    D3 r = D3::seed(u[0], 0), th = D3::seed(u[1], 1), ph = D3::seed(u[2], 2);
    D3 H = hamiltonian<D3>(r, th, ph, D3(u[3] * erg), D3(u[4] * erg), D3(u[5] * erg), D3(time), D3(E), P,
                           Mass_NS, iso, -1.0);
    for (int i = 0; i < 3; ++i) du[3 + i] = -H.d[i] * c_km * t * (gu.grr / E) / erg;
  }
  {  // :85  grad_k H . c t g_rr / E ; clamps u[1] in place
    if (u[0] < P.rNS) u[0] = P.rNS;
    D3 k1 = D3::seed(u[3] * erg, 0), k2 = D3::seed(u[4] * erg, 1), k3 = D3::seed(u[5] * erg, 2);
    D3 H = hamiltonian<D3>(D3(u[0]), D3(u[1]), D3(u[2]), k1, k2, k3, D3(time), D3(E), P, Mass_NS, iso, -1.0);
    for (int i = 0; i < 3; ++i) du[i] = H.d[i] * c_km * t * (gu.grr / E);
  }
  if (u[0] <= P.rNS * 1.01) for (int i = 0; i < 7; ++i) du[i] = 0.0;  // :86
  {  // :88  dH/dt . t g_rr / E  (with bndry_lyr)
    D1 T = D1::seed(time, 0);
    D1 H = hamiltonian<D1>(D1(u[0]), D1(u[1]), D1(u[2]), D1(u[3] * erg), D1(u[4] * erg), D1(u[5] * erg), T,
                           D1(E), P, Mass_NS, iso, P.bndry_lyr);
    du[6] = H.d[0] * t * (gu.grr / E);
  }
}

// func_axion! -- RayTracer.jl:95-123
void rhs_axion(const art_params& P, const double u[7], double lnt, double erg, double du[7]) {
  const double t = std::exp(lnt);
  const double Mass_NS = P.flat ? 0.0 : P.mass_ns;
  Metric<double> gu = g_schwartz(u[0], u[1], Mass_NS);
  {
    D3 r = D3::seed(u[0], 0), th = D3::seed(u[1], 1);
    D3 H = hamiltonian_axion<D3>(r, th, D3(u[3] * erg), D3(u[4] * erg), D3(u[5] * erg), D3(erg), Mass_NS);
    for (int i = 0; i < 3; ++i) du[3 + i] = -H.d[i] * c_km * t * (gu.grr / erg) / erg;
  }
  {
    D3 k1 = D3::seed(u[3] * erg, 0), k2 = D3::seed(u[4] * erg, 1), k3 = D3::seed(u[5] * erg, 2);
    D3 H = hamiltonian_axion<D3>(D3(u[0]), D3(u[1]), k1, k2, k3, D3(erg), Mass_NS);
    for (int i = 0; i < 3; ++i) du[i] = H.d[i] * c_km * t * (gu.grr / erg);
  }
  du[6] = 0.0;
}

// Resonance condition -- RayTracer.jl:254-298 (thick_surface = true branch)
double condition(const art_params& P, const double u[7], double lnt) {
  const double Mass_NS = P.flat ? 0.0 : P.mass_ns;
  const double erg_inf = u[6];
  const double t0 = std::exp(lnt);
  Metric<double> g = g_schwartz(u[0], u[1], Mass_NS);
  double w[3] = {u[3], u[4], u[5]};
  double NrmSq = (-sq(erg_inf) * g.gtt - sq(P.mass_a)) / (sq(w[0]) * g.grr + sq(w[1]) * g.gthth + sq(w[2]) * g.gpp);
  double s = std::sqrt(NrmSq);
  for (double& wi : w) wi *= s;
  double omP = GJ_wp_vecSPH(u[0], u[1], u[2], t0, P, true, P.bndry_lyr, P.mass_a);
  double kpar = P.isotropic ? 0.0 : K_par(u[0], u[1], u[2], w[0], w[1], w[2], t0, P, Mass_NS);
  double ksqr = g.gtt * sq(erg_inf) + g.grr * sq(w[0]) + g.gthth * sq(w[1]) + g.gpp * sq(w[2]);
  return 0.5 * (ksqr + sq(omP) * (sq(erg_inf) / g.grr - sq(kpar)) / (sq(erg_inf) / g.grr)) / sq(erg_inf);
}

// Cartesian -> covariant "celerity" components used by k_norm_Cart (:656-664),
// propagate (:193-212), k_sphere (:995-1007) and the sampler condition (:1557-1564).
struct Sph { double r, th, ph; };
inline Sph cart_to_sph(const double x[3]) {
  Sph s;
  s.r = std::sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
  s.th = std::acos(x[2] / s.r);
  s.ph = std::atan2(x[1], x[0]);
  return s;
}
inline void celerity(const double x[3], const double k[3], const Sph& s, double AA, double w[3]) {
  double dr_dt = (x[0] * k[0] + x[1] * k[1] + x[2] * k[2]) / s.r;
  double st = std::sin(s.th);
  double v0[3] = {dr_dt, (x[2] * dr_dt - s.r * k[2]) / (s.r * st), (-x[1] * k[0] + x[0] * k[1]) / (s.r * st)};
  w[0] = v0[0] / std::sqrt(AA) / AA;
  w[1] = v0[1] / s.r * sq(s.r) / AA;
  w[2] = v0[2] / (s.r * st) * sq(s.r * st) / AA;
}

// k_norm_Cart with ax_fix=true or is_photon=false -- RayTracer.jl:643-685
void k_norm_cart_axion_shell(const double x0[3], const double khat[3], double erg, const art_params& P,
                             double Mass_NS, double out[3]) {
  Sph s = cart_to_sph(x0);
  double r_s0 = 2.0 * Mass_NS * GNew / (c_km * c_km);
  double w0[3];
  celerity(x0, khat, s, 1.0 - r_s0 / s.r, w0);
  Metric<double> g = g_schwartz(s.r, s.th, Mass_NS);
  double NrmSq = (-sq(erg) * g.gtt - sq(P.mass_a)) / (sq(w0[0]) * g.grr + sq(w0[1]) * g.gthth + sq(w0[2]) * g.gpp);
  double f = std::sqrt(NrmSq);
  for (int i = 0; i < 3; ++i) out[i] = f * khat[i];
}

// propagate initial state -- RayTracer.jl:171-216
void initial_state(const art_params& P, const double x0[3], const double k0[3], double erg, double dw,
                   double u0[7]) {
  double kn[3];
  k_norm_cart_axion_shell(x0, k0, erg, P, P.mass_ns, kn);  // GR mass even when flat (:181-185)
  const double Mass_NS = P.flat ? 0.0 : P.mass_ns;         // :187-189
  double r_s0 = 2.0 * Mass_NS * GNew / (c_km * c_km);
  Sph s = cart_to_sph(x0);
  double w0[3];
  celerity(x0, kn, s, 1.0 - r_s0 / s.r, w0);
  u0[0] = s.r; u0[1] = s.th; u0[2] = s.ph;
  for (int i = 0; i < 3; ++i) u0[3 + i] = w0[i] * (1.0 / erg);
  u0[6] = erg * dw;
}

// Final Cartesian x, k -- RayTracer.jl:393-416 (per saved point; interior Mass scaling :398-406)
void back_transform(const art_params& P, const double u[7], double erg, double x[3], double k[3]) {
  double Mass = P.flat ? 0.0 : P.mass_ns;
  if (u[0] < P.rNS) Mass *= cube(u[0]) / cube(P.rNS);
  double r_s = 2.0 * Mass * GNew / (c_km * c_km);
  double om = 1.0 - r_s / u[0];
  double st = std::sin(u[1]), ct = std::cos(u[1]), sp = std::sin(u[2]), cp = std::cos(u[2]);
  double kr = u[3] * erg, kt = u[4] * erg, kp = u[5] * erg;
  double v[3] = {kr * std::sqrt(om) * om, kt / u[0] * om, kp / (u[0] * st) * om};
  x[0] = u[0] * st * cp; x[1] = u[0] * st * sp; x[2] = u[0] * ct;
  k[0] = cp * (st * v[0] + ct * v[1]) - st * sp * v[2] / st;
  k[1] = sp * (st * v[0] + ct * v[1]) + st * cp * v[2] / st;
  k[2] = ct * v[0] - st * v[1];
}

// ---------------------------------------------------------------------------
// get_Prob_nonAD -- MainRunner.jl:67-124 with conversion_prob RayTracer.jl:1405-1473,
// k_sphere :983-1009, spatial_dot :973-981, Cristoffel :503-527, for ONE call with Nc
// crossings. Julia's Nc x 3 matrices are column-major; the reference's linear indexing
// ksphere[1..3], Bsphere[1..3], x0_pl[1..2] (:1432-1443, :510-511) is reproduced via lin().
void get_prob_nonad(const art_params& P, int Nc, const double* pos, const double* kpos,
                    const double* erg_inf, double* out) {
  const double Mass_NS = P.mass_ns;  // global Mass_NS (Gen_Samples.jl:144; MainRunner.jl:75)
  const bool flat = P.flat != 0, iso = P.isotropic != 0;
  std::vector<double> x0pl(3 * Nc), Bs(3 * Nc), ks(3 * Nc), grr(Nc), gthth(Nc), gpp(Nc);
  std::vector<double> Bmag(Nc), kmag(Nc), cth(Nc), sth(Nc), ergax(Nc), wp(Nc);
  auto lin = [&](const std::vector<double>& m, int idx) { return m[idx]; };  // column-major storage
  for (int i = 0; i < Nc; ++i) {
    double x[3] = {pos[i], pos[Nc + i], pos[2 * Nc + i]};
    double k[3] = {kpos[i], kpos[Nc + i], kpos[2 * Nc + i]};
    Sph s = cart_to_sph(x);
    x0pl[i] = s.r; x0pl[Nc + i] = s.th; x0pl[2 * Nc + i] = s.ph;
    Metric<double> g = g_schwartz(s.r, s.th, Mass_NS);
    grr[i] = g.grr; gthth[i] = g.gthth; gpp[i] = g.gpp;
    double B[3];
    GJ_Sphereical(s.r, s.th, s.ph, 0.0, P, Mass_NS, flat, B);  // sphericalX=false recomputes the same r,θ,φ
    for (int c = 0; c < 3; ++c) Bs[c * Nc + i] = B[c];
    double Mk = flat ? 0.0 : Mass_NS;  // k_sphere :987-989
    double r_s0 = 2.0 * Mk * GNew / (c_km * c_km);
    double w[3];
    celerity(x, k, s, 1.0 - r_s0 / s.r, w);
    for (int c = 0; c < 3; ++c) ks[c * Nc + i] = w[c];
    auto sd = [&](const double* a, const double* b) { return g.grr * a[0] * b[0] + g.gthth * a[1] * b[1] + g.gpp * a[2] * b[2]; };
    Bmag[i] = std::sqrt(sd(B, B)) * 1.95e-2;
    kmag[i] = std::sqrt(sd(w, w));
    cth[i] = sd(B, w) * 1.95e-2 / (kmag[i] * Bmag[i]);
    sth[i] = std::sin(std::acos(cth[i]));
    if (iso) { cth[i] *= 0.0; sth[i] /= sth[i]; }
    ergax[i] = erg_inf[i] / std::sqrt(1.0 - 2 * GNew * Mass_NS / s.r / (c_km * c_km));
    wp[i] = GJ_wp_vecSPH(s.r, s.th, s.ph, 0.0, P, true, P.bndry_lyr, 1e-5);  // Mass_a default (:97)
  }
  // Cristoffel(x0_pl, ...) reads r = x0_pl[1], theta = x0_pl[2] (linear indices, :510-511)
  const double r_c = lin(x0pl, 0), th_c = lin(x0pl, 1);
  const double GM = GNew * Mass_NS / (c_km * c_km);  // uses Mass_NS even when flat (:512)
  const double G_rrr = -GM / (r_c * (r_c - 2 * GM)), G_rtt = -(r_c - 2 * GM);
  const double G_rpp = -(r_c - 2 * GM) * sq(std::sin(th_c)), G_trt = 1.0 / r_c;
  const double G_tpp = -std::sin(th_c) * std::cos(th_c), G_prp = 1.0 / r_c;
  const double G_ptp = std::cos(th_c) / std::sin(th_c), G_ttr = 1.0 / r_c, G_ppr = 1.0 / r_c;
  const double G_ppt = std::cos(th_c) / std::sin(th_c);
  const double k1 = lin(ks, 0), k2 = lin(ks, 1), k3 = lin(ks, 2);
  const double B1 = lin(Bs, 0), B2 = lin(Bs, 1), B3 = lin(Bs, 2);
  for (int i = 0; i < Nc; ++i) {
    const double wE = ergax[i];
    const double vloc = std::sqrt(sq(wE) - sq(P.mass_a)) / wE;  // :1410
    double dmu_E[3];
    if (iso) {
      // isotropic branch (:1421-1422): grad_x omega_function(seed(x0_pl), ..., kmag=kmag) =
      // grad sqrt(kmag^2 + ωp^2), omega_function clamping r < rNS (:560) and using its defaults
      // zeroIn=false, bndry_lyr=-1 (:1421 passes neither).
      D3 r = D3::seed(x0pl[i], 0), th = D3::seed(x0pl[Nc + i], 1), ph = D3::seed(x0pl[2 * Nc + i], 2);
      if (r.v < P.rNS) r = D3(P.rNS);
      D3 omP = GJ_wp_vecSPH<D3>(r, th, ph, D3(0.0), P, false, -1.0, P.mass_a);
      D3 om = sqrt(D3(sq(kmag[i])) + sq(omP));
      for (int c = 0; c < 3; ++c) dmu_E[c] = om.d[c];
    } else {
      D3 r = D3::seed(x0pl[i], 0), th = D3::seed(x0pl[Nc + i], 1), ph = D3::seed(x0pl[2 * Nc + i], 2);
      D3 dwp = GJ_wp_vecSPH<D3>(r, th, ph, D3(0.0), P, true, P.bndry_lyr, P.mass_a);     // :1427
      D3 dB = GJ_Sphereical_comp<D3>(r, th, ph, D3(0.0), P, Mass_NS, flat, 0);            // :1429
      D3 c1 = GJ_Sphereical_comp<D3>(r, th, ph, D3(0.0), P, Mass_NS, flat, 1);            // :1432
      D3 c2 = GJ_Sphereical_comp<D3>(r, th, ph, D3(0.0), P, Mass_NS, flat, 2);
      D3 c3 = GJ_Sphereical_comp<D3>(r, th, ph, D3(0.0), P, Mass_NS, flat, 3);
      double term1[3], term2[3];
      for (int c = 0; c < 3; ++c) term1[c] = k1 * c1.d[c] + k2 * c2.d[c] + k3 * c3.d[c];
      term2[0] = k1 * (grr[i] * B1 * 1.95e-2) * G_rrr + k2 * G_trt * (B2 * gthth[i] * 1.95e-2) +
                 k3 * G_prp * (B3 * gpp[i] * 1.95e-2);
      term2[1] = k1 * (gthth[i] * B2 * 1.95e-2) * G_rtt + k3 * G_ptp * (B3 * gpp[i] * 1.95e-2) +
                 k2 * (grr[i] * B1 * 1.95e-2) * G_ttr;
      term2[2] = k1 * (gpp[i] * B3 * 1.95e-2) * G_rpp + k2 * G_tpp * (B3 * gpp[i] * 1.95e-2) +
                 k3 * G_ppr * (B1 * grr[i] * 1.95e-2) + k3 * G_ppt * (B2 * gthth[i] * 1.95e-2);
      double dmu_ct[3];
      for (int c = 0; c < 3; ++c)
        dmu_ct[c] = (term1[c] + term2[c]) / (kmag[i] * Bmag[i]) - cth[i] * dB.d[c] / Bmag[i];  // :1438
      const double w = wp[i];
      double preF = w / std::abs(std::pow(wE, 5) + sq(cth[i]) * wE * (std::pow(w, 4) - 2 * sq(w) * sq(wE)));
      for (int c = 0; c < 3; ++c)
        dmu_E[c] = preF * (std::pow(wE, 4) * sq(sth[i]) * dwp.d[c] -
                           sq(wE) * cth[i] * w * (sq(wE) - sq(w)) * dmu_ct[c]);  // :1449
    }
    const double kh[3] = {ks[i] / kmag[i], ks[Nc + i] / kmag[i], ks[2 * Nc + i] / kmag[i]};
    const double vhat_gradE = grr[i] * kh[0] * dmu_E[0] + gthth[i] * kh[1] * dmu_E[1] + gpp[i] * kh[2] * dmu_E[2];
    const double w = wp[i];
    const double prefactor = std::pow(wE, 4) * sq(sth[i]) / (sq(cth[i]) * sq(w) * (sq(w) - 2 * sq(wE)) + std::pow(wE, 4));
    out[i] = PI / 2.0 * prefactor * sq(P.g_agg * 1e-9 * Bmag[i]) / (std::abs(vhat_gradE) * vloc * c_km * hbar);  // :1467-1468
  }
}

// ---------------------------------------------------------------------------
// Vern6 tableau (OrdinaryDiffEq "Vern6", Verner's most efficient 6(5) pair, FSAL:
// b == A[8,:]). Checked against all 37 sixth-order and 17 fifth-order conditions in
// tests/test_tableau.py.
struct Vern6 {
  static constexpr double c[9] = {0.0, 0.06, 0.09593333333333333, 0.1439, 0.4973, 0.9725, 0.9995, 1.0, 1.0};
  double A[9][9];
  double b[9], bhat[9];
  Vern6() {
    std::memset(A, 0, sizeof(A));
    A[1][0] = 0.06;
    A[2][0] = 0.019239962962962962; A[2][1] = 0.07669337037037037;
    A[3][0] = 0.035975; A[3][2] = 0.107925;
    A[4][0] = 1.3186834152331484; A[4][2] = -5.042058063628562; A[4][3] = 4.220674648395414;
    A[5][0] = -41.872591664327516; A[5][2] = 159.4325621631375; A[5][3] = -122.11921356501003; A[5][4] = 5.531743066200053;
    A[6][0] = -54.430156935316504; A[6][2] = 207.06725136501848; A[6][3] = -158.61081378459; A[6][4] = 6.991816585950242;
    A[6][5] = -0.018597231062309313;
    A[7][0] = -54.66374178728198; A[7][2] = 207.95280625538937; A[7][3] = -159.2889574744995; A[7][4] = 7.018743740796944;
    A[7][5] = -0.018338785905045722; A[7][6] = -0.0005119484997882099;
    A[8][0] = 0.03438957868357036; A[8][3] = 0.2582624555633503; A[8][4] = 0.4209371189673537;
    A[8][5] = 4.40539646966931; A[8][6] = -176.48311902429865; A[8][7] = 172.36413340141507;
    for (int j = 0; j < 9; ++j) b[j] = A[8][j];
    const double bh[9] = {0.04909967648382489, 0, 0, 0.2251112229516524, 0.4694682253029562, 0.8065792249988868, 0.0,
                          -0.6071194891777959, 0.05686113944047569};
    for (int j = 0; j < 9; ++j) bhat[j] = bh[j];
  }
};
constexpr double Vern6::c[9];
static const Vern6 V6;

// ---------------------------------------------------------------------------
// One segment: propagate's solve(...) with callbacks (RayTracer.jl:251-391).
struct Crossing { double pos[3], k[3], t, dw, p; };

class Segment {
 public:
  Segment(const art_params& P, int species, double erg, const double x0[3], int max_crossings)
      : P(P), photon(species == ART_PHOTON), erg(erg), max_crossings(max_crossings) {
    for (int i = 0; i < 3; ++i) x0c[i] = x0[i];
  }

  void f(double u[7], double tau, double du[7]) {
    if (photon) rhs_photon(P, u, tau, erg, du); else rhs_axion(P, u, tau, erg, du);
  }
  double cond(const double u[7], double tau) const { return condition(P, u, tau); }

  // one Vern6 attempt from (u, k1=f(u)) with step h; writes unew, k9, EEst
  double vern6_step(const double u[7], const double k1[7], double tau, double h, double unew[7], double k9[7]) {
    double k[9][7], tmp[7];
    std::memcpy(k[0], k1, sizeof(double) * 7);
    for (int s = 1; s < 9; ++s) {
      for (int i = 0; i < 7; ++i) {
        double acc = 0.0;
        for (int j = 0; j < s; ++j) acc += V6.A[s][j] * k[j][i];
        tmp[i] = u[i] + h * acc;
      }
      f(tmp, tau + Vern6::c[s] * h, k[s]);  // stage 9 at u_{n+1}: FSAL; f may clamp tmp[0] (quirk 1)
    }
    std::memcpy(unew, tmp, sizeof(double) * 7);
    std::memcpy(k9, k[8], sizeof(double) * 7);
    double acc2 = 0.0;
    for (int i = 0; i < 7; ++i) {
      double e = 0.0;
      for (int j = 0; j < 9; ++j) e += (V6.b[j] - V6.bhat[j]) * k[j][i];
      e *= h;
      double sc = P.abstol + std::max(std::abs(u[i]), std::abs(unew[i])) * P.reltol;
      acc2 += sq(e / sc);
    }
    return std::sqrt(acc2 / 7.0);
  }

  void rk4_step(const double u[7], const double k1[7], double tau, double h, double unew[7], double fnew[7]) {
    double k2[7], k3[7], k4[7], tmp[7];
    for (int i = 0; i < 7; ++i) tmp[i] = u[i] + 0.5 * h * k1[i];
    f(tmp, tau + 0.5 * h, k2);
    for (int i = 0; i < 7; ++i) tmp[i] = u[i] + 0.5 * h * k2[i];
    f(tmp, tau + 0.5 * h, k3);
    for (int i = 0; i < 7; ++i) tmp[i] = u[i] + h * k3[i];
    f(tmp, tau + h, k4);
    for (int i = 0; i < 7; ++i) unew[i] = u[i] + h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
    f(unew, tau + h, fnew);  // next step's k1 (may clamp unew[0])
  }

  double step(const double u[7], const double k1[7], double tau, double h, double unew[7], double fnew[7]) {
    if (P.integrator == ART_RK4) { rk4_step(u, k1, tau, h, unew, fnew); return 0.0; }
    return vern6_step(u, k1, tau, h, unew, fnew);
  }

  static double rms7(const double* a) {
    double s = 0.0;
    for (int i = 0; i < 7; ++i) s += a[i] * a[i];
    return std::sqrt(s / 7.0);
  }

  // ode_determine_initdt (DiffEqBase), order 6
  double initdt(double u0[7], const double f0[7], double tau0, double dtmax) {
    double sk[7], tmp[7];
    for (int i = 0; i < 7; ++i) sk[i] = P.abstol + std::abs(u0[i]) * P.reltol;
    for (int i = 0; i < 7; ++i) tmp[i] = u0[i] / sk[i];
    double d0 = rms7(tmp);
    for (int i = 0; i < 7; ++i) tmp[i] = f0[i] / sk[i];
    double d1 = rms7(tmp);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * (d0 / d1);
    dt0 = std::min(dt0, dtmax);
    double eps_t = std::nextafter(std::abs(tau0), INFINITY) - std::abs(tau0);
    if (dt0 < 10 * eps_t) return std::max(1e-6, P.dtmin);
    double u1[7], f1[7];
    for (int i = 0; i < 7; ++i) u1[i] = u0[i] + dt0 * f0[i];
    f(u1, tau0 + dt0, f1);
    bool same = true;
    for (int i = 0; i < 7; ++i) same = same && (f0[i] == f1[i]);
    if (same) return std::max(P.dtmin, 100 * dt0);
    for (int i = 0; i < 7; ++i) tmp[i] = (f1[i] - f0[i]) / sk[i];
    double d2 = rms7(tmp) / dt0;
    double mx = std::max(d1, d2);
    double dt1 = (mx <= 1e-15) ? std::max(1e-6, dt0 * 1e-3) : std::pow(10.0, -(2.0 + std::log10(mx)) / 6.0);
    return std::max(P.dtmin, std::min(std::min(100 * dt0, dt1), dtmax));
  }

  static void hermite(const double u0[7], const double f0[7], const double u1[7], const double f1[7], double h,
                      double th, double out[7]) {
    for (int i = 0; i < 7; ++i)
      out[i] = (1 - th) * u0[i] + th * u1[i] +
               th * (th - 1) * ((1 - 2 * th) * (u1[i] - u0[i]) + (th - 1) * h * f0[i] + th * h * f1[i]);
  }
  static int sgn(double x) { return (x > 0) - (x < 0); }

  // Root of the condition along the cubic Hermite interpolant in [tha, thb] (Illinois).
  double illinois_interp(const double u0[7], const double f0[7], const double u1[7], const double f1[7], double tau,
                         double h, double tha, double thb, double ca, double cb) const {
    double tr = tha - ca * (thb - tha) / (cb - ca);
    int side = 0;
    for (int it = 0; it < 40; ++it) {
      double ui[7];
      hermite(u0, f0, u1, f1, h, tr, ui);
      double cr = cond(ui, tau + tr * h);
      if (cr == 0.0 || std::isnan(cr) || (thb - tha) < 1e-12) break;
      if (sgn(cr) == sgn(ca)) { tha = tr; ca = cr; if (side == -1) cb *= 0.5; side = -1; }
      else { thb = tr; cb = cr; if (side == 1) ca *= 0.5; side = 1; }
      double tn = tha - ca * (thb - tha) / (cb - ca);
      if (tn == tr) break;
      tr = tn;
    }
    return tr;
  }

  // Bracketed root polish on the true trajectory (same algorithm as the kernel's ROOT mode).
  struct RootBracket {
    double tha, ca, thb, cb, t, slope;
    int side = 0, rit = 0;
    RootBracket(double a, double fa, double b, double fb, double t_int)
        : tha(a), ca(fa), thb(b), cb(fb), t(t_int), slope((fb - fa) / (b - a)) {
      if (!(t > tha && t < thb)) t = 0.5 * (tha + thb);
    }
    // feed the true condition at t; returns true when t is the accepted root
    bool update(double c, double h) {
      ++rit;
      if (!(std::abs(c) > 1e-12)) return true;  // converged (or NaN: stop here)
      if (sgn(c) == sgn(ca)) { tha = t; ca = c; if (side == -1) cb *= 0.5; side = -1; }
      else { thb = t; cb = c; if (side == 1) ca *= 0.5; side = 1; }
      if ((thb - tha) * h < 1e-13 || rit >= 9) return true;
      double tn = (rit == 1) ? t - c / slope : tha - ca * (thb - tha) / (cb - ca);
      if (!(tn > tha && tn < thb)) tn = 0.5 * (tha + thb);
      t = tn;
      return false;
    }
  };

  // affect! (RayTracer.jl:301-350). Returns 0 skip, 1 recorded, 2 recorded + terminate
  int affect(const double u[7], double tau) {
    const double s = 1.0001;
    if (callback_count == 0) {
      double pos[3] = {std::sin(u[1]) * std::cos(u[2]), std::sin(u[1]) * std::sin(u[2]), std::cos(u[1])};
      bool all_lt = true, all_gt = true;
      for (int i = 0; i < 3; ++i) {
        pos[i] *= u[0];
        all_lt = all_lt && (std::abs(pos[i]) < std::abs(x0c[i]) * s);
        all_gt = all_gt && (std::abs(pos[i]) > std::abs(x0c[i]) / s);
      }
      if (all_lt && all_gt) return 0;
    }
    Crossing c;
    c.pos[0] = u[0] * std::sin(u[1]) * std::cos(u[2]);
    c.pos[1] = u[0] * std::sin(u[1]) * std::sin(u[2]);
    c.pos[2] = u[0] * std::cos(u[1]);
    if (std::sqrt(sq(c.pos[0]) + sq(c.pos[1]) + sq(c.pos[2])) < P.rNS * 1.01) return 0;
    c.t = std::exp(tau);
    c.dw = u[6] / erg;
    const double Mass_NS = P.flat ? 0.0 : P.mass_ns;
    double r_s = 2.0 * Mass_NS * GNew / (c_km * c_km);
    double om = 1.0 - r_s / u[0];
    double v[3] = {u[3] * std::sqrt(om), u[4] / u[0], u[5] / (u[0] * std::sin(u[1]))};
    for (double& vi : v) vi *= erg * om;
    double vt = std::sin(u[1]) * v[0] + std::cos(u[1]) * v[1];
    c.k[0] = std::cos(u[2]) * vt - std::sin(u[2]) * v[2];
    c.k[1] = std::sin(u[2]) * vt + std::cos(u[2]) * v[2];
    c.k[2] = std::cos(u[1]) * v[0] - std::sin(u[1]) * v[1];
    double pos_soa[3] = {c.pos[0], c.pos[1], c.pos[2]}, k_soa[3] = {c.k[0], c.k[1], c.k[2]};
    double eeff = erg * std::abs(c.dw);  // get_tree: erg_inf_ini .* abs.(Δωc) (MainRunner.jl:265)
    get_prob_nonad(P, 1, pos_soa, k_soa, &eeff, &c.p);
    crossings.push_back(c);
    callback_count += 1;
    int maxc = max_crossings <= 0 ? -1 : max_crossings;
    if (callback_count >= maxc) return 2;
    return 1;
  }

  // Run the segment from u (state), tau0 to P.ln_t_end.
  int run(double u[7], double& tau, int& n_acc, int& n_rej) {
    const double tend = P.ln_t_end;
    double fcur[7];
    f(u, tau, fcur);
    double dt;
    const bool rk4 = P.integrator == ART_RK4;
    const double dtmax = tend - tau;  // DiffEq default dtmax = tspan length
    if (rk4) dt = (tend - tau) / P.n_fixed;
    else dt = initdt(u, fcur, tau, tend - tau);
    double qold = 1e-4;
    const double beta1 = 7.0 / 60.0, beta2 = 1.0 / 15.0, gam = 0.9, qmin = 0.2, qmax = 10.0;
    double cprev = cond(u, tau);
    int sprev = std::isnan(cprev) ? 0 : sgn(cprev);
    int64_t iter = 0;
    bool just_evented = false;
    n_acc = n_rej = 0;
    const int npts = std::max(P.interp_points, 2);
    while (true) {
      if (tau >= tend) return ART_STATUS_SUCCESS;
      if (iter >= P.maxiters) return ART_STATUS_MAXITERS;
      ++iter;
      double h = dt;
      bool last = false, forced = false;
      if (tau + h >= tend) { h = tend - tau; last = true; }
      if (!rk4 && h < P.dtmin && !last) { h = P.dtmin; forced = true; }
      double unew[7], fnew[7];
      double EEst = step(u, fcur, tau, h, unew, fnew);
      if (trace) std::fprintf(stderr, "it=%lld tau=%.6f h=%.3e EEst=%.3e r=%.6f th=%.6f u7=%.6e rnew=%.6f\n",
                              (long long)iter, tau, h, EEst, u[0], u[1], u[6], unew[0]);
      bool finite = std::isfinite(EEst);
      for (int i = 0; i < 7; ++i) finite = finite && std::isfinite(unew[i]);
      if (!finite) return ART_STATUS_NONFINITE;
      double q = 1.0, q11 = 1.0;
      if (!rk4) {
        if (EEst == 0.0) q = 1.0 / qmax;
        else {
          q11 = std::pow(EEst, beta1);
          q = q11 / std::pow(qold, beta2);
          q = std::max(1.0 / qmax, std::min(1.0 / qmin, q / gam));
        }
        if (!(EEst <= 1.0) && !forced) {  // reject
          dt = h / std::min(1.0 / qmin, q11 / gam);
          ++n_rej;
          continue;
        }
      }
      ++n_acc;
      double dtnext = dt;
      if (!rk4) {  // qsteady_min = qsteady_max = 1: only q == 1 is "steady"
        qold = std::max(EEst, 1e-4);
        dtnext = h / q;
      }
      // ContinuousCallback sign scan on the step (interp_points points, :358)
      // Samples whose condition is NaN carry no sign: the reference would raise DomainError
      // in sqrt(NrmSq) (:281-282) once |u7| < m_a. A NaN sample resets the sign memory, so a
      // crossing needs defined condition values on both sides ("no resonance possible").
      double last_c = cprev, last_th = 0.0;
      int last_s = sprev;
      bool evented = false;
      // make_tree = false installs no callbacks at all (RayTracer.jl:361-377): no scan, no cb_r
      const bool cbs = max_crossings != INT32_MIN;
      for (int ip = 1; cbs && ip < npts && !evented; ++ip) {
        double th = double(ip) / double(npts - 1);
        double ui[7];
        hermite(u, fcur, unew, fnew, h, th, ui);
        double ci = cond(ui, tau + th * h);
        if (std::isnan(ci)) { last_s = 0; continue; }
        int si = sgn(ci);
        if (!(last_s != 0 && si != 0 && si != last_s)) {
          if (si != 0) { last_s = si; last_c = ci; last_th = th; }
          continue;
        }
        // Sign change in (last_th, th]. (1) Illinois on the cubic Hermite interpolant (cheap
        // condition evaluations only); (2) polish on the TRUE trajectory by re-stepping from
        // (u, fcur), always inside the detection bracket so time never runs backwards: a
        // Newton step with the interpolant's slope, then Illinois, until |condition| <= 1e-12
        // (above the ~1e-13 noise floor of a re-stepped condition), the bracket is below
        // 1e-13 in ln t, or 9 re-steps. After an event, DiffEq takes the sign from a point
        // nudged 1/100 of a step ahead (repeat_nudge); sign changes before it are ignored.
        const double t_int = illinois_interp(u, fcur, unew, fnew, tau, h, last_th, th, last_c, ci);
        if (just_evented && t_int < 0.01) {
          last_s = si; last_c = ci; last_th = th;
          continue;
        }
        RootBracket rb(last_th, last_c, th, ci, t_int);
        last_s = si; last_c = ci; last_th = th;
        double ur[7], fr[7];
        for (;;) {
          step(u, fcur, tau, rb.t * h, ur, fr);
          const double c1 = cond(ur, tau + rb.t * h);
          ++n_root_steps;
          if (trace) std::fprintf(stderr, "  root it=%d th=%.17g c=%.6e\n", rb.rit, rb.t, c1);
          if (rb.update(c1, h)) break;
        }
        const double tr = rb.t;
        const double tau_r = tau + tr * h;
        const int a = affect(ur, tau_r);
        std::memcpy(u, ur, sizeof(double) * 7);
        std::memcpy(fcur, fr, sizeof(double) * 7);
        tau = tau_r;
        cprev = ci;  // post-event side: DiffEq keeps it so the same root is not re-found
        sprev = si;
        just_evented = true;
        evented = true;
        if (a == 2) return ART_STATUS_CROSSING;
        if (photon && u[0] < P.rNS * 1.01) return ART_STATUS_HIT_NS;  // cb_r after the event
        if (!rk4) dt = std::min(dtnext, dtmax);  // fixed-step RK4 keeps its dt (last step clipped)
      }
      if (evented) continue;
      std::memcpy(u, unew, sizeof(double) * 7);
      std::memcpy(fcur, fnew, sizeof(double) * 7);
      tau = last ? tend : tau + h;
      cprev = last_c;
      sprev = last_s;
      just_evented = false;
      if (cbs && photon && u[0] < P.rNS * 1.01) return ART_STATUS_HIT_NS;  // cb_r (:352-359)
      if (last) return ART_STATUS_SUCCESS;
      if (!rk4) dt = std::min(dtnext, dtmax);
    }
  }

  const art_params& P;
  bool photon;
  double erg;
  double x0c[3];
  int max_crossings;
  int callback_count = 0;
  int64_t n_root_steps = 0;
  std::vector<Crossing> crossings;
  bool trace = std::getenv("ORACLE_TRACE") != nullptr;
};

// ---------------------------------------------------------------------------
// Event weight of one sampled conversion point (MainRunner.jl:498-557): the incoming-axion
// rate sln_prob (npy column 8 before the final division by f_inx), built from cos_w of
// dwp_ds (RayTracer.jl:1327-1403) and jacobian_GR = g_det (:734-754).

// omega_function (RayTracer.jl:558-589) as dwp_ds calls it (:1367): time0 = 0, the
// defaults flat = false, zeroIn = false, bndry_lyr = -1, melrose = true; r < rNS is
// clamped in place (a constant for the dual numbers). erg is unused by the reference.
template <class T>
T omega_function(T r, const T& th, const T& ph, const double k[3], const art_params& P, double Mass_NS, bool iso) {
  if (val(r) < P.rNS) r = T(P.rNS);
  T omP = GJ_wp_vecSPH(r, th, ph, T(0.0), P, false, -1.0, P.mass_a);
  Metric<T> g = g_schwartz(r, th, Mass_NS);
  T ksqr = g.grr * sq(k[0]) + g.gthth * sq(k[1]) + g.gpp * sq(k[2]);
  if (iso) return sqrt(ksqr + sq(omP));
  T kpar = K_par(r, th, ph, T(k[0]), T(k[1]), T(k[2]), T(0.0), P, Mass_NS);
  T Ham = (ksqr + sq(omP) + sqrt(sq(ksqr) + 2.0 * ksqr * sq(omP) - 4.0 * sq(kpar) * sq(omP) + pow(omP, 4.0))) /
          std::sqrt(2.0);
  return sqrt(Ham);
}

struct EventWeight { double cos_w, jacobian_GR, sln_prob, erg_inf_ini, vel_eng; };

EventWeight event_weight(const art_params& P, const double x[3], const double k_init[3], const double vIfty[3],
                         double maxR, double rho_DM, double mcmc_weight) {
  const double Mass_NS = P.mass_ns, Mass_a = P.mass_a;
  EventWeight E{};
  // MainRunner.jl:505-517
  const double rmag = std::sqrt(sq(x[0]) + sq(x[1]) + sq(x[2]));
  const double vmag2 = sq(vIfty[0]) + sq(vIfty[1]) + sq(vIfty[2]);
  E.vel_eng = (sq(vIfty[0] / c_km) + sq(vIfty[1] / c_km) + sq(vIfty[2] / c_km)) / 2.0;
  const double vIfty_mag = std::sqrt(vmag2);
  const double gammaA = 1.0 / std::sqrt(1.0 - sq(vIfty_mag));
  E.erg_inf_ini = Mass_a * std::sqrt(1.0 + sq(vIfty_mag * gammaA));
  // k_sphere (:983-1009, flat honoured) at the sample point
  Sph s = cart_to_sph(x);
  const double Mk = P.flat ? 0.0 : Mass_NS;
  double ks[3];
  celerity(x, k_init, s, 1.0 - 2.0 * Mk * GNew / (c_km * c_km) / s.r, ks);
  // dwp_ds cos_w (:1367-1371): gradient of omega_function over (r, θ, φ) at fixed k
  D3 r = D3::seed(s.r, 0), th = D3::seed(s.th, 1), ph = D3::seed(s.ph, 2);
  D3 om = omega_function(r, th, ph, ks, P, Mass_NS, P.isotropic != 0);
  Metric<double> g = g_schwartz(s.r, s.th, Mass_NS);
  const double gn = std::sqrt(g.grr * sq(om.d[0]) + g.gthth * sq(om.d[1]) + g.gpp * sq(om.d[2]));
  const double kmag = std::sqrt(g.grr * sq(ks[0]) + g.gthth * sq(ks[1]) + g.gpp * sq(ks[2]));
  E.cos_w = std::abs(g.grr * ks[0] / kmag * om.d[0] / gn + g.gthth * ks[1] / kmag * om.d[1] / gn +
                     g.gpp * ks[2] / kmag * om.d[2] / gn);
  // g_det (:734-754), zeroIn = false, with the run's bndry_lyr and Mass_a
  if (P.flat) {
    E.jacobian_GR = 1.0;
  } else {
    D3 w = GJ_wp_vecSPH(r, th, ph, D3(0.0), P, false, P.bndry_lyr, Mass_a);
    const double dr_th = w.d[1] / w.d[0], dr_p = w.d[2] / w.d[0];
    const double A = g.grr, st2 = sq(std::sin(s.th));
    const double det = s.r * std::sqrt(st2 * (A * sq(s.r) + sq(dr_th)) + sq(dr_p));
    const double det0 = s.r * std::sqrt(st2 * (sq(s.r) + sq(dr_th)) + sq(dr_p));
    E.jacobian_GR = det / det0;
  }
  // MainRunner.jl:545-554
  const double dense_extra = 2.0 / std::sqrt(PI) * (1.0 / (220.0 / c_km)) *
                             std::sqrt(2.0 * Mass_NS * GNew / (c_km * c_km) / rmag);
  const double redshift = std::sqrt(1.0 - 2.0 * GNew * Mass_NS / rmag / (c_km * c_km));
  const double phaseS = dense_extra * (2.0 * PI * sq(maxR)) * (rho_DM * 1e9) / Mass_a * E.jacobian_GR;
  E.sln_prob = E.cos_w * redshift * phaseS * (1e5 * 1e5) * c_km * 1e5 * mcmc_weight;
  return E;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11) -- the counter-based stream that replaces
// Julia's global Random stream (SURVEY §7 hard part iv).
inline void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = uint64_t(0xD2511F53u) * c0, p1 = uint64_t(0xCD9E8D57u) * c2;
    uint32_t hi0 = uint32_t(p0 >> 32), lo0 = uint32_t(p0), hi1 = uint32_t(p1 >> 32), lo1 = uint32_t(p1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

inline double u01(uint32_t a, uint32_t b) {  // 53-bit uniform in [0, 1)
  return (double(a >> 5) * 67108864.0 + double(b >> 6)) * (1.0 / 9007199254740992.0);
}

// The 10 uniforms of one find_samples_new attempt, drawn in the reference's order:
// θi, ϕi, θi_loc, ϕi_loc, ϕRND, rRND (:1486-1497), vIfty x3 (:1531), randInx (:1623).
inline void attempt_uniforms(uint64_t seed, uint64_t ray, uint32_t attempt, double U[10]) {
  uint32_t key[2] = {uint32_t(seed), uint32_t(seed >> 32)};
  for (uint32_t blk = 0; blk < 5; ++blk) {
    uint32_t ctr[4] = {uint32_t(ray), uint32_t(ray >> 32), attempt, blk}, o[4];
    philox4x32_10(ctr, key, o);
    U[2 * blk] = u01(o[0], o[1]);
    U[2 * blk + 1] = u01(o[2], o[3]);
  }
}

// Sampler condition -- RayTracer.jl:1547-1583 (thick_surface = true), on the line point x
double sampler_condition(const art_params& P, const double x[3], const double vloc[3], double E) {
  const double Mass_NS = P.mass_ns;
  Sph s = cart_to_sph(x);
  double r_s0 = 2.0 * Mass_NS * GNew / (c_km * c_km);
  double AA = 1.0 - r_s0 / s.r;
  if (s.r < P.rNS) AA = 1.0;
  double w[3];
  celerity(x, vloc, s, AA, w);
  Metric<double> g = g_schwartz(s.r, s.th, Mass_NS);
  double NrmSq = (-sq(E) * g.gtt - sq(P.mass_a)) / (sq(w[0]) * g.grr + sq(w[1]) * g.gthth + sq(w[2]) * g.gpp);
  double f = std::sqrt(NrmSq);
  for (double& wi : w) wi *= f;
  double omP = GJ_wp_vec(x, 0.0, P, P.bndry_lyr, P.mass_a);
  double kpar = P.isotropic ? 0.0 : K_par(s.r, s.th, s.ph, w[0], w[1], w[2], 0.0, P, Mass_NS);
  double ksqr = g.gtt * sq(E) + g.grr * sq(w[0]) + g.gthth * sq(w[1]) + g.gpp * sq(w[2]);
  return 0.5 * (ksqr + sq(omP) * (sq(E) / g.grr - sq(kpar)) / (sq(E) / g.grr)) / sq(E);
}

struct SampleAttempt {
  int n_found;  // crossings accepted by affect!
  bool ok;
  double x[3], vel[3], vifty_c[3];
};

// One find_samples_new call (RayTracer.jl:1480-1653) with the Euler line scan
// (dt = 0.5 km over [0, 2.2 maxR], :1611-1613) and ContinuousCallback(interp_points=20).
SampleAttempt find_samples_attempt(const art_params& P, double maxR, const double U[10]) {
  const double thi = std::acos(1.0 - 2.0 * U[0]), phi = U[1] * 2 * PI;
  const double thl = std::acos(1.0 - 2.0 * U[2]), phl = U[3] * 2 * PI;
  const double phR = U[4] * 2 * PI, rR = std::sqrt(U[5]) * maxR;
  const double va[3] = {std::sin(thi) * std::cos(phi), std::sin(thi) * std::sin(phi), std::cos(thi)};
  const double vl[3] = {std::sin(thl) * std::cos(phl), std::sin(thl) * std::sin(phl), std::cos(thl)};
  const double x1 = rR * std::cos(phR), x2 = rR * std::sin(phR);
  double x0[3] = {x1 * std::cos(-phi) * std::cos(-thi) + x2 * std::sin(-phi),
                  x2 * std::cos(-phi) - x1 * std::sin(-phi) * std::cos(-thi), x1 * std::sin(-thi)};
  double vI[3];
  for (int i = 0; i < 3; ++i) vI[i] = (220.0 + U[6 + i] * 1.0e-5) / std::sqrt(3.0);
  const double vmag = std::sqrt((sq(vI[0]) + sq(vI[1])) + sq(vI[2]));
  const double gammaA = 1 / std::sqrt(1.0 - sq(vmag / c_km));
  const double E = P.mass_a * std::sqrt(1 + sq(vmag / c_km * gammaA));
  for (int i = 0; i < 3; ++i) x0[i] += va[i] * (-maxR * 1.1);
  auto line = [&](double s, double x[3]) { for (int i = 0; i < 3; ++i) x[i] = x0[i] + va[i] * s; };
  auto cf = [&](double s) { double x[3]; line(s, x); return sampler_condition(P, x, vl, E); };
  std::vector<double> found;
  const double send = 2.2 * maxR, ds = 0.5;
  const int np = 20;
  double s0 = 0.0, c0 = cf(0.0);
  while (s0 < send) {
    double s1 = std::min(s0 + ds, send);
    double sl = s0, cl = c0;
    for (int ip = 1; ip < np; ++ip) {
      double sc = s0 + (s1 - s0) * double(ip) / double(np - 1);
      double cc = cf(sc);
      if (std::signbit(cl) != std::signbit(cc) && cl != 0.0 && cc != 0.0) {
        double a = sl, b = sc, fa = cl, fb = cc, root = sc;  // Illinois on the exact line
        int side = 0;
        for (int it = 0; it < 100; ++it) {
          root = a - fa * (b - a) / (fb - fa);
          double fr = cf(root);
          if (fr == 0.0 || (b - a) < 1e-13 * std::max(1.0, std::abs(root))) break;
          if (std::signbit(fr) == std::signbit(fa)) { a = root; fa = fr; if (side == -1) fb *= 0.5; side = -1; }
          else { b = root; fb = fr; if (side == 1) fa *= 0.5; side = 1; }
        }
        double xr[3];
        line(root, xr);
        // affect! (:1585-1597)
        Sph s = cart_to_sph(xr);
        double omP = GJ_wp_vec(xr, 0.0, P, P.bndry_lyr, P.mass_a);
        Metric<double> g = g_schwartz(s.r, s.th, P.mass_ns);
        double ergL = E / std::sqrt(g.grr);
        if (s.r > P.rNS && ergL > omP) for (int i = 0; i < 3; ++i) found.push_back(xr[i]);
      }
      sl = sc; cl = cc;
    }
    s0 = s1; c0 = cl;
  }
  SampleAttempt out{};
  out.n_found = int(found.size() / 3);
  out.ok = false;
  if (out.n_found == 0) return out;
  int randInx = 1 + int(U[9] * 6.0);  // rand(1:n_max), n_max = n_maxSample = 6
  if (randInx > 6) randInx = 6;
  if (out.n_found < randInx) return out;
  for (int i = 0; i < 3; ++i) out.x[i] = found[3 * (randInx - 1) + i];
  double rmag = std::sqrt((sq(out.x[0]) + sq(out.x[1])) + sq(out.x[2]));
  double vmag_loc = std::sqrt(sq(vmag) + 2 * GNew * P.mass_ns / rmag) / c_km;
  for (int i = 0; i < 3; ++i) { out.vel[i] = vl[i] * vmag_loc; out.vifty_c[i] = vI[i] / c_km; }
  out.ok = true;
  return out;
}

}  // namespace oracle

// ============================================================================
// extern "C" surface (ctypes) -- names prefixed oracle_.
// ============================================================================
using namespace oracle;

extern "C" {

void oracle_philox4x32_10(const uint32_t* ctr, const uint32_t* key, uint32_t* out) { philox4x32_10(ctr, key, out); }

void oracle_attempt_uniforms(uint64_t seed, uint64_t ray, uint32_t attempt, double* U) {
  attempt_uniforms(seed, ray, attempt, U);
}

void oracle_vern6_tableau(double* c, double* A, double* b, double* bhat) {
  for (int i = 0; i < 9; ++i) {
    c[i] = Vern6::c[i]; b[i] = V6.b[i]; bhat[i] = V6.bhat[i];
    for (int j = 0; j < 9; ++j) A[9 * i + j] = V6.A[i][j];
  }
}

void oracle_metric(double r, double th, double Mass_NS, double* g4) {
  Metric<double> g = g_schwartz(r, th, Mass_NS);
  g4[0] = g.gtt; g4[1] = g.grr; g4[2] = g.gthth; g4[3] = g.gpp;
}

double oracle_omega_p(const art_params* P, double r, double th, double ph, double t, int zeroIn, double bndry) {
  return GJ_wp_vecSPH(r, th, ph, t, *P, zeroIn != 0, bndry, P->mass_a);
}

// H, dH/dx (3), dH/dk (3), dH/dT at (x, k, T, E); flat handled like func! (Mass_NS -> 0)
void oracle_hamiltonian(const art_params* P, const double* x, const double* k, double T, double E, double* H,
                        double* dHdx, double* dHdk, double* dHdT) {
  const double M = P->flat ? 0.0 : P->mass_ns;
  const bool iso = P->isotropic != 0;
  D3 r = D3::seed(x[0], 0), th = D3::seed(x[1], 1), ph = D3::seed(x[2], 2);
  D3 Hx = hamiltonian<D3>(r, th, ph, D3(k[0]), D3(k[1]), D3(k[2]), D3(T), D3(E), *P, M, iso, P->bndry_lyr);
  D3 k1 = D3::seed(k[0], 0), k2 = D3::seed(k[1], 1), k3 = D3::seed(k[2], 2);
  D3 Hk = hamiltonian<D3>(D3(x[0]), D3(x[1]), D3(x[2]), k1, k2, k3, D3(T), D3(E), *P, M, iso, P->bndry_lyr);
  D1 Ht = hamiltonian<D1>(D1(x[0]), D1(x[1]), D1(x[2]), D1(k[0]), D1(k[1]), D1(k[2]), D1::seed(T, 0), D1(E), *P, M,
                          iso, P->bndry_lyr);
  *H = Hx.v;
  for (int i = 0; i < 3; ++i) { dHdx[i] = Hx.d[i]; dHdk[i] = Hk.d[i]; }
  *dHdT = Ht.d[0];
}

void oracle_rhs(const art_params* P, int species, const double* u_in, double tau, double erg, double* du) {
  double u[7];
  std::memcpy(u, u_in, sizeof(u));
  if (species == ART_PHOTON) rhs_photon(*P, u, tau, erg, du); else rhs_axion(*P, u, tau, erg, du);
}

double oracle_condition(const art_params* P, const double* u, double tau) { return condition(*P, u, tau); }

void oracle_initial_state(const art_params* P, const double* x0, const double* k0, double erg, double dw, double* u0) {
  initial_state(*P, x0, k0, erg, dw, u0);
}

void oracle_back_transform(const art_params* P, const double* u, double erg, double* x, double* k) {
  back_transform(*P, u, erg, x, k);
}

double oracle_find_conversion_surface(const art_params* P) {
  // Find_Conversion_Surface(Mass_a, fix_time=0, θm, ω, B0, rNS, 1, false) -- RayTracer.jl:1250-1263
  double thEV = P->theta_m < (PI / 2.0) ? P->theta_m / 2.0 : (P->theta_m + PI) / 2.0;
  double x[3] = {P->rNS * std::sin(thEV), 0.0, P->rNS * std::cos(thEV)};
  double om = GJ_wp_scalar(x, 0.0, *P);
  double rc = P->rNS * std::pow(om / P->mass_a, 2.0 / 3.0);
  return rc * 1.01;
}

// get_Prob_nonAD over groups (group_start == NULL: one crossing per group)
void oracle_get_prob_nonad(const art_params* P, int64_t nc, const double* pos, const double* kpos,
                           const double* erg_eff, int64_t n_groups, const int64_t* group_start, double* out) {
  for (int64_t g = 0; g < n_groups; ++g) {
    int64_t a = group_start ? group_start[g] : g, b = group_start ? group_start[g + 1] : g + 1;
    int m = int(b - a);
    std::vector<double> ps(3 * m), kk(3 * m);
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < m; ++i) { ps[c * m + i] = pos[c * nc + a + i]; kk[c * m + i] = kpos[c * nc + a + i]; }
    get_prob_nonad(*P, m, ps.data(), kk.data(), erg_eff + a, out + a);
  }
}

// RT.propagate for n segments; outputs mirror art_segment_out / art_crossing_buf.
void oracle_propagate(const art_params* P, int64_t n, const double* x0, const double* k0, const double* erg,
                      const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                      double* x_end, double* k_end, double* u7_end, double* tau_end, int32_t* status,
                      int32_t* n_accept, int32_t* n_reject, int32_t cap, int32_t* xcount, double* xpos, double* xk,
                      double* xt, double* xdw, double* xp, int32_t nthreads) {
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads > 0 ? nthreads : 1)
  for (int64_t i = 0; i < n; ++i) {
    double xi[3] = {x0[i], x0[n + i], x0[2 * n + i]}, ki[3] = {k0[i], k0[n + i], k0[2 * n + i]};
    double u[7];
    initial_state(*P, xi, ki, erg[i], dw[i], u);
    Segment seg(*P, species[i], erg[i], xi, max_crossings);
    double tau = ln_t0[i];
    int na = 0, nr = 0;
    int st = seg.run(u, tau, na, nr);
    double xe[3], ke[3];
    back_transform(*P, u, erg[i], xe, ke);
    for (int c = 0; c < 3; ++c) { x_end[c * n + i] = xe[c]; k_end[c * n + i] = ke[c]; }
    u7_end[i] = u[6]; tau_end[i] = tau; status[i] = st; n_accept[i] = na; n_reject[i] = nr;
    if (xcount) {
      xcount[i] = int32_t(seg.crossings.size());
      for (int j = 0; j < std::min<int>(cap, int(seg.crossings.size())); ++j) {
        const Crossing& c = seg.crossings[j];
        for (int q = 0; q < 3; ++q) {
          xpos[(q * cap + j) * n + i] = c.pos[q];
          xk[(q * cap + j) * n + i] = c.k[q];
        }
        xt[j * n + i] = c.t; xdw[j * n + i] = c.dw; xp[j * n + i] = c.p;
      }
    }
  }
}

// find_samples_new + main_runner's k_init (MainRunner.jl:463-529), one accepted sample per ray.
void oracle_sample(const art_params* P, double maxR, uint64_t seed, int64_t ray_offset, int64_t n, double* x,
                   double* k_init, double* erg_inf, double* vifty, int32_t* weights, int32_t* attempts,
                   int32_t nthreads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int64_t i = 0; i < n; ++i) {
    uint64_t ray = uint64_t(ray_offset + i);
    for (uint32_t a = 0; a < 1000000u; ++a) {
      double U[10];
      attempt_uniforms(seed, ray, a, U);
      SampleAttempt s = find_samples_attempt(*P, maxR, U);
      if (!s.ok) continue;
      double vm = std::sqrt((sq(s.vifty_c[0]) + sq(s.vifty_c[1])) + sq(s.vifty_c[2]));  // :514 (unitless)
      double gA = 1 / std::sqrt(1.0 - sq(vm));
      double E = P->mass_a * std::sqrt(1 + sq(vm * gA));
      double kn[3];
      k_norm_cart_axion_shell(s.x, s.vel, E, *P, P->mass_ns, kn);  // :529, ax_fix=true
      for (int c = 0; c < 3; ++c) { x[c * n + i] = s.x[c]; k_init[c * n + i] = kn[c]; vifty[c * n + i] = s.vifty_c[c]; }
      erg_inf[i] = E; weights[i] = s.n_found; attempts[i] = int32_t(a + 1);
      break;
    }
  }
}

void oracle_event_weight(const art_params* P, int64_t n, const double* x, const double* k_init,
                         const double* vIfty, double maxR, double rho_DM, double mcmc_weight, double* out5) {
  // x, k_init, vIfty: 3n SoA; out5: 5n SoA (cos_w, jacobian_GR, sln_prob, erg_inf_ini, vel_eng)
  for (int64_t i = 0; i < n; ++i) {
    const double xi[3] = {x[i], x[n + i], x[2 * n + i]}, ki[3] = {k_init[i], k_init[n + i], k_init[2 * n + i]};
    const double vi[3] = {vIfty[i], vIfty[n + i], vIfty[2 * n + i]};
    EventWeight E = event_weight(*P, xi, ki, vi, maxR, rho_DM, mcmc_weight);
    out5[i] = E.cos_w; out5[n + i] = E.jacobian_GR; out5[2 * n + i] = E.sln_prob;
    out5[3 * n + i] = E.erg_inf_ini; out5[4 * n + i] = E.vel_eng;
  }
}

double oracle_sampler_condition(const art_params* P, const double* x, const double* vloc, double E) {
  return sampler_condition(*P, x, vloc, E);
}

}  // extern "C"
