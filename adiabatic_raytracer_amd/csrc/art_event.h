// art_event.h -- per-sample event weight of the conversion-surface sampler
// (MainRunner.jl:498-557): sln_prob, the incoming-axion rate that becomes column 8 of
// every npy row of the event, from cos_w of dwp_ds (RayTracer.jl:1327-1403) and
// jacobian_GR = g_det (:734-754). Evaluated once per sampled point (not on the ray hot
// loop), so the spatial gradients are taken with a 3-tangent forward-mode number over
// (r, θ, φ), exactly what the reference's ForwardDiff seed/grad pair computes.
#pragma once

#include "art_core.h"

namespace art {

// value + gradient over (r, θ, φ)
struct Tan3 {
  double v, d[3];
  __host__ __device__ Tan3() : v(0.0), d{0.0, 0.0, 0.0} {}
  __host__ __device__ Tan3(double x) : v(x), d{0.0, 0.0, 0.0} {}
  __host__ __device__ static Tan3 var(double x, int k) {
    Tan3 t(x);
    t.d[k] = 1.0;
    return t;
  }
};

__host__ __device__ inline Tan3 lin3(const Tan3& a, double f, double fp) {  // f(a) with f'(a) = fp
  Tan3 r(f);
  for (int k = 0; k < 3; ++k) r.d[k] = fp * a.d[k];
  return r;
}
__host__ __device__ inline Tan3 operator+(const Tan3& a, const Tan3& b) {
  Tan3 r(a.v + b.v);
  for (int k = 0; k < 3; ++k) r.d[k] = a.d[k] + b.d[k];
  return r;
}
__host__ __device__ inline Tan3 operator-(const Tan3& a, const Tan3& b) {
  Tan3 r(a.v - b.v);
  for (int k = 0; k < 3; ++k) r.d[k] = a.d[k] - b.d[k];
  return r;
}
__host__ __device__ inline Tan3 operator-(const Tan3& a) { return lin3(a, -a.v, -1.0); }
__host__ __device__ inline Tan3 operator*(const Tan3& a, const Tan3& b) {
  Tan3 r(a.v * b.v);
  for (int k = 0; k < 3; ++k) r.d[k] = a.d[k] * b.v + a.v * b.d[k];
  return r;
}
__host__ __device__ inline Tan3 operator/(const Tan3& a, const Tan3& b) {
  const double q = a.v / b.v;
  Tan3 r(q);
  for (int k = 0; k < 3; ++k) r.d[k] = (a.d[k] - q * b.d[k]) / b.v;
  return r;
}
__host__ __device__ inline Tan3 operator+(const Tan3& a, double b) { return lin3(a, a.v + b, 1.0); }
__host__ __device__ inline Tan3 operator+(double a, const Tan3& b) { return lin3(b, a + b.v, 1.0); }
__host__ __device__ inline Tan3 operator-(const Tan3& a, double b) { return lin3(a, a.v - b, 1.0); }
__host__ __device__ inline Tan3 operator-(double a, const Tan3& b) { return lin3(b, a - b.v, -1.0); }
__host__ __device__ inline Tan3 operator*(const Tan3& a, double b) { return lin3(a, a.v * b, b); }
__host__ __device__ inline Tan3 operator*(double a, const Tan3& b) { return lin3(b, a * b.v, a); }
__host__ __device__ inline Tan3 operator/(const Tan3& a, double b) { return lin3(a, a.v / b, 1.0 / b); }
__host__ __device__ inline Tan3 operator/(double a, const Tan3& b) { return lin3(b, a / b.v, -a / (b.v * b.v)); }
__host__ __device__ inline bool operator<(const Tan3& a, double b) { return a.v < b; }
__host__ __device__ inline bool operator<=(const Tan3& a, double b) { return a.v <= b; }
__host__ __device__ inline bool operator>(const Tan3& a, double b) { return a.v > b; }
__host__ __device__ inline bool operator>=(const Tan3& a, double b) { return a.v >= b; }

__host__ __device__ inline Tan3 msqrt(const Tan3& a) {
  const double s = sqrt(a.v);
  return lin3(a, s, 0.5 / s);
}
__host__ __device__ inline Tan3 mexp(const Tan3& a) {
  const double e = exp(a.v);
  return lin3(a, e, e);
}
__host__ __device__ inline Tan3 mabs(const Tan3& a) { return lin3(a, fabs(a.v), signbit(a.v) ? -1.0 : 1.0); }
__host__ __device__ inline void msincos(const Tan3& a, Tan3& s, Tan3& c) {
  double sv, cv;
  msincos(a.v, sv, cv);
  s = lin3(a, sv, cv);
  c = lin3(a, cv, -sv);
}

// GJ_Model_ωp_vecSPH (RayTracer.jl:1120-1170) at t, zeroIn = false; the boundary layer
// (:1155-1162, r >= rNS) when with_layer and bndry_lyr > 0, with the run's Mass_a.
template <class T>
__host__ __device__ inline T gj_wp(const KParams& P, const T& r, const T& th, const T& ph, double t, bool with_layer,
                                   DipoleAng<T>* dout = nullptr) {
  T st, ct, sp, cp;
  msincos(th, st, ct);
  msincos(ph - P.omega * t, sp, cp);
  const DipoleAng<T> d = dipole_ang(P, st, ct, sp, cp);
  if (dout) *dout = d;
  T wp = msqrt(P.wp2n / (r * r * r) * mabs(d.b));  // n_e = |2 ω Bz ...|: either sign of B0
  if (with_layer && P.bndry_lyr > 0.0 && r >= P.rNS) wp = wp + layer_wp(P, r, P.rmax);
  return wp;
}

// omega_function (RayTracer.jl:558-589) as dwp_ds calls it (:1367): t = 0, the reference's
// defaults flat = false (GR metric with the run's Mass_NS), zeroIn = false, bndry_lyr = -1,
// melrose = true; r < rNS clamped in place (a constant); k is the covariant k_sphere.
template <class T>
__host__ __device__ inline T omega_fn(const KParams& P, T r, const T& th, const T& ph, const double k[3]) {
  if (r < P.rNS) r = T(P.rNS);
  DipoleAng<T> d;
  const T wp = gj_wp(P, r, th, ph, 0.0, false, &d);
  T gtt, grr;
  metric_tr(r, P.rs_gr, gtt, grr);
  T st, ct;
  msincos(th, st, ct);
  const T gthth = 1.0 / (r * r);
  const T gpp = gthth / (st * st);
  const T ksqr = grr * (k[0] * k[0]) + gthth * (k[1] * k[1]) + gpp * (k[2] * k[2]);
  const T wp2 = wp * wp;
  if (P.isotropic) return msqrt(ksqr + wp2);
  // K_par (:1044-1058): B covariant (Br/√g^rr, Bθ/√g^θθ, Bφ/√g^φφ), flat = false
  const T Bn = P.Bn_coef / (r * r * r);
  const T Bs0 = 2.0 * Bn * d.a1 / msqrt(grr);
  const T Bs1 = Bn * d.a2 / msqrt(gthth);
  const T Bs2 = Bn * d.a3 / msqrt(gpp);
  const T Bmag = msqrt(grr * Bs0 * Bs0 + gthth * Bs1 * Bs1 + gpp * Bs2 * Bs2);
  const T kpar = (grr * k[0] * Bs0 + gthth * k[1] * Bs1 + gpp * k[2] * Bs2) / Bmag;
  const T Ham = (ksqr + wp2 + msqrt(ksqr * ksqr + 2.0 * ksqr * wp2 - 4.0 * kpar * kpar * wp2 + wp2 * wp2)) /
                1.4142135623730951;  // sqrt(2) (:584)
  return msqrt(Ham);
}

struct EventW {
  double cos_w, jacobian_GR, sln_prob, erg_inf_ini, vel_eng;
};

// x: sampled conversion point [km]; k_init: k_norm_Cart onto the axion shell at erg_inf_ini
// (MainRunner.jl:528-529); vifty: vIfty/c from find_samples_new (unitless).
__host__ __device__ inline EventW event_weight(const KParams& P, const double x[3], const double k_init[3],
                                               const double vifty[3], double maxR, double rho_DM, double mcmc_weight) {
  EventW E;
  // MainRunner.jl:505-526
  const double rmag = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  const double v1 = vifty[0] / C_KM, v2 = vifty[1] / C_KM, v3 = vifty[2] / C_KM;
  E.vel_eng = (v1 * v1 + v2 * v2 + v3 * v3) / 2.0;
  const double vm = sqrt(vifty[0] * vifty[0] + vifty[1] * vifty[1] + vifty[2] * vifty[2]);
  const double gA = 1.0 / sqrt(1.0 - vm * vm);
  E.erg_inf_ini = P.mass_a * sqrt(1.0 + (vm * gA) * (vm * gA));
  // k_sphere (:983-1009) at the sample point, flat honoured
  double r, th, ph;
  cart_to_sph(x, r, th, ph);
  double ks[3];
  celerity(x, k_init, r, sin(th), P.rs_eff, ks);
  // cos_w (:1367-1371): ∇ω over (r, θ, φ) at fixed k, normalised with the GR metric
  const Tan3 tr = Tan3::var(r, 0), tt = Tan3::var(th, 1), tp = Tan3::var(ph, 2);
  const Tan3 om = omega_fn(P, tr, tt, tp, ks);
  double gtt, grr;
  metric_tr(r, P.rs_gr, gtt, grr);
  const double gthth = 1.0 / (r * r), gpp = gthth / (sin(th) * sin(th));
  const double gn = sqrt(grr * om.d[0] * om.d[0] + gthth * om.d[1] * om.d[1] + gpp * om.d[2] * om.d[2]);
  const double kmag = sqrt(grr * ks[0] * ks[0] + gthth * ks[1] * ks[1] + gpp * ks[2] * ks[2]);
  E.cos_w = fabs(grr * (ks[0] / kmag) * (om.d[0] / gn) + gthth * (ks[1] / kmag) * (om.d[1] / gn) +
                 gpp * (ks[2] / kmag) * (om.d[2] / gn));
  // g_det (:734-754): ratio of √det with and without the GR g_rr, from ∇ωp (zeroIn = false)
  if (P.flat) {
    E.jacobian_GR = 1.0;
  } else {
    const Tan3 w = gj_wp(P, tr, tt, tp, 0.0, true);
    const double dr_th = w.d[1] / w.d[0], dr_p = w.d[2] / w.d[0];
    const double st2 = sin(th) * sin(th);
    const double det = r * sqrt(st2 * (grr * r * r + dr_th * dr_th) + dr_p * dr_p);
    const double det0 = r * sqrt(st2 * (r * r + dr_th * dr_th) + dr_p * dr_p);
    E.jacobian_GR = det / det0;
  }
  // MainRunner.jl:545-554
  const double GM2 = 2.0 * P.GM_c2;  // 2 GNew Mass_NS / c^2
  const double dense_extra = 2.0 / sqrt(PI) * (1.0 / (220.0 / C_KM)) * sqrt(GM2 / rmag);
  const double redshift = sqrt(1.0 - GM2 / rmag);
  const double phaseS = dense_extra * (2.0 * PI * maxR * maxR) * (rho_DM * 1e9) / P.mass_a * E.jacobian_GR;
  E.sln_prob = E.cos_w * redshift * phaseS * 1e10 * C_KM * 1e5 * mcmc_weight;
  return E;
}

}  // namespace art
