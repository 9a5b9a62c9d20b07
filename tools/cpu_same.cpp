// CPU BASELINE ONLY (bench.py's cpu_baseline leg): the engine's own algorithm on the host
// cores, so the GPU/CPU ratio compares like with like ("the build's C++
// restatement, same kernel header, OpenMP over rays"). Never loaded by the product.
//
// Per ray, RT.propagate's forward segment (RayTracer.jl:171-452) with the product's physics
// header compiled for the host (art_core.h: the hand-derived one-pass RHS rhs_photon_gj, the
// closed-form condition, the scan certificates, prob_nonad_single) and the integrator the
// kernel runs, written as a scalar loop: Vern6 with OrdinaryDiffEq's PI controller and
// Hairer's initial dt, the 50-point cubic-Hermite sign scan with its certificates, the
// bracket polished on the true trajectory by re-stepping, affect! and cb_r. The dual-number
// oracle (oracle/art_oracle.cpp) is the other CPU figure: the reference's ForwardDiff cost.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../adiabatic_raytracer_amd/csrc/art_core.h"

#ifndef CPU_SAME_ATTEMPT_HOOK  // (tools/exp_gr_predict.cpp: per-attempt probes of the same loop)
#define CPU_SAME_ATTEMPT_HOOK(attempts, tau, u, dt)
#define CPU_SAME_RAY_HOOK(ray)
#endif

using namespace art;

namespace {

inline int sgn(double x) { return (x > 0) - (x < 0); }

struct Segment {
  const KParams& P;
  bool photon, gj;
  double erg;
  double x0c[3];
  int max_crossings;
  int count = 0;
  double xc[8] = {0};  // first recorded crossing: pos (3), k (3), t, dw
  double xp = 0.0;

  Segment(const KParams& P_, bool photon_, double erg_, const double* x0, int maxc)
      : P(P_), photon(photon_), gj(!(P_.bndry_lyr > 0.0) && !P_.isotropic), erg(erg_), max_crossings(maxc) {
    for (int i = 0; i < 3; ++i) x0c[i] = x0[i];
  }

  // the RHS with the hamiltonian's in-place clamp of the stage state (RayTracer.jl:531);
  // aux = {Bz/B_n, t} for the scan certificate
  void f(double* u, double tau, double* du, double* aux) {
    if (!photon) {
      rhs_axion(P, u, tau, erg, du);
      aux[0] = aux[1] = NAN;
    } else if (gj) {
      rhs_photon_gj(P, u, tau, erg, du, aux);
    } else {
      rhs_photon(P, u, tau, erg, du, aux);
    }
    if (photon && u[0] < P.rNS) u[0] = P.rNS;
  }

  double vern6(const double* u, const double* k1, double tau, double h, double* un, double* k9, double* aux) {
    using V = Vern6;
    double k[9][7], y[7];
    std::memcpy(k[0], k1, sizeof(double) * 7);
    static constexpr double c[9] = {0.0, V::c2, V::c3, V::c4, V::c5, V::c6, V::c7, 1.0, 1.0};
    static constexpr double A[9][8] = {
        {0}, {V::a21}, {V::a31, V::a32}, {V::a41, 0, V::a43}, {V::a51, 0, V::a53, V::a54},
        {V::a61, 0, V::a63, V::a64, V::a65}, {V::a71, 0, V::a73, V::a74, V::a75, V::a76},
        {V::a81, 0, V::a83, V::a84, V::a85, V::a86, V::a87}, {V::a91, 0, 0, V::a94, V::a95, V::a96, V::a97, V::a98}};
    for (int s = 1; s < 9; ++s) {
      for (int i = 0; i < 7; ++i) {
        double acc = 0.0;
        for (int j = 0; j < s; ++j) acc += A[s][j] * k[j][i];
        y[i] = u[i] + h * acc;
      }
      f(y, tau + c[s] * h, k[s], aux);
    }
    std::memcpy(un, y, sizeof(double) * 7);
    std::memcpy(k9, k[8], sizeof(double) * 7);
    static constexpr double e[9] = {V::e1, 0, 0, V::e4, V::e5, V::e6, V::e7, V::e8, V::e9};
    double acc2 = 0.0;
    for (int i = 0; i < 7; ++i) {
      double ei = 0.0;
      for (int j = 0; j < 9; ++j) ei += e[j] * k[j][i];
      ei *= h;
      const double sc = P.abstol + std::max(std::fabs(u[i]), std::fabs(un[i])) * P.reltol;
      acc2 += (ei / sc) * (ei / sc);
    }
    return std::sqrt(acc2 / 7.0);
  }

  double initdt(double* u0, const double* f0, double tau0, double dtmax) {
    double d0 = 0.0, d1 = 0.0;
    for (int i = 0; i < 7; ++i) {
      const double sk = P.abstol + std::fabs(u0[i]) * P.reltol;
      d0 += (u0[i] / sk) * (u0[i] / sk);
      d1 += (f0[i] / sk) * (f0[i] / sk);
    }
    d0 = std::sqrt(d0 / 7.0);
    d1 = std::sqrt(d1 / 7.0);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * (d0 / d1);
    dt0 = std::min(dt0, dtmax);
    const double eps_t = std::nextafter(std::fabs(tau0), INFINITY) - std::fabs(tau0);
    if (dt0 < 10 * eps_t) return std::max(1e-6, P.dtmin);
    double u1[7], f1[7], aux[2];
    for (int i = 0; i < 7; ++i) u1[i] = u0[i] + dt0 * f0[i];
    f(u1, tau0 + dt0, f1, aux);
    double d2 = 0.0;
    bool same = true;
    for (int i = 0; i < 7; ++i) {
      const double sk = P.abstol + std::fabs(u0[i]) * P.reltol;
      d2 += ((f1[i] - f0[i]) / sk) * ((f1[i] - f0[i]) / sk);
      same = same && f0[i] == f1[i];
    }
    if (same) return std::max(P.dtmin, 100 * dt0);
    d2 = std::sqrt(d2 / 7.0) / dt0;
    const double mx = std::max(d1, d2);
    const double dt1 = (mx <= 1e-15) ? std::max(1e-6, dt0 * 1e-3) : std::pow(10.0, -(2.0 + std::log10(mx)) / 6.0);
    return std::max(P.dtmin, std::min(std::min(100 * dt0, dt1), dtmax));
  }

  static void hermite(const double* u0, const double* f0, const double* u1, const double* f1, double h, double th,
                      double* out) {
    for (int i = 0; i < 7; ++i)
      out[i] = (1 - th) * u0[i] + th * u1[i] +
               th * (th - 1) * ((1 - 2 * th) * (u1[i] - u0[i]) + (th - 1) * h * f0[i] + th * h * f1[i]);
  }
  double cond(const double* u, double tau) const { return condition(P, u, tau); }

  double illinois_interp(const double* u0, const double* f0, const double* u1, const double* f1, double tau,
                         double h, double tha, double thb, double ca, double cb) const {
    double tr = tha - ca * (thb - tha) / (cb - ca);
    int side = 0;
    for (int it = 0; it < 40; ++it) {
      double ui[7];
      hermite(u0, f0, u1, f1, h, tr, ui);
      const double cr = cond(ui, tau + tr * h);
      if (cr == 0.0 || std::isnan(cr) || (thb - tha) < 1e-12) break;
      if (sgn(cr) == sgn(ca)) { tha = tr; ca = cr; if (side == -1) cb *= 0.5; side = -1; }
      else { thb = tr; cb = cr; if (side == 1) ca *= 0.5; side = 1; }
      const double tn = tha - ca * (thb - tha) / (cb - ca);
      if (tn == tr) break;
      tr = tn;
    }
    return tr;
  }

  // affect! (RayTracer.jl:301-350): 0 skip, 1 recorded, 2 recorded + terminate
  int affect(const double* u, double tau) {
    double x[3], k[3];
    back_transform(P, u, erg, x, k);
    if (count == 0) {
      bool lt = true, gt = true;
      for (int i = 0; i < 3; ++i) {
        lt = lt && std::fabs(x[i]) < std::fabs(x0c[i]) * 1.0001;
        gt = gt && std::fabs(x[i]) > std::fabs(x0c[i]) / 1.0001;
      }
      if (lt && gt) return 0;
    }
    if (std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) < P.rNS101) return 0;
    if (count == 0) {
      for (int i = 0; i < 3; ++i) { xc[i] = x[i]; xc[3 + i] = k[i]; }
      xc[6] = std::exp(tau);
      xc[7] = u[6] / erg;
      double pos[3] = {x[0], x[1], x[2]}, kp[3] = {k[0], k[1], k[2]};
      xp = prob_nonad_single(P, pos, kp, erg * std::fabs(xc[7]));
    }
    count += 1;
    const int maxc = max_crossings <= 0 ? -1 : max_crossings;
    return count >= maxc ? 2 : 1;
  }

  int run(double* u, double& tau, int& n_acc, int& n_rej) {
    const double tend = P.ln_t_end;
    const bool cbs = max_crossings != ART_NO_CALLBACKS;
    double fcur[7], aux[2];
    f(u, tau, fcur, aux);
    double bstart = NAN;
    double dt = initdt(u, fcur, tau, tend - tau);
    const double dtmax = tend - tau;
    double qold = 1e-4;
    const double beta1 = 7.0 / 60.0, beta2 = 1.0 / 15.0, gam = 0.9, qmin = 0.2, qmax = 10.0;
    double cprev = cond(u, tau);
    int sprev = std::isnan(cprev) ? 0 : sgn(cprev);
    bool just_evented = false;
    n_acc = n_rej = 0;
    const int npts = P.interp_points;
    for (int64_t iter = 0;; ++iter) {
      if (tau >= tend) return ART_STATUS_SUCCESS;
      if (iter >= P.maxiters) return ART_STATUS_MAXITERS;
      CPU_SAME_ATTEMPT_HOOK(n_acc + n_rej, tau, u, dt);
      double h = dt;
      bool last = false, forced = false;
      if (tau + h >= tend) { h = tend - tau; last = true; }
      if (h < P.dtmin && !last) { h = P.dtmin; forced = true; }
      double un[7], fn[7], aux1[2];
      const double EEst = vern6(u, fcur, tau, h, un, fn, aux1);
      bool finite = std::isfinite(EEst);
      for (int i = 0; i < 7; ++i) finite = finite && std::isfinite(un[i]);
      if (!finite) return ART_STATUS_NONFINITE;
      double q = 1.0 / qmax, q11 = 1.0;
      if (EEst != 0.0) {
        q11 = std::pow(EEst, beta1);
        q = std::max(1.0 / qmax, std::min(1.0 / qmin, q11 / std::pow(qold, beta2) / gam));
      }
      if (!(EEst <= 1.0) && !forced) {
        dt = h / std::min(1.0 / qmin, q11 / gam);
        ++n_rej;
        continue;
      }
      ++n_acc;
      qold = std::max(EEst, 1e-4);
      const double dtnext = h / q;
      // the ContinuousCallback scan (:357-358): certified steps need no grid point
      int code = (cbs && photon) ? scan_certified_code(P, u, fcur, un, fn, h, aux1[0], aux1[1], bstart) : 0;
      if (code == 1 || code == 2) {
        const int s = code == 1 ? 1 : -1;
        if (sprev != 0 && s != sprev) code = 0;  // a change at the first grid point: scan it
      }
      double last_c = cprev, last_th = 0.0;
      int last_s = sprev;
      bool evented = false;
      if (code == 3) {
        last_s = 0;  // all NaN: the sign memory resets
      } else if (code != 0) {
        last_s = code == 1 ? 1 : -1;
        last_th = 1.0;
        last_c = NAN;  // (its value is needed only by a bracket, which a certified step cannot open)
      } else {
        for (int ip = 1; cbs && ip < npts && !evented; ++ip) {
          const double th = double(ip) / double(npts - 1);
          double ui[7];
          hermite(u, fcur, un, fn, h, th, ui);
          const double ci = cond(ui, tau + th * h);
          if (std::isnan(ci)) { last_s = 0; continue; }
          const int si = sgn(ci);
          if (!(last_s != 0 && si != 0 && si != last_s)) {
            if (si != 0) { last_s = si; last_c = ci; last_th = th; }
            continue;
          }
          double ca = last_c;
          if (std::isnan(ca)) {  // the bracket's start value after a certified step
            double ua[7];
            hermite(u, fcur, un, fn, h, last_th, ua);
            ca = cond(ua, tau + last_th * h);
          }
          const double t_int = illinois_interp(u, fcur, un, fn, tau, h, last_th, th, ca, ci);
          if (just_evented && t_int < 0.01) { last_s = si; last_c = ci; last_th = th; continue; }
          // polish on the true trajectory by re-stepping (Newton with the interpolant's slope, then Illinois)
          double tha = last_th, cA = ca, thb = th, cB = ci, t = t_int;
          if (!(t > tha && t < thb)) t = 0.5 * (tha + thb);
          const double slope = (cB - cA) / (thb - tha);
          int side = 0;
          double ur[7], fr[7], auxr[2];
          for (int rit = 1;; ++rit) {
            vern6(u, fcur, tau, t * h, ur, fr, auxr);
            const double c1 = cond(ur, tau + t * h);
            if (!(std::fabs(c1) > 1e-12)) break;
            if (sgn(c1) == sgn(cA)) { tha = t; cA = c1; if (side == -1) cB *= 0.5; side = -1; }
            else { thb = t; cB = c1; if (side == 1) cA *= 0.5; side = 1; }
            if ((thb - tha) * h < 1e-13 || rit >= 9) break;
            double tn = (rit == 1) ? t - c1 / slope : tha - cA * (thb - tha) / (cB - cA);
            if (!(tn > tha && tn < thb)) tn = 0.5 * (tha + thb);
            t = tn;
          }
          const double tau_r = tau + t * h;
          const int a = affect(ur, tau_r);
          std::memcpy(u, ur, sizeof(double) * 7);
          std::memcpy(fcur, fr, sizeof(double) * 7);
          tau = tau_r;
          cprev = ci;
          sprev = si;
          bstart = auxr[0];
          just_evented = true;
          evented = true;
          if (a == 2) return ART_STATUS_CROSSING;
          if (photon && u[0] < P.rNS101) return ART_STATUS_HIT_NS;
          dt = std::min(dtnext, dtmax);
        }
      }
      if (evented) continue;
      std::memcpy(u, un, sizeof(double) * 7);
      std::memcpy(fcur, fn, sizeof(double) * 7);
      bstart = aux1[0];
      tau = last ? tend : tau + h;
      cprev = last_c;  // (NaN after a certified step: evaluated at th = 0 if a bracket opens there)
      sprev = last_s;
      just_evented = false;
      if (cbs && photon && u[0] < P.rNS101) return ART_STATUS_HIT_NS;
      if (last) return ART_STATUS_SUCCESS;
      dt = std::min(dtnext, dtmax);
    }
  }
};

}  // namespace

extern "C" {
// art_propagate_host's arguments and SoA layout (include/art.h), crossing capacity 1.
void cpu_same_propagate(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                        const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                        double* x_end, double* k_end, double* u7_end, double* tau_end, int32_t* status,
                        int32_t* n_accept, int32_t* n_reject, int32_t* n_cross, double* xc_pos, double* xc_k,
                        double* xc_t, double* xc_dw, double* xc_p, int32_t nthreads) {
  const KParams P = make_kparams(*p);
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
  for (int64_t i = 0; i < n; ++i) {
    CPU_SAME_RAY_HOOK(i);
    const double xi[3] = {x0[i], x0[n + i], x0[2 * n + i]}, ki[3] = {k0[i], k0[n + i], k0[2 * n + i]};
    const bool photon = species[i] != ART_AXION;
    double u[7];
    initial_state(P, xi, ki, erg[i], dw[i], u);
    Segment seg(P, photon, erg[i], xi, max_crossings);
    double tau = ln_t0[i];
    int na = 0, nr = 0;
    const int st = seg.run(u, tau, na, nr);
    double xe[3], ke[3];
    back_transform(P, u, erg[i], xe, ke);
    for (int c = 0; c < 3; ++c) {
      x_end[c * n + i] = xe[c];
      k_end[c * n + i] = ke[c];
      xc_pos[c * n + i] = seg.xc[c];
      xc_k[c * n + i] = seg.xc[3 + c];
    }
    u7_end[i] = u[6];
    tau_end[i] = tau;
    status[i] = st;
    n_accept[i] = na;
    n_reject[i] = nr;
    n_cross[i] = seg.count;
    xc_t[i] = seg.xc[6];
    xc_dw[i] = seg.xc[7];
    xc_p[i] = seg.xp;
  }
}
}
