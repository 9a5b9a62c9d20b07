// Dev: statistics of the sampler's 0.5 km scan steps (find_samples_new, RayTracer.jl:1547-1613)
// on the host, one line at a time, with sample_kernel's certificates: how many steps need
// their 19 grid points, how many of those hold a sign change, and how far the others stay
// from zero against the condition's slope along the line -- the data for a tighter
// certificate. Host build of the product header (art_core.h); never part of the product.
// Build: hipcc -O2 -std=c++17 tools/sampler_steps.cpp -o tools/build/sampler_steps
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../adiabatic_raytracer_amd/csrc/art_core.h"

using namespace art;

static double rmin2_line(const double* x0, const double* va, double s0, double s1) {
  const double sd = -(x0[0] * va[0] + x0[1] * va[1] + x0[2] * va[2]);
  const double sm = std::fmin(std::fmax(sd, s0), s1);
  double r2 = 0;
  for (int i = 0; i < 3; ++i) r2 += (x0[i] + va[i] * sm) * (x0[i] + va[i] * sm);
  return r2;
}

int main(int argc, char** argv) {
  const long nrays = argc > 1 ? atol(argv[1]) : 20000;
  const double theta_m = argc > 2 ? atof(argv[2]) : 0.2;
  const double mass_a = argc > 3 ? atof(argv[3]) : 1e-5;
  const double B0 = argc > 4 ? atof(argv[4]) : 1e14;
  art_params p{};
  p.theta_m = theta_m; p.omega_pul = 1.0; p.B0 = B0; p.rNS = 10.0; p.mass_ns = 1.0; p.mass_a = mass_a;
  p.g_agg = 1e-12; p.bndry_lyr = -1.0; p.ln_t_end = 0.0; p.abstol = 1e-6; p.reltol = 1e-7; p.dtmin = 1e-13;
  p.maxiters = 100000; p.flat = 1; p.isotropic = 0; p.melrose = 1; p.integrator = ART_VERN6; p.n_fixed = 2000;
  p.interp_points = 50;
  const KParams P = make_kparams(p);
  // Find_Conversion_Surface (art_find_conversion_surface)
  const double th = p.theta_m < PI / 2.0 ? p.theta_m / 2.0 : (p.theta_m + PI) / 2.0;
  const double xs[3] = {p.rNS * std::sin(th), 0.0, p.rNS * std::cos(th)};
  const double r = std::sqrt(xs[0] * xs[0] + xs[2] * xs[2]);
  const double t = std::acos(xs[2] / r);
  const double Bn = p.B0 * std::pow(p.rNS / r, 3) / 2.0;
  const double Br = 2.0 * Bn * (std::cos(p.theta_m) * std::cos(t) + std::sin(p.theta_m) * std::sin(t));
  const double Bt = Bn * (std::cos(p.theta_m) * std::sin(t) - std::sin(p.theta_m) * std::cos(t));
  const double Bz = Br * std::cos(t) - Bt * std::sin(t);
  const double ne = std::fabs(2.0 * p.omega_pul * Bz / std::sqrt(4 * PI / 137) * 1.95e-2 * HBAR);
  const double wp = std::sqrt(4 * PI * ne / 137 / 5.0e5);
  const double maxR = p.rNS * std::pow(wp / p.mass_a, 2.0 / 3.0) * 1.01;
  const double send = 2.2 * maxR;
  const int nsteps = (int)std::ceil(send / 0.5);
  const int np = 20, nper = 19;
  const double cert_lhs = 2.0 * P.wp2n, cert_rhs = P.mass_a2 * (1.0 - 1e-6);
  long attempts = 0, steps = 0, cert_old = 0, cert_tight = 0, unc = 0, unc_br = 0, samples = 0;
  // no-bracket uncertified steps: margin m = (|c_a| + |c_b|) / (Δs · slope_max) where slope_max is
  // the largest |Δc|/δ between consecutive grid points of the step; histogram of m
  const int NB = 12;
  const double edges[NB] = {0.5, 1, 1.5, 2, 3, 4, 6, 8, 12, 16, 32, 64};
  long hist[NB + 1] = {0};
  long span_hist[8] = {0};  // wave-free view: uncertified steps per attempt
  std::vector<long> unc_per_attempt;
  for (long ray = 0; ray < nrays; ++ray) {
    for (uint32_t attempt = 0;; ++attempt) {
      double U[10];
      attempt_uniforms(1769, (uint64_t)ray, attempt, U);
      const double cti = 1.0 - 2.0 * U[0], sti = std::sin(std::acos(cti));
      const double spi = std::sin(U[1] * 2.0 * PI), cpi = std::cos(U[1] * 2.0 * PI);
      const double ctl = 1.0 - 2.0 * U[2], stl = std::sin(std::acos(ctl));
      const double spl = std::sin(U[3] * 2.0 * PI), cpl = std::cos(U[3] * 2.0 * PI);
      const double sR = std::sin(U[4] * 2.0 * PI), cR = std::cos(U[4] * 2.0 * PI);
      const double rR = std::sqrt(U[5]) * maxR;
      const double va[3] = {sti * cpi, sti * spi, cti};
      const double vl[3] = {stl * cpl, stl * spl, ctl};
      const double x1 = rR * cR, x2 = rR * sR;
      double x0[3] = {x1 * cpi * cti - x2 * spi, x2 * cpi + x1 * spi * cti, -x1 * sti};
      double vI[3];
      for (int i = 0; i < 3; ++i) vI[i] = (220.0 + U[6 + i] * 1.0e-5) / std::sqrt(3.0);
      const double vmag = std::sqrt(vI[0] * vI[0] + vI[1] * vI[1] + vI[2] * vI[2]);
      const double gammaA = 1.0 / std::sqrt(1.0 - (vmag / C_KM) * (vmag / C_KM));
      const double E = P.mass_a * std::sqrt(1.0 + (vmag / C_KM * gammaA) * (vmag / C_KM * gammaA));
      const double iE2 = 1.0 / (E * E);
      for (int i = 0; i < 3; ++i) x0[i] += va[i] * (-maxR * 1.1);
      int randInx = 1 + (int)(U[9] * 6.0);
      if (randInx > 6) randInx = 6;
      ++attempts;
      auto cond = [&](double s) {
        double x[3];
        for (int i = 0; i < 3; ++i) x[i] = x0[i] + va[i] * s;
        return sampler_condition_e(P, x, vl, E, iE2);
      };
      double c_prev = cond(0.0);
      int count = 0;
      long unc_here = 0;
      for (int st = 0; st < nsteps; ++st) {
        ++steps;
        const double s0 = st * 0.5, s1 = std::fmin(s0 + 0.5, send);
        bool c1 = false, c2 = false;
        const double rm2 = rmin2_line(x0, va, s0, s1), rmin = std::sqrt(rm2);
        double xa[3], xb[3];
        for (int i = 0; i < 3; ++i) { xa[i] = x0[i] + va[i] * s0; xb[i] = x0[i] + va[i] * s1; }
        const double ra2 = xa[0] * xa[0] + xa[1] * xa[1] + xa[2] * xa[2];
        const double rb2 = xb[0] * xb[0] + xb[1] * xb[1] + xb[2] * xb[2];
        const double ba = (P.cm * (3.0 * xa[2] * xa[2] - ra2) + 3.0 * P.sm * xa[0] * xa[2]) / ra2;
        const double bb = (P.cm * (3.0 * xb[2] * xb[2] - rb2) + 3.0 * P.sm * xb[0] * xb[2]) / rb2;
        if (c_prev != 0.0 && !std::isnan(c_prev)) {
          const double db = (3.0 + 3.0 * std::fabs(P.sm)) * (s1 - s0) / rmin * (1.0 + 1e-9) + 1e-9;
          const double al = (s1 - s0) / rmin;
          const double db2 = 0.75 * al * al * (1.0 + 1e-9) + 1e-12;  // quadratic form on a great-circle arc
          if (c_prev < 0.0) {
            c1 = cert_lhs * 0.5 * std::fmin(2.0, std::fabs(ba) + db) < cert_rhs * (rm2 * rmin);
            c2 = cert_lhs * 0.5 * std::fmin(2.0, std::fmax(std::fabs(ba), std::fabs(bb)) + db2) < cert_rhs * (rm2 * rmin);
          } else if (rmin > 10.0) {
            const double rmax2 = std::fmax(ra2, rb2), grr = 1.0 - P.rs_gr / rmin;
            const double bmin = std::fabs(ba) - db;
            c1 = bmin > 0.0 && P.wp2n * bmin * grr > E * E * (1.0 + 1e-6) * (rmax2 * std::sqrt(rmax2));
            const double bmin2 = (ba * bb > 0.0) ? std::fmin(std::fabs(ba), std::fabs(bb)) - db2 : -1.0;
            c2 = bmin2 > 0.0 && P.wp2n * bmin2 * grr > E * E * (1.0 + 1e-6) * (rmax2 * std::sqrt(rmax2));
          }
        }
        cert_old += c1;
        cert_tight += c2;
        double v[20];
        v[0] = c_prev;
        for (int j = 1; j < np; ++j) v[j] = cond(s0 + (s1 - s0) * double(j) / double(np - 1));
        bool br = false;
        double slope = 0.0;
        for (int j = 1; j < np; ++j) {
          if (std::signbit(v[j]) != std::signbit(v[j - 1]) && v[j] != 0.0 && v[j - 1] != 0.0) br = true;
          slope = std::fmax(slope, std::fabs(v[j] - v[j - 1]) / ((s1 - s0) / nper));
        }
        if (!(c1 || c2)) {
          ++unc;
          ++unc_here;
          if (br) ++unc_br;
          else {
            const double m = (std::fabs(v[0]) + std::fabs(v[nper])) / ((s1 - s0) * slope);
            int b = 0;
            while (b < NB && m > edges[b]) ++b;
            ++hist[b];
          }
        }
        if (c1 || c2) {  // a certified step: every grid value has the sign of the point before
          for (int j = 1; j < np; ++j)
            if (std::signbit(v[j]) != std::signbit(v[0]) || v[j] == 0.0) {
              std::printf("BUG: certified step (old %d tight %d) with value %g at point %d\n", c1, c2, v[j], j);
              return 1;
            }
        }
        if (br) {  // count valid crossings exactly as flush() (Illinois + affect!)
          for (int j = 1; j < np; ++j) {
            if (!(std::signbit(v[j]) != std::signbit(v[j - 1]) && v[j] != 0.0 && v[j - 1] != 0.0)) continue;
            double a = s0 + (s1 - s0) * double(j - 1) / double(np - 1), b = s0 + (s1 - s0) * double(j) / double(np - 1);
            double fa = cond(a), fb = cond(b), root = b;
            int side = 0;
            for (int it = 0; it < 100; ++it) {
              root = a - fa * (b - a) / (fb - fa);
              const double fr = cond(root);
              if (fr == 0.0 || (b - a) < 1e-13 * std::fmax(1.0, std::fabs(root))) break;
              if (std::signbit(fr) == std::signbit(fa)) { a = root; fa = fr; if (side == -1) fb *= 0.5; side = -1; }
              else { b = root; fb = fr; if (side == 1) fa *= 0.5; side = 1; }
            }
            double xr[3];
            for (int i = 0; i < 3; ++i) xr[i] = x0[i] + va[i] * root;
            const double rr = std::sqrt(xr[0] * xr[0] + xr[1] * xr[1] + xr[2] * xr[2]);
            double gtt, grr;
            metric_tr(rr, P.rs_gr, gtt, grr);
            if (rr > P.rNS && E / std::sqrt(grr) > wp_cart(P, xr)) ++count;
          }
        }
        c_prev = v[nper];
      }
      unc_per_attempt.push_back(unc_here);
      int hb = unc_here == 0 ? 0 : unc_here < 5 ? 1 : unc_here < 10 ? 2 : unc_here < 20 ? 3 : unc_here < 40 ? 4 : unc_here < 80 ? 5 : 6;
      ++span_hist[hb];
      if (count >= randInx || attempt + 1 >= 1000000u) { ++samples; break; }
    }
  }
  std::printf("{\"maxR\": %.4f, \"nsteps\": %d, \"rays\": %ld, \"attempts\": %ld, \"steps\": %ld, \"cert_old\": %ld, "
              "\"cert_tight\": %ld, \"uncertified\": %ld, \"uncertified_with_bracket\": %ld, \"margin_hist_edges\": [",
              maxR, nsteps, nrays, attempts, steps, cert_old, cert_tight, unc, unc_br);
  for (int b = 0; b < NB; ++b) std::printf("%s%g", b ? ", " : "", edges[b]);
  std::printf("], \"margin_hist\": [");
  for (int b = 0; b <= NB; ++b) std::printf("%s%ld", b ? ", " : "", hist[b]);
  std::printf("], \"unc_per_attempt_hist(0,<5,<10,<20,<40,<80,>=80)\": [");
  for (int b = 0; b < 7; ++b) std::printf("%s%ld", b ? ", " : "", span_hist[b]);
  std::printf("]}\n");
  return 0;
}
