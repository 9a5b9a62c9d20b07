// art_core.h -- physics of the adiabatic axion<->photon ray-tracing hot path for CDNA4.
//
// Every function restates a reference function of SamWitte/Adiabatic_RayTracer
// (file:line under /root/reference/src). Gradients that the reference takes with
// ForwardDiff dual numbers (RayTracer.jl:21,24,84-88,1427-1432) are HAND-DERIVED here:
// one fused pass yields H's 7 partial derivatives with ~5x fewer operations than the
// reference's three dual-number passes, and no transcendental is evaluated twice.
//
// Everything is templated on the scalar type T so the same source compiles
//   * as T = double in the gfx950 kernels (art_kernels.hip), and
//   * as an op-counting type on the host (tools/count_flops.cpp) -- the
//     "instrumented restatement" that fixes the algorithmic FLOPs per ray-step.
// Branch conditions compare T against doubles, so the counting type carries a value.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/art.h"

// FMA contraction. libart.so is compiled with -ffp-contract=on: a multiply and an add are
// fused only inside one source expression, so a shared function rounds the same in every
// kernel it is inlined into (the bulk integrator and the one-wave-per-ray tail kernel must
// agree bit for bit; with the backend's cross-statement fusion ("fast") the choice depends on
// how many uses each product has at the inlined site, and it differed between the two in the
// scan and the back-transform). The ray equations' right-hand side keeps "fast" contraction
// (ART_FP_FAST at the top of its functions): it is 2% of the headline kernel's time faster
// that way, and its roundings were checked equal between the kernels (the ART_TRACE per-attempt build; the trace tools are in git history).
#if defined(__clang__)
#define ART_FP_FAST _Pragma("clang fp contract(fast)")
#else
#define ART_FP_FAST
#endif

// ART_EXP_ASM (off by default): three-operand FMA Horner steps in exp_fma and a
// one-instruction radius clamp in inline asm. The backend otherwise keeps the polynomial's
// coefficients in VGPRs and copies one into the accumulator before every two-address
// v_fmac_f64. 1e7 flat rays: 84.34 -> 83.37 ms (profiles/r04b_ab.txt), but (1) the tail kernel
// and the persistent integrator then no longer agree bit for bit (tests/test_edges.py,
// test_gpu_tail_donation.py, profiles/r04d_bitexact.log) and (2) the streamed instantiation's
// register allocation gets worse (100.8 -> 117.6 ms, profiles/r04d_stream_ab.jsonl). Not kept.

namespace art {

// Constants.jl:3-5
constexpr double C_KM = 2.99792e5;
constexpr double HBAR = 6.582119e-16;
constexpr double GNEW = 132712000000.0;
constexpr double PI = 3.141592653589793;

// ---- scalar math for T = double (the op-counting type provides its own overloads) ----
__host__ __device__ inline double msqrt(double x) { return sqrt(x); }
__host__ __device__ inline double mexp(double x) { return exp(x); }
__host__ __device__ inline double mabs(double x) { return fabs(x); }
__host__ __device__ inline double msign(double x) { return copysign(1.0, x); }  // ForwardDiff abs: signbit
// sin and cos together: FMA Cody-Waite reduction by π/2 (3 parts) + the fdlibm kernels on
// [-π/4, π/4]; <= 1 ulp against glibc for |x| <= 200 (tests/test_corecheck.py). The ray's
// angles θ and ψ = φ - ωt stay small, so the large-argument (Payne-Hanek) path that
// ocml's sincos carries -- ~200 instructions of code per call site -- is never needed.
__host__ __device__ inline void msincos(double x, double& s, double& c) {
  ART_FP_FAST
  const double n = rint(x * 0.63661977236758134308);
  double r = fma(-n, 1.5707963267948966, x);
  r = fma(-n, 6.123233995736766e-17, r);
  r = fma(-n, -1.4973849048591698e-33, r);
  const double z = r * r;
  const double ps = 8.33333333332248946124e-03 +
                    z * (-1.98412698298579493134e-04 +
                         z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
  const double sr = r + r * z * (-1.66666666666666324348e-01 + z * ps);
  const double pc =
      z * (4.16666666666666019037e-02 +
           z * (-1.38888888888741095749e-03 +
                z * (2.48015872894767294178e-05 +
                     z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cr = w + (((1.0 - w) - hz) + z * pc);
  const int q = ((int)n) & 3;
  const double ss = (q & 1) ? cr : sr;
  const double cc = (q & 1) ? sr : cr;
  // the quadrant's signs by flipping the sign bit (an XOR of the high word instead of a
  // compare and a select of both words): -x exactly
  const unsigned long long ms = (unsigned long long)(q & 2) << 62, mc = (unsigned long long)((q + 1) & 2) << 62;
  s = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, ss) ^ ms);
  c = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, cc) ^ mc);
}
// max(|a|, |b|), min(a, b) and max(a, b) as one instruction each. LLVM's fmax/fmin in IEEE
// mode first quiet signaling NaNs with a v_max x, x per operand it cannot prove canonical
// (anything loaded or passed in); the integrator never holds signaling NaNs, and a quiet NaN
// operand gives the other operand either way.
__host__ __device__ inline double fmax_abs(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fmax(fabs(a), fabs(b));
#endif
}
__host__ __device__ inline double fmin_q(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fmin(a, b);
#endif
}
__host__ __device__ inline double fmax_q(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fmax(a, b);
#endif
}
// The radius clamped to rNS (:531): max(r, rNS) for the double path (one v_max_f64 instead
// of a compare and two selects; a NaN radius gives rNS here, and the NaN state itself is
// what the integrator reports), the select for the op-counting and dual types.
__host__ __device__ inline double rclamp(double r, double rns) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(ART_EXP_ASM)
  double m;
  asm("v_max_f64 %0, %1, %2" : "=v"(m) : "v"(r), "s"(rns));
  return m;
#else
  return fmax(r, rns);
#endif
}
template <class T>
__host__ __device__ inline T rclamp(const T& r, double rns) {
  return (r < rns) ? T(rns) : r;
}
// 1/x from the hardware reciprocal and two Newton steps (~0.5 ulp; 1/0 and 1/inf give NaN,
// which the integrator reports as a non-finite state either way). The host build, which the
// CPU tests compare with the oracle, divides.
__host__ __device__ inline double frcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
#else
  return 1.0 / x;
#endif
}
// e^x in 19 FMA-pipe instructions (ocml's exp_f64: 34): Cody-Waite reduction by ln 2 with a
// two-part constant (the first FMA is exact for |k| < 2^11), the degree-13 Taylor polynomial
// on |r| <= ln2/2 (truncation < 0.05 ulp) and one ldexp. <= 1 ulp for |x| < 708
// (tests/test_corecheck.py); no overflow/underflow/NaN special-casing beyond what the
// arithmetic propagates (the integrator's arguments are moderate ln t and ln EEst values).
// Horner step p r + c as one three-operand v_fma_f64 (the backend otherwise picks the two-
// address v_fmac_f64 with the coefficient copied into the accumulator: a v_mov_b64 per step)
__host__ __device__ inline double horner_fma(double p, double r, double c) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(ART_EXP_ASM)
  double o;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(o) : "v"(p), "v"(r), "v"(c));
  return o;
#else
  return fma(p, r, c);
#endif
}
__host__ __device__ inline double exp_fma(double x) {
  ART_FP_FAST
  const double k = rint(x * 1.4426950408889634);
  double r = fma(-k, 0.6931471805599453, x);
  r = fma(-k, 2.3190468138462996e-17, r);
  double p = 1.0 / 6227020800.0;  // 1/13!
  p = horner_fma(p, r, 1.0 / 479001600.0);
  p = horner_fma(p, r, 1.0 / 39916800.0);
  p = horner_fma(p, r, 1.0 / 3628800.0);
  p = horner_fma(p, r, 1.0 / 362880.0);
  p = horner_fma(p, r, 1.0 / 40320.0);
  p = horner_fma(p, r, 1.0 / 5040.0);
  p = horner_fma(p, r, 1.0 / 720.0);
  p = horner_fma(p, r, 1.0 / 120.0);
  p = horner_fma(p, r, 1.0 / 24.0);
  p = horner_fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)k);
}
// ln x for finite x > 0 (the step-size controller's ln EEst): x = m 2^e with m in
// [√½, √2), ln m = 2 atanh(s), s = (m - 1)/(m + 1), |s| <= 0.1716, odd series to s^21.
// ~30 instructions against ocml's 105; <= 2 ulp (tests/test_corecheck.py).
__host__ __device__ inline double log_fma(double x) {
  int e;
  double m = frexp(x, &e);  // [0.5, 1)
  if (m < 0.70710678118654752) { m += m; e -= 1; }
  const double f = m - 1.0;
#if defined(__HIP_DEVICE_COMPILE__)
  const double d = 2.0 + f;
  double id = __builtin_amdgcn_rcp(d);
  id = fma(id, fma(-d, id, 1.0), id);
  id = fma(id, fma(-d, id, 1.0), id);
  const double s = f * id;
#else
  const double s = f / (2.0 + f);
#endif
  const double z = s * s;
  double p = 1.0 / 21.0;
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  // ln m = 2s + 2s z p; e ln2 in two parts so the sum keeps the small terms
  const double de = (double)e;
  const double lo = fma(2.0 * s * z, p, de * 2.3190468138462996e-17);
  return fma(de, 0.6931471805599453, fma(2.0, s, lo));
}
// device: exp_fma / log_fma; host (the CPU tests against the oracle): libm
__host__ __device__ inline double fexp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return exp_fma(x);
#else
  return exp(x);
#endif
}
__host__ __device__ inline double flog(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return log_fma(x);
#else
  return log(x);
#endif
}
// 1/x for the templated physics: frcp for double, a plain division for the counting and
// dual types of tools/ and oracle/
template <class T>
__host__ __device__ inline T trcp(const T& x) {
  return T(1.0) / x;
}
template <>
__host__ __device__ inline double trcp<double>(const double& x) {
  return frcp(x);
}
__host__ __device__ inline double msin(double x) { return sin(x); }
__host__ __device__ inline double mcos(double x) { return cos(x); }
__host__ __device__ inline double macos(double x) { return acos(x); }
__host__ __device__ inline double matan2(double y, double x) { return atan2(y, x); }
__host__ __device__ inline double mpow(double x, double p) { return pow(x, p); }
__host__ __device__ inline bool misnan(double x) { return isnan(x); }
__host__ __device__ inline double mmax(double a, double b) { return a > b ? a : b; }

// Kernel-side parameters: art_params plus derived constants, passed by value (kernarg ->
// SGPRs: the NS parameters are wave-uniform scalars, never per-lane data).
struct KParams {
  double cm, sm;          // cos θm, sin θm
  double omega;           // ωPul
  double Bn_coef;         // B0 rNS^3 / 2  (B_n = Bn_coef / r^3, RayTracer.jl:1143)
  double rNS, rNS101;     // rNS, 1.01 rNS
  double rs_gr, rs_eff;   // 2 GNew M / c^2 (GR); flat ? 0 : rs_gr
  double wp2_coef;        // ωp^2 = wp2_coef |Bz| (RayTracer.jl:1153-1154)
  double wp2n;            // wp2_coef |Bn_coef|: ωp^2 = wp2n |b| / r^3 for either sign of B0
  double mass_a, mass_a2; // m_a, m_a^2
  double g_agg;
  double bndry_lyr, pole_val, rmax, rmax_def;  // boundary layer (RayTracer.jl:1155-1162)
  double GM_c2;           // GNew M / c^2 (Cristoffel, get_Prob_nonAD erg_ax)
  double ln_t_end, abstol, reltol, dtmin;
  // certified-negative resonance scan (scan_certified_negative): margin
  // factor on ωp² (+inf disables the certificate), the smallest radius it trusts (10 km in
  // GR: g_schwartz's interior patch) and m_a² with a margin
  double cert_fac, cert_rmin, cert_e2;
  int64_t maxiters;
  int32_t flat, isotropic, integrator, n_fixed, interp_points, pad;
};

inline KParams make_kparams(const art_params& p) {
  KParams k{};
  k.cm = cos(p.theta_m);
  k.sm = sin(p.theta_m);
  k.omega = p.omega_pul;
  k.Bn_coef = 0.5 * p.B0 * p.rNS * p.rNS * p.rNS;
  k.rNS = p.rNS;
  k.rNS101 = p.rNS * 1.01;
  k.rs_gr = 2.0 * GNEW * p.mass_ns / (C_KM * C_KM);
  k.rs_eff = p.flat ? 0.0 : k.rs_gr;
  const double ne_coef = fabs(2.0 * p.omega_pul / sqrt(4.0 * PI / 137.0) * 1.95e-2 * HBAR);
  k.wp2_coef = 4.0 * PI * ne_coef / 137.0 / 5.0e5;
  k.wp2n = k.wp2_coef * fabs(k.Bn_coef);  // n_e = |2 ω Bz ...| (RayTracer.jl:1153): the sign of B0 drops out
  k.mass_a = p.mass_a;
  k.mass_a2 = p.mass_a * p.mass_a;
  k.g_agg = p.g_agg;
  k.bndry_lyr = p.bndry_lyr;
  const double ne_pole = fabs(2.0 * p.omega_pul * p.B0 / sqrt(4.0 * PI / 137.0) * 1.95e-2 * HBAR);
  k.pole_val = sqrt(4.0 * PI * ne_pole / 137.0 / 5.0e5);
  k.rmax = p.rNS * pow(k.pole_val / p.mass_a, 2.0 / 3.0);
  k.rmax_def = p.rNS * pow(k.pole_val / 1e-5, 2.0 / 3.0);  // get_Prob_nonAD passes no Mass_a (:97)
  k.GM_c2 = GNEW * p.mass_ns / (C_KM * C_KM);
  // certified-negative scan: ωp² = wp2n |b| / r³ needs GJ plasma without a boundary layer
  k.cert_fac = (p.bndry_lyr > 0.0 || !(p.mass_a > 0.0)) ? __builtin_inf() : 1.0 + 1e-6;
  k.cert_rmin = k.rs_eff == 0.0 ? 0.0 : 10.0;
  k.cert_e2 = k.mass_a2 * (1.0 + 1e-9);
  k.ln_t_end = p.ln_t_end;
  k.abstol = p.abstol;
  k.reltol = p.reltol;
  k.dtmin = p.dtmin;
  k.maxiters = p.maxiters;
  k.flat = p.flat;
  k.isotropic = p.isotropic;
  k.integrator = p.integrator;
  k.n_fixed = p.n_fixed;
  k.interp_points = p.interp_points < 2 ? 2 : p.interp_points;
  return k;
}

// ---------------------------------------------------------------------------
// g_schwartz (RayTracer.jl:455-501): g^tt, g^rr and d/dr. The interior patch is switched
// on r <= 10 km, the keyword default that hot-path callers never override (:455).
template <class T>
__host__ __device__ inline void metric_tr(const T& r, double rs, T& gtt, T& grr) {
  ART_FP_FAST
  if (rs == 0.0) {  // flat space: exactly what both branches below give for rs = 0
    grr = 1.0;
    gtt = -1.0;
  } else if (r <= 10.0) {
    const T rsp = rs * (r * r * r) * 1e-3;  // rs (r/10)^3 (:463)
    grr = 1.0 - r * r * rsp * 1e-3;
    const T D = 3.0 * msqrt(1.0 - rsp * 0.1) - msqrt(grr);
    gtt = -4.0 / (D * D);
  } else {
    grr = 1.0 - rs / r;
    gtt = -1.0 / grr;
  }
}

template <class T>
__host__ __device__ inline void metric_tr_d(const T& r, double rs, T& gtt, T& grr, T& dgtt, T& dgrr) {
  ART_FP_FAST
  if (rs == 0.0) {  // flat space (wave-uniform branch): no divisions
    grr = 1.0;
    gtt = -1.0;
    dgrr = 0.0;
    dgtt = 0.0;
  } else if (r <= 10.0) {
    const T r2 = r * r;
    const T rsp = rs * (r2 * r) * 1e-3;
    grr = 1.0 - r2 * rsp * 1e-3;                  // 1 - rs r^5 / 1e6
    dgrr = -5e-6 * rs * (r2 * r2);
    const T S1 = msqrt(1.0 - rsp * 0.1);          // sqrt(1 - rs r^3 / 1e4)
    const T dS1 = (-1.5e-4 * rs * r2) / S1;
    const T S2 = msqrt(grr);
    const T dS2 = 0.5 * dgrr / S2;
    const T D = 3.0 * S1 - S2;
    const T iD = 1.0 / D;
    gtt = -4.0 * iD * iD;
    dgtt = 8.0 * (3.0 * dS1 - dS2) * iD * iD * iD;
  } else {
    const T ir = trcp(r);
    grr = 1.0 - rs * ir;
    dgrr = rs * ir * ir;
    const T ig = trcp(grr);
    gtt = -ig;
    dgtt = dgrr * ig * ig;
  }
}

// ---------------------------------------------------------------------------
// Rotating oblique dipole (RayTracer.jl:1142-1151): B = B_n (2 a1, a2, a3) with
// a1 = cosθm cosθ + sinθm sinθ cosψ, a2 = cosθm sinθ - sinθm cosθ cosψ, a3 = sinθm sinψ,
// ψ = φ - ωt, B_n = B0 (rNS/r)^3 / 2. The GJ density uses b = Bz/B_n = 2 a1 cosθ - a2 sinθ.
template <class T>
struct DipoleAng {
  T a1, a2, a3;        // angular factors
  T a1t, a1p, a2p, a3p;  // ∂θ a1, ∂φ a1, ∂φ a2, ∂φ a3  (∂θ a2 = a1, ∂θ a3 = 0)
  T b, bt, bp;         // Bz/B_n and its θ, φ derivatives
};

template <class T>
__host__ __device__ inline DipoleAng<T> dipole_ang(const KParams& P, const T& st, const T& ct, const T& sp,
                                                   const T& cp) {
  ART_FP_FAST
  DipoleAng<T> d;
  d.a1 = P.cm * ct + P.sm * st * cp;
  d.a2 = P.cm * st - P.sm * ct * cp;
  d.a3 = P.sm * sp;
  d.a1t = P.sm * ct * cp - P.cm * st;
  d.a1p = -P.sm * st * sp;
  d.a2p = P.sm * ct * sp;
  d.a3p = P.sm * cp;
  d.b = 2.0 * d.a1 * ct - d.a2 * st;
  d.bt = 2.0 * d.a1t * ct - 3.0 * d.a1 * st - d.a2 * ct;
  d.bp = 2.0 * d.a1p * ct - d.a2p * st;
  return d;
}

// Boundary-layer increment of ωp (RayTracer.jl:1158-1161), r >= rNS.
template <class T>
__host__ __device__ inline T layer_wp(const KParams& P, const T& r, double rmax) {
  ART_FP_FAST
  const T x = P.rNS / r;
  return P.pole_val * x * msqrt(x) * mexp(-(r - rmax * P.bndry_lyr) / (0.1 * rmax));
}

// ---------------------------------------------------------------------------
// func! (RayTracer.jl:71-91) with hamiltonian (:530-556, melrose=true), GJ_Model_ωp_vecSPH
// (:1120-1170), K_par (:1044-1058), g_schwartz (:455-501), all partials hand-derived:
//   H = ½[K + ωp²(1 - Q)],  K = g^tt E² + g^rr k_r² + g^θθ k_θ² + g^φφ k_φ²,
//   Q = g^rr k∥²/E²,  k∥² = p²/β,  p = 2√g^rr k_r a1 + (k_θ a2 + k_φ a3/|sinθ|)/r,
//   β = 4a1² + a2² + a3²  (|B|² = B_n² β, so B_n cancels from k∥),  ωp² = C |B_n b|.
// du[1:3] = ∂H/∂k c t g^rr/E, du[4:6] = -∂H/∂x c t g^rr/(E erg), du[7] = ∂H/∂t t g^rr/E,
// E = -u[7], k = w erg; rows 1..6 zeroed for r <= 1.01 rNS (:86); H is evaluated at the
// radius clamped to rNS (:531) while the prefactor's g^rr uses the raw radius (:82).
// bndry_lyr enters only the ∂t pass (:84-88).
template <class T>
__host__ __device__ inline void rhs_photon(const KParams& P, const T* u, const T& tau, double erg, T* du,
                                           T* aux = nullptr) {
  ART_FP_FAST
  const T t = fexp(tau);
  const T r = u[0];
  const T E = -u[6];
  const T rc = (r < P.rNS) ? T(P.rNS) : r;
  T st, ct, sp, cp;
  msincos(u[1], st, ct);
  msincos(u[2] - P.omega * t, sp, cp);  // ψ = φ - ω (time0 + t), time0 = 0 (MainRunner.jl:177)
  const T ast = mabs(st);
  const T sgn_st = msign(st);
  const T kr = u[3] * erg, kt = u[4] * erg, kp = u[5] * erg;
  // one division for 1/r, 1/|sinθ|, 1/E and 1/erg (it needs only r, θ and u7, so it does not
  // wait for ψ: a lone long ray is latency-bound), and one for 1/β
  const T X1 = rc * ast, X2 = E * erg;
  const T R = frcp(X1 * X2);
  const T inv_rs = R * X2;       // 1/(r |sinθ|)
  const T iE = R * X1 * erg;     // 1/E
  const T ierg = R * X1 * E;     // 1/erg
  const DipoleAng<T> d = dipole_ang(P, st, ct, sp, cp);
  const T ibeta = frcp(4.0 * d.a1 * d.a1 + d.a2 * d.a2 + d.a3 * d.a3);  // |B|²/B_n² = 1 + 3 a1² >= 1
  const T ir = inv_rs * ast;
  const T ir2 = ir * ir;
  const T iast = inv_rs * rc;
  const T sgb = msign(d.b);
  const T cB = P.wp2n * ir2 * ir;               // ∂ωp² = cB sgn(b) ∂b, ωp² ∝ r^-3
  const T wp2 = cB * mabs(d.b);
  const T dwp2_r = -3.0 * wp2 * ir;
  const T dwp2_t = cB * sgb * d.bt;
  const T dwp2_p = cB * sgb * d.bp;
  T gtt, grr, dgtt, dgrr;
  metric_tr_d(rc, P.rs_eff, gtt, grr, dgtt, dgrr);
  // the prefactor's g^rr at the raw radius (:82) differs from the clamped one only inside the
  // star: a second metric evaluation only for lanes there
  T grr_u = grr;
  if (!(P.rs_eff == 0.0) && r < P.rNS) {
    T gtt_u;
    metric_tr(r, P.rs_eff, gtt_u, grr_u);
  }
  const T gpp = ir2 * iast * iast;
  const T E2 = E * E;
  const T iE2 = iE * iE;
  const bool flat = P.rs_eff == 0.0;  // wave-uniform: g^rr = 1, ∂g^rr = 0
  const T sq = flat ? T(1.0) : msqrt(grr);
  // k∥ part (vanishes for isotropic plasma, kpar = 0)
  T Q = 0.0, Q_r = 0.0, Q_t = 0.0, Q_p = 0.0, Q_kr = 0.0, Q_kt = 0.0, Q_kp = 0.0;
  if (!P.isotropic) {
    const T pa = kt * d.a2 + kp * d.a3 * iast;
    const T p = 2.0 * sq * kr * d.a1 + ir * pa;
    const T G = grr * p * ibeta * iE2;  // Q = G p
    Q = G * p;
    const T p_r = flat ? -ir2 * pa : dgrr / sq * kr * d.a1 - ir2 * pa;
    const T p_t = 2.0 * sq * kr * d.a1t + ir * (kt * d.a1 - kp * d.a3 * sgn_st * ct * iast * iast);
    const T p_p = 2.0 * sq * kr * d.a1p + ir * (kt * d.a2p + kp * d.a3p * iast);
    const T beta_t = 8.0 * d.a1 * d.a1t + 2.0 * d.a2 * d.a1;
    const T beta_p = 8.0 * d.a1 * d.a1p + 2.0 * d.a2 * d.a2p + 2.0 * d.a3 * d.a3p;
    Q_r = dgrr * p * p * ibeta * iE2 + 2.0 * G * p_r;
    Q_t = 2.0 * G * p_t - Q * beta_t * ibeta;
    Q_p = 2.0 * G * p_p - Q * beta_p * ibeta;
    const T G2 = 2.0 * G;
    Q_kr = G2 * 2.0 * sq * d.a1;
    Q_kt = G2 * ir * d.a2;
    Q_kp = G2 * ir * d.a3 * iast;
  }
  const T omQ = 1.0 - Q;
  const T fac = C_KM * t * grr_u * iE;
  const T ir3 = ir2 * ir;
  const T H_r = 0.5 * (dgtt * E2 + dgrr * kr * kr - 2.0 * ir3 * (kt * kt + iast * iast * kp * kp) +
                       dwp2_r * omQ - wp2 * Q_r);
  const T H_t = 0.5 * (-2.0 * ct * ir2 * iast * iast * (sgn_st * iast) * kp * kp + dwp2_t * omQ - wp2 * Q_t);
  const T H_p = 0.5 * (dwp2_p * omQ - wp2 * Q_p);
  // rows 1..6 vanish for r <= 1.01 rNS (:86): one select on their common factor
  const T facx = (r <= P.rNS101) ? T(0.0) : fac;
  const T fx = -facx * ierg;
  du[0] = (grr * kr - 0.5 * wp2 * Q_kr) * facx;
  du[1] = (ir2 * kt - 0.5 * wp2 * Q_kt) * facx;
  du[2] = (gpp * kp - 0.5 * wp2 * Q_kp) * facx;
  du[3] = H_r * fx;
  du[4] = H_t * fx;
  du[5] = H_p * fx;
  // ∂H/∂t = -ω ∂H/∂ψ (K is static); with a boundary layer ωp² -> (sqrt(ωp²) + L)²
  T dwp2_T = -P.omega * dwp2_p;
  T wp2_T = wp2;
  if (P.bndry_lyr > 0.0) {
    const T wgj = msqrt(wp2);
    const T wtot = wgj + layer_wp(P, rc, P.rmax);
    wp2_T = wtot * wtot;
    dwp2_T = dwp2_T * (wtot / wgj);
  }
  const T H_T = 0.5 * (dwp2_T * omQ + wp2_T * P.omega * Q_p);
  du[6] = H_T * t * grr_u * iE;
  if (aux) {  // for the scan certificate: Bz/B_n and t at this point
    aux[0] = d.b;
    aux[1] = t;
  }
}

// rhs_photon for GJ plasma without a boundary layer, anisotropic (the headline workload in
// flat space, configs[3] in Schwarzschild), with the algebra the general form leaves to the
// hardware done by hand: with a1t = ∂θ a1 = -a2, ∂θ b = -3(a2 cosθ + a1 sinθ),
// ∂φ b = 3 a1p cosθ, ∂θ β = -6 a1 a2, w = ωp² G (= ½ ωp² ∂Q/∂p) and ∂H/∂t = -ω ∂H/∂φ, the
// same derivatives as rhs_photon in about a third fewer operations (equal up to rounding;
// tests/test_gpu_pointwise.py and tests/test_corecheck.py check it against the oracle's dual
// numbers). In flat space (rs_eff == 0, compile-time in the GEOM_FLAT kernel) the metric
// terms drop out; in Schwarzschild
//   H_r += ½ ∂g^tt E² + ½ ∂g^rr k_r² - ½ ωp² ∂g^rr Q/g^rr - w ∂g^rr/√g^rr k_r a1.
// ψ = φ - ω (time0 + t), time0 = 0 (MainRunner.jl:177): the argument of rhs_photon_gj's second sincos
template <class T>
__host__ __device__ inline T psi_of(const KParams& P, const T& phi, const T& t) {
  ART_FP_FAST
  return phi - P.omega * t;
}

// A branch condition the caller knows to be wave-uniform (UNI: the one-wave-per-ray tail kernel,
// whose lanes hold the ray alike): a scalar branch on lane 0's value instead of an exec-mask
// branch; elsewhere the condition itself. The values either way are the same.
template <bool UNI>
__host__ __device__ inline bool uni_if(bool c) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (UNI) return __builtin_amdgcn_readfirstlane((int)c) != 0;
#endif
  return c;
}

// rhs_photon_gj from its transcendental inputs: t = e^τ, (sin, cos) of θ = u[1] and of ψ = psi_of(u[2], t).
// The one-ray-per-wave tail kernel evaluates the two sincos on two lanes at once and every
// stage's e^τ ahead of the stage (and takes its branches as wave-uniform, UNI); the values and
// the arithmetic here are the same.
template <class T, bool UNI = false>
__host__ __device__ inline void rhs_photon_gj_tr(const KParams& P, const T* u, const T& t, const T& st, const T& ct,
                                                 const T& sp, const T& cp, double erg, T* du, T* aux = nullptr);

template <class T>
__host__ __device__ inline void rhs_photon_gj(const KParams& P, const T* u, const T& tau, double erg, T* du,
                                              T* aux = nullptr) {
  ART_FP_FAST
  const T t = fexp(tau);
  T st, ct, sp, cp;
  msincos(u[1], st, ct);
  msincos(psi_of(P, u[2], t), sp, cp);
  rhs_photon_gj_tr(P, u, t, st, ct, sp, cp, erg, du, aux);
}

template <class T, bool UNI>
__host__ __device__ inline void rhs_photon_gj_tr(const KParams& P, const T* u, const T& t, const T& st, const T& ct,
                                                 const T& sp, const T& cp, double erg, T* du, T* aux) {
  ART_FP_FAST
  const bool flat = P.rs_eff == 0.0;
  const T r = u[0];
  const T E = -u[6];
  const T rc = rclamp(r, P.rNS);  // max(r, rNS) in one instruction
  const T ast = mabs(st);
  const T sgn_st = msign(st);
  const T kr = u[3] * erg, kt = u[4] * erg, kp = u[5] * erg;
  // one division for 1/r, 1/|sinθ|, 1/E and 1/erg, one for 1/β
  const T X1 = rc * ast, X2 = E * erg;
  const T R = frcp(X1 * X2);
  const T RX1 = R * X1;
  const T iE = RX1 * erg;
  const T ierg = RX1 * E;
  const T inv_rs = R * X2;
  const T ir = inv_rs * ast, iast = inv_rs * rc;
  // Schwarzschild: g^rr at the clamped radius, its derivatives, and g^rr at the raw radius for
  // the prefactor (:82), which differs only inside the star
  T grr = 1.0, dgtt = 0.0, dgrr = 0.0, grr_u = 1.0, sq = 1.0, isq = 1.0;
  if (!flat) {
    if (uni_if<UNI>(rc <= 10.0)) {  // g_schwartz's interior patch (a radius clamped to rNS <= 10 km)
      T gtt;
      metric_tr_d(rc, P.rs_eff, gtt, grr, dgtt, dgrr);
      sq = msqrt(grr);
      isq = trcp(sq);
    } else {  // metric_tr_d's exterior branch on the shared 1/r: one reciprocal, 1/g^rr
      grr = 1.0 - P.rs_eff * ir;
      dgrr = P.rs_eff * ir * ir;
      const T ig = trcp(grr);
      dgtt = dgrr * ig * ig;
      sq = msqrt(grr);
      isq = sq * ig;  // 1/√g^rr = √g^rr / g^rr
    }
    grr_u = grr;
    if (uni_if<UNI>(r < P.rNS)) {
      T gtt_u;
      metric_tr(r, P.rs_eff, gtt_u, grr_u);
    }
  }
  // rotating dipole (dipole_ang)
  const T cmst = P.cm * st, smct = P.sm * ct, smst = P.sm * st;
  const T a1 = P.cm * ct + smst * cp;
  const T a2 = cmst - smct * cp;
  const T a3 = P.sm * sp;
  const T a1p = -smst * sp, a2p = smct * sp, a3p = P.sm * cp;
  const T b = 2.0 * a1 * ct - a2 * st;
  const T ibeta = frcp(4.0 * a1 * a1 + a2 * a2 + a3 * a3);
  const T ir2 = ir * ir, ir3 = ir2 * ir;
  const T cB = P.wp2n * ir3;  // ωp² = cB |b|
  const T wp2 = cB * mabs(b);
  const T cBs = cB * msign(b);
  const T iast2 = iast * iast;
  const T kpa3 = kp * a3;
  const T krs = flat ? kr : sq * kr;  // √g^rr k_r
  const T pa = kt * a2 + kpa3 * iast;
  const T p = 2.0 * krs * a1 + ir * pa;  // k∥ √β r |sinθ| / (r |sinθ|)
  const T Gp = p * ibeta * (iE * iE);   // G / g^rr
  const T G = flat ? Gp : grr * Gp;
  const T Q = G * p;
  const T w = wp2 * G;
  const T omQ = 1.0 - Q;
  const T p_t = -2.0 * krs * a2 + ir * (kt * a1 - kpa3 * sgn_st * ct * iast2);
  const T p_p = 2.0 * krs * a1p + ir * (kt * a2p + kp * a3p * iast);
  const T Qib = wp2 * Q * ibeta;
  const T beta_p = 8.0 * a1 * a1p + 2.0 * (a2 * a2p + a3 * a3p);
  const T kp2 = kp * kp;
  T H_r = w * ir2 * pa - ir3 * (kt * kt + iast2 * kp2) - 1.5 * wp2 * ir * omQ;
  if (!flat)
    H_r += 0.5 * (dgtt * (E * E) + dgrr * (kr * kr) - wp2 * dgrr * Gp * p) - w * dgrr * isq * kr * a1;
  const T H_t = -ct * ir2 * iast2 * iast * sgn_st * kp2 - 1.5 * cBs * (a2 * ct + a1 * st) * omQ - w * p_t -
                3.0 * Qib * a1 * a2;
  const T H_p = 1.5 * cBs * a1p * ct * omQ - w * p_p + 0.5 * Qib * beta_p;
  // rows 1..6 vanish for r <= 1.01 rNS (:86)
  const T tg = flat ? t : t * grr_u;
  const T facx = (r <= P.rNS101) ? T(0.0) : C_KM * tg * iE;
  const T fx = -facx * ierg;
  du[0] = flat ? (kr - 2.0 * w * a1) * facx : (grr * kr - 2.0 * w * (sq * a1)) * facx;
  du[1] = (ir2 * kt - w * ir * a2) * facx;
  du[2] = (ir2 * iast2 * kp - w * ir * a3 * iast) * facx;
  du[3] = H_r * fx;
  du[4] = H_t * fx;
  du[5] = H_p * fx;
  du[6] = -P.omega * H_p * tg * iE;  // ∂H/∂t = -ω ∂H/∂φ
  if (aux) {
    aux[0] = b;
    aux[1] = t;
  }
}

// func_axion! (RayTracer.jl:95-123) with hamiltonian_axion (:632-640): H = K/2 at fixed
// energy erg, no clamp, no NS cut, du[7] = 0.
template <class T>
__host__ __device__ inline void rhs_axion(const KParams& P, const T* u, const T& tau, double erg, T* du) {
  ART_FP_FAST
  const T t = fexp(tau);
  const T r = u[0];
  T st, ct;
  msincos(u[1], st, ct);
  T gtt, grr, dgtt, dgrr;
  metric_tr_d(r, P.rs_eff, gtt, grr, dgtt, dgrr);
  const T ir = 1.0 / r;
  const T ir2 = ir * ir;
  const T is2 = 1.0 / (st * st);
  const T kr = u[3] * erg, kt = u[4] * erg, kp = u[5] * erg;
  const T fac = C_KM * t * grr / erg;
  const T fx = -fac / erg;
  du[0] = grr * kr * fac;
  du[1] = ir2 * kt * fac;
  du[2] = ir2 * is2 * kp * fac;
  du[3] = 0.5 * (dgtt * erg * erg + dgrr * kr * kr - 2.0 * ir2 * ir * (kt * kt + is2 * kp * kp)) * fx;
  du[4] = 0.5 * (-2.0 * ct * ir2 * is2 / st * kp * kp) * fx;
  du[5] = 0.0;
  du[6] = 0.0;
}

template <class T>
__host__ __device__ inline void rhs(const KParams& P, bool photon, const T* u, const T& tau, double erg, T* du) {
  if (!photon) rhs_axion(P, u, tau, erg, du);
  else if (!(P.bndry_lyr > 0.0) && !P.isotropic) rhs_photon_gj(P, u, tau, erg, du);
  else rhs_photon(P, u, tau, erg, du);
}

// hamiltonian value + all partials at (x, k, T, E) for parity tests (RayTracer.jl:530-556).
// bndry_lyr is applied in all partials here (unlike func!, which applies it to ∂t only).
template <class T>
__host__ __device__ inline void hamiltonian_full(const KParams& P, const T* x, const T* k, const T& Tm, const T& E,
                                                 T* H, T* dHdx, T* dHdk, T* dHdT) {
  const T r = x[0];
  const bool clamped = r < P.rNS;
  const T rc = clamped ? T(P.rNS) : r;
  T st, ct, sp, cp;
  msincos(x[1], st, ct);
  msincos(x[2] - P.omega * Tm, sp, cp);
  const T ir = 1.0 / rc, ir2 = ir * ir, iast = 1.0 / mabs(st), sgn_st = msign(st);
  const DipoleAng<T> d = dipole_ang(P, st, ct, sp, cp);
  const T sgb = msign(d.b);
  const T cB = P.wp2n * ir2 * ir;
  T wp2 = cB * mabs(d.b);
  T dwp2_r = -3.0 * wp2 * ir, dwp2_t = cB * sgb * d.bt, dwp2_p = cB * sgb * d.bp;
  if (P.bndry_lyr > 0.0) {
    const T wgj = msqrt(wp2);
    const T L = layer_wp(P, rc, P.rmax);
    const T wt = wgj + L;
    const T dL_r = L * (-1.5 * ir - 1.0 / (0.1 * P.rmax));
    const T s = wt / wgj;
    dwp2_r = dwp2_r * s + 2.0 * wt * dL_r;
    dwp2_t = dwp2_t * s;
    dwp2_p = dwp2_p * s;
    wp2 = wt * wt;
  }
  T gtt, grr, dgtt, dgrr;
  metric_tr_d(rc, P.rs_eff, gtt, grr, dgtt, dgrr);
  // the prefactor's g^rr at the raw radius (:82) differs from the clamped one only inside the
  // star: a second metric evaluation only for lanes there
  T grr_u = grr;
  if (!(P.rs_eff == 0.0) && r < P.rNS) {
    T gtt_u;
    metric_tr(r, P.rs_eff, gtt_u, grr_u);
  }
  const T gpp = ir2 * iast * iast;
  const T E2 = E * E, iE2 = 1.0 / E2, sq = msqrt(grr);
  T Q = 0.0, Q_r = 0.0, Q_t = 0.0, Q_p = 0.0, Q_kr = 0.0, Q_kt = 0.0, Q_kp = 0.0;
  if (!P.isotropic) {
    const T pa = k[1] * d.a2 + k[2] * d.a3 * iast;
    const T p = 2.0 * sq * k[0] * d.a1 + ir * pa;
    const T ibeta = 1.0 / (4.0 * d.a1 * d.a1 + d.a2 * d.a2 + d.a3 * d.a3);
    const T G = grr * p * ibeta * iE2;
    Q = G * p;
    const T p_r = dgrr / sq * k[0] * d.a1 - ir2 * pa;
    const T p_t = 2.0 * sq * k[0] * d.a1t + ir * (k[1] * d.a1 - k[2] * d.a3 * sgn_st * ct * iast * iast);
    const T p_p = 2.0 * sq * k[0] * d.a1p + ir * (k[1] * d.a2p + k[2] * d.a3p * iast);
    const T beta_t = 8.0 * d.a1 * d.a1t + 2.0 * d.a2 * d.a1;
    const T beta_p = 8.0 * d.a1 * d.a1p + 2.0 * d.a2 * d.a2p + 2.0 * d.a3 * d.a3p;
    Q_r = dgrr * p * p * ibeta * iE2 + 2.0 * G * p_r;
    Q_t = 2.0 * G * p_t - Q * beta_t * ibeta;
    Q_p = 2.0 * G * p_p - Q * beta_p * ibeta;
    Q_kr = 4.0 * G * sq * d.a1;
    Q_kt = 2.0 * G * ir * d.a2;
    Q_kp = 2.0 * G * ir * d.a3 * iast;
  }
  const T omQ = 1.0 - Q;
  const T K = gtt * E2 + grr * k[0] * k[0] + ir2 * k[1] * k[1] + gpp * k[2] * k[2];
  *H = 0.5 * (K + wp2 * omQ);
  const T ir3 = ir2 * ir;
  const T rmask = clamped ? 0.0 : 1.0;  // the clamp makes r a constant (zero partial)
  dHdx[0] = rmask * 0.5 * (dgtt * E2 + dgrr * k[0] * k[0] - 2.0 * ir3 * (k[1] * k[1] + iast * iast * k[2] * k[2]) +
                           dwp2_r * omQ - wp2 * Q_r);
  dHdx[1] = 0.5 * (-2.0 * ct * ir2 * iast * iast / st * k[2] * k[2] + dwp2_t * omQ - wp2 * Q_t);
  dHdx[2] = 0.5 * (dwp2_p * omQ - wp2 * Q_p);
  dHdk[0] = grr * k[0] - 0.5 * wp2 * Q_kr;
  dHdk[1] = ir2 * k[1] - 0.5 * wp2 * Q_kt;
  dHdk[2] = gpp * k[2] - 0.5 * wp2 * Q_kp;
  *dHdT = -P.omega * dHdx[2];
}

// ---------------------------------------------------------------------------
// Resonance condition of propagate's ContinuousCallback (RayTracer.jl:254-298,
// thick_surface = true): rescale w onto the axion mass shell with E = u[7], then
// H_photon/E² with ωp at t (zeroIn = true), k∥ and the raw radius.
// The reference computes w' = w √nrm, nrm = (-E² g^tt - m_a²)/(g^rr w_r² + g^θθ w_θ² +
// g^φφ w_φ²) (:281-282), then ½[g^tt E² + Σ g^ii w'_i² + ωp²(1 - g^rr k∥(w')²/E²)]/E².
// By construction Σ g^ii w'_i² = nrm·den = -E² g^tt - m_a², so the kinetic part is exactly
// -m_a², and k∥(w')² = nrm·k∥(w)². This evaluates that closed form: no square root, one
// division, the same value up to rounding. It is NaN where √nrm is (nrm < 0: |u7| has
// dropped below m_a, where the reference would raise DomainError).
template <class T>
__host__ __device__ inline void condition_nd(const KParams& P, const T* u, const T& t0, T& N, T& D) {
  // With s = |sinθ|: k∥(w)² = p²/β, p = 2√g^rr w_r a1 + (w_θ a2 + w_φ a3/s)/r, and
  // den = g^rr w_r² + (w_θ² + w_φ²/s²)/r². Scaling both by r s gives PP = p r s and
  // DEN = den r² s², so X = g^rr k∥(w')²/E² = g^rr num PP²/(DEN β E²) with no 1/r, 1/s.
  // ωp² = wpn/wpd (wpd = r³ without a boundary layer). One division in total:
  //   cond = ½ [wpn (A - B) - m_a² wpd A] / (wpd A E²),  A = DEN β E²,  B = g^rr num PP².
  const T r = u[0];
  T gtt, grr;
  metric_tr(r, P.rs_eff, gtt, grr);
  T st, ct;
  msincos(u[1], st, ct);
  const T E2 = u[6] * u[6];
  const T num = -E2 * gtt - P.mass_a2;
  if (num < 0.0) {
    N = T(NAN);
    D = T(1.0);
    return;
  }
  T wpn = 0.0, wpd = r * r * r;
  T A = 1.0, B = 0.0;
  if (r > P.rNS || !P.isotropic) {
    T sp, cp;
    msincos(u[2] - P.omega * t0, sp, cp);
    const DipoleAng<T> d = dipole_ang(P, st, ct, sp, cp);
    if (r > P.rNS) {  // zeroIn = true
      wpn = P.wp2n * mabs(d.b);
      if (P.bndry_lyr > 0.0) {
        const T w = msqrt(wpn / wpd) + layer_wp(P, r, P.rmax);
        wpn = w * w;
        wpd = 1.0;
      }
    }
    if (!P.isotropic) {
      const T as = mabs(st);
      const T sq = (P.rs_eff == 0.0) ? T(1.0) : msqrt(grr);
      const T ur = u[3] * r * as, ut = u[4] * as;
      const T DEN = grr * ur * ur + ut * ut + u[5] * u[5];
      const T PP = 2.0 * sq * ur * d.a1 + ut * d.a2 + u[5] * d.a3;
      const T beta = 4.0 * d.a1 * d.a1 + d.a2 * d.a2 + d.a3 * d.a3;
      A = DEN * beta * E2;
      B = grr * num * PP * PP;
    }
  }
  N = wpn * (A - B) - P.mass_a2 * wpd * A;
  D = wpd * A * E2;
}

// The condition's value: cond = ½ N / D (condition_nd). The grid pass of the scan only needs
// its sign, which is the sign of N whenever D > 0 (propagate_kernel, sign_code_nd).
template <class T>
__host__ __device__ inline T condition_t(const KParams& P, const T* u, const T& t0) {
  T N, D;
  condition_nd(P, u, t0, N, D);
  return 0.5 * N / D;
}

// ---------------------------------------------------------------------------
// Certified steps of the resonance scan (propagate_kernel).
// The scanned interpolant -- the cubic Hermite of (u0, f0) -> (u1, f1) over h -- lies in the
// convex hull of its Bernstein control points u0, u0 + h f0/3, u1 - h f1/3, u1. That bounds
// r and |u7| from below and θ, φ around the end point over the whole step. With
// b = Bz/B_n = cosθm (3cos²θ - 1) + 3 sinθm sinθ cosθ cosψ one has |∂b/∂θ| <= 3 and
// |∂b/∂ψ| <= 1.5 |sinθm|, so |b| <= |b(end)| + 3Δθ + 1.5|sinθm|Δψ (and |b| <= 2). If then
// ωp² <= wp2n |b|max / r_min³ < m_a² and u7² > m_a² (so num > 0: no NaN), the numerator of
// condition_nd, wpn (A - B) - m_a² r³ A, is < 0 at every point (B >= 0, A > 0): every grid
// code of the step is "negative" without evaluating it. The margins (1e-6 on ωp², 1e-9 on
// u7², a hull slack of 1e-12 of the terms) are far above the rounding of the interpolant
// and of the condition. The only uncovered case is measure-zero: A = 0, which needs sinθ
// and w_φ both exactly zero at a grid point. Likewise, where u7² (-g^tt) < m_a² over the
// whole hull (the photon has lost energy below the axion shell), every grid point's NrmSq
// is negative and every code is "NaN".
struct Hull {
  double lo, hi;
};

__host__ __device__ inline Hull bernstein_hull(double a, double fa, double b, double fb, double h) {
  const double h3 = h * (1.0 / 3.0);
  const double c1 = a + h3 * fa, c2 = b - h3 * fb;
  const double s = 1e-12 * (fabs(a) + fabs(b) + fabs(h * fa) + fabs(h * fb));
  if (!(fabs(c1) + fabs(c2) + s < __builtin_inf())) return {NAN, NAN};  // non-finite: no bound
  return {fmin_q(fmin_q(a, b), fmin_q(c1, c2)) - s, fmax_q(fmax_q(a, b), fmax_q(c1, c2)) + s};
}

// Returns the certified sign code of every grid point of the step: 2 (negative, above), 1
// (positive: ωp² g^rr > u7² all along the step, below), 3 (NaN: u7² (-g^tt) < m_a² all along
// the step, where the reference's √NrmSq is undefined and condition_nd returns NaN), or 0
// when nothing is certain.
// b1 = Bz/B_n and t1 = e^(τ + h) at the end point come from the step's last RHS evaluation
// (rhs_photon's aux), so the certificate needs no transcendental of its own. b0, b at the
// start point (the previous step's last RHS; NaN when unknown), tightens the range of b.
__host__ __device__ inline int scan_certified_code(const KParams& P, const double* u0, const double* f0,
                                                   const double* u1, const double* f1, double h, double b1,
                                                   double t1, double b0 = NAN) {
  if (!(P.cert_fac < 1e300)) return 0;
  const Hull r = bernstein_hull(u0[0], f0[0], u1[0], f1[0], h);
  if (!(r.lo > P.cert_rmin)) return 0;
  const Hull e = bernstein_hull(u0[6], f0[6], u1[6], f1[6], h);
  const double elo = e.lo > 0.0 ? e.lo : (e.hi < 0.0 ? -e.hi : 0.0);
  const double ehi = fmax(fabs(e.lo), fabs(e.hi));
  // -g^tt <= 1 / (1 - rs / r_min) for r > 10 km (flat: exactly 1)
  const double gmax = P.rs_eff == 0.0 ? 1.0 : 1.0 / (1.0 - P.rs_eff / r.lo);
  if (ehi * ehi * gmax * (1.0 + 1e-9) < P.mass_a2) return 3;
  if (!(elo * elo > P.cert_e2)) return 0;
  const Hull th = bernstein_hull(u0[1], f0[1], u1[1], f1[1], h);
  const Hull ph = bernstein_hull(u0[2], f0[2], u1[2], f1[2], h);
  // t = e^(τ + θh) rises monotonically over the step, by t1 - t0 = t1 (1 - e^-h) <= t1 h
  const double dth = fmax(th.hi - u1[1], u1[1] - th.lo);
  const double dps = fmax(ph.hi - u1[2], u1[2] - ph.lo) + fabs(P.omega) * t1 * h * (1.0 + 1e-12);
  const double db = 3.0 * dth + 1.5 * fabs(P.sm) * dps + 1e-12;
  double bmax = fmin(2.0, fabs(b1) + db);
  double bmin = fabs(b1) - db;
  if (b0 == b0) {
    // Two-sided: along the step b moves by at most ℓ = 3 TV(θ) + 1.5|sinθm| TV(ψ) in total
    // (TV: total variation; a Bézier curve's is at most its control polygon's, and
    // TV(ψ) <= TV(φ) + |ω| (t1 - t0)). A point at variation d0 from the start and d1 from the
    // end (d0 + d1 <= ℓ) has b >= max(b0 - d0, b1 - d1) >= (b0 + b1 - ℓ)/2, and likewise
    // b <= (b0 + b1 + ℓ)/2: half the one-sided slack when the path is monotone.
    const double h3 = h * (1.0 / 3.0);
    const double tvt = fabs(h3 * f0[1]) + fabs((u1[1] - h3 * f1[1]) - (u0[1] + h3 * f0[1])) + fabs(h3 * f1[1]);
    const double tvp = fabs(h3 * f0[2]) + fabs((u1[2] - h3 * f1[2]) - (u0[2] + h3 * f0[2])) + fabs(h3 * f1[2]);
    const double ell = (3.0 * tvt + 1.5 * fabs(P.sm) * (tvp + fabs(P.omega) * t1 * h)) * (1.0 + 1e-12) + 1e-12;
    const double lo = 0.5 * (b0 + b1 - ell), hi = 0.5 * (b0 + b1 + ell);
    bmax = fmin(bmax, fmax(fabs(lo), fabs(hi)));
    bmin = fmax(bmin, lo > 0.0 ? lo : (hi < 0.0 ? -hi : 0.0));
  }
  if (P.wp2n * bmax * P.cert_fac < P.mass_a2 * (r.lo * r.lo * r.lo)) return 2;
  // positive: with ωp² g^rr > u7² everywhere. Cauchy-Schwarz gives B/A = g^rr num PP²/(DEN β E²)
  // <= g^rr num / E² = 1 - g^rr m_a² / E² (g^rr (-g^tt) = 1 outside 10 km), so
  // N / (r³ A) >= ωp² g^rr m_a² / E² - m_a² > 0. It needs r > rNS everywhere (zeroIn).
  const double grr_lo = P.rs_eff == 0.0 ? 1.0 : 1.0 - P.rs_eff / r.lo;
  if (r.lo > P.rNS && bmin > 0.0 &&
      P.wp2n * bmin * grr_lo > ehi * ehi * P.cert_fac * (r.hi * r.hi * r.hi))
    return 1;
  return 0;
}


template <class T>
__host__ __device__ inline T condition(const KParams& P, const T* u, const T& tau) {
  return condition_t(P, u, fexp(tau));
}

// ---------------------------------------------------------------------------
// The ContinuousCallback's sign walk over one step's grid codes (DiffEqBase's sequential
// scan of interp_points values, RayTracer.jl:357-358): 2-bit codes (0 zero, 1 positive,
// 2 negative, 3 NaN) of points 1..nper, 16 per word. A NaN resets the remembered sign; a
// nonzero point of the other sign than the remembered one is a change. State: the next
// point ip, the remembered sign last_s, the last nonzero point last_j, and lc_ok (the value
// at last_j is known: cleared by every nonzero point passed).
struct WalkState {
  int ip, last_s, last_j;
  bool lc_ok;
};

// The sequential reference form.
__host__ __device__ inline void walk_codes_loop(const unsigned cw[4], int nper, WalkState& st, bool& found) {
  found = false;
  for (; st.ip <= nper; ++st.ip) {
    const unsigned code = (cw[(st.ip - 1) >> 4] >> (2 * ((st.ip - 1) & 15))) & 3u;
    if (code == 3u) {
      st.last_s = 0;
      continue;
    }
    const int si = (code == 1u) ? 1 : (code == 2u ? -1 : 0);
    if (st.last_s != 0 && si != 0 && si != st.last_s) {
      found = true;
      return;
    }
    if (si != 0) {
      st.last_s = si;
      st.last_j = st.ip;
      st.lc_ok = false;
    }
  }
}

// Bit-parallel form for the usual case, no exact-zero code from ip on: every remaining
// point is then positive, negative or NaN, its predecessor is the point before it (at ip:
// the remembered sign), and a change is a P after an N or an N after a P. 32 points per
// 64-bit word (bit 2(p-1) of word 0 for p <= 32, bit 2(p-33) of word 1 above). Returns
// false, with st untouched, when a zero code needs the sequential form; otherwise leaves
// exactly the state walk_codes_loop would (tests/test_walk_codes.py). nper <= 64.
__host__ __device__ inline bool walk_codes_bits(const unsigned cw[4], int nper, WalkState& st, bool& found) {
  constexpr unsigned long long M = 0x5555555555555555ull;
  const int ip = st.ip;
  if (ip > nper) {
    found = false;
    return true;
  }
  const unsigned long long c[2] = {(unsigned long long)cw[0] | ((unsigned long long)cw[1] << 32),
                                   (unsigned long long)cw[2] | ((unsigned long long)cw[3] << 32)};
  unsigned long long Pm[2], Nm[2], R[2];
  unsigned long long zero = 0ull;
  for (int k = 0; k < 2; ++k) {
    int a = ip - 1 - 32 * k, b = nper - 1 - 32 * k;  // the range ip..nper in chunk positions
    a = a < 0 ? 0 : a;
    b = b > 31 ? 31 : b;
    unsigned long long r = 0ull;
    if (a <= b) {
      const unsigned long long hi = (b == 31) ? ~0ull : ((1ull << (2 * b + 2)) - 1ull);
      r = hi & ~((1ull << (2 * a)) - 1ull) & M;
    }
    R[k] = r;
    const unsigned long long x = c[k], xs = c[k] >> 1;
    Pm[k] = x & ~xs & M;
    Nm[k] = xs & ~x & M;
    zero |= ~(x | xs) & M & r;
  }
  if (zero != 0ull) return false;
  const int q = ip - 1;
  const unsigned long long ib0 = (q < 32) ? (1ull << (2 * q)) : 0ull;
  const unsigned long long ib1 = (q >= 32) ? (1ull << (2 * (q - 32))) : 0ull;
  const unsigned long long sP = st.last_s > 0 ? ~0ull : 0ull, sN = st.last_s < 0 ? ~0ull : 0ull;
  const unsigned long long Pp0 = ((Pm[0] << 2) & ~ib0) | (ib0 & sP);
  const unsigned long long Np0 = ((Nm[0] << 2) & ~ib0) | (ib0 & sN);
  const unsigned long long Pp1 = (((Pm[1] << 2) | (Pm[0] >> 62)) & ~ib1) | (ib1 & sP);
  const unsigned long long Np1 = (((Nm[1] << 2) | (Nm[0] >> 62)) & ~ib1) | (ib1 & sN);
  const unsigned long long T0 = R[0] & ((Pm[0] & Np0) | (Nm[0] & Pp0));
  const unsigned long long T1 = R[1] & ((Pm[1] & Np1) | (Nm[1] & Pp1));
  if ((T0 | T1) != 0ull) {
    const int j = T0 ? 1 + (__builtin_ctzll(T0) >> 1) : 33 + (__builtin_ctzll(T1) >> 1);
    const bool jp = T0 ? ((Pm[0] >> (2 * (j - 1))) & 1ull) : ((Pm[1] >> (2 * (j - 33))) & 1ull);
    if (j > ip) {  // the point before j is nonzero, of the other sign
      st.last_j = j - 1;
      st.lc_ok = false;
    }
    st.last_s = jp ? -1 : 1;
    st.ip = j;
    found = true;
    return true;
  }
  const unsigned long long g0 = (Pm[0] | Nm[0]) & R[0], g1 = (Pm[1] | Nm[1]) & R[1];
  if (g1) {
    st.last_j = 33 + ((63 - __builtin_clzll(g1)) >> 1);
    st.lc_ok = false;
  } else if (g0) {
    st.last_j = 1 + ((63 - __builtin_clzll(g0)) >> 1);
    st.lc_ok = false;
  }
  // the sign remembered after the last point: its own (no zeros), none after a NaN
  const int e = nper - 1;
  const unsigned code = (unsigned)(((e < 32) ? (c[0] >> (2 * e)) : (c[1] >> (2 * (e - 32)))) & 3ull);
  st.last_s = (code == 1u) ? 1 : (code == 2u ? -1 : 0);
  st.ip = nper + 1;
  found = false;
  return true;
}

// ---------------------------------------------------------------------------
// Cartesian -> (r, θ, φ) and the covariant "celerity" of k (RayTracer.jl:193-212,
// k_norm_Cart :656-664, k_sphere :995-1007).
template <class T>
__host__ __device__ inline void cart_to_sph(const T* x, T& r, T& th, T& ph) {
  r = msqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  th = macos(x[2] / r);
  ph = matan2(x[1], x[0]);
}

template <class T>
__host__ __device__ inline void celerity(const T* x, const T* k, const T& r, const T& st, double rs, T* w) {
  const T AA = 1.0 - rs / r;
  const T iAA = 1.0 / AA;
  const T dr_dt = (x[0] * k[0] + x[1] * k[1] + x[2] * k[2]) / r;
  w[0] = dr_dt / msqrt(AA) * iAA;
  w[1] = (x[2] * dr_dt - r * k[2]) / st * iAA;   // v_θ r
  w[2] = (x[0] * k[1] - x[1] * k[0]) * iAA;      // v_φ r sinθ
}

// k_norm_Cart (RayTracer.jl:643-685) with ax_fix = true / is_photon = false: rescale k
// onto the axion mass shell at erg, always with the GR mass (:181-185).
template <class T>
__host__ __device__ inline void k_norm_axion_shell(const KParams& P, const T* x, const T* k, double erg, T* out) {
  T r, th, ph;
  cart_to_sph(x, r, th, ph);
  const T st = msin(th);
  T w[3];
  celerity(x, k, r, st, P.rs_gr, w);
  T gtt, grr;
  metric_tr(r, P.rs_gr, gtt, grr);
  const T ir2 = 1.0 / (r * r);
  const T nrm = (-erg * erg * gtt - P.mass_a2) / (grr * w[0] * w[0] + ir2 * w[1] * w[1] + ir2 / (st * st) * w[2] * w[2]);
  const T f = msqrt(nrm);
  out[0] = f * k[0];
  out[1] = f * k[1];
  out[2] = f * k[2];
}

// propagate's initial state u0 = [r θ φ | w/erg | erg Δω] (RayTracer.jl:179-216).
template <class T>
__host__ __device__ inline void initial_state(const KParams& P, const T* x0, const T* k0, double erg, double dw, T* u) {
  T kn[3];
  k_norm_axion_shell(P, x0, k0, erg, kn);
  T r, th, ph;
  cart_to_sph(x0, r, th, ph);
  T w[3];
  celerity(x0, kn, r, msin(th), P.rs_eff, w);
  const double ie = 1.0 / erg;
  u[0] = r; u[1] = th; u[2] = ph;
  u[3] = w[0] * ie; u[4] = w[1] * ie; u[5] = w[2] * ie;
  u[6] = T(erg * dw);
}

// Covariant (w erg) -> Cartesian momentum with ω = 1 - r_s/r (affect! :331-342 and the
// back-transform :393-416, which scales the mass inside the star :398-406).
template <class T>
__host__ __device__ inline void sph_to_cart(const T* u, double erg, const T& rs, T* x, T* k) {
  T st, ct, sp, cp;
  msincos(u[1], st, ct);
  msincos(u[2], sp, cp);
  const T om = 1.0 - rs / u[0];
  const T s = erg * om;
  const T v0 = u[3] * msqrt(om) * s, v1 = u[4] / u[0] * s, v2 = u[5] / (u[0] * st) * s;
  const T vt = st * v0 + ct * v1;
  x[0] = u[0] * st * cp;
  x[1] = u[0] * st * sp;
  x[2] = u[0] * ct;
  k[0] = cp * vt - sp * v2;
  k[1] = sp * vt + cp * v2;
  k[2] = ct * v0 - st * v1;
}

// Final state -> Cartesian (RayTracer.jl:393-416); the mass is scaled by (r/rNS)^3 inside.
template <class T>
__host__ __device__ inline void back_transform(const KParams& P, const T* u, double erg, T* x, T* k) {
  T rs = P.rs_eff;
  if (u[0] < P.rNS) rs = rs * (u[0] * u[0] * u[0]) / (P.rNS * P.rNS * P.rNS);
  sph_to_cart(u, erg, rs, x, k);
}

// ---------------------------------------------------------------------------
// get_Prob_nonAD (MainRunner.jl:67-124) -> conversion_prob (RayTracer.jl:1405-1473),
// one_D = false, melrose = true. Per-crossing ("local") quantities first; the group-level
// linear-indexed values (ksphere[1..3], Bsphere[1..3], x0_pl[1..2], :1432-1443, :510-511)
// come in separately so groups of Nc > 1 crossings reproduce the reference exactly.
template <class T>
struct ProbLocal {
  T r, th, ph, st, ct;
  T grr, gthth, gpp;     // GR metric (global Mass_NS, MainRunner.jl:75)
  T B[3];                // Bsphere (GJ_Model_Sphereical, flat honoured)
  T ks[3];               // k_sphere (flat honoured)
  T Bmag, kmag, cth, sth;
  T ergax, wp;
};

template <class T>
__host__ __device__ inline ProbLocal<T> prob_local(const KParams& P, const T* pos, const T* kpos, const T& erg_eff) {
  ProbLocal<T> L;
  cart_to_sph(pos, L.r, L.th, L.ph);
  msincos(L.th, L.st, L.ct);
  T gtt;
  metric_tr(L.r, P.rs_gr, gtt, L.grr);
  const T ir = 1.0 / L.r;
  L.gthth = ir * ir;
  L.gpp = L.gthth / (L.st * L.st);
  T sp, cp;
  msincos(L.ph, sp, cp);  // t_start = 0
  const DipoleAng<T> d = dipole_ang(P, L.st, L.ct, sp, cp);
  const T Bn = P.Bn_coef * ir * ir * ir;
  T gtt_f, grr_f;
  metric_tr(L.r, P.rs_eff, gtt_f, grr_f);
  L.B[0] = 2.0 * Bn * d.a1 / msqrt(grr_f);
  L.B[1] = Bn * d.a2 * L.r;
  L.B[2] = Bn * d.a3 * L.r * mabs(L.st);
  celerity(pos, kpos, L.r, L.st, P.rs_eff, L.ks);
  const T BB = L.grr * L.B[0] * L.B[0] + L.gthth * L.B[1] * L.B[1] + L.gpp * L.B[2] * L.B[2];
  const T kk = L.grr * L.ks[0] * L.ks[0] + L.gthth * L.ks[1] * L.ks[1] + L.gpp * L.ks[2] * L.ks[2];
  const T Bk = L.grr * L.B[0] * L.ks[0] + L.gthth * L.B[1] * L.ks[1] + L.gpp * L.B[2] * L.ks[2];
  L.Bmag = msqrt(BB) * 1.95e-2;
  L.kmag = msqrt(kk);
  L.cth = Bk * 1.95e-2 / (L.kmag * L.Bmag);
  L.sth = msqrt(1.0 - L.cth * L.cth);  // sin(acos(c))
  if (P.isotropic) {
    L.cth = 0.0;
    L.sth = 1.0;
  }
  L.ergax = erg_eff / msqrt(1.0 - 2.0 * P.GM_c2 / L.r);
  L.wp = 0.0;
  if (L.r > P.rNS) {  // zeroIn = true
    L.wp = msqrt(P.wp2n * ir * ir * ir * mabs(d.b));
    if (P.bndry_lyr > 0.0) L.wp = L.wp + layer_wp(P, L.r, P.rmax_def);
  }
  return L;
}

// Group-level values: linear index q of a column-major m x 3 matrix -> row q % m, col q / m.
template <class T>
struct ProbLin {
  T k1, k2, k3, B1, B2, B3;  // ksphere[1..3], Bsphere[1..3]
  T r_c, th_c;               // x0_pl[1], x0_pl[2] (Cristoffel's r, theta)
};

template <class T>
__host__ __device__ inline T prob_eval(const KParams& P, double g_agg, const ProbLocal<T>& L, const ProbLin<T>& G) {
  const T wE = L.ergax;
  const T wE2 = wE * wE;
  const T vloc = msqrt(wE2 - P.mass_a2) / wE;
  T st, ct, sp, cp;
  msincos(L.th, st, ct);
  msincos(L.ph, sp, cp);
  const T ir = 1.0 / L.r, ir2 = ir * ir;
  const T iast = 1.0 / mabs(st), sgn_st = msign(st);
  const DipoleAng<T> d = dipole_ang(P, st, ct, sp, cp);
  const T Bn = P.Bn_coef * ir2 * ir;
  T dmu_E[3];
  if (P.isotropic) {
    // grad_x sqrt(kmag² + ωp²), omega_function defaults zeroIn=false, bndry_lyr=-1 (:1421)
    const T wp2 = P.wp2n * ir2 * ir * mabs(d.b);
    const T cB = 0.5 * P.wp2n * ir2 * ir * msign(d.b);
    const T inv = 1.0 / msqrt(L.kmag * L.kmag + wp2);
    dmu_E[0] = -1.5 * wp2 * ir * inv;
    dmu_E[1] = cB * d.bt * inv;
    dmu_E[2] = cB * d.bp * inv;
  } else {
    // ∇ωp (zeroIn = true, bndry_lyr, Mass_a = m_a; :1427)
    T dwp[3] = {0.0, 0.0, 0.0};
    if (L.r > P.rNS) {
      const T wgj = msqrt(P.wp2n * ir2 * ir * mabs(d.b));
      const T c = P.wp2n * ir2 * ir * msign(d.b) / (2.0 * wgj);
      dwp[0] = -1.5 * wgj * ir;
      dwp[1] = c * d.bt;
      dwp[2] = c * d.bp;
      if (P.bndry_lyr > 0.0) {
        const T Ly = layer_wp(P, L.r, P.rmax);
        dwp[0] = dwp[0] + Ly * (-1.5 * ir - 1.0 / (0.1 * P.rmax));
      }
    }
    // ∇(|B| 1.95e-2) (return_comp = 0, :1429)
    const T beta = 4.0 * d.a1 * d.a1 + d.a2 * d.a2 + d.a3 * d.a3;
    const T sb = msqrt(beta);
    const T beta_t = 8.0 * d.a1 * d.a1t + 2.0 * d.a2 * d.a1;
    const T beta_p = 8.0 * d.a1 * d.a1p + 2.0 * d.a2 * d.a2p + 2.0 * d.a3 * d.a3p;
    const T f = 1.95e-2 * Bn;        // signed: the components B^i (return_comp 1..3)
    const T fa = 1.95e-2 * mabs(Bn);  // |B| (return_comp 0) for either sign of B0
    const T dB[3] = {-3.0 * fa * sb * ir, fa * beta_t / (2.0 * sb), fa * beta_p / (2.0 * sb)};
    // ∇ of B^r √g^rr, B^θ/r, B^φ/(r|sinθ|) times 1.95e-2 (return_comp 1..3, :1432)
    T gtt_f, grr_f, dgtt_f, dgrr_f;
    metric_tr_d(L.r, P.rs_eff, gtt_f, grr_f, dgtt_f, dgrr_f);
    const T sgf = msqrt(grr_f);
    const T dc1[3] = {2.0 * f * d.a1 * (-3.0 * ir * sgf + 0.5 * dgrr_f / sgf), 2.0 * f * d.a1t * sgf,
                      2.0 * f * d.a1p * sgf};
    const T dc2[3] = {-4.0 * f * d.a2 * ir2, f * d.a1 * ir, f * d.a2p * ir};
    const T dc3[3] = {-4.0 * f * d.a3 * ir2 * iast, -f * d.a3 * ir * sgn_st * ct * iast * iast, f * d.a3p * ir * iast};
    // Christoffel symbols at (x0_pl[1], x0_pl[2]) with the GR mass (:503-527)
    const T GM = P.GM_c2;
    T stc, ctc;
    msincos(G.th_c, stc, ctc);
    const T G_rrr = -GM / (G.r_c * (G.r_c - 2.0 * GM));
    const T G_rtt = -(G.r_c - 2.0 * GM);
    const T G_rpp = -(G.r_c - 2.0 * GM) * stc * stc;
    const T G_trt = 1.0 / G.r_c;
    const T G_tpp = -stc * ctc;
    const T G_ptp = ctc / stc;
    const T s = 1.95e-2;
    const T t2r = G.k1 * (L.grr * G.B1 * s) * G_rrr + G.k2 * G_trt * (G.B2 * L.gthth * s) +
                  G.k3 * G_trt * (G.B3 * L.gpp * s);
    const T t2t = G.k1 * (L.gthth * G.B2 * s) * G_rtt + G.k3 * G_ptp * (G.B3 * L.gpp * s) +
                  G.k2 * (L.grr * G.B1 * s) * G_trt;
    const T t2p = G.k1 * (L.gpp * G.B3 * s) * G_rpp + G.k2 * G_tpp * (G.B3 * L.gpp * s) +
                  G.k3 * G_trt * (G.B1 * L.grr * s) + G.k3 * G_ptp * (G.B2 * L.gthth * s);
    const T t2[3] = {t2r, t2t, t2p};
    const T ikB = 1.0 / (L.kmag * L.Bmag);
    const T wp = L.wp;
    const T wp2 = wp * wp;
    const T preF = wp / mabs(wE2 * wE2 * wE + L.cth * L.cth * wE * (wp2 * wp2 - 2.0 * wp2 * wE2));
    const T A1 = wE2 * wE2 * L.sth * L.sth;
    const T A2 = wE2 * L.cth * wp * (wE2 - wp2);
    for (int c = 0; c < 3; ++c) {
      const T term1 = G.k1 * dc1[c] + G.k2 * dc2[c] + G.k3 * dc3[c];
      const T dct = (term1 + t2[c]) * ikB - L.cth * dB[c] / L.Bmag;
      dmu_E[c] = preF * (A1 * dwp[c] - A2 * dct);
    }
  }
  const T ik = 1.0 / L.kmag;
  const T vhat = L.grr * L.ks[0] * ik * dmu_E[0] + L.gthth * L.ks[1] * ik * dmu_E[1] + L.gpp * L.ks[2] * ik * dmu_E[2];
  const T wp2 = L.wp * L.wp;
  const T pref = wE2 * wE2 * L.sth * L.sth / (L.cth * L.cth * wp2 * (wp2 - 2.0 * wE2) + wE2 * wE2);
  const T gB = g_agg * 1e-9 * L.Bmag;
  return PI / 2.0 * pref * gB * gB / (mabs(vhat) * vloc * C_KM * HBAR);
}

// Nc = 1: the group values are the crossing's own (forward trees, MainRunner.jl:265).
template <class T>
__host__ __device__ inline T prob_nonad_single(const KParams& P, const T* pos, const T* kpos, const T& erg_eff) {
  const ProbLocal<T> L = prob_local(P, pos, kpos, erg_eff);
  ProbLin<T> G;
  G.k1 = L.ks[0]; G.k2 = L.ks[1]; G.k3 = L.ks[2];
  G.B1 = L.B[0]; G.B2 = L.B[1]; G.B3 = L.B[2];
  G.r_c = L.r; G.th_c = L.th;
  return prob_eval(P, P.g_agg, L, G);
}

// ---------------------------------------------------------------------------
// Sampler condition (find_samples_new :1547-1583, thick_surface = true) at the Cartesian
// line point x with local velocity direction vl. sinθ, cosθ, sinφ, cosφ are taken
// algebraically from x instead of through acos/atan2 + sin/cos (identical values up to
// rounding); the metric always uses the GR mass (the sampler gets no `flat`). Divisions are
// hardware reciprocals with two Newton steps (trcp) on the device.
template <class T>
__host__ __device__ inline T sampler_condition_e(const KParams& P, const T* x, const T* vl, double E, double iE2);

template <class T>
__host__ __device__ inline T sampler_condition(const KParams& P, const T* x, const T* vl, double E) {
  const double iE2 = 1.0 / (E * E);  // per attempt: hoisted out of a scan by the compiler
  return sampler_condition_e(P, x, vl, E, iE2);
}

// The same with 1/E² given (the cooperative scan of sample_kernel evaluates other lanes' lines).
//
// Algebra (round 3): the reference builds w = (ṙ/√AA, (z ṙ - r v_z)/sinθ, x v_y - y v_x)/AA,
// rescales it onto the axion shell, w' = √nrm w with nrm = (-E² g^tt - m_a²)/|w|²_g, and
// evaluates ½(ksqr + ωp²(1 - g^rr k∥(w')²/E²))/E². After the rescale the kinetic part is
// ksqr = g^tt E² + |w'|²_g = -m_a² by construction, and k∥(w')² = nrm k∥(w)², so neither √nrm
// nor the rescaled w is needed, and the common factor 1/AA of w cancels in nrm k∥(w)². Scaling
// k∥'s numerator and |w|²_g by sin²θ clears the 1/sinθ's:
//   g^rr k∥(w')² = g^rr (-E² g^tt - m_a²) p²/(D (4a1² + a2² + a3²)),
//   p = 2 √(g^rr/AA) ṙ a1 sinθ + ((z ṙ - r v_z) a2 + (x v_y - y v_x) a3)/r,
//   D = (g^rr/AA) ṙ² sin²θ + ((z ṙ - r v_z)² + (x v_y - y v_x)²)/r²,
// one reciprocal instead of the reference's divisions and two square roots. Equal to the
// reference's value to rounding (tests/test_corecheck.py against the oracle's literal form);
// NaN where it is (r = 0 or on the z axis).
template <class T>
__host__ __device__ inline T sampler_condition_e(const KParams& P, const T* x, const T* vl, double E, double iE2) {
  ART_FP_FAST
  const T rho2 = x[0] * x[0] + x[1] * x[1];
  const T r = msqrt(rho2 + x[2] * x[2]);
  const T ir = trcp(r);
  const T rho = msqrt(rho2);
  const T st = rho * ir, ct = x[2] * ir;
  const T irho = trcp(rho);
  const T cp = x[0] * irho, sp = x[1] * irho;  // ψ = φ at t0 = 0
  const T dr = (x[0] * vl[0] + x[1] * vl[1] + x[2] * vl[2]) * ir;
  const T u1 = x[2] * dr - r * vl[2];          // sinθ w1 AA
  const T u2 = x[0] * vl[1] - x[1] * vl[0];    // w2 AA
  const T ds = dr * st;
  const DipoleAng<T> d = dipole_ang(P, st, ct, sp, cp);
  T wp2 = P.wp2n * (ir * ir) * ir * mabs(d.b);  // GJ_Model_ωp_vec: no zeroIn
  if (P.bndry_lyr > 0.0 && r >= P.rNS) {
    const T w = msqrt(wp2) + layer_wp(P, r, P.rmax);
    wp2 = w * w;
  }
  T kn = 0.0;  // g^rr k∥(w')²
  if (!P.isotropic) {
    if (r > 10.0 && r >= P.rNS) {
      // outside the star and g_schwartz's interior patch, g^rr = 1 - rs/r = AA, so g = 1 and
      // g^rr (-E² g^tt - m_a²) = E² - g^rr m_a²: no square root and no division (the same
      // value to rounding; the general form below divides twice and takes √g)
      const T gx = 1.0 - P.rs_gr * ir;
      const T p = 2.0 * ds * d.a1 + (u1 * d.a2 + u2 * d.a3) * ir;
      const T D = ds * ds + (u1 * u1 + u2 * u2) * (ir * ir);
      kn = (E * E - gx * P.mass_a2) * (p * p) * trcp(D * (4.0 * d.a1 * d.a1 + d.a2 * d.a2 + d.a3 * d.a3));
    } else {
      T AA = 1.0 - P.rs_gr * ir;
      if (r < P.rNS) AA = 1.0;
      T gtt, grr;
      metric_tr(r, P.rs_gr, gtt, grr);
      const T g = grr * trcp(AA);  // 1 outside the star, up to rounding
      const T p = 2.0 * msqrt(g) * ds * d.a1 + (u1 * d.a2 + u2 * d.a3) * ir;
      const T D = g * ds * ds + (u1 * u1 + u2 * u2) * (ir * ir);
      kn = grr * (-(E * E) * gtt - P.mass_a2) * (p * p) * trcp(D * (4.0 * d.a1 * d.a1 + d.a2 * d.a2 + d.a3 * d.a3));
    }
  }
  return 0.5 * (wp2 * (1.0 - kn * iE2) - P.mass_a2) * iE2;
}

// The SIGN of sampler_condition_e at x without evaluating it (the sampler's grid needs only the
// signs of its points and whether they are nonzero): 1 negative, 2 positive, 0 undecided (then
// evaluate the condition). GJ plasma without a boundary layer, outside r_lim (r_lim2 =
// (max(10 km, rNS) (1 + 1e-9))²: the exterior branch above). With G = |x|² B̂-direction
// = 3 M x - |x|² m̂ (M = m̂·x, m̂ = (sinθm, 0, cosθm)): b = ẑ·G/|x|², and the algebra of
// sampler_condition_e's k∥ gives p²/(D β) = (v̂l·G)²/W, W = |x|² (3M² + |x|²) (p = sinθ v̂l·B,
// D = sin²θ |v̂l|², β = |B|²), so the condition has the sign of
//   T1 - T2 = wp2n |ẑ·G| (W r - κ r (v̂l·G)²) - m_a² |x|⁶ W,  κ r = r (1 - m_a²/E²) + rs m_a²/E²
// (the condition times |x|⁴ r² W 2E² > 0): one square root, no division. Decided only where
// |T1 - T2| exceeds 1e-9 of S, the sum of the magnitudes before cancellation, while both
// evaluations round at ~1e-14 of it; the 1e-9 band (and r = 0, the z axis, where the condition
// is NaN) goes to the full evaluation. tests/test_corecheck.py checks the signs against the
// condition and the oracle.
template <class T>
__host__ __device__ inline int sampler_sign_fast(const KParams& P, const T* x, const T* vl, double mE2,
                                                 double r_lim2) {
  const T rho2 = x[0] * x[0] + x[1] * x[1];
  const T R2 = rho2 + x[2] * x[2];
  if (!(R2 > r_lim2) || !(rho2 > 1e-100 * R2)) return 0;
  const T r = msqrt(R2);
  const T M = P.sm * x[0] + P.cm * x[2];
  const T zs = 3.0 * M * x[2], zc = R2 * P.cm;
  const T l = vl[0] * x[0] + vl[1] * x[1] + vl[2] * x[2];
  const T vm = P.sm * vl[0] + P.cm * vl[2];
  const T V = 3.0 * M * l - R2 * vm;
  const T W = R2 * (3.0 * M * M + R2);
  const T kr = P.isotropic ? 0.0 : r * (1.0 - mE2) + P.rs_gr * mE2;
  const T wz = P.wp2n * mabs(zs - zc);
  const T T2 = P.mass_a2 * (R2 * R2) * (R2 * W);
  const T d = wz * (W * r - kr * (V * V)) - T2;
  const T S = P.wp2n * (mabs(zs) + mabs(zc)) * (W * r + kr * (V * V)) + T2;
  if (!(mabs(d) > 1e-9 * S)) return 0;
  return d < 0.0 ? 1 : 2;
}

// ωp from GJ_Model_ωp_vec (no zeroIn) at Cartesian x, t = 0 (sampler affect!, :1587)
template <class T>
__host__ __device__ inline T wp_cart(const KParams& P, const T* x) {
  const T rho2 = x[0] * x[0] + x[1] * x[1];
  const T r = msqrt(rho2 + x[2] * x[2]);
  const T ir = trcp(r);
  const T rho = msqrt(rho2);
  const T irho = trcp(rho);
  const DipoleAng<T> d = dipole_ang(P, rho * ir, x[2] * ir, x[1] * irho, x[0] * irho);
  T wp = msqrt(P.wp2n * ir * ir * ir * mabs(d.b));
  if (P.bndry_lyr > 0.0 && r >= P.rNS) wp = wp + layer_wp(P, r, P.rmax);
  return wp;
}

// ---------------------------------------------------------------------------
// Verner 6(5) "most efficient" pair as used by OrdinaryDiffEq's Vern6 (FSAL: b = A[8,:]).
// Order conditions verified in tests/test_tableau.py.
struct Vern6 {
  static constexpr double c2 = 0.06, c3 = 0.09593333333333333, c4 = 0.1439, c5 = 0.4973, c6 = 0.9725,
                          c7 = 0.9995;
  static constexpr double a21 = 0.06;
  static constexpr double a31 = 0.019239962962962962, a32 = 0.07669337037037037;
  static constexpr double a41 = 0.035975, a43 = 0.107925;
  static constexpr double a51 = 1.3186834152331484, a53 = -5.042058063628562, a54 = 4.220674648395414;
  static constexpr double a61 = -41.872591664327516, a63 = 159.4325621631375, a64 = -122.11921356501003,
                          a65 = 5.531743066200053;
  static constexpr double a71 = -54.430156935316504, a73 = 207.06725136501848, a74 = -158.61081378459,
                          a75 = 6.991816585950242, a76 = -0.018597231062309313;
  static constexpr double a81 = -54.66374178728198, a83 = 207.95280625538937, a84 = -159.2889574744995,
                          a85 = 7.018743740796944, a86 = -0.018338785905045722, a87 = -0.0005119484997882099;
  static constexpr double a91 = 0.03438957868357036, a94 = 0.2582624555633503, a95 = 0.4209371189673537,
                          a96 = 4.40539646966931, a97 = -176.48311902429865, a98 = 172.36413340141507;
  static constexpr double bh1 = 0.04909967648382489, bh4 = 0.2251112229516524, bh5 = 0.4694682253029562,
                          bh6 = 0.8065792249988868, bh8 = -0.6071194891777959, bh9 = 0.05686113944047569;
  // btilde = b - bhat (error weights)
  static constexpr double e1 = a91 - bh1, e4 = a94 - bh4, e5 = a95 - bh5, e6 = a96 - bh6, e7 = a97, e8 = a98 - bh8,
                          e9 = -bh9;
};

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011): counter-based stream keyed by (seed, ray id), so
// every initial condition is independent of batch split and GPU count.
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = uint64_t(0xD2511F53u) * c[0];
    const uint64_t p1 = uint64_t(0xCD9E8D57u) * c[2];
    const uint32_t n0 = uint32_t(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = uint32_t(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = uint32_t(p1);
    c[2] = n2;
    c[3] = uint32_t(p0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__host__ __device__ inline double u01(uint32_t a, uint32_t b) {
  return (double(a >> 5) * 67108864.0 + double(b >> 6)) * (1.0 / 9007199254740992.0);
}

// The 10 uniforms of one find_samples_new attempt, in the reference's draw order:
// θi, ϕi, θi_loc, ϕi_loc, ϕRND, rRND (:1486-1497), vIfty x3 (:1531), randInx (:1623).
__host__ __device__ inline void attempt_uniforms(uint64_t seed, uint64_t ray, uint32_t attempt, double* U) {
#pragma unroll
  for (uint32_t blk = 0; blk < 5; ++blk) {
    uint32_t c[4] = {uint32_t(ray), uint32_t(ray >> 32), attempt, blk};
    philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
    U[2 * blk] = u01(c[0], c[1]);
    U[2 * blk + 1] = u01(c[2], c[3]);
  }
}

}  // namespace art
