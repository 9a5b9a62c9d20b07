// art_kernels.hip -- gfx950 kernels for the ray-tracing hot path.
//
// propagate_kernel: RT.propagate (RayTracer.jl:171-452) for a batch of segments.
//   * one wavefront lane per ray; the 7-D state u = [r θ φ | w | u7] and its FSAL
//     derivative live in VGPRs; NS parameters are kernel arguments (SGPRs);
//   * persistent lanes with a wave-aggregated work queue: a lane whose segment ends pulls
//     the next ray id from a 64-ray chunk the wave claimed with ONE global atomicAdd, so
//     short and long segments (12 vs 5000 steps) never idle a wave;
//   * every loop iteration is ONE integrator step attempt for every live lane: ordinary
//     adaptive steps, and the re-steps that polish a resonance root on the true
//     trajectory (mode ROOT), run the same unrolled stage code in lockstep;
//   * HBM is touched only to load a segment's initial conditions and to store its end
//     state and its crossings (Σ ≈ 220 B per segment).
#include <hip/hip_runtime.h>

#include <atomic>

#include <cstdio>
#include <cstdlib>

#include "art_core.h"
#include "art_event.h"
#include "art_internal.h"
#ifndef ART_NOLICM_TU
#include <hipcub/hipcub.hpp>
#endif

namespace art {


// stats[]: totals over the launch, for the roofline accounting (tools/count_flops.cpp)
enum { ST_ATTEMPTS = 0, ST_ACCEPTED, ST_ROOT_STEPS, ST_SCAN_EVALS, ST_INTERP_EVALS, ST_RAYS, ST_INIT_RHS, ST_CERT,
       ST_NSTATS = 8 };


// ---------------------------------------------------------------------------
// One Verner 6(5) attempt from (u, k1 = f(u)) over h: writes u_{n+1}, its FSAL derivative
// k9 and returns the RMS error norm of OrdinaryDiffEq (abstol + max(|u|,|u_new|) reltol).
template <class T>
__host__ __device__ inline T vern6_attempt(const KParams& P, bool photon, double erg, const T* u, const T* k1,
                                           const T& tau, const T& h, T* un, T* k9) {
  using V = Vern6;
  T k2[7], k3[7], k4[7], k5[7], k6[7], k7[7], k8[7], y[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h * (V::a21 * k1[i]);
  rhs(P, photon, y, tau + V::c2 * h, erg, k2);
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h * (V::a31 * k1[i] + V::a32 * k2[i]);
  rhs(P, photon, y, tau + V::c3 * h, erg, k3);
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h * (V::a41 * k1[i] + V::a43 * k3[i]);
  rhs(P, photon, y, tau + V::c4 * h, erg, k4);
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h * (V::a51 * k1[i] + V::a53 * k3[i] + V::a54 * k4[i]);
  rhs(P, photon, y, tau + V::c5 * h, erg, k5);
#pragma unroll
  for (int i = 0; i < 7; ++i)
    y[i] = u[i] + h * (V::a61 * k1[i] + V::a63 * k3[i] + V::a64 * k4[i] + V::a65 * k5[i]);
  rhs(P, photon, y, tau + V::c6 * h, erg, k6);
#pragma unroll
  for (int i = 0; i < 7; ++i)
    y[i] = u[i] + h * (V::a71 * k1[i] + V::a73 * k3[i] + V::a74 * k4[i] + V::a75 * k5[i] + V::a76 * k6[i]);
  rhs(P, photon, y, tau + V::c7 * h, erg, k7);
#pragma unroll
  for (int i = 0; i < 7; ++i)
    y[i] = u[i] + h * (V::a81 * k1[i] + V::a83 * k3[i] + V::a84 * k4[i] + V::a85 * k5[i] + V::a86 * k6[i] +
                       V::a87 * k7[i]);
  rhs(P, photon, y, tau + h, erg, k8);
#pragma unroll
  for (int i = 0; i < 7; ++i)
    un[i] = u[i] + h * (V::a91 * k1[i] + V::a94 * k4[i] + V::a95 * k5[i] + V::a96 * k6[i] + V::a97 * k7[i] +
                        V::a98 * k8[i]);
  rhs(P, photon, un, tau + h, erg, k9);
  if (photon && un[0] < P.rNS) un[0] = P.rNS;  // hamiltonian's in-place clamp on the FSAL stage (:531)
  T acc = 0.0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const T e = h * (V::e1 * k1[i] + V::e4 * k4[i] + V::e5 * k5[i] + V::e6 * k6[i] + V::e7 * k7[i] + V::e8 * k8[i] +
                     V::e9 * k9[i]);
    const T au = mabs(u[i]), an = mabs(un[i]);
    const T sc = P.abstol + (au > an ? au : an) * P.reltol;
    const T q = e / sc;
    acc = acc + q * q;
  }
  return msqrt(acc * (1.0 / 7.0));
}

// Classical RK4 over h; k_next = f(u_{n+1}) doubles as the next step's k1.
template <class T>
__host__ __device__ inline void rk4_attempt(const KParams& P, bool photon, double erg, const T* u, const T* k1,
                                            const T& tau, const T& h, T* un, T* kn) {
  T k2[7], k3[7], k4[7], y[7];
  const T h2 = 0.5 * h;
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h2 * k1[i];
  rhs(P, photon, y, tau + h2, erg, k2);
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h2 * k2[i];
  rhs(P, photon, y, tau + h2, erg, k3);
#pragma unroll
  for (int i = 0; i < 7; ++i) y[i] = u[i] + h * k3[i];
  rhs(P, photon, y, tau + h, erg, k4);
#pragma unroll
  for (int i = 0; i < 7; ++i) un[i] = u[i] + h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
  rhs(P, photon, un, tau + h, erg, kn);
  if (photon && un[0] < P.rNS) un[0] = P.rNS;
}

// cubic Hermite dense output between (u0, f0) and (u1, f1) over h at fraction th
template <class T>
__host__ __device__ inline void hermite7(const T* u0, const T* f0, const T* u1, const T* f1, const T& h,
                                         const T& th, T* out) {
  const T a = 1.0 - th;
  const T b = th * (th - 1.0);
  const T c1 = 1.0 - 2.0 * th;
  const T c2 = (th - 1.0) * h;
  const T c3 = th * h;
#pragma unroll
  for (int i = 0; i < 7; ++i) out[i] = a * u0[i] + th * u1[i] + b * (c1 * (u1[i] - u0[i]) + c2 * f0[i] + c3 * f1[i]);
}

// one component of hermite7
__device__ inline double hermite1(double u0, double f0, double u1, double f1, double h, double th) {
  return (1.0 - th) * u0 + th * u1 + th * (th - 1.0) * ((1.0 - 2.0 * th) * (u1 - u0) + (th - 1.0) * h * f0 + th * h * f1);
}

__device__ inline int sgn(double x) { return (x > 0.0) - (x < 0.0); }

// One point of the resonance scan: the condition on the cubic Hermite interpolant of the
// step (u0, f0) -> (u1, f1) over h, at fraction th and t = e^(τ + th h). Both the
// wave-cooperative grid pass and the per-lane bracket/Illinois evaluations call this, so a
// recomputed grid value is bit-identical to the one whose sign the grid pass recorded.
__device__ inline double scan_point(const KParams& P, const double* u0, const double* f0, const double* u1,
                                    const double* f1, double h, double tau, double th) {
  double ui[7];
  hermite7(u0, f0, u1, f1, h, th, ui);
  const double tt = tau + th * h;
  return condition_t(P, ui, fexp(tt));
}

// scan_point on an interpolant parked in LDS: S = the lane's base in the [slot][component]
// [lane] layout, slots 0-3 = u0, f0, u1, f1, slot 4 = (h, τ). The cooperative grid pass and
// the per-lane bracket evaluations both go through here.
__device__ inline void scan_nd_lds(const KParams& P, const double* S, int stride, double th, double& N, double& D) {
  double u0[7], f0[7], u1[7], f1[7], ui[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    u0[i] = S[(0 * 7 + i) * stride];
    f0[i] = S[(1 * 7 + i) * stride];
    u1[i] = S[(2 * 7 + i) * stride];
    f1[i] = S[(3 * 7 + i) * stride];
  }
  const double h = S[(4 * 7 + 0) * stride], tau = S[(4 * 7 + 1) * stride];
  hermite7(u0, f0, u1, f1, h, th, ui);
#pragma unroll
  for (int i = 0; i < 7; ++i) ui[i] = (th == 1.0) ? u1[i] : ui[i];  // the step's end point exactly
  condition_nd(P, ui, fexp(tau + th * h), N, D);
}

__device__ inline double scan_point_lds(const KParams& P, const double* S, int stride, double th) {
  double N, D;
  scan_nd_lds(P, S, stride, th, N, D);
  return 0.5 * N / D;  // = condition_t, bit for bit
}

// The integrator's span from in-kernel clock stamps (stats[ST_T0], stats[ST_T1]: the earliest
// wave start as the max of ~t, the latest wave end): s_memrealtime is the device's one 100 MHz
// constant clock, so the figure is the launch's own duration without a profiler's completion
// signals (art_recent_kernel_span_ms). Two atomics per wave.
__device__ inline void span_stamp(unsigned long long* stats, bool end) {
  if ((threadIdx.x & 63) == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    atomicMax(stats + (end ? ST_T1 : ST_T0), end ? t : ~t);
  }
}

// Completes this wave's LDS traffic before other lanes of the same wave read it.
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 2-bit sign code of a scan value: 0 zero, 1 positive, 2 negative, 3 NaN
__device__ inline unsigned sign_code(double c) { return isnan(c) ? 3u : (c > 0.0 ? 1u : (c < 0.0 ? 2u : 0u)); }

// sign_code(½ N / D) without the division where its sign is certain: D > 0 and finite, N a
// normal number and the quotient far from underflow. Otherwise the division decides.
__device__ inline unsigned sign_code_nd(double N, double D) {
  const double aN = fabs(N);
  if (D > 0.0 && D < INFINITY && aN >= 1e-290 && !(aN < 1e-290 * D)) return N > 0.0 ? 1u : 2u;
  return sign_code(0.5 * N / D);
}

// ode_determine_initdt (DiffEqBase) for an order-6 method, in two halves around its one extra RHS
// evaluation (init_one evaluates both RHS at ONE inlined site). initdt_begin returns the step when
// no probe is needed, else NaN with the probe point u1 = u0 + dt0 f0 at tau0 + dt0.
struct InitDt {
  double sk[7], d1, dt0;
};
__device__ inline double initdt_begin(const KParams& P, const double* u0, const double* f0, double tau0, double dtmax,
                                      InitDt& s, double* u1) {
  double d0 = 0.0, d1 = 0.0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    s.sk[i] = P.abstol + fabs(u0[i]) * P.reltol;
    d0 += (u0[i] / s.sk[i]) * (u0[i] / s.sk[i]);
    d1 += (f0[i] / s.sk[i]) * (f0[i] / s.sk[i]);
  }
  d0 = sqrt(d0 / 7.0);
  d1 = sqrt(d1 / 7.0);
  double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * (d0 / d1);
  dt0 = fmin(dt0, dtmax);
  const double at = fabs(tau0);
  const double eps_t = nextafter(at, INFINITY) - at;
  if (dt0 < 10.0 * eps_t) return fmax(1e-6, P.dtmin);
#pragma unroll
  for (int i = 0; i < 7; ++i) u1[i] = u0[i] + dt0 * f0[i];
  s.d1 = d1;
  s.dt0 = dt0;
  return NAN;
}
__device__ inline double initdt_end(const KParams& P, const double* f0, const double* f1, double dtmax, const InitDt& s) {
  bool same = true;
  double d2 = 0.0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    same = same && (f0[i] == f1[i]);
    const double q = (f1[i] - f0[i]) / s.sk[i];
    d2 += q * q;
  }
  if (same) return fmax(P.dtmin, 100.0 * s.dt0);
  d2 = sqrt(d2 / 7.0) / s.dt0;
  const double mx = fmax(s.d1, d2);
  const double dt1 = (mx <= 1e-15) ? fmax(1e-6, s.dt0 * 1e-3) : pow(10.0, -(2.0 + log10(mx)) / 6.0);
  return fmax(P.dtmin, fmin(fmin(100.0 * s.dt0, dt1), dtmax));
}

// Root of the condition along the Hermite interpolant inside (tha, thb] (Illinois).
__device__ inline double illinois_interp(const KParams& P, const double* u0, const double* f0, const double* u1,
                                         const double* f1, double tau, double h, double tha, double thb, double ca,
                                         double cb, int& nevals) {
  double tr = tha - ca * (thb - tha) / (cb - ca);
  int side = 0;
  for (int it = 0; it < 40; ++it) {
    double ui[7];
    hermite7(u0, f0, u1, f1, h, tr, ui);
    const double cr = condition(P, ui, tau + tr * h);
    ++nevals;
    if (cr == 0.0 || isnan(cr) || (thb - tha) < 1e-12) break;
    if (sgn(cr) == sgn(ca)) {
      tha = tr; ca = cr;
      if (side == -1) cb *= 0.5;
      side = -1;
    } else {
      thb = tr; cb = cr;
      if (side == 1) ca *= 0.5;
      side = 1;
    }
    const double tn = tha - ca * (thb - tha) / (cb - ca);
    if (tn == tr) break;
    tr = tn;
  }
  return tr;
}

// ---------------------------------------------------------------------------
// affect! (RayTracer.jl:301-350). Returns 0 = skipped, 1 = recorded, 2 = recorded + terminate.
__device__ inline int affect(const KParams& P, const SegIn& in, const SegOut& out, int64_t n, int64_t ray,
                             const double* u, double tau, double erg, int& ncross, int max_crossings) {
  double st, ct, sp, cp;
  msincos(u[1], st, ct);
  msincos(u[2], sp, cp);
  if (ncross == 0) {  // a "crossing" at the start point is not new (:303-314)
    const double s = 1.0001;
    const double pos[3] = {st * cp * u[0], st * sp * u[0], ct * u[0]};
    bool all_lt = true, all_gt = true;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double x0i = fabs(in.x0[i * n + ray]);
      all_lt = all_lt && (fabs(pos[i]) < x0i * s);
      all_gt = all_gt && (fabs(pos[i]) > x0i / s);
    }
    if (all_lt && all_gt) return 0;
  }
  double x[3], k[3];
  sph_to_cart(u, erg, P.rs_eff, x, k);
  if (sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) < P.rNS101) return 0;  // :322-324
  const int j = ncross;
  if (out.xcount && j < out.cap) {
    const double dwc = u[6] / erg;  // P_nonAD: finalize_kernel
    double2* rq = reinterpret_cast<double2*>(out.xrec + ((int64_t)ray * out.cap + j) * X_REC);
    rq[0] = make_double2(x[0], x[1]);
    rq[1] = make_double2(x[2], k[0]);
    rq[2] = make_double2(k[1], k[2]);
    rq[3] = make_double2(exp(tau), dwc);
  }
  ncross = j + 1;
  const int maxc = max_crossings <= 0 ? -1 : max_crossings;
  return (ncross >= maxc) ? 2 : 1;
}

// ---------------------------------------------------------------------------
// Stage glue, table-driven. Slot s (0-based) of an attempt evaluates the next stage at
//   y = u + h (cf[s] f + cA[s] kA + Σ_q cL[s][q] L_q),   t = τ + ct[s] h,
// where kA is ONE register-resident stage vector (k2, later k8 -- their lifetimes do not
// overlap) and L_0..L_4 are stage vectors parked in LDS (k3..k7 for Vern6; k3, k4 for RK4).
// Coefficients are wave-uniform scalar loads; the RHS is inlined once.
constexpr int LDS_SLOTS = 5;
// The wave-uniform scalars of one slot in one 48-byte row: a single scalar load and wait at
// the slot's start (the cL coefficients are loaded inside the LDS loop, where their latency
// overlaps the LDS reads).
struct alignas(16) SlotRow {
  double cf, cA, ct;
  int lmask;   // bit q: cL[s][q] != 0 -- the LDS slots stage s reads, one contiguous range
  int storeA;  // after the slot: kk -> kA?
  int storeL;  // after the slot: kk -> L[storeL] (-1: no)
  int pad;
};
struct StageTable {
  SlotRow row[8];
  double cL[8][LDS_SLOTS];
  double e_f, e_A, e_L[LDS_SLOTS], e_k;  // error weights (Vern6): btilde of f, kA(=k8), L, k9
};

// (static: both translation units, art_kernels.hip and art_kernels_nolicm.hip, hold their own copy)
static __constant__ StageTable c_vern6 = {
    // {cf = a_{s+2,1}, cA (k2 for slots 0..6, k8 for slot 7), ct, lmask, storeA, storeL}
    {{Vern6::a21, 0.0, Vern6::c2, 0x0, 1, -1, 0},
     {Vern6::a31, Vern6::a32, Vern6::c3, 0x0, 0, 0, 0},
     {Vern6::a41, 0.0, Vern6::c4, 0x1, 0, 1, 0},
     {Vern6::a51, 0.0, Vern6::c5, 0x3, 0, 2, 0},
     {Vern6::a61, 0.0, Vern6::c6, 0x7, 0, 3, 0},
     {Vern6::a71, 0.0, Vern6::c7, 0xf, 0, 4, 0},
     {Vern6::a81, 0.0, 1.0, 0x1f, 1, -1, 0},
     {Vern6::a91, Vern6::a98, 1.0, 0x1e, 0, -1, 0}},
    // cL: coefficients of k3..k7
    {{0, 0, 0, 0, 0},
     {0, 0, 0, 0, 0},
     {Vern6::a43, 0, 0, 0, 0},
     {Vern6::a53, Vern6::a54, 0, 0, 0},
     {Vern6::a63, Vern6::a64, Vern6::a65, 0, 0},
     {Vern6::a73, Vern6::a74, Vern6::a75, Vern6::a76, 0},
     {Vern6::a83, Vern6::a84, Vern6::a85, Vern6::a86, Vern6::a87},
     {0, Vern6::a94, Vern6::a95, Vern6::a96, Vern6::a97}},
    Vern6::e1, Vern6::e8, {0.0, Vern6::e4, Vern6::e5, Vern6::e6, Vern6::e7}, Vern6::e9};

static __constant__ StageTable c_rk4 = {
    {{0.5, 0.0, 0.5, 0x0, 1, -1, 0},
     {0.0, 0.5, 0.5, 0x0, 0, 0, 0},
     {0.0, 0.0, 1.0, 0x1, 0, 1, 0},
     {1.0 / 6.0, 2.0 / 6.0, 1.0, 0x3, 0, -1, 0},
     {0, 0, 0, 0, 0, -1, 0}, {0, 0, 0, 0, 0, -1, 0}, {0, 0, 0, 0, 0, -1, 0}, {0, 0, 0, 0, 0, -1, 0}},
    {{0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {1.0, 0, 0, 0, 0}, {2.0 / 6.0, 1.0 / 6.0, 0, 0, 0},
     {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}},
    0.0, 0.0, {0, 0, 0, 0, 0}, 0.0};

enum LaneMode { M_IDLE = 0, M_STEP = 2, M_ROOT = 3 };

// Lanes per block of the persistent integrator. A block retires only when all its waves are
// done, so smaller blocks free their CU slots sooner while a launch drains (the next launch,
// on another stream, fills them).
#ifndef ART_BLOCK
#define ART_BLOCK 256
#endif
constexpr int BLOCK = ART_BLOCK;
constexpr int SCAN_WORDS = 4;  // 2-bit codes for up to 64 grid points (interp_points <= 65)
// Waves per SIMD the integrator is register-budgeted for (1: 512 VGPR+AGPR, 2: 256).
// Loop-carried per-lane flags: bool lets the compiler keep them as 64-bit lane masks in SGPR
// pairs, which the integrator's SGPR pressure spills to VGPR lanes; int keeps them in VGPRs.
#ifndef ART_LBOOL
#define ART_LBOOL int
#endif
#ifndef ART_LBOOL2
#define ART_LBOOL2 int  // per-iteration flags too (A/B: 1e7 flat -0.7%)
#endif
#ifndef ART_SUNROLL
#define ART_SUNROLL 1  // the stage slot loop: one RHS site
#endif
#ifndef ART_SUNROLL_GR
#define ART_SUNROLL_GR 2  // GR: two RHS sites (A/B: lone GR tail ray -6%; flat: bulk +-0, lone +1%)
#endif
#ifndef ART_QUNROLL
#define ART_QUNROLL 5  // = LDS_SLOTS: the slot range fully unrolled (A/B: -0.8% bulk, -3% lone ray)
#endif
#ifndef ART_PRIO_ITERS
#define ART_PRIO_ITERS 1024
#endif
#ifndef ART_WAVES_PER_SIMD
#define ART_WAVES_PER_SIMD 2
#endif
#ifndef ART_STREAM_FLUSH
// (DON = 3) a wave's finished-ray counts go out every 128 iterations (~2.5 ms of a flat ray's
// steps; every 8: -3%, every 32: -1%, profiles/r03sg_flush.jsonl)
#define ART_STREAM_FLUSH 127
#endif

// ---------------------------------------------------------------------------
// One loop iteration = one step attempt for every live lane: a runtime loop over the
// stage slots with the RHS inlined once. A lane that takes a new ray loads its fresh state
// (init_kernel) and steps in the same iteration; lanes polishing a crossing (M_ROOT)
// re-step from the step start. After the slots, the wave-cooperative scan and one per-lane
// condition call site (brackets, Illinois, root polish) serve the ContinuousCallback.
// GEOM_FLAT: flat space, no boundary layer, anisotropic plasma (the headline workload). The
// kernel then works on a copy of the parameters whose rs_eff, bndry_lyr and isotropic are
// compile-time constants, so the Schwarzschild, boundary-layer and isotropic branches of
// the physics fold away instead of holding registers. GEOM_ANY reads them at run time.
// GEOM_GR: Schwarzschild (rs > 0), no boundary layer, anisotropic (configs[3]): only the
// boundary-layer and isotropic branches fold away, and rs != 0 is assumed.
enum { GEOM_ANY = 0, GEOM_FLAT = 1, GEOM_GR = 2 };

// (DON = 3) a wave's LDS histogram of finished rays per piece (lane l: piece l) into the
// pieces' global counts: the wave's end-record stores released once (agent scope), then one
// atomic add per piece with a count (the helpers poll piece_cnt)
__device__ inline void stream_flush(const SegOut& out, unsigned* hist, int lane) {
  const unsigned c = hist[lane];
  if (__ballot(c != 0u) == 0ull) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the write-back done before the counts, always)
  if (c != 0u) {
    hist[lane] = 0u;
    __hip_atomic_fetch_add(out.piece_cnt + lane, (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One ray's complete integrator state as a CONT_REC record (tail donation, graduation):
// [u (7) | f (7) | τ, dt, qpow, cprev, bstart, erg | int4 {ray, n_acc, n_rej, ncross} |
//  int4 {iter, sprev, flags, save_k}]
__device__ inline void write_cont_rec(double* rec, const double* u, const double* f, double tau, double dt, double qpow,
                                      double cprev, double bstart, double erg, int ray, int n_acc, int n_rej,
                                      int ncross, int iter, int sprev, bool photon, bool cprev_ok, bool just_evented,
                                      int save_k) {
  double2* rq = reinterpret_cast<double2*>(rec);
  const double v[20] = {u[0], u[1], u[2], u[3], u[4], u[5], u[6], f[0], f[1], f[2],
                        f[3], f[4], f[5], f[6], tau, dt, qpow, cprev, bstart, erg};
#pragma unroll
  for (int i = 0; i < 10; ++i) rq[i] = make_double2(v[2 * i], v[2 * i + 1]);
  int4* ri = reinterpret_cast<int4*>(rq + 10);
  ri[0] = make_int4(ray, n_acc, n_rej, ncross);
  ri[1] = make_int4(iter, sprev, (photon ? 1 : 0) | (cprev_ok ? 2 : 0) | (just_evented ? 4 : 0), save_k);
}

template <int GEOM>
__device__ inline KParams specialize(const KParams& P) {
  KParams Q = P;
  if (GEOM == GEOM_FLAT) {
    Q.rs_eff = 0.0;
    Q.bndry_lyr = -1.0;
    Q.isotropic = 0;
    Q.cert_rmin = 0.0;
  } else if (GEOM == GEOM_GR) {
    __builtin_assume(Q.rs_eff > 0.0);
    Q.bndry_lyr = -1.0;
    Q.isotropic = 0;
  }
  return Q;
}

// Fresh state of ray i (init_kernel; the maskless streamed integrator, DON = 3, runs it for
// each chunk it claims): u0 (RayTracer.jl:179-216: k_norm_Cart onto the axion shell, Cartesian
// -> (r, θ, φ), covariant celerity), f(u0) with the hamiltonian's in-place clamp (:531), the
// initial dt (ode_determine_initdt, order 6, with its probe RHS; RK4: the fixed step) and the
// condition value that seeds the callback's sign memory, into the ray's fresh-state record
// (U0_REC doubles at in.u0 + i U0_REC: [u0 (7) | f0 (7) | dt | c0 | erg | ln t0 | species | 0]),
// ten 16-byte stores. Returns the RHS evaluations it took.
__device__ inline unsigned init_one(const KParams& P, int64_t n, int64_t i, const SegIn& in) {
  const double xs[3] = {in.x0[i], in.x0[n + i], in.x0[2 * n + i]};
  const double ks[3] = {in.k0[i], in.k0[n + i], in.k0[2 * n + i]};
  const double erg = in.erg[i], tau = in.lnt0[i];
  const bool photon = in.species[i] != ART_AXION;
  double u[7], f[7], y[7];
  initial_state(P, xs, ks, erg, in.dw[i], u);
  // pass 0: f(u0); pass 1 (Vern6, when initdt asks for it): its probe f(u1). One inlined RHS site:
  // with two, the helper kernel needed more than the 256 VGPRs of 2 waves per SIMD and spilled
  double dt = P.integrator == ART_RK4 ? (P.ln_t_end - tau) / P.n_fixed : NAN;
  InitDt ids;
  unsigned nrhs = 0;
#pragma unroll
  for (int c = 0; c < 7; ++c) y[c] = u[c];
  double ty = tau;
  for (int pass = 0; pass < 2; ++pass) {
    double r[7];
    rhs(P, photon, y, ty, erg, r);
    ++nrhs;
    if (pass == 0) {
#pragma unroll
      for (int c = 0; c < 7; ++c) f[c] = r[c];
      if (photon && u[0] < P.rNS) u[0] = P.rNS;  // hamiltonian's in-place clamp (:531)
      if (P.integrator == ART_RK4) break;
      dt = initdt_begin(P, u, f, tau, P.ln_t_end - tau, ids, y);
      if (!isnan(dt)) break;
      ty = tau + ids.dt0;
    } else {
      dt = initdt_end(P, f, r, P.ln_t_end - tau, ids);
    }
  }
  const double c0 = condition_t(P, u, fexp(tau));
  const double v[U0_REC] = {u[0], u[1], u[2], u[3], u[4], u[5], u[6], f[0], f[1], f[2],
                            f[3], f[4], f[5], f[6], dt,   c0,   erg,  tau,  photon ? 1.0 : 0.0, 0.0};
  double2* rq = reinterpret_cast<double2*>(in.u0 + i * U0_REC);
#pragma unroll
  for (int c = 0; c < U0_REC / 2; ++c) rq[c] = make_double2(v[2 * c], v[2 * c + 1]);
  return nrhs;
}

// np.histogram's bin of x for `nbins` equal bins over [-π, π] (numpy 2.x histogram: the
// index from (x - lo) / (hi - lo) * nbins, then corrected against the edges of
// linspace(lo, hi, nbins + 1) = i * ((hi - lo) / nbins) + lo, the right edge in the last bin),
// with the same roundings: no contraction into FMAs. -1 outside [lo, hi] (and for NaN).
// The range defaults to flux_kernel's fixed [-π, π]; flux_phi_kernel also takes a data-dependent
// one (np.histogram(a, bins) without `range` bins over [a.min(), a.max()], plot/flux.py:43-47).
__device__ inline int np_hist_bin(double x, int nbins, double lo = -PI, double hi = PI) {
#pragma clang fp contract(off)  // numpy rounds every product and sum (HIP's __dmul_rn would still fuse)
  if (!(x >= lo && x <= hi)) return -1;
  const double span = hi - lo;
  int i = (int)(((x - lo) / span) * (double)nbins);
  if (i == nbins) i -= 1;
  const double step = span / (double)nbins;
  const double e0 = (double)i * step + lo;
  if (x < e0) i -= 1;
  const double e1 = (i + 1 == nbins) ? hi : (double)(i + 1) * step + lo;
  if (x >= e1 && i != nbins - 1) i += 1;
  return i;
}

// The radiated-flux bin of one segment's end state (plot/flux.py:38-48 over a batch's escaping
// segments): is_final -- no crossing and escaped beyond 1.1 rNS (MainRunner.jl:203-209) -- and
// the azimuth of its momentum binned as np.histogram(range = (-π, π)); -1 = not counted.
// flux_kernel and the streamed pipeline's helpers (finalize_one) both bin through here.
__device__ inline int flux_bin_of(const KParams& P, const double* x, const double* k, int status, int nbins) {
  const double xr = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  if (status == ART_STATUS_CROSSING || !(xr > 1.1 * P.rNS)) return -1;
  return np_hist_bin(atan2(k[1], k[0]), nbins);
}

// End state of ray i in Cartesian form (back-transform, RayTracer.jl:393-416) from the raw end
// record the integrator left in out.rec, spread into the SoA outputs at o (row stride m), and
// the conversion probability of every recorded crossing (get_Prob_nonAD with Nc = 1,
// MainRunner.jl:265). finalize_kernel runs it one thread per ray; the maskless streamed
// integrator (DON = 3) for each chunk whose rays have all finished.
__device__ inline void finalize_one(const KParams& P, int64_t n, int64_t i, int64_t o, int64_t m, const SegIn& in,
                                    const SegOut& out, double* fl = nullptr, int fl_nbins = 0) {
  const double erg = in.erg[i];
  int ncross = 0;
  {
    const double2* rq = reinterpret_cast<const double2*>(out.rec + i * END_REC);
    double u[7], xe[3], ke[3];
    const double2 q0 = rq[0], q1 = rq[1], q2 = rq[2], q3 = rq[3];
    const int4 ri = reinterpret_cast<const int4*>(rq + 4)[0];
    u[0] = q0.x; u[1] = q0.y; u[2] = q1.x; u[3] = q1.y; u[4] = q2.x; u[5] = q2.y; u[6] = q3.x;
    back_transform(P, u, erg, xe, ke);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      out.x_end[c * m + o] = xe[c];
      out.k_end[c * m + o] = ke[c];
    }
    out.u7_end[o] = u[6];
    out.tau_end[o] = q3.y;
    out.status[o] = ri.x;
    out.n_acc[o] = ri.y;
    out.n_rej[o] = ri.z;
    ncross = ri.w;
    if (out.xcount) out.xcount[o] = ncross;
    if (out.ntimes >= 2) out.traj_n[o] = reinterpret_cast<const int4*>(rq + 4)[1].x;
    if (fl) {  // (the streamed pipeline's helpers: the ray's radiated-flux bin, an exact count)
      const int bin = flux_bin_of(P, xe, ke, ri.x, fl_nbins);
      if (bin >= 0) atomicAdd(&fl[(in.species[i] == ART_AXION ? 0 : 1) * fl_nbins + bin], 1.0);
    }
  }
  if (out.ntimes >= 2) {  // saveat: start (u0 back-transformed), interior to Cartesian, end
    double u0[7], xs[3], ks[3];
#pragma unroll
    for (int c = 0; c < 7; ++c) u0[c] = in.u0[i * U0_REC + c];
    back_transform(P, u0, erg, xs, ks);
    const int mt = out.traj_n[o];
    for (int k = 0; k < mt; ++k) {
      double x[3];
      if (k == 0) {
        x[0] = xs[0]; x[1] = xs[1]; x[2] = xs[2];
        out.traj_t[o] = in.lnt0[i];
      } else if (k == mt - 1) {
        x[0] = out.x_end[o]; x[1] = out.x_end[m + o]; x[2] = out.x_end[2 * m + o];
        out.traj_t[int64_t(k) * m + o] = out.tau_end[o];
      } else {
        const double r = out.traj[(int64_t(0) * out.ntimes + k) * m + o];
        double st, ct, sp, cp;
        msincos(out.traj[(int64_t(1) * out.ntimes + k) * m + o], st, ct);
        msincos(out.traj[(int64_t(2) * out.ntimes + k) * m + o], sp, cp);
        x[0] = r * st * cp; x[1] = r * st * sp; x[2] = r * ct;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) out.traj[(int64_t(c) * out.ntimes + k) * m + o] = x[c];
    }
  }
  if (!out.xcount) return;
  const int mc = ncross < out.cap ? ncross : out.cap;
  for (int j = 0; j < mc; ++j) {
    const double2* rq = reinterpret_cast<const double2*>(out.xrec + (i * out.cap + j) * X_REC);
    const double2 q0 = rq[0], q1 = rq[1], q2 = rq[2], q3 = rq[3];
    const double x[3] = {q0.x, q0.y, q1.x}, k[3] = {q1.y, q2.x, q2.y};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      out.xpos[(int64_t(c) * out.cap + j) * m + o] = x[c];
      out.xk[(int64_t(c) * out.cap + j) * m + o] = k[c];
    }
    out.xt[int64_t(j) * m + o] = q3.x;
    const double dwc = q3.y;
    out.xdw[int64_t(j) * m + o] = dwc;
    out.xp[int64_t(j) * m + o] = prob_nonad_single(P, x, k, erg * fabs(dwc));  // erg_inf_ini .* abs.(Δωc)
  }
  if (out.nan_fill) {
    for (int j = mc; j < out.cap; ++j) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        out.xpos[(int64_t(c) * out.cap + j) * m + o] = NAN;
        out.xk[(int64_t(c) * out.cap + j) * m + o] = NAN;
      }
      out.xt[int64_t(j) * m + o] = NAN;
      out.xdw[int64_t(j) * m + o] = NAN;
      out.xp[int64_t(j) * m + o] = NAN;
    }
  }
}

// (DON = 3) the SoA output blob of piece p (art_capi.cpp, propagate_host_maskless: the same
// layout and 256-byte alignments), its rows m long
__device__ inline SegOut piece_blob(const SegOut& out, int64_t n, int p, int64_t& m) {
  const int64_t lo = (int64_t)p << out.piece_shift;
  const int64_t full = (int64_t)1 << out.piece_shift;
  m = (n - lo) < full ? n - lo : full;
  auto up = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  char* db = out.blob + (int64_t)p * out.blob_stride;
  double* dd = (double*)db;
  int32_t* di32 = (int32_t*)(dd + 8 * m);
  SegOut ol{};
  ol.x_end = dd; ol.k_end = dd + 3 * m; ol.u7_end = dd + 6 * m; ol.tau_end = dd + 7 * m;
  ol.status = di32; ol.n_acc = di32 + m; ol.n_rej = di32 + 2 * m;
  ol.rec = out.rec;
  if (out.cap) {
    const int64_t cnt = up(m * 8 * 8 + m * 3 * 4);
    double* x = (double*)(db + cnt + up(m * 4));
    ol.cap = out.cap;
    ol.xcount = (int32_t*)(db + cnt);
    ol.xpos = x; ol.xk = x + 3 * out.cap * m; ol.xt = x + 6 * out.cap * m; ol.xdw = x + 7 * out.cap * m;
    ol.xp = x + 8 * out.cap * m;
    ol.xrec = out.xrec;
    ol.nan_fill = 1;
  }
  return ol;
}

// ---- the maskless streamed pipeline's helper duty (DON = 3, SegOut::helpers) ----
constexpr int S3_TILE = HELPER_TILE;  // (4 rays per thread: the claim, the barriers and the L2 write-back of
                                     // the hand-off amortised over 4 rays)
constexpr unsigned long long S3_WAIT_TICKS = 2000000000ull;  // 20 s of s_memrealtime without progress: give up

__device__ inline unsigned long long ld_sys(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline bool ld_abort(const SegOut& out) {
  return __hip_atomic_load(out.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

// (DON = 3) the claimed chunk's fresh state: its flag as the leader lane reads it now, or after
// a bounded wait (false: the wait timed out or another wave gave up; the wave stops taking rays)
__device__ inline bool chunk_flag(const SegOut& out, int wnext, int leader) {
  unsigned v = 0;
  if ((int)(threadIdx.x & 63) == leader)
    v = __hip_atomic_load(out.chunk_ready + wnext / CHUNK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readlane((int)v, leader) != 0;
}
__device__ inline bool chunk_wait(const SegOut& out, int wnext, int leader) {
  int ok = 1;
  if ((int)(threadIdx.x & 63) == leader) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(out.chunk_ready + wnext / CHUNK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      if (__hip_atomic_load(out.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
          __builtin_amdgcn_s_memrealtime() - t0 > out.wait_ticks) {
        __hip_atomic_store(out.abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(32);
    }
  }
  return __shfl(ok, leader) != 0;
}

// The hot rule (SegOut::hot): a ray that has advanced less than hot_dtau + hot_slope
// log2(attempts / 256) in ln t since its start
__device__ inline bool hot_lags(const SegOut& out, double dtau, double log2_att_256) {
  return dtau < out.hot_dtau + out.hot_slope * log2_att_256;
}

// DON: the tail-donation instantiations (SegOut::donate / cont_mode honoured); the others
// carry none of that code, so a lone pass pays nothing for it
// WPS: waves per SIMD the registers are budgeted for (the default 2; the GR continuation
// launch, below, uses 1)
template <int INTEG, int GEOM, bool SAVE, int DON, int WPS = ART_WAVES_PER_SIMD>
__global__ __launch_bounds__(BLOCK, WPS) void propagate_kernel(const KParams P_in, const int64_t n,
                                                                              const SegIn in, const SegOut out,
                                                                              const int32_t max_crossings,
                                                                              unsigned long long* __restrict__ queue,
                                                                              unsigned long long* __restrict__ stats) {
  const KParams P = specialize<GEOM>(P_in);
  constexpr bool RK4 = (INTEG == ART_RK4);
  // the work queue: fresh rays [0, n), or in a continuation launch the donated records
  const bool cont = DON == 1 && out.cont_mode;
  const int64_t nq = cont ? (int64_t)*out.cont_src_count : n;
  unsigned long long* const rqueue = cont ? out.cont_queue : queue;
  // the callbacks (RayTracer.jl:357-368) are installed only when make_tree (:361-377)
  const bool cbs = max_crossings != ART_NO_CALLBACKS;
  constexpr int NSLOT = RK4 ? 4 : 8;
  constexpr int SUNROLL = GEOM == GEOM_GR ? ART_SUNROLL_GR : ART_SUNROLL;
  const StageTable& T = RK4 ? c_rk4 : c_vern6;
  __shared__ double lds[LDS_SLOTS * 7 * BLOCK];  // [slot][component][lane]: conflict-free ds_read_b64
  __shared__ unsigned codes[SCAN_WORDS * BLOCK];  // [word][lane]: 2-bit sign codes of the grid scan
  __shared__ double lastv[BLOCK];                 // value at the last grid point (before: b at the step's end)
  __shared__ double lastt[BLOCK];                 // t at the step's end (the scan certificate)
  __shared__ unsigned char srcl[BLOCK];           // compact list of the wave's scanning lanes
  __shared__ double thgrid[SCAN_WORDS * 16 + 1];  // Θs = j/(npts-1): range(0, 1, length = npts)
  __shared__ unsigned pend_lds[BLOCK / 64][64];  // (DON = 3) per wave: finished rays per piece, not yet counted
  double* const L = lds + threadIdx.x;
  const int wbase = threadIdx.x & ~63;
  const int lane = threadIdx.x & 63;
  const double tend = P.ln_t_end;
  const int npts = P.interp_points;
  for (int j = threadIdx.x; j < npts; j += BLOCK) thgrid[j] = double(j) / double(npts - 1);
  if constexpr (DON == 3) {
    pend_lds[threadIdx.x >> 6][threadIdx.x & 63] = 0u;
    if (out.waves_started && (threadIdx.x & 63) == 0) {
      const unsigned long long old =
          __hip_atomic_fetch_add(out.waves_started, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (out.resident_host && old + 1ull == (unsigned long long)out.waves_total)  // (a vector store to host memory)
        __hip_atomic_store(out.resident_host, out.resident_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  span_stamp(stats, false);
  __syncthreads();

  int mode = M_IDLE;
  int ray = -1;
  ART_LBOOL photon = true;
  double erg = 0.0;
  // qpow = qold^(1/15) of the PI controller, updated only when qold changes (on accept)
  const double qpow_init = pow(1e-4, 1.0 / 15.0);
  double u[7], f[7], tau = 0.0, dt = 0.0, qpow = qpow_init;
  double cprev = 0.0;
  double bstart = NAN;  // Bz/B_n at u (the previous step's last RHS) for the scan certificate
  ART_LBOOL cprev_ok = true;  // cprev holds the condition at the step start (false after a certified step)
  int sprev = 0;
  ART_LBOOL just_evented = false;
  int n_acc = 0, n_rej = 0, ncross = 0, iter = 0;
  double hroot = 0.0, r_tha = 0.0, r_ca = 0.0, r_thb = 0.0, r_cb = 0.0, r_t = 0.0, r_slope = 1.0, post_c = 0.0;
  int post_s = 0, r_side = 0, r_it = 0;
  int wnext = 0, wend = 0;
  int tick = 0;                          // (DON = 3) iterations, for the flushes of the piece counts
  bool cready = false;                   // (DON = 3) the claimed chunk's fresh state is in
  int save_k = 1;  // SAVE: the next interior saveat index
  bool exhausted = false;
  unsigned s_att = 0, s_acc = 0, s_root = 0, s_scan = 0, s_interp = 0, s_rays = 0, s_cert = 0;
#ifdef ART_SECTION_TIMING
  // dev build: s_memtime cycles per main-loop section, summed over the wave's iterations
  unsigned long long t_sec[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#define ART_TMARK(k)                                                  \
  {                                                                   \
    const unsigned long long t_now_ = __builtin_amdgcn_s_memtime();   \
    t_sec[k] += t_now_ - t_last;                                      \
    t_last = t_now_;                                                  \
  }
#else
#define ART_TMARK(k)
#endif
#pragma unroll
  for (int i = 0; i < 7; ++i) { u[i] = 0.0; f[i] = 0.0; }

  while (true) {
    // ---- refill idle lanes from the wave's chunk (one atomicAdd per 64 rays) ----
    if (!exhausted) {
      unsigned long long need = __ballot(mode == M_IDLE);
      while (need != 0ull) {
        if (wnext >= wend) {
          unsigned long long base = 0;
          const int leader = __ffsll((long long)need) - 1;
          if (lane == leader) base = atomicAdd(rqueue, (unsigned long long)CHUNK);
          base = __shfl(base, leader);
          if ((int64_t)base >= nq) { exhausted = true; break; }
          wnext = __builtin_amdgcn_readfirstlane((int)base);
          wend = __builtin_amdgcn_readfirstlane((int)((int64_t)base + CHUNK < nq ? (int64_t)base + CHUNK : nq));
          cready = false;
        }
        int lim = wend;
        if constexpr (DON == 3) {
          // the chunk's fresh state (the helpers' chunk flag); while it is not in, a wave with
          // other rays goes on integrating them, and an empty wave waits (bounded)
          if (!cready) {
            const int leader = __ffsll((long long)need) - 1;
            if (!chunk_flag(out, wnext, leader)) {
              if (lane == leader) atomicAdd(out.init_next + 2, 1ull);  // (the misses, for the host's trace)
              if (__ballot(mode != M_IDLE) != 0ull) break;
              if (!chunk_wait(out, wnext, leader)) { exhausted = true; break; }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            cready = true;
          }
        }
        const int rank = __popcll(need & ((1ull << lane) - 1ull));
        const int cnt = __popcll(need);
        const int take = (lim - wnext) < cnt ? (lim - wnext) : cnt;
        if (mode == M_IDLE && rank < take && cont) {
          // a donated ray: its complete state from the tail-donation record
          mode = M_STEP;
          const double2* rq = reinterpret_cast<const double2*>(out.cont_src + (int64_t)(wnext + rank) * CONT_REC);
          double v[20];
#pragma unroll
          for (int i = 0; i < 10; ++i) {
            const double2 q = rq[i];
            v[2 * i] = q.x;
            v[2 * i + 1] = q.y;
          }
#pragma unroll
          for (int i = 0; i < 7; ++i) {
            u[i] = v[i];
            f[i] = v[7 + i];
          }
          tau = v[14];
          dt = v[15];
          qpow = v[16];
          cprev = v[17];
          bstart = v[18];
          erg = v[19];
          const int4 i0 = reinterpret_cast<const int4*>(rq + 10)[0], i1 = reinterpret_cast<const int4*>(rq + 10)[1];
          ray = i0.x;
          n_acc = i0.y;
          n_rej = i0.z;
          ncross = i0.w;
          iter = i1.x;
          sprev = i1.y;
          save_k = i1.w;
          photon = i1.z & 1;
          cprev_ok = (i1.z >> 1) & 1;
          just_evented = (i1.z >> 2) & 1;
        } else if (mode == M_IDLE && rank < take) {
          ray = (DON == 1 && out.order) ? out.order[wnext + rank] : wnext + rank;
          mode = M_STEP;
          // fresh segment: u0, f(u0), the initial dt and the initial condition value, all
          // precomputed by the init pass, with erg, ln t0 and the species: one 160-byte record
          const double2* rq = reinterpret_cast<const double2*>(in.u0 + (int64_t)ray * U0_REC);
          double v[U0_REC - 2];
#pragma unroll
          for (int i = 0; i < U0_REC / 2 - 1; ++i) {
            const double2 q = rq[i];
            v[2 * i] = q.x;
            v[2 * i + 1] = q.y;
          }
          const double sp = rq[U0_REC / 2 - 1].x;
#pragma unroll
          for (int i = 0; i < 7; ++i) {
            u[i] = v[i];
            f[i] = v[7 + i];
          }
          dt = v[14];
          cprev = v[15];
          erg = v[16];
          tau = v[17];
          photon = sp != 0.0;
          cprev_ok = true;
          bstart = NAN;
          sprev = isnan(cprev) ? 0 : sgn(cprev);
          n_acc = n_rej = ncross = iter = 0;
          save_k = 1;
          just_evented = false;
          qpow = qpow_init;  // qoldinit = 1e-4
          s_rays += 1;
        }
        wnext += take;
        need = __ballot(mode == M_IDLE);
      }
    }
    if (__ballot(mode != M_IDLE) == 0ull) break;  // every lane idle and the queue drained
    // A wave holding an outlier ray (ART_PRIO_ITERS attempts and more: ~20x the mean) asks the
    // SIMD's arbiter for issue priority. The one ray that sets a launch's (or a scan point's)
    // drain time then runs at close to its lone-wave speed while the bulk of the batch still
    // shares its SIMD; the other waves fill the issue slots it leaves.
    const bool outlier = __ballot(iter >= ART_PRIO_ITERS) != 0ull;
    if (outlier) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(0);
    ART_TMARK(0)  // refill

    // ---- this iteration's step size ----
    ART_LBOOL2 last = false, forced = false;
    double hs = 0.0;
    if (mode == M_ROOT) {
      hs = r_t * hroot;
    } else if (mode == M_STEP) {
      hs = dt;  // (min(dt, dtmax) is implied: the span end clips every step)
      if (tau + hs >= tend) { hs = tend - tau; last = true; }
      else if (!RK4 && hs < P.dtmin) { hs = P.dtmin; forced = true; }
    }

    // ---- stage slots: one RHS per slot per lane ----
    double kA[7], y[7], kk[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) kA[i] = 0.0;  // read (times a zero coefficient) before its first store
    // flat builds: the next slot's row of scalars is loaded before this slot's RHS, so its
    // scalar-load latency hides behind the RHS instead of opening the next slot: 1e7 flat device
    // launch 84.0 -> 83.4 ms (3 interleaved pairs, profiles/r05c_ab_prefetch.jsonl); the GR build
    // (slot loop unrolled by two) lost 0.5% with it (profiles/r05d_ab_gr_prefetch.txt)
    constexpr bool PF = GEOM == GEOM_FLAT;
    SlotRow Rnext = T.row[0];
#pragma unroll SUNROLL
    for (int s = 0; s < NSLOT; ++s) {
      const SlotRow R = PF ? Rnext : T.row[s];
      const double cf = R.cf, cA = R.cA;
      double acc[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) acc[i] = cf * f[i];
      if (cA != 0.0) {  // wave-uniform: only Vern6's a32 and a98 rows use the register stage
#pragma unroll
        for (int i = 0; i < 7; ++i) acc[i] = fma(cf, f[i], cA * kA[i]);  // (the rounding of the general form)
      }
      // the LDS slots this stage reads form one contiguous range [qlo, qhi) (lmask): no
      // per-slot load-compare-branch, and each coefficient load overlaps the slot's LDS reads
      const int lm = R.lmask;
      if (lm != 0) {
        const int qhi = 32 - __builtin_clz(lm);
#pragma unroll ART_QUNROLL
        for (int q = __builtin_ctz(lm); q < qhi; ++q) {
          const double c = T.cL[s][q];
#pragma unroll
          for (int i = 0; i < 7; ++i) acc[i] += c * L[(q * 7 + i) * BLOCK];
        }
      }
#pragma unroll
      for (int i = 0; i < 7; ++i) y[i] = u[i] + hs * acc[i];
      const double ty = tau + R.ct * hs;
      if constexpr (PF) Rnext = T.row[s + 1 < NSLOT ? s + 1 : s];
      // Every lane evaluates the photon RHS -- idle lanes (a draining wave) on stale state,
      // whose results nothing reads -- so the slot has no divergent control flow. Axion
      // segments (the tree driver's batches) take a wave-uniform detour and a select.
      double aux[2];
      if constexpr (GEOM != GEOM_ANY) rhs_photon_gj(P, y, ty, erg, kk, aux);
      else rhs_photon(P, y, ty, erg, kk, aux);
      if (s == NSLOT - 1) {  // the end point's b and t for the scan certificate (lastv and codes are free)
        lastv[threadIdx.x] = aux[0];
        lastt[threadIdx.x] = aux[1];
      }
      if (__ballot(!photon) != 0ull) {
        double ka[7];
        rhs_axion(P, y, ty, erg, ka);
#pragma unroll
        for (int i = 0; i < 7; ++i) kk[i] = photon ? kk[i] : ka[i];
      }
      if (R.storeA) {
#pragma unroll
        for (int i = 0; i < 7; ++i) kA[i] = kk[i];
      }
      const int sl = R.storeL;
      if (sl >= 0) {
#pragma unroll
        for (int i = 0; i < 7; ++i) L[(sl * 7 + i) * BLOCK] = kk[i];
      }
    }
    ART_TMARK(1)  // step size and stage slots
    // The rest of the iteration -- error norm, controller, certificate, scan, walk, refill --
    // is latency-bound (short dependent chains, LDS round trips, the loads of a refill), the
    // stage slots issue-bound. At a higher issue priority than the partner wave's stage slots,
    // its instructions issue as soon as they are ready and the slots fill the gaps, instead of
    // the older wave's slots taking every issue cycle while this wave's chain waits behind
    // them (the arbiter goes by priority, then age). The priority drops back to the slots' level
    // at the top of the next iteration. 1e7 flat rays: 84.34 -> 82.53 ms (profiles/r04b_ab.txt,
    // 3 interleaved runs each); the grid pass at the slots' priority instead: 81.69 against
    // 81.42 (profiles/r04c_ab_grid_prio.txt). ART_NO_PRIO_PHASE switches it off (A/B).
    if (outlier) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(1);
    // y = u_{n+1}, kk = f(u_{n+1}) for stepping lanes
    // EEst² = mean of the 7 squared scaled errors: the controller needs EEst only through
    // EEst <= 1 and its logarithm (ln EEst = ½ ln EEst²), so no square root is taken
    double EEst2 = 0.0;
    if (mode == M_STEP || mode == M_ROOT) {
      if (photon && y[0] < P.rNS) y[0] = P.rNS;  // clamp on the FSAL stage (:531)
      if (!RK4) {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 7; ++i) {
          // explicit FMAs: the contraction of a sum of three products is the compiler's choice
          // (it prefers the product with fewer uses), so written out it could round differently
          // in the tail kernel's straight-line code (tests/test_gpu_tail_donation.py)
          double e = fma(T.e_k, kk[i], fma(T.e_A, kA[i], T.e_f * f[i]));
#pragma unroll
          for (int q = 1; q < LDS_SLOTS; ++q) e = fma(T.e_L[q], L[(q * 7 + i) * BLOCK], e);
          e *= hs;
          const double q = e * frcp(P.abstol + fmax_abs(u[i], y[i]) * P.reltol);
          acc += q * q;
        }
        EEst2 = acc * (1.0 / 7.0);
      }
    }

    // ---- controller (STEP lanes) ----
    int finish = -1;
    ART_LBOOL2 scan = false;  // accepted step to be scanned for sign changes
    double dtnext = dt;
    if (mode == M_STEP) {
      s_att += 1;
      ++iter;
      bool finite = !isnan(EEst2) && !isinf(EEst2);
#pragma unroll
      for (int i = 0; i < 7; ++i) finite = finite && !isnan(y[i]) && !isinf(y[i]);
      if (!finite) {
        finish = ART_STATUS_NONFINITE;
      } else {
        // PI controller (OrdinaryDiffEq: beta1 = 7/60, beta2 = 1/15, gamma = 0.9, qmin = 0.2, qmax = 10)
        // EEst^(7/60) and max(EEst, 1e-4)^(1/15) are the 7th and 4th powers of y = EEst^(1/60)
        // = (EEst²)^(1/120): one logarithm and one exponential (OrdinaryDiffEq itself uses
        // FastPower.fastpower, an exp2/log2 approximation)
        double q = 1.0, q11 = 1.0, y60 = 0.0;
        bool accept = true;
        if (!RK4) {
          if (EEst2 == 0.0) {
            q = 0.1;
          } else {
            y60 = fexp(flog(EEst2) * (1.0 / 120.0));
            const double y2 = y60 * y60;
            q11 = (y2 * y2) * (y2 * y60);
            q = q11 * frcp(qpow);
            q = fmax(0.1, fmin(5.0, q * (1.0 / 0.9)));
          }
          accept = (EEst2 <= 1.0) || forced;
        }
        if (!accept) {
          dt = hs * frcp(fmin(5.0, q11 * (1.0 / 0.9)));
          ++n_rej;
          if (iter >= P.maxiters) finish = ART_STATUS_MAXITERS;
        } else {
          ++n_acc;
          s_acc += 1;
          if (!RK4) {
            const double ym = fmax(y60, 0.8576958985908941);  // (1e-4)^(1/60)
            qpow = (ym * ym) * (ym * ym);
            dtnext = hs * frcp(q);
          }
          scan = true;
        }
      }
    }

    // ---- resonance scan of the accepted steps (ContinuousCallback, RayTracer.jl:357-358) ----
    // (a) Wave-cooperative grid pass: every lane of the wave evaluates (source lane, grid
    //     point) items of all the wave's accepted steps, so lanes whose attempt was rejected
    //     (and the idle lanes of a draining wave) share the 49-point scans instead of waiting.
    //     Each item leaves a 2-bit sign code in the source lane's LDS words.
    const int nper = npts - 1;
    // (0) certified steps (scan_certified_code, art_core.h): every grid point of the step
    //     provably has a positive (1), negative (2) or undefined (3, NaN) condition, so its codes are
    //     known without evaluating them; its end value is not needed unless the next step
    //     opens a bracket at its start (then it is recomputed there, bit-identically:
    //     cprev_ok = false).
    // without callbacks (make_tree = false: ART_NO_CALLBACKS) every step is "certified NaN":
    // no sign change can open a bracket, so nothing is scanned or recorded
    const double bend = lastv[threadIdx.x];
    const int ccode =
        !scan ? 0 : (cbs ? scan_certified_code(P, u, f, y, kk, hs, bend, lastt[threadIdx.x], bstart) : 3);
    const ART_LBOOL2 cert = ccode != 0;
    s_cert += cert ? 1u : 0u;
    // every lane parks (u, f, y, kk, h, τ) in its LDS slots (free after the error estimate):
    // the scan reads the interpolants from there, and the registers stay free until the
    // state is reloaded after the scan
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      L[(0 * 7 + i) * BLOCK] = u[i];
      L[(1 * 7 + i) * BLOCK] = f[i];
      L[(2 * 7 + i) * BLOCK] = y[i];
      L[(3 * 7 + i) * BLOCK] = kk[i];
    }
    L[(4 * 7 + 0) * BLOCK] = hs;
    L[(4 * 7 + 1) * BLOCK] = tau;
    const ART_LBOOL2 grid = scan && !cert;
    const unsigned long long smask = __ballot(grid);
    // lanes polishing a crossing need the condition at the end of their re-step (th = 1 of the
    // parked step): those items ride in the same pass, after the grid items
    const unsigned long long rmask = __ballot(mode == M_ROOT);
    const int ns_g = __popcll(smask), crank = __popcll(smask & ((1ull << lane) - 1ull));
    // N and D of the items this lane evaluates in the first two passes (see (c0) below)
    double gN0 = 0.0, gD0 = 1.0, gN1 = 0.0, gD1 = 1.0;
    ART_TMARK(2)  // error norm, controller, certificate and parking
    if ((smask | rmask) != 0ull) {
      const int ns = __popcll(smask), nr = __popcll(rmask);
      if (grid) {
        srcl[wbase + __popcll(smask & ((1ull << lane) - 1ull))] = lane;
#pragma unroll
        for (int w = 0; w < SCAN_WORDS; ++w) codes[w * BLOCK + threadIdx.x] = 0u;
      }
      if (mode == M_ROOT) srcl[wbase + ns + __popcll(rmask & ((1ull << lane) - 1ull))] = lane;
      wave_lds_sync();
      // grid item w = (j - 1) ns + c: point-major, advanced by 64 items per pass; then the
      // root items
      const int tg = ns * nper, total = tg + nr;
      const int dj = ns ? 64 / ns : 0, dc = ns ? 64 % ns : 0;
      int c = ns ? lane % ns : 0, j = ns ? lane / ns + 1 : 0;
#pragma unroll 1
      for (int w0 = 0; w0 < total; w0 += 64) {
        const int t = w0 + lane;
        if (t < total) {  // one evaluation site for both kinds of item (no divergent second copy)
          const bool gi = t < tg;
          const int src = srcl[wbase + (gi ? c : ns + (t - tg))];
          double N, D;
          scan_nd_lds(P, lds + wbase + src, BLOCK, gi ? thgrid[j] : 1.0, N, D);
          if (w0 == 0) {
            gN0 = N;
            gD0 = D;
          } else if (w0 == 64) {
            gN1 = N;
            gD1 = D;
          }
          if (!gi || j == nper) {  // a root item's value; the end value opens the next step's brackets
            const double cv = 0.5 * N / D;  // = scan_point_lds, bit for bit
            lastv[wbase + src] = cv;
          }
          if (gi) {
            const unsigned code = (j == nper) ? sign_code(lastv[wbase + src]) : sign_code_nd(N, D);
            atomicOr(&codes[((j - 1) >> 4) * BLOCK + wbase + src], code << (2 * ((j - 1) & 15)));
            s_scan += 1;
          }
        }
        c += dc;
        j += dj;
        if (c >= ns) {
          c -= ns;
          j += 1;
        }
      }
      wave_lds_sync();
    }

    ART_TMARK(3)  // grid pass
    // (b) Per lane: walk the sign codes exactly as the sequential scan would (NaN resets the
    //     sign memory; a sign change opens an Illinois search on the interpolant, ignored
    //     right after an event -- DiffEq repeat_nudge), plus the single evaluations of fresh
    //     lanes (initial sign) and of lanes polishing a crossing. Condition evaluations
    //     here only happen at brackets, Illinois points and root polish steps.
    //     ph: 0 done, 1 single point (INIT / ROOT), 2 walk codes, 3 Illinois, 5 value at the
    //     change point, 6 value at the bracket start, 7 value at the step's last nonzero point.
    int ph = scan ? 2 : 0;  // (polishing lanes: their value came with the grid pass, below)
    int ip = 1, last_j = 0;
    int last_s = sprev;
    double last_c = cprev;
    ART_LBOOL2 lc_ok = cprev_ok;  // last_c is the value at grid point last_j (0: the step start)
    unsigned cw[SCAN_WORDS] = {0u, 0u, 0u, 0u};
    if (ph == 2) {
#pragma unroll
      for (int w = 0; w < SCAN_WORDS; ++w)
        cw[w] = cert ? 0x55555555u * (unsigned)ccode : codes[w * BLOCK + threadIdx.x];
      // fast path: every grid point has the previous sign (or the previous sign is unknown
      // and every point has one common nonzero sign)
      const unsigned s0 = cw[0] & 3u;
      if (s0 == 1u || s0 == 2u) {
        bool same = (last_s == 0) || (last_s == (s0 == 1u ? 1 : -1));
#pragma unroll
        for (int w = 0; w < SCAN_WORDS; ++w) {
          const int nw = nper - 16 * w;
          if (nw <= 0) break;
          const unsigned m = nw >= 16 ? 0xffffffffu : ((1u << (2 * nw)) - 1u);
          same = same && ((cw[w] & m) == ((s0 * 0x55555555u) & m));
        }
        if (same) {
          last_s = (s0 == 1u) ? 1 : -1;
          last_j = nper;
          if (!cert) last_c = lastv[threadIdx.x];
          lc_ok = !cert;
          ph = 0;
        }
      } else if (s0 == 3u) {  // every point NaN: no resonance possible, the sign memory resets
        bool all = true;
#pragma unroll
        for (int w = 0; w < SCAN_WORDS; ++w) {
          const int nw = nper - 16 * w;
          if (nw <= 0) break;
          const unsigned m = nw >= 16 ? 0xffffffffu : ((1u << (2 * nw)) - 1u);
          all = all && ((cw[w] & m) == m);
        }
        if (all) {  // with no sign remembered, the bracket-start value is never read
          last_s = 0;
          lc_ok = false;
          ph = 0;
        }
      }
    }
    double i_tha = 0.0, i_ca = 0.0, i_thb = 0.0, i_cb = 0.0, i_tr = 0.0, i_cg = 0.0;
    int i_side = 0, i_it = 0;
    ART_LBOOL2 hit = false, root_done = false;
    // a crossing in (θ_last, θ_ip]: polish it on the true trajectory (mode ROOT), from t_int
    auto open_root = [&](double t_int) {
      const double thg = thgrid[ip];
      const double last_th = thgrid[last_j];
      hit = true;
      hroot = hs;
      r_tha = last_th; r_ca = last_c; r_thb = thg; r_cb = i_cg;
      r_slope = (i_cg - last_c) / (thg - last_th);
      r_t = (t_int > last_th && t_int < thg) ? t_int : 0.5 * (last_th + thg);
      r_side = 0;
      r_it = 0;
      post_c = i_cg;
      post_s = sgn(i_cg);
      dt = dtnext;
    };
    // the values at the change point (i_cg) and at the bracket start (last_c) are known
    auto open_bracket = [&]() {
      lc_ok = true;
      i_tha = thgrid[last_j];
      i_ca = last_c;
      i_thb = thgrid[ip];
      i_cb = i_cg;
      i_tr = i_tha - i_ca * (i_thb - i_tha) / (i_cb - i_ca);
      i_side = 0;
      i_it = 0;
      // The interpolant's root only seeds the polish on the true trajectory -- except right
      // after an event, where DiffEq's repeat_nudge asks whether it lies below θ = 0.01. Only
      // then is it refined by Illinois on the interpolant (ph 3); otherwise Vern6 starts the
      // polish from the secant point, which saves the ~6.6 lone-lane Illinois iterations a
      // bracket would cost the whole wave. (The fixed-step RK4 path keeps the Illinois seed:
      // with its tiny steps the oracle's own 1-ulp sensitivity is ~1e-12, and a different seed
      // moves grazing crossings by more.)
      if (RK4 || (just_evented && i_tha < 0.01)) {
        ph = 3;
      } else {
        open_root(i_tr);
        ph = 0;
      }
    };
    // walk the codes from grid point ip (no evaluations): ph 5 at a sign change, 7 when the
    // value at the last nonzero point is still needed, else 0
    auto walk = [&]() {
      WalkState ws{ip, last_s, last_j, lc_ok != 0};
      bool found = false;
      if (!walk_codes_bits(cw, nper, ws, found)) walk_codes_loop(cw, nper, ws, found);
      ip = ws.ip;
      last_s = ws.last_s;
      last_j = ws.last_j;
      lc_ok = ws.lc_ok;
      if (found) {
        ph = 5;
      } else if (!lc_ok && last_j == nper) {
        if (!cert) {  // a certified step leaves it to the next step's start (th = 0)
          last_c = lastv[threadIdx.x];
          lc_ok = true;
        }
        ph = 0;
      } else if (!lc_ok && last_s != 0) {
        ph = 7;
      } else {  // (with no sign remembered the bracket-start value is never read)
        ph = 0;
      }
    };
    // bracketed polish on the true trajectory (Newton with the interpolant slope, then Illinois)
    auto polish = [&](double ci) {
      ++r_it;
      bool done = !(fabs(ci) > 1e-12);
      if (!done) {
        if (sgn(ci) == sgn(r_ca)) { r_tha = r_t; r_ca = ci; if (r_side == -1) r_cb *= 0.5; r_side = -1; }
        else { r_thb = r_t; r_cb = ci; if (r_side == 1) r_ca *= 0.5; r_side = 1; }
        done = (r_thb - r_tha) * hroot < 1e-13 || r_it >= 9;
        if (!done) {
          double tn = (r_it == 1) ? r_t - ci / r_slope : r_tha - r_ca * (r_thb - r_tha) / (r_cb - r_ca);
          if (!(tn > r_tha && tn < r_thb)) tn = 0.5 * (r_tha + r_thb);
          r_t = tn;
        }
      }
      root_done = done;
      ph = 0;
    };
    if (mode == M_ROOT) {  // the re-stepped end's value, from the grid pass
      s_root += 1;
      polish(lastv[threadIdx.x]);
    }
    ART_TMARK(4)  // sign-code fast paths
    if (ph == 2) walk();
    ART_TMARK(5)  // code walk
    // (c0) The values a bracket (ph 5: at the change point and, when unknown, at the last
    //      nonzero point before it) or the next step's bracket start (ph 7) needs are grid
    //      points of this step: item (j - 1) ns + c of the grid pass (c: this lane's rank among
    //      the sources), evaluated by lane w & 63 in pass w >> 6, whose N and D from the first
    //      two passes are still in that lane's registers. ½ N / D there is scan_point_lds's
    //      value bit for bit, so no second evaluation is needed. (The step's start point,
    //      last_j = 0, and later passes go to the cooperative pass.)
    {
      const bool want = grid && (ph == 5 || ph == 7);
      const int ja = (ph == 5) ? ip : last_j;
      const int wa = (want && ja >= 1) ? (ja - 1) * ns_g + crank : (want ? 1 << 20 : 0);
      const bool needb = want && ph == 5 && !lc_ok;
      const int wb = needb ? (last_j >= 1 ? (last_j - 1) * ns_g + crank : 1 << 20) : 0;
      if (__ballot(want) != 0ull) {
        const int la = wa & 63, lb = wb & 63;
        const double nA0 = __shfl(gN0, la), dA0 = __shfl(gD0, la), nA1 = __shfl(gN1, la), dA1 = __shfl(gD1, la);
        const double nB0 = __shfl(gN0, lb), dB0 = __shfl(gD0, lb), nB1 = __shfl(gN1, lb), dB1 = __shfl(gD1, lb);
        if (want && wa < 128 && wb < 128) {
          const double va = 0.5 * ((wa >> 6) ? nA1 : nA0) / ((wa >> 6) ? dA1 : dA0);
          if (ph == 7) {
            last_c = va;
            lc_ok = true;
            ph = 0;
          } else {
            i_cg = va;
            if (needb) last_c = 0.5 * ((wb >> 6) ? nB1 : nB0) / ((wb >> 6) ? dB1 : dB0);
            open_bracket();
          }
        }
      }
    }
    // (c) One cooperative pass evaluates the pending condition values of the whole wave at
    //     once: the re-stepped end of polishing lanes (ph 1, th = 1 of their parked step), the
    //     change point of a bracket (ph 5) and its start when unknown, and the step's last
    //     nonzero grid point (ph 7). Requests (source lane, th) go to LDS and any lane
    //     evaluates any request, so a lane with two values needs one pass, not two.
    {
      const int nq = (ph == 1 || ph == 7) ? 1 : (ph == 5 ? (lc_ok ? 1 : 2) : 0);
      const unsigned long long lt = (1ull << lane) - 1ull;
      const unsigned long long b1 = __ballot(nq >= 1), b2 = __ballot(nq == 2);
      const int total = __popcll(b1) + __popcll(b2);
      if (total > 0 && total <= 64) {
        const int off = __popcll(b1 & lt) + __popcll(b2 & lt);
        wave_lds_sync();  // the walk's lastv reads are done
        if (nq >= 1) {
          srcl[wbase + off] = lane;
          lastv[wbase + off] = (ph == 1) ? 1.0 : (ph == 7 ? thgrid[last_j] : thgrid[ip]);
        }
        if (nq == 2) {
          srcl[wbase + off + 1] = lane;
          lastv[wbase + off + 1] = thgrid[last_j];
        }
        wave_lds_sync();
        if (lane < total) {
          const int src = srcl[wbase + lane];
          lastt[wbase + lane] = scan_point_lds(P, lds + wbase + src, BLOCK, lastv[wbase + lane]);
        }
        wave_lds_sync();
        if (nq >= 1) {
          const double r1 = lastt[wbase + off];
          if (ph == 1) {
            s_root += 1;
            polish(r1);
          } else if (ph == 7) {  // value at the step's last nonzero grid point (next step's bracket start)
            s_interp += 1;
            last_c = r1;
            lc_ok = true;
            ph = 0;
          } else {  // ph 5
            s_interp += (unsigned)nq;
            i_cg = r1;
            if (nq == 2) last_c = lastt[wbase + off + 1];
            open_bracket();
          }
        }
      }
    }
    ART_TMARK(6)  // cooperative pass
    // (d) Per lane, for the rare rest: more than 64 pending values, Illinois on the interpolant
    //     (repeat_nudge), and walking on after an ignored crossing.
    //     ph: 0 done, 1 re-stepped end (ROOT), 2 walk codes, 3 Illinois, 5 value at the change
    //     point, 6 value at the bracket start, 7 value at the step's last nonzero point.
#pragma unroll 1
    while (ph != 0) {
      if (ph == 2) {
        walk();
        if (ph == 0) break;
      }
      double th = 1.0;  // ph 1: the re-stepped end y at τ + h is the parked step's th = 1
      if (ph == 3) th = i_tr;
      else if (ph == 5) th = thgrid[ip];
      else if (ph == 6 || ph == 7) th = thgrid[last_j];
      const double ci = scan_point_lds(P, L, BLOCK, th);
      if (ph == 1) {
        s_root += 1;
        polish(ci);
        continue;
      }
      s_interp += 1;
      if (ph == 7) {
        last_c = ci;
        lc_ok = true;
        ph = 0;
      } else if (ph == 5 || ph == 6) {
        if (ph == 5) i_cg = ci;
        else last_c = ci;
        if (ph == 5 && !lc_ok) ph = 6;
        else open_bracket();
      } else {  // ph == 3: Illinois on the interpolant inside (i_tha, i_thb]
        bool stop = ci == 0.0 || isnan(ci) || (i_thb - i_tha) < 1e-12;
        bool below = false;
        if (!stop) {
          if (sgn(ci) == sgn(i_ca)) { i_tha = i_tr; i_ca = ci; if (i_side == -1) i_cb *= 0.5; i_side = -1; }
          else { i_thb = i_tr; i_cb = ci; if (i_side == 1) i_ca *= 0.5; i_side = 1; }
          // Every later iterate stays in [i_tha, i_thb]: once that lies below θ = 0.01 right
          // after an event, the root is ignored (repeat_nudge) wherever Illinois would end,
          // so the search stops here with the same outcome
          below = just_evented && i_thb < 0.01;
          if (below) {
            stop = true;
          } else {
            const double tn = i_tha - i_ca * (i_thb - i_tha) / (i_cb - i_ca);
            if (tn == i_tr) stop = true;
            else i_tr = tn;
            if (++i_it >= 40) stop = true;
          }
        }
        if (stop) {
          const double t_int = i_tr;
          if (!below && !(just_evented && t_int < 0.01)) {  // DiffEq repeat_nudge after an event
            open_root(t_int);
            ph = 0;
          } else {  // ignored: continue the walk after the change point
            last_s = sgn(i_cg);
            last_c = i_cg;
            last_j = ip;
            lc_ok = true;
            ++ip;
            ph = 2;
          }
        }
      }
    }
    ART_TMARK(7)  // per-lane fallback loop
    if constexpr (SAVE) {
      // saveat (RayTracer.jl:176, 383): the interior save times ln t0 + kΔ that this completed
      // step passed -- an accepted step without a crossing, or the polish step that ends at a
      // root -- from the step's parked interpolant. finalize_kernel adds the start and the end.
      if (((scan && !hit) || root_done) && save_k < out.ntimes - 1) {
        const double t0 = in.lnt0[ray];
        const double D = (tend - t0) / double(out.ntimes - 1);
        const double tb = (last && !root_done) ? tend : tau + hs;
        while (save_k < out.ntimes - 1) {
          const double ts = t0 + double(save_k) * D;
          if (!(ts <= tb)) break;
          const double th = (ts - tau) / hs;
#pragma unroll
          for (int c = 0; c < 3; ++c)
            out.traj[(int64_t(c) * out.ntimes + save_k) * n + ray] =
                hermite1(L[(0 * 7 + c) * BLOCK], L[(1 * 7 + c) * BLOCK], L[(2 * 7 + c) * BLOCK],
                         L[(3 * 7 + c) * BLOCK], hs, th);
          out.traj_t[int64_t(save_k) * n + ray] = ts;
          ++save_k;
        }
      }
    }
    // reload the state each lane continues from: the step's end (y, kk: slots 2-3) after an
    // accepted step or a finished polish, else its start (u, f: slots 0-1)
    {
      const double* Ls = L + ((root_done || (scan && !hit)) ? 2 * 7 * BLOCK : 0);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        u[i] = Ls[i * BLOCK];
        f[i] = Ls[(7 + i) * BLOCK];
      }
    }
    if (hit) mode = M_ROOT;
    if (root_done || (scan && !hit)) bstart = bend;
    if (root_done) {
      const double tau_r = tau + hs;
      const int a = affect(P, in, out, n, ray, u, tau_r, erg, ncross, max_crossings);
      tau = tau_r;
      cprev = post_c;  // the post-event side (DiffEq repeat_nudge): the root is not re-found
      cprev_ok = true;
      sprev = post_s;
      just_evented = true;
      mode = M_STEP;
      if (a == 2) finish = ART_STATUS_CROSSING;
      else if (photon && u[0] < P.rNS101) finish = ART_STATUS_HIT_NS;  // cb_r after the event
      else if (iter >= P.maxiters) finish = ART_STATUS_MAXITERS;
    }
    if (scan && !hit) {
      tau = last ? tend : tau + hs;
      cprev = last_c;
      cprev_ok = lc_ok;
      sprev = last_s;
      just_evented = false;
      dt = dtnext;
      if (cbs && photon && u[0] < P.rNS101) finish = ART_STATUS_HIT_NS;  // cb_r (:352-368)
      else if (last) finish = ART_STATUS_SUCCESS;
      else if (iter >= P.maxiters) finish = ART_STATUS_MAXITERS;
    }

    int fin_piece = -1;  // (DON = 3) the piece of a ray finishing now
    if (finish >= 0) {  // the raw end record; finalize_kernel back-transforms it (RayTracer.jl:393-416)
      if constexpr (DON == 3) fin_piece = ray >> out.piece_shift;
      double2* rq = reinterpret_cast<double2*>(out.rec + (int64_t)ray * END_REC);
      rq[0] = make_double2(u[0], u[1]);
      rq[1] = make_double2(u[2], u[3]);
      rq[2] = make_double2(u[4], u[5]);
      rq[3] = make_double2(u[6], tau);
      int4* ri = reinterpret_cast<int4*>(rq + 4);
      ri[0] = make_int4(finish, n_acc, n_rej, ncross);
      if constexpr (SAVE) ri[1] = make_int4(save_k + 1, 0, 0, 0);  // start + interior + end
      ray = -1;
      mode = M_IDLE;
    }
    if constexpr (DON == 3) {
      // the streamed host pipelines: each finishing lane counts its ray into its wave's LDS
      // histogram over the pieces; every ART_STREAM_FLUSH + 1 iterations (and once the queue is
      // drained) the wave releases its stores and adds the histogram to the pieces' global
      // counts, one lane per piece (stream_flush). Kept out of registers: a per-wave pending
      // count held across the loop cost the integrator 7.5% in spills
      // (profiles/r04s2_streamed_kernel_ab.jsonl)
      if (fin_piece >= 0) atomicAdd(&pend_lds[threadIdx.x >> 6][fin_piece], 1u);
#ifndef ART_DRAIN_FLUSH_MASK
#define ART_DRAIN_FLUSH_MASK 7  // (once the queue is drained: every 8th iteration, so the drain pays few write-backs)
#endif
      ++tick;
      if ((tick & ART_STREAM_FLUSH) == 0 || (exhausted && (tick & ART_DRAIN_FLUSH_MASK) == 0))
        stream_flush(out, pend_lds[threadIdx.x >> 6], lane);
    }
    ART_TMARK(0)  // saveat, reload, events, finish and the output stores (+ refill)
    // graduation (SegOut::graduate): a ray past `graduate` attempts, at a step boundary, leaves
    // for the tail kernel now instead of running on as one lane of this wave until the wave
    // drains; its lane takes the next ray. The record is the donation record, so the ray's
    // arithmetic does not change.
    // early graduation (SegOut::hot): a ray whose progress in ln t lags the hot rule at a
    // power-of-two attempt count, or when its drained wave donates it, leaves for the hot
    // records, which a tail_kernel launch beside this one resumes at once (one wave per ray)
    auto to_hot = [&](bool h) {
      const unsigned long long hm = __ballot(h);
      if (hm == 0ull) return;
      const int leader = __ffsll((long long)hm) - 1;
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(out.hot_count, (unsigned long long)__popcll(hm));
      base = __shfl(base, leader);
      const int64_t slot = (int64_t)base + __popcll(hm & ((1ull << lane) - 1ull));
      if (h && slot < (int64_t)out.hot_cap) {  // (no slot left: the ray stays)
        write_cont_rec(out.hot + slot * CONT_REC, u, f, tau, dt, qpow, cprev, bstart, erg, ray, n_acc, n_rej, ncross,
                       iter, sprev, photon, cprev_ok, just_evented, save_k);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(out.hot_ready + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ray = -1;
        mode = M_IDLE;
      }
    };
    if (DON == 1 && out.hot_at > 0) {
      bool h = mode == M_STEP && iter >= out.hot_at && (iter & (iter - 1)) == 0;
      if (__ballot(h) != 0ull) {
        if (h) h = hot_lags(out, tau - in.lnt0[ray], (double)(__builtin_ctz((unsigned)iter) - 8));
        to_hot(h);
      }
    }
    // graduation (SegOut::graduate): a ray past `graduate` attempts, at a step boundary, leaves
    // for the tail kernel now instead of running on as one lane of this wave until the wave
    // drains; its lane takes the next ray. The record is the donation record, so the ray's
    // arithmetic does not change.
    if (DON == 1 && out.graduate > 0) {
      const bool g = mode == M_STEP && iter >= out.graduate;
      const unsigned long long gm = __ballot(g);
      if (gm != 0ull) {
        const int leader = __ffsll((long long)gm) - 1;
        unsigned long long base = 0;
        if (lane == leader) base = atomicAdd(out.grad_count, (unsigned long long)__popcll(gm));
        base = __shfl(base, leader);
        const int64_t slot = (int64_t)base + __popcll(gm & ((1ull << lane) - 1ull));
        if (g && slot < (int64_t)out.grad_cap) {  // (no slot left: the ray stays)
          write_cont_rec(out.grad + slot * CONT_REC, u, f, tau, dt, qpow, cprev, bstart, erg, ray, n_acc, n_rej,
                         ncross, iter, sprev, photon, cprev_ok, just_evented, save_k);
          ray = -1;
          mode = M_IDLE;
        }
      }
    }
    // tail donation (SegOut::donate): the drained wave's last few rays, all at a step
    // boundary, leave for the continuation launch and the wave retires
    if (DON == 1 && exhausted && out.donate > 0) {
      unsigned long long live = __ballot(mode != M_IDLE);
      if (live != 0ull && __popcll(live) <= out.donate && __ballot(mode == M_ROOT) == 0ull) {
        if (out.hot_at > 0) {  // (the lagging ones to the hot records instead)
          bool h = mode == M_STEP && iter >= out.hot_at;
          if (__ballot(h) != 0ull) {
            if (h) h = hot_lags(out, tau - in.lnt0[ray], log2((double)iter) - 8.0);
            to_hot(h);
            live = __ballot(mode != M_IDLE);
          }
        }
        if (live != 0ull) {
          const int leader = __ffsll((long long)live) - 1;
          unsigned long long base = 0;
          if (lane == leader) base = atomicAdd(out.cont_count, (unsigned long long)__popcll(live));
          base = __shfl(base, leader);
          if (mode != M_IDLE) {
            const int64_t slot = (int64_t)base + __popcll(live & ((1ull << lane) - 1ull));
            write_cont_rec(out.cont + slot * CONT_REC, u, f, tau, dt, qpow, cprev, bstart, erg, ray, n_acc, n_rej,
                           ncross, iter, sprev, photon, cprev_ok, just_evented, save_k);
            ray = -1;
            mode = M_IDLE;
          }
        }
      }
    }
  }

  // wave-reduce the statistics and add them once per wave (DON = 3: before the wave counts itself
  // done and flushes its last piece counts, so the helper that ends the call finds them complete)
#if defined(ART_SECTION_TIMING)
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(&stats[k], t_sec[k]);
  }
#else
  const unsigned v[7] = {s_att, s_acc, s_root, s_scan, s_interp, s_rays, s_cert};
  const int slot[7] = {ST_ATTEMPTS, ST_ACCEPTED, ST_ROOT_STEPS, ST_SCAN_EVALS, ST_INTERP_EVALS, ST_RAYS, ST_CERT};
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    unsigned long long x = v[k];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if (lane == 0 && x) atomicAdd(&stats[slot[k]], x);
  }
#endif
  span_stamp(stats, true);
  if constexpr (DON == 3) {
    if (out.waves_done) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (lane == 0) __hip_atomic_fetch_add(out.waves_done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stream_flush(out, pend_lds[threadIdx.x >> 6], lane);
  }
}

// ---------------------------------------------------------------------------
// tail_kernel: the long rays that set a launch's drain time, ONE WAVE PER RAY.
//
// A persistent pass ends with a drain: once its queue is empty, its last long rays run alone
// in their waves, and a lone lane issues every instruction of its wave (configs[3]'s ray
// 717277 alone takes ~0.3 s of the 1e6-ray GR batch). With tail donation (SegOut::donate) such
// rays leave the bulk kernel with their complete state; when few remain, this kernel resumes
// each of them on a wave of its own and spreads the attempt's independent work across lanes:
//   * the e^τ of all eight stages of an attempt in one pass on lanes 0..7 (stage times are
//     known at the attempt's start), instead of one exp per stage on the critical path;
//   * sin/cos of θ and of ψ = φ - ωt in ONE sincos on lanes 0 and 1 (same code, two arguments);
//   * the 49 grid points of an uncertified step's resonance scan on lanes 0..48 at once, their
//     sign codes gathered with two ballots;
//   * all the stage vectors in registers (one wave per SIMD: 512 VGPRs), the Vern6 stages fully
//     unrolled with compile-time coefficients, the ray's control state wave-uniform.
// Everything else is the bulk kernel's arithmetic on the same operands in the same order, so a
// donated ray's result is bit-identical to its never-donated one (tests/test_gpu_tail_donation.py).
// Vern6 without saveat only (the other launches keep the packed continuation).
static __constant__ double c_tail_ct[8] = {Vern6::c2, Vern6::c3, Vern6::c4, Vern6::c5, Vern6::c6, Vern6::c7, 1.0, 1.0};

// a wave-uniform double from lane l (two v_readlane_b32)
__device__ inline double rdlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// the 16 bits b[15:0] spread to the even bit positions of 32
__device__ inline unsigned spread16(unsigned x) {
  x &= 0xffffu;
  x = (x | (x << 8)) & 0x00ff00ffu;
  x = (x | (x << 4)) & 0x0f0f0f0fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

// scan_nd_lds on register arrays (the same arithmetic)
__device__ inline void scan_nd_regs(const KParams& P, const double* u0, const double* f0, const double* u1,
                                    const double* f1, double h, double tau, double th, double& N, double& D) {
  double ui[7];
  hermite7(u0, f0, u1, f1, h, th, ui);
#pragma unroll
  for (int i = 0; i < 7; ++i) ui[i] = (th == 1.0) ? u1[i] : ui[i];
  condition_nd(P, ui, fexp(tau + th * h), N, D);
}

__device__ inline double scan_point_regs(const KParams& P, const double* u0, const double* f0, const double* u1,
                                         const double* f1, double h, double tau, double th) {
  double N, D;
  scan_nd_regs(P, u0, f0, u1, f1, h, tau, th, N, D);
  return 0.5 * N / D;
}

// The photon RHS at stage point y, t = e^(τ_s) given: θ's and ψ's sincos on lanes 0 and 1.
template <int GEOM>
__device__ inline void tail_rhs(const KParams& P, int lane, const double* y, double ty, double t, double erg,
                                double* kk, double* aux) {
  if constexpr (GEOM != GEOM_ANY) {
    const double arg = (lane == 1) ? psi_of(P, y[2], t) : y[1];
    double sn, cs;
    msincos(arg, sn, cs);
    const double st = rdlane(sn, 0), ct = rdlane(cs, 0), sp = rdlane(sn, 1), cp = rdlane(cs, 1);
    rhs_photon_gj_tr(P, y, t, st, ct, sp, cp, erg, kk, aux);
  } else {
    rhs_photon(P, y, ty, erg, kk, aux);
  }
}

// The next hot record (SegOut::hot) for this wave, -1 once none is left: claimed as the records
// arrive until *hot_done is raised (then the count is final) or the wait passes HOT_WAIT_TICKS,
// and read only once its hot_ready word is up.
__device__ inline int64_t claim_hot(const SegOut& out, int lane) {
  long long rec = -1;
  if (lane == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long cap = (unsigned long long)out.hot_cap;
    while (true) {
      const bool done = __hip_atomic_load(out.hot_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      unsigned long long q = __hip_atomic_load(out.hot_queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned long long c = __hip_atomic_load(out.hot_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      c = c < cap ? c : cap;
      if (q < c) {
        if (__hip_atomic_compare_exchange_strong(out.hot_queue, &q, q + 1ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          rec = (long long)q;
          break;
        }
        continue;
      }
      if (done || __builtin_amdgcn_s_memrealtime() - t0 > HOT_WAIT_TICKS) break;
      __builtin_amdgcn_s_sleep(64);
    }
    if (rec >= 0) {  // (its producer raises it right after the record; bounded all the same)
      while (__hip_atomic_load(out.hot_ready + rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2ull * HOT_WAIT_TICKS) {
          rec = -1;
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
  }
  rec = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)rec, 0)) |
                    ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)((unsigned long long)rec >> 32), 0) << 32));
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return (int64_t)rec;
}

// (blocks of up to 4 waves, each wave a ray of its own: the hot rays' launch packs its waves
// into few CUs, the others launch one wave a block)
template <int GEOM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void tail_kernel(
    const KParams P_in, const int64_t n, const SegIn in, const SegOut out, const int32_t max_crossings,
    const int32_t max_rays, unsigned long long* __restrict__ stats) {
  const KParams P = specialize<GEOM>(P_in);
  using V = Vern6;
  const int lane = threadIdx.x & 63;
  // Every lane holds the ray's state alike, so its control decisions are wave-uniform: U() makes
  // that visible to the compiler (a scalar branch on lane 0's value instead of an exec-mask
  // branch with its saved masks -- SGPRs the kernel otherwise spills to VGPR lanes); the values
  // and the arithmetic do not change
  auto U = [](bool c) { return __builtin_amdgcn_readfirstlane((int)c) != 0; };
  const int64_t nq = (int64_t)*out.cont_count;
  (void)max_rays;
  __builtin_amdgcn_s_setprio(3);  // the rays that set the launch's end
  const bool cbs = max_crossings != ART_NO_CALLBACKS;
  const double tend = P.ln_t_end;
  const int npts = P.interp_points;
  const int nper = npts - 1;
  const double my_ct = c_tail_ct[lane & 7];
  const double my_th = double(lane + 1) / double(npts - 1);  // grid point lane + 1 (Julia's range(0, 1, length = npts))
  unsigned s_att = 0, s_acc = 0, s_root = 0, s_scan = 0, s_interp = 0, s_cert = 0;
  // the graduated rays (SegOut::grad, the pass's outliers) first, then the drained waves' records
  const int64_t ng = out.grad ? ((int64_t)*out.grad_count < (int64_t)out.grad_cap ? (int64_t)*out.grad_count
                                                                                   : (int64_t)out.grad_cap)
                              : 0;
  bool grads = ng > 0;
  bool hots = out.hot != nullptr;
  span_stamp(stats, false);
  while (true) {
    const double* src = nullptr;
    if (hots) {  // the hot rays first (a launch beside the bulk pass waits for them)
      const int64_t rec = claim_hot(out, lane);
      if (rec >= 0) src = out.hot + rec * CONT_REC;
      else hots = false;
    }
    while (src == nullptr) {
      unsigned long long* q = grads ? out.grad_queue : out.cont_queue;
      unsigned long long ix = 0;
      if (lane == 0) ix = atomicAdd(q, 1ull);
      const int64_t rec = (int64_t)__builtin_amdgcn_readfirstlane((unsigned)ix) |
                          ((int64_t)__builtin_amdgcn_readfirstlane((unsigned)(ix >> 32)) << 32);
      if (grads) {
        if (rec < ng) src = out.grad + rec * CONT_REC;
        else grads = false;
      } else {
        if (rec >= nq) break;
        src = out.cont + rec * CONT_REC;
      }
    }
    if (src == nullptr) break;
    // ---- the donated ray's complete state (the bulk kernel's CONT_REC) ----
    double u[7], f[7];
    double tau, dt, qpow, cprev, bstart, erg;
    int ray, n_acc, n_rej, ncross, iter, sprev;
    bool photon, cprev_ok, just_evented;
    {
      const double2* rq = reinterpret_cast<const double2*>(src);
      double v[20];
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const double2 q = rq[i];
        v[2 * i] = q.x;
        v[2 * i + 1] = q.y;
      }
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        u[i] = v[i];
        f[i] = v[7 + i];
      }
      tau = v[14]; dt = v[15]; qpow = v[16]; cprev = v[17]; bstart = v[18]; erg = v[19];
      const int4 i0 = reinterpret_cast<const int4*>(rq + 10)[0], i1 = reinterpret_cast<const int4*>(rq + 10)[1];
      ray = i0.x; n_acc = i0.y; n_rej = i0.z; ncross = i0.w;
      iter = i1.x; sprev = i1.y;
      photon = i1.z & 1; cprev_ok = (i1.z >> 1) & 1; just_evented = (i1.z >> 2) & 1;
    }
    int mode = M_STEP;
    double hroot = 0.0, r_tha = 0.0, r_ca = 0.0, r_thb = 0.0, r_cb = 0.0, r_t = 0.0, r_slope = 1.0, post_c = 0.0;
    int post_s = 0, r_side = 0, r_it = 0;
    int finish = -1;
    while (U(finish < 0)) {
      // ---- this attempt's step size (the bulk kernel's rules) ----
      bool last = false, forced = false;
      double hs;
      if (U(mode == M_ROOT)) {
        hs = r_t * hroot;
      } else {
        hs = dt;
        if (U(tau + hs >= tend)) { hs = tend - tau; last = true; }
        else if (U(hs < P.dtmin)) { hs = P.dtmin; forced = true; }
      }
      // ---- e^τ of the eight stages at once (lane s: stage s) ----
      const double tl = fexp(tau + my_ct * hs);
      // ---- the Vern6 stages, unrolled (c_vern6's rows with their coefficients folded) ----
      // The bulk kernel forms each stage point in the order acc = cf f (rounded), then
      // acc = fma(c_q, L_q, acc) per parked stage, y = fma(h, acc, u): its product cf f and the
      // stage loop's additions sit in different basic blocks, so they are never contracted into
      // one FMA. Written straight-line, `cf * f + c * L` would be (fma(cf, f, c L)); the explicit
      // fma calls below keep the bulk kernel's roundings, bit for bit.
      double kA[7], L0[7], L1[7], L2[7], L3[7], L4[7], y[7], kk[7], aux[2] = {0.0, 0.0};
      auto stage = [&](int s, double ct) {
        const double ty = tau + ct * hs;
        const double t = rdlane(tl, s);
        tail_rhs<GEOM>(P, lane, y, ty, t, erg, kk, aux);
        if (U(!photon)) {
          double ka[7];
          rhs_axion(P, y, ty, erg, ka);
#pragma unroll
          for (int i = 0; i < 7; ++i) kk[i] = ka[i];
        }
      };
#pragma unroll
      for (int i = 0; i < 7; ++i) y[i] = u[i] + hs * (V::a21 * f[i]);
      stage(0, V::c2);
#pragma unroll
      for (int i = 0; i < 7; ++i) kA[i] = kk[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) y[i] = u[i] + hs * fma(V::a31, f[i], V::a32 * kA[i]);
      stage(1, V::c3);
#pragma unroll
      for (int i = 0; i < 7; ++i) L0[i] = kk[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        double acc = V::a41 * f[i];
        acc = fma(V::a43, L0[i], acc);
        y[i] = u[i] + hs * acc;
      }
      stage(2, V::c4);
#pragma unroll
      for (int i = 0; i < 7; ++i) L1[i] = kk[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        double acc = V::a51 * f[i];
        acc = fma(V::a53, L0[i], acc);
        acc = fma(V::a54, L1[i], acc);
        y[i] = u[i] + hs * acc;
      }
      stage(3, V::c5);
#pragma unroll
      for (int i = 0; i < 7; ++i) L2[i] = kk[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        double acc = V::a61 * f[i];
        acc = fma(V::a63, L0[i], acc);
        acc = fma(V::a64, L1[i], acc);
        acc = fma(V::a65, L2[i], acc);
        y[i] = u[i] + hs * acc;
      }
      stage(4, V::c6);
#pragma unroll
      for (int i = 0; i < 7; ++i) L3[i] = kk[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        double acc = V::a71 * f[i];
        acc = fma(V::a73, L0[i], acc);
        acc = fma(V::a74, L1[i], acc);
        acc = fma(V::a75, L2[i], acc);
        acc = fma(V::a76, L3[i], acc);
        y[i] = u[i] + hs * acc;
      }
      stage(5, V::c7);
#pragma unroll
      for (int i = 0; i < 7; ++i) L4[i] = kk[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        double acc = V::a81 * f[i];
        acc = fma(V::a83, L0[i], acc);
        acc = fma(V::a84, L1[i], acc);
        acc = fma(V::a85, L2[i], acc);
        acc = fma(V::a86, L3[i], acc);
        acc = fma(V::a87, L4[i], acc);
        y[i] = u[i] + hs * acc;
      }
      stage(6, 1.0);
#pragma unroll
      for (int i = 0; i < 7; ++i) kA[i] = kk[i];  // k8
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        double acc = fma(V::a91, f[i], V::a98 * kA[i]);
        acc = fma(V::a94, L1[i], acc);
        acc = fma(V::a95, L2[i], acc);
        acc = fma(V::a96, L3[i], acc);
        acc = fma(V::a97, L4[i], acc);
        y[i] = u[i] + hs * acc;
      }
      stage(7, 1.0);
      const double bend = aux[0], tlast = aux[1];
      // ---- error estimate (y = u_{n+1}, kk = f(u_{n+1})) ----
      if (photon && y[0] < P.rNS) y[0] = P.rNS;  // clamp on the FSAL stage (:531)
      double EEst2;
      {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 7; ++i) {
          double e = fma(V::e9, kk[i], fma(V::e8, kA[i], V::e1 * f[i]));  // as the bulk kernel
          e = fma(V::e4, L1[i], e);
          e = fma(V::e5, L2[i], e);
          e = fma(V::e6, L3[i], e);
          e = fma(V::e7, L4[i], e);
          e *= hs;
          const double q = e * frcp(P.abstol + fmax_abs(u[i], y[i]) * P.reltol);
          acc += q * q;
        }
        EEst2 = acc * (1.0 / 7.0);
      }
      // ---- controller (STEP) ----
      bool scan = false;
      double dtnext = dt;
      if (U(mode == M_STEP)) {
        s_att += 1;
        ++iter;
        bool finite = !isnan(EEst2) && !isinf(EEst2);
#pragma unroll
        for (int i = 0; i < 7; ++i) finite = finite && !isnan(y[i]) && !isinf(y[i]);
        if (U(!finite)) {
          finish = ART_STATUS_NONFINITE;
        } else {
          double q = 1.0, q11 = 1.0, y60 = 0.0;
          if (U(EEst2 == 0.0)) {
            q = 0.1;
          } else {
            y60 = fexp(flog(EEst2) * (1.0 / 120.0));
            const double y2 = y60 * y60;
            q11 = (y2 * y2) * (y2 * y60);
            q = q11 * frcp(qpow);
            q = fmax(0.1, fmin(5.0, q * (1.0 / 0.9)));
          }
          const bool accept = U((EEst2 <= 1.0) || forced);
          if (!accept) {
            dt = hs * frcp(fmin(5.0, q11 * (1.0 / 0.9)));
            ++n_rej;
            if (iter >= P.maxiters) finish = ART_STATUS_MAXITERS;
          } else {
            ++n_acc;
            s_acc += 1;
            const double ym = fmax(y60, 0.8576958985908941);  // (1e-4)^(1/60)
            qpow = (ym * ym) * (ym * ym);
            dtnext = hs * frcp(q);
            scan = true;
          }
        }
      }
      if (U(finish >= 0)) break;
      // ---- resonance scan of an accepted step: certificate, else the 49 grid points at once ----
      const int ccode = !scan ? 0 : (cbs ? scan_certified_code(P, u, f, y, kk, hs, bend, tlast, bstart) : 3);
      const bool cert = U(ccode != 0);
      s_cert += cert ? 1u : 0u;
      const bool grid = U(scan && !cert);
      double gN = 0.0, gD = 1.0;  // lane l: N, D at grid point l + 1
      unsigned cw[SCAN_WORDS] = {0u, 0u, 0u, 0u};
      double lastv = 0.0;  // value at the last grid point
      if (grid) {
        if (lane < nper) scan_nd_regs(P, u, f, y, kk, hs, tau, my_th, gN, gD);
        const double cv = 0.5 * gN / gD;
        const unsigned code = (lane == nper - 1) ? sign_code(cv) : sign_code_nd(gN, gD);
        const unsigned long long b0 = __ballot(lane < nper && (code & 1u)), b1 = __ballot(lane < nper && (code & 2u));
#pragma unroll
        for (int w = 0; w < SCAN_WORDS; ++w)
          cw[w] = spread16((unsigned)(b0 >> (16 * w))) | (spread16((unsigned)(b1 >> (16 * w))) << 1);
        lastv = rdlane(cv, nper - 1);
        s_scan += (unsigned)nper;
      } else if (ccode != 0) {
#pragma unroll
        for (int w = 0; w < SCAN_WORDS; ++w) cw[w] = 0x55555555u * (unsigned)ccode;
      }
      auto gval = [&](int j) {  // the condition at grid point j of this step (from the grid pass when it ran)
        if (U(grid && j >= 1)) return 0.5 * rdlane(gN, j - 1) / rdlane(gD, j - 1);
        s_interp += 1;
        return scan_point_regs(P, u, f, y, kk, hs, tau, double(j) / double(npts - 1));
      };
      // ---- the sign walk, brackets and root polish: the bulk kernel's per-lane logic ----
      int ph = scan ? 2 : 0;
      int ip = 1, last_j = 0;
      int last_s = sprev;
      double last_c = cprev;
      bool lc_ok = cprev_ok;
      if (U(ph == 2)) {
        const unsigned s0 = cw[0] & 3u;
        if (U(s0 == 1u || s0 == 2u)) {
          bool same = (last_s == 0) || (last_s == (s0 == 1u ? 1 : -1));
#pragma unroll
          for (int w = 0; w < SCAN_WORDS; ++w) {
            const int nw = nper - 16 * w;
            if (nw <= 0) break;
            const unsigned m = nw >= 16 ? 0xffffffffu : ((1u << (2 * nw)) - 1u);
            same = same && ((cw[w] & m) == ((s0 * 0x55555555u) & m));
          }
          if (U(same)) {
            last_s = (s0 == 1u) ? 1 : -1;
            last_j = nper;
            if (!cert) last_c = lastv;
            lc_ok = !cert;
            ph = 0;
          }
        } else if (U(s0 == 3u)) {
          bool all = true;
#pragma unroll
          for (int w = 0; w < SCAN_WORDS; ++w) {
            const int nw = nper - 16 * w;
            if (nw <= 0) break;
            const unsigned m = nw >= 16 ? 0xffffffffu : ((1u << (2 * nw)) - 1u);
            all = all && ((cw[w] & m) == m);
          }
          if (U(all)) {
            last_s = 0;
            lc_ok = false;
            ph = 0;
          }
        }
      }
      double i_tha = 0.0, i_ca = 0.0, i_thb = 0.0, i_cb = 0.0, i_tr = 0.0, i_cg = 0.0;
      int i_side = 0, i_it = 0;
      bool hit = false, root_done = false;
      auto thg = [&](int j) { return double(j) / double(npts - 1); };
      auto open_root = [&](double t_int) {
        const double tg = thg(ip), lth = thg(last_j);
        hit = true;
        hroot = hs;
        r_tha = lth; r_ca = last_c; r_thb = tg; r_cb = i_cg;
        r_slope = (i_cg - last_c) / (tg - lth);
        r_t = (t_int > lth && t_int < tg) ? t_int : 0.5 * (lth + tg);
        r_side = 0;
        r_it = 0;
        post_c = i_cg;
        post_s = sgn(i_cg);
        dt = dtnext;
      };
      auto open_bracket = [&]() {
        lc_ok = true;
        i_tha = thg(last_j);
        i_ca = last_c;
        i_thb = thg(ip);
        i_cb = i_cg;
        i_tr = i_tha - i_ca * (i_thb - i_tha) / (i_cb - i_ca);
        i_side = 0;
        i_it = 0;
        if (U(just_evented && i_tha < 0.01)) {
          ph = 3;
        } else {
          open_root(i_tr);
          ph = 0;
        }
      };
      auto walk = [&]() {
        WalkState ws{ip, last_s, last_j, lc_ok};
        bool found = false;
        if (!walk_codes_bits(cw, nper, ws, found)) walk_codes_loop(cw, nper, ws, found);
        ip = ws.ip;
        last_s = ws.last_s;
        last_j = ws.last_j;
        lc_ok = ws.lc_ok;
        if (U(found)) {
          ph = 5;
        } else if (U(!lc_ok && last_j == nper)) {
          if (!cert) {
            last_c = lastv;
            lc_ok = true;
          }
          ph = 0;
        } else if (!lc_ok && last_s != 0) {
          ph = 7;
        } else {
          ph = 0;
        }
      };
      auto polish = [&](double ci) {
        ++r_it;
        bool done = !(fabs(ci) > 1e-12);
        if (!done) {
          if (sgn(ci) == sgn(r_ca)) { r_tha = r_t; r_ca = ci; if (r_side == -1) r_cb *= 0.5; r_side = -1; }
          else { r_thb = r_t; r_cb = ci; if (r_side == 1) r_ca *= 0.5; r_side = 1; }
          done = (r_thb - r_tha) * hroot < 1e-13 || r_it >= 9;
          if (!done) {
            double tn = (r_it == 1) ? r_t - ci / r_slope : r_tha - r_ca * (r_thb - r_tha) / (r_cb - r_ca);
            if (!(tn > r_tha && tn < r_thb)) tn = 0.5 * (r_tha + r_thb);
            r_t = tn;
          }
        }
        root_done = done;
        ph = 0;
      };
      if (U(mode == M_ROOT)) {  // the re-stepped end's value (th = 1 of this step)
        s_root += 1;
        polish(scan_point_regs(P, u, f, y, kk, hs, tau, 1.0));
      }
      if (U(ph == 2)) walk();
#pragma unroll 1
      while (U(ph != 0)) {
        if (U(ph == 2)) {
          walk();
          if (U(ph == 0)) break;
        }
        if (U(ph == 5)) {  // the values at the change point and, when unknown, at the bracket start
          i_cg = gval(ip);
          if (U(!lc_ok)) last_c = gval(last_j);
          open_bracket();
        } else if (U(ph == 7)) {
          last_c = gval(last_j);
          lc_ok = true;
          ph = 0;
        } else {  // ph 3: Illinois on the interpolant inside (i_tha, i_thb] (repeat_nudge)
          s_interp += 1;
          const double ci = scan_point_regs(P, u, f, y, kk, hs, tau, i_tr);
          bool stop = ci == 0.0 || isnan(ci) || (i_thb - i_tha) < 1e-12;
          bool below = false;
          if (!stop) {
            if (sgn(ci) == sgn(i_ca)) { i_tha = i_tr; i_ca = ci; if (i_side == -1) i_cb *= 0.5; i_side = -1; }
            else { i_thb = i_tr; i_cb = ci; if (i_side == 1) i_ca *= 0.5; i_side = 1; }
            below = just_evented && i_thb < 0.01;
            if (below) {
              stop = true;
            } else {
              const double tn = i_tha - i_ca * (i_thb - i_tha) / (i_cb - i_ca);
              if (tn == i_tr) stop = true;
              else i_tr = tn;
              if (++i_it >= 40) stop = true;
            }
          }
          if (U(stop)) {
            const double t_int = i_tr;
            if (U(!below && !(just_evented && t_int < 0.01))) {
              open_root(t_int);
              ph = 0;
            } else {
              last_s = sgn(i_cg);
              last_c = i_cg;
              last_j = ip;
              lc_ok = true;
              ++ip;
              ph = 2;
            }
          }
        }
      }
      // ---- the state the ray continues from (the bulk kernel's reload and event logic) ----
      if (U(root_done || (scan && !hit))) {
#pragma unroll
        for (int i = 0; i < 7; ++i) {
          u[i] = y[i];
          f[i] = kk[i];
        }
        bstart = bend;
      }
      if (U(hit)) mode = M_ROOT;
      if (U(root_done)) {
        const double tau_r = tau + hs;
        int a = 0;
        {  // affect! (RayTracer.jl:301-350) as the bulk kernel's affect(), stored by lane 0
          double st, ct, sp, cp;
          msincos(u[1], st, ct);
          msincos(u[2], sp, cp);
          bool skip = false;
          if (ncross == 0) {
            const double sc = 1.0001;
            const double pos[3] = {st * cp * u[0], st * sp * u[0], ct * u[0]};
            bool all_lt = true, all_gt = true;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              const double x0i = fabs(in.x0[i * n + ray]);
              all_lt = all_lt && (fabs(pos[i]) < x0i * sc);
              all_gt = all_gt && (fabs(pos[i]) > x0i / sc);
            }
            skip = all_lt && all_gt;
          }
          if (!skip) {
            double x[3], k[3];
            sph_to_cart(u, erg, P.rs_eff, x, k);
            if (!(sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) < P.rNS101)) {
              const int j = ncross;
              if (lane == 0 && out.xcount && j < out.cap) {
                double2* rq = reinterpret_cast<double2*>(out.xrec + ((int64_t)ray * out.cap + j) * X_REC);
                rq[0] = make_double2(x[0], x[1]);
                rq[1] = make_double2(x[2], k[0]);
                rq[2] = make_double2(k[1], k[2]);
                rq[3] = make_double2(exp(tau_r), u[6] / erg);
              }
              ncross = j + 1;
              const int maxc = max_crossings <= 0 ? -1 : max_crossings;
              a = (ncross >= maxc) ? 2 : 1;
            }
          }
        }
        tau = tau_r;
        cprev = post_c;
        cprev_ok = true;
        sprev = post_s;
        just_evented = true;
        mode = M_STEP;
        if (a == 2) finish = ART_STATUS_CROSSING;
        else if (photon && u[0] < P.rNS101) finish = ART_STATUS_HIT_NS;
        else if (iter >= P.maxiters) finish = ART_STATUS_MAXITERS;
      }
      if (U(scan && !hit)) {
        tau = last ? tend : tau + hs;
        cprev = last_c;
        cprev_ok = lc_ok;
        sprev = last_s;
        just_evented = false;
        dt = dtnext;
        if (cbs && photon && u[0] < P.rNS101) finish = ART_STATUS_HIT_NS;
        else if (last) finish = ART_STATUS_SUCCESS;
        else if (iter >= P.maxiters) finish = ART_STATUS_MAXITERS;
      }
    }
    if (lane == 0) {  // the raw end record; finalize_kernel back-transforms it
      double2* rq = reinterpret_cast<double2*>(out.rec + (int64_t)ray * END_REC);
      rq[0] = make_double2(u[0], u[1]);
      rq[1] = make_double2(u[2], u[3]);
      rq[2] = make_double2(u[4], u[5]);
      rq[3] = make_double2(u[6], tau);
      int4* ri = reinterpret_cast<int4*>(rq + 4);
      ri[0] = make_int4(finish, n_acc, n_rej, ncross);
    }
  }
  if (lane == 0) {
    const unsigned v[6] = {s_att, s_acc, s_root, s_scan, s_interp, s_cert};
    const int slot[6] = {ST_ATTEMPTS, ST_ACCEPTED, ST_ROOT_STEPS, ST_SCAN_EVALS, ST_INTERP_EVALS, ST_CERT};
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (v[k]) atomicAdd(&stats[slot[k]], (unsigned long long)v[k]);
  }
  span_stamp(stats, true);
}

#ifndef ART_NOLICM_TU  // (non-template kernels: this translation unit only)
// Small batches (SegOut::small_tail): every fresh ray as a CONT_REC record for tail_kernel, the
// state the persistent integrator gives a ray it takes from the queue (its refill: u0, f0, dt
// and c0 from init_kernel, the controller's qold power at qoldinit = 1e-4, no b at the step
// start, counters at zero, the sign memory from c0), so a ray's arithmetic is the same whether
// a lane or a wave of its own integrates it (tests/test_edges.py compares small batches with
// large ones bit for bit).
__global__ __launch_bounds__(256) void pack_fresh_kernel(const int64_t n, const SegIn in, const SegOut out,
                                                         unsigned long long* __restrict__ stats) {
  const int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ray == 0) {
    *out.cont_count = (unsigned long long)n;
    atomicAdd(&stats[ST_RAYS], (unsigned long long)n);
  }
  if (ray >= n) return;
  const double qpow_init = pow(1e-4, 1.0 / 15.0);
  double v[20];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    v[i] = in.u0[ray * U0_REC + i];
    v[7 + i] = in.u0[ray * U0_REC + 7 + i];
  }
  const double cprev = in.u0[ray * U0_REC + 15];
  v[14] = in.lnt0[ray];
  v[15] = in.u0[ray * U0_REC + 14];
  v[16] = qpow_init;
  v[17] = cprev;
  v[18] = NAN;
  v[19] = in.erg[ray];
  double2* rq = reinterpret_cast<double2*>(out.cont + ray * CONT_REC);
#pragma unroll
  for (int i = 0; i < 10; ++i) rq[i] = make_double2(v[2 * i], v[2 * i + 1]);
  const int photon = in.species[ray] != ART_AXION;
  const int sprev = isnan(cprev) ? 0 : sgn(cprev);
  int4* ri = reinterpret_cast<int4*>(rq + 10);
  ri[0] = make_int4((int)ray, 0, 0, 0);
  ri[1] = make_int4(0, sprev, photon | 2 /* cprev_ok */, 1 /* save_k */);
}

#endif  // ART_NOLICM_TU
// Every initialisation and finalization of the library runs in helper_kernel, through ONE call
// site of init_one and ONE of finalize_one: their arithmetic (the right-hand side's "fast"
// contraction included) is then the same machine code for every path -- the single launch, the
// chunked and CU-masked pipelines and the maskless streamed one -- so their outputs agree bit
// for bit (tests/test_edges.py). (Inlined into two kernels, the photon RHS of init_one had
// contracted differently: profiles/r04m_pytest.log.)
//   HK_INIT  rays [i0, i1): fresh state into in.u0 (grid-stride over 256-ray tiles);
//   HK_FIN   rays [i0, i1): the end state into `out` at o = i - i0, row stride i1 - i0;
//   HK_TILES the maskless streamed pipeline's helper duty (SegOut::host_ready ...): claim
//            1024-ray tiles (S3_TILE) to initialise once the host's copies of their inputs have landed,
//            and tiles of each finished piece to finalize into its blob; flag each initialised
//            chunk (chunk_ready, which the integrator's waves poll) and each finalized piece
//            (host_flags, which the host polls). init_limit >= 0: initialise only, until every
//            tile below it is claimed (the pass that starts the launch); -1: serve until every
//            tile is initialised and finalized. announce: count this block into *host_started
//            (the host launches the integrator once every persistent helper block is resident).
//            Each hand-off: the block's stores, s_waitcnt, barrier, one agent-scope release,
//            then the flag (MI355X_MICROARCH.md, inter-workgroup visibility); readers poll the
//            flag and take one agent-scope acquire.
enum { HK_INIT = 0, HK_FIN = 1, HK_TILES = 2 };
// Instantiated per geometry like the integrator (the same folded physics), for 2 waves per SIMD:
// a helper wave then shares a SIMD with one integrator wave, so the streamed pipeline's persistent
// helpers take one integrator block slot each instead of a whole CU. The builds need 158-203
// VGPRs and no scratch (-disable-machine-licm, build.py); helper_waves_per_simd checks that at
// run time, because a scratch-spilling persistent helper stalled the next launch on another
// queue for seconds (the runtime growing that queue's scratch while the helpers held theirs).
#ifdef ART_NOLICM_TU
template <int GEOM>
__global__ __launch_bounds__(256, 2) void helper_kernel(
    const KParams P_in, const int64_t n, const SegIn in, const SegOut out, const int mode, const int64_t i0,
    const int64_t i1, const int64_t init_limit, const int announce, unsigned long long* __restrict__ stats) {
  const KParams P = specialize<GEOM>(P_in);
  __shared__ long long cmd[2];  // HK_TILES: [what, tile]: 0 nothing now, 1 initialise, 2 finalize, 3 done
  __shared__ double hfl[2 * FLUX_HELPER_BINS];  // (HK_TILES with SegOut::flux_hist) this block's flux counts
  __shared__ int last_out, complete;
  const int tid = threadIdx.x;
  // the persistent helpers share their SIMDs with integrator waves (2 waves per SIMD): their claims,
  // hand-offs and tiles run at the top issue priority, so the initialisation keeps ahead of the
  // integrator's chunk claims (at the integrator's priorities the idle polls starved and the calls
  // gave up); between polls they sleep
  if (mode == HK_TILES) __builtin_amdgcn_s_setprio(3);
  const bool flb = mode == HK_TILES && out.flux_hist != nullptr;
  if (flb)
    for (int b = tid; b < 2 * out.flux_nbins; b += 256) hfl[b] = 0.0;
  __syncthreads();
  const int64_t full = (int64_t)1 << out.piece_shift;
  auto piece_rays = [&](int p) {
    const int64_t lo = (int64_t)p << out.piece_shift;
    return (n - lo) < full ? n - lo : full;
  };
  const int64_t TS = mode == HK_TILES ? S3_TILE : 256;  // rays per tile
  int64_t tile = blockIdx.x;
  unsigned long long hr = 0;  // (HK_TILES, thread 0) host_ready as last read: it only grows
  long long pend = -1;  // (HK_TILES, thread 0) a claimed finalize tile whose piece is still running
  unsigned long long t_idle = __builtin_amdgcn_s_memrealtime();
  unsigned npoll = 0;  // (HK_TILES, thread 0) claim rounds: every 16th reads the abort word
  unsigned nrhs = 0;
  if (mode == HK_TILES && announce && tid == 0)
    __hip_atomic_fetch_add(out.host_flags + 64, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  while (true) {
    long long what = 0, t = -1;
    if (mode != HK_TILES) {
      t = (long long)(i0 + tile * TS);
      if (t >= i1) break;
      what = mode == HK_INIT ? 1 : 2;
      tile += gridDim.x;
    } else {
      if (tid == 0) {
        // a given-up call (the host's or a wave's abort word) ends here: every 16th claim round
        // reads the word (a host-memory load, ~2 us), every wait below reads it each time
        if ((++npoll & 15u) == 0u && ld_abort(out)) what = 3;
        const unsigned long long inext = ld_agent(out.init_next);
        if (what == 0 && init_limit >= 0 && (int64_t)inext >= init_limit) what = 3;
        if (what == 0 && (int64_t)inext < n && inext >= hr) hr = ld_sys(out.host_ready);
        if (what == 0 && (int64_t)inext < n && inext < hr) {
          if (init_limit >= 0) {
            // the pass that starts the launch claims tiles below init_limit only (compare-and-
            // swap: with a blind add, every block that saw init_next below the limit claimed a
            // tile, far past the landed inputs, and the integrator behind this pass waited for them)
            unsigned long long cur = inext;
            while ((int64_t)cur < init_limit && (int64_t)cur < n) {
              const unsigned long long seen = atomicCAS(out.init_next, cur, cur + (unsigned long long)S3_TILE);
              if (seen == cur) {
                what = 1;
                t = (long long)cur;
                break;
              }
              cur = seen;
            }
            if (what == 0) what = 3;
          } else {
            const unsigned long long c = atomicAdd(out.init_next, (unsigned long long)S3_TILE);
            if ((int64_t)c < n) {  // (a tile past the landed inputs waits for them below)
              what = 1;
              t = (long long)c;
            }
          }
        }
        if (what == 0 && init_limit < 0) {
          if (pend < 0) {
            const unsigned long long fnext = ld_agent(out.fin_next);
            if ((int64_t)fnext < n) {
              const int p = (int)(fnext >> out.piece_shift);
              if ((int64_t)ld_agent(out.piece_cnt + p) == piece_rays(p)) {
                const unsigned long long c = atomicAdd(out.fin_next, (unsigned long long)S3_TILE);
                if ((int64_t)c < n) pend = (long long)c;
              }
            }
          }
          if (pend >= 0) {
            const int p = (int)(pend >> out.piece_shift);
            if ((int64_t)ld_agent(out.piece_cnt + p) == piece_rays(p)) {
              what = 2;
              t = pend;
              pend = -1;
            }
          }
          if (what == 0 && pend < 0 && (int64_t)inext >= n && (int64_t)ld_agent(out.fin_next) >= n) what = 3;
        }
        if (what == 1) {  // the tile's inputs (bounded wait)
          const int64_t t1 = (int64_t)t + S3_TILE < n ? (int64_t)t + S3_TILE : n;
          const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
          while ((int64_t)ld_sys(out.host_ready) < t1) {
            if (__hip_atomic_load(out.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
                __builtin_amdgcn_s_memrealtime() - w0 > S3_WAIT_TICKS) {
              __hip_atomic_store(out.abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              what = 3;
              break;
            }
            __builtin_amdgcn_s_sleep(32);
          }
        }
        if (what == 0 && (__hip_atomic_load(out.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
                          __builtin_amdgcn_s_memrealtime() - t_idle > S3_WAIT_TICKS)) {
          __hip_atomic_store(out.abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          what = 3;
        }
        // aborted: drain the integrator's work queue, so each of its waves stops at its next
        // chunk claim instead of integrating every chunk the helpers had flagged
        if (what == 3 && out.queue_word && ld_abort(out)) atomicAdd(out.queue_word, 1ull << 40);
        if (what == 1 || what == 2) {
          t_idle = __builtin_amdgcn_s_memrealtime();
          // the inputs the DMA engines wrote / the end records other CUs wrote
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        cmd[0] = what;
        cmd[1] = t;
      }
      __syncthreads();
      // (block-uniform: said so, so the tile's SegOut and bounds stay in scalar registers --
      // read as per-lane values they took ~100 VGPRs across the tile loop)
      what = (long long)__builtin_amdgcn_readfirstlane((int)cmd[0]);
      {
        const unsigned long long tw = (unsigned long long)cmd[1];
        t = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(tw >> 32)) << 32) |
                        (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)tw));
      }
      __syncthreads();
      if (what == 3) break;
      if (what == 0) {
        __builtin_amdgcn_s_sleep(16);
        continue;
      }
    }
    const int64_t t1 = t + TS < (mode == HK_TILES ? n : i1) ? t + TS : (mode == HK_TILES ? n : i1);
    if (what == 1) {  // (one call site of each)
#pragma unroll 1
      for (int64_t i = t + tid; i < t1; i += 256) nrhs += init_one(P, n, i, in);
    } else {
      SegOut ol = out;
      int64_t ob = i0, m = i1 - i0;
      if (mode == HK_TILES) {
        const int p = (int)(t >> out.piece_shift);
        ol = piece_blob(out, n, p, m);
        ob = (int64_t)p << out.piece_shift;
      }
#pragma unroll 1
      for (int64_t i = t + tid; i < t1; i += 256) finalize_one(P, n, i, i - ob, m, in, ol, flb ? hfl : nullptr, out.flux_nbins);
    }
    if (mode == HK_TILES) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (what == 2 && out.blob_host) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (the blob in host memory)
        else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (what == 1) {
          for (int64_t c = t / CHUNK; c * CHUNK < t1; ++c)
            __hip_atomic_store(out.chunk_ready + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          const int p = (int)(t >> out.piece_shift);
          const unsigned long long tiles = (unsigned long long)((piece_rays(p) + S3_TILE - 1) / S3_TILE);
          const unsigned long long old =
              __hip_atomic_fetch_add(out.piece_fin + p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (old + 1ull == tiles) {  // the piece's last tile: its blob is complete in memory
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(out.host_flags + p, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
      }
    }
  }
  unsigned long long x = nrhs;  // init RHS evaluations -> stats[6]
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  if ((tid & 63) == 0 && x) atomicAdd(&stats[6], x);
  if (mode == HK_TILES && init_limit < 0 && out.exit_count) {
    // the end of the call (SegOut::done_host): this block's flux counts into the call's histogram
    // (sums of 1.0: exact in any order), then the last serving block out copies the statistics
    // and the flux into host memory and raises the flag the host waits for
    __syncthreads();
    if (flb)
      for (int b = tid; b < 2 * out.flux_nbins; b += 256)
        if (hfl[b] != 0.0) atomicAdd(out.flux_hist + b, hfl[b]);
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long old = __hip_atomic_fetch_add(out.exit_count, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_out = (old + 1ull == (unsigned long long)out.exit_expected) ? 1 : 0;
    }
    __syncthreads();
    if (last_out) {
      if (tid == 0) {  // the integrator's started waves have added their statistics (they count themselves after)
        const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        const unsigned long long started = ld_agent(out.waves_started);
        while (ld_agent(out.waves_done) < started) {
          if (ld_abort(out) || __builtin_amdgcn_s_memrealtime() - w0 > STREAM_WAIT_TICKS) { ok = false; break; }
          __builtin_amdgcn_s_sleep(8);
        }
        complete = ok ? 1 : 2;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      __syncthreads();
      for (int k = tid; k < N_STATS_DEV; k += 256)
        __hip_atomic_store(out.done_host + DONE_STATS + k, ld_agent(stats + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (out.flux_hist)
        for (int b = tid; b < 2 * out.flux_nbins; b += 256)
          __hip_atomic_store(out.done_host + DONE_FLUX + b, ld_agent(reinterpret_cast<const unsigned long long*>(out.flux_hist) + b),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope)
        __hip_atomic_store(out.done_host, (unsigned long long)complete, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// the helper instantiation of the integrator's geometry (launch_propagate, launch_integrator_streamed)
HFn pick_helper(const KParams& P) {
  const bool flat = P.rs_eff == 0.0 && !(P.bndry_lyr > 0.0) && !P.isotropic;
  const bool sch = P.rs_eff > 0.0 && !(P.bndry_lyr > 0.0) && !P.isotropic;
  return flat ? helper_kernel<GEOM_FLAT> : (sch ? helper_kernel<GEOM_GR> : helper_kernel<GEOM_ANY>);
}
int helper_waves_per_simd(const KParams& P) {
  // 2 when the build for these parameters fits 2 waves per SIMD without scratch (read once per build)
  static std::atomic<int> cached[3];
  const HFn fn = pick_helper(P);
  const int g = fn == helper_kernel<GEOM_FLAT> ? 1 : (fn == helper_kernel<GEOM_GR> ? 2 : 0);
  int w = cached[g].load(std::memory_order_relaxed);
  if (!w) {
    hipFuncAttributes a{};
    const bool ok = hipFuncGetAttributes(&a, (const void*)fn) == hipSuccess;
    (void)hipGetLastError();
    w = (ok && a.localSizeBytes == 0 && a.numRegs > 0 && a.numRegs <= 256) ? 2 : 1;
    cached[g].store(w, std::memory_order_relaxed);
  }
  return w;
}

// The integrator and tail instantiations compiled here, without MachineLICM (art_kernels_nolicm.hip):
// every geometry but flat's Vern6/RK4 integrator. GR: the bulk launch 235.2-236.7 -> 227.3-228.7
// ms per 10^6 rays, the lone tail ray 7.69 -> 7.54 us per attempt (no spills: 256 VGPRs + 60 spilled
// -> 226), bit-identical (profiles/r06q_gr_licm.jsonl); the flat integrator stays in art_kernels.hip,
// 3% faster with the pass (profiles/r06o_ab_device_licm_off_everywhere.jsonl).
KFn nl_propagate(int integ, int geom, bool save, int don, int wps) {
#define ART_NL(I, G, S, D, W) \
  if (integ == I && geom == G && save == S && don == D && wps == W) return propagate_kernel<I, G, S, D, W>;
  ART_NL(ART_VERN6, GEOM_GR, true, 0, 2) ART_NL(ART_VERN6, GEOM_GR, true, 1, 2)
  ART_NL(ART_VERN6, GEOM_ANY, true, 0, 2) ART_NL(ART_VERN6, GEOM_ANY, true, 1, 2)
  ART_NL(ART_RK4, GEOM_ANY, true, 0, 2) ART_NL(ART_RK4, GEOM_ANY, true, 1, 2)
  ART_NL(ART_RK4, GEOM_ANY, false, 0, 2) ART_NL(ART_RK4, GEOM_ANY, false, 1, 2)
  ART_NL(ART_VERN6, GEOM_GR, false, 0, 2) ART_NL(ART_VERN6, GEOM_GR, false, 1, 2) ART_NL(ART_VERN6, GEOM_GR, false, 3, 2)
  ART_NL(ART_VERN6, GEOM_ANY, false, 0, 2) ART_NL(ART_VERN6, GEOM_ANY, false, 1, 2) ART_NL(ART_VERN6, GEOM_ANY, false, 3, 2)
  ART_NL(ART_VERN6, GEOM_GR, false, 0, 1) ART_NL(ART_VERN6, GEOM_GR, false, 1, 1)
#undef ART_NL
  return nullptr;
}
TFn nl_tail(int geom) { return geom == GEOM_FLAT ? tail_kernel<GEOM_FLAT> : (geom == GEOM_GR ? tail_kernel<GEOM_GR> : tail_kernel<GEOM_ANY>); }
#endif  // ART_NOLICM_TU


// ---------------------------------------------------------------------------
// find_samples_new (RayTracer.jl:1480-1653) + main_runner's erg and k_init
// (MainRunner.jl:511-529): persistent lanes, one ray per lane, one attempt per lane per outer
// iteration; all lanes of a wave walk their lines' 0.5 km Euler steps in lockstep.
//
// Per step, the ContinuousCallback(interp_points = 20) scan (:1603-1613) is WAVE-COOPERATIVE:
//   * a step whose every point is provably below the resonance (certified negative, below)
//     needs only its last point -- the value the next step's first bracket starts from;
//   * every other step needs its 19 points.
// Those items (source lane, point) of the whole wave are evaluated 64 at a time by all lanes
// on the source lines (kept in LDS), so one lane's uncertified step no longer makes the whole
// wave evaluate 19 points. Each item leaves the signbit and nonzero-ness of its value in its
// source lane's bit masks; a lane then finds its sign changes (the reference's brackets:
// signbit differs, both values nonzero) with bit operations. Brackets are queued (in each
// lane's order of discovery) and resolved 64 at a time -- Illinois on the exact line and the
// affect! test (rr > rNS, E_loc > ωp, :1585-1597) -- and each lane then counts its valid
// crossings in order and keeps the randInx-th (:1623-1636). Every value is computed by the same
// expression on the same operands as a per-lane scan would, so the samples do not change.
constexpr int SQCAP = 128;  // bracket queue entries per wave

// closest approach of the line x0 + va s to the centre within [s0, s1], squared
__device__ inline double line_rmin2(const double* x0, const double* va, double s0, double s1) {
  const double sd = -(x0[0] * va[0] + x0[1] * va[1] + x0[2] * va[2]);
  const double sm = fmin(fmax(sd, s0), s1);
  double xm[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) xm[i] = x0[i] + va[i] * sm;
  return xm[0] * xm[0] + xm[1] * xm[1] + xm[2] * xm[2];
}

// The sampler's certificates on the segment [s0, s1] of a line (x0 + va s, energy E): 1 when every
// point of it provably has a negative condition, 2 when every point provably has a positive one,
// 0 otherwise. The bounds are derived at sample_kernel's step loop; both hold for a segment of any
// length (a block of steps as well as one step) and whatever the sign of the point before it.
__device__ inline int seg_cert(const KParams& P, const double* X0, const double* VA, double E, double s0, double s1,
                               double cert_lhs, double cert_rhs) {
  // The radii's square root and the three reciprocals in single precision (v_sqrt_f32, v_rcp_f32 of
  // the rounded operand: relative error < 3e-7 each): every bound below is widened by 2e-6 (db, the
  // negative test) or 1e-6 (g^rr, bmin, rmin > 10) to stay conservative, and the negative test's
  // own 1e-6 margin on m_a² is kept whole; a certified segment is still provably one-signed.
  const double rm2 = line_rmin2(X0, VA, s0, s1);
  const double rmin = (double)__builtin_amdgcn_sqrtf((float)rm2);
  double xa[3], xb[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) { xa[i] = X0[i] + VA[i] * s0; xb[i] = X0[i] + VA[i] * s1; }
  const double ra2 = xa[0] * xa[0] + xa[1] * xa[1] + xa[2] * xa[2];
  const double rb2 = xb[0] * xb[0] + xb[1] * xb[1] + xb[2] * xb[2];
  const double ba = (P.cm * (3.0 * xa[2] * xa[2] - ra2) + 3.0 * P.sm * xa[0] * xa[2]) * (double)__builtin_amdgcn_rcpf((float)ra2);
  const double bb = (P.cm * (3.0 * xb[2] * xb[2] - rb2) + 3.0 * P.sm * xb[0] * xb[2]) * (double)__builtin_amdgcn_rcpf((float)rb2);
  const double irmin = (double)__builtin_amdgcn_rcpf((float)rmin);
  const double al = (s1 - s0) * irmin;
  const double db = 0.75 * al * al * (1.0 + 2e-6) + 1e-12;
  const double bmax = fmin(2.0, fmax(fabs(ba), fabs(bb)) * (1.0 + 1e-6) + db);
  if (cert_lhs * 0.5 * bmax < cert_rhs * (rm2 * rmin) * (1.0 - 2e-6)) return 1;
  if (rmin > 10.0 * (1.0 + 1e-6)) {
    const double bmin = (ba * bb > 0.0) ? fmin(fabs(ba), fabs(bb)) * (1.0 - 1e-6) - db : -1.0;
    const double rmax2 = fmax(ra2, rb2);
    const double grr = 1.0 - P.rs_gr * irmin * (1.0 + 1e-6);  // (rounded down: a smaller g^rr)
    if (bmin > 0.0 && P.wp2n * bmin * grr > E * E * (1.0 + 1e-6) * (rmax2 * sqrt(rmax2))) return 2;
  }
  return 0;
}

// Two builds, by waves per SIMD (the LDS allows 3): at 3 the kernel spills a few
// loop-invariant values, reloaded once per scan step -- a good trade where a line has ~111
// steps with uncertified ones among them, not where it has ~650 mostly skipped ones
// (launch_sample picks by the line length).
template <int WPS, bool BLOCKS>
__global__ __launch_bounds__(256, WPS) void sample_kernel(const KParams P, const double maxR, const uint64_t seed,
                                                     const int64_t ray_offset, const int64_t n, double* __restrict__ xo,
                                                     double* __restrict__ ko, double* __restrict__ ergo,
                                                     double* __restrict__ vifo, int32_t* __restrict__ wo,
                                                     int32_t* __restrict__ ao, unsigned long long* __restrict__ queue) {
  // line data of every lane [component][lane]: x0 (3), va (3), vl (3), E, 1/E², vIfty (3).
  // A lane reads its own line from here too (its registers hold none of it across the step
  // loop: the kernel fits 2 waves/SIMD without spills)
  __shared__ double sline[14 * 256];
  __shared__ double slast[256];           // value at the step's last point
  __shared__ unsigned char ssrc[2 * 256];  // compact lists: uncertified lanes, certified lanes
  __shared__ double sqa[4 * SQCAP], sqb[4 * SQCAP];  // bracket queue: ends -> root
  __shared__ unsigned char sqsrc[4 * SQCAP], sqok[4 * SQCAP];
  __shared__ double sgrid[32];  // (0.5 j)/19: a full step's grid offsets, the same rounding as the division
  __shared__ unsigned char spair[4 * 64 * 3];  // a wave's (lane, step of the block) pairs to scan: lane << 2 | step
  __shared__ unsigned sbm[256];  // (step-by-step scan) a lane's sign changes of the step not queued yet
  const int lane = threadIdx.x & 63;
  const int wb = threadIdx.x & ~63;
  const int wq = (threadIdx.x >> 6) * SQCAP;
  double* const Lx = sline + threadIdx.x;
  int64_t ray = -1;
  uint32_t attempt = 0;
  int64_t wnext = 0, wend = 0;
  bool exhausted = false;
  const double send = 2.2 * maxR;
  const int nsteps = (int)ceil(send / 0.5);
  const int np = 20;  // ContinuousCallback(interp_points=20) (:1603)
  const int nper = np - 1;
  // certified-negative scan steps: GJ plasma without a boundary layer only (ART_SCAN_CERT=0: off)
  const bool cert_ok = !(P.bndry_lyr > 0.0) && P.mass_a > 0.0 && P.cert_fac < 1e300;
  const double cert_lhs = 2.0 * P.wp2n, cert_rhs = P.mass_a2 * (1.0 - 1e-6);
  // r_win³ = 2 wp2n / (m_a² (1 - 1e-6)) with a margin: ωp² < m_a² (1 - 1e-6) beyond it
  const double r_win2 = cert_ok ? pow(cert_lhs / cert_rhs, 2.0 / 3.0) * (1.0 + 3e-6) : 0.0;
  // sampler_sign_fast's domain (the condition's exterior branch: r > 10 km, r >= rNS) with a margin,
  // and the radius below which both ends of a step put all of it inside the star
  const double r_lim = fmax(10.0, P.rNS) * (1.0 + 1e-9), r_lim2 = r_lim * r_lim;
  const double r_in2 = (P.rNS * (1.0 - 1e-9)) * (P.rNS * (1.0 - 1e-9));
  const unsigned long long lt = (1ull << lane) - 1ull;
  if (threadIdx.x < np) sgrid[threadIdx.x] = 0.5 * double(threadIdx.x) / double(np - 1);
  __syncthreads();
#ifdef ART_SAMPLER_SECTIONS
  // dev build: s_memtime cycles per section, summed over the wave's iterations, into queue[8..15]
  // [refill + line set-up, step loop control + window, certificate, grid pass, brackets + flush,
  //  sample out]; queue[14] wave-steps with a grid pass, queue[15] wave-steps run
  unsigned long long q_sec[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long q_last = __builtin_amdgcn_s_memtime();
#define ART_QMARK(k)                                                \
  {                                                                 \
    const unsigned long long q_now_ = __builtin_amdgcn_s_memtime(); \
    q_sec[k] += q_now_ - q_last;                                    \
    q_last = q_now_;                                                \
  }
#else
#define ART_QMARK(k)
#endif
  while (true) {
    if (!exhausted) {
      unsigned long long need = __ballot(ray < 0);
      while (need != 0ull && !exhausted) {
        if (wnext >= wend) {
          unsigned long long base = 0;
          const int leader = __ffsll((long long)need) - 1;
          if (lane == leader) base = atomicAdd(queue, (unsigned long long)CHUNK);
          base = __shfl(base, leader);
          if ((int64_t)base >= n) { exhausted = true; break; }
          wnext = (int64_t)base;
          wend = (wnext + CHUNK < n) ? wnext + CHUNK : n;
        }
        const int rank = __popcll(need & lt);
        const int64_t avail = wend - wnext;
        const int take = (int)(avail < (int64_t)__popcll(need) ? avail : (int64_t)__popcll(need));
        if (ray < 0 && rank < take) { ray = wnext + rank; attempt = 0; }
        wnext += take;
        need = __ballot(ray < 0);
      }
    }
    if (__ballot(ray >= 0) == 0ull) break;
    const bool active = ray >= 0;

    // ---- one attempt of every active lane: its line (:1486-1531) ----
    double U[10];
    attempt_uniforms(seed, uint64_t(ray_offset + (active ? ray : 0)), attempt, U);
    // sin(acos c) as √((1 - c)(1 + c)) and the FMA sincos of the integrator (arguments in
    // [0, 2π)): equal to the reference's values to an ulp, without ocml's acos and its
    // large-argument sincos path, whose registers set the kernel's occupancy
    double sti, cti, spi, cpi, stl, ctl, spl, cpl, sR, cR;
    cti = 1.0 - 2.0 * U[0];
    sti = sqrt((1.0 - cti) * (1.0 + cti));
    msincos(U[1] * 2.0 * PI, spi, cpi);
    ctl = 1.0 - 2.0 * U[2];
    stl = sqrt((1.0 - ctl) * (1.0 + ctl));
    msincos(U[3] * 2.0 * PI, spl, cpl);
    msincos(U[4] * 2.0 * PI, sR, cR);
    const double rR = sqrt(U[5]) * maxR;
    const double va[3] = {sti * cpi, sti * spi, cti};
    const double vl[3] = {stl * cpl, stl * spl, ctl};
    const double x1 = rR * cR, x2 = rR * sR;
    // rotate (x1, x2, 0) by Inv[EulerMatrix(ϕi, θi, 0)] (:1523-1524); cos(-a) = cos a, sin(-a) = -sin a
    double x0[3] = {x1 * cpi * cti - x2 * spi, x2 * cpi + x1 * spi * cti, -x1 * sti};
    double vI[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) vI[i] = (220.0 + U[6 + i] * 1.0e-5) / sqrt(3.0);
    const double vmag = sqrt(vI[0] * vI[0] + vI[1] * vI[1] + vI[2] * vI[2]);
    const double gammaA = 1.0 / sqrt(1.0 - (vmag / C_KM) * (vmag / C_KM));
    const double E = P.mass_a * sqrt(1.0 + (vmag / C_KM * gammaA) * (vmag / C_KM * gammaA));
    const double iE2 = 1.0 / (E * E);
#pragma unroll
    for (int i = 0; i < 3; ++i) x0[i] += va[i] * (-maxR * 1.1);
    int randInx = 1 + (int)(U[9] * 6.0);
    if (randInx > 6) randInx = 6;
    int count = 0;
    double xsel[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      Lx[i * 256] = x0[i];
      Lx[(3 + i) * 256] = va[i];
      Lx[(6 + i) * 256] = vl[i];
    }
    Lx[9 * 256] = E;
    Lx[10 * 256] = iE2;
#pragma unroll
    for (int i = 0; i < 3; ++i) Lx[(11 + i) * 256] = vI[i];
    double c_prev = sampler_condition_e(P, x0, vl, E, iE2);
    int qn = 0;  // queued brackets (wave-uniform)
    // This line's window: its chord through the sphere r <= r_win, outside which
    // ωp² <= 2 wp2n / r³ < m_a² (1 - 1e-6) on every point (|b| <= 2), so every step there is
    // certified negative once the point before is negative -- the certificate below would say
    // so too, step by step; here it costs one comparison, and a wave whose lanes are all
    // outside their windows jumps to the next window (the big-maxR scan points walk ~650
    // steps per line, ~99% of them certified).
    double w_in = 1e300, w_out = -1e300;
    if (active && cert_ok) {
      const double sc = -(x0[0] * va[0] + x0[1] * va[1] + x0[2] * va[2]);
      const double h2 = r_win2 - ((x0[0] * x0[0] + x0[1] * x0[1] + x0[2] * x0[2]) - sc * sc);
      if (h2 > 0.0) {
        const double h = sqrt(h2);
        w_in = sc - h - 1e-6;
        w_out = sc + h + 1e-6;
      }
    }

    // resolve the queued brackets: Illinois on the exact line (the lane that found one owns
    // it), then each owner counts its valid crossings in queue order and keeps the randInx-th
    auto flush = [&]() {
      wave_lds_sync();
      #pragma unroll 1
      for (int t = lane; t < qn; t += 64) {
        const int src = sqsrc[wq + t];
        const double* S = sline + wb + src;
        const double X0[3] = {S[0], S[256], S[2 * 256]}, VA[3] = {S[3 * 256], S[4 * 256], S[5 * 256]};
        const double VL[3] = {S[6 * 256], S[7 * 256], S[8 * 256]};
        const double Es = S[9 * 256], iEs = S[10 * 256];
        double a = sqa[wq + t], b = sqb[wq + t], root = b;
        double xr[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) xr[i] = X0[i] + VA[i] * a;
        double fa = sampler_condition_e(P, xr, VL, Es, iEs);
#pragma unroll
        for (int i = 0; i < 3; ++i) xr[i] = X0[i] + VA[i] * b;
        double fb = sampler_condition_e(P, xr, VL, Es, iEs);
        int side = 0;
        #pragma unroll 1
        for (int it = 0; it < 100; ++it) {  // Illinois on the exact line
          root = a - fa * (b - a) / (fb - fa);
#pragma unroll
          for (int i = 0; i < 3; ++i) xr[i] = X0[i] + VA[i] * root;
          const double fr = sampler_condition_e(P, xr, VL, Es, iEs);
          if (fr == 0.0 || (b - a) < 1e-13 * fmax(1.0, fabs(root))) break;
          if (signbit(fr) == signbit(fa)) { a = root; fa = fr; if (side == -1) fb *= 0.5; side = -1; }
          else { b = root; fb = fr; if (side == 1) fa *= 0.5; side = 1; }
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) xr[i] = X0[i] + VA[i] * root;
        // affect! (:1585-1597): keep crossings outside the star with E_loc > ωp
        const double rr = sqrt(xr[0] * xr[0] + xr[1] * xr[1] + xr[2] * xr[2]);
        double gtt, grr;
        metric_tr(rr, P.rs_gr, gtt, grr);
        sqa[wq + t] = root;
        sqok[wq + t] = (rr > P.rNS && Es / sqrt(grr) > wp_cart(P, xr)) ? 1 : 0;
      }
      wave_lds_sync();
      for (int t = 0; t < qn; ++t) {
        if (sqsrc[wq + t] == lane && sqok[wq + t] && active) {
          ++count;
          if (count == randInx) {
            const double r = sqa[wq + t];
#pragma unroll
            for (int i = 0; i < 3; ++i) xsel[i] = Lx[i * 256] + Lx[(3 + i) * 256] * r;
          }
        }
      }
      qn = 0;
      wave_lds_sync();
    };

    ART_QMARK(0)
    if constexpr (BLOCKS) {
    // Blocks of KB = 3 steps (1.5 km). Per block: ONE certificate of the whole block per lane (most
    // blocks away from the conversion surface pass it); the steps of the lanes whose block failed
    // are certified one by one as wave-cooperative items (lane, step); the grid points of every
    // uncertified (lane, step) pair of the block are evaluated together, 64 items a pass, so a pass
    // is rarely left part-empty. A certificate holds whatever the point before it (the sign logic
    // below sees a certified point as the value it provably has: nonzero, of the certified sign),
    // so a block or step is certified whatever c_prev is, and a sign change at its first point is
    // found by the same bit logic as an evaluated one. The evaluated points and their arithmetic
    // are those of the step-by-step scan (ART_SAMPLER_STEPWISE), so the samples do not change.
    // (the step masks of a block share 64-bit words: at most 3 steps; blocks of 2 measured slower,
    // 128 vs 119 ms per 1e7 flat samples, profiles/r05h_ab_sampler.txt)
    constexpr int KB = 3;
    const int wp = (threadIdx.x >> 6) * 64 * KB;  // this wave's pair list in spair
    for (int st0 = 0; st0 < nsteps; st0 += KB) {
#ifdef ART_SAMPLER_SECTIONS
      q_sec[7] += 1;
#endif
      const int kmax = min(KB, nsteps - st0);
      const double S0 = st0 * 0.5;
      const double S1 = fmin((st0 + kmax - 1) * 0.5 + 0.5, send);
      const bool quiet = !active || (cert_ok && c_prev < 0.0 && (S1 < w_in || S0 > w_out));
      if (__ballot(!quiet) == 0ull) {
        // every lane outside its window: jump to one step before the earliest next window start
        int nxt = (active && S1 < w_in && w_in < send) ? (int)floor(w_in * 2.0) - 1 : nsteps;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) nxt = min(nxt, __shfl_xor(nxt, o));
        nxt = __builtin_amdgcn_readfirstlane(nxt);  // (wave-uniform: keeps the step counter and kmax scalar)
        if (nxt > st0 + KB) st0 = nxt - KB;
        continue;
      }
      ART_QMARK(1)
      int bc = 0;  // the whole block certified: 1 negative, 2 positive
      if (active && quiet) {
        bc = 1;  // outside its window after a negative point
      } else if (active && cert_ok) {
        const double X0[3] = {Lx[0], Lx[256], Lx[2 * 256]}, VA[3] = {Lx[3 * 256], Lx[4 * 256], Lx[5 * 256]};
        bc = seg_cert(P, X0, VA, E, S0, S1, cert_lhs, cert_rhs);
      }
      const unsigned kmask = (1u << kmax) - 1u;
      unsigned cneg = bc == 1 ? kmask : 0u, cpos = bc == 2 ? kmask : 0u;  // certified steps, bit k
      // the steps of the lanes whose block failed, certified as items (lane u, step k), t = u kmax + k
      const bool fail = active && cert_ok && bc == 0 && kmax > 1;
      const unsigned long long mF = __ballot(fail);
      if (mF != 0ull) {
        const int nF = __popcll(mF);
        const int fix = __popcll(mF & lt);
        if (fail) ssrc[wb + fix] = (unsigned char)lane;
        wave_lds_sync();
        const int totc = nF * kmax;
        #pragma unroll 1
        for (int w0 = 0; w0 < totc; w0 += 64) {
          const int t = w0 + lane;
          int r = 0;
          if (t < totc) {
            const int u = t / kmax;
            const int k = t - u * kmax;
            const double* S = sline + wb + ssrc[wb + u];
            const double X0[3] = {S[0], S[256], S[2 * 256]}, VA[3] = {S[3 * 256], S[4 * 256], S[5 * 256]};
            const double s0 = (st0 + k) * 0.5;
            r = seg_cert(P, X0, VA, S[9 * 256], s0, fmin(s0 + 0.5, send), cert_lhs, cert_rhs);
          }
          const unsigned long long mn = __ballot(r == 1), mp = __ballot(r == 2);
          if (fail) {
            const int a = fix * kmax;
            const int lo = max(a, w0), hi = min(a + kmax, w0 + 64);
            if (lo < hi) {
              const unsigned long long run = (1ull << (hi - lo)) - 1ull;
              cneg |= (unsigned)((mn >> (lo - w0)) & run) << (lo - a);
              cpos |= (unsigned)((mp >> (lo - w0)) & run) << (lo - a);
            }
          }
        }
        wave_lds_sync();
      }
      ART_QMARK(2)
      // the uncertified (lane, step) pairs, lane-major, each lane's in step order: their grid points
      // are the items t = pair nper + j - 1, and each owner takes its pairs' runs of the ballots
      const unsigned unc = active ? (kmask & ~(cneg | cpos)) : 0u;
      const int m = __popc(unc);
      const unsigned long long b0 = __ballot(m & 1), b1 = __ballot(m & 2);
      const int off = __popcll(b0 & lt) + 2 * __popcll(b1 & lt);
      const int npairs = __popcll(b0) + 2 * __popcll(b1);
      // bits [20 k, 20 k + 20): signbit / nonzero-ness of step k's point j (bit 0: the point before it)
      unsigned long long sb = 0ull, nz = 0ull;
      if (npairs > 0) {
#ifdef ART_SAMPLER_SECTIONS
        q_sec[6] += 1;
#endif
        {
          unsigned rem = unc;
          for (int i = 0; rem != 0u; ++i) {
            spair[wp + off + i] = (unsigned char)(lane << 2 | __builtin_ctz(rem));
            rem &= rem - 1u;
          }
        }
        wave_lds_sync();
        const int tot = npairs * nper;
        __builtin_amdgcn_s_setprio(0);
        #pragma unroll 1
        for (int w0 = 0; w0 < tot; w0 += 64) {
          const int t = w0 + lane;
          bool neg = false, nonz = false;
          if (t < tot) {
            const int pr = t / nper;
            const int j = t - pr * nper + 1;
            const int e = spair[wp + pr];
            const int src = e >> 2, k = e & 3;
            const double* S = sline + wb + src;
            const double s0 = (st0 + k) * 0.5;
            const double s1 = fmin(s0 + 0.5, send);
            // (s1 - s0) j / 19: from the table for a full 0.5 km step, else divided
            const double sc = s0 + (s1 - s0 == 0.5 ? sgrid[j] : (s1 - s0) * double(j) / double(np - 1));
            double xl[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) xl[i] = S[i * 256] + S[(3 + i) * 256] * sc;
            const double VL[3] = {S[6 * 256], S[7 * 256], S[8 * 256]};
            const int fs = cert_ok ? sampler_sign_fast(P, xl, VL, P.mass_a2 * S[10 * 256], r_lim2) : 0;
            double v = fs == 1 ? -1.0 : 1.0;  // (a decided point: only its sign and nonzero-ness are read)
            if (fs == 0) v = sampler_condition_e(P, xl, VL, S[9 * 256], S[10 * 256]);
            if (j == nper && k == kmax - 1) slast[wb + src] = v;
            neg = signbit(v);
            nonz = v != 0.0;
          }
          const unsigned long long mneg = __ballot(neg), mnz = __ballot(nonz);
          unsigned rem = unc;
          for (int i = 0; rem != 0u; ++i) {
            const int k = __builtin_ctz(rem);
            rem &= rem - 1u;
            const int a = (off + i) * nper;
            const int lo = max(a, w0), hi = min(a + nper, w0 + 64);
            if (lo < hi) {
              const unsigned long long run = (1ull << (hi - lo)) - 1ull;
              const int at = 20 * k + (lo - a) + 1;
              sb |= ((mneg >> (lo - w0)) & run) << at;
              nz |= ((mnz >> (lo - w0)) & run) << at;
            }
          }
        }
        __builtin_amdgcn_s_setprio(1);
        wave_lds_sync();
      }
      ART_QMARK(3)
      if (active) {
        // certified steps: points 1..19 nonzero and of the certified sign
        const unsigned long long p19 = 0xFFFFEull;
        for (int k = 0; k < kmax; ++k) {
          if ((cneg >> k) & 1u) { sb |= p19 << (20 * k); nz |= p19 << (20 * k); }
          else if ((cpos >> k) & 1u) nz |= p19 << (20 * k);
        }
        // bit 0 of each step: the point before it (c_prev, then the previous step's point 19)
        sb |= signbit(c_prev) ? 1ull : 0ull;
        nz |= (c_prev != 0.0) ? 1ull : 0ull;
        for (int k = 1; k < kmax; ++k) {
          sb |= ((sb >> (20 * k - 1)) & 1ull) << (20 * k);
          nz |= ((nz >> (20 * k - 1)) & 1ull) << (20 * k);
        }
        const int kl = kmax - 1;  // the value the next block's first bracket starts from (read for its sign)
        if ((unc >> kl) & 1u) c_prev = slast[threadIdx.x];
        else if ((cneg >> kl) & 1u) c_prev = -1.0;
        else if ((cpos >> kl) & 1u) c_prev = 1.0;
      }
      // queue the sign changes in (point j-1, point j] of each step (signbits differ, both nonzero),
      // step by step, so each lane's brackets stay in their order along the line
      for (int k = 0; k < kmax; ++k) {
        const int st = st0 + k;
        const double s0 = st * 0.5;
        const double s1 = fmin(s0 + 0.5, send);
        const unsigned sbk = (unsigned)(sb >> (20 * k)) & 0xFFFFFu, nzk = (unsigned)(nz >> (20 * k)) & 0xFFFFFu;
        unsigned br = active ? (sbk ^ (sbk << 1)) & nzk & (nzk << 1) & (((1u << np) - 1u) & ~1u) : 0u;
        unsigned long long bm = __ballot(br != 0u);
        if (bm == 0ull) continue;
        // the previous step's last grid point, where a bracket at point 1 opens
        const double ps0 = (st - 1) * 0.5;
        const double pds = fmin(ps0 + 0.5, send) - ps0;
        const double s_start = st == 0 ? 0.0 : ps0 + (pds == 0.5 ? sgrid[nper] : pds * double(nper) / double(np - 1));
        while (bm != 0ull) {
          if (qn + 64 > SQCAP) flush();
          if (br != 0u) {
            const int ip = __builtin_ctz(br);
            const int slot = qn + __popcll(bm & lt);
            sqa[wq + slot] = (ip == 1) ? s_start : s0 + (s1 - s0) * double(ip - 1) / double(np - 1);
            sqb[wq + slot] = s0 + (s1 - s0) * double(ip) / double(np - 1);
            sqsrc[wq + slot] = (unsigned char)lane;
            br &= br - 1u;
          }
          qn = __builtin_amdgcn_readfirstlane(qn + __popcll(bm));  // (wave-uniform)
          bm = __ballot(br != 0u);
        }
      }
      ART_QMARK(4)
    }
    } else {  // step by step (round 4)
    // The bracket queue is resolved (flush: Illinois with its three inlined conditions) at the top
    // of this loop and after it, not inside the insertion below: a queue that fills up there ends
    // the pass, the rest wait in sbm, and the loop comes back to the same step after resolving it.
    // Inside the insertion the flush's registers stacked on the step's live state: 71 spilled VGPRs
    // in the 3-wave build, 51 now; 10^7 flat samples 118 -> 115 ms, bit-identical
    // (profiles/r05q_ab_sampler_flush.txt). (The block scan, 2 waves/SIMD, does not spill.)
    bool sres = false;  // (wave-uniform) this step's brackets wait behind a full queue
    for (int st = 0; st < nsteps;) {
      const double s0 = st * 0.5;
      const double s1 = fmin(s0 + 0.5, send);
      if (sres) {
        flush();
      } else {
#ifdef ART_SAMPLER_SECTIONS
      q_sec[7] += 1;
#endif
      const bool quiet = !active || (cert_ok && c_prev < 0.0 && (s1 < w_in || s0 > w_out));
      if (__ballot(!quiet) == 0ull) {
        // every lane is certified outside its window: jump to one step before the earliest
        // next window start (certified steps change nothing but the step counter)
        int nxt = (active && s1 < w_in && w_in < send) ? (int)floor(w_in * 2.0) - 1 : nsteps;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) nxt = min(nxt, __shfl_xor(nxt, o));
        nxt = __builtin_amdgcn_readfirstlane(nxt);  // (wave-uniform: keeps the step counter scalar)
        st = nxt > st + 1 ? nxt : st + 1;
        continue;
      }
      // Certified-negative step: with the axion shell imposed (w normalised), the condition
      // is ½(-m_a² + ωp² (1 - g^rr k∥²/E²))/E² with 0 <= g^rr k∥² <= E² (Cauchy-Schwarz, the
      // factor is at most 1), and ωp² = wp2n |b| / r³ <= 2 wp2n / r³ (|b| <= √(4a1² + a2²)
      // <= 2). Where 2 wp2n / r_min³ stays below m_a² on the whole segment (r_min: the line's
      // closest approach to the centre within [s0, s1]), all its points are negative. If the
      // point before is negative too, no sign change can occur: only the last point is
      // evaluated, for the value a bracket opening at the next step's first point starts from.
      //
      // Both bounds use b = Bz/B_n at the step's two end points, b = cosθm (3z² - r²)/r² +
      // 3 sinθm x z / r² (ψ = φ at t = 0): a quadratic form n̂ᵀ M n̂ of the direction n̂, M with
      // eigenvalues -cosθm and (cosθm ± 3)/2, so λmax - λmin = 3. The step projects onto a
      // great-circle arc of angle α <= L/r_min (the radial projection shrinks lengths by 1/|x|),
      // along which b(φ) = C + A cos 2φ + B sin 2φ with √(A² + B²) <= (λmax - λmin)/2, so
      // |b''| <= 6 and b stays within 6 α²/8 of the chord between its end values:
      // |b| <= min(2, max(|b_a|, |b_b|) + 0.75 α²), and where b_a, b_b share a sign,
      // |b| >= min(|b_a|, |b_b|) - 0.75 α². (Until round 3 the bound was the first-order
      // |b_a| ± (3 + 3|sinθm|) α, about 100x wider at 0.5 km steps: the uncertified steps
      // drop by a third)
      //  * negative: ωp² <= wp2n |b|max / r_min³ < m_a² (see above);
      //  * positive (the point before positive too): outside g_schwartz's interior patch
      //    (r > 10 km), g^rr g^tt = -1, so Cauchy-Schwarz on k∥ with w on the axion shell gives
      //    1 - g^rr k∥²/E² >= g^rr m_a²/E² and the condition >= ½ m_a² (ωp² g^rr/E² - 1)/E² > 0
      //    when wp2n |b|min g^rr(r_min) > E² r_max³ (r_max: at an end of the step).
      ART_QMARK(1)
      bool cert = active && quiet;
      if (active && !quiet && cert_ok && c_prev != 0.0 && !isnan(c_prev)) {
        const double X0[3] = {Lx[0], Lx[256], Lx[2 * 256]}, VA[3] = {Lx[3 * 256], Lx[4 * 256], Lx[5 * 256]};
        const double rm2 = line_rmin2(X0, VA, s0, s1);
        const double rmin = (double)__builtin_amdgcn_sqrtf((float)rm2);
        double xa[3], xb[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) { xa[i] = X0[i] + VA[i] * s0; xb[i] = X0[i] + VA[i] * s1; }
        const double ra2 = xa[0] * xa[0] + xa[1] * xa[1] + xa[2] * xa[2];
        const double rb2 = xb[0] * xb[0] + xb[1] * xb[1] + xb[2] * xb[2];
        // (the square root and reciprocals in single precision, < 3e-7 relative each, with the bounds
        // widened as in seg_cert; the 1e-6 margin on m_a² kept whole: a certified step is still
        // provably one-signed)
        const double ba = (P.cm * (3.0 * xa[2] * xa[2] - ra2) + 3.0 * P.sm * xa[0] * xa[2]) * (double)__builtin_amdgcn_rcpf((float)ra2);
        const double bb = (P.cm * (3.0 * xb[2] * xb[2] - rb2) + 3.0 * P.sm * xb[0] * xb[2]) * (double)__builtin_amdgcn_rcpf((float)rb2);
        const double irmin = (double)__builtin_amdgcn_rcpf((float)rmin);
        const double al = (s1 - s0) * irmin;
        const double db = 0.75 * al * al * (1.0 + 2e-6) + 1e-12;
        if (c_prev < 0.0) {
          const double bmax = fmin(2.0, fmax(fabs(ba), fabs(bb)) * (1.0 + 1e-6) + db);
          cert = cert_lhs * 0.5 * bmax < cert_rhs * (rm2 * rmin) * (1.0 - 2e-6);
        } else if (rmin > 10.0 * (1.0 + 1e-6)) {
          const double bmin = (ba * bb > 0.0) ? fmin(fabs(ba), fabs(bb)) * (1.0 - 1e-6) - db : -1.0;
          const double rmax2 = fmax(ra2, rb2);
          const double grr = 1.0 - P.rs_gr * irmin * (1.0 + 1e-6);  // (rounded down: a smaller g^rr)
          cert = bmin > 0.0 && P.wp2n * bmin * grr > E * E * (1.0 + 1e-6) * (rmax2 * sqrt(rmax2));
        }
      }
      const bool unc = active && !cert;
      // A step wholly inside the star (both ends below rNS, so the whole segment is) holds no
      // crossing affect! keeps (rr > rNS, :1585-1597): its brackets would all be resolved and
      // dropped, so none is queued, and only its last point is evaluated -- the value the next
      // step's first bracket starts from. (~40% of the flat workload's uncertified steps.)
      bool inner = false;
      if (unc && cert_ok) {
        const double X0[3] = {Lx[0], Lx[256], Lx[2 * 256]}, VA[3] = {Lx[3 * 256], Lx[4 * 256], Lx[5 * 256]};
        double xa[3], xb[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) { xa[i] = X0[i] + VA[i] * s0; xb[i] = X0[i] + VA[i] * s1; }
        inner = fmax(xa[0] * xa[0] + xa[1] * xa[1] + xa[2] * xa[2], xb[0] * xb[0] + xb[1] * xb[1] + xb[2] * xb[2]) < r_in2;
      }
      const unsigned long long mU = __ballot(unc && !inner), mI = __ballot(inner);
      const int nU = __popcll(mU), nI = __popcll(mI);
      ART_QMARK(2)
      if (nU + nI == 0) {  // all certified: no point, no bracket, c_prev unchanged
        ++st;
        continue;
      }
#ifdef ART_SAMPLER_SECTIONS
      q_sec[6] += 1;
#endif
      // this lane's rank among the uncertified ones (the inner steps' lanes after the others)
      const int uix = inner ? nU + __popcll(mI & lt) : __popcll(mU & lt);
      if (unc) ssrc[wb + uix] = (unsigned char)lane;
      // bit j: signbit / nonzero-ness of point j (bit 0: the step start)
      unsigned sb = signbit(c_prev) ? 1u : 0u, nz = (c_prev != 0.0) ? 1u : 0u;
      wave_lds_sync();
      // items: (uncertified lane u, point j = 1..nper) lane-major, t = u nper + j - 1. A certified
      // step needs no point at all: its last point -- the next step's bracket start -- has the
      // certified sign, and c_prev is only ever read for its sign (the next certificate, the
      // bit-0 sign and nonzero-ness of the next scan), so it keeps the value it had. Each pass's
      // signs come back as two ballots, from which every owner takes the run of its own items'
      // bits (round 4: until then point-major items ORed their bits into LDS words with two LDS
      // atomics each, ~13 lanes deep on one word, and divided by the variable nU: 3.3 LDS
      // bank-conflict cycles per LDS instruction. Samples bit-identical, time unchanged: the
      // kernel is VALU-bound, profiles/r04aq_sampler_pmc.txt).
      // items: the other lanes' 19 points each, then the inner lanes' last points
      const int totN = nU * nper, tot = totN + nI;
      __builtin_amdgcn_s_setprio(0);  // brackets: short dependent chains) at the high one: 118.5 -> 117.1 ms
      #pragma unroll 1
      for (int w0 = 0; w0 < tot; w0 += 64) {
        const int t = w0 + lane;
        bool neg = false, nonz = false;
        if (t < tot) {
          int src, j;
          if (t < totN) {
            const int u = t / nper;
            j = t - u * nper + 1;
            src = ssrc[wb + u];
          } else {
            j = nper;
            src = ssrc[wb + nU + (t - totN)];
          }
          const double* S = sline + wb + src;
          // (s1 - s0) j / 19: from the table for a full 0.5 km step (wave-uniform), else divided
          const double sc = s0 + (s1 - s0 == 0.5 ? sgrid[j] : (s1 - s0) * double(j) / double(np - 1));
          double xl[3];
#pragma unroll
          for (int i = 0; i < 3; ++i) xl[i] = S[i * 256] + S[(3 + i) * 256] * sc;
          const double VL[3] = {S[6 * 256], S[7 * 256], S[8 * 256]};
          // the point's sign without the condition where it is decided (sampler_sign_fast), else the
          // condition itself; a decided point carries ±1 (only its sign and nonzero-ness are read)
          const int fs = cert_ok ? sampler_sign_fast(P, xl, VL, P.mass_a2 * S[10 * 256], r_lim2) : 0;
          double v = fs == 1 ? -1.0 : 1.0;
          if (fs == 0) v = sampler_condition_e(P, xl, VL, S[9 * 256], S[10 * 256]);
          if (j == nper) slast[wb + src] = v;
          neg = signbit(v);
          nonz = v != 0.0;
        }
        const unsigned long long mneg = __ballot(neg), mnz = __ballot(nonz);
        if (unc && !inner) {
          const int a = uix * nper;
          const int lo = max(a, w0), hi = min(a + nper, w0 + 64);
          if (lo < hi) {
            const unsigned long long run = (1ull << (hi - lo)) - 1ull;
            const int at = lo - a + 1;
            sb |= (unsigned)((mneg >> (lo - w0)) & run) << at;
            nz |= (unsigned)((mnz >> (lo - w0)) & run) << at;
          }
        }
      }
      __builtin_amdgcn_s_setprio(1);
      wave_lds_sync();
      // this lane's sign changes in (point j-1, point j]: signbits differ, both values nonzero
      unsigned br = 0u;
      if (unc) {
        if (!inner) br = (sb ^ (sb << 1)) & nz & (nz << 1) & (((1u << np) - 1u) & ~1u);
        c_prev = slast[threadIdx.x];
      }
      ART_QMARK(3)
      if (__ballot(br != 0u) == 0ull) {
        ++st;
        continue;
      }
      sbm[threadIdx.x] = br;
      }
      // the previous step's last grid point, where a bracket at point 1 opens
      const double ps0 = (st - 1) * 0.5;
      const double pds = fmin(ps0 + 0.5, send) - ps0;
      const double s_start = st == 0 ? 0.0 : ps0 + (pds == 0.5 ? sgrid[nper] : pds * double(nper) / double(np - 1));
      // queue the brackets, each lane's in its order along the line
      unsigned br = sbm[threadIdx.x];
      unsigned long long bm = __ballot(br != 0u);
      sres = false;
      while (bm != 0ull) {
        if (qn + 64 > SQCAP) {  // (the rest wait in sbm; the loop's top resolves the queue)
          sres = true;
          sbm[threadIdx.x] = br;
          break;
        }
        if (br != 0u) {
          const int ip = __builtin_ctz(br);
          const int slot = qn + __popcll(bm & lt);
          sqa[wq + slot] = (ip == 1) ? s_start : s0 + (s1 - s0) * double(ip - 1) / double(np - 1);
          sqb[wq + slot] = s0 + (s1 - s0) * double(ip) / double(np - 1);
          sqsrc[wq + slot] = (unsigned char)lane;
          br &= br - 1u;
        }
        qn = __builtin_amdgcn_readfirstlane(qn + __popcll(bm));  // (wave-uniform)
        bm = __ballot(br != 0u);
      }
      ART_QMARK(4)
      if (!sres) ++st;
    }
    }
    if (qn > 0) flush();
    ART_QMARK(4)

    if (active) {
      const bool give_up = attempt + 1 >= 1000000u;  // bounded: no conversion surface reachable
      if (count >= randInx || give_up) {
        if (count < randInx) { xsel[0] = xsel[1] = xsel[2] = NAN; count = 0; }
        const double rmag = sqrt(xsel[0] * xsel[0] + xsel[1] * xsel[1] + xsel[2] * xsel[2]);
        const double vIl[3] = {Lx[11 * 256], Lx[12 * 256], Lx[13 * 256]};
        const double vmagl = sqrt(vIl[0] * vIl[0] + vIl[1] * vIl[1] + vIl[2] * vIl[2]);  // = vmag
        const double vml = sqrt(vmagl * vmagl + 2.0 * P.GM_c2 * C_KM * C_KM / rmag) / C_KM;  // :1644
        double vel[3], vc[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) { vel[i] = Lx[(6 + i) * 256] * vml; vc[i] = vIl[i] / C_KM; }
        // MainRunner.jl:514-529: erg_inf_ini from vIfty/c, k_init = k_norm_Cart(ax_fix = true)
        const double vm = sqrt(vc[0] * vc[0] + vc[1] * vc[1] + vc[2] * vc[2]);
        const double gA = 1.0 / sqrt(1.0 - vm * vm);
        const double Ei = P.mass_a * sqrt(1.0 + (vm * gA) * (vm * gA));
        double kn[3];
        k_norm_axion_shell(P, xsel, vel, Ei, kn);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          xo[c * n + ray] = xsel[c];
          ko[c * n + ray] = kn[c];
          vifo[c * n + ray] = vc[c];
        }
        ergo[ray] = Ei;
        wo[ray] = count;
        ao[ray] = (int32_t)(attempt + 1);
        ray = -1;
      } else {
        ++attempt;
      }
    }
    ART_QMARK(5)
  }
#ifdef ART_SAMPLER_SECTIONS
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(queue + 8 + k, q_sec[k]);
#endif
}

#ifdef ART_NOLICM_TU
// the sampler's builds, compiled here without MachineLICM (art_kernels_nolicm.hip)
SFn nl_sample(int wps, bool blocks) {
  return wps == 3 ? (blocks ? sample_kernel<3, true> : sample_kernel<3, false>)
                  : (blocks ? sample_kernel<2, true> : sample_kernel<2, false>);
}
#endif  // ART_NOLICM_TU

#ifndef ART_NOLICM_TU
// ---------------------------------------------------------------------------
// get_Prob_nonAD over groups; one thread per group (groups are one segment's crossings).
__global__ __launch_bounds__(256) void prob_kernel(const KParams P, const int64_t nc, const double* __restrict__ pos,
                                                   const double* __restrict__ kpos, const double* __restrict__ erg,
                                                   const int64_t n_groups, const int64_t* __restrict__ gstart,
                                                   double* __restrict__ outp) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const int64_t a = gstart ? gstart[g] : g;
  const int64_t b = gstart ? gstart[g + 1] : g + 1;
  const int64_t m = b - a;
  if (m <= 0) return;
  // linear-indexed group values (column-major m x 3): index q -> row q % m, col q / m
  double ks_lin[3], B_lin[3], x0pl_lin[2];
  for (int q = 0; q < 3; ++q) {
    const int64_t row = q % m, col = q / m;
    const double p3[3] = {pos[a + row], pos[nc + a + row], pos[2 * nc + a + row]};
    const double k3[3] = {kpos[a + row], kpos[nc + a + row], kpos[2 * nc + a + row]};
    const ProbLocal<double> Lq = prob_local(P, p3, k3, erg[a + row]);
    ks_lin[q] = Lq.ks[col];
    B_lin[q] = Lq.B[col];
    if (q < 2) {
      const double sph[3] = {Lq.r, Lq.th, Lq.ph};
      x0pl_lin[q] = sph[col];
    }
  }
  ProbLin<double> G;
  G.k1 = ks_lin[0]; G.k2 = ks_lin[1]; G.k3 = ks_lin[2];
  G.B1 = B_lin[0]; G.B2 = B_lin[1]; G.B3 = B_lin[2];
  G.r_c = x0pl_lin[0]; G.th_c = x0pl_lin[1];
  for (int64_t i = a; i < b; ++i) {
    const double p3[3] = {pos[i], pos[nc + i], pos[2 * nc + i]};
    const double k3[3] = {kpos[i], kpos[nc + i], kpos[2 * nc + i]};
    const ProbLocal<double> L = prob_local(P, p3, k3, erg[i]);
    outp[i] = prob_eval(P, P.g_agg, L, G);
  }
}


// ---------------------------------------------------------------------------
// Binned flux (plot/flux.py:38-48): φf = atan2(k_y, k_x) of final particles, per species.
__global__ __launch_bounds__(256) void flux_kernel(const KParams P, const int64_t n, const double* __restrict__ x_end,
                                                   const double* __restrict__ k_end, const int32_t* __restrict__ status,
                                                   const int8_t* __restrict__ species, const double* __restrict__ w,
                                                   const int32_t nbins, double* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x) sh[i] = 0.0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x[3] = {x_end[i], x_end[n + i], x_end[2 * n + i]}, k[3] = {k_end[i], k_end[n + i], k_end[2 * n + i]};
    const int bin = flux_bin_of(P, x, k, status[i], nbins);
    if (bin < 0) continue;
    const int row = (species && species[i] == ART_AXION) ? 0 : 1;
    atomicAdd(&sh[row * nbins + bin], w ? w[i] : 1.0);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x)
    if (sh[i] != 0.0) atomicAdd(&hist[i], sh[i]);
}

// Binned flux of npy rows (plot/flux.py:38-48): histogram of the given φf with weights w.
__global__ __launch_bounds__(256) void flux_phi_kernel(const int64_t n, const double* __restrict__ phi,
                                                       const int8_t* __restrict__ species,
                                                       const double* __restrict__ w, const int32_t nbins,
                                                       const double lo, const double hi,
                                                       double* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x) sh[i] = 0.0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int bin = np_hist_bin(phi[i], nbins, lo, hi);
    if (bin < 0) continue;
    const int row = (species && species[i] == ART_AXION) ? 0 : 1;
    atomicAdd(&sh[row * nbins + bin], w ? w[i] : 1.0);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x)
    if (sh[i] != 0.0) atomicAdd(&hist[i], sh[i]);
}

// ---------------------------------------------------------------------------
// Pointwise physics for parity tests.
__global__ void eval_rhs_kernel(const KParams P, const int64_t n, const double* __restrict__ u,
                                const double* __restrict__ tau, const double* __restrict__ erg,
                                const int8_t* __restrict__ species, double* __restrict__ du) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double ui[7], d[7];
  for (int c = 0; c < 7; ++c) ui[c] = u[c * n + i];
  rhs(P, species[i] != ART_AXION, ui, tau[i], erg[i], d);
  for (int c = 0; c < 7; ++c) du[c * n + i] = d[c];
}

__global__ void eval_hamiltonian_kernel(const KParams P, const int64_t n, const double* __restrict__ x,
                                        const double* __restrict__ k, const double* __restrict__ Tm,
                                        const double* __restrict__ E, double* __restrict__ H,
                                        double* __restrict__ dHdx, double* __restrict__ dHdk,
                                        double* __restrict__ dHdT) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double xi[3] = {x[i], x[n + i], x[2 * n + i]};
  const double ki[3] = {k[i], k[n + i], k[2 * n + i]};
  double h, gx[3], gk[3], gT;
  hamiltonian_full(P, xi, ki, Tm[i], E[i], &h, gx, gk, &gT);
  H[i] = h;
  dHdT[i] = gT;
  for (int c = 0; c < 3; ++c) {
    dHdx[c * n + i] = gx[c];
    dHdk[c * n + i] = gk[c];
  }
}

__global__ void eval_condition_kernel(const KParams P, const int64_t n, const double* __restrict__ u,
                                      const double* __restrict__ tau, double* __restrict__ outc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double ui[7];
  for (int c = 0; c < 7; ++c) ui[c] = u[c * n + i];
  outc[i] = condition(P, ui, tau[i]);
}

// Event weight of every sampled point (MainRunner.jl:498-557, art_event.h); out: 5n SoA.
__global__ __launch_bounds__(256) void event_weight_kernel(const KParams P, const int64_t n, const double* __restrict__ x,
                                                           const double* __restrict__ k, const double* __restrict__ v,
                                                           const double maxR, const double rho, const double mcmc,
                                                           double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double xi[3] = {x[i], x[n + i], x[2 * n + i]};
  const double ki[3] = {k[i], k[n + i], k[2 * n + i]};
  const double vi[3] = {v[i], v[n + i], v[2 * n + i]};
  const EventW E = event_weight(P, xi, ki, vi, maxR, rho, mcmc);
  out[i] = E.cos_w;
  out[n + i] = E.jacobian_GR;
  out[2 * n + i] = E.sln_prob;
  out[3 * n + i] = E.erg_inf_ini;
  out[4 * n + i] = E.vel_eng;
}

// ---------------------------------------------------------------------------
// host-side launch wrappers (art_internal.h)
// Resident blocks of `func` per CU from its own resource use: the unified 512-entry VGPR file
// of a CDNA SIMD (arch VGPRs + AGPRs, granule 8), 8 waves per SIMD at most, and the 160 KB of
// LDS per CU.
static int blocks_per_cu_from_attributes(const void* func, int block, int fallback) {
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, func) != hipSuccess) {
    (void)hipGetLastError();
    return fallback;
  }
  const int regs = a.numRegs > 0 ? ((a.numRegs + 7) / 8) * 8 : 8;
  int wps = 512 / regs;
  wps = wps > 8 ? 8 : wps;
  const int waves = (block + 63) / 64;
  int per_cu = (4 * wps) / waves;
  if (a.sharedSizeBytes > 0) {
    const int by_lds = (int)(163840 / a.sharedSizeBytes);
    per_cu = per_cu < by_lds ? per_cu : by_lds;
  }
  return per_cu < 1 ? 1 : per_cu;
}

int persistent_blocks(const void* func, int64_t work, int block, int fallback_per_cu) {
  int dev = 0, ncu = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, func, block, 0);
  if (oe != hipSuccess || per_cu < 1) {
    // The runtime's occupancy calculator returns hipErrorUnknown (and 0 blocks) for the
    // 1-wave/SIMD flat integrator (270 unified VGPRs: 256 arch + 14 AGPRs), a kernel that
    // launches and runs correctly. That error stays the thread's last error, and the
    // hipGetLastError() after the next launch then reported the launch as failed (round 2's
    // "unknown error" on a 2000-ray flat batch, profiles/r03a_w1_launch_debug.txt). Clear it
    // and size the grid from the kernel's own resource use instead.
    (void)hipGetLastError();
    per_cu = blocks_per_cu_from_attributes(func, block, fallback_per_cu);
  }
  const int64_t need = (work + block - 1) / block;
  const int64_t full = (int64_t)ncu * per_cu;
  return (int)(need < full ? need : full);
}


// flat's instantiations live here; every other one comes from art_kernels_nolicm.hip (nl_propagate)
template <int DON>
static KFn pick_propagate(bool save, bool rk4, bool flat, bool sch) {
  if (save)  // saveat requested: the saving instantiations
    return (!rk4 && flat) ? propagate_kernel<ART_VERN6, GEOM_FLAT, true, DON>
                          : nl_propagate(rk4 ? ART_RK4 : ART_VERN6, (!rk4 && sch) ? GEOM_GR : GEOM_ANY, true, DON,
                                         ART_WAVES_PER_SIMD);
  if (flat) return rk4 ? propagate_kernel<ART_RK4, GEOM_FLAT, false, DON> : propagate_kernel<ART_VERN6, GEOM_FLAT, false, DON>;
  return nl_propagate(rk4 ? ART_RK4 : ART_VERN6, (!rk4 && sch) ? GEOM_GR : GEOM_ANY, false, DON, ART_WAVES_PER_SIMD);
}

int64_t small_tail_limit() {
  const char* e = std::getenv("ART_SMALL_TAIL");  // read per launch (tests switch it)
  if (e && *e) return std::atoll(e);
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return (int64_t)ncu * 4;
}

// The one-wave-per-ray tail kernel for donated rays: ART_TAIL=0 off, ART_TAIL=k at most k rays
// (default 1: one per SIMD of the device).
static int tail_rays() {
  const char* e = std::getenv("ART_TAIL");  // read per launch (tests switch it)
  return (e && *e) ? std::atoi(e) : 1;
}

// lanes a drained wave of the packed continuation hands to the tail kernel (ART_TAIL_DONATE)
static int tail_donate() {
  const char* e = std::getenv("ART_TAIL_DONATE");
  const int v = (e && *e) ? std::atoi(e) : 4;
  return v < 1 ? 1 : (v > 63 ? 63 : v);
}

// The 1-wave/SIMD instantiations (small batches, GR continuations) are on unless ART_W1=0.
static bool w1_builds() {
  static const bool on = [] {
    const char* e = std::getenv("ART_W1");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The claim order (SegOut::order): 32-bit keys of the rays' initial step sizes (positive floats sort
// as their bits), the ray ids beside them, one stable radix sort.
__global__ void order_keys_kernel(int64_t n, const double* __restrict__ u0, unsigned* __restrict__ keys,
                                  int32_t* __restrict__ ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    keys[i] = __float_as_uint((float)u0[i * U0_REC + 14]);
    ids[i] = (int32_t)i;
  }
}
struct OrderLayout {
  size_t keys_in, keys_out, ids_in, ids_out, tmp, tmp_bytes, total;
};
static OrderLayout order_layout(int64_t n) {
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  OrderLayout L{};
  size_t tb = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const unsigned*)nullptr, (unsigned*)nullptr,
                                           (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  const size_t k = al((size_t)n * 4);
  L.keys_in = 0;
  L.keys_out = k;
  L.ids_in = 2 * k;
  L.ids_out = 3 * k;
  L.tmp = 4 * k;
  L.tmp_bytes = tb;
  L.total = 4 * k + al(tb);
  return L;
}
size_t claim_order_bytes(int64_t n) { return n > 0 && n < INT32_MAX ? order_layout(n).total : 0; }

// Raises a launch's *hot_done once the kernels that write hot records have ended (stream order).
__global__ void hot_done_kernel(unsigned* w) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

hipError_t launch_propagate(const KParams& P, int64_t n, const SegIn& in, const SegOut& out_arg, int32_t max_crossings,
                            unsigned long long* queue, unsigned long long* stats, hipStream_t s, int* grid_out,
                            hipEvent_t ev0, hipEvent_t ev1, hipStream_t fs, const HotSide& hs) {
  const int64_t gr = (n + 255) / 256;
  const unsigned g1 = (unsigned)((n + 255) / 256);
#define ART_DBG(stage)
  hipLaunchKernelGGL(pick_helper(P), dim3((unsigned)(gr < 2048 ? gr : 2048)), dim3(256), 0, s, P, n, in, out_arg, (int)HK_INIT,
                     (int64_t)0, n, (int64_t)-1, 0, stats);
  ART_DBG("helper_kernel (init)")
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const bool flat = P.rs_eff == 0.0 && !(P.bndry_lyr > 0.0) && !P.isotropic;
  const bool sch = P.rs_eff > 0.0 && !(P.bndry_lyr > 0.0) && !P.isotropic;
  const bool rk4 = P.integrator == ART_RK4;
  // graduation (SegOut::grad) only where the tail kernel runs after the continuation to resume
  // the graduated rays
  SegOut out = out_arg;
  if (out.small_tail || !(out.donate > 0 && tail_rays() != 0 && !rk4 && out.ntimes < 2 && out.cont2)) {
    out.grad = nullptr;
    out.graduate = 0;
  }
  // early graduation (SegOut::hot): only with graduation, and with the side stream that the hot
  // rays' tail launch runs on beside the bulk pass and the continuation
  const bool hot = out.graduate > 0 && out.hot && out.hot_ready && out.hot_done && out.hot_at > 0 &&
                   out.hot_cap > 0 &&
                   hs.stream && hs.fork && hs.join && hs.zero_word;
  if (!hot) {
    out.hot = nullptr;
    out.hot_at = 0;
  }
  out.order = nullptr;
  if (hot && out.order_tmp && !out.small_tail && n < INT32_MAX) {
    // the bulk pass claims the rays smallest initial step first (SegOut::order)
    const OrderLayout L = order_layout(n);
    char* b = (char*)out.order_tmp;
    hipLaunchKernelGGL(order_keys_kernel, dim3(g1), dim3(256), 0, s, n, in.u0, (unsigned*)(b + L.keys_in),
                       (int32_t*)(b + L.ids_in));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = L.tmp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(b + L.tmp, tb, (const unsigned*)(b + L.keys_in),
                                                (unsigned*)(b + L.keys_out), (const int32_t*)(b + L.ids_in),
                                                (int32_t*)(b + L.ids_out), (int)n, 0, 32, s)) != hipSuccess)
      return e;
    out.order = (const int32_t*)(b + L.ids_out);
  }
  if (out.small_tail) {  // a small Vern6 batch: every ray on a wave of its own (tail_kernel)
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    SegOut ot = out;
    ot.cont_count = out.cont_count;
    ot.cont_queue = out.cont_queue;
    hipLaunchKernelGGL(pack_fresh_kernel, dim3(g1), dim3(256), 0, s, n, in, ot, stats);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int waves = (int)(n < (int64_t)ncu * 4 ? n : (int64_t)ncu * 4);
    if (grid_out) *grid_out = waves;
    if (ev0 && (e = hipEventRecord(ev0, s)) != hipSuccess) return e;
    const TFn tfn = nl_tail(flat ? GEOM_FLAT : (sch ? GEOM_GR : GEOM_ANY));
    hipLaunchKernelGGL(tfn, dim3(waves), dim3(64), 0, s, P, n, in, ot, max_crossings, waves, stats);
    ART_DBG("tail_kernel (small batch)")
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev1 && (e = hipEventRecord(ev1, s)) != hipSuccess) return e;
    hipStream_t sf = s;
    if (fs && ev1 && fs != s) {
      if ((e = hipStreamWaitEvent(fs, ev1, 0)) != hipSuccess) return e;
      sf = fs;
    }
    hipLaunchKernelGGL(pick_helper(P), dim3(g1), dim3(256), 0, sf, P, n, in, out, (int)HK_FIN, (int64_t)0, n,
                       (int64_t)-1, 0, stats);
    return hipGetLastError();
  }
  KFn fn = out.donate > 0 ? pick_propagate<1>(out.ntimes >= 2, rk4, flat, sch)
                           : pick_propagate<0>(out.ntimes >= 2, rk4, flat, sch);
  // A batch that fits one ray per lane of 1 wave per SIMD runs the 1-wave/SIMD build, which
  // does not spill: lone GR tail ray -3%, flat -4.5% per attempt, bit-identical
  // (profiles/r02j_small_batch_w1_ab.txt, tests/test_edges.py). ART_W1=0 switches it off (A/B).
  bool w1 = false;
  if (w1_builds() && out.donate <= 0 && out.ntimes < 2 && !rk4 && (flat || sch)) {
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
#ifndef ART_W1_ALWAYS
    if (n <= (int64_t)ncu * 4 * 64) {
#else
    if (true) {  // (dev A/B build: the 1-wave/SIMD integrator for every batch, the occupancy sensitivity)
#endif
      fn = flat ? propagate_kernel<ART_VERN6, GEOM_FLAT, false, 0, 1> : nl_propagate(ART_VERN6, GEOM_GR, false, 0, 1);
      w1 = true;
    }
  }
  // (the integrator's blocks per CU by design: its waves per SIMD, 4 waves a block)
  int grid = persistent_blocks((const void*)fn, n, BLOCK, w1 ? 1 : ART_WAVES_PER_SIMD * 4 / (BLOCK / 64));
  ART_DBG("persistent_blocks")
  // the hot rays' launch: HOT_BLOCKS blocks of 4 waves, each beside one integrator block on a CU
  // (one wave of each per SIMD), so the bulk pass gives up that many of its blocks
  if (hot) grid = grid > 2 * HOT_BLOCKS ? grid - HOT_BLOCKS : grid;
  if (grid_out) *grid_out = grid;
  if (ev0 && (e = hipEventRecord(ev0, s)) != hipSuccess) return e;
  if (hot) {
    // on the side stream from the bulk pass's start: each wave resumes a hot record as soon as
    // one is written (one wave per ray, the tail kernel's arithmetic) and leaves once *hot_done is
    // raised after the continuation and none is left
    if ((e = hipEventRecord(hs.fork, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(hs.stream, hs.fork, 0)) != hipSuccess) return e;
    SegOut oh = out;
    oh.grad = nullptr;
    oh.graduate = 0;
    oh.hot_at = 0;
    oh.cont_count = hs.zero_word;  // (no drained-wave records: word 0 stays zero, word 1 is its queue)
    oh.cont_queue = hs.zero_word + 1;
    hipLaunchKernelGGL(nl_tail(flat ? GEOM_FLAT : (sch ? GEOM_GR : GEOM_ANY)), dim3(HOT_BLOCKS), dim3(256), 0,
                       hs.stream, P, n, in, oh, max_crossings, 4 * HOT_BLOCKS, stats);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipEventRecord(hs.join, hs.stream)) != hipSuccess) return e;
  }
  // (from here on every return raises *hot_done first, so the hot waves never wait past it)
  auto hot_done = [&](hipError_t err) {
    if (hot) {
      hipLaunchKernelGGL(hot_done_kernel, dim3(1), dim3(64), 0, s, out.hot_done);
      if (err == hipSuccess) err = hipGetLastError();
    }
    return err;
  };
  hipLaunchKernelGGL(fn, dim3(grid), dim3(BLOCK), 0, s, P, n, in, out, max_crossings, queue, stats);
  ART_DBG("propagate_kernel")
  if ((e = hipGetLastError()) != hipSuccess) return hot_done(e);
  if (out.donate > 0) {  // the donated tail rays, packed into full waves (at most waves x donate of them)
    // with the tail kernel (ART_TAIL != 0, Vern6 without saveat) the packed continuation donates
    // in its turn: its drained waves' last rays (at most ART_TAIL_DONATE each, default 4) go to
    // the second-level records, and tail_kernel resumes each of those on a wave of its own
    const bool tail = tail_rays() != 0 && !rk4 && out.ntimes < 2 && out.cont2;
    SegOut oc = out;  // (the continuation sends its lagging rays to the hot records too)
    oc.cont_mode = 1;
    oc.cont_src = out.cont;
    oc.cont_src_count = out.cont_count;
    oc.donate = tail ? tail_donate() : 0;
    oc.cont = out.cont2;
    oc.cont_count = out.cont2_count;
    const int64_t maxc = (int64_t)grid * (BLOCK / 64) * out.donate;
    const int cgrid = (int)((maxc + BLOCK - 1) / BLOCK);
    // GR continuations at 1 wave/SIMD: no spills (68 VGPRs spill to scratch at 2). A/B on the
    // configs[3] bench line: 3.21e8 -> 3.35e8 ray-steps/s, bit-identical
    // (profiles/r02h_continuation_w1_ab.txt); flat stays at 2 (measured -3.5% at 1).
    const KFn cfn = (w1_builds() && sch && !rk4 && out.ntimes < 2) ? nl_propagate(ART_VERN6, GEOM_GR, false, 1, 1) : fn;
    hipLaunchKernelGGL(cfn, dim3(cgrid), dim3(BLOCK), 0, s, P, n, in, oc, max_crossings, queue, stats);
    ART_DBG("continuation")
    if ((e = hipGetLastError()) != hipSuccess) return hot_done(e);
    if ((e = hot_done(hipSuccess)) != hipSuccess) return e;
    if (tail) {
      int dev = 0, ncu = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      // one wave per ray, at most one per SIMD of the device (ART_TAIL=k: k waves); more
      // second-level rays queue behind them
      const int64_t maxc2 = (int64_t)cgrid * (BLOCK / 64) * oc.donate + (out.grad ? (int64_t)out.grad_cap : 0);
      const int waves = tail_rays() == 1 ? ncu * 4 : tail_rays();
      const int tgrid = (int)(maxc2 < waves ? maxc2 : waves);
      SegOut ot = out;
      ot.cont = out.cont2;
      ot.cont_count = out.cont2_count;
      ot.cont_queue = out.cont2_queue;
      const TFn tfn = nl_tail(flat ? GEOM_FLAT : (sch ? GEOM_GR : GEOM_ANY));
      if (tgrid > 0) hipLaunchKernelGGL(tfn, dim3(tgrid), dim3(64), 0, s, P, n, in, ot, max_crossings, waves, stats);
      ART_DBG("tail_kernel")
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
  } else if ((e = hot_done(hipSuccess)) != hipSuccess) {
    return e;
  }
  if (hot && (e = hipStreamWaitEvent(s, hs.join, 0)) != hipSuccess) return e;
  if (ev1 && (e = hipEventRecord(ev1, s)) != hipSuccess) return e;
  hipStream_t sf = s;
  if (fs && ev1 && fs != s) {
    if ((e = hipStreamWaitEvent(fs, ev1, 0)) != hipSuccess) return e;
    sf = fs;
  }
  hipLaunchKernelGGL(pick_helper(P), dim3(g1), dim3(256), 0, sf, P, n, in, out, (int)HK_FIN, (int64_t)0, n, (int64_t)-1,
                     0, stats);
  ART_DBG("helper_kernel (finalize)")
  return hipGetLastError();
}

// The streamed pipeline's integrator: Vern6 (flat / GR / general geometry), no saveat, no
// donation, at most `blocks` persistent blocks (the block slots it leaves free run the init and
// finalize kernels of the pieces).
hipError_t launch_integrator_streamed(const KParams& P, int64_t n, const SegIn& in, const SegOut& out,
                                      int32_t max_crossings, unsigned long long* queue, unsigned long long* stats,
                                      int blocks, hipStream_t s, int* grid_out) {
  const bool flat = P.rs_eff == 0.0 && !(P.bndry_lyr > 0.0) && !P.isotropic;
  const bool sch = P.rs_eff > 0.0 && !(P.bndry_lyr > 0.0) && !P.isotropic;
  const KFn fn = flat ? propagate_kernel<ART_VERN6, GEOM_FLAT, false, 3>
                      : nl_propagate(ART_VERN6, sch ? GEOM_GR : GEOM_ANY, false, 3, ART_WAVES_PER_SIMD);
  const int64_t need = (n + BLOCK - 1) / BLOCK;
  const int grid = (int)(need < (int64_t)blocks ? need : (int64_t)blocks);
  if (grid_out) *grid_out = grid;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(BLOCK), 0, s, P, n, in, out, max_crossings, queue, stats);
  return hipGetLastError();
}

hipError_t launch_helpers(const KParams& P, int64_t n, const SegIn& in, const SegOut& out, int blocks, int64_t init_limit,
                          int announce, unsigned long long* stats, hipStream_t s) {
  hipLaunchKernelGGL(pick_helper(P), dim3((unsigned)blocks), dim3(256), 0, s, P, n, in, out, (int)HK_TILES, (int64_t)0, n,
                     init_limit, announce, stats);
  return hipGetLastError();
}

hipError_t launch_sample(const KParams& P, double maxR, uint64_t seed, int64_t ray_offset, int64_t n, double* x,
                         double* k, double* erg, double* vifty, int32_t* w, int32_t* att, unsigned long long* queue,
                         hipStream_t s, int waves) {
  // lines of up to 2.2 x 60 km (264 steps): the 3-wave build, step by step (blocks of steps: no
  // faster there, 118 vs 119 ms per 1e7 flat samples); longer lines, mostly certified far from the
  // conversion surface: 2 waves, blocks of 3 steps (the scan's largest-maxR point 55 -> 43 ms,
  // profiles/r05h_ab_sampler.txt). waves (art_set_sampler_waves) = 2 or 3 takes that build for every
  // line; ART_SAMPLER_WPS=2|3 and ART_SAMPLER_BLOCKS=0|1 force a build (A/B)
  int wps = waves == 2 || waves == 3 ? waves : (maxR <= 60.0 ? 3 : 2);
  bool blocks = maxR > 60.0;
  if (const char* e = std::getenv("ART_SAMPLER_WPS"))
    if (e[0] == '2' || e[0] == '3') wps = e[0] - '0';
  if (const char* e = std::getenv("ART_SAMPLER_BLOCKS"))
    if (e[0] == '0' || e[0] == '1') blocks = e[0] == '1';

  const SFn fn = nl_sample(wps, blocks);
  const int grid = persistent_blocks((const void*)fn, n, 256, 1);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, s, P, maxR, seed, ray_offset, n, x, k, erg, vifty, w, att, queue);
  return hipGetLastError();
}

hipError_t launch_prob(const KParams& P, int64_t nc, const double* pos, const double* kpos, const double* erg,
                       int64_t n_groups, const int64_t* gstart, double* out, hipStream_t s) {
  const int64_t grid = (n_groups + 255) / 256;
  hipLaunchKernelGGL(prob_kernel, dim3((unsigned)grid), dim3(256), 0, s, P, nc, pos, kpos, erg, n_groups, gstart, out);
  return hipGetLastError();
}

hipError_t launch_flux(const KParams& P, int64_t n, const double* x_end, const double* k_end, const int32_t* status,
                       const int8_t* species, const double* w, int32_t nbins, double* hist, hipStream_t s) {
  int64_t grid = (n + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(flux_kernel, dim3((unsigned)grid), dim3(256), 2 * nbins * sizeof(double), s, P, n, x_end, k_end,
                     status, species, w, nbins, hist);
  return hipGetLastError();
}

hipError_t launch_flux_phi(int64_t n, const double* phi, const int8_t* species, const double* w, int32_t nbins,
                           double lo, double hi, double* hist, hipStream_t s) {
  int64_t grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(flux_phi_kernel, dim3((unsigned)grid), dim3(256), 2 * nbins * sizeof(double), s, n, phi, species, w,
                     nbins, lo, hi, hist);
  return hipGetLastError();
}

hipError_t launch_eval_rhs(const KParams& P, int64_t n, const double* u, const double* tau, const double* erg,
                           const int8_t* species, double* du, hipStream_t s) {
  hipLaunchKernelGGL(eval_rhs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, n, u, tau, erg, species, du);
  return hipGetLastError();
}

hipError_t launch_eval_hamiltonian(const KParams& P, int64_t n, const double* x, const double* k, const double* T,
                                   const double* E, double* H, double* dHdx, double* dHdk, double* dHdT,
                                   hipStream_t s) {
  hipLaunchKernelGGL(eval_hamiltonian_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, n, x, k, T, E, H,
                     dHdx, dHdk, dHdT);
  return hipGetLastError();
}

hipError_t launch_event_weight(const KParams& P, int64_t n, const double* x, const double* k, const double* v,
                               double maxR, double rho, double mcmc, double* out, hipStream_t s) {
  hipLaunchKernelGGL(event_weight_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, n, x, k, v, maxR, rho,
                     mcmc, out);
  return hipGetLastError();
}

hipError_t launch_eval_condition(const KParams& P, int64_t n, const double* u, const double* tau, double* out,
                                 hipStream_t s) {
  hipLaunchKernelGGL(eval_condition_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, n, u, tau, out);
  return hipGetLastError();
}

#endif  // ART_NOLICM_TU

}  // namespace art

