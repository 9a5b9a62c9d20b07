// TEST INFRASTRUCTURE ONLY -- never linked into the product library.
//
// Forward-mode dual numbers restating what ForwardDiff.jl does for the reference
// (RayTracer.jl:10 `using ForwardDiff: gradient, derivative, Dual`; the `seed`/`grad`
// helpers at RayTracer.jl:21,24). The oracle evaluates every reference gradient with
// these duals so that the product kernel's hand-derived gradients are checked against
// an independent, mechanically differentiated restatement.
#pragma once
#include <cmath>

namespace oracle {

template <int N>
struct Dual {
  double v;
  double d[N];
  Dual() : v(0.0) { for (int i = 0; i < N; ++i) d[i] = 0.0; }
  Dual(double x) : v(x) { for (int i = 0; i < N; ++i) d[i] = 0.0; }  // NOLINT: implicit like Julia promotion
  static Dual seed(double x, int k) { Dual r(x); r.d[k] = 1.0; return r; }
};

inline double val(double x) { return x; }
template <int N> inline double val(const Dual<N>& x) { return x.v; }

#define ORACLE_DUAL_BINOP(OP, VEXPR, DEXPR)                                                    \
  template <int N> inline Dual<N> operator OP(const Dual<N>& a, const Dual<N>& b) {          \
    Dual<N> r; r.v = VEXPR; for (int i = 0; i < N; ++i) r.d[i] = DEXPR; return r; }           \
  template <int N> inline Dual<N> operator OP(const Dual<N>& a, double bv) {                 \
    Dual<N> b(bv); return a OP b; }                                                            \
  template <int N> inline Dual<N> operator OP(double av, const Dual<N>& b) {                 \
    Dual<N> a(av); return a OP b; }

ORACLE_DUAL_BINOP(+, a.v + b.v, a.d[i] + b.d[i])
ORACLE_DUAL_BINOP(-, a.v - b.v, a.d[i] - b.d[i])
ORACLE_DUAL_BINOP(*, a.v * b.v, a.d[i] * b.v + a.v * b.d[i])
// ForwardDiff: d(a/b) = (da*b - a*db)/b^2, evaluated as da/b - (a/b)*db/b
ORACLE_DUAL_BINOP(/, a.v / b.v, (a.d[i] - (a.v / b.v) * b.d[i]) / b.v)
#undef ORACLE_DUAL_BINOP

template <int N> inline Dual<N> operator-(const Dual<N>& a) {
  Dual<N> r; r.v = -a.v; for (int i = 0; i < N; ++i) r.d[i] = -a.d[i]; return r;
}

template <int N> inline Dual<N> chain(const Dual<N>& a, double fv, double dfdx) {
  Dual<N> r; r.v = fv; for (int i = 0; i < N; ++i) r.d[i] = dfdx * a.d[i]; return r;
}

template <int N> inline Dual<N> sqrt(const Dual<N>& a) { double s = std::sqrt(a.v); return chain(a, s, 0.5 / s); }
template <int N> inline Dual<N> sin(const Dual<N>& a) { return chain(a, std::sin(a.v), std::cos(a.v)); }
template <int N> inline Dual<N> cos(const Dual<N>& a) { return chain(a, std::cos(a.v), -std::sin(a.v)); }
template <int N> inline Dual<N> exp(const Dual<N>& a) { double e = std::exp(a.v); return chain(a, e, e); }
template <int N> inline Dual<N> acos(const Dual<N>& a) {
  return chain(a, std::acos(a.v), -1.0 / std::sqrt(1.0 - a.v * a.v));
}
// ForwardDiff's abs: flips the whole dual when the sign bit of the value is set.
template <int N> inline Dual<N> abs(const Dual<N>& a) { return std::signbit(a.v) ? -a : a; }
template <int N> inline Dual<N> pow(const Dual<N>& a, double p) {
  double f = std::pow(a.v, p); return chain(a, f, p * std::pow(a.v, p - 1.0));
}
template <int N> inline Dual<N> atan2(const Dual<N>& y, const Dual<N>& x) {
  Dual<N> r; double den = x.v * x.v + y.v * y.v; r.v = std::atan2(y.v, x.v);
  for (int i = 0; i < N; ++i) r.d[i] = (x.v * y.d[i] - y.v * x.d[i]) / den;
  return r;
}

using std::abs; using std::sqrt; using std::sin; using std::cos; using std::exp;
using std::acos; using std::pow; using std::atan2;

// Julia's literal integer powers x^2, x^3 lower to repeated multiplication.
template <class T> inline T sq(const T& x) { return x * x; }
template <class T> inline T cube(const T& x) { return x * x * x; }

}  // namespace oracle
