// TEST TOOL ONLY: host build of the product's physics header (art_core.h) so the CPU test
// suite can check the hand-derived analytic gradients against the oracle's dual numbers
// without a GPU. Never loaded by the product (adiabatic_raytracer_amd).
#include "../adiabatic_raytracer_amd/csrc/art_core.h"

using namespace art;

extern "C" {
void cc_rhs(const art_params* p, int species, const double* u, double tau, double erg, double* du) {
  KParams K = make_kparams(*p);
  rhs(K, species != ART_AXION, u, tau, erg, du);
}
double cc_condition(const art_params* p, const double* u, double tau) {
  KParams K = make_kparams(*p);
  return condition(K, u, tau);
}
void cc_hamiltonian(const art_params* p, const double* x, const double* k, double T, double E, double* H, double* gx,
                    double* gk, double* gT) {
  KParams K = make_kparams(*p);
  hamiltonian_full(K, x, k, T, E, H, gx, gk, gT);
}
void cc_initial_state(const art_params* p, const double* x0, const double* k0, double erg, double dw, double* u) {
  KParams K = make_kparams(*p);
  initial_state(K, x0, k0, erg, dw, u);
}
void cc_back_transform(const art_params* p, const double* u, double erg, double* x, double* k) {
  KParams K = make_kparams(*p);
  back_transform(K, u, erg, x, k);
}
double cc_prob_single(const art_params* p, const double* pos, const double* kpos, double erg) {
  KParams K = make_kparams(*p);
  return prob_nonad_single(K, pos, kpos, erg);
}
double cc_sampler_condition(const art_params* p, const double* x, const double* vl, double E) {
  KParams K = make_kparams(*p);
  return sampler_condition(K, x, vl, E);
}
// n points: the condition (sampler_condition) and sampler_sign_fast's verdict on each
void cc_sampler_signs(const art_params* p, int64_t n, const double* x, const double* vl, const double* E, double* cond,
                      int* sgn) {
  KParams K = make_kparams(*p);
  const double rl = (K.rNS > 10.0 ? K.rNS : 10.0) * (1.0 + 1e-9);
  for (int64_t i = 0; i < n; ++i) {
    cond[i] = sampler_condition(K, x + 3 * i, vl + 3 * i, E[i]);
    sgn[i] = sampler_sign_fast(K, x + 3 * i, vl + 3 * i, K.mass_a2 / (E[i] * E[i]), rl * rl);
  }
}
}

extern "C" {
void cc_attempt_uniforms(uint64_t seed, uint64_t ray, uint32_t attempt, double* U) { attempt_uniforms(seed, ray, attempt, U); }
void cc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  philox4x32_10(c, key[0], key[1]);
  for (int i = 0; i < 4; ++i) out[i] = c[i];
}
void cc_sincos(const double* x, int64_t n, double* s, double* c) {
  for (int64_t i = 0; i < n; ++i) msincos(x[i], s[i], c[i]);
}
// walk_codes_loop / walk_codes_bits (art_core.h); st = {ip, last_s, last_j, lc_ok} in/out.
// Returns found (0/1), or -1 when the bit-parallel form declines (a zero code).
int cc_walk(const unsigned* cw, int nper, int* st, int bits) {
  WalkState w{st[0], st[1], st[2], st[3] != 0};
  bool found = false;
  if (bits) {
    if (!walk_codes_bits(cw, nper, w, found)) return -1;
  } else {
    walk_codes_loop(cw, nper, w, found);
  }
  st[0] = w.ip; st[1] = w.last_s; st[2] = w.last_j; st[3] = w.lc_ok ? 1 : 0;
  return found ? 1 : 0;
}
void cc_exp_fma(const double* x, int64_t n, double* y) {
  for (int64_t i = 0; i < n; ++i) y[i] = exp_fma(x[i]);
}
void cc_log_fma(const double* x, int64_t n, double* y) {
  for (int64_t i = 0; i < n; ++i) y[i] = log_fma(x[i]);
}
void cc_metric_d(double r, double rs, double* out) {
  double gtt, grr, dgtt, dgrr;
  metric_tr_d(r, rs, gtt, grr, dgtt, dgrr);
  out[0] = gtt; out[1] = grr; out[2] = dgtt; out[3] = dgrr;
}
}

extern "C" {
// scan_certified_code (art_core.h) for one step (u0, f0) -> (u1, f1) over h from τ
// (two_sided: with b at the start point too, as the kernel has it after its first step)
int cc_certified_code(const art_params* p, const double* u0, const double* f0, const double* u1,
                          const double* f1, double h, double tau, int two_sided) {
  KParams K = make_kparams(*p);
  double du[7], aux[2], aux0[2];  // b and t at the end point, as the kernel takes them from its last RHS
  rhs_photon(K, u1, tau + h, 1.0, du, aux);
  rhs_photon(K, u0, tau, 1.0, du, aux0);
  return scan_certified_code(K, u0, f0, u1, f1, h, aux[0], aux[1], two_sided ? aux0[0] : NAN);
}
}
