// oracle_backend.cpp -- TEST INFRASTRUCTURE ONLY (sanitizer build, tools/asan/Makefile).
// CPU stand-ins for the three libart entry points the batched tree driver (art_forest.cpp)
// calls -- art_propagate_host, art_propagate_traj_host and art_get_prob_nonad_host -- built
// on the oracle restatement (oracle/art_oracle.cpp), so the driver's host C++ runs under
// AddressSanitizer / UndefinedBehaviorSanitizer in a container without a GPU. The saveat
// variant returns the start and the end point only.
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/art.h"

extern "C" {
void oracle_propagate(const art_params* P, int64_t n, const double* x0, const double* k0, const double* erg,
                      const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                      double* x_end, double* k_end, double* u7_end, double* tau_end, int32_t* status,
                      int32_t* n_accept, int32_t* n_reject, int32_t cap, int32_t* n_cross, double* xc_pos,
                      double* xc_k, double* xc_t, double* xc_dw, double* xc_p, int nthreads);
void oracle_get_prob_nonad(const art_params* P, int64_t nc, const double* pos, const double* kpos,
                           const double* erg_eff, int64_t n_groups, const int64_t* group_start, double* out);

int art_propagate_host(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                       const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                       art_segment_out* out, art_crossing_buf* xc) {
  if (!p || n < 0 || !out) return ART_E_INVALID;
  if (n == 0) return ART_OK;
  const int cap = (xc && xc->count) ? xc->capacity : 1;
  std::vector<int32_t> cnt(n);
  std::vector<double> pos(3 * (size_t)cap * n), k(3 * (size_t)cap * n), t((size_t)cap * n), dwc((size_t)cap * n),
      pc((size_t)cap * n);
  oracle_propagate(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out->x_end, out->k_end, out->u7_end,
                   out->tau_end, out->status, out->n_accept, out->n_reject, cap, cnt.data(), pos.data(), k.data(),
                   t.data(), dwc.data(), pc.data(), 1);
  if (xc && xc->count) {
    for (int64_t i = 0; i < n; ++i) xc->count[i] = cnt[i];
    for (size_t q = 0; q < pos.size(); ++q) { xc->pos[q] = pos[q]; xc->k[q] = k[q]; }
    for (size_t q = 0; q < t.size(); ++q) { xc->t[q] = t[q]; xc->dw[q] = dwc[q]; xc->p_nonad[q] = pc[q]; }
  }
  return ART_OK;
}

int art_propagate_traj_host(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                            const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                            art_segment_out* out, art_crossing_buf* xc, int32_t ntimes, double* traj, double* traj_t,
                            int32_t* traj_n) {
  if (ntimes < 2) return ART_E_INVALID;
  int rc = art_propagate_host(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc);
  if (rc) return rc;
  for (int64_t i = 0; i < n; ++i) {
    traj_n[i] = 2;
    for (int c = 0; c < 3; ++c) {
      traj[((int64_t)c * ntimes + 0) * n + i] = x0[c * n + i];
      traj[((int64_t)c * ntimes + 1) * n + i] = out->x_end[c * n + i];
    }
    traj_t[i] = ln_t0[i];
    traj_t[n + i] = out->tau_end[i];
  }
  return ART_OK;
}

int art_get_prob_nonad_host(const art_params* p, int64_t nc, const double* pos, const double* kpos,
                            const double* erg_eff, int64_t n_groups, const int64_t* group_start, double* out) {
  if (!p || nc < 0) return ART_E_INVALID;
  if (nc == 0) return ART_OK;
  oracle_get_prob_nonad(p, nc, pos, kpos, erg_eff, group_start ? n_groups : nc, group_start, out);
  return ART_OK;
}
}
