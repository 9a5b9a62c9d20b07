// capi_main.cpp -- TEST INFRASTRUCTURE ONLY: the host code of the C boundary
// (art_capi.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer, in a container
// without a GPU: the pure host entry points, every argument check, and the paths that
// reach the HIP runtime (which then reports that no device is present). The kernels'
// launch wrappers are replaced by stubs (launch_stubs.cpp). Prints "capi OK".
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/art.h"

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  art_params p{};
  p.theta_m = 0.2; p.omega_pul = 1.0; p.B0 = 1e14; p.rNS = 10.0; p.mass_ns = 1.0; p.mass_a = 1e-5;
  p.g_agg = 1e-12; p.bndry_lyr = -1.0; p.ln_t_end = 0.0; p.abstol = 1e-6; p.reltol = 1e-7; p.dtmin = 1e-13;
  p.maxiters = 100000; p.flat = 1; p.melrose = 1; p.integrator = ART_VERN6; p.n_fixed = 2000; p.interp_points = 50;
  CHECK(art_abi_version() == ART_ABI_VERSION);
  CHECK(art_last_error() != nullptr);
  const double mr = art_find_conversion_surface(&p);
  CHECK(mr > 25.0 && mr < 26.0);  // 25.167 km
  double c[9], A[81], b[9], bh[9];
  CHECK(art_vern6_tableau(c, A, b, bh) == ART_OK);
  double sb = 0.0;
  for (double v : b) sb += v;
  CHECK(std::fabs(sb - 1.0) < 1e-14);
  const int64_t n = 4;
  std::vector<double> x(3 * n, 20.0), k(3 * n, 1e-6), e(n, 1e-5), dw(n, -1.0), lt(n, -30.0), xe(3 * n), ke(3 * n),
      u7(n), tau(n);
  std::vector<int8_t> sp(n, ART_PHOTON);
  std::vector<int32_t> st(n), acc(n), rej(n);
  art_segment_out so{xe.data(), ke.data(), u7.data(), tau.data(), st.data(), acc.data(), rej.data()};
  CHECK(art_propagate_host(nullptr, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, &so,
                           nullptr) == ART_E_INVALID);
  art_params q = p;
  q.melrose = 0;
  CHECK(art_propagate_host(&q, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, &so, nullptr) ==
        ART_E_UNSUPPORTED);
  q = p; q.interp_points = 70;
  CHECK(art_propagate_host(&q, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, &so, nullptr) ==
        ART_E_INVALID);
  q = p; q.integrator = ART_RK4; q.n_fixed = 0;
  CHECK(art_propagate_host(&q, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, &so, nullptr) ==
        ART_E_INVALID);
  q = p; q.abstol = 0.0;
  CHECK(art_propagate_host(&q, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, &so, nullptr) ==
        ART_E_INVALID);
  CHECK(std::strlen(art_last_error()) > 0);
  CHECK(art_propagate_host(&p, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, -1, &so, nullptr) == ART_OK);
  CHECK(art_propagate_device(&p, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, nullptr,
                             nullptr, nullptr) == ART_E_INVALID);
  // reaches the HIP runtime: no device in this container
  int rc = art_propagate_host(&p, n, x.data(), k.data(), e.data(), dw.data(), lt.data(), sp.data(), -1, &so, nullptr);
  CHECK(rc == ART_E_HIP || rc == ART_E_NOMEM || rc == ART_OK);
  // get_Prob_nonAD groups must tile [0, nc)
  std::vector<double> out(n);
  int64_t bad[3] = {0, 3, 2};
  CHECK(art_get_prob_nonad_host(&p, n, x.data(), k.data(), e.data(), 2, bad, out.data()) == ART_E_INVALID);
  CHECK(art_get_prob_nonad_host(&p, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr) == ART_OK);
  // sampler / event weight / flux argument checks
  std::vector<int32_t> wi(n), ai(n);
  CHECK(art_sample_conversion_points_host(&p, 5.0, 1, 0, n, x.data(), k.data(), e.data(), x.data(), wi.data(),
                                          ai.data()) != ART_OK);
  CHECK(art_sample_conversion_points_host(&p, mr, 1, 0, -1, x.data(), k.data(), e.data(), x.data(), wi.data(),
                                          ai.data()) == ART_E_INVALID);
  CHECK(art_event_weight_host(&p, mr, 0.45, 6.0, 0, nullptr, nullptr, nullptr, nullptr) == ART_OK);
  CHECK(art_flux_histogram_device(&p, n, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr) ==
        ART_E_INVALID);
  CHECK(art_flux_histogram_phi_device(n, nullptr, nullptr, nullptr, 50, nullptr, nullptr) == ART_E_INVALID);
  CHECK(art_flux_histogram_phi_device(-1, nullptr, nullptr, nullptr, 50, nullptr, nullptr) == ART_E_INVALID);
  // the reduction: nothing to reduce without a communicator, bad ranks rejected
  double h[4] = {1, 2, 3, 4};
  CHECK(art_flux_allreduce(h, 4, nullptr) == ART_E_INVALID);
  CHECK(art_flux_allreduce_host(h, 4) == ART_E_INVALID);
  art_rccl_id id{};
  CHECK(art_comm_init(2, 2, &id) == ART_E_INVALID);
  CHECK(art_comm_init(0, 0, &id) == ART_E_INVALID);
  CHECK(art_comm_init(0, 1, nullptr) == ART_E_INVALID);
  CHECK(art_comm_destroy() == ART_OK);
  double ms[2];
  CHECK(art_recent_kernel_ms(-1, ms) != ART_OK);
  std::printf("capi OK\n");
  return 0;
}
