// forest_main.cpp -- TEST INFRASTRUCTURE ONLY: drives the batched tree driver
// (art_forest.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer on the CPU, with the
// oracle standing in for the GPU segments (oracle_backend.cpp). Forward trees (full and
// Monte-Carlo), the backtrace, the saveMode 3 variant, determinism, capacity and argument
// errors. Prints "forest OK" on success.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/art.h"

extern "C" {
void oracle_sample(const art_params* P, double maxR, uint64_t seed, int64_t ray_offset, int64_t n, double* x,
                   double* k_init, double* erg_inf, double* vifty, int32_t* weights, int32_t* attempts,
                   int32_t nthreads);
double oracle_find_conversion_surface(const art_params* P);
}

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

static art_params params(double B0) {
  art_params p{};
  p.theta_m = 0.2; p.omega_pul = 1.0; p.B0 = B0; p.rNS = 10.0; p.mass_ns = 1.0; p.mass_a = 1e-5;
  p.g_agg = 1e-12; p.bndry_lyr = -1.0; p.ln_t_end = 0.0; p.abstol = 1e-6; p.reltol = 1e-7; p.dtmin = 1e-13;
  p.maxiters = 100000; p.flat = 1; p.isotropic = 0; p.melrose = 1; p.integrator = ART_VERN6; p.n_fixed = 2000;
  p.interp_points = 50;
  return p;
}

static int grow(const art_params& p, int64_t n, const std::vector<double>& x, const std::vector<double>& k,
                const std::vector<double>& erg, int8_t species, const art_tree_opts& o, std::vector<art_tree_node>& nodes,
                std::vector<int32_t>& counts, std::vector<int32_t>& infos, const art_tree_traj* tj = nullptr) {
  std::vector<int8_t> sp(n, species);
  int64_t nn = 0;
  nodes.assign((size_t)n * 60, art_tree_node{});
  counts.assign(n, 0);
  infos.assign(n, 0);
  int rc = tj ? art_grow_trees_traj(&p, n, x.data(), k.data(), erg.data(), sp.data(), &o, (int64_t)nodes.size(),
                                    nodes.data(), &nn, counts.data(), infos.data(), tj)
              : art_grow_trees(&p, n, x.data(), k.data(), erg.data(), sp.data(), &o, (int64_t)nodes.size(),
                               nodes.data(), &nn, counts.data(), infos.data());
  if (rc) return rc;
  nodes.resize(nn);
  return 0;
}

int main() {
  const int64_t n = 12;
  art_params p = params(1e14);
  const double maxr = oracle_find_conversion_surface(&p);
  std::vector<double> x(3 * n), k(3 * n), erg(n), vif(3 * n), mk(3 * n);
  std::vector<int32_t> w(n), att(n);
  oracle_sample(&p, maxr, 1769, 0, n, x.data(), k.data(), erg.data(), vif.data(), w.data(), att.data(), 1);
  for (int64_t i = 0; i < 3 * n; ++i) mk[i] = -k[i];
  std::vector<art_tree_node> a, b;
  std::vector<int32_t> ca, ia, cb, ib;
  for (int mc : {1000, 2}) {  // full tree, then Monte-Carlo after 2 nodes
    art_tree_opts o{5, mc, 50, -1, 64, 7, 1e-10, 1769};
    CHECK(grow(p, n, x, k, erg, ART_PHOTON, o, a, ca, ia) == 0);
    CHECK(grow(p, n, x, k, erg, ART_PHOTON, o, b, cb, ib) == 0);
    CHECK(a.size() == b.size() && a.size() >= (size_t)n);
    CHECK(std::memcmp(a.data(), b.data(), a.size() * sizeof(art_tree_node)) == 0);  // deterministic
    CHECK(ca == cb && ia == ib);
    for (const art_tree_node& e : a) CHECK(e.tree >= 0 && e.tree < n && std::isfinite(e.weight));
  }
  // backtrace: axion, -k, -B0, every crossing, root only
  art_params pb = params(-1e14);
  art_tree_opts ob{0, 5, 50, 100000, 256, 0, 1e-10, 1769};
  CHECK(grow(pb, n, x, mk, erg, ART_AXION, ob, a, ca, ia) == 0);
  CHECK((int64_t)a.size() == n);
  for (int64_t i = 0; i < n; ++i) CHECK(ca[i] == 1 && a[i].weight > 0.0 && a[i].weight <= 1.0);
  // saveMode 3: the saveNode data of every node
  {
    art_tree_opts o{5, 5, 50, -1, 64, 0, 1e-10, 1769};
    const int nt = 3, xcap = 4;
    const size_t cap = (size_t)n * 60;
    std::vector<double> traj(cap * nt * 3), times(cap * nt), xc(cap * xcap * 4);
    std::vector<int32_t> cnt(cap);
    art_tree_traj tj{nt, xcap, traj.data(), times.data(), cnt.data(), xc.data()};
    CHECK(grow(p, n, x, k, erg, ART_PHOTON, o, a, ca, ia, &tj) == 0);
    for (size_t q = 0; q < a.size(); ++q) CHECK(cnt[q] >= 2 && cnt[q] <= nt);
  }
  // too small a node buffer: ART_E_NOMEM and the count needed
  {
    art_tree_opts o{5, 1000, 50, -1, 64, 0, 1e-10, 1769};
    std::vector<int8_t> sp(n, ART_PHOTON);
    std::vector<art_tree_node> small(2);
    int64_t nn = 0;
    CHECK(art_grow_trees(&p, n, x.data(), k.data(), erg.data(), sp.data(), &o, 2, small.data(), &nn, nullptr, nullptr) ==
          ART_E_NOMEM);
    CHECK(nn > 2);
    CHECK(art_grow_trees(&p, -1, x.data(), k.data(), erg.data(), sp.data(), &o, 2, small.data(), &nn, nullptr,
                         nullptr) == ART_E_INVALID);
    CHECK(art_grow_trees(&p, n, nullptr, k.data(), erg.data(), sp.data(), &o, 2, small.data(), &nn, nullptr,
                         nullptr) == ART_E_INVALID);
    CHECK(art_grow_trees(&p, 0, nullptr, nullptr, nullptr, nullptr, &o, 0, nullptr, &nn, nullptr, nullptr) == ART_OK);
    CHECK(nn == 0);
  }
  std::printf("forest OK\n");
  return 0;
}
