// art_forest.cpp -- batched tree driver: get_tree (MainRunner.jl:126-352) for many trees at
// once. The reference grows one tree at a time, propagating one node per iteration
// (batchsize = 1, :139). Here every active tree pops its next node and all of them are
// propagated in ONE GPU launch per round, so a forest of N trees costs at most
// max_nodes + 1 launches instead of N x (max_nodes + 1) single-ray solves. Per tree, the
// reference's order and rules are kept exactly:
//   * the event stack is popped from the end after a stable sort by weight (:166, :348),
//     i.e. highest weight first;
//   * a segment stops at its first new crossing when splittings_cutoff <= 0 (forward
//     trees) and records every crossing otherwise (backtrace, :588);
//   * full-tree splitting while count <= MC_nodes, one Monte-Carlo branch after (:281-305),
//     the draw being Philox4x32-10 keyed by (seed, tree, count) instead of Julia's global
//     rand(Float64);
//   * the "rare fail" rule (|kc| > 1, :213-225), the merge of crossings closer than 1e-5
//     km (:227-245), and the stop rules and info codes 1-4 (:325-350), negative when the
//     tree went Monte-Carlo.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/art.h"
#include "art_core.h"

namespace {

struct Cross {
  double pos[3], k[3], t, dw, P;
};

struct Node {
  double x[3], k[3], t, dw;
  int species;
  double prob, weight, parent_weight, prob_conv, prob_conv0;
  // filled once propagated
  int status = -1, is_final = 0, n_cross = 0;
  double x_end[3] = {0, 0, 0}, k_end[3] = {0, 0, 0}, u7_end = 0.0, tau_end = 0.0;
  Cross first{};
  // saveMode 3 (saveNode): the saved points and every kept crossing of the segment
  std::vector<double> traj, times;
  std::vector<Cross> xcs;
};

struct Tree {
  std::vector<Node> events, done;
  int count = 0, count_main = 0, info = 1;
  double tot_prob = 0.0;
  double erg = 0.0;
  bool active = true;
};

double mc_uniform(uint64_t seed, uint64_t tree, uint32_t count) {
  uint32_t ctr[4] = {(uint32_t)tree, (uint32_t)(tree >> 32), count, 0x54524545u /* "TREE" */};
  art::philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
  return art::u01(ctr[0], ctr[1]);
}

Node make_child(const Cross& c, int species, double prob, double weight, double parent_weight, double prob_conv,
                double prob_conv0) {
  Node n{};
  for (int i = 0; i < 3; ++i) {
    n.x[i] = c.pos[i];
    n.k[i] = c.k[i];
  }
  n.t = c.t;
  n.dw = c.dw;
  n.species = species;
  n.prob = prob;
  n.weight = weight;
  n.parent_weight = parent_weight;
  n.prob_conv = prob_conv;
  n.prob_conv0 = prob_conv0;
  return n;
}

int grow_trees_impl(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                    const int8_t* species, const art_tree_opts* opts, int64_t node_capacity, art_tree_node* nodes,
                    int64_t* n_nodes, int32_t* counts, int32_t* infos, const art_tree_traj* tj) {
  if (!p || !opts || !n_nodes || n < 0) return ART_E_INVALID;
  if (tj && (tj->ntimes < 2 || tj->crossing_cap < 0 || !tj->traj || !tj->times || !tj->count ||
             (tj->crossing_cap > 0 && !tj->xc)))
    return ART_E_INVALID;
  const int nt = tj ? tj->ntimes : 0;
  *n_nodes = 0;
  if (n == 0) return ART_OK;
  if (!x0 || !k0 || !erg || !species) return ART_E_INVALID;
  const bool split_all = opts->splittings_cutoff > 0;
  const int cap = split_all ? std::max(1, opts->crossing_cap) : 1;
  const double dt0 = std::exp(-30.0);  // NumerPass[1] = ln_t_start = -30 (MainRunner.jl:410)
  const double rNS = p->rNS;

  // roots: RT.node(x, k, t = 0, Δω = -1, species, prob = 1, weight = 1, -1, -1, -1) with
  // first.prob = 1 - exp(-P_nonAD) at the root, erg_inf_ini |Δω| = erg (:132-137)
  std::vector<Tree> trees((size_t)n);
  {
    std::vector<double> pos(3 * n), kp(3 * n), ee(n), pn(n);
    for (int64_t i = 0; i < n; ++i) {
      for (int c = 0; c < 3; ++c) {
        pos[c * n + i] = x0[c * n + i];
        kp[c * n + i] = k0[c * n + i];
      }
      ee[i] = erg[i];
    }
    int rc = art_get_prob_nonad_host(p, n, pos.data(), kp.data(), ee.data(), n, nullptr, pn.data());
    if (rc) return rc;
    for (int64_t i = 0; i < n; ++i) {
      Node r{};
      for (int c = 0; c < 3; ++c) {
        r.x[c] = x0[c * n + i];
        r.k[c] = k0[c * n + i];
      }
      r.t = 0.0;
      r.dw = -1.0;
      r.species = species[i] == ART_AXION ? ART_AXION : ART_PHOTON;
      r.prob = 1.0 - std::exp(-pn[i]);
      r.weight = 1.0;
      r.parent_weight = -1.0;
      r.prob_conv = -1.0;
      r.prob_conv0 = -1.0;
      trees[i].erg = erg[i];
      trees[i].events.push_back(r);
    }
  }

  std::vector<int64_t> idx;
  std::vector<Node> cur;
  std::vector<double> bx, bk, be, bdw, blt, sx, sk, su7, stau, cpos, ck, ct, cdw, cpn;
  std::vector<int8_t> bsp;
  std::vector<int32_t> sst, sacc, srej, ccount, trn;
  std::vector<double> trx, trt;
  while (true) {
    idx.clear();
    cur.clear();
    for (int64_t i = 0; i < n; ++i) {
      Tree& T = trees[i];
      if (!T.active) continue;
      if (T.events.empty()) {
        T.active = false;
        continue;
      }
      T.count += 1;
      cur.push_back(T.events.back());
      T.events.pop_back();
      idx.push_back(i);
    }
    const int64_t m = (int64_t)idx.size();
    if (m == 0) break;
    // ---- one batched RT.propagate for the popped node of every active tree ----
    bx.assign(3 * m, 0.0); bk.assign(3 * m, 0.0); be.assign(m, 0.0); bdw.assign(m, 0.0); blt.assign(m, 0.0);
    bsp.assign(m, 0);
    for (int64_t j = 0; j < m; ++j) {
      const Node& e = cur[j];
      for (int c = 0; c < 3; ++c) {
        bx[c * m + j] = e.x[c];
        bk[c * m + j] = e.k[c];
      }
      be[j] = trees[idx[j]].erg;
      bdw[j] = e.dw;                            // event.Δω[end]
      blt[j] = std::log(std::max(e.t, dt0));    // NumerPass[1] = log(max(event.t, dt0)) (:164)
      bsp[j] = (int8_t)e.species;
    }
    sx.assign(3 * m, 0.0); sk.assign(3 * m, 0.0); su7.assign(m, 0.0); stau.assign(m, 0.0);
    sst.assign(m, 0); sacc.assign(m, 0); srej.assign(m, 0);
    ccount.assign(m, 0); cpos.assign(3 * cap * m, 0.0); ck.assign(3 * cap * m, 0.0);
    ct.assign(cap * m, 0.0); cdw.assign(cap * m, 0.0); cpn.assign(cap * m, 0.0);
    art_segment_out so{sx.data(), sk.data(), su7.data(), stau.data(), sst.data(), sacc.data(), srej.data()};
    art_crossing_buf xb{cap, ccount.data(), cpos.data(), ck.data(), ct.data(), cdw.data(), cpn.data()};
    int rc;
    if (nt) {
      trx.assign(3 * (size_t)nt * m, 0.0); trt.assign((size_t)nt * m, 0.0); trn.assign(m, 0);
      rc = art_propagate_traj_host(p, m, bx.data(), bk.data(), be.data(), bdw.data(), blt.data(), bsp.data(),
                                   opts->splittings_cutoff, &so, &xb, nt, trx.data(), trt.data(), trn.data());
    } else {
      rc = art_propagate_host(p, m, bx.data(), bk.data(), be.data(), bdw.data(), blt.data(), bsp.data(),
                              opts->splittings_cutoff, &so, &xb);
    }
    if (rc) return rc;

    // ---- crossings of each segment: merge near-duplicates, probabilities ----
    std::vector<std::vector<Cross>> xcs((size_t)m);
    std::vector<char> rare((size_t)m, 0);  // the "rare fail" |kc| > 1 (:213-225), before the merge (:227)
    std::vector<int64_t> gstart(1, 0);
    std::vector<double> gpos, gk, ge;
    for (int64_t j = 0; j < m; ++j) {
      const int nc = std::min(ccount[j], cap);
      std::vector<Cross>& L = xcs[j];
      for (int q = 0; q < nc; ++q) {
        Cross c{};
        for (int a = 0; a < 3; ++a) {
          c.pos[a] = cpos[((int64_t)a * cap + q) * m + j];
          c.k[a] = ck[((int64_t)a * cap + q) * m + j];
        }
        c.t = ct[(int64_t)q * m + j];
        c.dw = cdw[(int64_t)q * m + j];
        c.P = 1.0 - std::exp(-cpn[(int64_t)q * m + j]);  // Nc = 1 semantics (forward trees)
        L.push_back(c);
        for (int a = 0; a < 3; ++a) rare[j] = rare[j] || std::abs(c.k[a]) > 1.0;
      }
      if (L.size() > 1) {  // two crossings at the same point are one (:227-245)
        std::vector<Cross> keep;
        for (size_t q = 0; q < L.size(); ++q) {
          bool k = true;
          if (q + 1 < L.size()) {
            const double d = std::sqrt(std::pow(std::abs(L[q + 1].pos[0] - L[q].pos[0]), 2) +
                                       std::pow(std::abs(L[q + 1].pos[1] - L[q].pos[1]), 2) +
                                       std::pow(std::abs(L[q + 1].pos[2] - L[q].pos[2]), 2));
            k = d > 1e-5;
          }
          if (k) keep.push_back(L[q]);
        }
        L.swap(keep);
      }
      if (L.size() > 1) {  // one get_Prob_nonAD call with Nc > 1: the reference's indexing (:265)
        for (const Cross& c : L) {
          for (int a = 0; a < 3; ++a) {
            gpos.push_back(c.pos[a]);
            gk.push_back(c.k[a]);
          }
          ge.push_back(trees[idx[j]].erg * std::abs(c.dw));
        }
        gstart.push_back(gstart.back() + (int64_t)L.size());
      }
    }
    if (gstart.size() > 1) {
      const int64_t nc = gstart.back();
      // SoA for the ABI
      std::vector<double> P3(3 * nc), K3(3 * nc), out(nc);
      for (int64_t q = 0; q < nc; ++q)
        for (int a = 0; a < 3; ++a) {
          P3[a * nc + q] = gpos[3 * q + a];
          K3[a * nc + q] = gk[3 * q + a];
        }
      rc = art_get_prob_nonad_host(p, nc, P3.data(), K3.data(), ge.data(), (int64_t)gstart.size() - 1,
                                   gstart.data(), out.data());
      if (rc) return rc;
      int64_t g = 0;
      for (int64_t j = 0; j < m; ++j) {
        if (xcs[j].size() <= 1) continue;
        for (size_t q = 0; q < xcs[j].size(); ++q) xcs[j][q].P = 1.0 - std::exp(-out[gstart[g] + q]);
        ++g;
      }
    }

    // ---- the per-tree bookkeeping of get_tree (:199-350) ----
    for (int64_t j = 0; j < m; ++j) {
      Tree& T = trees[idx[j]];
      Node e = cur[j];
      for (int c = 0; c < 3; ++c) {
        e.x_end[c] = sx[c * m + j];
        e.k_end[c] = sk[c * m + j];
      }
      e.u7_end = su7[j];
      e.tau_end = stau[j];
      e.status = sst[j];
      const std::vector<Cross>& L = xcs[j];
      e.n_cross = (int)L.size();
      if (!L.empty()) e.first = L[0];
      if (nt) {
        for (int k = 0; k < trn[j]; ++k) {
          for (int c = 0; c < 3; ++c) e.traj.push_back(trx[((size_t)c * nt + k) * m + j]);
          e.times.push_back(trt[(size_t)k * m + j]);
        }
        e.xcs = L;
      }
      if (L.empty()) {  // no crossings (:200-207)
        T.count_main += 1;
        T.tot_prob += e.weight;
        const double rr = std::sqrt(e.x_end[0] * e.x_end[0] + e.x_end[1] * e.x_end[1] + e.x_end[2] * e.x_end[2]);
        if (rr > rNS * 1.1) e.is_final = 1;
      } else {
        if (rare[j]) {  // (:213-225), judged on the unmerged crossings
          T.done.push_back(e);
          T.tot_prob += e.weight;
          continue;  // no stop checks, no sort (the reference's `continue`)
        }
        const int new_species = e.species == ART_PHOTON ? ART_AXION : ART_PHOTON;
        const double P1 = L[0].P;
        if (!split_all) {
          if (T.count > opts->mc_nodes) {  // pure MC (:281-292)
            const double r = mc_uniform(opts->seed, (uint64_t)(opts->tree_offset + idx[j]), (uint32_t)T.count);
            if (r < P1)
              T.events.push_back(make_child(L[0], new_species, P1, e.weight, e.weight, P1, P1));
            else
              T.events.push_back(make_child(L[0], e.species, 1.0 - P1, e.weight, e.weight, P1, e.prob_conv));
          } else {  // full tree (:294-305)
            T.events.push_back(make_child(L[0], new_species, P1, P1 * e.weight, e.weight, P1, P1));
            T.events.push_back(
                make_child(L[0], e.species, 1.0 - P1, (1.0 - P1) * e.weight, e.weight, P1, e.prob_conv));
          }
        } else {  // follow one particle over all its crossings (:309-316)
          for (const Cross& c : L) {
            T.events.push_back(make_child(c, new_species, c.P, c.P * e.weight, e.weight, P1, P1));
            e.weight = e.weight * (1.0 - c.P);
          }
          T.tot_prob += e.weight;
        }
      }
      T.done.push_back(e);
      // stop rules (:325-345)
      if (T.tot_prob >= 1.0 - opts->prob_cutoff) {
        T.info = 2;
        T.active = false;
      } else if (opts->num_cutoff <= 0 && split_all) {
        T.active = false;
      } else if (T.count_main >= opts->num_cutoff) {
        T.info = 3;
        T.active = false;
      } else if (T.count > opts->max_nodes) {
        T.info = 4;
        T.active = false;
      } else {
        std::stable_sort(T.events.begin(), T.events.end(),
                         [](const Node& a, const Node& b) { return a.weight < b.weight; });  // (:348)
      }
    }
  }

  // ---- flatten: trees in order, each tree's nodes in the order they were pushed ----
  int64_t total = 0;
  for (const Tree& T : trees) total += (int64_t)T.done.size();
  *n_nodes = total;
  if (total > node_capacity || !nodes) return total > node_capacity ? ART_E_NOMEM : ART_OK;
  int64_t o = 0;
  for (int64_t i = 0; i < n; ++i) {
    Tree& T = trees[i];
    if (counts) counts[i] = T.count;
    if (infos) infos[i] = T.count > opts->mc_nodes ? -std::abs(T.info) : T.info;
    for (const Node& e : T.done) {
      art_tree_node& r = nodes[o++];
      std::memset(&r, 0, sizeof r);
      r.tree = (int32_t)i;
      r.species = e.species;
      r.is_final = e.is_final;
      r.n_cross = e.n_cross;
      r.status = e.status;
      r.weight = e.weight;
      r.prob = e.prob;
      r.parent_weight = e.parent_weight;
      r.prob_conv = e.prob_conv;
      r.prob_conv0 = e.prob_conv0;
      for (int c = 0; c < 3; ++c) {
        r.x0[c] = e.x[c];
        r.k0[c] = e.k[c];
        r.x_end[c] = e.x_end[c];
        r.k_end[c] = e.k_end[c];
        r.xc[c] = e.first.pos[c];
        r.kc[c] = e.first.k[c];
      }
      r.t0 = e.t;
      r.dw0 = e.dw;
      r.u7_end = e.u7_end;
      r.tau_end = e.tau_end;
      r.tc = e.first.t;
      r.dwc = e.first.dw;
      r.pc = e.first.P;
      if (tj) {
        const int64_t q = o - 1;
        const int cnt = (int)e.times.size();
        tj->count[q] = cnt;
        for (int k = 0; k < nt; ++k) {
          for (int c = 0; c < 3; ++c) tj->traj[(q * nt + k) * 3 + c] = k < cnt ? e.traj[3 * k + c] : 0.0;
          tj->times[q * nt + k] = k < cnt ? e.times[k] : 0.0;
        }
        for (int jx = 0; jx < tj->crossing_cap; ++jx) {
          const bool have = jx < (int)e.xcs.size();
          for (int c = 0; c < 3; ++c) tj->xc[(q * tj->crossing_cap + jx) * 4 + c] = have ? e.xcs[jx].pos[c] : 0.0;
          tj->xc[(q * tj->crossing_cap + jx) * 4 + 3] = have ? e.xcs[jx].t : 0.0;
        }
      }
    }
  }
  return ART_OK;
}

}  // namespace

extern "C" int art_grow_trees(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                              const int8_t* species, const art_tree_opts* opts, int64_t node_capacity,
                              art_tree_node* nodes, int64_t* n_nodes, int32_t* counts, int32_t* infos) {
  return grow_trees_impl(p, n, x0, k0, erg, species, opts, node_capacity, nodes, n_nodes, counts, infos, nullptr);
}

extern "C" int art_grow_trees_traj(const art_params* p, int64_t n, const double* x0, const double* k0,
                                   const double* erg, const int8_t* species, const art_tree_opts* opts,
                                   int64_t node_capacity, art_tree_node* nodes, int64_t* n_nodes, int32_t* counts,
                                   int32_t* infos, const art_tree_traj* traj) {
  return grow_trees_impl(p, n, x0, k0, erg, species, opts, node_capacity, nodes, n_nodes, counts, infos, traj);
}
