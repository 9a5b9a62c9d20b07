"""TEST INFRASTRUCTURE ONLY: sequential restatement of get_tree (MainRunner.jl:126-352) and
of the row assembly of main_runner_tree (:498-761) on top of the CPU oracle. The
reference grows one tree at a time, one node per iteration; so does this. It is the
checker for the batched native driver (art_grow_trees) and adiabatic_raytracer_amd.trees.

The reference's global rand(Float64) in Monte-Carlo mode (:283) is replaced by the same
Philox4x32-10 draw the product uses: key = seed, counter = (tree, count, "TREE").
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import oracle as O

AXION, PHOTON = 0, 1
_TREE = 0x54524545


@dataclass
class Node:  # RT.node (RayTracer.jl:126-163), the fields get_tree touches
    x: np.ndarray
    k: np.ndarray
    t: float
    dw: float
    species: int
    prob: float
    weight: float
    parent_weight: float
    prob_conv: float
    prob_conv0: float
    xc: list = field(default_factory=list)  # [(pos, k, t, dw, P)]
    is_final: bool = False
    x_end: np.ndarray = None
    k_end: np.ndarray = None
    u7_end: float = 0.0
    status: int = -1


def mc_uniform(seed: int, tree: int, count: int) -> float:
    o = O.philox4x32_10([tree & 0xFFFFFFFF, tree >> 32, count, _TREE], [seed & 0xFFFFFFFF, seed >> 32])
    return ((o[0] >> 5) * 67108864.0 + (o[1] >> 6)) * (1.0 / 9007199254740992.0)


def get_tree(p, first: Node, erg: float, tree_id: int, *, num_cutoff=5, prob_cutoff=1e-10, splittings_cutoff=-1,
             MC_nodes=5, max_nodes=50, cap=256, seed=1769):
    """get_tree (MainRunner.jl:126-352) with p = oracle params (B0 already signed)."""
    pn = O.get_prob_nonad(p, first.x, first.k, [erg * abs(first.dw)])
    first.prob = 1.0 - math.exp(-pn[0])  # :132-137
    events, tree = [first], []
    tot_prob, count, count_main, info = 0.0, 0, 0, 1
    dt0 = math.exp(-30.0)
    rNS = p.rNS
    while events:
        count += 1
        event = events.pop()
        ln_t0 = math.log(max(event.t, dt0))  # :164
        r = O.propagate(p, event.x, event.k, erg, event.dw, ln_t0, event.species, max_crossings=splittings_cutoff,
                        cap=cap if splittings_cutoff > 0 else 1, nthreads=1)
        event.x_end, event.k_end, event.u7_end = r["x_end"].copy(), r["k_end"].copy(), float(r["u7_end"][0])
        event.status = int(r["status"][0])
        nc = min(int(r["n_cross"][0]), cap if splittings_cutoff > 0 else 1)
        capn = cap if splittings_cutoff > 0 else 1
        xc = [(r["xc_pos"].reshape(3, capn)[:, q].copy(), r["xc_k"].reshape(3, capn)[:, q].copy(),
               float(r["xc_t"][q]), float(r["xc_dw"][q]), float(r["xc_p"][q])) for q in range(nc)]
        if not xc:  # :200-207
            count_main += 1
            tot_prob += event.weight
            if np.linalg.norm(event.x_end) > rNS * 1.1:
                event.is_final = True
        else:
            if any(np.any(np.abs(c[1]) > 1) for c in xc):  # :213-225
                tree.append(event)
                tot_prob += event.weight
                continue
            if len(xc) > 1:  # :227-245
                keep = [np.linalg.norm(np.abs(xc[q + 1][0] - xc[q][0])) > 1e-5 for q in range(len(xc) - 1)] + [True]
                xc = [c for c, kp in zip(xc, keep) if kp]
            if len(xc) > 1:  # one get_Prob_nonAD call with Nc crossings (:265)
                pos = np.array([c[0] for c in xc]).T.reshape(-1)
                kp = np.array([c[1] for c in xc]).T.reshape(-1)
                pn = O.get_prob_nonad(p, pos, kp, [erg * abs(c[3]) for c in xc], group_start=[0, len(xc)])
            else:
                pn = [xc[0][4]]  # Nc = 1: the oracle's own crossing probability
            P = [1.0 - math.exp(-v) for v in pn]
            event.xc = [(c[0], c[1], c[2], c[3], P[q]) for q, c in enumerate(xc)]
            new_species = AXION if event.species == PHOTON else PHOTON
            c0 = event.xc[0]
            if splittings_cutoff <= 0:
                if count > MC_nodes:  # :281-292
                    if mc_uniform(seed, tree_id, count) < P[0]:
                        events.append(Node(c0[0], c0[1], c0[2], c0[3], new_species, P[0], event.weight, event.weight,
                                           P[0], P[0]))
                    else:
                        events.append(Node(c0[0], c0[1], c0[2], c0[3], event.species, 1 - P[0], event.weight,
                                           event.weight, P[0], event.prob_conv))
                else:  # :294-305
                    events.append(Node(c0[0], c0[1], c0[2], c0[3], new_species, P[0], P[0] * event.weight,
                                       event.weight, P[0], P[0]))
                    events.append(Node(c0[0], c0[1], c0[2], c0[3], event.species, 1 - P[0],
                                       (1 - P[0]) * event.weight, event.weight, P[0], event.prob_conv))
            else:  # :309-316
                for c in event.xc:
                    events.append(Node(c[0], c[1], c[2], c[3], new_species, c[4], c[4] * event.weight, event.weight,
                                       P[0], P[0]))
                    event.weight = event.weight * (1 - c[4])
                tot_prob += event.weight
        tree.append(event)
        if tot_prob >= 1 - prob_cutoff:
            info = 2
            break
        if num_cutoff <= 0 and splittings_cutoff > 0:
            break
        if count_main >= num_cutoff:
            info = 3
            break
        if count > max_nodes:
            info = 4
            break
        events.sort(key=lambda e: e.weight)  # stable, as Julia's sort! (:348)
    if count > MC_nodes:
        info = -abs(info)
    return tree, count, info


def main_runner_rows(p, Ntajs, *, seed=1769, rho_DM=0.45, n_maxSample=6, num_cutoff=5, MC_nodes=5, max_nodes=50,
                     prob_cutoff=1e-10, saveMode=0):
    """Rows of main_runner_tree (MainRunner.jl:498-747) for Ntajs - 1 events, sample by sample."""
    n_ev = max(0, int(Ntajs) - 1)
    max_r = O.find_conversion_surface(p)
    s = O.sample(p, max_r, seed, 0, n_ev, nthreads=1)
    w = O.event_weight(p, s["x"], s["k_init"], s["vifty"], max_r, rho_DM, n_maxSample)
    x, k, erg = s["x"].reshape(3, n_ev).T, s["k_init"].reshape(3, n_ev).T, s["erg"]
    f_inx = int(np.sum(s["attempts"].astype(np.int64) - 1))
    pb = _copy_params(p)
    pb.B0 = -p.B0  # the backtrace runs with -B0 (:585)
    rows = []
    for i in range(n_ev):
        root = Node(x[i].copy(), -k[i].copy(), 0.0, -1.0, AXION, 1.0, 1.0, -1.0, -1.0, -1.0)
        nbt, c_bck, _ = get_tree(pb, root, erg[i], i, num_cutoff=0, splittings_cutoff=100000, prob_cutoff=prob_cutoff,
                                 seed=seed)
        nb = nbt[0]
        samp_back_weight = nb.prob * nb.weight
        root = Node(x[i].copy(), k[i].copy(), 0.0, -1.0, PHOTON, 1.0, 1.0, -1.0, -1.0, -1.0)
        tree, c, info = get_tree(p, root, erg[i], i, num_cutoff=num_cutoff, MC_nodes=MC_nodes, max_nodes=max_nodes,
                                 prob_cutoff=prob_cutoff, seed=seed)
        for e in tree:
            if not e.is_final:
                continue
            absf, absfX = np.linalg.norm(e.k_end), np.linalg.norm(e.x_end)
            θf, ϕf = math.acos(e.k_end[2] / absf), math.atan2(e.k_end[1], e.k_end[0])
            θfX, ϕfX = math.acos(e.x_end[2] / absfX), math.atan2(e.x_end[1], e.x_end[0])
            ident = 0 if e.species == AXION else 1
            e.weight *= samp_back_weight
            if ident == 1:
                f_inx += 1
            dω = e.u7_end / p.mass_a + w["vel_eng"][i]
            row = [i + 1, ident, θf, ϕf, θfX, ϕfX, absfX, w["sln_prob"][i], e.weight, x[i, 0], x[i, 1], x[i, 2], dω]
            if saveMode > 0:
                row += [e.weight, 0.0, 1.0, k[i, 0], k[i, 1], k[i, 2], w["cos_w"][i], c, info, e.prob, e.prob_conv,
                        e.prob_conv0, samp_back_weight, absfX, c_bck, nb.prob]
            rows.append(row)
    rows = np.array(rows, np.float64).reshape(len(rows), -1)
    if len(rows):
        rows[:, 7] /= float(f_inx)
    return rows


def _copy_params(p):
    q = type(p)()
    for name, _ in p._fields_:
        setattr(q, name, getattr(p, name))
    return q
