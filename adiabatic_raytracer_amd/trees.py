"""Trees and events on the GPU engine: the host side of main_runner_tree (MainRunner.jl:354-763).

grow_trees()        get_tree (MainRunner.jl:126-352) for many trees at once, through the
                    native batched driver art_grow_trees (csrc/art_forest.cpp).
main_runner_tree()  the event loop: sample conversion points, weight them (sln_prob),
                    backtrace each one (axion, -k, -B0, every crossing), grow its forward
                    photon tree, and write the reference's npy rows, with the same columns
                    and the same file name (MainRunner.jl:715-761), so Combine_Files.py and
                    plot/*.py read them unchanged.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import replace

import numpy as np

from . import _lib
from ._lib import TreeOpts, TreeTraj, check
from .raytracer import Params, event_weight, sample_conversion_points

AXION, PHOTON = 0, 1


# include/art.h art_tree_node, as a numpy record (checked against the C layout in tests)
NODE_DTYPE = np.dtype([
    ("tree", np.int32), ("species", np.int32), ("is_final", np.int32), ("n_cross", np.int32),
    ("status", np.int32), ("pad", np.int32),
    ("weight", np.float64), ("prob", np.float64), ("parent_weight", np.float64), ("prob_conv", np.float64),
    ("prob_conv0", np.float64),
    ("x0", np.float64, 3), ("k0", np.float64, 3), ("t0", np.float64), ("dw0", np.float64),
    ("x_end", np.float64, 3), ("k_end", np.float64, 3), ("u7_end", np.float64), ("tau_end", np.float64),
    ("xc", np.float64, 3), ("kc", np.float64, 3), ("tc", np.float64), ("dwc", np.float64), ("pc", np.float64),
], align=True)


def grow_trees(params: Params, x0, k0, erg, species, *, num_cutoff=5, mc_nodes=5, max_nodes=50,
               splittings_cutoff=-1, crossing_cap=64, prob_cutoff=1e-10, seed=1769, ntimes=None, tree_offset=0):
    """get_tree for n roots RT.node(x0, k0, 0, -1, species, 1, 1, -1, -1, -1) (MainRunner.jl:578-590,
    :653-667). x0, k0: (n, 3) or SoA 3n; erg: erg_inf_ini per root. Returns (nodes, counts,
    infos): nodes is a NODE_DTYPE record array grouped by tree in get_tree's push order.
    With ntimes (>= 2, saveMode 3) a fourth item holds every node's saveNode data
    (art_grow_trees_traj): traj (nodes, ntimes, 3) Cartesian saved points, times (nodes,
    ntimes) their ln t, count (nodes,), xc (nodes, cap, 4) the kept crossings (x, y, z, tc).
    tree_offset: global id of root 0 (the Monte-Carlo draws are keyed by the global tree id)."""
    x0, k0 = np.asarray(x0, np.float64), np.asarray(k0, np.float64)
    erg = np.ascontiguousarray(erg, np.float64).reshape(-1)
    n = erg.size
    if x0.ndim == 2:
        x0, k0 = x0.T, k0.T
    x0, k0 = np.ascontiguousarray(x0).reshape(-1), np.ascontiguousarray(k0).reshape(-1)
    sp = np.ascontiguousarray(np.broadcast_to(np.asarray(species, np.int8), (n,)))
    opts = TreeOpts(num_cutoff, mc_nodes, max_nodes, splittings_cutoff, crossing_cap, int(tree_offset), prob_cutoff,
                    seed)
    per_tree = 1 if (splittings_cutoff > 0 and num_cutoff <= 0) else max_nodes + 2
    cap = max(1, n * per_tree)
    lib = _lib.load()
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    xcap = max(1, crossing_cap) if splittings_cutoff > 0 else 1
    while True:
        nodes = np.zeros(cap, NODE_DTYPE)
        nn = C.c_int64(0)
        counts, infos = np.zeros(n, np.int32), np.zeros(n, np.int32)
        if ntimes:
            tr = {"traj": np.zeros((cap, ntimes, 3)), "times": np.zeros((cap, ntimes)),
                  "count": np.zeros(cap, np.int32), "xc": np.zeros((cap, xcap, 4))}
            tt = TreeTraj(int(ntimes), xcap, *[ptr(tr[k]) for k in ("traj", "times", "count", "xc")])
            rc = lib.art_grow_trees_traj(C.byref(params.to_c()), n, ptr(x0), ptr(k0), ptr(erg), ptr(sp),
                                         C.byref(opts), cap, ptr(nodes), C.byref(nn), ptr(counts), ptr(infos),
                                         C.byref(tt))
        else:
            rc = lib.art_grow_trees(C.byref(params.to_c()), n, ptr(x0), ptr(k0), ptr(erg), ptr(sp), C.byref(opts),
                                    cap, ptr(nodes), C.byref(nn), ptr(counts), ptr(infos))
        if rc == -3 and nn.value > cap:  # ART_E_NOMEM: grow and redo (pathological trees only)
            cap = nn.value
            continue
        check(rc)
        if ntimes:
            return nodes[:nn.value], counts, infos, {k: v[:nn.value] for k, v in tr.items()}
        return nodes[:nn.value], counts, infos


def _angles(v):
    a = np.linalg.norm(v, axis=-1)
    return np.arccos(v[..., 2] / a), np.arctan2(v[..., 1], v[..., 0]), a


def jl(x) -> str:
    """Julia's string(::Float64): shortest round-trip digits, scientific notation (1.0e14,
    2.0e-5) outside [1e-4, 1e6)."""
    x = float(x)
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    if not math.isfinite(x):
        return "NaN" if math.isnan(x) else ("Inf" if x > 0 else "-Inf")
    if 1e-4 <= abs(x) < 1e6:
        r = repr(x)
        return r if ("." in r or "e" in r) else r + ".0"
    m, e = np.format_float_scientific(x, unique=True, trim="-").split("e")
    return f"{m if '.' in m else m + '.0'}e{int(e)}"


def tree_file_name(dir_tag, Mass_a, Ax_g, θm, ωPul, B0, Ntajs, ntimes, num_cutoff, MC_nodes, max_nodes, file_tag):
    """The npy name of MainRunner.jl:750-760, with Julia's number formatting."""
    name = (f"tree_MassAx_{jl(Mass_a)}_AxionG_{jl(Ax_g)}_ThetaM_{jl(θm)}_rotPulsar_{jl(ωPul)}_B0_{jl(B0)}"
            f"_Ax_trajs_{int(Ntajs)}_N_Times_{int(ntimes)}_num_cutoff_{int(num_cutoff)}_MC_nodes_{int(MC_nodes)}"
            f"_max_nodes_{int(max_nodes)}_{file_tag}.npy")
    return os.path.join(dir_tag, "npy", name)


def _write_event_text(dir_tag, file_tag, n_ev, s, w, x, k, tree, fin, ev, wgt, ident, counts, elapsed=None,
                      ev_offset=0):
    """event_<file_tag> and final_<file_tag> of saveMode > 1 (MainRunner.jl:438-444, 592-609,
    690-702, 735-741), Julia number formatting. The reference's per-event wall time
    time() - time0 has no per-event meaning in a batched run; the mean per event is written."""
    d = os.path.join(dir_tag, "event")
    os.makedirs(d, exist_ok=True)
    v = s["vifty"].reshape(3, n_ev).T
    t_ev = 0.0 if elapsed is None else elapsed / max(1, n_ev)
    with open(os.path.join(d, "event_" + file_tag), "w") as fe:
        for i in range(n_ev):
            vals = [*v[i], w["sln_prob"][i], *x[i], *(-k[i]), *x[i], *k[i]]
            fe.write(f"{ev_offset + i + 1} " + " ".join(jl(a) for a in vals) + f" {jl(t_ev)} {int(counts[i])}\n")
    θf, ϕf, absf = _angles(fin["k_end"])
    θfX, ϕfX, absfX = _angles(fin["x_end"])
    # node.t: the root's is the integer literal 0 of RT.node(..., 0, ...) (MainRunner.jl:661)
    first = np.zeros(len(tree), bool)
    first[np.r_[0, np.flatnonzero(np.diff(tree["tree"])) + 1]] = True
    is_root = first[tree["is_final"] != 0]
    with open(os.path.join(d, "final_" + file_tag), "w") as ff:
        for q in range(len(fin)):
            t = "0" if is_root[q] else jl(fin["t0"][q])
            vals = [θf[q], ϕf[q], absf[q], θfX[q], ϕfX[q], absfX[q]]
            ff.write(f"{ev_offset + int(ev[q]) + 1} {jl(wgt[q])} {int(ident[q])} " + " ".join(jl(a) for a in vals) + f" {t}\n")


SPECIES_NAME = {AXION: "axion", PHOTON: "photon"}


def save_node(fh, node, tr, q):
    """saveNode(f, n) (MainRunner.jl:17-65) for node q of a grow_trees(..., ntimes) result:
    species, weight, prob, parent_weight; the crossing x, y, z and tc lines (or "-" x 3);
    the saved trajectory's x, y, z and ln t lines. Julia number formatting."""
    fh.write(f"{SPECIES_NAME[int(node['species'])]} {jl(node['weight'])} {jl(node['prob'])} "
             f"{jl(node['parent_weight'])}\n")
    m = min(int(node["n_cross"]), tr["xc"].shape[1])
    if m > 0:
        for c in range(3):
            fh.write("".join("  " + jl(tr["xc"][q, j, c]) for j in range(m)) + "\n")
        fh.write("".join("  " + jl(tr["xc"][q, j, 3]) for j in range(m)))
    else:
        fh.write("-\n-\n-")
    fh.write("\n")
    cnt = int(tr["count"][q])
    for c in range(3):
        fh.write("".join("  " + jl(tr["traj"][q, k, c]) for k in range(cnt)) + "\n")
    fh.write("".join("  " + jl(tr["times"][q, k]) for k in range(cnt)) + "\n")


def main_runner_tree(params: Params, Ntajs: int, *, seed=1769, ntimes=1000, rho_DM=0.45, n_maxSample=6,
                     num_cutoff=5, MC_nodes=5, max_nodes=50, prob_cutoff=1e-10, saveMode=0, dir_tag=None,
                     file_tag="", backtrace_cap=256, rank=0, world=1, nbins=50, run_info=None):
    """main_runner_tree (MainRunner.jl:354-763) for Ntajs - 1 events (the reference's
    `while photon_trajs < desired_trajs` loop), all events batched on the GPU. Returns the
    row matrix (13 columns, 29 with saveMode > 0) after the final division of column 8 by
    f_inx, and writes it to the reference's npy path when dir_tag is given; saveMode > 1
    also writes the event_/final_ text files and saveMode > 2 one tree_<file_tag><event>
    file per event with saveNode of the backtrace node and of every forward-tree node
    (MainRunner.jl:573-577, :612, :671), each segment saved at ntimes points.

    Sharding, world > 1 with torch.distributed initialised (one process per
    GPU): the Ntajs - 1 events of ONE logical run are split by global event id
    (shard.shard_range). Rank r samples its block (Philox keyed by the global event id),
    backtraces it and grows its trees (Monte-Carlo draws keyed by the global tree id), and
    numbers its rows by global event id, so the ranks' rows in rank order are the
    single-process rows. f_inx (MainRunner.jl:469,477,711-713) is all-reduced and column 8
    is divided by the GLOBAL f_inx (:747): the normalisation of one large run, not the
    per-file /Nruns of Gen_Samples.jl:220. Rank r writes file_tag + str(r) (:750-761).

    run_info (a dict, optional) receives the run's reduced totals: f_inx (global), the
    binned radiated flux of plot/flux.py:38-48 -- np.histogram(φf, nbins, range=(-π, π),
    weights = weight * sln_prob) of the rows, axions in flux[0], photons in flux[1], after
    the f_inx division, binned on the GPU and summed over ranks in the same all-reduce --
    Σ weight * sln_prob per species and the global row count."""
    if saveMode < 3:
        ntimes = 3  # "Times to store in ODE" (MainRunner.jl:379-381): also names the npy file
    import time
    from .shard import allreduce_sum, shard_range
    t_start = time.perf_counter()
    n_glob = max(0, int(Ntajs) - 1)
    lo, hi = shard_range(n_glob, rank, world)
    n_ev = hi - lo
    tag = f"{file_tag}{rank}" if world > 1 else file_tag
    max_r = params.max_r()
    if max_r < params.rNS:
        raise ValueError("maxR < rNS: this neutron star has no conversion surface (MainRunner.jl:387-396)")
    s = sample_conversion_points(params, n_ev, seed=seed, ray_offset=lo, max_r=max_r)
    w = event_weight(params, s["x"], s["k_init"], s["vifty"], max_r=max_r, rho_DM=rho_DM, n_maxSample=n_maxSample)
    x = s["x"].reshape(3, n_ev).T
    k = s["k_init"].reshape(3, n_ev).T
    erg = s["erg"]
    # f_inx: find_samples_new calls minus accepted samples (MainRunner.jl:463-481)
    f_inx = int(np.sum(s["attempts"].astype(np.int64) - 1))
    # backtrace: axion, -k, -B0, every crossing, only the root is processed (:578-590)
    dumps = saveMode > 2 and dir_tag is not None
    got = grow_trees(replace(params, B0=-params.B0), x, -k, erg, AXION, num_cutoff=0, splittings_cutoff=100000,
                     crossing_cap=backtrace_cap, prob_cutoff=prob_cutoff, seed=seed, ntimes=ntimes if dumps else None,
                     tree_offset=lo)
    nb, c_bck = got[0], got[1]
    samp_back_weight = nb["prob"] * nb["weight"]  # (:635)
    prob0 = nb["prob"]
    # forward photon tree from the sample (:653-667)
    fwd = grow_trees(params, x, k, erg, PHOTON, num_cutoff=num_cutoff, mc_nodes=MC_nodes, max_nodes=max_nodes,
                     prob_cutoff=prob_cutoff, seed=seed, ntimes=ntimes if dumps else None, tree_offset=lo)
    tree, counts, infos = fwd[:3]
    if dumps:  # saveMode > 2: one file per event, the backtrace node then the forward tree
        d = os.path.join(dir_tag, "tree")
        os.makedirs(d, exist_ok=True)
        for e in range(n_ev):
            with open(os.path.join(d, f"tree_{file_tag}{lo + e + 1}"), "w") as fh:
                save_node(fh, nb[e], got[3], e)
                for q in np.flatnonzero(tree["tree"] == e):
                    save_node(fh, tree[q], fwd[3], q)
    fin = tree[tree["is_final"] != 0]
    ev = fin["tree"]
    θf, ϕf, _ = _angles(fin["k_end"])
    θfX, ϕfX, absfX = _angles(fin["x_end"])
    wgt = fin["weight"] * samp_back_weight[ev]  # tree[ii].weight *= samp_back_weight (:690)
    ident = np.where(fin["species"] == AXION, 0.0, 1.0)
    f_inx += int(np.sum(ident == 1.0))
    dω = fin["u7_end"] / params.mass_a + w["vel_eng"][ev]  # (:713)
    photon_trajs = lo + ev + 1.0  # global event number
    cols = [photon_trajs, ident, θf, ϕf, θfX, ϕfX, absfX, w["sln_prob"][ev], wgt, x[ev, 0], x[ev, 1], x[ev, 2], dω]
    if saveMode > 0:
        zero = np.zeros_like(wgt)
        cols += [wgt, zero, zero + 1.0, k[ev, 0], k[ev, 1], k[ev, 2], w["cos_w"][ev], counts[ev].astype(float),
                 infos[ev].astype(float), fin["prob"], fin["prob_conv"], fin["prob_conv0"], samp_back_weight[ev],
                 absfX, c_bck[ev].astype(float), prob0[ev]]
    rows = np.stack(cols, axis=1) if len(fin) else np.zeros((0, len(cols)))
    if saveMode > 1 and dir_tag is not None:
        _write_event_text(dir_tag, tag, n_ev, s, w, x, k, tree, fin, ev, wgt, ident, counts,
                          elapsed=time.perf_counter() - t_start, ev_offset=lo)
    # the run's totals: [flux (2 nbins, weight * sln_prob before the f_inx division) | f_inx |
    # Σ weight * sln_prob (axions, photons) | rows], ONE sum over the ranks
    # the binned flux (a GPU histogram) only when someone reads it: the reduced run_info, or the
    # other ranks' sum (every rank must contribute its part); f_inx alone normalises column 8
    want_flux = len(rows) and (world > 1 or run_info is not None)
    flux = radiated_flux(rows[:, 3], rows[:, 1], rows[:, 8] * rows[:, 7], nbins) if want_flux else np.zeros(2 * nbins)
    pps = rows[:, 8] * rows[:, 7] if len(rows) else np.zeros(0)
    tot = np.concatenate([flux, [float(f_inx), float(pps[rows[:, 1] == 0].sum()) if len(rows) else 0.0,
                                 float(pps[rows[:, 1] == 1].sum()) if len(rows) else 0.0, float(len(rows))]])
    if world > 1:
        tot = allreduce_sum(tot)
    f_glob = tot[2 * nbins]
    if len(rows):
        rows[:, 7] /= f_glob  # saveAll[:, 8] ./= f_inx (:747), the whole run's f_inx
    if run_info is not None:
        run_info.update(f_inx=int(round(f_glob)), flux=(tot[:2 * nbins] / f_glob).reshape(2, nbins),
                        sum_weight_sln_prob=(tot[2 * nbins + 1] / f_glob, tot[2 * nbins + 2] / f_glob),
                        rows=int(round(tot[2 * nbins + 3])), events=(lo, hi), n_events=n_glob)
    if dir_tag is not None:
        path = tree_file_name(dir_tag, params.mass_a, params.g_agg, params.theta_m, params.omega_pul, params.B0, Ntajs,
                              ntimes, num_cutoff, MC_nodes, max_nodes, tag)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.save(path, rows)
    return rows


def radiated_flux(phif, ident, weights, nbins=50, range=(-np.pi, np.pi)) -> np.ndarray:
    """The binned flux of plot/flux.py:38-48 on the GPU: np.histogram(phif, nbins,
    range=range, weights=weights) for axion rows (ident 0) and photon rows (ident 1), as a
    (2 * nbins,) array [axions | photons]. The reference's radiated flux is the photon half with
    weights = weight * sln_prob (npy columns 9 and 8). range=None bins like flux.py:43-47 itself,
    np.histogram(phif, bins=nbins) without a range: over [min φf, max φf] of ALL the rows
    (numpy's rule, ±0.5 when they are equal); `flux_edges` gives those edges."""
    import torch
    lib = _lib.load()
    n = len(phif)
    lo, hi = flux_range(phif) if range is None else (float(range[0]), float(range[1]))
    dev = torch.device("cuda", torch.cuda.current_device())
    f = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(dev)  # noqa: E731
    ph, sp, ww = f(phif), f(np.asarray(ident) != 0, torch.int8), f(weights)
    hist = torch.zeros(2 * nbins, dtype=torch.float64, device=dev)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    check(lib.art_flux_histogram_phi_range_device(n, C.c_void_p(ph.data_ptr()), C.c_void_p(sp.data_ptr()),
                                                  C.c_void_p(ww.data_ptr()), int(nbins), lo, hi,
                                                  C.c_void_p(hist.data_ptr()), stream))
    return hist.cpu().numpy()


def flux_range(phif):
    """np.histogram's range when none is given: (min, max) of the data, widened by 0.5 on each
    side when they are equal, (0, 1) for no data."""
    a = np.asarray(phif, np.float64)
    if a.size == 0:
        return 0.0, 1.0
    lo, hi = float(a.min()), float(a.max())
    return (lo - 0.5, hi + 0.5) if lo == hi else (lo, hi)


def flux_edges(lo, hi, nbins=50):
    """The bin edges np.histogram uses for `nbins` equal bins of [lo, hi] (np.linspace)."""
    return np.linspace(lo, hi, nbins + 1)


def gather_rank_rows(dir_tag, params: Params, Ntajs, world, file_tag="", ntimes=3, num_cutoff=5, MC_nodes=5,
                     max_nodes=50) -> np.ndarray:
    """The rows of a sharded run: its per-rank files (file_tag + str(rank)) concatenated in rank
    order -- the rows the single-process run writes."""
    return np.concatenate([np.load(tree_file_name(dir_tag, params.mass_a, params.g_agg, params.theta_m,
                                                  params.omega_pul, params.B0, Ntajs, ntimes, num_cutoff, MC_nodes,
                                                  max_nodes, f"{file_tag}{r}")) for r in range(int(world))], axis=0)


def combine_files(Mass_a, Ax_g, θm, ωPul, B0, Ntajs, Nruns, file_tag, ntimes=3, dir_tag="results", num_cutoff=5,
                  MC_nodes=5, max_nodes=50, remove=True):
    """Gen_Samples.jl --run_Combine 1 (combine_files, Gen_Samples.jl:195-239): concatenate the
    npy rows of runs file_tag + "0" .. file_tag + str(Nruns - 1), divide column 8 (1-based,
    sln_prob) by Nruns, write them to dir_tag/<name with Ax_trajs = Ntajs * Nruns>.npy and
    delete the inputs. Returns the combined path."""
    files = [tree_file_name(dir_tag, Mass_a, Ax_g, θm, ωPul, B0, Ntajs, ntimes, num_cutoff, MC_nodes, max_nodes,
                            f"{file_tag}{i}") for i in range(int(Nruns))]
    hold = np.concatenate([np.load(f) for f in files], axis=0)
    hold[:, 7] /= Nruns  # hold[:, 8] ./= Nruns (Julia 1-based, :220)
    name = os.path.basename(tree_file_name(dir_tag, Mass_a, Ax_g, θm, ωPul, B0, Ntajs * Nruns, ntimes, num_cutoff,
                                           MC_nodes, max_nodes, file_tag))
    out = os.path.join(dir_tag, name[len("tree_"):])  # dir_tag/MassAx_... (:223-231)
    np.save(out, hold)
    if remove:
        for f in files:
            os.remove(f)
    return out


def combine_files_py(out_path, files) -> np.ndarray:
    """Combine_Files.py OUT IN... (the reference's Python combine, Combine_Files.py:1-31):
    the row files in the given order, each file's event numbers (column 1) offset by the last
    event number combined so far (:22), and -- its quirk -- column 10 (0-based 9, the sampled
    x position) divided by the number of files (:28). Writes out_path and returns the rows.
    (Gen_Samples.jl --run_Combine divides the sln_prob column instead: combine_files.)"""
    data = None
    for f in files:
        name = os.path.basename(f)
        if not (name[:5] == "tree_" and name[-4:] == ".npy"):
            raise ValueError(f"{f} is not a tree_*.npy row file")
        tmp = np.load(f).T.copy()
        if data is None:
            data = tmp
        else:
            tmp[0, :] += data[0, -1]
            data = np.append(data, tmp, axis=1)
    if data is None:
        raise ValueError("no input files")
    data[9, :] /= len(files)
    np.save(out_path, data.T)
    return data.T

