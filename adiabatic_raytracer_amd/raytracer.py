"""Host-side mirror of the reference's ray-tracing operator interface (module `RT`).

The reference calls its hot path as (RayTracer.jl:171-172, MainRunner.jl:179-190):

    RT.propagate(x0, k0, nsteps, Mvars, NumerP, rhs, make_tree, is_axion, Mass_a,
                 max_crossings, Δω)
    get_Prob_nonAD(pos, kpos, Mass_a, Ax_g, θm, ωPul, B0, rNS, erg_inf_ini, vIfty_mag,
                   flat, isotropic, bndry_lyr)                          (MainRunner.jl:67)

`propagate` and `get_Prob_nonAD` below take the same arguments with the same meaning and
order; x0/k0 may hold N rows (the reference always passes one), and every row is
integrated on the GPU by libart.so. Device-resident batches (torch tensors in HBM) use
`Engine`. There is no CPU fallback: if libart.so is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import NamedTuple, Optional

import numpy as np

from . import _lib
from ._lib import ART_AXION, ART_PHOTON, ART_RK4, ART_VERN6, ArtParams, CrossingBuf, SegmentOut, check

ART_NO_CALLBACKS = -(2 ** 31)  # include/art.h: max_crossings for make_tree = false

# Constants.jl:3-5
c_km = 2.99792e5
hbar = 6.582119e-16
GNew = 132712000000.0

# sentinels standing for the reference's RHS functions (RayTracer.jl:71, :95)
func_photon = "func!"
func_axion = "func_axion!"


@dataclass
class Params:
    """Physics + numerics of one run (Gen_Samples.jl:139-170, RayTracer.jl:383-384)."""
    theta_m: float = 0.0        # --ThetaM
    omega_pul: float = 1.0      # --rotW
    B0: float = 1e14            # --B0
    rNS: float = 10.0           # --rNS
    mass_ns: float = 1.0        # --Mass_NS
    mass_a: float = 1e-5        # --MassA
    g_agg: float = 1e-12        # --Axg
    bndry_lyr: float = -1.0     # --bndry_lyr
    ln_t_end: Optional[float] = None  # NumerP[2]; default log(1/ωPul) (MainRunner.jl:412)
    abstol: float = 1e-6        # ode_err (Gen_Samples.jl:162)
    reltol: float = 1e-7
    dtmin: float = 1e-13
    maxiters: int = 100000
    flat: bool = False          # Gen_Samples.jl:165
    isotropic: bool = False     # Gen_Samples.jl:166
    integrator: str = "vern6"   # "vern6" (reference) | "rk4" (fixed step)
    n_fixed: int = 2000         # RK4 steps per segment
    interp_points: int = 50     # ContinuousCallback interp_points (RayTracer.jl:358)

    def to_c(self) -> ArtParams:
        ln_t_end = self.ln_t_end if self.ln_t_end is not None else float(np.log(1.0 / self.omega_pul))
        integ = {"vern6": ART_VERN6, "rk4": ART_RK4}[self.integrator]
        return ArtParams(self.theta_m, self.omega_pul, self.B0, self.rNS, self.mass_ns, self.mass_a, self.g_agg,
                         self.bndry_lyr, ln_t_end, self.abstol, self.reltol, self.dtmin, int(self.maxiters),
                         int(self.flat), int(self.isotropic), 1, integ, int(self.n_fixed), int(self.interp_points))

    def max_r(self) -> float:
        return Find_Conversion_Surface(self)


def params_from_mvars(Mvars, NumerP, is_axion: bool, Ax_g: float = 1e-12, **numerics) -> tuple:
    """Unpack the reference's untyped Mvars vector (MainRunner.jl:177-178 photon order,
    :185-186 axion order) and NumerP = [ln_tstart, ln_tend, ode_err] into Params plus the
    per-ray energy `erg` and start time."""
    if is_axion:
        θm, ωPul, B0, rNS, _gammaF, _time0, Mass_NS, erg, flat, isotropic, melrose, Mass_a, bndry_lyr = Mvars
    else:
        θm, ωPul, B0, rNS, _gammaF, _time0, Mass_NS, Mass_a, erg, flat, isotropic, melrose, bndry_lyr = Mvars
    if not melrose:
        raise ValueError("melrose=false is not supported (the reference hard-codes melrose=true, Gen_Samples.jl:167)")
    ln_t0, ln_t_end, ode_err = NumerP
    p = Params(theta_m=float(θm), omega_pul=float(ωPul), B0=float(B0), rNS=float(rNS), mass_ns=float(Mass_NS),
               mass_a=float(Mass_a), g_agg=float(Ax_g), bndry_lyr=float(bndry_lyr), ln_t_end=float(ln_t_end),
               abstol=float(ode_err), flat=bool(flat), isotropic=bool(isotropic), **numerics)
    return p, np.atleast_1d(np.asarray(erg, np.float64)), float(ln_t0)


class Propagated(NamedTuple):
    """RayTracer.jl:448's 14-tuple for N rows, final saved point only (nsave = 1), plus the
    per-row status / step counts / conversion probability at each crossing."""
    x: np.ndarray          # (N, 3, 1) Cartesian position [km]
    v: np.ndarray          # (N, 3, 1) Cartesian momentum [eV]
    dt: np.ndarray         # (N, 1) u[7] = erg Δω
    fail: np.ndarray       # (N,) 0 if the final radius <= 1.01 rNS (:436-437)
    cut_short: np.ndarray  # (N,) terminated by max_crossings
    xc: list               # per row: array of crossing x
    yc: list
    zc: list
    kxc: list
    kyc: list
    kzc: list
    tc: list               # exp(τ) at the crossings
    Δωc: list              # u7/erg at the crossings
    times: np.ndarray      # (N, 1) final ln t
    status: np.ndarray     # (N,) ART_STATUS_*
    n_accept: np.ndarray
    n_reject: np.ndarray
    p_nonad: list          # per row: get_Prob_nonAD at each crossing (Nc = 1 semantics)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _soa(a, n):
    a = np.asarray(a, np.float64)
    if a.ndim == 1 and a.size == 3 and n == 1:
        a = a.reshape(1, 3)
    if a.shape != (n, 3):
        raise ValueError(f"expected an (N, 3) array, got {a.shape}")
    return np.ascontiguousarray(a.T).reshape(-1)  # Julia column-major N x 3


class PropagatedPlain(NamedTuple):
    """RayTracer.jl:450's 4-tuple (make_tree = false), final saved point only."""
    x: np.ndarray          # (N, 3, 1)
    v: np.ndarray          # (N, 3, 1)
    dt: np.ndarray         # (N, 1)
    fail: np.ndarray       # (N,)


def propagate(x0, k0, nsteps, Mvars, NumerP, rhs=func_photon, make_tree=False, is_axion=False, Mass_a=1e-6,
              max_crossings=3, Δω=-1.0, *, Ax_g=1e-12, capacity=None, **numerics):
    """Batched RT.propagate (RayTracer.jl:171-452): integrate N segments on the GPU.

    Arguments keep the reference's meaning and defaults; `nsteps` only controls saved
    interior points in the reference (saveat) and does not influence the integration, so
    only the final point is returned. `Mass_a` is taken from Mvars, as the reference does.
    make_tree = true installs the resonance callback (and, for photons, the NS cut) and
    returns the 14-tuple (:448, as `Propagated`, with status / step counts / P per row);
    make_tree = false integrates with no callbacks and returns the 4-tuple (:450)."""
    del nsteps, Mass_a
    if (rhs == func_axion) != bool(is_axion):
        raise ValueError("rhs and is_axion disagree (func_axion! <=> is_axion)")
    x0 = np.atleast_2d(np.asarray(x0, np.float64))
    n = x0.shape[0]
    params, erg, ln_t0 = params_from_mvars(Mvars, NumerP, is_axion, Ax_g=Ax_g, **numerics)
    erg = np.broadcast_to(erg, (n,)).astype(np.float64)
    dw = np.broadcast_to(np.asarray(Δω, np.float64), (n,)).copy()
    lnt = np.full(n, ln_t0)
    species = np.full(n, ART_AXION if is_axion else ART_PHOTON, np.int8)
    res = propagate_batch(params, _soa(x0, n), _soa(k0, n), erg, dw, lnt, species,
                          max_crossings=max_crossings if make_tree else ART_NO_CALLBACKS,
                          capacity=capacity or (1 if max_crossings <= 1 or not make_tree else min(int(max_crossings), 64)))
    xe, ke = res["x_end"].reshape(3, n).T, res["k_end"].reshape(3, n).T
    r_end = np.linalg.norm(xe, axis=1)
    fail = np.where(r_end <= params.rNS * 1.01, 0.0, 1.0)  # fail_indx (:436-437)
    if not make_tree:
        return PropagatedPlain(x=xe[:, :, None], v=ke[:, :, None], dt=res["u7_end"][:, None], fail=fail)
    cap = res["capacity"]
    cnt = np.minimum(res["n_cross"], cap)

    def col(a, c, i):
        return np.array([a[(c * cap + j) * n + i] for j in range(cnt[i])])

    def sc(a, i):
        return np.array([a[j * n + i] for j in range(cnt[i])])

    return Propagated(
        x=xe[:, :, None], v=ke[:, :, None], dt=res["u7_end"][:, None], fail=fail, cut_short=res["status"] == 1,
        xc=[col(res["xc_pos"], 0, i) for i in range(n)], yc=[col(res["xc_pos"], 1, i) for i in range(n)],
        zc=[col(res["xc_pos"], 2, i) for i in range(n)], kxc=[col(res["xc_k"], 0, i) for i in range(n)],
        kyc=[col(res["xc_k"], 1, i) for i in range(n)], kzc=[col(res["xc_k"], 2, i) for i in range(n)],
        tc=[sc(res["xc_t"], i) for i in range(n)], Δωc=[sc(res["xc_dw"], i) for i in range(n)],
        times=res["tau_end"][:, None], status=res["status"], n_accept=res["n_accept"], n_reject=res["n_reject"],
        p_nonad=[sc(res["xc_p"], i) for i in range(n)])


def propagate_batch(params: Params, x0, k0, erg, dw, ln_t0, species, max_crossings=-1, capacity=1,
                    ntimes=None, flux_nbins=None) -> dict:
    """Low-level host entry (art_propagate_host): SoA numpy inputs, dict of numpy outputs.
    With ntimes >= 2 (art_propagate_traj_host) also the saved points of RayTracer.jl:176,383:
    traj (3, ntimes, n) Cartesian positions, traj_t (ntimes, n) ln t, traj_n (n) points.
    With flux_nbins (art_propagate_host_flux) also `flux` (2, flux_nbins): the batch's binned
    radiated flux (plot/flux.py:38-48), axions in row 0, photons in row 1. The two are separate
    entry points of the C ABI: asking for both raises ValueError."""
    if ntimes and flux_nbins:
        raise ValueError("ntimes (saveat) and flux_nbins are separate entry points: ask for one of them")
    lib = _lib.load()
    n = int(np.asarray(erg).size)
    f64 = lambda a: np.ascontiguousarray(a, np.float64)  # noqa: E731
    x0, k0, erg, dw, ln_t0 = f64(x0), f64(k0), f64(erg), f64(dw), f64(ln_t0)
    species = np.ascontiguousarray(species, np.int8)
    if x0.size != 3 * n or k0.size != 3 * n or dw.size != n or ln_t0.size != n or species.size != n:
        raise ValueError("inconsistent batch sizes")
    out = {"x_end": np.zeros(3 * n), "k_end": np.zeros(3 * n), "u7_end": np.zeros(n), "tau_end": np.zeros(n),
           "status": np.zeros(n, np.int32), "n_accept": np.zeros(n, np.int32), "n_reject": np.zeros(n, np.int32),
           "n_cross": np.zeros(n, np.int32), "xc_pos": np.zeros(3 * capacity * n), "xc_k": np.zeros(3 * capacity * n),
           "xc_t": np.zeros(capacity * n), "xc_dw": np.zeros(capacity * n), "xc_p": np.zeros(capacity * n),
           "capacity": capacity}
    so = SegmentOut(*[_ptr(out[k]) for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept",
                                               "n_reject")])
    xb = CrossingBuf(capacity, *[_ptr(out[k]) for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")])
    cp = params.to_c()
    if ntimes:
        out.update(traj=np.zeros(3 * ntimes * n), traj_t=np.zeros(ntimes * n), traj_n=np.zeros(n, np.int32))
        check(lib.art_propagate_traj_host(C.byref(cp), n, _ptr(x0), _ptr(k0), _ptr(erg), _ptr(dw), _ptr(ln_t0),
                                          _ptr(species), int(max_crossings), C.byref(so), C.byref(xb), int(ntimes),
                                          _ptr(out["traj"]), _ptr(out["traj_t"]), _ptr(out["traj_n"])))
        out["traj"] = out["traj"].reshape(3, ntimes, n)
        out["traj_t"] = out["traj_t"].reshape(ntimes, n)
    elif flux_nbins:
        out["flux"] = np.zeros(2 * int(flux_nbins))
        check(lib.art_propagate_host_flux(C.byref(cp), n, _ptr(x0), _ptr(k0), _ptr(erg), _ptr(dw), _ptr(ln_t0),
                                          _ptr(species), int(max_crossings), C.byref(so), C.byref(xb),
                                          int(flux_nbins), _ptr(out["flux"])))
        out["flux"] = out["flux"].reshape(2, int(flux_nbins))
    else:
        check(lib.art_propagate_host(C.byref(cp), n, _ptr(x0), _ptr(k0), _ptr(erg), _ptr(dw), _ptr(ln_t0),
                                     _ptr(species), int(max_crossings), C.byref(so), C.byref(xb)))
    out["kernel_ms"] = lib.art_last_kernel_ms()
    out["stats"] = last_stats()
    return out


class HostCall:
    """An asynchronous art_propagate_host_flux call (propagate_batch_async): holds the call's
    arrays until wait() returns its outputs (the dict propagate_batch returns)."""

    def __init__(self, ticket, out, keep):
        self.ticket, self.out, self._keep = ticket, out, keep
        self._waited = False

    def wait(self) -> dict:
        if not self._waited:
            self._waited = True
            check(_lib.load().art_host_wait(self.ticket))
            self.out["flux"] = self.out["flux"].reshape(2, -1)
            self._keep = None
        return self.out

    def __del__(self):
        # the library's worker writes through raw pointers into the arrays this object holds:
        # a call dropped without wait() (an exception between submit and wait) must not free
        # them while the GPU and the host threads still write into them
        if not getattr(self, "_waited", True):
            self._waited = True
            try:
                _lib.load().art_host_wait(self.ticket)
            except Exception:  # noqa: BLE001 -- interpreter shutdown: nothing left to report to
                pass
            self._keep = None


def propagate_batch_async(params: Params, x0, k0, erg, dw, ln_t0, species, flux_nbins, max_crossings=-1,
                          capacity=1) -> HostCall:
    """art_propagate_host_flux_async: the call runs on a library worker thread (two per device
    in flight, the next batch's uploads and first rays overlapping this one's drain); wait() on
    the returned HostCall gives propagate_batch's dict, bit for bit the synchronous call's."""
    lib = _lib.load()
    n = int(np.asarray(erg).size)
    f64 = lambda a: np.ascontiguousarray(a, np.float64)  # noqa: E731
    x0, k0, erg, dw, ln_t0 = f64(x0), f64(k0), f64(erg), f64(dw), f64(ln_t0)
    species = np.ascontiguousarray(species, np.int8)
    if x0.size != 3 * n or k0.size != 3 * n or dw.size != n or ln_t0.size != n or species.size != n:
        raise ValueError("inconsistent batch sizes")
    out = {"x_end": np.zeros(3 * n), "k_end": np.zeros(3 * n), "u7_end": np.zeros(n), "tau_end": np.zeros(n),
           "status": np.zeros(n, np.int32), "n_accept": np.zeros(n, np.int32), "n_reject": np.zeros(n, np.int32),
           "n_cross": np.zeros(n, np.int32), "xc_pos": np.zeros(3 * capacity * n), "xc_k": np.zeros(3 * capacity * n),
           "xc_t": np.zeros(capacity * n), "xc_dw": np.zeros(capacity * n), "xc_p": np.zeros(capacity * n),
           "capacity": capacity, "flux": np.zeros(2 * int(flux_nbins))}
    so = SegmentOut(*[_ptr(out[k]) for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept",
                                               "n_reject")])
    xb = CrossingBuf(capacity, *[_ptr(out[k]) for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")])
    cp = params.to_c()
    ticket = C.c_int64(-1)
    check(lib.art_propagate_host_flux_async(C.byref(cp), n, _ptr(x0), _ptr(k0), _ptr(erg), _ptr(dw), _ptr(ln_t0),
                                            _ptr(species), int(max_crossings), C.byref(so), C.byref(xb),
                                            int(flux_nbins), _ptr(out["flux"]), C.byref(ticket)))
    return HostCall(ticket.value, out, (x0, k0, erg, dw, ln_t0, species, so, xb, cp))


def last_stats() -> dict:
    lib = _lib.load()
    s = (C.c_uint64 * 8)()
    g = C.c_int32()
    check(lib.art_last_stats(s, C.byref(g)))
    keys = ("attempts", "accepted", "root_steps", "scan_evals", "interp_evals", "rays", "init_rhs", "cert_steps")
    d = {k: int(s[i]) for i, k in enumerate(keys)}
    d["grid"] = int(g.value)
    return d


HOST_PATH_KEYS = ("calls", "streamed", "stream_giveups", "chunked", "single")


def recent_kernel_span_ms(n: int = 1) -> list:
    """The last n propagate launches' integrator spans [ms] from in-kernel clock stamps (first
    wave start to last wave end, art_recent_kernel_span_ms), oldest first: the launch's own
    duration, free of a profiler's completion signals; -1 where a launch left no stamps."""
    lib = _lib.load()
    buf = (C.c_double * max(1, n))()
    got = lib.art_recent_kernel_span_ms(int(n), buf)
    if got < 0:
        check(got)
    return list(buf)[:got]


def host_path_counters(reset=False) -> dict:
    """What this process's art_propagate_host* calls ran as (art_host_path_counters): calls,
    streamed-pipeline completions, streamed give-ups (rerun as one launch), chunked and
    single-launch calls."""
    c = (C.c_uint64 * len(HOST_PATH_KEYS))()
    rc = _lib.load().art_host_path_counters(c, len(HOST_PATH_KEYS), 1 if reset else 0)
    if rc < 0:
        check(rc)
    return {k: int(c[i]) for i, k in enumerate(HOST_PATH_KEYS)}


def Find_Conversion_Surface(params: Params) -> float:
    """RT.Find_Conversion_Surface (RayTracer.jl:1250-1263) with fix_time = 0."""
    cp = params.to_c()
    return float(_lib.load().art_find_conversion_surface(C.byref(cp)))


def get_Prob_nonAD(pos, kpos, Mass_a, Ax_g, θm, ωPul, B0, rNS, erg_inf_ini, vIfty_mag, flat, isotropic, bndry_lyr,
                   *, Mass_NS=1.0, group_start=None) -> np.ndarray:
    """get_Prob_nonAD (MainRunner.jl:67-124) on the GPU. One call of the reference = one
    group; pass `group_start` (len n_groups + 1) to evaluate many calls at once. Mass_NS is
    the reference's global (Gen_Samples.jl:144)."""
    del vIfty_mag  # unused by the reference's probability (only printed)
    pos = np.atleast_2d(np.asarray(pos, np.float64))
    nc = pos.shape[0]
    e = np.broadcast_to(np.asarray(erg_inf_ini, np.float64).reshape(-1), (nc,)).copy()
    p = Params(theta_m=θm, omega_pul=ωPul, B0=B0, rNS=rNS, mass_ns=Mass_NS, mass_a=Mass_a, g_agg=Ax_g,
               bndry_lyr=bndry_lyr, flat=bool(flat), isotropic=bool(isotropic)).to_c()
    out = np.zeros(nc)
    gs = None if group_start is None else np.ascontiguousarray(group_start, np.int64)
    ng = nc if gs is None else gs.size - 1
    check(_lib.load().art_get_prob_nonad_host(C.byref(p), nc, _ptr(_soa(pos, nc)), _ptr(_soa(kpos, nc)), _ptr(e), ng,
                                              _ptr(gs), _ptr(out)))
    return out


def sample_conversion_points(params: Params, n: int, seed: int = 1769, ray_offset: int = 0, max_r=None) -> dict:
    """find_samples_new (RayTracer.jl:1480-1653) + k_norm_Cart (MainRunner.jl:529) on the
    GPU: one accepted conversion point per ray, Philox stream keyed by (seed, ray id)."""
    max_r = params.max_r() if max_r is None else max_r
    out = {"x": np.zeros(3 * n), "k_init": np.zeros(3 * n), "erg": np.zeros(n), "vifty": np.zeros(3 * n),
           "weights": np.zeros(n, np.int32), "attempts": np.zeros(n, np.int32)}
    cp = params.to_c()
    check(_lib.load().art_sample_conversion_points_host(
        C.byref(cp), float(max_r), int(seed), int(ray_offset), int(n), *[_ptr(out[k]) for k in
                                                                        ("x", "k_init", "erg", "vifty", "weights",
                                                                         "attempts")]))
    return out


EVENT_FIELDS = ("cos_w", "jacobian_GR", "sln_prob", "erg_inf_ini", "vel_eng")


def event_weight(params: Params, x, k_init, vifty, max_r=None, rho_DM=0.45, n_maxSample=6) -> dict:
    """Per-sample event weight of main_runner_tree (MainRunner.jl:498-557) on the GPU:
    cos_w of RT.dwp_ds, jacobian_GR = RT.g_det and sln_prob = |cos_w| redshift phaseS
    (1e5)^2 c 1e5 mcmc_weights (before the final division by f_inx, :722). x, k_init and
    vifty are the sampler's SoA outputs (3n)."""
    max_r = params.max_r() if max_r is None else max_r
    x, k_init, vifty = (np.ascontiguousarray(a, np.float64).reshape(-1) for a in (x, k_init, vifty))
    n = x.size // 3
    out = np.zeros(5 * n)
    check(_lib.load().art_event_weight_host(C.byref(params.to_c()), float(max_r), float(rho_DM), float(n_maxSample),
                                            n, _ptr(x), _ptr(k_init), _ptr(vifty), _ptr(out)))
    o = out.reshape(5, n)
    return {k: o[i].copy() for i, k in enumerate(EVENT_FIELDS)}


def vern6_tableau():
    c, A, b, bh = np.zeros(9), np.zeros(81), np.zeros(9), np.zeros(9)
    check(_lib.load().art_vern6_tableau(_ptr(c), _ptr(A), _ptr(b), _ptr(bh)))
    return c, A.reshape(9, 9), b, bh
