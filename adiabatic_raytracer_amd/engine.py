"""Device-resident batches: inputs and outputs live in HBM as torch tensors (PyTorch is
plumbing for device memory and streams here); every compute call goes through libart.so
on the caller's current HIP stream."""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import CrossingBuf, SegmentOut, check
from .raytracer import Params

F64 = torch.float64


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class Engine:
    def __init__(self, params: Params, device: int | None = None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.ArtError("no GPU visible: the engine has no CPU fallback")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        torch.cuda.set_device(self.device)
        check(self.lib.art_set_device(self.device.index))
        self.params = params
        self.cp = params.to_c()

    def empty(self, *shape, dtype=F64):
        return torch.empty(*shape, dtype=dtype, device=self.device)

    # ---- conversion-surface sampler (RayTracer.jl:1480-1653, MainRunner.jl:463-529)
    def sample(self, n: int, seed: int = 1769, ray_offset: int = 0, max_r=None) -> dict:
        max_r = self.params.max_r() if max_r is None else max_r
        o = {"x": self.empty(3 * n), "k_init": self.empty(3 * n), "erg": self.empty(n), "vifty": self.empty(3 * n),
             "weights": self.empty(n, dtype=torch.int32), "attempts": self.empty(n, dtype=torch.int32)}
        check(self.lib.art_sample_conversion_points_device(
            C.byref(self.cp), float(max_r), int(seed), int(ray_offset), int(n),
            *[_p(o[k]) for k in ("x", "k_init", "erg", "vifty", "weights", "attempts")], _stream()))
        return o

    def forward_roots(self, n: int, seed: int = 1769, ray_offset: int = 0) -> dict:
        """Segment inputs of the forward-tree roots (MainRunner.jl:653-664 -> :179): photons
        at the sampled conversion points, Δω = -1, ln t0 = -30."""
        s = self.sample(n, seed, ray_offset)
        return {"x0": s["x"], "k0": s["k_init"], "erg": s["erg"],
                "dw": torch.full((n,), -1.0, dtype=F64, device=self.device),
                "ln_t0": torch.full((n,), -30.0, dtype=F64, device=self.device),
                "species": torch.ones(n, dtype=torch.int8, device=self.device), "sample": s}

    def alloc_out(self, n: int, capacity: int = 1) -> dict:
        # crossing slots a ray does not fill stay as allocated (include/art.h): NaN here, once
        nan = lambda m: self.empty(m).fill_(float("nan"))  # noqa: E731
        return {"x_end": self.empty(3 * n), "k_end": self.empty(3 * n), "u7_end": self.empty(n),
                "tau_end": self.empty(n), "status": self.empty(n, dtype=torch.int32),
                "n_accept": self.empty(n, dtype=torch.int32), "n_reject": self.empty(n, dtype=torch.int32),
                "n_cross": self.empty(n, dtype=torch.int32), "xc_pos": nan(3 * capacity * n),
                "xc_k": nan(3 * capacity * n), "xc_t": nan(capacity * n),
                "xc_dw": nan(capacity * n), "xc_p": nan(capacity * n), "capacity": capacity}

    # ---- RT.propagate (RayTracer.jl:171-452), asynchronous on the current stream
    def propagate(self, inp: dict, out: dict | None = None, max_crossings: int = -1, capacity: int = 1) -> dict:
        n = inp["erg"].numel()
        out = out or self.alloc_out(n, capacity)
        so = SegmentOut(*[out[k].data_ptr() for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept",
                                                    "n_reject")])
        xb = CrossingBuf(out["capacity"], *[out[k].data_ptr() for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw",
                                                                        "xc_p")])
        check(self.lib.art_propagate_device(
            C.byref(self.cp), n, *[_p(inp[k]) for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")],
            int(max_crossings), C.byref(so), C.byref(xb), _stream()))
        return out

    def set_tail_donation(self, lanes: int) -> None:
        """Tail donation for launches pipelined with others on other streams
        (art_set_tail_donation, include/art.h): a drained wave with <= lanes live rays hands
        them to a continuation launch and retires. Bit-identical results; 0 = off, -1 = the
        library's default by geometry (16 for Schwarzschild batches, else 0)."""
        check(self.lib.art_set_tail_donation(int(lanes)))

    def set_graduation(self, attempts: int) -> None:
        """Graduation of a launch's outlier rays to the one-wave-per-ray tail kernel
        (art_set_graduation, include/art.h): 0 = off (several batches in flight), -1 = the
        default (2048 attempts). Bit-identical results."""
        check(self.lib.art_set_graduation(int(attempts)))

    def set_sampler_waves(self, waves: int) -> None:
        """Waves per SIMD of the sampler (art_set_sampler_waves, include/art.h): 0 = by line
        length (the default), 3 = the 3-wave build for every line (several sampler launches in
        flight). Bit-identical samples."""
        check(self.lib.art_set_sampler_waves(int(waves)))

    def kernel_ms(self) -> float:
        """Duration of the last propagate kernel (HIP events on its stream); synchronizes."""
        check(self.lib.art_synchronize())
        return float(self.lib.art_last_kernel_ms())

    # ---- binned flux (plot/flux.py:38-48)
    def flux_histogram(self, out: dict, species, weights=None, nbins: int = 50, hist=None):
        n = out["status"].numel()
        hist = torch.zeros(2 * nbins, dtype=F64, device=self.device) if hist is None else hist
        check(self.lib.art_flux_histogram_device(C.byref(self.cp), n, _p(out["x_end"]), _p(out["k_end"]),
                                                 _p(out["status"]), _p(species), _p(weights), int(nbins), _p(hist),
                                                 _stream()))
        return hist

    # ---- get_Prob_nonAD (MainRunner.jl:67-124)
    def get_prob_nonad(self, pos, kpos, erg_eff, group_start=None):
        nc = erg_eff.numel()
        out = self.empty(nc)
        ng = nc if group_start is None else group_start.numel() - 1
        check(self.lib.art_get_prob_nonad_device(C.byref(self.cp), nc, _p(pos), _p(kpos), _p(erg_eff), ng,
                                                 _p(group_start), _p(out), _stream()))
        return out

    # ---- per-sample event weight (MainRunner.jl:498-557): 5 x n SoA
    def event_weight(self, sample: dict, max_r=None, rho_DM=0.45, n_maxSample=6):
        n = sample["erg"].numel()
        max_r = self.params.max_r() if max_r is None else max_r
        out = self.empty(5 * n)
        check(self.lib.art_event_weight_device(C.byref(self.cp), float(max_r), float(rho_DM), float(n_maxSample), n,
                                               _p(sample["x"]), _p(sample["k_init"]), _p(sample["vifty"]), _p(out),
                                               _stream()))
        return out.view(5, n)

    # ---- pointwise physics (parity tests)
    def eval_rhs(self, u, tau, erg, species):
        n = tau.numel()
        du = self.empty(7 * n)
        check(self.lib.art_eval_rhs_device(C.byref(self.cp), n, _p(u), _p(tau), _p(erg), _p(species), _p(du),
                                           _stream()))
        return du

    def eval_hamiltonian(self, x, k, T, E):
        n = T.numel()
        H, gx, gk, gT = self.empty(n), self.empty(3 * n), self.empty(3 * n), self.empty(n)
        check(self.lib.art_eval_hamiltonian_device(C.byref(self.cp), n, _p(x), _p(k), _p(T), _p(E), _p(H), _p(gx),
                                                   _p(gk), _p(gT), _stream()))
        return H, gx, gk, gT

    def eval_condition(self, u, tau):
        n = tau.numel()
        c = self.empty(n)
        check(self.lib.art_eval_condition_device(C.byref(self.cp), n, _p(u), _p(tau), _p(c), _stream()))
        return c
