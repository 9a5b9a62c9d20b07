"""Generate the committed golden fixtures from the CPU oracle (oracle/art_oracle.cpp).

The reference (Julia) cannot run here and ships no fixtures, so these vectors pin the GPU
engine to the oracle's restatement on fixed, seeded inputs (seed 1769, the reference's
canonical seed, jonas_test_analyses/runner_tree.sh:1). Regenerate with:
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402

CASES = {
    "segments_flat": dict(theta_m=0.2, mass_a=1e-5, flat=True),   # BASELINE configs[0..2]
    "segments_gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),    # BASELINE configs[3]
}


def make(name, kw, n=256):
    p = O.make_params(**kw)
    maxr = O.find_conversion_surface(p)
    s = O.sample(p, maxr, 1769, 0, n, nthreads=1)
    dw, lnt, sp = -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8)
    r = O.propagate(p, s["x"], s["k_init"], s["erg"], dw, lnt, sp, max_crossings=-1, cap=1, nthreads=1)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"), x0=s["x"], k0=s["k_init"], erg=s["erg"], dw=dw, ln_t0=lnt, species=sp,
        attempts=s["attempts"], weights=s["weights"], max_r=maxr, x_end=r["x_end"], k_end=r["k_end"],
        u7_end=r["u7_end"], tau_end=r["tau_end"], status=r["status"], n_accept=r["n_accept"],
        n_reject=r["n_reject"], n_cross=r["n_cross"], xc_pos=r["xc_pos"], xc_k=r["xc_k"], xc_t=r["xc_t"],
        xc_dw=r["xc_dw"], xc_p=r["xc_p"], **{"params_" + k: v for k, v in kw.items()})


if __name__ == "__main__":
    for name, kw in CASES.items():
        make(name, kw)
        print("wrote", name)
