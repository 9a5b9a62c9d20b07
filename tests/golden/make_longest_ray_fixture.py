"""Writes tests/golden/gr_longest_rays.json: the oracle (oracle/, test infrastructure) on
configs[3]'s two longest rays (717277, 913293 of the 1e6-ray GR batch, seed 1769) and on 1-ulp
perturbations of their start positions -- the spread of step attempts, accepted steps and end
point that the reference's arithmetic itself shows for these chaotic rays, against which
tests/test_longest_ray.py reads the GPU's counts for the same rays.
Usage: python3 tests/golden/make_longest_ray_fixture.py"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402

RAYS = (717277, 913293)
CONFIG = dict(theta_m=0.0, mass_a=1e-6, flat=False)  # configs[3]


def oracle_runs(ray, perturb=True):
    """The unperturbed ray, then x, y, z one ulp up and one ulp down (RayTracer.jl:176 solve
    through the oracle's restatement, oracle/art_oracle.cpp)."""
    p = O.make_params(**CONFIG)
    mr = O.find_conversion_surface(p)
    s = O.sample(p, mr, 1769, ray, 1, nthreads=1)
    runs = []
    for k in range(7 if perturb else 1):
        x = s["x"].copy()
        if k:
            c = (k - 1) % 3
            x[c] = np.nextafter(x[c], np.inf if k <= 3 else -np.inf)
        r = O.propagate(p, x, s["k_init"], s["erg"], -1.0, -30.0, 1, max_crossings=-1, nthreads=1)
        runs.append({"perturbed": "none" if k == 0 else f"x[{(k - 1) % 3}] {'+' if k <= 3 else '-'}1 ulp",
                     "attempts": int(r["n_accept"][0] + r["n_reject"][0]), "accepted": int(r["n_accept"][0]),
                     "status": int(r["status"][0]), "x_end": np.asarray(r["x_end"]).reshape(-1).tolist()})
    return runs


if __name__ == "__main__":
    O.build()
    out = {"config": "configs[3] GR (theta_m 0, m_a 1e-6, seed 1769)", "rays": {}}
    for ray in RAYS:
        out["rays"][str(ray)] = oracle_runs(ray)
    with open(os.path.join(HERE, "gr_longest_rays.json"), "w") as f:
        json.dump(out, f, indent=1)
