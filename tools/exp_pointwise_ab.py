"""Dev: pointwise RHS / condition of the library named by ART_LIB on fixed random states,
saved for an exact comparison between builds. Usage: ART_LIB=... exp_pointwise_ab.py OUT.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402
from conftest import random_states  # noqa: E402

N = 65536
eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True))
U, tau = random_states(N, seed=3)
dev = lambda a, dt=torch.float64: torch.tensor(np.ascontiguousarray(a), dtype=dt, device="cuda")  # noqa: E731
du = eng.eval_rhs(dev(U.reshape(-1)), dev(tau), dev(np.full(N, 1.0000002692622573e-05)), dev(np.ones(N), torch.int8))
c = eng.eval_condition(dev(U.reshape(-1)), dev(tau))
np.savez(sys.argv[1], du=du.cpu().numpy(), c=c.cpu().numpy())
