"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle (oracle/art_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package -- as the checker, never as the thing measured or shipped. The product
(adiabatic_raytracer_amd) never imports it. Parity status: see art_oracle.cpp header
("parity unpinned" against the Julia reference, which cannot run here).
"""
from .oracle import *  # noqa: F401,F403
