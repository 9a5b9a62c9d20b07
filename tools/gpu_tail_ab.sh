#!/bin/bash
# Dev: lone-ray latency (µs per attempt) of the GR tail ray and the scan-point-6 tail ray, for
# the current build and the libraries given as arguments.
cd "$GRAFT_REPO_ROOT" || exit 1
P6='{"mass_a": 1e-6, "B0": 2e14, "omega_pul": 12.566370614359172, "theta_m": 0.2, "flat": true}'
for lib in adiabatic_raytracer_amd/lib/libart.so "$@"; do
  echo "== $lib"
  ART_LIB=$lib timeout -k 10 100 python3 tools/exp_gr_tail.py 1 717277 2>&1 | grep -v amdgpu.ids || exit 1
  ART_LIB=$lib TAIL_KW="$P6" timeout -k 10 100 python3 tools/exp_gr_tail.py 1 14856 2>&1 | grep -v amdgpu.ids || exit 1
done
