#!/bin/bash
# Dev: interleaved 1e7 flat kernel timings of the current build and the given variants, plus
# the lone tail rays.
cd "$GRAFT_REPO_ROOT" || exit 1
REPS=${REPS:-3} bash tools/ab_multi.sh adiabatic_raytracer_amd/lib/libart.so "$@" || exit 1
[ -n "$TAIL" ] && bash tools/gpu_tail_ab.sh "$@"
exit 0
