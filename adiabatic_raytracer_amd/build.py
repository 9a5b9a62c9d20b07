"""Build libart.so (gfx950) in-tree with hipcc: adiabatic_raytracer_amd/lib/libart.so."""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libart.so")
SOURCES = ["art_kernels.hip", "art_capi.cpp", "art_forest.cpp", "art_kernels_nolicm.hip"]
HEADERS = ["art_core.h", "art_internal.h", "art_event.h"]
ARCH = os.environ.get("ART_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=on: FMA fusion within one source expression only ("FMA contraction").
# -amdgpu-use-amdgpu-trackers: AMDGPU's own register-pressure trackers in the machine scheduler:
#   fewer spills of the 256-VGPR integrator and 1% faster (A/B on the 1e7-ray flat batch, round 3).
# art_kernels_nolicm.hip adds -disable-machine-licm (see its header): the helper, the non-flat
#   integrators and the tail kernel spill nothing without MachineLICM's hoisted constants (and the GR
#   ones run 2-3% faster); the flat integrator (art_kernels.hip) runs 3% faster with it.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=on", "-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
# art_kernels.hip (the flat integrator) keeps MachineLICM but lets it sink hoisted instructions back
#   into the loop where they would spill (-sink-insts-to-avoid-spills): 12-18 spilled VGPRs -> 2-6;
#   device launch 83.2-83.5 -> 82.5-83.0 ms, 1e7 host-path call 91.0-91.6 -> 89.5-90.7 ms, three
#   interleaved pairs (profiles/r06t_ab_*_sink.jsonl).
TU_FLAGS = {"art_kernels_nolicm.hip": ["-mllvm", "-disable-machine-licm"],
            "art_kernels.hip": ["-mllvm", "-sink-insts-to-avoid-spills"]}


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: libart.so cannot be built")


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(HERE, "..", "include", "art.h"),
                                                                  os.path.abspath(__file__)]  # (the flags too)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    _compile_link(LIB, (), (), verbose)
    return LIB


def _compile_link(out, defines, extra, verbose=False):
    """Each translation unit compiled on its own (in parallel, its TU_FLAGS added), then linked."""
    obj_dir = os.path.join(os.path.dirname(os.path.abspath(out)), "obj_" + os.path.basename(out))
    os.makedirs(obj_dir, exist_ok=True)
    procs, objs = [], []
    for src in SOURCES:
        obj = os.path.join(obj_dir, src + ".o")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", *FLAGS, *TU_FLAGS.get(src, []), *[f"-D{d}" for d in defines],
               *extra, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    bad = [p.args for p in procs if p.wait() != 0]
    if bad:
        raise subprocess.CalledProcessError(1, bad[0])
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    shutil.rmtree(obj_dir, ignore_errors=True)


def build_variant(out, defines=(), extra=()):
    """Dev builds (tools/gpu_final.sh: the section-timing one): the same sources with extra -D defines / flags into
    `out` (e.g. tools/build/libart_x.so, loaded with ART_LIB)."""
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    _compile_link(out, defines, extra)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":  # --variant OUT [-DNAME ...]
        print(build_variant(sys.argv[2], [a[2:] for a in sys.argv[3:] if a.startswith("-D")],
                            [a for a in sys.argv[3:] if not a.startswith("-D")]))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
