"""Pins the build's radiated flux and its event_/final_ text files against the reference's own
post-processing scripts, run unchanged on build-written files (as make_combine_fixture.py does
for Combine_Files.py).

Stage "gpu" (on the GPU box): one trees.main_runner_tree run with saveMode 2 writes the
event_/final_ text files (MainRunner.jl:592-609, 690-702) under <dir>/results/event/, named
with the tag analysis.py reads first ("convergence_1e-10", jonas_test_analyses/analysis.py:35).

Stage "ref" (in the build container only, where /root/reference exists):
  * plot/flux.py runs unchanged (MPLBACKEND=Agg) in a scratch directory whose
    results/combined.npy is tests/golden/combine_py/expected_mode1.npy -- the reference's
    Combine_Files.py output over two build-written 29-column row files. A wrapper records the
    (hist, bin_edges) of every np.histogram call the script makes (flux.py:43-47 first: the
    photon and axion flux over data-dependent bins) and its stdout -> tests/golden/flux_py/;
  * jonas_test_analyses/analysis.py runs unchanged on the stage-"gpu" text files; afterwards
    the wrapper calls the script's own load_event_info / load_final_info (analysis.py:8-33) on
    them and stores the columns they return, and the np.histogram calls the script made
    (analysis.py:91-96) -> tests/golden/analysis_py/ (with the two input files).
Nothing from the reference is copied: the fixtures are data (npy/npz arrays, text files the
build wrote, the scripts' printed output).

    python tests/golden/make_postproc_fixture.py gpu gpurun_out/pp
    python tests/golden/make_postproc_fixture.py ref gpurun_out/pp
"""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src"
TAG = "convergence_1e-10"
KW = dict(theta_m=0.2, mass_a=1e-5, flat=True)
NTAJS = 65
SEED = 1769

# runs a reference script unchanged (runpy, as __main__) with np.histogram recording its calls;
# argv: script, out.npz [, tag: then also the script's load_event_info / load_final_info(tag)]
WRAPPER = r"""
import sys, runpy
import numpy as np
import matplotlib
matplotlib.use("Agg")
script, out = sys.argv[1], sys.argv[2]
calls = []
_hist = np.histogram
def _rec(*a, **k):
    r = _hist(*a, **k)
    calls.append(r)
    return r
np.histogram = _rec
err = ""
try:
    g = runpy.run_path(script, run_name="__main__")
except BaseException as e:  # the script's own failure is part of what it does
    g, err = {}, repr(e)
res = {"error": np.array(err)}
for i, (h, e) in enumerate(calls):
    res[f"hist{i}"], res[f"edges{i}"] = np.asarray(h), np.asarray(e)
if len(sys.argv) > 3:
    ev = g["load_event_info"](sys.argv[3])
    fi = g["load_final_info"](sys.argv[3])
    for name, v in zip(("num", "vIfty", "sln_prob", "x_in", "k_in", "x0", "k0", "time", "nodes"), ev):
        res["event_" + name] = np.asarray(v)
    for name, v in zip(("num", "weight", "species", "theta_f", "phi_f", "abs_f", "theta_Xf", "phi_Xf", "abs_Xf", "t"), fi):
        res["final_" + name] = np.asarray(v)
np.savez(out, **res)
"""


def stage_gpu(d):
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import adiabatic_raytracer_amd as A
    A.trees.main_runner_tree(A.Params(**KW), NTAJS, seed=SEED, saveMode=2, dir_tag=os.path.join(d, "results"),
                             file_tag=TAG)


def run_ref(script, cwd, out, *extra):
    env = dict(os.environ, MPLBACKEND="Agg")
    r = subprocess.run([sys.executable, "-c", WRAPPER, script, out, *extra], cwd=cwd, capture_output=True, text=True,
                       env=env)
    assert r.returncode == 0, r.stderr
    return r.stdout


def stage_ref(d):
    fdir, adir = os.path.join(HERE, "flux_py"), os.path.join(HERE, "analysis_py")
    os.makedirs(fdir, exist_ok=True)
    os.makedirs(adir, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "results"))
        shutil.copyfile(os.path.join(HERE, "combine_py", "expected_mode1.npy"), os.path.join(tmp, "results", "combined.npy"))
        out = run_ref(os.path.join(REF, "plot", "flux.py"), tmp, os.path.join(fdir, "flux_calls.npz"))
        with open(os.path.join(fdir, "flux_stdout.txt"), "w") as fh:
            fh.write(out)
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "results", "event"))
        for kind in ("event_", "final_"):
            src = os.path.join(os.path.abspath(d), "results", "event", kind + TAG)
            shutil.copyfile(src, os.path.join(tmp, "results", "event", kind + TAG))
            shutil.copyfile(src, os.path.join(adir, kind + TAG))
        out = run_ref(os.path.join(REF, "jonas_test_analyses", "analysis.py"), tmp,
                      os.path.join(adir, "analysis_calls.npz"), TAG)
        with open(os.path.join(adir, "analysis_stdout.txt"), "w") as fh:
            fh.write(out)
    print("fixtures in", fdir, sorted(os.listdir(fdir)), adir, sorted(os.listdir(adir)))


if __name__ == "__main__":
    {"gpu": stage_gpu, "ref": stage_ref}[sys.argv[1]](sys.argv[2])
