"""Pins the npy layout of the build against the reference's own post-processing.

Stage "gpu" (on the GPU box): two independent runs of trees.main_runner_tree, the way two
reference processes with different --ftag and --seed would run (runner_example.sh:4-7),
write their npy rows (MainRunner.jl:715-761) for saveMode 0 (13 columns) and 1 (29
columns) under <dir>/npy/.

Stage "ref" (in the build container only, where /root/reference exists): the reference's
Combine_Files.py (run unchanged, as a subprocess) combines each pair; the build-produced
inputs and the reference-produced outputs are stored as fixtures in tests/golden/combine_py/.
Nothing from the reference is copied: the fixtures are data (npy arrays).

    python tests/golden/make_combine_fixture.py gpu gpurun_out/pin
    python tests/golden/make_combine_fixture.py ref gpurun_out/pin
"""
import glob
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "combine_py")
REF_SCRIPT = "/root/reference/src/Combine_Files.py"
RUNS = [("pin0", 1769), ("pin1", 1770)]
KW = dict(theta_m=0.2, mass_a=1e-5, flat=True)
NTAJS = 33


def stage_gpu(d):
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import adiabatic_raytracer_amd as A
    for save_mode in (0, 1):
        for tag, seed in RUNS:
            A.trees.main_runner_tree(A.Params(**KW), NTAJS, seed=seed, saveMode=save_mode,
                                     dir_tag=os.path.join(d, f"mode{save_mode}"), file_tag=tag)


def stage_ref(d):
    os.makedirs(OUT, exist_ok=True)
    for save_mode in (0, 1):
        files = sorted(glob.glob(os.path.join(os.path.abspath(d), f"mode{save_mode}", "npy", "tree_*.npy")))
        assert len(files) == 2, files
        ins = []
        for k, f in enumerate(files):
            dst = os.path.join(OUT, f"input_mode{save_mode}_{k}.npy")
            shutil.copyfile(f, dst)
            ins.append(f)
        with tempfile.TemporaryDirectory() as tmp:
            out = os.path.join(tmp, "combined.npy")
            # Combine_Files.py OUT IN... : its argv[2:] are globs, combined in the given order
            r = subprocess.run([sys.executable, REF_SCRIPT, out, *ins], cwd=tmp, capture_output=True, text=True)
            assert r.returncode == 0, r.stderr
            shutil.copyfile(out, os.path.join(OUT, f"expected_mode{save_mode}.npy"))
        with open(os.path.join(OUT, f"names_mode{save_mode}.txt"), "w") as fh:
            fh.write("\n".join(os.path.basename(f) for f in files) + "\n")
    print("fixtures in", OUT, sorted(os.listdir(OUT)))


if __name__ == "__main__":
    {"gpu": stage_gpu, "ref": stage_ref}[sys.argv[1]](sys.argv[2])
