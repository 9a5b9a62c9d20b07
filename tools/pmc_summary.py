"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) into profiles/pmc_summary.json.

HBM bytes per propagate launch = FETCH_SIZE x c_read + WRITE_SIZE x c_write (KB -> B).
The correction factors c come from tools/calib_hbm.hip, a kernel with the engine's own
access width (8 B per lane, coalesced SoA) and a known byte count, measured in the same
session. MI355X_MICROARCH.md calibrates only 16-B/lane streams, where FETCH_SIZE reads
1/2 of the bytes; that variant is also measured, as a cross-check.

    python tools/pmc_summary.py PMC_DIR WORKLOAD_KEY [OUT_JSON]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_counters(pmc_dir):
    """{kernel name: {counter: [per-dispatch values]}} over every pass CSV under pmc_dir."""
    out = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                out[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return out


def pick(counters, prefix):
    for name, c in counters.items():
        if name.startswith(prefix) or prefix in name:
            return name, c
    raise KeyError(prefix)


def main():
    pmc_dir, workload = sys.argv[1], sys.argv[2]
    out_json = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                 "pmc_summary.json")
    truth = json.load(open(os.path.join(pmc_dir, "calib_truth.json")))
    cal = read_counters(os.path.join(pmc_dir, "calib"))
    _, c8 = pick(cal, "copy8")
    _, c16 = pick(cal, "copy16")
    kb = 1024.0
    c_read = truth["copy8_read_bytes"] / (c8["FETCH_SIZE"][0] * kb)
    c_write = truth["copy8_write_bytes"] / (c8["WRITE_SIZE"][0] * kb)
    c16_read = truth["copy16_read_bytes"] / (c16["FETCH_SIZE"][0] * kb)

    k = read_counters(os.path.join(pmc_dir, "kernel"))
    import hashlib
    import re
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adiabatic_raytracer_amd", "lib", "libart.so")

    def summary(name, pc):
        fetch = pc["FETCH_SIZE"][-1] * kb
        write = pc["WRITE_SIZE"][-1] * kb
        return {"kernel": name, "hbm_bytes_per_launch": fetch * c_read + write * c_write,
                "fetch_bytes_raw": fetch, "write_bytes_raw": write,
                "other_counters_per_launch": {c: v[-1] for c, v in pc.items() if c not in ("FETCH_SIZE", "WRITE_SIZE")}}
    # the Vern6 integrator's instantiations: <INTEG, GEOM, SAVE, DON, WPS>; DON = 3 is the
    # maskless streamed host pipeline's (bench.py's headline), DON = 0 the device-resident pass's
    kernels = {}
    for name, pc in k.items():
        m = re.search(r"propagate_kernel<0, \d, false, (\d),", name)
        if m and "FETCH_SIZE" in pc and "WRITE_SIZE" in pc:
            kernels[{"3": "streamed", "0": "device"}.get(m.group(1), "don" + m.group(1))] = summary(name, pc)
    top = kernels.get("streamed") or kernels["device"]
    res = {
        "workload": workload,
        "libart_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None,
        **top,
        "calibration": {"access": "8 B/lane coalesced f64 (tools/calib_hbm.hip copy8)",
                        "read_factor": c_read, "write_factor": c_write,
                        "read_factor_16B_per_lane": c16_read},
        "kernels": kernels,
    }
    os.makedirs(os.path.dirname(os.path.abspath(out_json)), exist_ok=True)
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
