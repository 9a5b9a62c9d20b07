"""Per-kernel PMC table from rocprofv3 --pmc passes (one directory per pass under DIR): for each
kernel whose name matches REGEX, every counter's value in each dispatch, and a few derived
ratios. Usage: python tools/pmc_table.py DIR REGEX [OUT_JSON]"""
import json
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import read_counters  # noqa: E402


def derived(c):
    d = {}
    g = lambda k: c.get(k)  # noqa: E731
    if g("SQ_INSTS_VALU") and g("SQ_INSTS_VALU_FMA_F64") is not None:
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        d["fp64_share_of_valu"] = f64 / g("SQ_INSTS_VALU")
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if g(k) is not None:
                d[k.lower() + "_per_wave_cycle"] = g(k) / g("SQ_WAVE_CYCLES")
    return d


def main():
    root, rx = sys.argv[1], re.compile(sys.argv[2])
    k = read_counters(root)
    res = {}
    for name, pc in k.items():
        if not rx.search(name):
            continue
        nd = max(len(v) for v in pc.values())
        per = [{c: v[i] for c, v in pc.items() if i < len(v)} for i in range(nd)]
        res[name] = {"dispatches": nd, "per_dispatch": per, "derived_last": derived(per[-1])}
    out = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(out)
    print(out)


if __name__ == "__main__":
    main()
