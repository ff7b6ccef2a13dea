"""Summarise tools/pmc_stalls.sh's passes into a profiles/ file (default profiles/r06_pmc_stalls.json):
per kernel the SQ counters per dispatch, VALU per wave and wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES,
stamped with the SHA-256 of the library they measured (tools/shape_tags.lib_sha256).
  python3 tools/pmc_stalls_summary.py TAG [OUT]"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from shape_tags import lib_sha256  # noqa: E402

tag = sys.argv[1]
dest = sys.argv[2] if len(sys.argv) > 2 else "profiles/r06_pmc_stalls.json"
out = {"what": "rocprofv3 --pmc SQ_* stall counters per kernel (per dispatch) of the measured build; "
               "wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES, VALU/wave = SQ_INSTS_VALU / SQ_WAVES",
       "lib_sha256": lib_sha256(), "runs": {}}
for c in ("c5", "c3", "c4"):
    fs = glob.glob(f"gpurun_out/{tag}/stall_{c}/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    ks = {}
    for k, a in agg.items():
        if not (k.startswith("k_prep") or k.startswith("k_cand") or k.startswith("k_emit") or k.startswith("k_winner")):
            continue
        n = max(len(disp[k]), 1)
        e = {kk: v / n for kk, v in a.items()}
        if e.get("SQ_WAVES"):
            e["VALU_per_wave"] = e["SQ_INSTS_VALU"] / e["SQ_WAVES"]
        if e.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"]
        ks[k] = e
    out["runs"][c] = {"source": f"gpurun_out/{tag}/stall_{c}", "kernels": ks}
json.dump(out, open(dest, "w"), indent=1)
for c, r in out["runs"].items():
    for k, e in r["kernels"].items():
        print(c, k, round(e.get("VALU_per_wave", 0)), round(e.get("wait_frac", 0), 3))
