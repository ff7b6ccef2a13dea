"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) into per-kernel per-launch averages and write
profiles/pmc_summary.json (read by bench.py for roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads (x2 applied); WRITE_SIZE is exact for 16-B/lane streaming stores.
Both counters are in KiB.

  python3 tools/pmc_summarize.py <dir> <tag> [parts]

parts: the dispatches of each kernel per pp_eval call (a split batch launches every kernel once per
part: 2 or 3 for a shard, 6 for BASELINE config 5's two chunks of 3 parts since round 6). The
profiler reports counters per dispatch; a call's figures are the per-dispatch average x parts."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

from shape_tags import DOMINANT, lib_sha256, parse_tag

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
tag = sys.argv[2] if len(sys.argv) > 2 else None
nparts = int(sys.argv[3]) if len(sys.argv) > 3 else 1
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "").split("(")[0].replace("void ", "").strip()
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
summary = {}
for k, d in vals.items():
    # rocprofv3 reports one row per dispatch per counter (already summed over XCDs/SEs)
    summary[k] = {c: sum(v) / len(v) * nparts for c, v in d.items()}
print(json.dumps(summary, indent=1))


STEP_KERNELS = ("k_prep", "k_prep_g2", "k_prep_g4", "k_prep_g8", "k_prep_g16", "k_cand", "k_cand_small",
                "k_step_small", "k_emit", "k_winner", "k_winner_st")
if tag:
    shape = parse_tag(tag)
    parts = [v for k, v in summary.items() if k.startswith(DOMINANT)]
    kc = {c: sum(p.get(c, 0.0) for p in parts) for c in set().union(*parts)} if parts else {}
    out = {}
    p = "profiles/pmc_summary.json"
    if os.path.exists(p):
        out = json.load(open(p))
    fetch = kc.get("FETCH_SIZE")
    write = kc.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        # every kernel of one evaluation: the step's whole HBM traffic, beside the dominant kernel's
        per_kernel = {k: (2 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)) * 1024.0
                      for k, v in summary.items() if k.split("<")[0] in STEP_KERNELS}
        out[tag] = dict(shape, **{
            "kernels": sorted(k for k in summary if k.startswith(DOMINANT)),
            "hbm_bytes_per_launch": (2 * fetch + write) * 1024.0,
            "pipeline_bytes_per_step": sum(per_kernel.values()),
            "pipeline_bytes_by_kernel": per_kernel,
            "fetch_kib_raw": fetch, "write_kib": write, "parts": nparts,
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py ({src}, summarised into profiles/); FETCH_SIZE x2 (gfx950), dominant-kernel instantiations summed, per-dispatch averages x {nparts} dispatches per call",
            "counters": kc, "lib_sha256": lib_sha256()})
        json.dump(out, open(p, "w"), indent=1)
        print("wrote", p, tag)
