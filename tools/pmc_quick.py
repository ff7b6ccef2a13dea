"""Per-kernel SQ counters per wave from a rocprofv3 --pmc counter_collection.csv (A/B scratch runs).
  python3 tools/pmc_quick.py DIR [DIR ...]   (kernels whose name contains k_prep or k_cand)"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    fs = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(d, "none")
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, a in agg.items():
        w = a.get("SQ_WAVES", 0)
        if not w or not ("k_prep" in k or "k_cand" in k):
            continue
        line = f"{d} {k[:24]:24s} VALU/wave={a['SQ_INSTS_VALU'] / w:8.0f}"
        if "SQ_INSTS_SALU" in a:
            line += f" SALU/wave={a['SQ_INSTS_SALU'] / w:7.0f}"
        if "SQ_THREAD_CYCLES_VALU" in a and a.get("SQ_ACTIVE_INST_VALU"):
            line += f" lane_util={a['SQ_THREAD_CYCLES_VALU'] / a['SQ_ACTIVE_INST_VALU'] / 64:.3f}"
        if "SQ_WAIT_ANY" in a and a.get("SQ_WAVE_CYCLES"):
            line += f" wait={a['SQ_WAIT_ANY'] / a['SQ_WAVE_CYCLES']:.3f} cyc/wave={a['SQ_WAVE_CYCLES'] / w:8.0f}"
        print(line)
