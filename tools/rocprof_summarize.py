"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into profiles/rocprof_summary.json
(read by bench.py for roofline.frac_rocprof: the same roofline fraction from the profiler's average
kernel duration instead of the bench's own HIP events).

  python3 tools/rocprof_summarize.py <dir with *kernel_stats.csv> <tag> [launches_per_step]

<tag> is bench.py's launch-shape tag k_cand_S<scenes>_C<cands>_N<points>[_paths][_D<draws>];
launches_per_step is the number of K2 launches per pp_eval call (2 where pp_eval splits a
shard-sized batch over two streams, include/pp.h PP_DBG_SPLIT)."""
import csv
import glob
import json
import os
import sys

from shape_tags import DOMINANT, parse_tag


def main():
    src, tag = sys.argv[1], sys.argv[2]
    per_step = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    files = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"rocprof_summarize: no *kernel_stats.csv under {src}")
    kernels = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row["Name"].split("(")[0].replace("void ", "").strip()
            kernels[name] = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) * 1e-6,
                             "total_ms": float(row["TotalDurationNs"]) * 1e-6}
    dom = {k: v for k, v in kernels.items() if k.startswith(DOMINANT)}
    if not dom:
        raise SystemExit(f"rocprof_summarize: no dominant kernel ({DOMINANT}) in {src}")
    # one K2 launch = one dispatch of each dominant instantiation (k_cand<false>, k_cand<true>)
    calls = max(v["calls"] for v in dom.values())
    dom_ms = sum(v["total_ms"] for v in dom.values()) / calls
    shape = parse_tag(tag)
    shape["candidates_per_launch"] //= per_step
    p = "profiles/rocprof_summary.json"
    out = json.load(open(p)) if os.path.exists(p) else {}
    out[tag] = dict(shape, **{"launches_per_step": per_step, "dominant_ms_per_launch": dom_ms,
                              "dominant_launches": calls, "kernels": kernels,
                              "source": f"rocprofv3 --kernel-trace --stats of bench.py ({src}, summarised into profiles/)"})
    json.dump(out, open(p, "w"), indent=1, sort_keys=True)
    print("wrote", p, tag, f"dominant {dom_ms:.4f} ms per launch")


if __name__ == "__main__":
    main()
