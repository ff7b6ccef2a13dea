"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into profiles/rocprof_summary.json
(read by bench.py for roofline.frac_rocprof: the same roofline fraction from the profiler's average
kernel duration instead of the bench's own HIP events).

  python3 tools/rocprof_summarize.py <dir with *kernel_stats.csv> <tag> [parts [chunks]]

<tag> is bench.py's launch-shape tag k_cand_S<scenes>_C<cands>_N<points>[_paths][_D<draws>];
parts is the number of streams pp_eval splits the batch over (include/pp.h PP_DBG_SPLIT): their K2
launches overlap, so the K2 time of a call is the span from the first of its k_cand dispatches'
start to the last one's end, read from the kernel trace (run_kernel_trace.csv), as pp_timing_read
reports it; parts = 1 takes the profiler's per-dispatch averages. chunks (round 6): a call runs as
that many sequential chunks of `parts` parts (batches beyond 1,572,864 scenes), and its K2 time is
the sum of the chunks' spans."""
import csv
import glob
import json
import os
import sys

from shape_tags import DOMINANT, lib_sha256, parse_tag


def main():
    src, tag = sys.argv[1], sys.argv[2]
    parts = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 1
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
    how = "per-dispatch averages"
    if parts > 1:
        # the dominant dispatches in launch order, 2 per part (k_cand<false>, k_cand<true>) per call
        tr = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
        if not tr:
            raise SystemExit(f"rocprof_summarize: parts > 1 needs the kernel trace under {src}")
        rows = [r for r in csv.DictReader(open(tr[0]))
                if r["Kernel_Name"].split("(")[0].replace("void ", "").strip().startswith(DOMINANT)]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        per = 2 * parts
        spans = []
        for c0 in range(0, len(rows) - per * chunks + 1, per * chunks):
            tot = 0.0
            for k in range(chunks):
                grp = rows[c0 + k * per:c0 + (k + 1) * per]
                tot += (max(int(r["End_Timestamp"]) for r in grp) - min(int(r["Start_Timestamp"]) for r in grp)) * 1e-6
            spans.append(tot)
        if not spans:
            raise SystemExit("rocprof_summarize: no complete call in the kernel trace")
        # the median call: the first call's parts load the code object one after the other
        dom_ms = sorted(spans)[len(spans) // 2]
        calls = len(spans)
        how = (f"median span of a call's {per} k_cand dispatches ({parts} overlapping parts), kernel trace"
               if chunks == 1 else
               f"median over calls of the summed spans of {chunks} sequential chunks of {per} k_cand dispatches "
               f"({parts} overlapping parts each), kernel trace")
    shape = parse_tag(tag)
    p = "profiles/rocprof_summary.json"
    out = json.load(open(p)) if os.path.exists(p) else {}
    out[tag] = dict(shape, **{"launches_per_step": 1, "parts": parts, "chunks": chunks, "dominant_ms_per_launch": dom_ms,
                              "dominant_launches": calls, "dominant_time": how, "kernels": kernels,
                              "source": f"rocprofv3 --kernel-trace --stats of bench.py ({src}, summarised into profiles/)",
                              "lib_sha256": lib_sha256()})
    json.dump(out, open(p, "w"), indent=1, sort_keys=True)
    print("wrote", p, tag, f"dominant {dom_ms:.4f} ms per launch")


if __name__ == "__main__":
    main()
