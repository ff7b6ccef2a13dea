"""Per-region instruction census of k_cand's candidate loop.

Static part: the ISA of a -DPP_CENSUS build (tools/variants.sh census "-DPP_CENSUS", then
`make asm`-style -S output), whose run_candidate regions start with an assembly comment
";@R <output mode> <region>". Every instruction of the kernel belongs to the region of the nearest
marker before it in layout order (out-of-line blocks start with their own marker); instructions
before the first marker or after a region "end" are "other" (phase A, prologue, epilogue).

Dynamic part: how many wave-steps execute each region, from a PP_DIAG run (tools/diag_events.py
JSON: wave_frac per event, wave_steps in total).

  python3 tools/valu_census.py census.s KERNEL_SUBSTRING [diag.json] [--measured VALU_PER_WAVE]

Prints one JSON object: per region its static VALU / SALU / VMEM / LDS counts, the wave-step
fraction that executes it, and VALU per wave-step (static x fraction)."""
import json
import re
import sys

# region -> diag event (tools/diag_events.py NAMES) giving the fraction of wave-steps executing it;
# None: every wave-step (the loop body's straight-line regions)
REGION_EVENT = {"head": None, "seg": "seg_reload", "segback": "seg_back", "eval": None, "dir": None,
                "dirfix": "not_dok", "cross": None, "asin": None, "wide": "wide_turn", "acc": None,
                "lim": "limiter", "ovr": "override", "lim2": "limiter", "adj": "curv_adjust",
                "adjwide": "adjust_wide", "adjn": "adjust_narrow", "sqrtslow": "not_dok", "tail": None, "tailfix": "not_dok", "tail2": None, "out": None,
                "outw": "winner_out", "out2": None, "latch": None}


def classify(op):
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "valu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_endpgm", "s_setprio", "s_sleep")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return None


def kernel_lines(path, sub):
    out, inside = [], False
    for ln in open(path):
        if not inside:
            m = re.match(r"^(_Z\w+):", ln)
            if m and sub in m.group(1):
                inside = True
            continue
        if re.match(r"^\.Lfunc_end\d+:", ln):
            break
        out.append(ln.rstrip("\n"))
    if not out:
        raise SystemExit(f"valu_census: no kernel matching {sub!r} in {path}")
    return out


def blocks(lines):
    """Basic blocks in layout order: [(markers, [instruction classes with the marker count before
    each])]."""
    out, cur = [], None
    for ln in lines:
        if re.match(r"^\.LBB\d+_\d+:", ln) or re.match(r"^; %bb\.\d+:", ln):
            cur = {"marks": [], "ins": []}
            out.append(cur)
            continue
        if cur is None:
            cur = {"marks": [], "ins": []}
            out.append(cur)
        m = re.search(r";@R (\d+) (\w+)", ln)
        if m:
            cur["marks"].append(f"m{m.group(1)}:{m.group(2)}" if m.group(2) != "end" else "other")
            continue
        t = ln.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        c = classify(t.split()[0])
        if c is not None:
            cur["ins"].append((len(cur["marks"]), c))
    return out


def static_counts(lines):
    """Region of an instruction: a block holding markers gives its instructions before the first
    marker to that marker's region (the scheduler hoists work above an assembly comment) and the
    rest to the marker before them; a block without one continues the region of the block laid out
    before it (a join or a compiler-made block of the same source region)."""
    regions = {}
    cur = "other"
    for b in blocks(lines):
        marks = b["marks"]
        for k, c in b["ins"]:
            r = marks[max(k - 1, 0)] if marks else cur
            regions.setdefault(r, {"valu": 0, "salu": 0, "vmem": 0, "lds": 0, "wait": 0})[c] += 1
        if marks:
            cur = marks[-1]
    return regions


def main(argv):
    measured = None
    if "--measured" in argv:
        i = argv.index("--measured")
        measured = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    asm, sub = argv[0], argv[1]
    diag = json.load(open(argv[2])) if len(argv) > 2 else None
    st = static_counts(kernel_lines(asm, sub))
    out = {"kernel": sub, "regions": {}}
    per_step = 0.0
    for r, c in sorted(st.items()):
        name = r.split(":")[-1]
        e = REGION_EVENT.get(name, "n/a") if r != "other" else "n/a"
        frac = None
        if diag is not None and e != "n/a":
            frac = 1.0 if e is None else diag.get(e, {}).get("wave_frac")
        d = dict(c)
        if frac is not None:
            d["wave_step_frac"] = frac
            d["valu_per_wave_step"] = c["valu"] * frac
            per_step += c["valu"] * frac
        out["regions"][r] = d
    if diag is not None:
        steps = diag["wave_steps"] / max(diag.get("waves", 0) or 1, 1) if diag.get("waves") else None
        out["loop_valu_per_wave_step"] = per_step
        out["wave_steps"] = diag["wave_steps"]
        if steps:
            out["wave_steps_per_wave"] = steps
            out["loop_valu_per_wave"] = per_step * steps
            if measured:
                out["measured_valu_per_wave"] = measured
                out["outside_loop_valu_per_wave"] = measured - per_step * steps
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
