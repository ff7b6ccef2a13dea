"""bench.py's launch-shape tags and the dominant kernel of a step (shared by pmc_summarize.py and
rocprof_summarize.py)."""
import hashlib
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(REPO, "carnd-path-planning-project_amd", "ppamd", "libppamd.so")


def lib_sha256(path=None):
    """SHA-256 of the product library a profiled run loaded (PPAMD_LIB, else the in-tree build):
    every summary entry carries it, and bench.py uses an entry's counters only for that library."""
    path = path or os.environ.get("PPAMD_LIB") or DEFAULT_LIB
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()

# the dominant kernel of a step: k_cand (both instantiations); the small-batch shapes fuse it
# into k_cand_small / k_step_small
DOMINANT = ("k_cand<", "k_cand_small", "k_step_small")


def parse_tag(tag):
    """Launch shape from a bench tag k_cand_S<scenes>_C<cands>_N<points>[_paths][_D<draws>][_comfort]
    (_comfort: the comfort cost mode, the data-dependent argmin; its kernels differ from the
    reference decision's)."""
    m = re.match(r"k_cand_S(\d+)_C(\d+)_N(\d+)(_paths)?(?:_D(\d+))?(_comfort)?$", tag)
    if not m:
        raise SystemExit(f"tag {tag!r} is not k_cand_S<S>_C<C>_N<N>[_paths][_D<D>][_comfort]")
    S, C, N = int(m.group(1)), int(m.group(2)), int(m.group(3))
    return {"scenes": S, "candidates_per_scene": C, "n_points": N, "emit_paths": bool(m.group(4)),
            "draws": int(m.group(5) or 1), "comfort": bool(m.group(6)), "candidates_per_launch": S * C}
