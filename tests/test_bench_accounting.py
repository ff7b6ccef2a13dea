"""bench.py's roofline accounting (CPU): the PMC counters of a profiled launch are scaled to the
measured launch per candidate, using the launch size the summary records, and every bench line
names the BASELINE config it measures (a config-3 line divided a 262,144-scene launch's
counters by the config-5 launch size)."""
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = json.load(open(os.path.join(REPO, "profiles", "pmc_summary.json")))


def test_every_pmc_entry_states_its_launch():
    for tag, e in PMC.items():
        assert e["candidates_per_launch"] == e["scenes"] * e["candidates_per_scene"], tag
        assert bench.pmc_tag(e["scenes"], e["candidates_per_scene"], e["n_points"], e["emit_paths"],
                             e.get("draws", 1), e.get("comfort", False)) == tag


@pytest.mark.parametrize("tag", [t for t in PMC if PMC[t]["emit_paths"]])
def test_paths_traffic_covers_the_written_paths(tag):
    """All-paths mode writes 16 B per point of every candidate: counted traffic below that is
    impossible, at the profiled size and scaled to any other batch size of the same shape."""
    e = PMC[tag]
    C, N = e["candidates_per_scene"], e["n_points"]
    for S in (e["scenes"], 4096, 1_000_003):
        pmc = bench.pmc_for(PMC, S, C, N, True, 1)
        assert pmc is e
        bpc = bench.algorithmic_bytes_per_candidate(C, N, True)
        traffic, pipe = bench.roofline_fields(pmc, S * C, bpc, 1.0)
        written = 16.0 * N * C * S
        assert traffic >= written, (S, traffic, written)
        assert pipe >= traffic
        # the algorithmic figure and the counters agree within the counted over-fetch (<= 1.3x)
        assert traffic <= 1.3 * bpc * S * C


def test_config5_entry_scales_to_shards():
    """A shard size with its own profiled entry uses it (the 8-GPU shard, 262,144 scenes, round 5);
    another size of the same shape scales the largest profiled launch per candidate."""
    e = PMC["k_cand_S2097152_C15_N50"]
    assert bench.pmc_for(PMC, 262144, 15, 50, False, 1) is PMC.get("k_cand_S262144_C15_N50", e)
    pmc = bench.pmc_for(PMC, 131072, 15, 50, False, 1)      # an unprofiled shard size
    assert pmc is e
    t_full, _ = bench.roofline_fields(pmc, 2097152 * 15, 104.3, 1.0)
    t_shard, _ = bench.roofline_fields(pmc, 131072 * 15, 104.3, 1.0)
    assert t_full == pytest.approx(e["hbm_bytes_per_launch"])
    assert t_shard == pytest.approx(t_full / 16)


def test_unprofiled_shape_has_no_traffic_and_unsized_entry_fails():
    assert bench.pmc_for(PMC, 4096, 9, 50, False, 1) is None
    bad = {"k_cand_S10_C15_N50": {"candidates_per_scene": 15, "n_points": 50, "emit_paths": False,
                                  "hbm_bytes_per_launch": 1.0, "source": "test"}}
    with pytest.raises(ValueError):
        bench.pmc_for(bad, 10, 15, 50, False, 1)


def test_workload_names():
    w = bench.workload_name
    assert w(4096, 15, 5, 50, False, 1, 0) == "BASELINE config 2"
    assert w(262144, 24, 8, 100, True, 1, 0) == "BASELINE config 3"
    assert w(16384, 192, 1, 50, False, 64, 0) == "BASELINE config 4"
    assert w(2097152, 15, 5, 50, False, 1, 0) == "BASELINE config 5"
    assert w(262144, 15, 5, 50, False, 1, 0) == "BASELINE config 5"     # a shard of it
    assert w(65536, 15, 5, 50, False, 1, 100).startswith("closed-loop")


def test_rocprof_summary_entries():
    """profiles/rocprof_summary.json (tools/rocprof_summarize.py): every entry names its launch shape
    and its K2 stages per step (1: a batch split over streams is timed as the span of its parts),
    the candidates of one stage are the shape's, and the recomputed fraction of HBM peak is the one
    a bench line of that shape reports as roofline.frac_rocprof."""
    rp = bench.load_rocprof_all()
    assert rp, "profiles/rocprof_summary.json missing"
    for tag, e in rp.items():
        lps = e["launches_per_step"]
        assert lps in (1, 2, 3, 4), tag
        assert e["candidates_per_launch"] == e["scenes"] * e["candidates_per_scene"] // lps, tag
        assert bench.pmc_tag(e["scenes"], e["candidates_per_scene"], e["n_points"], e["emit_paths"],
                             e.get("draws", 1), e.get("comfort", False)) == tag
        assert 0 < e["dominant_ms_per_launch"] < 100, tag
        bpc = bench.algorithmic_bytes_per_candidate(e["candidates_per_scene"], e["n_points"], e["emit_paths"])
        frac = bpc * e["candidates_per_launch"] / (e["dominant_ms_per_launch"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS
        assert 0 < frac < 1, tag
    # the shard is split in two: its entry says so, and times the two parts as one span
    assert rp["k_cand_S262144_C15_N50"]["parts"] == 2
    assert rp["k_cand_S262144_C15_N50"]["launches_per_step"] == 1


def test_rocprof_summarize_tool(tmp_path):
    """tools/rocprof_summarize.py on a synthetic kernel-stats CSV: the dominant kernel's time per
    launch sums both k_cand instantiations per dispatch, the other kernels are listed."""
    import subprocess
    import sys
    d = tmp_path / "stats" / "host"
    d.mkdir(parents=True)
    rows = ['"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"',
            '"void k_cand<false, 1>(MapG, pp_scene_batch)",26,26000000,1000000.0,70,1,1,0',
            '"void k_cand<true, 1>(MapG, pp_scene_batch)",26,260000,10000.0,1,1,1,0',
            '"void k_prep<true, false>(MapG)",26,5200000,200000.0,20,1,1,0']
    (d / "run_kernel_stats.csv").write_text("\n".join(rows) + "\n")
    # the kernel trace of 3 calls split in 2 parts: part 1 starts 0.1 ms after part 0 and each part's
    # k_cand<false> runs 1 ms, k_cand<true> 0.01 ms after it -> 1.11 ms per call; the first call is
    # slow (3 ms) and the median skips it
    tr = ['"Kernel_Name","Start_Timestamp","End_Timestamp"']
    for c, t0 in enumerate((0, 10_000_000, 20_000_000)):
        stretch = 3 if c == 0 else 1
        for h in range(2):
            a = t0 + h * 100_000 * stretch
            tr.append(f'"void k_cand<false, 1>(MapG, pp_scene_batch)",{a},{a + 1_000_000 * stretch}')
            tr.append(f'"void k_cand<true, 1>(MapG, pp_scene_batch)",{a + 1_000_000 * stretch},{a + 1_010_000 * stretch}')
        tr.append(f'"void k_prep<true, false>(MapG)",{t0 - 300_000},{t0 - 100_000}')
    (d / "run_kernel_trace.csv").write_text("\n".join(tr) + "\n")
    (tmp_path / "profiles").mkdir()
    tool = os.path.join(REPO, "tools", "rocprof_summarize.py")
    r = subprocess.run([sys.executable, tool, str(tmp_path / "stats"), "k_cand_S4096_C15_N50"],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([sys.executable, tool, str(tmp_path / "stats"), "k_cand_S262144_C15_N50", "2"],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    summary = json.load(open(tmp_path / "profiles" / "rocprof_summary.json"))
    one = summary["k_cand_S4096_C15_N50"]
    assert one["dominant_ms_per_launch"] == pytest.approx(1.01) and one["parts"] == 1
    out = summary["k_cand_S262144_C15_N50"]
    assert out["dominant_ms_per_launch"] == pytest.approx(1.11)
    assert out["launches_per_step"] == 1 and out["parts"] == 2 and out["dominant_launches"] == 3
    assert out["candidates_per_launch"] == 262144 * 15
    assert "k_prep<true, false>" in out["kernels"]


def test_profile_entries_need_the_loaded_librarys_stamp():
    """Counters and profiler durations measured on another library build describe another binary:
    bench.py drops traffic, valu_roofline and frac_rocprof unless the entry's lib_sha256 is the
    loaded library's, and records which entries it dropped."""
    sha = "ab" * 32
    pmc = {"candidates_per_launch": 10, "hbm_bytes_per_launch": 1.0, "lib_sha256": sha}
    rp = {"dominant_ms_per_launch": 1.0, "lib_sha256": sha}
    p, r, st = bench.profile_entries(pmc, rp, sha)
    assert p is pmc and r is rp and st["pmc"] == "match" and st["rocprof"] == "match"
    p, r, st = bench.profile_entries(pmc, dict(rp, lib_sha256="cd" * 32), sha)
    assert p is pmc and r is None and st["rocprof"].startswith("stale")
    p, r, st = bench.profile_entries({k: v for k, v in pmc.items() if k != "lib_sha256"}, None, sha)
    assert p is None and r is None and st["pmc"].startswith("stale") and st["rocprof"] is None
    assert bench.roofline_fields(p, 10, 1.0, 1.0) == (None, None)


def test_shard_projection_arithmetic():
    pr = bench.shard_projection(0.010, {2: 0.005, 4: 0.0026, 8: 0.00135})
    assert pr["2"]["speedup"] == pytest.approx(2.0) and pr["2"]["efficiency"] == pytest.approx(1.0)
    assert pr["8"]["speedup"] == pytest.approx(0.010 / 0.00135)
    assert pr["8"]["efficiency"] == pytest.approx(0.010 / 0.00135 / 8)
    assert pr["4"]["shard_ms_per_step"] == pytest.approx(2.6)
    # a shard faster than its share: the one-GPU baseline is the shards in sequence (like with like)
    pr = bench.shard_projection(0.010, {2: 0.0048, 8: 0.0013})
    assert pr["2"]["speedup"] == pytest.approx(2.0) and pr["2"]["efficiency"] <= 1.0
    assert pr["2"]["one_gpu_policy"] == "2 shard calls in sequence"
    assert pr["2"]["speedup_vs_one_call"] == pytest.approx(0.010 / 0.0048)
    assert pr["8"]["speedup"] == pytest.approx(0.010 / 0.0013) and pr["8"]["one_gpu_policy"] == "one call"
    assert all(v["efficiency"] <= 1.0 for v in pr.values())


def test_ppamd_and_tools_hash_the_same_library():
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import shape_tags
    from oracle_lib import ppamd
    assert ppamd.lib_sha256() == shape_tags.lib_sha256(ppamd.LIB_PATH)


def test_committed_summaries_are_stamped():
    """Every committed PMC and kernel-trace summary entry names the library build it measured
    (64 hex digits); bench.py uses an entry only while that build is the loaded one."""
    import re
    for name, d in (("pmc_summary.json", PMC), ("rocprof_summary.json", bench.load_rocprof_all())):
        for tag, e in d.items():
            assert re.fullmatch(r"[0-9a-f]{64}", str(e.get("lib_sha256"))), (name, tag)
