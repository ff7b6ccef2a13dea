"""NUM_LANES other than the reference default. The library, the
restatement and the reference are each built a second time with four lanes (PP_NUM_LANES=4 /
NUM_LANES=4; carnd-path-planning-project_amd/Makefile `lanes4`, oracle/Makefile), and the cases in
tests/lanes4_cases.py run against those builds in one child process (a process loads one
PP_NUM_LANES: the C-ABI structs are sized by it)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB4 = os.path.join(REPO, "carnd-path-planning-project_amd", "ppamd", "libppamd_l4.so")
ORACLE4 = os.path.join(REPO, "oracle", "liboracle_l4.so")
REF4 = os.path.join(REPO, "oracle", "_ref", "libppref_l4.so")


def run_cases(marker, timeout):
    for p in (LIB4, ORACLE4):
        assert os.path.exists(p), f"{p} not built (run __graft_entry__.build())"
    env = dict(os.environ, PPAMD_LIB=LIB4, PP_ORACLE_SO=ORACLE4, PP_REF_SO=REF4)
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.join(REPO, "tests", "lanes4_cases.py"),
                        "-x", "-q", "-s", "-m", marker, "-p", "no:cacheprovider"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-3000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-3000:]


def test_four_lane_build_cpu():
    run_cases("not gpu", 600)


@pytest.mark.gpu
def test_four_lane_build_gpu():
    run_cases("gpu", 600)
