"""bench.py helpers that need no GPU: PMC records are found by the bench's kernel label whether
rocprof's demangled name carries the interior-point template flag or not."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import bench  # noqa: E402


def test_counters_lookup_ignores_template_flag():
    rec_a, rec_b = {"SQ_INSTS_MFMA": 1.0}, {"SQ_INSTS_MFMA": 2.0}
    new = {"void cmpc::solve_group_kernel<192, 160, false>": rec_b,
           "void cmpc::solve_group_kernel<128, 96, false>": rec_a}
    old = {"void cmpc::solve_group_kernel<192, 160>": rec_b,
           "void cmpc::solve_group_kernel<128, 96>": rec_a}
    for c in (new, old):
        assert bench._counters_of(c, "solve_group_kernel<128, 96>") is rec_a
        assert bench._counters_of(c, "solve_group_kernel<192, 160>") is rec_b
        assert bench._counters_of(c, "solve_team_kernel<4>") is None
    assert bench._counters_of(None, "solve_group_kernel<128, 96>") is None
