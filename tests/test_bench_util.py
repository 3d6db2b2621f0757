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
        assert bench._counters_of(c, "solve_team_kernel<4, 1>") is None
    assert bench._counters_of(None, "solve_group_kernel<128, 96>") is None


class _StubPlan:
    def __init__(self, names):
        self.names = names

    def solve_kernels(self, B):
        return list(self.names)


def _batch(n_light, n_heavy, N=16, n_mid=0):
    import numpy as np
    c = np.zeros((n_light + n_mid + n_heavy, 4, N), np.uint8)
    c[:n_light, :, :10] = 1          # 40 stance legs: 120 free forces (NC 128 bin)
    c[n_light:n_light + n_mid, :, :13] = 1  # 52 stance legs: 156 free forces (NC 160 bin)
    c[n_light + n_mid:] = 1          # 64 stance legs: 192 free forces (NC 192 bin)
    return c, np.full(n_light + n_mid + n_heavy, 8, np.int32)


def test_bins_and_kernels():
    """Five bins (NC 96 / 128 / 144 / 160 / 192) map onto the three solve kernels."""
    import numpy as np
    contact, _ = _batch(3, 2, n_mid=4)
    bins = bench.bins_of(contact)
    assert bins.tolist() == [1, 1, 1, 3, 3, 3, 3, 4, 4]
    assert bench.kernel_of_bins(np.arange(5)).tolist() == [0, 0, 1, 1, 2]


def test_roofline_dominant_and_critical_kernels():
    """Three kernels: the dominant one processes the most solves, the critical one has the
    longest live time (it sets the step); the HBM fraction is algorithmic bytes / live time."""
    contact, iters = _batch(900, 100, n_mid=50)
    bins = bench.bins_of(contact)
    plan = _StubPlan(["solve_group_kernel<128, 96, false>", "solve_group_kernel<160, 144, false>",
                      "solve_group_kernel<192, 0, false>"])
    roof, comp, crit = bench.kernel_roofline(plan, 1050, bins, contact, iters, [9.0, 4.0, 12.0],
                                             [1, 1, 1], step_ms=12.5)
    assert roof["kernel"].startswith("solve_group_kernel<128") and roof["solves_per_launch"] == 900
    assert crit["kernel"].startswith("solve_group_kernel<192") and crit["solves_per_launch"] == 100
    assert roof["solves_per_kernel"]["solve_group_kernel<160, 144, false>"] == 50
    assert not crit["same_as_dominant"] and abs(crit["step_share"] - 12.0 / 12.5) < 1e-12
    assert abs(roof["achieved"] - bench.BYTES_PER_SOLVE * 900 / 9e-3 / 1e9) < 1e-9
    assert abs(crit["frac"] - bench.BYTES_PER_SOLVE * 100 / 12e-3 / 1e9 / bench.HBM_PEAK_GBS) < 1e-12
    assert comp["kernel"] == roof["kernel"] and crit["compute"]["kernel"] == crit["kernel"]


def test_roofline_single_kernel():
    """One solve kernel for every bin (pair kernel): dominant == critical, all solves counted."""
    contact, iters = _batch(900, 100)
    plan = _StubPlan(["solve_pair_kernel<false>", None, None])
    roof, comp, crit = bench.kernel_roofline(plan, 1000, bench.bins_of(contact), contact, iters,
                                             [10.0, 0.0, 0.0], [2, 0, 0], step_ms=5.2)
    assert roof["kernel"] == crit["kernel"] == "solve_pair_kernel<false>"
    assert roof["solves_per_launch"] == 1000 and roof["kernel_avg_ms"] == 5.0
    assert crit["same_as_dominant"] and list(roof["kernel_avg_ms_all"]) == ["solve_pair_kernel<false>"]
