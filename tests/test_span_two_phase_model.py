"""CPU model of the two-phase span row kernels (k_span_plan / k_span_write) against the
sequential T5Data::put_data loop the oracle restates, on random rows and draw sequences --
default-like, tiny gaps (more passes than the plan holds), gaps and sizes past the row.
The device kernels are checked against the C oracle in tests/test_gpu_span.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "sim"))
import span_two_phase_sim as sim  # noqa: E402


def test_two_phase_model_equals_sequential_rows():
    checked, overflow = sim.run(trials=3000, seed=7)
    assert checked > 2000 and overflow > 100  # both branches exercised


def test_rows_within_the_label_width_fit_the_plan():
    # every pass but the last writes >= 2 labels, so a row without label overflow has at most
    # LW // 2 + 1 passes: gap 0 / size 1 is the most passes a valid row can hold
    for S in (8, 64, 512):
        LW = S // 4
        n = S
        draws = lambda p: (0, 1)  # noqa: E731
        want = sim.sequential(list(range(1, n + 1)), n, S, LW, draws)
        got = sim.plan(n, S, LW, draws, LW // 2 + 2)
        assert want[2] > 0 and got is None  # this many passes overflow the labels
