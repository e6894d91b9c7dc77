"""bench.py's host-side helpers (no GPU): the positions the timed decode steps take, and the
correctness fields that invalidate a bench line (a false one fails the run)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)      # no GPU work at import (main() is behind __name__)
    return mod


@pytest.mark.parametrize("steps", [1, 20, 96, 495, 496])
def test_spread_positions_cover_the_window(bench, steps):
    pos = [bench.spread_pos(i, steps, 512) for i in range(steps)]
    assert pos[0] == 16 and all(16 <= p <= 511 for p in pos)
    assert pos == sorted(pos) and len(set(pos)) == steps      # distinct, in order
    if steps > 1:
        assert pos[-1] >= 511 - 496 // steps                  # reaches the end of the window


def test_spread_positions_wrap_past_the_window(bench):
    pos = [bench.spread_pos(i, 600, 512) for i in range(600)]
    assert pos[:496] == list(range(16, 512)) and pos[496] == 16


def test_collect_checks_passes_when_every_check_holds(bench):
    out = {"decode_greedy_device": {"stream_check": {"digests_equal": True}, "chained": {"tokens_match_eval_greedy": True}},
           "decode_13b_q4_1": {"stream_check": {"digests_equal": True}}, "decode_65b_q4_0": None,
           "layer_split": None}
    c = bench.collect_checks(out)
    assert c["passed"] and c["failed"] == []


@pytest.mark.parametrize("path,value", [
    (("decode_greedy_device", "stream_check", "digests_equal"), False),
    (("decode_65b_q4_0", "stream_check", "digests_equal"), False),
    (("layer_split", "greedy_check", "forced_steps", "logits_bit_identical_every_step"), False),
    (("layer_split", "greedy_check", "match"), None),            # a check that did not run is not a pass
])
def test_collect_checks_names_every_failure(bench, path, value):
    out = {}
    node = out
    for k in path[:-1]:
        node = node.setdefault(k, {})
    node[path[-1]] = value
    c = bench.collect_checks(out)
    assert not c["passed"] and c["failed"] == [".".join(path)]
