"""CPU tests of the close-call margin gate (tests/margin_gate.py) that the bf16 / fp8 parity cases use."""
import pytest

from margin_gate import assert_diverges_only_at_close_calls as gate

GAP = 2.0


def test_identical_passes():
    exp = list(range(10))
    assert gate(list(exp), exp, [5.0] * 10, GAP, 4) == 10


def test_divergence_on_confident_step_fails():
    exp = list(range(10))
    got = exp[:5] + [99] + exp[6:]
    with pytest.raises(AssertionError, match="margin"):
        gate(got, exp, [5.0] * 10, GAP, 4)


def test_divergence_at_step0_is_vacuous():
    exp = list(range(10))
    margins = [0.5] + [5.0] * 9
    with pytest.raises(AssertionError, match="confident"):
        gate([99] + exp[1:], exp, margins, GAP, 4)


def test_close_call_after_confident_prefix_passes():
    # 4 confident tokens, two close calls, flip at token 6 (the round-3 large-v3-2L case)
    exp = list(range(12))
    margins = [5.0, 5.0, 5.0, 5.0, 1.1, 0.5, 0.3] + [5.0] * 5
    got = exp[:6] + [99] + exp[7:]
    assert gate(got, exp, margins, GAP, 4) == 6


def test_long_prefix_of_close_calls_passes():
    # 12 identical tokens, only 3 of them confident, flip of a 0.1-nat call at token 12
    exp = list(range(20))
    margins = [1.3, 0.6, 0.1, 0.1, 1.5, 2.5, 3.0, 0.4, 2.9, 0.2, 1.9, 1.0, 0.1] + [5.0] * 7
    got = exp[:12] + [99] + exp[13:]
    assert gate(got, exp, margins, GAP, 4) == 12


def test_short_prefix_of_close_calls_fails():
    exp = list(range(20))
    margins = [1.3, 0.6, 3.0, 0.1, 0.2] + [5.0] * 15
    got = exp[:4] + [99] + exp[5:]
    with pytest.raises(AssertionError, match="confident"):
        gate(got, exp, margins, GAP, 4)


def test_run_ending_early_on_close_call():
    exp = list(range(10))
    margins = [5.0] * 8 + [0.5, 5.0]
    assert gate(exp[:8], exp, margins, GAP, 4) == 8
