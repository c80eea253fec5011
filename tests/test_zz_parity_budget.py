"""Runs last (file order): the near-tie escapes of the session's GPU plan comparisons stay rare."""
import pytest

from parity_util import TIES

pytestmark = pytest.mark.gpu


def test_near_tie_escapes_are_rare():
    n = TIES["full"] + TIES["escaped"]
    print(f"plan comparisons: {TIES['full']} full, {TIES['escaped']} near-tie escapes {TIES['where']}")
    if n == 0:
        pytest.skip("no plan comparison ran in this session")
    assert TIES["full"] >= 0.9 * n, f"{TIES['escaped']} of {n} plan comparisons escaped on near ties: {TIES['where']}"
