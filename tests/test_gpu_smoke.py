"""The driver's round-end smoke check (__graft_entry__.smoke) run as a GPU test, so a
broken smoke shows up in `pytest -m gpu` first."""
import pytest

pytestmark = pytest.mark.gpu


def test_graft_entry_smoke():
    import __graft_entry__ as g
    g.smoke()
