"""vgan.gcscope.gc_frozen: the objects alive at entry sit in the permanent
generation for the body (nested scopes freeze once) and are handed back on
exit; vgan.affinity's cpulist parser."""
import gc

from vgan.affinity import _parse_cpulist
from vgan.gcscope import gc_frozen


def test_gc_frozen_nests_and_restores():
    keep = [[i] for i in range(1000)]  # tracked containers alive at entry
    gc.unfreeze()
    assert gc.get_freeze_count() == 0
    with gc_frozen():
        n = gc.get_freeze_count()
        assert n >= len(keep)
        with gc_frozen():
            assert gc.get_freeze_count() == n  # the inner scope does not refreeze
        assert gc.get_freeze_count() == n  # ... nor unfreeze the outer one's objects
    assert gc.get_freeze_count() == 0
    try:
        with gc_frozen():
            raise KeyError
    except KeyError:
        pass
    assert gc.get_freeze_count() == 0
    del keep


def test_parse_cpulist():
    assert _parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert _parse_cpulist("") == set()
