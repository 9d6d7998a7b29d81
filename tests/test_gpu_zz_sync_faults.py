"""Runs after the other GPU tests (file order): no device-wide barrier of the
fused class-side launches timed out anywhere in the suite (pfsgnn_sync_faults;
a time-out also traps its launch, so a failing count here means a launch was
abandoned without the process dying)."""
import pytest

pytestmark = pytest.mark.gpu


def test_no_barrier_timed_out_in_the_suite():
    from pfsgnn import native
    assert native.sync_faults() == 0
