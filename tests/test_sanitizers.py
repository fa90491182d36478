"""Host-side race/memory checks of the native engine: the randomised stress
driver built with ASan+UBSan and with TSan (ThreadPool parallel filter/score)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.parametrize("variant", ["asan-ubsan", "tsan"])
def test_engine_stress_under_sanitizers(variant):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import sanitize
    assert sanitize.run(variant) == 0


@pytest.mark.slow
def test_sniffer_json_under_sanitizers():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import sanitize
    assert sanitize.run_sniffer("asan-ubsan") == 0


@pytest.mark.slow
@pytest.mark.parametrize("variant", ["asan-ubsan", "tsan"])
def test_native_lane_under_sanitizers(variant):
    """Lane thread × transport I/O thread × caller (native/core/lane_stress.cpp) under ASan+UBSan
    and TSan: no race, no leak, exact ledger after every burst and deletion wave."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import sanitize
    assert sanitize.run_lane(variant) == 0
