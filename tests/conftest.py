import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running parity case")
    config.addinivalue_line("markers", "late: host-side machinery around the kernels (child processes, "
                                       "concurrent callers, streamed files, GiB of temp files); runs after the "
                                       "kernel parity tests so that a failure there under -x does not hide them")
    config.addinivalue_line("markers", "firstrun: kernels that have not yet run on hardware (written while the "
                                       "round's GPU access was closed); run last, after the late tests, so that a "
                                       "fault there under -x cannot hide any test of hardware-validated code")


def pytest_collection_modifyitems(config, items):
    # stable: order otherwise unchanged.  Validated kernels, then host machinery, then
    # kernels on their first hardware run.
    items.sort(key=lambda it: (it.get_closest_marker("firstrun") is not None, it.get_closest_marker("late") is not None))


@pytest.fixture(scope="session")
def oracle_c():
    from oracle import oracle

    return oracle.C()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    import sy_amd.device as dev  # raises if libsydelta.so is missing

    return dev
