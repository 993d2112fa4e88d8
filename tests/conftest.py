import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
sys.path.insert(0, ROOT)

import pytest  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblrl.so on cuda:0)")
    config.addinivalue_line("markers", "multiproc: spawns several processes (ranks); collected after every other test")


def pytest_collection_modifyitems(session, config, items):
    """The multi-process rehearsals run last: under -x a failure in one of them must not hide the single-process
    parity record (the 8-rank test aborted at test 10 of 150 and blanked the rest)."""
    def ranks(it):  # among the rehearsals, fewer ranks first (the 8-rank one last)
        cs = getattr(it, "callspec", None)
        return cs.params.get("world", 2) if cs is not None else 2
    multi = [it for it in items if it.get_closest_marker("multiproc") is not None]
    items[:] = [it for it in items if it.get_closest_marker("multiproc") is None] + sorted(multi, key=ranks)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
