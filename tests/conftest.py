import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def scene1():
    from pathtracerdemo_amd.scene.world import compile_scene
    return compile_scene("dummy_scene_1")


@pytest.fixture(scope="session")
def scene3():
    """Config C3: the build-defined many-light interior (scenes/make_c3.py, 32 rect lights)."""
    from pathtracerdemo_amd.scene.world import compile_scene
    return compile_scene("c3_interior_32")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle
