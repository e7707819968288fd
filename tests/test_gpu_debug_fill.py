"""Uninitialised device memory: the library run with every new buffer filled with a fixed byte
(PTX_AB=DEBUG_FILL, read once per process -- hence a child process, tests/fill_check.py) must
still render bit-exact frames.  0xFF makes every uninitialised word a NaN / all-ones index
(the spatial combine's folded job step once read such a word as a pending ray index); 0x00
the opposite extreme."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("byte", [255, 0])
def test_frames_bit_exact_over_filled_buffers(byte):
    env = dict(os.environ, PTX_AB=f"DEBUG_FILL={byte}")
    p = subprocess.run([sys.executable, os.path.join(HERE, "fill_check.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), (p.stdout[-2000:], p.stderr[-2000:])
