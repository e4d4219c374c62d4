"""The map kernels built with -DSKQ_DEBUG_LDS (make debuglds): the hashing loop's LDS slot counter
clamps at 0 instead of wrapping below LDS address 0 (skq_map1.h lds_slot_next). The results must be
the same, per read, as the oracle's — so the wrapped-store trick of the shipped build is only a
speed choice, and a lane running past row 0 is exercised in both builds (the k = 21 pass)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "ab", "debug_lds", "libskq.so")


def test_debug_lds_build_is_bit_exact():
    assert os.path.exists(DBG), "build it first: make debuglds"
    env = dict(os.environ, SKQ_LIB=DBG)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "_debug_lds_run.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "debug-lds ok" in r.stdout
