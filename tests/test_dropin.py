"""GPU: the reference's own FEC tests (sim_test/fec_test/test_func.c, with the
reference flex_fec_sender.c / flex_fec_receiver.c, unchanged) linked against
librazor_fec.so instead of flex_fec_xor.c print exactly what the reference
prints (tests/golden/ref_fec_test_stdout.txt).  The binary is built in this
container by `make -C oracle dropin` and travels with the repo."""
import os
import subprocess

import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu


def test_reference_tests_linked_to_razor():
    exe = po.REFDIR / "fec_test_on_razor"
    if not exe.exists():
        pytest.skip("oracle/_ref/fec_test_on_razor not built (needs /root/reference at build time)")
    env = dict(os.environ)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout == (po.GOLDEN / "ref_fec_test_stdout.txt").read_text()
