"""CPU checks of the C++ host's argument handling (dxrpathtracer_amd/lib/dxrpt_render): bad arguments fail
before any GPU call, with a message and exit status 1."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "dxrpathtracer_amd", "lib", "dxrpt_render")


@pytest.mark.parametrize("args,msg", [(["--bogus"], "unknown option"), (["--scene", "nope"], "unknown scene"),
                                      (["--world", "2", "--rank", "0"], "--uid-file"),
                                      (["--world", "2", "--rank", "2", "--uid-file", "x"], "--rank < N"),
                                      (["--path-length", "9"], "--path-length 2..8"), (["--width"], "missing value")])
def test_cli_rejects_bad_arguments(args, msg):
    if not os.path.exists(CLI):
        pytest.skip("dxrpt_render not built (make -C dxrpathtracer_amd/csrc)")
    p = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and msg in p.stderr, (p.returncode, p.stderr)
