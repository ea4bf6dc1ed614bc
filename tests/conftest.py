"""Shared fixtures.  `-m gpu` tests need a ROCm GPU and the HIP library (lib/libdxrpt.so); everything
else runs on CPU: the oracle against the reference's golden vectors, the host logic, the C-ABI
export check and the multi-rank (gloo) sharding path."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

LIB_DIR = os.path.join(REPO, "dxrpathtracer_amd", "lib")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP path")


def _ensure_built():
    need = [os.path.join(LIB_DIR, "libdxrpt.so"), os.path.join(LIB_DIR, "libdxrpt_host.so"),
            os.path.join(REPO, "oracle", "_build", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "dxrpathtracer_amd", "csrc")], check=True)
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    _ensure_built()


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def pytest_terminal_summary(terminalreporter):
    """Max relative error of every GPU-vs-oracle parity check run in this session."""
    try:
        from tests._common import PARITY_LOG
    except Exception:
        return
    if not PARITY_LOG:
        return
    terminalreporter.section("parity: max relative error per check (gate 1e-4)")
    for what, err, n in PARITY_LOG:
        terminalreporter.write_line(f"{err:.3e}  {n:8d} px  {what}")
    terminalreporter.write_line(f"overall max {max(e for _, e, _ in PARITY_LOG):.3e} over {len(PARITY_LOG)} checks")
