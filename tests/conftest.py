"""Shared pytest setup.

Markers:
  gpu   needs a real MI355X (run with -m gpu on the GPU box); everything else
        runs on the CPU container (oracle, host state machines, host-compiled
        engine logic, C-ABI load/symbol checks, gloo multi-process tests).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "open_spiel-1_amd")
TESTS = os.path.join(ROOT, "tests")
for p in (PKG, TESTS):
  if p not in sys.path:
    sys.path.insert(0, p)


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP kernels)")
  config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
  need = [os.path.join(ROOT, "oracle", "build", "liboracle.so"),
          os.path.join(ROOT, "tests", "hostcheck", "build", "libhostcheck.so"),
          os.path.join(PKG, "os_amd", "libos_mcts.so")]
  if all(os.path.exists(p) for p in need):
    return
  for d in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "hostcheck"),
            os.path.join(PKG, "csrc")):
    subprocess.check_call(["make", "-s", "-j8", "-C", d])


_ensure_built()


def gpu_available():
  try:
    import torch
    return torch.cuda.is_available()
  except Exception:  # pragma: no cover
    return False


@pytest.fixture(scope="session")
def require_gpu():
  if not gpu_available():
    pytest.fail("GPU test selected but no GPU is visible")
