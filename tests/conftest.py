import os
import sys

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (REPO, os.path.join(REPO, "clip-ebc_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")
BINS = [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (3.0, 3.0), (4.0, float("inf"))]
ANCHORS_NWPU = [0.0, 1.0, 2.0, 3.0, 4.21931]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libebc_hip.so")
    mexpr = config.getoption("markexpr", "") or ""
    if "gpu" in mexpr and "not gpu" not in mexpr:
        # Multi-process GPU tests (test_gpu_ddp.py) start their ranks from a forkserver launched NOW, before
        # this process touches the GPU: a process that has initialised HIP must never exec (the ranks are
        # forked from the server, which never initialises HIP).  PYTHONPATH lets the server import the
        # rank bodies.
        import multiprocessing as mp
        from multiprocessing import forkserver
        here = os.path.dirname(os.path.abspath(__file__))
        os.environ["PYTHONPATH"] = os.pathsep.join([here, REPO, os.path.join(REPO, "clip-ebc_amd")] +
                                                   [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
        mp.get_context("forkserver")
        forkserver.ensure_running()


def golden(name: str):
    return np.load(os.path.join(GOLDEN, name))


def _np(a):
    if hasattr(a, "detach"):                      # torch tensors (any device, grad or not)
        a = a.detach().float().cpu().numpy() if a.dtype.is_floating_point and a.dtype.itemsize < 4 else a.detach().cpu().numpy()
    return np.asarray(a, np.float64)


def rel_l2(a, b) -> float:
    a = _np(a); b = _np(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def rel_max(a, b) -> float:
    a = _np(a); b = _np(b)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def split_points(d):
    offs = d["offsets"]; pts = d["points"]
    return [pts[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
