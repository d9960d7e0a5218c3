"""Sliding-window eval under torch.distributed (utils/eval_utils.py:26-96, trainer.py:161-177,194).

(1) The reference evaluates on rank 0 only while the other ranks wait in dist.barrier(): the default call
must not issue a collective (round 1 sharded whenever a process group existed and deadlocked there).
(2) shard=True (every rank calls) splits the tiles of one image over the ranks and all-gathers them: the
result equals the unsharded one.  Both ranks share cuda:0 over gloo; they are forked from the forkserver
conftest.py starts before any GPU use."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

import _ddp_worker as W

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_eval_rank0_only_and_sharded(tmp_path):
    from multiprocessing import forkserver
    if getattr(forkserver._forkserver, "_forkserver_pid", None) is None:
        pytest.skip("run with -m gpu: the ranks need the forkserver conftest.py starts before GPU init")
    ctx = mp.get_context("forkserver")
    port = _free_port()
    procs = [ctx.Process(target=W.eval_main, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=110)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes                      # a collective in the rank-0-only call would hang here
    from ebc_amd.eval_utils import sliding_window_predict
    m = W.build(torch.device("cuda:0")).eval()
    want = sliding_window_predict(m, torch.from_numpy(W.eval_image()).cuda(), 224, 112).numpy()
    r0 = torch.load(os.path.join(tmp_path, "eval_rank0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "eval_rank1.pt"), weights_only=True)
    np.testing.assert_allclose(r0["rank0_only"].numpy(), want, rtol=1e-5, atol=1e-6)
    for r in (r0, r1):
        np.testing.assert_allclose(r["sharded"].numpy(), want, rtol=1e-5, atol=1e-6)
