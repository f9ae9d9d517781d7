"""The ctx's own stream is a blocking stream (include/ewal.h,
ewal_ctx_set_stream): device inputs a caller writes on the legacy default
stream (torch's default stream) right before a call are complete when the
call's kernels read them.  With a non-blocking ctx stream the kernel below
starts while the default stream is still busy and reads the zeroed records
(bench.py's N=2 rehearsal caught exactly that in its commit sub-line).
Reference for the computation: raft/raft.go:248-258, raft/log.go:148-154."""
import ctypes as C

import numpy as np
import pytest

from etcd_amd import _lib as L
from etcd_amd import raftcommit as RC

pytestmark = pytest.mark.gpu


def test_ctx_kernels_wait_for_default_stream_writes(ctx):
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(31)
    G = 1 << 18
    nv = np.where(rng.random(G) < 0.5, 5, 7).astype(np.uint8)
    committed = rng.integers(0, 1 << 20, size=G, dtype=np.uint64)
    match = (committed[None, :] + rng.integers(0, 12, size=(7, G), dtype=np.uint64)).astype(np.uint64)
    term = np.ones(G, np.uint64)
    log_offset = committed.copy()
    ptr = (np.arange(G + 1, dtype=np.uint64) * np.uint64(16))
    lt = np.ones(G * 16, np.uint64)
    rec = RC.pack_groups(match, nv, committed, term, log_offset, ptr, lt).reshape(-1).view(np.int64)
    host = torch.from_numpy(rec).pin_memory()
    d_rec = torch.empty(host.numel(), dtype=torch.int64, device=dev)
    d_ptr = torch.from_numpy(ptr.view(np.int64)).to(dev)
    d_lt = torch.from_numpy(lt.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    P = lambda t: C.c_void_p(t.data_ptr())   # noqa: E731
    outs = []
    for racing in (False, True):
        co = torch.zeros(G, dtype=torch.int64, device=dev)
        ch = torch.zeros(G, dtype=torch.uint8, device=dev)
        st = torch.zeros(G, dtype=torch.uint8, device=dev)
        d_rec.zero_()
        if racing:
            busy = torch.empty(1 << 27, dtype=torch.float32, device=dev)   # keep stream 0 busy for a few ms
            for _ in range(16):
                busy.add_(1.0)
        else:
            torch.cuda.synchronize()
        d_rec.copy_(host, non_blocking=True)   # on stream 0, behind the busy work
        if not racing:
            torch.cuda.synchronize()
        assert L.lib.ecommit_batch_rec_device(ctx.handle, G, P(d_rec), P(d_ptr), P(d_lt), P(co), P(ch), P(st), None) == 0
        outs.append((co.cpu().numpy(), ch.cpu().numpy(), st.cpu().numpy()))
    (co0, ch0, st0), (co1, ch1, st1) = outs
    assert ch0.sum() > G // 4 and not st0.any()
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(ch1, ch0)
    np.testing.assert_array_equal(co1, co0)
