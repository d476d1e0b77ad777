"""GPU: the fused device path with concurrent pipelines (jx_engine.cpp `pipes_for`, debug option 4):
the launches of one jx_helper_prep_aggregate_device call alternate over P child engines (own stream and
staging) and only their accumulations are ordered. Verdicts, prep messages, aggregate, count and checksum
must equal the oracle's for P = 1..4, with a ragged last launch, with the inputs produced on torch's stream
behind a long kernel (the entry ordering), and with torch reading the outputs without a host sync (the join).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from janus_amd.distributed import P64, P128
from janus_amd.engine import HelperEngine
from janus_amd.vdaf import Prio3
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _batch(v, vk, n, seed):
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    rng = np.random.default_rng(seed)
    meas = rng.integers(0, 1 << v.bits, size=(n, v.length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
    lps[::37, 0] ^= 1  # rejected reports
    return orc, nonces, ps, his, lps


@pytest.mark.parametrize("name,vdaf", [("sumvec", Prio3.sum_vec(8, 100, 10)), ("histogram", Prio3.histogram(64, 8)),
                                       ("sum", Prio3.sum(16))])
def test_pipes_match_oracle(name, vdaf):
    import torch

    vk = bytes(range(7, 23))
    n = 4 * 1024 + 333  # 5 launches of 1,024 (the last one ragged) at 1,024 reports per launch
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=sum(map(ord, name)))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    dev = torch.device("cuda", 0)
    pinned = [torch.from_numpy(np.array(a, copy=True)).pin_memory() for a in (nonces, ps, his, lps)]
    engs = [HelperEngine(vdaf, vk) for _ in range(4)]
    for _e in engs:
        _e.debug(5, 1024)  # 1024 reports per launch
    try:
        for P, eng in zip((1, 2, 3, 4), engs):
            eng.debug(4, P)
            d_in = [torch.empty(t.shape, dtype=torch.uint8, device=dev) for t in pinned]
            d_v = torch.empty(n, dtype=torch.uint8, device=dev)
            d_m = torch.empty((n, 16), dtype=torch.uint8, device=dev)
            torch.cuda._sleep(200_000_000)  # the producer: inputs written behind a long kernel on torch's stream
            for d, h in zip(d_in, pinned):
                d.copy_(h, non_blocking=True)
            for _ in range(2):  # twice: the pipelines' staging is reused across calls
                eng.prep_and_aggregate_device(d_in[0].data_ptr(), d_in[1].data_ptr() if ps.shape[1] else None,
                                              d_in[2].data_ptr(), d_in[3].data_ptr(), n, 0, d_m.data_ptr(),
                                              d_v.data_ptr())
            got_v, got_m = d_v.cpu().numpy(), d_m.cpu().numpy()  # torch's stream, no engine sync
            np.testing.assert_array_equal(got_v, want["verdicts"], err_msg=f"P={P}")
            fin = want["verdicts"] == 0
            if eng.prep_msg_len:
                np.testing.assert_array_equal(got_m[fin, :eng.prep_msg_len], want["prep_msgs"][fin], err_msg=f"P={P}")
            agg, cnt, cs = eng.aggregate_share(0)
            assert cnt == 2 * want["count"], P
            fb = eng.field_bytes
            p = P64 if fb == 8 else P128
            exp = b"".join(((2 * int.from_bytes(want["agg"][i:i + fb], "little")) % p).to_bytes(fb, "little")
                           for i in range(0, len(want["agg"]), fb))
            assert agg == exp, P
            assert cs == bytes(32), P  # every report id twice: the XOR checksum cancels
            eng.timing(True)
            eng.prep_and_aggregate_device(d_in[0].data_ptr(), d_in[1].data_ptr() if ps.shape[1] else None,
                                          d_in[2].data_ptr(), d_in[3].data_ptr(), n, 0, d_m.data_ptr(), d_v.data_ptr())
            kt = eng.timing_read()
            assert kt["xof"]["launches"] == 5 and kt["accumulate"]["launches"] == 5, (P, kt)
    finally:
        for eng in engs:
            eng.close()


@pytest.mark.parametrize("P", [1, 2, 3])
def test_host_path_pipes_match_oracle(P):
    """jx_helper_prep_aggregate (host buffers) over P pipelines: verdicts and prep messages come back once
    for the whole call; aggregate, count and checksum as the oracle's."""
    vdaf = Prio3.sum_vec(8, 100, 10)
    vk = bytes(range(3, 19))
    n = 3 * 1024 + 77
    orc, nonces, ps, his, lps = _batch(vdaf, vk, n, seed=P)
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16)
    eng = HelperEngine(vdaf, vk)
    eng.debug(5, 1024)  # 1024 reports per launch
    with eng:
        eng.debug(4, P)
        v, m = eng.prep_and_aggregate(nonces, ps, his, lps)
        np.testing.assert_array_equal(v, want["verdicts"])
        fin = want["verdicts"] == 0
        np.testing.assert_array_equal(m[fin], want["prep_msgs"][fin])
        assert eng.aggregate_share(0) == (want["agg"], want["count"], want["checksum"])
        # aggregate_share's scratch must not free the host path's output buffer.
        # Call again, after the read, with a larger batch: verdicts, prep messages and the running
        # aggregate (now both calls) still equal the oracle's.
        n2 = n + 1500
        orc2, nonces2, ps2, his2, lps2 = _batch(vdaf, vk, n2, seed=100 + P)
        want2 = orc2.helper_prep_batch(vk, nonces2, ps2, his2, lps2, nthreads=16)
        v2, m2 = eng.prep_and_aggregate(nonces2, ps2, his2, lps2)
        np.testing.assert_array_equal(v2, want2["verdicts"])
        fin2 = want2["verdicts"] == 0
        np.testing.assert_array_equal(m2[fin2], want2["prep_msgs"][fin2])
        agg, cnt, cs = eng.aggregate_share(0)
        both = [(int.from_bytes(want["agg"][i:i + 16], "little") + int.from_bytes(want2["agg"][i:i + 16], "little"))
                % P128 for i in range(0, len(want["agg"]), 16)]
        assert agg == b"".join(x.to_bytes(16, "little") for x in both)
        assert cnt == want["count"] + want2["count"]
        assert cs == bytes(a ^ b for a, b in zip(want["checksum"], want2["checksum"]))
        assert eng.memory()["last_pipelines"] == P
