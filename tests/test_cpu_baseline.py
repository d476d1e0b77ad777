"""The CPU baseline engine (cpu_baseline/jc_cpu_engine.cpp, bench.py's cpu_baseline leg) is
byte-exact with the golden fixtures: verdicts, prepare messages, aggregate share, count, checksum."""
import json
import os

import numpy as np
import pytest

from cpu_baseline import cpu_engine as CE

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("threads", [1, 5])
@pytest.mark.parametrize("name", ["sumvec_8x1000_88", "sumvec_small", "histogram_16_4", "histogram_256_16"])
def test_cpu_engine_matches_fixtures(name, threads):
    doc = json.load(open(os.path.join(GOLDEN, name + ".json")))
    reps = doc["reports"]
    n = len(reps)

    def cat(k):
        return np.frombuffer(b"".join(bytes.fromhex(r[k]) for r in reps), np.uint8).reshape(n, -1)

    v = doc["vdaf"]
    res = CE.helper_prep_aggregate(v["algo_id"], v["bits"], v["length"], v["chunk_length"],
                                   bytes.fromhex(doc["verify_key"]), cat("nonce"), cat("public_share"),
                                   cat("helper_input_share"), cat("leader_prep_share"), nthreads=threads)
    assert res["verdicts"].tolist() == [r["verdict"] for r in reps]
    for i, r in enumerate(reps):
        if r["verdict"] == 0:
            assert res["prep_msgs"][i].tobytes().hex() == r["prep_msg"]
    assert res["agg"].hex() == doc["aggregate_share"]
    assert res["count"] == doc["report_count"] and res["checksum"].hex() == doc["checksum"]


def test_cpu_engine_random_batch_vs_oracle():
    from oracle import oracle as O

    orc = O.Prio3Oracle(O.SUMVEC, 3, 37, 5)
    rng = np.random.default_rng(4)
    n = 64
    vk = bytes(range(16))
    meas = rng.integers(0, 8, size=(n, 37), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=8)
    for i in range(0, n, 5):
        lps[i, int(rng.integers(0, lps.shape[1]))] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=8)
    got = CE.helper_prep_aggregate(2, 3, 37, 5, vk, nonces, ps, his, lps, nthreads=3)
    assert got["verdicts"].tolist() == want["verdicts"].tolist()
    assert (got["agg"], got["count"], got["checksum"]) == (want["agg"], want["count"], want["checksum"])
