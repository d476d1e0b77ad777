"""The CPU baseline engine (cpu_baseline/jc_cpu_engine.cpp, bench.py's cpu_baseline leg) is
byte-exact with the golden fixtures: verdicts, prepare messages, aggregate share, count, checksum."""
import json
import os

import numpy as np
import pytest

from cpu_baseline import cpu_engine as CE

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("threads", [1, 5])
@pytest.mark.parametrize("name", ["sumvec_8x1000_88", "sumvec_small", "histogram_16_4", "histogram_256_16", "count",
                                  "sum8", "sum32", "fixedpoint16_3", "fixedpoint16_37", "fixedpoint32_3",
                                  "fixedpoint32_100", "fixedpoint16_10000"])
def test_cpu_engine_matches_fixtures(name, threads):
    doc = json.load(open(os.path.join(GOLDEN, name + ".json")))
    reps = doc["reports"]
    n = len(reps)

    def cat(k):
        return np.frombuffer(b"".join(bytes.fromhex(r[k]) for r in reps), np.uint8).reshape(n, -1)

    v = doc["vdaf"]
    ps = cat("public_share") if reps[0]["public_share"] else np.zeros((n, 0), np.uint8)
    res = CE.helper_prep_aggregate(v["algo_id"], v["bits"], v["length"], v["chunk_length"],
                                   bytes.fromhex(doc["verify_key"]), cat("nonce"), ps,
                                   cat("helper_input_share"), cat("leader_prep_share"), nthreads=threads)
    assert res["verdicts"].tolist() == [r["verdict"] for r in reps]
    for i, r in enumerate(reps):
        if r["verdict"] == 0 and r["prep_msg"]:
            assert res["prep_msgs"][i].tobytes().hex() == r["prep_msg"]
    if "aggregate_share" in doc:
        assert res["agg"].hex() == doc["aggregate_share"]
    else:
        import hashlib
        assert hashlib.sha256(res["agg"]).hexdigest() == doc["aggregate_share_sha256"]
    assert res["count"] == doc["report_count"] and res["checksum"].hex() == doc["checksum"]


@pytest.mark.parametrize("algo,bits,length,chunk", [(2, 3, 37, 5), (0, 0, 0, 0), (1, 13, 0, 0), (3, 0, 21, 4),
                                                    (5, 16, 11, 0), (5, 32, 7, 0)],
                         ids=["sumvec", "count", "sum13", "histogram", "fixedpoint16", "fixedpoint32"])
def test_cpu_engine_random_batch_vs_oracle(algo, bits, length, chunk):
    """Random honest and tampered reports (every 5th leader prep share has a flipped bit): verdicts,
    aggregate, count and checksum == the C oracle's."""
    from oracle import oracle as O

    orc = O.Prio3Oracle(algo, bits, length, chunk)
    rng = np.random.default_rng(4 + algo)
    n = 64
    vk = bytes(range(16))
    if algo == 0:
        meas = rng.integers(0, 2, size=(n, 1), dtype=np.uint64)
    elif algo == 1:
        meas = rng.integers(0, 1 << bits, size=(n, 1), dtype=np.uint64)
    elif algo == 3:
        meas = rng.integers(0, length, size=(n, 1), dtype=np.uint64)
    elif algo == 5:  # small fixed-point entries (norm within bounds), as two's-complement words
        meas = rng.integers(-(1 << (bits - 5)), 1 << (bits - 5), size=(n, length)).astype(np.int64).view(np.uint64)
        meas &= np.uint64((1 << bits) - 1)
    else:
        meas = rng.integers(0, 1 << bits, size=(n, length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=8)
    for i in range(0, n, 5):
        lps[i, int(rng.integers(0, lps.shape[1]))] ^= 1 << int(rng.integers(0, 8))
    want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=8)
    got = CE.helper_prep_aggregate(algo, bits, length, chunk, vk, nonces, ps, his, lps, nthreads=3)
    assert got["verdicts"].tolist() == want["verdicts"].tolist()
    assert (want["verdicts"] == 0).sum() > n // 2 and (want["verdicts"] != 0).any()
    assert (got["agg"], got["count"], got["checksum"]) == (want["agg"], want["count"], want["checksum"])


@pytest.mark.parametrize("algo,bits,length,chunk", [(2, 3, 37, 5), (1, 13, 0, 0), (3, 0, 21, 4), (5, 16, 11, 0)],
                         ids=["sumvec", "sum13", "histogram", "fixedpoint16"])
def test_cpu_engine_leader_ping_pong_vs_oracle(algo, bits, length, chunk):
    """The CPU engine's leader (configs[4] is a leader+helper ping-pong): prep shares == the oracle's
    prepare_init(agg_id 0); CPU leader -> CPU helper -> CPU leader finish gives output shares that add up
    with the helper's to the measurement sums, with the helper's rejects failing the leader."""
    from oracle import oracle as O

    orc = O.Prio3Oracle(algo, bits, length, chunk)
    rng = np.random.default_rng(40 + algo)
    n = 40
    vk = bytes(range(3, 19))
    if algo == 1:
        meas = rng.integers(0, 1 << bits, size=(n, 1), dtype=np.uint64)
    elif algo == 3:
        meas = rng.integers(0, length, size=(n, 1), dtype=np.uint64)
    elif algo == 5:
        meas = rng.integers(-(1 << (bits - 5)), 1 << (bits - 5), size=(n, length)).astype(np.int64).view(np.uint64)
        meas &= np.uint64((1 << bits) - 1)
    else:
        meas = rng.integers(0, 1 << bits, size=(n, length), dtype=np.uint64)
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    rands = rng.integers(0, 256, size=(n, orc.sizes.client_rand), dtype=np.uint8)
    sh = [orc.shard(meas[i], nonces[i].tobytes(), rands[i].tobytes()) for i in range(n)]
    ps, lis, his = (np.frombuffer(b"".join(s[k] for s in sh), np.uint8).reshape(n, -1) for k in range(3))
    lead = CE.leader_prep_init(algo, bits, length, chunk, vk, nonces, ps, lis, orc.sizes.prep_share, nthreads=3)
    for i in range(n):
        rc, share, _, _ = orc.prep_init(vk, 0, nonces[i].tobytes(), ps[i].tobytes(), lis[i].tobytes())
        assert rc == lead["verdicts"][i] == 0 and lead["prep_shares"][i].tobytes() == share, i
    lps = lead["prep_shares"].copy()
    lps[7, 3] ^= 1  # the helper rejects report 7
    helper = CE.helper_prep_aggregate(algo, bits, length, chunk, vk, nonces, ps, his, lps, nthreads=2)
    assert helper["verdicts"][7] != 0 and (helper["verdicts"] != 0).sum() == 1
    fin = CE.leader_finish_aggregate(algo, bits, length, chunk, nonces, lis, lead["seeds"], lead["verdicts"],
                                     helper["prep_msgs"], helper["verdicts"], nthreads=2)
    assert fin["verdicts"][7] == 5 and (fin["verdicts"] != 0).sum() == 1
    assert fin["count"] == helper["count"] == n - 1 and fin["checksum"] == helper["checksum"]
    p = 2**128 - 28 * 2**64 + 1
    ok = np.arange(n) != 7
    tot = [(int.from_bytes(fin["agg"][16 * j:16 * j + 16], "little") +
            int.from_bytes(helper["agg"][16 * j:16 * j + 16], "little")) % p for j in range(len(fin["agg"]) // 16)]
    if algo == 3:
        want = [int((meas[ok, 0] == j).sum()) for j in range(length)]
    elif algo == 5:
        want = [int(sum(int(meas[i, j]) ^ (1 << (bits - 1)) for i in np.nonzero(ok)[0])) for j in range(length)]
    else:
        want = [int(meas[ok, j].astype(object).sum()) for j in range(meas.shape[1])]
    assert tot == want
