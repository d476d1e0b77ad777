"""Child process of tests/test_gpu_coalesce.py::test_two_engines_under_a_small_arena_budget (run with a small
JX_ARENA_GB): two SumVec 8x1000/88 engines with different verify keys, each in its own thread, run fused device
prep + aggregate calls whose launch size changes every call (debug option 5), so the device arena keeps trimming
one engine's idle staging for the other's check-outs. Prints one JSON line: verified (every verdict, prep
message and both aggregates against the C oracle) and the arena counters."""
from __future__ import annotations

import json
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

P128 = 2**128 - 28 * 2**64 + 1


def main():
    import torch

    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3
    from oracle import oracle as O

    v = Prio3.sum_vec(8, 1000, 88)
    vks = [bytes(range(16)), bytes(range(16, 32))]
    K, R = 1024, 49152
    orc = O.Prio3Oracle(v.algo_id, v.bits, v.length, v.chunk_length)
    pools = []
    for k, vk in enumerate(vks):
        rng = np.random.default_rng(700 + k)
        meas = rng.integers(0, 256, size=(K, v.length), dtype=np.uint64)
        nonces = rng.integers(0, 256, size=(K, 16), dtype=np.uint8)
        rands = rng.integers(0, 256, size=(K, orc.sizes.client_rand), dtype=np.uint8)
        ps, his, lps, _ = orc.client_leader_batch(vk, meas, nonces, rands, nthreads=16)
        lps[::37, 5] ^= 4
        want = orc.helper_prep_batch(vk, nonces, ps, his, lps, nthreads=16, want_out_shares=True)
        pools.append((nonces, ps, his, lps, want))
    dev = torch.device("cuda", 0)
    idx = np.arange(R) % K
    d_idx = torch.from_numpy(idx).to(dev)
    tiles = [[torch.from_numpy(np.ascontiguousarray(a)).to(dev).index_select(0, d_idx).contiguous() for a in p[:4]]
             for p in pools]
    outs = [(torch.empty(R, dtype=torch.uint8, device=dev), torch.empty((R, 16), dtype=torch.uint8, device=dev))
            for _ in vks]
    torch.cuda.synchronize()
    engs = [HelperEngine(v, vk) for vk in vks]
    sizes = [[16384, 4096, 12288, 2048], [3072, 16384, 6144, 8192]]
    errs = []
    amax = [0]
    lock = threading.Lock()

    def worker(k):
        try:
            d_n, d_ps, d_his, d_lps = tiles[k]
            d_v, d_m = outs[k]
            for c, size in enumerate(sizes[k]):
                engs[k].debug(5, size)
                engs[k].prep_and_aggregate_device(d_n.data_ptr(), d_ps.data_ptr(), d_his.data_ptr(), d_lps.data_ptr(),
                                                  R, 0, d_m.data_ptr(), d_v.data_ptr(), stream=False)
                m = engs[k].memory()
                with lock:
                    amax[0] = max(amax[0], m["arena_allocated"])
            engs[k].sync()
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    ok = not errs
    calls = len(sizes[0])
    for k, (nonces, ps, his, lps, want) in enumerate(pools):
        d_v, d_m = outs[k]
        got_v = d_v.cpu().numpy()
        ok = ok and np.array_equal(got_v, want["verdicts"][idx])
        f = got_v == 0
        ok = ok and np.array_equal(d_m.cpu().numpy()[f], want["prep_msgs"][idx][f])
        fin = want["verdicts"] == 0
        mult = np.bincount(idx, minlength=K) * calls
        words = want["out_shares"].reshape(K, v.length, 4, 4).astype(np.uint64)
        words = words[..., 0] | (words[..., 1] << 8) | (words[..., 2] << 16) | (words[..., 3] << 24)
        sums = np.einsum("k,kew->ew", np.where(fin, mult, 0).astype(np.uint64), words)
        exp = b"".join((sum(int(sums[e, w]) << (32 * w) for w in range(4)) % P128).to_bytes(16, "little")
                       for e in range(v.length))
        agg, cnt, _ = engs[k].aggregate_share(0)
        ok = ok and cnt == int(np.where(fin, mult, 0).sum()) and agg == exp
    m = engs[0].memory()
    for e in engs:
        e.close()
    print(json.dumps({"verified": bool(ok), "errors": errs[:2], "arena_frees": m["arena_frees"],
                      "arena_budget": m["arena_budget"], "arena_allocated_max": amax[0], "arena_waits": m["arena_waits"],
                      "arena_allocs": m["arena_allocs"], "arena_reuses": m["arena_reuses"]}))


if __name__ == "__main__":
    main()
