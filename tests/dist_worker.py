"""One rank of tests/test_gpu_distributed.py (run as a child process, not collected by pytest).

Each rank prepares its contiguous shard of a golden batch on the real engine (cuda:0 on a 1-GPU
box: both ranks share the card), then exports its shard record, all-gathers the records over
torch.distributed (argv[2]: "gloo", host-staged, or "nccl" = RCCL on device tensors -- world size 1
on a 1-GPU box, RCCL refuses two ranks on one device) and merges them on the device
(ShardCombiner), the compute_aggregate_share step (aggregator/src/aggregator/aggregate_share.rs:
55-96). Prints one JSON line with the merged record.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from janus_amd import distributed as D
    from janus_amd.engine import HelperEngine
    from janus_amd.vdaf import Prio3

    name = sys.argv[1]
    backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    doc = json.load(open(os.path.join(ROOT, "tests", "golden", name)))
    reps = doc["reports"]
    n = len(reps)

    def cat(k):
        return np.frombuffer(b"".join(bytes.fromhex(r[k]) for r in reps), np.uint8).reshape(n, -1)

    v = doc["vdaf"]
    vdaf = Prio3(v["algo_id"], v["bits"], v["length"], v["chunk_length"], v.get("num_proofs", 1))
    a, b = D.shard_range(n, rank, world)
    ps = cat("public_share") if reps[0]["public_share"] else np.zeros((n, 0), np.uint8)
    with HelperEngine(vdaf, bytes.fromhex(doc["verify_key"]), device=0) as eng:
        eng.prep_and_aggregate(cat("nonce")[a:b], ps[a:b], cat("helper_input_share")[a:b],
                               cat("leader_prep_share")[a:b], segment=0)
        comb = D.ShardCombiner(eng)
        comb.combine(0)
        # a second round on the same buffers, queued without a host sync in between: the
        # stream ordering alone must keep export -> gather -> merge in order
        comb.combine(0)
        agg, count, checksum = comb.result()
        own = eng.aggregate_share(0)
    print(json.dumps({"rank": rank, "backend": dist.get_backend(), "agg_sha": __import__("hashlib").sha256(agg).hexdigest(),
                      "count": count, "checksum": checksum.hex(), "own_count": own[1], "shard": [a, b]}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
