"""One rank started by lvgpu.shard.launch (tests/test_dist.py launcher tests).

    python dist_rank_main.py <gpus> <spec.json> <result.json>

Reads its rank from torchrun's variables exactly as bench.py does
(shard.world_from_env), joins a gloo group over env://, and runs the shared
rank body of test_dist.py (RankShard, timed_steps, gather, aggregate; the CPU
oracle as the compute).  `fail_rank` in the spec makes that rank exit 3
before the group forms, to test that the launcher ends the job."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "leveldb-rs_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def main():
    import torch.distributed as dist

    from lvgpu import shard
    import test_dist
    gpus, spec_path, out = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    world, rank, _ = shard.world_from_env(gpus)
    with open(spec_path) as f:
        spec = json.load(f)
    if spec.get("fail_rank") == rank:
        sys.exit(3)
    dist.init_process_group("gloo")
    test_dist.rank_body(rank, world, dist, spec["kind"], spec["spec"], out)


if __name__ == "__main__":
    main()
