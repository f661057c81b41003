"""Stand-in for bench.py's worker under bench.spawn_ranks (CPU, gloo): checks the launcher's
environment and prints one JSON line from rank 0, the way bench.py's ranks do."""
import json
import os
import sys

import torch
import torch.distributed as dist

world = int(os.environ["WORLD_SIZE"])
rank = int(os.environ["RANK"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
assert os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
dist.init_process_group("gloo")
ones = torch.ones(1)
dist.all_reduce(ones)
if rank == 0:
    print(json.dumps({"n_gpus": dist.get_world_size(), "rccl_ranks": int(ones.item()), "argv": sys.argv[1:]}),
          flush=True)
dist.destroy_process_group()
