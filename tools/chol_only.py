"""bench.time_cholesky alone (n = 4096 factor + inverse, and the batched
shapes), for rocprofv3 kernel stats (development tool)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    Xtr, _, _ = bench.build_problem(dev, 1)
    print(json.dumps(bench.time_cholesky(Xtr, dev)))
