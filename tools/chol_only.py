"""bench.time_cholesky alone (n = 4096 factor + inverse, and the batched
shapes), for rocprofv3 kernel stats (development tool).  argv "single": the
n = 4096 launch only (a PMC pass then measures one shape's bytes)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    Xtr, _, _ = bench.build_problem(dev, 1)
    single = len(sys.argv) > 1 and sys.argv[1] == "single"
    print(json.dumps(bench.time_cholesky(Xtr, dev, shapes=() if single else
                                         ((3, 2048), (4, 4096), (8, 4096)), ainv=not single)))
