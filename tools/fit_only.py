"""The bench's GP-fit leg alone (fit_gpytorch_mll at n = 4096 from default
init), for rocprofv3 kernel stats of the MLL closure (development tool)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    Xtr, Ytr, _ = bench.build_problem(dev, 1)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    for _ in range(reps):
        out = bench.time_gp_fit(Xtr, Ytr, dev, cpu=False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
