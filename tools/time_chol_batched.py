import sys, json, torch
sys.path.insert(0, '.')
import bench
from botorch_amd.utils_sampling import draw_sobol_samples
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 4096, 1, seed=0).squeeze(1)
r = bench.time_cholesky(X, torch.device("cuda", 0))
print(json.dumps(r))
