"""Step time of the sep kernel vs D (waves = D/2) at fixed N (GPU only)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np
import torch
from viabel_amd import _native as nat, targets, vb

dev = torch.device('cuda', 0)
s = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(s)
nat.use_stream(0, s.cuda_stream)
N = int(os.environ.get('N', '128'))
out = {}
for D in [int(x) for x in os.environ.get('DS', '2048,4096,6144,8192,8194,10000,12288,16384,20000').split(',')]:
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    run = vb.DeviceRun(vb.black_box_klvi(fam, targets.isogauss(D), N), 4096,
                       np.concatenate([np.zeros(D), np.ones(D)])[None], learning_rate=0.01)
    run.advance_philox(1024, 0, 1, 0)
    best = 1e9
    for r in range(3):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s); run.advance_philox(1024, 0, 1, 1024 * (r + 1)); e1.record(s); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / 1024)
    out[D] = {'us_per_step': best, 'waves': (D + 1) // 2, 'ns_per_col_step': best * 1e3 / D,
              'mc_samples_per_s': N * D / (best * 1e-6)}
print(json.dumps({'N': N, 'sweep': out}))
