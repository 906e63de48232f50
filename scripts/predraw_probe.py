"""One block-kernel run (mean-field t, mixture D=5, N=300, 2 problems, KLVI,
700 Philox steps) in the draw mode named by argv[1] ('0' in-kernel draws,
'all' pre-drawn); prints a checksum of the result."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['VIABEL_AMD_PREDRAW'] = sys.argv[1]
from viabel_amd import vb, targets
D, N = int(os.environ.get('PD_D', 5)), int(os.environ.get('PD_N', 300))
fam = vb.mean_field_t_variational_family(D, 40.0, rng='philox')
obj = vb.black_box_klvi(fam, targets.mixture(D), N)
rs = np.random.RandomState(40)
init = np.stack([np.concatenate([rs.randn(D) * 0.7, rs.randn(D) * 0.3 - 0.2]) for _ in range(2)])
run = vb.DeviceRun(obj, 700, init, learning_rate=0.01)
run.advance_philox(3, 7, 5, 0)
run.advance_philox(697, 7, 5, 3)
lam, hist, vals, smooth = run.result()
print(sys.argv[1], 'D', D, 'N', N, 'lam', repr(float(lam.sum())), 'vals', repr(float(vals.sum())))
