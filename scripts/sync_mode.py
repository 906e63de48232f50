"""Host completion latency of the headline's timed region under the HIP device
scheduling flags (hipSetDeviceFlags before the context exists): 0 auto, 1 spin,
2 yield, 4 blocking sync; -1 leaves the runtime default.  Times the bench.py
protocol (synchronize, one 20-step advance_philox, synchronize) 40 times and
prints the median wall time per step.  One JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    flag = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    rc = None
    if flag >= 0:
        hip = ctypes.CDLL('libamdhip64.so')
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(flag))
    import torch
    from viabel_amd import _native as nat, targets, vb
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    nat.use_stream(0, stream.cuda_stream)
    D, N = 10_000, 128
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    reps, K, W = 40, 20, 5
    run = vb.DeviceRun(obj, reps * (K + W) + 10, init[None, :])
    run.set_timing(True)
    step, wall, sync_only = 0, [], []
    for _ in range(reps):
        run.advance_philox(W, 0, 1, step)
        step += W
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run.advance_philox(K, 0, 1, step)
        step += K
        torch.cuda.synchronize(dev)
        wall.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        sync_only.append(time.perf_counter() - t0)
    lt = run.launch_times()
    timed = [t for k, t in lt if k == K]
    print(json.dumps({'flag': flag, 'rc': rc, 'us_per_step_median': round(float(np.median(wall)) / K * 1e6, 3),
                      'us_per_step_min': round(float(np.min(wall)) / K * 1e6, 3),
                      'launch_us_median': round(float(np.median(timed)) * 1e6, 2),
                      'idle_sync_us': round(float(np.median(sync_only)) * 1e6, 2)}), flush=True)


if __name__ == '__main__':
    main()
