"""The driver's headline timed region as bench.py runs it -- one warm-up advance of W
steps, synchronize, launch_times(), synchronize, then ONE timed K-step advance +
synchronize -- followed by 20 more timed repetitions in the same process, to
separate first-shot costs from the steady state.  One JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    flag = int(sys.argv[3]) if len(sys.argv) > 3 else -1   # hipSetDeviceFlags before the context
    if flag >= 0:
        import ctypes
        ctypes.CDLL('libamdhip64.so').hipSetDeviceFlags(ctypes.c_uint(flag))
    import torch
    from viabel_amd import _native as nat, targets, vb
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    nat.use_stream(0, stream.cuda_stream)
    D, N, K, W = 10_000, 128, 20, 5
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, 30 * (K + W), init[None, :])
    run.set_timing(True)
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 1   # warm-up advance calls per W steps
    idle = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # seconds idle before each timed call
    step, walls, spans = 0, [], []
    for rep in range(21):
        for c in range(calls):
            k = W // calls + (1 if c < W % calls else 0)
            run.advance_philox(k, 0, 1, step)
            step += k
        torch.cuda.synchronize(dev)
        run.launch_times()
        torch.cuda.synchronize(dev)
        if idle:
            time.sleep(idle)
        t0 = time.perf_counter()
        run.advance_philox(K, 0, 1, step)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        step += K
        walls.append((t2 - t0, t1 - t0))
        spans.append(run.launch_times()[-1][1])
    first = walls[0]
    rest = np.array(walls[1:])
    print(json.dumps({'warmup_calls': calls, 'idle_s': idle, 'flag': flag, 'first_us_per_step': round(first[0] / K * 1e6, 3),
                      'first_submit_us': round(first[1] * 1e6, 2),
                      'first_span_us': round(spans[0] * 1e6, 2),
                      'rest_us_per_step_median': round(float(np.median(rest[:, 0])) / K * 1e6, 3),
                      'rest_submit_us_median': round(float(np.median(rest[:, 1])) * 1e6, 2),
                      'rest_span_us_median': round(float(np.median(spans[1:])) * 1e6, 2)}), flush=True)


if __name__ == '__main__':
    main()
