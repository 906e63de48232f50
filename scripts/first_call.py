"""bench.py's timed region in a fresh process: warm-up of 5 steps (one call,
or `--split` five 1-step calls), then one timed 20-step advance.  Prints the
host submit time, the wall time to synchronisation and the launch's event
span, to locate the extra wall time of a first timed call."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--split', action='store_true')
    ap.add_argument('--sleep', type=float, default=0.0)
    ap.add_argument('--repeat', type=int, default=1)
    ap.add_argument('--spin', action='store_true', help='poll the stream before synchronising')
    a = ap.parse_args()
    import numpy as np
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
    run = vb.DeviceRun(obj, 25 + 20 * a.repeat, init[None, :])
    run.set_timing(True)
    if a.split:
        for k in range(5):
            run.advance_philox(1, 0, 1, k)
    else:
        run.advance_philox(5, 0, 1, 0)
    torch.cuda.synchronize(dev)
    run.launch_times()
    if a.sleep:
        time.sleep(a.sleep)
    step = 5
    for r in range(a.repeat):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run.advance_philox(20, 0, 1, step)
        t1 = time.perf_counter()
        if a.spin:
            while not stream.query():
                pass
        torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        step += 20
        span = run.launch_times()[0][1]
        print(json.dumps({'spin': a.spin, 'split': a.split, 'sleep': a.sleep, 'rep': r,
                          'submit_us': round((t1 - t0) * 1e6, 2),
                          'wall_us': round((t2 - t0) * 1e6, 2), 'span_us': round(span * 1e6, 2)}),
              flush=True)


if __name__ == '__main__':
    main()
