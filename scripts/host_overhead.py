"""Host-side cost of the pieces of bench.py's timed region (config 3, 20-step
launches): submit time of advance_philox with and without the library's launch
events, the wall time from submit to synchronisation, an idle synchronize, and
the event span, median of 20 repetitions each."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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
    run = vb.DeviceRun(obj, 100000, init[None, :])
    step = [5]
    run.advance_philox(5, 0, 1, 0)
    torch.cuda.synchronize(dev)
    ctx = nat.context()

    def trial(timing, sync):
        run.set_timing(timing)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run.advance_philox(20, 0, 1, step[0])
        t1 = time.perf_counter()
        if sync == 'torch':
            torch.cuda.synchronize(dev)
        else:
            ctx.synchronize()
        t2 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        step[0] += 20
        span = run.launch_times()
        return {'submit_us': (t1 - t0) * 1e6, 'wall_us': (t2 - t0) * 1e6,
                'idle_sync_us': (t3 - t2) * 1e6,
                'span_us': span[0][1] * 1e6 if span else float('nan')}

    for timing in (False, True):
        for sync in ('torch', 'native'):
            rs = [trial(timing, sync) for _ in range(20)]
            med = {k: round(float(np.median([r[k] for r in rs])), 2) for k in rs[0]}
            print(json.dumps({'timing': timing, 'sync': sync, **med}), flush=True)


if __name__ == '__main__':
    main()
