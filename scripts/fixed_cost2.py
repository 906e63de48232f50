"""Host-side latency around one short device run (config 3, 20 steps).

For each completion strategy, after an idle gap, times: host wall from just
before the launch to completion, and the HIP-event span of the launch.
wall - span = submission latency + completion-notification latency.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from viabel_amd import _native as nat, targets, vb

D, N = 10_000, 128


def main():
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    nat.use_stream(0, stream.cuda_stream)
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, 100000, init[None, :])
    step = [0]
    run.advance_philox(5, 0, 1, 0)
    step[0] = 5
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(200)]
    k = [0]

    def once(mode, gap):
        if gap:
            time.sleep(gap)
        e0, e1 = evs[k[0]]
        k[0] += 1
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record(stream)
        run.advance_philox(20, 0, 1, step[0])
        e1.record(stream)
        t1 = time.perf_counter()
        if mode == 'spin':
            while not e1.query():
                pass
        elif mode == 'evsync':
            e1.synchronize()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        step[0] += 20
        return {'wall_us': (t2 - t0) * 1e6, 'submit_us': (t1 - t0) * 1e6,
                'span_us': e0.elapsed_time(e1) * 1e3}

    for gap in (0.0, 0.001, 0.05):
        for mode in ('sync', 'spin', 'evsync'):
            rs = [once(mode, gap) for _ in range(6)]
            print(json.dumps({'gap_s': gap, 'mode': mode,
                              'wall_us': [round(r['wall_us'], 1) for r in rs],
                              'span_us': [round(r['span_us'], 1) for r in rs],
                              'submit_us': [round(r['submit_us'], 1) for r in rs]}), flush=True)


if __name__ == '__main__':
    main()
