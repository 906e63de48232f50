"""Where does a short device-resident adagrad run spend its time?

Times vb_run_advance for config 3 (mean-field Gaussian KLVI, isogauss D=1e4,
N=128, Philox) at several step counts, back to back and after idle gaps, with
HIP events on the launch stream and host wall time around the ctypes call.
Distinguishes a per-call host cost, a per-launch kernel prologue and GPU clock
ramp-up after idle.
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
    total = 200000
    run = vb.DeviceRun(obj, total, init[None, :])
    step = [0]
    out = {}

    def adv(k):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        run.advance_philox(k, 0, 1, step[0])
        e1.record(stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        step[0] += k
        return {'steps': k, 'ev_us': e0.elapsed_time(e1) * 1e3, 'call_us': (t1 - t0) * 1e6,
                'wall_us': (t2 - t0) * 1e6}

    out['first5'] = adv(5)
    out['then20'] = [adv(20) for _ in range(5)]
    out['then256'] = [adv(256) for _ in range(3)]
    out['then20_hot'] = [adv(20) for _ in range(5)]
    time.sleep(0.5)
    out['after_sleep_20'] = [adv(20) for _ in range(3)]
    # many back-to-back short launches without syncs: per-launch cost in a queue
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(50):
        run.advance_philox(20, 0, 1, step[0])
        step[0] += 20
    e1.record(stream)
    torch.cuda.synchronize(dev)
    out['queued_50x20_us_per_step'] = e0.elapsed_time(e1) * 1e3 / 1000
    out['long_2560'] = adv(2560)
    for k, v in out.items():
        print(k, json.dumps(v), flush=True)


if __name__ == '__main__':
    main()
