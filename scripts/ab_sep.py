"""In-process A/B timing of sep_kernel variants (cdna guide §5.4 rule 24:
interleaved rounds in one process).  GPU only; prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np
import torch

from viabel_amd import _native as nat, targets, vb


def time_steps(run, steps, seed, stream, step0, tstream):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(tstream)
    run.advance_philox(steps, seed, stream, step0)
    e1.record(tstream)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps  # us per step


def main():
    variants = os.environ.get('VARIANTS', '1,2,mix').split(',')
    Ns = [int(v) for v in os.environ.get('NS', '128').split(',')]
    D = int(os.environ.get('D', '10000'))
    rounds = int(os.environ.get('ROUNDS', '3'))
    steps = int(os.environ.get('STEPS', '2048'))
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    nat.use_stream(0, s.cuda_stream)
    res = {}
    for N in Ns:
        fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
        obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
        init = np.concatenate([np.zeros(D), np.ones(D)])
        total = steps * (rounds * len(variants) + 1)
        run = vb.DeviceRun(obj, total, init[None], learning_rate=0.01)
        done = 0
        os.environ['VB_SEP_MODE'] = variants[0]
        run.advance_philox(steps, 0, 1, 0)   # warm-up
        done += steps
        for r in range(rounds):
            for v in variants:
                os.environ['VB_SEP_MODE'] = v
                us = time_steps(run, steps, 0, 1, done, s)
                done += steps
                res.setdefault('N%d_%s' % (N, v), []).append(us)
    out = {k: {'us_per_step_min': min(v), 'us_per_step_med': float(np.median(v)),
               'mc_samples_per_s': None} for k, v in res.items()}
    for k in out:
        N = int(k.split('_')[0][1:])
        out[k]['mc_samples_per_s'] = N * D / (out[k]['us_per_step_min'] * 1e-6)
    print(json.dumps({'D': D, 'results': out}))


if __name__ == '__main__':
    main()
