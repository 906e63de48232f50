"""sep_kernel launch time vs steps per launch (config 3, N = 128): HIP-event
span of one advance_philox(k) after a synchronisation, for k = 1 .. 256.
Separates a per-launch constant from a per-step cost that changes over the
launch."""
import json
import os
import sys

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
    D, N = 10_000, int(os.environ.get('NS', '128'))
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, 200000, init[None, :])
    step = 0
    run.advance_philox(5, 0, 1, 0)
    step = 5
    torch.cuda.synchronize(dev)
    out = {}
    for k in (1, 2, 4, 8, 12, 16, 20, 24, 32, 48, 64, 96, 128, 192, 256):
        spans = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            e0.record(stream)
            run.advance_philox(k, 0, 1, step)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            step += k
            spans.append(e0.elapsed_time(e1) * 1e3)
        out[k] = float(np.median(spans))
        print(json.dumps({'k': k, 'span_us_median': round(out[k], 2),
                          'us_per_step': round(out[k] / k, 3),
                          'spans': [round(x, 1) for x in spans]}), flush=True)
    # a 20-step launch right behind a heater launch of h steps (no synchronisation
    # between): does a warm GPU run the short launch faster?
    for h in (0, 5, 64, 256, 1024):
        spans = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            left = h
            while left > 0:
                c = min(256, left)
                run.advance_philox(c, 0, 1, step)
                step += c
                left -= c
            e0.record(stream)
            run.advance_philox(20, 0, 1, step)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            step += 20
            spans.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({'heater_steps': h, 'span20_us_median': round(float(np.median(spans)), 2),
                          'spans': [round(x, 1) for x in spans]}), flush=True)
    # increments: marginal cost per added step between lengths
    ks = sorted(out)
    for a, b in zip(ks, ks[1:]):
        print('marginal %3d -> %3d: %.3f us/step' % (a, b, (out[b] - out[a]) / (b - a)))


if __name__ == '__main__':
    main()
