"""Per-wave timeline of one short sep_kernel launch (config 3, N = 128).

Run with the instrumented build (make -C viabel_amd/csrc variant V=sepprof
EXTRA=-DVB_SEP_PROF=5) selected through VIABEL_AMD_LIB: every wave of the launch
whose first step is 5 prints "SEPW ppw pair hw_id xcc t_entry t_start t_loop t_end"
(s_memrealtime, 100 MHz).  `--parse FILE` summarises such output: where the
launch's fixed cost goes (dispatch spread, prologue, loop, tail)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(steps):
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
    run = vb.DeviceRun(obj, 5 + steps, init[None, :])
    run.advance_philox(5, 0, 1, 0)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    run.advance_philox(steps, 0, 1, 5)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    sys.stdout.flush()
    print('EVENT_SPAN_US %.2f' % (e0.elapsed_time(e1) * 1e3), flush=True)
    print('STEPS %d' % steps, flush=True)


def parse(path):
    import numpy as np
    rows = []
    nsteps = 20
    for line in open(path):
        if line.startswith('STEPS'):
            nsteps = int(line.split()[1])
        if line.startswith('SEPW'):
            f = line.split()
            rows.append([int(x) for x in f[1:]])
        elif line.startswith('EVENT_SPAN_US'):
            print(line.strip())
    a = np.array(rows, dtype=np.int64)
    ppw, te, ts, tl, tn = a[:, 0], a[:, 4], a[:, 5], a[:, 6], a[:, 7]
    s0, s1, s2 = a[:, 8], a[:, 9], a[:, 10]
    t0 = te.min()
    us = lambda x: (x - t0) / 100.0
    print('waves %d (4-pair %d, 1-pair %d)' % (len(a), (ppw == 4).sum(), (ppw == 1).sum()))
    for name, x in (('entry', te), ('start (tables loaded)', ts), ('loop start', tl), ('end', tn)):
        q = np.percentile(us(x), [0, 10, 50, 90, 100])
        print('%-22s us from first entry: min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f' % (name, *q))
    for p in (4, 1):
        m = ppw == p
        if m.any():
            print('ppw %d: prologue (entry->loop) p50 %.2f us, loop p50 %.2f us, max end %.2f us'
                  % (p, np.median((tl - te)[m]) / 100, np.median((tn - tl)[m]) / 100,
                     us(tn[m]).max()))
            print('       step 0 %.2f us, step 1 %.2f us, step 2 %.2f us, later steps %.2f us/step (p50)'
                  % (np.median((s0 - tl)[m]) / 100, np.median((s1 - s0)[m]) / 100,
                     np.median((s2 - s1)[m]) / 100, np.median((tn - s2)[m]) / 100 / max(1, nsteps - 3)))


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--parse':
        parse(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
