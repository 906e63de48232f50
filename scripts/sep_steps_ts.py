"""Per-wave progress through one sep_kernel launch (config 3, N = 128) from the
VB_SEP_TS build (make -C viabel_amd/csrc variant V=septs EXTRA=-DVB_SEP_TS=5;
VIABEL_AMD_LIB=.../libviabel_amd_septs.so): timestamps (s_memrealtime, 100 MHz)
at steps 0, 1, 2, 4, ... and the last step of the launch whose first step is 5.
Prints, per wave type, the median time of each checkpoint and the per-step cost
between checkpoints."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from viabel_amd import _native as nat, targets, vb
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 256
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
    span = e0.elapsed_time(e1) * 1e3
    nw = 8192
    buf = (ctypes.c_ulonglong * (32 * nw))()
    rc = nat.lib().vb_debug_sep_ts(buf, nw)
    assert rc == 0, rc
    both = np.frombuffer(buf, dtype=np.uint64).reshape(2, nw, 16).astype(np.int64)
    a, clk = both[0], both[1]
    keep = a[:, 15] > 0
    a, clk = a[keep], clk[keep]
    t0 = a[:, 15].min()
    print('launch of %d steps: event span %.1f us, waves %d' % (steps, span, len(a)))
    ks = [0] + [1 << j for j in range(12) if (1 << j) < steps - 1]
    cols = list(range(len(ks))) + [13]
    labels = ks + [steps - 1]
    for ppw in (4, 2, 1):
        m = a[:, 14] == ppw
        if not m.any():
            continue
        med = [np.median((a[m, c] - t0) / 100.0) for c in cols]
        mx = [np.max((a[m, c] - t0) / 100.0) for c in cols]
        ent = np.median((a[m, 15] - t0) / 100.0)
        print('PPW %d (%d waves): entry p50 %.2f us' % (ppw, m.sum(), ent))
        prev = None
        for lab, md, mxx in zip(labels, med, mx):
            rate = '' if prev is None else ' | %.3f us/step since step %d' % (
                (md - prev[1]) / (lab - prev[0]), prev[0])
            if prev is not None:
                c0, c1 = cols[labels.index(prev[0])], cols[labels.index(lab)]
                ghz = np.median((clk[m, c1] - clk[m, c0]) / ((a[m, c1] - a[m, c0]) * 10.0))
                rate += ', core clock %.3f GHz' % ghz
            print('   end of step %4d: p50 %8.2f us  max %8.2f us%s' % (lab, md, mxx, rate))
            prev = (lab, md)


if __name__ == '__main__':
    main()
