"""Throughput benchmark of the MC-VI hot path on MI355X (driver contract).

Workload (BASELINE.json metric: "MC-samples/sec (N x D / step) for KLVI
adagrad, D=1e4 N=128"): mean-field Gaussian KLVI on the synthetic isotropic
Gaussian target N(0, I_D), D = 10 000, N = 128 Monte Carlo draws per step,
adagrad (window 10, lr .01 constant, eps .1), init lambda = [0, 1]
(SURVEY.md §8d config 3).  A step = one pass of the hot path: draw N x D noise,
reparameterise, target log density + gradient, reduce over N, adagrad update,
value and tail-quarter history bookkeeping.  Draws come from the in-kernel
Philox generator (rng='philox'); everything is resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: independent optimisation restarts (one per rank, distinct Philox
streams) with no data-path collective -> weak scaling; an RCCL all_gather of
the per-restart summaries closes the run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

D, N, WINDOW, LR, EPS = 10_000, 128, 10, 0.01, 0.1
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_PEAK_GINSTR = 256 * 4 * 2.4 / 4  # wave64 fp64 VALU issue: 4 cycles/instr/SIMD (profiles/r01/ubench_instr_costs.txt)
CHUNK = 256                    # steps per sep_kernel launch (vb_capi.hip max_chunk)


def algorithmic_bytes_per_step(n, d, w):
    """one fp64 draw of the N x D sample matrix + lambda read/write,
    gradient write and the W-window read (2D params x 8 B)."""
    return 8 * n * d + 16 * d * (3 + w)


def cpu_baseline(seconds=12.0):
    """The oracle (numpy restatement of vb.py:236-245 + 345-389, legacy RNG like
    the reference) timed on this host, one thread, on a bounded sample."""
    import numpy as np
    from oracle import vb_oracle
    fam = vb_oracle.Family('gauss', D)
    lam = np.concatenate([np.zeros(D), np.ones(D)])
    grads = []
    acc_steps = 0
    t_end = None
    for i in range(3):                                    # warm-up
        vb_oracle.klvi_value_grad(fam, 'isogauss', lam, N)
    t0 = time.perf_counter()
    while True:
        val, g = vb_oracle.klvi_value_grad(fam, 'isogauss', lam, N)
        grads.append(g)
        if len(grads) > WINDOW:
            grads.pop(0)
        acc = np.sum(np.array(grads) ** 2, axis=0)
        lam = lam - LR * g / np.sqrt(EPS + acc)
        acc_steps += 1
        t_end = time.perf_counter()
        if t_end - t0 >= seconds:
            break
    dt = t_end - t0
    return {'value': acc_steps * N * D / dt, 'unit': 'MC-samples/s', 'cores': 1, 'kind': 'port',
            'sample': '%d KLVI adagrad steps at N=%d, D=%d (oracle/vb_oracle.py, numpy legacy '
                      'RandomState noise, OMP/OPENBLAS threads = 1), %.1f s' % (acc_steps, N, D, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20000)
    ap.add_argument('--warmup', type=int, default=1000)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    args = ap.parse_args()

    import numpy as np
    import torch

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device('cuda', local)

    from viabel_amd import _native as nat, targets
    from viabel_amd import vb
    # a dedicated (non-NULL) stream: the kernels and the timing events share it
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    nat.use_stream(local, stream.cuda_stream)

    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), N)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    K, W = args.steps, args.warmup
    run = vb.DeviceRun(obj, W + K, init[None, :], window=WINDOW, learning_rate=LR, epsilon=EPS)
    seed, strm = 0, 1 + rank       # one restart per rank, independent Philox streams

    # warm-up (untimed)
    run.advance_philox(W, seed, strm, 0)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)

    # timed region: K steps in launches of CHUNK steps, each bracketed by events
    evs = []
    t0 = time.perf_counter()
    done = 0
    while done < K:
        cs = min(CHUNK, K - done)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run.advance_philox(cs, seed, strm, W + done)
        e1.record(stream)
        evs.append((cs, e0, e1))
        done += cs
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    # per-launch durations of full chunks (sep_kernel + its value-partial reduction)
    full = [(cs, a.elapsed_time(b) * 1e-3) for cs, a, b in evs if cs == CHUNK]
    launch_s = float(np.mean([t for _, t in full])) if full else elapsed
    bytes_launch = CHUNK * algorithmic_bytes_per_step(N, D, WINDOW)
    achieved = bytes_launch / launch_s / 1e9

    # restart summaries gathered over RCCL (the only collective)
    lam, hist, vals, smooth = run.result()
    summary = torch.tensor([float(vals[0, -1]), float(np.mean(vals[0, -100:])),
                            float(np.linalg.norm(smooth[0]))], dtype=torch.float64, device=dev)
    if dist:
        gathered = [torch.empty_like(summary) for _ in range(world)]
        dist.all_gather(gathered, summary)
        gathered = torch.stack(gathered).cpu().numpy()
    else:
        gathered = summary.cpu().numpy()[None]

    total_units = world * K * N * D
    value = total_units / elapsed
    if rank == 0:
        line = {
            'metric': 'MC-samples/sec (N*D/step) for KLVI adagrad, D=1e4 N=128',
            'value': value, 'unit': 'MC-samples/s', 'n_gpus': world, 'steps': K, 'warmup': W,
            'ms_per_step': elapsed / K * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
            'config': {'workload': 'mean-field Gaussian KLVI + adagrad on isotropic Gaussian '
                                   'target (SURVEY config 3)',
                       'D': D, 'N': N, 'window': WINDOW, 'learning_rate': LR, 'epsilon': EPS,
                       'rng': 'philox', 'restarts': world,
                       'parallelism': 'restarts sharded 1/GPU, RCCL all_gather of summaries'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                         'kernel': 'sep_kernel<IsoGauss,gauss,philox> (+ sep_values_kernel)',
                         'launch_ms': launch_s * 1e3, 'steps_per_launch': CHUNK,
                         'algorithmic_bytes_per_launch': bytes_launch},
            'restart_summaries': gathered.tolist(),
        }
        prof = os.path.join(ROOT, 'profiles', 'traffic.json')
        if os.path.exists(prof):
            try:
                tr = json.load(open(prof))
                line['roofline']['traffic'] = tr.get('bytes_per_launch')
                line['roofline']['traffic_source'] = tr.get('source')
                if tr.get('valu_instr_per_launch'):
                    # the kernel's real ceiling: fp64 VALU issue
                    ins = float(tr['valu_instr_per_launch'])
                    rate = ins / launch_s / 1e9
                    line['valu'] = {'instr_per_launch': ins, 'achieved': rate,
                                    'peak': VALU_PEAK_GINSTR, 'unit': 'G wave-instr/s',
                                    'frac': rate / VALU_PEAK_GINSTR,
                                    'source': 'SQ_INSTS_VALU (rocprofv3 --pmc, '
                                              'profiles/r01/bench_pmc_summary.json) / live '
                                              'launch time; peak = 256 CUs x 4 SIMDs x 2.4 GHz '
                                              '/ 4 cycles per wave64 fp64 instruction'}
            except Exception:
                pass
        if not args.no_cpu_baseline and world == 1:   # rank 0 at N = 1 only
            line['cpu_baseline'] = cpu_baseline(args.cpu_seconds)
            line['speedup_vs_cpu_baseline'] = value / line['cpu_baseline']['value']
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    # the CPU-baseline leg is single-threaded numpy (set before numpy loads)
    for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ.setdefault(k, '1')
    main()
