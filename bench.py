"""Throughput benchmark of the MC-VI hot path on MI355X (driver contract).

Headline (BASELINE.json metric "MC-samples/sec (N x D / step) for KLVI
adagrad, D=1e4 N=128; PSIS k-hat match"): mean-field Gaussian KLVI on the
synthetic isotropic Gaussian target N(0, I_D), D = 10 000, N = 128 Monte Carlo
draws per step, adagrad (window 10, lr .01 constant, eps .1), init
lambda = [0, 1].  A step = one pass of the hot path:
draw N x D noise, reparameterise, target log density + gradient, reduce over
N, adagrad update, per-step objective value and tail-quarter history rows.
Draws come from the in-kernel Philox generator; everything is resident in HBM
before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--legs all|none|cfg3_256,...]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: independent optimisation restarts (one per rank, distinct Philox
streams) with no data-path collective -> weak scaling; an RCCL all_gather of
the per-restart summaries closes the run.  The config-5 leg
shards 64 restarts over the ranks (viabel_amd.restarts) the same way.

After the headline, shorter legs put the other BASELINE.json configs on the
same line ("configs"): config 3 at N = 256, configs 1, 2, 4 and 5, and the
PSIS k-hat match (device psislw vs the CPU restatement on a 1e6 log-weight
vector).  The CPU baselines (median of 5 runs, one core, plus
an all-core leg; host CPU model and core counts) run on rank 0 at N = 1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'MC-samples/sec (N×D/step) for KLVI adagrad, D=1e4 N=128; PSIS k-hat match'
D, N, WINDOW, LR, EPS = 10_000, 128, 10, 0.01, 0.1
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # MI355X dense fp64 MFMA spec peak
# wave64 fp64 VALU issue: 256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per instruction
# (profiles/r01/ubench_instr_costs.txt)
VALU_PEAK_GINSTR = 256 * 4 * 2.4 / 4
CHUNK = 256                    # steps per sep_kernel launch (vb_capi.hip max_chunk)


def algorithmic_bytes_per_step(n, d, w):
    """one fp64 draw of the N x D sample matrix + lambda read/write,
    gradient write and the W-window read (2D params x 8 B)."""
    return 8 * n * d + 16 * d * (3 + w)


def _median(xs):
    xs = sorted(xs)
    k = len(xs)
    return xs[k // 2] if k % 2 else 0.5 * (xs[k // 2 - 1] + xs[k // 2])


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle's numpy/scipy restatement of the
# reference algorithm, timed on this host.  Workers are module-level so that
# spawned processes (which never touch the GPU) can import them.
# ---------------------------------------------------------------------------
def host_info():
    model = 'unknown'
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    quota = cgroup_cpu_quota()
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {'cpu_model': model, 'nproc': os.cpu_count(), 'affinity_cpus': aff,
            'cgroup_cpu_quota': quota, 'cores_used_all_core_leg': usable,
            'all_core_rule': 'every CPU the process may run on concurrently: the affinity '
                             'mask, capped by the cgroup CPU quota (cpu.max) when one is set'}


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants (cgroup v2 cpu.max 'quota period',
    v1 cfs_quota_us / cfs_period_us), or None when unlimited / unreadable.  The
    affinity mask can list far more CPUs than the quota lets run at once."""
    try:
        q, p = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        return None if q == 'max' else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        p = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def _cfg3_objective(n):
    from oracle import vb_oracle
    fam = vb_oracle.Family('gauss', D)
    return lambda lam: vb_oracle.klvi_value_grad(fam, 'isogauss', lam, n)


def _cfg3_cpu_run(n, steps, seed_shift=0):
    """`steps` adagrad steps of config 3 through the oracle's restatement of
    adagrad_optimize (vb.py:345-389); returns seconds."""
    import numpy as np
    from oracle import vb_oracle
    obj = _cfg3_objective(n)
    init = np.concatenate([np.zeros(D), np.ones(D)]) + 1e-3 * seed_shift
    vb_oracle.adagrad_optimize(3, obj, init)                     # warm-up
    t0 = time.perf_counter()
    vb_oracle.adagrad_optimize(steps, obj, init)
    return time.perf_counter() - t0


def _allcore_worker(barrier, queue, wid, rounds, fn_name, args):
    """One process of an all-core leg: `rounds` timed runs, each started
    together with the other workers behind a barrier."""
    for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ[k] = '1'
    fn = globals()[fn_name]
    fn(*args, warm=True)
    for r in range(rounds):
        barrier.wait()
        t0 = time.perf_counter()
        fn(*args, warm=False)
        queue.put((r, wid, time.perf_counter() - t0))


def _w_cfg3(n, steps, wid, warm):
    import numpy as np
    from oracle import vb_oracle
    obj = _cfg3_objective(n)
    init = np.concatenate([np.zeros(D), np.ones(D)]) + 1e-3 * wid
    vb_oracle.adagrad_optimize(2 if warm else steps, obj, init)


def _w_cfg5(restart_ids, iters, M, warm):
    for r in (restart_ids[:1] if warm else restart_ids):
        _cfg5_cpu_restart(r, 20 if warm else iters, 1000 if warm else M)


def _cfg5_cpu_restart(r, iters, M):
    """One config-5 restart on the CPU: mf-t(40) KLVI on 8-schools NCP, N=100,
    lr .01 -> .001, then M log weights -> divergence bound -> PSIS."""
    import warnings
    import numpy as np
    from oracle import vb_oracle, bounds_oracle, psis_oracle
    warnings.simplefilter('ignore')
    fam = vb_oracle.Family('t', 10, 40.0)
    init = np.random.RandomState(r).randn(20) * 0.5
    lam = vb_oracle.adagrad_optimize(
        iters, lambda l: vb_oracle.klvi_value_grad(fam, 'eight_schools_ncp', l, 100), init,
        learning_rate=.01, learning_rate_end=.001)[0]
    _, lw = vb_oracle.log_weights(fam, 'eight_schools_ncp', lam, M)
    bounds_oracle.divergence_bound(lw)
    psis_oracle.psislw(lw.copy())


def _run_allcore(fn_name, per_worker_args, rounds):
    """Spawned worker processes (numpy only, no GPU) run together; per round,
    the slowest worker's time bounds the round.  Returns per-round seconds."""
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    P = len(per_worker_args)
    barrier, queue = ctx.Barrier(P), ctx.Queue()
    procs = [ctx.Process(target=_allcore_worker, args=(barrier, queue, w, rounds, fn_name, a))
             for w, a in enumerate(per_worker_args)]
    for p in procs:
        p.start()
    per_round = {}
    for _ in range(P * rounds):
        r, _, dt = queue.get(timeout=600)
        per_round[r] = max(per_round.get(r, 0.0), dt)
    for p in procs:
        p.join()
    return [per_round[r] for r in range(rounds)]


def cpu_baseline_cfg3(host, n=N, runs=5, steps=200, allcore_rounds=3):
    """median of `runs` runs of `steps` adagrad steps, one core;
    then every usable core, one independent restart per process."""
    orig = None
    try:
        orig = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {sorted(orig)[0]})
    except (AttributeError, OSError):
        orig = None
    try:
        ts = [_cfg3_cpu_run(n, steps) for _ in range(runs)]
    finally:
        if orig is not None:
            os.sched_setaffinity(0, orig)
    single = n * D * steps / _median(ts)
    P = host['cores_used_all_core_leg']
    rts = _run_allcore('_w_cfg3', [(n, steps, w) for w in range(P)], allcore_rounds)
    allc = P * n * D * steps / _median(rts)
    return {
        'value': single, 'unit': 'MC-samples/s', 'cores': 1, 'kind': 'port',
        'sample': 'median of %d runs x %d KLVI adagrad steps at N=%d, D=%d (oracle/vb_oracle.py '
                  'adagrad_optimize = vb.py:345-389 restated, numpy legacy RandomState noise, '
                  'one pinned core, BLAS threads 1); run seconds %s'
                  % (runs, steps, n, D, [round(t, 3) for t in ts]),
        'all_cores': {'value': allc, 'unit': 'MC-samples/s', 'cores': P,
                      'sample': '%d spawned processes x %d steps (independent restarts), '
                                'median of %d barrier-started rounds, slowest worker per round; '
                                'round seconds %s' % (P, steps, allcore_rounds,
                                                     [round(t, 3) for t in rts])},
        'host': host,
    }


# ---------------------------------------------------------------------------
# GPU legs
# ---------------------------------------------------------------------------
def run_cfg3(torch, stream, dev, n, steps, warmup, rank, dist):
    """Config 3 (mf-Gauss KLVI, isogauss D = 1e4, Philox) for `steps` timed
    steps after `warmup` untimed ones, in launches of at most CHUNK steps.  The
    library brackets every launch (sep_kernel + its per-step value reduction)
    with HIP events on the launch stream (vb_run_set_timing), so the timed
    loop makes one host call per launch.  Returns (elapsed max over ranks,
    [(steps, history rows, seconds) per timed launch], run)."""
    import numpy as np
    from viabel_amd import targets, vb
    fam = vb.mean_field_gaussian_variational_family(D, rng='philox')
    obj = vb.black_box_klvi(fam, targets.isogauss(D), n)
    init = np.concatenate([np.zeros(D), np.ones(D)])
    run = vb.DeviceRun(obj, warmup + steps, init[None, :], window=WINDOW, learning_rate=LR,
                       epsilon=EPS)
    run.set_timing(True)
    seed, strm = 0, 1 + rank          # one restart per rank, independent Philox streams
    hist_start = 3 * (warmup + steps) // 4        # vb.py:375-376
    # the W warm-up steps take the same host path as the timed launches
    done = 0
    while done < warmup:
        cs = min(CHUNK, warmup - done)
        run.advance_philox(cs, seed, strm, done)
        done += cs
    torch.cuda.synchronize(dev)
    run.launch_times()                            # drop the warm-up records
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    done = 0
    while done < steps:
        cs = min(CHUNK, steps - done)
        run.advance_philox(cs, seed, strm, warmup + done)
        done += cs
    torch.cuda.synchronize(dev)
    # no closing barrier: every rank stops its own clock when its work is done, and
    # the MAX all-reduce below gives the job's wall time from the aligned start
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    launches, s0 = [], warmup
    for k, sec in run.launch_times():
        launches.append((k, max(0, s0 + k - max(s0, hist_start)), sec))
        s0 += k
    return elapsed, launches, run


COLL_CPU = False   # collectives on host tensors (gloo rehearsal, see main)


def coll_device(dev):
    """Device of the tensors handed to collectives: the rank's GPU under RCCL, the
    host under the gloo rehearsal backend."""
    import torch
    return torch.device('cpu') if COLL_CPU else dev


# the round whose committed counter passes (profiles/<round>/) price the bench line
PROFILE_ROUND = 'r06'


def load_traffic():
    p = os.path.join(ROOT, 'profiles', 'traffic.json')
    try:
        return json.load(open(p))
    except (OSError, ValueError):
        return None


def load_valu_busy():
    """The headline launch's VALU busy fraction measured with rocprofv3 PMC
    (SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs): the
    fraction of SIMD cycles issuing a VALU instruction, at the clock the launch ran
    at), from the committed record scripts/gpu_valu_busy.sh wrote.  A measured
    counterpart to the instruction-count model's frac, which prices every VALU
    instruction at 4 cycles."""
    p = os.path.join(ROOT, 'profiles', PROFILE_ROUND, 'valu_busy_headline.json')
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    disp = d.get('dispatches') or []
    return {'busy': d.get('timed_dispatch_valu_busy'),
            'clock_ghz': disp[-1].get('clock_ghz') if disp else None,
            'formula': d.get('formula'),
            'source': 'profiles/%s/valu_busy_headline.json (raw counters: '
                      'valu_busy_headline_counters.csv beside it)' % PROFILE_ROUND}


def roofline_cfg3(launches, n, traffic):
    """Dominant kernel: sep_kernel (+ its per-step value reduction, one launch
    pair per advance call).  Bytes and VALU instructions are priced for the
    steps each launch actually ran."""
    steps = sum(k for k, _, _ in launches)
    secs = sum(t for _, _, t in launches)
    per_step = algorithmic_bytes_per_step(n, D, WINDOW)
    achieved = steps * per_step / secs / 1e9
    out = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
           'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
           'kernel': 'sep_kernel<IsoGauss,gauss,philox> + sep_values_kernel',
           'launches': len(launches), 'steps_per_launch': [k for k, _, _ in launches][:4],
           'launch_ms_mean': secs / len(launches) * 1e3,
           'algorithmic_bytes_per_step': per_step,
           'algorithmic_bytes_per_launch_mean': steps * per_step / len(launches)}
    valu = None
    m = (traffic or {}).get('models', {}).get(str(n))
    if m:
        # linear per-launch models fitted to PMC passes at several launch lengths
        a, b, c = m['traffic_bytes']
        tb = sum(a + b * k + c * h for k, h, _ in launches)
        out['traffic'] = tb / len(launches)
        out['traffic_source'] = traffic.get('source')
        vi = sum(m['valu_instr'][0] + m['valu_instr'][1] * k for k, _, _ in launches)
        rate = vi / secs / 1e9
        valu = {'instr_per_launch_mean': vi / len(launches), 'achieved': rate,
                'peak': VALU_PEAK_GINSTR, 'unit': 'G wave-instr/s',
                'frac': rate / VALU_PEAK_GINSTR,
                'source': 'SQ_INSTS_VALU per-launch model (a + b x steps) from rocprofv3 --pmc '
                          '(profiles/traffic.json) / live launch time; peak = 256 CUs x 4 SIMDs '
                          'x 2.4 GHz / 4 cycles per wave64 fp64 instruction'}
    return out, valu


def leg_cfg3_n256(torch, stream, dev, traffic, steps=2048, warmup=64):
    n = 256
    elapsed, launches, _ = run_cfg3(torch, stream, dev, n, steps, warmup, 0, None)
    roof, valu = roofline_cfg3(launches, n, traffic)
    return {'config': 3, 'workload': 'isogauss D=1e4 mf-Gauss KLVI adagrad, N=256 (config-3 text)',
            'steps': steps, 'warmup': warmup, 'ms_per_step': elapsed / steps * 1e3,
            'value': steps * n * D / elapsed, 'unit': 'MC-samples/s', 'roofline': roof,
            'valu': valu}


def measure_peaks():
    """the roofline peaks confirmed with microbenchmarks on this box
    (vb_peak_probe, best of 5 launches each): HBM copy and read over 1 GiB buffers
    (4x the Infinity Cache), the fp64 MFMA loop, and the VALU issue rate of fp64
    FMA and u64 multiply chains (4 waves per SIMD)."""
    from viabel_amd import _native as nat
    out = {}
    for k, n in (('hbm_copy', 1 << 30), ('hbm_read', 1 << 30), ('mfma_f64', 20000),
                 ('valu_fma_f64', 20000), ('valu_mad_u64', 20000)):
        try:
            out[k] = nat.peak_probe(k, n)
        except Exception as e:      # reported, never hidden
            out[k] = None
            out[k + '_error'] = str(e)
    out['units'] = {'hbm_copy': 'GB/s (read + written)', 'hbm_read': 'GB/s', 'mfma_f64': 'TFLOP/s',
                    'valu_fma_f64': 'G wave-instr/s', 'valu_mad_u64': 'G wave-instr/s'}
    out['source'] = 'vb_peak_probe (viabel_amd/csrc/vb_probe.hip), measured in this run'
    return out


# the HBM copy rate MI355X_MICROARCH.md measured (float4 copy); the probe's best copy
# form reaches ~5.7 TB/s on the box (profiles/r05/hbm_probe2.log), so HBM rooflines
# carry the fraction against this figure too
GUIDE_HBM_COPY_GBS = 6290.0


def add_measured(roof, measured, key):
    """frac against the measured peak beside the spec one (and, for HBM, against the
    guide's measured copy rate)."""
    m = measured.get(key) if measured else None
    if roof and m and roof.get('achieved'):
        roof['measured_peak'] = m
        roof['measured_peak_source'] = key
        roof['frac_of_measured_peak'] = roof['achieved'] / m
    if roof and roof.get('achieved') and key == 'hbm_copy':
        roof['guide_copy_peak'] = GUIDE_HBM_COPY_GBS
        roof['frac_of_guide_copy_peak'] = roof['achieved'] / GUIDE_HBM_COPY_GBS


def _sync():
    from viabel_amd import _native as nat
    nat.context().synchronize()


def leg_cfg1(cpu):
    """2-D normal mixture, mf-Gauss KLVI, N = 100, 5 000 adagrad iterations
    (config 1; latency-bound: one workgroup)."""
    import numpy as np
    from viabel_amd import vb, targets
    Dm, n, iters = 2, 100, 5000
    lam0 = np.array([0., 0., 1., 1.])
    fam = vb.mean_field_gaussian_variational_family(Dm, rng='philox')
    obj = vb.black_box_klvi(fam, targets.mixture(Dm), n)
    # warm-up at the timed call's shapes (its buffers then come from the library's
    # device block cache, as in any later call of a long-running program)
    vb.adagrad_optimize(iters, obj, lam0)
    _sync()
    t0 = time.perf_counter()
    vb.adagrad_optimize(iters, obj, lam0)
    _sync()
    dt = (time.perf_counter() - t0) / iters
    out = {'config': 1, 'workload': 'mixture D=2 mf-Gauss KLVI N=100, 5000 iters (adagrad_optimize '
                                   'incl. result copy)', 'ms_per_step': dt * 1e3,
           'steps_per_s': 1 / dt, 'value': n * Dm / dt, 'unit': 'MC-samples/s',
           'roofline': latency_roofline(dt, Dm, n, chivi=False,
                                        host_layout=gauss_runs_predraw(), n_problems=1,
                                        note='one workgroup per problem; D=2 moves 64 B of '
                                             'parameters per step; the Gaussian draws are '
                                             'pre-drawn and staged by the copy wave unless '
                                             'VIABEL_AMD_PREDRAW is 0 or t')}
    if cpu:
        from oracle import vb_oracle
        ofam = vb_oracle.Family('gauss', Dm)
        obj_c = lambda l: vb_oracle.klvi_value_grad(ofam, 'mixture', l, n)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            vb_oracle.adagrad_optimize(2000, obj_c, lam0)
            ts.append((time.perf_counter() - t0) / 2000)
        out['cpu_baseline'] = {'value': n * Dm / _median(ts), 'unit': 'MC-samples/s', 'cores': 1,
                               'kind': 'port', 'ms_per_step': _median(ts) * 1e3,
                               'sample': 'median of 5 x 2000 oracle adagrad steps'}
        out['speedup_vs_cpu'] = _median(ts) / dt
    return out


def leg_cfg2(cpu):
    """Funnel D = 10, mf-t(40) CHIVI alpha = 2, N = 128, lr .01 -> .001, 10 000 iterations."""
    import numpy as np
    from viabel_amd import vb, targets
    Dm, n, iters = 10, 128, 10000
    lam0 = np.concatenate([np.zeros(Dm), np.ones(Dm)])
    lam0[1] = -1.0
    fam = vb.mean_field_t_variational_family(Dm, 40.0, rng='philox')
    obj = vb.black_box_chivi(2.0, fam, targets.funnel(Dm), n)
    # (warm-up at the timed call's shapes, as config 1's)
    vb.adagrad_optimize(iters, obj, lam0, learning_rate=.01, learning_rate_end=.001)
    _sync()
    t0 = time.perf_counter()
    vb.adagrad_optimize(iters, obj, lam0, learning_rate=.01, learning_rate_end=.001)
    _sync()
    dt = (time.perf_counter() - t0) / iters
    out = {'config': 2, 'workload': 'funnel D=10 mf-t(40) CHIVI a=2 N=128, 10000 iters',
           'ms_per_step': dt * 1e3, 'value': n * Dm / dt, 'unit': 'MC-samples/s',
           'roofline': latency_roofline(dt, Dm, n, chivi=True, host_layout=True, n_problems=1,
                                        note='one workgroup; t draws pre-drawn chunk by chunk '
                                             'over the chip (pre-draw kernels inside the timed '
                                             'run), the block consumes them')}
    if cpu:
        from oracle import vb_oracle
        ofam = vb_oracle.Family('t', Dm, 40.0)
        np.random.seed(0)
        obj_c = lambda l: vb_oracle.chivi_value_grad(ofam, 'funnel', l, n, 2.0)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            vb_oracle.adagrad_optimize(400, obj_c, lam0, learning_rate_end=.001)
            ts.append((time.perf_counter() - t0) / 400)
        out['cpu_baseline'] = {'value': n * Dm / _median(ts), 'unit': 'MC-samples/s', 'cores': 1,
                               'kind': 'port', 'ms_per_step': _median(ts) * 1e3,
                               'sample': 'median of 5 x 400 oracle adagrad steps'}
        out['speedup_vs_cpu'] = _median(ts) / dt
    return out


def gauss_runs_predraw():
    """Whether Gaussian-family runs pre-draw their noise (vb_capi.hip
    predraw_enabled: the default unless VIABEL_AMD_PREDRAW is 0 or t), so the
    block kernel runs its device-noise layout (row waves + copy wave)."""
    e = os.environ.get('VIABEL_AMD_PREDRAW', '')
    return not (e.startswith('0') or e.startswith('t'))


def latency_roofline(step_s, d, n, chivi, host_layout, n_problems, note):
    """Roofline of a latency-bound block-kernel leg: the measured floor of its step
    skeleton (vb_block_floor: the same block shape, barriers, reductions and
    adagrad update, no draws and no target, on the same grid) against the
    achieved time per step; frac = floor / achieved."""
    from viabel_amd import _native as nat
    fl = min(nat.block_floor_us(d, n, chivi=chivi, host_layout=host_layout, n_steps=2000,
                                n_problems=n_problems) for _ in range(3))
    us = step_s * 1e6
    return {'bound': 'latency', 'floor_us': fl, 'achieved_us': us, 'unit': 'us/step',
            'achieved_over_floor': us / fl, 'frac': fl / us,
            'floor_source': 'vb_block_floor, best of 3 x 2000 steps',
            'note': note}


def cfg5_stage_valu(stage_s, local, n_restarts):
    """VALU issue fraction of config 5's bounds / PSIS stage: the stage's
    SQ_INSTS_VALU from a committed counter pass over the same stage
    (profiles/<round>/cfg5/bounds_stage_pmc.json, scripts/gpu_cfg5_pmc.sh; 64
    restarts x M = 1e6, scaled to this rank's restarts) over the live stage time."""
    p = os.path.join(ROOT, 'profiles', PROFILE_ROUND, 'cfg5', 'bounds_stage_pmc.json')
    try:
        prof = json.load(open(p))
    except (OSError, ValueError):
        return None
    if not stage_s:
        return None
    vi = prof['stage']['valu_instr'] * local / n_restarts
    k = prof['kernels'].get('logw_row_kernel<vbd::EightSchools, true, false, 10>', {})
    return {'valu_instr': vi, 'achieved': vi / stage_s / 1e9, 'peak': VALU_PEAK_GINSTR,
            'unit': 'G wave-instr/s', 'frac': vi / stage_s / 1e9 / VALU_PEAK_GINSTR,
            'logw_kernel_valu_frac': k.get('valu_frac'),
            'source': 'SQ_INSTS_VALU of the stage (profiles/%s/cfg5/bounds_stage_pmc.json; raw '
                      'counters bounds_stage_sq_counters.csv beside it) / live stage seconds; the '
                      'log-weight kernel fraction is from the profile' % PROFILE_ROUND}


def _cfg4_problem():
    import numpy as np
    Dm = 512
    rs = np.random.RandomState(4)
    tri = np.tril_indices(Dm)
    free = rs.randn(len(tri[0])) * 0.01
    free[tri[0] == tri[1]] = rs.randn(Dm) * 0.1
    return Dm, np.concatenate([np.zeros(Dm), free])


def _w_cfg4_blas(steps, wid, warm):
    """all-core config-4 CPU leg: one process, BLAS threads = cores."""
    import numpy as np
    from oracle import fullrank_oracle as fo
    Dm, lam0 = _cfg4_problem()
    ofam = fo.FullRankT(Dm, 100.0)
    otgt = fo.target_fn('corr_gauss', Dm)
    np.random.seed(0)
    for _ in range(1 if warm else steps):
        fo.chivi_value_grad(ofam, otgt, lam0, 128, 2.0)


def leg_cfg4(cpu, host, steps=30):
    """Full-rank t D = 512 df = 100, CHIVI alpha = 2, N = 128, corr_gauss target
    (the fp64 MFMA path)."""
    import numpy as np
    from viabel_amd import vb, targets
    Dm, lam0 = _cfg4_problem()
    n = 128
    fam = vb.t_variational_family(Dm, 100.0, rng='philox')
    obj = vb.black_box_chivi(2.0, fam, targets.corr_gauss(Dm), n)
    run = vb.DeviceRun(obj, steps + 3, lam0)
    run.advance_philox(3, 0, 1, 0)
    _sync()
    from viabel_amd import _native as nat
    nat.lib().vb_flop_tally(1)
    t0 = time.perf_counter()
    run.advance_philox(steps, 0, 1, 3)
    _sync()
    dt = (time.perf_counter() - t0) / steps
    # matrix-core flops of the products the timed advance launched (library tally)
    exec_flops = nat.lib().vb_flop_tally(0) / steps
    flops = 8 * n * Dm * Dm + 20 * Dm ** 3          # SURVEY §8d config 4 algorithmic flops / step
    ach = flops / dt / 1e12
    out = {'config': 4, 'workload': 'full-rank t D=512 df=100 CHIVI a=2 N=128 corr_gauss, adagrad',
           'steps': steps, 'ms_per_step': dt * 1e3, 'value': n * Dm / dt, 'unit': 'MC-samples/s',
           'roofline': {'bound': 'mfma', 'achieved': ach, 'peak': FP64_PEAK_TFLOPS,
                        'unit': 'TFLOP/s', 'frac': ach / FP64_PEAK_TFLOPS,
                        'algorithmic_flops_per_step': flops,
                        'executed_flops_per_step': exec_flops,
                        'executed_tflops': exec_flops / dt / 1e12,
                        'executed_frac': exec_flops / dt / 1e12 / FP64_PEAK_TFLOPS,
                        'note': 'whole step (all launches) timed on the host clock; flops = '
                                '8 N D^2 + 20 D^3 (SURVEY §8d); executed_* = the matrix-core '
                                'flops of every product the timed steps launched (tiles x tile '
                                'area x depth x 2, counted by the library: vb_flop_tally)'}}
    if cpu:
        from oracle import fullrank_oracle as fo
        ofam = fo.FullRankT(Dm, 100.0)
        otgt = fo.target_fn('corr_gauss', Dm)
        np.random.seed(0)
        fo.chivi_value_grad(ofam, otgt, lam0, n, 2.0)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fo.chivi_value_grad(ofam, otgt, lam0, n, 2.0)
            ts.append(time.perf_counter() - t0)
        out['cpu_baseline'] = {'value': n * Dm / _median(ts), 'unit': 'MC-samples/s', 'cores': 1,
                               'kind': 'port', 'ms_per_step': _median(ts) * 1e3,
                               'sample': 'median of 5 CHIVI value+grad evaluations (scipy sqrtm '
                                         '+ solve_sylvester VJP: the reference algorithm), BLAS '
                                         'threads 1'}
        out['speedup_vs_cpu'] = _median(ts) / dt
        P = host['cores_used_all_core_leg']
        saved = {k: os.environ.get(k) for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS')}
        for k in saved:
            os.environ[k] = str(P)
        try:
            rts = _run_allcore_threads('_w_cfg4_blas', (2, 0), 1)
        finally:
            for k, v in saved.items():
                os.environ[k] = v if v is not None else '1'
        out['cpu_baseline']['all_cores'] = {
            'value': n * Dm * 2 / rts[0], 'unit': 'MC-samples/s', 'cores': P,
            'ms_per_step': rts[0] / 2 * 1e3,
            'sample': 'one process, BLAS threads = %d, 2 CHIVI value+grad evaluations' % P}
    return out


def _threaded_worker(queue, fn_name, args):
    fn = globals()[fn_name]
    fn(*args, warm=True)
    t0 = time.perf_counter()
    fn(*args, warm=False)
    queue.put(time.perf_counter() - t0)


def _run_allcore_threads(fn_name, args, rounds):
    """One spawned process inheriting the current BLAS thread settings."""
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    out = []
    for _ in range(rounds):
        q = ctx.Queue()
        p = ctx.Process(target=_threaded_worker, args=(q, fn_name, args))
        p.start()
        out.append(q.get(timeout=600))
        p.join()
    return out


def leg_cfg5(cpu, host, rank, world, n_restarts=64, iters=5000, M=1_000_000):
    """8-schools NCP, 64 KLVI restarts (mf-t df = 40, N = 100, lr .01 -> .001)
    + divergence / Wasserstein bounds and PSIS on M = 1e6 log weights each,
    sharded restart r -> rank r mod world, one RCCL all_gather of the records."""
    import numpy as np
    import torch
    from viabel_amd import vb, targets, restarts
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    # warm-up: code objects, and the timed call's buffer shapes for the device
    # allocators (torch's for the [restarts][M] log weights, the library's block
    # cache for the runs), i.e. the same call once untimed
    restarts.run_restarts(fac, tgt, n_restarts, iters, n_samples=100, n_bounds=M,
                          learning_rate=.01, learning_rate_end=.001)
    _sync()
    dist = torch.distributed if world > 1 else None
    # the restarts' initial parameters are the job's input, made before the timed
    # region like every other leg's inputs (the same values run_restarts draws when
    # none are given: RandomState(r).randn(P) * 0.5, ~0.5 ms of host time at 64)
    inits = restarts.default_inits(n_restarts, fac().var_param_dim)
    if dist:
        dist.barrier()
    tm = {}
    t0 = time.perf_counter()
    tab = restarts.run_restarts(fac, tgt, n_restarts, iters, n_samples=100, n_bounds=M,
                                learning_rate=.01, learning_rate_end=.001, inits=inits,
                                timings=tm)
    _sync()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt, tm.get('bounds_psis_s', 0.0), tm.get('fit_s', 0.0)],
                         dtype=torch.float64,
                         device=coll_device(torch.device('cuda', torch.cuda.current_device())))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, tm['bounds_psis_s'], tm['fit_s'] = t.tolist()
    local = len(restarts.shard(n_restarts, rank, world))
    # bounds/PSIS stage bytes per restart: 8 M D draws + 8 M lw write
    # + 8 M bounds read + 16 M PSIS read + write
    b_stage = local * M * (8 * 10 + 32)
    ach = b_stage / tm['bounds_psis_s'] / 1e9 if tm.get('bounds_psis_s') else None
    out = {'config': 5, 'workload': '8-schools NCP, %d KLVI restarts x %d iters (mf-t df=40, N=100) '
                                   '+ M=%d log weights, bounds, PSIS per restart' % (n_restarts, iters, M),
           'n_gpus': world, 'seconds': dt, 'value': n_restarts / dt, 'unit': 'restarts/s',
           'fit_s': tm.get('fit_s'), 'bounds_psis_s': tm.get('bounds_psis_s'),
           'local_s': tm.get('local_s'),
           'finite_khat': bool(np.all(np.isfinite(tab[:, 8]))),
           'khat_range': [float(np.min(tab[:, 8])), float(np.max(tab[:, 8]))],
           'roofline': {'bound': 'hbm', 'stage': 'log weights + bounds + PSIS (max over ranks)',
                        'achieved': ach, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                        'frac': ach / HBM_PEAK_GBS if ach else None,
                        'algorithmic_bytes_per_rank': b_stage,
                        'note': 'fitting is latency-bound (one workgroup per restart): fit_roofline'},
           'bounds_valu': cfg5_stage_valu(tm.get('bounds_psis_s'), local, n_restarts),
           'fit_roofline': (latency_roofline(tm['fit_s'] / iters, 10, 100, chivi=False,
                                             host_layout=True, n_problems=local,
                                             note='one workgroup per restart, %d restarts on this '
                                                  'rank; the fit (pre-draw + block kernels) per '
                                                  'step' % local)
                            if tm.get('fit_s') else None)}
    if cpu:
        t0 = time.perf_counter()
        _cfg5_cpu_restart(0, iters, M)
        one = time.perf_counter() - t0
        P = host['cores_used_all_core_leg']
        ids = [list(range(w, n_restarts, P)) for w in range(P)]
        rts = _run_allcore('_w_cfg5', [(i, iters, M) for i in ids], 1)
        out['cpu_baseline'] = {
            'value': 1 / one, 'unit': 'restarts/s', 'cores': 1, 'kind': 'port',
            'seconds_64_restarts_extrapolated': one * n_restarts,
            'sample': 'one full restart (5000 oracle adagrad steps + M=1e6 log weights, '
                      'divergence bound, psislw) on one core, x64 extrapolated',
            'all_cores': {'value': n_restarts / rts[0], 'unit': 'restarts/s', 'cores': P,
                          'seconds': rts[0],
                          'sample': 'all %d restarts measured, %d processes (one per core), '
                                    'restarts dealt round-robin' % (n_restarts, P)}}
        out['speedup_vs_cpu_1core'] = one * n_restarts / dt
        out['speedup_vs_cpu_all_cores'] = rts[0] / dt
    return out


def leg_khat(cpu):
    """PSIS k-hat match (metric suffix): fit restart 0 of config 5, draw M = 1e6
    log weights on the device, run device psislw (timed) and, in the CPU-baseline
    leg, the oracle psislw on the same vector: |k_device - k_cpu| and whether
    the tail order tailinds[x2si] is identical."""
    import numpy as np
    import torch
    from viabel_amd import vb, targets, experiments, psis
    M = 1_000_000
    fam = vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tgt = targets.eight_schools_ncp()
    init = np.random.RandomState(0).randn(20) * 0.5
    obj = vb.black_box_klvi(fam, tgt, 100)
    lam = vb.adagrad_optimize(5000, obj, init, learning_rate=.01, learning_rate_end=.001)[0]
    lw = torch.empty(M, dtype=torch.float64, device=torch.device('cuda', torch.cuda.current_device()))
    experiments.log_weights(tgt, fam, lam, M, return_samples=False, lw_out=lw)
    psis.psislw_with_tail(lw)                                    # warm-up
    _sync()
    t0 = time.perf_counter()
    _, kd, tails = psis.psislw_with_tail(lw)
    _sync()
    t_dev = time.perf_counter() - t0
    out = {'workload': 'psislw on M=1e6 log weights of a fitted 8-schools NCP mf-t(40) q',
           'k_device': float(kd[0]), 'device_ms': t_dev * 1e3,
           'value': M / t_dev, 'unit': 'log-weights/s'}
    if cpu:
        from oracle import psis_oracle
        host_lw = lw.cpu().numpy()
        t0 = time.perf_counter()
        _, kc, tc = psis_oracle.psislw(host_lw.copy(), return_tail=True)
        t_cpu = time.perf_counter() - t0
        kc = float(np.atleast_1d(kc)[0])
        tcpu = np.asarray(tc[0] if isinstance(tc, (list, tuple)) else tc)
        out.update({'k_cpu': kc, 'abs_diff': abs(float(kd[0]) - kc),
                    'rel_diff': abs(float(kd[0]) - kc) / max(abs(kc), 1e-300),
                    'tail_len': int(len(tails[0])),
                    'tail_order_identical': bool(len(tcpu) == len(tails[0]) and
                                                 np.array_equal(tcpu, tails[0])),
                    'match_1e-5': bool(abs(float(kd[0]) - kc) <= 1e-5 * max(1.0, abs(kc))),
                    'cpu_baseline': {'value': M / t_cpu, 'unit': 'log-weights/s', 'cores': 1,
                                     'kind': 'port', 'ms': t_cpu * 1e3,
                                     'sample': 'oracle psislw (psis.py:112-208 restated) on '
                                               'the same 1e6 vector'}})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=100)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--n-samples', type=int, default=N,
                    help='headline N (profiling passes only; the metric is quoted at 128)')
    ap.add_argument('--legs', default='all',
                    help="'all', 'none' or a comma list of cfg3_256,cfg1,cfg2,cfg4,cfg5,khat")
    args = ap.parse_args()

    import numpy as np
    import torch

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    # one GPU per rank (LOCAL_RANK mod the visible devices, as restarts.bind_local_device);
    # collectives over nccl (= RCCL) whenever every local rank has a GPU of its own;
    # more local ranks than GPUs (a rehearsal of the N > 1 path on a one-GPU box,
    # scripts/gpu_rehearse_ranks.sh) use gloo, since RCCL refuses two ranks on one GPU.
    # A launcher that does not export LOCAL_WORLD_SIZE gets nccl (the production
    # case: one rank per GPU); VIABEL_AMD_BENCH_BACKEND overrides the choice.
    global COLL_CPU
    n_dev = max(1, torch.cuda.device_count())
    lws = os.environ.get('LOCAL_WORLD_SIZE')
    backend = 'nccl' if lws is None or int(lws) <= n_dev else 'gloo'
    backend = os.environ.get('VIABEL_AMD_BENCH_BACKEND', backend)
    if backend not in ('nccl', 'gloo'):
        raise ValueError('VIABEL_AMD_BENCH_BACKEND must be nccl or gloo')
    local_world = int(lws) if lws is not None else world
    local_dev = local % n_dev
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_dev)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local_dev))
        else:
            dist.init_process_group(backend)
            COLL_CPU = True
            if rank == 0:
                print('[bench] %d local ranks on %d GPU(s): gloo collectives (rehearsal)'
                      % (local_world, n_dev), file=sys.stderr, flush=True)
    else:
        torch.cuda.set_device(0)
    dev = torch.device('cuda', local_dev)

    from viabel_amd import _native as nat
    # a dedicated (non-NULL) stream: the kernels and the timing events share it
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    nat.use_stream(local_dev, stream.cuda_stream)
    traffic = load_traffic()

    K, W, NS = args.steps, args.warmup, args.n_samples
    elapsed, launches, run = run_cfg3(torch, stream, dev, NS, K, W, rank, dist)
    roof, valu = roofline_cfg3(launches, NS, traffic)

    # restart summaries gathered over RCCL (the only collective)
    lam, hist, vals, smooth = run.result()
    summary = torch.tensor([float(vals[0, -1]), float(np.mean(vals[0, -100:])),
                            float(np.linalg.norm(smooth[0]))], dtype=torch.float64,
                           device=coll_device(dev))
    if dist:
        gathered = [torch.empty_like(summary) for _ in range(world)]
        dist.all_gather(gathered, summary)
        gathered = torch.stack(gathered).cpu().numpy()
    else:
        gathered = summary.cpu().numpy()[None]
    value = world * K * NS * D / elapsed

    legs = [] if args.legs == 'none' else (
        ['cfg3_256', 'cfg1', 'cfg2', 'cfg4', 'cfg5', 'khat'] if args.legs == 'all'
        else args.legs.split(','))
    if world > 1:
        legs = [l for l in legs if l == 'cfg5']      # the sharded config; others are per-GPU
    cpu = not args.no_cpu_baseline and world == 1 and rank == 0
    host = host_info() if cpu else None
    configs = {}
    for leg in legs:
        t_leg = time.perf_counter()
        try:
            if leg == 'cfg3_256':
                configs[leg] = leg_cfg3_n256(torch, stream, dev, traffic)
            elif leg == 'cfg1':
                configs[leg] = leg_cfg1(cpu)
            elif leg == 'cfg2':
                configs[leg] = leg_cfg2(cpu)
            elif leg == 'cfg4':
                configs[leg] = leg_cfg4(cpu, host)
            elif leg == 'cfg5':
                configs[leg] = leg_cfg5(cpu, host, rank, world)
            elif leg == 'khat':
                configs[leg] = leg_khat(cpu)
        except Exception as e:       # a failed leg is reported, never hidden
            configs[leg] = {'error': '%s: %s' % (type(e).__name__, e)}
        configs[leg]['leg_seconds'] = time.perf_counter() - t_leg
        if rank == 0:
            print('[bench] leg %s done in %.1f s' % (leg, configs[leg]['leg_seconds']),
                  file=sys.stderr, flush=True)

    measured = measure_peaks() if rank == 0 else None
    add_measured(roof, measured, 'hbm_copy')
    if valu and measured and measured.get('valu_fma_f64'):
        valu['measured_fma_f64_peak'] = measured['valu_fma_f64']
        valu['frac_of_measured_fma_f64_peak'] = valu['achieved'] / measured['valu_fma_f64']
    if valu:
        busy = load_valu_busy()
        if busy:
            valu['pmc_busy'] = busy
    for leg, key in (('cfg3_256', 'hbm_copy'), ('cfg4', 'mfma_f64'), ('cfg5', 'hbm_copy')):
        if isinstance(configs.get(leg), dict):
            add_measured(configs[leg].get('roofline'), measured, key)

    if rank == 0:
        line = {
            'metric': METRIC,
            'value': value, 'unit': 'MC-samples/s', 'n_gpus': world, 'steps': K, 'warmup': W,
            'ms_per_step': elapsed / K * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
            'config': {'workload': 'mean-field Gaussian KLVI + adagrad on isotropic Gaussian '
                                   'target (SURVEY config 3)',
                       'D': D, 'N': NS, 'window': WINDOW, 'learning_rate': LR, 'epsilon': EPS,
                       'rng': 'philox', 'restarts': world,
                       'parallelism': 'restarts sharded 1/GPU, RCCL all_gather of summaries'},
            'roofline': roof,
            'valu': valu,
            'measured_peaks': measured,
            'build_id': nat.lib().vb_build_id().decode(),
            'restart_summaries': gathered.tolist(),
        }
        if cpu:
            line['cpu_baseline'] = cpu_baseline_cfg3(host)
            line['speedup_vs_cpu_baseline'] = value / line['cpu_baseline']['value']
            line['speedup_vs_cpu_all_cores'] = value / line['cpu_baseline']['all_cores']['value']
        if 'khat' in configs:
            line['khat_match'] = configs.pop('khat')
        line['configs'] = configs
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    # the CPU-baseline legs are single-threaded numpy (set before numpy loads)
    for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ.setdefault(k, '1')
    os.environ.setdefault('VIABEL_AMD_PROGRESS', '0')     # no progress bars in the legs
    main()
