"""Independent optimisation restarts sharded over GPUs.

The reference's restart loop (rmsprop_IA_optimize_with_rhat, viabel/vb.py:
417-421) runs restarts one after another on one CPU.  Here restart r lives on
rank r % world; each rank runs all of its restarts in ONE device-resident
adagrad launch chain (vb_run with n_problems = local restarts, one workgroup
per restart), then, per restart, draws M log weights on the device and reduces
them to the divergence / Wasserstein bounds (viabel/bounds.py) and the PSIS
k-hat (notebooks/psis.py).  The only collective is one all_gather of a
fixed-size summary record per restart at the end (RCCL over xGMI on the GPU
pool; gloo in the CPU tests).  There is no data-path collective.

Summary record (float64), per restart:
  [restart id, ELBO estimate (mean log weight), CUBO-based d2, W1, W2,
   mean_error, std_error, cov_error, k_hat, final objective value, lambda*(P)]
"""
import os
import time

import numpy as np

from . import _native as nat

__all__ = ['shard', 'run_restarts', 'gather_records', 'bind_local_device', 'bounds_records',
           'RECORD_HEAD']

RECORD_HEAD = ['restart', 'elbo', 'd2', 'W1', 'W2', 'mean_error', 'std_error', 'cov_error',
               'khat', 'final_value']


def shard(n_restarts, rank, world):
    """Restart ids owned by `rank`: r = rank, rank + world, ..."""
    return list(range(rank, n_restarts, world))


def default_inits(n_restarts, P, scale=0.5, base=None):
    """init_r = base + RandomState(r).randn(P) * scale (SURVEY §8d config 5,
    the fixed-scale variant of vb.py:420-421)."""
    base = np.zeros(P) if base is None else np.asarray(base, dtype=float)
    # one generator re-seeded per restart: the same streams as RandomState(r),
    # without constructing 64 generator objects (~15 ms of host time)
    rs = np.random.RandomState(0)
    out = np.empty((n_restarts, P))
    for r in range(n_restarts):
        rs.seed(r)
        out[r] = base + rs.randn(P) * scale
    return out


def bind_local_device(rank=0):
    """Select this rank's GPU before any allocation: LOCAL_RANK (set by
    torchrun) or the global rank, modulo the visible device count.  The vb
    context (nat.set_device) and torch's current device (used by the NCCL
    all_gather) then name the same GPU."""
    import torch
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError('run_restarts: no GPU visible to rank %d' % rank)
    dev = int(os.environ.get('LOCAL_RANK', rank)) % n
    torch.cuda.set_device(dev)
    nat.set_device(dev)
    return dev


def _sync():
    nat.context().synchronize()


# the batched bound-draw kernel (vb_log_weights_rows) covers the block kernel's
# target dimensions (vb_internal.hpp kBlockDMax) or separable targets at any D
_ROWS_DMAX = 16


def _rows_supported(fam, target):
    """Whether vb_log_weights_rows accepts this family and target
    (vb_capi.hip vb_log_weights_rows: mean-field family, device target,
    separable or D <= 16)."""
    from .targets import Target
    if fam.kind == nat.FAMILY_FR_T or not isinstance(target, Target):
        return False
    if target.kind == nat.TARGET_CALLBACK:
        return False
    return target.separable or fam.dim <= _ROWS_DMAX


def _native_compute(ids, inits, family_factory, target, n_iters, n_samples, n_bounds,
                    learning_rate, learning_rate_end, window, seed, stream_base, stride,
                    timings=None):
    """Fit this rank's restarts in ONE device run (one workgroup per restart;
    restart r draws from Philox stream 1 + r whatever the sharding) and
    summarise each with device log weights, bounds and PSIS.  `timings`, if a
    dict, receives the seconds of the fitting and of the bounds/PSIS stage."""
    t_entry = time.perf_counter()
    from . import vb, bounds, psis, experiments
    fam = family_factory()
    if fam.rng != 'philox':
        raise ValueError("run_restarts needs a family_factory with rng='philox' (restart r "
                         "draws from its own Philox stream; a numpy-stream family would give "
                         "every restart the same RandomState(0) noise)")
    t0 = time.perf_counter()
    obj = vb.black_box_klvi(fam, target, n_samples)
    run = vb.DeviceRun(obj, n_iters, inits, window=window, learning_rate=learning_rate,
                       learning_rate_end=learning_rate_end)
    run.advance_philox(n_iters, seed, stream_base, 0, stream_stride=stride)
    _, _, vals, smooth = run.result(history=False)
    t1 = time.perf_counter()
    # the M log weights of every restart stay in HBM from the draws through the
    # bounds and PSIS: row j of one [restarts][M] buffer; PSIS then runs all
    # restarts' columns in one batched pipeline (the buffer's transpose is the
    # reference's Fortran-ordered (M, restarts) log-weight matrix)
    import torch
    lw = torch.empty((len(ids), int(n_bounds)), dtype=torch.float64,
                     device=torch.device('cuda', nat.context().device))
    # bound draws: restart r uses Philox stream 2^20 + r of its own; all of this
    # rank's restarts (ids = r0, r0 + stride, ...) in one launch where the
    # batched kernel covers the family and target (mean-field family, a device
    # target that is separable or has D <= 16), else one launch per restart
    bfam = family_factory()
    batched = (_rows_supported(bfam, target)
               and ids == list(range(ids[0], ids[0] + stride * len(ids), stride)))
    if batched:
        experiments.log_weights_rows(target, bfam, smooth, n_bounds, (1 << 20) + ids[0],
                                     stride, lw_out=lw)
    else:
        for j, r in enumerate(ids):
            fj = family_factory()
            fj.stream = (1 << 20) + r
            experiments.log_weights(target, fj, smooth[j], n_bounds, return_samples=False,
                                    lw_out=lw[j])
    # the divergence statistics of all restarts in one batched reduction chain,
    # then the O(D) bound algebra and the Monte Carlo warnings of all restarts on the
    # host, then the PSIS k-hats (psis.py:112-208's kss; the smoothed weights are not
    # needed here).  VIABEL_AMD_PSIS_WORKER=1 runs the k-hats on a worker thread beside
    # the bound algebra instead: the thread hand-off cost more than the ~0.15 ms of
    # algebra it hides (config 5's stage 4.05-4.18 vs 3.81-3.90 ms,
    # profiles/r06/cfg5/stage_logq_product_worker_ab.log)
    div = bounds.divergence_rows(lw)
    khat_fn = lambda: psis.psis_khat(lw.t()) if len(ids) > 1 else np.array([psis.psis_khat(lw[0])])
    # (a full-rank family's moments below call the library: no concurrent calls
    # on the context, so the k-hats run first there)
    use_worker = bfam.kind != nat.FAMILY_FR_T and os.environ.get('VIABEL_AMD_PSIS_WORKER', '0') == '1'
    khat_job = _psis_worker().submit(khat_fn) if use_worker else None
    khat = khat_fn() if (khat_job is None and bfam.kind == nat.FAMILY_FR_T) else None
    if bfam.kind == nat.FAMILY_FR_T:
        # full-rank q: the family's own moments and covariance (eigenvalues of
        # Sigma on the device), restart by restart, as all_bounds does
        recs = []
        for j, r in enumerate(ids):
            res = bounds.all_bounds_from_divergence(
                div[j], lambda p, lam=smooth[j]: bfam.pth_moment(p, lam),
                q_var=bfam.mean_and_cov(smooth[j])[1])
            recs.append([r, float(div[j, 1]), res['d2'], res['W1'], res['W2'],
                         res['mean_error'], res['std_error'], res['cov_error']])
    else:
        recs = bounds_records(ids, div, smooth, bfam)
    if khat_job is not None:
        khat = khat_job.result()
    elif khat is None:
        khat = khat_fn()
    if timings is not None:
        _sync()
        t2 = time.perf_counter()
        timings['fit_s'] = t1 - t0
        timings['bounds_psis_s'] = t2 - t1
        timings['pre_s'] = t0 - t_entry
    # [records | k-hat | final value | lambda*] of every restart, one array op
    # (a per-restart concatenate took ~0.3 ms at 64 restarts)
    out = np.column_stack([np.asarray(recs, dtype=float), np.asarray(khat, dtype=float),
                           np.asarray(vals, dtype=float)[:, -1], np.asarray(smooth, dtype=float)])
    if timings is not None:
        timings['post_s'] = time.perf_counter() - t2
    return out


_WORKER = []


def _psis_worker():
    """One persistent worker thread for the restart table's PSIS calls (made on
    first use; a new thread per call costs more than the overlap gains)."""
    if not _WORKER:
        import concurrent.futures
        _WORKER.append(concurrent.futures.ThreadPoolExecutor(max_workers=1,
                                                             thread_name_prefix='viabel_amd_psis'))
    return _WORKER[0]


def bounds_records(ids, div, lams, fam):
    """Per-restart [id, elbo, d2, W1, W2, mean_error, std_error, cov_error]:
    `all_bounds(lw, moment_bound_fn=fam.pth_moment, q_var=fam.mean_and_cov)`
    (bounds.py:13-61) for every row of `divergence_rows` at once.  The family's
    2nd / 4th moments (vb.py:72-82, 168-182) and the spectral norm of its
    diagonal covariance (bounds.py:64-67) are evaluated for all rows as arrays
    instead of 64 sets of per-restart calls; the Monte Carlo warnings
    (bounds.py:187-191) are issued per row as all_bounds does."""
    from . import bounds
    if fam.kind not in (nat.FAMILY_MF_GAUSSIAN, nat.FAMILY_MF_T):
        raise ValueError('bounds_records: mean-field families only (a full-rank q needs its '
                         'own moments: all_bounds_from_divergence per restart)')
    div = np.asarray(div, dtype=float)
    lams = np.atleast_2d(np.asarray(lams, dtype=float))
    D = fam.dim
    for row in div:
        bounds._mc_warning(row[2], row[3], 'CUBO')
        bounds._mc_warning(row[4], row[5], 'ELBO')
    d2 = div[:, 0]
    v = np.exp(2 * lams[:, D:])                       # variances (Gaussian) / squared scales (t)
    if fam.kind == nat.FAMILY_MF_GAUSSIAN:
        C2 = np.sum(v, axis=1)
        C4 = 2 * np.sum(v ** 2, axis=1) + np.sum(v, axis=1) ** 2
        qnorm = np.max(v, axis=1)
    else:
        df = fam.df
        if df <= 4:
            raise ValueError('df must be greater than p')
        c = df / (df - 2)
        s = np.exp(lams[:, D:])
        C2 = c * np.sum(s ** 2, axis=1)
        C4 = c ** 2 * (2 * (df - 1) / (df - 4) * np.sum(s ** 4, axis=1) + np.sum(s ** 2, axis=1) ** 2)
        qnorm = np.max(np.abs(c * v), axis=1)
    W1 = 2 * C2 ** .5 * np.expm1(d2) ** .5
    W2 = 2 * C4 ** .25 * np.expm1(d2) ** .25
    cov_error = 2 * (np.sqrt(qnorm) * W2 + W2 ** 2)
    return [[r, float(div[j, 1]), d2[j], W1[j], W2[j], min(W1[j], W2[j]), W2[j], cov_error[j]]
            for j, r in enumerate(ids)]


def gather_records(local, n_restarts, width, group=None):
    """all_gather of the fixed-size per-restart records; returns the full
    [n_restarts, width] table ordered by restart id on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    per_rank = -(-n_restarts // world)
    backend = dist.get_backend(group)
    dev = torch.device('cuda', torch.cuda.current_device()) if backend == 'nccl' else torch.device('cpu')
    buf = torch.full((per_rank, width), float('nan'), dtype=torch.float64, device=dev)
    if len(local):
        buf[:len(local)] = torch.as_tensor(np.asarray(local), dtype=torch.float64, device=dev)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    table = torch.cat(out).cpu().numpy()
    table = table[~np.isnan(table[:, 0])]
    return table[np.argsort(table[:, 0])]


def run_restarts(family_factory, target, n_restarts, n_iters, n_samples=100, n_bounds=1_000_000,
                 learning_rate=.01, learning_rate_end=.001, window=10, inits=None, seed=0,
                 group=None, compute=None, timings=None):
    """Fit n_restarts KLVI restarts sharded over the ranks of `group` (or this
    process alone when torch.distributed is not initialised) and return the
    gathered summary table (RECORD_HEAD + lambda*) on every rank.

    `compute(ids, inits) -> records` replaces the device computation (tests use
    it to run the sharding and the collective without a GPU).  With the device
    computation under torch.distributed, each rank first binds its own GPU
    (bind_local_device).  `timings` (a dict) receives this rank's fit and
    bounds/PSIS stage seconds."""
    try:
        import torch.distributed as dist
        dist_on = dist.is_available() and dist.is_initialized()
    except ImportError:
        dist_on = False
    t_in = time.perf_counter()
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if dist_on else (0, 1)
    fam0 = family_factory()
    P = fam0.var_param_dim
    if inits is None:
        inits = default_inits(n_restarts, P)
    if compute is None and dist_on:
        bind_local_device(rank)
    ids = shard(n_restarts, rank, world)
    local_inits = np.asarray(inits)[ids] if ids else np.zeros((0, P))
    if compute is None:
        local = (_native_compute(ids, local_inits, family_factory, target, n_iters, n_samples,
                                 n_bounds, learning_rate, learning_rate_end, window, seed,
                                 1 + rank, world, timings)
                 if ids else np.zeros((0, len(RECORD_HEAD) + P)))
    else:
        local = compute(ids, local_inits)
    if timings is not None:
        # this rank's whole call before the gather (the fit and bounds stages plus
        # the host setup and the record table around them)
        timings['local_s'] = time.perf_counter() - t_in
    width = len(RECORD_HEAD) + P
    if not dist_on:
        return np.asarray(local)[np.argsort(np.asarray(local)[:, 0])]
    return gather_records(local, n_restarts, width, group)


# ---------------------------------------------------------------------------
# RMSProp-IA / Adam-IA chains with R-hat, sharded over ranks (vb.py:392-712)

class DeviceIAOps:
    """run_ia_chains' per-rank work on the device: the rank's chains in one
    launch chain (one workgroup per chain, chain o on Philox stream
    family.stream + o whatever the sharding), the first R-hat stage
    (vb_rhat_stats), the combine (vb_rhat_combine) and the cumulative means
    (vb_iterate_average).  Tests substitute other ops to run the sharding and
    the collective without a GPU."""

    @staticmethod
    def chains(opt, obj, inits, ids, world, n_iters, window, learning_rate, epsilon,
               learning_rate_end):
        from . import vb
        fam = obj.family
        run = vb.DeviceRun(obj, n_iters, inits, window, learning_rate, epsilon,
                           learning_rate_end, optimizer=opt)
        run.advance_philox(n_iters, fam.seed, fam.stream + ids[0], fam.step, stream_stride=world)
        lam, hist, vals, _ = run.result()
        return lam, hist, vals

    @staticmethod
    def stats(hist, segs):
        from . import functions
        return functions.rhat_stats(hist, segs)

    @staticmethod
    def combine(mean, ss, lens):
        from . import functions
        return functions.rhat_combine(mean, ss, lens)

    @staticmethod
    def average(x, start):
        from . import functions
        return functions.stochastic_iterate_averaging(x, start)[0]


def run_ia_chains(opt, n_iters, objective_and_grad, init_param, K, has_log_norm=False,
                  window=500, learning_rate=.01, epsilon=1e-6, rhat_window=500, n_optimisers=1,
                  r_mean_threshold=1.15, r_sigma_threshold=1.20, tail_avg_iters=2000,
                  learning_rate_end=None, perturb_scale=0.5, avg_grad_norm=False, group=None,
                  gather_histories=False, ops=None):
    """rmsprop_IA_optimize_with_rhat / adam_IA_optimize_with_rhat (vb.py:392-712,
    `opt` = OPT_RMSPROP_IA / OPT_ADAM_IA) with the n_optimisers chains of the
    reference's loop (vb.py:417-421) dealt to the ranks of `group`: chain o on
    rank o % world.  Each rank runs its chains, then reduces each to the
    statistics split-chain R-hat needs (per window / halfway segment, half-chain
    and parameter: the half-chain mean and centred sum of squares,
    functions.rhat_stats).  ONE all_gather of fixed-size per-chain records
    (chain id, final parameters, value history, those statistics) gives every
    rank all chains' statistics; the R-hat combine (functions.py:8-31's B / W
    algebra) then runs on them in chain order, so r_hat_mean / r_hat_sigma (and
    the halfway ones) and the averaging starts equal the one-process run's bit
    for bit.  Returns the one-process tuple (final parameters of the last chain,
    history chains, averaged means, averaged sigmas, values of all chains, log
    norms, log); history chains and averages are this rank's chains (ids in
    log['chain_ids']) unless gather_histories=True, which all-gathers the
    histories as well (a second collective of n_optimisers x history x P).

    The objective must be a native Philox-noise objective: chain o's noise is
    then its own stream.  (The numpy-stream path draws the chains one after
    another from shared generators, vb.py:419 / the family stream, and a
    caller's objective runs where the caller's code runs: neither shards.)"""
    from . import vb, functions
    if ops is None:
        if not isinstance(objective_and_grad, vb.NativeObjective) or \
                objective_and_grad.family.rng != 'philox':
            raise ValueError("sharded IA chains need a native objective with rng='philox' "
                             "(chain o draws from its own Philox stream)")
        if has_log_norm:
            raise ValueError('not enough values to unpack (expected 3, got 2)')
        if avg_grad_norm:
            raise ValueError('avg_grad_norm runs the host-side update path, which is not sharded')
        ops = DeviceIAOps
    if learning_rate <= 0:
        raise ValueError('learning rate must be positive')
    if learning_rate_end is not None and learning_rate <= learning_rate_end:
        raise ValueError('initial learning rate must be greater than final learning rate')
    try:
        import torch.distributed as dist
        dist_on = dist.is_available() and dist.is_initialized()
    except ImportError:
        dist_on = False
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if dist_on else (0, 1)
    n_iters = int(n_iters)
    init_param = np.asarray(init_param, dtype=float)
    P = init_param.size
    inits = vb._ia_inits(init_param, n_optimisers, perturb_scale)
    n_hist = min(n_iters, 100 * int(window))              # vb.py:465-466
    segs_w = functions.adaptive_segments(n_optimisers, n_hist, P, rhat_window)
    segs_h = functions.halfway_segments(n_optimisers, n_hist, P, 100, 200)
    segs = segs_w + segs_h
    J = len(segs)
    if ops is DeviceIAOps and dist_on:
        bind_local_device(rank)
    ids = shard(n_optimisers, rank, world)
    width = 1 + P + n_iters + 4 * J * P
    local = np.zeros((len(ids), width))
    hist = np.zeros((0, n_hist, P))
    if ids:
        lam, hist, vals = ops.chains(opt, objective_and_grad, np.stack([inits[o] for o in ids]),
                                     ids, world, n_iters, int(window), learning_rate, epsilon,
                                     learning_rate_end)
        hist = np.asarray(hist)
        mean, ss = ops.stats(hist, segs)                  # [J][2 n_local][P]
        nl = len(ids)
        per_chain = lambda a: np.asarray(a).reshape(J, nl, 2, P).transpose(1, 0, 2, 3).reshape(nl, -1)
        local = np.concatenate([np.asarray(ids, dtype=float)[:, None], np.asarray(lam),
                                np.asarray(vals), per_chain(mean), per_chain(ss)], axis=1)
    if ops is DeviceIAOps:
        objective_and_grad.family.step += n_iters        # as the one-process run leaves it
    table = gather_records(local, n_optimisers, width, group) if dist_on else local
    o1, o2 = 1 + P, 1 + P + n_iters
    o3 = o2 + 2 * J * P
    to_halves = lambda a: a.reshape(n_optimisers, J, 2, P).transpose(1, 0, 2, 3).reshape(
        J, 2 * n_optimisers, P)
    lens = np.array([m for _, m in segs], dtype=np.int64)
    rhats = ops.combine(np.ascontiguousarray(to_halves(table[:, o2:o3])),
                        np.ascontiguousarray(to_halves(table[:, o3:])), lens)
    rw = rhats[:len(segs_w)]
    rh = rhats[len(segs_w):] if segs_h else np.zeros((0,))
    rm, rs = rw[:, :K], rw[:, K:]
    start_m, start_s = vb._ia_avg_starts(rm, rs, n_iters, rhat_window, r_mean_threshold,
                                         r_sigma_threshold, tail_avg_iters)
    chain_ids = list(ids)
    if gather_histories:
        hrec = np.concatenate([np.asarray(ids, dtype=float)[:, None], hist.reshape(len(ids), -1)],
                              axis=1) if ids else np.zeros((0, 1 + n_hist * P))
        htab = gather_records(hrec, n_optimisers, 1 + n_hist * P, group) if dist_on else hrec
        hist = htab[:, 1:].reshape(n_optimisers, n_hist, P)
        chain_ids = list(range(n_optimisers))
    means = [ops.average(np.ascontiguousarray(hist[j, :, :K]), start_m) for j in range(len(chain_ids))]
    sigmas = [ops.average(np.ascontiguousarray(hist[j, :, K:]), start_s)
              for j in range(len(chain_ids))]
    values = table[:, o1:o2].reshape(-1)
    log = {'start_avg_mean_iters': start_m, 'start_avg_sigma_iters': start_s,
           'r_hat_mean': rm, 'r_hat_sigma': rs,
           'r_hat_mean_halfway': rh[:, :K], 'r_hat_sigma_halfway': rh[:, K:],
           'chain_ids': chain_ids}
    return (table[-1, 1:1 + P].copy(), hist, means, sigmas, values, np.zeros(len(values)), log)
