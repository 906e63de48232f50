"""Monte Carlo VI on the GPU behind the viabel.vb API.

Mirrors the reference module viabel/vb.py (names, signatures, return shapes,
error messages) for the hot path:

  mean_field_gaussian_variational_family  vb.py:48-82
  mean_field_t_variational_family         vb.py:140-182
  t_variational_family (full rank)        vb.py:185-233, _distributions.py:8-38
  black_box_klvi                          vb.py:236-245
  black_box_chivi                         vb.py:248-266
  black_box_klvi_pd / black_box_klvi_pd2  vb.py:268-295
  learning_rate_schedule                  vb.py:324-342
  adagrad_optimize                        vb.py:345-389
  rmsprop_IA_optimize_with_rhat           vb.py:392-553
  adam_IA_optimize_with_rhat              vb.py:556-712

Computation runs in libviabel_amd.so (HIP, gfx950).  Two noise sources:

* ``rng='numpy'`` (default): the family owns ``RandomState(0)`` exactly like the
  reference (vb.py:49, 143) and CHIVI draws its per-call seed from the global
  numpy RNG (vb.py:258); the standardized draws are generated on the host with
  the same calls in the same order and streamed to the kernels, so results
  match the reference on identical seeds.
* ``rng='philox'``: draws come from an in-kernel Philox4x32-10 counter RNG
  (counter = column pair, sample, step, stream); nothing is transferred per
  step.  Statistically equivalent, not stream-identical, to the reference.
  This is the throughput path (bench.py).

The module-wide default is taken from $VIABEL_AMD_RNG or set_default_rng().
"""
import itertools
import math
import os
from collections import namedtuple

import numpy as np

from . import _native as nat
from . import targets as _targets
from .targets import Target

__all__ = [
    'make_stan_log_density',
    'mean_field_gaussian_variational_family',
    'mean_field_t_variational_family',
    'full_rank_gaussian_variational_family',
    't_variational_family',
    'black_box_klvi',
    'black_box_chivi',
    'black_box_klvi_pd',
    'black_box_klvi_pd2',
    'learning_rate_schedule',
    'adagrad_optimize',
    'rmsprop_IA_optimize_with_rhat',
    'adam_IA_optimize_with_rhat',
    'set_default_rng',
]

VariationalFamily = namedtuple('VariationalFamily',
                               ['sample', 'entropy',
                                'logdensity', 'mean_and_cov',
                                'pth_moment', 'var_param_dim'])

_DEFAULT_RNG = [os.environ.get('VIABEL_AMD_RNG', 'numpy')]
_STREAMS = itertools.count(1)
LOG2PI = math.log(2 * math.pi)


def set_default_rng(kind):
    if kind not in ('numpy', 'philox'):
        raise ValueError("rng must be 'numpy' or 'philox'")
    _DEFAULT_RNG[0] = kind


class NativeVariationalFamily(VariationalFamily):
    """VariationalFamily namedtuple carrying the device descriptor and RNG state."""

    def _struct(self):
        return nat.Family(self.kind, 0, self.dim, float(self.df or 0.0))

    # the family's own RandomState(0) (vb.py:49 / 143 / 195), made on first use:
    # constructing one costs ~0.25 ms of host time (MT19937 seeding), and a Philox
    # family never draws from it (config 5 built three families per call)
    @property
    def rs(self):
        r = self.__dict__.get('_rs')
        if r is None:
            r = self.__dict__['_rs'] = np.random.RandomState(0)
        return r

    @rs.setter
    def rs(self, value):
        self.__dict__['_rs'] = value

    # standardized draws exactly as the reference draws them
    def _draw(self, n, seed=None):
        rs = self.rs if seed is None else np.random.RandomState(seed)
        if self.kind == nat.FAMILY_MF_GAUSSIAN:
            return rs.randn(n, self.dim)
        if self.kind == nat.FAMILY_FR_T:
            # vb.py:204-206: chisquare first, then randn; flat [s (n), z (n x D)]
            s = np.sqrt(rs.chisquare(self.df, n) / self.df)
            return np.concatenate([s, rs.randn(n, self.dim).ravel()])
        return rs.standard_t(self.df, size=(n, self.dim))

    def _philox_noise(self, seed=None, steps=1):
        """Noise descriptor for the next `steps` Philox steps of this family."""
        if seed is None:
            nz = nat.Noise(nat.NOISE_PHILOX, self.stream, self.seed, self.step, None)
            self.step += steps
        else:
            nz = nat.Noise(nat.NOISE_PHILOX, 0, int(seed) & 0xFFFFFFFFFFFFFFFF, 0, None)
        return nz


def _make_family(kind, dim, df, rng):
    rng = _DEFAULT_RNG[0] if rng is None else rng
    if rng not in ('numpy', 'philox'):
        raise ValueError("rng must be 'numpy' or 'philox'")

    def unpack(var_param):
        var_param = np.asarray(var_param, dtype=float)
        return var_param[:dim], var_param[dim:]

    def sample(var_param, n_samples, seed=None):
        lam = nat.as_f64(var_param)
        out = np.empty((int(n_samples), dim))
        if fam.rng == 'numpy':
            eps = nat.as_f64(fam._draw(int(n_samples), seed))
            nz = nat.Noise(nat.NOISE_HOST, 0, 0, 0, nat.dptr(eps))
        else:
            nz = fam._philox_noise(seed)
        nat.check(nat.lib().vb_family_sample(nat.context().handle, fam._struct(), nat.dptr(lam),
                                             int(n_samples), nz, nat.dptr(out)))
        return out

    def logdensity(x, var_param):
        lam = nat.as_f64(var_param)
        xx = np.asarray(x, dtype=float)
        one_d = xx.ndim == 1
        xx = nat.as_f64(np.atleast_2d(xx))
        out = np.empty(xx.shape[0])
        nat.check(nat.lib().vb_family_logdensity(nat.context().handle, fam._struct(),
                                                 nat.dptr(lam), nat.dptr(xx), xx.shape[0],
                                                 nat.dptr(out)))
        if one_d and kind == nat.FAMILY_MF_GAUSSIAN:
            return out[0]            # mvn.logpdf of one point is a scalar
        return out

    if kind == nat.FAMILY_MF_GAUSSIAN:
        def entropy(var_param):
            _, log_std = unpack(var_param)
            return 0.5 * dim * (1.0 + np.log(2 * np.pi)) + np.sum(log_std)   # vb.py:61

        def mean_and_cov(var_param):
            mean, log_std = unpack(var_param)
            return mean, np.diag(np.exp(2 * log_std))                       # vb.py:69

        def pth_moment(p, var_param):
            if p not in [2, 4]:
                raise ValueError('only p = 2 or 4 supported')
            _, log_std = unpack(var_param)
            v = np.exp(2 * log_std)
            if p == 2:
                return np.sum(v)
            return 2 * np.sum(v ** 2) + np.sum(v) ** 2
    else:
        def entropy(var_param):
            _, log_scale = unpack(var_param)
            return np.sum(log_scale)                                          # vb.py:156

        def mean_and_cov(var_param):
            mean, log_scale = unpack(var_param)
            return mean, df / (df - 2) * np.diag(np.exp(2 * log_scale))       # vb.py:166

        def pth_moment(p, var_param):
            if p not in [2, 4]:
                raise ValueError('only p = 2 or 4 supported')
            if df <= p:
                raise ValueError('df must be greater than p')
            _, log_scale = unpack(var_param)
            s = np.exp(log_scale)
            c = df / (df - 2)
            if p == 2:
                return c * np.sum(s ** 2)
            return c ** 2 * (2 * (df - 1) / (df - 4) * np.sum(s ** 4) + np.sum(s ** 2) ** 2)

    fam = NativeVariationalFamily(sample, entropy, logdensity, mean_and_cov, pth_moment, 2 * dim)
    fam.kind, fam.dim, fam.df, fam.rng = kind, int(dim), df, rng
    fam.seed, fam.stream, fam.step = 0, next(_STREAMS) & 0xFFFFFF, 0
    return fam


def t_variational_family(dim, df, rng=None):
    """vb.py:192-233.  var_param = [mu (dim), tril(M) (dim (dim + 1) / 2)] in
    paragami's free layout: row-major lower triangle, log diagonal,
    Sigma = L L^T.  Every method runs on the device (sqrtm / eigh through the
    eigendecomposition of Sigma)."""
    if df <= 2:
        raise ValueError('df must be greater than 2')
    rng = _DEFAULT_RNG[0] if rng is None else rng
    if rng not in ('numpy', 'philox'):
        raise ValueError("rng must be 'numpy' or 'philox'")
    dim = int(dim)
    df = float(df)
    P = dim + dim * (dim + 1) // 2

    def _lam(var_param):
        lam = nat.as_f64(var_param)
        if lam.shape != (P,):
            raise ValueError('var_param must have shape (%d,)' % P)
        return lam

    def sample(var_param, n_samples, seed=None):
        lam = _lam(var_param)
        out = np.empty((int(n_samples), dim))
        if fam.rng == 'numpy':
            eps = nat.as_f64(fam._draw(int(n_samples), seed))
            nz = nat.Noise(nat.NOISE_HOST, 0, 0, 0, nat.dptr(eps))
        else:
            nz = fam._philox_noise(seed)
        nat.check(nat.lib().vb_family_sample(nat.context().handle, fam._struct(), nat.dptr(lam),
                                             int(n_samples), nz, nat.dptr(out)))
        return out

    def logdensity(x, var_param):
        lam = _lam(var_param)
        xx = np.asarray(x, dtype=float)
        one_d = xx.ndim == 1
        xx = nat.as_f64(np.atleast_2d(xx))
        out = np.empty(xx.shape[0])
        nat.check(nat.lib().vb_family_logdensity(nat.context().handle, fam._struct(),
                                                 nat.dptr(lam), nat.dptr(xx), xx.shape[0],
                                                 nat.dptr(out)))
        return out[0] if one_d else out

    def _moments(var_param, sigma=False):
        lam = _lam(var_param)
        eig = np.empty(dim)
        sig = np.empty((dim, dim)) if sigma else None
        nat.check(nat.lib().vb_family_moments(nat.context().handle, fam._struct(), nat.dptr(lam),
                                              nat.dptr(sig) if sigma else None, nat.dptr(eig)))
        return eig, sig

    def entropy(var_param):
        # .5 log det Sigma (vb.py:210-213), from the device eigenvalues
        return .5 * np.sum(np.log(_moments(var_param)[0]))

    def mean_and_cov(var_param):
        lam = _lam(var_param)
        sig = np.empty((dim, dim))
        nat.check(nat.lib().vb_family_moments(nat.context().handle, fam._struct(), nat.dptr(lam),
                                              nat.dptr(sig), None))
        return lam[:dim].copy(), df / (df - 2.) * sig                      # vb.py:215-217

    def pth_moment(p, var_param):
        if p not in [2, 4]:
            raise ValueError('only p = 2 or 4 supported')
        if df <= p:
            raise ValueError('df must be greater than p')
        sq_scales = _moments(var_param)[0]                                  # vb.py:225
        c = df / (df - 2)
        if p == 2:
            return c * np.sum(sq_scales)
        return c ** 2 * (2 * (df - 1) / (df - 4) * np.sum(sq_scales ** 2) + np.sum(sq_scales) ** 2)

    fam = NativeVariationalFamily(sample, entropy, logdensity, mean_and_cov, pth_moment, P)
    fam.kind, fam.dim, fam.df, fam.rng = nat.FAMILY_FR_T, dim, df, rng
    fam.seed, fam.stream, fam.step = 0, next(_STREAMS) & 0xFFFFFF, 0
    return fam


def mean_field_gaussian_variational_family(dim, rng=None):
    """vb.py:48-82.  var_param = [mean (dim), log_std (dim)]."""
    return _make_family(nat.FAMILY_MF_GAUSSIAN, dim, None, rng)


def full_rank_gaussian_variational_family(dim):
    """Importable for the reference notebooks' import cells (vb.py:85-137); not
    built: the reference's own version is broken, and the
    full-rank path here is t_variational_family (a large df approaches it)."""
    raise NotImplementedError(
        'full_rank_gaussian_variational_family is out of scope for viabel_amd; '
        'use t_variational_family(dim, df) with a large df')


def mean_field_t_variational_family(dim, df, rng=None):
    """vb.py:140-182.  var_param = [mean (dim), log_scale (dim)]."""
    if df <= 2:
        raise ValueError('df must be greater than 2')
    return _make_family(nat.FAMILY_MF_T, dim, float(df), rng)


class NativeObjective:
    """objective_and_grad(var_param) -> (value, grad) evaluated on the GPU."""

    def __init__(self, kind, var_family, logdensity, n_samples, alpha=None):
        if not isinstance(var_family, NativeVariationalFamily):
            raise TypeError('var_family must come from viabel_amd.vb')
        # device targets pass through; torch-differentiable callables are wrapped
        # (targets.as_target); anything else raises TypeError
        logdensity = _targets.as_target(logdensity, var_family.dim).bind(var_family.dim)
        if logdensity.dim != var_family.dim:
            raise ValueError('target dimension %d != family dimension %d'
                             % (logdensity.dim, var_family.dim))
        self.kind, self.family, self.target = kind, var_family, logdensity
        self.n_samples = int(n_samples)
        self.alpha = float(alpha) if alpha is not None else 2.0

    def _structs(self):
        return (self.family._struct(), self.target._struct(),
                nat.Objective(self.kind, 0, self.alpha, self.n_samples))

    def _eps_one_call(self):
        """Host draws for one call, in the reference's order (numpy mode)."""
        fam = self.family
        if self.kind != nat.OBJ_CHIVI:
            return fam._draw(self.n_samples)                        # vb.py:239, 271
        seed = np.random.randint(2 ** 32)                           # vb.py:258
        return fam._draw(self.n_samples, seed)                      # vb.py:251

    def __call__(self, var_param):
        lam = nat.as_f64(var_param)
        if lam.shape != (self.family.var_param_dim,):
            raise ValueError('var_param must have shape (%d,)' % self.family.var_param_dim)
        fam = self.family
        if fam.rng == 'numpy':
            eps = nat.as_f64(self._eps_one_call())
            nz = nat.Noise(nat.NOISE_HOST, 0, 0, 0, nat.dptr(eps))
        elif self.kind == nat.OBJ_CHIVI:
            nz = fam._philox_noise(np.random.randint(2 ** 32))
            nz.stream = fam.stream
        else:
            nz = fam._philox_noise()
        f, t, o = self._structs()
        val = np.empty(1)
        grad = np.empty(lam.size)
        nat.check(nat.lib().vb_objective_value_grad(nat.context().handle, f, t, o, nat.dptr(lam),
                                                    nz, nat.dptr(val), nat.dptr(grad)))
        return val[0], grad


def black_box_klvi(var_family, logdensity, n_samples):
    """vb.py:236-245: returns objective_and_grad(var_param) -> (-ELBO, grad)."""
    return NativeObjective(nat.OBJ_KLVI, var_family, logdensity, n_samples)


def black_box_chivi(alpha, var_family, logdensity, n_samples):
    """vb.py:248-266: returns objective_and_grad(var_param) -> (CUBO, grad)."""
    return NativeObjective(nat.OBJ_CHIVI, var_family, logdensity, n_samples, alpha)


def black_box_klvi_pd(var_family, logdensity, n_samples):
    """vb.py:268-278: value -(mean log p - mean log q(x)) on the family's draws;
    autograd differentiates log q through x and lambda, whose total derivative
    reduces to the entropy's, so the gradient is black_box_klvi's."""
    return NativeObjective(nat.OBJ_KLVI_PD, var_family, logdensity, n_samples)


def black_box_klvi_pd2(var_family, logdensity, n_samples):
    """vb.py:281-295: the same objective written with a partial over var_param
    (autograd still differentiates through it): identical value and gradient."""
    return NativeObjective(nat.OBJ_KLVI_PD, var_family, logdensity, n_samples)


def make_stan_log_density(fitobj):
    """vb.py:314-321: a fitted Stan model's log_prob / grad_log_prob as the
    target (evaluated on the host per sample row; its dimension is the
    family's, as in the reference)."""
    from .targets import from_stan
    return from_stan(fitobj)


def learning_rate_schedule(n_iters, learning_rate, learning_rate_end):
    """vb.py:324-342 (generator); the device evaluates the same expression."""
    if learning_rate <= 0:
        raise ValueError('learning rate must be positive')
    if learning_rate_end is not None:
        if learning_rate <= learning_rate_end:
            raise ValueError('initial learning rate must be greater than final learning rate')
        b = n_iters * learning_rate_end / (2 * (learning_rate - learning_rate_end))
        a = learning_rate * b
        start_decrease_at = n_iters // 4
        end_decrease_at = 3 * n_iters // 4
    for i in range(n_iters):
        if learning_rate_end is None or i < start_decrease_at:
            yield learning_rate
        elif i < end_decrease_at:
            yield a / (b + i - start_decrease_at + 1)
        else:
            yield learning_rate_end


# host draws per device chunk in numpy mode (bounded host memory)
_HOST_CHUNK_ELEMS = 1 << 24


class DeviceRun:
    """Device-resident adagrad state for one or more problems (vb_run)."""

    def __init__(self, objective, n_iters, init_params, window=10, learning_rate=.01,
                 epsilon=.1, learning_rate_end=None, optimizer=nat.OPT_ADAGRAD):
        init = nat.as_f64(np.atleast_2d(init_params))
        self.optimizer = optimizer
        self.window = int(window)
        self.obj = objective
        self.n_iters = int(n_iters)
        self.n_problems = init.shape[0]
        self.P = init.shape[1]
        f, t, o = objective._structs()
        cfg = nat.AdagradConfig(self.n_iters, int(window), int(optimizer), float(learning_rate),
                                nat.NAN if learning_rate_end is None else float(learning_rate_end),
                                float(epsilon))
        import ctypes
        h = ctypes.c_void_p()
        nat.check(nat.lib().vb_run_create(nat.context().handle, f, t, o, cfg, self.n_problems,
                                          nat.dptr(init), ctypes.byref(h)))
        self.handle = h
        self.done = 0

    def advance_philox(self, n_steps, seed, stream, step, stream_stride=1):
        """Problem q draws from Philox stream `stream + q * stream_stride`.
        The noise descriptor is reused across calls (short runs are host-bound)."""
        nz = self.__dict__.get('_nz')
        if nz is None:
            nz = self._nz = nat.Noise(nat.NOISE_PHILOX, 0, 0, 0, None, 1)
            self._advance = nat.lib().vb_run_advance
        nz.stream = stream & 0xFFFFFF
        nz.seed = seed
        nz.step = step
        nz.stream_stride = stream_stride
        nat.check(self._advance(self.handle, int(n_steps), nz))
        self.done += int(n_steps)

    def set_timing(self, enable=True):
        """Bracket later advances' device work with HIP events (vb_run_set_timing)."""
        nat.check(nat.lib().vb_run_set_timing(self.handle, 1 if enable else 0))

    def launch_times(self, max_records=4096):
        """[(steps, seconds)] of the bracketed launches since the last call."""
        import ctypes
        steps = (ctypes.c_int64 * max_records)()
        ms = (ctypes.c_float * max_records)()
        n = ctypes.c_int64()
        nat.check(nat.lib().vb_run_launch_times(self.handle, max_records, steps, ms,
                                                ctypes.byref(n)))
        return [(int(steps[k]), float(ms[k]) * 1e-3) for k in range(n.value)]

    def advance_host(self, eps):
        """eps: [n_problems][n_steps][N][D] standardized draws."""
        eps = nat.as_f64(eps)
        n_steps = eps.shape[1]
        nz = nat.Noise(nat.NOISE_HOST, 0, 0, 0, nat.dptr(eps))
        nat.check(nat.lib().vb_run_advance(self.handle, n_steps, nz))
        self.done += n_steps

    def result(self, history=True):
        """(lam, hist, vals, smooth) of every problem; history=False skips the
        history copy (hist is None) -- at config 5's 64 x 1 250 x 20 it is
        12.8 MB of device-to-host traffic that the restart table never reads."""
        if self.optimizer == nat.OPT_ADAGRAD:
            n_hist = self.n_iters - 3 * self.n_iters // 4
        else:
            n_hist = min(self.n_iters, 100 * self.window)
        lam = np.empty((self.n_problems, self.P))
        hist = np.empty((self.n_problems, n_hist, self.P)) if history else None
        vals = np.empty((self.n_problems, self.n_iters))
        smooth = np.empty((self.n_problems, self.P))
        nat.check(nat.lib().vb_run_result(self.handle, nat.dptr(lam),
                                          nat.dptr(hist) if history else None,
                                          nat.dptr(vals), nat.dptr(smooth)))
        return lam, hist, vals, smooth

    def values(self):
        """Objective values of problem 0 so far ([n_iters], steps not yet run are
        undefined)."""
        vals = np.empty((self.n_problems, self.n_iters))
        nat.check(nat.lib().vb_run_result(self.handle, None, None, nat.dptr(vals), None))
        return vals[0]

    def values_async(self, count):
        """Queue a snapshot of problem 0's first `count` values behind the work
        already queued (vb_run_values_async); values_wait() returns it."""
        nat.check(nat.lib().vb_run_values_async(self.handle, int(count)))

    def values_wait(self):
        """Wait for the last values_async snapshot only and return it."""
        import ctypes
        out = np.empty(max(1, self.n_iters))
        n = ctypes.c_int64()
        nat.check(nat.lib().vb_run_values_wait(self.handle, nat.dptr(out), ctypes.byref(n)))
        return out[:n.value]

    def steps_done(self):
        """Steps the library has run (vb_run_steps_done): the truth after an
        interrupt, whatever the caller's own counter says."""
        import ctypes
        n = ctypes.c_int64()
        nat.check(nat.lib().vb_run_steps_done(self.handle, ctypes.byref(n)))
        return int(n.value)

    def fr_retries(self):
        """Full-rank runs: advances run again after a warm Newton-Schulz root
        launched too few iterations (vb_run_fr_retries)."""
        import ctypes
        n = ctypes.c_int64()
        nat.check(nat.lib().vb_run_fr_retries(self.handle, ctypes.byref(n)))
        return int(n.value)

    def synchronize(self):
        nat.context().synchronize()

    def __del__(self):
        try:
            if getattr(self, 'handle', None) and nat._lib is not None and not nat.shutting_down():
                nat._lib.vb_run_destroy(self.handle)
        except Exception:
            pass


def _progress(n_iters):
    """The reference's tqdm.trange progress bar (vb.py:354), or None without
    tqdm; VIABEL_AMD_PROGRESS=0 turns it off."""
    if os.environ.get('VIABEL_AMD_PROGRESS', '1') == '0':
        return None
    try:
        import tqdm
    except ImportError:
        return None
    return tqdm.tqdm(total=n_iters)


def _native_adagrad(n_iters, obj, init_param, window, learning_rate, epsilon,
                    learning_rate_end):
    """The device-resident loop in chunks of about a tenth of the run (>= 1000
    steps): between chunks the progress bar shows the reference's 'Average Loss'
    (mean of the last 1000 values, vb.py:378-381), and a KeyboardInterrupt stops
    the run with the steps done so far, like the reference's (vb.py:382-389)."""
    fam = obj.family
    run = DeviceRun(obj, n_iters, init_param[None, :], window, learning_rate, epsilon,
                    learning_rate_end)
    chunk = max(1000, -(-n_iters // 10))
    if fam.rng != 'philox':
        per_step = obj.n_samples * (fam.dim + 1)
        chunk = max(1, min(chunk, _HOST_CHUNK_ELEMS // max(per_step, 1)))
    bar = _progress(n_iters)
    done = 0
    step0 = fam.step if fam.rng == 'philox' else None
    shown = 0

    def show():
        # the snapshot queued after the previous chunk: waiting for it leaves the
        # chunk queued since then running (the device never idles for the bar)
        nonlocal shown
        vals = run.values_wait()
        upto = len(vals)
        bar.update(upto - shown)
        shown = upto
        bar.set_description('Average Loss = {:,.5g}'.format(
            np.mean(vals[max(0, upto - 1 - 1000):upto])))

    try:
        if bar is not None and fam.rng == 'philox':
            pending = False
            while done < n_iters:
                cs = min(chunk, n_iters - done)
                run.advance_philox(cs, fam.seed, fam.stream, step0 + done)
                done += cs
                if pending:
                    show()
                run.values_async(done)
                pending = True
            if pending:
                show()
        else:
            while done < n_iters:
                cs = min(chunk, n_iters - done)
                if fam.rng == 'philox':
                    run.advance_philox(cs, fam.seed, fam.stream, step0 + done)
                else:
                    run.advance_host(np.stack([obj._eps_one_call() for _ in range(cs)])[None])
                done += cs
                if bar is not None:
                    vals = run.values()
                    bar.update(cs)
                    bar.set_description('Average Loss = {:,.5g}'.format(
                        np.mean(vals[max(0, done - 1 - 1000):done])))
    except KeyboardInterrupt:
        pass
    finally:
        if bar is not None:
            bar.close()
    # a ctypes call cannot be interrupted, but the interrupt may land between an
    # advance returning and `done` being updated: the run's own count is the truth
    done = run.steps_done()
    if step0 is not None:
        # the family's Philox counter follows the steps the run really took, so a
        # later call never reuses draws whatever point an interrupt landed at
        fam.step = step0 + done
    _, hist, vals, smooth = run.result()
    if done == n_iters:
        return smooth[0], hist[0], vals[0], np.zeros(n_iters)
    # interrupted: what the reference returns at that point
    rows = max(0, done - 3 * n_iters // 4)
    hist = hist[0, :rows]
    smoothed = np.mean(hist, axis=0) if rows else np.full(run.P, np.nan)
    return smoothed, hist, vals[0, :done], np.zeros(done)


def _foreign_adagrad(n_iters, objective_and_grad, init_param, has_log_norm, window,
                     learning_rate, epsilon, learning_rate_end):
    """Adagrad for a caller-supplied objective: the objective is the caller's
    Python; the update (vb.py:364-374) runs in the device kernel vb_adagrad_update
    on device-resident state."""
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError('viabel_amd.adagrad_optimize needs a GPU')
    dev = torch.device('cuda', nat.context().device)
    lam = torch.tensor(np.asarray(init_param, dtype=float), dtype=torch.float64, device=dev)
    ring = torch.zeros((window, lam.numel()), dtype=torch.float64, device=dev)
    values, hist, log_norms, local_log_norms = [], [], [], []
    sched = learning_rate_schedule(n_iters, learning_rate, learning_rate_end)
    for i, lr in zip(range(n_iters), sched):
        torch.cuda.synchronize(dev)
        if has_log_norm:
            val, g, log_norm = objective_and_grad(lam.cpu().numpy())
        else:
            val, g = objective_and_grad(lam.cpu().numpy())
            log_norm = 0
        values.append(val)
        log_norms.append(log_norm)
        g = nat.as_f64(g)
        if has_log_norm:
            # vb.py:365-373: the window's gradients scaled by exp(min - log_norm_j)
            local_log_norms.append(log_norm)
            if len(local_log_norms) > window:
                local_log_norms.pop(0)
            scale = nat.as_f64(np.exp(np.min(local_log_norms) - np.array(local_log_norms)))
            nat.check(nat.lib().vb_adagrad_update_scaled(
                nat.context().handle, lam.numel(), nat.dptr(lam), nat.dptr(g), nat.dptr(ring),
                window, i, lr, epsilon, nat.dptr(scale)))
        else:
            nat.check(nat.lib().vb_adagrad_update(nat.context().handle, lam.numel(),
                                                  nat.dptr(lam), nat.dptr(g), nat.dptr(ring),
                                                  window, i, lr, epsilon))
        if i >= 3 * n_iters // 4:
            hist.append(lam.cpu().numpy().copy())
    hist = np.array(hist)
    smooth = np.mean(hist, axis=0) if len(hist) else np.full(lam.numel(), np.nan)
    return smooth, hist, np.array(values), np.array(log_norms, dtype=float)


def adagrad_optimize(n_iters, objective_and_grad, init_param,
                     has_log_norm=False, window=10, learning_rate=.01,
                     epsilon=.1, learning_rate_end=None):
    """vb.py:345-389.  Returns (smoothed_opt_param, variational_param_history,
    value_history, log_norm_history).  Native objectives run the whole loop on
    the device (one kernel chain, no per-step host work in philox mode)."""
    # validate like the reference's schedule generator
    if learning_rate <= 0:
        raise ValueError('learning rate must be positive')
    if learning_rate_end is not None and learning_rate <= learning_rate_end:
        raise ValueError('initial learning rate must be greater than final learning rate')
    init_param = np.asarray(init_param, dtype=float)
    if isinstance(objective_and_grad, NativeObjective):
        if has_log_norm:
            raise ValueError('not enough values to unpack (expected 3, got 2)')
        return _native_adagrad(int(n_iters), objective_and_grad, init_param, int(window),
                               learning_rate, epsilon, learning_rate_end)
    return _foreign_adagrad(int(n_iters), objective_and_grad, init_param, has_log_norm,
                            int(window), learning_rate, epsilon, learning_rate_end)


def _ia_optimize(opt, n_iters, objective_and_grad, init_param, K, has_log_norm, window,
                 learning_rate, epsilon, rhat_window, n_optimisers, r_mean_threshold,
                 r_sigma_threshold, tail_avg_iters, learning_rate_end, perturb_scale,
                 avg_grad_norm):
    native = isinstance(objective_and_grad, NativeObjective)
    if native and has_log_norm:
        raise ValueError('not enough values to unpack (expected 3, got 2)')
    if learning_rate <= 0:
        raise ValueError('learning rate must be positive')
    if learning_rate_end is not None and learning_rate <= learning_rate_end:
        raise ValueError('initial learning rate must be greater than final learning rate')
    if not native or avg_grad_norm:
        lams, hists, values, log_norms = _ia_host_chains(
            opt, int(n_iters), objective_and_grad, np.asarray(init_param, dtype=float),
            has_log_norm, window, learning_rate, epsilon, learning_rate_end, n_optimisers,
            perturb_scale, avg_grad_norm)
        return _ia_finish(lams, hists, values, log_norms, int(n_iters), K, rhat_window,
                          r_mean_threshold, r_sigma_threshold, tail_avg_iters, n_optimisers)
    obj = objective_and_grad
    fam = obj.family
    init_param = np.asarray(init_param, dtype=float)
    n_iters = int(n_iters)
    inits = []
    for o in range(n_optimisers):
        np.random.seed(seed=o)                                       # vb.py:418 / 584
        if o == 0:
            inits.append(init_param.copy())
        else:
            inits.append(init_param + np.random.randn(len(init_param)) * (o + 1) * perturb_scale)
        if fam.rng == 'numpy':
            # chains run one after another like the reference: the objective's
            # draws (family stream / global-RNG CHIVI seeds) follow seed(o)
            run = DeviceRun(obj, n_iters, inits[o][None, :], window, learning_rate, epsilon,
                            learning_rate_end, optimizer=opt)
            per_step = obj.n_samples * (fam.dim + 1)
            chunk = max(1, min(n_iters, _HOST_CHUNK_ELEMS // max(per_step, 1)))
            done = 0
            while done < n_iters:
                cs = min(chunk, n_iters - done)
                run.advance_host(np.stack([obj._eps_one_call() for _ in range(cs)])[None])
                done += cs
            lam, hist, vals, _ = run.result()
            if o == 0:
                lams, hists, valss = [], [], []
            lams.append(lam[0])
            hists.append(hist[0])
            valss.append(vals[0])
    if fam.rng == 'philox':
        # independent chains: one launch chain, one Philox stream per chain
        run = DeviceRun(obj, n_iters, np.stack(inits), window, learning_rate, epsilon,
                        learning_rate_end, optimizer=opt)
        run.advance_philox(n_iters, fam.seed, fam.stream, fam.step, stream_stride=1)
        fam.step += n_iters
        lam, hist, vals, _ = run.result()
        lams, hists, valss = list(lam), list(hist), list(vals)
    values = np.concatenate(valss)
    return _ia_finish(lams, hists, values, np.zeros(len(values)), n_iters, K, rhat_window,
                      r_mean_threshold, r_sigma_threshold, tail_avg_iters, n_optimisers)


def _ia_host_chains(opt, n_iters, objective_and_grad, init_param, has_log_norm, window,
                    learning_rate, epsilon, learning_rate_end, n_optimisers, perturb_scale,
                    avg_grad_norm):
    """RMSProp-IA / Adam-IA chains for a caller-supplied objective (or with
    avg_grad_norm): the objective runs where the caller's code runs, each
    update in the device kernel vb_ia_update on device-resident state
    (vb.py:417-468, 583-631).  Returns the final parameters and pre-update
    histories per chain plus the value / log-norm histories of all chains."""
    import collections
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError('viabel_amd IA optimisers need a GPU')
    dev = torch.device('cuda', nat.context().device)
    P = init_param.size
    lams, hists, values, log_norms = [], [], [], []
    alpha = 0.9
    for o in range(n_optimisers):
        np.random.seed(seed=o)                                        # vb.py:418 / 584
        init = init_param.copy() if o == 0 else (
            init_param + np.random.randn(P) * (o + 1) * perturb_scale)
        lam = torch.tensor(init, dtype=torch.float64, device=dev)
        state = torch.zeros((2, P), dtype=torch.float64, device=dev)
        hist = collections.deque(maxlen=100 * window)                 # vb.py:465-466
        sched = learning_rate_schedule(n_iters, learning_rate, learning_rate_end)
        for i, lr in zip(range(n_iters), sched):
            cur = lam.cpu().numpy()
            if has_log_norm:
                val, g, log_norm = objective_and_grad(cur)
            else:
                val, g = objective_and_grad(cur)
                log_norm = 0
            values.append(val)
            log_norms.append(log_norm)
            g = nat.as_f64(g)
            kind, norm2 = opt, 0.0
            if avg_grad_norm:
                # vb.py:443-451 (the reference's own arithmetic, on the host scalar)
                grad_norm = np.exp(log_norm) if has_log_norm else np.sum(g ** 2, axis=0)
                norm2 = grad_norm if i == 0 else grad_norm * alpha + (1. - alpha) * grad_norm
                kind = nat.OPT_RMSPROP_IA_NORM
            nat.check(nat.lib().vb_ia_update(nat.context().handle, kind, P, nat.dptr(lam),
                                             nat.dptr(g), nat.dptr(state), i, lr, epsilon,
                                             float(norm2), None))
            hist.append(cur.copy())
        lams.append(lam.cpu().numpy())
        hists.append(np.array(hist))
    return lams, hists, np.array(values), np.array(log_norms, dtype=float)


def _ia_avg_starts(rm, rs, n_iters, rhat_window, r_mean_threshold, r_sigma_threshold,
                   tail_avg_iters):
    """First window pair whose R-hats are all below the thresholds (vb.py:495-512)."""
    start_m = start_s = n_iters - tail_avg_iters
    for ee in range(rm.shape[0] - 1):
        if (rm[ee] < r_mean_threshold).all() and (rm[ee + 1] < r_mean_threshold).all():
            start_m = ee * rhat_window
            break
    for ee in range(rs.shape[0] - 1):
        if (rs[ee] < r_sigma_threshold).all() and (rs[ee + 1] < r_sigma_threshold).all():
            start_s = ee * rhat_window
            break
    return start_m, start_s


def _ia_inits(init_param, n_optimisers, perturb_scale):
    """Chain o's start: init_param for o = 0, else init_param + randn * (o + 1) *
    perturb_scale after np.random.seed(o) (vb.py:418-421 / 583-586); the global
    RNG is left where the reference leaves it."""
    inits = []
    for o in range(n_optimisers):
        np.random.seed(seed=o)
        if o == 0:
            inits.append(init_param.copy())
        else:
            inits.append(init_param + np.random.randn(len(init_param)) * (o + 1) * perturb_scale)
    return inits


def _ia_finish(lams, hists, values, log_norms, n_iters, K, rhat_window, r_mean_threshold,
               r_sigma_threshold, tail_avg_iters, n_optimisers):
    """R-hat windows and iterate averaging of the chains (vb.py:486-553)."""
    from . import functions
    chains = np.stack(hists, axis=0)
    rhats = functions.compute_R_hat_adaptive_numpy(chains, window_size=rhat_window)
    rhats_halfway = functions.compute_R_hat_halfway(chains, interval=100, start=200)
    rm, rs = rhats[:, :K], rhats[:, K:]
    start_m, start_s = _ia_avg_starts(rm, rs, n_iters, rhat_window, r_mean_threshold,
                                      r_sigma_threshold, tail_avg_iters)
    means, sigmas = [], []
    for o in range(n_optimisers):
        means.append(functions.stochastic_iterate_averaging(chains[o, :, :K], start_m)[0])
        sigmas.append(functions.stochastic_iterate_averaging(chains[o, :, K:], start_s)[0])
    log = {'start_avg_mean_iters': start_m, 'start_avg_sigma_iters': start_s,
           'r_hat_mean': rm, 'r_hat_sigma': rs,
           'r_hat_mean_halfway': rhats_halfway[:, :K], 'r_hat_sigma_halfway': rhats_halfway[:, K:]}
    return (lams[-1], chains, means, sigmas, values, log_norms, log)


def rmsprop_IA_optimize_with_rhat(n_iters, objective_and_grad, init_param, K,
                                  has_log_norm=False, window=500, learning_rate=.01,
                                  epsilon=.000001, rhat_window=500, averaging=True,
                                  n_optimisers=1, r_mean_threshold=1.15, r_sigma_threshold=1.20,
                                  tail_avg_iters=2000, avg_grad_norm=False,
                                  learning_rate_end=None, sharded=False, group=None,
                                  gather_histories=False):
    """vb.py:392-553: RMSProp (decay .9) chains, windowed / halfway R-hat, and
    iterate averaging from the first pair of windows whose R-hat is below the
    thresholds.  Returns (final param of the last chain, history chains
    [n_optimisers, n_hist, P], averaged means per chain, averaged sigmas per
    chain, values, log norms, log dict).  The updates run on the device
    (vb_run, optimizer RMSPROP_IA); R-hat and averaging too (vb_rhat,
    vb_iterate_average).

    sharded=True (a Philox-noise native objective under torch.distributed): the
    chains are dealt to the ranks of `group` (restarts.run_ia_chains: chain o on
    rank o % world, one gather of per-chain R-hat statistics); the R-hat
    diagnostics and averaging starts equal the one-process run's.  The returned
    histories and averages are then this rank's chains unless gather_histories."""
    if sharded:
        from . import restarts
        return restarts.run_ia_chains(
            nat.OPT_RMSPROP_IA, n_iters, objective_and_grad, init_param, K,
            has_log_norm=has_log_norm, window=window, learning_rate=learning_rate,
            epsilon=epsilon, rhat_window=rhat_window, n_optimisers=n_optimisers,
            r_mean_threshold=r_mean_threshold, r_sigma_threshold=r_sigma_threshold,
            tail_avg_iters=tail_avg_iters, learning_rate_end=learning_rate_end,
            perturb_scale=0.5, avg_grad_norm=avg_grad_norm, group=group,
            gather_histories=gather_histories)
    return _ia_optimize(nat.OPT_RMSPROP_IA, n_iters, objective_and_grad, init_param, K,
                        has_log_norm, window, learning_rate, epsilon, rhat_window, n_optimisers,
                        r_mean_threshold, r_sigma_threshold, tail_avg_iters, learning_rate_end,
                        0.5, avg_grad_norm)


def adam_IA_optimize_with_rhat(n_iters, objective_and_grad, init_param, K,
                               has_log_norm=False, window=500, learning_rate=.01,
                               epsilon=.000001, rhat_window=500, averaging=True, n_optimisers=1,
                               r_mean_threshold=1.15, r_sigma_threshold=1.20,
                               tail_avg_iters=2000, learning_rate_end=None, sharded=False,
                               group=None, gather_histories=False):
    """vb.py:556-712: Adam (beta1 .9, beta2 .999, bias correction with i + 2)
    chains; same diagnostics, return value and sharding as
    rmsprop_IA_optimize_with_rhat."""
    if sharded:
        from . import restarts
        return restarts.run_ia_chains(
            nat.OPT_ADAM_IA, n_iters, objective_and_grad, init_param, K,
            has_log_norm=has_log_norm, window=window, learning_rate=learning_rate,
            epsilon=epsilon, rhat_window=rhat_window, n_optimisers=n_optimisers,
            r_mean_threshold=r_mean_threshold, r_sigma_threshold=r_sigma_threshold,
            tail_avg_iters=tail_avg_iters, learning_rate_end=learning_rate_end,
            perturb_scale=0.2, avg_grad_norm=False, group=group,
            gather_histories=gather_histories)
    return _ia_optimize(nat.OPT_ADAM_IA, n_iters, objective_and_grad, init_param, K,
                        has_log_norm, window, learning_rate, epsilon, rhat_window, n_optimisers,
                        r_mean_threshold, r_sigma_threshold, tail_avg_iters, learning_rate_end,
                        0.2, False)
