"""Pin the vb restatement (oracle/vb_oracle.py).  The reference vb module is not
importable here (autograd/paragami absent), so its gradients are checked by
independent AD: torch.autograd in fp64 differentiating the REFERENCE's forward
formulas (sample -> logdensity -> objective, vb.py:237-241 and 249-263) with
the same injected noise, plus central finite differences.  CPU only."""
import math

import numpy as np
import pytest
import torch

from oracle import targets_oracle, vb_oracle

torch.set_default_dtype(torch.float64)
LOG2PI = math.log(2 * math.pi)


# ---- torch versions of the reference forward formulas -----------------------
def t_norm_logpdf(x, loc, scale):
    z = (x - loc) / scale
    return -0.5 * z * z - torch.log(scale) - 0.5 * LOG2PI


def t_target(name, x):
    if name == 'isogauss':
        return torch.sum(-0.5 * x * x - 0.5 * LOG2PI, dim=1)
    if name == 'mixture':
        one = torch.tensor(1.0)
        a = t_norm_logpdf(x, -2.0, one)
        b = t_norm_logpdf(x, 2.0, one)
        return torch.sum(torch.logaddexp(a, b) - math.log(2), dim=1)
    if name == 'funnel':
        v = x[:, 1]
        lp = t_norm_logpdf(v, 0.0, torch.tensor(1.35))
        for d in range(x.shape[1]):
            if d != 1:
                lp = lp + t_norm_logpdf(x[:, d], 0.0, torch.exp(v))
        return lp
    if name == 'eight_schools_ncp':
        y = torch.tensor(targets_oracle.ES_Y)
        sg = torch.tensor(targets_oracle.ES_SIGMA)
        mu, u, th = x[:, 0], x[:, 1], x[:, 2:]
        tau = torch.exp(u)
        theta = mu[:, None] + tau[:, None] * th
        return (-0.5 * (mu / 5) ** 2 - torch.log1p((tau / 5) ** 2) + u
                - 0.5 * torch.sum(th ** 2, 1) - 0.5 * torch.sum(((y - theta) / sg) ** 2, 1))
    raise KeyError(name)


def t_logq(kind, df, x, mu, ls):
    """mvn.logpdf with diag cov (vb.py:65) / sum of t.logpdf (vb.py:162)."""
    if kind == 'gauss':
        cov = torch.diag(torch.exp(2 * ls))
        dist = torch.distributions.MultivariateNormal(mu, covariance_matrix=cov)
        return dist.log_prob(x)
    dist = torch.distributions.StudentT(df, mu, torch.exp(ls))
    return torch.sum(dist.log_prob(x), dim=1)


def t_klvi(kind, df, target, lam, eps):
    D = eps.shape[1]
    mu, ls = lam[:D], lam[D:]
    x = eps * torch.exp(ls) + mu if kind == 'gauss' else mu + torch.exp(ls) * eps
    ent = (0.5 * D * (1 + LOG2PI) + torch.sum(ls)) if kind == 'gauss' else torch.sum(ls)
    return -(ent + torch.mean(t_target(target, x)))


def t_chivi(kind, df, target, lam, eps, alpha):
    D = eps.shape[1]
    mu, ls = lam[:D], lam[D:]
    x = eps * torch.exp(ls) + mu if kind == 'gauss' else mu + torch.exp(ls) * eps
    lw = t_target(target, x) - t_logq(kind, df, x, mu, ls)
    # vb.py:260-263: grad = alpha * VJP(lw)(w) / N with w held constant
    log_norm = torch.max(lw).detach()
    w = (torch.exp(lw - log_norm) ** alpha).detach()
    value = torch.log(torch.mean(w)) / alpha + log_norm
    (alpha * torch.sum(w * lw) / w.numel()).backward()
    return value.item(), lam.grad.numpy().copy()


CASES = [('gauss', None, 'isogauss', 6), ('gauss', None, 'mixture', 5), ('gauss', None, 'funnel', 4),
         ('t', 40.0, 'funnel', 10), ('t', 8.0, 'eight_schools_ncp', 10), ('gauss', None, 'eight_schools_ncp', 10),
         ('t', 5.0, 'mixture', 3)]


def _lam(D, seed):
    rs = np.random.RandomState(seed)
    return np.concatenate([rs.randn(D) * 0.7, rs.randn(D) * 0.3 - 0.2])


@pytest.mark.parametrize('kind,df,target,D', CASES)
def test_klvi_gradient_vs_torch_autograd(kind, df, target, D):
    fam = vb_oracle.Family(kind, D, df)
    lam = _lam(D, 3)
    eps = fam.draw(64)
    val, grad = vb_oracle.klvi_value_grad(fam, target, lam, 64, eps=eps)
    tl = torch.tensor(lam, requires_grad=True)
    tv = t_klvi(kind, df, target, tl, torch.tensor(eps))
    tv.backward()
    np.testing.assert_allclose(val, tv.item(), rtol=1e-12)
    np.testing.assert_allclose(grad, tl.grad.numpy(), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize('kind,df,target,D', CASES)
@pytest.mark.parametrize('alpha', [2.0, 1.5])
def test_chivi_gradient_vs_torch_autograd(kind, df, target, D, alpha):
    fam = vb_oracle.Family(kind, D, df)
    lam = _lam(D, 4)
    eps = fam.draw(50, seed=123)
    val, grad = vb_oracle.chivi_value_grad(fam, target, lam, 50, alpha, eps=eps)
    tl = torch.tensor(lam, requires_grad=True)
    tval, tgrad = t_chivi(kind, df, target, tl, torch.tensor(eps), alpha)
    np.testing.assert_allclose(val, tval, rtol=1e-11)
    np.testing.assert_allclose(grad, tgrad, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize('kind,df,target,D', CASES)
def test_klvi_pd_gradient_vs_torch_autograd(kind, df, target, D):
    """black_box_klvi_pd (vb.py:268-278): autograd through samples AND lambda in log q."""
    fam = vb_oracle.Family(kind, D, df)
    lam = _lam(D, 5)
    eps = fam.draw(40)
    val, grad = vb_oracle.klvi_pd_value_grad(fam, target, lam, 40, eps=eps)
    tl = torch.tensor(lam, requires_grad=True)
    mu, ls = tl[:D], tl[D:]
    te = torch.tensor(eps)
    x = te * torch.exp(ls) + mu
    tv = -(torch.mean(t_target(target, x)) - torch.mean(t_logq(kind, df, x, mu, ls)))
    tv.backward()
    np.testing.assert_allclose(val, tv.item(), rtol=1e-11)
    np.testing.assert_allclose(grad, tl.grad.numpy(), rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize('target', ['isogauss', 'mixture', 'funnel', 'eight_schools_ncp'])
def test_target_grad_finite_differences(target):
    D = 10 if target == 'eight_schools_ncp' else 4
    x = np.random.RandomState(5).randn(3, D) * 0.8
    lp, g = targets_oracle.TARGETS[target](x)
    h = 1e-6
    for d in range(D):
        e = np.zeros(D)
        e[d] = h
        fd = (targets_oracle.TARGETS[target](x + e)[0] - targets_oracle.TARGETS[target](x - e)[0]) / (2 * h)
        np.testing.assert_allclose(g[:, d], fd, rtol=1e-6, atol=1e-6)
    tx = torch.tensor(x)
    np.testing.assert_allclose(lp, t_target(target, tx).numpy(), rtol=1e-13)


@pytest.mark.parametrize('kind,df', [('gauss', None), ('t', 40.0)])
def test_family_logdensity_matches_scipy(kind, df):
    from scipy.stats import multivariate_normal, t
    D = 4
    fam = vb_oracle.Family(kind, D, df)
    lam = _lam(D, 9)
    x = fam.sample(lam, 7)
    ref = (multivariate_normal.logpdf(x, lam[:D], np.diag(np.exp(2 * lam[D:])))
           if kind == 'gauss' else np.sum(t.logpdf(x, df, lam[:D], np.exp(lam[D:])), axis=-1))
    np.testing.assert_allclose(fam.logdensity(x, lam), ref, rtol=1e-12)


def test_learning_rate_schedule_shape():
    lrs = vb_oracle.learning_rate_schedule(100, 0.01, 0.001)
    assert lrs[0] == 0.01 and lrs[24] == 0.01 and lrs[75] == 0.001 and lrs[-1] == 0.001
    assert all(lrs[i] >= lrs[i + 1] for i in range(99))
    assert vb_oracle.learning_rate_schedule(5, 0.1, None) == [0.1] * 5
    with pytest.raises(ValueError, match='learning rate must be positive'):
        vb_oracle.learning_rate_schedule(5, 0.0, None)
    with pytest.raises(ValueError, match='initial learning rate must be greater'):
        vb_oracle.learning_rate_schedule(5, 0.01, 0.1)


def test_klvi_adagrad_converges_on_isogauss():
    D = 3
    fam = vb_oracle.Family('gauss', D)
    obj = lambda l: vb_oracle.klvi_value_grad(fam, 'isogauss', l, 200)
    sm, hist, vals, ln = vb_oracle.adagrad_optimize(2000, obj, np.ones(2 * D), learning_rate=0.1)
    assert hist.shape == (500, 2 * D) and vals.shape == (2000,) and np.all(ln == 0)
    np.testing.assert_allclose(sm, np.zeros(2 * D), atol=0.05)
