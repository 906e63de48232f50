"""Pin the full-rank t restatement (oracle/fullrank_oracle.py): its analytic
KLVI / CHIVI gradients (Sylvester VJP of sqrtm, det VJP, (G + G^T) L chain,
exp-diagonal free parametrisation) against torch.autograd in fp64 through the
reference's forward formulas (sqrtm and multivariate_t_logpdf via eigh, as
_distributions.py does), on identical draws.  CPU only."""
import math

import numpy as np
import pytest
import torch

from oracle import fullrank_oracle as fo

torch.set_default_dtype(torch.float64)


def t_unpack(lam, D):
    mu = lam[:D]
    idx = torch.tril_indices(D, D)
    M = torch.zeros(D, D)
    M = M.index_put((idx[0], idx[1]), lam[D:])
    L = torch.tril(M, -1) + torch.diag(torch.exp(torch.diagonal(M)))
    return mu, L, L @ L.T


def t_sqrtm(S):
    w, V = torch.linalg.eigh(S)
    return V @ torch.diag(torch.sqrt(w)) @ V.T


def t_mvt_logpdf(x, m, S, df):
    d = m.shape[-1]
    s, u = torch.linalg.eigh(S)
    U = u * torch.sqrt(1 / s)
    out = math.lgamma(.5 * (df + d)) - math.lgamma(.5 * df) - .5 * d * math.log(math.pi * df)
    out = out - .5 * torch.sum(torch.log(s))
    maha = torch.sum(((x - m) @ U) ** 2, dim=-1)
    return out - .5 * (df + d) * torch.log(1 + maha / df)


def t_target(name, x, tgt):
    if name == 'corr_gauss':
        P = torch.tensor(tgt.prec)
        return -0.5 * torch.sum(x * (x @ P), dim=1) + tgt.const
    if name == 'isogauss':
        return torch.sum(-0.5 * x * x - 0.5 * math.log(2 * math.pi), dim=1)
    raise KeyError(name)


def _lam(D, seed=4):
    rs = np.random.RandomState(seed)
    lam = np.concatenate([rs.randn(D) * 0.3, np.zeros(D * (D + 1) // 2)])
    tri = np.tril_indices(D)
    free = rs.randn(len(tri[0])) * 0.05
    free[tri[0] == tri[1]] = rs.randn(D) * 0.1          # log-diagonal: non-degenerate
    lam[D:] = free
    return lam


@pytest.mark.parametrize('target,D', [('corr_gauss', 6), ('isogauss', 5), ('corr_gauss', 17)])
def test_fullrank_klvi_grad_vs_autograd(target, D):
    fam = fo.FullRankT(D, 100.0)
    tgt = fo.target_fn(target, D)
    lam = _lam(D)
    draws = fam.draw(40)
    val, grad = fo.klvi_value_grad(fam, tgt, lam, 40, draws=draws)
    tl = torch.tensor(lam, requires_grad=True)
    mu, L, Sig = t_unpack(tl, D)
    s, z = (torch.tensor(a) for a in draws)
    x = mu + (z @ t_sqrtm(Sig)) / s[:, None]
    f = -(.5 * torch.logdet(Sig) + torch.mean(t_target(target, x, tgt)))
    f.backward()
    np.testing.assert_allclose(val, f.item(), rtol=1e-11)
    np.testing.assert_allclose(grad, tl.grad.numpy(), rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize('target,D', [('corr_gauss', 6), ('isogauss', 4)])
@pytest.mark.parametrize('alpha', [2.0, 1.5])
def test_fullrank_chivi_grad_vs_autograd(target, D, alpha):
    fam = fo.FullRankT(D, 100.0)
    tgt = fo.target_fn(target, D)
    lam = _lam(D, 7)
    draws = fam.draw(30, seed=11)
    val, grad = fo.chivi_value_grad(fam, tgt, lam, 30, alpha, draws=draws)
    tl = torch.tensor(lam, requires_grad=True)
    mu, L, Sig = t_unpack(tl, D)
    s, z = (torch.tensor(a) for a in draws)
    x = mu + (z @ t_sqrtm(Sig)) / s[:, None]
    lw = t_target(target, x, tgt) - t_mvt_logpdf(x, mu, Sig, 100.0)
    top = torch.max(lw).detach()
    w = (torch.exp(lw - top) ** alpha).detach()
    (alpha * torch.sum(w * lw) / w.numel()).backward()
    np.testing.assert_allclose(val, (torch.log(torch.mean(w)) / alpha + top).item(), rtol=1e-11)
    np.testing.assert_allclose(grad, tl.grad.numpy(), rtol=1e-7, atol=1e-9)


def test_family_helpers():
    D = 5
    fam = fo.FullRankT(D, 7.0)
    lam = _lam(D, 2)
    mu, L, Sig = fo.unpack(lam, D)
    np.testing.assert_allclose(Sig, Sig.T)
    assert np.all(np.linalg.eigvalsh(Sig) > 0)
    x = fam.sample(lam, 4000)
    assert x.shape == (4000, D)
    from scipy.stats import multivariate_t
    ref = multivariate_t(mu, Sig, df=7.0).logpdf(x[:5])
    np.testing.assert_allclose(fam.logdensity(x[:5], lam), ref, rtol=1e-10)
    assert fam.var_param_dim == D + D * (D + 1) // 2
    with pytest.raises(ValueError, match='df must be greater than 2'):
        fo.FullRankT(3, 2)


def test_fullrank_klvi_pd_vs_autograd():
    D = 6
    fam = fo.FullRankT(D, 100.0)
    tgt = fo.target_fn('corr_gauss', D)
    lam = _lam(D, 9)
    draws = fam.draw(30, seed=5)
    val, grad = fo.klvi_pd_value_grad(fam, tgt, lam, 30, draws=draws)
    tl = torch.tensor(lam, requires_grad=True)
    mu, L, Sig = t_unpack(tl, D)
    s, z = (torch.tensor(a) for a in draws)
    x = mu + (z @ t_sqrtm(Sig)) / s[:, None]
    f = -(torch.mean(t_target('corr_gauss', x, tgt)) - torch.mean(t_mvt_logpdf(x, mu, Sig, 100.0)))
    f.backward()
    np.testing.assert_allclose(val, f.item(), rtol=1e-11)
    np.testing.assert_allclose(grad, tl.grad.numpy(), rtol=1e-7, atol=1e-9)
