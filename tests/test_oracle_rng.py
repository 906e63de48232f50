"""Pin the C restatement of the device noise (oracle/vbrng.c): Random123
known-answer vectors for Philox4x32-10 and distributional checks of the normal
and t transforms.  CPU only."""
import numpy as np
import pytest
from scipy import stats

from oracle import rng_oracle

# Random123 kat_vectors, philox4x32 with 10 rounds: (counter, key) -> output
KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize('ctr,key,out', KAT)
def test_philox_known_answers(ctr, key, out):
    assert rng_oracle.philox(ctr, key) == out


def test_normal_draws_are_standard_normal():
    z = rng_oracle.noise(seed=11, stream=3, step=0, n=20000, dim=10)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert stats.kstest(z.ravel(), 'norm').pvalue > 1e-3


def test_t_draws_match_student_t():
    df = 8.0
    z = rng_oracle.noise(seed=5, stream=1, step=2, n=20000, dim=6, family='t', df=df)
    assert abs(z.var() - df / (df - 2)) < 0.03
    assert stats.kstest(z.ravel(), 't', args=(df,)).pvalue > 1e-3


@pytest.mark.parametrize('df', [3.0, 8.0, 40.0])
def test_bailey_t_draws_match_student_t(df):
    """Bailey's trigonometric t (the log-weight draws of the t family, vbrng.c
    family 2): KS against scipy's t, the variance, and no correlation between a
    row's consecutive variates (a pair's two variates use disjoint words)."""
    z = rng_oracle.noise(seed=5, stream=1, step=2, n=40000, dim=6, family='t_bailey', df=df)
    assert stats.kstest(z.ravel(), 't', args=(df,)).pvalue > 1e-3
    if df > 4:
        assert abs(z.var() / (df / (df - 2)) - 1) < 0.03
    r = np.corrcoef(z[:, :-1].ravel(), z[:, 1:].ravel())[0, 1]
    assert abs(r) < 0.01
    # counter addressing by column pair: a row's first variates do not depend on D
    z3 = rng_oracle.noise(seed=5, stream=1, step=2, n=50, dim=3, family='t_bailey', df=df)
    np.testing.assert_array_equal(z3, z[:50, :3])


def test_counter_addressing():
    """Draws depend only on (seed, stream, step, sample, column): any row block
    regenerates identically, different steps/streams differ."""
    a = rng_oracle.noise(1, 7, 4, 6, 5)
    b = rng_oracle.noise(1, 7, 4, 3, 5)
    np.testing.assert_array_equal(a[:3], b)
    assert not np.allclose(a, rng_oracle.noise(1, 7, 5, 6, 5))
    assert not np.allclose(a, rng_oracle.noise(1, 8, 4, 6, 5))
    assert not np.allclose(a, rng_oracle.noise(2, 7, 4, 6, 5))
