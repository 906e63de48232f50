"""Coefficients of vbd::exp_fast (vb_device.hpp): exp(r) = 1 + r + r^2 q(r) on
|r| <= ln2 / 2, q of degree 9 fitted by least squares on 200 Chebyshev nodes in
long double (iterative refinement of a float64 solve).  Prints the C array."""
import numpy as np

ld = np.longdouble
a = ld(np.log(2)) / 2
deg, n = 9, 200
k = np.arange(n, dtype=ld)
nodes = np.cos((2 * k + 1) * ld(np.pi) / (2 * n)) * a


def expm1_series(x):
    s, t = ld(0), ld(1)
    for i in range(1, 40):
        t = t * x / i
        s += t
    return s


q = np.array([(expm1_series(x) - x) / (x * x) for x in nodes], dtype=ld)
V = np.vander(nodes / a, deg + 1, increasing=True).astype(ld)
c = np.linalg.lstsq(V.astype(np.float64), q.astype(np.float64), rcond=None)[0].astype(ld)
for _ in range(5):
    c = c + np.linalg.lstsq(V.astype(np.float64), (q - V.dot(c)).astype(np.float64),
                            rcond=None)[0].astype(ld)
coef = [float(c[i] / a ** i) for i in range(deg + 1)]
print('max fit error of q: %.3g' % float(np.max(np.abs(q - V.dot(c)))))
print('{' + ', '.join(repr(v) for v in coef) + '}')
