"""viabel_amd -- MI355X (gfx950) implementation of viabel's Monte Carlo VI hot path.

Mirrors the reference package layout: ``viabel_amd`` re-exports the bounds
(reference viabel/__init__.py:1), ``viabel_amd.vb`` holds the variational
families, estimators and adagrad, ``viabel_amd.psis`` the PSIS routines of
notebooks/psis.py, ``viabel_amd.targets`` the device log densities.
All arithmetic runs in the HIP library libviabel_amd.so (include/viabel_amd.h).
"""
from .bounds import *  # noqa: F401,F403

__version__ = '0.1.0'
