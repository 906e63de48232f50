"""Drop-in ``viabel`` namespace over viabel_amd (the reference's import paths).

The reference's users and its own tests write ``from viabel import all_bounds,
...`` (viabel/__init__.py:1 re-exports viabel/bounds.py) and ``from viabel.vb
import ...``, ``import viabel.functions``.  These names resolve to the
MI355X implementation: ``viabel.bounds``, ``viabel.vb`` and
``viabel.functions`` ARE the modules viabel_amd.bounds / .vb / .functions
(aliased in sys.modules, so ``import viabel.vb`` and attribute access see the
same objects); the top-level ``psis`` and ``experiments`` modules stand in for
the reference's notebooks/psis.py and notebooks/experiments.py.  Nothing here
computes: every call runs in libviabel_amd.so.
"""
import sys as _sys

from viabel_amd import bounds, vb, functions  # noqa: F401
from viabel_amd.bounds import *  # noqa: F401,F403  (viabel/__init__.py:1)

for _name, _mod in (('bounds', bounds), ('vb', vb), ('functions', functions)):
    _sys.modules[__name__ + '.' + _name] = _mod
del _name, _mod

__version__ = '0.1.0'
