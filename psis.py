"""Top-level ``psis`` module of the reference's notebooks (notebooks/psis.py:
psislw, gpdfitnew, gpinv, sumlogs; psisloo is out of scope): this name IS
viabel_amd.psis, the device implementation, so ``from psis import psislw``
keeps working."""
import sys as _sys

import viabel_amd.psis as _impl

_sys.modules[__name__] = _impl
