"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference algorithms on the hot path, used as the
checker for the HIP implementation in ``viabel_amd``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything from this package; the product (``viabel_amd``) never does and fails
loudly when its HIP library is missing.

Modules
-------
vb_oracle      numpy restatement of viabel/vb.py:48-82, 140-182, 236-266, 324-389
               (families, KLVI, CHIVI, learning-rate schedule, adagrad) with
               analytic gradients in place of autograd's tape, drawing noise
               from numpy's legacy RandomState exactly as the reference does.
targets_oracle target log densities + gradients.
bounds_oracle  restatement of viabel/bounds.py:13-213.
psis_oracle    restatement of notebooks/psis.py:112-395.
rng_oracle     ctypes binding of vbrng.c, the C restatement of the device
               Philox noise (VB_NOISE_PHILOX).

Pinning: bounds_oracle and psis_oracle are checked
against golden vectors produced by the importable reference (tests/golden/);
rng_oracle against the Random123 known-answer vectors; numpy RNG streams
against golden draws; vb_oracle's analytic gradients against torch.autograd
(fp64) of the reference's forward formulas and central finite differences.
The reference's vb module itself cannot be imported here (autograd and
paragami are absent), so vb_oracle / fullrank_oracle are pinned by the
reference's own published outputs instead: re-running the notebooks'
reproducible KLVI runs (funnel; robust regression, mean-field t and full-rank t)
reproduces every printed digit (tests/golden/notebook_outputs.json,
tests/test_oracle_notebooks.py), with torch.autograd and finite differences as
an independent check of the analytic gradients.  functions_oracle (R-hat,
iterate averaging) is pinned by a textbook split-R-hat only: the reference's
functions.py imports autograd, so no reference output exists for it here.
"""
