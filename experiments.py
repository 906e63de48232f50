"""Top-level ``experiments`` module of the reference's notebooks
(notebooks/experiments.py: get_samples_and_log_weights, psis_correction,
improve_with_psis, check_accuracy, check_approx_accuracy): this name IS
viabel_amd.experiments, the device implementation."""
import sys as _sys

import viabel_amd.experiments as _impl

_sys.modules[__name__] = _impl
