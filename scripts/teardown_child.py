"""A program that uses the library and exits WITHOUT _native.release_all():
a >= 8-problem mean-field t DeviceRun (its pre-draw overlaps the block kernel on
CU-masked streams, vb_capi.hip predraw_overlap_streams), a full-rank call (the
fr workspace) and a short config-5 restart table (log weights, bounds, PSIS).
Round 5 saw the process teardown crash under rocprofv3 with such streams alive;
the library and _native now release them before the HIP runtime's own teardown.
tests/test_gpu_teardown.py runs this in a child process (plain and under
rocprofv3) and asserts rc 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    from viabel_amd import vb, targets, restarts
    os.environ.setdefault('VIABEL_AMD_PROGRESS', '0')
    fam = vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    obj = vb.black_box_klvi(fam, targets.eight_schools_ncp(), 100)
    run = vb.DeviceRun(obj, 600, restarts.default_inits(16, fam.var_param_dim), window=10,
                       learning_rate=.01, learning_rate_end=.001)
    run.advance_philox(600, 0, 1, 0, stream_stride=1)
    lam, _, vals, _ = run.result(history=False)
    assert np.isfinite(vals).all()
    fr = vb.t_variational_family(8, 40.0, rng='philox')
    fobj = vb.black_box_chivi(2.0, fr, targets.isogauss(8), 64)
    v, g = fobj(np.zeros(fr.var_param_dim))
    assert np.isfinite(v) and np.isfinite(g).all()
    fac = lambda: vb.mean_field_t_variational_family(10, 40.0, rng='philox')
    tab = restarts.run_restarts(fac, targets.eight_schools_ncp(), 8, 200, n_bounds=20000)
    assert tab.shape[0] == 8
    print('teardown child done: %d problems, k-hat %.3f..%.3f' % (
        lam.shape[0], tab[:, 8].min(), tab[:, 8].max()), flush=True)
    # objects still referenced at exit on purpose: `run`, `fobj`
    globals()['_keep'] = (run, fobj)


if __name__ == '__main__':
    main()
