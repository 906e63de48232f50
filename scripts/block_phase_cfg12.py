"""Phase profile of the block kernel at configs 1 and 2 (run with the VB_BLOCK_PROF
build: VIABEL_AMD_LIB=viabel_amd/libviabel_amd_prof.so): one 2000-step advance each,
the kernel prints per-phase clock64 cycles of a row wave (BLOCKPROF lines)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from viabel_amd import vb, targets, _native as nat
    for name, fam, tgt, D, N, chivi in [
            ('cfg1', 'gauss', 'mixture', 2, 100, False),
            ('cfg2', 't', 'funnel', 10, 128, True),
            ('cfg5', 't', 'eight_schools_ncp', 10, 100, False)]:
        f = (vb.mean_field_gaussian_variational_family(D, rng='philox') if fam == 'gauss'
             else vb.mean_field_t_variational_family(D, 40.0, rng='philox'))
        t = (targets.eight_schools_ncp() if tgt == 'eight_schools_ncp'
             else {'mixture': targets.mixture, 'funnel': targets.funnel}[tgt](D))
        obj = vb.black_box_chivi(2.0, f, t, N) if chivi else vb.black_box_klvi(f, t, N)
        init = np.concatenate([np.zeros(D), np.zeros(D)])
        run = vb.DeviceRun(obj, 2100, init[None], learning_rate=.001)
        run.advance_philox(100, 0, 1, 0)
        print('==', name, flush=True)
        run.advance_philox(2000, 0, 1, 100)
        nat.context().synchronize()


if __name__ == '__main__':
    main()
