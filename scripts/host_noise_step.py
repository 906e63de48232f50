"""Step time of the block kernel when the standardized draws are already on the
device (vb_run_advance with device-resident noise: the block kernel's HOST
path) vs in-kernel Philox draws, for the block-kernel configs."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main():
    import torch
    from viabel_amd import vb, targets, _native as nat
    steps = 2000
    for fam_kind, tgt, D, N, objk in [('t', 'funnel', 10, 128, 'chivi'), ('t', 'eight_schools_ncp', 10, 100, 'klvi'),
                                      ('gauss', 'mixture', 2, 100, 'klvi')]:
        fam = (vb.mean_field_gaussian_variational_family(D, rng='philox') if fam_kind == 'gauss'
               else vb.mean_field_t_variational_family(D, 40.0, rng='philox'))
        t = targets.eight_schools_ncp() if tgt == 'eight_schools_ncp' else getattr(targets, tgt)(D)
        obj = vb.black_box_klvi(fam, t, N) if objk == 'klvi' else vb.black_box_chivi(2.0, fam, t, N)
        init = np.zeros(2 * D)
        eps = torch.randn(1, steps, N, D, dtype=torch.float64, device='cuda')
        for mode in ['philox', 'device_noise', 'philox', 'device_noise']:
            run = vb.DeviceRun(obj, 2 * steps, init[None], learning_rate=.001)
            if mode == 'philox':
                run.advance_philox(100, 0, 1, 0)
            nat.context().synchronize()
            t0 = time.perf_counter()
            if mode == 'philox':
                run.advance_philox(steps, 0, 1, 100)
            else:   # device-resident noise, used in place (no PCIe)
                nz = nat.Noise(nat.NOISE_HOST, 0, 0, 0, nat.dptr(eps))
                nat.check(nat.lib().vb_run_advance(run.handle, steps, nz))
            nat.context().synchronize()
            dt = (time.perf_counter() - t0) / steps
            print(json.dumps({'fam': fam_kind, 'target': tgt, 'D': D, 'N': N, 'obj': objk, 'mode': mode,
                              'us_per_step': round(dt * 1e6, 3)}), flush=True)


if __name__ == '__main__':
    main()
