"""AddressSanitizer + UndefinedBehaviorSanitizer build of the C noise oracle
(oracle/vbrng.c through oracle/sanitize_main.c): the Random123 known answers and
every entry point over ragged shapes run clean under both sanitizers, and the
sanitized build draws the same bits as the plain build the other tests load
(oracle/liboracle_rng.so).  CPU only; skipped when gcc or its sanitizer runtimes
are missing."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from oracle import rng_oracle

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle')

# the cases of sanitize_main.c: (seed, stream, step, rows, D, family, df)
CASES = [(0, 1, 0, 3, 1, 'gauss', 0.0), (7, 5, 11, 5, 7, 'gauss', 0.0),
         (123456789, 3, 2, 4, 9, 't', 40.0), (1 << 40, 2, 1, 2, 3, 't', 3.0),
         (42, 9, 0, 0, 5, 'gauss', 0.0), (42, 9, 4, 1, 16, 't', 100.0)]


@pytest.fixture(scope='module')
def sanitized_run(tmp_path_factory):
    gcc = shutil.which('gcc')
    if gcc is None:
        pytest.skip('gcc not available')
    exe = str(tmp_path_factory.mktemp('asan') / 'vbrng_asan')
    cmd = [gcc, '-std=gnu11', '-g', '-O1', '-fsanitize=address,undefined',
           '-fno-sanitize-recover=all', '-fno-omit-frame-pointer', '-ffp-contract=off',
           '-I', ORACLE, '-o', exe, os.path.join(ORACLE, 'sanitize_main.c'), '-lm']
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0:
        pytest.skip('sanitizer runtimes not available: ' + b.stderr[-500:])
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:halt_on_error=1',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1')
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    return r


def test_sanitized_oracle_runs_clean(sanitized_run):
    r = sanitized_run
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'runtime error' not in r.stderr and 'AddressSanitizer' not in r.stderr, r.stderr[-3000:]
    assert r.stdout.splitlines()[0] == 'kat ok'


def _parse(stdout):
    out = {}
    for line in stdout.splitlines()[1:]:
        tag, n, *words = line.split()
        assert int(n) == len(words)
        out[tag] = np.array([struct.unpack('<d', bytes.fromhex(w)[::-1])[0] for w in words])
    return out


def test_sanitized_oracle_draws_equal_the_plain_build(sanitized_run):
    got = _parse(sanitized_run.stdout)
    for c, (seed, stream, step, rows, D, fam, df) in enumerate(CASES):
        want = rng_oracle.noise(seed, stream, step, rows, D, fam, df).ravel()
        np.testing.assert_array_equal(got['fill%d' % c], want)
    s, _ = rng_oracle.fr_noise(99, 4, 3, 6, 1, 100.0)
    np.testing.assert_array_equal(got['frscale'], s)
