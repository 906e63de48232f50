"""The XCD-grouped block order of the symmetric-sum products
(vb_symsum.hpp geo_xcd) is a permutation of geo()'s units for every tile count:
every (row half, column tile) of the upper triangle and every diagonal tile is
computed by exactly one block.  Host code compiled with hipcc (no GPU needed)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = '/opt/rocm/bin/hipcc'

_SRC = r'''
#include "vb_symsum.hpp"
#include <cstdio>
#include <set>
#include <tuple>
int main() {
  for (int nt = 1; nt <= 40; ++nt) {
    std::set<std::tuple<int, int, int>> a, b;
    for (int i = 0; i < nt * nt; ++i) {
      const auto g = vbk::symsum::geo(i, nt);
      const auto h = vbk::symsum::geo_xcd(i, nt);
      a.insert(std::make_tuple(g.r0, g.c0, (int)g.diag));
      b.insert(std::make_tuple(h.r0, h.c0, (int)h.diag));
      const bool ok = h.c0 == 32 * h.bj && h.bi <= h.bj && (h.diag == (h.bi == h.bj)) &&
                      h.r0 == 32 * h.bi + (h.diag ? 0 : h.r0 - 32 * h.bi) &&
                      (h.r0 - 32 * h.bi == 0 || h.r0 - 32 * h.bi == 16) && h.bj < nt;
      if (!ok) { printf("nt %d block %d: bad geometry\n", nt, i); return 1; }
    }
    if (a != b || (int)a.size() != nt * nt) { printf("nt %d: not a permutation\n", nt); return 1; }
  }
  printf("ok\n");
  return 0;
}
'''


@pytest.mark.skipif(not os.path.exists(HIPCC), reason='needs hipcc')
def test_xcd_order_is_a_permutation_of_the_units(tmp_path):
    src = tmp_path / 'geo.cpp'
    src.write_text(_SRC)
    exe = tmp_path / 'geo'
    r = subprocess.run([HIPCC, '--offload-arch=gfx950', '-std=c++17', '-O1',
                        '-I', os.path.join(ROOT, 'viabel_amd', 'csrc'), str(src), '-o', str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == 'ok', out.stdout + out.stderr
