"""Disassembly checks of the built gfx950 code (no GPU).

The block kernel's copy-wave instances (`block_kernel<..., PF = true>`) read each
noise row from the LDS ring with hand-written `ds_read_b64` and wait for them with
an explicit `s_waitcnt lgkmcnt(0)` (vb_mf.hip `LdsRowWait`): the hardware has no
interlock between an LDS load and a later read of its destination register, so no
instruction may touch those registers between the reads and the wait.  Reads and
wait are one asm statement; this test guards that the emitted code keeps them
adjacent (a compiler upgrade or an edit that splits the statement would show up
here) and that the instances do not spill to scratch."""
import os
import re
import shutil
import subprocess

import pytest

from tests.conftest import ROOT

OBJ = os.path.join(ROOT, 'viabel_amd', 'csrc', 'build', 'vb_mf.o')
OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'


@pytest.fixture(scope='module')
def disasm(tmp_path_factory):
    if not (os.path.exists(OBJ) and os.path.exists(OBJDUMP)):
        pytest.skip('needs the in-tree build objects and llvm-objdump')
    d = tmp_path_factory.mktemp('co')
    o = str(d / 'vb_mf.o')
    shutil.copy(OBJ, o)
    subprocess.check_call([OBJDUMP, '--offloading', o], cwd=str(d), stdout=subprocess.DEVNULL)
    dev = [str(d / f) for f in os.listdir(str(d)) if 'gfx950' in f]
    assert dev, os.listdir(str(d))
    txt = subprocess.check_output([OBJDUMP, '-d', '--demangle', dev[0]], text=True)
    funcs, cur = {}, None
    for line in txt.split('\n'):
        m = re.match(r'^[0-9a-f]+ <(.*)>:', line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        ins = line.split('//')[0].strip()
        if cur and ins:
            funcs[cur].append(ins)
    return funcs


PF_RE = re.compile(r'block_kernel<vbd::\w+, (true|false), true, (\d+), true, (?:true|false)>')


def test_copy_wave_row_reads_are_waited_before_any_other_instruction(disasm):
    pf = {f: b for f, b in disasm.items() if PF_RE.search(f)}
    assert len(pf) >= 8, sorted(disasm)[:5]
    for f, body in pf.items():
        dmax = int(PF_RE.search(f).group(2))
        runs = 0
        for i, ins in enumerate(body):
            m = re.match(r'ds_read_b64 v\[\d+:\d+\], (v\d+)$', ins)
            if not m:
                continue
            base = m.group(1)
            seq = body[i:i + dmax]
            want = ['offset:%d' % (8 * k) for k in range(1, dmax)]
            if not all(s.startswith('ds_read_b64') and s.split(', ')[1].split()[0] == base
                       for s in seq) or [s.split()[-1] for s in seq[1:]] != want:
                continue
            runs += 1
            nxt = body[i + dmax]
            if nxt.startswith('ds_read_b64'):          # the row's log q partial
                assert 'offset' not in nxt, (f, nxt)
                nxt = body[i + dmax + 1]
            assert nxt == 's_waitcnt lgkmcnt(0)', (f, body[i:i + dmax + 2])
        assert runs >= 1, f


def test_copy_wave_instances_do_not_spill(disasm):
    for f, body in disasm.items():
        if PF_RE.search(f):
            assert not any(i.startswith('scratch_') or i.startswith('buffer_store') for i in body), f
