"""Disassembly checks of the built gfx950 code (no GPU).

1. The block kernel's copy-wave instances (`block_kernel<..., PF = true>`) read each
noise row from the LDS ring with hand-written `ds_read_b64` and wait for them with
an explicit `s_waitcnt lgkmcnt(0)` (vb_mf.hip `LdsRowWait`): the hardware has no
interlock between an LDS load and a later read of its destination register, so no
instruction may touch those registers between the reads and the wait.  Reads and
wait are one asm statement; this test guards that the emitted code keeps them
adjacent (a compiler upgrade or an edit that splits the statement would show up
here) and that the instances do not spill to scratch.

2. The fp64 MFMA GEMM's main loop (vb_gemm.hpp, every `gemm_f64_kernel` /
`gemm_f64_hook_kernel` instance, and the symmetric-sum products of vb_symsum.hpp
in `fr_pcg_ss_kernel`) issues its operand fragment reads as
inline-asm `ds_read_b64` and waits for them with hand-counted `s_waitcnt
lgkmcnt(N)` statements (4 steps' reads in flight).  `lds_wait_violations`
replays each instance's instruction stream against a model of the LGKM
counter (LDS operations complete in issue order; scalar-memory loads only at
lgkmcnt(0)): no instruction may read or write a `ds_read` destination register
before a wait that guarantees the read has landed.  A compiler that copied a
fragment register between its read and its wait, or an edit that made a count
too large, fails here rather than as a parity error at the tested shapes.  The
instances must not use scratch either."""
import os
import re
import shutil
import subprocess

import pytest

from tests.conftest import ROOT

BUILD = os.path.join(ROOT, 'viabel_amd', 'csrc', 'build')
OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'


def _disassemble(tmp_path_factory, name):
    obj = os.path.join(BUILD, name)
    if not (os.path.exists(obj) and os.path.exists(OBJDUMP)):
        pytest.skip('needs the in-tree build objects and llvm-objdump')
    d = tmp_path_factory.mktemp('co')
    o = str(d / name)
    shutil.copy(obj, o)
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


@pytest.fixture(scope='module')
def disasm(tmp_path_factory):
    return _disassemble(tmp_path_factory, 'vb_mf.o')


@pytest.fixture(scope='module')
def disasm_gemm(tmp_path_factory):
    funcs = {}
    for name in ('vb_fr.o', 'vb_bounds.o'):
        funcs.update({(name, f): b for f, b in _disassemble(tmp_path_factory, name).items()
                      if 'gemm_f64_kernel<' in f or 'gemm_f64_hook_kernel<' in f
                      or 'fr_pcg_ss_kernel' in f or 'symsum_plain_kernel' in f})
    return funcs


PF_RE = re.compile(r'block_kernel<vbd::\w+, (true|false), true, (\d+), true, (?:true|false)(?:, \d+)?>')


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


_REG = re.compile(r'\b([vas])(?:(\d+)\b|\[(\d+):(\d+)\])')


def _regs(text):
    out = set()
    for k, one, lo, hi in _REG.findall(text):
        if one:
            out.add(k + one)
        else:
            out.update(k + str(r) for r in range(int(lo), int(hi) + 1))
    return out


def lds_wait_violations(body):
    """Replay an instruction list against the LGKM counter.  Queue entries are
    (kind, destination registers, index) in issue order; `s_waitcnt lgkmcnt(N)`
    retires an LDS entry once at least N LDS operations were issued after it
    (they complete in issue order) and a scalar-memory entry only at N = 0;
    scalar-memory loads complete out of order, so one issued after an LDS read
    does not count towards that read's N.  Returns the
    (index, instruction, pending register) of every access to the destination of
    an LDS read still in flight.  The replay follows the listing: an
    unconditional branch ends the straight-line run (the following instruction is
    a jump target, replayed from an empty counter)."""
    queue, bad = [], []
    for i, ins in enumerate(body):
        op = ins.split()[0]
        if op == 's_waitcnt':
            m = re.search(r'lgkmcnt\((\d+)\)', ins)
            if m:
                n = int(m.group(1))
                lds_after = [sum(1 for q in queue[j + 1:] if q[0] == 'lds') for j in range(len(queue))]
                queue = [q for j, q in enumerate(queue)
                         if not ((q[0] == 'lds' and lds_after[j] >= n) or n == 0)]
            continue
        if op in ('s_branch', 's_endpgm', 's_setpc_b64'):
            # the next instruction in the listing is not this one's successor (it
            # is reached by a jump, from other waits): start from an empty counter
            queue = []
            continue
        pending = set().union(*[q[1] for q in queue if q[0] == 'lds']) if queue else set()
        hit = _regs(ins) & pending
        if hit:
            bad.append((i, ins, sorted(hit)))
        if op.startswith('ds_'):
            dest = _regs(ins.split(',')[0]) if op.startswith('ds_read') else set()
            queue.append(('lds', dest, i))
        elif op.startswith('s_load') or op.startswith('s_buffer_load') or op == 's_memtime':
            queue.append(('smem', set(), i))
    return bad


def test_lds_wait_model_catches_a_copy_before_the_wait():
    ok = ['ds_read_b64 v[60:61], v59', 'ds_read_b64 v[62:63], v58', 's_waitcnt lgkmcnt(1)',
          'v_mov_b32_e32 v1, v60', 's_waitcnt lgkmcnt(0)', 'v_mov_b32_e32 v2, v62']
    assert lds_wait_violations(ok) == []
    early = ['ds_read_b64 v[60:61], v59', 'ds_read_b64 v[62:63], v58', 's_waitcnt lgkmcnt(1)',
             'v_mov_b32_e32 v2, v63', 's_waitcnt lgkmcnt(0)']
    assert [b[2] for b in lds_wait_violations(early)] == [['v63']]
    loose = ['ds_read_b64 v[60:61], v59', 's_load_dwordx2 s[4:5], s[0:1], 0x0',
             's_waitcnt lgkmcnt(1)', 'v_mov_b32_e32 v1, v60']
    assert lds_wait_violations(loose) == [(3, 'v_mov_b32_e32 v1, v60', ['v60'])]


def test_gemm_fragment_reads_are_waited_before_use(disasm_gemm):
    assert len(disasm_gemm) >= 20, len(disasm_gemm)
    mains = 0
    for (obj, f), body in disasm_gemm.items():
        assert lds_wait_violations(body) == [], (obj, f, lds_wait_violations(body)[:5])
        # the main loop is there: MFMAs fed by waited ds_read_b64 fragments
        if any(i.startswith('v_mfma_f64_16x16x4') for i in body):
            mains += 1
    assert mains == len(disasm_gemm)
    # and the replay sees a real stream's hazards: a copy of a fragment register
    # placed right after its read is flagged in every instance with the asm
    # fragment reads (the register-staged instances' LDS reads are the compiler's)
    n_asm = 0
    for (obj, f), body in disasm_gemm.items():
        i = next((k for k, ins in enumerate(body) if ins.startswith('ds_read_b64 v[')), None)
        if i is None:
            continue
        n_asm += 1
        reg = _REG.search(body[i]).group(0).replace('[', '').split(':')[0]
        hurt = body[:i + 1] + ['v_mov_b32_e32 v0, %s' % reg] + body[i + 1:]
        assert lds_wait_violations(hurt), (obj, f)
    assert n_asm >= 16, n_asm


def test_gemm_instances_do_not_spill(disasm_gemm):
    for (obj, f), body in disasm_gemm.items():
        assert not any(i.startswith('scratch_') or i.startswith('buffer_store') for i in body), f
