"""The build's device-assembly pass (probayes_amd/csrc/isa_e64.py): VOP2 lane
selects become the VOP3 encoding of the same operation only where VOP3 can
encode them, and only in functions small enough to keep every branch in the
16-bit range the compiler's relaxation assumed."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
  spec = importlib.util.spec_from_file_location(
      'isa_e64', os.path.join(ROOT, 'probayes_amd', 'csrc', 'isa_e64.py'))
  m = importlib.util.module_from_spec(spec)
  spec.loader.exec_module(m)
  return m


ASM = """\t.text
small_kernel:
\ts_mov_b32 s0, 0
\ts_mov_b32 s1, 0
\tv_cndmask_b32_e32 v1, v2, v3, vcc
\tv_cndmask_b32_e32 v4, 0, v5, vcc    ; inline constant
\tv_cndmask_b32_e32 v6, -16, v7, vcc
\tv_cndmask_b32_e32 v8, 0x3ff00000, v9, vcc
\tv_cndmask_b32_e32 v10, s4, v11, vcc
\tv_cndmask_b32_e32 v12, 65, v13, vcc
\ts_endpgm
.Lfunc_end0:
big_kernel:
\tv_cndmask_b32_e32 v1, v2, v3, vcc
\ts_endpgm
.Lfunc_end1:
hazard_kernel:
\tv_cndmask_b32_e32 v1, v2, v3, vcc
\ts_mov_b32 s0, 0
\ts_mov_b32 s1, 0
\tv_cmp_lt_f32_e32 vcc, v1, v2
\tv_cndmask_b32_e32 v4, v5, v6, vcc
\tv_cmp_lt_f64_e64 vcc, v[0:1], v[2:3]
\tv_mov_b32_e32 v7, 0
\tv_cndmask_b32_e32 v8, v9, v10, vcc
\tv_add_co_u32_e32 v11, vcc, v12, v13
\ts_nop 0
\tv_cndmask_b32_e32 v14, v15, v16, vcc
\tv_cmp_eq_u32_e32 vcc, 0, v17
\tv_mov_b32_e32 v18, 0
\tv_mov_b32_e32 v19, 0
\tv_cndmask_b32_e32 v20, v21, v22, vcc
\ts_and_b64 vcc, exec, s[2:3]
\tv_cndmask_b32_e32 v23, v24, v25, vcc
.LBB2_1:
\tv_cndmask_b32_e32 v26, v27, v28, vcc
\ts_endpgm
.Lfunc_end2:
"""

SIZES = """Symbol table '.symtab' contains 4 entries:
   Num:    Value          Size Type    Bind   Vis       Ndx Name
     1: 0000000000000000    64 FUNC    GLOBAL PROTECTED   2 small_kernel
     2: 0000000000000100 131000 FUNC    GLOBAL PROTECTED   2 big_kernel
     3: 0000000000020100   256 FUNC    GLOBAL PROTECTED   2 hazard_kernel
"""


def _run(tmp_path):
  m = _mod()
  src, dst, sz = tmp_path / 'in.s', tmp_path / 'out.s', tmp_path / 'sizes'
  src.write_text(ASM)
  sz.write_text(SIZES)
  import sys
  argv = sys.argv
  sys.argv = ['isa_e64.py', str(src), str(dst), str(sz)]
  try:
    m.main()
  finally:
    sys.argv = argv
  return dst.read_text().splitlines()


def test_rewrites_only_encodable_selects_in_small_functions(tmp_path):
  out = _run(tmp_path)
  small = out[out.index('small_kernel:') + 3:out.index('.Lfunc_end0:')]
  assert small[0].strip() == 'v_cndmask_b32_e64 v1, v2, v3, vcc'
  assert small[1].strip() == 'v_cndmask_b32_e64 v4, 0, v5, vcc'
  assert small[2].strip() == 'v_cndmask_b32_e64 v6, -16, v7, vcc'
  # a literal, an SGPR (second constant-bus read beside VCC) and an
  # integer outside the inline range stay VOP2
  assert small[3].strip().startswith('v_cndmask_b32_e32 v8, 0x3ff00000')
  assert small[4].strip().startswith('v_cndmask_b32_e32 v10, s4')
  assert small[5].strip().startswith('v_cndmask_b32_e32 v12, 65')
  big = out[out.index('big_kernel:') + 1:out.index('.Lfunc_end1:')]
  assert big[0].strip() == 'v_cndmask_b32_e32 v1, v2, v3, vcc'   # 128 KB limit
  # everything else is untouched
  keep = lambda ls: [l for l in ls if 'cndmask' not in l and 's_nop' not in l]
  assert keep(out) == keep(ASM.splitlines())


def test_vcc_write_read_hazard_gets_its_wait_states(tmp_path):
  """A VALU write of VCC needs two wait states before a VOP3 read of it
  (the compiler's own `s_nop 1` between v_cmp_*_e64 and v_cndmask_b32_e64):
  the pass adds what is missing -- also right after a label -- and nothing
  after SALU writes or when two instructions already separate them."""
  out = _run(tmp_path)
  h = [l.strip() for l in out[out.index('hazard_kernel:') + 1:out.index('.Lfunc_end2:')]]
  assert h[0:2] == ['s_nop 1', 'v_cndmask_b32_e64 v1, v2, v3, vcc']   # after the label
  i = h.index('v_cmp_lt_f32_e32 vcc, v1, v2')
  assert h[i + 1:i + 3] == ['s_nop 1', 'v_cndmask_b32_e64 v4, v5, v6, vcc']
  i = h.index('v_cmp_lt_f64_e64 vcc, v[0:1], v[2:3]')
  assert h[i + 1:i + 4] == ['v_mov_b32_e32 v7, 0', 's_nop 0',
                            'v_cndmask_b32_e64 v8, v9, v10, vcc']
  i = h.index('v_add_co_u32_e32 v11, vcc, v12, v13')
  assert h[i + 1:i + 4] == ['s_nop 0', 's_nop 0', 'v_cndmask_b32_e64 v14, v15, v16, vcc']
  i = h.index('v_cmp_eq_u32_e32 vcc, 0, v17')
  assert h[i + 3] == 'v_cndmask_b32_e64 v20, v21, v22, vcc'
  i = h.index('s_and_b64 vcc, exec, s[2:3]')
  assert h[i + 1] == 'v_cndmask_b32_e64 v23, v24, v25, vcc'
  i = h.index('.LBB2_1:')
  assert h[i + 1:i + 3] == ['s_nop 1', 'v_cndmask_b32_e64 v26, v27, v28, vcc']
