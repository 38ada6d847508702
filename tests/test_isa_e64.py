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
"""

SIZES = """Symbol table '.symtab' contains 3 entries:
   Num:    Value          Size Type    Bind   Vis       Ndx Name
     1: 0000000000000000    64 FUNC    GLOBAL PROTECTED   2 small_kernel
     2: 0000000000000100 131000 FUNC    GLOBAL PROTECTED   2 big_kernel
"""


def test_rewrites_only_encodable_selects_in_small_functions(tmp_path):
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
  out = dst.read_text().splitlines()
  small = out[out.index('small_kernel:') + 1:out.index('.Lfunc_end0:')]
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
  assert [l for l in out if 'cndmask' not in l] == \
         [l for l in ASM.splitlines() if 'cndmask' not in l]
