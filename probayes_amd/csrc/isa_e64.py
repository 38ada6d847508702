#!/usr/bin/env python3
"""Device-assembly pass of the build (hip_e64.sh): rewrites the VOP2 lane
select `v_cndmask_b32_e32 vD, src0, vS1, vcc` into its VOP3 encoding
`v_cndmask_b32_e64 vD, src0, vS1, vcc` -- the same operation on the same
registers.  On gfx950 the VOP2 form issues at ~23 cycles per wave
instruction at any occupancy and the VOP3 form at ~5
(tools/ubench/isa_cost.hip, profiles/r02y_isa_cnd.txt); the compiler always
shrinks to VOP2 when the mask was allocated to VCC.  Forms VOP3 cannot encode
on gfx9 are left alone: a literal src0, and an SGPR src0 (with VCC it would
be a second constant-bus read).
A function is rewritten only if its assembled size plus 4 bytes per
rewritten select (and per added s_nop) stays below 128 KB: then every branch inside it still fits
the 16-bit dword offset the compiler's branch relaxation assumed (larger
functions keep their VOP2 selects).
Hazard: VOP2 reads VCC implicitly, VOP3 as an explicit SGPR source, and a
VALU write of an SGPR followed by a VALU read of it as an SGPR operand needs
two wait states on gfx950 -- the compiler's hazard recognizer puts `s_nop 1`
between a v_cmp_*_e64 writing a mask and the v_cndmask_b32_e64 reading it
(every such pair in this build), and nothing between a VALU VCC write and
a VOP2 select.  So a rewritten select whose VCC was written by a VALU
instruction less than two wait states before it (counting instructions and
s_nop N as N + 1), or that follows a label within that window (a writer may
sit in any predecessor block), gets the missing wait states as an s_nop.
usage: isa_e64.py <in.s> <out.s> [<llvm-readelf -s of the assembled in.s>]"""
import re
import sys

PAT = re.compile(r'^(\s*)v_cndmask_b32_e32(\s+)(v\d+|v\[\d+:\d+\]),\s*([^,]+),\s*(v\d+),\s*vcc(\s*(;.*)?)$')
INLINE_INT = re.compile(r'^-?\d+$')


def ok_src0(s):
  s = s.strip()
  if re.fullmatch(r'v\d+', s):
    return True
  if INLINE_INT.match(s):
    return -16 <= int(s) <= 64
  return s in ('0.5', '-0.5', '1.0', '-1.0', '2.0', '-2.0', '4.0', '-4.0')


FUNC = re.compile(r'^([A-Za-z_.$][\w.$]*):')
LABEL = re.compile(r'^\s*([A-Za-z_.$%][\w.$]*):')
# VALU instructions that write VCC: VOPC e32 compares, carry-out e32 forms,
# and VOP3 forms with vcc as the scalar destination (second operand)
VCC_E32 = re.compile(r'^v_(cmpx?_\w+|add_co_u32|sub_co_u32|subrev_co_u32|addc_co_u32|'
                     r'subb_co_u32|subbrev_co_u32)_e32\b')
VCC_SDST = re.compile(r'^v_\w+\s+[^,]+,\s*vcc\s*,')
VCC_VOPC3 = re.compile(r'^v_cmpx?_\w+_e64\s+vcc\s*,')


def writes_vcc(ins):
  return bool(VCC_E32.match(ins) or VCC_SDST.match(ins) or VCC_VOPC3.match(ins))


def wait_needed(prev):
  """Wait states to add before a VOP3 read of VCC, given the instructions
  before it (nearest last; None marks a label)."""
  ws = 0
  for ins in reversed(prev):
    if ws >= 2:
      return 0
    if ins is None:
      return 2 - ws
    if ins.startswith('s_nop'):
      ws += int(ins.split()[1], 0) + 1
      continue
    if ins.startswith('v_') and writes_vcc(ins):
      return 2 - ws
    ws += 1
  return 0
LIMIT = 128 * 1024 - 256


def sizes(path):
  """symbol -> byte size from `llvm-readelf -s` output"""
  out = {}
  if path:
    with open(path) as f:
      for line in f:
        t = line.split()
        if len(t) == 8 and t[0].endswith(':') and t[3] == 'FUNC':
          out[t[7]] = int(t[2], 0)
  return out


def rewrite(lines, owner, allowed):
  """The rewritten lines, (selects rewritten, s_nops added, selects kept) and
  the bytes each function grows by."""
  n = kept = nops = 0
  out, grow = [], {}
  prev = []   # the last few instructions (None for a label)
  for line, func in zip(lines, owner):
    m = PAT.match(line.rstrip('\n'))
    if m and ok_src0(m.group(4)) and func in allowed:
      w = wait_needed(prev)
      if w:
        out.append('{}s_nop {}\n'.format(m.group(1), w - 1))
        prev.append('s_nop {}'.format(w - 1))
        nops += 1
        grow[func] = grow.get(func, 0) + 4
      line = '{}v_cndmask_b32_e64{}{}, {}, {}, vcc\n'.format(
          m.group(1), m.group(2), m.group(3), m.group(4).strip(), m.group(5))
      grow[func] = grow.get(func, 0) + 4
      n += 1
    elif 'v_cndmask_b32_e32' in line:
      kept += 1
    out.append(line)
    t = line.split(';')[0].strip()
    if LABEL.match(line) and not t.startswith('.set'):
      prev.append(None)
    elif t and not t.startswith('.'):
      prev.append(t)
    prev = prev[-4:]
  return out, (n, nops, kept), grow


# ---------------------------------------------------------------------------
# Second rewrite: an fp64 accumulate whose accumulator is a fresh copy,
#     v_mov_b64_e32 vD, vS            (vD = vS)
#     ...                              (nothing reads or writes vD, writes vS)
#     v_fmac_f64_e32 vD, A, B          (vD = A B + vD)
# becomes the one VOP3 instruction v_fma_f64 vD, A, B, vS: the same value in
# the same register, one VALU instruction fewer (the compiler selects the
# two-address VOP2 form and copies the accumulator when its old value stays
# live, e.g. x' = fma(r, scale, x) with x kept for the accept select).  Same
# bytes (4 + 4 -> 8), so branch offsets keep their range.  Only within a
# basic block; A must be VOP3-encodable (a VGPR, an SGPR pair -- vS is a
# VGPR, so one constant-bus read -- or an inline constant; no literal).
# ---------------------------------------------------------------------------
REG = re.compile(r'\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]')
MOV64 = re.compile(r'^(\s*)v_mov_b64_e32\s+v\[(\d+):(\d+)\],\s*v\[(\d+):(\d+)\]\s*(;.*)?$')
FMAC64 = re.compile(r'^(\s*)v_fmac_f64_e32\s+v\[(\d+):(\d+)\],\s*([^,]+),\s*(v\[\d+:\d+\])\s*(;.*)?$')
INLINE_F = {'0.5', '-0.5', '1.0', '-1.0', '2.0', '-2.0', '4.0', '-4.0', '0', '1'}


def regs(text, kind='v'):
  """VGPR numbers mentioned in an operand text"""
  out = set()
  for m in REG.finditer(text):
    if m.group(1) == kind:
      out.add(int(m.group(2)))
    elif m.group(3) == kind:
      out.update(range(int(m.group(4)), int(m.group(5)) + 1))
  return out


def ok_a(a):
  a = a.strip()
  if re.fullmatch(r'v\[\d+:\d+\]|s\[\d+:\d+\]', a):
    return True
  return a in INLINE_F or (INLINE_INT.match(a) is not None and -16 <= int(a) <= 64)


def fuse_fmac(lines, allowed, owner):
  """(rewritten lines, fused count)"""
  out = list(lines)
  n = 0
  pending = {}   # vD lo -> (index of the mov, vD set, vS set, vS text)
  for i, line in enumerate(lines):
    body = line.split(';')[0].strip()
    if LABEL.match(line) or not body or body.startswith('.') or \
        body.startswith('s_cbranch') or body.startswith('s_branch') or \
        body.startswith('s_setpc') or body.startswith('s_swappc') or \
        body.startswith('s_endpgm') or owner[i] not in allowed:
      pending = {}
      continue
    fm = FMAC64.match(line.rstrip('\n'))
    if fm:
      d = (int(fm.group(2)), int(fm.group(3)))
      p = pending.get(d[0])
      a, b = fm.group(4), fm.group(5)
      if p is not None and p[1] == set(range(d[0], d[1] + 1)) and ok_a(a) and \
          not (regs(a) & p[1]) and not (regs(b) & p[1]):
        out[p[0]] = ''
        out[i] = '{}v_fma_f64 v[{}:{}], {}, {}, {}\n'.format(
            fm.group(1), d[0], d[1], a.strip(), b, p[3])
        n += 1
        del pending[d[0]]
        continue
    mm = MOV64.match(line.rstrip('\n'))
    # any other instruction: operands it touches end the pending copies
    # (reads of vD, writes of vD or vS; a conservative textual check: any
    # mention of the registers)
    touched = regs(body)
    for k in [k for k, p in pending.items() if (touched & p[1]) or (touched & p[2])]:
      del pending[k]
    if mm:
      dset = set(range(int(mm.group(2)), int(mm.group(3)) + 1))
      sset = set(range(int(mm.group(4)), int(mm.group(5)) + 1))
      if not (dset & sset):
        pending[int(mm.group(2))] = (i, dset, sset,
                                     'v[{}:{}]'.format(mm.group(4), mm.group(5)))
  return [l for l in out if l != ''], n


def main():
  src, dst = sys.argv[1], sys.argv[2]
  size = sizes(sys.argv[3] if len(sys.argv) > 3 else None)
  lines = open(src).readlines()
  func, owner = None, []
  for line in lines:
    fm = FUNC.match(line)
    if fm and not fm.group(1).startswith('.L'):
      func = fm.group(1)
    owner.append(func)
  # the growth of every function if rewritten, then only those that stay in
  # the branch range
  _, _, grow = rewrite(lines, owner, set(owner) - {None})
  allowed = {f for f, g in grow.items() if f in size and size[f] + g < LIMIT}
  out, (n, nops, kept), _ = rewrite(lines, owner, allowed)
  # the fma fusion keeps every function's size (4 + 4 -> 8 bytes): all of them
  o2 = []
  func = None
  for line in out:
    fm = FUNC.match(line)
    if fm and not fm.group(1).startswith('.L'):
      func = fm.group(1)
    o2.append(func)
  out, nf = fuse_fmac(out, set(o2) - {None}, o2)
  with open(dst, 'w') as f:
    f.writelines(out)
  sys.stderr.write('isa_e64: {} mov + fmac_f64 pairs -> v_fma_f64\n'.format(nf))
  big = sorted(set(grow) - allowed)
  sys.stderr.write('isa_e64: {} VOP2 selects -> VOP3 ({} behind an s_nop), {} kept '
                   '({}; {} functions too large to rewrite)\n'.format(
                       n, nops, kept, src, len(big)))


if __name__ == '__main__':
  main()
