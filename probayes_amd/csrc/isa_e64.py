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
rewritten select stays below 128 KB: then every branch inside it still fits
the 16-bit dword offset the compiler's branch relaxation assumed (larger
functions keep their VOP2 selects).
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


def main():
  src, dst = sys.argv[1], sys.argv[2]
  size = sizes(sys.argv[3] if len(sys.argv) > 3 else None)
  lines = open(src).readlines()
  # per function: the number of convertible selects, to decide whether the
  # grown function still keeps every branch within range
  func, grow, owner = None, {}, []
  for line in lines:
    fm = FUNC.match(line)
    if fm and not fm.group(1).startswith('.L'):
      func = fm.group(1)
    m = PAT.match(line.rstrip('\n'))
    if m and ok_src0(m.group(4)) and func is not None:
      grow[func] = grow.get(func, 0) + 4
    owner.append(func)
  allowed = {f for f, g in grow.items() if f in size and size[f] + g < LIMIT}
  n = kept = 0
  out = []
  for line, func in zip(lines, owner):
    if True:
      m = PAT.match(line.rstrip('\n'))
      if m and ok_src0(m.group(4)) and func in allowed:
        line = '{}v_cndmask_b32_e64{}{}, {}, {}, vcc\n'.format(
            m.group(1), m.group(2), m.group(3), m.group(4).strip(), m.group(5))
        n += 1
      elif 'v_cndmask_b32_e32' in line:
        kept += 1
      out.append(line)
  with open(dst, 'w') as f:
    f.writelines(out)
  big = sorted(set(grow) - allowed)
  sys.stderr.write('isa_e64: {} VOP2 selects -> VOP3, {} kept ({}; {} functions '
                   'too large to rewrite)\n'.format(n, kept, src, len(big)))


if __name__ == '__main__':
  main()
