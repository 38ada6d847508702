#!/usr/bin/env python3
"""Static instruction mix of one kernel in a compiled device assembly file.

usage: isa_stats.py <file.s> <mangled-name-substring> [--blocks] [--dump LABEL]

Prints, per basic block of the kernel (label to label), the count of VALU,
SALU, LDS, VMEM and other instructions, and marks the blocks that branch
backwards (loop latches).  Used to price a change to a hot loop before a
GPU run (the PMC per-wave-step figures are the measured counterpart).
"""
import collections
import re
import sys


def kernel_lines(path, sub):
  out, inside = [], False
  for line in open(path):
    if not inside:
      if re.match(r'^_Z\S*' + re.escape(sub) + r'\S*:', line):
        inside = True
      continue
    if line.startswith('.Lfunc_end'):
      break
    out.append(line.rstrip('\n'))
  return out


def category(op):
  if op.startswith('v_readlane') or op.startswith('v_writelane'):
    return 'spill'
  if op.startswith('ds_'):
    return 'lds'
  if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
    return 'vmem'
  if op.startswith('v_'):
    if '_f64' in op or 'mfma' in op:
      return 'valu64'
    return 'valu'
  if op.startswith('s_waitcnt') or op.startswith('s_nop'):
    return 'wait'
  if op.startswith(('s_cbranch', 's_branch')):
    return 'branch'
  if op.startswith(('s_load', 's_buffer')):
    return 'smem'
  if op.startswith('s_'):
    return 'salu'
  return 'other'


def blocks(lines):
  cur, name, order = [], 'entry', []
  res = collections.OrderedDict()
  for l in lines:
    m = re.match(r'^(\.LBB\S+|\.L\S+):', l) or re.match(r'^; (%bb\.\d+):', l)
    if m:
      res[name] = cur
      order.append(name)
      name, cur = m.group(1), []
      continue
    t = l.strip()
    if not t or t.startswith(('.', ';')):
      continue
    cur.append(t.split(';')[0].strip())
  res[name] = cur
  return res


def main():
  path, sub = sys.argv[1], sys.argv[2]
  dump = sys.argv[sys.argv.index('--dump') + 1] if '--dump' in sys.argv else None
  bl = blocks(kernel_lines(path, sub))
  names = list(bl)
  tot = collections.Counter()
  for i, (n, ins) in enumerate(bl.items()):
    c = collections.Counter(category(x.split()[0]) for x in ins if x)
    tot.update(c)
    back = [x for x in ins if x.startswith(('s_cbranch', 's_branch')) and
            x.split()[-1] in names and names.index(x.split()[-1]) <= i]
    if '--blocks' in sys.argv or back:
      print('{:14s} n={:4d} {} {}'.format(n, len(ins), dict(c),
                                          'LOOP->' + back[0].split()[-1] if back else ''))
    if dump == n:
      ops = collections.Counter(x.split()[0] for x in ins)
      for op, k in ops.most_common():
        print('    {:32s} {}'.format(op, k))
  print('total', dict(tot))


if __name__ == '__main__':
  main()
