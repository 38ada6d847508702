"""Per-kernel averages of PMC passes (rocprofv3 --pmc, one directory per
pass under <dir>), plus per-wave-step figures when the step count is given.
usage: pmc_summary.py <dir> [kernel-substr] [steps-per-launch]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ''
spl = float(sys.argv[3]) if len(sys.argv) > 3 else 250.
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
  run = os.path.relpath(f, d).split(os.sep)[0].rsplit('_p', 1)[0]
  for r in csv.DictReader(open(f)):
    if sub in r['Kernel_Name']:
      key = (run, r['Kernel_Name'][:80])
      agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
for (run, k), cs in sorted(agg.items()):
  print(run, k)
  m = {c: sum(v) / len(v) for c, v in cs.items()}
  for c, v in sorted(m.items()):
    print('  {:26s} {:18.1f}'.format(c, v))
  w = m.get('SQ_WAVES')
  if w:
    per = lambda c: m[c] / w / spl if c in m else float('nan')
    print('  per wave-step: VALU {:.1f} SALU {:.1f} LDS {:.1f} VMEM_WR {:.2f}'
          .format(per('SQ_INSTS_VALU'), per('SQ_INSTS_SALU'),
                  per('SQ_INSTS_LDS'), per('SQ_INSTS_VMEM_WR')))
    if 'SQ_WAVE_CYCLES' in m:
      # SQ cycle counters are in quad-cycles (MI355X_MICROARCH.md)
      print('  per wave-step cycles: wave {:.0f} busy-frac {:.2f} wait_any {:.0f} '
            'wait_inst {:.0f}'.format(4 * per('SQ_WAVE_CYCLES'),
                                      m['SQ_BUSY_CYCLES'] / max(m['SQ_WAVE_CYCLES'], 1),
                                      4 * per('SQ_WAIT_ANY'), 4 * per('SQ_WAIT_INST_ANY')))
    if 'SQ_ACTIVE_INST_VALU' in m:
      print('  per wave-step: active_valu {:.0f} active_any {:.0f} vmem_wr_cyc {:.0f} '
            'wait_lds {:.0f}'.format(4 * per('SQ_ACTIVE_INST_VALU'),
                                      4 * per('SQ_ACTIVE_INST_ANY'),
                                      4 * per('SQ_INST_CYCLES_VMEM_WR'),
                                      4 * per('SQ_WAIT_INST_LDS')))
