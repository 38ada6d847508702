"""Summary of scripts/pmc_cmd.sh passes: per kernel, the counters averaged
over dispatches, the dispatch time, the effective clock (GRBM_GUI_ACTIVE / 8
XCDs / time) and per-wave-step instruction counts.
usage: pmc_report.py <dir> <kernel-substr> <steps-per-dispatch>"""
import collections
import csv
import glob
import sys

d, sub, steps = sys.argv[1], sys.argv[2], float(sys.argv[3])
agg = collections.defaultdict(list)
dur = []
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
  for r in csv.DictReader(open(f)):
    if sub in r['Kernel_Name']:
      agg[r['Counter_Name']].append(float(r['Counter_Value']))
      dur.append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
m = {k: sum(v) / len(v) for k, v in agg.items()}
t = sum(dur) / len(dur) * 1e-9
w = m['SQ_WAVES']
print('dispatch {:.1f} us, clock {:.2f} GHz, waves {:.0f}'.format(
    t * 1e6, m['GRBM_GUI_ACTIVE'] / 8 / t / 1e9, w))
for k in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM_WR'):
  print('  {:20s} per wave-step {:8.1f}'.format(k, m[k] / w / steps))
for k in ('SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY',
          'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_SCA',
          'SQ_WAIT_INST_LDS'):
  if k in m:
    print('  {:20s} {:14.0f}  / wave-cycles {:.3f}'.format(
        k, m[k], m[k] / m['SQ_WAVE_CYCLES']))
