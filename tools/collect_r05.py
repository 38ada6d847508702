"""Copy scripts/profile_r05.sh's output (gpurun_out/prof5) into profiles/:
per shape the kernel stats / trace CSVs, the FETCH_SIZE / WRITE_SIZE passes,
the bench lines, and a traffic JSON keyed by (kernel, chains, steps per
launch, rng) that bench.py's measured_traffic reads.  FETCH_SIZE is doubled
per MI355X_MICROARCH.md (gfx950 counts half of a wide coalesced read);
WRITE_SIZE is taken as reported (KiB).

usage: python tools/collect_r05.py <tag>      e.g. r05z

Every traffic JSON carries the sha256 of the library the passes ran
(gpurun_out/prof5/lib.sha256): bench.py takes roofline.traffic only from a
profile of the binary it loads.

The timed dispatches are the steady-state (FULL) form of the lane-pair
kernel: the first launch of a run (step 1) takes the general form.  The
driver's shape runs as a resident-server command; its traffic is taken from
the same 20 steps launched (PBH_SERVER=0, the same step code: the launched
form also reads and writes the chain state once, an upper bound), and the
server run itself is kept beside it (s20srv: kernel trace, bench lines,
per-command device stamps).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, 'gpurun_out', 'prof5')
KERNEL = 'mh_pair_kernel<10, 1, false, true, true, false>'   # FULL, loc 0, launched


def rows(path):
  return [r for r in csv.DictReader(open(path)) if KERNEL in r['Kernel_Name']]


def sq_summary(path, last):
  """The SQ counters of the last `last` FULL dispatches, averaged, plus
  VALU / SALU per wave-step and the LDS bank-conflict share."""
  by = {}
  for r in rows(path):
    by.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
  out = {k: sum(v[-last:]) / last for k, v in by.items()}
  return out


def main(tag):
  sha = open(os.path.join(PROF, 'lib.sha256')).read().split()[0]
  for shape, spl in (('s20', 20), ('s1000', 250)):
    src = os.path.join(PROF, shape)
    dst = lambda name: os.path.join(ROOT, 'profiles',
                                    '{}_{}_{}'.format(tag, shape, name))
    for a, b in (('trace/run_kernel_stats.csv', 'kernel_stats.csv'),
                 ('trace/run_kernel_trace.csv', 'kernel_trace.csv'),
                 ('fetch/run_counter_collection.csv', 'pmc_fetch_size.csv'),
                 ('write/run_counter_collection.csv', 'pmc_write_size.csv'),
                 ('sq/run_counter_collection.csv', 'pmc_sq.csv')):
      shutil.copy(os.path.join(src, a), dst(b))
    with open(dst('bench_lines.jsonl'), 'w') as f:
      for log in ('bench.log', 'bench_trace.log', 'bench_sq.log'):
        for line in open(os.path.join(src, log)):
          if line.startswith('{'):
            f.write(line)
    # the timed launches: spl steps each (the warm-up launch is shorter
    # at s20); pick the dispatches by their trace duration rank
    tr = rows(os.path.join(src, 'trace/run_kernel_trace.csv'))
    dur = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in tr]
    fetch = [float(r['Counter_Value']) for r in
             rows(os.path.join(src, 'fetch/run_counter_collection.csv'))]
    write = [float(r['Counter_Value']) for r in
             rows(os.path.join(src, 'write/run_counter_collection.csv'))]
    if shape == 's20':   # FULL dispatches: 4 one-step warm-ups, the timed 20
      sel_t, sel_f, sel_w = [dur[-1]], [fetch[-1]], [write[-1]]
    else:                # 250-step launches: the 4 timed (the warm-up is general)
      sel_t, sel_f, sel_w = dur[-4:], fetch[-4:], write[-4:]
    fk, wk = sum(sel_f) / len(sel_f), sum(sel_w) / len(sel_w)
    b = (2 * fk + wk) * 1024
    alg = 88.125 * 65536 * spl
    json.dump({'kernel': 'mh_pair_kernel<10, PHILOX, MOM=0, FULL>', 'chains': 65536,
               'steps_per_launch': spl, 'rng': 'philox',
               'fetch_size_kb': fk, 'write_size_kb': wk,
               'bytes_per_launch': b, 'algorithmic_bytes_per_launch': alg,
               'traffic_over_algorithmic': b / alg,
               'avg_launch_ns_trace': sum(sel_t) / len(sel_t),
               'dispatches': len(sel_t),
               'lib_sha256': sha,
               'sq_per_dispatch': sq_summary(os.path.join(src, 'sq/run_counter_collection.csv'),
                                             len(sel_t)),
               'source': 'scripts/profile_r05.sh ({}): rocprofv3 --pmc FETCH_SIZE '
                         '/ --pmc WRITE_SIZE in separate passes of bench.py; '
                         'FETCH_SIZE doubled (MI355X_MICROARCH.md)'.format(shape)},
              open(os.path.join(ROOT, 'profiles', '{}_traffic_{}.json'.format(
                  tag, shape)), 'w'), indent=1)
  srv = os.path.join(PROF, 's20srv')
  for a, b in (('trace/run_kernel_stats.csv', 'kernel_stats.csv'),
               ('trace/run_kernel_trace.csv', 'kernel_trace.csv'),
               ('probe.jsonl', 'server_probe.jsonl')):
    shutil.copy(os.path.join(srv, a),
                os.path.join(ROOT, 'profiles', '{}_s20srv_{}'.format(tag, b)))
  with open(os.path.join(ROOT, 'profiles', '{}_s20srv_bench_lines.jsonl'.format(tag)),
            'w') as f:
    for log in ('bench.log', 'bench_trace.log'):
      for line in open(os.path.join(srv, log)):
        if line.startswith('{'):
          f.write(line)
  with open(os.path.join(ROOT, 'profiles', '{}_bench_driver.jsonl'.format(tag)),
            'w') as f:
    for line in open(os.path.join(PROF, 'bench_driver.log')):
      if line.startswith('{'):
        f.write(line)
  src = os.path.join(PROF, 'bench_default.log')
  with open(os.path.join(ROOT, 'profiles', '{}_bench_default.jsonl'.format(tag)),
            'w') as f:
    for line in open(src):
      if line.startswith('{'):
        f.write(line)


if __name__ == '__main__':
  main(sys.argv[1])
